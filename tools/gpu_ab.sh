#!/bin/bash
# A/B of two libm3d builds on one box: tools/ab/libm3d_{old,new}.so swapped in turn (new, old, new, old)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in new old new old; do
  cp tools/ab/libm3d_$v.so 3d-matching_amd/m3d/libm3d.so
  timeout -k 10 300 python3 -u bench.py --no-ransac --no-ransac-api --no-cpu-baseline --steps 3 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
  python3 - "$v" <<'P'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
out = {"headline": round(d["value"], 1)}
for k, v in d.items():
    if isinstance(v, dict) and "value" in v and k != "cpu_baseline":
        out[k] = round(v["value"], 3)
print(sys.argv[1], json.dumps(out), flush=True)
P
  timeout -k 10 300 python3 -u tools/cfg4_refine_timing.py --reps 3 2>&1 | grep -v amdgpu | tail -1 | sed "s/^/$v /" || exit 1
done
cp tools/ab/libm3d_new.so 3d-matching_amd/m3d/libm3d.so
M3D_GRID_STATS=1 timeout -k 10 300 python3 -u tools/cfg4_icp_trace.py 2>&1 | grep -v amdgpu | cut -c1-150
