#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/cfg4_icp_trace.py 2>&1 | grep -v amdgpu || exit 1
timeout -k 10 300 python3 -u tools/cfg4_refine_timing.py --reps 3 2>&1 | grep -v amdgpu | tail -1 || exit 1
timeout -k 10 400 python3 -u bench.py > gpurun_out/r4n_bench.json 2> gpurun_out/r4n_bench.err || exit 1
python3 - <<'P'
import json
d=json.loads(open("gpurun_out/r4n_bench.json").read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"])
for k,v in d.items():
    if isinstance(v, dict) and "value" in v and k not in ("cpu_baseline",):
        print(k, v.get("value"), v.get("ms_per_iteration", v.get("ms_per_run", "")))
P
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4n_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r4n_pytest.log; exit $rc
