#!/bin/bash
# per-kernel A/B of libm3d builds (tools/ab/libm3d_<v>.so, v in $VARIANTS) on the cfg1 grid loop,
# plus the cfg4 cold refine stages per build
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abprof
for v in ${VARIANTS:-old new}; do
  cp tools/ab/libm3d_$v.so 3d-matching_amd/m3d/libm3d.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof/$v -o k --output-format csv -- python3 tools/grid_loop_min.py > gpurun_out/abprof/$v.log 2>&1 || exit 1
  f=$(find gpurun_out/abprof/$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'P'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("grid_nn", "terms", "solve", "reduce")):
        print(sys.argv[2], n[:60], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
P
  if [ "${CFG4:-1}" = 1 ]; then
    timeout -k 10 300 python3 -u tools/cfg4_refine_timing.py --reps 3 2>&1 | grep -v amdgpu | tail -1 | sed "s/^/$v /" || exit 1
  fi
done
