#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python3 -u tools/grid_loop_min.py 2>&1 | grep "grid loop" | sed "s/^/default: /" || exit 1
  M3D_GRID_HEAVY=1000000 timeout -k 10 120 python3 -u tools/grid_loop_min.py 2>&1 | grep "grid loop" | sed "s/^/amb-to-heavy: /" || exit 1
done
M3D_GRID_HEAVY=1000000 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4v -o k --output-format csv -- python3 tools/grid_loop_min.py > gpurun_out/r4v.log 2>&1 || exit 1
python3 - $(find gpurun_out/r4v -name "*kernel_stats.csv" | head -1) <<'P'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("grid_nn", "terms", "solve", "reduce", "heavy")):
        print("amb-to-heavy", n[:60], r["Calls"], r["AverageNs"])
P
