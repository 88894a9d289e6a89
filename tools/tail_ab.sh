#!/bin/bash
# Round 6 (second session): the fused ICP tail — finer tail-clock stamps (reduce: loads landed / LDS
# sum; solve: fitness-rmse / before the solve) of the in-tree code, then grid_timing alternated
# between the in-tree library and tools/ab/$1.so (cfg1 three times each, 1M x 1M once each).
# Needs tools/ab/$1.so (and, for the stamps, tools/ab/tclk_new.so; tools/ab_build.sh).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
v=${1:-head}
if [ -f tools/ab/tclk_new.so ]; then
  AB_LIB=tools/ab/tclk_new.so timeout -k 10 120 python3 tools/tail_clock.py grid > gpurun_out/tclk_new.log 2>&1 || exit $?
fi
for rep in 1 2 3; do
  timeout -k 10 200 python3 tools/grid_timing.py 50 cfg1 > gpurun_out/gt_new_$rep.log 2>&1 || exit $?
  AB_LIB=tools/ab/$v.so timeout -k 10 200 python3 tools/grid_timing.py 50 cfg1 > gpurun_out/gt_${v}_$rep.log 2>&1 || exit $?
done
timeout -k 10 200 python3 tools/grid_timing.py 50 "1M x" > gpurun_out/gt_new_1m.log 2>&1 || exit $?
AB_LIB=tools/ab/$v.so timeout -k 10 200 python3 tools/grid_timing.py 50 "1M x" > gpurun_out/gt_${v}_1m.log 2>&1 || exit $?
for f in gpurun_out/tclk_new.log gpurun_out/gt_*.log; do [ -f $f ] || continue; echo "== $f"; grep -v amdgpu $f; done
