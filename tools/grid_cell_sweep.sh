#!/bin/bash
# Grid NN cell-size sweep (M3D_GRID_CELL_DIV: cell = radius / div) at the three grid geometries,
# with per-launch candidate statistics (M3D_GRID_STATS=1) in a separate short pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gridsweep
for div in ${DIVS:-1 2 3 4}; do
  timeout -k 10 300 env M3D_GRID_CELL_DIV=$div python3 tools/grid_timing.py 20 > gpurun_out/gridsweep/t_$div.log 2>&1
  rc=$?; echo "div=$div rc=$rc"; cat gpurun_out/gridsweep/t_$div.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 env M3D_GRID_CELL_DIV=$div M3D_GRID_STATS=1 python3 tools/grid_timing.py 3 > gpurun_out/gridsweep/s_$div.log 2>&1
  rc=$?; grep "grid stats" gpurun_out/gridsweep/s_$div.log | sort | uniq -c | sort -rn | head -12; [ $rc -eq 0 ] || exit $rc
done
