#!/bin/bash
# Grid NN launch-shape sweep: lanes per query (M3D_GRID_LANES) x row/point batching (M3D_GRID_RB)
# x cell divisor (M3D_GRID_CELL_DIV) at the three grid geometries (tools/grid_timing.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gridlanes
for div in ${DIVS:-1 3}; do for L in ${LANES:-1 2 4}; do for rb in ${RBS:-22 24}; do
  f=gpurun_out/gridlanes/d${div}_L${L}_rb${rb}.log
  timeout -k 10 300 env M3D_GRID_CELL_DIV=$div M3D_GRID_LANES=$L M3D_GRID_RB=$rb python3 tools/grid_timing.py 20 > $f 2>&1
  rc=$?; echo "div=$div L=$L rb=$rb rc=$rc"; grep -v amdgpu.ids $f | sed 's/ (.*of 8 TB\/s)//'; [ $rc -eq 0 ] || exit $rc
done; done; done
