#!/bin/bash
# 1M x 1M grid NN sweep (>= 0.08 of 8 TB/s): target cell divisor x lanes per
# query x (rows, points) batching, events per launch (tools/grid_timing.py, 1M x 1M only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/grid1m
for div in 2 3 4; do for L in 1 2 4; do for RB in 22 42 24; do
  timeout -k 10 120 env M3D_GRID_CELL_DIV=$div M3D_GRID_LANES=$L M3D_GRID_RB=$RB python3 tools/grid_timing.py 20 "1M x 1M" > gpurun_out/grid1m/t_${div}_${L}_${RB}.log 2>&1
  rc=$?; echo "div=$div L=$L RB=$RB rc=$rc $(grep -v amdgpu.ids gpurun_out/grid1m/t_${div}_${L}_${RB}.log | tail -1)"; [ $rc -eq 0 ] || exit $rc
done; done; done
