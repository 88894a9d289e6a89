#!/bin/bash
# GPU tests with the current library, then grid ICP timing A/B over library variants built in
# 3d-matching_amd/m3d/ab/ (base = previous tree, sr8 = ambiguous queries resolved in the scan + 8 waves/EU cap, sr = without the cap, sroff = sr8 with M3D_GRID_SCANRES=0).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=3d-matching_amd/m3d
cp $L/libm3d.so $L/ab/libm3d_cur.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base sr8 sr sroff; do
    if [ $v = sroff ]; then cp $L/ab/libm3d_sr8.so $L/libm3d.so; export M3D_GRID_SCANRES=0; else cp $L/ab/libm3d_$v.so $L/libm3d.so; unset M3D_GRID_SCANRES; fi
    echo "== $v rep $rep" >> gpurun_out/ab_grid.log
    timeout -k 10 180 python tools/grid_timing.py 50 >> gpurun_out/ab_grid.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "timing rc=$rc ($v)"; exit $rc; }
  done
done
unset M3D_GRID_SCANRES
cp $L/ab/libm3d_cur.so $L/libm3d.so
cat gpurun_out/ab_grid.log
