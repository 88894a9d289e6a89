#!/bin/bash
# Cold setup: stream-ordered grid-build temporaries (M3D_GRID_ASYNC_TMP=1) against hipMalloc/hipFree
# ones (the default) on the tree's library: ICP/prep/multi GPU tests with the option on, then
# alternating tools/cold_timing.py runs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
M3D_GRID_ASYNC_TMP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_icp.py tests/test_gpu_prep.py tests/test_gpu_multi.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gtmp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gtmp.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  timeout -k 10 120 python tools/cold_timing.py --tag sync || exit 1
  M3D_GRID_ASYNC_TMP=1 timeout -k 10 120 python tools/cold_timing.py --tag async || exit 1
done
