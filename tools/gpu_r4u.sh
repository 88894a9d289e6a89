#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp tools/ab/libm3d_dbg.so 3d-matching_amd/m3d/libm3d.so
M3D_GRID_HEAVY=8 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4u_dbg.log 2>&1
rc=$?; echo "debug forced rc=$rc guards=$(grep -c '\[guard\]' gpurun_out/r4u_dbg.log)"; tail -2 gpurun_out/r4u_dbg.log; [ $rc -eq 0 ] || exit $rc
cp tools/ab/libm3d_new.so 3d-matching_amd/m3d/libm3d.so
M3D_GRID_HEAVY=8 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_prep.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4u_forced.log 2>&1
rc=$?; tail -2 gpurun_out/r4u_forced.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="defer1 new defer1 new" bash tools/gpu_ab_prof.sh
