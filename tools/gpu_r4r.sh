#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py -x -q --timeout 200 --timeout-method thread -k "dense or deferred or identical_to_brute" > gpurun_out/r4r_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4r_pytest.log; [ $rc -eq 0 ] || exit $rc
M3D_GRID_HEAVY=8 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_icp.py tests/test_gpu_prep.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4r_pytest_forced.log 2>&1
rc=$?; tail -2 gpurun_out/r4r_pytest_forced.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="defer1 new defer1 new" bash tools/gpu_ab_prof.sh
