#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_icp.py \
  -k "host_cloud or chunks or corr_pairs or refine or empty" > gpurun_out/r4d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4d_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r4d_tests.log | head -20; exit $rc; }
M3D_RUN_PROF=1 timeout -k 10 180 python3 -u tools/refine_timing.py --reps 5 > gpurun_out/refine_prof.log 2>&1
rc=$?; grep -v "m3d run" gpurun_out/refine_prof.log | tail -3; grep "m3d run" gpurun_out/refine_prof.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -u tools/refine_timing.py > gpurun_out/refine_timing.log 2>&1
rc=$?; tail -2 gpurun_out/refine_timing.log; [ $rc -eq 0 ] || exit $rc
M3D_UPLOAD=pageable timeout -k 10 180 python3 -u tools/refine_timing.py > gpurun_out/refine_timing_pageable.log 2>&1
rc=$?; tail -2 gpurun_out/refine_timing_pageable.log; exit $rc
