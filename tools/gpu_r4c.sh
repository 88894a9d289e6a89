#!/bin/bash
# Round 4: chunked m3d_icp_run + device correspondence compaction — the new/affected GPU tests,
# then the refine_registration stage split.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_icp.py \
  -k "chunks or corr_pairs or refine or step_loop or graph or empty or icp_grid_identical" > gpurun_out/r4c_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4c_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r4c_tests.log | head -20; exit $rc; }
timeout -k 10 180 python3 -u tools/refine_timing.py > gpurun_out/refine_timing.log 2>&1
rc=$?; tail -3 gpurun_out/refine_timing.log; exit $rc
