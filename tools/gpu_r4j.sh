#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_ransac.py -k "culling or bench_batch or gui_loop" > gpurun_out/r4j_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|assert" gpurun_out/r4j_tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/cull_timing.py 10 2>&1 | grep -v amdgpu.ids
bash tools/gpu_r4i.sh
