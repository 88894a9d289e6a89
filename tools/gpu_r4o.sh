#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py -x -q --timeout 200 --timeout-method thread -k "dense or deferred or identical_to_brute" > gpurun_out/r4o_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4o_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh
