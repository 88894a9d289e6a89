#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_icp.py -x -q --timeout 200 --timeout-method thread -k "dense or deferred or identical_to_brute" > gpurun_out/r4p_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4p_pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old new old new" bash tools/gpu_ab_prof.sh || exit 1
bash tools/gpu_ab.sh 2>&1 | grep -v "^step\|grid stats\|^points"
