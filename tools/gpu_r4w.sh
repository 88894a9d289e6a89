#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4w_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4w_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/multipair_timing.py 2>&1 | grep -v amdgpu || exit 1
M3D_BLOCK_CACHE=0 timeout -k 10 200 python3 -u tools/multipair_timing.py 2>&1 | grep -v amdgpu | sed "s/^/nocache: /" || exit 1
timeout -k 10 200 python3 -u tools/cloud_upload_timing.py --ns 100000 --nt 100000 --reps 15 2>&1 | grep -v amdgpu | head -5
