#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ransac_batch_det.py 4 > gpurun_out/ransac_det.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ransac_det.log | tail -40; exit $rc
