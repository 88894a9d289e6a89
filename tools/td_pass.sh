#!/bin/bash
# The grid scan's texture-data path at cfg1 (TD_TD_BUSY share): one rocprofv3 --pmc
# pass of tools/prof_kernels.py over the cfg1 grid loop -> gpurun_out/td/.  Run on the GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/td
timeout -k 10 -s KILL 120 rocprofv3 --pmc TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE -d gpurun_out/td/p3 -o p3 \
  --output-format csv -- python3 tools/prof_kernels.py --nn grid --skip-ransac --icp-iters 10 \
  > gpurun_out/td/p3.log 2>&1
rc=$?; echo "td pass rc=$rc"; exit $rc
