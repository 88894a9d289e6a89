#!/bin/bash
# quick per-kernel timing of the ICP loops (brute + grid) under rocprofv3 --kernel-trace --stats
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/icpprof -o icp --output-format csv -- \
  python3 tools/prof_kernels.py --skip-ransac --icp-iters ${ICP_ITERS:-30} > gpurun_out/icpprof.log 2>&1
rc=$?; echo "icp prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py gpurun_out/icpprof | cut -c1-110
