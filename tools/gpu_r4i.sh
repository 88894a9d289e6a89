#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cullprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cullprof/t -o cull --output-format csv -- python3 tools/cull_timing.py 3 > gpurun_out/cullprof/run.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/cullprof/run.log
f=$(find gpurun_out/cullprof/t -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-8

python3 tools/split_kernel_trace.py $(find gpurun_out/cullprof/t -name "*kernel_trace.csv" | head -1) | grep -E "score|cull|kabsch" | head -12
