#!/bin/bash
# Copy the judged rocprof summaries from gpurun_out/ (scratch) into profiles/ (tracked).
set -eu
TAG=${TAG:-r01}
cd "$(dirname "$0")/.."
ks=$(find gpurun_out/benchprof/trace -name "*kernel_stats.csv" | head -1)
cp "$ks" profiles/${TAG}_bench_kernel_stats.csv
grep -h '^{' gpurun_out/benchprof/bench_under_rocprof.log | tail -1 > profiles/${TAG}_bench_under_rocprof.json
grep -h '^{' gpurun_out/benchprof/bench_plain.log | tail -1 > profiles/${TAG}_bench_plain.json
ks2=$(find gpurun_out/prof/trace -name "*kernel_stats.csv" | head -1)
cp "$ks2" profiles/${TAG}_prof_kernels_stats.csv
python3 tools/prof_summary.py gpurun_out/prof --json profiles/pmc_${TAG}.json > profiles/${TAG}_pmc_summary.txt
echo "profiles/ updated for $TAG"
