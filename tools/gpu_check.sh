#!/bin/bash
# GPU-box run: tests, smoke, bench.  Each GPU step has its own time limit; after a fault,
# abort, segfault or timeout nothing else touches the GPU (exit codes other than 0/1 stop).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after $1 rc=$2"; exit "$2"; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -rf \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || stop pytest $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || stop smoke $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
