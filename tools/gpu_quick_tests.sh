#!/bin/bash
# GPU box: a selection of GPU tests (PYTEST_K) then an optional short bench (BENCH_ARGS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "${PYTEST_K:-.}" > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|PASSED|FAILED|Error" gpurun_out/quick_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/quick_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/quick_bench.log; exit $rc
fi
