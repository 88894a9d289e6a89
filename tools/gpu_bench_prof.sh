#!/bin/bash
# rocprofv3 kernel-trace/stats of the bench command itself, then PMC passes on the short driver.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/benchprof
BARGS=${BARGS:---steps 3 --warmup 1 --no-cpu-baseline}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof/trace -o bench --output-format csv -- \
  python3 bench.py $BARGS > gpurun_out/benchprof/bench_under_rocprof.log 2>&1
rc=$?; echo "bench trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py $BARGS > gpurun_out/benchprof/bench_plain.log 2>&1
rc=$?; echo "bench plain rc=$rc"; [ $rc -eq 0 ] || exit $rc
PROF_ARGS="${PROF_ARGS:---icp-iters 10 --hyps 20000}" bash tools/gpu_prof.sh
