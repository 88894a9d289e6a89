set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_quick.log | tail -3 | cut -c1-600
exit $rc
