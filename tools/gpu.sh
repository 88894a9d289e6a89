#!/bin/bash
# The one GPU-box script (run through gpurun):  bash tools/gpu.sh STEP [STEP ...]
#   tests    pytest -m gpu, one process, per-test timeout ($PYTEST_ARGS; $PYTEST_K: a -k expression)
#            -> gpurun_out/pytest_gpu.log
#   smoke    __graft_entry__.smoke()                                       -> gpurun_out/smoke.log
#   bench    bench.py $BENCH_ARGS                                          -> gpurun_out/bench.log
#   launch   bench.py --gpus 2 on this one-GPU box: must refuse (exit != 0, no JSON line)
#   dist1    the N > 1 code path at world 1: torch.distributed.run, nccl pg + libm3d's RCCL comm
#   multi    the N > 1 path with 2 ranks on cuda:0 over gloo (functional; RCCL needs a GPU per rank)
#   large    cfg3 per-GPU geometry (1M sources x 125k-target shard) + a 1M x 1M grid ICP
#   prof     rocprofv3 --kernel-trace --stats of bench.py $PROF_BENCH_ARGS, and the plain bench
#            -> gpurun_out/benchprof/
#   pmc      tools/prof_kernels.py at the bench's shapes: a trace pass, then one --pmc pass per
#            counter group; the 1M x 1M grid NN's FETCH/WRITE   -> gpurun_out/prof/, prof1m/
#   py:FILE  python FILE $PY_ARGS (a timing / probe script)       -> gpurun_out/<FILE>.log
# Every GPU step runs under its own time limit; the first failing step ends the script, so
# nothing touches the GPU after a fault, abort, segfault or timeout.  tools/collect_profiles.sh
# (in the container) copies the prof / pmc summaries into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "stopping after $1 rc=$2"; exit "$2"; }
pmc_run() {  # dir name "args" rocprof-args...
  local dir=$1 name=$2 args=$3; shift 3
  mkdir -p gpurun_out/$dir
  timeout -k 10 300 rocprofv3 "$@" -d gpurun_out/$dir/$name -o $name --output-format csv -- \
    python3 tools/prof_kernels.py $args > gpurun_out/$dir/$name.log 2>&1
  local rc=$?; echo "$dir/$name rc=$rc"; [ $rc -eq 0 ] || stop "$dir/$name" $rc
}
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
        --timeout-method thread -rf ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
      [ $rc -eq 0 ] || stop tests $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
      [ $rc -eq 0 ] || stop smoke $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.log; echo
      [ $rc -eq 0 ] || stop bench $rc ;;
    launch)
      timeout -k 10 300 python bench.py --gpus 2 --steps 1 --warmup 0 > gpurun_out/launch2.log 2>&1
      rc=$?; echo "bench --gpus 2 on one GPU: rc=$rc (expect != 0)"; tail -3 gpurun_out/launch2.log
      if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then stop launch $rc; fi
      if [ $rc -eq 0 ] || grep -q '^{' gpurun_out/launch2.log; then stop launch 1; fi ;;
    dist1)
      M3D_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 2 --warmup 1 \
        --no-cpu-baseline --cfg3-n 200000 --cfg3-iters 5 --no-ransac-api --no-cfg4 > gpurun_out/dist1.log 2>&1
      rc=$?; echo "dist1 rc=$rc"; tail -c 400 gpurun_out/dist1.log; echo
      [ $rc -eq 0 ] || stop dist1 $rc ;;
    multi)
      M3D_BENCH_SAME_DEVICE=1 M3D_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 1 \
        --warmup 1 --icp-iters 10 --no-cpu-baseline --comm torch --cfg3-n 200000 --cfg3-iters 3 \
        --no-ransac-api --no-cfg4 > gpurun_out/multi.log 2>&1
      rc=$?; echo "multi rc=$rc"; grep '^{' gpurun_out/multi.log | tail -1 | cut -c1-400
      [ $rc -eq 0 ] || stop multi $rc ;;
    large)
      timeout -k 10 300 python3 bench.py --ns 1000000 --nt 125000 --icp-iters 5 --steps 1 --warmup 1 \
        --no-ransac --no-cpu-baseline --no-ransac-api --no-cfg4 --no-cfg3 > gpurun_out/large_cfg3.log 2>&1
      rc=$?; echo "large rc=$rc"; tail -c 400 gpurun_out/large_cfg3.log; echo
      [ $rc -eq 0 ] || stop large $rc ;;
    prof)
      mkdir -p gpurun_out/benchprof
      PB=${PROF_BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof/trace -o bench \
        --output-format csv -- python3 bench.py $PB > gpurun_out/benchprof/bench_under_rocprof.log 2>&1
      rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || stop prof $rc
      timeout -k 10 600 python3 bench.py > gpurun_out/benchprof/bench_plain.log 2>&1
      rc=$?; echo "bench plain rc=$rc"; [ $rc -eq 0 ] || stop bench_plain $rc ;;
    pmc)
      P="--icp-iters 10 --hyps 100000"
      pmc_run prof trace "$P" --kernel-trace --stats
      pmc_run prof pmc1 "$P" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
      pmc_run prof pmc2 "$P" --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA
      pmc_run prof pmc3 "$P" --pmc FETCH_SIZE
      pmc_run prof pmc4 "$P" --pmc WRITE_SIZE
      P1="--n 1000000 --nn grid --skip-ransac --icp-iters 4"
      pmc_run prof1m trace "$P1" --kernel-trace --stats
      pmc_run prof1m pmc3 "$P1" --pmc FETCH_SIZE
      pmc_run prof1m pmc4 "$P1" --pmc WRITE_SIZE ;;
    py:*)
      f=${step#py:}; b=$(basename "$f" .py)
      timeout -k 10 600 python -u "$f" ${PY_ARGS:-} > "gpurun_out/$b.log" 2>&1
      rc=$?; echo "$f rc=$rc"; tail -c 1500 "gpurun_out/$b.log"; echo
      [ $rc -eq 0 ] || stop "$f" $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
