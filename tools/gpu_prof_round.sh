#!/bin/bash
# Round profile set (TAG): rocprofv3 kernel trace + stats of the bench command itself, the plain
# bench, then the short driver (tools/prof_kernels.py at the bench's shapes: H = 1e5) under a
# trace pass and separate PMC passes (one counter group per run), and the 1M x 1M grid NN's
# FETCH/WRITE.  Every step has its own time limit; a failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/benchprof gpurun_out/prof gpurun_out/prof1m
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof/trace -o bench --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/benchprof/bench_under_rocprof.log 2>&1
step $? bench_trace
timeout -k 10 600 python3 bench.py > gpurun_out/benchprof/bench_plain.log 2>&1
step $? bench_plain
P="--icp-iters 10 --hyps 100000"
run() { local dir=$1 name=$2; shift 2; local args=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d gpurun_out/$dir/$name -o $name --output-format csv -- \
    python3 tools/prof_kernels.py $args > gpurun_out/$dir/$name.log 2>&1
  step $? $dir/$name; }
run prof trace "$P" --kernel-trace --stats
run prof pmc1 "$P" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run prof pmc2 "$P" --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA
run prof pmc3 "$P" --pmc FETCH_SIZE
run prof pmc4 "$P" --pmc WRITE_SIZE
P1="--n 1000000 --nn grid --skip-ransac --icp-iters 4"
run prof1m trace "$P1" --kernel-trace --stats
run prof1m pmc3 "$P1" --pmc FETCH_SIZE
run prof1m pmc4 "$P1" --pmc WRITE_SIZE
