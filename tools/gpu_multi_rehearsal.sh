#!/bin/bash
# Functional rehearsal of bench.py's N > 1 path on a one-GPU box: 2 ranks on cuda:0 over gloo
# (RCCL needs one GPU per rank).  Checks that the sharded ICP / RANSAC protocol runs end to end
# and that rank 0 prints the JSON line; the timing is not meaningful.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
M3D_BENCH_SAME_DEVICE=1 M3D_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus ${NPROC:-2} --steps 1 --warmup 1 --icp-iters 10 --no-cpu-baseline --comm torch --cfg3-n 200000 --cfg3-iters 3 ${ARGS:-} \
  > gpurun_out/multi_rehearsal.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; grep '^{' gpurun_out/multi_rehearsal.log | tail -1 | cut -c1-600; exit $rc
