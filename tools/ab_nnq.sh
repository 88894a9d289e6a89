#!/bin/bash
# A/B of the NN queries-per-lane knob (M3D_NN_Q) on the cfg1 bench, ICP only.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for q in ${QS:-4 2}; do
  M3D_NN_Q=$q timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ransac > gpurun_out/bench_q$q.log 2>&1
  rc=$?; echo "bench q=$q rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
