#!/bin/bash
# Large-size sanity runs on one GPU: cfg3 per-GPU geometry (1M sources x 125k-target shard)
# and a 1M x 1M grid-NN ICP; each step under its own time limit.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --ns 1000000 --nt 125000 --icp-iters 5 --steps 1 --warmup 1 \
  --no-ransac --no-cpu-baseline > gpurun_out/large_cfg3.log 2>&1
rc=$?; echo "cfg3-geometry rc=$rc"; tail -c 600 gpurun_out/large_cfg3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 - > gpurun_out/large_grid.log 2>&1 <<'PY'
import sys, time
sys.path.insert(0, "3d-matching_amd")
import numpy as np, torch
from m3d import synth
from m3d.core import Cloud, icp, nn1
src, tgt, nrm, T = synth.icp_pair(1_000_000, seed=3)
s, t = Cloud(src), Cloud(tgt, nrm)
torch.cuda.synchronize(); t0 = time.perf_counter()
out = icp(s, t, 0.04, np.eye(4), relative_fitness=-1, relative_rmse=-1, max_iteration=20, nn="grid")
torch.cuda.synchronize(); el = time.perf_counter() - t0
print("1M x 1M grid ICP: %.1f ms for 21 evaluations, fitness %.4f, err %.2e" % (
    el * 1e3, out.fitness, np.abs(out.transformation - T).max()))
idx_b, d_b = nn1(s, t, T, 0.04, nn="brute")
idx_g, d_g = nn1(s, t, T, 0.04, nn="grid")
print("1M x 1M nn1 brute == grid:", bool(torch.equal(idx_b, idx_g)), bool(torch.equal(d_b, d_g)))
PY
rc=$?; echo "grid-1M rc=$rc"; cat gpurun_out/large_grid.log | tail -3; exit $rc
