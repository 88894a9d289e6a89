#!/usr/bin/env python3
"""Grid ICP on partial overlaps (AB_LIB: another build of libm3d.so): cfg1's 100k x 100k pair with
half of the target removed (x above its median), and 1M x 1M likewise — half of the sources have
no target within r (the round-6 empty-ball certificate experiment, docs/EXPERIMENTS.md §R6).
Per-launch average of the grid NN over the evaluations (library HIP events), fitness.
Usage: python tools/partial_overlap_timing.py [iters]"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import _lib, synth

if os.environ.get("AB_LIB"):
    _lib.LIB_PATH = Path(os.environ["AB_LIB"]).resolve()
from m3d.core import Cloud, IcpLoop, context

it = int(sys.argv[1]) if len(sys.argv) > 1 else 30
torch.cuda.set_device(0)
ctx = context()
for name, n in (("100k x 50k (half the target)", 100_000), ("1M x 500k (half the target)", 1_000_000)):
    src, tgt, nrm, _ = synth.icp_pair(n, n, seed=0)
    keep = tgt[:, 0] < np.median(tgt[:, 0])
    lp = IcpLoop(Cloud(src), Cloud(tgt[keep], nrm[keep]), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=it, nn="grid")
    lp.reset(np.eye(4))
    lp.steps(it + 1)  # warm-up; the timed run uses a fresh loop
    torch.cuda.synchronize()
    lp = IcpLoop(Cloud(src), Cloud(tgt[keep], nrm[keep]), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=it, nn="grid")
    lp.reset(np.eye(4))
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_read(_lib.KERNEL_NN)
    lp.steps(it + 1)
    nn_ms, k = ctx.profile_read(_lib.KERNEL_NN)
    ctx.profile(False)
    r = lp.result()
    print(f"{name}: grid_nn {nn_ms / k * 1e3:.1f} us per launch ({k} launches), fitness {r.fitness:.4f}", flush=True)
