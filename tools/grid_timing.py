#!/usr/bin/env python3
"""Grid-NN ICP timing (AB_LIB=path: another build of libm3d.so) at cfg1 (100k x 100k) and cfg3's per-rank geometry (1M sources x one 125k
target shard) and 1M x 1M: per-launch averages of the NN and terms kernels (library HIP events).
Usage: [WARM=k] python tools/grid_timing.py [iters] [all|cfg1|1M x 1M|...]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

import os

from m3d import _lib, synth

if os.environ.get("AB_LIB"):  # time another build of the library (tools/ab/*.so)
    _lib.LIB_PATH = Path(os.environ["AB_LIB"]).resolve()
from m3d.core import Cloud, IcpLoop, context

it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
only = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "all" else None
warm = int(os.environ.get("WARM", "0"))  # WARM=k: kernel events over evaluations k .. iters only
torch.cuda.set_device(0)
ctx = context()
for name, ns, nt_all, shard in (("cfg1 100k x 100k", 100_000, 100_000, 1), ("1M x 125k shard", 1_000_000, 1_000_000, 8),
                                ("1M x 1M", 1_000_000, 1_000_000, 1)):
    if only and only not in name:
        continue
    src, tgt, nrm, _ = synth.icp_pair(ns, nt_all, seed=0)
    nt = nt_all // shard
    tc = Cloud(tgt[:nt], nrm[:nt], center=tgt.mean(axis=0)) if shard > 1 else Cloud(tgt, nrm)
    lp = IcpLoop(Cloud(src), tc, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=it, nn="grid")
    lp.reset(np.eye(4))
    lp.steps(it + 1)
    torch.cuda.synchronize()
    lp.reset(np.eye(4))
    if warm:  # the first evaluations untimed (stale seeds while the transform still moves)
        lp.steps(warm)
        torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_read(_lib.KERNEL_NN), ctx.profile_read(_lib.KERNEL_TERMS)
    lp.steps(it + 1 - warm)
    nn_ms, n = ctx.profile_read(_lib.KERNEL_NN)
    t_ms, tn = ctx.profile_read(_lib.KERNEL_TERMS)
    ctx.profile(False)
    lp.reset(np.eye(4))
    lp.steps(it + 1)  # a sequence requested twice is captured into a graph (m3d_icp_steps)
    lp.reset(np.eye(4))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lp.steps(it + 1)
    e1.record()
    torch.cuda.synchronize()
    wall_us = e0.elapsed_time(e1) * 1e3 / (it + 1)
    nn = nn_ms / n
    b = 28 * ns + 16 * nt
    print(f"{name}: grid_nn {nn * 1e3:.1f} us ({b / (nn * 1e-3) / 1e9:.0f} GB/s algorithmic, "
          f"{b / (nn * 1e-3) / 8e12 * 100:.1f}% of 8 TB/s), terms {t_ms / max(tn, 1) * 1e3:.1f} us, iteration {wall_us:.1f} us (no kernel events), fitness {lp.result().fitness:.4f}",
          flush=True)
