#!/usr/bin/env python3
"""Brute-force NN timing at cfg1 (100k x 100k): per-launch average of nn_mfma_kernel and of the
fused terms tail over `iters` seeded evaluations (library HIP events), for A/B runs under the
M3D_NN_* knobs (M3D_NN_EXP=1: the sweep without the exact path — keys then wrong, timing only).
Usage: python tools/nn_timing.py [iters]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

import os

from m3d import _lib, synth

if os.environ.get("AB_LIB"):  # time another build of the library (tools/ab_build.sh)
    _lib.LIB_PATH = Path(os.environ["AB_LIB"]).resolve()
from m3d.core import Cloud, IcpLoop, context

it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
torch.cuda.set_device(0)
ctx = context()
src, tgt, nrm, _ = synth.icp_pair(100_000, 100_000, seed=0)
lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1,
             max_iteration=it, nn="brute")
lp.reset(np.eye(4))
lp.steps(it + 1)
torch.cuda.synchronize()
ctx.profile(True)
ctx.profile_read(_lib.KERNEL_NN), ctx.profile_read(_lib.KERNEL_TERMS)
lp.reset(np.eye(4))
lp.steps(it + 1)
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
print(f"cfg1 brute: nn {nn_ms / n * 1e3:.1f} us per launch ({n} launches), terms {t_ms / tn * 1e3:.1f} us, "
      f"iteration {e0.elapsed_time(e1) * 1e3 / (it + 1):.1f} us (no kernel events), "
      f"fitness {lp.result().fitness:.4f}", flush=True)
