#!/usr/bin/env python3
"""A/B timing of ICP loop kernels across libm3d builds (development tool).

Usage: python tools/terms_ab.py <libm3d.so> [nn] — runs the cfg1 ICP loop (100k ↔ 100k, 30
iterations) from that library build and prints the per-launch NN / terms times (library HIP
events; run with M3D_ICP_FUSED=0 to time the terms pass alone)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import _lib

_lib.LIB_PATH = Path(sys.argv[1]).resolve()
from m3d import synth  # noqa: E402
from m3d.core import Cloud, IcpLoop, context  # noqa: E402

nn = sys.argv[2] if len(sys.argv) > 2 else "grid"
torch.cuda.set_device(0)
ctx = context()
src, tgt, nrm, _ = synth.icp_pair(100_000, 100_000, seed=0)
lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=30, nn=nn)
for rep in range(2):
    lp.reset(np.eye(4))
    if rep == 1:
        ctx.profile(True)
        ctx.profile_read(_lib.KERNEL_NN), ctx.profile_read(_lib.KERNEL_TERMS)
    lp.steps(31)
    torch.cuda.synchronize()
nn_ms, n = ctx.profile_read(_lib.KERNEL_NN)
t_ms, tn = ctx.profile_read(_lib.KERNEL_TERMS)
print(f"{Path(sys.argv[1]).name} {nn}: nn {nn_ms / n * 1e3:.2f} us, terms {t_ms / max(tn, 1) * 1e3:.2f} us, "
      f"fitness {lp.result().fitness:.5f}", flush=True)
