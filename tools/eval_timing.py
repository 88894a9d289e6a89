"""Per-evaluation grid NN scan time of a cfg1 grid ICP loop (library HIP events): the first,
unseeded evaluation against the seeded ones.  AB_LIB=tools/ab/NAME.so times another build.
Usage: python tools/eval_timing.py [evaluations] [ns]"""
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

n_eval = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
torch.cuda.set_device(0)
ctx = context()
src, tgt, nrm, _ = synth.icp_pair(ns, ns, seed=0)
lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=50, nn="grid")
for rep in range(3):
    lp.reset(np.eye(4))
    ctx.profile(True)
    ctx.profile_read(_lib.KERNEL_NN), ctx.profile_read(_lib.KERNEL_TERMS)
    out = []
    for k in range(n_eval):
        lp.step()
        torch.cuda.synchronize()
        nn_ms, n = ctx.profile_read(_lib.KERNEL_NN)
        t_ms, tn = ctx.profile_read(_lib.KERNEL_TERMS)
        out.append((nn_ms / max(n, 1) * 1e3, t_ms / max(tn, 1) * 1e3))
    ctx.profile(False)
    print(f"ns {ns}, rep {rep}: scan / tail us per evaluation: " + " ".join(f"{a:.1f}/{b:.1f}" for a, b in out),
          flush=True)
