"""Per-phase time of the fused ICP terms pass at cfg1 (diagnostic build: tools/ab_build.sh tph
-DM3D_TERMS_CLOCK=1, then AB_LIB=tools/ab/tph.so python tools/terms_phases.py [grid|brute]).  Each
stamp follows an s_waitcnt 0, so a phase's loads complete inside it: the phases serialise, and the
sum is longer than the undisturbed pass (the stamps stay in registers until the end).  Phases: 1 key / runner-up / point loads (+ point write-back),
2 fp64 decision (+ the ambiguous queries' grid walk), 3 winner record gather, 4 fp64 terms,
5 wave reduction, 6 block barrier, 7 LDS sum + partial store."""
import ctypes as C
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import _lib, synth

_lib.LIB_PATH = Path(os.environ["AB_LIB"]).resolve()
from m3d.core import Cloud, IcpLoop, context

torch.cuda.set_device(0)
ctx = context()
nn = sys.argv[1] if len(sys.argv) > 1 else "grid"
src, tgt, nrm, _ = synth.icp_pair(100_000, 100_000, seed=0)
lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=50, nn=nn)
lp.reset(np.eye(4))
lp.steps(20)
torch.cuda.synchronize()
buf = (C.c_ulonglong * (4096 * 8))()
ctx.lib.m3d_debug_terms_clock(buf, C.c_int(4096 * 8))
a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(-1, 8)
a = a[a[:, 7] > 0]
t0 = a[:, 0].min()
d = np.diff(a, axis=1) * 1e-2
print(f"{nn}: {len(a)} waves; start spread {(a[:, 0].max() - t0) * 1e-2:.2f} us; last end {(a[:, 7].max() - t0) * 1e-2:.2f} us")
names = ["loads", "decision+walk", "gather", "terms", "wave sum", "barrier", "store"]
for k, n in enumerate(names):
    print(f"  {n:14s} mean {d[:, k].mean():.2f}  p90 {np.percentile(d[:, k], 90):.2f}  max {d[:, k].max():.2f} us")
print(f"  total per wave mean {(a[:, 7] - a[:, 0]).mean() * 1e-2:.2f} us")
