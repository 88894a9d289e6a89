"""Timeline of the last fused ICP tail (terms_solve_kernel) of a cfg1 grid loop (diagnostic build:
tools/ab_build.sh tclk -DM3D_TAIL_CLOCK=1, then AB_LIB=tools/ab/tclk.so python tools/tail_clock.py [grid|brute]):
per-wave terms time, the last block's ticket, reduction and solve, and the terms time of the
waves that resolved ambiguous queries against the others.  s_memrealtime ticks at 100 MHz."""
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
NW = 4096
buf = (C.c_ulonglong * (3 * NW + 24))()
ctx.lib.m3d_debug_tail_clock(buf, C.c_int(3 * NW + 24))
a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
w = a[: 2 * NW].reshape(-1, 2)
keep = w[:, 1] > 0
w = w[keep]
amb = a[2 * NW + 8:3 * NW + 8][keep]
t0 = w[:, 0].min()
st, en = (w[:, 0] - t0) * 1e-2, (w[:, 1] - t0) * 1e-2
du = en - st
tk, rd, sv, l0, l1, v6, mm, rf = [(a[2 * NW + k] - t0) * 1e-2 for k in range(8)]
print(f"{nn}: waves {len(w)}; start max {st.max():.2f} us; terms per wave mean {du.mean():.2f} p90 "
      f"{np.percentile(du, 90):.2f} max {du.max():.2f}; last wave done {en.max():.2f}; ticket won {tk:.2f}; "
      f"reduced {rd:.2f}; solved {sv:.2f} us | solve: ldlt in {l0:.2f} out {l1:.2f}, vec6 {v6:.2f}, "
      f"T stored {mm:.2f}, refresh {rf:.2f}")
ld, lr, fr, pv = [(a[3 * NW + k] - t0) * 1e-2 if a[3 * NW + k] > 0 else float("nan") for k in (8, 9, 10, 11)]
print(f"  reduce: loads landed {ld:.2f}, LDS sum {lr:.2f}; solve: fitness/rmse {fr:.2f}, before solve {pv:.2f} us")
has = amb > 0
if has.any():
    print(f"  waves with ambiguous queries: {has.sum()} ({amb.sum()} queries), terms mean {du[has].mean():.2f} "
          f"max {du[has].max():.2f} us; the others mean {du[~has].mean():.2f} max {du[~has].max():.2f} us")
slow = np.argsort(du)[-10:][::-1]
print("  10 slowest waves (us, ambiguous queries, wave index): " +
      ", ".join(f"{du[k]:.2f}/{amb[k]}/{k}" for k in slow))
