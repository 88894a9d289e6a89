"""Per-wave timeline of the last grid scan (diagnostic build: tools/ab_build.sh clk -DM3D_SCAN_CLOCK=1,
then AB_LIB=tools/ab/clk.so python tools/scan_clock.py).  s_memrealtime ticks at 100 MHz (10 ns)."""
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
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
src, tgt, nrm, _ = synth.icp_pair(n, n, seed=0)
lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=50, nn="grid")
lp.reset(np.eye(4))
lp.steps(20)
torch.cuda.synchronize()
L = 4 if n <= 300000 else 2
nw = (n * L + 63) // 64
nw = min(nw, 65536)
buf = (C.c_ulonglong * (2 * 65536))()
rc = ctx.lib.m3d_debug_scan_clock(buf, C.c_int(2 * nw))
a = np.frombuffer(buf, dtype=np.uint64)[: 2 * nw].reshape(-1, 2).astype(np.int64)
a = a[a[:, 1] > 0]
t0 = a[:, 0].min()
st = (a[:, 0] - t0) * 10e-3  # us
du = (a[:, 1] - a[:, 0]) * 10e-3
en = st + du
print(f"waves {len(a)}: span {en.max():.2f} us; start: median {np.median(st):.2f} p90 {np.percentile(st, 90):.2f} max {st.max():.2f}")
print(f"duration: mean {du.mean():.2f} median {np.median(du):.2f} p90 {np.percentile(du, 90):.2f} p99 {np.percentile(du, 99):.2f} max {du.max():.2f} us")
print(f"end: median {np.median(en):.2f} p90 {np.percentile(en, 90):.2f} p99 {np.percentile(en, 99):.2f} max {en.max():.2f}")
hist, edges = np.histogram(st, bins=12)
print("starts per bin:", " ".join(f"{e:.1f}:{h}" for e, h in zip(edges[:-1], hist)))
hist, edges = np.histogram(en, bins=12)
print("ends per bin:  ", " ".join(f"{e:.1f}:{h}" for e, h in zip(edges[:-1], hist)))
