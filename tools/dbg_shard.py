#!/usr/bin/env python3
"""Diagnostics: the target-sharded NN (3 shards emulated on one device) against the unsharded NN
under the SAME transform every iteration; prints per-iteration key mismatches."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import synth
from m3d.core import Cloud, IcpLoop

nn = sys.argv[1] if len(sys.argv) > 1 else "brute"
src, tgt, nrm, _ = synth.icp_pair(20000, 30000, seed=13)
s = Cloud(src)
bounds = [0, 7000, 19001, 30000]
c = tgt.mean(axis=0)
shards = [Cloud(tgt[a:b], nrm[a:b], center=c) for a, b in zip(bounds[:-1], bounds[1:])]
kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=6, nn=nn)
loops = [IcpLoop(s, sh, 0.12, **kw) for sh in shards]
ref = IcpLoop(s, Cloud(tgt, nrm, center=c), 0.12, **kw)
for lp in loops + [ref]:
    lp.reset(np.eye(4))
ns = len(src)
NONE = 0x7FFFFFFFFFFFFFFF
for it in range(7):
    keys = [torch.empty(ns, dtype=torch.int64, device="cuda") for _ in loops]
    for lp, off, k in zip(loops, bounds, keys):
        lp.shard_nn(off, k)
    kmin = torch.stack(keys).min(dim=0).values
    kref = torch.empty(ns, dtype=torch.int64, device="cuda")
    ref.shard_nn(0, kref)
    a, b = kmin.cpu().numpy(), kref.cpu().numpy()
    pseudo = (a != NONE) & ((a & 0xFFFFFFFF) == 0xFFFFFFFF)
    a2 = np.where(pseudo, NONE, a)
    bad = np.nonzero(a2 != b)[0]
    print(f"it {it}: pseudo in MIN {pseudo.sum()}, mismatches {len(bad)}")
    for i in bad[:5]:
        per = [int(k[i].item()) for k in keys]
        print("   i", i, "sharded", hex(int(a[i])), "ref", hex(int(b[i])), "per-shard", [hex(x) for x in per])
    sums = [torch.empty(32, dtype=torch.float64, device="cuda") for _ in loops]
    for lp, off, sm in zip(loops, bounds, sums):
        lp.shard_terms(off, kmin, sm)
    tot = torch.stack(sums).sum(dim=0)
    sref = torch.empty(32, dtype=torch.float64, device="cuda")
    ref.shard_terms(0, kref, sref)
    print("   sums max rel diff", float(((tot - sref).abs() / sref.abs().clamp_min(1e-300)).max()))
    for lp in loops + [ref]:
        lp.solve(tot)
