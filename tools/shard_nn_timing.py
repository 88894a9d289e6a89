#!/usr/bin/env python3
"""Per-rank NN time of target-sharded ICP, emulated on one GPU: 100k sources against an 800k-point
target in 8 shards of 100k (the bench's N = 8 geometry).  Runs the protocol (NN on every shard,
MIN of the keys, terms, SUM, solve) for a few iterations and times one shard's brute-force NN
launches with HIP events, once with per-shard centring (no bounds: non-owning shards search with
the radius) and once with one shared frame (m3d_cloud_create_framed: distance-bound seeds)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import _lib, synth
from m3d.core import Cloud, IcpLoop, context

W, NS, NT = 8, 100_000, 100_000
src, tgt, nrm, _ = synth.icp_pair(NS, NT * W, seed=0)
s = Cloud(src)
ctx = context()
for framed in (False, True):
    c = tgt.mean(axis=0) if framed else None
    shards = [Cloud(tgt[k * NT:(k + 1) * NT], nrm[k * NT:(k + 1) * NT], center=c) for k in range(W)]
    loops = [IcpLoop(s, sh, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=8, nn="brute")
             for sh in shards]
    for lp in loops:
        lp.reset(np.eye(4))
    per_rank = np.zeros(W)
    for it in range(6):
        keys = [torch.empty(NS, dtype=torch.int64, device="cuda") for _ in loops]
        for k, lp in enumerate(loops):
            torch.cuda.synchronize()
            ctx.profile(True)
            ctx.profile_read(_lib.KERNEL_NN)
            lp.shard_nn(k * NT, keys[k])
            torch.cuda.synchronize()
            ms, n = ctx.profile_read(_lib.KERNEL_NN)
            ctx.profile(False)
            if it >= 2:
                per_rank[k] += ms / max(n, 1)
        kmin = torch.stack(keys).min(dim=0).values
        sums = [torch.empty(32, dtype=torch.float64, device="cuda") for _ in loops]
        for k, (lp, sm) in enumerate(zip(loops, sums)):
            lp.shard_terms(k * NT, kmin, sm)
        tot = torch.stack(sums).sum(dim=0)
        for lp in loops:
            lp.solve(tot)
    per_rank /= 4
    r = loops[0].result()
    print(f"{'shared frame (bounds)' if framed else 'per-shard frames    '}: NN ms per rank "
          f"{np.round(per_rank, 3).tolist()}  max {per_rank.max():.3f}  fitness {r.fitness:.5f}")
