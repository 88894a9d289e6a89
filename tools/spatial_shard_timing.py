#!/usr/bin/env python3
"""Per-rank NN time of the target-sharded ICP at cfg3's N = 8 geometry, emulated on one GPU
(VERDICT r5 #2): 1M sources against a 1M target in 8 shards of 125k, INDEX shards (ranges of the
unordered cloud: every shard spans the whole surface) against SPATIAL shards (m3d.dist.
spatial_shards: slabs along the longest axis).  The protocol runs as on 8 ranks (NN on every shard,
MIN of the d64 keys, claims, MIN, terms, SUM, solve); each shard's NN launches are timed with
library events after two warm iterations.  Prints per-shard ms and the max (the per-rank time of a
real 8-GPU run), and checks that both shardings end at the same transform."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-matching_amd"))
import numpy as np
import torch

from m3d import _lib, synth
from m3d import dist as D
from m3d.core import Cloud, IcpLoop, context

W = 8
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
NNS = tuple(sys.argv[2].split(",")) if len(sys.argv) > 2 else ("grid", "brute")
ITERS = 6
src, tgt, nrm, _ = synth.icp_pair(N, N, seed=0)
s = Cloud(src)
ctx = context()
c = tgt.mean(axis=0)
res = {}
for kind in ("index", "spatial"):
    if kind == "index":
        perm, bounds = np.arange(N), np.array([k * N // W for k in range(W + 1)])
    else:
        perm, bounds = D.spatial_shards(tgt, W)
    ts, ns_ = tgt[perm], nrm[perm]
    shards = [Cloud(ts[a:b], ns_[a:b], center=c) for a, b in zip(bounds[:-1], bounds[1:])]
    for nn in NNS:
        loops = [IcpLoop(s, sh, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=ITERS, nn=nn)
                 for sh in shards]
        for lp in loops:
            lp.reset(np.eye(4))
        per = np.zeros(W)
        per_nn = np.zeros(W)  # scan + fp64 winner (shard_nn: what a rank runs before the MIN)
        timed = 0
        for it in range(ITERS + 1):
            keys = [torch.empty(N, dtype=torch.int64, device="cuda") for _ in loops]
            for k, lp in enumerate(loops):
                torch.cuda.synchronize()
                ctx.profile(True)
                ctx.profile_read(_lib.KERNEL_NN)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                lp.shard_nn(int(bounds[k]), keys[k])
                e1.record()
                torch.cuda.synchronize()
                ms, n = ctx.profile_read(_lib.KERNEL_NN)
                ctx.profile(False)
                if it >= 2:
                    per[k] += ms / max(n, 1)
                    per_nn[k] += e0.elapsed_time(e1)
            timed += it >= 2
            kmin = torch.stack(keys).min(dim=0).values
            claims = [torch.empty(N, dtype=torch.int32, device="cuda") for _ in loops]
            for lp, cl in zip(loops, claims):
                lp.shard_claim(kmin, cl)
            cmin = torch.stack(claims).min(dim=0).values
            sums = [torch.empty(32, dtype=torch.float64, device="cuda") for _ in loops]
            for k, (lp, sm) in enumerate(zip(loops, sums)):
                lp.shard_terms(int(bounds[k]), kmin, cmin, sm)
            tot = torch.stack(sums).sum(dim=0)
            for lp in loops:
                lp.solve(tot)
        per /= max(timed, 1)
        per_nn /= max(timed, 1)
        r = loops[0].result()
        res[(kind, nn)] = r
        print(f"{kind:7s} {nn:5s}: NN ms per shard {np.round(per, 4).tolist()}  max {per.max():.4f}  "
              f"mean {per.mean():.4f}  | scan + winner ms max {per_nn.max():.4f} mean {per_nn.mean():.4f}  "
              f"fitness {r.fitness:.6f}", flush=True)
        del loops
        torch.cuda.empty_cache()
for nn in NNS:
    a, b = res[("index", nn)], res[("spatial", nn)]
    print(f"{nn}: same transform index vs spatial: {np.array_equal(a.transformation, b.transformation)}, "
          f"same fitness {a.fitness == b.fitness}")
