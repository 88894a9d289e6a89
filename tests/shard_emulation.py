"""Multi-GPU protocols emulated on one device (test helpers for the -m gpu tests): one IcpLoop
per shard, the all-reduces done with torch min/sum over the shards' buffers."""
import numpy as np

from m3d.core import Cloud, IcpLoop


def shard_step(lp, off, ns, sums):
    """One iteration of the target-shard protocol on a single shard (no exchange needed)."""
    import torch

    dk = torch.empty(ns, dtype=torch.int64, device="cuda")
    cl = torch.empty(ns, dtype=torch.int32, device="cuda")
    lp.shard_nn(off, dk)
    lp.shard_claim(dk, cl)
    lp.shard_terms(off, dk, cl, sums)
    lp.solve(sums)


def run_target_shards(src, tgt, nrm, bounds, iters, nn, r=0.12, check_keys=None):
    """The multi-GPU target-shard protocol (MIN on the d64 keys, MIN on the claims, SUM on the
    terms) emulated with one IcpLoop per shard on one device.  Returns the loops."""
    import torch

    s = Cloud(src)
    c = tgt.mean(axis=0)  # one frame for all shards: seed bounds on non-owning shards
    shards = [Cloud(tgt[a:b], nrm[a:b], center=c) for a, b in zip(bounds[:-1], bounds[1:])]
    loops = [IcpLoop(s, sh, r, relative_fitness=-1, relative_rmse=-1, max_iteration=iters, nn=nn)
             for sh in shards]
    for lp in loops:
        lp.reset(np.eye(4))
    ns = len(src)
    for it in range(iters + 1):
        keys = [torch.empty(ns, dtype=torch.int64, device="cuda") for _ in loops]
        for lp, off, k in zip(loops, bounds, keys):
            lp.shard_nn(off, k)
        kmin = torch.stack(keys).min(dim=0).values
        claims = [torch.empty(ns, dtype=torch.int32, device="cuda") for _ in loops]
        for lp, cl in zip(loops, claims):
            lp.shard_claim(kmin, cl)
        cmin = torch.stack(claims).min(dim=0).values
        if check_keys is not None:
            check_keys(it, loops[0], kmin, cmin)
        sums = [torch.empty(32, dtype=torch.float64, device="cuda") for _ in loops]
        for lp, off, sm in zip(loops, bounds, sums):
            lp.shard_terms(off, kmin, cmin, sm)
        tot = torch.stack(sums).sum(dim=0)
        for lp in loops:
            lp.solve(tot)
    return loops


