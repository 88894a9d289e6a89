"""Multi-GPU protocols over torch.distributed (backend "nccl" = RCCL over xGMI; "gloo" in tests).

One process per GPU.  Hot-path shardings; the source-sharded ICP variant
(``SourceShardedIcp``: sources split, target replicated, one 256-B SUM per iteration) is the
cheaper exchange whenever the target fits one GPU; the target-sharded one is the north-star's:

* ICP, target-sharded (cfg3).  Rank r owns target points [off_r, off_r + n_r) (points + normals)
  and a replica of the source.  Per iteration:
    1. local NN over the shard → packed key per source: (bits(d²_f32) << 32) | global_idx
       (d² ≥ 0 so float bits order like the values; the low word breaks exact ties towards the
       lowest index; KEY_NONE = INT64_MAX = "no target inside the radius");
    2. all_reduce(keys, MIN)               — Ns × 8 B (0.8 MB at 100k, 8 MB at 1M);
    3. each rank accumulates the fp64 estimation terms of the sources whose winner it owns
       (it holds that target's point and normal) → 32 doubles;
    4. all_reduce(sums, SUM)               — 256 B;
    5. every rank runs the identical solve/update → identical T everywhere (no broadcast).
* RANSAC, hypothesis-sharded (cfg2 at N>1).  Rank r evaluates hypothesis ids
  [hyp0_r, hyp0_r + H_r) with the counter-based sampler (ids are global, so the union equals the
  single-GPU run); the winner is all_reduce(MAX) of (count << 32) | (0xFFFFFFFF − id) — highest
  count, lowest id on ties (the reference's first strict improvement) — and every rank
  recomputes the winner's transform from its id (the sampler is a pure function of the id).

The driver below is backend-agnostic: the GPU backend is ``m3d.core.IcpLoop``; the CPU tests
plug in an oracle-backed backend and run the identical protocol over gloo.
"""

from __future__ import annotations

import numpy as np

KEY_NONE = 0x7FFFFFFFFFFFFFFF
_LOW = 0xFFFFFFFF


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Balanced contiguous shard [off, off + cnt) of n items for `rank`."""
    base, extra = divmod(n, world)
    off = rank * base + min(rank, extra)
    return off, base + (1 if rank < extra else 0)


def pack_nn_key(d2_f32, idx):
    """numpy: (float32 bits << 32) | idx as int64; KEY_NONE where idx < 0."""
    d2 = np.asarray(d2_f32, np.float32)
    idx = np.asarray(idx, np.int64)
    k = (d2.view(np.uint32).astype(np.int64) << 32) | (idx & _LOW)
    return np.where(idx < 0, np.int64(KEY_NONE), k)


def unpack_nn_key(keys):
    k = np.asarray(keys, np.int64)
    none = k == KEY_NONE
    d2 = (k >> 32).astype(np.uint32).view(np.float32)
    idx = (k & _LOW).astype(np.int64)
    return np.where(none, np.float32(np.inf), d2), np.where(none, -1, idx)


def best_key(count: int, hyp_id: int) -> int:
    return (int(count) << 32) | (_LOW - int(hyp_id))


def unpack_best_key(key: int) -> tuple[int, int]:
    return int(key) >> 32, _LOW - (int(key) & _LOW)


class ShardedIcp:
    """Target-sharded ICP driver: backend has shard_nn / shard_terms / solve / reset."""

    def __init__(self, backend, offset: int, ns: int, device, group=None):
        import torch

        self.b = backend
        self.off = int(offset)
        self.group = group
        self.keys = torch.empty(ns, dtype=torch.int64, device=device)
        self.sums = torch.empty(32, dtype=torch.float64, device=device)

    def iteration(self):
        import torch.distributed as dist

        self.b.shard_nn(self.off, self.keys)
        dist.all_reduce(self.keys, op=dist.ReduceOp.MIN, group=self.group)
        self.b.shard_terms(self.off, self.keys, self.sums)
        dist.all_reduce(self.sums, op=dist.ReduceOp.SUM, group=self.group)
        self.b.solve(self.sums)

    def run(self, init, max_iteration: int):
        """Open3D loop structure: Eval + up to max_iteration updates (max_iteration + 1 passes)."""
        self.b.reset(init)
        for _ in range(max_iteration + 1):
            self.iteration()
        return self.b.result()


class SourceShardedIcp:
    """Source-sharded ICP driver (SURVEY §8(e) "ICP alternative"): rank r owns sources
    [off_r, off_r + n_r) and the whole target.  Per iteration: local NN + local terms →
    all_reduce(sums, SUM) (256 B, the only exchange) → identical solve on every rank, whose
    fitness denominator is the global source count (backend.set_source_total)."""

    def __init__(self, backend, ns_local: int, ns_total: int, device, group=None):
        import torch

        self.b = backend
        self.group = group
        self.b.set_source_total(ns_total)
        self.keys = torch.empty(ns_local, dtype=torch.int64, device=device)
        self.sums = torch.empty(32, dtype=torch.float64, device=device)

    def iteration(self):
        import torch.distributed as dist

        self.b.shard_nn(0, self.keys)
        self.b.shard_terms(0, self.keys, self.sums)
        dist.all_reduce(self.sums, op=dist.ReduceOp.SUM, group=self.group)
        self.b.solve(self.sums)

    def run(self, init, max_iteration: int):
        self.b.reset(init)
        for _ in range(max_iteration + 1):
            self.iteration()
        return self.b.result()


def ransac_sharded(cs, params, group=None):
    """Hypothesis-sharded a4 without early stop: returns (best_count, best_id, T) on every rank.

    ``params.hyp0`` / ``params.max_iter`` must already describe this rank's id range."""
    import torch
    import torch.distributed as dist

    out = cs.run(params)
    gid = params.hyp0 + out.best_index
    key = torch.tensor([best_key(out.best_count, gid)], dtype=torch.int64,
                       device="cuda" if torch.cuda.is_available() else "cpu")
    dist.all_reduce(key, op=dist.ReduceOp.MAX, group=group)
    count, wid = unpack_best_key(int(key.item()))
    T, _ = cs.kabsch3(1, seed=params.seed, hyp0=wid)
    return count, wid, T[0].cpu().numpy()
