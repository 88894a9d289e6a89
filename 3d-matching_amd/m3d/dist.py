"""Multi-GPU protocols: one process per GPU.

The collectives go through a communicator object with three in-place all-reduces (min_, sum_,
max_).  ``TorchComm`` uses torch.distributed (backend "nccl" = RCCL over xGMI, "gloo" in the CPU
tests); ``m3d.comm.LibComm`` issues RCCL from inside libm3d.so on the library's stream
(m3d_comm_*), with torch.distributed used only for the rendezvous.

* ICP, target-sharded (cfg3; the north-star variant).  Rank r owns target points
  [off_r, off_r + n_r) (points + normals, one shared fp32 frame) and a replica of the source.
  Per iteration (include/m3d.h "Multi-GPU pieces"):
    1. shard NN → each source's fp64 winner on this shard; exchange key = bits(d64) (d64 ≥ +0 so
       the integer order is the fp64 order; KEY_NONE = INT64_MAX = none within the radius);
    2. MIN(dkeys)            — Ns × 8 B (8 MB at 1M);
    3. claim = own winner's global index where its d64 is the global minimum, else INT32_MAX;
    4. MIN(claim)            — Ns × 4 B: exact fp64 ties across shards go to the lowest index, so
       the result is the lexicographic (d64, index) minimum — the single-device answer;
    5. the rank owning each winner accumulates its fp64 estimation terms → 32 doubles;
    6. SUM(sums)             — 256 B;
    7. every rank runs the identical solve/update → identical T everywhere (no broadcast).
* ICP, source-sharded (SURVEY §8(e) "ICP alternative"): rank r owns sources and the whole target;
  per iteration local NN + local terms → SUM(sums) → identical solve (global fitness
  denominator).  The cheaper exchange whenever the target fits one GPU.
* RANSAC, hypothesis-sharded (cfg2 at N>1).  Rank r evaluates hypothesis ids
  [hyp0_r, hyp0_r + H_r) with the counter-based sampler (ids are global, so the union equals the
  single-GPU run); the winner is MAX of (count << 32) | (0xFFFFFFFF − id) — highest count, lowest
  id on ties (the reference's first strict improvement) — and every rank recomputes the winner's
  transform from its id (the sampler is a pure function of the id).

The drivers are backend-agnostic: the GPU backend is ``m3d.core.IcpLoop``; the CPU tests plug in
an oracle-backed backend and run the identical protocol over gloo.

Failure contract (the native loops' in comm.cpp): the drivers' setup (the backend's reset) is
followed by one MAX of a failed flag, so a rank that fails before the first exchange raises its
own error and its peers ``M3DCommError`` — no rank is left inside an all-reduce its peers never
join; ``ransac_sharded`` is fail-soft (a failed local run still joins the exchanges with neutral
values and a failure count).  Source slots: per-source exchange buffers follow the backend's own
source order (``IcpLoop``: its Morton slots, identical on every rank that holds the same source).
"""

from __future__ import annotations

import numpy as np

from ._lib import M3DCommError

KEY_NONE = 0x7FFFFFFFFFFFFFFF
CLAIM_NONE = 0x7FFFFFFF
_LOW = 0xFFFFFFFF


class TorchComm:
    """All-reduces through torch.distributed (the default process group, or `group`)."""

    def __init__(self, group=None):
        self.group = group

    def _ar(self, t, op):
        import torch.distributed as dist

        dist.all_reduce(t, op=op, group=self.group)

    def min_(self, t):
        import torch.distributed as dist

        self._ar(t, dist.ReduceOp.MIN)

    def sum_(self, t):
        import torch.distributed as dist

        self._ar(t, dist.ReduceOp.SUM)

    def max_(self, t):
        import torch.distributed as dist

        self._ar(t, dist.ReduceOp.MAX)

    def min_async(self, t):
        """In-place MIN started in the background; returns a handle with .wait()."""
        import torch.distributed as dist

        return dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group, async_op=True)


def agree(comm, exc, device):
    """Setup agreement: MAX over ranks of "my setup failed".  Re-raises this rank's own exception,
    or M3DCommError when only a peer failed."""
    import torch

    flag = torch.tensor([0 if exc is None else 1], dtype=torch.int32, device=device)
    comm.max_(flag)
    if exc is not None:
        raise exc
    if int(flag.item()) != 0:
        raise M3DCommError("a peer rank failed before the collective loop")


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Balanced contiguous shard [off, off + cnt) of n items for `rank`."""
    base, extra = divmod(n, world)
    off = rank * base + min(rank, extra)
    return off, base + (1 if rank < extra else 0)


def spatial_shards(points, world: int):
    """Spatial target shards (cfg3 at N > 1): slabs along the cloud's longest
    axis, cut at the (k / world)-quantiles of that coordinate.  Returns (perm, bounds): the
    target reordered as points[perm] holds rank r's slab at [bounds[r], bounds[r + 1]), each slab
    in increasing original index.

    Why: index shards of an unordered cloud each span the whole surface, so every rank scans every
    source query against its sparse shard.  A slab's grid covers one region, and a query whose
    search box misses it leaves at once (nnkey.h grid_miss); the keys, claims and terms are the
    protocol's own, so the result is the single-device result ON THE REORDERED CLOUD (tie rule:
    exact fp64 ties go to the lower index of points[perm]).  Cuts fall between distinct coordinate
    values, so equal points (duplicates) always share a slab and keep their original order; a tie
    between distinct points in two slabs is the only case where the original cloud's lowest-index
    rule could pick the other point.  Map a correspondence c of the reordered cloud back with
    perm[c]."""
    p = np.asarray(points, np.float64)
    n = len(p)
    world = int(world)
    if world < 1:
        raise ValueError("world must be >= 1")
    if n == 0 or world == 1:
        return np.arange(n, dtype=np.int64), np.array([0] + [n] * world, dtype=np.int64)
    ext = p.max(axis=0) - p.min(axis=0)
    x = p[:, int(np.argmax(ext))]
    xs = np.sort(x)
    cuts = xs[(np.arange(1, world) * n) // world]  # slab k: cuts[k-1] <= x < cuts[k]
    slab = np.searchsorted(cuts, x, side="right")
    perm = np.argsort(slab, kind="stable").astype(np.int64)  # stable: original order inside a slab
    counts = np.bincount(slab, minlength=world)
    bounds = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return perm, bounds


def pack_nn_key(d2_f32, idx):
    """numpy: (float32 bits << 32) | idx as int64; KEY_NONE where idx < 0 (the scan's key)."""
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


def pack_d64(d2, valid):
    """numpy: the target-shard exchange key, bits of the fp64 d² (KEY_NONE where not valid)."""
    d = np.ascontiguousarray(np.asarray(d2, np.float64))
    return np.where(np.asarray(valid, bool), d.view(np.int64), np.int64(KEY_NONE))


def unpack_d64(keys):
    k = np.ascontiguousarray(np.asarray(keys, np.int64))
    return np.where(k == KEY_NONE, np.inf, k.view(np.float64))


def best_key(count: int, hyp_id: int) -> int:
    return (int(count) << 32) | (_LOW - int(hyp_id))


def unpack_best_key(key: int) -> tuple[int, int]:
    return int(key) >> 32, _LOW - (int(key) & _LOW)


def split_point(ns: int) -> int:
    """The two source halves of the split exchange meet on a 4096-slot boundary (comm.cpp)."""
    return (ns // 2 + 4095) // 4096 * 4096 if ns >= 2 * 4096 else ns


class ShardedIcp:
    """Target-sharded ICP driver: backend has shard_nn / shard_claim / shard_terms / solve /
    reset / result (and shard_nn_range for split=True).

    split=True: the half-split exchange of m3d_icp_shard_steps — the first source half's MIN runs
    (async) while the second half's NN runs; the same keys, so the same result."""

    def __init__(self, backend, offset: int, ns: int, device, comm=None, split: bool = False):
        import torch

        self.b = backend
        self.off = int(offset)
        self.comm = comm or TorchComm()
        self.device = device
        self.ns = int(ns)
        # split: True → split_point(ns); an int → that slot (tests); False → one piece
        h = split_point(self.ns) if split is True else (int(split) if split else self.ns)
        self.h = h if 0 < h < self.ns else self.ns
        self.split = self.h < self.ns
        self.dkeys = torch.empty(ns, dtype=torch.int64, device=device)
        self.claim = torch.empty(ns, dtype=torch.int32, device=device)
        self.sums = torch.empty(32, dtype=torch.float64, device=device)

    def _nn_exchange(self):
        if not self.split:
            self.b.shard_nn(self.off, self.dkeys)
            self.comm.min_(self.dkeys)
            return
        h = self.h
        self.b.shard_nn_range(self.off, 0, h, self.dkeys)
        a = self.dkeys[:h]
        start = getattr(self.comm, "min_async", None)
        work = start(a) if start is not None else None
        if work is None:
            self.comm.min_(a)
        self.b.shard_nn_range(self.off, h, self.ns, self.dkeys)
        if work is not None:
            work.wait()
        self.comm.min_(self.dkeys[h:])

    def iteration(self):
        self._nn_exchange()
        self.b.shard_claim(self.dkeys, self.claim)
        self.comm.min_(self.claim)
        self.b.shard_terms(self.off, self.dkeys, self.claim, self.sums)
        self.comm.sum_(self.sums)
        self.b.solve(self.sums)

    def run(self, init, max_iteration: int):
        """Open3D loop structure: Eval + up to max_iteration updates (max_iteration + 1 passes)."""
        err = None
        try:
            self.b.reset(init)
        except Exception as e:  # noqa: BLE001 - re-raised by agree() after the peers learned of it
            err = e
        agree(self.comm, err, self.device)
        for _ in range(max_iteration + 1):
            self.iteration()
        return self.b.result()


class SourceShardedIcp:
    """Source-sharded ICP driver (SURVEY §8(e) "ICP alternative"): rank r owns sources
    [off_r, off_r + n_r) and the whole target.  Per iteration: local NN + local terms →
    SUM(sums) (256 B, the only exchange) → identical solve on every rank, whose fitness
    denominator is the global source count (backend.set_source_total)."""

    def __init__(self, backend, ns_local: int, ns_total: int, device, comm=None):
        import torch

        self.b = backend
        self.comm = comm or TorchComm()
        self.device = device
        self.b.set_source_total(ns_total)
        self.sums = torch.empty(32, dtype=torch.float64, device=device)

    def iteration(self):
        self.b.shard_nn(0, None)
        self.b.shard_terms(0, None, None, self.sums)
        self.comm.sum_(self.sums)
        self.b.solve(self.sums)

    def run(self, init, max_iteration: int):
        err = None
        try:
            self.b.reset(init)
        except Exception as e:  # noqa: BLE001 - re-raised by agree()
            err = e
        agree(self.comm, err, self.device)
        for _ in range(max_iteration + 1):
            self.iteration()
        return self.b.result()


def ransac_sharded(cs, params, comm=None):
    """Hypothesis-sharded a4 without early stop: returns (best_count, best_id, T) on every rank.

    ``params.hyp0`` / ``params.max_iter`` must already describe this rank's id range.  The
    shards are scored without early stop (each rank would otherwise stop on its own id range and
    the MAX over ranks would not be the single-device loop's best)."""
    import torch

    if params.early_stop:
        raise ValueError("ransac_sharded runs without early stop: set params.early_stop = False")
    comm = comm or TorchComm()
    err, k = None, 0
    try:
        out = cs.run(params)
        if out.best_index >= 0:
            k = best_key(out.best_count, params.hyp0 + out.best_index)
    except Exception as e:  # noqa: BLE001 - fail-soft: join the exchanges, raise after them
        err = e
    key = torch.tensor([k], dtype=torch.int64, device=cs.device)
    comm.max_(key)
    failed = torch.tensor([0 if err is None else 1], dtype=torch.int64, device=cs.device)
    comm.sum_(failed)
    if err is not None:
        raise err
    if int(failed.item()) != 0:
        raise M3DCommError(f"{int(failed.item())} peer rank(s) failed their local run")
    kv = int(key.item())
    if kv == 0:  # no rank found a winner: identity and no index, as comm.cpp's native driver
        return 0, -1, np.eye(4)
    count, wid = unpack_best_key(kv)
    T, _ = cs.kabsch3(1, seed=params.seed, hyp0=wid)
    return count, wid, T[0].cpu().numpy()
