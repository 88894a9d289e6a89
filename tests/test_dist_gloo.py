"""Multi-process (world_size 2 and 3, gloo, CPU) tests of the N>1 protocols in m3d/dist.py.

The driver (ShardedIcp) is the code bench.py runs over RCCL; here its backend is an oracle-backed
CPU implementation of the same calls (shard_nn / shard_claim / shard_terms / solve), so the
protocol — d64 exchange keys, MIN on keys and claims, SUM on terms, ownership of terms,
identical solve on every rank — is checked against the single-process oracle.  The GPU kernels behind the same calls are covered by
tests/test_gpu_icp.py::test_target_sharded_loop_matches_single_device.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from scipy.spatial import cKDTree

import icp_oracle as I
from m3d import dist as D
from m3d import synth


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class OracleShard:
    """CPU stand-in for IcpLoop on one shard: the exact fp64 NN of the oracle, the d64 exchange
    keys and claims of the target-shard protocol, fp64 terms."""

    def __init__(self, src, tgt, nrm, r, max_iteration):
        self.src, self.tgt, self.nrm, self.r = src, tgt, nrm, r
        self.tree = cKDTree(tgt)
        self.max_iteration = max_iteration
        self.ns_total = len(src)

    def set_source_total(self, n):
        self.ns_total = n

    def reset(self, init):
        self.T = np.array(init, np.float64)
        self.pcd = I.initial_points(self.T, self.src)  # RegistrationICP's copy of the source
        self.iters = 0
        self.evals = 0
        self.done = False
        self.fitness = self.rmse = 0.0

    def _local(self, off):
        j, d2 = I.nn_exact(self.tree, self.tgt, self.pcd, self.r)
        return np.where(j >= 0, j + off, -1), d2

    def shard_nn(self, off, dkeys):
        if self.done:
            return
        self.lj, self.ld = self._local(off)
        if dkeys is not None:
            dkeys.copy_(torch.from_numpy(D.pack_d64(self.ld, self.lj >= 0)))

    def shard_nn_range(self, off, q0, q1, dkeys):
        """The split exchange's piece: sources [q0, q1) only (entries outside stay untouched)."""
        if self.done:
            return
        j, d2 = self._local(off)
        if q0 == 0:
            self.lj, self.ld = j.copy(), d2.copy()
        else:
            self.lj[q0:q1], self.ld[q0:q1] = j[q0:q1], d2[q0:q1]
        dkeys[q0:q1].copy_(torch.from_numpy(D.pack_d64(d2[q0:q1], j[q0:q1] >= 0)))

    def shard_claim(self, dmin, claim):
        if self.done:
            return
        own = (self.lj >= 0) & (D.pack_d64(self.ld, self.lj >= 0) == dmin.numpy())
        claim.copy_(torch.from_numpy(np.where(own, self.lj, D.CLAIM_NONE).astype(np.int32)))

    def shard_terms(self, off, dmin, claim, sums):
        if self.done:
            return
        if claim is None:  # source shard: the local winners are the global ones
            idx = self.lj
        else:
            idx = claim.numpy().astype(np.int64)
            idx[idx == D.CLAIM_NONE] = -1
        mine = (idx >= off) & (idx < off + len(self.tgt))
        i = np.nonzero(mine)[0]
        j = idx[mine] - off
        pcd = self.pcd
        out = np.zeros(32)
        if len(i):
            JTJ, JTr, r2 = I.point_to_plane_terms(pcd, self.tgt, self.nrm, np.stack([i, j], 1))
            out[:21] = JTJ[np.triu_indices(6)]
            out[21:27] = JTr
            out[27] = r2
            out[28] = len(i)
            out[29] = np.sum(I.sq_dist(pcd[i], self.tgt[j]))
        sums.copy_(torch.from_numpy(out))

    def solve(self, sums):
        if self.done:
            return
        s = sums.numpy()
        count = s[28]
        self.fitness = count / self.ns_total
        self.rmse = np.sqrt(s[29] / count) if count else 0.0
        self.evals += 1
        if self.iters >= self.max_iteration:
            self.done = True
            return
        if count > 0:
            A = np.zeros((6, 6))
            A[np.triu_indices(6)] = s[:21]
            A = A + np.triu(A, 1).T
            upd = I.vec6_to_matrix(I.ldlt_solve(A, -s[21:27]))
            self.T = I.matmul4(upd, self.T)
            self.pcd = I.transform_points(upd, self.pcd)  # pcd.Transform(update)
        self.iters += 1

    def result(self):
        return self.T, self.fitness, self.rmse, self.iters


def _icp_worker(rank, world, port, path, split=False, spatial=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    src, tgt, nrm, _ = synth.icp_pair(4000, 6001, seed=21)
    off, cnt = D.shard_bounds(len(tgt), world, rank)
    if spatial:  # slabs of the longest axis on the reordered target (bench.py's cfg3 default)
        perm, b = D.spatial_shards(tgt, world)
        tgt, nrm = tgt[perm], nrm[perm]
        off, cnt = int(b[rank]), int(b[rank + 1] - b[rank])
    b = OracleShard(src, tgt[off:off + cnt], nrm[off:off + cnt], 0.12, 8)
    drv = D.ShardedIcp(b, off, len(src), "cpu", split=split)
    assert drv.split == bool(split)
    T, fit, rmse, iters = drv.run(np.eye(4), 8)
    np.savez(f"{path}/rank{rank}.npz", T=T, fit=fit, rmse=rmse, iters=iters)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,split,spatial", [(2, False, False), (2, 1733, False), (3, False, False),
                                                 (3, 1733, False), (2, False, True), (3, 1733, True)])
def test_sharded_icp_protocol_matches_single_process(tmp_path, world, split, spatial):
    """Target shards over gloo equal the single-process oracle, with the exchange in one piece
    and split (the first slot half's MIN in flight — async — while the second half's NN runs,
    m3d_icp_shard_steps' schedule); world 3 gives uneven shards (6001 targets); spatial: the slabs
    of m3d.dist.spatial_shards on the reordered target give the original cloud's transform."""
    mp.spawn(_icp_worker, args=(world, free_port(), str(tmp_path), split, spatial), nprocs=world, join=True)
    src, tgt, nrm, _ = synth.icp_pair(4000, 6001, seed=21)
    ref = I.registration_icp(src, tgt, 0.12, np.eye(4), tgt_normals=nrm, relative_fitness=-1,
                             relative_rmse=-1, max_iteration=8)
    r0 = np.load(tmp_path / "rank0.npz")
    for r in range(1, world):  # every rank holds the identical transform
        np.testing.assert_array_equal(r0["T"], np.load(tmp_path / f"rank{r}.npz")["T"])
    np.testing.assert_allclose(r0["T"], ref["transformation"], atol=1e-10)
    assert abs(float(r0["fit"]) - ref["fitness"]) < 1e-12
    assert int(r0["iters"]) == 8


def _icp_source_worker(rank, world, port, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    src, tgt, nrm, _ = synth.icp_pair(4001, 6000, seed=22)
    off, cnt = D.shard_bounds(len(src), world, rank)
    b = OracleShard(src[off:off + cnt], tgt, nrm, 0.12, 8)
    drv = D.SourceShardedIcp(b, cnt, len(src), "cpu")
    T, fit, rmse, iters = drv.run(np.eye(4), 8)
    np.savez(f"{path}/rank{rank}.npz", T=T, fit=fit, rmse=rmse, iters=iters)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_source_sharded_icp_protocol_matches_single_process(tmp_path, world):
    mp.spawn(_icp_source_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    src, tgt, nrm, _ = synth.icp_pair(4001, 6000, seed=22)
    ref = I.registration_icp(src, tgt, 0.12, np.eye(4), tgt_normals=nrm, relative_fitness=-1,
                             relative_rmse=-1, max_iteration=8)
    r0 = np.load(tmp_path / "rank0.npz")
    for r in range(1, world):
        np.testing.assert_array_equal(r0["T"], np.load(tmp_path / f"rank{r}.npz")["T"])
    np.testing.assert_allclose(r0["T"], ref["transformation"], atol=1e-10)
    assert abs(float(r0["fit"]) - ref["fitness"]) < 1e-12  # global denominator
    assert abs(float(r0["rmse"]) - ref["inlier_rmse"]) < 1e-12
    assert int(r0["iters"]) == 8


def _ransac_worker(rank, world, port, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    counts = np.load(f"{path}/counts.npy")
    off, cnt = D.shard_bounds(len(counts), world, rank)
    local = counts[off:off + cnt]
    li = int(np.argmax(local))  # first max in this shard
    key = torch.tensor([D.best_key(local[li], off + li)], dtype=torch.int64)
    dist.all_reduce(key, op=dist.ReduceOp.MAX)
    np.save(f"{path}/best{rank}.npy", np.array(D.unpack_best_key(int(key.item()))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ransac_best_key_allreduce_first_max(tmp_path, world):
    rng = np.random.default_rng(0)
    counts = rng.integers(0, 50, 1001)
    counts[[100, 700, 900]] = 77  # ties across shards: the lowest id must win
    np.save(tmp_path / "counts.npy", counts)
    mp.spawn(_ransac_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert tuple(np.load(tmp_path / f"best{r}.npy")) == (77, 100)


def test_key_packing_is_order_preserving():
    rng = np.random.default_rng(1)
    d2 = np.sort(rng.random(1000).astype(np.float32) * 10)
    idx = rng.integers(0, 1 << 31, 1000)
    k = D.pack_nn_key(d2, idx)
    assert np.all(np.diff(k[np.argsort(d2, kind="stable")]) >= 0) or np.all(np.diff(k) >= 0)
    dd, ii = D.unpack_nn_key(k)
    np.testing.assert_array_equal(dd, d2)
    np.testing.assert_array_equal(ii, idx)
    assert D.pack_nn_key(np.float32(1.0), -1) == D.KEY_NONE
    # equal distances: lower index wins under MIN
    a = D.pack_nn_key(np.float32(0.5), 7)
    b = D.pack_nn_key(np.float32(0.5), 3)
    assert min(a, b) == b


@pytest.mark.parametrize("n,world", [(10, 3), (100_000, 8), (7, 8)])
def test_shard_bounds_cover(n, world):
    spans = [D.shard_bounds(n, world, r) for r in range(world)]
    assert spans[0][0] == 0
    for (o1, c1), (o2, _) in zip(spans, spans[1:]):
        assert o1 + c1 == o2
    assert sum(c for _, c in spans) == n


class _FailingShard(OracleShard):
    def reset(self, init):
        raise RuntimeError("injected setup failure")


class _RansacStub:
    """CorrSet stand-in for the fail-soft protocol test: a fixed local best, or a failing run."""

    device = "cpu"

    def __init__(self, count, fail):
        self.count, self.fail = count, fail

    def run(self, params):
        if self.fail:
            raise RuntimeError("injected run failure")
        from types import SimpleNamespace
        return SimpleNamespace(best_index=3, best_count=self.count)

    def kabsch3(self, n, seed, hyp0):
        return torch.eye(4, dtype=torch.float64)[None], None


def _failure_worker(rank, world, port, path, what):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    src, tgt, nrm, _ = synth.icp_pair(500, 600, seed=3)
    got = "ok"
    try:
        if what == "setup":
            cls = _FailingShard if rank == 1 else OracleShard
            D.ShardedIcp(cls(src, tgt, nrm, 0.12, 2), 0, len(src), "cpu").run(np.eye(4), 2)
        else:
            from m3d.core import RansacParams
            p = RansacParams(max_iter=10, seed=1, thr=0.45, early_stop=False, hyp0=10 * rank)
            D.ransac_sharded(_RansacStub(5 + rank, fail=rank == 1), p)
    except Exception as e:  # noqa: BLE001
        got = type(e).__name__ + ": " + str(e)
    with open(f"{path}/rank{rank}.txt", "w") as f:
        f.write(got)
    dist.destroy_process_group()


@pytest.mark.parametrize("what", ["setup", "ransac"])
def test_rank_failure_reaches_every_rank(tmp_path, what):
    """A failure on one rank before (ICP setup) or during (the local RANSAC run) the exchange:
    every rank raises from the same call instead of waiting in an all-reduce forever — the
    failing rank its own error, the peer M3DCommError (m3d.dist.agree / the fail-soft RANSAC
    exchange, the protocol of comm.cpp)."""
    mp.spawn(_failure_worker, args=(2, free_port(), str(tmp_path), what), nprocs=2, join=True)
    r0 = (tmp_path / "rank0.txt").read_text()
    r1 = (tmp_path / "rank1.txt").read_text()
    assert r0.startswith("M3DCommError"), r0
    assert r1.startswith("RuntimeError: injected"), r1


def test_spatial_shards_partition_and_keep_duplicates_together():
    """m3d.dist.spatial_shards: a permutation whose slabs are contiguous, balanced, ordered along
    the longest axis, each in increasing original index; equal points never straddle a cut."""
    from m3d import dist as D

    rng = np.random.default_rng(3)
    p = rng.normal(size=(10_001, 3)) * np.array([1.0, 5.0, 0.5])  # longest axis: y
    p[5000:5400] = p[17]  # a block of duplicates
    for world in (1, 2, 3, 8):
        perm, b = D.spatial_shards(p, world)
        assert sorted(perm.tolist()) == list(range(len(p)))
        assert b[0] == 0 and b[-1] == len(p) and len(b) == world + 1
        y = p[perm, 1]
        for k in range(world):
            seg = perm[b[k]:b[k + 1]]
            assert (np.diff(seg) > 0).all()  # original order inside a slab
            if k + 1 < world and b[k + 1] < len(p) and b[k + 1] > b[k]:
                assert y[b[k]:b[k + 1]].max() < y[b[k + 1]:].min()  # slabs ordered, disjoint in y
        slab_of = np.empty(len(p), int)
        for k in range(world):
            slab_of[perm[b[k]:b[k + 1]]] = k
        assert len(set(slab_of[5000:5400].tolist()) | {slab_of[17]}) == 1
        if world == 8:
            assert np.abs(np.diff(b) - len(p) / 8).max() <= 401  # balanced up to the duplicate block
    perm, b = D.spatial_shards(np.zeros((0, 3)), 4)
    assert len(perm) == 0 and list(b) == [0, 0, 0, 0, 0]
