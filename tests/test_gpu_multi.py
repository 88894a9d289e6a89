"""GPU tests of the multi-GPU paths on a one-GPU box.

* cfg3's per-rank geometry — 1M sources × 8 target shards of 125k (BASELINE.json cfg3, the
  sharded NN of /root/reference/src/matcher/icp.py:42-48) — emulated with 8 loops on one device:
  the MIN-reduced exchange equals the unsharded NN bit for bit, and 3 iterations end at the
  single-device transform.
* 2 ranks on cuda:0 over gloo with the REAL HIP backend (IcpLoop behind m3d.dist's drivers),
  both ICP shardings and the hypothesis-sharded RANSAC: every rank ends with the single-device
  result.
* The library's own RCCL communicator (m3d_comm_*, m3d_icp_shard_steps, m3d_ransac_run_sharded)
  at world size 1 — RCCL refuses two ranks on one GPU, so this is the plumbing test; the same
  calls run one rank per GPU in bench.py at N > 1.
"""
import os
import socket

import numpy as np
import pytest
from scipy.spatial import cKDTree

import icp_oracle as I
from m3d import _lib, synth
from m3d.core import Cloud, CorrSet, IcpLoop, RansacParams, icp, nn1
from shard_emulation import run_target_shards

pytestmark = pytest.mark.gpu


def test_cfg3_geometry_eight_shards_match_unsharded():
    """1M ↔ 1M, target split into 8 shards of 125k: at every evaluation the reduced claims are
    the unsharded correspondences (grid and brute-force shards agree bit for bit with the
    single-device grid run and with the oracle at the first evaluation); after 3 iterations the
    transform equals the single-device run."""
    import torch

    n = 1_000_000
    src, tgt, nrm, _ = synth.icp_pair(n, n, seed=0)
    bounds = [k * n // 8 for k in range(9)]
    single = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1,
                     max_iteration=3, nn="grid")
    single.reset(np.eye(4))
    ref_corr = []
    for _ in range(4):
        single.step()
        ref_corr.append(single.correspondences().cpu().numpy())
    ref = single.result()
    first = {}

    def check(it, lp, kmin, cmin):
        slot_claims = cmin.cpu().numpy().astype(np.int64)   # indexed by the loop's source slot
        got = np.empty_like(slot_claims)
        got[lp.source_slots().cpu().numpy()] = slot_claims
        got[got == 0x7FFFFFFF] = -1
        np.testing.assert_array_equal(got, ref_corr[it], err_msg=f"evaluation {it}")
        if it == 0:
            first["claims"] = got

    for nn in ("grid", "brute"):
        loops = run_target_shards(src, tgt, nrm, bounds, 3, nn, check_keys=check)
        r = loops[0].result()
        np.testing.assert_allclose(r.transformation, ref.transformation, rtol=0, atol=1e-9)
        assert r.fitness == ref.fitness
        del loops
        torch.cuda.empty_cache()
    # the first evaluation (identity transform) against the oracle's exact fp64 NN
    ref_j, _ = I.nn_exact(cKDTree(tgt), tgt, src, 0.12)
    np.testing.assert_array_equal(first["claims"], ref_j)
    # SPATIAL shards (m3d.dist.spatial_shards: 8 slabs of the longest axis, bench.py's cfg3
    # default): the protocol on the reordered target; its claims mapped back through perm are the
    # unsharded correspondences of the ORIGINAL cloud at every evaluation, the fitness is the
    # single-device run's and the transform too (to the SUM's reassociation of the terms)
    from m3d import dist as D

    perm, sb = D.spatial_shards(tgt, 8)
    assert sorted(perm.tolist()) == list(range(n)) and sb[0] == 0 and sb[-1] == n
    assert (np.diff(sb) > n // 8 - n // 50).all()  # balanced within 2 %

    def check_sp(it, lp, kmin, cmin):
        slot_claims = cmin.cpu().numpy().astype(np.int64)
        got = np.empty_like(slot_claims)
        got[lp.source_slots().cpu().numpy()] = slot_claims
        got = np.where(got == 0x7FFFFFFF, -1, perm[np.minimum(got, n - 1)])
        np.testing.assert_array_equal(got, ref_corr[it], err_msg=f"spatial shards, evaluation {it}")

    for nn in ("grid", "brute"):
        loops = run_target_shards(src, tgt[perm], nrm[perm], sb, 3, nn, check_keys=check_sp)
        r = loops[0].result()
        np.testing.assert_allclose(r.transformation, ref.transformation, rtol=0, atol=1e-9)
        assert r.fitness == ref.fitness
        del loops
        torch.cuda.empty_cache()


# ---------------------------------------------------------------------------- 2 ranks, gloo
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)  # both ranks share the one GPU of the box
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from m3d import dist as D

    comm = D.TorchComm()
    src, tgt, nrm, _ = synth.icp_pair(40_000, 60_001, seed=41)
    out = {}
    # target-sharded: ragged shards, one shared frame
    off, cnt = D.shard_bounds(len(tgt), world, rank)
    sh = Cloud(tgt[off:off + cnt], nrm[off:off + cnt], center=tgt.mean(axis=0))
    for nn in ("brute", "grid"):
        lp = IcpLoop(Cloud(src), sh, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=6, nn=nn)
        r = D.ShardedIcp(lp, off, len(src), "cuda", comm=comm).run(np.eye(4), 6)
        out[f"target_{nn}_T"], out[f"target_{nn}_fit"] = r.transformation, r.fitness
    # source-sharded
    off, cnt = D.shard_bounds(len(src), world, rank)
    lp = IcpLoop(Cloud(src[off:off + cnt]), Cloud(tgt, nrm), 0.12, relative_fitness=-1,
                 relative_rmse=-1, max_iteration=6, nn="brute")
    r = D.SourceShardedIcp(lp, cnt, len(src), "cuda", comm=comm).run(np.eye(4), 6)
    out["source_T"], out["source_fit"] = r.transformation, r.fitness
    # hypothesis-sharded RANSAC (no early stop)
    s, t, c, _ = synth.ransac_pair(20_000, seed=5, noise_ratio=2.0)
    cs = CorrSet(s, t, c)
    H = 3000
    h0, hn = D.shard_bounds(H, world, rank)
    count, wid, T = D.ransac_sharded(cs, RansacParams(max_iter=hn, seed=9, thr=0.45, mode=_lib.SCORE_NORM,
                                                      early_stop=False, hyp0=h0), comm=comm)
    out["ransac"] = np.array([count, wid])
    out["ransac_T"] = T
    np.savez(f"{path}/rank{rank}.npz", **out)
    dist.destroy_process_group()


def test_two_ranks_gloo_real_backend(tmp_path):
    import torch.multiprocessing as mp

    mp.spawn(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (np.load(tmp_path / f"rank{k}.npz") for k in range(2))
    src, tgt, nrm, _ = synth.icp_pair(40_000, 60_001, seed=41)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=6)
    full = icp(Cloud(src), Cloud(tgt, nrm), 0.12, np.eye(4), nn="brute", **kw)
    for key in ("target_brute", "target_grid", "source"):
        np.testing.assert_array_equal(r0[f"{key}_T"], r1[f"{key}_T"])  # identical on every rank
        np.testing.assert_allclose(r0[f"{key}_T"], full.transformation, rtol=0, atol=1e-9)
        assert float(r0[f"{key}_fit"]) == full.fitness
    s, t, c, _ = synth.ransac_pair(20_000, seed=5, noise_ratio=2.0)
    one = CorrSet(s, t, c).run(RansacParams(max_iter=3000, seed=9, thr=0.45, mode=_lib.SCORE_NORM,
                                            early_stop=False))
    for r in (r0, r1):
        assert tuple(r["ransac"]) == (one.best_count, one.best_index)
        np.testing.assert_array_equal(r["ransac_T"], one.transformation)


# ---------------------------------------------------------------------------- library RCCL
@pytest.fixture(scope="module")
def comm1():
    from m3d.comm import LibComm, unique_id

    return LibComm(0, 1, uid=unique_id())


def test_libcomm_allreduce_world1(comm1):
    import torch

    for dt in (torch.int32, torch.int64, torch.float64):
        t = torch.arange(1000, dtype=dt, device="cuda") * 3
        ref = t.clone()
        comm1.min_(t)
        comm1.sum_(t)
        comm1.max_(t)
        assert torch.equal(t, ref)
    with pytest.raises(ValueError):
        comm1.sum_(torch.zeros(4, dtype=torch.float32, device="cuda"))


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_lib_shard_steps_world1_match_single_device(comm1, nn):
    """m3d_icp_shard_steps / m3d_icp_source_shard_steps (exchanges issued by libm3d over RCCL)
    with one rank: the same bits as the fused single-device loop."""
    src, tgt, nrm, _ = synth.icp_pair(50_000, 40_000, seed=43)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=7, nn=nn)
    full = icp(s, t, 0.12, np.eye(4), **kw)
    a = IcpLoop(s, t, 0.12, **kw)
    a.reset(np.eye(4))
    a.shard_steps(comm1, 0, 8)
    b = IcpLoop(s, t, 0.12, **kw)
    b.reset(np.eye(4))
    b.source_shard_steps(comm1, 8)
    for lp in (a, b):
        r = lp.result()
        np.testing.assert_array_equal(r.transformation, full.transformation)
        assert (r.fitness, r.inlier_rmse, r.iterations) == (full.fitness, full.inlier_rmse, 7)


def test_lib_ransac_sharded_world1_matches_run(comm1):
    s, t, c, _ = synth.ransac_pair(30_000, seed=6, noise_ratio=2.0)
    cs = CorrSet(s, t, c)
    p = RansacParams(max_iter=5000, seed=4, thr=0.45, mode=_lib.SCORE_NORM, early_stop=False)
    one = cs.run(p)
    sh = cs.run_sharded(comm1, p)
    assert (sh.best_index, sh.best_count, sh.iterations) == (one.best_index, one.best_count, 5000)
    np.testing.assert_array_equal(sh.transformation, one.transformation)
    with pytest.raises(ValueError):
        cs.run_sharded(comm1, RansacParams(max_iter=10, seed=4, thr=0.45, early_stop=True))


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_split_exchange_driver_matches_single_device(comm1, nn):
    """The half-split target-shard schedule through the Python driver (IcpLoop.shard_nn_range
    pieces, m3d.dist.ShardedIcp(split=True)) over the library communicator: the same bits as the
    fused single-device loop, at a ragged split point and at the default one."""
    from m3d import dist as D

    src, tgt, nrm, _ = synth.icp_pair(30_001, 40_000, seed=44)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=5, nn=nn)
    full = icp(s, t, 0.12, np.eye(4), **kw)
    for split in (True, 12_345):
        lp = IcpLoop(s, t, 0.12, **kw)
        r = D.ShardedIcp(lp, 0, len(src), "cuda", comm=comm1, split=split).run(np.eye(4), 5)
        np.testing.assert_array_equal(r.transformation, full.transformation)
        assert (r.fitness, r.inlier_rmse) == (full.fitness, full.inlier_rmse)


def test_comm_failure_contract_world1():
    """Failure injection (m3d_debug_comm_inject) at world size 1: a failed local RANSAC run
    raises from run_sharded without poisoning the communicator (fail-soft exchange; the next run
    is exact); a failure inside an ICP shard loop aborts the communicator — that call raises, and
    every later call raises M3DCommError."""
    from m3d._lib import M3DCommError, M3DError
    from m3d.comm import LibComm, unique_id

    c = LibComm(0, 1, uid=unique_id())
    s, t, cc, _ = synth.ransac_pair(20_000, seed=6, noise_ratio=1.0)
    cs = CorrSet(s, t, cc)
    p = RansacParams(max_iter=2000, seed=4, thr=0.45, mode=_lib.SCORE_NORM, early_stop=False)
    one = cs.run(p)
    c.inject_failure(1)
    with pytest.raises(M3DError, match="injected"):
        cs.run_sharded(c, p)
    assert not c.poisoned
    sh = cs.run_sharded(c, p)
    assert (sh.best_index, sh.best_count) == (one.best_index, one.best_count)
    np.testing.assert_array_equal(sh.transformation, one.transformation)
    src, tgt, nrm, _ = synth.icp_pair(20_000, 20_000, seed=45)
    lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=4, nn="grid")
    lp.reset(np.eye(4))
    lp.shard_steps(c, 0, 1)
    c.inject_failure(2)
    with pytest.raises(M3DError, match="injected"):
        lp.shard_steps(c, 0, 2)
    assert c.poisoned
    with pytest.raises(M3DCommError):
        lp.shard_steps(c, 0, 1)
    with pytest.raises(M3DCommError):
        cs.run_sharded(c, p)


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_empty_target_shard_and_empty_target(nn):
    """A target shard may be empty (m3d.dist.spatial_shards on heavily duplicated data can leave a
    slab with no point): the emulated 3-shard protocol with an empty middle shard ends at the
    single-device transform and fitness; an empty target on one device gives Open3D's empty result
    (identity, fitness 0)."""
    src, tgt, nrm, _ = synth.icp_pair(20_000, 30_000, seed=7)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=4, nn=nn)
    single = icp(Cloud(src), Cloud(tgt, nrm), 0.12, np.eye(4), **kw)
    loops = run_target_shards(src, tgt, nrm, [0, 15_000, 15_000, 30_000], 4, nn)
    r = loops[0].result()
    np.testing.assert_allclose(r.transformation, single.transformation, rtol=0, atol=1e-9)
    assert r.fitness == single.fitness
    out = icp(Cloud(src), Cloud(np.zeros((0, 3)), np.zeros((0, 3))), 0.12, np.eye(4), **kw)
    assert out.fitness == 0.0 and out.inlier_rmse == 0.0
    np.testing.assert_array_equal(out.transformation, np.eye(4))


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_tiny_targets_nn1_and_icp(nn):
    """Targets of 0, 1 and 2 points: nn1 returns no / the exact fp64 neighbour (icp_oracle.nn_exact),
    and ICP against a 1-point target (a rank-deficient point-to-plane system: the pivoted LDLT
    fallback; Open3D's own answer there is arbitrary) runs to a finite transform."""
    src, tgt, nrm, _ = synth.icp_pair(5_000, 5_000, seed=9)
    q = Cloud(src)
    for k in (0, 1, 2):
        t, n = src[:k] + 0.01, nrm[:k]  # inside the radius of a few sources
        i, d = nn1(q, Cloud(t, n), np.eye(4), 0.3, nn=nn)
        if k == 0:
            assert (i.cpu().numpy() == -1).all()
            continue
        ref_j, _ = I.nn_exact(cKDTree(t), t, src, 0.3)
        np.testing.assert_array_equal(i.cpu().numpy(), ref_j)
        assert (ref_j >= 0).sum() >= 5
    out = icp(Cloud(src), Cloud(src[:1] + 0.01, nrm[:1]), 0.3, np.eye(4), nn=nn, relative_fitness=-1,
              relative_rmse=-1, max_iteration=3)
    assert np.isfinite(out.transformation).all()
