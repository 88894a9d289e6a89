"""GPU parity for the ICP half: the HIP NN + point-to-plane/point-to-point loop vs the CPU oracle
(Open3D 0.19 semantics restated; parity against Open3D itself is unpinned — SURVEY.md §8(c)).

NN contract (nnkey.h, icp_oracle.nn_exact): for every source point the exact lexicographic
(d64, index) minimum over the targets with d64 < r², d64 the fp64 d² of the fp64 transformed
point — checked BIT FOR BIT (indices and d²) against the oracle, for brute force and the grid.
ICP loops follow RegistrationICP's incremental points (pcd.Transform(init) unless init
isIdentity(), then pcd.Transform(update) per iteration).  The device reduces the fp64 terms in a
different order than numpy, so a loop's updates differ from the oracle's by rounding (~1e-15);
per evaluation the device's points are checked bit for bit against its previous points moved by
its own update, and its correspondence set against the oracle's exact NN of those points
(_check_evaluations); whole runs within 1e-9 / fitness exactly where stated.
"""
import numpy as np
import pytest
from scipy.spatial import cKDTree

import icp_oracle as I
from m3d import _lib, synth
from m3d.core import Cloud, IcpLoop, icp, nn1
from shard_emulation import run_target_shards, shard_step

pytestmark = pytest.mark.gpu


def check_nn(src, tgt, T, r, idx, d2):
    """Device NN == the oracle's exact fp64 NN at transform T, bit for bit."""
    ref_j, ref_d2 = I.nn_exact(cKDTree(tgt), tgt, I.transform_points(T, src), r)
    np.testing.assert_array_equal(idx, ref_j)
    np.testing.assert_array_equal(d2, ref_d2)


@pytest.mark.parametrize("nn", ["brute", "grid"])
@pytest.mark.parametrize("ns,nt", [(1, 1), (5, 3000), (1000, 1000), (20000, 30011), (100_000, 100_000)])
def test_nn1_matches_kdtree(ns, nt, nn):
    tgt, _ = synth.surface_points(nt, seed=1)
    src, _ = synth.surface_points(ns, seed=2)
    T = synth.random_rigid(3, rot_range=0.02, trans_range=0.05)
    r = 0.3 if nt < 5000 else 0.12
    idx, d2 = nn1(Cloud(src), Cloud(tgt), T, r, nn=nn)
    check_nn(src, tgt, T, r, idx.cpu().numpy(), d2.cpu().numpy())


def _grid_cases():
    rng = np.random.default_rng(21)
    sph, _ = synth.surface_points(30000, seed=3)
    plane = np.c_[rng.uniform(-3, 3, (20000, 2)), np.zeros(20000)]  # zero extent along z
    line = np.c_[np.linspace(-1, 1, 5000), np.zeros((5000, 2))]
    dup = np.repeat(rng.normal(size=(50, 3)), 40, axis=0)  # exact duplicates → index ties
    wide = rng.uniform(-5e3, 5e3, (40000, 3))  # cell-count cap (r ≪ extent)
    offset = sph + np.array([1e5, -2e5, 3e4])  # large absolute coordinates
    # a few far outliers make the fp16-scaled queries overflow: the MFMA kernel's exact scan
    outl = sph[::3].copy()
    outl[::500] += 2e4
    # a vertex fan: 3000 targets within 0.004 of one surface point (≥ 256 in one cell at r: the
    # loop defers the queries near it to grid_nn_heavy_kernel)
    fan = np.vstack([sph, sph[7] + rng.normal(scale=0.002, size=(3000, 3))])
    # a dense volume (≈ 100 points per r-cell: the loop's cells are r/4, so an unseeded query's
    # box is 9 cells wide and the scan takes its half-cell first pass, grid.hip M3D_SCAN_PHASE1)
    cube = rng.uniform(-0.5, 0.5, (60000, 3))
    return {
        "dense_volume": (cube[::3] + 1e-3, cube, 0.12),
        "dense_cluster": (np.vstack([sph[::3] * 1.001, sph[7] + rng.normal(scale=0.03, size=(2000, 3))]), fan, 0.12),
        "sphere": (sph[::3] * 1.002, sph, 0.12),
        "sphere_big_r": (sph[::7], sph, 50.0),  # radius larger than the cloud
        "sphere_tiny_r": (sph[::5] + 1e-4, sph, 1e-3),
        "plane": (plane[::4] + [0, 0, 0.01], plane, 0.05),
        "line": (line + [0.0001, 0.02, 0], line, 0.03),
        "duplicates": (dup + 1e-3, dup, 0.5),
        "wide": (wide[::2] + 0.3, wide, 0.01),
        "offset": (offset[::3] * 1.0000001, offset, 0.12),
        "far": (sph[:100] + 1e3, sph, 0.12),
        "outliers": (outl * 1.002, sph, 0.12),
        "single_target": (sph[:500], sph[:1], 10.0),
    }


@pytest.mark.parametrize("case", list(_grid_cases()))
def test_grid_nn_identical_to_brute_force(case):
    """Grid and brute-force NN return bit-identical (index, d²) for every query, equal to the
    oracle's exact fp64 NN (exact duplicates: lowest index)."""
    src, tgt, r = _grid_cases()[case]
    T = synth.random_rigid(17, rot_range=0.01, trans_range=0.01)
    s, t = Cloud(src), Cloud(tgt)
    ib, db = nn1(s, t, T, r, nn="brute")
    ig, dg = nn1(s, t, T, r, nn="grid")
    np.testing.assert_array_equal(ig.cpu().numpy(), ib.cpu().numpy())
    np.testing.assert_array_equal(dg.cpu().numpy(), db.cpu().numpy())
    check_nn(src, tgt, T, r, ig.cpu().numpy(), dg.cpu().numpy())


@pytest.mark.parametrize("estimation", [_lib.EST_POINT_TO_PLANE, _lib.EST_POINT_TO_POINT])
def test_icp_grid_identical_to_brute_force(estimation):
    src, tgt, nrm, _ = synth.icp_pair(50000, 60000, seed=19)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=12, estimation=estimation)
    a = icp(s, t, 0.12, np.eye(4), nn="brute", **kw)
    b = icp(s, t, 0.12, np.eye(4), nn="grid", **kw)
    np.testing.assert_array_equal(b.transformation, a.transformation)
    assert (b.fitness, b.inlier_rmse, b.iterations) == (a.fitness, a.inlier_rmse, a.iterations)
    np.testing.assert_array_equal(b.correspondence_set, a.correspondence_set)


def test_icp_with_far_outliers_grid_identical_to_brute_force():
    """Far source outliers switch the brute-force NN to the MFMA kernel's exact in-kernel scan
    (operands beyond fp16); the fused loop must still match the grid path bit for bit."""
    src, tgt, nrm, _ = synth.icp_pair(30000, 40000, seed=29)
    src = src.copy()
    src[::1000] += 3e4
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=4)
    a = icp(s, t, 0.12, np.eye(4), nn="brute", **kw)
    b = icp(s, t, 0.12, np.eye(4), nn="grid", **kw)
    np.testing.assert_array_equal(a.transformation, b.transformation)
    assert (a.fitness, a.inlier_rmse) == (b.fitness, b.inlier_rmse) and a.fitness > 0.5


@pytest.mark.parametrize("drop", ["half", "slab"])
def test_partial_overlap_grid_identical_to_brute_force(drop):
    """Partial overlaps — half of the target cut away (the grid's box then excludes the
    unpartnered sources: the scan's far exit) or a slab from its middle (unpartnered sources
    inside the grid, full radius boxes that find nothing): the grid loop keeps the brute-force
    loop's bits at every iteration count."""
    src, tgt, nrm, _ = synth.icp_pair(30000, 40000, seed=31)
    lo, hi = np.quantile(tgt[:, 1], [0.3, 0.7])
    keep = tgt[:, 0] < np.median(tgt[:, 0]) if drop == "half" else (tgt[:, 1] < lo) | (tgt[:, 1] > hi)
    s, t = Cloud(src), Cloud(tgt[keep], nrm[keep])
    for mi in (1, 3, 8, 25):
        kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=mi)
        a = icp(s, t, 0.12, np.eye(4), nn="brute", **kw)
        b = icp(s, t, 0.12, np.eye(4), nn="grid", **kw)
        np.testing.assert_array_equal(b.transformation, a.transformation)
        assert (b.fitness, b.inlier_rmse, b.iterations) == (a.fitness, a.inlier_rmse, a.iterations)
        np.testing.assert_array_equal(b.correspondence_set, a.correspondence_set)
        assert 0.2 < a.fitness < 0.9, a.fitness  # a real partial overlap


def test_nn1_exact_ties_pick_lowest_index():
    tgt = np.array([[1.0, 0, 0], [-1.0, 0, 0], [0, 1.0, 0], [1.0, 0, 0]])
    src = np.zeros((3, 3))
    idx, d2 = nn1(Cloud(src), Cloud(tgt), np.eye(4), 2.0)
    assert idx.cpu().numpy().tolist() == [0, 0, 0]
    idx, _ = nn1(Cloud(src), Cloud(tgt), np.eye(4), 1.0)  # strict d² < r²: none
    assert idx.cpu().numpy().tolist() == [-1, -1, -1]


@pytest.mark.parametrize("estimation", ["point_to_plane", "point_to_point"])
def test_icp_matches_oracle(estimation):
    src, tgt, nrm, T_true = synth.icp_pair(20000, seed=5)
    if estimation == "point_to_point":
        src = synth.apply(np.linalg.inv(T_true), tgt)[::2]
    ref = I.registration_icp(src, tgt, 0.12, init=np.eye(4), tgt_normals=nrm, estimation=estimation,
                             max_iteration=30)
    est = _lib.EST_POINT_TO_PLANE if estimation == "point_to_plane" else _lib.EST_POINT_TO_POINT
    out = icp(Cloud(src), Cloud(tgt, nrm if est == _lib.EST_POINT_TO_PLANE else None), 0.12,
              np.eye(4), estimation=est, max_iteration=30)
    np.testing.assert_allclose(out.transformation[:3, :3], ref["transformation"][:3, :3], atol=1e-6)
    np.testing.assert_allclose(out.transformation[:3, 3], ref["transformation"][:3, 3], atol=1e-5)
    assert abs(out.fitness - ref["fitness"]) < 2e-4
    assert abs(out.inlier_rmse - ref["inlier_rmse"]) < 1e-4 * ref["inlier_rmse"] + 1e-9
    assert abs(out.iterations - ref["iterations"]) <= 1


def test_refine_registration_api_recovers_pose():
    from matcher.icp import refine_registration
    from ply import Ply

    src_pts, tgt_pts, nrm, T_true = synth.icp_pair(100_000, seed=7)
    src = Ply.from_arrays(src_pts)
    tgt = Ply.from_arrays(tgt_pts, normals=nrm)
    res = refine_registration(src, tgt, np.eye(4), 0.3)
    assert res.fitness > 0.95
    np.testing.assert_allclose(res.transformation, T_true, atol=5e-4)
    assert len(res.correspondence_set) == round(res.fitness * len(src_pts))


def test_fixed_iterations_and_missing_normals():
    src, tgt, nrm, _ = synth.icp_pair(5000, seed=9)
    out = icp(Cloud(src), Cloud(tgt, nrm), 0.12, np.eye(4), relative_fitness=-1, relative_rmse=-1,
              max_iteration=7)
    assert out.iterations == 7 and not out.converged
    from matcher.icp import registration_icp

    with pytest.raises(ValueError):
        registration_icp(src, tgt, 0.12, np.eye(4), "point_to_plane")
    with pytest.raises(ValueError):
        registration_icp(src, tgt, 0.0)


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_empty_source_icp_and_nn1(nn):
    """An empty source cloud (round-3 ADVICE: the Morton-slot copy must accept n = 0): nn1 returns
    empty arrays, ICP returns Open3D's empty result (identity, fitness 0, no correspondences) for
    both NN methods, and the same cloud objects keep working for a non-empty call afterwards."""
    tgt, nrm = synth.surface_points(3000, seed=2)
    empty = Cloud(np.zeros((0, 3)))
    t = Cloud(tgt, nrm)
    idx, d2 = nn1(empty, t, np.eye(4), 0.3, nn=nn)
    assert idx.numel() == 0 and d2.numel() == 0
    out = icp(empty, t, 0.12, np.eye(4), nn=nn, max_iteration=5)
    assert out.fitness == 0.0 and out.inlier_rmse == 0.0
    np.testing.assert_array_equal(out.transformation, np.eye(4))
    assert len(out.correspondence_set) == 0
    src, _ = synth.surface_points(500, seed=3)
    idx, _ = nn1(Cloud(src), t, np.eye(4), 0.3, nn=nn)
    assert idx.numel() == 500
    # the step-wise loop on the empty source: no points, the identity update, T = init
    init = synth.random_rigid(3, rot_range=0.01, trans_range=0.01)
    lp = IcpLoop(empty, t, 0.12, max_iteration=3, nn=nn)
    lp.reset(init)
    lp.steps(4)
    r = lp.result()
    assert lp.points().shape == (0, 3)
    np.testing.assert_array_equal(r.update, np.eye(4))
    np.testing.assert_array_equal(r.transformation, init)
    assert r.fitness == 0.0


def test_icp_result_update_and_points_api():
    """IcpOutcome.update is the identity after a reset and then the last update a solve produced:
    T_k = update_k · T_(k−1) (to rounding), the one-shot icp() reports the same update as the loop,
    and the loop's points before any evaluation are the source itself (init·source for a
    non-identity init), in the caller's order."""
    src, tgt, nrm, _ = synth.icp_pair(20_000, 20_000, seed=12)
    s, t = Cloud(src), Cloud(tgt, nrm)
    lp = IcpLoop(s, t, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=5, nn="grid")
    lp.reset(np.eye(4))
    np.testing.assert_array_equal(lp.result().update, np.eye(4))
    np.testing.assert_array_equal(lp.points().cpu().numpy(), src)  # before the first evaluation
    # a non-identity init: RegistrationICP's pcd is init·source before the first evaluation
    # (pcd.Transform(init), Eigen's non-FMA order) — bit for bit
    init = synth.random_rigid(3, rot_range=0.02, trans_range=0.02)
    lp.reset(init)
    R, tt = init[:3, :3], init[:3, 3]
    exp = ((src[:, 0:1] * R[:, 0] + src[:, 1:2] * R[:, 1]) + src[:, 2:3] * R[:, 2]) + tt
    np.testing.assert_array_equal(lp.points().cpu().numpy(), exp)
    lp.reset(np.eye(4))
    prev = lp.result().transformation
    for _ in range(5):
        lp.step()
        r = lp.result()
        np.testing.assert_allclose(r.transformation, r.update @ prev, rtol=0, atol=1e-14)
        prev = r.transformation
    lp.step()  # the 6th evaluation ends the run (max_iteration): no update, T and update kept
    r = lp.result()
    assert r.iterations == 5
    np.testing.assert_array_equal(r.transformation, prev)
    out = icp(s, t, 0.12, np.eye(4), relative_fitness=-1, relative_rmse=-1, max_iteration=5)
    np.testing.assert_array_equal(out.update, lp.result().update)
    np.testing.assert_array_equal(out.transformation, lp.result().transformation)


def test_morton_copies_stay_bounded_per_cloud():
    """nn1 with many different radii on one cloud pair (round-3 ADVICE): the per-cloud Morton
    source copies are capped (api.cpp kMortonKeep), results stay exact."""
    tgt, _ = synth.surface_points(4000, seed=4)
    src, _ = synth.surface_points(3000, seed=5)
    s, t = Cloud(src), Cloud(tgt)
    T = synth.random_rigid(6, rot_range=0.02, trans_range=0.05)
    for r in (0.1, 0.12, 0.15, 0.2, 0.25, 0.3, 0.35, 0.4):
        idx, d2 = nn1(s, t, T, r, nn="grid")
        check_nn(src, tgt, T, r, idx.cpu().numpy(), d2.cpu().numpy())


def test_no_overlap_gives_identity_and_zero_fitness():
    src, _ = synth.surface_points(2000, seed=1)
    tgt, nrm = synth.surface_points(2000, seed=2)
    out = icp(Cloud(src + 100.0), Cloud(tgt, nrm), 0.12, np.eye(4), max_iteration=5)
    assert out.fitness == 0.0 and out.inlier_rmse == 0.0
    np.testing.assert_array_equal(out.transformation, np.eye(4))


def test_step_loop_matches_run():
    src, tgt, nrm, _ = synth.icp_pair(30000, seed=11)
    s, t = Cloud(src), Cloud(tgt, nrm)
    full = icp(s, t, 0.12, np.eye(4), relative_fitness=-1, relative_rmse=-1, max_iteration=10)
    loop = IcpLoop(s, t, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=10)
    loop.reset(np.eye(4))
    for _ in range(11):
        loop.step()
    r = loop.result()
    np.testing.assert_array_equal(r.transformation, full.transformation)
    assert r.fitness == full.fitness and r.iterations == 10
    loop.reset(np.eye(4))
    loop.steps(13)  # native loop; the two extra iterations are device no-ops after the last
    r2 = loop.result()
    np.testing.assert_array_equal(r2.transformation, full.transformation)
    assert r2.fitness == full.fitness and r2.iterations == 10


@pytest.mark.parametrize("nn", ["brute", "grid"])
@pytest.mark.parametrize("max_iteration", [0, 1, 3, 7, 30])
def test_run_chunks_match_stepped_loop(nn, max_iteration):
    """m3d_icp_run enqueues its evaluations in chunks of 4, 8, 16, … and stops enqueueing once the
    state says done: converging (Open3D criteria) and non-converging runs give the loop's bits,
    iteration count and correspondence set."""
    import torch

    src, tgt, nrm, _ = synth.icp_pair(20000, seed=12)
    s, t = Cloud(src), Cloud(tgt, nrm)
    for crit in ((1e-6, 1e-6), (-1.0, -1.0)):
        full = icp(s, t, 0.12, np.eye(4), relative_fitness=crit[0], relative_rmse=crit[1],
                   max_iteration=max_iteration, nn=nn)
        loop = IcpLoop(s, t, 0.12, relative_fitness=crit[0], relative_rmse=crit[1],
                       max_iteration=max_iteration, nn=nn)
        loop.reset(np.eye(4))
        for _ in range(max_iteration + 1):
            loop.step()
        r = loop.result()
        np.testing.assert_array_equal(r.transformation, full.transformation)
        assert (r.fitness, r.iterations, r.converged) == (full.fitness, full.iterations, full.converged)
        jj = loop.correspondences().cpu().numpy()
        i = np.flatnonzero(jj >= 0)
        np.testing.assert_array_equal(full.correspondence_set, np.stack([i, jj[i]], 1))


@pytest.mark.parametrize("n", [0, 1, 5, 100_000, 3_000_000])
def test_host_cloud_equals_device_cloud(n):
    """m3d_cloud_create_host (the staged upload: 256 KB chunks, rounds past the 64 MB staging cap
    at 3M points with normals) builds the cloud m3d_cloud_create builds from device arrays: the
    same NN (indices and d²) and, with normals, the same ICP bits."""
    import torch

    rng = np.random.default_rng(n)
    pts = rng.normal(size=(n, 3)) * 3.0
    nrm = rng.normal(size=(n, 3))
    q = pts[: min(n, 20000)] + rng.normal(size=(min(n, 20000), 3)) * 0.01
    a_t, a_n = Cloud(pts, nrm), Cloud(torch.from_numpy(pts).cuda(), torch.from_numpy(nrm).cuda())
    assert a_t.n == a_n.n == n
    s = Cloud(q)
    T = synth.random_rigid(5, rot_range=0.001, trans_range=0.001)
    i1, d1 = nn1(s, a_t, T, 0.05, nn="grid")
    i2, d2 = nn1(s, a_n, T, 0.05, nn="grid")
    np.testing.assert_array_equal(i1.cpu().numpy(), i2.cpu().numpy())
    np.testing.assert_array_equal(d1.cpu().numpy(), d2.cpu().numpy())
    if n >= 5:
        r1 = icp(s, a_t, 0.05, np.eye(4), max_iteration=3)
        r2 = icp(s, a_n, 0.05, np.eye(4), max_iteration=3)
        np.testing.assert_array_equal(r1.transformation, r2.transformation)
        np.testing.assert_array_equal(r1.correspondence_set, r2.correspondence_set)


@pytest.mark.parametrize("n", [0, 1, 1023, 1024, 1025, 4096, 100_000, 3_000_001])
def test_corr_pairs_compaction(n):
    """m3d_corr_pairs: the (i, v[i]) pairs for v[i] >= 0 in increasing i, against numpy, at chunk
    edges, with none / all / a random half valid."""
    import torch

    from m3d.core import context, corr_pairs

    rng = np.random.default_rng(n)
    ctx = context()
    for frac in (0.0, 1.0, 0.5):
        v = np.where(rng.random(n) < frac, rng.integers(0, 1 << 30, n), -1).astype(np.int32)
        got = corr_pairs(ctx, torch.from_numpy(v).cuda(), n)
        i = np.flatnonzero(v >= 0)
        assert got.dtype == np.int32 and got.shape == (len(i), 2)
        np.testing.assert_array_equal(got, np.stack([i, v[i]], 1).astype(np.int32))


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_graph_replay_matches_enqueued_steps(nn):
    """m3d_icp_steps captures an n-step sequence into a HIP graph the second time it is requested
    (one graph per keys-clean state on entry) and replays it; it must compute what the steps
    enqueued one by one compute, bit for bit: plain first calls, the capturing call, replays,
    steps without a reset in between, another n, and with kernel profiling on (plain)."""
    from m3d.core import context

    src, tgt, nrm, _ = synth.icp_pair(30000, seed=13)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=80, nn=nn)
    a = IcpLoop(s, t, 0.12, **kw)
    b = IcpLoop(s, t, 0.12, **kw)

    def state(lp):
        r = lp.result()
        return r.transformation, r.fitness, r.inlier_rmse, r.iterations, lp.correspondences().cpu().numpy()

    def same(x, y):
        np.testing.assert_array_equal(x[0], y[0])
        assert x[1:4] == y[1:4]
        np.testing.assert_array_equal(x[4], y[4])

    def both(n):
        a.steps(n)
        for _ in range(n):
            b.step()
        same(state(a), state(b))

    T0 = synth.random_rigid(5, rot_range=0.02, trans_range=0.03)
    for rep in range(3):
        for lp in (a, b):
            lp.reset(T0 if rep != 1 else np.eye(4))
        both(6)
        both(6)  # without a reset: the keys-clean entry state (brute force) or the same one (grid)
    both(3)
    both(3)
    both(3)
    ctx = context()
    ctx.profile(True)
    a.steps(4)
    ctx.profile(False)
    for _ in range(4):
        b.step()
    same(state(a), state(b))


@pytest.mark.parametrize("estimation", [_lib.EST_POINT_TO_PLANE, _lib.EST_POINT_TO_POINT])
@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_fused_tail_matches_separate_kernels(nn, estimation):
    """m3d_icp_step fuses terms → reduce → solve into one launch (last-block ticket, ~400 blocks
    spread over all XCDs) and decides the fp64 winners inside the terms pass; the separate
    shard_nn / shard_claim / shard_terms / solve launches (keyinit-seeded scan, winners decided
    by shard_winner_kernel) must give the same bits."""
    import torch

    src, tgt, nrm, _ = synth.icp_pair(100000, 90000, seed=23)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=8, estimation=estimation, nn=nn)
    full = icp(s, t, 0.12, np.eye(4), **kw)
    lp = IcpLoop(s, t, 0.12, **kw)
    lp.reset(np.eye(4))
    sm = torch.empty(32, dtype=torch.float64, device="cuda")
    for _ in range(9):
        shard_step(lp, 0, len(src), sm)
    r = lp.result()
    np.testing.assert_array_equal(r.transformation, full.transformation)
    assert (r.fitness, r.inlier_rmse, r.iterations) == (full.fitness, full.inlier_rmse, 8)


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_mixed_fused_and_separate_steps(nn):
    """The fused m3d_icp_step hands the keys back as kKeyNone and its next brute-force scan seeds
    itself; separate shard_nn / shard_terms / solve calls (keyinit path) interleaved with fused
    steps on the same loop must give the bits of the all-separate loop."""
    import torch

    src, tgt, nrm, _ = synth.icp_pair(60000, 50000, seed=31)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=9,
              estimation=_lib.EST_POINT_TO_PLANE, nn=nn)
    sm = torch.empty(32, dtype=torch.float64, device="cuda")

    def separate(lp, n):
        for _ in range(n):
            shard_step(lp, 0, len(src), sm)

    ref = IcpLoop(s, t, 0.12, **kw)
    ref.reset(np.eye(4))
    separate(ref, 10)
    r_ref = ref.result()
    mix = IcpLoop(s, t, 0.12, **kw)
    for _ in range(2):  # the second pass starts from keys a finished fused run left behind
        mix.reset(np.eye(4))
        mix.steps(3)
        separate(mix, 2)
        mix.steps(3)
        separate(mix, 1)
        mix.steps(1)
        r = mix.result()
        np.testing.assert_array_equal(r.transformation, r_ref.transformation)
        assert (r.fitness, r.inlier_rmse, r.iterations) == (r_ref.fitness, r_ref.inlier_rmse, 9)


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_icp_rank_deficient_plane_matches_oracle(nn):
    """A planar target with exact (0, 0, 1) normals: the point-to-plane rows are
    (p_y, −p_x, 0, 0, 0, 1), so the 6×6 system has exact zero rows and columns for rz, tx and ty —
    the LDLT pivoting moves them last and zero pivots give zero components (Eigen::LDLT, as
    linalg.h ldlt6_solve and the oracle restate).  In-plane motion stays unobserved."""
    rng = np.random.default_rng(7)
    n = 20000
    tgt = np.zeros((n, 3))
    tgt[:, :2] = rng.uniform(-1, 1, (n, 2))
    nrm = np.tile([0.0, 0.0, 1.0], (n, 1))
    c, s_ = np.cos(0.02), np.sin(0.02)
    T = np.eye(4)
    T[:3, :3] = [[1, 0, 0], [0, c, -s_], [0, s_, c]]
    T[:3, 3] = [0.0, 0.0, 0.03]
    src = synth.apply(np.linalg.inv(T), tgt[rng.permutation(n)[: n // 2]]) + rng.normal(0, 1e-3, (n // 2, 3))
    ref = I.registration_icp(src, tgt, 0.1, init=np.eye(4), tgt_normals=nrm,
                             estimation="point_to_plane", max_iteration=20)
    out = icp(Cloud(src), Cloud(tgt, nrm), 0.1, np.eye(4), estimation=_lib.EST_POINT_TO_PLANE,
              max_iteration=20, nn=nn)
    assert np.all(np.isfinite(out.transformation))
    np.testing.assert_allclose(out.transformation[:3, :3], ref["transformation"][:3, :3], atol=1e-6)
    np.testing.assert_allclose(out.transformation[:3, 3], ref["transformation"][:3, 3], atol=1e-5)
    assert abs(out.fitness - ref["fitness"]) < 2e-4
    # the aligned source lies on the plane again
    aligned = synth.apply(out.transformation, src)
    assert np.abs(aligned[:, 2]).mean() < 5e-3


@pytest.mark.parametrize("keys_inside", [False, True])
@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_source_sharded_loop_matches_single_device(nn, keys_inside):
    """The source-sharded protocol (local NN + terms, SUM of the 32 term slots, global fitness
    denominator) emulated with three source shards on one device.  keys_inside: no key buffer
    passed (bench.py's form) — the keys stay in the loop, the terms hand them back as kKeyNone
    and the next brute-force scan seeds itself."""
    import torch

    src, tgt, nrm, _ = synth.icp_pair(30001, 20000, seed=14)
    t = Cloud(tgt, nrm)
    full = icp(Cloud(src), t, 0.12, np.eye(4), relative_fitness=-1, relative_rmse=-1,
               max_iteration=6, nn="brute")
    bounds = [0, 9000, 21000, 30001]
    loops = [IcpLoop(Cloud(src[a:b]), t, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=6,
                     nn=nn) for a, b in zip(bounds[:-1], bounds[1:])]
    for lp in loops:
        lp.set_source_total(len(src))
        lp.reset(np.eye(4))
    for _ in range(7):
        sums = []
        for lp in loops:
            sm = torch.empty(32, dtype=torch.float64, device="cuda")
            if keys_inside:
                lp.shard_nn(0, None)
                lp.shard_terms(0, None, None, sm)
            else:  # the target-shard calls with the whole target as the one shard
                dk = torch.empty(lp.src.n, dtype=torch.int64, device="cuda")
                cl = torch.empty(lp.src.n, dtype=torch.int32, device="cuda")
                lp.shard_nn(0, dk)
                lp.shard_claim(dk, cl)
                lp.shard_terms(0, dk, cl, sm)
            sums.append(sm)
        tot = torch.stack(sums).sum(dim=0)
        for lp in loops:
            lp.solve(tot)
    r = loops[0].result()
    np.testing.assert_allclose(r.transformation, full.transformation, atol=1e-9)
    assert abs(r.fitness - full.fitness) < 1e-12
    for lp in loops[1:]:
        np.testing.assert_array_equal(lp.result().transformation, r.transformation)


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_target_sharded_loop_matches_single_device(nn):
    """Three ragged target shards on one device: the reduced claims are the single-device
    correspondences at every iteration, and the run ends at the single-device transform."""
    src, tgt, nrm, _ = synth.icp_pair(20000, 30000, seed=13)
    full = icp(Cloud(src), Cloud(tgt, nrm), 0.12, np.eye(4), relative_fitness=-1, relative_rmse=-1,
               max_iteration=6, nn="brute")
    loops = run_target_shards(src, tgt, nrm, [0, 7000, 19001, 30000], 6, nn)
    r = loops[0].result()
    np.testing.assert_allclose(r.transformation, full.transformation, atol=1e-9)
    assert abs(r.fitness - full.fitness) < 1e-12
    for lp in loops[1:]:
        np.testing.assert_array_equal(lp.result().transformation, r.transformation)


def test_target_shard_duplicates_across_shards_lowest_index():
    """Exact fp64 ties between shards (the same target point stored on two shards): the claim
    exchange gives the lowest global index, as the single-device NN does."""
    import torch

    tgt, nrm = synth.surface_points(4000, seed=3)
    tgt = np.concatenate([tgt, tgt])  # index j and j + 4000 are the same point
    nrm = np.concatenate([nrm, nrm])
    src = tgt[:4000:3] + 1e-3
    seen = {}

    def keep(it, lp, kmin, cmin):  # claims are indexed by the loop's source slot
        got = np.empty(len(src), np.int64)
        got[lp.source_slots().cpu().numpy()] = cmin.cpu().numpy()
        seen[it] = got

    run_target_shards(src, tgt, nrm, [0, 2500, 8000], 0, "grid", r=0.3, check_keys=keep)
    ref_j, _ = I.nn_exact(cKDTree(tgt), tgt, src, 0.3)
    got = seen[0].astype(np.int64)
    got[got == 0x7FFFFFFF] = -1
    np.testing.assert_array_equal(got, ref_j)
    assert np.all(ref_j < 4000)


def _check_evaluations(lp, src, tgt, init, n_evals, r=0.12, keep=None):
    """Step lp n_evals times from reset(init).  At every evaluation the loop's points are
    RegistrationICP's incremental pcd, BIT FOR BIT: the source (init applied unless it
    isIdentity()) for the first, the previous points moved by the update the device produced
    (pcd.Transform(update)) after that; its correspondence set is the oracle's exact fp64 NN of
    those points, bit for bit."""
    tree = cKDTree(tgt)
    lp.reset(init)
    want = I.initial_points(init, src)
    for it in range(n_evals):
        lp.step()
        pts = lp.points().cpu().numpy()
        np.testing.assert_array_equal(pts, want, err_msg=f"points, evaluation {it}")
        ref_j, _ = I.nn_exact(tree, tgt, pts, r)
        corr = lp.correspondences().cpu().numpy()
        np.testing.assert_array_equal(corr, ref_j, err_msg=f"evaluation {it}")
        if keep is not None:
            keep.append((pts, corr))
        want = I.transform_points(lp.result().update, pts)
    return lp.result()


def _against_oracle_run(dev, src, tgt, nrm, r, n_iter, **kw):
    """The oracle's own incremental run beside the device's evaluations (dev: [(points, corr)]):
    per evaluation the number of correspondences that differ and the largest point difference
    (the two runs' updates differ only by the order of the fp64 term sums).  Stated bound: 0
    differing correspondences and ≤ 1e-12 per coordinate at every evaluation."""
    diffs = []

    def cmp(k, pcd, j):
        pts, corr = dev[k]
        diffs.append((k, int(np.count_nonzero(corr != j)), float(np.max(np.abs(pts - pcd)))))

    ref = I.registration_icp(src, tgt, r, init=np.eye(4), tgt_normals=nrm, relative_fitness=-1,
                             relative_rmse=-1, max_iteration=n_iter, on_eval=cmp, **kw)
    assert len(diffs) == len(dev)
    print("evaluation, correspondences differing from the incremental oracle, max |Δpoint|:")
    print(" ".join(f"{k}:{n}/{d:.1e}" for k, n, d in diffs))
    assert all(n == 0 for _, n, _ in diffs), diffs
    assert max(d for _, _, d in diffs) <= 1e-12, diffs
    return ref


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_icp_cfg1_matches_oracle(nn):
    """cfg1 itself (bench.py's pair: 100k ↔ 100k, seed 0, r = 0.12, 50 fixed point-to-plane
    iterations = 51 evaluations), every evaluation checked by _check_evaluations; the device's
    final transform and fitness agree with the oracle's own 50-iteration run (the only difference
    is the order of the fp64 term sums: measured ≲ 1e-15, bound stated 1e-9)."""
    src, tgt, nrm, T_true = synth.icp_pair(100_000, 100_000, seed=0)
    lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=50, nn=nn)
    dev = []
    r = _check_evaluations(lp, src, tgt, np.eye(4), 51, keep=dev)
    ref = _against_oracle_run(dev, src, tgt, nrm, 0.12, 50)
    assert r.iterations == ref["iterations"] == 50
    np.testing.assert_allclose(r.transformation, ref["transformation"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(lp.points().cpu().numpy(), ref["points"], rtol=0, atol=1e-9)
    assert r.fitness == ref["fitness"]
    assert abs(r.inlier_rmse - ref["inlier_rmse"]) < 1e-12
    np.testing.assert_allclose(r.transformation, T_true, atol=5e-4)


@pytest.mark.parametrize("which", ["rigid", "fuzzy_identity"])
def test_icp_init_applied_as_registration_icp(which):
    """A non-identity init moves the loop's points before the first evaluation; an init within
    Eigen's 1e-12 of I does not (the points stay the source's own bits), while T starts at init
    either way (Registration.cpp)."""
    src, tgt, nrm, _ = synth.icp_pair(30_000, 30_000, seed=6)
    if which == "rigid":
        init = synth.random_rigid(9, rot_range=0.01, trans_range=0.01)
    else:
        init = np.eye(4)
        init[0, 3] = 5e-13
        init[1, 2] = -3e-13
    lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=6, nn="grid")
    r = _check_evaluations(lp, src, tgt, init, 7)
    ref = I.registration_icp(src, tgt, 0.12, init=init, tgt_normals=nrm, relative_fitness=-1,
                             relative_rmse=-1, max_iteration=6)
    np.testing.assert_allclose(r.transformation, ref["transformation"], rtol=0, atol=1e-9)
    assert r.fitness == ref["fitness"]
    out = icp(Cloud(src), Cloud(tgt, nrm), 0.12, init, relative_fitness=-1, relative_rmse=-1,
              max_iteration=6)
    np.testing.assert_array_equal(out.transformation, r.transformation)
    np.testing.assert_array_equal(out.update, r.update)


@pytest.mark.parametrize("nn", ["brute", "grid"])
@pytest.mark.parametrize("ns", [1, 2, 63, 65, 255, 257, 511, 513, 4097])
def test_icp_ragged_sources_incremental_points(ns, nn):
    """Ragged source counts around the wave (64), terms-block (256 / 512) and tile sizes: every
    evaluation's points and correspondences as _check_evaluations requires (bit for bit), against
    a 20k target, from a rigid init; the final transform against the oracle's run where the 6 × 6
    system has full rank (ns ≥ 63: with 1–2 sources JTJ has rank ≤ 2, its other pivots are
    rounding noise, and any two LDLT implementations return different, equally meaningless
    solutions — Eigen's included)."""
    src_all, tgt, nrm, _ = synth.icp_pair(20_000, 20_000, seed=23)
    src = src_all[:ns].copy()
    init = synth.random_rigid(ns, rot_range=0.005, trans_range=0.005)
    lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=4, nn=nn)
    r = _check_evaluations(lp, src, tgt, init, 5)
    ref = I.registration_icp(src, tgt, 0.12, init=init, tgt_normals=nrm, relative_fitness=-1,
                             relative_rmse=-1, max_iteration=4)
    if ns >= 63:
        np.testing.assert_allclose(r.transformation, ref["transformation"], rtol=0, atol=1e-9)
        assert r.fitness == ref["fitness"]


@pytest.mark.parametrize("nn", ["brute", "grid"])
def test_icp_ambiguous_pairs_and_triples_exact(nn):
    """A target with exact duplicate pairs, exact triples and near-duplicate pairs (1e-9 apart,
    one fp32 point, two fp64 points): their queries are ambiguous (the runner-up inside the fp32
    error band).  The grid loop decides a query with exactly two targets in its band from the
    scan's runner-up (grid.hip alt) and walks the grid for three or more; the brute loop always
    walks.  Every evaluation's correspondences must equal the oracle's exact fp64 NN (ties: the
    lowest index) bit for bit."""
    src, tgt, nrm, _ = synth.icp_pair(20_000, 12_000, seed=31)
    near = tgt[6000:9000].copy()
    near[:, 0] += 1e-9
    tgt2 = np.concatenate([tgt, tgt[:3000], tgt[3000:6000], tgt[3000:6000], near])
    nrm2 = np.concatenate([nrm, nrm[:3000], nrm[3000:6000], nrm[3000:6000], nrm[6000:9000]])
    lp = IcpLoop(Cloud(src), Cloud(tgt2, nrm2), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=4, nn=nn)
    keep = []
    _check_evaluations(lp, src, tgt2, np.eye(4), 5, keep=keep)
    # the duplicate sets are met: some correspondences name a copy's lowest index, some a
    # near-duplicate decided in fp64
    corr = keep[-1][1]
    assert np.isin(corr, np.arange(3000)).any() and np.isin(corr, np.arange(3000, 6000)).any()
    assert np.isin(corr, np.arange(6000, 9000)).any() or np.isin(corr, np.arange(21000, 24000)).any()


def test_icp_cfg1_point_to_point_matches_oracle():
    """cfg1's pair with TransformationEstimationPointToPoint (a10: Umeyama over the 15 centred
    sums, rotation_from_cov shared with a1), 30 fixed iterations, grid NN: every evaluation
    checked by _check_evaluations, final transform / fitness / rmse against the oracle's own run."""
    src, tgt, nrm, _ = synth.icp_pair(100_000, 100_000, seed=0)
    lp = IcpLoop(Cloud(src), Cloud(tgt, nrm), 0.12, relative_fitness=-1, relative_rmse=-1,
                 max_iteration=30, nn="grid", estimation=_lib.EST_POINT_TO_POINT)
    dev = []
    r = _check_evaluations(lp, src, tgt, np.eye(4), 31, keep=dev)
    ref = _against_oracle_run(dev, src, tgt, None, 0.12, 30, estimation="point_to_point")
    assert r.iterations == ref["iterations"] == 30
    np.testing.assert_allclose(r.transformation, ref["transformation"], rtol=0, atol=1e-9)
    assert r.fitness == ref["fitness"]
    assert abs(r.inlier_rmse - ref["inlier_rmse"]) < 1e-12


def test_fused_tail_beyond_256_blocks_equals_separate():
    """Past 256 terms blocks the fused tail's last block reduces the partials in several batches
    (brute force keeps the fused form: it hands the keys back) and the grid loop switches to the
    separate terms / reduce / solve launches (api.cpp fused_tail).  A subprocess with
    M3D_ICP_FUSED=0 (all separate) and one with the default give the same bits at 300k sources
    (587 blocks)."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path

    code = r'''
import json, sys
import numpy as np
sys.path[:0] = [sys.argv[1]]
import torch
from m3d import synth
from m3d.core import Cloud, IcpLoop
src, tgt, nrm, _ = synth.icp_pair(300000, 120000, seed=41)
s, t = Cloud(src), Cloud(tgt, nrm)
out = {}
for nn in ("brute", "grid"):
    lp = IcpLoop(s, t, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=6, nn=nn)
    lp.reset(np.eye(4))
    lp.steps(7)
    r = lp.result()
    out[nn] = [r.transformation.tolist(), r.fitness, r.inlier_rmse, r.iterations]
print(json.dumps(out))
'''
    pkg = str(Path(__file__).resolve().parents[1] / "3d-matching_amd")
    res = {}
    for fused in ("0", "1"):
        env = dict(os.environ, M3D_ICP_FUSED=fused)
        r = subprocess.run([sys.executable, "-c", code, pkg], env=env, capture_output=True, text=True,
                           timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        res[fused] = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["0"] == res["1"]
    assert res["1"]["brute"] == res["1"]["grid"]


def test_deferred_dense_queries_give_the_same_bits():
    """grid_nn_heavy_kernel (one block per query with more than the candidate cap, and every
    ambiguous query decided in fp64) gives the per-query scan + terms pass's bits:
    M3D_GRID_HEAVY=8 defers nearly every query, =0 none; both give the brute-force loop's bits on
    a pair with a dense vertex fan (where the default defers some), over 41 steps enqueued back to
    back (the list's count is re-zeroed by the kernel, never by the host)."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path

    code = r'''
import json, sys
import numpy as np
sys.path[:0] = [sys.argv[1]]
import torch
from m3d import synth
from m3d.core import Cloud, IcpLoop, nn1
src, tgt, nrm, _ = synth.icp_pair(60000, 50000, seed=43)
rng = np.random.default_rng(5)
fan = tgt[11] + rng.normal(scale=0.002, size=(4000, 3))
tgt = np.vstack([tgt, fan]); nrm = np.vstack([nrm, np.repeat(nrm[11:12], 4000, 0)])
src = np.vstack([src, tgt[11] + rng.normal(scale=0.05, size=(3000, 3))])
s, t = Cloud(src), Cloud(tgt, nrm)
out = {}
for nn in ("brute", "grid"):
    lp = IcpLoop(s, t, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=40, nn=nn)
    lp.reset(synth.random_rigid(3, rot_range=0.03, trans_range=0.05))
    for _ in range(41):  # back to back, no host sync: each launch must start from an empty list
        lp.step()
    r = lp.result()
    c = lp.correspondences().cpu().numpy()
    out[nn] = [r.transformation.tolist(), r.fitness, r.inlier_rmse, r.iterations, int(c.sum()), int((c >= 0).sum())]
    # the same 41 steps as captured HIP graphs: a sequence requested twice is captured, then
    # replayed (api.cpp capture_steps) — the deferral list is used inside the graph too
    g = IcpLoop(s, t, 0.12, relative_fitness=-1, relative_rmse=-1, max_iteration=40, nn=nn)
    for _ in range(3):
        g.reset(synth.random_rigid(3, rot_range=0.03, trans_range=0.05))
        for _ in range(4):
            g.steps(10)
        g.step()
    r = g.result()
    c = g.correspondences().cpu().numpy()
    out[nn + "_graph"] = [r.transformation.tolist(), r.fitness, r.inlier_rmse, r.iterations, int(c.sum()), int((c >= 0).sum())]
i, d = nn1(Cloud(src), t, np.eye(4), 0.12, nn="grid")
out["nn1"] = [int(i.sum().item()), float(d.sum().item())]
print(json.dumps(out))
'''
    pkg = str(Path(__file__).resolve().parents[1] / "3d-matching_amd")
    res = {}
    for mode in ("0", "8", None):
        env = dict(os.environ)
        env.pop("M3D_GRID_HEAVY", None)
        if mode is not None:
            env["M3D_GRID_HEAVY"] = mode
        r = subprocess.run([sys.executable, "-c", code, pkg], env=env, capture_output=True, text=True,
                           timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        res[mode] = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["0"] == res["8"] == res[None]
    assert res[None]["brute"] == res[None]["grid"] == res[None]["brute_graph"] == res[None]["grid_graph"]


def test_deferral_list_survives_a_dirty_reused_block_and_flags_overflow():
    """the grid scan's deferral list (count, ticket, fault word) is zeroed before the
    loop's setup sync and by every reset on the caller's stream, and a slot past the list is
    dropped and flagged instead of written out of bounds.  A grid loop whose arrays come from a
    cache block pre-filled with 0xFF (m3d_debug_block_cache_fill), stepped on a non-blocking
    torch stream under M3D_GRID_HEAVY=8 (nearly every query deferred), gives the brute-force
    loop's bits; a forced count past the list makes result() fail (not fault), and a reset
    recovers the same bits."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path

    code = r'''
import ctypes as C, json, sys
import numpy as np
sys.path[:0] = [sys.argv[1]]
import torch
from m3d import synth
from m3d.core import Cloud, IcpLoop, context, stream_handle
src, tgt, nrm, _ = synth.icp_pair(60000, 50000, seed=43)
rng = np.random.default_rng(5)
fan = tgt[11] + rng.normal(scale=0.002, size=(4000, 3))
tgt = np.vstack([tgt, fan]); nrm = np.vstack([nrm, np.repeat(nrm[11:12], 4000, 0)])
src = np.vstack([src, tgt[11] + rng.normal(scale=0.05, size=(3000, 3))])
s, t = Cloud(src), Cloud(tgt, nrm)
kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=20)
init = synth.random_rigid(3, rot_range=0.03, trans_range=0.05)
def outcome(lp):
    r = lp.result()
    c = lp.correspondences().cpu().numpy()
    return [r.transformation.tolist(), r.fitness, r.inlier_rmse, r.iterations, int(c.sum()), int((c >= 0).sum())]
ref = IcpLoop(s, t, 0.12, nn="brute", **kw)
ref.reset(init)
ref.steps(21)
want = outcome(ref)
lib = context().lib
g0 = IcpLoop(s, t, 0.12, nn="grid", **kw)  # its arrays' block goes back to the cache
del g0
torch.cuda.synchronize()
filled = lib.m3d_debug_block_cache_fill(0xFF)
st = torch.cuda.Stream()
out = {"filled": filled}
with torch.cuda.stream(st):
    lp = IcpLoop(s, t, 0.12, nn="grid", **kw)  # reuses a 0xFF block
    lp.reset(init)
    for _ in range(21):  # back to back on the non-blocking stream
        lp.step()
    out["dirty"] = outcome(lp) == want
    lp.reset(init)  # (a finished loop's scans are no-ops: poke a running one)
    lp.step()
    rc = lib.m3d_debug_icp_defer_count(lp.h, C.c_uint32(0x7FFFFFF0), stream_handle())
    out["poke_rc"] = rc
    lp.step()
    try:
        lp.result()
        out["overflow"] = "no error"
    except RuntimeError as e:
        out["overflow"] = str(e)
    lp.reset(init)
    for _ in range(21):
        lp.step()
    out["recovered"] = outcome(lp) == want
print(json.dumps(out))
'''
    pkg = str(Path(__file__).resolve().parents[1] / "3d-matching_amd")
    env = dict(os.environ, M3D_GRID_HEAVY="8")
    r = subprocess.run([sys.executable, "-c", code, pkg], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["filled"] >= 1, res
    assert res["dirty"] is True, res
    assert res["poke_rc"] == 0, res
    assert "deferral list overflow" in res["overflow"], res
    assert res["recovered"] is True, res
