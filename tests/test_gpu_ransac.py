"""GPU parity: the HIP RANSAC path (through the C ABI) vs the reference's golden vectors and the
CPU oracle.  Bar: inlier counts bit-exact; Kabsch transforms within 1e-9 (rank-2 samples);
loop trajectories (best index, best fitness, stop iteration) exact."""
import numpy as np
import pytest

import ransac_oracle as O
from m3d import _lib, synth
from m3d.core import CorrSet, RansacParams

pytestmark = pytest.mark.gpu

THR = 0.3 * 1.5


def rank_deficient(a, b):
    H = (a - a.mean(0)).T @ (b - b.mean(0))
    s = np.linalg.svd(H, compute_uv=False)
    return s[1] <= 1e-10 * s[0]


@pytest.fixture(scope="module")
def sets(pts5k):
    out = {}
    for name in ("clean", "noise", "mid"):
        corr = pts5k[f"corr_{name}"]
        out[name] = (CorrSet(pts5k["src"], pts5k["tgt"], corr), corr)
    return out


@pytest.mark.parametrize("seed", (0, 1, 42))
@pytest.mark.parametrize("name", ("clean", "noise"))
def test_kabsch_replay_matches_reference(golden, pts5k, sets, seed, name):
    g = golden(f"ransac_5k_seed{seed}.npz")
    cs, corr = sets[name]
    T, st = cs.kabsch3(1000, triples=g[f"{name}_triples"])
    T = T.cpu().numpy()
    assert (st.cpu().numpy() == _lib.HYP_OK).all()
    p, q = pts5k["src"][corr[:, 0]], pts5k["tgt"][corr[:, 1]]
    tri = g[f"{name}_triples"]
    for h in range(1000):
        if rank_deficient(p[tri[h]], q[tri[h]]):
            R = T[h, :3, :3]
            np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
            continue
        np.testing.assert_allclose(T[h], g[f"{name}_T"][h], atol=1e-9, err_msg=f"hyp {h}")


@pytest.mark.parametrize("seed", (0, 1, 42))
@pytest.mark.parametrize("name", ("clean", "noise"))
def test_scores_exact_on_reference_transforms(golden, sets, seed, name):
    g = golden(f"ransac_5k_seed{seed}.npz")
    cs, _ = sets[name]
    Ts = g[f"{name}_T"]
    fast = cs.score(Ts, THR * THR, _lib.SCORE_SQUARED).cpu().numpy()
    slow = cs.score(Ts, THR, _lib.SCORE_NORM).cpu().numpy()
    np.testing.assert_array_equal(fast, g[f"{name}_count_fast"])
    np.testing.assert_array_equal(slow, g[f"{name}_count_slow"])


def test_native_sampler_matches_oracle(pts5k, sets):
    cs, corr = sets["noise"]
    H = 3000
    T, st = cs.kabsch3(H, seed=42, hyp0=17)
    T = T.cpu().numpy()
    tri = O.native_triples(42, 17, H, len(corr))
    p, q = pts5k["src"][corr[:, 0]], pts5k["tgt"][corr[:, 1]]
    for h in range(0, H, 3):
        if rank_deficient(p[tri[h]], q[tri[h]]):
            continue
        Tr, _ = O.kabsch3(p[tri[h]], q[tri[h]])
        np.testing.assert_allclose(T[h], Tr, atol=1e-9)


@pytest.mark.parametrize("name", ("clean", "noise", "mid"))
def test_loop_trajectory_matches_reference(golden, sets, name):
    t = golden("loop_trajectory.npz")
    cs, corr = sets[name]
    max_iter = int(t[f"{name}_max_iter"])
    tri, _ = O.replay_triples(int(t[f"{name}_seed"]), len(corr), max_iter)
    for batch in (0, 7, 64):
        out = cs.run(RansacParams(max_iter=max_iter, thr=THR * THR, mode=_lib.SCORE_SQUARED,
                                  early_stop=True, batch=batch), triples=tri)
        assert out.best_index == int(t[f"{name}_best_index"])
        assert out.fitness == float(t[f"{name}_best_fitness"])
        assert out.iterations == int(t[f"{name}_iterations"])


def test_loop_no_early_stop_argmax(pts5k, sets):
    cs, corr = sets["noise"]
    H = 5000
    out = cs.run(RansacParams(max_iter=H, seed=9, thr=THR, mode=_lib.SCORE_NORM, early_stop=False,
                              batch=1000))
    T, _ = cs.kabsch3(H, seed=9)
    counts = cs.score(T, THR, _lib.SCORE_NORM).cpu().numpy()
    assert out.iterations == H
    assert out.best_index == int(np.argmax(counts))
    assert out.best_count == counts.max()
    np.testing.assert_allclose(out.transformation, T[out.best_index].cpu().numpy(), atol=0)


def test_matcher_api_is_drop_in(golden, pts5k):
    from matcher import ransac as M
    from ply import Ply

    g = golden("ransac_5k_seed42.npz")
    corr = pts5k["corr_noise"]
    src = Ply.from_arrays(pts5k["src"])
    tgt = Ply.from_arrays(pts5k["tgt"])
    np.random.seed(42)
    p, q = pts5k["src"][corr[:, 0]], pts5k["tgt"][corr[:, 1]]
    for h in range(12):
        res = M.compute_step_transformation(src, tgt, corr)
        assert res.fitness == 0.0
        if not rank_deficient(p[g["noise_triples"][h]], q[g["noise_triples"][h]]):
            np.testing.assert_allclose(res.transformation, g["noise_T"][h], atol=1e-9)
        assert M.evaluate_inlier_ratio(src, tgt, corr, g["noise_T"][h], 0.3) == g["noise_ratio_slow"][h]
        assert M.evaluate_inlier_ratio_fast(p, q, g["noise_T"][h], float(g["thr_sq"])) == \
            g["noise_ratio_fast"][h]
    # RNG consumed exactly like the reference's 12 calls
    np.random.seed(42)
    for _ in range(12):
        np.random.choice(len(corr), 3, replace=False)
    ref_next = np.random.rand()
    np.random.seed(42)
    for _ in range(12):
        M.compute_step_transformation(src, tgt, corr)
    assert np.random.rand() == ref_next


def test_matcher_ransac_replay_equals_reference_loop(golden, pts5k):
    from matcher import ransac as M

    t = golden("loop_trajectory.npz")
    corr = pts5k["corr_mid"]
    np.random.seed(int(t["mid_seed"]))
    res, info = M.run_ransac(pts5k["src"], pts5k["tgt"], corr, voxel_size=0.3,
                         max_iter=int(t["mid_max_iter"]))
    assert info["iterations"] == int(t["mid_iterations"])
    assert info["best_index"] == int(t["mid_best_index"])
    assert res.fitness == float(t["mid_best_fitness"])
    # the global RNG advanced by exactly the iterations consumed
    after = np.random.rand()
    np.random.seed(int(t["mid_seed"]))
    for _ in range(int(t["mid_iterations"])):
        np.random.choice(len(corr), 3, replace=False)
    assert np.random.rand() == after


@pytest.mark.parametrize("max_iter", [5000, 8192])
def test_replay_rng_advance_across_checkpoints(pts5k, max_iter):
    """run_ransac's replay keeps an MT checkpoint every 4096 rows; without early stop the loop
    consumes max_iter rows (one checkpoint + a remainder, or exactly two checkpoints) and the
    global RNG must end where max_iter np.random.choice calls leave it."""
    from matcher import ransac as M

    corr = pts5k["corr_mid"]
    np.random.seed(77)
    _, info = M.run_ransac(pts5k["src"], pts5k["tgt"], corr, voxel_size=0.3, max_iter=max_iter,
                           early_stop=False)
    assert info["iterations"] == max_iter
    after = np.random.rand()
    np.random.seed(77)
    for _ in range(max_iter):
        np.random.choice(len(corr), 3, replace=False)
    assert np.random.rand() == after


def test_crash_kats_through_api(golden):
    from matcher import ransac as M

    k = golden("crash_kats.npz")
    c3 = np.array([[0, 0], [1, 1], [2, 2]], dtype=np.int32)
    col = k["collinear_pts"]
    np.random.seed(5)
    np.testing.assert_allclose(M.compute_step_transformation(col, col, c3).transformation,
                               k["collinear_T"], atol=1e-12)
    dup = k["duplicate_pts"]
    np.random.seed(9)
    np.testing.assert_allclose(M.compute_step_transformation(dup, dup, c3).transformation,
                               k["duplicate_T"], atol=1e-12)
    np.random.seed(8)
    np.testing.assert_allclose(M.compute_step_transformation(k["coplanar_src"], k["coplanar_tgt"],
                                                             c3).transformation,
                               k["coplanar_T"], atol=1e-12)
    for s in range(10):
        np.random.seed(200 + s)
        np.testing.assert_allclose(
            M.compute_step_transformation(k["minimal_src"][s], k["minimal_tgt"][s], c3).transformation,
            k["minimal_T"][s], atol=1e-12)
    ten = np.random.rand(10, 3)
    assert M.evaluate_inlier_ratio(ten, ten, np.zeros((0, 2), np.int32), np.eye(4), 0.3) == 0.0
    r = M.compute_step_transformation(ten, ten, c3[:2])
    np.testing.assert_array_equal(r.transformation, np.eye(4))


def test_crash_kat_ratios_through_api(golden, pts5k):
    from matcher import ransac as M

    k = golden("crash_kats.npz")
    src, tgt = pts5k["src"], pts5k["tgt"]
    assert M.evaluate_inlier_ratio(src, tgt, pts5k["corr_clean"], k["large_T"], 0.3) == k["large_ratio_clean"]
    assert M.evaluate_inlier_ratio(src, tgt, pts5k["corr_clean"], np.eye(4), 0.3) == k["identity_ratio_clean"]
    assert M.evaluate_inlier_ratio(src, tgt, pts5k["corr_clean"], pts5k["T_true"], 0.3) == k["true_ratio_clean"]
    assert M.evaluate_inlier_ratio(src, tgt, pts5k["corr_noise"], pts5k["T_true"], 0.3) == k["true_ratio_noise"]


def test_negative_and_out_of_range_indices():
    from matcher import ransac as M

    pts = np.random.default_rng(0).random((10, 3))
    c = np.array([[-1, -1], [0, 0], [1, 1]], dtype=np.int32)  # numpy wraps -1
    assert M.evaluate_inlier_ratio(pts, pts, c, np.eye(4), 0.3) == 1.0
    with pytest.raises(IndexError):  # numpy's error, as the reference's gather raises it
        M.evaluate_inlier_ratio(pts, pts, np.array([[0, 10]], np.int32), np.eye(4), 0.3)
    # compute_step_transformation reads only its 3 sampled rows (ransac.py:143-148): an
    # out-of-range row elsewhere is harmless, a sampled one raises IndexError
    bad = np.array([[0, 0], [1, 1], [2, 2], [3, 99]], np.int32)
    np.random.seed(0)  # choice(4, 3) = [2, 3, 1]: row 3 is sampled
    with pytest.raises(IndexError):
        M.compute_step_transformation(pts, pts, bad)
    np.random.seed(5)  # choice(4, 3) = [0, 1, 2]: row 3 is never read
    r = M.compute_step_transformation(pts, pts, bad)
    np.testing.assert_allclose(r.transformation, np.eye(4), atol=1e-9)
    # an unread int64 row beyond int32 range is harmless too, and the draw still happens
    wide = bad.astype(np.int64)
    wide[3, 1] = 1 << 40
    np.random.seed(5)
    r = M.compute_step_transformation(pts, pts, wide)
    np.testing.assert_allclose(r.transformation, np.eye(4), atol=1e-9)
    after = np.random.rand()
    np.random.seed(5)
    np.random.choice(4, 3, replace=False)
    assert np.random.rand() == after


@pytest.mark.parametrize("nc", [1, 2, 3, 5, 63, 2047, 2048, 2049, 10007])
def test_ragged_sizes_exact(nc):
    from m3d import synth

    src, tgt, corr, T = synth.ransac_pair(max(nc, 3), seed=nc)
    corr = corr[:nc]
    cs = CorrSet(src, tgt, corr)
    rng = np.random.default_rng(nc)
    Ts = np.stack([T] + [synth.random_rigid(int(s), rot_range=0.2, trans_range=0.3)
                         for s in rng.integers(0, 1 << 30, 70)])
    p, q = src[corr[:, 0]], tgt[corr[:, 1]]
    for mode, thr in ((_lib.SCORE_SQUARED, THR * THR), (_lib.SCORE_NORM, THR)):
        got = cs.score(Ts, thr, mode).cpu().numpy()
        np.testing.assert_array_equal(got, O.inlier_counts(p, q, Ts, thr, mode))


def test_guard_band_recheck_is_exercised_and_exact():
    """Pairs placed within ~1e-7 of the threshold force the fp64 recheck path."""
    from m3d.core import context

    rng = np.random.default_rng(3)
    n = 20000
    p = rng.uniform(-5, 5, (n, 3))
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    scale = THR * (1 + rng.uniform(-3e-7, 3e-7, n))
    q = p + d * scale[:, None]
    cs = CorrSet(p_src=p, p_tgt=q)
    ctx = context()
    before = ctx.stats()
    Ts = np.stack([np.eye(4)] * 5)
    for mode, thr in ((_lib.SCORE_SQUARED, THR * THR), (_lib.SCORE_NORM, THR)):
        got = cs.score(Ts, thr, mode).cpu().numpy()
        np.testing.assert_array_equal(got, O.inlier_counts(p, q, Ts, thr, mode))
    assert (ctx.stats() - before)[:2].sum() > 0  # rechecks happened


def test_full_size_counts_subsample_exact():
    """cfg2 geometry (Nc = 1e5): native-sampled hypotheses' counts equal the oracle's."""
    from m3d import synth

    src, tgt, corr, _ = synth.ransac_pair(100_000, seed=42)
    cs = CorrSet(src, tgt, corr)
    H = 20_000
    T, _ = cs.kabsch3(H, seed=42)
    counts = cs.score(T, THR, _lib.SCORE_NORM).cpu().numpy()
    Tn = T.cpu().numpy()
    p, q = src[corr[:, 0]], tgt[corr[:, 1]]
    pick = np.random.default_rng(0).choice(H, 60, replace=False)
    np.testing.assert_array_equal(counts[pick], O.inlier_counts(p, q, Tn[pick], THR, 1))
    out = cs.run(RansacParams(max_iter=H, seed=42, thr=THR, mode=_lib.SCORE_NORM, early_stop=False))
    assert out.best_count == counts.max() and out.best_index == int(np.argmax(counts))


def test_score_edge_transforms_exact():
    """Transforms outside the MFMA screen's rigid/near regime keep exact counts: a scaled
    (non-rigid) matrix (every pair re-evaluated in fp64), NaN entries and far translations
    (count 0 by the |d|∞ bound), and a threshold beyond the cloud extent (fp32 screen)."""
    from m3d import synth

    src, tgt, corr, T = synth.ransac_pair(5000, seed=8)
    cs = CorrSet(src, tgt, corr)
    p, q = src[corr[:, 0]], tgt[corr[:, 1]]
    scaled = T.copy()
    scaled[:3, :3] *= 1.5
    nan = T.copy()
    nan[0, 1] = np.nan
    far = T.copy()
    far[:3, 3] += 1e4
    near_far = T.copy()
    near_far[:3, 3] += 12.0  # just past the extent: the bound must not reject possible inliers
    Ts = np.stack([T, scaled, nan, far, near_far, np.eye(4)])
    for mode, thr in ((_lib.SCORE_SQUARED, THR * THR), (_lib.SCORE_NORM, THR),
                      (_lib.SCORE_NORM, 50.0), (_lib.SCORE_SQUARED, 1e-12)):
        got = cs.score(Ts, thr, mode).cpu().numpy()
        np.testing.assert_array_equal(got, O.inlier_counts(p, q, Ts, thr, mode))


@pytest.mark.parametrize("early_stop", [True, False])
def test_run_async_matches_run(early_stop):
    """m3d_ransac_run_async (no host round trip; bench.py enqueues runs back to back) gives the
    synchronous run's outcome bit for bit, batches of 2^18 included."""
    import torch

    from m3d import synth
    from m3d.core import RESULT_WORDS, RansacOutcome

    src, tgt, corr, _ = synth.ransac_pair(20000, seed=3, noise_ratio=1.0)
    cs = CorrSet(src, tgt, corr)
    p = RansacParams(max_iter=3000, seed=7, thr=THR, mode=_lib.SCORE_NORM, early_stop=early_stop)
    a = cs.run(p)
    buf = torch.zeros(RESULT_WORDS, dtype=torch.int64, device="cuda")
    cs.run_async(p, buf)
    b = RansacOutcome.from_device(buf, cs.nc)
    assert (a.best_index, a.iterations, a.best_count) == (b.best_index, b.iterations, b.best_count)
    np.testing.assert_array_equal(a.transformation, b.transformation)
    assert a.fitness == b.fitness


# ---------------------------------------------------------------- cfg2 scale (Nc = 1e5)
@pytest.fixture(scope="module")
def cfg2(golden):
    from golden_pairs import cfg2_pair

    g, src, tgt, corr, noise = cfg2_pair(golden)
    return g, src, tgt, corr, noise, CorrSet(src, tgt, corr), CorrSet(src, tgt, noise)


@pytest.mark.parametrize("key", ("s42", "s7", "noise"))
def test_cfg2_reference_calls_exact(cfg2, key):
    """benchmark_ransac.py:105-113 at Nc = 1e5 (3e5 with noise): the reference's own sampled rows
    replayed through a1 (transforms within 1e-9 of LAPACK) and its counts for both comparators
    bit-exact; the replay-mode loop picks the reference's best of those calls."""
    g, src, tgt, corr, noise, cs, csn = cfg2
    c, s = (noise, csn) if key == "noise" else (corr, cs)
    tri = g[f"{key}_triples"]
    T, st = s.kabsch3(len(tri), triples=tri)
    T = T.cpu().numpy()
    p, q = src[c[:, 0]], tgt[c[:, 1]]
    for h in range(len(tri)):
        if not rank_deficient(p[tri[h]], q[tri[h]]):
            np.testing.assert_allclose(T[h], g[f"{key}_T"][h], rtol=0, atol=1e-9, err_msg=f"hyp {h}")
    Tg = g[f"{key}_T"]
    np.testing.assert_array_equal(s.score(Tg, THR, _lib.SCORE_NORM).cpu().numpy(), g[f"{key}_count_slow"])
    np.testing.assert_array_equal(s.score(Tg, THR * THR, _lib.SCORE_SQUARED).cpu().numpy(),
                                  g[f"{key}_count_fast"])
    out = s.run(RansacParams(max_iter=len(tri), thr=THR, mode=_lib.SCORE_NORM, early_stop=False),
                triples=tri)
    ref_best = int(np.argmax(g[f"{key}_count_slow"]))  # first strict improvement = first max
    assert (out.best_index, out.best_count) == (ref_best, int(g[f"{key}_count_slow"][ref_best]))


def _run_batch(cs, H, thr, mode):
    """The exact batch bench.py times: one run of H native hypotheses (seed 42), no early stop;
    returns (per-hypothesis counts, outcome)."""
    import ctypes

    import torch

    from m3d.core import RESULT_WORDS, RansacOutcome, ptr, stream_handle

    counts = torch.zeros(H, dtype=torch.int32, device="cuda")
    buf = torch.zeros(RESULT_WORDS, dtype=torch.int64, device="cuda")
    p = RansacParams(max_iter=H, seed=42, thr=thr, mode=mode, early_stop=False)
    cs.ctx.check(cs.ctx.lib.m3d_ransac_run_async(cs.ctx.h, cs.h, ctypes.byref(p.to_c()), None,
                                                 ptr(counts), ptr(buf), stream_handle()), "run_async")
    return counts.cpu().numpy(), RansacOutcome.from_device(buf, cs.nc)


@pytest.mark.parametrize("key", ("n1e5", "n3e5"))
def test_cfg2_bench_batch_exact(golden, cfg2, key):
    """Every one of the 1e5 hypotheses of the exact batch bench.py times (counter sampler seed 42,
    one batch, no early stop) against the REFERENCE's counts (tools/gen_golden_full.py: the
    reference's evaluate_inlier_ratio on Nc = 1e5 — benchmark_ransac.py's comparator — and its
    evaluate_inlier_ratio_fast on the noise_ratio 2.0 set, Nc = 3e5 — the GUI's), each on the
    oracle's a1 transform (numpy SVD; bit-exact to the reference's own a1 at 5k,
    tests/test_oracle_golden.py).  The device scores its own transforms (within 1e-9 of those), so
    a count is compared bit for bit where no pair lies within 1e-7 of the threshold under the
    reference transform (the golden ``band``) and whose 3-point sample is not rank-deficient (a
    repeated or collinear sample leaves the rotation about its axis undetermined: any such
    rotation minimises the Kabsch objective and the count follows LAPACK's choice — 6 of the 1e5
    samples of the noise_ratio 2.0 set repeat a point); the banded and rank-deficient hypotheses
    are re-scored on the device with the oracle's transform and must then equal the reference's
    count exactly."""
    g, src, tgt, corr, noise, cs, csn = cfg2
    full = golden("ransac_cfg2_full.npz")
    assert str(full["digest"]) == str(g["digest"]) and str(full["noise_digest"]) == str(g["noise_digest"])
    H = int(full["h"])
    c, s = (corr, cs) if key == "n1e5" else (noise, csn)
    thr, mode = (THR, _lib.SCORE_NORM) if key == "n1e5" else (THR * THR, _lib.SCORE_SQUARED)
    want = full[f"batch_{key}_count"].astype(np.int64)
    band = full[f"batch_{key}_band"]
    counts, out = _run_batch(s, H, thr, mode)
    assert out.iterations == H
    pp, qq = src[c[:, 0]], tgt[c[:, 1]]
    tri = O.native_triples(42, 0, H, len(c))
    P, Q = pp[tri], qq[tri]
    P, Q = P - P.mean(1, keepdims=True), Q - Q.mean(1, keepdims=True)
    sv = np.linalg.svd(np.einsum("hki,hkj->hij", P, Q), compute_uv=False)
    rankdef = sv[:, 1] <= 1e-10 * sv[:, 0]  # rank_deficient() over the whole batch
    free = (band == 0) & ~rankdef
    assert free.mean() > 0.99 and rankdef.sum() <= 16
    np.testing.assert_array_equal(counts[free], want[free])
    banded = np.nonzero(~free)[0]
    To = np.stack([O.kabsch3(pp[tri[h]], qq[tri[h]])[0] for h in banded])
    np.testing.assert_array_equal(s.score(To, thr, mode).cpu().numpy(), want[banded])
    # the run's winner: the first maximum of its own counts, and the reference's maximum
    assert out.best_index == int(np.argmax(counts)) and out.best_count == counts.max() == want.max()
    T, _ = s.kabsch3(H, seed=42)
    np.testing.assert_array_equal(out.transformation, T[out.best_index].cpu().numpy())


@pytest.mark.parametrize("key", ("n1e5", "n3e5"))
def test_gui_loop_early_stop_at_baseline_scale(golden, cfg2, key):
    """The GUI step-RANSAC loop (_visualize_matcher.py:394-450: a1 + evaluate_inlier_ratio_fast,
    early stop at fitness > 0.5 with confidence 0.99, ransac_iteration 10000) at the BASELINE
    scale, replaying the reference's own rows from np.random.seed(42): Nc = 1e5 (noise 0, stops at
    iteration 2) and Nc = 3e5 (noise_ratio 2.0, the GUI default: best fitness ≈ 1/3, never stops
    early, all 10000 iterations).  The drop-in's run_ransac(sampler="replay", early_stop=True)
    must give the reference loop's best index, best fitness and stop iteration (golden from the
    reference's own a1 + a3, tools/gen_golden_full.py), and every iteration's count must equal
    the reference's (a count that differs is re-scored with the oracle's transform — bit-exact
    to the reference's a1 — and must then match)."""
    from matcher import ransac as M

    g, src, tgt, corr, noise, cs, csn = cfg2
    full = golden("ransac_cfg2_full.npz")
    c, s = (corr, cs) if key == "n1e5" else (noise, csn)
    np.random.seed(42)
    res, info = M.run_ransac(src, tgt, c, voxel_size=0.3, max_iter=int(full[f"loop_{key}_max_iter"]),
                             early_stop=True, sampler="replay", score="fast")
    assert info["best_index"] == int(full[f"loop_{key}_best_index"])
    assert info["iterations"] == int(full[f"loop_{key}_iterations"])
    assert res.fitness == float(full[f"loop_{key}_best_fitness"])
    want = full[f"loop_{key}_counts"].astype(np.int64)
    from m3d.core import replay_triples  # the library's MT19937 replay (= numpy's, tests/test_abi.py)

    tri, _ = replay_triples(len(c), len(want), state=np.random.RandomState(42).get_state())
    T, _ = s.kabsch3(len(want), triples=tri)
    got = s.score(T, THR * THR, _lib.SCORE_SQUARED).cpu().numpy()
    diff = np.nonzero(got != want)[0]
    assert len(diff) <= 3, diff
    if len(diff):
        pp, qq = src[c[:, 0]], tgt[c[:, 1]]
        To = np.stack([O.kabsch3(pp[tri[h]], qq[tri[h]])[0] for h in diff])
        np.testing.assert_array_equal(s.score(To, THR * THR, _lib.SCORE_SQUARED).cpu().numpy(), want[diff])


def test_fused_hyp16_equals_separate_launch():
    """For a4 batches kabsch3 writes the MFMA screen's per-hypothesis operands itself (ScoreFuse);
    m3d_ransac_score builds them in a separate hyp16 launch.  Both give identical counts for the
    same native hypotheses, at a ragged H whose padding hypotheses are exercised, both comparators,
    several batch sizes."""
    import ctypes

    import torch

    from m3d.core import ptr, stream_handle

    src, tgt, corr, _ = synth.ransac_pair(30011, seed=12, noise_ratio=1.5)
    cs = CorrSet(src, tgt, corr)
    H = 2049 + 30
    T, _ = cs.kabsch3(H, seed=5)
    counts = torch.zeros(H, dtype=torch.int32, device="cuda")
    buf = torch.zeros(64, dtype=torch.int64, device="cuda")
    for mode, thr in ((_lib.SCORE_NORM, 0.45), (_lib.SCORE_SQUARED, 0.45 * 0.45)):
        sep = cs.score(T, thr, mode).cpu().numpy()
        for batch in (1000, 0):
            p = RansacParams(max_iter=H, seed=5, thr=thr, mode=mode, early_stop=False, batch=batch)
            cs.ctx.check(cs.ctx.lib.m3d_ransac_run_async(cs.ctx.h, cs.h, ctypes.byref(p.to_c()), None, ptr(counts),
                                                         ptr(buf), stream_handle()), "run")
            np.testing.assert_array_equal(counts.cpu().numpy(), sep)
    pick = np.arange(0, H, 97)
    pp, qq = src[corr[:, 0]], tgt[corr[:, 1]]
    np.testing.assert_array_equal(cs.score(T, 0.45, _lib.SCORE_NORM).cpu().numpy()[pick],
                                  O.inlier_counts(pp, qq, T.cpu().numpy()[pick], 0.45, 1))


@pytest.mark.parametrize("nc", [3, 5, 2049, 100_000])
def test_one_hypothesis_calls_equal_batched(nc):
    """m3d_kabsch3_one / m3d_ransac_score_one (the per-call drop-in path: operands as kernel
    arguments, results through mapped pinned memory) give the batched kernels' bits."""
    src, tgt, corr, _ = synth.ransac_pair(nc, seed=11, noise_ratio=1.0)
    cs = CorrSet(src, tgt, corr)
    rng = np.random.RandomState(nc)
    n = len(corr)
    tri = np.array([rng.choice(n, 3, replace=False) for _ in range(16)], np.int32)
    T, st = cs.kabsch3(len(tri), triples=tri)
    T, st = T.cpu().numpy(), st.cpu().numpy()
    for h in range(len(tri)):
        T1, s1 = cs.kabsch3_one(tri[h])
        assert s1 == st[h]
        np.testing.assert_array_equal(T1, T[h])
    Ts = np.concatenate([T, np.eye(4)[None], synth.random_rigid(3, rot_range=3.0, trans_range=50.0)[None]])
    for thr, mode in ((0.45, _lib.SCORE_NORM), (0.2025, _lib.SCORE_SQUARED), (1e4, _lib.SCORE_NORM)):
        ref = cs.score(Ts, thr, mode).cpu().numpy()
        got = [cs.score_one(Ts[h], thr, mode) for h in range(len(Ts))]
        np.testing.assert_array_equal(got, ref)


@pytest.fixture(scope="module")
def ply_pair():
    """A synthetic Ply pair through the device preprocessing (ply.py:32-66): two samplings of
    the synthetic surface, the target moved by a known pose (the reference's 3d_data/ scans are
    absent)."""
    from ply import Ply

    T = synth.random_rigid(41, rot_range=0.4, trans_range=0.5)
    a, _ = synth.surface_points(20000, seed=42)
    b, _ = synth.surface_points(20000, seed=43)
    np.random.seed(1)
    return (Ply.from_arrays(a, voxel_size=0.3, preprocess=True),
            Ply.from_arrays(synth.apply(T, b), voxel_size=0.3, preprocess=True))


def test_crash_script_noise_ratios(ply_pair):
    """test_ransac_crash.py:227-236 as asserts: noise ratios 0/1/5/10/100 through
    compute_feature_correspondences give Nc·(1 + r) int32 rows, every index in range, and the
    noise-free rows all present (ransac.py:89-99 appends and shuffles)."""
    from matcher import ransac as M

    src, tgt = ply_pair
    ns, nt = len(src.pcd_down.points), len(tgt.pcd_down.points)
    base = M.compute_feature_correspondences(src, tgt, noise_ratio=0.0)
    assert base.dtype == np.int32 and base.shape == (ns, 2)      # one row per source (no mutual)
    key = lambda c: np.sort(c[:, 0].astype(np.int64) * nt + c[:, 1])
    for r in (0.0, 1.0, 5.0, 10.0, 100.0):
        np.random.seed(int(r) + 7)
        c = M.compute_feature_correspondences(src, tgt, noise_ratio=r)
        assert c.dtype == np.int32 and c.shape == (ns + int(ns * r), 2), (r, c.shape)
        assert c[:, 0].min() >= 0 and c[:, 0].max() < ns and c[:, 1].min() >= 0 and c[:, 1].max() < nt
        # multiset containment of the feature rows: the noise rows are extra
        kc, kb = key(c), key(base)
        pos = np.searchsorted(kc, kb)
        assert np.all(kc[np.minimum(pos, len(kc) - 1)] == kb)
        # the injected rows follow the reference's recipe on the global RNG
        np.random.seed(int(r) + 7)
        ref = O.inject_noise_legacy(base, ns, nt, r)
        np.testing.assert_array_equal(c, ref)


def test_crash_script_numerical_stability(ply_pair):
    """test_ransac_crash.py:239-274 as asserts: 1000 compute_step_transformation +
    evaluate_inlier_ratio(…, 0.3) calls on the Ply pair — every fitness finite (the script asks
    ≥ 95 %), each transform the oracle's (1e-9, rank-2 samples) and each ratio the oracle's exactly,
    and the global RNG advanced by exactly 1000 np.random.choice(n, 3, replace=False) draws."""
    from matcher import ransac as M

    src, tgt = ply_pair
    sp, tp = np.asarray(src.pcd_down.points), np.asarray(tgt.pcd_down.points)
    corr = M.compute_feature_correspondences(src, tgt, noise_ratio=0.0)
    np.random.seed(123)
    ref_rng = np.random.RandomState(123)
    for _ in range(1000):
        res = M.compute_step_transformation(src, tgt, corr)
        f = M.evaluate_inlier_ratio(src, tgt, corr, res.transformation, 0.3)
        assert np.isfinite(f) and np.all(np.isfinite(res.transformation))
        idx = ref_rng.choice(len(corr), 3, replace=False)
        T_ref, _ = O.kabsch3(sp[corr[idx, 0]], tp[corr[idx, 1]])
        if not rank_deficient(sp[corr[idx, 0]], tp[corr[idx, 1]]):
            np.testing.assert_allclose(res.transformation, T_ref, atol=1e-9)
        assert f == O.evaluate_inlier_ratio(sp, tp, corr, res.transformation, 0.3)
    assert np.random.rand() == ref_rng.rand()


def test_crash_script_large_transformation(ply_pair):
    """test_ransac_crash.py:277-294 as an assert: R ×1000 and t = (1000, 1000, 1000) give the
    oracle's ratio on the Ply pair's correspondences (0.0 here, exactly)."""
    from matcher import ransac as M

    src, tgt = ply_pair
    corr = M.compute_feature_correspondences(src, tgt, noise_ratio=0.0)
    big = np.eye(4)
    big[:3, :3] *= 1000.0
    big[:3, 3] = [1000, 1000, 1000]
    f = M.evaluate_inlier_ratio(src, tgt, corr, big, 0.3)
    assert f == O.evaluate_inlier_ratio(src.pcd_down.points, tgt.pcd_down.points, corr, big, 0.3)
    assert f == 0.0


def test_drop_in_sees_in_place_mutation_between_calls():
    """The per-call drop-in caches packed device objects by exact content (m3d.cache): editing
    the caller's arrays IN PLACE between calls (same buffers, same shapes) must give the
    reference's answer for the new contents, never the stale cached one — at Nc = 1e5, where the
    keys come from the library's parallel hash."""
    from matcher import ransac as M
    from ply import Ply

    s, t, corr, T = synth.ransac_pair(100_000, seed=8)
    src, tgt = Ply.from_arrays(s), Ply.from_arrays(t)
    sp, tp = src.pcd_down.points, tgt.pcd_down.points
    assert M.evaluate_inlier_ratio(src, tgt, corr, T, 0.3) == O.evaluate_inlier_ratio(sp, tp, corr, T, 0.3)
    sp[corr[:5000, 0]] += 1.0                       # move 5000 matched source points away
    f1 = M.evaluate_inlier_ratio(src, tgt, corr, T, 0.3)
    assert f1 == O.evaluate_inlier_ratio(sp, tp, corr, T, 0.3) and f1 < 0.96
    corr[:20000, 1] = corr[20000:40000, 1]          # rewire 20000 correspondences in place
    f2 = M.evaluate_inlier_ratio(src, tgt, corr, T, 0.3)
    assert f2 == O.evaluate_inlier_ratio(sp, tp, corr, T, 0.3) and f2 < f1
    tp[:] = tp[::-1].copy()                         # permute the target in place
    f3 = M.evaluate_inlier_ratio(src, tgt, corr, T, 0.3)
    assert f3 == O.evaluate_inlier_ratio(sp, tp, corr, T, 0.3)
    # compute_step_transformation reads the edited rows too
    np.random.seed(3)
    r = M.compute_step_transformation(src, tgt, corr)
    ref_rng = np.random.RandomState(3)
    idx = ref_rng.choice(len(corr), 3, replace=False)
    T_ref, _ = O.kabsch3(sp[corr[idx, 0]], tp[corr[idx, 1]])
    np.testing.assert_allclose(r.transformation, T_ref, atol=1e-9)
