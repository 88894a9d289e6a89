"""Pin the CPU oracle (oracle/ransac_oracle.py) to the reference's own outputs.

The golden vectors were produced by tools/gen_golden.py, which imports the reference's
``src/matcher/ransac.py`` (open3d stubbed) — SURVEY.md §8(c) G1-G3.
"""
import numpy as np
import pytest

import ransac_oracle as O

SEEDS = (0, 1, 42)
SETS = ("clean", "noise")


@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("name", SETS)
def test_replay_triples_match_reference_rng(golden, pts5k, seed, name):
    g = golden(f"ransac_5k_seed{seed}.npz")
    corr = pts5k[f"corr_{name}"]
    tri, _ = O.replay_triples(seed, len(corr), 1000)
    np.testing.assert_array_equal(tri, g[f"{name}_triples"])


@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("name", SETS)
def test_kabsch_and_scores_match_reference(golden, pts5k, seed, name):
    g = golden(f"ransac_5k_seed{seed}.npz")
    src, tgt, corr = pts5k["src"], pts5k["tgt"], pts5k[f"corr_{name}"]
    p_src, p_tgt = src[corr[:, 0]], tgt[corr[:, 1]]
    tri = g[f"{name}_triples"]
    for h in range(0, 1000, 7):
        T, st = O.kabsch3(p_src[tri[h]], p_tgt[tri[h]])
        assert st == O.HYP_OK
        np.testing.assert_array_equal(T, g[f"{name}_T"][h])
    Ts = g[f"{name}_T"][:200]
    thr = float(g["voxel"]) * 1.5
    np.testing.assert_array_equal(O.inlier_counts(p_src, p_tgt, Ts, thr * thr, 0),
                                  g[f"{name}_count_fast"][:200])
    np.testing.assert_array_equal(O.inlier_counts(p_src, p_tgt, Ts, thr, 1),
                                  g[f"{name}_count_slow"][:200])
    for h in range(0, 200, 13):
        assert O.evaluate_inlier_ratio(src, tgt, corr, Ts[h], 0.3) == g[f"{name}_ratio_slow"][h]
        assert O.evaluate_inlier_ratio_fast(p_src, p_tgt, Ts[h], float(g["thr_sq"])) == \
            g[f"{name}_ratio_fast"][h]


def test_compute_step_transformation_consumes_rng_like_reference(golden, pts5k):
    g = golden("ransac_5k_seed42.npz")
    src, tgt, corr = pts5k["src"], pts5k["tgt"], pts5k["corr_noise"]
    np.random.seed(42)
    for h in range(20):
        T, st, idx = O.compute_step_transformation(src, tgt, corr)
        np.testing.assert_array_equal(idx, g["noise_triples"][h])
        np.testing.assert_array_equal(T, g["noise_T"][h])


def test_crash_kats(golden):
    k = golden("crash_kats.npz")
    c3 = np.array([[0, 0], [1, 1], [2, 2]])
    for s in range(10):
        T, st = O.kabsch3(k["minimal_src"][s], k["minimal_tgt"][s])
        np.testing.assert_allclose(T, k["minimal_T"][s], atol=1e-13)
    for name, a, b in (("collinear", "collinear_pts", "collinear_pts"),
                       ("coplanar", "coplanar_src", "coplanar_tgt"),
                       ("coplanar_self", "coplanar_src", "coplanar_src"),
                       ("duplicate", "duplicate_pts", "duplicate_pts")):
        T, st = O.kabsch3(k[a][:3], k[b][:3])
        np.testing.assert_allclose(T, k[f"{name}_T"], atol=1e-12)
    assert k["zero_corr_ratio"] == 0.0
    T, st, _ = O.compute_step_transformation(np.zeros((10, 3)), np.zeros((10, 3)), c3[:2])
    assert st == O.HYP_DEGENERATE
    np.testing.assert_array_equal(T, k["two_corr_T"])


def test_crash_kat_ratios(golden, pts5k):
    k = golden("crash_kats.npz")
    src, tgt = pts5k["src"], pts5k["tgt"]
    for key, corr, T in (("large_ratio_clean", "corr_clean", k["large_T"]),
                         ("identity_ratio_clean", "corr_clean", np.eye(4)),
                         ("true_ratio_clean", "corr_clean", pts5k["T_true"]),
                         ("true_ratio_noise", "corr_noise", pts5k["T_true"])):
        assert O.evaluate_inlier_ratio(src, tgt, pts5k[corr], T, 0.3) == k[key]


@pytest.mark.parametrize("name", ("clean", "noise", "mid"))
def test_loop_trajectory(golden, pts5k, name):
    t = golden("loop_trajectory.npz")
    src, tgt, corr = pts5k["src"], pts5k["tgt"], pts5k[f"corr_{name}"]
    p_src, p_tgt = src[corr[:, 0]], tgt[corr[:, 1]]
    max_iter = int(t[f"{name}_max_iter"])
    tri, _ = O.replay_triples(int(t[f"{name}_seed"]), len(corr), max_iter)
    thr = 0.3 * 1.5
    bi, bf, it, counts, _ = O.ransac_loop(p_src, p_tgt, tri, thr * thr, max_iter)
    assert (bi, bf, it) == (int(t[f"{name}_best_index"]), float(t[f"{name}_best_fitness"]),
                            int(t[f"{name}_iterations"]))
    np.testing.assert_array_equal(counts / len(corr), t[f"{name}_fitness"])
    assert O.select_best(counts, len(corr), max_iter) == (bi, bf, it)


def test_noise_injection_recipe(pts5k):
    """a5 outlier injection restated on the legacy RNG reproduces the reference's corr set."""
    n = len(pts5k["src"])
    ident = np.stack([np.arange(n)] * 2, axis=1).astype(np.int32)
    np.random.seed(7)
    out = O.inject_noise_legacy(ident, n, n, 2.0)
    np.testing.assert_array_equal(out, pts5k["corr_noise"])
    np.random.seed(11)
    np.testing.assert_array_equal(O.inject_noise_legacy(ident, n, n, 0.6), pts5k["corr_mid"])


def test_native_sampler_properties():
    tri = O.native_triples(42, 0, 4000, 100)
    assert tri.min() >= 0 and tri.max() < 100
    assert np.all((tri[:, 0] != tri[:, 1]) & (tri[:, 0] != tri[:, 2]) & (tri[:, 1] != tri[:, 2]))
    np.testing.assert_array_equal(O.native_triples(42, 100, 50, 100), tri[100:150])
    small = O.native_triples(7, 0, 300, 3)
    assert np.all(np.sort(small, axis=1) == [0, 1, 2])
    # uniformity sanity
    big = O.native_triples(1, 0, 20000, 10)
    cnt = np.bincount(big.ravel(), minlength=10)
    assert cnt.min() > 0.9 * cnt.mean()


# ---------------------------------------------------------------- cfg2 scale (Nc = 1e5)
from golden_pairs import cfg2_pair  # noqa: E402


def test_cfg2_golden_pins_oracle(golden):
    """The oracle restatement reproduces the reference's own cfg2-scale calls: sampled rows
    (legacy RNG), transforms and both comparators' counts (first 25 of each set)."""
    g, src, tgt, corr, noise = cfg2_pair(golden)
    for key, c, seed in (("s42", corr, 42), ("s7", corr, 7), ("noise", noise, 42)):
        rng = np.random.RandomState(seed)
        p, q = src[c[:, 0]], tgt[c[:, 1]]
        for h in range(25):
            T, _, idx = O.compute_step_transformation(src, tgt, c, rng=rng)
            np.testing.assert_array_equal(idx, g[f"{key}_triples"][h])
            np.testing.assert_allclose(T, g[f"{key}_T"][h], rtol=0, atol=1e-12)
            assert O.inlier_count(p, q, g[f"{key}_T"][h], 0.45, 1) == g[f"{key}_count_slow"][h]
            assert O.inlier_count(p, q, g[f"{key}_T"][h], 0.45 * 0.45, 0) == g[f"{key}_count_fast"][h]
