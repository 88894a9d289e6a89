"""CPU checks of the preprocessing / feature-matching oracle (oracle/prep_oracle.py).

Open3D is not installed: these pin the restatement by construction —
hand-computed voxels, eigenvector identities, invariances and known-pose recovery — not by
Open3D's own outputs (parity with Open3D unpinned).
"""
import math

import numpy as np
import pytest

import prep_oracle as P
from m3d import synth


def test_voxel_down_sample_hand_example():
    pts = np.array([[0.0, 0.0, 0.0], [0.1, 0.0, 0.0], [1.0, 1.0, 1.0], [0.05, 0.2, 0.1],
                    [1.02, 1.01, 0.99]])
    down, _ = P.voxel_down_sample(pts, 0.5)
    # voxel_min = min − 0.25: (0,0,0),(0.1,0,0),(0.05,0.2,0.1) share voxel (0,0,0); the two near
    # (1,1,1) share voxel (2,2,2)
    np.testing.assert_allclose(down, [[0.05, 0.2 / 3, 0.1 / 3], [1.01, 1.005, 0.995]], rtol=1e-15)


def test_voxel_down_sample_normals_and_order():
    rng = np.random.default_rng(0)
    pts = rng.uniform(-1, 1, (2000, 3))
    nrm = rng.normal(size=(2000, 3))
    down, dn = P.voxel_down_sample(pts, 0.25, nrm)
    vmin = pts.min(0) - 0.125
    keys = np.floor((down - vmin) / 0.25).astype(int)
    assert np.all(np.diff(keys[:, 0]) >= 0)  # ascending ix
    assert len(np.unique(keys, axis=0)) == len(down)
    assert dn.shape == down.shape


def test_fast_eigen3x3_smallest_eigenvector():
    rng = np.random.default_rng(1)
    for _ in range(200):
        A = rng.normal(size=(3, 3))
        C = A @ A.T + np.diag(rng.uniform(0, 1e-3, 3))
        v = P.fast_eigen3x3(C)
        w, V = np.linalg.eigh(C)
        assert abs(abs(np.dot(v, V[:, 0])) - 1.0) < 1e-8
    # degenerate forms: diagonal (norm = 0 branch), zero, planar
    np.testing.assert_array_equal(P.fast_eigen3x3(np.diag([3.0, 1.0, 2.0])), [0, 1, 0])
    np.testing.assert_array_equal(P.fast_eigen3x3(np.zeros((3, 3))), [0, 0, 0])
    np.testing.assert_array_equal(P.fast_eigen3x3(np.eye(3)), [0, 0, 1])


def test_normals_of_plane_and_sphere():
    rng = np.random.default_rng(2)
    plane = np.c_[rng.uniform(-1, 1, (800, 2)), np.zeros(800)]
    n = P.estimate_normals(plane, 0.3, 30)
    np.testing.assert_allclose(np.abs(n[:, 2]), 1.0, atol=1e-12)
    pts, true = synth.surface_points(3000, seed=3)
    n = P.estimate_normals(pts, 0.8, 30, prev_normals=true)
    cos = np.sum(n * true, axis=1)
    assert np.all(cos > 0)  # oriented by the previous normals
    assert np.median(cos) > 0.99


def test_hybrid_search_semantics():
    pts = np.array([[0.0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 0, 0], [3, 0, 0]])
    idx, d2, cnt = P.hybrid_search(pts, 1.0, 3)
    assert cnt.tolist() == [1, 2, 1, 2, 1]  # strict d² < r²: the unit neighbours are excluded
    idx, d2, cnt = P.hybrid_search(pts, 1.5, 3)
    assert idx[0].tolist() == [0, 1, 2]     # ties (d² = 1) ordered by index; max_nn caps at 3
    assert idx[1].tolist() == [1, 3, 0]     # duplicate point first (d² = 0), then by d²


def test_fpfh_histograms_and_rigid_invariance():
    pts, nrm = synth.surface_points(1200, seed=4)
    r = 2.0
    f = P.compute_fpfh(pts, nrm, r, 100)
    nb = P.hybrid_search(pts, r, 100)
    spfh = P.compute_spfh(pts, nrm, nb[0], nb[2])
    ok = nb[2] > 1
    for g in range(3):
        np.testing.assert_allclose(spfh[ok, 11 * g:11 * g + 11].sum(1), 100.0, rtol=1e-12)
        np.testing.assert_allclose(f[ok, 11 * g:11 * g + 11].sum(1), 200.0, rtol=1e-12)
    T = synth.random_rigid(5, rot_range=math.pi, trans_range=3.0)
    f2 = P.compute_fpfh(synth.apply(T, pts), nrm @ T[:3, :3].T, r, 100)
    close = np.all(np.abs(f2 - f) < 1e-6, axis=1)
    assert close.mean() > 0.99  # bin flips only for features on a bin edge


def test_feature_correspondences_and_mutual_fallback():
    rng = np.random.default_rng(6)
    f = rng.uniform(0, 10, (300, 33))
    perm = rng.permutation(300)
    c = P.correspondences_from_features(f, f[perm])
    np.testing.assert_array_equal(perm[c[:, 1]], np.arange(300))
    c = P.correspondences_from_features(f, f[perm], mutual_filter=True)
    assert len(c) == 300
    # a single target feature: every source maps to it, only one pair is mutual → fallback
    c = P.correspondences_from_features(f, f[:1], mutual_filter=True)
    assert len(c) == 300 and np.all(c[:, 1] == 0)


def test_ransac_feature_recovers_pose():
    pts, _ = synth.surface_points(1500, seed=7)
    T = synth.random_rigid(8, rot_range=0.5, trans_range=1.0)
    tgt = synth.apply(T, pts)
    rng = np.random.default_rng(9)
    corr = np.c_[np.arange(1500), np.arange(1500)]
    bad = rng.random(1500) < 0.5  # half of the rows are outliers
    corr[bad, 1] = rng.integers(0, 1500, int(bad.sum()))
    out = P.ransac_feature(pts, tgt, corr, 0.45, lambda h: P.native_rows(42, h, len(corr)),
                           max_iteration=200, edge_length=0.9, distance=0.45)
    assert out["fitness"] > 0.99
    np.testing.assert_allclose(out["transformation"], T, atol=1e-8)
    assert out["validations"] <= 200 and out["best_index"] >= 0


def test_native_rows_with_replacement_range():
    rows = [P.native_rows(1, h, 7) for h in range(2000)]
    flat = np.array(rows).ravel()
    assert flat.min() == 0 and flat.max() == 6
    assert any(len(set(r)) < 3 for r in rows)  # duplicates occur: drawn with replacement


def test_est_k_update_c_semantics():
    """Open3D 0.19's exit update: est_k ← ceil(log(1−c)/log(1−r^n)) when smaller; r = 1 → 0
    (log(0) = −inf gives −0.0), r = 0 → stop (a division by +0.0 gives −inf), NaN leaves it."""
    assert P.est_k_update(30, 1.0, 0.999, 3) == 0
    assert P.est_k_update(30, 0.0, 0.999, 3) == 0
    assert P.est_k_update(30, float("nan"), 0.999, 3) == 30
    k = math.ceil(math.log(0.001) / math.log(1 - 0.3 ** 3))
    assert k == 253 and P.est_k_update(1000, 0.3, 0.999, 3) == 253
    assert P.est_k_update(30, 0.3, 0.999, 3) == 30     # not below the current est_k
    assert P.est_k_update(30, 0.9, 0.999, 3) == math.ceil(math.log(0.001) / math.log(1 - 0.729))


def test_corres_inlier_ratio_counts_input_correspondences():
    pts = np.array([[0.0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]])
    T = np.eye(4)
    T[0, 3] = 0.1
    corr = np.array([[0, 0], [1, 1], [2, 3], [3, 3]])
    # under T: rows 0, 1 and 3 lie 0.1 from their targets; row 2 lies √2-ish away
    assert P.corres_inlier_ratio(pts, pts, corr, 0.2, T) == 0.75
    assert P.corres_inlier_ratio(pts, pts, corr, 0.1, T) == 0.0  # strict <: 0.1² is not below


def test_ransac_feature_exit_follows_corres_ratio_not_fitness():
    """A well-overlapping pair (fitness ≈ 1 at the true pose) with 70 % outlier correspondences:
    the fitness rule exits after a handful of hypotheses, Open3D's correspondence-ratio rule
    (≈ 0.3 → est_k ≈ 253) keeps validating — the two restatements differ."""
    pts, _ = synth.surface_points(1500, seed=7)
    T = synth.random_rigid(8, rot_range=0.5, trans_range=1.0)
    # 0.01 noise: rmse values are then real distances, not rounding noise (an exact copy makes
    # every good hypothesis's rmse ~1e-15, and "lower rmse wins" compares rounding orders)
    tgt = synth.apply(T, pts) + np.random.default_rng(10).normal(scale=0.01, size=pts.shape)
    rng = np.random.default_rng(9)
    corr = np.c_[np.arange(1500), np.arange(1500)]
    bad = rng.random(1500) < 0.7
    corr[bad, 1] = rng.integers(0, 1500, int(bad.sum()))
    kw = dict(max_iteration=400, edge_length=0.9, distance=0.45)
    rows = lambda h: P.native_rows(3, h, len(corr))  # noqa: E731
    new = P.ransac_feature(pts, tgt, corr, 0.45, rows, **kw)
    old = P.ransac_feature(pts, tgt, corr, 0.45, rows, exit_rule="fitness", **kw)
    assert new["fitness"] > 0.98 and old["fitness"] > 0.98
    assert 0.25 < new["corres_ratio"] < 0.35
    assert old["validations"] < 10 < new["validations"]
