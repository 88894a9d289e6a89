"""ICP oracle self-checks (parity vs Open3D unpinned: Open3D is absent).

Pinned by: LDLT agrees with a dense solve, vec6→matrix composes Rz·Ry·Rx, and point-to-plane /
point-to-point ICP recover a known rigid transform on synthetic pairs.
"""
import numpy as np
import pytest

import icp_oracle as I
from m3d import synth


def test_ldlt_matches_dense_solve():
    rng = np.random.default_rng(0)
    for _ in range(20):
        J = rng.standard_normal((50, 6))
        A = J.T @ J
        b = rng.standard_normal(6)
        np.testing.assert_allclose(I.ldlt_solve(A, b), np.linalg.solve(A, b), rtol=1e-9, atol=1e-12)


def test_ldlt_zero_pivot_gives_zero_component():
    A = np.diag([2.0, 0.0, 1.0, 3.0, 0.0, 4.0])
    x = I.ldlt_solve(A, np.ones(6))
    np.testing.assert_allclose(x, [0.5, 0, 1, 1 / 3, 0, 0.25])


def test_vec6_to_matrix_is_zyx():
    x = np.array([0.1, -0.2, 0.3, 1.0, 2.0, 3.0])
    T = I.vec6_to_matrix(x)
    np.testing.assert_allclose(T[:3, :3], synth.euler_zyx(x[:3]), atol=1e-15)
    np.testing.assert_array_equal(T[:3, 3], x[3:])


@pytest.mark.parametrize("estimation", ["point_to_plane", "point_to_point"])
def test_icp_recovers_known_pose(estimation):
    src, tgt, nrm, T_true = synth.icp_pair(20000, seed=3)
    if estimation == "point_to_point":  # p2p crawls on independent samplings: use the same one
        src = synth.apply(np.linalg.inv(T_true), tgt)
    res = I.registration_icp(src, tgt, 0.12, init=np.eye(4), tgt_normals=nrm, estimation=estimation,
                             max_iteration=150)
    T = res["transformation"]
    assert res["fitness"] > 0.9
    np.testing.assert_allclose(T[:3, :3], T_true[:3, :3], atol=2e-3)
    np.testing.assert_allclose(T[:3, 3], T_true[:3, 3], atol=2e-2)


def test_registration_result_empty():
    fit, rmse, corr, _ = I.registration_result(np.zeros((5, 3)), np.ones((4, 3)) * 10, 0.1)
    assert fit == 0.0 and rmse == 0.0 and len(corr) == 0


def test_is_identity_is_eigens_fuzzy_test():
    T = np.eye(4)
    assert I.is_identity(T)
    for (i, j), e in [((0, 1), 5e-13), ((2, 2), 5e-13), ((3, 3), -5e-13), ((1, 3), -1e-12)]:
        U = T.copy()
        U[i, j] += e
        assert I.is_identity(U), (i, j, e)
    for (i, j), e in [((0, 1), 2e-12), ((2, 2), 2e-12), ((0, 3), 1e-9)]:
        U = T.copy()
        U[i, j] += e
        assert not I.is_identity(U), (i, j, e)


def test_initial_points_follow_registration_icp():
    """pcd = source, and pcd.Transform(init) only when init is not isIdentity(): an init within
    1e-12 of I leaves the points untouched (bit for bit), any other init moves them."""
    src, _ = synth.surface_points(1000, seed=1)
    near = np.eye(4)
    near[0, 3] = 4e-13
    np.testing.assert_array_equal(I.initial_points(near, src), src)
    T = synth.random_rigid(2, rot_range=0.01, trans_range=0.01)
    np.testing.assert_array_equal(I.initial_points(T, src), I.transform_points(T, src))


def test_registration_icp_points_are_incremental():
    """The evaluated points are the previous points moved by each update (pcd.Transform(update)),
    not T·source: the oracle's final points equal the fold of its updates over the source, and
    differ in the last bits from T·source (the two forms round differently)."""
    src, tgt, nrm, _ = synth.icp_pair(5000, seed=8)
    T0 = synth.random_rigid(4, rot_range=0.01, trans_range=0.01)
    pts = I.initial_points(T0, src)
    T = T0
    for n in range(1, 5):
        res = I.registration_icp(src, tgt, 0.12, init=T0, tgt_normals=nrm, relative_fitness=-1,
                                 relative_rmse=-1, max_iteration=n)
        pts = I.transform_points(res["update"], pts)
        T = I.matmul4(res["update"], T)
        np.testing.assert_array_equal(res["points"], pts)
        np.testing.assert_array_equal(res["transformation"], T)
    assert np.any(res["points"] != I.transform_points(res["transformation"], src))
    np.testing.assert_allclose(res["points"], I.transform_points(res["transformation"], src), atol=1e-12)
