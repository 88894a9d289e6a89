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
