"""C-ABI checks that need no GPU: the library loads, exports every symbol include/m3d.h declares,
and its host-side pieces (MT19937 replay, and the host-compiled copy of the device linear algebra)
agree with the reference's golden vectors / numpy."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

from m3d import _lib

ROOT = Path(__file__).resolve().parents[1]
P = C.POINTER(C.c_double)


def header_symbols():
    text = (ROOT / "include" / "m3d.h").read_text()
    return sorted(set(re.findall(r"\b(m3d_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} missing from the ctypes signature table"
    assert lib.m3d_abi_version() == _lib.ABI_VERSION == 13


def test_no_device_here_is_reported_not_crashed():
    lib = _lib.load()
    n = C.c_int(-1)
    assert lib.m3d_device_count(C.byref(n)) == 0
    if n.value == 0:
        h = C.c_void_p()
        assert lib.m3d_create(0, C.byref(h)) == _lib.M3D_ERR_NODEVICE


@pytest.mark.parametrize("nc", [3, 4, 5, 17, 1000, 65537])
def test_replay_triples_match_numpy_legacy_choice(nc):
    from m3d.core import replay_triples

    rs = np.random.RandomState(1234 + nc)
    st0 = rs.get_state()
    H = 40 if nc > 10000 else 300
    tri, st1 = replay_triples(nc, H, state=st0)
    exp = np.array([rs.choice(nc, 3, replace=False) for _ in range(H)])
    np.testing.assert_array_equal(tri, exp)
    st_np = rs.get_state()
    assert st1[2] == st_np[2]
    np.testing.assert_array_equal(st1[1], st_np[1])


def test_replay_triples_advance_global_rng():
    from m3d.core import replay_triples

    np.random.seed(42)
    tri, _ = replay_triples(5000, 10)
    after = np.random.rand()
    np.random.seed(42)
    exp = np.array([np.random.choice(5000, 3, replace=False) for _ in range(10)])
    np.testing.assert_array_equal(tri, exp)
    assert np.random.rand() == after


@pytest.mark.parametrize("nc", [3, 4, 7, 1024, 1025, 5000, 100000])
def test_choice3_is_numpy_choice_on_the_global_rng(nc):
    """matcher.ransac.compute_step_transformation draws through m3d.core.choice3: the rows of
    np.random.choice(nc, 3, replace=False) (ransac.py:143) and the identical global RNG state."""
    from m3d import core

    np.random.seed(nc)
    exp = [np.random.choice(nc, 3, replace=False) for _ in range(5)]
    st_exp = np.random.get_state()
    np.random.seed(nc)
    got = [core.choice3(nc) for _ in range(5)]
    st = np.random.get_state()
    assert core._choice3_fast, "numpy MT19937 state layout check failed: fast path disabled"
    for a, b in zip(exp, got):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(st_exp[1], st[1])
    assert st_exp[2] == st[2]
    assert np.random.rand() == (np.random.set_state(st_exp) or np.random.rand())


def host_kabsch(a, b):
    lib = _lib.load()
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    T = np.zeros(16)
    rc = lib.m3d_debug_kabsch3_host(a.ctypes.data_as(P), b.ctypes.data_as(P), T.ctypes.data_as(P))
    return T.reshape(4, 4), rc


def test_host_kabsch_matches_reference_kats(golden):
    k = golden("crash_kats.npz")
    for s in range(10):
        T, rc = host_kabsch(k["minimal_src"][s], k["minimal_tgt"][s])
        assert rc == 0
        np.testing.assert_allclose(T, k["minimal_T"][s], atol=1e-12)
    for name, a, b in (("collinear", "collinear_pts", "collinear_pts"),
                       ("coplanar", "coplanar_src", "coplanar_tgt"),
                       ("coplanar_self", "coplanar_src", "coplanar_src"),
                       ("duplicate", "duplicate_pts", "duplicate_pts")):
        T, rc = host_kabsch(k[a][:3], k[b][:3])
        np.testing.assert_allclose(T, k[f"{name}_T"], atol=1e-12, err_msg=name)


@pytest.mark.parametrize("seed", (0, 42))
def test_host_kabsch_matches_reference_5k(golden, pts5k, seed):
    g = golden(f"ransac_5k_seed{seed}.npz")
    src, tgt, corr = pts5k["src"], pts5k["tgt"], pts5k["corr_noise"]
    p, q = src[corr[:, 0]], tgt[corr[:, 1]]
    tri = g["noise_triples"]
    worst, n_rank1 = 0.0, 0
    for h in range(1000):
        T, rc = host_kabsch(p[tri[h]], q[tri[h]])
        assert rc == 0
        if rank_deficient(p[tri[h]], q[tri[h]]):
            # rotation not unique (LAPACK returns rounding noise): pin properness only
            n_rank1 += 1
            R = T[:3, :3]
            np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
            assert abs(np.linalg.det(R) - 1) < 1e-12
            continue
        worst = max(worst, np.abs(T - g["noise_T"][h]).max())
    assert worst < 1e-9, worst
    assert n_rank1 <= 5


def rank_deficient(a, b):
    """3-point sample whose cross-covariance has rank < 2 (collinear or repeated points)."""
    H = (a - a.mean(0)).T @ (b - b.mean(0))
    s = np.linalg.svd(H, compute_uv=False)
    return s[1] <= 1e-10 * s[0]


def test_host_ldlt_matches_dense_solve():
    lib = _lib.load()
    rng = np.random.default_rng(1)
    for _ in range(10):
        J = rng.standard_normal((40, 6))
        A = np.ascontiguousarray(J.T @ J)
        b = rng.standard_normal(6)
        x = np.zeros(6)
        lib.m3d_debug_ldlt6_host(A.ctypes.data_as(P), b.ctypes.data_as(P), x.ctypes.data_as(P))
        np.testing.assert_allclose(x, np.linalg.solve(A, b), rtol=1e-9, atol=1e-12)


def test_host_solve_rule_matches_oracle():
    """The device solve's rule (icp.hip solve_state, through the host-compiled hook): a full-rank
    JᵀJ takes the unpivoted LDLT and agrees with the oracle's pivoted, Eigen-order solve to the
    system's conditioning; an axis the correspondences never excite (a zero column of J, so a zero
    pivot) falls back to the pivoted factorisation and gets the zero component Eigen gives it."""
    import icp_oracle as I

    lib = _lib.load()
    rng = np.random.default_rng(3)

    def solve(A, b):
        x = np.zeros(6)
        rc = lib.m3d_debug_ldlt6_host(np.ascontiguousarray(A).ctypes.data_as(P), b.ctypes.data_as(P),
                                      x.ctypes.data_as(P))
        assert rc == 0
        return x

    for _ in range(20):
        J = rng.standard_normal((50, 6)) * np.array([3.0, 3.0, 3.0, 1.0, 1.0, 1.0])
        A, b = J.T @ J, rng.standard_normal(6)
        np.testing.assert_allclose(solve(A, b), I.ldlt_solve(A, b), rtol=1e-10, atol=1e-13)
    for zero in range(6):
        J = rng.standard_normal((50, 6))
        J[:, zero] = 0.0
        A, b = J.T @ J, rng.standard_normal(6)
        b[zero] = 0.0
        x, ref = solve(A, b), I.ldlt_solve(A, b)
        assert x[zero] == 0.0 and ref[zero] == 0.0
        np.testing.assert_allclose(x, ref, rtol=1e-10, atol=1e-13)


def test_acos_cr_is_correctly_rounded():
    """ddmath.h acos_cr (the FPFH swap test's acos, host-compiled copy of the device code) equals
    acos rounded to nearest from 200-bit mpmath on 20,000 arguments — uniform, near 1 (where acos
    is steep and glibc's own acos misrounds most often) and near 0 — while glibc's math.acos
    does not everywhere (it is not correctly rounded: the reason the swap test needs this)."""
    import math
    import random

    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.prec = 200
    lib = _lib.load()
    rnd = random.Random(11)
    u = np.array([[r, 1 - r * 1e-6, 1 - rnd.random() ** 8, r * 1e-9, 1 - 2.0 ** -53 * (1 + k % 50)][k % 5]
                  for k, r in ((k, rnd.random()) for k in range(20000))])
    out = np.empty_like(u)
    assert lib.m3d_debug_acos_cr(u.ctypes.data_as(C.c_void_p), len(u), out.ctypes.data_as(C.c_void_p)) == 0
    ref = np.array([float(mpmath.acos(mpmath.mpf(x))) for x in u])
    np.testing.assert_array_equal(out, ref)
    assert sum(math.acos(x) != r for x, r in zip(u, ref)) > 0  # glibc misrounds some of them
    edge = np.array([0.0, 1.0, 1.0 + 2.0 ** -52, np.nan])
    out = np.empty_like(edge)
    lib.m3d_debug_acos_cr(edge.ctypes.data_as(C.c_void_p), 4, out.ctypes.data_as(C.c_void_p))
    assert out[0] == math.acos(0.0) and out[1] == 0.0 and np.isnan(out[2]) and np.isnan(out[3])
