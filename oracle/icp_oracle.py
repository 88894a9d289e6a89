"""CPU oracle for the ICP half of the hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module.  The product path never does.

The reference ICP is one call into Open3D 0.19.0 (`src/matcher/icp.py:42-48`:
``registration_icp(src.pcd, tgt.pcd, 0.4·voxel, init, TransformationEstimationPointToPlane())``
with the default ``ICPConvergenceCriteria(1e-6, 1e-6, 30)``).  Open3D is a third-party wheel
(`uv.lock:741-742`) that is neither vendored nor installed here, so this module restates its
published algorithm (Open3D 0.19 ``pipelines/registration/Registration.cpp``,
``TransformationEstimation.cpp``, ``utility/Eigen.cpp``):

* ``registration_result``   — GetRegistrationResultAndCorrespondences: for each source point the
  nearest target strictly inside ``max_correspondence_distance`` (KDTreeFlann::SearchHybrid with
  max_nn = 1; nanoflann's radius result set keeps d² < r²); fitness = pairs/Ns,
  inlier_rmse = sqrt(Σd²/pairs), both 0 when there are no pairs.
* ``point_to_plane_update`` — r = (p−q)·n, J = [p×n ; n], JTJ/JTr/Σr² (ComputeJTJandJTr), solve
  JTJ·x = −JTr (SolveLinearSystemPSD → LDLT), x → Rz(x2)·Ry(x1)·Rx(x0) | t = x[3:6]
  (TransformVector6dToMatrix4d); identity for an empty correspondence set.
* ``point_to_point_update`` — Umeyama without scaling (Eigen::umeyama).
* ``registration_icp``      — the RegistrationICP loop (Registration.cpp): pcd = source, and
  pcd.Transform(init) only when ``!init.isIdentity()`` (``is_identity``: Eigen's dummy precision
  1e-12); Eval(pcd); for i < max_iteration: update from pcd; T ← update·T; pcd.Transform(update)
  (INCREMENTAL — the points are the previous points moved by the update, not T·source); re-Eval;
  break when |Δfitness| < rel_fitness and |Δrmse| < rel_rmse.

PARITY UNPINNED against Open3D itself (no Open3D in this container, and the reference's tests
pin no ICP output).  It is pinned instead by known-R|t recovery on synthetic pairs
(``tests/test_oracle_icp.py``) and the GPU path is checked against it within stated tolerances.

Arithmetic contract (shared with the device, 3d-matching_amd/csrc/nnkey.h):
* ``transform_points`` is Open3D's PointCloud::Transform (Eigen 4×4 · (x, y, z, 1)) in Eigen's
  non-FMA order, ((r0·x + r1·y) + r2·z) + t, written elementwise so that no BLAS kernel (whose
  FMA order depends on the host CPU) decides the rounding;
* d² = ((dx·dx + dy·dy) + dz·dz) in fp64;
* the nearest neighbour is the exact lexicographic (d², index) minimum over the targets with
  d² < r² (nanoflann's radius result set keeps d² < r²; exact ties → lowest index).  scipy's
  ``cKDTree`` proposes candidates; the decision is taken on the d² above (``nn_exact``).
"""

from __future__ import annotations

import numpy as np
from scipy.spatial import cKDTree


def transform_points(T: np.ndarray, pts: np.ndarray) -> np.ndarray:
    """Open3D PointCloud::Transform: ((r0·x + r1·y) + r2·z) + t per row, fp64, no FMA."""
    T = np.asarray(T, np.float64)
    p = np.asarray(pts, np.float64).reshape(-1, 3)
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    out = np.empty_like(p)
    for k in range(3):
        out[:, k] = ((T[k, 0] * x + T[k, 1] * y) + T[k, 2] * z) + T[k, 3]
    return out


def is_identity(T: np.ndarray, prec: float = 1e-12) -> bool:
    """Eigen's Matrix4d::isIdentity(): |a_ii − 1| ≤ prec·min(|a_ii|, 1), |a_ij| ≤ prec (i ≠ j)."""
    T = np.asarray(T, np.float64)
    for i in range(4):
        for j in range(4):
            a = T[i, j]
            if i == j:
                if not abs(a - 1.0) <= prec * min(abs(a), 1.0):
                    return False
            elif not abs(a) <= prec:
                return False
    return True


def matmul4(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """4×4 product with each entry summed ((a0·b0 + a1·b1) + a2·b2) + a3·b3 (no BLAS)."""
    A = np.asarray(A, np.float64)
    B = np.asarray(B, np.float64)
    out = np.empty((4, 4))
    for i in range(4):
        for j in range(4):
            out[i, j] = ((A[i, 0] * B[0, j] + A[i, 1] * B[1, j]) + A[i, 2] * B[2, j]) + A[i, 3] * B[3, j]
    return out


def initial_points(init: np.ndarray, src: np.ndarray) -> np.ndarray:
    """RegistrationICP's pcd before the first evaluation: the source, transformed by init only
    when init is not isIdentity()."""
    src = np.asarray(src, np.float64).reshape(-1, 3)
    return src.copy() if is_identity(init) else transform_points(init, src)


def sq_dist(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """((dx·dx + dy·dy) + dz·dz) row-wise, fp64."""
    d = a - b
    return (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]


def nn_exact(tree: cKDTree, tgt: np.ndarray, q: np.ndarray, max_dist: float, k: int = 8):
    """Radius-bounded exact 1-NN: for every query the lexicographic (d², index) minimum over the
    targets with d² < max_dist² (d² = ``sq_dist``).  Returns (idx int64, -1 = none; d² with inf).

    The kd-tree's own distances may round differently from ``sq_dist``, so k candidates are
    decided on ``sq_dist``; a query whose k-th candidate is not clearly farther than its best (a
    cluster of near-duplicates) is redone with every target inside a slightly larger ball."""
    nq = len(q)
    idx = np.full(nq, -1, np.int64)
    d2 = np.full(nq, np.inf)
    if nq == 0 or len(tgt) == 0 or max_dist <= 0:
        return idx, d2
    r2 = max_dist * max_dist
    k = min(k, len(tgt))
    dd, jj = tree.query(q, k=k, distance_upper_bound=max_dist * (1 + 1e-9), workers=-1)
    dd = dd.reshape(nq, k)
    jj = jj.reshape(nq, k).astype(np.int64)
    valid = jj < len(tgt)
    jc = np.where(valid, jj, 0)
    cand = np.full((nq, k), np.inf)
    for c in range(k):
        cand[:, c] = np.where(valid[:, c], sq_dist(q, tgt[jc[:, c]]), np.inf)
    cand = np.where(cand < r2, cand, np.inf)
    # lexicographic (d², index) minimum over the k candidates
    bd = cand.min(axis=1)
    tie = (cand == bd[:, None]) & np.isfinite(bd)[:, None]
    bj = np.where(tie, jc, np.iinfo(np.int64).max).min(axis=1)
    ok = np.isfinite(bd)
    idx[ok] = bj[ok]
    d2[ok] = bd[ok]
    # near-duplicate clusters: the k-th kd-tree candidate within 1e-9 of the best
    if k < len(tgt):
        dk = dd[:, k - 1]
        crowd = np.nonzero(ok & np.isfinite(dk) & (dk <= np.sqrt(bd) * (1 + 1e-9) + 1e-300))[0]
        for i in crowd:
            js = np.asarray(tree.query_ball_point(q[i], np.sqrt(bd[i]) * (1 + 1e-9) + 1e-300), np.int64)
            dj = sq_dist(np.repeat(q[i:i + 1], len(js), 0), tgt[js])
            m = dj < r2
            js, dj = js[m], dj[m]
            o = np.lexsort((js, dj))[0]
            idx[i], d2[i] = js[o], dj[o]
    return idx, d2


def registration_result(src_t: np.ndarray, tgt: np.ndarray, max_dist: float, tree=None):
    """Return (fitness, inlier_rmse, corr (M×2 int), d2 per source (inf when none))."""
    tree = cKDTree(tgt) if tree is None else tree
    ns = len(src_t)
    if ns == 0 or max_dist <= 0:
        return 0.0, 0.0, np.zeros((0, 2), dtype=np.int64), np.full(ns, np.inf)
    j, d2 = nn_exact(tree, tgt, src_t, max_dist)
    idx = np.nonzero(j >= 0)[0]
    corr = np.stack([idx, j[idx]], axis=1)
    if len(idx) == 0:
        return 0.0, 0.0, corr, d2
    fitness = len(idx) / ns
    rmse = float(np.sqrt(np.sum(d2[idx]) / len(idx)))
    return fitness, rmse, corr, d2


def vec6_to_matrix(x: np.ndarray) -> np.ndarray:
    """TransformVector6dToMatrix4d: AngleAxis(x2,Z)·AngleAxis(x1,Y)·AngleAxis(x0,X), t = x[3:6]."""
    a, b, c = x[0], x[1], x[2]
    rx = np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])
    ry = np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])
    rz = np.array([[np.cos(c), -np.sin(c), 0], [np.sin(c), np.cos(c), 0], [0, 0, 1]])
    T = np.eye(4)
    T[:3, :3] = rz @ ry @ rx
    T[:3, 3] = x[3:6]
    return T


def ldlt_solve(A: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Symmetric-pivoted LDLᵀ solve (Eigen::LDLT semantics: zero pivots give zero components)."""
    n = len(b)
    A = A.astype(np.float64).copy()
    perm = np.arange(n)
    L = np.eye(n)
    D = np.zeros(n)
    # Right-looking LDLT with diagonal pivoting (largest remaining |diag|).
    M = A.copy()
    for k in range(n):
        p = k + int(np.argmax(np.abs(np.diag(M)[k:])))
        if p != k:
            M[[k, p], :] = M[[p, k], :]
            M[:, [k, p]] = M[:, [p, k]]
            L[[k, p], :k] = L[[p, k], :k]
            perm[[k, p]] = perm[[p, k]]
        D[k] = M[k, k]
        if abs(D[k]) > np.finfo(np.float64).tiny:
            L[k + 1:, k] = M[k + 1:, k] / D[k]
        else:
            L[k + 1:, k] = 0.0
        M[k + 1:, k + 1:] -= np.outer(L[k + 1:, k], M[k, k + 1:])
    y = b[perm].astype(np.float64)
    for i in range(n):
        y[i] -= L[i, :i] @ y[:i]
    for i in range(n):
        y[i] = y[i] / D[i] if abs(D[i]) > np.finfo(np.float64).tiny else 0.0
    for i in reversed(range(n)):
        y[i] -= L[i + 1:, i] @ y[i + 1:]
    x = np.empty(n)
    x[perm] = y
    return x


def point_to_plane_terms(src_t, tgt, tgt_n, corr):
    """JTJ (6×6), JTr (6), Σr² over the correspondence set (ComputeJTJandJTr, L2 weights)."""
    vs = src_t[corr[:, 0]]
    vt = tgt[corr[:, 1]]
    nt = tgt_n[corr[:, 1]]
    r = np.sum((vs - vt) * nt, axis=1)
    J = np.concatenate([np.cross(vs, nt), nt], axis=1)
    return J.T @ J, J.T @ r, float(r @ r)


def point_to_plane_update(src_t, tgt, tgt_n, corr) -> np.ndarray:
    if len(corr) == 0:
        return np.eye(4)
    JTJ, JTr, _ = point_to_plane_terms(src_t, tgt, tgt_n, corr)
    return vec6_to_matrix(ldlt_solve(JTJ, -JTr))


def umeyama(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """Eigen::umeyama(src, dst, with_scaling=false) on N×3 arrays."""
    n = len(src)
    ms, md = src.mean(axis=0), dst.mean(axis=0)
    sigma = (dst - md).T @ (src - ms) / n
    U, _, Vt = np.linalg.svd(sigma)
    S = np.ones(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2] = -1
    R = U @ np.diag(S) @ Vt
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = md - R @ ms
    return T


def point_to_point_update(src_t, tgt, corr) -> np.ndarray:
    if len(corr) == 0:
        return np.eye(4)
    return umeyama(src_t[corr[:, 0]], tgt[corr[:, 1]])


def _report(on_eval, k, pcd, corr):
    if on_eval is not None:
        j = np.full(len(pcd), -1, np.int64)
        j[corr[:, 0]] = corr[:, 1]
        on_eval(k, pcd, j)


def registration_icp(src, tgt, max_dist, init=None, tgt_normals=None, estimation="point_to_plane",
                     relative_fitness=1e-6, relative_rmse=1e-6, max_iteration=30, on_eval=None):
    """RegistrationICP (Open3D 0.19).  Returns dict(transformation, fitness, inlier_rmse,
    correspondence_set, iterations (updates applied), history of (fitness, rmse), points (the
    last evaluation's pcd), update (the last update applied; I when none)).
    on_eval(k, pcd, j): called at every evaluation k with its points and per-source winner
    (-1 none) — the tests' per-evaluation comparison."""
    if max_dist <= 0:
        raise ValueError("Invalid max_correspondence_distance.")
    if estimation == "point_to_plane" and tgt_normals is None:
        raise ValueError("TransformationEstimationPointToPlane requires target normals.")
    T = np.eye(4) if init is None else np.asarray(init, dtype=np.float64).copy()
    tree = cKDTree(tgt)
    pcd = initial_points(T, src)
    fit, rmse, corr, _ = registration_result(pcd, tgt, max_dist, tree)
    _report(on_eval, 0, pcd, corr)
    hist = [(fit, rmse)]
    it = 0
    upd = np.eye(4)
    for it in range(1, max_iteration + 1):
        if estimation == "point_to_plane":
            upd = point_to_plane_update(pcd, tgt, tgt_normals, corr)
        else:
            upd = point_to_point_update(pcd, tgt, corr)
        T = matmul4(upd, T)
        pcd = transform_points(upd, pcd)
        bfit, brmse = fit, rmse
        fit, rmse, corr, _ = registration_result(pcd, tgt, max_dist, tree)
        _report(on_eval, it, pcd, corr)
        hist.append((fit, rmse))
        if abs(bfit - fit) < relative_fitness and abs(brmse - rmse) < relative_rmse:
            break
    return dict(transformation=T, fitness=fit, inlier_rmse=rmse, correspondence_set=corr,
                iterations=it, history=hist, points=pcd, update=upd)
