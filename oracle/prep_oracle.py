"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the preprocessing and feature-matching rows:
SURVEY.md §8(f) ranks 2-3 and §8(a) a5 (FPFH half) / a6.

The reference calls Open3D 0.19 for all of these (``src/ply/ply.py:106-120``,
``src/matcher/ransac.py:41-58,85``).  Open3D is not installed and not vendored,
so this module restates its published algorithms — **parity against Open3D itself is
unpinned**; the GPU path is checked against this restatement:

* ``voxel_down_sample``  — ``PointCloud::VoxelDownSample``: voxel_min = min_bound − v/2,
  index = floor((p − voxel_min)/v), per-voxel mean of the points (and normals) accumulated in
  input order.  Open3D emits voxels in ``unordered_map`` order (unspecified); here and on the
  device they come in ascending (ix, iy, iz) order.
* ``hybrid_search``      — ``KDTreeFlann::SearchHybrid(p, r, max_nn)`` (nanoflann radius search,
  strict d² < r², sorted by distance, first max_nn).  fp64 d² = (dx² + dy²) + dz²; exact ties
  are ordered by index (nanoflann leaves them unspecified).
* ``estimate_normals``   — ``PointCloud::EstimateNormals`` with ``ComputeCovariance`` (one-pass
  cumulants in neighbour order, identity below 3 neighbours) and ``FastEigen3x3`` (Eberly's
  robust symmetric 3×3 eigensolver, smallest-eigenvalue vector), re-oriented to agree with
  existing normals.
* ``compute_fpfh``       — ``ComputeFPFHFeature`` / ``ComputeSPFHFeature`` /
  ``ComputePairFeatures``: 3 × 11-bin SPFH with increments 100/(k−1), FPFH = Σ spfh_j / d²_j
  normalised per 11-bin group to 100, + own SPFH.  Layout here: N×33 (Open3D: 33×N).
* ``correspondences_from_features`` — ``CorrespondencesFromFeatures`` (exact 33-D 1-NN, optional
  mutual filter with the 0.1·Ns fallback).
* ``ransac_feature``     — ``RegistrationRANSACBasedOnCorrespondence`` restated sequentially:
  ransac_n rows drawn WITH replacement, Umeyama (PointToPoint, no scaling), EdgeLength and
  Distance checkers, validation = 1-NN within max_corr over all source points, best =
  IsBetterRANSACThan, early exit k = ceil(log(1−c)/log(1−ratio^n)) with ratio = the new best's
  CORRESPONDENCE inlier ratio (``EvaluateInlierCorrespondenceRatio``: the share of the input
  correspondences within max_corr under T — not the fitness; rounds 1–3 used the fitness here,
  fixed in round 4).  Open3D draws rows from a
  global RNG under OpenMP (non-deterministic); here the rows are an input (the device's counter
  sampler, restated in ``native_rows``).
"""

from __future__ import annotations

import math

import numpy as np
from scipy.spatial import cKDTree

MASK64 = (1 << 64) - 1


# ------------------------------------------------------------------------------------- voxel
def voxel_down_sample(points, voxel, normals=None):
    p = np.asarray(points, np.float64)
    if len(p) == 0:
        return np.zeros((0, 3)), (None if normals is None else np.zeros((0, 3)))
    vmin = p.min(axis=0) - voxel * 0.5
    idx = np.floor((p - vmin) / voxel).astype(np.int64)
    # ascending (ix, iy, iz) lexicographic (primary key ix), input order within a voxel
    order =np.lexsort((np.arange(len(p)), idx[:, 2], idx[:, 1], idx[:, 0]))
    si = idx[order]
    new = np.ones(len(p), bool)
    new[1:] = np.any(si[1:] != si[:-1], axis=1)
    starts = np.nonzero(new)[0]
    counts = np.diff(np.append(starts, len(p)))

    def seg_mean(a):
        a = a[order]
        acc = np.zeros((len(starts), 3))
        for k in range(int(counts.max())):     # sequential per voxel, in input order
            m = counts > k
            acc[m] += a[starts[m] + k]
        return acc / counts[:, None].astype(np.float64)

    # AccumulatedPoint::AddPoint skips a normal with a NaN component; the mean still divides by
    # every point of the voxel (GetAverageNormal, no re-normalisation)
    if normals is None:
        out_n = None
    else:
        nr = np.asarray(normals, np.float64)
        out_n = seg_mean(np.where(np.isnan(nr).any(axis=1)[:, None], 0.0, nr))
    return seg_mean(p), out_n


# ------------------------------------------------------------------------------------- search
def d2_exact(a, b):
    d = a - b
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def hybrid_search(points, radius, max_nn, queries=None):
    """→ (idx N×max_nn int32 (−1 pad), d2 N×max_nn f64, count N)."""
    p = np.asarray(points, np.float64)
    q = p if queries is None else np.asarray(queries, np.float64)
    tree = cKDTree(p)
    cand = tree.query_ball_point(q, radius * (1 + 1e-9) + 1e-300)
    idx = np.full((len(q), max_nn), -1, np.int32)
    d2 = np.zeros((len(q), max_nn))
    cnt = np.zeros(len(q), np.int64)
    r2 = radius * radius
    for i, c in enumerate(cand):
        c = np.asarray(c, np.int64)
        dd = d2_exact(p[c], q[i])
        keep = dd < r2
        c, dd = c[keep], dd[keep]
        o = np.lexsort((c, dd))[:max_nn]
        cnt[i] = len(o)
        idx[i, : len(o)] = c[o]
        d2[i, : len(o)] = dd[o]
    return idx, d2, cnt


# ------------------------------------------------------------------------------------- normals
def covariance(points, idx, cnt):
    """ComputeCovariance (Open3D utility/Eigen.cpp): cumulants in neighbour order."""
    n = len(idx)
    cum = np.zeros((n, 9))
    for s in range(idx.shape[1]):
        m = cnt > s
        if not m.any():
            break
        x = points[idx[m, s]]
        cum[m, 0] += x[:, 0]
        cum[m, 1] += x[:, 1]
        cum[m, 2] += x[:, 2]
        cum[m, 3] += x[:, 0] * x[:, 0]
        cum[m, 4] += x[:, 0] * x[:, 1]
        cum[m, 5] += x[:, 0] * x[:, 2]
        cum[m, 6] += x[:, 1] * x[:, 1]
        cum[m, 7] += x[:, 1] * x[:, 2]
        cum[m, 8] += x[:, 2] * x[:, 2]
    cum = cum / np.maximum(cnt, 1)[:, None].astype(np.float64)
    C = np.zeros((n, 3, 3))
    C[:, 0, 0] = cum[:, 3] - cum[:, 0] * cum[:, 0]
    C[:, 1, 1] = cum[:, 6] - cum[:, 1] * cum[:, 1]
    C[:, 2, 2] = cum[:, 8] - cum[:, 2] * cum[:, 2]
    C[:, 0, 1] = C[:, 1, 0] = cum[:, 4] - cum[:, 0] * cum[:, 1]
    C[:, 0, 2] = C[:, 2, 0] = cum[:, 5] - cum[:, 0] * cum[:, 2]
    C[:, 1, 2] = C[:, 2, 1] = cum[:, 7] - cum[:, 1] * cum[:, 2]
    C[cnt < 3] = np.eye(3)
    return C


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]])


def _dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def _eigvec0(A, e):
    r0 = np.array([A[0, 0] - e, A[0, 1], A[0, 2]])
    r1 = np.array([A[0, 1], A[1, 1] - e, A[1, 2]])
    r2 = np.array([A[0, 2], A[1, 2], A[2, 2] - e])
    r0xr1, r0xr2, r1xr2 = _cross(r0, r1), _cross(r0, r2), _cross(r1, r2)
    d0, d1, d2 = _dot(r0xr1, r0xr1), _dot(r0xr2, r0xr2), _dot(r1xr2, r1xr2)
    dmax, imax = d0, 0
    if d1 > dmax:
        dmax, imax = d1, 1
    if d2 > dmax:
        imax = 2
    if imax == 0:
        return r0xr1 / math.sqrt(d0)
    if imax == 1:
        return r0xr2 / math.sqrt(d1)
    return r1xr2 / math.sqrt(d2)


def _eigvec1(A, ev0, e1):
    if abs(ev0[0]) > abs(ev0[1]):
        inv = 1.0 / math.sqrt(ev0[0] * ev0[0] + ev0[2] * ev0[2])
        U = np.array([-ev0[2] * inv, 0.0, ev0[0] * inv])
    else:
        inv = 1.0 / math.sqrt(ev0[1] * ev0[1] + ev0[2] * ev0[2])
        U = np.array([0.0, ev0[2] * inv, -ev0[1] * inv])
    V = _cross(ev0, U)
    AU = np.array([A[0, 0] * U[0] + A[0, 1] * U[1] + A[0, 2] * U[2],
                   A[0, 1] * U[0] + A[1, 1] * U[1] + A[1, 2] * U[2],
                   A[0, 2] * U[0] + A[1, 2] * U[1] + A[2, 2] * U[2]])
    AV = np.array([A[0, 0] * V[0] + A[0, 1] * V[1] + A[0, 2] * V[2],
                   A[0, 1] * V[0] + A[1, 1] * V[1] + A[1, 2] * V[2],
                   A[0, 2] * V[0] + A[1, 2] * V[1] + A[2, 2] * V[2]])
    m00 = U[0] * AU[0] + U[1] * AU[1] + U[2] * AU[2] - e1
    m01 = U[0] * AV[0] + U[1] * AV[1] + U[2] * AV[2]
    m11 = V[0] * AV[0] + V[1] * AV[1] + V[2] * AV[2] - e1
    a00, a01, a11 = abs(m00), abs(m01), abs(m11)
    if a00 >= a11:
        if max(a00, a01) > 0:
            if a00 >= a01:
                m01 /= m00
                m00 = 1.0 / math.sqrt(1.0 + m01 * m01)
                m01 *= m00
            else:
                m00 /= m01
                m01 = 1.0 / math.sqrt(1.0 + m00 * m00)
                m00 *= m01
            return m01 * U - m00 * V
        return U
    if max(a11, a01) > 0:
        if a11 >= a01:
            m01 /= m11
            m11 = 1.0 / math.sqrt(1.0 + m01 * m01)
            m01 *= m11
        else:
            m11 /= m01
            m01 = 1.0 / math.sqrt(1.0 + m11 * m11)
            m11 *= m01
        return m11 * U - m01 * V
    return U


def fast_eigen3x3(cov):
    """Open3D FastEigen3x3 (Eberly, RobustEigenSymmetric3x3): eigenvector of the smallest
    eigenvalue (not normalised to a sign)."""
    A = np.array(cov, np.float64)
    mx = A.max()
    if mx == 0:
        return np.zeros(3)
    A = A / mx
    norm = A[0, 1] * A[0, 1] + A[0, 2] * A[0, 2] + A[1, 2] * A[1, 2]
    if norm > 0:
        q = (A[0, 0] + A[1, 1] + A[2, 2]) / 3
        b00, b11, b22 = A[0, 0] - q, A[1, 1] - q, A[2, 2] - q
        p = math.sqrt((b00 * b00 + b11 * b11 + b22 * b22 + norm * 2) / 6)
        c00 = b11 * b22 - A[1, 2] * A[1, 2]
        c01 = A[0, 1] * b22 - A[1, 2] * A[0, 2]
        c02 = A[0, 1] * A[1, 2] - b11 * A[0, 2]
        det = (b00 * c00 - A[0, 1] * c01 + A[0, 2] * c02) / (p * p * p)
        half_det = min(max(det * 0.5, -1.0), 1.0)
        angle = math.acos(half_det) / 3.0
        two_thirds_pi = 2.09439510239319549
        beta2 = math.cos(angle) * 2
        beta0 = math.cos(angle + two_thirds_pi) * 2
        beta1 = -(beta0 + beta2)
        e0, e1, e2 = q + p * beta0, q + p * beta1, q + p * beta2
        if half_det >= 0:
            v2 = _eigvec0(A, e2)
            if e2 < e0 and e2 < e1:
                return v2
            v1 = _eigvec1(A, v2, e1)
            if e1 < e0 and e1 < e2:
                return v1
            return _cross(v1, v2)
        v0 = _eigvec0(A, e0)
        if e0 < e1 and e0 < e2:
            return v0
        v1 = _eigvec1(A, v0, e1)
        if e1 < e0 and e1 < e2:
            return v1
        return _cross(v0, v1)
    if A[0, 0] < A[1, 1] and A[0, 0] < A[2, 2]:
        return np.array([1.0, 0.0, 0.0])
    if A[1, 1] < A[0, 0] and A[1, 1] < A[2, 2]:
        return np.array([0.0, 1.0, 0.0])
    return np.array([0.0, 0.0, 1.0])


def estimate_normals(points, radius, max_nn, prev_normals=None, nbrs=None):
    p = np.asarray(points, np.float64)
    idx, _, cnt = nbrs if nbrs is not None else hybrid_search(p, radius, max_nn)
    C = covariance(p, idx, cnt)
    out = np.zeros_like(p)
    for i in range(len(p)):
        n = fast_eigen3x3(C[i])
        if n[0] == 0 and n[1] == 0 and n[2] == 0:
            n = prev_normals[i].copy() if prev_normals is not None else np.array([0.0, 0.0, 1.0])
        if prev_normals is not None and _dot(n, prev_normals[i]) < 0.0:
            n = -n
        out[i] = n
    return out


# ------------------------------------------------------------------------------------- FPFH
def pair_features(p1, n1, p2, n2):
    """ComputePairFeatures (Open3D Feature.cpp) → (f0, f1, f2, f3)."""
    dp = p2 - p1
    f3 = math.sqrt(_dot(dp, dp))
    if f3 == 0.0:
        return (0.0, 0.0, 0.0, 0.0)
    a1 = _dot(n1, dp) / f3
    a2 = _dot(n2, dp) / f3
    if math.acos(abs(a1)) > math.acos(abs(a2)):
        n1, n2 = n2, n1
        dp = -dp
        f2 = -a2
    else:
        f2 = a1
    v = _cross(dp, n1)
    vn = math.sqrt(_dot(v, v))
    if vn == 0.0:
        return (0.0, 0.0, 0.0, 0.0)
    v = v / vn
    w = _cross(n1, v)
    return (math.atan2(_dot(w, n2), _dot(n1, n2)), _dot(v, n2), f2, f3)


def _bin(x):
    return min(max(int(math.floor(x)), 0), 10)


def compute_spfh(points, normals, idx, cnt):
    n = len(points)
    spfh = np.zeros((n, 33))
    for i in range(n):
        c = int(cnt[i])
        if c <= 1:
            continue
        incr = 100.0 / (c - 1)
        for k in range(1, c):
            j = idx[i, k]
            f = pair_features(points[i], normals[i], points[j], normals[j])
            spfh[i, _bin(11 * (f[0] + math.pi) / (2.0 * math.pi))] += incr
            spfh[i, 11 + _bin(11 * (f[1] + 1.0) * 0.5)] += incr
            spfh[i, 22 + _bin(11 * (f[2] + 1.0) * 0.5)] += incr
    return spfh


def spfh_edge_sensitive(points, normals, idx, cnt, delta=1e-12, delta_swap=2e-15):
    """Test aid for the FPFH parity bar: True for a point whose SPFH may legitimately differ
    between two correct fp64 implementations — one of its pair features lands within ``delta``
    of a bin edge (the bin arguments 11·(f0 + π)/2π, 11·(f1 + 1)/2, 11·(f2 + 1)/2), or the
    source/target swap test acos|a1| > acos|a2| has ||a1| − |a2|| < ``delta_swap``.  acos /
    atan2 of two libms (numpy's and the device's ocml) may differ by an ulp or two (≈ 1e-16
    relative: acos near π/2 has slope ≈ 1, so ≥ 10 ulps of acos for the swap test), which can
    move only such a feature across the edge."""
    p = np.asarray(points, np.float64)
    nr = np.asarray(normals, np.float64)
    out = np.zeros(len(p), bool)
    for i in range(len(p)):
        c = int(cnt[i])
        for k in range(1, c):
            j = idx[i, k]
            dp = p[j] - p[i]
            f3 = math.sqrt(_dot(dp, dp))
            if f3 == 0.0:
                continue
            a1, a2 = _dot(nr[i], dp) / f3, _dot(nr[j], dp) / f3
            if abs(abs(a1) - abs(a2)) < delta_swap:
                out[i] = True
                break
            f = pair_features(p[i], nr[i], p[j], nr[j])
            xs = (11 * (f[0] + math.pi) / (2.0 * math.pi), 11 * (f[1] + 1.0) * 0.5, 11 * (f[2] + 1.0) * 0.5)
            if any(abs(x - round(x)) < delta for x in xs):
                out[i] = True
                break
    return out


def compute_fpfh(points, normals, radius, max_nn, nbrs=None):
    p = np.asarray(points, np.float64)
    nr = np.asarray(normals, np.float64)
    idx, d2, cnt = nbrs if nbrs is not None else hybrid_search(p, radius, max_nn)
    spfh = compute_spfh(p, nr, idx, cnt)
    out = np.zeros((len(p), 33))
    for i in range(len(p)):
        c = int(cnt[i])
        if c <= 1:
            continue
        s = [0.0, 0.0, 0.0]
        f = np.zeros(33)
        for k in range(1, c):
            dist = d2[i, k]
            if dist == 0.0:
                continue
            row = spfh[idx[i, k]]
            for j in range(33):
                val = row[j] / dist
                s[j // 11] += val
                f[j] += val
        for g in range(3):
            if s[g] != 0.0:
                s[g] = 100.0 / s[g]
        for j in range(33):
            f[j] *= s[j // 11]
            f[j] += spfh[i, j]
        out[i] = f
    return out


# ------------------------------------------------------------------------------------- matching
def feature_nn(fq, fr):
    """Exact 33-D 1-NN of every row of fq in fr (fp64 Σ(a−b)² in dimension order; ties → lowest
    index)."""
    fq = np.asarray(fq, np.float64)
    fr = np.asarray(fr, np.float64)
    out = np.zeros(len(fq), np.int64)
    for a in range(0, len(fq), 256):
        blk = fq[a:a + 256]
        d = np.zeros((len(blk), len(fr)))
        for j in range(fq.shape[1]):
            t = blk[:, j, None] - fr[None, :, j]
            d += t * t
        out[a:a + 256] = np.argmin(d, axis=1)   # argmin: first (lowest) index on ties
    return out


def correspondences_from_features(fsrc, ftgt, mutual_filter=False, mutual_consistent_ratio=0.1):
    ij = feature_nn(fsrc, ftgt)
    c0 = np.stack([np.arange(len(fsrc)), ij], axis=1).astype(np.int32)
    if not mutual_filter:
        return c0
    ji = feature_nn(ftgt, fsrc)
    keep = ji[ij] == np.arange(len(fsrc))
    cm = c0[keep]
    if len(cm) >= int(mutual_consistent_ratio * len(fsrc)):
        return cm
    return c0


# ------------------------------------------------------------------------------------- a6 RANSAC
def _splitmix64(x):
    z = (x + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def native_rows(seed, h, nc, n=3):
    """Device sampler WITH replacement (Open3D draws ransac_n rows independently):
    row k = ((splitmix64(splitmix64(seed ^ h·φ) + k) >> 32) · nc) >> 32."""
    base = _splitmix64((seed ^ ((h * 0x9E3779B97F4A7C15) & MASK64)) & MASK64)
    return [(((_splitmix64((base + k) & MASK64) >> 32) * nc) >> 32) for k in range(n)]


def umeyama(src, dst):
    """Eigen::umeyama without scaling (TransformationEstimationPointToPoint)."""
    sm, dm = src.mean(axis=0), dst.mean(axis=0)
    sigma = (dst - dm).T @ (src - sm) / len(src)
    U, _, Vt = np.linalg.svd(sigma)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1
    R = U @ S @ Vt
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = dm - R @ sm
    return T


def check_edge_length(ps, pt, thr):
    for i in range(len(ps)):
        for j in range(i + 1, len(ps)):
            ds = math.sqrt(_dot(ps[i] - ps[j], ps[i] - ps[j]))
            dt = math.sqrt(_dot(pt[i] - pt[j], pt[i] - pt[j]))
            if ds < dt * thr or dt < ds * thr:
                return False
    return True


def check_distance(ps, pt, T, thr):
    for a, b in zip(ps, pt):
        x = T[:3, :3] @ a + T[:3, 3]
        if math.sqrt(_dot(b - x, b - x)) > thr:
            return False
    return True


def evaluate(src, tgt, T, max_corr, tree=None):
    """GetRegistrationResultAndCorrespondences: fitness, rmse of 1-NN within max_corr (the exact
    fp64 contract of icp_oracle.registration_result)."""
    import icp_oracle

    fit, rmse, _, _ = icp_oracle.registration_result(icp_oracle.transform_points(T, src), tgt,
                                                     max_corr, tree or cKDTree(tgt))
    return fit, rmse


def corres_inlier_ratio(src, tgt, corres, max_corr, T):
    """Open3D 0.19 EvaluateInlierCorrespondenceRatio (Registration.cpp, static): the share of the
    INPUT correspondences c with |T·p_c − q_c|² < max_corr² — the source transformed as
    PointCloud::Transform does (``icp_oracle.transform_points``), squaredNorm as
    ``icp_oracle.sq_dist``, strict <."""
    import icp_oracle

    corres = np.asarray(corres, np.int64).reshape(-1, 2)
    if len(corres) == 0:
        return 0.0
    pcd = icp_oracle.transform_points(T, np.asarray(src, np.float64)[corres[:, 0]])
    d2 = icp_oracle.sq_dist(pcd, np.asarray(tgt, np.float64)[corres[:, 1]])
    return int(np.count_nonzero(d2 < max_corr * max_corr)) / len(corres)


def est_k_update(est_k, ratio, confidence, ransac_n):
    """Open3D 0.19's exit update after a new best (RegistrationRANSACBasedOnCorrespondence):
    ``est_k_d = log(1 − confidence) / log(1 − pow(ratio, ransac_n))``, and est_k ← ceil(est_k_d)
    when est_k_d < est_k.  C semantics: ratio = 1 gives log(0) = −inf, est_k_d = −0.0 → 0 (stop);
    ratio = 0 gives a division by +0.0 → −inf, whose int cast is INT_MIN on x86 → stop (0 here)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        den = np.log(np.float64(1.0) - np.power(np.float64(ratio), np.float64(ransac_n)))
        d = np.float64(np.log(np.float64(1.0) - np.float64(confidence))) / den
    if not d < est_k:  # NaN compares false, as in C
        return est_k
    return int(math.ceil(d)) if math.isfinite(d) else 0


def ransac_feature(src, tgt, corres, max_corr, rows_fn, max_iteration=30, confidence=0.999,
                   ransac_n=3, edge_length=0.9, distance=None, exit_rule="open3d"):
    """RegistrationRANSACBasedOnCorrespondence (Open3D 0.19), sequential.  rows_fn(h) → ransac_n
    row ids.  The early exit follows upstream: after every new best the estimate est_k comes from
    the CORRESPONDENCE inlier ratio of that best (``corres_inlier_ratio``), not from its fitness
    (``exit_rule="fitness"`` keeps the round-1..3 restatement, for the divergence test only).
    Returns dict(transformation, fitness, inlier_rmse, best_index, validations, corres_ratio)."""
    src = np.asarray(src, np.float64)
    tgt = np.asarray(tgt, np.float64)
    corres = np.asarray(corres, np.int64).reshape(-1, 2)
    best = dict(transformation=np.eye(4), fitness=0.0, inlier_rmse=0.0, best_index=-1, validations=0,
                corres_ratio=0.0)
    if ransac_n < 3 or len(corres) < ransac_n or max_corr <= 0:
        return best
    tree = cKDTree(tgt)
    est_k = max_iteration
    for h in range(max_iteration):
        if h >= est_k:
            break
        rows = corres[rows_fn(h)]
        ps, pt = src[rows[:, 0]], tgt[rows[:, 1]]
        T = umeyama(ps, pt)
        if edge_length is not None and not check_edge_length(ps, pt, edge_length):
            continue
        if distance is not None and not check_distance(ps, pt, T, distance):
            continue
        fit, rmse = evaluate(src, tgt, T, max_corr, tree)
        best["validations"] += 1
        if fit > best["fitness"] or (fit == best["fitness"] and rmse < best["inlier_rmse"]):
            best.update(transformation=T, fitness=fit, inlier_rmse=rmse, best_index=h)
            if exit_rule == "fitness":
                ratio = fit
            else:
                ratio = corres_inlier_ratio(src, tgt, corres, max_corr, T)
                best["corres_ratio"] = ratio
            est_k = est_k_update(est_k, ratio, confidence, ransac_n)
    return best
