"""CPU oracle for the RANSAC half of the hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / CPU baseline.  The product path (``m3d``, ``matcher``)
never imports it and fails loudly when the HIP library is missing.

Restates, in numpy fp64, the reference functions of
``/root/reference/src/matcher/ransac.py`` (KTC-Security-Circle/3d-matching):

* ``compute_step_transformation``  — ransac.py:104-192 (3-point Kabsch, identity fallback)
* ``evaluate_inlier_ratio``        — ransac.py:195-236 (gather, transform, ``norm < thr``)
* ``evaluate_inlier_ratio_fast``   — ransac.py:239-277 (pre-gathered, ``Σd² < thr²``)
* noise injection of ``compute_feature_correspondences`` — ransac.py:88-99
* the step-RANSAC driver loop      — _visualize_matcher.py:343-470 (best tracking, early stop)
* the benchmark loop               — benchmark_ransac.py:87-125

plus the build's own counter-based hypothesis sampler (``native_triples``), which the HIP kernel
reproduces bit for bit.

Parity pinning: ``tests/test_oracle_golden.py`` checks this module against golden vectors that
``tools/gen_golden.py`` produced by importing the reference's own ``ransac.py`` in the build
container (open3d replaced by a type stub).
"""

from __future__ import annotations

import numpy as np

HYP_OK, HYP_DEGENERATE, HYP_NONFINITE = 0, 1, 2


# --------------------------------------------------------------------------------------------
# a1: 3-point Kabsch (ransac.py:104-192)
# --------------------------------------------------------------------------------------------
def kabsch3(src3: np.ndarray, tgt3: np.ndarray):
    """Kabsch on 3 sampled pairs exactly as ransac.py:150-188 does. Returns (T 4×4, status)."""
    try:
        centroid_src = np.mean(src3, axis=0)                      # :153
        centroid_tgt = np.mean(tgt3, axis=0)                      # :154
        p = src3 - centroid_src                                   # :157
        q = tgt3 - centroid_tgt                                   # :158
        H = np.dot(p.T, q)                                        # :161
        U, S, Vt = np.linalg.svd(H, full_matrices=False)          # :165
        R = np.dot(Vt.T, U.T)                                     # :168
        if np.linalg.det(R) < 0:                                  # :171-173
            Vt[2, :] *= -1
            R = np.dot(Vt.T, U.T)
        t = centroid_tgt - np.dot(R, centroid_src)                # :176
        trans = np.eye(4)
        trans[:3, :3] = R
        trans[:3, 3] = t
        if np.isnan(trans).any() or np.isinf(trans).any():        # :184-185
            return np.eye(4), HYP_NONFINITE
        return trans, HYP_OK
    except Exception:                                             # :190-192
        return np.eye(4), HYP_NONFINITE


def compute_step_transformation(src_pts, tgt_pts, corr, rng=None):
    """ransac.py:104-192.  ``rng`` defaults to the global legacy numpy RNG, like the reference."""
    rng = np.random if rng is None else rng
    corr = np.asarray(corr).reshape(-1, 2)
    if len(corr) < 3:                                             # :139-140
        return np.eye(4), HYP_DEGENERATE, None
    idxs = rng.choice(len(corr), 3, replace=False)                # :143
    sample = corr[idxs]
    T, st = kabsch3(np.asarray(src_pts)[sample[:, 0]], np.asarray(tgt_pts)[sample[:, 1]])
    return T, st, idxs


def replay_triples(seed_or_state, nc: int, H: int):
    """The exact index triples H successive reference calls draw (legacy MT19937 stream)."""
    rs = np.random.RandomState()
    if isinstance(seed_or_state, tuple):
        rs.set_state(seed_or_state)
    else:
        rs.seed(seed_or_state)
    out = np.empty((H, 3), dtype=np.int32)
    for h in range(H):
        out[h] = rs.choice(nc, 3, replace=False)
    return out, rs.get_state()


# --------------------------------------------------------------------------------------------
# the build's counter-based sampler (mirrored bit-exactly by csrc/ransac.hip::native_triple)
# --------------------------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_M64)
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(_M64)
        return z ^ (z >> np.uint64(31))


def native_triples(seed: int, hyp0: int, H: int, nc: int) -> np.ndarray:
    """Three distinct correspondence rows per hypothesis id h = hyp0..hyp0+H-1.

    base(h)    = splitmix64(seed ^ (h · 0x9E3779B97F4A7C15))
    draw(h, k) = splitmix64(base(h) + k)                     (uint64 wrap-around)
    index      = ((draw >> 32) · nc) >> 32                    (multiply-shift into [0, nc))
    Draws k = 0, 1, 2, ... are consumed until three distinct indices are found, in order.
    """
    if nc < 3:
        raise ValueError("need at least 3 correspondences")
    h = np.arange(hyp0, hyp0 + H, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = _splitmix64(np.uint64(seed) ^ (h * np.uint64(0x9E3779B97F4A7C15)))
    K = 8
    with np.errstate(over="ignore"):
        d = _splitmix64(base[:, None] + np.arange(K, dtype=np.uint64)[None, :])
    idx = ((d >> np.uint64(32)) * np.uint64(nc)) >> np.uint64(32)
    out = np.empty((H, 3), dtype=np.int32)
    for i in range(H):
        got = []
        for v in idx[i]:
            v = int(v)
            if v not in got:
                got.append(v)
                if len(got) == 3:
                    break
        k = K
        while len(got) < 3:  # only reachable for tiny nc
            with np.errstate(over="ignore"):
                v = int(((_splitmix64(np.array([base[i] + np.uint64(k)]))[0] >> np.uint64(32))
                         * np.uint64(nc)) >> np.uint64(32))
            k += 1
            if v not in got:
                got.append(v)
        out[i] = got
    return out


# --------------------------------------------------------------------------------------------
# a2 / a3: inlier scoring
# --------------------------------------------------------------------------------------------
def evaluate_inlier_ratio(src_pts, tgt_pts, corr, transform, voxel_size) -> float:
    """ransac.py:195-236 verbatim semantics (``norm < 1.5·voxel``)."""
    dist_thresh = voxel_size * 1.5                                # :218
    corres = np.asarray(corr).reshape(-1, 2)
    if len(corres) == 0:                                          # :220-221
        return 0.0
    p_src = np.asarray(src_pts)[corres[:, 0]]                     # :226
    p_tgt = np.asarray(tgt_pts)[corres[:, 1]]                     # :227
    p_t = (transform[:3, :3] @ p_src.T).T + transform[:3, 3]      # :230
    dists = np.linalg.norm(p_t - p_tgt, axis=1)                   # :233
    return np.sum(dists < dist_thresh) / len(corres)              # :236


def evaluate_inlier_ratio_fast(p_src, p_tgt, transform, dist_thresh_sq) -> float:
    """ransac.py:239-277 (``Σ(Δ²) < thr²`` on pre-gathered pairs)."""
    if len(p_src) == 0:                                           # :265-266
        return 0.0
    R = transform[:3, :3]
    t = transform[:3, 3]
    p_t = p_src @ R.T + t                                         # :271
    dists_sq = np.sum((p_t - p_tgt) ** 2, axis=1)                 # :274
    return np.sum(dists_sq < dist_thresh_sq) / len(p_src)         # :277


def inlier_count(p_src, p_tgt, transform, thr, mode: int) -> int:
    """Count form used by the batched checker: mode 0 = a3 (thr is thr²), mode 1 = a2 (thr)."""
    if len(p_src) == 0:
        return 0
    R = transform[:3, :3]
    t = transform[:3, 3]
    if mode == 0:
        d2 = np.sum((p_src @ R.T + t - p_tgt) ** 2, axis=1)
        return int(np.sum(d2 < thr))
    d = np.linalg.norm((R @ p_src.T).T + t - p_tgt, axis=1)
    return int(np.sum(d < thr))


def inlier_counts(p_src, p_tgt, transforms, thr, mode: int) -> np.ndarray:
    return np.array([inlier_count(p_src, p_tgt, T, thr, mode) for T in transforms], dtype=np.int64)


# --------------------------------------------------------------------------------------------
# a5: outlier injection (ransac.py:88-99) on the global legacy RNG, as the reference does it
# --------------------------------------------------------------------------------------------
def inject_noise_legacy(corr, n_src, n_tgt, noise_ratio, rng=None):
    rng = np.random if rng is None else rng
    corres_np = np.asarray(corr)
    if noise_ratio > 0:
        n_noise = int(len(corres_np) * noise_ratio)
        if n_noise > 0:
            src_indices = rng.randint(0, n_src, n_noise)
            tgt_indices = rng.randint(0, n_tgt, n_noise)
            noise_corres = np.stack((src_indices, tgt_indices), axis=1)
            corres_np = np.vstack((corres_np, noise_corres))
            rng.shuffle(corres_np)
    return corres_np


# --------------------------------------------------------------------------------------------
# a4: driver loops
# --------------------------------------------------------------------------------------------
def required_iterations(inlier_ratio, confidence, max_iter, sample_size=3) -> int:
    """_visualize_matcher.py:356-370 ``compute_required_iterations``."""
    if inlier_ratio < 0.01:
        return max_iter
    with np.errstate(divide="ignore"):
        return int(np.log(1 - confidence) / np.log(1 - inlier_ratio ** sample_size))


def select_best(counts, nc, max_iter, early_stop=True, es_threshold=0.5, es_confidence=0.99):
    """The loop semantics of _visualize_matcher.py:394-450 applied to a precomputed count stream.

    Returns ``(best_index, best_fitness, iterations)``; iterations = iter_num at exit.
    """
    best_idx, best_fit = -1, -1.0
    for h, c in enumerate(counts[:max_iter]):
        w = c / nc if nc else 0.0
        if best_idx < 0 or w > best_fit:                          # :426-429 strict '>'
            best_idx, best_fit = h, w
        iter_num = h + 1
        if early_stop and best_fit > es_threshold:                # :432
            if iter_num >= required_iterations(best_fit, es_confidence, max_iter):
                return best_idx, best_fit, iter_num
    return best_idx, best_fit, min(len(counts), max_iter)


def ransac_loop(p_src, p_tgt, triples, thr_sq, max_iter, early_stop=True, es_threshold=0.5,
                es_confidence=0.99):
    """Full a4 loop on pre-gathered pairs with given triples (a1 + a3 per iteration)."""
    counts, Ts = [], []
    nc = len(p_src)
    best_idx, best_fit = -1, -1.0
    for h in range(max_iter):
        i = triples[h]
        T, _ = kabsch3(p_src[i], p_tgt[i])
        c = inlier_count(p_src, p_tgt, T, thr_sq, 0)
        counts.append(c)
        Ts.append(T)
        w = c / nc
        if best_idx < 0 or w > best_fit:
            best_idx, best_fit = h, w
        if early_stop and best_fit > es_threshold:
            if h + 1 >= required_iterations(best_fit, es_confidence, max_iter):
                return best_idx, best_fit, h + 1, np.array(counts), np.array(Ts)
    return best_idx, best_fit, max_iter, np.array(counts), np.array(Ts)
