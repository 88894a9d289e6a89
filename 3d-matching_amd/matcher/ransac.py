"""Drop-in replacement of the reference's ``src/matcher/ransac.py`` on MI355X.

Same function names, arguments, defaults, return types and soft-failure behaviour as
KTC-Security-Circle/3d-matching ``src/matcher/ransac.py``; the arithmetic runs in libm3d.so
(HIP, gfx950) through the C ABI of ``include/m3d.h``.

* ``compute_step_transformation`` (ransac.py:104-192): draws its 3 rows from the GLOBAL legacy
  numpy RNG exactly like the reference (``np.random.choice(n, 3, replace=False)``: the same rows
  and the same RNG state afterwards, replayed natively by ``m3d.core.choice3``), so a seeded
  program sees the same hypotheses; the Kabsch estimate runs on the device (one launch, one sync:
  ``m3d_kabsch3_one``).
* ``evaluate_inlier_ratio`` (ransac.py:195-236) and ``evaluate_inlier_ratio_fast``
  (ransac.py:239-277): exact counts (fp32 screen + fp64 guard-band recheck on the device).
* ``compute_feature_correspondences`` (ransac.py:62-101): FPFH feature-space NN on the device
  plus the reference's outlier injection on the global numpy RNG.
* ``global_registration`` (ransac.py:20-59): ``m3d.prep`` feature correspondences + a6.

Additions (batched, device-resident): ``run_ransac`` runs the whole step-RANSAC loop of
``_visualize_matcher.py:343-470`` on the GPU; ``register`` is the coarse-to-fine façade
``main.py:34-38`` intends.
"""

from __future__ import annotations

import numpy as np

from m3d import _lib
from m3d import cache as _cache
from m3d.core import CorrSet, RansacParams, choice3, replay_triples
from m3d.types import RegistrationResult

__all__ = [
    "global_registration",
    "compute_feature_correspondences",
    "compute_step_transformation",
    "evaluate_inlier_ratio",
    "evaluate_inlier_ratio_fast",
    "run_ransac",
]


def _down_points(x) -> np.ndarray:
    """``src.pcd_down.points`` of a Ply-like (ransac.py:147-148), or the array itself."""
    if hasattr(x, "pcd_down"):
        x = x.pcd_down.points
    elif hasattr(x, "points"):
        x = x.points
    return np.asarray(x, dtype=np.float64).reshape(-1, 3)


def _corr_array(correspondences) -> np.ndarray:
    c = np.asarray(correspondences)
    if c.size == 0:
        return np.zeros((0, 2), np.int32)
    c = c.reshape(-1, 2)
    if c.dtype != np.int32:  # the device takes int32 rows: wider values must not wrap silently
        big = (c > np.iinfo(np.int32).max) | (c < np.iinfo(np.int32).min)
        if big.any():
            raise IndexError(f"index {int(c[big][0])} is out of bounds for axis 0")
    return c


def _check_gather(corr: np.ndarray, n_src: int, n_tgt: int) -> None:
    """numpy fancy-indexing semantics of the reference's gathers (ransac.py:147-148, 226-227):
    indices in [-n, n) are valid (negatives wrap — the device does the same), anything else
    raises numpy's IndexError."""
    for col, n in ((0, n_src), (1, n_tgt)):
        v = corr[:, col]
        bad = (v >= n) | (v < -n)
        if bad.any():
            raise IndexError(f"index {int(v[np.argmax(bad)])} is out of bounds for axis 0 with size {n}")


def _in_range(corr: np.ndarray, n_src: int, n_tgt: int) -> np.ndarray:
    return (corr[:, 0] < n_src) & (corr[:, 0] >= -n_src) & (corr[:, 1] < n_tgt) & (corr[:, 1] >= -n_tgt)


def _packed(s_pts: np.ndarray, t_pts: np.ndarray, corr: np.ndarray, need_all: bool):
    """The cached device correspondence set for (s_pts, t_pts, corr).

    need_all (evaluate_inlier_ratio / run_ransac read every row, ransac.py:226-227): an
    out-of-range index raises numpy's IndexError.  Otherwise (compute_step_transformation reads
    only its 3 sampled rows, checked by the caller) rows the reference never reads may hold
    anything: out-of-range entries are packed as 0.  Whether every index is in range is decided
    once per cached content (m3d.cache.memo)."""
    key = _cache.corr_key(s_pts, t_pts, corr)
    ok = _cache.memo(("in_range",) + key, lambda: bool(_in_range(corr, len(s_pts), len(t_pts)).all()))
    if ok:
        return _cache.get(key, lambda: CorrSet(s_pts, t_pts, corr))
    if need_all:
        _check_gather(corr, len(s_pts), len(t_pts))
    def make():
        c = corr.copy()
        c[~_in_range(corr, len(s_pts), len(t_pts))] = 0
        return CorrSet(s_pts, t_pts, c)
    return _cache.get(("clean",) + key, make)


def global_registration(src, tgt, voxel_size: float, iteration: int = 30) -> RegistrationResult:
    """ransac.py:20-59: feature-matching RANSAC (mutual filter, Point-to-Point, ransac_n=3,
    EdgeLength(0.9) + Distance(1.5·v) checkers, RANSACConvergenceCriteria(iteration, 0.999))."""
    # Open3D RegistrationRANSACBasedOnFeatureMatching = CorrespondencesFromFeatures (mutual) +
    # RegistrationRANSACBasedOnCorrespondence.  Open3D draws each hypothesis' rows from its global
    # RNG inside an OpenMP loop (not reproducible run to run); here the rows come from the counter
    # sampler (seed, hypothesis id) and the early exit follows the sequential semantics.
    from m3d import prep

    dist_thresh = voxel_size * 1.5
    if dist_thresh <= 0.0:  # Open3D: an empty RegistrationResult for a non-positive distance
        return RegistrationResult()
    corres = prep.feature_correspondences(src.pcd_fpfh, tgt.pcd_fpfh, True)
    out = prep.ransac_on_correspondences(_down_points(src), _down_points(tgt), corres, dist_thresh,
                                         ransac_n=3, edge_length=0.9, distance=dist_thresh,
                                         max_iteration=iteration, confidence=0.999)
    return RegistrationResult(out.transformation, out.fitness, out.inlier_rmse, out.correspondence_set)


def inject_noise(corres_np: np.ndarray, n_src: int, n_tgt: int, noise_ratio: float) -> np.ndarray:
    """ransac.py:89-99's outlier injection on the global legacy numpy RNG: int(N·ratio) random
    (source, target) rows appended, then the whole set shuffled in place."""
    if noise_ratio > 0:
        n_original = len(corres_np)
        n_noise = int(n_original * noise_ratio)
        if n_noise > 0:
            src_indices = np.random.randint(0, n_src, n_noise)
            tgt_indices = np.random.randint(0, n_tgt, n_noise)
            noise_corres = np.stack((src_indices, tgt_indices), axis=1)
            corres_np = np.vstack((corres_np, noise_corres))
            np.random.shuffle(corres_np)
    return np.asarray(corres_np, dtype=np.int32)


def compute_feature_correspondences(src, tgt, mutual_filter: bool = False,
                                    noise_ratio: float = 0.0) -> np.ndarray:
    """ransac.py:62-101.  Returns an (N,2) int32 array (the Vector2iVector's numpy view)."""
    from m3d import prep

    corres_np = prep.feature_correspondences(src.pcd_fpfh, tgt.pcd_fpfh, mutual_filter)
    return inject_noise(corres_np, len(_down_points(src)), len(_down_points(tgt)), noise_ratio)


def compute_step_transformation(src, tgt, correspondences) -> RegistrationResult:
    """ransac.py:104-192 — 3-point Kabsch with identity fallback (fitness stays 0.0)."""
    c = np.asarray(correspondences)
    corres_np = np.zeros((0, 2), np.int32) if c.size == 0 else c.reshape(-1, 2)
    res = RegistrationResult(np.eye(4), 0.0)
    n_corres = len(corres_np)
    if n_corres < 3:
        return res
    idxs = choice3(n_corres)  # np.random.choice(n, 3, replace=False): same rows, same RNG state
    s_pts, t_pts = _down_points(src), _down_points(tgt)
    _check_gather(corres_np[idxs], len(s_pts), len(t_pts))     # only the sampled rows are read
    if corres_np.dtype != np.int32:
        # rows the reference never reads may hold anything, wider than int32 included: packed
        # as 0 (the sampled rows were checked above)
        ok = _in_range(corres_np, len(s_pts), len(t_pts))
        corres_np = np.where(ok[:, None], corres_np, 0).astype(np.int32)
    cs = _packed(s_pts, t_pts, corres_np, need_all=False)
    T, status = cs.kabsch3_one(idxs)
    if status == _lib.HYP_OK:
        res.transformation = T
    return res


def evaluate_inlier_ratio(src, tgt, correspondences, transform, voxel_size) -> float:
    """ransac.py:195-236 — fraction of pairs with ‖T p − q‖ < 1.5·voxel_size."""
    dist_thresh = voxel_size * 1.5
    corres = _corr_array(correspondences)
    if len(corres) == 0:
        return 0.0
    s_pts, t_pts = _down_points(src), _down_points(tgt)
    cs = _packed(s_pts, t_pts, np.asarray(corres, np.int32), need_all=True)
    cnt = cs.score_one(transform, dist_thresh, _lib.SCORE_NORM)
    return np.int64(cnt) / len(corres)


def evaluate_inlier_ratio_fast(p_src, p_tgt, transform, dist_thresh_sq) -> float:
    """ransac.py:239-277 — fraction of pre-gathered pairs with Σ(T p − q)² < dist_thresh_sq."""
    p_src = np.asarray(p_src, np.float64).reshape(-1, 3)
    if len(p_src) == 0:
        return 0.0
    cs = _cache.corrset_gathered(p_src, np.asarray(p_tgt, np.float64).reshape(-1, 3))
    cnt = cs.score_one(transform, dist_thresh_sq, _lib.SCORE_SQUARED)
    return np.int64(cnt) / len(p_src)


_REPLAY_CHUNK = 4096  # rows per MT checkpoint of the replay sampler


def run_ransac(src, tgt, correspondences, voxel_size: float = 0.3, max_iter: int = 10000,
           early_stop: bool = True, early_stop_threshold: float = 0.5,
           early_stop_confidence: float = 0.99, sampler: str = "replay", seed=None,
           score: str = "fast"):
    """The step-RANSAC loop of _visualize_matcher.py:343-470 on the device.

    sampler="replay": the rows come from the global legacy numpy RNG exactly as successive
    ``compute_step_transformation`` calls would draw them (and the RNG is advanced by the number
    of iterations actually run), so the result is the reference loop's result.
    sampler="native": counter-based sampler keyed by ``seed`` (fast; no host RNG work).
    score="fast" compares Σd² < (1.5·v)² (evaluate_inlier_ratio_fast, the GUI loop);
    score="norm" compares ‖d‖ < 1.5·v (evaluate_inlier_ratio, benchmark_ransac.py).
    Returns (RegistrationResult, info dict with best_index / iterations / best_count).
    """
    corres = _corr_array(correspondences)
    nc = len(corres)
    dist_thresh = voxel_size * 1.5
    if score == "fast":
        thr, mode = dist_thresh * dist_thresh, _lib.SCORE_SQUARED
    elif score == "norm":
        thr, mode = dist_thresh, _lib.SCORE_NORM
    else:
        raise ValueError("score must be 'fast' or 'norm'")
    s_pts, t_pts = _down_points(src), _down_points(tgt)
    cs = _packed(s_pts, t_pts, np.asarray(corres, np.int32), need_all=True)
    params = RansacParams(max_iter=max_iter, thr=thr, mode=mode, early_stop=early_stop,
                          es_threshold=early_stop_threshold, es_confidence=early_stop_confidence)
    triples = None
    checkpoints = None
    if sampler == "replay" and nc >= 3:
        # the rows in chunks, keeping the MT state at each chunk start: after the run the RNG is
        # advanced from the checkpoint nearest the stop (< _REPLAY_CHUNK re-drawn rows), not
        # replayed from the start
        checkpoints = [np.random.get_state()]
        parts = []
        for h0 in range(0, max_iter, _REPLAY_CHUNK):
            t, st = replay_triples(nc, min(_REPLAY_CHUNK, max_iter - h0), state=checkpoints[-1])
            parts.append(t)
            checkpoints.append(st)
        triples = np.concatenate(parts) if parts else np.empty((0, 3), np.int32)
    elif sampler == "native":
        params.seed = 0 if seed is None else int(seed)
    elif sampler != "replay":
        raise ValueError("sampler must be 'replay' or 'native'")
    out = cs.run(params, triples=triples)
    if checkpoints is not None:
        # advance the global RNG by exactly the iterations the loop consumed
        k, rem = divmod(int(out.iterations), _REPLAY_CHUNK)
        st = checkpoints[k] if rem == 0 else replay_triples(nc, rem, state=checkpoints[k])[1]
        np.random.set_state(st)
    res = RegistrationResult(out.transformation, out.fitness)
    return res, dict(best_index=out.best_index, iterations=out.iterations, best_count=out.best_count,
                     n_correspondences=nc)
