"""Feature-matching RANSAC (a6) and feature-space correspondences (a5 FPFH half).

Reference: ``src/matcher/ransac.py:20-59`` (global_registration →
``o3d.pipelines.registration.registration_ransac_based_on_feature_matching``) and ``:85``
(``correspondences_from_features``).  Device path: ``m3d.prep`` (feat.hip); semantics restated
in ``oracle/prep_oracle.py``.

Open3D draws the ``ransac_n`` rows of every hypothesis from its global RNG inside an OpenMP loop,
so the reference's own result is not reproducible run to run.  Here the rows come from the
counter sampler (``seed``, hypothesis id) and the early exit follows the sequential semantics of
``RegistrationRANSACBasedOnCorrespondence`` — deterministic for a given seed.
"""

from __future__ import annotations

import numpy as np

from .types import Feature, RegistrationResult


def _rows(f) -> np.ndarray:
    """Feature rows (N×33) from an Open3D-style Feature (``.data`` 33×N) or an array."""
    if isinstance(f, Feature) or hasattr(f, "data") and not isinstance(f, np.ndarray):
        return np.ascontiguousarray(np.asarray(f.data, np.float64).T)
    return np.asarray(f, np.float64).reshape(-1, 33)


def correspondences_from_features(src_fpfh, tgt_fpfh, mutual_filter: bool = False,
                                  mutual_consistent_ratio: float = 0.1) -> np.ndarray:
    """CorrespondencesFromFeatures → (N, 2) int32 (source, target) rows."""
    from .prep import feature_correspondences

    return feature_correspondences(_rows(src_fpfh), _rows(tgt_fpfh), mutual_filter,
                                   mutual_consistent_ratio)


def registration_ransac_based_on_feature_matching(
        src_points, tgt_points, src_fpfh, tgt_fpfh, mutual_filter: bool,
        max_correspondence_distance: float, *, ransac_n: int = 3, edge_length: float | None = 0.9,
        distance: float | None = None, max_iteration: int = 100000, confidence: float = 0.999,
        seed: int = 0) -> RegistrationResult:
    """Open3D RegistrationRANSACBasedOnFeatureMatching (PointToPoint without scaling)."""
    from .prep import ransac_on_correspondences

    if ransac_n < 3 or max_correspondence_distance <= 0.0:
        return RegistrationResult()
    corres = correspondences_from_features(src_fpfh, tgt_fpfh, mutual_filter)
    out = ransac_on_correspondences(src_points, tgt_points, corres, max_correspondence_distance,
                                    ransac_n=ransac_n, edge_length=edge_length, distance=distance,
                                    max_iteration=max_iteration, confidence=confidence, seed=seed)
    return RegistrationResult(out.transformation, out.fitness, out.inlier_rmse, out.correspondence_set)
