"""Stub of the parts of ``open3d.pipelines.registration`` the reference numpy path touches.

``correspondences_from_features`` is replaced by a deterministic hook: the generator installs
the correspondence set it wants (identity pairs for synthetic clouds) so the reference's own
noise-injection code (`ransac.py:88-99`) runs for real on top of it.
"""
import numpy as _np


class RegistrationResult:
    def __init__(self):
        self.transformation = _np.eye(4)
        self.fitness = 0.0
        self.inlier_rmse = 0.0
        self.correspondence_set = _np.zeros((0, 2), dtype=_np.int32)


class Feature:
    def __init__(self):
        self.data = _np.zeros((33, 0))


_FEATURE_CORRESPONDENCES = None


def set_feature_correspondences(corr):
    global _FEATURE_CORRESPONDENCES
    _FEATURE_CORRESPONDENCES = _np.asarray(corr, dtype=_np.int32).reshape(-1, 2)


def correspondences_from_features(f1, f2, mutual_filter=False):
    if _FEATURE_CORRESPONDENCES is None:
        raise RuntimeError("stub: call set_feature_correspondences first")
    return _FEATURE_CORRESPONDENCES.copy()
