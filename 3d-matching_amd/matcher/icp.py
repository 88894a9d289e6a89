"""Drop-in replacement of the reference's ``src/matcher/icp.py`` on MI355X.

``refine_registration(src, tgt, init_trans, voxel_size)`` (icp.py:17-48) runs Open3D-semantics
point-to-plane ICP (``registration_icp(src.pcd, tgt.pcd, 0.4·voxel, init,
TransformationEstimationPointToPlane())`` with the default ``ICPConvergenceCriteria(1e-6, 1e-6,
30)``) entirely on the device: brute-force radius-bounded 1-NN, fp64 JTJ/JTr reduction, 6×6
LDLT and the SE(3) update, with no host round trip per iteration.
"""

from __future__ import annotations

import numpy as np

from m3d import _lib
from m3d import cache as _cache
from m3d.core import icp as _icp
from m3d.types import RegistrationResult

__all__ = ["refine_registration", "registration_icp"]


def _full_cloud(x):
    """``src.pcd`` of a Ply-like (icp.py:43-44): (points, normals or None)."""
    pc = x.pcd if hasattr(x, "pcd") else x
    if hasattr(pc, "points"):
        pts = np.asarray(pc.points, np.float64).reshape(-1, 3)
        nrm = getattr(pc, "normals", None)
        nrm = None if nrm is None or len(nrm) == 0 else np.asarray(nrm, np.float64).reshape(-1, 3)
        return pts, nrm
    return np.asarray(pc, np.float64).reshape(-1, 3), None


def registration_icp(source, target, max_correspondence_distance, init=None,
                     estimation="point_to_plane", relative_fitness=1e-6, relative_rmse=1e-6,
                     max_iteration=30) -> RegistrationResult:
    """Open3D ``pipelines.registration.registration_icp`` semantics on the device."""
    if max_correspondence_distance <= 0.0:
        raise ValueError("Invalid max_correspondence_distance.")
    sp, _ = _full_cloud(source)
    tp, tn = _full_cloud(target)
    est = {"point_to_plane": _lib.EST_POINT_TO_PLANE, "point_to_point": _lib.EST_POINT_TO_POINT}[estimation]
    if est == _lib.EST_POINT_TO_PLANE and tn is None:
        raise ValueError("TransformationEstimationPointToPlane and TransformationEstimationColoredICP "
                         "require pre-computed normal vectors for target PointCloud.")
    src, tgt = _cache.clouds([(sp, None), (tp, tn if est == _lib.EST_POINT_TO_PLANE else None)])
    out = _icp(src, tgt, max_correspondence_distance, init=np.eye(4) if init is None else init,
               estimation=est, relative_fitness=relative_fitness, relative_rmse=relative_rmse,
               max_iteration=max_iteration)
    return RegistrationResult(out.transformation, out.fitness, out.inlier_rmse, out.correspondence_set)


def refine_registration(src, tgt, init_trans, voxel_size) -> RegistrationResult:
    """icp.py:17-48 — point-to-plane ICP on the full-resolution clouds, radius 0.4·voxel_size."""
    dist_thresh = voxel_size * 0.4
    return registration_icp(src, tgt, dist_thresh, init_trans, "point_to_plane")
