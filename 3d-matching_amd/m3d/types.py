"""Host-side result/data types mirroring the reference's Open3D-facing types.

* ``RegistrationResult`` — Open3D ``pipelines.registration.RegistrationResult`` as the reference
  uses it (`ransac.py:134-136`, `icp.py:42`): ``transformation`` (4×4 f64), ``fitness``,
  ``inlier_rmse``, ``correspondence_set`` (M×2 int32).
* ``PointCloud`` — the two attributes the path reads from ``o3d.geometry.PointCloud``:
  ``points`` (N×3 f64) and ``normals`` (N×3 f64 or empty).
"""

from __future__ import annotations

import numpy as np


class RegistrationResult:
    def __init__(self, transformation=None, fitness=0.0, inlier_rmse=0.0, correspondence_set=None):
        self.transformation = np.eye(4) if transformation is None else np.asarray(transformation, np.float64)
        self.fitness = float(fitness)
        self.inlier_rmse = float(inlier_rmse)
        self.correspondence_set = (np.zeros((0, 2), np.int32) if correspondence_set is None
                                   else np.asarray(correspondence_set, np.int32).reshape(-1, 2))

    def __repr__(self):
        return (f"RegistrationResult with fitness={self.fitness:e}, inlier_rmse={self.inlier_rmse:e}, "
                f"and correspondence_set size of {len(self.correspondence_set)}")


class Feature:
    """Open3D ``pipelines.registration.Feature``: ``data`` is dimension × N (33×N for FPFH)."""

    def __init__(self, data=None):
        self.data = np.zeros((33, 0)) if data is None else np.asarray(data, np.float64)

    def dimension(self) -> int:
        return self.data.shape[0]

    def num(self) -> int:
        return self.data.shape[1]


class PointCloud:
    def __init__(self, points=None, normals=None):
        self.points = np.zeros((0, 3)) if points is None else np.asarray(points, np.float64).reshape(-1, 3)
        self.normals = np.zeros((0, 3)) if normals is None else np.asarray(normals, np.float64).reshape(-1, 3)

    def has_points(self) -> bool:
        return len(self.points) > 0

    def has_normals(self) -> bool:
        return len(self.normals) == len(self.points) and len(self.points) > 0

    def transform(self, T):
        T = np.asarray(T, np.float64)
        self.points = self.points @ T[:3, :3].T + T[:3, 3]
        if len(self.normals):
            self.normals = self.normals @ T[:3, :3].T
        return self
