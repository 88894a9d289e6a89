"""Point-cloud data holder mirroring the reference's ``src/ply/ply.py`` layout.

The hot path only needs the reference ``Ply``'s LAYOUT: ``pcd`` (full-resolution
points + normals, used by ICP), ``pcd_down`` (down-sampled points, used by RANSAC), ``pcd_fpfh``
(33×N features) and ``voxel_size``.  ``Ply.from_arrays`` builds one from arrays (synthetic
clouds, tests, benchmarks).  ``Ply(path, voxel_size)`` reads a PLY file (ASCII or binary
little-endian, float/double x y z [nx ny nz]) with ``m3d.plyio``; on-device preprocessing
(voxel down-sampling, normals, FPFH — SURVEY.md §8(f) rows 2-3) is applied when available.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np

from m3d.types import PointCloud


class Ply:
    def __init__(self, path, voxel_size: float = 0.3) -> None:
        self.path = Path(path)
        self.voxel_size = voxel_size
        if not self.path.exists():
            raise FileNotFoundError(f"Ply file not found: {self.path}")     # ply.py:46-48
        if self.path.suffix.lower() != ".ply":
            raise TypeError(f"File is not a ply file: {self.path}")         # ply.py:49-51
        from m3d import plyio

        pts, nrm = plyio.read_ply(self.path)
        if len(pts) == 0:
            raise ValueError(f"Point cloud is empty: {self.path}")          # ply.py:81-84
        self.pcd = PointCloud(pts, nrm)
        self.pcd_down = PointCloud(pts.copy())
        self.pcd_fpfh = None

    @classmethod
    def from_arrays(cls, points, normals=None, points_down=None, fpfh=None, voxel_size: float = 0.3):
        obj = cls.__new__(cls)
        obj.path = None
        obj.voxel_size = voxel_size
        obj.pcd = PointCloud(points, normals)
        obj.pcd_down = PointCloud(points if points_down is None else points_down)
        obj.pcd_fpfh = None if fpfh is None else np.asarray(fpfh, np.float64)
        return obj
