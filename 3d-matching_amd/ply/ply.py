"""Point-cloud data holder mirroring the reference's ``src/ply/ply.py``.

``Ply(path, voxel_size)`` follows ply.py:32-135 step by step, with every Open3D call replaced
by the device path of ``m3d.prep``:

1. read the PLY (``m3d.plyio``; Open3D ``read_point_cloud``)                       ply.py:80
2. ``pcd_down`` = voxel down-sample (voxel_size); file normals, when present, are averaged
   per voxel like Open3D's VoxelDownSample                                           ply.py:106
3. ``pcd_down`` normals: hybrid search (2·v, 30), oriented by those averaged normals ply.py:110-112
4. ``pcd_fpfh`` = FPFH on ``pcd_down`` (hybrid 5·v, 100) — an Open3D-style ``Feature``
   (``.data`` 33×N)                                                                  ply.py:117-120
5. Gaussian noise N(0, 0.05²) on ``pcd_down`` points from the GLOBAL numpy RNG, after the
   features (the reference's robustness test)                                        ply.py:61-62
6. ``pcd`` normals: hybrid search (2·v, 30), oriented by normals read from the file  ply.py:65,133

``Ply.from_arrays`` builds one from arrays (synthetic clouds, tests, benchmarks) without any
preprocessing unless ``preprocess=True``.
"""

from __future__ import annotations

import time
from pathlib import Path

import numpy as np

from m3d.types import Feature, PointCloud


class Ply:
    def __init__(self, path, voxel_size: float = 0.3) -> None:
        self.path = Path(path)
        self.voxel_size = voxel_size
        if not self.path.exists():
            raise FileNotFoundError(f"Ply file not found: {self.path}")     # ply.py:46-48
        if self.path.suffix.lower() != ".ply":
            raise TypeError(f"File is not a ply file: {self.path}")         # ply.py:49-51
        from m3d import plyio

        t0 = time.perf_counter()
        pts, nrm = plyio.read_ply(self.path)
        self.stage_ms = {"read": (time.perf_counter() - t0) * 1e3}
        if len(pts) == 0:
            raise ValueError(f"Point cloud is empty: {self.path}")          # ply.py:81-84
        self.pcd = PointCloud(pts, nrm)
        self._preprocess(voxel_size)

    def _preprocess(self, voxel_size: float) -> None:
        """ply.py:53-66.  Wall time of each stage lands in ``stage_ms`` (every stage returns host
        arrays, so the device work is complete when its timer stops)."""
        from m3d import prep
        from m3d.core import Cloud, to_device

        v = voxel_size
        ms = getattr(self, "stage_ms", None)
        if ms is None:
            ms = self.stage_ms = {}
        t = time.perf_counter()

        def lap(name):
            nonlocal t
            now = time.perf_counter()
            ms[name] = (now - t) * 1e3
            t = now

        # the full cloud goes to the device once (down-sampling, then its normals), the
        # down-sampled one once (its normals, then FPFH: the noise is added after, ply.py:61-62)
        p_dev = to_device(self.pcd.points)
        prev = self.pcd.normals if self.pcd.has_normals() else None
        # VoxelDownSample carries the file's normals (their plain per-voxel mean) into pcd_down,
        # and EstimateNormals then orients each new normal by that mean (ply.py:106-112)
        down, down_prev = prep.voxel_down_sample(p_dev, v, normals=prev)
        lap("voxel_down_sample")
        c_down = Cloud(down, down_prev)
        down_n = prep.estimate_normals(c_down, 2 * v, 30)
        lap("normals_down")
        self.pcd_down = PointCloud(down, down_n)
        self.pcd_fpfh = Feature(prep.compute_fpfh(c_down, down_n, 5 * v, 100).T)
        lap("fpfh")
        noise = 0.05 * np.random.randn(*self.pcd_down.points.shape)      # ply.py:61-62
        self.pcd_down.points = self.pcd_down.points + noise
        lap("noise")
        # existing normals orient the estimate like Open3D (the cloud carries them)
        self.pcd.normals = prep.estimate_normals(Cloud(p_dev, prev), 2 * v, 30)
        lap("normals_full")

    @classmethod
    def from_arrays(cls, points, normals=None, points_down=None, fpfh=None, voxel_size: float = 0.3,
                    preprocess: bool = False):
        obj = cls.__new__(cls)
        obj.path = None
        obj.voxel_size = voxel_size
        obj.pcd = PointCloud(points, normals)
        if preprocess:
            obj._preprocess(voxel_size)
            return obj
        obj.pcd_down = PointCloud(points if points_down is None else points_down)
        obj.pcd_fpfh = None if fpfh is None else Feature(np.asarray(fpfh, np.float64))
        return obj
