"""Stub point cloud: only ``points`` / ``normals`` attributes."""
import numpy as _np


class PointCloud:
    def __init__(self):
        self.points = _np.zeros((0, 3))
        self.normals = _np.zeros((0, 3))


class KDTreeSearchParamHybrid:
    def __init__(self, radius=0.0, max_nn=0):
        self.radius = radius
        self.max_nn = max_nn
