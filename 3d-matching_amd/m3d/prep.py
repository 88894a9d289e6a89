"""Device preprocessing and feature matching (prep.hip / feat.hip through the C ABI).

Open3D 0.19 calls of the reference path and their replacements (semantics restated in
oracle/prep_oracle.py; parity against Open3D itself unpinned — SURVEY.md §8(c)):

| reference (file:line)                                   | here                              |
|---------------------------------------------------------|-----------------------------------|
| ``pcd.voxel_down_sample(v)`` (src/ply/ply.py:106)        | ``voxel_down_sample``             |
| ``estimate_normals(Hybrid(2v, 30))`` (ply.py:110,133)    | ``estimate_normals``              |
| ``compute_fpfh_feature(pcd, Hybrid(5v, 100))`` (:117)    | ``compute_fpfh`` (N×33)           |
| ``correspondences_from_features`` (ransac.py:85)         | ``feature_correspondences``       |
| ``RegistrationRANSACBasedOnCorrespondence`` (a6)         | ``ransac_on_correspondences``     |

All entry points take host or device arrays and return numpy arrays (the reference works in
numpy / Open3D host containers); the arithmetic runs on the GPU.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .core import Cloud, _torch, context, corr_pairs, device_empty, ptr, stream_handle, to_device


def voxel_down_sample(points, voxel_size: float, normals=None):
    """→ (points M×3, normals M×3 or None), voxels in ascending (ix, iy, iz) order."""
    torch = _torch()
    ctx = context()
    p = to_device(points)
    nrm = None if normals is None else to_device(normals)
    n = p.shape[0]
    out = device_empty((max(n, 1), 3), torch.float64)
    out_n = device_empty((max(n, 1), 3), torch.float64) if nrm is not None else None
    m = C.c_int64()
    ctx.check(ctx.lib.m3d_voxel_down_sample(ctx.h, ptr(p), ptr(nrm), n, float(voxel_size), ptr(out),
                                            ptr(out_n), C.byref(m), stream_handle()), "voxel_down_sample")
    k = m.value
    return out[:k].cpu().numpy(), (None if out_n is None else out_n[:k].cpu().numpy())


def _cloud(points, normals=None):
    return points if isinstance(points, Cloud) else Cloud(points, normals)


def hybrid_search(points, radius: float, max_nn: int):
    """KDTreeFlann::SearchHybrid for every point → (idx N×k int32 (−1 pad), d2 N×k, count N)."""
    torch = _torch()
    c = _cloud(points)
    ctx = c.ctx
    n = max(c.n, 1)
    idx = device_empty((n, max_nn), torch.int32)
    d2 = device_empty((n, max_nn), torch.float64)
    cnt = device_empty((n,), torch.int32)
    ctx.check(ctx.lib.m3d_hybrid_search(ctx.h, c.h, float(radius), int(max_nn), ptr(idx), ptr(d2),
                                        ptr(cnt), stream_handle()), "hybrid_search")
    return idx[: c.n].cpu().numpy(), d2[: c.n].cpu().numpy(), cnt[: c.n].cpu().numpy()


def estimate_normals(points, radius: float, max_nn: int = 30, normals=None):
    """PointCloud::EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)); existing
    ``normals`` orient the result like Open3D."""
    torch = _torch()
    c = _cloud(points, normals)
    ctx = c.ctx
    out = device_empty((max(c.n, 1), 3), torch.float64)
    ctx.check(ctx.lib.m3d_estimate_normals(ctx.h, c.h, float(radius), int(max_nn), ptr(out),
                                           stream_handle()), "estimate_normals")
    return out[: c.n].cpu().numpy()


def compute_fpfh(points, normals, radius: float, max_nn: int = 100):
    """ComputeFPFHFeature → N×33 (Open3D's Feature.data is the 33×N transpose)."""
    torch = _torch()
    c = _cloud(points)
    ctx = c.ctx
    nrm = to_device(normals)
    if nrm.shape != (c.n, 3):
        raise ValueError("normals must be N×3")
    out = device_empty((max(c.n, 1), 33), torch.float64)
    ctx.check(ctx.lib.m3d_compute_fpfh(ctx.h, c.h, ptr(nrm), float(radius), int(max_nn), ptr(out),
                                       stream_handle()), "compute_fpfh")
    return out[: c.n].cpu().numpy()


def _feature_rows(f):
    """N×33 feature rows from an Open3D-style Feature (``.data`` is 33×N) or an array."""
    if not isinstance(f, np.ndarray) and hasattr(f, "data"):
        return np.ascontiguousarray(np.asarray(f.data, np.float64).T)
    return f


def feature_correspondences(f_src, f_tgt, mutual_filter: bool = False,
                            mutual_consistent_ratio: float = 0.1) -> np.ndarray:
    """CorrespondencesFromFeatures (ransac.py:85) on N×33 feature rows, or on Open3D-style
    Features (33×N ``.data``) → (M, 2) int32 (source, target)."""
    torch = _torch()
    ctx = context()
    f_src, f_tgt = _feature_rows(f_src), _feature_rows(f_tgt)
    fs = to_device(f_src, shape_tail=None)
    ft = to_device(f_tgt, shape_tail=None)
    if fs.ndim != 2 or ft.ndim != 2 or fs.shape[1] != ft.shape[1]:
        raise ValueError("features must be N×33 arrays")
    ns, nt = fs.shape[0], ft.shape[0]
    out = device_empty((max(ns, 1), 2), torch.int32)
    m = C.c_int64()
    ctx.check(ctx.lib.m3d_feature_correspondences(ctx.h, ptr(fs), ns, ptr(ft), nt, fs.shape[1],
                                                  int(bool(mutual_filter)), float(mutual_consistent_ratio),
                                                  ptr(out), C.byref(m), stream_handle()),
              "feature_correspondences")
    return out[: m.value].cpu().numpy()


@dataclass
class FeatureRansacOutcome:
    transformation: np.ndarray
    fitness: float
    inlier_rmse: float
    best_index: int
    validations: int
    correspondence_set: np.ndarray
    corres_ratio: float = 0.0  # the best's correspondence inlier ratio (Open3D's exit input)


def ransac_on_correspondences(src, tgt, corres, max_correspondence_distance: float, *,
                              ransac_n: int = 3, edge_length: float | None = 0.9,
                              distance: float | None = None, max_iteration: int = 100000,
                              confidence: float = 0.999, seed: int = 0) -> FeatureRansacOutcome:
    """RegistrationRANSACBasedOnCorrespondence (PointToPoint, no scaling) with the EdgeLength /
    Distance checkers (None disables a checker)."""
    torch = _torch()
    sc, tc = _cloud(src), _cloud(tgt)
    ctx = sc.ctx
    corr = to_device(np.asarray(corres).reshape(-1, 2), dtype="int32", shape_tail=(2,))
    p = _lib.FeatureRansacParams(float(max_correspondence_distance), float(confidence),
                                 float(edge_length) if edge_length is not None else 0.0,
                                 float(distance) if distance is not None else 0.0,
                                 int(seed) & ((1 << 64) - 1), int(max_iteration), int(ransac_n))
    r = _lib.FeatureRansacResult()
    cs = device_empty((max(sc.n, 1),), torch.int32)
    ctx.check(ctx.lib.m3d_ransac_on_correspondences(ctx.h, sc.h, tc.h, ptr(corr), corr.shape[0], C.byref(p),
                                                    C.byref(r), ptr(cs), stream_handle()),
              "ransac_on_correspondences")
    return FeatureRansacOutcome(np.array(r.T[:]).reshape(4, 4), r.fitness, r.inlier_rmse,
                                int(r.best_index), int(r.validations), corr_pairs(ctx, cs, sc.n),
                                float(r.corres_ratio))
