"""Stub: Open3D eigen-vector wrappers are plain ndarrays here."""
import numpy as _np


def Vector3dVector(a):  # noqa: N802 - mirrors the open3d name
    return _np.asarray(a, dtype=_np.float64).reshape(-1, 3)


def Vector2iVector(a):  # noqa: N802
    return _np.asarray(a, dtype=_np.int32).reshape(-1, 2)
