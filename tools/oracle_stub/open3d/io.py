"""Stub: no PLY reader offline."""


def read_point_cloud(path):  # pragma: no cover - never called by the generator
    raise RuntimeError("open3d stub has no IO")
