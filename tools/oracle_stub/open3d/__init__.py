"""Minimal type stub for ``open3d`` so the reference's numpy-only functions import offline.

Used ONLY by tools/gen_golden.py in the build container to generate golden vectors from the
reference (`/root/reference/src/matcher/ransac.py`).  Open3D 0.19.0 itself is not installed
(SURVEY.md §8c).  Nothing here is product code and nothing here travels to the GPU box.
"""
import numpy as _np

from . import geometry, io, pipelines, utility  # noqa: F401

__version__ = "0.0-stub"
