"""``register(source, target)`` — the coarse-to-fine pipeline `src/main.py:24-43` intends.

The reference's ``main()`` calls ``global_registration(src_ply, tgt_ply)`` and
``refine_registration(src_ply, tgt_ply, T)`` without the required ``voxel_size`` (TypeError as
written).  This façade supplies it (``Ply.voxel_size``, default 0.3) and composes
the same two stages on the device:

1. coarse: ``global_registration`` when both inputs carry FPFH features (``pcd_fpfh``), else the
   step-RANSAC loop (``run_ransac``) over the given ``correspondences``;
2. fine: ``refine_registration`` (point-to-plane ICP, radius 0.4·voxel) from the coarse result.
"""

from __future__ import annotations

from .icp import refine_registration
from .ransac import global_registration, run_ransac


def register(source, target, voxel_size=None, correspondences=None, ransac_iterations: int = 10000,
             refine: bool = True, iteration: int = 30, **ransac_kwargs):
    """Return the refined ``RegistrationResult`` mapping ``source`` onto ``target``.

    ``iteration``: RANSACConvergenceCriteria max_iteration of the feature path
    (global_registration's own default, 30); ``ransac_iterations``: hypotheses of the
    correspondence path."""
    v = voxel_size if voxel_size is not None else getattr(source, "voxel_size", 0.3)
    if correspondences is None and getattr(source, "pcd_fpfh", None) is not None \
            and getattr(target, "pcd_fpfh", None) is not None:
        coarse = global_registration(source, target, v, iteration=iteration)
    elif correspondences is not None:
        coarse, _ = run_ransac(source, target, correspondences, voxel_size=v, max_iter=ransac_iterations,
                           **ransac_kwargs)
    else:
        raise ValueError("register needs FPFH features on both inputs (pcd_fpfh) or correspondences")
    if not refine:
        return coarse
    return refine_registration(source, target, coarse.transformation, v)
