"""MI355X-native ``matcher`` package — drop-in for KTC-Security-Circle/3d-matching ``src/matcher``.

Put ``3d-matching_amd`` on ``PYTHONPATH`` where the reference put ``src``
(`.devcontainer/Dockerfile:39`) and ``from matcher.ransac import ...`` / ``from matcher.icp
import ...`` resolve to these modules.  (The package namespace keeps ``matcher.ransac`` and
``matcher.icp`` as the submodules, exactly like the reference's empty ``__init__``.)  ``register(source, target)`` is the coarse-to-fine
façade the reference's ``main()`` intends (`src/main.py:34-38`).
"""

from __future__ import annotations

from .icp import refine_registration, registration_icp
from .ransac import (
    compute_feature_correspondences,
    compute_step_transformation,
    evaluate_inlier_ratio,
    evaluate_inlier_ratio_fast,
    global_registration,
    run_ransac,
)
from .register import register

__all__ = [
    "compute_feature_correspondences",
    "compute_step_transformation",
    "evaluate_inlier_ratio",
    "evaluate_inlier_ratio_fast",
    "global_registration",
    "run_ransac",
    "refine_registration",
    "registration_icp",
    "register",
]
