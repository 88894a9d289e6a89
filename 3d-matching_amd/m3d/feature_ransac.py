"""Feature-matching RANSAC (Open3D RegistrationRANSACBasedOnFeatureMatching) — see DESIGN.md §6."""

from __future__ import annotations


def correspondences_from_features(src_fpfh, tgt_fpfh, mutual_filter=False):
    raise NotImplementedError("feature-space correspondences: SURVEY.md §8(f) rank 3, not built yet")


def registration_ransac_based_on_feature_matching(*args, **kwargs):
    raise NotImplementedError("feature-matching RANSAC (a6): not built yet")
