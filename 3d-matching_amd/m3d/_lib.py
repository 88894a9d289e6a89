"""ctypes binding of libm3d.so (include/m3d.h).

The library is built in-tree (``make -C 3d-matching_amd/csrc`` or ``__graft_entry__.build()``)
and loaded from this directory.  There is no fallback: if the shared object or a gfx950 device
is missing, the product path raises.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libm3d.so"

M3D_OK = 0
M3D_ERR_INVALID = -1
M3D_ERR_HIP = -2
M3D_ERR_OOM = -3
M3D_ERR_NODEVICE = -4
M3D_ERR_COMM = -5

HYP_OK, HYP_DEGENERATE, HYP_NONFINITE = 0, 1, 2
SCORE_SQUARED, SCORE_NORM = 0, 1
EST_POINT_TO_POINT, EST_POINT_TO_PLANE = 0, 1
KERNEL_NN, KERNEL_SCORE, KERNEL_KABSCH, KERNEL_TERMS, KERNEL_LOOP, KERNEL_COMM = 0, 1, 2, 3, 4, 5
ICP_NO_SPLIT = 2
NN_BRUTE, NN_GRID = 0, 1
COMM_ID_BYTES = 128
DT_I32, DT_I64, DT_F64 = 0, 1, 2
OP_SUM, OP_MIN, OP_MAX = 0, 1, 2
NN_METHODS = {"brute": NN_BRUTE, "grid": NN_GRID}
ABI_VERSION = 13

vp = C.c_void_p
i64 = C.c_int64
u64 = C.c_uint64
i32 = C.c_int32
dbl = C.c_double


class RansacParams(C.Structure):
    _fields_ = [("max_iter", i64), ("seed", u64), ("thr", dbl), ("mode", i32),
                ("early_stop", i32), ("es_threshold", dbl), ("es_confidence", dbl),
                ("batch", i64), ("hyp0", i64)]


class RansacResult(C.Structure):
    _fields_ = [("T", dbl * 16), ("fitness", dbl), ("best_index", i64), ("iterations", i64),
                ("best_count", i64), ("rechecked", i64)]


class IcpParams(C.Structure):
    _fields_ = [("relative_fitness", dbl), ("relative_rmse", dbl), ("max_iteration", i32),
                ("estimation", i32), ("nn_method", i32), ("flags", i32)]


class FeatureRansacParams(C.Structure):
    _fields_ = [("max_correspondence_distance", dbl), ("confidence", dbl), ("edge_length", dbl),
                ("distance", dbl), ("seed", u64), ("max_iteration", i32), ("ransac_n", i32)]


class FeatureRansacResult(C.Structure):
    _fields_ = [("T", dbl * 16), ("fitness", dbl), ("inlier_rmse", dbl), ("best_index", i64),
                ("validations", i64), ("corres_ratio", dbl)]


class IcpResult(C.Structure):
    _fields_ = [("T", dbl * 16), ("fitness", dbl), ("inlier_rmse", dbl),
                ("num_correspondences", i64), ("iterations", i32), ("converged", i32),
                ("update", dbl * 16)]


# name -> (restype, argtypes)
SIGNATURES = {
    "m3d_abi_version": (C.c_int, []),
    "m3d_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "m3d_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "m3d_destroy": (None, [vp]),
    "m3d_last_error": (C.c_char_p, [vp]),
    "m3d_get_stats": (C.c_int, [vp, C.POINTER(i64)]),
    "m3d_trim_block_cache": (C.c_int, [vp, C.POINTER(i64)]),
    "m3d_profile_enable": (C.c_int, [vp, C.c_int]),
    "m3d_profile_read": (C.c_int, [vp, C.c_int, C.POINTER(dbl), C.POINTER(i64)]),
    "m3d_corrset_create": (C.c_int, [vp, vp, i64, vp, i64, vp, i64, vp, C.POINTER(vp)]),
    "m3d_corrset_create_gathered": (C.c_int, [vp, vp, vp, i64, vp, C.POINTER(vp)]),
    "m3d_corrset_destroy": (None, [vp]),
    "m3d_corrset_size": (i64, [vp]),
    "m3d_kabsch3_batch": (C.c_int, [vp, vp, vp, u64, i64, i64, vp, vp, vp]),
    "m3d_ransac_score": (C.c_int, [vp, vp, vp, i64, dbl, C.c_int, vp, vp]),
    "m3d_kabsch3_one": (C.c_int, [vp, vp, C.POINTER(i32), C.POINTER(dbl), C.POINTER(i32), vp]),
    "m3d_ransac_score_one": (C.c_int, [vp, vp, C.POINTER(dbl), dbl, C.c_int, C.POINTER(i64), vp]),
    "m3d_ransac_run": (C.c_int, [vp, vp, C.POINTER(RansacParams), vp, C.POINTER(RansacResult), vp]),
    "m3d_ransac_run_async": (C.c_int, [vp, vp, C.POINTER(RansacParams), vp, vp, vp, vp]),
    "m3d_replay_triples": (C.c_int, [C.POINTER(C.c_uint32), C.POINTER(i32), i64, i64,
                                     C.POINTER(i32)]),
    "m3d_cloud_create": (C.c_int, [vp, vp, vp, i64, vp, C.POINTER(vp)]),
    "m3d_cloud_create_framed": (C.c_int, [vp, vp, vp, i64, C.POINTER(C.c_double), vp, C.POINTER(vp)]),
    "m3d_cloud_create_host": (C.c_int, [vp, vp, vp, i64, C.POINTER(C.c_double), vp, C.POINTER(vp)]),
    "m3d_cloud_destroy": (None, [vp]),
    "m3d_cloud_size": (i64, [vp]),
    "m3d_nn1": (C.c_int, [vp, vp, vp, C.POINTER(dbl), dbl, i32, vp, vp, vp]),
    "m3d_icp_run": (C.c_int, [vp, vp, vp, C.POINTER(dbl), dbl, C.POINTER(IcpParams),
                              C.POINTER(IcpResult), vp, vp]),
    "m3d_icp_create": (C.c_int, [vp, vp, vp, dbl, C.POINTER(IcpParams), C.POINTER(vp)]),
    "m3d_icp_destroy": (None, [vp]),
    "m3d_icp_reset": (C.c_int, [vp, C.POINTER(dbl), vp]),
    "m3d_icp_step": (C.c_int, [vp, vp]),
    "m3d_icp_steps": (C.c_int, [vp, C.c_int32, vp]),
    "m3d_icp_prepare_steps": (C.c_int, [vp, C.c_int32]),
    "m3d_icp_shard_nn": (C.c_int, [vp, i64, vp, vp]),
    "m3d_icp_shard_nn_range": (C.c_int, [vp, i64, i64, i64, vp, vp]),
    "m3d_icp_shard_claim": (C.c_int, [vp, vp, vp, vp]),
    "m3d_icp_shard_terms": (C.c_int, [vp, i64, vp, vp, vp, vp]),
    "m3d_icp_solve": (C.c_int, [vp, vp, vp]),
    "m3d_icp_result_get": (C.c_int, [vp, C.POINTER(IcpResult), vp]),
    "m3d_icp_set_source_total": (C.c_int, [vp, i64]),
    "m3d_icp_corr": (vp, [vp]),
    "m3d_icp_copy_corr": (C.c_int, [vp, vp, vp]),
    "m3d_corr_pairs": (C.c_int, [vp, vp, i64, vp, C.POINTER(i64), vp]),
    "m3d_icp_copy_slots": (C.c_int, [vp, vp, vp]),
    "m3d_icp_copy_points": (C.c_int, [vp, vp, vp]),
    "m3d_voxel_down_sample": (C.c_int, [vp, vp, vp, i64, dbl, vp, vp, C.POINTER(i64), vp]),
    "m3d_hybrid_search": (C.c_int, [vp, vp, dbl, i32, vp, vp, vp, vp]),
    "m3d_estimate_normals": (C.c_int, [vp, vp, dbl, i32, vp, vp]),
    "m3d_compute_fpfh": (C.c_int, [vp, vp, vp, dbl, i32, vp, vp]),
    "m3d_feature_correspondences": (C.c_int, [vp, vp, i64, vp, i64, i32, i32, dbl, vp,
                                              C.POINTER(i64), vp]),
    "m3d_ransac_on_correspondences": (C.c_int, [vp, vp, vp, vp, i64, C.POINTER(FeatureRansacParams),
                                                C.POINTER(FeatureRansacResult), vp, vp]),
    "m3d_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "m3d_comm_init": (C.c_int, [vp, C.POINTER(C.c_uint8), C.c_int, C.c_int, C.POINTER(vp)]),
    "m3d_comm_destroy": (None, [vp]),
    "m3d_comm_allreduce": (C.c_int, [vp, vp, i64, C.c_int, C.c_int, vp]),
    "m3d_icp_shard_steps": (C.c_int, [vp, vp, i64, i32, vp]),
    "m3d_icp_source_shard_steps": (C.c_int, [vp, vp, i32, vp]),
    "m3d_ransac_best_allreduce": (C.c_int, [vp, vp, i64, vp, vp]),
    "m3d_ransac_run_sharded": (C.c_int, [vp, vp, vp, C.POINTER(RansacParams), C.POINTER(RansacResult), vp]),
    "m3d_comm_poisoned": (C.c_int, [vp]),
    "m3d_debug_comm_inject": (C.c_int, [vp, C.c_int]),
    "m3d_debug_acos_cr": (C.c_int, [vp, C.c_int64, vp]),
    "m3d_debug_acos_device": (C.c_int, [vp, vp, C.c_int64, vp, C.c_int, vp]),
    "m3d_debug_block_cache_fill": (C.c_int, [C.c_int]),
    "m3d_debug_icp_defer_count": (C.c_int, [vp, C.c_uint32, vp]),
    "m3d_parse_ascii_rows": (C.c_int, [C.c_char_p, C.c_size_t, i64, i32, C.POINTER(dbl),
                                       C.POINTER(C.c_size_t)]),
    "m3d_format_ascii_rows": (C.c_int, [C.POINTER(dbl), i64, i32, vp, C.c_size_t, C.POINTER(C.c_size_t)]),
    "m3d_merge_vertices": (C.c_int, [C.POINTER(dbl), i64, C.POINTER(dbl), C.POINTER(i32), C.POINTER(i64)]),
    "m3d_content_keys": (C.c_int, [C.POINTER(vp), C.POINTER(C.c_size_t), i32, C.POINTER(u64)]),
    "m3d_debug_xxh64": (u64, [vp, C.c_size_t, u64]),
    "m3d_debug_xxh3_128": (C.c_int, [vp, C.c_size_t, C.POINTER(u64)]),
    "m3d_debug_kabsch3_host":(C.c_int, [C.POINTER(dbl), C.POINTER(dbl), C.POINTER(dbl)]),
    "m3d_debug_ldlt6_host": (C.c_int, [C.POINTER(dbl), C.POINTER(dbl), C.POINTER(dbl)]),
}

_lib = None


class M3DError(RuntimeError):
    pass


class M3DCommError(M3DError):
    """A peer rank failed, or the communicator was aborted after a failure (M3D_ERR_COMM)."""


def load() -> C.CDLL:
    """Load libm3d.so (once).  Raises ImportError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} not built: run `make -C {LIB_PATH.parent.parent / 'csrc'}` "
                          "(hipcc --offload-arch=gfx950)")
    # torch first: PyTorch-ROCm ships its own HIP/HSA runtime libraries.  Imported first, they
    # are the copies libm3d.so binds to (same sonames) and the process has ONE runtime; loaded
    # after libm3d.so (e.g. plyio's host text helpers before any device call), torch brings up a
    # second runtime and libm3d's then reports no device (measured on the MI355X box).
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - host-only use without torch
        pass
    lib = C.CDLL(os.fspath(LIB_PATH))
    lib.m3d_abi_version.restype = C.c_int
    if lib.m3d_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI {lib.m3d_abi_version()} != {ABI_VERSION}; rebuild it")
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc: int, ctx=None, what: str = "") -> None:
    if rc == M3D_OK:
        return
    msg = ""
    if ctx is not None:
        raw = load().m3d_last_error(ctx)
        msg = raw.decode() if raw else ""
    if rc == M3D_ERR_INVALID:
        raise ValueError(f"{what}: {msg}" if msg else what)
    if rc == M3D_ERR_COMM:
        raise M3DCommError(f"{what} failed (code {rc}): {msg}")
    raise M3DError(f"{what} failed (code {rc}): {msg}")
