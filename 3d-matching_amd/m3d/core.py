"""Python host layer over libm3d.so: contexts, device buffers, packed objects, batched calls.

PyTorch-ROCm is used only for device memory and streams (tensors' ``data_ptr()`` are passed
through the C ABI); every numerical step of the hot path runs in the HIP kernels.
"""

from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check

_tls = threading.local()


def _torch():
    import torch  # deferred: importing torch takes seconds on a cold image

    return torch


def require_device():
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("m3d needs a gfx950 (MI355X) GPU; torch.cuda is not available")
    return torch


class Context:
    """One m3d context per (host thread, device)."""

    def __init__(self, device: int = 0):
        lib = _lib.load()
        require_device()
        self.device = device
        h = C.c_void_p()
        rc = lib.m3d_create(device, C.byref(h))
        if rc == _lib.M3D_ERR_NODEVICE:
            n = C.c_int(-1)
            lib.m3d_device_count(C.byref(n))
            torch = _torch()
            arch = torch.cuda.get_device_properties(device).gcnArchName if torch.cuda.is_available() else "?"
            raise RuntimeError(f"device {device} is not a gfx950 (MI355X) GPU (libm3d sees {n.value} "
                               f"device(s); torch: {arch})")
        check(rc, None, "m3d_create")
        self.h = h
        self.lib = lib

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.lib.m3d_destroy(h)
            self.h = None

    def check(self, rc, what):
        check(rc, self.h, what)

    def trim_block_cache(self) -> int:
        """Give libm3d's idle cached device blocks back (m3d_trim_block_cache); bytes freed."""
        n = C.c_int64(0)
        self.check(self.lib.m3d_trim_block_cache(self.h, C.byref(n)), "m3d_trim_block_cache")
        return n.value

    def profile(self, enable: bool = True):
        """Record HIP events around every launch of the timed kernels (m3d_profile_enable)."""
        self.check(self.lib.m3d_profile_enable(self.h, int(enable)), "m3d_profile_enable")

    def profile_read(self, kernel: int):
        """(total_ms, launches) of `kernel` since the last read (synchronises)."""
        ms = C.c_double()
        n = C.c_int64()
        self.check(self.lib.m3d_profile_read(self.h, int(kernel), C.byref(ms), C.byref(n)),
                   "m3d_profile_read")
        return ms.value, n.value

    def stats(self) -> np.ndarray:
        out = (C.c_int64 * 8)()
        self.check(self.lib.m3d_get_stats(self.h, out), "m3d_get_stats")
        return np.array(out[:], dtype=np.int64)


def context(device: int | None = None) -> Context:
    torch = require_device()
    dev = torch.cuda.current_device() if device is None else int(device)
    cache = getattr(_tls, "ctx", None)
    if cache is None:
        cache = _tls.ctx = {}
    if dev not in cache:
        cache[dev] = Context(dev)
    return cache[dev]


def device_empty(shape, dtype):
    """torch.empty on the current cuda device.  On out-of-memory the idle blocks of libm3d's
    block cache (destroyed clouds) and torch's own cache are given back, and the allocation is
    retried once."""
    torch = _torch()
    try:
        return torch.empty(shape, dtype=dtype, device="cuda")
    except torch.cuda.OutOfMemoryError:
        context().trim_block_cache()
        torch.cuda.empty_cache()
        return torch.empty(shape, dtype=dtype, device="cuda")


def stream_handle():
    torch = _torch()
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> C.c_void_p:
    return C.c_void_p(0 if t is None else t.data_ptr())


def to_device(a, dtype="float64", shape_tail=(3,), device=None):
    """numpy / torch / sequence → contiguous torch tensor on the GPU (no copy if already there)."""
    torch = require_device()
    tdt = {"float64": torch.float64, "int32": torch.int32, "int64": torch.int64}[dtype]
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    if isinstance(a, torch.Tensor):
        t = a.to(device=dev, dtype=tdt)
    else:
        arr = np.ascontiguousarray(np.asarray(a), dtype=np.dtype(dtype))
        t = torch.from_numpy(arr).to(dev)
    if shape_tail is not None:
        t = t.reshape(-1, *shape_tail)
    return t.contiguous()


# --------------------------------------------------------------------------------- RANSAC
class CorrSet:
    """Packed correspondence set on the device (gathered fp64 pairs + centred fp32 SoA)."""

    def __init__(self, src_points=None, tgt_points=None, corr=None, *, p_src=None, p_tgt=None,
                 ctx: Context | None = None):
        self.ctx = ctx or context()
        self.device = _torch().device("cuda", self.ctx.device)
        lib = self.ctx.lib
        h = C.c_void_p()
        st = stream_handle()
        if p_src is not None:
            ps = to_device(p_src)
            pt = to_device(p_tgt)
            if ps.shape != pt.shape:
                raise ValueError("p_src and p_tgt must have the same shape")
            self.nc = ps.shape[0]
            self._keep = (ps, pt)
            self.ctx.check(lib.m3d_corrset_create_gathered(self.ctx.h, ptr(ps), ptr(pt), self.nc, st,
                                                           C.byref(h)), "corrset_create_gathered")
        else:
            s = to_device(src_points)
            t = to_device(tgt_points)
            c = to_device(corr, "int32", (2,))
            self.nc = c.shape[0]
            self._keep = (s, t, c)
            self.ctx.check(lib.m3d_corrset_create(self.ctx.h, ptr(s), s.shape[0], ptr(t), t.shape[0],
                                                  ptr(c), self.nc, st, C.byref(h)), "corrset_create")
        self.h = h
        self._keep = None  # the corrset holds its own gathered copy

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.ctx.lib.m3d_corrset_destroy(h)
            self.h = None

    def kabsch3(self, H: int, triples=None, seed: int = 0, hyp0: int = 0):
        """Batched a1: returns (T (H,4,4) torch f64 cuda, status (H,) uint8)."""
        torch = _torch()
        T = device_empty((H, 4, 4), torch.float64)
        status = device_empty((H,), torch.uint8)
        tri = None if triples is None else to_device(triples, "int32", (3,))
        self.ctx.check(self.ctx.lib.m3d_kabsch3_batch(self.ctx.h, self.h, ptr(tri), seed, hyp0, H,
                                                      ptr(T), ptr(status), stream_handle()),
                       "kabsch3_batch")
        return T, status

    def score(self, T, thr: float, mode: int = _lib.SCORE_SQUARED):
        """Batched a2/a3: inlier counts (H,) int32 for transforms T (H,4,4)."""
        torch = _torch()
        Td = to_device(T, "float64", (4, 4))
        H = Td.shape[0]
        counts = device_empty((H,), torch.int32)
        self.ctx.check(self.ctx.lib.m3d_ransac_score(self.ctx.h, self.h, ptr(Td), H, float(thr),
                                                     int(mode), ptr(counts), stream_handle()),
                       "ransac_score")
        return counts

    def kabsch3_one(self, triple):
        """a1 for one row triple (host) → (T (4,4) ndarray, status): one launch, one sync
        (m3d_kabsch3_one, the reference harness's per-call form)."""
        tri = (C.c_int32 * 3)(*(int(v) for v in triple))
        T = (C.c_double * 16)()
        st = C.c_int32(0)
        self.ctx.check(self.ctx.lib.m3d_kabsch3_one(self.ctx.h, self.h, tri, T, C.byref(st),
                                                    stream_handle()), "kabsch3_one")
        return np.array(T[:]).reshape(4, 4), int(st.value)

    def score_one(self, T, thr: float, mode: int = _lib.SCORE_SQUARED) -> int:
        """a2/a3 for one host transform → inlier count (m3d_ransac_score_one)."""
        Tc = (C.c_double * 16)(*np.asarray(T, np.float64).reshape(16).tolist())
        n = C.c_int64(0)
        self.ctx.check(self.ctx.lib.m3d_ransac_score_one(self.ctx.h, self.h, Tc, float(thr), int(mode),
                                                         C.byref(n), stream_handle()), "ransac_score_one")
        return int(n.value)

    def run(self, params: "RansacParams", triples=None) -> "RansacOutcome":
        """a4 on the device: the step-RANSAC loop with best tracking and early stop."""
        p = params.to_c()
        res = _lib.RansacResult()
        tri = None if triples is None else to_device(triples, "int32", (3,))
        self.ctx.check(self.ctx.lib.m3d_ransac_run(self.ctx.h, self.h, C.byref(p), ptr(tri),
                                                   C.byref(res), stream_handle()), "ransac_run")
        return RansacOutcome(np.array(res.T[:]).reshape(4, 4), res.fitness, res.best_index,
                             res.iterations, res.best_count, self.nc)

    def run_async(self, params: "RansacParams", result, triples=None) -> None:
        """a4 enqueued on the current stream, no host sync: the m3d_ransac_result lands in
        `result` (a cuda int64 tensor of RESULT_WORDS elements; best_index = result[17],
        best_count = result[19]).  Read it with RansacOutcome.from_device."""
        p = params.to_c()
        tri = None if triples is None else to_device(triples, "int32", (3,))
        self.ctx.check(self.ctx.lib.m3d_ransac_run_async(self.ctx.h, self.h, C.byref(p), ptr(tri), None,
                                                         ptr(result), stream_handle()), "ransac_run_async")


    def run_sharded(self, comm, params: "RansacParams") -> "RansacOutcome":
        """Hypothesis-sharded a4 over comm's ranks (m3d_ransac_run_sharded): params.hyp0 /
        max_iter = this rank's id range, no early stop; returns the global winner on every rank
        (best_index = its global id)."""
        p = params.to_c()
        res = _lib.RansacResult()
        self.ctx.check(self.ctx.lib.m3d_ransac_run_sharded(self.ctx.h, comm.h, self.h, C.byref(p),
                                                           C.byref(res), stream_handle()),
                       "ransac_run_sharded")
        return RansacOutcome(np.array(res.T[:]).reshape(4, 4), res.fitness, res.best_index,
                             res.iterations, res.best_count, self.nc)

    def best_allreduce(self, comm, result, hyp0: int, key):
        """MAX over ranks of this rank's packed best (count << 32 | ~global id) into key (cuda
        int64 (1,)), enqueued after run_async on the same stream (m3d_ransac_best_allreduce)."""
        self.ctx.check(self.ctx.lib.m3d_ransac_best_allreduce(comm.h, ptr(result), int(hyp0), ptr(key),
                                                              stream_handle()), "ransac_best_allreduce")


RESULT_WORDS = C.sizeof(_lib.RansacResult) // 8  # m3d_ransac_result as int64 words


@dataclass
class RansacParams:
    max_iter: int = 10000
    seed: int = 0
    thr: float = 0.45 * 0.45
    mode: int = _lib.SCORE_SQUARED
    early_stop: bool = True
    es_threshold: float = 0.5
    es_confidence: float = 0.99
    batch: int = 0
    hyp0: int = 0

    def to_c(self):
        return _lib.RansacParams(int(self.max_iter), int(self.seed) & ((1 << 64) - 1), float(self.thr),
                                 int(self.mode), int(bool(self.early_stop)), float(self.es_threshold),
                                 float(self.es_confidence), int(self.batch), int(self.hyp0))


@dataclass
class RansacOutcome:
    transformation: np.ndarray
    fitness: float
    best_index: int
    iterations: int
    best_count: int
    n_correspondences: int

    @staticmethod
    def from_device(result, nc: int) -> "RansacOutcome":
        """Decode the m3d_ransac_result written by CorrSet.run_async (synchronises)."""
        raw = result.detach().cpu().numpy().astype(np.int64).tobytes()
        r = _lib.RansacResult.from_buffer_copy(raw[:C.sizeof(_lib.RansacResult)])
        return RansacOutcome(np.array(r.T[:]).reshape(4, 4), r.fitness, r.best_index, r.iterations,
                             r.best_count, nc)


def replay_triples(nc: int, H: int, state=None):
    """Rows that H successive ``np.random.choice(nc, 3, replace=False)`` calls draw from the
    legacy MT19937 stream (ransac.py:143).  ``state`` defaults to the global numpy RNG, which is
    advanced exactly as the reference would advance it.  Returns (H,3) int32."""
    lib = _lib.load()
    use_global = state is None
    st = np.random.get_state() if use_global else state
    if st[0] != "MT19937":
        raise ValueError("legacy MT19937 state required")
    key = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
    pos = C.c_int32(int(st[2]))
    out = np.empty((H, 3), dtype=np.int32)
    rc = lib.m3d_replay_triples(key.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(pos), int(nc),
                                int(H), out.ctypes.data_as(C.POINTER(C.c_int32)))
    check(rc, None, "replay_triples")
    new_state = ("MT19937", key, pos.value, 0, 0.0)
    if use_global:
        np.random.set_state(new_state)
    return out, new_state


_MT_STATE_KEY_BYTES = 624 * 4  # numpy mt19937_state: uint32 key[624]; int pos
_choice3_fast = None


def _mt_state_ptrs(bitgen):
    addr = bitgen.ctypes.state_address
    return (C.cast(addr, C.POINTER(C.c_uint32)),
            C.cast(addr + _MT_STATE_KEY_BYTES, C.POINTER(C.c_int32)))


def _choice3_selftest() -> bool:
    """Whether numpy's MT19937 state can be advanced in place (layout check against numpy)."""
    try:
        lib = _lib.load()
        a, b = np.random.RandomState(20240), np.random.RandomState(20240)
        for n in (3, 50, 1025):
            exp = a.choice(n, 3, replace=False)
            key, pos = _mt_state_ptrs(b._bit_generator)
            out = (C.c_int32 * 3)()
            if lib.m3d_replay_triples(key, pos, n, 1, out) != 0 or list(out) != exp.tolist():
                return False
        sa, sb = a.get_state(), b.get_state()
        return bool(np.array_equal(sa[1], sb[1]) and sa[2] == sb[2])
    except Exception:
        return False


def choice3(nc: int) -> np.ndarray:
    """``np.random.choice(nc, 3, replace=False)`` on the global legacy RNG (ransac.py:143): the
    same three rows, and the RNG left in the same state.  numpy draws them through a full O(nc)
    permutation; the library replays the same MT19937 draws branch-free and traces only the
    first three positions (m3d_replay_triples), advancing numpy's state in place under its
    lock.  Falls back to numpy's own call if the state layout check fails."""
    global _choice3_fast
    if _choice3_fast is None:
        _choice3_fast = _choice3_selftest()
    rs = np.random.mtrand._rand
    bg = getattr(rs, "_bit_generator", None)
    if not _choice3_fast or nc < 3 or type(bg).__name__ != "MT19937":
        return np.random.choice(nc, 3, replace=False)
    out = (C.c_int32 * 3)()
    with bg.lock:
        key, pos = _mt_state_ptrs(bg)
        check(_lib.load().m3d_replay_triples(key, pos, int(nc), 1, out), None, "choice3")
    return np.array(out[:], dtype=np.int64)


# --------------------------------------------------------------------------------- ICP
class Cloud:
    """Packed point cloud on the device (fp64 AoS + centred fp32 float4, optional normals).

    center: the centring offset (3 floats) instead of the cloud's own mean.  Give every shard of
    a target-sharded cloud the same centre (e.g. the whole cloud's mean): the shards then share
    one fp32 frame and target-sharded ICP seeds non-owning ranks with a distance bound
    (m3d_cloud_create_framed)."""

    def __init__(self, points, normals=None, ctx: Context | None = None, center=None):
        """points / normals: torch cuda tensors (device arrays: m3d_cloud_create[_framed]) or
        host arrays (numpy / sequences: m3d_cloud_create_host, the library's staged upload)."""
        self.ctx = ctx or context()
        torch = _torch()
        on_dev = isinstance(points, torch.Tensor) and points.is_cuda
        if on_dev:
            p = to_device(points)
            nrm = None if normals is None else to_device(normals)
        else:
            require_device()
            p = np.ascontiguousarray(np.asarray(points, np.float64).reshape(-1, 3))
            nrm = None if normals is None else np.ascontiguousarray(
                np.asarray(normals.cpu() if isinstance(normals, torch.Tensor) else normals,
                           np.float64).reshape(-1, 3))
        if nrm is not None and nrm.shape != p.shape:
            raise ValueError("normals must match points")
        self.n = p.shape[0]
        h = C.c_void_p()
        c3 = None if center is None else (C.c_double * 3)(*[float(x) for x in np.asarray(center, np.float64).reshape(3)])
        if not on_dev:
            rc = self.ctx.lib.m3d_cloud_create_host(self.ctx.h, p.ctypes.data if self.n else None,
                                                    nrm.ctypes.data if nrm is not None else None, self.n, c3,
                                                    stream_handle(), C.byref(h))
        elif center is None:
            rc = self.ctx.lib.m3d_cloud_create(self.ctx.h, ptr(p), ptr(nrm), self.n, stream_handle(),
                                               C.byref(h))
        else:
            rc = self.ctx.lib.m3d_cloud_create_framed(self.ctx.h, ptr(p), ptr(nrm), self.n, c3,
                                                      stream_handle(), C.byref(h))
        self.ctx.check(rc, "cloud_create")
        self.h = h
        self.has_normals = nrm is not None

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.ctx.lib.m3d_cloud_destroy(h)
            self.h = None


def _T16(T):
    a = np.ascontiguousarray(np.asarray(T, dtype=np.float64).reshape(16))
    return (C.c_double * 16)(*a.tolist())


def _nn_method(nn: str) -> int:
    try:
        return _lib.NN_METHODS[nn]
    except KeyError:
        raise ValueError(f"nn must be one of {sorted(_lib.NN_METHODS)}, got {nn!r}") from None


def nn1(src: Cloud, tgt: Cloud, T, max_dist: float, nn: str = "grid"):
    """Radius-bounded 1-NN of T·src in tgt → (idx int32 (-1 none), d2 f64) torch cuda.

    nn="brute" scans every target, nn="grid" only the uniform-grid cells within the radius;
    both return the identical result (grid.hip header)."""
    torch = _torch()
    idx = device_empty((src.n,), torch.int32)
    d2 = device_empty((src.n,), torch.float64)
    src.ctx.check(src.ctx.lib.m3d_nn1(src.ctx.h, src.h, tgt.h, _T16(T), float(max_dist),
                                      _nn_method(nn), ptr(idx), ptr(d2), stream_handle()), "nn1")
    return idx, d2


@dataclass
class IcpOutcome:
    transformation: np.ndarray
    fitness: float
    inlier_rmse: float
    num_correspondences: int
    iterations: int
    converged: bool
    correspondence_set: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.int32))
    update: np.ndarray = field(default_factory=lambda: np.eye(4))  # the last ΔT (I since reset)


def corr_pairs(ctx: Context, corr, n: int) -> np.ndarray:
    """RegistrationResult.correspondence_set of a per-source index array (cuda int32, -1 none):
    the (i, corr[i]) pairs with corr[i] >= 0 in increasing i, compacted on the device
    (m3d_corr_pairs) — only the pairs cross to the host."""
    out = np.empty((max(n, 1), 2), np.int32)
    m = C.c_int64(0)
    ctx.check(ctx.lib.m3d_corr_pairs(ctx.h, ptr(corr) if n > 0 else None, int(n), out.ctypes.data, C.byref(m),
                                     stream_handle()), "corr_pairs")
    return out[: m.value]


def icp(src: Cloud, tgt: Cloud, max_dist: float, init=None, estimation=_lib.EST_POINT_TO_PLANE,
        relative_fitness=1e-6, relative_rmse=1e-6, max_iteration=30, with_correspondences=True,
        nn: str = "grid"):
    """registration_icp on the device (m3d_icp_run)."""
    torch = _torch()
    p = _lib.IcpParams(float(relative_fitness), float(relative_rmse), int(max_iteration), int(estimation),
                       _nn_method(nn), 0)
    res = _lib.IcpResult()
    corr = device_empty((max(src.n, 1),), torch.int32) if with_correspondences else None
    init16 = _T16(np.eye(4) if init is None else init)
    src.ctx.check(src.ctx.lib.m3d_icp_run(src.ctx.h, src.h, tgt.h, init16, float(max_dist), C.byref(p),
                                          C.byref(res), ptr(corr), stream_handle()), "icp_run")
    cs = corr_pairs(src.ctx, corr, src.n) if with_correspondences else np.zeros((0, 2), np.int32)
    return IcpOutcome(np.array(res.T[:]).reshape(4, 4), res.fitness, res.inlier_rmse,
                      res.num_correspondences, res.iterations, bool(res.converged), cs,
                      np.array(res.update[:]).reshape(4, 4))


class IcpLoop:
    """Step-wise device ICP (benchmarks, multi-GPU).  Every call only enqueues work."""

    def __init__(self, src: Cloud, tgt: Cloud, max_dist: float, estimation=_lib.EST_POINT_TO_PLANE,
                 relative_fitness=1e-6, relative_rmse=1e-6, max_iteration=30, nn: str = "brute",
                 split: bool = True):
        """split=False: the target-shard loop exchanges its keys in one piece (no overlap with
        the second half's NN)."""
        self.ctx = src.ctx
        self.src, self.tgt = src, tgt
        flags = 0 if split else _lib.ICP_NO_SPLIT
        self.p = _lib.IcpParams(float(relative_fitness), float(relative_rmse), int(max_iteration),
                                int(estimation), _nn_method(nn), flags)
        h = C.c_void_p()
        self.ctx.check(self.ctx.lib.m3d_icp_create(self.ctx.h, src.h, tgt.h, float(max_dist),
                                                   C.byref(self.p), C.byref(h)), "icp_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.ctx.lib.m3d_icp_destroy(h)
            self.h = None

    def reset(self, init=None):
        self.ctx.check(self.ctx.lib.m3d_icp_reset(self.h, _T16(np.eye(4) if init is None else init),
                                                  stream_handle()), "icp_reset")

    def step(self):
        self.ctx.check(self.ctx.lib.m3d_icp_step(self.h, stream_handle()), "icp_step")

    def steps(self, n: int):
        """n iterations enqueued by the library in one call (m3d_icp_steps; a sequence requested
        again is replayed from a captured HIP graph)."""
        self.ctx.check(self.ctx.lib.m3d_icp_steps(self.h, int(n), stream_handle()), "icp_steps")

    def prepare_steps(self, n: int):
        """Capture the n-step graph now for the current state (setup; m3d_icp_prepare_steps)."""
        self.ctx.check(self.ctx.lib.m3d_icp_prepare_steps(self.h, int(n)), "icp_prepare_steps")

    def shard_nn(self, offset: int, dkeys):
        """This shard's NN.  dkeys (cuda int64, ns) → target shard: bits of the shard's fp64
        winner d² per source (INT64_MAX none), to be MIN-reduced over ranks; None → source
        shard (the keys stay inside the loop object)."""
        self.ctx.check(self.ctx.lib.m3d_icp_shard_nn(self.h, int(offset), ptr(dkeys), stream_handle()),
                       "icp_shard_nn")

    def shard_nn_range(self, offset: int, q0: int, q1: int, dkeys):
        """shard_nn for the source slots [q0, q1) (the split exchange's pieces)."""
        self.ctx.check(self.ctx.lib.m3d_icp_shard_nn_range(self.h, int(offset), int(q0), int(q1), ptr(dkeys),
                                                           stream_handle()), "icp_shard_nn_range")

    def shard_claim(self, dmin, claim):
        """Target shard, after MIN(dkeys): claim (cuda int32, ns) = own winner's index where it
        has the global d², else INT32_MAX; MIN-reduce it over ranks."""
        self.ctx.check(self.ctx.lib.m3d_icp_shard_claim(self.h, ptr(dmin), ptr(claim), stream_handle()),
                       "icp_shard_claim")

    def shard_terms(self, offset: int, dmin, claim, sums):
        """Estimation terms of the owned winners → sums (cuda f64, 32), to be SUM-reduced.
        Source shard: dmin = claim = None."""
        self.ctx.check(self.ctx.lib.m3d_icp_shard_terms(self.h, int(offset), ptr(dmin), ptr(claim),
                                                        ptr(sums), stream_handle()), "icp_shard_terms")

    def solve(self, sums):
        self.ctx.check(self.ctx.lib.m3d_icp_solve(self.h, ptr(sums), stream_handle()), "icp_solve")

    def shard_steps(self, comm, offset: int, n: int):
        """n target-sharded iterations with the MIN / MIN / SUM all-reduces issued by libm3d
        (m3d_icp_shard_steps; comm = m3d.comm.LibComm)."""
        self.ctx.check(self.ctx.lib.m3d_icp_shard_steps(self.h, comm.h, int(offset), int(n), stream_handle()),
                       "icp_shard_steps")

    def source_shard_steps(self, comm, n: int):
        """n source-sharded iterations (one SUM all-reduce each) issued by libm3d."""
        self.ctx.check(self.ctx.lib.m3d_icp_source_shard_steps(self.h, comm.h, int(n), stream_handle()),
                       "icp_source_shard_steps")

    def set_source_total(self, ns_total: int):
        """Source-sharded runs: fitness denominator = sources over all ranks."""
        self.ctx.check(self.ctx.lib.m3d_icp_set_source_total(self.h, int(ns_total)), "icp_set_source_total")

    def result(self) -> IcpOutcome:
        r = _lib.IcpResult()
        self.ctx.check(self.ctx.lib.m3d_icp_result_get(self.h, C.byref(r), stream_handle()), "icp_result")
        return IcpOutcome(np.array(r.T[:]).reshape(4, 4), r.fitness, r.inlier_rmse,
                          r.num_correspondences, r.iterations, bool(r.converged),
                          update=np.array(r.update[:]).reshape(4, 4))

    def points(self):
        """The loop's fp64 points of the last evaluation (ns×3 f64 torch cuda, source order):
        RegistrationICP's transformed copy of the source (init applied unless it isIdentity(),
        then every update), from which that evaluation's correspondences and terms were taken;
        after a reset and before the first evaluation, init·source (the source itself when init
        isIdentity()), as RegistrationICP's pcd at that point."""
        torch = _torch()
        out = device_empty((max(self.src.n, 1), 3), torch.float64)
        self.ctx.check(self.ctx.lib.m3d_icp_copy_points(self.h, ptr(out), stream_handle()), "icp_copy_points")
        return out[: self.src.n]

    def source_slots(self):
        """Slot → source point index (int32 torch cuda): the loop holds its source in the Morton
        order of the source grid; exchange buffers (dkeys / claims) are indexed by slot."""
        torch = _torch()
        out = device_empty((max(self.src.n, 1),), torch.int32)
        self.ctx.check(self.ctx.lib.m3d_icp_copy_slots(self.h, ptr(out), stream_handle()), "icp_copy_slots")
        return out[: self.src.n]

    def correspondences(self):
        """Current correspondence target per source point (int32, -1 = none), torch cuda."""
        torch = _torch()
        out = device_empty((max(self.src.n, 1),), torch.int32)
        self.ctx.check(self.ctx.lib.m3d_icp_copy_corr(self.h, ptr(out), stream_handle()), "icp_copy_corr")
        return out[: self.src.n]
