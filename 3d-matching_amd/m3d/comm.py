"""RCCL inside libm3d.so (include/m3d.h "RCCL inside the library"): the multi-GPU collectives of
the hot path are issued by the library on the caller's stream; torch.distributed only carries the
128-byte RCCL unique id from rank 0 to the other ranks (the rendezvous).

``LibComm`` has the communicator interface of ``m3d.dist`` (in-place ``min_`` / ``sum_`` /
``max_`` on cuda tensors), so the protocol drivers there run unchanged over it, and the native
multi-GPU loops (``IcpLoop.shard_steps`` / ``source_shard_steps``, ``CorrSet.run_sharded``)
take it directly.
"""

from __future__ import annotations

import ctypes as C

from . import _lib
from .core import context, ptr, stream_handle


def unique_id() -> bytes:
    buf = (C.c_uint8 * _lib.COMM_ID_BYTES)()
    _lib.check(_lib.load().m3d_comm_unique_id(buf), None, "m3d_comm_unique_id")
    return bytes(buf)


class LibComm:
    """An RCCL communicator owned by libm3d for (this process's context, rank, world)."""

    def __init__(self, rank: int, world: int, uid: bytes | None = None, ctx=None, group=None):
        self.ctx = ctx or context()
        self.rank, self.world = int(rank), int(world)
        if uid is None:  # rendezvous: rank 0's id, broadcast with torch.distributed
            import torch.distributed as dist

            box = [unique_id() if self.rank == 0 else None]
            if world > 1:
                dist.broadcast_object_list(box, src=0, group=group)
            uid = box[0]
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        raw = (C.c_uint8 * _lib.COMM_ID_BYTES)(*uid)
        h = C.c_void_p()
        self.ctx.check(self.ctx.lib.m3d_comm_init(self.ctx.h, raw, self.rank, self.world, C.byref(h)),
                       "m3d_comm_init")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.ctx.lib.m3d_comm_destroy(h)
            self.h = None

    @property
    def poisoned(self) -> bool:
        """True once the communicator was aborted after a failure (calls raise M3DCommError)."""
        return self.ctx.lib.m3d_comm_poisoned(self.h) == 1

    def inject_failure(self, what: int):
        """Test hook (m3d_debug_comm_inject): 1 fails the next local run of run_sharded, 2 the
        next ICP shard-loop iteration."""
        self.ctx.check(self.ctx.lib.m3d_debug_comm_inject(self.h, int(what)), "m3d_debug_comm_inject")

    def _ar(self, t, op):
        import torch

        dt = {torch.int32: _lib.DT_I32, torch.int64: _lib.DT_I64, torch.float64: _lib.DT_F64}.get(t.dtype)
        if dt is None or not t.is_cuda or not t.is_contiguous():
            raise ValueError("LibComm all-reduces contiguous cuda int32 / int64 / float64 tensors")
        self.ctx.check(self.ctx.lib.m3d_comm_allreduce(self.h, ptr(t), t.numel(), dt, op, stream_handle()),
                       "m3d_comm_allreduce")

    def min_(self, t):
        self._ar(t, _lib.OP_MIN)

    def sum_(self, t):
        self._ar(t, _lib.OP_SUM)

    def max_(self, t):
        self._ar(t, _lib.OP_MAX)
