// comm.cpp — RCCL inside libm3d.so (include/m3d.h "RCCL inside the library").
//
// One communicator per (context, rank), one process per GPU.  The multi-GPU loops of the hot
// path enqueue their collectives on the caller's stream between the library's own kernels, so
// an iteration of target-sharded ICP is NN → MIN(d64 keys) → claim → MIN(claims) → terms →
// SUM(32 term slots) → solve with no host round trip (the reference's icp.py:42-48 with the
// correspondence search split over the node's GPUs).  xGMI is point-to-point: the 8·Ns-byte key
// MIN is one ring all-reduce per iteration (8 MB at 1M sources ≈ 0.1 ms per link ring), the
// claim MIN half that, the terms SUM 256 B (latency only).
//
// Failure contract (no rank may be left waiting inside a collective its peers never join):
//   * scratch is allocated before a loop's first collective, and every rank agrees on the outcome
//     (one 4-byte MAX, the loop object's first call only): a rank whose setup failed returns its
//     own error, its peers M3D_ERR_COMM — nobody enters the loop;
//   * the hypothesis-sharded RANSAC is fail-soft: a rank whose local run failed still joins both
//     collectives with neutral values and a failed-rank count in the SUM payload, so every rank
//     returns an error from the same call;
//   * a failure inside a collective loop (a launch or RCCL error mid-iteration) aborts the
//     communicator (ncclCommAbort) and poisons it: every later call on it returns M3D_ERR_COMM.
//     Peers already inside a collective are not reachable from here — the caller must tear down
//     every rank (torch.distributed.run stops the job when one worker exits with an error).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "m3d_internal.h"

struct m3d_comm {
  m3d_ctx* ctx = nullptr;
  ncclComm_t nccl = nullptr;
  int rank = 0, world = 1;
  bool poisoned = false;
  int inject = 0;           // test hook (m3d_debug_comm_inject): 1 = fail the next local RANSAC
                            // run, 2 = fail the next ICP loop iteration
  int64_t* key = nullptr;   // RANSAC key scratch (1 int64, m3d_ransac_best_allreduce)
  int64_t* rbuf = nullptr;  // run_sharded: [0] key (MAX), [1..19] SUM payload (ransac.hip)
  int64_t* hbuf = nullptr;  // pinned host copy of rbuf
  int32_t* flag = nullptr;  // setup agreement (MAX of the failed flags)
  m3d_ransac_result* dres = nullptr;  // run_sharded: this rank's local result
  hipStream_t xs = nullptr;           // target-shard loop: the exchange of the first source half
  hipEvent_t ev_a = nullptr, ev_x = nullptr;
};

using namespace m3d;

namespace {
int comm_fail(m3d_ctx* ctx, ncclResult_t r, const char* what) {
  return m3d_fail(ctx, M3D_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

// a failure inside a collective loop: abort the communicator, later calls fail fast
int poison(m3d_comm* c, int rc) {
  if (!c->poisoned) {
    if (c->nccl != nullptr) ncclCommAbort(c->nccl);
    c->nccl = nullptr;
    c->poisoned = true;
  }
  return rc;
}

int poisoned_error(m3d_comm* c) {
  return m3d_fail(c->ctx, M3D_ERR_COMM,
                  "communicator aborted after a failure inside a collective loop; tear down every rank");
}

int allreduce(m3d_comm* c, void* buf, int64_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t st) {
  if (count == 0) return M3D_OK;
  // profiling on: events around the collective on its own stream (M3D_KERNEL_COMM), so a run can
  // report exchange time beside NN and terms time
  KTimer kt(c->ctx, M3D_KERNEL_COMM, st);
  const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, dt, op, c->nccl, st);
  if (r != ncclSuccess) return poison(c, comm_fail(c->ctx, r, "ncclAllReduce"));
  return M3D_OK;
}

ncclDataType_t dtype_of(int dt) {
  return dt == M3D_DT_I32 ? ncclInt32 : (dt == M3D_DT_I64 ? ncclInt64 : ncclFloat64);
}
ncclRedOp_t op_of(int op) { return op == M3D_OP_MIN ? ncclMin : (op == M3D_OP_MAX ? ncclMax : ncclSum); }

template <class T>
int alloc_once(m3d_ctx* ctx, T** p, int64_t count) {
  if (*p != nullptr) return M3D_OK;
  if (dev_malloc(reinterpret_cast<void**>(p), sizeof(T) * (size_t)std::max<int64_t>(count, 1)) != hipSuccess) {
    *p = nullptr;
    return m3d_fail(ctx, M3D_ERR_OOM, "exchange buffer hipMalloc failed");
  }
  return M3D_OK;
}

// Setup agreement: MAX over ranks of "my setup failed"; one host sync.  Own error first, else
// M3D_ERR_COMM when a peer failed.
int agree(m3d_comm* c, int local_rc, hipStream_t st) {
  int32_t* h = reinterpret_cast<int32_t*>(c->hbuf);
  h[0] = local_rc != M3D_OK ? 1 : 0;
  hipError_t e = hipMemcpyAsync(c->flag, h, sizeof(int32_t), hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return poison(c, m3d_fail(c->ctx, M3D_ERR_HIP, "agreement copy"));
  int rc = allreduce(c, c->flag, 1, ncclInt32, ncclMax, st);
  if (rc) return rc;
  if (hipMemcpyAsync(h, c->flag, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return poison(c, m3d_fail(c->ctx, M3D_ERR_HIP, "agreement sync"));
  if (local_rc != M3D_OK) return local_rc;
  if (h[0] != 0) return m3d_fail(c->ctx, M3D_ERR_COMM, "a peer rank failed before the collective loop");
  return M3D_OK;
}

// Target-shard loop: split the sources into two slot halves so that the first half's d64 MIN
// runs on the exchange stream while the second half's NN runs (M3D_ICP_NO_SPLIT: one piece).
bool split_exchange(const m3d_icp* s) {
  return !(s->params.flags & M3D_ICP_NO_SPLIT) && s->src->n >= 2 * 4096 && icp_nn_range_ok(s);
}
}  // namespace

extern "C" {

int m3d_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return M3D_ERR_INVALID;
  static_assert(sizeof(ncclUniqueId) == M3D_COMM_ID_BYTES, "unique id size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return M3D_ERR_HIP;
  memcpy(id_out, &id, sizeof(id));
  return M3D_OK;
}

int m3d_comm_init(m3d_ctx* ctx, const uint8_t* id, int rank, int world, m3d_comm** out) {
  if (!ctx) return M3D_ERR_INVALID;
  if (!id || !out || world < 1 || rank < 0 || rank >= world)
    return m3d_fail(ctx, M3D_ERR_INVALID, "invalid communicator arguments");
  *out = nullptr;
  hipSetDevice(ctx->device);
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  m3d_comm* c = new m3d_comm();
  c->ctx = ctx;
  c->rank = rank;
  c->world = world;
  const ncclResult_t r = ncclCommInitRank(&c->nccl, world, uid, rank);
  if (r != ncclSuccess) {
    c->nccl = nullptr;
    delete c;
    return comm_fail(ctx, r, "ncclCommInitRank");
  }
  // every buffer the collectives use is allocated here, once (no allocation between collectives)
  if (dev_malloc(&c->key, sizeof(int64_t)) != hipSuccess || dev_malloc(&c->rbuf, 20 * sizeof(int64_t)) != hipSuccess ||
      dev_malloc(&c->flag, sizeof(int32_t)) != hipSuccess ||
      dev_malloc(&c->dres, sizeof(m3d_ransac_result)) != hipSuccess ||
      hipHostMalloc(&c->hbuf, 20 * sizeof(int64_t), hipHostMallocDefault) != hipSuccess ||
      hipStreamCreateWithFlags(&c->xs, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_a, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_x, hipEventDisableTiming) != hipSuccess) {
    m3d_comm_destroy(c);
    return m3d_fail(ctx, M3D_ERR_OOM, "communicator scratch");
  }
  *out = c;
  return M3D_OK;
}

void m3d_comm_destroy(m3d_comm* c) {
  if (!c) return;
  if (c->nccl) ncclCommDestroy(c->nccl);
  if (c->xs) hipStreamDestroy(c->xs);
  if (c->ev_a) hipEventDestroy(c->ev_a);
  if (c->ev_x) hipEventDestroy(c->ev_x);
  hipFree(c->key);
  hipFree(c->rbuf);
  hipFree(c->flag);
  hipFree(c->dres);
  hipHostFree(c->hbuf);
  delete c;
}

int m3d_comm_allreduce(m3d_comm* c, void* buf, int64_t count, int dtype, int op, void* stream) {
  if (!c) return M3D_ERR_INVALID;
  if (c->poisoned) return poisoned_error(c);
  if (count < 0 || (count > 0 && !buf) || dtype < M3D_DT_I32 || dtype > M3D_DT_F64 ||
      op < M3D_OP_SUM || op > M3D_OP_MAX)
    return m3d_fail(c->ctx, M3D_ERR_INVALID, "invalid all-reduce arguments");
  return allreduce(c, buf, count, dtype_of(dtype), op_of(op), reinterpret_cast<hipStream_t>(stream));
}

int m3d_icp_shard_steps(m3d_icp* s, m3d_comm* c, int64_t off, int32_t n, void* stream) {
  if (!s || !c) return M3D_ERR_INVALID;
  m3d_ctx* ctx = s->ctx;
  if (c->poisoned) return poisoned_error(c);
  if (n < 0) return m3d_fail(ctx, M3D_ERR_INVALID, "n must be >= 0");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  Touch tch{ctx, st};
  const int64_t ns = s->src->n;
  int rc;
  if (!s->xready_tgt) {  // scratch before the first collective, then every rank agrees
    rc = alloc_once(ctx, &s->xdk, ns);
    if (!rc) rc = alloc_once(ctx, &s->xcl, ns);
    if (!rc) rc = alloc_once(ctx, &s->xsums, kTermSlots);
    if ((rc = agree(c, rc, st))) return rc;
    s->xready_tgt = true;
  }
  const bool split = split_exchange(s);
  // the halves meet on a 4096-slot boundary (whole MFMA query blocks / grid blocks)
  const int64_t h = split ? (ns / 2 + 4095) / 4096 * 4096 : ns;
  for (int32_t k = 0; k < n; ++k) {
    if (c->inject == 2) {
      c->inject = 0;
      return poison(c, m3d_fail(ctx, M3D_ERR_HIP, "injected failure (m3d_debug_comm_inject)"));
    }
    if (split) {
      // half A: NN + winners, its MIN on the exchange stream while half B's NN runs here
      if ((rc = icp_shard_nn_range(s, off, 0, h, s->xdk, st))) return poison(c, rc);
      if (hipEventRecord(c->ev_a, st) != hipSuccess || hipStreamWaitEvent(c->xs, c->ev_a, 0) != hipSuccess)
        return poison(c, m3d_fail(ctx, M3D_ERR_HIP, "exchange stream hand-off"));
      if ((rc = allreduce(c, s->xdk, h, ncclInt64, ncclMin, c->xs))) return rc;
      if (hipEventRecord(c->ev_x, c->xs) != hipSuccess)
        return poison(c, m3d_fail(ctx, M3D_ERR_HIP, "exchange stream hand-off"));
      if ((rc = icp_shard_nn_range(s, off, h, ns, s->xdk, st))) return poison(c, rc);
      // the communicator's collectives run one after another: B's MIN after A's
      if (hipStreamWaitEvent(st, c->ev_x, 0) != hipSuccess)
        return poison(c, m3d_fail(ctx, M3D_ERR_HIP, "exchange stream hand-off"));
      if ((rc = allreduce(c, s->xdk + h, ns - h, ncclInt64, ncclMin, st))) return rc;
    } else {
      if ((rc = m3d_icp_shard_nn(s, off, s->xdk, stream))) return poison(c, rc);
      if ((rc = allreduce(c, s->xdk, ns, ncclInt64, ncclMin, st))) return rc;
    }
    if ((rc = m3d_icp_shard_claim(s, s->xdk, s->xcl, stream))) return poison(c, rc);
    if ((rc = allreduce(c, s->xcl, ns, ncclInt32, ncclMin, st))) return rc;
    if ((rc = m3d_icp_shard_terms(s, off, s->xdk, s->xcl, s->xsums, stream))) return poison(c, rc);
    if ((rc = allreduce(c, s->xsums, kTermSlots, ncclFloat64, ncclSum, st))) return rc;
    if ((rc = m3d_icp_solve(s, s->xsums, stream))) return poison(c, rc);
  }
  return M3D_OK;
}

int m3d_icp_source_shard_steps(m3d_icp* s, m3d_comm* c, int32_t n, void* stream) {
  if (!s || !c) return M3D_ERR_INVALID;
  m3d_ctx* ctx = s->ctx;
  if (c->poisoned) return poisoned_error(c);
  if (n < 0) return m3d_fail(ctx, M3D_ERR_INVALID, "n must be >= 0");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  Touch tch{ctx, st};
  int rc;
  if (!s->xready_src) {
    rc = alloc_once(ctx, &s->xsums, kTermSlots);
    if ((rc = agree(c, rc, st))) return rc;
    s->xready_src = true;
  }
  for (int32_t k = 0; k < n; ++k) {
    if (c->inject == 2) {
      c->inject = 0;
      return poison(c, m3d_fail(ctx, M3D_ERR_HIP, "injected failure (m3d_debug_comm_inject)"));
    }
    if ((rc = m3d_icp_shard_nn(s, 0, nullptr, stream))) return poison(c, rc);
    if ((rc = m3d_icp_shard_terms(s, 0, nullptr, nullptr, s->xsums, stream))) return poison(c, rc);
    if ((rc = allreduce(c, s->xsums, kTermSlots, ncclFloat64, ncclSum, st))) return rc;
    if ((rc = m3d_icp_solve(s, s->xsums, stream))) return poison(c, rc);
  }
  return M3D_OK;
}

int m3d_ransac_best_allreduce(m3d_comm* c, const m3d_ransac_result* result_dev, int64_t hyp0,
                              int64_t* key_dev, void* stream) {
  if (!c) return M3D_ERR_INVALID;
  if (c->poisoned) return poisoned_error(c);
  if (!result_dev || !key_dev) return m3d_fail(c->ctx, M3D_ERR_INVALID, "null device pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (launch_ransac_pack_key(result_dev, hyp0, key_dev, st) != hipSuccess)
    return poison(c, m3d_fail(c->ctx, M3D_ERR_HIP, "key pack"));
  return allreduce(c, key_dev, 1, ncclInt64, ncclMax, st);
}

int m3d_ransac_run_sharded(m3d_ctx* ctx, m3d_comm* c, const m3d_corrset* cs,
                           const m3d_ransac_params* p, m3d_ransac_result* out, void* stream) {
  if (!ctx || !c) return M3D_ERR_INVALID;
  if (c->poisoned) return poisoned_error(c);
  if (!cs || !p || !out) return m3d_fail(ctx, M3D_ERR_INVALID, "invalid arguments");
  if (p->early_stop)
    return m3d_fail(ctx, M3D_ERR_INVALID,
                    "hypothesis-sharded RANSAC runs without early stop (each rank would stop on "
                    "its own id range)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // the local run; on failure this rank still joins both collectives (fail-soft, see the header)
  int local = M3D_OK;
  std::string local_err;
  if (c->inject == 1) {
    c->inject = 0;
    local = m3d_fail(ctx, M3D_ERR_HIP, "injected failure (m3d_debug_comm_inject)");
  } else {
    local = m3d_ransac_run_async(ctx, cs, p, nullptr, nullptr, c->dres, stream);
  }
  if (local != M3D_OK) local_err = m3d_last_error(ctx);
  const m3d_ransac_result* r = local == M3D_OK ? c->dres : nullptr;
  if (launch_ransac_shard_key(r, p->hyp0, c->rbuf, st) != hipSuccess)
    return poison(c, m3d_fail(ctx, M3D_ERR_HIP, "key pack"));
  int rc = allreduce(c, c->rbuf, 1, ncclInt64, ncclMax, st);
  if (rc) return rc;
  if (launch_ransac_shard_pack(r, p->hyp0, c->rbuf, st) != hipSuccess)
    return poison(c, m3d_fail(ctx, M3D_ERR_HIP, "result pack"));
  if ((rc = allreduce(c, c->rbuf + 1, 19, ncclInt64, ncclSum, st))) return rc;
  if (hipMemcpyAsync(c->hbuf, c->rbuf, 20 * sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return poison(c, m3d_fail(ctx, M3D_ERR_HIP, "result copy"));
  const int64_t* h = c->hbuf;
  if (local != M3D_OK) return m3d_fail(ctx, local, local_err);
  if (h[19] != 0)
    return m3d_fail(ctx, M3D_ERR_COMM, std::to_string(h[19]) + " peer rank(s) failed their local run");
  memset(out, 0, sizeof(*out));
  for (int k = 0; k < 16; ++k) out->T[k] = (k % 5 == 0) ? 1.0 : 0.0;
  out->best_index = -1;
  out->iterations = h[1];
  out->rechecked = h[2];
  const int64_t key = h[0];
  if (key > 0) {
    out->best_count = (int64_t)((uint64_t)key >> 32);
    out->best_index = (int64_t)(0xFFFFFFFFull - ((uint64_t)key & 0xFFFFFFFFull));
    out->fitness = cs->nc > 0 ? (double)out->best_count / (double)cs->nc : 0.0;
    memcpy(out->T, h + 3, sizeof(out->T));  // the winner's bits (the other ranks added zeros)
  }
  return M3D_OK;
}

int m3d_debug_comm_inject(m3d_comm* c, int what) {
  if (!c || what < 0 || what > 2) return M3D_ERR_INVALID;
  c->inject = what;
  return M3D_OK;
}

int m3d_comm_poisoned(const m3d_comm* c) { return c ? (c->poisoned ? 1 : 0) : -1; }

}  // extern "C"
