// comm.cpp — RCCL inside libm3d.so (include/m3d.h "RCCL inside the library").
//
// One communicator per (context, rank), one process per GPU.  The multi-GPU loops of the hot
// path enqueue their collectives on the caller's stream between the library's own kernels, so
// an iteration of target-sharded ICP is NN → MIN(d64 keys) → claim → MIN(claims) → terms →
// SUM(32 term slots) → solve with no host round trip (the reference's icp.py:42-48 with the
// correspondence search split over the node's GPUs).  xGMI is point-to-point: the 8·Ns-byte key
// MIN is one ring all-reduce per iteration (8 MB at 1M sources ≈ 0.1 ms per link ring), the
// claim MIN half that, the terms SUM 256 B (latency only).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <string>

#include "m3d_internal.h"

struct m3d_comm {
  m3d_ctx* ctx = nullptr;
  ncclComm_t nccl = nullptr;
  int rank = 0, world = 1;
  int64_t* key = nullptr;  // RANSAC key scratch (1 int64)
};

using namespace m3d;

namespace {
int comm_fail(m3d_ctx* ctx, ncclResult_t r, const char* what) {
  return m3d_fail(ctx, M3D_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}
#define NCCLX(ctx, expr)                                 \
  do {                                                   \
    ncclResult_t r_ = (expr);                            \
    if (r_ != ncclSuccess) return comm_fail(ctx, r_, #expr); \
  } while (0)
#define HIPC(ctx, expr) M3D_HIP_CHECK(ctx, expr)

ncclDataType_t dtype_of(int dt) {
  return dt == M3D_DT_I32 ? ncclInt32 : (dt == M3D_DT_I64 ? ncclInt64 : ncclFloat64);
}
ncclRedOp_t op_of(int op) { return op == M3D_OP_MIN ? ncclMin : (op == M3D_OP_MAX ? ncclMax : ncclSum); }

template <class T>
int alloc_once(m3d_ctx* ctx, T** p, int64_t count) {
  if (*p != nullptr) return M3D_OK;
  if (hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (size_t)std::max<int64_t>(count, 1)) != hipSuccess) {
    *p = nullptr;
    return m3d_fail(ctx, M3D_ERR_OOM, "exchange buffer hipMalloc failed");
  }
  return M3D_OK;
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
    delete c;
    return comm_fail(ctx, r, "ncclCommInitRank");
  }
  if (hipMalloc(&c->key, sizeof(int64_t)) != hipSuccess) {
    m3d_comm_destroy(c);
    return m3d_fail(ctx, M3D_ERR_OOM, "communicator scratch");
  }
  *out = c;
  return M3D_OK;
}

void m3d_comm_destroy(m3d_comm* c) {
  if (!c) return;
  if (c->nccl) ncclCommDestroy(c->nccl);
  hipFree(c->key);
  delete c;
}

int m3d_comm_allreduce(m3d_comm* c, void* buf, int64_t count, int dtype, int op, void* stream) {
  if (!c) return M3D_ERR_INVALID;
  if (count < 0 || (count > 0 && !buf) || dtype < M3D_DT_I32 || dtype > M3D_DT_F64 ||
      op < M3D_OP_SUM || op > M3D_OP_MAX)
    return m3d_fail(c->ctx, M3D_ERR_INVALID, "invalid all-reduce arguments");
  if (count == 0) return M3D_OK;
  NCCLX(c->ctx, ncclAllReduce(buf, buf, (size_t)count, dtype_of(dtype), op_of(op), c->nccl,
                              reinterpret_cast<hipStream_t>(stream)));
  return M3D_OK;
}

int m3d_icp_shard_steps(m3d_icp* s, m3d_comm* c, int64_t off, int32_t n, void* stream) {
  if (!s || !c) return M3D_ERR_INVALID;
  m3d_ctx* ctx = s->ctx;
  if (n < 0) return m3d_fail(ctx, M3D_ERR_INVALID, "n must be >= 0");
  const int64_t ns = s->src->n;
  int rc = alloc_once(ctx, &s->xdk, ns);
  if (!rc) rc = alloc_once(ctx, &s->xcl, ns);
  if (!rc) rc = alloc_once(ctx, &s->xsums, kTermSlots);
  if (rc) return rc;
  for (int32_t k = 0; k < n; ++k) {
    if ((rc = m3d_icp_shard_nn(s, off, s->xdk, stream))) return rc;
    if ((rc = m3d_comm_allreduce(c, s->xdk, ns, M3D_DT_I64, M3D_OP_MIN, stream))) return rc;
    if ((rc = m3d_icp_shard_claim(s, s->xdk, s->xcl, stream))) return rc;
    if ((rc = m3d_comm_allreduce(c, s->xcl, ns, M3D_DT_I32, M3D_OP_MIN, stream))) return rc;
    if ((rc = m3d_icp_shard_terms(s, off, s->xdk, s->xcl, s->xsums, stream))) return rc;
    if ((rc = m3d_comm_allreduce(c, s->xsums, kTermSlots, M3D_DT_F64, M3D_OP_SUM, stream))) return rc;
    if ((rc = m3d_icp_solve(s, s->xsums, stream))) return rc;
  }
  return M3D_OK;
}

int m3d_icp_source_shard_steps(m3d_icp* s, m3d_comm* c, int32_t n, void* stream) {
  if (!s || !c) return M3D_ERR_INVALID;
  m3d_ctx* ctx = s->ctx;
  if (n < 0) return m3d_fail(ctx, M3D_ERR_INVALID, "n must be >= 0");
  int rc = alloc_once(ctx, &s->xsums, kTermSlots);
  if (rc) return rc;
  for (int32_t k = 0; k < n; ++k) {
    if ((rc = m3d_icp_shard_nn(s, 0, nullptr, stream))) return rc;
    if ((rc = m3d_icp_shard_terms(s, 0, nullptr, nullptr, s->xsums, stream))) return rc;
    if ((rc = m3d_comm_allreduce(c, s->xsums, kTermSlots, M3D_DT_F64, M3D_OP_SUM, stream))) return rc;
    if ((rc = m3d_icp_solve(s, s->xsums, stream))) return rc;
  }
  return M3D_OK;
}

int m3d_ransac_best_allreduce(m3d_comm* c, const m3d_ransac_result* result_dev, int64_t hyp0,
                              int64_t* key_dev, void* stream) {
  if (!c) return M3D_ERR_INVALID;
  if (!result_dev || !key_dev) return m3d_fail(c->ctx, M3D_ERR_INVALID, "null device pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIPC(c->ctx, launch_ransac_pack_key(result_dev, hyp0, key_dev, st));
  return m3d_comm_allreduce(c, key_dev, 1, M3D_DT_I64, M3D_OP_MAX, stream);
}

int m3d_ransac_run_sharded(m3d_ctx* ctx, m3d_comm* c, const m3d_corrset* cs,
                           const m3d_ransac_params* p, m3d_ransac_result* out, void* stream) {
  if (!ctx || !c) return M3D_ERR_INVALID;
  if (!cs || !p || !out) return m3d_fail(ctx, M3D_ERR_INVALID, "invalid arguments");
  if (p->early_stop)
    return m3d_fail(ctx, M3D_ERR_INVALID,
                    "hypothesis-sharded RANSAC runs without early stop (each rank would stop on "
                    "its own id range)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  m3d_ransac_result* dres = nullptr;
  double* Tw = nullptr;
  int64_t* cnt = nullptr;
  int rc = M3D_OK;
  if (hipMalloc(&dres, sizeof(*dres)) != hipSuccess || hipMalloc(&Tw, 16 * sizeof(double)) != hipSuccess ||
      hipMalloc(&cnt, 2 * sizeof(int64_t)) != hipSuccess)
    rc = m3d_fail(ctx, M3D_ERR_OOM, "hipMalloc failed");
  m3d_ransac_result loc{};
  int64_t key = 0, sums[2] = {0, 0};
  if (!rc) rc = hipMemsetAsync(dres, 0, sizeof(*dres), st) == hipSuccess ? M3D_OK : M3D_ERR_HIP;
  if (!rc) rc = m3d_ransac_run_async(ctx, cs, p, nullptr, nullptr, dres, stream);
  if (!rc) rc = m3d_ransac_best_allreduce(c, dres, p->hyp0, c->key, stream);
  if (!rc && hipMemcpyAsync(&loc, dres, sizeof(loc), hipMemcpyDeviceToHost, st) != hipSuccess)
    rc = m3d_fail(ctx, M3D_ERR_HIP, "result copy");
  if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = m3d_fail(ctx, M3D_ERR_HIP, "sync");
  if (!rc) {
    sums[0] = loc.iterations;
    sums[1] = loc.rechecked;
    if (hipMemcpyAsync(cnt, sums, sizeof(sums), hipMemcpyHostToDevice, st) != hipSuccess)
      rc = m3d_fail(ctx, M3D_ERR_HIP, "copy");
  }
  if (!rc) rc = m3d_comm_allreduce(c, cnt, 2, M3D_DT_I64, M3D_OP_SUM, stream);
  if (!rc && (hipMemcpyAsync(&key, c->key, sizeof(key), hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipMemcpyAsync(sums, cnt, sizeof(sums), hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipStreamSynchronize(st) != hipSuccess))
    rc = m3d_fail(ctx, M3D_ERR_HIP, "key copy");
  if (!rc) {
    memset(out, 0, sizeof(*out));
    for (int k = 0; k < 16; ++k) out->T[k] = (k % 5 == 0) ? 1.0 : 0.0;
    out->best_index = -1;
    out->iterations = sums[0];
    out->rechecked = sums[1];
    if (key > 0) {
      const int64_t count = (int64_t)((uint64_t)key >> 32);
      const int64_t wid = (int64_t)(0xFFFFFFFFull - ((uint64_t)key & 0xFFFFFFFFull));
      out->best_count = count;
      out->best_index = wid;
      out->fitness = cs->nc > 0 ? (double)count / (double)cs->nc : 0.0;
      rc = m3d_kabsch3_batch(ctx, cs, nullptr, p->seed, wid, 1, Tw, nullptr, stream);
      if (!rc && (hipMemcpyAsync(out->T, Tw, sizeof(out->T), hipMemcpyDeviceToHost, st) != hipSuccess ||
                  hipStreamSynchronize(st) != hipSuccess))
        rc = m3d_fail(ctx, M3D_ERR_HIP, "transform copy");
    }
  }
  hipFree(dres);
  hipFree(Tw);
  hipFree(cnt);
  return rc;
}

}  // extern "C"
