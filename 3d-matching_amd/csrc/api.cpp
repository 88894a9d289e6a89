// api.cpp — the C ABI of libm3d.so (include/m3d.h): contexts, packed objects, batching and
// the host-side drivers of the device loops.  No numerical work happens here except the
// MT19937 replay of the reference RNG (m3d_replay_triples) and O(1) bookkeeping.
#include <cfloat>
#include <chrono>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "linalg.h"
#include "m3d_internal.h"
#include "ddmath.h"

namespace m3d {
hipError_t launch_icp_reset(const m3d_icp* s, const double* T, bool apply_init, hipStream_t st);
hipError_t launch_copy_points(const m3d_icp* s, double* dst, hipStream_t st);
hipError_t launch_icp_terms_solve(const m3d_icp* s, bool reset_keys, hipStream_t st);
hipError_t launch_nn_finalize(const m3d_icp* s, int32_t* idx, double* d2, hipStream_t st);
int64_t terms_blocks(int64_t ns);
}  // namespace m3d

using namespace m3d;

int m3d_fail(m3d_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

KTimer::KTimer(m3d_ctx* c, int kid, hipStream_t s) : ctx(c), id(kid), st(s) {
  if (!ctx || !ctx->profiling) return;
  auto& v = ctx->ev[id];
  size_t k = ctx->ev_used[id];
  if (k >= 65536) return;  // cap; read regularly
  if (k == v.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return;
    if (hipEventCreate(&b) != hipSuccess) {
      hipEventDestroy(a);
      return;
    }
    v.emplace_back(a, b);
  }
  if (hipEventRecord(v[k].first, st) != hipSuccess) return;
  end = v[k].second;
  ctx->ev_used[id] = k + 1;
}

KTimer::~KTimer() {
  if (end) hipEventRecord(end, st);
}

#define CHECK_ARG(ctx, cond, msg) \
  do {                            \
    if (!(cond)) return m3d_fail((ctx), M3D_ERR_INVALID, (msg)); \
  } while (0)

#define HIPX(ctx, expr) M3D_HIP_CHECK(ctx, expr)

static hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }


namespace m3d {
// ------------------------------------------------------------------------------- block cache
// Released device blocks (clouds, grids, Morton copies, target records, MFMA tiles) wait in a
// process-wide cache for an allocation of a size in [need, 2·need].  Each carries the RELEASE
// MARK of the object that freed it: an event recorded, on its context's order stream, after
// every stream the context had enqueued work on (ctx_touch) up to the release — so a reuse only
// makes the ALLOCATING stream wait on the device (hipStreamWaitEvent) for the work that could
// still read the block, never the host, and never work on streams the context never used.
// Blocks freed outside a release scope (a rebuild inside a call) have no mark and are reused
// after a hipDeviceSynchronize, as before round 5.  Bounded (M3D_BLOCK_CACHE MiB, default
// 2048; 64 blocks; oldest freed first); trimmed when the last context of a device is destroyed,
// by m3d_trim_block_cache, and before any device allocation of the library is retried after
// an out-of-memory failure (dev_malloc_raw).
namespace {
struct CachedBlock {
  void* p;
  size_t bytes;
  int dev;
  std::shared_ptr<ReleaseMark> mark;  // null: unknown users, device sync before reuse
};
// The cache's state lives in one heap object that is never destroyed: objects (and their
// marks) may still be released while static destructors run at process exit.
struct CacheState {
  std::mutex mu;
  std::vector<CachedBlock> blocks;  // released, oldest first
  std::unordered_map<void*, std::pair<size_t, int>> live;  // from block_alloc: size, device
  std::mutex ev_mu;  // guards ev_retired; taken after mu (a mark may die under mu)
  std::vector<hipEvent_t> ev_retired;  // marks' events, destroyed once complete
  std::unordered_map<int, int> ctx_per_dev;  // live contexts per device
  std::unordered_map<const m3d_ctx*, uint64_t> ctx_ids;  // live contexts and their ids
  uint64_t next_id = 1;
  size_t bytes = 0;
};
CacheState& cache_state() {
  static CacheState* p = new CacheState();
  return *p;
}
std::mutex& g_bc_mu = cache_state().mu;
std::vector<CachedBlock>& g_bc = cache_state().blocks;
std::unordered_map<void*, std::pair<size_t, int>>& g_bc_live = cache_state().live;
std::mutex& g_ev_mu = cache_state().ev_mu;
std::vector<hipEvent_t>& g_ev_retired = cache_state().ev_retired;
std::unordered_map<int, int>& g_ctx_live = cache_state().ctx_per_dev;
size_t& g_bc_bytes = cache_state().bytes;
constexpr size_t kBcMaxCount = 64;
thread_local std::shared_ptr<ReleaseMark> t_mark;  // the active ReleaseScope's mark

size_t bc_cap() {
  static const size_t cap = [] {
    const char* e = getenv("M3D_BLOCK_CACHE");
    const long long mib = e ? atoll(e) : 2048;
    return mib > 0 ? (size_t)mib << 20 : (size_t)0;
  }();
  return cap;
}
bool bc_on() { return bc_cap() > 0; }

void retire_events(bool wait) {
  std::lock_guard<std::mutex> lk(g_ev_mu);
  for (size_t k = 0; k < g_ev_retired.size();) {
    hipEvent_t ev = g_ev_retired[k];
    if (wait) (void)hipEventSynchronize(ev);
    if (hipEventQuery(ev) == hipSuccess) {
      (void)hipEventDestroy(ev);
      g_ev_retired[k] = g_ev_retired.back();
      g_ev_retired.pop_back();
    } else {
      ++k;
    }
  }
  (void)hipGetLastError();
}

// free cached blocks (of device dev, or every device when dev < 0) until the cache holds at most
// max_bytes / max_count; a block is freed only after its release point has passed on the device
size_t bc_trim_locked(int dev, size_t max_bytes, size_t max_count) {
  size_t freed = 0;
  for (size_t k = 0; k < g_bc.size() && (g_bc_bytes > max_bytes || g_bc.size() > max_count);) {
    CachedBlock& b = g_bc[k];
    if (dev >= 0 && b.dev != dev) {
      ++k;
      continue;
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != b.dev) (void)hipSetDevice(b.dev);
    if (b.mark && b.mark->ev) (void)hipEventSynchronize(b.mark->ev);
    (void)hipFree(b.p);  // (hipFree itself waits for the device)
    if (cur != b.dev) (void)hipSetDevice(cur);
    g_bc_bytes -= b.bytes;
    freed += b.bytes;
    g_bc.erase(g_bc.begin() + (ptrdiff_t)k);
  }
  retire_events(false);
  return freed;
}
}  // namespace

ReleaseMark::~ReleaseMark() {
  if (ev == nullptr) return;
  std::lock_guard<std::mutex> lk(g_ev_mu);
  g_ev_retired.push_back(ev);
}

size_t block_cache_trim(int dev) {
  std::lock_guard<std::mutex> lk(g_bc_mu);
  return bc_trim_locked(dev, 0, 0);
}

hipError_t dev_malloc_raw(void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
    (void)hipGetLastError();
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (block_cache_trim(dev) > 0) e = hipMalloc(p, bytes);
  }
  if (e != hipSuccess) *p = nullptr;
  return e;
}

hipError_t block_alloc(void** out, size_t bytes, hipStream_t st) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (bc_on()) {
    std::unique_lock<std::mutex> lk(g_bc_mu);
    int best = -1;
    for (int k = 0; k < (int)g_bc.size(); ++k) {
      const CachedBlock& b = g_bc[(size_t)k];
      if (b.dev == dev && b.bytes >= bytes && b.bytes <= 2 * bytes && (best < 0 || b.bytes < g_bc[(size_t)best].bytes))
        best = k;
    }
    if (best >= 0) {
      const CachedBlock b = g_bc[(size_t)best];
      g_bc.erase(g_bc.begin() + best);
      g_bc_bytes -= b.bytes;
      g_bc_live[b.p] = {b.bytes, dev};
      lk.unlock();
      hipError_t e = hipSuccess;
      if (!b.mark)
        e = hipDeviceSynchronize();  // released outside a scope: unknown users
      else if (b.mark->ev != nullptr)
        e = hipStreamWaitEvent(st, b.mark->ev, 0);  // stream order: the allocating stream waits
      if (e != hipSuccess) {
        block_release(b.p);
        return e;
      }
      *out = b.p;
      return hipSuccess;
    }
  }
  void* p = nullptr;
  const hipError_t e = dev_malloc_raw(&p, bytes);
  if (e != hipSuccess) return e;
  if (bc_on()) {
    std::lock_guard<std::mutex> lk(g_bc_mu);
    g_bc_live[p] = {bytes, dev};
  }
  *out = p;
  return hipSuccess;
}

void block_release(void* p) {
  if (p == nullptr) return;
  if (bc_on()) {
    std::lock_guard<std::mutex> lk(g_bc_mu);
    auto it = g_bc_live.find(p);
    if (it != g_bc_live.end()) {
      g_bc.push_back(CachedBlock{p, it->second.first, it->second.second, t_mark});
      g_bc_bytes += it->second.first;
      g_bc_live.erase(it);
      bc_trim_locked(-1, bc_cap(), kBcMaxCount);
      return;
    }
  }
  (void)hipFree(p);
}

void ctx_touch(m3d_ctx* ctx, hipStream_t st) {
  if (ctx == nullptr) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();  // a capture: its graph launch is touched when it is replayed
    return;
  }
  std::lock_guard<std::mutex> lk(ctx->uses_mu);
  hipEvent_t ev = nullptr;
  for (auto& u : ctx->uses)
    if (u.first == st) ev = u.second;
  if (ev == nullptr) {
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      ctx->uses_lost = true;  // no event: releases fall back to a device sync before reuse
      return;
    }
    ctx->uses.emplace_back(st, ev);
  }
  if (hipEventRecord(ev, st) != hipSuccess) ctx->uses_lost = true;
}

ReleaseScope::ReleaseScope(m3d_ctx* ctx, uint64_t ctx_id) {
  prev = t_mark;
  std::shared_ptr<ReleaseMark> m;
  if (ctx != nullptr) {  // a destroyed context (e.g. Python teardown order): no mark, device sync
    std::lock_guard<std::mutex> lk(g_bc_mu);
    auto it = cache_state().ctx_ids.find(ctx);
    if (it == cache_state().ctx_ids.end() || it->second != ctx_id) ctx = nullptr;
  }
  if (ctx != nullptr) {
    std::lock_guard<std::mutex> lk(ctx->uses_mu);  // destroys may run on finaliser threads
    // streams whose last touched work has completed need no wait: drop them (a destroyed
    // stream's entry goes this way too), so the list stays as long as the streams still busy
    for (size_t k = 0; k < ctx->uses.size();) {
      if (hipEventQuery(ctx->uses[k].second) == hipSuccess) {
        (void)hipEventDestroy(ctx->uses[k].second);
        ctx->uses[k] = ctx->uses.back();
        ctx->uses.pop_back();
      } else {
        ++k;
      }
    }
    (void)hipGetLastError();
    if (!ctx->uses_lost) {
      m = std::make_shared<ReleaseMark>();
      if (!ctx->uses.empty()) {
        int cur = 0;
        (void)hipGetDevice(&cur);  // the caller's (e.g. torch's) current device is left as it was
        if (cur != ctx->device) (void)hipSetDevice(ctx->device);
        bool ok = ctx->order != nullptr || hipStreamCreateWithFlags(&ctx->order, hipStreamNonBlocking) == hipSuccess;
        hipEvent_t ev = nullptr;
        ok = ok && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
        for (auto& u : ctx->uses) ok = ok && hipStreamWaitEvent(ctx->order, u.second, 0) == hipSuccess;
        ok = ok && hipEventRecord(ev, ctx->order) == hipSuccess;
        if (ok) {
          m->ev = ev;
        } else {
          if (ev != nullptr) (void)hipEventDestroy(ev);
          m.reset();
          (void)hipGetLastError();
        }
        if (cur != ctx->device) (void)hipSetDevice(cur);
      }
    }
  }
  t_mark = m;
}

ReleaseScope::~ReleaseScope() { t_mark = prev; }

void ctx_register(m3d_ctx* ctx, bool live) {
  std::lock_guard<std::mutex> lk(g_bc_mu);
  if (live) {
    ctx->id = cache_state().next_id++;
    cache_state().ctx_ids[ctx] = ctx->id;
  } else {
    cache_state().ctx_ids.erase(ctx);
  }
}

void ctx_count(int dev, int delta) {
  std::lock_guard<std::mutex> lk(g_bc_mu);
  const int n = (g_ctx_live[dev] += delta);
  if (n <= 0) {
    g_ctx_live.erase(dev);
    bc_trim_locked(dev, 0, 0);  // the last context of the device: give the cache back
  }
}
}  // namespace m3d

namespace {

constexpr int64_t kCorrPad = 2048;  // score kernel block footprint (ransac.hip kBlockCorr)
constexpr int64_t kCloudPad = 1024; // NN tile multiple
constexpr float kFar = 1.0e18f;

template <class T>
int dev_alloc(m3d_ctx* ctx, T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) return M3D_OK;
  hipError_t e = dev_malloc(reinterpret_cast<void**>(p), sizeof(T) * (size_t)count);
  if (e != hipSuccess) {
    *p = nullptr;
    return m3d_fail(ctx, M3D_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  return M3D_OK;
}

// Bump allocator over the context scratch arena.  Growing synchronises the device.
// The scratch arena and the RANSAC loop state (ctx->rstate) are shared by every call on the
// context, and each call only enqueues work on its caller's stream: a call on a different stream
// than the previous scratch user first waits (device-side) for that user's work, and records its
// own completion event when it is done enqueueing — calls on several streams are serialised on
// the device, never racing on the scratch.
struct Arena {
  m3d_ctx* ctx;
  hipStream_t st;
  size_t off = 0;
  Arena(m3d_ctx* c, hipStream_t s) : ctx(c), st(s) {
    if (ctx->scratch_ev != nullptr && ctx->scratch_used && ctx->scratch_stream != st)
      (void)hipStreamWaitEvent(st, ctx->scratch_ev, 0);
  }
  ~Arena() {
    if (ctx->scratch_ev != nullptr && hipEventRecord(ctx->scratch_ev, st) == hipSuccess) {
      ctx->scratch_used = true;
      ctx->scratch_stream = st;
    }
  }
  size_t take(size_t bytes) {
    size_t o = (off + 255) & ~size_t(255);
    off = o + bytes;
    return o;
  }
  int commit() {
    if (off <= ctx->scratch_bytes) return M3D_OK;
    if (ctx->scratch) {
      hipDeviceSynchronize();
      hipFree(ctx->scratch);
      ctx->scratch = nullptr;
      ctx->scratch_bytes = 0;
    }
    size_t want = std::max(off, ctx->scratch_bytes * 3 / 2);
    hipError_t e = dev_malloc(&ctx->scratch, want);
    if (e != hipSuccess) {
      ctx->scratch = nullptr;
      return m3d_fail(ctx, M3D_ERR_OOM, "scratch hipMalloc failed");
    }
    ctx->scratch_bytes = want;
    return M3D_OK;
  }
  template <class T>
  T* at(size_t o) const {
    return reinterpret_cast<T*>(static_cast<char*>(ctx->scratch) + o);
  }
};

// deterministic mean of an n×3 device array (block partials summed in fixed order on host)
int device_mean3(m3d_ctx* ctx, const double* a, int64_t n, double out[3], hipStream_t st) {
  out[0] = out[1] = out[2] = 0.0;
  if (n == 0) return M3D_OK;
  const int blocks = 128;
  double* part = nullptr;
  int rc = dev_alloc(ctx, &part, blocks * 3);
  if (rc) return rc;
  hipError_t e = launch_sum3(a, n, part, blocks, st);
  std::vector<double> h(blocks * 3);
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), part, sizeof(double) * blocks * 3,
                                          hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  hipFree(part);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  for (int b = 0; b < blocks; ++b)
    for (int k = 0; k < 3; ++k) out[k] += h[3 * b + k];
  for (int k = 0; k < 3; ++k) out[k] /= (double)n;
  return M3D_OK;
}

// A cloud's centre (mean, unless given), centred fp32 copy, rmax and grid bounds with ONE host
// sync (ransac.hip cloud_pack_kernel); the same values as device_mean3 + center_pack + the grid
// build's bounds pass, which took three syncs.  Temporaries from the context's arena.
// mapped pinned memory of the context (pin_ensure): kernels write their few results into it and
// the host reads them after one stream sync — no device-to-host copy (a pageable copy is a staging
// blit plus its own wait: ≈ 20 µs per readback on the cold path)
int pin_ensure(m3d_ctx* ctx);
constexpr size_t kPinRead = 2048;  // the cold path's readbacks: cloud summary, grid occupancy
template <class T>
T* pin_read(const m3d_ctx* ctx, bool dev) {
  return reinterpret_cast<T*>(static_cast<char*>(dev ? ctx->pin_dev : ctx->pin) + kPinRead);
}

int cloud_pack(m3d_ctx* ctx, m3d_cloud* c, int64_t n, bool mean, hipStream_t st) {
  c->rmax = 0.0;
  c->has_bounds = false;
  if (c->n_pad == 0) return M3D_OK;
  int rc = pin_ensure(ctx);
  if (rc) return rc;
  const int sblocks = 128;
  const int blocks = (int)std::min<int64_t>(1024, (c->n_pad + 255) / 256);
  // scratch [block sums | centre | block (rmax, lo, hi)]; the summary goes to pinned memory
  const size_t o_sum = 0, o_c = tmp_align(sizeof(double) * 3 * sblocks), o_p7 = o_c + tmp_align(3 * sizeof(double));
  const size_t bytes = o_p7 + tmp_align(sizeof(float) * 7 * blocks);
  hipError_t e = ctx->tmp.reserve(bytes);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_OOM, "cloud scratch");
  char* b = ctx->tmp.base;
  double* cdev = reinterpret_cast<double*>(b + o_c);
  double* sum_part = reinterpret_cast<double*>(b + o_sum);
  float* p7 = reinterpret_cast<float*>(b + o_p7);
  const bool dmean = mean && n > 0;
  double* pin_c = pin_read<double>(ctx, true);
  float* pin7 = reinterpret_cast<float*>(pin_c + 3);
  if (dmean) e = launch_sum3(c->xyz64, n, sum_part, sblocks, st);
  if (e == hipSuccess)
    e = launch_cloud_pack(c->xyz64, n, c->n_pad, dmean ? sum_part : nullptr, sblocks, cdev, c->center, c->xyz32,
                          kFar, p7, blocks, pin_c, pin7, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  const volatile double* hc = pin_read<double>(ctx, false);
  const volatile float* h = reinterpret_cast<const volatile float*>(hc + 3);
  if (dmean)
    for (int k = 0; k < 3; ++k) c->center[k] = hc[k];
  for (int k = 0; k < 3; ++k) {
    c->lo[k] = h[1 + k];
    c->hi[k] = h[4 + k];
  }
  c->rmax = (double)h[0] * (1.0 + 1e-6);
  c->has_bounds = n > 0;
  return M3D_OK;
}

int center_pack(m3d_ctx* ctx, const double* a, int64_t n, int64_t n_pad, const double c[3],
                float4* out, float pad, double* maxv, hipStream_t st) {
  *maxv = 0.0;
  if (n_pad == 0) return M3D_OK;
  const int blocks = (int)std::min<int64_t>(1024, (n_pad + 255) / 256);
  float* part = nullptr;
  int rc = dev_alloc(ctx, &part, blocks);
  if (rc) return rc;
  hipError_t e = launch_center_pack(a, n, n_pad, c, out, pad, part, blocks, 1, st);
  std::vector<float> h(blocks);
  if (e == hipSuccess)
    e = hipMemcpyAsync(h.data(), part, sizeof(float) * blocks, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  hipFree(part);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  float m = 0.0f;
  for (float v : h) m = std::max(m, v);
  *maxv = (double)m * (1.0 + 1e-6);
  return M3D_OK;
}

int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// Host arrays → device: pageable hipMemcpyAsync straight into the cloud's buffers (the runtime
// stages them itself).  Measured against pinned staging through the host pool and against
// hipHostRegister of the caller's arrays (round 3): both were slower at cfg1 sizes.
int upload_host(m3d_ctx* ctx, int narr, void* const* dst, const void* const* src, const size_t* bytes,
                hipStream_t st) {
  for (int i = 0; i < narr; ++i)
    if (bytes[i] > 0) HIPX(ctx, hipMemcpyAsync(dst[i], src[i], bytes[i], hipMemcpyHostToDevice, st));
  return M3D_OK;
}

}  // namespace

extern "C" {

int m3d_abi_version(void) { return M3D_ABI_VERSION; }

int m3d_device_count(int* count) {
  if (!count) return M3D_ERR_INVALID;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return M3D_OK;
}

int m3d_create(int device, m3d_ctx** out) {
  if (!out) return M3D_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return M3D_ERR_NODEVICE;
  if (device < 0 || device >= n) return M3D_ERR_INVALID;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return M3D_ERR_HIP;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return M3D_ERR_NODEVICE;
  if (hipSetDevice(device) != hipSuccess) return M3D_ERR_HIP;
  m3d_ctx* ctx = new m3d_ctx();
  ctx->device = device;
  if (dev_malloc(&ctx->stats, 8 * sizeof(int64_t)) != hipSuccess ||
      dev_malloc(&ctx->rstate, sizeof(RansacState)) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->scratch_ev, hipEventDisableTiming) != hipSuccess ||
      hipMemset(ctx->stats, 0, 8 * sizeof(int64_t)) != hipSuccess) {
    m3d_destroy(ctx);
    return M3D_ERR_OOM;
  }
  ctx_register(ctx, true);
  ctx_count(device, +1);
  ctx->counted = true;
  *out = ctx;
  return M3D_OK;
}

void m3d_destroy(m3d_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipDeviceSynchronize();
  for (auto& u : ctx->uses) hipEventDestroy(u.second);
  if (ctx->order) hipStreamDestroy(ctx->order);
  if (ctx->scratch) hipFree(ctx->scratch);
  if (ctx->stats) hipFree(ctx->stats);
  if (ctx->rstate) hipFree(ctx->rstate);
  if (ctx->scratch_ev) hipEventDestroy(ctx->scratch_ev);
  if (ctx->pin) hipHostFree(ctx->pin);
  if (ctx->one_ticket) hipFree(ctx->one_ticket);
  if (ctx->prep) hipFree(ctx->prep);
  ctx->tmp.release();
  ctx->run.release();
  for (auto& v : ctx->ev)
    for (auto& pr : v) {
      hipEventDestroy(pr.first);
      hipEventDestroy(pr.second);
    }
  const int dev = ctx->device;
  const bool counted = ctx->counted;
  if (counted) ctx_register(ctx, false);
  delete ctx;
  if (counted) ctx_count(dev, -1);  // the device's last context gives the block cache back
}

int m3d_trim_block_cache(m3d_ctx* ctx, int64_t* freed_bytes) {
  if (!ctx) return M3D_ERR_INVALID;
  const size_t f = block_cache_trim(ctx->device);
  if (freed_bytes) *freed_bytes = (int64_t)f;
  return M3D_OK;
}

const char* m3d_last_error(const m3d_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int m3d_get_stats(m3d_ctx* ctx, int64_t* out8) {
  CHECK_ARG(ctx, out8 != nullptr, "null output");
  HIPX(ctx, hipMemcpy(out8, ctx->stats, 8 * sizeof(int64_t), hipMemcpyDeviceToHost));
  return M3D_OK;
}

int m3d_profile_enable(m3d_ctx* ctx, int enable) {
  if (!ctx) return M3D_ERR_INVALID;
  ctx->profiling = enable != 0;
  return M3D_OK;
}

int m3d_profile_read(m3d_ctx* ctx, int kernel, double* total_ms, int64_t* launches) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, kernel >= 0 && kernel < 6 && total_ms && launches, "invalid arguments");
  double tot = 0.0;
  const size_t n = ctx->ev_used[kernel];
  for (size_t k = 0; k < n; ++k) {
    auto& pr = ctx->ev[kernel][k];
    HIPX(ctx, hipEventSynchronize(pr.second));
    float ms = 0.0f;
    HIPX(ctx, hipEventElapsedTime(&ms, pr.first, pr.second));
    tot += ms;
  }
  ctx->ev_used[kernel] = 0;
  *total_ms = tot;
  *launches = (int64_t)n;
  return M3D_OK;
}

// ------------------------------------------------------------------------------- corrset
static int corrset_build(m3d_ctx* ctx, const double* src, int64_t ns, const double* tgt, int64_t nt,
                         const int32_t* corr, const double* p_src, const double* p_tgt, int64_t nc,
                         void* stream, m3d_corrset** out) {
  CHECK_ARG(ctx, out != nullptr, "null output");
  CHECK_ARG(ctx, nc >= 0 && nc < (int64_t)1 << 31, "correspondence count out of range");
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  std::vector<int32_t> fixed;
  const int32_t* corr_dev = corr;
  int32_t* corr_tmp = nullptr;
  if (corr != nullptr && nc > 0) {
    // validate rows like numpy fancy indexing: negative indices wrap once, others raise
    fixed.resize(2 * nc);
    HIPX(ctx, hipMemcpyAsync(fixed.data(), corr, sizeof(int32_t) * 2 * nc, hipMemcpyDeviceToHost, st));
    HIPX(ctx, hipStreamSynchronize(st));
    bool changed = false;
    for (int64_t i = 0; i < nc; ++i) {
      for (int c = 0; c < 2; ++c) {
        int64_t lim = c == 0 ? ns : nt;
        int64_t v = fixed[2 * i + c];
        if (v < 0) {
          v += lim;
          changed = true;
        }
        if (v < 0 || v >= lim)
          return m3d_fail(ctx, M3D_ERR_INVALID, "correspondence index " +
                                                    std::to_string(fixed[2 * i + c]) +
                                                    " out of bounds for axis 0 with size " +
                                                    std::to_string(lim));
        fixed[2 * i + c] = (int32_t)v;
      }
    }
    if (changed) {
      int rc = dev_alloc(ctx, &corr_tmp, 2 * nc);
      if (rc) return rc;
      HIPX(ctx, hipMemcpyAsync(corr_tmp, fixed.data(), sizeof(int32_t) * 2 * nc,
                               hipMemcpyHostToDevice, st));
      corr_dev = corr_tmp;
    }
  }
  m3d_corrset* cs = new m3d_corrset();
  cs->ctx = ctx;
  cs->nc = nc;
  cs->nc_pad = nc > 0 ? round_up(nc, kCorrPad) : 0;
  int rc = dev_alloc(ctx, &cs->p64, 3 * nc);
  if (!rc) rc = dev_alloc(ctx, &cs->q64, 3 * nc);
  if (!rc) rc = dev_alloc(ctx, &cs->p32, cs->nc_pad);
  if (!rc) rc = dev_alloc(ctx, &cs->q32, cs->nc_pad);
  if (rc) {
    if (corr_tmp) hipFree(corr_tmp);
    m3d_corrset_destroy(cs);
    return rc;
  }
  hipError_t e = launch_pack_corr(src, tgt, corr_dev, nc, p_src, p_tgt, cs->p64, cs->q64, st);
  if (e != hipSuccess) {
    if (corr_tmp) hipFree(corr_tmp);
    m3d_corrset_destroy(cs);
    return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  }
  rc = device_mean3(ctx, cs->p64, nc, cs->cs, st);
  if (!rc) rc = device_mean3(ctx, cs->q64, nc, cs->ct, st);
  // pad: source 0, target far away → padded pairs are never inliers nor ambiguous
  if (!rc) rc = center_pack(ctx, cs->p64, nc, cs->nc_pad, cs->cs, cs->p32, 0.0f, &cs->pmax2, st);
  if (!rc) rc = center_pack(ctx, cs->q64, nc, cs->nc_pad, cs->ct, cs->q32, kFar, &cs->qmaxinf, st);
  if (!rc) {
    hipError_t e2 = launch_corr16(cs, st);  // MFMA scoring operands (ransac.hip)
    if (e2 != hipSuccess) rc = m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e2));
  }
  if (corr_tmp) {
    hipStreamSynchronize(st);
    hipFree(corr_tmp);
  }
  if (rc) {
    m3d_corrset_destroy(cs);
    return rc;
  }
  *out = cs;
  return M3D_OK;
}

int m3d_corrset_create(m3d_ctx* ctx, const double* src_xyz, int64_t ns, const double* tgt_xyz,
                       int64_t nt, const int32_t* corr, int64_t nc, void* stream,
                       m3d_corrset** out) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, nc == 0 || (src_xyz && tgt_xyz && corr), "null device pointer");
  CHECK_ARG(ctx, ns >= 0 && nt >= 0, "negative size");
  return corrset_build(ctx, src_xyz, ns, tgt_xyz, nt, corr, nullptr, nullptr, nc, stream, out);
}

int m3d_corrset_create_gathered(m3d_ctx* ctx, const double* p_src, const double* p_tgt,
                                int64_t nc, void* stream, m3d_corrset** out) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, nc == 0 || (p_src && p_tgt), "null device pointer");
  return corrset_build(ctx, nullptr, 0, nullptr, 0, nullptr, p_src, p_tgt, nc, stream, out);
}

void m3d_corrset_destroy(m3d_corrset* cs) {
  if (!cs) return;
  hipFree(cs->p64);
  hipFree(cs->q64);
  hipFree(cs->p32);
  hipFree(cs->q32);
  hipFree(cs->ca16);
  delete cs;
}

int64_t m3d_corrset_size(const m3d_corrset* cs) { return cs ? cs->nc : -1; }

// ------------------------------------------------------------------------------- a1
int m3d_kabsch3_batch(m3d_ctx* ctx, const m3d_corrset* cs, const int32_t* triples, uint64_t seed,
                      int64_t hyp0, int64_t H, double* T_out, uint8_t* status, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, cs != nullptr && H >= 0 && (H == 0 || T_out), "invalid arguments");
  CHECK_ARG(ctx, triples != nullptr || cs->nc >= 3 || cs->nc < 3, "");
  hipSetDevice(ctx->device);
  Arena a(ctx, S(stream));
  size_t o_h = a.take(sizeof(HypF32) * (size_t)std::max<int64_t>(H, 1));
  int rc = a.commit();
  if (rc) return rc;
  hipError_t e = launch_kabsch3(cs, triples, seed, hyp0, H, 0.0, T_out, status,
                                a.at<HypF32>(o_h), nullptr, ZeroArgs{}, S(stream));
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  return M3D_OK;
}

// ------------------------------------------------------------------------------- a2/a3
namespace {
extern "C++" {
struct ScoreScratch {
  HypF32* hypf;
  ScoreMf mf;
};

constexpr int kScoreSlots = 3;
void score_layout(Arena& a, int64_t H, size_t* o) {
  const int64_t hp = score_mf_hpad(std::max<int64_t>(H, 1));
  o[0] = a.take(sizeof(HypF32) * std::max<int64_t>(H, 1));
  o[1] = a.take(sizeof(uint4) * 6 * hp);
  o[2] = a.take(sizeof(float) * hp);
}

ScoreScratch score_bind(const Arena& a, const size_t* o) {
  ScoreScratch s;
  s.hypf = a.at<HypF32>(o[0]);
  s.mf.hb16 = a.at<uint4>(o[1]);
  s.mf.heps = a.at<float>(o[2]);
  return s;
}
}  // extern "C++"

double thr_sq_of(double thr, int mode) { return mode == M3D_SCORE_SQUARED ? thr : thr * thr; }

// score H transforms T (device) whose fp32 blocks are already in s.hypf and whose counts were
// zeroed by the kernel that produced them
hipError_t score_enqueue(m3d_ctx* ctx, const m3d_corrset* cs, const double* T, int64_t H,
                         double thr, int mode, int32_t* counts, const ScoreScratch& s,
                         const int32_t* done, hipStream_t st, bool prepared = false) {
  // prepared: kabsch3 already wrote the MFMA operands (ScoreFuse)
  hipError_t e = prepared ? hipSuccess : launch_score_prep(cs, T, H, thr, mode, s.mf, st);
  if (e != hipSuccess) return e;
  KTimer kt(ctx, M3D_KERNEL_SCORE, st);
  return launch_score(cs, s.hypf, H, counts, T, thr, mode, ctx->stats, done, s.mf, st);
}
}  // namespace

int m3d_ransac_score(m3d_ctx* ctx, const m3d_corrset* cs, const double* T, int64_t H, double thr,
                     int mode, int32_t* counts, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, cs != nullptr && H >= 0, "invalid arguments");
  CHECK_ARG(ctx, H == 0 || (T && counts), "null device pointer");
  CHECK_ARG(ctx, mode == M3D_SCORE_SQUARED || mode == M3D_SCORE_NORM, "unknown score mode");
  if (H == 0) return M3D_OK;
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  if (cs->nc == 0) {  // ransac.py:220-221 — ratio 0.0
    HIPX(ctx, hipMemsetAsync(counts, 0, sizeof(int32_t) * H, st));
    return M3D_OK;
  }
  Arena a(ctx, S(stream));
  size_t o[kScoreSlots];
  score_layout(a, H, o);
  int rc = a.commit();
  if (rc) return rc;
  ScoreScratch s = score_bind(a, o);
  hipError_t e = launch_hypf_from_T(cs, T, H, thr_sq_of(thr, mode), s.hypf, ZeroArgs{counts}, st);
  if (e == hipSuccess) e = score_enqueue(ctx, cs, T, H, thr, mode, counts, s, nullptr, st);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  return M3D_OK;
}

// ------------------------------------------------------------------------------- one hypothesis
namespace {
constexpr size_t kPinT = 0, kPinStatus = 128, kPinCount = 136, kPinBytes = 4096;
int pin_ensure(m3d_ctx* ctx) {
  if (ctx->pin != nullptr) return M3D_OK;
  void* h = nullptr;
  if (hipHostMalloc(&h, kPinBytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return m3d_fail(ctx, M3D_ERR_OOM, "pinned staging hipHostMalloc failed");
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    hipHostFree(h);
    return m3d_fail(ctx, M3D_ERR_HIP, "hipHostGetDevicePointer failed");
  }
  uint32_t* tk = nullptr;
  if (dev_malloc(&tk, sizeof(uint32_t)) != hipSuccess || hipMemset(tk, 0, sizeof(uint32_t)) != hipSuccess) {
    if (tk) hipFree(tk);
    hipHostFree(h);
    return m3d_fail(ctx, M3D_ERR_OOM, "ticket hipMalloc failed");
  }
  ctx->pin = h;
  ctx->pin_dev = d;
  ctx->one_ticket = tk;
  return M3D_OK;
}
extern "C++" {
template <class T>
T* pin_at(const m3d_ctx* ctx, size_t o, bool dev) {
  return reinterpret_cast<T*>(static_cast<char*>(dev ? ctx->pin_dev : ctx->pin) + o);
}
}  // extern "C++"
}  // namespace

int m3d_kabsch3_one(m3d_ctx* ctx, const m3d_corrset* cs, const int32_t* triple, double* T_out,
                    int32_t* status, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, cs != nullptr && triple != nullptr && T_out != nullptr, "invalid arguments");
  hipSetDevice(ctx->device);
  int rc = pin_ensure(ctx);
  if (rc) return rc;
  hipStream_t st = S(stream);
  // the library's own staging: ordered after earlier scratch users on other streams
  Arena a(ctx, st);
  hipError_t e = launch_kabsch3_one(cs, triple, pin_at<double>(ctx, kPinT, true),
                                    pin_at<int32_t>(ctx, kPinStatus, true), st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  memcpy(T_out, pin_at<double>(ctx, kPinT, false), sizeof(double) * 16);
  if (status) *status = *pin_at<int32_t>(ctx, kPinStatus, false);
  return M3D_OK;
}

int m3d_ransac_score_one(m3d_ctx* ctx, const m3d_corrset* cs, const double* T, double thr, int mode,
                         int64_t* count, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, cs != nullptr && T != nullptr && count != nullptr, "invalid arguments");
  CHECK_ARG(ctx, mode == M3D_SCORE_SQUARED || mode == M3D_SCORE_NORM, "unknown score mode");
  if (cs->nc == 0) {  // ransac.py:220-221
    *count = 0;
    return M3D_OK;
  }
  hipSetDevice(ctx->device);
  int rc = pin_ensure(ctx);
  if (rc) return rc;
  hipStream_t st = S(stream);
  hipError_t e;
  {
    Arena a(ctx, st);
    const int64_t nb = count_one_blocks(cs->nc);
    const size_t o_p = a.take(sizeof(int32_t) * nb);
    rc = a.commit();
    if (rc) return rc;
    e = launch_count_one(cs, T, thr, mode, a.at<int32_t>(o_p), nb, ctx->one_ticket,
                         pin_at<int64_t>(ctx, kPinCount, true), st);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  *count = *pin_at<int64_t>(ctx, kPinCount, false);
  return M3D_OK;
}

// ------------------------------------------------------------------------------- a4
int m3d_ransac_run_async(m3d_ctx* ctx, const m3d_corrset* cs, const m3d_ransac_params* p,
                         const int32_t* triples, int32_t* counts_out,
                         m3d_ransac_result* result_dev, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, cs && p && result_dev, "invalid arguments");
  CHECK_ARG(ctx, p->max_iter >= 0, "max_iter must be >= 0");
  CHECK_ARG(ctx, p->mode == M3D_SCORE_SQUARED || p->mode == M3D_SCORE_NORM, "unknown score mode");
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  const int64_t nc = cs->nc;
  const int64_t max_iter = p->max_iter;
  int64_t B = p->batch;
  if (B <= 0) {
    // ~1e10 pair evaluations per batch (≤ 2^18 hypotheses, ~80 MB of scratch) amortise the
    // per-batch kabsch3/select latency and give the scoring grid more blocks (cfg2, 1e5
    // hypotheses: 10k per batch 2.15 ms, 25k 1.66 ms, 100k 1.55 ms — tools/ransac_batch.py);
    // early stop caps it (the stop is decided per batch)
    B = nc > 0 ? std::max<int64_t>(1024, std::min<int64_t>((int64_t)1 << 18,
                                                           (int64_t)1e10 / std::max<int64_t>(nc, 1)))
               : 1024;
    if (p->early_stop) B = std::min<int64_t>(B, 16384);
  }
  B = std::max<int64_t>(1, std::min<int64_t>(B, std::max<int64_t>(max_iter, 1)));
  const double thr_sq = thr_sq_of(p->thr, p->mode);
  Arena a(ctx, S(stream));
  size_t o[kScoreSlots];
  score_layout(a, B, o);
  size_t o_T = a.take(sizeof(double) * 16 * B);
  size_t o_c = a.take(sizeof(int32_t) * B);
  int rc = a.commit();
  if (rc) return rc;
  ScoreScratch s = score_bind(a, o);
  double* Tb = a.at<double>(o_T);
  int32_t* cb = a.at<int32_t>(o_c);
  // counts of the hypotheses after an early stop are never scored: they read 0
  if (counts_out != nullptr && max_iter > 0)
    HIPX(ctx, hipMemsetAsync(counts_out, 0, sizeof(int32_t) * max_iter, st));
  HIPX(ctx, launch_ransac_init(ctx->rstate, ctx->stats, max_iter == 0 ? 1 : 0, st));
  const int32_t* done = &ctx->rstate->done;
  for (int64_t b0 = 0; b0 < max_iter; b0 += B) {
    const int64_t n = std::min(B, max_iter - b0);
    const int32_t* tri = triples ? triples + 3 * b0 : nullptr;
    int32_t* cnt = counts_out ? counts_out + b0 : cb;
    hipError_t e;
    {
      KTimer kt(ctx, M3D_KERNEL_KABSCH, st);
      const ScoreFuse fz{&s.mf, p->thr, p->mode};
      e = launch_kabsch3(cs, tri, p->seed, p->hyp0 + b0, n, thr_sq, Tb, nullptr, s.hypf, done,
                         ZeroArgs{cnt}, st, nc > 0 ? &fz : nullptr);
    }
    if (e == hipSuccess) {
      if (nc > 0) {
        e = score_enqueue(ctx, cs, Tb, n, p->thr, p->mode, cnt, s, done, st, true);
      } else {
        e = hipMemsetAsync(cnt, 0, sizeof(int32_t) * n, st);
      }
    }
    if (e == hipSuccess)
      e = launch_select(cnt, b0, n, std::max<int64_t>(nc, 1), max_iter, p->early_stop,
                        p->es_threshold, p->es_confidence, Tb, ctx->rstate, st);
    if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  }
  hipError_t e = launch_copy_result(ctx->rstate, nc, ctx->stats, result_dev, st);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  return M3D_OK;
}

int m3d_ransac_run(m3d_ctx* ctx, const m3d_corrset* cs, const m3d_ransac_params* p,
                   const int32_t* triples, m3d_ransac_result* out, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, out != nullptr, "null output");
  m3d_ransac_result* dres = nullptr;
  int rc = dev_alloc(ctx, &dres, 1);
  if (rc) return rc;
  hipMemsetAsync(dres, 0, sizeof(*dres), S(stream));
  rc = m3d_ransac_run_async(ctx, cs, p, triples, nullptr, dres, stream);
  if (!rc) {
    hipError_t e = hipMemcpyAsync(out, dres, sizeof(*out), hipMemcpyDeviceToHost, S(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(S(stream));
    if (e != hipSuccess) rc = m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  }
  hipFree(dres);
  return rc;
}

// ------------------------------------------------------------------------------- MT19937 replay
namespace {
struct MT {
  uint32_t key[624];
  int pos;
  void gen() {
    const uint32_t A = 0x9908b0dfu, UP = 0x80000000u, LO = 0x7fffffffu;
    int i;
    uint32_t y;
    for (i = 0; i < 624 - 397; ++i) {
      y = (key[i] & UP) | (key[i + 1] & LO);
      key[i] = key[i + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
    }
    for (; i < 623; ++i) {
      y = (key[i] & UP) | (key[i + 1] & LO);
      key[i] = key[i + (397 - 624)] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
    }
    y = (key[623] & UP) | (key[0] & LO);
    key[623] = key[396] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
    pos = 0;
  }
  static uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  uint32_t next() {
    if (pos >= 624) gen();
    return temper(key[pos++]);
  }
};
}  // namespace

int m3d_replay_triples(uint32_t* mt_key, int32_t* mt_pos, int64_t nc, int64_t H,
                       int32_t* triples_out) {
  if (!mt_key || !mt_pos || (H > 0 && !triples_out)) return M3D_ERR_INVALID;
  if (nc < 3 || nc > 0xffffffffll) return M3D_ERR_INVALID;
  if (*mt_pos < 0 || *mt_pos > 624) return M3D_ERR_INVALID;
  MT mt;
  memcpy(mt.key, mt_key, sizeof(mt.key));
  mt.pos = *mt_pos;
  // legacy RandomState.choice(nc, 3, replace=False) == permutation(nc)[:3]; permutation shuffles
  // arange(nc) with i = nc-1 .. 1, j_i = random_interval(i), swap(x[i], x[j_i]).  Only positions
  // 0..2 are needed: the draws are stored (sequential writes), then each position is traced back
  // through the swaps in reverse order (i = 1 .. nc-1: p == i → j_i, p == j_i → i), which lands
  // on the initial index, i.e. the value.  Sequential passes, no O(nc) value array.
  thread_local std::vector<uint32_t> jbuf;
  if (jbuf.size() < (size_t)nc + 64) jbuf.resize((size_t)nc + 64);
  uint32_t* j = jbuf.data();
  uint32_t tk[624];  // the tempered outputs of the current key block
  auto temper_block = [&](int from) {
    for (int k = from; k < 624; ++k) tk[k] = MT::temper(mt.key[k]);  // vectorised
  };
  if (mt.pos < 624) temper_block(mt.pos);
  for (int64_t h = 0; h < H; ++h) {
    // random_interval(i) for i = nc-1 .. 1, branch-free: every MT output is a candidate
    // (y & mask(i), mask = 2^(⌊log2 i⌋+1) − 1) that is kept iff ≤ i — the rejection loop's
    // outcome is unpredictable, a branch on it costs more than the generator.  The mask is
    // constant while i stays above mask >> 1, so the dependency chain per output is the compare
    // and the decrement.
    int64_t i = nc - 1;
    while (i >= 1) {
      const uint32_t mask = 0xFFFFFFFFu >> __builtin_clz((uint32_t)i);
      const int64_t lo = (int64_t)(mask >> 1);
      while (i > lo) {
        if (mt.pos >= 624) {
          mt.gen();
          temper_block(0);
        }
        // at least i − lo more outputs are needed before i reaches lo (each output lowers i by
        // at most one), so that many run without a bound check
        const int k0 = mt.pos;
        const int n = (int)std::min<int64_t>(624 - k0, i - lo);
        uint32_t ii = (uint32_t)i;
        for (int k = k0; k < k0 + n; ++k) {
          const uint32_t v = tk[k] & mask;
          j[ii] = v;
          ii -= (uint32_t)(v <= ii);
        }
        mt.pos = k0 + n;
        i = ii;
      }
    }
    // trace positions 0..2 back through the swaps (i ascending).  After step i a traced
    // position p is ≤ i, so from i = 3 on it can only move when j_i == p (then p := i): a
    // vectorised search for the next index whose draw equals one of the three positions
    uint32_t p[3] = {0, 1, 2};
    for (int64_t a = 1; a < std::min<int64_t>(nc, 3); ++a) {
      const uint32_t ji = j[a], ia = (uint32_t)a;
      for (int q = 0; q < 3; ++q) p[q] = p[q] == ia ? ji : (p[q] == ji ? ia : p[q]);
    }
    int64_t a = 3;
    constexpr int kW = 32;
    while (a < nc) {
      const int64_t e = std::min<int64_t>(nc, a + kW);
      uint32_t any = 0;
      if (e - a == kW) {
        const uint32_t p0 = p[0], p1 = p[1], p2 = p[2];
        for (int t = 0; t < kW; ++t) {
          const uint32_t v = j[a + t];
          any |= (uint32_t)(v == p0) | (uint32_t)(v == p1) | (uint32_t)(v == p2);
        }
      } else {
        any = 1;
      }
      if (any) {
        for (int64_t b = a; b < e; ++b)
          for (int q = 0; q < 3; ++q) p[q] = j[b] == p[q] ? (uint32_t)b : p[q];
      }
      a = e;
    }
    triples_out[3 * h + 0] = (int32_t)p[0];
    triples_out[3 * h + 1] = (int32_t)p[1];
    triples_out[3 * h + 2] = (int32_t)p[2];
  }
  memcpy(mt_key, mt.key, sizeof(mt.key));
  *mt_pos = mt.pos;
  return M3D_OK;
}

// ------------------------------------------------------------------------------- clouds
int m3d_cloud_create(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                     void* stream, m3d_cloud** out) {
  return m3d_cloud_create_framed(ctx, xyz, normals, n, nullptr, stream, out);
}

namespace {
int cloud_create(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n, const double* center,
                 bool host, void* stream, m3d_cloud** out);
}

int m3d_cloud_create_framed(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                            const double* center, void* stream, m3d_cloud** out) {
  return cloud_create(ctx, xyz, normals, n, center, false, stream, out);
}

int m3d_cloud_create_host(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                          const double* center, void* stream, m3d_cloud** out) {
  return cloud_create(ctx, xyz, normals, n, center, true, stream, out);
}

namespace {
int cloud_create(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n, const double* center,
                 bool host, void* stream, m3d_cloud** out) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, out != nullptr, "null output");
  CHECK_ARG(ctx, n >= 0 && n < (int64_t)1 << 31, "point count out of range");
  CHECK_ARG(ctx, n == 0 || xyz != nullptr, "null device pointer");
  CHECK_ARG(ctx, center == nullptr || (std::isfinite(center[0]) && std::isfinite(center[1]) &&
                                       std::isfinite(center[2])),
            "non-finite centre");
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  Touch tch{ctx, st};
  m3d_cloud* c = new m3d_cloud();
  c->ctx = ctx;
  c->ctx_id = ctx->id;
  c->n = n;
  c->n_pad = round_up(std::max<int64_t>(n, 1), kCloudPad);
  int rc = M3D_OK;
  {
    Carve cv;  // the three point arrays in one allocation
    if (n > 0) cv.add(&c->xyz64, 3 * (size_t)n);
    if (n > 0 && normals) cv.add(&c->nrm64, 3 * (size_t)n);
    cv.add(&c->xyz32, (size_t)c->n_pad);
    if (cv.alloc(&c->block, &c->block_bytes, st) != hipSuccess) rc = m3d_fail(ctx, M3D_ERR_OOM, "device allocation failed (cloud)");
  }
  if (rc) {
    m3d_cloud_destroy(c);
    return rc;
  }
  if (n > 0 && host) {
    void* const dst[2] = {c->xyz64, c->nrm64};
    const void* const srcs[2] = {xyz, normals};
    const size_t bytes[2] = {sizeof(double) * 3 * (size_t)n, normals ? sizeof(double) * 3 * (size_t)n : 0};
    rc = upload_host(ctx, 2, dst, srcs, bytes, st);
    if (rc) {
      m3d_cloud_destroy(c);
      return rc;
    }
  } else if (n > 0) {
    hipError_t e = hipMemcpyAsync(c->xyz64, xyz, sizeof(double) * 3 * n, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && normals)
      e = hipMemcpyAsync(c->nrm64, normals, sizeof(double) * 3 * n, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) {
      m3d_cloud_destroy(c);
      return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
    }
  }
  if (center != nullptr) {
    for (int k = 0; k < 3; ++k) c->center[k] = center[k];
    c->center_given = 1;
  }
  rc = cloud_pack(ctx, c, n, center == nullptr, st);
  if (!rc) {
    // fp16 screen operand scale: a power of two with |S·x|∞ ≤ 32 (icp.hip pack16_sorted)
    int ex = 0;
    std::frexp(std::max(c->rmax, 1e-30) / 32.0, &ex);
    c->s16 = std::ldexp(1.0, -std::min(std::max(ex, -100), 100));
  }
  if (rc) {
    m3d_cloud_destroy(c);
    return rc;
  }
  *out = c;
  return M3D_OK;
}
}  // namespace

void m3d_cloud_destroy(m3d_cloud* c) {
  if (!c) return;
  // the blocks go back to the cache marked after every stream the context used (stream-ordered
  // reuse, no device sync)
  ReleaseScope rs(c->ctx, c->ctx_id);
  for (Grid* g : c->grids) {
    grid_free(g);
    delete g;
  }
  // Morton copies a live ICP loop still runs on are detached, not freed: the last loop to go
  // frees them (m3d_icp_destroy), so destroying the source before its loops stays safe
  for (auto& m : c->morton) {
    if (m.second->refs > 0)
      m.second->orphan = true;
    else
      m3d_cloud_destroy(m.second);
  }
  for (void** p : {reinterpret_cast<void**>(&c->slot), reinterpret_cast<void**>(&c->xyz64),
                   reinterpret_cast<void**>(&c->nrm64), reinterpret_cast<void**>(&c->xyz32)})
    if (in_block(*p, c->block, c->block_bytes)) *p = nullptr;
  block_release(c->block);
  hipFree(c->slot);
  hipFree(c->xyz64);
  hipFree(c->nrm64);
  hipFree(c->xyz32);
  block_release(c->rec64);
  delete c;
}

int64_t m3d_cloud_size(const m3d_cloud* c) { return c ? c->n : -1; }

// ------------------------------------------------------------------------------- ICP
namespace {
// uniform grid of a cloud for cell size `cell` (built once, synchronously, and cached on the
// cloud per cell size)
int ensure_grid(m3d_ctx* ctx, const m3d_cloud* c, double cell, hipStream_t st, const Grid** out) {
  for (Grid* g : c->grids)
    if (g->cell_req == cell && g->n_pts == c->n) {
      *out = g;
      return M3D_OK;
    }
  Grid* g = new Grid();
  float lohi[6];
  for (int k = 0; k < 3; ++k) {
    lohi[k] = c->lo[k];
    lohi[3 + k] = c->hi[k];
  }
  // asynchronous: the cloud's packing pass gave the bounds, the temporaries come from the arena
  hipError_t e = grid_build(c->xyz32, c->n, cell, st, g, &ctx->tmp, c->has_bounds ? lohi : nullptr);
  if (e != hipSuccess) {
    grid_free(g);
    delete g;
    return m3d_fail(ctx, M3D_ERR_HIP, std::string("grid build: ") + hipGetErrorString(e));
  }
  g->cell_req = cell;
  c->grids.push_back(g);
  *out = g;
  return M3D_OK;
}

// The ICP source in Morton slot order for cell size `cell` (grid.hip morton_source), built once and
// cached on the caller's cloud; sg = the caller's grid at that cell size.
int ensure_morton_source(m3d_ctx* ctx, const m3d_cloud* c, double cell, const m3d_cloud** out,
                         const Grid** gout) {
  for (auto& m : c->morton)
    if (m.first == cell && m.second->n == c->n) {
      *out = m.second;
      *gout = m.second->grids.front();
      return M3D_OK;
    }
  // straight from the points (grid.hip morton_source: the slots without the source's cell grid)
  m3d_cloud* mc = new m3d_cloud();
  mc->ctx = ctx;
  mc->ctx_id = ctx->id;
  Grid* g = new Grid();
  mc->grids.push_back(g);
  hipError_t e = morton_source(c, cell, mc, g, &ctx->tmp, nullptr);
  if (e != hipSuccess) {
    m3d_cloud_destroy(mc);
    return m3d_fail(ctx, M3D_ERR_HIP, std::string("morton source: ") + hipGetErrorString(e));
  }
  c->morton.emplace_back(cell, mc);
  // bounded cache: callers that query with many different radii (m3d_nn1, the a6 validation) would
  // otherwise keep one full source copy per cell size for the cloud's lifetime
  constexpr size_t kMortonKeep = 4;
  for (size_t k = 0; c->morton.size() > kMortonKeep && k + 1 < c->morton.size();) {
    if (c->morton[k].second->refs == 0) {
      m3d_cloud_destroy(c->morton[k].second);
      c->morton.erase(c->morton.begin() + (ptrdiff_t)k);
    } else {
      ++k;
    }
  }
  *out = mc;
  *gout = g;
  return M3D_OK;
}

// NN evaluation for the current transform → s->keys (brute: keyinit + scan; grid: one kernel).
// self_seed (m3d_icp_step's fused loop): when the previous fused tail left every key at
// kKeyNone (s->keys_clean), the brute-force scan seeds itself and the keyinit launch is skipped.
// [q0, q1): a slot range of the sources (q1 < 0: all), see icp_nn_splits.
hipError_t enqueue_nn(m3d_icp* s, int64_t off, hipStream_t st, bool self_seed = false, int64_t q0 = 0,
                      int64_t q1 = -1) {
  m3d_ctx* ctx = s->ctx;
  const bool whole = q0 == 0 && (q1 < 0 || q1 == s->src->n);
  const bool seeded = self_seed && s->keys_clean && off == 0 && whole;
  s->keys_clean = false;
  if (s->params.nn_method == M3D_NN_GRID) {
    KTimer kt(ctx, M3D_KERNEL_NN, st);
    return launch_grid_nn(s->src->xyz32, s->src->n, s->sgrid, s->tgrid, off, s->state, s->keys,
                          s->near2, s->corr, s->dprev, s->tgt->xyz32, s->tgt->n, st, q0, q1,
                          s->hlist, s->hcnt, s->cand_cap, s->pcd64, s->tgt->xyz64, s->hcap, s->scan_xchunk);
  }
  if (!seeded) {
    hipError_t e = launch_icp_keyinit(s, off, st, q0, q1);
    if (e != hipSuccess) return e;
  }
  KTimer kt(ctx, M3D_KERNEL_NN, st);
  return launch_icp_nn(s, off, seeded, st, q0, q1);
}
}  // namespace

extern "C++" {
namespace m3d {
int icp_shard_nn_range(m3d_icp* s, int64_t off, int64_t q0, int64_t q1, int64_t* dkeys, hipStream_t st) {
  hipError_t e = enqueue_nn(s, off, st, false, q0, q1);
  if (e == hipSuccess) e = launch_shard_winner(s, off, dkeys, st, q0, q1);
  if (e != hipSuccess) return m3d_fail(s->ctx, M3D_ERR_HIP, std::string("shard NN: ") + hipGetErrorString(e));
  return M3D_OK;
}
}  // namespace m3d
}  // extern "C++"

namespace {
int icp_create(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt, double max_dist,
               const m3d_icp_params* params, m3d_icp** out, bool run_arena);
constexpr int kLoopArrays = 11;
struct LoopLayout {
  bool heavy;
};
}

int m3d_icp_create(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt, double max_dist,
                   const m3d_icp_params* params, m3d_icp** out) {
  return icp_create(ctx, src, tgt, max_dist, params, out, false);
}

namespace {
// Dense target cells (a cell at ≈ r holding ≥ kHeavyCell points — e.g. the vertex fan at a
// UV-sphere pole, ~30× the mean density): queries with more than kHeavyCand candidates are
// deferred to grid_nn_heavy_kernel (one block per query) so that the few waves of such queries
// do not set the launch time (cfg4: up to 250 µs per evaluation).  M3D_GRID_HEAVY=0: never,
// =N: always, with cap N (tests).  Off on evenly dense clouds (cfg1's largest cell ≈ 20).
int32_t heavy_cap(const m3d_icp_params* params, int64_t coarse_max_occ) {
  constexpr int64_t kHeavyCell = 256;
  constexpr int32_t kHeavyCand = 256;
  static const int heavy_env = [] {
    const char* e = getenv("M3D_GRID_HEAVY");
    return e ? std::max(0, atoi(e)) : -1;
  }();
  if (params->nn_method != M3D_NN_GRID) return 0;
  return heavy_env > 0 ? heavy_env : (heavy_env < 0 && coarse_max_occ >= kHeavyCell ? kHeavyCand : 0);
}

// the loop's arrays: state, keys, near2, dprev, ld64, lidx, corr, partials + sums, hlist, hcnt
// (+ ticket), pcd64 — offsets into one block
LoopLayout loop_layout(int64_t ns, int32_t cand_cap, size_t* off, size_t* tot) {
  const size_t n1 = (size_t)std::max<int64_t>(ns, 1);
  const size_t nh = cand_cap > 0 ? n1 : 0;
  const size_t sz[kLoopArrays] = {sizeof(IcpState), 8 * n1, 4 * n1, 8 * n1, 8 * n1, 4 * n1, 4 * n1,
                                  sizeof(double) * (size_t)(terms_blocks(ns) * kTermSlots + kTermSlots), 4 * nh,
                                  kDeferWords * sizeof(uint32_t), 24 * n1};
  *tot = 0;
  for (int k = 0; k < kLoopArrays; ++k) {
    off[k] = *tot;
    *tot += tmp_align(sz[k]);
  }
  return LoopLayout{nh > 0};
}

// run_arena: the loop's arrays come from the context's run arena (kept between calls) instead of
// their own allocation — for the synchronous one-shot entry points (m3d_icp_run, m3d_nn1), whose
// loop object dies inside the call: no hipMalloc / hipFree (≈0.2 ms, the free waits for the
// device and unmaps) per call
int icp_create(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt, double max_dist,
               const m3d_icp_params* params, m3d_icp** out, bool run_arena) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, src && tgt && params && out, "invalid arguments");
  CHECK_ARG(ctx, max_dist > 0.0, "Invalid max_correspondence_distance.");
  CHECK_ARG(ctx, params->estimation == M3D_EST_POINT_TO_PLANE ||
                     params->estimation == M3D_EST_POINT_TO_POINT,
            "unknown estimation");
  CHECK_ARG(ctx, params->estimation != M3D_EST_POINT_TO_PLANE || tgt->nrm64 != nullptr || tgt->n == 0,
            "TransformationEstimationPointToPlane requires pre-computed normal vectors for target "
            "PointCloud.");
  CHECK_ARG(ctx, params->max_iteration >= 0, "max_iteration must be >= 0");
  CHECK_ARG(ctx, params->nn_method == M3D_NN_BRUTE || params->nn_method == M3D_NN_GRID,
            "unknown nn_method");
  hipSetDevice(ctx->device);
  const Grid *tg = nullptr, *sg = nullptr;
  const m3d_cloud* src_m = nullptr;
  int64_t coarse_max_occ = 0;  // most target points in one cell at cell ≈ r (grid NN)
  int32_t cand_cap = 0;
  size_t off[kLoopArrays] = {}, tot = 0;
  LoopLayout layout{};
  void* blk = nullptr;
  {
    // Grid NN: cell ≈ the search radius, a query visits 3 cells per axis.  Brute force: the
    // same grids only ORDER the points (targets and queries in cell order make the MFMA
    // screen's 32-target sub-tiles and 64-query waves spatially compact); every pair is still
    // screened.
    const double cell = max_dist * 1.001;
    int grc = ensure_grid(ctx, tgt, cell, nullptr, &tg);
    // the loop runs on the source in Morton slot order (sg: the copy's query grid)
    const m3d_cloud* ms = nullptr;
    if (!grc) grc = ensure_morton_source(ctx, src, cell, &ms, &sg);
    if (!grc) src_m = ms;
    if (!grc) {
      hipError_t e = ensure_target_rec(tgt, nullptr);
      if (e != hipSuccess) grc = m3d_fail(ctx, M3D_ERR_HIP, std::string("target records: ") + hipGetErrorString(e));
    }
    // (after the source grid, Morton copy and target records are enqueued: the occupancy's one
    // sync then also covers them instead of stalling the queue in between)
    // Grid NN on a dense target: a seeded query's box is ~1–2 cells per axis, so the candidates
    // it scans grow with the points per cell.  Shrink the target cell by div = ⌊√(m / 3.5)⌋
    // (m = points per occupied cell at cell ≈ r; any cell size gives the same keys, grid.hip):
    // measured (tools/grid_cell_sweep.sh) 1M × 1M (m ≈ 33) 206 → 128 µs per scan at div 3;
    // cfg1 (m ≈ 3.9) and the 1M × 125k shard (m ≈ 4.7) are fastest at div 1.
    if (!grc && params->nn_method == M3D_NN_GRID) {
      hipError_t e = pin_ensure(ctx) == M3D_OK ? hipSuccess : hipErrorOutOfMemory;
      if (e == hipSuccess)  // one sync, once per grid
        e = grid_occupancy(const_cast<Grid*>(tg), &ctx->tmp, nullptr, pin_read<unsigned long long>(ctx, true),
                           pin_read<unsigned long long>(ctx, false));
      if (e != hipSuccess) grc = m3d_fail(ctx, M3D_ERR_HIP, std::string("grid occupancy: ") + hipGetErrorString(e));
    }
    if (!grc && params->nn_method == M3D_NN_GRID && tg->n_occ > 0) {
      coarse_max_occ = tg->max_occ;
      const double m = (double)tg->n_pts / (double)tg->n_occ;
      const int div = std::min(4, std::max(1, (int)std::floor(std::sqrt(m / 3.5))));
      if (div > 1) grc = ensure_grid(ctx, tgt, cell / div, nullptr, &tg);
    }
    if (!grc) {  // the terms pass's fp64 walk for ambiguous queries (nnkey.h resolve_wave)
      hipError_t e = build_grid_pts64(tgt, const_cast<Grid*>(tg), nullptr);
      if (e != hipSuccess) grc = m3d_fail(ctx, M3D_ERR_HIP, std::string("grid fp64 points: ") + hipGetErrorString(e));
    }
    if (!grc && params->nn_method == M3D_NN_BRUTE && tg->mf16 == nullptr) {
      hipError_t e = build_mfma_tiles(tgt, const_cast<Grid*>(tg), nullptr);
      if (e != hipSuccess) grc = m3d_fail(ctx, M3D_ERR_HIP, std::string("mfma tiles: ") + hipGetErrorString(e));
    }
    // the loop's arrays in ONE block (from the block cache: a reused block's release mark is
    // waited for on the null stream, and so covered by the sync below)
    if (!grc) {
      cand_cap = heavy_cap(params, coarse_max_occ);
      layout = loop_layout(src->n, cand_cap, off, &tot);
      if (!run_arena && block_alloc(&blk, tot, nullptr) != hipSuccess)
        grc = m3d_fail(ctx, M3D_ERR_OOM, "device allocation failed (ICP loop arrays)");
      if (!grc && run_arena && ctx->run.reserve(tot) != hipSuccess)
        grc = m3d_fail(ctx, M3D_ERR_OOM, "device allocation failed (ICP loop arrays)");
    }
    // the deferral list's count / ticket / fault word start at zero BEFORE the sync below: a block
    // from the cache may hold any bytes of its previous owner (e.g. 0xFF fills), and a memset left
    // queued on the null stream is not ordered before a caller's non-blocking stream
    if (!grc && layout.heavy) {
      char* b0 = run_arena ? ctx->run.base : static_cast<char*>(blk);
      if (hipMemsetAsync(b0 + off[9], 0, kDeferWords * sizeof(uint32_t), nullptr) != hipSuccess)
        grc = m3d_fail(ctx, M3D_ERR_HIP, "loop arrays: deferral counter");
    }
    // the setup above ran asynchronously on the null stream: finish it before the loop object is
    // used on the caller's streams
    if (!grc) {
      hipError_t e = hipStreamSynchronize(nullptr);
      if (e != hipSuccess) grc = m3d_fail(ctx, M3D_ERR_HIP, std::string("loop setup: ") + hipGetErrorString(e));
    }
    if (grc) {
      block_release(blk);
      return grc;
    }
  }
  m3d_icp* s = new m3d_icp();
  s->ctx = ctx;
  s->ctx_id = ctx->id;
  s->src = src_m;
  src_m->refs += 1;  // the Morton copy stays cached while this loop runs on it
  s->user_src = src;
  s->tgt = tgt;
  s->params = *params;
  s->max_dist = max_dist;
  s->nblocks = terms_blocks(src->n);
  s->tgrid = tg;
  // brute-force query order: the Morton slots themselves (compact 64-query waves, contiguous
  // slot ranges for the split exchange of the target-shard loop)
  s->sgrid = sg;
  s->cand_cap = cand_cap;
  // a target whose extent along some axis is under half the source's (a spatial shard, m3d.dist
  // spatial_shards): the scan's real work concentrates in the Morton ranges near the target, so its
  // blocks go to the XCDs in chunks of 8 (tools/xchunk_sweep.sh: 8 slabs of 1M × 1M, per-shard
  // scan 39.8 → 32.6 µs; a whole-extent target keeps one contiguous eighth per XCD)
  if (src->has_bounds && tgt->has_bounds)
    for (int k = 0; k < 3; ++k)
      if ((double)(tgt->hi[k] - tgt->lo[k]) * 2.0 < (double)(src->hi[k] - src->lo[k])) s->scan_xchunk = 8;
  int rc = M3D_OK;
  char* b = static_cast<char*>(blk);
  if (run_arena) {
    b = ctx->run.base;  // reserved (and its deferral words zeroed) before the setup sync
  } else {
    s->block = blk;
  }
  if (b == nullptr) {
    rc = m3d_fail(ctx, M3D_ERR_OOM, "device allocation failed (ICP loop arrays)");
  } else {
    s->state = reinterpret_cast<IcpState*>(b + off[0]);
    s->keys = reinterpret_cast<int64_t*>(b + off[1]);
    s->near2 = reinterpret_cast<uint32_t*>(b + off[2]);
    s->dprev = reinterpret_cast<int64_t*>(b + off[3]);
    s->ld64 = reinterpret_cast<int64_t*>(b + off[4]);
    s->lidx = reinterpret_cast<int32_t*>(b + off[5]);
    s->corr = reinterpret_cast<int32_t*>(b + off[6]);
    s->partials = reinterpret_cast<double*>(b + off[7]);
    s->sums = s->partials + s->nblocks * kTermSlots;
    s->pcd64 = reinterpret_cast<double*>(b + off[10]);
    if (layout.heavy) {  // zeroed above; grid_nn_heavy_kernel re-zeroes count + ticket, icp_reset all
      s->hlist = reinterpret_cast<int32_t*>(b + off[8]);
      s->hcnt = reinterpret_cast<uint32_t*>(b + off[9]);
      s->hcap = (int32_t)std::max<int64_t>(src->n, 1);
    }
  }
  if (rc) {
    m3d_icp_destroy(s);
    return rc;
  }
  *out = s;
  return M3D_OK;
}
}  // namespace

void m3d_icp_destroy(m3d_icp* s) {
  if (!s) return;
  for (hipGraphExec_t g : s->graph)
    if (g != nullptr) hipGraphExecDestroy(g);
  if (s->cap_stream != nullptr) hipStreamDestroy(s->cap_stream);
  if (s->src != nullptr) {
    m3d_cloud* ms = const_cast<m3d_cloud*>(s->src);
    if (--ms->refs == 0 && ms->orphan) m3d_cloud_destroy(ms);  // its parent cloud is gone
  }
  {
    ReleaseScope rs(s->ctx, s->ctx_id);  // back to the block cache, marked after the loop's work
    block_release(s->block);             // state, keys, near2, dprev, ld64, lidx, corr, partials, sums
  }
  hipFree(s->xdk);
  hipFree(s->xcl);
  hipFree(s->xsums);
  delete s;
}

namespace {
// Eigen's Matrix4d::isIdentity() (dummy precision 1e-12), as RegistrationICP tests its init:
// |a_ii − 1| ≤ 1e-12·min(|a_ii|, 1), |a_ij| ≤ 1e-12
bool eigen_is_identity(const double* T) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      const double a = T[4 * i + j];
      if (i == j ? !(std::fabs(a - 1.0) <= 1e-12 * std::min(std::fabs(a), 1.0)) : !(std::fabs(a) <= 1e-12))
        return false;
    }
  return true;
}

int icp_reset(m3d_icp* s, const double* init, bool open3d_init, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  m3d_ctx* ctx = s->ctx;
  double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  const double* T = init ? init : I;
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  HIPX(ctx, hipMemsetAsync(s->corr, 0xFF, sizeof(int32_t) * std::max<int64_t>(s->src->n, 1), st));
  // all-ones bits = a NaN distance: no bound seed until a target-shard exchange wrote dprev
  HIPX(ctx, hipMemsetAsync(s->dprev, 0xFF, sizeof(int64_t) * std::max<int64_t>(s->src->n, 1), st));
  // the deferral list's count, ticket and fault word start at zero on the caller's stream (the
  // heavy kernel re-zeroes count and ticket after each scan; a reset also clears a fault)
  if (s->hcnt != nullptr) HIPX(ctx, hipMemsetAsync(s->hcnt, 0, kDeferWords * sizeof(uint32_t), st));
  // RegistrationICP (Registration.cpp): pcd = source; if (!init.isIdentity()) pcd.Transform(init)
  HIPX(ctx, launch_icp_reset(s, T, !(open3d_init && eigen_is_identity(T)), st));
  s->keys_clean = false;
  return M3D_OK;
}
}  // namespace

int m3d_icp_reset(m3d_icp* s, const double* init, void* stream) { return icp_reset(s, init, true, stream); }

int m3d_icp_copy_points(const m3d_icp* s, double* dst, void* stream) {
  if (!s || (!dst && s->src->n > 0)) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  HIPX(s->ctx, launch_copy_points(s, dst, S(stream)));
  return M3D_OK;
}

namespace {
// Whether an iteration's tail runs as ONE launch (terms + last-block reduce [+ solve]).  The
// fused last block reduces every block partial alone, with 256 threads: past ~256 blocks the
// separate 1024-thread reduce_kernel is faster (1M sources, grid loop: fused 60.7 µs against
// terms 33.1 + reduce 8.8 + solve 6.5 µs, rocprof).  Where the fused tail hands the keys back
// (brute force: the next scan then seeds itself, no keyinit launch) it stays fused.  Both forms
// sum in the same fixed order: the same bits.
bool fused_tail(const m3d_icp* s, bool keys_back) {
  static const bool env = [] {
    const char* e = getenv("M3D_ICP_FUSED");
    return !(e && atoi(e) == 0);
  }();
  return env && (keys_back || s->nblocks <= 256);
}
}  // namespace

int m3d_icp_step(m3d_icp* s, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  m3d_ctx* ctx = s->ctx;
  hipStream_t st = S(stream);
  // brute force: the fused tail hands the keys back as kKeyNone, the next NN seeds itself
  const bool reset = s->params.nn_method != M3D_NN_GRID && s->src->n > 0;
  const bool fused = fused_tail(s, reset);
  HIPX(ctx, enqueue_nn(s, 0, st, fused));
  if (fused) {
    KTimer kt(ctx, M3D_KERNEL_TERMS, st);
    HIPX(ctx, launch_icp_terms_solve(s, reset, st));
    s->keys_clean = reset;
    return M3D_OK;
  }
  { KTimer kt(ctx, M3D_KERNEL_TERMS, st); HIPX(ctx, launch_icp_terms_mode(s, 0, nullptr, nullptr, st)); }
  HIPX(ctx, launch_icp_reduce_solve(s, st));
  return M3D_OK;
}

namespace {
// n steps as ONE graph launch: the sequence (NN scan [+ keyinit] + fused tail per step, 2–3
// kernels each) is captured on a loop-owned stream the second time the same (n, keys_clean on
// entry) is requested — a one-shot run never pays the capture — and then replayed on the
// caller's stream — the per-kernel host enqueues and the stream's per-dispatch
// gaps become one graph launch.  Every kernel argument is a device pointer into the loop's state,
// so a replay computes exactly what the enqueued steps would (tests: test_gpu_icp graph cases).
// Not used while kernel profiling records events, or after a failed capture (plain enqueues).
bool icp_graphs_on() {
  static const bool on = [] {
    const char* e = getenv("M3D_ICP_GRAPH");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

int capture_steps(m3d_icp* s, int32_t n) {
  if (s->cap_stream == nullptr &&
      hipStreamCreateWithFlags(&s->cap_stream, hipStreamNonBlocking) != hipSuccess) {
    s->cap_stream = nullptr;
    return M3D_ERR_HIP;
  }
  const bool kc0 = s->keys_clean;
  const int slot = kc0 ? 1 : 0;
  if (hipStreamBeginCapture(s->cap_stream, hipStreamCaptureModeThreadLocal) != hipSuccess)
    return M3D_ERR_HIP;
  int rc = M3D_OK;
  for (int32_t k = 0; k < n && rc == M3D_OK; ++k) rc = m3d_icp_step(s, s->cap_stream);
  hipGraph_t g = nullptr;
  const hipError_t ee = hipStreamEndCapture(s->cap_stream, &g);
  const bool kc1 = s->keys_clean;
  s->keys_clean = kc0;  // nothing ran yet
  hipGraphExec_t ex = nullptr;
  if (rc == M3D_OK && ee == hipSuccess && g != nullptr &&
      hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) == hipSuccess) {
    if (s->graph[slot] != nullptr) hipGraphExecDestroy(s->graph[slot]);
    s->graph[slot] = ex;
    s->graph_n[slot] = n;
    s->graph_kc_out[slot] = kc1;
  } else {
    rc = rc ? rc : M3D_ERR_HIP;
  }
  if (g != nullptr) hipGraphDestroy(g);
  (void)hipGetLastError();
  return rc;
}
}  // namespace

int m3d_icp_prepare_steps(m3d_icp* s, int32_t n) {
  if (!s) return M3D_ERR_INVALID;
  CHECK_ARG(s->ctx, n >= 0, "n must be >= 0");
  if (n < 2 || !icp_graphs_on() || s->graph_off) return M3D_OK;  // plain enqueues then
  hipSetDevice(s->ctx->device);
  if (capture_steps(s, n) != M3D_OK) {
    s->graph_off = true;
    (void)hipGetLastError();
  }
  return M3D_OK;
}

int m3d_icp_steps(m3d_icp* s, int32_t n, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  CHECK_ARG(s->ctx, n >= 0, "n must be >= 0");
  if (n >= 2 && icp_graphs_on() && !s->graph_off && !s->ctx->profiling) {
    const int slot = s->keys_clean ? 1 : 0;
    const bool have = s->graph[slot] != nullptr && s->graph_n[slot] == n;
    const bool again = s->seen_n[slot] == n;
    s->seen_n[slot] = n;
    if (!have && again) {
      hipSetDevice(s->ctx->device);
      if (capture_steps(s, n) != M3D_OK) s->graph_off = true;
    }
    if ((have || again) && !s->graph_off) {
      HIPX(s->ctx, hipGraphLaunch(s->graph[slot], S(stream)));
      s->keys_clean = s->graph_kc_out[slot];
      return M3D_OK;
    }
  }
  for (int32_t k = 0; k < n; ++k) {
    const int rc = m3d_icp_step(s, stream);
    if (rc) return rc;
  }
  return M3D_OK;
}

int m3d_icp_shard_nn(m3d_icp* s, int64_t off, int64_t* dkeys, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  m3d_ctx* ctx = s->ctx;
  CHECK_ARG(ctx, off >= 0, "negative shard offset");
  CHECK_ARG(ctx, dkeys != nullptr || off == 0, "a target shard (offset > 0) needs the dkeys exchange buffer");
  hipStream_t st = S(stream);
  // dkeys == NULL: source-sharded protocol, the keys stay inside and the keyinit-free scan may
  // run; else target shard: this shard's fp64 winners → the MIN exchange buffer
  HIPX(ctx, enqueue_nn(s, off, st, dkeys == nullptr));
  if (dkeys != nullptr) HIPX(ctx, launch_shard_winner(s, off, dkeys, st));
  return M3D_OK;
}

int m3d_icp_shard_nn_range(m3d_icp* s, int64_t off, int64_t q0, int64_t q1, int64_t* dkeys, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  m3d_ctx* ctx = s->ctx;
  CHECK_ARG(ctx, off >= 0, "negative shard offset");
  CHECK_ARG(ctx, dkeys != nullptr, "null dkeys");
  CHECK_ARG(ctx, 0 <= q0 && q0 <= q1 && q1 <= s->src->n, "slot range outside [0, ns]");
  CHECK_ARG(ctx, icp_nn_range_ok(s), "this loop's NN cannot run on a slot range (fp32 VALU / per-query form)");
  return icp_shard_nn_range(s, off, q0, q1, dkeys, S(stream));
}

int m3d_icp_shard_claim(m3d_icp* s, const int64_t* dmin, int32_t* claim, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};  // reads the loop's block: its release mark must cover this launch
  CHECK_ARG(s->ctx, dmin != nullptr && claim != nullptr, "null exchange buffer");
  HIPX(s->ctx, launch_shard_claim(s, dmin, claim, S(stream)));
  return M3D_OK;
}

int m3d_icp_shard_terms(m3d_icp* s, int64_t off, const int64_t* dmin, const int32_t* claim,
                        double* sums, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  m3d_ctx* ctx = s->ctx;
  CHECK_ARG(ctx, sums != nullptr, "null sums");
  CHECK_ARG(ctx, (dmin == nullptr) == (claim == nullptr), "dmin and claim go together");
  CHECK_ARG(ctx, claim != nullptr || off == 0, "a target shard (offset > 0) needs dmin and claim");
  hipStream_t st = S(stream);
  s->keys_clean = false;
  // keys kept inside (source shard): the fused tail hands them back as kKeyNone like m3d_icp_step
  const bool reset = claim == nullptr && s->src->n > 0 && s->params.nn_method != M3D_NN_GRID;
  if (fused_tail(s, reset)) {  // terms + fixed-order reduce in one launch (same bits as the two kernels)
    KTimer kt(ctx, M3D_KERNEL_TERMS, st);
    HIPX(ctx, launch_icp_terms_reduce(s, off, claim, dmin, sums, reset, st));
    s->keys_clean = reset;
    return M3D_OK;
  }
  { KTimer kt(ctx, M3D_KERNEL_TERMS, st); HIPX(ctx, launch_icp_terms_mode(s, off, claim, dmin, st)); }
  HIPX(ctx, launch_icp_reduce(s, sums, st));
  return M3D_OK;
}

int m3d_icp_solve(m3d_icp* s, const double* sums, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};  // writes IcpState (the loop's block)
  HIPX(s->ctx, launch_icp_solve(s, sums ? sums : s->sums, S(stream)));
  return M3D_OK;
}

int m3d_icp_set_source_total(m3d_icp* s, int64_t ns_total) {
  if (!s) return M3D_ERR_INVALID;
  CHECK_ARG(s->ctx, ns_total >= 0 && (ns_total == 0 || ns_total >= s->src->n),
            "source total must be 0 or at least the shard's source count");
  s->ns_total = ns_total;
  s->graph_n[0] = s->graph_n[1] = -1;  // the captured solve carries the fitness denominator
  return M3D_OK;
}

int m3d_icp_result_get(m3d_icp* s, m3d_icp_result* out, void* stream) {
  if (!s || !out) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  m3d_ctx* ctx = s->ctx;
  IcpState h;
  uint32_t defer[kDeferWords] = {0, 0, 0, 0};
  HIPX(ctx, hipMemcpyAsync(&h, s->state, sizeof(h), hipMemcpyDeviceToHost, S(stream)));
  if (s->hcnt != nullptr)
    HIPX(ctx, hipMemcpyAsync(defer, s->hcnt, sizeof(defer), hipMemcpyDeviceToHost, S(stream)));
  HIPX(ctx, hipStreamSynchronize(S(stream)));
  // the grid scan's deferral list overflowed (a count the scan found larger than the list — the
  // loop's own writes were dropped, never out of bounds): the keys of this run are not trustworthy
  if (defer[kDeferFault] != 0)
    return m3d_fail(ctx, M3D_ERR_HIP,
                    "grid NN deferral list overflow (count " + std::to_string(defer[0]) +
                        "): results since the last m3d_icp_reset are invalid");
  for (int k = 0; k < 16; ++k) {
    out->T[k] = h.T[k];
    out->update[k] = h.last_upd[k];
  }
  out->fitness = h.fitness;
  out->inlier_rmse = h.rmse;
  out->num_correspondences = h.count;
  out->iterations = h.iters;
  out->converged = h.converged;
  return M3D_OK;
}

int m3d_corr_pairs(m3d_ctx* ctx, const int32_t* corr_idx, int64_t n, int32_t* pairs_out, int64_t* count,
                   void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, count != nullptr && n >= 0 && n < (int64_t)1 << 31, "invalid arguments");
  CHECK_ARG(ctx, n == 0 || (corr_idx != nullptr && pairs_out != nullptr), "null array");
  *count = 0;
  if (n == 0) return M3D_OK;
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  const int64_t nb = (n + 1023) / 1024;
  const size_t o_p = tmp_align(sizeof(int32_t) * (size_t)(nb + 1));
  if (ctx->tmp.reserve(o_p + sizeof(int32_t) * 2 * (size_t)n) != hipSuccess)
    return m3d_fail(ctx, M3D_ERR_OOM, "correspondence pairs scratch");
  int32_t* cnt = reinterpret_cast<int32_t*>(ctx->tmp.base);
  int32_t* pairs = reinterpret_cast<int32_t*>(ctx->tmp.base + o_p);
  int32_t m = 0;
  hipError_t e = launch_corr_pairs(corr_idx, n, cnt, pairs, st);
  if (e == hipSuccess) e = hipMemcpyAsync(&m, cnt + nb, sizeof(m), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess && m > 0) {
    e = hipMemcpyAsync(pairs_out, pairs, sizeof(int32_t) * 2 * (size_t)m, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  *count = m;
  return M3D_OK;
}

const int32_t* m3d_icp_corr(const m3d_icp* s) { return s ? s->corr : nullptr; }

int m3d_icp_copy_corr(const m3d_icp* s, int32_t* dst, void* stream) {
  if (!s || !dst) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  if (s->src->n == 0) return M3D_OK;
  HIPX(s->ctx, launch_scatter_i32(s->corr, s->src->slot, s->src->n, dst, S(stream)));
  return M3D_OK;
}

int m3d_icp_copy_slots(const m3d_icp* s, int32_t* dst, void* stream) {
  if (!s || !dst) return M3D_ERR_INVALID;
  Touch tch{s->ctx, S(stream)};
  if (s->src->n == 0) return M3D_OK;
  HIPX(s->ctx, hipMemcpyAsync(dst, s->src->slot, sizeof(int32_t) * s->src->n, hipMemcpyDeviceToDevice,
                              S(stream)));
  return M3D_OK;
}

int m3d_icp_run(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt, const double* init,
                double max_dist, const m3d_icp_params* params, m3d_icp_result* out,
                int32_t* corr_idx, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  Touch tch{ctx, S(stream)};
  CHECK_ARG(ctx, out != nullptr, "null output");
  m3d_icp* s = nullptr;
  int rc = icp_create(ctx, src, tgt, max_dist, params, &s, true);
  if (rc) return rc;
  rc = m3d_icp_reset(s, init, stream);
  // max_iteration + 1 evaluations, enqueued in
  // growing chunks (4, 8, 16, …) with a look at the state's `done` between chunks — a converged
  // loop (often after a handful of evaluations) then does not enqueue the remaining ~2 launches
  // per evaluation that would only read `done` and return.  The evaluations that run are the
  // same; only the early-exit launches are skipped.
  if (!rc) {
    const int32_t total = params->max_iteration + 1;
    s->graph_off = true;  // a one-shot loop: no HIP graph capture (two equal chunks would trigger one)
    int32_t left = total, chunk = 4;
    while (!rc && left > 0) {
      const int32_t k = std::min(chunk, left);
      rc = m3d_icp_steps(s, k, stream);
      left -= k;
      chunk *= 2;
      if (rc || left == 0) break;
      int32_t done = 0;
      hipError_t e = hipMemcpyAsync(&done, &s->state->done, sizeof(done), hipMemcpyDeviceToHost, S(stream));
      if (e == hipSuccess) e = hipStreamSynchronize(S(stream));
      if (e != hipSuccess) rc = m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
      if (done) break;
    }
  }
  if (!rc) rc = m3d_icp_result_get(s, out, stream);
  if (!rc && corr_idx && src->n > 0) {
    hipError_t e = launch_scatter_i32(s->corr, s->src->slot, src->n, corr_idx, S(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(S(stream));
    if (e != hipSuccess) rc = m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  }
  m3d_icp_destroy(s);
  return rc;
}

int m3d_nn1(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt, const double* T_host,
            double max_dist, int32_t nn_method, int32_t* idx, double* d2, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  Touch tch{ctx, S(stream)};
  CHECK_ARG(ctx, src && tgt && (idx || src->n == 0), "invalid arguments");
  CHECK_ARG(ctx, max_dist > 0.0, "max_dist must be > 0");
  m3d_icp_params p{1e-6, 1e-6, 0, M3D_EST_POINT_TO_POINT, nn_method, 0};
  m3d_icp* s = nullptr;
  int rc = icp_create(ctx, src, tgt, max_dist, &p, &s, true);
  if (rc) return rc;
  hipStream_t st = S(stream);
  rc = icp_reset(s, T_host, false, stream);  // the 1-NN of T·src for any T
  hipError_t e = hipSuccess;
  if (!rc) e = enqueue_nn(s, 0, st);
  if (e == hipSuccess) e = launch_nn_finalize(s, idx, d2, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (!rc && e != hipSuccess) rc = m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  m3d_icp_destroy(s);
  return rc;
}

// ------------------------------------------------------------------------------- preprocessing
extern "C++" {
namespace {
// device scratch released on scope exit (after the synchronous entry point has synchronised)
template <class T>
struct DevTmp {
  T* p = nullptr;
  ~DevTmp() { hipFree(p); }
};

// the grids of a hybrid search: cell = radius, plus the finer first-stage grid when the cloud is
// dense enough (prep.hip hybrid_fine_radius; both cached on the cloud)
int search_grids(m3d_ctx* ctx, const m3d_cloud* c, double radius, int k, hipStream_t st,
                 const Grid** g, const Grid** gf, double* hf) {
  int rc = ensure_grid(ctx, c, radius, st, g);
  if (rc) return rc;
  hipError_t e = grid_occupancy(const_cast<Grid*>(*g), &ctx->tmp, st);  // hybrid_fine_radius reads it
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, std::string("grid occupancy: ") + hipGetErrorString(e));
  *gf = nullptr;
  *hf = hybrid_fine_radius(*g, radius, k);
  if (*hf > 0.0) rc = ensure_grid(ctx, c, *hf, st, gf);
  return rc;
}

// Neighbour lists of the synchronous preprocessing calls (estimate_normals, compute_fpfh): a
// context-owned device buffer, grown on demand and reused — the lists of a 180k-point cloud at
// k = 30 take 65 MB, whose hipMalloc + hipFree per call cost more than the normals kernel.  Safe
// to reuse because those entry points synchronise their stream before returning and a context
// serves one host thread (m3d.h).
struct NbrLists {
  int32_t* idx = nullptr;
  double* d2 = nullptr;
  int32_t* cnt = nullptr;
  double* extra = nullptr;  // caller's n × extra_per_point doubles (FPFH: the SPFH rows)
};

// the context's preprocessing buffer with at least `need` bytes (grown, never shrunk)
int prep_buffer(m3d_ctx* ctx, size_t need, char** out) {
  if (need > ctx->prep_bytes) {
    if (ctx->prep) hipFree(ctx->prep);
    ctx->prep = nullptr;
    ctx->prep_bytes = 0;
    if (dev_malloc(&ctx->prep, need) != hipSuccess) {
      ctx->prep = nullptr;
      return m3d_fail(ctx, M3D_ERR_OOM, "hipMalloc: preprocessing scratch");
    }
    ctx->prep_bytes = need;
  }
  *out = static_cast<char*>(ctx->prep);
  return M3D_OK;
}

int prep_lists(m3d_ctx* ctx, int64_t n, int k, int64_t extra_per_point, NbrLists* L) {
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t bi = up(sizeof(int32_t) * (size_t)n * k), bd = up(sizeof(double) * (size_t)n * k);
  const size_t bc = up(sizeof(int32_t) * (size_t)n), be = up(sizeof(double) * (size_t)(n * extra_per_point));
  char* b = nullptr;
  const int rc = prep_buffer(ctx, bi + bd + bc + be, &b);
  if (rc) return rc;
  L->idx = reinterpret_cast<int32_t*>(b);
  L->d2 = reinterpret_cast<double*>(b + bi);
  L->cnt = reinterpret_cast<int32_t*>(b + bi + bd);
  L->extra = reinterpret_cast<double*>(b + bi + bd + bc);
  return M3D_OK;
}

// hybrid neighbourhoods of every point of `c` (grid cell = radius)
int neighbourhoods(m3d_ctx* ctx, const m3d_cloud* c, double radius, int k, hipStream_t st,
                   int64_t extra_per_point, NbrLists* L) {
  const Grid *g = nullptr, *gf = nullptr;
  double hf = 0.0;
  int rc = search_grids(ctx, c, radius, k, st, &g, &gf, &hf);
  if (rc) return rc;
  rc = prep_lists(ctx, std::max<int64_t>(c->n, 1), k, extra_per_point, L);
  if (rc) return rc;
  HIPX(ctx, hybrid_search(c, g, radius, k, L->idx, L->d2, L->cnt, st, gf, hf));
  return M3D_OK;
}
}  // namespace
}  // extern "C++"

int m3d_voxel_down_sample(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                          double voxel_size, double* out_xyz, double* out_normals, int64_t* out_n,
                          void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, out_n != nullptr && n >= 0 && n < ((int64_t)1 << 31), "invalid arguments");
  CHECK_ARG(ctx, voxel_size > 0.0, "voxel_size <= 0.");
  CHECK_ARG(ctx, n == 0 || (xyz && out_xyz), "null device pointer");
  hipSetDevice(ctx->device);
  std::string why;
  // scratch from the context's preprocessing buffer: the call synchronises before returning
  char* scratch = nullptr;
  int rc = n > 0 ? prep_buffer(ctx, voxel_scratch_bytes(n), &scratch) : M3D_OK;
  if (rc) return rc;
  hipError_t e = voxel_down_sample(xyz, normals, n, voxel_size, out_xyz, normals ? out_normals : nullptr,
                                   out_n, scratch, S(stream), &why);
  if (e != hipSuccess)
    return m3d_fail(ctx, why.empty() ? M3D_ERR_HIP : M3D_ERR_INVALID,
                    why.empty() ? std::string("voxel_down_sample: ") + hipGetErrorString(e) : why);
  return M3D_OK;
}

int m3d_hybrid_search(m3d_ctx* ctx, const m3d_cloud* cloud, double radius, int32_t max_nn,
                      int32_t* idx, double* d2, int32_t* count, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, cloud && idx && d2 && count, "invalid arguments");
  CHECK_ARG(ctx, radius > 0.0 && max_nn >= 1 && max_nn <= 256, "radius > 0 and 1 <= max_nn <= 256");
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  Touch tch{ctx, st};
  const Grid *g = nullptr, *gf = nullptr;
  double hf = 0.0;
  int rc = search_grids(ctx, cloud, radius, max_nn, st, &g, &gf, &hf);
  if (rc) return rc;
  HIPX(ctx, hybrid_search(cloud, g, radius, max_nn, idx, d2, count, st, gf, hf));
  HIPX(ctx, hipStreamSynchronize(st));
  return M3D_OK;
}

int m3d_estimate_normals(m3d_ctx* ctx, const m3d_cloud* cloud, double radius, int32_t max_nn,
                         double* normals_out, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, cloud && (normals_out || cloud->n == 0), "invalid arguments");
  CHECK_ARG(ctx, radius > 0.0 && max_nn >= 1 && max_nn <= 256, "radius > 0 and 1 <= max_nn <= 256");
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  Touch tch{ctx, st};
  NbrLists L;
  int rc = neighbourhoods(ctx, cloud, radius, max_nn, st, 0, &L);
  if (rc) return rc;
  HIPX(ctx, launch_normals(cloud, L.idx, max_nn, L.cnt, cloud->nrm64, normals_out, st));
  HIPX(ctx, hipStreamSynchronize(st));
  return M3D_OK;
}

int m3d_compute_fpfh(m3d_ctx* ctx, const m3d_cloud* cloud, const double* normals, double radius,
                     int32_t max_nn, double* fpfh_out, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, cloud && ((normals && fpfh_out) || cloud->n == 0),
            "Failed because input point cloud has no normal.");
  CHECK_ARG(ctx, radius > 0.0 && max_nn >= 1 && max_nn <= 256, "radius > 0 and 1 <= max_nn <= 256");
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  Touch tch{ctx, st};
  NbrLists L;
  int rc = neighbourhoods(ctx, cloud, radius, max_nn, st, 33, &L);
  if (rc) return rc;
  HIPX(ctx, launch_fpfh(cloud, normals, L.idx, L.d2, max_nn, L.cnt, L.extra, fpfh_out, st));
  HIPX(ctx, hipStreamSynchronize(st));
  return M3D_OK;
}

// ------------------------------------------------------------------------------- feature matching
int m3d_feature_correspondences(m3d_ctx* ctx, const double* f_src, int64_t ns, const double* f_tgt,
                                int64_t nt, int32_t dim, int32_t mutual_filter,
                                double mutual_consistent_ratio, int32_t* corr_out, int64_t* n_out,
                                void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, dim == 33, "feature dimension must be 33 (FPFH)");
  CHECK_ARG(ctx, n_out && ns >= 0 && nt >= 0 && ns < ((int64_t)1 << 31) && nt < ((int64_t)1 << 31),
            "invalid arguments");
  CHECK_ARG(ctx, (ns == 0 || (f_src && corr_out)) && (nt == 0 || f_tgt), "null device pointer");
  hipSetDevice(ctx->device);
  HIPX(ctx, feature_correspondences(f_src, ns, f_tgt, nt, mutual_filter, mutual_consistent_ratio,
                                    corr_out, n_out, S(stream)));
  return M3D_OK;
}

int m3d_ransac_on_correspondences(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt,
                                  const int32_t* corr, int64_t nc,
                                  const m3d_feature_ransac_params* p,
                                  m3d_feature_ransac_result* out, int32_t* corr_set_out,
                                  void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, src && tgt && p && out, "invalid arguments");
  CHECK_ARG(ctx, p->ransac_n <= 3, "ransac_n > 3 is not supported (the reference uses 3)");
  CHECK_ARG(ctx, p->max_iteration >= 0, "max_iteration must be >= 0");
  hipSetDevice(ctx->device);
  hipStream_t st = S(stream);
  Touch tch{ctx, st};
  memset(out, 0, sizeof(*out));
  for (int k = 0; k < 16; ++k) out->T[k] = (k % 5 == 0) ? 1.0 : 0.0;
  out->best_index = -1;
  const int64_t ns = src->n;
  if (corr_set_out && ns > 0) HIPX(ctx, hipMemsetAsync(corr_set_out, 0xFF, 4 * ns, st));
  // Open3D returns an empty RegistrationResult for these (Registration.cpp)
  if (p->ransac_n < 3 || nc < p->ransac_n || !(p->max_correspondence_distance > 0.0) ||
      p->max_iteration == 0 || ns == 0 || tgt->n == 0) {
    HIPX(ctx, hipStreamSynchronize(st));
    return M3D_OK;
  }
  CHECK_ARG(ctx, corr != nullptr, "null correspondence pointer");
  const int64_t H = p->max_iteration;
  DevTmp<double> T;
  DevTmp<int32_t> pass;
  int rc = dev_alloc(ctx, &T.p, 16 * H);
  if (!rc) rc = dev_alloc(ctx, &pass.p, H);
  if (rc) return rc;
  HIPX(ctx, launch_feat_hyp(src->xyz64, tgt->xyz64, corr, nc, p->seed, H, p->edge_length,
                            p->distance, T.p, pass.p, st));
  std::vector<int32_t> hpass(H);
  HIPX(ctx, hipMemcpyAsync(hpass.data(), pass.p, 4 * H, hipMemcpyDeviceToHost, st));
  HIPX(ctx, hipStreamSynchronize(st));
  m3d_icp_params ip{1e-6, 1e-6, 0, M3D_EST_POINT_TO_POINT, M3D_NN_GRID, 0};
  m3d_icp* s = nullptr;
  rc = m3d_icp_create(ctx, src, tgt, p->max_correspondence_distance, &ip, &s);
  if (rc) return rc;
  // Validation of the checker-passing hypotheses in batches (grid.hip validate_kernel: one launch
  // evaluates a whole batch), each batch followed by Open3D's sequential selection over it:
  // IsBetterRANSACThan and the early exit at est_k (a hypothesis at or past est_k is never
  // validated).  Batches grow from 64 so the reference's iteration = 30 costs one small launch;
  // a batch that straddles est_k only computes results the selection then ignores.
  std::vector<int32_t> list;
  for (int64_t h = 0; h < H; ++h)
    if (hpass[h]) list.push_back((int32_t)h);
  const int64_t npass = (int64_t)list.size();
  const int64_t cap = std::min<int64_t>(
      npass, std::max<int64_t>(64, std::min<int64_t>(8192, ((int64_t)1 << 23) / std::max<int64_t>(ns, 1))));
  const int64_t nbq = validate_blocks(ns);
  DevTmp<int32_t> dlist, vcorr;
  DevTmp<IcpState> vst;
  DevTmp<double> vpart, vres;
  if (npass > 0) {
    rc = dev_alloc(ctx, &dlist.p, npass);
    if (!rc) rc = dev_alloc(ctx, &vst.p, cap);
    if (!rc) rc = dev_alloc(ctx, &vpart.p, cap * nbq * 2);
    if (!rc) rc = dev_alloc(ctx, &vres.p, cap * 2);
    if (!rc) rc = dev_alloc(ctx, &vcorr.p, cap);
    if (rc) {
      m3d_icp_destroy(s);
      return rc;
    }
  }
  hipError_t e = hipSuccess;
  if (npass > 0)
    e = hipMemcpyAsync(dlist.p, list.data(), 4 * npass, hipMemcpyHostToDevice, st);
  int64_t est_k = H, best = -1;
  double best_fit = 0.0, best_rmse = 0.0, corres_ratio = 0.0;
  std::vector<double> hs;
  std::vector<int32_t> hc;
  for (int64_t c0 = 0, bsz = std::min<int64_t>(64, cap); c0 < npass && e == hipSuccess;
       c0 += bsz, bsz = std::min<int64_t>(cap, 2 * bsz)) {
    if (list[c0] >= est_k) break;
    const int64_t n = std::min<int64_t>(bsz, npass - c0);
    e = launch_val_states(s, T.p, dlist.p + c0, n, vst.p, st);
    if (e == hipSuccess)
      e = launch_validate(s->sgrid, ns, s->src->xyz64, s->tgrid, tgt->xyz64, tgt->n, vst.p, n, vpart.p,
                          vres.p, st);
    // the exit rule's correspondence inlier counts of the same batch (one small launch; only a
    // new best's is read)
    if (e == hipSuccess)
      e = launch_corres_inlier(src->xyz64, tgt->xyz64, corr, nc, T.p, dlist.p + c0, n,
                               p->max_correspondence_distance, vcorr.p, st);
    hs.resize(2 * (size_t)n);
    hc.resize((size_t)n);
    if (e == hipSuccess)
      e = hipMemcpyAsync(hs.data(), vres.p, sizeof(double) * 2 * n, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
      e = hipMemcpyAsync(hc.data(), vcorr.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) break;
    for (int64_t k = 0; k < n; ++k) {
      const int64_t h = list[c0 + k];
      if (h >= est_k) break;
      out->validations += 1;
      const double cnt = hs[2 * k], se = hs[2 * k + 1];
      const double fit = cnt > 0.0 ? cnt / (double)ns : 0.0;
      const double rmse = cnt > 0.0 ? std::sqrt(se / cnt) : 0.0;
      if (fit > best_fit || (fit == best_fit && rmse < best_rmse)) {  // IsBetterRANSACThan
        best = h;
        best_fit = fit;
        best_rmse = rmse;
        // Open3D 0.19 (Registration.cpp RegistrationRANSACBasedOnCorrespondence): the exit
        // estimate comes from the new best's CORRESPONDENCE inlier ratio
        // (EvaluateInlierCorrespondenceRatio), not from its fitness:
        //   est_k_d = log(1 − confidence) / log(1 − ratio^ransac_n); est_k ← ceil(est_k_d) if smaller.
        // ratio = 1: log(0) = −inf, est_k_d = −0.0 → 0.  ratio = 0: a division by +0.0 → −inf,
        // whose int conversion upstream is INT_MIN on x86 → stop (0 here).  NaN: no change.
        const double ratio = (double)hc[k] / (double)nc;
        corres_ratio = ratio;
        const double kd = std::log(1.0 - p->confidence) /
                          std::log(1.0 - std::pow(ratio, (double)p->ransac_n));
        if (kd < (double)est_k) est_k = std::isfinite(kd) ? (int64_t)std::ceil(kd) : 0;
      }
    }
  }
  if (e != hipSuccess) {
    m3d_icp_destroy(s);
    return m3d_fail(ctx, M3D_ERR_HIP, std::string("feature RANSAC: ") + hipGetErrorString(e));
  }
  if (best >= 0) {
    e = hipMemcpyAsync(out->T, T.p + 16 * best, sizeof(double) * 16, hipMemcpyDeviceToHost, st);
    out->fitness = best_fit;
    out->inlier_rmse = best_rmse;
    out->best_index = best;
    out->corres_ratio = corres_ratio;
    if (e == hipSuccess && corr_set_out) {
      e = launch_icp_set_T(s, T.p + 16 * best, st);
      if (e == hipSuccess) e = enqueue_nn(s, 0, st);
      if (e == hipSuccess) e = launch_icp_terms_mode(s, 0, nullptr, nullptr, st);
      if (e == hipSuccess)
        e = launch_scatter_i32(s->corr, s->src->slot, ns, corr_set_out, st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  m3d_icp_destroy(s);
  if (e != hipSuccess) return m3d_fail(ctx, M3D_ERR_HIP, hipGetErrorString(e));
  return M3D_OK;
}

// ------------------------------------------------------------------------------- test hooks
int m3d_debug_kabsch3_host(const double* src9, const double* tgt9, double* T16) {
  if (!src9 || !tgt9 || !T16) return M3D_ERR_INVALID;
  double ps[3][3], qs[3][3];
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) {
      ps[i][k] = src9[3 * i + k];
      qs[i][k] = tgt9[3 * i + k];
    }
  return kabsch3(ps, qs, T16);
}

int m3d_debug_ldlt6_host(const double* A36, const double* b6, double* x6) {
  if (!A36 || !b6 || !x6) return M3D_ERR_INVALID;
  if (!ldlt6_solve_spd(A36, b6, x6)) ldlt6_solve(A36, b6, x6);  // the device solve's rule (icp.hip)
  return M3D_OK;
}

int m3d_debug_acos_cr(const double* u, int64_t n, double* out) {
  if (n < 0 || (n > 0 && (!u || !out))) return M3D_ERR_INVALID;
  for (int64_t k = 0; k < n; ++k) out[k] = acos_cr(u[k]);  // the device's code, compiled for the host
  return M3D_OK;
}

int m3d_debug_acos_device(m3d_ctx* ctx, const double* u, int64_t n, double* out, int mode, void* stream) {
  if (!ctx) return M3D_ERR_INVALID;
  CHECK_ARG(ctx, n >= 0 && (n == 0 || (u && out)) && (mode == 0 || mode == 1), "invalid arguments");
  hipSetDevice(ctx->device);
  HIPX(ctx, launch_acos_probe(u, n, out, mode, S(stream)));
  return M3D_OK;
}

int m3d_debug_block_cache_fill(int byte) {
  // synchronous: every idle block's release point has passed before, and the fill is complete
  // after, so the next owner sees exactly these bytes
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (hipDeviceSynchronize() != hipSuccess) return M3D_ERR_HIP;
  std::lock_guard<std::mutex> lk(g_bc_mu);
  int n = 0;
  for (const CachedBlock& b : g_bc) {
    if (b.dev != cur) continue;
    if (hipMemset(b.p, byte & 0xFF, b.bytes) != hipSuccess) return M3D_ERR_HIP;
    ++n;
  }
  if (hipDeviceSynchronize() != hipSuccess) return M3D_ERR_HIP;
  return n;
}

int m3d_debug_icp_defer_count(m3d_icp* s, uint32_t count, void* stream) {
  if (!s) return M3D_ERR_INVALID;
  CHECK_ARG(s->ctx, s->hcnt != nullptr, "this loop has no deferral list (grid NN with a candidate cap only)");
  Touch tch{s->ctx, S(stream)};
  HIPX(s->ctx, hipMemcpyAsync(s->hcnt, &count, sizeof(count), hipMemcpyHostToDevice, S(stream)));
  HIPX(s->ctx, hipStreamSynchronize(S(stream)));
  return M3D_OK;
}

}  // extern "C"
