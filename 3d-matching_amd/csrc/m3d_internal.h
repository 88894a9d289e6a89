// m3d_internal.h — library-private types shared by the HIP translation units and the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <utility>
#include <functional>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/m3d.h"

// Uniform (wave-invariant) loads: a pointer in the constant address space makes the AMDGPU
// backend emit scalar s_load / s_buffer_load, which put the data in SGPRs and broadcast it to
// every lane for free (the hypothesis block in scoring, the target tile in the NN scan).
#define M3D_CONST __attribute__((address_space(4)))

namespace m3d {

constexpr int kWave = 64;

// fp32 hypothesis block for the scoring screen (64 B = one s_load_dwordx16).
// r: rotation row-major, t: translation in the centred frames (T p + t - q evaluated as
// R p_c + t' - q_c with p_c = p - c_src, q_c = q - c_tgt), lo/hi: guard band around thr².
struct alignas(64) HypF32 {
  float r[9];
  float t[3];
  float lo, hi;
  float pad[2];
};

// Plain 16-B point for constant-address-space (scalar) loads; HIP's float4 has no
// address-space-qualified copy constructor.
struct alignas(16) Pt4 {
  float x, y, z, w;
};

// Per-batch scoring state zeroed by the kernel that runs before the screen.
struct ZeroArgs {
  int32_t* counts = nullptr;
};

// Running state of the a4 loop across batches (device resident).
struct RansacState {
  double T_best[16];
  int64_t best_count;
  int64_t best_index;
  int64_t iterations;
  int64_t rechecked;
  int32_t done;
  uint32_t ticket;     // select_best_kernel's block ticket (the last block finalises the batch)
  int32_t pad[2];
  uint64_t batch_key;  // select_best_kernel's blocks → its last block (no-early-stop batches)
};

// ICP loop state (device resident), Open3D RegistrationICP semantics.
struct IcpState {
  double T[16];       // current transformation (world frame)
  float Rt32[12];     // fp32 R (row-major) + t' mapping centred source to centred target
  double fitness, rmse;
  double prev_fitness, prev_rmse;
  int64_t count;      // correspondences of the last evaluation
  int32_t evals;      // evaluations done
  int32_t iters;      // updates applied
  int32_t done;
  int32_t converged;
  double r2;          // max_dist² (fp64, strict <)
  float r2_hi;        // fp32 search bound (≥ r2 plus guard)
  float screen_eps;   // NN screen error bound (icp.hip refresh_rt32)
  float screen_eps_m; // NN screen error bound of the fp16-split MFMA screen
  float mfma_scale;   // power-of-two scale of the fp16 operands (the target cloud's s16)
  int32_t mfma_ok;    // scaled query magnitudes fit fp16: the MFMA screen may run
  uint32_t ticket;    // fused terms→reduce→solve: blocks done this iteration (last one resets)
  float Rt32_prev[12];  // Rt32 of the previous evaluation (nnkey.h seed_key bounds)
  int32_t bound_ok;     // Rt32_prev, keys and corr belong to the previous evaluation
  float band_e;         // 2·e_q·1.01: absolute term of nnkey.h band_of (fp32 → fp64 ambiguity)
  float eq;             // e_q: bound on |fp32 distance − fp64 distance| for the current T
  float eq_prev;        // e_q of the previous evaluation (seed_key bounds)
  // the transform the next evaluation applies to the loop's points: its fp64 queries are
  // dT·pcd64[i], written back (Open3D transforms its copy of the source by every update,
  // pcd.Transform(update)); after a reset, init (or I when init isIdentity()), then each ΔT
  double dT[16];
  double last_upd[16];  // the last ΔT a solve produced (I since the reset): m3d_icp_result.update
};

// Uniform grid over a cloud's centred fp32 points (grid.hip): kernel view + owner.
struct GridDev {
  float o[3];
  float inv_h;
  int n[3];
  int64_t ncells = 0;
  const int32_t* start = nullptr;  // ncells + 1 sorted-array offsets
  const float4* pts = nullptr;     // points sorted by cell, w = index bits
  const double4* pts64 = nullptr;  // the same points in fp64, w = index bits (ICP loops' target
                                   // grid, nnkey.h resolve_wave), or null
};

struct Grid {
  GridDev dev;
  int32_t* start = nullptr;
  float4* pts = nullptr;
  int32_t* order = nullptr;  // point indices in cell order
  // the points in Morton (Z-curve) order of their cells (w = index bits) and each point's position
  // in that order: the query order of the grid NN (grid.hip grid_morton); built on first use
  float4* mpts = nullptr;
  int32_t* minv = nullptr;
  int64_t n_pts = 0;
  int64_t n_occ = 0;      // occupied cells (grid_occupancy; 0: not counted)
  int64_t max_occ = 0;    // most points in one cell (grid_occupancy)
  bool occ_known = false;
  double cell = 0.0;      // cell size used
  double cell_req = 0.0;  // cell size requested
  // brute-force MFMA screen operands in this grid's cell order (icp.hip pack16_sorted), padded
  // to mf_npad: fp16 hi/lo split (2 × uint4 per point) + fp32 (x, y, z, original index bits)
  uint4* mf16 = nullptr;
  float4* mf32 = nullptr;
  int64_t mf_npad = 0;
  double4* pts64 = nullptr;  // dev.pts64 (build_grid_pts64, icp.hip)
  // one allocation holding several of the arrays above (Carve; grid_free frees it, not them)
  void* block = nullptr;
  size_t block_bytes = 0;
};

// Device scratch for the temporaries of setup work (grid sorts, Morton copies, cloud packing):
// grown on demand and owned by the context.  Setup work runs in stream order, so consecutive
// users on one stream reuse it without a host sync; an outgrown buffer is retired (freed with the
// context), never freed under work still in flight.  Replaces a hipMalloc/hipFree pair per
// temporary (hipFree waits for the device).
hipError_t dev_malloc_raw(void** p, size_t bytes);  // (below: the block cache)
struct TmpArena {
  char* base = nullptr;
  size_t cap = 0;
  std::vector<void*> retired;
  hipError_t reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    const size_t want = std::max(bytes, 2 * cap);
    void* p = nullptr;
    const hipError_t e = dev_malloc_raw(&p, want);
    if (e != hipSuccess) return e;
    if (base != nullptr) retired.push_back(base);
    base = static_cast<char*>(p);
    cap = want;
    return hipSuccess;
  }
  void release() {
    for (void* p : retired) (void)hipFree(p);
    retired.clear();
    if (base != nullptr) (void)hipFree(base);
    base = nullptr;
    cap = 0;
  }
};
// hostio.cpp's worker pool: fn(0 .. n-1) over the pool's threads and the caller; in_order(k) runs
// on the caller's thread once items 0..k are all done, in index order
void host_pipeline(int64_t n, const std::function<void(int64_t)>& fn, const std::function<void(int64_t)>& in_order);
// 256-B aligned carve-out of a TmpArena reservation
inline size_t tmp_align(size_t b) { return (b + 255) & ~(size_t)255; }

// Device block cache (api.cpp): the blocks of clouds, grids, Morton copies, target records and
// MFMA tiles go back to a process-wide cache when their object dies, and a later allocation of
// a size in [need, 2·need] takes one.  hipFree of a 2–5 MB block costs ≈ 160 µs on the box
// (unmapping; tools/ubench_alloc.hip), which a caller registering many pairs paid on every call
// that evicted older clouds from the drop-in cache (tools/multipair_timing.py).  Reuse is
// stream-ordered: a block released inside a ReleaseScope carries that scope's mark (an event
// after all work its context had enqueued, on every stream it used: ctx_touch), and the
// allocating stream waits for it on the device.
struct ReleaseMark {
  hipEvent_t ev = nullptr;  // null: nothing had been enqueued
  ~ReleaseMark();
};
// record that ctx enqueued work on st (entry points that read or write cached blocks)
void ctx_touch(m3d_ctx* ctx, hipStream_t st);
// an entry point that enqueues work reading or writing cached device blocks (clouds, grids, loop
// sources) records, when it returns, that its context used this stream
struct Touch {
  m3d_ctx* ctx;
  hipStream_t st;
  ~Touch() { ctx_touch(ctx, st); }
};
// blocks released while a scope is alive carry its mark (m3d_cloud_destroy, m3d_icp_destroy)
struct ReleaseScope {
  std::shared_ptr<ReleaseMark> prev;
  ReleaseScope(m3d_ctx* ctx, uint64_t ctx_id);  // ctx_id: m3d_ctx::id when the object was made
  ~ReleaseScope();
};
hipError_t block_alloc(void** p, size_t bytes, hipStream_t st = nullptr);
void block_release(void* p);
size_t block_cache_trim(int dev);  // free the cached blocks of device dev; returns bytes freed
void ctx_count(int dev, int delta);  // live contexts per device (the last one trims the cache)
void ctx_register(m3d_ctx* ctx, bool live);  // the live-context registry (ReleaseScope checks it)
// hipMalloc that trims the block cache and retries once on out-of-memory
hipError_t dev_malloc_raw(void** p, size_t bytes);
template <class T>
hipError_t dev_malloc(T** p, size_t bytes) {
  return dev_malloc_raw(reinterpret_cast<void**>(p), bytes);
}

// Several device arrays in ONE allocation (256-B aligned pieces): the setup paths make one
// hipMalloc per object instead of one per array, and the owner one hipFree.
struct Carve {
  std::vector<std::pair<void**, size_t>> parts;
  template <class T>
  void add(T** p, size_t count) {
    parts.emplace_back(reinterpret_cast<void**>(p), tmp_align(sizeof(T) * std::max<size_t>(count, 1)));
  }
  hipError_t alloc(void** block, size_t* bytes, hipStream_t st = nullptr) {
    size_t tot = 0;
    for (auto& q : parts) tot += q.second;
    void* b = nullptr;
    const hipError_t e = block_alloc(&b, std::max<size_t>(tot, 1), st);
    *block = e == hipSuccess ? b : nullptr;
    *bytes = e == hipSuccess ? tot : 0;
    if (e != hipSuccess) return e;
    size_t o = 0;
    for (auto& q : parts) {
      *q.first = static_cast<char*>(b) + o;
      o += q.second;
    }
    return hipSuccess;
  }
};
// whether p lies inside [block, block + bytes) (the arrays a Carve block holds)
inline bool in_block(const void* p, const void* block, size_t bytes) {
  return block != nullptr && p >= block && static_cast<const char*>(p) < static_cast<const char*>(block) + bytes;
}

// the grid NN's deferral list header (m3d_icp::hcnt): [0] count, [1] grid_nn_heavy_kernel's block
// ticket, [2] fault (a count beyond the list: the write was dropped), [3] pad
constexpr int kDeferWords = 4;
constexpr int kDeferFault = 2;
constexpr int kTermSlots = 32;  // 21 JTJ + 6 JTr + r² + count + Σd² (+2 pad)
constexpr int64_t kKeyNone = 0x7FFFFFFFFFFFFFFFll;

}  // namespace m3d

struct m3d_ctx {
  int device = 0;
  std::string err;
  // kernel timing (m3d_profile_*): event pairs per kernel id
  bool profiling = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[6];
  size_t ev_used[6] = {0, 0, 0, 0, 0, 0};
  // scratch (grown on demand)
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  int64_t* stats = nullptr;  // [8] device counters
  m3d::RansacState* rstate = nullptr;
  // cross-stream ordering of the scratch/rstate users (api.cpp Arena)
  hipEvent_t scratch_ev = nullptr;
  hipStream_t scratch_stream = nullptr;
  bool scratch_used = false;
  // mapped pinned host memory for the one-hypothesis calls (m3d_kabsch3_one / _score_one):
  // kernels write their few results straight into it (pin_dev), read after one stream sync
  void* pin = nullptr;
  void* pin_dev = nullptr;
  uint32_t* one_ticket = nullptr;  // device: last-block ticket of count_one_kernel (kept at 0)
  // neighbour lists of the synchronous preprocessing calls (api.cpp prep_lists), grown on demand
  void* prep = nullptr;
  size_t prep_bytes = 0;
  m3d::TmpArena tmp;  // setup temporaries (grids, Morton copies, cloud packing)
  m3d::TmpArena run;  // loop arrays of the synchronous one-shot ICP / NN calls (api.cpp icp_create)
  // streams this context enqueued work on, each with an event re-recorded at every such call
  // (api.cpp ctx_touch): the release marks of the block cache wait for all of them on `order`
  std::vector<std::pair<hipStream_t, hipEvent_t>> uses;  // (pruned of completed entries per mark)
  std::mutex uses_mu;  // ctx_touch vs ReleaseScope (destroys may run on finaliser threads)
  bool uses_lost = false;  // an event could not be made: releases fall back to a device sync
  hipStream_t order = nullptr;
  bool counted = false;  // counted among its device's live contexts (api.cpp ctx_count)
  uint64_t id = 0;       // unique per process (api.cpp ctx_register)
};

struct m3d_corrset {
  m3d_ctx* ctx = nullptr;
  int64_t nc = 0, nc_pad = 0;
  double* p64 = nullptr;  // nc×3 gathered source points (original frame)
  double* q64 = nullptr;  // nc×3 gathered target points
  float4* p32 = nullptr;  // nc_pad centred source (w = 0), pad = 0
  float4* q32 = nullptr;  // nc_pad centred target, pad = far away
  double cs[3] = {0, 0, 0}, ct[3] = {0, 0, 0};
  double pmax2 = 0.0;    // max |p_c|∞ (guard-band bound)
  double qmaxinf = 0.0;  // max |q_c|∞
  // MFMA scoring operands (ransac.hip score_mfma_kernel): 4 planes × nc_pad of fp16 hi/lo
  // splits of S·p_c / S·q_c (plane 0: the p part, planes 1-3: the q_x / q_y / q_z parts)
  uint4* ca16 = nullptr;
  double s16 = 0.0;  // the power-of-two scale S (0: MFMA scoring unavailable)
};

struct m3d_cloud {
  m3d_ctx* ctx = nullptr;
  uint64_t ctx_id = 0;  // ctx->id at creation (a cloud may outlive its context at teardown)
  int64_t n = 0, n_pad = 0;
  double* xyz64 = nullptr;  // n×3
  double* nrm64 = nullptr;  // n×3 or null
  float4* xyz32 = nullptr;  // n_pad centred (pad = far away)
  double center[3] = {0, 0, 0};
  double rmax = 0.0;  // max |x_c|∞ (guard-band bound)
  // per-axis min / max of the centred fp32 points (the grid bounds; from the packing pass)
  float lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  bool has_bounds = false;
  double s16 = 1.0;  // power-of-two scale of the fp16 MFMA screen operands (|s16·x|∞ ≤ 32)
  int center_given = 0;  // centre supplied by the caller (a frame shared by target shards)
  mutable std::vector<m3d::Grid*> grids;  // uniform grids built on demand, one per cell size
  // target records for the ICP terms pass (icp.hip pack_rec): point + normal (zeros without
  // normals) as 8 doubles per point, 64-B aligned, so the gather of a source's winner touches one
  // 64-B segment instead of one in each of xyz64 and nrm64; built on first use as an ICP target
  mutable double* rec64 = nullptr;
  // ICP sources: copies of this cloud in the Morton order of its grid, one per cell size (grid.hip
  // morton_copy), built on first use by m3d_icp_create; in a copy, slot[k] = the index in this
  // (parent) cloud of the copy's point k
  mutable std::vector<std::pair<double, m3d_cloud*>> morton;
  int32_t* slot = nullptr;
  // a Morton copy: live ICP loops running on it (m3d_icp_create / _destroy); the parent keeps at
  // most kMortonKeep copies and evicts the oldest unreferenced one beyond that (api.cpp)
  mutable int refs = 0;
  bool orphan = false;  // a Morton copy whose parent was destroyed while loops still ran on it
  // one allocation holding the point arrays (Carve; m3d_cloud_destroy frees it, not them)
  void* block = nullptr;
  size_t block_bytes = 0;
};

struct m3d_icp {
  m3d_ctx* ctx = nullptr;
  uint64_t ctx_id = 0;  // the context's registry id (release marks only while it lives)
  // the loop's source: the caller's cloud in Morton slot order (user_src->morton); every per-source
  // array below is indexed by slot, src->slot maps a slot to the caller's point index
  const m3d_cloud* src = nullptr;
  const m3d_cloud* user_src = nullptr;
  const m3d_cloud* tgt = nullptr;
  m3d_icp_params params{};
  double max_dist = 0.0;
  void* block = nullptr;           // device: one allocation holding the arrays below (api.cpp)
  m3d::IcpState* state = nullptr;  // device
  int64_t* keys = nullptr;         // ns packed NN keys: k1 = (d2f, index) minimum of the scan
  uint32_t* near2 = nullptr;       // ns: bits of the smallest d2f of any other target evaluated
  int64_t* dprev = nullptr;        // ns: target-sharded loops, bits of the global winner's d64
  int64_t* ld64 = nullptr;         // ns: target-sharded loops, bits of this shard's winner's d64
  int32_t* lidx = nullptr;         // ns: target-sharded loops, this shard's fp64 winner (-1 none)
  // grid NN on a target with dense cells (grid.hip grid_nn_heavy_kernel): the queries deferred
  // by the per-query scan (ns slots), their count and the kernel's block ticket; cand_cap = 0: no
  // deferral
  int32_t* hlist = nullptr;
  uint32_t* hcnt = nullptr;  // kDeferWords: count, ticket, fault
  int32_t hcap = 0;          // hlist entries (the scan drops, and flags, a slot at or past it)
  int32_t cand_cap = 0;
  // grid scan block → XCD mapping (grid.hip): 0 = one contiguous eighth of the Morton order per
  // XCD; C > 0 = chunks of C blocks dealt round-robin — for a target that covers a slab of the
  // source's extent (a spatial shard), whose queries' work sits in a few Morton ranges
  int32_t scan_xchunk = 0;
  bool keys_clean = false;         // host view: every key is kKeyNone (fused tail reset them)
  int32_t* corr = nullptr;         // ns current correspondence (-1 none)
  double* pcd64 = nullptr;         // ns×3: the source as Open3D's RegistrationICP holds it — the
                                   // points after every update but the last (dT, IcpState)
  double* partials = nullptr;      // nblocks × kTermSlots
  double* sums = nullptr;          // kTermSlots
  int64_t nblocks = 0;
  const m3d::Grid* sgrid = nullptr;  // the source's grid (Morton query order of the grid NN)
  const m3d::Grid* tgrid = nullptr;  // grid NN: the target's grid (owned by the target cloud)
  int64_t ns_total = 0;  // source-sharded multi-GPU: sources over all ranks (fitness denominator)
  // exchange buffers of the library-driven multi-GPU loops (m3d_icp_*shard_steps), lazily
  // exchange buffers allocated and every rank agreed (comm.cpp), one flag per loop kind: the
  // target-shard loop needs xdk/xcl/xsums, the source-shard loop only xsums
  bool xready_tgt = false;
  bool xready_src = false;
  int64_t* xdk = nullptr;   // ns: d64 keys, MIN-reduced
  int32_t* xcl = nullptr;   // ns: claims, MIN-reduced
  double* xsums = nullptr;  // kTermSlots, SUM-reduced
  // m3d_icp_steps replays: an n-step sequence captured into a HIP graph (api.cpp), one slot per
  // keys_clean state on entry; a slot captures a sequence requested a second time
  hipStream_t cap_stream = nullptr;
  hipGraphExec_t graph[2] = {nullptr, nullptr};
  int32_t graph_n[2] = {-1, -1};
  bool graph_kc_out[2] = {false, false};  // keys_clean after the sequence
  int32_t seen_n[2] = {-1, -1};           // the slot's last request (n)
  bool graph_off = false;                 // a capture failed: plain enqueues from then on
};

// error plumbing ------------------------------------------------------------------------
int m3d_fail(m3d_ctx* ctx, int code, const std::string& msg);

// kernel timing: RAII bracket recording events around one launch when profiling is on
struct KTimer {
  m3d_ctx* ctx;
  int id;
  hipStream_t st;
  hipEvent_t end = nullptr;
  KTimer(m3d_ctx* c, int kid, hipStream_t s);
  ~KTimer();
};
#define M3D_HIP_CHECK(ctx, expr)                                                        \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return m3d_fail((ctx), M3D_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// kernel launchers (defined in the .hip translation units) ------------------------------
namespace m3d {
hipError_t launch_pack_corr(const double* src, const double* tgt, const int32_t* corr, int64_t nc,
                            const double* p_src, const double* p_tgt, double* p64, double* q64,
                            hipStream_t st);
hipError_t launch_sum3(const double* a, int64_t n, double* partial /*[blocks*3]*/, int blocks,
                       hipStream_t st);
hipError_t launch_center_pack(const double* a, int64_t n, int64_t n_pad, const double c[3],
                              float4* out, float pad_value, float* maxnorm_partial, int blocks,
                              int maxinf, hipStream_t st);
// m3d_cloud_create: sum_part (sum3_kernel partials, sum_blocks of them) → mean into cdev (device),
// or the given centre c when sum_part is null; centred fp32 copy + 7 floats per block (max |x|∞,
// lo[3], hi[3])
hipError_t launch_cloud_pack(const double* a, int64_t n, int64_t n_pad, const double* sum_part,
                             int sum_blocks, double* cdev, const double c[3], float4* out, float pad_value,
                             float* part7, int blocks, double* pin_c /*[3], mapped pinned*/,
                             float* pin7 /*[7], mapped pinned*/, hipStream_t st);
struct ScoreMf;
// a4 batches: kabsch3_kernel also writes the MFMA screen's per-hypothesis operands (hyp16) for
// the score launch that follows (thr/mode of that launch; no effect when it will not use them)
struct ScoreFuse {
  const ScoreMf* mf;
  double thr;
  int mode;
};
hipError_t launch_kabsch3(const m3d_corrset* cs, const int32_t* triples, uint64_t seed,
                          int64_t hyp0, int64_t H, double thr_sq, double* T_out, uint8_t* status,
                          HypF32* hypf, const int32_t* done, ZeroArgs z, hipStream_t st,
                          const ScoreFuse* fuse = nullptr);
// one hypothesis, host operands by value (m3d_kabsch3_one / m3d_ransac_score_one)
hipError_t ensure_target_rec(const m3d_cloud* c, hipStream_t st);  // icp.hip: c->rec64
hipError_t build_grid_pts64(const m3d_cloud* c, Grid* g, hipStream_t st);  // icp.hip: g->pts64
hipError_t launch_kabsch3_one(const m3d_corrset* cs, const int32_t* tri, double* T_out,
                              int32_t* status, hipStream_t st);
int64_t count_one_blocks(int64_t nc);
hipError_t launch_count_one(const m3d_corrset* cs, const double* T, double thr, int mode,
                            int32_t* partials, int64_t max_blocks, uint32_t* ticket, int64_t* out,
                            hipStream_t st);
hipError_t launch_hypf_from_T(const m3d_corrset* cs, const double* T, int64_t H, double thr_sq,
                              HypF32* hypf, ZeroArgs z, hipStream_t st);
// MFMA scoring (score_mfma_kernel): per-batch hypothesis operands built from the fp64
// transforms; null hb16 → the fp32 VALU screen (score_kernel)
struct ScoreMf {
  uint4* hb16 = nullptr;  // 6 planes × h_pad (fp16 hi/lo splits of R rows and S·t')
  float* heps = nullptr;  // h_pad: guard band of v = S²(thr² − d²) per hypothesis (< 0: none)
  int64_t h_pad = 0;
};
int64_t score_mf_hpad(int64_t H);
hipError_t launch_corr16(m3d_corrset* cs, hipStream_t st);  // cs->ca16, cs->s16
hipError_t launch_score_prep(const m3d_corrset* cs, const double* T64, int64_t H, double thr,
                             int mode, const ScoreMf& mf, hipStream_t st);
hipError_t launch_score(const m3d_corrset* cs, const HypF32* hypf, int64_t H, int32_t* counts,
                        const double* T64, double thr, int mode, int64_t* stats,
                        const int32_t* done, const ScoreMf& mf, hipStream_t st);
hipError_t launch_select(const int32_t* counts, int64_t h_begin, int64_t n, int64_t nc,
                         int64_t max_iter, int early_stop, double es_thr, double es_conf,
                         const double* T_batch, RansacState* rs, hipStream_t st);
hipError_t launch_ransac_init(RansacState* rs, const int64_t* stats, int done, hipStream_t st);
hipError_t launch_copy_result(const RansacState* rs, int64_t nc, const int64_t* stats,
                              m3d_ransac_result* out_dev, hipStream_t st);
hipError_t launch_ransac_pack_key(const m3d_ransac_result* r, int64_t hyp0, int64_t* key,
                                  hipStream_t st);
// m3d_ransac_run_sharded: buf[0] ← this rank's key (r == null: a failed rank, 0); after the MAX,
// buf[1..19] ← the SUM payload (ransac.hip ransac_shard_pack_kernel)
hipError_t launch_ransac_shard_key(const m3d_ransac_result* r, int64_t hyp0, int64_t* buf,
                                   hipStream_t st);
hipError_t launch_ransac_shard_pack(const m3d_ransac_result* r, int64_t hyp0, int64_t* buf,
                                    hipStream_t st);
// target-shard loop pieces (api.cpp): the NN + this shard's winners of source slots [q0, q1), and
// whether the loop's NN can run on a slot range (grid NN; brute force with MFMA tiles in slot order)
int icp_shard_nn_range(m3d_icp* s, int64_t off, int64_t q0, int64_t q1, int64_t* dkeys, hipStream_t st);
bool icp_nn_range_ok(const m3d_icp* s);

// ICP
// [q0, q1): the sources (slots; brute force: positions of s->qorder) one launch evaluates,
// q1 < 0 = all (the target-shard loop splits its sources to overlap the exchange, comm.cpp)
hipError_t launch_icp_keyinit(const m3d_icp* s, int64_t shard_offset, hipStream_t st, int64_t q0 = 0,
                              int64_t q1 = -1);
hipError_t launch_icp_nn(const m3d_icp* s, int64_t shard_offset, bool self_seed, hipStream_t st,
                         int64_t q0 = 0, int64_t q1 = -1);
hipError_t launch_icp_reduce(const m3d_icp* s, double* sums, hipStream_t st);
hipError_t launch_icp_reduce_solve(const m3d_icp* s, hipStream_t st);
// claim/dmin: target-shard exchange results (m3d_icp_shard_claim), or null
hipError_t launch_icp_terms_mode(const m3d_icp* s, int64_t off, const int32_t* claim,
                                 const int64_t* dmin, hipStream_t st);
hipError_t launch_icp_terms_reduce(const m3d_icp* s, int64_t off, const int32_t* claim,
                                   const int64_t* dmin, double* sums, bool reset_keys,
                                   hipStream_t st);
hipError_t launch_shard_winner(const m3d_icp* s, int64_t off, int64_t* dkey, hipStream_t st,
                               int64_t q0 = 0, int64_t q1 = -1);
hipError_t launch_shard_claim(const m3d_icp* s, const int64_t* dmin, int32_t* claim, hipStream_t st);
hipError_t launch_icp_solve(const m3d_icp* s, const double* sums, hipStream_t st);
// grid over xyz32[0, n) with cell ≈ `cell`: asynchronous when `lohi` (per-axis min[3], max[3] of
// the points) is given, else one sync for the bounds; temporaries from `ta` (null: hipMalloc)
hipError_t grid_build(const float4* xyz32, int64_t n, double cell, hipStream_t st, Grid* g,
                      TmpArena* ta = nullptr, const float* lohi = nullptr);
// g->n_occ, counted on first use (one sync)
// pin_dev / pin_host: 16 B of mapped pinned memory the counts are written to (no device-to-host
// copy), or null (a copy into host memory)
hipError_t grid_occupancy(Grid* g, TmpArena* ta, hipStream_t st, unsigned long long* pin_dev = nullptr,
                          const unsigned long long* pin_host = nullptr);
void grid_free(Grid* g);
// prev/dprev/tgt32/nt_shard: seed each query with seed_key (nnkey.h); prev == nullptr: no seeds
// qgrid: the query cloud's Morton-slot grid (its Morton-ordered points, morton_source)
hipError_t launch_grid_nn(const float4* src32, int64_t ns, const Grid* qgrid, const Grid* g,
                          int64_t off, const IcpState* s, int64_t* keys, uint32_t* near2,
                          const int32_t* prev, const int64_t* dprev, const float4* tgt32, int64_t nt_shard,
                          hipStream_t st, int64_t q0 = 0, int64_t q1 = -1, int32_t* hlist = nullptr,
                          uint32_t* hcnt = nullptr, int32_t cand_cap = 0, const double* src64 = nullptr,
                          const double* tgt64 = nullptr, int32_t hcap = 0, int32_t xchunk = 0);
// the ICP source's Morton-slot copy (out, gout freshly allocated structs): grid.hip morton_source
hipError_t morton_source(const m3d_cloud* src, double cell, m3d_cloud* out, Grid* gout, TmpArena* ta,
                         hipStream_t st);
// dst[slot[k]] = v[k], k < n (slot-ordered loop arrays → the caller's source order)
// correspondence pairs (i, v[i]) for v[i] >= 0 in increasing i; cnt: (n + 1023) / 1024 + 1 ints of
// scratch, the total in cnt[(n + 1023) / 1024] (cnt[0] when n == 0)
hipError_t launch_corr_pairs(const int32_t* v, int64_t n, int32_t* cnt, int32_t* pairs, hipStream_t st);
hipError_t launch_scatter_i32(const int32_t* v, const int32_t* slot, int64_t n, int32_t* dst,
                              hipStream_t st);
hipError_t launch_keys_to_idx(const int64_t* keys, int64_t n, int32_t* idx, hipStream_t st);
hipError_t launch_icp_set_T(const m3d_icp* s, const double* T_dev, hipStream_t st);
// a6 batched validation: states[k] ← evaluation state of T[list[k]] (icp_set_T semantics), then
// out[2k], out[2k + 1] = (correspondence count, Σd²) of hypothesis k (grid.hip validate_kernel);
// part: validate_blocks(ns) × 2 doubles per hypothesis of scratch
hipError_t launch_val_states(const m3d_icp* s, const double* T_dev, const int32_t* list, int64_t n,
                             IcpState* states, hipStream_t st);
int64_t validate_blocks(int64_t ns);
hipError_t launch_validate(const Grid* qgrid, int64_t ns, const double* src64, const Grid* g,
                           const double* tgt64, int64_t nt, const IcpState* states, int64_t nhyp,
                           double* part, double* out, hipStream_t st);
hipError_t build_mfma_tiles(const m3d_cloud* c, Grid* g, hipStream_t st);

// preprocessing (prep.hip) and feature matching (feat.hip)
size_t voxel_scratch_bytes(int64_t n);  // device scratch voxel_down_sample needs for n points
hipError_t voxel_down_sample(const double* xyz, const double* nrm, int64_t n, double voxel,
                             double* out_xyz, double* out_nrm, int64_t* out_n, void* scratch,
                             hipStream_t st, std::string* why);
// hybrid (radius + max_nn) neighbour lists; gf / hfine: optional first-stage grid and radius
// (hybrid_fine_radius), the result is the same list
double hybrid_fine_radius(const Grid* g, double radius, int k);
hipError_t hybrid_search(const m3d_cloud* c, const Grid* g, double radius, int k, int32_t* idx,
                         double* d2, int32_t* cnt, hipStream_t st, const Grid* gf = nullptr,
                         double hfine = 0.0);
hipError_t launch_normals(const m3d_cloud* c, const int32_t* nbr, int k, const int32_t* cnt,
                          const double* prev, double* out, hipStream_t st);
hipError_t launch_acos_probe(const double* u, int64_t n, double* out, int mode, hipStream_t st);
hipError_t launch_fpfh(const m3d_cloud* c, const double* nrm, const int32_t* nbr, const double* d2,
                       int k, const int32_t* cnt, double* spfh, double* out, hipStream_t st);
hipError_t feature_nn(const double* fq, int64_t nq, const double* fr, int64_t nr, int32_t* out,
                      hipStream_t st);
hipError_t feature_correspondences(const double* fs, int64_t ns, const double* ft, int64_t nt,
                                   int mutual, double ratio, int32_t* corr_out, int64_t* n_out,
                                   hipStream_t st);
// a6 exit rule: count[k] = #{c : |T_k·p_c − q_c|² < max_corr²}, T_k = T_all + 16·list[k], k < n
hipError_t launch_corres_inlier(const double* src, const double* tgt, const int32_t* corr, int64_t nc,
                                const double* T_all, const int32_t* list, int64_t n, double max_corr,
                                int32_t* count, hipStream_t st);
hipError_t launch_feat_hyp(const double* src, const double* tgt, const int32_t* corr, int64_t nc,
                           uint64_t seed, int64_t H, double edge, double dist, double* T_out,
                           int32_t* pass, hipStream_t st);
}  // namespace m3d
