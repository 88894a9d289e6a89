// ransac.hip — RANSAC hypothesis generation and inlier scoring for gfx950.
//
// Reference path (all CPU, numpy fp64):
//   compute_step_transformation  src/matcher/ransac.py:104-192   → kabsch3_kernel
//   evaluate_inlier_ratio[_fast] src/matcher/ransac.py:195-277   → score_mfma_kernel (matrix cores,
//                                                                   see "MFMA screen" below) or the
//                                                                   fp32 VALU score_kernel
//   step-RANSAC loop             _visualize_matcher.py:343-470   → select_kernel (batched, on device)
//
// fp32 VALU scoring design (score_kernel: the fallback when the MFMA operands do not apply):
//   * One lane holds kScoreK = 8 correspondences (centred fp32, 6 VGPRs each) for the whole block;
//     a block of 4 waves covers 2048 correspondences and sweeps 64 hypotheses.
//   * The block's 64 hypothesis blocks (R, t', guard band: 64 B each) are staged in LDS and read
//     with broadcast ds_read_b128 → VGPR operands (SGPR operands cost 1.65x issue time).
//   * Per (hypothesis, correspondence): 12 ops for d = R p + t' − q, 3 for d², 2 compares.  The
//     compares are folded into wave masks (v_cmp → s_bcnt1 → s_add): counting is scalar work.
//   * Exactness: the fp32 screen counts d² < lo (certainly inside) and flags lo ≤ d² < hi; lo/hi
//     bracket thr² by a rounding-error bound.  A flagged 64-pair group is
//     re-evaluated in fp64 with numpy's operation order inside the same kernel (rare branch), so
//     the counts equal an fp64 evaluation of the reference formula.
//   * Counts are integers: atomics are exact and order-independent → deterministic results.
#include <float.h>
#include <stdlib.h>

#include <hipcub/hipcub.hpp>

#include "lds_dma.h"
#include "linalg.h"
#include "m3d_internal.h"

namespace m3d {

constexpr int kScoreK = 8;
constexpr int kScoreBlock = 256;
constexpr int kScoreHyps = 64;
constexpr int kChunk = kScoreK * kWave;  // 512 correspondences per wave
constexpr int kBlockCorr = kChunk * 4;   // 2048 per block
constexpr double kU32 = 5.9604644775390625e-08;  // 2^-24

// ------------------------------------------------------------------------------- packing
__global__ void pack_corr_kernel(const double* __restrict__ src, const double* __restrict__ tgt,
                                 const int32_t* __restrict__ corr, int64_t nc,
                                 const double* __restrict__ p_src, const double* __restrict__ p_tgt,
                                 double* __restrict__ p64, double* __restrict__ q64) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc) return;
  const double* a;
  const double* b;
  if (corr != nullptr) {
    a = src + 3 * (int64_t)corr[2 * i];
    b = tgt + 3 * (int64_t)corr[2 * i + 1];
  } else {
    a = p_src + 3 * i;
    b = p_tgt + 3 * i;
  }
  for (int k = 0; k < 3; ++k) {
    p64[3 * i + k] = a[k];
    q64[3 * i + k] = b[k];
  }
}

// deterministic per-block partial sums of an n×3 f64 array (fixed grid, fixed tree)
__global__ __launch_bounds__(256) void sum3_kernel(const double* __restrict__ a, int64_t n,
                                                   double* __restrict__ partial) {
  __shared__ double s[3][256];
  double acc[3] = {0.0, 0.0, 0.0};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    for (int k = 0; k < 3; ++k) acc[k] += a[3 * i + k];
  for (int k = 0; k < 3; ++k) s[k][threadIdx.x] = acc[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < 3; ++k) s[k][threadIdx.x] += s[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int k = 0; k < 3; ++k) partial[3 * blockIdx.x + k] = s[k][0];
}

// centre + convert to padded float4; per-block max of ‖x_c‖₂ (or |x_c|∞)
__global__ __launch_bounds__(256) void center_pack_kernel(const double* __restrict__ a, int64_t n,
                                                          int64_t n_pad, double c0, double c1,
                                                          double c2, float4* __restrict__ out,
                                                          float pad_value,
                                                          float* __restrict__ maxpart, int maxinf) {
  __shared__ float s[256];
  float m = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pad;
       i += (int64_t)gridDim.x * 256) {
    float4 v;
    if (i < n) {
      double x = a[3 * i] - c0, y = a[3 * i + 1] - c1, z = a[3 * i + 2] - c2;
      const float fx = (float)x, fy = (float)y, fz = (float)z;
      // w = |x̃|² of the fp32-rounded coordinates (fp64, one rounding): the NN screen's |t|²
      const double w = (double)fx * fx + (double)fy * fy + (double)fz * fz;
      v = make_float4(fx, fy, fz, (float)w);
      double mm = maxinf ? fmax(fabs(x), fmax(fabs(y), fabs(z))) : sqrt(x * x + y * y + z * z);
      m = fmaxf(m, (float)mm * (1.0f + 1e-6f));
    } else {
      v = make_float4(pad_value, pad_value, pad_value, 3.0f * pad_value * pad_value);
    }
    out[i] = v;
  }
  s[threadIdx.x] = m;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) s[threadIdx.x] = fmaxf(s[threadIdx.x], s[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) maxpart[blockIdx.x] = s[0];
}

// Cloud packing (m3d_cloud_create): the mean from sum3_kernel's partials reduced on the device by
// one wave in a fixed order (lane l adds partials l, l + 64, …, then a fixed xor butterfly; every
// lane ends with the same bits), ÷ n; then the centred fp32 copy with, per block, max |x_c|∞ and
// the per-axis min / max of the fp32 coordinates (the grid bounds, grid.hip minmax3_kernel's
// values) — one host sync for the whole cloud.  (Round 4 summed the partials in one thread:
// 384 dependent loads, 13-19 µs per cloud.)
__global__ __launch_bounds__(64) void mean3_final_kernel(const double* __restrict__ part, int blocks, int64_t n,
                                                         double* __restrict__ c) {
  const int l = threadIdx.x;
  double o[3] = {0.0, 0.0, 0.0};
  for (int b = l; b < blocks; b += 64)
    for (int k = 0; k < 3; ++k) o[k] += part[3 * b + k];
#pragma unroll
  for (int m = 32; m > 0; m >>= 1)
    for (int k = 0; k < 3; ++k) o[k] += __shfl_xor(o[k], m, 64);
  if (l < 3) c[l] = o[l] / (double)n;
}

__global__ __launch_bounds__(256) void cloud_pack_kernel(const double* __restrict__ a, int64_t n,
                                                         int64_t n_pad, const double* __restrict__ cdev,
                                                         double c0, double c1, double c2,
                                                         float4* __restrict__ out, float pad_value,
                                                         float* __restrict__ part7) {
  __shared__ float s[7][256];
  if (cdev != nullptr) {
    c0 = cdev[0];
    c1 = cdev[1];
    c2 = cdev[2];
  }
  float m = 0.0f, lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * 256) {
    float4 v;
    if (i < n) {
      double x = a[3 * i] - c0, y = a[3 * i + 1] - c1, z = a[3 * i + 2] - c2;
      const float fx = (float)x, fy = (float)y, fz = (float)z;
      const double w = (double)fx * fx + (double)fy * fy + (double)fz * fz;  // as center_pack_kernel
      v = make_float4(fx, fy, fz, (float)w);
      m = fmaxf(m, (float)fmax(fabs(x), fmax(fabs(y), fabs(z))) * (1.0f + 1e-6f));
      lo[0] = fminf(lo[0], fx);
      lo[1] = fminf(lo[1], fy);
      lo[2] = fminf(lo[2], fz);
      hi[0] = fmaxf(hi[0], fx);
      hi[1] = fmaxf(hi[1], fy);
      hi[2] = fmaxf(hi[2], fz);
    } else {
      v = make_float4(pad_value, pad_value, pad_value, 3.0f * pad_value * pad_value);
    }
    out[i] = v;
  }
  s[0][threadIdx.x] = m;
  for (int k = 0; k < 3; ++k) {
    s[1 + k][threadIdx.x] = lo[k];
    s[4 + k][threadIdx.x] = hi[k];
  }
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      s[0][threadIdx.x] = fmaxf(s[0][threadIdx.x], s[0][threadIdx.x + w]);
      for (int k = 0; k < 3; ++k) {
        s[1 + k][threadIdx.x] = fminf(s[1 + k][threadIdx.x], s[1 + k][threadIdx.x + w]);
        s[4 + k][threadIdx.x] = fmaxf(s[4 + k][threadIdx.x], s[4 + k][threadIdx.x + w]);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x < 7) part7[7 * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

// The cloud's host-side summary straight into mapped pinned memory (no device-to-host copy, the
// host reads it after one stream sync): the centre (3 f64, when computed on the device) and the
// max / min / max of the block partials — order-free, so the same bits as the host fold it replaces.
__global__ __launch_bounds__(256) void cloud_summary_kernel(const float* __restrict__ part7, int blocks,
                                                            const double* __restrict__ cdev,
                                                            double* __restrict__ out_c, float* __restrict__ out7) {
  __shared__ float s[7][256];
  float v[7] = {0.0f, FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int b = threadIdx.x; b < blocks; b += 256) {
    v[0] = fmaxf(v[0], part7[7 * b]);
    for (int k = 1; k < 4; ++k) v[k] = fminf(v[k], part7[7 * b + k]);
    for (int k = 4; k < 7; ++k) v[k] = fmaxf(v[k], part7[7 * b + k]);
  }
  for (int k = 0; k < 7; ++k) s[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      s[0][threadIdx.x] = fmaxf(s[0][threadIdx.x], s[0][threadIdx.x + w]);
      for (int k = 1; k < 4; ++k) s[k][threadIdx.x] = fminf(s[k][threadIdx.x], s[k][threadIdx.x + w]);
      for (int k = 4; k < 7; ++k) s[k][threadIdx.x] = fmaxf(s[k][threadIdx.x], s[k][threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 7) out7[threadIdx.x] = s[threadIdx.x][0];
  if (cdev != nullptr && threadIdx.x < 3) out_c[threadIdx.x] = cdev[threadIdx.x];
}

// ------------------------------------------------------------------------------- sampler
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Counter-based sampler; oracle/ransac_oracle.py::native_triples restates it bit for bit.
__device__ void native_triple(uint64_t seed, int64_t h, int64_t nc, int out[3]) {
  const uint64_t base = splitmix64(seed ^ ((uint64_t)h * 0x9E3779B97F4A7C15ull));
  int got = 0;
  for (uint64_t k = 0; got < 3 && k < (1u << 20); ++k) {
    const uint64_t v = splitmix64(base + k);
    const int idx = (int)(((v >> 32) * (uint64_t)nc) >> 32);
    bool dup = false;
    for (int j = 0; j < got; ++j) dup |= (out[j] == idx);
    if (!dup) out[got++] = idx;
  }
  for (; got < 3; ++got) out[got] = got;  // unreachable for nc >= 3
}

// ------------------------------------------------------------------------------- Kabsch
struct GuardParams {
  double cs[3], ct[3];
  double pinf;  // max |p_c|∞
  double qinf;  // max |q_c|∞
  double thr_sq;
};

// fp32 screen block for transform T (row-major 4×4, world frame) with a proven guard band.
__device__ HypF32 make_hypf(const double* T, const GuardParams& g) {
  HypF32 hp;
  double tp[3], rowl1 = 0.0, tinf = 0.0;
  for (int i = 0; i < 3; ++i) {
    const double* r = T + 4 * i;
    tp[i] = fma(r[2], g.cs[2], fma(r[1], g.cs[1], r[0] * g.cs[0])) + r[3] - g.ct[i];
    for (int j = 0; j < 3; ++j) hp.r[3 * i + j] = (float)r[j];
    hp.t[i] = (float)tp[i];
    rowl1 = fmax(rowl1, fabs(r[0]) + fabs(r[1]) + fabs(r[2]));
    tinf = fmax(tinf, fabs(tp[i]));
  }
  // Per-component error of the fp32 evaluation d = fma(r0,p0,fma(r1,p1,fma(r2,p2,t'−q)))
  // (DESIGN.md §3.2): inputs (p, q, R, t' rounded to fp32) 2S + |t'| + |q|, the four roundings
  // |t'−q| + |a1| + |a2| + |d| ≤ 2S + 3(|t'| + |q|) + thr  →  E ≤ u(4S + 4|t'| + 4|q| + thr),
  // S = Σ|r_j||p_j| ≤ ‖r‖₁|p|∞.  (1 + 1e-3) absorbs the O(u²) terms.
  const double thr = sqrt(g.thr_sq);
  const double E = kU32 * (4.0 * rowl1 * g.pinf + 4.0 * tinf + 4.0 * g.qinf + thr) * 1.001;
  double eps = 3.0 * kU32 * (thr + 1.7320508075688772 * E) * (thr + 1.7320508075688772 * E) +
               2.0 * 1.7320508075688772 * E * thr + 3.0 * E * E;
  eps = 1.25 * eps + 4.0 * DBL_EPSILON * g.thr_sq;
  double lo = g.thr_sq - eps, hi = g.thr_sq + eps;
  if (!(lo > 0.0)) lo = 0.0;
  hp.lo = __double2float_rd(lo);
  hp.hi = __double2float_ru(hi);
  if (!isfinite(hp.hi)) hp.hi = FLT_MAX;
  hp.pad[0] = hp.pad[1] = 0.0f;
  return hp;
}

// Zero the per-batch counts in the kernel that precedes the screen (saves a memset launch).
__device__ __forceinline__ void zero_scoring_state(const ZeroArgs& z, int64_t h, int64_t H) {
  if (h < H && z.counts) z.counts[h] = 0;
}

struct Mf16Params {
  double cs[3], ct[3];
  double S, pinf, qinf, thr_sq;
};

// hyp16_kernel's per-hypothesis body folded into kabsch3_kernel (the transform is already in
// registers there): one launch less per RANSAC batch when the MFMA screen scores it
struct Hyp16Fuse {
  Mf16Params m;
  uint4* hb16;
  float* heps;
  int64_t h_pad;
  int on;
};
// (defined with the MFMA screen below; declared inline here as it is there)
__device__ __forceinline__ void hyp16_one(const double* T, bool valid, int64_t j, int64_t h_pad,
                                          const Mf16Params& m, uint4* __restrict__ hb16,
                                          float* __restrict__ heps);

__global__ __launch_bounds__(256) void kabsch3_kernel(const double* __restrict__ p64,
                                                      const double* __restrict__ q64, int64_t nc,
                                                      const int32_t* __restrict__ triples,
                                                      uint64_t seed, int64_t hyp0, int64_t H,
                                                      GuardParams g, double* __restrict__ T_out,
                                                      uint8_t* __restrict__ status,
                                                      HypF32* __restrict__ hypf,
                                                      const int32_t* __restrict__ done,
                                                      ZeroArgs z, Hyp16Fuse hf) {
  if (done != nullptr && *done) return;
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  zero_scoring_state(z, h, H);
  if (h >= H) {  // padding hypotheses of the MFMA operands
    if (hf.on && h < hf.h_pad) hyp16_one(nullptr, false, h, hf.h_pad, hf.m, hf.hb16, hf.heps);
    return;
  }
  double T[16];
  int st = M3D_HYP_OK;
  if (nc < 3) {  // ransac.py:139-140
    for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
    st = M3D_HYP_DEGENERATE;
  } else {
    int id[3];
    if (triples != nullptr) {
      for (int k = 0; k < 3; ++k) {
        int v = triples[3 * h + k];
        id[k] = (v < 0 || v >= nc) ? 0 : v;
      }
    } else {
      native_triple(seed, hyp0 + h, nc, id);
    }
    double ps[3][3], qs[3][3];
    for (int k = 0; k < 3; ++k)
      for (int c = 0; c < 3; ++c) {
        ps[k][c] = p64[3 * (int64_t)id[k] + c];
        qs[k][c] = q64[3 * (int64_t)id[k] + c];
      }
    st = kabsch3(ps, qs, T) ? M3D_HYP_NONFINITE : M3D_HYP_OK;
  }
  if ((reinterpret_cast<uintptr_t>(T_out) & 15u) == 0) {  // 8 × 16-B stores (library buffers)
    double2* To = reinterpret_cast<double2*>(T_out + 16 * h);
#pragma unroll
    for (int k = 0; k < 8; ++k) To[k] = make_double2(T[2 * k], T[2 * k + 1]);
  } else {  // a caller's buffer at an 8-B offset (m3d_kabsch3)
    for (int k = 0; k < 16; ++k) T_out[16 * h + k] = T[k];
  }
  if (status != nullptr) status[h] = (uint8_t)st;
  // the fp32 VALU screen's block: not written when the MFMA screen scores this batch (hf.on)
  if (hypf != nullptr) hypf[h] = make_hypf(T, g);
  if (hf.on) hyp16_one(T, true, h, hf.h_pad, hf.m, hf.hb16, hf.heps);
}

__global__ __launch_bounds__(256) void hypf_from_T_kernel(const double* __restrict__ T, int64_t H,
                                                          GuardParams g,
                                                          HypF32* __restrict__ hypf, ZeroArgs z) {
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  zero_scoring_state(z, h, H);
  if (h < H) hypf[h] = make_hypf(T + 16 * h, g);
}

// ------------------------------------------------------------------------------- fp64 recheck
// numpy order (verified in the build container): p @ R.T is fma(r2,z,fma(r1,y,r0*x)), then + t,
// (.)**2 summed left to right; evaluate_inlier_ratio takes sqrt of the same sum.
__device__ __forceinline__ bool exact_inlier(const double* T, const double* p, const double* q,
                                             double thr, int mode) {
  const double x = fma(T[2], p[2], fma(T[1], p[1], T[0] * p[0])) + T[3];
  const double y = fma(T[6], p[2], fma(T[5], p[1], T[4] * p[0])) + T[7];
  const double z = fma(T[10], p[2], fma(T[9], p[1], T[8] * p[0])) + T[11];
  const double dx = x - q[0], dy = y - q[1], dz = z - q[2];
  const double s = (dx * dx + dy * dy) + dz * dz;
  return mode == M3D_SCORE_SQUARED ? (s < thr) : (sqrt(s) < thr);
}

// ------------------------------------------------------------------------------- fp32 screen
struct ExactArgs {
  const double* T64;  // [H][16] fp64 transforms of the batch
  const double* p64;  // [nc][3]
  const double* q64;  // [nc][3]
  int64_t nc;
  double thr;
  int mode;
  int64_t* stats;  // [0] pairs re-evaluated in fp64
};

__global__ __launch_bounds__(kScoreBlock) void score_kernel(
    const float4* __restrict__ p32, const float4* __restrict__ q32,
    const float4* __restrict__ hyp4, int64_t H, int64_t hbase, int32_t* __restrict__ counts,
    ExactArgs ex, const int32_t* __restrict__ done) {
  if (done != nullptr && *done) return;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int64_t chunk = (int64_t)blockIdx.x * 4 + wave;
  float px[kScoreK], py[kScoreK], pz[kScoreK], qx[kScoreK], qy[kScoreK], qz[kScoreK];
#pragma unroll
  for (int k = 0; k < kScoreK; ++k) {
    const int64_t i = chunk * kChunk + k * kWave + lane;  // padded: always in range
    const float4 a = p32[i];
    const float4 b = q32[i];
    px[k] = a.x; py[k] = a.y; pz[k] = a.z;
    qx[k] = b.x; qy[k] = b.y; qz[k] = b.z;
  }
  const int64_t h0 = hbase + (int64_t)blockIdx.y * kScoreHyps;
  const int nh = (int)((H - h0) < kScoreHyps ? (H - h0) : kScoreHyps);
  int cnt = 0;
  // The block's 64 hypothesis blocks (4 KB) are staged in LDS once; each wave reads one with
  // four broadcast ds_read_b128 into VGPRs, so the FMAs have no SGPR operand (an SGPR source
  // costs 1.65x issue time on gfx950, tools/ubench_valu.hip).
  __shared__ float4 hs[kScoreHyps * 4];
  {
    const int64_t hh = h0 + threadIdx.x / 4;
    hs[threadIdx.x] = hh < H ? hyp4[hh * 4 + (threadIdx.x & 3)] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  for (int hl = 0; hl < nh; ++hl) {
    const float4 ha = hs[4 * hl], hb = hs[4 * hl + 1], hc = hs[4 * hl + 2], hd = hs[4 * hl + 3];
    const float r0 = ha.x, r1 = ha.y, r2 = ha.z;
    const float r3 = ha.w, r4 = hb.x, r5 = hb.y;
    const float r6 = hb.z, r7 = hb.w, r8 = hc.x;
    const float t0 = hc.y, t1 = hc.z, t2 = hc.w;
    const float lo_t = hd.x, hi_t = hd.y;
    // all K distances first (independent chains), then the compares into independent masks,
    // so the VALU→SGPR→SALU hand-offs overlap instead of serialising on one mask register
    float d2[kScoreK];
#pragma unroll
    for (int k = 0; k < kScoreK; ++k) {
      const float dx = fmaf(r0, px[k], fmaf(r1, py[k], fmaf(r2, pz[k], t0 - qx[k])));
      const float dy = fmaf(r3, px[k], fmaf(r4, py[k], fmaf(r5, pz[k], t1 - qy[k])));
      const float dz = fmaf(r6, px[k], fmaf(r7, py[k], fmaf(r8, pz[k], t2 - qz[k])));
      d2[k] = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
    }
    uint64_t mlo[kScoreK], mband[kScoreK];
#pragma unroll
    for (int k = 0; k < kScoreK; ++k) {
      mlo[k] = __ballot(d2[k] < lo_t);
      mband[k] = __ballot(d2[k] < hi_t);
    }
    uint32_t lo = 0;
    uint64_t band = 0;
#pragma unroll
    for (int k = 0; k < kScoreK; ++k) {
      lo += (uint32_t)__popcll(mlo[k]);
      band |= mband[k] & ~mlo[k];
    }
    if (band != 0) {
      // rare (wave-uniform): a 64-pair group holds a pair inside the guard band — re-evaluate
      // that group in fp64 with numpy's operation order and replace its screen count.  The
      // dependent loads stall only this wave; the SIMD's other waves keep the VALU busy.
      double Th[12];
#pragma unroll
      for (int k = 0; k < 12; ++k) Th[k] = ex.T64[16 * (h0 + hl) + k];
      int groups = 0;
#pragma unroll
      for (int k = 0; k < kScoreK; ++k) {
        if (mband[k] & ~mlo[k]) {
          const int64_t i = chunk * kChunk + k * kWave + lane;
          const bool in = i < ex.nc && exact_inlier(Th, ex.p64 + 3 * i, ex.q64 + 3 * i, ex.thr, ex.mode);
          lo += (uint32_t)__popcll(__ballot(in)) - (uint32_t)__popcll(mlo[k]);
          ++groups;
        }
      }
      if (lane == 0 && ex.stats)
        atomicAdd((unsigned long long*)&ex.stats[0], (unsigned long long)(groups * kWave));
    }
    cnt = (lane == hl) ? (int)lo : cnt;
  }
  __shared__ int red[4][kWave];
  red[wave][lane] = cnt;
  __syncthreads();
  if (threadIdx.x < nh) {
    const int t = threadIdx.x;
    atomicAdd(&counts[h0 + t], red[0][t] + red[1][t] + red[2][t] + red[3][t]);
  }
}

// ------------------------------------------------------------------------------- MFMA screen
// The residual VECTOR d = R p_c + t' − q_c per (correspondence, hypothesis) is three rank-13
// contractions, one v_mfma_f32_32x32x16_f16 per component and 32 × 32 block, from fp16 hi/lo
// splits of the power-of-two-scaled operands (S = cs->s16, |S·p_c|∞, |S·q_c|∞ ≤ 1024):
//   A (correspondence row i, component c): [ph0, pl0, ph0, ph1, pl1, ph1, ph2, pl2 |
//                                           ph2, 1, 1, qh_c, ql_c, 0, 0, 0]
//   B (hypothesis column j, component c):  [Rh0, Rh0, Rl0, Rh1, Rh1, Rl1, Rh2, Rh2 |
//                                           Rl2, th_c, tl_c, −1, −1, 0, 0, 0]
// (R = row c of the rotation, t = S·t'_c; Rl·pl is dropped).  The VALU then forms
// v = S²thr² − dx² − dy² − dz² (3 packed FMAs per 2 pairs) and counts sign bits per lane (a lane
// owns one hypothesis column): 3.5 VALU per pair against ≈ 9 for the fp32 screen.  Exactness:
// |v − S²(thr² − d²)| < ε_j (per hypothesis, hyp16_kernel: split remainders, the MFMA's fp32
// accumulation of 13 exact products with cancellation, the three FMA roundings, thr² rounding
// and the fp64 reference's own rounding), so pairs with |v| ≥ ε_j are classified exactly and the
// rest are re-evaluated in fp64 with numpy's operation order (exact_inlier) — the counts equal
// the fp32 screen's and the reference formula's.
typedef _Float16 s_half8 __attribute__((ext_vector_type(8)));
typedef float s_floatx16 __attribute__((ext_vector_type(16)));
typedef float s_float2 __attribute__((ext_vector_type(2)));
union SH8 {
  uint4 u;
  s_half8 h;
};

constexpr int kSGroups = 2;                   // 32-hypothesis groups per wave
constexpr int kSBlock = 512;                  // 8 waves
template <int kSMG>
constexpr int shyps() { return (kSBlock / 64) * kSMG * 32; }  // hypotheses per block
constexpr int kSHypPad = shyps<4>();          // batch padding: a multiple of every variant's
constexpr int kSTile = 512;                   // correspondences per LDS tile
static_assert(kSTile % 64 == 0 && (4 * kSTile) % 512 == 0, "a wave stages 64 consecutive rows");
constexpr double kU16 = 4.8828125e-04;        // 2^-11
constexpr double kSig16 = 2.98023223876953125e-08;  // 2^-25: half the fp16 subnormal spacing
constexpr float kPadQ = 30000.0f;             // padded rows: q far away (exact in fp16)
constexpr float kFarT = 16384.0f;             // hypotheses that cannot have inliers
constexpr int kSQueue = 1024;                 // guard-band pairs queued per block (8 KB LDS)

__device__ __forceinline__ void split16d(double x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (double)hi);
}

__global__ __launch_bounds__(256) void corr16_kernel(const double* __restrict__ p64,
                                                     const double* __restrict__ q64, int64_t nc,
                                                     int64_t nc_pad, double cs0, double cs1,
                                                     double cs2, double ct0, double ct1,
                                                     double ct2, double S,
                                                     uint4* __restrict__ ca16) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nc_pad) return;
  const _Float16 one = (_Float16)1.0f, zero = (_Float16)0.0f;
  SH8 P, Q[3];
  if (i < nc) {
    const int64_t r = i;
    _Float16 h[3], l[3];
    split16d(S * (p64[3 * r] - cs0), h[0], l[0]);
    split16d(S * (p64[3 * r + 1] - cs1), h[1], l[1]);
    split16d(S * (p64[3 * r + 2] - cs2), h[2], l[2]);
    P.h = s_half8{h[0], l[0], h[0], h[1], l[1], h[1], h[2], l[2]};
    const double qc[3] = {q64[3 * r] - ct0, q64[3 * r + 1] - ct1, q64[3 * r + 2] - ct2};
    for (int c = 0; c < 3; ++c) {
      _Float16 qh, ql;
      split16d(S * qc[c], qh, ql);
      Q[c].h = s_half8{h[2], one, one, qh, ql, zero, zero, zero};
    }
  } else {
    P.u = make_uint4(0, 0, 0, 0);
    for (int c = 0; c < 3; ++c)
      Q[c].h = s_half8{zero, one, one, (_Float16)kPadQ, zero, zero, zero, zero};
  }
  ca16[i] = P.u;
  for (int c = 0; c < 3; ++c) ca16[(1 + c) * nc_pad + i] = Q[c].u;
}

// B operands + guard band of hypotheses [0, h_pad) of a batch (fp64 transforms T64).
// hypothesis j's B operands + guard band from its fp64 transform T (valid: j < H; the padding
// hypotheses get far operands)
__device__ __forceinline__ void hyp16_one(const double* T, bool valid, int64_t j, int64_t h_pad,
                                          const Mf16Params& m, uint4* __restrict__ hb16,
                                          float* __restrict__ heps) {
  const _Float16 zero = (_Float16)0.0f, mone = (_Float16)-1.0f;
  SH8 B0[3], B1[3];
  float eps = -1.0f;  // no guard band: v is never inside (−1, 1)·ε
  bool far = true, general = false;
  if (valid) {
    double tp[3], rowl1 = 0.0, tinf = 0.0;
    bool finite = true;
    for (int c = 0; c < 3; ++c) {
      const double* r = T + 4 * c;
      tp[c] = fma(r[2], m.cs[2], fma(r[1], m.cs[1], r[0] * m.cs[0])) + r[3] - m.ct[c];
      rowl1 = fmax(rowl1, fabs(r[0]) + fabs(r[1]) + fabs(r[2]));
      tinf = fmax(tinf, fabs(tp[c]));
      finite = finite && isfinite(r[0]) && isfinite(r[1]) && isfinite(r[2]) && isfinite(tp[c]);
    }
    const double thr = sqrt(m.thr_sq);
    // |d|∞ ≥ |t'|∞ − ‖R‖∞|p_c|∞ − |q_c|∞: beyond thr (with margin) no correspondence is an
    // inlier, in any arithmetic — such a hypothesis gets count 0 (NaN transforms too, as the
    // fp32 screen and numpy's comparisons give)
    far = !finite || tinf > 1.01 * (rowl1 * m.pinf + m.qinf + thr) + 1e-30;
    // not a rotation (only m3d_ransac_score takes arbitrary transforms): no fp16 operands for
    // R — every pair of the hypothesis goes to the fp64 re-evaluation
    general = !far && rowl1 > 2.0;
    if (general) {
      for (int c = 0; c < 3; ++c) {
        B0[c].u = make_uint4(0, 0, 0, 0);
        B1[c].h = s_half8{zero, zero, zero, mone, mone, zero, zero, zero};
      }
      eps = FLT_MAX;  // v = S²thr² − |S·q_c|² is finite: |v| < ε for every pair
    } else if (!far) {
      const double S = m.S;
      for (int c = 0; c < 3; ++c) {
        const double* r = T + 4 * c;
        _Float16 rh[3], rl[3], th, tl;
        for (int k = 0; k < 3; ++k) split16d(r[k], rh[k], rl[k]);
        split16d(S * tp[c], th, tl);
        B0[c].h = s_half8{rh[0], rh[0], rl[0], rh[1], rh[1], rl[1], rh[2], rh[2]};
        B1[c].h = s_half8{rl[2], th, tl, mone, mone, zero, zero, zero};
      }
      // per-component error of the scaled d (see the section comment): products exact in fp32,
      // accumulation ≤ 32u·Σ|terms| in any order even with truncating adds, split remainders
      // 3u16²|R||p| + 4σ(|R| + 3|p|) summed over the row, u16²|x| + σ for t and q
      const double Pt = S * m.pinf, Qt = S * m.qinf, Tt = S * tinf;
      const double sum_terms = (rowl1 * Pt + Tt + Qt) * (1.0 + 4.0 * kU16);
      const double Ed = 1.05 * (32.0 * kU32 * sum_terms + 3.0 * kU16 * kU16 * rowl1 * Pt +
                                4.0 * kSig16 * (rowl1 + 3.0 * Pt) + kU16 * kU16 * (Tt + Qt) +
                                4.0 * kSig16);
      const double Ts = S * thr, T2 = S * S * m.thr_sq;
      const double dm = Ts + 1.7320508075688772 * Ed;       // |d| of a pair that could flip
      const double dc = Ts + 2.0 * 1.7320508075688772 * Ed;  // its computed |d|
      const double e = kU32 * T2 + 2.0 * 1.7320508075688772 * dm * Ed + 3.0 * Ed * Ed +
                       3.0 * kU32 * (T2 + dc * dc);
      eps = __double2float_ru(1.25 * e + 8.0 * DBL_EPSILON * T2);
    }
  }
  if (far) {
    for (int c = 0; c < 3; ++c) {
      B0[c].u = make_uint4(0, 0, 0, 0);
      B1[c].h = s_half8{zero, (_Float16)kFarT, zero, mone, mone, zero, zero, zero};
    }
  }
  for (int c = 0; c < 3; ++c) {
    hb16[c * h_pad + j] = B0[c].u;
    hb16[(3 + c) * h_pad + j] = B1[c].u;
  }
  heps[j] = eps;
}

__global__ __launch_bounds__(256) void hyp16_kernel(const double* __restrict__ T64, int64_t H,
                                                    int64_t h_pad, Mf16Params m,
                                                    uint4* __restrict__ hb16,
                                                    float* __restrict__ heps) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= h_pad) return;
  hyp16_one(j < H ? T64 + 16 * j : nullptr, j < H, j, h_pad, m, hb16, heps);
}

// acc − x·x as one scalar v_fma_f32 (single rounding, = fma(−x, x, acc)).  The empty asm makes
// each operand an opaque scalar so that no pass pairs neighbours into v_pk_fma_f32: beside MFMAs
// a packed fp32 op costs ≈ 22 cycles more than the two scalar FMAs it replaces
// (MI355X_MICROARCH.md, filler prices; measured here 0.189 → 0.178 ms per 1e9 pairs).  The FMA
// itself stays compiler-generated: an asm FMA reading an MFMA result would bypass the hazard
// recogniser's wait states.
__device__ __forceinline__ float fnmsq(float x, float acc) {
  asm volatile("" : "+v"(x));
  return __builtin_fmaf(-x, x, acc);
}

__device__ __forceinline__ float vmin3a(float a, float b, float c) {
  return __builtin_elementwise_minimum(__builtin_elementwise_minimum(fabsf(a), fabsf(b)), fabsf(c));
}

// units of score_mfma_kernel's per-lane outlier counter (the v_perm count adds 8 per outlier)
constexpr uint32_t kOutlUnit = 8u;

// grid: x = hypothesis blocks of shyps<kSMG>(), y = correspondence slices of slice_len (multiple
// of kSTile); block = 8 waves, wave w owns hypotheses hb + (w·kSMG + g)·32 + (lane & 31).
template <int kSMG>
__global__ __launch_bounds__(kSBlock) void score_mfma_kernel(
    const uint4* __restrict__ ca16, int64_t nc_pad, const uint4* __restrict__ hb16,
    const float* __restrict__ heps, int64_t h_pad, int64_t H, int64_t slice_len, float T2,
    int32_t* __restrict__ counts, ExactArgs ex, const int32_t* __restrict__ done, int xcd) {
  if (done != nullptr && *done) return;
  // xcd: the dispatch order is remapped so that each XCD (linear block id mod 8) walks one
  // contiguous run of a group-major order — hypothesis blocks in 4 groups, within a group slice
  // by slice — so an XCD's L2 holds its group's B operands (≈ 2.4 MB) and one correspondence
  // slice at a time, instead of every XCD streaming every block's operands
  int64_t bxi = blockIdx.x, byi = blockIdx.y;
  if (xcd) {
    const int64_t nbx = gridDim.x, nby = gridDim.y, nb = nbx * nby;
    const int64_t b = blockIdx.x + blockIdx.y * nbx;
    const int64_t k = b % 8, pos = b / 8;
    const int64_t t = k * (nb / 8) + min(k, nb % 8) + pos;  // this XCD's run starts after the others'
    constexpr int64_t kG = 4;
    const int64_t gx = (nbx + kG - 1) / kG;
    const int64_t g = min(t / (gx * nby), (nbx - 1) / gx);  // full groups hold gx × nby blocks
    const int64_t r = t - g * gx * nby;
    const int64_t w = min(gx, nbx - g * gx);
    byi = r / w;
    bxi = g * gx + r % w;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  s_half8 bx[kSMG], by[kSMG], bz[kSMG];
  float eps[kSMG];
  uint32_t outl[kSMG];
  int64_t hyp[kSMG];
#pragma unroll
  for (int g = 0; g < kSMG; ++g) {
    const int64_t j = bxi * shyps<kSMG>() + (wave * kSMG + g) * 32 + c;  // < h_pad
    hyp[g] = j;
    SH8 t;
    t.u = hb16[(3 * h + 0) * h_pad + j];
    bx[g] = t.h;
    t.u = hb16[(3 * h + 1) * h_pad + j];
    by[g] = t.h;
    t.u = hb16[(3 * h + 2) * h_pad + j];
    bz[g] = t.h;
    eps[g] = heps[j];
    outl[g] = 0;
  }
  const s_floatx16 zacc = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f,
                           0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  // the threshold as a VGPR operand (a uniform value would be kept in SGPRs, and an SGPR source
  // costs 1.65x VALU issue time on gfx950: tools/ubench_valu.hip)
  float t2r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t2r) : "s"(T2));
  // [buffer][plane][correspondence]: plane 0 = p part (lane half 0 of every component),
  // planes 1-3 = the q_x / q_y / q_z parts (lane half 1).  The threads stage the tile's
  // 4 × kSTile 16-B operands (kStage of them: below).
  __shared__ uint4 a16[2][4][kSTile];
  __shared__ uint32_t qn;                 // guard-band queue: entries used
  __shared__ uint2 qbuf[kSQueue];         // (correspondence, hypothesis | screen sign << 31)
  if (threadIdx.x == 0) qn = 0;
  // grid.y block y visits every gridDim.y-th correspondence tile (slice_len = 0) or a contiguous
  // slice of slice_len rows
  const int64_t tstep = slice_len == 0 ? (int64_t)gridDim.y * kSTile : (int64_t)kSTile;
  const int64_t jb = slice_len == 0 ? byi * kSTile : byi * slice_len;
  const int64_t je = slice_len == 0 ? nc_pad : min(nc_pad, jb + slice_len);
  // thread t stages elements e = t + u·kSBlock of the tile's 4 × kSTile operands: plane e / kSTile,
  // row e % kSTile (a wave's 64 lanes: 64 consecutive rows of one plane)
  constexpr int kStage = 4 * kSTile / kSBlock;
#pragma unroll
  for (int u = 0; u < kStage; ++u) {
    const int e = threadIdx.x + u * kSBlock;
    a16[0][e / kSTile][e % kSTile] = ca16[(e / kSTile) * nc_pad + jb + e % kSTile];
  }
  __syncthreads();
  int buf = 0;
  const int pa = h == 0 ? 0 : 1;  // planes read by this lane for x, y, z: pa·(1 + comp)
  uint32_t tiles_seen = 0;
  for (int64_t j0 = jb; j0 < je; j0 += tstep) {
    ++tiles_seen;
    const bool has_next = j0 + tstep < je;
    // the next tile goes global → LDS by DMA (global_load_lds_dwordx4: wave-uniform base + lane ×
    // 16 B; the a16 rows are lane-linear) while this tile is swept, so no prefetch registers.  The
    // register prefetch (2 × uint4 live across the sweep) was spilled to scratch at the 128-VGPR
    // cap: a scratch store + reload per tile (78 of the launch's 83 MB of HBM writes at H = 1e5)
    // and a wait for the load before the sweep began.  The sweep issues no other vector-memory
    // load (the rare in-place exact fallback's waits stay correct: lds_dma.h); the wait before
    // the barrier below retires the copy.
    if (has_next) {
#pragma unroll
      for (int u = 0; u < kStage; ++u) {
        const int e = threadIdx.x + u * kSBlock;
        lds_dma16(ca16 + (e / kSTile) * nc_pad + j0 + tstep + e % kSTile, &a16[buf ^ 1][e / kSTile][(e % kSTile) & ~63]);
      }
    }
#pragma unroll 2
    for (int sub = 0; sub < kSTile / 32; ++sub) {
      SH8 ax, ay, az;
      ax.u = a16[buf][pa * 1][sub * 32 + c];
      ay.u = a16[buf][pa * 2][sub * 32 + c];
      az.u = a16[buf][pa * 3][sub * 32 + c];
#pragma unroll
      for (int g = 0; g < kSMG; ++g) {
#ifndef M3D_SCORE_PRICE
#define M3D_SCORE_PRICE 0  // pricing builds (timing only, wrong counts): 1 MFMA only, 2 VALU only
#endif
#if M3D_SCORE_PRICE == 2
        s_floatx16 dx, dy, dz;  // the LDS operands' bits as stand-in residuals (no MFMA)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t w[4] = {ax.u.x, ax.u.y, ay.u.z, az.u.w};
          dx[r] = __uint_as_float(w[r & 3] & 0x3FFFFFFFu);
          dy[r] = __uint_as_float(w[(r + 1) & 3] & 0x3FFFFFFFu);
          dz[r] = __uint_as_float(w[(r + 2) & 3] & 0x3FFFFFFFu);
        }
#else
        const s_floatx16 dx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax.h, bx[g], zacc, 0, 0, 0);
        const s_floatx16 dy = __builtin_amdgcn_mfma_f32_32x32x16_f16(ay.h, by[g], zacc, 0, 0, 0);
        const s_floatx16 dz = __builtin_amdgcn_mfma_f32_32x32x16_f16(az.h, bz[g], zacc, 0, 0, 0);
#endif
#if M3D_SCORE_PRICE == 1
        outl[g] += __float_as_uint(dx[g]) ^ __float_as_uint(dy[5]) ^ __float_as_uint(dz[11]);
        continue;
#endif
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = fnmsq(dz[r], fnmsq(dy[r], fnmsq(dx[r], t2r)));
        // v > 0 ⇔ inlier (outside the band): count sign bits (outliers) per lane
        uint32_t s = 0;
        // v_perm selectors 9 / 11 give a byte of 0xFF when S1 / S0 is negative: two sign masks
        // per word, and one full-rate OR joins two such words, so one v_bcnt (accumulating) counts
        // four sign bytes — 8 per outlier, so outl holds 8× the count (per 4 values 2 perm + 1 or
        // + 1 bcnt instead of 4 shifts + 2 add3)
#pragma unroll
        for (int r = 0; r < 16; r += 4)
          s += __builtin_popcount(
              __builtin_amdgcn_perm(__float_as_uint(v[r]), __float_as_uint(v[r + 1]), 0x0C0C0B09u) |
              __builtin_amdgcn_perm(__float_as_uint(v[r + 2]), __float_as_uint(v[r + 3]), 0x0B090C0Cu));
        outl[g] += s;
        const float m0 = vmin3a(v[0], v[1], v[2]), m1 = vmin3a(v[3], v[4], v[5]);
        const float m2 = vmin3a(v[6], v[7], v[8]), m3 = vmin3a(v[9], v[10], v[11]);
        const float m4 = vmin3a(v[12], v[13], v[14]);
        const float m = __builtin_elementwise_minimum(
            __builtin_elementwise_minimum(__builtin_elementwise_minimum(m0, m1),
                                          __builtin_elementwise_minimum(m2, m3)),
            __builtin_elementwise_minimum(m4, fabsf(v[15])));
        if (__any(m < eps[g])) {
          // rare (wave-uniform): pairs inside their hypothesis's guard band.  They are queued in
          // LDS (correspondence, hypothesis, screen sign) and re-evaluated in fp64 by the whole
          // block after the sweep, so no wave waits on the dependent fp64 loads here; a full
          // queue falls back to evaluating in place.
          uint32_t bm = 0, sm = 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            bm |= (fabsf(v[r]) < eps[g] ? 1u : 0u) << r;
            sm |= (__float_as_uint(v[r]) >> 31) << r;
          }
          const uint32_t nb = __builtin_popcount(bm);
          uint32_t slot = nb ? atomicAdd(&qn, nb) : 0u;
          while (bm != 0) {
            const int r = __builtin_ctz(bm);
            bm &= bm - 1;
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t i = j0 + sub * 32 + row;  // < nc (pads are never in a band)
            const uint32_t sgn = (sm >> r) & 1u;
            if (slot < kSQueue) {
              qbuf[slot] = make_uint2((uint32_t)i, (uint32_t)hyp[g] | (sgn << 31));
            } else {
              const bool in = hyp[g] < H && i < ex.nc &&
                              exact_inlier(ex.T64 + 16 * hyp[g], ex.p64 + 3 * i, ex.q64 + 3 * i,
                                           ex.thr, ex.mode);
              outl[g] += kOutlUnit * ((in ? 0u : 1u) - sgn);
            }
            ++slot;
          }
        }
      }
    }
    lds_dma_wait();
    __syncthreads();
    buf ^= 1;
  }
  // inliers of hypothesis column c over this slice: rows − outliers, the two lane halves summed
  const uint32_t rows = tiles_seen * (kSTile / 2);  // each lane half sees half of every 32-row block
#pragma unroll
  for (int g = 0; g < kSMG; ++g) {
    const uint32_t in = 2 * rows - (outl[g] + (uint32_t)__shfl_xor((int)outl[g], 32)) / kOutlUnit;
    if (h == 0 && hyp[g] < H && in != 0) atomicAdd(&counts[hyp[g]], (int32_t)in);
  }
  // the queued guard-band pairs, one per thread: fp64 in numpy order, count correction
  // (screen sign − exact outlier flag) for that hypothesis
  const uint32_t nq = min(qn, (uint32_t)kSQueue);  // the last barrier of the loop published qn
  for (uint32_t e = threadIdx.x; e < nq; e += kSBlock) {
    const uint2 q = qbuf[e];
    const int64_t i = (int64_t)q.x;
    const int64_t j = (int64_t)(q.y & 0x7FFFFFFFu);
    const int sgn = (int)(q.y >> 31);
    const bool in = j < H && i < ex.nc &&
                    exact_inlier(ex.T64 + 16 * j, ex.p64 + 3 * i, ex.q64 + 3 * i, ex.thr, ex.mode);
    const int corr = sgn - (in ? 0 : 1);  // +1: a screen outlier is an inlier, −1: the reverse
    if (corr != 0 && j < H) atomicAdd(&counts[j], corr);
  }
  if (threadIdx.x == 0 && ex.stats && qn != 0)
    atomicAdd((unsigned long long*)&ex.stats[0], (unsigned long long)qn);
}

int64_t score_mf_hpad(int64_t H) { return (H + kSHypPad - 1) / kSHypPad * kSHypPad; }

// ------------------------------------------------------------------------------- a4 select
struct BestPair {
  int64_t c, i;
};
__device__ __forceinline__ BestPair combine(BestPair l, BestPair r) { return (r.c > l.c) ? r : l; }

// exact cube (double-double, then one rounding) so r**3 matches a correctly rounded pow(r, 3)
__device__ __forceinline__ double cube_rn(double r) {
  const double r2 = r * r;
  const double e2 = fma(r, r, -r2);
  const double hi = r2 * r;
  const double e3 = fma(r2, r, -hi);
  return hi + (e3 + e2 * r);
}

__device__ __forceinline__ int64_t required_iters(double ratio, double conf, int64_t max_iter) {
  if (ratio < 0.01) return max_iter;  // _visualize_matcher.py:367-368
  const double v = log(1.0 - conf) / log(1.0 - cube_rn(ratio));
  if (!(v < 9.0e18)) return INT64_MAX;
  return (int64_t)v;  // int() truncation (v >= 0 here)
}

// Batch end without early stop: the batch's best (count desc, index asc — the first strict
// improvement of the sequential walk) is order-free, given as one packed key.
__device__ void finish_batch(RansacState* __restrict__ rs, uint64_t key, int64_t h_begin, int64_t n,
                             int64_t max_iter, const double* __restrict__ T_batch) {
  if (key == 0) {  // empty batch (n == 0): no candidate, only the iteration count moves
    rs->iterations = h_begin + n;
    if (rs->iterations >= max_iter) rs->done = 1;
    return;
  }
  const BestPair bb{(int64_t)(key >> 32), h_begin + (int64_t)(0xFFFFFFFFu - (uint32_t)key)};
  const BestPair fin = combine(BestPair{rs->best_count, rs->best_index}, bb);
  if (fin.i != rs->best_index && fin.i >= h_begin) {
    for (int k = 0; k < 16; ++k) rs->T_best[k] = T_batch[16 * (fin.i - h_begin) + k];
  }
  rs->best_count = fin.c;
  rs->best_index = fin.i;
  rs->iterations = h_begin + n;
  if (rs->iterations >= max_iter) rs->done = 1;
}

// Batch best for the no-early-stop select: key = (count << 32) | (2³² − 1 − k), k the batch
// position, so the MAX is the highest count at the lowest position; one 64-bit atomicMax per
// wave into rs->batch_key (0 = empty: below every real key).  Many blocks — a single-block
// reduction of 1e5 counts was latency-bound at 20–40 µs.  The last block to take a ticket reads
// and clears the key and finishes the batch (one launch fewer than a separate select_kernel).
constexpr int kSelBestBlock = 256, kSelBestPer = 8;
__global__ __launch_bounds__(kSelBestBlock) void select_best_kernel(
    const int32_t* __restrict__ counts, int64_t h_begin, int64_t n, int64_t max_iter,
    const double* __restrict__ T_batch, RansacState* __restrict__ rs) {
  if (rs->done) return;  // same value for every block: either all take a ticket or none does
  uint64_t best = 0;
  const int64_t base = (int64_t)blockIdx.x * kSelBestBlock * kSelBestPer + threadIdx.x;
  int32_t v[kSelBestPer];
#pragma unroll
  for (int u = 0; u < kSelBestPer; ++u) v[u] = counts[min(base + u * kSelBestBlock, n - 1)];
#pragma unroll
  for (int u = 0; u < kSelBestPer; ++u) {
    const int64_t k = base + u * kSelBestBlock;
    const uint64_t key = ((uint64_t)(uint32_t)v[u] << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)k);
    if (k < n && key > best) best = key;
  }
#pragma unroll
  for (int w = 32; w > 0; w >>= 1) {
    const uint64_t o = ((uint64_t)(uint32_t)__shfl_xor((int)(best >> 32), w) << 32) |
                       (uint32_t)__shfl_xor((int)(uint32_t)best, w);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & 63) == 0 && best != 0)
    atomicMax((unsigned long long*)&rs->batch_key, (unsigned long long)best);
  __threadfence();
  __syncthreads();
  __shared__ bool last;
  if (threadIdx.x == 0) last = atomicAdd(&rs->ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __threadfence();
  const uint64_t key = atomicExch((unsigned long long*)&rs->batch_key, 0ull);  // for the next batch
  rs->ticket = 0;
  finish_batch(rs, key, h_begin, n, max_iter, T_batch);
}

__global__ __launch_bounds__(1024) void select_kernel(const int32_t* __restrict__ counts,
                                                      int64_t h_begin, int64_t n, int64_t nc,
                                                      int64_t max_iter, int early, double es_thr,
                                                      double es_conf,
                                                      const double* __restrict__ T_batch,
                                                      RansacState* __restrict__ rs) {
  // The batch in chunks of 1024 × kSelPer counts, staged into LDS with coalesced loads (thread t
  // owns the contiguous run [t·kSelPer, (t+1)·kSelPer) of the chunk): per-thread first-max,
  // inclusive block scan with the first-max combine, the running best carried from chunk to
  // chunk, and — early stop — each thread walks its run from its prefix and the first stopping
  // iteration is a block min.  Same result as a sequential walk; per-thread contiguous segments
  // of the whole batch read straight from memory were uncoalesced (81 µs at 1e5 counts).
  constexpr int kSelPer = 8;
  constexpr int kChunk = 1024 * kSelPer;
  __shared__ int32_t cbuf[kChunk];
  __shared__ int64_t sc[1024], si[1024];
  __shared__ int64_t stop_s[1024];
  __shared__ int32_t done_s;
  const int t = threadIdx.x;
  if (t == 0) done_s = rs->done;
  __syncthreads();
  if (done_s) return;
  if (!early) {  // n == 0 only (key 0: no candidate): select_best_kernel finishes non-empty batches
    if (t == 0) finish_batch(rs, 0ull, h_begin, n, max_iter, T_batch);
    return;
  }
  BestPair carry{rs->best_count, rs->best_index};  // running best before the current chunk
  int64_t first_stop = INT64_MAX;
  BestPair fin = carry;
  bool writer = false;
  for (int64_t c0 = 0; c0 < n; c0 += kChunk) {
    const int m = (int)min((int64_t)kChunk, n - c0);
    int32_t ld[kSelPer];
#pragma unroll
    for (int u = 0; u < kSelPer; ++u) {
      const int k = u * 1024 + t;
      ld[u] = k < m ? counts[c0 + k] : 0;
    }
#pragma unroll
    for (int u = 0; u < kSelPer; ++u)
      if (u * 1024 + t < m) cbuf[u * 1024 + t] = ld[u];
    __syncthreads();
    const int b = t * kSelPer, e = min(m, b + kSelPer);
    BestPair loc{-1, -1};
    for (int k = b; k < e; ++k) loc = combine(loc, BestPair{cbuf[k], h_begin + c0 + k});
    sc[t] = loc.c;
    si[t] = loc.i;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele scan
      BestPair v{sc[t], si[t]};
      if (t >= off) v = combine(BestPair{sc[t - off], si[t - off]}, v);
      __syncthreads();
      sc[t] = v.c;
      si[t] = v.i;
      __syncthreads();
    }
    if (early) {
      BestPair cur = carry;
      if (t > 0) cur = combine(carry, BestPair{sc[t - 1], si[t - 1]});
      int64_t stop = INT64_MAX;
      BestPair at_stop = cur;
      for (int k = b; k < e; ++k) {
        cur = combine(cur, BestPair{cbuf[k], h_begin + c0 + k});
        const double fit = (double)cur.c / (double)nc;
        if (fit > es_thr) {
          const int64_t it = h_begin + c0 + k + 1;
          if (it >= required_iters(fit, es_conf, max_iter)) {
            stop = c0 + k;
            at_stop = cur;
            break;
          }
        }
      }
      stop_s[t] = stop;
      __syncthreads();
      for (int w = 512; w > 0; w >>= 1) {
        if (t < w) stop_s[t] = min(stop_s[t], stop_s[t + w]);
        __syncthreads();
      }
      first_stop = stop_s[0];
      if (first_stop != INT64_MAX) {
        writer = (stop == first_stop);
        fin = at_stop;
        break;  // uniform: every thread read the same stop_s[0]
      }
    }
    carry = combine(carry, BestPair{sc[1023], si[1023]});
    __syncthreads();  // before the next chunk overwrites cbuf / sc / stop_s
  }
  if (first_stop == INT64_MAX) {
    writer = (t == 0);
    fin = carry;
  }
  if (writer) {
    if (fin.i != rs->best_index && fin.i >= h_begin) {
      for (int k = 0; k < 16; ++k) rs->T_best[k] = T_batch[16 * (fin.i - h_begin) + k];
    }
    rs->best_count = fin.c;
    rs->best_index = fin.i;
    if (first_stop != INT64_MAX) {
      rs->iterations = h_begin + first_stop + 1;
      rs->done = 1;
    } else {
      rs->iterations = h_begin + n;
      if (rs->iterations >= max_iter) rs->done = 1;
    }
  }
}

__global__ void copy_result_kernel(const RansacState* __restrict__ rs, int64_t nc,
                                   const int64_t* __restrict__ stats,
                                   m3d_ransac_result* __restrict__ out) {
  if (threadIdx.x != 0) return;
  for (int k = 0; k < 16; ++k) out->T[k] = rs->T_best[k];
  out->best_count = rs->best_count;
  out->best_index = rs->best_index;
  out->iterations = rs->iterations;
  out->fitness = nc > 0 ? (double)rs->best_count / (double)nc : 0.0;
  // rs->rechecked holds the recheck counter's value when the run started
  out->rechecked = stats ? stats[0] - rs->rechecked : 0;
}

// ------------------------------------------------------------------------------- launchers
static inline int blocks_for(int64_t n, int t) { return (int)((n + t - 1) / t); }

hipError_t launch_pack_corr(const double* src, const double* tgt, const int32_t* corr, int64_t nc,
                            const double* p_src, const double* p_tgt, double* p64, double* q64,
                            hipStream_t st) {
  if (nc == 0) return hipSuccess;
  pack_corr_kernel<<<blocks_for(nc, 256), 256, 0, st>>>(src, tgt, corr, nc, p_src, p_tgt, p64, q64);
  return hipGetLastError();
}

hipError_t launch_sum3(const double* a, int64_t n, double* partial, int blocks, hipStream_t st) {
  sum3_kernel<<<blocks, 256, 0, st>>>(a, n, partial);
  return hipGetLastError();
}

hipError_t launch_cloud_pack(const double* a, int64_t n, int64_t n_pad, const double* sum_part,
                             int sum_blocks, double* cdev, const double c[3], float4* out, float pad_value,
                             float* part7, int blocks, double* pin_c, float* pin7, hipStream_t st) {
  if (sum_part != nullptr) {  // mean on the device from sum3 partials (else c is given)
    mean3_final_kernel<<<1, 64, 0, st>>>(sum_part, sum_blocks, n, cdev);
  }
  cloud_pack_kernel<<<blocks, 256, 0, st>>>(a, n, n_pad, sum_part != nullptr ? cdev : nullptr, c[0], c[1], c[2],
                                            out, pad_value, part7);
  cloud_summary_kernel<<<1, 256, 0, st>>>(part7, blocks, sum_part != nullptr ? cdev : nullptr, pin_c, pin7);
  return hipGetLastError();
}

hipError_t launch_center_pack(const double* a, int64_t n, int64_t n_pad, const double c[3],
                              float4* out, float pad_value, float* maxnorm_partial, int blocks,
                              int maxinf, hipStream_t st) {
  center_pack_kernel<<<blocks, 256, 0, st>>>(a, n, n_pad, c[0], c[1], c[2], out, pad_value,
                                             maxnorm_partial, maxinf);
  return hipGetLastError();
}

static GuardParams guard_of(const m3d_corrset* cs, double thr_sq) {
  GuardParams g;
  for (int k = 0; k < 3; ++k) {
    g.cs[k] = cs->cs[k];
    g.ct[k] = cs->ct[k];
  }
  g.pinf = cs->pmax2;
  g.qinf = cs->qmaxinf;
  g.thr_sq = thr_sq;
  return g;
}

static bool score_prep_params(const m3d_corrset* cs, int64_t H, double thr, int mode,
                              const ScoreMf& mf, Mf16Params* m, int64_t* hp);

hipError_t launch_kabsch3(const m3d_corrset* cs, const int32_t* triples, uint64_t seed,
                          int64_t hyp0, int64_t H, double thr_sq, double* T_out, uint8_t* status,
                          HypF32* hypf, const int32_t* done, ZeroArgs z, hipStream_t st,
                          const ScoreFuse* fuse) {
  if (H == 0) return hipSuccess;
  Hyp16Fuse hf{};
  hf.on = 0;
  if (fuse != nullptr && score_prep_params(cs, H, fuse->thr, fuse->mode, *fuse->mf, &hf.m, &hf.h_pad)) {
    hf.hb16 = fuse->mf->hb16;
    hf.heps = fuse->mf->heps;
    hf.on = 1;
  }
  const int64_t n = hf.on ? hf.h_pad : H;
  kabsch3_kernel<<<blocks_for(n, 256), 256, 0, st>>>(cs->p64, cs->q64, cs->nc, triples, seed,
                                                     hyp0, H, guard_of(cs, thr_sq), T_out, status,
                                                     hf.on ? nullptr : hypf, done, z, hf);
  return hipGetLastError();
}

hipError_t launch_hypf_from_T(const m3d_corrset* cs, const double* T, int64_t H, double thr_sq,
                              HypF32* hypf, ZeroArgs z, hipStream_t st) {
  if (H == 0) return hipSuccess;
  hypf_from_T_kernel<<<blocks_for(H, 256), 256, 0, st>>>(T, H, guard_of(cs, thr_sq), hypf, z);
  return hipGetLastError();
}

hipError_t launch_corr16(m3d_corrset* cs, hipStream_t st) {
  cs->s16 = 0.0;
  if (cs->nc == 0) return hipSuccess;
  const double mx = fmax(cs->pmax2, cs->qmaxinf);
  if (!(mx < 1e30)) return hipSuccess;  // non-finite input: the fp32 screen handles it
  double S = 1.0;
  if (mx > 0.0) S = exp2(floor(log2(1024.0 / mx)));
  S = fmin(fmax(S, 0x1p-40), 0x1p40);
  hipError_t e = dev_malloc(&cs->ca16, sizeof(uint4) * 4 * cs->nc_pad);
  if (e != hipSuccess) {
    cs->ca16 = nullptr;
    return e;
  }
  corr16_kernel<<<blocks_for(cs->nc_pad, 256), 256, 0, st>>>(
      cs->p64, cs->q64, cs->nc, cs->nc_pad, cs->cs[0], cs->cs[1], cs->cs[2], cs->ct[0], cs->ct[1],
      cs->ct[2], S, cs->ca16);
  e = hipGetLastError();
  if (e == hipSuccess) cs->s16 = S;
  return e;
}

// MFMA scoring applies when the operands exist and the threshold stays inside the cloud's
// scaled range (S·thr ≤ 1024: thresholds beyond the cloud extent use the fp32 screen)
static bool use_mfma_score(const m3d_corrset* cs, const ScoreMf& mf, double thr_sq) {
  return mf.hb16 != nullptr && cs->ca16 != nullptr && cs->s16 > 0.0 &&
         cs->s16 * sqrt(thr_sq) <= 1024.0;
}

static double thr_sq_mode(double thr, int mode) { return mode == M3D_SCORE_SQUARED ? thr : thr * thr; }

// the MFMA screen's per-batch parameters; false: the batch is not scored by the MFMA screen
static bool score_prep_params(const m3d_corrset* cs, int64_t H, double thr, int mode,
                              const ScoreMf& mf, Mf16Params* m, int64_t* hp) {
  const double thr_sq = thr_sq_mode(thr, mode);
  if (H == 0 || cs->nc == 0 || !use_mfma_score(cs, mf, thr_sq)) return false;
  for (int k = 0; k < 3; ++k) {
    m->cs[k] = cs->cs[k];
    m->ct[k] = cs->ct[k];
  }
  m->S = cs->s16;
  m->pinf = cs->pmax2;
  m->qinf = cs->qmaxinf;
  m->thr_sq = thr_sq;
  *hp = score_mf_hpad(H);
  return true;
}

hipError_t launch_score_prep(const m3d_corrset* cs, const double* T64, int64_t H, double thr,
                             int mode, const ScoreMf& mf, hipStream_t st) {
  Mf16Params m;
  int64_t hp = 0;
  if (!score_prep_params(cs, H, thr, mode, mf, &m, &hp)) return hipSuccess;
  hyp16_kernel<<<blocks_for(hp, 256), 256, 0, st>>>(T64, H, hp, m, mf.hb16, mf.heps);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------- one hypothesis
// The per-call drop-in (compute_step_transformation / evaluate_inlier_ratio as
// benchmark_ransac.py:105-113 calls them, one hypothesis per call): the triple and the transform
// travel as kernel arguments and the results go straight into mapped pinned memory, so a call
// is one launch and one stream sync, with no staging copies (a2/a3: count_one_kernel below).
struct Tri3 {
  int32_t i[3];
};
struct T16 {
  double v[16];
};

__global__ void kabsch3_one_kernel(const double* __restrict__ p64, const double* __restrict__ q64,
                                   int64_t nc, Tri3 tri, double* __restrict__ T_out,
                                   int32_t* __restrict__ status) {
  if (threadIdx.x != 0) return;
  double T[16];
  int st = M3D_HYP_OK;
  if (nc < 3) {  // ransac.py:139-140
    for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
    st = M3D_HYP_DEGENERATE;
  } else {
    double ps[3][3], qs[3][3];
    for (int k = 0; k < 3; ++k) {
      const int64_t r = (tri.i[k] < 0 || tri.i[k] >= nc) ? 0 : tri.i[k];
      for (int c = 0; c < 3; ++c) {
        ps[k][c] = p64[3 * r + c];
        qs[k][c] = q64[3 * r + c];
      }
    }
    st = kabsch3(ps, qs, T) ? M3D_HYP_NONFINITE : M3D_HYP_OK;
  }
  for (int k = 0; k < 16; ++k) T_out[k] = T[k];
  *status = st;
}

hipError_t launch_kabsch3_one(const m3d_corrset* cs, const int32_t* tri, double* T_out,
                              int32_t* status, hipStream_t st) {
  Tri3 t{{tri[0], tri[1], tri[2]}};
  kabsch3_one_kernel<<<1, 64, 0, st>>>(cs->p64, cs->q64, cs->nc, t, T_out, status);
  return hipGetLastError();
}

// One transform against every correspondence: the reference formula itself in fp64 (numpy's
// operation order, exact_inlier) — for a single hypothesis that is ~30 fp64 flop per pair, less
// than the MFMA screen's 1024-hypothesis padding costs.  Block counts go out write-through, the
// last block (ticket) adds them in block order and stores the total straight into the caller's
// mapped pinned memory: one launch, no memset, no copy.
constexpr int kOneBlock = 256, kOnePerThread = 4;
__global__ __launch_bounds__(kOneBlock) void count_one_kernel(T16 T, const double* __restrict__ p64,
                                                              const double* __restrict__ q64,
                                                              int64_t nc, double thr, int mode,
                                                              int32_t* partials, uint32_t* ticket,
                                                              int64_t* out) {
  __shared__ int32_t wsum[kOneBlock / 64];
  __shared__ int last;
  int32_t n = 0;
#pragma unroll
  for (int u = 0; u < kOnePerThread; ++u) {
    const int64_t i = ((int64_t)blockIdx.x * kOnePerThread + u) * kOneBlock + threadIdx.x;
    if (i < nc) n += exact_inlier(T.v, p64 + 3 * i, q64 + 3 * i, thr, mode) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int32_t b = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __hip_atomic_store(&partials[blockIdx.x], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  int64_t t = 0;
  for (uint32_t b = threadIdx.x; b < gridDim.x; b += kOneBlock)
    t += __hip_atomic_load(&partials[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  __shared__ int64_t tw[kOneBlock / 64];
  if ((threadIdx.x & 63) == 0) tw[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    *out = tw[0] + tw[1] + tw[2] + tw[3];
    *ticket = 0u;
  }
}

hipError_t launch_count_one(const m3d_corrset* cs, const double* T, double thr, int mode,
                            int32_t* partials, int64_t max_blocks, uint32_t* ticket, int64_t* out,
                            hipStream_t st) {
  T16 t;
  for (int k = 0; k < 16; ++k) t.v[k] = T[k];
  const int64_t per = (int64_t)kOneBlock * kOnePerThread;
  const int64_t nb = (cs->nc + per - 1) / per;
  if (nb < 1 || nb > max_blocks) return hipErrorInvalidValue;
  count_one_kernel<<<(unsigned)nb, kOneBlock, 0, st>>>(t, cs->p64, cs->q64, cs->nc, thr, mode, partials,
                                                        ticket, out);
  return hipGetLastError();
}

int64_t count_one_blocks(int64_t nc) {
  const int64_t per = (int64_t)kOneBlock * kOnePerThread;
  return std::max<int64_t>(1, (nc + per - 1) / per);
}

// grid.y of the MFMA screen for bx hypothesis blocks
static int64_t score_grid_y(const m3d_corrset* cs, int64_t bx) {
  // correspondence tiles over grid.y so that ≥ ~2048 blocks fill the chip: block y visits
  // every sy-th tile (slice 0), sy chosen in [S0, 2·S0] to fill the resident block slots in
  // whole rounds (20 × 98 contiguous slices = 3.8 rounds of 512 slots ran as 4)
  const int64_t tiles = cs->nc_pad / kSTile;
  int64_t sy = std::min<int64_t>(std::max<int64_t>((2048 + bx - 1) / bx, 1), tiles);
  {
    static const int64_t slots = [] {
      int dev = 0, per = 0;
      hipDeviceProp_t p;
      if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return (int64_t)0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, score_mfma_kernel<kSGroups>, kSBlock, 0) != hipSuccess)
        return (int64_t)0;
      return (int64_t)p.multiProcessorCount * (per > 0 ? per : 1);
    }();
    if (slots > 0) {
      const int64_t s0 = sy;
      double best_eff = 0.0;
      for (int64_t S = s0; S <= std::min<int64_t>(2 * s0, tiles); ++S) {
        const int64_t blocks = bx * S, rounds = (blocks + slots - 1) / slots;
        const double eff = (double)blocks / (double)(rounds * slots);
        if (eff > best_eff + 1e-9) {
          best_eff = eff;
          sy = S;
        }
      }
    }
  }
  return sy;
}

hipError_t launch_score(const m3d_corrset* cs, const HypF32* hypf, int64_t H, int32_t* counts,
                        const double* T64, double thr, int mode, int64_t* stats,
                        const int32_t* done, const ScoreMf& mf, hipStream_t st) {
  if (H == 0 || cs->nc == 0) return hipSuccess;
  ExactArgs ex{T64, cs->p64, cs->q64, cs->nc, thr, mode, stats};
  const double thr_sq = thr_sq_mode(thr, mode);
  if (use_mfma_score(cs, mf, thr_sq)) {
    const int64_t hp = score_mf_hpad(H);
    const int64_t bx = hp / shyps<kSGroups>();
    const int64_t sy = score_grid_y(cs, bx);
    const float T2 = (float)(cs->s16 * cs->s16 * thr_sq);
    // slice_len 0: block y visits every sy-th correspondence tile; xcd 1: the XCD-aware dispatch
    score_mfma_kernel<kSGroups><<<dim3((unsigned)bx, (unsigned)sy), kSBlock, 0, st>>>(
        cs->ca16, cs->nc_pad, mf.hb16, mf.heps, hp, H, 0, T2, counts, ex, done, 1);
    return hipGetLastError();
  }
  const int64_t per_launch = (int64_t)65535 * kScoreHyps;  // grid.y limit
  for (int64_t hb = 0; hb < H; hb += per_launch) {
    const int64_t nh = (H - hb) < per_launch ? (H - hb) : per_launch;
    dim3 grid((unsigned)(cs->nc_pad / kBlockCorr), (unsigned)((nh + kScoreHyps - 1) / kScoreHyps));
    score_kernel<<<grid, kScoreBlock, 0, st>>>(cs->p32, cs->q32, (const float4*)hypf, H, hb,
                                               counts, ex, done);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_select(const int32_t* counts, int64_t h_begin, int64_t n, int64_t nc,
                         int64_t max_iter, int early_stop, double es_thr, double es_conf,
                         const double* T_batch, RansacState* rs, hipStream_t st) {
  if (!early_stop && n > 0) {
    const int64_t per = (int64_t)kSelBestBlock * kSelBestPer;
    select_best_kernel<<<(unsigned)((n + per - 1) / per), kSelBestBlock, 0, st>>>(
        counts, h_begin, n, max_iter, T_batch, rs);
    return hipGetLastError();
  }
  select_kernel<<<1, 1024, 0, st>>>(counts, h_begin, n, nc, max_iter, early_stop, es_thr, es_conf,
                                    T_batch, rs);
  return hipGetLastError();
}

// state of a fresh a4 run (one launch instead of a pageable H2D copy + a D2D copy: ~10 µs)
__global__ void ransac_init_kernel(RansacState* __restrict__ rs, const int64_t* __restrict__ stats,
                                   int done) {
  if (threadIdx.x != 0) return;
  for (int k = 0; k < 16; ++k) rs->T_best[k] = (k % 5 == 0) ? 1.0 : 0.0;
  rs->best_count = -1;
  rs->best_index = -1;
  rs->iterations = 0;
  rs->rechecked = stats != nullptr ? stats[0] : 0;  // copy_result reports the difference
  rs->done = done;
  rs->ticket = 0;
  for (int k = 0; k < 2; ++k) rs->pad[k] = 0;
  rs->batch_key = 0;
}

hipError_t launch_ransac_init(RansacState* rs, const int64_t* stats, int done, hipStream_t st) {
  ransac_init_kernel<<<1, 64, 0, st>>>(rs, stats, done);
  return hipGetLastError();
}

hipError_t launch_copy_result(const RansacState* rs, int64_t nc, const int64_t* stats,
                              m3d_ransac_result* out_dev, hipStream_t st) {
  copy_result_kernel<<<1, 64, 0, st>>>(rs, nc, stats, out_dev);
  return hipGetLastError();
}

// hypothesis-sharded a4: this rank's best as the MAX-reducible key (count << 32) | (2³²−1 − id)
__global__ void ransac_pack_key_kernel(const m3d_ransac_result* __restrict__ r, int64_t hyp0,
                                       int64_t* __restrict__ key) {
  if (threadIdx.x != 0) return;
  const int64_t c = r->best_count, bi = r->best_index;
  key[0] = (c < 0 || bi < 0) ? 0
                             : (int64_t)(((uint64_t)c << 32) | (0xFFFFFFFFull - (uint64_t)(hyp0 + bi)));
}

hipError_t launch_ransac_pack_key(const m3d_ransac_result* r, int64_t hyp0, int64_t* key,
                                  hipStream_t st) {
  ransac_pack_key_kernel<<<1, 64, 0, st>>>(r, hyp0, key);
  return hipGetLastError();
}

// m3d_ransac_run_sharded, after MAX(buf[0]) over ranks: the SUM payload buf[1..19] = this rank's
// iterations, rechecked, the bits of its best T if its key is the global one (else 0: exactly one
// rank holds the winner, ids are disjoint, so the integer SUM is the winner's bits, -0.0
// included) and the failed-rank count.  A rank whose local run failed (r == null) contributes
// zeros and 1: every rank learns of the failure from the same collective, none waits forever.
__global__ void ransac_shard_pack_kernel(const m3d_ransac_result* __restrict__ r, int64_t hyp0,
                                         int64_t* __restrict__ buf) {
  const int t = threadIdx.x;
  int64_t lkey = 0;
  if (r != nullptr) {
    const int64_t c = r->best_count, bi = r->best_index;
    lkey = (c < 0 || bi < 0) ? 0 : (int64_t)(((uint64_t)c << 32) | (0xFFFFFFFFull - (uint64_t)(hyp0 + bi)));
  }
  const bool win = lkey != 0 && lkey == buf[0];
  if (t < 16) buf[3 + t] = win ? __double_as_longlong(r->T[t]) : 0;
  if (t == 16) buf[1] = r != nullptr ? r->iterations : 0;
  if (t == 17) buf[2] = r != nullptr ? r->rechecked : 0;
  if (t == 18) buf[19] = r != nullptr ? 0 : 1;
}

hipError_t launch_ransac_shard_key(const m3d_ransac_result* r, int64_t hyp0, int64_t* buf,
                                   hipStream_t st) {
  if (r == nullptr) return hipMemsetAsync(buf, 0, sizeof(int64_t), st);
  ransac_pack_key_kernel<<<1, 64, 0, st>>>(r, hyp0, buf);
  return hipGetLastError();
}

hipError_t launch_ransac_shard_pack(const m3d_ransac_result* r, int64_t hyp0, int64_t* buf,
                                    hipStream_t st) {
  ransac_shard_pack_kernel<<<1, 64, 0, st>>>(r, hyp0, buf);
  return hipGetLastError();
}

}  // namespace m3d
