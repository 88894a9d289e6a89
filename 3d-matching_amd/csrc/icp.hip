// icp.hip — ICP refinement for gfx950.
//
// Reference: src/matcher/icp.py:42-48 → Open3D 0.19 RegistrationICP with
// TransformationEstimationPointToPlane and ICPConvergenceCriteria(1e-6, 1e-6, 30).
// One iteration = Eval(T) [1-NN within r, fitness, rmse] + ComputeTransformation + T ← ΔT·T.
//
// Kernels per iteration (all device resident, no host round trip):
//   keyinit  O(Ns)      seeds each query's bound with its previous neighbour (fp32 d²)
//   nn       O(Ns·Nt)   brute-force scan, nn_mfma_kernel: screen key |t|² − 2q·t on the matrix
//                       cores (fp16 hi/lo split operands, proven error bound, refresh_rt32),
//                       v_minimum3 tree per 32×32 block, flagged sub-tiles take the exact path:
//                       direct fp32 d² with lexicographic (d², index) argmin — the same result as
//                       a full direct scan (nn_kernel: the fp32 VALU form of the same screen,
//                       used when a target has no MFMA tiles).  The target range is split into
//                       slices (grid.y); slices merge with a 64-bit atomicMin on packed
//                       (bits(d²) << 32 | idx): order independent → deterministic, lowest index
//                       wins exact ties.  (grid.hip: the radius-bounded grid search, same key.)
//   terms_solve O(Ns)   fp64: radius test d² < r² (strict, nanoflann), point-to-plane
//                       J = [p×n ; n], r = (p−q)·n → JTJ(21) JTr(6) Σr²; count; Σd² → block
//                       partials; the last block reduces them in a fixed order and one wave runs
//                       the solve (fitness/rmse, convergence test, LDLT(JTJ, −JTr),
//                       x → Rz·Ry·Rx|t, T ← ΔT·T).
// The multi-GPU paths use the same pieces as separate launches (terms_kernel, reduce_kernel,
// solve_kernel) with the RCCL MIN on keys / SUM on the 32 term slots between them.
#include <float.h>

#include <algorithm>
#include <string>
#include <vector>
#include <stdlib.h>

#include "lds_dma.h"
#include "linalg.h"
#include "m3d_internal.h"
#include "nnkey.h"

namespace m3d {

constexpr int kNNQ = 4;       // queries per lane (nn_kernel)
constexpr int kNNTile = 16;   // screen sub-tile (one branch per sub-tile)
constexpr int kNNLds = 512;   // targets per LDS tile (8 KB, double-buffered)
constexpr int kNNBlock = 256;
// terms pass geometry: 512-thread blocks, one source per thread (196 block partials at cfg1, as
// 256 × 2 gave): two waves per SIMD share the fp64 work and hide each other's round trips — the
// last terms wave of a cfg1 evaluation ends ≈ 1 µs sooner (docs/EXPERIMENTS.md §R6)
#ifndef M3D_TERMS_BLOCK
#define M3D_TERMS_BLOCK 512
#endif
constexpr int kTermsBlock = M3D_TERMS_BLOCK;
#ifndef M3D_TERMS_PTS
#define M3D_TERMS_PTS 1
#endif
constexpr int kTermsPtsDefault = M3D_TERMS_PTS;  // sources per terms thread (with 256-thread blocks
                                                 // 2 was fastest: 1 doubled the partials, 4 / 8
                                                 // lengthened each wave's chain)
static int terms_pts() { return kTermsPtsDefault; }
constexpr double kU = 5.9604644775390625e-08;
constexpr double kU64 = 1.1102230246251565e-16;


// ------------------------------------------------------------------------------- state
struct FrameParams {
  double cs[3], ct[3];
  double pinf, qinf;
  double s16;  // the target cloud's fp16 operand scale (power of two)
  int shared;  // the target's frame is shared by every shard (m3d_cloud_create_framed)
};

// Refresh the fp32 search transform and radius bound for transform T (device side; T and
// r2 = s->r2 passed in registers by the solve, which has them already).
// fp64 → fp32 rounded toward +inf on the vector unit (the library's __double2float_ru bounces the
// bits through the scalar unit, ≈ 20 dependent instructions each, five of them per refresh):
// the round-to-nearest value, moved one ulp up when it lies below d (−0 / +0 → the least denormal)
__device__ __forceinline__ float f32_ru(double d) {
  const float f = (float)d;
  const uint32_t u = __float_as_uint(f);
  const uint32_t up = f == 0.0f ? 1u : ((int32_t)u >= 0 ? u + 1u : u - 1u);
  return (double)f < d ? __uint_as_float(up) : f;
}

// r = √r2, taken by the caller (the solve computes it while its factorisation runs)
__device__ void refresh_rt32_from(IcpState* s, const double* T, double r2, double r, const FrameParams& f,
                                  int iters) {
  const double* cs = f.cs;
  const double* ct = f.ct;
  const double pinf = f.pinf, qinf = f.qinf;
  double rowl1 = 0.0, tinf = 0.0;
  for (int i = 0; i < 3; ++i) {
    const double* r = T + 4 * i;
    const double tp = fma(r[2], cs[2], fma(r[1], cs[1], r[0] * cs[0])) + r[3] - ct[i];
    for (int j = 0; j < 3; ++j) s->Rt32[3 * i + j] = (float)r[j];
    s->Rt32[9 + i] = (float)tp;
    rowl1 = fmax(rowl1, fabs(r[0]) + fabs(r[1]) + fabs(r[2]));
    tinf = fmax(tinf, fabs(tp));
  }
  // E: per-coordinate bound on |fp32 query − fp64 query| + |fp32 target − fp64 target| in the
  // centred frame: the fp32 roundings of p_c, R, t' and the three fmas (≤ 5u·Σ|r||p| + 4u|t'|),
  // the target's u|t_c|, and the fp64 query Q of the contract against T·p: Q is the source
  // transformed update by update (Open3D's pcd.Transform(update), IcpState::dT), so each of the
  // iters + 1 applications adds ≤ 4 roundings of 2⁻⁵³ of the magnitudes involved; the updates
  // are rotations to fp64 accuracy, which carry the earlier errors over without growth in the
  // 2-norm (√3 per coordinate).  The last term covers an init within 1e-12 of the identity,
  // which Open3D does not apply to the points (Eigen isIdentity) while T = init.
  double tabs = 0.0, csinf = 0.0, ctinf = 0.0;
  for (int i = 0; i < 3; ++i) {
    tabs = fmax(tabs, fabs(T[4 * i + 3]));
    csinf = fmax(csinf, fabs(cs[i]));
    ctinf = fmax(ctinf, fabs(ct[i]));
  }
  const double mag = rowl1 * (csinf + pinf) + tabs + ctinf + qinf;
  // the fp32 part, term by term (xform32: q = fma(r0, px, fma(r1, py, fma(r2, pz, t′)))):
  // p rounding u·Σ|r||p| + R rounding u·Σ|r||p| + three fma roundings ≤ 3u(Σ|r||p| + |t′|) +
  // t′ rounding u|t′| + the target's u|t_c|, Σ|r||p| ≤ ‖r‖₁·|p|∞; ×1.01 for the O(u²) products.
  // (Round 5 used 8u·(‖r‖₁|p|∞ + |t′| + |t|): 2.6× this at cfg1, and the fp32 → fp64 ambiguity
  // band, hence the terms pass's fp64 walks, scale with E.)
#ifndef M3D_TIGHT_E
#define M3D_TIGHT_E 1
#endif
  const double E32 = M3D_TIGHT_E ? 1.01 * kU * (5.0 * rowl1 * pinf + 4.0 * tinf + qinf)
                                 : 8.0 * kU * (rowl1 * pinf + tinf + qinf);
  const double E = E32 + 8.0 * kU64 * 1.7320508075688772 * (double)(iters + 2) * mag + 1e-11 * (mag + 1.0);
  // nnkey.h: |√d2f − |Q − t|| ≤ e_q + 3u√d2f with e_q = √3·E; band_of's absolute term 2·e_q
  const double eq = 1.7320508075688772 * E * 1.01;
  const float eqf = f32_ru(eq), bef = f32_ru(2.0 * eq * 1.01);
  s->eq = isfinite(eqf) ? eqf : FLT_MAX;
  s->band_e = isfinite(bef) ? bef : FLT_MAX;
  const double e = 2.0 * (3.0 * kU * (r + 1.7320508075688772 * E) * (r + 1.7320508075688772 * E) +
                          2.0 * 1.7320508075688772 * E * r + 3.0 * E * E);
  float hi = f32_ru(r2 + e);
  if (!isfinite(hi)) hi = FLT_MAX;
  s->r2_hi = hi;
  // Screen bound: |fl(|t|² − 2q·t) − (d² − |q|²)| + rounding of thr ≤ eps,
  // with |t|∞ ≤ qinf (target), |q|∞ ≤ Q = rowl1·pinf + |t'|∞ (query after the transform).
  const double Q = rowl1 * pinf + tinf;
  const double E1 = 5.0 * kU * (3.0 * qinf * qinf + 6.0 * Q * qinf);
  const double es = 2.0 * (E1 + 6.0 * kU * (double)hi + 12.0 * kU * Q * Q) + 1e-30;
  const float esf = f32_ru(es);
  s->screen_eps = isfinite(esf) ? esf : FLT_MAX;
  // MFMA screen (nn_mfma_kernel): the same key from fp16 hi/lo operands scaled
  // by S = s16, in S² units.  Per coordinate a = −2Sq, t = St split as x = xh + xl + r with
  // |r| ≤ u16²|x| + 2σ (u16 = 2⁻¹¹, σ = 2⁻²⁵ fp16 subnormal half-spacing); the dropped al·tl and
  // the split remainders cost ≤ 3u16²|a||t| + 4σ(|a| + |t|) per coordinate, the w = S²|t|² split
  // u16²|w| + 2σ; the 11 exact fp16 products are accumulated in fp32 by the MFMA in an
  // unspecified order: ≤ 32·u·Σ|products| (a bound for ≤ 16 additions even if each rounds by a
  // full ulp).  Back in unscaled units (÷ S²) plus the stored-|t|² rounding u·|t|².
  const double S = f.s16;
  const double As = 2.0 * Q * S, Ts = qinf * S;
  const double Ws = 3.0 * Ts * Ts * (1.0 + 1e-6);
  const double u16 = 4.8828125e-04, sig = 2.98023223876953125e-08;
  const double P = 3.0 * As * Ts;
  const double Esplit = 3.0 * u16 * u16 * P + 4.0 * sig * 3.0 * (As + Ts) + u16 * u16 * Ws + 2.0 * sig;
  const double Eacc = 32.0 * kU * 1.01 * (P + Ws);
  const double E1m = 1.05 * (Esplit + Eacc) / (S * S) + kU * 3.0 * qinf * qinf;
  const double esm = 2.0 * (E1m + 6.0 * kU * (double)hi + 12.0 * kU * Q * Q) + 1e-30;
  const float esmf = f32_ru(esm);
  s->screen_eps_m = isfinite(esmf) ? esmf : FLT_MAX;
  s->mfma_scale = (float)S;
  // operands must stay well inside the fp16 range (max 65504) and the bound finite
  s->mfma_ok = (As < 16384.0 && Ts < 16384.0 && Ws < 16384.0 && isfinite(esmf) &&
                hi < FLT_MAX && esmf < 0.25f * FLT_MAX) ? 1 : 0;
}

__device__ void refresh_rt32(IcpState* s, const FrameParams& f) {
  double T[16];
  for (int k = 0; k < 16; ++k) T[k] = s->T[k];
  refresh_rt32_from(s, T, s->r2, sqrt(s->r2), f, s->iters);
}

__device__ __forceinline__ void set_identity(double* M) {
  for (int k = 0; k < 16; ++k) M[k] = (k % 5 == 0) ? 1.0 : 0.0;
}

// apply_init: the points start as init·p (the loop's pcd64 holds p, dT = init); 0: as p (dT = I),
// Open3D's RegistrationICP for an init that isIdentity() — T still starts at init
__global__ void icp_init_kernel(IcpState* s, double T0, double T1, double T2, double T3, double T4,
                                double T5, double T6, double T7, double T8, double T9, double T10,
                                double T11, double r2, FrameParams f, int apply_init) {
  if (threadIdx.x != 0) return;
  const double T[12] = {T0, T1, T2, T3, T4, T5, T6, T7, T8, T9, T10, T11};
  for (int k = 0; k < 12; ++k) s->T[k] = T[k];
  s->T[12] = s->T[13] = s->T[14] = 0.0;
  s->T[15] = 1.0;
  for (int k = 0; k < 16; ++k) s->dT[k] = apply_init ? s->T[k] : ((k % 5 == 0) ? 1.0 : 0.0);
  set_identity(s->last_upd);
  s->fitness = s->rmse = s->prev_fitness = s->prev_rmse = 0.0;
  s->count = 0;
  s->evals = s->iters = s->done = s->converged = 0;
  s->ticket = 0;
  s->r2 = r2;
  s->bound_ok = 0;
  refresh_rt32(s, f);
  s->eq_prev = s->eq;
}

// state for evaluating transform T (device, row-major 4×4): feature-RANSAC validation (a6)
__global__ void icp_set_T_kernel(IcpState* s, const double* __restrict__ T, double r2, FrameParams f) {
  if (threadIdx.x != 0) return;
  for (int k = 0; k < 16; ++k) s->T[k] = s->dT[k] = T[k];  // the loop's pcd64 holds p
  set_identity(s->last_upd);
  s->fitness = s->rmse = s->prev_fitness = s->prev_rmse = 0.0;
  s->count = 0;
  s->evals = s->iters = s->done = s->converged = 0;
  s->ticket = 0;
  s->r2 = r2;
  s->bound_ok = 0;  // keys/corr of another transform: no bound seeds until the next update
  refresh_rt32(s, f);
  s->eq_prev = s->eq;
}

// a6 batched validation (grid.hip validate_kernel): one evaluation state per hypothesis, with
// icp_set_T's semantics, for the hypotheses list[0..n) of the transform array T
__global__ __launch_bounds__(64) void val_states_kernel(IcpState* __restrict__ states,
                                                        const double* __restrict__ T,
                                                        const int32_t* __restrict__ list, int64_t n,
                                                        double r2, FrameParams f) {
  const int64_t k = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (k >= n) return;
  IcpState* s = states + k;
  const double* Th = T + 16 * (int64_t)list[k];
  for (int j = 0; j < 16; ++j) s->T[j] = s->dT[j] = Th[j];  // validation reads the source itself
  s->fitness = s->rmse = s->prev_fitness = s->prev_rmse = 0.0;
  s->count = 0;
  s->evals = s->iters = s->done = s->converged = 0;
  s->ticket = 0;
  s->r2 = r2;
  s->bound_ok = 0;
  refresh_rt32(s, f);
  s->eq_prev = s->eq;
}

// ------------------------------------------------------------------------------- keyinit
__global__ __launch_bounds__(256) void keyinit_kernel(const float4* __restrict__ src32, int64_t ns,
                                                      const float4* __restrict__ tgt32,
                                                      int64_t nt_shard, int64_t off,
                                                      const IcpState* __restrict__ s,
                                                      const int32_t* __restrict__ prev,
                                                      const int64_t* __restrict__ dprev,
                                                      int64_t* __restrict__ keys,
                                                      uint32_t* __restrict__ near2, int64_t q0) {
  // keys ← seed_key (nnkey.h), near2 ← none; sources [q0, ns)
  if (s->done) return;
  const int64_t i = q0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ns) return;
  const float* Rt = s->Rt32;  // uniform → scalar loads (a local copy went to scratch)
  const float4 p = src32[i];
  float x, y, z;
  xform32(Rt, p, x, y, z);
  keys[i] = seed_key(s, i, p, x, y, z, tgt32, nt_shard, off, prev, dprev);
  near2[i] = kNearNone;
}

// ------------------------------------------------------------------------------- NN scan
// fp32 VALU form of the brute-force scan (fallback: a target without MFMA tiles).  Per query
// the scan state (k1, near2) of nnkey.h; the screen bound is search_bound(k1).
__global__ __launch_bounds__(kNNBlock) void nn_kernel(const float4* __restrict__ src32, int64_t ns,
                                                      const float4* __restrict__ tgt,
                                                      int64_t nt_pad, int64_t slice_len,
                                                      int64_t off, const IcpState* __restrict__ s,
                                                      int64_t* __restrict__ keys,
                                                      uint32_t* __restrict__ near2) {
  if (s->done) return;
  const float* Rt = s->Rt32;  // uniform → scalar loads (a local copy went to scratch)
  const float r2_hi = s->r2_hi, be = s->band_e;
  const float eps = s->screen_eps;
  // per query: q (exact-path coordinates), a = −2q (screen), qq = |q|², scan state (k1, k1d,
  // n2) and the screen threshold thr = search_bound(k1) − qq + eps (inactive: never fires)
  float qx[kNNQ], qy[kNNQ], qz[kNNQ], ax[kNNQ], ay[kNNQ], az[kNNQ], qq[kNNQ], thr[kNNQ];
  float k1d[kNNQ], n2[kNNQ];
  uint64_t k1[kNNQ], k10[kNNQ];
  int64_t qi[kNNQ];
#pragma unroll
  for (int q = 0; q < kNNQ; ++q) {
    const int64_t i = (int64_t)blockIdx.x * (kNNBlock * kNNQ) + q * kNNBlock + threadIdx.x;
    qi[q] = i;
    n2[q] = kInf;
    float X = -1.0f;
    if (i < ns) {
      xform32(Rt, src32[i], qx[q], qy[q], qz[q]);
      const int64_t key = keys[i];
      k1[q] = key == kKeyNone ? make_key(r2_hi, 0xFFFFFFFFu) : (uint64_t)key;
      X = search_bound(key_d2(k1[q]), be, r2_hi);
    } else {
      qx[q] = qy[q] = qz[q] = 0.0f;
      k1[q] = (uint64_t)kKeyNone;
    }
    k10[q] = k1[q];
    k1d[q] = key_real_d2(k1[q]);
    ax[q] = -2.0f * qx[q];
    ay[q] = -2.0f * qy[q];
    az[q] = -2.0f * qz[q];
    qq[q] = fmaf(qz[q], qz[q], fmaf(qy[q], qy[q], qx[q] * qx[q]));
    thr[q] = X < 0.0f ? -FLT_MAX : (X - qq[q]) + eps;
  }
  // Targets are staged through LDS (double-buffered tiles of kNNLds points): every wave reads
  // each target with one broadcast ds_read_b128 into VGPRs, so the FMAs have no SGPR operand
  // (an SGPR source costs 1.65x issue time on gfx950, tools/ubench_valu.hip).
  __shared__ float4 tile[2][kNNLds];
  const int64_t jb = (int64_t)blockIdx.y * slice_len;
  const int64_t je = min(nt_pad, jb + slice_len);
#pragma unroll
  for (int r = 0; r < kNNLds / kNNBlock; ++r)
    tile[0][r * kNNBlock + threadIdx.x] = tgt[jb + r * kNNBlock + threadIdx.x];
  __syncthreads();
  int buf = 0;
  for (int64_t j0 = jb; j0 < je; j0 += kNNLds) {
    // next tile: global loads issued now, written to the other buffer after this tile
    const bool has_next = j0 + kNNLds < je;
    float4 pre[kNNLds / kNNBlock];
    if (has_next) {
#pragma unroll
      for (int r = 0; r < kNNLds / kNNBlock; ++r) pre[r] = tgt[j0 + kNNLds + r * kNNBlock + threadIdx.x];
    }
    const float4* tl = tile[buf];
    for (int sb = 0; sb < kNNLds; sb += kNNTile) {
      // Screen: key = |t|² − 2 q·t (3 FMA per pair, |t|² precomputed in t.w) differs from
      // d² − |q|² by at most eps, so any target whose exact d² could reach the search bound has
      // key ≤ thr.  Sub-tiles whose screen minimum stays above thr are skipped exactly.
      float m[kNNQ];
#pragma unroll
      for (int q = 0; q < kNNQ; ++q) m[q] = FLT_MAX;
#pragma unroll
      for (int k = 0; k < kNNTile; ++k) {
        const float4 t = tl[sb + k];
#pragma unroll
        for (int q = 0; q < kNNQ; ++q)
          m[q] = fminf(m[q], fmaf(ax[q], t.x, fmaf(ay[q], t.y, fmaf(az[q], t.z, t.w))));
      }
      // one (almost always not-taken) branch per sub-tile for all queries
      bool hit = false;
#pragma unroll
      for (int q = 0; q < kNNQ; ++q) hit = hit || (m[q] <= thr[q]);
      if (!__any(hit)) continue;
#pragma unroll
      for (int q = 0; q < kNNQ; ++q) {
        if (__any(m[q] <= thr[q])) {
          // exact path: direct fp32 d², scan-state update
#pragma unroll
          for (int k = 0; k < kNNTile; ++k) {
            const float4 t = tl[sb + k];
            const float d2 = d2f(qx[q], qy[q], qz[q], t.x, t.y, t.z);
            if (d2 <= r2_hi)
              near_push(k1[q], k1d[q], n2[q], make_key(d2, (uint32_t)(off + j0 + sb + k)), d2);
          }
          if (qi[q] < ns) thr[q] = (search_bound(key_d2(k1[q]), be, r2_hi) - qq[q]) + eps;
        }
      }
    }
    if (has_next) {
#pragma unroll
      for (int r = 0; r < kNNLds / kNNBlock; ++r) tile[buf ^ 1][r * kNNBlock + threadIdx.x] = pre[r];
    }
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int q = 0; q < kNNQ; ++q)
    if (qi[q] < ns && (k1[q] != k10[q] || n2[q] < kInf))
      near_publish((unsigned long long*)&keys[qi[q]], &near2[qi[q]], k1[q], n2[q], k1[q] != k10[q]);
}

// ------------------------------------------------------------------------------- NN, MFMA screen
// The screen key |t|² − 2q·t is a rank-4 contraction over (x, y, z, 1): here it runs on the
// matrix cores.  One v_mfma_f32_32x32x16_f16 computes S²·(key − thr) for 32 targets (A rows) ×
// 32 queries (B columns) from fp16 hi/lo splits of the S-scaled operands, K = 16:
//   A (target) = [xh, xh, xl, yh, yh, yl, zh, zh | zl, wh, wl, 1,   1,   0, 0, 0]
//   B (query)  = [ah, al, ah, bh, bl, bh, ch, cl | ch, 1,  1,  −Th, −Tl, 0, 0, 0]
// (a,b,c) = −2S·q; Th + Tl = the query's threshold S²·thr split in fp16 (thr_split).  Products
// of fp16 are exact in fp32; the bound on the key error is screen_eps_m (refresh_rt32) plus the
// threshold terms' share of the accumulation and split error (thr_operand).  So a target can
// only be a candidate if its value is negative, and the screen is a sign test: per MFMA a lane
// ORs the bit patterns of its 16 values with v_bitop3_b32 — a full-rate 3-input op on gfx950,
// where v_min3/v_minimum3/v_or3 issue at half rate (tools/ubench_ops.hip) — and tests bit 31.
// A lane holds column c = lane & 31 (its query) and 16 of the 32 rows; the lane pair (c, c + 32)
// covers all 32.  A sub-tile that hits anywhere in the wave runs the fp32 exact path of
// nn_kernel (direct d², lexicographic (d², index)) over the lane's 16 rows, and the pair merges
// its two states with one shuffle.  Result: the same key as nn_kernel and the grid search.
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kMG = 2;        // 32-query groups per wave
constexpr int kMTile = 256;   // targets per half tile (8 sub-tiles of 32)
constexpr int kTH = 4;        // half tiles per LDS tile
constexpr int kMTilePad = 1024; // MFMA operand arrays are padded to a multiple of every tile size
constexpr int kMBlock = 512;  // 8 waves × kMG × 32 = 512 queries per block: every target tile
                              // staged in LDS serves 512 queries (L2→LDS traffic per pair halved)
constexpr int kMQueries = (kMBlock / 64) * kMG * 32;  // queries per block

__device__ __forceinline__ void split16(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

union H8 {
  uint4 u;
  half8 h;
};

// Sign bits of 16 screen values ORed by a full-rate tree: 7 v_bitop3_b32 (a | b | c) + 1 v_or.
__device__ __forceinline__ uint32_t or16(const floatx16& k) {
  const auto b = [&](int i) { return __float_as_uint(k[i]); };
  const uint32_t o0 = __builtin_amdgcn_bitop3_b32(b(0), b(1), b(2), 0xFE);
  const uint32_t o1 = __builtin_amdgcn_bitop3_b32(b(3), b(4), b(5), 0xFE);
  const uint32_t o2 = __builtin_amdgcn_bitop3_b32(b(6), b(7), b(8), 0xFE);
  const uint32_t o3 = __builtin_amdgcn_bitop3_b32(b(9), b(10), b(11), 0xFE);
  const uint32_t o4 = __builtin_amdgcn_bitop3_b32(b(12), b(13), b(14), 0xFE);
  const uint32_t o5 = __builtin_amdgcn_bitop3_b32(o0, o1, o2, 0xFE);
  const uint32_t o6 = __builtin_amdgcn_bitop3_b32(o3, o4, b(15), 0xFE);
  return o5 | o6;
}

// The query's threshold as B operand elements 11-12 (lane half 1), in S² units.  thr0 =
// ((best − |q|²) + eps)·S² carries the key's error bound; the threshold terms add their own
// share of the MFMA's accumulation bound (32u·|thr|, as for the other products) and of the fp16
// split (u16²|thr| + σ), with 5 % slack that also covers this sum's fp32 rounding, so that every
// candidate's value is strictly negative.  |thr| is clamped to 32768 (fp16 range): clamping a
// negative threshold up only adds false hits; a positive threshold that large (radius far
// beyond the cloud's extent) sets `force`, and the group then runs the exact path everywhere.
__device__ __forceinline__ void thr_operand(half8& b, float thr0, bool& force) {
  const float extra = 1.05f * ((32.0f * 1.01f * 5.9604645e-08f + 2.3841858e-07f) * fabsf(thr0) +
                               5.9604645e-08f);
  float thr = thr0 + extra;
  force = thr > 32768.0f;
  thr = fminf(fmaxf(thr, -32768.0f), 32768.0f);
  const _Float16 th = (_Float16)thr;
  const _Float16 tl = (_Float16)(thr - (float)th);
  b[3] = -th;
  b[4] = -tl;
}

// MFMA screen operands of a cloud in its grid's cell order (A rows of nn_mfma_kernel):
// mf16 = fp16 split (+ the two constant-1 threshold slots), mf32 = (x, y, z, original index
// bits).  Pads: key 65504 (never hit),
// far-away coordinates (never accepted by the exact path).
__global__ __launch_bounds__(256) void pack16_sorted_kernel(const float4* __restrict__ sorted,
                                                            const float4* __restrict__ xyz32,
                                                            int64_t n, int64_t n_pad, float S,
                                                            uint4* __restrict__ mf16,
                                                            float4* __restrict__ mf32) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n_pad) return;
  H8 a, b;
  a.u = make_uint4(0, 0, 0, 0);
  b.u = make_uint4(0, 0, 0, 0);
  if (k < n) {
    const int32_t idx = __float_as_int(sorted[k].w);
    const float4 t = xyz32[idx];  // w = |t|² (center_pack)
    _Float16 xh, xl, yh, yl, zh, zl, wh, wl;
    split16(t.x * S, xh, xl);
    split16(t.y * S, yh, yl);
    split16(t.z * S, zh, zl);
    split16(t.w * (S * S), wh, wl);
    a.h = half8{xh, xh, xl, yh, yh, yl, zh, zh};
    b.h = half8{zl, wh, wl, (_Float16)1, (_Float16)1, (_Float16)0, (_Float16)0, (_Float16)0};
    mf32[k] = make_float4(t.x, t.y, t.z, __int_as_float(idx));
  } else {
    b.h[1] = (_Float16)65504.0f;  // value ≥ 65504 − 32768 > 0: never a hit
    b.h[3] = (_Float16)1;
    b.h[4] = (_Float16)1;
    mf32[k] = make_float4(1.0e18f, 1.0e18f, 1.0e18f, __int_as_float(-1));
  }
  mf16[k] = a.u;  // two planes: elements 0-7 (lane half 0), elements 8-15 (lane half 1)
  mf16[n_pad + k] = b.u;
}

hipError_t build_mfma_tiles(const m3d_cloud* c, Grid* g, hipStream_t st) {
  const int64_t n = c->n;
  const int64_t n_pad = std::max<int64_t>((n + kMTilePad - 1) / kMTilePad * kMTilePad, kMTilePad);
  hipError_t e = block_alloc(reinterpret_cast<void**>(&g->mf16), sizeof(uint4) * 2 * n_pad, st);
  if (e == hipSuccess) e = block_alloc(reinterpret_cast<void**>(&g->mf32), sizeof(float4) * n_pad, st);
  if (e != hipSuccess) return e;
  g->mf_npad = n_pad;
  pack16_sorted_kernel<<<(unsigned)((n_pad + 255) / 256), 256, 0, st>>>(
      g->pts, c->xyz32, n, n_pad, (float)c->s16, g->mf16, g->mf32);
  return hipGetLastError();  // asynchronous (stream order); m3d_icp_create synchronises once
}

// Self-seeding (single-device fused loop, m3d_icp_step): the fused tail of the previous
// iteration left every key at kKeyNone, so instead of a keyinit launch every block computes
// its queries' starting key itself (nnkey.h seed_key: the previous correspondence, exact — one
// target load per query) and the blocks of grid.y == 0 also publish it; the MIN over the
// blocks' atomics is the keyinit → scan result bit for bit.
struct SeedArgs {
  const int32_t* prev;  // corr of the previous evaluation
  const float4* tgt;    // the target cloud's centred fp32 points, original order
  int64_t nt;           // its size
  int on;
};

__device__ __forceinline__ int64_t start_key(const SeedArgs& sa, const IcpState* __restrict__ s,
                                             int64_t i, float4 p, float qx, float qy, float qz,
                                             int64_t off, const int64_t* __restrict__ keys) {
  return sa.on ? seed_key(s, i, p, qx, qy, qz, sa.tgt, sa.nt, off, sa.prev, nullptr) : keys[i];
}

// whether a block publishes its k1: it changed, or (self-seeding) the grid.y = 0 blocks publish
// the seed every block started from
__device__ __forceinline__ bool publish_k1(const SeedArgs& sa, uint64_t k1, uint64_t k10) {
  return k1 != k10 || (sa.on && blockIdx.y == 0 && key_real(k1));
}

// Exact fallback of nn_mfma_kernel when the scaled operands do not fit fp16 (mfma_ok == 0, a
// far-off transform): the same scan state over the block's slice by a plain scan, one thread
// per query.  Keeps the fp32 VALU kernel off the launch path.
__device__ void nn_slice_scan(const float4* __restrict__ src32, int64_t ns, const float4* __restrict__ tgt32,
                              int64_t jb, int64_t je, int64_t off, const IcpState* __restrict__ s,
                              int64_t* __restrict__ keys, uint32_t* __restrict__ near2,
                              const SeedArgs& sa, int64_t q0) {
  const float* Rt = s->Rt32;
  const float r2_hi = s->r2_hi;
  for (int qs = threadIdx.x; qs < kMQueries; qs += kMBlock) {
    const int64_t slot = q0 + (int64_t)blockIdx.x * kMQueries + qs;
    if (slot >= ns) return;
    const int64_t i = slot;
    float qx, qy, qz;
    const float4 p = src32[i];
    xform32(Rt, p, qx, qy, qz);
    const int64_t key = start_key(sa, s, i, p, qx, qy, qz, off, keys);  // keyinit's starting key
    uint64_t k1 = key == kKeyNone ? make_key(r2_hi, 0xFFFFFFFFu) : (uint64_t)key;
    float k1d = key_real_d2(k1), n2 = kInf;
    const uint64_t k10 = k1;
    for (int64_t j = jb; j < je; ++j) {
      const float4 t = tgt32[j];
      if (__float_as_int(t.w) < 0) continue;  // pad
      const float d2 = d2f(qx, qy, qz, t.x, t.y, t.z);
      if (d2 <= r2_hi) near_push(k1, k1d, n2, make_key(d2, (uint32_t)(off + __float_as_int(t.w))), d2);
    }
    const bool pk = publish_k1(sa, k1, k10);
    if (pk || n2 < kInf) near_publish((unsigned long long*)&keys[i], &near2[i], k1, n2, pk);
  }
}

// Exact fp32 pass of nn_mfma_kernel over one flagged sub-tile (32 targets from `rows`), of which
// this lane takes its 16 MFMA rows: direct d² pushed into the lane's scan state.  Pads: far
// coordinates, d² ~ 1e36 > r2_hi.
__device__ __forceinline__ void nn_exact_rows(const float4* __restrict__ rows, int64_t off, int h,
                                              float qx, float qy, float qz, float r2_hi,
                                              uint64_t& k1, float& k1d, float& n2) {
  float4 t[16];  // all 16 loads in flight before the first use (one memory latency per sub-tile)
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) t[reg] = rows[(reg & 3) + 8 * (reg >> 2) + 4 * h];
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const float d2 = d2f(qx, qy, qz, t[reg].x, t[reg].y, t[reg].z);
    const uint64_t kc = make_key(d2, (uint32_t)(off + __float_as_int(t[reg].w)));
    if (d2 <= r2_hi) near_push(k1, k1d, n2, kc, d2);
  }
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

__global__ __launch_bounds__(kMBlock) __attribute__((amdgpu_waves_per_eu(4))) void nn_mfma_kernel(const float4* __restrict__ src32,
                                                          int64_t ns,
                                                          const uint4* __restrict__ tgt16,
                                                          const float4* __restrict__ tgt32,
                                                          int64_t nt_pad, int64_t off,
                                                          const IcpState* __restrict__ s,
                                                          int64_t* __restrict__ keys,
                                                          uint32_t* __restrict__ near2,
                                                          SeedArgs sa, int64_t q0) {
  if (s->done) return;
  // grid.y block y takes every gridDim.y-th target tile (strided: a query block's few candidate
  // tiles, adjacent in cell order, spread over gridDim.y blocks instead of landing in one)
  const int64_t tstep = (int64_t)gridDim.y * kTH * kMTile;
  const int64_t jb = (int64_t)blockIdx.y * kTH * kMTile;
  if (!s->mfma_ok) {  // the same tiles by a plain scan
    for (int64_t t0 = jb; t0 < nt_pad; t0 += tstep)
      nn_slice_scan(src32, ns, tgt32, t0, min(nt_pad, t0 + kTH * kMTile), off, s, keys, near2, sa, q0);
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const float* Rt = s->Rt32;
  const float r2_hi = s->r2_hi, eps = s->screen_eps_m, S = s->mfma_scale, be = s->band_e;
  const float S2 = S * S;
  float qx[kMG], qy[kMG], qz[kMG], qq[kMG];
  uint32_t force = 0;  // groups whose threshold exceeds the fp16 range: exact path everywhere
  uint32_t act = 0;    // groups whose query (column c) exists
  uint64_t k1[kMG], k10[kMG];
  float k1d[kMG], n2[kMG];
  int64_t qi[kMG];
  half8 bq[kMG];
#pragma unroll
  for (int g = 0; g < kMG; ++g) {
    // queries: positions [q0, ns) of the visit order (order, or the slots themselves)
    const int64_t slot = q0 + (int64_t)blockIdx.x * kMQueries + (wave * kMG + g) * 32 + c;
    const int64_t i = slot < ns ? slot : -1;
    qi[g] = i;
    n2[g] = kInf;
    float X = -1.0f;  // inactive: negative threshold, never hits
    if (i >= 0) {
      const float4 p = src32[i];
      xform32(Rt, p, qx[g], qy[g], qz[g]);
      const int64_t key = start_key(sa, s, i, p, qx[g], qy[g], qz[g], off, keys);
      k1[g] = key == kKeyNone ? make_key(r2_hi, 0xFFFFFFFFu) : (uint64_t)key;
      X = search_bound(key_d2(k1[g]), be, r2_hi);
      act |= 1u << g;
    } else {
      qx[g] = qy[g] = qz[g] = 0.0f;
      k1[g] = (uint64_t)kKeyNone;
    }
    k10[g] = k1[g];
    k1d[g] = key_real_d2(k1[g]);
    qq[g] = fmaf(qz[g], qz[g], fmaf(qy[g], qy[g], qx[g] * qx[g]));
    _Float16 ah, al, bh, bl, ch, cl;
    split16(-2.0f * S * qx[g], ah, al);
    split16(-2.0f * S * qy[g], bh, bl);
    split16(-2.0f * S * qz[g], ch, cl);
    const _Float16 one = (_Float16)1.0f, zero = (_Float16)0.0f;
    bq[g] = h == 0 ? half8{ah, al, ah, bh, bl, bh, ch, cl} : half8{ch, one, one, zero, zero, zero, zero, zero};
    bool fg;
    half8 bt = bq[g];
    thr_operand(bt, X < 0.0f ? -1.0f : ((X - qq[g]) + eps) * S2, fg);  // × power of two: exact
    if (h == 1) bq[g] = bt;
    if (__any(fg)) force |= 0xFFu << (g * 8);
  }
  const floatx16 zacc = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f,
                         0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  // Deferred exact passes: a group whose every query starts from a real seed already screens
  // with (nearly) its final threshold, so its flagged sub-tiles need not be resolved inside the
  // tile — where one wave's exact pass holds the block's other 7 waves at the tile barrier —
  // but can wait in a per-wave list (tile offset, flagged bits) until after the sweep.  The
  // candidates evaluated are the same sub-tiles' rows, so the key is the same.
  uint32_t dfr = 0;
#pragma unroll
  for (int g = 0; g < kMG; ++g)
    if (!((force >> (g * 8)) & 1u) && __all(qi[g] < 0 || key_real(k1[g]))) dfr |= 1u << g;
  // Tiles of kTH × 256 targets, [buffer][lane half][target]: a half-wave's 32 ds_read_b128 hit
  // 32 consecutive 16-B slots.  Thread t stages kTH elements (e = t + u·512: plane e / kTT, target
  // e % kTT; mf16 is stored as two planes, so the loads are coalesced).  The sweep runs the tile
  // in halves of 8 sub-tiles (8 A-operand registers live), one barrier per tile.  The fp32
  // coordinates are read from global memory by the (rare) exact path only.
  constexpr int kTT = kTH * kMTile;
  constexpr int kSub = kTT / 32;                  // sub-tiles per tile
  constexpr uint64_t kGMask = (kSub == 64) ? ~0ull : ((1ull << kSub) - 1ull);
  static_assert(kMBlock == 2 * kMTile, "one 16-B operand half per thread per half tile");
  static_assert(kSub * kMG <= 64, "hit mask holds every (group, sub-tile)");
  __shared__ uint4 t16[2][2][kTT];
  constexpr int kDefer = 16;  // deferred entries per wave (more: resolved in the tile as before)
  __shared__ uint64_t dlist[kMBlock / 64][kDefer];  // flagged (group, sub-tile) bits
  __shared__ uint32_t dtile[kMBlock / 64][kDefer];  // their tile's first target
  int dn = 0;
  uint64_t dmask = 0;  // (group, sub-tile) bits of the deferring groups
#pragma unroll
  for (int g = 0; g < kMG; ++g)
    if ((dfr >> g) & 1u) dmask |= kGMask << (g * kSub);
  dmask = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(dmask >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)dmask);  // wave-uniform: SGPRs
  const int64_t je = nt_pad;
#pragma unroll
  for (int u = 0; u < kTH; ++u) {
    const int e = threadIdx.x + u * kMBlock;
    t16[0][e / kTT][e % kTT] = tgt16[(e / kTT) * nt_pad + jb + e % kTT];
  }
  uint64_t force64 = 0;
#pragma unroll
  for (int g = 0; g < kMG; ++g)
    if ((force >> (g * 8)) & 1u) force64 |= kGMask << (g * kSub);
  __syncthreads();
  int buf = 0;
  for (int64_t j0 = jb; j0 < je; j0 += tstep) {
    const bool has_next = j0 + tstep < je;
    // the next tile global → LDS by DMA while this one is swept (lds_dma.h): no prefetch
    // registers (a wave's 64 elements are one plane's 64 consecutive targets)
    if (has_next) {
#pragma unroll
      for (int u = 0; u < kTH; ++u) {
        const int e = threadIdx.x + u * kMBlock;
        lds_dma16(tgt16 + (e / kTT) * nt_pad + j0 + tstep + e % kTT, &t16[buf ^ 1][e / kTT][(e % kTT) & ~63]);
      }
    }
    // Sweep: MFMA + sign-OR test for the tile's sub-tiles, branch-free; a sub-tile that hits
    // anywhere in the wave sets a bit of the wave-uniform mask (SALU).  Software-pipelined: the
    // MFMA of step t+1 is issued before step t's tree, so a wave never waits on its own MFMA.
    uint64_t hm = 0;
    constexpr int kSteps = 8 * kMG;  // (sub-tile, group) steps of one half tile
#pragma unroll
    for (int half = 0; half < kTH; ++half) {
      H8 av[8];
#pragma unroll
      for (int sub = 0; sub < 8; ++sub) av[sub].u = t16[buf][h][half * kMTile + sub * 32 + c];
      floatx16 kc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[0].h, bq[0], zacc, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < kSteps; ++t) {
        floatx16 kn;
        if (t + 1 < kSteps)
          kn = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[(t + 1) / kMG].h, bq[(t + 1) % kMG], zacc, 0, 0, 0);
        // keep the pipeline the source states: without this fence the scheduler sinks each
        // MFMA next to its consumer (same accumulator registers, the VALU then waits out the
        // whole MFMA latency every step and the matrix pipe idles under the tree)
        __builtin_amdgcn_sched_barrier(0);
        // a candidate's value is strictly negative: OR of the 16 bit patterns, test bit 31
        const int g = t % kMG, sub = half * 8 + t / kMG;
        if (__any((int32_t)or16(kc) < 0)) hm |= 1ull << (g * kSub + sub);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < kSteps) kc = kn;
      }
    }
    // Exact path for the flagged (group, sub-tile) pairs, every lane (exact for any lane): direct
    // fp32 d² over the lane's 16 rows, then the lane pair (c, c + 32) merges its two states.
    // A group whose queries all start from a real seed defers its flagged sub-tiles to the
    // per-wave list below (dlist/dtile, resolved after the sweep, off the tile barrier:
    // −2.2 % per launch at cfg1); unseeded groups and a full list resolve here,
    // where the threshold refresh still prunes the rest of the sweep.
    hm |= force64;
    {
      const uint64_t hd = hm & dmask;
      if (hd != 0 && dn < kDefer) {
        if (lane == 0) {
          dlist[wave][dn] = hd;
          dtile[wave][dn] = (uint32_t)j0;
        }
        ++dn;
        hm &= ~hd;
      }
    }
#pragma unroll
    for (int g = 0; g < kMG; ++g) {
      uint64_t mg = (hm >> (g * kSub)) & kGMask;
      if (mg == 0) continue;
      while (mg != 0) {
        const int sub = __builtin_ctzll(mg);
        mg &= mg - 1;
        nn_exact_rows(tgt32 + j0 + sub * 32, off, h, qx[g], qy[g], qz[g], r2_hi, k1[g], k1d[g], n2[g]);
        const uint64_t o1 = shfl_xor64(k1[g], 32);
        const float on2 = __shfl_xor(n2[g], 32);
        near_merge(k1[g], k1d[g], n2[g], o1, on2);
      }
      bool fg;
      half8 bt = bq[g];
      const float X = (act >> g) & 1u ? search_bound(key_d2(k1[g]), be, r2_hi) : -1.0f;
      thr_operand(bt, X < 0.0f ? -1.0f : ((X - qq[g]) + eps) * S2, fg);
      if (h == 1) bq[g] = bt;  // the threshold only ever tightens: force stays as it was
    }
    lds_dma_wait();
    __syncthreads();
    buf ^= 1;
  }
  // the deferred exact passes (rows from global memory: the tiles have left LDS)
  for (int e = 0; e < dn; ++e) {
    const uint64_t ent = dlist[wave][e];
    const int64_t jt = (int64_t)dtile[wave][e];
#pragma unroll
    for (int g = 0; g < kMG; ++g) {
      uint64_t mg = (ent >> (g * kSub)) & kGMask;
      while (mg != 0) {
        const int sub = __builtin_ctzll(mg);
        mg &= mg - 1;
        nn_exact_rows(tgt32 + jt + sub * 32, off, h, qx[g], qy[g], qz[g], r2_hi, k1[g], k1d[g], n2[g]);
        const uint64_t o1 = shfl_xor64(k1[g], 32);
        const float on2 = __shfl_xor(n2[g], 32);
        near_merge(k1[g], k1d[g], n2[g], o1, on2);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < kMG; ++g) {
    if (h != 0 || qi[g] < 0) continue;
    const bool pk = publish_k1(sa, k1[g], k10[g]);
    if (pk || n2[g] < kInf)
      near_publish((unsigned long long*)&keys[qi[g]], &near2[qi[g]], k1[g], n2[g], pk);
  }
}

// ------------------------------------------------------------------------------- terms
// Transposing wave reduction of 32 per-lane slots: each butterfly step halves the slots a lane
// keeps (the partner gets the other half), so 32 slots cost 31 pair exchanges instead of
// 32 × 6 full butterflies.  Steps 32 and 16 use the gfx950 permlane swaps (no selects);
// 8, 4, 2 exchange by shuffles; the last step adds the two lanes of a pair.  Afterwards lanes
// 2k and 2k+1 both hold the wave's sum of slot k.  A fixed tree: deterministic.
template <bool k32>
__device__ __forceinline__ double swap_add(double a, double b) {
  const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
  const uint32_t alo = (uint32_t)ua, ahi = (uint32_t)(ua >> 32);
  const uint32_t blo = (uint32_t)ub, bhi = (uint32_t)(ub >> 32);
  const auto rl = k32 ? __builtin_amdgcn_permlane32_swap(alo, blo, false, false)
                      : __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
  const auto rh = k32 ? __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false)
                      : __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
  const double na = __longlong_as_double((long long)(((uint64_t)rh[0] << 32) | rl[0]));
  const double nb = __longlong_as_double((long long)(((uint64_t)rh[1] << 32) | rl[1]));
  return na + nb;  // lanes of bit 0: a-slot over both halves; bit 1: b-slot
}

#ifndef M3D_SUM_DPP
#define M3D_SUM_DPP 1
#endif
// v from lane ^ kOff (all lanes active): DPP for 1 and 2 (quad permutes), 4 (two moves, xor4_dpp)
// and 8 (a rotation by 8 inside a 16-lane row is lane ^ 8), without the LDS unit's round trip; a
// shuffle otherwise
template <int kOff>
__device__ __forceinline__ double xor_lane64(double v) {
  constexpr int ctrl = kOff == 1 ? 0xB1 : kOff == 2 ? 0x4E : kOff == 8 ? 0x128 : -1;
  if (M3D_SUM_DPP && M3D_DPP_X4 && kOff == 4) {
    const long long b = __double_as_longlong(v);
    const int lo = xor4_dpp((int)(uint32_t)b), hi = xor4_dpp((int)(uint32_t)(b >> 32));
    return __longlong_as_double(((long long)(uint32_t)hi << 32) | (uint32_t)lo);
  }
  if (M3D_SUM_DPP && ctrl >= 0) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, ctrl < 0 ? 0 : ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), ctrl < 0 ? 0 : ctrl, 0xF, 0xF, false);
    return __longlong_as_double(((long long)(uint32_t)hi << 32) | (uint32_t)lo);
  }
  return __shfl_xor(v, kOff, kWave);
}
template <int kOff>
__device__ __forceinline__ double xchg_add(double a, double b, int lane) {
  const bool hi = (lane & kOff) != 0;
  const double keep = hi ? b : a, send = hi ? a : b;
  return keep + xor_lane64<kOff>(send);
}

__device__ __forceinline__ double wave_transpose_sum32(const double (&v)[32], int lane) {
  double w16[16], w8[8], w4[4], w2[2];
#pragma unroll
  for (int j = 0; j < 16; ++j) w16[j] = swap_add<true>(v[j], v[j + 16]);
#pragma unroll
  for (int j = 0; j < 8; ++j) w8[j] = swap_add<false>(w16[j], w16[j + 8]);
#pragma unroll
  for (int j = 0; j < 4; ++j) w4[j] = xchg_add<8>(w8[j], w8[j + 4], lane);
#pragma unroll
  for (int j = 0; j < 2; ++j) w2[j] = xchg_add<4>(w4[j], w4[j + 2], lane);
  const double w1 = xchg_add<2>(w2[0], w2[1], lane);
  return w1 + xor_lane64<1>(w1);  // slot lane >> 1
}

// One source's contribution to the 30 term slots (layout below), in a fixed operation order:
// every terms pass (terms_block, single device or shard) adds a source through this function,
// so equal winners give equal bits.  Q = the fp64 transformed source, q / n its winner's point and
// normal, d2 = the winner's fp64 d², c = the source centre (point-to-point).
template <int kEst>
__device__ __forceinline__ void terms_add(double (&acc)[30], const double (&Q)[3], const double (&q)[3],
                                          const double (&n)[3], double d2, const double (&c)[3]) {
  const double d[3] = {Q[0] - q[0], Q[1] - q[1], Q[2] - q[2]};
  acc[28] += 1.0;
  acc[29] += d2;
  if (kEst == M3D_EST_POINT_TO_PLANE) {
    const double r = d[0] * n[0] + d[1] * n[1] + d[2] * n[2];
    double J[6];
    cross3(Q, n, J);
    J[3] = n[0];
    J[4] = n[1];
    J[5] = n[2];
    int k = 0;
#pragma unroll
    for (int x = 0; x < 6; ++x)
#pragma unroll
      for (int y = x; y < 6; ++y) acc[k++] += J[x] * J[y];
#pragma unroll
    for (int x = 0; x < 6; ++x) acc[21 + x] += J[x] * r;
    acc[27] += r * r;
  } else {
    const double pc[3] = {Q[0] - c[0], Q[1] - c[1], Q[2] - c[2]};
    const double qc[3] = {q[0] - c[0], q[1] - c[1], q[2] - c[2]};
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      acc[x] += pc[x];
      acc[3 + x] += qc[x];
#pragma unroll
      for (int y = 0; y < 3; ++y) acc[6 + 3 * x + y] += pc[x] * qc[y];
    }
  }
}

// Inputs of the terms pass.  Winner of source i:
//  * claim == nullptr (one device, or a source shard against the whole target): the fp64 winner
//    decided from the scan keys (nnkey.h winner_fp64; ambiguous queries resolved over the
//    target grid g);
//  * claim != nullptr (target shard, after the two MIN exchanges of m3d_icp_shard_*): claim[i],
//    the global winner (INT32_MAX none), whose fp64 d² every rank knows from dmin; the rank
//    owning the target adds its terms.  dmin is kept in dprev for the next bound seeds.
struct TermsArgs {
  double* pcd64;          // the loop's fp64 points: the query is dT·pcd64[i], written back (Open3D's
                          // pcd.Transform(update): the next update applies to these)
  const float4* src32;
  int64_t ns;
  const double* tgt64;
  const double* nrm64;
  const double* rec64;    // the target's 64-B records (point, normal), or null: tgt64 / nrm64
  int64_t nt_shard, off;
  const int64_t* keys;
  uint32_t* near2;
  GridDev g;
  const int32_t* claim;
  const int64_t* dmin;
  int64_t* dprev;
  int32_t* corr;
  int est;
  double c[3];
  int64_t* reset_keys;   // fused single-device loop: hand the keys back as kKeyNone
};

// est: M3D_EST_POINT_TO_PLANE → slots 0..20 JTJ (upper, row-major), 21..26 JTr, 27 Σr²
//      M3D_EST_POINT_TO_POINT → slots 0..2 Σp_c, 3..5 Σq_c, 6..14 Σ p_c q_cᵀ (row-major)
// both: 28 count, 29 Σd²  (c = source centre: identical on every shard)
// kWT: write the block partial through to memory (sc1 store) for the fused last-block reduce.
// kP sources per thread, in two load rounds so that a thread's chains overlap: (1) every
// source's key / runner-up / fp64 point (or claim / dmin), (2) after the fp64 decision, every
// winner's fp64 target (and normal); the rare ambiguous queries are resolved by the whole wave in
// between (nnkey.h resolve_wave, one ballot when there are none).
#if M3D_TAIL_CLOCK  // diagnostic builds only (tools/tail_clock.py): per-wave start / end of the
                    // terms pass, the last block's ticket, reduce and solve steps (100 MHz), and
                    // per wave the number of ambiguous queries it resolved
__device__ unsigned long long g_tail_clock[3 * 4096 + 24];  // + 16 finer stamps at 3·4096 + 8
#endif
#ifndef M3D_WALK64
#define M3D_WALK64 1  // build_grid_pts64 (0: resolve_wave gathers fp64 points after an fp32 screen)
#endif
#ifndef M3D_AMB_SKIP
#define M3D_AMB_SKIP 0  // timing only (wrong winners on ambiguous queries): their cost
#endif
// kEst: the estimator as a template parameter (one path compiled per kernel: a runtime branch
// between the two accumulation forms kept two accumulators in scratch memory)
#if M3D_TERMS_CLOCK  // diagnostic builds only (tools/terms_phases.py): per wave, stamps at the terms
                     // pass's phase ends, each after s_waitcnt 0 (the phases serialise), kept in
                     // registers and stored at the end
__device__ unsigned long long g_terms_clock[4096 * 8];
#define M3D_TPH(k)                               \
  do {                                           \
    __builtin_amdgcn_s_waitcnt(0);               \
    tph_[k] = __builtin_amdgcn_s_memrealtime();  \
  } while (0)
#else
#define M3D_TPH(k) \
  do {             \
  } while (0)
#endif
template <bool kWT, int kP, int kEst>
__device__ __forceinline__ void terms_block(const TermsArgs& a, const IcpState* __restrict__ s,
                                            double* __restrict__ partials) {
  __shared__ double red[kTermSlots][kTermsBlock / kWave];
#if M3D_TERMS_CLOCK
  unsigned long long tph_[8];
#endif
  M3D_TPH(0);
  double acc[30];
#pragma unroll
  for (int k = 0; k < 30; ++k) acc[k] = 0.0;
  int64_t ii[kP];
  bool valid[kP];
  double vs[kP][3];
  int64_t gj[kP];
  double d2[kP];
  bool fixed[kP];  // winner and d² already final (resolved in fp64, or given by the claim)
  uint64_t k1[kP];
  float n2[kP];
#pragma unroll
  for (int u = 0; u < kP; ++u) {
    const int64_t i = ((int64_t)blockIdx.x * kP + u) * kTermsBlock + threadIdx.x;
    valid[u] = i < a.ns;
    ii[u] = valid[u] ? i : 0;
    gj[u] = -1;
    d2[u] = 0.0;
    fixed[u] = true;
    if (a.claim == nullptr) {
      k1[u] = valid[u] ? (uint64_t)a.keys[ii[u]] : (uint64_t)kKeyNone;
      n2[u] = valid[u] ? __uint_as_float(a.near2[ii[u]]) : kInf;
    } else if (valid[u]) {
      const int32_t cj = a.claim[ii[u]];
      const int64_t dm = a.dmin[ii[u]];
      if (cj != 0x7FFFFFFF) {
        gj[u] = cj;
        d2[u] = __longlong_as_double(dm);
      }
      if (a.dprev != nullptr) a.dprev[ii[u]] = dm;
    }
    q64_of(s->dT, a.pcd64 + 3 * ii[u], vs[u]);
    if (valid[u])
      for (int k = 0; k < 3; ++k) a.pcd64[3 * ii[u] + k] = vs[u][k];
  }
  M3D_TPH(1);
  if (a.claim == nullptr) {
    bool amb[kP];
    float X[kP], qx[kP], qy[kP], qz[kP];
    int64_t bj[kP];
    double bd[kP];
#pragma unroll
    for (int u = 0; u < kP; ++u) {
      if (valid[u] && a.reset_keys != nullptr) {
        a.reset_keys[ii[u]] = kKeyNone;
        a.near2[ii[u]] = kNearNone;
      }
      // nnkey.h winner_fp64, split: ambiguous queries resolved here by the wave, the others'
      // candidate (k1's target) re-evaluated in fp64 after the batched target loads below
      X[u] = valid[u] && k1[u] != (uint64_t)kKeyNone ? search_bound(key_d2(k1[u]), s->band_e, s->r2_hi) : -1.0f;
      amb[u] = !M3D_AMB_SKIP && X[u] >= 0.0f && n2[u] <= X[u];
#if M3D_TAIL_CLOCK
      {
        const int64_t gw = (int64_t)blockIdx.x * (kTermsBlock / kWave) + threadIdx.x / kWave;
        const int na = __popcll(__ballot(amb[u]));
        if ((threadIdx.x & (kWave - 1)) == 0 && gw < 4096)
          g_tail_clock[2 * 4096 + 8 + gw] = (u == 0 ? 0ull : g_tail_clock[2 * 4096 + 8 + gw]) + na;
      }
#endif
      qx[u] = qy[u] = qz[u] = 0.0f;
      if (amb[u]) xform32(s->Rt32, a.src32[ii[u]], qx[u], qy[u], qz[u]);
      bj[u] = -1;
      bd[u] = 0.0;
    }
    // every source round's ambiguous queries in one walk, two at a time (nnkey.h)
    resolve_wave_kp<kP>(amb, a.g, a.tgt64, a.off, qx, qy, qz, X, vs, s->r2, bj, bd);
#pragma unroll
    for (int u = 0; u < kP; ++u) {
      if (amb[u]) {
        gj[u] = bj[u];
        d2[u] = bd[u];
      } else if (valid[u] && key_real(k1[u])) {
        const int64_t c = (int64_t)(uint32_t)k1[u];
        if (c >= a.off && c < a.off + a.nt_shard) {
          gj[u] = c;
          fixed[u] = false;
        }
      }
    }
  }
  M3D_TPH(2);
  double tq[kP][3], tn[kP][3];
#pragma unroll
  for (int u = 0; u < kP; ++u) {
    const bool own = valid[u] && gj[u] >= a.off && gj[u] < a.off + a.nt_shard;
    // branch-free: a source whose winner is not on this shard loads target 0 and drops it — but
    // an EMPTY target shard has no target 0 (no arrays at all): nothing is loaded there
    const int64_t l = own ? gj[u] - a.off : 0;
    if (a.nt_shard == 0) {
      for (int k = 0; k < 3; ++k) tq[u][k] = tn[u][k] = 0.0;
    } else if (a.rec64 != nullptr) {
      const double4 r0 = reinterpret_cast<const double4*>(a.rec64)[2 * l];
      const double4 r1 = reinterpret_cast<const double4*>(a.rec64)[2 * l + 1];
      tq[u][0] = r0.x;
      tq[u][1] = r0.y;
      tq[u][2] = r0.z;
      tn[u][0] = r0.w;
      tn[u][1] = r1.x;
      tn[u][2] = r1.y;
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        tq[u][k] = a.tgt64[3 * l + k];
        tn[u][k] = kEst == M3D_EST_POINT_TO_PLANE ? a.nrm64[3 * l + k] : 0.0;
      }
    }
  }
  M3D_TPH(3);
#pragma unroll
  for (int u = 0; u < kP; ++u) {
    if (!valid[u]) continue;
    if (!fixed[u]) {  // k1's target: the fp64 winner iff its d64 < r²
      const double d = d2_64(vs[u], tq[u]);
      if (d < s->r2) {
        d2[u] = d;
      } else {
        gj[u] = -1;
      }
    }
    const int64_t i = ii[u];
    if (a.corr != nullptr) a.corr[i] = (int32_t)gj[u];
    if (gj[u] < a.off || gj[u] >= a.off + a.nt_shard) continue;  // none, or another shard's target
    terms_add<kEst>(acc, vs[u], tq[u], tn[u], d2[u], a.c);
  }
  M3D_TPH(4);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  {
    double v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = k < 30 ? acc[k] : 0.0;
    const double w = wave_transpose_sum32(v, lane);
    if ((lane & 1) == 0) red[lane >> 1][wave] = w;
  }
  M3D_TPH(5);
  __syncthreads();
  M3D_TPH(6);
  if (threadIdx.x < kTermSlots) {
    double v = 0.0;
    if (threadIdx.x < 30)
      for (int w = 0; w < kTermsBlock / kWave; ++w) v += red[threadIdx.x][w];
    double* dst = partials + (int64_t)blockIdx.x * kTermSlots + threadIdx.x;
    if (kWT)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst), __double_as_longlong(v),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      *dst = v;
  }
  M3D_TPH(7);
#if M3D_TERMS_CLOCK
  {
    const int64_t gw = (int64_t)blockIdx.x * (kTermsBlock / kWave) + threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0 && gw < 4096)
      for (int k = 0; k < 8; ++k) g_terms_clock[8 * gw + k] = tph_[k];
  }
#endif
}

template <int kP, int kEst>
__global__ __launch_bounds__(kTermsBlock) void terms_kernel(TermsArgs a, const IcpState* __restrict__ s,
                                                            double* __restrict__ partials) {
  if (s->done) return;
  terms_block<false, kP, kEst>(a, s, partials);
}

// Target-sharded evaluation, step 1 (m3d_icp_shard_nn): this shard's fp64 winner of every query
// (winner_fp64 over the shard's targets) → lidx / ld64 and the exchange key dkey = bits(d64)
// (INT64_MAX none; d64 ≥ +0, so the integer MIN over ranks is the fp64 minimum).
__global__ __launch_bounds__(256) void shard_winner_kernel(
    const double* __restrict__ pcd64, const float4* __restrict__ src32, int64_t ns,
    const double* __restrict__ tgt64, int64_t nt_shard, int64_t off, GridDev g,
    const IcpState* __restrict__ s, const int64_t* __restrict__ keys,
    const uint32_t* __restrict__ near2, int32_t* __restrict__ lidx, int64_t* __restrict__ ld64,
    int64_t* __restrict__ dkey, int64_t q0) {
  if (s->done) return;
  const int64_t i0 = q0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = i0 < ns;
  const int64_t i = valid ? i0 : 0;
  // a query with no candidate on this shard (kKeyNone: e.g. every query whose box missed a spatial
  // shard's grid) has no winner here and is never ambiguous: its fp64 point and fp32 source are
  // not read (at 1M sources on one of 8 slabs, ~7/8 of the queries)
  const uint64_t k1 = valid ? (uint64_t)keys[i] : (uint64_t)kKeyNone;
  const bool need = k1 != (uint64_t)kKeyNone;
  double Q[3] = {0.0, 0.0, 0.0};
  if (need) q64_of(s->dT, pcd64 + 3 * i, Q);
  const float4 p32 = need ? src32[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  int64_t gj;
  double d;
  winner_fp64(valid, k1, need ? __uint_as_float(near2[i]) : kInf, s, g, tgt64, off, nt_shard, p32, Q, gj, d);
  if (!valid) return;
  const int64_t k = gj >= 0 ? __double_as_longlong(d) : kKeyNone;
  lidx[i] = (int32_t)gj;
  ld64[i] = k;
  dkey[i] = k;
}

// Step 2 (m3d_icp_shard_claim): after MIN(dkey) over ranks, the ranks whose own winner has the
// global minimum d64 claim it with their target index; MIN(claim) over ranks then breaks exact
// fp64 ties between shards by the lowest index (the lexicographic (d64, index) minimum).
__global__ __launch_bounds__(256) void shard_claim_kernel(int64_t ns, const IcpState* __restrict__ s,
                                                          const int32_t* __restrict__ lidx,
                                                          const int64_t* __restrict__ ld64,
                                                          const int64_t* __restrict__ dmin,
                                                          int32_t* __restrict__ claim) {
  if (s->done) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ns) return;
  claim[i] = (lidx[i] >= 0 && ld64[i] == dmin[i]) ? lidx[i] : 0x7FFFFFFF;
}

// ------------------------------------------------------------------------------- reduce
// 32 groups × 32 slots: group g sums blocks g, g+32, … (independent loads in flight), then the
// 32 group sums are added in group order — a fixed order, so the result is deterministic.
constexpr int kReduceGroups = 32;
__device__ __forceinline__ double group_sum(const double* __restrict__ partials, int64_t nblocks,
                                            int g, int slot) {
  double v = 0.0;
#pragma unroll 4
  for (int64_t b = g; b < nblocks; b += kReduceGroups) v += partials[b * kTermSlots + slot];
  return v;
}

__global__ __launch_bounds__(kReduceGroups * kTermSlots) void reduce_kernel(
    const double* __restrict__ partials, int64_t nblocks, double* __restrict__ sums,
    const IcpState* __restrict__ s) {
  if (s != nullptr && s->done) return;
  __shared__ double red[kReduceGroups][kTermSlots];
  const int slot = threadIdx.x & (kTermSlots - 1);
  const int g = threadIdx.x / kTermSlots;
  red[g][slot] = group_sum(partials, nblocks, g, slot);
  __syncthreads();
  if (threadIdx.x < kTermSlots) {
    double t = 0.0;
    for (int k = 0; k < kReduceGroups; ++k) t += red[k][threadIdx.x];
    sums[threadIdx.x] = t;
  }
}

// ------------------------------------------------------------------------------- solve
struct SolveParams {
  double rel_fit, rel_rmse;
  int max_iter, est;
  int64_t ns;
  double c[3];  // centre used by point-to-point sums
  FrameParams f;
};

// vec6_to_matrix with the three sincos evaluated in lanes 0..2 at once (whole wave calls it)
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// sin / cos of |a| ≤ 0.5 by their Taylor series in z = a² (Horner, sine to a¹⁷, cosine to a¹⁸: the
// first dropped terms are < 2e-20 relative), ≈ 2 ulp; an ICP update's angles are far inside this
#ifndef M3D_SMALL_SINCOS
#define M3D_SMALL_SINCOS 1
#endif
__device__ __forceinline__ void sincos_small(double a, double* sn, double* cs) {
  const double z = a * a;
  double ps = 1.0 / 355687428096000.0;  // 1/17!
  ps = fma(ps, z, -1.0 / 1307674368000.0);
  ps = fma(ps, z, 1.0 / 6227020800.0);
  ps = fma(ps, z, -1.0 / 39916800.0);
  ps = fma(ps, z, 1.0 / 362880.0);
  ps = fma(ps, z, -1.0 / 5040.0);
  ps = fma(ps, z, 1.0 / 120.0);
  ps = fma(ps, z, -1.0 / 6.0);
  double pc = 1.0 / 6402373705728000.0;  // 1/18!
  pc = fma(pc, z, -1.0 / 20922789888000.0);
  pc = fma(pc, z, 1.0 / 87178291200.0);
  pc = fma(pc, z, -1.0 / 479001600.0);
  pc = fma(pc, z, 1.0 / 3628800.0);
  pc = fma(pc, z, -1.0 / 40320.0);
  pc = fma(pc, z, 1.0 / 720.0);
  pc = fma(pc, z, -1.0 / 24.0);
  pc = fma(pc, z, 0.5);
  *sn = fma(a * z, ps, a);
  *cs = fma(-z, pc, 1.0);
}

__device__ __forceinline__ void vec6_to_matrix_wave(const double x[6], double T[16]) {
  const int lane = threadIdx.x & (kWave - 1);
  double sn, cs;
  const double ang = lane == 0 ? x[0] : (lane == 1 ? x[1] : x[2]);
  // x is the same in every lane: the branch is uniform
  if (M3D_SMALL_SINCOS && fmax(fabs(x[0]), fmax(fabs(x[1]), fabs(x[2]))) <= 0.5)
    sincos_small(ang, &sn, &cs);
  else
    sincos(ang, &sn, &cs);
  // lanes 0..2 hold the results: v_readlane into SGPRs (a ds_bpermute per half costs an LDS trip)
  vec6_to_matrix_sc(x, readlane_f64(cs, 0), readlane_f64(sn, 0), readlane_f64(cs, 1),
                    readlane_f64(sn, 1), readlane_f64(cs, 2), readlane_f64(sn, 2), T);
}

// The state fields the solve reads, loaded by solve_in — in the fused tail before the partial
// sums, so that their global round trip overlaps the reduction's.
struct SolveIn {
  int32_t evals, iters;
  double prev_fit, prev_rmse, r2;
  float eq;
  double T[16];
  float rt[12];
};

__device__ __forceinline__ void solve_in(const IcpState* s, SolveIn& in) {
  in.evals = s->evals;
  in.iters = s->iters;
  in.prev_fit = s->prev_fitness;
  in.prev_rmse = s->prev_rmse;
  in.r2 = s->r2;
  in.eq = s->eq;
#pragma unroll
  for (int k = 0; k < 16; ++k) in.T[k] = s->T[k];
#pragma unroll
  for (int k = 0; k < 12; ++k) in.rt[k] = s->Rt32[k];
}

#if M3D_TAIL_CLOCK
#define M3D_TCLK(k)                                                                   \
  do {                                                                                \
    if (threadIdx.x == 0)                                                             \
      g_tail_clock[(k) < 8 ? 2 * 4096 + (k) : 3 * 4096 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define M3D_TCLK(k) \
  do {              \
  } while (0)
#endif
template <int kEst>
__device__ void solve_state(const double* sums, IcpState* s, const SolveParams& sp, const SolveIn& in) {
  double sm[30];
#pragma unroll
  for (int k = 0; k < 30; ++k) sm[k] = sums[k];
  const int32_t evals = in.evals, iters = in.iters;
  const double prev_fit = in.prev_fit, prev_rmse = in.prev_rmse, r2 = in.r2;
  const float eq = in.eq;
  double T[16];
  float rt[12];
#pragma unroll
  for (int k = 0; k < 16; ++k) T[k] = in.T[k];
#pragma unroll
  for (int k = 0; k < 12; ++k) rt[k] = in.rt[k];
  const double count = sm[28];
  const double r = sqrt(in.r2);  // for refresh_rt32_from; independent of everything below
#ifndef M3D_SOLVE_SPEC
#define M3D_SOLVE_SPEC 1
#endif
  // point-to-plane: the unpivoted LDLT of JᵀJ does not depend on the convergence test, so it is
  // written first, in the same basic block as fitness / rmse, for the scheduler to interleave the
  // chains (measured neutral against M3D_SOLVE_SPEC=0, docs/EXPERIMENTS.md §R6; the same bits);
  // its result is used only if the loop goes on
  double A[36], b[6], x[6];
  bool spd_ok = false;
  if (M3D_SOLVE_SPEC && kEst == M3D_EST_POINT_TO_PLANE) {
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int c = a; c < 6; ++c) {
        A[a * 6 + c] = sm[k];
        A[c * 6 + a] = sm[k];
        ++k;
      }
#pragma unroll
    for (int a = 0; a < 6; ++a) b[a] = -sm[21 + a];
    spd_ok = ldlt6_solve_spd(A, b, x);  // straight-line; x garbage (unused) when it fails
  }
  const double fit = count > 0.0 ? count / (double)sp.ns : 0.0;
  const double rmse = count > 0.0 ? sqrt(sm[29] / count) : 0.0;
  M3D_TCLK(10);
  bool stop = false;
  if (evals > 0 && fabs(prev_fit - fit) < sp.rel_fit && fabs(prev_rmse - rmse) < sp.rel_rmse) {
    s->converged = 1;
    stop = true;
  } else if (iters >= sp.max_iter) {
    stop = true;
  }
  s->fitness = fit;
  s->rmse = rmse;
  s->count = (int64_t)count;
  s->prev_fitness = fit;
  s->prev_rmse = rmse;
  s->evals = evals + 1;
  if (stop) {
    s->done = 1;
    return;
  }
#if M3D_SOLVE_SKIP  // timing only: the solve's cost
  return;
#endif
  double upd[16];
  for (int k = 0; k < 16; ++k) upd[k] = (k % 5 == 0) ? 1.0 : 0.0;
  // the search transform of the evaluation just reduced: seed_key's bound for the next one
#pragma unroll
  for (int k = 0; k < 12; ++k) s->Rt32_prev[k] = rt[k];
  s->eq_prev = eq;
  s->bound_ok = sp.f.shared;  // bounds compare keys across ranks: only in a shared frame
  M3D_TCLK(11);
  if (count > 0.0) {
    if (kEst == M3D_EST_POINT_TO_PLANE) {
      if (!M3D_SOLVE_SPEC) {
        int k = 0;
        for (int a = 0; a < 6; ++a)
          for (int c = a; c < 6; ++c) {
            A[a * 6 + c] = sm[k];
            A[c * 6 + a] = sm[k];
            ++k;
          }
        for (int a = 0; a < 6; ++a) b[a] = -sm[21 + a];
      }
      M3D_TCLK(3);
#ifndef M3D_SOLVE_SPD
#define M3D_SOLVE_SPD 1
#endif
      // a full-rank JᵀJ unpivoted (no scalar-unit row swaps: 1.6 µs of the tail); a
      // (near-)singular one through Eigen's pivot order, which decides its zero components
      if (!M3D_SOLVE_SPEC) spd_ok = M3D_SOLVE_SPD && ldlt6_solve_spd(A, b, x);
      if (!spd_ok) ldlt6_solve(A, b, x);
      M3D_TCLK(4);
      vec6_to_matrix_wave(x, upd);
      M3D_TCLK(5);
    } else {
      const double n = count;
      double mp[3], mq[3], Hm[9], R[9];
      for (int a = 0; a < 3; ++a) {
        mp[a] = sm[a] / n;
        mq[a] = sm[3 + a] / n;
      }
      for (int a = 0; a < 3; ++a)
        for (int c = 0; c < 3; ++c) Hm[3 * a + c] = sm[6 + 3 * a + c] / n - mp[a] * mq[c];
      rotation_from_cov(Hm, R);
      for (int a = 0; a < 3; ++a) {
        const double mpw[3] = {mp[0] + sp.c[0], mp[1] + sp.c[1], mp[2] + sp.c[2]};
        for (int c = 0; c < 3; ++c) upd[4 * a + c] = R[3 * a + c];
        upd[4 * a + 3] = (mq[a] + sp.c[a]) - (R[3 * a] * mpw[0] + R[3 * a + 1] * mpw[1] + R[3 * a + 2] * mpw[2]);
      }
    }
  }
  bool finite = true;
  for (int k = 0; k < 16; ++k) finite = finite && isfinite(upd[k]);
  if (!finite)
    for (int k = 0; k < 16; ++k) upd[k] = (k % 5 == 0) ? 1.0 : 0.0;
  // T ← ΔT·T and the points ← ΔT·points (applied by the next evaluation's query, IcpState::dT)
#pragma unroll
  for (int k = 0; k < 16; ++k) s->dT[k] = s->last_upd[k] = upd[k];
  // both are affine (bottom row 0 0 0 1): the 12 products that are not 0 or 1 (the same sums as
  // matmul4 without its exact-zero terms)
  matmul4_affine(upd, T, T);
#pragma unroll
  for (int k = 0; k < 16; ++k) s->T[k] = T[k];
  s->iters = iters + 1;
  M3D_TCLK(6);
  refresh_rt32_from(s, T, r2, r, sp.f, iters + 1);
  M3D_TCLK(7);
}

template <int kEst>
__global__ void solve_kernel(const double* __restrict__ sums, IcpState* __restrict__ s,
                             SolveParams sp) {
  if (threadIdx.x >= kWave || s->done) return;
  SolveIn in;
  solve_in(s, in);
  solve_state<kEst>(sums, s, sp, in);
}

// Past 256 partials (the separate tail of a large source, 1M: 1,954 rows) the same order on 32
// blocks instead of one: block g adds group g (blocks g, g + 32, …; 32 loads in flight per batch),
// stores the group sum write-through into partials row g (a row only this block reads), drains it
// and takes the ticket; the last block adds rows 0..31 in group order with sc1 loads — the same
// sums, bit for bit, as reduce_kernel — and, for a single-device step (do_solve), runs the solve
// on them (solve_kernel's work without its launch).
template <int kEst>
__global__ __launch_bounds__(kTermSlots) void reduce_groups_kernel(double* __restrict__ partials,
                                                                   int64_t nblocks, double* __restrict__ sums,
                                                                   IcpState* __restrict__ s, SolveParams sp,
                                                                   int do_solve) {
  if (s->done) return;
  const int g = blockIdx.x, slot = threadIdx.x;
  double v = 0.0;
  for (int64_t b0 = g; b0 < nblocks; b0 += (int64_t)kReduceGroups * 32) {
    double t[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int64_t b = b0 + (int64_t)k * kReduceGroups;
      t[k] = b < nblocks ? partials[b * kTermSlots + slot] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (b0 + (int64_t)k * kReduceGroups < nblocks) v += t[k];
  }
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials + (int64_t)g * kTermSlots + slot),
                     __double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ int last;
  __syncthreads();
  if (slot == 0)
    last = __hip_atomic_fetch_add(&s->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (uint32_t)(kReduceGroups - 1);
  __syncthreads();
  if (!last) return;
  SolveIn in;
  if (do_solve) solve_in(s, in);  // its loads overlap the group rows'
  double tot = 0.0;
  for (int k = 0; k < kReduceGroups; ++k)
    tot += __longlong_as_double(__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(partials + (int64_t)k * kTermSlots + slot), __ATOMIC_RELAXED,
        __HIP_MEMORY_SCOPE_AGENT));
  sums[slot] = tot;
  __shared__ double out[kTermSlots];
  out[slot] = tot;
  __syncthreads();
  if (slot == 0) s->ticket = 0;
  if (do_solve) solve_state<kEst>(out, s, sp, in);
}

// Fused single-device iteration tail: terms → block partial → the last block to finish (ticket)
// reduces all partials in reduce_kernel's exact order and runs solve_state.  Cross-XCD hand-off
// (MI355X_MICROARCH.md, visibility table, "last adder" row): each block stores its partial
// write-through (sc1), drains it (vmcnt(0)) and one lane adds to the agent-scope ticket; the
// block whose add returned nblocks − 1 reads every partial with sc1 loads.  No L2 write-back or
// invalidate fences are needed.
template <int kP, int kEst>
__global__ __launch_bounds__(kTermsBlock) void terms_solve_kernel(
    TermsArgs a, IcpState* s, double* partials, int64_t nblocks, double* __restrict__ sums,
    SolveParams sp, int do_solve) {
  // do_solve = 0: the sharded tail (m3d_icp_shard_terms) — terms + the fixed-order reduce into
  // `sums` in one launch; the caller all-reduces them and runs m3d_icp_solve
  if (s->done) return;
#if M3D_TAIL_CLOCK
  const unsigned long long clk0 = __builtin_amdgcn_s_memrealtime();
#endif
  terms_block<true, kP, kEst>(a, s, partials);
#if M3D_TAIL_CLOCK
  {
    const unsigned long long clk1 = __builtin_amdgcn_s_memrealtime();
    const int64_t gw = (int64_t)blockIdx.x * (kTermsBlock / kWave) + threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0 && gw < 4096) {
      g_tail_clock[2 * gw] = clk0;
      g_tail_clock[2 * gw + 1] = clk1;
    }
  }
#endif
  __shared__ double red[kReduceGroups][kTermSlots];
  __shared__ int last;
  // the partial went out write-through (sc1): drain it, then one lane takes the ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t =
        __hip_atomic_fetch_add(&s->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == (uint32_t)(nblocks - 1));
  }
  __syncthreads();
  if (!last) return;
  M3D_TCLK(0);
  SolveIn in;
  if (do_solve && threadIdx.x < kWave) solve_in(s, in);
  // every load of the other blocks' partials is an sc1 load (L2-coherent, bypasses L1)
  const int slot = threadIdx.x & (kTermSlots - 1);
  constexpr int kG = kReduceGroups / (kTermsBlock / kTermSlots);  // groups per thread
  double gv[kG];
#pragma unroll
  for (int u = 0; u < kG; ++u) gv[u] = 0.0;
  const int g0 = threadIdx.x / kTermSlots;
  constexpr int kR = 8;  // rounds of kReduceGroups blocks in flight per batch (kR·kG loads):
                         // 256 blocks (cfg1: 196) in ONE batch of dependent loads
  for (int64_t b0 = 0; b0 < nblocks; b0 += kR * kReduceGroups) {
    double t[kR][kG];
#pragma unroll
    for (int r = 0; r < kR; ++r)
#pragma unroll
      for (int u = 0; u < kG; ++u) {
        const int64_t b = b0 + r * kReduceGroups + g0 + u * (kTermsBlock / kTermSlots);
        t[r][u] = b < nblocks
                      ? __longlong_as_double(__hip_atomic_load(
                            reinterpret_cast<unsigned long long*>(partials + b * kTermSlots + slot),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                      : 0.0;
      }
#pragma unroll
    for (int r = 0; r < kR; ++r)
#pragma unroll
      for (int u = 0; u < kG; ++u) gv[u] += t[r][u];
  }
  M3D_TCLK(8);  // thread 0's loads landed and added
#pragma unroll
  for (int u = 0; u < kG; ++u) red[g0 + u * (kTermsBlock / kTermSlots)][slot] = gv[u];
  __syncthreads();
  if (threadIdx.x < kTermSlots) {
    double t = 0.0;
    for (int k = 0; k < kReduceGroups; ++k) t += red[k][threadIdx.x];
    red[0][threadIdx.x] = t;  // row 0 is consumed by this thread only before the overwrite
    sums[threadIdx.x] = t;
  }
  M3D_TCLK(9);
  __syncthreads();
  M3D_TCLK(1);
  if (threadIdx.x < kWave) {
    if (threadIdx.x == 0) s->ticket = 0;
    if (do_solve) solve_state<kEst>(red[0], s, sp, in);
  }
  M3D_TCLK(2);
}

// finalize standalone NN (m3d_nn1): the fp64 winner (nnkey.h winner_fp64) and its d64
__global__ __launch_bounds__(256) void nn_finalize_kernel(const double* __restrict__ pcd64,
                                                          const float4* __restrict__ src32,
                                                          int64_t ns,
                                                          const double* __restrict__ tgt64,
                                                          int64_t nt, GridDev g,
                                                          const IcpState* __restrict__ s,
                                                          const int64_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ near2,
                                                          const int32_t* __restrict__ slot,
                                                          int32_t* __restrict__ idx,
                                                          double* __restrict__ d2out) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = i0 < ns;
  const int64_t i = valid ? i0 : 0;
  double Q[3];
  q64_of(s->dT, pcd64 + 3 * i, Q);
  int64_t gj;
  double d;
  winner_fp64(valid, valid ? (uint64_t)keys[i] : (uint64_t)kKeyNone,
              valid ? __uint_as_float(near2[i]) : kInf, s, g, tgt64, 0, nt, src32[i], Q, gj, d);
  if (!valid) return;
  const int64_t o = slot != nullptr ? (int64_t)slot[i] : i;  // slot → the caller's source order
  idx[o] = (int32_t)gj;
  if (d2out != nullptr) d2out[o] = gj >= 0 ? d : INFINITY;
}

__global__ void scatter_i32_kernel(const int32_t* __restrict__ v, const int32_t* __restrict__ slot,
                                   int64_t n, int32_t* __restrict__ dst) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n) dst[slot[k]] = v[k];
}

// ------------------------------------------------------------------------------- pairs
// The correspondence set (Open3D RegistrationResult.correspondence_set): (i, v[i]) for every i
// with v[i] ≥ 0, in increasing i.  An order-preserving compaction in three launches over chunks
// of 1024 entries (256 threads × 4, entry base + u·256 + t): per-chunk counts, one block's
// exclusive scan of the counts, placement (per-wave ballots, LDS prefix over the chunk's 16
// (u, wave) groups in index order).
constexpr int kPairChunk = 1024;

__global__ __launch_bounds__(256) void pair_count_kernel(const int32_t* __restrict__ v, int64_t n,
                                                         int32_t* __restrict__ cnt) {
  __shared__ int part[4];
  const int64_t base = (int64_t)blockIdx.x * kPairChunk;
  int c = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = base + u * 256 + threadIdx.x;
    c += __popcll(__ballot(i < n && v[i] >= 0));
  }
  if ((threadIdx.x & (kWave - 1)) == 0) part[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// one block: cnt[0..nb) → exclusive offsets in place, the total in cnt[nb]
__global__ __launch_bounds__(1024) void pair_scan_kernel(int32_t* __restrict__ cnt, int64_t nb) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t carry_s;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < nb; b0 += 1024) {
    const int64_t b = b0 + threadIdx.x;
    const int32_t x = b < nb ? cnt[b] : 0;
    int32_t incl = x;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int32_t y = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += y;
    }
    if (lane == kWave - 1) wsum[w] = incl;
    __syncthreads();
    int32_t before = carry_s;
    for (int k = 0; k < w; ++k) before += wsum[k];
    if (b < nb) cnt[b] = before + incl - x;
    __syncthreads();
    if (threadIdx.x == 1023) carry_s = before + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) cnt[nb] = carry_s;
}

__global__ __launch_bounds__(256) void pair_place_kernel(const int32_t* __restrict__ v, int64_t n,
                                                         const int32_t* __restrict__ off,
                                                         int32_t* __restrict__ pairs) {
  __shared__ int grp[16];  // popcount of group (u, wave), index order u·4 + wave
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int64_t base = (int64_t)blockIdx.x * kPairChunk;
  bool hit[4];
  int32_t val[4];
  uint64_t m[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = base + u * 256 + threadIdx.x;
    val[u] = i < n ? v[i] : -1;
    hit[u] = val[u] >= 0;
    m[u] = __ballot(hit[u]);
    if (lane == 0) grp[u * 4 + w] = __popcll(m[u]);
  }
  __syncthreads();
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int32_t o = off[blockIdx.x];  // entries of the chunk's rows before row u
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    int32_t before = o;
    for (int k = 0; k < w; ++k) before += grp[u * 4 + k];
    if (hit[u]) {
      const int32_t k = before + __popcll(m[u] & below);
      pairs[2 * (int64_t)k] = (int32_t)(base + u * 256 + threadIdx.x);
      pairs[2 * (int64_t)k + 1] = val[u];
    }
    for (int k = 0; k < 4; ++k) o += grp[u * 4 + k];
  }
}

__global__ void keys_to_idx_kernel(const int64_t* __restrict__ keys, int64_t n,
                                   int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) idx[i] = keys[i] == kKeyNone ? -1 : (int32_t)(uint32_t)keys[i];
}

// ------------------------------------------------------------------------------- launchers
static FrameParams frame_of(const m3d_icp* s) {
  FrameParams f;
  for (int k = 0; k < 3; ++k) {
    f.cs[k] = s->src->center[k];
    f.ct[k] = s->tgt->center[k];
  }
  f.pinf = s->src->rmax;
  f.qinf = s->tgt->rmax;
  f.s16 = s->tgt->s16;
  f.shared = s->tgt->center_given;
  return f;
}

// the loop's fp64 points start as the source itself (the init, if applied, is dT)
static hipError_t reset_points(const m3d_icp* s, hipStream_t st) {
  if (s->src->n == 0) return hipSuccess;
  return hipMemcpyAsync(s->pcd64, s->src->xyz64, sizeof(double) * 3 * s->src->n, hipMemcpyDeviceToDevice, st);
}

hipError_t launch_icp_reset(const m3d_icp* s, const double* T, bool apply_init, hipStream_t st) {
  hipError_t e = reset_points(s, st);
  if (e != hipSuccess) return e;
  icp_init_kernel<<<1, 64, 0, st>>>(s->state, T[0], T[1], T[2], T[3], T[4], T[5], T[6], T[7],
                                    T[8], T[9], T[10], T[11], s->max_dist * s->max_dist,
                                    frame_of(s), apply_init ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_icp_set_T(const m3d_icp* s, const double* T_dev, hipStream_t st) {
  hipError_t e = reset_points(s, st);
  if (e != hipSuccess) return e;
  icp_set_T_kernel<<<1, 64, 0, st>>>(s->state, T_dev, s->max_dist * s->max_dist, frame_of(s));
  return hipGetLastError();
}

// m3d_icp_copy_points: the loop's points in the caller's order.  Before the first evaluation the
// init is still in dT (pcd64 = the source): apply it as the evaluation will (q64_of, Eigen's
// order) — RegistrationICP's pcd at that point is init·source — unless dT is exactly I
// (init isIdentity(): Open3D leaves pcd untouched, and I·p could turn a −0 into +0).
__global__ void copy_points_kernel(const IcpState* __restrict__ s, const double* __restrict__ v,
                                   const int32_t* __restrict__ slot, int64_t n, double* __restrict__ dst) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const int64_t o = (int64_t)slot[k];
  bool apply = s->evals == 0;
  if (apply) {
    bool eye = true;
    for (int e = 0; e < 16; ++e) eye = eye && s->dT[e] == ((e % 5) == 0 ? 1.0 : 0.0);
    apply = !eye;
  }
  if (apply) {
    double q[3];
    q64_of(s->dT, v + 3 * k, q);
    for (int c = 0; c < 3; ++c) dst[3 * o + c] = q[c];
  } else {
    for (int c = 0; c < 3; ++c) dst[3 * o + c] = v[3 * k + c];
  }
}

hipError_t launch_copy_points(const m3d_icp* s, double* dst, hipStream_t st) {
  const int64_t n = s->src->n;
  if (n == 0) return hipSuccess;
  copy_points_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(s->state, s->pcd64, s->src->slot, n, dst);
  return hipGetLastError();
}

hipError_t launch_val_states(const m3d_icp* s, const double* T_dev, const int32_t* list, int64_t n,
                             IcpState* states, hipStream_t st) {
  if (n == 0) return hipSuccess;
  val_states_kernel<<<(unsigned)((n + 63) / 64), 64, 0, st>>>(states, T_dev, list, n,
                                                              s->max_dist * s->max_dist, frame_of(s));
  return hipGetLastError();
}

hipError_t launch_icp_keyinit(const m3d_icp* s, int64_t off, hipStream_t st, int64_t q0, int64_t q1) {
  const int64_t ns = q1 < 0 ? s->src->n : q1;
  if (ns <= q0) return hipSuccess;
  keyinit_kernel<<<(unsigned)((ns - q0 + 255) / 256), 256, 0, st>>>(
      s->src->xyz32, ns, s->tgt->xyz32, s->tgt->n, off, s->state, s->corr, s->dprev, s->keys,
      s->near2, q0);
  return hipGetLastError();
}

// target slices over grid.y so that ≥ ~2048 blocks fill the chip; slices ≥ 1024 targets and a
// multiple of `mult`
static dim3 nn_grid(int64_t bx, int64_t nt_pad, int64_t mult, int64_t* slice_out) {
  int64_t S = (2048 + bx - 1) / bx;
  const int64_t max_s = nt_pad / 1024 > 0 ? nt_pad / 1024 : 1;
  if (S > max_s) S = max_s;
  if (S < 1) S = 1;
  int64_t slice = (nt_pad + S - 1) / S;
  slice = (slice + mult - 1) / mult * mult;
  S = (nt_pad + slice - 1) / slice;
  *slice_out = slice;
  return dim3((unsigned)bx, (unsigned)S);
}

static bool icp_nn_uses_mfma(const m3d_icp* s) {
  return s->tgrid != nullptr && s->tgrid->mf16 != nullptr;
}

bool icp_nn_range_ok(const m3d_icp* s) {
  if (s->params.nn_method == M3D_NN_GRID) return s->sgrid != nullptr && s->sgrid->mpts != nullptr;
  return icp_nn_uses_mfma(s);
}

// Brute-force NN into s->keys (after launch_icp_keyinit, or self_seed: keys all kKeyNone, see
// SeedArgs).  MFMA tiles present: nn_mfma_kernel alone (its exact in-kernel scan covers
// transforms whose operands do not fit fp16); otherwise the fp32 VALU nn_kernel.
hipError_t launch_icp_nn(const m3d_icp* s, int64_t off, bool self_seed, hipStream_t st, int64_t q0,
                         int64_t q1) {
  const int64_t ns = q1 < 0 ? s->src->n : q1;  // queries: visit positions [q0, ns)
  const int64_t nt_pad = s->tgt->n_pad;
  if (ns <= q0 || s->tgt->n == 0) return hipSuccess;
  const Grid* tg = s->tgrid;
  int64_t slice = 0;
  if (icp_nn_uses_mfma(s)) {
    const int64_t tt = (int64_t)kTH * kMTile;
    if (tg->mf_npad % tt != 0) return hipErrorInvalidValue;  // pack16 pads to kMTilePad
    dim3 gm = nn_grid((ns - q0 + kMQueries - 1) / kMQueries, tg->mf_npad, tt, &slice);
    // Strided tiles decouple grid.y from slice boundaries: pick S in [S0, 2·S0] so that the
    // block count fills the resident block slots in whole rounds (the last partial round of
    // equal-length blocks idles the rest of the chip: 196 × 11 blocks on 512 slots = 4.2
    // rounds ran as 5).
    static const int64_t slots = [] {
      int dev = 0, per = 0;
      hipDeviceProp_t p;
      if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return (int64_t)0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, nn_mfma_kernel, kMBlock, 0) != hipSuccess)
        return (int64_t)0;
      return (int64_t)p.multiProcessorCount * (per > 0 ? per : 1);
    }();
    const int64_t bx = gm.x, ntiles = tg->mf_npad / tt;
    if (slots > 0 && ntiles > 1) {
      int64_t s0 = std::min<int64_t>(std::max<int64_t>((2048 + bx - 1) / bx, 1), ntiles);
      int64_t best = s0;
      double best_eff = 0.0;
      for (int64_t S = s0; S <= std::min<int64_t>(2 * s0, ntiles); ++S) {
        const int64_t blocks = bx * S, rounds = (blocks + slots - 1) / slots;
        const double eff = (double)blocks / (double)(rounds * slots);
        if (eff > best_eff + 1e-9) {
          best_eff = eff;
          best = S;
        }
      }
      gm.y = (unsigned)best;
    }
    const SeedArgs sa{s->corr, s->tgt->xyz32, s->tgt->n, self_seed ? 1 : 0};
    nn_mfma_kernel<<<gm, kMBlock, 0, st>>>(s->src->xyz32, ns, tg->mf16, tg->mf32, tg->mf_npad, off,
                                           s->state, s->keys, s->near2, sa, q0);
    return hipGetLastError();
  }
  if (q0 != 0 || ns != s->src->n) return hipErrorInvalidValue;  // the VALU form scans every source
  if (self_seed) {  // the fp32 VALU kernel reads its starting keys
    const hipError_t e = launch_icp_keyinit(s, off, st);
    if (e != hipSuccess) return e;
  }
  const dim3 grid = nn_grid((ns + kNNBlock * kNNQ - 1) / (kNNBlock * kNNQ), nt_pad, kNNLds, &slice);
  nn_kernel<<<grid, kNNBlock, 0, st>>>(s->src->xyz32, ns, s->tgt->xyz32, nt_pad, slice, off, s->state,
                                             s->keys, s->near2);
  return hipGetLastError();
}


__global__ __launch_bounds__(256) void pack_rec_kernel(const double* __restrict__ xyz,
                                                       const double* __restrict__ nrm, int64_t n,
                                                       double* __restrict__ rec) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double r[8];
  for (int k = 0; k < 3; ++k) {
    r[k] = xyz[3 * i + k];
    r[3 + k] = nrm != nullptr ? nrm[3 * i + k] : 0.0;
  }
  r[6] = r[7] = 0.0;
  for (int k = 0; k < 8; ++k) rec[8 * i + k] = r[k];
}

hipError_t ensure_target_rec(const m3d_cloud* c, hipStream_t st) {
  if (c->rec64 != nullptr || c->n == 0) return hipSuccess;
  double* rec = nullptr;
  hipError_t e = block_alloc(reinterpret_cast<void**>(&rec), sizeof(double) * 8 * c->n, st);
  if (e != hipSuccess) return e;
  pack_rec_kernel<<<(unsigned)((c->n + 255) / 256), 256, 0, st>>>(c->xyz64, c->nrm64, c->n, rec);
  e = hipGetLastError();  // asynchronous (stream order); m3d_icp_create synchronises once
  if (e != hipSuccess) {
    block_release(rec);
    return e;
  }
  c->rec64 = rec;
  return hipSuccess;
}

// The target grid's points in fp64, in the grid's cell order (w = index bits): resolve_wave then
// reads an ambiguous query's box candidates with their fp64 coordinates in one load instead of the
// fp32 point and then a gather of the fp64 one
__global__ __launch_bounds__(256) void pack_pts64_kernel(const float4* __restrict__ pts,
                                                         const double* __restrict__ xyz, int64_t n,
                                                         double4* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const int32_t j = __float_as_int(pts[k].w);
  out[k] = make_double4(xyz[3 * (int64_t)j], xyz[3 * (int64_t)j + 1], xyz[3 * (int64_t)j + 2],
                        __longlong_as_double((long long)j));
}

hipError_t build_grid_pts64(const m3d_cloud* c, Grid* g, hipStream_t st) {
  if (g->pts64 != nullptr || g->n_pts == 0 || M3D_WALK64 == 0) return hipSuccess;
  double4* p = nullptr;
  hipError_t e = block_alloc(reinterpret_cast<void**>(&p), sizeof(double4) * g->n_pts, st);
  if (e != hipSuccess) return e;
  pack_pts64_kernel<<<(unsigned)((g->n_pts + 255) / 256), 256, 0, st>>>(g->pts, c->xyz64, g->n_pts, p);
  e = hipGetLastError();  // asynchronous (stream order); m3d_icp_create synchronises once
  if (e != hipSuccess) {
    block_release(p);
    return e;
  }
  g->pts64 = p;
  g->dev.pts64 = p;
  return hipSuccess;
}

static TermsArgs terms_args(const m3d_icp* s, int64_t off, const int32_t* claim,
                            const int64_t* dmin, bool reset_keys) {
  TermsArgs a;
  a.pcd64 = s->pcd64;
  a.src32 = s->src->xyz32;
  a.ns = s->src->n;
  a.tgt64 = s->tgt->xyz64;
  a.nrm64 = s->tgt->nrm64;
  a.rec64 = s->tgt->rec64;
  a.nt_shard = s->tgt->n;
  a.off = off;
  a.keys = s->keys;
  a.near2 = s->near2;
  a.g = s->tgrid->dev;
  a.claim = claim;
  a.dmin = dmin;
  a.dprev = claim != nullptr ? s->dprev : nullptr;
  a.corr = s->corr;
  a.est = s->params.estimation;
  for (int k = 0; k < 3; ++k) a.c[k] = s->src->center[k];
  a.reset_keys = reset_keys ? s->keys : nullptr;
  return a;
}

hipError_t launch_icp_terms_mode(const m3d_icp* s, int64_t off, const int32_t* claim,
                                 const int64_t* dmin, hipStream_t st) {
  const int64_t ns = s->src->n;
  if (ns == 0) return hipMemsetAsync(s->partials, 0, sizeof(double) * kTermSlots, st);
  const TermsArgs ta = terms_args(s, off, claim, dmin, false);
  const unsigned nb = (unsigned)s->nblocks;
  if (ta.est == M3D_EST_POINT_TO_PLANE)
    terms_kernel<kTermsPtsDefault, M3D_EST_POINT_TO_PLANE><<<nb, kTermsBlock, 0, st>>>(ta, s->state, s->partials);
  else
    terms_kernel<kTermsPtsDefault, M3D_EST_POINT_TO_POINT><<<nb, kTermsBlock, 0, st>>>(ta, s->state, s->partials);
  return hipGetLastError();
}

hipError_t launch_icp_reduce(const m3d_icp* s, double* sums, hipStream_t st) {
  if (s->nblocks > 256)  // group g's first row is block g's: rows 0..31 exist
    reduce_groups_kernel<M3D_EST_POINT_TO_PLANE><<<kReduceGroups, kTermSlots, 0, st>>>(
        s->partials, s->nblocks, sums, s->state, SolveParams{}, 0);
  else
    reduce_kernel<<<1, kReduceGroups * kTermSlots, 0, st>>>(s->partials, s->nblocks, sums, s->state);
  return hipGetLastError();
}

static SolveParams solve_params(const m3d_icp* s);

// the single-device separate tail after the terms pass: reduce + solve (one launch past 256
// partials, reduce_groups_kernel's last block solving; two below)
hipError_t launch_icp_reduce_solve(const m3d_icp* s, hipStream_t st) {
  if (s->nblocks <= 256) {
    hipError_t e = launch_icp_reduce(s, s->sums, st);
    return e == hipSuccess ? launch_icp_solve(s, s->sums, st) : e;
  }
  if (s->params.estimation == M3D_EST_POINT_TO_PLANE)
    reduce_groups_kernel<M3D_EST_POINT_TO_PLANE><<<kReduceGroups, kTermSlots, 0, st>>>(
        s->partials, s->nblocks, s->sums, s->state, solve_params(s), 1);
  else
    reduce_groups_kernel<M3D_EST_POINT_TO_POINT><<<kReduceGroups, kTermSlots, 0, st>>>(
        s->partials, s->nblocks, s->sums, s->state, solve_params(s), 1);
  return hipGetLastError();
}

static SolveParams solve_params(const m3d_icp* s) {
  SolveParams sp;
  sp.rel_fit = s->params.relative_fitness;
  sp.rel_rmse = s->params.relative_rmse;
  sp.max_iter = s->params.max_iteration;
  sp.est = s->params.estimation;
  sp.ns = s->ns_total > 0 ? s->ns_total : s->src->n;
  for (int k = 0; k < 3; ++k) sp.c[k] = s->src->center[k];
  sp.f = frame_of(s);
  return sp;
}

// sharded tail: terms (shard offset off; claim/dmin: the target-shard exchange results, or null
// for a source shard) + reduce into sums, one launch
static void launch_terms_solve(const TermsArgs& ta, const m3d_icp* s, double* sums, int do_solve,
                               hipStream_t st) {
  const unsigned nb = (unsigned)s->nblocks;
  const SolveParams sp = solve_params(s);
  if (ta.est == M3D_EST_POINT_TO_PLANE)
    terms_solve_kernel<kTermsPtsDefault, M3D_EST_POINT_TO_PLANE><<<nb, kTermsBlock, 0, st>>>(ta, s->state, s->partials, s->nblocks,
                                                                             sums, sp, do_solve);
  else
    terms_solve_kernel<kTermsPtsDefault, M3D_EST_POINT_TO_POINT><<<nb, kTermsBlock, 0, st>>>(ta, s->state, s->partials, s->nblocks,
                                                                             sums, sp, do_solve);
}

hipError_t launch_icp_terms_reduce(const m3d_icp* s, int64_t off, const int32_t* claim,
                                   const int64_t* dmin, double* sums, bool reset_keys,
                                   hipStream_t st) {
  const int64_t ns = s->src->n;
  if (ns == 0) {
    hipError_t e = launch_icp_terms_mode(s, off, claim, dmin, st);
    return e == hipSuccess ? launch_icp_reduce(s, sums, st) : e;
  }
  launch_terms_solve(terms_args(s, off, claim, dmin, reset_keys), s, sums, 0, st);
  return hipGetLastError();
}

hipError_t launch_icp_solve(const m3d_icp* s, const double* sums, hipStream_t st) {
  if (s->params.estimation == M3D_EST_POINT_TO_PLANE)
    solve_kernel<M3D_EST_POINT_TO_PLANE><<<1, 64, 0, st>>>(sums, s->state, solve_params(s));
  else
    solve_kernel<M3D_EST_POINT_TO_POINT><<<1, 64, 0, st>>>(sums, s->state, solve_params(s));
  return hipGetLastError();
}

hipError_t launch_icp_terms_solve(const m3d_icp* s, bool reset_keys, hipStream_t st) {
  const int64_t ns = s->src->n;
  if (ns == 0) {  // no blocks to take tickets: the unfused tail handles the empty source
    hipError_t e = launch_icp_terms_mode(s, 0, nullptr, nullptr, st);
    if (e == hipSuccess) e = launch_icp_reduce(s, s->sums, st);
    return e == hipSuccess ? launch_icp_solve(s, s->sums, st) : e;
  }
  launch_terms_solve(terms_args(s, 0, nullptr, nullptr, reset_keys), s, s->sums, 1, st);
  return hipGetLastError();
}

hipError_t launch_nn_finalize(const m3d_icp* s, int32_t* idx, double* d2, hipStream_t st) {
  const int64_t ns = s->src->n;
  if (ns == 0) return hipSuccess;
  nn_finalize_kernel<<<(unsigned)((ns + 255) / 256), 256, 0, st>>>(
      s->pcd64, s->src->xyz32, ns, s->tgt->xyz64, s->tgt->n, s->tgrid->dev, s->state, s->keys,
      s->near2, s->src->slot, idx, d2);
  return hipGetLastError();
}

hipError_t launch_scatter_i32(const int32_t* v, const int32_t* slot, int64_t n, int32_t* dst,
                              hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (slot == nullptr) return hipMemcpyAsync(dst, v, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st);
  scatter_i32_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(v, slot, n, dst);
  return hipGetLastError();
}

hipError_t launch_corr_pairs(const int32_t* v, int64_t n, int32_t* cnt, int32_t* pairs, hipStream_t st) {
  if (n <= 0) return hipMemsetAsync(cnt, 0, sizeof(int32_t), st);
  const int64_t nb = (n + kPairChunk - 1) / kPairChunk;
  pair_count_kernel<<<(unsigned)nb, 256, 0, st>>>(v, n, cnt);
  pair_scan_kernel<<<1, 1024, 0, st>>>(cnt, nb);
  pair_place_kernel<<<(unsigned)nb, 256, 0, st>>>(v, n, cnt, pairs);
  return hipGetLastError();
}

hipError_t launch_shard_winner(const m3d_icp* s, int64_t off, int64_t* dkey, hipStream_t st,
                               int64_t q0, int64_t q1) {
  const int64_t ns = q1 < 0 ? s->src->n : q1;
  if (ns <= q0) return hipSuccess;
  shard_winner_kernel<<<(unsigned)((ns - q0 + 255) / 256), 256, 0, st>>>(
      s->pcd64, s->src->xyz32, ns, s->tgt->xyz64, s->tgt->n, off, s->tgrid->dev, s->state,
      s->keys, s->near2, s->lidx, s->ld64, dkey, q0);
  return hipGetLastError();
}

hipError_t launch_shard_claim(const m3d_icp* s, const int64_t* dmin, int32_t* claim, hipStream_t st) {
  const int64_t ns = s->src->n;
  if (ns == 0) return hipSuccess;
  shard_claim_kernel<<<(unsigned)((ns + 255) / 256), 256, 0, st>>>(ns, s->state, s->lidx, s->ld64,
                                                                   dmin, claim);
  return hipGetLastError();
}

hipError_t launch_keys_to_idx(const int64_t* keys, int64_t n, int32_t* idx, hipStream_t st) {
  if (n == 0) return hipSuccess;
  keys_to_idx_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(keys, n, idx);
  return hipGetLastError();
}

int64_t terms_blocks(int64_t ns) {
  const int64_t per = (int64_t)kTermsBlock * terms_pts();
  return ns > 0 ? (ns + per - 1) / per : 1;
}

}  // namespace m3d

#if M3D_TERMS_CLOCK
extern "C" int m3d_debug_terms_clock(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(m3d::g_terms_clock), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif
#if M3D_TAIL_CLOCK
extern "C" int m3d_debug_tail_clock(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(m3d::g_tail_clock), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif
