// feat.hip — feature-space correspondences and feature-matching RANSAC on gfx950
// (SURVEY.md §8 a5 FPFH half, a6; §8(f) rank 3).
//
// Reference: src/matcher/ransac.py:41-58 (global_registration → Open3D
// RegistrationRANSACBasedOnFeatureMatching) and :85 (correspondences_from_features), restated in
// oracle/prep_oracle.py (parity against Open3D itself unpinned).
//
//   feature_nn_kernel   exact fp64 33-D 1-NN, d² = Σ_j (a_j − b_j)² in dimension order (the
//                       oracle's order).  Queries in VGPRs (one per lane), reference features
//                       staged through LDS tiles and read by broadcast; the reference range is
//                       sliced over grid.y and the slices merged by a second kernel in slice
//                       order (lexicographic (d², index) → deterministic, lowest index on ties).
//   mutual_kernel       corres_ij[i] kept iff corres_ji[corres_ij[i]] == i (order preserved by
//                       hipcub DeviceSelect::Flagged).
//   feat_hyp_kernel     per hypothesis: ransac_n = 3 rows drawn WITH replacement from the counter
//                       sampler, Umeyama/Kabsch (linalg.h kabsch3), EdgeLength + Distance checkers.
//   validation          the ICP evaluation pieces (grid NN + terms + reduce, icp.hip/grid.hip)
//                       per surviving hypothesis; the sequential best / early-exit selection of
//                       RegistrationRANSACBasedOnCorrespondence runs on the host over ≤ max_iter
//                       (count, Σd²) pairs.
#include <float.h>

#include <algorithm>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "linalg.h"
#include "m3d_internal.h"
#include "nnkey.h"

namespace m3d {

constexpr int kFeatDim = 33;
constexpr int kFnnBlock = 128;  // queries per block (one per lane)
constexpr int kFnnTile = 64;    // reference features per LDS tile (64 × 33 × 8 B = 16.9 KB)

__global__ __launch_bounds__(kFnnBlock) void feature_nn_kernel(const double* __restrict__ fq, int64_t nq,
                                                               const double* __restrict__ fr, int64_t nr,
                                                               int64_t slice_len,
                                                               double* __restrict__ best_d,
                                                               int32_t* __restrict__ best_i) {
  __shared__ double tile[kFnnTile][kFeatDim];
  const int64_t i = (int64_t)blockIdx.x * kFnnBlock + threadIdx.x;
  double a[kFeatDim];
#pragma unroll
  for (int j = 0; j < kFeatDim; ++j) a[j] = i < nq ? fq[i * kFeatDim + j] : 0.0;
  double bd = DBL_MAX;
  int32_t bi = -1;
  const int64_t rb = (int64_t)blockIdx.y * slice_len;
  const int64_t re = min(nr, rb + slice_len);
  for (int64_t t0 = rb; t0 < re; t0 += kFnnTile) {
    const int tn = (int)min((int64_t)kFnnTile, re - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < tn * kFeatDim; e += kFnnBlock)
      tile[e / kFeatDim][e % kFeatDim] = fr[t0 * kFeatDim + e];
    __syncthreads();
    // four references per step: four independent dimension-order chains (each d² still sums
    // its 33 terms in the oracle's order) instead of one 33-long dependent fp64 chain
    int r = 0;
    for (; r + 4 <= tn; r += 4) {
      double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
#pragma unroll
      for (int j = 0; j < kFeatDim; ++j) {
        const double t0 = a[j] - tile[r][j], t1 = a[j] - tile[r + 1][j];
        const double t2 = a[j] - tile[r + 2][j], t3 = a[j] - tile[r + 3][j];
        d0 += t0 * t0;
        d1 += t1 * t1;
        d2 += t2 * t2;
        d3 += t3 * t3;
      }
      // references in increasing index: strict < keeps the lowest
      if (d0 < bd) { bd = d0; bi = (int32_t)(t0 + r); }
      if (d1 < bd) { bd = d1; bi = (int32_t)(t0 + r + 1); }
      if (d2 < bd) { bd = d2; bi = (int32_t)(t0 + r + 2); }
      if (d3 < bd) { bd = d3; bi = (int32_t)(t0 + r + 3); }
    }
    for (; r < tn; ++r) {
      double d = 0.0;
#pragma unroll
      for (int j = 0; j < kFeatDim; ++j) {
        const double t = a[j] - tile[r][j];
        d += t * t;
      }
      if (d < bd) {
        bd = d;
        bi = (int32_t)(t0 + r);
      }
    }
  }
  if (i < nq) {
    best_d[(int64_t)blockIdx.y * nq + i] = bd;
    best_i[(int64_t)blockIdx.y * nq + i] = bi;
  }
}

__global__ __launch_bounds__(256) void feature_nn_merge_kernel(const double* __restrict__ best_d,
                                                               const int32_t* __restrict__ best_i,
                                                               int64_t nq, int slices,
                                                               int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nq) return;
  double bd = DBL_MAX;
  int32_t bi = -1;
  for (int s = 0; s < slices; ++s) {  // slice order = index order: strict < keeps the lowest
    const double d = best_d[(int64_t)s * nq + i];
    const int32_t k = best_i[(int64_t)s * nq + i];
    if (k >= 0 && (bi < 0 || d < bd)) {
      bd = d;
      bi = k;
    }
  }
  out[i] = bi;
}

hipError_t feature_nn(const double* fq, int64_t nq, const double* fr, int64_t nr, int32_t* out,
                      hipStream_t st) {
  if (nq == 0) return hipSuccess;
  const int64_t bx = (nq + kFnnBlock - 1) / kFnnBlock;
  // ≥ ~2048 blocks (≥ 4 waves per SIMD: each lane's chains are latency-bound): slice the
  // references, slices of ≥ 1 tile
  int64_t S = std::max<int64_t>(1, std::min<int64_t>((2048 + bx - 1) / bx, (nr + kFnnTile - 1) / kFnnTile));
  S = std::min<int64_t>(S, 65535);
  int64_t slice = (nr + S - 1) / S;
  slice = (slice + kFnnTile - 1) / kFnnTile * kFnnTile;
  S = std::max<int64_t>(1, (nr + slice - 1) / slice);
  double* bd = nullptr;
  int32_t* bi = nullptr;
  hipError_t e = dev_malloc(&bd, sizeof(double) * S * nq);
  if (e == hipSuccess) e = dev_malloc(&bi, sizeof(int32_t) * S * nq);
  if (e == hipSuccess) {
    feature_nn_kernel<<<dim3((unsigned)bx, (unsigned)S), kFnnBlock, 0, st>>>(fq, nq, fr, nr, slice, bd, bi);
    feature_nn_merge_kernel<<<(unsigned)((nq + 255) / 256), 256, 0, st>>>(bd, bi, nq, (int)S, out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);  // scratch freed below
  hipFree(bd);
  hipFree(bi);
  return e;
}

__global__ __launch_bounds__(256) void mutual_kernel(const int32_t* __restrict__ ij,
                                                     const int32_t* __restrict__ ji, int64_t ns,
                                                     int32_t* __restrict__ pairs,
                                                     uint8_t* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ns) return;
  const int32_t j = ij[i];
  pairs[2 * i] = (int32_t)i;
  pairs[2 * i + 1] = j;
  if (keep != nullptr) keep[i] = (j >= 0 && ji[j] == (int32_t)i) ? 1 : 0;
}

// corr_out [device] ns×2; returns the pair count in *n_out (synchronous)
hipError_t feature_correspondences(const double* fs, int64_t ns, const double* ft, int64_t nt,
                                   int mutual, double ratio, int32_t* corr_out, int64_t* n_out,
                                   hipStream_t st) {
  *n_out = 0;
  if (ns == 0 || nt == 0) return hipSuccess;
  int32_t *ij = nullptr, *ji = nullptr, *pairs = nullptr, *nsel = nullptr;
  uint8_t* keep = nullptr;
  void* tmp = nullptr;
  auto cleanup = [&]() {
    hipFree(ij);
    hipFree(ji);
    hipFree(pairs);
    hipFree(nsel);
    hipFree(keep);
    hipFree(tmp);
  };
  hipError_t e = dev_malloc(&ij, 4 * ns);
  if (e == hipSuccess) e = feature_nn(fs, ns, ft, nt, ij, st);
  if (e == hipSuccess && !mutual) {  // corres_ij only: (i, nn(i)) for every source feature
    mutual_kernel<<<(unsigned)((ns + 255) / 256), 256, 0, st>>>(ij, nullptr, ns, corr_out, nullptr);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    cleanup();
    *n_out = ns;
    return e;
  }
  if (e == hipSuccess) e = dev_malloc(&ji, 4 * nt);
  if (e == hipSuccess) e = feature_nn(ft, nt, fs, ns, ji, st);
  if (e == hipSuccess) e = dev_malloc(&pairs, 8 * ns);
  if (e == hipSuccess) e = dev_malloc(&keep, ns);
  if (e == hipSuccess) e = dev_malloc(&nsel, 4);
  if (e == hipSuccess) {
    mutual_kernel<<<(unsigned)((ns + 255) / 256), 256, 0, st>>>(ij, ji, ns, pairs, keep);
    e = hipGetLastError();
  }
  size_t tb = 0;
  if (e == hipSuccess)
    e = hipcub::DeviceSelect::Flagged(nullptr, tb, (const int2*)pairs, keep, (int2*)corr_out, nsel, (int)ns, st);
  if (e == hipSuccess) e = dev_malloc(&tmp, std::max<size_t>(tb, 1));
  if (e == hipSuccess)
    e = hipcub::DeviceSelect::Flagged(tmp, tb, (const int2*)pairs, keep, (int2*)corr_out, nsel, (int)ns, st);
  int32_t h = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&h, nsel, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess && (int64_t)h < (int64_t)(ratio * (double)ns)) {
    // too few mutual pairs: Open3D falls back to the one-directional set
    e = hipMemcpyAsync(corr_out, pairs, 8 * ns, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    h = (int32_t)ns;
  }
  cleanup();
  *n_out = h;
  return e;
}

// ------------------------------------------------------------------------------- a6 hypotheses
__device__ __forceinline__ uint64_t fsplitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void feat_hyp_kernel(const double* __restrict__ src, const double* __restrict__ tgt,
                                const int32_t* __restrict__ corr, int64_t nc, uint64_t seed,
                                int64_t H, double edge, double dist, double* __restrict__ T_out,
                                int32_t* __restrict__ pass) {
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  const uint64_t base = fsplitmix64(seed ^ ((uint64_t)h * 0x9E3779B97F4A7C15ull));
  double ps[3][3], qs[3][3];
  for (int k = 0; k < 3; ++k) {  // WITH replacement, like Open3D's rand_gen() per row
    const uint64_t v = fsplitmix64(base + (uint64_t)k);
    const int64_t r = (int64_t)(((v >> 32) * (uint64_t)nc) >> 32);
    const int64_t a = corr[2 * r], b = corr[2 * r + 1];
    for (int c = 0; c < 3; ++c) {
      ps[k][c] = src[3 * a + c];
      qs[k][c] = tgt[3 * b + c];
    }
  }
  double* T = T_out + 16 * h;
  kabsch3(ps, qs, T);
  bool ok = true;
  if (edge > 0.0) {  // CorrespondenceCheckerBasedOnEdgeLength
    for (int i = 0; i < 3 && ok; ++i)
      for (int j = i + 1; j < 3 && ok; ++j) {
        double ds = 0.0, dt = 0.0;
        {
          const double x = ps[i][0] - ps[j][0], y = ps[i][1] - ps[j][1], z = ps[i][2] - ps[j][2];
          ds = sqrt((x * x + y * y) + z * z);
        }
        {
          const double x = qs[i][0] - qs[j][0], y = qs[i][1] - qs[j][1], z = qs[i][2] - qs[j][2];
          dt = sqrt((x * x + y * y) + z * z);
        }
        if (ds < dt * edge || dt < ds * edge) ok = false;
      }
  }
  if (dist > 0.0) {  // CorrespondenceCheckerBasedOnDistance
    for (int k = 0; k < 3 && ok; ++k) {
      double d[3];
      for (int r = 0; r < 3; ++r)
        d[r] = qs[k][r] - (((T[4 * r] * ps[k][0] + T[4 * r + 1] * ps[k][1]) + T[4 * r + 2] * ps[k][2]) + T[4 * r + 3]);
      if (sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]) > dist) ok = false;
    }
  }
  pass[h] = ok ? 1 : 0;
}

// Open3D 0.19 EvaluateInlierCorrespondenceRatio (Registration.cpp): for hypothesis k of a
// validation batch (T = T_all + 16·list[k]) the number of INPUT correspondences c with
// |T·p_c − q_c|² < r2 — the source transformed as PointCloud::Transform does and squaredNorm in
// Eigen's order (nnkey.h q64_of / d2_64, fp64, no contraction), strict <.  Integer counts summed
// with atomics: exact and order-free.  grid.y = hypothesis of the batch, grid.x strides over nc.
__global__ __launch_bounds__(256) void corres_inlier_kernel(
    const double* __restrict__ src, const double* __restrict__ tgt, const int32_t* __restrict__ corr,
    int64_t nc, const double* __restrict__ T_all, const int32_t* __restrict__ list, double r2,
    int32_t* __restrict__ count) {
  const int h = blockIdx.y;
  double T[12];
  const double* Tg = T_all + 16 * (int64_t)list[h];
#pragma unroll
  for (int k = 0; k < 12; ++k) T[k] = Tg[k];
  int n = 0;
  for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < nc; c += (int64_t)gridDim.x * 256) {
    const int64_t a = corr[2 * c], b = corr[2 * c + 1];
    double Q[3];
    q64_of(T, src + 3 * a, Q);
    n += d2_64(Q, tgt + 3 * b) < r2 ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0 && n != 0) atomicAdd(count + h, n);
}

hipError_t launch_corres_inlier(const double* src, const double* tgt, const int32_t* corr, int64_t nc,
                                const double* T_all, const int32_t* list, int64_t n, double max_corr,
                                int32_t* count, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(count, 0, sizeof(int32_t) * (size_t)n, st);
  if (e != hipSuccess || nc <= 0) return e;
  const unsigned bx = (unsigned)std::min<int64_t>((nc + 255) / 256, 64);
  corres_inlier_kernel<<<dim3(bx, (unsigned)n), 256, 0, st>>>(src, tgt, corr, nc, T_all, list,
                                                              max_corr * max_corr, count);
  return hipGetLastError();
}

hipError_t launch_feat_hyp(const double* src, const double* tgt, const int32_t* corr, int64_t nc,
                           uint64_t seed, int64_t H, double edge, double dist, double* T_out,
                           int32_t* pass, hipStream_t st) {
  if (H == 0) return hipSuccess;
  feat_hyp_kernel<<<(unsigned)((H + 63) / 64), 64, 0, st>>>(src, tgt, corr, nc, seed, H, edge, dist,
                                                            T_out, pass);
  return hipGetLastError();
}

}  // namespace m3d
