// prep.hip — point-cloud preprocessing on gfx950 (a5 FPFH half).
//
// Reference: src/ply/ply.py:106-135 → Open3D 0.19 VoxelDownSample, EstimateNormals
// (KDTreeSearchParamHybrid(2v, 30)), ComputeFPFHFeature (KDTreeSearchParamHybrid(5v, 100)).
// Restated in oracle/prep_oracle.py (parity against Open3D itself unpinned).
//
// All arithmetic is fp64 in the oracle's operation order (-ffp-contract=off):
//   voxel   keys floor((p − vmin)/v) → stable radix sort (key, index) → run-length encode →
//           one thread per voxel sums its points in input order, divides by the count.
//   search  hybrid radius/k search on the cloud's uniform grid (grid.hip layout, cell = r):
//           one lane per query keeps its k best (d², index) in a sorted LDS list (insertion;
//           d² exact fp64 (dx²+dy²)+dz², strict d² < r², ties by index).  The fp32 grid box is
//           widened by the fp32 centring error so every exact candidate is visited.
//   normals cumulants in neighbour order → covariance → FastEigen3x3 (Eberly) → orientation.
//   FPFH    SPFH pair features (fp64 acos/atan2) into 3×11 bins, then the 1/d²-weighted
//           neighbour sum, per-group normalisation to 100, + own SPFH.
// These kernels are O(N·k) and run once per cloud: latency/HBM-bound, not a roofline concern
// next to the per-iteration loops; they are timed in bench.py's preprocessing line.
#include <float.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "m3d_internal.h"
#include "ddmath.h"

namespace m3d {

constexpr int kPrepBlock = 256;

// ------------------------------------------------------------------------------- voxel
__global__ __launch_bounds__(kPrepBlock) void minmax3d_kernel(const double* __restrict__ p, int64_t n,
                                                              double* __restrict__ part) {
  __shared__ double s[6][kPrepBlock];
  double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (int64_t i = (int64_t)blockIdx.x * kPrepBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kPrepBlock)
    for (int k = 0; k < 3; ++k) {
      lo[k] = fmin(lo[k], p[3 * i + k]);
      hi[k] = fmax(hi[k], p[3 * i + k]);
    }
  for (int k = 0; k < 3; ++k) {
    s[k][threadIdx.x] = lo[k];
    s[3 + k][threadIdx.x] = hi[k];
  }
  __syncthreads();
  for (int w = kPrepBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < 3; ++k) {
        s[k][threadIdx.x] = fmin(s[k][threadIdx.x], s[k][threadIdx.x + w]);
        s[3 + k][threadIdx.x] = fmax(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + w]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 6) part[6 * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

__global__ __launch_bounds__(kPrepBlock) void voxel_key_kernel(const double* __restrict__ p, int64_t n,
                                                               double v0, double v1, double v2,
                                                               double voxel,
                                                               uint64_t* __restrict__ key,
                                                               int32_t* __restrict__ val) {
  const int64_t i = (int64_t)blockIdx.x * kPrepBlock + threadIdx.x;
  if (i >= n) return;
  const uint64_t ix = (uint64_t)(int64_t)floor((p[3 * i] - v0) / voxel);
  const uint64_t iy = (uint64_t)(int64_t)floor((p[3 * i + 1] - v1) / voxel);
  const uint64_t iz = (uint64_t)(int64_t)floor((p[3 * i + 2] - v2) / voxel);
  key[i] = (ix << 42) | (iy << 21) | iz;
  val[i] = (int32_t)i;
}

__global__ __launch_bounds__(kPrepBlock) void voxel_mean_kernel(
    const double* __restrict__ p, const double* __restrict__ nrm, const int32_t* __restrict__ order,
    const int32_t* __restrict__ counts, const int32_t* __restrict__ offsets,
    const int32_t* __restrict__ nvox, double* __restrict__ out_p, double* __restrict__ out_n) {
  const int64_t v = (int64_t)blockIdx.x * kPrepBlock + threadIdx.x;
  if (v >= *nvox) return;
  const int32_t b = offsets[v], c = counts[v];
  double sp[3] = {0.0, 0.0, 0.0}, sn[3] = {0.0, 0.0, 0.0};
  for (int32_t k = 0; k < c; ++k) {
    const int64_t i = order[b + k];
    for (int a = 0; a < 3; ++a) sp[a] += p[3 * i + a];
    if (nrm != nullptr) {
      // AccumulatedPoint::AddPoint: a normal with a NaN component is skipped (still counted)
      const double n0 = nrm[3 * i], n1 = nrm[3 * i + 1], n2 = nrm[3 * i + 2];
      if (!(isnan(n0) || isnan(n1) || isnan(n2))) {
        sn[0] += n0;
        sn[1] += n1;
        sn[2] += n2;
      }
    }
  }
  for (int a = 0; a < 3; ++a) out_p[3 * v + a] = sp[a] / (double)c;
  if (nrm != nullptr && out_n != nullptr)
    for (int a = 0; a < 3; ++a) out_n[3 * v + a] = sn[a] / (double)c;
}

// ------------------------------------------------------------------------------- hybrid search
__device__ __forceinline__ int prep_coord(float x, float o, float inv_h, int n) {
  float f = (x - o) * inv_h;  // == grid.hip grid_coord
  f = fminf(fmaxf(f, 0.0f), (float)(n - 1));
  return (int)f;
}

__device__ __forceinline__ double d2_exact(const double* a, const double* b) {
  const double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
  return (dx * dx + dy * dy) + dz * dz;
}

// fp32 prefilter of a candidate against an exact fp64 threshold thr (inclusive): with e the
// bound on |fp32 distance − fp64 distance| of two centred points (both coordinate roundings,
// √3·2·u·rmax), any point whose fp64 d² ≤ thr has a directly computed fp32 d² (three roundings
// of relative u each, covered by the 4e-6 factors) ≤ this bound — so a candidate above it can be
// skipped without its fp64 gather.
__device__ __forceinline__ float prefilter_bound(double thr, double e) {
  const double b = (sqrt(thr) + e) * (1.0 + 4e-6);
  const float f = __double2float_ru(b * b * (1.0 + 4e-6));
  return isfinite(f) ? f : FLT_MAX;
}

// Block = L lanes (one query each); dynamic LDS: d²[k][L] doubles then idx[k][L] ints.
// Candidates are screened in fp32 from the grid's own sorted points first (prefilter_bound of
// r² and, once k are held, of the k-th d²): most of a box lies outside the sphere, and past the
// first k most candidates cannot enter the list, so the exact path (fp64 gather + insertion)
// runs for few.  The list is exactly the one without the screen.
__global__ void hybrid_search_kernel(const double* __restrict__ xyz64, const float4* __restrict__ xyz32,
                                     int64_t n, GridDev g, float Rf, double r2, double eabs, int k,
                                     int32_t* __restrict__ out_idx, double* __restrict__ out_d2,
                                     int32_t* __restrict__ out_cnt) {
  extern __shared__ double lds[];
  const int L = blockDim.x, lane = threadIdx.x;
  double* ld = lds;                          // [k][L]
  int32_t* li = (int32_t*)(lds + (size_t)k * L);  // [k][L]
  const int64_t i = (int64_t)blockIdx.x * L + lane;
  if (i >= n) return;
  const double q[3] = {xyz64[3 * i], xyz64[3 * i + 1], xyz64[3 * i + 2]};
  const float4 qf = xyz32[i];
  int cnt = 0;
  float bf = prefilter_bound(r2, eabs);
  if (g.ncells > 0) {
    const int x0 = prep_coord(qf.x - Rf, g.o[0], g.inv_h, g.n[0]);
    const int x1 = prep_coord(qf.x + Rf, g.o[0], g.inv_h, g.n[0]);
    const int y0 = prep_coord(qf.y - Rf, g.o[1], g.inv_h, g.n[1]);
    const int y1 = prep_coord(qf.y + Rf, g.o[1], g.inv_h, g.n[1]);
    const int z0 = prep_coord(qf.z - Rf, g.o[2], g.inv_h, g.n[2]);
    const int z1 = prep_coord(qf.z + Rf, g.o[2], g.inv_h, g.n[2]);
    for (int cz = z0; cz <= z1; ++cz)
      for (int cy = y0; cy <= y1; ++cy) {
        const int64_t row = ((int64_t)cz * g.n[1] + cy) * g.n[0];
        const int32_t j0 = g.start[row + x0], j1 = g.start[row + x1 + 1];
        for (int32_t j = j0; j < j1; ++j) {
          const float4 tp = g.pts[j];
          const float fx = qf.x - tp.x, fy = qf.y - tp.y, fz = qf.z - tp.z;
          if ((fx * fx + fy * fy) + fz * fz > bf) continue;
          const int32_t t = __float_as_int(tp.w);
          const double d2 = d2_exact(xyz64 + 3 * (int64_t)t, q);
          if (!(d2 < r2)) continue;
          int pos;
          if (cnt < k) {
            pos = cnt++;
          } else {
            const double dl = ld[(k - 1) * L + lane];
            const int32_t il = li[(k - 1) * L + lane];
            if (d2 > dl || (d2 == dl && t > il)) continue;
            pos = k - 1;
          }
          while (pos > 0) {
            const double dp = ld[(pos - 1) * L + lane];
            const int32_t ip = li[(pos - 1) * L + lane];
            if (dp < d2 || (dp == d2 && ip < t)) break;
            ld[pos * L + lane] = dp;
            li[pos * L + lane] = ip;
            --pos;
          }
          ld[pos * L + lane] = d2;
          li[pos * L + lane] = t;
          if (cnt == k) bf = prefilter_bound(ld[(k - 1) * L + lane], eabs);
        }
      }
  }
  for (int s = 0; s < k; ++s) {
    out_idx[i * k + s] = s < cnt ? li[s * L + lane] : -1;
    out_d2[i * k + s] = s < cnt ? ld[s * L + lane] : 0.0;
  }
  out_cnt[i] = cnt;
}

// The same search with ONE WAVE per query (k ≤ 64·kS): the wave reads the box's cell rows 64
// points at a time (coalesced: the rows are contiguous in the sorted grid), screens them in fp32
// against prefilter_bound of the current threshold, evaluates the survivors' exact fp64 d², and
// inserts the qualifying ones into a sorted list held across the lanes (entry e in lane e % 64,
// slot e / 64): position = number of held entries below the candidate (a ballot), entries at
// and above it move up one place (a lane shift), the k-th entry sets the next threshold.  The
// list order is the total order (d², index), so it is the per-lane kernel's list exactly, with
// every candidate read once per wave instead of once per lane and no divergent insertion chains.
__device__ __forceinline__ bool key_less(double d, int32_t t, double D, int32_t T) {
  return d < D || (d == D && t < T);
}

// lane l ← lane l − 1 across the whole wave (gfx9 DPP wave_shr:1; lane 0 keeps `old`): a VALU
// move, no LDS round trip like ds_bpermute
__device__ __forceinline__ int32_t wave_shr1(int32_t old, int32_t v) {
  return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ double wave_shr1(double old, double v) {
  const uint64_t o = (uint64_t)__double_as_longlong(old), x = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)wave_shr1((int32_t)(uint32_t)o, (int32_t)(uint32_t)x);
  const uint32_t hi = (uint32_t)wave_shr1((int32_t)(uint32_t)(o >> 32), (int32_t)(uint32_t)(x >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const uint64_t x = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)(x >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Two-stage form (gf.ncells > 0): the wave first searches the box of radius h on a finer grid
// gf (hybrid_search picks h so that ~2.5k points are expected within it).  The box holds every
// point within h of the query (the same covering argument as for r), so if k entries are then
// held and the k-th d² is below h²(1 − 1e-12), every unscanned point — exact distance > h, its
// fp64 d² at least h²(1 − 4u) — is beyond the k-th entry: the list is final.  Otherwise the list
// is discarded and the radius-r box is searched as before.  Either way the list is the same.
template <int kS>
__global__ __launch_bounds__(256) void hybrid_search_wave_kernel(
    const double* __restrict__ xyz64, const float4* __restrict__ xyz32, int64_t n, GridDev g,
    float Rf, double r2, double eabs, int k, GridDev gf, float Hf, double h2safe,
    int32_t* __restrict__ out_idx, double* __restrict__ out_d2, int32_t* __restrict__ out_cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;  // wave-uniform
  const double q[3] = {xyz64[3 * i], xyz64[3 * i + 1], xyz64[3 * i + 2]};
  const float4 qf = xyz32[i];
  double D[kS];
  int32_t T[kS];
#pragma unroll
  for (int u = 0; u < kS; ++u) {
    D[u] = 0.0;
    T[u] = -1;
  }
  int cnt = 0;             // entries held (wave-uniform)
  double thr = r2;         // exact threshold: r² until k are held, then the k-th entry (inclusive)
  int32_t thr_t = INT32_MAX;
  float bf = prefilter_bound(r2, eabs);
  auto scan = [&](const GridDev& g, float Rf) {
    if (g.ncells <= 0) return;
    const int x0 = prep_coord(qf.x - Rf, g.o[0], g.inv_h, g.n[0]);
    const int x1 = prep_coord(qf.x + Rf, g.o[0], g.inv_h, g.n[0]);
    const int y0 = prep_coord(qf.y - Rf, g.o[1], g.inv_h, g.n[1]);
    const int y1 = prep_coord(qf.y + Rf, g.o[1], g.inv_h, g.n[1]);
    const int z0 = prep_coord(qf.z - Rf, g.o[2], g.inv_h, g.n[2]);
    const int z1 = prep_coord(qf.z + Rf, g.o[2], g.inv_h, g.n[2]);
    for (int cz = z0; cz <= z1; ++cz)
      for (int cy = y0; cy <= y1; ++cy) {
        const int64_t row = ((int64_t)cz * g.n[1] + cy) * g.n[0];
        const int32_t j0 = g.start[row + x0], j1 = g.start[row + x1 + 1];
        for (int32_t jb = j0; jb < j1; jb += 64) {
          const int32_t j = jb + lane;
          bool cand = false;
          double d = 0.0;
          int32_t t = -1;
          if (j < j1) {
            const float4 tp = g.pts[j];
            const float fx = qf.x - tp.x, fy = qf.y - tp.y, fz = qf.z - tp.z;
            if ((fx * fx + fy * fy) + fz * fz <= bf) {
              t = __float_as_int(tp.w);
              d = d2_exact(xyz64 + 3 * (int64_t)t, q);
              cand = d < r2 && (cnt < k ? true : key_less(d, t, thr, thr_t));
            }
          }
          uint64_t m = __ballot(cand);
          if constexpr (kS == 1) {
            // Many candidates at once (the list is filling): merge them in one step instead of
            // one insertion each.  Every element's place in the union of the held list and the
            // chunk's candidates is its rank (the keys (d², index) are distinct): a list entry
            // is preceded by its own index and the candidates below it, a candidate by the list
            // entries below it (binary search over the sorted list) and the candidates below
            // it.  Elements ranked below k are written to LDS at their rank and read back.
            const int c = __popcll(m);
            if (c >= 3) {
              __shared__ double s_d[4][64];
              __shared__ int32_t s_t[4][64];
              const int w = threadIdx.x >> 6;
              int rl = lane, rc = 0;
              for (uint64_t mm = m; mm != 0; mm &= mm - 1) {
                const int s = __builtin_ctzll(mm);
                const double x = readlane_f64(d, s);
                const int32_t xt = __builtin_amdgcn_readlane(t, s);
                rl += key_less(x, xt, D[0], T[0]) ? 1 : 0;
                rc += key_less(x, xt, d, t) ? 1 : 0;
              }
              int lo = 0, hi = cnt;  // list entries below this lane's candidate: the first
              for (int it = 0; it < 7; ++it) {  // index whose key is not below it
                const int mid = (lo + hi) >> 1;
                const int src = mid < 64 ? mid : 63;
                const double dm = __shfl(D[0], src);
                const int32_t tm = __shfl(T[0], src);
                if (lo < hi) {
                  if (key_less(dm, tm, d, t))
                    lo = mid + 1;
                  else
                    hi = mid;
                }
              }
              rc += lo;
              const int ncnt = cnt + c < k ? cnt + c : k;
              if (lane < cnt && rl < k) {
                s_d[w][rl] = D[0];
                s_t[w][rl] = T[0];
              }
              if (cand && rc < k) {
                s_d[w][rc] = d;
                s_t[w][rc] = t;
              }
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              if (lane < ncnt) {
                D[0] = s_d[w][lane];
                T[0] = s_t[w][lane];
              }
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              cnt = ncnt;
              if (cnt == k) {
                thr = readlane_f64(D[0], k - 1);
                thr_t = __builtin_amdgcn_readlane(T[0], k - 1);
              }
              m = 0;
            }
          }
          while (m != 0) {
            const int src = __builtin_ctzll(m);
            m &= m - 1;
            const double x = readlane_f64(d, src);
            const int32_t xt = __builtin_amdgcn_readlane(t, src);
            if (cnt == k && !key_less(x, xt, thr, thr_t)) continue;  // the threshold moved
            int pos = 0;
#pragma unroll
            for (int u = 0; u < kS; ++u) {
              const int e = u * 64 + lane;
              pos += __popcll(__ballot(e < cnt && key_less(D[u], T[u], x, xt)));
            }
            // move entries pos .. up by one place (slot u takes lane 63 of slot u − 1)
#pragma unroll
            for (int u = kS - 1; u >= 0; --u) {
              // lane 0 of slot u takes lane 63 of slot u − 1 (a uniform read), the others
              // their left neighbour
              const double d63 = u > 0 ? readlane_f64(D[u > 0 ? u - 1 : 0], 63) : 0.0;
              const int32_t t63 = u > 0 ? __builtin_amdgcn_readlane(T[u > 0 ? u - 1 : 0], 63) : -1;
              const double dc = wave_shr1(d63, D[u]);
              const int32_t tc = wave_shr1(t63, T[u]);
              const int e = u * 64 + lane;
              if (e > pos) {
                D[u] = dc;
                T[u] = tc;
              } else if (e == pos) {
                D[u] = x;
                T[u] = xt;
              }
            }
            cnt = cnt < k ? cnt + 1 : k;
            if (cnt == k) {
              const int u = (k - 1) / 64, l = (k - 1) % 64;
              double dk = D[0];
              int32_t tk = T[0];
#pragma unroll
              for (int v = 0; v < kS; ++v)
                if (v == u) {
                  dk = D[v];
                  tk = T[v];
                }
              thr = readlane_f64(dk, l);
              thr_t = __builtin_amdgcn_readlane(tk, l);
            }
          }
          // the fp32 screen bound follows the k-th entry once per chunk (the entries above were
          // tested against the exact thr; bf only screens the next chunk)
          if (cnt == k) bf = prefilter_bound(thr, eabs);
        }
      }
  };
  bool done = false;
  if (gf.ncells > 0) {
    scan(gf, Hf);
    done = cnt == k && thr < h2safe;  // wave-uniform
    if (!done) {
#pragma unroll
      for (int u = 0; u < kS; ++u) {
        D[u] = 0.0;
        T[u] = -1;
      }
      cnt = 0;
      thr = r2;
      thr_t = INT32_MAX;
      bf = prefilter_bound(r2, eabs);
    }
  }
  if (!done) scan(g, Rf);
#pragma unroll
  for (int u = 0; u < kS; ++u) {
    const int e = u * 64 + lane;
    if (e < k) {
      out_idx[i * k + e] = e < cnt ? T[u] : -1;
      out_d2[i * k + e] = e < cnt ? D[u] : 0.0;
    }
  }
  if (lane == 0) out_cnt[i] = cnt;
}

// ------------------------------------------------------------------------------- normals
__device__ __forceinline__ void pcross(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ __forceinline__ double pdot(const double a[3], const double b[3]) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}

__device__ void eigvec0(const double A[3][3], double e, double out[3]) {
  const double r0[3] = {A[0][0] - e, A[0][1], A[0][2]};
  const double r1[3] = {A[0][1], A[1][1] - e, A[1][2]};
  const double r2[3] = {A[0][2], A[1][2], A[2][2] - e};
  double a[3], b[3], c[3];
  pcross(r0, r1, a);
  pcross(r0, r2, b);
  pcross(r1, r2, c);
  const double d0 = pdot(a, a), d1 = pdot(b, b), d2 = pdot(c, c);
  double dmax = d0;
  int imax = 0;
  if (d1 > dmax) {
    dmax = d1;
    imax = 1;
  }
  if (d2 > dmax) imax = 2;
  const double* v = imax == 0 ? a : (imax == 1 ? b : c);
  const double s = sqrt(imax == 0 ? d0 : (imax == 1 ? d1 : d2));
  for (int k = 0; k < 3; ++k) out[k] = v[k] / s;
}

__device__ void eigvec1(const double A[3][3], const double ev0[3], double e1, double out[3]) {
  double U[3], V[3];
  if (fabs(ev0[0]) > fabs(ev0[1])) {
    const double inv = 1.0 / sqrt(ev0[0] * ev0[0] + ev0[2] * ev0[2]);
    U[0] = -ev0[2] * inv;
    U[1] = 0.0;
    U[2] = ev0[0] * inv;
  } else {
    const double inv = 1.0 / sqrt(ev0[1] * ev0[1] + ev0[2] * ev0[2]);
    U[0] = 0.0;
    U[1] = ev0[2] * inv;
    U[2] = -ev0[1] * inv;
  }
  pcross(ev0, U, V);
  const double AU[3] = {A[0][0] * U[0] + A[0][1] * U[1] + A[0][2] * U[2],
                        A[0][1] * U[0] + A[1][1] * U[1] + A[1][2] * U[2],
                        A[0][2] * U[0] + A[1][2] * U[1] + A[2][2] * U[2]};
  const double AV[3] = {A[0][0] * V[0] + A[0][1] * V[1] + A[0][2] * V[2],
                        A[0][1] * V[0] + A[1][1] * V[1] + A[1][2] * V[2],
                        A[0][2] * V[0] + A[1][2] * V[1] + A[2][2] * V[2]};
  double m00 = U[0] * AU[0] + U[1] * AU[1] + U[2] * AU[2] - e1;
  double m01 = U[0] * AV[0] + U[1] * AV[1] + U[2] * AV[2];
  double m11 = V[0] * AV[0] + V[1] * AV[1] + V[2] * AV[2] - e1;
  const double a00 = fabs(m00), a01 = fabs(m01), a11 = fabs(m11);
  double cu, cv;  // out = cu·U − cv·V
  if (a00 >= a11) {
    if (fmax(a00, a01) > 0) {
      if (a00 >= a01) {
        m01 /= m00;
        m00 = 1.0 / sqrt(1.0 + m01 * m01);
        m01 *= m00;
      } else {
        m00 /= m01;
        m01 = 1.0 / sqrt(1.0 + m00 * m00);
        m00 *= m01;
      }
      cu = m01;
      cv = m00;
    } else {
      cu = 1.0;
      cv = 0.0;
    }
  } else {
    if (fmax(a11, a01) > 0) {
      if (a11 >= a01) {
        m01 /= m11;
        m11 = 1.0 / sqrt(1.0 + m01 * m01);
        m01 *= m11;
      } else {
        m11 /= m01;
        m01 = 1.0 / sqrt(1.0 + m11 * m11);
        m11 *= m01;
      }
      cu = m11;
      cv = m01;
    } else {
      cu = 1.0;
      cv = 0.0;
    }
  }
  for (int k = 0; k < 3; ++k) out[k] = (cv == 0.0 && cu == 1.0) ? U[k] : cu * U[k] - cv * V[k];
}

// Open3D FastEigen3x3: eigenvector of the smallest eigenvalue (oracle fast_eigen3x3)
__device__ void fast_eigen3x3(const double C[3][3], double out[3]) {
  double mx = C[0][0];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) mx = fmax(mx, C[r][c]);
  if (mx == 0.0) {
    out[0] = out[1] = out[2] = 0.0;
    return;
  }
  double A[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) A[r][c] = C[r][c] / mx;
  const double norm = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
  if (norm > 0) {
    const double q = (A[0][0] + A[1][1] + A[2][2]) / 3;
    const double b00 = A[0][0] - q, b11 = A[1][1] - q, b22 = A[2][2] - q;
    const double p = sqrt((b00 * b00 + b11 * b11 + b22 * b22 + norm * 2) / 6);
    const double c00 = b11 * b22 - A[1][2] * A[1][2];
    const double c01 = A[0][1] * b22 - A[1][2] * A[0][2];
    const double c02 = A[0][1] * A[1][2] - b11 * A[0][2];
    const double det = (b00 * c00 - A[0][1] * c01 + A[0][2] * c02) / (p * p * p);
    const double half_det = fmin(fmax(det * 0.5, -1.0), 1.0);
    const double angle = acos(half_det) / 3.0;
    const double two_thirds_pi = 2.09439510239319549;
    const double beta2 = cos(angle) * 2;
    const double beta0 = cos(angle + two_thirds_pi) * 2;
    const double beta1 = -(beta0 + beta2);
    const double e0 = q + p * beta0, e1 = q + p * beta1, e2 = q + p * beta2;
    double va[3], vb[3];
    if (half_det >= 0) {
      eigvec0(A, e2, va);
      if (e2 < e0 && e2 < e1) {
        for (int k = 0; k < 3; ++k) out[k] = va[k];
        return;
      }
      eigvec1(A, va, e1, vb);
      if (e1 < e0 && e1 < e2) {
        for (int k = 0; k < 3; ++k) out[k] = vb[k];
        return;
      }
      pcross(vb, va, out);
    } else {
      eigvec0(A, e0, va);
      if (e0 < e1 && e0 < e2) {
        for (int k = 0; k < 3; ++k) out[k] = va[k];
        return;
      }
      eigvec1(A, va, e1, vb);
      if (e1 < e0 && e1 < e2) {
        for (int k = 0; k < 3; ++k) out[k] = vb[k];
        return;
      }
      pcross(va, vb, out);
    }
    return;
  }
  out[0] = out[1] = out[2] = 0.0;
  if (A[0][0] < A[1][1] && A[0][0] < A[2][2])
    out[0] = 1.0;
  else if (A[1][1] < A[0][0] && A[1][1] < A[2][2])
    out[1] = 1.0;
  else
    out[2] = 1.0;
}

__global__ __launch_bounds__(kPrepBlock) void normals_kernel(const double* __restrict__ xyz64, int64_t n,
                                                             const int32_t* __restrict__ nbr, int k,
                                                             const int32_t* __restrict__ cnt,
                                                             const double* __restrict__ prev,
                                                             double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kPrepBlock + threadIdx.x;
  if (i >= n) return;
  const int c = cnt[i];
  double C[3][3];
  if (c < 3) {
    for (int r = 0; r < 3; ++r)
      for (int s = 0; s < 3; ++s) C[r][s] = r == s ? 1.0 : 0.0;
  } else {
    double cum[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < c; ++s) {
      const double* x = xyz64 + 3 * (int64_t)nbr[i * k + s];
      cum[0] += x[0];
      cum[1] += x[1];
      cum[2] += x[2];
      cum[3] += x[0] * x[0];
      cum[4] += x[0] * x[1];
      cum[5] += x[0] * x[2];
      cum[6] += x[1] * x[1];
      cum[7] += x[1] * x[2];
      cum[8] += x[2] * x[2];
    }
    for (int a = 0; a < 9; ++a) cum[a] /= (double)c;
    C[0][0] = cum[3] - cum[0] * cum[0];
    C[1][1] = cum[6] - cum[1] * cum[1];
    C[2][2] = cum[8] - cum[2] * cum[2];
    C[0][1] = C[1][0] = cum[4] - cum[0] * cum[1];
    C[0][2] = C[2][0] = cum[5] - cum[0] * cum[2];
    C[1][2] = C[2][1] = cum[7] - cum[1] * cum[2];
  }
  double nv[3];
  fast_eigen3x3(C, nv);
  if (nv[0] == 0.0 && nv[1] == 0.0 && nv[2] == 0.0) {
    if (prev != nullptr) {
      for (int a = 0; a < 3; ++a) nv[a] = prev[3 * i + a];
    } else {
      nv[2] = 1.0;
    }
  }
  if (prev != nullptr && pdot(nv, prev + 3 * i) < 0.0)
    for (int a = 0; a < 3; ++a) nv[a] = -nv[a];
  for (int a = 0; a < 3; ++a) out[3 * i + a] = nv[a];
}

// ------------------------------------------------------------------------------- FPFH
// ComputePairFeatures → (f0, f1, f2); returns false for the all-zero feature
__device__ bool pair_features(const double* p1, const double* n1in, const double* p2,
                              const double* n2in, double f[3]) {
  double dp[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  const double f3 = sqrt(pdot(dp, dp));
  f[0] = f[1] = f[2] = 0.0;
  if (f3 == 0.0) return true;
  const double a1 = pdot(n1in, dp) / f3, a2 = pdot(n2in, dp) / f3;
  const double* n1 = n1in;
  const double* n2 = n2in;
  double f2;
  // Open3D's swap test acos(|a1|) > acos(|a2|), decided as correctly rounded acos values would
  // (ddmath.h acos_gt: the device libm's ulp on a near tie would otherwise pick the other side)
#ifndef M3D_FPFH_CR_SWAP
#define M3D_FPFH_CR_SWAP 1  // 0: the device libm's acos on both sides (round 5; A/B only)
#endif
  if (M3D_FPFH_CR_SWAP ? acos_gt(fabs(a1), fabs(a2)) : acos(fabs(a1)) > acos(fabs(a2))) {
    n1 = n2in;
    n2 = n1in;
    for (int a = 0; a < 3; ++a) dp[a] = -dp[a];
    f2 = -a2;
  } else {
    f2 = a1;
  }
  double v[3], w[3];
  pcross(dp, n1, v);
  const double vn = sqrt(pdot(v, v));
  if (vn == 0.0) return true;
  for (int a = 0; a < 3; ++a) v[a] /= vn;
  pcross(n1, v, w);
  f[1] = pdot(v, n2);
  f[0] = atan2(pdot(w, n2), pdot(n1, n2));
  f[2] = f2;
  return true;
}

__device__ __forceinline__ int fbin(double x) {
  const int h = (int)floor(x);
  return h < 0 ? 0 : (h >= 11 ? 10 : h);
}

constexpr int kFeatBlock = 64;

__global__ __launch_bounds__(kFeatBlock) void spfh_kernel(const double* __restrict__ xyz64,
                                                          const double* __restrict__ nrm64, int64_t n,
                                                          const int32_t* __restrict__ nbr, int k,
                                                          const int32_t* __restrict__ cnt,
                                                          double* __restrict__ spfh) {
  __shared__ double h[33][kFeatBlock];
  const int lane = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * kFeatBlock + lane;
  for (int b = 0; b < 33; ++b) h[b][lane] = 0.0;
  if (i >= n) return;
  const int c = cnt[i];
  if (c > 1) {
    const double incr = 100.0 / (double)(c - 1);
    const double* p1 = xyz64 + 3 * i;
    const double* n1 = nrm64 + 3 * i;
    for (int s = 1; s < c; ++s) {
      const int64_t j = nbr[i * k + s];
      double f[3];
      pair_features(p1, n1, xyz64 + 3 * j, nrm64 + 3 * j, f);
      h[fbin(11 * (f[0] + M_PI) / (2.0 * M_PI))][lane] += incr;
      h[11 + fbin(11 * (f[1] + 1.0) * 0.5)][lane] += incr;
      h[22 + fbin(11 * (f[2] + 1.0) * 0.5)][lane] += incr;
    }
  }
  for (int b = 0; b < 33; ++b) spfh[i * 33 + b] = h[b][lane];
}

__global__ __launch_bounds__(kFeatBlock) void fpfh_kernel(const double* __restrict__ spfh, int64_t n,
                                                          const int32_t* __restrict__ nbr,
                                                          const double* __restrict__ d2, int k,
                                                          const int32_t* __restrict__ cnt,
                                                          double* __restrict__ out) {
  __shared__ double f[33][kFeatBlock];
  const int lane = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * kFeatBlock + lane;
  for (int b = 0; b < 33; ++b) f[b][lane] = 0.0;
  if (i >= n) return;
  const int c = cnt[i];
  if (c > 1) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int s = 1; s < c; ++s) {
      const double dist = d2[i * k + s];
      if (dist == 0.0) continue;
      const double* row = spfh + 33 * (int64_t)nbr[i * k + s];
      for (int b = 0; b < 11; ++b) {
        const double val = row[b] / dist;
        s0 += val;
        f[b][lane] += val;
      }
      for (int b = 11; b < 22; ++b) {
        const double val = row[b] / dist;
        s1 += val;
        f[b][lane] += val;
      }
      for (int b = 22; b < 33; ++b) {
        const double val = row[b] / dist;
        s2 += val;
        f[b][lane] += val;
      }
    }
    if (s0 != 0.0) s0 = 100.0 / s0;
    if (s1 != 0.0) s1 = 100.0 / s1;
    if (s2 != 0.0) s2 = 100.0 / s2;
    for (int b = 0; b < 33; ++b) {
      const double sc = b < 11 ? s0 : (b < 22 ? s1 : s2);
      f[b][lane] = f[b][lane] * sc + spfh[i * 33 + b];
    }
  }
  for (int b = 0; b < 33; ++b) out[i * 33 + b] = f[b][lane];
}

// ------------------------------------------------------------------------------- host side
static void free_all(std::initializer_list<void*> ps) {
  for (void* p : ps) hipFree(p);
}

// Device scratch of voxel_down_sample for n points (the caller's buffer, api.cpp): block
// partials of the bounds, 64-bit keys (in / sorted / unique), indices (in / sorted), run counts,
// offsets, the run count, and hipcub's temporary storage.
namespace {
struct VoxelScratch {
  size_t part, kin, kout, uniq, vin, vout, counts, offs, nruns, tmp, total, tmp_bytes;
};
VoxelScratch voxel_layout(int64_t n, int nb) {
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  VoxelScratch L{};
  size_t tb = 0, tb2 = 0, tb3 = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 63, (hipStream_t)0);
  hipcub::DeviceRunLengthEncode::Encode(nullptr, tb2, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                        (int32_t*)nullptr, (int32_t*)nullptr, (int)n, (hipStream_t)0);
  hipcub::DeviceScan::ExclusiveSum(nullptr, tb3, (int32_t*)nullptr, (int32_t*)nullptr, (int)n,
                                   (hipStream_t)0);
  L.tmp_bytes = std::max({tb, tb2, tb3, (size_t)1});
  size_t o = 0;
  L.part = o, o += up(sizeof(double) * 6 * (size_t)nb);
  L.kin = o, o += up(8 * (size_t)n);
  L.kout = o, o += up(8 * (size_t)n);
  L.uniq = o, o += up(8 * (size_t)n);
  L.vin = o, o += up(4 * (size_t)n);
  L.vout = o, o += up(4 * (size_t)n);
  L.counts = o, o += up(4 * (size_t)n);
  L.offs = o, o += up(4 * (size_t)n);
  L.nruns = o, o += up(4);
  L.tmp = o, o += up(L.tmp_bytes);
  L.total = o;
  return L;
}
int voxel_blocks(int64_t n) { return (int)std::min<int64_t>(1024, (n + kPrepBlock - 1) / kPrepBlock); }
}  // namespace

size_t voxel_scratch_bytes(int64_t n) { return n > 0 ? voxel_layout(n, voxel_blocks(n)).total : 0; }

hipError_t voxel_down_sample(const double* xyz, const double* nrm, int64_t n, double voxel,
                             double* out_xyz, double* out_nrm, int64_t* out_n, void* scratch,
                             hipStream_t st, std::string* why) {
  *out_n = 0;
  if (n == 0) return hipSuccess;
  const int nb = voxel_blocks(n);
  const VoxelScratch L = voxel_layout(n, nb);
  char* S = static_cast<char*>(scratch);
  double* part = reinterpret_cast<double*>(S + L.part);
  minmax3d_kernel<<<nb, kPrepBlock, 0, st>>>(xyz, n, part);
  std::vector<double> hp(6 * (size_t)nb);
  hipError_t e = hipMemcpyAsync(hp.data(), part, sizeof(double) * 6 * nb, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return e;
  double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (int b = 0; b < nb; ++b)
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], hp[6 * b + a]);
      hi[a] = std::max(hi[a], hp[6 * b + 3 + a]);
    }
  double vmin[3];
  for (int a = 0; a < 3; ++a) {
    vmin[a] = lo[a] - voxel * 0.5;
    const double cells = (hi[a] + voxel * 0.5 - vmin[a]) / voxel;
    if (!(cells < (double)(1 << 21))) {
      *why = "voxel_size is too small for the cloud extent (more than 2^21 voxels per axis)";
      return hipErrorInvalidValue;
    }
  }
  uint64_t* kin = reinterpret_cast<uint64_t*>(S + L.kin);
  uint64_t* kout = reinterpret_cast<uint64_t*>(S + L.kout);
  uint64_t* uniq = reinterpret_cast<uint64_t*>(S + L.uniq);
  int32_t* vin = reinterpret_cast<int32_t*>(S + L.vin);
  int32_t* vout = reinterpret_cast<int32_t*>(S + L.vout);
  int32_t* counts = reinterpret_cast<int32_t*>(S + L.counts);
  int32_t* offs = reinterpret_cast<int32_t*>(S + L.offs);
  int32_t* nruns = reinterpret_cast<int32_t*>(S + L.nruns);
  void* tmp = S + L.tmp;
  size_t tb = L.tmp_bytes;
  const unsigned blocks = (unsigned)((n + kPrepBlock - 1) / kPrepBlock);
  voxel_key_kernel<<<blocks, kPrepBlock, 0, st>>>(xyz, n, vmin[0], vmin[1], vmin[2], voxel, kin, vin);
  e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin, vout, (int)n, 0, 63, st);
  // counts past the number of runs stay zero, so the scan is well defined over all n entries
  if (e == hipSuccess) e = hipMemsetAsync(counts, 0, 4 * n, st);
  tb = L.tmp_bytes;
  if (e == hipSuccess)
    e = hipcub::DeviceRunLengthEncode::Encode(tmp, tb, kout, uniq, counts, nruns, (int)n, st);
  tb = L.tmp_bytes;
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, counts, offs, (int)n, st);
  if (e == hipSuccess) {
    voxel_mean_kernel<<<blocks, kPrepBlock, 0, st>>>(xyz, nrm, vout, counts, offs, nruns, out_xyz,
                                                     out_nrm);
    e = hipGetLastError();
  }
  int32_t h_runs = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&h_runs, nruns, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  *out_n = h_runs;
  return e;
}

// the fp32 box half-width that covers every point within `radius` (fp64) of a query: the
// radius plus the centring/rounding error of both fp32 coordinates
static float box_half_width(const m3d_cloud* c, double radius) {
  const double Rd = (radius + 2.0 * c->rmax * 5.9604644775390625e-08 * 1.01) * (1.0 + 1e-6);
  return (float)Rd * (1.0f + 1e-6f);
}

double hybrid_fine_radius(const Grid* g, double radius, int k) {
  constexpr double c = 0.5;  // the expected-count factor below
  if (k > 128 || g == nullptr || g->n_occ <= 0) return 0.0;
  // m = points per occupied radius-cell.  On a scanned surface ≈ 8 m (h / r)² points lie within
  // h (measured: the cfg4 scan, 1144 points within r against m = 139), so h = r·√(c·k / m)
  // expects ≈ 4 k of them at c = 0.5 (measured best of 0.3 / 0.5 / 0.8 once chunks merge in one
  // step; 0.3 before that).  The cost of the search is mostly the insertions, about
  // k·(1 + ln(N / k)) for N points within the searched radius, so a small h pays even though a
  // query with fewer than k points within it searches again; worth a second grid only well
  // below r.
  const double m = (double)g->n_pts / (double)g->n_occ;
  const double h = radius * sqrt(c * k / m);
  return h <= 0.6 * radius ? h : 0.0;
}

hipError_t hybrid_search(const m3d_cloud* c, const Grid* g, double radius, int k, int32_t* idx,
                         double* d2, int32_t* cnt, hipStream_t st, const Grid* gf, double hfine) {
  if (c->n == 0) return hipSuccess;
  const float Rf = box_half_width(c, radius);
  GridDev gfd{};
  gfd.ncells = 0;
  float Hf = 0.0f;
  double h2safe = 0.0;
  if (gf != nullptr && hfine > 0.0 && hfine < radius) {
    gfd = gf->dev;
    Hf = box_half_width(c, hfine);
    h2safe = hfine * hfine * (1.0 - 1e-12);
  }
  const int L = k <= 40 ? 64 : (k <= 80 ? 32 : (k <= 160 ? 16 : 8));
  const size_t lds = (size_t)k * L * (sizeof(double) + sizeof(int32_t));
  const double eabs = 3.4641016151377544 * c->rmax * 5.9604644775390625e-08 * 1.01;
  const unsigned wb = (unsigned)((c->n + 3) / 4);  // 4 waves (queries) per 256-thread block
  if (k <= 64) {
    hybrid_search_wave_kernel<1><<<wb, 256, 0, st>>>(c->xyz64, c->xyz32, c->n, g->dev, Rf,
                                                     radius * radius, eabs, k, gfd, Hf, h2safe,
                                                     idx, d2, cnt);
  } else if (k <= 128) {
    hybrid_search_wave_kernel<2><<<wb, 256, 0, st>>>(c->xyz64, c->xyz32, c->n, g->dev, Rf,
                                                     radius * radius, eabs, k, gfd, Hf, h2safe,
                                                     idx, d2, cnt);
  } else {
    hybrid_search_kernel<<<(unsigned)((c->n + L - 1) / L), L, lds, st>>>(
        c->xyz64, c->xyz32, c->n, g->dev, Rf, radius * radius, eabs, k, idx, d2, cnt);
  }
  return hipGetLastError();
}

hipError_t launch_normals(const m3d_cloud* c, const int32_t* nbr, int k, const int32_t* cnt,
                          const double* prev, double* out, hipStream_t st) {
  if (c->n == 0) return hipSuccess;
  normals_kernel<<<(unsigned)((c->n + kPrepBlock - 1) / kPrepBlock), kPrepBlock, 0, st>>>(
      c->xyz64, c->n, nbr, k, cnt, prev, out);
  return hipGetLastError();
}

// m3d_debug_acos_device: the swap test's acos on the device (mode 0: acos_cr, 1: the libm's acos)
__global__ void acos_probe_kernel(const double* __restrict__ u, int64_t n, double* __restrict__ out, int mode) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n) out[k] = mode == 0 ? acos_cr(u[k]) : acos(u[k]);
}

hipError_t launch_acos_probe(const double* u, int64_t n, double* out, int mode, hipStream_t st) {
  if (n == 0) return hipSuccess;
  acos_probe_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(u, n, out, mode);
  return hipGetLastError();
}

hipError_t launch_fpfh(const m3d_cloud* c, const double* nrm, const int32_t* nbr, const double* d2,
                       int k, const int32_t* cnt, double* spfh, double* out, hipStream_t st) {
  if (c->n == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((c->n + kFeatBlock - 1) / kFeatBlock);
  spfh_kernel<<<blocks, kFeatBlock, 0, st>>>(c->xyz64, nrm, c->n, nbr, k, cnt, spfh);
  fpfh_kernel<<<blocks, kFeatBlock, 0, st>>>(spfh, c->n, nbr, d2, k, cnt, out);
  return hipGetLastError();
}

}  // namespace m3d
