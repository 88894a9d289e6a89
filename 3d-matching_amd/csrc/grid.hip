// grid.hip — radius-bounded uniform-grid 1-NN for gfx950.
//
// Reference semantics: Open3D KDTreeFlann::SearchHybrid(p, r, max_nn = 1) inside
// GetRegistrationResultAndCorrespondences (a8).  The brute-force scan (icp.hip nn_kernel) and
// this path return the SAME key for every query: the lexicographic (fp32 d², index) minimum over
// the targets with d² ≤ r2_hi, where d² is the identical fp32 expression (d2f) of the identical
// fp32 query (xform32).  The grid only restricts which targets are visited, and it provably
// visits every target that can satisfy d² ≤ r2_hi:
//   * cell coordinate c(x) = trunc(clamp((x − o)·inv_h, 0, n−1)) is monotone in x (fp32
//     subtraction and multiplication by a positive constant are monotone under rounding);
//   * d2f(q, t) ≤ r2_hi ⇒ |q_k − t_k| ≤ R = 1.001·√r2_hi for every axis (each rounding of the
//     three-term sum shrinks by at most (1 − u)⁵ ≫ 1/1.001²);
//   * |q_k − t_k| ≤ R ⇒ fl(q_k − R) ≤ t_k ≤ fl(q_k + R) (t_k is representable) ⇒
//     c(fl(q_k − R)) ≤ c(t_k) ≤ c(fl(q_k + R)).
// So the cell box [c(q − R), c(q + R)] contains every candidate whatever the cell size; the cell
// size (≈ r) only sets how many cells a query visits (3 per axis).
//
// Layout in HBM: targets sorted by cell (row-major x fastest) as float4 (x, y, z, index bits),
// one int32 start offset per cell (+1).  For a query the cells of one (y, z) row are contiguous
// in the sorted array: ≤ 9 contiguous runs per query.  Queries are visited in the source cloud's
// own cell order (spatially coherent waves → the 9 runs of neighbouring lanes overlap in L2).
// Build: per-axis bounds (min/max reduction), cell ids, hipcub radix sort of (cell, index)
// pairs (stable → deterministic layout), cell starts by binary search, gather.
#include <float.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "m3d_internal.h"
#include "nnkey.h"

namespace m3d {

constexpr int kGridBlock = 256;
constexpr int64_t kMaxCells = (int64_t)1 << 25;

__global__ __launch_bounds__(kGridBlock) void minmax3_kernel(const float4* __restrict__ p, int64_t n,
                                                             float* __restrict__ part) {
  __shared__ float s[6][kGridBlock];
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t i = (int64_t)blockIdx.x * kGridBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGridBlock) {
    const float4 v = p[i];
    const float c[3] = {v.x, v.y, v.z};
    for (int k = 0; k < 3; ++k) {
      lo[k] = fminf(lo[k], c[k]);
      hi[k] = fmaxf(hi[k], c[k]);
    }
  }
  for (int k = 0; k < 3; ++k) {
    s[k][threadIdx.x] = lo[k];
    s[3 + k][threadIdx.x] = hi[k];
  }
  __syncthreads();
  for (int w = kGridBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < 3; ++k) {
        s[k][threadIdx.x] = fminf(s[k][threadIdx.x], s[k][threadIdx.x + w]);
        s[3 + k][threadIdx.x] = fmaxf(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + w]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 6) part[6 * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

__global__ __launch_bounds__(kGridBlock) void cell_id_kernel(const float4* __restrict__ p, int64_t n,
                                                             GridDev g, uint32_t* __restrict__ key,
                                                             int32_t* __restrict__ val) {
  const int64_t i = (int64_t)blockIdx.x * kGridBlock + threadIdx.x;
  if (i >= n) return;
  const float4 v = p[i];
  const int cx = grid_coord(v.x, g.o[0], g.inv_h, g.n[0]);
  const int cy = grid_coord(v.y, g.o[1], g.inv_h, g.n[1]);
  const int cz = grid_coord(v.z, g.o[2], g.inv_h, g.n[2]);
  key[i] = (uint32_t)(((int64_t)cz * g.n[1] + cy) * g.n[0] + cx);
  val[i] = (int32_t)i;
}

// Cell starts from the sorted keys without a search: the last point of each cell's run writes
// its end position into end[cell + 1] (end zeroed first), and start = the inclusive MAX scan of
// end (hipcub): start[c] = the end of the last occupied cell before c = the number of points whose
// cell is < c, start[ncells] = n.  Round 4 ran a binary search over all n keys for every cell: up
// to 207 µs at 1M points.
__global__ __launch_bounds__(kGridBlock) void cell_end_kernel(const uint32_t* __restrict__ key, int64_t n,
                                                              int32_t* __restrict__ end) {
  const int64_t k = (int64_t)blockIdx.x * kGridBlock + threadIdx.x;
  if (k < n && (k == n - 1 || key[k] != key[k + 1])) end[(int64_t)key[k] + 1] = (int32_t)(k + 1);
}

// occupied cells: sorted positions that start a new cell
__global__ __launch_bounds__(kGridBlock) void count_occupied_kernel(const uint32_t* __restrict__ key,
                                                                    int64_t n,
                                                                    unsigned long long* __restrict__ occ) {
  const int64_t k = (int64_t)blockIdx.x * kGridBlock + threadIdx.x;
  const bool first = k < n && (k == 0 || key[k] != key[k - 1]);
  const unsigned long long b = __ballot(first);
  if ((threadIdx.x & (kWave - 1)) == 0 && b != 0) atomicAdd(occ, (unsigned long long)__popcll(b));
}

__global__ __launch_bounds__(kGridBlock) void grid_gather_kernel(const float4* __restrict__ p,
                                                                 const int32_t* __restrict__ val,
                                                                 int64_t n,
                                                                 float4* __restrict__ pts) {
  const int64_t k = (int64_t)blockIdx.x * kGridBlock + threadIdx.x;
  if (k >= n) return;
  const int32_t j = val[k];
  const float4 v = p[j];
  pts[k] = make_float4(v.x, v.y, v.z, __int_as_float(j));
}

// ------------------------------------------------------------------------------- query

// ------------------------------------------------------------------------------- query
// kL lanes per query over the Morton query order (the scan state of nnkey.h per lane: packed
// (bits(d²) << 32 | index) minimum and runner-up near2, lanes combined by shuffles; a key compare
// is the lexicographic (d², index) compare of the brute-force scan), the queries straight from the
// Morton-sorted points (no order[] indirection).  Every lane of a query sees every cell row of
// its box and takes the row's points sub, sub + kL, …: the start offsets of kR rows are loaded
// together, then kR × kB point loads per lane go out at once, so a typical seeded query (≤ kR
// rows of ≤ kL·kB points) costs one round of start loads and one round of point loads instead of
// one dependent load per point.  Blocks are remapped XCD-contiguously (blocks b and b + 8 share
// an XCD's L2: each XCD gets one contiguous slice of the Morton order, so its L2 holds one
// region's targets and cell starts instead of every region's).
#if M3D_SCAN_CLOCK  // diagnostic builds only (tools/scan_clock.py): per-wave start / end of the
                    // grid scan, s_memrealtime (100 MHz)
__device__ unsigned long long g_scan_clock[2 * 65536];
#endif
#ifndef M3D_SCAN_PHASE1
#define M3D_SCAN_PHASE1 1
#endif
// append query t to the deferral list; a slot at or past the list's capacity (a count the loop
// did not produce: it starts at zero at creation and at every reset) is dropped and flagged in
// hcnt[kDeferFault] (m3d_icp_result_get then fails) — never written out of bounds
__device__ __forceinline__ void defer_push(int32_t* __restrict__ hlist, uint32_t* __restrict__ hcnt,
                                           uint32_t hcap, int32_t t) {
  const uint32_t slot = atomicAdd(hcnt, 1u);
  if (slot < hcap)
    hlist[slot] = t;
  else
    __hip_atomic_store(hcnt + kDeferFault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int kL, int kR, int kB, bool kDefer = false>
__global__ __launch_bounds__(kGridBlock) void grid_nn_batched_kernel(
    const float4* __restrict__ qpts, int64_t ns, GridDev g, int64_t off,
    const IcpState* __restrict__ s, int64_t* __restrict__ keys, uint32_t* __restrict__ near2,
    const int32_t* __restrict__ prev, const int64_t* __restrict__ dprev,
    const float4* __restrict__ tgt32, int64_t nt_shard, int64_t nblocks, int64_t q0,
    int32_t* __restrict__ hlist, uint32_t* __restrict__ hcnt, int cand_cap, uint32_t hcap, int xchunk) {
  if (s->done) return;
#if M3D_SCAN_CLOCK
  const unsigned long long clk0 = __builtin_amdgcn_s_memrealtime();
#endif
  // block b runs on XCD b % 8.  xchunk = 0: XCD k takes the k-th eighth of the Morton order (one
  // region per L2); xchunk = C: XCD k takes chunks k, k + 8, … of C consecutive blocks (the launch
  // is a multiple of 8·C blocks), so work concentrated in one part of the cloud — a spatial target
  // shard, whose queries are Morton-contiguous slabs — spreads over all eight XCDs
  int64_t blk;
  if (xchunk <= 0) {
    const int64_t per = (nblocks + 7) / 8;
    blk = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  } else {
    const int64_t j = blockIdx.x / 8, k = blockIdx.x % 8;
    blk = ((j / xchunk) * 8 + k) * xchunk + j % xchunk;
  }
  if (blk >= nblocks) return;
  const int64_t t = q0 + (blk * kGridBlock + threadIdx.x) / kL;  // queries [q0, ns) in Morton order
  const int sub = threadIdx.x & (kL - 1);
  const float r2_hi = s->r2_hi, be = s->band_e;
  const uint64_t key0 = ((uint64_t)__float_as_uint(r2_hi) << 32) | 0xFFFFFFFFull;
  uint64_t k1 = key0;
  float k1d = kInf, n2 = kInf;
  int64_t i = -1;
  if (t < ns) {
    // qpts are the loop's Morton copy (morton_copy_kernel: w = position = slot), so i = t, and the
    // previous correspondence is loaded beside the point instead of after it
    i = t;
    // (the point first: the prev load sits under a scalar branch whose wait would otherwise come
    // before the point load is issued — one round trip for both instead of two)
    const float4 p = qpts[t];
    const int32_t pj = prev != nullptr ? prev[t] : -1;
    float qx, qy, qz;
    xform32(s->Rt32, p, qx, qy, qz);
    // a query whose largest box (q ± 1.001·√r2_hi: any seed only shrinks it) misses this grid has
    // no target of the shard within r2_hi: no seed (an own previous target would lie in that box;
    // another shard's bound is a pseudo key, which every consumer reads as "none"), no scan — on a
    // spatial target shard (m3d.dist.spatial_shards) most queries leave here, before the dprev load
    const bool far = g.ncells > 0 && grid_box_miss(g, qx, qy, qz, sqrtf(r2_hi) * 1.001f);
    // seed: the previous correspondence re-evaluated (nnkey.h seed_key), or a bound
    const int64_t seed = far ? kKeyNone : seed_key_j(s, pj, i, p, qx, qy, qz, tgt32, nt_shard, off, dprev);
    if (seed != kKeyNone) k1 = (uint64_t)seed;
    k1d = key_real_d2(k1);
    if (g.ncells > 0 && !far) {
      float R = sqrtf(search_bound(key_d2(k1), be, r2_hi)) * 1.001f;
      if (M3D_SCAN_PHASE1 && 2.0f * R * g.inv_h > 3.0f) {
        // a box wider than ~4 cells per axis (no seed, or a seed the update moved far — the first
        // evaluations; a dense target, where the cells are r/2 … r/4): the half-cell box around
        // the query first, every lane over every point (so each lane's state holds the same
        // points: the second pass's repeats change neither k1 nor near2), then the box of the
        // bound that leaves
        grid_scan<1, kR, kB>(g, qx, qy, qz, 0.5f / g.inv_h, r2_hi, off, 0, k1, k1d, n2);
        R = fminf(R, sqrtf(search_bound(key_d2(k1), be, r2_hi)) * 1.001f);
      }
      int rows = 0, cand = 0;
      grid_scan<kL, kR, kB>(g, qx, qy, qz, R, r2_hi, off, sub, k1, k1d, n2, &rows, &cand,
                            kDefer ? cand_cap : 0x7FFFFFFF);
      if (kDefer && cand > cand_cap) {  // a dense box: grid_nn_heavy_kernel scans it with a whole block
        if (sub == 0) defer_push(hlist, hcnt, hcap, (int32_t)t);
        i = -1;
      }
    }
  }
  grid_merge_lanes<kL>(k1, k1d, n2);
  // deferral mode: an ambiguous query (the terms pass's test, nnkey.h winner_fp64) is decided in
  // fp64 by grid_nn_heavy_kernel too — a dense cluster makes whole waves ambiguous, and the terms
  // pass resolves a wave's queries one after another.  (Deciding them here in the scan for every
  // loop was measured in round 5: the scan grew by what the terms pass saved)
  const float X = kDefer && i >= 0 && k1 != key0 ? search_bound(key_d2(k1), be, r2_hi) : -1.0f;
  const bool amb = X >= 0.0f && n2 <= X;
  if (i >= 0 && sub == 0) {
    keys[i] = k1 == key0 ? kKeyNone : (int64_t)k1;
    near2[i] = __float_as_uint(n2);
    if (kDefer && amb) defer_push(hlist, hcnt, hcap, (int32_t)t);
  }
#if M3D_SCAN_CLOCK
  {
    const unsigned long long clk1 = __builtin_amdgcn_s_memrealtime();
    const int64_t gw = (int64_t)blockIdx.x * (kGridBlock / kWave) + threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0 && gw < 65536) {
      g_scan_clock[2 * gw] = clk0;
      g_scan_clock[2 * gw + 1] = clk1;
    }
  }
#endif
}

// Deferred queries of grid_nn_batched_kernel<..., true>: those with more than cand_cap candidates
// in their box (the cells of a dense cluster, where kL lanes would walk hundreds of points each
// and one wave would hold the whole launch) and the ambiguous ones (runner-up within the band).
// One block per query, its 4 waves over the box's rows and each wave's 64 lanes over a row's
// points: same seed, same box, same pushes as the per-query scan, merged by the same near_merge
// — the same (k1, near2) bits; an ambiguous query is then decided in fp64 here (below).  The
// list's count is re-zeroed by the last block (hcnt[1] = block ticket).
__global__ __launch_bounds__(kGridBlock) void grid_nn_heavy_kernel(
    const float4* __restrict__ qpts, GridDev g, int64_t off, const IcpState* __restrict__ s,
    int64_t* __restrict__ keys, uint32_t* __restrict__ near2, const int32_t* __restrict__ prev, const int64_t* __restrict__ dprev,
    const float4* __restrict__ tgt32, int64_t nt_shard, const int32_t* __restrict__ hlist,
    uint32_t* __restrict__ hcnt, const double* __restrict__ src64,
    const double* __restrict__ tgt64, int64_t nq, uint32_t hcap) {
  constexpr int kWaves = kGridBlock / kWave;
  constexpr int kHU = 4;
  __shared__ uint64_t wk[kWaves];
  __shared__ float wn[kWaves];
  __shared__ double wd[kWaves];
  __shared__ int64_t wj[kWaves];
  if (s->done) return;
  uint32_t nh = __hip_atomic_load(hcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (nh > hcap) {  // an overflowed list (flagged by the scan's defer_push): nothing is read from it
    nh = 0;
    if (threadIdx.x == 0) __hip_atomic_store(hcnt + kDeferFault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const float r2_hi = s->r2_hi, be = s->band_e;
  const uint64_t key0 = ((uint64_t)__float_as_uint(r2_hi) << 32) | 0xFFFFFFFFull;
  for (uint32_t h = blockIdx.x; h < nh; h += gridDim.x) {
    const int64_t t = hlist[h];
    if (t < 0 || t >= nq) {  // (cannot happen for a list this loop wrote; flagged, never dereferenced)
      if (threadIdx.x == 0) __hip_atomic_store(hcnt + kDeferFault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    const float4 p = qpts[t];
    const int64_t i = (int64_t)__float_as_int(p.w);
#ifdef M3D_DEBUG_GUARDS
    if (i < 0 || i >= nq) {
      if (threadIdx.x == 0) printf("[guard] heavy t %lld: i %lld outside [0, %lld)\n", (long long)t, (long long)i, (long long)nq);
      continue;
    }
#endif
    float qx, qy, qz;
    xform32(s->Rt32, p, qx, qy, qz);
    const int64_t seed = seed_key(s, i, p, qx, qy, qz, tgt32, nt_shard, off, prev, dprev);
    uint64_t k1 = seed != kKeyNone ? (uint64_t)seed : key0;
    float k1d = key_real_d2(k1), n2 = kInf;
    const float R = sqrtf(search_bound(key_d2(k1), be, r2_hi)) * 1.001f;
    const int x0 = grid_coord(qx - R, g.o[0], g.inv_h, g.n[0]);
    const int x1 = grid_coord(qx + R, g.o[0], g.inv_h, g.n[0]);
    const int y0 = grid_coord(qy - R, g.o[1], g.inv_h, g.n[1]);
    const int y1 = grid_coord(qy + R, g.o[1], g.inv_h, g.n[1]);
    const int z0 = grid_coord(qz - R, g.o[2], g.inv_h, g.n[2]);
    const int z1 = grid_coord(qz + R, g.o[2], g.inv_h, g.n[2]);
    const int ny = y1 - y0 + 1;
    const int rows = ny * (z1 - z0 + 1);
    for (int r = wave; r < rows; r += kWaves) {
      const int64_t row = ((int64_t)(z0 + r / ny) * g.n[1] + (y0 + r % ny)) * g.n[0];
      const int32_t a = g.start[row + x0], b = g.start[row + x1 + 1];
      // kHU points per lane per round trip (unconditional loads, slot 0 past the row's end)
      for (int32_t j0 = a + lane; j0 < b; j0 += kHU * kWave) {
        float4 v[kHU];
#pragma unroll
        for (int u = 0; u < kHU; ++u) v[u] = g.pts[j0 + u * kWave < b ? j0 + u * kWave : 0];
#pragma unroll
        for (int u = 0; u < kHU; ++u)
          if (j0 + u * kWave < b)
            push_within(k1, k1d, n2, d2f(qx, qy, qz, v[u].x, v[u].y, v[u].z), r2_hi,
                        (uint32_t)(off + __float_as_int(v[u].w)));
      }
    }
    grid_merge_lanes<kWave>(k1, k1d, n2);
    if (lane == 0) {
      wk[wave] = k1;
      wn[wave] = n2;
    }
    __syncthreads();
    for (int w = 0; w < kWaves; ++w)  // every thread merges the same states in the same order
      if (w != wave) near_merge(k1, k1d, n2, wk[w], wn[w]);
    // the terms pass's ambiguity test (nnkey.h winner_fp64); an ambiguous query is decided here by
    // the whole block as resolve_wave does: every target of the q ± 1.001·√X box with d2f ≤ X
    // re-evaluated in fp64, the lexicographic (d64, index) minimum among d64 < r2 — written as the
    // key with near2 = none, which the terms pass then takes as it is (its fp64 re-check of k1's
    // target gives the same d64)
    const float X = k1 != key0 ? search_bound(key_d2(k1), be, r2_hi) : -1.0f;
    if (!(X >= 0.0f && n2 <= X)) {
      if (threadIdx.x == 0) {
        keys[i] = k1 == key0 ? kKeyNone : (int64_t)k1;
        near2[i] = __float_as_uint(n2);
      }
    } else {
      double Q[3];
      q64_of(s->dT, src64 + 3 * i, Q);  // src64: the loop's points (dT·pcd64, icp.hip)
      double dl = kInf;
      int64_t jl = INT64_MAX;
      const float RX = sqrtf(X) * 1.001f;
      const int a0 = grid_coord(qx - RX, g.o[0], g.inv_h, g.n[0]);
      const int a1 = grid_coord(qx + RX, g.o[0], g.inv_h, g.n[0]);
      const int b0 = grid_coord(qy - RX, g.o[1], g.inv_h, g.n[1]);
      const int b1 = grid_coord(qy + RX, g.o[1], g.inv_h, g.n[1]);
      const int c0 = grid_coord(qz - RX, g.o[2], g.inv_h, g.n[2]);
      const int c1 = grid_coord(qz + RX, g.o[2], g.inv_h, g.n[2]);
      const int nby = b1 - b0 + 1;
      const int xrows = nby * (c1 - c0 + 1);
      for (int r = wave; r < xrows; r += kWaves) {
        const int64_t row = ((int64_t)(c0 + r / nby) * g.n[1] + (b0 + r % nby)) * g.n[0];
        const int32_t b = g.start[row + a1 + 1];
        for (int32_t j = g.start[row + a0] + lane; j < b; j += kWave) {
          const float4 v = g.pts[j];
          if (!(d2f(qx, qy, qz, v.x, v.y, v.z) <= X)) continue;
          const int64_t lj = (int64_t)__float_as_int(v.w);
#ifdef M3D_DEBUG_GUARDS
          if (lj < 0 || lj >= nt_shard) { printf("[guard] heavy resolve lj %lld nt %lld j %d\n", (long long)lj, (long long)nt_shard, j); continue; }
#endif
          const double* tp = tgt64 + 3 * lj;
          const double dx = Q[0] - tp[0], dy = Q[1] - tp[1], dz = Q[2] - tp[2];
          const double d = (dx * dx + dy * dy) + dz * dz;
          const int64_t gj = off + lj;
          if (d < s->r2 && (d < dl || (d == dl && gj < jl))) {
            dl = d;
            jl = gj;
          }
        }
      }
#pragma unroll
      for (int o = kWave / 2; o > 0; o >>= 1) {
        const double od = __shfl_xor(dl, o);
        const int64_t oj = __shfl_xor(jl, o);
        if (od < dl || (od == dl && oj < jl)) {
          dl = od;
          jl = oj;
        }
      }
      if (lane == 0) {
        wd[wave] = dl;
        wj[wave] = jl;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        for (int w = 1; w < kWaves; ++w)
          if (wd[w] < dl || (wd[w] == dl && wj[w] < jl)) {
            dl = wd[w];
            jl = wj[w];
          }
        keys[i] = jl == INT64_MAX ? kKeyNone : (int64_t)make_key(__double2float_ru(dl), (uint32_t)jl);
        near2[i] = kNearNone;
      }
    }
    __syncthreads();
  }
  // the list is consumed: the last block to finish zeroes the count (and this ticket) for the
  // next launch, so a loop needs no per-step memset node (count, ticket and fault word are zeroed
  // at loop creation before the setup sync, and by every m3d_icp_reset on the caller's stream).
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(hcnt + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
    __hip_atomic_store(hcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(hcnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------------------- a6 validation
// Feature-RANSAC validation of many hypotheses in one launch (Open3D
// RegistrationRANSACBasedOnCorrespondence evaluates every checker-passing hypothesis with
// GetRegistrationResultAndCorrespondences — 1-NN within the distance threshold, fitness =
// count / Ns, rmse = √(Σd² / count)).  blockIdx.y = hypothesis k of the batch (its evaluation
// state states[k], icp.hip val_states_kernel); kL lanes per source point, the source in its
// Morton order.  Per point: the unseeded scan of the grid NN (r2_hi box, packed-key minimum and
// runner-up), then nnkey.h winner_fp64 — the same fp64 decision as the single-hypothesis chain
// (set_T → grid NN → terms) it replaces, so the (count, Σd²) pairs are the same up to the
// summation order.  Block partials (count, Σd²) go out in a fixed tree order; val_reduce_kernel
// adds them per hypothesis in block order: deterministic.
template <int kL>
__global__ __launch_bounds__(kGridBlock) void validate_kernel(const float4* __restrict__ qpts,
                                                              int64_t ns,
                                                              const double* __restrict__ src64,
                                                              GridDev g,
                                                              const double* __restrict__ tgt64,
                                                              int64_t nt,
                                                              const IcpState* __restrict__ states,
                                                              double* __restrict__ part) {
  __shared__ double red[2][kGridBlock / kWave];
  const IcpState* s = states + blockIdx.y;
  const int64_t t = ((int64_t)blockIdx.x * kGridBlock + threadIdx.x) / kL;
  const int sub = threadIdx.x & (kL - 1);
  const float r2_hi = s->r2_hi;
  const uint64_t key0 = ((uint64_t)__float_as_uint(r2_hi) << 32) | 0xFFFFFFFFull;
  uint64_t k1 = key0;
  float k1d = kInf, n2 = kInf;
  int64_t i = -1;
  float4 p = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (t < ns) {
    p = qpts[t];
    i = (int64_t)__float_as_int(p.w);
    float qx, qy, qz;
    xform32(s->Rt32, p, qx, qy, qz);
    if (g.ncells > 0) {
      const float R = sqrtf(r2_hi) * 1.001f;
      // the grid scan's batched rows and points (nnkey.h grid_scan: kL lanes over each row, the
      // loads of 2 rows × 2 points per lane in one round trip); the (k1, near2) of the merged
      // lanes do not depend on which lane pushed which target
      grid_scan<kL, 2, 2>(g, qx, qy, qz, R, r2_hi, 0, sub, k1, k1d, n2);
    }
  }
#pragma unroll
  for (int o = kL / 2; o > 0; o >>= 1) {
    const uint64_t b1 = ((uint64_t)(uint32_t)__shfl_xor((int)(k1 >> 32), o, kL) << 32) |
                        (uint32_t)__shfl_xor((int)(uint32_t)k1, o, kL);
    const float bn2 = __shfl_xor(n2, o, kL);
    near_merge(k1, k1d, n2, b1, bn2);
  }
  const bool valid = i >= 0 && sub == 0;
  double Q[3] = {0.0, 0.0, 0.0};
  if (valid) q64_of(s->T, src64 + 3 * i, Q);
  int64_t bj = -1;
  double bd = 0.0;
  winner_fp64(valid, k1 == key0 ? (uint64_t)kKeyNone : k1, n2, s, g, tgt64, 0, nt, p, Q, bj, bd);
  double c = valid && bj >= 0 ? 1.0 : 0.0;
  double e = valid && bj >= 0 ? bd : 0.0;
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    e += __shfl_xor(e, o);
  }
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) {
    red[0][wave] = c;
    red[1][wave] = e;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double v = 0.0;
    for (int w = 0; w < kGridBlock / kWave; ++w) v += red[threadIdx.x][w];
    part[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 2 + threadIdx.x] = v;
  }
}

// out[2k] = count, out[2k + 1] = Σd² of hypothesis k: its nb block partials in block order
__global__ __launch_bounds__(kWave) void val_reduce_kernel(const double* __restrict__ part, int64_t nb,
                                                          double* __restrict__ out) {
  const double* p = part + (int64_t)blockIdx.x * nb * 2;
  double c = 0.0, e = 0.0;
  for (int64_t b = threadIdx.x; b < nb; b += kWave) {
    c += p[2 * b];
    e += p[2 * b + 1];
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    e += __shfl_xor(e, o);
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = c;
    out[2 * blockIdx.x + 1] = e;
  }
}

int64_t validate_blocks(int64_t ns) { return (ns * 4 + kGridBlock - 1) / kGridBlock; }

hipError_t launch_validate(const Grid* qgrid, int64_t ns, const double* src64, const Grid* g,
                           const double* tgt64, int64_t nt, const IcpState* states, int64_t nhyp,
                           double* part, double* out, hipStream_t st) {
  if (nhyp == 0) return hipSuccess;
  if (ns == 0) return hipMemsetAsync(out, 0, sizeof(double) * 2 * nhyp, st);
  if (qgrid == nullptr || qgrid->mpts == nullptr) return hipErrorInvalidValue;
  const int64_t nb = validate_blocks(ns);
  if (nb > INT32_MAX || nhyp > 65535) return hipErrorInvalidValue;
  validate_kernel<4><<<dim3((unsigned)nb, (unsigned)nhyp), kGridBlock, 0, st>>>(
      qgrid->mpts, ns, src64, g->dev, tgt64, nt, states, part);
  val_reduce_kernel<<<(unsigned)nhyp, kWave, 0, st>>>(part, nb, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------- host side
static hipError_t grid_fail(hipError_t e, void* a, void* b, void* c, void* d, void* tmp) {
  hipFree(a);
  hipFree(b);
  hipFree(c);
  hipFree(d);
  hipFree(tmp);
  return e;
}

// Occupied cells from the built grid itself: sorted positions whose cell differs from the
// previous point's (the cell of a point recomputed from its coordinates as cell_id_kernel does),
// and the most points in one cell (the first point of each cell reads its cell's range).  Per
// block (grid-stride, a fixed grid) a count and a max into part[2·block], then occ_final_kernel
// adds / maxes the partials — no atomics: round 4 had every wave add into the same two words
// (up to 367 µs at 1M points).
constexpr int kOccBlocks = 1024;
__global__ __launch_bounds__(kGridBlock) void count_occupied_pts_kernel(const float4* __restrict__ pts,
                                                                        int64_t n, GridDev g,
                                                                        uint32_t* __restrict__ part) {
  auto cell_of = [&](int64_t j) {
    const float4 v = pts[j];
    const int cx = grid_coord(v.x, g.o[0], g.inv_h, g.n[0]);
    const int cy = grid_coord(v.y, g.o[1], g.inv_h, g.n[1]);
    const int cz = grid_coord(v.z, g.o[2], g.inv_h, g.n[2]);
    return ((int64_t)cz * g.n[1] + cy) * g.n[0] + cx;
  };
  uint32_t cnt = 0, run = 0;
  for (int64_t k = (int64_t)blockIdx.x * kGridBlock + threadIdx.x; k < n; k += (int64_t)gridDim.x * kGridBlock) {
    const int64_t c = cell_of(k);
    if (k == 0 || c != cell_of(k - 1)) {
      ++cnt;
      run = max(run, (uint32_t)(g.start[c + 1] - g.start[c]));
    }
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    run = max(run, (uint32_t)__shfl_xor(run, o));
  }
  __shared__ uint32_t sc[kGridBlock / kWave], sr[kGridBlock / kWave];
  if ((threadIdx.x & (kWave - 1)) == 0) {
    sc[threadIdx.x / kWave] = cnt;
    sr[threadIdx.x / kWave] = run;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0, r = 0;
    for (int w = 0; w < kGridBlock / kWave; ++w) {
      c += sc[w];
      r = max(r, sr[w]);
    }
    part[2 * blockIdx.x] = c;
    part[2 * blockIdx.x + 1] = r;
  }
}

__global__ __launch_bounds__(kOccBlocks) void occ_final_kernel(const uint32_t* __restrict__ part, int nb,
                                                               unsigned long long* __restrict__ occ) {
  __shared__ unsigned long long sc[kOccBlocks / kWave];
  __shared__ uint32_t sr[kOccBlocks / kWave];
  unsigned long long c = threadIdx.x < nb ? part[2 * threadIdx.x] : 0;
  uint32_t r = threadIdx.x < nb ? part[2 * threadIdx.x + 1] : 0;
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    r = max(r, (uint32_t)__shfl_xor(r, o));
  }
  if ((threadIdx.x & (kWave - 1)) == 0) {
    sc[threadIdx.x / kWave] = c;
    sr[threadIdx.x / kWave] = r;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kOccBlocks / kWave; ++w) {
      c += sc[w];
      r = max(r, sr[w]);
    }
    occ[0] = c;
    occ[1] = r;
  }
}

// The dense cell array over [lo, hi] for a requested cell size: origin, cells per axis, 1/h; the
// cell grows until the grid has at most kMaxCells cells.  Returns the cell size h.
static double grid_params(const float lo[3], const float hi[3], double cell, GridDev& d) {
  double h = cell > 0.0 && std::isfinite(cell) ? cell : 1.0;
  int64_t nn[3], total = 0;
  for (;;) {
    total = 1;
    for (int k = 0; k < 3; ++k) {
      const double ext = std::isfinite((double)hi[k] - lo[k]) ? (double)hi[k] - lo[k] : 0.0;
      nn[k] = (int64_t)std::floor(ext / h) + 1;
      total *= nn[k];
      if (total > kMaxCells) break;
    }
    if (total <= kMaxCells) break;
    h *= 1.26;
  }
  for (int k = 0; k < 3; ++k) {
    d.o[k] = lo[k];
    d.n[k] = (int)nn[k];
  }
  d.inv_h = (float)(1.0 / h);
  d.ncells = total;
  return h;
}

hipError_t grid_build(const float4* xyz32, int64_t n, double cell, hipStream_t st, Grid* g, TmpArena* ta,
                      const float* lohi) {
  g->n_pts = n;
  g->cell = cell;
  g->n_occ = 0;
  g->occ_known = n == 0;
  GridDev& d = g->dev;
  d.ncells = 0;
  if (n == 0) return hipSuccess;
  hipError_t e = hipSuccess;
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  if (lohi != nullptr) {  // the cloud's packing pass already reduced them: no pass, no sync
    for (int k = 0; k < 3; ++k) {
      lo[k] = lohi[k];
      hi[k] = lohi[3 + k];
    }
  } else {  // per-axis bounds: one pass + one sync
    const int nb = (int)std::min<int64_t>(1024, (n + kGridBlock - 1) / kGridBlock);
    float* part = nullptr;
    e = dev_malloc(&part, sizeof(float) * 6 * nb);
    if (e != hipSuccess) return e;
    minmax3_kernel<<<nb, kGridBlock, 0, st>>>(xyz32, n, part);
    std::vector<float> hp(6 * (size_t)nb);
    e = hipMemcpyAsync(hp.data(), part, sizeof(float) * 6 * nb, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    hipFree(part);
    if (e != hipSuccess) return e;
    for (int b = 0; b < nb; ++b)
      for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(lo[k], hp[6 * b + k]);
        hi[k] = std::max(hi[k], hp[6 * b + 3 + k]);
      }
  }
  const double h = grid_params(lo, hi, cell, d);
  const int64_t total = d.ncells;
  g->cell = h;
  // (cell, index) pairs → stable radix sort; the sorted indices land in g->order
  uint32_t *kin = nullptr, *kout = nullptr;
  int32_t* vin = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  int bits = 1;
  while (bits < 32 && ((int64_t)1 << bits) < total) ++bits;
  if (g->block != nullptr) {  // a rebuild: the previous cell arrays (one block)
    block_release(g->block);
    g->block = nullptr;
    g->block_bytes = 0;
  } else {
    hipFree(g->start);
    hipFree(g->pts);
    hipFree(g->order);
  }
  g->start = nullptr;
  g->pts = nullptr;
  g->order = nullptr;
  int32_t* cnt = nullptr;
  size_t scan_bytes = 0;
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin, g->order, (int)n, 0, bits, st);
  if (e == hipSuccess)
    e = hipcub::DeviceScan::InclusiveScan(nullptr, scan_bytes, cnt, g->start, hipcub::Max(), (int)(total + 1), st);
  if (e != hipSuccess) return e;
  tmp_bytes = std::max<size_t>({tmp_bytes, scan_bytes, 1});  // the sort's and the scan's temporaries
  const size_t a4 = tmp_align(sizeof(uint32_t) * (size_t)n);
  const size_t ac = tmp_align(sizeof(int32_t) * (size_t)(total + 1));
  if (ta != nullptr) {
    if ((e = ta->reserve(3 * a4 + ac + tmp_align(tmp_bytes))) != hipSuccess) return e;
    kin = reinterpret_cast<uint32_t*>(ta->base);
    kout = reinterpret_cast<uint32_t*>(ta->base + a4);
    vin = reinterpret_cast<int32_t*>(ta->base + 2 * a4);
    cnt = reinterpret_cast<int32_t*>(ta->base + 3 * a4);
    tmp = ta->base + 3 * a4 + ac;
  } else if ((e = dev_malloc(&kin, a4)) != hipSuccess || (e = dev_malloc(&kout, a4)) != hipSuccess ||
             (e = dev_malloc(&vin, a4)) != hipSuccess || (e = dev_malloc(&cnt, ac)) != hipSuccess ||
             (e = dev_malloc(&tmp, tmp_bytes)) != hipSuccess) {
    return grid_fail(e, kin, kout, vin, cnt, tmp);
  }
  auto done = [&](hipError_t r) { return ta != nullptr ? r : grid_fail(r, kin, kout, vin, cnt, tmp); };
  {
    Carve cv;
    cv.add(&g->order, (size_t)n);
    cv.add(&g->start, (size_t)total + 1);
    cv.add(&g->pts, (size_t)n);
    if ((e = cv.alloc(&g->block, &g->block_bytes, st)) != hipSuccess) return done(e);
  }
  const unsigned blocks = (unsigned)((n + kGridBlock - 1) / kGridBlock);
  if ((e = hipMemsetAsync(cnt, 0, sizeof(int32_t) * (size_t)(total + 1), st)) != hipSuccess) return done(e);
  cell_id_kernel<<<blocks, kGridBlock, 0, st>>>(xyz32, n, d, kin, vin);
  if ((e = hipGetLastError()) != hipSuccess) return done(e);
  e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, g->order, (int)n, 0, bits, st);
  if (e == hipSuccess) {
    cell_end_kernel<<<blocks, kGridBlock, 0, st>>>(kout, n, cnt);
    e = hipcub::DeviceScan::InclusiveScan(tmp, tmp_bytes, cnt, g->start, hipcub::Max(), (int)(total + 1), st);
  }
  if (e != hipSuccess) return done(e);
  grid_gather_kernel<<<blocks, kGridBlock, 0, st>>>(xyz32, g->order, n, g->pts);
  e = hipGetLastError();
  d.start = g->start;
  d.pts = g->pts;
  // without an arena the temporaries are freed here (hipFree waits for the device)
  return done(e);
}

hipError_t grid_occupancy(Grid* g, TmpArena* ta, hipStream_t st, unsigned long long* pin_dev,
                          const unsigned long long* pin_host) {
  if (g->occ_known) return hipSuccess;
  if (g->n_pts == 0 || g->dev.ncells == 0) {
    g->n_occ = 0;
    g->occ_known = true;
    return hipSuccess;
  }
  unsigned long long* cnt = nullptr;
  uint32_t* part = nullptr;
  hipError_t e = hipSuccess;
  const size_t pbytes = sizeof(uint32_t) * 2 * kOccBlocks;
  if (ta != nullptr) {
    if ((e = ta->reserve(256 + pbytes)) != hipSuccess) return e;
    cnt = reinterpret_cast<unsigned long long*>(ta->base);
    part = reinterpret_cast<uint32_t*>(ta->base + 256);
  } else if ((e = dev_malloc(&cnt, 256 + pbytes)) != hipSuccess) {
    return e;
  } else {
    part = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(cnt) + 256);
  }
  unsigned long long occ[2] = {0, 0};
  const int nb = (int)std::min<int64_t>(kOccBlocks, (g->n_pts + kGridBlock - 1) / kGridBlock);
  count_occupied_pts_kernel<<<(unsigned)nb, kGridBlock, 0, st>>>(g->pts, g->n_pts, g->dev, part);
  occ_final_kernel<<<1, kOccBlocks, 0, st>>>(part, nb, pin_dev != nullptr ? pin_dev : cnt);
  e = hipGetLastError();
  if (e == hipSuccess && pin_dev == nullptr) e = hipMemcpyAsync(occ, cnt, sizeof(occ), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (ta == nullptr) hipFree(cnt);
  if (e != hipSuccess) return e;
  if (pin_dev != nullptr) {
    occ[0] = reinterpret_cast<const volatile unsigned long long*>(pin_host)[0];
    occ[1] = reinterpret_cast<const volatile unsigned long long*>(pin_host)[1];
  }
  g->n_occ = (int64_t)occ[0];
  g->max_occ = (int64_t)occ[1];
  g->occ_known = true;
  return hipSuccess;
}

void grid_free(Grid* g) {
  if (!g) return;
  for (void** p : {reinterpret_cast<void**>(&g->start), reinterpret_cast<void**>(&g->pts),
                   reinterpret_cast<void**>(&g->order), reinterpret_cast<void**>(&g->mpts),
                   reinterpret_cast<void**>(&g->minv)})
    if (in_block(*p, g->block, g->block_bytes)) *p = nullptr;
  block_release(g->block);
  g->block = nullptr;
  g->block_bytes = 0;
  hipFree(g->start);
  hipFree(g->pts);
  hipFree(g->order);
  hipFree(g->mpts);
  hipFree(g->minv);
  g->mpts = nullptr;
  g->minv = nullptr;
  block_release(g->mf16);
  block_release(g->mf32);
  block_release(g->pts64);
  g->pts64 = nullptr;
  g->dev.pts64 = nullptr;
  g->start = nullptr;
  g->pts = nullptr;
  g->order = nullptr;
  g->mf16 = nullptr;
  g->mf32 = nullptr;
  g->mf_npad = 0;
}

// ------------------------------------------------------------------------------- Morton copy
// The ICP loop's source in the Morton (Z-curve) order of its cells (m3d_icp_create): slot k holds
// source point slot[k].  Every per-source array of the loop (keys, runner-ups, correspondences,
// exchange buffers) is indexed by slot, so the grid scan's key writes and seed reads and the terms
// pass's source loads are coalesced and its winner gathers spatially coherent; the ABI translates
// back to source order (m3d_icp_copy_corr).  The Morton key of each point's cell under the grid
// parameters grid_build would choose (the cloud's bounds, cell size; 10 bits per axis, finer grids
// coarsened — only locality matters, any order gives the same keys), one stable radix sort of
// (key, index) from index order, one copy pass.  The copy's grid keeps only what the loop reads of
// a query grid (its Morton points and slot map, grid parameters); its cell arrays are not built
// (ncells = 0, and cell_req = −1 so no cell-size request ever matches it).
__device__ __forceinline__ uint32_t spread3(uint32_t v) {
  v &= 0x3FF;
  v = (v | (v << 16)) & 0x030000FF;
  v = (v | (v << 8)) & 0x0300F00F;
  v = (v | (v << 4)) & 0x030C30C3;
  v = (v | (v << 2)) & 0x09249249;
  return v;
}

__global__ __launch_bounds__(kGridBlock) void morton_key_src_kernel(const float4* __restrict__ pts, int64_t n,
                                                                    GridDev g, int sx, int sy, int sz,
                                                                    uint32_t* __restrict__ key,
                                                                    int32_t* __restrict__ val) {
  const int64_t k = (int64_t)blockIdx.x * kGridBlock + threadIdx.x;
  if (k >= n) return;
  const float4 v = pts[k];
  const uint32_t cx = (uint32_t)grid_coord(v.x, g.o[0], g.inv_h, g.n[0]) >> sx;
  const uint32_t cy = (uint32_t)grid_coord(v.y, g.o[1], g.inv_h, g.n[1]) >> sy;
  const uint32_t cz = (uint32_t)grid_coord(v.z, g.o[2], g.inv_h, g.n[2]) >> sz;
  key[k] = spread3(cx) | (spread3(cy) << 1) | (spread3(cz) << 2);
  val[k] = (int32_t)k;
}

__global__ __launch_bounds__(kGridBlock) void morton_src_copy_kernel(
    const double* __restrict__ xyz64, const double* __restrict__ nrm64, const float4* __restrict__ xyz32,
    const int32_t* __restrict__ perm, int64_t n, double* __restrict__ oxyz64, double* __restrict__ onrm64,
    float4* __restrict__ oxyz32, int32_t* __restrict__ slot, float4* __restrict__ ompts,
    int32_t* __restrict__ ominv) {
  const int64_t k = (int64_t)blockIdx.x * kGridBlock + threadIdx.x;
  if (k >= n) return;
  const int64_t j = perm[k];
  slot[k] = (int32_t)j;
  for (int a = 0; a < 3; ++a) oxyz64[3 * k + a] = xyz64[3 * j + a];
  if (onrm64 != nullptr)
    for (int a = 0; a < 3; ++a) onrm64[3 * k + a] = nrm64[3 * j + a];
  const float4 v = xyz32[j];
  oxyz32[k] = v;
  ompts[k] = make_float4(v.x, v.y, v.z, __int_as_float((int32_t)k));
  ominv[k] = (int32_t)k;
}

hipError_t morton_source(const m3d_cloud* src, double cell, m3d_cloud* out, Grid* gout, TmpArena* ta,
                         hipStream_t st) {
  const int64_t n = src->n;
  out->n = n;
  out->n_pad = src->n_pad;
  for (int k = 0; k < 3; ++k) out->center[k] = src->center[k];
  out->rmax = src->rmax;
  for (int k = 0; k < 3; ++k) {
    out->lo[k] = src->lo[k];
    out->hi[k] = src->hi[k];
  }
  out->has_bounds = src->has_bounds;
  out->s16 = src->s16;
  out->center_given = src->center_given;
  gout->n_pts = n;
  gout->n_occ = 0;
  gout->occ_known = false;
  gout->cell_req = -1.0;
  GridDev d;
  d.ncells = 0;
  float lo[3] = {0.0f, 0.0f, 0.0f}, hi[3] = {0.0f, 0.0f, 0.0f};
  if (src->has_bounds)
    for (int k = 0; k < 3; ++k) {
      lo[k] = src->lo[k];
      hi[k] = src->hi[k];
    }
  gout->cell = grid_params(lo, hi, cell, d);
  gout->dev = d;
  gout->dev.ncells = 0;  // no cell arrays
  gout->dev.start = nullptr;
  gout->dev.pts = nullptr;
  const size_t n1 = (size_t)std::max<int64_t>(n, 1);
  hipError_t e;
  {
    Carve cc, cg;
    cc.add(&out->xyz64, 3 * n1);
    if (src->nrm64 != nullptr) cc.add(&out->nrm64, 3 * n1);
    cc.add(&out->xyz32, (size_t)std::max<int64_t>(src->n_pad, 1));
    cc.add(&out->slot, n1);
    cg.add(&gout->mpts, n1);
    cg.add(&gout->minv, n1);
    if ((e = cc.alloc(&out->block, &out->block_bytes, st)) != hipSuccess ||
        (e = cg.alloc(&gout->block, &gout->block_bytes, st)) != hipSuccess)
      return e;
  }
  if (n == 0) return hipSuccess;
  int sh[3];
  for (int k = 0; k < 3; ++k) {
    sh[k] = 0;
    while ((d.n[k] >> sh[k]) > 1024) ++sh[k];
  }
  uint32_t *kin = nullptr, *kout = nullptr;
  int32_t *vin = nullptr, *vout = nullptr;
  size_t tmp_bytes = 0;
  if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin, vout, (int)n, 0, 30, st)) !=
      hipSuccess)
    return e;
  tmp_bytes = std::max<size_t>(tmp_bytes, 1);
  const size_t a4 = tmp_align(sizeof(uint32_t) * (size_t)n);
  if ((e = ta->reserve(4 * a4 + tmp_align(tmp_bytes))) != hipSuccess) return e;
  kin = reinterpret_cast<uint32_t*>(ta->base);
  kout = reinterpret_cast<uint32_t*>(ta->base + a4);
  vin = reinterpret_cast<int32_t*>(ta->base + 2 * a4);
  vout = reinterpret_cast<int32_t*>(ta->base + 3 * a4);
  void* tmp = ta->base + 4 * a4;
  const unsigned blocks = (unsigned)((n + kGridBlock - 1) / kGridBlock);
  morton_key_src_kernel<<<blocks, kGridBlock, 0, st>>>(src->xyz32, n, d, sh[0], sh[1], sh[2], kin, vin);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, vout, (int)n, 0, 30, st)) !=
      hipSuccess)
    return e;
  morton_src_copy_kernel<<<blocks, kGridBlock, 0, st>>>(src->xyz64, src->nrm64, src->xyz32, vout, n, out->xyz64,
                                                        out->nrm64, out->xyz32, out->slot, gout->mpts, gout->minv);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (src->n_pad > n &&
      (e = hipMemcpyAsync(out->xyz32 + n, src->xyz32 + n, sizeof(float4) * (size_t)(src->n_pad - n),
                          hipMemcpyDeviceToDevice, st)) != hipSuccess)
    return e;
  return hipSuccess;
}

#if M3D_SCAN_CLOCK
}  // namespace m3d
extern "C" int m3d_debug_scan_clock(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(m3d::g_scan_clock), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
namespace m3d {
#endif
hipError_t launch_grid_nn(const float4* src32, int64_t ns, const Grid* qgrid, const Grid* g,
                          int64_t off, const IcpState* s, int64_t* keys, uint32_t* near2,
                          const int32_t* prev, const int64_t* dprev, const float4* tgt32, int64_t nt_shard,
                          hipStream_t st, int64_t q0, int64_t q1, int32_t* hlist, uint32_t* hcnt,
                          int32_t cand_cap, const double* src64, const double* tgt64, int32_t hcap,
                          int32_t xchunk_loop) {
  if (q1 >= 0) ns = q1;
  if (ns <= q0) return hipSuccess;
  if (qgrid == nullptr || qgrid->mpts == nullptr) return hipErrorInvalidValue;  // Morton query order
  // lanes per query by size: 4 while the queries fill about one occupancy round (cfg1: 15.1 µs vs
  // 18.3 at 2), 2 beyond (1M × 125k 71.6 → 60.1 µs, 1M × 1M 117.7 → 112.1 µs: twice the queries in
  // flight per wave); 2 rows × 2 points per lane and load batch
  const int L = (ns - q0) > 300000 ? 2 : 4;
  const int64_t nb = ((ns - q0) * L + kGridBlock - 1) / kGridBlock;
  static const int xchunk_env = [] {
    const char* e = getenv("M3D_SCAN_XCHUNK");
    return e ? std::max(0, atoi(e)) : -1;
  }();
  const int xchunk = xchunk_env >= 0 ? xchunk_env : std::max(0, xchunk_loop);
  const int64_t unit = 8 * (int64_t)std::max(xchunk, 1);
  const unsigned launch = (unsigned)((nb + unit - 1) / unit * unit);
  // deferral of dense-cell and ambiguous queries to grid_nn_heavy_kernel (api.cpp icp_create)
  const bool defer = hlist != nullptr && hcnt != nullptr && cand_cap > 0 && hcap > 0 && g->dev.ncells > 0 &&
                     src64 != nullptr && tgt64 != nullptr;
  const int cap = defer ? cand_cap : 0x7FFFFFFF;
#define M3D_GB(LV, DV)                                                                              \
  grid_nn_batched_kernel<LV, 2, 2, DV><<<launch, kGridBlock, 0, st>>>(qgrid->mpts, ns, g->dev, off, s, keys, \
                                                                     near2, prev, dprev, tgt32, nt_shard, nb, \
                                                                     q0, hlist, hcnt, cap, (uint32_t)hcap, xchunk)
  if (defer) {
    if (L == 4) M3D_GB(4, true); else M3D_GB(2, true);
  } else {
    if (L == 4) M3D_GB(4, false); else M3D_GB(2, false);
  }
#undef M3D_GB
  if (defer) {  // a fixed grid striding over the deferred queries (their count stays on the device)
    const unsigned hb = (unsigned)std::min<int64_t>(512, ns - q0);
    grid_nn_heavy_kernel<<<hb, kGridBlock, 0, st>>>(qgrid->mpts, g->dev, off, s, keys, near2, prev, dprev,
                                                    tgt32, nt_shard, hlist, hcnt, src64, tgt64, ns,
                                                    (uint32_t)hcap);
  }
  return hipGetLastError();
}

}  // namespace m3d
