// nnkey.h — the fp32 query/distance expressions, packed keys and the fp64 resolution shared by
// every NN kernel (icp.hip nn_mfma_kernel / nn_kernel / keyinit / terms, grid.hip grid_nn_kernel).
//
// Result contract (Open3D KDTreeFlann::SearchHybrid(p, r, 1) in fp64): for each
// source point the lexicographic (d64, index) minimum over the targets with d64 < r², where
//   Q   = T·p in fp64 in Eigen's (non-FMA) order: ((T00·px + T01·py) + T02·pz) + T03  (q64_of)
//   d64 = ((dx·dx + dy·dy) + dz·dz), d = Q − t in fp64                                 (d2_64)
// (oracle/icp_oracle.py uses the same expressions in numpy).  The kernels search in fp32 on
// centred coordinates: d2f = the fp32 d² of the fp32 query and target.  Two values per query
// come out of the scan: the key k1 = the lexicographic (d2f, index) minimum, and near2 = the
// smallest d2f of any OTHER target the scan evaluated (+inf none).  The fp64 winner can differ
// from k1 only if some other target lies inside the error band of k1 (band_of), which the scan
// always evaluates, so
//   near2 ≤ band_of(d2f(k1))  ⇔  "ambiguous": re-evaluate in fp64 (resolve_wave)
//   otherwise                     the winner is k1's target (if its d64 < r²).
// Error bound (refresh_rt32): |√d2f − |Q − t|| ≤ e_q + 3u·√d2f, e_q = √3·E with E a
// per-coordinate bound on the fp32 query/target rounding plus the fp64 evaluation of Q.  If
// d64(c) ≤ d64(w) then √d2f(c) ≤ (√d2f(w)(1 + 3u) + e_q)(1 + 5ε) + e_q)(1 + 3u), which
// band_of(d2f(w)) over-covers (×(1 + 4e-6) on the root and on the square, 2·e_q·1.01 absolute).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "m3d_internal.h"

namespace m3d {

__device__ __forceinline__ float d2f(float qx, float qy, float qz, float tx, float ty, float tz) {
  const float dx = qx - tx, dy = qy - ty, dz = qz - tz;
  return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

// centred source point → centred fp32 query under the search transform Rt (R row-major, t')
__device__ __forceinline__ void xform32(const float* Rt, float4 p, float& x, float& y, float& z) {
  x = fmaf(Rt[0], p.x, fmaf(Rt[1], p.y, fmaf(Rt[2], p.z, Rt[9])));
  y = fmaf(Rt[3], p.x, fmaf(Rt[4], p.y, fmaf(Rt[5], p.z, Rt[10])));
  z = fmaf(Rt[6], p.x, fmaf(Rt[7], p.y, fmaf(Rt[8], p.z, Rt[11])));
}

// the fp64 query of the contract (Open3D PointCloud::Transform, Eigen non-FMA order; the
// library is built with -ffp-contract=off, so these products and sums are not fused)
__device__ __forceinline__ void q64_of(const double* __restrict__ T, const double* __restrict__ p,
                                       double q[3]) {
  q[0] = ((T[0] * p[0] + T[1] * p[1]) + T[2] * p[2]) + T[3];
  q[1] = ((T[4] * p[0] + T[5] * p[1]) + T[6] * p[2]) + T[7];
  q[2] = ((T[8] * p[0] + T[9] * p[1]) + T[10] * p[2]) + T[11];
}

__device__ __forceinline__ double d2_64(const double q[3], const double* __restrict__ t) {
  const double dx = q[0] - t[0], dy = q[1] - t[1], dz = q[2] - t[2];
  return (dx * dx + dy * dy) + dz * dz;
}

// (bits(d²) << 32) | index: for d² ≥ +0 the integer order is the lexicographic (d², index) order
__device__ __forceinline__ uint64_t make_key(float d2, uint32_t j) {
  return ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)j;
}
__device__ __forceinline__ float key_d2(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }
// a key naming a target (not kKeyNone, not a radius or distance-bound pseudo key)
__device__ __forceinline__ bool key_real(uint64_t k) { return (uint32_t)k != 0xFFFFFFFFu; }

// The fp32 band around a best d2f inside which another target may still win in fp64.
__device__ __forceinline__ float band_of(float d2, float be) {
  const float s = fmaf(sqrtf(d2), 1.000004f, be);
  return s * s * 1.000004f;
}
// the fp32 search bound a query with current best `d2` screens against
__device__ __forceinline__ float search_bound(float d2, float be, float r2_hi) {
  return d2 < 0.0f ? d2 : fminf(band_of(d2, be), r2_hi);
}

constexpr float kInf = __builtin_huge_valf();
constexpr uint32_t kNearNone = 0x7F800000u;  // bits of +inf: "no other target evaluated"

// d2f of a key that names a target, +inf for kKeyNone and pseudo keys
__device__ __forceinline__ float key_real_d2(uint64_t k) { return key_real(k) ? key_d2(k) : kInf; }

// Scan state of one query: k1 (lexicographic (d2f, index) minimum), k1d = key_real_d2(k1), and
// near2 = min d2f over the evaluated targets other than k1's.  Push a candidate target key kc
// with d2f d2c (a real target; kc == k1 only when the seed's target is met again).  Branch-free.
__device__ __forceinline__ void near_push(uint64_t& k1, float& k1d, float& near2, uint64_t kc,
                                          float d2c) {
  const bool lt = kc < k1;
  const float dd = lt ? k1d : (kc == k1 ? kInf : d2c);  // the value not kept as k1
  k1 = lt ? kc : k1;
  k1d = lt ? d2c : k1d;
  near2 = fminf(near2, dd);
}
// push target idx at d2f d2 if d2 ≤ r2_hi, branch-free (else a key above every scan key — k1 is at
// most (r2_hi, 0xFFFFFFFF) — and +inf: no change), so the point's index is read with its
// coordinates in one 16-B load instead of by a second dependent load under the branch
__device__ __forceinline__ void push_within(uint64_t& k1, float& k1d, float& near2, float d2, float r2_hi,
                                            uint32_t idx) {
  const bool ok = d2 <= r2_hi;
  near_push(k1, k1d, near2, ok ? make_key(d2, idx) : ~0ull, ok ? d2 : kInf);
}
// merge another state (b1, bn2) of the same query into (k1, k1d, near2)
__device__ __forceinline__ void near_merge(uint64_t& k1, float& k1d, float& near2, uint64_t b1,
                                           float bn2) {
  near_push(k1, k1d, near2, b1, key_real_d2(b1));
  near2 = fminf(near2, bn2);
}
// Publish a block's (k1, near2) into the global (keys, near2g) such that, after every block has
// published, keys = the minimum of all published keys and near2g = the minimum d2f of the
// published real keys other than it and of the published near2: the key an atomicMin on keys
// rejects or displaces goes to near2g.  publish_k1 = false: k1 is already in keys (an unchanged
// seed).  near2g holds float bits (d2f ≥ +0: the unsigned order is the float order).
__device__ __forceinline__ void near_publish(unsigned long long* keys, unsigned int* near2g,
                                             uint64_t k1, float near2, bool publish_k1) {
  float n2 = near2;
  if (publish_k1) {
    const uint64_t old = atomicMin(keys, (unsigned long long)k1);
    if (old != k1) n2 = fminf(n2, key_real_d2(old > k1 ? old : k1));
  }
  if (n2 < kInf) atomicMin(near2g, __float_as_uint(n2));
}

__device__ __forceinline__ int grid_coord(float x, float o, float inv_h, int n) {
  float f = (x - o) * inv_h;
  f = fminf(fmaxf(f, 0.0f), (float)(n - 1));
  return (int)f;
}

// whether [x − R, x + R] misses every target of an n-cell axis, by grid_coord's unclamped
// coordinates (same expressions) of its two ends: below 0 (every target has x − o ≥ 0, exactly),
// or at / past n + 1 (a target's coordinate is < n up to the fp32 rounding of (x − o)·inv_h, which
// can reach n only for a point within ~1e-7 of the top edge: one cell of margin)
__device__ __forceinline__ bool grid_miss(float x, float R, float o, float inv_h, int n) {
  return ((x + R) - o) * inv_h < 0.0f || ((x - R) - o) * inv_h >= (float)(n + 1);
}

__device__ __forceinline__ bool grid_box_miss(const GridDev& g, float qx, float qy, float qz, float R) {
  return grid_miss(qx, R, g.o[0], g.inv_h, g.n[0]) || grid_miss(qy, R, g.o[1], g.inv_h, g.n[1]) ||
         grid_miss(qz, R, g.o[2], g.inv_h, g.n[2]);
}

#ifndef M3D_SCAN_FLATLOAD
#define M3D_SCAN_FLATLOAD 1
#endif
// The start / end offsets of rows r0 .. r0 + kR − 1 of a query's box (rows past `rows`: a = b = 0).
// Every load is unconditional (a row past the box reads row r0's starts, dropped by the select):
// loads under a per-lane branch compile to load → s_waitcnt vmcnt(0) → copy, one round trip each;
// straight-line loads go out together and are waited for once.  The point loads below likewise
// read slot 0 for a lane past its row's end.
template <int kR>
__device__ __forceinline__ void scan_row_starts(const GridDev& g, int r0, int rows, int ny, int x0, int x1,
                                                int y0, int z0, int32_t* a, int32_t* b) {
#pragma unroll
  for (int k = 0; k < kR; ++k) {
    const int r = r0 + k;
    if (M3D_SCAN_FLATLOAD) {
      const int rr = r < rows ? r : r0;  // r0 < rows
      const int64_t row = ((int64_t)(z0 + rr / ny) * g.n[1] + (y0 + rr % ny)) * g.n[0];
      const int32_t sa = g.start[row + x0], sb = g.start[row + x1 + 1];
      a[k] = r < rows ? sa : 0;
      b[k] = r < rows ? sb : 0;
    } else {
      a[k] = b[k] = 0;
      if (r < rows) {
        const int64_t row = ((int64_t)(z0 + r / ny) * g.n[1] + (y0 + r % ny)) * g.n[0];
        a[k] = g.start[row + x0];
        b[k] = g.start[row + x1 + 1];
      }
    }
  }
}

// Grid scan of one query by kL cooperating lanes (grid.hip grid_nn_batched_kernel): every lane
// of the query sees every cell row of the box q ± R and takes the row's points sub, sub + kL, …;
// the start offsets of kR rows are loaded together, then kR × kB point loads per lane go out at
// once.  Each lane pushes the targets with d2f ≤ r2_hi into its (k1, k1d, near2) state;
// grid_merge_lanes combines the kL states.  A query whose rows hold more than cand_cap points
// stops at the batch that crosses it (*ncand > cand_cap: the caller defers it, see
// grid.hip grid_nn_heavy_kernel).
template <int kL, int kR, int kB>
__device__ __forceinline__ void grid_scan(const GridDev& g, float qx, float qy, float qz, float R,
                                          float r2_hi, int64_t off, int sub, uint64_t& k1,
                                          float& k1d, float& n2, int* nrows = nullptr,
                                          int* ncand = nullptr, int cand_cap = 0x7FFFFFFF) {
  const int x0 = grid_coord(qx - R, g.o[0], g.inv_h, g.n[0]);
  const int x1 = grid_coord(qx + R, g.o[0], g.inv_h, g.n[0]);
  const int y0 = grid_coord(qy - R, g.o[1], g.inv_h, g.n[1]);
  const int y1 = grid_coord(qy + R, g.o[1], g.inv_h, g.n[1]);
  const int z0 = grid_coord(qz - R, g.o[2], g.inv_h, g.n[2]);
  const int z1 = grid_coord(qz + R, g.o[2], g.inv_h, g.n[2]);
  const int ny = y1 - y0 + 1;
  // a box that misses the grid on some axis (the unclamped cell range lies wholly below cell 0 or
  // at / past cell n) holds none of its cells: the clamped range would scan an edge column of
  // targets outside the box.  A spatial target shard (m3d.dist.spatial_shards) sees most queries
  // leave here.
  const int rows = grid_box_miss(g, qx, qy, qz, R) ? 0 : ny * (z1 - z0 + 1);
  if (nrows != nullptr) *nrows = rows;
  int cand = 0;
  for (int r0 = 0; r0 < rows; r0 += kR) {
    int32_t a[kR], b[kR];
    int32_t len = 0;
    scan_row_starts<kR>(g, r0, rows, ny, x0, x1, y0, z0, a, b);
#pragma unroll
    for (int k = 0; k < kR; ++k) {
      len = max(len, b[k] - a[k]);
      cand += b[k] - a[k];
    }
    if (cand > cand_cap) break;  // deferred (same rows on every lane of the query)
    for (int32_t base = sub; base < len; base += kL * kB) {
      float4 v[kR][kB];
#pragma unroll
      for (int k = 0; k < kR; ++k)
#pragma unroll
        for (int m = 0; m < kB; ++m) {
          const int32_t j = a[k] + base + m * kL;
          if (M3D_SCAN_FLATLOAD)
            v[k][m] = g.pts[j < b[k] ? j : 0];
          else if (j < b[k])
            v[k][m] = g.pts[j];
        }
#pragma unroll
      for (int k = 0; k < kR; ++k)
#pragma unroll
        for (int m = 0; m < kB; ++m) {
          const int32_t j = a[k] + base + m * kL;
          if (j < b[k]) {
            const float d2 = d2f(qx, qy, qz, v[k][m].x, v[k][m].y, v[k][m].z);
            push_within(k1, k1d, n2, d2, r2_hi, (uint32_t)(off + __float_as_int(v[k][m].w)));
          }
        }
    }
  }
  if (ncand != nullptr) *ncand = cand;
}

#ifndef M3D_MERGE_DPP
#define M3D_MERGE_DPP 1
#endif
#ifndef M3D_DPP_X4
#define M3D_DPP_X4 1
#endif
// v from lane ^ 4 by two DPP moves: lane ^ 3 (quad permute [3,2,1,0]), then lane ^ 7 (the mirror
// inside each 8 lanes, row_half_mirror): (i ^ 7) ^ 3 = i ^ 4
__device__ __forceinline__ int xor4_dpp(int v) {
  return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(v, 0x1B, 0xF, 0xF, false), 0x141, 0xF, 0xF, false);
}
// v from lane ^ o: DPP for o = 1, 2 (quad permutes), 4 (two moves) and 8 (row_ror:8), with no
// LDS round trip; a shuffle otherwise
__device__ __forceinline__ int xor_lane(int v, int o, int width) {
  if (M3D_MERGE_DPP && o == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  if (M3D_MERGE_DPP && o == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  if (M3D_MERGE_DPP && M3D_DPP_X4 && o == 4) return xor4_dpp(v);
  if (M3D_MERGE_DPP && o == 8) return __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return __shfl_xor(v, o, width);
}
__device__ __forceinline__ double xor_lane_f64(double v, int o) {
  const long long b = __double_as_longlong(v);
  const int lo = xor_lane((int)(uint32_t)b, o, kWave), hi = xor_lane((int)(uint32_t)(b >> 32), o, kWave);
  return __longlong_as_double(((long long)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t xor_lane_i64(int64_t v, int o) {
  const int lo = xor_lane((int)(uint32_t)v, o, kWave), hi = xor_lane((int)(uint32_t)((uint64_t)v >> 32), o, kWave);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int kL>
__device__ __forceinline__ void grid_merge_lanes(uint64_t& k1, float& k1d, float& n2) {
#pragma unroll
  for (int o = kL / 2; o > 0; o >>= 1) {
    const uint64_t b1 = ((uint64_t)(uint32_t)xor_lane((int)(k1 >> 32), o, kL) << 32) |
                        (uint32_t)xor_lane((int)(uint32_t)k1, o, kL);
    const float bn2 = __int_as_float(xor_lane(__float_as_int(n2), o, kL));
    near_merge(k1, k1d, n2, b1, bn2);
  }
}

// Exact fp64 decision for the ambiguous queries of a wave (every lane of the wave calls it, with
// amb set on the lanes whose query needs it).  For each such query the whole wave scans the
// cell box of q ± 1.001·√X (grid.hip header lemma: it holds every target with d2f ≤ X), lanes
// split over the box's (y, z) rows and the points of a row; every target with d2f(q, t) ≤ X is
// re-evaluated with the contract's fp64 d² from its fp64 coordinates, and a butterfly takes the
// lexicographic (d64, global index) minimum among d64 < r2 (bj = −1: none).  With the grid's fp64
// points (g.pts64, the ICP loops' target grid) every target of the box is evaluated from one
// 32-B load — a superset holding the same minimum — instead of an fp32 screen and a gather.
#ifndef M3D_WALK_PAIRS
#define M3D_WALK_PAIRS 1
#endif
template <int kP, typename T>
__device__ __forceinline__ T item_of(const T (&v)[kP], int u) {  // v[u] for a wave-uniform u
  T r = v[0];
#pragma unroll
  for (int k = 1; k < kP; ++k)
    if (u == k) r = v[k];
  return r;
}
template <int kP>
__device__ __forceinline__ double item_q(const double (&Q)[kP][3], int u, int c) {
  double r = Q[0][c];
#pragma unroll
  for (int k = 1; k < kP; ++k)
    if (u == k) r = Q[k][c];
  return r;
}
// resolve_wave over kP queries per lane (the terms pass's sources per thread): the ambiguous
// (u, lane) items of all kP rounds are walked two at a time, one per half-wave (M3D_WALK_PAIRS),
// so a wave holding two walks them side by side instead of one after the other — its block waits
// for it.  Any box lane split gives the same minimum.
template <int kP>
__device__ __forceinline__ void resolve_wave_kp(const bool (&amb)[kP], const GridDev& g,
                                                const double* __restrict__ tgt64, int64_t off,
                                                const float (&qx)[kP], const float (&qy)[kP],
                                                const float (&qz)[kP], const float (&X)[kP],
                                                const double (&Q)[kP][3], double r2,
                                                int64_t (&bj)[kP], double (&bd)[kP]) {
  const int lane = threadIdx.x & (kWave - 1);
  uint64_t m[kP];
#pragma unroll
  for (int u = 0; u < kP; ++u) m[u] = __ballot(amb[u]);
  auto next = [&](int& u, int& L) {  // the next (u, lane) item, u = −1: none
    u = -1;
    L = 0;
#pragma unroll
    for (int k = 0; k < kP; ++k)
      if (u < 0 && m[k] != 0) {
        u = k;
        L = __builtin_ctzll(m[k]);
        m[k] &= m[k] - 1;
      }
  };
  for (;;) {
    int uA, LA, uB = -1, LB = 0;
    next(uA, LA);
    if (uA < 0) break;
    if (M3D_WALK_PAIRS) next(uB, LB);
    const bool two = uB >= 0;
    const int W = two ? kWave / 2 : kWave;  // lanes per query (wave-uniform)
    const int sl = lane & (W - 1);           // this lane's place among them
    const bool hb = two && lane >= kWave / 2;
    float lx = __shfl(item_of(qx, uA), LA), ly = __shfl(item_of(qy, uA), LA);
    float lz = __shfl(item_of(qz, uA), LA), lX = __shfl(item_of(X, uA), LA);
    double Q0 = __shfl(item_q(Q, uA, 0), LA), Q1 = __shfl(item_q(Q, uA, 1), LA);
    double Q2 = __shfl(item_q(Q, uA, 2), LA);
    if (two) {
      const float bx = __shfl(item_of(qx, uB), LB), by = __shfl(item_of(qy, uB), LB);
      const float bz = __shfl(item_of(qz, uB), LB), bX = __shfl(item_of(X, uB), LB);
      const double b0 = __shfl(item_q(Q, uB, 0), LB), b1 = __shfl(item_q(Q, uB, 1), LB);
      const double b2 = __shfl(item_q(Q, uB, 2), LB);
      if (hb) {
        lx = bx;
        ly = by;
        lz = bz;
        lX = bX;
        Q0 = b0;
        Q1 = b1;
        Q2 = b2;
      }
    }
    double dl = kInf;
    int64_t jl = INT64_MAX;
    if (g.ncells > 0 && lX >= 0.0f) {
      const float R = sqrtf(lX) * 1.001f;
      const int x0 = grid_coord(lx - R, g.o[0], g.inv_h, g.n[0]);
      const int x1 = grid_coord(lx + R, g.o[0], g.inv_h, g.n[0]);
      const int y0 = grid_coord(ly - R, g.o[1], g.inv_h, g.n[1]);
      const int y1 = grid_coord(ly + R, g.o[1], g.inv_h, g.n[1]);
      const int z0 = grid_coord(lz - R, g.o[2], g.inv_h, g.n[2]);
      const int z1 = grid_coord(lz + R, g.o[2], g.inv_h, g.n[2]);
      const int ny = y1 - y0 + 1;
      const int rows = ny * (z1 - z0 + 1);
      const int lpr = rows >= W ? 1 : W / rows;  // lanes per row
      const int rstep = W / lpr;
      for (int r = sl / lpr; r < rows; r += rstep) {
        const int cz = z0 + r / ny, cy = y0 + r % ny;
        const int64_t row = ((int64_t)cz * g.n[1] + cy) * g.n[0];
        const int32_t j1 = g.start[row + x1 + 1];
        if (g.pts64 != nullptr) {
          // every target of the box in fp64 (a superset of those with d2f ≤ X: the same
          // minimum), coordinates and index in one load
          for (int32_t j = g.start[row + x0] + sl % lpr; j < j1; j += lpr) {
            const double4 v = g.pts64[j];
            const double dx = Q0 - v.x, dy = Q1 - v.y, dz = Q2 - v.z;
            const double d = (dx * dx + dy * dy) + dz * dz;
            const int64_t gj = off + (int64_t)__double_as_longlong(v.w);
            if (d < r2 && (d < dl || (d == dl && gj < jl))) {
              dl = d;
              jl = gj;
            }
          }
          continue;
        }
        for (int32_t j = g.start[row + x0] + sl % lpr; j < j1; j += lpr) {
          const float4 v = g.pts[j];
          if (!(d2f(lx, ly, lz, v.x, v.y, v.z) <= lX)) continue;
          const int64_t lj = (int64_t)__float_as_int(v.w);
          const double* t = tgt64 + 3 * lj;
          const double dx = Q0 - t[0], dy = Q1 - t[1], dz = Q2 - t[2];
          const double d = (dx * dx + dy * dy) + dz * dz;
          const int64_t gj = off + lj;
          if (d < r2 && (d < dl || (d == dl && gj < jl))) {
            dl = d;
            jl = gj;
          }
        }
      }
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      if (o >= W) continue;  // two queries: the butterfly stays inside each half
      const double od = xor_lane_f64(dl, o);
      const int64_t oj = xor_lane_i64(jl, o);
      if (od < dl || (od == dl && oj < jl)) {
        dl = od;
        jl = oj;
      }
    }
    // the lower half (lane 0) holds item A's result, the upper half (lane 32) item B's
    const double dA = __shfl(dl, 0);
    const int64_t jA = __shfl(jl, 0);
    const double dB = __shfl(dl, kWave / 2);
    const int64_t jB = __shfl(jl, kWave / 2);
#pragma unroll
    for (int k = 0; k < kP; ++k) {
      if (uA == k && lane == LA) {
        bj[k] = jA == INT64_MAX ? -1 : jA;
        bd[k] = dA;
      }
      if (two && uB == k && lane == LB) {
        bj[k] = jB == INT64_MAX ? -1 : jB;
        bd[k] = dB;
      }
    }
  }
}

__device__ __forceinline__ void resolve_wave(bool amb, const GridDev& g,
                                             const double* __restrict__ tgt64, int64_t off,
                                             float qx, float qy, float qz, float X,
                                             const double Q[3], double r2, int64_t& bj,
                                             double& bd) {
  const bool a1[1] = {amb};
  const float x1[1] = {qx}, y1[1] = {qy}, z1[1] = {qz}, X1[1] = {X};
  const double Q1[1][3] = {{Q[0], Q[1], Q[2]}};
  int64_t b1[1] = {bj};
  double d1[1] = {bd};
  resolve_wave_kp<1>(a1, g, tgt64, off, x1, y1, z1, X1, Q1, r2, b1, d1);
  bj = b1[0];
  bd = d1[0];
}

// The fp64 winner of query i from its scan results (k1, near2) — see the header.  Q = its fp64
// query, p32 its centred fp32 source point.  Called by every lane of the wave (valid = the lane
// has a query).
__device__ __forceinline__ void winner_fp64(bool valid, uint64_t k1, float near2,
                                            const IcpState* __restrict__ s, const GridDev& g,
                                            const double* __restrict__ tgt64, int64_t off,
                                            int64_t nt_shard, const float4& p32, const double Q[3],
                                            int64_t& bj, double& bd) {
  bj = -1;
  bd = 0.0;
  const float X = valid && k1 != (uint64_t)kKeyNone ? search_bound(key_d2(k1), s->band_e, s->r2_hi)
                                                    : -1.0f;
  const bool amb = X >= 0.0f && near2 <= X;
  float qx = 0.0f, qy = 0.0f, qz = 0.0f;
  if (amb) xform32(s->Rt32, p32, qx, qy, qz);
  resolve_wave(amb, g, tgt64, off, qx, qy, qz, X, Q, s->r2, bj, bd);
  if (amb || !valid || !key_real(k1)) return;
  const int64_t gj = (int64_t)(uint32_t)k1;
  if (gj < off || gj >= off + nt_shard) return;
  const double d = d2_64(Q, tgt64 + 3 * (gj - off));
  if (d < s->r2) {
    bj = gj;
    bd = d;
  }
}

// Distance-bound pseudo key for a query whose previous winner lies in another shard: d64o ≥ the
// previous global winner's fp64 d² (rounded up to fp32); see seed_key.
__device__ __forceinline__ int64_t bound_key(const IcpState* __restrict__ s, float d64o, float4 p,
                                             float qx, float qy, float qz) {
  float ox, oy, oz;
  xform32(s->Rt32_prev, p, ox, oy, oz);
  const float mx = qx - ox, my = qy - oy, mz = qz - oz;
  const float b = (sqrtf(d64o) * 1.000001f + s->eq_prev + sqrtf(fmaf(mz, mz, fmaf(my, my, mx * mx))) * 1.000001f) *
                  1.00001f;
  const float B = b * b * 1.00001f;
  return B < s->r2_hi ? (int64_t)make_key(B, 0xFFFFFFFFu) : kKeyNone;
}

// Starting key of query i (source point p, current fp32 query q) for the scan.
// prev[i] = j is the previous correspondence (the fp64 winner of the last evaluation; −1 none):
//  * j in this shard: the candidate (d2f(q, t_j), j) itself — one of the targets, so the search
//    only has to look for something smaller (or inside its band);
//  * j in another shard (target-sharded loops, after an update: bound_ok): a bound only, the
//    pseudo key (B, 0xFFFFFFFF) with B ≥ d2f(q, t_j).  dprev[i] holds the bits of the previous
//    global fp64 winner's d64 = |Q_old − t_j|² (±ε); the fp32 distance of the old fp32 query is
//    ≤ √d64 + e_q_prev, and by the triangle inequality |q − t_j| ≤ |q − q_old| + |q_old − t_j|
//    (q_old from Rt32_prev).  A local target c that could beat t_j in fp64 has d2f(c) ≤
//    band_of(B), which is the bound the scan screens with (search_bound), so the rank owning
//    the new winner still finds it, and the MIN over ranks is unchanged.  Without the bound those
//    ranks searched with r2_hi: on N ranks, N − 1 of every N queries.
// (j = prev[i], loaded by the caller: the grid scan issues it beside the query's point load)
__device__ __forceinline__ int64_t seed_key_j(const IcpState* __restrict__ s, int64_t j, int64_t i, float4 p,
                                              float qx, float qy, float qz,
                                              const float4* __restrict__ tgt32, int64_t nt_shard,
                                              int64_t off, const int64_t* __restrict__ dprev) {
  if (j < 0) return kKeyNone;
  if (j >= off && j < off + nt_shard) {
    const float4 t = tgt32[j - off];
    const float d2 = d2f(qx, qy, qz, t.x, t.y, t.z);
    return d2 <= s->r2_hi ? (int64_t)make_key(d2, (uint32_t)j) : kKeyNone;
  }
  if (!s->bound_ok || dprev == nullptr) return kKeyNone;
  const int64_t dp = dprev[i];
  if (dp == kKeyNone) return kKeyNone;
  return bound_key(s, __double2float_ru(__longlong_as_double(dp)), p, qx, qy, qz);
}

__device__ __forceinline__ int64_t seed_key(const IcpState* __restrict__ s, int64_t i, float4 p,
                                            float qx, float qy, float qz,
                                            const float4* __restrict__ tgt32, int64_t nt_shard,
                                            int64_t off, const int32_t* __restrict__ prev,
                                            const int64_t* __restrict__ dprev) {
  if (prev == nullptr) return kKeyNone;
  return seed_key_j(s, (int64_t)prev[i], i, p, qx, qy, qz, tgt32, nt_shard, off, dprev);
}

}  // namespace m3d
