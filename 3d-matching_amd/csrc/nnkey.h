// nnkey.h — the fp32 query/distance expressions and packed keys shared by every NN kernel
// (icp.hip nn_kernel / nn_mfma_kernel / keyinit, grid.hip grid_nn_kernel), so that all of them
// compute bit-identical (d², index) keys.
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

// (bits(d²) << 32) | index: for d² ≥ +0 the integer order is the lexicographic (d², index) order
__device__ __forceinline__ uint64_t make_key(float d2, uint32_t j) {
  return ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)j;
}

// Starting key of query i (source point p, current fp32 query q) for the lexicographic
// (fp32 d², index) minimum over the targets with d² ≤ r2_hi that every NN kernel computes.
// prev[i] = j is the previous correspondence (the winner of the last evaluation; −1 none):
//  * j in this shard: the candidate (d2f(q, t_j), j) itself — exact, it is one of the targets,
//    so the search only has to look for something smaller;
//  * j in another shard (target-sharded loops, after an update: bound_ok): a bound only, the
//    key (B, 0xFFFFFFFF) with B ≥ d2f(q, t_j).  By the triangle inequality
//    |q − t_j| ≤ |q − q_old| + |q_old − t_j|, q_old = the previous query (Rt32_prev), and
//    keys_prev[i] holds the previous reduced key (d2f(q_old, t_j), j); each fp32 evaluation is
//    within ~5u of its exact value and the 1e-5 factors cover that 20× over.  Every real target
//    beats the pseudo index, so the rank owning t_j still finds it (or better) and the MIN over
//    ranks is unchanged; a rank whose shard holds nothing within B keeps the bound, whose index
//    no shard owns (the terms kernels skip it).  Without the bound those ranks searched with
//    r2_hi: on N ranks, N − 1 of every N queries.
__device__ __forceinline__ int64_t seed_key(const IcpState* __restrict__ s, int64_t i, float4 p,
                                            float qx, float qy, float qz,
                                            const float4* __restrict__ tgt32, int64_t nt_shard,
                                            int64_t off, const int32_t* __restrict__ prev,
                                            const int64_t* __restrict__ keys_prev) {
  if (prev == nullptr) return kKeyNone;
  const int64_t j = (int64_t)prev[i];
  if (j < 0) return kKeyNone;
  if (j >= off && j < off + nt_shard) {
    const float4 t = tgt32[j - off];
    const float d2 = d2f(qx, qy, qz, t.x, t.y, t.z);
    return d2 < s->r2_hi ? (int64_t)make_key(d2, (uint32_t)j) : kKeyNone;
  }
  if (!s->bound_ok || keys_prev == nullptr) return kKeyNone;
  const int64_t kp = keys_prev[i];
  if (kp == kKeyNone || (uint32_t)kp != (uint32_t)j) return kKeyNone;
  const float d2o = __uint_as_float((uint32_t)((uint64_t)kp >> 32));
  float ox, oy, oz;
  xform32(s->Rt32_prev, p, ox, oy, oz);
  const float mx = qx - ox, my = qy - oy, mz = qz - oz;
  const float b = (sqrtf(d2o) + sqrtf(fmaf(mz, mz, fmaf(my, my, mx * mx)))) * 1.00001f;
  const float B = b * b * 1.00001f;
  return B < s->r2_hi ? (int64_t)make_key(B, 0xFFFFFFFFu) : kKeyNone;
}

}  // namespace m3d
