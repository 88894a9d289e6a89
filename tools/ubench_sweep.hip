// Microbenchmark: the NN screen's sweep step (one v_mfma_f32_32x32x16_f16 + a 16-value minimum
// tree + one threshold test per step) with every operand in registers — no LDS, no global
// traffic, no barriers — to separate the step's own issue ceiling from the memory structure
// around it in nn_mfma_kernel.  Variants:
//   mfma      MFMAs only (results folded once per tile so they are not dead)
//   valu      the minimum tree + test on register data, no MFMA
//   sweep     MFMA + v_minimum3 tree + test (nn_mfma_kernel's step, pipelined one step ahead)
//   sweep_min v_min3_f32 tree (fminf semantics) instead of v_minimum3
//   sweep_nb  sweep without the sched_barrier fences
//   sweep_or  sign test: OR of the 16 bit patterns by full-rate v_bitop3_b32 (nn_mfma_kernel)
//   sweep_or_nb  the same without fences
//   mix       waves 4-7 of a block MFMA-only, waves 0-3 the sign-OR tree only (same SIMDs):
//             do the two pipes overlap across waves of one SIMD?
//   valu_or   the sign-OR tree only, every wave
//   sweep_or_prio  sweep_or with s_setprio 1 around each MFMA issue
//   sweep_c   threshold folded into the accumulator (C = −thr): tree over 2 groups at once,
//             one test per two MFMAs
// 512-thread blocks, 2048 blocks (≈2 blocks/CU at ≤128 VGPRs).  Prints ms per launch, the
// shader clock measured with s_memtime against s_memrealtime (100 MHz), and cycles per MFMA per
// SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_sweep tools/ubench_sweep.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kTiles = 64;   // loop iterations (tiles) per wave
constexpr int kSub = 8;      // sub-tiles per tile
constexpr int kG = 2;        // query groups per wave

__device__ __forceinline__ float vmin3(float a, float b, float c) {
  return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ float fmin3(float a, float b, float c) { return fminf(fminf(a, b), c); }

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

template <int kV>
__device__ __forceinline__ float tree(const floatx16& k) {
  if (kV == 1) {
    const float m0 = fmin3(k[0], k[1], k[2]), m1 = fmin3(k[3], k[4], k[5]);
    const float m2 = fmin3(k[6], k[7], k[8]), m3 = fmin3(k[9], k[10], k[11]);
    const float m4 = fmin3(k[12], k[13], k[14]);
    return fminf(fmin3(m0, m1, m2), fmin3(m3, m4, k[15]));
  }
  const float m0 = vmin3(k[0], k[1], k[2]), m1 = vmin3(k[3], k[4], k[5]);
  const float m2 = vmin3(k[6], k[7], k[8]), m3 = vmin3(k[9], k[10], k[11]);
  const float m4 = vmin3(k[12], k[13], k[14]);
  return __builtin_elementwise_minimum(vmin3(m0, m1, m2), vmin3(m3, m4, k[15]));
}

// kV: 0 sweep (minimum3), 1 sweep_min (min3), 2 mfma only, 3 valu only, 4 sweep_c,
// 5 sweep without the scheduling fences (compiler's own order), 6 sign-OR tree (v_bitop3, the
// threshold folded into the MFMA), 7 the same without fences
template <int kV>
__global__ __launch_bounds__(512) void sweep(const uint4* __restrict__ in, float thr0,
                                             uint32_t* __restrict__ out, uint64_t* __restrict__ clk) {
  const int lane = threadIdx.x & 63;
  union U { uint4 u; half8 h; };
  U av[kSub], bq[kG];
  for (int s = 0; s < kSub; ++s) av[s].u = in[(s * 64 + lane) & 1023];
  for (int g = 0; g < kG; ++g) bq[g].u = in[(512 + g * 64 + lane) & 1023];
  float thr[kG];
  floatx16 cacc[kG];
  for (int g = 0; g < kG; ++g) {
    thr[g] = thr0 + 0.001f * g;
    for (int r = 0; r < 16; ++r) cacc[g][r] = -thr[g];
  }
  const floatx16 zacc = {};
  floatx16 vdat = {};
  for (int r = 0; r < 16; ++r) vdat[r] = (float)(lane * 16 + r);
  uint32_t hm_all = 0;
  float fold = 0.0f;
  uint64_t t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < kTiles; ++it) {
    for (int s = 0; s < kSub; ++s) asm volatile("" : "+v"(av[s].u.x), "+v"(av[s].u.y), "+v"(av[s].u.z), "+v"(av[s].u.w));
    uint32_t hm = 0;
    constexpr int kSteps = kSub * kG;
    if (kV == 8 || kV == 10) {
      const bool mfma_wave = kV == 8 && ((threadIdx.x >> 6) & 4) != 0;
      if (mfma_wave) {
        floatx16 a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[0].h, bq[0].h, zacc, 0, 0, 0);
#pragma unroll
        for (int t = 1; t < kSteps; ++t)
          a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[t / kG].h, bq[t % kG].h, a0, 0, 0, 0);
        fold += a0[lane & 15];
      } else {
#pragma unroll
        for (int t = 0; t < kSteps; ++t) {
          asm volatile("" : "+v"(vdat[0]), "+v"(vdat[5]), "+v"(vdat[10]), "+v"(vdat[15]));
          if (__any((int32_t)or16(vdat) < 0)) hm |= 1u << t;
        }
      }
    } else if (kV == 3) {
#pragma unroll
      for (int t = 0; t < kSteps; ++t) {
        asm volatile("" : "+v"(vdat[0]), "+v"(vdat[5]), "+v"(vdat[10]), "+v"(vdat[15]));
        const float m = tree<0>(vdat);
        if (__any(m <= thr[t % kG])) hm |= 1u << t;
      }
    } else if (kV == 2) {
      floatx16 a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[0].h, bq[0].h, zacc, 0, 0, 0);
#pragma unroll
      for (int t = 1; t < kSteps; ++t)
        a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[t / kG].h, bq[t % kG].h, a0, 0, 0, 0);
      fold += a0[lane & 15];
    } else if (kV == 4) {
      // C = −thr per group: both groups' values compare against 0, one tree over 32 values
#pragma unroll
      for (int s = 0; s < kSub; ++s) {
        const floatx16 k0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s].h, bq[0].h, cacc[0], 0, 0, 0);
        const floatx16 k1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s].h, bq[1].h, cacc[1], 0, 0, 0);
        const float m = __builtin_elementwise_minimum(tree<0>(k0), tree<0>(k1));
        if (__any(m <= 0.0f)) hm |= 1u << s;
      }
    } else {
      floatx16 kc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[0].h, bq[0].h, zacc, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < kSteps; ++t) {
        floatx16 kn;
        if (kV == 9) __builtin_amdgcn_s_setprio(1);
        if (t + 1 < kSteps)
          kn = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[(t + 1) / kG].h, bq[(t + 1) % kG].h, zacc, 0, 0, 0);
        if (kV == 9) __builtin_amdgcn_s_setprio(0);
        if (kV != 5 && kV != 7) __builtin_amdgcn_sched_barrier(0);
        if (kV >= 6 && kV != 8) {
          if (__any((int32_t)or16(kc) < 0)) hm |= 1u << t;
        } else {
          const float m = tree<kV == 1 ? 1 : 0>(kc);
          if (__any(m <= thr[t % kG])) hm |= 1u << t;
        }
        if (kV != 5 && kV != 7) __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < kSteps) kc = kn;
      }
    }
    hm_all ^= hm + it;
  }
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  out[blockIdx.x * 512 + threadIdx.x] = hm_all + (uint32_t)fold;
}

template <int kV>
void run(const char* name, const uint4* in, uint32_t* out, uint64_t* clk, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  sweep<kV><<<blocks, 512>>>(in, 1.0f, out, clk);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a);
    sweep<kV><<<blocks, 512>>>(in, 1.0f, out, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  uint64_t h[2];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / ((double)h[1] * 10.0);  // memrealtime ticks at 100 MHz
  const double mfma = (double)blocks * 8 * kTiles * kSub * kG;  // step count (one MFMA each)
  const double cyc = best * 1e-3 * ghz * 1e9 * 1024.0 / mfma;  // per step per SIMD (1024 SIMDs)
  printf("%-10s %8.3f ms  clock %.2f GHz (block 0)  %6.1f cycles/step/SIMD  (nominal 2.4 GHz: %6.1f)\n",
         name, best, ghz, cyc, best * 1e-3 * 2.4e9 * 1024.0 / mfma);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  const int blocks = 2048;
  uint4* in;
  uint32_t* out;
  uint64_t* clk;
  hipMalloc(&in, 1024 * sizeof(uint4));
  hipMalloc(&out, (size_t)blocks * 512 * 4);
  hipMalloc(&clk, (size_t)blocks * 16);
  // small fp16 values (0x3c00 = 1.0 pattern + noise): finite keys
  uint4 h[1024];
  for (int i = 0; i < 1024; ++i) {
    uint32_t v = 0x3c003c00u ^ (uint32_t)(i * 2654435761u & 0x03ff03ffu);
    h[i] = make_uint4(v, v ^ 0x00010001u, v ^ 0x00020002u, v ^ 0x00030003u);
  }
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  run<2>("mfma", in, out, clk, blocks);
  run<3>("valu", in, out, clk, blocks);
  run<0>("sweep", in, out, clk, blocks);
  run<1>("sweep_min", in, out, clk, blocks);
  run<4>("sweep_c", in, out, clk, blocks);
  run<5>("sweep_nb", in, out, clk, blocks);
  run<6>("sweep_or", in, out, clk, blocks);
  run<7>("sweep_or_nb", in, out, clk, blocks);
  run<8>("mix", in, out, clk, blocks);
  run<10>("valu_or", in, out, clk, blocks);
  run<9>("sweep_or_prio", in, out, clk, blocks);
  hipFree(in);
  hipFree(out);
  hipFree(clk);
  return 0;
}
