// Microbenchmark: issue cost of the f16 MFMA shapes on gfx950 (back-to-back, 4 independent
// accumulators per wave, operands in registers, one or two waves per SIMD).  Question it answers:
// does the legacy K = 8 form (32x32x8) take fewer cycles than the K = 16 form the screens use?
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma_k.hip -o /tmp/ubench_mfma_k
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

template <int kV>
__global__ __launch_bounds__(256) void k(const float* in, float* out) {
  const float s = in[threadIdx.x & 63];
  half8 a8, b8;
  half4 a4, b4;
  for (int i = 0; i < 8; ++i) {
    a8[i] = (_Float16)(s + i);
    b8[i] = (_Float16)(s - i);
  }
  for (int i = 0; i < 4; ++i) {
    a4[i] = a8[i];
    b4[i] = b8[i];
  }
  floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  floatx4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
  for (int it = 0; it < kIters; ++it) {
    if constexpr (kV == 0) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, c3, 0, 0, 0);
    } else if constexpr (kV == 1) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, c3, 0, 0, 0);
    } else if constexpr (kV == 2) {
      d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, d3, 0, 0, 0);
    } else {
      d0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, d3, 0, 0, 0);
    }
  }
  float r = 0.0f;
  for (int i = 0; i < 16; ++i) r += c0[i] + c1[i] + c2[i] + c3[i];
  for (int i = 0; i < 4; ++i) r += d0[i] + d1[i] + d2[i] + d3[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int kV>
static void run(const char* name, const float* in, float* out, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<kV><<<blocks, 256>>>(in, out);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    k<kV><<<blocks, 256>>>(in, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  // waves per SIMD = blocks * 4 / 1024; MFMAs per SIMD = that * 4 * kIters
  const double per_simd = (double)blocks * 4 / 1024 * 4 * kIters;
  printf("%-12s blocks %5d  %.3f ms  %.2f ns per MFMA per SIMD (%.1f cycles at 2.4 GHz)\n", name,
         blocks, best, best * 1e6 / per_simd, best * 1e6 / per_simd * 2.4);
}

int main() {
  float *in, *out;
  hipMalloc(&in, 64 * sizeof(float));
  hipMemset(in, 0, 64 * sizeof(float));
  hipMalloc(&out, 2048 * 256 * sizeof(float));
  for (int blocks : {256, 512}) {
    run<0>("32x32x16", in, out, blocks);
    run<1>("32x32x8", in, out, blocks);
    run<2>("16x16x32", in, out, blocks);
    run<3>("16x16x16", in, out, blocks);
  }
  return 0;
}
