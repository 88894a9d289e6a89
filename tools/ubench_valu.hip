// Microbenchmark: fp32 VALU throughput on gfx950 (v_fma_f32 vs v_pk_fma_f32, VGPR vs SGPR
// operands, v_min3_f32).  Each kernel runs 8 independent chains per lane; grid = 256 CUs ×
// 8 waves/SIMD.  Prints GFLOP/s (FMA = 2 flop) or Gop/s.
//   hipcc --offload-arch=gfx950 -O3 -o ubench_valu tools/ubench_valu.hip && ./ubench_valu
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void fma_v(float* out, float b, float c) {
  float a[8];
  const float bv = b + threadIdx.x * 1e-9f, cv = c - threadIdx.x * 1e-9f;
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k;
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = fmaf(a[k], bv, cv);
  float s = 0;
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_s(float* out, float b, float c) {  // SGPR operand
  float a[8];
  const float cv = c - threadIdx.x * 1e-9f;
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k;
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = fmaf(a[k], b, cv);
  float s = 0;
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_pk(float* out, float b, float c) {
  f2 a[8];
  const f2 bv = {b + threadIdx.x * 1e-9f, b}, cv = {c, c - threadIdx.x * 1e-9f};
  for (int k = 0; k < 8; ++k) a[k] = (f2){(float)threadIdx.x + k, (float)k};
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = __builtin_elementwise_fma(a[k], bv, cv);
  float s = 0;
  for (int k = 0; k < 8; ++k) s += a[k].x + a[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void min3_v(float* out, float b, float c) {
  float a[8];
  const float bv = b + threadIdx.x, cv = c - threadIdx.x;
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k;
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = fminf(fminf(a[k], bv + k), cv - k);
  float s = 0;
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
static void run(const char* name, K kern, double ops_per_thread_iter, float* out) {
  const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  kern<<<blocks, 256>>>(out, 1.0001f, 0.999f);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) kern<<<blocks, 256>>>(out, 1.0001f, 0.999f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double ops = 5.0 * blocks * 256.0 * kIters * ops_per_thread_iter;
  printf("%-8s %8.3f ms  %8.1f Gop/s per launch-set -> %7.1f T(ops)/s\n", name, ms, ops / ms / 1e6,
         ops / ms / 1e9);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
  run("fma_v", fma_v, 16, out);    // 8 FMA = 16 flop
  run("fma_s", fma_s, 16, out);
  run("fma_pk", fma_pk, 32, out);  // 8 × 2 FMA = 32 flop
  run("min3", min3_v, 16, out);    // 8 × 2 min (as ops)
  hipFree(out);
  return 0;
}
