// Microbenchmark: per-lane gathers in the grid scan's pattern (grid.hip grid_scan, kL = 4 lanes
// per query, kR = 2 rows × kB = 2 points per lane per round) from an L2-resident point array, by
// record width: 16 B (float4, today's records), 8 B (uint2) and 4 B.  Each round's rows depend on
// the previous round's data (the scan's start → points chain), 8 waves per SIMD resident.  Prints
// the launch time and ns per wave-round: whether halving the bytes a gather returns shortens it.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_gather tools/ubench_gather.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kRounds = 64;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <typename T>
__device__ __forceinline__ uint32_t bits_of(const T& v);
template <> __device__ __forceinline__ uint32_t bits_of<float4>(const float4& v) {
  return __float_as_uint(v.x) ^ __float_as_uint(v.y) ^ __float_as_uint(v.z) ^ __float_as_uint(v.w);
}
template <> __device__ __forceinline__ uint32_t bits_of<uint2>(const uint2& v) { return v.x ^ v.y; }
template <> __device__ __forceinline__ uint32_t bits_of<uint32_t>(const uint32_t& v) { return v; }

// NOTE: rows of 8 consecutive records (a lane takes sub and sub + 4), 2 rows per round; lanes of a
// query (4) share their rows; a wave holds 16 queries at unrelated positions (spatially coherent
// in the real scan: neighbouring queries' rows overlap — `span` limits the rows to a window)
template <typename T>
__global__ __launch_bounds__(256) void gather_kernel(const T* __restrict__ a, uint32_t n, uint32_t span,
                                                     uint32_t* __restrict__ out) {
  const uint32_t q = (blockIdx.x * 256 + threadIdx.x) >> 2, sub = threadIdx.x & 3;
  const uint32_t w0 = hash32(blockIdx.x * 4 + (threadIdx.x >> 6)) % (n - span - 16);
  uint32_t acc = 0;
  for (int r = 0; r < kRounds; ++r) {
    const uint32_t h = hash32(q * 977u + r * 131u + (acc & 1u));
    const uint32_t r0 = w0 + (h % span), r1 = w0 + ((h >> 12) % span);
    const T v0 = a[r0 + sub], v1 = a[r0 + sub + 4], v2 = a[r1 + sub], v3 = a[r1 + sub + 4];
    acc += bits_of(v0) + bits_of(v1) + bits_of(v2) + bits_of(v3);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// The scan's per-query loads (query point, seed, row starts) are the same address on the 4 lanes
// of a query: every lane loading it (quad-uniform addresses) against one lane per quad loading it
// and a DPP broadcast to the other three
template <bool kOneLane>
__global__ __launch_bounds__(256) void quad_kernel(const float4* __restrict__ a, uint32_t n, uint32_t span,
                                                   uint32_t* __restrict__ out) {
  const uint32_t q = (blockIdx.x * 256 + threadIdx.x) >> 2, sub = threadIdx.x & 3;
  const uint32_t w0 = hash32(blockIdx.x * 4 + (threadIdx.x >> 6)) % (n - span - 16);
  uint32_t acc = 0;
  for (int r = 0; r < kRounds; ++r) {
    const uint32_t h = hash32(q * 977u + r * 131u + (acc & 1u));
    const uint32_t r0 = w0 + (h % span), r1 = w0 + ((h >> 12) % span);
    uint32_t x = 0;
    if (!kOneLane || sub == 0) {
      const float4 v0 = a[r0], v1 = a[r1];
      x = bits_of(v0) + bits_of(v1);
    }
    if (kOneLane) x = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x00, 0xF, 0xF, false);
    acc += x;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static void run_quad(bool one, uint32_t n, uint32_t span, int blocks) {
  float4* a; uint32_t* out;
  hipMalloc(&a, sizeof(float4) * n);
  hipMalloc(&out, sizeof(uint32_t) * 256 * blocks);
  hipMemset(a, 0x3c, sizeof(float4) * n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float best = 1e30f;
  for (int it = 0; it < 12; ++it) {
    hipEventRecord(e0);
    if (one) quad_kernel<true><<<blocks, 256>>>(a, n, span, out);
    else quad_kernel<false><<<blocks, 256>>>(a, n, span, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (it > 1 && ms < best) best = ms;
  }
  printf("quad-uniform 16-B loads, %s: n=%u span=%u: %8.2f us\n", one ? "one lane + DPP" : "all 4 lanes", n, span,
         best * 1e3);
  hipFree(a); hipFree(out);
}

template <typename T>
static void run(const char* name, uint32_t n, uint32_t span, int blocks) {
  T* a; uint32_t* out;
  hipMalloc(&a, sizeof(T) * n);
  hipMalloc(&out, sizeof(uint32_t) * 256 * blocks);
  hipMemset(a, 0x3c, sizeof(T) * n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float best = 1e30f;
  for (int it = 0; it < 12; ++it) {
    hipEventRecord(e0);
    gather_kernel<T><<<blocks, 256>>>(a, n, span, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (it > 1 && ms < best) best = ms;
  }
  const double waves = blocks * 4.0;
  printf("%-6s n=%8u (%6.1f MB) span=%6u blocks=%5d: %8.2f us, %6.2f ns per wave-round chip-wide, %.2f TB/s returned\n",
         name, n, sizeof(T) * (double)n / 1e6, span, blocks, best * 1e3, best * 1e6 / (waves * kRounds),
         waves * kRounds * 64 * 4 * sizeof(T) / (best * 1e-3) / 1e12);
  hipFree(a); hipFree(out);
}

int main() {
  for (uint32_t n : {100000u, 1000000u}) {
    run_quad(false, n, 2048, 1560);
    run_quad(true, n, 2048, 1560);
  }
  for (uint32_t n : {100000u, 1000000u}) {
    for (uint32_t span : {2048u, 65536u}) {
      const int blocks = 1560;  // ≈ cfg1's 6,234 waves
      run<float4>("16B", n, span, blocks);
      run<uint2>("8B", n, span, blocks);
      run<uint32_t>("4B", n, span, blocks);
    }
  }
  return 0;
}
