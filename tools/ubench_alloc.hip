// hipMalloc / hipFree against the stream-ordered pool (hipMallocAsync / hipFreeAsync) at the
// cloud-block sizes of cfg1 (2.4 + 4.8 MB) — is the per-cloud allocation worth pooling?
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <algorithm>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipSetDevice(0);
  hipFree(nullptr);
  const size_t sz[2] = {(size_t)100000 * 24 + 100352 * 16, (size_t)100000 * 48 + 100352 * 16};
  std::vector<double> m, f, ma, fa;
  for (int r = 0; r < 25; ++r) {
    void *a = nullptr, *b = nullptr;
    double t0 = now_us();
    hipMalloc(&a, sz[0]);
    hipMalloc(&b, sz[1]);
    double t1 = now_us();
    hipMemset(a, 0, 64);
    hipMemset(b, 0, 64);
    hipDeviceSynchronize();
    double t2 = now_us();
    hipFree(a);
    hipFree(b);
    double t3 = now_us();
    m.push_back(t1 - t0);
    f.push_back(t3 - t2);
  }
  hipMemPool_t pool;
  hipDeviceGetDefaultMemPool(&pool, 0);
  uint64_t thr = UINT64_MAX;
  hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
  hipStream_t st = nullptr;
  for (int r = 0; r < 25; ++r) {
    void *a = nullptr, *b = nullptr;
    double t0 = now_us();
    hipMallocAsync(&a, sz[0], st);
    hipMallocAsync(&b, sz[1], st);
    double t1 = now_us();
    hipMemsetAsync(a, 0, 64, st);
    hipMemsetAsync(b, 0, 64, st);
    hipStreamSynchronize(st);
    double t2 = now_us();
    hipFreeAsync(a, st);
    hipFreeAsync(b, st);
    double t3 = now_us();
    hipStreamSynchronize(st);
    ma.push_back(t1 - t0);
    fa.push_back(t3 - t2);
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin() + 1, v.end()); return v[1 + (v.size() - 1) / 2]; };
  printf("hipMalloc x2 %.1f us, hipFree x2 %.1f us; hipMallocAsync x2 %.1f us, hipFreeAsync x2 %.1f us (medians, first excluded)\n",
         med(m), med(f), med(ma), med(fa));
  return 0;
}
