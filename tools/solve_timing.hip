// Latency of the single-thread ICP solve pieces on one lane (s_memrealtime, 100 MHz ticks).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I3d-matching_amd/csrc \
//          tools/solve_timing.hip -o gpurun_out/solve_timing
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "linalg.h"

using namespace m3d;

__global__ void timing_kernel(const double* in, double* out, long long* ticks) {
  if (threadIdx.x != 0) return;
  double A[36], b[6], x[6], upd[16], T[16];
  for (int k = 0; k < 36; ++k) A[k] = in[k];
  for (int k = 0; k < 6; ++k) b[k] = in[36 + k];
  for (int k = 0; k < 16; ++k) T[k] = in[42 + k];
  long long t0 = wall_clock64();
  ldlt6_solve(A, b, x);
  __builtin_amdgcn_s_waitcnt(0);
  long long t1 = wall_clock64();
  vec6_to_matrix(x, upd);
  long long t2 = wall_clock64();
  matmul4(upd, T, T);
  long long t3 = wall_clock64();
  double s = 0.0;
  for (int k = 0; k < 16; ++k) s += sqrt(T[k] * T[k] + 1.0) / (T[k] + 3.0);
  long long t4 = wall_clock64();
  for (int k = 0; k < 16; ++k) out[k] = T[k] + s;
  ticks[0] = t1 - t0;
  ticks[1] = t2 - t1;
  ticks[2] = t3 - t2;
  ticks[3] = t4 - t3;
}

int main() {
  double h[58];
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) h[i * 6 + j] = (i == j ? 50.0 + i : 0.0) + 1.0 / (1.0 + i + j);
  for (int k = 0; k < 6; ++k) h[36 + k] = 0.01 * (k + 1);
  for (int k = 0; k < 16; ++k) h[42 + k] = (k % 5 == 0) ? 1.0 : 0.0;
  double *din, *dout;
  long long* dt;
  hipMalloc(&din, sizeof(h));
  hipMalloc(&dout, 16 * sizeof(double));
  hipMalloc(&dt, 4 * sizeof(long long));
  hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  long long t[4];
  for (int rep = 0; rep < 3; ++rep) {
    timing_kernel<<<1, 64>>>(din, dout, dt);
    hipMemcpy(t, dt, sizeof(t), hipMemcpyDeviceToHost);
    printf("ldlt6 %.2f us  vec6_to_matrix %.2f us  matmul4 %.2f us  16x(sqrt+div) %.2f us\n",
           t[0] / 100.0, t[1] / 100.0, t[2] / 100.0, t[3] / 100.0);
  }
  // whole-kernel launch-to-completion for reference
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int rep = 0; rep < 100; ++rep) timing_kernel<<<1, 64>>>(din, dout, dt);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("kernel back-to-back %.2f us per launch\n", ms * 10.0);
  return 0;
}
