// Microbenchmark: issue rate of single VALU instructions on gfx950 (wave64, SIMD-32), 8
// independent chains per lane, 512-thread blocks at 4 and 8 waves/SIMD.  Pins the instruction
// with inline asm so the compiler cannot substitute forms.  Prints ns per instruction per SIMD
// (chip-wide: 1024 SIMDs) and the per-wave cycle cost at the s_memtime clock.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_ops tools/ubench_ops.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int kIters = 2048;

#define OP_KERNEL(NAME, ASM)                                                                     \
  __global__ __launch_bounds__(512) void NAME(float* out, float b, float c, uint64_t* clk) {    \
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
          a6 = a0 + 6, a7 = a0 + 7;                                                              \
    float bv = b + threadIdx.x, cv = c - threadIdx.x;                                            \
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();           \
    for (int i = 0; i < kIters; ++i) {                                                           \
      asm volatile(ASM " %0, %0, %8, %9\n" ASM " %1, %1, %8, %9\n" ASM " %2, %2, %8, %9\n" ASM     \
                   " %3, %3, %8, %9\n" ASM " %4, %4, %8, %9\n" ASM " %5, %5, %8, %9\n" ASM         \
                   " %6, %6, %8, %9\n" ASM " %7, %7, %8, %9\n"                                   \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),       \
                     "+v"(a7)                                                                    \
                   : "v"(bv), "v"(cv));                                                          \
    }                                                                                            \
    if (threadIdx.x == 0) {                                                                      \
      clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;                                   \
      clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;                           \
    }                                                                                            \
    out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                 \
  }

#define OP2_KERNEL(NAME, ASM)                                                                    \
  __global__ __launch_bounds__(512) void NAME(float* out, float b, float c, uint64_t* clk) {    \
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
          a6 = a0 + 6, a7 = a0 + 7;                                                              \
    float bv = b + threadIdx.x;                                                                  \
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();           \
    for (int i = 0; i < kIters; ++i) {                                                           \
      asm volatile(ASM " %0, %0, %8\n" ASM " %1, %1, %8\n" ASM " %2, %2, %8\n" ASM " %3, %3, %8\n"  \
                   ASM " %4, %4, %8\n" ASM " %5, %5, %8\n" ASM " %6, %6, %8\n" ASM " %7, %7, %8\n"    \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),       \
                     "+v"(a7)                                                                    \
                   : "v"(bv));                                                                   \
    }                                                                                            \
    if (threadIdx.x == 0) {                                                                      \
      clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;                                   \
      clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;                           \
    }                                                                                            \
    out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                 \
  }

OP2_KERNEL(op_min, "v_min_f32")
OP2_KERNEL(op_or, "v_or_b32")
OP2_KERNEL(op_pkminf16, "v_pk_min_f16")
OP2_KERNEL(op_pkmini16, "v_pk_min_i16")
OP2_KERNEL(op_cvtpk, "v_cvt_pk_f16_f32")
OP2_KERNEL(op_lshr, "v_lshrrev_b32")
OP2_KERNEL(op_bcnt, "v_bcnt_u32_b32")
OP_KERNEL(op_fma, "v_fma_f32")
OP_KERNEL(op_min3, "v_min3_f32")
OP_KERNEL(op_minimum3, "v_minimum3_f32")
OP_KERNEL(op_max3, "v_max3_f32")
OP_KERNEL(op_add3, "v_add3_u32")
OP_KERNEL(op_or3, "v_or3_b32")
OP_KERNEL(op_alignbit, "v_alignbit_b32")
OP_KERNEL(op_mad24, "v_mad_u32_u24")
OP_KERNEL(op_lshlor, "v_lshl_or_b32")
OP_KERNEL(op_andor, "v_and_or_b32")
OP_KERNEL(op_lshladd, "v_lshl_add_u32")

OP_KERNEL(op_perm, "v_perm_b32")
OP_KERNEL(op_med3, "v_med3_f32")
OP_KERNEL(op_fmamix, "v_fma_mix_f32")
OP2_KERNEL(op_mini32, "v_min_i32")
OP2_KERNEL(op_minu32, "v_min_u32")
OP2_KERNEL(op_addu32, "v_add_u32")
OP2_KERNEL(op_subf32, "v_sub_f32")
OP2_KERNEL(op_and, "v_and_b32")
OP2_KERNEL(op_mulf32, "v_mul_f32")


__global__ __launch_bounds__(512) void op_bitop3(float* out, float b, float c, uint64_t* clk) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7;
  float bv = b + threadIdx.x, cv = c - threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < kIters; ++i) {
#define B3(X) "v_bitop3_b32 " X ", " X ", %8, %9 bitop3:0xfe\n"
    asm volatile(B3("%0") B3("%1") B3("%2") B3("%3") B3("%4") B3("%5") B3("%6") B3("%7")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 : "v"(bv), "v"(cv));
#undef B3
  }
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// VOPC compare into VCC + v_cndmask reading it: counted as two instructions per chain step
__global__ __launch_bounds__(512) void op_cmpcnd(float* out, float b, float c, uint64_t* clk) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  float bv = b + threadIdx.x, cv = c - threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < kIters; ++i) {
#define CC(X) "v_cmp_lt_f32 vcc, " X ", %4\nv_cndmask_b32 " X ", " X ", %5, vcc\n"
    asm volatile(CC("%0") CC("%1") CC("%2") CC("%3")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
                 : "v"(bv), "v"(cv)
                 : "vcc");
#undef CC
  }
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3;
}

typedef void (*kfn)(float*, float, float, uint64_t*);

void run(const char* name, kfn k, int blocks_per_cu, float* out, uint64_t* clk) {
  const int blocks = 256 * blocks_per_cu;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k<<<blocks, 512>>>(out, 1.0f, 2.0f, clk);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a);
    k<<<blocks, 512>>>(out, 1.0f, 2.0f, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  uint64_t h[2];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / ((double)h[1] * 10.0);
  const double instr_per_simd = (double)blocks * 8 * kIters * 8 / 1024.0;  // wave-instructions
  const double ns = best * 1e6 / instr_per_simd;
  printf("%-16s %d waves/SIMD  %7.3f ms  %.3f ns/instr/SIMD  clock %.2f GHz -> %.2f cycles\n", name,
         2 * blocks_per_cu, best, ns, ghz, ns * ghz);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  float* out;
  uint64_t* clk;
  hipMalloc(&out, (size_t)256 * 4 * 512 * 4);
  hipMalloc(&clk, (size_t)256 * 4 * 16);
  const struct { const char* n; kfn k; } ks[] = {
      {"v_fma_f32", op_fma},       {"v_min3_f32", op_min3}, {"v_minimum3_f32", op_minimum3},
      {"v_max3_f32", op_max3},     {"v_add3_u32", op_add3}, {"v_or3_b32", op_or3},
      {"v_alignbit_b32", op_alignbit}, {"v_min_f32", op_min}, {"v_or_b32", op_or},
      {"v_pk_min_f16", op_pkminf16}, {"v_pk_min_i16", op_pkmini16}, {"v_cvt_pk_f16_f32", op_cvtpk},
      {"v_lshrrev_b32", op_lshr}, {"v_bcnt_u32_b32", op_bcnt}, {"v_mad_u32_u24", op_mad24},
      {"v_lshl_or_b32", op_lshlor}, {"v_and_or_b32", op_andor}, {"v_lshl_add_u32", op_lshladd},
      {"v_perm_b32", op_perm}, {"v_med3_f32", op_med3},
      {"v_fma_mix_f32", op_fmamix}, {"v_min_i32", op_mini32}, {"v_min_u32", op_minu32},
      {"v_add_u32", op_addu32}, {"v_sub_f32", op_subf32}, {"v_and_b32", op_and},
      {"v_mul_f32", op_mulf32}, {"v_bitop3_b32", op_bitop3},
      {"v_cmp+cndmask", op_cmpcnd}};
  for (int bpc : {4})
    for (const auto& k : ks) run(k.n, k.k, bpc, out, clk);
  hipFree(out);
  hipFree(clk);
  return 0;
}
