// lds_dma.h — the double-buffered tile loaders' global → LDS copy (score_mfma_kernel,
// nn_mfma_kernel): global_load_lds_dwordx4 writes 16 B per lane straight into LDS at a
// wave-uniform base + lane × 16 B, so the next tile needs no prefetch registers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace m3d {

// Issue one wave's 64 × 16-B copy: lane l's `src` lands at wave_dst + 16·l (wave_dst: the
// address lane 0 writes, the same in every lane).  Inline asm rather than
// __builtin_amdgcn_global_load_lds: through the builtin hipcc cannot tell the DMA's buffer from
// the one being swept and waits for the DMA before the sweep's first ds_read.  The caller retires
// the copy with lds_dma_wait() before the barrier that publishes the buffer; ordinary loads the
// compiler issues meanwhile keep correct waits (an older pending copy only makes them stricter).
// M0 is a register the compiler reserves (it never honours an M0 clobber), so the asm saves it
// in an SGPR of its own and restores it after the copy: whatever the compiler keeps in M0 (a
// v_writelane lane index, say) survives the call.
__device__ __forceinline__ void lds_dma16(const void* src, void* wave_dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)wave_dst);
  uint32_t saved;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(src), "s"(lds)
      : "memory");
}

// every copy this wave issued has landed in LDS
__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace m3d
