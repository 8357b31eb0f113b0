// LDS / LDS-DMA helpers shared by the implicit-GEMM 3x3 conv kernels (conv3x3_fwd.hip,
// conv3x3_res.hip).
//
//   * LDS rows are 64 B (one pixel or one weight row of a 32-channel chunk) holding four
//     16-B pieces; piece q of row r is stored at q ^ swz(r) — conflict-free for the gfx950
//     ds_read_b128 lane groups when 16 lanes read 16 consecutive rows;
//   * operands arrive by LDS-DMA (buffer_load ... lds): 64 lanes x 16 B land LANE-LINEARLY
//     at a wave-uniform LDS base, so the swizzle is applied on the SOURCE address;
//   * an out-of-range buffer offset (kOOB) reads as zero: free zero padding.
#pragma once

#include "common.h"

namespace ddlpc {
namespace convlds {

constexpr int BK = 32;                 // channels per K chunk
constexpr int ROWB = BK * 2;           // bytes per LDS row
constexpr unsigned kOOB = 0x80000000u; // buffer offset that reads as zero

DDLPC_DEVICE int swz(int row) { return ((row >> 2) & 1) << 1; }
DDLPC_DEVICE int lds_off(int row, int piece) { return row * ROWB + ((piece ^ swz(row)) << 4); }

// LDS writes of this wave done + workgroup barrier (raw s_barrier: __syncthreads() would
// also drain the in-flight LDS-DMA loads we deliberately keep outstanding)
DDLPC_DEVICE void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
DDLPC_DEVICE void dma_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (an immediate per case; n <= 47 here)
DDLPC_DEVICE void vm_wait_dyn(int n) {
#define VW4(b) case b: dma_wait<b>(); break; case b + 1: dma_wait<b + 1>(); break; \
               case b + 2: dma_wait<b + 2>(); break; case b + 3: dma_wait<b + 3>(); break;
  switch (n) {
    VW4(0) VW4(4) VW4(8) VW4(12) VW4(16) VW4(20) VW4(24) VW4(28) VW4(32) VW4(36) VW4(40) VW4(44)
    default: dma_wait<0>();
  }
#undef VW4
}

DDLPC_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

DDLPC_DEVICE void dma16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)((size_t)lds_wave_base), 16, (int)voff, 0, 0, 0);
}

DDLPC_DEVICE uint4 lds128(const char* p) { return *reinterpret_cast<const uint4*>(p); }

}  // namespace convlds
}  // namespace ddlpc
