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

// 8-byte buffer load into VGPRs, issued unconditionally (masked lanes pass kOOB and read
// zeros): the per-wave load count stays fixed for the counted vmcnt waits
DDLPC_DEVICE uint2 buf_load8(__amdgpu_buffer_rsrc_t r, unsigned off) {
  asm volatile("" : "+v"(off));
  const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_uint2(v.x, v.y);
}

// 16-byte epilogue stores from the 16x16 MFMA D layout (A = weights, B = pixels): lane l
// holds channels 4g..4g+3 (g = l >> 4) of pixel l & 15 for each 16-channel tile.  For two
// adjacent tiles (lo, hi) one v_permlane16_swap per dword leaves every lane 8 consecutive
// channels of its pixel — lanes 0-15: lo 0-7, 16-31: hi 0-7, 32-47: lo 8-15, 48-63: hi 8-15
// (channel offset pair16_ch within the 32-channel pair): half the store instructions of the
// 8-byte layout, whole 64-byte pixel rows per instruction
DDLPC_DEVICE uint4 pair16(uint2 lo, uint2 hi) {
  const auto x = __builtin_amdgcn_permlane16_swap(lo.x, hi.x, false, false);
  const auto y = __builtin_amdgcn_permlane16_swap(lo.y, hi.y, false, false);
  return make_uint4(x[0], y[0], x[1], y[1]);
}
DDLPC_DEVICE int pair16_ch(int lane) { return ((lane >> 4) & 1) * 16 + (lane >> 5) * 8; }

// prologue constants (BN scale, shift) of the 8 consecutive input channels c8 .. c8 + 7
// (clamped to lim - 1) straight from global memory into registers: channels >= C1 belong to
// the second input tensor (psc2 / psh2).  For kernels whose lanes keep one channel group for
// the whole launch, so the in-LDS transform needs no per-piece LDS table reads
DDLPC_DEVICE void pro8_load(const float* psc, const float* psh, const float* psc2, const float* psh2,
                            int C1, int c8, int lim, float (&sc)[8], float (&sh)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = min(c8 + j, lim - 1);
    sc[j] = c < C1 ? psc[c] : psc2[c - C1];
    sh[j] = c < C1 ? psh[c] : psh2[c - C1];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(sc[j]), "v"(sh[j]));   // consumed here: before any DMA
}

// ---- BN-backward epilogue (ConvFwdArgs::bnb_y): LDS table [4][nb] of (scale, shift,
// invstd, -mean*invstd) for the channels [co0, co0 + nb) of a workgroup's n tile
DDLPC_DEVICE void bnb_fill(float* tab, int nb, int co0, int Cout, const float* s4, int tid, int nth) {
  for (int i = tid; i < nb; i += nth) {
    const int c = co0 + i;
    const bool ok = c < Cout;
    const float is = ok ? s4[Cout + c] : 0.f;
    tab[i] = ok ? s4[2 * Cout + c] : 0.f;
    tab[nb + i] = ok ? s4[3 * Cout + c] : 0.f;
    tab[2 * nb + i] = is;
    tab[3 * nb + i] = ok ? -s4[c] * is : 0.f;
  }
}
// the constants of 4 consecutive channels (table column col)
struct BnbC { float4 sc, sh, is, nm; };
// (restrict: alias scopes, so the compiler does not drain in-flight LDS-DMA before the reads)
DDLPC_DEVICE BnbC bnb_load(const float* __restrict__ tab, int nb, int col) {
  tab += opaque_zero();              // re-read per use, not hoisted into live VGPRs
  BnbC k;
  k.sc = *reinterpret_cast<const float4*>(tab + col);
  k.sh = *reinterpret_cast<const float4*>(tab + nb + col);
  k.is = *reinterpret_cast<const float4*>(tab + 2 * nb + col);
  k.nm = *reinterpret_cast<const float4*>(tab + 3 * nb + col);
  return k;
}
// (sum dyh, sum dyh*xhat) of those 4 channels of one pixel: d = the fp32 dA (before its bf16
// store; masked lanes pass zeros), yv = y; the arithmetic of bn_bwd2_kernel's reduction pass
// as packed fp32 pairs
DDLPC_DEVICE void bnb_accum(const float (&d)[4], uint2 yv, const BnbC& k, float (&s1)[4], float (&s2)[4]) {
  const f32x2_t y01 = {lo_bf(yv.x), hi_bf(yv.x)}, y23 = {lo_bf(yv.y), hi_bf(yv.y)};
  const f32x2_t a01 = __builtin_elementwise_fma(y01, f32x2_t{k.sc.x, k.sc.y}, f32x2_t{k.sh.x, k.sh.y});
  const f32x2_t a23 = __builtin_elementwise_fma(y23, f32x2_t{k.sc.z, k.sc.w}, f32x2_t{k.sh.z, k.sh.w});
  const f32x2_t x01 = __builtin_elementwise_fma(y01, f32x2_t{k.is.x, k.is.y}, f32x2_t{k.nm.x, k.nm.y});
  const f32x2_t x23 = __builtin_elementwise_fma(y23, f32x2_t{k.is.z, k.is.w}, f32x2_t{k.nm.z, k.nm.w});
  const f32x2_t d01 = {a01.x > 0.f ? d[0] : 0.f, a01.y > 0.f ? d[1] : 0.f};
  const f32x2_t d23 = {a23.x > 0.f ? d[2] : 0.f, a23.y > 0.f ? d[3] : 0.f};
  f32x2_t p01 = {s1[0], s1[1]}, p23 = {s1[2], s1[3]}, q01 = {s2[0], s2[1]}, q23 = {s2[2], s2[3]};
  p01 += d01; p23 += d23;
  q01 = __builtin_elementwise_fma(d01, x01, q01);
  q23 = __builtin_elementwise_fma(d23, x23, q23);
  s1[0] = p01.x; s1[1] = p01.y; s1[2] = p23.x; s1[3] = p23.y;
  s2[0] = q01.x; s2[1] = q01.y; s2[2] = q23.x; s2[3] = q23.y;
}
// bnb_accum with the xhat term factored out of the pixel loop: s2 sums dyh * y (not dyh *
// xhat); bnb_xhat_sum turns the reduced sums into sum dyh * xhat = invstd * sum dyh * y +
// (-mean * invstd) * sum dyh — two packed FMAs per 4 channels fewer per pixel
DDLPC_DEVICE void bnb_accum_y(const float (&d)[4], uint2 yv, const BnbC& k, float (&s1)[4], float (&s2)[4]) {
  const f32x2_t y01 = {lo_bf(yv.x), hi_bf(yv.x)}, y23 = {lo_bf(yv.y), hi_bf(yv.y)};
  const f32x2_t a01 = __builtin_elementwise_fma(y01, f32x2_t{k.sc.x, k.sc.y}, f32x2_t{k.sh.x, k.sh.y});
  const f32x2_t a23 = __builtin_elementwise_fma(y23, f32x2_t{k.sc.z, k.sc.w}, f32x2_t{k.sh.z, k.sh.w});
  const f32x2_t d01 = {a01.x > 0.f ? d[0] : 0.f, a01.y > 0.f ? d[1] : 0.f};
  const f32x2_t d23 = {a23.x > 0.f ? d[2] : 0.f, a23.y > 0.f ? d[3] : 0.f};
  f32x2_t p01 = {s1[0], s1[1]}, p23 = {s1[2], s1[3]}, q01 = {s2[0], s2[1]}, q23 = {s2[2], s2[3]};
  p01 += d01; p23 += d23;
  q01 = __builtin_elementwise_fma(d01, y01, q01);
  q23 = __builtin_elementwise_fma(d23, y23, q23);
  s1[0] = p01.x; s1[1] = p01.y; s1[2] = p23.x; s1[3] = p23.y;
  s2[0] = q01.x; s2[1] = q01.y; s2[2] = q23.x; s2[3] = q23.y;
}
DDLPC_DEVICE float bnb_xhat_sum(const BnbC& k, int i, float sd, float sdy) {
  const float is = i == 0 ? k.is.x : i == 1 ? k.is.y : i == 2 ? k.is.z : k.is.w;
  const float nm = i == 0 ? k.nm.x : i == 1 ? k.nm.y : i == 2 ? k.nm.z : k.nm.w;
  return __builtin_fmaf(is, sdy, nm * sd);
}

}  // namespace convlds
}  // namespace ddlpc
