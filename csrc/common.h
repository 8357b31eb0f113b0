// Shared helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Conventions used by every kernel in csrc/:
//   * activations are NHWC / NDHWC bf16 (channel fastest), stored as uint16_t;
//   * accumulation, BatchNorm statistics and optimizer state are fp32 (fp64 for the final
//     BN reductions);
//   * wave = 64 lanes; MFMA tiles are v_mfma_f32_16x16x32_bf16 (A/B: 8 bf16 per lane,
//     C/D: 4 fp32 per lane, col = lane&15, row = 4*(lane>>4) + i).
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#define DDLPC_HOST_DEVICE __host__ __device__ __forceinline__
#define DDLPC_DEVICE __device__ __forceinline__

typedef uint16_t bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short i16x8_t __attribute__((ext_vector_type(8)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

// 8-byte store of 4 bf16 (an ext-vector type carries its 8-byte alignment, so this is one
// global_store_dwordx2 — a HIP uint2 store through a computed pointer can be split)
DDLPC_DEVICE void store_bf16x4(bf16_t* dst, uint32_t lo, uint32_t hi) {
  *reinterpret_cast<u32x2_t*>(dst) = u32x2_t{lo, hi};
}

constexpr int kWave = 64;

DDLPC_HOST_DEVICE float bf2f(bf16_t h) {
  union { uint32_t u; float f; } v;
  v.u = static_cast<uint32_t>(h) << 16;
  return v.f;
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef short i16x2_t __attribute__((ext_vector_type(2)));

// round-to-nearest-even (NaN kept quiet).  Device code: the gfx950 hardware conversion
// (v_cvt_pk_bf16_f32, RNE); host code: the same rounding in integer arithmetic.
DDLPC_HOST_DEVICE bf16_t f2bf(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(bf16_t, (__bf16)f);
#else
  union { uint32_t u; float f; } v;
  v.f = f;
  uint32_t u = v.u;
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return static_cast<bf16_t>((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<bf16_t>(u >> 16);
#endif
}

// two floats -> packed bf16x2 in ONE v_cvt_pk_bf16_f32
DDLPC_DEVICE uint32_t pack2(float a, float b) {
  const f32x2_t f = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
}

DDLPC_DEVICE float lo_bf(uint32_t w) { return __builtin_bit_cast(float, w << 16); }
DDLPC_DEVICE float hi_bf(uint32_t w) { return __builtin_bit_cast(float, w & 0xffff0000u); }

// 16-byte (8 x bf16) vector <-> 8 floats
DDLPC_DEVICE void unpack8(const uint4& v, float (&f)[8]) {
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
  f[4] = lo_bf(v.z); f[5] = hi_bf(v.z); f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
}
DDLPC_DEVICE uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

DDLPC_DEVICE f32x4_t mfma16x16x32(const uint4& a, const uint4& b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

typedef float f32x16_t __attribute__((ext_vector_type(16)));
// v_mfma_f32_32x32x16_bf16: A 32(m) x 16(k), B 16(k) x 32(n); lane l holds A[l & 31][8 (l >> 5) ..
// + 7] and B[8 (l >> 5) .. + 7][l & 31]; D element i of lane l is D[8 (i / 4) + 4 (l >> 5) + i % 4][l & 31]
DDLPC_DEVICE f32x16_t mfma32x32x16(const uint4& a, const uint4& b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// sum over the 16 lanes of each DPP row (lanes 16r .. 16r+15), the same value in all 16
// lanes: quad xor 1, quad xor 2, half-row mirror, row mirror — VALU DPP moves instead of
// __shfl_xor's LDS-crossbar ds_bpermute (order fixed: deterministic)
template <int CTRL>
DDLPC_DEVICE float dpp_movf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
DDLPC_DEVICE float row16_sum(float v) {
  v += dpp_movf<0xB1>(v);
  v += dpp_movf<0x4E>(v);
  v += dpp_movf<0x141>(v);
  v += dpp_movf<0x140>(v);
  return v;
}

DDLPC_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DDLPC_DEVICE double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DDLPC_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies &M[row q][cols 4p..4p+3];
// lane i receives column i of the 4 rows (row q in element q).  EXEC must be all ones.
DDLPC_DEVICE uint2 lds_read_tr16(const void* lds_ptr) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  // address-space cast (not an integer round trip) keeps pointer provenance, so the read
  // inherits the alias scope of a restrict-qualified LDS operand pointer
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds_ptr));
  return __builtin_bit_cast(uint2, r);
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5, T1): blocks that share
// an XCD (hardware round-robin: id % 8) receive a contiguous range of logical ids.
DDLPC_DEVICE int xcd_remap(int bid, int nblocks) {
  constexpr int kX = 8;
  if (nblocks < kX) return bid;
  const int q = nblocks / kX, r = nblocks % kX, x = bid % kX;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / kX;
}

// m / d (m >= 0) for a wave-uniform divisor: a shift when d is a power of two (the usual
// U-Net widths), the integer division otherwise
DDLPC_DEVICE int udiv_pow2(int m, int d) {
  if ((d & (d - 1)) == 0) return m >> __builtin_ctz((unsigned)d);
  return m / d;
}

// An offset the compiler cannot prove loop-invariant (an SGPR through an empty asm): LDS
// tables indexed with it are re-read where used instead of being hoisted into live VGPRs.
DDLPC_DEVICE int opaque_zero() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}

inline int ceil_div(long a, long b) { return static_cast<int>((a + b - 1) / b); }
