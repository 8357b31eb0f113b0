// Weight gradient of the 2-D 32-output-channel CONCAT conv (dec1.a at width/2: cat(skip 32,
// up 64) -> 32 at 256², ref.py:579 / SURVEY K3), ALL input chunks per workgroup.
//
//     dW[co][kh][kw][ci] = sum_p dY[p][co] X[p + (kh, kw) - 1][ci]
//
// The v3 weight gradient gives each workgroup one 32-channel input chunk, so the 256² × 32 dY
// is streamed once per chunk (3× for dec1.a) and the layer is HBM-bound at ~0.65 PF/s.  Here
// one persistent 8-wave workgroup per CU walks a contiguous range of 16 × 16 pixel tiles and
// stages, per tile, the dY tile (16 KB) and the halos of ALL NC input chunks (18 × 18 × 32
// each) by LDS-DMA into a two-stage ring (counted vmcnt waits, the next tile's operands in
// flight under this tile's MFMAs): dY is read once.  The 9·NC (chunk, tap) units are split
// over the waves (NC = 3: 4,4,4,3,3,3,3,3 — per SIMD 7,7,7,6, as the 3-D depth-streaming weight
// gradient's (kd, kh, kw) units, conv3x3x3_wgrad_ds.hip, whose compute loop this is with the
// depth taps replaced by input chunks), each unit a 32×32 fp32 accumulator of
// v_mfma_f32_32x32x16_bf16 on transposed ds_read_b64_tr_b16 operands, fragments register
// double-buffered.  A wave's units are complete per workgroup: it writes its slab rows
// part[wg][32][9][Cin] once at the end (reduce_rows_scatter sums the workgroups in a fixed
// order).  The BN prologues of either concat input are applied in place by the lanes that
// DMA'd each piece (constants in an LDS table per chunk).
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

#include <cstdlib>
#include <type_traits>

namespace ddlpc {

namespace {

using namespace convlds;

constexpr int C32_T = 16, C32_HW2 = 18;
constexpr int C32_HALO = C32_HW2 * C32_HW2;               // 324
constexpr int C32_XINSTR = (C32_HALO * 4 + 63) / 64;      // 21 DMA wave-instructions per halo
constexpr int C32_XITERS = (C32_XINSTR + 7) / 8;          // 3 / 2 per wave
constexpr int C32_XBYTES = C32_XINSTR * 1024;
constexpr int C32_YBYTES = C32_T * C32_T * 64;            // 16 KB (16 instructions)
constexpr int C32_PRO = 3 * 64 * 4;                       // prologue table [3 chunks][scale|shift][32]
constexpr int C32_DYP = 7 * 32 * 4;                       // dY prologue table [7][32]
template <int NC>
constexpr int c32_smem() { return C32_PRO + C32_DYP + 2 * (C32_YBYTES + NC * C32_XBYTES); }
static_assert(c32_smem<3>() <= 160 * 1024, "LDS budget");

template <int NC>
__global__ __launch_bounds__(512, 1) void conv3_wgrad_c32_kernel(ConvWgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_pro = reinterpret_cast<float*>(smem);
  float* s_dy = s_pro + C32_PRO / 4;                 // dY prologue: [7][32]
  char* base = smem + C32_PRO + C32_DYP;
  constexpr int STAGE = C32_YBYTES + NC * C32_XBYTES;
  auto sY = [&](int b) { return base + b * STAGE; };
  auto sX = [&](int b, int c) { return base + b * STAGE + C32_YBYTES + c * C32_XBYTES; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesH = p.tilesH, tilesW = p.tilesW;
  const int t_begin = (int)((long long)p.nTiles * blockIdx.x / gridDim.x);
  const int t_end = (int)((long long)p.nTiles * (blockIdx.x + 1) / gridDim.x);
  const long long img_px = (long long)p.H * p.W;

  // ---- per chunk: source tensor, channel offset, prologue (table in LDS)
  bool has_pro[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const bool second = c * 32 >= p.C1;
    const float* psc = second ? p.pscale2 : p.pscale;
    const float* psh = second ? p.pshift2 : p.pshift;
    const int cs0 = second ? c * 32 - p.C1 : c * 32;
    has_pro[c] = psc != nullptr;
    if (has_pro[c] && tid < 32) {
      s_pro[c * 64 + tid] = psc[cs0 + tid];
      s_pro[c * 64 + 32 + tid] = psh[cs0 + tid];
    }
  }
  bool any_pro = false;
#pragma unroll
  for (int c = 0; c < NC; ++c) any_pro = any_pro || has_pro[c];
  // dY prologue (BN backward on load, bn_bwd2_kernel's apply arithmetic): the staged tile
  // holds dA; dY = k (dA [y*scale + shift > 0] - m1 - xhat m2) is formed in place by the lanes
  // that DMA'd each piece (y of the same piece loaded to registers with the DMA) and stored
  // to dyout for the conv's data gradient.  Table: scale, shift, invstd, -mean*invstd, k, m1, m2
  const bool has_dyp = p.dyy != nullptr;
  if (has_dyp && tid < 32) {
    const float is = p.dys4[32 + tid];
    s_dy[tid] = p.dys4[64 + tid];
    s_dy[32 + tid] = p.dys4[96 + tid];
    s_dy[64 + tid] = is;
    s_dy[96 + tid] = -p.dys4[tid] * is;
    s_dy[128 + tid] = p.dycoef[tid];
    s_dy[160 + tid] = p.dycoef[32 + tid];
    s_dy[192 + tid] = p.dycoef[64 + tid];
  }
  uint4 yv[2];                                       // (dY prologue) y of the lane's 2 dA pieces
  uint32_t ybits = 0;                                // in-image dA pieces, 2 bits per stage

  // ---- DMA of tile t into stage b: dY (piece e -> tile pixel e >> 2) and each chunk's halo
  // (piece e -> halo pixel e >> 2, channel piece e & 3, unswizzled: transposed reads)
  const int nxi = (C32_XINSTR - wave + 7) / 8;       // halo instructions of this wave per chunk
  const int nper = 2 + NC * nxi;                     // DMA instructions per tile (this wave)
  uint32_t vbits = 0;                                // in-image halo pieces, 4 bits per stage
  auto issue = [&](int t, int b) __attribute__((always_inline)) {
    const int tw_ = t % tilesW, q = t / tilesW;
    const int th_ = q % tilesH, n = q / tilesH;
    const int h0 = th_ * C32_T, w0 = tw_ * C32_T;
    {
      const auto r = make_rsrc(p.dY + (long long)n * img_px * 32, (unsigned)(img_px * 64));
      uint32_t yb = 0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int px = ((i * 8 + wave) * 64 + lane) >> 2;
        const int gh = h0 + (px >> 4), gw = w0 + (px & 15);
        const bool ok = gh < p.H && gw < p.W;
        const unsigned off = ok ? ((unsigned)(gh * p.W + gw) * 32 + (lane & 3) * 8) * 2u : kOOB;
        dma16(r, sY(b) + (i * 8 + wave) * 1024, off);
        if (has_dyp) {
          const auto ry = make_rsrc(p.dyy + (long long)n * img_px * 32, (unsigned)(img_px * 64));
          const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
          yv[i] = make_uint4(v.x, v.y, v.z, v.w);
          yb |= (ok ? 1u : 0u) << i;
        }
      }
      ybits = (ybits & ~(0x3u << (2 * b))) | (yb << (2 * b));
    }
    uint32_t valid = 0;
    int pix[C32_XITERS];
#pragma unroll
    for (int i = 0; i < C32_XITERS; ++i) {
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;
      const int gh = h0 + px / C32_HW2 - 1, gw = w0 + px % C32_HW2 - 1;
      const bool ok = i * 8 + wave < C32_XINSTR && px < C32_HALO && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W;
      pix[i] = ok ? gh * p.W + gw : -1;
      valid |= (ok ? 1u : 0u) << i;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const bool second = c * 32 >= p.C1;
      const int Cs = second ? p.C2 : p.C1;
      const int cs0 = second ? c * 32 - p.C1 : c * 32;
      const auto r = make_rsrc((second ? p.X2 : p.X1) + (long long)n * img_px * Cs, (unsigned)(img_px * Cs * 2));
#pragma unroll
      for (int i = 0; i < C32_XITERS; ++i) {
        if (i * 8 + wave >= C32_XINSTR) break;
        dma16(r, sX(b, c) + (i * 8 + wave) * 1024,
              pix[i] >= 0 ? ((unsigned)pix[i] * Cs + cs0 + (lane & 3) * 8) * 2u : kOOB);
      }
    }
    vbits = (vbits & ~(0xfu << (4 * b))) | (valid << (4 * b));
  };
  // prologue BN + ReLU on this lane's own landed pieces of chunk c (restrict: alias scopes)
  auto transform_body = [&](char* __restrict__ X, int c, uint32_t valid) __attribute__((always_inline)) {
    const float4* kp = reinterpret_cast<const float4*>(s_pro + opaque_zero() + c * 64 + (lane & 3) * 8);
    const float4 sa = kp[0], sb = kp[1], ha = kp[8], hb = kp[9];
    const float sc[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float sh[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
    uint4 v[C32_XITERS];
#pragma unroll
    for (int i = 0; i < C32_XITERS; ++i)
      if (i * 8 + wave < C32_XINSTR) v[i] = *reinterpret_cast<const uint4*>(X + ((i * 8 + wave) * 64 + lane) * 16);
#pragma unroll
    for (int i = 0; i < C32_XITERS; ++i) {
      if (i * 8 + wave >= C32_XINSTR) break;
      const bool ok = (valid >> i) & 1u;
      const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x2_t x = {lo_bf(w[j]), hi_bf(w[j])};
        const f32x2_t y2 = __builtin_elementwise_fma(x, f32x2_t{sc[2 * j], sc[2 * j + 1]},
                                                     f32x2_t{sh[2 * j], sh[2 * j + 1]});
        const uint32_t pk = __builtin_bit_cast(uint32_t, __builtin_convertvector(y2, bf16x2_t));
        const i16x2_t m = __builtin_elementwise_max(__builtin_bit_cast(i16x2_t, pk), i16x2_t{0, 0});
        o[j] = ok ? __builtin_bit_cast(uint32_t, m) : 0u;
      }
      *reinterpret_cast<uint4*>(X + ((i * 8 + wave) * 64 + lane) * 16) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  };

  // dY prologue on the lane's own 2 landed dA pieces of stage b (tile t): in place, and the
  // formed dY stored (the same element offsets the DMA read from)
  auto transform_dy = [&](char* __restrict__ Yb, int t, int b) __attribute__((always_inline)) {
    const int tw_ = t % tilesW, q2 = t / tilesW;
    const int th_ = q2 % tilesH, n = q2 / tilesH;
    const int h0 = th_ * C32_T, w0 = tw_ * C32_T;
    const auto ro = make_rsrc(p.dyout + (long long)n * img_px * 32, (unsigned)(img_px * 64));
    const uint32_t yb = (ybits >> (2 * b)) & 0x3u;
    const float* tb = s_dy + opaque_zero() + (lane & 3) * 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = (i * 8 + wave) * 64 + lane;
      const int px = e >> 2;
      const bool ok = (yb >> i) & 1u;
      uint4* qd = reinterpret_cast<uint4*>(Yb + e * 16);
      float fd[8], fy[8], o[8];
      unpack8(*qd, fd);
      unpack8(yv[i], fy);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = fmaf(fy[j], tb[j], tb[32 + j]);
        const float dyh = a > 0.f ? fd[j] : 0.f;
        const float xh = fmaf(fy[j], tb[64 + j], tb[96 + j]);
        o[j] = tb[128 + j] * (dyh - tb[160 + j] - xh * tb[192 + j]);
      }
      const uint4 pk = ok ? pack8(o) : make_uint4(0, 0, 0, 0);
      *qd = pk;
      const int gh = h0 + (px >> 4), gw = w0 + (px & 15);
      unsigned off = ok ? ((unsigned)(gh * p.W + gw) * 32 + (lane & 3) * 8) * 2u : kOOB;
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{pk.x, pk.y, pk.z, pk.w}, ro, off, 0, 0);
    }
  };

  // ---- this wave's (chunk, tap) units: U = 9 NC over 8 waves, the first U % 8 waves one more
  constexpr int U = 9 * NC, UQ = U / 8, UR = U % 8;
  const int nunit = UQ + (wave < UR ? 1 : 0);
  const int u0 = wave * UQ + (wave < UR ? wave : UR);
  const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int fr0 = ((g4 >> 1) * 8 + q) * ROWB + (g4 & 1) * 32 + 8 * pq;   // + 4 rows: + 4 * ROWB
  constexpr int NTMAX = UQ + (UR ? 1 : 0);
  f32x16_t acc[NTMAX];
#pragma unroll
  for (int t = 0; t < NTMAX; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  // one tile: the wave's units against the staged dY tile and chunk halos (restrict PARAMETERS:
  // the compiler does not drain the next tile's in-flight LDS-DMA before these reads)
  auto compute = [&](const char* __restrict__ Y0, const char* __restrict__ X0,
                     const char* __restrict__ X1, const char* __restrict__ X2, auto ntc)
                     __attribute__((always_inline)) {
    constexpr int NT = decltype(ntc)::value;
    const char* Y = Y0 + fr0;
    const char* xt[NT];
#pragma unroll
    for (int lt = 0; lt < NT; ++lt) {
      const int u = u0 + lt;
      const int c = u / 9, tap = u % 9;
      xt[lt] = (c == 0 ? X0 : c == 1 ? X1 : X2) + ((tap / 3) * C32_HW2 + tap % 3) * ROWB + fr0;
    }
    uint4 af[2], bf[2][NT];
    auto load = [&](int ks, int b) __attribute__((always_inline)) {   // tile row = 16-pixel k-step
      const uint2 alo = lds_read_tr16(Y + ks * 16 * ROWB);
      const uint2 ahi = lds_read_tr16(Y + (ks * 16 + 4) * ROWB);
      af[b] = make_uint4(alo.x, alo.y, ahi.x, ahi.y);
#pragma unroll
      for (int lt = 0; lt < NT; ++lt) {
        const uint2 lo = lds_read_tr16(xt[lt] + ks * C32_HW2 * ROWB);
        const uint2 hi = lds_read_tr16(xt[lt] + (ks * C32_HW2 + 4) * ROWB);
        bf[b][lt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    };
    load(0, 0);
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      if (ks + 1 < 16) load(ks + 1, (ks + 1) & 1);
#pragma unroll
      for (int lt = 0; lt < NT; ++lt) acc[lt] = mfma32x32x16(af[ks & 1], bf[ks & 1][lt], acc[lt]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto compute_tile = [&](int b) __attribute__((always_inline)) {
    const char* x2 = sX(b, NC > 2 ? 2 : NC - 1);
    if (nunit == NTMAX) compute(sY(b), sX(b, 0), sX(b, NC > 1 ? 1 : 0), x2, std::integral_constant<int, NTMAX>{});
    else compute(sY(b), sX(b, 0), sX(b, NC > 1 ? 1 : 0), x2, std::integral_constant<int, (NTMAX > 1 ? NTMAX - 1 : 1)>{});
  };

  // ---- tiles: two-stage ring, counted waits (per-wave ledger of issued DMA instructions)
  __syncthreads();                                   // prologue tables visible
  int issued = 0;
  if (t_begin < t_end) { issue(t_begin, 0); issued += nper; }
  int b = 0;
  for (int t = t_begin; t < t_end; ++t) {
    vm_wait_dyn(0);                                  // this tile's operands landed
    if (has_dyp) transform_dy(sY(b), t, b);
    if (any_pro) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (has_pro[c]) transform_body(sX(b, c), c, (vbits >> (4 * b)) & 0xfu);
    }
    lds_sync();                                      // visible; tile t-1 done by all
    if (t + 1 < t_end) { issue(t + 1, b ^ 1); issued += nper; }
    compute_tile(b);
    b ^= 1;
  }
  (void)issued;
  // ---- slab rows of this wave's units: part[wg][co][tap][ci] (32x32 D layout: column
  // n = lane & 31 = ci within the chunk, row m = 8 (i / 4) + 4 (lane >> 5) + i % 4 = co)
  float* slab = p.partial + (long long)blockIdx.x * 32 * 9 * p.Cin;
#pragma unroll
  for (int lt = 0; lt < NTMAX; ++lt) {
    if (lt >= nunit) break;
    const int u = u0 + lt, c = u / 9, tap = u % 9;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int co = 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
      slab[((long long)co * 9 + tap) * p.Cin + c * 32 + (lane & 31)] = acc[lt][i];
    }
  }
}

}  // namespace

// planner: 2-D, 32 output channels, 2 or 3 whole 32-channel input chunks (a concat conv), no
// BN groups / dY prologue, enough 16x16 tiles for one workgroup per CU with >= 8 tiles each
int conv3_wgrad_c32_plan(ConvWgradArgs& a, int num_cus) {
  if (a.dims != 2 || a.Cout != 32 || a.C1 % 32 != 0 || a.C2 % 32 != 0 || a.groups > 1 ||
      (a.dyy != nullptr && a.dyout == nullptr) || a.Cin < 64 || a.Cin > 96 || a.W < 16)
    return -1;
  const int cmax = a.C1 > a.C2 ? a.C1 : a.C2;
  if ((long long)a.H * a.W * (cmax > 32 ? cmax : 32) * 2 >= (1LL << 31)) return -1;
  const int tilesH = (a.H + C32_T - 1) / C32_T, tilesW = (a.W + C32_T - 1) / C32_T;
  const long long nt = (long long)a.N * tilesH * tilesW;
  if (nt < 8LL * num_cus || nt >= (1LL << 31)) return -1;
  a.tilesH = tilesH;
  a.tilesW = tilesW;
  a.nTiles = (int)nt;
  a.ciChunks = a.Cin / 32;
  a.splits = num_cus;
  return num_cus;
}

void conv3_wgrad_c32_launch(ConvWgradArgs& a, int grid, hipStream_t st) {
  if (a.ciChunks == 3)
    hipLaunchKernelGGL(conv3_wgrad_c32_kernel<3>, dim3(grid), dim3(512), c32_smem<3>(), st, a);
  else
    hipLaunchKernelGGL(conv3_wgrad_c32_kernel<2>, dim3(grid), dim3(512), c32_smem<2>(), st, a);
}

}  // namespace ddlpc
