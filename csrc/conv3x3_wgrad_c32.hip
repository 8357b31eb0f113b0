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
template <int NC>
constexpr int c32_smem() { return C32_PRO + 2 * (C32_YBYTES + NC * C32_XBYTES); }
static_assert(c32_smem<3>() <= 160 * 1024, "LDS budget");

template <int NC>
__global__ __launch_bounds__(512, 1) void conv3_wgrad_c32_kernel(ConvWgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_pro = reinterpret_cast<float*>(smem);
  char* base = smem + C32_PRO;
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
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int px = ((i * 8 + wave) * 64 + lane) >> 2;
        const int gh = h0 + (px >> 4), gw = w0 + (px & 15);
        const bool ok = gh < p.H && gw < p.W;
        dma16(r, sY(b) + (i * 8 + wave) * 1024,
              ok ? ((unsigned)(gh * p.W + gw) * 32 + (lane & 3) * 8) * 2u : kOOB);
      }
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
      a.dyy != nullptr || a.Cin < 64 || a.Cin > 96 || a.W < 16)
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
