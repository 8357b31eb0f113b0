// Weight gradient of the 3-D U-Net's 32-output-channel 3x3x3 convs (enc1.b / dec1.b: 32 -> 32,
// dec1.a: 96 -> 32 at 128^3; BASELINE config #5) — DEPTH-STREAMING, the
// weight-gradient counterpart of conv3x3x3_ds.hip.
//
//     dW[co][kd][kh][kw][ci] = sum_p dY[p][co] X[p + (kd, kh, kw) - 1][ci]
//
// The v3 weight gradient runs a 3-D layer as three depth-tap planes, each a 2-D weight
// gradient over all (n, d) slices: dY and X are each streamed three times.  Here a persistent
// 8-wave workgroup owns one 32-channel input chunk and walks 16 x 16 (h, w) tile COLUMNS
// through every depth d: output-gradient plane d (16 x 16 x 32, no halo) and a ring of four
// 18 x 18 x 32 input planes (d-1, d, d+1 in use, d+2 arriving) arrive by LDS-DMA, so dY and
// X are read once; every step accumulates all 27 taps.  The 27 taps are split over the 8 waves
// (waves 0-2 four taps, 3-7 three — per SIMD 7, 7, 7, 6), each tap a 32 x 32 fp32
// accumulator of v_mfma_f32_32x32x16_bf16 (A = dY^T, B = the shifted X plane, both
// ds_read_b64_tr_b16 transposed reads of 64-B pixel rows: conflict-free), A shared by the
// wave's taps: 0.078 B of LDS per MAC.  A wave's taps are complete per workgroup (no k-split),
// so it writes its slab rows directly: part[split][co][27 taps][Cin] with split = the
// workgroup's index within its chunk (reduce_rows_scatter sums the splits).  The X prologue
// (the previous BatchNorm + ReLU) is applied in place by the lanes that DMA'd each piece.
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

namespace ddlpc {

namespace {

using namespace convlds;

constexpr int WD_T = 16, WD_HW2 = 18;
constexpr int WD_HALO = WD_HW2 * WD_HW2;                // 324
constexpr int WD_XINSTR = (WD_HALO * 4 + 63) / 64;      // 21 DMA wave-instructions per X plane
constexpr int WD_XITERS = (WD_XINSTR + 7) / 8;          // 3 / 2 per wave
constexpr int WD_XBYTES = WD_XINSTR * 1024;
constexpr int WD_YINSTR = WD_T * WD_T * 4 / 64;         // 16 per dY plane (2 per wave)
constexpr int WD_YBYTES = WD_YINSTR * 1024;
constexpr int WD_SMEM = 2 * 32 * 4 + 4 * WD_XBYTES + 2 * WD_YBYTES;

__global__ __launch_bounds__(512, 1) void conv3d_wgrad_ds_kernel(ConvWgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_pro = reinterpret_cast<float*>(smem);                 // X prologue scale | shift
  char* sX = smem + 2 * 32 * 4;
  char* sY = sX + 4 * WD_XBYTES;
  auto xslot = [&](int plane) { return sX + (plane & 3) * WD_XBYTES; };
  auto yslot = [&](int plane) { return sY + (plane & 1) * WD_YBYTES; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // workgroup -> (input chunk, split): chunk-major blocks (launcher: grid = ciChunks * R)
  const int R = (int)gridDim.x / p.ciChunks;
  const int cic = (int)blockIdx.x / R, split = (int)blockIdx.x - cic * R;
  const int ci0 = cic * 32;
  const bool second = ci0 >= p.C1;                   // chunk of X2 (C1 % 32 == 0)
  const int Cs = second ? p.C2 : p.C1;
  const int cs0 = second ? ci0 - p.C1 : ci0;
  const bf16_t* xsrc = second ? p.X2 : p.X1;
  const float* psc = second ? p.pscale2 : p.pscale;
  const float* psh = second ? p.pshift2 : p.pshift;
  const bool has_pro = psc != nullptr;
  if (has_pro && tid < 32) {
    s_pro[tid] = psc[cs0 + tid];
    s_pro[32 + tid] = psh[cs0 + tid];
  }
  const int tilesH = (p.H + WD_T - 1) / WD_T, tilesW = (p.W + WD_T - 1) / WD_T;
  const int ncol = p.N * tilesH * tilesW;
  const long long plane_px = (long long)p.H * p.W;
  const long long vol_px = (long long)p.D * plane_px;

  // ---- DMA: X plane halo (piece e -> halo pixel e >> 2, channel piece e & 3, unswizzled) and
  // the dY plane tile (piece e -> tile pixel e >> 2)
  const int nxi = (WD_XINSTR - wave + 7) / 8;        // X instructions of this wave (3 or 2)
  uint32_t vmasks = 0;                               // in-image X pieces per ring slot
  int col_n = 0, col_h0 = 0, col_w0 = 0;
  auto issue_x = [&](int d) {
    const auto r = make_rsrc(xsrc + (long long)col_n * vol_px * Cs, (unsigned)(vol_px * Cs * 2));
    uint32_t valid = 0;
#pragma unroll
    for (int i = 0; i < WD_XITERS; ++i) {
      if (i * 8 + wave >= WD_XINSTR) break;
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;
      const int gh = col_h0 + px / WD_HW2 - 1, gw = col_w0 + px % WD_HW2 - 1;
      const bool ok = px < WD_HALO && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W;
      const unsigned pix = (unsigned)(d * plane_px + gh * p.W + gw);
      dma16(r, xslot(d) + (i * 8 + wave) * 1024, ok ? (pix * Cs + cs0 + (lane & 3) * 8) * 2u : kOOB);
      valid |= (ok ? 1u : 0u) << i;
    }
    vmasks = (vmasks & ~(0xffu << (8 * (d & 3)))) | (valid << (8 * (d & 3)));
  };
  auto issue_y = [&](int d) {
    const auto r = make_rsrc(p.dY + (long long)col_n * vol_px * 32, (unsigned)(vol_px * 64));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;       // tile pixel 0 .. 255
      const int gh = col_h0 + (px >> 4), gw = col_w0 + (px & 15);
      const bool ok = gh < p.H && gw < p.W;
      dma16(r, yslot(d) + (i * 8 + wave) * 1024,
            ok ? ((unsigned)(d * plane_px + gh * p.W + gw) * 32 + (lane & 3) * 8) * 2u : kOOB);
    }
  };
  auto transform_body = [&](char* __restrict__ X, int d) __attribute__((always_inline)) {
    const uint32_t valid = (vmasks >> (8 * (d & 3))) & 0xffu;
    const float4* kp = reinterpret_cast<const float4*>(s_pro + opaque_zero() + (lane & 3) * 8);
    const float4 sa = kp[0], sb = kp[1], ha = kp[8], hb = kp[9];
    const float sc[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float sh[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
    uint4 v[WD_XITERS];
#pragma unroll
    for (int i = 0; i < WD_XITERS; ++i)
      if (i * 8 + wave < WD_XINSTR) v[i] = *reinterpret_cast<const uint4*>(X + ((i * 8 + wave) * 64 + lane) * 16);
#pragma unroll
    for (int i = 0; i < WD_XITERS; ++i) {
      if (i * 8 + wave >= WD_XINSTR) break;
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

  // ---- this wave's taps: waves 0-2 own 4 consecutive taps, waves 3-7 three (27 in all)
  const int ntap = wave < 3 ? 4 : 3;
  const int tap0 = wave < 3 ? 4 * wave : 12 + 3 * (wave - 3);
  // transposed-read geometry (v3's BCO-32 layout): 16-lane group g4 = lane >> 4, row q, column
  // group pq; A rows = tile pixels (k), B rows = halo pixels shifted by the tap
  const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int ya0 = ((g4 >> 1) * 8 + q) * ROWB + (g4 & 1) * 32 + 8 * pq;   // + 4 rows: + 4 * ROWB
  const int xb0 = ((g4 >> 1) * 8 + q) * ROWB + (g4 & 1) * 32 + 8 * pq;
  f32x16_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  // one output-gradient plane d against input planes d-1, d, d+1: the wave's taps whose input
  // plane exists (wave-uniform)
  auto compute = [&](int d, const char* __restrict__ Y, const char* __restrict__ Xm,
                     const char* __restrict__ X0, const char* __restrict__ Xp) __attribute__((always_inline)) {
    const char* __restrict__ xt[4];
    bool ok[4];
#pragma unroll
    for (int lt = 0; lt < 4; ++lt) {
      const int tap = tap0 + lt;
      const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
      const int pl = d + kd - 1;
      ok[lt] = lt < ntap && pl >= 0 && pl < p.D;
      xt[lt] = (kd == 0 ? Xm : kd == 1 ? X0 : Xp) + (kh * WD_HW2 + kw) * ROWB + xb0;
    }
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {                // tile row = 16-pixel k-step
      const uint2 alo = lds_read_tr16(Y + ya0 + ks * 16 * ROWB);
      const uint2 ahi = lds_read_tr16(Y + ya0 + (ks * 16 + 4) * ROWB);
      const uint4 af = make_uint4(alo.x, alo.y, ahi.x, ahi.y);
#pragma unroll
      for (int lt = 0; lt < 4; ++lt) {
        if (!ok[lt]) continue;                       // (wave-uniform)
        const uint2 lo = lds_read_tr16(xt[lt] + ks * WD_HW2 * ROWB);
        const uint2 hi = lds_read_tr16(xt[lt] + (ks * WD_HW2 + 4) * ROWB);
        acc[lt] = mfma32x32x16(af, make_uint4(lo.x, lo.y, hi.x, hi.y), acc[lt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- columns of this workgroup's chunk: c = split + k * R, each marched through d; counted
  // waits from a per-wave ledger (a step: nxi X + 2 dY DMAs)
  __syncthreads();
  int issued = 0;
  for (int c = split; c < ncol; c += R) {
    col_n = c / (tilesH * tilesW);
    const int rr = c - col_n * tilesH * tilesW;
    col_h0 = (rr / tilesW) * WD_T;
    col_w0 = (rr % tilesW) * WD_T;
    issue_x(0);
    issue_y(0);
    issued += nxi + 2;
    const int mark0 = issued;
    int m0 = mark0;                                  // mark after the DMAs of step d's operands
    if (p.D > 1) { issue_x(1); issued += nxi; m0 = issued; }
    vm_wait_dyn(issued - mark0);                     // X(0), dY(0) landed
    if (has_pro) transform_body(xslot(0), 0);
    for (int d = 0; d < p.D; ++d) {
      vm_wait_dyn(issued - m0);                      // X(d+1) (and dY(d)) landed
      if (has_pro && d + 1 < p.D) transform_body(xslot(d + 1), d + 1);
      lds_sync();                                    // visible; step d-1 done by all
      int m1 = m0;
      if (d + 1 < p.D) {                             // operands of step d+1: X(d+2), dY(d+1)
        if (d + 2 < p.D) { issue_x(d + 2); issued += nxi; }
        issue_y(d + 1);
        issued += 2;
        m1 = issued;
      }
      compute(d, yslot(d), xslot(d + 3), xslot(d), xslot(d + 1));
      m0 = m1;
    }
    lds_sync();                                      // the column's planes read by all
  }
  // ---- this wave's taps -> slab rows part[split][co][tap][ci] (32x32 D layout: column n =
  // lane & 31 = ci, row m = 8 (i / 4) + 4 (lane >> 5) + i % 4 = co)
  float* out = p.partial + (long long)split * p.Cout * 27 * p.Cin;
#pragma unroll
  for (int lt = 0; lt < 4; ++lt) {
    if (lt >= ntap) break;
    const int tap = tap0 + lt;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int co = 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
      out[((long long)co * 27 + tap) * p.Cin + ci0 + (lane & 31)] = acc[lt][i];
    }
  }
}

}  // namespace

// planner: 3-D, 32 output channels, whole 32-channel input chunks (concat included), enough
// (chunk, column) work to fill the chip; -> grid (ciChunks x R), splits = R
int conv3d_wgrad_ds_plan(ConvWgradArgs& a, int num_cus) {
  if (a.dims != 3 || a.Cout != 32 || a.C1 % 32 != 0 || a.C2 % 32 != 0 || a.groups > 1 ||
      a.dyy != nullptr)
    return -1;
  const int cmax = a.C1 > a.C2 ? (a.C1 > 32 ? a.C1 : 32) : a.C2;
  if ((long long)a.D * a.H * a.W * cmax * 2 >= (1LL << 31)) return -1;
  const int ncol = a.N * ((a.H + WD_T - 1) / WD_T) * ((a.W + WD_T - 1) / WD_T);
  const int chunks = a.Cin / 32;
  if (chunks < 1 || ncol * chunks < num_cus || chunks > num_cus) return -1;
  a.ciChunks = chunks;
  const int r = num_cus / chunks;
  a.splits = r < ncol ? r : ncol;
  return a.ciChunks * a.splits;
}

void conv3d_wgrad_ds_launch(ConvWgradArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL(conv3d_wgrad_ds_kernel, dim3(grid), dim3(512), WD_SMEM, st, a);
}

}  // namespace ddlpc
