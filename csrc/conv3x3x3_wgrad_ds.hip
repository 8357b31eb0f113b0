// Weight gradient of the 3-D U-Net's 32-output-channel 3x3x3 convs (enc1.b / dec1.b: 32 -> 32,
// dec1.a: 96 -> 32 at 128^3; BASELINE config #5) — DEPTH-STREAMING, the
// weight-gradient counterpart of conv3x3x3_ds.hip.
//
//     dW[co][kd][kh][kw][ci] = sum_p dY[p][co] X[p + (kd, kh, kw) - 1][ci]
//
// The v3 weight gradient runs a 3-D layer as three depth-tap planes, each a 2-D weight
// gradient over all (n, d) slices: dY and X are each streamed three times.  Here a persistent
// 8-wave workgroup walks work ITEMS = (32-channel input chunk, 16 x 16 (h, w) tile column,
// depth segment) through depth: output-gradient plane d (16 x 16 x 32, no halo) and
// 18 x 18 x 32 input planes arrive by LDS-DMA into rings (X: 5 slots — d-1, d, d+1 in use,
// d+2 and d+3 in flight; dY: 3 slots), two steps ahead of the MFMAs, so dY and X are read
// once and every step accumulates all 27 taps.  The 27 taps are split over the 8 waves (waves
// 0-2 four taps, 3-7 three — per SIMD 7, 7, 7, 6), each tap a 32 x 32 fp32 accumulator of
// v_mfma_f32_32x32x16_bf16 (A = dY^T, B = the shifted X plane, both ds_read_b64_tr_b16
// transposed reads of 64-B pixel rows: conflict-free), A shared by the wave's taps.
// Items are dealt to the workgroups as contiguous ranges of the chunk-major item order (even
// shares whatever the chunk count: dec1.a's 3 x 512 columns are 6 per CU), so a workgroup
// meets at most a few chunks: at a chunk change each wave writes its taps' rows of the
// finished chunk to the workgroup's slab part[wg][co][27 taps][Cin] and restarts from zero;
// rows of chunks it never met are written as zeros (reduce_rows_scatter sums the slabs in a
// fixed order: deterministic).  The X prologue (the previous BatchNorm + ReLU) is applied in
// place by the lanes that DMA'd each piece, its 8 constants per lane in registers.
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

#include <cstdlib>
#include <type_traits>

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
// PF: steps of operands in flight ahead of the MFMAs; ring slots X 3 + PF, dY 1 + PF
template <int PF>
constexpr int wd_smem() { return (3 + PF) * WD_XBYTES + (1 + PF) * WD_YBYTES; }
static_assert(wd_smem<2>() <= 160 * 1024, "LDS budget");

template <int PF>
__global__ __launch_bounds__(512, 1) void conv3d_wgrad_ds_kernel(ConvWgradArgs p) {
  constexpr int WD_XS = 3 + PF, WD_YS = 1 + PF;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sX = smem;
  char* sY = smem + WD_XS * WD_XBYTES;
  auto xslot = [&](int plane) { return sX + ((plane + WD_XS) % WD_XS) * WD_XBYTES; };   // plane >= -1
  auto yslot = [&](int plane) { return sY + (plane % WD_YS) * WD_YBYTES; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesH = p.tilesH, tilesW = p.tilesW, nseg = p.tilesD;
  const int ncol = p.N * tilesH * tilesW;
  const int per_chunk = ncol * nseg;
  const int it_begin = (int)((long long)p.nTiles * blockIdx.x / gridDim.x);
  const int it_end = (int)((long long)p.nTiles * (blockIdx.x + 1) / gridDim.x);
  const long long plane_px = (long long)p.H * p.W;
  const long long vol_px = (long long)p.D * plane_px;

  // ---- the current item's chunk pair k = co chunk * ciChunks + ci chunk: source tensor,
  // channel offset, prologue constants of the input chunk; the output chunk's channel co0
  int cic = -1, Cs = 0, cs0 = 0, co0 = 0;
  const bf16_t* xsrc = nullptr;
  bool has_pro = false;
  float sc[8], sh[8];
  auto set_chunk = [&](int k) {
    cic = k;
    const int c = k % p.ciChunks;
    co0 = (k / p.ciChunks) * 32;
    const int ci0 = c * 32;
    const bool second = ci0 >= p.C1;                 // chunk of X2 (C1 % 32 == 0)
    Cs = second ? p.C2 : p.C1;
    cs0 = second ? ci0 - p.C1 : ci0;
    xsrc = second ? p.X2 : p.X1;
    const float* psc = second ? p.pscale2 : p.pscale;
    const float* psh = second ? p.pshift2 : p.pshift;
    has_pro = psc != nullptr;
    if (has_pro) {                                   // (before any DMA of the item is issued)
      const float4* a = reinterpret_cast<const float4*>(psc + cs0 + (lane & 3) * 8);
      const float4* b = reinterpret_cast<const float4*>(psh + cs0 + (lane & 3) * 8);
      const float4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
      sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
      sh[0] = b0.x; sh[1] = b0.y; sh[2] = b0.z; sh[3] = b0.w; sh[4] = b1.x; sh[5] = b1.y; sh[6] = b1.z; sh[7] = b1.w;
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(sc[j]), "v"(sh[j]));
    }
  };

  // ---- DMA: X plane halo (piece e -> halo pixel e >> 2, channel piece e & 3, unswizzled) and
  // the dY plane tile (piece e -> tile pixel e >> 2)
  const int nxi = (WD_XINSTR - wave + 7) / 8;        // X instructions of this wave (3 or 2)
  uint32_t vmasks = 0;                               // in-image X pieces per ring slot (4 bits)
  int col_n = 0, col_h0 = 0, col_w0 = 0;
  auto issue_x = [&](int d) {
    const auto r = make_rsrc(xsrc + (long long)col_n * vol_px * Cs, (unsigned)(vol_px * Cs * 2));
    char* dst = xslot(d);
    uint32_t valid = 0;
#pragma unroll
    for (int i = 0; i < WD_XITERS; ++i) {
      if (i * 8 + wave >= WD_XINSTR) break;
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;
      const int gh = col_h0 + px / WD_HW2 - 1, gw = col_w0 + px % WD_HW2 - 1;
      const bool ok = px < WD_HALO && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && d >= 0 && d < p.D;
      const unsigned pix = (unsigned)(d * plane_px + gh * p.W + gw);
      dma16(r, dst + (i * 8 + wave) * 1024, ok ? (pix * Cs + cs0 + (lane & 3) * 8) * 2u : kOOB);
      valid |= (ok ? 1u : 0u) << i;
    }
    const int sh4 = 4 * ((d + WD_XS) % WD_XS);
    vmasks = (vmasks & ~(0xfu << sh4)) | (valid << sh4);
  };
  auto issue_y = [&](int d) {
    const auto r = make_rsrc(p.dY + (long long)col_n * vol_px * p.Cout, (unsigned)(vol_px * p.Cout * 2));
    char* dst = yslot(d);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;       // tile pixel 0 .. 255
      const int gh = col_h0 + (px >> 4), gw = col_w0 + (px & 15);
      const bool ok = gh < p.H && gw < p.W;
      dma16(r, dst + (i * 8 + wave) * 1024,
            ok ? ((unsigned)(d * plane_px + gh * p.W + gw) * p.Cout + co0 + (lane & 3) * 8) * 2u : kOOB);
    }
  };
  // (restrict parameter: see compute)
  auto transform_body = [&](char* __restrict__ X, int d) __attribute__((always_inline)) {
    const uint32_t valid = (vmasks >> (4 * ((d + WD_XS) % WD_XS))) & 0xfu;
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

  auto transform = [&](int d) __attribute__((always_inline)) { transform_body(xslot(d), d); };

  // ---- this wave's taps: waves 0-2 own 4 consecutive taps, waves 3-7 three (27 in all)
  const int ntap = wave < 3 ? 4 : 3;
  const int tap0 = wave < 3 ? 4 * wave : 12 + 3 * (wave - 3);
  // transposed-read geometry (the v3 weight gradient's 32-channel layout): 16-lane group
  // g4 = lane >> 4, row q, column group pq; A rows = tile pixels (k), B rows = halo pixels
  // shifted by the tap
  const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int fr0 = ((g4 >> 1) * 8 + q) * ROWB + (g4 & 1) * 32 + 8 * pq;   // + 4 rows: + 4 * ROWB
  f32x16_t acc[4];
  auto zero_acc = [&]() {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  };
  zero_acc();
  // slab rows of this wave's taps for chunk pair k (32x32 D layout: column n = lane & 31 = ci,
  // row m = 8 (i / 4) + 4 (lane >> 5) + i % 4 = co within the output chunk)
  float* slab = p.partial + (long long)blockIdx.x * p.Cout * 27 * p.Cin;
  auto write_rows = [&](int k, bool zeros) {
    const int c = k % p.ciChunks, kco = (k / p.ciChunks) * 32;
    float* __restrict__ base = slab + opaque_zero() + c * 32 + (lane & 31) + (kco + 4 * (lane >> 5)) * 27 * p.Cin;
#pragma unroll
    for (int lt = 0; lt < 4; ++lt) {
      if (lt >= ntap) break;
      const int tap = tap0 + lt;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int co = 8 * (i >> 2) + (i & 3);          // (+ 4 (lane >> 5): in base)
        base[(co * 27 + tap) * p.Cin] = zeros ? 0.f : acc[lt][i];
      }
    }
  };

  // one output-gradient plane d against input planes d-1, d, d+1 (planes outside the volume
  // were DMA'd as zeros: no per-tap tests), NT = the wave's tap count
  // (restrict PARAMETERS: alias scopes, so the compiler does not drain the in-flight LDS-DMA
  // of the next steps before these reads)
  auto compute = [&](const char* __restrict__ Y0, const char* __restrict__ Xm,
                     const char* __restrict__ Xc, const char* __restrict__ Xp, auto ntc)
                     __attribute__((always_inline)) {
    constexpr int NT = decltype(ntc)::value;
    const char* Y = Y0 + fr0;
    const char* xt[NT];
#pragma unroll
    for (int lt = 0; lt < NT; ++lt) {
      const int tap = tap0 + lt;
      const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
      xt[lt] = (kd == 0 ? Xm : kd == 1 ? Xc : Xp) + (kh * WD_HW2 + kw) * ROWB + fr0;
    }
    // register double buffer: the fragments of k-step ks + 1 are read before the MFMAs of ks
    uint4 af[2], bf[2][NT];
    auto load = [&](int ks, int b) __attribute__((always_inline)) {   // tile row = 16-pixel k-step
      const uint2 alo = lds_read_tr16(Y + ks * 16 * ROWB);
      const uint2 ahi = lds_read_tr16(Y + (ks * 16 + 4) * ROWB);
      af[b] = make_uint4(alo.x, alo.y, ahi.x, ahi.y);
#pragma unroll
      for (int lt = 0; lt < NT; ++lt) {
        const uint2 lo = lds_read_tr16(xt[lt] + ks * WD_HW2 * ROWB);
        const uint2 hi = lds_read_tr16(xt[lt] + (ks * WD_HW2 + 4) * ROWB);
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

  // ---- items.  Operand group k of an item starting at depth d0 = {X(d0+k+1), dY(d0+k)}
  // (group -1: X(d0-1), X(d0)); step d needs groups <= d - d0 and issues group d - d0 + PF
  // after its barrier.  Counted waits from a per-wave ledger (issued DMA instructions; mk[j]:
  // the ledger mark after group d - d0 + j, or after the last group issued).
  unsigned long long met = 0;                        // chunk pairs this workgroup accumulated
  int issued = 0;
  for (int it = it_begin; it < it_end; ++it) {
    const int c = it / per_chunk;
    const int rem = it - c * per_chunk;
    const int col = rem / nseg, seg = rem - col * nseg;
    if (c != cic) {
      if (cic >= 0) {
        write_rows(cic, false);
        zero_acc();
        dma_wait<0>();                               // (stores count in vmcnt: keep the ledger exact)
      }
      set_chunk(c);
      met |= 1ull << c;
    }
    col_n = col / (tilesH * tilesW);
    const int rr = col - col_n * tilesH * tilesW;
    col_h0 = (rr / tilesW) * WD_T;
    col_w0 = (rr % tilesW) * WD_T;
    const int d0 = (int)((long long)p.D * seg / nseg), d1 = (int)((long long)p.D * (seg + 1) / nseg);
    auto issue_group = [&](int k) {                  // k >= 0, d0 + k < d1 (X(D): zeros)
      issue_x(d0 + k + 1);
      issued += nxi;
      issue_y(d0 + k);
      issued += 2;
    };
    issue_x(d0 - 1);                                 // (X(-1): zeros)
    issue_x(d0);
    issued += 2 * nxi;
    const int mark_pre = issued;
    int mk[PF];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      if (d0 + j < d1) issue_group(j);
      mk[j] = issued;
    }
    vm_wait_dyn(issued - mark_pre);                  // X(d0-1), X(d0) landed
    if (has_pro) {
      transform(d0 - 1);
      transform(d0);
    }
    for (int d = d0; d < d1; ++d) {
      vm_wait_dyn(issued - mk[0]);                   // X(d+1), dY(d) landed
      if (has_pro) transform(d + 1);
      lds_sync();                                    // visible; step d-1 done by all
      if (d + PF < d1) issue_group(d + PF - d0);
      if (ntap == 4) compute(yslot(d), xslot(d - 1), xslot(d), xslot(d + 1), std::integral_constant<int, 4>{});
      else compute(yslot(d), xslot(d - 1), xslot(d), xslot(d + 1), std::integral_constant<int, 3>{});
#pragma unroll
      for (int j = 0; j + 1 < PF; ++j) mk[j] = mk[j + 1];
      mk[PF - 1] = issued;
    }
    lds_sync();                                      // the item's planes read by all
  }
  if (cic >= 0) write_rows(cic, false);
  for (int c = 0; c < p.ciChunks * (p.Cout / 32); ++c)
    if (!((met >> c) & 1ull)) write_rows(c, true);
}

}  // namespace

// planner: 3-D, whole 32-channel input and output chunks (concat included, <= 64 chunk
// pairs), >= 4 planes per depth segment; items = chunk pairs x tile columns x depth segments
// dealt as even contiguous ranges to one workgroup per CU.  The segment count minimises the busiest
// workgroup's planes (each segment re-loads its two boundary planes)
int conv3d_wgrad_ds_plan(ConvWgradArgs& a, int num_cus) {
  if (a.dims != 3 || a.Cout % 32 != 0 || a.C1 % 32 != 0 || a.C2 % 32 != 0 || a.groups > 1 ||
      a.dyy != nullptr || a.Cin < 32 || a.Cin > 32 * 32 || a.D < 4)
    return -1;
  // >= 64 x 64 planes: at 32^3 (enc3.b, 128 -> 128) the streaming kernel measured 17% slower
  // than v3 (351 vs 409 us, profiles/r5/wgrad3d_ds/m_*_g35.log): 4 tile columns per volume
  if (a.H * a.W < 64 * 64) return -1;
  int cmax = a.C1 > a.C2 ? a.C1 : a.C2;
  if (a.Cout > cmax) cmax = a.Cout;
  if ((long long)a.D * a.H * a.W * cmax * 2 >= (1LL << 31)) return -1;
  const int tilesH = (a.H + WD_T - 1) / WD_T, tilesW = (a.W + WD_T - 1) / WD_T;
  const long long ncol = (long long)a.N * tilesH * tilesW;
  const int chunks = a.Cin / 32;
  if (chunks * (a.Cout / 32) > 64) return -1;        // (the chunk-pair bitmask)
  const long long base = ncol * chunks * (a.Cout / 32);
  int best = 0;
  long long best_cost = -1, best_items = 0;
  for (int nseg = 1; nseg <= 16 && a.D / nseg >= 4; ++nseg) {
    const long long items = base * nseg;
    const long long g = items < num_cus ? items : num_cus;
    const long long per = (items + g - 1) / g;       // items of the busiest workgroup
    const long long cost = per * ((a.D + nseg - 1) / nseg + (nseg > 1 ? 2 : 0));
    if (best_cost < 0 || cost < best_cost) { best_cost = cost; best = nseg; best_items = items; }
  }
  if (best == 0 || best_items < num_cus / 2 || best_items >= (1LL << 31)) return -1;
  // the slab [grid][Cout][27][Cin] (rows of unmet chunk pairs are zeros): <= 512 MB
  const long long g = best_items < num_cus ? best_items : num_cus;
  if (g * a.Cout * 27 * a.Cin * 4 > (512LL << 20)) return -1;
  a.tilesH = tilesH;
  a.tilesW = tilesW;
  a.ciChunks = chunks;
  a.tilesD = best;
  a.nTiles = (int)best_items;
  a.splits = (int)(best_items < num_cus ? best_items : num_cus);
  return a.splits;
}

// (operands one step ahead: two steps measured 1-2% slower, docs/PERF.md round 5)
void conv3d_wgrad_ds_launch(ConvWgradArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL(conv3d_wgrad_ds_kernel<1>, dim3(grid), dim3(512), wd_smem<1>(), st, a);
}

}  // namespace ddlpc
