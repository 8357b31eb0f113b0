// Fused backward of the 32 -> 32-channel 3x3 conv whose input is relu(bn1(y)) — the second
// conv of a DoubleConv at the U-Net's 32-channel level (enc1 / dec1 at width/2: ref.py:582
// nn.Conv2d(32, 32, 3, padding=1) after BatchNorm2d + ReLU).  Its two backward GEMMs both
// stream the output gradient dY, and the weight gradient's input a1 = relu(bn1(y)) is formed
// from the same y that the data gradient's BN-backward epilogue needs:
//
//     data gradient  dA[p][ci]      = sum_{tap, co} dY[p + tap][co] W'[ci][tap][co]  (K2)
//                    + BN1-backward partials (sum dyh, sum dyh * xhat) of dA against y
//     weight grad.   dW[co][tap][ci] = sum_p dY[p][co] a1[p + tap][ci]               (K3)
//
// At 32 channels both passes are HBM-bound (conv3x3_wgrad.hip / conv3x3_res.hip notes: the
// operands cost more time than the MFMAs), so ONE kernel reads each 16x16 tile's dY halo and y
// halo once for both: 2 x 1.27 T in + 1 T out instead of 5.5 T (T = one activation tensor).
//
// MI355X design: one persistent 8-wave workgroup per CU (two waves per SIMD), WAVE-
// SPECIALISED — waves 0-3 run the data gradient (each a 64-pixel x 32-channel tile of
// v_mfma_f32_16x16x32_bf16, weights resident in LDS, the resident conv's swizzled halo
// reads), waves 4-7 the weight gradient (each a quarter of the tile's 16 pixel rows, all 9
// taps of v_mfma_f32_32x32x16_bf16 in registers, ds_read_b64_tr_b16 transposed operand reads
// as conv3x3_wgrad.hip's v3).  The two roles issue the same MFMA cycles per tile (72 x 16 and
// 36 x 32), one of each per SIMD.  Tiles are double-buffered: the next tile's two halos
// arrive by LDS-DMA (buffer_load ... lds) while this tile computes; the y halo is turned into
// a1 in place by the lanes that DMA'd it (padding stays zero).  The data-gradient epilogue
// reads y at its output pixels for the BN-backward partials from a raw copy of the halo
// interior the transform keeps in LDS.  Outputs: dA (bf16), one BN-partial row [2][32] per workgroup, one fp32 weight-
// gradient slab [32][9][32] per workgroup (reduced by reduce_rows_scatter).
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

namespace ddlpc {

namespace {

using namespace convlds;

constexpr int B32_TH = 16, B32_TW = 16, B32_HW2 = 18;
constexpr int B32_HALO = 18 * 18;                     // halo pixels of a 16x16 tile
constexpr int B32_ITERS = 3;                          // DMA instructions per wave per halo
constexpr int B32_HBYTES = B32_ITERS * 8 * 1024;      // 1536 pieces (>= 4 x 324) per halo
constexpr int B32_WBYTES = 9 * 32 * ROWB;             // resident dgrad weights (9 taps x 32 rows)
constexpr int B32_YBYTES = 256 * ROWB;               // raw y of the tile's 256 output pixels
constexpr int B32_SMEM = 4 * 32 * 4 + B32_WBYTES + 2 * (2 * B32_HBYTES + B32_YBYTES);

__global__ __launch_bounds__(512, 1) void conv3_bwd32_kernel(Bwd32Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_bnb = reinterpret_cast<float*>(smem);               // BN1 table [4][32]
  char* sW = smem + 4 * 32 * 4;
  char* sH = sW + B32_WBYTES;
  constexpr int STG = 2 * B32_HBYTES + B32_YBYTES;
  auto sDY = [&](int b) { return sH + b * STG; };                      // dY halo (swizzled rows)
  auto sX = [&](int b) { return sH + b * STG + B32_HBYTES; };          // y -> a1 halo
  auto sYi = [&](int b) { return sH + b * STG + 2 * B32_HBYTES; };     // raw y, tile interior

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool dgrad = wave < 4;                                 // wave-uniform role
  const int my_tiles = p.nTiles > (int)blockIdx.x ? (p.nTiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const long long img_px = (long long)p.H * p.W;

  bnb_fill(s_bnb, 32, 0, 32, p.s4, tid, 512);
  // resident data-gradient weights: rows (tap, ci) of 32 co (64 B), swizzled pieces
  {
    const auto rW = make_rsrc(p.Wd, 32u * 9u * 32u * 2u);
    for (int b = wave * 64; b < B32_WBYTES / 16; b += 512) {
      const int e = b + lane;
      const int row = e >> 2;
      const int sub = (e & 3) ^ swz(row);
      const int t = row / 32, ci = row % 32;
      dma16(rW, sW + b * 16, (unsigned)((ci * 9 + t) * 32 + sub * 8) * 2u);
    }
  }

  // ---- per-lane halo DMA geometry: piece e = (i * 8 + wave) * 64 + lane, pixel e >> 2 (its
  // halo row / column recomputed per issue: registers are the wgrad role's budget)
  const int sub_dy = lane & 3;                       // (the swizzle flips it by the row below)
  uint32_t xvalid = 0;                               // in-image y pieces of the tile last issued
  auto tile_geo = [&](int t, int& n, int& h0, int& w0) {
    n = t / (p.tilesH * p.tilesW);
    const int r = t - n * p.tilesH * p.tilesW;
    h0 = (r / p.tilesW) * B32_TH;
    w0 = (r % p.tilesW) * B32_TW;
  };
  auto issue = [&](int t, int buf) {
    int n, h0, w0;
    tile_geo(t, n, h0, w0);
    const auto rdy = make_rsrc(p.dY + n * img_px * 32, (unsigned)(img_px * 64));
    const auto ry = make_rsrc(p.Y + n * img_px * 32, (unsigned)(img_px * 64));
    xvalid = 0;
#pragma unroll
    for (int i = 0; i < B32_ITERS; ++i) {
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;
      const int gh = h0 + px / B32_HW2 - 1, gw = w0 + px % B32_HW2 - 1;
      const bool ok = px < B32_HALO && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W;
      const unsigned pix = (unsigned)(gh * p.W + gw);
      // dY: LDS piece (e & 3) of row px holds source piece (e & 3) ^ swz(px)
      dma16(rdy, sDY(buf) + (i * 8 + wave) * 1024, ok ? (pix * 32 + ((sub_dy ^ swz(px)) << 3)) * 2u : kOOB);
      // y: unswizzled (the weight gradient's transposed reads are conflict-free on 64-B rows)
      dma16(ry, sX(buf) + (i * 8 + wave) * 1024, ok ? (pix * 32 + (sub_dy << 3)) * 2u : kOOB);
      xvalid |= (ok ? 1u : 0u) << i;
    }
  };
  // a1 = relu(bf16(y * scale + shift)) on this lane's own landed y pieces; padding stays 0.  The
  // raw y of interior pixels is kept (the data gradient's BN-backward epilogue needs y itself)
  // (the lane's 8 channels, 8 (lane & 3) .. + 7 — an unswizzled y piece a lane DMAs — read
  // from the BN table per tile rather than held in 16 VGPRs across the loop)
  auto transform = [&](int buf) {
    char* X = sX(buf);
    const float4* kp = reinterpret_cast<const float4*>(s_bnb + opaque_zero() + (lane & 3) * 8);
    const float4 sa = kp[0], sb = kp[1], ha = kp[8], hb = kp[9];
    const float psc[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float psh[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
    uint4 v[B32_ITERS];
#pragma unroll
    for (int i = 0; i < B32_ITERS; ++i) v[i] = *reinterpret_cast<const uint4*>(X + ((i * 8 + wave) * 64 + lane) * 16);
#pragma unroll
    for (int i = 0; i < B32_ITERS; ++i) {
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;
      const int hr = px / B32_HW2, hc = px % B32_HW2;
      if (px < B32_HALO && hr >= 1 && hr <= B32_TH && hc >= 1 && hc <= B32_TW)
        *reinterpret_cast<uint4*>(sYi(buf) + ((hr - 1) * B32_TW + hc - 1) * ROWB + (lane & 3) * 16) = v[i];
    }
#pragma unroll
    for (int i = 0; i < B32_ITERS; ++i) {
      const bool ok = (xvalid >> i) & 1u;
      const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x2_t x = {lo_bf(w[j]), hi_bf(w[j])};
        const f32x2_t y2 = __builtin_elementwise_fma(x, f32x2_t{psc[2 * j], psc[2 * j + 1]},
                                                     f32x2_t{psh[2 * j], psh[2 * j + 1]});
        const uint32_t pk = __builtin_bit_cast(uint32_t, __builtin_convertvector(y2, bf16x2_t));
        const i16x2_t m = __builtin_elementwise_max(__builtin_bit_cast(i16x2_t, pk), i16x2_t{0, 0});
        o[j] = ok ? __builtin_bit_cast(uint32_t, m) : 0u;
      }
      *reinterpret_cast<uint4*>(X + ((i * 8 + wave) * 64 + lane) * 16) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  };

  // The two roles run separate tile loops (same DMA / transform / barrier sequence per
  // tile) so their accumulators are never live together: one kernel, each wave's registers
  // sized for its own role.
  if (dgrad) {
    // ---- data-gradient waves: wave w owns tile pixels 64 w .. 64 w + 63 (MT = 4 rows of 16)
    // x 32 ci (NT = 2); A = weights (rows ci), B = dY halo pixels (K = 32 co)
    const int g = lane >> 4;
    int hp0[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) hp0[mt] = (wave * 4 + mt) * B32_HW2 + (lane & 15);
    float s1[2][4], s2[2][4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) { s1[nt][i] = 0.f; s2[nt][i] = 0.f; }
    auto compute = [&](int t, const char* __restrict__ A, const char* __restrict__ Wc,
                       const char* __restrict__ Yi) {
      int n, h0, w0;
      tile_geo(t, n, h0, w0);
      f32x4_t acc[4][2];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      uint4 xf[2][4], wf[2][2];
      // (the 36 swizzled (row, tap) addresses are recomputed per read — an opaque offset keeps
      // them from being hoisted out of the tile loop into 36 live VGPRs, which spilled)
      auto load = [&](int j, uint4 (&x)[4], uint4 (&w)[2]) __attribute__((always_inline)) {
        const int toff = (j / 3) * B32_HW2 + j % 3 + opaque_zero();
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) x[mt] = lds128(A + lds_off(hp0[mt] + toff, g));
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) w[nt] = lds128(Wc + lds_off(j * 32 + nt * 16 + (lane & 15), g));
      };
      load(0, xf[0], wf[0]);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        if (j + 1 < 9) load(j + 1, xf[(j + 1) & 1], wf[(j + 1) & 1]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma16x16x32(wf[j & 1][nt], xf[j & 1][mt], acc[mt][nt]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // epilogue: dA (bf16, 16-byte channel-pair stores) and the BN1-backward partials of
      // the fp32 values against y (lane: channels nt*16 + 4g .. + 3 of pixel lane & 15)
      const auto rA = make_rsrc(p.dA + n * img_px * 32, (unsigned)(img_px * 64));
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int gh = h0 + wave * 4 + mt, gw = w0 + (lane & 15);
        const bool ok = gh < p.H && gw < p.W;
        uint2 pk[2];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          pk[nt] = make_uint2(pack2(acc[mt][nt][0], acc[mt][nt][1]), pack2(acc[mt][nt][2], acc[mt][nt][3]));
          const BnbC kb = bnb_load(s_bnb, 32, nt * 16 + 4 * g);
          const float d[4] = {ok ? acc[mt][nt][0] : 0.f, ok ? acc[mt][nt][1] : 0.f,
                              ok ? acc[mt][nt][2] : 0.f, ok ? acc[mt][nt][3] : 0.f};
          const uint2 yv = *reinterpret_cast<const uint2*>(Yi + ((wave * 4 + mt) * B32_TW + (lane & 15)) * ROWB +
                                                           (nt * 16 + 4 * g) * 2);
          bnb_accum(d, yv, kb, s1[nt], s2[nt]);
        }
        const uint4 qv = pair16(pk[0], pk[1]);
        unsigned off = ok ? (unsigned)((gh * p.W + gw) * 32 + pair16_ch(lane)) * 2u : kOOB;
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{qv.x, qv.y, qv.z, qv.w}, rA, off, 0, 0);
        __builtin_amdgcn_sched_barrier(0);           // (one row's table / y reads at a time)
      }
    };
    if (my_tiles > 0) issue(blockIdx.x, 0);
    for (int k = 0; k < my_tiles; ++k) {
      const int t = (int)blockIdx.x + k * (int)gridDim.x;
      const int buf = k & 1;
      dma_wait<0>();                                 // this wave's halo DMAs of tile k
      transform(buf);
      lds_sync();                                    // every halo piece visible; tile k-1 done by all
      if (k + 1 < my_tiles) issue(t + (int)gridDim.x, buf ^ 1);
      compute(t, sDY(buf), sW, sYi(buf));
    }
    dma_wait<0>();
    lds_sync();
    // BN-backward partial row: 16 pixel lanes, then the 4 waves in a fixed order
    float* red = reinterpret_cast<float*>(sH);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a1 = row16_sum(s1[nt][i]), a2 = row16_sum(s2[nt][i]);
        if ((lane & 15) == 0) {
          const int c = nt * 16 + 4 * g + i;
          red[(wave * 2) * 32 + c] = a1;
          red[(wave * 2 + 1) * 32 + c] = a2;
        }
      }
    lds_sync();
    if (tid < 64) {
      const int half = tid >> 5, c = tid & 31;
      float v = 0.f;
      for (int w = 0; w < 4; ++w) v += red[(w * 2 + half) * 32 + c];
      p.bnpart[(long long)blockIdx.x * 64 + half * 32 + c] = v;
    }
    lds_sync();
#pragma unroll
    for (int tg = 0; tg < 6; ++tg) lds_sync();       // (the weight-gradient waves' reduction)
  } else {
    // ---- weight-gradient waves: k-steps (tile rows) ks = kw, kw + 4, kw + 8, kw + 12
    const int kw = wave & 3;
    const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
    f32x16_t wacc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) wacc[t][i] = 0.f;
    auto compute = [&](const char* __restrict__ DY, const char* __restrict__ X) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int ks = kk * 4 + kw;                  // tile row = 16-pixel k-step
        uint2 av[2];
        // A = dY^T (rows co, k = the row's 16 pixels) from the swizzled halo interior
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int px = (g4 >> 1) * 8 + 4 * h + q;  // pixel within the tile row
          const int hr = (ks + 1) * B32_HW2 + 1 + px;
          const int piece = ((g4 & 1) * 2 + (pq >> 1)) ^ swz(hr);
          av[h] = lds_read_tr16(DY + hr * ROWB + piece * 16 + (pq & 1) * 8);
        }
        const uint4 af = make_uint4(av[0].x, av[0].y, av[1].x, av[1].y);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int base = (ks + tap / 3) * B32_HW2 + tap % 3;   // halo row of pixel 0 at this tap
          const uint2 lo = lds_read_tr16(X + (base + (g4 >> 1) * 8 + q) * ROWB + (g4 & 1) * 32 + 8 * pq);
          const uint2 hi = lds_read_tr16(X + (base + (g4 >> 1) * 8 + 4 + q) * ROWB + (g4 & 1) * 32 + 8 * pq);
          wacc[tap] = mfma32x32x16(af, make_uint4(lo.x, lo.y, hi.x, hi.y), wacc[tap]);
        }
        __builtin_amdgcn_sched_barrier(0);           // (operand reads one k-step ahead at most)
      }
    };
    if (my_tiles > 0) issue(blockIdx.x, 0);
    for (int k = 0; k < my_tiles; ++k) {
      const int t = (int)blockIdx.x + k * (int)gridDim.x;
      const int buf = k & 1;
      dma_wait<0>();
      transform(buf);
      lds_sync();
      if (k + 1 < my_tiles) issue(t + (int)gridDim.x, buf ^ 1);
      compute(sDY(buf), sX(buf));
    }
    dma_wait<0>();
    lds_sync();
    lds_sync();                                      // (the data-gradient waves' partial row)
    lds_sync();
    // weight-gradient slab: the 4 k-split waves summed in LDS in a fixed order, one tap group
    // at a time (32x32 D layout: column n = lane & 31 = ci, row m = 8 (i / 4) + 4 (lane >> 5)
    // + i % 4 = co)
    float* red = reinterpret_cast<float*>(sH);
    float* out = p.wpart + (long long)blockIdx.x * 32 * 9 * 32;
#pragma unroll
    for (int tg = 0; tg < 3; ++tg) {
      if (kw > 0) {
#pragma unroll
        for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
          for (int i = 0; i < 16; ++i) red[(((kw - 1) * 3 + t3) * 16 + i) * 64 + lane] = wacc[tg * 3 + t3][i];
      }
      lds_sync();
      if (kw == 0) {
#pragma unroll
        for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float v = wacc[tg * 3 + t3][i];
#pragma unroll
            for (int w2 = 1; w2 < 4; ++w2) v += red[(((w2 - 1) * 3 + t3) * 16 + i) * 64 + lane];
            const int co = 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
            out[(co * 9 + tg * 3 + t3) * 32 + (lane & 31)] = v;
          }
      }
      lds_sync();
    }
  }
}

}  // namespace

int conv3_bwd32_grid(int nTiles, int num_cus) { return std::max(1, std::min(nTiles, num_cus)); }

void conv3_bwd32_launch(const Bwd32Args& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL(conv3_bwd32_kernel, dim3(grid), dim3(512), B32_SMEM, st, a);
}

}  // namespace ddlpc
