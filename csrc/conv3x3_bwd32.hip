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
constexpr int B32_INSTR = (B32_HALO * 4 + 63) / 64;  // 21 DMA wave-instructions per halo
constexpr int B32_ITERS = (B32_INSTR + 7) / 8;        // per wave: 3 (waves 0-4) or 2 (5-7)
constexpr int B32_HBYTES = B32_INSTR * 1024;          // 1344 pieces (>= 4 x 324) per halo
constexpr int B32_WBYTES = 9 * 32 * ROWB;             // resident dgrad weights (9 taps x 32 rows)
constexpr int B32_NBUF = 3;                           // halo ring depth
constexpr int B32_SMEM = 4 * 32 * 4 + B32_WBYTES + B32_NBUF * 2 * B32_HBYTES;

__global__ __launch_bounds__(512, 1) void conv3_bwd32_kernel(Bwd32Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_bnb = reinterpret_cast<float*>(smem);               // BN1 table [4][32]
  char* sW = smem + 4 * 32 * 4;
  char* sH = sW + B32_WBYTES;
  constexpr int STG = 2 * B32_HBYTES;
  auto sDY = [&](int b) { return sH + b * STG; };                      // dY halo (swizzled rows)
  auto sX = [&](int b) { return sH + b * STG + B32_HBYTES; };          // y -> a1 halo

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool dgrad = wave < 4;                                 // wave-uniform role
  // tiles t0 + k * tstride.  One group: t0 = blockIdx.x, tstride = gridDim.x.  BN groups
  // (Bwd32Args::groups, a batched window): group-major — workgroup b serves only the tiles of
  // group b / R (R = gridDim.x / groups), so its BN-partial row belongs to that group and the
  // BN1 constants are that group's
  const int NG_ = p.groups > 1 ? p.groups : 1;
  const int R = (int)gridDim.x / NG_;
  const int grp = (int)blockIdx.x / R;
  const int Tg = p.nTiles / NG_;                     // tiles per group
  const int r_blk = (int)blockIdx.x - grp * R;
  const int t0 = grp * Tg + r_blk, tstride = R;
  const int my_tiles = r_blk < Tg ? (Tg - 1 - r_blk) / R + 1 : 0;
  const long long img_px = (long long)p.H * p.W;

  bnb_fill(s_bnb, 32, 0, 32, p.s4 + grp * 4 * 32, tid, 512);
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
  // in-image y pieces of the tile staged in each ring slot, 8 bits per slot (a runtime-indexed
  // array would live in scratch)
  uint32_t vmasks = 0;
  // DMA wave-instructions per halo for this wave (21 over 8 waves: 3 for waves 0-4, 2 after)
  const int nins = (B32_INSTR - wave + 7) / 8;
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
    uint32_t xvalid = 0;
#pragma unroll
    for (int i = 0; i < B32_ITERS; ++i) {
      if (i * 8 + wave >= B32_INSTR) break;          // (wave-uniform)
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;
      const int gh = h0 + px / B32_HW2 - 1, gw = w0 + px % B32_HW2 - 1;
      const bool ok = px < B32_HALO && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W;
      const unsigned pix = (unsigned)(gh * p.W + gw);
      // dY: LDS piece (e & 3) of row px holds source piece (e & 3) ^ swz(halo column) — the
      // swizzle follows the column (bit 2 still flips between lanes 4 pixels apart: conflict-
      // free 16-pixel reads), so a read's XOR depends on the tap's column offset only and the
      // row / tap-row terms of every fragment address are immediates
      dma16(rdy, sDY(buf) + (i * 8 + wave) * 1024,
            ok ? (pix * 32 + ((sub_dy ^ swz(px % B32_HW2)) << 3)) * 2u : kOOB);
      // y: unswizzled (the weight gradient's transposed reads are conflict-free on 64-B rows)
      dma16(ry, sX(buf) + (i * 8 + wave) * 1024, ok ? (pix * 32 + (sub_dy << 3)) * 2u : kOOB);
      xvalid |= (ok ? 1u : 0u) << i;
    }
    vmasks = (vmasks & ~(0xffu << (8 * buf))) | (xvalid << (8 * buf));
  };
  // a1 = relu(bf16(y * scale + shift)) on this lane's own landed y pieces; padding stays 0.  The
  // raw y of interior pixels is kept (the data gradient's BN-backward epilogue needs y itself)
  // (the lane's 8 channels, 8 (lane & 3) .. + 7 — an unswizzled y piece a lane DMAs — read
  // from the BN table per tile rather than held in 16 VGPRs across the loop)
  // (the buffer comes in restrict-qualified so its LDS accesses carry alias scopes: the
  // compiler would otherwise drain the other ring slots' in-flight DMA before them)
  auto transform_body = [&](char* __restrict__ X, int buf) __attribute__((always_inline)) {
    const uint32_t xvalid = (vmasks >> (8 * buf)) & 0xffu;
    const float4* kp = reinterpret_cast<const float4*>(s_bnb + opaque_zero() + (lane & 3) * 8);
    const float4 sa = kp[0], sb = kp[1], ha = kp[8], hb = kp[9];
    const float psc[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float psh[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
    uint4 v[B32_ITERS];
#pragma unroll
    for (int i = 0; i < B32_ITERS; ++i)
      if (i * 8 + wave < B32_INSTR) v[i] = *reinterpret_cast<const uint4*>(X + ((i * 8 + wave) * 64 + lane) * 16);
#pragma unroll
    for (int i = 0; i < B32_ITERS; ++i) {
      if (i * 8 + wave >= B32_INSTR) break;
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
  auto transform = [&](int buf) __attribute__((always_inline)) { transform_body(sX(buf), buf); };

  // ---- the tile loop (each role passes its own work; both run the same DMA / transform /
  // barrier sequence per tile).  Ring of B32_NBUF slots: tile k's halos are issued two tiles
  // ahead; before transforming tile k a wave waits, with a COUNTED vmcnt, only for its own
  // DMAs of tile k — `issued` counts this wave's vector-memory ops in issue order (the DMAs,
  // the data-gradient role's y loads and dA stores), m0 / m1 its count right after the DMAs
  // of tiles k and k+1.  after_sync / work return how many vector-memory ops they issued.
  auto pipeline = [&](auto after_sync, auto work) __attribute__((always_inline)) {
    const int nd = 2 * nins;
    int issued = 0, m0 = 0, m1 = 0;
    if (my_tiles > 0) { issue(t0, 0); issued += nd; m0 = issued; }
    if (my_tiles > 1) { issue(t0 + tstride, 1); issued += nd; m1 = issued; }
    int buf = 0;
    for (int k = 0; k < my_tiles; ++k) {
      const int t = t0 + k * tstride;
      vm_wait_dyn(issued - m0);                      // this wave's halo DMAs of tile k landed
      transform(buf);
      lds_sync();                                    // every halo piece visible; tile k-1 done by all
      issued += after_sync(k, t, buf);
      int m2 = m1;
      if (k + 2 < my_tiles) {                        // into the slot tile k-1 used
        issue(t + 2 * tstride, buf == 0 ? 2 : buf - 1);
        issued += nd;
        m2 = issued;
      }
      issued += work(t, buf);
      m0 = m1;
      m1 = m2;
      buf = buf == 2 ? 0 : buf + 1;
    }
  };

  // The two roles run separate tile loops (same DMA / transform / barrier sequence per
  // tile) so their accumulators are never live together: one kernel, each wave's registers
  // sized for its own role.
  if (dgrad) {
    // ---- data-gradient waves: wave w owns tile pixels 64 w .. 64 w + 63 (MT = 4 rows of 16)
    // x 32 ci (NT = 2); A = weights (rows ci), B = dY halo pixels (K = 32 co)
    const int g = lane >> 4;
    // per-lane byte offsets: dY halo pixel (wave*4 rows down, column c + dw) with its column
    // swizzle, for the three tap columns dw; the weight row c of a 16-row block (rows j*32 +
    // nt*16 + c keep c's bit 2)
    const int c16 = lane & 15;
    int xo[3];
#pragma unroll
    for (int dw = 0; dw < 3; ++dw)
      xo[dw] = (wave * 4 * B32_HW2 + c16 + dw) * ROWB + ((g ^ swz(c16 + dw)) << 4);
    const int wo = c16 * ROWB + ((g ^ swz(c16)) << 4);
    float s1[2][4], s2[2][4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) { s1[nt][i] = 0.f; s2[nt][i] = 0.f; }
    // y at this wave's output pixels for the BN-backward partials: loaded right after the
    // tile's barrier, before the next halo DMA is issued (L2 hits: the halo just landed), so
    // the epilogue's wait for them leaves that DMA in flight
    uint2 ybuf[4][2];
    auto load_y = [&](int t) {
      int n, h0, w0;
      tile_geo(t, n, h0, w0);
      const auto ry = make_rsrc(p.Y + n * img_px * 32, (unsigned)(img_px * 64));
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int gh = h0 + wave * 4 + mt, gw = w0 + (lane & 15);
        const bool ok = gh < p.H && gw < p.W;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          ybuf[mt][nt] = buf_load8(ry, ok ? (unsigned)((gh * p.W + gw) * 32 + nt * 16 + 4 * g) * 2u : kOOB);
      }
    };
    auto compute = [&](int t, const char* __restrict__ A, const char* __restrict__ Wc) {
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
        const int dh = j / 3, dw = j % 3;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) x[mt] = lds128(A + xo[dw] + (mt + dh) * B32_HW2 * ROWB);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) w[nt] = lds128(Wc + wo + (j * 32 + nt * 16) * ROWB);
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
          bnb_accum(d, ybuf[mt][nt], kb, s1[nt], s2[nt]);
        }
        const uint4 qv = pair16(pk[0], pk[1]);
        unsigned off = ok ? (unsigned)((gh * p.W + gw) * 32 + pair16_ch(lane)) * 2u : kOOB;
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{qv.x, qv.y, qv.z, qv.w}, rA, off, 0, 0);
        __builtin_amdgcn_sched_barrier(0);           // (one row's table / y reads at a time)
      }
    };
    pipeline([&](int k, int t, int buf) { load_y(t); (void)k; return 8; },
             [&](int t, int buf) { compute(t, sDY(buf), sW); return 4; });
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
    // per-lane byte offsets of the transposed A reads: halo column 1 + px of the tile row, the
    // chunk XOR of that column (the k-step row term is an immediate)
    int ao[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int px = (g4 >> 1) * 8 + 4 * h + q;      // pixel within the tile row
      ao[h] = (1 + px) * ROWB + ((((g4 & 1) * 2 + (pq >> 1)) ^ swz(1 + px)) << 4) + (pq & 1) * 8;
    }
    // X fragment rows of the lane (+ the tap's halo row: an immediate / SGPR term)
    int xb[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) xb[h] = ((g4 >> 1) * 8 + 4 * h + q) * ROWB + (g4 & 1) * 32 + 8 * pq;
    // the wave's k phase (tile row kw of every 4) folded into both bases: the k-step / tap
    // terms below are immediates.  (The dY halo's column swizzle does not depend on the row.)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ao[h] += kw * B32_HW2 * ROWB;
      xb[h] += kw * B32_HW2 * ROWB;
    }
    // the (k-step, tap) sequence flattened and software-pipelined: the X fragment of step
    // i + LA (and the dY fragment of the next k-step) is read before the MFMA of step i (the
    // per-k-step form waited lgkmcnt(0) at every k-step boundary)
    auto compute = [&](const char* __restrict__ DY, const char* __restrict__ X) {
      constexpr int NI = 4 * 9, LA = 3;
      uint4 af[2], bq[LA + 1];
      auto ldA = [&](int kk, uint4& a) __attribute__((always_inline)) {
        const int ks = kk * 4;                       // tile row = 16-pixel k-step (+ kw: in ao)
        uint2 av[2];
        // A = dY^T (rows co, k = the row's 16 pixels) from the halo interior (column swizzle)
#pragma unroll
        for (int h = 0; h < 2; ++h) av[h] = lds_read_tr16(DY + ao[h] + (ks + 1) * B32_HW2 * ROWB);
        a = make_uint4(av[0].x, av[0].y, av[1].x, av[1].y);
      };
      auto ldB = [&](int i, uint4& b) __attribute__((always_inline)) {
        const int ks = (i / 9) * 4, tap = i % 9;      // (+ kw: in xb)
        const int base = (ks + tap / 3) * B32_HW2 + tap % 3;   // halo row of pixel 0 at this tap
        const uint2 lo = lds_read_tr16(X + base * ROWB + xb[0]);
        const uint2 hi = lds_read_tr16(X + base * ROWB + xb[1]);
        b = make_uint4(lo.x, lo.y, hi.x, hi.y);
      };
      ldA(0, af[0]);
#pragma unroll
      for (int i = 0; i < LA; ++i) ldB(i, bq[i]);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int j = i + LA;
        if (j < NI) {
          if (j % 9 == 0) ldA(j / 9, af[(j / 9) & 1]);
          ldB(j, bq[j % (LA + 1)]);
        }
        wacc[i % 9] = mfma32x32x16(af[(i / 9) & 1], bq[i % (LA + 1)], wacc[i % 9]);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    pipeline([&](int, int, int) { return 0; },
             [&](int, int buf) { compute(sDY(buf), sX(buf)); return 0; });
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

int conv3_bwd32_grid(int nTiles, int num_cus, int groups) {
  if (groups > 1) return groups * std::max(1, std::min(nTiles / groups, num_cus / groups));
  return std::max(1, std::min(nTiles, num_cus));
}

void conv3_bwd32_launch(const Bwd32Args& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL(conv3_bwd32_kernel, dim3(grid), dim3(512), B32_SMEM, st, a);
}

}  // namespace ddlpc
