// 3x3 (2-D) / 3x3x3 (3-D) convolution, stride 1, zero padding 1, as an MFMA implicit GEMM
// over NHWC / NDHWC bf16 activations — the U-Net's K1 (forward) and K2 (data gradient)
// of SURVEY.md §2.5.  Reference ops: nn.Conv2d(k=3, padding=1) in DoubleConv (ref.py:579,582).
//
// GEMM view:  M = output pixels, N = output channels, K = taps x input channels.
//
// Tiling (one workgroup = 4 or 8 waves as WM x WN):
//   * output tile BM pixels (a TD x TH x TW box) x BN channels; each wave owns
//     (16*MT) px x (16*NT) ch = MT x NT tiles of v_mfma_f32_16x16x32_bf16;
//   * K runs over 32-channel chunks; per chunk the (TD+2)(TH+2)(TW+2) input HALO is staged
//     ONCE in LDS and re-read by all 9 (27) taps (vs 9x re-reads of a per-tap im2col);
//   * pipeline: stage = (chunk, 3-tap kernel row).  Both operands arrive by LDS-DMA
//     (buffer_load ... lds, 16 B per lane, no VGPR round trip) into DOUBLE-BUFFERED LDS:
//     the weights of stage s+1 and the halo of chunk c+1 are in flight while stage s
//     computes.  The halo of chunk c+1 is issued at the first stage of chunk c and left in
//     flight across the next barrier with a COUNTED s_waitcnt vmcnt (raw s_barrier, never
//     __syncthreads(), which would drain it);
//   * zero padding is free: out-of-image pixels get an out-of-range buffer offset and the
//     hardware returns zeros; per-image buffer descriptors keep offsets 32-bit;
//   * LDS rows (64 B = one pixel or one weight row of a chunk) carry a 16-B chunk XOR
//     swizzle, chunk ^= 2*((row>>2)&1), applied on the DMA SOURCE address (the DMA writes
//     LDS lane-linearly) and on the ds_read_b128 fragment reads: conflict-free for the
//     gfx950 b128 lane groups {0-3,12-15,20-27}/{4-11,16-19,28-31}/...;
//   * the previous layer's BatchNorm-apply + ReLU (prologue) is applied IN LDS once per
//     chunk after the halo lands (padding stays zero), so BN outputs never round-trip HBM;
//   * two input tensors are one channel-concatenated input (zero-copy
//     torch.cat([up, skip], 1), ref.py:616) — one buffer descriptor per 32-channel chunk;
//   * epilogue: + bias, bf16, tile staged in LDS, 16-B coalesced stores (optionally split
//     across two outputs: the data gradient of a concat conv), and per-channel
//     (sum, sum^2) partials of the fp32 outputs for BatchNorm statistics (K4), one partial
//     row per M tile (deterministic; reduced by bn_finalize).
//
// The data gradient (K2) is this same kernel run on dY with the flipped, transposed
// weights W'[ci][8-t][co] (packed by weight_pack).
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

#include <cstdlib>

// Timing-decomposition builds only (scripts/build_diag.sh; never the shipped library):
// 1 = no fragment LDS reads (MFMAs on register operands), 2 = no operand DMA, 4 = no MFMA,
// 8 = no epilogue stores, 16 = no epilogue of items 0 .. n-2
#ifndef DDLPC_CONV_DIAG
#define DDLPC_CONV_DIAG 0
#endif

namespace ddlpc {

namespace {

using namespace convlds;

template <int DIMS, int WM, int WN, int MT, int NT, int HALO, int NBB>
struct Cfg {
  static constexpr int NW = WM * WN;                            // waves per workgroup (4 or 8)
  static constexpr int NTH = NW * 64;
  static constexpr int BM = WM * MT * 16;
  static constexpr int BN = WN * NT * 16;
  static constexpr int A_ITERS = (HALO / 16 + NW - 1) / NW;     // DMA instrs / wave / chunk
  static constexpr int A_BYTES = A_ITERS * NW * 1024;           // one halo buffer
  static constexpr int B_ITERS = (3 * BN * 4 / 64 + NW - 1) / NW;  // DMA instrs / wave / stage
  static constexpr int B_BYTES = B_ITERS * NW * 1024;           // one weight buffer
  static constexpr int SS_BYTES = 2 * 512 * 4;                  // prologue scale/shift
  // LEAN (accumulator of 32+ tiles per wave): bias and the BN-statistics accumulators live
  // in LDS instead of 48 VGPRs — per-wave-row slots [WM][2][BN], each (wave, column) owned
  // by one lane (no atomics: the order of the sums is fixed) + the bias of the n tile
  // (the BN-backward epilogue variants keep their partial sums in the same LDS slots: LSTAT)
  static constexpr bool LEAN = MT * NT >= 32;
  static constexpr int LEAN_BYTES = (WM * 2 * BN + BN) * 4;
  static constexpr int SMEM = SS_BYTES + LEAN_BYTES + 2 * A_BYTES + NBB * B_BYTES;   // NBB weight buffers
};

// Persistent workgroups walk (m tile, n tile) items; the stage stream runs across item
// boundaries, so the next item's first halo and weights are in flight while the current
// item finishes (and no LDS is needed by the epilogue: results leave straight from the
// accumulators).
//
// Operand roles: the MFMA A operand is the weight tile (rows = output channels) and the B
// operand the pixel tile, so each lane's accumulator holds 4 CONSECUTIVE channels of one
// pixel -> 8-byte bf16x4 stores; BN statistics are reduced with 4 lane shuffles and
// written as one partial row per (m tile, wave row).
// XL: 2-D 16-wide pixel tiles with the halo rows at stride 20 (see HWR) — launcher-chosen when
// TW == 16 and (TH + 2) * 20 halo pixels fit the halo buffer
template <int DIMS, int WM, int WN, int MT, int NT, int HALO, int NBB, int FDB, bool BNB, bool XL>
__global__ __launch_bounds__(WM * WN * 64, WM * WN == 4 ? 2 : 1) void conv3_fwd_kernel(ConvFwdArgs p) {
  using C = Cfg<DIMS, WM, WN, MT, NT, HALO, NBB>;
  static_assert(NBB == 2 || NBB == 3 || (NBB == 4 && DIMS == 2), "2 / 3 weight-stage buffers, or 4 (super-stages)");
  // BN-backward epilogue: 2-D, and not with the counted waits of the 3-deep weight ring
  static_assert(!BNB || (DIMS == 2 && NBB != 3), "BNB: 2-D, NBB 2 or 4");
  constexpr bool FRAG_DB = FDB == 1;            // (FDB 2: rolling pipeline, pipe_taps)
  constexpr int BM = C::BM, BN = C::BN;
  constexpr int NG = DIMS == 2 ? 3 : 9;           // (kd, r) kernel rows per chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_scale = reinterpret_cast<float*>(smem);
  float* s_shift = s_scale + 512;
  char* base = smem + C::SS_BYTES + C::LEAN_BYTES;
  constexpr bool LEAN = C::LEAN;                    // bias / statistics in LDS
  // (3-D XL: 16 x 4 (w, h) tile planes — TH = 4, launcher-enforced with TW == 16)
  static_assert(!LEAN || XL, "LEAN tiles use the XL addressing");
  constexpr bool LSTAT = C::LEAN || BNB;           // bias + statistics / BN-backward partials in LDS
  float* s_red = reinterpret_cast<float*>(smem + C::SS_BYTES);    // LSTAT: [WM][2][BN]
  float* s_bias = s_red + WM * 2 * BN;                             // LSTAT: [BN]
  static_assert(!LSTAT || C::LEAN_BYTES > 0, "LDS slots for the statistics");
  // double buffers addressed arithmetically (a runtime-indexed pointer array would spill)
  auto sA = [&](int b) { return base + b * C::A_BYTES; };
  auto sB = [&](int b) { return base + 2 * C::A_BYTES + b * C::B_BYTES; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN;
  const int wn = wave % WN;
  const int HW2 = p.TW + 2, HH2 = p.TH + 2;
  // halo row STRIDE in LDS rows: XL tiles (TW = 16, 18-pixel halo rows) pad it to 20 — 20 is
  // 4 mod 8, so bit 2 of a halo row index (the chunk swizzle) is bit 2 of its column XOR the
  // parity of its halo row, and a fragment address is a per-lane register XOR a wave-uniform
  // term plus an immediate (one VALU op per fragment instead of six); columns 18-19 are never
  // read (DMA'd as zeros)
  const int HWR = XL ? 20 : HW2;
  const int halo = (DIMS == 3 ? p.TD + 2 : 1) * HH2 * HWR;
  const long long img_px = (long long)p.D * p.H * p.W;
  // channel-chunk split (small layers); the BN-backward epilogue variant is launched with
  // ksplit 1 only (launch_mode), so its epilogue has no split-K / split-output branches
  const int KS = BNB ? 1 : p.ksplit;
  // M-tile walk: workgroup b = blockIdx.x / (KS * nTilesN) serves M tiles m0 + k * Gs.  One
  // group: m0 = b, Gs = the workgroups per n tile.  BN groups (ConvFwdArgs::groups): group-
  // major — b = grp * Gs + r serves tiles grp * Mg + r + k * Gs of its own group only
  const int Q = KS * p.nTilesN;
  const int NG_ = p.groups > 1 ? p.groups : 1;
  const int Gs = (int)gridDim.x / (Q * NG_);
  const int Mg = p.nTilesM / NG_;                  // M tiles per group
  const int grp = (int)blockIdx.x / Q / Gs;
  const int r_blk = (int)blockIdx.x / Q % Gs;
  const int my_items = r_blk < Mg ? (Mg - 1 - r_blk) / Gs + 1 : 0;
  const int nchunks = ((p.Cin + BK - 1) / BK) / KS;  // chunks per item (KS divides the total)
  const int spi = nchunks * NG;                   // stages per item
  const int S = my_items * spi;

  const bool has_pro = p.pscale != nullptr;
  const bool has_pro2 = p.pscale2 != nullptr;         // deferred skip: X2 channels at C1 + c
  if (has_pro) {
    const float* psc = p.pscale + grp * p.gstride;    // (BN groups: this workgroup's group)
    const float* psh = p.pshift + grp * p.gstride;
    for (int c = tid; c < p.C1; c += C::NTH) { s_scale[c] = psc[c]; s_shift[c] = psh[c]; }
  }
  if (has_pro2)
    for (int c = tid; c < p.C2; c += C::NTH) { s_scale[p.C1 + c] = p.pscale2[c]; s_shift[p.C1 + c] = p.pshift2[c]; }

  const auto rW = make_rsrc(p.Wt, (unsigned)((long long)p.Cout * p.taps * p.CinW * 2));

  struct Item { int n_img, d0, h0, w0, co0, ks; };
  // work item k of this workgroup: gridDim.x is a multiple of KS * nTilesN (launcher), so its
  // channel split ks and n tile are the block's own and its M tile is m0 + k * Gs: the item
  // geometry comes from carry-walkers (one add-and-carry step per item) instead of five
  // runtime integer divisions per call; one walker per consumer (halo issue, epilogue, BNB y
  // loads), each visiting the items in order
  const int ks_blk = (int)blockIdx.x % KS;
  const int co0_item = (int)blockIdx.x / KS % p.nTilesN * BN;
  struct Walk { int k, tw, th, td, n; };
  int g_w, g_h, g_d, g_n;
  {
    int q = Gs;
    g_w = q % p.tilesW; q /= p.tilesW;
    g_h = q % p.tilesH; q /= p.tilesH;
    g_d = q % p.tilesD; g_n = q / p.tilesD;
  }
  Walk w0;
  {
    int m = grp * Mg + r_blk;
    w0.k = 0;
    w0.tw = m % p.tilesW; m /= p.tilesW;
    w0.th = m % p.tilesH; m /= p.tilesH;
    w0.td = m % p.tilesD; w0.n = m / p.tilesD;
  }
  auto walk_item = [&](Walk& w, int k) __attribute__((always_inline)) {
    while (w.k < k) {
      w.tw += g_w;
      const int c1 = w.tw >= p.tilesW ? 1 : 0;
      w.tw -= c1 * p.tilesW;
      w.th += g_h + c1;
      const int c2 = w.th >= p.tilesH ? 1 : 0;
      w.th -= c2 * p.tilesH;
      w.td += g_d + c2;
      const int c3 = w.td >= p.tilesD ? 1 : 0;
      w.td -= c3 * p.tilesD;
      w.n += g_n + c3;
      ++w.k;
    }
    Item it;
    it.ks = ks_blk;
    it.n_img = w.n;
    it.d0 = w.td * p.TD; it.h0 = w.th * p.TH; it.w0 = w.tw * p.TW;
    it.co0 = co0_item;
    return it;
  };
  Walk wA = w0, wE = w0, wY = w0;
  // ---- per-lane DMA geometry.  Element e = (i*NW + wave)*64 + lane of a halo / weight
  // buffer holds row e >> 2 = (i*NW + wave)*16 + (lane >> 2), so the swizzled 8-channel
  // sub-chunk ((e & 3) ^ swz(row)) * 8 is the same for every i (swz depends on bit 2 of the
  // row = bit 4 of the lane): one register, and the halo position of piece i is recomputed
  // once per item (set_item_pixels) instead of held in 3 x A_ITERS registers (VGPR budget of
  // two waves per SIMD: the held geometry made the BM-512 / BN-backward variants spill to
  // scratch, and every scratch reload waits vmcnt(0) on the in-flight operand DMA)
  const int sub8 = ((lane & 3) ^ (((lane >> 4) & 1) << 1)) << 3;
  int a_pix[C::A_ITERS];       // in-image pixel of the item last issued, -1 = zero padding
#pragma unroll
  for (int i = 0; i < C::A_ITERS; ++i) a_pix[i] = -1;
  // B: row (tap-in-group, channel) -> byte offset without the (chunk, group) term
  // every item of a block has the same n tile (launcher: grid % (KS * nTilesN) == 0)
  const int co0_blk = (int)blockIdx.x / KS % p.nTilesN * BN;
  // BNB (a data gradient: no prologue, so the prologue constants' LDS holds the BN-backward
  // table [4][BN]; published by the first stage barrier)
  if constexpr (BNB) bnb_fill(s_scale, BN, co0_blk, p.Cout, p.bnb_s4 + grp * p.gstride, tid, C::NTH);
  int b_off[C::B_ITERS];
#pragma unroll
  for (int i = 0; i < C::B_ITERS; ++i) {
    const int row = ((i * C::NW + wave) * 64 + lane) >> 2;
    const int tl = row / BN, col = row % BN;
    const int co = co0_blk + col;
    b_off[i] = (tl < 3 && co < p.Cout) ? ((co * p.taps + tl) * p.CinW + sub8) * 2 : -1;
  }
  int a_item = -1;                 // item whose pixels a_pix currently holds
  int a_nimg = 0;
  auto set_item_pixels = [&](int k) {
    const Item it = walk_item(wA, k);
    a_item = k;
    a_nimg = it.n_img;
#pragma unroll
    for (int i = 0; i < C::A_ITERS; ++i) {
      // (opaque_zero: recomputed per item, not hoisted into 2 x A_ITERS live registers)
      const int px = (i * C::NW + wave) * 16 + (lane >> 2) + (XL ? opaque_zero() : 0);
      const int hw = px % HWR, hh = (px / HWR) % HH2;
      const int hd = DIMS == 3 ? px / (HWR * HH2) : 1;
      const int gw = it.w0 + hw - 1, gh = it.h0 + hh - 1, gd = it.d0 + hd - 1;
      const bool ok = px < halo && hw < HW2 && gw >= 0 && gw < p.W && gh >= 0 && gh < p.H && gd >= 0 && gd < p.D;
      a_pix[i] = ok ? (gd * p.H + gh) * p.W + gw : -1;
    }
  };
  auto chunk0_of = [&](int) { return ks_blk * nchunks; };     // (the block's own split)
  auto issue_A = [&](int k, int chunk, int buf) {
    if (k != a_item) set_item_pixels(k);
    const int cbase = (chunk0_of(k) + chunk) * BK;
    const bool second = cbase >= p.C1;              // chunk served by X2 (C1 % 32 == 0)
    const int Cs = second ? p.C2 : p.C1;
    const int c0 = second ? cbase - p.C1 : cbase;
    const bf16_t* src = second ? p.X2 : p.X1;
    const auto r = make_rsrc(src + a_nimg * img_px * Cs, (unsigned)(img_px * Cs * 2));
#pragma unroll
    for (int i = 0; i < C::A_ITERS; ++i) {
      const int c8 = c0 + sub8;
      unsigned off = (a_pix[i] >= 0 && c8 < Cs) ? (unsigned)(a_pix[i] * Cs + c8) * 2u : kOOB;
      if constexpr (!(DDLPC_CONV_DIAG & 2)) dma16(r, sA(buf) + (i * C::NW + wave) * 1024, off);
    }
  };
  auto issue_B = [&](int k, int chunk_local, int grp, int buf) {
    const int chunk = chunk0_of(k) + chunk_local;
    const int soff = (grp * 3 * p.CinW + chunk * BK) * 2;
#pragma unroll
    for (int i = 0; i < C::B_ITERS; ++i) {
      const bool ok = b_off[i] >= 0 && chunk * BK + sub8 < p.CinW;
      if constexpr (!(DDLPC_CONV_DIAG & 2)) dma16(rW, sB(buf) + (i * C::NW + wave) * 1024, ok ? (unsigned)(b_off[i] + soff) : kOOB);
    }
  };
  // prologue BN+ReLU applied in LDS on the landed halo (padding stays zero); a_pix holds
  // this chunk's item (the next item's pixels are only loaded after this transform)
  // (the halo buffer goes in as a restrict-qualified parameter so its LDS writes carry alias
  // scopes: the compiler would otherwise drain the in-flight weight DMA before them)
  auto transform_body = [&](int k, int chunk, char* __restrict__ Abuf) __attribute__((always_inline)) {
    const int cbase = (chunk0_of(k) + chunk) * BK;
    const bool x2ch = cbase >= p.C1;                // X2 channels: prologue only if deferred
    if (x2ch ? !has_pro2 : !has_pro) return;
    const int climit = x2ch ? p.Cin : p.C1;
    // batched form (<= 6 pieces per lane — larger 3-D halos would spill):
    // the lane's 8-channel group is the same in every piece, so its 16 constants are read
    // once; all piece reads issue before the math, and padding is re-zeroed by a select
    // instead of a branch around each piece
    if (C::A_ITERS <= 6) {
      const int c8 = cbase + sub8;
      const bool cok = c8 < climit;
      const float4* scp = reinterpret_cast<const float4*>(s_scale + (cok ? c8 : 0));
      const float4* shp = reinterpret_cast<const float4*>(s_shift + (cok ? c8 : 0));
      const float4 sa = scp[0], sb = scp[1], ha = shp[0], hb = shp[1];
      const float scf[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
      const float shf[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
      constexpr int NI = C::A_ITERS <= 6 ? C::A_ITERS : 1;
      uint4 v[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i)
        v[i] = *reinterpret_cast<const uint4*>(Abuf + ((i * C::NW + wave) * 64 + lane) * 16);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const bool ok = cok && a_pix[i] >= 0;
        const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x2_t x = {lo_bf(w[j]), hi_bf(w[j])};
          const f32x2_t sc2 = {scf[2 * j], scf[2 * j + 1]};
          const f32x2_t sh2 = {shf[2 * j], shf[2 * j + 1]};
          const f32x2_t y2 = __builtin_elementwise_fma(x, sc2, sh2);
          const uint32_t pk = __builtin_bit_cast(uint32_t, __builtin_convertvector(y2, bf16x2_t));
          const i16x2_t m = __builtin_elementwise_max(__builtin_bit_cast(i16x2_t, pk), i16x2_t{0, 0});
          o[j] = ok ? __builtin_bit_cast(uint32_t, m) : 0u;
        }
        *reinterpret_cast<uint4*>(Abuf + ((i * C::NW + wave) * 64 + lane) * 16) = make_uint4(o[0], o[1], o[2], o[3]);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < C::A_ITERS; ++i) {
      const int e = (i * C::NW + wave) * 64 + lane;    // same element this lane DMA'd
      const int c8 = cbase + sub8;
      if (c8 < climit && a_pix[i] >= 0) {
        uint4* q = reinterpret_cast<uint4*>(Abuf + e * 16);
        float f[8];
        unpack8(*q, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], s_scale[c8 + j], s_shift[c8 + j]), 0.0f);
        *q = pack8(f);
      }
    }
  };
  auto transform_A = [&](int k, int chunk, int buf) __attribute__((always_inline)) {
    transform_body(k, chunk, sA(buf));
  };

  // ---- per-lane fragment geometry (item independent)
  const int g = lane >> 4;
  // tile pixel -> (w, h, d) without integer division: TW is 8 or 16 and TW * TH (2-D) /
  // TW * TH * TD with TH = 4 (3-D) is the tile (bindings.cpp conv_tile)
  const int tw_sh = p.TW == 16 ? 4 : 3;
  auto pix_geo = [&](int pix, int& pw, int& ph, int& pd) __attribute__((always_inline)) {
    pw = pix & (p.TW - 1);
    ph = DIMS == 3 ? (pix >> tw_sh) & 3 : pix >> tw_sh;
    pd = DIMS == 3 ? pix >> (tw_sh + 2) : 0;
  };
  // (XL: 16-wide pixel tiles, TW == 16 — launcher-enforced — so the halo pixel of tile mt
  // is hp_lean + mt * HWR: one register instead of MT.  Its fragment byte offsets for tap
  // column dw: xo_lean[dw] ^ (32 * parity of the halo row) + halo row * HWR * 64)
  const int hp_lean = (wm * MT) * HWR + (lane & 15);
  int xo_lean[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int col = (lane & 15) + dw;               // (2-D: halo row wm * MT is even, no parity term;
    xo_lean[dw] = ((DIMS == 2 ? wm * MT : 0) * HWR + col) * ROWB + ((g ^ swz(col)) << 4);   // 3-D: row in xload)
  }
  int hp0[XL ? 1 : MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int pix = wm * (MT * 16) + mt * 16 + (lane & 15);
    const int pw = pix % p.TW;
    const int ph = (pix / p.TW) % p.TH;
    const int pd = DIMS == 3 ? pix / (p.TW * p.TH) : 0;
    if (!XL) hp0[XL ? 0 : mt] = (pd * HH2 + ph) * HW2 + pw;
  }

  f32x4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // BN statistics accumulate in registers across all items of this workgroup: every item
  // of a workgroup has the same n tile (grid % nTilesN == 0, enforced by the launcher)
  float s1[NT][4], s2[NT][4];                        // (LSTAT: unused)
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) { s1[nt][i] = 0.f; s2[nt][i] = 0.f; }
  if constexpr (LSTAT) {
    // published to every wave by the first stage barrier
    for (int i = tid; i < WM * 2 * BN; i += C::NTH) s_red[i] = 0.f;
    for (int i = tid; i < BN; i += C::NTH) {
      const int co = co0_blk + i;
      s_bias[i] = (p.bias != nullptr && co < p.Cout) ? p.bias[co] : 0.0f;
    }
  }

  // bias of this block's channel tile, loaded once (a global load inside the epilogue would
  // make the compiler wait vmcnt(0) — on in-flight stores and DMA — before every use)
  float bias_r[NT][4];                               // (LSTAT: unused, bias in LDS)
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0_blk + wn * (NT * 16) + nt * 16 + 4 * g + i;
      bias_r[nt][i] = (!LSTAT && p.bias != nullptr && co < p.Cout) ? p.bias[co] : 0.0f;
    }

  // ---- epilogue of item k straight from the accumulators:
  // lane holds channels co..co+3 (co = co0 + wn*NT*16 + nt*16 + 4*(lane>>4)) of pixel
  // (wm*MT*16 + mt*16 + (lane&15)) of the tile
  // Stores are buffer stores with an out-of-range offset for masked lanes: every wave issues
  // exactly EPI_STORES per epilogue (no exec branches), so counted vmcnt waits stay exact.
  // stores per epilogue: single bf16 output -> 16-byte stores of channel-tile pairs (pair16);
  // split output / split-K fp32 partials -> one store per tile
  static_assert(NT % 2 == 0, "channel tiles come in pairs");
  // (a split output takes pairs too when it splits at a 32-channel boundary: each pair lies
  // wholly in one output)
  const bool pairs = BNB || (KS == 1 && (p.Y2 == nullptr || p.Co1 % 32 == 0));   // (BNB: single output)
  const int EPI_STORES = pairs ? MT * NT / 2 : MT * NT;
  // BNB: y at an item's output pixels, loaded into VGPRs at the item's last stage (after that
  // stage's DMA) and consumed by its epilogue after the next stage's full wait
  uint2 ybuf[MT][NT];
  auto issue_Y = [&](int kk) __attribute__((always_inline)) {
    const Item it = walk_item(wY, kk);
    const auto ry = make_rsrc(p.bnb_y + it.n_img * img_px * p.Cout, (unsigned)(img_px * p.Cout * 2));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int pix = wm * (MT * 16) + mt * 16 + (lane & 15);
      int pw, ph, pd;
      pix_geo(pix, pw, ph, pd);
      const int gw = it.w0 + pw, gh = it.h0 + ph;
      const bool valid = gw < p.W && gh < p.H;
      const int lpix = gh * p.W + gw;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int co = it.co0 + wn * (NT * 16) + nt * 16 + 4 * g;
        ybuf[mt][nt] = buf_load8(ry, valid && co < p.Cout ? (unsigned)(lpix * p.Cout + co) * 2u : kOOB);
      }
    }
  };
  auto epilogue = [&](int k) __attribute__((always_inline)) {
    const Item it = walk_item(wE, k);
    const int Co2 = p.Cout - p.Co1;
    const auto r1 = KS > 1 ? make_rsrc(p.part + ((long long)it.ks * p.npix + (long long)it.n_img * img_px) * p.Cout,
                                       (unsigned)(img_px * p.Cout * 4))
                           : make_rsrc(p.Y1 + it.n_img * img_px * p.Co1, (unsigned)(img_px * p.Co1 * 2));
    const auto r2 = make_rsrc(p.Y2 != nullptr ? p.Y2 + it.n_img * img_px * Co2 : p.Y1,
                              p.Y2 != nullptr ? (unsigned)(img_px * Co2 * 2) : 0u);
    // pass 1, channel tiles outer: the BNB constants of one tile are read once (the scheduler
    // barrier below keeps the next tile's reads from being hoisted: VGPR pressure)
    uint2 pkv[MT][NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int co = it.co0 + wn * (NT * 16) + nt * 16 + 4 * g;
      BnbC kb;
      if constexpr (BNB) kb = bnb_load(s_scale, BN, wn * (NT * 16) + nt * 16 + 4 * g);
      // LEAN: this tile's bias from LDS, statistics of its 4 channels summed over the mt
      // tiles here, then over the 16 pixel lanes into the wave's LDS slot below
      float bl[4] = {0.f, 0.f, 0.f, 0.f}, t1[4] = {0.f, 0.f, 0.f, 0.f}, t2[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (LSTAT && !BNB) {                    // (BNB: no bias)
        const float4 b4 = *reinterpret_cast<const float4*>(s_bias + opaque_zero() + wn * (NT * 16) + nt * 16 + 4 * g);
        bl[0] = b4.x; bl[1] = b4.y; bl[2] = b4.z; bl[3] = b4.w;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int pix = wm * (MT * 16) + mt * 16 + (lane & 15);
        int pw, ph, pd;
        pix_geo(pix, pw, ph, pd);
        const int gw = it.w0 + pw, gh = it.h0 + ph, gd = it.d0 + pd;
        const bool valid = gw < p.W && gh < p.H && gd < p.D;
        const int lpix = (gd * p.H + gh) * p.W + gw;        // pixel within the image (32-bit)
        const bool ok = valid && co < p.Cout;
        if (KS > 1) {            // split-K partial: fp32 [ks][pixel][Cout], finalized later
          unsigned off = ok ? (unsigned)(lpix * p.Cout + co) * 4u : kOOB;
          asm volatile("" : "+v"(off));
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4_t{__float_as_uint(acc[mt][nt][0]), __float_as_uint(acc[mt][nt][1]),
                      __float_as_uint(acc[mt][nt][2]), __float_as_uint(acc[mt][nt][3])}, r1, off, 0, 0);
          acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          continue;
        }
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[mt][nt][i] + (BNB ? 0.f : LSTAT ? bl[i] : bias_r[nt][i]);
        const uint2 pk = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        pkv[mt][nt] = pk;
        if (!pairs) {
          // the 16-channel tile lies in one output (Co1 % 16 == 0): wave-uniform descriptor
          const bool in1 = it.co0 + wn * (NT * 16) + nt * 16 < p.Co1 || p.Y2 == nullptr;
          unsigned off = ok ? (unsigned)(in1 ? lpix * p.Co1 + co : lpix * Co2 + co - p.Co1) * 2u : kOOB;
          asm volatile("" : "+v"(off));
          __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk.x, pk.y}, in1 ? r1 : r2, off, 0, 0);
        }
        if constexpr (BNB) {
          const float d[4] = {ok ? v[0] : 0.f, ok ? v[1] : 0.f, ok ? v[2] : 0.f, ok ? v[3] : 0.f};
          bnb_accum_y(d, ybuf[mt][nt], kb, t1, t2);
        } else if (ok) {
          // statistics of the fp32 outputs (before the bf16 store; ops.h ConvFwdArgs::stats)
          const float r0 = v[0], q1 = v[1], q2 = v[2], q3 = v[3];
          if constexpr (LSTAT) {
            t1[0] += r0; t2[0] += r0 * r0;
            t1[1] += q1; t2[1] += q1 * q1;
            t1[2] += q2; t2[2] += q2 * q2;
            t1[3] += q3; t2[3] += q3 * q3;
          } else {
            s1[nt][0] += r0; s2[nt][0] += r0 * r0;
            s1[nt][1] += q1; s2[nt][1] += q1 * q1;
            s1[nt][2] += q2; s2[nt][2] += q2 * q2;
            s1[nt][3] += q3; s2[nt][3] += q3 * q3;
          }
        }
        acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (LSTAT) {
        if (BNB || (p.stats != nullptr && KS == 1)) {   // (BNB: the stats rows always exist)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float a1 = t1[i], a2 = t2[i];
            a1 = row16_sum(a1); a2 = row16_sum(a2);
            // BNB: t2 summed dyh * y; sum dyh * xhat = invstd * that - mean * invstd * sum dyh
            if constexpr (BNB) a2 = bnb_xhat_sum(kb, i, a1, a2);
            if ((lane & 15) == 0) {
              const int col = wn * (NT * 16) + nt * 16 + 4 * g + i;
              s_red[(2 * wm) * BN + col] += a1;       // one owner lane per (wave, column)
              s_red[(2 * wm + 1) * BN + col] += a2;
            }
          }
        }
      }
      if constexpr (BNB) __builtin_amdgcn_sched_barrier(0);
    }
    if (!pairs) return;
    // pass 2: 16-byte stores of channel-tile pairs
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int pix = wm * (MT * 16) + mt * 16 + (lane & 15);
      int pw, ph, pd;
      pix_geo(pix, pw, ph, pd);
      const int gw = it.w0 + pw, gh = it.h0 + ph, gd = it.d0 + pd;
      const bool valid = gw < p.W && gh < p.H && gd < p.D;
      const int lpix = (gd * p.H + gh) * p.W + gw;
#pragma unroll
      for (int np = 0; np < NT / 2; ++np) {
        const uint4 q = pair16(pkv[mt][2 * np], pkv[mt][2 * np + 1]);
        const int co = it.co0 + wn * (NT * 16) + np * 32 + pair16_ch(lane);
        const bool in1 = p.Y2 == nullptr || it.co0 + wn * (NT * 16) + np * 32 < p.Co1;   // wave-uniform
        unsigned off = valid && co < p.Cout ? (unsigned)(in1 ? lpix * p.Co1 + co : lpix * Co2 + co - p.Co1) * 2u
                                            : kOOB;
        asm volatile("" : "+v"(off));
        if constexpr (!(DDLPC_CONV_DIAG & 8))
          __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{q.x, q.y, q.z, q.w}, in1 ? r1 : r2, off, 0, 0);
      }
    }
  };

  // ---- compute one stage: the 3 taps of kernel row (kd, r).  The operand pointers are
  // restrict-qualified so the LDS reads carry alias scopes and the compiler does not make
  // them wait (vmcnt) for the NEXT stage's in-flight LDS-DMA; vmcnt is managed by hand.
  //
  // FDB == 2: ROLLING fragment pipeline.  Step s = (tap tt, pixel tile mt) runs the NT MFMAs
  // of pixel fragment s against the tap's NT weight fragments; pixel fragments rotate through
  // XD register sets, each read XD-1 steps (>= 96 MFMA cycles) before its use, and a tap's
  // weight fragments are read one tap ahead.  Live fragment registers: 4 (XD + 2 NT) instead
  // of the whole-tap double buffer's 8 (MT + NT) — 64 fewer with the BM-512 tiles (MT = 8),
  // which otherwise spill to scratch (a scratch reload waits vmcnt(0), i.e. on the operand
  // DMA in flight for the next stage)
  constexpr int XD = 1 + 12 / NT;     // (6 for BM-512: +0.1%, noise — profiles/r6/cfg5_xd_ab_r6d.json)
  auto pipe_taps = [&](auto TTc, const char* __restrict__ A0, const char* __restrict__ B0, int off0,
                       const char* __restrict__ A1, const char* __restrict__ B1, int off1, auto&& hook)
      __attribute__((always_inline)) {
    constexpr int TT = decltype(TTc)::value;
    constexpr int NS = TT * MT;
    auto xload = [&](int s) __attribute__((always_inline)) {
      const int tt = s / MT, mt = s % MT;
      if constexpr (DDLPC_CONV_DIAG & 1) return make_uint4(lane, lane + 1, 0u, 0u);
      const char* A = tt < 3 ? A0 : A1;
      if constexpr (XL && DIMS == 2) {
        // off = the kernel row r (XL call sites): halo row wm*MT + mt + r, wm*MT even
        const int r = tt < 3 ? off0 : off1;
        const int par = ((mt & 1) ^ r) & 1;
        return lds128(A + ((xo_lean[tt % 3] ^ (par << 5)) + (mt + r) * HWR * ROWB));
      }
      if constexpr (XL && DIMS == 3) {
        // off = kd * HH2 + r (XL call sites); the tile's pixel group q = wm*MT + mt is the
        // (d, h) row pair (q >> 2, q & 3) of the 16 x 4 plane tiles: halo (d, h) row
        // hr = (q >> 2) * HH2 + (q & 3) + off (wave-uniform), parity = bit 2 term of its rows
        const int q = wm * MT + mt;
        const int hr = (q >> 2) * HH2 + (q & 3) + (tt < 3 ? off0 : off1);
        return lds128(A + ((xo_lean[tt % 3] ^ ((hr & 1) << 5)) + hr * HWR * ROWB));
      }
      const int row = hp0[XL ? 0 : mt] + (tt < 3 ? off0 : off1) + tt % 3;
      return lds128(A + lds_off(row, g));
    };
    auto wload = [&](int tt, uint4 (&wf)[NT]) __attribute__((always_inline)) {
      const char* B = tt < 3 ? B0 : B1;
      if constexpr (DDLPC_CONV_DIAG & 1) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) wf[nt] = make_uint4(lane + nt, lane, 0u, 0u);
        return;
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        wf[nt] = lds128(B + lds_off((tt % 3) * BN + wn * (NT * 16) + nt * 16 + (lane & 15), g));
    };
    uint4 xf[XD], wf[2][NT];
    wload(0, wf[0]);
#pragma unroll
    for (int s = 0; s < XD - 1; ++s)
      if (s < NS) xf[s] = xload(s);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int tt = s / MT, mt = s % MT;
      if (s + XD - 1 < NS) xf[(s + XD - 1) % XD] = xload(s + XD - 1);
      if (mt == 0 && tt + 1 < TT) wload(tt + 1, wf[(tt + 1) & 1]);
      if (mt == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        if constexpr (!(DDLPC_CONV_DIAG & 4)) acc[mt][nt] = mfma16x16x32(wf[tt & 1][nt], xf[s % XD], acc[mt][nt]);
      if (mt == MT - 1) {
        __builtin_amdgcn_s_setprio(0);
        hook(tt);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto compute = [&](const char* __restrict__ A, const char* __restrict__ B, int kd, int r) __attribute__((always_inline)) {
    if constexpr (FDB == 2) {
      // (XL: the kernel row itself; see xload)
      const int off = XL ? kd * HH2 + r : (kd * HH2 + r) * HW2;
      pipe_taps(std::integral_constant<int, 3>{}, A, B, off, A, B, 0, [](int) {});
      return;
    }
    // register double buffer: the fragments of tap t+1 are read while the MFMAs of tap t
    // run (the sched barrier keeps the compiler from sinking the reads next to their use,
    // which exposed the LDS latency between every 4 MFMAs: ~31% MFMA busy)
    auto load_frags = [&](int t, uint4 (&xf)[MT], uint4 (&wf)[NT]) __attribute__((always_inline)) {
      const int tapoff = (kd * HH2 + r) * HWR + t;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        xf[mt] = lds128(A + lds_off((XL ? hp_lean + mt * HWR : hp0[XL ? 0 : mt]) + tapoff, g));
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        wf[nt] = lds128(B + lds_off(t * BN + wn * (NT * 16) + nt * 16 + (lane & 15), g));
    };
    uint4 xf[2][MT], wf[2][NT];
    load_frags(0, xf[0], wf[0]);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      if (t + 1 < 3) load_frags(t + 1, xf[(t + 1) & 1], wf[(t + 1) & 1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(wf[t & 1][nt], xf[t & 1][mt], acc[mt][nt]);
      __builtin_amdgcn_s_setprio(0);
      if (FRAG_DB) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // super-stage body: taps of row r0 (halo A0, weights B0) then row r1 (A1, B1), fragments
  // of tap t+1 read while tap t's MFMAs run, across the row boundary too
  auto compute2 = [&](const char* __restrict__ A0, const char* __restrict__ B0, int r0,
                      const char* __restrict__ A1, const char* __restrict__ B1, int r1, auto&& hook)
      __attribute__((always_inline)) {
    if constexpr (FDB == 2) {
      pipe_taps(std::integral_constant<int, 6>{}, A0, B0, XL ? r0 : r0 * HW2, A1, B1, XL ? r1 : r1 * HW2, hook);
      return;
    }
    auto load_frags = [&](int tt, uint4 (&xf)[MT], uint4 (&wf)[NT]) __attribute__((always_inline)) {
      const int t = tt % 3;
      const char* A = tt < 3 ? A0 : A1;
      const char* B = tt < 3 ? B0 : B1;
      const int tapoff = (tt < 3 ? r0 : r1) * HWR + t;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        xf[mt] = lds128(A + lds_off((XL ? hp_lean + mt * HWR : hp0[XL ? 0 : mt]) + tapoff, g));
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        wf[nt] = lds128(B + lds_off(t * BN + wn * (NT * 16) + nt * 16 + (lane & 15), g));
    };
    uint4 xf[2][MT], wf[2][NT];
    load_frags(0, xf[0], wf[0]);
#pragma unroll
    for (int tt = 0; tt < 6; ++tt) {
      if (tt + 1 < 6) load_frags(tt + 1, xf[(tt + 1) & 1], wf[(tt + 1) & 1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(wf[tt & 1][nt], xf[tt & 1][mt], acc[mt][nt]);
      __builtin_amdgcn_s_setprio(0);
      hook(tt);
      if (FRAG_DB) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // stage s computes kernel row grp of chunk `chunk` of item k.  NBB = 2: the weights of
  // stage s+1 are issued at stage s; NBB = 3: those of stage s+2 (two stages of latency
  // cover for the weight stream).  The next chunk's halo is issued at the chunk's first
  // stage.  Per stage a wave issues [epilogue stores] [B] [A]; with NBB = 3 the wait for
  // B(s) is the count of ops issued after it (snapshots of a per-wave issue counter).
  auto stage_of = [&](int t, int& k1, int& chunk1, int& grp1) {
    k1 = t / spi;
    const int r1 = t % spi;
    chunk1 = r1 / NG;
    grp1 = r1 % NG;
  };
  // wave priorities (MI355X_MICROARCH.md, two waves per SIMD: the second-dispatched half of an
  // 8-wave workgroup loses VALU / issue arbitration; one s_setprio 1 for it, no flips)
  if constexpr (NBB <= 3) {
    int ops = 0, snap0 = 0, snap1 = 0;           // NBB = 3: ops issued so far; after B(s), B(s+1)
    if (S > 0) {
      issue_A(0, 0, 0);
      issue_B(0, 0, 0, 0);
      ops = C::A_ITERS + C::B_ITERS;
      snap0 = ops;
      if (NBB == 3 && S > 1) {
        int k1, c1, g1;
        stage_of(1, k1, c1, g1);
        issue_B(k1, c1, g1, 1);
        ops += C::B_ITERS;
        snap1 = ops;
      }
    }
    // (late epilogue stores, not with the BN-backward epilogue: per layer fwd -0.5%, dgrad
    // -0.55%, dgradbn +0.2%, bench +0.17% — profiles/r6/epi_late_r6p/)
    constexpr bool epi_late = NBB == 2 && !BNB;
    int late_st = 0;                                // stores issued after the previous stage's DMA
    for (int s = 0; s < S; ++s) {
      const int k = s / spi, rem = s % spi;
      const int chunk = rem / NG, grp = rem % NG;
      const int cseq = k * nchunks + chunk;           // global chunk sequence -> A buffer
      const bool more_chunks = cseq + 1 < my_items * nchunks;
      if (NBB == 2) {
        // stage s needs B(s) (issued during s-1) and, at grp 0, A(cseq).  At grp 1 the next
        // chunk's halo (issued after B(s) during s-1) may stay in flight.  epi_late: the
        // previous item's epilogue stores were issued after that stage's DMA and may stay in
        // flight one more stage
        if (late_st > 0) vm_wait_dyn((NG > 1 && grp == 1 && more_chunks ? C::A_ITERS : 0) + late_st);
        else if (NG > 1 && grp == 1 && more_chunks) dma_wait<C::A_ITERS>();
        else dma_wait<0>();
        late_st = 0;
      } else {
        // A(cseq) was issued before B(s) (at the previous chunk's first stage or the prologue)
        vm_wait_dyn(ops - snap0);
      }
      // prologue BN + ReLU on the pieces this lane DMA'd (own vmcnt covers them): before the
      // stage barrier, which then also publishes the transformed halo (one barrier, not two)
      if (grp == 0 && (has_pro || has_pro2)) transform_A(k, chunk, cseq & 1);
      lds_sync();
      // the previous item's epilogue runs here, BEFORE this stage's DMA is issued, so its
      // stores drain under this stage's compute (vmcnt retires in order)
      if (rem == 0 && s > 0 && !epi_late) {
        if constexpr (!(DDLPC_CONV_DIAG & 16)) epilogue(k - 1);
        ops += EPI_STORES;
      }
      const int sn = s + NBB - 1;                     // stage whose weights are issued now
      int snapn = 0;
      if (sn < S) {
        int k1, c1, g1;
        stage_of(sn, k1, c1, g1);
        issue_B(k1, c1, g1, sn % NBB);
        ops += C::B_ITERS;
        snapn = ops;
      }
      if (grp == 0 && more_chunks) {
        const int k1 = (cseq + 1) / nchunks;
        issue_A(k1, (cseq + 1) % nchunks, (cseq + 1) & 1);
        ops += C::A_ITERS;
      }
      if (rem == 0 && s > 0 && epi_late) {
        if constexpr (!(DDLPC_CONV_DIAG & 16)) epilogue(k - 1);
        late_st = EPI_STORES;
      }
      // BNB: the item's last stage loads y for its epilogue (next stage: grp 0, full wait)
      if (BNB && KS == 1 && rem == spi - 1) issue_Y(k);
      if (NBB == 3) { snap0 = snap1; snap1 = snapn; }
      compute(sA(cseq & 1), sB(s % NBB), DIMS == 3 ? grp / 3 : 0, DIMS == 3 ? grp % 3 : grp);
    }
  } else {
    // NBB = 4, SUPER-STAGES (2-D): a barrier per TWO kernel rows (6 taps, 96 MFMAs per
    // wave) instead of one — the per-stage barrier and the exposed first-tap LDS latency
    // were most of the gap to the MFMA rate (operand DMA skipped: only 15-20% faster).
    // Pairs p = (chunk sequence c, row r) in order; super-stage j computes pairs 2j, 2j+1
    // (an item has 3 * nchunks pairs, nchunks even: items never straddle a super-stage).
    // Weights of super-stage j+1 (two rows, B slots 2*((j+1)&1) + h) are issued at j; the
    // halo of chunk c at super-stage floor((3c-4)/2)+1 (after chunk c-2's last use), one
    // super-stage before its first use floor(3c/2), where it is transformed (prologue)
    // before the barrier.  Everything issued at j-1 is awaited at j (dma_wait<0>).
    const int P = my_items * nchunks * NG;
    const int J = (P + 1) / 2;
    const int total_chunks = my_items * nchunks;
    auto issue_Bj = [&](int j) __attribute__((always_inline)) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pp = 2 * j + h;
        if (pp < P) {
          const int cs = pp / NG;
          issue_B(cs / nchunks, cs % nchunks, pp % NG, 2 * (j & 1) + h);
        }
      }
    };
    auto issue_Ac = [&](int c) __attribute__((always_inline)) {
      if (c < total_chunks) issue_A(c / nchunks, c % nchunks, c & 1);
    };
    if (J > 0) {
      issue_Ac(0);
      issue_Ac(1);
      issue_Bj(0);
    }
    // BNB with ylead 2: an item's y is loaded at its second-to-last super-stage (after that
    // stage's DMAs: the youngest MT * NT loads), so the last super-stage waits for everything
    // but y and y has two super-stages to arrive from HBM instead of one
    constexpr bool y2 = false;           // (y two super-stages ahead: 1-3% slower, profiles/r3s)
    for (int j = 0; j < J; ++j) {
      if (y2 && j > 0 && (2 * j + 2) % spi == 0) dma_wait<MT * NT>();
      else dma_wait<0>();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pp = 2 * j + h;
        if (pp < P && pp % NG == 0 && (has_pro || has_pro2)) {
          const int cs = pp / NG;
          transform_A(cs / nchunks, cs % nchunks, cs & 1);
        }
      }
      lds_sync();
      const int k0 = (2 * j) / spi;
      if ((2 * j) % spi == 0 && j > 0) epilogue(k0 - 1);
      // chunk whose halo is issued at this super-stage (-1: none)
      const int cA = j % 3 == 2 ? 2 * ((j + 1) / 3) : (j % 3 == 0 && j > 0) ? 2 * (j / 3) + 1 : -1;
      if (j + 1 < J) issue_Bj(j + 1);
      if (cA >= 0) issue_Ac(cA);
      // BNB: an item's last (ylead 2: second-to-last) super-stage loads y for its epilogue
      if (BNB && KS == 1) {
        if (y2) {
          if ((2 * j + 4) % spi == 0) issue_Y((2 * j + 4) / spi - 1);
        } else if ((2 * j + 2) % spi == 0) {
          issue_Y((2 * j + 2) / spi - 1);
        }
      }
      // P is even (nchunks even): both pairs exist; one 6-tap fragment pipeline across them
      const int c0 = (2 * j) / NG, c1 = (2 * j + 1) / NG;
      compute2(sA(c0 & 1), sB(2 * (j & 1)), (2 * j) % NG, sA(c1 & 1), sB(2 * (j & 1) + 1),
               (2 * j + 1) % NG, [](int) {});
    }
  }
  if (S > 0) {
    if (BNB) dma_wait<0>();
    epilogue(my_items - 1);
  }

  // ---- one BN-statistics partial row per workgroup: shuffle over the 16 pixel lanes,
  // per-wave-row LDS slots summed in a fixed order (bit-reproducible), one row write
  if (p.stats != nullptr && KS == 1) {
    dma_wait<0>();
    lds_sync();
    float* red = LSTAT ? s_red : reinterpret_cast<float*>(base);   // halo buffers are free now
    const int co0 = co0_item;
#pragma unroll
    for (int nt = 0; nt < (LSTAT ? 0 : NT); ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a1 = s1[nt][i], a2 = s2[nt][i];
        a1 = row16_sum(a1); a2 = row16_sum(a2);
        if ((lane & 15) == 0) {
          const int col = wn * (NT * 16) + nt * 16 + 4 * (lane >> 4) + i;
          red[(2 * wm) * BN + col] = a1;           // one writer per (wave row, column)
          red[(2 * wm + 1) * BN + col] = a2;
        }
      }
    lds_sync();
    float* row = p.stats + (long long)blockIdx.x * 2 * p.Cout;
    for (int c = tid; c < p.Cout; c += C::NTH) {   // full row: zeros outside this n tile
      const bool mine = c >= co0 && c < co0 + BN;
      float t1 = 0.f, t2 = 0.f;                    // fixed-order sum over wave rows
      if (mine)
        for (int r = 0; r < WM; ++r) { t1 += red[(2 * r) * BN + c - co0]; t2 += red[(2 * r + 1) * BN + c - co0]; }
      row[c] = t1;
      row[p.Cout + c] = t2;
    }
  }
}

// split-K finalize: sum the KS fp32 partials (fixed order), + bias, bf16 store (optionally
// split into two outputs), per-workgroup BN statistic rows of the fp32 outputs
__global__ void conv_splitk_finalize_kernel(const float* __restrict__ part, int KS, long long npix,
                                            int Cout, int Co1, const float* __restrict__ bias,
                                            bf16_t* __restrict__ Y1, bf16_t* __restrict__ Y2,
                                            float* __restrict__ stats, const bf16_t* __restrict__ bnb_y,
                                            const float* __restrict__ bnb_s4) {
  const int G = Cout / 8;
  const int per = (blockDim.x / G) * G;
  const int tid = threadIdx.x;
  const int cg = tid % G;
  const int c8 = cg * 8;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  // BN-backward partials (ConvFwdArgs::bnb_y): constants of this thread's 8 channels
  float bsc[8], bsh[8], bis[8], bnm[8];
  if (bnb_y != nullptr && tid < per)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bsc[j] = bnb_s4[2 * Cout + c8 + j]; bsh[j] = bnb_s4[3 * Cout + c8 + j];
      bis[j] = bnb_s4[Cout + c8 + j]; bnm[j] = -bnb_s4[c8 + j] * bis[j];
    }
  if (tid < per) {
    for (long long px = blockIdx.x * (long long)(per / G) + tid / G; px < npix;
         px += (long long)gridDim.x * (per / G)) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bias != nullptr ? bias[c8 + j] : 0.f;
      for (int k = 0; k < KS; ++k) {
        const float4* q = reinterpret_cast<const float4*>(part + ((long long)k * npix + px) * Cout + c8);
        const float4 a = q[0], b = q[1];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
        v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      }
      const uint4 pk = pack8(v);
      if (c8 < Co1) *reinterpret_cast<uint4*>(Y1 + px * Co1 + c8) = pk;
      else *reinterpret_cast<uint4*>(Y2 + px * (Cout - Co1) + (c8 - Co1)) = pk;
      if (stats != nullptr) {
        if (bnb_y != nullptr) {                  // (BN backward: the fp32 dA, as the epilogues)
          float yy[8];
          unpack8(*reinterpret_cast<const uint4*>(bnb_y + px * Cout + c8), yy);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float a = fmaf(yy[j], bsc[j], bsh[j]);
            const float dyh = a > 0.f ? v[j] : 0.f;
            s1[j] += dyh;
            s2[j] = fmaf(dyh, fmaf(yy[j], bis[j], bnm[j]), s2[j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) { s1[j] += v[j]; s2[j] += v[j] * v[j]; }
        }
      }
    }
  }
  if (stats == nullptr) return;
  __shared__ float red[256];
  for (int half = 0; half < 2; ++half)
    for (int j = 0; j < 8; ++j) {
      __syncthreads();
      red[tid] = tid < per ? (half ? s2[j] : s1[j]) : 0.f;
      __syncthreads();
      for (int g2 = tid; g2 < G; g2 += blockDim.x) {
        float t = 0.f;
        for (int q = g2; q < per; q += G) t += red[q];
        stats[((long long)blockIdx.x * 2 + half) * Cout + g2 * 8 + j] = t;
      }
    }
}

}  // namespace

// persistent grid of the streaming kernel: one workgroup per item up to persist_blocks, a
// multiple of KS * nTilesN (every block stays on one n tile and channel split); BN groups:
// groups x R x (KS * nTilesN) with R workgroups per (group, n tile) — as many as fit the
// persistent grid, at least one, at most the group's M tiles
int conv3_fwd_grid(const ConvFwdArgs& a) {
  const int q = a.nTilesN * a.ksplit;
  if (a.groups > 1) {
    const int Mg = a.nTilesM / a.groups;
    const int cap = a.persist_blocks > 0 ? a.persist_blocks : a.nTilesM * q;
    const int R = std::max(1, std::min(Mg, cap / (a.groups * q)));
    return a.groups * R * q;
  }
  int grid = a.nTilesM * q;
  if (a.persist_blocks > 0 && grid > a.persist_blocks) grid = a.persist_blocks / q * q;
  return grid;
}

namespace {

// (per-tap s_setprio flips around the MFMA blocks: a static priority for waves NW/2.. or no
// s_setprio measured -0.2 / -0.3%, noise — profiles/r6/prio_ab_r6b.json)
template <int DIMS, int WM, int WN, int MT, int NT, int HALO, int NBB, int FDB, bool XL>
void launch_mode(ConvFwdArgs& a, int grid, hipStream_t st) {
  using C = Cfg<DIMS, WM, WN, MT, NT, HALO, NBB>;
  if constexpr (DIMS == 2 && NBB != 3 && !C::LEAN) {
    // (split-K: fp32 partials, the BN-backward reduction in conv_splitk_finalize_kernel)
    if (a.bnb_y != nullptr && a.ksplit == 1) {
      hipLaunchKernelGGL((conv3_fwd_kernel<DIMS, WM, WN, MT, NT, HALO, NBB, FDB, true, XL>), dim3(grid),
                         dim3(C::NTH), C::SMEM, st, a);
      return;
    }
  }
  hipLaunchKernelGGL((conv3_fwd_kernel<DIMS, WM, WN, MT, NT, HALO, NBB, FDB, false, XL>), dim3(grid),
                     dim3(C::NTH), C::SMEM, st, a);
}

template <int DIMS, int WM, int WN, int MT, int NT, int HALO, int NBB = 2>
void launch_cfg(ConvFwdArgs& a, hipStream_t st) {
  const int grid = conv3_fwd_grid(a);
  a.stat_rows = grid;
  // rolling fragment pipeline (pipe_taps): every configuration (the whole-tap register
  // double buffer and no buffering measured slower: profiles/r3s/conv_ab_pipe_r3s1.txt).
  // 2-D 16-wide tiles whose stride-20 halo fits the buffer: the XL fragment addressing
  {
    const int halo_xl = (DIMS == 3 ? a.TD + 2 : 1) * (a.TH + 2) * 20;
    if (a.TW == 16 && (DIMS == 2 || a.TH == 4) && halo_xl <= HALO) {
      launch_mode<DIMS, WM, WN, MT, NT, HALO, NBB, 2, true>(a, grid, st);
      return;
    }
  }
  launch_mode<DIMS, WM, WN, MT, NT, HALO, NBB, 2, false>(a, grid, st);
}

// cfg 5 (BM-512, LEAN tiles: never with the BN-backward epilogue) on the rolling pipeline
void launch_cfg5(ConvFwdArgs& a, hipStream_t st) {
  using C = Cfg<2, 4, 2, 8, 4, 704, 2>;      // (34 halo rows of stride 20: 680 pixels)
  const int grid = conv3_fwd_grid(a);
  a.stat_rows = grid;
  hipLaunchKernelGGL((conv3_fwd_kernel<2, 4, 2, 8, 4, 704, 2, 2, false, true>), dim3(grid),
                     dim3(C::NTH), C::SMEM, st, a);
}

int cfg_wm(int cfg) { return cfg == 6 || cfg == 9 ? 8 : cfg == 8 ? 2 : cfg <= 1 || cfg >= 4 ? 4 : cfg == 2 ? 2 : 1; }

}  // namespace

// Tile configurations (cfg id -> BN, BM, halo capacity):
//   0: BN 32,  BM 256 (4x1 waves, 4x2 tiles)     2-D 16x16 / 32x8   3-D 4x4x16 / 8x4x8
//   1: BN 64,  BM 256 (4x1 waves, 4x4 tiles)     2-D 16x16 / 32x8   3-D 4x4x16 / 8x4x8
//   2: BN 128, BM 128 (2x2 waves, 4x4 tiles)     2-D 8x16 / 16x8    3-D 2x4x16 / 4x4x8
//   3: BN 128, BM 64  (1x4 waves, 4x2 tiles)     2-D 4x16 / 8x8     3-D 1x4x16 / 2x4x8
//   4: BN 128, BM 256 (4x2 waves = 512 threads, 4x4 tiles; 2-D only) 16x16 / 32x8: half the
//      weight-stream traffic per MFMA of cfg 2 (one workgroup per CU)
//   5: BN 128, BM 512 (4x2 waves = 512 threads, 8x4 tiles: 128 px x 64 ch per wave; 2-D
//      only) 32x16: half cfg 4's weight-stream DMA per MFMA and a quarter fewer LDS fragment
//      reads per MFMA (each wave's weight fragments serve 8 pixel tiles)
//   3-D with 8 waves (two per SIMD; the 4-wave 3-D configs fit one workgroup per CU in LDS,
//   i.e. ONE wave per SIMD and no latency hiding):
//   6: BN 32,  BM 384 (8x1 waves, 3x2 tiles) 6x4x16, halo 8x6x18
//   7: BN 64,  BM 256 (4x2 waves, 4x2 tiles) 4x4x16
//   8: BN 128, BM 128 (2x4 waves, 4x2 tiles) 2x4x16
//   9: BN 96,  BM 256 (8x1 waves, 2x6 tiles) 4x4x16 — the 96-channel data gradient of the
//      first decoder conv (d[up | skip] = 64 + 32 channels), which the 128-channel tiles
//      would pad by a third
// (halo capacity = DMA instructions per wave x 64 pixels)
int conv3_fwd_cfg_wm(int cfg) { return cfg_wm(cfg); }
int conv3_fwd_cfg_bn(int cfg) { return cfg == 0 || cfg == 6 ? 32 : cfg == 1 || cfg == 7 ? 64 : cfg == 9 ? 96 : 128; }
int conv3_fwd_cfg_bm(int cfg) {
  return cfg == 5 ? 512 : cfg == 6 ? 384 : cfg <= 1 || cfg == 4 || cfg == 7 || cfg == 9 ? 256 : cfg == 2 || cfg == 8 ? 128 : 64;
}
int conv3_fwd_cfg_halo(int dims, int cfg) {
  if (dims == 2) return cfg == 5 ? 612 : cfg <= 1 || cfg == 4 ? 384 : cfg == 2 ? 192 : 128;   // (cfg 5: 34 x 18, stored at stride 20)
  return cfg == 6 ? 896 : cfg <= 1 || cfg == 7 || cfg == 9 ? 704 : cfg == 2 || cfg == 8 ? 448 : 384;
}

void conv3_splitk_finalize_launch(ConvFwdArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL(conv_splitk_finalize_kernel, dim3(grid), dim3(256), 0, st, a.part, a.ksplit,
                     a.npix, a.Cout, a.Co1, a.bias, a.Y1, a.Y2, a.stats, a.bnb_y, a.bnb_s4);
}

void conv3_fwd_launch(ConvFwdArgs& a, int cfg, hipStream_t st) {
  if (a.dims == 2) {
    switch (cfg) {
      case 0: launch_cfg<2, 4, 1, 4, 2, 384>(a, st); break;
      case 1: launch_cfg<2, 4, 1, 4, 4, 384>(a, st); break;
      case 2: launch_cfg<2, 2, 2, 4, 4, 192>(a, st); break;
      case 4: {  // one workgroup per CU: super-stages (two kernel rows per barrier)
        const int nch = (a.Cin + 31) / 32 / a.ksplit;
        if (nch % 2 == 0) launch_cfg<2, 4, 2, 4, 4, 384, 4>(a, st);
        else launch_cfg<2, 4, 2, 4, 4, 384, 2>(a, st);
        break;
      }
      case 5: launch_cfg5(a, st); break;
      default: launch_cfg<2, 1, 4, 4, 2, 128>(a, st); break;
    }
  } else {
    switch (cfg) {
      // (halo capacities 720 / 480: the XL stride-20 halos of 4x4x16 / 2x4x16 tiles)
      case 0: launch_cfg<3, 4, 1, 4, 2, 720>(a, st); break;
      case 1: launch_cfg<3, 4, 1, 4, 4, 720>(a, st); break;
      case 2: launch_cfg<3, 2, 2, 4, 4, 480>(a, st); break;
      case 6: launch_cfg<3, 8, 1, 3, 2, 960>(a, st); break;   // (960: the XL halo of 6x4x16 tiles)
      case 7: launch_cfg<3, 4, 2, 4, 2, 720>(a, st); break;
      case 8: launch_cfg<3, 2, 4, 4, 2, 480>(a, st); break;
      case 9: launch_cfg<3, 8, 1, 2, 6, 704>(a, st); break;
      default: launch_cfg<3, 1, 4, 4, 2, 384>(a, st); break;
    }
  }
}

}  // namespace ddlpc
