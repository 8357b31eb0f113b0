// Weight gradient of the 3x3 (3x3x3) convolution — K3 of SURVEY.md §2.5.
//
//   dW[co][tap][ci] = sum_p dY[p][co] * A(X)[p + off(tap)][ci]
//
// GEMM view: M = Cout, N = taps x Cin, K = pixels (up to B*H*W = millions) -> split-K.
// Both operands are pixel-major in NHWC memory, so they are staged in LDS in their natural
// [pixel][channel] layout and fed to v_mfma_f32_16x16x32_bf16 through the gfx950 hardware
// transpose read ds_read_b64_tr_b16 (8 consecutive pixels per lane = the MFMA k run).
// The input side is staged as a (TD+2)(TH+2)(TW+2) halo per pixel tile, with the forward
// pass's prologue (BatchNorm-apply + ReLU of the previous layer) and the two-tensor concat
// re-applied on the fly, so the activation is never materialised; every tap of a 3-tap
// row re-reads the same halo.
//
// Each workgroup owns (co tile, 32-channel ci chunk, kd plane) and a contiguous range of
// pixel tiles; it writes an fp32 partial slab that reduce_rows (reduce.hip) sums over splits in a
// fixed order (bit-reproducible, so all data-parallel ranks stay bit-identical) and
// accumulates into the fp32 OIHW parameter gradient.
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

#include <cstdlib>

#include <stdexcept>
#include <type_traits>

namespace ddlpc {

// pixel tiles t_begin, t_begin + 1, ... of a (slices, tilesW, tilesH, images) grid visited in
// order: the integer divisions once, then a carry step per tile (per-tile divisions cost ~100
// scalar / vector instructions per tile against 36-54 MFMAs).  3-D: the depth slice d is the
// FASTEST index, so the three depth-tap-plane workgroups of a split (which run side by side
// on one XCD) re-read the input plane a neighbour fetched one tile earlier — from L2, not
// HBM.  n = image * D + d is the slice (2-D: D = 1, the plain w, h, image order).
struct TileWalk {
  int t, w, h, n, d, nb;
  DDLPC_DEVICE void init(int t0, int tilesW, int tilesH, int D) {
    t = t0;
    d = t0 % D;
    int q = t0 / D;
    w = q % tilesW;
    q /= tilesW;
    h = q % tilesH;
    nb = q / tilesH * D;
    n = nb + d;
  }
  DDLPC_DEVICE void to(int tile, int tilesW, int tilesH, int D) {
    while (t < tile) {
      ++t;
      ++n;
      if (++d == D) {
        d = 0;
        if (++w == tilesW) {
          w = 0;
          if (++h == tilesH) { h = 0; nb += D; }
        }
        n = nb;
      }
    }
  }
};

namespace {

constexpr int CI = 32;          // ci per workgroup
constexpr int PT = 128;         // pixels per K step tile

template <int DIMS>
struct WgHalo { static constexpr int value = DIMS == 2 ? 208 : 448; };

// Wave tiling: every wave holds ALL BCO output channels (NCO = BCO/16 A fragments) and a
// strided subset of the 18 (tap, ci-half) pairs (5,5,4,4 across the 4 waves), so each dY
// fragment read feeds up to 5 MFMAs and each input fragment up to NCO: per 32-pixel k-step
// a wave issues 2*NCO + 2*5 transposed reads for 5*NCO MFMAs.
template <int DIMS, int BCO>
struct WgCfg {
  static constexpr int NCO = BCO / 16;                 // 2 or 4
  static constexpr int NP = 5;                         // max (tap, ci-half) pairs per wave
  static constexpr int HALO = WgHalo<DIMS>::value;
  static constexpr int Y_ROWB = BCO * 2;
  static constexpr int X_ROWB = CI * 2;
  static constexpr int Y_BYTES = PT * Y_ROWB;
  static constexpr int X_BYTES = HALO * X_ROWB;
  static constexpr int Y_ELEMS = PT * BCO / 8;
  static constexpr int Y_PER_T = (Y_ELEMS + 255) / 256;
  static constexpr int X_ELEMS = HALO * CI / 8;
  static constexpr int X_PER_T = (X_ELEMS + 255) / 256;
  static constexpr int SMEM = Y_BYTES + X_BYTES;
};

template <int DIMS, int BCO>
__global__ __launch_bounds__(256, 2) void conv3_wgrad_kernel(ConvWgradArgs p) {
  using Cfg = WgCfg<DIMS, BCO>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sY = smem;
  char* sX = smem + Cfg::Y_BYTES;
  __shared__ float s_scale[512], s_shift[512];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // block -> (plane, ci chunk, co tile, split), the first three innermost in XCD-contiguous
  // order: workgroups streaming the same pixel range share one XCD's L2
  int b = xcd_remap(blockIdx.x, gridDim.x);
  const int plane = b % p.planes; b /= p.planes;
  const int cic = b % p.ciChunks; b /= p.ciChunks;
  const int cot = b % p.coTiles; b /= p.coTiles;
  const int split = b;
  const int co0 = cot * BCO, ci0 = cic * CI;

  const bool has_pro = p.pscale != nullptr;
  if (has_pro)
    for (int c = tid; c < p.C1; c += 256) { s_scale[c] = p.pscale[c]; s_shift[c] = p.pshift[c]; }

  const int HW2 = p.TW + 2, HH2 = p.TH + 2;
  const int halo = (p.TD + (DIMS == 3 ? 2 : 0)) * HH2 * HW2;
  const int tiles_per_img = p.tilesD * p.tilesH * p.tilesW;
  const int t_begin = (int)((long long)p.nTiles * split / p.splits);
  const int t_end = (int)((long long)p.nTiles * (split + 1) / p.splits);

  // per-lane pixel rows for the transposed reads: pixel = kb + 8*(lane>>4) + q + 4*h
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  int hp0[8];                                     // [kstep*2 + h]
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pix = ks * 32 + 8 * g + q + 4 * h;
      const int pw = pix % p.TW, ph = (pix / p.TW) % p.TH;
      const int pd = DIMS == 3 ? pix / (p.TW * p.TH) : 0;
      hp0[ks * 2 + h] = (pd * HH2 + ph) * HW2 + pw;
    }

  f32x4_t acc[Cfg::NCO][Cfg::NP];
#pragma unroll
  for (int j = 0; j < Cfg::NCO; ++j)
#pragma unroll
    for (int q2 = 0; q2 < Cfg::NP; ++q2) acc[j][q2] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 ry[Cfg::Y_PER_T], rx[Cfg::X_PER_T];
  uint32_t x_valid = 0;

  auto load = [&](int tile) {
    int t = tile;
    const int tw_i = t % p.tilesW; t /= p.tilesW;
    const int th_i = t % p.tilesH; t /= p.tilesH;
    const int td_i = t % p.tilesD; t /= p.tilesD;
    const int n = t;
    const int d0 = td_i * p.TD, h0 = th_i * p.TH, w0 = tw_i * p.TW;
    // dY tile [PT px][BCO co]
#pragma unroll
    for (int i = 0; i < Cfg::Y_PER_T; ++i) {
      const int e = tid + 256 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < Cfg::Y_ELEMS) {
        const int px = e / (BCO / 8), cg = e % (BCO / 8);
        const int pw = px % p.TW, ph = (px / p.TW) % p.TH;
        const int pd = DIMS == 3 ? px / (p.TW * p.TH) : 0;
        const int gw = w0 + pw, gh = h0 + ph, gd = d0 + pd;
        const int co = co0 + cg * 8;
        if (gw < p.W && gh < p.H && gd < p.D && co < p.Cout) {
          const long long pix = ((long long)(n * p.D + gd) * p.H + gh) * p.W + gw;
          v = *reinterpret_cast<const uint4*>(p.dY + pix * p.Cout + co);
        }
      }
      ry[i] = v;
    }
    // X halo [halo px][CI ci] (+ prologue flag)
    x_valid = 0;
    const int kd_off = DIMS == 3 ? plane : 1;     // plane kd -> halo depth offset
    (void)kd_off;
#pragma unroll
    for (int i = 0; i < Cfg::X_PER_T; ++i) {
      const int e = tid + 256 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      const int px = e >> 2, cq = e & 3;
      if (px < halo) {
        const int hw = px % HW2, hh = (px / HW2) % HH2;
        const int hd = DIMS == 3 ? px / (HW2 * HH2) : 1;
        const int gw = w0 + hw - 1, gh = h0 + hh - 1, gd = d0 + hd - 1;
        const int c8 = ci0 + cq * 8;
        if (gw >= 0 && gw < p.W && gh >= 0 && gh < p.H && gd >= 0 && gd < p.D && c8 < p.Cin) {
          const long long pix = ((long long)(n * p.D + gd) * p.H + gh) * p.W + gw;
          const bf16_t* src;
          int C, c;
          if (c8 < p.C1) { src = p.X1; C = p.C1; c = c8; }
          else { src = p.X2; C = p.C2; c = c8 - p.C1; }
          const bf16_t* ptr = src + pix * C + c;
          if ((C & 7) == 0) {
            v = *reinterpret_cast<const uint4*>(ptr);
          } else {
            uint16_t tt[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) tt[j] = (c + j < C) ? ptr[j] : (uint16_t)0;
            v = make_uint4(tt[0] | (tt[1] << 16), tt[2] | (tt[3] << 16), tt[4] | (tt[5] << 16),
                           tt[6] | (tt[7] << 16));
          }
          if (c8 < p.C1) x_valid |= 1u << i;
        }
      }
      rx[i] = v;
    }
  };

  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < Cfg::Y_PER_T; ++i) {
      const int e = tid + 256 * i;
      if (e < Cfg::Y_ELEMS) {
        const int px = e / (BCO / 8), cg = e % (BCO / 8);
        *reinterpret_cast<uint4*>(sY + px * Cfg::Y_ROWB + cg * 16) = ry[i];
      }
    }
#pragma unroll
    for (int i = 0; i < Cfg::X_PER_T; ++i) {
      const int e = tid + 256 * i;
      const int px = e >> 2, cq = e & 3;
      if (px < halo) {
        uint4 v = rx[i];
        if (has_pro && ((x_valid >> i) & 1u)) {
          const int c8 = ci0 + cq * 8;
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int c = c8 + j < p.C1 ? c8 + j : p.C1 - 1;
            f[j] = fmaxf(fmaf(f[j], s_scale[c], s_shift[c]), 0.0f);
          }
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(sX + px * Cfg::X_ROWB + cq * 16) = v;
      }
    }
  };

  if (t_begin < t_end) load(t_begin);
  __syncthreads();
  const int kd = DIMS == 3 ? plane : 0;
  for (int tile = t_begin; tile < t_end; ++tile) {
    __syncthreads();
    store();
    __syncthreads();
    if (tile + 1 < t_end) load(tile + 1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      // A = dY^T fragments (16 co x 32 px each): rows = pixels, cols = co
      uint4 af[Cfg::NCO];
      const int r0 = ks * 32 + 8 * g + q;
#pragma unroll
      for (int j = 0; j < Cfg::NCO; ++j) {
        const uint2 lo = lds_read_tr16(sY + r0 * Cfg::Y_ROWB + (j * 16 + 4 * pp) * 2);
        const uint2 hi = lds_read_tr16(sY + (r0 + 4) * Cfg::Y_ROWB + (j * 16 + 4 * pp) * 2);
        af[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int pi = 0; pi < Cfg::NP; ++pi) {
        const int pair = wave + 4 * pi;                 // wave-uniform
        if (pair < 18) {
          const int tap = pair >> 1, cih = pair & 1;
          const int tapoff = (kd * HH2 + tap / 3) * HW2 + tap % 3;
          const int cc = cih * 16 + 4 * pp;
          const uint2 lo = lds_read_tr16(sX + (hp0[ks * 2] + tapoff) * Cfg::X_ROWB + cc * 2);
          const uint2 hi = lds_read_tr16(sX + (hp0[ks * 2 + 1] + tapoff) * Cfg::X_ROWB + cc * 2);
          const uint4 bfr = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
          for (int j = 0; j < Cfg::NCO; ++j) acc[j][pi] = mfma16x16x32(af[j], bfr, acc[j][pi]);
        }
      }
    }
  }

  // ---- partial slab: part[split][co][tap][ci]   (tap = kd*9 + r*3 + s)
  float* out = p.partial + (long long)split * p.Cout * p.taps * p.Cin;
#pragma unroll
  for (int pi = 0; pi < Cfg::NP; ++pi) {
    const int pair = wave + 4 * pi;
    if (pair >= 18) continue;
    const int tap = kd * 9 + (pair >> 1);
    const int ci = ci0 + (pair & 1) * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < Cfg::NCO; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = co0 + j * 16 + 4 * (lane >> 4) + i;
        if (co < p.Cout && ci < p.Cin) out[((long long)co * p.taps + tap) * p.Cin + ci] = acc[j][pi][i];
      }
  }
  (void)tiles_per_img;
}

// ============================================================================ v2 (2-D; 3-D as 1-deep tiles per depth tap plane)
// Same GEMM and partial-slab contract, restructured like the forward kernels:
//   * both operands arrive by LDS-DMA into DOUBLE-BUFFERED LDS (no VGPR round trip, no
//     integer division in the tile loop: per-lane source geometry is tile independent);
//     the tile t+1 DMA is in flight while tile t computes, ONE barrier per tile;
//   * the prologue (BN-apply + ReLU) runs in LDS on the pieces each lane DMA'd, before the
//     barrier;
//   * dY rows carry an XOR swizzle on 32-B segments so the transposed A reads are bank-
//     conflict free (x = row bit 1 | row bit 3 << 1 for 128-B rows, row bit 3 for 64-B);
//     the swizzle is lane-constant, so every read address folds into the offset field;
//   * X halo rows stay linear (tap offsets fold into immediates; the B reads are 2-way).
template <int BCO, int PT>
struct Wg2Cfg {
  static constexpr int NCO = BCO / 16;
  static constexpr int NP = 5;
  static constexpr int TH = PT / 16;
  static constexpr int HALO = (TH + 2) * 18;
  static constexpr int Y_ROWB = BCO * 2;
  static constexpr int Y_PIECES = PT * BCO / 8;
  static constexpr int Y_INSTR = Y_PIECES / 64;
  static constexpr int Y_ITERS = (Y_INSTR + 3) / 4;
  static constexpr int Y_BYTES = Y_INSTR * 1024;
  static constexpr int X_PIECES = HALO * 4;
  static constexpr int X_INSTR = (X_PIECES + 63) / 64;
  static constexpr int X_ITERS = (X_INSTR + 3) / 4;
  static constexpr int X_BYTES = X_INSTR * 1024;
  static constexpr int SS_BYTES = 2 * 512 * 4 + 7 * BCO * 4;   // X prologue | dY prologue tables
  static constexpr int SMEM = SS_BYTES + 2 * (Y_BYTES + X_BYTES);
  static constexpr int KSTEPS = PT / 32;
};

template <int BCO>
DDLPC_DEVICE int wg2_yswz(int row) {             // XOR on the 16-B piece index
  return BCO == 64 ? ((((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1) : (((row >> 3) & 1) << 1);
}

template <int BCO, int PT>
__global__ __launch_bounds__(256, PT <= 96 ? 3 : 2) void conv3_wgrad2_kernel(ConvWgradArgs p) {
  using namespace convlds;
  using Cfg = Wg2Cfg<BCO, PT>;
  constexpr int TH = Cfg::TH, HW2 = 18;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_scale = reinterpret_cast<float*>(smem);
  float* s_shift = s_scale + 512;
  char* base = smem + Cfg::SS_BYTES;
  auto sY = [&](int b) { return base + b * (Cfg::Y_BYTES + Cfg::X_BYTES); };
  auto sX = [&](int b) { return base + b * (Cfg::Y_BYTES + Cfg::X_BYTES) + Cfg::Y_BYTES; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // (ci chunk, co tile) innermost in the XCD-contiguous logical order: the workgroups that
  // stream the SAME pixel range (same dY and X tiles) run together on one XCD and share its
  // L2 instead of each re-reading the operands from HBM
  int b = xcd_remap(blockIdx.x, gridDim.x);
  const int cic = b % p.ciChunks; b /= p.ciChunks;
  const int cot = b % p.coTiles; b /= p.coTiles;
  // 3-D: one depth tap plane kd per workgroup (planes = 3).  With 1-deep pixel tiles the
  // plane's 9 taps are a 2-D weight gradient of dY slice d against X slice d + kd - 1, so
  // the (n, d) slices are the "images" and the X image is shifted by kd - 1
  const int plane = b % p.planes; b /= p.planes;
  const int split = b;
  const int co0 = cot * BCO, ci0 = cic * BK;
  const int dshift = p.planes == 3 ? plane - 1 : 0;

  const bool has_pro = p.pscale != nullptr;
  const bool has_pro2 = p.pscale2 != nullptr;           // deferred skip: X2 channels at C1 + c
  if (has_pro)
    for (int c = tid; c < p.C1; c += 256) { s_scale[c] = p.pscale[c]; s_shift[c] = p.pshift[c]; }
  if (has_pro2)
    for (int c = tid; c < p.C2; c += 256) { s_scale[p.C1 + c] = p.pscale2[c]; s_shift[p.C1 + c] = p.pshift2[c]; }
  // dY prologue (BN backward on load): table [7][BCO] = scale, shift, invstd, -mean*invstd,
  // k, m1, m2 of this workgroup's output channels
  const bool has_dyp = p.dyy != nullptr;
  float* s_dy = s_scale + 1024;
  if (has_dyp)
    for (int i = tid; i < BCO; i += 256) {
      const int c = co0 + i;
      const bool ok = c < p.Cout;
      const float is = ok ? p.dys4[p.Cout + c] : 0.f;
      s_dy[i] = ok ? p.dys4[2 * p.Cout + c] : 0.f;
      s_dy[BCO + i] = ok ? p.dys4[3 * p.Cout + c] : 0.f;
      s_dy[2 * BCO + i] = is;
      s_dy[3 * BCO + i] = ok ? -p.dys4[c] * is : 0.f;
      s_dy[4 * BCO + i] = ok ? p.dycoef[c] : 0.f;
      s_dy[5 * BCO + i] = ok ? p.dycoef[p.Cout + c] : 0.f;
      s_dy[6 * BCO + i] = ok ? p.dycoef[2 * p.Cout + c] : 0.f;
    }
  const int t_begin = (int)((long long)p.nTiles * split / p.splits);
  const int t_end = (int)((long long)p.nTiles * (split + 1) / p.splits);
  const long long img_px = (long long)p.H * p.W;

  // ---- tile-independent per-lane DMA geometry
  int y_pw[Cfg::Y_ITERS], y_ph[Cfg::Y_ITERS], y_rel[Cfg::Y_ITERS];
  // dY prologue: the lane's pieces of y (loaded to registers with the dA DMA of the same
  // tile) and whether each piece is a real (pixel, channel group)
  uint4 yv[Cfg::Y_ITERS];
  bool y_ok[Cfg::Y_ITERS];
#pragma unroll
  for (int i = 0; i < Cfg::Y_ITERS; ++i) {
    const int e = (i * 4 + wave) * 64 + lane;
    const int row = e / (BCO / 8), pc = e % (BCO / 8);
    const int sp = pc ^ wg2_yswz<BCO>(row);        // source piece stored at LDS piece pc
    y_pw[i] = row % 16;
    y_ph[i] = row / 16;
    const int co = co0 + sp * 8;
    y_rel[i] = co < p.Cout ? (y_ph[i] * p.W + y_pw[i]) * p.Cout + co : -1;
  }
  int x_dw[Cfg::X_ITERS], x_dh[Cfg::X_ITERS], x_pix[Cfg::X_ITERS];
#pragma unroll
  for (int i = 0; i < Cfg::X_ITERS; ++i) {
    const int e = (i * 4 + wave) * 64 + lane;
    const int px = e >> 2;
    x_dw[i] = px < Cfg::HALO ? px % HW2 - 1 : -(1 << 20);
    x_dh[i] = px / HW2 - 1;
    x_pix[i] = -1;
  }
  const int c8l = ci0 + (lane & 3) * 8;              // this lane's X channel group
  const bool second = ci0 >= p.C1;                   // chunk served by X2 (C1 % 32 == 0)
  const int Cs = second ? p.C2 : p.C1;
  const int cs0 = second ? c8l - p.C1 : c8l;
  const bf16_t* xsrc = second ? p.X2 : p.X1;
  const bool xch_ok = cs0 < Cs;
  // (prologue constants stay in LDS here: 16 more live VGPRs would cost the 96-pixel-tile
  // variant its third workgroup per CU — measured 55% slower on dec3.a / dec2.a)

  TileWalk tw;                                     // the issue stream's tile geometry
  tw.init(t_begin, p.tilesW, p.tilesH, p.D);
  auto issue = [&](int tile, int buf) {
    tw.to(tile, p.tilesW, p.tilesH, p.D);
    const int n = tw.n;                              // (n, d) slice
    const int dx = tw.d + dshift;
    const bool dok = dx >= 0 && dx < p.D;
    const int h0 = tw.h * TH, w0 = tw.w * 16;
    const auto ry = make_rsrc(p.dY + n * img_px * p.Cout, (unsigned)(img_px * p.Cout * 2));
    const int ybase = (h0 * p.W + w0) * p.Cout;
#pragma unroll
    for (int i = 0; i < Cfg::Y_ITERS; ++i) {
      if ((i * 4 + wave) >= Cfg::Y_INSTR) break;
      const bool ok = y_rel[i] >= 0 && w0 + y_pw[i] < p.W && h0 + y_ph[i] < p.H;
      dma16(ry, sY(buf) + (i * 4 + wave) * 1024, ok ? (unsigned)(ybase + y_rel[i]) * 2u : kOOB);
      if (has_dyp) {
        const auto ryy = make_rsrc(p.dyy + n * img_px * p.Cout, (unsigned)(img_px * p.Cout * 2));
        const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(ryy, ok ? (unsigned)(ybase + y_rel[i]) * 2u : kOOB, 0, 0);
        yv[i] = make_uint4(v.x, v.y, v.z, v.w);
        y_ok[i] = ok;
      }
    }
    const auto rx = make_rsrc(xsrc + (n + (dok ? dshift : 0)) * img_px * Cs, (unsigned)(img_px * Cs * 2));
#pragma unroll
    for (int i = 0; i < Cfg::X_ITERS; ++i) {
      if ((i * 4 + wave) >= Cfg::X_INSTR) break;
      const int gw = w0 + x_dw[i], gh = h0 + x_dh[i];
      x_pix[i] = (gw >= 0 && gw < p.W && gh >= 0 && gh < p.H && xch_ok && dok) ? gh * p.W + gw : -1;
      dma16(rx, sX(buf) + (i * 4 + wave) * 1024, x_pix[i] >= 0 ? (unsigned)(x_pix[i] * Cs + cs0) * 2u : kOOB);
    }
  };
  // dY = k (dA [y*scale + shift > 0] - m1 - xhat m2) on the lane's own landed pieces
  auto transform_dy = [&](int buf) {
#pragma unroll
    for (int i = 0; i < Cfg::Y_ITERS; ++i) {
      if ((i * 4 + wave) < Cfg::Y_INSTR && y_ok[i]) {
        const int e = (i * 4 + wave) * 64 + lane;
        const int row = e / (BCO / 8), pc = e % (BCO / 8);
        const int cl = (pc ^ wg2_yswz<BCO>(row)) * 8;   // channel offset within the co tile
        uint4* qd = reinterpret_cast<uint4*>(sY(buf) + e * 16);
        float fd[8], fy[8], o[8];
        unpack8(*qd, fd);
        unpack8(yv[i], fy);
        const float* t = s_dy + opaque_zero() + cl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = fmaf(fy[j], t[j], t[BCO + j]);
          const float dyh = a > 0.f ? fd[j] : 0.f;
          const float xh = fmaf(fy[j], t[2 * BCO + j], t[3 * BCO + j]);
          o[j] = t[4 * BCO + j] * (dyh - t[5 * BCO + j] - xh * t[6 * BCO + j]);
        }
        *qd = pack8(o);
      }
    }
  };
  auto transform = [&](int buf) {
#pragma unroll
    for (int i = 0; i < Cfg::X_ITERS; ++i) {
      const int e = (i * 4 + wave) * 64 + lane;
      if ((i * 4 + wave) < Cfg::X_INSTR && x_pix[i] >= 0) {
        uint4* q = reinterpret_cast<uint4*>(sX(buf) + e * 16);
        float f[8];
        unpack8(*q, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = min(c8l + j, (second ? p.Cin : p.C1) - 1);
          f[j] = fmaxf(fmaf(f[j], s_scale[c], s_shift[c]), 0.0f);
        }
        *q = pack8(f);
      }
    }
  };

  // ---- per-lane transposed-read geometry
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  // A (dY): rows ks*32 + 8g + 4h + q; swizzle depends only on (g, h, q)
  int ya[2][Cfg::NCO];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < Cfg::NCO; ++j) {
      const int row = 8 * g + 4 * h + q;
      const int pc = 2 * j + (pp >> 1);
      ya[h][j] = row * Cfg::Y_ROWB + ((pc ^ wg2_yswz<BCO>(row)) << 4) + (pp & 1) * 8;
    }
  // B (X): tile pixel ks*32 + 8g + 4h + q -> halo row; + tap offset
  int xb[Cfg::KSTEPS][2];
#pragma unroll
  for (int ks = 0; ks < Cfg::KSTEPS; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pix = ks * 32 + 8 * g + 4 * h + q;
      xb[ks][h] = ((pix / 16) * HW2 + pix % 16) * 64 + (pp >> 1) * 16 + (pp & 1) * 8;
    }

  f32x4_t acc[Cfg::NCO][Cfg::NP];
#pragma unroll
  for (int j = 0; j < Cfg::NCO; ++j)
#pragma unroll
    for (int q2 = 0; q2 < Cfg::NP; ++q2) acc[j][q2] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // input chunks with at most 16 valid channels (the 8-channel padded image layer): only
  // the first 16-channel half carries data, so the 9 (tap, half 0) pairs are spread over
  // the waves instead of 18 pairs of which half are all-zero
  const bool half_only = p.Cin - ci0 <= 16;
  const int npairs = half_only ? 9 : 18;
  auto compute = [&](const char* __restrict__ Y, const char* __restrict__ X) {
#pragma unroll
    for (int ks = 0; ks < Cfg::KSTEPS; ++ks) {
      uint4 af[Cfg::NCO];
#pragma unroll
      for (int j = 0; j < Cfg::NCO; ++j) {
        const uint2 lo = lds_read_tr16(Y + ks * 32 * Cfg::Y_ROWB + ya[0][j]);
        const uint2 hi = lds_read_tr16(Y + ks * 32 * Cfg::Y_ROWB + ya[1][j]);
        af[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int pi = 0; pi < Cfg::NP; ++pi) {
        const int pair = wave + 4 * pi;                 // wave-uniform
        if (pair < npairs) {
          const int tap = half_only ? pair : pair >> 1, cih = half_only ? 0 : pair & 1;
          const int toff = ((tap / 3) * HW2 + tap % 3) * 64 + cih * 32;
          const uint2 lo = lds_read_tr16(X + xb[ks][0] + toff);
          const uint2 hi = lds_read_tr16(X + xb[ks][1] + toff);
          const uint4 bfr = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
          for (int j = 0; j < Cfg::NCO; ++j) acc[j][pi] = mfma16x16x32(af[j], bfr, acc[j][pi]);
        }
      }
    }
  };

  if (has_dyp) __syncthreads();                       // s_dy visible
  if (t_begin < t_end) issue(t_begin, 0);
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int buf = (tile - t_begin) & 1;
    dma_wait<0>();
    if (second ? has_pro2 : has_pro) transform(buf);
    if (has_dyp) transform_dy(buf);
    lds_sync();
    if (tile + 1 < t_end) issue(tile + 1, buf ^ 1);
    compute(sY(buf), sX(buf));
  }

  // ---- partial slab: part[split][co][tap][ci]
  float* out = p.partial + (long long)split * p.Cout * p.taps * p.Cin;
#pragma unroll
  for (int pi = 0; pi < Cfg::NP; ++pi) {
    const int pair = wave + 4 * pi;
    if (pair >= npairs) continue;
    const int tap = plane * 9 + (half_only ? pair : pair >> 1);
    const int ci = ci0 + (half_only ? 0 : (pair & 1) * 16) + (lane & 15);
#pragma unroll
    for (int j = 0; j < Cfg::NCO; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = co0 + j * 16 + 4 * g + i;
        if (co < p.Cout && ci < p.Cin) out[((long long)co * p.taps + tap) * p.Cin + ci] = acc[j][pi][i];
      }
  }
}

// ============================================================================ v3: 32x32x16 MFMA
// Same GEMM, tiles, DMA pipeline and partial-slab contract as v2, but the MFMA is
// v_mfma_f32_32x32x16_bf16 with M = 32 output channels and N = one tap x the 32-channel ci
// chunk.  That operand shape makes every transposed read conflict-free on the natural
// layouts: a 32-lane half-wave reads 4 consecutive pixel rows x 32 channels = 256
// contiguous bytes of the X halo (64-B rows, any tap shift) — v2's 16x16x32 B reads took 8
// pixels x 16 channels, 2-way bank conflicts on nearly every LDS instruction — and of dY
// (64-B rows for 32 channels; 128-B rows get a 64-B-half XOR on row bit 1).
// Waves split the pixel k-steps (BCO 32: 4-way; BCO 64: 2 co halves x 2-way), each wave
// holds all 9 taps (9 x 16 fp32 accumulators), and the k-split partials are summed in LDS
// in a fixed order at the end (deterministic).
template <int BCO>
DDLPC_DEVICE int wg3_yswz(int row) {             // XOR on the 16-B piece index
  // (256-B rows, 128 channels: the 64-B quarter XOR row bits 0-1 — the 4 consecutive rows a
  // 32-lane half-wave reads land in 4 different quarters of the bank row)
  return BCO == 128 ? ((row & 3) << 2) : BCO == 64 ? (((row >> 1) & 1) << 2) : 0;
}

// Stages: a double buffer, one full vmcnt drain per tile (rejected: a 3-deep ring with
// counted waits, 12-18% slower per layer: profiles/wgrad_micro_b128_ring*_s2.txt)
// CIW: 32-channel input chunks per workgroup (2: each staged dY tile feeds two X halos — the
// concat layers' many input chunks re-read dY half as often; the waves split (co tile, chunk)
// instead of the k-steps)
template <int BCO, int PT, int CIW = 1, bool PIPE = true>
__global__ __launch_bounds__(256, 2) void conv3_wgrad3_kernel(ConvWgradArgs p) {
  using namespace convlds;
  using Cfg = Wg2Cfg<BCO, PT>;                     // DMA geometry / LDS budget as v2
  constexpr int TH = Cfg::TH, HW2 = 18;
  constexpr int NJ = BCO / 32;                     // 32-channel co tiles
  constexpr int KW = 4 / (NJ * CIW);               // waves sharing a (co tile, chunk) (k-split)
  static_assert(NJ * CIW * KW == 4, "4 waves = co tiles x input chunks x k phases");
  constexpr int KS16 = PT / 16;                    // 16-pixel k-steps per tile
  static_assert(KS16 % KW == 0, "k-steps must split evenly over the waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* base = smem + Cfg::SS_BYTES;
  constexpr int STAGE = Cfg::Y_BYTES + CIW * Cfg::X_BYTES;
  auto sY = [&](int b) { return base + b * STAGE; };
  auto sX = [&](int b) { return base + b * STAGE + Cfg::Y_BYTES; };   // + cw * X_BYTES: chunk cw

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // (KW == 1: the k phase is the constant 0, so every fragment offset below is an immediate)
  const int wj = wave % NJ, wc = (wave / NJ) % CIW, wk = KW == 1 ? 0 : wave / (NJ * CIW);   // co tile, chunk, k phase
  int b = xcd_remap(blockIdx.x, gridDim.x);
  const int cic = b % p.ciChunks; b /= p.ciChunks;
  const int cot = b % p.coTiles; b /= p.coTiles;
  const int plane = b % p.planes; b /= p.planes;
  const int split = b;
  const int co0 = cot * BCO, ci0 = cic * BK * CIW;
  const int dshift = p.planes == 3 ? plane - 1 : 0;

  const bool has_pro = p.pscale != nullptr;
  const bool has_pro2 = p.pscale2 != nullptr;           // deferred skip: X2 channels at C1 + c
  const int t_begin = (int)((long long)p.nTiles * split / p.splits);
  const int t_end = (int)((long long)p.nTiles * (split + 1) / p.splits);
  const long long img_px = (long long)p.H * p.W;

  // ---- tile-independent per-lane DMA geometry (v2's, with the v3 dY swizzle)
  int y_pw[Cfg::Y_ITERS], y_ph[Cfg::Y_ITERS], y_rel[Cfg::Y_ITERS];
#pragma unroll
  for (int i = 0; i < Cfg::Y_ITERS; ++i) {
    const int e = (i * 4 + wave) * 64 + lane;
    const int row = e / (BCO / 8), pc = e % (BCO / 8);
    const int sp = pc ^ wg3_yswz<BCO>(row);
    y_pw[i] = row % 16;
    y_ph[i] = row / 16;
    const int co = co0 + sp * 8;
    y_rel[i] = co < p.Cout ? (y_ph[i] * p.W + y_pw[i]) * p.Cout + co : -1;
  }
  int x_dw[Cfg::X_ITERS], x_dh[Cfg::X_ITERS], x_pix[Cfg::X_ITERS];
#pragma unroll
  for (int i = 0; i < Cfg::X_ITERS; ++i) {
    const int e = (i * 4 + wave) * 64 + lane;
    const int px = e >> 2;
    x_dw[i] = px < Cfg::HALO ? px % HW2 - 1 : -(1 << 20);
    x_dh[i] = px / HW2 - 1;
    x_pix[i] = -1;
  }
  // per input chunk cw: source tensor, channel offset, validity, prologue constants
  bool second[CIW], xch_ok[CIW], xpro[CIW], xfull[CIW];
  int Cs[CIW], cs0[CIW];
  const bf16_t* xsrc[CIW];
  float psc[CIW][8] = {}, psh[CIW][8] = {};          // this lane's prologue constants
#pragma unroll
  for (int cw = 0; cw < CIW; ++cw) {
    const int cc = ci0 + cw * BK;
    const int c8l = cc + (lane & 3) * 8;
    second[cw] = cc >= p.C1;
    Cs[cw] = second[cw] ? p.C2 : p.C1;
    cs0[cw] = second[cw] ? c8l - p.C1 : c8l;
    xsrc[cw] = second[cw] ? p.X2 : p.X1;
    xch_ok[cw] = cs0[cw] < Cs[cw];
    xfull[cw] = (second[cw] ? cc - p.C1 : cc) + BK <= Cs[cw];   // the whole 32-channel chunk
    xpro[cw] = second[cw] ? has_pro2 : has_pro;
    if (xpro[cw])
      pro8_load(p.pscale, p.pshift, p.pscale2, p.pshift2, p.C1, c8l, second[cw] ? p.Cin : p.C1, psc[cw], psh[cw]);
  }

  // 32-channel tiles (one input chunk): the element offset of halo piece i relative to the
  // tile's first pixel, pieces outside the halo / past the channels pushed beyond any tensor
  // (>= 2^31 bytes: the DMA reads zeros) — an interior tile's DMAs need no per-piece test
  // (wave-uniform path; its prologue takes the batched unmasked form, so x_pix is not
  // refreshed).  enc1.b / dec1.a / dec1.b -6..-9%; the 64 / 128-channel tiles measured
  // 1-5% slower with it: profiles/r4/wgrad_ab_fastdma_r5c.txt
  constexpr bool FASTDMA = CIW == 1 && BCO == 32 && Cfg::X_ITERS <= 6;
  int x_relC[FASTDMA ? Cfg::X_ITERS : 1];
  if constexpr (FASTDMA) {
#pragma unroll
    for (int i = 0; i < Cfg::X_ITERS; ++i)
      x_relC[i] = x_dw[i] > -2 && xch_ok[0] ? (x_dh[i] * p.W + x_dw[i]) * Cs[0] + cs0[0] : (1 << 30);
  }
  const bool co_full = co0 + BCO <= p.Cout;          // every dY piece's channels exist
  TileWalk tw;                                     // the issue stream's tile geometry
  tw.init(t_begin, p.tilesW, p.tilesH, p.D);
  bool x_int = false;
  auto issue = [&](int tile, int buf) __attribute__((always_inline)) {
    tw.to(tile, p.tilesW, p.tilesH, p.D);
    const int n = tw.n;
    const int dx = tw.d + dshift;
    const bool dok = dx >= 0 && dx < p.D;
    const int h0 = tw.h * TH, w0 = tw.w * 16;
    x_int = dok && h0 >= 1 && w0 >= 1 && h0 + TH < p.H && w0 + 16 < p.W;
    const auto ry = make_rsrc(p.dY + n * img_px * p.Cout, (unsigned)(img_px * p.Cout * 2));
    const int ybase = (h0 * p.W + w0) * p.Cout;
    if (FASTDMA && x_int && co_full && xfull[0]) {
      // interior tile, full channel tiles: no per-piece tests (x_pix is not needed: the
      // prologue of such a tile takes its unmasked path)
#pragma unroll
      for (int i = 0; i < Cfg::Y_ITERS; ++i) {
        if ((i * 4 + wave) >= Cfg::Y_INSTR) break;
        dma16(ry, sY(buf) + (i * 4 + wave) * 1024, (unsigned)(ybase + y_rel[i]) * 2u);
      }
      const auto rx = make_rsrc(xsrc[0] + (n + dshift) * img_px * Cs[0], (unsigned)(img_px * Cs[0] * 2));
      const int xbase = (h0 * p.W + w0) * Cs[0];
#pragma unroll
      for (int i = 0; i < Cfg::X_ITERS; ++i) {
        if ((i * 4 + wave) >= Cfg::X_INSTR) break;
        dma16(rx, sX(buf) + (i * 4 + wave) * 1024, (unsigned)(xbase + x_relC[i]) * 2u);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < Cfg::Y_ITERS; ++i) {
      if ((i * 4 + wave) >= Cfg::Y_INSTR) break;
      const bool ok = y_rel[i] >= 0 && w0 + y_pw[i] < p.W && h0 + y_ph[i] < p.H;
      dma16(ry, sY(buf) + (i * 4 + wave) * 1024, ok ? (unsigned)(ybase + y_rel[i]) * 2u : kOOB);
    }
#pragma unroll
    for (int i = 0; i < Cfg::X_ITERS; ++i) {
      if ((i * 4 + wave) >= Cfg::X_INSTR) break;
      const int gw = w0 + x_dw[i], gh = h0 + x_dh[i];
      x_pix[i] = (gw >= 0 && gw < p.W && gh >= 0 && gh < p.H && dok) ? gh * p.W + gw : -1;
    }
#pragma unroll
    for (int cw = 0; cw < CIW; ++cw) {
      const auto rx = make_rsrc(xsrc[cw] + (n + (dok ? dshift : 0)) * img_px * Cs[cw],
                                (unsigned)(img_px * Cs[cw] * 2));
#pragma unroll
      for (int i = 0; i < Cfg::X_ITERS; ++i) {
        if ((i * 4 + wave) >= Cfg::X_INSTR) break;
        const bool ok = x_pix[i] >= 0 && xch_ok[cw];
        dma16(rx, sX(buf) + cw * Cfg::X_BYTES + (i * 4 + wave) * 1024,
              ok ? (unsigned)(x_pix[i] * Cs[cw] + cs0[cw]) * 2u : kOOB);
      }
    }
  };
  // x_pix still holds this tile's validity (the next tile's DMA is issued after the barrier
  // that follows this transform); x_int: the tile's whole halo lies inside the image
  auto transform = [&](char* __restrict__ X0) __attribute__((always_inline)) {
    // (batched form on the 32-output-channel tiles: enc1.b / dec1.b -7%; the 64 / 128-channel
    // tiles measured 0-2% slower with it, profiles/r3s/wgrad_xform_ab_b256_r3s36.txt)
    if (Cfg::X_ITERS <= 6 && BCO == 32) {
      // batched form: all piece reads issue before the math (packed fp32 FMA, bf16 rounding,
      // ReLU as a packed 16-bit max), padding re-zeroed by a select instead of a branch —
      // none at all on an interior tile with a full chunk (wave-uniform; pieces past the
      // halo are never read)
      constexpr int NI = Cfg::X_ITERS <= 6 ? Cfg::X_ITERS : 1;
      auto run = [&](char* __restrict__ X, int cw, auto maskc) __attribute__((always_inline)) {
        constexpr bool MASK = decltype(maskc)::value;
        uint4 v[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i)
          if ((i * 4 + wave) < Cfg::X_INSTR) v[i] = *reinterpret_cast<const uint4*>(X + ((i * 4 + wave) * 64 + lane) * 16);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          if ((i * 4 + wave) >= Cfg::X_INSTR) break;
          const bool ok = !MASK || (x_pix[i] >= 0 && xch_ok[cw]);
          const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
          uint32_t o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x2_t x = {lo_bf(w[j]), hi_bf(w[j])};
            const f32x2_t sc2 = {psc[cw][2 * j], psc[cw][2 * j + 1]};
            const f32x2_t sh2 = {psh[cw][2 * j], psh[cw][2 * j + 1]};
            const f32x2_t y2 = __builtin_elementwise_fma(x, sc2, sh2);
            const uint32_t pk = __builtin_bit_cast(uint32_t, __builtin_convertvector(y2, bf16x2_t));
            const i16x2_t m = __builtin_elementwise_max(__builtin_bit_cast(i16x2_t, pk), i16x2_t{0, 0});
            o[j] = ok ? __builtin_bit_cast(uint32_t, m) : 0u;
          }
          *reinterpret_cast<uint4*>(X + ((i * 4 + wave) * 64 + lane) * 16) = make_uint4(o[0], o[1], o[2], o[3]);
        }
      };
#pragma unroll
      for (int cw = 0; cw < CIW; ++cw) {
        if (!xpro[cw]) continue;
        if (x_int && xfull[cw]) run(X0 + cw * Cfg::X_BYTES, cw, std::false_type{});
        else run(X0 + cw * Cfg::X_BYTES, cw, std::true_type{});
      }
      return;
    }
#pragma unroll
    for (int cw = 0; cw < CIW; ++cw) {
      if (!xpro[cw]) continue;
      char* X = X0 + cw * Cfg::X_BYTES;
#pragma unroll
      for (int i = 0; i < Cfg::X_ITERS; ++i) {
        const int e = (i * 4 + wave) * 64 + lane;
        const bool ok = x_pix[i] >= 0 && xch_ok[cw];
        if ((i * 4 + wave) < Cfg::X_INSTR && ok) {
          uint4* q = reinterpret_cast<uint4*>(X + e * 16);
          float f[8];
          unpack8(*q, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], psc[cw][j], psh[cw][j]), 0.0f);
          *q = pack8(f);
        }
      }
    }
  };
  bool any_pro = false;
#pragma unroll
  for (int cw = 0; cw < CIW; ++cw) any_pro = any_pro || xpro[cw];

  // ---- per-lane transposed-read geometry.  16-lane group g4 = lane >> 4: columns
  // (g4 & 1) * 16 + 4 * pq, pixel rows (g4 >> 1) * 8 + 4 * h + q within the 16-pixel k-step
  // (Rejected: on the 128-channel tiles, waves splitting (co half, tap group) instead of co
  // quarters — 2 dY + 5 X fragment reads per 9 MFMAs instead of 1 + 9 — measured 14-23%
  // slower per layer: profiles/r4/wgrad_ab_tapsplit_r4r.txt)
  const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  int ya[2], xb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = (g4 >> 1) * 8 + 4 * h + q;     // + 16 * ks (row bits 0..3 unchanged)
    const int byte = wj * 64 + (g4 & 1) * 32 + 8 * pq;
    const int pc = (byte >> 4) ^ wg3_yswz<BCO>(row);
    ya[h] = row * Cfg::Y_ROWB + (pc << 4) + (byte & 15);
    xb[h] = row * 64 + (g4 & 1) * 32 + 8 * pq;      // halo pixel row (+ 18 * ks + tap offset)
    // the wave's k phase folded in: k-step ks = kk * KW + wk, the kk terms are immediates
    // (row bits 0..3 and the swizzle are unchanged by whole 16-pixel k-steps)
    ya[h] += wk * 16 * Cfg::Y_ROWB;
    xb[h] += wk * HW2 * 64;
  }
  f32x16_t acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  auto compute = [&](const char* __restrict__ Y, const char* __restrict__ X0) __attribute__((always_inline)) {
    const char* X = X0 + wc * Cfg::X_BYTES;          // this wave's input chunk
    if constexpr (PIPE) {
      // software-pipelined: the (k-step, tap) sequence flattened, the X fragment of step i + LA
      // (and the dY fragment of the next k-step) read before the MFMA of step i — LA MFMAs
      // of LDS latency cover instead of none (the plain loop waits lgkmcnt(0) before every
      // MFMA: the compiler keeps one fragment in flight at 222-240 VGPRs)
      constexpr int NI = KS16 / KW * 9, LA = 3;      // LA: X-fragment lookahead (steps)
      uint4 af[2], bq[LA + 1];
      auto ldA = [&](int kk, uint4& a) __attribute__((always_inline)) {
        const int ks = kk * KW;                      // (+ wk: in ya)
        const uint2 lo = lds_read_tr16(Y + ks * 16 * Cfg::Y_ROWB + ya[0]);
        const uint2 hi = lds_read_tr16(Y + ks * 16 * Cfg::Y_ROWB + ya[1]);
        a = make_uint4(lo.x, lo.y, hi.x, hi.y);
      };
      auto ldB = [&](int i, uint4& b) __attribute__((always_inline)) {
        const int ks = (i / 9) * KW, tap = i % 9;    // (+ wk: in xb)
        const int toff = (ks * HW2 + (tap / 3) * HW2 + tap % 3) * 64;
        const uint2 lo = lds_read_tr16(X + toff + xb[0]);
        const uint2 hi = lds_read_tr16(X + toff + xb[1]);
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
        acc[i % 9] = mfma32x32x16(af[(i / 9) & 1], bq[i % (LA + 1)], acc[i % 9]);
        __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
#pragma unroll
    for (int kk = 0; kk < KS16 / KW; ++kk) {
      const int ks = kk * KW;                        // (+ wk: in ya / xb)
      const uint2 alo = lds_read_tr16(Y + ks * 16 * Cfg::Y_ROWB + ya[0]);
      const uint2 ahi = lds_read_tr16(Y + ks * 16 * Cfg::Y_ROWB + ya[1]);
      const uint4 af = make_uint4(alo.x, alo.y, ahi.x, ahi.y);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = (ks * HW2 + (tap / 3) * HW2 + tap % 3) * 64;
        const uint2 lo = lds_read_tr16(X + toff + xb[0]);
        const uint2 hi = lds_read_tr16(X + toff + xb[1]);
        acc[tap] = mfma32x32x16(af, make_uint4(lo.x, lo.y, hi.x, hi.y), acc[tap]);
      }
    }
  };

  // BN groups (ConvWgradArgs::groups, X1 prologue only): the tile's image decides its group;
  // a workgroup's tiles are contiguous, so the constants reload only at a group boundary —
  // after the full drain below, with no DMA in flight
  // (v3 chunks are whole 32-channel chunks of X1: the lane's 8 constants are two float4s)
  int grp_end = p.groups > 1 ? p.gimg : (1 << 30);  // first image past the current group
  long long goff = 0;
  if (t_begin < t_end) issue(t_begin, 0);
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int buf = (tile - t_begin) & 1;
    dma_wait<0>();
    if (tw.n >= grp_end) {                           // (tw: this tile, the last one issued)
      while (tw.n >= grp_end) { grp_end += p.gimg; goff += p.gstride; }
      const float4* bs = reinterpret_cast<const float4*>(p.pscale + goff + ci0 + (lane & 3) * 8);
      const float4* bh = reinterpret_cast<const float4*>(p.pshift + goff + ci0 + (lane & 3) * 8);
#pragma unroll
      for (int cw = 0; cw < CIW; ++cw) {
        const float4 s0 = bs[cw * BK / 4], s1 = bs[cw * BK / 4 + 1];
        const float4 h0 = bh[cw * BK / 4], h1 = bh[cw * BK / 4 + 1];
        psc[cw][0] = s0.x; psc[cw][1] = s0.y; psc[cw][2] = s0.z; psc[cw][3] = s0.w;
        psc[cw][4] = s1.x; psc[cw][5] = s1.y; psc[cw][6] = s1.z; psc[cw][7] = s1.w;
        psh[cw][0] = h0.x; psh[cw][1] = h0.y; psh[cw][2] = h0.z; psh[cw][3] = h0.w;
        psh[cw][4] = h1.x; psh[cw][5] = h1.y; psh[cw][6] = h1.z; psh[cw][7] = h1.w;
      }
    }
    if (any_pro) transform(sX(buf));
    lds_sync();
    if (tile + 1 < t_end) issue(tile + 1, buf ^ 1);
    compute(sY(buf), sX(buf));
  }

  // ---- k-split reduction over the KW waves of each co tile (fixed order, in LDS, one tap
  // group at a time), then the partial slab part[split][co][tap][ci]
  dma_wait<0>();
  lds_sync();
  float* red = reinterpret_cast<float*>(base);     // [KW-1][NJ * CIW][3 taps][16][64] floats
  const int wjc = wc * NJ + wj;                    // (chunk, co tile) of this wave
  float* out = p.partial + (long long)split * p.Cout * p.taps * p.Cin;
#pragma unroll
  for (int tg = 0; tg < 3; ++tg) {
    if (wk > 0) {
#pragma unroll
      for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          red[((((wk - 1) * NJ * CIW + wjc) * 3 + t3) * 16 + i) * 64 + lane] = acc[tg * 3 + t3][i];
    }
    lds_sync();
    if (wk == 0) {
#pragma unroll
      for (int t3 = 0; t3 < 3; ++t3) {
        const int tap = plane * 9 + tg * 3 + t3;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float v = acc[tg * 3 + t3][i];
#pragma unroll
          for (int w2 = 1; w2 < KW; ++w2) v += red[((((w2 - 1) * NJ * CIW + wjc) * 3 + t3) * 16 + i) * 64 + lane];
          // D layout of 32x32: column n = lane & 31 (ci), row m = 8 (i / 4) + 4 (lane >> 5) + i % 4
          const int co = co0 + wj * 32 + 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
          const int ci = ci0 + wc * BK + (lane & 31);
          if (co < p.Cout && ci < p.Cin) out[((long long)co * p.taps + tap) * p.Cin + ci] = v;
        }
      }
    }
    lds_sync();
  }
}

// ============================================================================ image layer
// The first conv's weight gradient (2-D, one 8-channel padded image of which at most 4
// channels are real: ref.py:588's Conv2d(3, 32)).  v2 runs it as 9 taps x a 16-channel half
// chunk (9 x 2 MFMA per 32-pixel k-step, 13 of every 16 columns zero).  Here the GEMM's N
// packs (tap, channel) as n = 4 tap + c (c < 4): three 16-wide MFMA tiles (taps 0-3, 4-7,
// 8; columns of taps 9-11 are computed from tap 8's pixels and discarded), a third of the
// MFMA work.  Each lane of a transposed B read supplies its own row address, so a tap's 4
// channels (8 bytes) are gathered straight from the 16-B-per-pixel halo rows — no im2col.
// dY arrives and is optionally BN-backward-transformed exactly as in v2 (same layout, same
// swizzle); the waves split the k-steps and their partials are summed in LDS in a fixed
// order; the slab keeps the [co][tap][ci] contract with ci >= 4 written as zeros.
// 3-D (Conv3d(3, 32)): one workgroup per depth tap plane as in v2 / v3 — the 2-D kernel over
// depth slices, the input slice shifted by the plane, writing taps 9 plane + t.
template <int BCO, int PT>
struct WgImgCfg {
  using Y = Wg2Cfg<BCO, PT>;                       // dY staging exactly as v2
  static constexpr int TH = PT / 16;
  static constexpr int HALO = (TH + 2) * 18;       // one 16-B piece (8 channels) per pixel
  static constexpr int X_INSTR = (HALO + 63) / 64;
  static constexpr int X_ITERS = (X_INSTR + 3) / 4;
  static constexpr int X_BYTES = X_INSTR * 1024;
  static constexpr int STAGE = Y::Y_BYTES + X_BYTES;
  static constexpr int RED_BYTES = 3 * (BCO / 16) * 3 * 4 * 64 * 4;   // k-split partials of waves 1-3
  static constexpr int SMEM = Y::SS_BYTES + (2 * STAGE > RED_BYTES ? 2 * STAGE : RED_BYTES);
  static constexpr int KSTEPS = PT / 32;
};

template <int BCO, int PT>
__global__ __launch_bounds__(256, 2) void conv3_wgrad_img_kernel(ConvWgradArgs p) {
  using namespace convlds;
  using Cfg = WgImgCfg<BCO, PT>;
  using YC = typename Cfg::Y;
  constexpr int NCO = BCO / 16, HW2 = 18;
  static_assert(Cfg::KSTEPS % 4 == 0, "k-steps split evenly over the 4 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_dy = reinterpret_cast<float*>(smem) + 1024;   // dY-prologue table (v2's offset)
  char* base = smem + YC::SS_BYTES;
  auto sY = [&](int b) { return base + b * Cfg::STAGE; };
  auto sX = [&](int b) { return base + b * Cfg::STAGE + YC::Y_BYTES; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int b = xcd_remap(blockIdx.x, gridDim.x);
  const int cot = b % p.coTiles; b /= p.coTiles;
  const int plane = b % p.planes; b /= p.planes;
  const int split = b;
  const int co0 = cot * BCO;
  const int dshift = p.planes == 3 ? plane - 1 : 0;

  const bool has_dyp = p.dyy != nullptr;
  if (has_dyp)
    for (int i = tid; i < BCO; i += 256) {
      const int c = co0 + i;
      const bool ok = c < p.Cout;
      const float is = ok ? p.dys4[p.Cout + c] : 0.f;
      s_dy[i] = ok ? p.dys4[2 * p.Cout + c] : 0.f;
      s_dy[BCO + i] = ok ? p.dys4[3 * p.Cout + c] : 0.f;
      s_dy[2 * BCO + i] = is;
      s_dy[3 * BCO + i] = ok ? -p.dys4[c] * is : 0.f;
      s_dy[4 * BCO + i] = ok ? p.dycoef[c] : 0.f;
      s_dy[5 * BCO + i] = ok ? p.dycoef[p.Cout + c] : 0.f;
      s_dy[6 * BCO + i] = ok ? p.dycoef[2 * p.Cout + c] : 0.f;
    }
  const int t_begin = (int)((long long)p.nTiles * split / p.splits);
  const int t_end = (int)((long long)p.nTiles * (split + 1) / p.splits);
  const long long img_px = (long long)p.H * p.W;

  // ---- tile-independent per-lane DMA geometry
  int y_pw[YC::Y_ITERS], y_ph[YC::Y_ITERS], y_rel[YC::Y_ITERS];
  uint4 yv[YC::Y_ITERS];
  bool y_ok[YC::Y_ITERS];
#pragma unroll
  for (int i = 0; i < YC::Y_ITERS; ++i) {
    const int e = (i * 4 + wave) * 64 + lane;
    const int row = e / (BCO / 8), pc = e % (BCO / 8);
    const int sp = pc ^ wg2_yswz<BCO>(row);
    y_pw[i] = row % 16;
    y_ph[i] = row / 16;
    const int co = co0 + sp * 8;
    y_rel[i] = co < p.Cout ? (y_ph[i] * p.W + y_pw[i]) * p.Cout + co : -1;
    y_ok[i] = false;
  }
  TileWalk tw;                                     // the issue stream's tile geometry
  tw.init(t_begin, p.tilesW, p.tilesH, p.D);
  auto issue = [&](int tile, int buf) {
    tw.to(tile, p.tilesW, p.tilesH, p.D);
    const int n = tw.n;                              // (image, d) slice
    const int dx = tw.d + dshift;
    const bool dok = dx >= 0 && dx < p.D;            // the plane's input slice exists
    const int h0 = tw.h * Cfg::TH, w0 = tw.w * 16;
    const auto ry = make_rsrc(p.dY + n * img_px * p.Cout, (unsigned)(img_px * p.Cout * 2));
    const int ybase = (h0 * p.W + w0) * p.Cout;
#pragma unroll
    for (int i = 0; i < YC::Y_ITERS; ++i) {
      if ((i * 4 + wave) >= YC::Y_INSTR) break;
      const bool ok = y_rel[i] >= 0 && w0 + y_pw[i] < p.W && h0 + y_ph[i] < p.H;
      dma16(ry, sY(buf) + (i * 4 + wave) * 1024, ok ? (unsigned)(ybase + y_rel[i]) * 2u : kOOB);
      if (has_dyp) {
        const auto ryy = make_rsrc(p.dyy + n * img_px * p.Cout, (unsigned)(img_px * p.Cout * 2));
        const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(ryy, ok ? (unsigned)(ybase + y_rel[i]) * 2u : kOOB, 0, 0);
        yv[i] = make_uint4(v.x, v.y, v.z, v.w);
        y_ok[i] = ok;
      }
    }
    const auto rx = make_rsrc(p.X1 + (n + (dok ? dshift : 0)) * img_px * p.C1, (unsigned)(img_px * p.C1 * 2));
#pragma unroll
    for (int i = 0; i < Cfg::X_ITERS; ++i) {
      if ((i * 4 + wave) >= Cfg::X_INSTR) break;
      const int px = (i * 4 + wave) * 64 + lane;          // halo pixel (one piece each)
      const int gw = w0 + px % HW2 - 1, gh = h0 + px / HW2 - 1;
      const bool ok = dok && px < Cfg::HALO && gw >= 0 && gw < p.W && gh >= 0 && gh < p.H;
      dma16(rx, sX(buf) + (i * 4 + wave) * 1024, ok ? (unsigned)(gh * p.W + gw) * (unsigned)(p.C1 * 2) : kOOB);
    }
  };
  // dY = k (dA [y*scale + shift > 0] - m1 - xhat m2) on the lane's own landed pieces (v2's)
  auto transform_dy = [&](int buf) {
#pragma unroll
    for (int i = 0; i < YC::Y_ITERS; ++i) {
      if ((i * 4 + wave) < YC::Y_INSTR && y_ok[i]) {
        const int e = (i * 4 + wave) * 64 + lane;
        const int row = e / (BCO / 8), pc = e % (BCO / 8);
        const int cl = (pc ^ wg2_yswz<BCO>(row)) * 8;
        uint4* qd = reinterpret_cast<uint4*>(sY(buf) + e * 16);
        float fd[8], fy[8], o[8];
        unpack8(*qd, fd);
        unpack8(yv[i], fy);
        const float* t = s_dy + opaque_zero() + cl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = fmaf(fy[j], t[j], t[BCO + j]);
          const float dyh = a > 0.f ? fd[j] : 0.f;
          const float xh = fmaf(fy[j], t[2 * BCO + j], t[3 * BCO + j]);
          o[j] = t[4 * BCO + j] * (dyh - t[5 * BCO + j] - xh * t[6 * BCO + j]);
        }
        *qd = pack8(o);
      }
    }
  };

  // ---- transposed-read geometry: 16-lane group g, row q within 4, column quad pp
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  int ya[2][NCO];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < NCO; ++j) {
      const int row = 8 * g + 4 * h + q;
      const int pc = 2 * j + (pp >> 1);
      ya[h][j] = row * YC::Y_ROWB + ((pc ^ wg2_yswz<BCO>(row)) << 4) + (pp & 1) * 8;
    }
  // B: column quad pp of tile n = tap 4n + pp (taps past 8 re-read tap 8: discarded columns)
  int toff[3];
#pragma unroll
  for (int n = 0; n < 3; ++n) {
    const int tap = min(4 * n + pp, 8);
    toff[n] = ((tap / 3) * HW2 + tap % 3) * 16;
  }
  constexpr int KW = Cfg::KSTEPS / 4;              // k-steps per wave per tile
  int xb[KW][2];
#pragma unroll
  for (int kk = 0; kk < KW; ++kk)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pix = (kk * 4 + wave) * 32 + 8 * g + 4 * h + q;
      xb[kk][h] = ((pix / 16) * HW2 + pix % 16) * 16;
    }

  f32x4_t acc[NCO][3];
#pragma unroll
  for (int j = 0; j < NCO; ++j)
#pragma unroll
    for (int n = 0; n < 3; ++n) acc[j][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const char* __restrict__ Y, const char* __restrict__ X) {
#pragma unroll
    for (int kk = 0; kk < KW; ++kk) {
      const int ks = kk * 4 + wave;
      uint4 af[NCO];
#pragma unroll
      for (int j = 0; j < NCO; ++j) {
        const uint2 lo = lds_read_tr16(Y + ks * 32 * YC::Y_ROWB + ya[0][j]);
        const uint2 hi = lds_read_tr16(Y + ks * 32 * YC::Y_ROWB + ya[1][j]);
        af[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int n = 0; n < 3; ++n) {
        const uint2 lo = lds_read_tr16(X + xb[kk][0] + toff[n]);
        const uint2 hi = lds_read_tr16(X + xb[kk][1] + toff[n]);
        const uint4 bfr = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
        for (int j = 0; j < NCO; ++j) acc[j][n] = mfma16x16x32(af[j], bfr, acc[j][n]);
      }
    }
  };

  if (has_dyp) __syncthreads();                       // s_dy visible
  if (t_begin < t_end) issue(t_begin, 0);
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int buf = (tile - t_begin) & 1;
    dma_wait<0>();
    if (has_dyp) transform_dy(buf);
    lds_sync();
    if (tile + 1 < t_end) issue(tile + 1, buf ^ 1);
    compute(sY(buf), sX(buf));
  }

  // ---- k-split reduction over the 4 waves (fixed order), then the partial slab
  dma_wait<0>();
  lds_sync();
  float* red = reinterpret_cast<float*>(base);        // [3][NCO][3][4][64]
  if (wave > 0) {
#pragma unroll
    for (int j = 0; j < NCO; ++j)
#pragma unroll
      for (int n = 0; n < 3; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[((((wave - 1) * NCO + j) * 3 + n) * 4 + i) * 64 + lane] = acc[j][n][i];
  }
  lds_sync();
  float* out = p.partial + (long long)split * p.Cout * p.taps * p.Cin;
  if (wave == 0) {
#pragma unroll
    for (int j = 0; j < NCO; ++j)
#pragma unroll
      for (int n = 0; n < 3; ++n) {
        const int col = 16 * n + (lane & 15);           // n = 4 tap + c
        const int tap = col >> 2, ci = col & 3;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[j][n][i];
#pragma unroll
          for (int w2 = 1; w2 < 4; ++w2) v += red[((((w2 - 1) * NCO + j) * 3 + n) * 4 + i) * 64 + lane];
          const int co = co0 + j * 16 + 4 * g + i;
          if (tap < 9 && co < p.Cout && ci < p.Cin) out[((long long)co * p.taps + plane * 9 + tap) * p.Cin + ci] = v;
        }
      }
  }
  // padding input channels (4 .. Cin-1: zero in the image, so their gradient is exactly 0)
  for (int e = tid; e < BCO * 9 * (p.Cin - 4); e += 256) {
    const int ci = 4 + e % (p.Cin - 4), tap = plane * 9 + (e / (p.Cin - 4)) % 9, co = co0 + e / ((p.Cin - 4) * 9);
    if (co < p.Cout) out[((long long)co * p.taps + tap) * p.Cin + ci] = 0.f;
  }
}

template <int DIMS, int BCO>
void launch_wg(ConvWgradArgs& a, hipStream_t st) {
  using Cfg = WgCfg<DIMS, BCO>;
  const int grid = a.coTiles * a.ciChunks * a.planes * a.splits;
  hipLaunchKernelGGL((conv3_wgrad_kernel<DIMS, BCO>), dim3(grid), dim3(256), Cfg::SMEM, st, a);
}

}  // namespace

// pixel-tile size of the 2-D v2 kernel.  BCO 64: 128-pixel tiles (two 60 KB workgroups per
// CU) except for the large concat layers (two input tensors, >= 64x64 images), which measured
// 25% faster with 96-pixel tiles (three 46 KB workgroups per CU) and slower elsewhere
// (conv_micro, batch 128)
int conv3_wgrad2_pt(int bco, int C2, int H, int W) {
  if (bco == 32) return 256;
  return (C2 > 0 && H * W >= 64 * 64) ? 96 : 128;
}
void conv3_wgrad2_launch(ConvWgradArgs& a, int bco, hipStream_t st) {
  const int grid = a.coTiles * a.ciChunks * a.planes * a.splits;
  const int pt = a.TH * 16;
  if (bco == 32)
    hipLaunchKernelGGL((conv3_wgrad2_kernel<32, 256>), dim3(grid), dim3(256), (Wg2Cfg<32, 256>::SMEM), st, a);
  else if (pt == 96)
    hipLaunchKernelGGL((conv3_wgrad2_kernel<64, 96>), dim3(grid), dim3(256), (Wg2Cfg<64, 96>::SMEM), st, a);
  else
    hipLaunchKernelGGL((conv3_wgrad2_kernel<64, 128>), dim3(grid), dim3(256), (Wg2Cfg<64, 128>::SMEM), st, a);
}

// v3 tiles: 32 output channels on 256-pixel tiles; 64 on 128-pixel tiles, or two 32-channel
// input chunks per workgroup on 96-pixel tiles (ciw 2); 128 on 96-pixel tiles.  (Rejected:
// 128-pixel 32-channel tiles with a 3-deep ring, 12-18% slower per layer:
// profiles/wgrad_micro_b128_ring*_s2.txt.)
// (the compute loop is always the software-pipelined one: the plain loop measured 2-9%
// slower per layer, profiles/r5/wgrad_pipe/)
void conv3_wgrad3_launch(ConvWgradArgs& a, int bco, hipStream_t st) {
  constexpr bool PIPE = true;
  const int grid = a.coTiles * a.ciChunks * a.planes * a.splits;
  // (64 output channels x two input chunks, 96-pixel tiles: dY + two halos per stage)
  constexpr int SMEM64C2 = Wg2Cfg<64, 96>::SS_BYTES + 2 * (Wg2Cfg<64, 96>::Y_BYTES + 2 * Wg2Cfg<64, 96>::X_BYTES);
  static_assert(2 * SMEM64C2 <= 160 * 1024, "two workgroups per CU");
  if (a.TH * 16 != (bco == 32 ? 256 : (bco == 128 || a.ciw == 2) ? 96 : 128))
    throw std::runtime_error("conv3_wgrad3_launch: pixel tile does not match the v3 variant");
  if (bco == 32)
    hipLaunchKernelGGL((conv3_wgrad3_kernel<32, 256, 1, PIPE>), dim3(grid), dim3(256), (Wg2Cfg<32, 256>::SMEM), st, a);
  else if (bco == 64 && a.ciw == 2)   // two input chunks per workgroup, 96-pixel tiles
    hipLaunchKernelGGL((conv3_wgrad3_kernel<64, 96, 2, PIPE>), dim3(grid), dim3(256), SMEM64C2, st, a);
  else if (bco == 128)   // 96-pixel tiles: two 74 KB workgroups per CU
    hipLaunchKernelGGL((conv3_wgrad3_kernel<128, 96, 1, PIPE>), dim3(grid), dim3(256), (Wg2Cfg<128, 96>::SMEM), st, a);
  else
    hipLaunchKernelGGL((conv3_wgrad3_kernel<64, 128, 1, PIPE>), dim3(grid), dim3(256), (Wg2Cfg<64, 128>::SMEM), st, a);
}

void conv3_wgrad_img_launch(ConvWgradArgs& a, int bco, hipStream_t st) {
  const int grid = a.coTiles * a.planes * a.splits;
  if (bco == 32)
    hipLaunchKernelGGL((conv3_wgrad_img_kernel<32, 256>), dim3(grid), dim3(256), (WgImgCfg<32, 256>::SMEM), st, a);
  else
    hipLaunchKernelGGL((conv3_wgrad_img_kernel<64, 128>), dim3(grid), dim3(256), (WgImgCfg<64, 128>::SMEM), st, a);
}
int conv3_wgrad_img_pt(int bco) { return bco == 32 ? 256 : 128; }

void conv3_wgrad_launch(ConvWgradArgs& a, int bco, hipStream_t st) {
  if (a.dims == 2) {
    if (bco == 32) launch_wg<2, 32>(a, st); else launch_wg<2, 64>(a, st);
  } else {
    if (bco == 32) launch_wg<3, 32>(a, st); else launch_wg<3, 64>(a, st);
  }
}

int conv3_wgrad_halo_cap(int dims) { return dims == 2 ? WgHalo<2>::value : WgHalo<3>::value; }

}  // namespace ddlpc
