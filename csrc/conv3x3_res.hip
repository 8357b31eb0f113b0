// 3x3 2-D convolution (stride 1, pad 1) for the HIGH-RESOLUTION, FEW-CHANNEL U-Net layers
// (256^2 / 128^2 x 32..96 channels: enc1, enc2, dec2.b, dec1 and their data gradients) —
// the layers where the streaming kernel (conv3x3_fwd.hip) spends most of its time on
// per-stage overhead rather than MFMA work.  Reference ops: DoubleConv's nn.Conv2d(k=3,
// padding=1) (ref.py:579,582) and the first conv on the 3-channel image (ref.py:588).
//
// Design (MI355X / gfx950):
//   * RESIDENT WEIGHTS: every workgroup is persistent and owns ONE output-channel tile, so
//     all its weights (9 taps x Cin x BN bf16, <= ~74 KB) are DMA'd into LDS once and stay
//     there; only the input halo streams;
//   * one pipeline stage = (pixel tile, 32-channel chunk) with ALL 9 taps: 9*MT*NT MFMAs
//     per wave per stage behind ONE barrier (the streaming kernel: 3 taps per barrier);
//   * the halo of stage s+1 is in flight (LDS-DMA, double-buffered) while stage s computes;
//   * the BatchNorm+ReLU prologue of the previous layer is applied in LDS by the lane that
//     DMA'd each 16-B piece, right after its own DMA lands and BEFORE the stage barrier —
//     no extra barrier (padding stays zero);
//   * the epilogue of a tile (bias, bf16, 8-B stores, BN (sum, sum^2) in registers) runs
//     after the NEXT stage's barrier, just before that stage's DMA is issued, so its stores
//     drain under the next tile's compute instead of stalling the next vmcnt wait;
//   * TAP8 (the image layer, Cin <= 8): K packs (tap, channel) as k = 8*tap + c, 12 taps
//     (3 zero-weight) = 3 MFMA k-steps instead of 9 on a 4x zero-padded chunk; the halo row
//     is one 16-B pixel.  TAP8 = 3: the 3-D image layer (ref.py:588 with Conv3d) as depth
//     slices — an item is a TH x TW tile of one slice, its halo the 3 neighbouring planes,
//     28 taps (1 zero-weight) = 7 k-steps instead of 27 on a 4x zero-padded chunk.
// Output / statistics contracts are those of conv3_fwd_kernel (ops.h ConvFwdArgs).
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

#include <type_traits>

namespace ddlpc {

namespace {

using namespace convlds;

template <int WM, int WN, int MT, int NT, int HALO, int TAP8, int NBUF>
struct RCfg {
  static constexpr int NW = WM * WN;
  static constexpr int NTH = NW * 64;
  static constexpr int BM = WM * MT * 16;
  static constexpr int BN = WN * NT * 16;
  static constexpr int PIECES = TAP8 ? HALO : HALO * 4;   // 16-B pieces per halo buffer
  static constexpr int INSTR = (PIECES + 63) / 64;         // DMA wave-instructions per halo
  // EVERY wave issues exactly A_ITERS DMA instructions per stage (surplus ones land
  // zeros past the halo), so the counted vmcnt waits below are exact
  static constexpr int A_ITERS = (INSTR + NW - 1) / NW;
  static constexpr int A_BYTES = A_ITERS * NW * 1024;
};

template <int N>
DDLPC_DEVICE void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

DDLPC_HOST_DEVICE int res_ss_bytes(int C1, bool pro) { return pro ? ((8 * C1 + 15) / 16) * 16 : 0; }
DDLPC_HOST_DEVICE constexpr int tap8_ksteps(int tap8) { return tap8 == 3 ? 7 : 3; }
DDLPC_HOST_DEVICE int res_w_bytes(int Cin, int BN, int tap8) {
  return tap8 ? tap8_ksteps(tap8) * BN * ROWB : ((Cin + BK - 1) / BK) * 9 * BN * ROWB;
}

// SPLIT: 0 = one output; 1 = two outputs (concat data gradient), 8-byte stores; 2 = two
// outputs split at a 32-channel boundary (Co1 % 32 == 0, launcher-checked): 16-byte pair
// stores, each pair wholly in one output (a quarter of mode 1's store instructions)
// BNB: the BN-backward epilogue (statistics of dA against y).  (Rejected: the epilogue
// interleaved between the next stage's tap steps from a second accumulator set, 10-20%
// slower: profiles/r3s/res_ilv_ab_b256_r3s24.txt)
template <int WM, int WN, int MT, int NT, int HALO, int TAP8, int NBUF, int SPLIT, bool BNB>
__global__ __launch_bounds__(WM * WN * 64, WM * WN == 4 ? 2 : 1) void conv3_res_kernel(ConvFwdArgs p) {
  using C = RCfg<WM, WN, MT, NT, HALO, TAP8, NBUF>;
  static_assert(NBUF == 2 || NBUF == 3, "halo ring depth");
  static_assert(!BNB || (!SPLIT && !TAP8), "BN-backward epilogue: single output, no image layer");
  constexpr int NW = C::NW, BN = C::BN;
  // the 96-channel variant serves the data gradient of the first decoder conv only (planner:
  // single input, no prologue, no bias): its statistics rows carry the column SUMS only (the
  // up-conv's bias gradient; the sum^2 rows are written as zeros) — 24 VGPRs fewer, which
  // keeps it inside 256
  constexpr bool NOSTAT = BN == 96;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const bool has_pro = p.pscale != nullptr;
  const bool has_pro2 = p.pscale2 != nullptr;          // deferred skip: X2 channels at C1 + c
  const int NSS = has_pro2 ? p.Cin : p.C1;             // channels with prologue constants
  // BNB (a data gradient: no prologue): the LDS table of the BN-backward constants instead
  const int ss_bytes = BNB ? 16 * BN : res_ss_bytes(NSS, has_pro || has_pro2);
  float* s_scale = reinterpret_cast<float*>(smem);
  float* s_shift = s_scale + NSS;
  char* sW = smem + ss_bytes;
  char* sA0 = sW + res_w_bytes(p.Cin, BN, TAP8);
  auto sA = [&](int b) { return sA0 + b * C::A_BYTES; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN;
  const int wn = wave % WN;
  const int HW2 = p.TW + 2, HH2 = p.TH + 2;
  constexpr int NPL = TAP8 == 3 ? 3 : 1;              // halo planes (3-D image layer: 3)
  const int PL = HH2 * HW2;
  const int halo = NPL * PL;
  const long long img_px = (long long)p.H * p.W;      // one slice
  const long long vol_px = NPL == 3 ? (long long)p.D * img_px : img_px;   // one image
  // M-tile walk (conv3_fwd_kernel's): workgroup b = blockIdx.x / nTilesN serves M tiles
  // grp * Mg + r + k * Gs — one group: grp = 0, r = b; BN groups: group-major blocks
  const int NG_ = p.groups > 1 ? p.groups : 1;
  const int Gs = (int)gridDim.x / (p.nTilesN * NG_);
  const int Mg = p.nTilesM / NG_;
  const int grp = (int)blockIdx.x / p.nTilesN / Gs;
  const int r_blk = (int)blockIdx.x / p.nTilesN % Gs;
  const int my_items = r_blk < Mg ? (Mg - 1 - r_blk) / Gs + 1 : 0;
  const int nch = TAP8 ? 1 : (p.Cin + BK - 1) / BK;
  const int S = my_items * nch;
  // every item of a block has the same n tile (launcher: grid % nTilesN == 0)
  const int co0 = (int)blockIdx.x % p.nTilesN * BN;

  if (has_pro) {
    const float* psc = p.pscale + grp * p.gstride;      // (BN groups: this workgroup's group)
    const float* psh = p.pshift + grp * p.gstride;
    for (int c = tid; c < p.C1; c += C::NTH) { s_scale[c] = psc[c]; s_shift[c] = psh[c]; }
  }
  if (has_pro2)
    for (int c = tid; c < p.C2; c += C::NTH) { s_scale[p.C1 + c] = p.pscale2[c]; s_shift[p.C1 + c] = p.pshift2[c]; }
  float* s_bnb = reinterpret_cast<float*>(smem);       // BNB: [4][BN] (published by the first barrier)
  if constexpr (BNB) bnb_fill(s_bnb, BN, co0, p.Cout, p.bnb_s4 + grp * p.gstride, tid, C::NTH);

  // bias of this block's channel tile, loaded once (a global load inside the epilogue would
  // make the compiler wait vmcnt(0) — on this tile's stores — before every use); loaded
  // BEFORE any DMA is issued, so no later wait of ours is affected by it
  float bias_r[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + wn * (NT * 16) + nt * 16 + 4 * (lane >> 4) + i;
      bias_r[nt][i] = (!NOSTAT && p.bias != nullptr && co < p.Cout) ? p.bias[co] : 0.0f;
    }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)                     // consume now: the compiler's wait
    asm volatile("" ::"v"(bias_r[nt][0]), "v"(bias_r[nt][1]), "v"(bias_r[nt][2]), "v"(bias_r[nt][3]));
  // ---- resident weights: rows (chunk, tap, col) [TAP8: (k-step, col)], 64 B each
  {
    const auto rW = make_rsrc(p.Wt, (unsigned)((long long)p.Cout * p.taps * p.CinW * 2));
    const int pieces = res_w_bytes(p.Cin, BN, TAP8) / 16;
    for (int b = wave * 64; b < pieces; b += NW * 64) {
      const int e = b + lane;
      const int row = e >> 2;
      const int sub = (e & 3) ^ swz(row);
      const int col = row % BN;
      const int co = co0 + col;
      unsigned off = kOOB;
      if (TAP8) {
        const int tap = (row / BN) * 4 + sub;
        if (tap < p.taps && co < p.Cout) off = (unsigned)((co * p.taps + tap) * p.CinW) * 2u;
      } else {
        const int t = (row / BN) % 9, c = row / (9 * BN);
        const int ci = c * BK + sub * 8;
        if (co < p.Cout && ci < p.CinW) off = (unsigned)((co * 9 + t) * p.CinW + ci) * 2u;
      }
      dma16(rW, sW + b * 16, off);
    }
  }

  // n_img: the slice (image * D + d; 2-D: the image) — outputs are slice-addressed
  struct Item { int n_img, img, d, h0, w0; };
  // item geometry without integer division in the stage loop: item k of this workgroup is
  // M tile m0 + k * Gs (gridDim.x a multiple of nTilesN: launcher); a walker steps (tw, th,
  // slice) by Gs with carries, the slice as (image, d).  One walker per consumer (halo issue,
  // epilogue, BNB y loads), each visiting the items in order
  struct Walk { int k, tw, th, img, d; };
  const int g_w = Gs % p.tilesW, g_q = Gs / p.tilesW;
  const int g_h = g_q % p.tilesH, g_n = g_q / p.tilesH;
  const int g_d = NPL == 3 ? g_n % p.D : 0, g_i = NPL == 3 ? g_n / p.D : g_n;
  Walk w0;
  {
    int m = grp * Mg + r_blk;
    w0.k = 0; w0.tw = m % p.tilesW; m /= p.tilesW; w0.th = m % p.tilesH; m /= p.tilesH;
    w0.d = NPL == 3 ? m % p.D : 0; w0.img = NPL == 3 ? m / p.D : m;
  }
  auto walk_item = [&](Walk& w, int k) __attribute__((always_inline)) {
    while (w.k < k) {
      w.tw += g_w;
      const int c1 = w.tw >= p.tilesW ? 1 : 0;
      w.tw -= c1 * p.tilesW;
      w.th += g_h + c1;
      const int c2 = w.th >= p.tilesH ? 1 : 0;
      w.th -= c2 * p.tilesH;
      if constexpr (NPL == 3) {
        w.d += g_d + c2;
        const int c3 = w.d >= p.D ? 1 : 0;
        w.d -= c3 * p.D;
        w.img += g_i + c3;
      } else {
        w.img += g_n + c2;                              // 2-D: D = 1, d = 0
      }
      ++w.k;
    }
    Item it;
    it.img = w.img; it.d = NPL == 3 ? w.d : 0; it.n_img = NPL == 3 ? w.img * p.D + w.d : w.img;
    it.h0 = w.th * p.TH; it.w0 = w.tw * p.TW;
    return it;
  };
  Walk wA = w0, wE = w0, wY = w0;
  // ---- per-lane halo DMA geometry (no integer division in the stage loop).  Interior
  // tiles (the common case) need no bounds checks: pixel = tile base + a_rel.
  int a_dw[C::A_ITERS], a_dh[C::A_ITERS], a_dd[C::A_ITERS], a_sub8[C::A_ITERS];
  uint32_t a_inhalo = 0;
#pragma unroll
  for (int i = 0; i < C::A_ITERS; ++i) {
    const int e = (i * NW + wave) * 64 + lane;
    const int px = TAP8 ? e : e >> 2;
    a_sub8[i] = TAP8 ? 0 : ((e & 3) ^ swz(px)) << 3;
    const int pr = NPL == 1 ? px : px % PL;
    a_dd[i] = NPL == 1 ? 0 : px / PL - 1;
    a_dw[i] = pr % HW2 - 1;
    a_dh[i] = pr / HW2 - 1;
    if (px < halo && e < C::PIECES) a_inhalo |= 1u << i;
  }
  // element offset of piece i relative to the item / chunk base, per input tensor (a runtime
  // multiply per piece per stage otherwise); pieces past the halo get an offset beyond any
  // tensor (>= 2^31 bytes: the DMA reads zeros), so an interior item's pieces need no mask
  // (X2 chunks of the concat layers compute theirs per stage: VGPR budget of the 96-channel
  // variant)
  int a_relC1[C::A_ITERS];
#pragma unroll
  for (int i = 0; i < C::A_ITERS; ++i)
    a_relC1[i] = (a_inhalo >> i) & 1u ? (((NPL == 3 ? a_dd[i] * p.H : 0) + a_dh[i]) * p.W + a_dw[i]) * p.C1 + a_sub8[i]
                                      : (1 << 30);
  uint32_t a_valid = 0;            // pieces of the item last issued that are inside the image
  // a_valid of the stage held by each ring slot, 8 bits per slot in one register (a
  // runtime-indexed array would live in scratch: vm ops that break the counted waits)
  static_assert(C::A_ITERS <= 8, "valid mask packing");
  uint32_t vmasks = 0;
  auto set_vmask = [&](int buf, uint32_t m) {
    vmasks = (vmasks & ~(0xffu << (8 * buf))) | (m << (8 * buf));
  };
  auto get_vmask = [&](int buf) { return (vmasks >> (8 * buf)) & 0xffu; };
  // wave-uniform: bit b = the item staged in ring slot b is interior (every halo piece inside
  // the image): its prologue needs no masking
  uint32_t ibits = 0;
  bool a_int = false;
  int a_item = -1, a_nimg = 0, a_base = 0;
  auto issue_A = [&](int k, int chunk, int buf) {
    if (k != a_item) {
      const Item it = walk_item(wA, k);
      a_item = k;
      a_nimg = it.img;
      a_base = ((NPL == 3 ? it.d * p.H : 0) + it.h0) * p.W + it.w0;   // pixel within the image volume
      const bool interior = it.w0 >= 1 && it.h0 >= 1 && it.w0 + p.TW < p.W && it.h0 + p.TH < p.H &&
                            (NPL == 1 || (it.d >= 1 && it.d + 1 < p.D));
      a_int = interior;
      if (interior) {
        a_valid = a_inhalo;
      } else {
        a_valid = 0;
#pragma unroll
        for (int i = 0; i < C::A_ITERS; ++i) {
          const int gw = it.w0 + a_dw[i], gh = it.h0 + a_dh[i], gd = it.d + a_dd[i];
          if (gw >= 0 && gw < p.W && gh >= 0 && gh < p.H && (NPL == 1 || (gd >= 0 && gd < p.D)))
            a_valid |= 1u << i;
        }
        a_valid &= a_inhalo;
      }
    }
    const int cbase = chunk * BK;
    const bool second = cbase >= p.C1;                 // chunk served by X2 (C1 % 32 == 0)
    const int Cs = second ? p.C2 : p.C1;
    const int c0 = second ? cbase - p.C1 : cbase;
    const bool full = c0 + BK <= Cs;                   // wave-uniform: no channel check
    const bf16_t* src = second ? p.X2 : p.X1;
    set_vmask(buf, a_valid);
    ibits = (ibits & ~(1u << buf)) | ((a_int ? 1u : 0u) << buf);
    const auto r = make_rsrc(src + a_nimg * vol_px * Cs, (unsigned)(vol_px * Cs * 2));
    const int s0 = a_base * Cs + c0;                   // scalar part of the element offset
    // (wave-uniform branches: interior item and full chunk = no per-piece mask at all)
    auto pieces = [&](const int (&rel)[C::A_ITERS], auto maskc) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < C::A_ITERS; ++i) {
        unsigned off = (unsigned)(rel[i] + s0) * 2u;
        if constexpr (decltype(maskc)::value) {
          const bool ok = ((a_valid >> i) & 1u) && (full || c0 + a_sub8[i] < Cs);
          off = ok ? off : kOOB;
        }
        dma16(r, sA(buf) + (i * NW + wave) * 1024, off);
      }
    };
    if (second) {
      int rel2[C::A_ITERS];
#pragma unroll
      for (int i = 0; i < C::A_ITERS; ++i)
        rel2[i] = (a_inhalo >> i) & 1u ? (((NPL == 3 ? a_dd[i] * p.H : 0) + a_dh[i]) * p.W + a_dw[i]) * Cs + a_sub8[i]
                                       : (1 << 30);
      pieces(rel2, std::true_type{});
    } else if (a_int && full) {
      pieces(a_relC1, std::false_type{});
    } else {
      pieces(a_relC1, std::true_type{});
    }
  };
  // prologue on the pieces THIS lane DMA'd (a_valid still describes the chunk's item), in a
  // batched form: a lane's 8-channel group is the same in every piece it DMAs (the XOR
  // swizzle flips bit 1 of the piece index by bit 4 of the lane only), so the chunk's 16
  // constants are read once per stage instead of once per piece, all A_ITERS piece reads
  // issue before any math, and padding / masked pieces are re-zeroed by a select instead of
  // a branch around each piece
  const int sub8_l = TAP8 ? 0 : ((lane & 3) ^ (((lane >> 4) & 1) << 1)) << 3;
  auto transform_batched = [&](char* __restrict__ Ab, const float* __restrict__ scl,
                               const float* __restrict__ shf_, int cbase, uint32_t vm, int climit,
                               auto maskc) {
    constexpr bool MASK = decltype(maskc)::value;   // false: interior item, full chunk
    const int c8 = cbase + sub8_l;
    const bool cok = c8 < climit;
    const float4* scp = reinterpret_cast<const float4*>(scl + (cok ? c8 : 0));
    const float4* shp = reinterpret_cast<const float4*>(shf_ + (cok ? c8 : 0));
    const float4 sa = scp[0], sb = scp[1], ha = shp[0], hb = shp[1];
    const float scf[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float shf[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
    uint4 v[C::A_ITERS];
#pragma unroll
    for (int i = 0; i < C::A_ITERS; ++i)
      v[i] = *reinterpret_cast<const uint4*>(Ab + ((i * NW + wave) * 64 + lane) * 16);
#pragma unroll
    for (int i = 0; i < C::A_ITERS; ++i) {
      const bool ok = !MASK || (((vm >> i) & 1u) && cok);
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
      *reinterpret_cast<uint4*>(Ab + ((i * NW + wave) * 64 + lane) * 16) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  };
  // (restrict-qualified LDS pointers: alias scopes keep the compiler from waiting on the
  // in-flight halo DMAs of later ring slots before these reads)
  auto transform_A = [&](int chunk, int buf) {
    const int cbase = chunk * BK;
    const bool x2ch = cbase >= p.C1;                   // X2 chunk: prologue only if deferred
    if (x2ch ? !has_pro2 : !has_pro) return;
    const int climit = x2ch ? p.Cin : p.C1;
    // interior item and a full chunk: no piece needs re-zeroing (pieces past the halo are
    // never read by the fragment loads)
    if (((ibits >> buf) & 1u) && cbase + BK <= climit)
      transform_batched(sA(buf), s_scale, s_shift, cbase, 0u, climit, std::false_type{});
    else
      transform_batched(sA(buf), s_scale, s_shift, cbase, get_vmask(buf), climit, std::true_type{});
  };

  // ---- per-lane fragment geometry
  const int g = lane >> 4;
  int hp0[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int pix = wm * (MT * 16) + mt * 16 + (lane & 15);
    hp0[mt] = (NPL == 3 ? PL : 0) + (pix / p.TW) * HW2 + pix % p.TW;   // (3-D: the centre plane)
  }
  constexpr int KS8 = tap8_ksteps(TAP8);
  int toff8[KS8];                                      // TAP8: this lane group's tap offsets
#pragma unroll
  for (int ks = 0; ks < KS8; ++ks) {
    // taps past the last are zero-weight: any in-halo address will do
    const int tap = min(ks * 4 + g, NPL * 9 - 1);
    const int t9 = tap % 9;
    toff8[ks] = (NPL == 3 ? (tap / 9 - 1) * PL : 0) + (t9 / 3) * HW2 + t9 % 3;
  }
  const int wrow0 = wn * (NT * 16) + (lane & 15);

  // accumulators start at the bias and the epilogue resets them to it (no bias add per value)
  f32x4_t bias4[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) bias4[nt] = f32x4_t{bias_r[nt][0], bias_r[nt][1], bias_r[nt][2], bias_r[nt][3]};
  f32x4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = bias4[j];
  float s1[NT][4], s2[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) { s1[nt][i] = 0.f; s2[nt][i] = 0.f; }

  // epilogue of item k straight from the accumulators: lane holds channels co..co+3 of
  // tile pixel (wm*MT*16 + mt*16 + (lane&15))
  // Stores are buffer stores with an out-of-range offset for masked lanes: every wave
  // issues exactly EPI_STORES of them per epilogue (no exec branches), which keeps the
  // counted vmcnt waits exact.
  // PAIRS: 16-byte stores of channel-tile pairs (pair16).  Measured per layer at batch 128
  // (profiles/conv_micro_b128_pair16_r2.txt): 5-10% faster on the BN 64 and image-layer
  // variants, 4-6% slower on the 32-channel 3x3 layers (BN 32) -> 8-byte stores there
  constexpr bool PAIRS = (!SPLIT && (TAP8 || BN >= 64) && NT % 2 == 0) || SPLIT == 2;
  static_assert(SPLIT != 2 || (NT % 2 == 0 && BN % 32 == 0), "split pairs: 32-channel pairs");
  constexpr int EPI_STORES = SPLIT == 1 ? MT * NT * 2 : PAIRS ? MT * NT / 2 : MT * NT;
  // ---- per-lane output geometry relative to an item's first pixel (item-independent): the
  // element offset of tile (mt, nt) is item_base * Co + orel[mt] + 16 nt (pairs: + 32 np) —
  // one add per store instead of a 64-bit multiply-add chain (the epilogue was VALU-issue
  // bound).  q: the MFMA's 4-channel lane layout, p: the pair16 layout.
  const int Co2 = p.Cout - p.Co1;
  int prow[MT], pcol[MT], orel1q[MT], orel2q[MT], orel1p[MT], orel2p[MT];
  {
    const int coq = co0 + wn * (NT * 16) + 4 * g;
    const int cop = co0 + wn * (NT * 16) + pair16_ch(lane);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int pix = wm * (MT * 16) + mt * 16 + (lane & 15);
      prow[mt] = pix / p.TW;
      pcol[mt] = pix % p.TW;
      const int lr = prow[mt] * p.W + pcol[mt];
      orel1q[mt] = lr * p.Co1 + coq;
      orel2q[mt] = SPLIT == 1 ? lr * Co2 + coq - p.Co1 : 0;
      orel1p[mt] = PAIRS ? lr * p.Co1 + cop : 0;
      orel2p[mt] = SPLIT == 2 ? lr * Co2 + cop - p.Co1 : 0;
    }
  }
  // per item: output descriptors, element bases, the in-image extent, and whether the whole
  // tile (pixels and channels) is inside the output — wave-uniform, then no masks at all
  struct EpiCtx { __amdgpu_buffer_rsrc_t r1, r2; int b1, b2, wlim, hlim; bool full; };
  auto epi_ctx = [&](Walk& w, int kk) __attribute__((always_inline)) {
    const Item it = walk_item(w, kk);
    EpiCtx e;
    e.r1 = make_rsrc(p.Y1 + (long long)it.n_img * img_px * p.Co1, (unsigned)(img_px * p.Co1 * 2));
    e.r2 = SPLIT ? make_rsrc(p.Y2 + (long long)it.n_img * img_px * Co2, (unsigned)(img_px * Co2 * 2)) : e.r1;
    const int base = it.h0 * p.W + it.w0;
    e.b1 = base * p.Co1;
    e.b2 = SPLIT ? base * Co2 : 0;
    e.wlim = p.W - it.w0;
    e.hlim = p.H - it.h0;
    e.full = it.w0 + p.TW <= p.W && it.h0 + p.TH <= p.H && co0 + BN <= p.Cout;
    return e;
  };
  // one 16-pixel row (mt) of tiles: bf16 stores, and the BN statistics of the tiles' fp32
  // values as packed pairs (masked lanes add zeros); FULL: every lane is valid
  auto epi_row = [&](const EpiCtx& e, int mt, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    const bool pv = FULL || (pcol[mt] < e.wlim && prow[mt] < e.hlim);
    uint2 pkv[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int co = co0 + wn * (NT * 16) + nt * 16 + 4 * g;
      const bool ok = FULL || (pv && co < p.Cout);
      const f32x2_t v01 = {acc[mt][nt][0], acc[mt][nt][1]};
      const f32x2_t v23 = {acc[mt][nt][2], acc[mt][nt][3]};
      const uint2 pk = make_uint2(pack2(v01.x, v01.y), pack2(v23.x, v23.y));
      pkv[nt] = pk;
      if constexpr (!PAIRS) {
        const u32x2_t d = u32x2_t{pk.x, pk.y};
        if constexpr (!SPLIT) {
          unsigned o1 = ok ? (unsigned)(e.b1 + orel1q[mt] + nt * 16) * 2u : kOOB;
          asm volatile("" : "+v"(o1));
          __builtin_amdgcn_raw_buffer_store_b64(d, e.r1, o1, 0, 0);
        } else {
          const bool in1 = co < p.Co1;
          unsigned o1 = (ok && in1) ? (unsigned)(e.b1 + orel1q[mt] + nt * 16) * 2u : kOOB;
          unsigned o2 = (ok && !in1) ? (unsigned)(e.b2 + orel2q[mt] + nt * 16) * 2u : kOOB;
          asm volatile("" : "+v"(o1), "+v"(o2));
          __builtin_amdgcn_raw_buffer_store_b64(d, e.r1, o1, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(d, e.r2, o2, 0, 0);
        }
      }
      const f32x2_t z = {0.f, 0.f};
      const f32x2_t r01 = ok ? v01 : z, r23 = ok ? v23 : z;
      f32x2_t a01 = {s1[nt][0], s1[nt][1]}, a23 = {s1[nt][2], s1[nt][3]};
      a01 += r01; a23 += r23;
      s1[nt][0] = a01.x; s1[nt][1] = a01.y; s1[nt][2] = a23.x; s1[nt][3] = a23.y;
      if constexpr (!NOSTAT) {
        f32x2_t q01 = {s2[nt][0], s2[nt][1]}, q23 = {s2[nt][2], s2[nt][3]};
        q01 = __builtin_elementwise_fma(r01, r01, q01);
        q23 = __builtin_elementwise_fma(r23, r23, q23);
        s2[nt][0] = q01.x; s2[nt][1] = q01.y; s2[nt][2] = q23.x; s2[nt][3] = q23.y;
      }
    }
    if constexpr (PAIRS) {
#pragma unroll
      for (int np = 0; np < NT / 2; ++np) {
        const uint4 q = pair16(pkv[2 * np], pkv[2 * np + 1]);
        const int co = co0 + wn * (NT * 16) + np * 32 + pair16_ch(lane);
        const bool ok = FULL || (pv && co < p.Cout);
        if constexpr (SPLIT == 2) {
          // the pair's 32 channels lie in one output (wave-uniform choice)
          const bool in1 = co0 + wn * (NT * 16) + np * 32 < p.Co1;
          unsigned o = ok ? (unsigned)(in1 ? e.b1 + orel1p[mt] + np * 32 : e.b2 + orel2p[mt] + np * 32) * 2u
                          : kOOB;
          asm volatile("" : "+v"(o));
          __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{q.x, q.y, q.z, q.w}, in1 ? e.r1 : e.r2, o, 0, 0);
        } else {
          unsigned o1 = ok ? (unsigned)(e.b1 + orel1p[mt] + np * 32) * 2u : kOOB;
          asm volatile("" : "+v"(o1));
          __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{q.x, q.y, q.z, q.w}, e.r1, o1, 0, 0);
        }
      }
    }
  };
  // BNB: y at this item's output pixels, loaded into VGPRs at the item's last stage (before
  // that stage's halo DMA) and consumed by its epilogue one stage later (Co1 = Cout)
  constexpr int YL = BNB ? MT * NT : 0;
  uint2 ybuf[MT][NT];
  auto issue_Y = [&](int kk) __attribute__((always_inline)) {
    const Item it = walk_item(wY, kk);
    const auto ry = make_rsrc(p.bnb_y + (long long)it.n_img * img_px * p.Cout, (unsigned)(img_px * p.Cout * 2));
    const int b = (it.h0 * p.W + it.w0) * p.Cout;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const bool valid = pcol[mt] < p.W - it.w0 && prow[mt] < p.H - it.h0;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int co = co0 + wn * (NT * 16) + nt * 16 + 4 * g;
        ybuf[mt][nt] = buf_load8(ry, valid && co < p.Cout ? (unsigned)(b + orel1q[mt] + nt * 16) * 2u : kOOB);
      }
    }
  };
  // BNB epilogue (a data gradient dA; no bias): channel tiles outer, so the BN-backward
  // constants of one tile are read once; the scheduler barrier keeps the next tile's reads
  // from being hoisted (VGPR pressure)
  auto epilogue_bnb_f = [&](const EpiCtx& e, auto fullc) __attribute__((always_inline)) {
    constexpr bool FULL = decltype(fullc)::value;
    uint2 pkv[MT][NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int co = co0 + wn * (NT * 16) + nt * 16 + 4 * g;
      const BnbC kb = bnb_load(s_bnb, BN, wn * (NT * 16) + nt * 16 + 4 * g);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bool ok = FULL || (pcol[mt] < e.wlim && prow[mt] < e.hlim && co < p.Cout);
        const uint2 pk = make_uint2(pack2(acc[mt][nt][0], acc[mt][nt][1]), pack2(acc[mt][nt][2], acc[mt][nt][3]));
        pkv[mt][nt] = pk;
        if constexpr (!PAIRS) {
          unsigned o1 = ok ? (unsigned)(e.b1 + orel1q[mt] + nt * 16) * 2u : kOOB;
          asm volatile("" : "+v"(o1));
          __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk.x, pk.y}, e.r1, o1, 0, 0);
        }
        const float d[4] = {ok ? acc[mt][nt][0] : 0.f, ok ? acc[mt][nt][1] : 0.f,
                            ok ? acc[mt][nt][2] : 0.f, ok ? acc[mt][nt][3] : 0.f};
        bnb_accum(d, ybuf[mt][nt], kb, s1[nt], s2[nt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PAIRS) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bool pv = FULL || (pcol[mt] < e.wlim && prow[mt] < e.hlim);
#pragma unroll
        for (int np = 0; np < NT / 2; ++np) {
          const uint4 q = pair16(pkv[mt][2 * np], pkv[mt][2 * np + 1]);
          const int co = co0 + wn * (NT * 16) + np * 32 + pair16_ch(lane);
          unsigned o1 = FULL || (pv && co < p.Cout) ? (unsigned)(e.b1 + orel1p[mt] + np * 32) * 2u : kOOB;
          asm volatile("" : "+v"(o1));
          __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{q.x, q.y, q.z, q.w}, e.r1, o1, 0, 0);
        }
      }
    }
  };
  auto epilogue_bnb = [&](int kk) __attribute__((always_inline)) {
    const EpiCtx e = epi_ctx(wE, kk);
    if (e.full) epilogue_bnb_f(e, std::true_type{});
    else epilogue_bnb_f(e, std::false_type{});
  };

  auto epilogue = [&](int kk) __attribute__((always_inline)) {
    if constexpr (BNB) {
      epilogue_bnb(kk);
    } else {
      const EpiCtx e = epi_ctx(wE, kk);
      if (e.full) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) epi_row(e, mt, std::true_type{});
      } else {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) epi_row(e, mt, std::false_type{});
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = bias4[nt];
  };

  // ---- pipeline: the halo of stage s+NBUF-1 is issued at stage s (ring of NBUF buffers).
  // Per stage a wave issues: [epilogue stores of the previous item] [BNB: y loads, at an
  // item's last stage] then [A_ITERS DMAs], so at stage s the ops younger than DMA(s) are
  // exactly those of stage s-1 (NBUF = 3) or none (NBUF = 2) plus the prologue's extra DMA
  // at s = 0.
  auto next_of = [&](int k0, int c0, int& k1, int& c1) {
    k1 = k0; c1 = c0 + 1;
    if (c1 == nch) { c1 = 0; ++k1; }
  };
  int kp = 0, cp = 0;                                 // stage whose halo is issued next
  for (int j = 0; j < NBUF - 1 && j < S; ++j) {
    issue_A(kp, cp, j % NBUF);
    int k1, c1;
    next_of(kp, cp, k1, c1);
    kp = k1; cp = c1;
  }
  // (wave priority: s_setprio 1 around every MFMA cluster, in compute below)
  int k = 0, c = 0;
  bool epi_prev = false;                              // stage s-1 ran an epilogue
  for (int s = 0; s < S; ++s) {
    if (NBUF == 2) {
      vm_wait<0>();                                   // DMA(s) is the youngest op
    } else {
      // younger than DMA(s): s == 0 -> DMA(1); s >= 1 -> [stores(s-1)] + [DMA(s+1)]
      const bool dma_next = s + 1 < S;
      if (BNB && s > 0) {
        // stage s-1 issued [stores if it ran an epilogue] [y loads if it was an item's last]
        // [DMA(s+1)]
        vm_wait_dyn((epi_prev ? EPI_STORES : 0) + (c == 0 ? YL : 0) + (dma_next ? C::A_ITERS : 0));
      } else if (s == 0) {
        if (dma_next) vm_wait<C::A_ITERS>(); else vm_wait<0>();
      } else if (epi_prev) {
        if (dma_next) vm_wait<C::A_ITERS + EPI_STORES>(); else vm_wait<EPI_STORES>();
      } else {
        if (dma_next) vm_wait<C::A_ITERS>(); else vm_wait<0>();
      }
    }
    const int buf = s % NBUF;
    if (!TAP8 && (has_pro || has_pro2)) transform_A(c, buf);
    lds_sync();
    epi_prev = (c == 0 && s > 0);
    if (epi_prev) {
      // BNB, 3-deep ring: the y loads (issued before DMA(s+1)) must have landed
      if (BNB && NBUF == 3) { if (s + 1 < S) vm_wait<C::A_ITERS>(); else vm_wait<0>(); }
      epilogue(k - 1);
    }
    if (BNB && c == nch - 1) issue_Y(k);              // before this stage's DMA
    if (s + NBUF - 1 < S) {
      issue_A(kp, cp, (s + NBUF - 1) % NBUF);
      int k1, c1;
      next_of(kp, cp, k1, c1);
      kp = k1; cp = c1;
    }
    int k1 = k, c1 = c + 1;
    if (c1 == nch) { c1 = 0; ++k1; }
    // compute: fragments of step j+1 are read while the MFMAs of step j run (register
    // double buffer; the sched barrier keeps the compiler from hoisting all 9 steps' reads)
    // (restrict-qualified operand pointers give the LDS reads alias scopes, so the compiler
    // does not make them wait for the next stage's in-flight LDS-DMA: vmcnt is managed by
    // hand above)
    auto compute = [&](const char* __restrict__ A, const char* __restrict__ Wc, auto hook) {
    constexpr int KSTEPS = TAP8 ? KS8 : 9;
    auto load_frags = [&](int j, uint4 (&xf)[MT], uint4 (&wf)[NT]) {
      if (TAP8) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xf[mt] = lds128(A + (hp0[mt] + toff8[j]) * 16);
      } else {
        const int tapoff = (j / 3) * HW2 + j % 3;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xf[mt] = lds128(A + lds_off(hp0[mt] + tapoff, g));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) wf[nt] = lds128(Wc + lds_off(j * BN + wrow0 + nt * 16, g));
    };
    uint4 xf[2][MT], wf[2][NT];
    load_frags(0, xf[0], wf[0]);
#pragma unroll
    for (int j = 0; j < KSTEPS; ++j) {
      if (j + 1 < KSTEPS) load_frags(j + 1, xf[(j + 1) & 1], wf[(j + 1) & 1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = mfma16x16x32(wf[j & 1][nt], xf[j & 1][mt], acc[mt][nt]);
      __builtin_amdgcn_s_setprio(0);
      hook(j);
      __builtin_amdgcn_sched_barrier(0);
    }
    };
    const char* Wst = TAP8 ? sW : sW + c * 9 * BN * ROWB;
    auto no_hook = [](int) {};
    compute(sA(buf), Wst, no_hook);
    k = k1; c = c1;
  }
  if (S > 0) {
    if (BNB) vm_wait<0>();
    epilogue(k - 1);
  }

  // ---- one BN-statistics partial row per workgroup (layout of conv3_fwd_kernel)
  if (p.stats != nullptr) {
    dma_wait<0>();
    lds_sync();
    float* red = reinterpret_cast<float*>(sA0);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a1 = s1[nt][i], a2 = s2[nt][i];
        a1 = row16_sum(a1); a2 = row16_sum(a2);
        if ((lane & 15) == 0) {
          const int col = wn * (NT * 16) + nt * 16 + 4 * g + i;
          red[(2 * wm) * BN + col] = a1;           // one writer per (wave row, column)
          red[(2 * wm + 1) * BN + col] = a2;
        }
      }
    lds_sync();
    float* row = p.stats + (long long)blockIdx.x * 2 * p.Cout;
    for (int i = tid; i < p.Cout; i += C::NTH) {
      const bool mine = i >= co0 && i < co0 + BN;
      float t1 = 0.f, t2 = 0.f;                    // fixed-order sum over wave rows
      if (mine)
        for (int r = 0; r < WM; ++r) { t1 += red[(2 * r) * BN + i - co0]; t2 += red[(2 * r + 1) * BN + i - co0]; }
      row[i] = t1;
      row[p.Cout + i] = t2;
    }
  }
}

struct ResVariant { int wm, wn, mt, nt, halo, tap8, tw, th, nbuf; };
// BN 32 = 4x2 16x16 MFMA tiles per wave column, BN 64 = two wave columns; NBUF = halo ring
constexpr ResVariant kRes[10] = {
    {4, 1, 4, 2, 324, 0, 16, 16, 2},       // 0: BM 256 BN 32, 4 waves, 2-deep (2 WG / CU)
    {8, 1, 4, 2, 612, 0, 32, 16, 3},       // 1: BM 512 BN 32, 8 waves, 3-deep
    {4, 2, 4, 2, 324, 0, 16, 16, 3},       // 2: BM 256 BN 64, 8 waves, 3-deep
    {4, 1, 4, 2, 324, 2, 16, 16, 2},       // 3: image layer (TAP8), 4 waves, 2-deep
    {8, 1, 4, 2, 612, 2, 32, 16, 3},       // 4: image layer (TAP8), 8 waves, 3-deep
    {8, 1, 4, 2, 612, 0, 32, 16, 2},       // 5: BM 512 BN 32, 8 waves, 2-deep (large Cin)
    {4, 2, 4, 2, 324, 0, 16, 16, 2},       // 6: BM 256 BN 64, 8 waves, 2-deep (large Cin)
    // 7: BM 256 BN 96, 8 waves x (2 x 6 tiles), 3-deep — the 96-channel data gradient of the
    //    first decoder conv (dY: 32 ch -> d[up | skip]: 64 + 32 ch).  One workgroup covers all
    //    96 output channels, so the dY halo is read once instead of once per 32-channel tile.
    {8, 1, 2, 6, 324, 0, 16, 16, 3},
    // 8 / 9: the 3-D image layer (TAP8 = 3): 3-plane halos of 16x16 / 32x16 slice tiles
    {4, 1, 4, 2, 972, 3, 16, 16, 2},
    {8, 1, 4, 2, 1836, 3, 32, 16, 3}};

int res_smem(const ResVariant& v, int Cin, int C1, bool pro, bool bnb) {   // C1: channels with constants
  const int bn = v.wn * v.nt * 16;
  const int nw = v.wm * v.wn;
  const int instr = ((v.tap8 ? v.halo : v.halo * 4) + 63) / 64;
  const int a_bytes = (instr + nw - 1) / nw * nw * 1024;
  return (bnb ? 16 * bn : res_ss_bytes(C1, pro)) + res_w_bytes(Cin, bn, v.tap8) + v.nbuf * a_bytes;
}

template <int WM, int WN, int MT, int NT, int HALO, int TAP8, int NBUF>
void launch_res(ConvFwdArgs& a, int grid, int smem, hipStream_t st) {
  constexpr int BNc = WN * NT * 16;
  if (a.Co1 < a.Cout) {
    // split output at a 32-channel boundary: 16-byte pair stores
    if constexpr (NT % 2 == 0 && BNc % 32 == 0 && !TAP8) {
      if (a.Co1 % 32 == 0) {
        hipLaunchKernelGGL((conv3_res_kernel<WM, WN, MT, NT, HALO, TAP8, NBUF, 2, false>), dim3(grid),
                           dim3(WM * WN * 64), smem, st, a);
        return;
      }
    }
    hipLaunchKernelGGL((conv3_res_kernel<WM, WN, MT, NT, HALO, TAP8, NBUF, 1, false>), dim3(grid),
                       dim3(WM * WN * 64), smem, st, a);
  } else if constexpr (!TAP8 && BNc != 96) {
    if (a.bnb_y != nullptr)
      hipLaunchKernelGGL((conv3_res_kernel<WM, WN, MT, NT, HALO, TAP8, NBUF, 0, true>), dim3(grid),
                         dim3(WM * WN * 64), smem, st, a);
    else
      hipLaunchKernelGGL((conv3_res_kernel<WM, WN, MT, NT, HALO, TAP8, NBUF, 0, false>), dim3(grid),
                         dim3(WM * WN * 64), smem, st, a);
  } else {
    hipLaunchKernelGGL((conv3_res_kernel<WM, WN, MT, NT, HALO, TAP8, NBUF, 0, false>), dim3(grid),
                       dim3(WM * WN * 64), smem, st, a);
  }
}

}  // namespace

// Planner: returns a variant id (and fills tiles / persistent grid) or -1 when the layer
// belongs to the streaming kernel.  LDS budget: 160 KB per CU; two workgroups per CU when
// a workgroup needs <= 80 KB.
int conv3_res_plan(ConvFwdArgs& a, int num_cus, int& grid, int& smem) {
  if (a.W < 16 || a.H < 16) return -1;
  const bool pro = a.pscale != nullptr;
  const bool tap8 = a.Cin <= 8 && a.C2 == 0 && a.CinW == 8 && !pro;
  // 3-D: the image layer only (depth slices, a 3-plane halo addressed within one image
  // volume through one buffer descriptor: 32-bit offsets)
  const bool d3 = a.dims == 3;
  if (d3 && (!tap8 || (long long)a.D * a.H * a.W * a.CinW * 2 >= (1LL << 31))) return -1;
  const int bn = a.Cout == 96 ? 96 : (a.Cout <= 32 || a.Cout % 64 != 0) ? 32 : 64;
  // halo ring depth: 2 for the 64-channel tiles (variant 6: BN-backward data gradients 9-11%
  // faster, the others 1-3.5%), 3 for the 32-channel tiles (the 2-deep 4-wave variant is
  // 5-11% slower forward): profiles/r3s/res_depth_ab_b256_r3s33.txt
  const int depth = bn == 64 ? 2 : 3;
  int cand[3];
  int nc = 0;
  if (tap8) {
    if (bn != 32 || a.bnb_y != nullptr) return -1;
    if (d3) { cand[nc++] = 9; cand[nc++] = 8; }
    else if (depth == 2) { cand[nc++] = 3; } else { cand[nc++] = 4; cand[nc++] = 3; }
  } else if (bn == 96) {
    // BN 96: the concat data gradient only — no BN-backward epilogue, single input, no
    // prologue, no bias; its statistics rows hold the column sums only (sum^2 rows zero)
    if (a.bnb_y != nullptr || a.bias != nullptr || a.C2 != 0 || pro || a.pscale2 != nullptr) return -1;
    cand[nc++] = 7;
  } else if (bn == 32) {
    if (depth == 2) { cand[nc++] = 0; cand[nc++] = 5; }
    else { cand[nc++] = 1; cand[nc++] = 5; cand[nc++] = 0; }
  } else {
    if (depth == 2) { cand[nc++] = 6; } else { cand[nc++] = 2; cand[nc++] = 6; }
  }
  for (int i = 0; i < nc; ++i) {
    const ResVariant& v = kRes[cand[i]];
    const int sm = res_smem(v, a.Cin, a.pscale2 != nullptr ? a.Cin : a.C1, pro || a.pscale2 != nullptr,
                            a.bnb_y != nullptr);
    const int nw = v.wm * v.wn;
    // 4-wave blocks need 2 per CU (2 waves / SIMD); 8-wave blocks use ~200 VGPRs: 1 per CU
    const int bpc = nw == 4 ? (sm <= 80 * 1024 ? 2 : 0) : (sm <= 160 * 1024 ? 1 : 0);
    if (bpc == 0) continue;
    a.TD = 1; a.TW = v.tw; a.TH = v.th;
    a.tilesD = a.D;                                     // 3-D: one tile per slice
    a.tilesH = (a.H + a.TH - 1) / a.TH;
    a.tilesW = (a.W + a.TW - 1) / a.TW;
    a.nTilesM = a.N * a.D * a.tilesH * a.tilesW;
    a.nTilesN = (a.Cout + bn - 1) / bn;
    const int items = a.nTilesM * a.nTilesN;
    const int cap = bpc * num_cus;
    if (items < cap) return -1;                         // too small: streaming kernel
    grid = cap / a.nTilesN * a.nTilesN;
    if (a.groups > 1) {
      // BN groups: group-major blocks, R per (group, n tile) (conv3_res_kernel's walk)
      const int R = std::max(1, std::min(a.nTilesM / a.groups, cap / (a.groups * a.nTilesN)));
      grid = a.groups * R * a.nTilesN;
    }
    smem = sm;
    a.ksplit = 1;
    a.persist_blocks = cap;
    a.stat_rows = grid;
    return cand[i];
  }
  return -1;
}

void conv3_res_launch(ConvFwdArgs& a, int variant, int grid, int smem, hipStream_t st) {
  switch (variant) {
    case 0: launch_res<4, 1, 4, 2, 324, 0, 2>(a, grid, smem, st); break;
    case 1: launch_res<8, 1, 4, 2, 612, 0, 3>(a, grid, smem, st); break;
    case 2: launch_res<4, 2, 4, 2, 324, 0, 3>(a, grid, smem, st); break;
    case 3: launch_res<4, 1, 4, 2, 324, 2, 2>(a, grid, smem, st); break;
    case 4: launch_res<8, 1, 4, 2, 612, 2, 3>(a, grid, smem, st); break;
    case 5: launch_res<8, 1, 4, 2, 612, 0, 2>(a, grid, smem, st); break;
    case 7: launch_res<8, 1, 2, 6, 324, 0, 3>(a, grid, smem, st); break;
    case 8: launch_res<4, 1, 4, 2, 972, 3, 2>(a, grid, smem, st); break;
    case 9: launch_res<8, 1, 4, 2, 1836, 3, 3>(a, grid, smem, st); break;
    default: launch_res<4, 2, 4, 2, 324, 0, 2>(a, grid, smem, st); break;
  }
}

}  // namespace ddlpc
