// 3x3 (2-D) / 3x3x3 (3-D) convolution, stride 1, zero padding 1, as an MFMA implicit GEMM
// over NHWC / NDHWC bf16 activations — the U-Net's K1 (forward) and K2 (data gradient)
// of SURVEY.md §2.5.  Reference ops: nn.Conv2d(k=3, padding=1) in DoubleConv (ref.py:579,582).
//
// GEMM view:  M = output pixels, N = output channels, K = taps x input channels.
//
// Tiling (one 256-thread workgroup = 4 waves as WM x WN):
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
//     (sum, sum^2) partials of the stored values for BatchNorm statistics (K4), one partial
//     row per M tile (deterministic; reduced by bn_finalize).
//
// The data gradient (K2) is this same kernel run on dY with the flipped, transposed
// weights W'[ci][8-t][co] (packed by weight_pack).
#include "common.h"
#include "ops.h"

namespace ddlpc {

namespace {

constexpr int BK = 32;                 // channels per K chunk
constexpr int ROWB = BK * 2;           // bytes per LDS row (one pixel / one weight row)
constexpr unsigned kOOB = 0x80000000u; // buffer offset that reads as zero

DDLPC_DEVICE int swz(int row) { return ((row >> 2) & 1) << 1; }
DDLPC_DEVICE int lds_off(int row, int chunk) { return row * ROWB + ((chunk ^ swz(row)) << 4); }

DDLPC_DEVICE void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
DDLPC_DEVICE void dma_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

DDLPC_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

DDLPC_DEVICE void dma16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)((size_t)lds_wave_base), 16, (int)voff, 0, 0, 0);
}

template <int DIMS, int WM, int WN, int MT, int NT, int HALO>
struct Cfg {
  static constexpr int BM = WM * MT * 16;
  static constexpr int BN = WN * NT * 16;
  static constexpr int A_ITERS = (HALO + 63) / 64;              // DMA instrs / wave / chunk
  static constexpr int A_BYTES = A_ITERS * 4 * 1024;            // one halo buffer
  static constexpr int B_ITERS = (3 * BN * 4 + 255) / 256;      // DMA instrs / wave / stage
  static constexpr int B_BYTES = B_ITERS * 4 * 1024;            // one weight buffer
  static constexpr int SS_BYTES = 2 * 512 * 4;                  // prologue scale/shift
  static constexpr int MAIN = 2 * A_BYTES + 2 * B_BYTES;
  static constexpr int OUT = BM * BN * 2 + 2 * 256 * 4;         // epilogue tile + stats
  static constexpr int SMEM = SS_BYTES + (MAIN > OUT ? MAIN : OUT);
};

template <int DIMS, int WM, int WN, int MT, int NT, int HALO>
__global__ __launch_bounds__(256, 2) void conv3_fwd_kernel(ConvFwdArgs p) {
  using C = Cfg<DIMS, WM, WN, MT, NT, HALO>;
  constexpr int BM = C::BM, BN = C::BN;
  constexpr int NG = DIMS == 2 ? 3 : 9;           // (kd, r) kernel rows per chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_scale = reinterpret_cast<float*>(smem);
  float* s_shift = s_scale + 512;
  char* base = smem + C::SS_BYTES;
  // double buffers addressed arithmetically (a runtime-indexed pointer array would spill)
  auto sA = [&](int b) { return base + b * C::A_BYTES; };
  auto sB = [&](int b) { return base + 2 * C::A_BYTES + b * C::B_BYTES; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN;
  const int wn = wave % WN;

  // ---- block -> (m tile, n tile); the n tiles of one m tile share an XCD (halo reuse)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = bid % p.nTilesN;
  int mt_id = bid / p.nTilesN;
  const int mtile = mt_id;
  const int tw_i = mt_id % p.tilesW; mt_id /= p.tilesW;
  const int th_i = mt_id % p.tilesH; mt_id /= p.tilesH;
  const int td_i = mt_id % p.tilesD; mt_id /= p.tilesD;
  const int n_img = mt_id;
  const int d0 = td_i * p.TD, h0 = th_i * p.TH, w0 = tw_i * p.TW;
  const int co0 = ntile * BN;
  const int HW2 = p.TW + 2, HH2 = p.TH + 2;
  const int halo = (DIMS == 3 ? p.TD + 2 : 1) * HH2 * HW2;

  const bool has_pro = p.pscale != nullptr;
  if (has_pro)
    for (int c = tid; c < p.C1; c += 256) { s_scale[c] = p.pscale[c]; s_shift[c] = p.pshift[c]; }

  // ---- buffer descriptors (per image: 32-bit offsets for any batch size)
  const long long img_px = (long long)p.D * p.H * p.W;
  const unsigned x1_bytes = (unsigned)(img_px * p.C1 * 2);
  const unsigned x2_bytes = (unsigned)(img_px * p.C2 * 2);
  const auto rX1 = make_rsrc(p.X1 + n_img * img_px * p.C1, x1_bytes);
  const auto rX2 = make_rsrc(p.C2 > 0 ? p.X2 + n_img * img_px * p.C2 : p.X1, x2_bytes);
  const auto rW = make_rsrc(p.Wt, (unsigned)((long long)p.Cout * p.taps * p.CinW * 2));

  // ---- per-lane DMA geometry (constant over chunks): halo pixel -> source pixel offset
  int a_pix[C::A_ITERS];   // pixel index within the image, -1 if padding / outside
  int a_sub[C::A_ITERS];   // source 8-channel sub-chunk (swizzle applied)
#pragma unroll
  for (int i = 0; i < C::A_ITERS; ++i) {
    const int e = (i * 4 + wave) * 64 + lane;
    const int px = e >> 2;
    a_sub[i] = (e & 3) ^ swz(px);
    a_pix[i] = -1;
    if (px < halo) {
      const int hw = px % HW2, hh = (px / HW2) % HH2;
      const int hd = DIMS == 3 ? px / (HW2 * HH2) : 1;
      const int gw = w0 + hw - 1, gh = h0 + hh - 1, gd = d0 + hd - 1;
      if (gw >= 0 && gw < p.W && gh >= 0 && gh < p.H && gd >= 0 && gd < p.D)
        a_pix[i] = (gd * p.H + gh) * p.W + gw;
    }
  }
  auto issue_A = [&](int chunk, int buf) {
    const int cbase = chunk * BK;
    const bool second = cbase >= p.C1;              // chunk served by X2 (C1 % 32 == 0)
    const auto r = second ? rX2 : rX1;
    const int Cs = second ? p.C2 : p.C1;
    const int c0 = second ? cbase - p.C1 : cbase;
#pragma unroll
    for (int i = 0; i < C::A_ITERS; ++i) {
      const int c8 = c0 + a_sub[i] * 8;
      const unsigned off = (a_pix[i] >= 0 && c8 < Cs) ? (unsigned)(a_pix[i] * Cs + c8) * 2u : kOOB;
      dma16(r, sA(buf) + (i * 4 + wave) * 1024, off);
    }
  };
  auto issue_B = [&](int stage, int buf) {
    const int chunk = stage / NG, grp = stage % NG;
#pragma unroll
    for (int i = 0; i < C::B_ITERS; ++i) {
      const int e = (i * 4 + wave) * 64 + lane;
      const int row = e >> 2;
      const int sub = (e & 3) ^ swz(row);
      const int tl = row / BN, col = row % BN;
      const int co = co0 + col;
      const int c8 = chunk * BK + sub * 8;
      unsigned off = kOOB;
      if (tl < 3 && co < p.Cout && c8 < p.CinW)
        off = (unsigned)(((co * p.taps) + grp * 3 + tl) * p.CinW + c8) * 2u;
      dma16(rW, sB(buf) + (i * 4 + wave) * 1024, off);
    }
  };
  // prologue BN+ReLU applied in LDS on the landed halo (padding stays zero)
  auto transform_A = [&](int chunk, int buf) {
    const int cbase = chunk * BK;
    if (cbase >= p.C1) return;                      // X2 channels: no prologue
#pragma unroll
    for (int i = 0; i < C::A_ITERS; ++i) {
      const int e = (i * 4 + wave) * 64 + lane;    // same element this lane DMA'd
      const int c8 = cbase + a_sub[i] * 8;
      if (a_pix[i] >= 0 && c8 < p.C1) {
        uint4* q = reinterpret_cast<uint4*>(sA(buf) + e * 16);
        float f[8];
        unpack8(*q, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], s_scale[c8 + j], s_shift[c8 + j]), 0.0f);
        *q = pack8(f);
      }
    }
  };

  // ---- per-lane fragment geometry
  const int g = lane >> 4;
  int hp0[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int pix = wm * (MT * 16) + mt * 16 + (lane & 15);
    const int pw = pix % p.TW;
    const int ph = (pix / p.TW) % p.TH;
    const int pd = DIMS == 3 ? pix / (p.TW * p.TH) : 0;
    hp0[mt] = (pd * HH2 + ph) * HW2 + pw;
  }

  f32x4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nchunks = (p.Cin + BK - 1) / BK;
  const int S = nchunks * NG;

  issue_A(0, 0);
  issue_B(0, 0);
  for (int s = 0; s < S; ++s) {
    const int chunk = s / NG, grp = s % NG;
    // stage s operands: B(s) (issued during s-1) and, at grp 0, A(chunk).  At grp 1 the
    // next chunk's halo (issued after B(s) during s-1... see issue order below) may stay
    // in flight.
    if (grp == 1 && chunk + 1 < nchunks) dma_wait<C::A_ITERS>();
    else dma_wait<0>();
    lds_sync();
    if (grp == 0 && has_pro) {
      transform_A(chunk, chunk & 1);
      lds_sync();
    }
    if (s + 1 < S) issue_B(s + 1, (s + 1) & 1);
    if (grp == 0 && chunk + 1 < nchunks) issue_A(chunk + 1, (chunk + 1) & 1);
    // ---- compute: the 3 taps of kernel row (kd, r)
    const char* A = sA(chunk & 1);
    const char* B = sB(s & 1);
    const int kd = DIMS == 3 ? grp / 3 : 0;
    const int r = DIMS == 3 ? grp % 3 : grp;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int tapoff = (kd * HH2 + r) * HW2 + t;
      uint4 af[MT], bfr[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int hp = hp0[mt] + tapoff;
        af[mt] = *reinterpret_cast<const uint4*>(A + lds_off(hp, g));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int row = t * BN + wn * (NT * 16) + nt * 16 + (lane & 15);
        bfr[nt] = *reinterpret_cast<const uint4*>(B + lds_off(row, g));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(af[mt], bfr[nt], acc[mt][nt]);
    }
  }

  // ---- epilogue: bias, bf16, stage [BM][BN] in LDS
  dma_wait<0>();
  lds_sync();
  bf16_t* sO = reinterpret_cast<bf16_t*>(base);
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = wn * (NT * 16) + nt * 16 + (lane & 15);
    const float b = (p.bias != nullptr && co0 + col < p.Cout) ? p.bias[co0 + col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * (MT * 16) + mt * 16 + 4 * (lane >> 4) + i;
        sO[row * BN + col] = f2bf(acc[mt][nt][i] + b);
      }
    }
  }
  lds_sync();

  // ---- coalesced 16-B stores (optionally split into Y1 [0, Co1) / Y2 [Co1, Cout))
  constexpr int CH = BN / 8;
  for (int e = tid; e < BM * CH; e += 256) {
    const int row = e / CH, cg = e % CH;
    const int co = co0 + cg * 8;
    const int pw = row % p.TW, ph = (row / p.TW) % p.TH;
    const int pd = DIMS == 3 ? row / (p.TW * p.TH) : 0;
    const int gw = w0 + pw, gh = h0 + ph, gd = d0 + pd;
    if (gw >= p.W || gh >= p.H || gd >= p.D || co >= p.Cout) continue;
    const long long pix = ((long long)(n_img * p.D + gd) * p.H + gh) * p.W + gw;
    const uint4 v = *reinterpret_cast<const uint4*>(sO + row * BN + cg * 8);
    if (co < p.Co1) *reinterpret_cast<uint4*>(p.Y1 + pix * p.Co1 + co) = v;
    else *reinterpret_cast<uint4*>(p.Y2 + pix * (p.Cout - p.Co1) + (co - p.Co1)) = v;
  }

  // ---- BatchNorm statistics partials over the stored (bf16) values
  if (p.stats != nullptr) {
    constexpr int GROUPS = 256 / BN > 0 ? 256 / BN : 1;
    float* red = reinterpret_cast<float*>(base + BM * BN * 2);
    for (int c0 = 0; c0 < BN; c0 += 256) {
      const int col = c0 + tid % (BN < 256 ? BN : 256);
      const int grp = BN < 256 ? tid / BN : 0;
      float s1 = 0.f, s2 = 0.f;
      if (col < BN) {
        for (int row = grp; row < BM; row += GROUPS) {
          const int pw = row % p.TW, ph = (row / p.TW) % p.TH;
          const int pd = DIMS == 3 ? row / (p.TW * p.TH) : 0;
          if (w0 + pw >= p.W || h0 + ph >= p.H || d0 + pd >= p.D) continue;
          const float v = bf2f(sO[row * BN + col]);
          s1 += v;
          s2 += v * v;
        }
      }
      lds_sync();
      red[tid] = s1;
      red[256 + tid] = s2;
      lds_sync();
      if (grp == 0 && col < BN && co0 + col < p.Cout) {
        float t1 = 0.f, t2 = 0.f;
        for (int q = 0; q < GROUPS; ++q) { t1 += red[q * BN + col]; t2 += red[256 + q * BN + col]; }
        p.stats[(long long)mtile * 2 * p.Cout + co0 + col] = t1;
        p.stats[(long long)mtile * 2 * p.Cout + p.Cout + co0 + col] = t2;
      }
    }
  }
}

template <int DIMS, int WM, int WN, int MT, int NT, int HALO>
void launch_cfg(ConvFwdArgs& a, hipStream_t st) {
  using C = Cfg<DIMS, WM, WN, MT, NT, HALO>;
  const int grid = a.nTilesM * a.nTilesN;
  hipLaunchKernelGGL((conv3_fwd_kernel<DIMS, WM, WN, MT, NT, HALO>), dim3(grid), dim3(256),
                     C::SMEM, st, a);
}

}  // namespace

// Tile configurations (cfg id -> BN, BM, halo capacity):
//   0: BN 32,  BM 256 (4x1 waves, 4x2 tiles)     2-D 16x16 / 32x8   3-D 4x4x16 / 8x4x8
//   1: BN 64,  BM 256 (4x1 waves, 4x4 tiles)     2-D 16x16 / 32x8   3-D 4x4x16 / 8x4x8
//   2: BN 128, BM 128 (2x2 waves, 4x4 tiles)     2-D 8x16 / 16x8    3-D 2x4x16 / 4x4x8
//   3: BN 128, BM 64  (1x4 waves, 4x2 tiles)     2-D 4x16 / 8x8     3-D 1x4x16 / 2x4x8
// (halo capacity = DMA instructions per wave x 64 pixels)
int conv3_fwd_cfg_bn(int cfg) { return cfg == 0 ? 32 : cfg == 1 ? 64 : 128; }
int conv3_fwd_cfg_bm(int cfg) { return cfg <= 1 ? 256 : cfg == 2 ? 128 : 64; }
int conv3_fwd_cfg_halo(int dims, int cfg) {
  if (dims == 2) return cfg <= 1 ? 384 : cfg == 2 ? 192 : 128;
  return cfg <= 1 ? 704 : cfg == 2 ? 448 : 384;
}

void conv3_fwd_launch(ConvFwdArgs& a, int cfg, hipStream_t st) {
  if (a.dims == 2) {
    switch (cfg) {
      case 0: launch_cfg<2, 4, 1, 4, 2, 384>(a, st); break;
      case 1: launch_cfg<2, 4, 1, 4, 4, 384>(a, st); break;
      case 2: launch_cfg<2, 2, 2, 4, 4, 192>(a, st); break;
      default: launch_cfg<2, 1, 4, 4, 2, 128>(a, st); break;
    }
  } else {
    switch (cfg) {
      case 0: launch_cfg<3, 4, 1, 4, 2, 704>(a, st); break;
      case 1: launch_cfg<3, 4, 1, 4, 4, 704>(a, st); break;
      case 2: launch_cfg<3, 2, 2, 4, 4, 448>(a, st); break;
      default: launch_cfg<3, 1, 4, 4, 2, 384>(a, st); break;
    }
  }
}

}  // namespace ddlpc
