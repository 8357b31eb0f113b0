// 3x3 (2-D) / 3x3x3 (3-D) convolution, stride 1, zero padding 1, as an MFMA implicit GEMM
// over NHWC / NDHWC bf16 activations — the U-Net's K1 (forward) and K2 (data gradient)
// of SURVEY.md §2.5.  Reference ops: nn.Conv2d(k=3, padding=1) in DoubleConv (ref.py:579,582).
//
// GEMM view:  M = output pixels, N = output channels, K = taps x input channels.
//
// Tiling (one 256-thread workgroup = 4 waves):
//   * output tile BM pixels (TD x TH x TW box) x BN channels; each wave owns 64 px x 32 ch
//     (4 x 2 tiles of v_mfma_f32_16x16x32_bf16); BM * BN = 8192 for BN in {32, 64, 128};
//   * K loop over 32-channel chunks; for each chunk the (TD+2)(TH+2)(TW+2) input HALO is
//     staged ONCE in LDS and re-read by all 9 (27) taps (vs 9x global re-reads of a
//     per-tap im2col), with the previous layer's BatchNorm-apply + ReLU fused into the
//     staging (so BN outputs never round-trip HBM) and zero padding applied after it;
//   * weights stream per (chunk, 3-tap row) group; staging is register double-buffered:
//     the next group's global loads are issued before the current group's MFMAs;
//   * LDS images use a 16-B chunk XOR swizzle (chunk ^= 2*((row>>2)&1)) that makes every
//     ds_read_b128 fragment read conflict-free for the gfx950 lane groups
//     {0-3,12-15,20-27}/{4-11,16-19,28-31}/... on 64-B rows;
//   * two input tensors are read as one channel-concatenated input (zero-copy
//     torch.cat([up, skip], 1), ref.py:616);
//   * epilogue: + bias, bf16 rounding, tile staged in LDS, 16-B coalesced stores (optionally
//     split across two output tensors: the data gradient of a concat conv), and per-channel
//     (sum, sum^2) partials of the stored values for the BatchNorm statistics (K4), one
//     partial row per M tile (deterministic; reduced by bn_finalize).
//
// The data gradient (K2) is this same kernel run on dY with the flipped, transposed
// weights W'[ci][8-t][co] (packed by weight_pack).
#include "common.h"
#include "ops.h"

namespace ddlpc {

namespace {

constexpr int BK = 32;                 // channels per K chunk
constexpr int ROWB = BK * 2;           // bytes per LDS row (one pixel / one weight row)

DDLPC_DEVICE int swz(int row, int chunk) { return chunk ^ (((row >> 2) & 1) << 1); }
DDLPC_DEVICE int lds_off(int row, int chunk) { return row * ROWB + (swz(row, chunk) << 4); }

template <int DIMS>
struct HaloCap { static constexpr int value = DIMS == 2 ? 352 : 656; };

template <int DIMS, int BN>
struct ConvFwdCfg {
  static constexpr int WAVES_N = BN / 32;
  static constexpr int WAVES_M = 4 / WAVES_N;
  static constexpr int BM = 64 * WAVES_M;
  static constexpr int HALO = HaloCap<DIMS>::value;
  static constexpr int A_ELEMS = HALO * 4;                       // 16-B elements
  static constexpr int A_PER_T = (A_ELEMS + 255) / 256;
  static constexpr int B_ELEMS = 3 * BN * 4;
  static constexpr int B_PER_T = (B_ELEMS + 255) / 256;
  static constexpr int A_BYTES = HALO * ROWB;
  static constexpr int B_BYTES = 3 * BN * ROWB;
  static constexpr int OUT_BYTES = BM * BN * 2;
  static constexpr int MAIN_BYTES = A_BYTES + B_BYTES;
  static constexpr int SMEM = (MAIN_BYTES > OUT_BYTES ? MAIN_BYTES : OUT_BYTES);
};

template <int DIMS, int BN>
__global__ __launch_bounds__(256, 1) void conv3_fwd_kernel(ConvFwdArgs p) {
  using Cfg = ConvFwdCfg<DIMS, BN>;
  constexpr int BM = Cfg::BM;
  constexpr int NTAPS_ROW = 3;                    // taps per (kd, r) group
  constexpr int NGROUPS = DIMS == 2 ? 3 : 9;      // (kd, r) groups
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sA = smem;
  char* sB = smem + Cfg::A_BYTES;
  __shared__ float s_scale[512], s_shift[512];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / Cfg::WAVES_N;
  const int wn = wave % Cfg::WAVES_N;

  // ---- block -> (m tile, n tile), XCD-aware: the n tiles of one m tile share an XCD
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
  const int HW2 = (p.TW + 2), HH2 = (p.TH + 2);
  const int halo = (p.TD + (DIMS == 3 ? 2 : 0)) * HH2 * HW2;

  const bool has_pro = p.pscale != nullptr;
  if (has_pro) {
    for (int c = tid; c < p.C1; c += 256) { s_scale[c] = p.pscale[c]; s_shift[c] = p.pshift[c]; }
  }

  // ---- per-lane fragment geometry
  // A: row (pixel) = lane & 15 of each 16-pixel m sub-tile, k-group g = lane >> 4
  const int g = lane >> 4;
  int hp0[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int pix = wm * 64 + mt * 16 + (lane & 15);
    const int pw = pix % p.TW;
    const int ph = (pix / p.TW) % p.TH;
    const int pd = DIMS == 3 ? pix / (p.TW * p.TH) : 0;
    hp0[mt] = (pd * HH2 + ph) * HW2 + pw;
  }

  const int nchunks = (p.Cin + BK - 1) / BK;
  const int total_it = nchunks * NGROUPS;

  uint4 ra[Cfg::A_PER_T];
  uint4 rb[Cfg::B_PER_T];
  uint32_t a_valid = 0;     // bit i: element i is an in-bounds pixel (apply prologue)

  const long long strideW = 1;
  (void)strideW;

  auto load_A = [&](int chunk) {
    a_valid = 0;
#pragma unroll
    for (int i = 0; i < Cfg::A_PER_T; ++i) {
      const int e = tid + 256 * i;
      const int px = e >> 2, cq = e & 3;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (px < halo) {
        const int hw = px % HW2;
        const int hh = (px / HW2) % HH2;
        const int hd = DIMS == 3 ? px / (HW2 * HH2) : 1;
        const int gw = w0 + hw - 1, gh = h0 + hh - 1, gd = d0 + hd - 1;
        const int c8 = chunk * BK + cq * 8;
        if (gw >= 0 && gw < p.W && gh >= 0 && gh < p.H && gd >= 0 && gd < p.D && c8 < p.Cin) {
          const long long pix = ((long long)(n_img * p.D + gd) * p.H + gh) * p.W + gw;
          const bf16_t* src;
          int C, c;
          if (c8 < p.C1) { src = p.X1; C = p.C1; c = c8; }
          else { src = p.X2; C = p.C2; c = c8 - p.C1; }
          const bf16_t* ptr = src + pix * C + c;
          if ((C & 7) == 0) {
            v = *reinterpret_cast<const uint4*>(ptr);
          } else {                                   // C not a multiple of 8 (first layer)
            uint16_t t[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) t[j] = (c + j < C) ? ptr[j] : (uint16_t)0;
            v = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16),
                           t[6] | (t[7] << 16));
          }
          if (c8 < p.C1) a_valid |= (1u << i);
        }
      }
      ra[i] = v;
    }
  };

  auto load_B = [&](int chunk, int grp) {
#pragma unroll
    for (int i = 0; i < Cfg::B_PER_T; ++i) {
      const int e = tid + 256 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < Cfg::B_ELEMS) {
        const int row = e >> 2, cq = e & 3;
        const int tl = row / BN, col = row % BN;
        const int co = co0 + col;
        const int c8 = chunk * BK + cq * 8;
        if (co < p.Cout && c8 < p.CinW) {
          const int tap = grp * NTAPS_ROW + tl;
          v = *reinterpret_cast<const uint4*>(p.Wt + ((long long)co * p.taps + tap) * p.CinW + c8);
        }
      }
      rb[i] = v;
    }
  };

  auto store_A = [&](int chunk) {
#pragma unroll
    for (int i = 0; i < Cfg::A_PER_T; ++i) {
      const int e = tid + 256 * i;
      const int px = e >> 2, cq = e & 3;
      if (px < halo) {
        uint4 v = ra[i];
        if (has_pro && (a_valid >> i) & 1u) {
          const int c8 = chunk * BK + cq * 8;
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int c = c8 + j < p.C1 ? c8 + j : p.C1 - 1;
            f[j] = fmaxf(fmaf(f[j], s_scale[c], s_shift[c]), 0.0f);
          }
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(sA + lds_off(px, cq)) = v;
      }
    }
  };

  auto store_B = [&]() {
#pragma unroll
    for (int i = 0; i < Cfg::B_PER_T; ++i) {
      const int e = tid + 256 * i;
      if (e < Cfg::B_ELEMS) {
        const int row = e >> 2, cq = e & 3;
        *reinterpret_cast<uint4*>(sB + lds_off(row, cq)) = rb[i];
      }
    }
  };

  f32x4_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  load_A(0);
  load_B(0, 0);
  __syncthreads();   // s_scale/s_shift visible

  for (int it = 0; it < total_it; ++it) {
    const int chunk = it / NGROUPS;
    const int grp = it % NGROUPS;
    __syncthreads();                       // previous compute finished reading LDS
    if (grp == 0) store_A(chunk);
    store_B();
    __syncthreads();
    if (it + 1 < total_it) {               // prefetch next group into registers
      const int nchunk = (it + 1) / NGROUPS, ngrp = (it + 1) % NGROUPS;
      if (ngrp == 0) load_A(nchunk);
      load_B(nchunk, ngrp);
    }
    // ---- compute: 3 taps of this (kd, r) row
    const int kd = DIMS == 3 ? grp / 3 : 0;
    const int r = DIMS == 3 ? grp % 3 : grp;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int tapoff = (kd * HH2 + r) * HW2 + s;
      uint4 af[4], bfr[2];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int hp = hp0[mt] + tapoff;
        af[mt] = *reinterpret_cast<const uint4*>(sA + lds_off(hp, g));
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int row = s * BN + wn * 32 + nt * 16 + (lane & 15);
        bfr[nt] = *reinterpret_cast<const uint4*>(sB + lds_off(row, g));
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma16x16x32(af[mt], bfr[nt], acc[mt][nt]);
    }
  }

  // ---- epilogue: bias, bf16, stage [BM][BN] in LDS
  __syncthreads();
  bf16_t* sO = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int col = wn * 32 + nt * 16 + (lane & 15);
    const float b = (p.bias != nullptr && co0 + col < p.Cout) ? p.bias[co0 + col] : 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + mt * 16 + 4 * (lane >> 4) + i;
        sO[row * BN + col] = f2bf(acc[mt][nt][i] + b);
      }
    }
  }
  __syncthreads();

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
    constexpr int GROUPS = 256 / BN;
    const int col = tid % BN, grp = tid / BN;
    float s1 = 0.f, s2 = 0.f;
    for (int row = grp; row < BM; row += GROUPS) {
      const int pw = row % p.TW, ph = (row / p.TW) % p.TH;
      const int pd = DIMS == 3 ? row / (p.TW * p.TH) : 0;
      if (w0 + pw >= p.W || h0 + ph >= p.H || d0 + pd >= p.D) continue;
      const float v = bf2f(sO[row * BN + col]);
      s1 += v;
      s2 += v * v;
    }
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem + Cfg::OUT_BYTES);
    red[tid] = s1;
    red[256 + tid] = s2;
    __syncthreads();
    if (grp == 0 && co0 + col < p.Cout) {
      float t1 = 0.f, t2 = 0.f;
      for (int q = 0; q < GROUPS; ++q) { t1 += red[q * BN + col]; t2 += red[256 + q * BN + col]; }
      p.stats[(long long)mtile * 2 * p.Cout + co0 + col] = t1;
      p.stats[(long long)mtile * 2 * p.Cout + p.Cout + co0 + col] = t2;
    }
  }
}

template <int DIMS, int BN>
void launch_fwd(ConvFwdArgs& a, hipStream_t st) {
  using Cfg = ConvFwdCfg<DIMS, BN>;
  int smem = Cfg::SMEM;
  if (a.stats != nullptr && smem < Cfg::OUT_BYTES + 2048) smem = Cfg::OUT_BYTES + 2048;
  const int grid = a.nTilesM * a.nTilesN;
  hipLaunchKernelGGL((conv3_fwd_kernel<DIMS, BN>), dim3(grid), dim3(256), smem, st, a);
}

}  // namespace

int conv3_fwd_bm(int bn) { return 8192 / bn; }

void conv3_fwd_launch(ConvFwdArgs& a, int bn, hipStream_t st) {
  if (a.dims == 2) {
    if (bn == 32) launch_fwd<2, 32>(a, st);
    else if (bn == 64) launch_fwd<2, 64>(a, st);
    else launch_fwd<2, 128>(a, st);
  } else {
    if (bn == 32) launch_fwd<3, 32>(a, st);
    else if (bn == 64) launch_fwd<3, 64>(a, st);
    else launch_fwd<3, 128>(a, st);
  }
}

int conv3_halo_cap(int dims) { return dims == 2 ? HaloCap<2>::value : HaloCap<3>::value; }

}  // namespace ddlpc
