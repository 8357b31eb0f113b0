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
#include "ops.h"

namespace ddlpc {

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

  // block -> (split, plane, ci chunk, co tile); splits innermost share operand tiles
  int b = blockIdx.x;
  const int split = b % p.splits; b /= p.splits;
  const int plane = b % p.planes; b /= p.planes;
  const int cic = b % p.ciChunks; b /= p.ciChunks;
  const int cot = b;
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

template <int DIMS, int BCO>
void launch_wg(ConvWgradArgs& a, hipStream_t st) {
  using Cfg = WgCfg<DIMS, BCO>;
  const int grid = a.coTiles * a.ciChunks * a.planes * a.splits;
  hipLaunchKernelGGL((conv3_wgrad_kernel<DIMS, BCO>), dim3(grid), dim3(256), Cfg::SMEM, st, a);
}

}  // namespace

void conv3_wgrad_launch(ConvWgradArgs& a, int bco, hipStream_t st) {
  if (a.dims == 2) {
    if (bco == 32) launch_wg<2, 32>(a, st); else launch_wg<2, 64>(a, st);
  } else {
    if (bco == 32) launch_wg<3, 32>(a, st); else launch_wg<3, 64>(a, st);
  }
}

int conv3_wgrad_halo_cap(int dims) { return dims == 2 ? WgHalo<2>::value : WgHalo<3>::value; }

}  // namespace ddlpc
