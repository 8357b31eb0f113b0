// ConvTranspose 2x2 stride 2 (and 2x2x2 for 3-D) as MFMA GEMMs — K8 of SURVEY.md §2.5.
// Reference: UpBlock.up_sample = nn.ConvTranspose2d(in-out, in-out, kernel_size=2, stride=2)
// (ref.py:606-607,615).  The kernel windows do not overlap, so
//
//   forward  out[2h+i, 2w+j, co] = b[co] + sum_ci x[h,w,ci] W[ci][co][i][j]
//            = GEMM  M = input pixels, N = S*Cout (S = 4 or 8 sub-positions), K = Cin,
//              with a pixel-shuffle scatter epilogue (+ bias);
//   dgrad    dx[h,w,ci] = sum_{sub,co} dOut[up(h,w,sub), co] W[ci][co][sub]
//            = GEMM  M = input pixels, N = Cin, K = S*Cout with a gathering A loader;
//   wgrad    dW[ci][(sub,co)] = sum_px x[px][ci] dOut[up(px,sub)][co]
//            = "TN" GEMM (both operands pixel-major), split-K over pixels, operands read
//              through ds_read_b64_tr_b16, fp32 partial slabs reduced in fixed order.
//
// NT tile: 128 x 64 per 256-thread workgroup, 4 waves of 64 x 32 (4 x 2 v_mfma 16x16x32),
// 32-deep K chunks staged through swizzled LDS with register prefetch (same scheme as the
// 3x3 conv).  TN tile: 64 x 64, 4 waves of 32 x 32, 64-pixel K chunks.
#include <type_traits>

#include "common.h"
#include "conv_lds.h"
#include "ops.h"

namespace ddlpc {

namespace {

constexpr int BK = 32;
DDLPC_DEVICE int swz(int row, int chunk) { return chunk ^ (((row >> 2) & 1) << 1); }
DDLPC_DEVICE int lds_off(int row, int chunk) { return row * 64 + (swz(row, chunk) << 4); }

// output (high-res) pixel of input pixel m and sub-position sub, in 32-bit arithmetic
// (pixel counts < 2^31): with q = m / W (= n*H + h for 2-D), the 2x up-sampled pixel is
// (2q + i) * 2W + 2w + j — one integer division for 2-D, two for 3-D
DDLPC_DEVICE int up_pixel(int m, int sub, int dims, int D, int H, int W) {
  const int q = udiv_pow2(m, W), w = m - q * W;
  if (dims == 2) {
    const int i = sub >> 1, j = sub & 1;
    return (2 * q + i) * (2 * W) + 2 * w + j;
  }
  const int q2 = udiv_pow2(q, H), h = q - q2 * H; // q2 = n*D + d
  const int kd = sub >> 2, i = (sub >> 1) & 1, j = sub & 1;
  (void)D;
  return ((2 * q2 + kd) * (2 * H) + 2 * h + i) * (2 * W) + 2 * w + j;
}

// NT GEMM, KC 32-wide k chunks per pipeline step: every thread has 2*KC A pieces and KC B
// pieces (16 B each) in flight while the previous step's 8*KC MFMAs per wave run, so a
// block exposes the memory latency once per 32*KC of K instead of once per 32 (these GEMMs
// are skinny — K or N is 64..1024 against M up to millions of pixels — and memory bound).
// The dgrad gather addresses are formed without division in the k loop: a step's chunk
// sits inside one sub-position (Cout % 32 == 0), whose up-sampled pixel is the row's base
// pixel plus a per-sub offset.
template <int MODE, int KC, int BN>
__global__ __launch_bounds__(256) void gemm_nt_kernel(GemmArgs p) {
  constexpr int BM = 128;
  constexpr int NT = BN / 32;            // 16-col MFMA tiles per wave (2 wave columns)
  constexpr int NBP = BN / 64;           // B pieces per thread per chunk
  constexpr int A_BYTES = KC * BM * 64, B_BYTES = KC * BN * 64;
  // deferred-BN constants live in otherwise idle LDS: FWD (scale|shift, 2 x 512 floats)
  // behind the operand tiles, used in the k loop; DGRAD (scale|shift|mean|invstd) behind the
  // 16 KB output staging tile, used in the epilogue only
  constexpr int BN_OFF = MODE == GEMM_CONVT_FWD ? A_BYTES + B_BYTES : BM * BN * 2;
  constexpr int BN_BYTES = MODE == GEMM_CONVT_FWD ? 2 * 512 * 4 : 4 * 512 * 4;
  constexpr int SMEM0 = A_BYTES + B_BYTES > BM * BN * 2 ? A_BYTES + B_BYTES : BM * BN * 2;
  constexpr int SMEM = SMEM0 > BN_OFF + BN_BYTES ? SMEM0 : BN_OFF + BN_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  float* s_bn = reinterpret_cast<float*>(smem + BN_OFF);
  char* sA = smem;                       // [KC][BM rows][64 B]
  char* sB = smem + A_BYTES;             // [KC][BN rows][64 B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Cbn = MODE == GEMM_CONVT_FWD ? p.K : p.N;   // channels of the deferred tensor
  const bool bn = p.bn4 != nullptr;
  if (bn && MODE == GEMM_CONVT_FWD) {
    for (int i = tid; i < Cbn; i += 256) {
      s_bn[i] = p.bn4[2 * Cbn + i];              // scale
      s_bn[512 + i] = p.bn4[3 * Cbn + i];        // shift
    }
    __syncthreads();
  }
  const int wm = wave >> 1, wn = wave & 1;
  const int nTilesN = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = bid % nTilesN, mtile = bid / nTilesN;
  const int m0 = mtile * BM;
  const int n0 = ntile * BN;
  const int g = lane >> 4;

  // per-thread rows: A rows (tid>>2) and (tid>>2)+64, B row tid>>2; 8-channel piece tid&3
  const int cq = tid & 3;
  long long arow_off[2];                 // FWD: m*K ; DGRAD: up-pixel base * Cout (-1: none)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + (tid >> 2) + 64 * i;
    if (m >= p.M) { arow_off[i] = -1; continue; }
    if (MODE == GEMM_CONVT_FWD) arow_off[i] = (long long)m * p.K;
    else arow_off[i] = (long long)up_pixel(m, 0, p.dims, p.D, p.H, p.W) * p.Cout;
  }
  int brow_off[NBP];
#pragma unroll
  for (int i = 0; i < NBP; ++i) {
    const int n_b = n0 + (tid >> 2) + 64 * i;
    brow_off[i] = n_b < p.N ? n_b * p.K : -1;
  }
  const int W2 = 2 * p.W, HW4 = 4 * p.H * p.W;
  auto sub_off = [&](int sub) {          // up-pixel offset of sub-position sub (x Cout)
    const int o = (p.dims == 2 ? (sub >> 1) * W2 + (sub & 1)
                               : (sub >> 2) * HW4 + ((sub >> 1) & 1) * W2 + (sub & 1));
    return o * p.Cout;
  };

  uint4 ra[KC][2], rb[KC][NBP];
  int kcur = 0;                          // k base of the step held in ra (FWD prologue)
  auto load = [&](int it) {
    kcur = it * KC * BK;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const int kb = (it * KC + j) * BK;           // chunk base (uniform)
      const int k8 = kb + cq * 8;
      int aoff;                                    // element offset added to the row base
      if (MODE == GEMM_CONVT_FWD) aoff = k8;
      else {
        const int sub = kb / p.Cout;               // uniform per chunk
        aoff = sub_off(sub) + (kb - sub * p.Cout) + cq * 8;
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (arow_off[i] >= 0 && k8 < p.K)
          v = *reinterpret_cast<const uint4*>(p.A + arow_off[i] + aoff);
        ra[j][i] = v;
      }
#pragma unroll
      for (int i = 0; i < NBP; ++i) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (brow_off[i] >= 0 && k8 < p.K) v = *reinterpret_cast<const uint4*>(p.B + (long long)brow_off[i] + k8);
        rb[j][i] = v;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        uint4 v = ra[j][i];
        const int k8 = kcur + j * BK + cq * 8;
        if (MODE == GEMM_CONVT_FWD && bn && arow_off[i] >= 0 && k8 < p.K) {
          float f[8];                    // deferred BN + ReLU of the input activation
          unpack8(v, f);
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = fmaxf(fmaf(f[q], s_bn[k8 + q], s_bn[512 + k8 + q]), 0.f);
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(sA + j * BM * 64 + lds_off((tid >> 2) + 64 * i, cq)) = v;
      }
#pragma unroll
      for (int i = 0; i < NBP; ++i)
        *reinterpret_cast<uint4*>(sB + j * BN * 64 + lds_off((tid >> 2) + 64 * i, cq)) = rb[j][i];
    }
  };

  f32x4_t acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nit = (p.K + BK * KC - 1) / (BK * KC);
  load(0);
  for (int it = 0; it < nit; ++it) {
    __syncthreads();
    store();
    __syncthreads();
    if (it + 1 < nit) load(it + 1);
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      uint4 af[4], bfr[NT];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        af[mt] = *reinterpret_cast<const uint4*>(sA + j * BM * 64 + lds_off(wm * 64 + mt * 16 + (lane & 15), g));
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        bfr[nt] = *reinterpret_cast<const uint4*>(sB + j * BN * 64 + lds_off(wn * (BN / 2) + nt * 16 + (lane & 15), g));
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(af[mt], bfr[nt], acc[mt][nt]);
    }
  }

  __syncthreads();
  bf16_t* sO = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = wn * (BN / 2) + nt * 16 + (lane & 15);
    float b = 0.f;
    if (MODE == GEMM_CONVT_FWD && p.bias != nullptr && n0 + col < p.N) b = p.bias[(n0 + col) % p.Cout];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        sO[(wm * 64 + mt * 16 + 4 * (lane >> 4) + i) * BN + col] = f2bf(acc[mt][nt][i] + b);
  }
  const bool bnst = MODE == GEMM_CONVT_DGRAD && p.bnpart != nullptr;
  if (bnst)
    for (int i = tid; i < Cbn; i += 256) {
      s_bn[i] = p.bn4[2 * Cbn + i];              // scale
      s_bn[512 + i] = p.bn4[3 * Cbn + i];        // shift
      s_bn[1024 + i] = p.bn4[i];                 // mean
      s_bn[1536 + i] = p.bn4[Cbn + i];           // invstd
    }
  __syncthreads();
  bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
  float s1[8], s2[8];                    // BN-backward partials of this thread's 8 channels
#pragma unroll
  for (int q = 0; q < 8; ++q) { s1[q] = 0.f; s2[q] = 0.f; }
  for (int e = tid; e < BM * (BN / 8); e += 256) {
    const int row = e / (BN / 8), cg = e % (BN / 8);
    const int m = m0 + row;
    const int n = n0 + cg * 8;
    if (m >= p.M || n >= p.N) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(sO + row * BN + cg * 8);
    if (MODE == GEMM_CONVT_FWD) {
      const int sub = n / p.Cout, co = n % p.Cout;
      const int up = up_pixel(m, sub, p.dims, p.D, p.H, p.W);
      *reinterpret_cast<uint4*>(C + (long long)up * p.Cout + co) = v;
    } else {
      *reinterpret_cast<uint4*>(C + (long long)m * p.N + n) = v;
      if (bnst) {                        // dyh = dx [y*scale+shift > 0], xhat = (y-mean)*invstd
        float dx[8], yv[8];
        unpack8(v, dx);
        unpack8(*reinterpret_cast<const uint4*>(p.bny + (long long)m * p.N + n), yv);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int c = n + q;
          const float dyh = fmaf(yv[q], s_bn[c], s_bn[512 + c]) > 0.f ? dx[q] : 0.f;
          s1[q] += dyh;
          s2[q] = fmaf(dyh, (yv[q] - s_bn[1024 + c]) * s_bn[1536 + c], s2[q]);
        }
      }
    }
  }
  if (bnst) {
    // threads with equal tid % (BN/8) hold the same channels: fixed-order LDS reduction,
    // then one full-width row per workgroup (zeros outside this channel tile)
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);     // [2][8][256]
#pragma unroll
    for (int q = 0; q < 8; ++q) { red[q * 256 + tid] = s1[q]; red[2048 + q * 256 + tid] = s2[q]; }
    __syncthreads();
    float* row = p.bnpart + (long long)blockIdx.x * 2 * p.N;
    for (int c = tid; c < 2 * p.N; c += 256) {
      const int half = c / p.N, ch = c - half * p.N;
      float t = 0.f;
      if (ch >= n0 && ch < n0 + BN) {
        const int cg = (ch - n0) >> 3, q = (ch - n0) & 7;
        for (int k = cg; k < 256; k += BN / 8) t += red[half * 2048 + q * 256 + k];
      }
      row[c] = t;
    }
  }
}

// ---------------------------------------------------------------- NT forward v2
// The transposed-conv forward GEMM (M = input pixels, N = S*Cout, K = Cin) restructured like
// the 3x3 conv kernels: 8 waves on a 256-pixel x 128-column tile (4 x 2 waves of 64 x 64),
// both operands by LDS-DMA (buffer_load ... lds) into a 3-deep swizzled LDS ring, KS
// 32-channel sub-chunks per stage behind ONE barrier (v1: register staging, two barriers
// per 32 channels, LDS-staged scalar epilogue), the deferred BN + ReLU of x applied in LDS
// by the lane that DMA'd each piece.  The MFMA computes D^T (weights as the A operand), so
// every lane holds 4 consecutive output channels of one pixel; one v_permlane16_swap per
// dword pairs two 16-column tiles into 8 channels and the result leaves as 16-byte stores
// at the pixel-shuffled output position (+ bias), straight from the accumulators.
// Persistent workgroups walk their tiles with the DMA pipeline running across tile
// boundaries: a tile's epilogue stores drain under the next tile's first stages (the
// one-tile-per-workgroup form spent half of the 32^2 -> 64^2 x 256-channel up-sampling in
// its store tail: 165 us without stores, 347 us with them).
// Requires Cin % 32 == 0, (S*Cout) % 128 == 0, Cout % 32 == 0 and Cout <= 512 (launcher-checked).
template <int KS, int BN_ = 128>
struct Nt2Cfg {
  static constexpr int BM = 256, BN = BN_;
  static constexpr int A_BYTES = KS * BM * 64, B_BYTES = KS * BN * 64;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  // ring depth: 3 at KS = 1 (76 KB: still two workgroups per CU), so the DMA of stage s + 2
  // is in flight during two stages' MFMAs instead of one
  static constexpr int NS = KS == 1 ? 3 : 2;
  static constexpr int SS_BYTES = 2 * 512 * 4;                   // BN scale | shift
  static constexpr int SMEM = SS_BYTES + NS * STAGE;             // 76 KB at KS = 1 (BN 256: 100 KB)
  static constexpr int A_IT = KS * BM * 4 / 512;                 // DMA pieces per thread
  static constexpr int B_IT = KS * BN * 4 / 512;
};

// BN 256 (one workgroup per CU, waves of 64 x 128): each A tile is read from L2 half as often
template <int KS, int BN_ = 128>
__global__ __launch_bounds__(512, KS == 1 && BN_ == 128 ? 2 : 1) void gemm_nt_fwd2_kernel(GemmArgs p) {
  using C = Nt2Cfg<KS, BN_>;
  constexpr int BM = C::BM, BN = C::BN;
  constexpr int NTW = BN / 32;                                    // 16-column tiles per wave
  constexpr int NPW = BN / 64;                                    // 32-column pairs per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_bn = reinterpret_cast<float*>(smem);                   // scale [512] | shift [512]
  char* base = smem + C::SS_BYTES;
  auto sA = [&](int b) { return base + b * C::STAGE; };
  auto sB = [&](int b) { return base + b * C::STAGE + C::A_BYTES; };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const bool bn = p.bn4 != nullptr;
  if (bn)
    for (int i = tid; i < p.K; i += 512) { s_bn[i] = p.bn4[2 * p.K + i]; s_bn[512 + i] = p.bn4[3 * p.K + i]; }
  // persistent, XCD-aware: workgroup b sits on XCD x = b % 8 (round-robin dispatch) in slot
  // i = b / 8 of that XCD; the slot keeps ONE column tile n = i % nTilesN for the whole launch
  // (bias and weight rows fixed) and walks the m tiles congruent to x mod 8 with stride
  // 8 * R (R = slots per column tile).  So all nTilesN column tiles of an m tile run at the
  // same time on one XCD and share its A rows in L2.  (Launcher: gridDim.x = 8 * R * nTilesN.)
  const int nTilesN = p.N / BN;
  const int nTilesM = (p.M + BM - 1) / BM;
  const int xcd = (int)blockIdx.x % 8, slot = (int)blockIdx.x / 8;
  const int R = (int)gridDim.x / (8 * nTilesN);
  const int n0 = (slot % nTilesN) * BN;
  const int mfirst = (slot / nTilesN) * 8 + xcd, mstep = 8 * R;
  const int my_tiles = nTilesM > mfirst ? (nTilesM - 1 - mfirst) / mstep + 1 : 0;
  const int nk = p.K / (32 * KS);
  const int S = my_tiles * nk;                                    // pipeline stages
  auto m0_of = [&](int j) __attribute__((always_inline)) { return (mfirst + j * mstep) * BM; };
  const auto rB = convlds::make_rsrc(p.B + (long long)n0 * p.K, (unsigned)((long long)BN * p.K * 2));
  // bias of this lane's output columns, loaded once before any DMA is in flight (a load in the
  // epilogue would make the compiler wait vmcnt(0) on the ring's DMAs)
  float bias_r[NPW][8];
#pragma unroll
  for (int np = 0; np < NPW; ++np) {
    const int c0 = n0 + wn * (BN / 2) + np * 32, cob = c0 % p.Cout;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bias_r[np][i] = p.bias != nullptr ? p.bias[cob + 4 * (lane >> 4) + i] : 0.f;
      bias_r[np][4 + i] = p.bias != nullptr ? p.bias[cob + 16 + 4 * (lane >> 4) + i] : 0.f;
    }
  }
  // per-lane DMA geometry: piece e = i * 512 + tid -> row e >> 2, source piece swizzled
  const int sub8 = ((lane & 3) ^ (((lane >> 4) & 1) << 1)) << 3;   // same for every i
  // issue stage (tile j, chunk kc): A rows past M read as zeros (resource clipped to M)
  auto issue = [&](int j, int kc, int b) __attribute__((always_inline)) {
    const int m0 = m0_of(j);
    const auto rA = convlds::make_rsrc(p.A + (long long)m0 * p.K,
                                       (unsigned)((long long)(p.M - m0 < BM ? p.M - m0 : BM) * p.K * 2));
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) {
      const int e = i * 512 + tid, row = (e >> 2) % BM, sc = (e >> 2) / BM;
      convlds::dma16(rA, sA(b) + (i * 8 + wave) * 1024,
                     (unsigned)((row * p.K + (kc * KS + sc) * 32 + sub8) * 2));
    }
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int e = i * 512 + tid, row = (e >> 2) % BN, sc = (e >> 2) / BN;
      convlds::dma16(rB, sB(b) + (i * 8 + wave) * 1024,
                     (unsigned)((row * p.K + (kc * KS + sc) * 32 + sub8) * 2));
    }
  };
  // deferred BN + ReLU of x on this lane's landed A pieces (rows past M stay zero)
  auto transform = [&](int m0, int kc, char* __restrict__ A) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) {
      const int e = i * 512 + tid, row = (e >> 2) % BM, sc = (e >> 2) / BM;
      if (m0 + row < p.M) {
        const int c8 = (kc * KS + sc) * 32 + sub8;
        uint4* q = reinterpret_cast<uint4*>(A + e * 16);
        float f[8];
        unpack8(*q, f);
        // (the 8 constants as two 16-B LDS reads each, not 16 scalar reads)
        const float4* vs = reinterpret_cast<const float4*>(s_bn + c8);
        const float4* vh = reinterpret_cast<const float4*>(s_bn + 512 + c8);
        const float4 s0 = vs[0], s1 = vs[1], h0 = vh[0], h1 = vh[1];
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
        *q = pack8(f);
      }
    }
  };
  const int g = lane >> 4;
  f32x4_t acc[4][NTW];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const char* __restrict__ A, const char* __restrict__ B) __attribute__((always_inline)) {
#pragma unroll
    for (int sc = 0; sc < KS; ++sc) {
      uint4 af[4], bf[NTW];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        af[mt] = *reinterpret_cast<const uint4*>(A + sc * BM * 64 + lds_off(wm * 64 + mt * 16 + (lane & 15), g));
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt)
        bf[nt] = *reinterpret_cast<const uint4*>(B + sc * BN * 64 + lds_off(wn * (BN / 2) + nt * 16 + (lane & 15), g));
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) acc[mt][nt] = mfma16x16x32(bf[nt], af[mt], acc[mt][nt]);
    }
  };
  // ---- epilogue of tile (m0, n0): lane holds columns n0 + wn*64 + nt*16 + 4g .. +3 of pixel
  // wm*64 + mt*16 + (lane & 15); paired into 16-B stores at the pixel-shuffled output position
  // (+ bias).  Exactly EPI buffer stores per wave (rows past M: out-of-range offset), so the
  // counted waits of the next tile's stages stay exact while they drain
  constexpr int EPI = 4 * NPW;                                    // column pairs x 4 m tiles
  auto epilogue = [&](int m0) __attribute__((always_inline)) {
    const int m_last = min(m0 + BM, p.M) - 1;
    const long long up_lo = up_pixel(m0, 0, p.dims, p.D, p.H, p.W);
    const long long up_hi = up_pixel(m_last, p.dims == 2 ? 3 : 7, p.dims, p.D, p.H, p.W);
    const auto rO = convlds::make_rsrc(reinterpret_cast<bf16_t*>(p.C) + up_lo * p.Cout,
                                       (unsigned)((up_hi - up_lo + 1) * p.Cout * 2));
    int upr[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = m0 + wm * 64 + mt * 16 + (lane & 15);
      upr[mt] = m < p.M ? (int)(up_pixel(m, 0, p.dims, p.D, p.H, p.W) - up_lo) : -1;
    }
#pragma unroll
    for (int np = 0; np < NPW; ++np) {
      const int c0 = n0 + wn * (BN / 2) + np * 32;                // 32 columns in one sub-position
      const int sub = c0 / p.Cout, cob = c0 - sub * p.Cout;
      const int soff = p.dims == 2 ? (sub >> 1) * 2 * p.W + (sub & 1)
                                   : (sub >> 2) * 4 * p.H * p.W + ((sub >> 1) & 1) * 2 * p.W + (sub & 1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4_t& a0 = acc[mt][2 * np];
        const f32x4_t& a1 = acc[mt][2 * np + 1];
        const float* bb = bias_r[np];
        const uint2 lo = make_uint2(pack2(a0[0] + bb[0], a0[1] + bb[1]), pack2(a0[2] + bb[2], a0[3] + bb[3]));
        const uint2 hi = make_uint2(pack2(a1[0] + bb[4], a1[1] + bb[5]), pack2(a1[2] + bb[6], a1[3] + bb[7]));
        const uint4 q = convlds::pair16(lo, hi);
        unsigned off = upr[mt] >= 0 ? (unsigned)(((upr[mt] + soff) * p.Cout + cob + convlds::pair16_ch(lane)) * 2)
                                    : convlds::kOOB;
        asm volatile("" : "+v"(off));                              // store count must not depend on data
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{q.x, q.y, q.z, q.w}, rO, off, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  };
  if (bn) __syncthreads();                                        // s_bn visible
  constexpr int NS = C::NS, PER = C::A_IT + C::B_IT;             // DMAs per thread per stage
  static_assert(NS == 3 || NS == 2, "ring depth");
  // stage s = (tile j, chunk kc); the issue walker (ji, ki) runs NS - 1 stages ahead
  int ji = 0, ki = 0;
  auto advance = [&](int& j1, int& k1) __attribute__((always_inline)) { if (++k1 == nk) { k1 = 0; ++j1; } };
  for (int s = 0; s < NS - 1 && s < S; ++s) { issue(ji, ki, s); advance(ji, ki); }
  int b = 0, bi = NS - 1;                                         // ring slot of stage s / s + NS - 1
  int j = 0, kc = 0, m0 = 0;
  unsigned epi_hist = 0;                                          // bit t: an epilogue at stage s-1-t
  for (int s = 0; s < S; ++s) {
    if (kc == 0) m0 = m0_of(j);
    // stage s landed; younger than its DMA: the DMAs of stages s+1 .. s+NS-2 and the epilogue
    // stores of stages s-NS+1 .. s-1 (issued after DMA(s) within their stage)
    const int dmas = min(S - 1 - s, NS - 2);
    const int epis = __builtin_popcount(epi_hist & ((1u << (NS - 1)) - 1u));
    convlds::vm_wait_dyn(dmas * PER + epis * EPI);
    if (bn) transform(m0, kc, sA(b));
    convlds::lds_sync();
    if (s + NS - 1 < S) { issue(ji, ki, bi); advance(ji, ki); }
    compute(sA(b), sB(b));
    const bool epi = kc == nk - 1;
    epi_hist = (epi_hist << 1) | (epi ? 1u : 0u);
    if (epi) epilogue(m0);
    b = b + 1 == NS ? 0 : b + 1;
    bi = bi + 1 == NS ? 0 : bi + 1;
    advance(j, kc);
  }
}

// ---------------------------------------------------------------- NT data gradient v2
// dx[m][ci] = sum_(sub, co) dOut[up(m, sub)][co] Wd[ci][(sub, co)] (M = input pixels, N = Cin,
// K = S*Cout) on the forward v2 geometry: 8 waves on a 256-pixel x 128-channel tile, both
// operands LDS-DMA'd into a 3-deep swizzled ring, one 32-deep k chunk per stage behind one
// barrier (v1: register staging, two barriers per 4 chunks).  The A operand is a gather: a
// chunk lies inside one sub-position (Cout % 32 == 0), so a lane's piece address is its
// row's up-sampled base pixel (computed once) plus a per-chunk uniform offset.  Epilogue:
// 16-B stores from the accumulators (v_permlane16_swap pairs) and, with the deferred BN of x,
// the BN-backward partials (sum dyh, sum dyh * xhat) of the stored dx against y, one
// full-width row per workgroup (zeros outside its channel tile).
struct Dg2Cfg {
  static constexpr int BM = 256, BN = 128, NS = 3;
  static constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64, STAGE = A_BYTES + B_BYTES;
  static constexpr int SMEM = NS * STAGE;                        // 72 KB: two workgroups per CU
};

__global__ __launch_bounds__(512, 2) void gemm_nt_dgrad2_kernel(GemmArgs p) {
  using C = Dg2Cfg;
  constexpr int BM = C::BM, BN = C::BN, NS = C::NS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto sA = [&](int b) { return smem + b * C::STAGE; };
  auto sB = [&](int b) { return smem + b * C::STAGE + C::A_BYTES; };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4;
  const int nTilesN = p.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / nTilesN) * BM, n0 = (bid % nTilesN) * BN;
  const int sub8 = ((lane & 3) ^ (((lane >> 4) & 1) << 1)) << 3;   // same for every piece
  // A: pieces e = i * 512 + tid -> tile row e >> 2; its up-sampled base pixel x Cout
  int arow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + ((i * 512 + tid) >> 2);
    arow[i] = m < p.M ? up_pixel(m, 0, p.dims, p.D, p.H, p.W) * p.Cout + sub8 : -1;
  }
  const long long a_bytes = (long long)p.M * p.K * 2;            // dOut (launcher: < 2^31)
  const auto rA = convlds::make_rsrc(p.A, (unsigned)a_bytes);
  const auto rB = convlds::make_rsrc(p.B + (long long)n0 * p.K, (unsigned)((long long)BN * p.K * 2));
  const int W2 = 2 * p.W, HW4 = 4 * p.H * p.W;
  const int nk = p.K / 32;
  auto issue = [&](int kc, int b) __attribute__((always_inline)) {
    const int kb = kc * 32, sub = kb / p.Cout;                    // uniform
    const int so = (p.dims == 2 ? (sub >> 1) * W2 + (sub & 1)
                                : (sub >> 2) * HW4 + ((sub >> 1) & 1) * W2 + (sub & 1)) * p.Cout +
                   (kb - sub * p.Cout);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      convlds::dma16(rA, sA(b) + (i * 8 + wave) * 1024, arow[i] >= 0 ? (unsigned)((arow[i] + so) * 2) : convlds::kOOB);
    convlds::dma16(rB, sB(b) + wave * 1024, (unsigned)(((tid >> 2) * p.K + kb + sub8) * 2));
  };
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const char* __restrict__ A, const char* __restrict__ B) __attribute__((always_inline)) {
    uint4 af[4], bf[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) af[mt] = *reinterpret_cast<const uint4*>(A + lds_off(wm * 64 + mt * 16 + (lane & 15), g));
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bf[nt] = *reinterpret_cast<const uint4*>(B + lds_off(wn * 64 + nt * 16 + (lane & 15), g));
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16x16x32(bf[nt], af[mt], acc[mt][nt]);
  };
  constexpr int PER = 3;                                          // DMAs per thread per stage
  for (int j = 0; j < NS - 1 && j < nk; ++j) issue(j, j);
  int b = 0, bi = NS - 1;
  for (int kc = 0; kc < nk; ++kc) {
    if (kc + 1 < nk) convlds::dma_wait<PER>();                    // stage kc landed, kc + 1 in flight
    else convlds::dma_wait<0>();
    convlds::lds_sync();
    if (kc + NS - 1 < nk) issue(kc + NS - 1, bi);
    compute(sA(b), sB(b));
    b = b + 1 == NS ? 0 : b + 1;
    bi = bi + 1 == NS ? 0 : bi + 1;
  }
  // ---- epilogue: lane holds channels n0 + wn*64 + nt*16 + 4g .. +3 of pixel
  // m0 + wm*64 + mt*16 + (lane & 15); pairs of 16-column tiles -> 8 channels per lane
  const bool bnst = p.bnpart != nullptr;
  float* s_bn = reinterpret_cast<float*>(smem);                   // scale|shift|mean|invstd [4][BN]
  // y tile [BM][BN] bf16 (64 KB) LDS-DMA'd into the idle ring in one burst (a load per
  // (pixel tile, column pair) in the epilogue exposed its latency 8 times per wave); 16-B
  // slot sp of row r holds channel piece sp ^ (r & 15): conflict-free row-strided reads
  char* ys = smem + 8192;
  if (bnst) {
    __syncthreads();                                              // every wave is done with the ring
    const auto rY = convlds::make_rsrc(p.bny, (unsigned)((long long)p.M * p.N * 2));
#pragma unroll
    for (int i = 0; i < BM * BN * 2 / 16 / 512; ++i) {
      const int e = i * 512 + tid, r = e >> 4, pc = (e & 15) ^ (r & 15);
      const int m = m0 + r;
      convlds::dma16(rY, ys + (i * 8 + wave) * 1024,
                     m < p.M ? (unsigned)(((long long)m * p.N + n0 + pc * 8) * 2) : convlds::kOOB);
    }
    for (int i = tid; i < 4 * BN; i += 512) {
      const int q = i / BN, c = n0 + i % BN;
      s_bn[i] = p.bn4[(q == 0 ? 2 : q == 1 ? 3 : q == 2 ? 0 : 1) * p.N + c];
    }
    convlds::dma_wait<0>();
    __syncthreads();
  }
  bf16_t* dx = reinterpret_cast<bf16_t*>(p.C);
  const int cl = wn * 64 + convlds::pair16_ch(lane);              // + np * 32: tile-local channel
  float* red = s_bn + 4 * BN;                                     // [wm][2][BN] partials
  // column halves one after the other (16 live partial sums instead of 32: two workgroups
  // per CU need <= 128 VGPRs)
#pragma unroll
  for (int np = 0; np < 2; ++np) {
    float s1[8], s2[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) { s1[q] = 0.f; s2[q] = 0.f; }
    const int c = cl + np * 32;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = m0 + wm * 64 + mt * 16 + (lane & 15);
      const f32x4_t& a0 = acc[mt][2 * np];
      const f32x4_t& a1 = acc[mt][2 * np + 1];
      const uint2 lo = make_uint2(pack2(a0[0], a0[1]), pack2(a0[2], a0[3]));
      const uint2 hi = make_uint2(pack2(a1[0], a1[1]), pack2(a1[2], a1[3]));
      const uint4 q = convlds::pair16(lo, hi);
      if (m < p.M) {
        const long long off = (long long)m * p.N + n0 + c;
        *reinterpret_cast<uint4*>(dx + off) = q;
        if (bnst) {                     // dyh = dx [y*scale+shift > 0], xhat = (y-mean)*invstd
          float d8[8], y8[8];
          unpack8(q, d8);
          const int r = wm * 64 + mt * 16 + (lane & 15);
          unpack8(*reinterpret_cast<const uint4*>(ys + r * 256 + (((c >> 3) ^ (r & 15)) << 4)), y8);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float dyh = fmaf(y8[j], s_bn[c + j], s_bn[BN + c + j]) > 0.f ? d8[j] : 0.f;
            s1[j] += dyh;
            s2[j] = fmaf(dyh, (y8[j] - s_bn[2 * BN + c + j]) * s_bn[3 * BN + c + j], s2[j]);
          }
        }
      }
    }
    if (bnst) {
      // lanes with equal bits 4, 5 hold the same channels: butterfly over the pixel bits
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
          s1[j] += __shfl_xor(s1[j], sh);
          s2[j] += __shfl_xor(s2[j], sh);
        }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          red[(wm * 2 + 0) * BN + c + j] = s1[j];
          red[(wm * 2 + 1) * BN + c + j] = s2[j];
        }
      }
    }
  }
  if (bnst) {
    // the 4 m waves of a column half summed in a fixed order
    __syncthreads();
    float* row = p.bnpart + (long long)blockIdx.x * 2 * p.N;
    for (int e = tid; e < 2 * p.N; e += 512) {
      const int half = e / p.N, ch = e - half * p.N;
      float t = 0.f;
      if (ch >= n0 && ch < n0 + BN) {
        const int c = ch - n0;
        for (int w = 0; w < 4; ++w) t += red[(w * 2 + half) * BN + c];
      }
      row[e] = t;
    }
  }
}

// the v2 data gradient where its shape constraints hold (else gemm_nt_kernel)
bool gemm_nt_dgrad2_ok(const GemmArgs& a) {
  return a.mode == GEMM_CONVT_DGRAD && a.N % 128 == 0 && a.K % 32 == 0 && a.Cout % 32 == 0 &&
         (long long)a.M * a.K * 2 < (1LL << 31) && (long long)a.M * a.N * 2 < (1LL << 31);
}

// 1 = the v2 forward (one 32-channel chunk per stage, two persistent workgroups per CU) where
// its shape constraints hold, 0 = the v1 kernel
int gemm_nt_fwd2_mode(const GemmArgs& a) {
  const bool ok = a.mode == GEMM_CONVT_FWD && a.K % 32 == 0 && a.K <= 512 && a.N % 128 == 0 &&
                  a.Cout % 32 == 0 && a.Cout <= 512;
  return ok ? 1 : 0;
}

// compute units of the current device (the persistent forward's grid)
int device_cus() {
  static int n[64] = {};
  int d = 0;
  (void)hipGetDevice(&d);
  if (d < 0 || d >= 64) d = 0;
  if (n[d] == 0) {
    int v = 0;
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d);
    n[d] = v > 0 ? v : 256;
  }
  return n[d];
}

// ---------------------------------------------------------------- TN (weight gradient)
// C[m = ci][n = (sub, co)] = sum_px x[px][ci] * dOut[up(px, sub)][co]
__global__ __launch_bounds__(256, 2) void gemm_tn_wgrad_kernel(GemmArgs p) {
  constexpr int BM = 64, BN = 64, KT = 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * KT * 128];
  __shared__ float s_bn[2 * 512];
  char* sA = smem;               // [KT px][BM ci]   128-B rows
  char* sB = smem + KT * 128;    // [KT px][BN n]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (p.bn4 != nullptr) {
    for (int i = tid; i < p.M; i += 256) { s_bn[i] = p.bn4[2 * p.M + i]; s_bn[512 + i] = p.bn4[3 * p.M + i]; }
    __syncthreads();
  }
  const int wm = wave >> 1, wn = wave & 1;
  const int nTilesN = (p.N + BN - 1) / BN, nTilesM = (p.M + BM - 1) / BM;
  // tiles of one pixel range innermost in XCD-contiguous order (shared operands hit L2)
  int b = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = b % nTilesN; b /= nTilesN;
  const int mtile = b % nTilesM; b /= nTilesM;
  const int split = b;
  const int m0 = mtile * BM, n0 = ntile * BN;
  const long long npx = (long long)p.K;
  const long long per = (npx + p.splits - 1) / p.splits;
  const long long k_begin = per * split;
  const long long k_end = k_begin + per < npx ? k_begin + per : npx;
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;

  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 ra[2], rb[2];
  auto load = [&](long long k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i;               // 512 elements: 64 rows x 8 chunks
      const int row = e >> 3, cg = e & 7;
      const long long px = k0 + row;
      uint4 va = make_uint4(0, 0, 0, 0), vb = make_uint4(0, 0, 0, 0);
      if (px < k_end) {
        const int ci = m0 + cg * 8;
        if (ci < p.M) va = *reinterpret_cast<const uint4*>(p.A + px * p.Cin + ci);
        const int n = n0 + cg * 8;
        if (n < p.N) {
          const int sub = n / p.Cout, co = n % p.Cout;
          const int up = up_pixel((int)px, sub, p.dims, p.D, p.H, p.W);
          vb = *reinterpret_cast<const uint4*>(p.B + (long long)up * p.Cout + co);
        }
      }
      ra[i] = va;
      rb[i] = vb;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i;
      const int row = e >> 3, cg = e & 7;
      *reinterpret_cast<uint4*>(sA + row * 128 + cg * 16) = ra[i];
      *reinterpret_cast<uint4*>(sB + row * 128 + cg * 16) = rb[i];
    }
  };

  if (k_begin < k_end) load(k_begin);
  for (long long k0 = k_begin; k0 < k_end; k0 += KT) {
    __syncthreads();
    if (p.bn4 != nullptr) {               // deferred BN + ReLU of x (valid pieces only)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + 256 * i;
        const int row = e >> 3, ci = m0 + (e & 7) * 8;
        if (k0 + row < k_end && ci < p.M) {
          float f[8];
          unpack8(ra[i], f);
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = fmaxf(fmaf(f[q], s_bn[ci + q], s_bn[512 + ci + q]), 0.f);
          ra[i] = pack8(f);
        }
      }
    }
    store();
    __syncthreads();
    if (k0 + KT < k_end) load(k0 + KT);
#pragma unroll
    for (int ks = 0; ks < KT / 32; ++ks) {
      uint4 af[2], bfr[2];
      const int r0 = ks * 32 + 8 * g + q;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int c = wm * 32 + mt * 16 + 4 * pp;
        const uint2 lo = lds_read_tr16(sA + r0 * 128 + c * 2);
        const uint2 hi = lds_read_tr16(sA + (r0 + 4) * 128 + c * 2);
        af[mt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int c = wn * 32 + nt * 16 + 4 * pp;
        const uint2 lo = lds_read_tr16(sB + r0 * 128 + c * 2);
        const uint2 hi = lds_read_tr16(sB + (r0 + 4) * 128 + c * 2);
        bfr[nt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma16x16x32(af[mt], bfr[nt], acc[mt][nt]);
    }
  }
  float* out = p.partial + (long long)split * p.M * p.N;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = n0 + wn * 32 + nt * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 32 + mt * 16 + 4 * (lane >> 4) + i;
        if (m < p.M && n < p.N) out[(long long)m * p.N + n] = acc[mt][nt][i];
      }
    }
}

// ---------------------------------------------------------------- TN v2 (weight gradient)
// Same product as gemm_tn_wgrad_kernel with MFMA-sized per-wave tiles: 4 waves of 64 x 64
// (4 x 4 v_mfma 16x16x32 per 32-pixel k step: 16 transposed LDS reads per 16 MFMAs, a
// quarter of the v1 kernel's LDS traffic per FLOP, which saturated the LDS array), a
// BM x BN = 128 x 128 (or 64 x 256 for 64 input channels) workgroup tile, 64-pixel stages
// that arrive by LDS-DMA (buffer_load ... lds, double-buffered, counted vmcnt waits) and
// an XOR swizzle on 32-byte groups so every ds_read_b64_tr_b16 half-wave (8 pixel rows x
// 32 B) touches all 64 banks once.  The gathered dOut rows (4 / 8 sub-positions per input
// pixel) and x are addressed through per-workgroup buffer descriptors (32-bit offsets
// relative to the split's first row: tensors beyond 4 GB are fine).  The deferred BN + ReLU
// of x is applied in LDS by the lane that DMA'd each piece, before the stage barrier.
template <int BM>
struct Tn2Cfg {
  static constexpr int BN = BM == 128 ? 128 : 256;
  static constexpr int WN = BN / 64;                  // waves along n (BM / 64 along m)
  // 64 input channels (the 256^2-level transposed conv: 1.3 GB of operands, 69 GFLOP per
  // pass at batch 128 — memory bound): 32-pixel stages in a 3-deep ring, the DMA of stage
  // s + 2 in flight while s computes.  Wider layers (compute heavier): 64-pixel stages,
  // double-buffered.  (measured per shape, profiles/convt_wgrad_micro_*_s2.txt)
  static constexpr int KT = BM == 64 ? 32 : 64;
  static constexpr int NBUF = BM == 64 ? 3 : 2;
  static constexpr int A_RB = BM * 2, B_RB = BN * 2;  // LDS row bytes
  static constexpr int A_BYTES = KT * A_RB, B_BYTES = KT * B_RB;
  static constexpr int NA = A_BYTES / 4096;           // DMA instructions per wave per stage
  static constexpr int NB = B_BYTES / 4096;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int BN_FLOATS = BM == 128 ? 512 : 64;   // deferred-BN table (M <= 512 / 64)
  static constexpr int SMEM = NBUF * STAGE + 2 * BN_FLOATS * 4;
};
// 32-byte group swizzle of LDS row `row` (rows of >= 256 B: 3 bits; 128-B rows: 2 bits) —
// conflict-free for the half-wave row sets {r..r+3, r+8..r+11} of the transposed reads
template <int RB>
DDLPC_DEVICE int tn2_swz(int row) {
  return RB >= 256 ? ((row & 3) | (((row >> 3) & 1) << 2)) : (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
}

template <int BM>
__global__ __launch_bounds__(256, 2) void gemm_tn_wgrad2_kernel(GemmArgs p) {
  using namespace convlds;
  using Cf = Tn2Cfg<BM>;
  constexpr int BN = Cf::BN, KT = Cf::KT, WN = Cf::WN;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NBUF = Cf::NBUF, NBF = Cf::BN_FLOATS;
  float* s_bn = reinterpret_cast<float*>(smem + NBUF * Cf::STAGE);  // scale [NBF] | shift [NBF]
  auto sA = [&](int b) { return smem + b * Cf::STAGE; };
  auto sB = [&](int b) { return smem + b * Cf::STAGE + Cf::A_BYTES; };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const bool has_bn = p.bn4 != nullptr;
  if (has_bn)
    for (int i = tid; i < p.M; i += 256) { s_bn[i] = p.bn4[2 * p.M + i]; s_bn[NBF + i] = p.bn4[3 * p.M + i]; }
  const int nTilesN = (p.N + BN - 1) / BN, nTilesM = (p.M + BM - 1) / BM;
  int b = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = b % nTilesN; b /= nTilesN;
  const int mtile = b % nTilesM; b /= nTilesM;
  const int split = b;
  const int m0 = mtile * BM, n0 = ntile * BN;
  const long long npx = (long long)p.K;
  const long long per = ((npx + p.splits - 1) / p.splits + KT - 1) / KT * KT;
  const long long k_begin = per * split;
  const long long k_end = k_begin + per < npx ? k_begin + per : npx;
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  if (k_begin < k_end) {
    const int S = p.dims == 2 ? 4 : 8;
    // buffer descriptors relative to this split's first rows (32-bit offsets)
    const long long a_lo = k_begin;
    const auto ra = make_rsrc(p.A + a_lo * p.Cin, (unsigned)((k_end - a_lo) * p.Cin * 2));
    const long long kb0 = k_begin - k_begin % p.W;           // row start: up_pixel is monotone
    const long long b_lo = up_pixel((int)kb0, 0, p.dims, p.D, p.H, p.W);
    const long long b_hi = (long long)up_pixel((int)(k_end - 1), S - 1, p.dims, p.D, p.H, p.W) + 1;
    const auto rb = make_rsrc(p.B + b_lo * p.Cout, (unsigned)((b_hi - b_lo) * p.Cout * 2));
    // per-lane DMA geometry (tile independent): LDS piece e = (i*4 + wave)*64 + lane
    int a_row[Cf::NA], a_col[Cf::NA], b_row[Cf::NB], b_col[Cf::NB], b_sub[Cf::NB];
#pragma unroll
    for (int i = 0; i < Cf::NA; ++i) {
      const int e = (i * 4 + wave) * 64 + lane;
      const int ppr = Cf::A_RB / 16;
      const int row = e / ppr, pc = e % ppr;
      const int lp = (((pc >> 1) ^ tn2_swz<Cf::A_RB>(row)) << 1) | (pc & 1);
      a_row[i] = row;
      a_col[i] = m0 + lp * 8 < p.M ? m0 + lp * 8 : -1;
    }
#pragma unroll
    for (int i = 0; i < Cf::NB; ++i) {
      const int e = (i * 4 + wave) * 64 + lane;
      const int ppr = Cf::B_RB / 16;
      const int row = e / ppr, pc = e % ppr;
      const int lp = (((pc >> 1) ^ tn2_swz<Cf::B_RB>(row)) << 1) | (pc & 1);
      const int n = n0 + lp * 8;
      b_row[i] = row;
      b_sub[i] = n < p.N ? n / p.Cout : -1;
      b_col[i] = n < p.N ? n % p.Cout : 0;
    }
    // 2-D: each B piece's up-sampled pixel walked by carries (the stages are issued in k
    // order, KT pixels apart): (w, 4qW + 2w) of its input pixel plus the sub-position offset,
    // no integer division per piece and stage
    int b_w[Cf::NB], b_base[Cf::NB], b_so[Cf::NB];
    const int W = p.W, dq = KT / W, dw = KT % W, dbase = 4 * W * dq + 2 * dw;
#pragma unroll
    for (int i = 0; i < Cf::NB; ++i) {
      const long long px0 = k_begin + b_row[i];
      const int qq = (int)(px0 / W);
      b_w[i] = (int)(px0 - (long long)qq * W);
      b_base[i] = 4 * qq * W + 2 * b_w[i];
      b_so[i] = b_sub[i] >= 0 ? (b_sub[i] >> 1) * 2 * W + (b_sub[i] & 1) : 0;
    }
    auto issue = [&](long long k0, int buf) {
#pragma unroll
      for (int i = 0; i < Cf::NA; ++i) {
        const long long px = k0 + a_row[i];
        const bool ok = px < k_end && a_col[i] >= 0;
        dma16(ra, sA(buf) + (i * 4 + wave) * 1024,
              ok ? (unsigned)(((px - a_lo) * p.Cin + a_col[i]) * 2) : kOOB);
      }
#pragma unroll
      for (int i = 0; i < Cf::NB; ++i) {
        const long long px = k0 + b_row[i];
        const bool ok = px < k_end && b_sub[i] >= 0;
        long long up;
        if (p.dims == 2) {
          up = ok ? (long long)(b_base[i] + b_so[i]) : b_lo;
          b_w[i] += dw;
          b_base[i] += dbase;
          if (b_w[i] >= W) { b_w[i] -= W; b_base[i] += 2 * W; }
        } else {
          up = ok ? up_pixel((int)px, b_sub[i], p.dims, p.D, p.H, p.W) : b_lo;
        }
        dma16(rb, sB(buf) + (i * 4 + wave) * 1024,
              ok ? (unsigned)(((up - b_lo) * p.Cout + b_col[i]) * 2) : kOOB);
      }
    };
    auto transform = [&](long long k0, int buf) {      // deferred BN + ReLU of this lane's x pieces
#pragma unroll
      for (int i = 0; i < Cf::NA; ++i) {
        if (k0 + a_row[i] < k_end && a_col[i] >= 0) {
          uint4* q = reinterpret_cast<uint4*>(sA(buf) + ((i * 4 + wave) * 64 + lane) * 16);
          float f[8];
          unpack8(*q, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], s_bn[a_col[i] + j], s_bn[NBF + a_col[i] + j]), 0.f);
          *q = pack8(f);
        }
      }
    };
    // transposed-read geometry: lane (g, q, pp) reads row 8g + q (+4) of a 32-row k step,
    // columns 4pp..4pp+3 of a 16-wide m / n fragment
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    auto frag_off = [&](int row, int col, auto rb_tag) {
      constexpr int RB = decltype(rb_tag)::value;
      const int grp = (col >> 4) ^ tn2_swz<RB>(row);
      return row * RB + grp * 32 + (col & 15) * 2;
    };
    using RA = std::integral_constant<int, Cf::A_RB>;
    using RBt = std::integral_constant<int, Cf::B_RB>;
    const int nst = (int)((k_end - k_begin + KT - 1) / KT);
    __syncthreads();                                     // s_bn visible
    // prologue: stages 0 .. NBUF-2 in flight (empty stages past the end are not issued;
    // the waits below count only what was issued)
#pragma unroll
    for (int j = 0; j < NBUF - 1; ++j)
      if (j < nst) issue(k_begin + (long long)j * KT, j);
    constexpr int PER = Cf::NA + Cf::NB;
#pragma unroll 1
    for (int st = 0; st < nst; ++st) {
      const int buf = st % NBUF;
      const long long k0 = k_begin + (long long)st * KT;
      if constexpr (NBUF == 2) {
        // double buffer: stage st + 1 goes out before waiting for st (its buffer was freed
        // by the trailing barrier of the previous iteration)
        if (st + 1 < nst) { issue(k0 + KT, buf ^ 1); dma_wait<PER>(); }
        else dma_wait<0>();
        if (has_bn) transform(k0, buf);
        lds_sync();
      } else {
        // ring: stages issued after st = min(NBUF - 2, nst - 1 - st)
        const int after = min(NBUF - 2, nst - 1 - st);
        if (NBUF >= 4 && after >= 2) dma_wait<2 * PER>();
        else if (after >= 1) dma_wait<PER>();
        else dma_wait<0>();
        if (has_bn) transform(k0, buf);
        lds_sync();
        // the buffer of stage st - 1 is free (every wave is past its compute): refill it
        if (st + NBUF - 1 < nst) issue(k0 + (long long)(NBUF - 1) * KT, (st + NBUF - 1) % NBUF);
      }
      const char* A_ = sA(buf);
      const char* B_ = sB(buf);
#pragma unroll
      for (int ks = 0; ks < KT / 32; ++ks) {
      const int r0 = ks * 32 + 8 * g + q;
      uint4 af[4], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int c = wm * 64 + mt * 16 + 4 * pp;
        const uint2 lo = lds_read_tr16(A_ + frag_off(r0, c, RA{}));
        const uint2 hi = lds_read_tr16(A_ + frag_off(r0 + 4, c, RA{}));
        af[mt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int c = wn * 64 + nt * 16 + 4 * pp;
        const uint2 lo = lds_read_tr16(B_ + frag_off(r0, c, RBt{}));
        const uint2 hi = lds_read_tr16(B_ + frag_off(r0 + 4, c, RBt{}));
        bfr[nt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16x16x32(af[mt], bfr[nt], acc[mt][nt]);
      }
      // 2-deep ring: the next iteration refills THIS buffer right after its barrier, so
      // every wave must be done reading it first
      if (NBUF == 2) lds_sync();
    }
  }
  float* out = p.partial + (long long)split * p.M * p.N;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n = n0 + wn * 64 + nt * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + mt * 16 + 4 * (lane >> 4) + i;
        if (m < p.M && n < p.N) out[(long long)m * p.N + n] = acc[mt][nt][i];
      }
    }
}

// ---------------------------------------------------------------- fused backward (64 ch)
// The 256^2-level transposed conv of the U-Net (64 -> 64 channels, 2-D): its output
// gradient dOut (64 channels at 4x the pixels: the largest tensor of the backward) is read
// ONCE for both gradients instead of once by the data-gradient kernel and again by the
// weight-gradient kernel.  Per 32-pixel stage the workgroup holds x [32 px][64 ci] and the
// gathered dOut rows [32 px][256 (sub, co)] in LDS (the TN v2 pipeline, double-buffered)
// plus the packed data-gradient weights Wd [64 ci][256] resident, and runs
//   weight gradient  dW[ci][n] += x^T dOut        (16 MFMAs / wave, as gemm_tn_wgrad2_kernel)
//   data gradient    dx[px][ci] = dOut Wd^T       (16 MFMAs / wave: wave w owns ci 16w..16w+15)
// The data gradient is stored from registers (8-byte buffer stores, fixed count per wave so
// the counted vmcnt waits stay exact) and, with the deferred BatchNorm of x (bn4), its
// backward partial sums (sum dyh, sum dyh*xhat of the stored dx) accumulate against the
// raw x still in LDS — one [2][64] row per workgroup.  The deferred BN + ReLU of x for the
// weight gradient is applied in registers after the transposed reads (raw x stays in LDS).
struct FbCfg {
  static constexpr int KT = 32, A_RB = 128, B_RB = 512;
  static constexpr int A_BYTES = KT * A_RB, B_BYTES = KT * B_RB;     // 4 KB + 16 KB
  static constexpr int NA = A_BYTES / 4096, NB = B_BYTES / 4096;     // 1 + 4 DMAs / wave
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int WD_BYTES = 64 * 512;                          // resident Wd
  static constexpr int SMEM = 2 * STAGE + WD_BYTES + 4 * 64 * 4;     // + BN table
};

__global__ __launch_bounds__(256, 2) void convt_bwd_fused_kernel(GemmArgs p) {
  using namespace convlds;
  using Cf = FbCfg;
  constexpr int KT = Cf::KT, PER = Cf::NA + Cf::NB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sWd = smem + 2 * Cf::STAGE;
  float* s_bn = reinterpret_cast<float*>(sWd + Cf::WD_BYTES);   // scale | shift | invstd | -mean*invstd
  auto sA = [&](int b) { return smem + b * Cf::STAGE; };
  auto sB = [&](int b) { return smem + b * Cf::STAGE + Cf::A_BYTES; };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool has_bn = p.bn4 != nullptr;
  if (has_bn && tid < 64) {
    const float is = p.bn4[64 + tid];
    s_bn[tid] = p.bn4[128 + tid];
    s_bn[64 + tid] = p.bn4[192 + tid];
    s_bn[128 + tid] = is;
    s_bn[192 + tid] = -p.bn4[tid] * is;
  }
  const int split = xcd_remap(blockIdx.x, gridDim.x);
  const long long npx = (long long)p.K;
  const long long per = ((npx + p.splits - 1) / p.splits + KT - 1) / KT * KT;
  const long long k_begin = per * split;
  const long long k_end = k_begin + per < npx ? k_begin + per : npx;
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float bs1[4] = {0.f, 0.f, 0.f, 0.f}, bs2[4] = {0.f, 0.f, 0.f, 0.f};   // BN partials
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int ci4 = 16 * wave + 4 * g;                  // this lane's 4 dx channels
  if (k_begin < k_end) {
    const long long a_lo = k_begin;
    const auto ra = make_rsrc(p.A + a_lo * 64, (unsigned)((k_end - a_lo) * 64 * 2));
    const long long kb0 = k_begin - k_begin % p.W;
    const long long b_lo = up_pixel((int)kb0, 0, 2, 1, p.H, p.W);
    const long long b_hi = (long long)up_pixel((int)(k_end - 1), 3, 2, 1, p.H, p.W) + 1;
    const auto rb = make_rsrc(p.B + b_lo * 64, (unsigned)((b_hi - b_lo) * 64 * 2));
    const auto rx = make_rsrc(static_cast<bf16_t*>(p.C) + a_lo * 64, (unsigned)((k_end - a_lo) * 64 * 2));
    // resident Wd [ci][n]: 16-B piece pc of row ci stored at pc ^ (ci & 15)
    {
      const auto rw = make_rsrc(p.Wd2, 64 * 256 * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = (i * 4 + wave) * 64 + lane;
        const int row = e >> 5, pc = e & 31;
        dma16(rw, sWd + (i * 4 + wave) * 1024, (unsigned)((row * 256 + ((pc ^ (row & 15)) * 8)) * 2));
      }
    }
    int a_row, a_col, b_row[Cf::NB], b_col[Cf::NB], b_sub[Cf::NB];
    {
      const int e = wave * 64 + lane;
      const int row = e / 8, pc = e % 8;
      a_row = row;
      a_col = ((((pc >> 1) ^ tn2_swz<Cf::A_RB>(row)) << 1) | (pc & 1)) * 8;
    }
#pragma unroll
    for (int i = 0; i < Cf::NB; ++i) {
      const int e = (i * 4 + wave) * 64 + lane;
      const int row = e / 32, pc = e % 32;
      const int n = ((((pc >> 1) ^ tn2_swz<Cf::B_RB>(row)) << 1) | (pc & 1)) * 8;
      b_row[i] = row;
      b_sub[i] = n >> 6;
      b_col[i] = n & 63;
    }
    auto issue = [&](long long k0, int buf) {
      {
        const long long px = k0 + a_row;
        dma16(ra, sA(buf) + wave * 1024, px < k_end ? (unsigned)(((px - a_lo) * 64 + a_col) * 2) : kOOB);
      }
#pragma unroll
      for (int i = 0; i < Cf::NB; ++i) {
        const long long px = k0 + b_row[i];
        const bool ok = px < k_end;
        const long long up = ok ? up_pixel((int)px, b_sub[i], 2, 1, p.H, p.W) : b_lo;
        dma16(rb, sB(buf) + (i * 4 + wave) * 1024, ok ? (unsigned)(((up - b_lo) * 64 + b_col[i]) * 2) : kOOB);
      }
    };
    auto frag_off = [&](int row, int col, auto rb_tag) {
      constexpr int RB = decltype(rb_tag)::value;
      const int grp = (col >> 4) ^ tn2_swz<RB>(row);
      return row * RB + grp * 32 + (col & 15) * 2;
    };
    using RA = std::integral_constant<int, Cf::A_RB>;
    using RBt = std::integral_constant<int, Cf::B_RB>;
    // deferred BN of the weight-gradient A operand, in registers: lane column ci = 16 mt +
    // (lane & 15) for fragment mt
    float asc[4], ash[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) { asc[mt] = 0.f; ash[mt] = 0.f; }
    const int nst = (int)((k_end - k_begin + KT - 1) / KT);
    dma_wait<0>();
    __syncthreads();                                  // Wd + BN table resident
    if (has_bn)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) { asc[mt] = s_bn[16 * mt + (lane & 15)]; ash[mt] = s_bn[64 + 16 * mt + (lane & 15)]; }
    float ysc[4], ysh[4], yis[4], ynm[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ysc[i] = has_bn ? s_bn[ci4 + i] : 0.f;
      ysh[i] = has_bn ? s_bn[64 + ci4 + i] : 0.f;
      yis[i] = has_bn ? s_bn[128 + ci4 + i] : 0.f;
      ynm[i] = has_bn ? s_bn[192 + ci4 + i] : 0.f;
    }
    issue(k_begin, 0);
#pragma unroll 1
    for (int st = 0; st < nst; ++st) {
      const int buf = st & 1;
      const long long k0 = k_begin + (long long)st * KT;
      // in flight (issue order): DMA(st) [, stores(st - 1)], DMA(st + 1)
      if (st + 1 < nst) {
        issue(k0 + KT, buf ^ 1);
        if (st > 0) dma_wait<PER + 2>(); else dma_wait<PER>();
      } else {
        if (st > 0) dma_wait<2>(); else dma_wait<0>();
      }
      lds_sync();
      const char* A_ = sA(buf);
      const char* B_ = sB(buf);
      // ---- weight gradient: dW[ci][n] += sum_px x[px][ci] dOut[px][n]
      {
        const int r0 = 8 * g + q;
        uint4 af[4], bfr[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int c = mt * 16 + 4 * pp;
          const uint2 lo = lds_read_tr16(A_ + frag_off(r0, c, RA{}));
          const uint2 hi = lds_read_tr16(A_ + frag_off(r0 + 4, c, RA{}));
          uint4 v = make_uint4(lo.x, lo.y, hi.x, hi.y);
          if (has_bn) {
            // rows 8g..8g+7 of the stage; rows past the end stay zero
            float f[8];
            unpack8(v, f);
#pragma unroll
            for (int j = 0; j < 8; ++j)
              f[j] = k0 + 8 * g + j < k_end ? fmaxf(fmaf(f[j], asc[mt], ash[mt]), 0.f) : 0.f;
            v = pack8(f);
          }
          af[mt] = v;
        }
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int c = wave * 64 + nt * 16 + 4 * pp;
          const uint2 lo = lds_read_tr16(B_ + frag_off(r0, c, RBt{}));
          const uint2 hi = lds_read_tr16(B_ + frag_off(r0 + 4, c, RBt{}));
          bfr[nt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16x16x32(af[mt], bfr[nt], acc[mt][nt]);
      }
      // ---- data gradient: dx^T[ci][px] = Wd[ci][n] dOut^T[n][px]; wave owns ci 16w..16w+15
      f32x4_t dacc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
      {
        const int wrow = 16 * wave + (lane & 15);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const int lp = 4 * kk + g;                  // logical 16-B piece (8 n) of the k step
          const uint4 aw = lds128(sWd + wrow * 512 + ((lp ^ (wrow & 15)) << 4));
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int prow = 16 * t + (lane & 15);
            const uint4 bx = lds128(B_ + prow * 512 + ((((lp >> 1) ^ tn2_swz<Cf::B_RB>(prow)) << 1 | (lp & 1)) << 4));
            dacc[t] = mfma16x16x32(aw, bx, dacc[t]);
          }
        }
      }
      // dx stores (lane: channels ci4..ci4+3 of pixel 16t + (lane & 15)) + BN partials of
      // the stored values against the raw x in LDS
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int prow = 16 * t + (lane & 15);
        const long long px = k0 + prow;
        const bool ok = px < k_end;
        const uint32_t lo = pack2(dacc[t][0], dacc[t][1]), hi = pack2(dacc[t][2], dacc[t][3]);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{lo, hi}, rx,
                                              ok ? (unsigned)(((px - a_lo) * 64 + ci4) * 2) : kOOB, 0, 0);
        if (has_bn && ok) {
          const uint2 yv = *reinterpret_cast<const uint2*>(A_ + frag_off(prow, ci4, RA{}));
          const float d[4] = {lo_bf(lo), hi_bf(lo), lo_bf(hi), hi_bf(hi)};
          const float y[4] = {lo_bf(yv.x), hi_bf(yv.x), lo_bf(yv.y), hi_bf(yv.y)};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float a = fmaf(y[i], ysc[i], ysh[i]);
            const float dyh = a > 0.f ? d[i] : 0.f;
            const float xh = fmaf(y[i], yis[i], ynm[i]);
            bs1[i] += dyh;
            bs2[i] = fmaf(dyh, xh, bs2[i]);
          }
        }
      }
      lds_sync();                                     // buffer free for stage st + 2
    }
  }
  // weight-gradient partial of this split
  float* out = p.partial + (long long)split * 64 * 256;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n = wave * 64 + nt * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) out[(long long)(mt * 16 + 4 * g + i) * 256 + n] = acc[mt][nt][i];
    }
  if (has_bn) {
    // lanes with equal g hold the same 4 channels: sum over lane & 15, fixed order
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int i = 0; i < 4; ++i) { bs1[i] += __shfl_xor(bs1[i], o, 64); bs2[i] += __shfl_xor(bs2[i], o, 64); }
    if ((lane & 15) == 0) {
      float* row = p.bnpart + (long long)split * 128;
#pragma unroll
      for (int i = 0; i < 4; ++i) { row[ci4 + i] = bs1[i]; row[64 + ci4 + i] = bs2[i]; }
    }
  }
}

}  // namespace

void convt_bwd_fused_launch(GemmArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(convt_bwd_fused_kernel, dim3(a.splits), dim3(256), FbCfg::SMEM, st, a);
}
// (Rejected: one 8-wave workgroup per CU with a 4-slot ring — three 20 KB stages in flight
// instead of one per workgroup — measured 1.5% slower end to end: profiles/r6/convt_fb8_ab_rejected_r6e.log)
int convt_bwd_fused_splits(long long K, int num_cus) {
  return (int)std::max<long long>(1, std::min<long long>(2LL * num_cus, K / 128));   // two per CU
}

int convt_wgrad2_tiles(const GemmArgs& a) {
  const int bm = a.M <= 64 ? 64 : 128;
  const int bn = bm == 64 ? 256 : 128;
  return ((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
}

int gemm_nt_bn(const GemmArgs& a) {
  return a.N % 128 == 0 ? 128 : 64;      // 128-wide N tiles (fwd -9%, dgrad -7%: docs/PERF.md)
}

// workgroups of the NT (forward / data-gradient) launch: one BN-partial row each
long long gemm_nt_grid(const GemmArgs& a) {
  if (gemm_nt_dgrad2_ok(a)) return ((a.M + Dg2Cfg::BM - 1) / Dg2Cfg::BM) * (long long)(a.N / Dg2Cfg::BN);
  const int bn = gemm_nt_bn(a);
  return ((a.M + 127) / 128) * (long long)((a.N + bn - 1) / bn);
}

void gemm_launch(GemmArgs& a, hipStream_t st) {
  if (a.mode == GEMM_CONVT_WGRAD && a.wg2) {
    const int grid = convt_wgrad2_tiles(a) * a.splits;
    if (a.M <= 64)
      hipLaunchKernelGGL(gemm_tn_wgrad2_kernel<64>, dim3(grid), dim3(256), Tn2Cfg<64>::SMEM, st, a);
    else
      hipLaunchKernelGGL(gemm_tn_wgrad2_kernel<128>, dim3(grid), dim3(256), Tn2Cfg<128>::SMEM, st, a);
    return;
  }
  if (a.mode == GEMM_CONVT_WGRAD) {
    const int grid = ((a.M + 63) / 64) * ((a.N + 63) / 64) * a.splits;
    hipLaunchKernelGGL(gemm_tn_wgrad_kernel, dim3(grid), dim3(256), 0, st, a);
    return;
  }
  // measured (B=64 U-Net shapes): the gathered data-gradient A operand gains from wide
  // steps; the forward (contiguous A, K = Cin) runs best at one chunk per step.  The forward
  // uses 128-wide N tiles when N allows (each A tile is read from L2 half as often)
  if (gemm_nt_fwd2_mode(a)) {
    // persistent: 8 XCDs x R slots per column tile x nTilesN column tiles, about two
    // workgroups per CU (76 KB of LDS each; BN 256: one of 100 KB), R no larger than the m
    // tiles need
    // (BN 256 where the m tiles fill the chip: 32^2 -> 64^2 x 256 channels 450 -> 361 us,
    // 16^2 -> 32^2 93 -> 85 us at batch 384; 8^2 -> 16^2 (24k pixels) 29 -> 33 us, so not
    // there — profiles/r6/convt_fwd_bn256_r6t/)
    const bool w256 = a.N % 256 == 0 && a.M >= 65536;
    const int bnt = w256 ? 256 : 128;
    const int ntn = a.N / bnt;
    const long long mt = (a.M + 255) / 256;
    const long long rneed = (mt + 7) / 8;
    const int per_cu = w256 ? 1 : 2;
    const int R = (int)std::max<long long>(1, std::min<long long>(rneed, (long long)per_cu * device_cus() / (8 * ntn)));
    const unsigned grid2 = (unsigned)(8 * R * ntn);
    if (w256)
      hipLaunchKernelGGL((gemm_nt_fwd2_kernel<1, 256>), dim3(grid2), dim3(512), (Nt2Cfg<1, 256>::SMEM), st, a);
    else
      hipLaunchKernelGGL((gemm_nt_fwd2_kernel<1>), dim3(grid2), dim3(512), Nt2Cfg<1>::SMEM, st, a);
    return;
  }
  if (gemm_nt_dgrad2_ok(a)) {
    hipLaunchKernelGGL(gemm_nt_dgrad2_kernel, dim3((unsigned)gemm_nt_grid(a)), dim3(512), Dg2Cfg::SMEM, st, a);
    return;
  }
  const int bn = gemm_nt_bn(a);
  const long long grid = gemm_nt_grid(a);
  const int kc = a.mode == GEMM_CONVT_FWD ? 1 : a.K <= 64 ? 2 : 4;
  if (a.mode == GEMM_CONVT_FWD) {
    if (bn == 128) hipLaunchKernelGGL((gemm_nt_kernel<GEMM_CONVT_FWD, 1, 128>), dim3((unsigned)grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((gemm_nt_kernel<GEMM_CONVT_FWD, 1, 64>), dim3((unsigned)grid), dim3(256), 0, st, a);
  } else if (bn == 128) {
    if (kc == 2) hipLaunchKernelGGL((gemm_nt_kernel<GEMM_CONVT_DGRAD, 2, 128>), dim3((unsigned)grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((gemm_nt_kernel<GEMM_CONVT_DGRAD, 4, 128>), dim3((unsigned)grid), dim3(256), 0, st, a);
  } else if (kc == 2) {
    hipLaunchKernelGGL((gemm_nt_kernel<GEMM_CONVT_DGRAD, 2, 64>), dim3((unsigned)grid), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((gemm_nt_kernel<GEMM_CONVT_DGRAD, 4, 64>), dim3((unsigned)grid), dim3(256), 0, st, a);
  }
}

}  // namespace ddlpc
