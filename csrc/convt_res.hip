// ConvTranspose 2x2(x2) stride 2 with RESIDENT WEIGHTS — K8 of SURVEY.md §2.5, the
// up-sampling of UpBlock (ref.py:606-607,615): forward and data gradient.
//
//   FWD   out[up(m, sub)][co] = b[co] + sum_ci x[m][ci] Wt[(sub, co)][ci]   (M = px, N = S*Cout, K = Cin)
//   DGRAD dx[m][ci] = sum_(sub, co) dOut[up(m, sub)][co] Wd[ci][(sub, co)]  (M = px, N = Cin, K = S*Cout)
//
// Both GEMMs are memory bound (K = 64..512, and the up-sampled side is 4x the other), so the
// design streams the pixel operand once at HBM rate instead of re-staging both operands per
// output tile (gemm_nt_kernel):
//   * each persistent workgroup owns ONE n tile (64 or 128 columns); its weight rows
//     (<= 64 KB bf16) are LDS-DMA'd once and stay resident;
//   * the pixel operand streams as (128-pixel m tile, 32-channel chunk) stages through a
//     3-deep LDS-DMA ring.  FWD reads x rows; DGRAD gathers the 64-B runs of dOut at the
//     up-sampled positions (a chunk lies inside one sub-position: Cout % 32 == 0);
//   * FWD: the deferred BatchNorm + ReLU of x (a block whose output feeds only this conv
//     keeps its pre-BN tensor) is applied in LDS by the lane that DMA'd each 16-B piece;
//     DGRAD: the epilogue accumulates the BatchNorm-backward partials of the stored dx
//     (sum dyh, sum dyh*xhat with dyh = dx [relu active]) — one row per workgroup;
//   * MFMA operand roles as in the 3x3 conv: A = weight rows (n), B = pixels (m), so a
//     lane's accumulator holds 4 consecutive output channels of one pixel and the epilogue
//     writes 8-byte bf16x4 stores from registers (no LDS staging);
//   * every wave issues a FIXED number of DMAs per stage and stores per epilogue (buffer
//     stores, out-of-range offset for masked lanes), so the vmcnt waits are exact counts
//     (the conv3x3_res.hip pipeline).
// The launcher splits the batch into image groups whose tensors fit 31-bit buffer offsets.
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

namespace ddlpc {

namespace {

using namespace convlds;

constexpr int TBM = 128;                    // pixels per m tile
constexpr int TNW = 4;                      // waves: 2 (m) x 2 (n)
constexpr int TMT = 4;                      // 16-pixel MFMA tiles per wave (64 pixels)
constexpr int T_ITERS = TBM * 4 / 64 / TNW; // DMA instructions per wave per stage (= 2)
constexpr int T_ABYTES = TBM * ROWB;        // one ring slot (8 KB)

template <int N>
DDLPC_DEVICE void vmw() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// up(m, 0): the up-sampled pixel of sub-position 0 of low-res pixel m (image-group relative)
DDLPC_DEVICE int up0_of(int m, int dims, int H, int W) {
  const int q = udiv_pow2(m, W), w = m - q * W;
  if (dims == 2) return 4 * q * W + 2 * w;
  const int q2 = udiv_pow2(q, H), h = q - q2 * H;
  return (4 * q2 * H + 2 * h) * (2 * W) + 2 * w;
}
DDLPC_DEVICE int sub_off(int sub, int dims, int H, int W) {
  const int W2 = 2 * W;
  return dims == 2 ? (sub >> 1) * W2 + (sub & 1)
                   : (sub >> 2) * (2 * H) * W2 + ((sub >> 1) & 1) * W2 + (sub & 1);
}

// LDS: [BN constants][resident weights nch x TBN x 64 B][ring NBUF x 8 KB][4 x 16 x (TBN+16) B staging]
//      [DGRAD + stats: 4 x YL KB y slots]
template <int MODE, int TBN, bool BN, int NBUF>
__global__ __launch_bounds__(256, 2) void convt_res_kernel(GemmArgs p, int M, int ss_floats) {
  static_assert(NBUF == 3, "the y-prefetch wait below assumes a 3-deep ring");
  constexpr int TNT = TBN / 32;             // 16-col MFMA tiles per wave (TBN / 2 columns)
  constexpr bool FWD = MODE == GEMM_CONVT_FWD;
  constexpr bool STATS = !FWD && BN;        // DGRAD: BN-backward partials of dx
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_bn = reinterpret_cast<float*>(smem);        // FWD: scale|shift of x; DGRAD: 4 x N
  const int K = p.K, nch = K / BK;
  char* sW = smem + ss_floats * 4;
  char* sX0 = sW + nch * TBN * ROWB;
  auto sX = [&](int b) { return sX0 + b * T_ABYTES; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4;
  const int nTilesN = p.N / TBN;
  const int nTilesM = (M + TBM - 1) / TBM;
  // XCD-aware (launcher: gridDim.x = 8 R nTilesN): workgroup b sits on XCD b % 8 in slot
  // b / 8, keeps column tile slot % nTilesN and walks the m tiles congruent to its XCD, so
  // the nTilesN workgroups of an m tile share its pixel rows in that XCD's L2 (blocks of one
  // m tile on different XCDs read them from HBM once per column tile: up2 forward -6..-11%;
  // with two column tiles (up1) measured +1%, so from four on).  Other grids: b % nTilesN.
  const bool xcd_map = nTilesN >= 4 && (int)gridDim.x % (8 * nTilesN) == 0;
  const int slot = xcd_map ? (int)blockIdx.x / 8 : (int)blockIdx.x;
  const int n0 = slot % nTilesN * TBN;
  const int mstride = (int)gridDim.x / nTilesN;
  const int mfirst = xcd_map ? (slot / nTilesN) * 8 + (int)blockIdx.x % 8 : (int)blockIdx.x / nTilesN;
  const int my_items = mfirst < nTilesM ? (nTilesM - 1 - mfirst) / mstride + 1 : 0;
  const int S = my_items * nch;

  if (BN) {
    const int Cb = FWD ? K : p.N;
    for (int c = tid; c < Cb; c += 256) {
      s_bn[c] = p.bn4[2 * Cb + c];                       // scale
      s_bn[Cb + c] = p.bn4[3 * Cb + c];                  // shift
      if (!FWD) { s_bn[2 * Cb + c] = p.bn4[c]; s_bn[3 * Cb + c] = p.bn4[Cb + c]; }  // mean, invstd
    }
    __syncthreads();
  }
  // bias of this lane's 4 x TNT output channels (FWD), loaded before any DMA is in flight
  float bias_r[TNT][4];
#pragma unroll
  for (int nt = 0; nt < TNT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * (TBN / 2) + nt * 16 + 4 * g + i;
      bias_r[nt][i] = FWD && p.bias != nullptr ? p.bias[n % p.Cout] : 0.f;
    }
#pragma unroll
  for (int nt = 0; nt < TNT; ++nt)
    asm volatile("" ::"v"(bias_r[nt][0]), "v"(bias_r[nt][1]), "v"(bias_r[nt][2]), "v"(bias_r[nt][3]));
  // ---- resident weights: rows n0..n0+TBN-1 of [N][K], chunk-major in LDS
  {
    const auto rW = make_rsrc(p.B + (long long)n0 * K, (unsigned)(TBN * K * 2));
    const int pieces = nch * TBN * 4;
    for (int b = wave * 64; b < pieces; b += TNW * 64) {
      const int e = b + lane;
      const int row = (e >> 2) % TBN, c = (e >> 2) / TBN;
      const int sp = (e & 3) ^ swz(row);
      dma16(rW, sW + b * 16, (unsigned)((row * K + c * BK + sp * 8) * 2));
    }
  }
  // ---- per-lane pixel-operand DMA geometry: element e -> tile row (pixel), source piece
  int x_row[T_ITERS], x_sp8[T_ITERS];
#pragma unroll
  for (int i = 0; i < T_ITERS; ++i) {
    const int e = (i * TNW + wave) * 64 + lane;
    x_row[i] = e >> 2;
    x_sp8[i] = ((e & 3) ^ swz(e >> 2)) * 8;
  }
  const auto rD = make_rsrc(p.A, FWD ? 0u : (unsigned)((long long)M * K * 2));   // DGRAD: dOut
  auto issue = [&](int k, int c, int buf) __attribute__((always_inline)) {
    const int m0 = (mfirst + k * mstride) * TBM;
    if (FWD) {
      const auto r = make_rsrc(p.A + (long long)m0 * K, (unsigned)(TBM * K * 2));
#pragma unroll
      for (int i = 0; i < T_ITERS; ++i) {
        const bool ok = m0 + x_row[i] < M;
        dma16(r, sX(buf) + (i * TNW + wave) * 1024,
              ok ? (unsigned)((x_row[i] * K + c * BK + x_sp8[i]) * 2) : kOOB);
      }
    } else {
      const int kb = c * BK, sub = kb / p.Cout;                     // uniform
      const int koff = sub_off(sub, p.dims, p.H, p.W) * p.Cout + (kb - sub * p.Cout);
#pragma unroll
      for (int i = 0; i < T_ITERS; ++i) {
        const int m = m0 + x_row[i];
        const bool ok = m < M;
        const int up = ok ? up0_of(m, p.dims, p.H, p.W) : 0;
        dma16(rD, sX(buf) + (i * TNW + wave) * 1024,
              ok ? (unsigned)((up * p.Cout + koff + x_sp8[i]) * 2) : kOOB);
      }
    }
  };
  auto transform_body = [&](int k, int c, char* __restrict__ X) __attribute__((always_inline)) {   // FWD deferred BN + ReLU
    const int m0 = (mfirst + k * mstride) * TBM;
    const int o = opaque_zero();
#pragma unroll
    for (int i = 0; i < T_ITERS; ++i) {
      if (m0 + x_row[i] >= M) continue;
      const int e = (i * TNW + wave) * 64 + lane;
      uint4* q = reinterpret_cast<uint4*>(X + e * 16);
      float f[8];
      unpack8(*q, f);
      const int c8 = c * BK + x_sp8[i] + o;
      // (the 16 constants as four 16-B LDS reads, not 16 scalar ones)
      const float4* vs = reinterpret_cast<const float4*>(s_bn + c8);
      const float4* vh = reinterpret_cast<const float4*>(s_bn + K + c8);
      const float4 s0 = vs[0], s1 = vs[1], h0 = vh[0], h1 = vh[1];
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
      *q = pack8(f);
    }
  };
  
  f32x4_t acc[TMT][TNT];
#pragma unroll
  for (int i = 0; i < TMT; ++i)
#pragma unroll
    for (int j = 0; j < TNT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- epilogue: per 16-pixel MFMA row block, the wave stages its bf16 tile (16 px x TBN/2
  // columns, rows padded to TBN + 16 B: conflict-free b64 writes) in a private LDS slot and
  // re-reads it as 16-B pieces, so every store instruction writes whole 64..128-B runs of
  // output rows (the accumulator layout alone gives 32-B runs).  A lane always handles the
  // same piece (column run) pc of pixel rows pxl, pxl + 64/P, ...
  constexpr int P = TBN / 16;                   // 16-B pieces per staged row
  constexpr int RS = TBN + 16;                  // staged row stride (bytes)
  constexpr int EPJ = 16 * P / 64;              // pieces per lane per row block
  constexpr int EPI_STORES = TMT * EPJ;
  char* const stg_w = sX0 + NBUF * T_ABYTES + wave * 16 * RS;
  const int pc = lane % P, pxl = lane / P;
  int col_off;                                  // FWD: off(sub) * Cout + co; DGRAD: n
  {
    const int n = n0 + wn * (TBN / 2) + pc * 8;
    if (FWD) {
      const int sub = n / p.Cout;
      col_off = sub_off(sub, p.dims, p.H, p.W) * p.Cout + (n - sub * p.Cout);
    } else {
      col_off = n;
    }
  }
  float s1[STATS ? 8 : 1], s2[STATS ? 8 : 1];   // BN-backward partials of channels col_off..+7
#pragma unroll
  for (int i = 0; i < (STATS ? 8 : 1); ++i) { s1[i] = 0.f; s2[i] = 0.f; }
  const auto rO = make_rsrc(p.C, (unsigned)((long long)M * p.N * 2));   // < 2^31 (launcher)
  const auto rY = make_rsrc(p.bny, STATS ? (unsigned)((long long)M * p.N * 2) : 0u);
  auto out_off = [&](int m) __attribute__((always_inline)) -> unsigned {
    if (m >= M) return kOOB;
    return (unsigned)((FWD ? up0_of(m, p.dims, p.H, p.W) * p.Cout : m * p.N) + col_off) * 2u;
  };
  // (the staging slot goes in as a restrict-qualified parameter: its LDS accesses then carry
  // alias scopes and do not wait for the ring's in-flight LDS-DMA)
  // DGRAD + stats: the pre-BN y of the pieces a lane stores is LDS-DMA'd one stage AHEAD of
  // the epilogue that consumes it (at the item's last chunk, before that stage's ring DMA)
  // into a per-wave slot, lane-linearly: each lane reads back exactly the 16-B pieces it
  // fetched.  (Loads into registers would make the compiler wait on vmcnt for every DMA
  // and store in flight.)
  constexpr int YL = STATS ? TMT * EPJ : 0;     // DMA instructions per wave per item
  char* const ys_w = stg_w + TNW * 16 * RS - wave * 16 * RS + wave * YL * 1024;
  auto load_y = [&](int k) __attribute__((always_inline)) {
    const int mb = (mfirst + k * mstride) * TBM + wm * 64;
#pragma unroll
    for (int mt = 0; mt < TMT; ++mt)
#pragma unroll
      for (int j = 0; j < EPJ; ++j)
        dma16(rY, ys_w + (mt * EPJ + j) * 1024, out_off(mb + mt * 16 + pxl + j * (64 / P)));
  };
  auto epilogue_body = [&](int k, char* __restrict__ stg, const char* __restrict__ ys)
      __attribute__((always_inline)) {
    const int mb = (mfirst + k * mstride) * TBM + wm * 64;
#pragma unroll
    for (int mt = 0; mt < TMT; ++mt) {
#pragma unroll
      for (int nt = 0; nt < TNT; ++nt) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[mt][nt][i] + bias_r[nt][i];
        *reinterpret_cast<uint2*>(stg + (lane & 15) * RS + (nt * 16 + 4 * g) * 2) =
            make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < EPJ; ++j) {
        const int px = pxl + j * (64 / P);
        const uint4 v = lds128(stg + px * RS + pc * 16);
        unsigned off = out_off(mb + mt * 16 + px);
        asm volatile("" : "+v"(off));                  // store count must not depend on data
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rO, off, 0, 0);
        if (STATS) {      // dyh = dx [y*scale+shift > 0], xhat = (y - mean) * invstd (bf16 dx)
          float dx[8], y[8];
          unpack8(v, dx);
          unpack8(lds128(ys + (mt * EPJ + j) * 1024 + lane * 16), y);
          const int Cb = p.N;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int ch = col_off + i;
            const float dyh = fmaf(y[i], s_bn[ch], s_bn[Cb + ch]) > 0.f ? dx[i] : 0.f;
            s1[STATS ? i : 0] += dyh;
            s2[STATS ? i : 0] = fmaf(dyh, (y[i] - s_bn[2 * Cb + ch]) * s_bn[3 * Cb + ch], s2[STATS ? i : 0]);
          }
        }
      }
    }
  };

  // ---- pipeline (conv3x3_res.hip): the pixel stage s + NBUF - 1 is issued at stage s; per
  // stage a wave issues [epilogue stores of the previous item] [y loads of the current item
  // (DGRAD + stats, last chunk)] then [T_ITERS DMAs].  At the wait of stage s the ops
  // younger than DMA(s) are those issued at stages s-NBUF+2..s-1 (bit j of epi_hist /
  // yl_hist: an epilogue / y loads at stage s-1-j).
  int kp = 0, cp = 0;
  auto advance = [&](int& k1, int& c1) __attribute__((always_inline)) { if (++c1 == nch) { c1 = 0; ++k1; } };
  for (int j = 0; j < NBUF - 1 && j < S; ++j) { issue(kp, cp, j % NBUF); advance(kp, cp); }
  int k = 0, c = 0;
  unsigned epi_hist = 0, yl_hist = 0;
  constexpr unsigned HMASK = (1u << (NBUF - 2)) - 1u;
  for (int s = 0; s < S; ++s) {
    const int dmas = min(S - 1 - s, NBUF - 2);
    const int epis = __builtin_popcount(epi_hist & HMASK);
    const int yls = STATS ? __builtin_popcount(yl_hist & HMASK) : 0;
    // an epilogue stage with stats also needs the y DMAs of stage s-1, which are younger
    // than DMA(s): only DMA(s+1) may stay in flight
    if (STATS && c == 0 && s > 0) vm_wait_dyn(dmas * T_ITERS);
    else vm_wait_dyn(dmas * T_ITERS + epis * EPI_STORES + yls * YL);
    const int buf = s % NBUF;
    if (FWD && BN) transform_body(k, c, sX(buf));
    lds_sync();
    const bool epi = (c == 0 && s > 0);
    epi_hist = (epi_hist << 1) | (epi ? 1u : 0u);
    if (epi) epilogue_body(k - 1, stg_w, ys_w);
    const bool yl = STATS && c == nch - 1;
    yl_hist = (yl_hist << 1) | (yl ? 1u : 0u);
    if (yl) load_y(k);
    if (s + NBUF - 1 < S) { issue(kp, cp, (s + NBUF - 1) % NBUF); advance(kp, cp); }
    // (restrict-qualified lambda parameters give the LDS reads alias scopes, so the
    // compiler does not make them wait for the in-flight LDS-DMA of later stages)
    auto compute = [&](const char* __restrict__ X, const char* __restrict__ Wc) __attribute__((always_inline)) {
      uint4 xf[TMT], wf[TNT];
#pragma unroll
      for (int mt = 0; mt < TMT; ++mt) xf[mt] = lds128(X + lds_off(wm * 64 + mt * 16 + (lane & 15), g));
#pragma unroll
      for (int nt = 0; nt < TNT; ++nt)
        wf[nt] = lds128(Wc + lds_off(wn * (TBN / 2) + nt * 16 + (lane & 15), g));
#pragma unroll
      for (int mt = 0; mt < TMT; ++mt)
#pragma unroll
        for (int nt = 0; nt < TNT; ++nt) acc[mt][nt] = mfma16x16x32(wf[nt], xf[mt], acc[mt][nt]);
    };
    compute(sX(buf), sW + c * TBN * ROWB);
    advance(k, c);
  }
  if (STATS) vmw<0>();                                 // the last item's y DMAs
  if (S > 0) epilogue_body(k - 1, stg_w, ys_w);

  if (STATS) {
    // lanes with equal pc hold the same 8 channels: butterfly over the other lane bits, then
    // a fixed-order sum of the two wm waves in LDS; one [2][N] row per workgroup (zeros
    // outside the n tile)
#pragma unroll
    for (int i = 0; i < (STATS ? 8 : 1); ++i)
#pragma unroll
      for (int sh = P; sh < 64; sh <<= 1) {
        s1[i] += __shfl_xor(s1[i], sh);
        s2[i] += __shfl_xor(s2[i], sh);
      }
    vmw<0>();
    lds_sync();
    float* red = reinterpret_cast<float*>(sX0);        // [wm][2][TBN]
    if (lane < P) {
#pragma unroll
      for (int i = 0; i < (STATS ? 8 : 1); ++i) {
        const int col = wn * (TBN / 2) + pc * 8 + i;
        red[(wm * 2 + 0) * TBN + col] = s1[i];
        red[(wm * 2 + 1) * TBN + col] = s2[i];
      }
    }
    lds_sync();
    float* row = p.bnpart + (long long)blockIdx.x * 2 * p.N;
    for (int e = tid; e < 2 * p.N; e += 256) {
      const int half = e / p.N, ch = e - half * p.N;
      float t = 0.f;
      if (ch >= n0 && ch < n0 + TBN) t = red[half * TBN + ch - n0] + red[(2 + half) * TBN + ch - n0];
      row[e] = t;
    }
  }
}

struct ResPlan {
  int tbn = 0;           // 0: not covered
  int smem = 0, ss_floats = 0, per_cu = 0, nbuf = 3;   // nbuf: ring depth
  long long imgs_per = 0;
  long long img_in = 0;
};

ResPlan plan_of(const GemmArgs& a) {
  ResPlan r;
  if (a.mode == GEMM_CONVT_WGRAD || a.K % BK != 0 || a.Cout % 32 != 0) return r;
  const int S = a.dims == 2 ? 4 : 8;
  int tbn = 0;
  if (a.N % 128 == 0 && 128 * a.K * 2 <= 64 * 1024) tbn = 128;
  else if (a.N % 64 == 0 && 64 * a.K * 2 <= 64 * 1024) tbn = 64;
  if (tbn == 0) return r;
  r.img_in = (long long)a.D * a.H * a.W;
  const long long big_img_bytes = r.img_in * S * a.Cout * 2;    // the up-sampled side
  const long long small_img_bytes = r.img_in * (a.mode == GEMM_CONVT_FWD ? a.K : a.N) * 2;
  if (big_img_bytes >= (1LL << 31) || small_img_bytes >= (1LL << 31)) return r;
  r.tbn = tbn;
  r.ss_floats = a.bn4 == nullptr ? 0 : a.mode == GEMM_CONVT_FWD ? 2 * a.K : 4 * a.N;
  // ring depth 3 (measured: a 6-deep ring is slower on every up-sampling shape at batch 128)
  r.nbuf = 3;
  const bool stats = a.mode == GEMM_CONVT_DGRAD && a.bn4 != nullptr;
  r.smem = r.ss_floats * 4 + a.K / BK * tbn * ROWB + TNW * 16 * (tbn + 16) + r.nbuf * T_ABYTES +
           (stats ? TNW * TMT * (tbn / 64) * 1024 : 0);    // + per-wave y slots (YL KB each)
  // one resident workgroup per CU cannot hide the DMA latency (measured 1.3-2x slower than
  // the GEMM kernel): those shapes keep gemm_nt_kernel
  // (the DGRAD+stats 128-wide variant needs 237 VGPRs: 2 waves per SIMD)
  const int vgpr_cap = (a.mode == GEMM_CONVT_DGRAD && a.bn4 != nullptr && tbn == 128) ? 2 : 3;
  r.per_cu = std::min(vgpr_cap, 160 * 1024 / r.smem);
  if (r.per_cu < 2) { r.tbn = 0; return r; }
  r.imgs_per = std::max<long long>(1, ((1LL << 31) - 1) / std::max(big_img_bytes, small_img_bytes));
  return r;
}

int launch_grid(const ResPlan& r, const GemmArgs& a, int M, int num_cus) {
  const int nTilesN = a.N / r.tbn;
  const int nTilesM = (M + TBM - 1) / TBM;
  const int cap = std::max(1, r.per_cu * num_cus / nTilesN) * nTilesN;
  // XCD-aware grid (the kernel's mapping): 8 XCDs x R slots x nTilesN column tiles
  const int unit = 8 * nTilesN;
  if (nTilesN >= 4 && cap >= unit) return std::min(cap / unit, (nTilesM + 7) / 8) * unit;
  return std::min(cap, nTilesM * nTilesN);
}

}  // namespace

int convt_res_rows(const GemmArgs& a, int num_cus) {
  const ResPlan r = plan_of(a);
  if (r.tbn == 0) return 0;
  int rows = 0;
  for (long long i0 = 0; i0 < a.Nimg; i0 += r.imgs_per) {
    const long long ni = std::min<long long>(r.imgs_per, a.Nimg - i0);
    rows += launch_grid(r, a, (int)(ni * r.img_in), num_cus);
  }
  return rows;
}

bool convt_res_launch(GemmArgs& a, int num_cus, hipStream_t st) {
  const ResPlan r = plan_of(a);
  if (r.tbn == 0) return false;
  const int S = a.dims == 2 ? 4 : 8;
  const bool fwd = a.mode == GEMM_CONVT_FWD, bn = a.bn4 != nullptr;
  int row0 = 0;
  for (long long i0 = 0; i0 < a.Nimg; i0 += r.imgs_per) {
    const long long ni = std::min<long long>(r.imgs_per, a.Nimg - i0);
    const int M = (int)(ni * r.img_in);
    GemmArgs b = a;
    const long long small_c = fwd ? a.K : a.N;        // channels of the low-res tensor
    const long long px0 = i0 * r.img_in;
    if (fwd) {
      b.A = a.A + px0 * small_c;
      b.C = reinterpret_cast<bf16_t*>(a.C) + px0 * S * a.Cout;
    } else {
      b.A = a.A + px0 * S * a.Cout;
      b.C = reinterpret_cast<bf16_t*>(a.C) + px0 * small_c;
      if (bn) { b.bny = a.bny + px0 * small_c; b.bnpart = a.bnpart + (long long)row0 * 2 * a.N; }
    }
    const int grid = launch_grid(r, a, M, num_cus);
    row0 += grid;
#define CT_LAUNCH(MODE, TBN, BNF)                                                               \
  hipLaunchKernelGGL((convt_res_kernel<MODE, TBN, BNF, 3>), dim3(grid), dim3(256), r.smem, st, b, M, \
                     r.ss_floats)
    if (fwd) {
      if (r.tbn == 128) { if (bn) CT_LAUNCH(GEMM_CONVT_FWD, 128, true); else CT_LAUNCH(GEMM_CONVT_FWD, 128, false); }
      else { if (bn) CT_LAUNCH(GEMM_CONVT_FWD, 64, true); else CT_LAUNCH(GEMM_CONVT_FWD, 64, false); }
    } else {
      if (r.tbn == 128) { if (bn) CT_LAUNCH(GEMM_CONVT_DGRAD, 128, true); else CT_LAUNCH(GEMM_CONVT_DGRAD, 128, false); }
      else { if (bn) CT_LAUNCH(GEMM_CONVT_DGRAD, 64, true); else CT_LAUNCH(GEMM_CONVT_DGRAD, 64, false); }
    }
#undef CT_LAUNCH
  }
  return true;
}

}  // namespace ddlpc
