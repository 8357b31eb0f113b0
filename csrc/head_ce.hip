// Fused 1x1 head + softmax cross-entropy + pixel accuracy — K11-K13 of SURVEY.md §2.5.
// Reference: conv_last = nn.Conv2d(64//N, out_classes, 1) (ref.py:641,655),
// nn.CrossEntropyLoss() with mean reduction / ignore_index=-100 (ref.py:703,755) and the
// per-iteration pixel accuracy argmax(outputs,1)==y (ref.py:775).
//
// The logits never touch HBM during training: the forward kernel computes per-pixel logits
// from the bf16 activation (C in {8,16,32,64} channels, any K <= 16 classes, fp32 math), the
// log-sum-exp loss, the arg-max hit and the valid-pixel count, reduced per block.  The
// backward kernel recomputes the logits (192 MACs/pixel: far cheaper than storing them),
// forms dlogits = (softmax - onehot) * dL / count, writes dA = dlogits . Wh (bf16) and
// reduces dWh = sum a (x) dlogits, dbh = sum dlogits through an LDS tile per 256 pixels.
// With the last decoder block's BatchNorm deferred into the head (the training default) the
// backward runs in two passes: a stats pass (dWh, dbh, that BN's backward partial sums; no
// dA store) and head_bn_apply_kernel, which recomputes dA and writes the BN's dY directly —
// y + labels are read twice, but dA never round-trips through HBM and the separate BN-apply
// pass over (dA, y) disappears (256^2 x 128: 5.1 -> 3.2 tensor-sized HBM transfers).
#include "common.h"
#include "ops.h"

namespace ddlpc {

namespace {

constexpr int MAXC = 64, MAXK = 16;

// Classes: the kernels are instantiated for KP in {2, 4, 8, 16} (and 6, the
// Vaihingen class count, unpadded) logit slots and take
// the real class count K <= KP at run time; padded slots carry bias -inf and zero weights
// (sW/sb staged that way in LDS), so they add exp(-inf) = 0 to the softmax, never win the
// arg-max and receive a zero gradient.

// (opaque_zero, common.h: the K*C head weights stay in LDS — uniform-address broadcast
// reads — instead of being hoisted out of the pixel loop into K*C live VGPRs; measured
// 150-256 VGPRs, occupancy 1-3 and spills at C=64 without it)

// The head's input activation, 8 channels at c8.  With a deferred BatchNorm (sBN != null:
// scale [C] | shift [C] in LDS) the tensor holds the block's PRE-BN conv output y and the
// activation relu(y*scale + shift) is formed here, rounded to bf16 exactly as a
// materialised activation would be — the last decoder block never writes it to HBM.
template <int C, bool DEFER>
DDLPC_DEVICE void act8(const bf16_t* ap, int c8, const float* sBN, float (&f)[8]) {
  const uint4 v = *reinterpret_cast<const uint4*>(ap + c8);
  unpack8(v, f);
  if (DEFER) {
    // opaque LDS offset: the compiler would otherwise hoist all 2*C constants out of the
    // pixel loop into live registers and halve the kernel's occupancy
    const float* vb = sBN + opaque_zero();
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], vb[c8 + j], vb[C + c8 + j]), 0.f);
    unpack8(pack8(f), f);
  }
}

// stage Wh [K][C] / bh [K] into LDS as KP padded rows
template <int C, int KP>
DDLPC_DEVICE void load_head(const float* Wh, const float* bh, int K, float* sW, float* sb) {
  for (int i = threadIdx.x; i < KP * C; i += blockDim.x) sW[i] = i < K * C ? Wh[i] : 0.f;
  if (threadIdx.x < KP) sb[threadIdx.x] = (int)threadIdx.x < K ? bh[threadIdx.x] : -INFINITY;
}

// stage != nullptr: also store the (bf16) activation row to LDS for the weight-gradient pass
template <int C, int K, bool DEFER>
DDLPC_DEVICE void logits_of(const bf16_t* ap, const float* sW, const float* sb, const float* sBN,
                            float (&z)[K], bf16_t* stage = nullptr) {
  const int o = opaque_zero();
  sW += o;
  sb += o;
#pragma unroll
  for (int k = 0; k < K; ++k) z[k] = sb[k];
#pragma unroll 1
  for (int c8 = 0; c8 < C; c8 += 8) {
    float f[8];
    act8<C, DEFER>(ap, c8, sBN, f);
    if (stage != nullptr) *reinterpret_cast<uint4*>(stage + c8) = pack8(f);
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) z[k] = fmaf(f[j], sW[k * C + c8 + j], z[k]);
  }
}

// bn4 = [mean | invstd | scale | shift] (C each) -> LDS: scale, shift (+ mean, invstd)
template <int C>
DDLPC_DEVICE const float* load_bn(const float* bn4, float* sBN, bool need_stats) {
  if (bn4 == nullptr) return nullptr;
  for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) sBN[i] = bn4[2 * C + i];
  if (need_stats)
    for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) sBN[2 * C + i] = bn4[i];
  return sBN;
}

template <int C, int K, bool DEFER>
__global__ __launch_bounds__(256) void head_ce_fwd_kernel(
    const bf16_t* __restrict__ a, const float* __restrict__ Wh, const float* __restrict__ bh,
    const int64_t* __restrict__ labels, float* __restrict__ partial, long long P,
    int ignore_index, const float* __restrict__ bn4, int Kreal) {
  __shared__ __attribute__((aligned(16))) float sBNm[4 * C];
  __shared__ float sW[K * C], sb[K];
  load_head<C, K>(Wh, bh, Kreal, sW, sb);
  const float* sBN = DEFER ? load_bn<C>(bn4, sBNm, false) : nullptr;
  __syncthreads();
  float loss = 0.f, correct = 0.f, count = 0.f;
  for (long long px = blockIdx.x * (long long)blockDim.x + threadIdx.x; px < P;
       px += (long long)gridDim.x * blockDim.x) {
    float z[K];
    logits_of<C, K, DEFER>(a + px * C, sW, sb, sBN, z);
    const int64_t y = labels[px];
    float m = z[0];
    int am = 0;
#pragma unroll
    for (int k = 1; k < K; ++k)
      if (z[k] > m) { m = z[k]; am = k; }
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) se += __expf(z[k] - m);
    const float lse = m + __logf(se);
    float zy = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) zy = (k == y) ? z[k] : zy;
    if (y != ignore_index) {
      loss += lse - zy;
      count += 1.f;
    }
    correct += (am == y) ? 1.f : 0.f;
  }
  __shared__ float red[3][4];
  loss = wave_sum(loss);
  correct = wave_sum(correct);
  count = wave_sum(count);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = loss; red[1][w] = correct; red[2][w] = count; }
  __syncthreads();
  if (threadIdx.x < 3) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[threadIdx.x][i];
    partial[blockIdx.x * 3 + threadIdx.x] = t;
  }
}

// out[0] = sum loss / count, out[1] = correct, out[2] = count
__global__ void ce_finalize_kernel(const float* __restrict__ partial, int nb, float* out) {
  double s[3] = {0, 0, 0};
  for (int i = threadIdx.x; i < nb; i += blockDim.x)
    for (int j = 0; j < 3; ++j) s[j] += partial[i * 3 + j];
  __shared__ double red[3][4];
  for (int j = 0; j < 3; ++j) {
    s[j] = wave_sum_d(s[j]);
    if ((threadIdx.x & 63) == 0) red[j][threadIdx.x >> 6] = s[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[3] = {0, 0, 0};
    for (int j = 0; j < 3; ++j)
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t[j] += red[j][w];
    out[0] = (float)(t[0] / (t[2] > 0 ? t[2] : 1.0));
    out[1] = (float)t[1];
    out[2] = (float)t[2];
  }
}

// Backward, channel-split: G = C/8 consecutive lanes share one pixel, each owning 8 channels
// (one 16-B activation load).  Per pixel: partial logits over the lane's channels, summed over
// the G lanes by shuffles; softmax-CE gradient d (fp32, identical on the G lanes); the lane's
// 8 channels of dA = d . Wh (bf16 store); and per-lane accumulators for
//   dWh[k][c8..c8+7] += a * d[k],   dbh[k] += d[k]  (lane c8 == 0),
//   and, with a deferred BatchNorm (bn4 != null), the BN-backward partial sums of the
//   stored dA:  sum dyh, sum dyh * xhat  with dyh = dA * [y*scale + shift > 0]
// — so the last decoder block's BN backward skips its reduction pass.  Accumulators are
// reduced once per (persistent) workgroup: shuffles over the lanes with equal c8, then a
// fixed-order sum over the waves (deterministic), one partial row per workgroup.
// One pixel of the channel-split backward (shared by head_ce_bwd_kernel and
// head_bn_apply_kernel so both form bit-identical values): from this lane's 8 raw input
// channels av and the label, the activation f (the deferred BN + ReLU, bf16-rounded), the
// softmax-CE gradient d[K] (identical on the G lanes of the pixel) and the lane's 8
// channels of dA = d . Wh, rounded to bf16 (pk) exactly as stored.
template <int CTRL>
DDLPC_DEVICE float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// head_pixel with the extras of the fused forward + statistics pass: dA before rounding
// (o8), the log-sum-exp, the label's logit and the arg-max class
template <int C, int K, bool DEFER>
DDLPC_DEVICE void head_pixel_x(const uint4 av, const int64_t lab, const float* __restrict__ w,
                               const float (&bk)[K], const float (&sc)[8], const float (&sh)[8],
                               float gs, int ignore_index, float (&y8)[8], float (&f)[8],
                               float (&d)[K], uint4& pk, float (&o8)[8], float& lse, float& zy,
                               int& am) {
  constexpr int G = C / 8;
  unpack8(av, y8);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = DEFER ? fmaxf(fmaf(y8[j], sc[j], sh[j]), 0.f) : y8[j];
  if (DEFER) unpack8(pack8(f), f);                // the activation rounded as materialised
  // packed f32 math (v_pk_fma_f32: two channels per instruction) — this kernel pair is
  // VALU-issue bound; the per-channel operation order of dA and dWh is unchanged
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const f2_t* w2 = reinterpret_cast<const f2_t*>(w);
  f2_t f2[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) f2[jj] = f2_t{f[2 * jj], f[2 * jj + 1]};
  float z[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    f2_t t2 = f2_t{0.f, 0.f};
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) t2 = __builtin_elementwise_fma(f2[jj], w2[(k * C) / 2 + jj], t2);
    z[k] = t2.x + t2.y;
  }
  // sum over the G lanes of the pixel: DPP lane swaps (xor 1, xor 2 within quads, then the
  // half-row mirror — the quads are uniform by then), no LDS-crossbar permutes
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (G >= 2) z[k] += dpp_f<0xB1>(z[k]);
    if (G >= 4) z[k] += dpp_f<0x4E>(z[k]);
    if (G >= 8) z[k] += dpp_f<0x141>(z[k]);
  }
  float m = -INFINITY;
  am = 0;
  zy = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    z[k] += bk[k];
    if (z[k] > m) { m = z[k]; am = k; }              // first maximum (padded classes: -inf)
    zy = k == lab ? z[k] : zy;
  }
  float se = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) { z[k] = __expf(z[k] - m); se += z[k]; }
  lse = m + __logf(se);
  const float inv = __builtin_amdgcn_rcpf(se);      // (se >= 1: the max term is exp(0))
#pragma unroll
  for (int k = 0; k < K; ++k) d[k] = lab != ignore_index ? (z[k] * inv - (k == lab ? 1.f : 0.f)) * gs : 0.f;
  f2_t o2[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) o2[jj] = f2_t{0.f, 0.f};
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      o2[jj] = __builtin_elementwise_fma(f2_t{d[k], d[k]}, w2[(k * C) / 2 + jj], o2[jj]);
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) { o8[2 * jj] = o2[jj].x; o8[2 * jj + 1] = o2[jj].y; }
  pk = pack8(o8);
}

template <int C, int K, bool DEFER>
DDLPC_DEVICE void head_pixel(const uint4 av, const int64_t lab, const float* __restrict__ w,
                             const float (&bk)[K], const float (&sc)[8], const float (&sh)[8],
                             float gs, int ignore_index, float (&y8)[8], float (&f)[8],
                             float (&d)[K], uint4& pk) {
  float o8[8], lse, zy;
  int am;
  head_pixel_x<C, K, DEFER>(av, lab, w, bk, sc, sh, gs, ignore_index, y8, f, d, pk, o8, lse, zy, am);
}

// STORE = false (deferred BN only): the stats pass of the two-pass head backward — dWh,
// dbh and the BN-backward partials, no dA (head_bn_apply_kernel recomputes it)
//
// LOSS = true (training forward with the deferred BN): the forward itself — loss, pixel hits
// and valid count per workgroup (lossp rows [nb][3]) — fused with the statistics pass at a
// UNIT gradient scale: dWh, dbh and the BN partials (from the unrounded dA) are linear in
// the scale dL/count, which the backward applies on the device (head_wgrad_from_rows,
// head_ce_bn_bwd's pscale) — one pass over the activation and labels instead of two.
template <int C, int K, bool DEFER, bool STORE = true, bool LOSS = false>
__global__ __launch_bounds__(256) void head_ce_bwd_kernel(
    const bf16_t* __restrict__ a, const float* __restrict__ Wh, const float* __restrict__ bh,
    const int64_t* __restrict__ labels, const float* __restrict__ gscale,
    const float* __restrict__ stats3, bf16_t* __restrict__ dA, float* __restrict__ dWp,
    long long P, int ignore_index, const float* __restrict__ bn4, float* __restrict__ bnpart,
    int Kreal, float* __restrict__ lossp = nullptr) {
  static_assert(STORE || DEFER, "the stats-only pass exists for the deferred BatchNorm");
  static_assert(!LOSS || (DEFER && !STORE), "the fused forward is the deferred stats pass");
  constexpr int G = C / 8;                          // lanes per pixel
  constexpr int PPB = 256 / G;                      // pixels per workgroup step
  constexpr int NACC = 8 * K + K + (DEFER ? 16 : 0) + (LOSS ? 3 : 0);
  constexpr int LA = 8 * K + K + (DEFER ? 16 : 0);  // loss | correct | count accumulators
  __shared__ float sred[4][G][NACC];
  __shared__ __attribute__((aligned(16))) float sW[K * C];      // Wh, padded classes zero
  __shared__ __attribute__((aligned(16))) float sXh[2 * C];     // invstd | -mean*invstd
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = lane % G, c8 = cg * 8;
  for (int i = tid; i < K * C; i += 256) sW[i] = i < Kreal * C ? Wh[i] : 0.f;
  if (DEFER)
    for (int i = tid; i < C; i += 256) { sXh[i] = bn4[C + i]; sXh[C + i] = -bn4[i] * bn4[C + i]; }
  // registers: bias (padded classes -inf) and the deferred BN's scale / shift (the ReLU
  // mask); the K x 8 weights and the xhat constants are re-read from LDS per pixel
  float bk[K], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < K; ++k) bk[k] = k < Kreal ? bh[k] : -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = DEFER ? bn4[2 * C + c8 + j] : 0.f;
    sh[j] = DEFER ? bn4[3 * C + c8 + j] : 0.f;
  }
  __syncthreads();
  const float cnt = LOSS ? 1.f : stats3[2];
  const float gs = LOSS ? 1.f : (gscale != nullptr ? gscale[0] : 1.0f) / (cnt > 0.f ? cnt : 1.f);
  float acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = 0.f;
  typedef float f2_t __attribute__((ext_vector_type(2)));
  f2_t accw[K][4];                                  // dWh[k][c8 + 2jj, +1] (packed pairs)
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) accw[k][jj] = f2_t{0.f, 0.f};
  const long long stride = (long long)gridDim.x * PPB;
  // software pipeline: the next pixel's activation + label loads are in flight while this
  // pixel computes.  (Two slots in ping-pong were measured: SQ_WAIT_ANY 0.46 -> 0.25 but
  // VALU-active 0.37 -> 0.68 with 15% more VALU instructions, 442 -> 475 us — this loop is
  // VALU-issue bound, not latency bound; profiles/head_pmc_*_s2.txt)
  long long px = (long long)blockIdx.x * PPB + tid / G;
  uint4 a_nx = make_uint4(0, 0, 0, 0);
  int64_t l_nx = 0;
  if (px < P) { a_nx = *reinterpret_cast<const uint4*>(a + px * C + c8); l_nx = labels[px]; }
#pragma unroll 1
  for (; px < P; px += stride) {
    const uint4 a_cur = a_nx;
    const int64_t lab = l_nx;
    if (px + stride < P) {
      a_nx = *reinterpret_cast<const uint4*>(a + (px + stride) * C + c8);
      l_nx = labels[px + stride];
    }
    float y8[8], f[8], d[K], o8[8], lse, zy;
    int am;
    uint4 pk;
    head_pixel_x<C, K, DEFER>(a_cur, lab, sW + opaque_zero() + c8, bk, sc, sh, gs, ignore_index,
                              y8, f, d, pk, o8, lse, zy, am);
    if (STORE) *reinterpret_cast<uint4*>(dA + px * C + c8) = pk;
    if (LOSS && cg == 0) {
      if (lab != ignore_index) { acc[LA] += lse - zy; acc[LA + 2] += 1.f; }
      acc[LA + 1] += am == lab ? 1.f : 0.f;
    }
    {
      f2_t f2[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) f2[jj] = f2_t{f[2 * jj], f[2 * jj + 1]};
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) accw[k][jj] = __builtin_elementwise_fma(f2[jj], f2_t{d[k], d[k]}, accw[k][jj]);
    }
    if (cg == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) acc[8 * K + k] += d[k];
    }
    if (DEFER) {
      float r[8];
      if (LOSS) {                                    // unit scale: the unrounded dA
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = o8[j];
      } else {
        unpack8(pk, r);                              // BN backward sees the stored dA
      }
      const float* xh = sXh + opaque_zero() + c8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dyh = fmaf(y8[j], sc[j], sh[j]) > 0.f ? r[j] : 0.f;
        acc[9 * K + j] += dyh;
        acc[9 * K + 8 + j] = fmaf(dyh, fmaf(y8[j], xh[j], xh[C + j]), acc[9 * K + 8 + j]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) { acc[k * 8 + 2 * jj] = accw[k][jj].x; acc[k * 8 + 2 * jj + 1] = accw[k][jj].y; }
  // ---- workgroup reduction: lanes with equal c8 (xor over the pixel-slot bits), then waves
#pragma unroll
  for (int o = G; o < 64; o <<= 1)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] += __shfl_xor(acc[i], o, 64);
  if (lane < G)
#pragma unroll
    for (int i = 0; i < NACC; ++i) sred[wave][lane][i] = acc[i];
  __syncthreads();
  const int nout = Kreal * C + Kreal;
  for (int o = tid; o < nout; o += 256) {            // [dW (k, c) | db (k)]
    float t = 0.f;
    if (o < Kreal * C) {
      const int k = o / C, c = o % C;
      for (int wv = 0; wv < 4; ++wv) t += sred[wv][c / 8][k * 8 + c % 8];
    } else {
      const int k = o - Kreal * C;
      for (int wv = 0; wv < 4; ++wv) t += sred[wv][0][8 * K + k];
    }
    dWp[(long long)blockIdx.x * nout + o] = t;
  }
  if (DEFER)
    for (int o = tid; o < 2 * C; o += 256) {        // [sum dyh (c) | sum dyh*xhat (c)]
      const int half = o / C, c = o % C;
      float t = 0.f;
      for (int wv = 0; wv < 4; ++wv) t += sred[wv][c / 8][9 * K + 8 * half + c % 8];
      bnpart[(long long)blockIdx.x * 2 * C + o] = t;
    }
  if (LOSS && tid < 3) {                             // lanes cg == 0 hold them
    float t = 0.f;
    for (int wv = 0; wv < 4; ++wv) t += sred[wv][0][LA + tid];
    lossp[(long long)blockIdx.x * 3 + tid] = t;
  }
}

// The fused training forward + statistics pass for the flagship head (C = 32, deferred
// BatchNorm) with dWh on the matrix cores.  head_ce_bwd_kernel<.., LOSS> keeps the K x 8
// dWh accumulators of each lane's channels in registers (48 VGPRs at K = 6: 200 in all, two
// waves per SIMD, ~1.5 TB/s — latency-bound on its one-pixel prefetch).  Here each wave
// stages its 16 pixels' activation [16 px][32 ch] and dlogits [16 px][16 classes] (split
// into bf16 hi + lo parts: products exact to ~2^-17) in LDS and accumulates
//   dWh^T[class][ch] += dlogits^T[class][px] . act[px][ch]
// with v_mfma_f32_16x16x16_bf16 (the transposed ds_read_b64_tr_b16 gives both operands in
// MFMA layout): 8 accumulator VGPRs instead of 48.  Everything else is head_pixel_x's
// arithmetic.  The pixel loop is wave-uniform (the transposed reads need EXEC all ones):
// tail lanes run with zeroed contributions.
DDLPC_DEVICE f32x4_t mfma16x16x16(const uint2& a, const uint2& b, f32x4_t c) {
  typedef short s4_t __attribute__((ext_vector_type(4)));
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s4_t, a), __builtin_bit_cast(s4_t, b),
                                                   c, 0, 0, 0);
}

template <int K>
__global__ __launch_bounds__(256, 3) void head_fwd_stats_mdw_kernel(
    const bf16_t* __restrict__ a, const float* __restrict__ Wh, const float* __restrict__ bh,
    const int64_t* __restrict__ labels, float* __restrict__ dWp, long long P, int ignore_index,
    const float* __restrict__ bn4, float* __restrict__ bnpart, int Kreal, float* __restrict__ lossp) {
  constexpr int C = 32, G = 4, PPB = 64;
  static_assert(K <= 16, "one 16-class MFMA tile");
  constexpr int NACC = K + 16 + 3;                  // db | BN partials (8 + 8) | loss, hits, count
  constexpr int LB = K + 16;                        // loss accumulators at LB, LB + 1, LB + 2
  __shared__ float sred[4][G][NACC];
  __shared__ __attribute__((aligned(16))) float sW[K * C];      // Wh, padded classes zero
  __shared__ __attribute__((aligned(16))) float sXh[2 * C];     // invstd | -mean*invstd
  // per wave: act [16][32] bf16 (1 KB) | dlogits hi [16][16] (512 B) | lo [16][16]; the end
  // of the kernel reuses it as the wave's dWh^T [16][32] fp32 (2 KB)
  __shared__ __attribute__((aligned(16))) char sT[4][2048];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = lane % G, c8 = cg * 8;
  for (int i = tid; i < K * C; i += 256) sW[i] = i < Kreal * C ? Wh[i] : 0.f;
  for (int i = tid; i < C; i += 256) { sXh[i] = bn4[C + i]; sXh[C + i] = -bn4[i] * bn4[C + i]; }
  float bk[K], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < K; ++k) bk[k] = k < Kreal ? bh[k] : -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = bn4[2 * C + c8 + j]; sh[j] = bn4[3 * C + c8 + j]; }
  __syncthreads();
  char* tA = sT[wave];
  char* tDh = tA + 1024;
  char* tDl = tA + 1536;
  float acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = 0.f;
  f32x4_t dw[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  // transposed-read geometry: 16-lane group g reads pixel rows 4g..4g+3, lane 4q + p of the
  // group supplies row 4g + q, columns 4p..4p+3 (+16 for the second channel tile)
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int rA = (4 * g + q) * 64 + pq * 8;          // act row: 32 ch x 2 B
  const int rD = (4 * g + q) * 32 + pq * 8;          // dlogit row: 16 classes x 2 B
  const int p16 = lane >> 2;                         // this lane's pixel within the wave's 16
  const long long stride = (long long)gridDim.x * PPB;
  long long base = (long long)blockIdx.x * PPB;
  long long px = base + tid / G;
  // (rejected: a second pixel of prefetch spills at three workgroups per CU)
  uint4 a_nx = make_uint4(0, 0, 0, 0);
  int64_t l_nx = ignore_index;
  if (px < P) { a_nx = *reinterpret_cast<const uint4*>(a + px * C + c8); l_nx = labels[px]; }
#pragma unroll 1
  for (; base < P; base += stride, px += stride) {   // wave-uniform trip count
    const bool valid = px < P;
    const uint4 a_cur = a_nx;
    const int64_t lab = l_nx;
    if (px + stride < P) {
      a_nx = *reinterpret_cast<const uint4*>(a + (px + stride) * C + c8);
      l_nx = labels[px + stride];
    }
    float y8[8], f[8], d[K], o8[8], lse, zy;
    int am;
    uint4 pk;
    head_pixel_x<C, K, true>(a_cur, lab, sW + opaque_zero() + c8, bk, sc, sh, 1.f, ignore_index,
                             y8, f, d, pk, o8, lse, zy, am);
    if (!valid) {                                     // tail lane: contributes nothing
#pragma unroll
      for (int j = 0; j < 8; ++j) { f[j] = 0.f; o8[j] = 0.f; }
#pragma unroll
      for (int k = 0; k < K; ++k) d[k] = 0.f;
    }
    // stage: act row (this lane's 8 channels), dlogit hi / lo (classes 4 cg .. 4 cg + 3)
    *reinterpret_cast<uint4*>(tA + p16 * 64 + cg * 16) = pack8(f);
    {
      float dh[4], dl[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) v = (4 * cg + i == k) ? d[k] : v;
        const uint32_t h2 = pack2(v, 0.f);
        dh[i] = lo_bf(h2);
        dl[i] = v - dh[i];
      }
      *reinterpret_cast<uint2*>(tDh + p16 * 32 + cg * 8) = make_uint2(pack2(dh[0], dh[1]), pack2(dh[2], dh[3]));
      *reinterpret_cast<uint2*>(tDl + p16 * 32 + cg * 8) = make_uint2(pack2(dl[0], dl[1]), pack2(dl[2], dl[3]));
    }
    const uint2 ah = lds_read_tr16(tDh + rD);
    const uint2 al = lds_read_tr16(tDl + rD);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const uint2 b = lds_read_tr16(tA + rA + nt * 32);
      dw[nt] = mfma16x16x16(ah, b, dw[nt]);
      dw[nt] = mfma16x16x16(al, b, dw[nt]);
    }
    if (valid) {
      if (cg == 0) {
        if (lab != ignore_index) { acc[LB] += lse - zy; acc[LB + 2] += 1.f; }
        acc[LB + 1] += am == lab ? 1.f : 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] += d[k];
      }
      const float* xh = sXh + opaque_zero() + c8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {                   // unit scale: the unrounded dA
        const float dyh = fmaf(y8[j], sc[j], sh[j]) > 0.f ? o8[j] : 0.f;
        acc[K + j] += dyh;
        acc[K + 8 + j] = fmaf(dyh, fmaf(y8[j], xh[j], xh[C + j]), acc[K + 8 + j]);
      }
    }
  }
  // ---- workgroup reduction.  dWh: each wave's D (lane: class 4g + i, channel 16 nt + (lane & 15))
  // to its LDS slot, then the 4 waves summed in a fixed order
  float* wd = reinterpret_cast<float*>(tA);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) wd[(4 * g + i) * 32 + nt * 16 + (lane & 15)] = dw[nt][i];
  // db / BN partials / loss: lanes with equal cg (xor over the pixel-slot bits), then waves
#pragma unroll
  for (int o = G; o < 64; o <<= 1)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] += __shfl_xor(acc[i], o, 64);
  if (lane < G)
#pragma unroll
    for (int i = 0; i < NACC; ++i) sred[wave][lane][i] = acc[i];
  __syncthreads();
  const int nout = Kreal * C + Kreal;
  for (int o = tid; o < nout; o += 256) {            // [dW (k, c) | db (k)]
    float t = 0.f;
    if (o < Kreal * C) {
      const int k = o / C, c = o % C;
      for (int wv = 0; wv < 4; ++wv) t += reinterpret_cast<const float*>(sT[wv])[k * 32 + c];
    } else {
      const int k = o - Kreal * C;
      for (int wv = 0; wv < 4; ++wv) t += sred[wv][0][k];
    }
    dWp[(long long)blockIdx.x * nout + o] = t;
  }
  for (int o = tid; o < 2 * C; o += 256) {           // [sum dyh (c) | sum dyh*xhat (c)]
    const int half = o / C, c = o % C;
    float t = 0.f;
    for (int wv = 0; wv < 4; ++wv) t += sred[wv][c / 8][K + 8 * half + c % 8];
    bnpart[(long long)blockIdx.x * 2 * C + o] = t;
  }
  if (tid < 3) {                                     // lanes cg == 0 hold them
    float t = 0.f;
    for (int wv = 0; wv < 4; ++wv) t += sred[wv][0][LB + tid];
    lossp[(long long)blockIdx.x * 3 + tid] = t;
  }
}

// Second pass of the two-pass head backward (deferred BatchNorm of the last decoder
// block): recomputes dA exactly as head_ce_bwd_kernel stores it (head_pixel) and applies
// that BatchNorm's backward to it in registers,
//   dY = k * (dyh - m1 - xhat * m2),  dyh = dA * [y*scale + shift > 0]
// (coefs = [k | m1 | m2] x C from the stats pass's partial rows; the arithmetic of
// bn_bwd2_kernel's apply, same operand order) — dA never reaches HBM and the separate
// BN-apply pass (read dA + y, write dY) is gone: y + labels in, dY out.
// Two pixels per lane per iteration with all loads first (memory-level parallelism).
template <int C, int K>
__global__ __launch_bounds__(256) void head_bn_apply_kernel(
    const bf16_t* __restrict__ a, const float* __restrict__ Wh, const float* __restrict__ bh,
    const int64_t* __restrict__ labels, const float* __restrict__ gscale,
    const float* __restrict__ stats3, const float* __restrict__ bn4,
    const float* __restrict__ coefs, bf16_t* __restrict__ dY, long long P, int ignore_index,
    int Kreal) {
  constexpr int G = C / 8;
  constexpr int PPB = 256 / G;
  constexpr int U = 4;                               // pixels per lane in flight
  __shared__ __attribute__((aligned(16))) float sW[K * C];
  const int tid = threadIdx.x, lane = tid & 63;
  const int cg = lane % G, c8 = cg * 8;
  for (int i = tid; i < K * C; i += 256) sW[i] = i < Kreal * C ? Wh[i] : 0.f;
  float bk[K], sc[8], sh[8], is[8], nm[8], k1[8], m1[8], m2[8];
#pragma unroll
  for (int k = 0; k < K; ++k) bk[k] = k < Kreal ? bh[k] : -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = bn4[2 * C + c8 + j]; sh[j] = bn4[3 * C + c8 + j];
    is[j] = bn4[C + c8 + j]; nm[j] = -bn4[c8 + j] * is[j];
    k1[j] = coefs[c8 + j]; m1[j] = coefs[C + c8 + j]; m2[j] = coefs[2 * C + c8 + j];
  }
  __syncthreads();
  const float cnt = stats3[2];
  const float gs = (gscale != nullptr ? gscale[0] : 1.0f) / (cnt > 0.f ? cnt : 1.f);
  const long long stride = (long long)gridDim.x * PPB;
#pragma unroll 1
  for (long long px0 = (long long)blockIdx.x * PPB + tid / G; px0 < P; px0 += U * stride) {
    uint4 av[U];
    int64_t lab[U];
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const long long px = px0 + r * stride;
      const long long pq = px < P ? px : px0;
      av[r] = *reinterpret_cast<const uint4*>(a + pq * C + c8);
      lab[r] = labels[pq];
    }
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const long long px = px0 + r * stride;
      if (px >= P) break;                            // uniform over the G lanes of a pixel
      float y8[8], f[8], d[K];
      uint4 pk;
      head_pixel<C, K, true>(av[r], lab[r], sW + opaque_zero() + c8, bk, sc, sh, gs,
                             ignore_index, y8, f, d, pk);
      float rr[8], o[8];
      unpack8(pk, rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float av2 = fmaf(y8[j], sc[j], sh[j]);
        const float dyh = av2 > 0.f ? rr[j] : 0.f;
        const float xh = fmaf(y8[j], is[j], nm[j]);
        o[j] = k1[j] * (dyh - m1[j] - xh * m2[j]);
      }
      *reinterpret_cast<uint4*>(dY + px * C + c8) = pack8(o);
    }
  }
}

// ===================================================================== the C = 32 head on MFMA
// The flagship head (32 input channels, up to 16 classes) with the per-pixel arithmetic on the
// matrix cores.  A wave works on 16 pixels at a time; lane l holds pixel n = l & 15 and
// channel group g = l >> 4 (channels 8g..8g+7: one 16-B load, the same bytes the channel-split
// kernels read), which is exactly the B operand of v_mfma_f32_16x16x32_bf16:
//   logits^T [16 classes][16 px] = Wh [16][32] . act^T        (Wh as bf16 hi + lo: 2 MFMAs)
// and its output layout (lane: classes 4g..4g+3 of pixel n) is exactly the B operand of
// v_mfma_f32_16x16x16_bf16 for the head's input gradient:
//   dA^T [channels][16 px] = Wh^T . dlogits^T                  (hi/lo products: 3 MFMAs per
//                                                                 16-channel tile, 2 tiles)
// with the A rows permuted so the output lane again holds channels 8g..8g+7 of pixel n (the
// lane's own y for the BatchNorm-backward arithmetic and a 16-B store).  The softmax runs on
// the 4 class values per lane; its max / sum over a pixel's 4 lanes (rows of the wave) are
// two v_permlane{16,32}_swap steps.  The channel-split kernels (one lane per 8 channels of a
// pixel, 48 FMAs for the logits and 48 for dA per lane, the softmax repeated on the 4 lanes
// of a pixel) were VALU-issue bound at ~1.5-2.6 TB/s (profiles/r4/pmc_head_r6e.txt); here the
// VALU work per pixel is the BatchNorm transform, 4 exponentials and the stats.  Products are
// exact bf16 x bf16 (hi + lo splits of the fp32 weights and dlogits: ~2^-16 relative), sums fp32.
// dWh^T [class][ch] += dlogits^T . act uses the LDS-transposed operands of the former MDW kernel.

// sum / max of a value over the 4 rows of the wave (the 4 channel / class groups of a pixel):
// permlane16_swap pairs rows (0,1), (2,3); permlane32_swap pairs halves — every lane gets the
// same result, summed in the same order
DDLPC_DEVICE float rows4_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                            false, false);
  const float s = __builtin_bit_cast(float, (unsigned)a[0]) + __builtin_bit_cast(float, (unsigned)a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, s), __builtin_bit_cast(unsigned, s),
                                            false, false);
  return __builtin_bit_cast(float, (unsigned)b[0]) + __builtin_bit_cast(float, (unsigned)b[1]);
}
DDLPC_DEVICE float rows4_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                            false, false);
  const float s = fmaxf(__builtin_bit_cast(float, (unsigned)a[0]), __builtin_bit_cast(float, (unsigned)a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, s), __builtin_bit_cast(unsigned, s),
                                            false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)b[0]), __builtin_bit_cast(float, (unsigned)b[1]));
}
DDLPC_DEVICE int rows4_min_i(int v) {
  auto a = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  const int s = min((int)a[0], (int)a[1]);
  auto b = __builtin_amdgcn_permlane32_swap((unsigned)s, (unsigned)s, false, false);
  return min((int)b[0], (int)b[1]);
}

// the lane's constant MFMA operands: logits A = Wh[class n][8g..8g+7] (hi, lo), dA tiles
// A = Wh[4g..4g+3][ch(n, t)] with ch(m, t) = 8 (m >> 2) + 4 t + (m & 3) (hi, lo), and the
// logit bias of classes 4g..4g+3 (padded classes: zero weights, bias -inf)
struct Head32W { uint4 zh, zl; uint2 th[2], tl[2]; f32x4_t b4; };
DDLPC_DEVICE Head32W head32_weights(const float* __restrict__ Wh, const float* __restrict__ bh, int Kreal,
                                    int lane) {
  const int n = lane & 15, g = lane >> 4;
  Head32W w;
  float hi[8], lo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = n < Kreal ? Wh[n * 32 + 8 * g + j] : 0.f;
    hi[j] = lo_bf(pack2(v, 0.f));
    lo[j] = v - hi[j];
  }
  w.zh = pack8(hi);
  w.zl = pack8(lo);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ch = 8 * (n >> 2) + 4 * t + (n & 3);
    float h4[4], l4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 4 * g + i;
      const float v = k < Kreal ? Wh[k * 32 + ch] : 0.f;
      h4[i] = lo_bf(pack2(v, 0.f));
      l4[i] = v - h4[i];
    }
    w.th[t] = make_uint2(pack2(h4[0], h4[1]), pack2(h4[2], h4[3]));
    w.tl[t] = make_uint2(pack2(l4[0], l4[1]), pack2(l4[2], l4[3]));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) w.b4[i] = 4 * g + i < Kreal ? bh[4 * g + i] : -INFINITY;
  return w;
}

// one 16-pixel step of a wave: from the lane's 8 raw channels yv (pixel n, channels 8g..),
// its label and validity -> the activation f (BN + ReLU when DEFER, bf16-rounded), the 4
// dlogits d (classes 4g..4g+3, scaled by gs; zero for ignored / tail pixels), dA before
// rounding (o8, the lane's 8 channels) and rounded (pk); LOSS extras: lse, the label's
// logit, the arg-max class (valid on every lane of the pixel)
template <bool DEFER, bool LOSS>
DDLPC_DEVICE void head32_step(const uint4 yv, const int lab, const bool valid, const Head32W* __restrict__ wl,
                              const float (&sc)[8], const float (&sh)[8], float gs, int ignore_index,
                              int g, float (&y8)[8], uint4& fb, float (&d)[4], uint2& bh2, uint2& bl2,
                              float (&o8)[8], uint4& pk, float& lse, float& zy, int& am) {
  unpack8(yv, y8);
  if (DEFER) {
    // the activation as materialised (bf16 of relu(y * scale + shift)), packed: two channels
    // per v_pk_fma_f32, one v_cvt_pk_bf16_f32, ReLU as a packed 16-bit max on the bf16 bits
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2_t r2 = __builtin_elementwise_fma(f32x2_t{y8[2 * j], y8[2 * j + 1]},
                                                   f32x2_t{sc[2 * j], sc[2 * j + 1]},
                                                   f32x2_t{sh[2 * j], sh[2 * j + 1]});
      const uint32_t pb = __builtin_bit_cast(uint32_t, __builtin_convertvector(r2, bf16x2_t));
      o[j] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2_t, pb),
                                                                    i16x2_t{0, 0}));
    }
    fb = make_uint4(o[0], o[1], o[2], o[3]);
  } else {
    fb = yv;
  }
  const uint4 fz = valid ? fb : make_uint4(0, 0, 0, 0);
  // (the lane's constant operands are read from LDS where they are used: held in VGPRs across
  // the step loop they cost 20 registers and a wave per SIMD of occupancy)
  f32x4_t z = mfma16x16x32(wl->zh, fz, wl->b4);
  z = mfma16x16x32(wl->zl, fz, z);
  float m = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
  m = rows4_max(m);
  float e[4], se = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) { e[i] = __expf(z[i] - m); se += e[i]; }
  se = rows4_sum(se);
  const float inv = __builtin_amdgcn_rcpf(se);     // (se >= 1: the max term is exp(0))
  const bool live = valid && lab != ignore_index;
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = live ? (e[i] * inv - (4 * g + i == lab ? 1.f : 0.f)) * gs : 0.f;
  if (LOSS) {
    lse = m + __logf(se);
    float t = 0.f;
    int c = 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      t = (4 * g + i == lab) ? z[i] : t;
      c = (z[i] == m && c == 16) ? 4 * g + i : c;   // first maximum
    }
    zy = rows4_sum(t);
    am = rows4_min_i(c);
  }
  // dA: hi / lo splits of the dlogits as the B operand (classes 4g..4g+3 of pixel n; also the
  // caller's dWh staging)
  {
    const uint32_t h01 = pack2(d[0], d[1]), h23 = pack2(d[2], d[3]);
    const float dl0 = d[0] - lo_bf(h01), dl1 = d[1] - hi_bf(h01);
    const float dl2 = d[2] - lo_bf(h23), dl3 = d[3] - hi_bf(h23);
    bh2 = make_uint2(h01, h23);
    bl2 = make_uint2(pack2(dl0, dl1), pack2(dl2, dl3));
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    f32x4_t o = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const uint2 th = wl->th[t], tl = wl->tl[t];
    o = mfma16x16x16(th, bh2, o);
    o = mfma16x16x16(th, bl2, o);
    o = mfma16x16x16(tl, bh2, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) o8[4 * t + i] = o[i];
  }
  pk = pack8(o8);
}

// Loads run HEAD32_D steps ahead (a wave's 1 KB activation tile + its 16 labels per step): the
// channel-split kernels and a first one-step-prefetch form of these were latency-bound at
// 1.9 TB/s (12 waves x 1.1 KB in flight per CU); the per-lane channel constants live in LDS
// (re-read per step; an opaque offset keeps the compiler from hoisting them into VGPRs) to pay
// for the deeper register pipeline.
constexpr int HEAD32_D = 3;             // head32_kernel (three steps ahead at four workgroups per CU, <= 128 VGPRs)
constexpr int HEAD32_DA = 4;            // head32_apply_kernel

template <int D>
struct Head32Ld {
  uint4 y[D];
  int l[D];                             // (the low word of the int64 label: ids and -100 fit)
};

// The C = 32 counterpart of head_ce_bwd_kernel<32, K, DEFER, STORE, LOSS> (same outputs, same
// row layouts): stats of the backward (dWh, dbh; with DEFER the deferred BatchNorm's backward
// partials), the dA store (STORE), and with LOSS the training forward's loss / hits / count at
// a unit gradient scale.
template <bool DEFER, bool STORE, bool LOSS>
__global__ __launch_bounds__(256, 4) void head32_kernel(
    const bf16_t* __restrict__ a, const float* __restrict__ Wh, const float* __restrict__ bh,
    const int64_t* __restrict__ labels, const float* __restrict__ gscale,
    const float* __restrict__ stats3, bf16_t* __restrict__ dA, float* __restrict__ dWp,
    long long P, int ignore_index, const float* __restrict__ bn4, float* __restrict__ bnpart,
    int Kreal, float* __restrict__ lossp, int groups, long long gsteps) {
  static_assert(!LOSS || (DEFER && !STORE), "the fused forward is the deferred stats pass");
  constexpr int C = 32;
  // BN groups (a batched window, groups > 1): the deferred BatchNorm has per-group statistics
  // bn4 [groups][4][C]; the grid is groups x Rb workgroups and workgroup b walks only the
  // 16-pixel steps of group b / Rb (gsteps per group: a step never straddles two groups), so
  // its BN partial row belongs to that group (rows [groups][Rb][2][C])
  const int Rb = groups > 1 ? (int)gridDim.x / groups : (int)gridDim.x;
  const int grp = groups > 1 ? (int)blockIdx.x / Rb : 0;
  if (DEFER) bn4 += (long long)grp * 4 * C;
  // per wave: act [16][32] bf16 (1 KB) | dlogits hi [16][16] | lo [16][16]; reused at the end
  // as the wave's dWh^T [16][32] fp32 (2 KB)
  __shared__ __attribute__((aligned(16))) char sT[4][2048];
  __shared__ float sred[4][4][24];                 // [wave][row g][db 4 | bn 16 | loss 3]
  __shared__ __attribute__((aligned(16))) float sK[4][C];   // scale | shift | invstd | -mean*invstd
  __shared__ Head32W sW[64];                       // the lanes' constant MFMA operands
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // (uniform: scalar step indices)
  const int n = lane & 15, g = lane >> 4;
  if (tid < 64) sW[tid] = head32_weights(Wh, bh, Kreal, lane);
  if (DEFER && tid < C) {
    sK[0][tid] = bn4[2 * C + tid];
    sK[1][tid] = bn4[3 * C + tid];
    sK[2][tid] = bn4[C + tid];
    sK[3][tid] = -bn4[tid] * bn4[C + tid];
  }
  __syncthreads();
  const float cnt = LOSS ? 1.f : stats3[2];
  const float gs = LOSS ? 1.f : (gscale != nullptr ? gscale[0] : 1.0f) / (cnt > 0.f ? cnt : 1.f);
  char* tA = sT[wave];
  char* tDh = tA + 1024;
  char* tDl = tA + 1536;
  const int q = (lane & 15) >> 2, pq = lane & 3;
  const int rA = (4 * g + q) * 64 + pq * 8;          // transposed reads (see the MDW notes)
  const int rD = (4 * g + q) * 32 + pq * 8;
  f32x4_t dw[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  float db[4] = {0.f, 0.f, 0.f, 0.f}, b1[8], b2[8], ls[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) { b1[j] = 0.f; b2[j] = 0.f; }
  const long long steps = groups > 1 ? (long long)(grp + 1) * gsteps : (P + 15) / 16;   // (end step)
  const long long wstride = (long long)Rb * 4;
  const long long s0 = (long long)grp * gsteps + (long long)((int)blockIdx.x - grp * Rb) * 4 + wave;
  auto load = [&](long long st, uint4& yv, int& lb) __attribute__((always_inline)) {
    const long long px = st * 16 + n;
    const long long pc = px < P ? px : 0;
    yv = *reinterpret_cast<const uint4*>(a + pc * C + 8 * g);
    lb = reinterpret_cast<const int*>(labels)[2 * pc];
  };
  Head32Ld<HEAD32_D> q4;
#pragma unroll
  for (int j = 0; j < HEAD32_D; ++j) load(s0 + j * wstride < steps ? s0 + j * wstride : s0, q4.y[j], q4.l[j]);
#pragma unroll 1
  for (long long sb = s0; sb < steps; sb += HEAD32_D * wstride) {   // wave-uniform trip count
#pragma unroll
    for (int j = 0; j < HEAD32_D; ++j) {
      // branch-free steps (a step past the end is masked) whose slot is refilled only after
      // its last use (end of the step, clamped address): the loaded registers are then the
      // loop-carried ones.  With the load issued before the step and guarded by a branch, the
      // compiler rotated the slots with register copies at the loop back edge — each copy of
      // a register with a load in flight a vmcnt(0), i.e. the whole prefetch drained once per
      // HEAD32_D steps
      const long long s = sb + j * wstride;
      const uint4 yv = q4.y[j];
      const int lab = q4.l[j];
      const long long px = s * 16 + n;
      const bool valid = s < steps && px < P;
      float sc[8], sh[8];
      if (DEFER) {
        const float4* kp = reinterpret_cast<const float4*>(&sK[0][0] + opaque_zero() + 8 * g);
        const float4 a0 = kp[0], a1 = kp[1], c0 = kp[8], c1 = kp[9];
        sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
        sh[0] = c0.x; sh[1] = c0.y; sh[2] = c0.z; sh[3] = c0.w; sh[4] = c1.x; sh[5] = c1.y; sh[6] = c1.z; sh[7] = c1.w;
      } else {
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) { sc[jj] = 0.f; sh[jj] = 0.f; }
      }
      float y8[8], d[4], o8[8], lse = 0.f, zy = 0.f;
      int am = 0;
      uint4 pk, fb;
      uint2 bh2, bl2;
      head32_step<DEFER, LOSS>(yv, lab, valid, sW + opaque_zero() + lane, sc, sh, gs, ignore_index, g, y8, fb, d, bh2, bl2, o8, pk,
                               lse, zy, am);
      if (STORE && valid) *reinterpret_cast<uint4*>(dA + px * C + 8 * g) = pk;
      // dWh via the LDS transpose: act row (the lane's 8 channels; zero for tail pixels),
      // dlogits hi / lo (the lane's 4 classes; zero for tail pixels already)
      *reinterpret_cast<uint4*>(tA + n * 64 + g * 16) = valid ? fb : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint2*>(tDh + n * 32 + g * 8) = bh2;
      *reinterpret_cast<uint2*>(tDl + n * 32 + g * 8) = bl2;
      const uint2 ah = lds_read_tr16(tDh + rD);
      const uint2 al = lds_read_tr16(tDl + rD);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const uint2 b = lds_read_tr16(tA + rA + nt * 32);
        dw[nt] = mfma16x16x16(ah, b, dw[nt]);
        dw[nt] = mfma16x16x16(al, b, dw[nt]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) db[i] += d[i];
      if (LOSS) {                                    // (branch-free: row g = 0 counts a pixel)
        const bool cnt_px = g == 0 && valid;
        const bool lv = cnt_px && lab != ignore_index;
        ls[0] += lv ? lse - zy : 0.f;
        ls[2] += lv ? 1.f : 0.f;
        ls[1] += (cnt_px && am == lab) ? 1.f : 0.f;
      }
      if (DEFER) {
        float r[8];
        if (LOSS) {                                  // unit scale: the unrounded dA
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) r[jj] = o8[jj];
        } else {
          unpack8(pk, r);                            // BN backward sees the stored dA
        }
        const float4* kp = reinterpret_cast<const float4*>(&sK[2][0] + opaque_zero() + 8 * g);
        const float4 a0 = kp[0], a1 = kp[1], c0 = kp[8], c1 = kp[9];
        const float xi[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float xm[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        // (packed: two channels per v_pk_fma / v_pk_add; the ReLU mask compares the fp32
        // y * scale + shift like bn_bwd2_kernel)
#pragma unroll
        for (int jj = 0; jj < 8; jj += 2) {
          const f32x2_t y2 = {y8[jj], y8[jj + 1]};
          const f32x2_t a2 = __builtin_elementwise_fma(y2, f32x2_t{sc[jj], sc[jj + 1]},
                                                       f32x2_t{sh[jj], sh[jj + 1]});
          const f32x2_t x2 = __builtin_elementwise_fma(y2, f32x2_t{xi[jj], xi[jj + 1]},
                                                       f32x2_t{xm[jj], xm[jj + 1]});
          const f32x2_t d2 = {(valid && a2.x > 0.f) ? r[jj] : 0.f, (valid && a2.y > 0.f) ? r[jj + 1] : 0.f};
          f32x2_t s1 = {b1[jj], b1[jj + 1]}, s2 = {b2[jj], b2[jj + 1]};
          s1 += d2;
          s2 = __builtin_elementwise_fma(d2, x2, s2);
          b1[jj] = s1.x; b1[jj + 1] = s1.y; b2[jj] = s2.x; b2[jj + 1] = s2.y;
        }
      }
      const long long sl = s + HEAD32_D * wstride;
      load(sl < steps ? sl : s0, q4.y[j], q4.l[j]);
    }
  }
  // ---- workgroup reduction (fixed order): dWh^T of each wave to its LDS tile (lane: class
  // 4g + i, channel 16 nt + n), db / BN partials / loss summed over the 16 pixel lanes of
  // each row, then the 4 waves
  float* wd = reinterpret_cast<float*>(tA);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) wd[(4 * g + i) * 32 + nt * 16 + n] = dw[nt][i];
  float red[23];
#pragma unroll
  for (int i = 0; i < 4; ++i) red[i] = row16_sum(db[i]);
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[4 + j] = DEFER ? row16_sum(b1[j]) : 0.f; red[12 + j] = DEFER ? row16_sum(b2[j]) : 0.f; }
#pragma unroll
  for (int i = 0; i < 3; ++i) red[20 + i] = LOSS ? row16_sum(ls[i]) : 0.f;
  if (n == 0)
#pragma unroll
    for (int i = 0; i < 23; ++i) sred[wave][g][i] = red[i];
  __syncthreads();
  const int nout = Kreal * C + Kreal;
  for (int o = tid; o < nout; o += 256) {            // [dW (k, c) | db (k)]
    float t = 0.f;
    if (o < Kreal * C) {
      const int k = o / C, c = o % C;
      for (int wv = 0; wv < 4; ++wv) t += reinterpret_cast<const float*>(sT[wv])[k * 32 + c];
    } else {
      const int k = o - Kreal * C;
      for (int wv = 0; wv < 4; ++wv) t += sred[wv][k >> 2][k & 3];
    }
    dWp[(long long)blockIdx.x * nout + o] = t;
  }
  if (DEFER)
    for (int o = tid; o < 2 * C; o += 256) {         // [sum dyh (c) | sum dyh * xhat (c)]
      const int half = o / C, c = o % C;
      float t = 0.f;
      for (int wv = 0; wv < 4; ++wv) t += sred[wv][c >> 3][4 + 8 * half + (c & 7)];
      bnpart[(long long)blockIdx.x * 2 * C + o] = t;
    }
  if (LOSS && tid < 3) {                             // row g = 0 holds them
    float t = 0.f;
    for (int wv = 0; wv < 4; ++wv) t += sred[wv][0][20 + tid];
    lossp[(long long)blockIdx.x * 3 + tid] = t;
  }
}

// The C = 32 counterpart of head_bn_apply_kernel: dA recomputed exactly as head32_kernel
// stores it, the deferred BatchNorm's backward applied in registers (bn_bwd2_kernel's apply
// arithmetic), dY stored.  A HEAD32_DA-deep load pipeline.
__global__ __launch_bounds__(256, 4) void head32_apply_kernel(
    const bf16_t* __restrict__ a, const float* __restrict__ Wh, const float* __restrict__ bh,
    const int64_t* __restrict__ labels, const float* __restrict__ gscale,
    const float* __restrict__ stats3, const float* __restrict__ bn4,
    const float* __restrict__ coefs, bf16_t* __restrict__ dY, long long P, int ignore_index,
    int Kreal, int groups, long long gsteps) {
  constexpr int C = 32;
  // scale | shift | invstd | -mean*invstd | k | m1 | m2 (the BN backward coefficients)
  __shared__ __attribute__((aligned(16))) float sK[7][C];
  __shared__ Head32W sW[64];                       // the lanes' constant MFMA operands
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // (uniform: scalar step indices)
  const int n = lane & 15, g = lane >> 4;
  // BN groups: group-major workgroups as head32_kernel (bn4 [groups][4][C], coefs [groups][3][C])
  const int Rb = groups > 1 ? (int)gridDim.x / groups : (int)gridDim.x;
  const int grp = groups > 1 ? (int)blockIdx.x / Rb : 0;
  bn4 += (long long)grp * 4 * C;
  coefs += (long long)grp * 3 * C;
  if (tid < 64) sW[tid] = head32_weights(Wh, bh, Kreal, lane);
  if (tid < C) {
    sK[0][tid] = bn4[2 * C + tid]; sK[1][tid] = bn4[3 * C + tid];
    sK[2][tid] = bn4[C + tid]; sK[3][tid] = -bn4[tid] * bn4[C + tid];
    sK[4][tid] = coefs[tid]; sK[5][tid] = coefs[C + tid]; sK[6][tid] = coefs[2 * C + tid];
  }
  __syncthreads();
  const float cnt = stats3[2];
  const float gs = (gscale != nullptr ? gscale[0] : 1.0f) / (cnt > 0.f ? cnt : 1.f);
  const long long steps = groups > 1 ? (long long)(grp + 1) * gsteps : (P + 15) / 16;   // (end step)
  const long long wstride = (long long)Rb * 4;
  const long long s0 = (long long)grp * gsteps + (long long)((int)blockIdx.x - grp * Rb) * 4 + wave;
  auto load = [&](long long st, uint4& yv, int& lb) __attribute__((always_inline)) {
    const long long px = st * 16 + n;
    const long long pc = px < P ? px : 0;
    yv = *reinterpret_cast<const uint4*>(a + pc * C + 8 * g);
    lb = reinterpret_cast<const int*>(labels)[2 * pc];
  };
  auto k8 = [&](int r, float (&v)[8]) __attribute__((always_inline)) {
    const float4* kp = reinterpret_cast<const float4*>(&sK[r][0] + opaque_zero() + 8 * g);
    const float4 a0 = kp[0], a1 = kp[1];
    v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
  };
  Head32Ld<HEAD32_DA> q4;
#pragma unroll
  for (int j = 0; j < HEAD32_DA; ++j) load(s0 + j * wstride < steps ? s0 + j * wstride : s0, q4.y[j], q4.l[j]);
#pragma unroll 1
  for (long long sb = s0; sb < steps; sb += HEAD32_DA * wstride) {
#pragma unroll
    for (int j = 0; j < HEAD32_DA; ++j) {
      // (branch-free, slot refilled after its last use: see head32_kernel)
      const long long s = sb + j * wstride;
      const uint4 yv = q4.y[j];
      const int lab = q4.l[j];
      const long long px = s * 16 + n;
      const bool valid = s < steps && px < P;
      float sc[8], sh[8];
      k8(0, sc);
      k8(1, sh);
      float y8[8], d[4], o8[8], lse, zy;
      int am;
      uint4 pk, fb;
      uint2 bh2, bl2;
      head32_step<true, false>(yv, lab, valid, sW + opaque_zero() + lane, sc, sh, gs, ignore_index, g, y8, fb, d, bh2, bl2, o8, pk,
                               lse, zy, am);
      float rr[8], o[8], is[8], nm[8], k1[8], m1[8], m2[8];
      unpack8(pk, rr);
      k8(2, is); k8(3, nm); k8(4, k1); k8(5, m1); k8(6, m2);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const float av2 = fmaf(y8[jj], sc[jj], sh[jj]);
        const float dyh = av2 > 0.f ? rr[jj] : 0.f;
        const float xh = fmaf(y8[jj], is[jj], nm[jj]);
        o[jj] = k1[jj] * (dyh - m1[jj] - xh * m2[jj]);
      }
      if (valid) *reinterpret_cast<uint4*>(dY + px * C + 8 * g) = pack8(o);
      const long long sl = s + HEAD32_DA * wstride;
      load(sl < steps ? sl : s0, q4.y[j], q4.l[j]);
    }
  }
}

template <int C, int K, bool DEFER>
__global__ __launch_bounds__(256) void head_logits_kernel(const bf16_t* __restrict__ a, const float* __restrict__ Wh,
                                   const float* __restrict__ bh, float* __restrict__ out,
                                   long long P, long long HW, const float* __restrict__ bn4,
                                   int Kreal) {
  __shared__ __attribute__((aligned(16))) float sBNm[4 * C];
  __shared__ float sW[K * C], sb[K];
  load_head<C, K>(Wh, bh, Kreal, sW, sb);
  const float* sBN = DEFER ? load_bn<C>(bn4, sBNm, false) : nullptr;
  __syncthreads();
#pragma unroll 1
  for (long long px = blockIdx.x * (long long)blockDim.x + threadIdx.x; px < P;
       px += (long long)gridDim.x * blockDim.x) {
    float z[K];
    logits_of<C, K, DEFER>(a + px * C, sW, sb, sBN, z);
    const long long n = px / HW, s = px % HW;
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < Kreal) out[(n * Kreal + k) * HW + s] = z[k];
  }
}

// C in {8, 16, 32, 64} (64 / width_divisor channels) x padded class slots KP >= K
#define HEAD_SWITCH_K(C_, K_, ...)                                                  \
  if (K_ <= 2) { constexpr int KK = 2; __VA_ARGS__; }                               \
  else if (K_ <= 4) { constexpr int KK = 4; __VA_ARGS__; }                          \
  else if (K_ == 6) { constexpr int KK = 6; __VA_ARGS__; }                          \
  else if (K_ <= 8) { constexpr int KK = 8; __VA_ARGS__; }                          \
  else { constexpr int KK = 16; __VA_ARGS__; }
#define HEAD_SWITCH(C_, K_, ...)                                                    \
  [&] {                                                                             \
    if ((K_) < 1 || (K_) > MAXK) return false;                                      \
    if (C_ == 8) { constexpr int CC = 8; HEAD_SWITCH_K(C_, K_, __VA_ARGS__) }         \
    else if (C_ == 16) { constexpr int CC = 16; HEAD_SWITCH_K(C_, K_, __VA_ARGS__) }  \
    else if (C_ == 32) { constexpr int CC = 32; HEAD_SWITCH_K(C_, K_, __VA_ARGS__) }  \
    else if (C_ == 64) { constexpr int CC = 64; HEAD_SWITCH_K(C_, K_, __VA_ARGS__) }  \
    else { return false; }                                                          \
    return true;                                                                    \
  }()

}  // namespace

bool head_supported(int C, int K) {
  return HEAD_SWITCH(C, K, (void)0);
}

void head_ce_fwd_launch(const bf16_t* a, const float* Wh, const float* bh, const int64_t* labels,
                        float* partial, float* out3, const float* bn4, int nblocks, long long P,
                        int C, int K, int ignore_index, hipStream_t st) {
  if (bn4 != nullptr)
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_ce_fwd_kernel<CC, KK, true>), dim3(nblocks), dim3(256), 0,
                                         st, a, Wh, bh, labels, partial, P, ignore_index, bn4, K));
  else
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_ce_fwd_kernel<CC, KK, false>), dim3(nblocks), dim3(256), 0,
                                         st, a, Wh, bh, labels, partial, P, ignore_index, bn4, K));
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(256), 0, st, partial, nblocks, out3);
}

// persistent grid of the channel-split backward: every workgroup resident at once (the
// occupancy of the instantiation, from the HIP occupancy API), capped by the pixel count
// (the SAME grid with and without the deferred BatchNorm — the smaller occupancy of the two
// — so both paths reduce dWh in the same order: bit-identical weight gradients)
namespace {
// resident workgroups per CU of a head32 kernel (occupancy API)
int head32_per_cu(const void* fn) {
  int n = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 256, 0) == hipSuccess && n > 0 ? n : 1;
}
int head32_grid(long long P, int per_cu, int num_cus) {
  const long long steps4 = ((P + 15) / 16 + 3) / 4;        // 4 waves x 16 pixels per workgroup step
  return (int)std::max<long long>(1, std::min<long long>(steps4, (long long)per_cu * num_cus));
}
int head32_bwd_per_cu() {
  static int n = std::min({head32_per_cu(reinterpret_cast<const void*>(&head32_kernel<true, true, false>)),
                           head32_per_cu(reinterpret_cast<const void*>(&head32_kernel<true, false, false>)),
                           head32_per_cu(reinterpret_cast<const void*>(&head32_kernel<false, true, false>))});
  return n;
}
}  // namespace

int head_ce_bwd_blocks(int C, int K, bool /*defer*/, long long P, int num_cus) {
  // C = 32: the MFMA kernels — the same grid for every variant, so the deferred / plain /
  // stats-only paths reduce dWh in the same order (bit-identical weight gradients)
  if (C == 32) return head32_grid(P, head32_bwd_per_cu(), num_cus);
  int per_cu = 8;
  auto occ = [&](const void* fn) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 256, 0) == hipSuccess && n > 0)
      per_cu = std::min(per_cu, n);
    else
      per_cu = std::min(per_cu, 1);
  };
  HEAD_SWITCH(C, K, occ(reinterpret_cast<const void*>(&head_ce_bwd_kernel<CC, KK, true>)));
  HEAD_SWITCH(C, K, occ(reinterpret_cast<const void*>(&head_ce_bwd_kernel<CC, KK, false>)));
  // (the resident workgroups per CU: 4 / 6 / 8 / 12 measured 3-4% slower, docs/PERF.md)
  const long long ppb = 256 / (C / 8);
  return (int)std::max<long long>(1, std::min<long long>((P + ppb - 1) / ppb, (long long)per_cu * num_cus));
}

void head_ce_bwd_launch(const bf16_t* a, const float* Wh, const float* bh, const int64_t* labels,
                        const float* gscale, const float* stats3, int /*unused*/, bf16_t* dA,
                        float* dW_partial, int nblocks, long long P, int C, int K,
                        int ignore_index, const float* bn4, float* bnpart, hipStream_t st) {
  if (C == 32 && K <= MAXK) {
    if (bn4 != nullptr && dA == nullptr)
      hipLaunchKernelGGL((head32_kernel<true, false, false>), dim3(nblocks), dim3(256), 0, st, a, Wh, bh,
                         labels, gscale, stats3, dA, dW_partial, P, ignore_index, bn4, bnpart, K, nullptr, 1, 0LL);
    else if (bn4 != nullptr)
      hipLaunchKernelGGL((head32_kernel<true, true, false>), dim3(nblocks), dim3(256), 0, st, a, Wh, bh,
                         labels, gscale, stats3, dA, dW_partial, P, ignore_index, bn4, bnpart, K, nullptr, 1, 0LL);
    else
      hipLaunchKernelGGL((head32_kernel<false, true, false>), dim3(nblocks), dim3(256), 0, st, a, Wh, bh,
                         labels, gscale, stats3, dA, dW_partial, P, ignore_index, bn4, bnpart, K, nullptr, 1, 0LL);
    return;
  }
  if (bn4 != nullptr && dA == nullptr)               // stats pass of the two-pass backward
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_ce_bwd_kernel<CC, KK, true, false>), dim3(nblocks), dim3(256), 0,
                                         st, a, Wh, bh, labels, gscale, stats3, dA, dW_partial, P,
                                         ignore_index, bn4, bnpart, K));
  else if (bn4 != nullptr)
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_ce_bwd_kernel<CC, KK, true>), dim3(nblocks), dim3(256), 0,
                                         st, a, Wh, bh, labels, gscale, stats3, dA, dW_partial, P,
                                         ignore_index, bn4, bnpart, K));
  else
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_ce_bwd_kernel<CC, KK, false>), dim3(nblocks), dim3(256), 0,
                                         st, a, Wh, bh, labels, gscale, stats3, dA, dW_partial, P,
                                         ignore_index, bn4, bnpart, K));
}

// the fused forward + statistics pass on the matrix-core dWh kernel (C = 32; other shapes: the
// register-accumulator kernel)
// (K <= 6: the 8- and 16-class instantiations exceed the 168-VGPR budget of three
// workgroups per CU and spill)
bool head_mdw(int C, int K) { return C == 32 && K <= 6; }

int head_fwd_stats_blocks(int C, int K, long long P, int num_cus, int groups) {
  if (C == 32 && K <= MAXK) {
    static const int n = head32_per_cu(reinterpret_cast<const void*>(&head32_kernel<true, false, true>));
    const int nb = head32_grid(P, n, num_cus);
    return groups > 1 ? groups * std::max(1, nb / groups) : nb;   // (groups x Rb, group-major)
  }
  if (!head_mdw(C, K)) return head_ce_bwd_blocks(C, K, true, P, num_cus);
  int per_cu = 8;
  HEAD_SWITCH(C, K, if constexpr (KK <= 6) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&head_fwd_stats_mdw_kernel<KK>),
                                                     256, 0) == hipSuccess && n > 0)
      per_cu = std::min(per_cu, n);
    else
      per_cu = 1;
  });
  const long long ppb = 64;
  return (int)std::max<long long>(1, std::min<long long>((P + ppb - 1) / ppb, (long long)per_cu * num_cus));
}

void head_ce_fwd_stats_launch(const bf16_t* a, const float* Wh, const float* bh,
                              const int64_t* labels, const float* bn4, float* dW_partial,
                              float* bnpart, float* loss_partial, float* out3, int nblocks,
                              long long P, int C, int K, int ignore_index, hipStream_t st, int groups) {
  if (C == 32 && K <= MAXK)
    hipLaunchKernelGGL((head32_kernel<true, false, true>), dim3(nblocks), dim3(256), 0, st, a, Wh, bh, labels,
                       nullptr, nullptr, nullptr, dW_partial, P, ignore_index, bn4, bnpart, K, loss_partial,
                       groups, groups > 1 ? P / groups / 16 : 0LL);
  else if (head_mdw(C, K))
    HEAD_SWITCH(C, K, if constexpr (KK <= 6) {
      hipLaunchKernelGGL((head_fwd_stats_mdw_kernel<KK>), dim3(nblocks), dim3(256), 0, st, a, Wh, bh, labels,
                         dW_partial, P, ignore_index, bn4, bnpart, K, loss_partial);
    });
  else
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_ce_bwd_kernel<CC, KK, true, false, true>), dim3(nblocks),
                                         dim3(256), 0, st, a, Wh, bh, labels, nullptr, nullptr, nullptr,
                                         dW_partial, P, ignore_index, bn4, bnpart, K, loss_partial));
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(256), 0, st, loss_partial, nblocks, out3);
}

int head_bn_apply_blocks(long long P, int C) {
  const long long ppb = 256 / (C / 8);
  const int cap = 4096;
  return (int)std::max<long long>(1, std::min<long long>((P + 2 * ppb - 1) / (2 * ppb), cap));
}

void head_bn_apply_launch(const bf16_t* a, const float* Wh, const float* bh, const int64_t* labels,
                          const float* gscale, const float* stats3, const float* bn4,
                          const float* coefs, bf16_t* dY, long long P, int C, int K,
                          int ignore_index, hipStream_t st, int groups) {
  if (C == 32 && K <= MAXK) {
    static const int per_cu = head32_per_cu(reinterpret_cast<const void*>(&head32_apply_kernel));
    static const int cus = [] {
      hipDeviceProp_t prop;
      int dev = 0;
      hipGetDevice(&dev);
      return hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    }();
    const int nb = head32_grid(P, per_cu, cus);
    const int grid = groups > 1 ? groups * std::max(1, nb / groups) : nb;
    hipLaunchKernelGGL(head32_apply_kernel, dim3(grid), dim3(256), 0, st, a, Wh, bh,
                       labels, gscale, stats3, bn4, coefs, dY, P, ignore_index, K, groups,
                       groups > 1 ? P / groups / 16 : 0LL);
    return;
  }
  const int nb = head_bn_apply_blocks(P, C);
  HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_bn_apply_kernel<CC, KK>), dim3(nb), dim3(256), 0, st,
                                       a, Wh, bh, labels, gscale, stats3, bn4, coefs, dY, P,
                                       ignore_index, K));
}

void head_logits_launch(const bf16_t* a, const float* Wh, const float* bh, float* logits,
                        long long P, long long HW, int C, int K, const float* bn4, hipStream_t st) {
  const int grid = (int)std::min<long long>((P + 255) / 256, 4096);
  if (bn4 != nullptr)
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_logits_kernel<CC, KK, true>), dim3(grid), dim3(256), 0, st,
                                         a, Wh, bh, logits, P, HW, bn4, K));
  else
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_logits_kernel<CC, KK, false>), dim3(grid), dim3(256), 0, st,
                                         a, Wh, bh, logits, P, HW, bn4, K));
}

}  // namespace ddlpc
