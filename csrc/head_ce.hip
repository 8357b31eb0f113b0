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

// bn4 != null: deferred BatchNorm of the last decoder block (see act8).  (Its backward
// partial sums are NOT reduced here: 2*C per-thread accumulators cost the kernel its
// occupancy — measured slower than the separate reduction pass.)
template <int C, int K, bool DEFER>
__global__ __launch_bounds__(256) void head_ce_bwd_kernel(
    const bf16_t* __restrict__ a, const float* __restrict__ Wh, const float* __restrict__ bh,
    const int64_t* __restrict__ labels, const float* __restrict__ gscale,
    const float* __restrict__ stats3, bf16_t* __restrict__ dA, float* __restrict__ dWp,
    long long P, int ignore_index, const float* __restrict__ bn4, int Kreal) {
  __shared__ __attribute__((aligned(16))) float sBNm[4 * C];
  __shared__ float sW[K * C], sb[K];
  __shared__ __attribute__((aligned(16))) bf16_t sA[256 * C];
  __shared__ float sD[256 * K];
  load_head<C, K>(Wh, bh, Kreal, sW, sb);
  const float* sBN = DEFER ? load_bn<C>(bn4, sBNm, false) : nullptr;
  __syncthreads();
  const float cnt = stats3[2];
  const float gs = (gscale != nullptr ? gscale[0] : 1.0f) / (cnt > 0.f ? cnt : 1.f);
  const int t = threadIdx.x;
  // per-block partial row [dW (Kreal*C) | db (Kreal)]: output o = t + 256*r of thread t
  constexpr int NO = (K * C + K + 255) / 256;
  const int nout = Kreal * C + Kreal;
  float accw[NO];
#pragma unroll
  for (int r = 0; r < NO; ++r) accw[r] = 0.f;
  const long long nper = (long long)gridDim.x * blockDim.x;
#pragma unroll 1
  for (long long base = blockIdx.x * (long long)blockDim.x; base < P; base += nper) {
    const long long px = base + t;
    float d[K];
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = 0.f;
    if (px < P) {
      float z[K];
      logits_of<C, K, DEFER>(a + px * C, sW, sb, sBN, z, sA + t * C);
      const int64_t y = labels[px];
      float m = z[0];
#pragma unroll
      for (int k = 1; k < K; ++k) m = fmaxf(m, z[k]);
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) { z[k] = __expf(z[k] - m); se += z[k]; }
      const float inv = 1.f / se;
      if (y != ignore_index) {
#pragma unroll
        for (int k = 0; k < K; ++k) d[k] = (z[k] * inv - (k == y ? 1.f : 0.f)) * gs;
      }
    } else {
#pragma unroll
      for (int c8 = 0; c8 < C; c8 += 8) *reinterpret_cast<uint4*>(sA + t * C + c8) = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) sD[t * K + k] = d[k];
    if (px < P) {
      // dA = d . Wh, one class row at a time (k loop kept rolled: C accumulators live, the
      // weights stream from LDS as broadcast reads instead of K*C hoisted registers)
      float o[C];
#pragma unroll
      for (int c = 0; c < C; ++c) o[c] = 0.f;
#pragma unroll 1
      for (int k = 0; k < Kreal; ++k) {
        const float dk = sD[t * K + k];
        const float* wr = sW + k * C;
#pragma unroll
        for (int c = 0; c < C; ++c) o[c] = fmaf(dk, wr[c], o[c]);
      }
#pragma unroll
      for (int c8 = 0; c8 < C; c8 += 8) {
        float q[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = o[c8 + j];
        *reinterpret_cast<uint4*>(dA + px * C + c8) = pack8(q);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NO; ++r) {
      const int o = t + 256 * r;
      if (o < Kreal * C) {
        const int k = o / C, c = o % C;
        float s = 0.f;
#pragma unroll 8
        for (int i = 0; i < 256; ++i) s = fmaf(bf2f(sA[i * C + c]), sD[i * K + k], s);
        accw[r] += s;
      } else if (o < nout) {
        const int k = o - Kreal * C;
        float s = 0.f;
#pragma unroll 8
        for (int i = 0; i < 256; ++i) s += sD[i * K + k];
        accw[r] += s;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < NO; ++r) {
    const int o = t + 256 * r;
    if (o < nout) dWp[(long long)blockIdx.x * nout + o] = accw[r];
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

void head_ce_bwd_launch(const bf16_t* a, const float* Wh, const float* bh, const int64_t* labels,
                        const float* gscale, const float* stats3, int /*unused*/, bf16_t* dA,
                        float* dW_partial, int nblocks, long long P, int C, int K,
                        int ignore_index, const float* bn4, float* /*bnpart: unused*/,
                        hipStream_t st) {
  if (bn4 != nullptr)
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_ce_bwd_kernel<CC, KK, true>), dim3(nblocks), dim3(256), 0,
                                         st, a, Wh, bh, labels, gscale, stats3, dA, dW_partial, P,
                                         ignore_index, bn4, K));
  else
    HEAD_SWITCH(C, K, hipLaunchKernelGGL((head_ce_bwd_kernel<CC, KK, false>), dim3(nblocks), dim3(256), 0,
                                         st, a, Wh, bh, labels, gscale, stats3, dA, dW_partial, P,
                                         ignore_index, bn4, K));
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
