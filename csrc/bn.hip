// Training-mode BatchNorm + ReLU (+ 2x max-pool) — K4-K7 of SURVEY.md §2.5.
// Reference: nn.BatchNorm2d -> nn.ReLU(inplace=True) inside DoubleConv (ref.py:580-584) and
// nn.MaxPool2d(2) in DownBlock (ref.py:595,599).
//
// Forward data flow (per conv):  conv epilogue writes y (bf16, pre-BN) + per-tile channel
// (sum, sum^2)  ->  bn_finalize (fp64 reduction: mean, invstd, scale = gamma*invstd,
// shift = beta - mean*scale, running stats with momentum 0.1 and the unbiased variance)
// ->  consumers apply relu(y*scale + shift) on the fly (next conv prologue) or
// bn_relu_apply materialises it once, writing the 2x2(x2) max-pooled tensor in the same
// pass for encoder blocks.
//
// Backward:  bn_bwd_reduce recomputes a = relu(y*scale+shift) and the pool arg-max from y,
// forms dyhat = (dA + unpool(dP)) * [a > 0] (times the loss-gradient scale), and reduces
// per-channel sum(dyhat), sum(dyhat*xhat); bn_bwd_finalize turns them into dgamma, dbeta
// and the three coefficients of dY = gamma*invstd*(dyhat - mean(dyhat) - xhat*mean(dyhat*xhat));
// bn_bwd_apply writes dY (bf16) for the conv's data/weight gradients.  The pool backward
// and the skip-gradient sum are folded into both passes (no unpooled tensor is stored).
#include "common.h"
#include "ops.h"

namespace ddlpc {

namespace {

// --------------------------------------------------------------------- apply (+ pool)
template <int DIMS, bool POOL>
__global__ void bn_relu_apply_kernel(const bf16_t* __restrict__ y, const float* __restrict__ scale,
                                     const float* __restrict__ shift, bf16_t* __restrict__ out,
                                     bf16_t* __restrict__ pooled, int N, int D, int H, int W,
                                     int C, long long sstride) {
  const int G = C / 8;
  // per-micro-batch BatchNorm groups (bn_group_apply): blockIdx.y = group, N = its images
  // and the group's (scale, shift) rows sstride floats apart; one group: blockIdx.y = 0
  {
    const long long gpix = (long long)N * D * H * W;
    const int grp = blockIdx.y;
    y += grp * gpix * C;
    if (out != nullptr) out += grp * gpix * C;
    if (POOL) pooled += grp * (gpix / (DIMS == 3 ? 8 : 4)) * C;
    scale += grp * sstride;
    shift += grp * sstride;
  }
  if (!POOL) {
    const long long total = (long long)N * D * H * W * G;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
      const int c8 = (int)(e % G) * 8;
      float f[8];
      unpack8(reinterpret_cast<const uint4*>(y)[e], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], scale[c8 + j], shift[c8 + j]), 0.f);
      reinterpret_cast<uint4*>(out)[e] = pack8(f);
    }
    return;
  }
  const int Do = DIMS == 3 ? D / 2 : 1, Ho = H / 2, Wo = W / 2;
  const long long total = (long long)N * Do * Ho * Wo * G;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(e % G);
    long long q = e / G;
    const int wo = (int)(q % Wo); q /= Wo;
    const int ho = (int)(q % Ho); q /= Ho;
    const int dd = DIMS == 3 ? (int)(q % Do) : 0;
    const int n = (int)(DIMS == 3 ? q / Do : q);
    const int c8 = cg * 8;
    float sc[8], sh[8], mx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = scale[c8 + j]; sh[j] = shift[c8 + j]; mx[j] = -INFINITY; }
#pragma unroll
    for (int kd = 0; kd < (DIMS == 3 ? 2 : 1); ++kd)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int kw = 0; kw < 2; ++kw) {
          const int d = DIMS == 3 ? 2 * dd + kd : 0;
          const long long pix = ((long long)(n * D + d) * H + 2 * ho + kh) * W + 2 * wo + kw;
          float f[8];
          unpack8(*reinterpret_cast<const uint4*>(y + pix * C + c8), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
          }
          const uint4 v = pack8(f);
          if (out != nullptr) *reinterpret_cast<uint4*>(out + pix * C + c8) = v;
          float r[8];
          unpack8(v, r);                       // pool the bf16-rounded activations
#pragma unroll
          for (int j = 0; j < 8; ++j) mx[j] = fmaxf(mx[j], r[j]);
        }
    const long long opix = ((long long)(n * Do + dd) * Ho + ho) * Wo + wo;
    *reinterpret_cast<uint4*>(pooled + opix * C + c8) = pack8(mx);
  }
}

// Apply + pool, v2 (bn_bwd2_kernel's mapping): unit = 2x2 (3-D: 2x2x2) window; lanes (kw, cg)
// cover the window's top-row pixel pair contiguously (2 x C channels), each lane also handles
// the pixels below it (kh) and, in 3-D, in the next slice (kd); the window maximum is
// completed with the kw partner lane (lane ^ G), whose kw = 0 lane stores the pooled value.
// 32-bit unit geometry (no 64-bit division per element) and UNROLL units' loads in flight
// per thread.  Requires G = C/8 a power of two <= 32 and even D, H, W.
template <int DIMS>
__global__ __launch_bounds__(256) void bn_relu_pool2_kernel(
    const bf16_t* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    bf16_t* __restrict__ out, bf16_t* __restrict__ pooled, int N, int H, int W, int C, long long sstride) {
  constexpr int UNROLL = 2;
  constexpr int NK = DIMS == 3 ? 4 : 2;            // pixels per lane per unit (k = 2*kd + kh)
  const int G = C / 8;
  {
    const int grp = blockIdx.y;                    // per-micro-batch BN groups (N = slices per group)
    const long long gel = (long long)N * H * W * C;
    y += grp * gel;
    if (out != nullptr) out += grp * gel;
    pooled += grp * (gel / (DIMS == 3 ? 8 : 4));
    scale += grp * sstride;
    shift += grp * sstride;
  }
  const int L = 2 * G;
  const int tid = threadIdx.x;
  const int cg = tid % G, c8 = cg * 8, kw = (tid / G) & 1;
  const int upb = 256 / L;
  const int Wo = W / 2, Ho = H / 2;
  const int units = (DIMS == 3 ? N / 2 : N) * Ho * Wo;   // N counts (n, d) slices
  const int stride = gridDim.x * upb;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = scale[c8 + j]; sh[j] = shift[c8 + j]; }
  for (int u0 = blockIdx.x * upb + tid / L; u0 < units; u0 += UNROLL * stride) {
    uint4 v[UNROLL][NK];
    long long off[UNROLL][NK];
    bool ok[UNROLL];
#pragma unroll
    for (int r = 0; r < UNROLL; ++r) {             // all loads first (memory-level parallelism)
      const int u = u0 + r * stride;
      ok[r] = u < units;
      const int uu = ok[r] ? u : u0;
      const int rr = uu / Wo, wo = uu - rr * Wo;
      long long pix0;
      if (DIMS == 3) {
        const int nd = rr / Ho, ho = rr - nd * Ho;
        pix0 = ((long long)(2 * nd) * H + 2 * ho) * W + 2 * wo + kw;
      } else {
        pix0 = (long long)rr * 2 * W + 2 * wo + kw;
      }
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        off[r][k] = (pix0 + (long long)(k >> 1) * H * W + (k & 1) * W) * C + c8;
        v[r][k] = *reinterpret_cast<const uint4*>(y + off[r][k]);
      }
    }
#pragma unroll
    for (int r = 0; r < UNROLL; ++r) {
      float mx[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) mx[j] = -INFINITY;
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        float f[8];
        unpack8(v[r][k], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
        const uint4 q = pack8(f);
        if (out != nullptr && ok[r]) *reinterpret_cast<uint4*>(out + off[r][k]) = q;
        float rq[8];
        unpack8(q, rq);                            // pool the bf16-rounded activations
#pragma unroll
        for (int j = 0; j < 8; ++j) mx[j] = fmaxf(mx[j], rq[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) mx[j] = fmaxf(mx[j], __shfl_xor(mx[j], G, 64));
      if (ok[r] && kw == 0) {
        const int u = u0 + r * stride;
        *reinterpret_cast<uint4*>(pooled + (long long)u * C + c8) = pack8(mx);
      }
    }
  }
}

// --------------------------------------------------------------------- backward passes
// Per work item: 8 channels of one pixel (no pool) or of one pooling window (pool).
// MODE 0: reduce (write per-block partial sums), MODE 1: apply (write dY).
template <int DIMS, bool POOL, int MODE>
__global__ void bn_bwd_kernel(const bf16_t* __restrict__ dA, const bf16_t* __restrict__ dP,
                              const bf16_t* __restrict__ y, const float* __restrict__ scale,
                              const float* __restrict__ shift, const float* __restrict__ mean,
                              const float* __restrict__ invstd, const float* __restrict__ coefs,
                              const float* __restrict__ gscale, float* __restrict__ partial,
                              bf16_t* __restrict__ dY, int N, int D, int H, int W, int C) {
  const int G = C / 8;
  const int per_block = (blockDim.x / G) * G;           // threads with a fixed channel group
  const int tid = threadIdx.x;
  const bool active = tid < per_block;
  const int cg = tid % G;
  const int c8 = cg * 8;
  const float gs = gscale != nullptr ? gscale[0] : 1.0f;
  float sc[8], sh[8], mu[8], is[8], k1[8], m1[8], m2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[c8 + j]; sh[j] = shift[c8 + j]; mu[j] = mean[c8 + j]; is[j] = invstd[c8 + j];
    if (MODE == 1) { k1[j] = coefs[c8 + j]; m1[j] = coefs[C + c8 + j]; m2[j] = coefs[2 * C + c8 + j]; }
  }
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }

  const int Do = POOL ? (DIMS == 3 ? D / 2 : 1) : D;
  const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
  const long long items = (long long)N * Do * Ho * Wo;
  const long long stride = (long long)gridDim.x * (per_block / G);
  if (active) {
    for (long long it = blockIdx.x * (long long)(per_block / G) + tid / G; it < items; it += stride) {
      if (!POOL) {
        const long long off = it * C + c8;
        float fy[8], fd[8];
        unpack8(*reinterpret_cast<const uint4*>(y + off), fy);
        unpack8(*reinterpret_cast<const uint4*>(dA + off), fd);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = fmaf(fy[j], sc[j], sh[j]);
          const float dyh = a > 0.f ? fd[j] * gs : 0.f;
          const float xh = (fy[j] - mu[j]) * is[j];
          if (MODE == 0) { s1[j] += dyh; s2[j] += dyh * xh; }
          else o[j] = k1[j] * (dyh - m1[j] - xh * m2[j]);
        }
        if (MODE == 1) *reinterpret_cast<uint4*>(dY + off) = pack8(o);
      } else {
        long long q = it;
        const int wo = (int)(q % Wo); q /= Wo;
        const int ho = (int)(q % Ho); q /= Ho;
        const int dd = DIMS == 3 ? (int)(q % Do) : 0;
        const int n = (int)(DIMS == 3 ? q / Do : q);
        constexpr int NW = DIMS == 3 ? 8 : 4;
        float fy[NW][8];
        long long offs[NW];
        int best[8];
        float bv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = 0; bv[j] = -INFINITY; }
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const int kd = DIMS == 3 ? (w >> 2) : 0, kh = (w >> 1) & 1, kw = w & 1;
          const int d = DIMS == 3 ? 2 * dd + kd : 0;
          offs[w] = (((long long)(n * D + d) * H + 2 * ho + kh) * W + 2 * wo + kw) * C + c8;
          unpack8(*reinterpret_cast<const uint4*>(y + offs[w]), fy[w]);
          // arg-max over the bf16-rounded activations, first maximum wins (PyTorch order)
          float a[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] = fmaxf(fmaf(fy[w][j], sc[j], sh[j]), 0.f);
          const uint4 av = pack8(a);
          float ar[8];
          unpack8(av, ar);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (ar[j] > bv[j]) { bv[j] = ar[j]; best[j] = w; }
        }
        const long long popix = ((long long)(n * Do + dd) * Ho + ho) * Wo + wo;
        float fp[8];
        unpack8(*reinterpret_cast<const uint4*>(dP + popix * C + c8), fp);
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          float fd[8], o[8];
          if (dA != nullptr) unpack8(*reinterpret_cast<const uint4*>(dA + offs[w]), fd);
          else {
#pragma unroll
            for (int j = 0; j < 8; ++j) fd[j] = 0.f;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float a = fmaf(fy[w][j], sc[j], sh[j]);
            const float dt = fd[j] + (best[j] == w ? fp[j] : 0.f);
            const float dyh = a > 0.f ? dt * gs : 0.f;
            const float xh = (fy[w][j] - mu[j]) * is[j];
            if (MODE == 0) { s1[j] += dyh; s2[j] += dyh * xh; }
            else o[j] = k1[j] * (dyh - m1[j] - xh * m2[j]);
          }
          if (MODE == 1) *reinterpret_cast<uint4*>(dY + offs[w]) = pack8(o);
        }
      }
    }
  }
  if (MODE == 0) {
    // block reduction: threads with equal cg hold the same channels
    __shared__ float red[256 * 8];
    for (int half = 0; half < 2; ++half) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 8; ++j) red[j * 256 + tid] = active ? (half ? s2[j] : s1[j]) : 0.f;
      __syncthreads();
      for (int c = tid; c < C; c += blockDim.x) {
        const int g2 = c / 8, j = c % 8;
        float t = 0.f;
        for (int k = g2; k < per_block; k += G) t += red[j * 256 + k];
        partial[(long long)blockIdx.x * 2 * C + half * C + c] = t;
      }
    }
  }
}

// Backward, v2: fully coalesced and unrolled.  A thread keeps one 8-channel group
// (constants in registers); consecutive lanes walk consecutive 16-B pieces of memory:
//   no pool: unit = pixel, lanes (cg) cover the pixel's C channels (3-D: N*D slices);
//   pool:    unit = 2x2 (3-D: 2x2x2) window, lanes (kw, cg) cover the window's top-row pixel
//            pair contiguously and each lane also handles the pixels below it (kh) and, in
//            3-D, in the next slice (kd); the window arg-max is completed with the kw
//            partner lane (lane ^ G) — first maximum wins in PyTorch's (kd, kh, kw) scan
//            order.
//   pool, KWIN (G > 32: the kw partner would sit in another wave): unit = window, lanes (cg)
//            cover one pixel's channels and each lane handles both kw pixels of its rows
//            itself (no cross-lane exchange).
// Requires G = C/8 a power of two <= 256 and even D, H, W for pool.
template <int DIMS, bool POOL, int MODE, bool KWIN = false>
__global__ __launch_bounds__(256) void bn_bwd2_kernel(
    const bf16_t* __restrict__ dA, const bf16_t* __restrict__ dP, const bf16_t* __restrict__ y,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ coefs, const float* __restrict__ gscale,
    float* __restrict__ partial, bf16_t* __restrict__ dY, int N, int H, int W, int C,
    long long sstride) {
  constexpr int UNROLL = (POOL && KWIN && DIMS == 3) ? 1 : 2;
  const int G = C / 8;
  // per-micro-batch BatchNorm groups (bn_group_backward): blockIdx.y = group of N slices,
  // its statistics rows sstride floats apart, its coefficients [3][C] and partial rows
  // (gridDim.x per group) in group order; one group: blockIdx.y = 0
  {
    const int grp = blockIdx.y;
    const long long gel = (long long)N * H * W * C;
    y += grp * gel;
    if (dA != nullptr) dA += grp * gel;
    if (dY != nullptr) dY += grp * gel;
    if (POOL) dP += grp * (gel / (DIMS == 3 ? 8 : 4));
    scale += grp * sstride; shift += grp * sstride;
    mean += grp * sstride; invstd += grp * sstride;
    if (MODE == 1) coefs += grp * 3LL * C;
    if (MODE == 0) partial += (long long)grp * gridDim.x * 2 * C;
  }
  const int L = (POOL && !KWIN) ? 2 * G : G;     // lanes per unit (divides 256)
  const int tid = threadIdx.x;
  const int cg = tid % G, c8 = cg * 8;
  const int kw = (POOL && !KWIN) ? (tid / G) & 1 : 0;
  const int upb = 256 / L;                        // units per block per step
  const int Wo = W / 2, Ho = H / 2;
  // N counts (n, d) slices; a 3-D pooled unit row covers slices 2*nd and 2*nd + 1
  const int units = POOL ? (DIMS == 3 ? N / 2 : N) * Ho * Wo : N * H * W;
  const int stride = gridDim.x * upb;
  const float gs = gscale != nullptr ? gscale[0] : 1.0f;
  float sc[8], sh[8], is[8], nm[8], k1[8], m1[8], m2[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[c8 + j]; sh[j] = shift[c8 + j];
    is[j] = invstd[c8 + j]; nm[j] = -mean[c8 + j] * is[j];
    if (MODE == 1) { k1[j] = coefs[c8 + j]; m1[j] = coefs[C + c8 + j]; m2[j] = coefs[2 * C + c8 + j]; }
    s1[j] = 0.f; s2[j] = 0.f;
  }
  // pixels per lane per unit: k = 2*kd + kh, KWIN: k = 2 * (2*kd + kh) + kw
  constexpr int NK = POOL ? (DIMS == 3 ? 4 : 2) * (KWIN ? 2 : 1) : 1;
  for (int u0 = blockIdx.x * upb + tid / L; u0 < units; u0 += UNROLL * stride) {
    uint4 vy[UNROLL][NK], vd[UNROLL][NK], vp[UNROLL];
    long long off[UNROLL][NK];
    bool ok[UNROLL];
#pragma unroll
    for (int r = 0; r < UNROLL; ++r) {            // all loads first (memory-level parallelism)
      const int u = u0 + r * stride;
      ok[r] = u < units;
      const int uu = ok[r] ? u : u0;
      if (POOL) {
        const int rr = uu / Wo, wo = uu - rr * Wo;
        long long pix0;
        if (DIMS == 3) {
          const int nd = rr / Ho, ho = rr - nd * Ho;
          pix0 = ((long long)(2 * nd) * H + 2 * ho) * W + 2 * wo + kw;
        } else {
          pix0 = (long long)rr * 2 * W + 2 * wo + kw;
        }
#pragma unroll
        for (int k = 0; k < NK; ++k) {
          const int kk = KWIN ? k >> 1 : k;       // 2*kd + kh
          off[r][k] = (pix0 + (long long)(kk >> 1) * H * W + (kk & 1) * W + (KWIN ? (k & 1) : 0)) * C + c8;
        }
        vp[r] = *reinterpret_cast<const uint4*>(dP + (long long)uu * C + c8);
      } else {
        off[r][0] = (long long)uu * C + c8;
      }
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        vy[r][k] = *reinterpret_cast<const uint4*>(y + off[r][k]);
        vd[r][k] = dA != nullptr ? *reinterpret_cast<const uint4*>(dA + off[r][k]) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < UNROLL; ++r) {
      float fy[NK][8], fd[NK][8], fp[8];
      int bestk[8];
#pragma unroll
      for (int k = 0; k < NK; ++k) { unpack8(vy[r][k], fy[k]); unpack8(vd[r][k], fd[k]); }
      if (POOL) {
        unpack8(vp[r], fp);
        // bf16-rounded activations of my NK pixels, partner's via lane ^ G
        float a[NK][8];
#pragma unroll
        for (int k = 0; k < NK; ++k)
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const uint32_t w2 = pack2(fmaxf(fmaf(fy[k][j], sc[j], sh[j]), 0.f),
                                      fmaxf(fmaf(fy[k][j + 1], sc[j + 1], sh[j + 1]), 0.f));
            a[k][j] = lo_bf(w2); a[k][j + 1] = hi_bf(w2);
          }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // window values in scan order w = 2*k + kw (k = 2*kd + kh)
          int best = 0;
          float bv = 0.f;
          if (KWIN) {                             // my pixel k IS scan position k
#pragma unroll
            for (int k = 0; k < NK; ++k)
              if (k == 0 || a[k][j] > bv) { bv = a[k][j]; best = k; }
          } else {
#pragma unroll
            for (int k = 0; k < NK; ++k) {
              const float pk = __shfl_xor(a[k][j], G, 64);
              const float v0 = kw ? pk : a[k][j], v1 = kw ? a[k][j] : pk;
              if (k == 0 || v0 > bv) { bv = v0; best = 2 * k; }
              if (v1 > bv) { bv = v1; best = 2 * k + 1; }
            }
          }
          bestk[j] = best;                        // routed to (k, kw) = (best >> 1, best & 1)
        }
      }
      if (!ok[r]) continue;
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = fmaf(fy[k][j], sc[j], sh[j]);
          float dt = fd[k][j];
          if (POOL && bestk[j] == (KWIN ? k : 2 * k + kw)) dt += fp[j];
          const float dyh = a > 0.f ? dt * gs : 0.f;
          const float xh = fmaf(fy[k][j], is[j], nm[j]);
          if (MODE == 0) { s1[j] += dyh; s2[j] = fmaf(dyh, xh, s2[j]); }
          else o[j] = k1[j] * (dyh - m1[j] - xh * m2[j]);
        }
        if (MODE == 1) {
          // streaming store (non-temporal: dY is read back by the next kernels from HBM
          // anyway): -1.4% over all BN-backward passes, profiles/r4/bn_bwd_nt_ab_r4x.txt
          const uint4 q = pack8(o);
          __builtin_nontemporal_store(u32x4_t{q.x, q.y, q.z, q.w}, reinterpret_cast<u32x4_t*>(dY + off[r][k]));
        }
      }
    }
  }
  if (MODE == 0) {
    // block reduction: threads with equal cg hold the same channels
    __shared__ float red[256 * 8];
    for (int half = 0; half < 2; ++half) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 8; ++j) red[j * 256 + tid] = half ? s2[j] : s1[j];
      __syncthreads();
      for (int c = tid; c < C; c += 256) {
        const int g2 = c / 8, j = c % 8;
        float t = 0.f;
        for (int k = g2; k < 256; k += G) t += red[j * 256 + k];
        partial[(long long)blockIdx.x * 2 * C + half * C + c] = t;
      }
    }
  }
}

int grid_for(long long items, int per_block) {
  long long g = (items + per_block - 1) / per_block;
  return (int)std::max<long long>(1, std::min<long long>(g, 2048));
}

}  // namespace

int bn_bwd_reduce_blocks(long long items) {
  // <= 2048 partial rows (the per-channel finalize reads them in one kernel): enough
  // workgroups to keep HBM busy
  return (int)std::max<long long>(1, std::min<long long>((items + 63) / 64, 2048));
}

namespace {
bool bn_bwd2_ok(int dims, bool pool, int D, int H, int W, int C) {
  const int G = C / 8;
  if (C % 8 != 0 || (G & (G - 1)) != 0 || G > 256) return false;
  if (pool && (H % 2 != 0 || W % 2 != 0 || (dims == 3 && D % 2 != 0))) return false;
  return true;
}

template <int MODE>
void bn_bwd2_launch(int grid, int dims, bool pool, const bf16_t* dA, const bf16_t* dP,
                    const bf16_t* y, const float* scale, const float* shift, const float* mean,
                    const float* invstd, const float* coefs, const float* gscale, float* partial,
                    bf16_t* dY, int N, int D, int H, int W, int C, hipStream_t st,
                    int groups = 1, long long sstride = 0) {
  // (groups > 1: N = images per group, the groups' tensors follow each other)
  const int ND = N * (dims == 3 ? D : 1);
  const dim3 gr(grid, groups);
  if (pool && C / 8 > 32) {                        // window kw pair inside the lane
    if (dims == 3)
      hipLaunchKernelGGL((bn_bwd2_kernel<3, true, MODE, true>), gr, dim3(256), 0, st, dA, dP, y,
                         scale, shift, mean, invstd, coefs, gscale, partial, dY, ND, H, W, C, sstride);
    else
      hipLaunchKernelGGL((bn_bwd2_kernel<2, true, MODE, true>), gr, dim3(256), 0, st, dA, dP, y,
                         scale, shift, mean, invstd, coefs, gscale, partial, dY, ND, H, W, C, sstride);
    return;
  }
  if (dims == 3 && pool)
    hipLaunchKernelGGL((bn_bwd2_kernel<3, true, MODE>), gr, dim3(256), 0, st, dA, dP, y,
                       scale, shift, mean, invstd, coefs, gscale, partial, dY, ND, H, W, C, sstride);
  else if (pool)
    hipLaunchKernelGGL((bn_bwd2_kernel<2, true, MODE>), gr, dim3(256), 0, st, dA, dP, y,
                       scale, shift, mean, invstd, coefs, gscale, partial, dY, ND, H, W, C, sstride);
  else
    hipLaunchKernelGGL((bn_bwd2_kernel<2, false, MODE>), gr, dim3(256), 0, st, dA, dP, y,
                       scale, shift, mean, invstd, coefs, gscale, partial, dY, ND, H, W, C, sstride);
}
}  // namespace

void bn_relu_apply_launch(const bf16_t* y, const float* scale, const float* shift, bf16_t* out,
                          bf16_t* pooled, int dims, int N, int D, int H, int W, int C,
                          hipStream_t st, int groups, long long sstride) {
  // groups > 1: N = images per group (per-micro-batch BatchNorm, statistics rows sstride apart)
  const long long G = C / 8;
  const int cap = std::max(1, 8192 / groups);
  if (pooled == nullptr) {
    const long long items = (long long)N * D * H * W * G;
    const dim3 gr(std::min(grid_for(items, 256), cap), groups);
    if (dims == 2)
      hipLaunchKernelGGL((bn_relu_apply_kernel<2, false>), gr, dim3(256), 0,
                         st, y, scale, shift, out, pooled, N, D, H, W, C, sstride);
    else
      hipLaunchKernelGGL((bn_relu_apply_kernel<3, false>), gr, dim3(256), 0,
                         st, y, scale, shift, out, pooled, N, D, H, W, C, sstride);
    return;
  }
  const long long items = (long long)N * (dims == 3 ? D / 2 : 1) * (H / 2) * (W / 2) * G;
  const dim3 gr(std::min(grid_for(items, 256), cap), groups);
  const long long units = (long long)N * (dims == 3 ? D / 2 : 1) * (H / 2) * (W / 2);
  if ((G & (G - 1)) == 0 && G <= 32 && units < (1LL << 31)) {
    // v2: lanes (kw, cg) over the window's pixel pair, UNROLL units per thread in flight
    const int ND = N * (dims == 3 ? D : 1);
    const long long per = (256 / (2 * G)) * 2;       // units per block per grid-stride pass
    const dim3 g2((unsigned)std::max<long long>(1, std::min<long long>((units + per - 1) / per,
                                                                     std::max(1, 8192 / groups))), groups);
    if (dims == 2)
      hipLaunchKernelGGL((bn_relu_pool2_kernel<2>), g2, dim3(256), 0, st, y, scale, shift, out, pooled,
                         ND, H, W, C, sstride);
    else
      hipLaunchKernelGGL((bn_relu_pool2_kernel<3>), g2, dim3(256), 0, st, y, scale, shift, out, pooled,
                         ND, H, W, C, sstride);
    return;
  }
  if (dims == 2)
    hipLaunchKernelGGL((bn_relu_apply_kernel<2, true>), gr, dim3(256), 0, st, y, scale,
                       shift, out, pooled, N, D, H, W, C, sstride);
  else
    hipLaunchKernelGGL((bn_relu_apply_kernel<3, true>), gr, dim3(256), 0, st, y, scale,
                       shift, out, pooled, N, D, H, W, C, sstride);
}

#define BN_BWD_DISPATCH(MODE, grid)                                                         \
  do {                                                                                      \
    if (dims == 2) {                                                                        \
      if (pool) hipLaunchKernelGGL((bn_bwd_kernel<2, true, MODE>), dim3(grid), dim3(256), 0, \
                                   st, dA, dP, y, scale, shift, mean, invstd, coefs, gscale,  \
                                   partial, dY, N, D, H, W, C);                              \
      else hipLaunchKernelGGL((bn_bwd_kernel<2, false, MODE>), dim3(grid), dim3(256), 0, st,  \
                              dA, dP, y, scale, shift, mean, invstd, coefs, gscale, partial,  \
                              dY, N, D, H, W, C);                                           \
    } else {                                                                                \
      if (pool) hipLaunchKernelGGL((bn_bwd_kernel<3, true, MODE>), dim3(grid), dim3(256), 0, \
                                   st, dA, dP, y, scale, shift, mean, invstd, coefs, gscale,  \
                                   partial, dY, N, D, H, W, C);                              \
      else hipLaunchKernelGGL((bn_bwd_kernel<3, false, MODE>), dim3(grid), dim3(256), 0, st,  \
                              dA, dP, y, scale, shift, mean, invstd, coefs, gscale, partial,  \
                              dY, N, D, H, W, C);                                           \
    }                                                                                       \
  } while (0)

void bn_bwd_reduce_launch(const bf16_t* dA, const bf16_t* dP, const bf16_t* y,
                          const float* scale, const float* shift, const float* mean,
                          const float* invstd, const float* gscale, float* partial, int nblocks,
                          int dims, int N, int D, int H, int W, int C, hipStream_t st) {
  const bool pool = dP != nullptr;
  const float* coefs = nullptr;
  bf16_t* dY = nullptr;
  if (bn_bwd2_ok(dims, pool, D, H, W, C)) {
    bn_bwd2_launch<0>(nblocks, dims, pool, dA, dP, y, scale, shift, mean, invstd, coefs, gscale,
                      partial, dY, N, D, H, W, C, st);
    return;
  }
  BN_BWD_DISPATCH(0, nblocks);
}

void bn_bwd_apply_launch(const bf16_t* dA, const bf16_t* dP, const bf16_t* y, const float* scale,
                         const float* shift, const float* mean, const float* invstd,
                         const float* coefs, const float* gscale, bf16_t* dY, int dims, int N,
                         int D, int H, int W, int C, hipStream_t st) {
  const bool pool = dP != nullptr;
  float* partial = nullptr;
  const int G = C / 8;
  const long long items = (long long)N * (pool ? (dims == 3 ? D / 2 : 1) * (H / 2) * (W / 2)
                                                : (long long)D * H * W);
  const int per = std::max(1, 256 / G);
  if (bn_bwd2_ok(dims, pool, D, H, W, C)) {
    const int upb = 256 / ((pool && G <= 32) ? 2 * G : G);
    const int grid2 = (int)std::max<long long>(1, std::min<long long>((items + 2 * upb - 1) / (2 * upb), 8192));
    bn_bwd2_launch<1>(grid2, dims, pool, dA, dP, y, scale, shift, mean, invstd, coefs, gscale,
                      partial, dY, N, D, H, W, C, st);
    return;
  }
  const int grid = std::min(grid_for(items, per), 16384);
  BN_BWD_DISPATCH(1, grid);
}

// ===================================================================== per-micro-batch groups
// A window of accumulation micro-batches run as ONE batched pass (Trainer bn_window): the
// weights are fixed inside the window and a train-mode BatchNorm normalises over its own
// micro-batch (ref.py:580,583 with batch_size 1, ref.py:686), so every BatchNorm keeps one
// statistics group per micro-batch.  The batch is the groups' tensors one after another;
// statistics are [groups][4][C] (mean | invstd | scale | shift), coefficients [groups][3][C].
namespace {

// per-group channel (sum, sum^2) of y: grid (nb, groups), a thread keeps one 8-channel group
// (C / 8 lanes per pixel, a power of two dividing 256); partial rows [groups][nb][2][C]
__global__ __launch_bounds__(256) void bn_group_stats_kernel(const bf16_t* __restrict__ y,
                                                             long long gpix, int C,
                                                             float* __restrict__ partial) {
  const int G8 = C / 8;
  const int tid = threadIdx.x;
  const int c8 = (tid % G8) * 8;
  const int upb = 256 / G8;
  const int grp = blockIdx.y;
  y += grp * gpix * C;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  const long long stride = (long long)gridDim.x * upb;
  long long p = (long long)blockIdx.x * upb + tid / G8;
  for (; p + stride < gpix; p += 2 * stride) {     // two pixels' loads in flight
    const uint4 v0 = *reinterpret_cast<const uint4*>(y + p * C + c8);
    const uint4 v1 = *reinterpret_cast<const uint4*>(y + (p + stride) * C + c8);
    float f0[8], f1[8];
    unpack8(v0, f0);
    unpack8(v1, f1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s1[j] += f0[j] + f1[j];
      s2[j] = fmaf(f0[j], f0[j], fmaf(f1[j], f1[j], s2[j]));
    }
  }
  if (p < gpix) {
    float f0[8];
    unpack8(*reinterpret_cast<const uint4*>(y + p * C + c8), f0);
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[j] += f0[j]; s2[j] = fmaf(f0[j], f0[j], s2[j]); }
  }
  __shared__ float red[256 * 8];
  float* out = partial + ((long long)grp * gridDim.x + blockIdx.x) * 2 * C;
  for (int half = 0; half < 2; ++half) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[j * 256 + tid] = half ? s2[j] : s1[j];
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
      const int g2 = c / 8, j = c % 8;
      float t = 0.f;
      for (int k = g2; k < 256; k += G8) t += red[j * 256 + k];
      out[half * C + c] = t;
    }
  }
}

// Finalize kernels: grid (channel chunks of 64, groups), 256 threads = 64 channels x 4 row
// lanes.  A thread sums rows r = lane4, lane4 + 4, ... of its (group, channel) in fp64 —
// loads coalesced across the 64 channels (the partial rows are [groups][nb][2][C]) — and the
// 4 row lanes combine in LDS in a fixed order (deterministic).
constexpr int kFR = 4;                       // row lanes per finalize workgroup
DDLPC_DEVICE void group_rows_sum(const float* __restrict__ rows, int nb, int C, int c, int rl,
                                 double& a, double& b) {
  a = 0.0; b = 0.0;
  int r = rl;
  for (; r + 3 * kFR < nb; r += 4 * kFR) {   // four rows' loads in flight
    const float a0 = rows[(long long)r * 2 * C + c], b0 = rows[(long long)r * 2 * C + C + c];
    const float a1 = rows[(long long)(r + kFR) * 2 * C + c], b1 = rows[(long long)(r + kFR) * 2 * C + C + c];
    const float a2 = rows[(long long)(r + 2 * kFR) * 2 * C + c], b2 = rows[(long long)(r + 2 * kFR) * 2 * C + C + c];
    const float a3 = rows[(long long)(r + 3 * kFR) * 2 * C + c], b3 = rows[(long long)(r + 3 * kFR) * 2 * C + C + c];
    a += (double)a0 + (double)a1 + (double)a2 + (double)a3;
    b += (double)b0 + (double)b1 + (double)b2 + (double)b3;
  }
  for (; r < nb; r += kFR) {
    a += (double)rows[(long long)r * 2 * C + c];
    b += (double)rows[(long long)r * 2 * C + C + c];
  }
}

// stats4 per group (mean | invstd | scale | shift), and the group's (mean, unbiased var) into
// its arena row (the running statistics are then updated in micro-batch order:
// bn_running_apply)
__global__ __launch_bounds__(64 * kFR) void bn_group_finalize_kernel(
    const float* __restrict__ partial, int nb, int groups, int C, double count,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    float* __restrict__ out4, float* __restrict__ arena, long long astride) {
  __shared__ double red[2][kFR][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, g = blockIdx.y;
  double a = 0.0, b = 0.0;
  if (c < C) group_rows_sum(partial + (long long)g * nb * 2 * C, nb, C, c, rl, a, b);
  red[0][rl][cl] = a;
  red[1][rl][cl] = b;
  __syncthreads();
  if (rl != 0 || c >= C) return;
  a = 0.0; b = 0.0;
#pragma unroll
  for (int k = 0; k < kFR; ++k) { a += red[0][k][cl]; b += red[1][k][cl]; }
  const double mean = a / count;
  double var = b / count - mean * mean;
  if (var < 0) var = 0;
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * inv;
  float* o = out4 + (long long)g * 4 * C;
  o[c] = (float)mean;
  o[C + c] = inv;
  o[2 * C + c] = sc;
  o[3 * C + c] = beta[c] - (float)mean * sc;
  if (arena != nullptr) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    arena[g * astride + c] = (float)mean;
    arena[g * astride + C + c] = (float)unb;
  }
}

// BatchNorm-backward finalize per group: coefficients [k | m1 | m2] of every group and the
// group's fp64 sums into gsum [groups][2][C] (dbeta / dgamma terms) ...
__global__ __launch_bounds__(64 * kFR) void bn_group_grad_finalize_kernel(
    const float* __restrict__ partial, int nb, int groups, int C, double count,
    const float* __restrict__ gamma, const float* __restrict__ stats4, double* __restrict__ gsum,
    float* __restrict__ coefs, const float* __restrict__ dscale) {
  __shared__ double red[2][kFR][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, g = blockIdx.y;
  double a = 0.0, b = 0.0;
  if (c < C) group_rows_sum(partial + (long long)g * nb * 2 * C, nb, C, c, rl, a, b);
  red[0][rl][cl] = a;
  red[1][rl][cl] = b;
  __syncthreads();
  if (rl != 0 || c >= C) return;
  a = 0.0; b = 0.0;
#pragma unroll
  for (int k = 0; k < kFR; ++k) { a += red[0][k][cl]; b += red[1][k][cl]; }
  if (dscale != nullptr) { a *= (double)dscale[0]; b *= (double)dscale[0]; }
  gsum[((long long)g * 2) * C + c] = a;
  gsum[((long long)g * 2 + 1) * C + c] = b;
  float* k = coefs + (long long)g * 3 * C;
  k[c] = gamma[c] * stats4[(long long)g * 4 * C + C + c];
  k[C + c] = (float)(a / count);
  k[2 * C + c] = (float)(b / count);
}

// ... then dbeta / dgamma = those sums over the groups in group order (deterministic)
__global__ __launch_bounds__(256) void bn_group_grad_sum_kernel(const double* __restrict__ gsum, int groups,
                                                                int C, float* dgamma, float* dbeta,
                                                                int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, b = 0.0;
  for (int g = 0; g < groups; ++g) {
    a += gsum[((long long)g * 2) * C + c];
    b += gsum[((long long)g * 2 + 1) * C + c];
  }
  dbeta[c] = accumulate ? dbeta[c] + (float)a : (float)a;
  dgamma[c] = accumulate ? dgamma[c] + (float)b : (float)b;
}

int bn_group_rows(long long gpix, int C, int groups) {
  // rows per group: enough workgroups over all groups to fill the chip, each >= 16 steps
  const long long units = gpix * (C / 8);
  long long nb = (units + 256 * 16 - 1) / (256 * 16);
  nb = std::min<long long>(nb, std::max(1, 4096 / groups));
  return (int)std::max<long long>(1, std::min<long long>(nb, 256));
}

}  // namespace

bool bn_group_supported(int dims, bool pool, int D, int H, int W, int C) {
  const int G8 = C / 8;
  return C % 8 == 0 && (G8 & (G8 - 1)) == 0 && G8 <= 256 && bn_bwd2_ok(dims, pool, D, H, W, C);
}

void bn_group_stats_finalize_launch(const bf16_t* y, int groups, long long gpix, int C,
                                    const float* gamma, const float* beta, float eps, float* out4,
                                    float* arena, long long astride, float* partial_scratch,
                                    int nb, hipStream_t st) {
  hipLaunchKernelGGL(bn_group_stats_kernel, dim3(nb, groups), dim3(256), 0, st, y, gpix, C,
                     partial_scratch);
  hipLaunchKernelGGL(bn_group_finalize_kernel, dim3((C + 63) / 64, groups), dim3(64 * kFR), 0, st,
                     partial_scratch, nb, groups, C, (double)gpix, gamma, beta, eps, out4, arena, astride);
}

int bn_group_stats_rows(long long gpix, int C, int groups) { return bn_group_rows(gpix, C, groups); }

// statistics from partial rows a producer already wrote group-major ([groups][nb][2][C]: the
// conv epilogues' rows in BN-group mode, ConvFwdArgs::groups)
void bn_group_finalize_rows_launch(const float* partial, int nb, int groups, long long gpix, int C,
                                   const float* gamma, const float* beta, float eps, float* out4,
                                   float* arena, long long astride, hipStream_t st) {
  hipLaunchKernelGGL(bn_group_finalize_kernel, dim3((C + 63) / 64, groups), dim3(64 * kFR), 0, st,
                     partial, nb, groups, C, (double)gpix, gamma, beta, eps, out4, arena, astride);
}

void bn_group_backward_launch(const bf16_t* dA, const bf16_t* dP, const bf16_t* y,
                              const float* stats4, const float* gamma, float* dgamma, float* dbeta,
                              bool accumulate, float* coefs, float* partial_scratch, int nb,
                              bf16_t* dY, int dims, int groups, int N, int D, int H, int W, int C,
                              hipStream_t st, bool have_partial, double* gsum_scratch) {
  const bool pool = dP != nullptr;
  const long long sstride = 4LL * C;
  const float* s = stats4;
  // have_partial: the rows [groups][nb][2][C] came from the data-gradient conv's BN-backward
  // epilogue (ConvFwdArgs::bnb_y in group mode) — no reduction pass
  if (!have_partial)
    bn_bwd2_launch<0>(nb, dims, pool, dA, dP, y, s + 2 * C, s + 3 * C, s, s + C, nullptr, nullptr,
                      partial_scratch, nullptr, N, D, H, W, C, st, groups, sstride);
  const double count = (double)N * D * H * W;
  hipLaunchKernelGGL(bn_group_grad_finalize_kernel, dim3((C + 63) / 64, groups), dim3(64 * kFR), 0, st,
                     partial_scratch, nb, groups, C, count, gamma, stats4, gsum_scratch, coefs, nullptr);
  hipLaunchKernelGGL(bn_group_grad_sum_kernel, dim3((C + 255) / 256), dim3(256), 0, st, gsum_scratch,
                     groups, C, dgamma, dbeta, accumulate ? 1 : 0);
  const long long items = (long long)N * (pool ? (dims == 3 ? D / 2 : 1) * (H / 2) * (W / 2)
                                                : (long long)D * H * W);
  const int upb = 256 / ((pool && C / 8 <= 32) ? 2 * (C / 8) : C / 8);
  const int grid2 = (int)std::max<long long>(
      1, std::min<long long>((items + 2 * upb - 1) / (2 * upb), std::max(1, 8192 / groups)));
  bn_bwd2_launch<1>(grid2, dims, pool, dA, dP, y, s + 2 * C, s + 3 * C, s, s + C, coefs, nullptr,
                    nullptr, dY, N, D, H, W, C, st, groups, sstride);
}

void bn_group_grad_rows_launch(const float* partial, int nb, int groups, int C, double count,
                               const float* gamma, const float* stats4, float* dgamma, float* dbeta,
                               bool accumulate, float* coefs, double* gsum_scratch,
                               const float* dscale, hipStream_t st) {
  hipLaunchKernelGGL(bn_group_grad_finalize_kernel, dim3((C + 63) / 64, groups), dim3(64 * kFR), 0, st,
                     partial, nb, groups, C, count, gamma, stats4, gsum_scratch, coefs, dscale);
  hipLaunchKernelGGL(bn_group_grad_sum_kernel, dim3((C + 255) / 256), dim3(256), 0, st, gsum_scratch,
                     groups, C, dgamma, dbeta, accumulate ? 1 : 0);
}

int bn_group_bwd_rows(long long items, int groups) {
  return (int)std::max<long long>(1, std::min<long long>((items + 255) / 256, std::max(1, 4096 / groups)));
}

}  // namespace ddlpc
