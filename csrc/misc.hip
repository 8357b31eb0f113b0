// Optimizer, weight packing, gradient codec and small layout kernels.
//   * adam:        K14 — fused Adam over the flat fp32 parameter buffer (ref.py:704,437,552)
//   * weight_pack: fp32 OIHW/IOHW parameters -> bf16 kernel layouts (fwd + flipped dgrad),
//                  all conv weights of the model in ONE launch
//   * codec:       K16-K18 — absmax / quantise / dequantise-sum of the reference's lossy
//                  gradient compression (ref.py:328-545), multi-segment
//   * bilinear x2 up-sampling (align_corners=True), the alternative UpBlock mode (ref.py:609)
//   * NCHW -> NHWC bf16 input conversion, per-channel column sums (transposed-conv bias grad)
#include "common.h"
#include "ops.h"

namespace ddlpc {

namespace {

// dscal (optional, hipGraph replays): device [t, step_size, inv_sqrt_bc2] written by
// adam_scalars_kernel in the same graph, overriding the host-side scalars
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                            float* __restrict__ m, float* __restrict__ v, long long n, float b1,
                            float b2, float eps, float wd, float step_size, float inv_sqrt_bc2,
                            const float* __restrict__ dscal) {
  if (dscal != nullptr) { step_size = dscal[1]; inv_sqrt_bc2 = dscal[2]; }
  const long long n4 = n / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* P = &pp.x; float* G = &gg.x; float* M = &mm.x; float* V = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gr = wd != 0.f ? G[j] + wd * P[j] : G[j];
      M[j] = M[j] + (1.f - b1) * (gr - M[j]);            // lerp, as torch.optim.Adam
      V[j] = b2 * V[j] + (1.f - b2) * gr * gr;
      const float denom = sqrtf(V[j]) * inv_sqrt_bc2 + eps;
      P[j] = P[j] - step_size * M[j] / denom;
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  // tail
  for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float gr = wd != 0.f ? g[i] + wd * p[i] : g[i];
    m[i] = m[i] + (1.f - b1) * (gr - m[i]);
    v[i] = b2 * v[i] + (1.f - b2) * gr * gr;
    p[i] = p[i] - step_size * m[i] / (sqrtf(v[i]) * inv_sqrt_bc2 + eps);
  }
}

// LDS-tiled transposes: a workgroup loads one (32 x 32-channel) tile of the fp32 source
// with coalesced reads, then writes every packed layout from LDS as contiguous 64-B runs
// (both sides coalesced; all weights of the model in one launch, blockIdx.y = entry).
//   conv3 (OIHW [co][ci][tap]):  tile = 32 co x (32 ci x taps)   (10 ci for 27 taps)
//     fwd   [co][tap][CinW]      runs of 32 ci
//     dgrad [ci][taps-1-tap][CoutW] runs of 32 co
//   convT (IOHW [ci][co][sub]):  tile = 32 ci x (32 co x S)
//     fwd   [(sub, co)][Cin]     runs of 32 ci
//     dgrad [ci][(sub, co)]      runs of 32 co
// Packing pads (ci >= Cin) were zeroed at allocation and are never written.
constexpr int PT = 32;
__global__ __launch_bounds__(256) void weight_pack_kernel(const PackEntry* __restrict__ ents) {
  __shared__ float tile[PT][PT * 9 + 1];
  const PackEntry e = ents[blockIdx.y];
  const int T = e.taps;
  const int NC = min(PT, PT * 9 / T);                 // tile columns: 32, or 10 for 27 taps
  // tile grid: conv3 rows = co, cols = ci; convT rows = ci, cols = co
  const int R = e.kind == 0 ? e.Cout : e.Cin, Cc = e.kind == 0 ? e.Cin : e.Cout;
  const int tr = (R + PT - 1) / PT, tc = (Cc + NC - 1) / NC;
  const int tid = threadIdx.x;
  for (int t = blockIdx.x; t < tr * tc; t += gridDim.x) {
    const int r0 = (t / tc) * PT, c0 = (t % tc) * NC;
    const int nr = min(PT, R - r0), nc = min(NC, Cc - c0);
    __syncthreads();
    // load: row r, the nc*T contiguous floats of columns [c0, c0+nc)
    for (int i = tid; i < PT * NC * T; i += 256) {
      const int r = i / (NC * T), j = i % (NC * T);
      if (r < nr && j < nc * T)
        tile[r][j] = e.src[((long long)(r0 + r) * Cc + c0) * T + j];
    }
    __syncthreads();
    if (e.kind == 0) {
      // fwd: [co = r0+r][tap][ci = c0 + c] — a thread writes a (c, c+1) pair as one 4-byte
      // store (NC, c0, CinW even; a lone last channel of an odd Cin is written alone)
      for (int i = tid; i < PT * T * (NC / 2); i += 256) {
        const int c = 2 * (i % (NC / 2)), rt = i / (NC / 2), tap = rt % T, r = rt / T;
        if (r < nr && c < nc) {
          bf16_t* d = e.fwd + ((long long)(r0 + r) * T + tap) * e.CinW + c0 + c;
          if (c + 1 < nc)
            *reinterpret_cast<uint32_t*>(d) = pack2(tile[r][c * T + tap], tile[r][(c + 1) * T + tap]);
          else
            d[0] = f2bf(tile[r][c * T + tap]);
        }
      }
      // dgrad: [ci = c0 + c][tp][co = r0 + r], source tap = T-1-tp (co pairs: r0, CoutW even)
      if (e.dgrad != nullptr)
        for (int i = tid; i < (PT / 2) * T * NC; i += 256) {
          const int r = 2 * (i % (PT / 2)), ct = i / (PT / 2), tp = ct % T, c = ct / T;
          if (r < nr && c < nc) {
            bf16_t* d = e.dgrad + ((long long)(c0 + c) * T + tp) * e.CoutW + r0 + r;
            const int st = c * T + (T - 1 - tp);
            if (r + 1 < nr)
              *reinterpret_cast<uint32_t*>(d) = pack2(tile[r][st], tile[r + 1][st]);
            else
              d[0] = f2bf(tile[r][st]);
          }
        }
    } else {
      // fwd: [(sub, co = c0 + c)][ci = r0 + r]
      for (int i = tid; i < PT * T * NC; i += 256) {
        const int r = i % PT, cs = i / PT, c = cs % NC, sub = cs / NC;
        if (r < nr && c < nc)
          e.fwd[((long long)sub * e.Cout + c0 + c) * e.Cin + r0 + r] = f2bf(tile[r][c * T + sub]);
      }
      // dgrad: [ci = r0 + r][(sub, co = c0 + c)]
      if (e.dgrad != nullptr)
        for (int i = tid; i < PT * T * NC; i += 256) {
          const int c = i % NC, rs = i / NC, sub = rs % T, r = rs / T;
          if (r < nr && c < nc)
            e.dgrad[((long long)(r0 + r) * T + sub) * e.Cout + c0 + c] = f2bf(tile[r][c * T + sub]);
        }
    }
  }
}

// ---- codec -----------------------------------------------------------------------------
DDLPC_DEVICE void atomic_max_pos(float* addr, float v) {
  // non-negative floats order like their unsigned bit patterns
  atomicMax(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

__global__ void codec_absmax_kernel(const float* __restrict__ x, const int64_t* __restrict__ seg,
                                    float* __restrict__ scales) {
  const int s = blockIdx.y;
  const long long a = seg[2 * s], b = seg[2 * s + 1];
  float m = 0.f;
  for (long long i = a + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < b;
       i += (long long)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(x[i]));
  m = wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t = fmaxf(t, red[w]);
    atomic_max_pos(scales + s, t);
  }
}

__global__ void codec_encode_kernel(const float* __restrict__ x, const int64_t* __restrict__ seg,
                                    const float* __restrict__ scales, void* __restrict__ out,
                                    int codec) {
  const int s = blockIdx.y;
  const long long a = seg[2 * s], b = seg[2 * s + 1];
  const float sc = scales[s];
  const float L = codec == 0 ? 100.f : 10.f;
  for (long long i = a + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < b;
       i += (long long)gridDim.x * blockDim.x) {
    // torch.round(g / max * L): IEEE division then multiply, round half to even
    const float q = sc > 0.f ? rintf(__fdiv_rn(x[i], sc) * L) : 0.f;
    if (codec == 0) reinterpret_cast<__half*>(out)[i] = __float2half_rn(q);
    else reinterpret_cast<int8_t*>(out)[i] = (int8_t)q;
  }
}

__global__ void codec_decode_sum_kernel(float* __restrict__ out, const void* __restrict__ q,
                                        const float* __restrict__ scales,
                                        const float* __restrict__ w,
                                        const int64_t* __restrict__ seg, int nseg, int world,
                                        int codec, long long n) {
  const int s = blockIdx.y;
  const long long a = seg[2 * s], b = seg[2 * s + 1];
  const float L = codec == 0 ? 100.f : 10.f;
  for (long long i = a + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < b;
       i += (long long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int r = 0; r < world; ++r) {
      const float qv = codec == 0 ? __half2float(reinterpret_cast<const __half*>(q)[r * n + i])
                                  : (float)reinterpret_cast<const int8_t*>(q)[r * n + i];
      // reference decode: q.float() / L * max_grad  (ref.py:304,313)
      acc += w[r] * (__fdiv_rn(qv, L) * scales[r * nseg + s]);
    }
    out[i] = acc;
  }
}

// ---- bilinear x2, align_corners=True (2-D bilinear / 3-D trilinear), NHWC bf16 --------------
DDLPC_DEVICE void src_coord(int o, int in, int& i0, int& i1, float& f) {
  const float scale = in > 1 ? (float)(in - 1) / (float)(2 * in - 1) : 0.f;
  const float x = o * scale;
  i0 = (int)floorf(x);
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + 1 < in ? i0 + 1 : in - 1;
  f = x - i0;
}

template <int DIMS>
__global__ void bilinear_up2_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N,
                                        int D, int H, int W, int C) {
  const int Do = DIMS == 3 ? 2 * D : 1, Ho = 2 * H, Wo = 2 * W;
  const long long total = (long long)N * Do * Ho * Wo * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    long long q = e / C;
    const int wo = (int)(q % Wo); q /= Wo;
    const int ho = (int)(q % Ho); q /= Ho;
    const int dd = DIMS == 3 ? (int)(q % Do) : 0;
    const int n = (int)(DIMS == 3 ? q / Do : q);
    int h0, h1, w0, w1, d0 = 0, d1 = 0;
    float fh, fw, fd = 0.f;
    src_coord(ho, H, h0, h1, fh);
    src_coord(wo, W, w0, w1, fw);
    if (DIMS == 3) src_coord(dd, D, d0, d1, fd);
    auto at = [&](int d, int h, int w) {
      return bf2f(x[((((long long)n * D + d) * H + h) * W + w) * C + c]);
    };
    float v = (1 - fh) * ((1 - fw) * at(d0, h0, w0) + fw * at(d0, h0, w1)) +
              fh * ((1 - fw) * at(d0, h1, w0) + fw * at(d0, h1, w1));
    if (DIMS == 3) {
      const float v1 = (1 - fh) * ((1 - fw) * at(d1, h0, w0) + fw * at(d1, h0, w1)) +
                       fh * ((1 - fw) * at(d1, h1, w0) + fw * at(d1, h1, w1));
      v = (1 - fd) * v + fd * v1;
    }
    y[e] = f2bf(v);
  }
}

template <int DIMS>
__global__ void bilinear_up2_bwd_kernel(const bf16_t* __restrict__ dy, float* __restrict__ dx,
                                        int N, int D, int H, int W, int C) {
  const int Do = DIMS == 3 ? 2 * D : 1, Ho = 2 * H, Wo = 2 * W;
  const long long total = (long long)N * Do * Ho * Wo * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    long long q = e / C;
    const int wo = (int)(q % Wo); q /= Wo;
    const int ho = (int)(q % Ho); q /= Ho;
    const int dd = DIMS == 3 ? (int)(q % Do) : 0;
    const int n = (int)(DIMS == 3 ? q / Do : q);
    int h0, h1, w0, w1, d0 = 0, d1 = 0;
    float fh, fw, fd = 0.f;
    src_coord(ho, H, h0, h1, fh);
    src_coord(wo, W, w0, w1, fw);
    if (DIMS == 3) src_coord(dd, D, d0, d1, fd);
    const float g = bf2f(dy[e]);
    auto add = [&](int d, int h, int w, float wt) {
      atomicAdd(dx + ((((long long)n * D + d) * H + h) * W + w) * C + c, g * wt);
    };
    const float wd0 = DIMS == 3 ? 1 - fd : 1.f;
    add(d0, h0, w0, wd0 * (1 - fh) * (1 - fw));
    add(d0, h0, w1, wd0 * (1 - fh) * fw);
    add(d0, h1, w0, wd0 * fh * (1 - fw));
    add(d0, h1, w1, wd0 * fh * fw);
    if (DIMS == 3) {
      add(d1, h0, w0, fd * (1 - fh) * (1 - fw));
      add(d1, h0, w1, fd * (1 - fh) * fw);
      add(d1, h1, w0, fd * fh * (1 - fw));
      add(d1, h1, w1, fd * fh * fw);
    }
  }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

// strided [N][C][S] (fp32 or bf16; NCHW or channels-last memory) -> [N][S][Cp] bf16 with the
// channels zero-padded to Cp (the first conv reads 8-channel, 16-byte pixels)
// one thread per (pixel, 8-channel group): gathers up to 8 input channels (strided NCHW or
// channel-last, fp32 or bf16), pads with zeros, one 16-B store
__global__ void to_nhwc_generic_kernel(const void* __restrict__ x, int in_dtype, bf16_t* __restrict__ y,
                                       int N, int C, int Cp, long long S, long long sN, long long sC,
                                       long long sS) {
  const long long total = (long long)N * Cp * S;
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(o % Cp);
    const long long s = (o / Cp) % S;
    const long long n = o / ((long long)Cp * S);
    bf16_t v = 0;
    if (c < C) {
      const long long i = n * sN + c * sC + s * sS;
      v = in_dtype == 0 ? f2bf(reinterpret_cast<const float*>(x)[i])
                        : reinterpret_cast<const bf16_t*>(x)[i];
    }
    y[o] = v;
  }
}

template <typename IDX>
__global__ void to_nhwc_pad_kernel(const void* __restrict__ x, int in_dtype, bf16_t* __restrict__ y,
                                   int N, int C, int Cp, long long S, long long sN, long long sC,
                                   long long sS) {
  const int G = Cp / 8;
  const IDX total = (IDX)N * (IDX)S * G;
  for (IDX o = blockIdx.x * (IDX)blockDim.x + threadIdx.x; o < total;
       o += (IDX)gridDim.x * blockDim.x) {
    const int gi = (int)(o % G);
    const IDX ps = o / G;
    const IDX s = ps % (IDX)S, n = ps / (IDX)S;
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = gi * 8 + j;
      f[j] = 0.f;
      if (c < C) {
        const long long i = (long long)n * sN + (long long)c * sC + (long long)s * sS;
        f[j] = in_dtype == 0 ? reinterpret_cast<const float*>(x)[i]
                             : bf2f(reinterpret_cast<const bf16_t*>(x)[i]);
      }
    }
    reinterpret_cast<uint4*>(y)[o] = pack8(f);
  }
}

// per-block per-channel sums of a [P][C] bf16 tensor -> partial[block][C]
__global__ void channel_sum_kernel(const bf16_t* __restrict__ x, long long P, int C,
                                   float* __restrict__ partial) {
  __shared__ float red[256];
  const int G = C / 8;
  const int per = (blockDim.x / G) * G;
  const int tid = threadIdx.x;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (tid < per) {
    const int cg = tid % G;
    for (long long px = blockIdx.x * (long long)(per / G) + tid / G; px < P;
         px += (long long)gridDim.x * (per / G)) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + px * C + cg * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
  for (int j = 0; j < 8; ++j) {
    __syncthreads();
    red[tid] = tid < per ? s[j] : 0.f;
    __syncthreads();
    for (int cg = tid; cg < G; cg += blockDim.x) {
      float t = 0.f;
      for (int k = cg; k < per; k += G) t += red[k];
      partial[(long long)blockIdx.x * C + cg * 8 + j] = t;
    }
  }
}

}  // namespace

void adam_launch(float* p, const float* g, float* m, float* v, long long n, float b1, float b2,
                 float eps, float wd, float step_size, float inv_sqrt_bc2, hipStream_t st,
                 const float* dscal) {
  const int grid = (int)std::min<long long>((n / 4 + 255) / 256 + 1, 2048);
  hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(256), 0, st, p, g, m, v, n, b1, b2, eps, wd,
                     step_size, inv_sqrt_bc2, dscal);
}

// one thread: t += 1, step_size = lr / (1 - b1^t), inv_sqrt_bc2 = 1 / sqrt(1 - b2^t) in
// double (the host path's arithmetic), so a captured optimizer step stays correct on replay
__global__ void adam_scalars_kernel(float* s, double lr, double b1, double b2) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double t = (double)s[0] + 1.0;
  s[0] = (float)t;
  s[1] = (float)(lr / (1.0 - pow(b1, t)));
  s[2] = (float)(1.0 / sqrt(1.0 - pow(b2, t)));
}

void adam_scalars_launch(float* s, double lr, double b1, double b2, hipStream_t st) {
  hipLaunchKernelGGL(adam_scalars_kernel, dim3(1), dim3(64), 0, st, s, lr, b1, b2);
}

void weight_pack_launch(const PackEntry* entries_dev, int n_entries, long long max_elems,
                        hipStream_t st) {
  // one workgroup per 32 x 32-channel tile of the largest entry (smaller entries loop less)
  const int gx = (int)std::max<long long>(1, std::min<long long>((max_elems + 9215) / 9216, 1024));
  hipLaunchKernelGGL(weight_pack_kernel, dim3(gx, n_entries), dim3(256), 0, st, entries_dev);
}

void codec_absmax_launch(const float* x, const int64_t* seg, int nseg, float* scales,
                         hipStream_t st) {
  (void)hipMemsetAsync(scales, 0, sizeof(float) * nseg, st);
  hipLaunchKernelGGL(codec_absmax_kernel, dim3(64, nseg), dim3(256), 0, st, x, seg, scales);
}

void codec_encode_launch(const float* x, const int64_t* seg, int nseg, const float* scales,
                         void* out, int codec, long long n, hipStream_t st) {
  (void)n;
  hipLaunchKernelGGL(codec_encode_kernel, dim3(256, nseg), dim3(256), 0, st, x, seg, scales, out,
                     codec);
}

void codec_decode_sum_launch(float* out, const void* q, const float* scales, const float* w,
                             const int64_t* seg, int nseg, int world, int codec, long long n,
                             hipStream_t st) {
  hipLaunchKernelGGL(codec_decode_sum_kernel, dim3(256, nseg), dim3(256), 0, st, out, q, scales,
                     w, seg, nseg, world, codec, n);
}

void bilinear_up2_launch(const bf16_t* x, bf16_t* y, int dims, int N, int D, int H, int W, int C,
                         bool backward, hipStream_t st) {
  (void)backward;
  const long long total = (long long)N * (dims == 3 ? 2 * D : 1) * 2 * H * 2 * W * C;
  const int grid = (int)std::min<long long>((total + 255) / 256, 8192);
  if (dims == 2)
    hipLaunchKernelGGL((bilinear_up2_fwd_kernel<2>), dim3(grid), dim3(256), 0, st, x, y, N, D, H, W, C);
  else
    hipLaunchKernelGGL((bilinear_up2_fwd_kernel<3>), dim3(grid), dim3(256), 0, st, x, y, N, D, H, W, C);
}

void bilinear_up2_bwd_launch(const bf16_t* dy, float* dx_f32, bf16_t* dx, int dims, int N, int D,
                             int H, int W, int C, hipStream_t st) {
  const long long nin = (long long)N * D * H * W * C;
  (void)hipMemsetAsync(dx_f32, 0, sizeof(float) * nin, st);
  const long long total = (long long)N * (dims == 3 ? 2 * D : 1) * 2 * H * 2 * W * C;
  const int grid = (int)std::min<long long>((total + 255) / 256, 8192);
  if (dims == 2)
    hipLaunchKernelGGL((bilinear_up2_bwd_kernel<2>), dim3(grid), dim3(256), 0, st, dy, dx_f32, N, D, H, W, C);
  else
    hipLaunchKernelGGL((bilinear_up2_bwd_kernel<3>), dim3(grid), dim3(256), 0, st, dy, dx_f32, N, D, H, W, C);
  const int g2 = (int)std::min<long long>((nin + 255) / 256, 8192);
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(g2), dim3(256), 0, st, dx_f32, dx, nin);
}

void to_nhwc_pad_launch(const void* x, int in_dtype, bf16_t* y, int N, int C, int Cp, long long S,
                        long long sN, long long sC, long long sS, hipStream_t st) {
  if (Cp % 8 != 0) {
    const long long total = (long long)N * Cp * S;
    const int grid = (int)std::min<long long>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(to_nhwc_generic_kernel, dim3(grid), dim3(256), 0, st, x, in_dtype, y, N, C, Cp,
                       S, sN, sC, sS);
    return;
  }
  const long long total = (long long)N * S * (Cp / 8);
  const int grid = (int)std::min<long long>((total + 255) / 256, 8192);
  if (total < (1LL << 31))
    hipLaunchKernelGGL(to_nhwc_pad_kernel<int>, dim3(grid), dim3(256), 0, st, x, in_dtype, y, N, C, Cp,
                       S, sN, sC, sS);
  else
    hipLaunchKernelGGL(to_nhwc_pad_kernel<long long>, dim3(grid), dim3(256), 0, st, x, in_dtype, y, N,
                       C, Cp, S, sN, sC, sS);
}

void channel_sum_launch(const bf16_t* x, long long P, int C, float* partial, int nblocks,
                        hipStream_t st) {
  hipLaunchKernelGGL(channel_sum_kernel, dim3(nblocks), dim3(256), 0, st, x, P, C, partial);
}

}  // namespace ddlpc
