// Deterministic two-pass row reductions of fp32 partial slabs into fp64 sums, plus the small
// finishing kernels that consume them (BatchNorm statistics / gradient coefficients, weight
// gradient transpose + accumulate).
//
// Every split-K / per-tile partial in the library (conv and transposed-conv weight-gradient
// slabs, BatchNorm sum / sum^2 rows, head-gradient rows, channel sums) is reduced here in a
// FIXED order: pass 1 sums row chunks of 64 (one thread per column, coalesced across the
// wave), pass 2 sums the chunk results.  No float atomics, so every data-parallel rank
// computes bit-identical local gradients from identical inputs.
#include "common.h"
#include "ops.h"

namespace ddlpc {

namespace {

constexpr int RB = 64;   // rows per chunk

template <typename T>
__global__ void rows_chunk_sum_kernel(const T* __restrict__ in, int R, long long N,
                                      double* __restrict__ out, long long ld = -1) {
  const long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (j >= N) return;
  if (ld < 0) ld = N;
  const int r0 = blockIdx.y * RB;
  const int r1 = min(R, r0 + RB);
  double s = 0.0;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += (double)in[(long long)r * ld + j];
  out[(long long)blockIdx.y * N + j] = s;
}

// running <- (1 - m) running + m x, in one fixed fp32 form: the deferred (per-micro-batch
// slot) updates of bn_running_apply_kernel reproduce the in-kernel ones bit for bit; with
// m = 1 a slot receives x exactly
DDLPC_DEVICE float bn_momentum_update(float running, float x, float m) {
  return fmaf(m, x, (1.f - m) * running);
}

// mean / invstd / scale / shift + running statistics from fp64 (sum, sum^2)
__global__ void bn_stats_finalize_kernel(const double* __restrict__ sums, int C, double count,
                                         const float* __restrict__ gamma,
                                         const float* __restrict__ beta, float* running_mean,
                                         float* running_var, float momentum, float eps,
                                         float* __restrict__ out4, int update_running,
                                         int64_t* nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && update_running && nbt != nullptr) nbt[0] += 1;
  if (c >= C) return;
  const double mean = sums[c] / count;
  double var = sums[C + c] / count - mean * mean;
  if (var < 0) var = 0;
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * inv;
  out4[c] = (float)mean;
  out4[C + c] = inv;
  out4[2 * C + c] = sc;
  out4[3 * C + c] = beta[c] - (float)mean * sc;
  if (update_running) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    running_mean[c] = bn_momentum_update(running_mean[c], (float)mean, momentum);
    running_var[c] = bn_momentum_update(running_var[c], (float)unb, momentum);
  }
}

// dgamma, dbeta (accumulated if requested) and dY coefficients from fp64 (sum dyh, sum dyh*xhat)
// (dscale: optional device factor on both sums — partials reduced at a unit gradient scale)
__global__ void bn_grad_finalize_kernel(const double* __restrict__ sums, int C, double count,
                                        const float* __restrict__ gamma,
                                        const float* __restrict__ invstd, float* dgamma,
                                        float* dbeta, float* coefs, int accumulate,
                                        const float* __restrict__ dscale) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double ds = dscale != nullptr ? (double)dscale[0] : 1.0;
  const double t1 = sums[c] * ds, t2 = sums[C + c] * ds;
  dbeta[c] = accumulate ? dbeta[c] + (float)t1 : (float)t1;
  dgamma[c] = accumulate ? dgamma[c] + (float)t2 : (float)t2;
  coefs[c] = gamma[c] * invstd[c];
  coefs[C + c] = (float)(t1 / count);
  coefs[2 * C + c] = (float)(t2 / count);
}

// dst[perm(j)] (+)= scale * sums[j]; perm: conv slab [co][tap][ci] -> OIHW [co][ci][tap]
// (mode 0), convT slab [ci][(sub, co)] -> IOHW [ci][co][sub] (mode 1), identity (mode 2)
__global__ void scatter_sums_kernel(const double* __restrict__ sums, long long N, float* dst,
                                    int mode, int A, int T, int B, float scale, int accumulate) {
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < N;
       j += (long long)gridDim.x * blockDim.x) {
    long long d = j;
    if (mode == 0) {          // A = Cout, T = taps, B = Cin ; j = (co*T + tap)*B + ci
      const int ci = (int)(j % B);
      const int tap = (int)((j / B) % T);
      const long long co = j / ((long long)B * T);
      d = (co * B + ci) * T + tap;
    } else if (mode == 1) {   // A = Cin, T = subs, B = Cout ; j = ci*(T*B) + sub*B + co
      const int co = (int)(j % B);
      const int sub = (int)((j / B) % T);
      const long long ci = j / ((long long)B * T);
      d = (ci * B + co) * T + sub;
    }
    const float v = (float)sums[j] * scale;
    dst[d] = accumulate ? dst[d] + v : v;
  }
}

// dst[j] (+)= sums[j] * dscale[0]  (identity layout; device-side scale)
__global__ void scatter_sums_dscale_kernel(const double* __restrict__ sums, long long N, float* dst,
                                           const float* __restrict__ dscale, int accumulate) {
  const double ds = (double)dscale[0];
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < N;
       j += (long long)gridDim.x * blockDim.x) {
    const float v = (float)(sums[j] * ds);
    dst[j] = accumulate ? dst[j] + v : v;
  }
}

// deferred running-statistics updates (concurrent micro-batch streams): K slots of
// (batch mean, unbiased batch var) written by K forwards with momentum 1, applied here in
// micro-batch order — the sequence of updates the K forwards would have made one by one
__global__ void bn_running_apply_kernel(float* __restrict__ running_mean, float* __restrict__ running_var,
                                        const float* __restrict__ slots, int K, int C, long long stride,
                                        float momentum, int64_t* nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt != nullptr) nbt[0] += K;
  if (c >= C) return;
  float rm = running_mean[c], rv = running_var[c];
  for (int k = 0; k < K; ++k) {                   // slot k: [mean (C) | var (C)] at k * stride
    rm = bn_momentum_update(rm, slots[k * stride + c], momentum);
    rv = bn_momentum_update(rv, slots[k * stride + C + c], momentum);
  }
  running_mean[c] = rm;
  running_var[c] = rv;
}

// head gradient scale dL/count from the loss kernel's (loss, correct, count) and the incoming
// dL (null: 1) — one thread; replaces a handful of tiny elementwise launches per step
__global__ void head_grad_scale_kernel(const float* __restrict__ out3, const float* __restrict__ gs,
                                       float* __restrict__ scale) {
  if (threadIdx.x != 0) return;
  const float cnt = out3[2];
  scale[0] = (gs != nullptr ? gs[0] : 1.f) / (cnt > 0.f ? cnt : 1.f);
}

// training meter [sum loss, sum correct, sum pixels, micro-batches] += (loss * n, correct,
// pixels, n): n micro-batches whose mean loss is `loss` (a batched window counts n)
__global__ void meter_add_kernel(double* __restrict__ buf, const float* __restrict__ loss,
                                 const float* __restrict__ correct, double pixels, double n) {
  const int t = threadIdx.x;
  if (t == 0) buf[0] += (double)loss[0] * n;
  else if (t == 1) buf[1] += (double)correct[0];
  else if (t == 2) buf[2] += pixels;
  else if (t == 3) buf[3] += n;
}

// one block per channel: fp64 sum of P partial rows, then finalize (P <= a few thousand)
DDLPC_DEVICE void block_sum2(double& a, double& b) {
  __shared__ double r1[4], r2[4];
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  if ((threadIdx.x & 63) == 0) { r1[threadIdx.x >> 6] = a; r2[threadIdx.x >> 6] = b; }
  __syncthreads();
  a = r1[0] + r1[1] + r1[2] + r1[3];
  b = r2[0] + r2[1] + r2[2] + r2[3];
}

__global__ void bn_stats_rows_kernel(const float* __restrict__ partial, int P, int C, double count,
                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                     float* running_mean, float* running_var, float momentum,
                                     float eps, float* __restrict__ out4, int update_running,
                                     int64_t* nbt) {
  const int c = blockIdx.x;
  double a = 0.0, b = 0.0;
  for (int r = threadIdx.x; r < P; r += 256) {
    a += partial[(long long)r * 2 * C + c];
    b += partial[(long long)r * 2 * C + C + c];
  }
  block_sum2(a, b);
  if (threadIdx.x != 0) return;
  if (c == 0 && update_running && nbt != nullptr) nbt[0] += 1;
  const double mean = a / count;
  double var = b / count - mean * mean;
  if (var < 0) var = 0;
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * inv;
  out4[c] = (float)mean;
  out4[C + c] = inv;
  out4[2 * C + c] = sc;
  out4[3 * C + c] = beta[c] - (float)mean * sc;
  if (update_running) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    running_mean[c] = bn_momentum_update(running_mean[c], (float)mean, momentum);
    running_var[c] = bn_momentum_update(running_var[c], (float)unb, momentum);
  }
}

__global__ void bn_grad_rows_kernel(const float* __restrict__ partial, int P, int C, double count,
                                    const float* __restrict__ gamma,
                                    const float* __restrict__ invstd, float* dgamma, float* dbeta,
                                    float* coefs, int accumulate, const float* __restrict__ dscale) {
  const int c = blockIdx.x;
  double a = 0.0, b = 0.0;
  for (int r = threadIdx.x; r < P; r += 256) {
    a += partial[(long long)r * 2 * C + c];
    b += partial[(long long)r * 2 * C + C + c];
  }
  block_sum2(a, b);
  if (threadIdx.x != 0) return;
  if (dscale != nullptr) { a *= (double)dscale[0]; b *= (double)dscale[0]; }
  dbeta[c] = accumulate ? dbeta[c] + (float)a : (float)a;
  dgamma[c] = accumulate ? dgamma[c] + (float)b : (float)b;
  coefs[c] = gamma[c] * invstd[c];
  coefs[C + c] = (float)(a / count);
  coefs[2 * C + c] = (float)(b / count);
}

// final pass fused with the scatter/accumulate into the destination gradient
template <typename T>
__global__ void rows_sum_scatter_kernel(const T* __restrict__ in, int R, long long N, float* dst,
                                        int mode, int A, int Tt, int B, int accumulate,
                                        long long ld) {
  const long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (j >= N) return;
  double s = 0.0;
#pragma unroll 8
  for (int r = 0; r < R; ++r) s += (double)in[(long long)r * ld + j];
  long long d = j;
  if (mode == 0) {
    const int ci = (int)(j % B);
    const int tap = (int)((j / B) % Tt);
    const long long co = j / ((long long)B * Tt);
    d = (co * B + ci) * Tt + tap;
  } else if (mode == 1) {
    const int co = (int)(j % B);
    const int sub = (int)((j / B) % Tt);
    const long long ci = j / ((long long)B * Tt);
    d = (ci * B + co) * Tt + sub;
  }
  const float v = (float)s;
  dst[d] = accumulate ? dst[d] + v : v;
}

// one-launch form for R > 64 rows (the two-pass pair costs a second >= 4.5 us launch): a
// block of kWideWaves waves owns 64 columns, wave w sums the rows r = w (mod kWideWaves) of
// them (coalesced 256-B row segments), and wave 0 adds the partials in a fixed order
// (deterministic); optional permuted scatter / accumulate into the fp32 destination.
// Four waves, not sixteen: these reductions run on the weight-gradient stream next to the
// persistent data-gradient kernels, and a 1024-thread block (four waves on every SIMD of one
// CU) waited for a wholly free CU — 300-570 us per launch in the two-stream trace against
// 8-15 us alone (profiles/r5/tail_img_wgrad_main_g64_g65/)
constexpr int kWideWaves = 4;
template <bool SCATTER>
__global__ __launch_bounds__(64 * kWideWaves) void rows_sum_wide_kernel(const float* __restrict__ in, int R,
                                                                        long long N, long long ld,
                                                                        double* __restrict__ sums, float* dst,
                                                                        int mode, int A, int Tt, int B,
                                                                        int accumulate) {
  __shared__ double red[kWideWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long j = blockIdx.x * 64LL + lane;
  double s = 0.0;
  if (j < N) {
#pragma unroll 4
    for (int r = w; r < R; r += kWideWaves) s += (double)in[(long long)r * ld + j];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w != 0 || j >= N) return;
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < kWideWaves; ++k) t += red[k][lane];
  if (!SCATTER) { sums[j] = t; return; }
  long long d = j;
  if (mode == 0) {
    const int ci = (int)(j % B);
    const int tap = (int)((j / B) % Tt);
    const long long co = j / ((long long)B * Tt);
    d = (co * B + ci) * Tt + tap;
  } else if (mode == 1) {
    const int co = (int)(j % B);
    const int sub = (int)((j / B) % Tt);
    const long long ci = j / ((long long)B * Tt);
    d = (ci * B + co) * Tt + sub;
  }
  const float v = (float)t;
  dst[d] = accumulate ? dst[d] + v : v;
}

// (up to 64 rows per wave: longer serial chains lose to the two-pass form — measured 22 us vs
// 2 x 5 us for the head's 4096-row, 198-column reduction)
constexpr int kWideMaxRows = 1024;

}  // namespace

void bn_stats_finalize_rows_launch(const float* partial, int P, int C, double count,
                                   const float* gamma, const float* beta, float* running_mean,
                                   float* running_var, float momentum, float eps, float* out4,
                                   bool update_running, int64_t* nbt, hipStream_t st) {
  hipLaunchKernelGGL(bn_stats_rows_kernel, dim3(C), dim3(256), 0, st, partial, P, C, count, gamma,
                     beta, running_mean, running_var, momentum, eps, out4, update_running ? 1 : 0,
                     nbt);
}

void bn_grad_finalize_rows_launch(const float* partial, int P, int C, double count,
                                  const float* gamma, const float* invstd, float* dgamma,
                                  float* dbeta, float* coefs, bool accumulate, hipStream_t st,
                                  const float* dscale) {
  hipLaunchKernelGGL(bn_grad_rows_kernel, dim3(C), dim3(256), 0, st, partial, P, C, count, gamma,
                     invstd, dgamma, dbeta, coefs, accumulate ? 1 : 0, dscale);
}

// dst (+)= permute(sum over rows of in[R][N]); one pass when R <= 64, else chunk sums first
void reduce_rows_scatter_launch(const float* in, int R, long long N, double* tmp, float* dst,
                                int mode, int A, int T, int B, bool accumulate, hipStream_t st,
                                long long ld) {
  const unsigned gx = (unsigned)((N + 255) / 256);
  if (ld < 0) ld = N;
  if (R <= 64) {
    hipLaunchKernelGGL(rows_sum_scatter_kernel<float>, dim3(gx), dim3(256), 0, st, in, R, N, dst,
                       mode, A, T, B, accumulate ? 1 : 0, ld);
    return;
  }
  if (R <= kWideMaxRows) {
    hipLaunchKernelGGL(rows_sum_wide_kernel<true>, dim3((unsigned)((N + 63) / 64)), dim3(64 * kWideWaves), 0, st, in,
                       R, N, ld, nullptr, dst, mode, A, T, B, accumulate ? 1 : 0);
    return;
  }
  const int RC = (R + RB - 1) / RB;
  hipLaunchKernelGGL(rows_chunk_sum_kernel<float>, dim3(gx, RC), dim3(256), 0, st, in, R, N, tmp, ld);
  hipLaunchKernelGGL(rows_sum_scatter_kernel<double>, dim3(gx), dim3(256), 0, st, tmp, RC, N, dst,
                     mode, A, T, B, accumulate ? 1 : 0, N);
}

int reduce_rows_chunks(int R) { return (R + RB - 1) / RB; }

// sums[N] (fp64) = sum over R rows of in[R][N]; tmp must hold reduce_rows_chunks(R) * N doubles
void reduce_rows_launch(const float* in, int R, long long N, double* tmp, double* sums,
                        hipStream_t st) {
  const int RC = reduce_rows_chunks(R);
  const unsigned gx = (unsigned)((N + 255) / 256);
  if (RC == 1) {
    hipLaunchKernelGGL(rows_chunk_sum_kernel<float>, dim3(gx, 1), dim3(256), 0, st, in, R, N, sums, -1LL);
    return;
  }
  if (R <= kWideMaxRows) {
    hipLaunchKernelGGL(rows_sum_wide_kernel<false>, dim3((unsigned)((N + 63) / 64)), dim3(64 * kWideWaves), 0, st, in,
                       R, N, N, sums, nullptr, 2, 0, 0, 0, 0);
    return;
  }
  hipLaunchKernelGGL(rows_chunk_sum_kernel<float>, dim3(gx, RC), dim3(256), 0, st, in, R, N, tmp, -1LL);
  int R2 = RC;
  const double* cur = tmp;
  while (reduce_rows_chunks(R2) > 1) {       // (only for > 4096 rows)
    const int RC2 = reduce_rows_chunks(R2);
    double* nxt = tmp + (long long)RC * N;   // second half of tmp is free scratch
    hipLaunchKernelGGL(rows_chunk_sum_kernel<double>, dim3(gx, RC2), dim3(256), 0, st, cur, R2, N, nxt, -1LL);
    cur = nxt;
    R2 = RC2;
  }
  hipLaunchKernelGGL(rows_chunk_sum_kernel<double>, dim3(gx, 1), dim3(256), 0, st, cur, R2, N, sums, -1LL);
}

void bn_stats_finalize_launch(const double* sums, int C, double count, const float* gamma,
                              const float* beta, float* running_mean, float* running_var,
                              float momentum, float eps, float* out4, bool update_running,
                              int64_t* nbt, hipStream_t st) {
  hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, sums, C,
                     count, gamma, beta, running_mean, running_var, momentum, eps, out4,
                     update_running ? 1 : 0, nbt);
}

void bn_grad_finalize_launch(const double* sums, int C, double count, const float* gamma,
                             const float* invstd, float* dgamma, float* dbeta, float* coefs,
                             bool accumulate, hipStream_t st, const float* dscale) {
  hipLaunchKernelGGL(bn_grad_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, sums, C,
                     count, gamma, invstd, dgamma, dbeta, coefs, accumulate ? 1 : 0, dscale);
}

void scatter_sums_dscale_launch(const double* sums, long long N, float* dst, const float* dscale,
                                bool accumulate, hipStream_t st) {
  const int grid = (int)std::max<long long>(1, std::min<long long>((N + 255) / 256, 4096));
  hipLaunchKernelGGL(scatter_sums_dscale_kernel, dim3(grid), dim3(256), 0, st, sums, N, dst, dscale,
                     accumulate ? 1 : 0);
}

// every BatchNorm of the network in ONE launch (blockIdx.y = layer): entries [L][4] =
// (running_mean*, running_var*, num_batches_tracked* or 0, C | column offset << 32) into an
// arena of K rows (row stride `stride` floats); same arithmetic and order as
// bn_running_apply_kernel
__global__ void bn_running_apply_all_kernel(const int64_t* __restrict__ entries, const float* __restrict__ arena,
                                            int K, long long stride, float momentum) {
  const int64_t* e = entries + 4 * blockIdx.y;
  float* running_mean = reinterpret_cast<float*>(e[0]);
  float* running_var = reinterpret_cast<float*>(e[1]);
  int64_t* nbt = reinterpret_cast<int64_t*>(e[2]);
  const int C = (int)(e[3] & 0xffffffff);
  const long long off = (long long)((uint64_t)e[3] >> 32);
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt != nullptr) nbt[0] += K;
  if (c >= C) return;
  const float* slots = arena + off;
  float rm = running_mean[c], rv = running_var[c];
  for (int k = 0; k < K; ++k) {
    rm = bn_momentum_update(rm, slots[k * stride + c], momentum);
    rv = bn_momentum_update(rv, slots[k * stride + C + c], momentum);
  }
  running_mean[c] = rm;
  running_var[c] = rv;
}

void bn_running_apply_all_launch(const int64_t* entries, int L, int maxC, const float* arena, int K,
                                 long long stride, float momentum, hipStream_t st) {
  hipLaunchKernelGGL(bn_running_apply_all_kernel, dim3((maxC + 255) / 256, L), dim3(256), 0, st, entries,
                     arena, K, stride, momentum);
}

void bn_running_apply_launch(float* rm, float* rv, const float* slots, int K, int C, long long stride,
                             float momentum, int64_t* nbt, hipStream_t st) {
  hipLaunchKernelGGL(bn_running_apply_kernel, dim3((C + 255) / 256), dim3(256), 0, st, rm, rv, slots, K,
                     C, stride, momentum, nbt);
}

void head_grad_scale_launch(const float* out3, const float* gs, float* scale, hipStream_t st) {
  hipLaunchKernelGGL(head_grad_scale_kernel, dim3(1), dim3(64), 0, st, out3, gs, scale);
}

// a bucket all-reduce's memory footprint without a peer: `passes` read + write-back sweeps
// (values unchanged: the empty asm keeps the compiler from folding the store of a just-
// loaded value), 16-byte accesses, each workgroup on its own contiguous slice
__global__ __launch_bounds__(256) void comm_proxy_kernel(float* __restrict__ g, long long n, int passes) {
  const long long n4 = n / 4;
  const long long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long long lo = blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  for (int p = 0; p < passes; ++p) {
    for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      float4 v = reinterpret_cast<float4*>(g)[i];
      asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
      reinterpret_cast<float4*>(g)[i] = v;
    }
  }
}

void comm_proxy_launch(float* g, long long n, int blocks, int passes, hipStream_t st) {
  hipLaunchKernelGGL(comm_proxy_kernel, dim3(std::max(1, blocks)), dim3(256), 0, st, g, n, passes);
}

void meter_add_launch(double* buf, const float* loss, const float* correct, double pixels,
                      double n, hipStream_t st) {
  hipLaunchKernelGGL(meter_add_kernel, dim3(1), dim3(64), 0, st, buf, loss, correct, pixels, n);
}

void scatter_sums_launch(const double* sums, long long N, float* dst, int mode, int A, int T,
                         int B, float scale, bool accumulate, hipStream_t st) {
  const int grid = (int)std::max<long long>(1, std::min<long long>((N + 255) / 256, 4096));
  hipLaunchKernelGGL(scatter_sums_kernel, dim3(grid), dim3(256), 0, st, sums, N, dst, mode, A, T,
                     B, scale, accumulate ? 1 : 0);
}

}  // namespace ddlpc
