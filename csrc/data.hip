// Device-side input pipeline — K20 of SURVEY.md §2.5 (input normalise + layout).
//
// Reference: every micro-batch is a host tensor `float32/255`, reshaped to NCHW and copied
// to the GPU (ref.py:737,741,754-755); the dataset is re-read from disk every epoch
// (ref.py:732).  Here the batch is produced directly in HBM, in the layout the first conv
// consumes (channel-last bf16, channels zero-padded to 8 = one 16-byte pixel for its
// LDS-DMA), by ONE kernel per batch:
//
//   * synth_tiles_kernel: the synthetic Vaihingen-shape generator (benchmark / no-data
//     source).  Sample i depends only on (seed, i): a counter-based hash (no RNG state),
//     so a batch is the same whichever rank, batch position or resume point renders it.
//     Recipe (the CPU twin in data/datasets.py computes the identical bits):
//       key     = mix(mix(seed ^ 0x9E3779B9) ^ i)
//       coarse  = mix(key ^ mix(cell + 0x632BE5AB)) % classes   on a grid^dims lattice
//       label   = coarse[(h*grid)/tile][(w*grid)/tile]           (nearest up-sampling)
//       u_j     = (mix(key ^ mix(p*8 + ch + 0x1B873593) + j*0x9E3779B9) >> 8) * 2^-24
//       x       = clamp(palette[label][ch] + (((u0+u1)+u2)+u3 - 2) * k, 0, 1)   -> bf16
//     (Irwin-Hall noise: k = noise*sqrt(3) gives std `noise`; every float op rounds on its
//     own — no FMA contraction — so the host twin matches bit for bit.)
//   * tile_gather_kernel: a real dataset uploaded ONCE to HBM as uint8 NHWC (+ uint8 label
//     maps): gather the batch's sample indices, /255 (IEEE division, as the reference's
//     numpy op), pad, bf16; labels widen to int64.
#include "common.h"
#include "ops.h"

namespace ddlpc {

namespace {

DDLPC_DEVICE uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

DDLPC_DEVICE float u24(uint32_t h) { return (float)(h >> 8) * (1.0f / 16777216.0f); }

// a separately rounded fp32 multiply: HIP's __fmul_rn is a plain operator that the default
// -ffp-contract=fast still fuses into the following add (the PyTorch twin rounds twice)
DDLPC_DEVICE float mul_rn(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// one thread per pixel; spatial = tile^dims pixels per sample, row-major (d, h, w).
// POW2 (tile a power of two and B * tile^dims < 2^31, the benchmark shapes): the pixel
// geometry by 32-bit shifts and masks instead of 64-bit divisions (which made the kernel
// ALU-bound: 230 us for a 384 x 256^2 batch); the same integers, so the same bits
template <bool POW2>
__global__ __launch_bounds__(256) void synth_tiles_kernel(
    const int64_t* __restrict__ idx, int B, uint32_t seed, int classes, int in_ch, int tile,
    int dims, int grid, float k, const float* __restrict__ palette, int cpad,
    bf16_t* __restrict__ x, int64_t* __restrict__ y) {
  const long long S = dims == 3 ? (long long)tile * tile * tile : (long long)tile * tile;
  const long long total = (long long)B * S;
  const uint32_t skey = mix32(seed ^ 0x9E3779B9u);
  const int lt = POW2 ? __builtin_ctz((unsigned)tile) : 0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    int b, w, h, d, cw, ch, cd;
    long long p;
    if constexpr (POW2) {
      const unsigned e32 = (unsigned)e, m = (unsigned)tile - 1u;
      b = (int)(e32 >> (lt * dims));
      p = (long long)(e32 & ((1u << (lt * dims)) - 1u));
      w = (int)(e32 & m);
      h = (int)((e32 >> lt) & m);
      d = dims == 3 ? (int)((e32 >> (2 * lt)) & m) : 0;
      cw = (w * grid) >> lt; ch = (h * grid) >> lt; cd = (d * grid) >> lt;
    } else {
      b = (int)(e / S);
      p = e - (long long)b * S;
      w = (int)(p % tile);
      const long long q = p / tile;
      h = (int)(q % tile);
      d = dims == 3 ? (int)(q / tile) : 0;
      cw = (w * grid) / tile; ch = (h * grid) / tile; cd = (d * grid) / tile;
    }
    const uint32_t key = mix32(skey ^ (uint32_t)idx[b]);
    const uint32_t cell = (uint32_t)((cd * grid + ch) * grid + cw);
    const int lab = (int)(mix32(key ^ mix32(cell + 0x632BE5ABu)) % (uint32_t)classes);
    y[e] = lab;
    float f[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float v = 0.f;
      if (c < in_ch) {
        const uint32_t base = key ^ mix32((uint32_t)(p * 8 + c) + 0x1B873593u);
        float s = u24(mix32(base));
        s = __fadd_rn(s, u24(mix32(base + 0x9E3779B9u)));
        s = __fadd_rn(s, u24(mix32(base + 2u * 0x9E3779B9u)));
        s = __fadd_rn(s, u24(mix32(base + 3u * 0x9E3779B9u)));
        const float n = mul_rn(__fadd_rn(s, -2.0f), k);
        v = fminf(fmaxf(__fadd_rn(palette[lab * in_ch + c], n), 0.f), 1.f);
      }
      f[c] = v;
    }
    if (cpad == 8) {
      reinterpret_cast<uint4*>(x)[e] = pack8(f);
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (c < cpad) x[e * cpad + c] = f2bf(f[c]);
    }
  }
}

__global__ __launch_bounds__(256) void tile_gather_kernel(
    const uint8_t* __restrict__ src, const uint8_t* __restrict__ lab, const int64_t* __restrict__ idx,
    int B, long long S, int in_ch, int cpad, long long N, bf16_t* __restrict__ x,
    int64_t* __restrict__ y) {
  const long long total = (long long)B * S;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(e / S);
    const long long p = e - (long long)b * S;
    const long long n = idx[b];
    // an out-of-range sample index reads nothing: zero image, label -100 (CrossEntropy's
    // ignore_index).  Host indices are range-checked by DeviceTileDataset.get first; device
    // indices cannot raise without a blocking read-back
    const bool in_range = n >= 0 && n < N;
    const long long sp = in_range ? n * S + p : 0;
    y[e] = in_range ? (int64_t)lab[sp] : (int64_t)-100;
    float f[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      f[c] = (c < in_ch && in_range) ? __fdiv_rn((float)src[sp * in_ch + c], 255.0f) : 0.f;
    if (cpad == 8) {
      reinterpret_cast<uint4*>(x)[e] = pack8(f);
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (c < cpad) x[e * cpad + c] = f2bf(f[c]);
    }
  }
}

int data_grid(long long total) {
  return (int)std::max<long long>(1, std::min<long long>((total + 255) / 256, 16384));
}

}  // namespace

void synth_tiles_launch(const int64_t* idx, int B, uint32_t seed, int classes, int in_ch, int tile,
                        int dims, int grid, float k, const float* palette, int cpad, bf16_t* x,
                        int64_t* y, hipStream_t st) {
  const long long S = dims == 3 ? (long long)tile * tile * tile : (long long)tile * tile;
  const bool pow2 = tile > 0 && (tile & (tile - 1)) == 0 && (long long)B * S < (1LL << 31);
  if (pow2)
    hipLaunchKernelGGL(synth_tiles_kernel<true>, dim3(data_grid(B * S)), dim3(256), 0, st, idx, B, seed,
                       classes, in_ch, tile, dims, grid, k, palette, cpad, x, y);
  else
    hipLaunchKernelGGL(synth_tiles_kernel<false>, dim3(data_grid(B * S)), dim3(256), 0, st, idx, B, seed,
                       classes, in_ch, tile, dims, grid, k, palette, cpad, x, y);
}

void tile_gather_launch(const uint8_t* src, const uint8_t* lab, const int64_t* idx, int B,
                        long long S, int in_ch, int cpad, long long N, bf16_t* x, int64_t* y,
                        hipStream_t st) {
  hipLaunchKernelGGL(tile_gather_kernel, dim3(data_grid(B * S)), dim3(256), 0, st, src, lab, idx, B,
                     S, in_ch, cpad, N, x, y);
}

}  // namespace ddlpc
