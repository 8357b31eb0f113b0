// Micro-benchmark: can the LDS fragment reads of a 128 px x 64 ch wave tile hide under its MFMAs?
//
// One 8-wave workgroup per CU (two waves per SIMD), the streaming conv's wave tile
// (128 px x 64 ch, K = 32 per tap, 3 taps per stage, a barrier per stage), operands read
// from LDS as in csrc/conv3x3_fwd.hip (rolling fragment pipeline), in two MFMA shapes:
//   shape 0: v_mfma_f32_16x16x32_bf16, 8 x 4 tiles: per tap 12 ds_read_b128, 32 MFMAs (16 cyc)
//   shape 1: v_mfma_f32_32x32x16_bf16, 4 x 2 tiles: per tap 12 ds_read_b128, 16 MFMAs (32 cyc)
// and without the reads (operands from registers) for the MFMA-only rate.
//
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_lds_micro.hip -o mfma_lds_micro && ./mfma_lds_micro
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x4_t mfma16(const uint4& a, const uint4& b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x16_t mfma32(const uint4& a, const uint4& b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

constexpr int kLds = 64 * 1024;

template <int SHAPE, bool READS, int PRIO, int NWV = 8, int NT0 = 4, int XD0 = 4>
__global__ __launch_bounds__(NWV * 64, 1) void bench_kernel(float* out, int stages) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < kLds / 16; i += NWV * 64) {
    const unsigned h = i * 2654435761u;
    const unsigned v = (h & 0x007f007fu) | 0x3c003c00u;     // small random bf16 pairs
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(v, v ^ 0x00050003u, v ^ 0x00110007u, v ^ 0x00020009u);
  }
  __syncthreads();
  if (PRIO == 1 && wave >= 4) __builtin_amdgcn_s_setprio(1);
  // fragment f of a wave: 1 KB at ((f & 63) * 64 + lane) * 16, conflict-free
  auto rd = [&](int f) __attribute__((always_inline)) {
    return *reinterpret_cast<const uint4*>(smem + (((f & 63) * 64 + lane) << 4));
  };
  const uint4 c0 = make_uint4(0x3c003c01u + lane, 0x3c013c00u, 0x3c023c00u, 0x3c003c03u);
  float sum = 0.f;
  if constexpr (SHAPE == 0) {
    constexpr int MT = 8, NT = NT0, XD = XD0, NS = 3 * MT;
    f32x4_t acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < stages; ++s) {
      const int base = (s & 3) * 16 + wave;
      uint4 xf[XD], wf[2][NT];
      auto wload = [&](int tt, uint4 (&w)[NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) w[nt] = READS ? rd(base + 32 + tt * NT + nt) : c0;
      };
      wload(0, wf[0]);
#pragma unroll
      for (int q = 0; q < XD - 1; ++q) xf[q] = READS ? rd(base + q) : c0;
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        const int tt = st / MT, mt = st % MT;
        if (st + XD - 1 < NS) xf[(st + XD - 1) % XD] = READS ? rd(base + st + XD - 1) : c0;
        if (mt == 0 && tt + 1 < 3) wload(tt + 1, wf[(tt + 1) & 1]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16(wf[tt & 1][nt], xf[st % XD], acc[mt][nt]);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) sum += acc[i][j][0] + acc[i][j][3];
  } else {
    constexpr int MT = 4, NT = 2, NK = 6;                  // 3 taps x 2 k-steps of 16
    f32x16_t acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    for (int s = 0; s < stages; ++s) {
      const int base = (s & 3) * 16 + wave;
      uint4 xa[2][MT], wb[2][NT];
      auto load = [&](int k, uint4 (&x)[MT], uint4 (&w)[NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) x[mt] = READS ? rd(base + k * 6 + mt) : c0;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) w[nt] = READS ? rd(base + k * 6 + 4 + nt) : c0;
      };
      load(0, xa[0], wb[0]);
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        if (k + 1 < NK) load(k + 1, xa[(k + 1) & 1], wb[(k + 1) & 1]);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32(wb[k & 1][nt], xa[k & 1][mt], acc[mt][nt]);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) sum += acc[i][j][0] + acc[i][j][15];
  }
  out[blockIdx.x * 512 + tid] = sum;
}

template <int SHAPE, bool READS, int PRIO, int NWV = 8, int NT0 = 4, int XD0 = 4>
static void run(const char* name, float* out, int blocks, int stages) {
  auto kern = bench_kernel<SHAPE, READS, PRIO, NWV, NT0, XD0>;
  const size_t lds = 150 * 1024;                      // one workgroup per CU
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(NWV * 64), lds, 0, out, stages);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(NWV * 64), lds, 0, out, stages);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  // per stage per wave: 3 taps x 128 px x (16 NT) ch x 32 k x 2
  const double flops = (double)blocks * NWV * stages * 3 * 128.0 * (SHAPE == 0 ? 16 * NT0 : 64) * 32 * 2;
  printf("%-34s %8.3f ms  %7.1f TF/s  (%.1f ns per stage per workgroup)\n", name, best, flops / best / 1e9,
         best * 1e6 / ((double)stages * blocks / 256));
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 512 * sizeof(float));
  const int blocks = 256 * 4, stages = 2000;
  run<0, false, 0>("16x16x32, no reads", out, blocks, stages);
  run<0, true, 0>("16x16x32, rolling reads", out, blocks, stages);
  run<0, true, 1>("16x16x32, rolling reads, prio 4-7", out, blocks, stages);
  run<1, false, 0>("32x32x16, no reads", out, blocks, stages);
  run<1, true, 0>("32x32x16, double-buffered reads", out, blocks, stages);
  run<1, true, 1>("32x32x16, reads, prio 4-7", out, blocks, stages);
  run<0, false, 0, 4, 8, 3>("4 waves 128x128, no reads", out, blocks, stages);
  run<0, true, 0, 4, 8, 3>("4 waves 128x128, reads XD 3", out, blocks, stages);
  run<0, true, 0, 4, 8, 4>("4 waves 128x128, reads XD 4", out, blocks, stages);
  run<0, true, 0, 4, 8, 2>("4 waves 128x128, reads XD 2", out, blocks, stages);
  hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(hipGetLastError()));
  hipFree(out);
  return 0;
}
