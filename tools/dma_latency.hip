// Micro-benchmark: round-trip latency of LDS-DMA (buffer_load ... lds) vs register loads
// on gfx950, per wave, for L2-resident data, with N instructions in flight per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int N, int MODE>
__global__ void k(const char* src, unsigned bytes, unsigned long long* out, int iters, float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[64 * 1024];
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)bytes, 0x00020000);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned base = ((blockIdx.x * 4 + wave) * 16384u) % (bytes - 65536u);
  float acc = 0.f;
  unsigned long long t0 = clk();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const unsigned off = base + (i * 64 + lane) * 16u + (unsigned)it * 1024u % 8192u;
      if (MODE == 0) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)((size_t)(lds + (wave * N + i) % 64 * 1024)), 16,
            (int)off, 0, 0, 0);
      } else if (MODE == 1) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)((size_t)(lds + (wave * N + i) % 64 * 1024)), 16,
            (int)0x80000000u, 0, 0, 0);
      } else {
        float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
        acc += v.x;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  unsigned long long t1 = clk();
  if (lane == 0) out[blockIdx.x * 4 + wave] = (t1 - t0) / iters;
  if (acc == 1234.5f) sink[0] = acc;
}

template <int N, int MODE>
void run(const char* name, char* buf, unsigned bytes, int blocks) {
  unsigned long long* d;
  float* sink;
  hipMalloc(&d, blocks * 4 * 8);
  hipMalloc(&sink, 4);
  hipLaunchKernelGGL((k<N, MODE>), dim3(blocks), dim3(256), 0, 0, buf, bytes, d, 10, sink);
  hipLaunchKernelGGL((k<N, MODE>), dim3(blocks), dim3(256), 0, 0, buf, bytes, d, 200, sink);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), d, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (auto v : h) s += v;
  printf("%-28s N=%2d blocks=%4d : %8.0f cycles per round trip\n", name, N, blocks, s / h.size());
  hipFree(d);
  hipFree(sink);
}

int main() {
  char* buf;
  const unsigned bytes = 2u << 20;   // 2 MB: L2 resident
  hipMalloc(&buf, bytes);
  hipMemset(buf, 0, bytes);
  for (int blocks : {256, 512, 1024}) {
    run<1, 0>("lds-dma", buf, bytes, blocks);
    run<8, 0>("lds-dma", buf, bytes, blocks);
    run<8, 1>("lds-dma OOB", buf, bytes, blocks);
    run<1, 2>("buffer_load b128 (regs)", buf, bytes, blocks);
    run<8, 2>("buffer_load b128 (regs)", buf, bytes, blocks);
  }
  return 0;
}
