// Store-granularity probe (MI355X): HBM write rate when every store instruction writes
// 64-lane x 16-B data as runs of CH contiguous bytes at a 1 KB row stride (the rest of each
// row written by the same wave's next instructions), CH = 64 .. 1024 (1024 = fully
// contiguous).  The convT / conv epilogues write 64-B runs (4 lanes x 16 B per pixel row).
//   hipcc -O3 --offload-arch=gfx950 scripts/store_probe.hip -o /tmp/store_probe && /tmp/store_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(256) void store_runs(u32x4* out, long long blocks_total) {
  constexpr int LPS = CH / 16;               // lanes per run
  constexpr int RPI = 64 / LPS;              // rows per instruction (1 KB rows)
  constexpr int IPB = 1024 / CH;             // instructions per block of RPI rows
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long long nwaves = (long long)gridDim.x * 4;
  const int r = lane / LPS, c = lane % LPS;
  const u32x4 v = {(unsigned)lane, 1u, 2u, 3u};
  for (long long b = wave; b < blocks_total; b += nwaves) {
    char* base = reinterpret_cast<char*>(out) + b * (long long)RPI * 1024;
#pragma unroll
    for (int i = 0; i < IPB; ++i)
      *reinterpret_cast<u32x4*>(base + r * 1024 + i * CH + c * 16) = v;
  }
}

template <int CH>
float run(u32x4* buf, long long bytes) {
  constexpr int RPI = 64 / (CH / 16);
  const long long blocks_total = bytes / (RPI * 1024LL);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  store_runs<CH><<<2048, 256>>>(buf, blocks_total);
  hipEventRecord(e0);
  for (int it = 0; it < 10; ++it) store_runs<CH><<<2048, 256>>>(buf, blocks_total);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  const long long bytes = 1LL << 29;         // 512 MiB (the 32^2 -> 64^2 up-sampling output)
  u32x4* buf = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  float t;
  t = run<64>(buf, bytes);   printf("CH   64 B runs: %8.1f us  %6.2f TB/s\n", t * 1e3, bytes / (t * 1e-3) / 1e12);
  t = run<128>(buf, bytes);  printf("CH  128 B runs: %8.1f us  %6.2f TB/s\n", t * 1e3, bytes / (t * 1e-3) / 1e12);
  t = run<256>(buf, bytes);  printf("CH  256 B runs: %8.1f us  %6.2f TB/s\n", t * 1e3, bytes / (t * 1e-3) / 1e12);
  t = run<1024>(buf, bytes); printf("CH 1024 B runs: %8.1f us  %6.2f TB/s\n", t * 1e3, bytes / (t * 1e-3) / 1e12);
  t = run<64>(buf, bytes);   printf("CH   64 B runs: %8.1f us  %6.2f TB/s (again)\n", t * 1e3, bytes / (t * 1e-3) / 1e12);
  hipFree(buf);
  return 0;
}
