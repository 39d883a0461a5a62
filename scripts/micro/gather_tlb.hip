// Microbenchmark: random 128-B line gathers over growing footprints (0.5 .. 32 GiB).
// Does the rate fall once the footprint outgrows the GPU's TLB reach (C3 rows 1.28 GB,
// C5 6.4 GB, C4 25.6 GB)?  Mode "local": each wave's lines fall in one 64 MiB window
// that moves per workgroup, as when a level's nodes are walked in row order.
// build: hipcc --offload-arch=gfx950 -O3 gather_tlb.hip -o gather_tlb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <bool LOCAL>
__global__ __launch_bounds__(256) void k(const uint8_t* __restrict__ buf, uint64_t nline,
                                        int per_thread, uint32_t* out) {
  const int lane16 = threadIdx.x & 15;
  uint64_t x = (blockIdx.x * 256ull + threadIdx.x / 16) * 0x9E3779B97F4A7C15ull + 12345;
  const uint64_t win = (64ull << 20) / 128;  // lines per 64 MiB window
  const uint64_t base = LOCAL ? ((uint64_t)blockIdx.x * 2654435761ull % (nline / win)) * win : 0;
  uint32_t acc = 0;
#pragma unroll 8
  for (int i = 0; i < per_thread; i++) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    const uint64_t line = LOCAL ? base + ((x >> 20) % win) : ((x >> 20) % nline);
    const uint2 v = ((const uint2*)(buf + line * 128))[lane16];
    acc += v.x + v.y;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t maxb = 32ull << 30;
  uint8_t* buf;
  uint32_t* out;
  if (hipMalloc(&buf, maxb) != hipSuccess) return 1;
  hipMalloc(&out, 64);
  hipMemset(buf, 1, maxb);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = 256 * 16, per = 256;
  const double nl = (double)blocks * 16 * per;  // lines per launch
  for (int local = 0; local < 2; local++)
    for (size_t fp : {512ull << 20, 1ull << 30, 2ull << 30, 4ull << 30, 8ull << 30, 16ull << 30,
                      32ull << 30}) {
      auto f = local ? k<true> : k<false>;
      hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, buf, fp / 128, per, out);
      hipEventRecord(a);
      hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, buf, fp / 128, per, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("%s footprint %6.2f GiB: %.3f ms  %.2f G lines/s  %.0f GB/s\n",
             local ? "local " : "random", fp / 1073741824.0, ms, nl / ms / 1e6, nl * 128 / ms / 1e6);
    }
  return 0;
}
