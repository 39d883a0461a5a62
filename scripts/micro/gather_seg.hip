// Microbenchmark: random gather of 64-B vs 128-B row segments from a 2 GiB buffer
// (does a 64-B aligned half-line miss move 64 B or a whole 128-B line from HBM?).
// 16 lanes read one segment (dword per lane for 64 B, dwordx2 for 128 B).
// build: hipcc --offload-arch=gfx950 -O3 gather_seg.hip -o gather_seg
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int SEG>
__global__ __launch_bounds__(256) void k(const uint8_t* __restrict__ buf, uint64_t nseg_buf,
                                        int per_thread, uint32_t* out) {
  const int lane16 = threadIdx.x & 15;
  uint64_t x = (blockIdx.x * 256ull + threadIdx.x / 16) * 0x9E3779B97F4A7C15ull + 12345;
  uint32_t acc = 0;
#pragma unroll 8
  for (int i = 0; i < per_thread; i++) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    const uint64_t seg = (x >> 20) & (nseg_buf - 1);  // nseg_buf: power of two
    const uint8_t* p = buf + seg * SEG;
    if (SEG == 64) {
      acc += ((const uint32_t*)p)[lane16];
    } else {
      const uint2 v = ((const uint2*)p)[lane16];
      acc += v.x + v.y;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t bytes = 2ull << 30;
  uint8_t* buf;
  uint32_t* out;
  hipMalloc(&buf, bytes);
  hipMalloc(&out, 64);
  hipMemset(buf, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = 256 * 16, per = 256;
  const double nseg = (double)blocks * 16 * per;  // segments read per launch
  for (int rep = 0; rep < 2; rep++) {
    for (int seg : {64, 128}) {
      auto f = seg == 64 ? k<64> : k<128>;
      hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, buf, bytes / seg, per, out);
      hipEventRecord(a);
      hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, buf, bytes / seg, per, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("seg %3d B: %.3f ms  %.2f Gseg/s  %.0f GB/s useful\n", seg, ms, nseg / ms / 1e6,
             nseg * seg / ms / 1e6);
    }
  }
  return 0;
}
