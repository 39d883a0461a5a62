// Microbenchmark: LDS atomic / store throughput on gfx950 (cycles per wave-instruction per CU).
// build: hipcc --offload-arch=gfx950 -O3 lds_atomic.hip -o lds_atomic
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;

template <int MODE>
__global__ __launch_bounds__(512) void k(uint64_t* out, int wpl) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 65536 / 8; i += blockDim.x) ((uint64_t*)smem)[i] = 0;
  __syncthreads();
  // addresses: [bin][112 features] u64 layout, bins pseudo-random per lane and step
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  uint64_t acc = 0;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      x = x * 1664525u + 1013904223u;
      const uint32_t b = (x >> 27);  // 0..31
      const uint32_t addr = (b * 112 + lane) * 8;
      if (MODE == 0) atomicAdd((unsigned long long*)(smem + addr), (unsigned long long)x);
      if (MODE == 1) atomicAdd((uint32_t*)(smem + addr), x);
      if (MODE == 2) *(uint64_t*)(smem + addr) = x;
      if (MODE == 3) acc += *(volatile uint64_t*)(smem + addr);
      if (MODE == 4) atomicAdd((uint32_t*)(smem + (b * 128 + lane) * 4), x);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = ((uint64_t*)smem)[lane] + acc;
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 1 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"ds_add_u64", "ds_add_u32", "ds_write_b64", "ds_read_b64", "ds_add_u32 b*128"};
  for (int mode = 0; mode < 5; mode++) {
    for (int wgpc : {1, 2, 4}) {
      const int blocks = 256 * wgpc;
      const size_t lds = 160 * 1024 / wgpc - 1024;
      auto f = mode == 0 ? k<0> : mode == 1 ? k<1> : mode == 2 ? k<2> : mode == 3 ? k<3> : k<4>;
      hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipLaunchKernelGGL(f, dim3(blocks), dim3(512), lds, 0, d, 0);
      hipEventRecord(a);
      hipLaunchKernelGGL(f, dim3(blocks), dim3(512), lds, 0, d, 0);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double instr_per_cu = (double)wgpc * 8 * ITERS * 4;
      printf("%-18s wg/cu=%d  %.3f ms  %.2f cycles/wave-instr/CU (2.4GHz)\n", names[mode], wgpc, ms,
             ms * 1e-3 * 2.4e9 / instr_per_cu);
    }
  }
  return 0;
}
