// Microbenchmark: LDS ds_add_u64 / ds_add_u32 throughput of histogram address patterns
// (cycles per wave-instruction per CU).
//   lanes   lane = feature (k_hist's layout: 64 distinct features, random bins)
//   rl G    lane = (entry lane/G, feature (lane%G)*K + j): G features x 64/G entries
// bins uniform in [0, 32) or skewed (half the draws are bin 0).
// build: hipcc --offload-arch=gfx950 -O3 lds_rl.hip -o lds_rl
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 32768;

template <bool U64, int G, int K>
__global__ __launch_bounds__(512) void k(uint64_t* out, int FPH, int skew) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 40960 / 8; i += blockDim.x) ((uint64_t*)smem)[i] = 0;
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x * 97u;
  constexpr uint32_t WB = U64 ? 8 : 4;
  const uint32_t fbase = (G ? (uint32_t)(lane % G) * K : (uint32_t)lane) * WB;
  const uint32_t amul = (uint32_t)FPH * WB;
  const uint32_t smask = skew ? 0xffffffffu : 0u;
  for (int it = 0; it < ITERS / K; it++) {
#pragma unroll
    for (int j = 0; j < K; j++) {
      x = x * 1664525u + 1013904223u;
      // skew: half the draws (bit 26 set) land in bin 0
      const uint32_t b = (x >> 27) & ~(((x << 5) >> 31) * smask);
      const uint32_t addr = b * amul + fbase + (G ? j * WB : 0u);
      if (U64)
        atomicAdd((unsigned long long*)(smem + addr), (unsigned long long)x);
      else
        atomicAdd((uint32_t*)(smem + addr), x);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = ((uint64_t*)smem)[lane];
}

template <bool U64, int G, int K>
static void run(uint64_t* d, int FPH, int skew, hipEvent_t a, hipEvent_t b) {
  const int wgpc = 2, blocks = 256 * wgpc;
  const size_t lds = 40960;
  auto f = k<U64, G, K>;
  hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(512), lds, 0, d, FPH, skew);
  hipEventRecord(a);
  hipLaunchKernelGGL(f, dim3(blocks), dim3(512), lds, 0, d, FPH, skew);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double instr_per_cu = (double)wgpc * 8 * (ITERS / K) * K;
  printf("%s skew=%d G=%2d K=%2d FPH=%3d  %.3f ms  %.2f cycles/wave-instr/CU\n",
         U64 ? "ds_add_u64" : "ds_add_u32", skew, G, K, FPH, ms, ms * 1e-3 * 2.4e9 / instr_per_cu);
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 1 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int skew = 0; skew < 2; skew++)
    for (int fph : {112, 113}) {
      run<true, 0, 8>(d, fph, skew, a, b);
      run<true, 4, 25>(d, fph, skew, a, b);
      run<true, 8, 13>(d, fph, skew, a, b);
      run<true, 16, 7>(d, fph, skew, a, b);
      run<false, 0, 8>(d, fph, skew, a, b);
      run<false, 4, 25>(d, fph, skew, a, b);
      run<false, 8, 13>(d, fph, skew, a, b);
    }
  return 0;
}
