// Microbenchmark: fp64 accumulation into LDS cells owned by one lane (the fp64-label
// histogram's pattern, [bin][64 lanes] f64 layout): ds_add_f64 vs ds_add_u64 vs a plain
// read-add-write per entry (the lane owns its cells, so no atomicity is needed; LDS
// executes one wave's operations in order).  Cycles per wave-instruction (or per entry
// for the read-add-write) per CU.
// build: hipcc --offload-arch=gfx950 -O3 lds_f64.hip -o lds_f64
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int ITERS = 2048;
typedef __attribute__((address_space(3))) double lds_double;
typedef __attribute__((address_space(3))) unsigned long long lds_u64;

template <int MODE>
__global__ __launch_bounds__(256) void k(double* out) {
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // per wave: 32 bins x 64 lanes x 8 B = 16 KB
  lds_double* base = (lds_double*)smem + wave * 32 * 64;
  for (int i = lane; i < 32 * 64; i += 64) base[i] = 0.0;
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  const double w = 1.0 + lane * 1e-3;
  double acc = 0.0;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      x = x * 1664525u + 1013904223u;
      const uint32_t b = x >> 27;  // 0..31
      lds_double* p = base + b * 64 + lane;
      if (MODE == 0) __hip_atomic_fetch_add(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (MODE == 1)
        __hip_atomic_fetch_add((lds_u64*)p, (unsigned long long)x, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      if (MODE == 2) *p = *p + w;  // read, add, write (the lane owns the cell)
      if (MODE == 3) acc += *p;    // reads only
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = base[lane] + acc;
}

int main() {
  double* d;
  hipMalloc(&d, 1 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"ds_add_f64", "ds_add_u64", "read+add+write f64", "ds_read_b64"};
  for (int mode = 0; mode < 4; mode++) {
    for (int wgpc : {1, 2, 4, 8}) {  // 4 waves per workgroup: 4 .. 32 waves per CU
      const int blocks = 256 * wgpc;
      const size_t lds = 4 * 32 * 64 * 8;  // 64 KB
      auto f = mode == 0 ? k<0> : mode == 1 ? k<1> : mode == 2 ? k<2> : k<3>;
      hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (wgpc > 2) break;  // 64 KB per workgroup: at most 2 per CU
      hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, d);
      hipEventRecord(a);
      hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, d);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double instr_per_cu = (double)wgpc * 4 * ITERS * 4;
      printf("%-20s waves/cu=%2d  %.3f ms  %.2f cycles/wave-op/CU (2.4GHz)\n", names[mode],
             4 * wgpc, ms, ms * 1e-3 * 2.4e9 / instr_per_cu);
    }
  }
  return 0;
}
