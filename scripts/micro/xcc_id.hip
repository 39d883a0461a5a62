// Probe: the XCC_ID hardware register (s_getreg, hwreg 20 on gfx940+) of each workgroup,
// against blockIdx.x % 8 (the round-robin dispatch over the 8 XCDs).
// Build: hipcc --offload-arch=gfx950 -O3 -o xcc_id xcc_id.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void probe(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = (int)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));
}

int main() {
  constexpr int n = 64;
  int* d;
  (void)hipMalloc(&d, n * sizeof(int));
  hipLaunchKernelGGL(probe, dim3(n), dim3(64), 0, 0, d);
  int h[n];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int match = 0;
  for (int i = 0; i < n; i++) {
    printf("%d%c", h[i], i % 16 == 15 ? '\n' : ' ');
    match += (h[i] & 7) == i % 8;
  }
  printf("blocks with xcc == blockIdx %% 8: %d of %d\n", match, n);
  return 0;
}
