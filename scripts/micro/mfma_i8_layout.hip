// Probe: the A/B operand lane map of v_mfma_i32_32x32x32_i8 on gfx950, checked with exact
// integer data (asymmetric A and B).  Hypotheses for lane l (r = l & 31, h = l >> 5),
// element j = 0..15 of its 16 bytes:
//   H0: A[r][16h + j]                      (one contiguous 16-byte K run per lane half)
//   H1: A[r][8h + j] (j < 8), A[r][16 + 8h + j - 8] (j >= 8)   (two bf16-style K=16 halves)
// B likewise with B[k][col r].  C/D: col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h.
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/mfma_i8_layout mfma_i8_layout.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ int kmap(int hyp, int h, int j) {
  if (hyp == 0) return 16 * h + j;
  return j < 8 ? 8 * h + j : 16 + 8 * h + (j - 8);
}

__global__ void probe(const int8_t* A, const int8_t* B, int* D, int hyp) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; j++) {
    const int k = kmap(hyp, h, j);
    a[j] = A[r * 32 + k];  // A [32 rows][32 k]
    b[j] = B[k * 32 + r];  // B [32 k][32 cols]
  }
  v4i av, bv;
  for (int q = 0; q < 4; q++) {
    av[q] = (int)((uint32_t)(uint8_t)a[4 * q] | ((uint32_t)(uint8_t)a[4 * q + 1] << 8) |
                  ((uint32_t)(uint8_t)a[4 * q + 2] << 16) | ((uint32_t)(uint8_t)a[4 * q + 3] << 24));
    bv[q] = (int)((uint32_t)(uint8_t)b[4 * q] | ((uint32_t)(uint8_t)b[4 * q + 1] << 8) |
                  ((uint32_t)(uint8_t)b[4 * q + 2] << 16) | ((uint32_t)(uint8_t)b[4 * q + 3] << 24));
  }
  v16i c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int reg = 0; reg < 16; reg++) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    D[row * 32 + r] = c[reg];
  }
}

int main() {
  int8_t hA[32 * 32], hB[32 * 32];
  for (int i = 0; i < 32; i++)
    for (int k = 0; k < 32; k++) {
      hA[i * 32 + k] = (int8_t)(((i * 7 + k * 3) % 23) - 11);
      hB[i * 32 + k] = (int8_t)(((i * 5 + k * 11) % 19) - 9);  // B[k = i][col = k]
    }
  int ref[32 * 32];
  for (int i = 0; i < 32; i++)
    for (int j = 0; j < 32; j++) {
      int s = 0;
      for (int k = 0; k < 32; k++) s += hA[i * 32 + k] * hB[k * 32 + j];
      ref[i * 32 + j] = s;
    }
  int8_t *dA, *dB;
  int* dD;
  (void)hipMalloc(&dA, sizeof(hA));
  (void)hipMalloc(&dB, sizeof(hB));
  (void)hipMalloc(&dD, sizeof(ref));
  (void)hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  for (int hyp = 0; hyp < 2; hyp++) {
    (void)hipMemset(dD, 0, sizeof(ref));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, hyp);
    int out[32 * 32];
    (void)hipMemcpy(out, dD, sizeof(out), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32 * 32; i++) bad += out[i] != ref[i];
    printf("hypothesis H%d: %d of 1024 outputs differ\n", hyp, bad);
  }
  return 0;
}
