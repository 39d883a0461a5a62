// Probe: cycles per step of a lane-serial fp64 chain on gfx950 (one wave alone on a CU),
// the bound of k_fb_chain on long chains (the root's ~200k entries per bin).
//   mode 0: s1 += y; s2 += y*y           with y from registers (the add latency)
//   mode 1: the same with y read from LDS, 4 reads ahead (k_fb_chain's exploded loop)
//   mode 2: per entry (y, c) from LDS and a count loop (k_fb_chain's per-entry loop)
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o chain_lat chain_lat.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kN = 4096;

__global__ __launch_bounds__(64) void probe(int mode, int iters, double* out, long long* cyc) {
  __shared__ double s_y[kN];
  __shared__ uint8_t s_c[kN];
  const int lane = threadIdx.x;
  for (int i = lane; i < kN; i += 64) {
    s_y[i] = 1.0 + 1e-3 * i;
    s_c[i] = (uint8_t)(1 + (i * 7919 % 13 == 0) + (i * 104729 % 29 == 0));
  }
  __syncthreads();
  double s1 = 0.0, s2 = 0.0;
  uint64_t cnt = 0;
  const long long t0 = clock64();
  if (lane < 16) {
    for (int it = 0; it < iters; it++) {
      if (mode == 0) {
        double y = 1.0 + 1e-9 * it;
        for (int d = 0; d < kN; d++) {
          s1 += y;
          s2 += y * y;
          y += 1e-12;
        }
      } else if (mode == 1) {
        for (int d = 0; d < kN; d += 4) {
          const double y0 = s_y[d], y1 = s_y[d + 1], y2 = s_y[d + 2], y3 = s_y[d + 3];
          s1 += y0;
          s2 += y0 * y0;
          s1 += y1;
          s2 += y1 * y1;
          s1 += y2;
          s2 += y2 * y2;
          s1 += y3;
          s2 += y3 * y3;
        }
      } else {
        for (int d = 0; d < kN; d += 4) {
          const double y0 = s_y[d], y1 = s_y[d + 1], y2 = s_y[d + 2], y3 = s_y[d + 3];
          const uint32_t c0 = s_c[d], c1 = s_c[d + 1], c2 = s_c[d + 2], c3 = s_c[d + 3];
          auto add = [&](double y, uint32_t c) {
            const double wy = y * y;
            s1 += y;
            s2 += wy;
            for (uint32_t k = 1; k < c; k++) {
              s1 += y;
              s2 += wy;
            }
            cnt += c;
          };
          add(y0, c0);
          add(y1, c1);
          add(y2, c2);
          add(y3, c3);
        }
      }
    }
  }
  const long long t1 = clock64();
  if (lane == 0) *cyc = t1 - t0;
  out[lane] = s1 + s2 + (double)cnt;
}

int main() {
  double* d_out;
  long long* d_cyc;
  (void)hipMalloc(&d_out, 64 * sizeof(double));
  (void)hipMalloc(&d_cyc, sizeof(long long));
  const int iters = 20;
  for (int mode = 0; mode < 3; mode++) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, mode, iters, d_out, d_cyc);
    long long cyc = 0;
    (void)hipMemcpy(&cyc, d_cyc, sizeof(cyc), hipMemcpyDeviceToHost);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, mode, iters, d_out, d_cyc);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(&cyc, d_cyc, sizeof(cyc), hipMemcpyDeviceToHost);
    const double steps = (double)iters * kN;
    printf("mode %d: %.1f clock64 ticks per entry, %.2f ns per entry (event %.3f ms)\n", mode,
           cyc / steps, ms * 1e6 / steps, ms);
  }
  return 0;
}
