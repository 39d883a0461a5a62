// sbag_well.h — Well19937c helpers shared by the Poisson samplers (sbag_kernels.hip
// k_poisson / k_poisson2 / k_poisson3, sbag_poisson.hip k_poisson4).
//
// Expanding commons-math3 AbstractWell.next / Well19937c.next, the only value a step
// needs from the step before it is z4 (AbstractWell's v0 = z4 of the previous step):
//   z4[n] = L(z4[n-1]) ^ c[n],  L(x) = x<<9 ^ x>>21 ^ (x & 0x7f)<<4,
// with c[n] a function of ring words written >= 70 steps earlier.
// L^K is applied as a XOR of shifted, masked copies of x, the masks built at compile time.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sbag {

__device__ __forceinline__ int wrap624(int x) { return x < 0 ? x + 624 : (x >= 624 ? x - 624 : x); }

// Well19937c's tempering, then next(26)
__device__ __forceinline__ uint32_t well_temper26(uint32_t z4) {
  z4 ^= (z4 << 7) & 0xe46e1700u;
  z4 ^= (z4 << 15) & 0x9b868000u;
  return z4 >> 6;  // next(26)
}

namespace wellsp {
__host__ __device__ constexpr uint32_t L1(uint32_t x) {
  return (x << 9) ^ (x >> 21) ^ ((x & 0x7Fu) << 4);
}
struct Masks {
  uint32_t m[63];  // m[s + 31]: input bits i with output bit i + s
};
constexpr Masks lpow_masks(int k) {
  Masks r{};
  for (int i = 0; i < 32; i++) {
    uint32_t x = 1u << i;
    for (int s = 0; s < k; s++) x = L1(x);
    for (int j = 0; j < 32; j++)
      if ((x >> j) & 1u) r.m[j - i + 31] |= 1u << i;
  }
  return r;
}
template <int K>
struct LP {
  static constexpr Masks M = lpow_masks(K);
};
// L^K(x) as a XOR of shifted, masked copies of x (zero terms vanish at compile time)
template <int K, int S = 0>
__device__ __forceinline__ uint32_t lpow(uint32_t x) {
  if constexpr (S == 63) {
    return 0u;
  } else {
    constexpr uint32_t m = LP<K>::M.m[S];
    constexpr int sh = S - 31;
    if constexpr (m == 0u)
      return lpow<K, S + 1>(x);
    else if constexpr (sh >= 0)
      return ((x & m) << sh) ^ lpow<K, S + 1>(x);
    else
      return ((x & m) >> (-sh)) ^ lpow<K, S + 1>(x);
  }
}
// three-input bitwise ops (gfx950 v_bitop3_b32; LUT index = a << 2 | b << 1 | c)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t andxor(uint32_t a, uint32_t m, uint32_t c) {  // (a & m) ^ c
  return __builtin_amdgcn_bitop3_b32(a, m, c, 0x6A);
}
// L(x) ^ c in five instructions: x<<9 ^ x>>21 ^ ((x<<4) & 0x7f0) ^ c
__device__ __forceinline__ uint32_t L1x(uint32_t x, uint32_t c) {
  return xor3(x << 9, x >> 21, andxor(x << 4, 0x7F0u, c));
}
// L^K(x) ^ acc: one shift and one and-xor per nonzero shift diagonal
// (((x & m) << s) == (x << s) & (m << s))
template <int K, int S = 0>
__device__ __forceinline__ uint32_t lpowx(uint32_t x, uint32_t acc) {
  if constexpr (S == 63) {
    return acc;
  } else {
    constexpr uint32_t m = LP<K>::M.m[S];
    constexpr int sh = S - 31;
    if constexpr (m == 0u)
      return lpowx<K, S + 1>(x, acc);
    else if constexpr (sh >= 0)
      return lpowx<K, S + 1>(x, andxor(x << sh, m << sh, acc));
    else
      return lpowx<K, S + 1>(x, andxor(x >> (-sh), m >> (-sh), acc));
  }
}
// Well19937c's tempering without the final >> 6
__device__ __forceinline__ uint32_t temper_raw(uint32_t z4) {
  z4 = andxor(z4 << 7, 0xe46e1700u, z4);
  return andxor(z4 << 15, 0x9b868000u, z4);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {  // lanes without a source read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
template <int LANE>
__device__ __forceinline__ double row_bcast(double x) {  // DPP row_newbcast:LANE
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x150 + LANE, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x150 + LANE, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
}  // namespace wellsp

}  // namespace sbag
