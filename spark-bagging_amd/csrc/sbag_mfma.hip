// sbag_mfma.hip — the root histogram as an int8 MFMA contraction (v_mfma_i32_32x32x32_i8).
//
// RandomForest.findBestSplits' first level aggregates every in-bag row of every replica:
// for shared bins that are the value codes (the synthetic C3 / C4 workloads, any dataset
// whose features have <= maxBins values and no subspace), the root histogram of replica r,
// feature f, bin b is
//
//     count[r][f][b] = sum_n c[r][n] [X[n][f] == b]
//     sum_k[r][f][b] = sum_n c[r][n] k'[n] [X[n][f] == b],   k' = k + K0 >= 0
//
// -- a dense contraction over the N rows of A = counts [R x N] (u8, <= 127: int8) with
// B = onehot(X[:, f]) [N x NB] and, for the label, B_j = onehot * digit_j(k') (7-bit digits
// of k', int8; and for the exact path's squares B_j = onehot * digit_j(k^2)).  One MFMA tile is 32 replicas x one feature's 32 bins x 32 rows; every
// plane's int32 accumulator stays exact for 65536 rows (127 * 127 * 65536 < 2^31), so a
// workgroup takes a 65536-row slice, 8 features (one per wave) and all replicas, and adds
// its exact int64 partials to the histogram with atomics.  A (the counts) is staged in
// LDS per 256-row chunk and shared by the 8 waves; each wave builds its B fragments in
// registers from its feature's column (the column-major copy k_transpose keeps with the
// dataset) with SWAR byte compares.  The sums are integers: the result is the k_hist_rl
// root histogram bit for bit, in any order.
//
// Reference: ml/ensemble/ensembleParams.scala:113-115 -> DecisionTreeRegressor.train ->
// RandomForest.findBestSplits (DTStatsAggregator over the bagged rows).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "sbag_internal.h"

namespace sbag {

namespace {
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kMfWaves = 8;          // features per workgroup
constexpr int kMfChunk = 256;        // rows per LDS chunk of A
constexpr int kMfPitch = kMfChunk + 16;  // LDS bytes per replica row (bank spread)
constexpr int64_t kMfSlice = 65536;  // rows per workgroup (int32 accumulators exact)

// 4 bytes x of a column vs bin b: 0x80 in every byte equal to b.  The last step
// ~(s | t) & 0x80808080 is one gfx950 v_bitop3_b32 (LUT index a << 2 | b << 1 | c; the
// compiler emitted or, not, and: the B fragments' VALU is what bounds this kernel, §4.8)
__device__ __forceinline__ uint32_t eq_hi(uint32_t x, uint32_t bb) {
  const uint32_t t = x ^ bb;
  const uint32_t s = (t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return __builtin_amdgcn_bitop3_b32(s, t, 0x80808080u, 0x02);
}
}  // namespace

// MT: 32-replica tiles (R <= 32 MT); ND: 7-bit digit planes (ND1 of k', the rest of k^2)
template <int MT, int ND>
__global__ __launch_bounds__(kMfWaves * 64, 1) void k_hist_mfma(MfmaHistArgs A) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nfg = (A.F + kMfWaves - 1) / kMfWaves;
  const int fg = (int)(blockIdx.x % (unsigned)nfg);
  const int64_t slice = blockIdx.x / (unsigned)nfg;
  const int f = fg * kMfWaves + wave;
  const bool fok = f < A.F;  // wave-uniform
  const int64_t n0 = slice * kMfSlice;
  const int64_t n1 = min(A.N, n0 + kMfSlice);
  const int RP = MT * 32;
  // LDS, two buffers of: A [RP][kMfPitch], the 8 columns [8][kMfChunk], the digits [ND][kMfChunk]
  constexpr int kBuf = MT * 32 * kMfPitch + (kMfWaves + ND) * kMfChunk;
  const uint32_t b = (uint32_t)(lane & 31), h = (uint32_t)(lane >> 5);
  const uint32_t bb = b * 0x01010101u;
  v16i acc[MT][1 + ND];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int q = 0; q <= ND; q++) acc[m][q] = v16i{};
  // a chunk is rows [c0, c0 + kMfChunk) in 16-byte pieces (N % 16 == 0): thread tid loads A
  // pieces tid + 512 i (replica p >> 4, rows 16 (p & 15)), then threads 0..127 one column piece
  // and threads 128.. one digit piece; replicas past R, rows past N and features past F are 0.
  // Loads go to registers first and reach LDS after the current chunk's MFMAs.
  uint4 ra[MT], rx = make_uint4(0, 0, 0, 0);
  auto prefetch = [&](int64_t c0) {
#pragma unroll
    for (int i = 0; i < MT; i++) {
      const int p = tid + kMfWaves * 64 * i, r = p >> 4;
      const int64_t row = c0 + 16 * (p & 15);
      const bool ok = r < A.R && row < n1;
      const uint4 v = *(const uint4*)(A.counts + (int64_t)min(r, A.R - 1) * A.N + min(row, n1 - 16));
      ra[i] = ok ? v : make_uint4(0, 0, 0, 0);
    }
    const int q = tid & 15, g = tid >> 4;
    const int64_t row = c0 + 16 * q;
    const unsigned char* src;
    bool ok;
    if (g < kMfWaves) {
      const int fx = fg * kMfWaves + g;
      ok = fx < A.F && row < n1;
      src = A.cols + (int64_t)min(fx, A.F - 1) * A.npad;
    } else {
      const int j = min(g - kMfWaves, ND > 0 ? ND - 1 : 0);
      ok = ND > 0 && g - kMfWaves < ND && row < n1;
      src = ND > 0 ? A.digits + (int64_t)j * A.N : A.cols;
    }
    const uint4 v = *(const uint4*)(src + min(row, n1 - 16));
    rx = ok ? v : make_uint4(0, 0, 0, 0);
  };
  auto commit = [&](int buf) {
    unsigned char* d = smem + buf * kBuf;
#pragma unroll
    for (int i = 0; i < MT; i++) {
      const int p = tid + kMfWaves * 64 * i;
      *(uint4*)(d + (p >> 4) * kMfPitch + 16 * (p & 15)) = ra[i];
    }
    const int g = tid >> 4;
    if (g < kMfWaves + ND) *(uint4*)(d + RP * kMfPitch + g * kMfChunk + 16 * (tid & 15)) = rx;
  };
  int buf = 0;
  prefetch(n0);
  commit(0);
  block_sync();
  for (int64_t c0 = n0; c0 < n1; c0 += kMfChunk) {
    const bool more = c0 + kMfChunk < n1;
    if (more) prefetch(c0 + kMfChunk);
    const unsigned char* cA = smem + buf * kBuf;
    const unsigned char* cX = cA + RP * kMfPitch + wave * kMfChunk;
    const unsigned char* cD = cA + RP * kMfPitch + kMfWaves * kMfChunk;
    if (fok) {
      // rows past N are zeros in LDS: the last chunk runs whole
#pragma unroll 2
      for (int ks = 0; ks < kMfChunk; ks += 32) {
        // B: the column's 16 rows of this lane half vs bin b (rows past N are 0 with 0 counts)
        const uint4 x = *(const uint4*)(cX + ks + 16 * h);
        // 0x01 (count plane) and 0xFF (digit mask) in every matching byte: from the 0x80
        // mask by a shift, and (hi - lo) | hi -- not (lo << 8) - lo, which the compiler
        // turns into a quarter-rate v_mul_lo_u32 by 255
        const uint32_t h0 = eq_hi(x.x, bb), h1 = eq_hi(x.y, bb), h2 = eq_hi(x.z, bb), h3 = eq_hi(x.w, bb);
        v4i be;
        be.x = (int)(h0 >> 7);
        be.y = (int)(h1 >> 7);
        be.z = (int)(h2 >> 7);
        be.w = (int)(h3 >> 7);
        v4i bd[ND > 0 ? ND : 1];
        if constexpr (ND > 0) {
          v4i ff;
          ff.x = (int)((h0 - (h0 >> 7)) | h0);
          ff.y = (int)((h1 - (h1 >> 7)) | h1);
          ff.z = (int)((h2 - (h2 >> 7)) | h2);
          ff.w = (int)((h3 - (h3 >> 7)) | h3);
#pragma unroll
          for (int j = 0; j < ND; j++) {
            const uint4 d = *(const uint4*)(cD + j * kMfChunk + ks + 16 * h);
            bd[j].x = ff.x & (int)d.x;
            bd[j].y = ff.y & (int)d.y;
            bd[j].z = ff.z & (int)d.z;
            bd[j].w = ff.w & (int)d.w;
          }
        }
#pragma unroll
        for (int m = 0; m < MT; m++) {
          const uint4 a4 = *(const uint4*)(cA + (m * 32 + (int)b) * kMfPitch + ks + 16 * h);
          const v4i a = v4i{(int)a4.x, (int)a4.y, (int)a4.z, (int)a4.w};
          acc[m][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, be, acc[m][0], 0, 0, 0);
#pragma unroll
          for (int j = 0; j < ND; j++)
            acc[m][1 + j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bd[j], acc[m][1 + j], 0, 0, 0);
        }
      }
    }
    if (more) commit(buf ^ 1);
    block_sync();  // the next chunk is in LDS; this one may be overwritten
    buf ^= 1;
  }
  if (!fok || (int)b >= A.NB) return;
  // D: col = lane & 31 (bin), row = (reg & 3) + 8 (reg >> 2) + 4 h (replica in the tile)
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int reg = 0; reg < 16; reg++) {
      const int r = m * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (int)h;
      if (r >= A.R) continue;
      const int64_t cnt = acc[m][0][reg];
      if (cnt == 0) continue;
      int64_t sk = 0, sq = 0;
#pragma unroll
      for (int j = 0; j < ND; j++) {
        const int64_t v = acc[m][1 + j][reg];
        if (j < A.ND1)
          sk += v * ((int64_t)1 << (A.dbits * j));  // (v may be negative: balanced digits)
        else
          sq += v << (7 * (j - A.ND1));
      }
      sk -= (int64_t)A.K0 * cnt;
      unsigned long long* w = A.hist + (((int64_t)r * A.Fmax + f) * A.NB + b) * 3;
      atomicAdd(&w[0], (unsigned long long)cnt);
      atomicAdd(&w[1], (unsigned long long)sk);
      if (ND > A.ND1) atomicAdd(&w[2], (unsigned long long)sq);
    }
}

size_t mfma_hist_lds_bytes(int R, int ND) {
  const int MT = (R + 31) / 32;
  return (size_t)2 * (MT * 32 * kMfPitch + (kMfWaves + ND) * kMfChunk);
}

template <int MT, int ND>
static void launch_mfma_t(hipStream_t st, const MfmaHistArgs& a, int nblk, size_t lds) {
  if constexpr (MT * (1 + ND) <= 12) {
    (void)hipFuncSetAttribute((const void*)k_hist_mfma<MT, ND>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL((k_hist_mfma<MT, ND>), dim3(nblk), dim3(kMfWaves * 64), lds, st, a);
  }
}

template <int MT>
static void launch_mfma_m(hipStream_t st, const MfmaHistArgs& a, int nblk, size_t lds) {
  switch (a.ND) {
    case 1: launch_mfma_t<MT, 1>(st, a, nblk, lds); break;
    case 2: launch_mfma_t<MT, 2>(st, a, nblk, lds); break;
    case 3: launch_mfma_t<MT, 3>(st, a, nblk, lds); break;
    case 4: launch_mfma_t<MT, 4>(st, a, nblk, lds); break;
    case 5: launch_mfma_t<MT, 5>(st, a, nblk, lds); break;
    default: launch_mfma_t<MT, 6>(st, a, nblk, lds); break;
  }
}

// replicas go in launches of at most MT tiles, MT (1 + ND) <= 10 accumulators (160 VGPRs at
// two waves per SIMD, no spills)
int mfma_hist_tiles(int ND) {
  // (12 accumulators -- all 128 C3 replicas in one launch -- spill at two waves per SIMD: root
  // frac 0.49 -> 0.38, profiles/r05logs/r05s/; SBAG_MFMA_ACC overrides)
  static const int acc = getenv("SBAG_MFMA_ACC") ? atoi(getenv("SBAG_MFMA_ACC")) : 10;
  return std::max(1, std::min(4, std::min(12, acc) / (1 + ND)));
}

bool launch_hist_mfma(hipStream_t st, const MfmaHistArgs& a) {
  if (a.R <= 0 || a.ND < 1 || a.ND > 6 || a.ND1 < 1 || a.ND1 > a.ND || a.NB > 32 || a.F <= 0 || a.N <= 0 || a.N % 16 != 0)
    return false;
  const int mtmax = mfma_hist_tiles(a.ND);
  const int nfg = (a.F + kMfWaves - 1) / kMfWaves;
  const int64_t slices = (a.N + kMfSlice - 1) / kMfSlice;
  const int nblk = (int)(slices * nfg);
  for (int r0 = 0; r0 < a.R; r0 += 32 * mtmax) {
    MfmaHistArgs g = a;
    g.R = std::min(a.R - r0, 32 * mtmax);
    g.counts = a.counts + (int64_t)r0 * a.N;
    g.hist = a.hist + (int64_t)r0 * a.Fmax * a.NB * 3;
    const int MT = (g.R + 31) / 32;
    const size_t lds = mfma_hist_lds_bytes(g.R, g.ND);
    switch (MT) {
      case 1: launch_mfma_m<1>(st, g, nblk, lds); break;
      case 2: launch_mfma_m<2>(st, g, nblk, lds); break;
      case 3: launch_mfma_m<3>(st, g, nblk, lds); break;
      default: launch_mfma_m<4>(st, g, nblk, lds); break;
    }
  }
  return true;
}

// the digits of k' = k + K0: unsigned 7-bit, plane j = (k' >> 7j) & 127 (k' >= 0), or
// balanced base 256 (int8 digits d_j in [-128, 127], k' = Σ d_j 256^j: each digit the low
// byte read as signed, the rest carried up); then those of k^2, plane nd1 + j =
// (k^2 >> 7j) & 127 (j < nd2)
__global__ __launch_bounds__(256) void k_label_digits(const int32_t* __restrict__ labk, int64_t N,
                                                      int32_t K0, int nd1, int nd2, int balanced,
                                                      uint8_t* __restrict__ digits) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256) {
    const int64_t k = labk[i];
    const uint64_t kp = (uint64_t)(k + K0), k2 = (uint64_t)((int64_t)k * k);
    if (balanced) {
      int64_t v = k + K0;
      for (int j = 0; j < nd1; j++) {
        const int64_t d = (int64_t)(int8_t)(uint8_t)(v & 0xFF);
        digits[(int64_t)j * N + i] = (uint8_t)d;
        v = (v - d) / 256;  // (exact)
      }
    } else {
      for (int j = 0; j < nd1; j++) digits[(int64_t)j * N + i] = (uint8_t)((kp >> (7 * j)) & 127u);
    }
    for (int j = 0; j < nd2; j++) digits[(int64_t)(nd1 + j) * N + i] = (uint8_t)((k2 >> (7 * j)) & 127u);
  }
}

void launch_label_digits(hipStream_t st, const int32_t* labk, int64_t N, int32_t K0, int nd1, int nd2,
                         uint8_t* digits, bool balanced) {
  if (nd1 + nd2 <= 0 || N <= 0) return;
  const int blocks = (int)std::min<int64_t>((N + 255) / 256, 256 * 8);
  hipLaunchKernelGGL(k_label_digits, dim3(blocks), dim3(256), 0, st, labk, N, K0, nd1, nd2, balanced ? 1 : 0,
                     digits);
}

}  // namespace sbag
