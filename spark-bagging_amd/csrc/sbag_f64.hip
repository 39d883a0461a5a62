// sbag_f64.hip — gfx950 kernels for bagging regression on arbitrary fp64 labels.
//
// The integer engine (sbag_kernels.hip) needs dyadic labels: its histogram sums are exact
// integers, so their order does not matter.  For any other double the reference's result
// depends on the order: Spark's DTStatsAggregator.update adds every exploded row (a row
// drawn c times is c consecutive rows, sql/bfunctions.scala:42-44) to its (node, feature,
// bin) cell in row order, in fp64 (count += 1, sum += 1 * y, sumSq += 1 * y * y).  These
// kernels reproduce those sums bit for bit:
//
//   k_chunk_inbag / k_chunk_scan / k_compact_ordered  the bootstrap of each replica:
//                     one entry (row, count, fixed-point label) per in-bag row, in row
//                     order (a stable compaction); a row drawn c times adds its label c
//                     times in a row
//   k_f64_hist        one wave per (node, group of <= 64 features); lane = feature owns
//                     that feature's NB cells in LDS and walks the node's entries in row
//                     order, adding each row's label with LDS fp64 atomics (ds_add_f64):
//                     one lane's adds to one cell execute in issue order, so the sum is
//                     the sequential fp64 sum, while the wave never waits on a result
//   k_f64_split       RandomForest.binsToBestSplit in Spark's operation order, one wave
//                     per node, lane = feature (mergeForFeature prefixes, right = total -
//                     left, calculateImpurityStats, first max over splits then features)
//   (the stable partition of a split node's entries is k_fb_scatter's, sbag_f64s.hip)
//
// Reference call sites: ml/ensemble/ensembleParams.scala:113-115 (fitBaseLearner ->
// DecisionTreeRegressor.train), ml/regression/BaggingRegressor.scala:146-150,179-185.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "sbag_internal.h"

namespace sbag {

namespace {

__device__ __forceinline__ int f64_wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// block-wide exclusive scan of one int per thread (256 threads); returns the exclusive
// prefix and writes the block total to *total
__device__ __forceinline__ int block_excl_scan256(int v, int* s_wave, int* total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int incl = f64_wave_incl_scan(v, lane);
  if (lane == 63) s_wave[wave] = incl;
  block_sync();
  int before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    if (w < wave) before += s_wave[w];
    tot += s_wave[w];
  }
  block_sync();
  *total = tot;
  return before + incl - v;
}

constexpr int kChunkRows = 8192;

}  // namespace

// ---------------------------------------------------------------- ordered compaction
// The fp64 path keeps every replica's in-bag rows in row order (Spark adds a node's rows to
// its fp64 sums in that order): one entry row | (k << 8 | count) << 32 per in-bag row, k the
// labels' fixed-point image for the integer screening histograms (a row drawn c times is c
// consecutive rows in Spark, sql/bfunctions.scala:42-44: its label is added c times).
// per (replica, 8192-row chunk): in-bag rows; per replica Σ count and max count
__global__ __launch_bounds__(256) void k_chunk_inbag(const uint8_t* __restrict__ counts, int64_t N,
                                                     int R, int64_t chunks,
                                                     uint32_t* __restrict__ ncnt,
                                                     unsigned long long* __restrict__ wsum,
                                                     unsigned int* __restrict__ cmax) {
  const int r = blockIdx.x % R;
  const int64_t chunk = blockIdx.x / R;
  const uint8_t* cr = counts + (int64_t)r * N;
  unsigned int s = 0, m = 0, n = 0;
  const uint8_t* cc = cr + chunk * kChunkRows;
  if ((chunk + 1) * kChunkRows <= N && (((uintptr_t)cc) & 15) == 0) {
    // 16 counts per load: Σ by v_sad_u8, the nonzero bytes by (b & 0x7f) + 0x7f | b, the max
    // bytewise
    for (int k = threadIdx.x; k < kChunkRows / 16; k += 256) {
      const uint4 v = ((const uint4*)cc)[k];
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t w = w4[q];
        s = __builtin_amdgcn_sad_u8(w, 0u, s);
        n += (uint32_t)__builtin_popcount((((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u);
        m = max(m, max(max(w & 0xFFu, (w >> 8) & 0xFFu), max((w >> 16) & 0xFFu, w >> 24)));
      }
    }
  } else {
    for (int it = 0; it < kChunkRows / 256; it++) {
      const int64_t row = chunk * kChunkRows + it * 256 + threadIdx.x;
      if (row < N) {
        const unsigned int c = cr[row];
        s += c;
        n += c ? 1u : 0u;
        m = max(m, c);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_down(s, o);
    n += __shfl_down(n, o);
    m = max(m, (unsigned int)__shfl_down((int)m, o));
  }
  __shared__ unsigned int s_s[4], s_m[4], s_n[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_s[wave] = s;
    s_m[wave] = m;
    s_n[wave] = n;
  }
  block_sync();
  if (threadIdx.x == 0) {
    const unsigned int t = s_s[0] + s_s[1] + s_s[2] + s_s[3];  // <= 8192 * 255
    ncnt[(int64_t)r * chunks + chunk] = s_n[0] + s_n[1] + s_n[2] + s_n[3];
    if (t) atomicAdd(&wsum[r], (unsigned long long)t);
    const unsigned int mm = max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3]));
    if (mm) atomicMax(&cmax[r], mm);
  }
}

// per (replica, 8192-row chunk): in-bag rows only (the entry capacity's pre-count on the
// integer path), 16 counts per load: a byte is nonzero iff (b & 0x7f) + 0x7f or b has bit 7
__global__ __launch_bounds__(256) void k_chunk_rows(const uint8_t* __restrict__ counts, int64_t N,
                                                    int R, int64_t chunks, uint32_t* __restrict__ ncnt) {
  const int r = blockIdx.x % R;
  const int64_t chunk = blockIdx.x / R;
  const uint8_t* cr = counts + (int64_t)r * N + chunk * kChunkRows;
  const int64_t nrow = min((int64_t)kChunkRows, N - chunk * kChunkRows);
  uint32_t n = 0;
  auto nz = [](uint32_t w) {
    return (uint32_t)__builtin_popcount((((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u);
  };
  if (nrow == kChunkRows && (((uintptr_t)cr) & 15) == 0) {
    for (int k = threadIdx.x; k < kChunkRows / 16; k += 256) {
      const uint4 v = ((const uint4*)cr)[k];
      n += nz(v.x) + nz(v.y) + nz(v.z) + nz(v.w);
    }
  } else {
    for (int64_t k = threadIdx.x; k < nrow; k += 256) n += cr[k] ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o);
  __shared__ uint32_t s_n[4];
  if ((threadIdx.x & 63) == 0) s_n[threadIdx.x >> 6] = n;
  block_sync();
  if (threadIdx.x == 0) ncnt[(int64_t)r * chunks + chunk] = s_n[0] + s_n[1] + s_n[2] + s_n[3];
}

void launch_chunk_rows(hipStream_t st, const uint8_t* counts, int64_t N, int R, uint32_t* d_ncnt) {
  const int64_t chunks = compact_ordered_chunks(N);
  hipLaunchKernelGGL(k_chunk_rows, dim3((unsigned)(chunks * R)), dim3(256), 0, st, counts, N, R, chunks, d_ncnt);
}

// per replica: exclusive prefix of the chunks' entries; cursor[r] = the total
__global__ __launch_bounds__(256) void k_chunk_scan(const uint32_t* __restrict__ ncnt, int64_t chunks,
                                                    unsigned long long* __restrict__ base,
                                                    unsigned long long* __restrict__ cursor) {
  __shared__ int s_wave[4];
  const int r = blockIdx.x;
  unsigned long long carry = 0;
  for (int64_t k0 = 0; k0 < chunks; k0 += 256) {
    const int64_t k = k0 + threadIdx.x;
    const int v = k < chunks ? (int)ncnt[(int64_t)r * chunks + k] : 0;
    int tot;
    const int ex = block_excl_scan256(v, s_wave, &tot);
    if (k < chunks) base[(int64_t)r * chunks + k] = carry + (unsigned long long)ex;
    carry += (unsigned long long)tot;
  }
  if (threadIdx.x == 0) cursor[r] = carry;
}

// one entry per in-bag row, in row order.  STG: the block's entries of an iteration (and
// their labels), contiguous in the output, are staged in LDS and stored by consecutive
// threads, instead of each thread's up to 4 entries at its own scattered positions
template <bool STG>
__global__ __launch_bounds__(256) void k_compact_ordered(const uint8_t* __restrict__ counts,
                                                         const int32_t* __restrict__ labk, int64_t N,
                                                         int R, int64_t chunks,
                                                         const unsigned long long* __restrict__ base,
                                                         uint64_t* __restrict__ ent, int64_t cap,
                                                         const double* __restrict__ y,
                                                         double* __restrict__ ey) {
  __shared__ int s_wave[4];
  const int r = blockIdx.x % R;
  const int64_t chunk = blockIdx.x / R;
  const uint8_t* cr = counts + (int64_t)r * N;
  uint64_t* er = ent + (int64_t)r * cap;
  double* eyr = ey ? ey + (int64_t)r * cap : nullptr;  // (the carried fp64 labels, same positions)
  unsigned long long pos0 = base[(int64_t)r * chunks + chunk];
  __shared__ uint64_t s_e[STG ? 1024 : 1];
  __shared__ double s_y[STG ? 1024 : 1];
  const bool vec = ((N | (int64_t)(uintptr_t)cr) & 3) == 0;
  for (int it = 0; it < kChunkRows / 1024; it++) {
    const int64_t row0 = chunk * kChunkRows + (int64_t)it * 1024 + (int64_t)threadIdx.x * 4;
    uint32_t c[4];
    int n = 0;
    if (vec && row0 + 3 < N) {
      const uint32_t w = *(const uint32_t*)(cr + row0);
#pragma unroll
      for (int j = 0; j < 4; j++) c[j] = (w >> (8 * j)) & 0xffu;
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) c[j] = row0 + j < N ? cr[row0 + j] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) n += c[j] ? 1 : 0;
    int tot;
    const int ex = block_excl_scan256(n, s_wave, &tot);
    if (STG) {
      int lp = ex;
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (c[j]) {
          if (eyr) s_y[lp] = y[row0 + j];
          s_e[lp++] = pack_entry((uint32_t)(row0 + j), labk[row0 + j], c[j]);
        }
      block_sync();
      for (int q = threadIdx.x; q < tot; q += 256) {
        er[pos0 + q] = s_e[q];
        if (eyr) eyr[pos0 + q] = s_y[q];
      }
      block_sync();  // (the staging is rewritten by the next iteration)
    } else {
      unsigned long long pos = pos0 + (unsigned long long)ex;
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (c[j]) {
          if (eyr) eyr[pos] = y[row0 + j];
          er[pos++] = pack_entry((uint32_t)(row0 + j), labk[row0 + j], c[j]);
        }
    }
    pos0 += (unsigned long long)tot;
  }
}

void launch_chunk_draws(hipStream_t st, const uint8_t* counts, int64_t N, int R, uint32_t* d_ncnt,
                        unsigned long long* d_wsum, unsigned int* d_cmax) {
  const int64_t chunks = compact_ordered_chunks(N);
  hipLaunchKernelGGL(k_chunk_inbag, dim3((unsigned)(chunks * R)), dim3(256), 0, st, counts, N, R,
                     chunks, d_ncnt, d_wsum, d_cmax);
}

void launch_compact_ordered(hipStream_t st, const uint8_t* counts, const int32_t* labk, int64_t N,
                            int R, uint64_t* ent, int64_t cap, const uint32_t* d_ncnt,
                            unsigned long long* d_base, unsigned long long* d_cursor, const double* y,
                            double* ey) {
  const int64_t chunks = compact_ordered_chunks(N);
  hipLaunchKernelGGL(k_chunk_scan, dim3(R), dim3(256), 0, st, d_ncnt, chunks, d_base, d_cursor);
  static const bool stg = !getenv("SBAG_COMPACT_STG") || atoi(getenv("SBAG_COMPACT_STG")) != 0;  // (A/B)
  if (stg)
    hipLaunchKernelGGL(k_compact_ordered<true>, dim3((unsigned)(chunks * R)), dim3(256), 0, st, counts, labk,
                       N, R, chunks, d_base, ent, cap, y, ey);
  else
    hipLaunchKernelGGL(k_compact_ordered<false>, dim3((unsigned)(chunks * R)), dim3(256), 0, st, counts, labk,
                       N, R, chunks, d_base, ent, cap, y, ey);
}

int64_t compact_ordered_chunks(int64_t N) { return (N + kChunkRows - 1) / kChunkRows; }

// ---------------------------------------------------------------- row-order fp64 histogram
// LDS per wave: count u32 [NB][W] at byte 0, then sum and sumSq interleaved as f64
// [NB][2][W] (sum of lane l at bin k: 16·W·k + 8·l, its sumSq 8·W bytes further), W = 64
// lanes (32 when NB > 128 would not fit 160 KB).  Lane fl < Fr owns feature fl's cells,
// lane Fr (when in this group) the node total at bin 0, lanes past the group their own
// bin-0 cells (never read back).  A cell address is one 24-bit multiply-add, bin · M +
// lane offset, M = 0 for the total and the idle lanes.
//
// The wave walks the node's entries (one per in-bag row, compaction above; a row drawn c
// times adds its label c times in a row, its count c at once) two batches of 64
// at a time: lane i holds entry i and its label, and the bins of the next batch are
// gathered one per entry of the current one, right after that entry's atomics, so each
// gather has ~63 entries of work to land in (the most the 6-bit vmcnt counter tracks).
// Both batches of an iteration are one basic block and the bins are consumed exactly as
// loaded: any operation between a gather and its use (a mask, a widening the compiler
// sinks to the use or folds through the loop phi, a rotation copy) would wait on every
// gather in flight.  Per entry: two readlanes (the label), its square, two cell
// addresses, the LDS atomics and the next gather.  The node's last iteration runs whole:
// entries past the end repeat the last entry with label y[N] = +0.0 (an exact no-op for
// the sums, which start at +0.0 and so never become -0.0), and their count increments are
// taken back from the last row's cells after the walk.  (This kernel is now the fallback of
// the screened engine, sbag_f64s.hip: it histograms the nodes whose split the screen could
// not decide, and every node under SBAG_F64_SCREEN=0.)
//
// Parts: at shallow levels (few nodes, few waves) a (node, group) is split over two
// waves, one adding count and sum, the other sumSq: the two walks run in parallel and
// each issues part of the LDS atomics (the walk is the level's critical path there).
constexpr int kF64Batch = 64;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) double lds_double;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

template <int PART, int W>
__device__ __forceinline__ void f64_add_entry(lds_char* L, double y, uint32_t cnt, uint32_t bin, int j,
                                              uint32_t M1, uint32_t lo1, uint32_t M2, uint32_t lo2,
                                              bool act) {
  const uint64_t yb = (uint64_t)__double_as_longlong(y);
  const int ylo = __builtin_amdgcn_readlane((int)(uint32_t)yb, j);
  const int yhi = __builtin_amdgcn_readlane((int)(uint32_t)(yb >> 32), j);
  // the row's draw count (wave-uniform): Spark adds its exploded copies one after another
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cnt, j);
  const double v = __longlong_as_double((long long)(((uint64_t)(uint32_t)yhi << 32) | (uint32_t)ylo));
  const double w = 1.0 * v;   // instanceWeight * label
  if (W < 64 && !act) return;  // lanes past W hold no cells
  lds_double* s = (lds_double*)(L + (__umul24(bin, M1) + lo1));
  for (uint32_t k = 0; k < c; k++) {
    if (PART != 2) __hip_atomic_fetch_add(s, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (PART != 1)  // instanceWeight * label * label (its own array in part 2)
      __hip_atomic_fetch_add(PART == 2 ? s : s + W, w * v, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (PART != 2)
    __hip_atomic_fetch_add((lds_u32*)(L + (__umul24(bin, M2) + lo2)), c, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int PART, int W, bool BUF>
__device__ __forceinline__ void f64_hist_body(const F64HistArgs& A, const F64Node& nd, int group) {
  extern __shared__ double lds[];
  lds_char* L = (lds_char*)lds;
  const int lane = threadIdx.x;
  const int Fr = A.Fr[nd.r];
  const int f0 = group * A.FPW;
  const int fl = f0 + lane;
  const bool feat = lane < A.FPW && lane < W && fl < Fr;
  const bool tot = lane < A.FPW && lane < W && fl == Fr;
  const int NB = A.NB;
  // part 0: counts, then sum and sumSq interleaved; part 1: counts, then sums; part 2:
  // sumSq only
  const uint32_t B1 = PART == 2 ? 0u : (uint32_t)NB * W * 4;
  const uint32_t F64W = PART == 0 ? 2u : 1u;  // f64 arrays per bin row
  for (uint32_t k = lane * 4; k < B1 + (uint32_t)NB * W * 8 * F64W; k += 256) *(lds_u32*)(L + k) = 0u;
  block_sync();
  const int64_t a = nd.a, b = nd.b;
  if (a < b) {
    const bool act = lane < W;
    const uint32_t M1 = feat ? 8u * F64W * W : 0u, M2 = feat ? 4u * W : 0u;
    const uint32_t lo1 = B1 + 8u * (uint32_t)lane, lo2 = 4u * (uint32_t)lane;
    const uint8_t* bins_r = A.bins + (int64_t)nd.r * A.bins_rstride;
    // lanes without a feature read column 0 (valid memory) and multiply it by 0
    const uint32_t posl = feat ? (uint32_t)A.pos[(int64_t)nd.r * A.Fmax + fl] : 0u;
    const uint64_t S = (uint64_t)A.S;
    const uint32_t S32 = (uint32_t)A.S;
    const int64_t last = b - 1;
    // BUF: a replica's bins below 4 GB, a buffer load with the row offset in a scalar
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)bins_r, (short)0, (int)A.bins_bytes, 0x00020000);
    auto ld_row_bin = [&](uint32_t row) -> uint32_t {
      if (BUF) return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, posl, row * S32, 0);
      return (uint32_t)bins_r[(uint64_t)row * S + posl];
    };
    auto ld_bin = [&](uint64_t e, int j) -> uint32_t {
      return ld_row_bin((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)e, j));
    };
    auto ld_entry = [&](int64_t base) -> uint64_t { return A.ent[min(base + lane, last)]; };
    auto ld_y = [&](int64_t base, uint64_t e) -> double {
      return A.y[base + lane <= last ? (uint32_t)e : A.yzero];
    };
    auto cnt_of = [](uint64_t e) -> uint32_t { return (uint32_t)(e >> 32) & 0xffu; };
    // even batches: eE, yE, cE, bE; odd batches: eO, yO, cO, bO -- each updated in place
    uint64_t eE = ld_entry(a), eO = ld_entry(a + kF64Batch);
    double yE = ld_y(a, eE), yO = ld_y(a + kF64Batch, eO);
    uint32_t cE = cnt_of(eE), cO = cnt_of(eO);
    uint32_t bE[kF64Batch], bO[kF64Batch];
    // (the prologue's bins pass through an opaque xor, so the loop phi is not a widening
    // the compiler could fold to the top of the loop)
#pragma unroll
    for (int j = 0; j < kF64Batch; j++) bE[j] = ld_bin(eE, j) ^ A.zero;
    int64_t base = a;
    for (;; base += 2 * kF64Batch) {
      // batch k (bE, yE): gather batch k + 1's bins, fetch batch k + 2's entries
      eE = ld_entry(base + 2 * kF64Batch);
#pragma unroll
      for (int j = 0; j < kF64Batch; j++) {
        f64_add_entry<PART, W>(L, yE, cE, bE[j], j, M1, lo1, M2, lo2, act);
        bO[j] = ld_bin(eO, j);
        __builtin_amdgcn_sched_barrier(0);  // keep each gather next to its entry
      }
      yE = ld_y(base + 2 * kF64Batch, eE);
      cE = cnt_of(eE);
      // batch k + 1 (bO, yO): gather batch k + 2's bins, fetch batch k + 3's entries
      eO = ld_entry(base + 3 * kF64Batch);
#pragma unroll
      for (int j = 0; j < kF64Batch; j++) {
        f64_add_entry<PART, W>(L, yO, cO, bO[j], j, M1, lo1, M2, lo2, act);
        bE[j] = ld_bin(eE, j);
        __builtin_amdgcn_sched_barrier(0);
      }
      yO = ld_y(base + 3 * kF64Batch, eO);
      cO = cnt_of(eO);
      if (base + 2 * kF64Batch >= b) break;
    }
    // the padding [b, base + 128) repeated the last entry: its count went to the last
    // row's cells once per padding entry (its sums added +0.0)
    const uint32_t pad = (uint32_t)(base + 2 * kF64Batch - b);
    if (PART != 2 && pad != 0u && act) {
      const uint64_t el = A.ent[last];
      const uint32_t bl = ld_row_bin((uint32_t)el);
      __hip_atomic_fetch_sub((lds_u32*)(L + (__umul24(bl, M2) + lo2)), pad * cnt_of(el),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  block_sync();
  if (feat || tot) {
    double* out = A.hist + ((int64_t)blockIdx.x * (A.Fmax + 1) + fl) * NB * 3;
    const int nbk = tot ? 1 : NB;
    const lds_u32* cn = (const lds_u32*)L;
    const lds_double* s12 = (const lds_double*)(L + B1);
    for (int k = 0; k < nbk; k++) {
      if (PART != 2) {
        out[3 * k] = (double)cn[k * W + lane];
        out[3 * k + 1] = s12[F64W * k * W + lane];
      }
      if (PART != 1) out[3 * k + 2] = s12[(F64W * k + F64W - 1) * W + lane];
    }
  }
}

// grid (nodes, groups * parts): blockIdx.y = group * parts + part
template <int W, bool BUF>
__global__ __launch_bounds__(64) void k_f64_hist(F64HistArgs A) {
  const F64Node nd = A.nodes[blockIdx.x];
  const int group = (int)blockIdx.y / A.parts;
  const int part = (int)blockIdx.y % A.parts;
  if (group * A.FPW > A.Fr[nd.r]) return;  // past the node's features and total
  if (A.parts == 1)
    f64_hist_body<0, W, BUF>(A, nd, group);
  else if (part == 0)
    f64_hist_body<1, W, BUF>(A, nd, group);
  else
    f64_hist_body<2, W, BUF>(A, nd, group);
}

int f64_hist_width(int NB) { return (size_t)NB * 64 * 20 <= 160 * 1024 ? 64 : 32; }
// per wave: 20 B a cell (count, sum, sumSq), 12 B when split in parts (count + sum | sumSq)
size_t f64_hist_lds_bytes(int NB, int parts) {
  return (size_t)NB * f64_hist_width(NB) * (parts == 1 ? 20 : 12);
}

template <int W, bool BUF>
static void launch_f64_hist_t(hipStream_t st, const F64HistArgs& a, dim3 grid, size_t lds) {
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)k_f64_hist<W, BUF>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  hipLaunchKernelGGL((k_f64_hist<W, BUF>), grid, dim3(64), lds, st, a);
}

void launch_f64_hist(hipStream_t st, const F64HistArgs& a, int nnodes, int ngroups) {
  const size_t lds = f64_hist_lds_bytes(a.NB, a.parts);
  const dim3 grid(nnodes, ngroups * a.parts);
  const bool buf = a.bins_bytes != 0;
  if (f64_hist_width(a.NB) == 64) {
    if (buf)
      launch_f64_hist_t<64, true>(st, a, grid, lds);
    else
      launch_f64_hist_t<64, false>(st, a, grid, lds);
  } else {
    if (buf)
      launch_f64_hist_t<32, true>(st, a, grid, lds);
    else
      launch_f64_hist_t<32, false>(st, a, grid, lds);
  }
}

// ---------------------------------------------------------------- split (binsToBestSplit)
namespace {
__device__ __forceinline__ double var_impurity(double count, double sum, double sumsq) {
  if (count == 0) return 0.0;  // Variance.calculate
  const double squared_loss = sumsq - (sum * sum) / count;
  return squared_loss / count;
}
constexpr double kMinValue = -1.7976931348623157e308;  // Double.MinValue
}  // namespace

// hist [q][Fmax + 1][NB][3]: the node's per-feature bin stats (and its total at Fmax... at
// local index Fr).  Each lane takes features fl = lane, lane + 64, ...; per feature it
// forms the prefixes in bin order (mergeForFeature), evaluates every split against the
// node's chain state and keeps the first max; the wave then takes the first max over
// features (lowest index on ties).  At the root the chain state is the first candidate's
// left + right of the first feature with splits (calculateImpurityStats, stats == null).
__global__ __launch_bounds__(64) void k_f64_split(F64SplitArgs A) {
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  const F64Node nd = A.nodes[q];
  const int r = nd.r;
  const int Fr = A.Fr[r];
  const int NB = A.NB;
  const double* h = A.hist + (int64_t)q * (A.Fmax + 1) * NB * 3;
  const int32_t* nbins = A.nbins + (int64_t)r * A.Fmax;
  const F64Chain ch = A.chain[q];
  double pc0 = ch.calc[0], pc1 = ch.calc[1], pc2 = ch.calc[2], pimp = ch.impurity;
  if (!ch.set) {
    // first feature with splits; its first candidate fixes the parent
    int f0 = -1;
    for (int k = 0; k < Fr; k++)
      if (nbins[k] > 1) {
        f0 = k;
        break;
      }
    if (f0 >= 0) {
      const double* fa = h + (int64_t)f0 * NB * 3;
      const int nsp = nbins[f0] - 1;
      double t0 = 0, t1 = 0, t2 = 0;  // prefix through bin nsp, in bin order
      for (int s = 0; s <= nsp; s++) {
        if (s == 0) {
          t0 = fa[0];
          t1 = fa[1];
          t2 = fa[2];
        } else {
          t0 += fa[3 * s];
          t1 += fa[3 * s + 1];
          t2 += fa[3 * s + 2];
        }
      }
      const double l0 = fa[0], l1 = fa[1], l2 = fa[2];
      const double r0 = t0 - l0, r1 = t1 - l1, r2 = t2 - l2;
      pc0 = l0 + r0;
      pc1 = l1 + r1;
      pc2 = l2 + r2;
      pimp = var_impurity(pc0, pc1, pc2);
    }
  }
  double best_gain = 0.0;
  int best_f = -1, best_s = -1, best_valid = 0;
  const uint8_t* fm = A.fmask ? A.fmask + (int64_t)q * A.Fmax : nullptr;
  for (int fl = lane; fl < Fr; fl += 64) {
    const int nsp = nbins[fl] - 1;
    if (nsp <= 0 || (fm && !fm[fl])) continue;
    const double* fa = h + (int64_t)fl * NB * 3;
    double t0 = fa[0], t1 = fa[1], t2 = fa[2];
    for (int s = 1; s <= nsp; s++) {
      t0 += fa[3 * s];
      t1 += fa[3 * s + 1];
      t2 += fa[3 * s + 2];
    }
    double c0 = 0, c1 = 0, c2 = 0;
    double fg = 0.0;
    int fs = -1, fv = 0;
    for (int s = 0; s < nsp; s++) {
      if (s == 0) {
        c0 = fa[0];
        c1 = fa[1];
        c2 = fa[2];
      } else {
        c0 += fa[3 * s];
        c1 += fa[3 * s + 1];
        c2 += fa[3 * s + 2];
      }
      const double r0 = t0 - c0, r1 = t1 - c1, r2 = t2 - c2;
      const int64_t lc = (int64_t)c0, rc = (int64_t)r0;
      double gain;
      int valid;
      if (lc < A.min_inst || rc < A.min_inst) {
        gain = kMinValue;
        valid = 0;
      } else {
        const int64_t total = lc + rc;
        const double li = var_impurity(c0, c1, c2), ri = var_impurity(r0, r1, r2);
        const double lw = (double)lc / (double)total, rw = (double)rc / (double)total;
        gain = pimp - lw * li - rw * ri;
        valid = 1;
        if (gain < A.min_gain) {
          gain = kMinValue;
          valid = 0;
        }
      }
      if (fs < 0 || gain > fg) {
        fg = gain;
        fs = s;
        fv = valid;
      }
    }
    if (best_f < 0 || fg > best_gain) {  // features visited in increasing order per lane
      best_gain = fg;
      best_f = fl;
      best_s = fs;
      best_valid = fv;
    }
  }
  // wave: first max over features (the larger gain, on ties the lower feature index)
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(best_gain, o);
    const int of = __shfl_xor(best_f, o);
    const int os = __shfl_xor(best_s, o);
    const int ov = __shfl_xor(best_valid, o);
    const bool take = of >= 0 && (best_f < 0 || og > best_gain || (og == best_gain && of < best_f));
    if (take) {
      best_gain = og;
      best_f = of;
      best_s = os;
      best_valid = ov;
    }
  }
  if (lane != 0) return;
  F64SplitOut o{};
  o.f = best_f;
  o.s = best_s;
  if (best_f < 0) {  // no feature has a split: invalid stats on the node's total
    const double* par = h + (int64_t)Fr * NB * 3;
    o.calc[0] = par[0];
    o.calc[1] = par[1];
    o.calc[2] = par[2];
    o.gain = kMinValue;
    o.impurity = var_impurity(par[0], par[1], par[2]);
    o.valid = 0;
    A.out[q] = o;
    return;
  }
  o.calc[0] = pc0;
  o.calc[1] = pc1;
  o.calc[2] = pc2;
  o.gain = best_gain;
  o.impurity = pimp;
  o.valid = best_valid;
  const double* fa = h + (int64_t)best_f * NB * 3;
  const int nsp = nbins[best_f] - 1;
  double c0 = 0, c1 = 0, c2 = 0, t0 = 0, t1 = 0, t2 = 0;
  for (int s = 0; s <= nsp; s++) {
    if (s == 0) {
      t0 = fa[0];
      t1 = fa[1];
      t2 = fa[2];
    } else {
      t0 += fa[3 * s];
      t1 += fa[3 * s + 1];
      t2 += fa[3 * s + 2];
    }
    if (s == best_s) {
      c0 = t0;
      c1 = t1;
      c2 = t2;
    }
  }
  o.left[0] = c0;
  o.left[1] = c1;
  o.left[2] = c2;
  o.right[0] = t0 - c0;
  o.right[1] = t1 - c1;
  o.right[2] = t2 - c2;
  A.out[q] = o;
}

void launch_f64_split(hipStream_t st, const F64SplitArgs& a, int nnodes) {
  hipLaunchKernelGGL(k_f64_split, dim3(nnodes), dim3(64), 0, st, a);
}

// ---------------------------------------------------------------- imported codes
// sbag_dataset_import checks a received code matrix before any kernel indexes a table
// with it: feature columns hold codes < their dictionary size, the row padding is zero.
__global__ __launch_bounds__(256) void k_check_codes(const void* __restrict__ codes, int code_bytes,
                                                     int64_t N, int32_t S, int32_t F,
                                                     const int64_t* __restrict__ dict_off,
                                                     int* __restrict__ bad) {
  const int64_t total = N * (int64_t)S;
  int b = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(i % S);
    const uint32_t v = code_bytes == 1   ? ((const uint8_t*)codes)[i]
                       : code_bytes == 2 ? ((const uint16_t*)codes)[i]
                                         : ((const uint32_t*)codes)[i];
    if (f < F ? (int64_t)v >= dict_off[f + 1] - dict_off[f] : v != 0u) b = 1;
  }
  if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
}

void launch_check_codes(hipStream_t st, const void* codes, int code_bytes, int64_t N, int32_t S,
                        int32_t F, const int64_t* d_dict_off, int* d_bad) {
  const int64_t total = N * (int64_t)S;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 256 * 16));
  hipLaunchKernelGGL(k_check_codes, dim3(blocks), dim3(256), 0, st, codes, code_bytes, N, S, F,
                     d_dict_off, d_bad);
}

}  // namespace sbag
