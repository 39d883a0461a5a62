// sbag_kernels.hip — gfx950 kernels of the bagging engine.
//
// Kernels (DESIGN.md §3 gives the roofline and algorithmic bytes of each):
//   k_poisson     per-(learner, partition) Well19937c + PoissonDistribution streams
//                 (sql/catalyst/expressions/Poisson.scala:53-56,73)
//   k_bernoulli   counter-based XORShiftRandom streams via GF(2) jump-ahead
//                 (Rand at sql/bfunctions.scala:62-64)
//   k_compact     per-replica in-bag row lists (replaces explode/replicate_row,
//                 sql/bfunctions.scala:42-44, HasSubBag.scala:112-114)
//   k_hist        streaming LDS-privatized histogram (the hot loop of Spark's
//                 RandomForest.findBestSplits, reached via
//                 ml/ensemble/ensembleParams.scala:113-115)
//   k_partition   rows of each split node -> its children (RandomForest's
//                 node-index update of every TreePoint per level)
//   k_split       prefix scan over bins + fp64 gain + first-max argmax
//                 (RandomForest.binsToBestSplit / calculateImpurityStats)
//   k_subtract    sibling histogram = parent - smaller child
//   k_bin_cuts / k_bin_ranked   per-replica bins from value codes (TreePoint.findBin)
//   k_predict     slicer + tree walk + in-order mean / breeze mode
//                 (BaggingRegressor.scala:248-256, BaggingClassifier.scala:248-257)
//   k_synth       bench data generator
// Built with -ffp-contract=off: every fp64 op of the gain formula is rounded
// separately, as the JVM does.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <set>
#include <type_traits>
#include <utility>

#include "sbag_internal.h"
#include "sbag_well.h"

namespace sbag {

// Raise a kernel's dynamic-LDS cap once per (kernel, device).  Thread-safe: contexts on
// different devices launch from their own threads (ml.py trains one thread per device).
// A failure stays in hipGetLastError(), which every launch site checks (HIP_TRY).
static void set_max_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  std::lock_guard<std::mutex> g(mu);
  if (done.count({fn, dev})) return;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess)
    done.insert({fn, dev});
}

// ======================================================================
// Poisson sampler (withBag with replacement, sql/bfunctions.scala:46-68 -> Poisson.scala:53-56):
// k_poisson4 (sbag_poisson.hip), the step-parallel Well19937c of DESIGN §4.3.  (Rounds 1-3's
// k_poisson / k_poisson2 / k_poisson3 were measured slower and removed in round 6.)
// ======================================================================
void launch_poisson(hipStream_t st, uint8_t* counts, int64_t N, const int64_t* d_part_off, int P,
                    int R, int learner0, int64_t seed, double mean, double p_exp, int* d_err) {
  // PoissonDistribution.nextPoisson's `n < 1000 * mean` for integer n: n < ceil(1000 * mean);
  // the cap is only checked when it can end a row below the 255 limit.  SBAG_POISSON_LANES:
  // lanes per stream (8, 16 or 4; default by stream count -- read per launch, the tests switch it)
  const int icap = (int)std::min(ceil(1000.0 * mean), 1e9);
  const char* el = getenv("SBAG_POISSON_LANES");
  launch_poisson4(st, counts, N, d_part_off, P, R, learner0, seed, p_exp, icap, icap <= 255, el ? atoi(el) : 0,
                  d_err);
}

// ======================================================================
// RandomForest.findSplits' split-finding sample (Spark 2.4.3): for subbags of more than
// max(maxBins^2, 10^4) rows, thresholds come from RDD.sample(false, fraction, seed') over
// the exploded subbag: partition p's BernoulliSampler is an XORShiftRandom seeded with
// the p-th java.util.Random(seed').nextLong() (part_state = its hashed state, host);
// GapSampling when fraction <= 0.4 (countForDropping = (log(max(u, 5e-11)) / log1p(-f))
// .toInt, the first gap drawn at the first item), else one nextDouble() <= f per item.
// A thread walks one (replica, partition) in row order, each row standing for `count`
// consecutive items, and adds every sampled item's value codes to the replica's value
// counts (vcoff layout), as findSplitsBySorting's groupByKey would see them.
// ======================================================================
__device__ __forceinline__ uint64_t xs_step_s(uint64_t s) {
  s ^= s << 21;
  s ^= s >> 35;
  s ^= s << 4;
  return s;
}

// Phase 1, a thread per (replica, partition): the walk appends every sampled item's row
// to the replica's list (order is irrelevant to the counts).  It skips whole 64-row
// chunks (one cache line of counts) while the current gap covers them.  Phase 2
// (k_split_sample_vc) gathers the sampled rows' value codes with every lane busy: the
// walk's lanes sample at different times, so gathering inside it serialised the wave.
__device__ __forceinline__ uint32_t bytesum4(uint32_t x) {
  x = (x & 0x00ff00ffu) + ((x >> 8) & 0x00ff00ffu);
  return (x & 0xffffu) + (x >> 16);
}

__global__ __launch_bounds__(64) void k_split_sample(
    const uint8_t* __restrict__ counts, int64_t N, const int64_t* __restrict__ part_off, int P,
    const int32_t* __restrict__ reps, const uint64_t* __restrict__ part_state,
    const double* __restrict__ frac, const uint16_t* __restrict__ gsums,
    uint32_t* __restrict__ rows_out, int64_t cap, uint32_t* __restrict__ nrows) {
  __shared__ uint32_t s_take[64 * 33];
  const int ri = blockIdx.y;
  const int r = reps[ri];
  const int p = (int)blockIdx.x * 64 + (int)threadIdx.x;
  if (p >= P) return;
  // per replica: fraction = required / numExamples and log1p(-fraction) (host libm, as the
  // oracle computes it)
  const double fraction = frac[2 * ri], lnq = frac[2 * ri + 1];
  uint64_t s = part_state[p];
  auto next_double = [&]() {
    s = xs_step_s(s);
    const int64_t a = (int64_t)(s & ((1ull << 26) - 1));
    s = xs_step_s(s);
    const int64_t b = (int64_t)(s & ((1ull << 27) - 1));
    return (double)((a << 27) + b) * 0x1.0p-53;
  };
  auto gap = [&]() {
    const double u = fmax(next_double(), 5e-11);
    return (int32_t)(log(u) / lnq);
  };
  uint32_t* out = rows_out + (int64_t)ri * cap;
  // sampled rows wait in the thread's LDS buffer: one returning atomic per 32 samples
  // (lanes sample at different times, so per-sample atomics serialised the wave)
  uint32_t* tb = s_take + threadIdx.x * 33;
  int nt = 0;
  auto flush = [&]() {
    if (nt == 0) return;
    const uint32_t k = atomicAdd(&nrows[ri], (uint32_t)nt);
    for (int i = 0; i < nt; i++)
      if ((int64_t)k + i < cap) out[k + i] = tb[i];
    nt = 0;
  };
  auto take = [&](int64_t row) {
    tb[nt++] = (uint32_t)row;
    if (nt == 32) flush();
  };
  const uint8_t* cr = counts + (int64_t)r * N;
  const int64_t r0 = part_off[p], r1 = part_off[p + 1];
  if (fraction <= 0.4) {
    // Item positions: the partition's rows in order, row i standing for counts[i] items.
    // GapSampling takes items g1, g1 + 1 + g2, ... (the gaps are drawn in order, the
    // first at the first item; an empty partition takes nothing either way), so the lanes
    // step in lockstep from one taken item to the next.  A lane finds the 256-row group
    // holding its target from the group sums (8 per 16-byte chunk, k_group_sums; the
    // partition's head and tail groups are summed here with the rows outside it masked),
    // then the word and the byte inside the group's counts.
    const int64_t off0 = (int64_t)r * N + r0, off1 = (int64_t)r * N + r1;  // byte offsets
    if (off1 > off0) {
      const int64_t G0 = off0 >> 8, G1 = (off1 - 1) >> 8;
      uint4 v[16];
      auto load_group = [&](int64_t G) {
        const uint4* q = (const uint4*)(counts + (G << 8));
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = q[u];
        if ((G << 8) < off0 || (G << 8) + 256 > off1) {
#pragma unroll
          for (int u = 0; u < 16; u++) {
            uint32_t* w = (uint32_t*)&v[u];
#pragma unroll
            for (int e = 0; e < 4; e++) {
              const int64_t a0 = (G << 8) + 16 * u + 4 * e;
              uint32_t m = 0;
#pragma unroll
              for (int bb = 0; bb < 4; bb++)
                m |= (a0 + bb >= off0 && a0 + bb < off1) ? (0xffu << (8 * bb)) : 0u;
              w[e] &= m;
            }
          }
        }
      };
      auto vsum = [&]() {
        uint32_t t = 0;
#pragma unroll
        for (int u = 0; u < 16; u++)
          t += bytesum4(v[u].x) + bytesum4(v[u].y) + bytesum4(v[u].z) + bytesum4(v[u].w);
        return t;
      };
      load_group(G0);
      const uint32_t head = vsum();
      load_group(G1);
      const uint32_t tail = vsum();
      int64_t vg = G1;  // the group held in v
      uint32_t cs[8];
      const int64_t K1 = G1 >> 3;
      int64_t K = G0 >> 3;
      auto load_chunk = [&]() {
        const uint4 q = ((const uint4*)gsums)[K];
        const uint32_t qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const int64_t G = K * 8 + j;
          const uint32_t gsv = (qq[j >> 1] >> (16 * (j & 1))) & 0xffffu;
          cs[j] = (G < G0 || G > G1) ? 0u : G == G0 ? head : G == G1 ? tail : gsv;
        }
      };
      auto csum = [&]() {
        uint32_t t = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) t += cs[j];
        return t;
      };
      load_chunk();
      uint32_t ksum = csum();
      int64_t base = 0;  // items before chunk K
      int64_t target = gap();
      while (true) {
        while (base + ksum <= target) {
          base += ksum;
          if (++K > K1) break;
          load_chunk();
          ksum = csum();
        }
        if (K > K1) break;
        int gsel = 0;
        int64_t gb = base;
        {
          int64_t acc = base;
          bool found = false;
#pragma unroll
          for (int j = 0; j < 8; j++) {
            const bool hit = !found && target < acc + cs[j];
            gsel = hit ? j : gsel;
            gb = hit ? acc : gb;
            found = found || hit;
            acc += cs[j];
          }
        }
        const int64_t G = K * 8 + gsel;
        if (G != vg) {
          load_group(G);
          vg = G;
        }
        uint32_t o = (uint32_t)(target - gb);  // item offset inside the group
        int widx = 0;
        uint32_t wsel = 0;
        {
          uint32_t acc = 0;
          bool found = false;
#pragma unroll
          for (int u = 0; u < 16; u++) {
            const uint32_t ww[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
              const uint32_t ws = bytesum4(ww[e]);
              const bool hit = !found && o < acc + ws;
              widx = hit ? 4 * u + e : widx;
              wsel = hit ? ww[e] : wsel;
              o = hit ? o - acc : o;
              found = found || hit;
              acc += found ? 0u : ws;
            }
          }
        }
        int bsel = 3;
#pragma unroll
        for (int bb = 2; bb >= 0; bb--) {
          uint32_t pre = 0;
          for (int t = 0; t <= bb; t++) pre += (wsel >> (8 * t)) & 0xffu;
          bsel = o < pre ? bb : bsel;
        }
        take((G << 8) + 4 * widx + bsel - (int64_t)r * N);
        target += 1 + (int64_t)gap();
      }
    }
  } else {
    for (int64_t row = r0; row < r1; row++)
      for (int k = cr[row]; k > 0; k--)
        if (next_double() <= fraction) take(row);
  }
  flush();
}

// Few partitions (P < 64: a GBM booster's single partition, or any fit on one partition):
// k_split_sample's lanes are partitions, so one lane would walk the whole subbag with a
// dependent load per taken item.  Here a wave takes one (replica, partition): GapSampling's
// gaps depend only on its XORShift stream, so every lane steps the stream to its own draw of
// a block of 64 (the stream is sequential: each lane runs the 64 steps, keeps the one it
// owns), the gaps' prefix gives the block's 64 taken item positions, and the wave streams the
// partition's count bytes (4096 rows per chunk in aligned 16-byte loads, three chunks ahead);
// the lanes whose items fall in a chunk resolve their rows in parallel.  The same items as
// the one-lane walk, in the same order: the row list is identical.
__global__ __launch_bounds__(64) void k_split_sample_gap(
    const uint8_t* __restrict__ counts, int64_t N, const int64_t* __restrict__ part_off, int P,
    const int32_t* __restrict__ reps, const uint64_t* __restrict__ part_state,
    const double* __restrict__ frac, uint32_t* __restrict__ rows_out, int64_t cap,
    uint32_t* __restrict__ nrows, int64_t counts_len, int W) {
  constexpr int kGapBuf = 2048;
  __shared__ uint32_t s_incl[64];
  __shared__ uint32_t s_words[64 * 16];
  __shared__ uint32_t s_buf[kGapBuf];
  // W waves per (replica, partition): wave w resolves the items of its share of the chunks
  // (every wave steps the whole gap stream -- cheap scalar work -- and skips the items
  // before its share, whose count it sums from the counts first)
  const int ri = blockIdx.y, p = blockIdx.x / W, wv = blockIdx.x % W, lane = threadIdx.x;
  const int r = reps[ri];
  const double lnq = frac[2 * ri + 1];
  uint64_t st = part_state[p];
  const uint8_t* cr = counts + (int64_t)r * N;
  const int64_t r0 = part_off[p], r1 = part_off[p + 1];
  uint32_t* out = rows_out + (int64_t)ri * cap;
  // the current chunk: 4096 rows from the 16-byte aligned address at or below the
  // partition's first row, lane l's 64 rows [c0 + 64 l, c0 + 64 l + 64) as four aligned
  // 16-byte loads (clamped inside the counts buffer: every lane loads, no branch); rows
  // outside [r0, r1) count 0
  // (the buffer holds counts_len >= 1 bytes; device allocations come in >= 4 KB pages, so a
  // 16-byte load clamped to its start stays mapped)
  const uint8_t* cbase = counts;
  const uint8_t* climit = counts + max(counts_len - 16, (int64_t)0);
  const int64_t a0 = r0 - (int64_t)(((uintptr_t)(cr + r0)) & 15u);  // row of the aligned start
  // issue: the chunk's four 16-byte loads per lane, raw (the data is not touched here, so
  // the loads stay in flight behind the current chunk); finish: the chunk's words, shifted
  // into place where a load was clamped to the buffer's last 16 bytes, rows outside
  // [r0, r1) masked to 0
  auto issue = [&](int64_t c0, uint4 (&v)[4]) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint8_t* pa = cr + c0 + 64 * lane + 16 * q;
      const uint8_t* pc = pa < cbase ? cbase : (pa > climit ? climit : pa);
      v[q] = *(const uint4*)pc;
    }
  };
  auto finish = [&](int64_t c0, const uint4 (&v)[4], uint32_t (&w)[16]) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t row = c0 + 64 * lane + 16 * q;
      const uint8_t* pa = cr + row;
      const uint8_t* pc = pa < cbase ? cbase : (pa > climit ? climit : pa);
      // clamped at the buffer's end (its last < 16 rows): the wanted bytes pa.. are the
      // loaded bytes from pa - pc on, the rest past the buffer (0): a 128-bit right shift
      const uint32_t s8 = 8u * (uint32_t)(pa > pc ? pa - pc : 0);
      const uint64_t lo = ((uint64_t)v[q].y << 32) | v[q].x, hi = ((uint64_t)v[q].w << 32) | v[q].z;
      const uint64_t nlo = s8 == 0 ? lo : s8 < 64 ? (lo >> s8) | (hi << (64 - s8)) : hi >> (s8 - 64);
      const uint64_t nhi = s8 < 64 ? hi >> s8 : 0ull;
      const uint32_t vv[4] = {(uint32_t)nlo, (uint32_t)(nlo >> 32), (uint32_t)nhi, (uint32_t)(nhi >> 32)};
#pragma unroll
      for (int d = 0; d < 4; d++) {
        uint32_t m = 0;
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
          const int64_t rr = row + 4 * d + bb;
          m |= (rr >= r0 && rr < r1) ? (0xFFu << (8 * bb)) : 0u;
        }
        w[4 * q + d] = pa < cbase ? 0u : (vv[d] & m);
      }
    }
  };
  auto bsum = [](uint32_t x) {  // sum of the 4 bytes
    x = (x & 0x00FF00FFu) + ((x >> 8) & 0x00FF00FFu);
    return (x & 0xFFFFu) + (x >> 16);
  };
  // kAhead - 1 chunks in flight behind the current one (the wave walks the partition's counts
  // chunk after chunk)
  constexpr int kAhead = 4;
  const int64_t nch = r1 > a0 ? (r1 - a0 + 4095) / 4096 : 0;  // the partition's chunks
  const int64_t cs = nch * wv / W, ce = nch * (wv + 1) / W;    // this wave's share
  const int64_t c_end = min(r1, a0 + 4096 * ce);
  uint32_t cw[16];
  // ring of kAhead chunks in flight; the chunk loop is unrolled kAhead times so each slot
  // is a fixed set of registers (moving an in-flight load's destination would wait for it)
  uint4 ring[kAhead][4];
  // items before the share: the counts of chunks [0, cs), summed through the same ring
  int64_t c0 = a0;
  uint32_t before = 0;
  {
    const int64_t pre_end = a0 + 4096 * cs;
#pragma unroll
    for (int a = 0; a < kAhead; a++) issue(c0 + 4096 * a, ring[a]);
    bool pm = c0 < pre_end;
    while (pm) {
#pragma unroll
      for (int a = 0; a < kAhead; a++) {
        if (pm) {
          finish(c0, ring[a], cw);
          issue(c0 + 4096 * kAhead, ring[a]);
#pragma unroll
          for (int k = 0; k < 16; k++) before += bsum(cw[k]);
          c0 += 4096;
          pm = c0 < pre_end;
        }
      }
    }
    // (the ring now holds chunks c0 .. c0 + kAhead - 1 in slot order only when cs is a
    // multiple of kAhead: reissue them in slot order)
#pragma unroll
    for (int a = 0; a < kAhead; a++) issue(c0 + 4096 * a, ring[a]);
  }
  for (int o = 32; o > 0; o >>= 1) before += (uint32_t)__shfl_xor((int)before, o);
  // a block of 64 draws: lane j holds taken item j (every lane steps the shared stream and
  // keeps its own draw); bhi = the block's last item
  int64_t next = 0;  // item index of the next draw's gap origin
  auto gen_block = [&](int64_t& tgt) {
    double myu = 0.0;
    for (int j = 0; j < 64; j++) {
      st = xs_step_s(st);
      const int64_t a = (int64_t)(st & ((1ull << 26) - 1));
      st = xs_step_s(st);
      const int64_t b = (int64_t)(st & ((1ull << 27) - 1));
      const double u = (double)((a << 27) + b) * 0x1.0p-53;
      if (j == lane) myu = u;
    }
    // countForDropping = (log(u) / lnq).toInt (a JVM cast saturates)
    const double q = log(fmax(myu, 5e-11)) / lnq;
    const int64_t g = (int64_t)(q >= 2147483647.0 ? 2147483647.0 : q);
    // taken item = previous + 1 + gap (the first: gap): an inclusive scan of gap + 1
    int64_t d = g + 1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = __shfl_up(d, o);
      if (lane >= o) d += u;
    }
    tgt = next + d - 1;
    next = next + __shfl(d, 63);
  };
  int64_t tgt;
  gen_block(tgt);
  int nbuf = 0;  // rows in s_buf
  auto flush = [&]() {
    __builtin_amdgcn_wave_barrier();
    uint32_t k0 = 0;
    if (lane == 0) k0 = atomicAdd(&nrows[ri], (uint32_t)nbuf);
    k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k0);
    for (int i = lane; i < nbuf; i += 64)
      if ((int64_t)k0 + i < cap) out[k0 + i] = s_buf[i];
    __builtin_amdgcn_wave_barrier();
    nbuf = 0;
  };
  int64_t ib = (int64_t)before;  // items before the chunk
  // Chunk-major: each chunk's words and lane prefixes go to LDS, and every lane whose taken
  // item falls in the chunk resolves its row in parallel (the owner lane by a binary
  // search over the prefixes, then its 64 rows' bytes) -- no per-item serial loop
  auto process = [&]() {
    uint32_t lsum = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) lsum += bsum(cw[k]);
    uint32_t incl = lsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
    const uint32_t ctot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    s_incl[lane] = incl;
#pragma unroll
    for (int k = 0; k < 16; k++) s_words[16 * lane + k] = cw[k];
    __builtin_amdgcn_wave_barrier();
    const int64_t iend = ib + (int64_t)ctot;
    for (;;) {
      const bool in = tgt >= ib && tgt < iend;
      const uint64_t im = __ballot(in);
      if (im) {
        uint32_t row = 0;
        if (in) {
          const uint32_t o = (uint32_t)(tgt - ib);
          // owner: the first lane w with incl[w] > o
          int w = 0;
#pragma unroll
          for (int stp = 32; stp > 0; stp >>= 1)
            if (s_incl[w + stp - 1] <= o) w += stp;
          uint32_t acc = s_incl[w];
          uint32_t wv[16];
#pragma unroll
          for (int k = 0; k < 16; k++) wv[k] = s_words[16 * w + k];
#pragma unroll
          for (int k = 0; k < 16; k++) acc -= bsum(wv[k]);  // items before lane w's rows
          // the word, then the byte, holding item o
          int kk = 0;
          uint32_t run = acc;
#pragma unroll
          for (int k = 0; k < 16; k++) {
            const uint32_t nx = run + bsum(wv[k]);
            const bool before = nx <= o && k == kk;
            run = before ? nx : run;
            kk += before ? 1 : 0;
          }
          uint32_t x = wv[0];
#pragma unroll
          for (int k = 1; k < 16; k++) x = kk == k ? wv[k] : x;
          int bb = 0;
#pragma unroll
          for (int q = 0; q < 3; q++) {
            const uint32_t nx = run + ((x >> (8 * q)) & 0xFFu);
            const bool before = nx <= o && q == bb;
            run = before ? nx : run;
            bb += before ? 1 : 0;
          }
          row = (uint32_t)(c0 + 64 * w + 4 * kk + bb);
        }
        // the chunk's rows of this block, in item order, to the LDS buffer (appended to the
        // replica's list with one atomic per kGapBuf rows: a returning atomic in the chunk
        // loop would wait for the chunk loads in flight, vmcnt counting in order)
        const int n = __popcll(im);
        const int rk = __popcll(im & ((1ull << lane) - 1));
        if (in) s_buf[nbuf + rk] = row;
        nbuf += n;
        if (nbuf > kGapBuf - 64) flush();
      }
      // the whole block lies before the chunk's end: the next block (it may start here too)
      const int64_t bhi = (int64_t)__builtin_amdgcn_readlane((int)(uint32_t)tgt, 63) |
                          ((int64_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)tgt >> 32), 63) << 32);
      if (bhi < iend) {
        gen_block(tgt);
        continue;
      }
      break;
    }
    __builtin_amdgcn_wave_barrier();
    ib = iend;
  };
  bool more = c0 < c_end;
  while (more) {
#pragma unroll
    for (int a = 0; a < kAhead; a++) {
      if (more) {
        finish(c0, ring[a], cw);
        issue(c0 + 4096 * kAhead, ring[a]);
        process();
        c0 += 4096;
        more = c0 < c_end;
      }
    }
  }
  if (nbuf > 0) flush();
}

// Phase 2, grid (sample chunks of kSvcRows, replicas): each sampled row adds its value codes
// to the replica's counts, in LDS when they fit (`lds_words`), flushed once.
constexpr int kSvcRows = 1024;  // sampled rows per k_split_sample_vc workgroup
__global__ __launch_bounds__(256) void k_split_sample_vc(
    const uint32_t* __restrict__ rows, int64_t cap, const uint32_t* __restrict__ nrows,
    const int32_t* __restrict__ reps, const uint8_t* __restrict__ codes, int code_bytes, int32_t S,
    const int32_t* __restrict__ sub, const int32_t* __restrict__ Fr, int32_t Fmax,
    const int64_t* __restrict__ vcoff, uint32_t* __restrict__ vc, int lds_words) {
  extern __shared__ uint32_t s_vc[];
  const int ri = blockIdx.y;
  const int r = reps[ri];
  const int64_t n = min((int64_t)nrows[ri], cap);
  const int64_t k0 = (int64_t)blockIdx.x * kSvcRows;
  if (k0 >= n) return;  // whole block
  const int fr = Fr[r];
  const int32_t* sr = sub + (int64_t)r * Fmax;
  const int64_t* vo = vcoff + (int64_t)r * Fmax;
  const int64_t vbase = vo[0];
  const int nw = (int)(vcoff[(int64_t)r * Fmax + fr] - vbase);
  const bool use_lds = nw <= lds_words;
  if (use_lds)
    for (int i = threadIdx.x; i < nw; i += 256) s_vc[i] = 0u;
  block_sync();
  // lane = feature within a 64-feature group, wave = every 4th sampled row: a row's
  // codes are read by one wave from its cache line
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t k1 = min(n, k0 + kSvcRows);
  for (int fg = 0; fg < fr; fg += 64) {
    const int fl = fg + lane;
    if (fl >= fr) break;
    const int64_t col = sr[fl];
    const uint32_t* rr = rows + (int64_t)ri * cap;
    auto code_at = [&](int64_t k) {
      const int64_t pos = (int64_t)rr[k] * S + col;
      return code_bytes == 1 ? (uint32_t)codes[pos] : (uint32_t)((const uint16_t*)codes)[pos];
    };
    if (use_lds) {
      uint32_t* dst = s_vc + (vo[fl] - vbase);
#pragma unroll 4
      for (int64_t k = k0 + wv; k < k1; k += 4) atomicAdd(&dst[code_at(k)], 1u);
    } else {
      uint32_t* dst = vc + vo[fl];
      for (int64_t k = k0 + wv; k < k1; k += 4) atomicAdd(&dst[code_at(k)], 1u);
    }
  }
  if (use_lds) {
    block_sync();
    for (int i = threadIdx.x; i < nw; i += 256)
      if (s_vc[i]) atomicAdd(&vc[vbase + i], s_vc[i]);
  }
}

// byte sums of the counts buffer's 256-byte groups (k_split_sample's skip index); groups
// past the buffer (the padding to whole 8-group chunks) are 0
__global__ __launch_bounds__(256) void k_group_sums(const uint8_t* __restrict__ counts,
                                                    int64_t bytes, uint16_t* __restrict__ gsums,
                                                    int64_t ngroups) {
  const int64_t G = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (G >= ngroups) return;
  uint32_t t = 0;
  if ((G << 8) < bytes) {
    const uint4* q = (const uint4*)(counts + (G << 8));
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const uint4 v = q[u];
      t += bytesum4(v.x) + bytesum4(v.y) + bytesum4(v.z) + bytesum4(v.w);
    }
  }
  gsums[G] = (uint16_t)t;
}

void launch_split_sample(hipStream_t st, const uint8_t* counts, int64_t N, int64_t R,
                         const int64_t* d_part_off, int P, const int32_t* d_reps, int nrep,
                         const uint64_t* d_part_state, const double* d_frac, uint16_t* d_gsums,
                         uint32_t* d_rows, int64_t cap, uint32_t* d_nrows, bool gap_sampling) {
  if (nrep == 0 || P == 0) return;
  // few partitions and GapSampling (every fraction <= 0.4): a wave per (replica, partition);
  // else k_split_sample's lanes walk the partitions (SBAG_SPLIT_SAMPLE_LANES=1 forces them)
  static const bool lanes_env = getenv("SBAG_SPLIT_SAMPLE_LANES") && atoi(getenv("SBAG_SPLIT_SAMPLE_LANES"));
  if (P < 64 && gap_sampling && !lanes_env) {
    // waves per (replica, partition): enough for ~32 waves per replica (SBAG_GAP_WAVES)
    const int W = getenv("SBAG_GAP_WAVES") ? std::max(1, atoi(getenv("SBAG_GAP_WAVES")))
                                           : std::max(1, std::min(32, 64 / P));
    hipLaunchKernelGGL(k_split_sample_gap, dim3((unsigned)(P * W), (unsigned)nrep), dim3(64), 0, st, counts,
                       N, d_part_off, P, d_reps, d_part_state, d_frac, d_rows, cap, d_nrows, R * N, W);
    return;
  }
  const int64_t ng = split_sample_groups(R * N);
  hipLaunchKernelGGL(k_group_sums, dim3((unsigned)((ng + 255) / 256)), dim3(256), 0, st, counts,
                     R * N, d_gsums, ng);
  const dim3 grid((unsigned)((P + 63) / 64), (unsigned)nrep);
  hipLaunchKernelGGL(k_split_sample, grid, dim3(64), 0, st, counts, N, d_part_off, P, d_reps,
                     d_part_state, d_frac, d_gsums, d_rows, cap, d_nrows);
}

void launch_split_sample_vc(hipStream_t st, const uint32_t* d_rows, int64_t cap,
                            const uint32_t* d_nrows, const int32_t* d_reps, int nrep,
                            const void* codes, int code_bytes, int32_t S, const int32_t* d_sub,
                            const int32_t* d_Fr, int32_t Fmax, const int64_t* d_vcoff, uint32_t* vc,
                            int lds_words) {
  if (nrep == 0) return;
  set_max_lds((const void*)k_split_sample_vc, 64 * 1024);
  const dim3 grid((unsigned)((cap + kSvcRows - 1) / kSvcRows), (unsigned)nrep);
  hipLaunchKernelGGL(k_split_sample_vc, grid, dim3(256), (size_t)lds_words * 4, st, d_rows, cap,
                     d_nrows, d_reps, (const uint8_t*)codes, code_bytes, S, d_sub, d_Fr, Fmax,
                     d_vcoff, vc, lds_words);
}

// Spark 2.4.3 RandomForest.findSplitsForContinuousFeature (the spark-mllib dependency the
// reference's DecisionTree learners call; the host's find_splits is the same walk) for one (replica, feature) per wave, over its value counts on the device: the weighted
// (value, count) list is the dictionary order with zero counts dropped and 0.0 carrying
// numSamples - (non-zero count), inserted at its sorted place when the dictionary lacks it.
// Midpoints of consecutive values when there are at most numSplits + 1 of them; else the
// stride walk: with current the running int count, a value's midpoint with its predecessor is
// taken when |prev - target| < |current - target|, then target += stride.  prev and current are
// prefix sums that do not depend on the choices, so a chunk of 64 entries evaluates the test in
// every lane, takes the first lane that passes, advances target and retests the lanes after it
// -- the host loop's order and fp64 operations exactly.  The cuts (#{values <= t}) are a binary
// search of the dictionary per threshold.  It replaces the value counts' copy to the host (a
// C3-sized continuous fit: 4 bytes per (replica, feature, dictionary value), 0.5 GB per learner
// half) and the host walk over them.
constexpr int kFindSplitsMaxTc = 520;
__global__ __launch_bounds__(64) void k_find_splits(SplitFindArgs A) {
  __shared__ double s_thr[kFindSplitsMaxTc];
  const int lane = threadIdx.x;
  const int k = blockIdx.y, fl = blockIdx.x;
  const int r = A.reps[k];
  if (fl >= A.Fr[r]) return;
  const int64_t rf = (int64_t)r * A.Fmax + fl;
  const int g = A.sub[rf];
  const double* d = A.dict + A.dict_off[g];
  const int64_t D = A.dict_off[g + 1] - A.dict_off[g];
  const uint32_t* cn = A.cnt + A.vcoff[rf];
  const int64_t z = A.zero_code[g];
  // non-zero count and values other than 0.0 present
  unsigned long long nnz = 0, nvz = 0;
  for (int64_t c = lane; c < D; c += 64) {
    const uint32_t v = cn[c];
    if (c != z) {
      nnz += v;
      nvz += v != 0u ? 1ull : 0ull;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    nnz += __shfl_xor(nnz, o);
    nvz += __shfl_xor(nvz, o);
  }
  if (nnz == 0) {  // featureSamples.isEmpty
    if (lane == 0) A.nt[rf] = 0;
    return;
  }
  const int64_t n = A.nw[k], num_samples = A.nsamp[k];
  const int64_t num_splits = min((int64_t)A.max_bins, n) - 1;
  const int64_t zeros = num_samples - (int64_t)nnz;
  const int64_t possible = (int64_t)nvz + (zeros > 0 ? 1 : 0) - 1;
  if (possible == 0) {
    if (lane == 0) A.nt[rf] = 0;
    return;
  }
  const bool mids = possible <= num_splits;
  // the implied 0.0's place when the dictionary lacks it: #{values < 0}
  int64_t zp = -1;
  if (z < 0 && zeros > 0) {
    int64_t lo = 0, hi = D;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (d[mid] < 0.0)
        lo = mid + 1;
      else
        hi = mid;
    }
    zp = lo;
  }
  const int64_t X = D + (zp >= 0 ? 1 : 0);
  const int tc = A.tc;
  const double stride = (double)num_samples / (double)(num_splits + 1);
  double target = stride;
  bool have_prev = false;
  double prev_val = 0.0;
  uint32_t cur = 0;  // Java int running count (wraps as the host's int32_t)
  int64_t rank = 0;  // valid entries before the chunk
  int64_t nt = 0;
  for (int64_t x0 = 0; x0 < X; x0 += 64) {
    const int64_t x = x0 + lane;
    double v = 0.0;
    uint32_t cv = 0u;
    if (x < X) {
      if (x == zp) {
        cv = (uint32_t)zeros;
      } else {
        const int64_t c = (zp >= 0 && x > zp) ? x - 1 : x;
        if (c == z) {
          cv = zeros > 0 ? (uint32_t)zeros : 0u;
        } else {
          cv = cn[c];
          v = d[c];
        }
      }
    }
    const bool valid = cv != 0u;
    const uint64_t vm = __ballot(valid);
    if (!vm) continue;
    uint32_t s = cv;  // inclusive prefix of the chunk's counts
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(s, o);
      if (lane >= o) s += t;
    }
    const uint32_t cur_i = cur + s, prev_i = cur_i - cv;
    const uint64_t below = vm & ((1ull << lane) - 1ull);
    const int pl = below ? 63 - __clzll((long long)below) : 0;
    const double pv_l = __shfl(v, pl);
    const double pv = below ? pv_l : prev_val;
    const bool cand = valid && (below != 0ull || have_prev);
    const double mid = (pv + v) / 2.0;
    if (mids) {
      const int64_t rk = rank + __popcll(below);  // this entry's place among the valid ones
      if (cand && rk - 1 < tc) s_thr[rk - 1] = mid;
    } else {
      uint64_t left = __ballot(cand);
      while (left) {
        const bool p = cand && fabs((double)(int32_t)prev_i - target) < fabs((double)(int32_t)cur_i - target);
        const uint64_t pm = __ballot(p) & left;
        if (!pm) break;
        const int f = __ffsll((unsigned long long)pm) - 1;
        const double m = __shfl(mid, f);
        if (lane == 0 && nt < tc) s_thr[nt] = m;
        nt++;
        target += stride;
        left &= f == 63 ? 0ull : ~((2ull << f) - 1ull);
      }
    }
    const int lv = 63 - __clzll((long long)vm);
    prev_val = __shfl(v, lv);
    cur = __shfl(cur_i, 63);
    have_prev = true;
    rank += __popcll(vm);
  }
  if (mids) nt = possible;
  block_sync();
  if (lane == 0) A.nt[rf] = (int32_t)min<int64_t>(nt, 0x7fffffff);
  const int64_t m = min<int64_t>(nt, tc);
  for (int64_t j = lane; j < m; j += 64) {
    const double t = s_thr[j];
    int64_t lo = 0, hi = D;  // first value > t
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (d[mid] <= t)
        lo = mid + 1;
      else
        hi = mid;
    }
    A.thr[rf * tc + j] = t;
    A.cut[rf * tc + j] = (uint32_t)lo;
  }
}

void launch_find_splits(hipStream_t st, const SplitFindArgs& a) {
  if (a.nrep == 0 || a.Fmax == 0) return;
  hipLaunchKernelGGL(k_find_splits, dim3((unsigned)a.Fmax, (unsigned)a.nrep), dim3(64), 0, st, a);
}

// ======================================================================
// Bernoulli sampler: XORShiftRandom is GF(2)-linear; a thread jumps its
// stream to row j0 with precomputed M^(2^k) matrices and then steps 256 rows.
// ======================================================================
__device__ __forceinline__ uint32_t d_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t d_mix_last(uint32_t h, uint32_t k) {
  k *= 0xcc9e2d51u;
  k = d_rotl(k, 15);
  k *= 0x1b873593u;
  return h ^ k;
}
__device__ __forceinline__ uint32_t d_mix(uint32_t h, uint32_t k) {
  h = d_mix_last(h, k);
  h = d_rotl(h, 13);
  return h * 5u + 0xe6546b64u;
}
// MurmurHash3.bytesHash of Spark 2.4.3's 64-byte hashSeed buffer
// (ByteBuffer.allocate(java.lang.Long.SIZE): the seed's 8 big-endian bytes, then 56 zeros).
// A zero block leaves mix_last's h unchanged, so those 14 blocks are plain mix(h, 0).
__device__ uint32_t d_hash64(uint32_t k0, uint32_t k1, uint32_t seed) {
  uint32_t h = d_mix(d_mix(seed, k0), k1);
#pragma unroll
  for (int i = 0; i < 14; i++) h = d_rotl(h, 13) * 5u + 0xe6546b64u;
  h ^= 64u;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__device__ uint64_t d_hash_seed(int64_t seed) {  // XORShiftRandom.hashSeed (Spark 2.4.3)
  const uint64_t u = (uint64_t)seed;
  // big-endian bytes b0..b7; little-endian 4-byte blocks of that array
  const uint32_t b0 = (uint32_t)(u >> 56) & 0xff, b1 = (uint32_t)(u >> 48) & 0xff;
  const uint32_t b2 = (uint32_t)(u >> 40) & 0xff, b3 = (uint32_t)(u >> 32) & 0xff;
  const uint32_t b4 = (uint32_t)(u >> 24) & 0xff, b5 = (uint32_t)(u >> 16) & 0xff;
  const uint32_t b6 = (uint32_t)(u >> 8) & 0xff, b7 = (uint32_t)u & 0xff;
  const uint32_t k0 = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
  const uint32_t k1 = b4 | (b5 << 8) | (b6 << 16) | (b7 << 24);
  const uint32_t lo = d_hash64(k0, k1, 0x3c074a61u);
  const uint32_t hi = d_hash64(k0, k1, lo);
  return ((uint64_t)hi << 32) | (uint64_t)lo;
}
__device__ __forceinline__ uint64_t xs_step(uint64_t s) {
  s ^= s << 21;
  s ^= s >> 35;
  s ^= s << 4;
  return s;
}

__global__ __launch_bounds__(256) void k_bernoulli(uint8_t* __restrict__ counts, int64_t N,
                                                   const int64_t* __restrict__ part_off,
                                                   const int64_t* __restrict__ chunk_pre, int P,
                                                   int64_t chunks_total, int R, int learner0,
                                                   int64_t seed, double ratio,
                                                   const uint64_t* __restrict__ jump) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)R * chunks_total) return;
  const int r = (int)(t / chunks_total);
  const int64_t c = t % chunks_total;
  int lo = 0, hi = P;  // largest p with chunk_pre[p] <= c
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (chunk_pre[mid] <= c)
      lo = mid;
    else
      hi = mid;
  }
  const int p = lo;
  const int64_t j0 = (c - chunk_pre[p]) * 256;
  const int64_t row0 = part_off[p] + j0;
  const int64_t row1 = min(row0 + 256, part_off[p + 1]);
  const int i = learner0 + r;
  int64_t rs;
  if (seed >= (int64_t)INT_MIN && seed <= (int64_t)INT_MAX) {  // SQL Int addition (H15)
    const int32_t s32 = (int32_t)((uint32_t)(int32_t)seed + (uint32_t)i);
    rs = (int64_t)s32 + p;
  } else {
    rs = (int64_t)((uint64_t)seed + (uint64_t)(int64_t)i + (uint64_t)(int64_t)p);
  }
  uint64_t s = d_hash_seed(rs);
  const uint64_t steps = 2ull * (uint64_t)j0;
  for (int k = 0; k < 63; k++) {
    if ((steps >> k) & 1ull) {
      const uint64_t* m = jump + k * 64;
      uint64_t acc = 0, x = s;
      while (x) {
        const int b = __ffsll((long long)x) - 1;
        acc ^= m[b];
        x &= x - 1;
      }
      s = acc;
    }
  }
  uint8_t* out = counts + (int64_t)r * N;
  for (int64_t row = row0; row < row1; row++) {
    s = xs_step(s);
    const int64_t a = (int64_t)(s & ((1ull << 26) - 1));
    s = xs_step(s);
    const int64_t b = (int64_t)(s & ((1ull << 27) - 1));
    const double u = (double)((a << 27) + b) * 0x1.0p-53;
    out[row] = (u < ratio) ? 1 : 0;
  }
}

void launch_bernoulli(hipStream_t st, uint8_t* counts, int64_t N, const int64_t* d_part_off,
                      const int64_t* d_chunk_pre, int P, int64_t chunks_total, int R,
                      int learner0, int64_t seed, double ratio, const uint64_t* d_jump) {
  const int64_t threads = (int64_t)R * chunks_total;
  const int blocks = (int)((threads + 255) / 256);
  hipLaunchKernelGGL(k_bernoulli, dim3(blocks), dim3(256), 0, st, counts, N, d_part_off,
                     d_chunk_pre, P, chunks_total, R, learner0, seed, ratio, d_jump);
}

__global__ void k_fill(uint8_t* p, uint8_t v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
void launch_fill(hipStream_t st, uint8_t* p, uint8_t v, int64_t n) {
  int blocks = (int)std::min<int64_t>((n + 255) / 256, 65536);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, st, p, v, n);
}

// ======================================================================
// In-bag compaction: entries of rows with count > 0.  A block owns 8192 rows of
// one replica (replicas interleaved over the grid so concurrent blocks hit
// different cursors); per 1024 rows a block-wide scan and ONE atomic reserve the
// output slots.  Order inside a segment is irrelevant (integer stats).  Also
// reports the weighted row count and the largest count per replica.
// ======================================================================
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

template <bool STG>
__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ counts, int64_t N,
                                                 const int32_t* __restrict__ labk,
                                                 uint64_t* __restrict__ ent, int64_t cap,
                                                 unsigned long long* cursor,
                                                 unsigned long long* wsum, unsigned int* cmax,
                                                 unsigned long long* sqsum, int R) {
  const int r = blockIdx.x % R;
  const int64_t chunk = blockIdx.x / R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ unsigned long long s_base;
  __shared__ unsigned long long s_red[4];
  __shared__ unsigned int s_max[4];
  const uint8_t* cr = counts + (int64_t)r * N;
  uint64_t* er = ent + (int64_t)r * cap;
  unsigned long long mysum = 0, mysq = 0;
  unsigned int mymax = 0;
  // all 8 iterations' count words and labels are loaded up front (one dword and one
  // 16-byte load each when the rows are whole and aligned): the loop's barriers and cursor
  // atomic then no longer wait on them one iteration at a time
  const bool vec = ((N | (int64_t)(uintptr_t)cr) & 3) == 0 && ((uintptr_t)labk & 15) == 0;
  uint32_t cw[8];
  int4 lk[8];
#pragma unroll
  for (int it = 0; it < 8; it++) {
    const int64_t row0 = chunk * 8192 + (int64_t)it * 1024 + (int64_t)tid * 4;
    if (vec && row0 + 3 < N) {
      cw[it] = *(const uint32_t*)(cr + row0);
      lk[it] = *(const int4*)(labk + row0);
    } else {
      cw[it] = 0;
      int l4[4] = {0, 0, 0, 0};
      for (int j = 0; j < 4; j++)
        if (row0 + j < N) {
          cw[it] |= (uint32_t)cr[row0 + j] << (8 * j);
          l4[j] = labk[row0 + j];
        }
      lk[it] = make_int4(l4[0], l4[1], l4[2], l4[3]);
    }
  }
  // one cursor reservation for the workgroup's 8192 rows: the 8 iterations' wave scans first
  // (no barriers between them), their wave totals through LDS, one atomic, then the stores in
  // row order (8 reservations, each a round trip between two barriers, paced the kernel)
  __shared__ int s_it[8][4];
  __shared__ uint64_t s_stage[STG ? 4 : 1][STG ? 256 : 1];
  int incl[8], nn[8];
#pragma unroll
  for (int it = 0; it < 8; it++) {
    int n = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t c = (cw[it] >> (8 * j)) & 0xffu;
      n += c ? 1 : 0;
      mysum += c;
      mymax = max(mymax, c);
    }
    nn[it] = n;
    incl[it] = wave_incl_scan(n, lane);
    if (lane == 63) s_it[it][wave] = incl[it];
  }
  block_sync();
  if (tid == 0) {
    int total = 0;
#pragma unroll
    for (int it = 0; it < 8; it++)
#pragma unroll
      for (int w = 0; w < 4; w++) total += s_it[it][w];
    s_base = total ? atomicAdd(&cursor[r], (unsigned long long)total) : 0ull;
  }
  block_sync();
  unsigned long long itbase = s_base;
#pragma unroll
  for (int it = 0; it < 8; it++) {
    const int64_t row0 = chunk * 8192 + (int64_t)it * 1024 + (int64_t)tid * 4;
    const int32_t kk[4] = {lk[it].x, lk[it].y, lk[it].z, lk[it].w};
    int before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
      before += w < wave ? s_it[it][w] : 0;
      total += s_it[it][w];
    }
    if (STG) {
      // the wave's entries (contiguous in the output) go through its LDS run first, then out
      // as lane-consecutive 8-byte stores: one 512-byte line run per store instead of 64
      // lanes' entries scattered over the wave's ~1.3 KB (4 predicated stores per iteration)
      uint64_t* sw = s_stage[wave];
      int lp = incl[it] - nn[it];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t c = (cw[it] >> (8 * j)) & 0xffu;
        if (c) {
          const int32_t k = kk[j];
          mysq += (unsigned long long)c * (unsigned long long)((int64_t)k * k);
          sw[lp++] = pack_entry((uint32_t)(row0 + j), k, c);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int wn = s_it[it][wave];
      uint64_t* dst = er + itbase + (unsigned long long)before;
      for (int q = lane; q < wn; q += 64) dst[q] = sw[q];
      __builtin_amdgcn_wave_barrier();  // (the run is rewritten by the next iteration)
    } else {
      unsigned long long pos = itbase + (unsigned long long)(before + incl[it] - nn[it]);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t c = (cw[it] >> (8 * j)) & 0xffu;
        if (c) {
          const int32_t k = kk[j];
          mysq += (unsigned long long)c * (unsigned long long)((int64_t)k * k);
          er[pos++] = pack_entry((uint32_t)(row0 + j), k, c);
        }
      }
    }
    itbase += (unsigned long long)total;
  }
  __shared__ unsigned long long s_sq[4];
  for (int o = 32; o > 0; o >>= 1) {
    mysum += __shfl_down(mysum, o);
    mysq += __shfl_down(mysq, o);
    mymax = max(mymax, (unsigned int)__shfl_down((int)mymax, o));
  }
  if (lane == 0) {
    s_red[wave] = mysum;
    s_sq[wave] = mysq;
    s_max[wave] = mymax;
  }
  block_sync();
  if (tid == 0) {
    const unsigned long long s = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    const unsigned long long q = s_sq[0] + s_sq[1] + s_sq[2] + s_sq[3];
    const unsigned int m = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
    if (s) atomicAdd(&wsum[r], s);
    if (q) atomicAdd(&sqsum[r], q);
    if (m) atomicMax(&cmax[r], m);
  }
}

void launch_compact(hipStream_t st, const uint8_t* counts, int64_t N, int R, const int32_t* d_labk,
                    uint64_t* ent, int64_t cap, unsigned long long* d_cursor,
                    unsigned long long* d_wsum, unsigned int* d_cmax, unsigned long long* d_sqsum) {
  const int64_t chunks = (N + 8191) / 8192;
  static const bool stg = !getenv("SBAG_COMPACT_STG") || atoi(getenv("SBAG_COMPACT_STG")) != 0;  // (A/B)
  if (stg)
    hipLaunchKernelGGL(k_compact<true>, dim3((unsigned)(chunks * R)), dim3(256), 0, st, counts, N, d_labk,
                       ent, cap, d_cursor, d_wsum, d_cmax, d_sqsum, R);
  else
    hipLaunchKernelGGL(k_compact<false>, dim3((unsigned)(chunks * R)), dim3(256), 0, st, counts, N, d_labk,
                       ent, cap, d_cursor, d_wsum, d_cmax, d_sqsum, R);
}

// ======================================================================
// Histogram (the hot kernel) and the row partition that feeds it.
//
// k_hist streams the entries of the nodes being histogrammed; LDS holds only
// the histogram.  Grid (workgroups, feature tiles): workgroup w walks pieces
// [wg_piece[w], wg_piece[w+1]) -- contiguous slices of node segments, in node
// order -- and keeps the current node's histogram in LDS until the node changes
// (or flush_limit entries were added), so a flush of Fr x NB bins happens once
// per (workgroup, node run).  Inside a run the waves are independent (no
// barrier): each takes batches of 64 consecutive entries; lane i loads entry i
// and computes its stat words, then for every entry of the batch the wave
// broadcasts row and words (readlane), lane fl loads the aligned 4-byte word holding
// byte pos[fl] of that row straight from the row's cache line (SGPR row base + VGPR
// column; HistArgs.dw = 1: the byte itself) one group of entries ahead, extracts the
// byte, and adds the words into
// [plane][bin][feature] with one LDS atomic per plane.  The LDS atomic pipe is
// the only shared resource, and it only carries the atomics.
//
// Variance stats are two u64 planes per (bin, feature): (count << cshift) +
// count*(k + K0) and count*k^2 -- integers, so the result is order-independent
// and bit-exact; cshift and flush_limit are chosen on the host from the label
// range and the largest count.  Gini: one u32 plane per class.  Each plane has
// 64 trailing dump words: lanes past the tile's features add there (amul = 0),
// so the accumulation is branch-free.
//
// k_partition routes the entries of each split node into its two children
// (left block grows from the segment start, right block from its end), one
// cursor atomic per wave and side for 256 entries.
// ======================================================================
constexpr int kHistThreads = 512;  // 8 waves; two workgroups per CU at <= 80 KB of LDS
constexpr int kHistWaves = kHistThreads / 64;
// entries per pipeline group: row bytes of the next group are loaded while the current
// one is added, so a wave keeps up to 2 groups of row gathers in flight (k_hist is bound
// by their latency when the atomics are few: 16 for up to two 64-feature lane groups)
// (gini with one lane group: 8, so that the kernel fits 64 VGPRs at 8 waves per SIMD)
template <int MODE, int NJ, int GW>
constexpr int hist_group() {
  return (MODE == kHistGini && NJ == 1) || NJ > 2 ? 8 : 16;
}

static __host__ __device__ inline uint32_t hist_plane_bytes(int NB, int FPH, bool gini) {
  return (uint32_t)(NB * FPH + 64) * (gini ? 4u : 8u);
}

// MODE: kHistGini  u32 class counts, one plane per class  -> hist[.][cls]
//       kHistVar   u64 (count << cshift) + count*(k + K0)  -> hist[.][0], hist[.][1]
//       kHistSq    u64 count*k^2                           -> hist[.][2]
template <int MODE>
__device__ __forceinline__ void hist_flush(const HistArgs& A, const unsigned char* smem,
                                           uint32_t plane, int slot, int ft0, int ftn, int c0,
                                           int nct, bool store) {
  const int tid = threadIdx.x;
  const int NB = A.NB, NS = A.NS, FPH = A.FPH;
  const int64_t slot_words = (int64_t)A.Fmax * NB * NS;
  if (MODE == kHistGini) {
    // class planes [0, nct) of the LDS hold classes [c0, c0 + nct).  Lane q takes one
    // (feature, bin): features fastest, so the LDS reads of a class plane hit distinct
    // banks (planes and bin rows are multiples of 64 words apart), and the lane writes
    // its classes -- runs of 4 contiguous in the class-tile-major global layout
    // (gini_cell) -- as 16-byte stores.  With the workgroup's tile equal to the layout
    // tile (grouped C5) the flush writes one contiguous block that no other workgroup
    // shares a line of.
    uint32_t* gh = (uint32_t*)A.hist + (int64_t)slot * slot_words;
    const int hct = A.hct;
    const bool vec = store && ((hct | c0) & 3) == 0;
    if (vec && nct == 4 && hct == 4 && ftn <= 64) {
      // the workgroup's class tile is the layout tile (grouped C5): its block
      // [Fmax][NB][4] is contiguous; lane = feature, waves step the bins -- no index
      // division per (feature, bin) (the general loop below spent ~60 instructions on
      // each, which made the flush a third of the deep levels' histogram time)
      uint4* blk = (uint4*)(gh + (int64_t)(c0 >> 2) * A.Fmax * NB * 4) + (int64_t)ft0 * NB;
      const int f = tid & 63;
      if (f < ftn)
        for (int b = tid >> 6; b < NB; b += (int)(blockDim.x >> 6)) {
          const unsigned char* src = smem + ((size_t)b * FPH + f) * 4;
          uint4 v;
          v.x = *(const uint32_t*)(src);
          v.y = *(const uint32_t*)(src + plane);
          v.z = *(const uint32_t*)(src + 2 * (size_t)plane);
          v.w = *(const uint32_t*)(src + 3 * (size_t)plane);
          blk[f * NB + b] = v;
        }
      return;
    }
    for (int q = tid; q < ftn * NB; q += blockDim.x) {
      const int f = q % ftn, b = q / ftn;
      const unsigned char* src = smem + ((size_t)b * FPH + f) * 4;
      int cl = 0;
      if (vec)
        for (; cl + 4 <= nct; cl += 4) {
          uint4 v;
          v.x = *(const uint32_t*)(src + (size_t)cl * plane);
          v.y = *(const uint32_t*)(src + (size_t)(cl + 1) * plane);
          v.z = *(const uint32_t*)(src + (size_t)(cl + 2) * plane);
          v.w = *(const uint32_t*)(src + (size_t)(cl + 3) * plane);
          *(uint4*)(gh + gini_cell(ft0 + f, b, c0 + cl, NB, A.Fmax, hct)) = v;
        }
      // (a stored flush writes its zeros too: the host then leaves the slot's tile unzeroed)
      for (; cl < nct; cl++) {
        const uint32_t v = *(const uint32_t*)(src + (size_t)cl * plane);
        uint32_t* dst = gh + gini_cell(ft0 + f, b, c0 + cl, NB, A.Fmax, hct);
        if (store)
          *dst = v;
        else if (v)
          atomicAdd(dst, v);
      }
    }
  } else {
    unsigned long long* gh = (unsigned long long*)A.hist + (int64_t)slot * slot_words;
    const int cs = A.cshift;
    const uint64_t MS = (1ull << cs) - 1;
    for (int q = tid; q < ftn * NB; q += blockDim.x) {
      const int f = q % ftn, b = q / ftn;  // features fastest, as above
      const uint64_t w = *(const uint64_t*)(smem + ((size_t)b * FPH + f) * 8);
      if (w) {
        const int64_t gb = ((int64_t)(ft0 + f) * NB + b) * 3;
        if (MODE == kHistVar) {
          const uint64_t cnt = w >> cs;
          const int64_t sk = (int64_t)(w & MS) - (int64_t)A.K0 * (int64_t)cnt;
          if (store) {
            gh[gb] = (unsigned long long)cnt;
            gh[gb + 1] = (unsigned long long)sk;
          } else {
            atomicAdd(&gh[gb], (unsigned long long)cnt);
            atomicAdd(&gh[gb + 1], (unsigned long long)sk);
          }
        } else if (store) {
          gh[gb + 2] = (unsigned long long)w;
        } else {
          atomicAdd(&gh[gb + 2], (unsigned long long)w);
        }
      }
    }
  }
}

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// bytes of the NJ feature columns of entries [u0, u0 + KG) of the batch.  DW: each lane
// loads the aligned dword holding its byte (posr is then pos & ~3; the add extracts the
// byte): a wave's 64 lanes touch ~1/4 as many distinct addresses as with byte loads, which
// for a subspace's scattered columns is what the vector memory path is paced by
template <int NJ, int KG, int GW>
__device__ __forceinline__ void hist_load_group(const uint8_t* __restrict__ binsr, uint32_t S,
                                                uint32_t row, int u0, const uint32_t (&posr)[NJ],
                                                uint32_t (&buf)[KG][NJ]) {
#pragma unroll
  for (int t = 0; t < KG; t++) {
    // a buffer load per row: the resource's base is the row (SGPRs: the row index is
    // wave-uniform), the column the VGPR offset -- no VALU for the address (a global load
    // took a v_mov of the column or a 64-bit v_lshl_add per load)
    const uint8_t* rp = binsr + (size_t)rdlane(row, u0 + t) * S;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)rp, (short)0, (int)S, 0x00020000);
#pragma unroll
    for (int jj = 0; jj < NJ; jj++) {
      if (GW == 4)
        buf[t][jj] = __builtin_amdgcn_raw_buffer_load_b32(rs, posr[jj], 0, 0);
      else
        buf[t][jj] = __builtin_amdgcn_raw_buffer_load_b8(rs, posr[jj], 0, 0);
    }
  }
}

// one LDS atomic per entry and lane group: GINI adds count wl into class plane
// (offset wh); the u64 modes add (wh:wl)
// ONES (gini): every count of the batch is 1 (Bernoulli bags, C5): the added value is the
// constant 1 and the count readlane and its VGPR copy go away (5 VALU per entry, not 7)
template <int MODE, int NJ, int KG, int GW, bool ONES = false>
__device__ __forceinline__ void hist_add_group(unsigned char* smem, int u0,
                                               const uint32_t (&buf)[KG][NJ], uint32_t wl,
                                               uint32_t wh, const uint32_t (&amul)[NJ],
                                               const uint32_t (&abase)[NJ],
                                               const uint32_t (&bsh)[NJ]) {
  auto bin = [&](int t, int jj) -> uint32_t {
    return GW == 4 ? __builtin_amdgcn_ubfe(buf[t][jj], bsh[jj], 8) : buf[t][jj];
  };
#pragma unroll
  for (int t = 0; t < KG; t++) {
    const int u = u0 + t;
    if (MODE == kHistGini && ONES) {
      const uint32_t cou = rdlane(wh, u);
#pragma unroll
      for (int jj = 0; jj < NJ; jj++) {
        const uint32_t addr = __umul24(bin(t, jj), amul[jj]) + abase[jj] + cou;
        atomicAdd((uint32_t*)(smem + addr), 1u);
      }
    } else if (MODE == kHistGini) {
      const uint32_t cu = rdlane(wl, u), cou = rdlane(wh, u);
#pragma unroll
      for (int jj = 0; jj < NJ; jj++) {
        const uint32_t addr = __umul24(bin(t, jj), amul[jj]) + abase[jj] + cou;
        atomicAdd((uint32_t*)(smem + addr), cu);
      }
    } else {
      const unsigned long long a0 = ((unsigned long long)rdlane(wh, u) << 32) | rdlane(wl, u);
#pragma unroll
      for (int jj = 0; jj < NJ; jj++) {
        const uint32_t addr = __umul24(bin(t, jj), amul[jj]) + abase[jj];
        atomicAdd((unsigned long long*)(smem + addr), a0);
      }
    }
  }
}

// The second bound is waves per SIMD.  Gini with one lane group (C5's class tiles, ~34 KB
// of LDS, four workgroups per CU) needs 8 waves per SIMD, i.e. <= 64 VGPRs: at 85 VGPRs only
// two of the four workgroups were resident.
// NT threads per workgroup, KG entries per gather group.  The default (512, 8 or 16) keeps
// 8 waves per SIMD; the short-segment form (256, 32) is for deep levels, where a (node,
// class tile) sub-segment is a few hundred entries: each wave then holds one or two
// batches, the barriers around every sub-segment's flush expose the whole chain of gather
// groups, and 32-entry groups (4 waves per SIMD, 128 VGPRs) cut that chain by 4.
template <int MODE, int NJ, int GW, int NT = kHistThreads, int KG = hist_group<MODE, NJ, GW>()>
__global__ __launch_bounds__(NT, NT == kHistThreads ? (MODE == kHistGini && NJ == 1 ? 8 : 4) : 4) void k_hist(HistArgs A) {
  constexpr int kWaves = NT / 64;
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr bool GINI = MODE == kHistGini;
  const int tid = threadIdx.x, lane = tid & 63;
  // wave-uniform for the compiler too: batch bounds and the group loop's exits stay scalar
  // branches, so the row-byte loads of the next group stay in flight across them (with a
  // VGPR wave index the branches were exec-masked and each group waited for the next)
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NB = A.NB, FPH = A.FPH;
  const uint32_t S = (uint32_t)A.S;
  const int ft0 = (int)(blockIdx.y % (unsigned)A.ntf) * A.FT;
  // gini class tiling: this workgroup accumulates classes [c0, c0 + nct) only -- the
  // grid's tile, or (grouped) the tile of the current sub-segment
  int c0 = GINI && !A.grouped ? (int)(blockIdx.y / (unsigned)A.ntf) * A.CT : 0;
  int nct = GINI ? min(A.CT, A.NS - c0) : 1;
  const bool ctile = GINI && !A.count_only && A.CT < A.NS && !A.grouped;
  constexpr uint32_t WB = GINI ? 4u : 8u;
  const uint32_t plane = hist_plane_bytes(NB, FPH, GINI);
  const uint32_t hist_bytes = plane * (GINI ? (uint32_t)A.CT : 1u);
  const uint32_t dump = (uint32_t)NB * FPH * WB + (uint32_t)lane * WB;  // inside plane 0
  // per-wave staging of the batch entries that fall in the class tile
  uint64_t* stage = (uint64_t*)(smem + hist_bytes) + wave * 64;
  const uint64_t lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));

  for (uint32_t i = (uint32_t)tid * 16; i < hist_bytes; i += NT * 16)
    *(uint4*)(smem + i) = make_uint4(0, 0, 0, 0);

  const int p0 = A.wg_piece[blockIdx.x], p1 = A.wg_piece[blockIdx.x + 1];
  int cur_slot = -1, cur_ftn = 0, cur_r = -1, cur_tile = -1;
  bool cur_store = false;  // the current node run is this workgroup's alone and not yet flushed
  int64_t acc = 0;
  uint32_t posr[NJ], amul[NJ], abase[NJ], bsh[NJ];
#pragma unroll
  for (int j = 0; j < NJ; j++) {
    posr[j] = 0;
    bsh[j] = 0;
    amul[j] = 0;
    abase[j] = dump;
  }
  block_sync();

  // pieces carry their parent's replica, slot, tile and feature count (HistChunk), and the
  // next piece is loaded while this one runs; the first entries of a piece are loaded before
  // the flush of the previous node.  Deep levels are thousands of short pieces per
  // workgroup, where these dependent loads were most of the time.
  HistChunk pn = p0 < p1 ? A.chunks[p0] : HistChunk{};
  for (int p = p0; p < p1; p++) {
    const HistChunk pc = pn;
    if (p + 1 < p1) pn = A.chunks[p + 1];
    const int r = pc.r;
    const int ftn = min(A.FT, pc.fr - ft0);
    const int slot = pc.slot;
    if (ftn <= 0 || slot < 0) continue;
    const int64_t a = pc.a, b = pc.b;
    const int tile = A.grouped ? pc.tile : 0;
    // entries of the wave's next batch are loaded one batch ahead
    int64_t q0 = a + (int64_t)wave * 64;
    uint64_t e_next = (q0 + lane < b) ? A.ent_in[q0 + lane] : 0ull;
    if (slot != cur_slot || tile != cur_tile || acc + (b - a) > A.flush_limit) {
      if (cur_slot >= 0) {
        block_sync();
        if (!(A.ablate & 1)) hist_flush<MODE>(A, smem, plane, cur_slot, ft0, cur_ftn, c0, nct, cur_store);
        block_sync();
        if (!(A.ablate & 2))
          for (uint32_t i = (uint32_t)tid * 16; i < hist_bytes; i += NT * 16)
            *(uint4*)(smem + i) = make_uint4(0, 0, 0, 0);
        block_sync();
      }
      // a node split over several flushes by this workgroup adds from the second on
      cur_store = (slot != cur_slot || tile != cur_tile) && pc.excl != 0;
      cur_slot = slot;
      cur_tile = tile;
      cur_ftn = ftn;
      acc = 0;
      if (GINI && A.grouped) {
        c0 = tile * A.CT;
        nct = min(A.CT, A.NS - c0);
      }
    }
    acc += b - a;
    if (r != cur_r) {
#pragma unroll
      for (int j = 0; j < NJ; j++) {
        const int fl = lane + 64 * j;
        const bool ok = fl < ftn;
        const uint32_t pb = ok ? (uint32_t)A.pos[(int64_t)r * A.Fmax + ft0 + fl] : 0u;
        posr[j] = pb & ~(uint32_t)(GW - 1);
        bsh[j] = (pb & (uint32_t)(GW - 1)) * 8u;
        amul[j] = ok ? (uint32_t)FPH * WB : 0u;
        abase[j] = ok ? (uint32_t)fl * WB : dump;
      }
      cur_r = r;
    }
    const uint8_t* binsr = A.bins + (int64_t)r * A.bins_rstride;
    const int cs = A.cshift;
    const int64_t K0 = A.K0;
    const uint32_t cstride = A.count_only ? 0u : plane;
    for (; q0 < b; q0 += (int64_t)kWaves * 64) {
      int n = (int)min((int64_t)64, b - q0);
      uint64_t e = e_next;
      const int64_t qn = q0 + (int64_t)kWaves * 64 + lane;
      e_next = (qn < b) ? A.ent_in[qn] : 0ull;
      if (ctile) {  // keep the batch entries of classes [c0, c0 + nct), packed to the front
        const int32_t eh = (int32_t)(e >> 32);
        const int kc = eh >> 8;
        const bool m = ((eh & 0xff) != 0) && kc >= c0 && kc < c0 + nct;  // c = 0 past the piece
        const uint64_t mask = __ballot(m);
        if (m) stage[__popcll(mask & lt_mask)] = e;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        n = __popcll(mask);
        e = (lane < n) ? stage[lane] : 0ull;
        __builtin_amdgcn_wave_barrier();
        if (n == 0) continue;
      }
      const uint32_t row = (uint32_t)e;
      const int32_t hi = (int32_t)(e >> 32);
      const uint32_t c = (uint32_t)hi & 0xffu;  // 0 for lanes past the piece: they add zeros
      const int32_t k = hi >> 8;
      uint32_t wl, wh;
      if (MODE == kHistGini) {
        wl = c;
        wh = c ? (uint32_t)(k - c0) * cstride : 0u;  // class plane offset; c = 0 lanes add 0
      } else {
        const uint64_t w = MODE == kHistVar
                               ? ((uint64_t)c << cs) + (uint64_t)c * (uint64_t)((int64_t)k + K0)
                               : (uint64_t)c * (uint64_t)((int64_t)k * (int64_t)k);  // < 2^56
        wl = (uint32_t)w;
        wh = (uint32_t)(w >> 32);
      }
      constexpr int kG = KG;
      const uint32_t rowa = (A.ablate & 4) ? 0u : row;  // diagnostics: every gather hits row 0
      // the batch's group loop; ONES: a full batch whose counts are all 1 (lanes past a
      // piece have c = 0, so a partial batch takes the general path, which adds 0 for them)
      auto groups = [&](auto ones) {
        constexpr bool O = decltype(ones)::value;
        uint32_t bA[kG][NJ], bB[kG][NJ];
        hist_load_group<NJ, kG, GW>(binsr, S, rowa, 0, posr, bA);
#pragma unroll
        for (int g = 0; g < 64 / kG; g += 2) {
          if ((g + 1) * kG < n) hist_load_group<NJ, kG, GW>(binsr, S, rowa, (g + 1) * kG, posr, bB);
          if (!(A.ablate & 8))
            hist_add_group<MODE, NJ, kG, GW, O>(smem, g * kG, bA, wl, wh, amul, abase, bsh);
          if ((g + 1) * kG >= n) break;
          if (g + 2 < 64 / kG && (g + 2) * kG < n)
            hist_load_group<NJ, kG, GW>(binsr, S, rowa, (g + 2) * kG, posr, bA);
          if (!(A.ablate & 8))
            hist_add_group<MODE, NJ, kG, GW, O>(smem, (g + 1) * kG, bB, wl, wh, amul, abase, bsh);
          if ((g + 2) * kG >= n) break;
        }
      };
      if (GINI && __all(c == 1u))
        groups(std::true_type{});
      else
        groups(std::false_type{});
    }
  }
  if (cur_slot >= 0 && !(A.ablate & 1)) {
    block_sync();
    hist_flush<MODE>(A, smem, plane, cur_slot, ft0, cur_ftn, c0, nct, cur_store);
  }
}

// ----------------------------------------------------------------------
// k_hist_rl: the row-lane layout, for feature tiles that would leave lane groups
// idle (F = 100 fills 100 of k_hist's 128 lanes).  kRlG lanes share an entry and
// 64 / kRlG entries share a wave-instruction; lane (e, s) adds features
// [s*K, s*K + K) of entry e, K = ceil(FT / kRlG), so one wave-instruction carries
// roundup(FT, 16) useful-or-dump lanes per 4 entries instead of roundup(FT, 64) per
// entry (F = 100: 112 vs 128 LDS atomics per 4 entries).  Four lanes share a
// feature in each instruction; at 4 the bank conflicts of skewed bins stay at
// k_hist's level (scripts/micro/lds_rl.hip; 8 or 16 lanes per feature double them).
// A lane reads its K bytes with aligned dword loads realigned by v_alignbyte.
// Lanes past the tile add into the LDS row's pad columns [ftn, FPH), which the flush
// never reads: they read row padding or the next features' bins, all < NB (row
// padding and the buffers' slack are zero).  Requires the identity byte layout
// (pos[r][f] = f) and, for variance, cshift >= 32.
// ----------------------------------------------------------------------
constexpr int kRlG = 16;                 // lanes per entry
constexpr int kRlEP = 64 / kRlG;         // entries per wave-instruction

// raw dwords covering a lane's byte range [off, off + K) of one row (the buffers
// carry >= 64 bytes of slack, so the last row's over-read stays in bounds)
template <int K>
struct RlRaw {
  static constexpr int KW = (K + 3) / 4;
  uint32_t d[KW + 1];
};

// OFF32: rows * S < 2^32 and rows < 2^24, so the row offset is one v_mad_u32_u24 off an
// SGPR base; otherwise a 64-bit address per lane
template <int K, bool OFF32>
__device__ __forceinline__ void rl_load(const uint8_t* __restrict__ binsr, uint32_t loff,
                                        uint32_t S, uint32_t row, RlRaw<K>& r) {
  const uint32_t* p = OFF32 ? (const uint32_t*)(binsr + (uint32_t)(__umul24(row, S) + loff))
                            : (const uint32_t*)(binsr + (size_t)row * S + loff);
#pragma unroll
  for (int d = 0; d <= RlRaw<K>::KW; d++) r.d[d] = p[d];
}

// one pass: K LDS atomics of the lane's entry (weights wl/wh, LDS base lb)
template <int MODE, int K>
__device__ __forceinline__ void rl_add(unsigned char* smem, const RlRaw<K>& r, uint32_t sh,
                                       uint32_t amul, uint32_t lb, uint32_t wl, uint32_t wh) {
  constexpr int KW = RlRaw<K>::KW;
  constexpr uint32_t WB = MODE == kHistGini ? 4u : 8u;
  uint32_t w[KW];
#pragma unroll
  for (int q = 0; q < KW; q++) w[q] = __builtin_amdgcn_alignbyte(r.d[q + 1], r.d[q], sh);
  const unsigned long long a64 = ((unsigned long long)wh << 32) | wl;
#pragma unroll
  for (int j = 0; j < K; j++) {
    const uint32_t bin = __builtin_amdgcn_ubfe(w[j >> 2], 8 * (j & 3), 8);
    const uint32_t addr = __umul24(bin, amul) + lb + (uint32_t)j * WB;
    if (MODE == kHistGini)
      atomicAdd((uint32_t*)(smem + addr), wl);
    else
      atomicAdd((unsigned long long*)(smem + addr), a64);
  }
}

// stat words of one entry: u64 modes add (wh:wl); gini adds the count wl into its class
// plane (lb offset).  Variance: (c << cshift) + c*(k + K0) with cshift >= 32 and
// c*(k + K0) < 2^32, i.e. wh = c << (cshift - 32), wl = c*(k + K0).
template <int MODE>
__device__ __forceinline__ void rl_words(uint64_t e, int csh, int32_t K0, int c0, uint32_t cstride,
                                         uint32_t& wl, uint32_t& wh, uint32_t& lb) {
  const int32_t hi = (int32_t)(e >> 32);
  const uint32_t c = (uint32_t)hi & 0xffu;
  const int32_t k = hi >> 8;
  if (MODE == kHistGini) {
    wl = c;
    wh = 0;
    lb += c ? (uint32_t)(k - c0) * cstride : 0u;
  } else if (MODE == kHistVar) {
    wl = __umul24(c, (uint32_t)(k + K0));
    wh = c << csh;
  } else {
    const uint64_t w = (uint64_t)c * (uint64_t)((int64_t)k * (int64_t)k);
    wl = (uint32_t)w;
    wh = (uint32_t)(w >> 32);
  }
}

struct RlLane {  // per-lane constants of the current (replica, tile)
  const uint8_t* binsr;  // bins of the replica (wave-uniform)
  uint32_t loff;         // off & ~3: the lane's first aligned byte in a row
  uint32_t sh;           // off & 3
  uint32_t lb;           // LDS byte offset of feature s*K
};

// one batch of n <= 64 entries (16 passes of 4 entries), row bytes two passes ahead and
// entries three passes ahead.  FULL: n == 64 from global memory, no bounds checks.
// src: the batch's entries, global (ent_in + q0) or the wave's LDS stage.
template <int MODE, int K, bool OFF32, bool FULL, int PD>
__device__ __forceinline__ void rl_batch(unsigned char* smem, const uint64_t* src, int n,
                                         int eo, const RlLane& L, uint32_t S, uint32_t amul,
                                         int csh, int32_t K0, int c0, uint32_t cstride) {
  // rows PD passes ahead, entries PD + 1
  const int npass = FULL ? 16 : (n + kRlEP - 1) / kRlEP;
  auto fetch = [&](int t) -> uint64_t {
    const int i = t * kRlEP + eo;
    if (FULL) return src[i];
    return i < n ? src[i] : 0ull;
  };
  uint64_t ev[PD + 2];
  RlRaw<K> rb[PD + 1];
#pragma unroll
  for (int j = 0; j <= PD; j++) ev[j] = (FULL || j < npass) ? fetch(j) : 0ull;
  ev[PD + 1] = 0;
#pragma unroll
  for (int j = 0; j < PD; j++)
    if (FULL || j < npass) rl_load<K, OFF32>(L.binsr, L.loff, S, (uint32_t)ev[j], rb[j]);
#pragma unroll
  for (int t = 0; t < 16; t++) {
    if (!FULL && t >= npass) break;
    if (FULL ? t + PD + 1 < 16 : t + PD + 1 < npass) ev[PD + 1] = fetch(t + PD + 1);
    if (FULL ? t + PD < 16 : t + PD < npass)
      rl_load<K, OFF32>(L.binsr, L.loff, S, (uint32_t)ev[PD], rb[PD]);
    uint32_t wl, wh, lb = L.lb;
    rl_words<MODE>(ev[0], csh, K0, c0, cstride, wl, wh, lb);
    rl_add<MODE, K>(smem, rb[0], L.sh, amul, lb, wl, wh);
#pragma unroll
    for (int j = 0; j <= PD; j++) ev[j] = ev[j + 1];
#pragma unroll
    for (int j = 0; j < PD; j++) rb[j] = rb[j + 1];
  }
}

template <int MODE, int K, bool OFF32, int PD>
__global__ __launch_bounds__(kHistThreads, 2) void k_hist_rl(HistArgs A) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr bool GINI = MODE == kHistGini;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s = lane % kRlG, eo = lane / kRlG;
  const int NB = A.NB, FPH = A.FPH;
  const uint32_t S = (uint32_t)A.S;
  const int ft0 = (int)(blockIdx.y % (unsigned)A.ntf) * A.FT;
  int c0 = GINI && !A.grouped ? (int)(blockIdx.y / (unsigned)A.ntf) * A.CT : 0;
  int nct = GINI ? min(A.CT, A.NS - c0) : 1;
  const bool ctile = GINI && A.CT < A.NS && !A.grouped;
  constexpr uint32_t WB = GINI ? 4u : 8u;
  const uint32_t plane = hist_plane_bytes(NB, FPH, GINI);
  const uint32_t hist_bytes = plane * (GINI ? (uint32_t)A.CT : 1u);
  uint64_t* stage = (uint64_t*)(smem + hist_bytes) + wave * 64;
  const uint64_t lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  const uint32_t amul = (uint32_t)FPH * WB;
  const int csh = A.cshift - 32;
  const int32_t K0 = A.K0;

  for (uint32_t i = (uint32_t)tid * 16; i < hist_bytes; i += kHistThreads * 16)
    *(uint4*)(smem + i) = make_uint4(0, 0, 0, 0);

  const int p0 = A.wg_piece[blockIdx.x], p1 = A.wg_piece[blockIdx.x + 1];
  int cur_slot = -1, cur_ftn = 0, cur_ftn_lane = -1, cur_tile = -1;
  bool cur_store = false;
  int64_t acc = 0;
  // this lane's byte range of the tile: [off, off + K)
  RlLane L{A.bins, 0u, 0u, (uint32_t)(s * K) * WB};
  block_sync();

  HistChunk pn = p0 < p1 ? A.chunks[p0] : HistChunk{};  // next piece prefetched (k_hist)
  for (int p = p0; p < p1; p++) {
    const HistChunk pc = pn;
    if (p + 1 < p1) pn = A.chunks[p + 1];
    const int r = pc.r;
    const int ftn = min(A.FT, pc.fr - ft0);
    const int slot = pc.slot;
    if (ftn <= 0 || slot < 0) continue;
    const int64_t a = pc.a, b = pc.b;
    const int tile = A.grouped ? pc.tile : 0;
    if (slot != cur_slot || tile != cur_tile || acc + (b - a) > A.flush_limit) {
      if (cur_slot >= 0) {
        block_sync();
        hist_flush<MODE>(A, smem, plane, cur_slot, ft0, cur_ftn, c0, nct, cur_store);
        block_sync();
        for (uint32_t i = (uint32_t)tid * 16; i < hist_bytes; i += kHistThreads * 16)
          *(uint4*)(smem + i) = make_uint4(0, 0, 0, 0);
        block_sync();
      }
      cur_store = (slot != cur_slot || tile != cur_tile) && pc.excl != 0;
      cur_slot = slot;
      cur_tile = tile;
      cur_ftn = ftn;
      acc = 0;
      if (GINI && A.grouped) {
        c0 = tile * A.CT;
        nct = min(A.CT, A.NS - c0);
      }
    }
    acc += b - a;
    if (ftn != cur_ftn_lane) {
      // lanes wholly past the tile read its first bytes (into pad columns)
      const uint32_t off = (uint32_t)(ft0 + (s * K < ftn ? s * K : 0));
      L.loff = off & ~3u;
      L.sh = off & 3u;
      cur_ftn_lane = ftn;
    }
    L.binsr = A.bins + (int64_t)r * A.bins_rstride;
    for (int64_t q0 = a + (int64_t)wave * 64; q0 < b; q0 += (int64_t)kHistWaves * 64) {
      const int n = (int)min((int64_t)64, b - q0);
      if (ctile) {  // keep the batch entries of classes [c0, c0 + nct), packed to the front
        const uint64_t e = (lane < n) ? A.ent_in[q0 + lane] : 0ull;
        const int32_t eh = (int32_t)(e >> 32);
        const int kc = eh >> 8;
        const bool m = ((eh & 0xff) != 0) && kc >= c0 && kc < c0 + nct;
        const uint64_t mask = __ballot(m);
        const int nm = __popcll(mask);
        __builtin_amdgcn_wave_barrier();
        if (m) stage[__popcll(mask & lt_mask)] = e;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (nm > 0)
          rl_batch<MODE, K, OFF32, false, PD>(smem, stage, nm, eo, L, S, amul, csh, K0, c0, plane);
        __builtin_amdgcn_wave_barrier();
      } else if (n == 64) {
        rl_batch<MODE, K, OFF32, true, PD>(smem, A.ent_in + q0, 64, eo, L, S, amul, csh, K0, c0, plane);
      } else {
        rl_batch<MODE, K, OFF32, false, PD>(smem, A.ent_in + q0, n, eo, L, S, amul, csh, K0, c0, plane);
      }
    }
  }
  if (cur_slot >= 0) {
    block_sync();
    hist_flush<MODE>(A, smem, plane, cur_slot, ft0, cur_ftn, c0, nct, cur_store);
  }
}

template <int K, bool OFF32, int PD>
static void launch_hist_rl_kop(hipStream_t st, const HistArgs& a, dim3 grid, size_t lds, int mode) {
  for (const void* f : {(const void*)k_hist_rl<kHistGini, K, OFF32, PD>,
                        (const void*)k_hist_rl<kHistVar, K, OFF32, PD>,
                        (const void*)k_hist_rl<kHistSq, K, OFF32, PD>})
    set_max_lds(f, 160 * 1024);
  if (mode == kHistGini)
    hipLaunchKernelGGL((k_hist_rl<kHistGini, K, OFF32, PD>), grid, dim3(kHistThreads), lds, st, a);
  else if (mode == kHistVar)
    hipLaunchKernelGGL((k_hist_rl<kHistVar, K, OFF32, PD>), grid, dim3(kHistThreads), lds, st, a);
  else
    hipLaunchKernelGGL((k_hist_rl<kHistSq, K, OFF32, PD>), grid, dim3(kHistThreads), lds, st, a);
}

template <int K, bool OFF32>
static void launch_hist_rl_ko(hipStream_t st, const HistArgs& a, dim3 grid, size_t lds, int mode) {
  // rows four passes ahead (HistArgs.rlpd documents it; 2, 3 and 5 were measured, 4 is
  // the one built)
  launch_hist_rl_kop<K, OFF32, 4>(st, a, grid, lds, mode);
}

template <int K>
static void launch_hist_rl_k(hipStream_t st, const HistArgs& a, dim3 grid, size_t lds, int mode) {
  if (a.rl == 2)
    launch_hist_rl_ko<K, true>(st, a, grid, lds, mode);
  else
    launch_hist_rl_ko<K, false>(st, a, grid, lds, mode);
}

static void launch_hist_rl(hipStream_t st, const HistArgs& a, dim3 grid, size_t lds, int mode) {
  switch ((a.FT + kRlG - 1) / kRlG) {
    case 1: launch_hist_rl_k<1>(st, a, grid, lds, mode); break;
    case 2: launch_hist_rl_k<2>(st, a, grid, lds, mode); break;
    case 3: launch_hist_rl_k<3>(st, a, grid, lds, mode); break;
    case 4: launch_hist_rl_k<4>(st, a, grid, lds, mode); break;
    case 5: launch_hist_rl_k<5>(st, a, grid, lds, mode); break;
    case 6: launch_hist_rl_k<6>(st, a, grid, lds, mode); break;
    case 7: launch_hist_rl_k<7>(st, a, grid, lds, mode); break;
    case 8: launch_hist_rl_k<8>(st, a, grid, lds, mode); break;
    case 9: launch_hist_rl_k<9>(st, a, grid, lds, mode); break;
    case 10: launch_hist_rl_k<10>(st, a, grid, lds, mode); break;
    case 11: launch_hist_rl_k<11>(st, a, grid, lds, mode); break;
    case 12: launch_hist_rl_k<12>(st, a, grid, lds, mode); break;
    case 13: launch_hist_rl_k<13>(st, a, grid, lds, mode); break;
    case 14: launch_hist_rl_k<14>(st, a, grid, lds, mode); break;
    case 15: launch_hist_rl_k<15>(st, a, grid, lds, mode); break;
    default: launch_hist_rl_k<16>(st, a, grid, lds, mode); break;
  }
}

size_t hist_rl_lds_bytes(int NB, int CT, int FPH, bool gini) {
  return (size_t)hist_plane_bytes(NB, FPH, gini) * (gini ? (size_t)CT : 1u) +
         (size_t)kHistWaves * 64 * 8;
}
int hist_rl_lanes() { return kRlG; }

size_t hist_lds_bytes(int NB, int NS, int FPH, bool gini) {
  return (size_t)hist_plane_bytes(NB, FPH, gini) * (gini ? (size_t)NS : 1u);
}
size_t hist_stage_bytes() { return (size_t)kHistWaves * 64 * 8; }

template <int MODE, int NJ>
static void launch_hist_t(hipStream_t st, const HistArgs& a, dim3 grid, size_t lds_bytes) {
  if constexpr (MODE == kHistGini && NJ == 1) {
    if (a.small && a.dw == 4) {
      set_max_lds((const void*)k_hist<MODE, NJ, 4, 256, 32>, 160 * 1024);
      hipLaunchKernelGGL((k_hist<MODE, NJ, 4, 256, 32>), grid, dim3(256), lds_bytes, st, a);
      return;
    }
  }
  if (a.dw == 4) {
    set_max_lds((const void*)k_hist<MODE, NJ, 4>, 160 * 1024);
    hipLaunchKernelGGL((k_hist<MODE, NJ, 4>), grid, dim3(kHistThreads), lds_bytes, st, a);
  } else {
    set_max_lds((const void*)k_hist<MODE, NJ, 1>, 160 * 1024);
    hipLaunchKernelGGL((k_hist<MODE, NJ, 1>), grid, dim3(kHistThreads), lds_bytes, st, a);
  }
}

template <int MODE>
static void launch_hist_m(hipStream_t st, const HistArgs& a, dim3 grid, size_t lds_bytes) {
  switch ((a.FT + 63) / 64) {  // 64-feature lane groups per tile (FT <= 256)
    case 1: launch_hist_t<MODE, 1>(st, a, grid, lds_bytes); break;
    case 2: launch_hist_t<MODE, 2>(st, a, grid, lds_bytes); break;
    case 3: launch_hist_t<MODE, 3>(st, a, grid, lds_bytes); break;
    default: launch_hist_t<MODE, 4>(st, a, grid, lds_bytes); break;
  }
}

// ---- class-tile grouping (gini with more classes than one workgroup's LDS holds).
// Without it every class tile's workgroups stream all entries of a node and keep only
// their own (ballot + stage), so an entry is read once per tile.  Per level, the
// entries to be histogrammed are instead counted per (piece, tile) and scattered so
// that each (node, tile) is one contiguous sub-segment; the histogram kernels then
// read every entry once, in full batches.  Order inside a sub-segment is free: the
// class counts are integers.
constexpr int kTileThreads = 256;

__global__ __launch_bounds__(kTileThreads) void k_tile_count(const HistChunk* __restrict__ pieces,
                                                             const uint64_t* __restrict__ ent,
                                                             int CT, int ntc,
                                                             uint32_t* __restrict__ counts) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* cnt = (uint32_t*)smem;
  const HistChunk pc = pieces[blockIdx.x];
  for (int t = threadIdx.x; t < ntc; t += kTileThreads) cnt[t] = 0;
  block_sync();
  for (int64_t i = pc.a + threadIdx.x; i < pc.b; i += kTileThreads) {
    const int k = (int32_t)(ent[i] >> 32) >> 8;
    atomicAdd(&cnt[k / CT], 1u);
  }
  block_sync();
  for (int t = threadIdx.x; t < ntc; t += kTileThreads)
    counts[(int64_t)blockIdx.x * ntc + t] = cnt[t];
}

__global__ __launch_bounds__(kTileThreads) void k_tile_scatter(const HistChunk* __restrict__ pieces,
                                                               const uint64_t* __restrict__ ent,
                                                               int CT, int ntc,
                                                               const int64_t* __restrict__ base,
                                                               uint64_t* __restrict__ ent_out) {
  extern __shared__ __align__(16) unsigned char smem[];
  int64_t* cur = (int64_t*)smem;  // [ntc] next output position of each tile
  const HistChunk pc = pieces[blockIdx.x];
  for (int t = threadIdx.x; t < ntc; t += kTileThreads) cur[t] = base[(int64_t)blockIdx.x * ntc + t];
  block_sync();
  for (int64_t i = pc.a + threadIdx.x; i < pc.b; i += kTileThreads) {
    const uint64_t e = ent[i];
    const int k = (int32_t)(e >> 32) >> 8;
    const int64_t o = (int64_t)atomicAdd((unsigned long long*)&cur[k / CT], 1ull);
    ent_out[o] = e;
  }
}

// The grouping when every (segment, tile) size is known on the host (gini with every draw
// count 1, e.g. bags without replacement: the split's class counts are the children's entry
// counts): a workgroup takes a kTkPiece-entry piece of one segment (HistChunk.parent), ranks
// its entries per tile with returning LDS atomics, reserves each tile's run with one global
// atomic on the (segment, tile) cursor (set by the host to the tile's start), and writes the
// entries from registers -- no count pass and no host round trip between them.
constexpr int kTkPer = 16;                              // entries per thread
constexpr int kTkPiece = kTkPer * kTileThreads;         // 4096
__global__ __launch_bounds__(kTileThreads) void k_tile_scatter_known(const HistChunk* __restrict__ pieces,
                                                                     const uint64_t* __restrict__ ent,
                                                                     int CT, int ntc,
                                                                     unsigned long long* __restrict__ cursors,
                                                                     uint64_t* __restrict__ ent_out) {
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned long long* base = (unsigned long long*)smem;  // [ntc] the piece's run of each tile
  uint32_t* cnt = (uint32_t*)(base + ntc);                // [ntc]
  const HistChunk pc = pieces[blockIdx.x];
  const int tid = threadIdx.x;
  for (int t = tid; t < ntc; t += kTileThreads) cnt[t] = 0u;
  block_sync();
  uint64_t e[kTkPer];
  uint32_t tl[kTkPer], rk[kTkPer];
  const int64_t last = pc.b - 1;
#pragma unroll
  for (int u = 0; u < kTkPer; u++) e[u] = ent[min(pc.a + (int64_t)u * kTileThreads + tid, last)];
#pragma unroll
  for (int u = 0; u < kTkPer; u++) {
    const bool valid = pc.a + (int64_t)u * kTileThreads + tid < pc.b;
    tl[u] = (uint32_t)(((int32_t)(e[u] >> 32) >> 8) / CT);
    rk[u] = valid ? atomicAdd(&cnt[tl[u]], 1u) : 0u;
  }
  block_sync();
  for (int t = tid; t < ntc; t += kTileThreads)
    base[t] = cnt[t] ? atomicAdd(&cursors[(int64_t)pc.parent * ntc + t], (unsigned long long)cnt[t]) : 0ull;
  block_sync();
#pragma unroll
  for (int u = 0; u < kTkPer; u++)
    if (pc.a + (int64_t)u * kTileThreads + tid < pc.b) ent_out[base[tl[u]] + rk[u]] = e[u];
}

void launch_tile_scatter_known(hipStream_t st, const HistChunk* pieces, int npieces, const uint64_t* ent,
                               int CT, int ntc, unsigned long long* cursors, uint64_t* ent_out) {
  if (npieces <= 0) return;
  set_max_lds((const void*)k_tile_scatter_known, 160 * 1024);
  hipLaunchKernelGGL(k_tile_scatter_known, dim3((unsigned)npieces), dim3(kTileThreads), (size_t)ntc * 12, st,
                     pieces, ent, CT, ntc, cursors, ent_out);
}
int tile_scatter_known_piece() { return kTkPiece; }

void launch_tile_count(hipStream_t st, const HistChunk* pieces, int npieces, const uint64_t* ent,
                       int CT, int ntc, uint32_t* counts) {
  if (npieces <= 0) return;
  set_max_lds((const void*)k_tile_count, 160 * 1024);
  hipLaunchKernelGGL(k_tile_count, dim3((unsigned)npieces), dim3(kTileThreads), (size_t)ntc * 4, st,
                     pieces, ent, CT, ntc, counts);
}

void launch_tile_scatter(hipStream_t st, const HistChunk* pieces, int npieces, const uint64_t* ent,
                         int CT, int ntc, const int64_t* base, uint64_t* ent_out) {
  if (npieces <= 0) return;
  set_max_lds((const void*)k_tile_scatter, 160 * 1024);
  hipLaunchKernelGGL(k_tile_scatter, dim3((unsigned)npieces), dim3(kTileThreads), (size_t)ntc * 8, st,
                     pieces, ent, CT, ntc, base, ent_out);
}

void launch_hist(hipStream_t st, const HistArgs& a, int nwg, int ntiles, int mode,
                 size_t lds_bytes) {
  const dim3 grid((unsigned)nwg, (unsigned)ntiles);
  if (a.rl) {
    launch_hist_rl(st, a, grid, lds_bytes, mode);
    return;
  }
  if (mode == kHistGini)
    launch_hist_m<kHistGini>(st, a, grid, lds_bytes);
  else if (mode == kHistVar)
    launch_hist_m<kHistVar>(st, a, grid, lds_bytes);
  else
    launch_hist_m<kHistSq>(st, a, grid, lds_bytes);
}

size_t hist_lds_limit() { return 160 * 1024; }

// ---- partition: kPartK entries per lane per step, one cursor atomic per workgroup and
// side for 64 * 4 * kPartK entries.  Pieces are handed out dynamically in split-column order
// (parents of one column interleaved), so at any time the whole GPU gathers from
// one or two columns of the column-major bins copy: a column (N bytes) stays in
// the MALL / L2 while every node that splits on it is routed, instead of each
// sparse 1-byte gather costing its own memory sector.
constexpr int kPartThreads = 256;
constexpr int kPartWaves = kPartThreads / 64;
constexpr int kPartK = 16;  // entries per lane per step (8: C5 partition 30.4 ms per fit, 16: 25.7)

template <bool PLANES>
__global__ __launch_bounds__(kPartThreads) void k_partition(PartArgs A) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  __shared__ int64_t s_a, s_b;
  __shared__ int s_q;
  __shared__ int s_n[2][kPartWaves];
  __shared__ unsigned long long s_base[2];
  for (;;) {
    if (tid == 0) {
      const int64_t p = (int64_t)atomicAdd(A.counter, 1ull);
      const PartPiece pc = p < A.npieces ? A.pieces[p] : PartPiece{-1, 0, 0, 0};
      s_q = pc.q;
      s_a = pc.a;
      s_b = pc.b;
    }
    block_sync();
    const int q = s_q;
    const int64_t pa = s_a, pb = s_b;
    block_sync();
    if (q < 0) break;
    const ParentInfo pi = A.parents[q];
    const uint8_t* col = A.cols + (int64_t)pi.r * A.cols_rstride + (int64_t)pi.pos * A.npad;
    const uint32_t* plane = PLANES ? A.planes + ((int64_t)pi.pos * A.nsp + pi.s) * A.nw32 : nullptr;
    const uint32_t split = (uint32_t)pi.s;
    const bool wlp = pi.write_l != 0, wrp = pi.write_r != 0;
    unsigned long long* cur = A.cursors + 2 * (int64_t)q;
    // every wave runs the same number of steps (barriers inside)
    for (int64_t step0 = pa; step0 < pb; step0 += (int64_t)kPartWaves * 64 * kPartK) {
      const int64_t base = step0 + (int64_t)wave * 64 * kPartK;
      uint64_t e[kPartK];
      uint32_t byte[kPartK];
#pragma unroll
      for (int k = 0; k < kPartK; k++) {
        const int64_t i = base + k * 64 + lane;
        e[k] = i < pb ? A.ent_in[i] : 0ull;
      }
#pragma unroll
      for (int k = 0; k < kPartK; k++) {
        // 1 = goes right (bin > split): one bit of an L2-sized plane, or the column byte
        if (PLANES) {
          const uint32_t row = (uint32_t)e[k];
          byte[k] = (plane[row >> 5] >> (row & 31u)) & 1u;
        } else {
          byte[k] = col[(uint32_t)e[k]] > split ? 1u : 0u;
        }
      }
      uint64_t ml[kPartK], mr[kPartK];
      int nl = 0, nr = 0;
#pragma unroll
      for (int k = 0; k < kPartK; k++) {
        const bool valid = base + k * 64 + lane < pb;
        const bool right = byte[k] != 0u;
        ml[k] = __ballot(valid && !right && wlp);
        mr[k] = __ballot(valid && right && wrp);
        nl += __popcll(ml[k]);
        nr += __popcll(mr[k]);
      }
      if (A.sq_left) {  // exact sum of count*k^2 of the left child (variance stats)
        unsigned long long sq = 0;
#pragma unroll
        for (int k = 0; k < kPartK; k++) {
          const bool valid = base + k * 64 + lane < pb;
          if (valid && byte[k] == 0u) {
            const int32_t hi = (int32_t)(e[k] >> 32);
            const int64_t kk = hi >> 8;
            sq += (unsigned long long)(hi & 0xff) * (unsigned long long)(kk * kk);
          }
        }
        for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
        if (lane == 0 && sq) atomicAdd(&A.sq_left[q], sq);
      }
      if (lane == 0) {
        s_n[0][wave] = nl;
        s_n[1][wave] = nr;
      }
      block_sync();
      if (tid == 0) {
        int tl = 0, tr = 0;
#pragma unroll
        for (int w = 0; w < kPartWaves; w++) {
          tl += s_n[0][w];
          tr += s_n[1][w];
        }
        s_base[0] = tl ? atomicAdd(&cur[0], (unsigned long long)tl) : 0ull;
        s_base[1] = tr ? atomicAdd(&cur[1], (unsigned long long)(-(long long)tr)) - (unsigned long long)tr : 0ull;
      }
      block_sync();
      unsigned long long bl = s_base[0], br = s_base[1];
      for (int w = 0; w < wave; w++) {
        bl += (unsigned long long)s_n[0][w];
        br += (unsigned long long)s_n[1][w];
      }
#pragma unroll
      for (int k = 0; k < kPartK; k++) {
        const uint64_t bit = 1ull << lane;
        if (ml[k] & bit) A.ent_out[bl + __popcll(ml[k] & lt)] = e[k];
        if (mr[k] & bit) A.ent_out[br + __popcll(mr[k] & lt)] = e[k];
        bl += __popcll(ml[k]);
        br += __popcll(mr[k]);
      }
      block_sync();  // s_n / s_base are rewritten by the next step
    }
  }
}

// ---- column-major copy of a row-major byte matrix (the partition's split column:
// the sorted rows of a node segment read ~1 byte each instead of a 128-B line)
__global__ __launch_bounds__(256) void k_transpose(const uint8_t* __restrict__ src, int64_t N,
                                                   int S, int C, uint8_t* __restrict__ dst,
                                                   int64_t npad, int64_t src_rstride,
                                                   int64_t dst_rstride) {
  __shared__ __align__(16) uint8_t t[64][80];
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * 64;
  const int col0 = blockIdx.y * 64;
  src += (int64_t)blockIdx.z * src_rstride;
  dst += (int64_t)blockIdx.z * dst_rstride;
  {
    const int r = tid >> 2, part = tid & 3;
    const int cb = col0 + part * 16;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row0 + r < N && cb < S) v = *(const uint4*)(src + (row0 + r) * S + cb);
    *(uint4*)&t[r][part * 16] = v;
  }
  block_sync();
  const int cl = tid >> 2, rq = tid & 3;
  if (col0 + cl < C) {
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; q++)
      w[q] = (uint32_t)t[rq * 16 + 4 * q][cl] | ((uint32_t)t[rq * 16 + 4 * q + 1][cl] << 8) |
             ((uint32_t)t[rq * 16 + 4 * q + 2][cl] << 16) | ((uint32_t)t[rq * 16 + 4 * q + 3][cl] << 24);
    *(uint4*)(dst + (int64_t)(col0 + cl) * npad + row0 + rq * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

void launch_transpose(hipStream_t st, const uint8_t* src, int64_t N, int S, int C, uint8_t* dst,
                      int64_t npad, int R, int64_t src_rstride, int64_t dst_rstride) {
  const dim3 grid((unsigned)((N + 63) / 64), (unsigned)((C + 63) / 64), (unsigned)R);
  hipLaunchKernelGGL(k_transpose, grid, dim3(256), 0, st, src, N, S, C, dst, npad, src_rstride,
                     dst_rstride);
}

// piece list of k_partition: thread per piece.  A column group's pieces come in
// rounds (piece k of every parent that is long enough, longest parents first).
__global__ __launch_bounds__(256) void k_part_pieces(const PartRound* __restrict__ rounds,
                                                     int nrounds, int64_t npieces,
                                                     const int32_t* __restrict__ order,
                                                     const int64_t* __restrict__ seg, int64_t piece,
                                                     PartPiece* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= npieces) return;
  int lo = 0, hi = nrounds;  // rounds[lo].out0 <= p < rounds[hi].out0
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (rounds[mid].out0 <= p)
      lo = mid;
    else
      hi = mid;
  }
  const PartRound rd = rounds[lo];
  const int q = order[rd.o0 + (int)(p - rd.out0)];
  const int64_t x = seg[2 * q] + rd.off;
  out[p] = PartPiece{q, 0, x, min(x + piece, seg[2 * q + 1])};
}

void launch_part_pieces(hipStream_t st, const PartRound* rounds, int nrounds, int64_t npieces,
                        const int32_t* order, const int64_t* seg, int64_t piece, PartPiece* out) {
  if (npieces <= 0) return;
  hipLaunchKernelGGL(k_part_pieces, dim3((unsigned)((npieces + 255) / 256)), dim3(256), 0, st,
                     rounds, nrounds, npieces, order, seg, piece, out);
}

// side-bit planes of the shared bins for k_partition: bit (row & 31) of word
// row >> 5 of plane (f, s) = bins[row][f] > s.  A plane is N/8 bytes (1.25 MB for C3),
// small enough for an XCD's L2 while the whole GPU routes the nodes split at (f, s).
__global__ __launch_bounds__(256) void k_planes(const uint8_t* __restrict__ cols, int64_t npad,
                                                int nsp, int64_t nw32, uint32_t* __restrict__ planes) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int f = blockIdx.y;
  if (w >= nw32) return;
  const uint32_t* src = (const uint32_t*)(cols + (int64_t)f * npad + w * 32);
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = src[i];
  uint32_t* dst = planes + (int64_t)f * nsp * nw32 + w;
  if (nsp <= 127) {
    // bins < 128: per 4 bytes, (b | 0x80) - (s + 1) keeps bit 7 iff b > s; the four
    // bit-7s are gathered into a nibble with one multiply (no carries collide)
    for (int sp = 0; sp < nsp; sp++) {
      const uint32_t sub = (uint32_t)(sp + 1) * 0x01010101u;
      uint32_t word = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint32_t t = (((v[i] | 0x80808080u) - sub) & 0x80808080u) >> 7;
        word |= ((t * 0x00204081u) >> 21 & 0xfu) << (4 * i);
      }
      dst[(int64_t)sp * nw32] = word;
    }
    return;
  }
  for (int sp = 0; sp < nsp; sp++) {
    uint32_t word = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
      const uint32_t b = (v[i >> 2] >> ((i & 3) * 8)) & 0xffu;
      word |= (b > (uint32_t)sp ? 1u : 0u) << i;
    }
    dst[(int64_t)sp * nw32] = word;
  }
}

void launch_planes(hipStream_t st, const uint8_t* cols, int64_t npad, int ncol, int nsp, int64_t nw32,
                   uint32_t* planes) {
  if (ncol <= 0 || nsp <= 0) return;
  const dim3 grid((unsigned)((nw32 + 255) / 256), (unsigned)ncol);
  hipLaunchKernelGGL(k_planes, grid, dim3(256), 0, st, cols, npad, nsp, nw32, planes);
}

void launch_partition(hipStream_t st, const PartArgs& a, int nwg) {
  if (a.planes)
    hipLaunchKernelGGL(k_partition<true>, dim3((unsigned)nwg), dim3(kPartThreads), 0, st, a);
  else
    hipLaunchKernelGGL(k_partition<false>, dim3((unsigned)nwg), dim3(kPartThreads), 0, st, a);
}

// ======================================================================
// Split search: one workgroup per node slot; thread per local feature does
// the prefix scan over bins and the fp64 gain of every candidate in Spark's
// operation order; first max over splits, then first max over features.
// ======================================================================
__device__ __forceinline__ double var_impurity(int64_t cnt, int64_t sk, uint64_t sq, double is,
                                               double is2) {
  const double count = (double)cnt;
  if (count == 0) return 0.0;
  const double sum = (double)sk * is;
  const double sumsq = (double)sq * is2;
  const double squared_loss = sumsq - (sum * sum) / count;
  return squared_loss / count;
}

template <bool GINI>
__global__ __launch_bounds__(256) void k_split(SplitArgs A) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int slot = A.slot_ids ? A.slot_ids[blockIdx.x] : (int)blockIdx.x, tid = threadIdx.x;
  const int r = A.slot_r[slot];
  const int Fr = A.Fr[r];
  const int NB = A.NB, NS = A.NS;
  const int64_t slot_words = (int64_t)A.Fmax * NB * NS;
  double* s_gain = (double*)smem;
  int* s_fl = (int*)(s_gain + 256);
  int* s_s = s_fl + 256;
  int* s_valid = s_s + 256;
  int64_t* s_tot = (int64_t*)(s_valid + 256);  // [NS]
  uint32_t* s_left = (uint32_t*)(s_tot + NS);  // GINI: [NS][256]
  const int32_t* nb_r = A.nbins + (int64_t)r * A.Fmax;

  // node total = sum over the bins of local feature 0 (every feature sums to it)
  if (GINI) {
    const uint32_t* h = (const uint32_t*)A.hist + (int64_t)slot * slot_words;
    for (int c = tid; c < NS; c += 256) {
      int64_t t = 0;
      for (int b = 0; b < NB; b++) t += h[gini_cell(0, b, c, NB, A.Fmax, A.hct)];
      s_tot[c] = t;
    }
  } else {
    const uint64_t* h = (const uint64_t*)A.hist + (int64_t)slot * slot_words;
    if (tid < 3) {
      int64_t t = 0;
      for (int b = 0; b < NB; b++) t += (int64_t)h[(int64_t)b * 3 + tid];
      s_tot[tid] = t;
    }
  }
  block_sync();

  double bgain = -INFINITY;
  int bfl = INT_MAX, bs = -1, bvalid = 0;
  const double is = A.inv_scale, is2 = A.inv_scale2;
  if (GINI) {
    double ttot = 0.0;
    for (int c = 0; c < NS; c++) ttot += (double)s_tot[c];
    double imp = 0.0;
    if (ttot != 0) {
      imp = 1.0;
      for (int c = 0; c < NS; c++) {
        const double f = (double)s_tot[c] / ttot;
        imp -= f * f;
      }
    }
    const int64_t tcount = (int64_t)ttot;
    uint32_t* left = s_left + tid;  // stride 256
    for (int fl = tid; fl < Fr; fl += 256) {
      const int nsp = nb_r[fl] - 1;
      if (nsp <= 0) continue;
      const uint32_t* h = (const uint32_t*)A.hist + (int64_t)slot * slot_words;
      for (int c = 0; c < NS; c++) left[c * 256] = 0;
      double fg = 0.0;
      int fs = -1, fv = 0;
      for (int s = 0; s < nsp; s++) {
        double lt = 0.0;
        for (int c = 0; c < NS; c++) {
          const uint32_t v = left[c * 256] + h[gini_cell(fl, s, c, NB, A.Fmax, A.hct)];
          left[c * 256] = v;
          lt += (double)v;
        }
        const int64_t lc = (int64_t)lt;
        const int64_t rc = tcount - lc;
        double gain;
        int valid;
        if (lc < A.min_inst || rc < A.min_inst) {
          gain = -DBL_MAX;
          valid = 0;
        } else {
          double li = 0.0, ri = 0.0;
          if (lt != 0) {
            li = 1.0;
            for (int c = 0; c < NS; c++) {
              const double f = (double)left[c * 256] / lt;
              li -= f * f;
            }
          }
          double rt = 0.0;
          for (int c = 0; c < NS; c++) rt += (double)(s_tot[c] - (int64_t)left[c * 256]);
          if (rt != 0) {
            ri = 1.0;
            for (int c = 0; c < NS; c++) {
              const double f = (double)(s_tot[c] - (int64_t)left[c * 256]) / rt;
              ri -= f * f;
            }
          }
          const double lw = (double)lc / (double)(lc + rc);
          const double rw = (double)rc / (double)(lc + rc);
          gain = imp - lw * li - rw * ri;
          valid = 1;
          if (gain < A.min_gain) {
            gain = -DBL_MAX;
            valid = 0;
          }
        }
        if (fs < 0 || gain > fg) {
          fg = gain;
          fs = s;
          fv = valid;
        }
      }
      if (fg > bgain || (fg == bgain && fl < bfl)) {
        bgain = fg;
        bfl = fl;
        bs = fs;
        bvalid = fv;
      }
    }
  } else {
    const int64_t tc = s_tot[0], tsk = s_tot[1];
    const uint64_t tsq = (uint64_t)s_tot[2];
    const double imp = var_impurity(tc, tsk, tsq, is, is2);
    for (int fl = tid; fl < Fr; fl += 256) {
      const int nsp = nb_r[fl] - 1;
      if (nsp <= 0) continue;
      const uint64_t* h = (const uint64_t*)A.hist + (int64_t)slot * slot_words + (int64_t)fl * NB * 3;
      int64_t lc = 0, lsk = 0;
      uint64_t lsq = 0;
      double fg = 0.0;
      int fs = -1, fv = 0;
      for (int s = 0; s < nsp; s++) {
        lc += (int64_t)h[s * 3];
        lsk += (int64_t)h[s * 3 + 1];
        lsq += h[s * 3 + 2];
        const int64_t rc = tc - lc;
        double gain;
        int valid;
        if (lc < A.min_inst || rc < A.min_inst) {
          gain = -DBL_MAX;
          valid = 0;
        } else {
          const double li = var_impurity(lc, lsk, lsq, is, is2);
          const double ri = var_impurity(rc, tsk - lsk, tsq - lsq, is, is2);
          const double lw = (double)lc / (double)(lc + rc);
          const double rw = (double)rc / (double)(lc + rc);
          gain = imp - lw * li - rw * ri;
          valid = 1;
          if (gain < A.min_gain) {
            gain = -DBL_MAX;
            valid = 0;
          }
        }
        if (fs < 0 || gain > fg) {
          fg = gain;
          fs = s;
          fv = valid;
        }
      }
      if (fg > bgain || (fg == bgain && fl < bfl)) {
        bgain = fg;
        bfl = fl;
        bs = fs;
        bvalid = fv;
      }
    }
  }
  s_gain[tid] = bgain;
  s_fl[tid] = bfl;
  s_s[tid] = bs;
  s_valid[tid] = bvalid;
  block_sync();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const double g2 = s_gain[tid + o];
      const int f2 = s_fl[tid + o];
      if (g2 > s_gain[tid] || (g2 == s_gain[tid] && f2 < s_fl[tid])) {
        s_gain[tid] = g2;
        s_fl[tid] = f2;
        s_s[tid] = s_s[tid + o];
        s_valid[tid] = s_valid[tid + o];
      }
    }
    block_sync();
  }
  int64_t* so = A.stats + (int64_t)slot * NS;  // so[k * plane + c]: total, left, right
  if (tid == 0) {
    SplitOut o;
    const int fl = s_fl[0];
    if (fl == INT_MAX) {
      o.gain = -DBL_MAX;
      o.fl = -1;
      o.s = -1;
      o.valid = 0;
    } else {
      o.gain = s_gain[0];
      o.fl = fl;
      o.s = s_s[0];
      o.valid = s_valid[0];
    }
    o.pad = 0;
    A.out[slot] = o;
  }
  const int bf = s_fl[0], bsp = s_s[0];
  for (int c = tid; c < NS; c += 256) {
    int64_t l = 0;
    if (bf != INT_MAX) {
      if (GINI) {
        const uint32_t* h = (const uint32_t*)A.hist + (int64_t)slot * slot_words;
        for (int s = 0; s <= bsp; s++) l += h[gini_cell(bf, s, c, NB, A.Fmax, A.hct)];
      } else {
        const uint64_t* h = (const uint64_t*)A.hist + (int64_t)slot * slot_words + (int64_t)bf * NB * 3;
        for (int s = 0; s <= bsp; s++) l += (int64_t)h[s * 3 + c];
      }
    }
    so[c] = s_tot[c];
    so[A.plane + c] = l;
    so[2 * A.plane + c] = s_tot[c] - l;
  }
}

// ---- variance split screening from (count, sum) only.
// Spark's gain  impurity - wL*imp(L) - wR*imp(R),  imp = (sumSq - sum^2/n)/n,  equals
// g = (S1_L^2/n_L + S1_R^2/n_R - S1^2/n)/n exactly in real arithmetic: the sums of
// squares cancel.  In fp64 both Spark's value G and our g carry rounding errors
// bounded by a few ulps of sumSq/n (S1^2/n <= sumSq by Cauchy-Schwarz, every term of
// both formulas is at most sumSq/n), so |G - g| <= delta = 2^-47 * sumSq/n (= 64 u).
// A candidate whose g beats every other by more than 2*delta is Spark's argmax, and
// g > delta (g >= minInfoGain + delta) decides G > 0 (G >= minInfoGain).  A node
// where that does not hold is flagged (SplitOut.pad = 1): the host histograms its
// sums of squares and reruns the exact k_split on it.
__global__ __launch_bounds__(256) void k_split_screen(SplitArgs A) {
  const int slot = blockIdx.x, tid = threadIdx.x;
  const int r = A.slot_r[slot];
  const int Fr = A.Fr[r];
  const int NB = A.NB;
  const int64_t slot_words = (int64_t)A.Fmax * NB * 3;
  __shared__ double s_g[256];
  __shared__ int s_fl[256], s_s[256], s_cnt[256], s_any[256];
  __shared__ int64_t s_tot[2];
  const int32_t* nb_r = A.nbins + (int64_t)r * A.Fmax;
  const uint64_t* hs = (const uint64_t*)A.hist + (int64_t)slot * slot_words;
  if (tid < 2) {
    int64_t t = 0;
    for (int b = 0; b < NB; b++) t += (int64_t)hs[(int64_t)b * 3 + tid];
    s_tot[tid] = t;
  }
  block_sync();
  const int64_t tc = s_tot[0], tsk = s_tot[1];
  const uint64_t tsq = A.node_sq[slot];
  const double is2 = A.inv_scale2;
  const double n = (double)tc;
  const double delta = tc > 0 ? ldexp((double)tsq * is2 / n, -47) : 0.0;
  const double sp = (double)tsk * (double)tsk / n;
  const double lo_gain = A.min_gain - delta;  // below: invalid in Spark for sure
  // pass 1: best g per feature (first max), any feature with splits
  double fgb = -INFINITY;
  int ffl = INT_MAX, fs = -1, any = INT_MAX;
  for (int fl = tid; fl < Fr; fl += 256) {
    const int nsp = nb_r[fl] - 1;
    if (nsp <= 0) continue;
    any = min(any, fl);
    const uint64_t* h = hs + (int64_t)fl * NB * 3;
    int64_t lc = 0, lsk = 0;
    for (int s = 0; s < nsp; s++) {
      lc += (int64_t)h[s * 3];
      lsk += (int64_t)h[s * 3 + 1];
      const int64_t rc = tc - lc, rsk = tsk - lsk;
      if (lc < A.min_inst || rc < A.min_inst) continue;
      const double g = (((double)lsk * (double)lsk / (double)lc +
                         (double)rsk * (double)rsk / (double)rc) - sp) / n * is2;
      if (g < lo_gain) continue;
      if (g > fgb) {
        fgb = g;
        ffl = fl;
        fs = s;
      }
    }
  }
  s_g[tid] = fgb;
  s_fl[tid] = ffl;
  s_s[tid] = fs;
  s_any[tid] = any;
  block_sync();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const double g2 = s_g[tid + o];
      const int f2 = s_fl[tid + o];
      if (g2 > s_g[tid] || (g2 == s_g[tid] && f2 < s_fl[tid])) {
        s_g[tid] = g2;
        s_fl[tid] = f2;
        s_s[tid] = s_s[tid + o];
      }
      s_any[tid] = min(s_any[tid], s_any[tid + o]);
    }
    block_sync();
  }
  const double gb = s_g[0];
  const int bfl = s_fl[0], bs = s_s[0], first_fl = s_any[0];
  block_sync();
  // pass 2: contenders within 2*delta of the best
  int cnt = 0;
  if (bfl != INT_MAX) {
    const double thr = gb - 2.0 * delta;
    for (int fl = tid; fl < Fr; fl += 256) {
      const int nsp = nb_r[fl] - 1;
      const uint64_t* h = hs + (int64_t)fl * NB * 3;
      int64_t lc = 0, lsk = 0;
      for (int s = 0; s < nsp; s++) {
        lc += (int64_t)h[s * 3];
        lsk += (int64_t)h[s * 3 + 1];
        const int64_t rc = tc - lc, rsk = tsk - lsk;
        if (lc < A.min_inst || rc < A.min_inst) continue;
        const double g = (((double)lsk * (double)lsk / (double)lc +
                           (double)rsk * (double)rsk / (double)rc) - sp) / n * is2;
        if (g >= lo_gain && g >= thr) cnt++;
      }
    }
  }
  s_cnt[tid] = cnt;
  block_sync();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) s_cnt[tid] += s_cnt[tid + o];
    block_sync();
  }
  if (tid == 0) {
    SplitOut o;
    int64_t* so = A.stats + (int64_t)slot * 3;  // NS = 3; so[k * plane + c]
    const int64_t P = A.plane;
    so[0] = tc;
    so[1] = tsk;
    so[2] = (int64_t)tsq;
    if (bfl == INT_MAX) {  // every candidate is invalid in Spark: leaf
      o.gain = -DBL_MAX;
      o.fl = first_fl == INT_MAX ? -1 : first_fl;
      o.s = first_fl == INT_MAX ? -1 : 0;
      o.valid = 0;
      o.pad = 0;
      so[P] = so[P + 1] = so[P + 2] = so[2 * P] = so[2 * P + 1] = so[2 * P + 2] = 0;
    } else {
      const bool flag = s_cnt[0] > 1 || gb < A.min_gain + delta || gb <= delta;
      o.gain = gb;
      o.fl = bfl;
      o.s = bs;
      o.valid = 1;
      o.pad = flag ? 1 : 0;
      const uint64_t* h = hs + (int64_t)bfl * NB * 3;
      int64_t lc = 0, lsk = 0;
      for (int s = 0; s <= bs; s++) {
        lc += (int64_t)h[s * 3];
        lsk += (int64_t)h[s * 3 + 1];
      }
      so[P] = lc;
      so[P + 1] = lsk;
      so[P + 2] = -1;  // left sum of squares: from k_partition
      so[2 * P] = tc - lc;
      so[2 * P + 1] = tsk - lsk;
      so[2 * P + 2] = -1;
    }
    A.out[slot] = o;
  }
}

void launch_split_screen(hipStream_t st, const SplitArgs& a, int M) {
  hipLaunchKernelGGL(k_split_screen, dim3(M), dim3(256), 0, st, a);
}

// zero word `word` of every (feature, bin) cell of the listed slots
__global__ __launch_bounds__(256) void k_zero_word(uint64_t* __restrict__ hist,
                                                   const int32_t* __restrict__ slots,
                                                   int64_t slot_words, int stride, int word) {
  uint64_t* h = hist + (int64_t)slots[blockIdx.y] * slot_words;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < slot_words / stride;
       i += (int64_t)gridDim.x * 256)
    h[i * stride + word] = 0;
}

void launch_zero_word(hipStream_t st, uint64_t* hist, const int32_t* d_slots, int nslots,
                      int64_t slot_words, int stride, int word) {
  if (nslots <= 0) return;
  const unsigned gx = (unsigned)std::min<int64_t>((slot_words / stride + 255) / 256, 64);
  hipLaunchKernelGGL(k_zero_word, dim3(gx, (unsigned)nslots), dim3(256), 0, st, hist, d_slots,
                     slot_words, stride, word);
}

// ---- gini split search with every thread on a candidate.  k_split<true> ran one
// thread per feature (100 of 256 busy) through 31 splits x 2C fp64 divisions each;
// with 64 classes (BASELINE config 5) that dominated a level.  Here a block stages
// the bin-prefix counts of a group of G features in LDS ([f][bin][class] u32) and
// gives each thread one (feature, split) candidate; the arithmetic of a candidate is
// k_split<true>'s, in Spark's operation order (ImpurityCalculator.count = sequential
// class sum, Gini.calculate = 1 - sum freq^2 in class order), and the block argmax
// keeps Spark's first max (maxBy over splits, then over features).
// stage the raw [g][NB][NS] u32 histogram of features [f0, f0 + g) (contiguous in the
// slot) into LDS rows of NS + 1 words, features split_fstride() words apart, 16-byte
// loads with several in flight per thread, then prefix sums over bins in place (a
// thread per (feature, class)).  Candidate q = fl * (NB - 1) + sp reads row (fl, sp) at
// word q * (NS + 1) + c (mod 64): with NS + 1 odd the 64 candidates of a wave fall on 64
// distinct banks (a plain NB * (NS + 1) feature stride put features 0 and 2 of a wave on
// the same banks: 24 % of the kernel's LDS cycles were conflicts on C5)
__host__ __device__ inline int split_fstride(int NB, int NS) {
  const int NSP = NS + 1;
  return NB * NSP + (((NB - 1) * NSP - NB * NSP) % 64 + 64) % 64;
}
// (ps, hw: a derived slot -- the staged words are parent ps - smaller child hs, and are also
// written to hw, the slot's own histogram for the next level; hw null: no next level)
__device__ __forceinline__ void split_stage_prefix(const uint32_t* __restrict__ hs, int f0, int g,
                                                   int NB, int NS, int Fmax, int hct,
                                                   uint32_t* pre, const uint32_t* __restrict__ ps = nullptr,
                                                   uint32_t* __restrict__ hw = nullptr) {
  // features [f0, f0 + g) of each layout class tile t are one contiguous run of g*NB*hct
  // words (gini_cell); staged as pre[fl][b][c] with the class row padded to NS + 1
  const int tid = threadIdx.x;
  const int NSP = NS + 1, FS = split_fstride(NB, NS);
  const int ntc = NS / hct;
  const int64_t per_t = (int64_t)g * NB * hct;
  if ((hct & 3) == 0) {
    const int hct4 = hct >> 2, per_t4 = (int)(per_t >> 2), n4 = ntc * per_t4;
    auto src4 = [&](int q) {
      const int t = q / per_t4, rem = q - t * per_t4;
      const int64_t o = ((int64_t)t * Fmax + f0) * NB * hct;
      uint4 v = ((const uint4*)(hs + o))[rem];
      if (ps) {
        const uint4 pv = ((const uint4*)(ps + o))[rem];
        v = make_uint4(pv.x - v.x, pv.y - v.y, pv.z - v.z, pv.w - v.w);
        if (hw) ((uint4*)(hw + o))[rem] = v;
      }
      return v;
    };
    auto put = [&](int q, const uint4& v) {
      const int t = q / per_t4, rem = q - t * per_t4;
      const int row = rem / hct4, c = t * hct + (rem - row * hct4) * 4;
      const int fl = row / NB;
      uint32_t* d = pre + (size_t)fl * FS + (size_t)(row - fl * NB) * NSP + c;
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    };
    int q = tid;
    for (; q + 3 * 256 < n4; q += 4 * 256) {
      const uint4 v0 = src4(q), v1 = src4(q + 256), v2 = src4(q + 512), v3 = src4(q + 768);
      put(q, v0);
      put(q + 256, v1);
      put(q + 512, v2);
      put(q + 768, v3);
    }
    for (; q < n4; q += 256) put(q, src4(q));
  } else {
    const int64_t words = (int64_t)ntc * per_t;
    for (int64_t q = tid; q < words; q += 256) {
      const int t = (int)(q / per_t);
      const int64_t rem = q - (int64_t)t * per_t;
      const int row = (int)(rem / hct), c = t * hct + (int)(rem - (int64_t)row * hct);
      const int fl = row / NB;
      const int64_t o = ((int64_t)t * Fmax + f0) * NB * hct + rem;
      uint32_t v = hs[o];
      if (ps) {
        v = ps[o] - v;
        if (hw) hw[o] = v;
      }
      pre[(size_t)fl * FS + (size_t)(row - fl * NB) * NSP + c] = v;
    }
  }
  block_sync();
  // (16 bins read before any is written back: one LDS round trip per 16 bins -- the plain
  // read-add-write chain waited out a round trip per bin, 32 per group on C5)
  for (int q = tid; q < g * NS; q += 256) {
    const int fl = q / NS, c = q - fl * NS;
    uint32_t* o = pre + (size_t)fl * FS + c;
    uint32_t acc = 0;
    int b = 0;
    for (; b + 16 <= NB; b += 16) {
      uint32_t v[16];
#pragma unroll
      for (int u = 0; u < 16; u++) v[u] = o[(size_t)(b + u) * NSP];
#pragma unroll
      for (int u = 0; u < 16; u++) {
        acc += v[u];
        o[(size_t)(b + u) * NSP] = acc;
      }
    }
    for (; b < NB; b++) {
      acc += o[(size_t)b * NSP];
      o[(size_t)b * NSP] = acc;
    }
  }
  block_sync();
}

__global__ __launch_bounds__(256) void k_split_gini(SplitArgs A, int G) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int slot = A.slot_ids ? A.slot_ids[blockIdx.x] : (int)blockIdx.x, tid = threadIdx.x;
  const int r = A.slot_r[slot];
  const int Fr = A.Fr[r];
  const int NB = A.NB, NS = A.NS, NSP = NS + 1, FS = split_fstride(NB, NS);
  const int64_t slot_words = (int64_t)A.Fmax * NB * NS;
  const uint32_t* hs = (const uint32_t*)A.hist + (int64_t)slot * slot_words;
  // a derived slot (the larger child): staged as parent - smaller child, written to its own
  // histogram on the way (k_subtract fused in)
  const uint32_t* ps = nullptr;
  uint32_t* hw = nullptr;
  if (A.derive && A.derive[2 * slot] >= 0) {
    ps = (const uint32_t*)A.par_hist + (int64_t)A.derive[2 * slot] * slot_words;
    hw = A.hist_w ? (uint32_t*)A.hist_w + (int64_t)slot * slot_words : nullptr;
    hs = (const uint32_t*)A.hist + (int64_t)A.derive[2 * slot + 1] * slot_words;
  }
  const int32_t* nb_r = A.nbins + (int64_t)r * A.Fmax;
  int64_t* s_tot = (int64_t*)smem;                      // [NS]
  double* s_gain = (double*)(s_tot + NS);               // [256]
  int* s_key = (int*)(s_gain + 256);                    // [256] fl * 65536 + s (INT_MAX: none)
  int* s_valid = s_key + 256;                           // [256]
  double* s_wmax = (double*)(s_valid + 256);            // [2][4] per-wave best, by group parity
  uint32_t* pre = (uint32_t*)(s_wmax + 8);              // [G][NB][NS + 1] prefix over bins
  // group 0 first: the node totals are feature 0's last prefix
  split_stage_prefix(hs, 0, min(G, Fr), NB, NS, A.Fmax, A.hct, pre, ps, hw);
  for (int c = tid; c < NS; c += 256) s_tot[c] = (int64_t)pre[(size_t)(NB - 1) * NSP + c];
  block_sync();
  double ttot = 0.0;
  for (int c = 0; c < NS; c++) ttot += (double)s_tot[c];
  double imp = 0.0;
  if (ttot != 0) {
    imp = 1.0;
    for (int c = 0; c < NS; c++) {
      const double f = (double)s_tot[c] / ttot;
      imp -= f * f;
    }
  }
  const int64_t tcount = (int64_t)ttot;
  double bgain = -INFINITY;
  int bkey = INT_MAX, bvalid = 0;
  // Screen: a candidate whose cheap gain (1 - sum l^2 / lt^2: two divisions instead of
  // two per class) lies below the block's best exact gain of the earlier feature groups by
  // more than kGiniScreen cannot be the argmax or tie it (the two formulas differ by
  // rounding only, < 1e-11 for up to 4096 classes), so only the others run Spark's
  // per-class Gini.calculate.  thr is exact, so the chosen split is unchanged.
  constexpr double kGiniScreen = 1e-9;
  double thr = -INFINITY;
  int grp = 0;
  for (int f0 = 0; f0 < Fr; f0 += G, grp++) {
    const int g = min(G, Fr - f0);
    if (f0 > 0) {
      // per-wave maxima of the running best, written after the previous group
      const double* wm = s_wmax + ((grp - 1) & 1) * 4;
      block_sync();  // previous group's prefix no longer read; wm visible
      thr = fmax(fmax(wm[0], wm[1]), fmax(wm[2], wm[3]));
      split_stage_prefix(hs, f0, g, NB, NS, A.Fmax, A.hct, pre, ps, hw);
    }
    for (int q = tid; q < g * (NB - 1); q += 256) {
      const int fl = q / (NB - 1), sp = q - fl * (NB - 1);
      const int nsp = nb_r[f0 + fl] - 1;
      if (sp >= nsp) continue;
      const uint32_t* left = pre + (size_t)fl * FS + (size_t)sp * NSP;
      // class sums of integers: exact in any order
      double lt = 0.0, rt = 0.0;
#pragma unroll 8
      for (int c = 0; c < NS; c++) {
        const uint32_t l = left[c];
        lt += (double)l;
        rt += (double)(s_tot[c] - (int64_t)l);
      }
      const int64_t lc = (int64_t)lt;
      const int64_t rc = tcount - lc;
      double gain;
      int valid;
      const double lw = (double)lc / (double)(lc + rc);
      const double rw = (double)rc / (double)(lc + rc);
      bool screened = false;
      if (lc >= A.min_inst && rc >= A.min_inst && thr > -DBL_MAX) {
        double sl = 0.0, sr = 0.0;
#pragma unroll 8
        for (int c = 0; c < NS; c++) {
          const double l = (double)left[c], r = (double)(s_tot[c] - (int64_t)left[c]);
          sl = fma(l, l, sl);
          sr = fma(r, r, sr);
        }
        const double apx = imp - lw * (1.0 - sl / (lt * lt)) - rw * (1.0 - sr / (rt * rt));
        screened = apx < thr - kGiniScreen;
      }
      if (screened) continue;
      if (lc < A.min_inst || rc < A.min_inst) {
        gain = -DBL_MAX;
        valid = 0;
      } else {
        // Gini.calculate of both children: 1 - sum freq^2 in class order
        double li = lt != 0 ? 1.0 : 0.0, ri = rt != 0 ? 1.0 : 0.0;
#pragma unroll 8
        for (int c = 0; c < NS; c++) {
          const uint32_t l = left[c];
          const double fl_ = (double)l / lt;
          const double fr_ = (double)(s_tot[c] - (int64_t)l) / rt;
          if (lt != 0) li -= fl_ * fl_;
          if (rt != 0) ri -= fr_ * fr_;
        }
        gain = imp - lw * li - rw * ri;
        valid = 1;
        if (gain < A.min_gain) {
          gain = -DBL_MAX;
          valid = 0;
        }
      }
      const int key = (f0 + fl) * 65536 + sp;
      if (gain > bgain || (gain == bgain && key < bkey)) {
        bgain = gain;
        bkey = key;
        bvalid = valid;
      }
    }
    double wmx = bgain;  // this wave's best exact gain so far -> the next group's screen
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wmx = fmax(wmx, __shfl_xor(wmx, o));
    if ((tid & 63) == 0) s_wmax[(grp & 1) * 4 + (tid >> 6)] = wmx;
  }
  s_gain[tid] = bgain;
  s_key[tid] = bkey;
  s_valid[tid] = bvalid;
  block_sync();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const double g2 = s_gain[tid + o];
      const int k2 = s_key[tid + o];
      if (g2 > s_gain[tid] || (g2 == s_gain[tid] && k2 < s_key[tid])) {
        s_gain[tid] = g2;
        s_key[tid] = k2;
        s_valid[tid] = s_valid[tid + o];
      }
    }
    block_sync();
  }
  const int key = s_key[0];
  const int bf = key == INT_MAX ? -1 : key / 65536, bsp = key == INT_MAX ? -1 : key % 65536;
  int64_t* so = A.stats + (int64_t)slot * NS;  // so[k * plane + c]: total, left, right
  if (tid == 0) {
    SplitOut o;
    if (key == INT_MAX) {
      o.gain = -DBL_MAX;
      o.fl = -1;
      o.s = -1;
      o.valid = 0;
    } else {
      o.gain = s_gain[0];
      o.fl = bf;
      o.s = bsp;
      o.valid = s_valid[0];
    }
    o.pad = 0;
    A.out[slot] = o;
  }
  // left stats of the best split: bins [0, bsp] of feature bf, 8 loads in flight
  for (int c = tid; c < NS; c += 256) {
    int64_t l = 0;
    if (bf >= 0) {
      // bins of (bf, c) are hct words apart (gini_cell)
      const int hct = A.hct;
      auto bins_sum = [&](const uint32_t* h) {
        int64_t acc = 0;
        int sb = 0;
        for (; sb + 8 <= bsp + 1; sb += 8) {
          uint32_t v[8];
#pragma unroll
          for (int u = 0; u < 8; u++) v[u] = h[(int64_t)(sb + u) * hct];
#pragma unroll
          for (int u = 0; u < 8; u++) acc += v[u];
        }
        for (; sb <= bsp; sb++) acc += h[(int64_t)sb * hct];
        return acc;
      };
      const int64_t cell = gini_cell(bf, 0, c, NB, A.Fmax, hct);
      // (a derived slot: parent - smaller child, read where this block did not write)
      l = ps ? bins_sum(ps + cell) - bins_sum(hs + cell) : bins_sum(hs + cell);
    }
    so[c] = s_tot[c];
    so[A.plane + c] = l;
    so[2 * A.plane + c] = s_tot[c] - l;
  }
  block_sync_mem();  // tid 0 reads the other threads' global stats words
  if (tid == 0 && bf >= 0) {  // the children's Gini.calculate, as the host's Calc would
    double imp2[2];
    for (int side = 0; side < 2; side++) {
      const int64_t* st = so + (1 + side) * A.plane;
      double total = 0.0;
      for (int c = 0; c < NS; c++) total += (double)st[c];
      double im = 0.0;
      if (total != 0) {
        im = 1.0;
        for (int c = 0; c < NS; c++) {
          const double fq = (double)st[c] / total;
          im -= fq * fq;
        }
      }
      imp2[side] = im;
    }
    A.out[slot].imp_l = imp2[0];
    A.out[slot].imp_r = imp2[1];
    A.out[slot].pad = 2;
  }
}

void launch_split(hipStream_t st, const SplitArgs& a, int M, bool gini) {
  const size_t lds = 256 * (8 + 4 + 4 + 4) + 8 * (size_t)a.NS + (gini ? (size_t)a.NS * 256 * 4 : 0);
  set_max_lds((const void*)k_split<true>, 160 * 1024);
  set_max_lds((const void*)k_split<false>, 160 * 1024);
  if (gini) {
    // feature group: about one candidate per thread, and <= 40 KB of LDS in all so that
    // four blocks share a CU (the kernel waits on its staging loads; C5, 64 classes:
    // G = 4 -> 17.6 ms of splits per fit, G = 7 at two blocks per CU -> 21.5 ms)
    const size_t per_f = (size_t)split_fstride(a.NB, a.NS) * 4;
    const size_t fixed = (size_t)a.NS * 8 + 256 * (8 + 4 + 4) + 64;
    const size_t budget = 40 * 1024 > fixed ? 40 * 1024 - fixed : 0;
    int G = (int)std::max<size_t>(1, std::min<size_t>(budget / per_f, (size_t)(256 / std::max(1, a.NB - 1))));
    if (const char* e = getenv("SBAG_SPLIT_G")) G = atoi(e);
    G = std::max(1, std::min(G, a.Fmax));
    const size_t lds_g = fixed + (size_t)G * per_f;
    set_max_lds((const void*)k_split_gini, 160 * 1024);
    if (lds_g <= 160 * 1024 && !getenv("SBAG_SPLIT_GINI_V1")) {
      hipLaunchKernelGGL(k_split_gini, dim3(M), dim3(256), lds_g, st, a, G);
      return;
    }
    hipLaunchKernelGGL(k_split<true>, dim3(M), dim3(256), lds, st, a);
  } else {
    hipLaunchKernelGGL(k_split<false>, dim3(M), dim3(256), lds, st, a);
  }
}

// sibling = parent - smaller child  (triples: dst slot, parent slot, small slot)
template <typename W>
__global__ __launch_bounds__(256) void k_subtract(W* __restrict__ dst_hist,
                                                  const W* __restrict__ par_hist,
                                                  const int32_t* __restrict__ triples,
                                                  int64_t words) {
  const int t = blockIdx.y;
  const int64_t d = triples[3 * t], p = triples[3 * t + 1], s = triples[3 * t + 2];
  for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < words;
       w += (int64_t)gridDim.x * 256)
    dst_hist[d * words + w] = par_hist[p * words + w] - dst_hist[s * words + w];
}

// zero the listed histogram slots (u32 words): the slots the next level's histogram kernel
// accumulates; the subtraction writes every word of the others
__global__ __launch_bounds__(256) void k_zero_slots(uint32_t* __restrict__ hist,
                                                    const int32_t* __restrict__ slots,
                                                    int64_t words) {
  uint4* h = (uint4*)(hist + (int64_t)slots[blockIdx.y] * words);
  for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < words / 4; w += (int64_t)gridDim.x * 256)
    h[w] = make_uint4(0, 0, 0, 0);
  if (blockIdx.x == 0 && threadIdx.x < (words & 3))
    hist[(int64_t)slots[blockIdx.y] * words + (words & ~3ll) + threadIdx.x] = 0u;
}

void launch_zero_slots(hipStream_t st, void* hist, const int32_t* d_slots, int nslots,
                       int64_t u32_words_per_slot) {
  if (nslots <= 0) return;
  const unsigned gx = (unsigned)std::min<int64_t>((u32_words_per_slot / 4 + 255) / 256, 64);
  for (int k0 = 0; k0 < nslots; k0 += 65535)  // (grid.y is at most 65535)
    hipLaunchKernelGGL(k_zero_slots, dim3(std::max(gx, 1u), (unsigned)std::min(65535, nslots - k0)), dim3(256), 0,
                       st, (uint32_t*)hist, d_slots + k0, u32_words_per_slot);
}

void launch_subtract(hipStream_t st, void* dst_hist, const void* parent_hist, const int32_t* d_triples,
                     int ntriples, int64_t words_per_slot, bool u32words) {
  if (ntriples <= 0) return;
  const unsigned gx = (unsigned)std::min<int64_t>((words_per_slot + 255) / 256, 64);
  dim3 grid(gx, (unsigned)ntriples);
  if (u32words)
    hipLaunchKernelGGL(k_subtract<uint32_t>, grid, dim3(256), 0, st, (uint32_t*)dst_hist,
                       (const uint32_t*)parent_hist, d_triples, words_per_slot);
  else
    hipLaunchKernelGGL(k_subtract<uint64_t>, grid, dim3(256), 0, st, (uint64_t*)dst_hist,
                       (const uint64_t*)parent_hist, d_triples, words_per_slot);
}


// Per-replica bins by counting code cuts: bin(code) = #{j : cut_j <= code}, cut_j = #{dictionary
// values <= t_j} of the (replica, feature)'s thresholds t_j -- TreePoint.findBin's binary search
// over the thresholds (#{t < value}).  cut: [R][Fmax][ncp] u32 ascending, padded with 0xffffffff
// (never <= a code); ng: [R][Fmax] groups of 32 cuts to test.
//
// k_bin_cuts (round 5): a workgroup takes rb replicas and a chunk of row blocks.  The rb
// replicas' cuts go to LDS once, as keys cut - 1 (u16 for u8/u16 codes: a cut is at most the
// dictionary size, and a key 0xffff -- also the padding -- is never below a code; u32 for wide
// codes), and the bin of a code is a branch-free binary search over the (replica, feature)'s
// ncp keys: log2(ncp) steps of one LDS read (at most 16 distinct words of 32 consecutive banks
// per wave: no conflicts), a compare and a select.  Per row block of kRows rows the codes are
// staged in LDS (pitch S*sizeof(CT) + 4 bytes: a column read by 64 consecutive rows hits 64
// banks); for each replica every wave bins groups of 4 features for all the rows (kRows/64 per
// lane), packs a row's 4 bins into a word of an LDS tile [kRows][S_out + 4], and the tile goes
// out row-major (the histograms' rows) and as k_partition's column copy (4 rows per word).
// The LUT form it replaces gathered one byte per (row, feature, replica) from multi-MB tables
// in L2 (955 ms of a C3-sized continuous fit, profiles/r04bf/); a count of the cuts by VALU
// compares took 32 compares per bin (380 ms, profiles/r05logs/r05e/).
template <typename CT, typename KT, int kRows>
__global__ __launch_bounds__(256) void k_bin_cuts(const CT* __restrict__ codes, int64_t N, int32_t S_codes,
                                                  const int32_t* __restrict__ sub,
                                                  const int32_t* __restrict__ Fr, int32_t Fmax,
                                                  const uint32_t* __restrict__ cut, int32_t ncp, int32_t lg,
                                                  const uint8_t* __restrict__ z0,
                                                  uint8_t* __restrict__ out, int32_t S_out, int64_t out_rstride,
                                                  uint8_t* __restrict__ cols, int32_t ncol, int64_t npad,
                                                  int64_t cols_rstride, int R, int rb, int64_t rows_per_chunk) {
  extern __shared__ __align__(16) uint8_t smem[];
  constexpr int kRpl = kRows / 64;  // rows per lane
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r0 = blockIdx.y * rb, nrep = min(rb, R - r0);
  const int pc = S_codes * (int)sizeof(CT) + 4;  // code row pitch in LDS (bytes)
  // bin row pitch: an odd number of words (a row per lane writes 64 distinct banks)
  const int pb = ((S_out / 4) & 1) ? S_out : S_out + 4;
  KT* sk = (KT*)smem;                            // [rb][Fmax][ncp] keys
  const size_t kbytes = ((size_t)rb * Fmax * ncp * sizeof(KT) + 15) & ~(size_t)15;
  uint8_t* sz = smem + kbytes;                   // [rb][Fmax] leading zero cuts (with z0)
  const size_t zbytes = z0 ? ((size_t)rb * Fmax + 15) & ~(size_t)15 : 0;
  uint8_t* sc = sz + zbytes;
  uint8_t* sb = sc + (size_t)kRows * pc;
  for (int64_t k = tid; k < (int64_t)nrep * Fmax * ncp; k += 256) {
    const uint32_t c = cut[(int64_t)r0 * Fmax * ncp + k];
    sk[k] = c == 0xffffffffu ? (KT)~(KT)0 : (KT)(c - 1u);
  }
  if (z0)
    for (int k = tid; k < nrep * Fmax; k += 256) sz[k] = z0[(int64_t)r0 * Fmax + k];
  const int64_t c0 = (int64_t)blockIdx.x * rows_per_chunk, c1 = min(N, c0 + rows_per_chunk);
  const int ngrp4 = S_out / 4;
  // the code rows of a block as 16-byte pieces, kPv per thread, loaded one block ahead into
  // registers (a load-then-store loop waited out the memory latency for every piece)
  const int rq = S_codes * (int)sizeof(CT) / 16;  // 16-byte pieces per code row
  constexpr int kPv = kRows / 16;                  // pieces per thread (rows of <= 256 bytes)
  uint4 pv[kPv];
  // (unconditional loads, clamped to the last row: rows past a block's end are binned but never
  // stored; a select on a loaded value, or a branch around a load, makes the compiler wait)
  auto load_block = [&](int64_t nb) {
    nb = min(nb, N - 1);
    const uint4* src = (const uint4*)(codes + nb * S_codes);
    const int64_t lim = (min(N, nb + kRows) - nb) * rq;  // pieces of the block's real rows
#pragma unroll
    for (int v = 0; v < kPv; v++) pv[v] = src[min((int64_t)(tid + 256 * v), lim - 1)];
  };
  // (each piece's LDS place, computed once: the division by rq is not per block)
  int soff[kPv];
#pragma unroll
  for (int v = 0; v < kPv; v++) {
    const int k = tid + 256 * v;
    const int row = k / rq, w = k - row * rq;
    soff[v] = k < kRows * rq ? row * pc + 16 * w : -1;
  }
  if (c0 < c1) load_block(c0);
  for (int64_t n0 = c0; n0 < c1; n0 += kRows) {
    const int nr = (int)min<int64_t>(kRows, c1 - n0);
    block_sync();  // (the previous block's tile reads; the keys at the first block)
#pragma unroll
    for (int v = 0; v < kPv; v++) {
      if (soff[v] >= 0) {
        uint32_t* d = (uint32_t*)(sc + soff[v]);
        d[0] = pv[v].x;
        d[1] = pv[v].y;
        d[2] = pv[v].z;
        d[3] = pv[v].w;
      }
    }
    load_block(n0 + kRows);  // the next block's codes in flight
    block_sync();
    for (int ri = 0; ri < nrep; ri++) {
      const int r = r0 + ri;
      // the replica's feature count and this wave's features' code offsets, by vector loads
      // once per replica (lane 4 j + k: feature 4 (wave + 4 j) + k) -- scalar loads inside
      // the group loop would wait on lgkmcnt, which also counts the searches' LDS reads
      const int fr = __builtin_amdgcn_readfirstlane(Fr[r]);
      int gv;
      {
        const int fl = min(4 * (wave + 4 * (lane >> 2)) + (lane & 3), fr - 1);
        gv = sub[(int64_t)r * Fmax + fl] * (int)sizeof(CT);
      }
      for (int q = wave, j = 0; q < ngrp4; q += 4, j++) {
        if (4 * q >= fr) {  // past the replica's features: zero bins
#pragma unroll
          for (int i = 0; i < kRpl; i++) *(uint32_t*)(sb + (lane + 64 * i) * pb + 4 * q) = 0u;
          continue;
        }
        uint32_t wv[kRpl];
#pragma unroll
        for (int i = 0; i < kRpl; i++) wv[i] = 0u;
        // the group's 4 features x kRpl rows: 4 kRpl independent searches, their LDS reads
        // interleaved (one search alone waits out each read's latency)
        const KT* ks[4];
        uint32_t cv[4][kRpl], idx[4][kRpl];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int fl = min(4 * q + k, fr - 1);  // (features past F_r search a real one; masked below)
          const int gb = __builtin_amdgcn_readlane(gv, 4 * j + k);
          ks[k] = sk + ((size_t)ri * Fmax + fl) * ncp;
#pragma unroll
          for (int i = 0; i < kRpl; i++) {
            cv[k][i] = (uint32_t) * (const CT*)(sc + (lane + 64 * i) * pc + gb);
            idx[k][i] = 0u;
          }
        }
        // idx = #{keys < code} (keys ascending): steps of ncp / 2, ..., 1 (unrolled for the
        // common 32 keys)
        auto step = [&](uint32_t h) {
#pragma unroll
          for (int k = 0; k < 4; k++)
#pragma unroll
            for (int i = 0; i < kRpl; i++) idx[k][i] += (uint32_t)ks[k][idx[k][i] + h - 1u] < cv[k][i] ? h : 0u;
        };
        // (measured on a C3-sized continuous fit, 64 keys: a two-level search with packed u16
        // counts took the same 83.8 ms per launch, profiles/r05logs/r05z/; one search per pair
        // of replicas over their union of keys, half the searches, took 124 vs 78 ms -- its
        // tables halve the workgroups per CU, profiles/r05logs/r05z5/)
        if (lg == 5) {
          step(16u);
          step(8u);
          step(4u);
          step(2u);
          step(1u);
        } else if (lg == 6) {  // (a replica's 32nd threshold: common on continuous features)
          step(32u);
          step(16u);
          step(8u);
          step(4u);
          step(2u);
          step(1u);
        } else {
          for (int st = lg - 1; st >= 0; st--) step(1u << st);
        }
        // the steps count the keys of slots 0 .. ncp - 2; slot ncp - 1 (a 32nd cut in 32 slots,
        // else padding) by one more compare off the dependent chain, then the leading zero cuts
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t kl = (uint32_t)ks[k][ncp - 1];
          const uint32_t zk = z0 ? (uint32_t)sz[ri * Fmax + min(4 * q + k, fr - 1)] : 0u;
#pragma unroll
          for (int i = 0; i < kRpl; i++) idx[k][i] += (kl < cv[k][i] ? 1u : 0u) + zk;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (4 * q + k < fr)
#pragma unroll
            for (int i = 0; i < kRpl; i++) wv[i] |= idx[k][i] << (8 * k);
#pragma unroll
        for (int i = 0; i < kRpl; i++) *(uint32_t*)(sb + (lane + 64 * i) * pb + 4 * q) = wv[i];
      }
      block_sync();
      {
        uint8_t* o = out + (int64_t)r * out_rstride + n0 * S_out;
        if (pb == S_out) {  // the tile is the block's rows as they go out
          const int nb = nr * S_out;
          if ((((uintptr_t)o) & 15) == 0) {
            for (int k = tid; k < nb / 16; k += 256) ((uint4*)o)[k] = ((const uint4*)sb)[k];
            for (int k = nb / 16 * 4 + tid; k < nb / 4; k += 256) ((uint32_t*)o)[k] = ((const uint32_t*)sb)[k];
          } else {
            for (int k = tid; k < nb / 4; k += 256) ((uint32_t*)o)[k] = ((const uint32_t*)sb)[k];
          }
        } else {
          const int wpr = S_out / 4;  // output words per row
          for (int row = tid >> 5; row < nr; row += 8)
            for (int w = tid & 31; w < wpr; w += 32)
              ((uint32_t*)o)[row * wpr + w] = *(const uint32_t*)(sb + row * pb + 4 * w);
        }
      }
      if (cols) {  // per feature the block's rows are consecutive bytes (rows past N: 0)
        // a thread takes a 4 x 4 byte block (rows 4 rq.., features 4 fq..): four word reads of
        // the tile, a byte transpose by v_perm, one word per feature column
        constexpr int kRq = kRows / 4;
        uint8_t* cr = cols + (int64_t)r * cols_rstride + n0;
        for (int t = tid; t < (ncol + 3) / 4 * kRq; t += 256) {
          const int fq = t / kRq, rq4 = t % kRq;
          uint32_t d[4];
#pragma unroll
          for (int kk = 0; kk < 4; kk++) {
            const int row = 4 * rq4 + kk;
            const uint32_t x = *(const uint32_t*)(sb + row * pb + 4 * fq);
            d[kk] = row < nr ? x : 0u;
          }
          const uint32_t lo01 = __builtin_amdgcn_perm(d[1], d[0], 0x05010400u);
          const uint32_t hi01 = __builtin_amdgcn_perm(d[1], d[0], 0x07030602u);
          const uint32_t lo23 = __builtin_amdgcn_perm(d[3], d[2], 0x05010400u);
          const uint32_t hi23 = __builtin_amdgcn_perm(d[3], d[2], 0x07030602u);
          const uint32_t f4[4] = {__builtin_amdgcn_perm(lo23, lo01, 0x05040100u),
                                  __builtin_amdgcn_perm(lo23, lo01, 0x07060302u),
                                  __builtin_amdgcn_perm(hi23, hi01, 0x05040100u),
                                  __builtin_amdgcn_perm(hi23, hi01, 0x07060302u)};
#pragma unroll
          for (int i = 0; i < 4; i++)
            if (4 * fq + i < ncol) *(uint32_t*)(cr + (int64_t)(4 * fq + i) * npad + 4 * rq4) = f4[i];
        }
      }
      if (ri + 1 < nrep) block_sync();  // the tile is rewritten by the next replica
    }
  }
}

// Fallback for rows too wide for the staged tiles: a thread per row, a binary search over the
// cuts per feature (no column copy).
template <typename CT>
__global__ __launch_bounds__(256) void k_bin_cuts_rows(const CT* __restrict__ codes, int64_t N, int32_t S_codes,
                                                       const int32_t* __restrict__ sub,
                                                       const int32_t* __restrict__ Fr, int32_t Fmax,
                                                       const uint32_t* __restrict__ cut, int32_t ncp,
                                                       const uint8_t* __restrict__ z0,
                                                       uint8_t* __restrict__ out, int32_t S_out,
                                                       int64_t out_rstride) {
  const int r = blockIdx.y;
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= N) return;
  const int fr = Fr[r];
  uint8_t* o = out + (int64_t)r * out_rstride + row * S_out;
  const CT* cr = codes + row * S_codes;
  for (int fl = 0; fl < S_out; fl++) {
    uint32_t b = 0;
    if (fl < fr) {
      const uint32_t code = (uint32_t)cr[sub[(int64_t)r * Fmax + fl]];
      const uint32_t* cu = cut + ((int64_t)r * Fmax + fl) * ncp;
      int lo = 0, hi = ncp;  // first j with cu[j] > code
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cu[mid] <= code)
          lo = mid + 1;
        else
          hi = mid;
      }
      b = (uint32_t)lo + (z0 ? (uint32_t)z0[(int64_t)r * Fmax + fl] : 0u);
    }
    o[fl] = (uint8_t)b;
  }
}

template <typename CT, typename KT, int kRows>
static bool launch_bin_cuts_r(hipStream_t st, const CT* codes, int64_t N, int32_t S_codes, const int32_t* d_sub,
                              const int32_t* d_Fr, int32_t Fmax, int R, const uint32_t* d_cut, int32_t ncp,
                              const uint8_t* d_z0, uint8_t* out, int32_t S_out, int64_t out_rstride, uint8_t* cols,
                              int32_t ncol, int64_t npad, int64_t cols_rstride) {
  const int pb = ((S_out / 4) & 1) ? S_out : S_out + 4;  // (the kernel's bin row pitch)
  const size_t tiles = (size_t)kRows * (S_codes * sizeof(CT) + 4) + (size_t)kRows * pb;
  const size_t per_rep = (size_t)Fmax * ncp * sizeof(KT);
  // replicas per workgroup (they share the staged codes) within the LDS target.  One by default:
  // the occupancy it buys outweighs re-reading the codes per replica (C3-sized continuous fit,
  // 64 keys: 57.7 ms per launch at one, 65.9 at two; profiles/r05logs/r05z6/).  SBAG_BIN_RB /
  // SBAG_BIN_LDS_KB override
  static const int rb_env = getenv("SBAG_BIN_RB") ? atoi(getenv("SBAG_BIN_RB")) : 0;
  static const int lds_kb = getenv("SBAG_BIN_LDS_KB") ? atoi(getenv("SBAG_BIN_LDS_KB")) : 52;
  int rb = rb_env > 0 ? rb_env : 1;
  while (rb > 1 && tiles + rb * per_rep > (size_t)lds_kb * 1024) rb--;
  rb = std::max(1, std::min(rb, R));
  int lg = 0;
  while ((1 << lg) < ncp) lg++;
  const size_t lds = tiles + ((rb * per_rep + 15) & ~(size_t)15) + (d_z0 ? ((size_t)rb * Fmax + 15) & ~(size_t)15 : 0);
  // (the staged code rows: 16-byte pieces, at most kRows / 16 per thread per block)
  if (lds > 150 * 1024 || (1 << lg) != ncp || S_out % 4 != 0 || (S_codes * sizeof(CT)) % 16 != 0 ||
      (size_t)kRows * S_codes * sizeof(CT) > (size_t)kRows / 16 * 16 * 256 || npad % kRows != 0 ||
      getenv("SBAG_BIN_ROWWISE"))
    return false;
  // chunks of row blocks: about 65536 workgroups over the replica groups (SBAG_BIN_WGS; C3-sized
  // continuous fit 1024 / 4096 / 16384 / 65536 / 262144: 617 / 632 / 548 / 548 / 523 ms on one box,
  // profiles/r05logs/r05t/)
  static const int64_t wgs = getenv("SBAG_BIN_WGS") ? atoll(getenv("SBAG_BIN_WGS")) : 65536;
  const int ngrp = (R + rb - 1) / rb;
  const int64_t nblk = (N + kRows - 1) / kRows;
  const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(nblk, (wgs + ngrp - 1) / ngrp));
  const int64_t rpc = (nblk + nch - 1) / nch * kRows;
  const dim3 g((unsigned)((N + rpc - 1) / rpc), (unsigned)ngrp);
  set_max_lds((const void*)k_bin_cuts<CT, KT, kRows>, (int)lds);
  hipLaunchKernelGGL((k_bin_cuts<CT, KT, kRows>), g, dim3(256), lds, st, codes, N, S_codes, d_sub, d_Fr, Fmax,
                     d_cut, ncp, lg, d_z0, out, S_out, out_rstride, cols, ncol, npad, cols_rstride, R, rb, rpc);
  return true;
}

template <typename CT, typename KT>
static bool launch_bin_cuts_t(hipStream_t st, const CT* codes, int64_t N, int32_t S_codes, const int32_t* d_sub,
                              const int32_t* d_Fr, int32_t Fmax, int R, const uint32_t* d_cut, int32_t ncp,
                              const uint8_t* d_z0, uint8_t* out, int32_t S_out, int64_t out_rstride, uint8_t* cols,
                              int32_t ncol, int64_t npad, int64_t cols_rstride) {
  // 64-row blocks (one row per lane: ~50 KB of LDS with four replicas, three workgroups per CU)
  // unless SBAG_BIN_ROWS=128 (C3-sized continuous fit 563 vs 604 ms, profiles/r05logs/r05k/)
  static const int rows = getenv("SBAG_BIN_ROWS") ? atoi(getenv("SBAG_BIN_ROWS")) : 64;
  if (rows == 128)
    return launch_bin_cuts_r<CT, KT, 128>(st, codes, N, S_codes, d_sub, d_Fr, Fmax, R, d_cut, ncp, d_z0, out, S_out,
                                          out_rstride, cols, ncol, npad, cols_rstride);
  return launch_bin_cuts_r<CT, KT, 64>(st, codes, N, S_codes, d_sub, d_Fr, Fmax, R, d_cut, ncp, d_z0, out, S_out,
                                       out_rstride, cols, ncol, npad, cols_rstride);
}

template <typename CT>
static bool launch_bin_cuts_any(hipStream_t st, const CT* codes, int64_t N, int32_t S_codes, const int32_t* d_sub,
                                const int32_t* d_Fr, int32_t Fmax, int R, const uint32_t* d_cut, int32_t ncp,
                                const uint8_t* d_z0, uint8_t* out, int32_t S_out, int64_t out_rstride,
                                uint8_t* cols, int32_t ncol, int64_t npad, int64_t cols_rstride) {
  const bool ok = sizeof(CT) <= 2
                      ? launch_bin_cuts_t<CT, uint16_t>(st, codes, N, S_codes, d_sub, d_Fr, Fmax, R, d_cut, ncp, d_z0,
                                                        out, S_out, out_rstride, cols, ncol, npad, cols_rstride)
                      : launch_bin_cuts_t<CT, uint32_t>(st, codes, N, S_codes, d_sub, d_Fr, Fmax, R, d_cut, ncp, d_z0,
                                                        out, S_out, out_rstride, cols, ncol, npad, cols_rstride);
  if (ok) return cols != nullptr;
  // rows too wide for the staged tiles: a thread per row (no column copy)
  const dim3 grid((unsigned)((N + 255) / 256), (unsigned)R);
  hipLaunchKernelGGL(k_bin_cuts_rows<CT>, grid, dim3(256), 0, st, codes, N, S_codes, d_sub, d_Fr, Fmax, d_cut,
                     ncp, d_z0, out, S_out, out_rstride);
  return false;
}

bool launch_bin_cuts(hipStream_t st, const void* codes, int code_bytes, int64_t N, int32_t S_codes,
                     const int32_t* d_sub, const int32_t* d_Fr, int32_t Fmax, int R, const uint32_t* d_cut,
                     int32_t ncp, const uint8_t* d_z0, uint8_t* out, int32_t S_out, int64_t out_rstride,
                     uint8_t* cols, int32_t ncol, int64_t npad, int64_t cols_rstride) {
  if (code_bytes == 1)
    return launch_bin_cuts_any(st, (const uint8_t*)codes, N, S_codes, d_sub, d_Fr, Fmax, R, d_cut, ncp, d_z0,
                               out, S_out, out_rstride, cols, ncol, npad, cols_rstride);
  if (code_bytes == 2)
    return launch_bin_cuts_any(st, (const uint16_t*)codes, N, S_codes, d_sub, d_Fr, Fmax, R, d_cut, ncp, d_z0,
                               out, S_out, out_rstride, cols, ncol, npad, cols_rstride);
  return launch_bin_cuts_any(st, (const uint32_t*)codes, N, S_codes, d_sub, d_Fr, Fmax, R, d_cut, ncp, d_z0,
                             out, S_out, out_rstride, cols, ncol, npad, cols_rstride);
}

// k_bin_ranked: k_bin_cuts over a replica's in-bag rows only, stored by in-bag rank (the
// entry's index in the replica's row-ordered list): out[r][rank][S_out], cols[r][fl][rank].
// Out-of-bag rows' bins were never read; the in-bag list of a Poisson(1) bag is 63 % of the rows,
// so the searches and the stores shrink by as much.  The entries then carry ranks instead of
// rows (k_rank_entries).  A workgroup takes one replica and a chunk of ranks; each block of
// 64 ranks loads its rows' ids two blocks ahead and their code rows one block ahead (gathers of
// whole code rows, mostly consecutive), then searches and emits as k_bin_cuts does.
template <typename CT, typename KT, int kPv>
__global__ __launch_bounds__(256) void k_bin_ranked(const CT* __restrict__ codes, int32_t S_codes,
                                                    const uint64_t* __restrict__ ent, int64_t cap,
                                                    const unsigned long long* __restrict__ inbag,
                                                    const int32_t* __restrict__ sub, const int32_t* __restrict__ Fr,
                                                    int32_t Fmax, const uint32_t* __restrict__ cut, int32_t ncp,
                                                    int32_t lg, const uint8_t* __restrict__ z0,
                                                    uint8_t* __restrict__ out, int32_t S_out, int64_t out_rstride,
                                                    uint8_t* __restrict__ cols, int32_t ncol, int64_t npad,
                                                    int64_t cols_rstride, int64_t ranks_per_chunk) {
  extern __shared__ __align__(16) uint8_t smem[];
  constexpr int kRows = 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = blockIdx.y;
  const int64_t nin = (int64_t)inbag[r];
  const int64_t c0 = (int64_t)blockIdx.x * ranks_per_chunk, c1 = min(nin, c0 + ranks_per_chunk);
  if (c0 >= c1) return;  // (uniform: before any barrier)
  const int pc = S_codes * (int)sizeof(CT) + 4;
  const int pb = ((S_out / 4) & 1) ? S_out : S_out + 4;
  KT* sk = (KT*)smem;
  const size_t kbytes = ((size_t)Fmax * ncp * sizeof(KT) + 15) & ~(size_t)15;
  uint8_t* sz = smem + kbytes;
  const size_t zbytes = z0 ? ((size_t)Fmax + 15) & ~(size_t)15 : 0;
  uint8_t* sc = sz + zbytes;
  uint8_t* sb = sc + (size_t)kRows * pc;
  for (int64_t k = tid; k < (int64_t)Fmax * ncp; k += 256) {
    const uint32_t c = cut[(int64_t)r * Fmax * ncp + k];
    sk[k] = c == 0xffffffffu ? (KT)~(KT)0 : (KT)(c - 1u);
  }
  if (z0)
    for (int k = tid; k < Fmax; k += 256) sz[k] = z0[(int64_t)r * Fmax + k];
  const uint64_t* er = ent + (int64_t)r * cap;
  const int ngrp4 = S_out / 4;
  const int rq = S_codes * (int)sizeof(CT) / 16;  // (kPv 16-byte pieces per thread: rows <= 64 kPv bytes)
  int soff[kPv], srow[kPv], sw[kPv];
#pragma unroll
  for (int v = 0; v < kPv; v++) {
    const int k = tid + 256 * v;
    const int kk = min(k, kRows * rq - 1);
    srow[v] = kk / rq;
    sw[v] = kk - srow[v] * rq;
    soff[v] = k < kRows * rq ? srow[v] * pc + 16 * sw[v] : -1;
  }
  // the row of rank nb + lane (clamped to the chunk: ranks past it are binned, never stored)
  auto load_rows = [&](int64_t nb) { return (uint32_t)er[min(nb + lane, c1 - 1)]; };
  uint4 pv[kPv];
  auto load_block = [&](uint32_t rowv) {
#pragma unroll
    for (int v = 0; v < kPv; v++) {
      const uint32_t row = (uint32_t)__shfl((int)rowv, srow[v]);
      pv[v] = ((const uint4*)(codes + (int64_t)row * S_codes))[sw[v]];
    }
  };
  const int fr = __builtin_amdgcn_readfirstlane(Fr[r]);
  int gv;
  {
    const int fl = min(4 * (wave + 4 * (lane >> 2)) + (lane & 3), fr - 1);
    gv = sub[(int64_t)r * Fmax + fl] * (int)sizeof(CT);
  }
  load_block(load_rows(c0));
  uint32_t rows_next = load_rows(c0 + kRows);
  for (int64_t n0 = c0; n0 < c1; n0 += kRows) {
    const int nr = (int)min<int64_t>(kRows, c1 - n0);
    block_sync();  // (the previous block's tile reads; the keys at the first block)
#pragma unroll
    for (int v = 0; v < kPv; v++) {
      if (soff[v] >= 0) {
        uint32_t* d = (uint32_t*)(sc + soff[v]);
        d[0] = pv[v].x;
        d[1] = pv[v].y;
        d[2] = pv[v].z;
        d[3] = pv[v].w;
      }
    }
    load_block(rows_next);  // the next block's code rows in flight
    rows_next = load_rows(n0 + 2 * kRows);
    block_sync();
    for (int q = wave, j = 0; q < ngrp4; q += 4, j++) {
      if (4 * q >= fr) {
        *(uint32_t*)(sb + lane * pb + 4 * q) = 0u;
        continue;
      }
      const KT* ks[4];
      uint32_t cv[4], idx[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int fl = min(4 * q + k, fr - 1);
        const int gb = __builtin_amdgcn_readlane(gv, 4 * j + k);
        ks[k] = sk + (size_t)fl * ncp;
        cv[k] = (uint32_t) * (const CT*)(sc + lane * pc + gb);
        idx[k] = 0u;
      }
      auto step = [&](uint32_t h) {
#pragma unroll
        for (int k = 0; k < 4; k++) idx[k] += (uint32_t)ks[k][idx[k] + h - 1u] < cv[k] ? h : 0u;
      };
      if (lg == 5) {
        step(16u);
        step(8u);
        step(4u);
        step(2u);
        step(1u);
      } else if (lg == 6) {
        step(32u);
        step(16u);
        step(8u);
        step(4u);
        step(2u);
        step(1u);
      } else {
        for (int st = lg - 1; st >= 0; st--) step(1u << st);
      }
      uint32_t wv = 0u;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t kl = (uint32_t)ks[k][ncp - 1];
        const uint32_t zk = z0 ? (uint32_t)sz[min(4 * q + k, fr - 1)] : 0u;
        const uint32_t b = idx[k] + (kl < cv[k] ? 1u : 0u) + zk;
        if (4 * q + k < fr) wv |= b << (8 * k);
      }
      *(uint32_t*)(sb + lane * pb + 4 * q) = lane < nr ? wv : 0u;
    }
    block_sync();
    {
      // (the replica's last block also stores its zeroed rows past the last rank: the row-lane
      // histogram's aligned loads may read a few bytes past a row, which must be valid bins;
      // the caller leaves room for them)
      const int nst = n0 + kRows >= nin ? kRows : nr;
      uint8_t* o = out + (int64_t)r * out_rstride + n0 * S_out;
      if (pb == S_out) {
        const int nb = nst * S_out;
        if ((((uintptr_t)o) & 15) == 0) {
          for (int k = tid; k < nb / 16; k += 256) ((uint4*)o)[k] = ((const uint4*)sb)[k];
          for (int k = nb / 16 * 4 + tid; k < nb / 4; k += 256) ((uint32_t*)o)[k] = ((const uint32_t*)sb)[k];
        } else {
          for (int k = tid; k < nb / 4; k += 256) ((uint32_t*)o)[k] = ((const uint32_t*)sb)[k];
        }
      } else {
        const int wpr = S_out / 4;
        for (int row = tid >> 5; row < nst; row += 8)
          for (int w = tid & 31; w < wpr; w += 32)
            ((uint32_t*)o)[row * wpr + w] = *(const uint32_t*)(sb + row * pb + 4 * w);
      }
      // a full last block (nin a multiple of 64) leaves the row at rank nin to zero here
      // (it stayed stale workspace memory)
      if (n0 + nr == nin && nr == kRows)
        for (int w = tid; w < S_out / 4; w += 256) ((uint32_t*)(o + (int64_t)kRows * S_out))[w] = 0u;
    }
    if (cols) {
      constexpr int kRq = kRows / 4;
      uint8_t* cr = cols + (int64_t)r * cols_rstride + n0;
      for (int t = tid; t < (ncol + 3) / 4 * kRq; t += 256) {
        const int fq = t / kRq, rq4 = t % kRq;
        uint32_t d[4];
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
          const int row = 4 * rq4 + kk;
          const uint32_t x = *(const uint32_t*)(sb + row * pb + 4 * fq);
          d[kk] = row < nr ? x : 0u;
        }
        const uint32_t lo01 = __builtin_amdgcn_perm(d[1], d[0], 0x05010400u);
        const uint32_t hi01 = __builtin_amdgcn_perm(d[1], d[0], 0x07030602u);
        const uint32_t lo23 = __builtin_amdgcn_perm(d[3], d[2], 0x05010400u);
        const uint32_t hi23 = __builtin_amdgcn_perm(d[3], d[2], 0x07030602u);
        const uint32_t f4[4] = {__builtin_amdgcn_perm(lo23, lo01, 0x05040100u),
                                __builtin_amdgcn_perm(lo23, lo01, 0x07060302u),
                                __builtin_amdgcn_perm(hi23, hi01, 0x05040100u),
                                __builtin_amdgcn_perm(hi23, hi01, 0x07060302u)};
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (4 * fq + i < ncol) *(uint32_t*)(cr + (int64_t)(4 * fq + i) * npad + 4 * rq4) = f4[i];
      }
    }
  }
}

static size_t bin_ranked_lds(int code_bytes, int32_t S_codes, int32_t S_out, int32_t Fmax, int32_t ncp) {
  const int kb = code_bytes <= 2 ? 2 : 4;
  const int pb = ((S_out / 4) & 1) ? S_out : S_out + 4;
  return (((size_t)Fmax * ncp * kb + 15) & ~(size_t)15) + (((size_t)Fmax + 15) & ~(size_t)15) +
         (size_t)64 * (S_codes * code_bytes + 4) + (size_t)64 * pb;
}

bool bin_ranked_fits(int code_bytes, int32_t S_codes, int32_t S_out, int32_t Fmax, int32_t ncp) {
  return bin_ranked_lds(code_bytes, S_codes, S_out, Fmax, ncp) <= 150 * 1024 && (ncp & (ncp - 1)) == 0 &&
         S_out % 4 == 0 && ((int64_t)S_codes * code_bytes) % 16 == 0 && (int64_t)S_codes * code_bytes <= 1024;
}

template <typename CT, typename KT>
static bool launch_bin_ranked_t(hipStream_t st, const CT* codes, int32_t S_codes, const uint64_t* ent, int64_t cap,
                                const unsigned long long* d_inbag, int64_t capb, const int32_t* d_sub,
                                const int32_t* d_Fr, int32_t Fmax, int R, const uint32_t* d_cut, int32_t ncp,
                                const uint8_t* d_z0, uint8_t* out, int32_t S_out, int64_t out_rstride, uint8_t* cols,
                                int32_t ncol, int64_t npad, int64_t cols_rstride) {
  constexpr int kRows = 64;
  if (!bin_ranked_fits((int)sizeof(CT), S_codes, S_out, Fmax, ncp) || npad % kRows != 0 || !cols) return false;
  const size_t lds = bin_ranked_lds((int)sizeof(CT), S_codes, S_out, Fmax, ncp);
  int lg = 0;
  while ((1 << lg) < ncp) lg++;
  static const int64_t wgs = getenv("SBAG_BIN_WGS") ? atoll(getenv("SBAG_BIN_WGS")) : 65536;
  const int64_t nblk = (capb + kRows - 1) / kRows;
  const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(nblk, (wgs + R - 1) / R));
  const int64_t rpc = (nblk + nch - 1) / nch * kRows;
  const dim3 g((unsigned)((capb + rpc - 1) / rpc), (unsigned)R);
  const int64_t rowb = (int64_t)S_codes * sizeof(CT);  // code row bytes: 16-byte pieces per thread
  auto go = [&](const void* fn) {
    set_max_lds(fn, (int)lds);
    void* args[] = {(void*)&codes, (void*)&S_codes, (void*)&ent,   (void*)&cap,         (void*)&d_inbag,
                    (void*)&d_sub, (void*)&d_Fr,    (void*)&Fmax,  (void*)&d_cut,       (void*)&ncp,
                    (void*)&lg,    (void*)&d_z0,    (void*)&out,   (void*)&S_out,       (void*)&out_rstride,
                    (void*)&cols,  (void*)&ncol,    (void*)&npad,  (void*)&cols_rstride, (void*)&rpc};
    (void)hipLaunchKernel(fn, g, dim3(256), args, lds, st);
  };
  if (rowb <= 256)
    go((const void*)k_bin_ranked<CT, KT, 4>);
  else if (rowb <= 512)
    go((const void*)k_bin_ranked<CT, KT, 8>);
  else
    go((const void*)k_bin_ranked<CT, KT, 16>);
  return true;
}

bool launch_bin_ranked(hipStream_t st, const void* codes, int code_bytes, int32_t S_codes, const uint64_t* ent,
                       int64_t cap, const unsigned long long* d_inbag, int64_t capb, const int32_t* d_sub,
                       const int32_t* d_Fr, int32_t Fmax, int R, const uint32_t* d_cut, int32_t ncp,
                       const uint8_t* d_z0, uint8_t* out, int32_t S_out, int64_t out_rstride, uint8_t* cols,
                       int32_t ncol, int64_t npad, int64_t cols_rstride) {
  if (code_bytes == 1)
    return launch_bin_ranked_t<uint8_t, uint16_t>(st, (const uint8_t*)codes, S_codes, ent, cap, d_inbag, capb, d_sub,
                                                  d_Fr, Fmax, R, d_cut, ncp, d_z0, out, S_out, out_rstride, cols,
                                                  ncol, npad, cols_rstride);
  if (code_bytes == 2)
    return launch_bin_ranked_t<uint16_t, uint16_t>(st, (const uint16_t*)codes, S_codes, ent, cap, d_inbag, capb,
                                                   d_sub, d_Fr, Fmax, R, d_cut, ncp, d_z0, out, S_out, out_rstride,
                                                   cols, ncol, npad, cols_rstride);
  return launch_bin_ranked_t<uint32_t, uint32_t>(st, (const uint32_t*)codes, S_codes, ent, cap, d_inbag, capb, d_sub,
                                                 d_Fr, Fmax, R, d_cut, ncp, d_z0, out, S_out, out_rstride, cols,
                                                 ncol, npad, cols_rstride);
}

// entries' row field -> their in-bag rank (after k_bin_ranked)
__global__ __launch_bounds__(256) void k_rank_entries(uint64_t* __restrict__ ent, int64_t cap,
                                                      const unsigned long long* __restrict__ inbag) {
  const int r = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)inbag[r]) return;
  uint64_t* e = ent + (int64_t)r * cap + i;
  *e = (*e & 0xffffffff00000000ull) | (uint64_t)(uint32_t)i;
}

void launch_rank_entries(hipStream_t st, uint64_t* ent, int64_t cap, const unsigned long long* d_inbag, int R,
                         int64_t capb) {
  if (capb <= 0 || R <= 0) return;
  hipLaunchKernelGGL(k_rank_entries, dim3((unsigned)((capb + 255) / 256), (unsigned)R), dim3(256), 0, st, ent, cap,
                     d_inbag);
}

// Value counts with global atomics (u16 codes / dictionaries too large for LDS)
template <typename CT>
__global__ __launch_bounds__(256) void k_vc_global(const CT* __restrict__ codes, int32_t S,
                                                   const uint64_t* __restrict__ ent, int64_t cap,
                                                   const unsigned long long* __restrict__ inbag,
                                                   const int32_t* __restrict__ sub,
                                                   const int32_t* __restrict__ Fr, int32_t Fmax,
                                                   const int64_t* __restrict__ off, uint32_t* vc) {
  const int r = blockIdx.y;
  const int64_t n = (int64_t)inbag[r];
  const int fr = Fr[r];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = ent[(int64_t)r * cap + i];
    const uint32_t row = (uint32_t)e;
    const uint32_t cnt = (uint32_t)(e >> 32) & 0xffu;
    for (int fl = 0; fl < fr; fl++) {
      const int g = sub[(int64_t)r * Fmax + fl];
      atomicAdd(&vc[off[(int64_t)r * Fmax + fl] + (int64_t)codes[(int64_t)row * S + g]], cnt);
    }
  }
}

void launch_vc_global(hipStream_t st, const void* codes, int code_bytes, int32_t S, const uint64_t* ent,
                      int64_t cap, const unsigned long long* d_inbag, const int32_t* d_sub,
                      const int32_t* d_Fr, int32_t Fmax, int R, const int64_t* d_off, uint32_t* vc) {
  dim3 grid(256, (unsigned)R);
  if (code_bytes == 1)
    hipLaunchKernelGGL(k_vc_global<uint8_t>, grid, dim3(256), 0, st, (const uint8_t*)codes, S, ent,
                       cap, d_inbag, d_sub, d_Fr, Fmax, d_off, vc);
  else
    hipLaunchKernelGGL(k_vc_global<uint16_t>, grid, dim3(256), 0, st, (const uint16_t*)codes, S,
                       ent, cap, d_inbag, d_sub, d_Fr, Fmax, d_off, vc);
}

// ======================================================================
// Synthetic workload
// ======================================================================
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ codes, int32_t S, int64_t N,
                                               int32_t F, uint64_t seed, int32_t C,
                                               int32_t* __restrict__ labk) {
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= N) return;
  uint8_t* o = codes + row * S;
  int x[8];
  for (int f = 0; f < 8; f++) x[f] = 0;
  for (int f0 = 0; f0 < S; f0 += 4) {
    uint32_t w = 0;
    for (int j = 0; j < 4; j++) {
      const int f = f0 + j;
      uint32_t v = 0;
      if (f < F) v = (uint32_t)(splitmix64(seed ^ (uint64_t)(row * (int64_t)F + f)) & 31u);
      if (f < 8) x[f] = (int)v;
      w |= v << (8 * j);
    }
    *(uint32_t*)(o + f0) = w;
  }
  const uint64_t h2 = splitmix64(~seed ^ (uint64_t)row);
  if (C == 0) {
    int k = 0;
    for (int f = 0; f < 8 && f < F; f++) k += (f + 1) * x[f];
    labk[row] = k + (int)(h2 & 63u) - 32;
  } else {
    labk[row] = (x[0] + 3 * x[1] + 7 * x[2] + (int)(h2 & 7u)) % C;
  }
}

void launch_synth(hipStream_t st, uint8_t* codes, int32_t S, int64_t N, int32_t F, uint64_t seed,
                  int32_t num_classes, int32_t* labk) {
  hipLaunchKernelGGL(k_synth, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, codes, S, N, F,
                     seed, num_classes, labk);
}

// ======================================================================
// Prediction: thread per row, trees in learner order (breeze sum order /
// breeze mode "first value to reach the final max count").
// ======================================================================
// Global-memory node walk (trees too deep for the LDS-tiled kernel, per-tree fp64
// outputs, or more classes than the tiled kernel's counters fit).  One thread per row
// of [row_begin, row_end).  Mode counters are u16 [nclasses][256] in LDS, or, when
// `gcnt` is given (more than kLdsModeClasses classes), u16 [nclasses][row_end -
// row_begin] in global memory, zeroed by the launcher.
__global__ __launch_bounds__(256) void k_predict(const double* __restrict__ X,
                                                 const void* __restrict__ codes, int code_bytes,
                                                 const double* __restrict__ dict,
                                                 const int64_t* __restrict__ dict_off, int64_t N,
                                                 int32_t F, int32_t S,
                                                 const DevNode* __restrict__ nodes,
                                                 const int64_t* __restrict__ tree_off, int L,
                                                 int agg, int nclasses, double* __restrict__ out,
                                                 double* __restrict__ per_tree,
                                                 void* __restrict__ votes, int vote_bytes,
                                                 uint16_t* __restrict__ gcnt, int64_t row_begin,
                                                 int64_t row_end) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x;
  const int64_t row = row_begin + (int64_t)blockIdx.x * 256 + tid;
  if (row >= row_end) return;
  const int64_t cstride = gcnt ? row_end - row_begin : 256;
  uint16_t* cnt = gcnt ? gcnt + (row - row_begin) : (uint16_t*)smem + tid;
  if (agg == kAggMode && !gcnt)
    for (int c = 0; c < nclasses; c++) cnt[c * cstride] = 0;
  double sum = 0.0, mode = 0.0;
  int maxc = 0;
  for (int l = 0; l < L; l++) {
    const DevNode* t = nodes + tree_off[l];
    int id = 0;
    while (t[id].left >= 0) {
      const int g = t[id].gfeat;
      double v;
      if (X) {
        v = X[row * F + g];
      } else {
        const int64_t c = code_bytes == 1   ? (int64_t)((const uint8_t*)codes)[row * S + g]
                          : code_bytes == 2 ? (int64_t)((const uint16_t*)codes)[row * S + g]
                                            : (int64_t)((const uint32_t*)codes)[row * S + g];
        v = dict[dict_off[g] + c];
      }
      id = (v <= t[id].value) ? t[id].left : t[id].right;
    }
    const double pred = t[id].value;
    if (per_tree) per_tree[(int64_t)l * N + row] = pred;
    if (agg == kAggVotes) {
      if (vote_bytes == 1)
        ((uint8_t*)votes)[(int64_t)l * N + row] = (uint8_t)pred;
      else if (vote_bytes == 2)
        ((uint16_t*)votes)[(int64_t)l * N + row] = (uint16_t)pred;
      else
        ((double*)votes)[(int64_t)l * N + row] = pred;
    } else if (agg == kAggMode) {
      const int k = ++cnt[(int64_t)(int)pred * cstride];
      if (k > maxc) {
        maxc = k;
        mode = pred;
      }
    } else {
      sum += pred;
    }
  }
  if (agg != kAggVotes) out[row] = agg == kAggMean ? sum / (double)L : agg == kAggSum ? sum : mode;
}

// `gcnt` (u16 [nclasses][gcnt_rows], more than kLdsModeClasses classes) moves the mode
// counters to global memory; the rows then go in batches of gcnt_rows.
void launch_predict(hipStream_t st, const double* X, const void* codes, int code_bytes,
                    const double* dict, const int64_t* dict_off, int64_t N, int32_t F, int32_t S,
                    const DevNode* nodes, const int64_t* tree_off, int L, int agg, int nclasses,
                    double* out, double* per_tree, void* votes, int vote_bytes, uint16_t* gcnt,
                    int64_t gcnt_rows) {
  const bool global_cnt = agg == kAggMode && gcnt != nullptr;
  const size_t lds = (agg == kAggMode && !global_cnt) ? (size_t)nclasses * 256 * 2 : 0;
  set_max_lds((const void*)k_predict, 160 * 1024);
  const int64_t step = global_cnt ? std::max<int64_t>(gcnt_rows, 1) : std::max<int64_t>(N, 1);
  for (int64_t r0 = 0; r0 < N; r0 += step) {
    const int64_t r1 = std::min(N, r0 + step);
    if (global_cnt) (void)hipMemsetAsync(gcnt, 0, (size_t)nclasses * (size_t)(r1 - r0) * 2, st);
    hipLaunchKernelGGL(k_predict, dim3((unsigned)((r1 - r0 + 255) / 256)), dim3(256), lds, st, X,
                       codes, code_bytes, dict, dict_off, N, F, S, nodes, tree_off, L, agg,
                       nclasses, out, per_tree, global_cnt ? nullptr : votes, vote_bytes,
                       global_cnt ? gcnt : nullptr, r0, r1);
  }
}

// ---- LDS-tiled predict over device-resident rows (transform of large scoring
// sets).  A workgroup stages kPredRows rows of codes (pitch
// S + 4 bytes: rows on distinct banks) and walks them through the forest chunk by
// chunk (packed nodes + leaf values in LDS), trees in learner order: the sum is
// breeze's sequential sum (BaggingRegressor.scala:249-255), the vote breeze's
// mode (first class to reach the final max count, BaggingClassifier.scala:249-257).
// Thresholds are precompiled to code space (code <= tc  <=>  value <= threshold,
// the dictionary being sorted), so a level is two LDS reads and no fp64 compare.
constexpr int kPredRows = 512;  // 2 rows per thread (two independent walks in flight)
constexpr int kPredThreads = 256;

size_t predict_tiled_lds(const PredictArgs& a) {
  const size_t pitch = (size_t)a.S * a.code_bytes + 4;
  size_t b = (size_t)kPredRows * pitch + (size_t)a.chunk_bytes;
  if (a.agg == kAggMode) b += (size_t)a.nclasses * kPredRows * 2;
  return (b + 15) & ~(size_t)15;
}

template <typename CT>
__global__ __launch_bounds__(kPredThreads) void k_predict_tiled(PredictArgs A) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x;
  const int pitch = A.S * (int)sizeof(CT) + 4;
  unsigned char* rows = smem;
  unsigned char* chunk = smem + (size_t)kPredRows * pitch;
  uint16_t* cnt = (uint16_t*)(chunk + A.chunk_bytes);  // [nclasses][kPredRows]
  const int64_t row0 = (int64_t)blockIdx.x * kPredRows;
  const int rb = A.S * (int)sizeof(CT);  // bytes of one row
  for (int q = tid; q < kPredRows * (rb >> 2); q += kPredThreads) {
    const int r = q / (rb >> 2), w = q - r * (rb >> 2);
    uint32_t v = 0;
    if (row0 + r < A.N) v = *(const uint32_t*)((const unsigned char*)A.codes + (row0 + r) * rb + w * 4);
    *(uint32_t*)(rows + r * pitch + w * 4) = v;
  }
  if (A.agg == kAggMode)
    for (int i = tid; i < A.nclasses * kPredRows; i += kPredThreads) cnt[i] = 0;
  double sum0 = 0.0, sum1 = 0.0, mode0 = 0.0, mode1 = 0.0;
  int max0 = 0, max1 = 0;
  const unsigned char* r0p = rows + tid * pitch;
  const unsigned char* r1p = rows + (tid + kPredThreads) * pitch;
  for (int c = 0; c < A.nchunks; c++) {
    const PredictChunk ch = A.chunks[c];
    block_sync();  // previous chunk done (and the row tile written)
    const int nb = (int)(ch.n1 - ch.n0) * 8, lb = (int)(ch.l1 - ch.l0) * 8;
    for (int i = tid; i < (nb >> 3); i += kPredThreads)
      ((PNode*)chunk)[i] = A.nodes[ch.n0 + i];
    for (int i = tid; i < (lb >> 3); i += kPredThreads)
      ((double*)(chunk + nb))[i] = A.leaves[ch.l0 + i];
    block_sync();
    for (int t = ch.t0; t < ch.t1; t++) {
      const PNode* tn = (const PNode*)chunk + (A.tree_node[t] - ch.n0);
      const double* tl = (const double*)(chunk + nb) + (A.tree_leaf[t] - ch.l0);
      uint32_t i0 = 0, i1 = 0;
      PNode a0 = tn[0], a1 = tn[0];
      while (!((a0.a & a1.a) & 0x80000000u)) {  // until both walks reach a leaf
        if (!(a0.a & 0x80000000u)) {
          const uint32_t code = ((const CT*)r0p)[a0.b >> 17];
          i0 = a0.a + (code < (a0.b & 0x1ffffu) ? 0u : 1u);
          a0 = tn[i0];
        }
        if (!(a1.a & 0x80000000u)) {
          const uint32_t code = ((const CT*)r1p)[a1.b >> 17];
          i1 = a1.a + (code < (a1.b & 0x1ffffu) ? 0u : 1u);
          a1 = tn[i1];
        }
      }
      const double p0 = tl[a0.a & 0x7fffffffu], p1 = tl[a1.a & 0x7fffffffu];
      if (A.agg == kAggMean || A.agg == kAggSum) {
        sum0 += p0;
        sum1 += p1;
      } else if (A.agg == kAggVotes) {  // class id of tree t for both rows: [L][N] u8/u16
        const int64_t v0 = (int64_t)t * A.N + row0 + tid, v1 = v0 + kPredThreads;
        if (A.vote_bytes == 1) {
          if (row0 + tid < A.N) ((uint8_t*)A.votes)[v0] = (uint8_t)p0;
          if (row0 + tid + kPredThreads < A.N) ((uint8_t*)A.votes)[v1] = (uint8_t)p1;
        } else if (A.vote_bytes == 8) {  // per-tree fp64 predictions (any impurity)
          if (row0 + tid < A.N) ((double*)A.votes)[v0] = p0;
          if (row0 + tid + kPredThreads < A.N) ((double*)A.votes)[v1] = p1;
        } else {
          if (row0 + tid < A.N) ((uint16_t*)A.votes)[v0] = (uint16_t)p0;
          if (row0 + tid + kPredThreads < A.N) ((uint16_t*)A.votes)[v1] = (uint16_t)p1;
        }
      } else {
        const int k0 = ++cnt[(int)p0 * kPredRows + tid];
        if (k0 > max0) {
          max0 = k0;
          mode0 = p0;
        }
        const int k1 = ++cnt[(int)p1 * kPredRows + tid + kPredThreads];
        if (k1 > max1) {
          max1 = k1;
          mode1 = p1;
        }
      }
    }
  }
  if (A.agg == kAggVotes) return;
  const double o0 = A.agg == kAggMean ? sum0 / (double)A.L : A.agg == kAggSum ? sum0 : mode0;
  const double o1 = A.agg == kAggMean ? sum1 / (double)A.L : A.agg == kAggSum ? sum1 : mode1;
  if (row0 + tid < A.N) A.out[row0 + tid] = o0;
  if (row0 + tid + kPredThreads < A.N) A.out[row0 + tid + kPredThreads] = o1;
}

// rows -> u16 codes against the forest's thresholds of each feature:
// code = #{t < x} (binary search), so x <= t_k <=> code <= k; NaN compares false
// with everything in Spark (goes right) -> the code past every threshold
__global__ __launch_bounds__(256) void k_quantize(const double* __restrict__ X, int64_t n, int32_t F,
                                                  const double* __restrict__ thr,
                                                  const int64_t* __restrict__ toff,
                                                  uint16_t* __restrict__ codes, int32_t S) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n * S) return;
  const int64_t row = i / S;
  const int g = (int)(i - row * S);
  uint32_t code = 0;
  if (g < F) {
    const double x = X[row * F + g];
    int64_t lo = toff[g], hi = toff[g + 1];
    if (x != x) {
      lo = hi;
    } else {
      while (lo < hi) {  // first threshold >= x
        const int64_t mid = (lo + hi) >> 1;
        if (thr[mid] < x)
          lo = mid + 1;
        else
          hi = mid;
      }
    }
    code = (uint32_t)(lo - toff[g]);
  }
  codes[i] = (uint16_t)code;
}

void launch_quantize(hipStream_t st, const double* X, int64_t n, int32_t F, const double* thr,
                     const int64_t* toff, uint16_t* codes, int32_t S) {
  const int64_t total = n * S;
  hipLaunchKernelGGL(k_quantize, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, X, n, F,
                     thr, toff, codes, S);
}

void launch_predict_tiled(hipStream_t st, const PredictArgs& a) {
  const size_t lds = predict_tiled_lds(a);
  set_max_lds((const void*)k_predict_tiled<uint8_t>, 160 * 1024);
  set_max_lds((const void*)k_predict_tiled<uint16_t>, 160 * 1024);
  const dim3 grid((unsigned)((a.N + kPredRows - 1) / kPredRows));
  if (a.code_bytes == 1)
    hipLaunchKernelGGL(k_predict_tiled<uint8_t>, grid, dim3(kPredThreads), lds, st, a);
  else
    hipLaunchKernelGGL(k_predict_tiled<uint16_t>, grid, dim3(kPredThreads), lds, st, a);
}

// Ordered aggregation of K rows of per-row values [K][N] (K = learners, or ranks'
// partial sums): kAggMean -> (in-order sum) / num_learners, kAggMode -> breeze mode
// of class ids (first class to reach the final max count).  VT: fp64 values (host
// per-tree predictions / partial sums) or u8 / u16 class ids (device votes after the
// all-to-all).  Counters as in k_predict.
template <typename VT>
__global__ __launch_bounds__(256) void k_aggregate(const VT* __restrict__ votes, int K, int64_t N,
                                                   int agg, int nclasses, double num_learners,
                                                   double* __restrict__ out,
                                                   uint16_t* __restrict__ gcnt, int64_t row_begin,
                                                   int64_t row_end) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x;
  const int64_t row = row_begin + (int64_t)blockIdx.x * 256 + tid;
  if (row >= row_end) return;
  const int64_t cstride = gcnt ? row_end - row_begin : 256;
  uint16_t* cnt = gcnt ? gcnt + (row - row_begin) : (uint16_t*)smem + tid;
  if (agg == kAggMode && !gcnt)
    for (int c = 0; c < nclasses; c++) cnt[c * cstride] = 0;
  double sum = 0.0, mode = 0.0;
  int maxc = 0;
  for (int l = 0; l < K; l++) {
    const double v = (double)votes[(int64_t)l * N + row];
    if (agg == kAggMode) {
      const int k = ++cnt[(int64_t)(int)v * cstride];
      if (k > maxc) {
        maxc = k;
        mode = v;
      }
    } else {
      sum += v;
    }
  }
  out[row] = agg == kAggMode ? mode : sum / num_learners;
}

template <typename VT>
static void launch_aggregate_t(hipStream_t st, const VT* votes, int K, int64_t N, int agg,
                               int nclasses, double num_learners, double* out, uint16_t* gcnt,
                               int64_t gcnt_rows) {
  const bool global_cnt = agg == kAggMode && gcnt != nullptr;
  const size_t lds = (agg == kAggMode && !global_cnt) ? (size_t)nclasses * 256 * 2 : 0;
  set_max_lds((const void*)k_aggregate<VT>, 160 * 1024);
  const int64_t step = global_cnt ? std::max<int64_t>(gcnt_rows, 1) : std::max<int64_t>(N, 1);
  for (int64_t r0 = 0; r0 < N; r0 += step) {
    const int64_t r1 = std::min(N, r0 + step);
    if (global_cnt) (void)hipMemsetAsync(gcnt, 0, (size_t)nclasses * (size_t)(r1 - r0) * 2, st);
    hipLaunchKernelGGL(k_aggregate<VT>, dim3((unsigned)((r1 - r0 + 255) / 256)), dim3(256), lds, st,
                       votes, K, N, agg, nclasses, num_learners, out, global_cnt ? gcnt : nullptr,
                       r0, r1);
  }
}

void launch_aggregate(hipStream_t st, const void* votes, int vote_bytes, int K, int64_t N, int agg,
                      int nclasses, double num_learners, double* out, uint16_t* gcnt,
                      int64_t gcnt_rows) {
  if (vote_bytes == 1)
    launch_aggregate_t(st, (const uint8_t*)votes, K, N, agg, nclasses, num_learners, out, gcnt,
                       gcnt_rows);
  else if (vote_bytes == 2)
    launch_aggregate_t(st, (const uint16_t*)votes, K, N, agg, nclasses, num_learners, out, gcnt,
                       gcnt_rows);
  else
    launch_aggregate_t(st, (const double*)votes, K, N, agg, nclasses, num_learners, out, gcnt,
                       gcnt_rows);
}

}  // namespace sbag
