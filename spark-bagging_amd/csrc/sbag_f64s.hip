// sbag_f64s.hip — the screened fp64 engine: bagging regression on arbitrary fp64 labels
// without histogramming every feature in Spark's row order.
//
// Spark's DecisionTreeRegressor sums each (node, feature, bin) cell in fp64, row by row
// (DTStatsAggregator.update; a row drawn c times is c consecutive rows,
// sql/bfunctions.scala:42-44), so its gains depend on the summation order.  But only the
// CHOSEN split's statistics reach the model (node impurity, gain, the children's
// calculators); the other candidates matter only through the argmax.  So:
//
//   k_f64_screen   per node, every candidate's gain from the integer histograms of the
//                  labels' fixed-point image k = round(y 2^s) (k_hist / k_hist_rl: exact
//                  integer sums), with a rigorous bound on Spark's fp64 value: the
//                  fixed-point error (|y - k 2^-s| <= eps), the summation error of the
//                  row-order sums and Spark's rounding of the gain formula (host, dnode /
//                  dpar).  The first max is Spark's when no other candidate's upper bound
//                  reaches its lower bound and that lower bound is > 0 and >= minInfoGain;
//                  otherwise the node is flagged and histogrammed exactly (k_f64_hist,
//                  every feature in row order, then k_f64_split).
//   k_fb_count / k_fb_scan / k_fb_scatter   for every decided node (and, at the root,
//                  its first feature with splits, whose bins give Spark's parent stats):
//                  a stable bucketing of the node's entries (row order) by the chosen
//                  feature's bin, fused with the stable two-way partition of
//                  every split node into its children (left |= bin <= s), which keeps the
//                  children's entries in row order for the next level
//   k_fb_chainx    one partition: one lane per (task, bin), the bucket's rows in row order,
//                  each label added count times (a row drawn c times is c consecutive
//                  rows) -- Spark's cell sums bit for bit
//   k_fb_runs / k_fb_psum / k_fb_pmerge   several partitions: Spark's per-partition
//                  aggregates (row order inside a partition, a chain per (task, partition,
//                  bin), no buckets), merged per (task, bin) in partition order (reduceByKey)
//   k_fb_finish    binsToBestSplit over the chosen feature's exact bins (prefixes in bin
//                  order, right = total - left, calculateImpurityStats with the node's
//                  chained stats): the node's gain, impurity and children calculators
//
// Reference: ml/ensemble/ensembleParams.scala:113-115 (fitBaseLearner ->
// DecisionTreeRegressor.train), ml/regression/BaggingRegressor.scala:146-150 (any Double
// label); upstream RandomForest.findBestSplits / binsToBestSplit (Spark 2.4.3).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>

#include "sbag_internal.h"

namespace sbag {

namespace {
constexpr double kU = 1.1102230246251565e-16;          // 2^-53, unit roundoff
constexpr double kMinValueS = -1.7976931348623157e308;  // Double.MinValue

__device__ __forceinline__ double var_imp(double count, double sum, double sumsq) {
  if (count == 0) return 0.0;  // Variance.calculate
  const double squared_loss = sumsq - (sum * sum) / count;
  return squared_loss / count;
}

// block-wide exclusive scan of one int per thread (256 threads); block total in *total
__device__ __forceinline__ int64_t scan256(int64_t v, int64_t* s_wave, int64_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int64_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == 63) s_wave[wave] = incl;
  block_sync();
  int64_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    if (w < wave) before += s_wave[w];
    tot += s_wave[w];
  }
  block_sync();
  *total = tot;
  return before + incl - v;
}
}  // namespace

// ---------------------------------------------------------------- screen
// One candidate (lc, lsk) of a node (tc, tsk): the screened gain g = wL wR (muL - muR)^2
// (the variance gain in exact arithmetic: Spark's sums of squares cancel) and a bound a on
// |g - g*|, g* the exact-arithmetic gain of the true labels.  muL = lsk 2^-s / lc is within
// eps of the true left mean; D = muL - muR within eD of the true difference, rounding
// included; g = w D^2 within w ((|D| + eD)^2 - D^2) + 8u w (|D| + eD)^2.
__device__ __forceinline__ void screen_cand(int64_t lc, int64_t lsk, int64_t tc, int64_t tsk, double n,
                                            double is, double eps, double* g, double* a) {
  const int64_t rc = tc - lc, rsk = tsk - lsk;
  const double muL = (double)lsk * is / (double)lc;
  const double muR = (double)rsk * is / (double)rc;
  const double D = muL - muR;
  const double w = ((double)lc / n) * ((double)rc / n);
  *g = w * D * D;
  const double eD = 2.0 * eps + 2.0 * kU * (fabs(muL) + fabs(muR) + fabs(D));
  const double hiD = fabs(D) + eD;
  *a = (w * (hiD * hiD - D * D) + 8.0 * kU * w * hiD * hiD) * 1.0001;
}

__global__ __launch_bounds__(256) void k_f64_screen(F64ScreenArgs A) {
  const int slot = blockIdx.x, tid = threadIdx.x;
  const int r = A.slot_r[slot];
  const int Fr = A.Fr[r];
  const int NB = A.NB;
  const int64_t slot_words = (int64_t)A.Fmax * NB * 3;
  __shared__ double s_g[256], s_a[256];
  __shared__ int s_fl[256], s_s[256], s_cnt[256];
  __shared__ int64_t s_tot[2];
  const int32_t* nb_r = A.nbins + (int64_t)r * A.Fmax;
  const uint64_t* hs = A.hist + (int64_t)slot * slot_words;
  if (tid < 2) {  // the node's count and Σ c k (every feature's bins hold the same rows)
    int64_t t = 0;
    for (int b = 0; b < NB; b++) t += (int64_t)hs[(int64_t)b * 3 + tid];
    s_tot[tid] = t;
  }
  block_sync();
  const int64_t tc = s_tot[0], tsk = s_tot[1];
  const double n = (double)tc, is = A.inv_scale, eps = A.eps;
  // pass 1: first max of the screened gain (features in order, bins in order)
  double fgb = -INFINITY, fab = 0.0;
  int ffl = INT_MAX, fs = -1;
  for (int fl = tid; fl < Fr; fl += 256) {
    const int nsp = nb_r[fl] - 1;
    const uint64_t* h = hs + (int64_t)fl * NB * 3;
    int64_t lc = 0, lsk = 0;
    for (int s = 0; s < nsp; s++) {
      lc += (int64_t)h[s * 3];
      lsk += (int64_t)h[s * 3 + 1];
      if (lc < A.min_inst || tc - lc < A.min_inst) continue;  // invalid in Spark: MinValue
      double g, a;
      screen_cand(lc, lsk, tc, tsk, n, is, eps, &g, &a);
      if (g > fgb) {
        fgb = g;
        fab = a;
        ffl = fl;
        fs = s;
      }
    }
  }
  s_g[tid] = fgb;
  s_a[tid] = fab;
  s_fl[tid] = ffl;
  s_s[tid] = fs;
  block_sync();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const double g2 = s_g[tid + o];
      const int f2 = s_fl[tid + o];
      if (g2 > s_g[tid] || (g2 == s_g[tid] && f2 < s_fl[tid])) {
        s_g[tid] = g2;
        s_a[tid] = s_a[tid + o];
        s_fl[tid] = f2;
        s_s[tid] = s_s[tid + o];
      }
    }
    block_sync();
  }
  const double gb = s_g[0], ab = s_a[0];
  const int bfl = s_fl[0], bs = s_s[0];
  const double dn = A.dnode[slot], dp = A.dpar[slot];
  block_sync();
  // pass 2: candidates whose upper bound reaches the best's lower bound (the best too), and
  // per feature whether it holds one: a flagged node's exact fallback needs only those
  // features (every other candidate's exact gain is below the best's, so it can be neither
  // Spark's argmax nor tie with it)
  int cnt = 0;
  uint8_t* cm = A.cmask + (int64_t)slot * A.Fmax;
  const double thr = gb - ab - 2.0 * dn;
  for (int fl = tid; fl < Fr; fl += 256) {
    int fc = 0;
    if (bfl != INT_MAX) {
      const int nsp = nb_r[fl] - 1;
      const uint64_t* h = hs + (int64_t)fl * NB * 3;
      int64_t lc = 0, lsk = 0;
      for (int s = 0; s < nsp; s++) {
        lc += (int64_t)h[s * 3];
        lsk += (int64_t)h[s * 3 + 1];
        if (lc < A.min_inst || tc - lc < A.min_inst) continue;
        double g, a;
        screen_cand(lc, lsk, tc, tsk, n, is, eps, &g, &a);
        if (!(g + a < thr)) fc++;  // NaN counts as a contender
      }
    }
    cm[fl] = fc > 0 ? 1 : 0;
    cnt += fc;
  }
  s_cnt[tid] = cnt;
  block_sync();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) s_cnt[tid] += s_cnt[tid + o];
    block_sync();
  }
  if (tid == 0) {
    F64ScreenOut o{};
    if (bfl == INT_MAX) {  // no count-valid candidate: decided exactly (leaf stats)
      o.f = -1;
      o.s = -1;
      o.flag = 1;
    } else {
      // Spark's gain of the best lies in [gb - ab - dn - dp, ...]: a split (> 0) and
      // valid (>= minInfoGain) for sure, and no other candidate can reach it
      const double lo = gb - ab - dn - dp;
      const bool certain = s_cnt[0] == 1 && lo > 0.0 && lo >= A.min_gain;
      o.f = bfl;
      o.s = bs;
      o.flag = certain ? 0 : 1;
      o.gain = gb;
      o.margin = lo;
    }
    A.out[slot] = o;
  }
}

void launch_f64_screen(hipStream_t st, const F64ScreenArgs& a, int M) {
  hipLaunchKernelGGL(k_f64_screen, dim3(M), dim3(256), 0, st, a);
}

// ---------------------------------------------------------------- bucket + route
__device__ __forceinline__ const uint8_t* task_col(const F64BucketArgs& A, const F64Task& t) {
  return A.cols + (int64_t)t.r * A.cols_rstride + (int64_t)t.col * A.npad;
}

__device__ __forceinline__ uint32_t task_bin(const uint8_t* col, uint64_t e) {
  return col ? (uint32_t)col[(uint32_t)e] : 0u;
}

// Buffer resources make every lane's gather and store the same instruction whatever its
// entry: an offset past the resource's size reads 0 and drops a store.  (Exec-masked
// branches around memory operations leave the compiler's vmcnt counting uncertain on the
// merged path, and it then waits for every outstanding load and store.)
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(uint32_t)bytes, 0x00020000);
}
// the task's bin column (rows < 2^32 bytes); the node-total task (col < 0): size 0, bin 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t task_col_rsrc(const F64BucketArgs& A, const F64Task& t) {
  return t.col >= 0 ? rsrc_of(task_col(A, t), (uint64_t)A.npad) : rsrc_of(A.cols, 0);
}
__device__ __forceinline__ uint32_t rbin(__amdgpu_buffer_rsrc_t rc, uint64_t e) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rc, (int)(uint32_t)e, 0, 0);
}
__device__ __forceinline__ void rstore64(__amdgpu_buffer_rsrc_t r, uint32_t off, uint64_t v) {
  v2u32 w;
  w.x = (uint32_t)v;
  w.y = (uint32_t)(v >> 32);
  __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)off, 0, 0);
}

// per piece: entries per bin of the task's feature, entries going left (bin <= s).  Each
// thread takes 8 entries per step, their loads (clamped indices: no branches, so the
// gathers are issued back to back) and gathers before the atomics.
__global__ __launch_bounds__(256) void k_fb_count(F64BucketArgs A) {
  // (porder: the dispatch order of the pieces, XCD-aware; the outputs stay per piece)
  const int64_t pix = A.porder ? (int64_t)A.porder[blockIdx.x] : (int64_t)blockIdx.x;
  const F64TPiece pc = A.pieces[pix];
  const F64Task t = A.tasks[pc.task];
  const int NB = A.NB, tid = threadIdx.x;
  const bool counting = !A.psum;  // (the per-bin counts place buckets; psum has none)
  __shared__ uint32_t s_c[256];
  __shared__ uint32_t s_l[4];
  for (int b = tid; b < NB; b += 256) s_c[b] = 0u;
  block_sync();
  const __amdgpu_buffer_rsrc_t rc = task_col_rsrc(A, t);
  // the gathered bins with the draw counts (bin | count << 8), kept for k_fb_scatter and
  // k_fb_psum (which then read them in order)
  const __amdgpu_buffer_rsrc_t re = rsrc_of(A.ebin + t.ebase, (uint64_t)(t.b - t.a) * 2);
  uint32_t nl = 0;
  constexpr int U = 8;
  const int64_t last = pc.b - 1;
  for (int64_t i0 = pc.a; i0 < pc.b; i0 += 256 * U) {
    uint64_t e[U];
    uint32_t bin[U];
#pragma unroll
    for (int u = 0; u < U; u++) e[u] = A.ent_in[min(i0 + u * 256 + tid, last)];
#pragma unroll
    for (int u = 0; u < U; u++) bin[u] = rbin(rc, e[u]);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = i0 + u * 256 + tid;
      // (lanes past the piece store past the resource: dropped)
      __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(bin[u] | ((uint32_t)(e[u] >> 32) & 0xffu) << 8), re,
                                            i < pc.b ? (int)(uint32_t)(2 * (i - t.a)) : -1, 0, 0);
      if (i < pc.b) {
        if (counting) atomicAdd(&s_c[bin[u]], 1u);
        nl += bin[u] <= (uint32_t)t.s ? 1u : 0u;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) nl += __shfl_down(nl, o);
  if ((tid & 63) == 0) s_l[tid >> 6] = nl;
  block_sync();
  if (counting)
    for (int b = tid; b < NB; b += 256) A.pcnt[pix * NB + b] = s_c[b];
  if (tid == 0) A.plcnt[pix] = s_l[0] + s_l[1] + s_l[2] + s_l[3];
}

// per task: bucket bounds (bins in order, each bin's entries in row order), each piece's
// first position per bin, left entries before each piece, the task's left total
__global__ __launch_bounds__(256) void k_fb_scan(F64BucketArgs A) {
  const int task = blockIdx.x, tid = threadIdx.x, NB = A.NB;
  const F64Task t = A.tasks[task];
  __shared__ int64_t s_start[257];
  __shared__ int64_t s_wave[4];
  if (t.kbase >= 0 && !A.psum) {
    int64_t tot = 0;
    if (tid < NB)
      for (int64_t p = t.piece0; p < t.piece1; p++) tot += A.pcnt[p * NB + tid];
    int64_t all;
    const int64_t ex = scan256(tid < NB ? tot : 0, s_wave, &all);
    if (tid < NB) s_start[tid] = ex;
    if (tid == 0) s_start[NB] = all;
    block_sync();
    int64_t* ko = A.kb_off + (int64_t)task * (NB + 1);
    for (int b = tid; b <= NB; b += 256) ko[b] = t.kbase + s_start[b];
    if (tid < NB) {
      int64_t run = t.kbase + s_start[tid];
      for (int64_t p = t.piece0; p < t.piece1; p++) {
        A.pbase[p * NB + tid] = run;
        run += A.pcnt[p * NB + tid];
      }
    }
  }
  if (t.part) {
    int64_t carry = 0;
    for (int64_t p0 = t.piece0; p0 < t.piece1; p0 += 256) {
      const int64_t p = p0 + tid;
      int64_t tot;
      const int64_t ex = scan256(p < t.piece1 ? (int64_t)A.plcnt[p] : 0, s_wave, &tot);
      if (p < t.piece1) A.plbase[p] = carry + ex;
      carry += tot;
    }
    if (tid == 0) A.nleft[task] = carry;
  }
}

// one wave per piece: every entry to its bucket (stable: its rank among the round's
// entries of the same bin, from ballots over the bin's bits) and, for split nodes, to its
// child (left from the segment start, right after the left block, both in row order).
// Every lane issues the same memory operations each round (loads at clamped indices, one
// bucket store, one child store, buffer operations whose out-of-range offsets are dropped),
// so the compiler's vmcnt waits stay counted.  (The wave's LDS operations execute in
// order, and the compiler keeps a store to sb[x] before a later load of sb[y] it cannot
// prove distinct: no fence, which would drain the vector memory counter too.)
// A step's 512 entries are first ordered by bin in LDS, so the bucket stores leave as runs of
// consecutive positions (stored straight from the rounds, a 64-entry round spread over up to
// NB buckets: 2-entry runs of 8-byte labels and 1-byte counts, written back ~1.7x their bytes
// as measured by WRITE_SIZE; that variant was removed in round 6).
constexpr int kScU = 8;  // rounds of 64 entries per step
// kWide (datasets of >= 2^28 rows): the 8-byte labels, buckets and children are addressed by
// 64-bit pointers with predicated stores -- a buffer resource spans at most 4 GB, and a task's
// segment (up to a replica's every in-bag row) or the label column (8 N bytes) may not
template <bool kWide>
__global__ __launch_bounds__(256) void k_fb_scatter(F64BucketArgs A, int64_t npieces, int nbits) {
  // (the wave index in an SGPR: the piece, its task and the buffer resources built from them
  // are then wave-uniform, with no per-lane waterfall loop around the buffer operations)
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t pi = (int64_t)blockIdx.x * 4 + wv;
  __shared__ int64_t s_base[4][256];
  // staging: per wave the step's bin counts and offsets, and its entries by bin
  __shared__ uint32_t s_scnt[4][256], s_soff[4][256];
  __shared__ v2u32 s_sy[4][64 * kScU];
  __shared__ uint32_t s_skp[4][64 * kScU];
  __shared__ uint8_t s_sc[4][64 * kScU];
  if (pi >= npieces) return;  // whole waves only; no block-wide barrier below
  const F64TPiece pc = A.pieces[pi];
  const F64Task t = A.tasks[pc.task];
  const int NB = A.NB;
  // (uniform: SGPR resources; psum: k_fb_psum sums per partition without buckets, this only routes)
  const bool chain = __builtin_amdgcn_readfirstlane((int)(t.kbase >= 0 && !A.psum)) != 0;
  int64_t* sb = s_base[wv];
  for (int b = lane; b < NB; b += 64) sb[b] = chain ? A.pbase[pi * NB + b] : 0;
  uint32_t* scnt = s_scnt[wv];
  uint32_t* soff = s_soff[wv];
  for (int b = lane; b < 256; b += 64) scnt[b] = 0u;
  int64_t lrun = t.part ? A.plbase[pi] : 0;
  const int64_t nl = t.part ? A.nleft[pc.task] : 0;
  // the entries' bins as k_fb_count gathered them (in entry order: coalesced; bin | count << 8)
  const __amdgpu_buffer_rsrc_t re = rsrc_of(A.ebin + t.ebase, (uint64_t)(t.b - t.a) * 2);
  // the task's buckets (labels and counts) and its children's segment (each < 4 GB: a
  // node's entries); the labels (rows < 2^28 on this path; kWide takes 64-bit pointers)
  const uint64_t nk = chain ? (uint64_t)(t.b - t.a) : 0;
  const __amdgpu_buffer_rsrc_t rk = rsrc_of(A.bky + (chain ? t.kbase : 0), nk * 8);
  const __amdgpu_buffer_rsrc_t rkc = rsrc_of(A.bkc + (chain ? t.kbase : 0), nk);
  const __amdgpu_buffer_rsrc_t ro = rsrc_of(A.ent_out + t.a, t.part ? (uint64_t)(t.b - t.a) * 8 : 0);
  // the entries' labels: carried in entry order (coalesced; and the children's written),
  // or, without the carried copy (ey_in null: too big), gathered by row
  const bool carried = A.ey_in != nullptr;
  const __amdgpu_buffer_rsrc_t ry =
      carried ? rsrc_of(A.ey_in + t.a, (uint64_t)(t.b - t.a) * 8) : rsrc_of(A.y, 0xFFFFFFFFull);
  const __amdgpu_buffer_rsrc_t roy =
      rsrc_of(carried ? A.ey_out + t.a : A.ey_out, carried && t.part ? (uint64_t)(t.b - t.a) * 8 : 0);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t last = pc.b - 1;
  // kScU rounds of 64 entries per step: all their entry loads, then all their bin and label
  // gathers, then the rounds' ballots and stores -- one memory latency per step, not per
  // round (vmcnt counts stores and loads in order on gfx9, so loads carried across steps
  // would wait for the stores issued after them anyway)
  for (int64_t i0 = pc.a; i0 < pc.b; i0 += 64 * kScU) {
    uint64_t ev[kScU];
    uint32_t bv[kScU];
    v2u32 yv[kScU];
    uint32_t rs[kScU];  // rank among the step's entries of the same bin
#pragma unroll
    for (int u = 0; u < kScU; u++) ev[u] = A.ent_in[min(i0 + 64 * u + lane, last)];
#pragma unroll
    for (int u = 0; u < kScU; u++) {
      bv[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(re, (int)(uint32_t)(2 * (min(i0 + 64 * u + lane, last) - t.a)), 0, 0) & 0xffu;
      if constexpr (kWide) {
        const double* yp = carried ? A.ey_in + min(i0 + 64 * u + lane, last) : A.y + (uint32_t)ev[u];
        yv[u] = *(const v2u32*)yp;
      } else {
        const int yoff = carried ? (int)(min(i0 + 64 * u + lane, last) - t.a) * 8 : (int)((uint32_t)ev[u] * 8u);
        yv[u] = __builtin_amdgcn_raw_buffer_load_b64(ry, yoff, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < kScU; u++) {
      const int64_t i = i0 + 64 * u + lane;
      const bool valid = i < pc.b;
      const uint64_t e = ev[u];
      const uint32_t bin = valid ? bv[u] : 0u;
      // every store every round, whatever the task does (a task without buckets or
      // without children has zero-size resources: the stores are dropped) -- no branch
      uint64_t eq = __ballot(valid);
      for (int k = 0; k < (chain ? nbits : 0); k++) {  // (ranks by bin: only for the buckets)
        const bool bit = (bin >> k) & 1u;
        const uint64_t m = __ballot(bit);
        eq &= bit ? m : ~m;
      }
      const int rank = __popcll(eq & lt), cnt = __popcll(eq);
      {
        const uint32_t so = scnt[bin];
        rs[u] = so + (uint32_t)rank;
        if (valid && rank == cnt - 1) scnt[bin] = so + (uint32_t)cnt;
      }
      const bool left = valid && bin <= (uint32_t)t.s;
      const uint64_t lm = __ballot(left);
      const int64_t lr = __popcll(lm & lt);
      const int64_t pos = left ? lrun + lr : nl + (i - t.a - lrun - lr);  // within the segment
      if constexpr (kWide) {
        if (valid && t.part) {
          A.ent_out[t.a + pos] = e;
          if (carried) *(v2u32*)(A.ey_out + t.a + pos) = yv[u];
        }
      } else {
        rstore64(ro, valid ? (uint32_t)pos * 8u : 0xFFFFFFF0u, e);
        __builtin_amdgcn_raw_buffer_store_b64(yv[u], roy, valid ? (int)((uint32_t)pos * 8u) : -16, 0, 0);
      }
      lrun += __popcll(lm);
    }
    {
      if (chain) {
        // step offsets per bin (exclusive scan over the bins, 4 per lane), then every entry
        // to its slot: bins in order, row order inside a bin
        __builtin_amdgcn_wave_barrier();
        uint32_t c4[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          c4[k] = scnt[4 * lane + k];
          sum += c4[k];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t v = __shfl_up(incl, o);
          if (lane >= o) incl += v;
        }
        uint32_t run = incl - sum;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          soff[4 * lane + k] = run;
          run += c4[k];
        }
        __builtin_amdgcn_wave_barrier();
        v2u32* sy = s_sy[wv];
        uint32_t* skp = s_skp[wv];
        uint8_t* sc = s_sc[wv];
#pragma unroll
        for (int u = 0; u < kScU; u++) {
          const bool valid = i0 + 64 * u + lane < pc.b;
          const uint32_t bin = valid ? bv[u] : 0u;
          if (valid) {
            const uint32_t slot = soff[bin] + rs[u];
            sy[slot] = yv[u];
            sc[slot] = (uint8_t)(ev[u] >> 32);
            skp[slot] = (uint32_t)(sb[bin] - t.kbase) + rs[u];
          }
        }
        __builtin_amdgcn_wave_barrier();
        // bucket positions advance by the step's counts; the counts restart
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int b = 4 * lane + k;
          if (b < NB) sb[b] += c4[k];
          scnt[b] = 0u;
        }
        const int nst = (int)min((int64_t)(64 * kScU), pc.b - i0);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < kScU; k++) {
          const int q = 64 * k + lane;
          const bool ok = q < nst;
          const uint32_t kp = ok ? skp[q] : 0x1FFFFFFEu;
          const v2u32 y = sy[ok ? q : 0];
          const uint32_t cb = sc[ok ? q : 0];
          if constexpr (kWide) {
            if (ok) {
              *(v2u32*)(A.bky + t.kbase + kp) = y;
              A.bkc[t.kbase + kp] = (uint8_t)cb;
            }
          } else {
            __builtin_amdgcn_raw_buffer_store_b64(y, rk, (int)(kp * 8u), 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)cb, rkc, (int)kp, 0, 0);
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
}

// Spark's row-order fp64 sums of every bucket (one partition): one lane per (task, bin), kChC
// chains per wave.  A lane's adds are one dependent chain, so what paces a long chain is the
// instructions between two adds: the draws are exploded in LDS first.  The whole wave turns a
// stage of 512 entries (kChT per chain, kChC chains) into draw streams: the (sumSq term)
// products and the draw positions (a scan of the counts per chain) are computed in parallel,
// entry e of count c is written c times as (w, w*y), and every chain is padded to the wave's
// longest stream with (-0.0, -0.0), which leaves a sum unchanged (-0.0 included), so the serial
// loop is one 16-byte LDS read and two adds per draw with a uniform trip count.  A stage's
// draws beyond kDcap per chain go through further windows.  The count is the integer sum of
// the draws.  (Round 4: 22 cycles per draw against 100 with a per-entry count loop,
// scripts/micro/chain_lat.hip; the per-entry kernel and a 64-chains-per-wave variant were
// measured slower and removed in round 6.)
template <int kChC>
__global__ __launch_bounds__(64) void k_fb_chainx(F64BucketArgs A, int nchain) {
  constexpr int kChT = 512 / kChC;     // entries per chain per stage
  constexpr int kLd = 8;               // 512 entries = 8 loads of 64
  constexpr int kDcap = 2 * kChT;      // draws per chain per window
  constexpr int kDp = kDcap + 1;       // odd pitch (16-byte units): conflict-free serial reads
  __shared__ double2 s_d[kChC * kDp + 8];
  const int NB = A.NB, lane = threadIdx.x;
  const int nbits = min(8, 32 - (int)__builtin_clz((uint32_t)max(A.cmax, 1)));  // of a count
  const int64_t nlanes = (int64_t)nchain * NB;
  const int64_t g = (int64_t)blockIdx.x * kChC + lane;
  int64_t lo = 0, hi = 0;
  if (lane < kChC && g < nlanes) {
    const int64_t task = g / NB;
    const int b = (int)(g - task * NB);
    const int64_t* ko = A.kb_off + task * (NB + 1);
    lo = ko[b];
    hi = ko[b + 1];
  }
  const int64_t len = hi - lo;
  int64_t maxlen = len;
  for (int o = 32; o > 0; o >>= 1) maxlen = max(maxlen, (int64_t)__shfl_xor(maxlen, o));
  // load u, lane l: slot 64u + l = chain j's entry x of the stage
  int64_t ulo[kLd], ulen[kLd];
  int ux[kLd], uj[kLd];
#pragma unroll
  for (int u = 0; u < kLd; u++) {
    const int slot = 64 * u + lane;
    uj[u] = slot / kChT;
    ux[u] = slot % kChT;
    ulo[u] = __shfl(lo, uj[u]);
    ulen[u] = __shfl(len, uj[u]);
  }
  auto load = [&](int64_t off, double (&yv)[kLd], uint32_t (&cv)[kLd]) {
#pragma unroll
    for (int u = 0; u < kLd; u++) {
      const int64_t at = max(min(ulo[u] + off + ux[u], ulo[u] + ulen[u] - 1), (int64_t)0);
      yv[u] = A.bky[at];
      cv[u] = (uint32_t)A.bkc[at];
    }
  };
  double yA[kLd], yB[kLd];
  uint32_t cA[kLd], cB[kLd];
  if (maxlen > 0) {
    load(0, yA, cA);
    load(kChT, yB, cB);
  }
  double s1 = 0.0, s2 = 0.0;
  uint64_t cnt = 0;
  for (int64_t off = 0; off < maxlen; off += kChT) {
    uint32_t cc[kLd];
    double w[kLd], wy[kLd];
#pragma unroll
    for (int u = 0; u < kLd; u++) {
      cc[u] = off + ux[u] < ulen[u] ? cA[u] : 0u;
      w[u] = 1.0 * yA[u];    // instanceWeight * label
      wy[u] = w[u] * yA[u];  // instanceWeight * label * label
    }
#pragma unroll
    for (int u = 0; u < kLd; u++) {
      yA[u] = yB[u];
      cA[u] = cB[u];
    }
    if (off + 2 * kChT < maxlen) load(off + 2 * kChT, yB, cB);
    // draw positions: exclusive prefix of the counts per chain from ballots of their bits
    // (lanes below this one in its chain's segment: mbcnt), D[j] = chain j's draws
    uint32_t pre[kLd];
    int D[kChC], T[kLd];  // T: a whole load's draws (kChT >= 64)
#pragma unroll
    for (int u = 0; u < kLd; u++) {
      pre[u] = 0;
      T[u] = 0;
    }
#pragma unroll
    for (int j = 0; j < kChC; j++) D[j] = 0;
#pragma unroll
    for (int b = 0; b < 8; b++) {
      if (b >= nbits) break;
#pragma unroll
      for (int u = 0; u < kLd; u++) {
        const uint64_t bal = __ballot((cc[u] >> b) & 1u);
        uint32_t mlo, mhi;
        if constexpr (kChT >= 64) {
          mlo = (uint32_t)bal;
          mhi = (uint32_t)(bal >> 32);
        } else {  // this lane's kChT-lane segment
          const uint64_t seg = ((1ull << kChT) - 1) << (lane & ~(kChT - 1));
          mlo = (uint32_t)(bal & seg);
          mhi = (uint32_t)((bal & seg) >> 32);
        }
        pre[u] += __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u)) << b;
        if constexpr (kChT >= 64) {
          T[u] += __popcll(bal) << b;
        } else {
#pragma unroll
          for (int q = 0; q < 64 / kChT; q++)
            D[u * (64 / kChT) + q] += __popcll(bal & (((1ull << kChT) - 1) << (q * kChT))) << b;
        }
      }
    }
    if constexpr (kChT >= 64) {  // + the chain's earlier loads of the stage
      constexpr int kPer = kChT / 64;
#pragma unroll
      for (int u = 0; u < kLd; u++) {
#pragma unroll
        for (int v = u - u % kPer; v < u; v++) pre[u] += (uint32_t)T[v];
        D[u / kPer] += T[u];
      }
    }
    int maxD = 0, myD = 0;
#pragma unroll
    for (int j = 0; j < kChC; j++) {
      maxD = max(maxD, D[j]);
      myD = lane == j ? D[j] : myD;
    }
    cnt += (uint32_t)myD;  // count += 1.0 per draw (an integer sum: order-free)
    for (int wnd = 0; wnd < maxD; wnd += kDcap) {
#pragma unroll
      for (int u = 0; u < kLd; u++) {
        const int p = (int)pre[u] - wnd;
        const int k1 = min((int)cc[u], kDcap - p);
        double2 v;
        v.x = w[u];
        v.y = wy[u];
        for (int k = max(0, -p); k < k1; k++) s_d[uj[u] * kDp + p + k] = v;
      }
      block_sync();
      if (lane < kChC) {
        // this chain's draws of the window, padded to a multiple of 8 with (-0.0, -0.0) by
        // its own lane; 8 draws per step, the next 8 read ahead (the array's 8-entry tail
        // keeps the last chain's over-read inside it)
        const int n = min(max(myD - wnd, 0), kDcap);
        const int n8 = (n + 7) & ~7;
        double2* sd = s_d + lane * kDp;
        double2 z;
        z.x = -0.0;
        z.y = -0.0;
        for (int i = n; i < n8; i++) sd[i] = z;
        double2 a[8];
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = sd[k];
        for (int d = 0; d < n8; d += 8) {
          double2 b[8];
#pragma unroll
          for (int k = 0; k < 8; k++) b[k] = sd[d + 8 + k];
#pragma unroll
          for (int k = 0; k < 8; k++) {
            s1 += a[k].x;
            s2 += a[k].y;
          }
#pragma unroll
          for (int k = 0; k < 8; k++) a[k] = b[k];
        }
      }
      block_sync();
    }
  }
  if (lane < kChC && g < nlanes) {
    double* o = A.chist + g * 3;
    o[0] = (double)cnt;
    o[1] = s1;
    o[2] = s2;
  }
}


// ---------------------------------------------------------------- per-partition sums
// Several partitions (P > 1): RandomForest.findBestSplits aggregates each partition's rows on
// its own (mapPartitions -> binSeqOp: DTStatsAggregator.update, row order within the
// partition, sums from 0.0) and merges the partitions' aggregates per node with
// reduceByKey((a, b) => a.merge(b)), allStats(i) += other.allStats(i).  The merge order is the
// shuffle's; partition order is one order Spark produces (and the only one at P = 1), and the
// oracle restates the same (oracle/sbag_oracle.c fit_one).  So a (task, bin) cell is P
// independent row-order chains plus a P-term merge; a run (task, partition) is a contiguous
// range of the task's entries (a node's entries are in row order, partitions are row ranges).
//
// k_fb_psum: a wave per R runs with R = 64 / 2^nbits clamped to [1, 8] (C3's 32 bins: 2).  A
// step of 512 entries (512 / R per run) is loaded coalesced, ordered by key = (run, bin) in LDS
// (stable: an entry's rank among the step's entries of its key, from ballots over the key's
// bits, as k_fb_scatter orders its buckets), and then lane l adds the entries of its keys l,
// l + 64, ... in row order: a chain per (run, bin), ~512 / 64 entries long per step.  The run
// bounds come from k_fb_runs (one lane per run, two binary searches of the partition's row
// bounds).  The walk is VALU-issue bound, so every lane is kept busy and an entry's draws past
// the first are an exec-masked loop.  (Round 6 measured, per C3 fit: one lane per run, 64 runs
// per wave, 8 entries a stage, all of them walked by the run's lane -- 47.5 ms, the first
// levels' few long runs leaving most SIMDs idle; the same with 2-8 lanes per run splitting the
// bins -- 48 ms; one run per wave, 4 predicated draws per entry -- ~4 ms per level; this
// kernel -- 29 ms.)  k_fb_pmerge then adds the P partials of every (task, bin) in partition
// order.
constexpr int kPwU = 8;  // rounds of 64 entries per step
__global__ __launch_bounds__(256) void k_fb_runs(F64BucketArgs A, int64_t runs) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= runs) return;
  const int64_t task = g / A.P;
  const int q = (int)(g - task * A.P);
  const F64Task t = A.tasks[task];
  auto lower = [&](int64_t row) {  // first entry of the task with a row >= row
    int64_t a = t.a, b = t.b;
    while (a < b) {
      const int64_t mid = (a + b) >> 1;
      if ((int64_t)(uint32_t)A.ent_in[mid] < row)
        a = mid + 1;
      else
        b = mid;
    }
    return a;
  };
  const int64_t lo = lower(A.poff[q]);
  A.prun[2 * g] = lo;
  A.prun[2 * g + 1] = lower(A.poff[q + 1]) - lo;
}

template <int R, bool kCarried>
__global__ __launch_bounds__(256) void k_fb_psum(F64BucketArgs A, int64_t runs, int nbits) {
  constexpr int kRu = kPwU / R;  // rounds per run per step
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t g0 = ((int64_t)blockIdx.x * 4 + wv) * R;  // the wave's first run
  __shared__ uint32_t s_cnt[4][256], s_off[4][256];
  constexpr int kKeys = R == 1 ? 256 : 64;  // keys at most (R = 1: up to 256 bins)
  __shared__ uint64_t s_eq[4][kKeys + 1];     // per key: the round's lanes of that key (+ invalid)
  // key k's entries at soff[k] + k + rank: one slot of padding per key, so the walk's lanes
  // (reading soff[l] + l + j, ~8 entries per key apart) spread over the LDS banks
  __shared__ double s_y[4][64 * kPwU + kKeys];
  __shared__ uint8_t s_c[4][64 * kPwU + kKeys];
  if (g0 >= runs) return;  // whole waves only; no block-wide barrier below
  const int NB = A.NB;
  const int nkey = R << nbits;  // keys (run r, bin b) = r 2^nbits + b
  // per run (wave-uniform): its entries' bins and labels from 32-bit offsets (a run < 2^31)
  const uint16_t* rb[R];
  const double* ry[R];
  const uint64_t* re[R];
  int32_t len[R], lm1[R];
  int32_t steps = 0;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int64_t g = g0 + r;
    int64_t lo = 0, n = 0, eb = 0;
    if (g < runs) {
      const int64_t task = g / A.P;
      lo = A.prun[2 * g];
      n = A.prun[2 * g + 1];
      eb = A.tasks[task].ebase - A.tasks[task].a;
    }
    rb[r] = A.ebin + eb + lo;
    ry[r] = kCarried ? A.ey_in + lo : nullptr;
    re[r] = A.ent_in + lo;
    len[r] = (int32_t)n;
    lm1[r] = max((int32_t)n - 1, 0);
    steps = max(steps, (int32_t)((n + 64 * kRu - 1) / (64 * kRu)));
  }
  uint32_t* scnt = s_cnt[wv];
  uint32_t* soff = s_off[wv];
  uint64_t* seq = s_eq[wv];
  double* sy = s_y[wv];
  uint8_t* sc = s_c[wv];
  for (int b = lane; b < 256; b += 64) scnt[b] = 0u;
  double2 acc[4];
#pragma unroll
  for (int k = 0; k < 4; k++) acc[k] = make_double2(0.0, 0.0);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint64_t me = 1ull << lane;
  __builtin_amdgcn_wave_barrier();
  for (int32_t st = 0; st < steps; st++) {
    uint32_t kv[kPwU], rs[kPwU];
    double yv[kPwU];
    // round u: run u / kRu, its entry st 64 kRu + 64 (u % kRu) + lane (loads at clamped
    // offsets, unconditional: one memory latency per step)
#pragma unroll
    for (int u = 0; u < kPwU; u++) {
      const int r = u / kRu;
      const int32_t i = min(st * 64 * kRu + 64 * (u % kRu) + lane, lm1[r]);
      kv[u] = (uint32_t)rb[r][i];
      if constexpr (kCarried)
        yv[u] = ry[r][i];
      else
        yv[u] = A.y[(uint32_t)re[r][i]];
    }
    // ranks: the round's lanes of each key by an atomic OR of the lane bits into the key's
    // mask (the OR's result does not depend on the lanes' order), then the lanes before this
    // one in that mask
#pragma unroll
    for (int u = 0; u < kPwU; u++) {
      const int r = u / kRu;
      const bool valid = st * 64 * kRu + 64 * (u % kRu) + lane < len[r];
      const uint32_t key = valid ? ((uint32_t)r << nbits | (kv[u] & 0xffu)) : (uint32_t)kKeys;
      seq[key] = 0ull;
      __hip_atomic_fetch_or(&seq[key], me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      const uint64_t eq = seq[key];
      const int rank = __popcll(eq & lt), cnt = __popcll(eq);
      const uint32_t so = valid ? scnt[key] : 0u;
      rs[u] = so + (uint32_t)rank;
      if (valid && rank == cnt - 1) scnt[key] = so + (uint32_t)cnt;
      kv[u] = valid ? (key | (kv[u] >> 8) << 16) : 0xFFFFFFFFu;  // key | count << 16; invalid
    }
    __builtin_amdgcn_wave_barrier();
    // step offsets per key (exclusive scan, 4 keys per lane)
    uint32_t c4[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      c4[k] = scnt[4 * lane + k];
      sum += c4[k];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    uint32_t run = incl - sum;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      soff[4 * lane + k] = run + 4 * lane + k;  // (+ key: the padding)
      run += c4[k];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < kPwU; u++) {
      if (kv[u] != 0xFFFFFFFFu) {
        const uint32_t slot = soff[kv[u] & 0xffffu] + rs[u];
        sy[slot] = yv[u];
        sc[slot] = (uint8_t)(kv[u] >> 16);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // lane l: keys l + 64 k, each one chain in row order; an entry's draws past the first in
    // an exec-masked loop (every entry of a key is drawn: c >= 1)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (64 * k >= nkey) break;  // (uniform)
      const int key = lane + 64 * k;
      const uint32_t n = key < nkey ? scnt[key] : 0u, o = key < nkey ? soff[key] : 0u;
      double2 v = acc[k];
      for (uint32_t j = 0; j < n; j++) {
        const double w = 1.0 * sy[o + j];  // instanceWeight * label
        const double wy = w * sy[o + j];   // instanceWeight * label * label
        const uint32_t c = sc[o + j];
        v.x += w;
        v.y += wy;
        for (uint32_t d = 1; d < c; d++) {
          v.x += w;
          v.y += wy;
        }
      }
      acc[k] = v;
    }
    __builtin_amdgcn_wave_barrier();
    // the counts restart (after every lane's walk read them: in-order LDS operations)
#pragma unroll
    for (int k = 0; k < 4; k++) scnt[4 * lane + k] = 0u;
    __builtin_amdgcn_wave_barrier();
  }
  // lane l's keys: run (l + 64 k) >> nbits of the wave, bin (l + 64 k) & (2^nbits - 1)
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int key = lane + 64 * k;
    const int r = key >> nbits, b = key & ((1 << nbits) - 1);
    if (key < nkey && b < NB && g0 + r < runs) ((double2*)A.ppart)[(size_t)(g0 + r) * NB + b] = acc[k];
  }
}

// the partitions' partials of every (task, bin), added in partition order from 0.0 (the first
// partial is then itself: no sum is ever -0.0); the count is the (task, bin) cell of the
// level's integer histogram -- Spark's count += 1.0 per draw is the exact integer number of
// draws, which the integer engine counted (the node total for a task without a feature)
__global__ __launch_bounds__(256) void k_fb_pmerge(F64BucketArgs A, int nchain) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int NB = A.NB, P = A.P;
  if (i >= (int64_t)nchain * NB) return;
  const int64_t task = i / NB;
  const int b = (int)(i - task * NB);
  const double2* p = (const double2*)A.ppart + (size_t)task * P * NB + b;
  double s1 = 0.0, s2 = 0.0;
  for (int q = 0; q < P; q++) {
    const double2 v = p[(size_t)q * NB];
    s1 += v.x;
    s2 += v.y;
  }
  const F64Task t = A.tasks[task];
  const uint64_t* h = A.hist + ((size_t)t.slot * A.Fmax + (t.fl >= 0 ? t.fl : 0)) * NB * 3;
  uint64_t cnt = 0;
  if (t.a == t.b)
    cnt = 0;
  else if (t.fl >= 0)
    cnt = h[(size_t)b * 3];
  else if (b == 0)  // the node total: every entry in bin 0
    for (int k = 0; k < NB; k++) cnt += h[(size_t)k * 3];
  double* o = A.chist + (size_t)i * 3;
  o[0] = (double)cnt;
  o[1] = s1;
  o[2] = s2;
}

// the partials, then the run bounds (entry offset, length) k_fb_runs finds for k_fb_psum
size_t fb_psum_part_bytes(int64_t nchain, int P, int NB) { return (size_t)nchain * P * (NB + 1) * 2 * sizeof(double); }

// ---------------------------------------------------------------- label column
// analyze_labels (sbag_host.cpp) on the device: per label, finite / integral and the
// smallest s with y 2^s integral (from the exponent and the significand's trailing zeros),
// the range and the largest |y|; wave reductions, then one atomic per wave and quantity
__device__ __forceinline__ uint64_t dkey(double v) {  // order-preserving key of a double
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__global__ __launch_bounds__(256) void k_label_stats(const double* __restrict__ y, int64_t N,
                                                     uint64_t* __restrict__ acc) {
  uint32_t nf = 0, ni = 0;
  int smax = 0;
  uint64_t kmin = ~0ull, kmax = 0, amax = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256) {
    const double v = y[i];
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    const int E = (int)((bits >> 52) & 0x7FF);
    if (E == 0x7FF) {  // NaN / inf
      nf = 1;
      ni = 1;
      continue;
    }
    int si = 0;
    if (v != 0.0) {
      const uint64_t M = bits & ((1ull << 52) - 1);
      const uint64_t sig = E ? (M | (1ull << 52)) : M;
      const int low = (E ? E - 1075 : -1074) + (int)__builtin_ctzll(sig);  // v = odd 2^low
      si = low < 0 ? -low : 0;
    }
    smax = max(smax, si);
    if (!(v >= 0 && si == 0 && v < 8388608.0)) ni = 1;
    const uint64_t k = dkey(v);
    kmin = min(kmin, k);
    kmax = max(kmax, k);
    amax = max(amax, bits & 0x7FFFFFFFFFFFFFFFull);  // |v|: its bits order as the value
  }
  for (int o = 32; o > 0; o >>= 1) {
    nf |= (uint32_t)__shfl_xor((int)nf, o);
    ni |= (uint32_t)__shfl_xor((int)ni, o);
    smax = max(smax, __shfl_xor(smax, o));
    kmin = min(kmin, (uint64_t)__shfl_xor((long long)kmin, o));
    kmax = max(kmax, (uint64_t)__shfl_xor((long long)kmax, o));
    amax = max(amax, (uint64_t)__shfl_xor((long long)amax, o));
  }
  if ((threadIdx.x & 63) == 0) {
    if (nf) atomicOr((unsigned long long*)&acc[0], 1ull);
    if (ni) atomicOr((unsigned long long*)&acc[1], 1ull);
    atomicMax((unsigned long long*)&acc[2], (unsigned long long)smax);
    atomicMin((unsigned long long*)&acc[3], (unsigned long long)kmin);
    atomicMax((unsigned long long*)&acc[4], (unsigned long long)kmax);
    atomicMax((unsigned long long*)&acc[5], (unsigned long long)amax);
  }
}

void launch_label_stats(hipStream_t st, const double* y, int64_t N, uint64_t* acc) {
  const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((N + 255) / 256, 2048));
  hipLaunchKernelGGL(k_label_stats, dim3(bx), dim3(256), 0, st, y, N, acc);
}

__global__ __launch_bounds__(256) void k_label_image(const double* __restrict__ y, int64_t N,
                                                     int shift, int dyadic, int32_t* __restrict__ k) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256) {
    const double v = ldexp(y[i], shift);
    k[i] = (int32_t)(dyadic ? v : rint(v));
  }
}

void launch_label_image(hipStream_t st, const double* y, int64_t N, int shift, bool dyadic, int32_t* k) {
  const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((N + 255) / 256, 4096));
  hipLaunchKernelGGL(k_label_image, dim3(bx), dim3(256), 0, st, y, N, shift, dyadic ? 1 : 0, k);
}

void launch_fb_route(hipStream_t st, const F64BucketArgs& a, int64_t npieces, int nchain) {
  int nbits = 0;
  while ((1 << nbits) < a.NB) nbits++;
  if (npieces > 0)
    hipLaunchKernelGGL(k_fb_count, dim3((unsigned)npieces), dim3(256), 0, st, a);
  if (a.ntasks > 0)  // (tasks without pieces still get their bucket bounds)
    hipLaunchKernelGGL(k_fb_scan, dim3((unsigned)a.ntasks), dim3(256), 0, st, a);
  if (npieces > 0 && (a.route || !a.psum)) {
    const dim3 g((unsigned)((npieces + 3) / 4));
    if (a.wide)
      hipLaunchKernelGGL(k_fb_scatter<true>, g, dim3(256), 0, st, a, npieces, nbits);
    else
      hipLaunchKernelGGL(k_fb_scatter<false>, g, dim3(256), 0, st, a, npieces, nbits);
  }
  if (nchain <= 0) return;
  if (a.psum) {  // P > 1: per-partition runs of each chain task, then the merge in partition order
    const int64_t runs = (int64_t)nchain * a.P;
    hipLaunchKernelGGL(k_fb_runs, dim3((unsigned)((runs + 255) / 256)), dim3(256), 0, st, a, runs);
    const int R = nbits >= 6 ? 1 : nbits == 5 ? 2 : nbits == 4 ? 4 : 8;  // runs per wave
    const dim3 g((unsigned)((runs + 4 * R - 1) / (4 * R)));
    const bool cy = a.ey_in != nullptr;
#define SBAG_PSUMW(r)                                                                  \
  if (cy)                                                                              \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fb_psum<r, true>), g, dim3(256), 0, st, a, runs, nbits); \
  else                                                                                 \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fb_psum<r, false>), g, dim3(256), 0, st, a, runs, nbits)
    if (R == 1)
      SBAG_PSUMW(1);
    else if (R == 2)
      SBAG_PSUMW(2);
    else if (R == 4)
      SBAG_PSUMW(4);
    else
      SBAG_PSUMW(8);
#undef SBAG_PSUMW
    const int64_t cells = (int64_t)nchain * a.NB;
    hipLaunchKernelGGL(k_fb_pmerge, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, st, a, nchain);
    return;
  }
  // one partition: the buckets' chains.  The serial lanes are latency-bound, so a wave takes
  // as few chains as keep >= 2048 waves (two per SIMD: the VGPR budget's occupancy) -- C3
  // shape, serialized fit, ms: 16 everywhere 331, by this rule 305 (root 37 instead of 51); a
  // booster's few chains get a wave each (GBM 10M x 100: chains 71 -> 16 ms per booster)
  const int64_t lanes = (int64_t)nchain * a.NB;
  const int cw = lanes >= 16 * 2048 ? 16 : lanes >= 4 * 2048 ? 4 : 1;
  if (cw == 16)
    hipLaunchKernelGGL(k_fb_chainx<16>, dim3((unsigned)((lanes + 15) / 16)), dim3(64), 0, st, a, nchain);
  else if (cw == 4)
    hipLaunchKernelGGL(k_fb_chainx<4>, dim3((unsigned)((lanes + 3) / 4)), dim3(64), 0, st, a, nchain);
  else
    hipLaunchKernelGGL(k_fb_chainx<1>, dim3((unsigned)lanes), dim3(64), 0, st, a, nchain);
}

// ---------------------------------------------------------------- finish
// RandomForest.binsToBestSplit on the chosen feature's exact bins, in Spark's operation order
// (as k_f64_split): the parent stats chained from the node (or, at the root, the first
// feature with splits: its first candidate's left + right), the prefixes in bin order,
// right = total - left, the first max over the feature's splits.
__global__ __launch_bounds__(64) void k_fb_finish(F64FinishArgs A) {
  const int q = blockIdx.x * 64 + threadIdx.x;
  if (q >= A.n) return;
  const F64FinishNode nd = A.nodes[q];
  const int NB = A.NB;
  double pc0 = nd.ch.calc[0], pc1 = nd.ch.calc[1], pc2 = nd.ch.calc[2], pimp = nd.ch.impurity;
  if (!nd.ch.set) {
    const double* fa = A.chist + (int64_t)nd.t0 * NB * 3;
    double t0 = 0, t1 = 0, t2 = 0;
    for (int s = 0; s <= nd.nsp0; s++) {
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
    pimp = var_imp(pc0, pc1, pc2);
  }
  const double* fa = A.chist + (int64_t)nd.t * NB * 3;
  const int nsp = nd.nsp;
  double t0 = fa[0], t1 = fa[1], t2 = fa[2];
  for (int s = 1; s <= nsp; s++) {
    t0 += fa[3 * s];
    t1 += fa[3 * s + 1];
    t2 += fa[3 * s + 2];
  }
  double c0 = 0, c1 = 0, c2 = 0, fg = 0.0, bl[3] = {0, 0, 0};
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
      gain = kMinValueS;
      valid = 0;
    } else {
      const int64_t total = lc + rc;
      const double li = var_imp(c0, c1, c2), ri = var_imp(r0, r1, r2);
      const double lw = (double)lc / (double)total, rw = (double)rc / (double)total;
      gain = pimp - lw * li - rw * ri;
      valid = 1;
      if (gain < A.min_gain) {
        gain = kMinValueS;
        valid = 0;
      }
    }
    if (fs < 0 || gain > fg) {
      fg = gain;
      fs = s;
      fv = valid;
      bl[0] = c0;
      bl[1] = c1;
      bl[2] = c2;
    }
  }
  F64SplitOut o{};
  o.f = nd.f;
  o.s = fs;
  o.gain = fg;
  o.impurity = pimp;
  o.valid = fv;
  o.calc[0] = pc0;
  o.calc[1] = pc1;
  o.calc[2] = pc2;
  for (int k = 0; k < 3; k++) o.left[k] = bl[k];
  o.right[0] = t0 - bl[0];
  o.right[1] = t1 - bl[1];
  o.right[2] = t2 - bl[2];
  A.out[q] = o;
}

void launch_fb_finish(hipStream_t st, const F64FinishArgs& a) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(k_fb_finish, dim3((unsigned)((a.n + 63) / 64)), dim3(64), 0, st, a);
}

}  // namespace sbag
