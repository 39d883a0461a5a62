// sbag_internal.h — device-side structs and kernel launchers shared by
// sbag_kernels.hip (gfx950 kernels) and sbag_host.cpp (C-ABI orchestration).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sbag {

// Workgroup barrier with the waits spelled out.  gfx950 has the back-off barrier, so the
// compiler leaves the wait for a wave's outstanding LDS operations to the barrier's release
// fence, and on some loop paths that wait was dropped: a wave crossed s_barrier with a
// ds_write in flight and another wave read the old word (k_split_gini's per-wave maxima of
// the previous feature group: nondeterministic splits, found by scripts/fuzz_parity.py).
// block_sync: s_waitcnt lgkmcnt(0) first; block_sync_mem: vmcnt(0) too, for global
// memory written by one thread of the block and read by another after the barrier.
// The immediates are the gfx9 s_waitcnt encoding (other generations lay the fields out
// differently): the build refuses any other device target rather than drop the wait.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "sbag kernels are written for gfx9 (gfx950): block_sync's s_waitcnt encoding"
#endif
__device__ __forceinline__ void block_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt 63 (no wait), expcnt 7, lgkmcnt 0
  __syncthreads();
}
__device__ __forceinline__ void block_sync_mem() {
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt 0, expcnt 7, lgkmcnt 0
  __syncthreads();
}

// Entry of a replica's row list (one per in-bag row): low 32 bits row index,
// high 32 bits (label_fixed << 8) | count.  Replaces the reference's
// explode(array_repeat) replication (sql/bfunctions.scala:42-44) by a weight.
__host__ __device__ inline uint64_t pack_entry(uint32_t row, int32_t k, uint32_t c) {
  return (uint64_t)row | ((uint64_t)(uint32_t)(((uint32_t)k << 8) | (c & 0xffu)) << 32);
}

struct HistChunk {  // one workgroup: entries [a, b) of one parent segment
  int32_t parent;
  int32_t excl;      // the whole segment lies in this workgroup's pieces: flush with stores
  int64_t a, b;
  // the histogram kernels' copy of the parent's ParentInfo fields (set by the host, so a
  // piece is one load): replica, histogram slot, class tile, replica's feature count
  int32_t r, slot, tile, fr;
};

struct ParentInfo {  // a node of level d whose rows are routed to level d+1
  int32_t r;          // replica (local index)
  int32_t pos;        // byte position of the split feature in a bins row; -1: no routing
  int32_t s;          // split bin: left iff bin <= s (ContinuousSplit.shouldGoLeft)
  int32_t write_l;    // left child is not a leaf -> its entries are written
  int32_t write_r;
  int32_t hist_slot;  // histogram slot accumulated by this pass, -1 none
  int32_t hist_side;  // 0 = left child, 1 = right child
  int32_t tile;       // grouped gini histograms: class tile of this sub-segment
};

enum { kHistGini = 0, kHistVar = 1, kHistSq = 2 };  // k_hist modes

struct HistArgs {
  const uint8_t* bins;   // [R?][N][S] bins (or value codes in count mode)
  int64_t bins_rstride;  // bytes between replica matrices (0: shared)
  int32_t S;             // row stride in bytes (multiple of 16)
  int32_t Fmax;
  const int16_t* pos;    // [R][Fmax] byte position of local feature fl in a row
  const int32_t* Fr;     // [R]
  const HistChunk* chunks;   // pieces: slices of node segments, in node order
  const int32_t* wg_piece;   // [nwg + 1]: workgroup w walks pieces [wg_piece[w], wg_piece[w+1])
  const ParentInfo* parents; // unused by the histogram kernels (HistChunk carries r/slot/tile)
  const uint64_t* ent_in;
  void* hist;            // [slot][Fmax][NB][NS] u64 (variance) or u32 (gini / counts)
  int32_t NB, NS;
  int32_t K0;            // label offset for the packed LDS word (variance)
  int32_t cshift;        // bit position of the count field in the packed word
  int64_t flush_limit;   // max entries accumulated in LDS between flushes
  int32_t FT, FPH;       // features per tile, LDS pitch
  int32_t count_only;    // gini layout with the label ignored (value counts)
  int32_t CT;            // gini: classes per class tile (LDS holds CT class planes)
  int32_t ntf;           // feature tiles; blockIdx.y = class_tile * ntf + feature_tile
  int32_t rl;            // k_hist_rl (identity byte layout): 1 = 64-bit row addresses, 2 = 32-bit
  int32_t grouped;       // gini: entries grouped by class tile, ParentInfo.tile per segment;
                         // blockIdx.y walks feature tiles only
  int32_t dw;            // k_hist gather width: 1 (byte loads) or 4 (aligned words + extract)
  int32_t hct;           // gini layout class tile: hist[slot][NS / hct][Fmax][NB][hct]
  int32_t rlpd;          // k_hist_rl: rows loaded this many passes ahead (2 or 3)
  int32_t small;         // k_hist: short segments (deep levels): 256-thread workgroups with
                         // 32-entry gather groups (k_hist<.., 256, 32>)
  int32_t ablate;        // diagnostics only (SBAG_HIST_ABLATE, wrong results): 1 skips the
                         // flushes, 2 the LDS zeroing, 4 the row gathers, 8 the LDS atomics
  int32_t pad3_;
};

// Gini histogram cell (f, b, c) of one slot: class-tile-major, so that a class tile's
// flush writes one contiguous block (hct = NS: the plain [f][b][NS] layout)
__host__ __device__ inline int64_t gini_cell(int f, int b, int c, int NB, int Fmax, int hct) {
  const int t = c / hct;
  return (((int64_t)t * Fmax + f) * NB + b) * hct + (c - t * hct);
}

// k_partition: entries of each split node -> left block (from the segment start,
// cursors[2p] grows) and right block (from the segment end, cursors[2p+1] shrinks)
struct PartPiece {  // one dynamically scheduled piece of a parent segment
  int32_t q;         // parent
  int32_t pad;
  int64_t a, b;      // entries [a, b)
};

struct PartRound {   // round k of a column group: order[o0, o0 + m) each give one piece
  int64_t out0;      // first piece of the round in the piece list
  int32_t o0, m;     // parents of the group (longest first) that reach this round
  int64_t off;       // entry offset of the round's pieces inside their parents
};

struct PartArgs {
  const uint8_t* cols;   // column-major bins [R?][C][npad] (k_transpose)
  int64_t cols_rstride;  // bytes between replica copies (0: shared)
  int64_t npad;          // column stride (rows rounded up to 64)
  const uint32_t* planes;   // [ncol][nsp][nw32] side bits (bin > s) of shared bins, or NULL
  int64_t nw32;             // words per plane = ceil(N / 32)
  int32_t nsp;              // planes per column (maxBins - 1)
  int32_t pad2;
  const PartPiece* pieces;  // work order: split-column groups, parents interleaved
  int64_t npieces;
  unsigned long long* counter;  // dynamic piece counter (zeroed before the launch)
  const ParentInfo* parents;    // r, pos (split column), s (split bin), write_l, write_r
  const uint64_t* ent_in;
  uint64_t* ent_out;
  unsigned long long* cursors;
  unsigned long long* sq_left;  // [parents] sum of count*k^2 of the rows going left (or NULL)
};

struct SplitOut {
  double gain;  // Double.MinValue when invalid
  int32_t fl;   // best local feature, -1 when no feature has splits
  int32_t s;    // best split bin
  int32_t valid;
  int32_t pad;  // bit 0: variance screen undecided; bit 1: imp_l / imp_r are set
  double imp_l, imp_r;  // Gini.calculate of the chosen split's children (k_split_gini)
};

struct SplitArgs {
  const void* hist;
  int32_t Fmax, NB, NS;
  const int32_t* slot_r;  // [M] replica of each slot
  const int32_t* Fr;      // [R]
  const int32_t* nbins;   // [R][Fmax]  numSplits + 1
  int32_t min_inst;
  double min_gain;
  double inv_scale, inv_scale2;  // 2^-s, 2^-2s (fixed-point labels)
  SplitOut* out;                  // [M]
  int64_t* stats;                 // [3][M][NS] planes: total, left, right (integers)
  int64_t plane;                  // M * NS
  const int32_t* slot_ids;        // block -> slot (NULL: identity)
  const uint64_t* node_sq;        // screen: [M] exact sum of count*k^2 of each node
  int32_t hct;                    // gini layout class tile (HistArgs.hct)
  int32_t pad;
  // gini: slots whose histogram is the sibling = parent - smaller child, derived while staged
  // (k_subtract fused into the split search): derive[2 slot] = the parent's slot in par_hist,
  // derive[2 slot + 1] = the smaller child's slot in hist (-1: the slot's histogram is built);
  // the derived histogram is written to hist_w for the next level's parents
  const int32_t* derive;
  const void* par_hist;
  void* hist_w;
};

struct DevNode {  // packed tree node for predict
  double value;   // threshold (internal) or prediction (leaf)
  int32_t left;   // -1 for a leaf
  int32_t right;
  int32_t gfeat;  // global feature index (subspace resolved)
  int32_t pad;
};

// Packed tree for the LDS-tiled predict: children adjacent (right = left + 1).
// internal: a = left child, b = (global feature << 17) | (tc + 1), go left iff
//           code <= tc, tc = largest code whose value <= threshold (-1: none)
// leaf:     a = 0x80000000 | leaf index (prediction in the chunk's leaf values)
struct PNode {
  uint32_t a, b;
};

struct PredictChunk {  // consecutive trees whose nodes + leaves fit the LDS budget
  int32_t t0, t1;      // trees [t0, t1)
  int64_t n0, n1;      // packed nodes [n0, n1)
  int64_t l0, l1;      // leaf values [l0, l1)
};

struct PredictArgs {
  const void* codes;   // [N][S] u8 / u16
  int32_t code_bytes, S;
  int64_t N;
  const PNode* nodes;
  const double* leaves;
  const int64_t* tree_node;  // [L] first packed node of each tree
  const int64_t* tree_leaf;  // [L] first leaf value of each tree
  const PredictChunk* chunks;
  int32_t nchunks, L;
  int32_t agg, nclasses;
  int32_t chunk_bytes;       // LDS bytes reserved for one chunk
  int32_t vote_bytes;        // kAggVotes: 1 (u8) or 2 (u16) per vote
  double* out;
  void* votes;               // kAggVotes: [L][N] class ids
};

// aggregation kinds of the predict / aggregate kernels (SBAG_AGG_MEAN / _MODE and the
// device outputs of sbag_predict_dataset_device)
constexpr int kAggMean = 0, kAggMode = 1, kAggSum = 2, kAggVotes = 3;
// mode counters of k_predict / k_aggregate fit in LDS up to this many classes
// (u16 x 256 threads per class, 160 KB)
constexpr int kLdsModeClasses = 320;

// ---- launchers (sbag_kernels.hip) ----
void launch_poisson(hipStream_t st, uint8_t* counts, int64_t N, const int64_t* d_part_off, int P,
                    int R, int learner0, int64_t seed, double mean, double p_exp, int* d_err);
void launch_poisson4(hipStream_t st, uint8_t* counts, int64_t N, const int64_t* d_part_off, int P,
                     int R, int learner0, int64_t seed, double p_exp, int icap, bool cap, int lanes,
                     int* d_err);
void launch_bernoulli(hipStream_t st, uint8_t* counts, int64_t N, const int64_t* d_part_off,
                      const int64_t* d_chunk_pre, int P, int64_t chunks_total, int R,
                      int learner0, int64_t seed, double ratio, const uint64_t* d_jump);
void launch_fill(hipStream_t st, uint8_t* p, uint8_t v, int64_t n);
// 256-byte groups of a counts buffer of `bytes` bytes, padded to whole 8-group chunks
inline int64_t split_sample_groups(int64_t bytes) { return ((bytes + 255) / 256 + 7) / 8 * 8; }
void launch_split_sample(hipStream_t st, const uint8_t* counts, int64_t N, int64_t R,
                         const int64_t* d_part_off, int P, const int32_t* d_reps, int nrep,
                         const uint64_t* d_part_state,
                         const double* d_frac /*[nrep][2]: fraction, log1p(-fraction)*/,
                         uint16_t* d_gsums /*[split_sample_groups(R * N)]*/,
                         uint32_t* d_rows /*[nrep][cap]*/, int64_t cap, uint32_t* d_nrows,
                         bool gap_sampling /* every replica's fraction <= 0.4 */);
void launch_split_sample_vc(hipStream_t st, const uint32_t* d_rows, int64_t cap,
                            const uint32_t* d_nrows, const int32_t* d_reps, int nrep,
                            const void* codes, int code_bytes, int32_t S, const int32_t* d_sub,
                            const int32_t* d_Fr, int32_t Fmax, const int64_t* d_vcoff, uint32_t* vc,
                            int lds_words);
// RandomForest.findSplitsForContinuousFeature on the device for the replicas thresholded on their
// split-finding sample (k_find_splits: a wave per (replica, feature) over its value counts): the
// thresholds thr[r][fl][tc] and their code cuts cut[r][fl][tc] (#{dictionary values <= t}), and
// the threshold count nt[r][fl] (may exceed tc: the caller then falls back to the host)
struct SplitFindArgs {
  const uint32_t* cnt;     // value counts, the (replica, feature)'s at vcoff[r * Fmax + fl]
  const int64_t* vcoff;    // [R * Fmax + 1]
  const double* dict;      // sorted distinct values of every feature, flat
  const int64_t* dict_off; // [F + 1]
  const int32_t* zero_code;  // [F]: the code of 0.0, -1 when absent
  const int32_t* sub;      // [R][Fmax] global feature of a local one
  const int32_t* Fr;       // [R]
  const int32_t* reps;     // [nrep] replicas
  const int64_t* nw;       // [nrep] numExamples (the subbag's weighted size)
  const int64_t* nsamp;    // [nrep] numSamples ((fraction * numExamples).toInt)
  int32_t Fmax, max_bins, tc, nrep;
  int32_t* nt;             // [R * Fmax]
  double* thr;             // [R * Fmax][tc]
  uint32_t* cut;           // [R * Fmax][tc]
};
void launch_find_splits(hipStream_t st, const SplitFindArgs& a);
// launch_bin_cuts over the in-bag rows only, by rank: out[r][rank][fl], cols[r][fl][rank] for the
// ranks < inbag[r] of the replica's row-ordered entries ent[r][.] (capb >= every inbag[r]); false:
// not supported for this geometry (the caller bins every row)
bool launch_bin_ranked(hipStream_t st, const void* codes, int code_bytes, int32_t S_codes, const uint64_t* ent,
                       int64_t cap, const unsigned long long* d_inbag, int64_t capb, const int32_t* d_sub,
                       const int32_t* d_Fr, int32_t Fmax, int R, const uint32_t* d_cut, int32_t ncp,
                       const uint8_t* d_z0, uint8_t* out, int32_t S_out, int64_t out_rstride, uint8_t* cols,
                       int32_t ncol, int64_t npad, int64_t cols_rstride);
// whether launch_bin_ranked takes this geometry (decided before the bins are sized)
bool bin_ranked_fits(int code_bytes, int32_t S_codes, int32_t S_out, int32_t Fmax, int32_t ncp);
// ent[r][i] row field := i (i < inbag[r])
void launch_rank_entries(hipStream_t st, uint64_t* ent, int64_t cap, const unsigned long long* d_inbag, int R,
                         int64_t capb);
// per-replica bins out[r][n][fl] = #{j : cut[r][fl][j] <= codes[n][sub[r][fl]]} (cut [R][Fmax][ncp]
// ascending, every cut >= 1, padded with ~0u; ncp a power of two) + z0[r][fl] (leading zero cuts
// left out of the table; nullptr: none), zero past F_r; with cols the
// column copy cols[r][fl < ncol][npad] is written by the same pass when the kernel can (returns
// true; else the caller transposes)
bool launch_bin_cuts(hipStream_t st, const void* codes, int code_bytes, int64_t N, int32_t S_codes,
                     const int32_t* d_sub, const int32_t* d_Fr, int32_t Fmax, int R, const uint32_t* d_cut,
                     int32_t ncp, const uint8_t* d_z0, uint8_t* out, int32_t S_out, int64_t out_rstride, uint8_t* cols, int32_t ncol,
                     int64_t npad, int64_t cols_rstride);
void launch_compact(hipStream_t st, const uint8_t* counts, int64_t N, int R, const int32_t* d_labk,
                    uint64_t* ent, int64_t cap, unsigned long long* d_cursor,
                    unsigned long long* d_wsum, unsigned int* d_cmax, unsigned long long* d_sqsum);
void launch_hist(hipStream_t st, const HistArgs& a, int nwg, int ntiles, int mode,
                 size_t lds_bytes);
size_t hist_lds_bytes(int NB, int NS, int FPH, bool gini);
size_t hist_stage_bytes();
size_t hist_rl_lds_bytes(int NB, int CT, int FPH, bool gini);
int hist_rl_lanes();
void launch_partition(hipStream_t st, const PartArgs& a, int nwg);
void launch_planes(hipStream_t st, const uint8_t* cols, int64_t npad, int ncol, int nsp, int64_t nw32,
                   uint32_t* planes);
void launch_part_pieces(hipStream_t st, const PartRound* rounds, int nrounds, int64_t npieces,
                        const int32_t* order, const int64_t* seg, int64_t piece, PartPiece* out);
void launch_transpose(hipStream_t st, const uint8_t* src, int64_t N, int S, int C, uint8_t* dst,
                      int64_t npad, int R, int64_t src_rstride, int64_t dst_rstride);
void launch_split(hipStream_t st, const SplitArgs& a, int M, bool gini);
void launch_split_screen(hipStream_t st, const SplitArgs& a, int M);
void launch_zero_word(hipStream_t st, uint64_t* hist, const int32_t* d_slots, int nslots,
                      int64_t slot_words, int stride, int word);
void launch_zero_slots(hipStream_t st, void* hist, const int32_t* d_slots, int nslots,
                       int64_t u32_words_per_slot);
void launch_subtract(hipStream_t st, void* dst_hist, const void* parent_hist, const int32_t* d_triples,
                     int ntriples, int64_t words_per_slot, bool u32words);
void launch_synth(hipStream_t st, uint8_t* codes, int32_t S, int64_t N, int32_t F, uint64_t seed,
                  int32_t num_classes, int32_t* labk);
void launch_predict(hipStream_t st, const double* X, const void* codes, int code_bytes,
                    const double* dict, const int64_t* dict_off, int64_t N, int32_t F, int32_t S,
                    const DevNode* nodes, const int64_t* tree_off, int L, int agg, int nclasses,
                    double* out, double* per_tree, void* votes, int vote_bytes, uint16_t* gcnt,
                    int64_t gcnt_rows);
// vote_bytes: 8 = fp64 values, 1 / 2 = u8 / u16 class ids
void launch_aggregate(hipStream_t st, const void* votes, int vote_bytes, int K, int64_t N, int agg,
                      int nclasses, double num_learners, double* out, uint16_t* gcnt,
                      int64_t gcnt_rows);
size_t predict_tiled_lds(const PredictArgs& a);
void launch_quantize(hipStream_t st, const double* X, int64_t n, int32_t F, const double* thr,
                     const int64_t* toff, uint16_t* codes, int32_t S);
void launch_predict_tiled(hipStream_t st, const PredictArgs& a);
// class-tile grouping of gini histogram entries (one workgroup per piece)
// the grouping with known (segment, tile) sizes: cursors[q ntc + t] start at the tile's first
// position and advance by atomics; pieces of tile_scatter_known_piece() entries
void launch_tile_scatter_known(hipStream_t st, const HistChunk* pieces, int npieces, const uint64_t* ent,
                               int CT, int ntc, unsigned long long* cursors, uint64_t* ent_out);
int tile_scatter_known_piece();
void launch_tile_count(hipStream_t st, const HistChunk* pieces, int npieces, const uint64_t* ent,
                       int CT, int ntc, uint32_t* counts);
void launch_tile_scatter(hipStream_t st, const HistChunk* pieces, int npieces, const uint64_t* ent,
                         int CT, int ntc, const int64_t* base, uint64_t* ent_out);
void launch_vc_global(hipStream_t st, const void* codes, int code_bytes, int32_t S, const uint64_t* ent,
                      int64_t cap, const unsigned long long* d_inbag, const int32_t* d_sub,
                      const int32_t* d_Fr, int32_t Fmax, int R, const int64_t* d_off, uint32_t* vc);
size_t hist_lds_limit();

// ---- fp64 labels (sbag_f64.hip): bagging regression on labels that are not dyadic,
// Spark's row-order fp64 histogram sums reproduced bit for bit
struct F64Node {      // a node of the level: its entries [a, b) (row order) of replica r
  int64_t a, b;
  int32_t r, pad;
};
struct F64HistArgs {
  const uint64_t* ent;     // entries row | count << 32, row order inside every node
  const F64Node* nodes;    // [A]
  const double* y;         // [N] labels
  const uint8_t* bins;     // [R?][N][S]
  int64_t bins_rstride;
  int32_t S, Fmax;
  const int16_t* pos;      // [R][Fmax] byte of local feature fl in a bins row
  const int32_t* Fr;       // [R]
  int32_t NB, FPW;         // bins; features per wave (<= f64_hist_width; local Fr = total)
  int32_t parts;           // 1, or 2: count + sum and sumSq on separate waves
  uint32_t bins_bytes;     // one replica's bins (N·S) when below 4 GB (buffer loads), else 0
  uint32_t yzero, zero;    // y[yzero] = +0.0 (padding label); zero = 0 (opaque to the compiler)
  double* hist;            // [A][Fmax + 1][NB][3]: count, sum, sumSq
};
struct F64Chain {     // calculateImpurityStats' chain state: the node's stats (set) or none
  double calc[3];
  double impurity;
  int32_t set, pad;
};
struct F64SplitOut {
  double gain, impurity;   // Double.MinValue when invalid; the chain's parent impurity
  double calc[3];          // parent calculator
  double left[3], right[3];
  int32_t f, s, valid, pad;  // f = -1: no feature has splits (calc = the node total)
};
struct F64SplitArgs {
  const double* hist;
  const F64Node* nodes;
  const F64Chain* chain;
  const int32_t* Fr;       // [R]
  const int32_t* nbins;    // [R][Fmax] numSplits + 1
  int32_t Fmax, NB, min_inst, pad;
  double min_gain;
  F64SplitOut* out;
  const uint8_t* fmask;    // [node][Fmax] features to consider (null: all); the others hold
                           // no sums (the screen proved none of their candidates can win)
};
// the stable bootstrap compaction of the fp64 path: in-bag rows per (replica, chunk) and
// per replica (Σ count, max count), then one entry row | (k << 8 | count) << 32 per in-bag
// row, in row order (k: the labels' fixed-point image, labk)
void launch_chunk_draws(hipStream_t st, const uint8_t* counts, int64_t N, int R,
                        uint32_t* d_ncnt /*[R][chunks]*/, unsigned long long* d_wsum,
                        unsigned int* d_cmax);
void launch_compact_ordered(hipStream_t st, const uint8_t* counts, const int32_t* labk, int64_t N,
                            int R, uint64_t* ent, int64_t cap, const uint32_t* d_ncnt,
                            unsigned long long* d_base /*[R][chunks]*/, unsigned long long* d_cursor,
                            const double* y, double* ey /* null, or the carried fp64 labels [R][cap] */);

// ---- screened fp64 engine (sbag_f64s.hip): the split of a node is chosen from the integer
// histograms of the labels' fixed-point image with a rigorous bound on Spark's fp64 gain
// (k_f64_screen); only the chosen feature's bins are summed in Spark's row order
// (k_fb_count / k_fb_scan / k_fb_scatter bucket each node's entries by that feature's
// bin, stable, and route them to the children; k_fb_chain adds every bucket in row
// order); k_fb_finish evaluates the chosen feature exactly as binsToBestSplit does.
struct F64ScreenOut {
  int32_t f, s;      // best local feature / split bin by the screen (-1: none)
  int32_t flag;      // 1: undecided -> exact row-order histogram of every feature
  int32_t pad;
  double gain, margin;  // screened gain of the best candidate, its guaranteed lead
};
struct F64ScreenArgs {
  const uint64_t* hist;     // [slot][Fmax][NB][3] integer (count, Σ c k, -)
  const int32_t* slot_r;    // [M]
  const int32_t* Fr;        // [R]
  const int32_t* nbins;     // [R][Fmax]
  int32_t Fmax, NB, min_inst, pad;
  double min_gain;
  double inv_scale;         // 2^-s: k 2^-s approximates y
  double eps;               // max |y - k 2^-s| (2^-s-1)
  const double* dnode;      // [M] bound on Spark's summation and rounding error of a
                            //     candidate's child part (lw imp(L) + rw imp(R)) of the gain
  const double* dpar;       // [M] bound on the error of the node's own impurity
  F64ScreenOut* out;        // [M]
  uint8_t* cmask;           // [M][Fmax] the feature holds a contender (pass 2)
};
struct F64Task {            // one (node, feature) whose entries are bucketed / routed
  int64_t a, b;             // entries [a, b) of ent_in (row order)
  int64_t kbase;            // buckets at bucket[kbase, kbase + b - a); -1: no buckets
  int64_t piece0, piece1;   // its pieces
  int32_t r, col, s, part;  // replica, column of the column-major bins (-1: every entry in
                            // bin 0, the node total), split bin, route?
  int64_t ebase;            // its entries' bin | count << 8 at ebin[ebase, ebase + b - a) (k_fb_count)
  int32_t slot, fl;         // its node's slot in the level's integer histograms and the local
                            // feature (-1: the node total): k_fb_pmerge takes the draw counts there
};
struct F64TPiece {
  int64_t a, b;
  int32_t task, pad;
};
constexpr int64_t kFbPiece = 8192;
struct F64BucketArgs {
  const uint8_t* cols;      // [R?][C][npad]
  int64_t cols_rstride, npad;
  const F64Task* tasks;
  const F64TPiece* pieces;
  int32_t NB, ntasks;
  const uint64_t* ent_in;
  uint64_t* ent_out;        // children: left [a, a + nleft), right [a + nleft, b), row order
  double* bky;              // the buckets: the node's entries' labels grouped by bin, row
  uint8_t* bkc;             //   order kept, and their draw counts
  uint16_t* ebin;           // every task's entries' bin | draw count << 8, gathered once by k_fb_count
  uint32_t* pcnt;           // [piece][NB] entries per bin
  uint32_t* plcnt;          // [piece] entries going left
  int64_t* pbase;           // [piece][NB] bucket position of the piece's first entry per bin
  int64_t* plbase;          // [piece] left entries of the task before the piece
  int64_t* nleft;           // [task]
  int64_t* kb_off;          // [task][NB + 1] bucket bounds in entK
  const double* y;          // [N] labels
  const double* ey_in;      // the labels of ent_in's entries (same positions)
  double* ey_out;           // the labels of ent_out's entries
  double* chist;            // [task][NB][3] count, sum, sumSq in Spark's row order
  int32_t cmax;             // largest draw count of an entry (1: no count loop)
  int32_t psum;             // P > 1: k_fb_psum sums the chain tasks per partition (no buckets)
  int32_t wide, P;          // >= 2^28 rows: k_fb_scatter addresses by 64-bit pointers; partitions
  const int32_t* porder;    // k_fb_count's piece of each workgroup (null: in order)
  const int64_t* poff;      // [P + 1] the partitions' row offsets (psum)
  double* ppart;            // [chain task][P][NB][2] per-partition partials (psum): sum, sumSq
  const uint64_t* hist;     // (psum) the level's integer histograms [slot][Fmax][NB][3]: the
  int32_t Fmax, pad3;       //   draw counts per (task, bin) (count += 1.0 per draw: exact)
  int64_t* prun;            // [chain task][P][2] the runs' first entry and length (k_fb_psum)
  int32_t route, pad4;      // some task routes its entries to children (else, at P > 1, no
                            // k_fb_scatter: it only routes there -- the last split level)
};
// bytes of k_fb_psum's per-partition partials for nchain tasks
size_t fb_psum_part_bytes(int64_t nchain, int P, int NB);
// A label column's analysis on the device (sbag_fit_booster's residuals): acc[6] =
// {not finite, not integral, largest scale s making a label integral, order key of the
// smallest and of the largest label, bits of the largest |y|}; acc must hold the
// launch_label_stats_init values.  k_label_image: k = y 2^shift (dyadic) or
// rint(y 2^shift) (the fp64 screen's image).
void launch_label_stats(hipStream_t st, const double* y, int64_t N, uint64_t* acc);
void launch_label_image(hipStream_t st, const double* y, int64_t N, int shift, bool dyadic, int32_t* k);
struct F64FinishNode {
  int32_t t, t0;            // task of the chosen feature; task of the first feature with
                            // splits (root: the parent stats), -1 when not needed
  int32_t f, s;             // chosen local feature and split bin
  int32_t nsp, nsp0;        // numSplits of f and of the first feature
  int32_t pad[2];
  F64Chain ch;
};
struct F64FinishArgs {
  const double* chist;
  const F64FinishNode* nodes;
  int32_t n, NB, min_inst, pad;
  double min_gain;
  F64SplitOut* out;
};
// sbag_mfma.hip: the root histogram of shared identity bins as an int8 MFMA contraction
struct MfmaHistArgs {
  const uint8_t* counts;  // [R][N], every count <= 127
  const uint8_t* cols;    // [F][npad] column-major bin codes
  const uint8_t* digits;  // [ND][N] 7-bit digits: planes [0, ND1) of k + K0, then of k^2
  int64_t N, npad;
  int32_t R, F, Fmax, NB, ND1, ND, K0;
  unsigned long long* hist;  // [R][Fmax][NB][3] words: += count, += sum c k, (ND > ND1) += sum c k^2
  int32_t dbits, pad;        // the k planes' digit base: 7 (unsigned digits of k + K0) or 8
                             // (balanced int8 digits of k + K0)
};
bool launch_hist_mfma(hipStream_t st, const MfmaHistArgs& a);
void launch_label_digits(hipStream_t st, const int32_t* labk, int64_t N, int32_t K0, int nd1, int nd2,
                         uint8_t* digits, bool balanced);
void launch_f64_screen(hipStream_t st, const F64ScreenArgs& a, int M);
void launch_fb_route(hipStream_t st, const F64BucketArgs& a, int64_t npieces, int nchain);
void launch_fb_finish(hipStream_t st, const F64FinishArgs& a);
int64_t compact_ordered_chunks(int64_t N);
// in-bag rows per (replica, chunk) only (the entry capacity's pre-count)
void launch_chunk_rows(hipStream_t st, const uint8_t* counts, int64_t N, int R, uint32_t* d_ncnt);
int f64_hist_width(int NB);
size_t f64_hist_lds_bytes(int NB, int parts);
void launch_f64_hist(hipStream_t st, const F64HistArgs& a, int nnodes, int ngroups);
void launch_f64_split(hipStream_t st, const F64SplitArgs& a, int nnodes);
// sbag_dataset_import: *d_bad != 0 when a code is past its dictionary or padding is nonzero
void launch_check_codes(hipStream_t st, const void* codes, int code_bytes, int64_t N, int32_t S,
                        int32_t F, const int64_t* d_dict_off, int* d_bad);

}  // namespace sbag
