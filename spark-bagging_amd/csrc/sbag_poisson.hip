// sbag_poisson.hip — k_poisson4: the Poisson bag sampler of sql/catalyst/expressions/
// Poisson.scala:53-56,73 (one commons-math3 PoissonDistribution per (learner, partition),
// reseeded with seed + i + partitionIndex; one nextPoisson() per row).
//
// A stream is a Well19937c generator (624-word ring in LDS) parsed into counts by
// PoissonDistribution.nextPoisson (mean < 40: multiply nextDouble()s until the product
// drops below exp(-mean)).  Like k_poisson3 (sbag_kernels.hip) a batch of 64 steps of one
// stream runs on LANES lanes, SPL = 64 / LANES consecutive steps each (sbag_well.h has the
// algebra): the lanes read their steps' ring words, fold their c terms into one
// L^SPL-affine transfer, scan it across the stream's lanes with DPP, replay their steps,
// and parse their SPL / 2 doubles by relaxation.  Differences from k_poisson3:
//
//  * 8 lanes per stream by default (LANES = 16 kept for A/B): the scan has 3 rounds
//    instead of 4 for 64 steps, and with 4 doubles per lane the relaxation parse settles
//    in ~3.1 rounds instead of ~4.7 (a stream's lanes rarely run 4 doubles without a row
//    end), so the generator and the parse issue ~40 % fewer VALU per step;
//  * conflict-free ring reads: a stream's pitch is 626 words (= 2 mod 8), every window is
//    read with 8-byte ds_read_b64 at a compile-time parity (the batch start i is a
//    multiple of 16), and the 8 (16) lanes of a stream read 8 (4) words apart, so the 4 (2)
//    streams of a 32-lane group cover disjoint bank residues (k_poisson3's 4-word stride
//    with read2_b32 put lanes t and t+8 on one bank: 52 % of its LDS cycles were
//    conflicts);
//  * the next batch's ring reads are issued before the current batch's parse, so the parse
//    (fp64 multiplies, DPP, a wave-wide vote per round) hides their latency;
//  * the hb / lo windows (top bit of v[j-1], low bits of v[j-2]) are one window.
//
// Exactness: the same arithmetic as k_poisson3 / the oracle (oracle/sbag_oracle.c
// well_next / poisson_next): bit-exact bags, checked by tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "sbag_internal.h"
#include "sbag_well.h"

namespace sbag {

namespace {

constexpr int kP4Streams = 16;  // streams per block: 16 x 626 words = 40 KB, 4 blocks per CU
constexpr int kP4Pitch = 626;   // = 2 mod 8: the streams of a 32-lane group on disjoint banks
constexpr int kP4B = 64;        // steps per batch (<= 69: every read precedes the batch)

// bit m: a batch starting at ring index 16m reads every window without wrapping round
// the ring end.  The lane windows of offset `off` lie in [wrap(16m + off) - 65,
// wrap(16m + off) + 1] (the aligned 8-byte reads start up to 2 words early and end up to
// one word late, inside the 626-word pitch); off = 623 is the joint hb / lo window.
constexpr uint64_t p4_fast_mask() {
  uint64_t m = 0;
  const int offs[4] = {70, 179, 449, 623};
  for (int k = 0; k < 39; k++) {
    bool fast = true;
    for (int w = 0; w < 4; w++) {
      int x = 16 * k + offs[w];
      x = x >= 624 ? x - 624 : x;
      fast = fast && x >= 65;
    }
    if (fast) m |= 1ull << k;
  }
  return m;
}

// lanes t - s of the stream (t >= s), else 0: DPP row_shr within 16-lane rows; a stream of
// 8 (4) lanes masks the lanes that would read the previous stream's
template <int LANES, int S>
__device__ __forceinline__ uint32_t shr_in_stream(uint32_t x, int t) {
  const uint32_t y = wellsp::dpp<0x110 + S>(x);
  if constexpr (LANES >= 16)
    return y;
  else
    return t >= S ? y : 0u;
}

// the value of the stream's last lane, valid at lane 0 of the stream
template <int LANES>
__device__ __forceinline__ uint32_t last_to_first(uint32_t x) {
  if constexpr (LANES == 16)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x121, 0xF, 0xF, false);  // row_ror:1
  else if constexpr (LANES == 8)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  else
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x93, 0xF, 0xF, false);  // quad_perm [3,0,1,2]
}

// sum over the stream's lanes, in every lane (butterfly of DPP adds)
template <int LANES>
__device__ __forceinline__ int stream_sum(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  if constexpr (LANES >= 8) x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false);
  if constexpr (LANES >= 16) x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false);
  return x;
}

// NW consecutive ring words from an 8-byte aligned LDS address.  (The compiler pairs
// them into ds_read2_b64, whose 16-lane groups bank mod 32 dwords: with the 8-word lane
// stride lanes t and t+4 share a bank.  Unpaired ds_read_b64 through opaque addresses was
// measured too: conflicts 52 -> 46 % of LDS cycles, the kernel 1 % slower -- the LDS is
// not what paces it)
template <int NW>
__device__ __forceinline__ void lds_words(const uint32_t* __restrict__ p, uint32_t (&w)[NW]) {
  static_assert(NW % 2 == 0, "whole 8-byte reads");
  const uint2* q = (const uint2*)p;
#pragma unroll
  for (int u = 0; u < NW / 2; u++) {
    const uint2 v = q[u];
    w[2 * u] = v.x;
    w[2 * u + 1] = v.y;
  }
}

// The ring words of the lane's SPL steps (step q of the lane sits at ring index
// i - n0 - q): m1 = v[j+70], m2 = v[j+179], m3 = v[j+449], hb = v[j-1], lo = v[j-2].
template <int SPL>
struct P4Words {
  uint32_t m1[SPL], m2[SPL], m3[SPL], hb[SPL], lo[SPL];
};

template <int SPL, bool FAST>
__device__ __forceinline__ void p4_read(const uint32_t* __restrict__ st, int i, int n0,
                                        P4Words<SPL>& w) {
  if constexpr (FAST) {
    // i is a multiple of 16, n0 and SPL are even: the parity of every window start is fixed
    const int b70 = wrap624(i + 70), b179 = wrap624(i + 179), b449 = wrap624(i + 449);
    const int bh = wrap624(i + 623);
    {  // [b70 - n0 - SPL + 1, b70 - n0] starts odd: read [b70 - n0 - SPL, b70 - n0 + 1]
      uint32_t x[SPL + 2];
      lds_words<SPL + 2>(st + (b70 - n0 - SPL), x);
#pragma unroll
      for (int q = 0; q < SPL; q++) w.m1[q] = x[SPL - q];
    }
    {
      uint32_t x[SPL];
      lds_words<SPL>(st + (b179 - n0 - SPL + 1), x);
#pragma unroll
      for (int q = 0; q < SPL; q++) w.m2[q] = x[SPL - 1 - q];
    }
    {
      uint32_t x[SPL];
      lds_words<SPL>(st + (b449 - n0 - SPL + 1), x);
#pragma unroll
      for (int q = 0; q < SPL; q++) w.m3[q] = x[SPL - 1 - q];
    }
    {  // hb of step q at bh - n0 - q, lo at bh - 1 - n0 - q: one window [bh - n0 - SPL - 1, bh - n0]
      uint32_t x[SPL + 2];
      lds_words<SPL + 2>(st + (bh - n0 - SPL - 1), x);
#pragma unroll
      for (int q = 0; q < SPL; q++) {
        w.hb[q] = x[SPL + 1 - q];
        w.lo[q] = x[SPL - q];
      }
    }
  } else {
    const int b[5] = {wrap624(i + 70), wrap624(i + 179), wrap624(i + 449), wrap624(i + 623),
                      wrap624(i + 622)};
#pragma unroll
    for (int q = 0; q < SPL; q++) {
      int pos[5];
#pragma unroll
      for (int k = 0; k < 5; k++) {
        pos[k] = b[k] - n0 - q;
        pos[k] += pos[k] < 0 ? 624 : 0;
      }
      w.m1[q] = st[pos[0]];
      w.m2[q] = st[pos[1]];
      w.m3[q] = st[pos[2]];
      w.hb[q] = st[pos[3]];
      w.lo[q] = st[pos[4]];
    }
  }
}

template <int LANES, bool CAP>
__global__ __launch_bounds__(kP4Streams* LANES) void k_poisson4(
    uint8_t* __restrict__ counts, int64_t N, const int64_t* __restrict__ part_off, int P, int R,
    int learner0, int64_t seed, double p_exp, int icap, int* err) {
  constexpr int SPL = kP4B / LANES;  // steps per lane
  constexpr int DPL = SPL / 2;       // doubles per lane
  static_assert(LANES == 4 || LANES == 8 || LANES == 16, "a stream is a power-of-two lane group");
  __shared__ __align__(16) uint32_t sm[kP4Streams * kP4Pitch];
  const int t = threadIdx.x & (LANES - 1);
  const int slot = threadIdx.x / LANES;
  uint32_t* st = sm + slot * kP4Pitch;
  const int64_t sid = (int64_t)blockIdx.x * kP4Streams + slot;
  const bool active = sid < (int64_t)R * P;
  const int r = active ? (int)(sid / P) : 0;
  const int p = active ? (int)(sid % P) : 0;
  // PoissonDistribution.reseedRandomGenerator(seed + i + partitionIndex) ->
  // AbstractWell.setSeed(int[]{hi, lo}): v[i] = 1812433253 * (v[i-2] ^ v[i-2] >>> 30) + i,
  // two independent chains (even / odd i) on lanes 0 and 1; the pad words 624, 625 are
  // read (never used) by the aligned windows
  if (t < 2) {
    const uint64_t s64 = (uint64_t)seed + (uint64_t)(int64_t)(learner0 + r) + (uint64_t)(int64_t)p;
    uint32_t x = t == 0 ? (uint32_t)(s64 >> 32) : (uint32_t)s64;
    st[t] = x;
    for (int i = 2 + t; i < 624; i += 2) {
      x = 1812433253u * (x ^ (uint32_t)((int32_t)x >> 30)) + (uint32_t)i;
      st[i] = x;
    }
    st[624 + t] = 0u;
  }
  block_sync();
  int64_t row = active ? part_off[p] : 0;
  const int64_t row_end = active ? part_off[p + 1] : 0;
  uint8_t* out = counts + (int64_t)r * N;
  uint32_t carry = st[0];  // z4 "before" step 0 is v[0] (used by lane 0 of the stream)
  int i = 0, bad = 0;
  auto out_row = [&](int64_t q, int n) {
    out[q] = (uint8_t)min(n, 255);
    bad |= n > 255 ? 1 : 0;
  };
  const int n0 = SPL * t;
  constexpr uint64_t kFast = p4_fast_mask();
  P4Words<SPL> w;
  p4_read<SPL, (kFast & 1u) != 0>(st, i, n0, w);  // i = 0
  // A batch is "special" when its z3 block [i - 63, i] or the next batch's read windows
  // wrap round the ring end (5 of the 39 batch starts): per-word wrapped addresses then.
  auto special = [&]() {
    return i < kP4B - 1 || !((kFast >> (wrap624(i - kP4B) >> 4)) & 1u);
  };
  // Generator: the batch at ring index i from the words in w -> its doubles x; writes its
  // z3 block, moves i on and issues the next batch's ring reads (this wave wrote the words
  // they depend on; a stream's lanes share the wave).
  auto gen = [&](auto sp, double (&x)[DPL]) {
    constexpr bool SP = decltype(sp)::value;
    uint32_t az[SPL], c[SPL];
#pragma unroll
    for (int q = 0; q < SPL; q++) {
      const uint32_t a = w.m1[q] ^ (w.m1[q] >> 27);
      const uint32_t z2 = wellsp::xor3(w.m2[q] >> 9, w.m3[q], w.m3[q] >> 1);
      const uint32_t z0 = (w.hb[q] & 0x80000000u) | (w.lo[q] & 0x7FFFFFFFu);
      c[q] = wellsp::xor3(wellsp::xor3(a << 9, a >> 21, z0), z2 << 21, z2 >> 21);
      az[q] = a ^ z2;
    }
    // lane transfer: z4 after the lane's last step = L^SPL(z4 before) ^ C; then the
    // inclusive scan over the stream's lanes
    uint32_t C = c[0];
#pragma unroll
    for (int q = 1; q < SPL; q++) C = wellsp::L1x(C, c[q]);
    C = t == 0 ? wellsp::lpowx<SPL>(carry, C) : C;
    C = wellsp::lpowx<SPL>(shr_in_stream<LANES, 1>(C, t), C);
    C = wellsp::lpowx<2 * SPL>(shr_in_stream<LANES, 2>(C, t), C);
    if constexpr (LANES >= 8) C = wellsp::lpowx<4 * SPL>(shr_in_stream<LANES, 4>(C, t), C);
    if constexpr (LANES >= 16) C = wellsp::lpowx<8 * SPL>(shr_in_stream<LANES, 8>(C, t), C);
    uint32_t y;
    if constexpr (LANES == 16) {
      const uint32_t prevC = last_to_first<16>(C);  // row_ror:1: lane t-1, lane 0 gets lane 15
      y = t == 0 ? carry : prevC;
      carry = prevC;
    } else {
      const uint32_t prevC = wellsp::dpp<0x111>(C);  // lane t-1 (lane 0 takes the carry)
      y = t == 0 ? carry : prevC;
      carry = last_to_first<LANES>(C);
    }
    // replay: z3 = z4' ^ z4'<<25 ^ a ^ z2 (z4' = z4 of the step before), z4, tempered z4
    uint32_t o[SPL], z3[SPL];
#pragma unroll
    for (int q = 0; q < SPL; q++) {
      z3[q] = wellsp::xor3(y, y << 25, az[q]);
      y = wellsp::L1x(y, c[q]);
      o[q] = wellsp::temper_raw(y);
    }
    if constexpr (!SP) {  // the written block [i - 63, i] does not wrap
      uint32_t* pw = st + (i - n0 - (SPL - 1));
#pragma unroll
      for (int q = 0; q < SPL; q++) pw[SPL - 1 - q] = z3[q];
    } else {
#pragma unroll
      for (int q = 0; q < SPL; q++) {
        int pos = i - n0 - q;
        pos += pos < 0 ? 624 : 0;
        st[pos] = z3[q];
      }
    }
    i = wrap624(i - kP4B);
    p4_read<SPL, !SP>(st, i, n0, w);
    // BitsStreamGenerator.nextDouble = (next(26) << 26 | next(26)) * 2^-52, built exactly
    // as the bits of 1 + m * 2^-52 minus 1 (o = tempered z4; next(26) = o >> 6)
#pragma unroll
    for (int k = 0; k < DPL; k++) {
      const uint32_t hi = o[2 * k], lo = o[2 * k + 1];
      // next(26) << 26 | next(26): the low word is (hi >> 6) << 26 | lo >> 6
      x[k] = __hiloint2double((int)(0x3FF00000u | (hi >> 12)),
                              (int)(((hi << 20) & 0xFC000000u) | (lo >> 6))) - 1.0;
    }
  };
  // PoissonDistribution.nextPoisson (mean < 40) by relaxation: a lane's doubles map an
  // in-state (the open row's product and count) to an out-state; every lane re-evaluates
  // from its left neighbour's out-state (lane 0: the carry) until no in-state changes.  The
  // fixed point is unique and equals the sequential parse (k_poisson3's argument).  One
  // round: in-state -> ends, counts, out-state, and the in-state the left neighbour's
  // out-state gives for the next round (lane 0 of a stream keeps its carry in-state).
  struct Parse {
    double r;
    int n;
  };
  int nk[DPL];
  uint32_t emask = 0u;
  Parse pout{1.0, 0};  // the last round's out-state
  auto round = [&](const double (&x)[DPL], Parse in) {
    double r_ = in.r;
    int n_ = in.n;
    emask = 0u;
#pragma unroll
    for (int k = 0; k < DPL; k++) {
      // r *= nextDouble(); r >= p: n++ (and, capped, return n once n reaches the cap);
      // else return n
      const double rr = r_ * x[k];
      const bool ge = rr >= p_exp;
      const int n1 = n_ + 1;
      const bool e = CAP ? (!ge || n1 >= icap) : !ge;
      nk[k] = CAP ? (ge ? n1 : n_) : n_;
      emask |= e ? (1u << k) : 0u;
      r_ = e ? 1.0 : rr;
      n_ = e ? 0 : n1;
    }
    pout = Parse{r_, n_};
    const int ph = (int)wellsp::dpp<0x111>((uint32_t)__double2hiint(r_));
    const int pl = (int)wellsp::dpp<0x111>((uint32_t)__double2loint(r_));
    const int pnn = (int)wellsp::dpp<0x111>((uint32_t)n_);
    return t != 0 ? Parse{__hiloint2double(ph, pl), pnn} : in;
  };
  auto differs = [&](Parse a, Parse b) {
    return (int)((__double2hiint(a.r) != __double2hiint(b.r)) |
                 (__double2loint(a.r) != __double2loint(b.r)) | (a.n != b.n));
  };
  Parse carry_in{1.0, 0};  // the open row at the stream's batch boundary (lane 0)
  double xc[DPL];
  if (special())
    gen(std::true_type{}, xc);
  else
    gen(std::false_type{}, xc);
  // Each iteration parses the current batch, stores its counts and generates the next
  // one, whose gen issues the ring reads of the batch after it: they land during the next
  // iteration's parse.  (Interleaving the parse with the next batch's generation in one
  // basic block -- three unconditional relaxation rounds -- measured slower: 12.0 vs
  // 11.8 ms on C3.)
  auto step = [&](auto sp) {
    Parse in = t == 0 ? carry_in : Parse{1.0, 0};
    for (;;) {
      const Parse nx = round(xc, in);
      if (!__any(differs(nx, in))) break;
      in = nx;
    }
    // parse carry: the stream's last lane's out-state to lane 0
    carry_in.r = __hiloint2double((int)last_to_first<LANES>((uint32_t)__double2hiint(pout.r)),
                                  (int)last_to_first<LANES>((uint32_t)__double2loint(pout.r)));
    carry_in.n = (int)last_to_first<LANES>((uint32_t)pout.n);
    // rows of the emitted counts: an exclusive scan of the lanes' end counts
    const int mine = __builtin_popcount(emask);
    int inc = mine;
    inc += (int)shr_in_stream<LANES, 1>((uint32_t)inc, t);
    inc += (int)shr_in_stream<LANES, 2>((uint32_t)inc, t);
    if constexpr (LANES >= 8) inc += (int)shr_in_stream<LANES, 4>((uint32_t)inc, t);
    if constexpr (LANES >= 16) inc += (int)shr_in_stream<LANES, 8>((uint32_t)inc, t);
    const int total = stream_sum<LANES>(mine);
    int rk = inc - mine;
#pragma unroll
    for (int k = 0; k < DPL; k++) {  // one exec mask per store: an end inside the partition
      const int e = (emask >> k) & 1u;
      const int64_t q = row + rk;
      if (e & (q < row_end)) out_row(q, nk[k]);
      rk += e;
    }
    row += total;
    gen(sp, xc);
  };
  while (__any(row < row_end)) {
    if (special())
      step(std::true_type{});
    else
      step(std::false_type{});
  }
  if (bad) atomicOr(err, 1);
}

}  // namespace

// R * P streams, kP4Streams per block.  lanes: lanes per stream (4, 8 or 16); 0 picks by
// the stream count: 8 lanes when the streams fill one round of the device's 64 stream slots
// per CU (C3: 16 384 streams, 12.6 vs 14.5 ms), else 16 (the C4 shard's 8 192 streams leave
// half the slots idle, where 16 lanes per stream cut the chain per stream: 79 vs 117 ms;
// two or more rounds of slots: 12.7 vs 13.9 ms at C3 with P = 256).
void launch_poisson4(hipStream_t st, uint8_t* counts, int64_t N, const int64_t* d_part_off, int P,
                     int R, int learner0, int64_t seed, double p_exp, int icap, bool cap, int lanes,
                     int* d_err) {
  const int64_t streams = (int64_t)R * P;
  const int blocks = (int)((streams + kP4Streams - 1) / kP4Streams);
  if (lanes != 4 && lanes != 8 && lanes != 16) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    const int64_t slots = (int64_t)cus * 4 * kP4Streams;  // 4 blocks per CU (LDS)
    lanes = (streams * 4 > slots * 3 && streams <= slots) ? 8 : 16;
  }
#define SBAG_P4(LN, C)                                                                          \
  hipLaunchKernelGGL((k_poisson4<LN, C>), dim3(blocks), dim3(kP4Streams * LN), 0, st, counts, N, \
                     d_part_off, P, R, learner0, seed, p_exp, icap, d_err)
  if (lanes == 16) {
    if (cap) SBAG_P4(16, true); else SBAG_P4(16, false);
  } else if (lanes == 4) {
    if (cap) SBAG_P4(4, true); else SBAG_P4(4, false);
  } else {
    if (cap) SBAG_P4(8, true); else SBAG_P4(8, false);
  }
#undef SBAG_P4
}

}  // namespace sbag
