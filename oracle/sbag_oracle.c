/*
 * sbag_oracle.c — CPU restatement of the spark-ensemble bagging hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see sbag_oracle.h).  PARITY UNPINNED: no golden
 * vectors exist in the reference; this file is cross-checked against the
 * independent pure-Python restatement oracle/pyoracle.py.
 *
 * Every function cites the reference call site it restates
 * (paths relative to /root/reference/core/src/main/scala/org/apache/spark/)
 * and the upstream algorithm it follows (Spark 2.4.3, commons-math3 3.4.1,
 * scala-library 2.12.8, breeze 0.13.2; restated in SURVEY.md Appendix A).
 * Java integer semantics are reproduced with unsigned arithmetic.
 */
#include "sbag_oracle.h"
#include "or_fastmath.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================================================================
 * scala.util.hashing.MurmurHash3.bytesHash (scala-library 2.12.8) and
 * org.apache.spark.util.random.XORShiftRandom.hashSeed (Spark 2.4.3).
 * Used by ml/ensemble/HasSubBag.scala:97 and by Rand at sql/bfunctions.scala:64.
 * ==================================================================== */
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t mm3_mix_last(uint32_t h, uint32_t k) {
  k *= 0xcc9e2d51u;
  k = rotl32(k, 15);
  k *= 0x1b873593u;
  return h ^ k;
}
static uint32_t mm3_mix(uint32_t h, uint32_t k) {
  h = mm3_mix_last(h, k);
  h = rotl32(h, 13);
  return h * 5u + 0xe6546b64u;
}
static uint32_t mm3_finalize(uint32_t h, uint32_t len) {
  h ^= len;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
static uint32_t mm3_bytes_hash(const uint8_t* d, int len, uint32_t seed) {
  uint32_t h = seed;
  int i = 0, rem = len;
  while (rem >= 4) {
    uint32_t k = (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8) | ((uint32_t)d[i + 2] << 16) |
                 ((uint32_t)d[i + 3] << 24);
    h = mm3_mix(h, k);
    i += 4;
    rem -= 4;
  }
  uint32_t k = 0;
  if (rem == 3) k ^= (uint32_t)d[i + 2] << 16;
  if (rem >= 2) k ^= (uint32_t)d[i + 1] << 8;
  if (rem >= 1) {
    k ^= (uint32_t)d[i];
    h = mm3_mix_last(h, k);
  }
  return mm3_finalize(h, (uint32_t)len);
}

/* Spark 2.4.3 XORShiftRandom.hashSeed:
 *   ByteBuffer.allocate(java.lang.Long.SIZE).putLong(seed).array()
 * Long.SIZE is 64 (bits) but allocate() takes bytes, so the hashed buffer is 64 bytes: the
 * big-endian seed followed by 56 zero bytes (Spark 3.0 changed this to Long.BYTES = 8).
 * Pinned by tests/test_oracle.py: XORShiftRandom(0|30|5419823303878592871).nextDouble()
 * = 0.8446490682263027 | 0.31429268272540556 | 0.2304755080444375 (published 2.x values). */
#define OR_HASH_SEED_BYTES 64
uint64_t or_hash_seed(int64_t seed) {
  uint8_t b[OR_HASH_SEED_BYTES];
  memset(b, 0, sizeof b);
  uint64_t u = (uint64_t)seed;
  for (int i = 0; i < 8; i++) b[i] = (uint8_t)(u >> (56 - 8 * i)); /* ByteBuffer.putLong: big endian */
  uint32_t lo = mm3_bytes_hash(b, OR_HASH_SEED_BYTES, 0x3c074a61u); /* MurmurHash3.arraySeed */
  uint32_t hi = mm3_bytes_hash(b, OR_HASH_SEED_BYTES, lo);
  return ((uint64_t)hi << 32) | (uint64_t)lo;
}

typedef struct {
  uint64_t s;
} xs_t;
static void xs_init(xs_t* r, int64_t seed) { r->s = or_hash_seed(seed); }
/* XORShiftRandom.next(bits): low bits of the new state */
static int32_t xs_next(xs_t* r, int bits) {
  uint64_t s = r->s;
  s ^= s << 21;
  s ^= s >> 35;
  s ^= s << 4;
  r->s = s;
  return (int32_t)(uint32_t)(s & ((bits == 64) ? ~0ULL : ((1ULL << bits) - 1)));
}
/* java.util.Random.nextDouble: ((long)next(26) << 27) + next(27)) * 2^-53 */
static double xs_next_double(xs_t* r) {
  int64_t a = (int64_t)xs_next(r, 26);
  int64_t b = (int64_t)xs_next(r, 27);
  return (double)((a << 27) + b) * 0x1.0p-53;
}

void or_xorshift_next(int64_t seed, int bits, int n, int32_t* out) {
  xs_t r;
  xs_init(&r, seed);
  for (int i = 0; i < n; i++) out[i] = xs_next(&r, bits);
}
void or_xorshift_doubles(int64_t seed, int n, double* out) {
  xs_t r;
  xs_init(&r, seed);
  for (int i = 0; i < n; i++) out[i] = xs_next_double(&r);
}

/* ======================================================================
 * commons-math3 3.4.1 Well19937c (AbstractWell.setSeed(long/int[]),
 * Well19937c.next) + BitsStreamGenerator.nextDouble (52 bits).
 * Used through PoissonDistribution at sql/catalyst/expressions/Poisson.scala:53-56,73.
 * ==================================================================== */
typedef struct {
  uint32_t v[624];
  int index;
} well_t;

static void well_seed(well_t* w, int64_t seed) {
  uint64_t u = (uint64_t)seed;
  w->v[0] = (uint32_t)(u >> 32);
  w->v[1] = (uint32_t)(u & 0xffffffffULL);
  for (int i = 2; i < 624; i++) {
    int64_t l = (int64_t)(int32_t)w->v[i - 2];          /* int -> long sign extension */
    uint64_t t = 1812433253ULL * (uint64_t)(l ^ (l >> 30)) + (uint64_t)i;
    w->v[i] = (uint32_t)(t & 0xffffffffULL);
  }
  w->index = 0;
}

static int32_t well_next(well_t* w, int bits) {
  const int idx = w->index;
  const int iRm1 = (idx + 623) % 624, iRm2 = (idx + 622) % 624;
  const uint32_t v0 = w->v[idx];
  const uint32_t vM1 = w->v[(idx + 70) % 624];
  const uint32_t vM2 = w->v[(idx + 179) % 624];
  const uint32_t vM3 = w->v[(idx + 449) % 624];
  const uint32_t z0 = (0x80000000u & w->v[iRm1]) ^ (0x7FFFFFFFu & w->v[iRm2]);
  const uint32_t z1 = (v0 ^ (v0 << 25)) ^ (vM1 ^ (vM1 >> 27));
  const uint32_t z2 = (vM2 >> 9) ^ (vM3 ^ (vM3 >> 1));
  const uint32_t z3 = z1 ^ z2;
  uint32_t z4 = z0 ^ (z1 ^ (z1 << 9)) ^ (z2 ^ (z2 << 21)) ^ (z3 ^ (z3 >> 21));
  w->v[idx] = z3;
  w->v[iRm1] = z4;
  w->v[iRm2] &= 0x80000000u;
  w->index = iRm1;
  z4 ^= (z4 << 7) & 0xe46e1700u; /* Matsumoto-Kurita tempering */
  z4 ^= (z4 << 15) & 0x9b868000u;
  return (int32_t)(z4 >> (32 - bits));
}

static double well_next_double(well_t* w) {
  const int64_t high = ((int64_t)well_next(w, 26)) << 26;
  const int32_t low = well_next(w, 26);
  return (double)(high | (int64_t)low) * 0x1.0p-52;
}

/* PoissonDistribution.sample() -> nextPoisson(mean) for mean < 40.
   p = FastMath.exp(-mean), restated table for table in or_fastmath.h (FastMath is not
   correctly rounded: at mean 0.052 it is one ulp above libm's exp). */
static int poisson_sample(well_t* w, double mean, double p) {
  int64_t n = 0;
  double r = 1.0;
  while ((double)n < 1000.0 * mean) {
    const double rnd = well_next_double(w);
    r *= rnd;
    if (r >= p) {
      n++;
    } else {
      return (int)n;
    }
  }
  return (int)n;
}

void or_well_next(int64_t seed, int bits, int n, int32_t* out) {
  well_t w;
  well_seed(&w, seed);
  for (int i = 0; i < n; i++) out[i] = well_next(&w, bits);
}
void or_well_doubles(int64_t seed, int n, double* out) {
  well_t w;
  well_seed(&w, seed);
  for (int i = 0; i < n; i++) out[i] = well_next_double(&w);
}
void or_poisson(double lambda, int64_t seed, int n, int32_t* out) {
  well_t w;
  well_seed(&w, seed);
  const double p = or_fm_exp_neg(-lambda);
  for (int i = 0; i < n; i++) out[i] = poisson_sample(&w, lambda, p);
}

/* ======================================================================
 * bfunctions.bag (sql/bfunctions.scala:46-68)
 *   replacement:          Poisson(ratio, seed+i) seeded seed+i+partitionIndex
 *                          (Poisson.scala:53-56)
 *   !replacement, ratio==1: array_repeat(1, L)                       (:56-57)
 *   !replacement:          if(rand(seed+i) < ratio, 1, 0)            (:62-64)
 *                          `seed+i` is spliced into SQL text: Int addition
 *                          (wraps) when seed fits an Int.
 * ==================================================================== */
int or_bag(int replacement, double ratio, int lb, int le, int64_t seed, const int64_t* off, int P,
           int64_t N, uint8_t* counts) {
  if (!(ratio > 0)) return -1; /* require(sampleRatio > 0) */
  if (!replacement && ratio > 1) return -1;
  if (replacement && ratio >= 40.0) return -2; /* large-mean Poisson branch not restated */
  if (off[0] != 0 || off[P] != N) return -3;
  const double p = replacement ? or_fm_exp_neg(-ratio) : 0.0;
  for (int i = lb; i < le; i++) {
    uint8_t* c = counts + (int64_t)(i - lb) * N;
    for (int part = 0; part < P; part++) {
      const int64_t r0 = off[part], r1 = off[part + 1];
      if (replacement) {
        well_t w;
        well_seed(&w, (int64_t)((uint64_t)seed + (uint64_t)(int64_t)i + (uint64_t)(int64_t)part));
        for (int64_t r = r0; r < r1; r++) {
          int k = poisson_sample(&w, ratio, p);
          if (k > 255) return -4;
          c[r] = (uint8_t)k;
        }
      } else if (ratio == 1.0) {
        for (int64_t r = r0; r < r1; r++) c[r] = 1;
      } else {
        int64_t rseed;
        if (seed >= INT32_MIN && seed <= INT32_MAX) {
          int32_t s32 = (int32_t)((uint32_t)(int32_t)seed + (uint32_t)i);
          rseed = (int64_t)s32 + part;
        } else {
          rseed = (int64_t)((uint64_t)seed + (uint64_t)(int64_t)i + (uint64_t)(int64_t)part);
        }
        xs_t x;
        xs_init(&x, rseed);
        for (int64_t r = r0; r < r1; r++) c[r] = (xs_next_double(&x) < ratio) ? 1 : 0;
      }
    }
  }
  return 0;
}

/* HasSubBag.mkSubspace (ml/ensemble/HasSubBag.scala:90-106) */
int or_subspace(double ratio, int F, int64_t seed, int32_t* idx, int32_t* n_out) {
  int n = 0;
  if (ratio == 1.0) {
    for (int f = 0; f < F; f++) idx[n++] = f;
  } else {
    xs_t r;
    xs_init(&r, seed);
    for (int f = 0; f < F; f++)
      if (xs_next_double(&r) < ratio) idx[n++] = f;
  }
  *n_out = n;
  return 0;
}

/* ======================================================================
 * Spark 2.4.3 RandomForest.findSplitsForContinuousFeature over a replica's
 * subbag (rows replicated `count` times: sql/bfunctions.scala:42-44,
 * HasSubBag.scala:112-114).  Split-finding sample fraction per
 * RandomForest.samplesFractionForFindSplits; when fraction < 1 the reference
 * draws an RDD sample that is not reproduced: we use the whole subbag
 * (exact_out = 0 flags it).
 * ==================================================================== */
typedef struct {
  double v;
  int64_t c;
} vc_t;
static int cmp_double(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return (x < y) ? -1 : (x > y) ? 1 : 0;
}

/* Spark 2.4.3 RandomForest.findSplitsForContinuousFeature.  vals: the nonzero values of
   the split-finding sample with multiplicity (findSplitsBySorting drops zeros); n =
   metadata.numExamples; num_samples = (samplesFractionForFindSplits * numExamples).toInt,
   the expected sample size whose shortfall over nnz is the implied zero count. */
/* thr holds cap values: a split-finding sample larger than num_samples can pass one more
   target than numSplits (Spark then sets numSplits to the length it got); -1 past cap. */
static int find_splits_values(double* vals /*nonzero values with multiplicity, sorted in place*/,
                              int64_t nnz, int64_t n, int64_t num_samples, int64_t max_bins,
                              double* thr, int cap) {
  if (nnz == 0) return 0; /* featureSamples.isEmpty */
  const int64_t max_possible_bins = (max_bins < n) ? max_bins : n;
  const int64_t num_splits = max_possible_bins - 1;
  qsort(vals, (size_t)nnz, sizeof(double), cmp_double);
  vc_t* vc = (vc_t*)malloc(sizeof(vc_t) * (size_t)(nnz + 1));
  int64_t k = 0;
  /* distinct values with counts, plus valueCountMap + (0.0 -> numSamples - partNumSamples),
     merged in sorted position (values are nonzero, so zero sits between signs) */
  const int64_t zeros = num_samples - nnz;
  int zero_done = !(zeros > 0);
  for (int64_t i = 0; i < nnz;) {
    double v = vals[i];
    int64_t j = i;
    while (j < nnz && vals[j] == v) j++;
    if (!zero_done && v > 0.0) {
      vc[k].v = 0.0;
      vc[k].c = zeros;
      k++;
      zero_done = 1;
    }
    vc[k].v = v;
    vc[k].c = j - i;
    k++;
    i = j;
  }
  if (!zero_done) {
    vc[k].v = 0.0;
    vc[k].c = zeros;
    k++;
  }
  const int64_t possible = k - 1;
  int nt = 0;
  if (possible == 0) {
    nt = 0;
  } else if (possible <= num_splits) {
    for (int64_t i = 1; i <= possible; i++) thr[nt++] = (vc[i - 1].v + vc[i].v) / 2.0;
  } else {
    const double stride = (double)num_samples / (double)(num_splits + 1);
    int32_t current = (int32_t)vc[0].c; /* Scala Int */
    double target = stride;
    for (int64_t i = 1; i < k; i++) {
      const int32_t prev = current;
      current += (int32_t)vc[i].c;
      const double pg = fabs((double)prev - target);
      const double cg = fabs((double)current - target);
      if (pg < cg) {
        if (nt >= cap) {
          free(vc);
          return -1;
        }
        thr[nt++] = (vc[i - 1].v + vc[i].v) / 2.0;
        target += stride;
      }
    }
  }
  free(vc);
  return nt;
}

/* ======================================================================
 * The split-finding sample (Spark 2.4.3 RandomForest.findSplits):
 *   fraction = samplesFractionForFindSplits = required / numExamples when
 *     required = max(maxPossibleBins^2, 10000) < numExamples, else 1;
 *   input.sample(withReplacement = false, fraction, new XORShiftRandom(seed).nextInt())
 *   -> PartitionwiseSampledRDD: java.util.Random(sampleSeed).nextLong() per partition, in
 *      partition order, seeds that partition's BernoulliSampler (XORShiftRandom.setSeed);
 *   -> BernoulliSampler.sample per item: GapSampling when fraction <= 0.4
 *      (countForDropping = (log(max(u, 5e-11)) / log1p(-f)).toInt, first gap drawn at
 *      construction), else nextDouble() <= fraction.
 * The items are the replica's subbag rows in partition order, each row repeated `count`
 * times consecutively (replicate_row = explode(array_repeat), sql/bfunctions.scala:42-44).
 * `seed` is the base learner's seed param (HasSeed default: class-name hashCode).
 * Math.log / log1p are libm here (the JVM's may differ by 1 ulp; a draw flips only if the
 * quotient lands within that of an integer).
 * ==================================================================== */
typedef struct {
  uint64_t s;
} jr_t; /* java.util.Random */
static void jr_init(jr_t* r, int64_t seed) { r->s = ((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
static int32_t jr_next(jr_t* r, int bits) {
  r->s = (r->s * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
  return (int32_t)(uint32_t)(r->s >> (48 - bits));
}
static int64_t jr_next_long(jr_t* r) {
  const int64_t hi = (int64_t)jr_next(r, 32), lo = (int64_t)jr_next(r, 32);
  return (int64_t)((uint64_t)hi << 32) + lo;
}

double or_split_sample_fraction(int64_t num_examples, int max_bins) {
  const int64_t mpb = (max_bins < num_examples) ? max_bins : num_examples;
  const int64_t required = (mpb * mpb > 10000) ? mpb * mpb : 10000;
  return (required < num_examples) ? (double)required / (double)num_examples : 1.0;
}

void or_split_sample_seeds(int64_t dt_seed, int P, int64_t* part_seed) {
  xs_t x;
  xs_init(&x, dt_seed);
  const int64_t sample_seed = (int64_t)xs_next(&x, 32); /* XORShiftRandom.nextInt */
  jr_t j;
  jr_init(&j, sample_seed);
  for (int p = 0; p < P; p++) part_seed[p] = jr_next_long(&j);
}

int64_t or_split_sample(const uint8_t* cnt, const int64_t* off, int P, int64_t dt_seed,
                        double fraction, uint16_t* mult) {
  int64_t* ps = (int64_t*)malloc(sizeof(int64_t) * (size_t)(P > 0 ? P : 1));
  or_split_sample_seeds(dt_seed, P, ps);
  int64_t taken = 0;
  const double lnq = log1p(-fraction);
  for (int p = 0; p < P; p++) {
    for (int64_t r = off[p]; r < off[p + 1]; r++) mult[r] = 0;
    xs_t x;
    xs_init(&x, ps[p]);
    if (fraction <= 0.4) {
      int32_t cfd = 0, started = 0;
      for (int64_t r = off[p]; r < off[p + 1]; r++)
        for (int c = 0; c < cnt[r]; c++) {
          if (!started) { /* lazy GapSampling: its constructor draws the first gap */
            double u = xs_next_double(&x);
            if (u < 5e-11) u = 5e-11;
            cfd = (int32_t)(log(u) / lnq);
            started = 1;
          }
          if (cfd > 0) {
            cfd--;
          } else {
            double u = xs_next_double(&x);
            if (u < 5e-11) u = 5e-11;
            cfd = (int32_t)(log(u) / lnq);
            mult[r]++;
            taken++;
          }
        }
    } else {
      for (int64_t r = off[p]; r < off[p + 1]; r++)
        for (int c = 0; c < cnt[r]; c++)
          if (xs_next_double(&x) <= fraction) {
            mult[r]++;
            taken++;
          }
    }
  }
  free(ps);
  return taken;
}

int or_find_splits(const double* X, int64_t N, int F, int feature, const uint8_t* counts,
                   int max_bins, double* thr_out, int* exact_out) {
  int64_t n = 0, nnz = 0;
  for (int64_t r = 0; r < N; r++) {
    n += counts[r];
    if (counts[r] && X[r * F + feature] != 0.0) nnz += counts[r];
  }
  double* vals = (double*)malloc(sizeof(double) * (size_t)(nnz + 1));
  int64_t k = 0;
  for (int64_t r = 0; r < N; r++) {
    const double x = X[r * F + feature];
    if (x != 0.0)
      for (int c = 0; c < counts[r]; c++) vals[k++] = x;
  }
  *exact_out = or_split_sample_fraction(n, max_bins) >= 1.0;
  int nt = find_splits_values(vals, nnz, n, n, max_bins, thr_out, (int)max_bins);
  free(vals);
  return nt;
}

/* MurmurHash3_x86_32 (= scala.util.hashing.MurmurHash3.bytesHash), exported so the tests
   can pin it to SMHasher's published verification value. */
double or_fastmath_exp_neg(double x) { return (x < 0 && x > -41) ? or_fm_exp_neg(x) : NAN; }
uint32_t or_mm3_bytes_hash(const uint8_t* data, int len, uint32_t seed) {
  return mm3_bytes_hash(data, len, seed);
}

/* Feature matrix accessor: X is fp64 [N][F] (xkind 0) or u8 value codes whose fp64 value is
   the code itself (xkind 1; the synthetic workload of SURVEY.md §8d, 32 integer levels). */
static inline double xval(const void* X, int xkind, int64_t i) {
  return xkind ? (double)((const uint8_t*)X)[i] : ((const double*)X)[i];
}

/* Host restatement of the synthetic bench data (the product generates the same
   rows on the device): x[r,f] = splitmix64(seed ^ (r*F+f)) mod 32; h2 = splitmix64(~seed ^ r);
   regression y = (sum_{f<8} (f+1) x[r,f] + (h2 mod 64) - 32) / 64, class
   y = (x0 + 3 x1 + 7 x2 + h2 mod 8) mod C.  Rows [row_begin, row_begin + n). */
static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
void or_synth(int64_t row_begin, int64_t n, int F, uint64_t seed, int C, int nthreads, uint8_t* X,
              double* y) {
  if (nthreads <= 0) nthreads = 1;
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (int64_t i = 0; i < n; i++) {
    const uint64_t r = (uint64_t)(row_begin + i);
    int x[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int f = 0; f < F; f++) {
      const int v = (int)(splitmix64(seed ^ (r * (uint64_t)F + (uint64_t)f)) & 31u);
      X[i * F + f] = (uint8_t)v;
      if (f < 8) x[f] = v;
    }
    const uint64_t h2 = splitmix64(~seed ^ r);
    if (C == 0) {
      int64_t k = 0;
      for (int f = 0; f < 8 && f < F; f++) k += (int64_t)(f + 1) * x[f];
      k += (int64_t)(h2 & 63u) - 32;
      y[i] = ldexp((double)k, -6);
    } else {
      y[i] = (double)((x[0] + 3 * x[1] + 7 * x[2] + (int)(h2 & 7u)) % C);
    }
  }
}

/* ======================================================================
 * Spark 2.4.3 DecisionTree (RandomForest.run, numTrees=1, "all"),
 * invoked by HasBaseLearner.fitBaseLearner (ml/ensemble/ensembleParams.scala:99-117).
 * Level-wise growth over the replicated subbag; stats accumulate in fp64 in
 * row order exactly as DTStatsAggregator.update does.
 * ==================================================================== */
#define MAXS 256 /* max stats per calculator (classes) */

typedef struct { /* ImpurityStats of the chosen candidate */
  double gain, impurity;
  int valid;
  double calc[MAXS], left[MAXS], right[MAXS];
} istats_t;

typedef struct { /* LearningNode; children are nodes[child] and nodes[child + 1] */
  int exists, is_leaf, has_split, split_f, split_bin, processed;
  int64_t child;
  double threshold;
  istats_t st;
} lnode_t;

/* the tree's LearningNodes in creation order (level by level, heap order within a level:
   Spark's node ids 2h, 2h+1 are only ever compared within a level, so indices replace them
   and depth 30 needs no 2^31-entry heap) */
typedef struct {
  lnode_t* v;
  int64_t n, cap;
} lnodes_t;
static int64_t lnodes_push(lnodes_t* a) {
  if (a->n == a->cap) {
    a->cap = a->cap ? 2 * a->cap : 64;
    a->v = (lnode_t*)realloc(a->v, sizeof(lnode_t) * (size_t)a->cap);
  }
  memset(&a->v[a->n], 0, sizeof(lnode_t));
  return a->n++;
}

static double calc_count_d(const double* s, int ns, int gini) {
  if (!gini) return s[0];
  double t = 0.0;
  for (int i = 0; i < ns; i++) t += s[i];
  return t;
}
static int64_t calc_count(const double* s, int ns, int gini) {
  return (int64_t)calc_count_d(s, ns, gini);
}
/* Variance.calculate / Gini.calculate */
static double calc_impurity(const double* s, int ns, int gini) {
  if (!gini) {
    const double count = s[0], sum = s[1], sumsq = s[2];
    if (count == 0) return 0.0;
    const double squared_loss = sumsq - (sum * sum) / count;
    return squared_loss / count;
  }
  const double total = calc_count_d(s, ns, 1);
  if (total == 0) return 0.0;
  double imp = 1.0;
  for (int c = 0; c < ns; c++) {
    const double freq = s[c] / total;
    imp -= freq * freq;
  }
  return imp;
}
/* VarianceCalculator.predict / GiniCalculator.predict */
static double calc_predict(const double* s, int ns, int gini) {
  const int64_t count = calc_count(s, ns, gini);
  if (count == 0) return 0.0;
  if (!gini) return s[1] / (double)count;
  int best = -1;
  double bv = -1.7976931348623157e308;
  for (int c = 0; c < ns; c++)
    if (s[c] > bv) {
      bv = s[c];
      best = c;
    }
  return (double)best;
}

/* RandomForest.calculateImpurityStats.  The reference threads the previous
   candidate's ImpurityStats through every call (binsToBestSplit); only its
   impurityCalculator (the parent) and impurity are read, so the chain state is
   (chain_calc, chain_impurity), fixed by the node's stats or, at the root, by
   the first candidate's left+right.  Returns the gain (Double.MinValue when
   invalid) and sets *valid. */
static double candidate_gain(int* chain_set, double* chain_calc, double* chain_imp,
                             const double* left, const double* right, int ns, int gini,
                             const or_tree_params* p, int* valid) {
  if (!*chain_set) {
    for (int i = 0; i < ns; i++) chain_calc[i] = left[i] + right[i];
    *chain_imp = calc_impurity(chain_calc, ns, gini);
    *chain_set = 1;
  }
  const int64_t lc = calc_count(left, ns, gini), rc = calc_count(right, ns, gini);
  const int64_t total = lc + rc;
  if (lc < p->min_instances_per_node || rc < p->min_instances_per_node) {
    *valid = 0;
    return -1.7976931348623157e308; /* Double.MinValue */
  }
  const double li = calc_impurity(left, ns, gini), ri = calc_impurity(right, ns, gini);
  const double lw = (double)lc / (double)total, rw = (double)rc / (double)total;
  const double gain = *chain_imp - lw * li - rw * ri;
  if (gain < p->min_info_gain) {
    *valid = 0;
    return -1.7976931348623157e308;
  }
  *valid = 1;
  return gain;
}

typedef struct {
  or_node* nodes;
  double* stats;
  int stride, ns, count, max_nodes, overflow;
} emit_t;

typedef struct {
  int is_leaf;
  double prediction;
} tn_ret;

/* LearningNode.toNode(prune = true) emitted in NodeData pre-order */
static tn_ret to_node(const lnode_t* ln, int64_t hid, emit_t* e, int gini, int* out_id) {
  tn_ret ret;
  const lnode_t* n = &ln[hid];
  const int my = e->count++;
  if (my >= e->max_nodes) {
    e->overflow = 1;
    *out_id = my;
    ret.is_leaf = 1;
    ret.prediction = 0;
    return ret;
  }
  *out_id = my;
  or_node* o = &e->nodes[my];
  memset(o, 0, sizeof(*o));
  o->id = my;
  double* so = e->stats + (int64_t)my * e->stride;
  if (n->has_split) {
    const int mark = e->count;
    int lid, rid;
    tn_ret l = to_node(ln, n->child, e, gini, &lid);
    tn_ret r = to_node(ln, n->child + 1, e, gini, &rid);
    if (l.is_leaf && r.is_leaf && l.prediction == r.prediction) {
      /* pruned: LeafNode(l.prediction, stats.impurity, stats.impurityCalculator) */
      e->count = mark;
      o->left = o->right = -1;
      o->feature = -1;
      o->split_bin = -1;
      o->threshold = 0;
      o->prediction = l.prediction;
      o->impurity = n->st.impurity;
      o->gain = -1.0;
      memcpy(so, n->st.calc, sizeof(double) * (size_t)e->ns);
      ret.is_leaf = 1;
      ret.prediction = l.prediction;
      return ret;
    }
    o->left = lid;
    o->right = rid;
    o->feature = n->split_f;
    o->split_bin = n->split_bin;
    o->threshold = n->threshold;
    o->prediction = calc_predict(n->st.calc, e->ns, gini);
    o->impurity = n->st.impurity;
    o->gain = n->st.gain;
    memcpy(so, n->st.calc, sizeof(double) * (size_t)e->ns);
    ret.is_leaf = 0;
    ret.prediction = o->prediction;
    return ret;
  }
  o->left = o->right = -1;
  o->feature = -1;
  o->split_bin = -1;
  o->threshold = 0;
  o->prediction = calc_predict(n->st.calc, e->ns, gini);
  o->impurity = n->st.valid ? n->st.impurity : -1.0;
  o->gain = -1.0;
  memcpy(so, n->st.calc, sizeof(double) * (size_t)e->ns);
  ret.is_leaf = 1;
  ret.prediction = o->prediction;
  return ret;
}

static int fit_one(const void* X, int xkind, const double* y, int64_t N, int F, const uint8_t* cnt,
                   const int32_t* sub, int Fr, const or_tree_params* p, or_node* out_nodes,
                   int max_nodes, double* out_stats, int stride, int32_t* out_num_nodes,
                   int32_t* out_ns, int32_t* out_exact, int inner) {
  const int gini = p->impurity == 1;
  const int D = p->max_depth;
  if (D < 0 || D > 30 || p->max_bins < 2 || Fr <= 0) return -1;
  int64_t n = 0, nrows = 0;
  double maxlab = -1;
  for (int64_t r = 0; r < N; r++)
    if (cnt[r]) {
      n += cnt[r];
      nrows++;
      if (y[r] > maxlab) maxlab = y[r];
    }
  if (n == 0) return -2; /* DecisionTree requires size of input RDD > 0 */
  int ns = 3;
  if (gini) {
    ns = (int)maxlab + 1; /* Classifier.getNumClasses on the subbag */
    if (ns > MAXS || ns > stride) return -3;
  }
  if (stride < ns) return -3;
  int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * (size_t)nrows);
  {
    int64_t k = 0;
    for (int64_t r = 0; r < N; r++)
      if (cnt[r]) rows[k++] = r;
  }
  /* findSplits + TreePoint binning */
  const int tcap = p->max_bins + 64; /* thresholds per feature (find_splits_values) */
  double* thr = (double*)malloc(sizeof(double) * (size_t)Fr * (size_t)tcap);
  int* nthr = (int*)malloc(sizeof(int) * (size_t)Fr);
  uint16_t* bins = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)nrows * (size_t)Fr);
  int all_exact = 1;
  int too_many = 0;
  /* RandomForest.findSplits: the split-finding sample of the subbag */
  const double fraction = or_split_sample_fraction(n, p->max_bins);
  uint16_t* mult = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)N);
  int64_t num_samples = n;
  if (fraction < 1.0) {
    const int64_t one[2] = {0, N};
    const int64_t* off = p->part_off ? p->part_off : one;
    const int P = p->part_off ? p->num_partitions : 1;
    or_split_sample(cnt, off, P, p->seed, fraction, mult);
    num_samples = (int64_t)(int32_t)(fraction * (double)n); /* (fraction * numExamples).toInt */
  } else {
    for (int64_t r = 0; r < N; r++) mult[r] = cnt[r];
  }
  /* features are independent: split finding and binning run one feature per thread */
#pragma omp parallel for schedule(dynamic, 1) num_threads(inner)
  for (int fl = 0; fl < Fr; fl++) {
    const int fg = sub[fl];
    int64_t nnz = 0;
    for (int64_t k = 0; k < nrows; k++)
      if (xval(X, xkind, rows[k] * F + fg) != 0.0) nnz += mult[rows[k]];
    double* vals = (double*)malloc(sizeof(double) * (size_t)(nnz + 1));
    int64_t q = 0;
    for (int64_t k = 0; k < nrows; k++) {
      const double x = xval(X, xkind, rows[k] * F + fg);
      if (x != 0.0)
        for (int c = 0; c < mult[rows[k]]; c++) vals[q++] = x;
    }
    nthr[fl] = find_splits_values(vals, nnz, n, num_samples, p->max_bins, thr + (int64_t)fl * tcap, tcap);
    free(vals);
    if (nthr[fl] < 0) { /* more thresholds than tcap: refuse rather than overflow */
      nthr[fl] = 0;
      too_many = 1;
      continue;
    }
    const double* t = thr + (int64_t)fl * tcap;
    for (int64_t k = 0; k < nrows; k++) {
      const double x = xval(X, xkind, rows[k] * F + fg);
      int lo = 0, hi = nthr[fl]; /* #thresholds < x  == Arrays.binarySearch result */
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (t[mid] < x)
          lo = mid + 1;
        else
          hi = mid;
      }
      bins[k * Fr + fl] = (uint16_t)lo;
    }
  }
  lnodes_t tree = {NULL, 0, 0};
  lnodes_push(&tree); /* root: LearningNode.emptyNode(1), stats == null */
  tree.v[0].exists = 1;
  int64_t* node_of = (int64_t*)malloc(sizeof(int64_t) * (size_t)nrows);
  for (int64_t k = 0; k < nrows; k++) node_of[k] = 0;
  if (too_many) {
    free(rows);
    free(thr);
    free(nthr);
    free(bins);
    free(mult);
    return -6;
  }
  int nb = p->max_bins; /* bins per feature row: numSplits + 1, one more after a large sample */
  for (int fl = 0; fl < Fr; fl++)
    if (nthr[fl] + 1 > nb) nb = nthr[fl] + 1;
  int64_t first = 0, last = 0; /* this level's nodes: tree.v[first .. last] */
  for (int level = 0; level <= D && first <= last; level++) {
    int64_t nact = 0;
    for (int64_t h = first; h <= last; h++)
      if (tree.v[h].exists && !tree.v[h].is_leaf) nact++;
    if (nact == 0) break;
    const int64_t per_node = (int64_t)Fr * nb * ns;
    /* process active nodes in groups bounded by memory (mirrors selectNodesToSplit) */
    int64_t group = (int64_t)(256u << 20) / (int64_t)(per_node * 8 + 1);
    if (group < 1) group = 1;
    int64_t* slot = (int64_t*)malloc(sizeof(int64_t) * (size_t)(last - first + 1));
    int64_t h0 = first;
    while (h0 <= last) {
      for (int64_t h = first; h <= last; h++) slot[h - first] = -1;
      int64_t g = 0, h = h0;
      int64_t* members = (int64_t*)malloc(sizeof(int64_t) * (size_t)group);
      for (; h <= last && g < group; h++)
        if (tree.v[h].exists && !tree.v[h].is_leaf) {
          slot[h - first] = g;
          members[g++] = h;
        }
      h0 = h;
      if (g == 0) {
        free(members);
        continue;
      }
      double* agg = (double*)calloc((size_t)(g * per_node), sizeof(double));
      double* par = (double*)calloc((size_t)(g * ns), sizeof(double));
      /* the group's rows grouped by node, stably (row order kept within a node): a node's
         cells then stay in cache while its rows are added; every (node, feature, bin) cell
         still sees its rows in row order */
      int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nrows + 1));
      int64_t n_order = 0;
      {
        int64_t* start = (int64_t*)calloc((size_t)(g + 1), sizeof(int64_t));
        for (int64_t k = 0; k < nrows; k++) {
          const int64_t nd = node_of[k];
          if (nd < first || nd > last || slot[nd - first] < 0) continue;
          start[slot[nd - first] + 1]++;
        }
        for (int64_t s = 0; s < g; s++) start[s + 1] += start[s];
        n_order = start[g];
        for (int64_t k = 0; k < nrows; k++) {
          const int64_t nd = node_of[k];
          if (nd < first || nd > last || slot[nd - first] < 0) continue;
          order[start[slot[nd - first]]++] = k;
        }
        free(start);
      }
      /* RandomForest.findBestSplits: every partition aggregates its own rows
         (mapPartitions -> binSeqOp -> DTStatsAggregator.update, row order within the
         partition), and the per-node aggregates of the partitions are merged with
         reduceByKey((a, b) => a.merge(b)) -- allStats(i) += other.allStats(i).  The merge order
         is the shuffle's; partition order is one order Spark produces (and the only one at
         P = 1), so each (node, feature, bin) cell here is: per partition, its rows in row
         order from 0.0; then the partials added in partition order.  An empty partial adds
         +0.0, which changes no sum (no sum is ever -0.0), so only touched cells are merged.
         Gini cells are integer counts (order-free): summed directly.  Threads own disjoint
         feature ranges; the row order within a node segment ascends, so its partition index
         only advances. */
      const int64_t one_off[2] = {0, N};
      const int64_t* poff = p->part_off ? p->part_off : one_off;
      const int P = p->part_off ? p->num_partitions : 1;
#pragma omp parallel num_threads(inner)
      {
        int nth = 1, tid = 0;
#ifdef _OPENMP
        nth = omp_get_num_threads();
        tid = omp_get_thread_num();
#endif
        const int f0 = (int)((int64_t)Fr * tid / nth), f1 = (int)((int64_t)Fr * (tid + 1) / nth);
        /* the open partition's partial of the current node: cells (feature-major as agg) and
           the node total, with the list of touched cells */
        double* pa = gini ? NULL : (double*)calloc((size_t)(per_node + ns), sizeof(double));
        uint8_t* tf = gini ? NULL : (uint8_t*)calloc((size_t)per_node, 1);
        int64_t* tl = gini ? NULL : (int64_t*)malloc(sizeof(int64_t) * (size_t)(per_node > 0 ? per_node : 1));
        int64_t ntl = 0;
        int64_t open_s = -1; /* slot of the open partial, -1: none */
        int open_q = -1;
        int q = 0;
        for (int64_t o = 0; o < n_order; o++) {
          const int64_t k = order[o];
          const int64_t s = slot[node_of[k] - first];
          const double lab = y[rows[k]];
          double* a = agg + s * per_node;
          double* pp = par + s * ns;
          if (!gini) {
            if (s != open_s) q = 0;
            while (q + 1 < P && rows[k] >= poff[q + 1]) q++;
            if (s != open_s || q != open_q) { /* merge the closed partial (a.merge(b)) */
              if (open_s >= 0) {
                double* ca = agg + open_s * per_node;
                for (int64_t t = 0; t < ntl; t++) {
                  ca[tl[t]] += pa[tl[t]];
                  pa[tl[t]] = 0.0;
                  tf[tl[t]] = 0;
                }
                if (tid == 0)
                  for (int i = 0; i < ns; i++) {
                    par[open_s * ns + i] += pa[per_node + i];
                    pa[per_node + i] = 0.0;
                  }
              }
              ntl = 0;
              open_s = s;
              open_q = q;
            }
          }
          for (int c = 0; c < cnt[rows[k]]; c++) {
            for (int fl = f0; fl < f1; fl++) {
              const int64_t cell = ((int64_t)fl * nb + bins[k * Fr + fl]) * ns;
              if (!gini) {
                double* st = pa + cell;
                if (!tf[cell]) {
                  tf[cell] = 1;
                  tl[ntl++] = cell;
                  tl[ntl++] = cell + 1;
                  tl[ntl++] = cell + 2;
                }
                st[0] += 1.0;
                st[1] += 1.0 * lab;
                st[2] += 1.0 * lab * lab;
              } else {
                a[cell + (int)lab] += 1.0;
              }
            }
            if (tid == 0) {
              if (!gini) {
                double* pt = pa + per_node;
                pt[0] += 1.0;
                pt[1] += 1.0 * lab;
                pt[2] += 1.0 * lab * lab;
              } else {
                pp[(int)lab] += 1.0;
              }
            }
          }
        }
        if (!gini && open_s >= 0) {
          double* ca = agg + open_s * per_node;
          for (int64_t t = 0; t < ntl; t++) ca[tl[t]] += pa[tl[t]];
          if (tid == 0)
            for (int i = 0; i < ns; i++) par[open_s * ns + i] += pa[per_node + i];
        }
        free(pa);
        free(tf);
        free(tl);
      }
      /* binsToBestSplit for each node of the group */
      for (int64_t gi = 0; gi < g; gi++) {
        lnode_t* node = &tree.v[members[gi]];
        double* a = agg + gi * per_node;
        int chain_set = 0;
        double chain_calc[MAXS], chain_imp = 0.0;
        if (level > 0) {
          memcpy(chain_calc, node->st.calc, sizeof(double) * (size_t)ns);
          chain_imp = node->st.impurity;
          chain_set = 1;
        }
        int best_f = -1, best_s = -1, best_valid = 0;
        double best_gain = 0.0;
        double left[MAXS], right[MAXS];
        for (int fl = 0; fl < Fr; fl++) {
          const int nsp = nthr[fl];
          if (nsp == 0) continue;
          double* fa = a + (int64_t)fl * nb * ns;
          for (int s = 0; s < nsp; s++) /* mergeForFeature: prefix over bins */
            for (int i = 0; i < ns; i++) fa[(s + 1) * ns + i] += fa[s * ns + i];
          int fbest_s = -1, fbest_valid = 0;
          double fbest_gain = 0.0;
          for (int s = 0; s < nsp; s++) {
            for (int i = 0; i < ns; i++) {
              left[i] = fa[s * ns + i];
              right[i] = fa[nsp * ns + i];
            }
            for (int i = 0; i < ns; i++) right[i] -= left[i];
            int valid;
            const double gain = candidate_gain(&chain_set, chain_calc, &chain_imp, left, right,
                                               ns, gini, p, &valid);
            if (fbest_s < 0 || gain > fbest_gain) { /* maxBy: first max */
              fbest_gain = gain;
              fbest_s = s;
              fbest_valid = valid;
            }
          }
          if (best_f < 0 || fbest_gain > best_gain) {
            best_gain = fbest_gain;
            best_f = fl;
            best_s = fbest_s;
            best_valid = fbest_valid;
          }
        }
        istats_t* best = &node->st;
        if (best_f < 0) { /* no feature has splits: invalid stats on the parent aggregate */
          memcpy(best->calc, par + gi * ns, sizeof(double) * (size_t)ns);
          best->gain = -1.7976931348623157e308;
          best->impurity = calc_impurity(best->calc, ns, gini);
          best->valid = 0;
        } else {
          memcpy(best->calc, chain_calc, sizeof(double) * (size_t)ns);
          best->gain = best_gain;
          best->impurity = chain_imp;
          best->valid = best_valid;
          const double* fa = a + (int64_t)best_f * nb * ns;
          const int nsp = nthr[best_f];
          for (int i = 0; i < ns; i++) {
            best->left[i] = fa[best_s * ns + i];
            best->right[i] = fa[nsp * ns + i] - fa[best_s * ns + i];
          }
        }
        node->processed = 1;
        const int is_leaf = (best->gain <= 0) || (level == D);
        node->is_leaf = is_leaf;
        if (!is_leaf) {
          node->has_split = 1;
          node->split_f = best_f;
          node->split_bin = best_s;
          node->threshold = thr[(int64_t)best_f * tcap + best_s];
          const int child_leaf = (level + 1) == D;
          const int64_t ci = lnodes_push(&tree);
          lnodes_push(&tree);
          node = &tree.v[members[gi]]; /* the push may have moved the array */
          best = &node->st;
          node->child = ci;
          lnode_t* L = &tree.v[ci];
          lnode_t* R = &tree.v[ci + 1];
          L->exists = R->exists = 1;
          /* LearningNode(child, isLeaf, getEmptyImpurityStats(calculator)) */
          L->st.impurity = calc_impurity(best->left, ns, gini);
          R->st.impurity = calc_impurity(best->right, ns, gini);
          L->is_leaf = child_leaf || (L->st.impurity == 0.0);
          R->is_leaf = child_leaf || (R->st.impurity == 0.0);
          L->st.gain = R->st.gain = NAN;
          L->st.valid = R->st.valid = 1;
          memcpy(L->st.calc, best->left, sizeof(double) * (size_t)ns);
          memcpy(R->st.calc, best->right, sizeof(double) * (size_t)ns);
        }
      }
      free(agg);
      free(par);
      free(order);
      free(members);
    }
    free(slot);
    /* route rows: predictImpl on binned features (ContinuousSplit.shouldGoLeft) */
    for (int64_t k = 0; k < nrows; k++) {
      const int64_t nd = node_of[k];
      if (nd < first || nd > last) continue;
      const lnode_t* node = &tree.v[nd];
      if (!node->has_split) continue;
      node_of[k] = (bins[k * Fr + node->split_f] <= node->split_bin) ? node->child : node->child + 1;
    }
    first = last + 1;
    last = tree.n - 1;
  }
  emit_t e;
  e.nodes = out_nodes;
  e.stats = out_stats;
  e.stride = stride;
  e.ns = ns;
  e.count = 0;
  e.max_nodes = max_nodes;
  e.overflow = 0;
  int rid;
  to_node(tree.v, 0, &e, gini, &rid);
  *out_num_nodes = e.count;
  *out_ns = ns;
  free(mult);
  *out_exact = all_exact;
  free(tree.v);
  free(node_of);
  free(rows);
  free(thr);
  free(nthr);
  free(bins);
  return e.overflow ? -4 : 0;
}

int or_fit_x(const void* X, int xkind, const double* y, int64_t N, int F, const uint8_t* counts,
             int L, const int32_t* sub, const int32_t* nsub, const or_tree_params* p, int nthreads,
             or_node* nodes, int max_nodes, double* stats, int stats_stride, int32_t* num_nodes,
             int32_t* num_stats, int32_t* all_exact) {
  int err = 0;
  if (nthreads <= 0) nthreads = 1;
  const int outer = nthreads < L ? nthreads : (L > 0 ? L : 1);
  const int inner = nthreads / outer > 0 ? nthreads / outer : 1; /* spare threads per learner */
#ifdef _OPENMP
  if (inner > 1) omp_set_max_active_levels(2);
#endif
#pragma omp parallel for schedule(dynamic, 1) num_threads(outer)
  for (int l = 0; l < L; l++) {
    int32_t ex = 1;
    int rc = fit_one(X, xkind, y, N, F, counts + (int64_t)l * N, sub + (int64_t)l * F, nsub[l], p,
                     nodes + (int64_t)l * max_nodes, max_nodes,
                     stats + (int64_t)l * max_nodes * stats_stride, stats_stride, &num_nodes[l],
                     &num_stats[l], &ex, inner);
    all_exact[l] = ex;
    if (rc) {
#pragma omp critical
      err = rc;
    }
  }
  return err;
}

int or_fit(const double* X, const double* y, int64_t N, int F, const uint8_t* counts, int L,
           const int32_t* sub, const int32_t* nsub, const or_tree_params* p, int nthreads,
           or_node* nodes, int max_nodes, double* stats, int stats_stride, int32_t* num_nodes,
           int32_t* num_stats, int32_t* all_exact) {
  return or_fit_x(X, 0, y, N, F, counts, L, sub, nsub, p, nthreads, nodes, max_nodes, stats,
                  stats_stride, num_nodes, num_stats, all_exact);
}

/* BaggingRegressionModel.predict (ml/regression/BaggingRegressor.scala:248-256) and
   BaggingClassificationModel.predict (ml/classification/BaggingClassifier.scala:248-257):
   slicer (HasSubBag.scala:128-131) + Node.predictImpl + breeze sum / mode. */
void or_predict(const double* X, int64_t N, int F, int L, const int32_t* sub, const int32_t* nsub,
                const or_node* nodes, int max_nodes, int agg, double* out, double* per_tree) {
  (void)nsub;
  /* rows are independent: one row per iteration, per-thread vote buffers */
#pragma omp parallel
  {
    double* votes = (double*)malloc(sizeof(double) * (size_t)L);
    double* vv = (double*)malloc(sizeof(double) * (size_t)L);
    int* vc = (int*)malloc(sizeof(int) * (size_t)L);
#pragma omp for schedule(static)
    for (int64_t r = 0; r < N; r++) {
      const double* x = X + r * F;
      for (int l = 0; l < L; l++) {
        const or_node* t = nodes + (int64_t)l * max_nodes;
        int id = 0;
        while (t[id].left >= 0) {
          const double v = x[sub[(int64_t)l * F + t[id].feature]];
          id = (v <= t[id].threshold) ? t[id].left : t[id].right;
        }
        votes[l] = t[id].prediction;
        if (per_tree) per_tree[(int64_t)l * N + r] = votes[l];
      }
      if (agg == 0) {
        double s = 0.0;
        for (int l = 0; l < L; l++) s += votes[l];
        out[r] = s / (double)L;
      } else {
        /* breeze.stats.mode: first value to reach the final max count */
        int nd = 0, maxc = 0;
        double mode = 0.0;
        for (int l = 0; l < L; l++) {
          int j = 0;
          while (j < nd && vv[j] != votes[l]) j++;
          if (j == nd) {
            vv[nd] = votes[l];
            vc[nd] = 0;
            nd++;
          }
          vc[j]++;
          if (vc[j] > maxc) {
            maxc = vc[j];
            mode = votes[l];
          }
        }
        out[r] = mode;
      }
    }
    free(votes);
    free(vv);
    free(vc);
  }
}
