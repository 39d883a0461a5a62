/*
 * sbag_oracle.h — CPU restatement of the spark-ensemble bagging hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library; the product
 * (libsbag, spark-bagging_amd/) never links or calls it.
 *
 * PARITY UNPINNED: the reference (Scala on Spark 2.4.3, no JVM in this image)
 * ships no golden vectors for this path; this restatement is
 * checked against an independent pure-Python restatement (oracle/pyoracle.py),
 * Java-semantics known answers (String.hashCode seeds) and algebraic invariants.
 */
#ifndef SBAG_ORACLE_H
#define SBAG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG primitives (upstream Spark / commons-math3 / scala-library) ---- */
uint64_t or_hash_seed(int64_t seed);
void or_xorshift_next(int64_t seed, int bits, int n, int32_t* out);
void or_xorshift_doubles(int64_t seed, int n, double* out);
void or_well_next(int64_t seed, int bits, int n, int32_t* out);
void or_well_doubles(int64_t seed, int n, double* out);
void or_poisson(double lambda, int64_t seed, int n, int32_t* out);

/* ---- bag / subspace (sql/bfunctions.scala, ml/ensemble/HasSubBag.scala) ---- */
int or_bag(int replacement, double ratio, int learner_begin, int learner_end, int64_t seed,
           const int64_t* part_off, int P, int64_t N, uint8_t* counts /*[(end-begin)][N]*/);
int or_subspace(double ratio, int F, int64_t seed, int32_t* idx, int32_t* n_out);

/* ---- Spark 2.4.3 DecisionTree (RandomForest.run with numTrees=1, "all") ---- */
typedef struct {
  int32_t max_depth, max_bins, min_instances_per_node, impurity; /* 0 variance, 1 gini */
  double min_info_gain;
  int64_t seed;             /* the base learner's seed param (split-finding sample)       */
  const int64_t* part_off;  /* [num_partitions + 1] subbag partitions, NULL: one          */
  int32_t num_partitions, pad_;
} or_tree_params;

/* RandomForest.findSplits' sample: fraction for numExamples rows, the per-partition
   sampler seeds, and the multiplicity of each subbag row in the sample.            */
double or_split_sample_fraction(int64_t num_examples, int max_bins);
void or_split_sample_seeds(int64_t dt_seed, int P, int64_t* part_seed);
int64_t or_split_sample(const uint8_t* counts, const int64_t* part_off, int P, int64_t dt_seed,
                        double fraction, uint16_t* mult /*[N]*/);

typedef struct { /* pre-order NodeData layout (DecisionTreeModelReadWrite.NodeData) */
  int32_t id, left, right, feature; /* feature: subspace-local index, -1 for a leaf */
  int32_t split_bin, pad_;
  double threshold, prediction, impurity, gain;
} or_node;

/* thresholds of one feature from a replica's whole subbag (no sample); returns
   #thresholds.  exact_out = 1 when Spark's split-finding sample is the whole subbag. */
int or_find_splits(const double* X, int64_t N, int F, int feature, const uint8_t* counts,
                   int max_bins, double* thr_out, int* exact_out);

/* fit L trees.  counts [L][N]; sub [L][F] subspace lists, nsub [L].
   nodes [L][max_nodes], stats [L][max_nodes][stats_stride]. */
int or_fit(const double* X, const double* y, int64_t N, int F, const uint8_t* counts, int L,
           const int32_t* sub, const int32_t* nsub, const or_tree_params* p, int nthreads,
           or_node* nodes, int max_nodes, double* stats, int stats_stride, int32_t* num_nodes,
           int32_t* num_stats, int32_t* all_exact);

/* or_fit over fp64 X (xkind 0) or u8 value codes (xkind 1, value = code) */
int or_fit_x(const void* X, int xkind, const double* y, int64_t N, int F, const uint8_t* counts,
             int L, const int32_t* sub, const int32_t* nsub, const or_tree_params* p, int nthreads,
             or_node* nodes, int max_nodes, double* stats, int stats_stride, int32_t* num_nodes,
             int32_t* num_stats, int32_t* all_exact);

/* synthetic bench rows [row_begin, row_begin+n) as u8 codes + labels */
void or_synth(int64_t row_begin, int64_t n, int F, uint64_t seed, int C, int nthreads, uint8_t* X,
              double* y);
uint32_t or_mm3_bytes_hash(const uint8_t* data, int len, uint32_t seed);
/* commons-math3 FastMath.exp(x), -41 < x < 0 (NaN outside) */
double or_fastmath_exp_neg(double x);

/* ensemble prediction: agg 0 = mean (BaggingRegressionModel.predict),
   1 = breeze mode (BaggingClassificationModel.predict).                  */
void or_predict(const double* X, int64_t N, int F, int L, const int32_t* sub, const int32_t* nsub,
                const or_node* nodes, int max_nodes, int agg, double* out /*[N]*/,
                double* per_tree /*[L][N] or NULL*/);

#ifdef __cplusplus
}
#endif
#endif
