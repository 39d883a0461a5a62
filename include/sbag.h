/*
 * sbag.h — C ABI of the MI355X bagging engine (libsbag.so).
 *
 * Drop-in boundary for spark-ensemble's bagging hot path: BaggingRegressor /
 * BaggingClassifier `.fit` (train) and `.transform` (predict) with a
 * DecisionTree{Regressor,Classifier} base learner.  Every entry point cites the
 * reference interface it replaces (paths relative to
 * /root/reference/core/src/main/scala/org/apache/spark/).  The JNI binding a
 * maintainer adds on the Scala side is shown in INTEGRATION.md.
 *
 * Conventions
 *  - Every call returns an int status: SBAG_OK or one of the SBAG_E* codes below.
 *    The JNI shim maps SBAG_EINVAL to IllegalArgumentException (the reference's
 *    `require` / ParamValidators), SBAG_EEMPTY to SparkException ("ML algorithm
 *    was given empty dataset."), everything else to SparkException.
 *  - sbag_last_error() returns the message of the calling thread's last failure.
 *  - Host buffers passed in are read during the call only; the library owns
 *    device memory and the objects it returns until the matching *_free/_destroy.
 *  - A context is bound to one device.  Calls on one context are serialized by the
 *    library (a per-context lock): the reference runs learner Futures on a pool
 *    (ml/regression/BaggingRegressor.scala:169-191) and CrossValidator fits models
 *    concurrently, so several JVM threads may share a context.  Separate contexts
 *    run concurrently.  A dataset must be used with a context on its own device.
 */
#ifndef SBAG_H
#define SBAG_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBAG_OK 0
#define SBAG_EINVAL 1       /* IllegalArgumentException (require, ParamValidators)      */
#define SBAG_EEMPTY 2       /* SparkException: empty dataset / empty subbag             */
#define SBAG_EDEVICE 3      /* HIP runtime failure                                      */
#define SBAG_ENOMEM 4       /* device allocation failure                                */
#define SBAG_EUNSUPPORTED 5 /* input outside what the engine reproduces bit-exactly     */

#define SBAG_IMPURITY_VARIANCE 0 /* DecisionTreeRegressor (impurity "variance")  */
#define SBAG_IMPURITY_GINI 1     /* DecisionTreeClassifier (impurity "gini")     */

#define SBAG_AGG_MEAN 0 /* BaggingRegressionModel.predict (BaggingRegressor.scala:248-256)      */
#define SBAG_AGG_MODE 1 /* BaggingClassificationModel.predict (BaggingClassifier.scala:248-257) */

typedef struct sbag_ctx sbag_ctx;
typedef struct sbag_dataset sbag_dataset;
typedef struct sbag_forest sbag_forest;

/* ---- contexts ---------------------------------------------------------- */
int sbag_device_count(int32_t* n);
int sbag_ctx_create(int32_t device_ordinal, sbag_ctx** out);
int sbag_ctx_destroy(sbag_ctx* ctx);
const char* sbag_last_error(void);
const char* sbag_version(void);

/* ---- sampler: bfunctions.bag (sql/bfunctions.scala:46-68) --------------
 * Multiplicities of every row for learners [learner_begin, learner_end):
 *   replacement      -> Poisson(sample_ratio) reseeded seed+i+partitionIndex
 *                       (sql/catalyst/expressions/Poisson.scala:53-56,73)
 *   !replacement, 1  -> all ones (bfunctions.scala:56-57)
 *   !replacement     -> rand(seed+i) < sample_ratio (bfunctions.scala:62-64,
 *                       Spark Rand = XORShiftRandom(seed+i+partitionIndex))
 * partition_offsets[P+1] are the Spark partition boundaries of the DataFrame
 * rows (row j of partition p gets the j-th draw of stream (i, p)).           */
typedef struct {
  int32_t replacement;  /* HasSubBag.replacement (HasSubBag.scala:39-45)            */
  int32_t pad_;
  double sample_ratio;  /* HasSubBag.sampleRatio (HasSubBag.scala:52-62)            */
  int64_t seed;         /* HasSeed.seed (default: class-name hashCode)   */
  int32_t learner_begin, learner_end; /* global learner indices                    */
} sbag_sampler_params;

int sbag_sample(sbag_ctx* ctx, const sbag_sampler_params* p, const int64_t* partition_offsets,
                int32_t num_partitions, int64_t num_rows,
                uint8_t* counts_out /* host [(end-begin) x num_rows] */);

/* ---- subspace: HasSubBag.mkSubspace (ml/ensemble/HasSubBag.scala:90-106) */
int sbag_subspace(double ratio, int32_t num_features, int64_t seed, int32_t* idx_out,
                  int32_t* n_out);

/* ---- datasets (the DataFrame's label + features columns) ---------------- */
/* X row-major [num_rows x num_features] fp64, y [num_rows]; copied to HBM as
   per-feature value codes (exact distinct-value dictionaries; u8, u16 or u32
   codes by the widest feature) + labels.                                      */
int sbag_dataset_create(sbag_ctx* ctx, int64_t num_rows, int32_t num_features, const double* X,
                        const double* y, sbag_dataset** out);
/* SparseVector rows (CSR): indptr [num_rows+1] (indptr[0] == 0), per row strictly
   increasing indices in [0, num_features), values [indptr[num_rows]]; absent entries
   are 0.0 -- Spark's SparseVector semantics, which HasSubBag.slicer
   (ml/ensemble/HasSubBag.scala:128-131) and DecisionTree see.  No dense copy is made. */
int sbag_dataset_create_csr(sbag_ctx* ctx, int64_t num_rows, int32_t num_features,
                            const int64_t* indptr, const int32_t* indices, const double* values,
                            const double* y, sbag_dataset** out);
/* Columnar features (Arrow / Parquet column chunks, or values quantized upstream):
   columns[f] points to num_rows values of type col_type.                         */
#define SBAG_COL_F64 0
#define SBAG_COL_F32 1
#define SBAG_COL_U8 2
int sbag_dataset_create_columns(sbag_ctx* ctx, int64_t num_rows, int32_t num_features,
                                int32_t col_type, const void* const* columns, const double* y,
                                sbag_dataset** out);
/* Deterministic synthetic data generated directly in HBM (bench workload):
   x[r,f] = splitmix64(seed ^ (r*F+f)) mod 32; num_classes == 0 -> dyadic
   regression label, else a class label in [0, num_classes). */
int sbag_dataset_synthetic(sbag_ctx* ctx, int64_t num_rows, int32_t num_features, uint64_t seed,
                           int32_t num_classes, sbag_dataset** out);
int sbag_dataset_info(const sbag_dataset* ds, int64_t* num_rows, int32_t* num_features);
int sbag_dataset_labels(const sbag_dataset* ds, double* y_out);
int sbag_dataset_features(const sbag_dataset* ds, int64_t row_begin, int64_t row_end,
                          double* X_out /* [(row_end-row_begin) x F] */);
/* Replaces the label column (y [num_rows], host).  The reference selects whatever Double
   label column the DataFrame holds (ml/regression/BaggingRegressor.scala:146-150): labels
   that are not dyadic fixed point are fitted with Spark's row-order fp64 sums.          */
int sbag_dataset_set_labels(sbag_dataset* ds, const double* y);
/* Replication of an ingested dataset (every GPU holds the full binned matrix;
   the reference's learners share one persisted DataFrame, BaggingRegressor.scala:158-189):
   one rank ingests, exports the value codes (num_rows x row_stride x code_bytes bytes, into
   device memory of the dataset's device when codes_on_device, else host memory), the
   per-feature dictionaries (dict [dict_values], dict_off [num_features + 1]) and the labels;
   the others import them (after an RCCL broadcast of the codes, or a host copy) instead of
   re-ingesting rows.  Any of the export outputs may be NULL.  Import validates the
   dictionaries, the code width and every code on the device.                            */
int sbag_dataset_layout(const sbag_dataset* ds, int64_t* num_rows, int32_t* num_features,
                        int32_t* row_stride, int32_t* code_bytes, int64_t* dict_values);
int sbag_dataset_export(const sbag_dataset* ds, void* codes, int32_t codes_on_device, double* dict,
                        int64_t* dict_off, double* y);
int sbag_dataset_import(sbag_ctx* ctx, int64_t num_rows, int32_t num_features, int32_t row_stride,
                        int32_t code_bytes, const void* codes, int32_t codes_on_device,
                        const double* dict, const int64_t* dict_off, const double* y,
                        sbag_dataset** out);
/* datasets reference their context: free every dataset before sbag_ctx_destroy */
int sbag_dataset_free(sbag_dataset* ds);

/* ---- fit: BaggingRegressor.train / BaggingClassifier.train --------------
 * (ml/regression/BaggingRegressor.scala:121-199,
 *  ml/classification/BaggingClassifier.scala:121-199) with the base learner
 * DecisionTree{Regressor,Classifier}.fit reached through
 * HasBaseLearner.fitBaseLearner (ml/ensemble/ensembleParams.scala:99-117).     */
typedef struct {
  int32_t max_depth;              /* DecisionTree maxDepth (default 5)            */
  int32_t max_bins;               /* maxBins (default 32), 2..256                 */
  int32_t min_instances_per_node; /* default 1                                    */
  int32_t impurity;               /* SBAG_IMPURITY_*                              */
  double min_info_gain;           /* default 0.0                                  */
  int64_t seed;                   /* the base learner's seed param (HasSeed; default the
                                     class-name hashCode): seeds RandomForest.findSplits'
                                     split-finding sample of subbags > max(maxBins^2, 1e4) */
} sbag_tree_params;

typedef struct {
  sbag_sampler_params sampler;
  double subspace_ratio;       /* HasSubBag.subspaceRatio                          */
  int32_t subspace_bug_compat; /* 1: mkSubspace(getSampleRatio, ...) exactly as the
                                  reference does (BaggingRegressor.scala:174, H1)  */
  int32_t num_partitions;      /* 0 or 1 -> a single partition                    */
  const int64_t* partition_offsets; /* [num_partitions+1] or NULL                 */
  sbag_tree_params tree;
} sbag_fit_params;

int sbag_fit(sbag_ctx* ctx, sbag_dataset* ds, const sbag_fit_params* p, sbag_forest** out);

/* ---- GBM base learner: one boosting iteration's tree -----------------------
 * GBMRegressor.trainBoosters (ml/regression/GBMRegressor.scala:302-319): the subbag of
 * learner m (HasSubBag.extractSubBag of withBag's column m, HasSubBag.scala:108-126,
 * the bag drawn by sbag_sample), sliced to the booster's subspace (mkSubspace with the
 * boosting seed chain), fitted by DecisionTreeRegressor (fitBaseLearner,
 * ensembleParams.scala:99-117) on fp64 labels -- the pseudo-residuals -grad(y, F(x)).
 * Split statistics are fp64 sums in Spark's row order (DTStatsAggregator.update), so
 * trees and leaf values are those of the reference's DecisionTree on the same subbag.
 * Returns a forest of one tree (subspace = `subspace`).                           */
typedef struct {
  const uint8_t* counts;            /* host [num_rows]: the learner's bag column         */
  const int32_t* subspace;          /* the booster's feature indices, increasing          */
  int32_t subspace_len;
  int32_t num_partitions;           /* partitions of the split-finding sample (0/1: one) */
  const int64_t* partition_offsets; /* [num_partitions+1] or NULL                         */
  sbag_tree_params tree;            /* DecisionTreeRegressor params (impurity VARIANCE)   */
} sbag_booster_params;

int sbag_fit_booster(sbag_ctx* ctx, const sbag_dataset* ds, const double* labels /* host [N] */,
                     const sbag_booster_params* p, sbag_forest** out);

/* ---- forest (BaggingRegressionModel / BaggingClassificationModel fields
 *      `subspaces`, `models`, `numBaseModels`, BaggingRegressor.scala:235-246) */
typedef struct { /* DecisionTreeModelReadWrite.NodeData, pre-order ids */
  int32_t id, left, right, feature; /* feature: subspace-local index, -1 for a leaf */
  int32_t split_bin, pad_;
  double threshold, prediction, impurity, gain;
} sbag_node;

int sbag_forest_num_trees(const sbag_forest* f, int32_t* n);
/* exact_splits: 1 when the tree's thresholds are Spark's (always, since the split-finding
   sample of large subbags is replayed; kept for ABI compatibility) */
int sbag_forest_tree_info(const sbag_forest* f, int32_t t, int32_t* num_nodes, int32_t* num_stats,
                          int32_t* subspace_len, int32_t* exact_splits);
int sbag_forest_subspace(const sbag_forest* f, int32_t t, int32_t* idx_out);
int sbag_forest_nodes(const sbag_forest* f, int32_t t, sbag_node* nodes_out,
                      double* stats_out /* [num_nodes x num_stats] or NULL */);
/* rebuild a forest from node arrays (model load / JNI round trip) */
int sbag_forest_create(int32_t num_trees, const int32_t* num_nodes, const sbag_node* nodes,
                       const int32_t* subspace_len, const int32_t* subspaces, int32_t impurity,
                       sbag_forest** out);
int sbag_forest_free(sbag_forest* f);

/* device-side timing of the last fit (HIP events on the context stream) */
typedef struct {
  double total_ms, sample_ms, valuecount_ms, bin_ms, compact_ms, hist_ms, split_ms, subtract_ms;
  int64_t hist_launches;
  double hist_alg_bytes;   /* Σ over hist launches: entries x (F_r + 4)   */
  double hist_entries;     /* Σ entries processed by hist launches                    */
  double hist_upper_bytes; /* SURVEY §8d upper bound: Σ_r Σ_d inbag_r x (F_r + 4) + 3N */
  int64_t levels;
  double partition_ms;     /* k_partition: rows of split nodes -> child segments      */
  double hist_work_bytes;  /* SURVEY §8d algorithmic bytes of all histograms built:
                              Σ_(r,d) n(r,d) x (F_r + 4) + 3N, n = rows of every node
                              whose histogram exists (read or obtained by subtraction) */
  double fix_ms;           /* exact-split fallback of screened variance nodes */
  int64_t exact_fallbacks; /* nodes that needed it                                      */
  double hist_lds_atomics; /* LDS atomic wave-instructions issued by the hist launches   */
  double group_ms;         /* gini class tiles: entries regrouped by tile before the
                              histogram (k_tile_count / k_tile_scatter), not in hist_ms   */
  double chain_ms;         /* fp64 labels: the chosen features' bins summed in Spark's order
                              (routing + k_fb_chainx or k_fb_psum / k_fb_pmerge) */
  double root_ms;          /* root histogram as an int8 MFMA contraction (k_hist_mfma);
                              0 when the root went through k_hist_rl (then in hist_ms)     */
  double root_mfma_ops;    /* its int8 operations (2 x 32^3 per MFMA)                      */
} sbag_timing;
int sbag_forest_timing(const sbag_forest* f, sbag_timing* out);

/* ---- transform: PredictionModel.transform -> Bagging*Model.predict ------
 * slicer(subspace) (HasSubBag.scala:128-131) + tree walk + mean / breeze mode. */
int sbag_predict(sbag_ctx* ctx, const sbag_forest* f, const double* X, int64_t num_rows,
                 int32_t num_features, int32_t agg, double* out /* [num_rows] */,
                 double* per_tree_out /* [trees x num_rows] or NULL */);
int sbag_predict_dataset(sbag_ctx* ctx, const sbag_forest* f, const sbag_dataset* ds, int32_t agg,
                         double* out /* [num_rows] */);
/* ordered aggregation of per-learner predictions on the host:
   votes [num_learners x num_rows] fp64, learner order */
int sbag_aggregate(sbag_ctx* ctx, const double* votes, int32_t num_learners, int64_t num_rows,
                   int32_t agg, double* out);

/* ---- multi-GPU transform: device-resident outputs ----------
 * One process per GPU, each holding a learner shard [g*L/G, (g+1)*L/G) and the
 * replicated dataset.  The reference's aggregation is breeze's in-order sum / L
 * (BaggingRegressor.scala:248-256) and breeze mode (BaggingClassifier.scala:248-257);
 * across devices it becomes
 *   regression:      SBAG_OUT_SUM per rank (in-order sum of the shard's trees), an
 *                    RCCL all-to-all by row shard, then sbag_aggregate_device(MEAN) of
 *                    the G partial sums in rank order / L;
 *   classification:  SBAG_OUT_VOTES per rank ([trees x N] u8 / u16 class ids), an RCCL
 *                    all-to-all by row shard (rank order = learner order), then
 *                    sbag_aggregate_device(MODE) over all L votes of the shard's rows.
 * Pointers named d_* are device memory on the context's device (e.g. a torch tensor's
 * data_ptr()); both calls return after their work is complete on the device.       */
#define SBAG_OUT_SUM 2   /* fp64 [num_rows]: in-order sum of the forest's tree predictions */
#define SBAG_OUT_VOTES 3 /* [trees x num_rows] class ids, vote_bytes 1 (u8) or 2 (u16), or
                            vote_bytes 8: every tree's fp64 prediction (any impurity)  */
int sbag_predict_dataset_device(sbag_ctx* ctx, const sbag_forest* f, const sbag_dataset* ds,
                                int32_t out_kind, int32_t vote_bytes, void* d_out);
/* d_in [K x num_rows]: in_bytes 8 -> fp64 values, MEAN: out = (in-order sum of the K
   rows) / num_learners; in_bytes 1 / 2 -> u8 / u16 class ids < num_classes, MODE:
   breeze mode over the K votes in order.  d_out fp64 [num_rows].                   */
int sbag_aggregate_device(sbag_ctx* ctx, const void* d_in, int32_t in_bytes, int32_t K,
                          int64_t num_rows, int32_t agg, int32_t num_learners,
                          int32_t num_classes, double* d_out);

#ifdef __cplusplus
}
#endif
#endif
