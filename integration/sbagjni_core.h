/*
 * sbagjni_core.h -- the C core of the JNI shim shown in INTEGRATION.md §2.
 *
 * Every function takes its arguments in exactly the order of the Scala
 * `SbagNative` @native method it backs, with the JVM types mapped to C:
 * jlong -> int64_t (handles are sbag pointers cast to jlong), jint -> int32_t,
 * jboolean -> int, jdouble -> double, jdoubleArray / jlongArray -> pointer + length.
 * The JNI functions only pin arrays, call these, and turn a non-zero status into
 * the exception sbagb_exception_class() names.  tests/c/abi_driver.c drives them
 * from plain C (no ctypes) so the argument order the shim uses is tested.
 */
#ifndef SBAGJNI_CORE_H
#define SBAGJNI_CORE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* JVM class of the exception for a status (sbag.h conventions):
   SBAG_EINVAL -> java/lang/IllegalArgumentException (bfunctions.scala:52,59;
   HasSubBag.scala:57,74), anything else -> org/apache/spark/SparkException
   (HasSubBag.scala:141, ThreadUtils.awaitResult at BaggingRegressor.scala:191). */
const char* sbagb_exception_class(int status);

/* SbagNative.ctxCreate(device: Int): Long */
int sbagb_ctx_create(int32_t device, int64_t* ctx_out);
/* SbagNative.ctxDestroy(ctx: Long): Unit */
int sbagb_ctx_destroy(int64_t ctx);
/* SbagNative.datasetCreate(ctx: Long, n: Long, f: Int, X: Array[Double], y: Array[Double]): Long */
int sbagb_dataset_create(int64_t ctx, int64_t n, int32_t f, const double* X, const double* y,
                         int64_t* ds_out);
/* SbagNative.datasetFree(ds: Long): Unit */
int sbagb_dataset_free(int64_t ds);
/* SbagNative.fit(ctx, ds, replacement, sampleRatio, seed, learnerBegin, learnerEnd,
 *                subspaceRatio, bugCompat, partitionOffsets, maxDepth, maxBins,
 *                minInstancesPerNode, impurity, minInfoGain, treeSeed): Long
 * treeSeed is the base learner's HasSeed value (dt.getSeed): it seeds
 * RandomForest.findSplits' split-finding sample of every subbag > max(maxBins^2, 1e4) rows. */
int sbagb_fit(int64_t ctx, int64_t ds, int replacement, double sample_ratio, int64_t seed,
              int32_t learner_begin, int32_t learner_end, double subspace_ratio, int bug_compat,
              const int64_t* partition_offsets, int32_t num_offsets, int32_t max_depth,
              int32_t max_bins, int32_t min_instances_per_node, int32_t impurity,
              double min_info_gain, int64_t tree_seed, int64_t* forest_out);
/* sizes for the JVM arrays of SbagNative.forestNodes / forestSubspace */
int sbagb_forest_size(int64_t forest, int32_t t, int32_t* num_nodes, int32_t* subspace_len);
/* SbagNative.forestNodes(forest: Long, t: Int): Array[Double] -- 8 doubles per node:
   id, left, right, feature, threshold, prediction, impurity, gain (pre-order) */
int sbagb_forest_nodes(int64_t forest, int32_t t, double* packed_out);
/* SbagNative.forestSubspace(forest: Long, t: Int): Array[Int] */
int sbagb_forest_subspace(int64_t forest, int32_t t, int32_t* idx_out);
/* SbagNative.forestFree(forest: Long): Unit */
int sbagb_forest_free(int64_t forest);
/* SbagNative.predict(ctx, forest, X: Array[Double], n: Long, f: Int, agg: Int): Array[Double] */
int sbagb_predict(int64_t ctx, int64_t forest, const double* X, int64_t n, int32_t f, int32_t agg,
                  double* out);

/* SbagNative.datasetCreateCsr(ctx, n, f, indptr: Array[Long], indices: Array[Int],
 *                             values: Array[Double], y: Array[Double]): Long
 * SparseVector rows, Spark semantics (absent entries are 0.0) -- sbag_dataset_create_csr */
int sbagb_dataset_create_csr(int64_t ctx, int64_t n, int32_t f, const int64_t* indptr,
                             const int32_t* indices, const double* values, const double* y,
                             int64_t* ds_out);
/* SbagNative.sample(ctx, replacement, sampleRatio, seed, learnerBegin, learnerEnd,
 *                   partitionOffsets, n): Array[Byte] -- withBag's counts
 * (bfunctions.bag, sql/bfunctions.scala:46-68), [learners x n] */
int sbagb_sample(int64_t ctx, int replacement, double sample_ratio, int64_t seed,
                 int32_t learner_begin, int32_t learner_end, const int64_t* partition_offsets,
                 int32_t num_offsets, int64_t n, uint8_t* counts_out);
/* SbagNative.fitBooster(ctx, ds, labels, counts, subspace, partitionOffsets, maxDepth,
 *                       maxBins, minInstancesPerNode, minInfoGain, treeSeed): Long
 * one GBM booster (GBMRegressor.scala:311-319): DecisionTreeRegressor on the subbag
 * `counts` sliced to `subspace`, fp64 labels -- sbag_fit_booster */
int sbagb_fit_booster(int64_t ctx, int64_t ds, const double* labels, const uint8_t* counts,
                      const int32_t* subspace, int32_t subspace_len,
                      const int64_t* partition_offsets, int32_t num_offsets, int32_t max_depth,
                      int32_t max_bins, int32_t min_instances_per_node, double min_info_gain,
                      int64_t tree_seed, int64_t* forest_out);

#ifdef __cplusplus
}
#endif
#endif
