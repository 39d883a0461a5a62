/* sbagjni_core.c -- see sbagjni_core.h.  Plain C over include/sbag.h. */
#include "sbagjni_core.h"

#include <stdint.h>
#include <stdlib.h>

#include "sbag.h"

#define CTX(h) ((sbag_ctx*)(intptr_t)(h))
#define DS(h) ((sbag_dataset*)(intptr_t)(h))
#define FOREST(h) ((sbag_forest*)(intptr_t)(h))

const char* sbagb_exception_class(int status) {
  return status == SBAG_EINVAL ? "java/lang/IllegalArgumentException"
                               : "org/apache/spark/SparkException";
}

int sbagb_ctx_create(int32_t device, int64_t* ctx_out) {
  sbag_ctx* c = NULL;
  const int st = sbag_ctx_create(device, &c);
  *ctx_out = (int64_t)(intptr_t)c;
  return st;
}

int sbagb_ctx_destroy(int64_t ctx) { return sbag_ctx_destroy(CTX(ctx)); }

int sbagb_dataset_create(int64_t ctx, int64_t n, int32_t f, const double* X, const double* y,
                         int64_t* ds_out) {
  sbag_dataset* ds = NULL;
  const int st = sbag_dataset_create(CTX(ctx), n, f, X, y, &ds);
  *ds_out = (int64_t)(intptr_t)ds;
  return st;
}

int sbagb_dataset_free(int64_t ds) { return sbag_dataset_free(DS(ds)); }

int sbagb_fit(int64_t ctx, int64_t ds, int replacement, double sample_ratio, int64_t seed,
              int32_t learner_begin, int32_t learner_end, double subspace_ratio, int bug_compat,
              const int64_t* partition_offsets, int32_t num_offsets, int32_t max_depth,
              int32_t max_bins, int32_t min_instances_per_node, int32_t impurity,
              double min_info_gain, int64_t tree_seed, int64_t* forest_out) {
  sbag_fit_params p = {0};
  p.sampler.replacement = replacement ? 1 : 0;
  p.sampler.sample_ratio = sample_ratio;
  p.sampler.seed = seed;
  p.sampler.learner_begin = learner_begin;
  p.sampler.learner_end = learner_end;
  p.subspace_ratio = subspace_ratio;
  p.subspace_bug_compat = bug_compat ? 1 : 0;
  p.num_partitions = num_offsets > 0 ? num_offsets - 1 : 0;
  p.partition_offsets = num_offsets > 0 ? partition_offsets : NULL;
  p.tree.max_depth = max_depth;
  p.tree.max_bins = max_bins;
  p.tree.min_instances_per_node = min_instances_per_node;
  p.tree.impurity = impurity;
  p.tree.min_info_gain = min_info_gain;
  p.tree.seed = tree_seed;
  sbag_forest* f = NULL;
  const int st = sbag_fit(CTX(ctx), DS(ds), &p, &f);
  *forest_out = (int64_t)(intptr_t)f;
  return st;
}

int sbagb_forest_size(int64_t forest, int32_t t, int32_t* num_nodes, int32_t* subspace_len) {
  return sbag_forest_tree_info(FOREST(forest), t, num_nodes, NULL, subspace_len, NULL);
}

int sbagb_forest_nodes(int64_t forest, int32_t t, double* packed_out) {
  int32_t nn = 0;
  int st = sbag_forest_tree_info(FOREST(forest), t, &nn, NULL, NULL, NULL);
  if (st) return st;
  sbag_node* nodes = (sbag_node*)malloc(sizeof(sbag_node) * (size_t)(nn > 0 ? nn : 1));
  if (!nodes) return SBAG_ENOMEM;
  st = sbag_forest_nodes(FOREST(forest), t, nodes, NULL);
  for (int32_t i = 0; st == SBAG_OK && i < nn; i++) {
    double* o = packed_out + 8 * (int64_t)i;
    o[0] = nodes[i].id;
    o[1] = nodes[i].left;
    o[2] = nodes[i].right;
    o[3] = nodes[i].feature;
    o[4] = nodes[i].threshold;
    o[5] = nodes[i].prediction;
    o[6] = nodes[i].impurity;
    o[7] = nodes[i].gain;
  }
  free(nodes);
  return st;
}

int sbagb_forest_subspace(int64_t forest, int32_t t, int32_t* idx_out) {
  return sbag_forest_subspace(FOREST(forest), t, idx_out);
}

int sbagb_forest_free(int64_t forest) { return sbag_forest_free(FOREST(forest)); }

int sbagb_predict(int64_t ctx, int64_t forest, const double* X, int64_t n, int32_t f, int32_t agg,
                  double* out) {
  return sbag_predict(CTX(ctx), FOREST(forest), X, n, f, agg, out, NULL);
}

int sbagb_dataset_create_csr(int64_t ctx, int64_t n, int32_t f, const int64_t* indptr,
                             const int32_t* indices, const double* values, const double* y,
                             int64_t* ds_out) {
  sbag_dataset* ds = NULL;
  const int st = sbag_dataset_create_csr(CTX(ctx), n, f, indptr, indices, values, y, &ds);
  *ds_out = (int64_t)(intptr_t)ds;
  return st;
}

int sbagb_sample(int64_t ctx, int replacement, double sample_ratio, int64_t seed,
                 int32_t learner_begin, int32_t learner_end, const int64_t* partition_offsets,
                 int32_t num_offsets, int64_t n, uint8_t* counts_out) {
  sbag_sampler_params p;
  p.replacement = replacement ? 1 : 0;
  p.pad_ = 0;
  p.sample_ratio = sample_ratio;
  p.seed = seed;
  p.learner_begin = learner_begin;
  p.learner_end = learner_end;
  return sbag_sample(CTX(ctx), &p, partition_offsets, num_offsets - 1, n, counts_out);
}

int sbagb_fit_booster(int64_t ctx, int64_t ds, const double* labels, const uint8_t* counts,
                      const int32_t* subspace, int32_t subspace_len,
                      const int64_t* partition_offsets, int32_t num_offsets, int32_t max_depth,
                      int32_t max_bins, int32_t min_instances_per_node, double min_info_gain,
                      int64_t tree_seed, int64_t* forest_out) {
  sbag_booster_params p;
  p.counts = counts;
  p.subspace = subspace;
  p.subspace_len = subspace_len;
  p.num_partitions = num_offsets - 1;
  p.partition_offsets = partition_offsets;
  p.tree.max_depth = max_depth;
  p.tree.max_bins = max_bins;
  p.tree.min_instances_per_node = min_instances_per_node;
  p.tree.impurity = SBAG_IMPURITY_VARIANCE;
  p.tree.min_info_gain = min_info_gain;
  p.tree.seed = tree_seed;
  sbag_forest* f = NULL;
  const int st = sbag_fit_booster(CTX(ctx), DS(ds), labels, &p, &f);
  *forest_out = (int64_t)(intptr_t)f;
  return st;
}
