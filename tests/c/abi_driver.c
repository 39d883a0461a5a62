/* abi_driver.c -- drives libsbag from plain C through the JNI shim's core
 * (integration/sbagjni_core.c), in the argument order SbagNative's @native methods
 * use: ctxCreate -> datasetCreate -> fit(..., treeSeed) ->
 * forestNodes / forestSubspace -> predict -> free.  No ctypes: the struct layouts
 * and argument order are the C compiler's, as in the JNI library.
 *
 * usage: abi_driver data.bin out.bin replacement ratio seed lb le subRatio bugCompat
 *                   depth bins minInst impurity minGain treeSeed agg
 * data.bin: int64 N, int64 F, int64 num_offsets, int64 offsets[], f64 X[N*F], f64 y[N]
 * out.bin:  int32 status; when 0: int32 T, per tree {int32 nn, int32 sl, f64 nodes[nn*8],
 *           int32 sub[sl]}, f64 pred[N].  On failure stdout names the exception class
 *           the JNI shim would throw and sbag_last_error().
 * Built by __graft_entry__.build() (tests/c/Makefile); run by tests/test_gpu_c_abi.py. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sbag.h"
#include "sbagjni_core.h"

static void* read_all(const char* path, size_t* len) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *len = (size_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  void* b = malloc(*len ? *len : 1);
  if (fread(b, 1, *len, f) != *len) {
    free(b);
    b = NULL;
  }
  fclose(f);
  return b;
}

static int fail_out(FILE* out, int st, const char* where) {
  printf("%s: status=%d exception=%s message=%s\n", where, st, sbagb_exception_class(st),
         sbag_last_error());
  int32_t s = st;
  fwrite(&s, 4, 1, out);
  fclose(out);
  return 3;
}

int main(int argc, char** argv) {
  if (argc != 17) {
    fprintf(stderr, "usage: %s data.bin out.bin replacement ratio seed lb le subRatio bugCompat "
                    "depth bins minInst impurity minGain treeSeed agg\n", argv[0]);
    return 2;
  }
  size_t len = 0;
  char* buf = (char*)read_all(argv[1], &len);
  if (!buf || len < 24) return 2;
  const int64_t* h = (const int64_t*)buf;
  const int64_t N = h[0], F = h[1], np1 = h[2];
  const int64_t* offsets = h + 3;
  const double* X = (const double*)(offsets + np1);
  const double* y = X + N * F;
  if ((size_t)((const char*)(y + N) - buf) != len) return 2;
  const int replacement = atoi(argv[3]);
  const double ratio = atof(argv[4]);
  const int64_t seed = strtoll(argv[5], NULL, 10);
  const int32_t lb = atoi(argv[6]), le = atoi(argv[7]);
  const double sub_ratio = atof(argv[8]);
  const int bug_compat = atoi(argv[9]);
  const int32_t depth = atoi(argv[10]), bins = atoi(argv[11]), min_inst = atoi(argv[12]);
  const int32_t impurity = atoi(argv[13]);
  const double min_gain = atof(argv[14]);
  const int64_t tree_seed = strtoll(argv[15], NULL, 10);
  const int32_t agg = atoi(argv[16]);

  FILE* out = fopen(argv[2], "wb");
  if (!out) return 2;
  int64_t ctx = 0, ds = 0, forest = 0;
  int st = sbagb_ctx_create(0, &ctx);
  if (st) return fail_out(out, st, "ctxCreate");
  st = sbagb_dataset_create(ctx, N, (int32_t)F, X, y, &ds);
  if (st) return fail_out(out, st, "datasetCreate");
  st = sbagb_fit(ctx, ds, replacement, ratio, seed, lb, le, sub_ratio, bug_compat, offsets,
                 (int32_t)np1, depth, bins, min_inst, impurity, min_gain, tree_seed, &forest);
  if (st) return fail_out(out, st, "fit");
  int32_t zero = 0, T = le - lb;
  fwrite(&zero, 4, 1, out);
  fwrite(&T, 4, 1, out);
  for (int32_t t = 0; t < T; t++) {
    int32_t nn = 0, sl = 0;
    st = sbagb_forest_size(forest, t, &nn, &sl);
    if (st) return fail_out(out, st, "forestSize");
    double* packed = (double*)malloc(sizeof(double) * 8 * (size_t)nn);
    int32_t* sub = (int32_t*)malloc(sizeof(int32_t) * (size_t)(sl > 0 ? sl : 1));
    st = sbagb_forest_nodes(forest, t, packed);
    if (!st) st = sbagb_forest_subspace(forest, t, sub);
    if (st) return fail_out(out, st, "forestNodes");
    fwrite(&nn, 4, 1, out);
    fwrite(&sl, 4, 1, out);
    fwrite(packed, 8, 8 * (size_t)nn, out);
    fwrite(sub, 4, (size_t)sl, out);
    free(packed);
    free(sub);
  }
  double* pred = (double*)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
  st = sbagb_predict(ctx, forest, X, N, (int32_t)F, agg, pred);
  if (st) return fail_out(out, st, "predict");
  fwrite(pred, 8, (size_t)N, out);
  fclose(out);
  free(pred);
  sbagb_forest_free(forest);
  sbagb_dataset_free(ds);
  sbagb_ctx_destroy(ctx);
  free(buf);
  printf("ok: %d trees, %lld predictions\n", T, (long long)N);
  return 0;
}
