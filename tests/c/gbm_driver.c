/* gbm_driver.c -- GBMRegressor's boosting loop (ml/regression/GBMRegressor.scala:286-397,
 * squared loss, optimizedWeights = false, no validation) driven from plain C through the
 * JNI shim's core in SbagNative's argument order: sample -> per
 * iteration fitBooster on the residuals -> forestNodes -> predict the booster ->
 * current += prediction * learningRate.  The subspaces come from the caller (the
 * reference's mkSubspace seed chain, computed by the JVM side).
 *
 * usage: gbm_driver data.bin subs.bin out.bin L learningRate replacement sampleRatio seed
 *                   depth bins treeSeed
 * data.bin: int64 N, int64 F, f64 X[N*F], f64 y[N]
 * subs.bin: per iteration int32 len, int32 idx[len]
 * out.bin:  int32 status; when 0: per iteration {int32 nn, f64 nodes[nn*8]}, f64 F(x)[N]
 * Built by __graft_entry__.build() (tests/c/Makefile); run by tests/test_gpu_c_abi.py. */
#include <stdio.h>
#include <stdlib.h>

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
  if (argc != 12) {
    fprintf(stderr, "usage: %s data.bin subs.bin out.bin L learningRate replacement sampleRatio "
                    "seed depth bins treeSeed\n", argv[0]);
    return 2;
  }
  size_t len = 0, slen = 0;
  char* buf = (char*)read_all(argv[1], &len);
  char* sbuf = (char*)read_all(argv[2], &slen);
  if (!buf || !sbuf || len < 16) return 2;
  const int64_t N = ((const int64_t*)buf)[0], F = ((const int64_t*)buf)[1];
  const double* X = (const double*)(buf + 16);
  const double* y = X + N * F;
  if ((size_t)((const char*)(y + N) - buf) != len) return 2;
  const int32_t L = atoi(argv[4]);
  const double lr = atof(argv[5]);
  const int replacement = atoi(argv[6]);
  const double ratio = atof(argv[7]);
  const int64_t seed = strtoll(argv[8], NULL, 10);
  const int32_t depth = atoi(argv[9]), bins = atoi(argv[10]);
  const int64_t tree_seed = strtoll(argv[11], NULL, 10);
  FILE* out = fopen(argv[3], "wb");
  if (!out) return 2;
  int64_t ctx = 0, ds = 0;
  int st = sbagb_ctx_create(0, &ctx);
  if (st) return fail_out(out, st, "ctxCreate");
  st = sbagb_dataset_create(ctx, N, (int32_t)F, X, y, &ds);
  if (st) return fail_out(out, st, "datasetCreate");
  const int64_t off[2] = {0, N};
  uint8_t* bags = (uint8_t*)malloc((size_t)L * (size_t)N);
  st = sbagb_sample(ctx, replacement, ratio, seed, 0, L, off, 2, N, bags);
  if (st) return fail_out(out, st, "sample");
  double* cur = (double*)calloc((size_t)N, sizeof(double)); /* BLAS.dot running sum */
  double* res = (double*)malloc(sizeof(double) * (size_t)N);
  double* pred = (double*)malloc(sizeof(double) * (size_t)N);
  int32_t zero = 0;
  fwrite(&zero, 4, 1, out);
  const char* sp = sbuf;
  for (int32_t m = 0; m < L; m++) {
    const int32_t sl = *(const int32_t*)sp;
    const int32_t* sub = (const int32_t*)(sp + 4);
    sp += 4 + 4 * (size_t)sl;
    for (int64_t i = 0; i < N; i++) res[i] = -(-(y[i] - (cur[i] + 0.0))); /* -grad, const 0 */
    int64_t forest = 0;
    st = sbagb_fit_booster(ctx, ds, res, bags + (size_t)m * N, sub, sl, off, 2, depth, bins, 1,
                           0.0, tree_seed, &forest);
    if (st) return fail_out(out, st, "fitBooster");
    int32_t nn = 0, sl2 = 0;
    st = sbagb_forest_size(forest, 0, &nn, &sl2);
    double* packed = (double*)malloc(sizeof(double) * 8 * (size_t)nn);
    if (!st) st = sbagb_forest_nodes(forest, 0, packed);
    if (!st) st = sbagb_predict(ctx, forest, X, N, (int32_t)F, SBAG_AGG_MEAN, pred);
    if (st) return fail_out(out, st, "boosterPredict");
    fwrite(&nn, 4, 1, out);
    fwrite(packed, 8, 8 * (size_t)nn, out);
    free(packed);
    for (int64_t i = 0; i < N; i++) cur[i] = cur[i] + pred[i] * (lr * 1.0);
    sbagb_forest_free(forest);
  }
  for (int64_t i = 0; i < N; i++) pred[i] = cur[i] + 0.0;
  fwrite(pred, 8, (size_t)N, out);
  fclose(out);
  sbagb_dataset_free(ds);
  sbagb_ctx_destroy(ctx);
  free(bags);
  free(cur);
  free(res);
  free(pred);
  free(buf);
  free(sbuf);
  printf("ok: %d boosters, %lld predictions\n", L, (long long)N);
  return 0;
}
