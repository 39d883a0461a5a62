/* sanitize_main.c -- runs the oracle's whole path under AddressSanitizer + UBSan
 * (oracle/Makefile `san`; tests/test_oracle_sanitized.py).  TEST INFRASTRUCTURE.
 * Exercises RNG primitives, bag (Poisson, Bernoulli, all-ones), subspace, split
 * finding with and without the split-finding sample, variance and gini fits with
 * several depths / bin counts / partitionings, and both aggregations. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sbag_oracle.h"

static int run_case(int64_t N, int F, int C, int L, int depth, int bins, int replacement,
                    double ratio, int P, int threads) {
  uint8_t* X8 = malloc((size_t)N * F);
  double* X = malloc(sizeof(double) * (size_t)N * F);
  double* y = malloc(sizeof(double) * (size_t)N);
  or_synth(0, N, F, 99 + (uint64_t)N, C, threads, X8, y);
  for (int64_t i = 0; i < N * F; i++) X[i] = (double)X8[i] * 0.5 - 3.0;  /* negatives, zeros */
  int64_t* off = malloc(sizeof(int64_t) * (size_t)(P + 1));
  for (int p = 0; p <= P; p++) off[p] = N * p / P;
  uint8_t* counts = malloc((size_t)L * N);
  const int64_t seed = C ? 42087812 : -1395689524;
  if (or_bag(replacement, ratio, 0, L, seed, off, P, N, counts)) return 1;
  int32_t* sub = malloc(sizeof(int32_t) * (size_t)L * F);
  int32_t* nsub = malloc(sizeof(int32_t) * (size_t)L);
  for (int l = 0; l < L; l++) {
    if (or_subspace(ratio, F, seed + l, sub + (int64_t)l * F, &nsub[l])) return 2;
    if (nsub[l] == 0) {  /* mkSubspace drew nothing: use feature 0 for the sanitizer run */
      sub[(int64_t)l * F] = 0;
      nsub[l] = 1;
    }
  }
  or_tree_params tp = {depth, bins, 1, C ? 1 : 0, 0.0, 926680331, off, P, 0};
  const int max_nodes = (1 << (depth + 1)) + 1, stride = C ? C : 3;
  or_node* nodes = calloc((size_t)L * max_nodes, sizeof(or_node));
  double* stats = calloc((size_t)L * max_nodes * stride, sizeof(double));
  int32_t *nn = calloc(L, 4), *ns = calloc(L, 4), *ex = calloc(L, 4);
  const int rc = or_fit(X, y, N, F, counts, L, sub, nsub, &tp, threads, nodes, max_nodes, stats,
                        stride, nn, ns, ex);
  if (rc && rc != -3) {  /* -3: a learner's bag is empty (legitimate for tiny cases) */
    fprintf(stderr, "or_fit rc=%d\n", rc);
    return 3;
  }
  double* out = malloc(sizeof(double) * (size_t)N);
  double* pt = malloc(sizeof(double) * (size_t)N * L);
  if (!rc) or_predict(X, N, F, L, sub, nsub, nodes, max_nodes, C ? 1 : 0, out, pt);
  double thr[256];
  int exact = 0;
  or_find_splits(X, N, F, F - 1, counts, bins, thr, &exact);
  free(X8); free(X); free(y); free(off); free(counts); free(sub); free(nsub); free(nodes);
  free(stats); free(nn); free(ns); free(ex); free(out); free(pt);
  return 0;
}

int main(void) {
  int32_t ibuf[64];
  double dbuf[64];
  or_xorshift_next(-1, 32, 64, ibuf);
  or_xorshift_doubles(12345, 64, dbuf);
  or_well_next(-1395689524, 32, 64, ibuf);
  or_well_doubles(7, 64, dbuf);
  or_poisson(1.0, 99, 64, ibuf);
  or_poisson(0.0005, 3, 64, ibuf);
  uint8_t key[256];
  for (int i = 0; i < 256; i++) key[i] = (uint8_t)i;
  volatile uint32_t h = 0;
  for (int i = 0; i <= 256; i++) h ^= or_mm3_bytes_hash(key, i, 256 - i);
  const struct { int64_t N; int F, C, L, depth, bins, repl; double ratio; int P, thr; } cs[] = {
      {3000, 7, 0, 3, 6, 32, 1, 1.0, 3, 2},   {3000, 9, 5, 4, 5, 8, 1, 0.7, 1, 1},
      {20000, 5, 0, 2, 4, 16, 1, 1.0, 2, 4},  /* split-finding sample (> 1e4 rows) */
      {2500, 6, 3, 3, 7, 2, 0, 0.5, 4, 2},    {1200, 12, 0, 2, 0, 64, 0, 1.0, 1, 1},
      {4000, 10, 64, 2, 9, 32, 0, 0.5, 5, 3}, {17, 3, 2, 2, 3, 4, 1, 0.8, 4, 1},
  };
  for (size_t k = 0; k < sizeof(cs) / sizeof(cs[0]); k++) {
    const int rc = run_case(cs[k].N, cs[k].F, cs[k].C, cs[k].L, cs[k].depth, cs[k].bins,
                            cs[k].repl, cs[k].ratio, cs[k].P, cs[k].thr);
    if (rc) {
      fprintf(stderr, "case %zu failed rc=%d\n", k, rc);
      return rc;
    }
  }
  printf("oracle sanitizer run ok (%u)\n", (unsigned)h);
  return 0;
}
