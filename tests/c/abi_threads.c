#define _POSIX_C_SOURCE 200809L
/* abi_threads.c -- concurrent calls into libsbag through the JNI shim's core, as the
 * reference's CrossValidator.setParallelism(4) makes them (BaggingRegressorSuite.scala:38-43:
 * four estimators fitted at once from a JVM thread pool, each calling SbagNative.fit and
 * SbagNative.predict).  SURVEY §8b asks for a reentrant ABI: a per-context lock
 * (sbag_host.cpp) serialises calls on a shared context, separate contexts run side by side,
 * and sbag_last_error() is per thread.
 *
 * usage: abi_threads data.bin seed depth bins impurity agg [modes]
 *   modes: comma-separated subset of shared,separate,errors-shared,errors-separate (default all),
 *          or setup-only (threads create and destroy a context and a dataset, no fit)
 * data.bin: as tests/c/abi_driver.c (int64 N, F, num_offsets, offsets[], f64 X[N*F], y[N]).
 *
 * Four jobs (learner ranges [4j, 4j + 4) with subspace ratio 0.7 and Poisson bags) are first
 * fitted and predicted one after another on one context: the reference results.  Then:
 *   shared:   four threads, one context and one dataset, every job at once;
 *   separate: four threads, each with its own context and dataset;
 *   errors:   thread 0 passes sampleRatio 1.5 (SBAG_EINVAL) while threads 1-3 fit; thread
 *             0's sbag_last_error() names the ratio, the others' stay empty.
 * Every concurrent forest (all node fields, subspaces) and prediction must equal the serial
 * one byte for byte.  Prints "ok ..." per mode and exits 0, else prints what differed and
 * exits 1.  Built by tests/c/Makefile (also under host ASan); run by
 * tests/test_gpu_c_abi.py. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "sbag.h"
#include "sbagjni_core.h"

#define NJOBS 4
#define LPJ 4 /* learners per job */

static int64_t N, F, NOFF;
static const int64_t* OFFS;
static const double *X, *Y;
static int64_t SEED;
static int32_t DEPTH, BINS, IMPURITY, AGG;

typedef struct {
  int status;
  int32_t T;
  int32_t nn[LPJ], sl[LPJ];
  double* nodes[LPJ];
  int32_t* sub[LPJ];
  double* pred;
  char err[512];
} result_t;

typedef struct {
  int job;
  int64_t ctx, ds;   /* shared handles, or 0: create own */
  double ratio;      /* sampleRatio (1.5: the induced SBAG_EINVAL) */
  pthread_barrier_t* bar;
  result_t res;
} job_t;

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

static void free_result(result_t* r) {
  for (int t = 0; t < LPJ; t++) {
    free(r->nodes[t]);
    free(r->sub[t]);
  }
  free(r->pred);
  memset(r, 0, sizeof(*r));
}

/* fit job j and predict every row; the status and this thread's last error are recorded */
static void run_job(int j, int64_t ctx, int64_t ds, double ratio, result_t* r) {
  memset(r, 0, sizeof(*r));
  int64_t forest = 0;
  r->status = sbagb_fit(ctx, ds, 1, ratio, SEED, j * LPJ, (j + 1) * LPJ, 0.7, 1, OFFS, (int32_t)NOFF, DEPTH,
                        BINS, 1, IMPURITY, 0.0, IMPURITY == SBAG_IMPURITY_GINI ? 42087812LL : -1395689524LL,
                        &forest);
  snprintf(r->err, sizeof(r->err), "%s", sbag_last_error());
  if (r->status) return;
  r->T = LPJ;
  for (int t = 0; t < LPJ && !r->status; t++) {
    r->status = sbagb_forest_size(forest, t, &r->nn[t], &r->sl[t]);
    if (r->status) break;
    r->nodes[t] = (double*)malloc(sizeof(double) * 8 * (size_t)r->nn[t]);
    r->sub[t] = (int32_t*)malloc(sizeof(int32_t) * (size_t)(r->sl[t] > 0 ? r->sl[t] : 1));
    r->status = sbagb_forest_nodes(forest, t, r->nodes[t]);
    if (!r->status) r->status = sbagb_forest_subspace(forest, t, r->sub[t]);
  }
  if (!r->status) {
    r->pred = (double*)malloc(sizeof(double) * (size_t)N);
    r->status = sbagb_predict(ctx, forest, X, N, (int32_t)F, AGG, r->pred);
  }
  if (r->status) snprintf(r->err, sizeof(r->err), "%s", sbag_last_error());
  sbagb_forest_free(forest);
}

static void* setup_only_main(void* arg) {
  job_t* jb = (job_t*)arg;
  int64_t ctx = 0, ds = 0;
  pthread_barrier_wait(jb->bar);
  jb->res.status = sbagb_ctx_create(0, &ctx);
  if (!jb->res.status) jb->res.status = sbagb_dataset_create(ctx, N, (int32_t)F, X, Y, &ds);
  if (ds) sbagb_dataset_free(ds);
  if (ctx) sbagb_ctx_destroy(ctx);
  return NULL;
}

static void* thread_main(void* arg) {
  job_t* jb = (job_t*)arg;
  int64_t ctx = jb->ctx, ds = jb->ds;
  int own = 0;
  if (!ctx) {
    own = 1;
    int st = sbagb_ctx_create(0, &ctx);
    if (!st) st = sbagb_dataset_create(ctx, N, (int32_t)F, X, Y, &ds);
    if (st) {
      jb->res.status = st;
      snprintf(jb->res.err, sizeof(jb->res.err), "setup: %s", sbag_last_error());
      pthread_barrier_wait(jb->bar);
      return NULL;
    }
  }
  pthread_barrier_wait(jb->bar); /* every job's call starts together */
  run_job(jb->job, ctx, ds, jb->ratio, &jb->res);
  if (own) {
    sbagb_dataset_free(ds);
    sbagb_ctx_destroy(ctx);
  }
  return NULL;
}

static int same(const result_t* a, const result_t* b, const char* mode, int j) {
  if (a->status || b->status) {
    printf("%s job %d: status %d / %d (%s / %s)\n", mode, j, a->status, b->status, a->err, b->err);
    return 0;
  }
  for (int t = 0; t < LPJ; t++) {
    if (a->nn[t] != b->nn[t] || a->sl[t] != b->sl[t] ||
        memcmp(a->nodes[t], b->nodes[t], sizeof(double) * 8 * (size_t)a->nn[t]) ||
        memcmp(a->sub[t], b->sub[t], sizeof(int32_t) * (size_t)a->sl[t])) {
      printf("%s job %d: tree %d differs from the serial fit\n", mode, j, t);
      return 0;
    }
  }
  if (memcmp(a->pred, b->pred, sizeof(double) * (size_t)N)) {
    printf("%s job %d: predictions differ from the serial run\n", mode, j);
    return 0;
  }
  return 1;
}

/* run the four jobs on threads; shared handles when ctx != 0 */
static int concurrent(const char* mode, int64_t ctx, int64_t ds, const double* ratios, result_t* serial) {
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, NJOBS);
  job_t jobs[NJOBS];
  pthread_t th[NJOBS];
  for (int j = 0; j < NJOBS; j++) {
    memset(&jobs[j], 0, sizeof(jobs[j]));
    jobs[j].job = j;
    jobs[j].ctx = ctx;
    jobs[j].ds = ds;
    jobs[j].ratio = ratios[j];
    jobs[j].bar = &bar;
    pthread_create(&th[j], NULL, thread_main, &jobs[j]);
  }
  for (int j = 0; j < NJOBS; j++) pthread_join(th[j], NULL);
  pthread_barrier_destroy(&bar);
  int ok = 1;
  for (int j = 0; j < NJOBS; j++) {
    if (ratios[j] > 1.0) { /* the induced failure: its own thread's error, nobody else's */
      if (jobs[j].res.status != SBAG_EINVAL || !strstr(jobs[j].res.err, "atio")) {
        printf("%s job %d: expected SBAG_EINVAL naming the ratio, got %d '%s'\n", mode, j, jobs[j].res.status,
               jobs[j].res.err);
        ok = 0;
      } else {
        printf("%s job %d: %s (%s)\n", mode, j, sbagb_exception_class(jobs[j].res.status), jobs[j].res.err);
      }
    } else {
      if (jobs[j].res.err[0]) {
        printf("%s job %d: another thread's error leaked into this one: '%s'\n", mode, j, jobs[j].res.err);
        ok = 0;
      }
      ok &= same(&jobs[j].res, &serial[j], mode, j);
    }
    free_result(&jobs[j].res);
  }
  if (ok) printf("ok %s: %d concurrent jobs equal to the serial fits\n", mode, NJOBS);
  return ok;
}

/* is `m` one of the comma-separated names in `list`? */
static int has_mode(const char* list, const char* m) {
  const size_t n = strlen(m);
  for (const char* p = list; p && *p;) {
    const char* e = strchr(p, ',');
    const size_t k = e ? (size_t)(e - p) : strlen(p);
    if (k == n && !strncmp(p, m, n)) return 1;
    p = e ? e + 1 : NULL;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 7 && argc != 8) {
    fprintf(stderr, "usage: %s data.bin seed depth bins impurity agg [modes]\n", argv[0]);
    return 2;
  }
  setvbuf(stdout, NULL, _IOLBF, 0); /* (each verdict line out before any teardown) */
  const char* modes = argc == 8 ? argv[7] : "shared,separate,errors-shared,errors-separate";
  size_t len = 0;
  char* buf = (char*)read_all(argv[1], &len);
  if (!buf || len < 24) return 2;
  const int64_t* h = (const int64_t*)buf;
  N = h[0];
  F = h[1];
  NOFF = h[2];
  OFFS = h + 3;
  X = (const double*)(OFFS + NOFF);
  Y = X + N * F;
  if ((size_t)((const char*)(Y + N) - buf) != len) return 2;
  SEED = strtoll(argv[2], NULL, 10);
  DEPTH = atoi(argv[3]);
  BINS = atoi(argv[4]);
  IMPURITY = atoi(argv[5]);
  AGG = atoi(argv[6]);

  int64_t ctx = 0, ds = 0;
  if (sbagb_ctx_create(0, &ctx) || sbagb_dataset_create(ctx, N, (int32_t)F, X, Y, &ds)) {
    printf("setup failed: %s\n", sbag_last_error());
    return 1;
  }
  result_t serial[NJOBS];
  for (int j = 0; j < NJOBS; j++) {
    run_job(j, ctx, ds, 0.8, &serial[j]);
    if (serial[j].status) {
      printf("serial job %d failed: %d %s\n", j, serial[j].status, serial[j].err);
      return 1;
    }
  }
  const double good[NJOBS] = {0.8, 0.8, 0.8, 0.8};
  const double bad0[NJOBS] = {1.5, 0.8, 0.8, 0.8};
  int ok = 1;
  if (has_mode(modes, "setup-only")) {
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, NJOBS);
    job_t jobs[NJOBS];
    pthread_t th[NJOBS];
    memset(jobs, 0, sizeof(jobs));
    for (int j = 0; j < NJOBS; j++) {
      jobs[j].bar = &bar;
      pthread_create(&th[j], NULL, setup_only_main, &jobs[j]);
    }
    for (int j = 0; j < NJOBS; j++) pthread_join(th[j], NULL);
    pthread_barrier_destroy(&bar);
    int st = 0;
    for (int j = 0; j < NJOBS; j++) st |= jobs[j].res.status;
    printf(st ? "setup-only failed\n" : "ok setup-only: %d threads created and destroyed contexts\n", NJOBS);
    ok &= !st;
  }
  if (has_mode(modes, "shared")) ok &= concurrent("shared", ctx, ds, good, serial);
  if (has_mode(modes, "separate")) ok &= concurrent("separate", 0, 0, good, serial);
  if (has_mode(modes, "errors-shared")) ok &= concurrent("errors-shared", ctx, ds, bad0, serial);
  if (has_mode(modes, "errors-separate")) ok &= concurrent("errors-separate", 0, 0, bad0, serial);
  for (int j = 0; j < NJOBS; j++) free_result(&serial[j]);
  sbagb_dataset_free(ds);
  sbagb_ctx_destroy(ctx);
  free(buf);
#if defined(__SANITIZE_ADDRESS__)
#define ABI_ASAN 1
#elif defined(__has_feature)
#if __has_feature(address_sanitizer)
#define ABI_ASAN 1
#endif
#endif
#ifdef ABI_ASAN
  /* Under host ASan, leave without the runtime's static destructors: the HSA runtime's own
     teardown (libhsa-runtime64's destructors, after contexts were created on several threads)
     frees through ASan's device allocator after that allocator has been unloaded
     ("CHECK failed: sanitizer_allocator_device.h ... dev_runtime_unloaded_"), which is the
     toolchain's teardown order, not this library's code: every context, dataset and forest has
     been released above, and each verdict line is already out. */
  fflush(stdout);
  _exit(ok ? 0 : 1);
#endif
  return ok ? 0 : 1;
}
