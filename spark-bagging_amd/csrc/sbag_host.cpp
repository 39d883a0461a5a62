// sbag_host.cpp — C ABI (include/sbag.h) and host orchestration of the bagging
// engine.  The host mirrors the control flow of the reference's
// BaggingRegressor.train (ml/regression/BaggingRegressor.scala:121-199): bag ->
// per-learner subspace -> base-learner fit -> model of (subspaces, models), but
// all learners of a context are trained together, level by level, by the HIP
// kernels of sbag_kernels.hip.  The per-node bookkeeping of Spark 2.4.3's
// RandomForest (LearningNode, binsToBestSplit's ImpurityStats chain,
// toNode(prune = true)) lives here; every histogram and split search runs on
// the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <array>
#include <map>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "sbag.h"
#include "sbag_fastmath.h"
#include "sbag_internal.h"

using namespace sbag;

// ---------------------------------------------------------------- errors
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIP_TRY(x)                                                                   \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess)                                                            \
      return fail(e_ == hipErrorOutOfMemory ? SBAG_ENOMEM : SBAG_EDEVICE,            \
                  std::string(#x) + " failed: " + hipGetErrorString(e_));            \
  } while (0)
#define TRY(x)                   \
  do {                           \
    int rc_ = (x);               \
    if (rc_ != SBAG_OK) return rc_; \
  } while (0)

static const double kDoubleMinValue = -std::numeric_limits<double>::max();  // Scala Double.MinValue

// ---------------------------------------------------------------- context
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

// Persistent host workers for the per-level bookkeeping: run(n, f) calls f(0) on the
// caller and f(1..n-1) on workers, and returns when all are done (a per-level thread
// spawn cost about as much as the work it split).
struct HostPool {
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv, done;
  const std::function<void(int)>* job = nullptr;
  int n = 0, pending = 0;
  uint64_t gen = 0;
  bool stop = false;
  // host threads for node bookkeeping, thresholds, tree emission and ingest: 16 (the
  // CPU share of one GPU on an 8-GPU node) unless SBAG_HOST_THREADS says otherwise
  // host threads per context: 16, or the process's share of the cores when torchrun
  // starts one process per GPU (LOCAL_WORLD_SIZE) and sbag_fit runs two contexts each
  static int width() {
    static const int w = [] {
      const char* e = getenv("SBAG_HOST_THREADS");
      if (e) return std::max(1, std::min(atoi(e), 1024));
      const int hw = std::max(1, (int)std::thread::hardware_concurrency());
      const char* lw = getenv("LOCAL_WORLD_SIZE");
      const int procs = lw ? std::max(1, atoi(lw)) : 1;
      return std::max(2, std::min(16, hw / (2 * procs)));
    }();
    return w;
  }
  void run(int nw, const std::function<void(int)>& f) {
    nw = std::max(1, std::min(nw, width()));
    if (nw == 1) {
      f(0);
      return;
    }
    {
      std::unique_lock<std::mutex> lk(m);
      while ((int)th.size() < nw - 1) {
        const int id = (int)th.size() + 1;
        th.emplace_back([this, id] { loop(id); });
      }
      job = &f;
      n = nw;
      pending = nw - 1;
      gen++;
    }
    cv.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(m);
    done.wait(lk, [&] { return pending == 0; });
    job = nullptr;
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        if (id >= n) continue;
        f = job;
      }
      (*f)(id);
      std::lock_guard<std::mutex> lk(m);
      if (--pending == 0) done.notify_all();
    }
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(m);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
};

// Frees a finished fit's host containers on a thread of its own: C5's ~65 000 tree nodes
// with heap-held class counts (allocated on the pool's workers) took 3-14 ms to destroy
// on the fit's thread, after its last kernel and before the next fit could launch one
struct Reaper {
  std::mutex m;
  std::condition_variable cv;
  std::vector<std::shared_ptr<void>> q;
  bool stop = false;
  std::thread th;
  void post(std::shared_ptr<void> p) {
    {
      std::lock_guard<std::mutex> lk(m);
      if (!th.joinable()) th = std::thread([this] { loop(); });
      q.push_back(std::move(p));
    }
    cv.notify_one();
  }
  void loop() {
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
      cv.wait(lk, [&] { return stop || !q.empty(); });
      if (q.empty()) return;  // stopped and drained
      std::vector<std::shared_ptr<void>> w;
      w.swap(q);
      lk.unlock();
      w.clear();
      lk.lock();
    }
  }
  ~Reaper() {
    {
      std::lock_guard<std::mutex> lk(m);
      stop = true;
    }
    cv.notify_all();
    if (th.joinable()) th.join();
  }
};

struct sbag_ctx {
  HostPool pool;
  int device = 0;
  hipStream_t stream = nullptr;
  std::unordered_map<std::string, DevBuf> ws;
  uint64_t* d_jump = nullptr;
  // pinned staging for the per-level uploads (work lists, tables): a bump arena
  // that is reset whenever the stream is known to be idle (every d2h synchronizes)
  unsigned char* pin = nullptr;
  size_t pin_cap = 0, pin_used = 0;
  // every entry point that uses the context holds this: concurrent callers (learner
  // Futures, CrossValidator fits, executor threads) share its stream, workspace, pinned
  // arena and host pool, so their calls are serialized here (recursive: sbag_fit
  // re-enters itself when it splits a learner range)
  std::recursive_mutex mu;
  // a second stream and workspace on the same device: sbag_fit runs the two halves of a
  // learner range on the two contexts from two host threads, so one half's host work
  // (split bookkeeping between levels) overlaps the other half's kernels
  std::vector<sbag_ctx*> twins;
  // learner parts fitting concurrently on this device (sbag_fit's overlap): each part's
  // per-replica bins get 1/concurrent_parts of the device budget
  int concurrent_parts = 1;
  // the split stats planes copied back per level (C5's deep levels: ~50 MB), kept between
  // fits: a fresh buffer per fit page-faulted on every first copy and was unmapped at its end
  std::unique_ptr<int64_t[]> h_sst;
  size_t h_sst_cap = 0;
  Reaper reaper;  // (last: destroyed first, after its pending frees)
};
#define CTX_LOCK(c) std::lock_guard<std::recursive_mutex> ctx_lock_((c)->mu)

static int ws_get(sbag_ctx* c, const std::string& name, size_t bytes, void** out) {
  DevBuf& b = c->ws[name];
  if (bytes == 0) bytes = 16;
  if (b.cap < bytes) {
    if (b.p) HIP_TRY(hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    // 256 bytes of slack past every buffer: row-wise kernels may over-read the last row
    size_t want = bytes + bytes / 8 + 256;
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      want = bytes + 256;
      e = hipMalloc(&b.p, want);
    }
    if (e != hipSuccess) {
      (void)hipGetLastError();
      b.p = nullptr;
      return fail(SBAG_ENOMEM, "device allocation of " + std::to_string(bytes) + " bytes (" +
                                   name + ") failed: " + hipGetErrorString(e));
    }
    b.cap = want;
  }
  *out = b.p;
  return SBAG_OK;
}

template <typename T>
static int ws_typed(sbag_ctx* c, const std::string& name, size_t count, T** out) {
  void* p;
  TRY(ws_get(c, name, count * sizeof(T), &p));
  *out = (T*)p;
  return SBAG_OK;
}

template <typename T>
static int h2d(sbag_ctx* c, T* dst, const T* src, size_t count) {
  if (count == 0) return SBAG_OK;
  const size_t bytes = count * sizeof(T);
  if (bytes <= ((size_t)64 << 20)) {  // through the pinned arena: a true async DMA
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (c->pin_used + need > c->pin_cap) {
      HIP_TRY(hipStreamSynchronize(c->stream));  // earlier uploads have been consumed
      // an arena that ran out between two synchronizations grows (x2, to 256 MB), so a
      // level's uploads (C5's deep levels: ~10 MB of pieces and tile bases) fit in it and
      // the next level does not pay this synchronization again
      const bool grow = need > c->pin_cap || (c->pin_used > 0 && c->pin_cap < ((size_t)256 << 20));
      c->pin_used = 0;
      if (grow) {
        if (c->pin) HIP_TRY(hipHostFree(c->pin));
        c->pin = nullptr;
        const size_t cap = std::max<size_t>({need, (size_t)8 << 20, std::min<size_t>(2 * c->pin_cap, (size_t)256 << 20)});
        c->pin_cap = 0;
        HIP_TRY(hipHostMalloc((void**)&c->pin, cap, hipHostMallocDefault));
        c->pin_cap = cap;
      }
    }
    unsigned char* stage = c->pin + c->pin_used;
    c->pin_used += need;
    memcpy(stage, src, bytes);
    HIP_TRY(hipMemcpyAsync(dst, stage, bytes, hipMemcpyHostToDevice, c->stream));
    return SBAG_OK;
  }
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  return SBAG_OK;
}
template <typename T>
static int d2h(sbag_ctx* c, T* dst, const T* src, size_t count) {
  if (count == 0) return SBAG_OK;
  HIP_TRY(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->pin_used = 0;  // the stream is idle: every staged upload has completed
  return SBAG_OK;
}

// ---------------------------------------------------------------- host RNG (subspace, seeds)
// XORShiftRandom.hashSeed + nextDouble (Spark 2.4.3), used by mkSubspace
// (ml/ensemble/HasSubBag.scala:97-103) and to build the GF(2) jump tables.
static uint32_t h_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t h_mix_last(uint32_t h, uint32_t k) {
  k *= 0xcc9e2d51u;
  k = h_rotl(k, 15);
  k *= 0x1b873593u;
  return h ^ k;
}
static uint32_t h_mix(uint32_t h, uint32_t k) {
  h = h_mix_last(h, k);
  h = h_rotl(h, 13);
  return h * 5u + 0xe6546b64u;
}
// Spark 2.4.3 hashes ByteBuffer.allocate(java.lang.Long.SIZE).putLong(seed): Long.SIZE is 64
// bits used as a byte count, so the buffer is 64 bytes (big-endian seed + 56 zero bytes).
// Spark 3.0 switched to Long.BYTES; the reference pins 2.4.3 (build.sbt:1).
static constexpr int kHashSeedBytes = 64;
static uint32_t h_hash_buf(const uint8_t* d, uint32_t seed) {
  uint32_t h = seed;
  for (int i = 0; i < kHashSeedBytes; i += 4) {
    const uint32_t k = (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8) | ((uint32_t)d[i + 2] << 16) |
                       ((uint32_t)d[i + 3] << 24);
    h = h_mix(h, k);
  }
  h ^= (uint32_t)kHashSeedBytes;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
static uint64_t h_hash_seed(int64_t seed) {
  uint8_t b[kHashSeedBytes] = {};
  const uint64_t u = (uint64_t)seed;
  for (int i = 0; i < 8; i++) b[i] = (uint8_t)(u >> (56 - 8 * i));
  const uint32_t lo = h_hash_buf(b, 0x3c074a61u);
  const uint32_t hi = h_hash_buf(b, lo);
  return ((uint64_t)hi << 32) | lo;
}
static uint64_t h_xs_step(uint64_t s) {
  s ^= s << 21;
  s ^= s >> 35;
  s ^= s << 4;
  return s;
}
struct HostXS {
  uint64_t s;
  explicit HostXS(int64_t seed) : s(h_hash_seed(seed)) {}
  int32_t next(int bits) {
    s = h_xs_step(s);
    return (int32_t)(uint32_t)(s & ((1ull << bits) - 1));
  }
  double next_double() {
    const int64_t a = next(26);
    const int64_t b = next(27);
    return (double)((a << 27) + b) * 0x1.0p-53;
  }
};

static int ensure_jump(sbag_ctx* c) {
  if (c->d_jump) return SBAG_OK;
  // jump[k][b] = M^(2^k) e_b, M = one XORShift step (linear over GF(2))
  std::vector<uint64_t> J(63 * 64);
  for (int b = 0; b < 64; b++) J[b] = h_xs_step(1ull << b);
  for (int k = 1; k < 63; k++) {
    for (int b = 0; b < 64; b++) {
      uint64_t x = J[(k - 1) * 64 + b], acc = 0;
      for (int q = 0; q < 64; q++)
        if ((x >> q) & 1) acc ^= J[(k - 1) * 64 + q];
      J[k * 64 + b] = acc;
    }
  }
  HIP_TRY(hipMalloc(&c->d_jump, J.size() * 8));
  HIP_TRY(hipMemcpy(c->d_jump, J.data(), J.size() * 8, hipMemcpyHostToDevice));
  return SBAG_OK;
}

// ---------------------------------------------------------------- dataset
// A label column and its device images: the dataset's own, or (sbag_fit_booster) the
// pseudo-residuals of one boosting iteration over the same rows
struct LabelSet {
  std::vector<double> y;
  int32_t* d_labk = nullptr;              // labels as fixed point k = y * 2^shift
  double* d_y64 = nullptr;                // fp64 labels on the device (f64 fits; built lazily)
  int shift = 0;
  bool label_ok = false;                  // representable as |k| < 2^23
  int64_t kmin = 0, kmax = 0;
  bool integral = false;                  // all labels integers >= 0 (classifiable)
  bool finite = true;                     // no NaN / inf
  // labels that are not dyadic (fp64 path): the fixed-point image k = round(y 2^ashift),
  // |k| <= 2^22, which the integer histograms screen splits with (|y - k 2^-ashift| <=
  // 2^-ashift-1), and the labels' largest |y| and y*y (the screen's error bounds)
  bool approx_ok = false;
  int ashift = 0;
  int64_t akmin = 0, akmax = 0;
  double ymax_abs = 0.0, ymax_sq = 0.0;
};

struct sbag_dataset {
  sbag_ctx* ctx = nullptr;
  int64_t N = 0;
  int32_t F = 0, S = 0;     // S: row stride in code elements
  int code_bytes = 1;                     // 4: "wide" (a feature with > 65536 distinct values)
  void* d_codes = nullptr;
  std::vector<uint32_t> h_codes;          // wide datasets: the codes on the host too [N][S]
  std::vector<std::vector<double>> dict;  // sorted distinct values per feature (-0.0 == 0.0)
  std::vector<int32_t> zero_code;         // code of 0.0, -1 when absent
  LabelSet lab;                           // the label column (owns its device images)
  double* d_dict = nullptr;
  int64_t* d_dict_off = nullptr;
  // Layouts derived from the codes alone, for fits whose bins are the codes: the
  // column-major copy [cols_ncol][npad] and the side-bit planes [cols_ncol][planes_nsp][nw32]
  // of k_partition.  Part of ingest: built by the first such fit, kept with the dataset.
  std::mutex layout_mu;
  uint8_t* d_cols = nullptr;
  int32_t cols_ncol = 0;
  uint32_t* d_planes = nullptr;
  int32_t planes_nsp = 0;
  bool planes_done = false;  // the planes were built (or found not to fit) by a fit
  // every device buffer goes with the dataset, also when a constructor (create, import)
  // returns early after some of them were allocated
  ~sbag_dataset() {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (void* p : {(void*)d_codes, (void*)lab.d_labk, (void*)lab.d_y64, (void*)d_dict, (void*)d_dict_off,
                    (void*)d_cols, (void*)d_planes})
      if (p) (void)hipFree(p);
  }
};

static int32_t row_stride(int32_t F) {
  if (F <= 64) return (F + 15) / 16 * 16;
  return (F + 127) / 128 * 128;
}

// chunks of [0, N) on the host pool (one chunk per worker; serial without a pool)
static void par_range(HostPool* pool, int64_t N, const std::function<void(int64_t, int64_t, int)>& f,
                      int* nw_out = nullptr) {
  const int nw = pool && N >= (1 << 16) ? HostPool::width() : 1;
  if (nw_out) *nw_out = nw;
  auto body = [&](int w) {
    const int64_t lo = N * w / nw, hi = N * (w + 1) / nw;
    f(lo, hi, w);
  };
  if (nw == 1)
    body(0);
  else
    pool->run(nw, body);
}

// The label column's integer images: dyadic fixed point (k = y 2^s exactly, |k| < 2^23, s
// minimal and <= 40), or for any other finite labels the fp64 engine's screening image
// k = round(y 2^ashift), |k| <= 2^22; also whether the labels are class indices and their
// largest |y| (the screen's bounds).  One pass: the smallest s making y integral is read off
// y's binary exponent and trailing zeros, and k's range is y's range times 2^s.
static void set_label_stats(LabelSet& L, int64_t N, bool finite, bool integral, int smax, double ymin,
                            double ymax, double amax) {
  L.finite = finite;
  L.integral = integral;
  L.label_ok = false;
  if (finite && smax <= 40 && std::ldexp(amax, smax) < 8388608.0) {
    L.label_ok = true;
    L.shift = smax;
    L.kmin = N ? (int64_t)std::ldexp(ymin, smax) : 0;
    L.kmax = N ? (int64_t)std::ldexp(ymax, smax) : 0;
  }
  L.approx_ok = false;
  L.ymax_abs = finite ? amax : 0.0;
  L.ymax_sq = finite ? amax * amax : 0.0;
  if (!L.label_ok && finite && amax > 0.0) {
    // 2^e <= max|y| < 2^(e+1): max|y| 2^(21-e) < 2^22 (the image's range includes 0)
    L.ashift = 21 - std::ilogb(amax);
    L.akmin = std::min<int64_t>(0, (int64_t)std::nearbyint(std::ldexp(ymin, L.ashift)));
    L.akmax = std::max<int64_t>(0, (int64_t)std::nearbyint(std::ldexp(ymax, L.ashift)));
    L.approx_ok = true;
  }
}

static void analyze_labels(LabelSet& L, HostPool* pool = nullptr) {
  const int64_t N = (int64_t)L.y.size();
  struct Acc {
    bool finite = true, integral = true;
    int smax = 0;
    double ymin = INFINITY, ymax = -INFINITY, amax = 0.0;
  };
  std::vector<Acc> acc(std::max(1, HostPool::width()));
  int nw = 1;
  par_range(pool, N, [&](int64_t lo, int64_t hi, int w) {
    Acc a;
    for (int64_t i = lo; i < hi; i++) {
      const double v = L.y[i];
      if (!std::isfinite(v)) {
        a.finite = false;
        a.integral = false;
        continue;
      }
      int si = 0;
      if (v != 0.0) {
        uint64_t bits;
        std::memcpy(&bits, &v, 8);
        const int E = (int)((bits >> 52) & 0x7FF);
        const uint64_t M = bits & ((1ull << 52) - 1);
        const uint64_t sig = E ? (M | (1ull << 52)) : M;
        const int low = (E ? E - 1075 : -1074) + __builtin_ctzll(sig);  // v = odd * 2^low
        si = low < 0 ? -low : 0;
      }
      a.smax = std::max(a.smax, si);
      if (!(v >= 0 && si == 0 && v < 8388608.0)) a.integral = false;
      a.ymin = std::min(a.ymin, v);
      a.ymax = std::max(a.ymax, v);
      a.amax = std::max(a.amax, std::fabs(v));
    }
    acc[w] = a;
  }, &nw);
  Acc t;
  for (int w = 0; w < nw; w++) {
    t.finite = t.finite && acc[w].finite;
    t.integral = t.integral && acc[w].integral;
    t.smax = std::max(t.smax, acc[w].smax);
    t.ymin = std::min(t.ymin, acc[w].ymin);
    t.ymax = std::max(t.ymax, acc[w].ymax);
    t.amax = std::max(t.amax, acc[w].amax);
  }
  set_label_stats(L, N, t.finite, t.integral, t.smax, t.ymin, t.ymax, t.amax);
}
static void analyze_labels(sbag_dataset* ds) { analyze_labels(ds->lab, &ds->ctx->pool); }

// the labels' fixed point image (exact for dyadic labels, else the screening approximation
// of the fp64 path, else zeros) into dst [N] on the device
static int labk_image(const LabelSet& L, int32_t* dst, HostPool* pool = nullptr) {
  const int64_t N = (int64_t)L.y.size();
  if (!L.label_ok && !L.approx_ok) {
    HIP_TRY(hipMemset(dst, 0, (size_t)std::max<int64_t>(N, 1) * 4));
    return SBAG_OK;
  }
  std::vector<int32_t> k(N);
  par_range(pool, N, [&](int64_t lo, int64_t hi, int) {
    if (L.label_ok)
      for (int64_t i = lo; i < hi; i++) k[i] = (int32_t)std::ldexp(L.y[i], L.shift);
    else
      for (int64_t i = lo; i < hi; i++) k[i] = (int32_t)std::nearbyint(std::ldexp(L.y[i], L.ashift));
  });
  HIP_TRY(hipMemcpy(dst, k.data(), (size_t)N * 4, hipMemcpyHostToDevice));
  return SBAG_OK;
}

static int upload_labels(sbag_dataset* ds) {
  HIP_TRY(hipMalloc(&ds->lab.d_labk, std::max<int64_t>(ds->N, 1) * 4));
  return labk_image(ds->lab, ds->lab.d_labk, &ds->ctx->pool);
}

static int upload_dict(sbag_dataset* ds) {
  std::vector<int64_t> off(ds->F + 1, 0);
  for (int f = 0; f < ds->F; f++) off[f + 1] = off[f] + (int64_t)ds->dict[f].size();
  std::vector<double> flat(std::max<int64_t>(off[ds->F], 1));
  for (int f = 0; f < ds->F; f++)
    std::copy(ds->dict[f].begin(), ds->dict[f].end(), flat.begin() + off[f]);
  HIP_TRY(hipMalloc(&ds->d_dict, flat.size() * 8));
  HIP_TRY(hipMalloc(&ds->d_dict_off, off.size() * 8));
  HIP_TRY(hipMemcpy(ds->d_dict, flat.data(), flat.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ds->d_dict_off, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  return SBAG_OK;
}

// ---------------------------------------------------------------- forest
struct HTree {
  std::vector<int32_t> sub;
  std::vector<sbag_node> nodes;
  std::vector<double> stats;
  int32_t ns = 0;
  int32_t exact = 1;
};

struct sbag_forest {
  std::vector<HTree> trees;
  int32_t impurity = 0;
  sbag_timing timing{};
  // device copies of the node arrays for the global-memory walk, one per device, built on
  // first use: contexts on different devices (or threads predicting with one forest) each
  // read their own copy, and a copy is never freed while the forest lives
  struct DevCopy {
    DevNode* nodes = nullptr;
    int64_t* off = nullptr;
  };
  std::mutex dev_mu;
  std::map<int, DevCopy> dev;
  int32_t nclasses = 0;
  ~sbag_forest() {
    for (auto& kv : dev) {
      (void)hipSetDevice(kv.first);
      if (kv.second.nodes) (void)hipFree(kv.second.nodes);
      if (kv.second.off) (void)hipFree(kv.second.off);
    }
  }
};

// ---------------------------------------------------------------- impurity (host, fp64, Spark order)
struct Calc {  // ImpurityCalculator over exact integer stats
  const int64_t* st;
  int ns;
  bool gini;
  int shift;
  double count_d() const {
    if (!gini) return (double)st[0];
    double t = 0.0;
    for (int i = 0; i < ns; i++) t += (double)st[i];
    return t;
  }
  int64_t count() const { return (int64_t)count_d(); }
  double stat(int i) const {  // the fp64 stats the reference accumulates
    if (gini) return (double)st[i];
    if (i == 0) return (double)st[0];
    if (i == 1) return std::ldexp((double)st[1], -shift);
    return std::ldexp((double)(uint64_t)st[2], -2 * shift);
  }
  double impurity() const {
    if (!gini) {  // Variance.calculate
      const double count = stat(0), sum = stat(1), sumsq = stat(2);
      if (count == 0) return 0.0;
      const double squared_loss = sumsq - (sum * sum) / count;
      return squared_loss / count;
    }
    const double total = count_d();  // Gini.calculate
    if (total == 0) return 0.0;
    double imp = 1.0;
    for (int i = 0; i < ns; i++) {
      const double f = (double)st[i] / total;
      imp -= f * f;
    }
    return imp;
  }
  double predict() const {
    const int64_t cnt = count();
    if (cnt == 0) return 0.0;
    if (!gini) return stat(1) / (double)cnt;
    int best = -1;
    double bv = kDoubleMinValue;
    for (int i = 0; i < ns; i++)
      if ((double)st[i] > bv) {
        bv = (double)st[i];
        best = i;
      }
    return (double)best;
  }
};

constexpr int kMaxHostNS = 4096;  // classes + 1 (check_agg's bound on nclasses)

struct NodeStats {  // exact integer stats of a node: inline up to 8 words (no allocation)
  int64_t inl[8];
  std::vector<int64_t> heap;
  int n = 0;
  int64_t* data() { return n <= 8 ? inl : heap.data(); }
  const int64_t* data() const { return n <= 8 ? inl : heap.data(); }
  int64_t& operator[](size_t i) { return data()[i]; }
  int64_t operator[](size_t i) const { return data()[i]; }
  void assign(const int64_t* a, const int64_t* b) {
    n = (int)(b - a);
    if (n > 8)
      heap.assign(a, b);
    else
      std::copy(a, b, inl);
  }
};

struct HNode {  // LearningNode
  int left = -1, right = -1;
  bool is_leaf = false, has_split = false;
  int fl = -1, s = -1;
  double thr = 0.0;
  NodeStats stats;
  double impurity = 0.0, gain = NAN;
  bool valid = true;
};

struct ToNodeRet {
  bool leaf;
  double pred;
};

// LearningNode.toNode(prune = true), emitted as NodeData pre-order
static ToNodeRet emit(const std::vector<HNode>& nodes, int idx, HTree& t, int ns, bool gini,
                      int shift, int stats_out) {
  const HNode& n = nodes[idx];
  const int my = (int)t.nodes.size();
  t.nodes.push_back(sbag_node{});
  t.stats.resize((size_t)(my + 1) * stats_out);
  Calc c{n.stats.data(), ns, gini, shift};
  auto fill_stats = [&](int at) {
    for (int i = 0; i < stats_out; i++) t.stats[(size_t)at * stats_out + i] = c.stat(i);
  };
  if (n.has_split) {
    const size_t mark = t.nodes.size();
    const int lid = (int)t.nodes.size();
    ToNodeRet l = emit(nodes, n.left, t, ns, gini, shift, stats_out);
    const int rid = (int)t.nodes.size();
    ToNodeRet r = emit(nodes, n.right, t, ns, gini, shift, stats_out);
    sbag_node& o = t.nodes[my];
    if (l.leaf && r.leaf && l.pred == r.pred) {
      t.nodes.resize(mark);
      t.stats.resize(mark * stats_out);
      sbag_node& p = t.nodes[my];
      p = sbag_node{};
      p.id = my;
      p.left = p.right = -1;
      p.feature = -1;
      p.split_bin = -1;
      p.prediction = l.pred;
      p.impurity = n.impurity;
      p.gain = -1.0;
      fill_stats(my);
      return {true, l.pred};
    }
    o.id = my;
    o.left = lid;
    o.right = rid;
    o.feature = n.fl;
    o.split_bin = n.s;
    o.threshold = n.thr;
    o.prediction = c.predict();
    o.impurity = n.impurity;
    o.gain = n.gain;
    fill_stats(my);
    return {false, o.prediction};
  }
  sbag_node& o = t.nodes[my];
  o.id = my;
  o.left = o.right = -1;
  o.feature = -1;
  o.split_bin = -1;
  o.prediction = c.predict();
  o.impurity = n.valid ? n.impurity : -1.0;
  o.gain = -1.0;
  fill_stats(my);
  return {true, o.prediction};
}

// ---------------------------------------------------------------- split finding (host)
// RandomForest.findSplitsForContinuousFeature over a replica's weighted value
// counts (the subbag replicates each row `count` times).  `cnt[c]` is the
// weighted count of dictionary value `vals[c]` among the in-bag rows, or among the
// split-finding sample; n = numExamples, num_samples = n or (fraction * n).toInt, whose
// shortfall over the nonzero count is the implied count of 0.0.
static int find_splits(const std::vector<double>& vals, const uint32_t* cnt, int zero_code, int64_t n,
                       int64_t num_samples, int max_bins, std::vector<double>& thr) {
  thr.clear();
  int64_t nnz = 0;
  for (size_t c = 0; c < vals.size(); c++)
    if ((int)c != zero_code) nnz += cnt[c];
  if (nnz == 0) return 0;  // featureSamples.isEmpty
  const int64_t max_possible_bins = std::min<int64_t>(max_bins, n);
  const int64_t num_splits = max_possible_bins - 1;
  std::vector<std::pair<double, int64_t>> vc;
  vc.reserve(vals.size());
  const int64_t zeros = num_samples - nnz;
  for (size_t c = 0; c < vals.size(); c++) {
    if ((int)c == zero_code) {
      if (zeros > 0) vc.emplace_back(0.0, zeros);
      continue;
    }
    if (cnt[c] == 0) continue;
    vc.emplace_back(vals[c], (int64_t)cnt[c]);
  }
  if (zero_code < 0 && zeros > 0) {  // zeros implied by a sample short of numSamples
    vc.emplace_back(0.0, zeros);
    std::sort(vc.begin(), vc.end());
  }
  const int64_t possible = (int64_t)vc.size() - 1;
  if (possible == 0) return 0;
  if (possible <= num_splits) {
    for (int64_t i = 1; i <= possible; i++) thr.push_back((vc[i - 1].first + vc[i].first) / 2.0);
  } else {
    const double stride = (double)num_samples / (double)(num_splits + 1);
    int32_t current = (int32_t)vc[0].second;
    double target = stride;
    for (size_t i = 1; i < vc.size(); i++) {
      const int32_t prev = current;
      current += (int32_t)vc[i].second;
      if (std::fabs((double)prev - target) < std::fabs((double)current - target)) {
        thr.push_back((vc[i - 1].first + vc[i].first) / 2.0);
        target += stride;
      }
    }
  }
  return (int)thr.size();
}

// ---------------------------------------------------------------- timing
struct EventTimer {
  hipStream_t st;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev;  // category
  std::vector<int> lv;  // tree level of each event (-1 before the level loop)
  int level = -1;
  int begin(int cat) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -1;
    (void)hipEventRecord(a, st);
    ev.push_back({cat, {a, b}});
    lv.push_back(level);
    return (int)ev.size() - 1;
  }
  void end(int h) {
    if (h >= 0) (void)hipEventRecord(ev[h].second.second, st);
  }
  void collect(double* cats, std::vector<double>* hist_each, int hist_cat) {
    for (auto& e : ev) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e.second.first, e.second.second);
      cats[e.first] += ms;
      if (e.first == hist_cat && hist_each) hist_each->push_back(ms);
    }
  }
  ~EventTimer() {
    for (auto& e : ev) {
      (void)hipEventDestroy(e.second.first);
      (void)hipEventDestroy(e.second.second);
    }
  }
};
enum { T_SAMPLE, T_VC, T_BIN, T_COMPACT, T_HIST, T_SPLIT, T_SUB, T_PART, T_FIX, T_GROUP, T_CHAIN, T_ROOT, T_NCAT };

// ---------------------------------------------------------------- C ABI
extern "C" {

const char* sbag_last_error(void) { return g_err.c_str(); }
const char* sbag_version(void) { return "sbag 0.1 (gfx950)"; }

int sbag_device_count(int32_t* n) {
  int c = 0;
  HIP_TRY(hipGetDeviceCount(&c));
  *n = c;
  return SBAG_OK;
}

int sbag_ctx_create(int32_t device_ordinal, sbag_ctx** out) {
  if (!out) return fail(SBAG_EINVAL, "out is NULL");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device_ordinal < 0 || device_ordinal >= n)
    return fail(SBAG_EINVAL, "device ordinal " + std::to_string(device_ordinal) + " out of range");
  HIP_TRY(hipSetDevice(device_ordinal));
  auto* c = new sbag_ctx();
  c->device = device_ordinal;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(SBAG_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  *out = c;
  return SBAG_OK;
}

// frees the context's workspace (the caller holds its lock; the stream is drained first)
static void ws_release(sbag_ctx* c) {
  (void)hipStreamSynchronize(c->stream);
  for (auto& kv : c->ws)
    if (kv.second.p) (void)hipFree(kv.second.p);
  c->ws.clear();
}

// frees one named workspace buffer if it holds more than `keep` bytes (the stream is drained)
static void ws_trim(sbag_ctx* c, const std::string& name, size_t keep) {
  auto it = c->ws.find(name);
  if (it == c->ws.end() || it->second.cap <= keep) return;
  (void)hipStreamSynchronize(c->stream);
  if (it->second.p) (void)hipFree(it->second.p);
  c->ws.erase(it);
}

int sbag_ctx_destroy(sbag_ctx* c) {
  if (!c) return SBAG_OK;
  { CTX_LOCK(c); }  // no call is in flight on it any more
  for (sbag_ctx* t : c->twins) (void)sbag_ctx_destroy(t);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (auto& kv : c->ws)
    if (kv.second.p) (void)hipFree(kv.second.p);
  if (c->d_jump) (void)hipFree(c->d_jump);
  if (c->pin) (void)hipHostFree(c->pin);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return SBAG_OK;
}

int sbag_subspace(double ratio, int32_t F, int64_t seed, int32_t* idx, int32_t* n_out) {
  if (F < 0 || !idx || !n_out) return fail(SBAG_EINVAL, "bad arguments");
  int n = 0;
  if (ratio == 1.0) {
    for (int f = 0; f < F; f++) idx[n++] = f;
  } else {
    HostXS r(seed);
    for (int f = 0; f < F; f++)
      if (r.next_double() < ratio) idx[n++] = f;
  }
  *n_out = n;
  return SBAG_OK;
}

static int check_sampler(const sbag_sampler_params* p) {
  if (!(p->sample_ratio >= 0.0 && p->sample_ratio <= 1.0))
    return fail(SBAG_EINVAL, "sampleRatio given invalid value " + std::to_string(p->sample_ratio) +
                                 " (ParamValidators.inRange(0, 1))");
  if (!(p->sample_ratio > 0)) return fail(SBAG_EINVAL, "requirement failed: sampleRatio must be strictly positive");
  if (p->learner_end <= p->learner_begin || p->learner_begin < 0)
    return fail(SBAG_EINVAL, "numBaseLearners given invalid value (learner range empty)");
  return SBAG_OK;
}

// counts [R][N] on the device (bfunctions.bag)
// (check_now = false: the caller reads the Poisson overflow flag later, with its next copy
// from the device -- sbag_fit does after the compaction -- so the sampler and the compaction
// queue back to back instead of the host waiting out the sampler in between)
static int sampler_overflow(sbag_ctx* c) {
  int* d_err;
  TRY(ws_typed(c, "err", 1 + 16, &d_err));
  int err = 0;
  TRY(d2h(c, &err, d_err, 1));
  if (err) return fail(SBAG_EUNSUPPORTED, "a Poisson draw exceeded 255");
  return SBAG_OK;
}

static int run_sampler(sbag_ctx* c, const sbag_sampler_params* p, const std::vector<int64_t>& poff,
                       int64_t N, uint8_t* d_counts, bool check_now = true) {
  const int R = p->learner_end - p->learner_begin;
  const int P = (int)poff.size() - 1;
  int64_t* d_poff;
  TRY(ws_typed(c, "poff", poff.size(), &d_poff));
  TRY(h2d(c, d_poff, poff.data(), poff.size()));
  if (p->replacement) {
    int* d_err;
    TRY(ws_typed(c, "err", 1 + 16, &d_err));  // flag + 64-byte store sink for k_poisson
    HIP_TRY(hipMemsetAsync(d_err, 0, 4, c->stream));
    // PoissonDistribution.nextPoisson: p = FastMath.exp(-mean), restated table for table
    // (sbag_fastmath.h): FastMath is not correctly rounded (mean 0.052: one ulp above libm).
    const double p_exp = sbag_fm_exp_neg(-p->sample_ratio);
    launch_poisson(c->stream, d_counts, N, d_poff, P, R, p->learner_begin, p->seed, p->sample_ratio,
                   p_exp, d_err);
    HIP_TRY(hipGetLastError());
    if (check_now) TRY(sampler_overflow(c));
  } else if (p->sample_ratio == 1.0) {
    launch_fill(c->stream, d_counts, 1, (int64_t)R * N);
    HIP_TRY(hipGetLastError());
  } else {
    TRY(ensure_jump(c));
    std::vector<int64_t> cpre(P + 1, 0);
    for (int q = 0; q < P; q++) cpre[q + 1] = cpre[q] + (poff[q + 1] - poff[q] + 255) / 256;
    int64_t* d_cpre;
    TRY(ws_typed(c, "cpre", cpre.size(), &d_cpre));
    TRY(h2d(c, d_cpre, cpre.data(), cpre.size()));
    launch_bernoulli(c->stream, d_counts, N, d_poff, d_cpre, P, cpre[P], R, p->learner_begin,
                     p->seed, p->sample_ratio, c->d_jump);
    HIP_TRY(hipGetLastError());
  }
  return SBAG_OK;
}

static int check_partitions(int32_t P, const int64_t* off, int64_t N, std::vector<int64_t>& poff) {
  if (P <= 1 || !off) {
    poff = {0, N};
    return SBAG_OK;
  }
  poff.assign(off, off + P + 1);
  if (poff[0] != 0 || poff[P] != N)
    return fail(SBAG_EINVAL, "partition_offsets must start at 0 and end at num_rows");
  for (int i = 0; i < P; i++)
    if (poff[i + 1] < poff[i]) return fail(SBAG_EINVAL, "partition_offsets must be non-decreasing");
  return SBAG_OK;
}

int sbag_sample(sbag_ctx* c, const sbag_sampler_params* p, const int64_t* partition_offsets,
                int32_t P, int64_t N, uint8_t* counts_out) {
  if (!c || !p || !counts_out || N < 0) return fail(SBAG_EINVAL, "bad arguments");
  CTX_LOCK(c);
  TRY(check_sampler(p));
  std::vector<int64_t> poff;
  TRY(check_partitions(P, partition_offsets, N, poff));
  HIP_TRY(hipSetDevice(c->device));
  const int R = p->learner_end - p->learner_begin;
  uint8_t* d_counts;
  TRY(ws_typed(c, "counts", (size_t)R * std::max<int64_t>(N, 1), &d_counts));
  TRY(run_sampler(c, p, poff, N, d_counts));
  TRY(d2h(c, counts_out, d_counts, (size_t)R * N));
  return SBAG_OK;
}

// ---- dataset ingest.  Three layouts of the DataFrame's features column, one result:
// per-feature sorted dictionaries of the distinct values (-0.0 == 0.0, as Spark's
// `<=` splits and findSplitsBySorting's `!= 0.0` filter see them) and the [N][S] value
// codes in HBM.
//   dense    row-major fp64 [N x F] (DenseVector rows)
//   csr      SparseVector rows: indptr [N+1], strictly increasing indices per row,
//            values; absent entries are 0.0 (HasSubBag.scala:128-131 slices them the
//            same way)
//   columns  one pointer per feature to N values (fp64, fp32 or u8): Arrow / Parquet
//            column chunks, or features quantized upstream
// Codes are built and uploaded in row batches, so no dense fp64 copy of a sparse or
// columnar input is ever made.
struct DsSource {
  int kind = 0;  // 0 dense, 1 csr, 2 columns
  const double* X = nullptr;
  const int64_t* indptr = nullptr;
  const int32_t* indices = nullptr;
  const double* values = nullptr;
  const void* const* cols = nullptr;
  int col_type = SBAG_COL_F64;
  double col(int f, int64_t i) const {
    if (col_type == SBAG_COL_F32) return (double)((const float*)cols[f])[i];
    if (col_type == SBAG_COL_U8) return (double)((const uint8_t*)cols[f])[i];
    return ((const double*)cols[f])[i];
  }
};

static inline double canon(double v) { return v == 0.0 ? 0.0 : v; }  // -0.0 -> 0.0

static int check_source(const DsSource& src, int64_t N, int32_t F) {
  if (src.kind == 1) {
    if (!src.indptr || src.indptr[0] != 0) return fail(SBAG_EINVAL, "indptr must start at 0");
    const int64_t nnz = src.indptr[N];
    if (nnz > 0 && (!src.indices || !src.values)) return fail(SBAG_EINVAL, "bad arguments");
    for (int64_t i = 0; i < N; i++) {
      if (src.indptr[i + 1] < src.indptr[i]) return fail(SBAG_EINVAL, "indptr must be non-decreasing");
      for (int64_t k = src.indptr[i]; k < src.indptr[i + 1]; k++) {
        const int32_t j = src.indices[k];
        if (j < 0 || j >= F || (k > src.indptr[i] && j <= src.indices[k - 1]))
          return fail(SBAG_EINVAL, "row " + std::to_string(i) +
                                       ": indices must be strictly increasing in [0, numFeatures)");
        if (std::isnan(src.values[k])) return fail(SBAG_EINVAL, "NaN feature value");
      }
    }
  } else if (src.kind == 2) {
    if (!src.cols) return fail(SBAG_EINVAL, "bad arguments");
    if (src.col_type != SBAG_COL_F64 && src.col_type != SBAG_COL_F32 && src.col_type != SBAG_COL_U8)
      return fail(SBAG_EINVAL, "unknown column type");
    for (int f = 0; f < F; f++)
      if (!src.cols[f]) return fail(SBAG_EINVAL, "column " + std::to_string(f) + " is NULL");
  } else if (!src.X) {
    return fail(SBAG_EINVAL, "bad arguments");
  }
  return SBAG_OK;
}

static int build_dataset(sbag_ctx* c, int64_t N, int32_t F, const DsSource& src, const double* y,
                         sbag_dataset** out) {
  auto ds = std::make_unique<sbag_dataset>();
  ds->ctx = c;
  ds->N = N;
  ds->F = F;
  ds->S = row_stride(F);
  ds->dict.resize(F);
  ds->zero_code.assign(F, -1);
  // CSR: the explicit values of every feature (a CSC copy of the values only)
  std::vector<int64_t> coff;
  std::vector<double> cval;
  if (src.kind == 1) {
    const int64_t nnz = src.indptr[N];
    coff.assign(F + 1, 0);
    for (int64_t k = 0; k < nnz; k++) coff[src.indices[k] + 1]++;
    for (int f = 0; f < F; f++) coff[f + 1] += coff[f];
    cval.resize((size_t)std::max<int64_t>(nnz, 1));
    std::vector<int64_t> fill(coff.begin(), coff.end() - 1);
    for (int64_t k = 0; k < nnz; k++) cval[fill[src.indices[k]]++] = canon(src.values[k]);
  }
  std::atomic<int> nan_seen{0};
  const int nw = HostPool::width();
  c->pool.run(nw, [&](int w) {
    std::vector<double> col;
    for (int f = w; f < F; f += nw) {
      if (src.kind == 1) {
        col.assign(cval.begin() + coff[f], cval.begin() + coff[f + 1]);
        if (coff[f + 1] - coff[f] < N) col.push_back(0.0);  // implicit zeros
      } else {
        col.resize(N);
        for (int64_t i = 0; i < N; i++) {
          const double v = src.kind == 0 ? src.X[i * F + f] : src.col(f, i);
          if (std::isnan(v)) nan_seen = 1;
          col[i] = canon(v);
        }
      }
      std::sort(col.begin(), col.end());
      col.erase(std::unique(col.begin(), col.end()), col.end());
      ds->dict[f] = col;
    }
  });
  if (nan_seen) return fail(SBAG_EINVAL, "NaN feature value");
  size_t maxd = 0;
  for (int f = 0; f < F; f++) {
    const auto& d = ds->dict[f];
    maxd = std::max(maxd, d.size());
    const auto z = std::lower_bound(d.begin(), d.end(), 0.0);
    if (z != d.end() && *z == 0.0) ds->zero_code[f] = (int)(z - d.begin());
  }
  ds->code_bytes = maxd <= 256 ? 1 : maxd <= 65536 ? 2 : 4;
  const int cb = ds->code_bytes;
  const size_t row_bytes = (size_t)ds->S * cb;
  const size_t bytes = (size_t)N * row_bytes;
  HIP_TRY(hipMalloc(&ds->d_codes, bytes + 256));  // zero slack: k_hist_rl over-reads rows
  HIP_TRY(hipMemset((uint8_t*)ds->d_codes + bytes, 0, 256));
  if (cb == 4) ds->h_codes.resize((size_t)N * ds->S);  // split finding gathers wide codes on the host
  const int64_t batch = std::max<int64_t>(1, std::min<int64_t>(N, ((int64_t)256 << 20) / (int64_t)row_bytes));
  std::vector<uint8_t> buf((size_t)batch * row_bytes);
  std::vector<int> zfill;  // CSR: features whose 0.0 is not code 0 (negative values exist)
  for (int f = 0; f < F; f++)
    if (ds->zero_code[f] > 0) zfill.push_back(f);
  for (int64_t r0 = 0; r0 < N; r0 += batch) {
    const int64_t n = std::min(batch, N - r0);
    c->pool.run(nw, [&](int w) {
      const int64_t a = r0 + n * w / nw, b = r0 + n * (w + 1) / nw;
      for (int64_t i = a; i < b; i++) {
        uint8_t* row = buf.data() + (size_t)(i - r0) * row_bytes;
        auto put = [&](int f, size_t k) {
          if (cb == 1)
            row[f] = (uint8_t)k;
          else if (cb == 2)
            ((uint16_t*)row)[f] = (uint16_t)k;
          else
            ((uint32_t*)row)[f] = (uint32_t)k;
        };
        auto code = [&](int f, double v) {
          const auto& d = ds->dict[f];
          return (size_t)(std::lower_bound(d.begin(), d.end(), canon(v)) - d.begin());
        };
        std::memset(row, 0, row_bytes);
        if (src.kind == 1) {
          for (int f : zfill) put(f, (size_t)ds->zero_code[f]);
          for (int64_t k = src.indptr[i]; k < src.indptr[i + 1]; k++)
            put(src.indices[k], code(src.indices[k], src.values[k]));
        } else {
          for (int f = 0; f < F; f++) put(f, code(f, src.kind == 0 ? src.X[i * F + f] : src.col(f, i)));
        }
      }
    });
    HIP_TRY(hipMemcpy((uint8_t*)ds->d_codes + (size_t)r0 * row_bytes, buf.data(), (size_t)n * row_bytes,
                      hipMemcpyHostToDevice));
    if (cb == 4) std::memcpy((uint8_t*)ds->h_codes.data() + (size_t)r0 * row_bytes, buf.data(), (size_t)n * row_bytes);
  }
  ds->lab.y.assign(y, y + N);
  analyze_labels(ds.get());
  TRY(upload_labels(ds.get()));
  TRY(upload_dict(ds.get()));
  *out = ds.release();
  return SBAG_OK;
}

static int dataset_from(sbag_ctx* c, int64_t N, int32_t F, const DsSource& src, const double* y,
                        sbag_dataset** out) {
  if (!c || !out || N < 0 || F <= 0 || (N > 0 && !y)) return fail(SBAG_EINVAL, "bad arguments");
  if (N == 0) return fail(SBAG_EEMPTY, "ML algorithm was given empty dataset.");
  if (N >= (int64_t)1 << 32) return fail(SBAG_EUNSUPPORTED, "more than 2^32 rows");
  TRY(check_source(src, N, F));
  CTX_LOCK(c);
  HIP_TRY(hipSetDevice(c->device));
  return build_dataset(c, N, F, src, y, out);
}

int sbag_dataset_create(sbag_ctx* c, int64_t N, int32_t F, const double* X, const double* y,
                        sbag_dataset** out) {
  DsSource src;
  src.kind = 0;
  src.X = X;
  return dataset_from(c, N, F, src, y, out);
}

int sbag_dataset_create_csr(sbag_ctx* c, int64_t N, int32_t F, const int64_t* indptr,
                            const int32_t* indices, const double* values, const double* y,
                            sbag_dataset** out) {
  DsSource src;
  src.kind = 1;
  src.indptr = indptr;
  src.indices = indices;
  src.values = values;
  return dataset_from(c, N, F, src, y, out);
}

int sbag_dataset_create_columns(sbag_ctx* c, int64_t N, int32_t F, int32_t col_type,
                                const void* const* columns, const double* y, sbag_dataset** out) {
  DsSource src;
  src.kind = 2;
  src.cols = columns;
  src.col_type = col_type;
  return dataset_from(c, N, F, src, y, out);
}

int sbag_dataset_synthetic(sbag_ctx* c, int64_t N, int32_t F, uint64_t seed, int32_t num_classes,
                           sbag_dataset** out) {
  if (!c || !out || N <= 0 || F <= 0 || num_classes < 0 || num_classes > 256)
    return fail(SBAG_EINVAL, "bad arguments");
  if (N >= (int64_t)1 << 32) return fail(SBAG_EUNSUPPORTED, "more than 2^32 rows");
  CTX_LOCK(c);
  HIP_TRY(hipSetDevice(c->device));
  auto ds = std::make_unique<sbag_dataset>();
  ds->ctx = c;
  ds->N = N;
  ds->F = F;
  ds->S = row_stride(F);
  ds->code_bytes = 1;
  ds->dict.assign(F, std::vector<double>(32));
  for (int f = 0; f < F; f++)
    for (int v = 0; v < 32; v++) ds->dict[f][v] = (double)v;
  ds->zero_code.assign(F, 0);
  HIP_TRY(hipMalloc(&ds->d_codes, (size_t)N * ds->S + 256));
  HIP_TRY(hipMemset((uint8_t*)ds->d_codes + (size_t)N * ds->S, 0, 256));
  HIP_TRY(hipMalloc(&ds->lab.d_labk, (size_t)N * 4));
  launch_synth(c->stream, (uint8_t*)ds->d_codes, ds->S, N, F, seed, num_classes, ds->lab.d_labk);
  HIP_TRY(hipGetLastError());
  std::vector<int32_t> k(N);
  TRY(d2h(c, k.data(), ds->lab.d_labk, (size_t)N));
  ds->lab.shift = num_classes ? 0 : 6;
  ds->lab.y.resize(N);
  ds->lab.kmin = ds->lab.kmax = k[0];
  for (int64_t i = 0; i < N; i++) {
    ds->lab.y[i] = std::ldexp((double)k[i], -ds->lab.shift);
    ds->lab.kmin = std::min<int64_t>(ds->lab.kmin, k[i]);
    ds->lab.kmax = std::max<int64_t>(ds->lab.kmax, k[i]);
    ds->lab.ymax_abs = std::max(ds->lab.ymax_abs, std::fabs(ds->lab.y[i]));
    ds->lab.ymax_sq = std::max(ds->lab.ymax_sq, ds->lab.y[i] * ds->lab.y[i]);
  }
  ds->lab.label_ok = true;
  ds->lab.integral = ds->lab.kmin >= 0 && num_classes > 0;
  if (num_classes == 0) {
    ds->lab.integral = true;
    for (int64_t i = 0; i < N && ds->lab.integral; i++)
      if (ds->lab.y[i] < 0 || ds->lab.y[i] != std::floor(ds->lab.y[i])) ds->lab.integral = false;
  }
  TRY(upload_dict(ds.get()));
  *out = ds.release();
  return SBAG_OK;
}

int sbag_dataset_info(const sbag_dataset* ds, int64_t* N, int32_t* F) {
  if (!ds) return fail(SBAG_EINVAL, "dataset is NULL");
  if (N) *N = ds->N;
  if (F) *F = ds->F;
  return SBAG_OK;
}

int sbag_dataset_labels(const sbag_dataset* ds, double* y) {
  if (!ds || !y) return fail(SBAG_EINVAL, "bad arguments");
  std::copy(ds->lab.y.begin(), ds->lab.y.end(), y);
  return SBAG_OK;
}

// The label column replaced in place (Spark: a new DataFrame whose labelCol differs; the
// features' codes and dictionaries are kept)
int sbag_dataset_set_labels(sbag_dataset* ds, const double* y) {
  if (!ds || !y) return fail(SBAG_EINVAL, "bad arguments");
  sbag_ctx* c = ds->ctx;
  CTX_LOCK(c);
  HIP_TRY(hipSetDevice(c->device));
  std::lock_guard<std::mutex> lk(ds->layout_mu);
  HIP_TRY(hipStreamSynchronize(c->stream));  // no fit of this context still reads the labels
  ds->lab.y.assign(y, y + ds->N);
  analyze_labels(ds);
  if (ds->lab.d_labk) HIP_TRY(hipFree(ds->lab.d_labk));
  ds->lab.d_labk = nullptr;
  TRY(upload_labels(ds));
  if (ds->lab.d_y64) HIP_TRY(hipFree(ds->lab.d_y64));
  ds->lab.d_y64 = nullptr;
  return SBAG_OK;
}

// ---- replication of an ingested dataset to another device: the value codes
// (device), the dictionaries and the labels, so that one rank ingests and the others
// receive the binned matrix over RCCL (or a host copy) instead of re-ingesting rows
int sbag_dataset_layout(const sbag_dataset* ds, int64_t* num_rows, int32_t* num_features,
                        int32_t* row_stride, int32_t* code_bytes, int64_t* dict_values) {
  if (!ds) return fail(SBAG_EINVAL, "dataset is NULL");
  if (num_rows) *num_rows = ds->N;
  if (num_features) *num_features = ds->F;
  if (row_stride) *row_stride = ds->S;
  if (code_bytes) *code_bytes = ds->code_bytes;
  if (dict_values) {
    int64_t t = 0;
    for (const auto& d : ds->dict) t += (int64_t)d.size();
    *dict_values = t;
  }
  return SBAG_OK;
}

int sbag_dataset_export(const sbag_dataset* ds, void* codes, int32_t codes_on_device, double* dict,
                        int64_t* dict_off, double* y) {
  if (!ds) return fail(SBAG_EINVAL, "dataset is NULL");
  sbag_ctx* c = ds->ctx;
  CTX_LOCK(c);
  HIP_TRY(hipSetDevice(c->device));
  if (codes) {
    const size_t bytes = (size_t)ds->N * ds->S * ds->code_bytes;
    HIP_TRY(hipMemcpyAsync(codes, ds->d_codes, bytes,
                           codes_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  if (dict_off) {
    dict_off[0] = 0;
    for (int f = 0; f < ds->F; f++) dict_off[f + 1] = dict_off[f] + (int64_t)ds->dict[f].size();
  }
  if (dict) {
    int64_t o = 0;
    for (const auto& d : ds->dict) {
      std::copy(d.begin(), d.end(), dict + o);
      o += (int64_t)d.size();
    }
  }
  if (y) std::copy(ds->lab.y.begin(), ds->lab.y.end(), y);
  return SBAG_OK;
}

int sbag_dataset_import(sbag_ctx* c, int64_t N, int32_t F, int32_t S, int32_t cb, const void* codes,
                        int32_t codes_on_device, const double* dict, const int64_t* dict_off,
                        const double* y, sbag_dataset** out) {
  if (!c || !out || !codes || !dict || !dict_off || !y || N <= 0 || F <= 0)
    return fail(SBAG_EINVAL, "bad arguments");
  if (N >= (int64_t)1 << 32) return fail(SBAG_EUNSUPPORTED, "more than 2^32 rows");
  if (S != row_stride(F)) return fail(SBAG_EINVAL, "row stride does not match the engine's layout");
  if (dict_off[0] != 0) return fail(SBAG_EINVAL, "dictionary offsets must start at 0");
  size_t maxd = 0;
  for (int f = 0; f < F; f++) {
    if (dict_off[f + 1] <= dict_off[f]) return fail(SBAG_EINVAL, "every feature needs a dictionary");
    maxd = std::max(maxd, (size_t)(dict_off[f + 1] - dict_off[f]));
    for (int64_t k = dict_off[f]; k < dict_off[f + 1]; k++) {
      const double v = dict[k];
      if (std::isnan(v) || (v == 0.0 && std::signbit(v)) || (k > dict_off[f] && !(dict[k - 1] < v)))
        return fail(SBAG_EINVAL, "dictionaries must be strictly increasing, without NaN or -0.0");
    }
  }
  if (cb != (maxd <= 256 ? 1 : maxd <= 65536 ? 2 : 4))
    return fail(SBAG_EINVAL, "code width does not match the dictionaries");
  CTX_LOCK(c);
  HIP_TRY(hipSetDevice(c->device));
  auto ds = std::make_unique<sbag_dataset>();
  ds->ctx = c;
  ds->N = N;
  ds->F = F;
  ds->S = S;
  ds->code_bytes = cb;
  ds->dict.resize(F);
  ds->zero_code.assign(F, -1);
  for (int f = 0; f < F; f++) {
    ds->dict[f].assign(dict + dict_off[f], dict + dict_off[f + 1]);
    const auto& d = ds->dict[f];
    const auto z = std::lower_bound(d.begin(), d.end(), 0.0);
    if (z != d.end() && *z == 0.0) ds->zero_code[f] = (int)(z - d.begin());
  }
  const size_t bytes = (size_t)N * S * cb;
  HIP_TRY(hipMalloc(&ds->d_codes, bytes + 256));
  HIP_TRY(hipMemsetAsync((uint8_t*)ds->d_codes + bytes, 0, 256, c->stream));
  HIP_TRY(hipMemcpyAsync(ds->d_codes, codes, bytes,
                         codes_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
  TRY(upload_dict(ds.get()));
  int* d_bad;
  TRY(ws_typed(c, "import_bad", 1, &d_bad));
  HIP_TRY(hipMemsetAsync(d_bad, 0, 4, c->stream));
  launch_check_codes(c->stream, ds->d_codes, cb, N, S, F, ds->d_dict_off, d_bad);
  HIP_TRY(hipGetLastError());
  int bad = 0;
  TRY(d2h(c, &bad, d_bad, 1));
  if (bad) return fail(SBAG_EINVAL, "imported codes exceed their dictionaries (or padding is not zero)");
  if (cb == 4) {
    ds->h_codes.resize((size_t)N * S);
    HIP_TRY(hipMemcpy(ds->h_codes.data(), ds->d_codes, bytes, hipMemcpyDeviceToHost));
  }
  ds->lab.y.assign(y, y + N);
  analyze_labels(ds.get());
  TRY(upload_labels(ds.get()));
  *out = ds.release();
  return SBAG_OK;
}

int sbag_dataset_features(const sbag_dataset* ds, int64_t r0, int64_t r1, double* X) {
  if (!ds || !X || r0 < 0 || r1 > ds->N || r1 < r0) return fail(SBAG_EINVAL, "bad arguments");
  sbag_ctx* c = ds->ctx;
  CTX_LOCK(c);
  HIP_TRY(hipSetDevice(c->device));
  const int64_t n = r1 - r0;
  std::vector<uint8_t> buf((size_t)n * ds->S * ds->code_bytes);
  HIP_TRY(hipMemcpy(buf.data(), (const uint8_t*)ds->d_codes + (size_t)r0 * ds->S * ds->code_bytes,
                    buf.size(), hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < n; i++)
    for (int f = 0; f < ds->F; f++) {
      const size_t k = ds->code_bytes == 1   ? buf[(size_t)i * ds->S + f]
                       : ds->code_bytes == 2 ? ((uint16_t*)buf.data())[(size_t)i * ds->S + f]
                                             : ((uint32_t*)buf.data())[(size_t)i * ds->S + f];
      X[i * ds->F + f] = ds->dict[f][k];
    }
  return SBAG_OK;
}

int sbag_dataset_free(sbag_dataset* ds) {
  if (!ds) return SBAG_OK;
  CTX_LOCK(ds->ctx);
  (void)hipSetDevice(ds->ctx->device);
  (void)hipStreamSynchronize(ds->ctx->stream);
  delete ds;  // ~sbag_dataset frees the device buffers
  return SBAG_OK;
}

// ---------------------------------------------------------------- fit
struct HistGeom {
  bool grouped = false;  // gini class tiles over entries grouped by tile (group_tiles)
  int T, FT, FPH, ntf, CT, ntiles;
  int rl;  // row-lane kernel (k_hist_rl)
  size_t lds;
};

static int roundup(int x, int a) { return (x + a - 1) / a * a; }

// LDS geometry of one k_hist workgroup: FT features (lane groups of 64) and, for
// gini, CT class planes.  Aim at <= 80 KB (two 512-thread workgroups per CU).
// Many classes (BASELINE config 5: 64) are split into class tiles first: a class
// tile re-reads the 8-byte entries but loads the row bytes of its own entries only,
// whereas a feature tile re-reads every row.
// grouped: gini class tiles over entries grouped by tile (no staging area; a smaller LDS
// target so that four workgroups share a CU and keep more row gathers in flight)
static bool hist_geometry(int S, int Fmax, int NB, int NS, bool gini_layout, HistGeom& g,
                          int rl_mode = 0, bool grouped = false) {
  (void)S;
  g.T = 64;  // piece granularity (entries)
  const int align = gini_layout ? 32 : 16;
  size_t soft = grouped ? 38 * 1024 : 80 * 1024;
  if (const char* e = getenv(grouped ? "SBAG_HIST_GROUPED_LDS_KB" : "SBAG_HIST_LDS_KB"))
    soft = (size_t)atoi(e) * 1024;
  const size_t hard = 160 * 1024 - 256;
  const size_t stage = grouped ? 0 : hist_stage_bytes();
  auto lds_for = [&](int ft, int ct) {
    size_t b = hist_lds_bytes(NB, gini_layout ? ct : 1, roundup(ft, align), gini_layout);
    if (gini_layout && ct < NS) b += stage;
    return b;
  };
  int ft = std::min(256, roundup(Fmax, align));
  int ct = gini_layout ? NS : 1;
  for (;;) {
    if (!gini_layout) {
      if (lds_for(ft, 1) <= soft || ft <= align) break;
      ft -= align;
      continue;
    }
    const size_t P = hist_lds_bytes(NB, 1, roundup(ft, align), true);
    if ((size_t)NS * P <= soft) {
      ct = NS;
      break;
    }
    const long c = soft > stage ? (long)((soft - stage) / P) : 0;
    if (c >= 1) {
      const int nct = (NS + (int)c - 1) / (int)c;
      ct = (NS + nct - 1) / nct;  // balanced class tiles
      break;
    }
    if (ft <= align) {
      ct = 1;
      break;
    }
    ft -= align;
  }
  if (lds_for(ft, ct) > hard) return false;
  g.FT = std::min(ft, Fmax);
  g.FPH = roundup(g.FT, align);
  g.CT = ct;
  g.ntf = (Fmax + g.FT - 1) / g.FT;
  g.ntiles = g.ntf * ((gini_layout ? (NS + ct - 1) / ct : 1));
  g.lds = lds_for(g.FT, ct);
  g.rl = 0;
  // row lanes when they carry fewer dump lanes than 64-feature lane groups
  // (SBAG_HIST_RL_FORCE=1: whenever the layout allows them, for A/B)
  static const bool rl_force = getenv("SBAG_HIST_RL_FORCE") && atoi(getenv("SBAG_HIST_RL_FORCE")) != 0;
  if (rl_mode && (rl_force || roundup(g.FT, hist_rl_lanes()) < roundup(g.FT, 64))) {
    const size_t b = hist_rl_lds_bytes(NB, ct, g.FPH, gini_layout);
    if (b <= hard) {
      g.rl = rl_mode;
      g.lds = b;
    }
  }
  return true;
}

// Work of one histogram launch: pieces (slices of parent segments, parent order)
// and a balanced contiguous piece range per workgroup.
struct HistWork {
  std::vector<HistChunk> pieces;
  std::vector<int32_t> wg;
  int nwg = 0;
  double entries = 0;
};

static void build_work(const std::vector<std::pair<int64_t, int64_t>>& segs, int64_t ps_max,
                       int nwg_max, int T, HistWork& w) {
  int64_t tot = 0;
  for (auto& s : segs) tot += s.second - s.first;
  int64_t ps = tot / std::max<int64_t>(1, 2 * (int64_t)nwg_max);
  ps = std::max<int64_t>(T, std::min<int64_t>(ps_max, (ps + T - 1) / T * T));
  w.pieces.clear();
  w.pieces.reserve(segs.size() + (size_t)(tot / ps) + 1);
  for (size_t q = 0; q < segs.size(); q++)
    for (int64_t a = segs[q].first; a < segs[q].second; a += ps)
      w.pieces.push_back(HistChunk{(int32_t)q, 0, a, std::min(a + ps, segs[q].second), 0, 0, 0, 0});
  const int np = (int)w.pieces.size();
  w.nwg = std::max(1, std::min(np, nwg_max));
  w.wg.assign(w.nwg + 1, np);
  w.wg[0] = 0;
  int64_t run = 0;
  int cur = 0;
  for (int p = 0; p < np; p++) {
    const int64_t len = w.pieces[p].b - w.pieces[p].a;
    int target = tot > 0 ? (int)(((double)run + 0.5 * len) * w.nwg / (double)tot) : 0;
    target = std::min(std::max(target, cur), w.nwg - 1);
    while (cur < target) w.wg[++cur] = p;
    run += len;
  }
  while (cur < w.nwg) w.wg[++cur] = np;
  // a segment whose pieces all fall in one workgroup is flushed with plain stores
  std::vector<int> wg_of(np);
  for (int g = 0; g < w.nwg; g++)
    for (int p = w.wg[g]; p < w.wg[g + 1]; p++) wg_of[p] = g;
  for (int p0 = 0; p0 < np;) {
    int p1 = p0;
    while (p1 < np && w.pieces[p1].parent == w.pieces[p0].parent) p1++;
    const int ex = wg_of[p0] == wg_of[p1 - 1] ? 1 : 0;
    for (int p = p0; p < p1; p++) w.pieces[p].excl = ex;
    p0 = p1;
  }
  w.entries = (double)tot;
}

// fit_range's request to be called again on halves of its learner range: per-replica bins
// (thresholds that differ across replicas) of all its replicas exceed the device budget
static constexpr int kSplitRange = -1000;
// fit_range_impl's integer engine cannot hold the dyadic labels' sums exactly (the packed
// LDS word or the 2^53 bound on the sum of squares): fit_range refits on the fp64 engine
static constexpr int kIntRange = -1001;
// rows the fp64 engine (real-valued regression labels) accepts: the largest size it is tested at
static constexpr int64_t kF64MaxRows = (int64_t)1 << 30;

// device bytes per-replica bins may take: SBAG_BINS_BUDGET_MB, else 40 % of the device
static double bins_budget(sbag_ctx* c) {
  if (const char* e = getenv("SBAG_BINS_BUDGET_MB"))
    return atof(e) * (1 << 20) / std::max(1, c->concurrent_parts);
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    return 48.0 * (1ull << 30);
  }
  return 0.4 * (double)tot / std::max(1, c->concurrent_parts);
}

// sbag_fit_booster's base-learner fit: one learner whose bag, subspace and labels are given
// (GBM*.train: the iteration's bag column, its subspace, the pseudo-residuals)
struct FitExt {
  const uint8_t* counts;  // host [N]
  std::vector<int32_t> sub;
  const LabelSet* lab;    // labels with their device images
};
static int fit_range(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out,
                     const FitExt* ext = nullptr);

// Bins are u8 codes, so a feature may have at most 256 bins (255 thresholds).  Spark's
// findSplitsForContinuousFeature can return maxBins thresholds when the split-finding sample
// (subbags above max(maxBins^2, 10^4) rows) holds more nonzero values than numSamples; with
// maxBins = 256 that is 257 bins.  Whether it happens depends on the sample (the seed), so
// the combination that allows it -- maxBins 256, more than 65536 rows, a feature with more
// than 255 distinct values -- is refused up front, for every seed.  (Below 65536 rows a
// bag only reaches the sample when a with-replacement draw exceeds 65536 rows; the 257th
// bin is then still refused when it occurs.)
static int check_bins256(const sbag_tree_params& tp, int64_t rows, int max_distinct) {
  if (tp.max_bins == 256 && rows > 65536 && max_distinct > 255)
    return fail(SBAG_EUNSUPPORTED, "maxBins 256 on more than 65536 rows with a feature of more than 255 "
                                   "distinct values: Spark's split-finding sample may return 256 "
                                   "thresholds (257 bins) and bins are u8 codes; use maxBins <= 255");
  return SBAG_OK;
}

// Learners are independent (seed + i per learner), so a range whose per-replica
// bins do not fit is fitted as two halves and the trees concatenated in learner order.
// sum of two forests' learner-ordered trees and timings (a then b)
static void merge_forests(sbag_forest* fa, sbag_forest* fb) {
  for (auto& t : fb->trees) fa->trees.push_back(std::move(t));
  fa->nclasses = std::max(fa->nclasses, fb->nclasses);
  sbag_timing& T = fa->timing;
  const sbag_timing& U = fb->timing;
  T.total_ms += U.total_ms;
  T.sample_ms += U.sample_ms;
  T.valuecount_ms += U.valuecount_ms;
  T.bin_ms += U.bin_ms;
  T.compact_ms += U.compact_ms;
  T.hist_ms += U.hist_ms;
  T.split_ms += U.split_ms;
  T.subtract_ms += U.subtract_ms;
  T.hist_launches += U.hist_launches;
  T.hist_alg_bytes += U.hist_alg_bytes;
  T.hist_entries += U.hist_entries;
  T.hist_upper_bytes += U.hist_upper_bytes;
  T.levels = std::max(T.levels, U.levels);
  T.partition_ms += U.partition_ms;
  T.hist_work_bytes += U.hist_work_bytes;
  T.fix_ms += U.fix_ms;
  T.exact_fallbacks += U.exact_fallbacks;
  T.hist_lds_atomics += U.hist_lds_atomics;
  T.group_ms += U.group_ms;
}

// Two learner parts run side by side only when both workspaces fit the device next to what
// is already allocated: per replica the counts (N bytes) and the two entry buffers (16 N),
// plus the histogram slots.  C4's shard (10^8 rows, 64 learners: 2 x 54 GB) qualifies on a
// 288-GB MI355X; the context's own workspace is reused by its part.
static bool overlap_fits(sbag_ctx* c, const sbag_dataset* ds, int learners) {
  size_t fr = 0, tot = 0;
  if (hipSetDevice(c->device) != hipSuccess || hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  double mine = 0;  // this context's and its twins' workspaces are reused by the parts
  for (const auto& kv : c->ws) mine += (double)kv.second.cap;
  for (const sbag_ctx* t : c->twins)
    for (const auto& kv : t->ws) mine += (double)kv.second.cap;
  // bytes per (learner, row): the count and two 8-byte entry buffers; with fp64 labels
  // (§4.7) also the carried labels, the kept bins and the buckets of the chosen and first
  // features (C4 shape: the halves did not fit side by side, 2829 vs 2586 ms serialized)
  const double per = ds->lab.label_ok ? 17.0 : 45.0;
  const double part = (double)((learners + 1) / 2) * (double)ds->N * per + (double)(1ull << 30);
  return 2.0 * part <= 0.9 * ((double)fr + mine);
}

static int fit_learners_halving(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out);
static int fit_halves(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out);
// one context: fit_range, or halves of the learner range when per-replica bins exceed
// the device budget (learners are independent, so concatenation is exact)
static int fit_learners(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out) {
  // Continuous features (more distinct values than maxBins) get thresholds of their own per
  // replica, so their bins are materialized per replica: when those of the whole range
  // exceed the budget, split it up front into parts that fit -- a fit_range that finds out
  // only after the sampling and the split finding would redo them for every halving
  // (C3-sized continuous fit: 3 wasted attempts)
  {
    const int lb = fp->sampler.learner_begin, le = fp->sampler.learner_end;
    bool cont = false;
    for (const auto& d : ds->dict) cont = cont || (int64_t)d.size() > fp->tree.max_bins;
    // (every replica holds every row once -- bags without replacement at ratio 1 -- : the
    // thresholds are shared and one bins matrix serves all)
    const bool whole = !fp->sampler.replacement && fp->sampler.sample_ratio >= 1.0;
    if (cont && le - lb > 1 && !whole) {
      // the per-replica rows hold the subspace's features (not all of them), and
      // with integer labels only the in-bag rows (k_bin_ranked): 1 - e^-ratio of them for
      // Poisson bags, the ratio for Bernoulli ones (a short estimate falls back to halving)
      // (fit_range_impl's conditions: not the fp64 engine -- gini, or integer labels without
      // SBAG_F64=1 --, and k_bin_ranked's LDS geometry for a cut table of up to maxBins cuts;
      // the estimate had missed the last one)
      const bool force_f64 = getenv("SBAG_F64") && atoi(getenv("SBAG_F64")) != 0;
      const bool gini = fp->tree.impurity == SBAG_IMPURITY_GINI;
      bool ranked = (gini || (ds->lab.label_ok && !force_f64)) &&
                    (!getenv("SBAG_BIN_RANKED") || atoi(getenv("SBAG_BIN_RANKED")) != 0);
      const double ratio = fp->sampler.sample_ratio;
      const double frac = std::min(1.0, (fp->sampler.replacement ? 1.0 - std::exp(-ratio) : ratio) * 1.02 + 1e-3);
      const double sratio = fp->subspace_bug_compat ? fp->sampler.sample_ratio : fp->subspace_ratio;
      int fmax = 0;
      std::vector<int32_t> idx(ds->F);
      for (int l = lb; l < le; l++) {
        int n = 0;
        if (sbag_subspace(sratio, ds->F, (int64_t)((uint64_t)fp->sampler.seed + (uint64_t)(int64_t)l), idx.data(),
                          &n) != SBAG_OK) {
          fmax = ds->F;
          break;
        }
        fmax = std::max(fmax, n);
      }
      fmax = std::max(fmax, 1);
      {
        int32_t ncp = 32;
        while (ncp < fp->tree.max_bins) ncp *= 2;
        ranked = ranked && bin_ranked_fits(ds->code_bytes, ds->S, row_stride(fmax), fmax, ncp);
      }
      const double rows = (ranked ? frac : 1.0) * (double)ds->N + 192.0;
      const double per = rows * row_stride(fmax) + (double)fmax * rows;
      const double budget = bins_budget(c);
      const int fitn = (int)std::max(1.0, std::floor(budget / per));
      if (fitn < le - lb) {
        const int parts = (le - lb + fitn - 1) / fitn;
        std::unique_ptr<sbag_forest> acc;
        for (int k = 0; k < parts; k++) {
          sbag_fit_params h = *fp;
          h.sampler.learner_begin = lb + (int)((int64_t)(le - lb) * k / parts);
          h.sampler.learner_end = lb + (int)((int64_t)(le - lb) * (k + 1) / parts);
          sbag_forest* f = nullptr;
          {
            const int st = fit_range(c, ds, &h, &f);
            if (st == kSplitRange) {  // the estimate was short: halve this part (not refit it whole)
              TRY(fit_halves(c, ds, &h, &f));
            } else {
              TRY(st);
            }
          }
          std::unique_ptr<sbag_forest> ff(f);
          if (!acc) {
            acc = std::move(ff);
          } else {
            merge_forests(acc.get(), ff.get());
          }
        }
        *out = acc.release();
        return SBAG_OK;
      }
    }
  }
  return fit_learners_halving(c, ds, fp, out);
}

static int fit_learners_halving(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out) {
  const int st = fit_range(c, ds, fp, out);
  if (st != kSplitRange) return st;
  return fit_halves(c, ds, fp, out);
}

// the two halves of a learner range that fit_range refused whole, concatenated in learner order
static int fit_halves(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out) {
  const int lb = fp->sampler.learner_begin, le = fp->sampler.learner_end, mid = lb + (le - lb) / 2;
  sbag_fit_params h = *fp;
  h.sampler.learner_end = mid;
  sbag_forest* a = nullptr;
  TRY(fit_learners_halving(c, ds, &h, &a));
  std::unique_ptr<sbag_forest> fa(a);
  h.sampler.learner_begin = mid;
  h.sampler.learner_end = le;
  sbag_forest* b = nullptr;
  TRY(fit_learners_halving(c, ds, &h, &b));
  std::unique_ptr<sbag_forest> fb(b);
  merge_forests(fa.get(), fb.get());
  *out = fa.release();
  return SBAG_OK;
}

int sbag_fit(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out) {
  if (!c || !ds || !fp || !out) return fail(SBAG_EINVAL, "bad arguments");
  if (ds->ctx->device != c->device)
    return fail(SBAG_EINVAL, "dataset lives on device " + std::to_string(ds->ctx->device) +
                                 ", the context on device " + std::to_string(c->device));
  CTX_LOCK(c);
  const int lb = fp->sampler.learner_begin, le = fp->sampler.learner_end;
  // The two halves of the learner range on two streams from two threads: while one half's
  // host thread turns a level's split results into the next level's work lists, the
  // other half's kernels run (C3: 150 -> 136 ms per fit, C5 shard 265 -> 238).  Each
  // context keeps its own copy of the dataset-derived buffers (column copy, side-bit
  // planes: C4's 100M x 256 would need 2 x 125 GB), so by default only fits of up to 2^26
  // rows with at least 16 learners overlap; SBAG_OVERLAP=0/1
  // forces it off / on; SBAG_OVERLAP=k runs k parts (3 and 4 were slower on C3: 151, 152 ms).
  const char* ov = getenv("SBAG_OVERLAP");
  int parts = ov ? atoi(ov) : ((le - lb >= 16 && ds->N >= (1 << 20) && overlap_fits(c, ds, le - lb)) ? 2 : 0);
  if (parts == 1) parts = 2;  // SBAG_OVERLAP=1: on, two parts
  parts = std::min(parts, le - lb);
  if (parts < 2) return fit_learners(c, ds, fp, out);
  while ((int)c->twins.size() < parts - 1) {
    sbag_ctx* t = nullptr;
    TRY(sbag_ctx_create(c->device, &t));
    c->twins.push_back(t);
  }
  std::vector<sbag_fit_params> hp(parts, *fp);
  for (int k = 0; k < parts; k++) {
    hp[k].sampler.learner_begin = lb + (int)((int64_t)(le - lb) * k / parts);
    hp[k].sampler.learner_end = lb + (int)((int64_t)(le - lb) * (k + 1) / parts);
  }
  std::vector<sbag_forest*> fs(parts, nullptr);
  std::vector<int> sts(parts, SBAG_OK);
  std::vector<std::string> errs(parts);
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  // the parts share the device: each one's per-replica bins take a 1/parts budget
  c->concurrent_parts = parts;
  for (int k = 1; k < parts; k++) c->twins[k - 1]->concurrent_parts = parts;
  for (int k = 1; k < parts; k++)
    th.emplace_back([&, k] {
      sbag_ctx* t = c->twins[k - 1];
      CTX_LOCK(t);
      (void)hipSetDevice(c->device);
      sts[k] = fit_learners(t, ds, &hp[k], &fs[k]);
      if (sts[k] != SBAG_OK) errs[k] = g_err;  // g_err is thread-local
    });
  sts[0] = fit_learners(c, ds, &hp[0], &fs[0]);
  for (auto& t : th) t.join();
  const auto tj = std::chrono::steady_clock::now();
  c->concurrent_parts = 1;
  for (int k = 1; k < parts; k++) c->twins[k - 1]->concurrent_parts = 1;
  std::vector<std::unique_ptr<sbag_forest>> own;
  for (auto* f : fs) own.emplace_back(f);
  bool oom = false;
  for (int k = 0; k < parts; k++) oom = oom || sts[k] == SBAG_ENOMEM;
  if (oom) {
    // two workspaces did not fit next to each other: release the twins' device memory and
    // fit the whole range serially on this context (the result is the same forest)
    for (int k = 1; k < parts; k++) {
      sbag_ctx* t = c->twins[k - 1];
      CTX_LOCK(t);
      (void)hipSetDevice(c->device);
      ws_release(t);
    }
    own.clear();
    return fit_learners(c, ds, fp, out);
  }
  if (sts[0] != SBAG_OK) return sts[0];
  for (int k = 1; k < parts; k++)
    if (sts[k] != SBAG_OK) return fail(sts[k], errs[k]);
  for (int k = 1; k < parts; k++) merge_forests(own[0].get(), own[k].get());
  // the parts ran concurrently: the fit took the wall time, not the sum
  own[0]->timing.total_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (getenv("SBAG_PROFILE_HOST"))
    fprintf(stderr, "host ms: parts wall %.2f, joined -> merged %.2f\n", own[0]->timing.total_ms,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tj).count());
  *out = own[0].release();
  return SBAG_OK;
}

// ---------------------------------------------------------------- fp64-stat trees
// LearningNode with fp64 ImpurityStats: the booster engine (sbag_fit_booster) and the
// bagging engine's row-order path for labels that are not dyadic (fit_range, f64 mode)
namespace {
struct BtNode {  // LearningNode with fp64 ImpurityStats
  int left = -1, right = -1;
  bool is_leaf = false, has_split = false, valid = true;
  int fl = -1, s = -1;
  double thr = 0.0;
  double calc[3] = {0, 0, 0};  // stats.impurityCalculator (count, sum, sumSq)
  double impurity = 0.0, gain = NAN;
};

double bt_count(const double* s) { return s[0]; }
// Variance.calculate (count, sum, sumSq)
double bt_impurity(const double* s) {
  const double count = s[0], sum = s[1], sumsq = s[2];
  if (count == 0) return 0.0;
  const double squared_loss = sumsq - (sum * sum) / count;
  return squared_loss / count;
}
// VarianceCalculator.predict: sum / count (count as a Long)
double bt_predict(const double* s) {
  const int64_t cnt = (int64_t)s[0];
  if (cnt == 0) return 0.0;
  return s[1] / (double)cnt;
}

// LearningNode.toNode(prune = true), NodeData pre-order
struct BtRet {
  bool leaf;
  double pred;
};
BtRet bt_emit(const std::vector<BtNode>& nodes, int idx, HTree& t) {
  const BtNode& n = nodes[idx];
  const int my = (int)t.nodes.size();
  t.nodes.push_back(sbag_node{});
  t.stats.resize((size_t)(my + 1) * 3);
  auto fill = [&](int at) {
    for (int i = 0; i < 3; i++) t.stats[(size_t)at * 3 + i] = n.calc[i];
  };
  if (n.has_split) {
    const size_t mark = t.nodes.size();
    const int lid = (int)t.nodes.size();
    BtRet l = bt_emit(nodes, n.left, t);
    const int rid = (int)t.nodes.size();
    BtRet r = bt_emit(nodes, n.right, t);
    if (l.leaf && r.leaf && l.pred == r.pred) {
      t.nodes.resize(mark);
      t.stats.resize(mark * 3);
      sbag_node& p = t.nodes[my];
      p = sbag_node{};
      p.id = my;
      p.left = p.right = -1;
      p.feature = -1;
      p.split_bin = -1;
      p.prediction = l.pred;
      p.impurity = n.impurity;
      p.gain = -1.0;
      fill(my);
      return {true, l.pred};
    }
    sbag_node& o = t.nodes[my];
    o.id = my;
    o.left = lid;
    o.right = rid;
    o.feature = n.fl;
    o.split_bin = n.s;
    o.threshold = n.thr;
    o.prediction = bt_predict(n.calc);
    o.impurity = n.impurity;
    o.gain = n.gain;
    fill(my);
    return {false, o.prediction};
  }
  sbag_node& o = t.nodes[my];
  o.id = my;
  o.left = o.right = -1;
  o.feature = -1;
  o.split_bin = -1;
  o.prediction = bt_predict(n.calc);
  o.impurity = n.valid ? n.impurity : -1.0;
  o.gain = -1.0;
  fill(my);
  return {true, o.prediction};
}

}  // namespace

// fp64 labels (sbag_f64s.hip): level-wise growth whose node statistics are
// Spark's row-order fp64 sums.  Every level:
//   1. k_f64_screen picks each node's split from the integer histograms of the labels'
//      fixed-point image (built like the dyadic engine's: smaller child + subtraction)
//      when a rigorous bound proves it is binsToBestSplit's choice; other nodes are
//      flagged and histogrammed exactly (k_f64_hist over every feature in row order, then
//      k_f64_split);
//   2. k_fb_* buckets every decided node's entries by the chosen feature's bin (at the root
//      also by the first feature with splits, whose bins give Spark's parent stats), sums
//      each bucket in row order, and routes every split node's entries stably into its
//      children (their entries stay in row order);
//   3. k_fb_finish evaluates the chosen feature exactly: gain, impurity, children stats.
// Error bounds (host, per node): Spark's sums of n terms carry at most gamma_K sum|term|,
// K = n + NB + 2 additions per term, gamma_K = K u / (1 - K u); a right child's stats
// (total - left) carry the parent's total's error.  See DESIGN §4.7 for the derivation.
struct F64sGrow {
  sbag_ctx* c;
  sbag_dataset* ds;
  const LabelSet& lab;    // the fit's labels (the dataset's, or a booster's residuals)
  const sbag_tree_params& tp;
  int R;
  int64_t N;
  int Fmax, NB, S;
  const std::vector<int32_t>& h_Fr;
  const std::vector<int32_t>& h_nbins;
  const std::vector<std::vector<double>>& thr;  // [R * Fmax]
  const uint8_t* d_bins;
  int64_t bins_rstride;
  const int16_t* d_pos;
  const int32_t* d_Fr;
  const int32_t* d_nbins;
  const std::vector<int16_t>& h_pos;
  const uint8_t* d_cols;
  int64_t cols_rstride, npad;
  uint64_t* entA;
  uint64_t* entB;
  int64_t cap;
  const std::vector<unsigned long long>& inbag;  // [4R]: entries, Σ count, max count, -
  EventTimer& tm;
  void* hist_root;        // level-0 integer histograms, slot = replica
  int64_t slot_words;     // Fmax * NB * 3
  unsigned int cmax;      // largest draw count of a row
  double inv_scale, eps;  // the labels' fixed-point image: k 2^-s, |y - k 2^-s| <= eps
  // integer (count, Σ c k) histograms of node segments of `ent` into slots of `hist`
  std::function<int(const std::vector<std::pair<int64_t, int64_t>>&, const std::vector<ParentInfo>&,
                    const uint64_t*, void*)> int_hist;
  // SURVEY §8d work bytes of a level's node segments
  std::function<void(const std::vector<std::pair<int64_t, int64_t>>&, const std::vector<int>&)> add_work;
  const std::vector<int64_t>& poff;  // [P + 1] the partitions' row offsets (one: {0, N})
  double* d_y64;                     // the fp64 labels [N + 1]
  double* eyA;                       // the entries' labels carried beside entA (null: gathered by
  double* eyB;                       //   row), written by the ordered compaction
  int64_t fallbacks = 0;
  int levels = 0;
};

// the fp64 labels on the device, once per label set, published only when complete (+ one
// +0.0 at index N: the label of k_f64_hist's padding entries)
static int f64_device_labels(sbag_dataset* ds, const LabelSet& lab, int64_t N, double** out) {
  if (&lab != &ds->lab) {  // a booster's residuals: uploaded by sbag_fit_booster
    if (!lab.d_y64) return fail(SBAG_EDEVICE, "internal: booster labels not on the device");
    *out = lab.d_y64;
    return SBAG_OK;
  }
  std::lock_guard<std::mutex> lk(ds->layout_mu);
  if (!ds->lab.d_y64) {
    double* p = nullptr;
    HIP_TRY(hipMalloc(&p, (size_t)(N + 1) * 8));
    if (hipMemcpy(p, ds->lab.y.data(), (size_t)N * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(p + N, 0, 8) != hipSuccess) {
      (void)hipFree(p);
      return fail(SBAG_EDEVICE, "labels could not be copied to the device");
    }
    ds->lab.d_y64 = p;
  }
  *out = ds->lab.d_y64;
  return SBAG_OK;
}

static int grow_f64s(F64sGrow& G, std::vector<std::vector<BtNode>>& trees) {
  sbag_ctx* c = G.c;
  const int R = G.R, Fmax = G.Fmax, NB = G.NB, D = G.tp.max_depth;
  const int64_t cap = G.cap;
  double* d_y64 = G.d_y64;
  // the partitions (RandomForest.findBestSplits aggregates each one apart, §4.7)
  const int P = (int)G.poff.size() - 1;
  int64_t* d_poff = nullptr;
  if (P > 1) {
    TRY(ws_typed(c, "f64_poff", G.poff.size(), &d_poff));
    TRY(h2d(c, d_poff, G.poff.data(), G.poff.size()));
  }
  const double u = std::ldexp(1.0, -53);
  const double M1 = G.lab.ymax_abs, M2 = G.lab.ymax_sq, Msq = std::max(M2, M1 * M1);
  // gamma_K of a node of n draws (inf when K u >= 1: every screen then flags)
  auto gam = [&](double n) {
    const double k = (n + NB + 2.0) * u;
    return k < 0.5 ? k / (1.0 - k) : INFINITY;
  };
  struct LNode {
    int r, node;
    int64_t a, b;
    double n, e1, e2;  // draws; error bounds of the node's calculator sums (sum, sumSq)
  };
  trees.assign(R, {});
  std::vector<LNode> cur;
  for (int r = 0; r < R; r++) {
    trees[r].push_back(BtNode{});
    const double n = (double)G.inbag[R + r];
    // root: Spark's parent stats l0 + (total - l0) of the first feature with splits
    const double e = (2.0 * gam(n) + 4.0 * u) * 1.01 * n;
    cur.push_back(LNode{r, 0, (int64_t)r * cap, (int64_t)r * cap + (int64_t)G.inbag[r], n, e * M1, e * M2});
  }
  std::vector<int> f0(R, -1);  // first local feature with splits
  for (int r = 0; r < R; r++)
    for (int fl = 0; fl < G.h_Fr[r]; fl++)
      if (G.h_nbins[(size_t)r * Fmax + fl] > 1) {
        f0[r] = fl;
        break;
      }
  // SBAG_F64_SCREEN=0: every node takes the exact path (the unscreened engine, for A/B and
  // the parity tests)
  const bool screen_on = !getenv("SBAG_F64_SCREEN") || atoi(getenv("SBAG_F64_SCREEN")) != 0;
  void* hist_cur = G.hist_root;
  std::string hist_cur_name = "histA", hist_nxt_name = "histB";
  uint64_t* ent_cur = G.entA;
  uint64_t* ent_nxt = G.entB;
  // the entries' labels, carried beside them (the scatter reads them in order and writes
  // the children's; fit_range_impl decides, and the ordered compaction writes the first copy)
  double *ey_cur = G.eyA, *ey_nxt = G.eyB;
  const size_t node_words = (size_t)(Fmax + 1) * NB * 3;
  for (int level = 0; level <= D && !cur.empty(); level++) {
    G.levels++;
    G.tm.level = level;
    const int M = (int)cur.size();
    // ---- 1. screen (level D only happens for maxDepth 0: the root's stats, exactly)
    std::vector<F64ScreenOut> so(M);
    for (auto& o : so) o.flag = 1;
    // per node, the features whose exact sums a flagged node needs (the screen's contenders;
    // every feature when the screen did not run)
    std::vector<uint8_t> cmask((size_t)M * Fmax, 1);
    if (screen_on && level < D) {
      std::vector<int32_t> h_slot_r(M);
      std::vector<double> hdn(M), hdp(M);
      for (int i = 0; i < M; i++) {
        h_slot_r[i] = cur[i].r;
        const double n = cur[i].n, g = gam(n);
        hdn[i] = (7.0 * g + 30.0 * u + 4.0 * (g + u) * (g + u) * n) * Msq * 1.01;
        hdp[i] = (cur[i].e2 / n + cur[i].e1 * (2.0 * n * M1 + cur[i].e1) / (n * n) + 8.0 * u * Msq) * 1.01;
      }
      int32_t* d_slot_r;
      double *d_dn, *d_dp;
      F64ScreenOut* d_so;
      TRY(ws_typed(c, "slot_r", (size_t)M, &d_slot_r));
      TRY(ws_typed(c, "f64_dn", (size_t)M, &d_dn));
      TRY(ws_typed(c, "f64_dp", (size_t)M, &d_dp));
      TRY(ws_typed(c, "f64_so", (size_t)M, &d_so));
      TRY(h2d(c, d_slot_r, h_slot_r.data(), (size_t)M));
      TRY(h2d(c, d_dn, hdn.data(), (size_t)M));
      TRY(h2d(c, d_dp, hdp.data(), (size_t)M));
      F64ScreenArgs sa{};
      sa.hist = (const uint64_t*)hist_cur;
      sa.slot_r = d_slot_r;
      sa.Fr = G.d_Fr;
      sa.nbins = G.d_nbins;
      sa.Fmax = Fmax;
      sa.NB = NB;
      sa.min_inst = G.tp.min_instances_per_node;
      sa.min_gain = G.tp.min_info_gain;
      sa.inv_scale = G.inv_scale;
      sa.eps = G.eps;
      sa.dnode = d_dn;
      sa.dpar = d_dp;
      sa.out = d_so;
      uint8_t* d_cm;
      TRY(ws_typed(c, "f64_cmask", (size_t)M * Fmax, &d_cm));
      sa.cmask = d_cm;
      int h = G.tm.begin(T_SPLIT);
      launch_f64_screen(c->stream, sa, M);
      HIP_TRY(hipGetLastError());
      G.tm.end(h);
      TRY(d2h(c, so.data(), d_so, (size_t)M));
      const bool all_features = getenv("SBAG_F64_FALLBACK_ALL") != nullptr;  // (A/B, tests)
      if (!all_features) TRY(d2h(c, cmask.data(), d_cm, cmask.size()));
    }
    // ... and the first feature with splits of the node's replica (at the root its bins
    // give Spark's parent stats; a node without any valid candidate takes its first split)
    for (int i = 0; i < M; i++)
      if (f0[cur[i].r] >= 0) cmask[(size_t)i * Fmax + f0[cur[i].r]] = 1;
    // Buckets + routing of a task list (launch_fb_route): the chain sums of its first
    // `nchain` tasks land at chist (task-major [NB][3]); nleft (optional) gets the left
    // entries of every routing task.  Bucket space: the chain tasks' entries.
    auto run_tasks = [&](std::vector<F64Task>& tk, int nchain, int64_t nlabels, double* chist,
                         std::vector<int64_t>* nleft_out) -> int {
      if (tk.empty()) return SBAG_OK;
      std::vector<F64TPiece> pcs;
      int64_t ebase = 0;
      for (size_t ti = 0; ti < tk.size(); ti++) {
        tk[ti].ebase = ebase;
        ebase += tk[ti].b - tk[ti].a;
        tk[ti].piece0 = (int64_t)pcs.size();
        for (int64_t x = tk[ti].a; x < tk[ti].b; x += kFbPiece)
          pcs.push_back(F64TPiece{x, std::min(x + kFbPiece, tk[ti].b), (int32_t)ti, 0});
        tk[ti].piece1 = (int64_t)pcs.size();
      }
      const int64_t np = (int64_t)pcs.size();
      const int nt = (int)tk.size();
      F64Task* d_tk;
      F64TPiece* d_pc;
      uint32_t *d_pcnt, *d_plcnt;
      int64_t *d_pbase, *d_plbase, *d_nleft, *d_kboff;
      double* d_bky;
      uint8_t* d_bkc;
      TRY(ws_typed(c, "fb_tasks", (size_t)nt, &d_tk));
      TRY(ws_typed(c, "fb_pieces", (size_t)std::max<int64_t>(np, 1), &d_pc));
      TRY(ws_typed(c, "fb_pcnt", (size_t)std::max<int64_t>(np, 1) * NB, &d_pcnt));
      TRY(ws_typed(c, "fb_plcnt", (size_t)std::max<int64_t>(np, 1), &d_plcnt));
      TRY(ws_typed(c, "fb_pbase", (size_t)std::max<int64_t>(np, 1) * NB, &d_pbase));
      TRY(ws_typed(c, "fb_plbase", (size_t)std::max<int64_t>(np, 1), &d_plbase));
      TRY(ws_typed(c, "fb_nleft", (size_t)nt, &d_nleft));
      TRY(ws_typed(c, "fb_kboff", (size_t)nt * (NB + 1), &d_kboff));
      uint16_t* d_ebin;
      TRY(ws_typed(c, "fb_ebin", (size_t)std::max<int64_t>(1, ebase), &d_ebin));
      // several partitions: Spark's per-partition aggregates merged in partition order
      // (k_fb_psum + k_fb_pmerge, no buckets); one partition: the buckets' row-order chains
      const bool psum = P > 1;
      TRY(ws_typed(c, "fb_bky", (size_t)std::max<int64_t>(1, psum ? 1 : nlabels), &d_bky));
      TRY(ws_typed(c, "fb_bkc", (size_t)std::max<int64_t>(1, psum ? 1 : nlabels), &d_bkc));
      double* d_ppart = nullptr;
      if (psum && nchain > 0)
        TRY(ws_typed(c, "fb_ppart", fb_psum_part_bytes(nchain, P, NB) / sizeof(double), &d_ppart));
      TRY(h2d(c, d_tk, tk.data(), (size_t)nt));
      TRY(h2d(c, d_pc, pcs.data(), pcs.size()));
      F64BucketArgs ba{};
      ba.cols = G.d_cols;
      ba.cols_rstride = G.cols_rstride;
      ba.npad = G.npad;
      ba.tasks = d_tk;
      ba.pieces = d_pc;
      ba.NB = NB;
      ba.ntasks = nt;
      ba.ent_in = ent_cur;
      ba.ent_out = ent_nxt;
      ba.ey_in = ey_cur;
      ba.ey_out = ey_nxt;
      ba.ebin = d_ebin;
      ba.bky = d_bky;
      ba.bkc = d_bkc;
      ba.pcnt = d_pcnt;
      ba.plcnt = d_plcnt;
      ba.pbase = d_pbase;
      ba.plbase = d_plbase;
      ba.nleft = d_nleft;
      ba.kb_off = d_kboff;
      ba.y = d_y64;
      ba.chist = chist;
      ba.cmax = (int32_t)G.cmax;
      ba.psum = psum ? 1 : 0;
      ba.P = P;
      ba.poff = d_poff;
      ba.ppart = d_ppart;
      ba.prun = d_ppart ? (int64_t*)(d_ppart + (size_t)nchain * P * NB * 2) : nullptr;
      ba.hist = (const uint64_t*)hist_cur;
      ba.Fmax = Fmax;
      // (a task's 8-byte arrays or the label column past 2^31 bytes; SBAG_F64_WIDE=1 forces it)
      ba.wide = (G.N >= ((int64_t)1 << 28) || getenv("SBAG_F64_WIDE")) ? 1 : 0;
      // XCD-aware dispatch of k_fb_count (workgroup w runs on XCD w mod 8, each with its own
      // L2): a piece goes to the XCD of its position within its node's entries, a proxy of
      // its rows' slice of [0, N), so each XCD's bin gathers stay in one eighth of a column
      // (SBAG_F64_XCD_ORDER=0: in order)
      ba.porder = nullptr;
      {
        const char* xenv = getenv("SBAG_F64_XCD_ORDER");
        if (!(xenv && atoi(xenv) == 0) && np >= 64) {
          std::vector<std::vector<int32_t>> q(8);
          for (int64_t i = 0; i < np; i++) {
            const F64Task& t = tk[pcs[i].task];
            const int64_t len = std::max<int64_t>(1, t.b - t.a);
            const int64_t mid = (pcs[i].a + pcs[i].b) / 2 - t.a;
            q[(size_t)std::min<int64_t>(7, mid * 8 / len)].push_back((int32_t)i);
          }
          std::vector<int32_t> ord;
          ord.reserve((size_t)np);
          std::vector<size_t> head(8, 0);
          for (int64_t w = 0; w < np; w++) {
            int k = (int)(w & 7);
            if (head[k] >= q[k].size()) {  // that slice is done: the earliest remaining piece
              int best = -1;
              for (int j = 0; j < 8; j++)
                if (head[j] < q[j].size() && (best < 0 || q[j][head[j]] < q[best][head[best]])) best = j;
              k = best;
            }
            ord.push_back(q[k][head[k]++]);
          }
          int32_t* d_ord;
          TRY(ws_typed(c, "fb_porder", (size_t)np, &d_ord));
          TRY(h2d(c, d_ord, ord.data(), ord.size()));
          ba.porder = d_ord;
        }
      }
      ba.route = 0;
      for (const F64Task& t : tk) ba.route |= t.part;
      launch_fb_route(c->stream, ba, np, nchain);
      HIP_TRY(hipGetLastError());
      if (nleft_out) {
        nleft_out->assign(tk.size(), 0);
        TRY(d2h(c, nleft_out->data(), d_nleft, tk.size()));
      }
      return SBAG_OK;
    };
    // ---- exact fallback: flagged nodes, every feature's bins in Spark's row order, then
    // k_f64_split over them.  Nodes up to walk_max entries: k_f64_hist (one wave per (node,
    // feature group) walks the node's entries in order -- latency-bound per node, but the
    // nodes run side by side); bigger ones: one bucketing + chain task per (node, feature)
    // (the node total too when the replica has no feature with splits), throughput-bound,
    // in batches of bounded bucket space.  (C3 shape, 1.1 y + 0.3, serialized: 93 flagged
    // nodes of 8k-800k entries per fit; all walked 120 ms -- ~77 ns per entry of the largest
    // node of a batch -- all chained 53 ms.)
    // (read per level: the tests switch them between fits)
    const bool walk_all = getenv("SBAG_F64_FALLBACK") && !strcmp(getenv("SBAG_F64_FALLBACK"), "hist");
    const bool chain_all = getenv("SBAG_F64_FALLBACK") && !strcmp(getenv("SBAG_F64_FALLBACK"), "chain");
    const int64_t walk_max =
        getenv("SBAG_F64_WALK_MAX") ? atoll(getenv("SBAG_F64_WALK_MAX")) : (int64_t)8192;
    // (several partitions: the walk sums a node in one row order, so every flagged node takes
    // the per-partition tasks)
    auto walked = [&](int i) {
      if (P > 1) return false;
      return walk_all || (!chain_all && cur[i].b - cur[i].a <= walk_max);
    };
    std::vector<int> X, xi(M, -1);
    for (int pass = 0; pass < 2; pass++)  // walked nodes first
      for (int i = 0; i < M; i++)
        if (so[i].flag && walked(i) == (pass == 0)) {
          xi[i] = (int)X.size();
          X.push_back(i);
        }
    size_t nwalk = 0;
    while (nwalk < X.size() && walked(X[nwalk])) nwalk++;
    G.fallbacks += (int64_t)X.size();
    if (getenv("SBAG_LEVEL_TRACE")) {
      int64_t nof = 0, big = 0, ent = 0;
      for (int i : X) {
        nof += so[i].f < 0 ? 1 : 0;
        big = std::max<int64_t>(big, cur[i].b - cur[i].a);
        ent += cur[i].b - cur[i].a;
      }
      fprintf(stderr, "[sbag] f64 level %d nodes %d flagged %zu (no candidate %lld, walked %zu) entries %lld largest %lld\n",
              level, M, X.size(), (long long)nof, nwalk, (long long)ent, (long long)big);
    }
    std::vector<F64SplitOut> xo(X.size());
    for (size_t k0 = 0; k0 < X.size();) {
      // a batch: walked nodes (up to 4096), or chained nodes while their feature tasks'
      // draws fit the budget (one node at least)
      const bool walk_fallback = k0 < nwalk;
      const double budget = (double)((int64_t)1 << 29);  // bucket entries (4 GB)
      size_t k1 = k0;
      double used = 0;
      while (k1 < X.size() && (k1 < nwalk) == walk_fallback) {
        const LNode& q = cur[X[k1]];
        int nf = 1;
        for (int fl = 0; fl < G.h_Fr[q.r]; fl++) nf += cmask[(size_t)X[k1] * Fmax + fl];
        const double need = walk_fallback ? 1.0 : (double)(q.b - q.a) * nf;
        if (k1 > k0 && used + need > (walk_fallback ? 4096.0 : budget)) break;
        used += need;
        k1++;
      }
      const int A = (int)(k1 - k0);
      std::vector<F64Node> hn(A);
      std::vector<F64Chain> chain(A);
      for (int k = 0; k < A; k++) {
        const LNode& q = cur[X[k0 + k]];
        hn[k] = F64Node{q.a, q.b, q.r, 0};
        const BtNode& n = trees[q.r][q.node];
        F64Chain ch{};
        if (level > 0) {
          for (int j = 0; j < 3; j++) ch.calc[j] = n.calc[j];
          ch.impurity = n.impurity;
          ch.set = 1;
        }
        chain[k] = ch;
      }
      F64Node* d_nodes;
      F64Chain* d_chain;
      F64SplitOut* d_out;
      double* d_hist;
      TRY(ws_typed(c, "f64_nodes", (size_t)A, &d_nodes));
      TRY(ws_typed(c, "f64_chain", (size_t)A, &d_chain));
      TRY(ws_typed(c, "f64_sout", (size_t)A, &d_out));
      TRY(ws_typed(c, "f64_hist", (size_t)A * node_words, &d_hist));
      TRY(h2d(c, d_nodes, hn.data(), (size_t)A));
      TRY(h2d(c, d_chain, chain.data(), (size_t)A));
      int h = G.tm.begin(T_FIX);
      if (walk_fallback) {  // the row-order walk of every feature
        const int fpw_env = getenv("SBAG_F64_FPW") ? atoi(getenv("SBAG_F64_FPW")) : 64;
        const int FPW = std::max(1, std::min(f64_hist_width(NB), fpw_env));
        const int ngroups = (Fmax + 1 + FPW - 1) / FPW;
        const int parts = (int64_t)A * ngroups < 1024 ? 2 : 1;
        F64HistArgs ha{};
        ha.ent = ent_cur;
        ha.nodes = d_nodes;
        ha.y = d_y64;
        ha.bins = G.d_bins;
        ha.bins_rstride = G.bins_rstride;
        ha.S = G.S;
        ha.Fmax = Fmax;
        ha.pos = G.d_pos;
        ha.Fr = G.d_Fr;
        ha.NB = NB;
        ha.FPW = FPW;
        ha.parts = parts;
        ha.bins_bytes = (double)G.N * G.S < 4294967295.0 ? (uint32_t)(G.N * G.S) : 0u;
        ha.yzero = (uint32_t)G.N;
        ha.hist = d_hist;
        launch_f64_hist(c->stream, ha, A, ngroups);
        HIP_TRY(hipGetLastError());
      } else {
        // tasks [k][Fmax + 1] (the chain sums land in k_f64_split's [node][Fmax + 1][NB][3]
        // layout), run in chunks of consecutive tasks whose labels fit the budget
        std::vector<F64Task> ft;
        std::vector<int64_t> fdraws;
        ft.reserve((size_t)A * (Fmax + 1));
        for (int k = 0; k < A; k++) {
          const LNode& q = cur[X[k0 + k]];
          for (int fl = 0; fl <= Fmax; fl++) {
            F64Task t{};
            t.r = q.r;
            t.s = -1;
            t.part = 0;
            t.slot = X[k0 + k];
            t.fl = fl < G.h_Fr[q.r] ? fl : -1;
            const bool real = (fl < G.h_Fr[q.r] && cmask[(size_t)X[k0 + k] * Fmax + fl]) ||
                              (fl == G.h_Fr[q.r] && f0[q.r] < 0);
            if (real) {
              t.a = q.a;
              t.b = q.b;
              t.col = fl < G.h_Fr[q.r] ? G.h_pos[(size_t)q.r * Fmax + fl] : -1;
            } else {
              t.a = t.b = q.a;  // empty: zero sums (never read by k_f64_split)
              t.col = -1;
            }
            ft.push_back(t);
            fdraws.push_back(real ? q.b - q.a : 0);
          }
        }
        for (size_t t0 = 0; t0 < ft.size();) {
          size_t t1 = t0;
          int64_t kbc = 0;
          while (t1 < ft.size() && (t1 == t0 || (double)(kbc + fdraws[t1]) <= budget)) {
            ft[t1].kbase = kbc;
            kbc += fdraws[t1];
            t1++;
          }
          std::vector<F64Task> sub(ft.begin() + t0, ft.begin() + t1);
          TRY(run_tasks(sub, (int)sub.size(), kbc, d_hist + t0 * (size_t)NB * 3, nullptr));
          t0 = t1;
        }
      }
      F64SplitArgs sa{};
      sa.hist = d_hist;
      sa.nodes = d_nodes;
      sa.chain = d_chain;
      sa.Fr = G.d_Fr;
      sa.nbins = G.d_nbins;
      sa.Fmax = Fmax;
      sa.NB = NB;
      sa.min_inst = G.tp.min_instances_per_node;
      sa.min_gain = G.tp.min_info_gain;
      sa.out = d_out;
      {
        std::vector<uint8_t> fm((size_t)A * Fmax);
        for (int k = 0; k < A; k++)
          std::copy(cmask.begin() + (size_t)X[k0 + k] * Fmax, cmask.begin() + (size_t)(X[k0 + k] + 1) * Fmax,
                    fm.begin() + (size_t)k * Fmax);
        uint8_t* d_fm;
        TRY(ws_typed(c, "f64_fmask", fm.size(), &d_fm));
        TRY(h2d(c, d_fm, fm.data(), fm.size()));
        sa.fmask = d_fm;
      }
      launch_f64_split(c->stream, sa, A);
      HIP_TRY(hipGetLastError());
      G.tm.end(h);
      TRY(d2h(c, xo.data() + k0, d_out, (size_t)A));
      k0 = k1;
    }
    // ---- 2. bucket + route tasks.  Pass 0: the decided nodes' chosen features (buckets and
    // routing), then the flagged split nodes (routing only); pass 1 (root only): the first
    // feature with splits where it is not the chosen one (buckets only)
    std::vector<F64Task> tasks[2];
    std::vector<F64FinishNode> fin;
    std::vector<int> part_task(M, -1), fin_of(M, -1);
    int64_t kb[2] = {0, 0};
    auto add_task = [&](int pass, int node, int fl, int s, bool part, bool chain) {
      const LNode& q = cur[node];
      F64Task t{};
      t.slot = node;
      t.fl = fl;
      t.a = q.a;
      t.b = q.b;
      t.kbase = chain ? kb[pass] : -1;
      if (chain) kb[pass] += q.b - q.a;  // one bucket entry per in-bag row
      t.r = q.r;
      t.col = G.h_pos[(size_t)q.r * Fmax + fl];
      t.s = s;
      t.part = part ? 1 : 0;
      tasks[pass].push_back(t);
      return (int)tasks[pass].size() - 1;
    };
    // tasks in order of their bin column: k_fb_count's bin gathers (one byte per entry, a
    // line each where a deep node's rows are sparse) then hit the same column from the
    // many replicas' tasks in flight together (SBAG_F64_TASK_ORDER=0: node order)
    std::vector<int> norder(M);
    for (int i = 0; i < M; i++) norder[i] = i;
    {
      const char* oenv = getenv("SBAG_F64_TASK_ORDER");
      if (!(oenv && atoi(oenv) == 0)) {
        auto colkey = [&](int i) -> int64_t {
          return so[i].flag || so[i].f < 0 ? INT64_MAX : (int64_t)G.h_pos[(size_t)cur[i].r * Fmax + so[i].f];
        };
        std::stable_sort(norder.begin(), norder.end(), [&](int x, int y) { return colkey(x) < colkey(y); });
      }
    }
    for (int ii = 0; ii < M; ii++) {
      const int i = norder[ii];
      if (so[i].flag) continue;
      const LNode& q = cur[i];
      const int f = so[i].f, s = so[i].s;
      F64FinishNode fn{};
      // (children at maxDepth are leaves: nothing to route at the last split level)
      fn.t = add_task(0, i, f, s, level + 1 < D, true);
      part_task[i] = fn.t;
      fn.f = f;
      fn.s = s;
      fn.nsp = G.h_nbins[(size_t)q.r * Fmax + f] - 1;
      fn.t0 = -1;
      if (level == 0) {
        fn.ch.set = 0;
        fn.nsp0 = G.h_nbins[(size_t)q.r * Fmax + f0[q.r]] - 1;
        fn.t0 = f0[q.r] == f ? fn.t : -2 - add_task(1, i, f0[q.r], -1, false, true);  // pass 1: fixed below
      } else {
        const BtNode& n = trees[q.r][q.node];
        for (int j = 0; j < 3; j++) fn.ch.calc[j] = n.calc[j];
        fn.ch.impurity = n.impurity;
        fn.ch.set = 1;
      }
      fin_of[i] = (int)fin.size();
      fin.push_back(fn);
    }
    const int nchain0 = (int)tasks[0].size();
    for (int k = 0; k < (int)X.size(); k++) {  // flagged split nodes: routing only
      const int i = X[k];
      const F64SplitOut& o = xo[k];
      if (o.gain <= 0 || level == D || o.f < 0) continue;
      const double li = bt_impurity(o.left), ri = bt_impurity(o.right);
      const bool child_leaf = (level + 1) == D;
      if ((child_leaf || li == 0.0) && (child_leaf || ri == 0.0)) continue;
      part_task[i] = add_task(0, i, o.f, o.s, true, false);
    }
    for (F64FinishNode& fn : fin)
      if (fn.t0 <= -2) fn.t0 = nchain0 + (-2 - fn.t0);  // pass-1 chain sums follow pass 0's
    const int nchain1 = (int)tasks[1].size();
    std::vector<F64SplitOut> fo(fin.size());
    std::vector<int64_t> nleft;
    double* dbg_chist = nullptr;  // (SBAG_F64_DEBUG: the chain histograms, for a violation report)
    if (!tasks[0].empty()) {
      double* d_chist;
      TRY(ws_typed(c, "fb_chist", (size_t)std::max(1, nchain0 + nchain1) * NB * 3, &d_chist));
      dbg_chist = d_chist;
      int h = G.tm.begin(T_CHAIN);
      // one launch sequence for both passes: the root's chains of the chosen features and of
      // the first features run side by side (the root has few, long chains: 2 x 2048 per C3
      // half, each ~200k entries, and a lone chain's adds are latency-bound)
      std::vector<F64Task> all;
      all.reserve(tasks[0].size() + tasks[1].size());
      all.insert(all.end(), tasks[0].begin(), tasks[0].begin() + nchain0);
      for (F64Task t : tasks[1]) {
        t.kbase += kb[0];
        all.push_back(t);
      }
      all.insert(all.end(), tasks[0].begin() + nchain0, tasks[0].end());
      // ... in chunks of consecutive tasks whose bucket entries stay within a budget of 2^32
      // (39 GB of labels and counts; the C4 shard's root holds 2 x 4.0e9: two chunks).  The
      // chain tasks lead the list, so a chunk's chain sums land at its first task's index.
      const int nch = nchain0 + nchain1;
      std::vector<int64_t> nl_all;
      {
        const int64_t kBudget =
            getenv("SBAG_F64_BUCKET_BUDGET") ? atoll(getenv("SBAG_F64_BUCKET_BUDGET")) : ((int64_t)1 << 32);
        size_t t0 = 0;
        while (t0 < all.size()) {
          size_t t1 = t0;
          int64_t ent = 0;
          while (t1 < all.size()) {
            const int64_t e = (int)t1 < nch ? all[t1].b - all[t1].a : 0;
            if (t1 > t0 && ent + e > kBudget) break;
            ent += e;
            t1++;
          }
          std::vector<F64Task> sub(all.begin() + t0, all.begin() + t1);
          int64_t kbc = 0;
          for (size_t t = 0; t < sub.size(); t++)
            if ((int)(t0 + t) < nch) {
              sub[t].kbase = kbc;
              kbc += sub[t].b - sub[t].a;
            }
          const int sub_chains = (int)std::max<int64_t>(0, std::min<int64_t>((int64_t)t1, nch) - (int64_t)t0);
          std::vector<int64_t> nl;
          TRY(run_tasks(sub, sub_chains, kbc, d_chist + t0 * (size_t)NB * 3, &nl));
          nl_all.insert(nl_all.end(), nl.begin(), nl.end());
          t0 = t1;
        }
      }
      nleft.assign(tasks[0].size(), 0);
      for (size_t t = 0; t < tasks[0].size(); t++)
        nleft[t] = nl_all[(int)t < nchain0 ? t : t + nchain1];
      G.tm.end(h);
      if (!fin.empty()) {
        F64FinishNode* d_fn;
        F64SplitOut* d_fo;
        TRY(ws_typed(c, "fb_fin", fin.size(), &d_fn));
        TRY(ws_typed(c, "fb_fout", fin.size(), &d_fo));
        TRY(h2d(c, d_fn, fin.data(), fin.size()));
        F64FinishArgs fa{};
        fa.chist = d_chist;
        fa.nodes = d_fn;
        fa.n = (int)fin.size();
        fa.NB = NB;
        fa.min_inst = G.tp.min_instances_per_node;
        fa.min_gain = G.tp.min_info_gain;
        fa.out = d_fo;
        int hs = G.tm.begin(T_SPLIT);
        launch_fb_finish(c->stream, fa);
        HIP_TRY(hipGetLastError());
        G.tm.end(hs);
        TRY(d2h(c, fo.data(), d_fo, fo.size()));
      }
    }
    // ---- 3. node updates (RandomForest.findBestSplits, host part), next level
    std::vector<LNode> next;
    std::vector<std::pair<int64_t, int64_t>> nseg, hseg;
    std::vector<ParentInfo> hpar;
    std::vector<int32_t> triples;
    for (int i = 0; i < M; i++) {
      const LNode& q = cur[i];
      const bool decided = !so[i].flag;
      const F64SplitOut& o = decided ? fo[fin_of[i]] : xo[xi[i]];
      if (decided && (o.s != so[i].s || !o.valid || !(o.gain > 0.0) || o.gain < G.tp.min_info_gain)) {
        if (getenv("SBAG_F64_DEBUG")) {
          fprintf(stderr,
                  "[sbag] screen violation level %d slot %d r %d entries %lld: screen f %d s %d gain %.17g margin "
                  "%.17g | exact f %d s %d gain %.17g valid %d | min_gain %.17g | node calc %.17g %.17g %.17g\n",
                  level, i, q.r, (long long)(q.b - q.a), so[i].f, so[i].s, so[i].gain, so[i].margin, o.f, o.s,
                  o.gain, o.valid, G.tp.min_info_gain, trees[q.r][q.node].calc[0], trees[q.r][q.node].calc[1],
                  trees[q.r][q.node].calc[2]);
          std::vector<uint64_t> ih((size_t)NB * 3);
          (void)d2h(c, ih.data(), (const uint64_t*)hist_cur + ((size_t)i * Fmax + so[i].f) * NB * 3, ih.size());
          std::vector<double> ch((size_t)NB * 3, 0.0);
          if (dbg_chist) (void)d2h(c, ch.data(), dbg_chist + (size_t)fin[fin_of[i]].t * NB * 3, ch.size());
          const F64FinishNode& fnd = fin[fin_of[i]];
          fprintf(stderr, "[sbag]   finish t %d f %d s %d nsp %d set %d impurity %.17g calc %.17g %.17g %.17g NB %d\n",
                  fnd.t, fnd.f, fnd.s, fnd.nsp, fnd.ch.set, fnd.ch.impurity, fnd.ch.calc[0], fnd.ch.calc[1],
                  fnd.ch.calc[2], NB);
          for (int b = 0; b < NB; b++)
            if (ih[b * 3] || ch[b * 3] != 0.0)
              fprintf(stderr, "[sbag]   bin %d: int count %llu sck %lld | chain %.17g %.17g %.17g\n", b,
                      (unsigned long long)ih[b * 3], (long long)ih[b * 3 + 1], ch[b * 3], ch[b * 3 + 1], ch[b * 3 + 2]);
        }
        return fail(SBAG_EDEVICE, "internal: the fp64 screen's split is not Spark's (bound violated)");
      }
      const int r = q.r;
      {
        BtNode& n = trees[r][q.node];
        for (int j = 0; j < 3; j++) n.calc[j] = o.calc[j];
        n.gain = o.gain;
        n.impurity = o.impurity;
        n.valid = o.f >= 0 && o.valid != 0;
        n.is_leaf = (n.gain <= 0) || (level == D);
        if (n.is_leaf) continue;
        n.has_split = true;
        n.fl = o.f;
        n.s = o.s;
        n.thr = G.thr[(size_t)r * Fmax + o.f][o.s];
      }
      const bool child_leaf = (level + 1) == D;
      BtNode L, Rn;
      for (int j = 0; j < 3; j++) {
        L.calc[j] = o.left[j];
        Rn.calc[j] = o.right[j];
      }
      // LearningNode(child, isLeaf, ImpurityStats.getEmptyImpurityStats(calculator))
      L.impurity = bt_impurity(L.calc);
      Rn.impurity = bt_impurity(Rn.calc);
      L.is_leaf = child_leaf || L.impurity == 0.0;
      Rn.is_leaf = child_leaf || Rn.impurity == 0.0;
      const int li = (int)trees[r].size();
      trees[r][q.node].left = li;
      trees[r][q.node].right = li + 1;
      trees[r].push_back(L);
      trees[r].push_back(Rn);
      if (L.is_leaf && Rn.is_leaf) continue;  // nothing to route
      const int t = part_task[i];
      if (t < 0) return fail(SBAG_EDEVICE, "internal: split node without routing");
      const int64_t m = q.a + nleft[t];
      const double g = gam(q.n);
      const double nl = L.calc[0], nr = Rn.calc[0];
      const double el = g * nl * 1.01, er = 2.0 * (g + u) * (1.0 + g) * q.n * 1.01;
      int sl = -1, sr = -1;
      if (!L.is_leaf) {
        sl = (int)next.size();
        next.push_back(LNode{r, li, q.a, m, nl, el * M1, el * M2});
        nseg.push_back({q.a, m});
      }
      if (!Rn.is_leaf) {
        sr = (int)next.size();
        next.push_back(LNode{r, li + 1, m, q.b, nr, er * M1, er * M2});
        nseg.push_back({m, q.b});
      }
      // the smaller (or only) child is histogrammed, its sibling is parent - small
      int hs = sl >= 0 ? sl : sr;
      if (sl >= 0 && sr >= 0) {
        hs = nl <= nr ? sl : sr;
        triples.push_back(hs == sl ? sr : sl);
        triples.push_back(i);
        triples.push_back(hs);
      }
      hseg.push_back(nseg[hs]);
      hpar.push_back(ParentInfo{r, -1, 0, 0, 0, hs, 0, 0});
    }
    if (next.empty()) break;
    const int Mn = (int)next.size();
    {
      std::vector<int> seg_r(Mn);
      for (int k = 0; k < Mn; k++) seg_r[k] = next[k].r;
      G.add_work(nseg, seg_r);
    }
    void* hist_nxt;
    TRY(ws_get(c, hist_nxt_name, (size_t)Mn * G.slot_words * 8, &hist_nxt));
    {
      std::vector<int32_t> zs;
      for (const ParentInfo& p : hpar) zs.push_back(p.hist_slot);
      const int64_t u32w = G.slot_words * 2;
      if ((u32w & 3) == 0) {
        int32_t* d_zs;
        TRY(ws_typed(c, "zslots", zs.size(), &d_zs));
        TRY(h2d(c, d_zs, zs.data(), zs.size()));
        launch_zero_slots(c->stream, hist_nxt, d_zs, (int)zs.size(), u32w);
        HIP_TRY(hipGetLastError());
      } else {
        HIP_TRY(hipMemsetAsync(hist_nxt, 0, (size_t)Mn * G.slot_words * 8, c->stream));
      }
    }
    TRY(G.int_hist(hseg, hpar, ent_nxt, hist_nxt));
    if (!triples.empty()) {
      int32_t* d_tri;
      TRY(ws_typed(c, "triples", triples.size(), &d_tri));
      TRY(h2d(c, d_tri, triples.data(), triples.size()));
      int h = G.tm.begin(T_SUB);
      launch_subtract(c->stream, hist_nxt, hist_cur, d_tri, (int)triples.size() / 3, G.slot_words, false);
      HIP_TRY(hipGetLastError());
      G.tm.end(h);
    }
    cur.swap(next);
    std::swap(hist_cur_name, hist_nxt_name);
    hist_cur = hist_nxt;
    std::swap(ent_cur, ent_nxt);
    std::swap(ey_cur, ey_nxt);
  }
  return SBAG_OK;
}

static int fit_range_impl(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out,
                          const FitExt* ext, bool int_overflow_f64);

// Dyadic labels go to the exact integer engine unless their sums do not fit its words
// (integer targets of 10^5 at 10^6 rows, e.g. a GBM's first residuals): then the fit is
// redone on the screened fp64 engine, which sums dyadic labels bit-identically to Spark
// (SBAG_F64=1 forces it; tests/test_gpu_gbm.py::test_gbm_large_integer_labels).
static int fit_range(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out,
                     const FitExt* ext) {
  const int st = fit_range_impl(c, ds, fp, out, ext, false);
  if (st != kIntRange) return st;
  return fit_range_impl(c, ds, fp, out, ext, true);
}

static int fit_range_impl(sbag_ctx* c, sbag_dataset* ds, const sbag_fit_params* fp, sbag_forest** out,
                          const FitExt* ext, bool int_overflow_f64) {
  const LabelSet& lab = ext ? *ext->lab : ds->lab;
  const sbag_tree_params& tp = fp->tree;
  TRY(check_sampler(&fp->sampler));
  if (tp.max_depth < 0 || tp.max_depth > 30)
    return fail(SBAG_EINVAL, "maxDepth given invalid value (must be in [0, 30])");
  if (tp.max_bins < 2 || tp.max_bins > 256)
    return fail(SBAG_EINVAL, "maxBins given invalid value (must be in [2, 256])");
  if (tp.min_instances_per_node < 1)
    return fail(SBAG_EINVAL, "minInstancesPerNode given invalid value (must be >= 1)");
  if (!(tp.min_info_gain >= 0.0)) return fail(SBAG_EINVAL, "minInfoGain given invalid value");
  if (!fp->subspace_bug_compat && !(fp->subspace_ratio >= 0 && fp->subspace_ratio <= 1))
    return fail(SBAG_EINVAL, "subspaceRatio given invalid value");
  const bool gini = tp.impurity == SBAG_IMPURITY_GINI;
  if (tp.impurity != SBAG_IMPURITY_GINI && tp.impurity != SBAG_IMPURITY_VARIANCE)
    return fail(SBAG_EINVAL, "unknown impurity");
  // Regression labels that are not dyadic fixed point (|y * 2^s| < 2^23, s <= 40) take the
  // fp64 path (f64 mode, sbag_f64s.hip / sbag_f64.hip): Spark's sums depend on their order
  // there. SBAG_F64=1 forces it on dyadic labels too (both paths then agree bit for bit).
  const bool force_f64 = getenv("SBAG_F64") && atoi(getenv("SBAG_F64")) != 0;
  const bool f64 = !gini && (!lab.label_ok || force_f64 || int_overflow_f64);
  if (f64) {
    if (!lab.finite) return fail(SBAG_EINVAL, "labels must be finite");
    if (!lab.label_ok && !lab.approx_ok) return fail(SBAG_EINVAL, "labels must be finite");
    // the largest row count the fp64 engine is tested at (tests/test_gpu_f64.py,
    // test_fp64_engine_near_the_row_limit: 2^30 - 4096 rows, the 64-bit-addressed scatter);
    // kernels past it (32-bit entry row field up to 2^32) are untested
    if (ds->N > kF64MaxRows)
      return fail(SBAG_EUNSUPPORTED, "real-valued regression labels on more than 2^30 rows (the largest "
                                     "size the fp64 engine is tested at)");
  }
  // the labels' fixed-point image in the entries: exact for dyadic labels, else (f64 path)
  // the screening approximation k = round(y 2^ashift)
  const int lshift = lab.label_ok ? lab.shift : lab.ashift;
  const int64_t lkmin = lab.label_ok ? lab.kmin : lab.akmin;
  const int64_t lkmax = lab.label_ok ? lab.kmax : lab.akmax;
  if (gini && !lab.integral)
    return fail(SBAG_EINVAL, "Classifier was given dataset with invalid label: labels must be "
                             "integers in [0, 2^23)");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t N = ds->N;
  const int F = ds->F;
  // wide datasets (u32 codes): value counts are sparse (code, count) lists built on the
  // host from the subbag's rows or the split-finding sample's rows, bins are per replica
  const bool wide = ds->code_bytes == 4;
  const int lb = fp->sampler.learner_begin;
  const int R = fp->sampler.learner_end - lb;
  const int D = tp.max_depth;
  std::vector<int64_t> poff;
  TRY(check_partitions(fp->num_partitions, fp->partition_offsets, N, poff));

  // ---- subspaces: mkSubspace(getSampleRatio, numFeatures, getSeed + iter) (H1)
  const double sratio = fp->subspace_bug_compat ? fp->sampler.sample_ratio : fp->subspace_ratio;
  std::vector<std::vector<int32_t>> sub(R);
  int Fmax = 0;
  for (int r = 0; r < R; r++) {
    if (ext) {  // the booster's subspace (R = 1)
      sub[r] = ext->sub;
      Fmax = std::max(Fmax, (int)ext->sub.size());
      continue;
    }
    std::vector<int32_t> idx(F);
    int n = 0;
    TRY(sbag_subspace(sratio, F, (int64_t)((uint64_t)fp->sampler.seed + (uint64_t)(int64_t)(lb + r)),
                      idx.data(), &n));
    if (n == 0)
      return fail(SBAG_EINVAL, "requirement failed: VectorSlicer requires that at least one "
                               "feature be selected.");
    idx.resize(n);
    sub[r] = idx;
    Fmax = std::max(Fmax, n);
  }
  auto forest = std::make_unique<sbag_forest>();
  forest->impurity = tp.impurity;
  EventTimer tm{c->stream, {}};
  hipEvent_t ev_start, ev_stop;
  HIP_TRY(hipEventCreate(&ev_start));
  HIP_TRY(hipEventCreate(&ev_stop));
  HIP_TRY(hipEventRecord(ev_start, c->stream));
  // host-side phase timing (SBAG_PROFILE_HOST=1 prints it): where the GPU waits
  const bool hprof = getenv("SBAG_PROFILE_HOST") != nullptr;
  double hp[24] = {0};  // [16..19]: inside histogram launches (grouping, work lists, launch)
  auto hnow = [] {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  double ht = hnow();
  auto hmark = [&](int k) {
    const double t = hnow();
    hp[k] += t - ht;
    ht = t;
  };
  // (the fit's tail after the forest is built: every workspace-local container's destructor)
  struct HostTail {
    bool on;
    double t15;
    ~HostTail() {
      if (on && t15 > 0)
        fprintf(stderr, "host ms: destructors %.2f\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
                        .count() - t15);
    }
  } htail{hprof, 0.0};

  // ---- 1. bag: counts [R][N]
  uint8_t* d_counts;
  TRY(ws_typed(c, "counts", (size_t)R * N, &d_counts));
  {
    int h = tm.begin(T_SAMPLE);
    if (ext)  // the booster's bag column
      TRY(h2d(c, d_counts, ext->counts, (size_t)N));
    else
      TRY(run_sampler(c, &fp->sampler, poff, N, d_counts, false));
    tm.end(h);
  }
  // ---- 2. in-bag entry lists: two ping-pong buffers per replica.  Capacity N, or -- on the
  // fp64 path, and wherever the two lists pass 40 % of the device -- the largest in-bag count
  // (+ 4096 entries of slack for the kernels' clamped read-ahead): a Poisson(1) bag holds 63 %
  // of the rows.  The counts per (replica, 8192-row chunk) come first (k_chunk_inbag, also the
  // ordered compaction's offsets; k_chunk_rows on the integer path), then one copy of them to
  // the host.  The fp64 path also trims lists an earlier integer fit left at capacity N, so
  // that its carried labels fit (§4.7: round 5 took N everywhere, and the C4 shard's
  // real-label fit gathered its labels by row, 2.05 s).  The integer path keeps N below 40 %:
  // the host round trip before the compaction cost the C4 shard step 1062 -> 1088 ms
  // (profiles/r06logs/r06cap3/, SBAG_ENT_TIGHT=0/1)
  unsigned long long* d_inbag;
  TRY(ws_typed(c, "inbag", (size_t)R * 4, &d_inbag));
  unsigned long long* d_wsum = d_inbag + R;
  unsigned int* d_cmax = (unsigned int*)(d_inbag + 2 * R);
  unsigned long long* d_sqsum = d_inbag + 3 * R;
  HIP_TRY(hipMemsetAsync(d_inbag, 0, (size_t)R * 32, c->stream));
  const int64_t nchunk = compact_ordered_chunks(N);
  uint32_t* d_ncnt = nullptr;
  int64_t cap = N;
  size_t dev_free0 = 0, dev_total0 = 0;
  (void)hipMemGetInfo(&dev_free0, &dev_total0);
  static const int cap_env = getenv("SBAG_ENT_TIGHT") ? atoi(getenv("SBAG_ENT_TIGHT")) : -1;  // (A/B)
  const bool tight = cap_env >= 0 ? cap_env != 0 : f64 || (double)R * N * 16.0 > 0.4 * (double)dev_total0;
  if (tight) {
    TRY(ws_typed(c, "inbag_ncnt", (size_t)R * nchunk, &d_ncnt));
    {
      int h = tm.begin(T_COMPACT);
      if (f64)
        launch_chunk_draws(c->stream, d_counts, N, R, d_ncnt, d_wsum, d_cmax);
      else  // (launch_compact computes Σ count and max count itself)
        launch_chunk_rows(c->stream, d_counts, N, R, d_ncnt);
      HIP_TRY(hipGetLastError());
      tm.end(h);
    }
    std::vector<uint32_t> hn((size_t)R * nchunk);
    TRY(d2h(c, hn.data(), d_ncnt, hn.size()));
    int64_t mx = 1;
    for (int r = 0; r < R; r++) {
      int64_t n = 0;
      for (int64_t k = 0; k < nchunk; k++) n += hn[(size_t)r * nchunk + k];
      mx = std::max(mx, n);
    }
    cap = std::min<int64_t>(N, (mx + 4096 + 63) / 64 * 64);
    if (f64) {  // (ws_get's 1/8 slack, and a quarter more before a list is worth trimming)
      const size_t need = (size_t)R * cap * sizeof(uint64_t);
      ws_trim(c, "entA", need + need / 8 + need / 4);
      ws_trim(c, "entB", need + need / 8 + need / 4);
    }
  }
  // fp64 path: the entries' labels carried beside them (k_fb_scatter reads them in entry
  // order and writes the children's; the ordered compaction writes the root copy), when the
  // two copies leave 5 % of the device plus 12 GB free for the level's buffers (C4 shard:
  // ≈10 GB, most of it the (bin, count) words) -- else the scatter and k_fb_psum gather
  // y[row], ~1.4x the carried path's routing + sums on C3 (profiles/r06logs/r06u2/).  Round 5
  // sized the copies as N-entry lists and carried only below 15 % of the device, which left
  // the C4 shard on the gather path (real-label step 2.08 s, profiles/r06logs/r06c4/)
  double *d_y64 = nullptr, *eyA = nullptr, *eyB = nullptr;
  if (f64) {
    TRY(f64_device_labels(ds, lab, N, &d_y64));
    size_t dev_free = 0, dev_total = 0;
    (void)hipMemGetInfo(&dev_free, &dev_total);
    // (the copies' and the level buffers' own memory from an earlier fit counts as free:
    // the margin is for the latter; ws_get adds 1/8 slack)
    const double ey_bytes = (double)R * cap * 16.0 * 1.125;
    double ey_free = (double)dev_free;
    for (const auto& kv : c->ws)
      if (kv.first.rfind("f64_ey", 0) == 0 || kv.first.rfind("fb_", 0) == 0) ey_free += (double)kv.second.cap;
    // (and the entry lists, allocated below, where the workspace does not hold them yet)
    double ent_new = 0.0;
    for (const char* nm : {"entA", "entB"}) {
      auto it = c->ws.find(nm);
      const double need = (double)R * cap * 8.0;
      if (it == c->ws.end() || (double)it->second.cap < need) ent_new += need * 1.125;
    }
    const bool carry = ey_bytes + ent_new + 0.05 * (double)dev_total + 12e9 <= ey_free && !getenv("SBAG_F64_NO_CARRY");
    static const bool ey_trace = getenv("SBAG_LEVEL_TRACE") != nullptr;
    if (ey_trace)
      fprintf(stderr, "f64 labels %s: %d replicas x %lld entries, %.1f GB of copies, %.1f GB free\n",
              carry ? "carried" : "gathered by row", R, (long long)cap, ey_bytes / 1e9, ey_free / 1e9);
    if (carry) {
      TRY(ws_typed(c, "f64_eyA", (size_t)R * cap, &eyA));
      TRY(ws_typed(c, "f64_eyB", (size_t)R * cap, &eyB));
    }
  }
  uint64_t *entA, *entB;
  TRY(ws_typed(c, "entA", (size_t)R * cap, &entA));
  TRY(ws_typed(c, "entB", (size_t)R * cap, &entB));
  {
    int h = tm.begin(T_COMPACT);
    if (f64) {  // row order inside every replica (Spark's fp64 sums follow it)
      unsigned long long* d_cbase;
      TRY(ws_typed(c, "f64_cbase", (size_t)R * nchunk, &d_cbase));
      launch_compact_ordered(c->stream, d_counts, lab.d_labk, N, R, entA, cap, d_ncnt, d_cbase, d_inbag, d_y64, eyA);
    } else {
      launch_compact(c->stream, d_counts, N, R, lab.d_labk, entA, cap, d_inbag, d_wsum, d_cmax,
                     d_sqsum);
    }
    HIP_TRY(hipGetLastError());
    tm.end(h);
  }
  hmark(8);
  std::vector<unsigned long long> inbag(4 * R);
  TRY(d2h(c, inbag.data(), d_inbag, (size_t)4 * R));
  if (!ext && fp->sampler.replacement) TRY(sampler_overflow(c));  // (run_sampler left it to here)
  hmark(9);
  std::vector<int64_t> nw(R);
  unsigned int cmax = 1;
  for (int r = 0; r < R; r++) {
    nw[r] = (int64_t)inbag[R + r];
    cmax = std::max(cmax, ((const unsigned int*)(inbag.data() + 2 * R))[r]);
    if (nw[r] == 0)
      return fail(SBAG_EEMPTY, "DecisionTree requires size of input RDD > 0, but was given by "
                               "empty one (learner " + std::to_string(lb + r) + ")");
    if (gini && (double)nw[r] >= 4294967295.0)
      return fail(SBAG_EUNSUPPORTED, "class counts exceed 32 bits");
  }
  // ---- LDS packing: count field at bit cshift, flush_limit entries between flushes
  const int64_t K0 = -lkmin;
  const double kspan = (double)(lkmax - lkmin + 1);
  const double kabs = (double)std::max(std::llabs(lkmin), std::llabs(lkmax));
  int64_t flush_limit = (int64_t)1 << 22;
  int cshift = 40;
  for (;; flush_limit /= 2) {
    if (flush_limit < 256) {
      if (!gini && !f64) {
        (void)hipEventDestroy(ev_start);
        (void)hipEventDestroy(ev_stop);
        return kIntRange;
      }
      return fail(SBAG_EUNSUPPORTED, "label range too wide for the packed LDS histogram");
    }
    const double wmax = (double)flush_limit * cmax;
    if (gini) {
      if (wmax < 4294967295.0) break;
      continue;
    }
    cshift = (int)std::ceil(std::log2(wmax * kspan + 1.0));
    const int cbits = 64 - cshift;
    // (the sum-of-squares plane of the exact fallback needs wmax k^2 in 64 bits; the fp64
    // path never builds it)
    if (cbits >= 1 && std::ldexp(1.0, cbits) > wmax && (f64 || wmax * kabs * kabs < 1.8e19)) break;
  }
  // the row-lane histogram builds the word as (c << cshift) + c*(k + K0) with a 32-bit
  // low half: raise cshift to 32 when the count field keeps room for flush_limit * cmax
  if (!gini && cshift < 32 && (double)flush_limit * cmax < 4294967296.0) cshift = 32;
  if (!gini && !f64 && (double)N * cmax * kabs * kabs >= std::ldexp(1.0, 53)) {
    (void)hipEventDestroy(ev_start);
    (void)hipEventDestroy(ev_stop);
    return kIntRange;
  }

  // ---- per-replica tables
  std::vector<int32_t> h_sub((size_t)R * Fmax, 0), h_Fr(R);
  for (int r = 0; r < R; r++) {
    h_Fr[r] = (int32_t)sub[r].size();
    for (size_t k = 0; k < sub[r].size(); k++) h_sub[(size_t)r * Fmax + k] = sub[r][k];
  }
  int32_t *d_sub, *d_Fr;
  TRY(ws_typed(c, "sub", h_sub.size(), &d_sub));
  TRY(ws_typed(c, "Fr", (size_t)R, &d_Fr));
  TRY(h2d(c, d_sub, h_sub.data(), h_sub.size()));
  TRY(h2d(c, d_Fr, h_Fr.data(), (size_t)R));
  std::vector<int64_t> vcoff((size_t)R * Fmax + 1, 0);
  {
    int64_t o = 0;
    for (int r = 0; r < R; r++)
      for (int fl = 0; fl < Fmax; fl++) {
        vcoff[(size_t)r * Fmax + fl] = o;
        if (fl < h_Fr[r] && !wide) o += (int64_t)ds->dict[sub[r][fl]].size();
      }
    vcoff[(size_t)R * Fmax] = o;
  }
  const int64_t vc_total = vcoff[(size_t)R * Fmax];
  int ncmax = 0;
  if (!wide)
    for (int f = 0; f < F; f++) ncmax = std::max(ncmax, (int)ds->dict[f].size());
  TRY(check_bins256(tp, N, wide ? INT_MAX : ncmax));

  // root "parents": one per replica, no routing, histogram slot = replica
  std::vector<ParentInfo> h_par(R);
  std::vector<std::pair<int64_t, int64_t>> seg(R);
  for (int r = 0; r < R; r++) {
    h_par[r] = ParentInfo{r, -1, 0, 0, 0, r, 0, 0};
    seg[r] = {(int64_t)r * cap, (int64_t)r * cap + (int64_t)inbag[r]};
  }
  const int NS = gini ? (int)lab.kmax + 1 : 3;
  if (NS > kMaxHostNS) return fail(SBAG_EUNSUPPORTED, "more than 4095 classes");
  const size_t word_bytes = gini ? 4 : 8;
  HistWork work;
  ParentInfo* d_par;
  HistChunk* d_pieces;
  int32_t* d_wg;
  auto upload_work = [&](const std::vector<ParentInfo>& par) -> int {
    for (HistChunk& pc : work.pieces) {
      const ParentInfo& pi = par[pc.parent];
      pc.r = pi.r;
      pc.slot = pi.hist_slot;
      pc.tile = pi.tile;
      pc.fr = h_Fr[pi.r];
    }
    // (the parent list itself stays on the host: the kernels read the pieces' copies)
    TRY(ws_typed(c, "pieces", std::max<size_t>(work.pieces.size(), 1), &d_pieces));
    TRY(h2d(c, d_pieces, work.pieces.data(), work.pieces.size()));
    TRY(ws_typed(c, "wgp", work.wg.size(), &d_wg));
    TRY(h2d(c, d_wg, work.wg.data(), work.wg.size()));
    return SBAG_OK;
  };
  HistArgs ha{};
  ha.Fmax = Fmax;
  ha.Fr = d_Fr;
  ha.K0 = (int32_t)K0;
  ha.cshift = cshift;
  ha.flush_limit = flush_limit;
  double hist_entries = 0, hist_alg_bytes = 0, hist_upper = 0, hist_work = 0, hist_lds = 0;
  const int s_y = gini ? 1 : 4;  // label bytes per row in SURVEY 8d (u8 class / fp32 label)
  // SURVEY §8d work bytes of the histograms of a set of node segments
  auto add_work = [&](const std::vector<std::pair<int64_t, int64_t>>& segs,
                      const std::vector<int>& seg_r) {
    std::vector<char> act(R, 0);
    for (size_t q = 0; q < segs.size(); q++) {
      hist_work += (double)(segs[q].second - segs[q].first) * (h_Fr[seg_r[q]] + s_y);
      act[seg_r[q]] = 1;
    }
    for (int r = 0; r < R; r++) hist_work += act[r] ? 3.0 * N : 0.0;
  };
  int64_t hist_launches = 0;
  double root_mfma_ops = 0;  // int8 MFMA operations of the root histogram (0: k_hist_rl)
  static const bool trace = getenv("SBAG_LEVEL_TRACE") != nullptr;
  int trace_level = -1;
  static const bool group_off = getenv("SBAG_NO_TILE_GROUPING") != nullptr;
  std::vector<std::pair<int64_t, int64_t>> gsegs;
  std::vector<ParentInfo> gpar;
  // the last grouping's per-segment tile bounds [segs][ntc + 1], its class tile and buffer
  // (tile-resident entries start from the root's grouping, see the level loop)
  std::vector<int64_t> gtile_bounds;
  int gtile_ct = 0;
  uint64_t* gtile_ent = nullptr;
  bool hist_pregrouped = false;  // launch(): segments are (node, tile) sub-segments already
  // Gini class tiles: regroup the entries to be histogrammed so that each (segment,
  // class tile) is contiguous (k_tile_count / k_tile_scatter into "entG"), and hand the
  // histogram one sub-segment per (segment, tile) with ParentInfo.tile.
  // the (segment, class tile) entry counts of the next histogram when the host knows them
  // (gini with every draw count 1: the split's class counts), [segs][ntc]; else null
  const std::vector<int64_t>* known_tiles = nullptr;
  auto group_tiles = [&](const HistGeom& g, const std::vector<std::pair<int64_t, int64_t>>& segs,
                         const std::vector<ParentInfo>& par, uint64_t** ent_out) -> int {
    const int CT = g.CT, ntc = (NS + CT - 1) / CT;
    if (known_tiles && known_tiles->size() == segs.size() * (size_t)ntc) {
      // sub-segments from the known sizes; k_tile_scatter_known places the entries with
      // atomic (segment, tile) cursors (no count pass, no round trip)
      const std::vector<int64_t>& kt = *known_tiles;
      std::vector<HistChunk> pcs;
      const int64_t kp = tile_scatter_known_piece();
      std::vector<unsigned long long> cur0(segs.size() * (size_t)ntc);
      gsegs.clear();
      gpar.clear();
      gtile_bounds.assign(segs.size() * (ntc + 1), 0);
      gtile_ct = CT;
      for (size_t q = 0; q < segs.size(); q++) {
        int64_t o = segs[q].first;
        for (int t = 0; t < ntc; t++) {
          gtile_bounds[q * (ntc + 1) + t] = o;
          cur0[q * ntc + t] = (unsigned long long)o;
          const int64_t n = kt[q * ntc + t];
          if (n > 0) {
            gsegs.push_back({o, o + n});
            ParentInfo pi = par[q];
            pi.tile = t;
            gpar.push_back(pi);
          }
          o += n;
        }
        if (o != segs[q].second)
          return fail(SBAG_EDEVICE, "internal: class-tile sizes differ from the segment's entries");
        gtile_bounds[q * (ntc + 1) + ntc] = o;
        for (int64_t a = segs[q].first; a < segs[q].second; a += kp)
          pcs.push_back(HistChunk{(int32_t)q, 0, a, std::min(a + kp, segs[q].second), 0, 0, 0, 0});
      }
      const int np = (int)pcs.size();
      HistChunk* d_pcs;
      unsigned long long* d_cur;
      uint64_t* d_entg;
      TRY(ws_typed(c, "tg_pieces", std::max(np, 1), &d_pcs));
      TRY(ws_typed(c, "tg_cursors", std::max<size_t>(cur0.size(), 1), &d_cur));
      TRY(ws_typed(c, "entG", (size_t)R * cap, &d_entg));
      TRY(h2d(c, d_pcs, pcs.data(), pcs.size()));
      TRY(h2d(c, d_cur, cur0.data(), cur0.size()));
      launch_tile_scatter_known(c->stream, d_pcs, np, ha.ent_in, CT, ntc, d_cur, d_entg);
      HIP_TRY(hipGetLastError());
      if (getenv("SBAG_TILE_CHECK")) {  // (tests: every cursor ends at its tile's end)
        std::vector<unsigned long long> ce(cur0.size());
        TRY(d2h(c, ce.data(), d_cur, ce.size()));
        for (size_t q = 0; q < segs.size(); q++)
          for (int t = 0; t < ntc; t++)
            if ((int64_t)ce[q * ntc + t] != gtile_bounds[q * (ntc + 1) + t + 1])
              return fail(SBAG_EDEVICE, "internal: class-tile cursor does not end at its tile's end");
      }
      *ent_out = d_entg;
      gtile_ent = d_entg;
      return SBAG_OK;
    }
    std::vector<HistChunk> pcs;
    std::vector<int> pseg;
    constexpr int64_t kPiece = 1 << 16;
    for (size_t q = 0; q < segs.size(); q++)
      for (int64_t a = segs[q].first; a < segs[q].second; a += kPiece) {
        pcs.push_back(HistChunk{(int32_t)q, 0, a, std::min(a + kPiece, segs[q].second), 0, 0, 0, 0});
        pseg.push_back((int)q);
      }
    const int np = (int)pcs.size();
    HistChunk* d_pcs;
    uint32_t* d_cnt;
    int64_t* d_base;
    uint64_t* d_entg;
    TRY(ws_typed(c, "tg_pieces", std::max(np, 1), &d_pcs));
    TRY(ws_typed(c, "tg_counts", (size_t)std::max(np, 1) * ntc, &d_cnt));
    TRY(ws_typed(c, "tg_base", (size_t)std::max(np, 1) * ntc, &d_base));
    TRY(ws_typed(c, "entG", (size_t)R * cap, &d_entg));
    TRY(h2d(c, d_pcs, pcs.data(), pcs.size()));
    launch_tile_count(c->stream, d_pcs, np, ha.ent_in, CT, ntc, d_cnt);
    HIP_TRY(hipGetLastError());
    std::vector<uint32_t> cnt((size_t)np * ntc);
    double gt0 = hprof ? hnow() : 0.0;
    TRY(d2h(c, cnt.data(), d_cnt, cnt.size()));
    if (hprof) {
      const double t = hnow();
      hp[18] += t - gt0;  // waiting for the counts (and the queue ahead of them)
      gt0 = t;
    }
    // sub-segment of (q, t) at segs[q].first + sum of the tiles before t; pieces of q
    // fill it in piece order
    std::vector<int64_t> base((size_t)np * ntc);
    gsegs.clear();
    gpar.clear();
    gtile_bounds.assign(segs.size() * (ntc + 1), 0);
    gtile_ct = CT;
    gsegs.reserve((size_t)segs.size() * ntc);
    gpar.reserve((size_t)segs.size() * ntc);
    for (int p0 = 0; p0 < np;) {
      int p1 = p0;
      while (p1 < np && pseg[p1] == pseg[p0]) p1++;
      const int q = pseg[p0];
      int64_t o = segs[q].first;
      for (int t = 0; t < ntc; t++) {
        const int64_t start = o;
        gtile_bounds[(size_t)q * (ntc + 1) + t] = o;
        for (int p = p0; p < p1; p++) {
          base[(size_t)p * ntc + t] = o;
          o += cnt[(size_t)p * ntc + t];
        }
        if (o > start) {
          gsegs.push_back({start, o});
          ParentInfo pi = par[q];
          pi.tile = t;
          gpar.push_back(pi);
        }
      }
      gtile_bounds[(size_t)q * (ntc + 1) + ntc] = o;
      p0 = p1;
    }
    if (hprof) hp[19] += hnow() - gt0;  // host prefix and sub-segment lists
    TRY(h2d(c, d_base, base.data(), base.size()));
    launch_tile_scatter(c->stream, d_pcs, np, ha.ent_in, CT, ntc, d_base, d_entg);
    HIP_TRY(hipGetLastError());
    *ent_out = d_entg;
    gtile_ent = d_entg;
    return SBAG_OK;
  };
  // class tiles of a gini histogram: group the entries by tile (k_hist only)
  auto maybe_grouped = [&](HistGeom& g, int S_, int NB_) -> int {
    if (!gini || g.CT >= NS || g.rl || group_off) return SBAG_OK;
    HistGeom gg;
    if (hist_geometry(S_, Fmax, NB_, NS, true, gg, 0, true) && gg.CT < NS) {
      gg.grouped = true;
      g = gg;
    }
    return SBAG_OK;
  };
  // class tile of the gini histogram layout (gini_cell): the grouped kernels' tile when it
  // divides the classes, so each (node, tile) flush is one contiguous block; else NS
  auto hist_layout_tile = [&](const HistGeom& g) -> int32_t {
    if (!gini || getenv("SBAG_NO_TILE_LAYOUT")) return NS;
    return (g.grouped && g.CT < NS && NS % g.CT == 0) ? g.CT : NS;
  };
  std::function<int()> pre_hist;  // queued by launch() right before the histogram kernel
  // grouped gini launches: per histogram slot, the class tiles whose (node, tile) sub-segment
  // one workgroup flushes with stores (every cell of its features written, zeros included),
  // and whether any of the slot's sub-segments is shared between workgroups (then its flushes
  // add, and the slot must start from zero).  pre_hist then zeros only the shared slots and
  // the tiles no sub-segment covers (C5: most deep-level slots need no zeroing at all)
  bool zplan = false;
  int zplan_ntc = 0;
  std::vector<uint64_t> zplan_cov;  // [slot] bit t: tile t stored by one workgroup
  std::vector<uint8_t> zplan_shared;  // [slot]
  auto launch = [&](const HistGeom& g, int mode, int cat,
                    const std::vector<std::pair<int64_t, int64_t>>& segs_in,
                    const std::vector<ParentInfo>& par_in) -> int {
    const bool grouped = g.grouped && mode == kHistGini && !ha.count_only;
    // 16 waves per CU (two 512-thread workgroups), 32 for grouped class tiles
    static const int wpc_env = getenv("SBAG_HIST_WPC") ? atoi(getenv("SBAG_HIST_WPC")) : 0;
    const int wpc = std::max(1, std::min(wpc_env > 0 ? wpc_env : (grouped ? 4 : 2),
                                         (int)((160 * 1024) / g.lds)));
    const uint64_t* ent_saved = ha.ent_in;
    int ntiles = g.ntiles;
    double lt0 = hprof ? hnow() : 0.0;
    if (grouped && hist_pregrouped) {
      ntiles = g.ntf;  // (node, tile) sub-segments of tile-resident entries: nothing to group
    } else if (grouped) {  // timed apart from the histogram kernel (group_ms)
      const int hg = tm.begin(cat == T_HIST ? T_GROUP : cat);
      uint64_t* d_entg = nullptr;
      TRY(group_tiles(g, segs_in, par_in, &d_entg));
      tm.end(hg);
      ha.ent_in = d_entg;
      ntiles = g.ntf;
    }
    if (hprof) {
      const double t = hnow();
      hp[16] += t - lt0;
      lt0 = t;
    }
    ha.grouped = grouped ? 1 : 0;
    // k_hist gathers aligned 4-byte words (SBAG_HIST_GW=1: single bytes, as before round 2e;
    // 8-byte words were slower on C5, 134 vs 98 ms per fit)
    static const int hist_gw = getenv("SBAG_HIST_GW") ? atoi(getenv("SBAG_HIST_GW")) : 4;
    ha.dw = hist_gw == 1 ? 1 : 4;
    // k_hist_rl row prefetch distance in passes of 4 entries (C3, ms per fit: 2 -> hist 92.1,
    // 3 -> 90.2 and step 134, 4 -> hist 89.7 and step 130, 5 -> flat); only 4 is built
    ha.rlpd = 4;
    const bool regrouped = grouped && !hist_pregrouped;
    const std::vector<std::pair<int64_t, int64_t>>& segs = regrouped ? gsegs : segs_in;
    const std::vector<ParentInfo>& par = regrouped ? gpar : par_in;
    build_work(segs, flush_limit, 256 * wpc * (grouped ? 2 : 1), g.T, work);
    TRY(upload_work(par));
    static const bool zplan_off = getenv("SBAG_ZERO_ALL") && atoi(getenv("SBAG_ZERO_ALL")) != 0;  // (A/B)
    zplan = regrouped && mode == kHistGini && !zplan_off && ha.hct == g.CT && g.CT < NS && NS % g.CT == 0 &&
            NS / g.CT <= 64;
    static const bool ztrace = getenv("SBAG_LEVEL_TRACE") != nullptr;
    if (ztrace)
      fprintf(stderr, "[sbag] zero plan %d (CT %d, layout tile %d, pieces %zu)\n", zplan ? 1 : 0, g.CT, ha.hct,
              work.pieces.size());
    if (zplan) {
      zplan_ntc = NS / g.CT;
      int smax = 0;
      for (const HistChunk& pc : work.pieces) smax = std::max(smax, pc.slot + 1);
      zplan_cov.assign((size_t)smax, 0ull);
      zplan_shared.assign((size_t)smax, 0);
      for (const HistChunk& pc : work.pieces) {
        if (pc.slot < 0) continue;
        if (pc.excl)
          zplan_cov[pc.slot] |= 1ull << pc.tile;
        else
          zplan_shared[pc.slot] = 1;
      }
    }
    if (hprof) {
      const double t = hnow();
      hp[17] += t - lt0;
      lt0 = t;
    }
    ha.chunks = d_pieces;
    ha.wg_piece = d_wg;
    ha.parents = nullptr;
    // short (node, class tile) sub-segments (deep gini levels): the 256-thread k_hist with
    // 32-entry gather groups; SBAG_HIST_SMALL = mean entries per sub-segment below which it
    // is used (0: never)
    static const double small_seg =
        getenv("SBAG_HIST_SMALL") ? atof(getenv("SBAG_HIST_SMALL")) : 4096.0;
    ha.small = (grouped && !segs.empty() && work.entries < small_seg * (double)segs.size()) ? 1 : 0;
    ha.ablate = 0;
    ha.FT = g.FT;
    ha.FPH = g.FPH;
    ha.CT = g.CT;
    ha.ntf = g.ntf;
    ha.rl = g.rl;
    if (pre_hist) TRY(pre_hist());
    int h = tm.begin(cat);
    launch_hist(c->stream, ha, work.nwg, ntiles, mode, g.lds);
    HIP_TRY(hipGetLastError());
    tm.end(h);
    if (trace) {
      // SBAG_LEVEL_TRACE: one line per histogram launch (synchronizes; diagnostics only)
      float ms = 0;
      (void)hipEventSynchronize(tm.ev[h].second.second);
      (void)hipEventElapsedTime(&ms, tm.ev[h].second.first, tm.ev[h].second.second);
      int64_t ne = 0;
      for (auto& sg : segs) ne += sg.second - sg.first;
      fprintf(stderr, "[sbag] level %d cat %d mode %d grouped %d segs %zu entries %lld pieces %zu nwg %d ms %.3f\n",
              trace_level, cat, mode, grouped ? 1 : 0, segs.size(), (long long)ne, work.pieces.size(),
              work.nwg, ms);
    }
    if (trace && getenv("SBAG_HIST_ABLATE")) {
      // diagnostics: relaunch the same histogram with phases skipped (flushes always
      // skipped, so the real result stays intact) and time each relaunch
      for (int m : {1, 1 | 2, 1 | 4, 1 | 8, 1 | 2 | 4 | 8}) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        ha.ablate = m;
        (void)hipEventRecord(e0, c->stream);
        launch_hist(c->stream, ha, work.nwg, ntiles, mode, g.lds);
        (void)hipEventRecord(e1, c->stream);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        fprintf(stderr, "[sbag] ablate level %d mode %d ms %.3f\n", trace_level, m, ms);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
      }
      ha.ablate = 0;
    }
    ha.ent_in = ent_saved;
    ha.grouped = 0;
    if (cat == T_HIST) {
      hist_launches++;
      // LDS atomic wave-instructions per entry: per feature tile, k_hist one per 64-lane
      // group, k_hist_rl K/4 (16 lanes of K features per entry, 4 entries per instruction)
      const double per_entry =
          g.ntf * (g.rl ? (double)((g.FT + hist_rl_lanes() - 1) / hist_rl_lanes()) * hist_rl_lanes() / 64.0
                        : (double)((g.FT + 63) / 64));
      for (size_t q = 0; q < segs.size(); q++) {
        const double ne = (double)(segs[q].second - segs[q].first);
        hist_entries += ne;
        hist_lds += ne * per_entry;
        hist_alg_bytes += ne * (h_Fr[par[q].r] + s_y);
      }
    }
    return SBAG_OK;
  };

  // the column-major copy of the codes [F][npad] (the bins when they are the codes), once
  // per dataset (part of ingest: kept with it)
  auto ensure_cols = [&]() -> int {
    std::lock_guard<std::mutex> lk(ds->layout_mu);
    if (!ds->d_cols) {
      const int64_t np = (N + 63) / 64 * 64;
      HIP_TRY(hipMalloc(&ds->d_cols, (size_t)ds->F * np));
      launch_transpose(c->stream, (const uint8_t*)ds->d_codes, N, ds->S, ds->F, ds->d_cols, np, 1, 0, 0);
      HIP_TRY(hipGetLastError());
      ds->cols_ncol = ds->F;
      // other contexts (the learner-part twins) read it without this stream's order
      HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return SBAG_OK;
  };
  // ---- 3. value counts -> thresholds.  Optimistic path: when every feature has
  // at most maxBins distinct values, histogram the root over the value codes
  // directly; its count stats ARE the value counts, and if every replica's
  // thresholds turn out to be all midpoints (code == bin) that root histogram is
  // already the level-0 histogram.
  void* hist_cur;
  TRY(ws_get(c, "histA", (size_t)R * Fmax * std::max(ncmax, tp.max_bins) * NS * word_bytes, &hist_cur));
  std::vector<int16_t> h_pos_codes((size_t)R * Fmax, 0);
  for (int r = 0; r < R; r++)
    for (int fl = 0; fl < h_Fr[r]; fl++) h_pos_codes[(size_t)r * Fmax + fl] = (int16_t)sub[r][fl];
  int16_t* d_pos;
  TRY(ws_typed(c, "pos", h_pos_codes.size(), &d_pos));
  TRY(h2d(c, d_pos, h_pos_codes.data(), h_pos_codes.size()));
  std::vector<uint32_t> vc;  // the subbag's value counts (filled below when a replica uses them)
  const bool optimistic = ds->code_bytes == 1 && ncmax <= tp.max_bins;
  // row-lane histogram: identity byte layout, packed variance words with cshift >= 32
  // (SBAG_HIST_RL: 0 = never, 1 = always 64-bit row addresses; tests pin both paths)
  const int rl_env = getenv("SBAG_HIST_RL") ? atoi(getenv("SBAG_HIST_RL")) : -1;
  auto rl_mode_for = [&](const std::vector<int16_t>& pos, int32_t S_) {
    if (rl_env == 0 || !(gini || cshift >= 32)) return 0;
    for (int r = 0; r < R; r++)
      for (int fl = 0; fl < h_Fr[r]; fl++)
        if (pos[(size_t)r * Fmax + fl] != fl) return 0;
    return (rl_env != 1 && N < (1 << 24) && (double)N * S_ + S_ < 4294967296.0) ? 2 : 1;
  };
  bool root_done = false;
  HistGeom g0{};
  if (optimistic) {
    vc.assign((size_t)std::max<int64_t>(vc_total, 1), 0);
    if (!hist_geometry(ds->S, Fmax, ncmax, NS, gini, g0, rl_mode_for(h_pos_codes, ds->S)))
      return fail(SBAG_EUNSUPPORTED, "histogram of one feature does not fit in LDS");
    TRY(maybe_grouped(g0, ds->S, ncmax));
    ha.hct = hist_layout_tile(g0);
    HIP_TRY(hipMemsetAsync(hist_cur, 0, (size_t)R * Fmax * ncmax * NS * word_bytes, c->stream));
    ha.bins = (const uint8_t*)ds->d_codes;
    ha.bins_rstride = 0;
    ha.S = ds->S;
    ha.pos = d_pos;
    ha.ent_in = entA;
    ha.hist = hist_cur;
    ha.NB = ncmax;
    ha.NS = NS;
    ha.count_only = 0;
    // Variance with every replica on every feature of <= 32 codes, counts <= 127: the root
    // histogram as an int8 MFMA contraction (sbag_mfma.hip; SBAG_ROOT_MFMA=0: k_hist_rl)
    const int mfma_env = getenv("SBAG_ROOT_MFMA") ? atoi(getenv("SBAG_ROOT_MFMA")) : -1;
    // (its cost goes with ceil(R / 32) tiles, the atomics' with R: below 16 replicas -- a
    // booster's single tree -- the atomics are cheaper; SBAG_ROOT_MFMA=1 forces it)
    bool mfma_root = !gini && mfma_env != 0 && (R >= 16 || mfma_env == 1) && ncmax <= 32 &&
                     N % 16 == 0 && cmax <= 127 && Fmax == F && !getenv("SBAG_NO_LAYOUT_CACHE");
    for (int r = 0; r < R && mfma_root; r++) {
      if (h_Fr[r] != F) mfma_root = false;
      for (int fl = 0; fl < h_Fr[r] && mfma_root; fl++)
        if (h_pos_codes[(size_t)r * Fmax + fl] != fl) mfma_root = false;
    }
    // digit planes of the label image: 7-bit digits of k + K0 >= 0, or -- when fewer -- the
    // balanced base-256 digits (int8, [-128, 127]) of k - its range's midpoint (round 6: a
    // non-dyadic label's 23-bit image takes 3 planes instead of 4; |count x digit| <=
    // 127 x 128 keeps a 65536-row int32 sum exact).  The root needs no squares plane
    // (words [.][2]): the screen decides from (count, Σck), and the exact path's Σck² comes
    // from k_compact / k_partition reductions and kHistSq launches
    int nd1 = 1;
    while (nd1 < 10 && ((uint64_t)(lkmax - lkmin) >> (7 * nd1)) != 0) nd1++;
    const int64_t kmid = lkmin + (lkmax - lkmin) / 2;
    int nds = 1;  // balanced base-256 digits of k - kmid: n of them cover [-128 m, 127 m], m = (256^n - 1) / 255
    for (; nds < 8; nds++) {
      const int64_t m = (((int64_t)1 << (8 * nds)) - 1) / 255;
      if (lkmin - kmid >= -128 * m && lkmax - kmid <= 127 * m) break;
    }
    const int dig_env = getenv("SBAG_MFMA_DIGITS") ? atoi(getenv("SBAG_MFMA_DIGITS")) : 0;  // 7 / 8: force (tests)
    const bool signed_digits = dig_env == 8 || (dig_env != 7 && nds < nd1);
    if (signed_digits) nd1 = nds;
    const int64_t dK0 = signed_digits ? -kmid : K0;  // the digits are of k + dK0
    const int nd2 = 0;
    if (nd1 + nd2 > 6) mfma_root = false;
    if (mfma_root) {
      TRY(ensure_cols());
      uint8_t* d_dig;
      TRY(ws_typed(c, "mfma_digits", (size_t)(nd1 + nd2) * N, &d_dig));
      int h = tm.begin(T_ROOT);
      launch_label_digits(c->stream, lab.d_labk, N, (int32_t)dK0, nd1, nd2, d_dig, signed_digits);
      MfmaHistArgs ma{};
      ma.counts = d_counts;
      ma.cols = ds->d_cols;
      ma.digits = d_dig;
      ma.N = N;
      ma.npad = (N + 63) / 64 * 64;
      ma.R = R;
      ma.F = F;
      ma.Fmax = Fmax;
      ma.NB = ncmax;
      ma.ND1 = nd1;
      ma.ND = nd1 + nd2;
      ma.K0 = (int32_t)dK0;
      ma.dbits = signed_digits ? 8 : 7;
      ma.hist = (unsigned long long*)hist_cur;
      if (!launch_hist_mfma(c->stream, ma)) return fail(SBAG_EDEVICE, "internal: MFMA root histogram geometry");
      HIP_TRY(hipGetLastError());
      tm.end(h);
      root_mfma_ops += 2.0 * 32.0 * 32.0 * 32.0 * (double)((N + 31) / 32) * F *
                       (double)(((R + 31) / 32)) * (1 + nd1 + nd2);
    } else {
      TRY(launch(g0, gini ? kHistGini : kHistVar, T_HIST, seg, h_par));
    }
    // its counts are the value counts of replicas thresholded on their whole subbag (numExamples
    // <= required); replicas thresholded on their split-finding sample (3b: every C3 / C5
    // replica) need none, and the copy would wait for the root histogram
    bool any_whole = false;
    for (int r = 0; r < R; r++) {
      const int64_t mpb = std::min<int64_t>(tp.max_bins, nw[r]);
      any_whole = any_whole || std::max<int64_t>(mpb * mpb, 10000) >= nw[r];
    }
    const int64_t words = any_whole ? (int64_t)R * Fmax * ncmax * NS : 0;
    std::vector<uint8_t> tmp((size_t)words * word_bytes);
    if (any_whole) TRY(d2h(c, tmp.data(), (const uint8_t*)hist_cur, tmp.size()));
    for (int r = 0; r < R && any_whole; r++)
      for (int fl = 0; fl < h_Fr[r]; fl++) {
        const size_t nc = ds->dict[sub[r][fl]].size();
        for (size_t k = 0; k < nc; k++) {
          const int64_t wi = (((int64_t)r * Fmax + fl) * ncmax + (int64_t)k) * NS;
          uint64_t cnt = 0;
          if (gini) {
            const uint32_t* hs = (const uint32_t*)tmp.data() + (int64_t)r * Fmax * ncmax * NS;
            for (int q = 0; q < NS; q++) cnt += hs[gini_cell(fl, (int)k, q, ncmax, Fmax, ha.hct)];
          } else {
            cnt = ((const uint64_t*)tmp.data())[wi];
          }
          vc[vcoff[(size_t)r * Fmax + fl] + k] = (uint32_t)cnt;
        }
      }
  } else if (!wide && [&] {
               // the subbag's value counts serve only replicas whose thresholds come from the
               // whole subbag (numExamples <= required); the others are thresholded on their
               // split-finding sample (3b) -- a C3-sized continuous fit skips 8.1e10 atomics
               for (int r = 0; r < R; r++)
                 if (std::max<int64_t>(std::min<int64_t>(tp.max_bins, nw[r]) * std::min<int64_t>(tp.max_bins, nw[r]),
                                       10000) >= nw[r])
                   return true;
               return false;
             }()) {
    vc.assign((size_t)std::max<int64_t>(vc_total, 1), 0);
    int h = tm.begin(T_VC);
    HistGeom g;
    if (ds->code_bytes == 1 && hist_geometry(ds->S, Fmax, ncmax, 1, true, g)) {
      const int64_t slot_words = (int64_t)Fmax * ncmax;
      uint32_t* d_vch;
      TRY(ws_typed(c, "vch", (size_t)R * slot_words, &d_vch));
      HIP_TRY(hipMemsetAsync(d_vch, 0, (size_t)R * slot_words * 4, c->stream));
      HistArgs save = ha;
      ha.bins = (const uint8_t*)ds->d_codes;
      ha.bins_rstride = 0;
      ha.S = ds->S;
      ha.pos = d_pos;
      ha.ent_in = entA;
      ha.hist = d_vch;
      ha.NB = ncmax;
      ha.NS = 1;
      ha.hct = 1;
      ha.count_only = 1;
      TRY(launch(g, kHistGini, T_VC, seg, h_par));
      ha = save;
      std::vector<uint32_t> tmp((size_t)R * slot_words);
      TRY(d2h(c, tmp.data(), d_vch, tmp.size()));
      for (int r = 0; r < R; r++)
        for (int fl = 0; fl < h_Fr[r]; fl++) {
          const size_t nc = ds->dict[sub[r][fl]].size();
          std::copy(tmp.begin() + ((size_t)r * Fmax + fl) * ncmax,
                    tmp.begin() + ((size_t)r * Fmax + fl) * ncmax + nc,
                    vc.begin() + vcoff[(size_t)r * Fmax + fl]);
        }
    } else {
      uint32_t* d_vc;
      int64_t* d_vcoff;
      TRY(ws_typed(c, "vc", (size_t)std::max<int64_t>(vc_total, 1), &d_vc));
      TRY(ws_typed(c, "vcoff", vcoff.size(), &d_vcoff));
      TRY(h2d(c, d_vcoff, vcoff.data(), vcoff.size()));
      HIP_TRY(hipMemsetAsync(d_vc, 0, (size_t)std::max<int64_t>(vc_total, 1) * 4, c->stream));
      launch_vc_global(c->stream, ds->d_codes, ds->code_bytes, ds->S, entA, cap, d_inbag, d_sub,
                       d_Fr, Fmax, R, d_vcoff, d_vc);
      HIP_TRY(hipGetLastError());
      TRY(d2h(c, vc.data(), d_vc, (size_t)vc_total));
    }
    tm.end(h);
  }

  hmark(10);
  // ---- 3b. RandomForest.findSplits' split-finding sample: a subbag of more than
  // required = max(min(maxBins, n)^2, 10^4) rows is thresholded on
  // RDD.sample(false, required / n, new XORShiftRandom(seed).nextInt()) (k_split_sample);
  // findSplitsForContinuousFeature then sees numSamples = (fraction * n).toInt
  std::vector<double> sfrac(R, 1.0);
  std::vector<uint32_t> vcs;
  // the sampled replicas' thresholds and cuts from k_find_splits (dev_tc per (replica, feature));
  // SBAG_SPLITS_HOST=1: the host walk over the value counts copied back (A/B)
  bool dev_splits = false;
  const int dev_tc = std::min(520, tp.max_bins + 64);
  std::vector<int32_t> dev_nt;
  std::vector<double> dev_thr;
  std::vector<uint32_t> dev_cut;
  // wide datasets: per replica the (row, weight) items split finding counts
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> items(wide ? R : 0);
  {
    std::vector<int32_t> reps;
    std::vector<double> fl2;
    for (int r = 0; r < R; r++) {
      const int64_t mpb = std::min<int64_t>(tp.max_bins, nw[r]);
      const int64_t required = std::max<int64_t>(mpb * mpb, 10000);
      if (required < nw[r]) {
        sfrac[r] = (double)required / (double)nw[r];
        reps.push_back(r);
        fl2.push_back(sfrac[r]);
        fl2.push_back(std::log1p(-sfrac[r]));
      }
    }
    if (!reps.empty()) {
      const int P = (int)poff.size() - 1;
      // PartitionwiseSampledRDD: java.util.Random(sampleSeed).nextLong() per partition
      uint64_t js = ((uint64_t)(int64_t)HostXS(tp.seed).next(32) ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1);
      auto jnext = [&]() {
        js = (js * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        return (int64_t)(int32_t)(uint32_t)(js >> 16);
      };
      std::vector<uint64_t> pst(P);
      for (int q = 0; q < P; q++) {
        const int64_t hi = jnext(), lo = jnext();
        pst[q] = h_hash_seed((int64_t)((uint64_t)hi << 32) + lo);
      }
      int32_t* d_reps;
      double* d_frac;
      uint64_t* d_pst;
      int64_t *d_spoff, *d_svcoff;
      uint32_t* d_vcs;
      TRY(ws_typed(c, "ss_reps", reps.size(), &d_reps));
      TRY(ws_typed(c, "ss_frac", fl2.size(), &d_frac));
      TRY(ws_typed(c, "ss_pst", pst.size(), &d_pst));
      TRY(ws_typed(c, "ss_poff", poff.size(), &d_spoff));
      TRY(ws_typed(c, "ss_vcoff", vcoff.size(), &d_svcoff));
      TRY(ws_typed(c, "ss_vc", (size_t)std::max<int64_t>(vc_total, 1), &d_vcs));
      TRY(h2d(c, d_reps, reps.data(), reps.size()));
      TRY(h2d(c, d_frac, fl2.data(), fl2.size()));
      TRY(h2d(c, d_pst, pst.data(), pst.size()));
      TRY(h2d(c, d_spoff, poff.data(), poff.size()));
      TRY(h2d(c, d_svcoff, vcoff.data(), vcoff.size()));
      HIP_TRY(hipMemsetAsync(d_vcs, 0, (size_t)std::max<int64_t>(vc_total, 1) * 4, c->stream));
      int h = tm.begin(T_VC);
      // a replica's value counts accumulate in LDS when they fit in 64 KB
      int64_t maxw = 0, maxreq = 0;
      for (int r : reps) {
        maxw = std::max(maxw, vcoff[(size_t)r * Fmax + h_Fr[r]] - vcoff[(size_t)r * Fmax]);
        const int64_t mpb = std::min<int64_t>(tp.max_bins, nw[r]);
        maxreq = std::max(maxreq, std::max<int64_t>(mpb * mpb, 10000));
      }
      const int lds_words = maxw <= 16384 ? (int)maxw : 0;
      // sampled rows per replica: Binomial(n, required / n), capacity 8 sigma above
      const int64_t cap = maxreq + 8 * (int64_t)std::ceil(std::sqrt((double)maxreq)) + 1024;
      uint32_t *d_srows, *d_snr;
      TRY(ws_typed(c, "ss_rows", (size_t)reps.size() * cap, &d_srows));
      TRY(ws_typed(c, "ss_nrows", reps.size(), &d_snr));
      HIP_TRY(hipMemsetAsync(d_snr, 0, reps.size() * 4, c->stream));
      uint16_t* d_gsums;
      TRY(ws_typed(c, "ss_gsums", (size_t)split_sample_groups((int64_t)R * N), &d_gsums));
      bool gap_all = true;  // every sampled replica's fraction <= 0.4: GapSampling
      for (size_t k = 0; k < reps.size(); k++) gap_all = gap_all && fl2[2 * k] <= 0.4;
      launch_split_sample(c->stream, d_counts, N, R, d_spoff, P, d_reps, (int)reps.size(), d_pst,
                          d_frac, d_gsums, d_srows, cap, d_snr, gap_all);
      HIP_TRY(hipGetLastError());
      if (!wide)
        launch_split_sample_vc(c->stream, d_srows, cap, d_snr, d_reps, (int)reps.size(), ds->d_codes,
                               ds->code_bytes, ds->S, d_sub, d_Fr, Fmax, d_svcoff, d_vcs, lds_words);
      HIP_TRY(hipGetLastError());
      tm.end(h);
      const bool splits_host = getenv("SBAG_SPLITS_HOST") && atoi(getenv("SBAG_SPLITS_HOST")) != 0;
      if (!wide && !splits_host && !getenv("SBAG_DEBUG_SAMPLE") && ds->d_dict) {
        std::vector<int64_t> knw(reps.size()), kns(reps.size());
        for (size_t k = 0; k < reps.size(); k++) {
          const int r = reps[k];
          knw[k] = nw[r];
          kns[k] = (int64_t)(int32_t)(sfrac[r] * (double)nw[r]);  // (fraction * numExamples).toInt
        }
        int32_t *d_zc, *d_nt;
        int64_t *d_knw, *d_kns;
        double* d_thr;
        uint32_t* d_fcut;
        TRY(ws_typed(c, "fs_zero", (size_t)F, &d_zc));
        TRY(ws_typed(c, "fs_nw", knw.size(), &d_knw));
        TRY(ws_typed(c, "fs_ns", kns.size(), &d_kns));
        TRY(ws_typed(c, "fs_nt", (size_t)R * Fmax, &d_nt));
        TRY(ws_typed(c, "fs_thr", (size_t)R * Fmax * dev_tc, &d_thr));
        TRY(ws_typed(c, "fs_cut", (size_t)R * Fmax * dev_tc, &d_fcut));
        TRY(h2d(c, d_zc, ds->zero_code.data(), (size_t)F));
        TRY(h2d(c, d_knw, knw.data(), knw.size()));
        TRY(h2d(c, d_kns, kns.data(), kns.size()));
        HIP_TRY(hipMemsetAsync(d_nt, 0, (size_t)R * Fmax * 4, c->stream));
        SplitFindArgs fa{};
        fa.cnt = d_vcs;
        fa.vcoff = d_svcoff;
        fa.dict = ds->d_dict;
        fa.dict_off = ds->d_dict_off;
        fa.zero_code = d_zc;
        fa.sub = d_sub;
        fa.Fr = d_Fr;
        fa.reps = d_reps;
        fa.nw = d_knw;
        fa.nsamp = d_kns;
        fa.Fmax = Fmax;
        fa.max_bins = tp.max_bins;
        fa.tc = dev_tc;
        fa.nrep = (int)reps.size();
        fa.nt = d_nt;
        fa.thr = d_thr;
        fa.cut = d_fcut;
        launch_find_splits(c->stream, fa);
        HIP_TRY(hipGetLastError());
        dev_nt.resize((size_t)R * Fmax);
        TRY(d2h(c, dev_nt.data(), d_nt, dev_nt.size()));
        dev_splits = true;
        for (int32_t v : dev_nt)
          if (v > dev_tc) dev_splits = false;  // (more thresholds than the table holds: host walk)
        if (dev_splits) {
          dev_thr.resize((size_t)R * Fmax * dev_tc);
          dev_cut.resize((size_t)R * Fmax * dev_tc);
          TRY(d2h(c, dev_thr.data(), d_thr, dev_thr.size()));
          TRY(d2h(c, dev_cut.data(), d_fcut, dev_cut.size()));
        }
      }
      std::vector<uint32_t> snr(reps.size());
      TRY(d2h(c, snr.data(), d_snr, snr.size()));
      for (uint32_t k : snr)
        if ((int64_t)k > cap)
          return fail(SBAG_EDEVICE, "split-finding sample exceeds its capacity");
      if (wide) {
        std::vector<uint32_t> rows((size_t)reps.size() * cap);
        TRY(d2h(c, rows.data(), d_srows, rows.size()));
        for (size_t ri = 0; ri < reps.size(); ri++) {
          auto& it = items[reps[ri]];
          it.clear();
          for (uint32_t k = 0; k < snr[ri]; k++) it.emplace_back(rows[ri * cap + k], 1u);
        }
      }
      if (!dev_splits) {
        vcs.assign((size_t)std::max<int64_t>(vc_total, 1), 0);
        TRY(d2h(c, vcs.data(), d_vcs, vcs.size()));
      }
      if (getenv("SBAG_DEBUG_SAMPLE")) {
        for (int r : reps) {
          int64_t tot = 0;
          for (int64_t k = vcoff[(size_t)r * Fmax]; k < vcoff[(size_t)r * Fmax + 1]; k++) tot += vcs[k];
          fprintf(stderr, "split sample r=%d n=%lld frac=%.17g sampled=%lld seed=%lld pst0=%llx\n", r,
                  (long long)nw[r], sfrac[r], (long long)tot, (long long)tp.seed,
                  (unsigned long long)pst[0]);
        }
      }
    }
  }

  // ---- 4. thresholds, code cuts (bin(code) = #{j : cut_j <= code}), numSplits per (replica,
  // feature)
  std::vector<std::vector<double>> thr((size_t)R * Fmax);
  std::vector<std::vector<uint32_t>> cuts((size_t)R * Fmax);
  std::vector<int32_t> h_nbins((size_t)R * Fmax, 1);
  std::vector<int32_t> exact(R, 1);
  bool identity = ds->code_bytes == 1;
  int NB = 1;
  if (wide) {  // subbags within the split-finding limit: their in-bag rows with counts
    for (int r = 0; r < R; r++) {
      if (sfrac[r] < 1.0) continue;
      std::vector<uint64_t> e((size_t)inbag[r]);
      TRY(d2h(c, e.data(), entA + (size_t)r * cap, e.size()));
      items[r].resize(e.size());
      for (size_t k = 0; k < e.size(); k++)
        items[r][k] = {(uint32_t)e[k], (uint32_t)(e[k] >> 32) & 0xffu};
    }
  }
  {
    // replicas are independent: split finding runs on host threads
    const int nth = std::max(1, std::min<int>(R, HostPool::width()));
    std::vector<int> t_nb(nth, 1);
    std::vector<char> t_id(nth, 1);
    auto work = [&](int w) {
      for (int r = w; r < R; r += nth) {
        const bool sampled = sfrac[r] < 1.0;
        // (fraction * numExamples).toInt
        const int64_t nsamp = sampled ? (int64_t)(int32_t)(sfrac[r] * (double)nw[r]) : nw[r];
        if (wide) {
          // sparse value counts: the items' codes sorted and merged
          std::vector<std::pair<uint32_t, uint32_t>> cw;
          std::vector<double> sv;
          std::vector<uint32_t> sc;
          t_id[w] = 0;
          for (int fl = 0; fl < h_Fr[r]; fl++) {
            const int g = sub[r][fl];
            cw.clear();
            for (const auto& it : items[r])
              cw.emplace_back(ds->h_codes[(size_t)it.first * ds->S + g], it.second);
            std::sort(cw.begin(), cw.end());
            sv.clear();
            sc.clear();
            int szero = -1;
            for (size_t k = 0; k < cw.size(); k++) {
              if (k > 0 && cw[k].first == cw[k - 1].first) {
                sc.back() += cw[k].second;
                continue;
              }
              if ((int64_t)cw[k].first == ds->zero_code[g]) szero = (int)sv.size();
              sv.push_back(ds->dict[g][cw[k].first]);
              sc.push_back(cw[k].second);
            }
            std::vector<double>& t = thr[(size_t)r * Fmax + fl];
            const int nt = find_splits(sv, sc.data(), szero, nw[r], nsamp, tp.max_bins, t);
            h_nbins[(size_t)r * Fmax + fl] = nt + 1;
            t_nb[w] = std::max(t_nb[w], nt + 1);
            const auto& d = ds->dict[g];
            std::vector<uint32_t>& cu = cuts[(size_t)r * Fmax + fl];
            cu.resize(t.size());
            for (size_t j = 0; j < t.size(); j++)
              cu[j] = (uint32_t)(std::upper_bound(d.begin(), d.end(), t[j]) - d.begin());
          }
          continue;
        }
        for (int fl = 0; fl < h_Fr[r]; fl++) {
          const int g = sub[r][fl];
          const size_t rf = (size_t)r * Fmax + fl;
          const size_t o = (size_t)vcoff[rf];
          std::vector<double>& t = thr[rf];
          std::vector<uint32_t>& cu = cuts[rf];
          const auto& d = ds->dict[g];
          int nt;
          if (sampled && dev_splits) {  // k_find_splits' thresholds and cuts
            nt = dev_nt[rf];
            t.assign(dev_thr.begin() + rf * dev_tc, dev_thr.begin() + rf * dev_tc + nt);
            cu.assign(dev_cut.begin() + rf * dev_tc, dev_cut.begin() + rf * dev_tc + nt);
          } else {
            nt = find_splits(d, (sampled ? vcs.data() : vc.data()) + o, ds->zero_code[g], nw[r], nsamp,
                             tp.max_bins, t);
            // cut_j = #{dict values <= t_j}: #{t < d[k]} = #{j : cut_j <= k}
            cu.resize(t.size());
            for (size_t j = 0; j < t.size(); j++)
              cu[j] = (uint32_t)(std::upper_bound(d.begin(), d.end(), t[j]) - d.begin());
          }
          h_nbins[rf] = nt + 1;
          t_nb[w] = std::max(t_nb[w], nt + 1);
          // the codes are the bins when bin(k) = k for every code k < d.size() and there are no
          // more bins than codes (an implied 0.0 past a one-signed feature's values adds an empty
          // last bin, and the layouts are sized by the bin count: NB would fall one short)
          if ((int)d.size() != nt + 1) {
            t_id[w] = 0;
          } else {
            for (size_t j = 0; j + 1 < d.size(); j++)
              if (cu[j] != (uint32_t)(j + 1)) {
                t_id[w] = 0;
                break;
              }
          }
        }
      }
    };
    c->pool.run(nth, work);
    for (int w = 0; w < nth; w++) {
      NB = std::max(NB, t_nb[w]);
      identity = identity && t_id[w];
    }
    // thresholds beyond maxBins - 1 are Spark's (a split-finding sample larger than
    // numSamples passes one more target; RandomForest then sets numSplits to what it got):
    // NB follows them, but bins are u8 codes
    if (NB > 256)
      return fail(SBAG_EUNSUPPORTED, "more than 256 bins in a feature (maxBins 256 and a "
                                     "split-finding sample above numSamples)");
  }
  if (optimistic && identity) {
    NB = ncmax;  // the codes-as-bins root histogram already has this layout
    root_done = true;
  }
  // per global feature: are the cuts (the code -> bin map) the same for every replica that
  // uses it?
  bool shared = !wide;
  std::vector<int64_t> first_rf(F, -1);
  if (shared) {
    for (int r = 0; r < R && shared; r++)
      for (int fl = 0; fl < h_Fr[r] && shared; fl++) {
        const int g = sub[r][fl];
        const int64_t rf = (int64_t)r * Fmax + fl;
        if (first_rf[g] < 0)
          first_rf[g] = rf;
        else if (cuts[rf] != cuts[first_rf[g]])
          shared = false;
      }
  }
  // the cut table [rows][Fmax'][ncp] (padded with ~0u, ncp a power of two >= 32 holding the most
  // cuts: maxBins 32 with a 32nd threshold still takes 32 slots; k_bin_cuts binary-searches it)
  size_t maxcuts = 1;
  for (const auto& cu : cuts) maxcuts = std::max(maxcuts, cu.size());
  int32_t ncp = 32;
  while ((size_t)ncp < maxcuts) ncp *= 2;
  if (getenv("SBAG_DEBUG_BINS"))
    fprintf(stderr, "[sbag] cut table: maxcuts %zu ncp %d identity %d shared %d\n", maxcuts, ncp, (int)identity,
            (int)shared);
  // A threshold is a midpoint of two sampled values, so it lies above the smallest dictionary
  // value -- unless one of the two is the 0.0 that a sample short of numSamples implies for a
  // feature without zeros: a positive feature's first threshold (0 + v_0) / 2 lies below every
  // value (cut 0; the feature's bin 0 stays empty).  Such leading zero cuts leave the table
  // (k_bin_cuts' keys are cut - 1) and are added back per (row, feature) from d_z0.
  auto upload_cuts = [&](int rows, int fw, const std::function<const std::vector<uint32_t>*(int, int)>& at,
                         uint32_t** d_cut, const uint8_t** d_z0) -> int {
    std::vector<uint32_t> tab((size_t)rows * fw * ncp, 0xffffffffu);
    std::vector<uint8_t> z0((size_t)rows * fw, 0);
    bool any_z0 = false;
    for (int a = 0; a < rows; a++)
      for (int b = 0; b < fw; b++) {
        const std::vector<uint32_t>* cu = at(a, b);
        if (!cu) continue;
        size_t z = 0;
        while (z < cu->size() && (*cu)[z] == 0u) z++;
        if (z > 255) return fail(SBAG_EDEVICE, "internal: more than 255 thresholds below every value");
        z0[(size_t)a * fw + b] = (uint8_t)z;
        any_z0 = any_z0 || z > 0;
        std::copy(cu->begin() + z, cu->end(), tab.begin() + ((size_t)a * fw + b) * ncp);
      }
    TRY(ws_typed(c, "cut", tab.size(), d_cut));
    TRY(h2d(c, *d_cut, tab.data(), tab.size()));
    *d_z0 = nullptr;
    if (any_z0) {
      uint8_t* d;
      TRY(ws_typed(c, "cut_z0", z0.size(), &d));
      TRY(h2d(c, d, z0.data(), z0.size()));
      *d_z0 = d;
    }
    return SBAG_OK;
  };
  hmark(11);
  // ---- 5. bins
  const uint8_t* d_bins;
  int64_t bins_rstride = 0;
  const uint8_t* d_cols = nullptr;
  int64_t cols_rstride = 0, npad = 0;
  const uint32_t* d_planes = nullptr;
  int64_t plane_nw32 = 0;
  int plane_nsp = 0;
  int32_t S;
  std::vector<int16_t> h_pos((size_t)R * Fmax, 0);
  uint8_t* cols_direct = nullptr;  // per-replica column copy written by the materialization
  int64_t cols_direct_npad = 0;    // (its row padding)
  {
    int h = tm.begin(T_BIN);
    if (identity) {
      d_bins = (const uint8_t*)ds->d_codes;
      S = ds->S;
      h_pos = h_pos_codes;
    } else if (shared && (int64_t)N * row_stride(F) <= ((int64_t)64 << 30)) {
      // one bins matrix in global feature coordinates
      S = row_stride(F);
      std::vector<int32_t> gsub(F), gF(1, F);
      for (int g = 0; g < F; g++) gsub[g] = g;
      int32_t *d_gsub, *d_gF;
      uint32_t* d_cut;
      const uint8_t* d_z0;
      TRY(ws_typed(c, "gsub", (size_t)F, &d_gsub));
      TRY(ws_typed(c, "gF", 1, &d_gF));
      TRY(h2d(c, d_gsub, gsub.data(), (size_t)F));
      TRY(h2d(c, d_gF, gF.data(), 1));
      TRY(upload_cuts(1, F, [&](int, int g) { return first_rf[g] < 0 ? nullptr : &cuts[first_rf[g]]; },
                      &d_cut, &d_z0));
      uint8_t* d_b;
      TRY(ws_typed(c, "bins", (size_t)N * S + 256, &d_b));
      launch_bin_cuts(c->stream, ds->d_codes, ds->code_bytes, N, ds->S, d_gsub, d_gF, F, 1, d_cut, ncp, d_z0,
                      d_b, S, 0, nullptr, 0, 0, 0);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemsetAsync(d_b + (size_t)N * S, 0, 256, c->stream));  // zero slack
      d_bins = d_b;
      h_pos = h_pos_codes;
    } else {
      S = row_stride(Fmax);
      // integer labels: only the in-bag rows are binned, by rank (k_bin_ranked; the entries then
      // carry ranks).  SBAG_BIN_RANKED=0: every row (k_bin_cuts)
      const bool ranked = !f64 && (!getenv("SBAG_BIN_RANKED") || atoi(getenv("SBAG_BIN_RANKED")) != 0) &&
                          bin_ranked_fits(ds->code_bytes, ds->S, S, Fmax, ncp);
      int64_t capb = 0;
      for (int r = 0; r < R; r++) capb = std::max<int64_t>(capb, (int64_t)inbag[r]);
      const int64_t rows_b = ranked ? (capb + 1 + 63) / 64 * 64 : N;  // (room for the zero rows)
      // the bins and their column copy, per replica
      const double need = (double)R * rows_b * S + (double)R * Fmax * ((rows_b + 127) / 128 * 128);
      if (need > bins_budget(c)) {
        if (R > 1) {
          (void)hipEventDestroy(ev_start);
          (void)hipEventDestroy(ev_stop);
          return kSplitRange;
        }
        return fail(SBAG_EUNSUPPORTED, "per-replica bins of one learner exceed the device budget");
      }
      uint8_t* d_b;
      TRY(ws_typed(c, "bins", (size_t)R * rows_b * S + 256, &d_b));
      int ncol_r = 1;
      for (int r = 0; r < R; r++) ncol_r = std::max(ncol_r, (int)h_Fr[r]);
      {
        // bin(code) = #{t < dict[code]} = #{j : cut_j <= code} by VALU compares (k_bin_cuts),
        // the partition's column copy written by the same pass
        uint32_t* d_cut;
        const uint8_t* d_z0;
        TRY(upload_cuts(R, Fmax, [&](int r, int fl) { return fl < h_Fr[r] ? &cuts[(size_t)r * Fmax + fl] : nullptr; },
                        &d_cut, &d_z0));
        uint8_t* d_c;
        const int64_t npad_c = (rows_b + 127) / 128 * 128;
        TRY(ws_typed(c, "cols", (size_t)R * ncol_r * npad_c, &d_c));
        // (SBAG_BIN_NO_COLS=1: the column copy by k_transpose afterwards, A/B)
        static const bool no_cols = getenv("SBAG_BIN_NO_COLS") != nullptr;
        if (ranked) {
          if (!launch_bin_ranked(c->stream, ds->d_codes, ds->code_bytes, ds->S, entA, cap, d_inbag, capb, d_sub, d_Fr,
                                 Fmax, R, d_cut, ncp, d_z0, d_b, S, rows_b * S, d_c, ncol_r, npad_c,
                                 (int64_t)ncol_r * npad_c))
            return fail(SBAG_EDEVICE, "internal: ranked bins geometry");
          HIP_TRY(hipGetLastError());
          launch_rank_entries(c->stream, entA, cap, d_inbag, R, capb);
          cols_direct = d_c;
          cols_direct_npad = npad_c;
        } else if (launch_bin_cuts(c->stream, ds->d_codes, ds->code_bytes, N, ds->S, d_sub, d_Fr, Fmax, R, d_cut,
                                   ncp, d_z0, d_b, S, (int64_t)N * S, no_cols ? nullptr : d_c, ncol_r, npad_c,
                                   (int64_t)ncol_r * npad_c)) {
          cols_direct = d_c;
          cols_direct_npad = npad_c;
        }
      }
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemsetAsync(d_b + (size_t)R * rows_b * S, 0, 256, c->stream));  // zero slack
      d_bins = d_b;
      bins_rstride = rows_b * S;
      for (int r = 0; r < R; r++)
        for (int fl = 0; fl < h_Fr[r]; fl++) h_pos[(size_t)r * Fmax + fl] = (int16_t)fl;
    }
    // column-major copy for k_partition
    int ncol = 1;
    for (int r = 0; r < R; r++)
      for (int fl = 0; fl < h_Fr[r]; fl++) ncol = std::max(ncol, (int)h_pos[(size_t)r * Fmax + fl] + 1);
    const int Rc = bins_rstride ? R : 1;
    npad = cols_direct ? cols_direct_npad : (N + 63) / 64 * 64;
    cols_rstride = bins_rstride ? (int64_t)ncol * npad : 0;
    plane_nw32 = (N + 31) / 32;
    plane_nsp = NB - 1;
    // side-bit planes (bin > s) of the shared bins for the partition's gather, when
    // they fit in 24 GB (NB - 1 planes of N/8 bytes per column; C3 3.9 GB, C5 19.4 GB,
    // C4's 99 GB are left to the column gather).  C5, serialized: partition 38 -> 32 ms
    // per fit at levels with >= 1024 parents.
    auto planes_fit = [&](int nc, int nsp) {
      static const double cap_gb = getenv("SBAG_PLANES_MAX_GB") ? atof(getenv("SBAG_PLANES_MAX_GB")) : 24.0;
      return nsp >= 1 && (double)nc * nsp * plane_nw32 * 4 <= cap_gb * (1ull << 30) &&
             !getenv("SBAG_NO_PLANES");
    };
    if (identity && !getenv("SBAG_NO_LAYOUT_CACHE")) {
      // the codes are the bins: every column of every feature, once per dataset
      TRY(ensure_cols());
      std::lock_guard<std::mutex> lk(ds->layout_mu);
      if (!ds->planes_done) {
        ds->planes_done = true;
        const int nc = ds->cols_ncol;
        if (planes_fit(nc, plane_nsp)) {
          HIP_TRY(hipMalloc(&ds->d_planes, (size_t)nc * plane_nsp * plane_nw32 * 4));
          launch_planes(c->stream, ds->d_cols, npad, nc, plane_nsp, plane_nw32, ds->d_planes);
          HIP_TRY(hipGetLastError());
          ds->planes_nsp = plane_nsp;
          // other contexts (the learner-part twins) read them without this stream's order
          HIP_TRY(hipStreamSynchronize(c->stream));
        }
      }
      d_cols = ds->d_cols;
      if (ds->d_planes && ds->planes_nsp >= plane_nsp) {
        d_planes = ds->d_planes;
        plane_nsp = ds->planes_nsp;
      }
    } else {
      uint8_t* d_c = cols_direct;
      if (!d_c) {
        TRY(ws_typed(c, "cols", (size_t)Rc * ncol * npad, &d_c));
        launch_transpose(c->stream, d_bins, N, S, ncol, d_c, npad, Rc, bins_rstride, cols_rstride);
        HIP_TRY(hipGetLastError());
      }
      d_cols = d_c;
      if (bins_rstride == 0 && planes_fit(ncol, plane_nsp)) {
        uint32_t* d_pl;
        TRY(ws_typed(c, "planes", (size_t)ncol * plane_nsp * plane_nw32, &d_pl));
        launch_planes(c->stream, d_c, npad, ncol, plane_nsp, plane_nw32, d_pl);
        HIP_TRY(hipGetLastError());
        d_planes = d_pl;
      }
    }
    tm.end(h);
  }
  int32_t* d_nbins;
  TRY(ws_typed(c, "pos", h_pos.size(), &d_pos));
  TRY(ws_typed(c, "nbins", h_nbins.size(), &d_nbins));
  TRY(h2d(c, d_pos, h_pos.data(), h_pos.size()));
  TRY(h2d(c, d_nbins, h_nbins.data(), h_nbins.size()));

  // (the histograms read the bins rows in place: per-replica packed subspace rows were measured
  // on the C5 shard in round 4 -- hist 71.8 -> 69.8 ms per fit for 46 ms of packing, k_hist being
  // bound by its per-entry instructions, not the row bytes -- and removed in round 6)
  const uint8_t* hbins = d_bins;
  const int64_t hb_rstride = bins_rstride;
  const int32_t hS = S;
  const int16_t* hpos = d_pos;
  const std::vector<int16_t>& h_hpos = h_pos;

  hmark(12);
  // ---- 6. level-wise growth
  HistGeom g;
  if (!hist_geometry(hS, Fmax, NB, NS, gini, g, rl_mode_for(h_hpos, hS)))
    return fail(SBAG_EUNSUPPORTED, "histogram of one feature does not fit in LDS");
  TRY(maybe_grouped(g, hS, NB));
  if (ha.hct == 0) ha.hct = hist_layout_tile(g);  // else the optimistic root's layout
  const int64_t slot_words = (int64_t)Fmax * NB * NS;
  std::vector<std::vector<HNode>> trees(R);
  std::vector<std::pair<int, int>> slots(R);  // (replica, node index)
  for (int r = 0; r < R; r++) {
    trees[r].reserve((size_t)std::min<int64_t>((int64_t)1 << std::min(D + 1, 20), 2 * (int64_t)inbag[r] + 1));
    trees[r].push_back(HNode{});
    slots[r] = {r, 0};
  }
  ha.bins = hbins;
  ha.bins_rstride = hb_rstride;
  ha.S = hS;
  ha.pos = hpos;
  ha.NB = NB;
  ha.NS = NS;
  ha.count_only = 0;
  if (!root_done) {
    TRY(ws_get(c, "histA", (size_t)R * slot_words * word_bytes, &hist_cur));
    HIP_TRY(hipMemsetAsync(hist_cur, 0, (size_t)R * slot_words * word_bytes, c->stream));
    ha.ent_in = entA;
    ha.hist = hist_cur;
    TRY(launch(g, gini ? kHistGini : kHistVar, T_HIST, seg, h_par));
  }
  for (int r = 0; r < R; r++) hist_upper += (double)inbag[r] * (h_Fr[r] + s_y) * D + 3.0 * N * D;
  {
    std::vector<int> seg_r(R);
    for (int r = 0; r < R; r++) seg_r[r] = r;
    add_work(seg, seg_r);
  }
  if (f64) {
    // the integer histograms of the labels' fixed-point image (exact when the labels are
    // dyadic, SBAG_F64=1) screen the splits; Spark's row-order fp64 sums give the stats
    F64sGrow G{c, ds, lab, tp, R, N, Fmax, NB, S, h_Fr, h_nbins, thr, d_bins, bins_rstride, d_pos, d_Fr,
               d_nbins, h_pos, d_cols, cols_rstride, npad, entA, entB, cap, inbag, tm, hist_cur,
               slot_words, cmax, std::ldexp(1.0, -lshift),
               lab.label_ok ? 0.0 : std::ldexp(1.0, -lshift - 1),
               [&](const std::vector<std::pair<int64_t, int64_t>>& segs, const std::vector<ParentInfo>& par,
                   const uint64_t* ent, void* hist) -> int {
                 ha.ent_in = ent;
                 ha.hist = hist;
                 return launch(g, kHistVar, T_HIST, segs, par);
               },
               add_work, poff, d_y64, eyA, eyB};
    std::vector<std::vector<BtNode>> ftrees;
    TRY(grow_f64s(G, ftrees));
    HIP_TRY(hipEventRecord(ev_stop, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    forest->trees.resize(R);
    for (int r = 0; r < R; r++) {
      HTree& t = forest->trees[r];
      t.sub = sub[r];
      t.exact = exact[r];
      t.ns = 3;
      bt_emit(ftrees[r], 0, t);
    }
    forest->nclasses = 0;
    double cats[T_NCAT] = {0};
    tm.collect(cats, nullptr, -1);
    if (trace) {
      std::map<int, std::array<double, T_NCAT>> per;
      for (size_t i = 0; i < tm.ev.size(); i++) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, tm.ev[i].second.first, tm.ev[i].second.second);
        auto it = per.find(tm.lv[i]);
        if (it == per.end()) it = per.emplace(tm.lv[i], std::array<double, T_NCAT>{}).first;
        it->second[tm.ev[i].first] += ms;
      }
      for (auto& kv : per)
        fprintf(stderr, "[sbag] f64 level %d ms: hist %.2f screen+finish %.2f sub %.2f chain %.2f fix %.2f\n",
                kv.first, kv.second[T_HIST], kv.second[T_SPLIT], kv.second[T_SUB], kv.second[T_CHAIN],
                kv.second[T_FIX]);
    }
    float total_ms = 0;
    (void)hipEventElapsedTime(&total_ms, ev_start, ev_stop);
    (void)hipEventDestroy(ev_start);
    (void)hipEventDestroy(ev_stop);
    sbag_timing& T = forest->timing;
    T.total_ms = total_ms;
    T.sample_ms = cats[T_SAMPLE];
    T.valuecount_ms = cats[T_VC];
    T.bin_ms = cats[T_BIN];
    T.compact_ms = cats[T_COMPACT];
    T.hist_ms = cats[T_HIST];
    T.split_ms = cats[T_SPLIT];
    T.subtract_ms = cats[T_SUB];
    T.partition_ms = cats[T_PART];
    T.chain_ms = cats[T_CHAIN];
    T.root_ms = cats[T_ROOT];
    T.root_mfma_ops = root_mfma_ops;
    T.fix_ms = cats[T_FIX];
    T.exact_fallbacks = G.fallbacks;
    T.hist_launches = hist_launches;
    T.hist_alg_bytes = hist_alg_bytes;
    T.hist_entries = hist_entries;
    T.hist_lds_atomics = hist_lds;
    T.hist_work_bytes = hist_work;
    T.hist_upper_bytes = hist_upper;
    T.levels = G.levels;
    *out = forest.release();
    return SBAG_OK;
  }
  const double inv_scale = std::ldexp(1.0, -lab.shift), inv_scale2 = std::ldexp(1.0, -2 * lab.shift);
  uint64_t* ent_cur = entA;
  uint64_t* ent_nxt = entB;
  // Tile-resident gini entries (C5's class tiles): the root's class-tile grouping is kept
  // for the whole fit.  Every node is a list of ntc (node, class tile) sub-segments; the
  // partition splits each sub-segment in place (left from its front, right from its back:
  // k_partition with one parent per (node, tile)), so the children's entries are grouped
  // for their histograms and no level regroups -- k_tile_count / k_tile_scatter and their
  // host round trip ran before every histogram (18.9 ms per C5 shard fit, round 2).
  const int ntc_t = g.CT > 0 ? (NS + g.CT - 1) / g.CT : 1;
  // Off by default (SBAG_TILE_RESIDENT=1 turns it on): measured on the C5 shard it removed
  // the per-level grouping (18.9 -> 4.1 ms per fit) but the partition's (node, tile) pieces
  // cost as much (25.7 -> 40.2 ms) and their host setup more (serialized fit 181 -> 223 ms).
  const bool tile_res_env = getenv("SBAG_TILE_RESIDENT") && atoi(getenv("SBAG_TILE_RESIDENT")) != 0;
  const bool tile_res = tile_res_env && gini && g.grouped && !group_off &&
                        gtile_ent != nullptr && gtile_ct == g.CT &&
                        gtile_bounds.size() == (size_t)R * (ntc_t + 1);
  std::vector<std::pair<int64_t, int64_t>> tseg;  // [slot][ntc_t] sub-segments (tile_res)
  if (tile_res) {
    tseg.resize((size_t)R * ntc_t);
    for (int r = 0; r < R; r++)
      for (int t = 0; t < ntc_t; t++)
        tseg[(size_t)r * ntc_t + t] = {gtile_bounds[(size_t)r * (ntc_t + 1) + t],
                                       gtile_bounds[(size_t)r * (ntc_t + 1) + t + 1]};
    ent_cur = gtile_ent;
    hist_pregrouped = true;
  }
  std::string hist_nxt_name = "histB", hist_cur_name = "histA";
  // gini: the larger children's histograms are derived (parent - smaller child) inside the next
  // level's split search (k_split_gini), not by k_subtract; SBAG_NO_FUSED_SUB=1: k_subtract
  static const bool fused_sub = !getenv("SBAG_NO_FUSED_SUB");
  void* hist_prev = nullptr;        // the previous level's histograms (the derived slots' parents)
  std::vector<int32_t> derive;      // [2 slot] (parent slot, smaller-child slot) or -1
  int levels = 0;
  // exact sum of count*k^2 of every slot's node (variance screening): root from k_compact
  std::vector<uint64_t> slot_sq(R);
  for (int r = 0; r < R; r++) slot_sq[r] = inbag[3 * R + r];
  int64_t fallbacks = 0;
  std::unique_ptr<int64_t[]>& sst_buf = c->h_sst;  // split stats planes copied back per level
  size_t& sst_cap = c->h_sst_cap;
  for (int level = 0; level <= D; level++) {
    const int M = (int)slots.size();
    if (M == 0) break;
    levels++;
    trace_level = level;
    tm.level = level;
    hmark(7);
    // --- split search on the device
    std::vector<int32_t> h_slot_r(M);
    for (int i = 0; i < M; i++) h_slot_r[i] = slots[i].first;
    int32_t* d_slot_r;
    SplitOut* d_sout;
    int64_t* d_sstats;
    TRY(ws_typed(c, "slot_r", (size_t)M, &d_slot_r));
    TRY(ws_typed(c, "sout", (size_t)M, &d_sout));
    TRY(ws_typed(c, "sstats", (size_t)M * 3 * NS, &d_sstats));
    TRY(h2d(c, d_slot_r, h_slot_r.data(), (size_t)M));
    SplitArgs sa{};
    sa.hct = ha.hct;
    sa.hist = hist_cur;
    sa.Fmax = Fmax;
    sa.NB = NB;
    sa.NS = NS;
    sa.slot_r = d_slot_r;
    sa.Fr = d_Fr;
    sa.nbins = d_nbins;
    sa.min_inst = tp.min_instances_per_node;
    sa.min_gain = tp.min_info_gain;
    sa.inv_scale = inv_scale;
    sa.inv_scale2 = inv_scale2;
    sa.out = d_sout;
    sa.stats = d_sstats;
    sa.plane = (int64_t)M * NS;
    if (gini && fused_sub && !derive.empty()) {
      int32_t* d_der;
      TRY(ws_typed(c, "derive", derive.size(), &d_der));
      TRY(h2d(c, d_der, derive.data(), derive.size()));
      sa.derive = d_der;
      sa.par_hist = hist_prev;
      // (the derived histograms serve the next level's derivations: none after the last split)
      sa.hist_w = level + 1 < D ? hist_cur : nullptr;
    }
    if (!gini) {
      uint64_t* d_nsq;
      TRY(ws_typed(c, "node_sq", (size_t)M, &d_nsq));
      TRY(h2d(c, d_nsq, slot_sq.data(), (size_t)M));
      sa.node_sq = d_nsq;
    }
    {
      int h = tm.begin(T_SPLIT);
      if (gini)
        launch_split(c->stream, sa, M, true);
      else
        launch_split_screen(c->stream, sa, M);
      HIP_TRY(hipGetLastError());
      tm.end(h);
    }
    std::vector<SplitOut> sout(M);
    // stats planes [total][left][right] x [M][NS]; the host needs the left plane (a
    // node's total is known from its parent's split, right = total - left) and, at the
    // root, the totals
    // not value-initialized: at C5's deep levels M * 3 * NS words are ~50 MB, whose zero
    // fill was most of the host's per-level split setup (14 ms per fit)
    if (sst_cap < (size_t)M * 3 * NS) {
      sst_cap = (size_t)M * 3 * NS;
      sst_buf.reset(new int64_t[sst_cap]);
    }
    int64_t* sst = sst_buf.get();
    hmark(0);
    TRY(d2h(c, sout.data(), d_sout, (size_t)M));
    hmark(1);
    std::vector<char> exact(M, gini ? 1 : 0);
    if (!gini) {
      // nodes the screen could not decide: histogram their sums of squares (word 2)
      // from their own rows, then the exact Spark-order split
      std::vector<int32_t> fl_slots;
      for (int i = 0; i < M; i++)
        if (sout[i].pad) fl_slots.push_back(i);
      if (!fl_slots.empty()) {
        fallbacks += (int64_t)fl_slots.size();
        int h = tm.begin(T_FIX);
        int32_t* d_fs;
        TRY(ws_typed(c, "fix_slots", fl_slots.size(), &d_fs));
        TRY(h2d(c, d_fs, fl_slots.data(), fl_slots.size()));
        launch_zero_word(c->stream, (uint64_t*)hist_cur, d_fs, (int)fl_slots.size(), slot_words, 3, 2);
        HIP_TRY(hipGetLastError());
        tm.end(h);
        std::vector<std::pair<int64_t, int64_t>> fseg;
        std::vector<ParentInfo> fpar;
        for (int i : fl_slots) {
          fseg.push_back(seg[i]);
          fpar.push_back(ParentInfo{slots[i].first, -1, 0, 0, 0, i, 0, 0});
        }
        ha.ent_in = ent_cur;
        ha.hist = hist_cur;
        TRY(launch(g, kHistSq, T_FIX, fseg, fpar));
        SplitArgs sx = sa;
        sx.slot_ids = d_fs;
        h = tm.begin(T_FIX);
        launch_split(c->stream, sx, (int)fl_slots.size(), false);
        HIP_TRY(hipGetLastError());
        tm.end(h);
        TRY(d2h(c, sout.data(), d_sout, (size_t)M));
        for (int i : fl_slots) exact[i] = 1;
      }
    }
    if (level == 0)
      TRY(d2h(c, sst, d_sstats, (size_t)2 * M * NS));
    else
      TRY(d2h(c, sst + (size_t)M * NS, d_sstats + (size_t)M * NS, (size_t)M * NS));
    // --- node updates (RandomForest.findBestSplits, host part)
    struct Split {
      int slot, r, ni, li;
    };
    // a replica's slots are contiguous (slots keep replica order), so chunks of whole
    // replicas update their trees on host workers; concatenated in chunk order, the
    // parent lists are those of one sequential pass
    const int nch = M < 256 ? 1 : std::min(HostPool::width(), M / 128);
    std::vector<int> cb(nch + 1, M);
    cb[0] = 0;
    for (int w = 1; w < nch; w++) {
      int k = std::max(cb[w - 1], (int)((int64_t)M * w / nch));
      while (k > 0 && k < M && slots[k].first == slots[k - 1].first) k++;
      cb[w] = k;
    }
    std::vector<std::vector<ParentInfo>> cpar(nch);
    std::vector<std::vector<std::pair<int64_t, int64_t>>> cpseg(nch);
    std::vector<std::vector<Split>> cpsplit(nch);
    const std::function<void(int)> node_work = [&](int w) {
    std::vector<ParentInfo>& par = cpar[w];
    std::vector<std::pair<int64_t, int64_t>>& pseg = cpseg[w];
    std::vector<Split>& psplit = cpsplit[w];
    for (int i = cb[w]; i < cb[w + 1]; i++) {
      const int r = slots[i].first;
      const int ni = slots[i].second;
      const int64_t* lef = &sst[(size_t)M * NS + (size_t)i * NS];
      int64_t rig[kMaxHostNS];
      {
        HNode& n = trees[r][ni];
        if (level == 0) {
          const int64_t* tot = &sst[(size_t)i * NS];
          n.stats.assign(tot, tot + NS);
          n.impurity = Calc{n.stats.data(), NS, gini, lab.shift}.impurity();
        }
        for (int k = 0; k < NS; k++) rig[k] = n.stats[k] - lef[k];
        const SplitOut& so = sout[i];
        if (so.fl < 0) {  // no feature has splits: invalid stats on the parent aggregate
          n.gain = kDoubleMinValue;
          n.valid = false;
        } else {
          n.gain = so.gain;
          n.valid = so.valid != 0;
        }
        n.is_leaf = (n.gain <= 0) || (level == D);
        if (n.is_leaf) continue;
        n.has_split = true;
        n.fl = so.fl;
        n.s = so.s;
        n.thr = thr[(size_t)r * Fmax + so.fl][so.s];
      }
      const bool child_leaf = (level + 1) == D;
      HNode L, Rn;
      L.stats.assign(lef, lef + NS);
      Rn.stats.assign(rig, rig + NS);
      bool wl = !child_leaf, wr = !child_leaf;
      if (exact[i]) {  // children stats complete: leaf-by-purity known before routing
        if (gini && (sout[i].pad & 2)) {  // computed by k_split_gini
          L.impurity = sout[i].imp_l;
          Rn.impurity = sout[i].imp_r;
        } else {
          L.impurity = Calc{L.stats.data(), NS, gini, lab.shift}.impurity();
          Rn.impurity = Calc{Rn.stats.data(), NS, gini, lab.shift}.impurity();
        }
        wl = wl && L.impurity != 0.0;
        wr = wr && Rn.impurity != 0.0;
      }
      const int li = (int)trees[r].size();
      trees[r].push_back(std::move(L));
      trees[r].push_back(std::move(Rn));
      trees[r][ni].left = li;
      trees[r][ni].right = li + 1;
      if (!wl && !wr && exact[i]) {  // nothing to route, all stats known
        trees[r][li].is_leaf = trees[r][li + 1].is_leaf = true;
        continue;
      }
      ParentInfo p{};
      p.r = r;
      p.pos = h_pos[(size_t)r * Fmax + trees[r][ni].fl];
      p.s = trees[r][ni].s;
      p.write_l = wl;
      p.write_r = wr;
      p.hist_slot = -1;
      par.push_back(p);
      pseg.push_back(seg[i]);
      psplit.push_back(Split{i, r, ni, li});
    }
    };
    c->pool.run(nch, node_work);
    std::vector<ParentInfo> par;
    std::vector<std::pair<int64_t, int64_t>> pseg;
    std::vector<Split> psplit;
    for (int w = 0; w < nch; w++) {
      par.insert(par.end(), cpar[w].begin(), cpar[w].end());
      pseg.insert(pseg.end(), cpseg[w].begin(), cpseg[w].end());
      psplit.insert(psplit.end(), cpsplit[w].begin(), cpsplit[w].end());
    }
    const double hp2 = hp[2];
    hmark(2);
    if (par.empty()) {
      hp[23] = hp[2] - hp2;  // the last level's node updates
      break;
    }
    // tile-resident entries: one partition parent per (split node, non-empty class tile)
    const int NPn = (int)par.size();  // split nodes
    std::vector<int32_t> tq_first, tq_tile;
    if (tile_res) {
      std::vector<ParentInfo> tpar;
      std::vector<std::pair<int64_t, int64_t>> tps;
      tq_first.assign((size_t)NPn + 1, 0);
      for (int q = 0; q < NPn; q++) {
        tq_first[q] = (int)tpar.size();
        const size_t i = (size_t)psplit[q].slot;
        for (int t = 0; t < ntc_t; t++) {
          const auto& sub = tseg[i * ntc_t + t];
          if (sub.second <= sub.first) continue;
          tpar.push_back(par[q]);
          tps.push_back(sub);
          tq_tile.push_back(t);
        }
      }
      tq_first[NPn] = (int)tpar.size();
      par.swap(tpar);
      pseg.swap(tps);
    }
    // --- partition the rows of every split node into its children (and, for
    // variance, the exact sum of squares of each left child)
    const int NP = (int)par.size();
    std::vector<unsigned long long> cur((size_t)2 * NP), sql(NP, 0);
    for (int q = 0; q < NP; q++) {
      cur[2 * q] = (unsigned long long)pseg[q].first;
      cur[2 * q + 1] = (unsigned long long)pseg[q].second;
    }
    unsigned long long *d_cur, *d_sql = nullptr;
    TRY(ws_typed(c, "cursors", cur.size(), &d_cur));
    TRY(h2d(c, d_cur, cur.data(), cur.size()));
    if (!gini) {
      TRY(ws_typed(c, "sq_left", (size_t)NP, &d_sql));
      HIP_TRY(hipMemsetAsync(d_sql, 0, (size_t)NP * 8, c->stream));
    }
    hmark(13);
    {
      // work order: parents grouped by split column (replica copies apart), pieces of
      // 8192 entries interleaved round-robin across the parents of a group, so the
      // concurrent workgroups spread over the group's cursors while the GPU reads
      // one column
      static const int64_t piece =
          getenv("SBAG_PART_PIECE") ? std::max<int64_t>(1024, atoll(getenv("SBAG_PART_PIECE"))) : 8192;
      // the gathered object: a side-bit plane (column, split) once parents are many (with
      // few parents, finer groups would crowd the workgroups onto fewer cursors), else a
      // column byte array.  Crossover measured at 128-256 parents (C5 level 3 / 4: cols
      // 2.21 / 2.49 ms, planes 2.38 / 2.23; C3 flat within 0.1 ms from 128)
      static const int planes_min_np =
          getenv("SBAG_PLANES_MIN_PARENTS") ? atoi(getenv("SBAG_PLANES_MIN_PARENTS")) : 256;
      const bool lvl_planes = d_planes != nullptr && NP >= planes_min_np;
      auto colkey = [&](int q) {
        if (lvl_planes) return (int64_t)par[q].pos * plane_nsp + par[q].s;
        return (bins_rstride ? (int64_t)par[q].r * 65536 : 0) + (int64_t)par[q].pos;
      };
      // counting sort of the parents by column (pos < 65536; per replica when bins are)
      std::vector<int32_t> order(NP);
      {
        int64_t nkeys = 1;
        for (int q = 0; q < NP; q++) nkeys = std::max<int64_t>(nkeys, colkey(q) + 1);
        std::vector<int32_t> start;
        if (nkeys <= ((int64_t)1 << 24)) {
          start.assign((size_t)nkeys + 1, 0);
          for (int q = 0; q < NP; q++) start[(size_t)colkey(q) + 1]++;
          for (int64_t k = 0; k < nkeys; k++) start[(size_t)k + 1] += start[(size_t)k];
          for (int q = 0; q < NP; q++) order[start[(size_t)colkey(q)]++] = q;
        } else {
          for (int q = 0; q < NP; q++) order[q] = q;
          std::stable_sort(order.begin(), order.end(),
                           [&](int x, int y) { return colkey(x) < colkey(y); });
        }
      }
      // rounds: inside a column group (parents longest first), round k takes piece k
      // of every parent longer than k pieces; the piece list is written on the device
      std::vector<PartRound> rounds;
      std::vector<int64_t> segv((size_t)2 * NP);
      for (int q = 0; q < NP; q++) {
        segv[2 * q] = pseg[q].first;
        segv[2 * q + 1] = pseg[q].second;
      }
      int64_t npieces = 0;
      for (int g0 = 0; g0 < NP;) {
        int g1 = g0;
        while (g1 < NP && colkey(order[g1]) == colkey(order[g0])) g1++;
        std::sort(order.begin() + g0, order.begin() + g1, [&](int x, int y) {
          const int64_t lx = pseg[x].second - pseg[x].first, ly = pseg[y].second - pseg[y].first;
          return lx != ly ? lx > ly : x < y;
        });
        int act = g1 - g0;
        for (int64_t off = 0;; off += piece) {
          while (act > 0 && pseg[order[g0 + act - 1]].second - pseg[order[g0 + act - 1]].first <= off)
            act--;
          if (act == 0) break;
          rounds.push_back(PartRound{npieces, g0, act, off});
          npieces += act;
        }
        g0 = g1;
      }
      rounds.push_back(PartRound{npieces, NP, 0, 0});  // sentinel
      hmark(14);
      PartPiece* d_pp;
      PartRound* d_rounds;
      int32_t* d_order;
      int64_t* d_segv;
      unsigned long long* d_ctr;
      // sized once for the whole fit (a regrowth would hipFree = synchronize)
      TRY(ws_typed(c, "ppieces", (size_t)std::max<int64_t>(npieces, (int64_t)R * cap / piece + 65536),
                   &d_pp));
      TRY(ws_typed(c, "prounds", rounds.size(), &d_rounds));
      TRY(ws_typed(c, "porder", (size_t)NP, &d_order));
      TRY(ws_typed(c, "psegv", segv.size(), &d_segv));
      TRY(ws_typed(c, "pctr", 1, &d_ctr));
      TRY(h2d(c, d_rounds, rounds.data(), rounds.size()));
      TRY(h2d(c, d_order, order.data(), (size_t)NP));
      TRY(h2d(c, d_segv, segv.data(), segv.size()));
      launch_part_pieces(c->stream, d_rounds, (int)rounds.size() - 1, npieces, d_order, d_segv,
                         piece, d_pp);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemsetAsync(d_ctr, 0, 8, c->stream));
      TRY(ws_typed(c, "par", std::max<size_t>(par.size(), 1), &d_par));
      TRY(h2d(c, d_par, par.data(), par.size()));
      PartArgs pa{};
      pa.cols = d_cols;
      pa.cols_rstride = cols_rstride;
      pa.npad = npad;
      pa.planes = lvl_planes ? d_planes : nullptr;
      pa.nw32 = plane_nw32;
      pa.nsp = plane_nsp;
      pa.pieces = d_pp;
      pa.npieces = npieces;
      pa.counter = d_ctr;
      pa.parents = d_par;
      pa.ent_in = ent_cur;
      pa.ent_out = ent_nxt;
      pa.cursors = d_cur;
      pa.sq_left = d_sql;
      const int nwg = (int)std::max<int64_t>(1, std::min<int64_t>(npieces, 256 * 8));
      hmark(3);
      int h = tm.begin(T_PART);
      launch_partition(c->stream, pa, nwg);
      HIP_TRY(hipGetLastError());
      tm.end(h);
    }
    TRY(d2h(c, cur.data(), d_cur, cur.size()));
    hmark(4);
    if (!gini) TRY(d2h(c, sql.data(), d_sql, sql.size()));
    // --- children: complete stats, purity, the parent's exact gain; next slots
    std::vector<std::pair<int, int>> next_slots;
    std::vector<std::pair<int64_t, int64_t>> nseg;
    std::vector<uint64_t> next_sq;
    std::vector<int32_t> triples;
    std::vector<std::pair<int64_t, int64_t>> hseg;
    std::vector<ParentInfo> hpar;
    std::vector<std::pair<int64_t, int64_t>> ntseg;  // next slots' tile sub-segments
    // gini bags whose every draw count is 1 (without replacement): a child's class counts are
    // its entries per class, so the next histogram's class-tile grouping sizes are known
    // (SBAG_TILE_KNOWN=0: counted on the device as before)
    static const bool known_env = !(getenv("SBAG_TILE_KNOWN") && atoi(getenv("SBAG_TILE_KNOWN")) == 0);
    const int kct = g.CT > 0 ? g.CT : NS, kntc = (NS + kct - 1) / kct;
    const bool known_ok = gini && g.grouped && !tile_res && cmax <= 1 && known_env;
    std::vector<int64_t> hknown;
    for (int q = 0; q < NPn; q++) {
      const Split& sp = psplit[q];
      HNode& L = trees[sp.r][sp.li];
      HNode& Rn = trees[sp.r][sp.li + 1];
      if (!gini) {
        const uint64_t psq = (uint64_t)trees[sp.r][sp.ni].stats[2];
        if (exact[sp.slot]) {
          if ((uint64_t)L.stats[2] != sql[q])
            return fail(SBAG_EDEVICE, "internal: left sum of squares differs between histogram "
                                      "and partition");
        } else {
          L.stats[2] = (int64_t)sql[q];
          Rn.stats[2] = (int64_t)(psq - sql[q]);
          L.impurity = Calc{L.stats.data(), NS, gini, lab.shift}.impurity();
          Rn.impurity = Calc{Rn.stats.data(), NS, gini, lab.shift}.impurity();
          // Spark's gain of the chosen split (calculateImpurityStats, operation order)
          HNode& n = trees[sp.r][sp.ni];
          const double lc = (double)L.stats[0], rc = (double)Rn.stats[0];
          const double lw = lc / (lc + rc), rw = rc / (lc + rc);
          const double gain = n.impurity - lw * L.impurity - rw * Rn.impurity;
          if (!(gain > 0.0) || gain < tp.min_info_gain)
            return fail(SBAG_EDEVICE, "internal: screened split fails Spark's gain test");
          n.gain = gain;
        }
      }
      const bool child_leaf = (level + 1) == D;
      L.is_leaf = child_leaf || L.impurity == 0.0;
      Rn.is_leaf = child_leaf || Rn.impurity == 0.0;
      const bool wl = !L.is_leaf, wr = !Rn.is_leaf;
      int sl = -1, sr = -1;
      if (tile_res) {
        // child tile t: [sub.first, left cursor) and [right cursor, sub.second) of the
        // (node, tile) sub-segment; nseg keeps each child's entry count only
        for (int side = 0; side < 2; side++) {
          if (side == 0 ? !wl : !wr) continue;
          (side == 0 ? sl : sr) = (int)next_slots.size();
          next_slots.push_back({sp.r, sp.li + side});
          next_sq.push_back(0);
          const size_t b0 = ntseg.size();
          ntseg.resize(b0 + ntc_t, {0, 0});
          int64_t n = 0;
          for (int k = tq_first[q]; k < tq_first[q + 1]; k++) {
            const std::pair<int64_t, int64_t> sub =
                side == 0 ? std::make_pair(pseg[k].first, (int64_t)cur[2 * k])
                          : std::make_pair((int64_t)cur[2 * k + 1], pseg[k].second);
            ntseg[b0 + tq_tile[k]] = sub;
            n += sub.second - sub.first;
          }
          nseg.push_back({0, n});
        }
      } else {
        if (wl) {
          sl = (int)next_slots.size();
          next_slots.push_back({sp.r, sp.li});
          nseg.push_back({pseg[q].first, (int64_t)cur[2 * q]});
          next_sq.push_back(gini ? 0 : (uint64_t)L.stats[2]);
        }
        if (wr) {
          sr = (int)next_slots.size();
          next_slots.push_back({sp.r, sp.li + 1});
          nseg.push_back({(int64_t)cur[2 * q + 1], pseg[q].second});
          next_sq.push_back(gini ? 0 : (uint64_t)Rn.stats[2]);
        }
      }
      int hs = -1;
      if (wl && wr) {
        const bool small_left = Calc{L.stats.data(), NS, gini, lab.shift}.count() <=
                                Calc{Rn.stats.data(), NS, gini, lab.shift}.count();
        hs = small_left ? sl : sr;
        triples.push_back(small_left ? sr : sl);  // dst (larger child)
        triples.push_back(sp.slot);               // parent slot (current level)
        triples.push_back(hs);                    // small child
      } else if (wl || wr) {
        hs = wl ? sl : sr;
      }
      if (hs >= 0 && tile_res) {
        for (int t = 0; t < ntc_t; t++) {
          const auto& sub = ntseg[(size_t)hs * ntc_t + t];
          if (sub.second <= sub.first) continue;
          hseg.push_back(sub);
          hpar.push_back(ParentInfo{sp.r, -1, 0, 0, 0, hs, 0, t});
        }
      } else if (hs >= 0) {
        hseg.push_back(nseg[hs]);
        hpar.push_back(ParentInfo{sp.r, -1, 0, 0, 0, hs, 0, 0});
        if (known_ok) {  // its class counts are its entries per class: sizes per class tile
          const HNode& ch = trees[sp.r][sp.li + (hs == sl ? 0 : 1)];
          const size_t b0 = hknown.size();
          hknown.resize(b0 + (size_t)kntc, 0);
          for (int k = 0; k < NS; k++) hknown[b0 + (size_t)(k / kct)] += ch.stats[k];
        }
      }
    }
    hmark(5);
    if (next_slots.empty()) break;
    const int Mn = (int)next_slots.size();
    {
      std::vector<int> seg_r(Mn);
      for (int k = 0; k < Mn; k++) seg_r[k] = next_slots[k].first;
      add_work(nseg, seg_r);
    }
    // --- histograms of level+1: the smaller (or only) child of each split node
    void* hist_nxt;
    TRY(ws_get(c, hist_nxt_name, (size_t)Mn * slot_words * word_bytes, &hist_nxt));
    // only the slots histogrammed below start from zero (the subtraction overwrites the
    // rest): C5's deep levels memset ~10 GB per level otherwise.  A slot's u32 word count
    // is a multiple of 4 (16-byte aligned slots) when slot_words * word_bytes is.  Queued
    // by launch() after the class-tile grouping's count pass, so the host's wait for the
    // counts does not include the zeroing.
    pre_hist = [&, hist_nxt, Mn]() -> int {
      std::vector<int32_t> zs;
      zs.reserve(hpar.size());
      for (const ParentInfo& p : hpar)  // (a tile-resident slot's sub-segments are adjacent)
        if (zs.empty() || zs.back() != p.hist_slot) zs.push_back(p.hist_slot);
      const int64_t u32w = slot_words * (int64_t)word_bytes / 4;
      const int64_t tilew = zplan && zplan_ntc > 0 ? u32w / zplan_ntc : 0;
      if (zplan && (tilew & 3) == 0 && tilew * zplan_ntc == u32w) {
        // only shared slots whole, and the uncovered class tiles of the others (as blocks
        // of one tile's words: block index slot * ntc + tile)
        std::vector<int32_t> zfull, zblk;
        for (int32_t sl : zs) {
          const bool known = sl >= 0 && (size_t)sl < zplan_cov.size();
          if (!known || zplan_shared[sl]) {
            zfull.push_back(sl);
            continue;
          }
          for (int t = 0; t < zplan_ntc; t++)
            if (!((zplan_cov[sl] >> t) & 1ull)) zblk.push_back(sl * zplan_ntc + t);
        }
        static const bool ztrace = getenv("SBAG_LEVEL_TRACE") != nullptr;
        if (ztrace)
          fprintf(stderr, "[sbag] zeroed: %zu of %zu slots whole, %zu tile blocks\n", zfull.size(), zs.size(),
                  zblk.size());
        if (!zfull.empty()) {
          int32_t* d_zs;
          TRY(ws_typed(c, "zslots", zfull.size(), &d_zs));
          TRY(h2d(c, d_zs, zfull.data(), zfull.size()));
          launch_zero_slots(c->stream, hist_nxt, d_zs, (int)zfull.size(), u32w);
          HIP_TRY(hipGetLastError());
        }
        if (!zblk.empty()) {
          int32_t* d_zb;
          TRY(ws_typed(c, "zblocks", zblk.size(), &d_zb));
          TRY(h2d(c, d_zb, zblk.data(), zblk.size()));
          launch_zero_slots(c->stream, hist_nxt, d_zb, (int)zblk.size(), tilew);
          HIP_TRY(hipGetLastError());
        }
        return SBAG_OK;
      }
      if ((u32w & 3) == 0 && !zs.empty()) {
        int32_t* d_zs;
        TRY(ws_typed(c, "zslots", zs.size(), &d_zs));
        TRY(h2d(c, d_zs, zs.data(), zs.size()));
        launch_zero_slots(c->stream, hist_nxt, d_zs, (int)zs.size(), u32w);
        HIP_TRY(hipGetLastError());
      } else if (!zs.empty()) {
        HIP_TRY(hipMemsetAsync(hist_nxt, 0, (size_t)Mn * slot_words * word_bytes, c->stream));
      }
      return SBAG_OK;
    };
    ha.ent_in = ent_nxt;
    ha.hist = hist_nxt;
    known_tiles = known_ok && hknown.size() == hseg.size() * (size_t)kntc ? &hknown : nullptr;
    TRY(launch(g, gini ? kHistGini : kHistVar, T_HIST, hseg, hpar));
    known_tiles = nullptr;
    pre_hist = nullptr;
    derive.clear();
    if (!triples.empty() && gini && fused_sub) {
      // the next level's split search derives them (SplitArgs.derive)
      derive.assign((size_t)2 * Mn, -1);
      for (size_t k = 0; k + 2 < triples.size() + 1; k += 3) {
        derive[2 * (size_t)triples[k]] = triples[k + 1];
        derive[2 * (size_t)triples[k] + 1] = triples[k + 2];
      }
    } else if (!triples.empty()) {
      int32_t* d_tri;
      TRY(ws_typed(c, "triples", triples.size(), &d_tri));
      TRY(h2d(c, d_tri, triples.data(), triples.size()));
      int h = tm.begin(T_SUB);
      launch_subtract(c->stream, hist_nxt, hist_cur, d_tri, (int)triples.size() / 3, slot_words, gini);
      HIP_TRY(hipGetLastError());
      tm.end(h);
    }
    hist_prev = hist_cur;
    seg = nseg;
    if (tile_res) tseg.swap(ntseg);
    slots = next_slots;
    slot_sq = next_sq;
    std::swap(hist_cur_name, hist_nxt_name);
    hist_cur = hist_nxt;
    std::swap(ent_cur, ent_nxt);
    hmark(6);
  }
  HIP_TRY(hipEventRecord(ev_stop, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  hmark(20);

  // ---- 7. models (toNode(prune = true)) + subspaces, trees on host threads
  forest->trees.resize(R);
  int nclasses = 0;
  std::vector<int> ns_of(R, 3);
  for (int r = 0; r < R; r++) {
    if (gini) {  // Classifier.getNumClasses on the subbag: max label + 1
      int ns_out = 0;
      for (int k = 0; k < NS; k++)
        if (trees[r][0].stats[k] > 0) ns_out = k + 1;
      ns_of[r] = ns_out;
      nclasses = std::max(nclasses, ns_out);
    }
  }
  {
    const int nth = std::max(1, std::min<int>(R, HostPool::width()));
    const std::function<void(int)> work = [&](int w) {
      for (int r = w; r < R; r += nth) {
        HTree& t = forest->trees[r];
        t.sub = sub[r];
        t.exact = exact[r];
        t.ns = ns_of[r];
        // (at most one emitted node per learning node: no regrowth of C5's 4-MB stats arrays)
        t.nodes.reserve(trees[r].size());
        t.stats.reserve(trees[r].size() * (size_t)ns_of[r]);
        emit(trees[r], 0, t, NS, gini, lab.shift, ns_of[r]);
      }
    };
    c->pool.run(nth, work);
  }
  hmark(21);
  forest->nclasses = gini ? std::max(nclasses, (int)lab.kmax + 1) : 0;
  double cats[T_NCAT] = {0};
  tm.collect(cats, nullptr, -1);
  if (trace) {
    // per level and category: ms (categories as in enum T_*)
    std::map<int, std::array<double, T_NCAT>> per;
    for (size_t i = 0; i < tm.ev.size(); i++) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, tm.ev[i].second.first, tm.ev[i].second.second);
      auto it = per.find(tm.lv[i]);
      if (it == per.end()) it = per.emplace(tm.lv[i], std::array<double, T_NCAT>{}).first;
      it->second[tm.ev[i].first] += ms;
    }
    for (auto& kv : per) {
      fprintf(stderr, "[sbag] level %d ms: sample %.2f vc %.2f bin %.2f compact %.2f group %.2f hist %.2f "
              "split %.2f sub %.2f part %.2f fix %.2f\n", kv.first, kv.second[T_SAMPLE], kv.second[T_VC],
              kv.second[T_BIN], kv.second[T_COMPACT], kv.second[T_GROUP], kv.second[T_HIST],
              kv.second[T_SPLIT], kv.second[T_SUB], kv.second[T_PART], kv.second[T_FIX]);
    }
  }
  float total_ms = 0;
  (void)hipEventElapsedTime(&total_ms, ev_start, ev_stop);
  (void)hipEventDestroy(ev_start);
  (void)hipEventDestroy(ev_stop);
  sbag_timing& T = forest->timing;
  T.total_ms = total_ms;
  T.sample_ms = cats[T_SAMPLE];
  T.valuecount_ms = cats[T_VC];
  T.bin_ms = cats[T_BIN];
  T.compact_ms = cats[T_COMPACT];
  T.hist_ms = cats[T_HIST];
  T.split_ms = cats[T_SPLIT];
  T.subtract_ms = cats[T_SUB];
  T.partition_ms = cats[T_PART];
  T.hist_work_bytes = hist_work;
  T.fix_ms = cats[T_FIX];
  T.group_ms = cats[T_GROUP];
  T.root_ms = cats[T_ROOT];
  T.root_mfma_ops = root_mfma_ops;
  T.exact_fallbacks = fallbacks;
  T.hist_launches = hist_launches;
  T.hist_alg_bytes = hist_alg_bytes;
  T.hist_entries = hist_entries;
  T.hist_lds_atomics = hist_lds;
  T.hist_upper_bytes = hist_upper;
  T.levels = levels;
  hmark(15);
  if (hprof)
    fprintf(stderr, "host ms: setup+sample-launch %.2f compact-wait %.2f valuecounts %.2f thresholds %.2f "
                    "bins %.2f | split-prep %.2f split-wait %.2f nodes %.2f part-cursors %.2f part-sort %.2f "
                    "part-upload %.2f part-wait %.2f children %.2f hist-prep %.2f loop %.2f | emit %.2f"
                    " | in hist launches: grouping %.2f (count wait %.2f, prefix %.2f) work lists %.2f\n",
            hp[8], hp[9], hp[10], hp[11], hp[12], hp[0], hp[1], hp[2], hp[13], hp[14], hp[3], hp[4], hp[5],
            hp[6], hp[7], hp[15], hp[16], hp[18], hp[19], hp[17]);
  if (hprof) {
    fprintf(stderr, "host ms: tail: last level's nodes %.2f stream sync %.2f emit %.2f collect %.2f\n", hp[23], hp[20],
            hp[21], hp[15]);
    htail.t15 = hnow();
  }
  // the trees' nodes and the per-replica threshold tables are freed on the context's reaper
  // thread, not between this fit's last kernel and the next fit's first
  c->reaper.post(std::make_shared<std::tuple<std::vector<std::vector<HNode>>, std::vector<std::vector<double>>,
                                             std::vector<std::vector<uint32_t>>,
                                             std::vector<std::pair<int64_t, int64_t>>>>(
      std::move(trees), std::move(thr), std::move(cuts), std::move(tseg)));
  *out = forest.release();
  return SBAG_OK;
}

// ---------------------------------------------------------------- forest accessors
int sbag_forest_num_trees(const sbag_forest* f, int32_t* n) {
  if (!f || !n) return fail(SBAG_EINVAL, "bad arguments");
  *n = (int32_t)f->trees.size();
  return SBAG_OK;
}
int sbag_forest_tree_info(const sbag_forest* f, int32_t t, int32_t* nn, int32_t* ns, int32_t* sl,
                          int32_t* ex) {
  if (!f || t < 0 || t >= (int)f->trees.size()) return fail(SBAG_EINVAL, "tree index out of range");
  const HTree& h = f->trees[t];
  if (nn) *nn = (int32_t)h.nodes.size();
  if (ns) *ns = h.ns;
  if (sl) *sl = (int32_t)h.sub.size();
  if (ex) *ex = h.exact;
  return SBAG_OK;
}
int sbag_forest_subspace(const sbag_forest* f, int32_t t, int32_t* idx) {
  if (!f || !idx || t < 0 || t >= (int)f->trees.size()) return fail(SBAG_EINVAL, "bad arguments");
  std::copy(f->trees[t].sub.begin(), f->trees[t].sub.end(), idx);
  return SBAG_OK;
}
int sbag_forest_nodes(const sbag_forest* f, int32_t t, sbag_node* nodes, double* stats) {
  if (!f || !nodes || t < 0 || t >= (int)f->trees.size()) return fail(SBAG_EINVAL, "bad arguments");
  const HTree& h = f->trees[t];
  std::copy(h.nodes.begin(), h.nodes.end(), nodes);
  if (stats) std::copy(h.stats.begin(), h.stats.end(), stats);
  return SBAG_OK;
}
int sbag_forest_timing(const sbag_forest* f, sbag_timing* out) {
  if (!f || !out) return fail(SBAG_EINVAL, "bad arguments");
  *out = f->timing;
  return SBAG_OK;
}
// Model load / JNI round trip: the arrays come from disk or another process, so every
// link, index and class id the predict kernels will follow is checked first (a bad
// child link would walk out of the tree or loop forever on the device).
int sbag_forest_create(int32_t T, const int32_t* num_nodes, const sbag_node* nodes,
                       const int32_t* sub_len, const int32_t* subs, int32_t impurity,
                       sbag_forest** out) {
  if (T <= 0 || !num_nodes || !nodes || !sub_len || !subs || !out)
    return fail(SBAG_EINVAL, "bad arguments");
  if (impurity != SBAG_IMPURITY_VARIANCE && impurity != SBAG_IMPURITY_GINI)
    return fail(SBAG_EINVAL, "unknown impurity");
  auto f = std::make_unique<sbag_forest>();
  f->impurity = impurity;
  f->trees.resize(T);
  int64_t no = 0, so = 0;
  int nclasses = 0;
  for (int t = 0; t < T; t++) {
    const std::string bad = "malformed tree " + std::to_string(t) + ": ";
    if (num_nodes[t] <= 0 || sub_len[t] < 0) return fail(SBAG_EINVAL, bad + "empty");
    HTree& h = f->trees[t];
    h.nodes.assign(nodes + no, nodes + no + num_nodes[t]);
    h.sub.assign(subs + so, subs + so + sub_len[t]);
    for (int32_t g : h.sub)
      if (g < 0) return fail(SBAG_EINVAL, bad + "negative subspace index");
    const int n = num_nodes[t];
    for (int i = 0; i < n; i++) {
      const sbag_node& nd = h.nodes[i];
      if (nd.left >= 0 || nd.right >= 0) {
        // pre-order ids: both children exist, lie inside the tree and after their parent,
        // so every walk strictly advances and ends at a leaf
        if (!(nd.left > i && nd.right > i && nd.left < n && nd.right < n && nd.left != nd.right))
          return fail(SBAG_EINVAL, bad + "node " + std::to_string(i) + " has bad child links");
        if (nd.feature < 0 || nd.feature >= sub_len[t])
          return fail(SBAG_EINVAL, bad + "node " + std::to_string(i) + " splits outside the subspace");
      } else if (impurity == SBAG_IMPURITY_GINI) {
        const double v = nd.prediction;
        if (!(v >= 0 && v == std::floor(v) && v < 4096))
          return fail(SBAG_EINVAL, bad + "leaf " + std::to_string(i) + " predicts no class id");
        nclasses = std::max(nclasses, (int)v + 1);
      }
    }
    no += num_nodes[t];
    so += sub_len[t];
  }
  f->nclasses = nclasses;
  *out = f.release();
  return SBAG_OK;
}
int sbag_forest_free(sbag_forest* f) {
  delete f;
  return SBAG_OK;
}

// ---------------------------------------------------------------- predict
// this device's copy of the forest's nodes (built once per device under the forest's lock)
static int upload_forest(sbag_ctx* c, const sbag_forest* fc, const DevNode** d_nodes,
                         const int64_t** d_off) {
  sbag_forest* f = const_cast<sbag_forest*>(fc);
  std::lock_guard<std::mutex> lk(f->dev_mu);
  auto it = f->dev.find(c->device);
  if (it != f->dev.end()) {
    *d_nodes = it->second.nodes;
    *d_off = it->second.off;
    return SBAG_OK;
  }
  std::vector<DevNode> dn;
  std::vector<int64_t> off;
  for (const HTree& t : f->trees) {
    off.push_back((int64_t)dn.size());
    for (const sbag_node& n : t.nodes) {
      DevNode d{};
      d.left = n.left;
      d.right = n.right;
      d.value = n.left >= 0 ? n.threshold : n.prediction;
      d.gfeat = n.left >= 0 ? t.sub[n.feature] : 0;
      dn.push_back(d);
    }
  }
  sbag_forest::DevCopy cp;
  HIP_TRY(hipMalloc(&cp.nodes, std::max<size_t>(dn.size(), 1) * sizeof(DevNode)));
  if (hipMalloc(&cp.off, std::max<size_t>(off.size(), 1) * 8) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(cp.nodes);
    return fail(SBAG_ENOMEM, "device allocation of the forest failed");
  }
  f->dev[c->device] = cp;  // owned by the forest from here on
  HIP_TRY(hipMemcpy(cp.nodes, dn.data(), dn.size() * sizeof(DevNode), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(cp.off, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  *d_nodes = cp.nodes;
  *d_off = cp.off;
  return SBAG_OK;
}

static int check_agg(const sbag_forest* f, int agg) {
  if (agg != SBAG_AGG_MEAN && agg != SBAG_AGG_MODE) return fail(SBAG_EINVAL, "unknown aggregation");
  if (agg == SBAG_AGG_MODE && (f->nclasses <= 0 || f->nclasses > 4096))
    return fail(SBAG_EINVAL, "mode aggregation needs class-valued trees");
  return SBAG_OK;
}

// Mode counters past the LDS (more than kLdsModeClasses classes): u16 [nclasses][rows]
// in global memory, at most 256 MB, the rows then processed in batches of *rows_out.
static int mode_counters(sbag_ctx* c, int agg, int nclasses, int64_t N, uint16_t** d_out,
                         int64_t* rows_out) {
  *d_out = nullptr;
  *rows_out = 0;
  if (agg != SBAG_AGG_MODE || nclasses <= kLdsModeClasses) return SBAG_OK;
  const int64_t rows = std::max<int64_t>(256, std::min<int64_t>(N, ((int64_t)256 << 20) / (2 * nclasses)));
  TRY(ws_typed(c, "mode_cnt", (size_t)nclasses * rows, d_out));
  *rows_out = rows;
  return SBAG_OK;
}

}  // extern "C" (host helpers of the predict entry points)

// ---- LDS-tiled predict plan: trees relaid breadth first (children adjacent),
// thresholds compiled to code space by `tc_of(g, thr)` = the largest code whose
// value is <= thr, trees chunked to the LDS budget.  false: a tree does not fit
// (very deep trees / very wide rows) -> the global-memory walk.
struct TiledPlan {
  std::vector<PNode> pn;
  std::vector<double> lv;
  std::vector<int64_t> tn, tl;
  std::vector<PredictChunk> chunks;
};

template <typename TC>
static bool plan_tiled(const sbag_forest* f, PredictArgs& pa, int F, TC tc_of, TiledPlan& P) {
  const int L = (int)f->trees.size();
  pa.L = L;
  pa.nclasses = std::max(f->nclasses, 1);
  pa.chunk_bytes = 0;
  const size_t fixed = predict_tiled_lds(pa);
  const size_t lds_cap = 160 * 1024 - 512;
  if (F >= 32768 || fixed + 4096 > lds_cap) return false;
  const int budget = (int)std::min<size_t>(64 * 1024, lds_cap - fixed) & ~15;
  pa.chunk_bytes = budget;
  P.tn.assign(L, 0);
  P.tl.assign(L, 0);
  for (int t = 0; t < L; t++) {
    const HTree& h = f->trees[t];
    P.tn[t] = (int64_t)P.pn.size();
    P.tl[t] = (int64_t)P.lv.size();
    std::vector<int> order{0}, pos(h.nodes.size(), -1);
    pos[0] = 0;
    for (size_t k = 0; k < order.size(); k++) {
      const sbag_node& n = h.nodes[order[k]];
      if (n.left >= 0) {
        pos[n.left] = (int)order.size();
        order.push_back(n.left);
        pos[n.right] = (int)order.size();
        order.push_back(n.right);
      }
    }
    for (int k : order) {
      const sbag_node& n = h.nodes[k];
      PNode q{};
      if (n.left >= 0) {
        const int g = h.sub[n.feature];
        const int64_t tc = tc_of(g, n.threshold);
        if (tc + 1 >= (1 << 17)) return false;
        q.a = (uint32_t)pos[n.left];
        q.b = ((uint32_t)g << 17) | (uint32_t)(tc + 1);
      } else {
        q.a = 0x80000000u | (uint32_t)(P.lv.size() - P.tl[t]);
        P.lv.push_back(n.prediction);
      }
      P.pn.push_back(q);
    }
    const int64_t tb = (int64_t)(P.pn.size() - P.tn[t]) * 8 + (int64_t)(P.lv.size() - P.tl[t]) * 8;
    if (tb > budget) return false;
    if (P.chunks.empty() ||
        (P.chunks.back().n1 - P.chunks.back().n0 + P.chunks.back().l1 - P.chunks.back().l0) * 8 + tb > budget)
      P.chunks.push_back(PredictChunk{t, t, P.tn[t], P.tn[t], P.tl[t], P.tl[t]});
    PredictChunk& ch = P.chunks.back();
    ch.t1 = t + 1;
    ch.n1 = (int64_t)P.pn.size();
    ch.l1 = (int64_t)P.lv.size();
  }
  return true;
}

static int upload_plan(sbag_ctx* c, const TiledPlan& P, PredictArgs& pa) {
  PNode* d_pn;
  double* d_lv;
  int64_t *d_tn, *d_tl;
  PredictChunk* d_ch;
  TRY(ws_typed(c, "pd_nodes", P.pn.size(), &d_pn));
  TRY(ws_typed(c, "pd_leaves", std::max<size_t>(P.lv.size(), 1), &d_lv));
  TRY(ws_typed(c, "pd_tn", P.tn.size(), &d_tn));
  TRY(ws_typed(c, "pd_tl", P.tl.size(), &d_tl));
  TRY(ws_typed(c, "pd_chunks", P.chunks.size(), &d_ch));
  TRY(h2d(c, d_pn, P.pn.data(), P.pn.size()));
  TRY(h2d(c, d_lv, P.lv.data(), P.lv.size()));
  TRY(h2d(c, d_tn, P.tn.data(), P.tn.size()));
  TRY(h2d(c, d_tl, P.tl.data(), P.tl.size()));
  TRY(h2d(c, d_ch, P.chunks.data(), P.chunks.size()));
  pa.nodes = d_pn;
  pa.leaves = d_lv;
  pa.tree_node = d_tn;
  pa.tree_leaf = d_tl;
  pa.chunks = d_ch;
  pa.nchunks = (int)P.chunks.size();
  return SBAG_OK;
}

extern "C" {

int sbag_predict(sbag_ctx* c, const sbag_forest* f, const double* X, int64_t N, int32_t F, int32_t agg,
                 double* out, double* per_tree) {
  if (!c || !f || !X || !out || N < 0 || F <= 0) return fail(SBAG_EINVAL, "bad arguments");
  CTX_LOCK(c);
  TRY(check_agg(f, agg));
  for (const HTree& t : f->trees)
    for (int32_t g : t.sub)
      if (g >= F) return fail(SBAG_EINVAL, "feature vector shorter than a subspace index");
  if (N == 0) return SBAG_OK;
  HIP_TRY(hipSetDevice(c->device));
  const int L = (int)f->trees.size();
  double *d_out, *d_pt = nullptr;
  TRY(ws_typed(c, "pout", (size_t)N, &d_out));
  // batched transform: rows go up in batches, are binned on the device against the
  // forest's own thresholds (code = #{thresholds of the feature < x}, so
  // x <= threshold_k <=> code <= k, exact; NaN -> past every threshold) and walk
  // the LDS-tiled forest
  std::vector<std::vector<double>> T(F);
  for (const HTree& t : f->trees)
    for (const sbag_node& n : t.nodes)
      if (n.left >= 0) T[t.sub[n.feature]].push_back(n.threshold);
  std::vector<int64_t> toff(F + 1, 0);
  for (int g = 0; g < F; g++) {
    std::sort(T[g].begin(), T[g].end());
    T[g].erase(std::unique(T[g].begin(), T[g].end()), T[g].end());
    toff[g + 1] = toff[g] + (int64_t)T[g].size();
  }
  const int32_t Sq = (F + 15) / 16 * 16;
  PredictArgs pa{};
  pa.code_bytes = 2;
  pa.S = Sq;
  pa.agg = agg;
  TiledPlan P;
  const bool tiled = per_tree == nullptr &&
                     plan_tiled(f, pa, F, [&](int g, double thr) {
                       return (int64_t)(std::lower_bound(T[g].begin(), T[g].end(), thr) - T[g].begin());
                     }, P);
  if (tiled) {
    std::vector<double> tv((size_t)std::max<int64_t>(toff[F], 1));
    for (int g = 0; g < F; g++) std::copy(T[g].begin(), T[g].end(), tv.begin() + toff[g]);
    double* d_T;
    int64_t* d_toff;
    TRY(ws_typed(c, "pq_thr", tv.size(), &d_T));
    TRY(ws_typed(c, "pq_off", toff.size(), &d_toff));
    TRY(h2d(c, d_T, tv.data(), tv.size()));
    TRY(h2d(c, d_toff, toff.data(), toff.size()));
    TRY(upload_plan(c, P, pa));
    int64_t batch = std::max<int64_t>(1, std::min<int64_t>(N, ((int64_t)2 << 30) / (8 * (int64_t)F)));
    if (const char* e = getenv("SBAG_PREDICT_BATCH_ROWS")) batch = std::max<int64_t>(1, std::min<int64_t>(batch, atoll(e)));
    double* d_X;
    uint16_t* d_codes;
    TRY(ws_typed(c, "pX", (size_t)batch * F, &d_X));
    TRY(ws_typed(c, "pq_codes", (size_t)batch * Sq, &d_codes));
    for (int64_t r0 = 0; r0 < N; r0 += batch) {
      const int64_t n = std::min(batch, N - r0);
      HIP_TRY(hipMemcpyAsync(d_X, X + r0 * F, (size_t)n * F * 8, hipMemcpyHostToDevice, c->stream));
      launch_quantize(c->stream, d_X, n, F, d_T, d_toff, d_codes, Sq);
      pa.codes = d_codes;
      pa.N = n;
      pa.out = d_out + r0;
      launch_predict_tiled(c->stream, pa);
      HIP_TRY(hipGetLastError());
    }
    TRY(d2h(c, out, d_out, (size_t)N));
    return SBAG_OK;
  }
  const DevNode* f_nodes = nullptr;
  const int64_t* f_off = nullptr;
  TRY(upload_forest(c, f, &f_nodes, &f_off));
  double* d_X;
  TRY(ws_typed(c, "pX", (size_t)N * F, &d_X));
  if (per_tree) TRY(ws_typed(c, "ppt", (size_t)N * L, &d_pt));
  TRY(h2d(c, d_X, X, (size_t)N * F));
  uint16_t* d_gcnt = nullptr;
  int64_t gcnt_rows = 0;
  TRY(mode_counters(c, agg, f->nclasses, N, &d_gcnt, &gcnt_rows));
  launch_predict(c->stream, d_X, nullptr, 1, nullptr, nullptr, N, F, F, f_nodes, f_off, L, agg,
                 std::max(f->nclasses, 1), d_out, d_pt, nullptr, 0, d_gcnt, gcnt_rows);
  HIP_TRY(hipGetLastError());
  TRY(d2h(c, out, d_out, (size_t)N));
  if (per_tree) TRY(d2h(c, per_tree, d_pt, (size_t)N * L));
  return SBAG_OK;
}

// Forest over a device dataset into device memory: kAggMean / kAggMode -> fp64 [N],
// kAggSum -> fp64 [N] in-order sum over the forest's trees, kAggVotes -> [L][N] class
// ids (vote_bytes 1 or 2).  d_out == nullptr: into the context's workspace (*d_res).
static int predict_dataset_dev(sbag_ctx* c, const sbag_forest* f, const sbag_dataset* ds, int agg,
                               int vote_bytes, void* d_out, void** d_res) {
  for (const HTree& t : f->trees)
    for (int32_t g : t.sub)
      if (g >= ds->F) return fail(SBAG_EINVAL, "dataset has fewer features than the model");
  if (ds->ctx->device != c->device)
    return fail(SBAG_EINVAL, "dataset lives on device " + std::to_string(ds->ctx->device) +
                                 ", the context on device " + std::to_string(c->device));
  HIP_TRY(hipSetDevice(c->device));
  const int L = (int)f->trees.size();
  if (!d_out) {
    const size_t bytes = agg == kAggVotes ? (size_t)L * ds->N * vote_bytes : (size_t)ds->N * 8;
    TRY(ws_get(c, "pout", bytes, &d_out));
  }
  if (d_res) *d_res = d_out;
  if (ds->N == 0) return SBAG_OK;
  double* d_o = agg == kAggVotes ? nullptr : (double*)d_out;
  void* d_votes = agg == kAggVotes ? d_out : nullptr;
  PredictArgs pa{};
  pa.code_bytes = ds->code_bytes;
  pa.S = ds->S;
  pa.N = ds->N;
  pa.agg = agg;
  pa.vote_bytes = vote_bytes;
  TiledPlan P;
  // TreePoint's `value <= threshold` in the dataset's code space (dict sorted ascending)
  const bool tiled = ds->code_bytes != 4 && plan_tiled(f, pa, ds->F, [&](int g, double thr) {
    const std::vector<double>& d = ds->dict[g];
    return (int64_t)(std::upper_bound(d.begin(), d.end(), thr) - d.begin()) - 1;
  }, P);
  if (tiled) {
    TRY(upload_plan(c, P, pa));
    pa.codes = ds->d_codes;
    pa.out = d_o;
    pa.votes = d_votes;
    launch_predict_tiled(c->stream, pa);
  } else {  // very deep trees, very wide rows or many classes: node walk from global memory
    const DevNode* f_nodes = nullptr;
    const int64_t* f_off = nullptr;
    TRY(upload_forest(c, f, &f_nodes, &f_off));
    uint16_t* d_gcnt = nullptr;
    int64_t gcnt_rows = 0;
    TRY(mode_counters(c, agg, f->nclasses, ds->N, &d_gcnt, &gcnt_rows));
    launch_predict(c->stream, nullptr, ds->d_codes, ds->code_bytes, ds->d_dict, ds->d_dict_off, ds->N,
                   ds->F, ds->S, f_nodes, f_off, L, agg, std::max(f->nclasses, 1), d_o, nullptr,
                   d_votes, vote_bytes, d_gcnt, gcnt_rows);
  }
  HIP_TRY(hipGetLastError());
  return SBAG_OK;
}

int sbag_predict_dataset(sbag_ctx* c, const sbag_forest* f, const sbag_dataset* ds, int32_t agg,
                         double* out) {
  if (!c || !f || !ds || !out) return fail(SBAG_EINVAL, "bad arguments");
  CTX_LOCK(c);
  TRY(check_agg(f, agg));
  void* d_out = nullptr;
  TRY(predict_dataset_dev(c, f, ds, agg, 0, nullptr, &d_out));
  TRY(d2h(c, out, (const double*)d_out, (size_t)ds->N));
  return SBAG_OK;
}

int sbag_predict_dataset_device(sbag_ctx* c, const sbag_forest* f, const sbag_dataset* ds,
                                int32_t out_kind, int32_t vote_bytes, void* d_out) {
  if (!c || !f || !ds || !d_out) return fail(SBAG_EINVAL, "bad arguments");
  if (out_kind != SBAG_OUT_SUM && out_kind != SBAG_OUT_VOTES)
    return fail(SBAG_EINVAL, "unknown output kind");
  CTX_LOCK(c);
  if (out_kind == SBAG_OUT_VOTES && vote_bytes != 8) {
    if (f->impurity != SBAG_IMPURITY_GINI || f->nclasses <= 0)
      return fail(SBAG_EINVAL, "votes need class-valued trees");
    if (vote_bytes != 1 && vote_bytes != 2) return fail(SBAG_EINVAL, "vote_bytes must be 1, 2 or 8");
    if (f->nclasses > (vote_bytes == 1 ? 256 : 4096))
      return fail(SBAG_EINVAL, std::to_string(f->nclasses) + " classes do not fit " +
                                   std::to_string(vote_bytes) + "-byte votes");
  }
  TRY(predict_dataset_dev(c, f, ds, out_kind == SBAG_OUT_SUM ? kAggSum : kAggVotes, vote_bytes,
                          d_out, nullptr));
  HIP_TRY(hipStreamSynchronize(c->stream));  // the caller's stream reads d_out next
  return SBAG_OK;
}

int sbag_aggregate(sbag_ctx* c, const double* votes, int32_t L, int64_t N, int32_t agg, double* out) {
  if (!c || !votes || !out || L <= 0 || N < 0) return fail(SBAG_EINVAL, "bad arguments");
  if (agg != SBAG_AGG_MEAN && agg != SBAG_AGG_MODE) return fail(SBAG_EINVAL, "unknown aggregation");
  if (N == 0) return SBAG_OK;
  CTX_LOCK(c);
  int ncls = 1;
  if (agg == SBAG_AGG_MODE) {
    for (int64_t i = 0; i < (int64_t)L * N; i++) {
      const double v = votes[i];
      if (!(v >= 0 && v == std::floor(v) && v < 4096)) return fail(SBAG_EINVAL, "votes must be class ids");
      ncls = std::max(ncls, (int)v + 1);
    }
  }
  HIP_TRY(hipSetDevice(c->device));
  double *d_v, *d_out;
  TRY(ws_typed(c, "agv", (size_t)L * N, &d_v));
  TRY(ws_typed(c, "agout", (size_t)N, &d_out));
  TRY(h2d(c, d_v, votes, (size_t)L * N));
  uint16_t* d_gcnt = nullptr;
  int64_t gcnt_rows = 0;
  TRY(mode_counters(c, agg, ncls, N, &d_gcnt, &gcnt_rows));
  launch_aggregate(c->stream, d_v, 8, L, N, agg, ncls, (double)L, d_out, d_gcnt, gcnt_rows);
  HIP_TRY(hipGetLastError());
  TRY(d2h(c, out, d_out, (size_t)N));
  return SBAG_OK;
}

int sbag_aggregate_device(sbag_ctx* c, const void* d_in, int32_t in_bytes, int32_t K, int64_t N,
                          int32_t agg, int32_t num_learners, int32_t num_classes, double* d_out) {
  if (!c || !d_in || !d_out || K <= 0 || N < 0 || num_learners <= 0)
    return fail(SBAG_EINVAL, "bad arguments");
  if (in_bytes != 1 && in_bytes != 2 && in_bytes != 8) return fail(SBAG_EINVAL, "in_bytes must be 1, 2 or 8");
  if (agg == SBAG_AGG_MODE) {
    if (num_classes <= 0 || num_classes > 4096) return fail(SBAG_EINVAL, "num_classes out of range");
    if (in_bytes == 8) return fail(SBAG_EINVAL, "device mode aggregation takes u8 / u16 class ids");
    if (in_bytes == 1 && num_classes > 256) return fail(SBAG_EINVAL, "u8 votes hold at most 256 classes");
  } else if (agg == SBAG_AGG_MEAN) {
    if (in_bytes != 8) return fail(SBAG_EINVAL, "mean aggregation takes fp64 values");
  } else {
    return fail(SBAG_EINVAL, "unknown aggregation");
  }
  if (N == 0) return SBAG_OK;
  CTX_LOCK(c);
  HIP_TRY(hipSetDevice(c->device));
  uint16_t* d_gcnt = nullptr;
  int64_t gcnt_rows = 0;
  TRY(mode_counters(c, agg, num_classes, N, &d_gcnt, &gcnt_rows));
  launch_aggregate(c->stream, d_in, in_bytes, K, N, agg, std::max(num_classes, 1), (double)num_learners,
                   d_out, d_gcnt, gcnt_rows);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SBAG_OK;
}

}  // extern "C"

// ====================================================================== booster engine
// GBMRegressor's base-learner fit (ml/regression/GBMRegressor.scala:302-319): the subbag
// of learner m (extractSubBag of withBag's column m, HasSubBag.scala:108-126) sliced to
// the booster's subspace, labels = the pseudo-residuals -grad(y, F(x)) in fp64, through
// DecisionTreeRegressor.fit (HasBaseLearner.fitBaseLearner, ensembleParams.scala:99-117):
// the bagging engine with one learner (fit_range) -- screened fp64 splits and Spark's
// per-partition row-order sums (sbag_f64s.hip) for real-valued residuals, the integer
// engine for dyadic ones.  (Round 3's engine, one lane per (node, feature) walking a node's
// rows with host split selection, was removed in round 6.)

extern "C" {

int sbag_fit_booster(sbag_ctx* c, const sbag_dataset* ds, const double* labels,
                     const sbag_booster_params* bp, sbag_forest** out) {
  if (!c || !ds || !labels || !bp || !out || !bp->counts || !bp->subspace)
    return fail(SBAG_EINVAL, "bad arguments");
  if (ds->ctx->device != c->device)
    return fail(SBAG_EINVAL, "dataset lives on device " + std::to_string(ds->ctx->device) +
                                 ", the context on device " + std::to_string(c->device));
  CTX_LOCK(c);
  const sbag_tree_params& tp = bp->tree;
  if (tp.impurity != SBAG_IMPURITY_VARIANCE)
    return fail(SBAG_EINVAL, "the booster engine fits DecisionTreeRegressor (impurity variance)");
  if (tp.max_depth < 0 || tp.max_depth > 30)
    return fail(SBAG_EINVAL, "maxDepth given invalid value (must be in [0, 30])");
  if (tp.max_bins < 2 || tp.max_bins > 256)
    return fail(SBAG_EINVAL, "maxBins given invalid value (must be in [2, 256])");
  if (tp.min_instances_per_node < 1)
    return fail(SBAG_EINVAL, "minInstancesPerNode given invalid value (must be >= 1)");
  if (!(tp.min_info_gain >= 0.0)) return fail(SBAG_EINVAL, "minInfoGain given invalid value");
  const int64_t N = ds->N;
  const int F = ds->F;
  if (N >= ((int64_t)1 << 32)) return fail(SBAG_EUNSUPPORTED, "booster fit on 2^32 rows or more");
  {
    int maxd = 0;
    for (const auto& d : ds->dict) maxd = std::max(maxd, (int)d.size());
    TRY(check_bins256(tp, N, maxd));
  }
  const int Fr = bp->subspace_len;
  if (Fr <= 0)
    return fail(SBAG_EINVAL, "requirement failed: VectorSlicer requires that at least one "
                             "feature be selected.");
  std::vector<int32_t> sub(bp->subspace, bp->subspace + Fr);
  for (int k = 0; k < Fr; k++)
    if (sub[k] < 0 || sub[k] >= F || (k > 0 && sub[k] <= sub[k - 1]))
      return fail(SBAG_EINVAL, "subspace indices must be increasing and within [0, num_features)");
  // host-side phase timing of the booster set-up (SBAG_PROFILE_HOST=1 prints it)
  const bool bprof = getenv("SBAG_PROFILE_HOST") != nullptr;
  auto bnow = [] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  double bt[6] = {0}, b0 = bnow();
  auto bmark = [&](int k) {
    const double t = bnow();
    bt[k] += t - b0;
    b0 = t;
  };
  // the residuals as a label set: uploaded, then analyzed on the device (analyze_labels'
  // quantities, k_label_stats) -- no host pass over the column
  LabelSet lab;
  HIP_TRY(hipSetDevice(c->device));
  TRY(ws_typed(c, "bt_y64", (size_t)N + 1, &lab.d_y64));
  TRY(h2d(c, lab.d_y64, labels, (size_t)N));
  HIP_TRY(hipMemsetAsync(lab.d_y64 + N, 0, 8, c->stream));
  {
    uint64_t* d_acc;
    TRY(ws_typed(c, "bt_lacc", 6, &d_acc));
    const uint64_t init[6] = {0, 0, 0, ~0ull, 0, 0};
    TRY(h2d(c, d_acc, init, 6));
    launch_label_stats(c->stream, lab.d_y64, N, d_acc);
    HIP_TRY(hipGetLastError());
    uint64_t acc[6];
    TRY(d2h(c, acc, d_acc, 6));
    auto from_key = [](uint64_t k) {
      const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
      double v;
      std::memcpy(&v, &b, 8);
      return v;
    };
    double amax;
    std::memcpy(&amax, &acc[5], 8);
    const bool finite = acc[0] == 0;
    set_label_stats(lab, N, finite, acc[1] == 0, (int)acc[2], finite ? from_key(acc[3]) : 0.0,
                    finite ? from_key(acc[4]) : 0.0, amax);
  }
  if (!lab.finite) return fail(SBAG_EUNSUPPORTED, "booster labels must be finite");
  bmark(0);  // upload + analysis
  std::vector<int64_t> poff;
  TRY(check_partitions(bp->num_partitions, bp->partition_offsets, N, poff));
  HIP_TRY(hipSetDevice(c->device));
  // the bagging engine with one learner (fit_range): the iteration's bag column and
  // subspace, its residuals as labels -- screened fp64 splits and row-order sums
  // (sbag_f64s.hip) for real-valued residuals, the integer engine for dyadic ones
  {
    int64_t n_items = 0;
    for (int64_t r = 0; r < N; r++) n_items += bp->counts[r];
    if (n_items == 0)
      return fail(SBAG_EEMPTY, "DecisionTree requires size of input RDD > 0, but was given by "
                               "empty one.");
  }
  bmark(1);  // items
  TRY(ws_typed(c, "bt_labk", (size_t)N, &lab.d_labk));
  if (lab.label_ok || lab.approx_ok)
    launch_label_image(c->stream, lab.d_y64, N, lab.label_ok ? lab.shift : lab.ashift, lab.label_ok,
                       lab.d_labk);
  else
    HIP_TRY(hipMemsetAsync(lab.d_labk, 0, (size_t)N * 4, c->stream));
  HIP_TRY(hipGetLastError());
  bmark(2);  // fixed-point image
  FitExt ext{bp->counts, sub, &lab};
  sbag_fit_params fp{};
  fp.sampler.replacement = 1;
  fp.sampler.sample_ratio = 1.0;
  fp.sampler.seed = 0;
  fp.sampler.learner_begin = 0;
  fp.sampler.learner_end = 1;
  fp.subspace_ratio = 1.0;
  fp.subspace_bug_compat = 0;
  fp.num_partitions = bp->num_partitions;
  fp.partition_offsets = bp->partition_offsets;
  fp.tree = tp;
  sbag_forest* f = nullptr;
  const int rc = fit_range(c, const_cast<sbag_dataset*>(ds), &fp, &f, &ext);
  if (rc == kSplitRange) return fail(SBAG_EUNSUPPORTED, "the booster's bins exceed the device budget");
  TRY(rc);
  bmark(4);  // fit
  if (bprof)
    fprintf(stderr, "[sbag] booster host ms: upload+analysis %.2f items %.2f image %.2f fit %.2f\n",
            bt[0], bt[1], bt[2], bt[4]);
  *out = f;
  return SBAG_OK;
}

}  // extern "C"
