"""ctypes bindings to libsbag.so (include/sbag.h).

The product path: every compute call goes through the HIP library.  There is
no CPU fallback; if the library is missing or fails to load, importing the
compute entry points raises.
"""
import ctypes
import weakref
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsbag.so")

SBAG_OK, SBAG_EINVAL, SBAG_EEMPTY, SBAG_EDEVICE, SBAG_ENOMEM, SBAG_EUNSUPPORTED = range(6)
IMPURITY_VARIANCE, IMPURITY_GINI = 0, 1
AGG_MEAN, AGG_MODE = 0, 1
OUT_SUM, OUT_VOTES = 2, 3  # device outputs of sbag_predict_dataset_device
COL_F64, COL_F32, COL_U8 = 0, 1, 2  # sbag_dataset_create_columns

# every symbol include/sbag.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "sbag_device_count", "sbag_ctx_create", "sbag_ctx_destroy", "sbag_last_error", "sbag_version",
    "sbag_sample", "sbag_subspace", "sbag_dataset_create", "sbag_dataset_create_csr",
    "sbag_dataset_create_columns", "sbag_dataset_synthetic",
    "sbag_dataset_info", "sbag_dataset_labels", "sbag_dataset_features", "sbag_dataset_free",
    "sbag_dataset_set_labels", "sbag_dataset_layout", "sbag_dataset_export", "sbag_dataset_import",
    "sbag_fit", "sbag_fit_booster", "sbag_forest_num_trees", "sbag_forest_tree_info", "sbag_forest_subspace",
    "sbag_forest_nodes", "sbag_forest_create", "sbag_forest_free", "sbag_forest_timing",
    "sbag_predict", "sbag_predict_dataset", "sbag_aggregate", "sbag_predict_dataset_device",
    "sbag_aggregate_device",
]


class SbagError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[sbag error {code}] {msg}")
        self.code = code


class IllegalArgumentException(SbagError, ValueError):
    """SBAG_EINVAL: the reference raises IllegalArgumentException (require / ParamValidators)."""


class SparkException(SbagError):
    """SBAG_EEMPTY and device failures: the reference raises SparkException."""


class SamplerParams(ctypes.Structure):
    _fields_ = [("replacement", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("sample_ratio", ctypes.c_double), ("seed", ctypes.c_int64),
                ("learner_begin", ctypes.c_int32), ("learner_end", ctypes.c_int32)]


class TreeParams(ctypes.Structure):
    _fields_ = [("max_depth", ctypes.c_int32), ("max_bins", ctypes.c_int32),
                ("min_instances_per_node", ctypes.c_int32), ("impurity", ctypes.c_int32),
                ("min_info_gain", ctypes.c_double), ("seed", ctypes.c_int64)]


# base learners' HasSeed defaults (class-name hashCode): seed of RandomForest.findSplits'
# split-finding sample
DT_SEED_REGRESSOR = 926680331     # "org.apache.spark.ml.regression.DecisionTreeRegressor"
DT_SEED_CLASSIFIER = 159147643    # "org.apache.spark.ml.classification.DecisionTreeClassifier"


class FitParams(ctypes.Structure):
    _fields_ = [("sampler", SamplerParams), ("subspace_ratio", ctypes.c_double),
                ("subspace_bug_compat", ctypes.c_int32), ("num_partitions", ctypes.c_int32),
                ("partition_offsets", ctypes.c_void_p), ("tree", TreeParams)]


class BoosterParams(ctypes.Structure):
    _fields_ = [("counts", ctypes.c_void_p), ("subspace", ctypes.c_void_p),
                ("subspace_len", ctypes.c_int32), ("num_partitions", ctypes.c_int32),
                ("partition_offsets", ctypes.c_void_p), ("tree", TreeParams)]


class Timing(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in
                ("total_ms", "sample_ms", "valuecount_ms", "bin_ms", "compact_ms", "hist_ms",
                 "split_ms", "subtract_ms")] + [
        ("hist_launches", ctypes.c_int64), ("hist_alg_bytes", ctypes.c_double),
        ("hist_entries", ctypes.c_double), ("hist_upper_bytes", ctypes.c_double),
        ("levels", ctypes.c_int64), ("partition_ms", ctypes.c_double),
        ("hist_work_bytes", ctypes.c_double), ("fix_ms", ctypes.c_double),
        ("exact_fallbacks", ctypes.c_int64), ("hist_lds_atomics", ctypes.c_double),
        ("group_ms", ctypes.c_double), ("chain_ms", ctypes.c_double),
        ("root_ms", ctypes.c_double), ("root_mfma_ops", ctypes.c_double)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


NODE_DTYPE = np.dtype([("id", "<i4"), ("left", "<i4"), ("right", "<i4"), ("feature", "<i4"),
                       ("split_bin", "<i4"), ("pad", "<i4"), ("threshold", "<f8"),
                       ("prediction", "<f8"), ("impurity", "<f8"), ("gain", "<f8")])

_lib = None


def lib():
    """Load libsbag.so; raises if it is missing (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libsbag.so not built at {LIB_PATH}: run __graft_entry__.build()")
        try:
            # PyTorch-ROCm ships its own HIP runtime under the same soname
            # (libamdhip64.so.7).  Loaded first, it is the one libsbag binds to; loaded
            # after libsbag, torch would bring a second HIP/HSA runtime into the process
            # and device pointers of one (torch tensors handed to the multi-GPU
            # aggregation) would be foreign to the other.
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        P, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        sig = {
            "sbag_device_count": [P],
            "sbag_ctx_create": [i32, P],
            "sbag_ctx_destroy": [P],
            "sbag_sample": [P, ctypes.POINTER(SamplerParams), P, i32, i64, P],
            "sbag_subspace": [dbl, i32, i64, P, P],
            "sbag_dataset_create": [P, i64, i32, P, P, P],
            "sbag_dataset_synthetic": [P, i64, i32, ctypes.c_uint64, i32, P],
            "sbag_dataset_create_csr": [P, i64, i32, P, P, P, P, P],
            "sbag_dataset_create_columns": [P, i64, i32, i32, P, P, P],
            "sbag_dataset_info": [P, P, P],
            "sbag_dataset_labels": [P, P],
            "sbag_dataset_features": [P, i64, i64, P],
            "sbag_dataset_free": [P],
            "sbag_dataset_set_labels": [P, P],
            "sbag_dataset_layout": [P, P, P, P, P, P],
            "sbag_dataset_export": [P, P, i32, P, P, P],
            "sbag_dataset_import": [P, i64, i32, i32, i32, P, i32, P, P, P, P],
            "sbag_fit": [P, P, ctypes.POINTER(FitParams), P],
            "sbag_fit_booster": [P, P, P, ctypes.POINTER(BoosterParams), P],
            "sbag_forest_num_trees": [P, P],
            "sbag_forest_tree_info": [P, i32, P, P, P, P],
            "sbag_forest_subspace": [P, i32, P],
            "sbag_forest_nodes": [P, i32, P, P],
            "sbag_forest_create": [i32, P, P, P, P, i32, P],
            "sbag_forest_free": [P],
            "sbag_forest_timing": [P, ctypes.POINTER(Timing)],
            "sbag_predict": [P, P, P, i64, i32, i32, P, P],
            "sbag_predict_dataset": [P, P, P, i32, P],
            "sbag_aggregate": [P, P, i32, i64, i32, P],
            "sbag_predict_dataset_device": [P, P, P, i32, i32, P],
            "sbag_aggregate_device": [P, P, i32, i32, i64, i32, i32, i32, P],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        L.sbag_last_error.restype = ctypes.c_char_p
        L.sbag_last_error.argtypes = []
        L.sbag_version.restype = ctypes.c_char_p
        L.sbag_version.argtypes = []
        _lib = L
    return _lib


def check(rc):
    if rc == SBAG_OK:
        return
    msg = lib().sbag_last_error().decode(errors="replace")
    if rc == SBAG_EINVAL:
        raise IllegalArgumentException(rc, msg)
    raise SparkException(rc, msg)


def ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Context:
    """One device context (sbag_ctx).  The library serializes calls on a context (sbag.h)."""

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        check(lib().sbag_ctx_create(device, ctypes.byref(self._h)))
        self.device = device
        self._datasets = weakref.WeakSet()  # freed before the context (sbag.h ownership)

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            for ds in list(self._datasets):
                ds.free()
            lib().sbag_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}


def default_context(device=0):
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


def device_count():
    n = ctypes.c_int32()
    check(lib().sbag_device_count(ctypes.byref(n)))
    return n.value


class DeviceDataset:
    """Label + features columns resident in HBM (sbag_dataset)."""

    def __init__(self, ctx, handle):
        self.ctx, self._h = ctx, handle
        ctx._datasets.add(self)

    @classmethod
    def from_numpy(cls, X, y, ctx=None):
        ctx = ctx or default_context()
        X = np.ascontiguousarray(X, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        h = ctypes.c_void_p()
        check(lib().sbag_dataset_create(ctx.handle, X.shape[0], X.shape[1], ptr(X), ptr(y),
                                        ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_csr(cls, rows, y, ctx=None):
        """SparseVector rows (libsvm.SparseRows or a scipy.sparse CSR matrix): absent
        entries are 0.0; no dense copy is made (sbag_dataset_create_csr)."""
        ctx = ctx or default_context()
        n, f = rows.shape
        indptr = np.ascontiguousarray(rows.indptr, np.int64)
        indices = np.ascontiguousarray(rows.indices, np.int32)
        values = np.ascontiguousarray(rows.data, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        if len(indptr) != n + 1 or len(y) != n:
            raise IllegalArgumentException(SBAG_EINVAL, "indptr / labels do not match the row count")
        h = ctypes.c_void_p()
        check(lib().sbag_dataset_create_csr(ctx.handle, n, f, ptr(indptr), ptr(indices), ptr(values),
                                            ptr(y), ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_columns(cls, columns, y, ctx=None):
        """Columnar features: a list of F arrays of N values (fp64, fp32 or u8, one dtype),
        e.g. Arrow / Parquet column chunks (sbag_dataset_create_columns)."""
        ctx = ctx or default_context()
        kinds = {np.dtype(np.float64): COL_F64, np.dtype(np.float32): COL_F32,
                 np.dtype(np.uint8): COL_U8}
        cols = [np.ascontiguousarray(c) for c in columns]
        dts = {c.dtype for c in cols}
        if len(dts) != 1 or next(iter(dts)) not in kinds:
            raise IllegalArgumentException(SBAG_EINVAL, "columns must share one of fp64 / fp32 / u8")
        y = np.ascontiguousarray(y, np.float64)
        if any(len(c) != len(y) for c in cols):
            raise IllegalArgumentException(SBAG_EINVAL, "columns and labels differ in length")
        arr = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        h = ctypes.c_void_p()
        check(lib().sbag_dataset_create_columns(ctx.handle, len(y), len(cols), kinds[cols[0].dtype],
                                                arr, ptr(y), ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def synthetic(cls, num_rows, num_features, seed=20261015, num_classes=0, ctx=None):
        ctx = ctx or default_context()
        h = ctypes.c_void_p()
        check(lib().sbag_dataset_synthetic(ctx.handle, num_rows, num_features, seed, num_classes,
                                           ctypes.byref(h)))
        return cls(ctx, h)

    @property
    def handle(self):
        return self._h

    @property
    def shape(self):
        n, f = ctypes.c_int64(), ctypes.c_int32()
        check(lib().sbag_dataset_info(self._h, ctypes.byref(n), ctypes.byref(f)))
        return n.value, f.value

    def labels(self):
        y = np.zeros(self.shape[0], np.float64)
        check(lib().sbag_dataset_labels(self._h, ptr(y)))
        return y

    def set_labels(self, y):
        """Replace the label column (sbag_dataset_set_labels); non-dyadic regression labels
        are then fitted with Spark's row-order fp64 sums."""
        y = np.ascontiguousarray(y, np.float64)
        if y.shape != (self.shape[0],):
            raise IllegalArgumentException(SBAG_EINVAL, "labels do not match the row count")
        check(lib().sbag_dataset_set_labels(self._h, ptr(y)))

    def layout(self):
        """(num_rows, num_features, row_stride, code_bytes, dict_values) of the codes."""
        n, f, s, cb, dv = (ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(),
                           ctypes.c_int64())
        check(lib().sbag_dataset_layout(self._h, ctypes.byref(n), ctypes.byref(f), ctypes.byref(s),
                                        ctypes.byref(cb), ctypes.byref(dv)))
        return n.value, f.value, s.value, cb.value, dv.value

    def codes_nbytes(self):
        n, _, s, cb, _ = self.layout()
        return n * s * cb

    def export(self, codes_ptr=None, codes_on_device=False):
        """Export for replication: the codes into `codes_ptr` (device memory of this
        dataset's device when codes_on_device, else host memory of codes_nbytes() bytes;
        None: skipped), and (dict, dict_off, labels) as numpy arrays."""
        n, f, _, _, dv = self.layout()
        d = np.zeros(max(dv, 1), np.float64)
        off = np.zeros(f + 1, np.int64)
        y = np.zeros(n, np.float64)
        check(lib().sbag_dataset_export(self._h, ctypes.c_void_p(codes_ptr) if codes_ptr else None,
                                        1 if codes_on_device else 0, ptr(d), ptr(off), ptr(y)))
        return d[:dv], off, y

    @classmethod
    def import_codes(cls, ctx, layout, codes_ptr, codes_on_device, dict_values, dict_off, y):
        """A dataset from exported pieces (sbag_dataset_import): `layout` as layout()
        returns it, the codes at codes_ptr (device memory of ctx's device or host)."""
        n, f, s, cb, _ = layout
        d = np.ascontiguousarray(dict_values, np.float64)
        off = np.ascontiguousarray(dict_off, np.int64)
        y = np.ascontiguousarray(y, np.float64)
        h = ctypes.c_void_p()
        check(lib().sbag_dataset_import(ctx.handle, n, f, s, cb, ctypes.c_void_p(codes_ptr),
                                        1 if codes_on_device else 0, ptr(d), ptr(off), ptr(y),
                                        ctypes.byref(h)))
        return cls(ctx, h)

    def features(self, row_begin=0, row_end=None):
        n, f = self.shape
        row_end = n if row_end is None else row_end
        X = np.zeros((row_end - row_begin, f), np.float64)
        check(lib().sbag_dataset_features(self._h, row_begin, row_end, ptr(X)))
        return X

    def free(self):
        if self._h:
            lib().sbag_dataset_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class NativeForest:
    """Fitted trees (sbag_forest): pre-order NodeData arrays + subspaces."""

    def __init__(self, handle, impurity):
        self._h, self.impurity = handle, impurity

    @property
    def handle(self):
        return self._h

    def __len__(self):
        n = ctypes.c_int32()
        check(lib().sbag_forest_num_trees(self._h, ctypes.byref(n)))
        return n.value

    def tree(self, t):
        nn, ns, sl, ex = (ctypes.c_int32() for _ in range(4))
        check(lib().sbag_forest_tree_info(self._h, t, ctypes.byref(nn), ctypes.byref(ns),
                                          ctypes.byref(sl), ctypes.byref(ex)))
        nodes = np.zeros(nn.value, NODE_DTYPE)
        stats = np.zeros((nn.value, max(ns.value, 1)), np.float64)
        check(lib().sbag_forest_nodes(self._h, t, ptr(nodes), ptr(stats)))
        return nodes, stats[:, : ns.value]

    def subspace(self, t):
        nn, ns, sl, ex = (ctypes.c_int32() for _ in range(4))
        check(lib().sbag_forest_tree_info(self._h, t, ctypes.byref(nn), ctypes.byref(ns),
                                          ctypes.byref(sl), ctypes.byref(ex)))
        idx = np.zeros(max(sl.value, 1), np.int32)
        check(lib().sbag_forest_subspace(self._h, t, ptr(idx)))
        return idx[: sl.value]

    def exact(self, t):
        nn, ns, sl, ex = (ctypes.c_int32() for _ in range(4))
        check(lib().sbag_forest_tree_info(self._h, t, ctypes.byref(nn), ctypes.byref(ns),
                                          ctypes.byref(sl), ctypes.byref(ex)))
        return bool(ex.value)

    def timing(self):
        t = Timing()
        check(lib().sbag_forest_timing(self._h, ctypes.byref(t)))
        return t.as_dict()

    @classmethod
    def from_trees(cls, trees, subspaces, impurity):
        nn = np.array([len(n) for n in trees], np.int32)
        nodes = np.ascontiguousarray(np.concatenate(trees).astype(NODE_DTYPE))
        sl = np.array([len(s) for s in subspaces], np.int32)
        subs = np.ascontiguousarray(np.concatenate([np.asarray(s, np.int32) for s in subspaces]))
        h = ctypes.c_void_p()
        check(lib().sbag_forest_create(len(trees), ptr(nn), ptr(nodes), ptr(sl), ptr(subs),
                                       impurity, ctypes.byref(h)))
        return cls(h, impurity)

    def free(self):
        if self._h:
            lib().sbag_forest_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def sample(ctx, replacement, ratio, seed, learner_begin, learner_end, num_rows,
           partition_offsets=None):
    p = SamplerParams(int(replacement), 0, float(ratio), int(seed), learner_begin, learner_end)
    off = None
    P = 1
    if partition_offsets is not None:
        off = np.ascontiguousarray(partition_offsets, np.int64)
        P = len(off) - 1
    out = np.zeros((learner_end - learner_begin, num_rows), np.uint8)
    check(lib().sbag_sample(ctx.handle, ctypes.byref(p), ptr(off), P, num_rows, ptr(out)))
    return out


def subspace(ratio, num_features, seed):
    idx = np.zeros(max(num_features, 1), np.int32)
    n = ctypes.c_int32()
    check(lib().sbag_subspace(float(ratio), num_features, int(seed), ptr(idx), ctypes.byref(n)))
    return idx[: n.value].copy()


def fit(ctx, dataset, *, replacement, sample_ratio, seed, learner_begin, learner_end,
        subspace_ratio=1.0, subspace_bug_compat=True, partition_offsets=None, max_depth=5,
        max_bins=32, min_instances_per_node=1, min_info_gain=0.0, impurity=IMPURITY_VARIANCE,
        tree_seed=None):
    if tree_seed is None:
        tree_seed = DT_SEED_CLASSIFIER if impurity == IMPURITY_GINI else DT_SEED_REGRESSOR
    off = None
    P = 1
    if partition_offsets is not None:
        off = np.ascontiguousarray(partition_offsets, np.int64)
        P = len(off) - 1
    fp = FitParams(SamplerParams(int(replacement), 0, float(sample_ratio), int(seed),
                                 learner_begin, learner_end),
                   float(subspace_ratio), int(subspace_bug_compat), P,
                   off.ctypes.data if off is not None else None,
                   TreeParams(max_depth, max_bins, min_instances_per_node, impurity,
                              float(min_info_gain), int(tree_seed)))
    h = ctypes.c_void_p()
    check(lib().sbag_fit(ctx.handle, dataset.handle, ctypes.byref(fp), ctypes.byref(h)))
    return NativeForest(h, impurity)


def fit_booster(ctx, dataset, labels, counts, subspace, *, partition_offsets=None, max_depth=5,
                max_bins=32, min_instances_per_node=1, min_info_gain=0.0, tree_seed=None):
    """One GBM base-learner fit (sbag_fit_booster): DecisionTreeRegressor on the subbag
    `counts` (u8 per row) sliced to `subspace`, with fp64 labels (pseudo-residuals)."""
    if tree_seed is None:
        tree_seed = DT_SEED_REGRESSOR
    labels = np.ascontiguousarray(labels, np.float64)
    counts = np.ascontiguousarray(counts, np.uint8)
    sub = np.ascontiguousarray(subspace, np.int32)
    n = dataset.shape[0]
    if len(labels) != n or len(counts) != n:
        raise IllegalArgumentException(SBAG_EINVAL, "labels / counts do not match the row count")
    off = None
    P = 1
    if partition_offsets is not None:
        off = np.ascontiguousarray(partition_offsets, np.int64)
        P = len(off) - 1
    bp = BoosterParams(counts.ctypes.data, sub.ctypes.data, len(sub), P,
                       off.ctypes.data if off is not None else None,
                       TreeParams(max_depth, max_bins, min_instances_per_node, IMPURITY_VARIANCE,
                                  float(min_info_gain), int(tree_seed)))
    h = ctypes.c_void_p()
    check(lib().sbag_fit_booster(ctx.handle, dataset.handle, ptr(labels), ctypes.byref(bp),
                                 ctypes.byref(h)))
    return NativeForest(h, IMPURITY_VARIANCE)


def predict(ctx, forest, X, agg, per_tree=False):
    X = np.ascontiguousarray(X, np.float64)
    out = np.zeros(X.shape[0], np.float64)
    pt = np.zeros((len(forest), X.shape[0]), np.float64) if per_tree else None
    check(lib().sbag_predict(ctx.handle, forest.handle, ptr(X), X.shape[0], X.shape[1], agg,
                             ptr(out), ptr(pt)))
    return (out, pt) if per_tree else out


def predict_dataset(ctx, forest, dataset, agg):
    out = np.zeros(dataset.shape[0], np.float64)
    check(lib().sbag_predict_dataset(ctx.handle, forest.handle, dataset.handle, agg, ptr(out)))
    return out


def aggregate(ctx, votes, agg):
    votes = np.ascontiguousarray(votes, np.float64)
    out = np.zeros(votes.shape[1], np.float64)
    check(lib().sbag_aggregate(ctx.handle, ptr(votes), votes.shape[0], votes.shape[1], agg,
                               ptr(out)))
    return out


def predict_dataset_device(ctx, forest, dataset, out_kind, vote_bytes, d_out):
    """Device outputs for the multi-GPU aggregation (distributed.transform): d_out is a
    device pointer on the context's device (OUT_SUM: fp64 [N]; OUT_VOTES: [trees x N]
    u8 / u16 class ids)."""
    check(lib().sbag_predict_dataset_device(ctx.handle, forest.handle, dataset.handle, out_kind,
                                            vote_bytes, ctypes.c_void_p(d_out)))


def aggregate_device(ctx, d_in, in_bytes, K, N, agg, num_learners, num_classes, d_out):
    """Ordered mean of K fp64 partial-sum rows / num_learners, or breeze mode of K u8 /
    u16 vote rows; device pointers in and out (fp64 [N])."""
    check(lib().sbag_aggregate_device(ctx.handle, ctypes.c_void_p(d_in), in_bytes, K, N, agg,
                                      num_learners, num_classes, ctypes.c_void_p(d_out)))
