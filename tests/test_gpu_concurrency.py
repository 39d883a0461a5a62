"""GPU: concurrent calls into libsbag from Python threads, as the reference's cross-validation
drives the estimator (BaggingRegressorSuite.scala:38-43: CrossValidator.setParallelism(4)
fits four models at once, each through SbagNative.fit and .predict).  ctypes releases the GIL
around every foreign call, so the four threads really are inside the library together.

SURVEY §8b asks the ABI to be reentrant: calls on one context are serialized by its lock,
separate contexts run side by side, and sbag_last_error() is per thread.  Every concurrent
result must equal the serial one byte for byte, and an SBAG_EINVAL induced in one thread must
be that thread's error only."""
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import DATA

import spark_bagging_amd as sb
from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu

FIELDS = ("left", "right", "feature", "threshold", "prediction", "impurity", "gain")
JOBS = 4

CASES = [
    # (data, label divisor, partitions, impurity, agg): gini, integer variance, fp64 variance
    ("vehicle.svm", None, [0, 300, 846], nat.IMPURITY_GINI, nat.AGG_MODE),
    ("cpusmall.svm", None, [0, 4000, 8192], nat.IMPURITY_VARIANCE, nat.AGG_MEAN),
    ("cpusmall.svm", 10.0, [0, 2000, 5000, 8192], nat.IMPURITY_VARIANCE, nat.AGG_MEAN),
]


def _data(case):
    name, div, part, imp, agg = CASES[case]
    X, y = sb.load_libsvm(os.path.join(DATA, name))
    X = np.asarray(X, np.float64)
    if div:
        y = y / div
    return X, y, part, imp, agg


def _job(ctx, ds, X, part, imp, agg, j, ratio=0.8):
    """fit learners [4j, 4j + 4) and transform every row; the forest as bytes"""
    f = nat.fit(ctx, ds, replacement=True, sample_ratio=ratio, seed=11, learner_begin=4 * j,
                learner_end=4 * j + 4, subspace_ratio=0.7, partition_offsets=part, max_depth=6,
                max_bins=32, impurity=imp)
    try:
        trees = []
        for t in range(len(f)):
            nodes, stats = f.tree(t)
            trees.append(tuple(np.ascontiguousarray(nodes[k]).tobytes() for k in FIELDS))
            trees.append(np.ascontiguousarray(stats).tobytes())
            trees.append(np.asarray(f.subspace(t)).tobytes())
        pred = nat.predict(ctx, f, X, agg)
        return trees, pred.tobytes()
    finally:
        f.free()


@pytest.mark.parametrize("case", range(len(CASES)))
def test_threads_on_one_shared_context(case):
    X, y, part, imp, agg = _data(case)
    ctx = nat.Context(0)
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    serial = [_job(ctx, ds, X, part, imp, agg, j) for j in range(JOBS)]
    start = threading.Barrier(JOBS)

    def run(j):
        start.wait()
        return _job(ctx, ds, X, part, imp, agg, j)

    for rep in range(2):
        with ThreadPoolExecutor(JOBS) as ex:
            got = list(ex.map(run, range(JOBS)))
        for j in range(JOBS):
            assert got[j][0] == serial[j][0], f"rep {rep} job {j}: forest differs from the serial fit"
            assert got[j][1] == serial[j][1], f"rep {rep} job {j}: transform differs"
    ds.free()
    ctx.close()


@pytest.mark.parametrize("case", range(len(CASES)))
def test_threads_on_separate_contexts(case):
    X, y, part, imp, agg = _data(case)
    ctx0 = nat.Context(0)
    ds0 = nat.DeviceDataset.from_numpy(X, y, ctx0)
    serial = [_job(ctx0, ds0, X, part, imp, agg, j) for j in range(JOBS)]
    ds0.free()
    ctx0.close()
    start = threading.Barrier(JOBS)

    def run(j):
        ctx = nat.Context(0)
        ds = nat.DeviceDataset.from_numpy(X, y, ctx)
        try:
            start.wait()
            return _job(ctx, ds, X, part, imp, agg, j)
        finally:
            ds.free()
            ctx.close()

    with ThreadPoolExecutor(JOBS) as ex:
        got = list(ex.map(run, range(JOBS)))
    for j in range(JOBS):
        assert got[j] == serial[j], f"job {j}: differs from the serial fit"


@pytest.mark.parametrize("shared", [True, False])
def test_thread_local_error_under_concurrency(shared):
    """Thread 0 passes sampleRatio 1.5 while threads 1-3 fit: thread 0 gets
    IllegalArgumentException with its own message (read through sbag_last_error() on its own
    thread), the others succeed with the serial results and an empty sbag_last_error()."""
    X, y, part, imp, agg = _data(2)
    ctx0 = nat.Context(0)
    ds0 = nat.DeviceDataset.from_numpy(X, y, ctx0)
    serial = [_job(ctx0, ds0, X, part, imp, agg, j) for j in range(JOBS)]
    start = threading.Barrier(JOBS)

    def run(j):
        ctx, ds = (ctx0, ds0) if shared else (nat.Context(0), None)
        if ds is None:
            ds = nat.DeviceDataset.from_numpy(X, y, ctx)
        try:
            start.wait()
            try:
                out = _job(ctx, ds, X, part, imp, agg, j, ratio=1.5 if j == 0 else 0.8)
                err = None
            except nat.IllegalArgumentException as e:
                out, err = None, str(e)
            return out, err, nat.lib().sbag_last_error().decode()
        finally:
            if not shared:
                ds.free()
                ctx.close()

    with ThreadPoolExecutor(JOBS) as ex:
        got = list(ex.map(run, range(JOBS)))
    out0, err0, last0 = got[0]
    assert out0 is None and err0 is not None and "sampleRatio" in err0
    assert "sampleRatio" in last0
    for j in range(1, JOBS):
        out, err, last = got[j]
        assert err is None and last == "", f"job {j}: error leaked: {err!r} / {last!r}"
        assert out == serial[j], f"job {j}: differs from the serial fit"
    ds0.free()
    ctx0.close()
