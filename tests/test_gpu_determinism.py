"""GPU: run twice, byte-equal.  The histogram kernels accumulate with atomics in an
order that changes from run to run; the engine is exact because every histogram word
is an integer, so two fits of the same input must agree in every byte
of every node -- and so must two transforms.  Covers the variance row-lane path, the
gini class-tile path with entry grouping (atomic scatter order) and the sampler."""
import numpy as np
import pytest

import oracle

from spark_bagging_amd import _native as nat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = nat.Context(0)
    yield c
    c.close()


def _fit_bytes(ctx, ds, **kw):
    f = nat.fit(ctx, ds, **kw)
    out = []
    for t in range(len(f)):
        nodes, stats = f.tree(t)
        out.append(nodes.tobytes() + stats.tobytes() + f.subspace(t).tobytes())
    pred = nat.predict_dataset(ctx, f, ds, nat.AGG_MODE if kw["impurity"] else nat.AGG_MEAN)
    f.free()
    return out, pred.tobytes()


@pytest.mark.parametrize("cls", [False, True], ids=["variance", "gini-64-classes"])
def test_fit_twice_byte_equal(ctx, cls):
    n, F = 1_000_000, 100
    ds = nat.DeviceDataset.synthetic(n, F, seed=7, num_classes=64 if cls else 0, ctx=ctx)
    part = [int(round(i * n / 64)) for i in range(65)]
    kw = dict(replacement=not cls, sample_ratio=0.5 if cls else 1.0,
              seed=oracle.DEFAULT_SEED_CLASSIFIER if cls else oracle.DEFAULT_SEED_REGRESSOR,
              learner_begin=0, learner_end=8, partition_offsets=part, max_depth=10 if cls else 8,
              max_bins=32, impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
    a, pa = _fit_bytes(ctx, ds, **kw)
    b, pb = _fit_bytes(ctx, ds, **kw)
    assert len(a) == len(b) == 8
    for t in range(8):
        assert a[t] == b[t], f"tree {t} differs between two identical fits"
    assert pa == pb
    ds.free()
