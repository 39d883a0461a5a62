"""GPU: the device outputs and device aggregation behind multi-GPU transform
(spark_bagging_amd.distributed) and breeze mode beyond the LDS counters.

Two learner shards of one ensemble are predicted on the device exactly as two ranks
would (sbag_predict_dataset_device), their outputs stacked as the all-to-all delivers
them (rank order), and aggregated on the device (sbag_aggregate_device):
  * regression: each shard's SBAG_OUT_SUM is its trees' in-order sum, bit for bit;
    the mean is (s_0 + s_1) / L, within 1e-12 of BaggingRegressionModel.predict's
    sequential sum (ml/regression/BaggingRegressor.scala:248-256);
  * classification: u8 / u16 votes equal the per-tree class ids, and the device mode
    equals the single-forest vote (ml/classification/BaggingClassifier.scala:248-257).
World-size-1 RCCL runs distributed.transform end to end.
"""
import os

import numpy as np
import pytest
import torch

import oracle

from spark_bagging_amd import _native as nat
from spark_bagging_amd import synthetic

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def ctx():
    c = nat.Context(0)
    yield c
    c.close()


def _fit(ctx, ds, lb, le, cls, seed):
    return nat.fit(ctx, ds, replacement=True, sample_ratio=0.8, seed=seed, learner_begin=lb,
                   learner_end=le, partition_offsets=[0, 7000, 15000], max_depth=6,
                   impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)


def _seq_sum(per_tree):
    s = np.zeros(per_tree.shape[1])
    for t in range(per_tree.shape[0]):
        s = s + per_tree[t]
    return s


def _mode(votes):
    out = np.zeros(votes.shape[1])
    for r in range(votes.shape[1]):
        cnt, best, maxc = {}, 0.0, 0
        for v in votes[:, r]:
            cnt[v] = cnt.get(v, 0) + 1
            if cnt[v] > maxc:
                maxc, best = cnt[v], float(v)
        out[r] = best
    return out


@pytest.fixture(scope="module", params=[False, True], ids=["regression", "classification"])
def shards(request, ctx):
    cls = request.param
    X, y = synthetic.generate(15000, 12, seed=5, num_classes=7 if cls else 0)
    seed = oracle.DEFAULT_SEED_CLASSIFIER if cls else oracle.DEFAULT_SEED_REGRESSOR
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    fa, fb, full = _fit(ctx, ds, 0, 5, cls, seed), _fit(ctx, ds, 5, 9, cls, seed), \
        _fit(ctx, ds, 0, 9, cls, seed)
    _, per_tree = nat.predict(ctx, full, X, nat.AGG_MEAN, per_tree=True)
    yield cls, X, ds, fa, fb, full, per_tree
    for f in (fa, fb, full):
        f.free()
    ds.free()


def test_partial_sums_two_shards(ctx, shards):
    cls, X, ds, fa, fb, full, per_tree = shards
    if cls:
        pytest.skip("regression path")
    N = X.shape[0]
    parts = torch.zeros((2, N), dtype=torch.float64, device=DEV)
    torch.cuda.synchronize()
    nat.predict_dataset_device(ctx, fa, ds, nat.OUT_SUM, 0, parts[0].data_ptr())
    nat.predict_dataset_device(ctx, fb, ds, nat.OUT_SUM, 0, parts[1].data_ptr())
    p = parts.cpu().numpy()
    np.testing.assert_array_equal(p[0], _seq_sum(per_tree[:5]))
    np.testing.assert_array_equal(p[1], _seq_sum(per_tree[5:]))
    out = torch.empty(N, dtype=torch.float64, device=DEV)
    nat.aggregate_device(ctx, parts.data_ptr(), 8, 2, N, nat.AGG_MEAN, 9, 0, out.data_ptr())
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got, (p[0] + p[1]) / 9)
    np.testing.assert_allclose(got, nat.predict_dataset(ctx, full, ds, nat.AGG_MEAN), rtol=1e-12,
                               atol=0)


@pytest.mark.parametrize("vb", [1, 2])
def test_votes_two_shards(ctx, shards, vb):
    cls, X, ds, fa, fb, full, per_tree = shards
    if not cls:
        pytest.skip("classification path")
    N = X.shape[0]
    dt = torch.uint8 if vb == 1 else torch.int16
    votes = torch.zeros((9, N), dtype=dt, device=DEV)
    torch.cuda.synchronize()
    nat.predict_dataset_device(ctx, fa, ds, nat.OUT_VOTES, vb, votes[:5].data_ptr())
    nat.predict_dataset_device(ctx, fb, ds, nat.OUT_VOTES, vb, votes[5:].data_ptr())
    np.testing.assert_array_equal(votes.cpu().numpy().astype(np.float64), per_tree)
    out = torch.empty(N, dtype=torch.float64, device=DEV)
    nat.aggregate_device(ctx, votes.data_ptr(), vb, 9, N, nat.AGG_MODE, 9, 7, out.data_ptr())
    np.testing.assert_array_equal(out.cpu().numpy(), nat.predict_dataset(ctx, full, ds, nat.AGG_MODE))


def _leaf_forest(classes_per_tree):
    trees = []
    for c in classes_per_tree:
        n = np.zeros(1, nat.NODE_DTYPE)
        n["left"] = n["right"] = n["feature"] = -1
        n["prediction"] = c
        trees.append(n)
    return nat.NativeForest.from_trees(trees, [[0]] * len(trees), nat.IMPURITY_GINI)


def test_mode_first_to_reach_max_ties_h11(ctx):
    """Crafted ties: breeze's mode keeps the class that first reaches the
    final max count -- through the host-row, device-row and aggregate kernels."""
    cases = [([2, 1, 1, 2], 1.0), ([3, 3, 0, 0], 3.0), ([0, 1, 2], 0.0),
             ([4, 2, 2, 4, 4, 2], 4.0), ([1, 2, 2, 1], 2.0), ([5, 0, 0, 5, 5, 0, 0], 0.0)]
    X = np.zeros((3, 1))
    ds = nat.DeviceDataset.from_numpy(X, np.zeros(3), ctx)
    for votes, want in cases:
        f = _leaf_forest(votes)
        assert (nat.predict(ctx, f, X, nat.AGG_MODE) == want).all()
        assert (nat.predict_dataset(ctx, f, ds, nat.AGG_MODE) == want).all()
        v = np.array(votes, np.float64)[:, None].repeat(3, axis=1)
        assert (nat.aggregate(ctx, v, nat.AGG_MODE) == want).all()
        dv = torch.tensor(np.array(votes, np.uint8)[:, None].repeat(3, axis=1), device=DEV)
        out = torch.empty(3, dtype=torch.float64, device=DEV)
        torch.cuda.synchronize()
        nat.aggregate_device(ctx, dv.data_ptr(), 1, len(votes), 3, nat.AGG_MODE, len(votes), 6,
                             out.data_ptr())
        assert (out.cpu().numpy() == want).all()
        f.free()
    ds.free()


def test_mode_beyond_lds_counters_400_classes(ctx):
    """More classes than the LDS counters hold (kLdsModeClasses = 320): the counters move
    to global memory.  Depth-1 trees on one feature, 400 classes."""
    rng = np.random.default_rng(3)
    L, N = 25, 3000
    X = rng.integers(0, 4, size=(N, 1)).astype(np.float64)
    trees = []
    for t in range(L):
        n = np.zeros(3, nat.NODE_DTYPE)
        n["id"] = np.arange(3)
        n["left"] = n["right"] = n["feature"] = -1
        n[0]["left"], n[0]["right"], n[0]["feature"], n[0]["threshold"] = 1, 2, 0, 1.5
        n[1]["prediction"], n[2]["prediction"] = rng.integers(0, 400, size=2)
        trees.append(n)
    trees[0][1]["prediction"] = 399.0
    f = nat.NativeForest.from_trees(trees, [[0]] * L, nat.IMPURITY_GINI)
    per_tree = np.stack([np.where(X[:, 0] <= 1.5, t[1]["prediction"], t[2]["prediction"])
                         for t in trees])
    want = _mode(per_tree)
    np.testing.assert_array_equal(nat.predict(ctx, f, X, nat.AGG_MODE), want)
    ds = nat.DeviceDataset.from_numpy(X, np.zeros(N), ctx)
    np.testing.assert_array_equal(nat.predict_dataset(ctx, f, ds, nat.AGG_MODE), want)
    np.testing.assert_array_equal(nat.aggregate(ctx, per_tree, nat.AGG_MODE), want)
    votes = torch.zeros((L, N), dtype=torch.int16, device=DEV)
    torch.cuda.synchronize()
    nat.predict_dataset_device(ctx, f, ds, nat.OUT_VOTES, 2, votes.data_ptr())
    np.testing.assert_array_equal(votes.cpu().numpy(), per_tree)
    out = torch.empty(N, dtype=torch.float64, device=DEV)
    nat.aggregate_device(ctx, votes.data_ptr(), 2, L, N, nat.AGG_MODE, L, 400, out.data_ptr())
    np.testing.assert_array_equal(out.cpu().numpy(), want)
    with pytest.raises(nat.IllegalArgumentException):  # 400 classes do not fit u8 votes
        nat.predict_dataset_device(ctx, f, ds, nat.OUT_VOTES, 1, votes.data_ptr())
    f.free()
    ds.free()


@pytest.mark.parametrize("cls", [False, True])
def test_distributed_transform_world_one_rccl(cls):
    """distributed.transform end to end over a world-size-1 RCCL group (the 8-GPU run
    is the driver's; the collectives' N > 1 logic is covered on gloo in test_dist.py)."""
    import socket

    import torch.distributed as dist

    from spark_bagging_amd import distributed as D
    from spark_bagging_amd.ml import (BaggingClassifier, BaggingRegressor,
                                      DecisionTreeClassifier, DecisionTreeRegressor, Frame)

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=DEV)
    try:
        X, y = synthetic.generate(6000, 9, seed=2, num_classes=4 if cls else 0)
        est = (BaggingClassifier().setBaseLearner(DecisionTreeClassifier()) if cls else
               BaggingRegressor().setBaseLearner(DecisionTreeRegressor()))
        est.setNumBaseLearners(6).setReplacement(True).setSampleRatio(0.9)
        shard = D.fit_shard(est, Frame(X, y), dist)
        got = D.transform(shard, X, dist)
        want = shard.transform(X)
        if cls:
            np.testing.assert_array_equal(got, want)
        else:
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)
    finally:
        dist.destroy_process_group()
