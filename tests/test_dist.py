"""CPU, world_size 2 and 3 over gloo: the learner-sharded path (spark_bagging_amd.distributed).

Each rank trains its learner block; the per-rank compute here is the oracle (the HIP
path needs a GPU), so this test checks what is specific to N > 1: learner ranges,
all-gathering trees in learner order, and the aggregation collectives -- the
all-to-all by row shard of per-rank partial sums (regression) or u8 votes
(classification), the ordered reduction on each row shard, the all-gather of the
predictions -- against the single-process ensemble: votes bit for bit, means as
the shard-blocked in-order sum / L (and within 1e-12 of the sequential sum).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mode_rows(votes):
    """breeze mode per column of [L x n] class ids: first class to reach the max count."""
    L, n = votes.shape
    out = np.zeros(n)
    for r in range(n):
        cnt, best, maxc = {}, 0.0, 0
        for v in votes[:, r]:
            cnt[v] = cnt.get(v, 0) + 1
            if cnt[v] > maxc:
                maxc, best = cnt[v], float(v)
        out[r] = best
    return out


L, N, F, PART = 7, 900, 10, [0, 400, 900]


def _data(cls):
    from spark_bagging_amd import synthetic

    X, y = synthetic.generate(N, F, seed=8, num_classes=4 if cls else 0)
    return X, y, (42087812 if cls else -1395689524)


def _shard_forest(lb, le, cls):
    X, y, seed = _data(cls)
    counts = oracle.bag(True, 0.8, lb, le, seed, PART, N)
    subs = [oracle.subspace(0.8, F, seed + i) for i in range(lb, le)]
    return X, subs, oracle.fit(X, y, counts, subs, max_depth=4, classification=cls)


def _worker(rank, world, port, cls, q):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist

    import sbag_loader

    sbag_loader.load()
    from spark_bagging_amd import distributed as D
    from spark_bagging_amd.ml import (BaggingClassificationModel, BaggingRegressionModel,
                                      DecisionTreeModel)

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        lb, le = D.learner_range(L, rank, world)
        X, subs, f = _shard_forest(lb, le, cls)
        mcls = BaggingClassificationModel if cls else BaggingRegressionModel
        shard = mcls(subs, [DecisionTreeModel(f.tree(t)[0], f.tree(t)[1], int(cls))
                            for t in range(le - lb)])
        full = D.gather_model(shard, dist)
        _, per_tree = oracle.predict(f, X, classification=cls, per_tree=True)
        if cls:
            local = torch.from_numpy(per_tree.astype(np.uint8))  # [L_rank x N] u8 votes

            def reduce_fn(rows):
                assert rows.shape[0] == L and rows.dtype == torch.uint8
                return torch.from_numpy(_mode_rows(rows.numpy()))
        else:
            s = np.zeros(N)
            for t in range(per_tree.shape[0]):
                s = s + per_tree[t]
            local = torch.from_numpy(s[None, :])  # [1 x N] in-order partial sum

            def reduce_fn(rows):
                assert rows.shape[0] == world
                acc = rows[0].clone()
                for g in range(1, world):
                    acc = acc + rows[g]
                return acc / L
        pred = D.sharded_aggregate(local, N, dist, reduce_fn).numpy()
        q.put((rank, pred, [m.nodes for m in full.models], [np.asarray(s) for s in full.subspaces]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cls,world", [(False, 2), (True, 2), (True, 3), (False, 3)])
def test_sharded_ensemble_matches_single_process(cls, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cls, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            r, pred, nodes, subs = q.get(timeout=180)
            got[r] = (pred, nodes, subs)
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    X, y, seed = _data(cls)
    _, s_subs, f = _shard_forest(0, L, cls)
    want, per_tree = oracle.predict(f, X, classification=cls, per_tree=True)
    from spark_bagging_amd.distributed import learner_range

    for r in range(world):
        pred, nodes, subs = got[r]
        if cls:
            assert (pred == want).all()  # every rank holds all N predictions
        else:
            blocked = np.zeros(N)
            for g in range(world):
                lb, le = learner_range(L, g, world)
                s = np.zeros(N)
                for t in range(lb, le):
                    s = s + per_tree[t]
                blocked = blocked + s
            assert (pred == blocked / L).all()
            np.testing.assert_allclose(pred, want, rtol=1e-12, atol=0)
        for l in range(L):
            assert (nodes[l] == f.tree(l)[0]).all()
            assert list(subs[l]) == list(s_subs[l])


def test_learner_ranges_partition_in_order():
    import sbag_loader

    sbag_loader.load()
    from spark_bagging_amd.distributed import learner_range

    for L in (1, 5, 128, 512):
        for world in (1, 2, 3, 8):
            rs = [learner_range(L, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == L
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def _votes16_worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import sbag_loader

    sbag_loader.load()
    from spark_bagging_amd import distributed as D

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        lb, le = D.learner_range(11, rank, world)
        # votes of learners lb..le-1 for 777 rows, class ids up to 400 (> 256: u16)
        l = torch.arange(lb, le, dtype=torch.int32)[:, None]
        r = torch.arange(777, dtype=torch.int32)[None, :]
        local = ((l * 131 + r * 7) % 401).to(torch.int16)
        out = D.exchange_rows(local, dist)
        q.put((rank, out.dtype, out.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_rows_u16_votes_as_bytes(world):
    """Above 256 classes the votes are int16, which torch's NCCL binding cannot move; they
    cross as bytes. Every rank gets all 11 learners' votes of its row shard,
    in learner order, as int16."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_votes16_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            r, dt, arr = q.get(timeout=180)
            got[r] = (dt, arr)
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    import torch

    from spark_bagging_amd.distributed import row_range
    full = ((np.arange(11)[:, None] * 131 + np.arange(777)[None, :] * 7) % 401).astype(np.int16)
    for r in range(world):
        a, b = row_range(777, r, world)
        dt, arr = got[r]
        assert dt == torch.int16
        assert (arr == full[:, a:b]).all()
