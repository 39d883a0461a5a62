"""CPU, world_size 2 over gloo: the learner-sharded path (spark_bagging_amd.distributed).

Each rank trains its learner block; the per-rank compute here is the oracle (the
HIP path needs a GPU), so this test checks what is specific to N > 1: learner
ranges, all-gathering trees and per-tree predictions in learner order, and that
the ordered aggregation equals the single-process ensemble bit for bit.
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


def _mode(votes):
    out = np.zeros(votes.shape[1])
    for r in range(votes.shape[1]):
        cnt, best, maxc = {}, 0.0, 0
        for v in votes[:, r]:
            cnt[v] = cnt.get(v, 0) + 1
            if cnt[v] > maxc:
                maxc, best = cnt[v], v
        out[r] = best
    return out


def _mean(votes):
    s = np.zeros(votes.shape[1])
    for l in range(votes.shape[0]):
        s = s + votes[l]
    return s / votes.shape[0]


def _worker(rank, world, port, cls, q):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist

    import sbag_loader

    sbag_loader.load()
    from spark_bagging_amd import distributed as D
    from spark_bagging_amd import synthetic
    from spark_bagging_amd.ml import (BaggingClassificationModel, BaggingRegressionModel,
                                      DecisionTreeModel)

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        L, N, F = 7, 900, 10
        X, y = synthetic.generate(N, F, seed=8, num_classes=4 if cls else 0)
        seed = 42087812 if cls else -1395689524
        lb, le = D.learner_range(L, rank, world)
        part = [0, 400, 900]
        counts = oracle.bag(True, 0.8, lb, le, seed, part, N)
        subs = [oracle.subspace(0.8, F, seed + i) for i in range(lb, le)]
        f = oracle.fit(X, y, counts, subs, max_depth=4, classification=cls)
        mcls = BaggingClassificationModel if cls else BaggingRegressionModel
        shard = mcls(subs, [DecisionTreeModel(f.tree(t)[0], f.tree(t)[1], int(cls))
                            for t in range(le - lb)])
        full = D.gather_model(shard, dist)
        _, per_tree = oracle.predict(f, X, classification=cls, per_tree=True)
        votes = D.gather_votes(per_tree, dist)
        pred = (_mode if cls else _mean)(votes)
        if rank == 0:
            q.put((pred, [m.nodes for m in full.models], [np.asarray(s) for s in full.subspaces]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cls", [False, True])
def test_two_rank_sharded_ensemble_matches_single_process(cls):
    from spark_bagging_amd import synthetic

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cls, q)) for r in range(2)]
    for p in procs:
        p.start()
    pred, nodes, subs = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    L, N, F = 7, 900, 10
    X, y = synthetic.generate(N, F, seed=8, num_classes=4 if cls else 0)
    seed = 42087812 if cls else -1395689524
    counts = oracle.bag(True, 0.8, 0, L, seed, [0, 400, 900], N)
    s_subs = [oracle.subspace(0.8, F, seed + i) for i in range(L)]
    f = oracle.fit(X, y, counts, s_subs, max_depth=4, classification=cls)
    want = oracle.predict(f, X, classification=cls)
    assert (pred == want).all()
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
