"""GPU, world size 2 on one MI355X (gloo): the learner-sharded HIP fit end to end
(VERDICT r02 item 6).

Two ranks share cuda:0.  Rank 0 ingests cpusmall / vehicle once; replicate_dataset
hands the value codes, dictionaries and labels to rank 1 (host copy under gloo; one RCCL
broadcast with backend nccl on a multi-GPU node), which imports them.  Each rank fits its
learner block through libsbag (distributed.fit_shard), gather_model assembles the
ensemble in learner order, and distributed.transform aggregates the predictions across
the ranks.  Rank 0 compares all of it with a single-process HIP fit: the same nodes, the
same subspaces, learner order kept; votes bit-exact, means within 1e-12 of the sequential
sum (ml/regression/BaggingRegressor.scala:158-191, BaggingClassifier.scala:248-257).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import DATA, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cls, q):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist

    import sbag_loader

    sb = sbag_loader.load()
    from spark_bagging_amd import _native as nat
    from spark_bagging_amd import distributed as D

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        torch.cuda.set_device(0)
        ctx = nat.Context(0)
        name = "vehicle.svm" if cls else "cpusmall.svm"
        ds0 = None
        if rank == 0:
            X, y = sb.load_libsvm(os.path.join(DATA, name))
            if not cls:
                y = y / 10.0  # real-valued labels: the row-order fp64 path
            ds0 = nat.DeviceDataset.from_numpy(X, y, ctx)
        ds = D.replicate_dataset(ds0, dist, ctx)
        L = 9
        est = (sb.BaggingClassifier().setBaseLearner(sb.DecisionTreeClassifier().setMaxDepth(6))
               if cls else
               sb.BaggingRegressor().setBaseLearner(sb.DecisionTreeRegressor().setMaxDepth(6)))
        est = est.setNumBaseLearners(L).setReplacement(True).setSampleRatio(0.8)
        shard = D.fit_shard(est, ds, dist)
        full = D.gather_model(shard, dist)
        pred = D.transform(shard, ds, dist)
        # the replicated dataset is the ingested one, byte for byte
        mine = (ds.labels(), ds.features(0, 50), ds.layout())
        res = {"pred": pred, "nodes": [m.nodes for m in full.models],
               "subs": [np.asarray(s) for s in full.subspaces], "data": mine,
               "shard_learners": len(shard.models)}
        if rank == 0:
            ref = est.fit(ds)
            res["ref_nodes"] = [m.nodes for m in ref.models]
            res["ref_subs"] = [np.asarray(s) for s in ref.subspaces]
            res["ref_pred"], res["ref_pt"] = ref.transform(ds, per_tree=True)
        q.put((rank, res))
        ds.free()
        if ds0 is not None and ds0 is not ds:
            ds0.free()
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cls", [False, True])
def test_two_ranks_one_gpu_fit_gather_transform(cls):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cls, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=240)
            got[r] = res
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    a, b = got[0], got[1]
    assert a["shard_learners"] + b["shard_learners"] == 9
    # replication: rank 1's imported dataset equals rank 0's
    np.testing.assert_array_equal(a["data"][0], b["data"][0])
    np.testing.assert_array_equal(a["data"][1], b["data"][1])
    assert a["data"][2] == b["data"][2]
    for res in (a, b):
        assert len(res["nodes"]) == 9
        for l in range(9):
            assert res["nodes"][l].tobytes() == a["ref_nodes"][l].tobytes(), f"learner {l}"
            assert list(res["subs"][l]) == list(a["ref_subs"][l])
        if cls:
            np.testing.assert_array_equal(res["pred"], a["ref_pred"])
        else:
            # rank-order partial sums: the in-order sum re-associated at the shard boundary
            lb = 9 // 2
            pt = a["ref_pt"]
            s0, s1 = np.zeros(pt.shape[1]), np.zeros(pt.shape[1])
            for t in range(lb):
                s0 = s0 + pt[t]
            for t in range(lb, 9):
                s1 = s1 + pt[t]
            np.testing.assert_array_equal(res["pred"], (s0 + s1) / 9)
            np.testing.assert_allclose(res["pred"], a["ref_pred"], rtol=1e-12, atol=0)
