"""Learner sharding across processes (one process per GPU, torch.distributed).

Bagging learners are independent (ml/regression/BaggingRegressor.scala:169-189: one
Future per learner, no shared state), and every learner's bag and subspace depend
only on (seed + i, partition layout, data) -- so rank g trains learners
[g*L/G, (g+1)*L/G) with no data-path collective.  Collectives are
used only to assemble the model and to aggregate predictions IN LEARNER ORDER:

  regression      per-tree predictions all-gathered in learner order, then the
                  sequential sum / L of BaggingRegressionModel.predict
                  (ml/regression/BaggingRegressor.scala:248-256) -- bit-identical
                  to the single-process order;
  classification  per-tree votes all-gathered, then breeze mode with its
                  first-to-reach-the-max tie rule (BaggingClassifier.scala:248-257).

The backend is whatever process group is initialised: "nccl" (RCCL over xGMI)
on MI355X nodes, "gloo" in the CPU tests.
"""
import numpy as np


def learner_range(num_learners, rank, world):
    """Contiguous learner block of `rank`; blocks cover [0, L) in rank order."""
    return (rank * num_learners // world, (rank + 1) * num_learners // world)


def gather_votes(local_votes, dist, device=None):
    """All-gather per-tree predictions [L_rank x N] into [L x N] in learner order."""
    import torch

    world = dist.get_world_size()
    local = torch.as_tensor(np.ascontiguousarray(local_votes, np.float64), device=device)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    lmax = max(sizes)
    pad = torch.zeros((lmax, local.shape[1]), dtype=torch.float64, device=device)
    pad[: local.shape[0]] = local
    parts = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return np.concatenate([p[:s].cpu().numpy() for p, s in zip(parts, sizes)], axis=0)


def gather_model(shard, dist):
    """Assemble the full model on every rank: subspaces and trees in learner order."""
    world = dist.get_world_size()
    payload = [(np.asarray(s), m.nodes, m.stats, m.impurity)
               for s, m in zip(shard.subspaces, shard.models)]
    out = [None] * world
    dist.all_gather_object(out, payload)
    from .ml import DecisionTreeModel

    subs, models = [], []
    for part in out:
        for s, nodes, stats, imp in part:
            subs.append(s)
            models.append(DecisionTreeModel(nodes, stats, imp))
    full = type(shard)(subs, models, uid=shard.uid)
    full._values = dict(shard._values)
    return full


def fit_shard(estimator, frame, dist, devices=None):
    """Train this rank's learner block of `estimator` (no collective)."""
    L = estimator.getNumBaseLearners()
    lb, le = learner_range(L, dist.get_rank(), dist.get_world_size())
    return estimator.fit_range(frame, lb, le, devices=devices)


def transform(shard, X, dist, device=None, agg_fn=None):
    """Ensemble prediction of a learner-sharded model: local per-tree predictions
    (HIP kernel), all-gather in learner order, ordered aggregation."""
    from . import _native as nat

    _, per_tree = shard.transform(X, device=0 if device is None else device, per_tree=True)
    votes = gather_votes(per_tree, dist, device=None)
    if agg_fn is not None:
        return agg_fn(votes)
    return nat.aggregate(nat.default_context(0 if device is None else device), votes, shard._agg)
