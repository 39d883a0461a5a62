"""Learner sharding across processes (one process per GPU, torch.distributed).

Bagging learners are independent (ml/regression/BaggingRegressor.scala:169-189: one
Future per learner, no shared state), and every learner's bag and subspace depend
only on (seed + i, partition layout, data) -- so rank g trains learners
[g*L/G, (g+1)*L/G) with no data-path collective.  Collectives are
used only to assemble the model and to aggregate predictions in learner order, and
they move device tensors (backend "nccl" = RCCL over xGMI on MI355X; "gloo" with CPU
tensors in the CPU tests):

  regression      every rank sums its own trees' predictions in learner order on the
                  device (sbag_predict_dataset_device, SBAG_OUT_SUM: N fp64), an
                  all-to-all hands rank g the G partial sums of its row shard, which
                  it adds in rank order and divides by L (sbag_aggregate_device):
                  BaggingRegressionModel.predict's sequential sum / L
                  (ml/regression/BaggingRegressor.scala:248-256) re-associated at the
                  G shard boundaries -- within 1e-5 relative (north_star), and
                  deterministic.  8 bytes per row cross the links, not 8 L;
  classification  every rank writes its trees' class ids as u8 (u16 above 256
                  classes) [L_g x N]; an all-to-all by row shard gives rank g all L
                  votes of its rows in learner order (rank order = learner order),
                  and breeze's mode with its first-to-reach-the-max tie rule
                  (BaggingClassifier.scala:248-257) runs there -- bit-exact.
  Both finish with an all-gather of the N fp64 predictions by row shard.

Dataset replication (every GPU holds the full binned matrix; the reference's
learners share one persisted DataFrame, ml/regression/BaggingRegressor.scala:158-189):
replicate_dataset has rank 0 ingest once and broadcast the value codes -- device memory
over RCCL with backend "nccl", host memory with "gloo" -- plus dictionaries and labels;
the other ranks import them (sbag_dataset_import validates every code) instead of
re-ingesting rows.  Under gloo the collectives stage device tensors through host memory,
so the CPU tests and a one-GPU multi-rank run share the code path.
"""
import numpy as np


def learner_range(num_learners, rank, world):
    """Contiguous learner block of `rank`; blocks cover [0, L) in rank order."""
    return (rank * num_learners // world, (rank + 1) * num_learners // world)


def row_range(num_rows, rank, world):
    """Row shard of `rank` for the aggregation (contiguous, rank order)."""
    return (rank * num_rows // world, (rank + 1) * num_rows // world)


def _staged(dist, t):
    """gloo moves host tensors: a device tensor goes through host memory."""
    return dist.get_backend() == "gloo" and t.is_cuda


def _all_gather_ints(value, dist, device):
    import torch

    if dist.get_backend() == "gloo":
        device = "cpu"
    world = dist.get_world_size()
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [int(o.item()) for o in out]


def exchange_rows(local, dist):
    """All-to-all by row shard: this rank's [K_rank x N] tensor -> [K_total x n_rank],
    the rows of every rank's block stacked in rank order (= learner order)."""
    import torch

    if _staged(dist, local):
        return exchange_rows(local.cpu(), dist).to(local.device)
    world, rank = dist.get_world_size(), dist.get_rank()
    K, N = local.shape
    ks = _all_gather_ints(K, dist, local.device)
    shards = [row_range(N, s, world) for s in range(world)]
    a, b = shards[rank]
    n_me = b - a
    # torch's NCCL binding converts only float/half/double/bf16/int8/uint8/int32/int64/bool:
    # u16 votes (> 256 classes) cross the links as bytes, every column range scaled by 2
    w = 1
    src = local
    if local.dtype in (torch.int16, torch.uint16):
        w = local.element_size()
        src = local.contiguous().view(torch.uint8)  # [K x w N]
    send = torch.cat([src[:, w * s0:w * s1].reshape(-1) for s0, s1 in shards]) if K else \
        torch.empty(0, dtype=src.dtype, device=src.device)
    recv = torch.empty(sum(ks) * n_me * w, dtype=src.dtype, device=src.device)
    dist.all_to_all_single(recv, send, output_split_sizes=[k * n_me * w for k in ks],
                           input_split_sizes=[K * (s1 - s0) * w for s0, s1 in shards])
    out = recv.view(sum(ks), n_me * w)
    return out.view(local.dtype) if w > 1 else out


def gather_rows(part, num_rows, dist):
    """All-gather the row shards' predictions [n_rank] -> [N] in row order."""
    import torch

    if _staged(dist, part):
        return gather_rows(part.cpu(), num_rows, dist).to(part.device)
    world = dist.get_world_size()
    sizes = [row_range(num_rows, s, world) for s in range(world)]
    sizes = [s1 - s0 for s0, s1 in sizes]
    pad = torch.zeros(max(sizes), dtype=part.dtype, device=part.device)
    pad[: part.shape[0]] = part
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return torch.cat([o[:s] for o, s in zip(outs, sizes)])


def sharded_aggregate(local, num_rows, dist, reduce_fn):
    """exchange_rows -> reduce_fn([K_total x n_rank]) -> [n_rank] fp64 -> gather_rows."""
    rows = exchange_rows(local, dist)
    return gather_rows(reduce_fn(rows), num_rows, dist)


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


def replicate_dataset(dataset, dist, ctx):
    """Rank 0's DeviceDataset on every rank: rank 0 passes its ingested dataset, the others
    None.  The codes (N x row_stride x code_bytes bytes) cross as one broadcast -- in device
    memory over RCCL (backend "nccl"), through host memory with gloo -- with the
    dictionaries and labels; ranks > 0 import them on `ctx`'s device.  Returns this rank's
    dataset (rank 0: `dataset` itself)."""
    import torch

    from . import _native as nat

    rank = dist.get_rank()
    on_dev = dist.get_backend() == "nccl"
    dev = torch.device("cuda", ctx.device) if on_dev else torch.device("cpu")
    lay = torch.zeros(5, dtype=torch.int64, device=dev)
    if rank == 0:
        lay.copy_(torch.tensor(dataset.layout(), dtype=torch.int64))
    dist.broadcast(lay, 0)
    n, f, s, cb, dv = (int(v) for v in lay.cpu().tolist())
    codes = torch.empty(n * s * cb, dtype=torch.uint8, device=dev)
    dvals = torch.zeros(max(dv, 1), dtype=torch.float64, device=dev)
    doff = torch.zeros(f + 1, dtype=torch.int64, device=dev)
    y = torch.zeros(n, dtype=torch.float64, device=dev)
    if rank == 0:
        if on_dev:
            torch.cuda.synchronize(dev)  # the allocation precedes the library's copy into it
        d, off, yy = dataset.export(codes.data_ptr(), codes_on_device=on_dev)
        dvals[:dv].copy_(torch.from_numpy(d))
        doff.copy_(torch.from_numpy(off))
        y.copy_(torch.from_numpy(yy))
    for t in (codes, dvals, doff, y):
        dist.broadcast(t, 0)
    if rank == 0:
        out = dataset
    else:
        if on_dev:
            torch.cuda.synchronize(dev)  # the broadcast has landed before the library reads it
        out = nat.DeviceDataset.import_codes(ctx, (n, f, s, cb, dv), codes.data_ptr(), on_dev,
                                             dvals[:dv].cpu().numpy(), doff.cpu().numpy(),
                                             y.cpu().numpy())
    # the staging tensors (a full copy of the codes: 25.6 GB for C4) go back to the device:
    # the engine allocates with hipMalloc, which torch's caching allocator would otherwise
    # keep from it
    del codes, dvals, doff, y, lay
    if on_dev:
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
    return out


def fit_shard(estimator, frame, dist, devices=None):
    """Train this rank's learner block of `estimator` (no collective)."""
    L = estimator.getNumBaseLearners()
    lb, le = learner_range(L, dist.get_rank(), dist.get_world_size())
    return estimator.fit_range(frame, lb, le, devices=devices)


def _num_classes(models):
    c = 0
    for m in models:
        leaves = m.nodes["left"] < 0
        if leaves.any():
            c = max(c, int(m.nodes["prediction"][leaves].max()) + 1)
    return c


def transform(shard, dataset, dist, device=None):
    """Ensemble prediction of a learner-sharded model on every rank's device: the
    rank's trees over its replica of the rows (HIP kernels, device outputs), an RCCL
    all-to-all by row shard, the ordered aggregation on the device, an all-gather.
    `dataset` is a DeviceDataset on this rank's device or host rows [N x F].
    Returns the N predictions (numpy fp64) on every rank."""
    import torch

    from . import _native as nat
    from .ml import Frame

    if isinstance(dataset, nat.DeviceDataset):
        ctx, ds = dataset.ctx, dataset
    else:
        ctx = nat.default_context(0 if device is None else device)
        frame = dataset if isinstance(dataset, Frame) else Frame(dataset, np.zeros(dataset.shape[0]))
        ds = frame.device_dataset(ctx)  # dense or SparseVector rows
    dev = torch.device("cuda", ctx.device)

    def sync():
        # the library runs on its own stream: what torch's stream wrote (fills, the
        # collective's output) must be complete before a native call reads or overwrites it
        torch.cuda.current_stream(dev).synchronize()
    N = ds.shape[0]
    L_me = len(shard.models)
    L = sum(_all_gather_ints(L_me, dist, dev))
    forest = shard.native_forest() if L_me else None
    if shard._agg == nat.AGG_MEAN:
        part = torch.zeros((1, N), dtype=torch.float64, device=dev)
        if forest is not None:
            sync()
            nat.predict_dataset_device(ctx, forest, ds, nat.OUT_SUM, 0, part.data_ptr())

        def reduce_fn(rows):  # [G x n]: partial sums in rank order
            out = torch.empty(rows.shape[1], dtype=torch.float64, device=dev)
            rows = rows.contiguous()
            sync()
            nat.aggregate_device(ctx, rows.data_ptr(), 8, rows.shape[0],
                                 rows.shape[1], nat.AGG_MEAN, L, 0, out.data_ptr())
            return out
    else:
        C = max(_all_gather_ints(_num_classes(shard.models), dist, dev))
        vb = 1 if C <= 256 else 2
        part = torch.zeros((L_me, N), dtype=torch.uint8 if vb == 1 else torch.int16, device=dev)
        if forest is not None:
            sync()
            nat.predict_dataset_device(ctx, forest, ds, nat.OUT_VOTES, vb, part.data_ptr())

        def reduce_fn(rows):  # [L x n]: every learner's vote in learner order
            out = torch.empty(rows.shape[1], dtype=torch.float64, device=dev)
            rows = rows.contiguous()
            sync()
            nat.aggregate_device(ctx, rows.data_ptr(), vb, rows.shape[0],
                                 rows.shape[1], nat.AGG_MODE, L, C, out.data_ptr())
            return out
    pred = sharded_aggregate(part, N, dist, reduce_fn)
    torch.cuda.synchronize(dev)
    return pred.cpu().numpy()
