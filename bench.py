#!/usr/bin/env python3
"""Bench: BaggingRegressor(DecisionTreeRegressor).fit on the synthetic C3 workload
(BASELINE.json configs[2]: 10M rows x 100 features, 128 bootstrap depth-8 trees,
one MI355X).  One step = one full fit (Poisson bag -> split finding -> binning ->
8 tree levels for all 128 learners -> forest on the host), inputs resident in HBM.

With --gpus N (launched by torch.distributed.run) every rank trains its own
128 learners [rank*128, (rank+1)*128) of the same ensemble on its own GPU: weak
scaling, no collective on the data path (learners are independent).
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import sbag_loader  # noqa: E402

SEED_REG = -1395689524  # default seed of BaggingRegressor (class-name hashCode)
SEED_CLS = 42087812     # default seed of BaggingClassifier
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E (MI355X_MICROARCH.md)
MFMA_I8_PEAK_TOPS = 5000.0  # dense int8 MFMA, 2x the ~2.5 PF dense BF16 (MI355X_MICROARCH.md, matrix cores)
# ds_add_u64 throughput measured on MI355X by scripts/micro/lds_atomic.hip:
# 7.16 cycles per wave-instruction per CU (4 x 512-thread workgroups per CU), 256 CUs, 2.4 GHz
LDS_ATOMIC_PEAK = 256 * 2.4e9 / 7.16
# ds_add_u32 (the gini class counts): 5.97 cycles per wave-instruction, same micro-benchmark
LDS_ATOMIC_PEAK_U32 = 256 * 2.4e9 / 5.97
# committed rocprofv3 PMC summaries of this command per workload (scripts/profile.sh +
# scripts/pmc_summary.py); the newest one present is used
PMC_SUMMARIES = {"c3": ["profiles/r06/c3/summary.json", "profiles/r05pr/c3/summary.json", "profiles/r04bn/c3/summary.json", "profiles/r04ac/c3/summary.json", "profiles/r04o/c3/summary.json", "profiles/r03y/c3/summary.json", "profiles/r03r/c3/summary.json", "profiles/r03g/c3/summary.json", "profiles/r02g/c3/summary.json", "profiles/r02f/c3/summary.json",
                        "profiles/r02e/c3/summary.json", "profiles/r01g/summary.json"],
                 "c4": ["profiles/r06/c4/summary.json", "profiles/r05pr/c4/summary.json", "profiles/r04o/c4/summary.json", "profiles/r02g/c4/summary.json", "profiles/r02f/c4/summary.json"],
                 "c5": ["profiles/r06/c5/summary.json", "profiles/r05s/c5/summary.json", "profiles/r05a/c5/summary.json", "profiles/r03y/c5/summary.json", "profiles/r02g/c5/summary.json", "profiles/r02f/c5/summary.json",
                        "profiles/r02e/c5/summary.json", "profiles/r01g_c5/summary.json"]}


def pmc_traffic(workload):
    """HBM bytes per histogram launch from the committed PMC summary of this same command:
    2 x FETCH_SIZE (gfx950 reports half of 128-B reads) + WRITE_SIZE.  The counters need
    their own rocprofv3 passes, so they are not collected inside this run: the value is
    returned with the summary it came from (stale if the kernel changed since)."""
    for rel in PMC_SUMMARIES.get(workload, []):
        try:
            with open(os.path.join(ROOT, rel)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            # (the level histograms' kernel; the MFMA root is reported apart)
            if (k.startswith("sbag::k_hist<") or k.startswith("sbag::k_hist_rl<")) and "hbm_bytes_per_launch" in v:
                return round(v["hbm_bytes_per_launch"]), rel, k
    return None, None, None


# BASELINE.json configs as bench workloads (per GPU).  c3 is the headline (default);
# c4 / c5 are the shapes of configs[3] / configs[4] on one GPU's learner shard.
WORKLOADS = {
    "c3": dict(rows=10_000_000, features=100, learners=128, depth=8, classes=0,
               replacement=True, ratio=1.0,
               name="C3: BaggingRegressor(DecisionTreeRegressor) fit, synthetic {N} rows x {F} "
                    "features, {L} bootstrap depth-{D} trees per GPU"),
    "c4": dict(rows=100_000_000, features=256, learners=64, depth=8, classes=0,
               replacement=True, ratio=1.0,
               name="C4 shard: BaggingRegressor fit, synthetic {N} rows x {F} features, "
                    "{L} bootstrap depth-{D} trees per GPU (512 learners over 8 GPUs)"),
    "c5": dict(rows=50_000_000, features=100, learners=16, depth=12, classes=64,
               replacement=False, ratio=0.5,
               name="C5 shard: BaggingClassifier(DecisionTreeClassifier) fit, synthetic {N} rows "
                    "x {F} features, {C} classes, subsample 0.5 without replacement, {L} depth-{D} "
                    "trees per GPU (128 learners over 8 GPUs)"),
}


def hist_kernel_name(F, cls, N):
    """The k_hist variant the host picks for an F-feature tile (sbag_host.cpp
    hist_geometry): row lanes when roundup(F, 16) < roundup(F, 64)."""
    if cls:
        # gini tiles shrink features and classes to fit the LDS target; the variant is
        # not predicted here (C5 runs sbag::k_hist<0, 1, 4>: profiles/r02e/c5/)
        return "sbag::k_hist* (kHistGini, class tiles; variant per hist_geometry)"
    ft = min(F, 256)
    mode = "0" if cls else "1"
    tag = "kHistGini, class tiles" if cls else "kHistVar"
    if -(-ft // 16) * 16 < -(-ft // 64) * 64:
        k = -(-ft // 16)
        off32 = "true" if N < (1 << 24) else "false"
        return f"sbag::k_hist_rl<{mode}, {k}, {off32}> ({tag}, row lanes)"
    return f"sbag::k_hist<{mode}, {-(-ft // 64)}> ({tag}, {-(-ft // 64)} lane groups)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for --gpus > 1 (nccl = RCCL over xGMI; gloo "
                         "stages the collectives through host memory, so N ranks can share one "
                         "GPU: the multi-rank path rehearsed on a 1-GPU box)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--features", type=int, default=None)
    ap.add_argument("--learners", type=int, default=None, help="learners per GPU")
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--bins", type=int, default=32)
    ap.add_argument("--partitions", type=int, default=128)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--sampler-partitions", type=int, default=None,
                    help="also time one fit's sampler at this P (default: nproc)")
    ap.add_argument("--cpu-rows", type=int, default=1_000_000)
    ap.add_argument("--cpu-learners", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-nondyadic", action="store_true",
                    help="skip the extra timing of the same fit on real-valued (non-dyadic) labels")
    ap.add_argument("--nondyadic-steps", type=int, default=3)
    ap.add_argument("--no-continuous", action="store_true",
                    help="skip the extra timing of the C3 shape on continuous features")
    ap.add_argument("--continuous-steps", type=int, default=3)
    a = ap.parse_args()
    w = WORKLOADS[a.workload]
    for k in ("rows", "features", "learners", "depth"):
        if getattr(a, k) is None:
            setattr(a, k, w[k])
    a.classes, a.replacement, a.ratio = w["classes"], w["replacement"], w["ratio"]
    a.workload_name = w["name"].format(N=a.rows, F=a.features, L=a.learners, D=a.depth, C=a.classes)
    return a


def cpu_baseline(args):
    """The oracle (CPU restatement, OpenMP over learners) on a bounded sample of the
    same workload: cpu_rows rows x F features, cpu_learners learners, same depth/bins."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from spark_bagging_amd import synthetic

    n, L = args.cpu_rows, args.cpu_learners
    cores = nproc()  # all host cores this process may use (what `nproc` prints)
    cls = args.classes > 0
    seed = SEED_CLS if cls else SEED_REG
    X, y = synthetic.generate(n, args.features, args.seed, args.classes)
    part = [int(round(i * n / args.partitions)) for i in range(args.partitions + 1)]
    counts = oracle.bag(args.replacement, args.ratio, 0, L, seed, part, n)
    subs = [oracle.subspace(args.ratio, args.features, seed + i) for i in range(L)]
    t0 = time.perf_counter()
    oracle.fit(X, y, counts, subs, max_depth=args.depth, max_bins=args.bins, nthreads=cores,
               classification=cls)
    dt = time.perf_counter() - t0
    return {"value": L * n / dt, "unit": "estimator*rows/s", "cores": cores, "kind": "port",
            "sample": f"{n} rows x {args.features} features, {L} learners, depth {args.depth}, "
                      f"{args.partitions} partitions; oracle/sbag_oracle.c fit only "
                      f"({dt:.1f} s, restatement, not Spark)"}


def continuous_data(N, F, seed=20261017):
    """Continuous features of the C3 shape: ~2400-38000 distinct values per feature (tiles of one
    rounded-normal block, each shifted), dyadic labels."""
    import numpy as np

    rng = np.random.default_rng(seed)
    blk = min(N, 1_000_000)
    B = np.round(rng.standard_normal((blk, F), dtype=np.float32) * 300).astype(np.float64) / 8
    X = np.empty((N, F))
    for k in range(0, N, blk):
        n = min(blk, N - k)
        X[k:k + n] = B[:n] + (k // blk) / 16.0
    y = np.round((X[:, 0] * 0.37 - X[:, 1] * 1.3 + X[:, 2] * 0.05) * 16) / 16
    return X, y


def continuous_fit(nat, ctx, N, F, L, depth, bins, part, steps=1):
    """Fit the continuous-feature dataset (ingested from host fp64 rows, timed apart) with the
    headline's tree parameters; returns the report dict."""
    t0 = time.perf_counter()
    X, y = continuous_data(N, F)
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    del X
    t_ingest = time.perf_counter() - t0

    def fit(lend):
        return nat.fit(ctx, ds, replacement=True, sample_ratio=1.0, seed=SEED_REG, learner_begin=0,
                       learner_end=lend, partition_offsets=part, max_depth=depth, max_bins=bins,
                       impurity=nat.IMPURITY_VARIANCE)

    fit(L).free()  # warmup: the same fit (its workspace -- ~100 GB of per-replica bins -- is allocated here)
    import torch
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(steps):
        f = fit(L)
        tm = f.timing()
        f.free()
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    tser = serialized_timing(lambda: fit(L))
    ds.free()
    return {"data": "continuous: ~2400-38000 distinct values per feature (host fp64 rows), dyadic "
                    "labels; per-replica thresholds from each replica's split-finding sample, "
                    "per-replica bins materialized on the device",
            "rows": N, "features": F, "learners": L, "steps": steps,
            "ms_per_step": round(1000.0 * el / steps, 3), "value": round(L * N * steps / el, 1),
            "unit": "estimator*rows/s", "ingest_s_untimed": round(t_ingest, 2),
            "breakdown_ms": breakdown_of(tser),
            "breakdown_def": "a fit with the learner parts serialized (SBAG_OVERLAP=0, after one "
                             "such warm fit), HIP events per stage; the timed steps overlap the parts",
            "step_total_ms_overlapped": round(tm["total_ms"], 3)}


def nproc():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


STAGES = ("sample_ms", "valuecount_ms", "bin_ms", "compact_ms", "hist_ms", "split_ms", "subtract_ms",
          "partition_ms", "fix_ms", "group_ms", "chain_ms", "root_ms")


def serialized_timing(fit):
    """Per-stage HIP-event times of one fit with the learner parts serialized (SBAG_OVERLAP=0):
    each launch runs alone, on the stream it is launched on.  The serialized fit runs twice and
    the second is reported: a single-part fit of all the learners needs bigger per-fit buffers
    than the timed steps' parts, and the first such fit allocates them inside its event window
    (the C4 shard: 2.8 s of total_ms against a 1.06 s step before round 6)."""
    prev = os.environ.get("SBAG_OVERLAP")
    os.environ["SBAG_OVERLAP"] = "0"
    try:
        fit().free()
        f = fit()
        tm = f.timing()
        f.free()
    finally:
        if prev is None:
            os.environ.pop("SBAG_OVERLAP", None)
        else:
            os.environ["SBAG_OVERLAP"] = prev
    return tm


def breakdown_of(tm):
    """breakdown_ms of a timing dict, with the stage sum against total_ms: what the stages do
    not cover is host time between kernels on the fit's stream (each level's split results and
    partition cursors go to the host and the next level's work lists come back)."""
    b = {k: round(v, 3) for k, v in tm.items() if k.endswith("_ms")}
    ssum = sum(tm.get(k, 0.0) for k in STAGES)
    tot = tm.get("total_ms", 0.0)
    b["stage_sum_ms"] = round(ssum, 3)
    b["unattributed_ms"] = round(tot - ssum, 3)
    b["unattributed_is"] = ("host time between kernels on the fit's stream (per-level results to "
                            "the host, work lists back), not a kernel")
    return b


def build_record():
    """Whether the shipped libsbag.so is newer than every source it is built from (the driver
    runs __graft_entry__.build() in the build container; the GPU box runs the shipped .so)."""
    import datetime
    import glob

    csrc = os.path.join(ROOT, "spark-bagging_amd", "csrc")
    so = os.path.join(ROOT, "spark-bagging_amd", "libsbag.so")
    srcs = glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")) + \
        glob.glob(os.path.join(csrc, "*.h")) + [os.path.join(ROOT, "include", "sbag.h")]
    objs = glob.glob(os.path.join(csrc, "build", "*.o"))

    def iso(t):
        return datetime.datetime.fromtimestamp(t, datetime.timezone.utc).isoformat(timespec="seconds")

    try:
        so_t = os.path.getmtime(so)
    except OSError:
        return {"libsbag_so": None}
    src_t = max(os.path.getmtime(x) for x in srcs)
    rec = {"libsbag_so_mtime": iso(so_t), "newest_source_mtime": iso(src_t),
           "so_newer_than_sources": so_t >= src_t}
    if objs:
        rec["objects"] = len(objs)
        rec["newest_object_mtime"] = iso(max(os.path.getmtime(o) for o in objs))
        rec["so_newer_than_objects"] = so_t >= max(os.path.getmtime(o) for o in objs)
    else:
        rec["objects"] = 0  # (the object directory is not shipped to the GPU box)
    return rec


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    # ranks beyond the visible devices share them (gloo rehearsal of the multi-rank path on
    # one GPU); with one rank per GPU this is LOCAL_RANK
    dev = local % max(1, torch.cuda.device_count())
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(dev)
    # host tensors for the timing collectives under gloo
    tdev = "cuda" if args.backend == "nccl" else "cpu"
    sb = sbag_loader.load()
    nat = sb._native
    ctx = nat.Context(dev)
    N, F, L = args.rows, args.features, args.learners
    cls = args.classes > 0
    replication = None
    if world == 1:
        ds = nat.DeviceDataset.synthetic(N, F, seed=args.seed, num_classes=args.classes, ctx=ctx)
    else:
        # rank 0 ingests (here: generates) the dataset, the other ranks receive the
        # binned matrix over RCCL (distributed.replicate_dataset); timed apart from the fits
        from spark_bagging_amd import distributed as D
        dist.barrier()
        torch.cuda.synchronize()
        t_r = time.perf_counter()
        ds0 = (nat.DeviceDataset.synthetic(N, F, seed=args.seed, num_classes=args.classes, ctx=ctx)
               if rank == 0 else None)
        ds = D.replicate_dataset(ds0, dist, ctx)
        torch.cuda.synchronize()
        dist.barrier()
        t_rep = torch.tensor([time.perf_counter() - t_r], dtype=torch.float64, device=tdev)
        dist.all_reduce(t_rep, op=dist.ReduceOp.MAX)
        replication = {"seconds": round(float(t_rep.item()), 4), "bytes": ds.codes_nbytes() + 8 * N,
                       "how": "rank 0 generates the synthetic dataset; ranks > 0 import its value "
                              "codes, dictionaries and labels after %s broadcasts "
                              "(distributed.replicate_dataset)" % (
                                  "RCCL" if args.backend == "nccl" else "gloo (host-staged)")}
    part = [int(round(i * N / args.partitions)) for i in range(args.partitions + 1)]
    lb = rank * L

    def step():
        return nat.fit(ctx, ds, replacement=args.replacement, sample_ratio=args.ratio,
                       seed=SEED_CLS if cls else SEED_REG, learner_begin=lb, learner_end=lb + L,
                       partition_offsets=part, max_depth=args.depth, max_bins=args.bins,
                       impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)

    for _ in range(args.warmup):
        step().free()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timings = []
    for _ in range(args.steps):
        f = step()
        timings.append(f.timing())
        f.free()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    value = world * L * N * args.steps / elapsed

    # Kernel-level figures (roofline, breakdown) come from one more fit with the learner
    # halves serialized (SBAG_OVERLAP=0).  In the timed steps the two halves of the learner
    # range run on two streams (sbag_fit) and each kernel shares the GPU with
    # the other half's, which stretches its HIP-event duration; the serialized fit measures
    # each launch alone, on the stream it runs on.  The rocprofv3 profile uses the same
    # setting.
    kernel_fit = serialized_timing(step)
    timings = [kernel_fit]
    hist_ms = sum(t["hist_ms"] for t in timings)
    hist_launches = sum(t["hist_launches"] for t in timings)
    work_bytes = sum(t["hist_work_bytes"] for t in timings)
    read_bytes = sum(t["hist_alg_bytes"] for t in timings)
    nl = max(hist_launches, 1)
    avg_s = hist_ms / 1e3 / nl
    # achieved: the bytes one launch processes -- its entries x (F_r + 4): the in-bag
    # rows of the nodes it histograms (u8 bins of the replica's features + the 4-byte
    # label word) -- over the launch's average duration (HIP events on the context
    # stream, the stream the kernel runs on)
    achieved = read_bytes / nl / avg_s / 1e9 if hist_ms > 0 else 0.0
    # SURVEY 8d's work-defined figure also counts every sibling histogram obtained by
    # subtraction as if read: reported separately, it can exceed the peak
    effective = work_bytes / nl / avg_s / 1e9 if hist_ms > 0 else 0.0
    # LDS atomic co-limiter, counted by the host per launch (variance: ds_add_u64 of the
    # packed (count, sum) word after the screening of DESIGN.md §5; gini: ds_add_u32)
    lds_instr = sum(t["hist_lds_atomics"] for t in timings)
    lds_rate = lds_instr / (hist_ms / 1e3) if hist_ms > 0 else 0.0
    lds_peak = LDS_ATOMIC_PEAK_U32 if cls else LDS_ATOMIC_PEAK
    traffic, traffic_src, traffic_kernel = pmc_traffic(args.workload)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": (f"{traffic_src} ({traffic_kernel}; rocprofv3 PMC passes of this "
                                   "command, not re-measured inside this run)") if traffic else None,
                "kernel": hist_kernel_name(F, cls, N),
                "avg_launch_ms": round(hist_ms / nl, 4),
                "alg_bytes_per_launch": round(read_bytes / nl),
                "alg_bytes_def": "entries the launch histograms x (F_r + 4): u8 bin per feature of "
                                 "the replica's subspace + 4-byte label word (DESIGN.md §4)",
                # not a bandwidth (it counts bytes no kernel reads, and exceeds the peak on
                # C4), so it carries a ratio, never a frac
                "effective": {"work_rate": round(effective, 1),
                              "work_rate_over_peak": round(effective / HBM_PEAK_GBS, 4),
                              "bytes_per_launch": round(work_bytes / nl),
                              "def": "SURVEY 8d: sum over histograms built (read or by subtraction) "
                                     "of n(r,d)*(F_r+s_y) + 3N, s_y = 4 (regression) / 1 (class); "
                                     "sibling histograms from k_subtract count as if read"},
                "binding_limiter": "lds_atomic",
                "lds_atomic": {"achieved": round(lds_rate / 1e9, 2),
                               "peak": round(lds_peak / 1e9, 2),
                               "unit": "G wave-instr/s (%s peak, scripts/micro/lds_atomic.hip)"
                                       % ("ds_add_u32" if cls else "ds_add_u64"),
                               "frac": round(lds_rate / lds_peak, 4)}}
    # the root histogram as an int8 MFMA contraction (k_hist_mfma): its
    # dense int8 operations over its HIP-event time against the dense int8 MFMA peak
    root_ms = sum(t.get("root_ms", 0.0) for t in timings)
    root_ops = sum(t.get("root_mfma_ops", 0.0) for t in timings)
    if root_ms > 0 and root_ops > 0:
        tops = root_ops / (root_ms / 1e3) / 1e12
        roofline["root_mfma"] = {"kernel": "sbag::k_hist_mfma (root histogram, int8 MFMA)",
                                 "bound": "mfma", "achieved": round(tops, 1), "peak": MFMA_I8_PEAK_TOPS,
                                 "unit": "TOPS", "frac": round(tops / MFMA_I8_PEAK_TOPS, 4),
                                 "ms_per_fit": round(root_ms, 3),
                                 "ops_def": "2 x 32^3 int8 ops per v_mfma_i32_32x32x32_i8 issued: "
                                            "ceil(N/32) row steps x F x ceil(R/32) replica tiles "
                                            "x (1 + label digit planes)"}
    breakdown = breakdown_of(timings[-1])
    # the sampler's cost depends on rows per partition stream (Poisson.scala:53-56 reseeds
    # per partition): one extra fit, outside the timed region, at P = nproc
    sp = args.sampler_partitions or nproc()
    if sp != args.partitions:
        part_sp = [int(round(i * N / sp)) for i in range(sp + 1)]
        f = nat.fit(ctx, ds, replacement=args.replacement, sample_ratio=args.ratio,
                    seed=SEED_CLS if cls else SEED_REG, learner_begin=lb, learner_end=lb + L,
                    partition_offsets=part_sp, max_depth=args.depth, max_bins=args.bins,
                    impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
        tsp = f.timing()
        f.free()
        sampler_p = {"partitions": sp, "partitions_is": "nproc of this host" if not args.sampler_partitions
                     else "--sampler-partitions", "sample_ms": round(tsp["sample_ms"], 3),
                     "fit_ms": round(tsp["total_ms"], 3),
                     "headline_partitions": args.partitions, "headline_sample_ms": breakdown["sample_ms"]}
    else:
        sampler_p = {"partitions": sp, "sample_ms": breakdown["sample_ms"]}
    # The same fit on real-valued labels: y' = 1.1 y + 0.3 is not dyadic,
    # so sbag_fit takes the screened fp64 path (Spark's DTStatsAggregator row-order sums of the
    # chosen features, sbag_f64s.hip).
    # Reported beside the headline; not part of `value`.
    nondyadic = None
    if not cls and world == 1 and not args.no_nondyadic:
        y0 = ds.labels()
        ds.set_labels(y0 * 1.1 + 0.3)
        step().free()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        tl = []
        for _ in range(args.nondyadic_steps):
            f = step()
            tl.append(f.timing())
            f.free()
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        # per-stage times from a serialized fit, as for the headline's breakdown (the
        # overlapped steps stretch each stage by the other half's)
        tser = serialized_timing(step)
        ds.set_labels(y0)
        nondyadic = {"labels": "1.1 * y + 0.3 (fp64, not dyadic)", "steps": args.nondyadic_steps,
                     "ms_per_step": round(1000.0 * el / args.nondyadic_steps, 3),
                     "value": round(L * N * args.nondyadic_steps / el, 1),
                     "unit": "estimator*rows/s",
                     "breakdown_ms": breakdown_of(tser),
                     "breakdown_def": "a fit with the learner halves serialized (SBAG_OVERLAP=0, "
                                      "after one such warm fit), HIP events per stage",
                     "exact_fallbacks": int(tl[-1]["exact_fallbacks"]),
                     "engine": "screened fp64 engine: splits chosen from integer histograms of the "
                               "labels' fixed-point image under a rigorous error bound; the chosen "
                               "feature's bins summed as Spark's executors do -- each partition's "
                               "rows in row order, the partials merged in partition order "
                               "(k_fb_psum / k_fb_pmerge; 'chain_ms' includes the stable routing); "
                               "flagged nodes ('exact_fallbacks') summed the same way on every "
                               "contending feature (DESIGN.md §4.7)"}
    # The C3 shape on continuous features: thousands of distinct values per
    # feature, so every replica is thresholded on its own split-finding sample and its bins are
    # materialized per replica.  Reported beside the headline; not `value`.
    continuous = None
    if args.workload == "c3" and world == 1 and not args.no_continuous:
        ds.free()
        continuous = continuous_fit(nat, ctx, N, F, L, args.depth, args.bins, part, steps=args.continuous_steps)
    out = {
        "metric": "estimator×rows trained/sec", "value": round(value, 1),
        "unit": "estimator*rows/s", "n_gpus": world, "backend": args.backend if world > 1 else None,
        "devices_used": min(world, torch.cuda.device_count()), "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (device generator k_synth: splitmix64 codes mod 32, "
                + ("class labels)" if cls else "dyadic labels)"),
        "config": {"workload": args.workload_name,
                   "rows": N, "features": F, "learners_per_gpu": L, "learners_total": L * world,
                   "max_depth": args.depth, "max_bins": args.bins, "partitions": args.partitions,
                   "classes": args.classes, "replacement": args.replacement,
                   "sample_ratio": args.ratio, "parallelism": f"learner-shard x{world}"},
        "roofline": roofline, "breakdown_ms": breakdown, "sampler_at_nproc_partitions": sampler_p,
        "nondyadic_labels": nondyadic, "continuous_features": continuous, "replication": replication,
        "value_incl_replication": (round(world * L * N * args.steps / (elapsed + replication["seconds"]), 1)
                                   if replication else None),
        "kernel_timing": "roofline and breakdown_ms: a fit after the timed steps with the learner "
                         "halves serialized (SBAG_OVERLAP=0, after one such warm fit), so each "
                         "launch runs alone; the timed steps overlap the two halves on two streams",
        "build": build_record(),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
