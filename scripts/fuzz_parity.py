"""Randomized parity fuzzing at larger shapes than tests/test_gpu_random.py: every case a
fresh random dataset and parameter draw (rows up to ~150k, up to 140 features, up to 80
classes -- grouped class tiles --, 32-level u8 columns for the row-lane kernel, non-dyadic
fp64 labels for the fp64 engine, depth up to 14, several partitions), each forest checked
against the CPU oracle node by node.  Runs until the time budget is spent; prints one line
per case so a failure names its seed and replays with --start SEED --cases 1.

usage: python3 scripts/fuzz_parity.py [--start S] [--minutes M] [--cases K]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import sbag_loader  # noqa: E402

sb = sbag_loader.load()
nat = sb._native
import oracle  # noqa: E402
from parity_utils import assert_forest_equal, fuzz_case, fuzz_case_big, oracle_forest  # noqa: E402


draw = fuzz_case  # tests/parity_utils.py


draw_big = fuzz_case_big  # tests/parity_utils.py


def run(ctx, seed, extra=False, big=False):
    X, y, cls, f64, part, p, kind = (draw_big if big else draw)(seed)
    sd = oracle.DEFAULT_SEED_CLASSIFIER if cls else oracle.DEFAULT_SEED_REGRESSOR
    N, F = X.shape
    # --extra: a learner range that does not start at 0 and, half the time, a subspace
    # ratio of its own (subspace_bug_compat off); its own stream, so the draws above keep
    # their meaning (tests/test_gpu_random.py pins some)
    lb, sub_ratio, compat = 0, p["ratio"], True
    if extra:
        rng2 = np.random.default_rng(seed + 10**7)
        lb = int(rng2.choice([0, 1, 7, 129, 511]))
        if rng2.random() < 0.5:
            compat, sub_ratio = False, float(rng2.choice([1.0, 0.8, 0.3]))
    desc = (f"seed {seed} N {N} F {F} {kind} {'cls C=%d' % (int(y.max()) + 1) if cls else ('f64' if f64 else 'reg')} "
            f"P {len(part) - 1} lb {lb} sub {sub_ratio if not compat else 'H1'} {p}")
    ds = nat.DeviceDataset.from_numpy(X, y, ctx)
    try:
        forest = nat.fit(ctx, ds, replacement=p["replacement"], sample_ratio=p["ratio"], seed=sd,
                         learner_begin=lb, learner_end=lb + p["L"], partition_offsets=part,
                         subspace_ratio=sub_ratio, subspace_bug_compat=compat,
                         max_depth=p["depth"], max_bins=p["bins"],
                         min_instances_per_node=p["min_inst"], min_info_gain=p["min_gain"],
                         impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
    except sb.SparkException as e:
        ds.free()
        counts = oracle.bag(p["replacement"], p["ratio"], lb, lb + p["L"], sd, part, N)
        ok = e.code == nat.SBAG_EEMPTY and (counts.sum(axis=1) == 0).any()
        return ok, desc + f" -> {e}"
    except sb.IllegalArgumentException as e:
        ds.free()
        ok = any(len(oracle.subspace(sub_ratio, F, sd + i)) == 0 for i in range(lb, lb + p["L"]))
        return ok, desc + f" -> {e}"
    counts = oracle.bag(p["replacement"], p["ratio"], lb, lb + p["L"], sd, part, N)
    subs = [oracle.subspace(sub_ratio, F, sd + i) for i in range(lb, lb + p["L"])]
    orf = oracle_forest(X, y, counts, subs, p["depth"], p["bins"], cls, p["min_inst"], p["min_gain"],
                        part=part)
    try:
        assert_forest_equal(forest, orf)
        agg = nat.AGG_MODE if cls else nat.AGG_MEAN
        want = oracle.predict(orf, X, classification=cls)
        got = nat.predict(ctx, forest, X, agg)
        np.testing.assert_array_equal(got, want)
        if extra:  # rows already on the device: the binned transform
            np.testing.assert_array_equal(nat.predict_dataset(ctx, forest, ds, agg), want)
    except AssertionError as e:
        return False, desc + " FAIL " + str(e)[:400]
    finally:
        forest.free()
        ds.free()
    return True, desc


def run_booster(ctx, seed):
    """--booster: one GBM base learner (sbag_fit_booster, Spark's row-order fp64 sums) on a
    draw's rows with real-valued labels, a bag and a subspace, against the oracle's tree."""
    X, y, cls, f64, part, p, kind = draw(seed)
    rng = np.random.default_rng(seed + 2 * 10**7)
    N, F = X.shape
    lab = rng.normal(size=N) * 3.3 + (X[:, 0] if F else 0.0) * 0.1
    counts = oracle.bag(p["replacement"], p["ratio"], 5, 6, 77 + seed, part, N)[0]
    sub = oracle.subspace(p["ratio"], F, 1234 + seed)
    desc = f"booster seed {seed} N {N} F {F} {kind} P {len(part) - 1} {p}"
    if counts.sum() == 0 or len(sub) == 0:
        return True, desc + " (empty bag or subspace: skipped)"
    ds = nat.DeviceDataset.from_numpy(X, np.zeros(N), ctx)
    try:
        f = nat.fit_booster(ctx, ds, lab, counts, sub, partition_offsets=part, max_depth=min(p["depth"], 10),
                            max_bins=p["bins"], min_instances_per_node=p["min_inst"],
                            min_info_gain=p["min_gain"])
    finally:
        ds.free()
    orf = oracle.fit(X, lab, counts[None, :], [sub], max_depth=min(p["depth"], 10), max_bins=p["bins"],
                     min_instances_per_node=p["min_inst"], min_info_gain=p["min_gain"], part=part)
    try:
        from parity_utils import assert_tree_equal
        assert_tree_equal(f, 0, orf, 0)
    except AssertionError as e:
        return False, desc + " FAIL " + str(e)[:400]
    finally:
        f.free()
    return True, desc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=50_000)
    ap.add_argument("--minutes", type=float, default=5.0)
    ap.add_argument("--cases", type=int, default=10**9)
    ap.add_argument("--extra", action="store_true",
                    help="learner offsets, subspace ratios of their own, device transform")
    ap.add_argument("--big", action="store_true", help="1-3M rows, 16-32 learners (draw_big)")
    ap.add_argument("--booster", action="store_true", help="GBM base learners (run_booster)")
    a = ap.parse_args()
    ctx = sb.default_context(0)
    t0 = time.time()
    n = fails = 0
    seed = a.start
    while n < a.cases and time.time() - t0 < 60 * a.minutes:
        t1 = time.time()
        ok, desc = run_booster(ctx, seed) if a.booster else run(ctx, seed, a.extra, a.big)
        n += 1
        fails += 0 if ok else 1
        print(("ok   " if ok else "FAIL ") + f"{time.time() - t1:6.1f}s " + desc, flush=True)
        seed += 1
    print(f"fuzz: {n} cases, {fails} failures, seeds {a.start}..{seed - 1}", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
