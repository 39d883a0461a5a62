"""Fit one scripts/fuzz_parity.py case several times per engine switch (set between fits in
one process) and report, per run, the trees that differ from the oracle and from run 0."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import fuzz_parity as fz  # noqa: E402

np, nat, oracle, sb = fz.np, fz.nat, fz.oracle, fz.sb
seed, reps = int(sys.argv[1]), int(sys.argv[2])
switches = sys.argv[3:] or ["none"]
X, y, cls, f64, part, p, kind = fz.draw(seed)
sd = oracle.DEFAULT_SEED_CLASSIFIER if cls else oracle.DEFAULT_SEED_REGRESSOR
N, F = X.shape
ctx = sb.default_context(0)
ds = nat.DeviceDataset.from_numpy(X, y, ctx)
counts = oracle.bag(p["replacement"], p["ratio"], 0, p["L"], sd, part, N)
subs = [oracle.subspace(p["ratio"], F, sd + i) for i in range(p["L"])]
orf = fz.oracle_forest(X, y, counts, subs, p["depth"], p["bins"], cls, p["min_inst"], p["min_gain"],
                       part=part)
ref = [orf.tree(t)[0].tobytes() for t in range(p["L"])]
for sw in switches:
    if sw != "none":
        k, v = sw.split("=")
        os.environ[k] = v
    first = None
    for rep in range(reps):
        forest = nat.fit(ctx, ds, replacement=p["replacement"], sample_ratio=p["ratio"], seed=sd,
                         learner_begin=0, learner_end=p["L"], partition_offsets=part,
                         max_depth=p["depth"], max_bins=p["bins"],
                         min_instances_per_node=p["min_inst"], min_info_gain=p["min_gain"],
                         impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
        got = [forest.tree(t)[0].tobytes() for t in range(p["L"])]
        forest.free()
        first = first or got
        print(sw, "rep", rep, "vs oracle:", [t for t in range(p["L"]) if got[t] != ref[t]],
              "vs rep 0:", [t for t in range(p["L"]) if got[t] != first[t]], flush=True)
    if sw != "none":
        del os.environ[k]
