"""Replay one scripts/fuzz_parity.py case and print where the native forest and the
oracle part: the first differing node of each differing tree (fields and class stats)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import fuzz_parity as fz  # noqa: E402

np, nat, oracle, sb = fz.np, fz.nat, fz.oracle, fz.sb

seed = int(sys.argv[1])
X, y, cls, f64, part, p, kind = fz.draw(seed)
sd = oracle.DEFAULT_SEED_CLASSIFIER if cls else oracle.DEFAULT_SEED_REGRESSOR
N, F = X.shape
ctx = sb.default_context(0)
ds = nat.DeviceDataset.from_numpy(X, y, ctx)
forest = nat.fit(ctx, ds, replacement=p["replacement"], sample_ratio=p["ratio"], seed=sd,
                 learner_begin=0, learner_end=p["L"], partition_offsets=part,
                 max_depth=p["depth"], max_bins=p["bins"],
                 min_instances_per_node=p["min_inst"], min_info_gain=p["min_gain"],
                 impurity=nat.IMPURITY_GINI if cls else nat.IMPURITY_VARIANCE)
counts = oracle.bag(p["replacement"], p["ratio"], 0, p["L"], sd, part, N)
subs = [oracle.subspace(p["ratio"], F, sd + i) for i in range(p["L"])]
orf = fz.oracle_forest(X, y, counts, subs, p["depth"], p["bins"], cls, p["min_inst"], p["min_gain"],
                       part=part)
bad = 0
for t in range(p["L"]):
    nn, ns = forest.tree(t)
    on, os_ = orf.tree(t)
    # walk both trees from the root in the same order; report the first node that differs
    stack = [(0, 0, 0)]
    while stack:
        a, b, d = stack.pop()
        fa = {f: nn[f][a] for f in fz.__dict__.get("FIELDS", ("feature", "threshold", "gain", "impurity", "prediction", "left", "right"))}
        fb = {f: on[f][b] for f in fa}
        same = all((fa[f] == fb[f]) or (isinstance(fa[f], float) and np.isnan(fa[f]) and np.isnan(fb[f]))
                   for f in ("feature", "threshold", "gain", "impurity", "prediction"))
        leaf_a, leaf_b = nn["left"][a] < 0, on["left"][b] < 0
        if not same or leaf_a != leaf_b or (ns[a] != os_[b]).any():
            bad += 1
            print(f"tree {t} depth {d} node native {a} / oracle {b}")
            for f in ("feature", "threshold", "gain", "impurity", "prediction", "left", "right"):
                print(f"   {f:10s} {nn[f][a]!r:>28} {on[f][b]!r:>28}")
            print("   stats native", ns[a].tolist())
            print("   stats oracle", os_[b].tolist())
            break
        if not leaf_a:
            stack.append((int(nn["right"][a]), int(on["right"][b]), d + 1))
            stack.append((int(nn["left"][a]), int(on["left"][b]), d + 1))
print("trees with a differing node:", bad)
