#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run from the repo root).

PARITY UNPINNED: the reference ships no golden vectors and cannot run here (no JVM,
SURVEY.md §8c).  These fixtures are produced by the C oracle and cross-checked,
while generating, against the independent pure-Python restatement
(oracle/pyoracle.py); they pin the oracle (and through it the HIP path) against
regressions.  Inputs: the reference's own workloads data/cpusmall and data/vehicle
(copied to tests/golden/data) and the deterministic synthetic generator.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
import pyoracle as po  # noqa: E402
import sbag_loader  # noqa: E402

sb = sbag_loader.load()
OUT = os.path.join(ROOT, "tests", "golden")
SEED_REG, SEED_CLS = oracle.DEFAULT_SEED_REGRESSOR, oracle.DEFAULT_SEED_CLASSIFIER


def rng_fixtures():
    seeds = [0, 1, -1, 42, SEED_REG, SEED_CLS, 2**40 + 7, -(2**63), 2**63 - 1]
    out = {"seeds": seeds, "hash_seed": [], "xorshift_doubles": [], "xorshift_int": [],
           "well_doubles": [], "poisson": {}}
    for s in seeds:
        out["hash_seed"].append(str(oracle.hash_seed(s)))
        d = oracle.xorshift_doubles(s, 8)
        r = po.XORShiftRandom(s)
        assert list(d) == [r.next_double() for _ in range(8)]
        out["xorshift_doubles"].append([float(x).hex() for x in d])
        out["xorshift_int"].append([int(x) for x in oracle.xorshift_next(s, 32, 8)])
        w = oracle.well_doubles(s, 8)
        ww = po.Well19937c(s)
        assert list(w) == [ww.next_double() for _ in range(8)]
        out["well_doubles"].append([float(x).hex() for x in w])
    for lam in [1.0, 0.7, 0.5, 0.05]:
        out["poisson"][repr(lam)] = {str(s): [int(x) for x in oracle.poisson(lam, s, 64)]
                                     for s in seeds[:6]}
        g = po.poisson_stream(lam, SEED_REG)
        assert out["poisson"][repr(lam)][str(SEED_REG)] == [next(g) for _ in range(64)]
    # published Spark 2.x XORShiftRandom(seed).nextDouble() values (hashSeed over 64 bytes)
    out["spark2_anchors"] = {"0": 0.8446490682263027, "30": 0.31429268272540556,
                             "5419823303878592871": 0.2304755080444375}
    for s, want in out["spark2_anchors"].items():
        assert oracle.xorshift_doubles(int(s), 1)[0] == want, s
    with open(os.path.join(OUT, "rng.json"), "w") as fh:
        json.dump(out, fh, indent=0)


def forest_fixture(name, X, y, L, replacement, ratio, seed, depth, bins, cls, part=None):
    N, F = X.shape
    off = part if part is not None else [0, N]
    counts = oracle.bag(replacement, ratio, 0, L, seed, off, N)
    subs = [oracle.subspace(ratio, F, seed + i) for i in range(L)]
    f = oracle.fit(X, y, counts, subs, max_depth=depth, max_bins=bins, classification=cls)
    # cross-check two trees against the pure-Python restatement
    for t in range(min(L, 2)):
        nodes, stats = f.tree(t)
        pt = po.fit_tree(X.tolist(), y.tolist(), counts[t].tolist(), list(subs[t]),
                         max_depth=depth, max_bins=bins, gini=cls)
        assert len(pt) == len(nodes)
        for a, b in zip(nodes, pt):
            for k in ("left", "right", "feature", "threshold", "prediction", "impurity", "gain"):
                assert a[k] == b[k], (name, t, k)
    pred = oracle.predict(f, X, classification=cls)
    nn = f.num_nodes
    nodes = np.concatenate([f.tree(t)[0] for t in range(L)])
    stats = [f.tree(t)[1] for t in range(L)]
    ns = max(s.shape[1] for s in stats)
    stats = np.concatenate([np.pad(s, ((0, 0), (0, ns - s.shape[1]))) for s in stats])
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), counts=counts,
                        subspaces=np.array([np.pad(s, (0, F - len(s)), constant_values=-1)
                                            for s in subs], np.int32),
                        num_nodes=nn, num_stats=f.num_stats, nodes=nodes, stats=stats,
                        prediction=pred,
                        params=np.array([L, int(replacement), ratio, seed, depth, bins, int(cls)],
                                        np.float64),
                        partitions=np.array(off, np.int64))


def main():
    rng_fixtures()
    X, y = sb.load_libsvm(os.path.join(OUT, "data", "cpusmall.svm"))
    forest_fixture("cpusmall_c1", X, y, 10, True, 1.0, SEED_REG, 5, 32, False)
    Xv, yv = sb.load_libsvm(os.path.join(OUT, "data", "vehicle.svm"))
    forest_fixture("vehicle_c2", Xv, yv, 32, False, 1.0, SEED_CLS, 5, 32, True)
    forest_fixture("vehicle_repl07", Xv, yv, 32, True, 0.7, SEED_CLS, 6, 32, True)
    from spark_bagging_amd import synthetic
    Xs, ys = synthetic.generate(6000, 12, seed=3)
    forest_fixture("synth_p3", Xs, ys, 4, True, 1.0, SEED_REG, 6, 32, False,
                   part=[0, 1000, 3500, 6000])
    Xc, yc = synthetic.generate(5000, 10, seed=4, num_classes=6)
    forest_fixture("synth_bern", Xc, yc, 4, False, 0.5, SEED_CLS, 5, 16, True,
                   part=[0, 2500, 5000])
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
