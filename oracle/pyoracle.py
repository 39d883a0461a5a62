"""Pure-Python restatement of the bagging hot path (TEST INFRASTRUCTURE ONLY).

Second, independent restatement used to cross-check oracle/sbag_oracle.c on small
inputs.  PARITY UNPINNED: the reference ships no golden vectors for this path
 and no JVM exists here to run it.

Reference call sites (relative to /root/reference/core/src/main/scala/org/apache/spark/):
  bag                sql/bfunctions.scala:46-68
  Poisson            sql/catalyst/expressions/Poisson.scala:53-56,73
  mkSubspace         ml/ensemble/HasSubBag.scala:90-106
  extractSubBag      ml/ensemble/HasSubBag.scala:108-126 (rows replicated `count` times)
  fitBaseLearner     ml/ensemble/ensembleParams.scala:99-117 -> Spark 2.4.3 DecisionTree
  predict (mean)     ml/regression/BaggingRegressor.scala:248-256
  predict (mode)     ml/classification/BaggingClassifier.scala:248-257
Upstream arithmetic restated from SURVEY.md Appendix A.
"""
import math
import struct

import fastmath

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF
DOUBLE_MIN_VALUE = -1.7976931348623157e308  # Scala Double.MinValue


def _i32(x):
    x &= M32
    return x - (1 << 32) if x & 0x80000000 else x


def _i64(x):
    x &= M64
    return x - (1 << 64) if x & (1 << 63) else x


# ---------------------------------------------------------------- MurmurHash3
def _rotl(x, r):
    x &= M32
    return ((x << r) | (x >> (32 - r))) & M32


def _mix_last(h, k):
    k = (k * 0xCC9E2D51) & M32
    k = _rotl(k, 15)
    k = (k * 0x1B873593) & M32
    return (h ^ k) & M32


def _mix(h, k):
    h = _mix_last(h, k)
    h = _rotl(h, 13)
    return (h * 5 + 0xE6546B64) & M32


def bytes_hash(data, seed):
    """scala.util.hashing.MurmurHash3.bytesHash"""
    h = seed & M32
    n = len(data)
    i = 0
    while n - i >= 4:
        k = data[i] | (data[i + 1] << 8) | (data[i + 2] << 16) | (data[i + 3] << 24)
        h = _mix(h, k)
        i += 4
    rest = n - i
    k = 0
    if rest == 3:
        k ^= data[i + 2] << 16
    if rest >= 2:
        k ^= data[i + 1] << 8
    if rest >= 1:
        k ^= data[i]
        h = _mix_last(h, k)
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def hash_seed(seed):
    """XORShiftRandom.hashSeed (Spark 2.4.3).

    `ByteBuffer.allocate(java.lang.Long.SIZE).putLong(seed)`: Long.SIZE = 64 is a bit count
    used as a byte count, so 64 bytes are hashed -- the big-endian seed and 56 zero bytes
    (Spark 3.0 hashes 8). Anchors: tests/test_oracle.py::test_xorshift_spark2_anchors.
    """
    b = struct.pack(">q", _i64(seed)) + bytes(56)
    lo = bytes_hash(b, 0x3C074A61)
    hi = bytes_hash(b, lo)
    return ((hi << 32) | lo) & M64


class XORShiftRandom:
    def __init__(self, seed):
        self.s = hash_seed(seed)

    def next(self, bits):
        s = self.s
        s ^= (s << 21) & M64
        s ^= s >> 35
        s ^= (s << 4) & M64
        self.s = s
        return _i32(s & ((1 << bits) - 1))

    def next_int(self):
        return self.next(32)

    def next_double(self):
        a = self.next(26)
        b = self.next(27)
        return float((a << 27) + b) * 2.0 ** -53


class Well19937c:
    R = 624

    def __init__(self, seed):
        seed = _i64(seed)
        v = [0] * self.R
        v[0] = (seed >> 32) & M32
        v[1] = seed & M32
        for i in range(2, self.R):
            l = _i32(v[i - 2])
            v[i] = ((1812433253 * (l ^ (l >> 30)) + i) & M64) & M32
        self.v = v
        self.index = 0

    def next(self, bits):
        v, i, R = self.v, self.index, self.R
        rm1, rm2 = (i + R - 1) % R, (i + R - 2) % R
        v0, m1, m2, m3 = v[i], v[(i + 70) % R], v[(i + 179) % R], v[(i + 449) % R]
        z0 = (0x80000000 & v[rm1]) ^ (0x7FFFFFFF & v[rm2])
        z1 = (v0 ^ ((v0 << 25) & M32)) ^ (m1 ^ (m1 >> 27))
        z2 = (m2 >> 9) ^ (m3 ^ (m3 >> 1))
        z3 = z1 ^ z2
        z4 = z0 ^ (z1 ^ ((z1 << 9) & M32)) ^ (z2 ^ ((z2 << 21) & M32)) ^ (z3 ^ (z3 >> 21))
        v[i] = z3
        v[rm1] = z4
        v[rm2] &= 0x80000000
        self.index = rm1
        z4 ^= ((z4 << 7) & M32) & 0xE46E1700
        z4 ^= ((z4 << 15) & M32) & 0x9B868000
        return _i32(z4 >> (32 - bits))

    def next_double(self):
        high = self.next(26) << 26
        low = self.next(26)
        return float(high | low) * 2.0 ** -52


def poisson_stream(mean, seed):
    """PoissonDistribution(mean) reseeded with `seed`; yields sample() values."""
    rng = Well19937c(seed)
    p = fastmath.exp(-mean)  # FastMath.exp, not libm (oracle/fastmath.py)
    while True:
        n = 0
        r = 1.0
        while n < 1000 * mean:
            r *= rng.next_double()
            if r >= p:
                n += 1
            else:
                break
        yield n


# ---------------------------------------------------------------- bag, subspace
def bag(replacement, ratio, learners, seed, part_off):
    """list (per learner in `learners`) of per-row counts"""
    if not ratio > 0:
        raise ValueError("sampleRatio must be strictly positive")
    out = []
    for i in learners:
        row = []
        for p in range(len(part_off) - 1):
            nrows = part_off[p + 1] - part_off[p]
            if replacement:
                g = poisson_stream(ratio, _i64(seed + i + p))
                row += [next(g) for _ in range(nrows)]
            elif ratio == 1:
                row += [1] * nrows
            else:
                if ratio > 1:
                    raise ValueError("Without replacement, the sampleRatio cannot be greater to one")
                if -(1 << 31) <= seed < (1 << 31):
                    rs = _i32(seed + i) + p
                else:
                    rs = _i64(seed + i + p)
                rng = XORShiftRandom(rs)
                row += [1 if rng.next_double() < ratio else 0 for _ in range(nrows)]
        out.append(row)
    return out


def subspace(ratio, nfeat, seed):
    if ratio == 1:
        return list(range(nfeat))
    rng = XORShiftRandom(seed)
    return [f for f in range(nfeat) if rng.next_double() < ratio]


# ---------------------------------------------------------------- split-finding sample
class JavaRandom:
    """java.util.Random (48-bit LCG)."""

    def __init__(self, seed):
        self.s = (seed ^ 0x5DEECE66D) & ((1 << 48) - 1)

    def next(self, bits):
        self.s = (self.s * 0x5DEECE66D + 0xB) & ((1 << 48) - 1)
        return _i32(self.s >> (48 - bits))

    def next_long(self):
        return _i64((self.next(32) << 32) + self.next(32))


def split_sample_fraction(num_examples, max_bins):
    """RandomForest.samplesFractionForFindSplits (metadata.maxBins = min(maxBins, n))."""
    mpb = min(max_bins, num_examples)
    required = max(mpb * mpb, 10000)
    return required / num_examples if required < num_examples else 1.0


def split_sample(counts_row, part_off, dt_seed, fraction):
    """RDD.sample(false, fraction, new XORShiftRandom(seed).nextInt()) over the exploded
    subbag: per-partition java.util.Random seeds, BernoulliSampler with GapSampling
    (fraction <= 0.4) or a nextDouble test per item.  Returns the multiplicity per row."""
    import math
    jr = JavaRandom(XORShiftRandom(dt_seed).next_int())
    mult = [0] * len(counts_row)
    for p in range(len(part_off) - 1):
        rng = XORShiftRandom(jr.next_long())
        if fraction <= 0.4:
            lnq = math.log1p(-fraction)
            cfd = None
            for r in range(part_off[p], part_off[p + 1]):
                for _ in range(int(counts_row[r])):
                    if cfd is None:  # lazy GapSampling: construction draws the first gap
                        cfd = int(math.log(max(rng.next_double(), 5e-11)) / lnq)
                    if cfd > 0:
                        cfd -= 1
                    else:
                        cfd = int(math.log(max(rng.next_double(), 5e-11)) / lnq)
                        mult[r] += 1
        else:
            for r in range(part_off[p], part_off[p + 1]):
                for _ in range(int(counts_row[r])):
                    if rng.next_double() <= fraction:
                        mult[r] += 1
    return mult


# ---------------------------------------------------------------- DecisionTree
def find_splits(values_with_mult, n, max_bins, num_samples=None):
    """RandomForest.findSplitsForContinuousFeature on the whole subbag.

    values_with_mult: dict value -> multiplicity over the replicated subbag (all values).
    """
    nonzero = {v: c for v, c in values_with_mult.items() if v != 0.0}
    if not nonzero:
        return []
    num_splits = min(max_bins, n) - 1
    if num_samples is None:
        num_samples = n
    part = sum(nonzero.values())
    vc = dict(nonzero)
    if num_samples - part > 0:
        vc[0.0] = num_samples - part
    vals = sorted(vc.items())
    possible = len(vals) - 1
    if possible == 0:
        return []
    if possible <= num_splits:
        return [(vals[i - 1][0] + vals[i][0]) / 2.0 for i in range(1, possible + 1)]
    stride = num_samples / (num_splits + 1)
    out = []
    cur = vals[0][1]
    target = stride
    for i in range(1, len(vals)):
        prev = cur
        cur += vals[i][1]
        if abs(prev - target) < abs(cur - target):
            out.append((vals[i - 1][0] + vals[i][0]) / 2.0)
            target += stride
    return out


def _impurity(s, gini):
    if not gini:
        cnt, sm, sq = s
        if cnt == 0:
            return 0.0
        return (sq - (sm * sm) / cnt) / cnt
    tot = 0.0
    for c in s:
        tot += c
    if tot == 0:
        return 0.0
    imp = 1.0
    for c in s:
        f = c / tot
        imp -= f * f
    return imp


def _count(s, gini):
    if not gini:
        return int(s[0])
    t = 0.0
    for c in s:
        t += c
    return int(t)


def _predict(s, gini):
    if _count(s, gini) == 0:
        return 0.0
    if not gini:
        return s[1] / _count(s, gini)
    best, bv = -1, DOUBLE_MIN_VALUE
    for i, c in enumerate(s):
        if c > bv:
            best, bv = i, c
    return float(best)


def fit_tree(X, y, counts, sub, max_depth=5, max_bins=32, min_inst=1, min_gain=0.0, gini=False,
             part_off=None):
    """One base learner on the replicated subbag; returns the pruned tree as a list of
    NodeData dicts in pre-order (id, prediction, impurity, gain, left, right, feature,
    threshold, stats).  part_off: the partitions' row offsets -- each partition sums its own
    rows in row order and the partials are merged in partition order (RandomForest
    .findBestSplits: mapPartitions + reduceByKey(_ merge _)); None: one partition."""
    if part_off is None:
        part_off = [0, len(counts)]
    rows = [r for r in range(len(counts)) if counts[r] > 0]
    n = sum(counts[r] for r in rows)
    if n == 0:
        raise ValueError("empty subbag")
    ns = 3 if not gini else int(max(y[r] for r in rows)) + 1
    Fr = len(sub)
    thr = []
    for f in sub:
        mult = {}
        for r in rows:
            mult[X[r][f]] = mult.get(X[r][f], 0) + counts[r]
        thr.append(find_splits(mult, n, max_bins))
    binned = {r: [sum(1 for t in thr[fl] if t < X[r][sub[fl]]) for fl in range(Fr)] for r in rows}
    nodes = {1: dict(leaf=False, stats=None)}
    where = {r: 1 for r in rows}
    for level in range(max_depth + 1):
        active = [h for h in sorted(nodes) if (1 << level) <= h < (2 << level)
                  and not nodes[h]["leaf"]]
        if not active:
            break
        agg = {h: [[[0.0] * ns for _ in range(max_bins)] for _ in range(Fr)] for h in active}
        par = {h: [0.0] * ns for h in active}
        for q in range(len(part_off) - 1):
            # partition q's DTStatsAggregator per node, then a.merge(b) in partition order
            pagg = {h: [[[0.0] * ns for _ in range(max_bins)] for _ in range(Fr)] for h in active}
            ppar = {h: [0.0] * ns for h in active}
            for r in rows:
                if not part_off[q] <= r < part_off[q + 1]:
                    continue
                h = where[r]
                if h not in pagg:
                    continue
                for _ in range(counts[r]):
                    for fl in range(Fr):
                        st = pagg[h][fl][binned[r][fl]]
                        if gini:
                            st[int(y[r])] += 1.0
                        else:
                            st[0] += 1.0
                            st[1] += 1.0 * y[r]
                            st[2] += 1.0 * y[r] * y[r]
                    if gini:
                        ppar[h][int(y[r])] += 1.0
                    else:
                        ppar[h][0] += 1.0
                        ppar[h][1] += 1.0 * y[r]
                        ppar[h][2] += 1.0 * y[r] * y[r]
            for h in active:
                for fl in range(Fr):
                    for b in range(max_bins):
                        for i in range(ns):
                            agg[h][fl][b][i] += pagg[h][fl][b][i]
                for i in range(ns):
                    par[h][i] += ppar[h][i]
        for h in active:
            node = nodes[h]
            chain = None if level == 0 else (node["stats"]["calc"], node["stats"]["impurity"])
            best = None
            for fl in range(Fr):
                nsp = len(thr[fl])
                if nsp == 0:
                    continue
                a = agg[h][fl]
                for s in range(nsp):
                    a[s + 1] = [a[s + 1][i] + a[s][i] for i in range(ns)]
                fbest = None
                for s in range(nsp):
                    left = list(a[s])
                    right = [a[nsp][i] - left[i] for i in range(ns)]
                    if chain is None:
                        calc = [left[i] + right[i] for i in range(ns)]
                        chain = (calc, _impurity(calc, gini))
                    lc, rc = _count(left, gini), _count(right, gini)
                    if lc < min_inst or rc < min_inst:
                        gain, valid = DOUBLE_MIN_VALUE, False
                    else:
                        li, ri = _impurity(left, gini), _impurity(right, gini)
                        gain = chain[1] - (lc / float(lc + rc)) * li - (rc / float(lc + rc)) * ri
                        valid = True
                        if gain < min_gain:
                            gain, valid = DOUBLE_MIN_VALUE, False
                    if fbest is None or gain > fbest[0]:
                        fbest = (gain, s, valid, left, right)
                if best is None or fbest[0] > best[0]:
                    best = (fbest[0], fl, fbest[1], fbest[2], fbest[3], fbest[4])
            if best is None:
                calc = par[h]
                node["stats"] = dict(gain=DOUBLE_MIN_VALUE, impurity=_impurity(calc, gini),
                                     calc=calc, valid=False)
                node["leaf"] = True
                continue
            gain, fl, s, valid, left, right = best
            node["stats"] = dict(gain=gain, impurity=chain[1], calc=chain[0], valid=valid)
            if gain <= 0 or level == max_depth:
                node["leaf"] = True
                continue
            node["split"] = (fl, s, thr[fl][s])
            child_leaf = level + 1 == max_depth
            for cid, cs in ((2 * h, left), (2 * h + 1, right)):
                imp = _impurity(cs, gini)
                nodes[cid] = dict(leaf=child_leaf or imp == 0.0,
                                  stats=dict(gain=float("nan"), impurity=imp, calc=cs, valid=True))
        for r in rows:
            h = where[r]
            if "split" in nodes[h] and (1 << level) <= h < (2 << level):
                fl, s, _ = nodes[h]["split"]
                where[r] = 2 * h if binned[r][fl] <= s else 2 * h + 1

    out = []

    def build(h):
        node = nodes[h]
        idx = len(out)
        out.append(None)
        st = node["stats"]
        if "split" in node:
            mark = len(out)
            lid, lleaf, lpred = build(2 * h)
            rid, rleaf, rpred = build(2 * h + 1)
            if lleaf and rleaf and lpred == rpred:
                del out[mark:]
                out[idx] = dict(id=idx, prediction=lpred, impurity=st["impurity"], gain=-1.0,
                                left=-1, right=-1, feature=-1, threshold=0.0, stats=list(st["calc"]))
                return idx, True, lpred
            fl, s, t = node["split"]
            pred = _predict(st["calc"], gini)
            out[idx] = dict(id=idx, prediction=pred, impurity=st["impurity"], gain=st["gain"],
                            left=lid, right=rid, feature=fl, threshold=t, stats=list(st["calc"]))
            return idx, False, pred
        pred = _predict(st["calc"], gini)
        out[idx] = dict(id=idx, prediction=pred, impurity=st["impurity"] if st["valid"] else -1.0,
                        gain=-1.0, left=-1, right=-1, feature=-1, threshold=0.0,
                        stats=list(st["calc"]))
        return idx, True, pred

    build(1)
    return out


def predict_tree(tree, x_sliced):
    i = 0
    while tree[i]["left"] >= 0:
        i = tree[i]["left"] if x_sliced[tree[i]["feature"]] <= tree[i]["threshold"] else tree[i]["right"]
    return tree[i]["prediction"]


def predict_ensemble(trees, subs, x, mode):
    votes = [predict_tree(t, [x[f] for f in s]) for t, s in zip(trees, subs)]
    if not mode:
        tot = 0.0
        for v in votes:
            tot += v
        return tot / len(votes)
    counts, maxc, best = {}, 0, 0.0
    for v in votes:
        counts[v] = counts.get(v, 0) + 1
        if counts[v] > maxc:
            maxc, best = counts[v], v
    return best
