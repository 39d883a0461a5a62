"""CPU check of the algebra behind k_poisson4 (the step-parallel Well19937c sampler).

k_poisson4 (spark-bagging_amd/csrc/sbag_poisson.hip) does not run a Well19937c stream
one step at a time.  A batch of B = LANES * SPL consecutive steps is spread over LANES lanes
(SPL steps per lane): every value a step reads from the state ring was written at least
70 steps earlier, except z4 of the previous step (AbstractWell's v0), and

    z4[n] = L(z4[n-1]) ^ c[n],   L(x) = x<<9 ^ x>>21 ^ (x & 0x7f)<<4

is F2-linear in z4[n-1] (c[n] depends only on older ring words).  The lanes therefore
scan z4 with the powers L^(SPL*2^k) (each a handful of shift/mask terms).  This test
replays exactly that schedule in Python, lane by lane, and compares every next(26)
output against the sequential restatement of commons-math3's Well19937c
(oracle/pyoracle.py, AbstractWell.setSeed / Well19937c.next).
"""
import pytest

import pyoracle

M32 = 0xFFFFFFFF


def L1(x):
    return ((x << 9) & M32) ^ (x >> 21) ^ ((x & 0x7F) << 4)


def lpow_terms(k):
    """(shift, mask) terms of L^k: L^k(x) = XOR over terms of (x & mask) shifted."""
    cols = []
    for i in range(32):
        x = 1 << i
        for _ in range(k):
            x = L1(x)
        cols.append(x)
    terms = {}
    for i in range(32):
        for j in range(32):
            if cols[i] >> j & 1:
                terms[j - i] = terms.get(j - i, 0) | (1 << i)
    return sorted(terms.items())


def lpow(terms, x):
    y = 0
    for s, m in terms:
        y ^= ((x & m) << s) & M32 if s >= 0 else (x & m) >> -s
    return y


def temper26(z4):
    z4 ^= ((z4 << 7) & M32) & 0xE46E1700
    z4 ^= ((z4 << 15) & M32) & 0x9B868000
    return z4 >> 6


def step_parallel_outputs(seed, nsteps, spl, lanes=16):
    """next(26) outputs of the stream seeded `seed`, batch by batch as the kernel does
    (k_poisson4: 8 lanes x 8 steps, 16 x 4, 4 x 16; smaller batches check the algebra too)."""
    g = pyoracle.Well19937c(seed)  # only for the seeded initial ring
    st = list(g.v)
    B = lanes * spl
    T = {k: lpow_terms(k) for k in (spl * (1 << d) for d in range(5))}
    carry = st[0]  # z4 "before" step 0 is v[0]
    i = 0
    out = []
    while len(out) < nsteps:
        a = [[0] * spl for _ in range(lanes)]
        z2 = [[0] * spl for _ in range(lanes)]
        c = [[0] * spl for _ in range(lanes)]
        pos = [[0] * spl for _ in range(lanes)]
        for t in range(lanes):  # every read of the batch comes before any write
            for q in range(spl):
                j = (i - (spl * t + q)) % 624
                m1, m2, m3 = st[(j + 70) % 624], st[(j + 179) % 624], st[(j + 449) % 624]
                hb, lo = st[(j + 623) % 624], st[(j + 622) % 624]
                a[t][q] = m1 ^ (m1 >> 27)
                z2[t][q] = (m2 >> 9) ^ m3 ^ (m3 >> 1)
                z0 = (hb & 0x80000000) | (lo & 0x7FFFFFFF)
                S = ((a[t][q] << 9) & M32) ^ (a[t][q] >> 21)
                c[t][q] = S ^ z0 ^ ((z2[t][q] << 21) & M32) ^ (z2[t][q] >> 21)
                pos[t][q] = j
        # lane transfer C_t (Horner), carry folded into lane 0, Hillis-Steele scan
        C = []
        for t in range(lanes):
            x = c[t][0]
            for q in range(1, spl):
                x = L1(x) ^ c[t][q]
            C.append(x)
        C[0] ^= lpow(T[spl], carry)
        for d in (d for d in (1, 2, 4, 8) if d < lanes):
            C = [C[t] ^ (lpow(T[spl * d], C[t - d]) if t >= d else 0) for t in range(lanes)]
        for t in range(lanes):
            y = carry if t == 0 else C[t - 1]
            for q in range(spl):
                z3 = y ^ ((y << 25) & M32) ^ a[t][q] ^ z2[t][q]
                st[pos[t][q]] = z3
                y = L1(y) ^ c[t][q]
                out.append(temper26(y))
            assert y == C[t]
        carry = C[lanes - 1]
        i = (i - B) % 624
    return out[:nsteps]


@pytest.mark.parametrize("lanes,spl", [(16, 1), (16, 2), (16, 4), (8, 8), (4, 16)])
@pytest.mark.parametrize("seed", [0, 42, -1395689524 + 7, (1 << 40) + 3])
def test_step_parallel_well_matches_sequential(seed, lanes, spl):
    n = 3 * 624 + 100  # several trips round the ring, both wrap cases of every window
    got = step_parallel_outputs(seed, n, spl, lanes)
    g = pyoracle.Well19937c(seed)
    want = [g.next(26) for _ in range(n)]
    assert got == want


def test_lpow_terms_are_few():
    # the kernel applies L^(SPL*2^k) as shift/mask terms: keep them cheap
    for k in (1, 2, 4, 8, 16, 32, 64):
        assert len(lpow_terms(k)) <= 6
