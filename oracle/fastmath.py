"""Restatement of commons-math3 3.4.1 `FastMath.exp` (TEST INFRASTRUCTURE ONLY).

The Poisson bag of the reference (sql/catalyst/expressions/Poisson.scala:53-56,73) draws
with `PoissonDistribution.sample()` -> `nextPoisson(mean)`, whose small-mean branch compares
the running product of uniforms with `p = FastMath.exp(-mean)`. The engine and the C oracle
compute p with libm `exp`. This module restates FastMath's algorithm so that
tests/test_fastmath.py can show the two agree bit for bit on every mean the configurations
and tests use (SURVEY App-A.2 [verify]).

FastMath.exp(x, extra = 0, hiPrec = null), x in (-709, 0):
    intVal = (int) x - 1                                  (x < 0 branch: intVal--)
    intPartA/B = EXP_INT_TABLE_A/B[750 + intVal]           exp(intVal), split hi/lo
    intFrac = (int) ((x - intVal) * 1024.0)
    fracPartA/B = EXP_FRAC_TABLE_A/B[intFrac]              exp(intFrac/1024), split hi/lo
    epsilon = x - (intVal + intFrac / 1024.0)
    z = Remez polynomial for exp(epsilon) - 1 (coefficients below)
    tempA = intPartA * fracPartA                           (exact: both halves are short)
    tempB = intPartA * fracPartB + intPartB * fracPartA + intPartB * fracPartB
    tempC = tempB + tempA
    result = tempC * z + tempB + tempA

The tables are literal arrays in commons-math3 (FastMathLiteralArrays), produced by
FastMathCalc in double-double arithmetic; they are not available offline. Here every entry
is the FastMathCalc.split() of the value computed with 50-digit decimal arithmetic:
hi = (v + v * 2^30) - v * 2^30 of the double nearest v, lo = the double nearest v - hi.
A table entry that differs from commons-math3's in lo's last bits moves the result by
about 2^-76 relative; `margin_ulps` measures how far the exact exp(x) lies from the
rounding boundary between two doubles, so a result whose margin is far above that (and
above the Remez polynomial's error, ~2^-63 relative) is the same double under any such
table and equals the correctly rounded exp(x).
"""
import decimal
import struct

_D = decimal.Context(prec=50)

EXP_INT_TABLE_MAX_INDEX = 750
_TWO30 = float(2 ** 30)


def _split(v):
    """FastMathCalc.split: hi keeps the top ~22 bits of the double nearest v."""
    d = float(v)
    a = d * _TWO30
    hi = (d + a) - a
    lo = float(_D.subtract(v, decimal.Decimal(hi)))
    return hi, lo


def _exp_dec(x):
    return _D.exp(decimal.Decimal(x))


_int_cache = {}
_frac_cache = {}


def _int_entry(i):
    if i not in _int_cache:
        _int_cache[i] = _split(_exp_dec(i))
    return _int_cache[i]


def _frac_entry(k):
    if k not in _frac_cache:
        _frac_cache[k] = _split(_exp_dec(decimal.Decimal(k) / 1024))
    return _frac_cache[k]


def exp(x):
    """FastMath.exp for -709 < x < 0 (the branch nextPoisson reaches with 0 < mean < 40)."""
    x = float(x)
    if not (-709.0 < x < 0.0):
        raise ValueError("restated for -709 < x < 0 only")
    int_val = int(x)  # Java (int) truncates toward zero
    int_val -= 1
    ia, ib = _int_entry(int_val)
    int_frac = int((x - int_val) * 1024.0)
    fa, fb = _frac_entry(int_frac)
    epsilon = x - (int_val + int_frac / 1024.0)
    z = 0.04168701738764507
    z = z * epsilon + 0.1666666505023083
    z = z * epsilon + 0.5000000000042687
    z = z * epsilon + 1.0
    z = z * epsilon + -3.940510424527919e-20
    temp_a = ia * fa
    temp_b = ia * fb + ib * fa + ib * fb
    temp_c = temp_b + temp_a
    return temp_c * z + temp_b + temp_a


def correctly_rounded_exp(x):
    return float(_exp_dec(float(x)))


def margin_ulps(x):
    """Distance, in ulps of the result, from the exact exp(x) to the nearest rounding
    boundary (midpoint between adjacent doubles). Large means every evaluation whose error
    is far below that many ulps rounds to the same double."""
    v = _exp_dec(float(x))
    r = float(v)
    bits = struct.unpack("<q", struct.pack("<d", r))[0]
    up = struct.unpack("<d", struct.pack("<q", bits + 1))[0]
    ulp = _D.subtract(decimal.Decimal(up), decimal.Decimal(r))
    dist = abs(_D.subtract(v, decimal.Decimal(r)))
    half = ulp / 2
    return float((half - dist) / ulp)


__all__ = ["exp", "correctly_rounded_exp", "margin_ulps"]
