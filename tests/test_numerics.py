"""The device-side elementary functions of the hot path, restated in Python
(exact fma through fractions) and checked against a 120-bit reference:
log_fast (nemo_internal.h) and exp_lse (nemo_factored.hip / _i8.hip), plus
the fixed-point digit expansion of the int8 factored kernel."""
import math
from fractions import Fraction

import numpy as np
import pytest

mpmath = pytest.importorskip("mpmath")
mpmath.mp.prec = 120


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


LN2_HI = float.fromhex("0x1.62e42fefa3800p-1")
LN2_LO = 5.4956039718945254e-14
INV = [1.0 / (1.0 + (k + 0.5) / 128.0) for k in range(128)]
LTAB = [(v, -math.log(v)) for v in INV]


def log_fast(x):
    bits = np.float64(x).view(np.uint64)
    hi = int(bits >> np.uint64(32))
    k = ((hi >> 20) & 0x7FF) - 1023
    m = float(np.uint64((int(bits) & 0x000FFFFFFFFFFFFF) | 0x3FF0000000000000).view(np.float64))
    inv, lj = LTAB[(hi >> 13) & 127]
    r = fma(m, inv, -1.0)
    p = fma(r, -1.0 / 6.0, 0.2)
    p = fma(r, p, -0.25)
    p = fma(r, p, 1.0 / 3.0)
    p = fma(r, p, -0.5)
    p = fma(r, p, 1.0)
    p *= r
    return fma(k, LN2_HI, lj) + fma(k, LN2_LO, p)


ETAB = [2.0 ** (j / 256.0) for j in range(256)]


def exp_lse(x):
    t = fma(x, 369.32993046757462707, 6755399441055744.0)
    kf = t - 6755399441055744.0
    k = int(kf)
    r = fma(-kf, 2.7076061740622862e-03, x)
    p = fma(r, 1.0 / 24.0, 1.0 / 6.0)
    p = fma(r, p, 0.5)
    p = fma(r, p, 1.0)
    p = fma(r, p, 1.0)
    return math.ldexp(p * ETAB[k & 255], k >> 8)


def test_log_fast_within_one_ulp():
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(1e-3, 1, 400), rng.uniform(1, 40, 400),
                         np.exp(rng.uniform(-170, 170, 400)), 1 + rng.uniform(-1e-4, 1e-4, 200)])
    worst = 0.0
    for x in xs:
        ref = mpmath.log(mpmath.mpf(float(x)))
        err = abs(mpmath.mpf(log_fast(float(x))) - ref) / max(abs(float(ref)), 0.5)
        worst = max(worst, float(err) / 2.0 ** -52)
    assert worst <= 1.1  # ulps of max(|log x|, 0.5)


def test_exp_lse_relative_error():
    rng = np.random.default_rng(1)
    xs = np.concatenate([-rng.exponential(3.0, 600), rng.uniform(-700, 0, 300), [0.0, -1e-300]])
    worst = 0.0
    for x in xs:
        ref = mpmath.exp(mpmath.mpf(float(x)))
        if ref < mpmath.mpf(2) ** -1000:
            continue
        rel = abs(mpmath.mpf(exp_lse(float(x))) - ref) / ref
        # single-constant reduction: error ~ |x| * 1.6e-16, weighted by e^x in the LSE
        worst = max(worst, float(rel) / (1.0 + abs(float(x))))
    assert worst <= 4e-16


def test_int8_digit_expansion_exact():
    """Delta = 2^(c-6) * sum_s d_s 64^-s with |d_s| <= 32 and a truncation of
    at most 2^(c-6) * 64^-7 / 2 = 2^(c-49), as score_i8_kernel builds it
    (c = per-model scale)."""
    rng = np.random.default_rng(2)
    for c in (0, 3, 4, 7):
        for d in rng.uniform(-1, 1, 300) * 2.0 ** (c - 1):
            x = math.ldexp(d, 6 - c)
            digits = []
            for _ in range(8):
                q = float(np.rint(x))
                digits.append(int(q))
                x = (x - q) * 64.0
            assert all(abs(q) <= 32 for q in digits)
            back = sum(Fraction(q) * Fraction(64) ** -s for s, q in enumerate(digits)) * Fraction(2) ** (c - 6)
            assert abs(back - Fraction(d)) <= Fraction(2) ** (c - 49)
            # pairs (64 d_2t + d_2t+1) and the int32 recombination stay exact
            pairs = [64 * digits[2 * t] + digits[2 * t + 1] for t in range(4)]
            assert all(abs(v) * 64 < 2 ** 18 for v in pairs)
