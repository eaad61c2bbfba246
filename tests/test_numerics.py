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


# --- score_i8l_kernel (nemo_factored_i8.hip): log2 fixed point -------------
L2_SCALE = 1512775.3951951857          # 2^20 / ln 2 (kL2Scale)
L2_C = (1.0000000000000377, 2.521654728528023e-12, 3.179908378901339e-24)  # kL2C0..2


def l2_digits(d):
    """i8l_digits: v = d 2^20 / ln 2 -> h = rint(v) (4 digits), l = rint((v - h) 2^18)
    (3 digits), as the device writes them."""
    hd = float(np.rint(d * L2_SCALE))
    h = int(hd)
    l = int(np.rint(fma(d, L2_SCALE, -hd) * 262144.0))
    hb, lb = h + 32 * (1 + 64 + 4096), l + 32 * (1 + 64)
    hd4 = [hb >> 18, ((hb >> 12) & 63) - 32, ((hb >> 6) & 63) - 32, (hb & 63) - 32]
    ld3 = [lb >> 12, ((lb >> 6) & 63) - 32, (lb & 63) - 32]
    return h, l, hd4, ld3


def test_log2_digit_expansion_exact():
    """h 2^-20 + l 2^-38 is d / ln 2 within 2^-39 (+ the rounding of d * kL2Scale);
    the 7 slices are int8 (top digit of h in [-128, 127] up to |d| / ln 2 < 31.87,
    the others in [-32, 32]); the MFMA pairs rebuild h and l exactly."""
    rng = np.random.default_rng(3)
    ds = np.concatenate([rng.uniform(-1, 1, 400) * 5.2, rng.uniform(-22.0, 22.0, 200), [0.0, 1e-12, -3.7]])
    for d in ds:
        h, l, hd4, ld3 = l2_digits(float(d))
        assert -128 <= hd4[0] <= 127 and all(-32 <= q <= 31 for q in hd4[1:])
        assert -32 <= ld3[0] <= 32 and all(-32 <= q <= 31 for q in ld3[1:])
        assert (64 * hd4[0] + hd4[1]) * 4096 + (64 * hd4[2] + hd4[3]) == h
        assert ld3[0] * 4096 + (64 * ld3[1] + ld3[2]) == l
        back = Fraction(h) / 2 ** 20 + Fraction(l) / 2 ** 38
        ref = mpmath.mpf(float(d)) / mpmath.log(2)
        assert abs(mpmath.mpf(back.numerator) / back.denominator - ref) <= 2.0 ** -39 + abs(float(d)) * 2.0 ** -52


def _l2_table():
    tab = []
    for j in range(2048):
        v = float(mpmath.mpf(2) ** (mpmath.mpf(j) / 2048))
        b = int(np.float64(v).view(np.uint64))
        tab.append((b & 0xFFFFFFFF, ((b >> 32) & 0x800FFFFF) ^ (j << 9)))
    return tab


def exp2_fx(t0, t1, tab):
    """exp2_fx_load / _series / _apply on (T_0, T_1) with 32-bit integer semantics."""
    t0 &= 0xFFFFFFFF
    low = t0 & 511
    lo, hi_t = tab[(t0 >> 6 & 0x3FF8) >> 3]
    hi = (t0 & ~511 & 0xFFFFFFFF) ^ hi_t
    value = float(np.uint64((hi << 32) | lo).view(np.float64))
    r32 = ((low << 18) + t1) & 0xFFFFFFFF
    r = float(r32 - (1 << 32) if r32 >= 1 << 31 else r32)
    p = fma(r, fma(r, L2_C[2], L2_C[1]), L2_C[0])
    return value * p


def test_exp2_fixed_point_assembly():
    """2^y from the integer accumulators, y = (T_0 - 1023 2^20) 2^-20 + T_1 2^-38:
    table entry with the exponent added to its high dword, remainder through the
    degree-2 Chebyshev series; within 3e-13 relative over the staged range
    (|y| <= 995.5, |T_1| <= 65 2^17)."""
    tab = _l2_table()
    rng = np.random.default_rng(4)
    worst = 0.0
    for _ in range(1500):
        y_int = int(rng.integers(-995, 995))
        frac = int(rng.integers(0, 1 << 20))
        t1 = int(rng.integers(-65 * 2 ** 17, 65 * 2 ** 17 + 1))
        t0 = (1023 + y_int) * 2 ** 20 + frac
        y = mpmath.mpf(y_int) + mpmath.mpf(frac) / 2 ** 20 + mpmath.mpf(t1) / 2 ** 38
        ref = mpmath.mpf(2) ** y
        worst = max(worst, float(abs(mpmath.mpf(exp2_fx(t0, t1, tab)) / ref - 1)))
    assert worst <= 3.2e-13


def test_remainder_through_slice4_cinit():
    """score_i8l_kernel's two-tile walk (NEMO_I8L_RINIT): slice 4's MFMA starts
    from C = (T_0 & 511) 2^6, so R = l0' 2^12 + l1 in 32-bit wrap-around
    arithmetic is exactly exp2_fx_series' R = (T_0 & 511) 2^18 + (l0 2^12 + l1)
    over the accumulator ranges (|slice-4 sum| <= 65 * 128 * 1, |l1| <= 2^23)."""
    rng = np.random.default_rng(12)
    n = 200000
    t0 = rng.integers(0, 1 << 31, n, dtype=np.int64)
    l0 = rng.integers(-65 * 128, 65 * 128 + 1, n, dtype=np.int64)
    l1 = rng.integers(-(1 << 23), (1 << 23) + 1, n, dtype=np.int64)
    wrap = lambda v: ((v + (1 << 31)) % (1 << 32)) - (1 << 31)  # int32 two's complement
    r_old = wrap((t0 & 511) * (1 << 18) + wrap(l0 * 4096 + l1))
    l0c = wrap(l0 + (t0 & 511) * 64)  # the MFMA accumulates onto the C operand
    r_new = wrap(l0c * 4096 + l1)
    assert np.array_equal(r_old, r_new)


def _dpp(v, ctrl):
    """update_dpp over 64 lanes for the dpp_ctrl values nemo_internal.h uses."""
    lane = np.arange(64)
    base, i = lane & ~15, lane & 15
    if ctrl == 0xB1:  # quad_perm [1,0,3,2]
        src = lane ^ 1
    elif ctrl == 0x4E:  # quad_perm [2,3,0,1]
        src = lane ^ 2
    elif ctrl == 0x141:  # row_half_mirror
        src = base + (i & 8) + (7 - (i & 7))
    elif ctrl == 0x140:  # row_mirror
        src = base + (15 - i)
    else:
        raise ValueError(ctrl)
    return v[src]


def _rowsum4(v):
    """v_permlane16_swap then v_permlane32_swap, both outputs summed: every lane
    gets the sum over lanes (l & 15) + 16 k."""
    lane = np.arange(64)
    v = v + v[lane ^ 16]
    return v + v[lane ^ 32]


def test_dpp_wave_sums_cover_every_lane_once():
    """rowsum16 / wsum_dpp (nemo_internal.h): with integer-valued lanes (exact
    sums), rowsum16 leaves each 16-lane row's sum in all its lanes and wsum_dpp
    the wave's sum in every lane -- each lane counted exactly once."""
    rng = np.random.default_rng(13)
    for _ in range(50):
        x = rng.integers(-1000, 1000, 64).astype(np.float64)
        r = x.copy()
        for c in (0xB1, 0x4E, 0x141, 0x140):
            r = r + _dpp(r, c)
        rows = x.reshape(4, 16).sum(axis=1)
        assert np.array_equal(r, np.repeat(rows, 16))
        assert np.array_equal(_rowsum4(r), np.full(64, x.sum()))


# --- score_window2_kernel (nemo_window.hip): register walk of the capped tables ---

_MLO = {16: 0x0000FFFF, 8: 0x00FF00FF, 4: 0x0F0F0F0F, 2: 0x33333333, 1: 0x55555555}


def _rotr(x, s):
    x = x.astype(np.uint64)
    s = np.asarray(s, dtype=np.uint64)
    return (((x >> s) | (x << ((np.uint64(32) - s) % np.uint64(32)))) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def window_transpose(m):
    """The kernel's cross-lane transpose of a 64 x 64 bit block (lane r holds
    row r as lo / hi dwords): the v_permlane32_swap of the off-diagonal 32 x 32
    blocks, then the five butterfly stages of tr_stage (partner = lane ^ d, a
    rotate by d or 32 - d, a bit select by the stage mask)."""
    lo = (m & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    hi = (m >> np.uint64(32)).astype(np.uint32)
    lo2, hi2 = lo.copy(), hi.copy()
    lo2[32:], hi2[:32] = hi[:32], lo[32:]
    lo, hi = lo2, hi2
    lane = np.arange(64)
    for d in (16, 8, 4, 2, 1):
        up = (lane & d) != 0
        sh = np.where(up, d, 32 - d)
        msk = np.where(up, ~np.uint32(_MLO[d]), np.uint32(_MLO[d])).astype(np.uint32)
        lo = ((lo & msk) | (_rotr(lo[lane ^ d], sh) & ~msk)).astype(np.uint32)
        hi = ((hi & msk) | (_rotr(hi[lane ^ d], sh) & ~msk)).astype(np.uint32)
    return lo, hi


def test_window_transpose_is_a_transpose():
    rng = np.random.default_rng(3)
    m = rng.integers(0, 2**64, size=64, dtype=np.uint64)
    lo, hi = window_transpose(m)
    bits = (m[:, None] >> np.arange(64, dtype=np.uint64)[None, :]) & np.uint64(1)  # [row][col]
    for j in range(64):
        assert int(lo[j]) == sum(int(bits[t, j]) << t for t in range(32))
        assert int(hi[j]) == sum(int(bits[32 + t, j]) << t for t in range(32))


@pytest.mark.parametrize("s,cap", [(128, 6), (70, 3), (11, 6), (5, 6), (33, 1), (150, 5)])
def test_window_walk_offsets(s, cap):
    """The kernel's LDS offsets, restated: A rows at 128 q, B' rows at
    kB0 + 128 q (B'[m] = B[m & 7]), av = (X & 0x78) | 4096 g from the funnel
    shift X of the transposed bits, B'(q) read at row q-3's av.  The walk must
    give sum_q e^{U'} prod_d y_d for every effect, rows before the order
    start and past the cap contributing factor 1."""
    rng = np.random.default_rng(s + cap)
    nb = (s + 63) // 64
    rows, kb0, mask = 64 * nb, 64 * nb * 128 + 64, 0xFFFFFFFF
    perm = rng.permutation(s)
    bits = rng.integers(0, 2, size=(s, 64))
    y = rng.uniform(0.5, 2.0, size=(s, 7, 2))
    for q in range(s):
        for d in range(1, 7):
            if not (d <= cap and q >= d):
                y[q, d] = 1.0
    lds = {}
    for q in range(rows):
        for m in range(16):
            a = y[q, 0, (m >> 3) & 1] * y[q, 1, (m >> 2) & 1] * y[q, 2, (m >> 1) & 1] * y[q, 3, m & 1] if q < s else 0.0
            b = y[q, 4, (m >> 2) & 1] * y[q, 5, (m >> 1) & 1] * y[q, 6, m & 1] if q < s else 0.0
            lds[128 * q + 8 * m], lds[kb0 + 128 * q + 8 * m] = a, b
    for e in range(64):
        r = [0] * (2 * nb)
        for q in range(s):
            if bits[perm[q], e]:
                r[q >> 5] |= 1 << (q & 31)
        tot, ap, rp, rc = 0.0, [(-4096) & mask] * 3, 0, r[0]
        for g in range(2 * nb):
            av = [0] * 32
            for t in range(32):
                x = (rc >> (t - 6)) if t >= 6 else ((((rc << 32) | rp) >> (t + 26)) & mask)
                av[t] = (x & 0x78) | ((g << 12) & ~0x78 & mask)
                aq3 = av[t - 3] if t >= 3 else ap[t]
                tot += lds[(av[t] + 128 * t) & mask] * lds[(aq3 + kb0 + 128 * (t - 3 if t >= 3 else t + 29) + 384) & mask]
            ap, rp, r = av[29:], rc, r[1:] + [0]
            rc = r[0]
        direct = 0.0
        for q in range(s):
            v = y[q, 0, bits[perm[q], e]]
            for d in range(1, 7):
                v *= y[q, d, bits[perm[q - d], e] if q >= d else 0]
            direct += v
        assert abs(tot - direct) <= 1e-12 * abs(direct)
