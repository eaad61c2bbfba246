"""GPU parity of the capped lookup-table kernel (score_window_kernel,
nemo_window.hip): the order score under a parent-set cap (SURVEY.md 8(a) A4,
BASELINE config C5) against the streaming kernel, the oracle and the C5
golden; tolerance 1e-8 absolute on log-scores (north_star: 1e-6)."""
import numpy as np
import pytest
from conftest import golden
from scipy.special import expit

import nemo_oracle as no
from nemo import generator
from nemo.engine import Engine

pytestmark = pytest.mark.gpu

TOL = 1e-8


def _pos(perm):
    pos = np.empty(len(perm), dtype=np.int32)
    pos[np.asarray(perm)] = np.arange(len(perm))
    return pos


@pytest.mark.parametrize("s,e,cap", [(3, 1, 1), (5, 130, 3), (11, 184, 6), (16, 500, 2), (40, 333, 6),
                                     (64, 2000, 6), (128, 700, 6), (150, 65, 5), (256, 130, 6)])
def test_window_kernel_vs_stream_and_oracle(s, e, cap):
    """fact_kernel 9 (and auto, which takes it for ll-only capped calls):
    orders whose first positions have fewer than cap parents, ragged last
    word (E % 64 != 0), S up to 150; single-evaluation calls give the batch's
    bits (the block split does not change them)."""
    m = generator.synthetic_nem(s, e, 4)
    t = m.get_score_tensor()
    eng = Engine(m.U, t)
    assert eng.factored and eng.get_option("win") == 1
    rng = np.random.default_rng(7 * s + e)
    b = 37
    perms = [rng.permutation(s) for _ in range(b)]
    pos = np.array([_pos(p) for p in perms])
    w01 = expit(rng.uniform(-4, 4, (b, s, s)))
    eng.set_option("score_path", 1)
    ref = eng.score(pos, w01, cap=cap)
    eng.set_option("score_path", 2)
    eng.set_option("fact_kernel", 9)
    ll = eng.score(pos, w01, cap=cap)
    assert np.max(np.abs(ll - ref)) <= TOL
    for c in (0, 11, 36):
        assert eng.score(pos[c:c + 1], w01[c:c + 1], cap=cap)[0] == ll[c]
    for c in (0, 1):
        assert abs(ll[c] - no.order_score(m.U, t, perms[c], w01[c], cap=cap)) <= TOL
    eng.set_option("fact_kernel", 0)
    # auto on the fast kernels takes it; the default (option exact) computes
    # capped host-pointer scores in the reference's arithmetic instead
    assert np.max(np.abs(eng.score(pos, w01, cap=cap) - ll)) <= TOL
    try:
        eng.set_option("exact", 0)
        assert np.array_equal(eng.score(pos, w01, cap=cap), ll)
    finally:
        eng.set_option("exact", 1)
    # the round-1 form (row bits re-read from LDS, exp of summed logs): its own
    # bits, the same values
    eng.set_option("fact_kernel", 15)
    r1 = eng.score(pos, w01, cap=cap)
    assert np.max(np.abs(r1 - ll)) <= TOL
    assert eng.score(pos[5:6], w01[5:6], cap=cap)[0] == r1[5]
    eng.set_option("fact_kernel", 0)
    # weights at 0 and 1: every factor at its extremes
    for w in (0.0, 1.0):
        wz = np.full((2, s, s), w)
        a = eng.score(pos[:2], wz, cap=cap)
        eng.set_option("score_path", 1)
        assert np.max(np.abs(a - eng.score(pos[:2], wz, cap=cap))) <= TOL
        eng.set_option("score_path", 2)
    # uncapped calls never take it; fact_kernel 9 then fails loudly
    eng.set_option("fact_kernel", 9)
    with pytest.raises(RuntimeError):
        eng.score(pos[:2], w01[:2], cap=0)
    eng.close()


def test_window_kernel_c5_golden():
    """BASELINE config C5 (128 x 5000, cap 6) against the reference golden,
    fp64 and fp32 stagings."""
    z = golden("eval_C5cap.npz")
    m = generator.synthetic_nem(128, 5000, 0)
    pos = np.array([_pos(p) for p in z["perm"]])
    w01 = expit(z["W"])
    for dtype in ("f64", "f32"):
        eng = Engine.for_nem(m, dtype=dtype)
        assert eng.get_option("win") == 1
        eng.set_option("fact_kernel", 9)
        ll = eng.score(pos, w01, cap=6)
        assert np.max(np.abs(ll - z["ll"])) <= 1e-6, dtype
        eng.close()


def test_window_kernel_not_staged_for_generic_u():
    """A U whose U - U[S] is not two-valued per row: no lookup-table kernel;
    auto falls back to the fp64 factored kernels, fact_kernel 9 raises."""
    m = generator.synthetic_nem(20, 150, 5)
    t = m.get_score_tensor()
    rng = np.random.default_rng(9)
    u = m.U + rng.uniform(-0.5, 0.5, m.U.shape)
    eng = Engine(u, t)
    assert eng.factored and eng.get_option("win") == 0
    perms = [rng.permutation(20) for _ in range(3)]
    pos = np.array([_pos(p) for p in perms])
    w01 = expit(rng.uniform(-3, 3, (3, 20, 20)))
    ll = eng.score(pos, w01, cap=4)
    for c in range(3):
        assert abs(ll[c] - no.order_score(u, t, perms[c], w01[c], cap=4)) <= TOL
    eng.set_option("fact_kernel", 9)
    with pytest.raises(RuntimeError):
        eng.score(pos, w01, cap=4)
    eng.close()
