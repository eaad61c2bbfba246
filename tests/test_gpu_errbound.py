"""The fixed-point kernels' error budget on the GPU.

The int8 score kernels round every entry of their contraction once, and those
roundings repeat over the effects, so the worst-case ll error grows with E
(nemo_host.h fixed_point_bound).  Auto takes the log2 kernel
only while its bound stays within the "err_budget" option (default 1e-7, a
tenth of the north star's 1e-6), then the 8-slice kernel, then fp64.  These
tests check the bound against the oracle (the reference's compute_cell_ratios
+ calculate_ll restated, nem_order_mcmc.py:79-93) at the headline size and at
8x its effects, where auto must leave the log2 kernel."""
import numpy as np
import pytest
from conftest import golden
from scipy.special import expit

import nemo_oracle as no
from nemo import generator
from nemo.engine import Engine

pytestmark = pytest.mark.gpu

LL_TOL = 1e-6
FP64_NOISE = 2e-9   # fp64 rounding of the reference path itself at |ll| ~ 4e4 (observed ~1e-10)


def _pos(perm):
    pos = np.empty(len(perm), dtype=np.int32)
    pos[np.asarray(perm)] = np.arange(len(perm))
    return pos


def test_c3_auto_takes_log2_kernel_within_budget():
    z = golden("eval_C3.npz")
    m = generator.synthetic_nem(64, 2000, 0)
    eng = Engine.for_nem(m)
    fk, bound = eng.score_kernel(0)
    assert eng.get_option_f64("err_budget") == 1e-7
    assert fk == 10 and 0.0 < bound <= 1e-7
    assert bound == eng.get_option_f64("i8l_bound")
    # the 8-slice kernel carries 2^-45 per entry at this model's scale (c = 4)
    # against the log2 kernel's 2^-39 ln 2: ~45x tighter
    assert eng.get_option_f64("i8o_bound") < bound / 40
    pos = np.array([_pos(p) for p in z["perm"]])
    w01 = expit(z["W"])
    # every kernel within its own bound of the reference's ll (plus the fp64
    # noise all kernels share); the fp64 kernels have bound 0
    for k in (10, 16, 8, 4, 2, 1):
        eng.set_option("fact_kernel", k)
        kk, b = eng.score_kernel(0)
        assert kk == k
        ll = eng.score(pos, w01)
        err = np.max(np.abs(ll - z["ll"]))
        assert err <= b + FP64_NOISE, (k, err, b)
    eng.set_option("fact_kernel", 0)
    # capped calls: the lookup-table kernel (fp64 tables, no fixed point)
    assert eng.score_kernel(6) == (9, 0.0)
    # a cap lowers the int8 bound (fewer parents per cell)
    eng.set_option("fact_kernel", 10)
    assert eng.score_kernel(3)[1] < bound
    eng.set_option("fact_kernel", 0)
    # outputs beyond ll take the fp64 kernel
    assert eng.score_kernel(0, ll_only=False) == (1, 0.0)
    eng.close()


@pytest.fixture(scope="module")
def wide():
    """64 S-genes x 16000 effects: 8x the headline's effects.  The host-pointer
    score calls here test the fixed-point kernels' error budget, so option
    exact is 0 (E = 16000 is inside the exact path since round 6: numpy's
    pairwise sum in four plan parts)."""
    m = generator.synthetic_nem(64, 16000, 0)
    eng = Engine.for_nem(m)
    assert eng.get_option("exact_ok") == 1
    eng.set_option("exact", 0)
    return m, eng, m.get_score_tensor()


def test_wide_model_auto_leaves_log2_kernel(wide):
    m, eng, t = wide
    b_l2 = eng.get_option_f64("i8l_bound")
    b_nat = eng.get_option_f64("i8o_bound")
    assert b_l2 > 1e-7 >= b_nat   # the log2 kernel's bound trips at this E
    fk, bound = eng.score_kernel(0)
    assert fk == 8 and bound == b_nat
    rng = np.random.default_rng(16000)
    perms = [rng.permutation(64) for _ in range(3)]
    pos = np.array([_pos(p) for p in perms])
    # weights across the range: random, saturated, all 0, all 1
    w01 = np.stack([expit(rng.uniform(-3, 3, (64, 64))), expit(rng.uniform(-30, 30, (64, 64))),
                    np.ones((64, 64))])
    ref = np.array([no.order_score(m.U, t, perms[c], w01[c]) for c in range(3)])
    ll = eng.score(pos, w01)
    assert np.max(np.abs(ll - ref)) <= min(LL_TOL, bound + FP64_NOISE * 8)
    # forcing the log2 kernel: still within its own (larger) bound
    eng.set_option("fact_kernel", 10)
    ll10 = eng.score(pos, w01)
    assert np.max(np.abs(ll10 - ref)) <= b_l2 + FP64_NOISE * 8
    # a looser budget lets auto take it again; a zero budget forces fp64
    eng.set_option("fact_kernel", 0)
    eng.set_option_f64("err_budget", 1e-5)
    assert eng.score_kernel(0)[0] == 10
    assert np.array_equal(eng.score(pos, w01), ll10)
    eng.set_option_f64("err_budget", 0.0)
    fk0, b0 = eng.score_kernel(0)
    assert fk0 == 2 and b0 == 0.0
    llf = eng.score(pos, w01)
    assert np.max(np.abs(llf - ref)) <= FP64_NOISE * 8
    eng.set_option_f64("err_budget", 1e-7)
    with pytest.raises(RuntimeError, match="err_budget"):
        eng.set_option_f64("err_budget", -1.0)


def test_persistent_kernel_equals_default_past_its_grid():
    """fact_kernel 17 runs min(batch, 3 x CUs) persistent blocks; only batches
    above that (768 on MI355X) reach its double-buffered path (next
    evaluation's prep in the walk, buffer reuse): same bits as kernel 10."""
    m = generator.synthetic_nem(64, 2000, 0)
    eng = Engine.for_nem(m)
    rng = np.random.default_rng(17)
    b = 2048
    pos = np.array([rng.permutation(64) for _ in range(b)], dtype=np.int32)
    w01 = expit(rng.uniform(-3, 3, (b, 64, 64)))
    eng.set_option("fact_kernel", 10)
    ref = eng.score(pos, w01)
    eng.set_option("fact_kernel", 17)
    got = eng.score(pos, w01)
    assert np.array_equal(got, ref)
    eng.close()


def test_split_prep_walk_equals_default():
    """fact_kernel 20 (an experiment) runs kernel 10's prep and
    walk as two launches, the prep's LDS image going through HBM: same bits
    as kernel 10 at a split batch (B = 1, 16 blocks per evaluation), a ragged
    one and past one block per CU; an image buffer grows with the batch."""
    m = generator.synthetic_nem(64, 2000, 0)
    eng = Engine.for_nem(m)
    rng = np.random.default_rng(20)
    for b in (1, 7, 1100):
        pos = np.array([rng.permutation(64) for _ in range(b)], dtype=np.int32)
        w01 = expit(rng.uniform(-3, 3, (b, 64, 64)))
        eng.set_option("fact_kernel", 10)
        ref = eng.score(pos, w01)
        eng.set_option("fact_kernel", 20)
        got = eng.score(pos, w01)
        assert np.array_equal(got, ref), b
    eng.close()
