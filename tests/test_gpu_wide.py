"""The int8 log2 kernel for 64 < S <= 128 (score_i8w_kernel, fact_kernel 18).

Uncapped ll-only calls with more than 64 S-genes took the fp64 MFMA kernel
(13x fewer cells per second than the S <= 64 int8 kernel); score_i8w_kernel
runs the contraction as two K = 64 halves per row block.  Checked against the
oracle (the reference's compute_cell_ratios + calculate_ll restated,
nem_order_mcmc.py:79-93) within 1e-6 and within the kernel's own worst-case
bound, against the fp64 kernels, and for batch-independent bits."""
import numpy as np
import pytest
from scipy.special import expit

import nemo_oracle as no
from nemo import generator
from nemo.engine import Engine

pytestmark = pytest.mark.gpu

FP64_NOISE = 4e-9


def _pos(perm):
    pos = np.empty(len(perm), dtype=np.int32)
    pos[np.asarray(perm)] = np.arange(len(perm))
    return pos


@pytest.mark.parametrize("s,e", [(128, 700), (100, 2000), (65, 333), (96, 1000)])
def test_wide_kernel_vs_oracle(s, e):
    m = generator.synthetic_nem(s, e, 0)
    eng = Engine.for_nem(m)
    assert eng.get_option("i8w") == 1 and eng.get_option("i8l") == 0
    fk, bound = eng.score_kernel(0)
    assert fk == 18 and 0.0 < bound <= 1e-7
    t = m.get_score_tensor()
    rng = np.random.default_rng(s * 7 + e)
    n = 5
    perms = [rng.permutation(s) for _ in range(n)]
    pos = np.array([_pos(p) for p in perms])
    w01 = np.stack([expit(rng.uniform(-3, 3, (s, s))) for _ in range(n - 2)] +
                   [expit(rng.uniform(-30, 30, (s, s))), np.ones((s, s))])
    ll = eng.score(pos, w01)
    ref = np.array([no.order_score(m.U, t, perms[c], w01[c]) for c in range(n)])
    assert np.max(np.abs(ll - ref)) <= min(1e-6, bound + FP64_NOISE)
    # 19: the same kernel walking one tile per iteration (its own bits)
    eng.set_option("fact_kernel", 19)
    assert eng.score_kernel(0) == (19, bound)
    ll19 = eng.score(pos, w01)
    assert np.max(np.abs(ll19 - ref)) <= min(1e-6, bound + FP64_NOISE)
    assert eng.score(pos[1:2], w01[1:2])[0] == ll19[1]
    # the fp64 kernels on the same inputs (pipelined: ll only; chunked)
    for k in (1,):
        eng.set_option("fact_kernel", k)
        assert np.max(np.abs(eng.score(pos, w01) - ref)) <= FP64_NOISE
    eng.set_option("fact_kernel", 0)
    # bits independent of the batch and of the position in it
    for c in (0, n - 1):
        assert eng.score(pos[c:c + 1], w01[c:c + 1])[0] == ll[c]
    assert np.array_equal(eng.score(pos[::-1], w01[::-1]), ll[::-1])


def test_wide_kernel_caps_and_budget():
    s, e = 128, 700
    m = generator.synthetic_nem(s, e, 1)
    eng = Engine.for_nem(m)
    t = m.get_score_tensor()
    rng = np.random.default_rng(5)
    perm = rng.permutation(s)
    w01 = expit(rng.uniform(-3, 3, (1, s, s)))
    pos = _pos(perm)[None]
    # a cap the lookup-table kernel does not take (7 .. S-2): the wide kernel
    # with capped parent sets (nearest predecessors)
    for cap in (7, 70):
        assert eng.score_kernel(cap)[0] == 18
        got = eng.score(pos, w01, cap=cap)[0]
        assert abs(got - no.order_score(m.U, t, perm, w01[0], cap=cap)) <= 1e-6
    # a zero budget forces fp64; the wide kernel asked for explicitly still runs
    eng.set_option_f64("err_budget", 0.0)
    assert eng.score_kernel(0) == (1, 0.0)
    eng.set_option("fact_kernel", 18)
    fk, b = eng.score_kernel(0)
    assert fk == 18 and b > 0.0
    assert abs(eng.score(pos, w01)[0] - no.order_score(m.U, t, perm, w01[0])) <= 1e-6
    eng.set_option("fact_kernel", 0)
    eng.set_option_f64("err_budget", 1e-7)
    # outputs beyond ll take the fp64 kernel
    assert eng.score_kernel(0, ll_only=False)[0] == 1
