"""The exact path's limits (nemo.limits, INTEGRATION.md's table): every
limit walked on the CPU, on both sides of its bound."""
import numpy as np

from nemo import limits


def _numpy_leaves(E):
    # numpy's pairwise_sum recursion, counted directly
    def rec(n):
        if n <= 128:
            return 1
        n2 = n // 2
        n2 -= n2 % 8
        return rec(n2) + rec(n - n2)
    return rec(E)


def test_pairwise_parts_are_numpys_buffers():
    # np.sum past 8192 terms: one plan per numpy buffer (tests/test_exact_spec.py
    # checks the sums themselves against numpy)
    assert limits.pairwise_parts(2000) == [2000] and limits.pairwise_parts(8192) == [8192]
    assert limits.pairwise_parts(9000) == [8192, 808]
    assert limits.pairwise_parts(16384) == [8192, 8192]
    assert limits.pairwise_parts(64 * 8192) is not None and limits.pairwise_parts(64 * 8192 + 1) is None
    assert all(limits.pairwise_leaves(n) <= limits.MAX_LEAVES for n in limits.pairwise_parts(100001))


def test_pairwise_leaves_follow_numpys_recursion():
    for E in list(range(1, 300)) + [500, 1000, 2000, 3900, 4096, 4097, 5000, 8192, 8193, 8200, 9000, 16384]:
        assert limits.pairwise_leaves(E) == _numpy_leaves(E), E
    assert limits.pairwise_leaves(2000) == 16 and limits.pairwise_leaves(8192) == 64
    assert limits.pairwise_leaves(9000) > 64


def _status(**kw):
    a = dict(S=64, E=2000, factored=True, cap=0, host_blas="SkylakeX", exact_option=True)
    a.update(kw)
    return limits.exact_status_from(limits.exact_limits(**a))


def test_each_limit_on_both_sides():
    assert _status() == (True, "")                                   # C3
    assert _status(S=128, E=5000, cap=6) == (True, "")               # C5's shape: host inverse, same bits
    ok, why = _status(exact_option=False)
    assert not ok and why.startswith("option exact")
    ok, why = _status(factored=False)
    assert not ok and why.startswith("table form")
    assert _status(E=8192)[0] and _status(E=9000)[0] and _status(E=100001)[0]   # buffers from 8193
    assert not _status(E=64 * 8192 + 1)[0]                           # past 64 numpy buffers
    assert "E (effects)" in _status(E=64 * 8192 + 1)[1]
    assert "the step fails" in _status(E=64 * 8192 + 1)[1]           # past the fast local optima too
    for cap in (0, 1, 6, 63):
        assert _status(cap=cap)[0]


def test_device_ancestor_limit_keeps_the_bits():
    rows = {r.name: r for r in limits.exact_limits(65, 2000, True)}
    anc = rows["S (S-genes), ancestor_x on the device"]
    assert not anc.covered and anc.bits                              # S = 65: scipy on the host
    assert {r.name: r for r in limits.exact_limits(64, 2000, True)}["S (S-genes), ancestor_x on the device"].covered
    r = {r.name: r for r in limits.exact_limits(64, 2000, True, host_blas="Haswell")}
    assert not r["S (S-genes), ancestor_x on the device"].covered
    assert _status(S=65)[0] and _status(host_blas="Haswell")[0]      # the step itself keeps the bits


def test_table_renders_every_row():
    md = limits.limits_table_markdown(limits.exact_limits(64, 2000, True))
    assert md.count("\n") == 1 + len(limits.exact_limits(64, 2000, True))
    assert "E (effects)" in md and "ancestor_x" in md
