"""Host-side logic of the product package (no GPU): tables, RNG stream,
parent-set bookkeeping quirks, proposals, DAG helpers, network I/O."""
import os
import random

import numpy as np
import pytest
from conftest import GOLDEN, golden

import nemo_oracle as no
from nemo import NEM, generator, utils


def test_net2_model_bit_exact(net2):
    m, state = net2
    z = golden("net2_tables.npz")
    assert np.array_equal(m.observed_knockdown_mat, z["D"].astype(float))
    assert np.array_equal(m.real_knockdown_mat, z["D_real"].astype(float))
    assert m.A == z["A"] and m.B == z["B"]
    assert np.array_equal(m.U, z["U"])
    assert np.array_equal(m.get_score_tensor(), z["T"])
    assert np.array_equal(np.array(m.get_score_tables(m.observed_knockdown_mat)), z["T"])
    # RNG state after construction equals the reference's (proposals continue from it)
    assert np.array_equal(np.array(state[1]), z["rng_state_after_nem"])
    # compute_real_score's side effect: caller's adjacency diagonal zeroed
    assert np.array_equal(m.adj_matrix, z["adj_after"])


def test_lazy_tables_and_direct_u():
    """The constructor's U (closed form, no S*S*E table) equals the
    reference's get_node_lr_table(get_score_tables(D)) bit for bit, and the
    lazy table sequence behaves like the reference's list."""
    for s, e, seed in ((11, 184, 0), (16, 500, 0), (40, 300, 7)):
        m = generator.synthetic_nem(s, e, seed)
        tables = m.get_score_tables(m.observed_knockdown_mat)
        t = m.get_score_tensor()
        assert len(tables) == s
        assert np.array_equal(m.U, m.get_node_lr_table([t[i] for i in range(s)]))
        assert np.array_equal(np.asarray(tables), t)
        assert np.array_equal(tables[-1], t[s - 1]) and np.array_equal(tables[3][1], t[3][1])
        assert all(np.array_equal(a, b) for a, b in zip(tables, t))
        with pytest.raises(IndexError):
            tables[s]


def test_initial_order_guess(net2):
    m, _ = net2
    assert np.array_equal(utils.initial_order_guess(m.observed_knockdown_mat), golden("net2_tables.npz")["order0"])


def test_read_write_csv_roundtrip(tmp_path):
    adj, end, err, s, e = utils.read_csv_to_adj(os.path.join(GOLDEN, "network2.csv"))
    assert (s, e) == (11, 184) and adj.sum() > 0 and len(end) == e
    assert tuple(err) == (0.05, 0.08)
    p = tmp_path / "n.csv"
    utils.write_adj_to_csv(str(p), adj, end, err)
    adj2, end2, err2, s2, e2 = utils.read_csv_to_adj(str(p))
    assert np.array_equal(adj, adj2) and np.array_equal(end, end2) and (s2, e2) == (s, e)


def test_ancestor_matches_closure_and_wraps_like_reference():
    g = generator.synthetic_network(12, 10, 3)
    assert np.array_equal(utils.ancestor(g.adj), generator.transitive_closure(g.adj))
    # dense 64-node DAG: the reference's int64 path counts wrap around
    # (utils.py:37-54); the result must equal that arithmetic, restated by the
    # oracle, whatever the true closure is
    dense = np.triu(np.ones((64, 64), dtype=int), 1)
    assert np.array_equal(utils.ancestor(dense), no.OracleSampler.dag_weights(dense * 0.9, True))


def test_transitive_reduction_brute_force():
    rng = np.random.default_rng(5)
    for _ in range(5):
        g = generator.synthetic_network(9, 5, int(rng.integers(1000)), edge_p=0.3)
        red = utils.transitive_reduction(g.adj)
        # literal triple loop of the reference semantics
        ref = g.adj.copy()
        n = ref.shape[0]
        for k in range(n):
            for i in range(n):
                for j in range(n):
                    if i != j and ref[i][k] and ref[k][j]:
                        ref[i][j] = 0
        assert np.array_equal(red, ref)


def test_order_unorder_roundtrip():
    rng = np.random.default_rng(1)
    order = rng.permutation(7)
    a = rng.random((7, 7))
    assert np.array_equal(utils.unorder_arr(order, utils.order_arr(order, a)), a)
    idx = np.argsort(order)
    assert np.array_equal(utils.order_arr(order, a), a[idx][:, idx])


def test_synthetic_generator_deterministic():
    a = generator.synthetic_network(16, 50, 7)
    b = generator.synthetic_network(16, 50, 7)
    assert np.array_equal(a.adj, b.adj) and np.array_equal(a.end_nodes, b.end_nodes)
    # closure of a DAG: acyclic (no i->i) and transitive
    reach = a.adj.astype(bool)
    assert not np.any(np.diag(reach))
    assert np.array_equal((reach.astype(int) @ reach.astype(int) > 0) & ~reach, np.zeros_like(reach))


def test_permissible_mask_cap():
    pos = np.array([2, 0, 3, 1])
    m = generator.permissible_mask(pos)
    assert m.sum() == 6
    assert m[0, 1] and m[0, 3] and not m[0, 2]
    mc = generator.permissible_mask(pos, cap=1)
    assert mc.sum() == 3 and mc[0, 3] and not mc[0, 1]


class _HostOnly:
    """The product sampler's host state machine without its GPU engine."""

    def __init__(self, s, cap=0):
        from nemo.nem_order_mcmc import NEMOrderMCMC
        self.obj = NEMOrderMCMC.__new__(NEMOrderMCMC)
        self.obj.num_s = s
        self.obj.cap = cap
        self.obj.parent_weights = np.zeros((s, s))


def test_reset_quirks_match_oracle():
    """get_permissible_parents(init=False) mutates W exactly like the reference
    (checked against the oracle restatement over a random proposal sequence)."""
    s = 9
    h = _HostOnly(s)
    rng = np.random.default_rng(0)
    perm = rng.permutation(s)
    ref = no.OracleSampler(np.zeros((s + 1, 3)), np.zeros((s, s, 3)), perm)
    h.obj.get_permissible_parents(perm, init=True, init_value=1.0)
    assert np.array_equal(h.obj.parent_weights, ref.w)
    random.seed(11)
    st = random.getstate()
    for step in range(60):
        ref.w = ref.w + rng.random((s, s)) * (rng.random((s, s)) < 0.3)  # stale junk
        h.obj.parent_weights = ref.w.copy()
        random.setstate(st)
        p1, i1, i2 = ref.new_order(perm, 0.7)
        st_after = random.getstate()
        random.setstate(st)
        p2, j1, j2 = h.obj.get_new_order(perm, 0.7)
        assert random.getstate() == st_after
        assert np.array_equal(p1, p2) and (i1, i2) == (j1, j2)
        st = st_after
        ref.permissible(p1, i1, i2, init=False)
        h.obj.reset(p2, i1, i2)
        assert np.array_equal(h.obj.parent_weights, ref.w), step
        for i in range(s):
            assert np.array_equal(h.obj.parents_list[i], ref.parents[i])
        perm = p1 if step % 2 else perm


def test_inv_stack_bit_exact_to_scipy_inv():
    """The batched ancestor_x inverse (nemo.chains.inv_stack) returns
    scipy.linalg.inv's bits for every matrix, and its errors for a singular
    or non-finite one (nem_order_mcmc.py:185)."""
    from scipy.linalg import LinAlgError, inv
    from nemo.chains import inv_stack
    rng = np.random.default_rng(3)
    for s in (2, 11, 64):
        a = np.identity(s) - np.triu(rng.random((4, s, s)), 1) * 0.7 - np.tril(rng.random((4, s, s)), -1) * 0.01
        out = inv_stack(a)
        for k in range(4):
            assert np.array_equal(out[k], inv(a[k]))
    with pytest.raises(LinAlgError):
        inv_stack(np.zeros((1, 3, 3)))
    bad = np.identity(3)[None].copy()
    bad[0, 0, 1] = np.nan
    with pytest.raises(ValueError):
        inv_stack(bad)


def test_expit_parent_weights_and_dag():
    s = 5
    h = _HostOnly(s).obj
    perm = np.array([3, 1, 4, 0, 2])
    h.get_permissible_parents(perm, init=True, init_value=1.0)
    w = np.arange(25, dtype=float).reshape(5, 5) / 10 - 1.0
    ref = no.OracleSampler(np.zeros((s + 1, 2)), np.zeros((s, s, 2)), perm)
    assert np.array_equal(h.expit_parent_weights(w), ref._mapped(w))
    assert np.array_equal(h.create_dag(w)[1], 1 * (w > 0.5))
    assert np.array_equal(h.create_nem(w)[1], no.OracleSampler.dag_weights(w, True))
