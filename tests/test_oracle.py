"""Pin the oracle (oracle/nemo_oracle.py) to the reference's own outputs.

Every golden vector was produced by importing the reference itself
(tests/golden/make_goldens.py); this module checks the CPU restatement against
them, so the oracle can then stand in for the reference on the GPU box, where
/root/reference does not exist.
"""
import random

import numpy as np
import pytest
from conftest import golden

import nemo_oracle as no
from nemo import generator


def test_kat_knockdown_from_reference_test():
    # tests/utils.tests.py:11-27 of the reference: data only
    z = golden("kat_knockdown.npz")
    from nemo import utils
    got = utils.create_real_knockdown_mat(z["s_mat"].tolist(), z["e_arr"].tolist())
    assert np.array_equal(got, z["expected"])


def test_oracle_tables_net2_bit_exact():
    z = golden("net2_tables.npz")
    d = z["D"].astype(np.float64)
    t = no.score_tensor(d, float(z["A"]), float(z["B"]))
    assert np.array_equal(t, z["T"])
    u = no.node_lr_table(t, d, float(z["A"]))
    assert np.array_equal(u, z["U"])


def _unpack_d(z):
    s, e = int(z["S"]), int(z["E"])
    return np.unpackbits(z["D_packed"])[: s * e].reshape(s, e).astype(np.float64)


@pytest.mark.parametrize("name", ["net2", "C2"])
def test_oracle_eval_small(name):
    z = golden(f"eval_{name}.npz")
    if name == "net2":
        t = golden("net2_tables.npz")
        u, tt = t["U"], t["T"]
    else:
        d = _unpack_d(z)
        tt = no.score_tensor(d, float(z["A"]), float(z["B"]))
        u = no.node_lr_table(tt, d, float(z["A"]))
        assert np.array_equal(u, z["U"])
    from scipy.special import expit
    for c in range(len(z["ll"])):
        perm, w = z["perm"][c], z["W"][c]
        cell = no.cell_ratios(u, tt, no.parents_of(perm), expit(w))
        ow, ll, cs = no.calculate_ll(cell)
        assert ll == z["ll"][c]            # same operation order: bit-exact
        assert np.array_equal(cs, z["cs"][c])
        if c == 0:
            assert np.array_equal(ow, z["ow0"])


def test_oracle_eval_c3_and_c5cap():
    from scipy.special import expit
    import hashlib
    for name in ("C3", "C5cap"):
        z = golden(f"eval_{name}.npz")
        d = _unpack_d(z)
        a, b = float(z["A"]), float(z["B"])
        tt = no.score_tensor(d, a, b)
        u = no.node_lr_table(tt, d, a)
        assert hashlib.sha256(u.tobytes()).hexdigest() == str(z["U_sha256"])
        cap = int(z["cap"])
        for c in range(len(z["ll"])):
            cell = no.cell_ratios(u, tt, no.parents_of(z["perm"][c], cap), expit(z["W"][c]))
            _, ll, cs = no.calculate_ll(cell)
            assert ll == z["ll"][c]
            assert np.array_equal(cs, z["cs"][c])


def test_generator_reproduces_golden_knockdown():
    """The synthetic D used for C2/C3/C5 goldens is regenerated bit for bit
    by nemo.generator + nemo.NEM (reference knockdown semantics)."""
    for name, s, e in (("C2", 16, 500), ("C3", 64, 2000), ("C5cap", 128, 5000)):
        z = golden(f"eval_{name}.npz")
        m = generator.synthetic_nem(s, e, 0)
        assert np.array_equal(m.observed_knockdown_mat, _unpack_d(z))
        assert m.A == z["A"] and m.B == z["B"]


def _oracle_traj(u, t, order, gamma, swap_prob, n, use_nem=False):
    smp = no.OracleSampler(u, t, order)
    smp.method(swap_prob=swap_prob, gamma=gamma, n_iterations=n, use_nem=use_nem)
    return smp


def test_oracle_trajectory_net2_200(net2):
    """C1: the oracle sampler replays the reference's 200-step net2 run."""
    z = golden("traj_net2_200.npz")
    tz = golden("net2_tables.npz")
    m, state = net2
    random.setstate(state)
    assert np.array_equal(np.array(random.getstate()[1]), tz["rng_state_after_nem"])
    smp = _oracle_traj(tz["U"], tz["T"], z["order0"], float(z["gamma"]), float(z["swap_prob"]),
                       int(z["n_iter"]))
    assert np.array_equal(np.array(smp.traj["acc"]), z["acc"])
    assert np.array_equal(np.array(smp.traj["i1"]), z["i1"])
    assert np.array_equal(np.array(smp.traj["perm"]), z["perm"])
    assert np.array_equal(np.array(smp.all_scores), z["all_scores"])
    assert smp.best_score == float(z["best_score"])
    assert np.array_equal(smp.w, z["final_W"])


def test_oracle_trajectory_c2_20():
    z = golden("traj_C2_20.npz")
    m = generator.synthetic_nem(16, 500, 0)
    t = m.get_score_tensor()
    smp = _oracle_traj(m.U, t, z["order0"], float(z["gamma"]), float(z["swap_prob"]), int(z["n_iter"]))
    assert np.array_equal(np.array(smp.traj["acc"]), z["acc"])
    assert np.array_equal(np.array(smp.all_scores), z["all_scores"])
    assert np.array_equal(np.array(random.getstate()[1]), z["rng_state_after"])


def test_oracle_trajectory_net2_use_nem_50(net2):
    """method(use_nem=True) (nem_order_mcmc.py:203-204, 283-284; the closure
    of utils.py:37-54): the oracle replays the reference's 50-step net2 run."""
    z = golden("traj_net2_nem_50.npz")
    tz = golden("net2_tables.npz")
    assert bool(z["use_nem"])
    _m, state = net2
    random.setstate(state)
    smp = _oracle_traj(tz["U"], tz["T"], z["order0"], float(z["gamma"]), float(z["swap_prob"]),
                       int(z["n_iter"]), use_nem=True)
    assert np.array_equal(np.array(smp.traj["acc"]), z["acc"])
    assert np.array_equal(np.array(smp.traj["perm"]), z["perm"])
    assert np.array_equal(np.array(smp.all_scores), z["all_scores"])
    assert smp.best_score == float(z["best_score"])
    assert np.array_equal(smp.best_order, z["best_order"])
    assert np.array_equal(smp.w, z["final_W"])
    assert np.array_equal(np.array(random.getstate()[1]), z["rng_state_after"])


def test_oracle_capped_step_equals_reference_capture():
    """The capped step (the C5 shape, parent lists cut to the last 6
    predecessors): OracleSampler(cap=6)'s get_optimal_weights(init=True)
    equals the reference's own step on the same cut lists
    (tests/golden/make_goldens.py capture_capped_step, nem_order_mcmc.py:
    172-208 with :186-189 over the overridden parents_list) -- ll, dag_ll,
    ancestor_x, the new weights and every local optimum's x*, nit and nfev, to
    the bit.  This pins the oracle's cap branch (nemo_oracle.py permissible)."""
    z = golden("step_C5cap_40x333.npz")
    d = _unpack_d(z)
    a, b = float(z["A"]), float(z["B"])
    tt = no.score_tensor(d, a, b)
    u = no.node_lr_table(tt, d, a)
    cap = int(z["cap"])
    for c in range(int(z["n_cases"])):
        ora = no.OracleSampler(u, tt, z[f"c{c}_perm"], record_local=True, cap=cap)
        ora.w = np.array(z[f"c{c}_W"], copy=True)
        dag_ll = ora.optimal_weights()
        assert ora.ll1 == z[f"c{c}_ll"] and dag_ll == z[f"c{c}_dag_ll"]
        assert np.array_equal(ora.anc, z[f"c{c}_anc"])
        assert np.array_equal(ora.w, z[f"c{c}_W_new"])
        ik = z[f"c{c}_local"]
        assert [(r[0], r[1]) for r in ora.local_log] == [tuple(x) for x in ik.tolist()]
        got_f = np.array([(r[4], r[3], r[5]) for r in ora.local_log])   # x0, anc, x*
        assert np.array_equal(got_f, z[f"c{c}_local_f"][:, :3])
        assert np.array_equal(np.array([(r[6], r[7]) for r in ora.local_log]), z[f"c{c}_local_n"])
