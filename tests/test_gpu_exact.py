"""GPU: the fused step in the reference's own arithmetic (option "exact",
the default; csrc/refmath.h, csrc/lbfgsb_exact.h, csrc/nemo_exact.hip),
checked bit for bit -- no tolerance -- against numpy / scipy and against the
reference's own recorded outputs."""
import math
import random

import numpy as np
import pytest
from conftest import golden
from scipy.special import expit

import nemo_oracle as no
from nemo import _lib, generator
from nemo.engine import Engine

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


def test_refmath_on_the_device_equals_numpy_scipy_glibc():
    """np.log / np.exp (SVML), scipy's expit, np.logaddexp and glibc's exp /
    log1p: the device restatements give the libraries' bits."""
    rng = np.random.default_rng(11)
    n = 1 << 20
    x = np.exp(rng.uniform(np.log(1e-3), np.log(1e6), n))
    assert _bits_equal(_lib.refmath_probe("log", x), np.log(x))
    x = 1.0 + np.exp(rng.uniform(np.log(1e-12), np.log(1e-2), n))
    assert _bits_equal(_lib.refmath_probe("log", x), np.log(x))
    x = rng.uniform(-707, 707, n)
    assert _bits_equal(_lib.refmath_probe("exp", x), np.exp(x))
    x = rng.uniform(-50, 0, n)
    assert _bits_equal(_lib.refmath_probe("exp", x), np.exp(x))
    x = rng.normal(0, 6, n)
    assert _bits_equal(_lib.refmath_probe("expit", x), expit(x))
    a, b = rng.normal(-60, 25, n), rng.normal(-60, 25, n)
    b[::7] = a[::7]
    assert _bits_equal(_lib.refmath_probe("logaddexp", a, b), np.logaddexp(a, b))
    x = rng.uniform(-745, 709, 1 << 16)
    assert _bits_equal(_lib.refmath_probe("glibc_exp", x), [math.exp(v) for v in x])
    x = np.exp(rng.uniform(np.log(1e-300), 0, 1 << 16))
    assert _bits_equal(_lib.refmath_probe("glibc_log1p", x), [math.log1p(v) for v in x])
    # logaddexp's log1p on [0, 1] (its normalising branch from 0.41422, the
    # divisions without scaling): dense near the branch points and the ends
    x = np.concatenate([rng.uniform(0, 1, 1 << 17), rng.uniform(0.41, 0.42, 1 << 15),
                        np.exp(rng.uniform(np.log(1e-320), 0, 1 << 15)), 1.0 - rng.uniform(0, 1e-6, 1 << 14),
                        [0.0, 1.0, 0.41421356, 2.0 ** -29, 2.0 ** -54, 5e-324]])
    assert _bits_equal(_lib.refmath_probe("log1p_unit", x), [math.log1p(v) for v in x])
    a = rng.normal(-60, 25, n)
    b = a + rng.normal(0, 1.0, n)     # |a - b| < 0.88 for most: the normalising branch
    b[::5] = a[::5] + rng.normal(0, 1e-9, len(b[::5]))
    assert _bits_equal(_lib.refmath_probe("logaddexp", a, b), np.logaddexp(a, b))
    # the IEEE operations the optimiser's control needs correctly rounded
    x = np.exp(rng.uniform(-700, 700, n))
    assert _bits_equal(_lib.refmath_probe("sqrt", x), np.sqrt(x))
    y = rng.normal(size=n) * np.exp(rng.uniform(-300, 300, n))
    assert _bits_equal(_lib.refmath_probe("div", x, y), x / y)


@pytest.mark.parametrize("name", ["net2_200", "C2_20"])
def test_exact_local_optima_equal_scipy_records(name):
    """Every recorded reference optimisation (c, anc, x0 -> scipy's x*, f*,
    nit, nfev): the same bits."""
    z = golden(f"localopt_{name}.npz")
    e = z["c"].shape[1]
    eng = Engine(np.zeros((3, e)), np.zeros((2, 2, e)))
    assert eng.get_option("exact") == 1 and eng.get_option("exact_ok") == 1
    xs, fs, nit, nfev, st = eng.local_opt(z["c"], z["anc"], z["x0"])
    assert np.array_equal(nit, z["nit"]) and np.array_equal(nfev, z["nfev"])
    assert _bits_equal(xs, z["xstar"]), int((xs != z["xstar"]).sum())
    assert _bits_equal(fs, z["fun"])
    eng.close()


def test_exact_long_local_optima_equal_scipy():
    """The longest C3 optima (nit up to 11: the m = 10 memory full and its
    oldest pair dropped; tests/golden/make_localopt_long.py)."""
    import os
    import sys
    from conftest import REPO
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from make_localopt_long import long_cases
    c, anc, x0, rec = long_cases()
    eng = Engine(np.zeros((3, c.shape[1])), np.zeros((2, 2, c.shape[1])))
    xs, fs, nit, nfev, st = eng.local_opt(c, anc, x0)
    assert np.array_equal(nit, rec["nit"]) and np.array_equal(nfev, rec["nfev"])
    assert _bits_equal(xs, rec["xstar"]) and _bits_equal(fs, rec["fun"])
    eng.close()


@pytest.mark.parametrize("name,s,e", [("C2", 16, 500), ("C3", 64, 2000)])
def test_exact_scores_equal_reference_goldens(name, s, e):
    """calculate_ll of the golden orders and weights (<= 64 orders: a
    sampler's ll-only call): the reference's ll to the bit."""
    z = golden(f"eval_{name}.npz")
    m = generator.synthetic_nem(s, e, 0)
    eng = Engine.for_nem(m)
    pos = np.array([np.argsort(p) for p in z["perm"]], dtype=np.int32)
    ll = eng.score(pos, expit(z["W"]))
    assert _bits_equal(ll, z["ll"])
    # calculate_ll's column sums and order weights (nem_order_mcmc.py:89-93)
    r = eng.score(pos, expit(z["W"]), want_cs=True, want_ow=True)
    assert _bits_equal(r["ll"], z["ll"]) and _bits_equal(r["cs"], z["cs"])
    assert _bits_equal(r["ow"][0], z["ow0"])
    eng.close()


def test_exact_score_dev_equals_reference_goldens():
    """Option exact_dev: the batched device entry in the reference's
    arithmetic -- the golden ll, cs and order weights to the bit, and the
    host-pointer exact path's bits at a batch of 300."""
    import torch
    z = golden("eval_C3.npz")
    m = generator.synthetic_nem(64, 2000, 0)
    eng = Engine.for_nem(m)
    eng.set_option("exact_dev", 1)
    assert eng.get_option("exact_dev") == 1
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    s, e = 64, 2000

    def run(pos, w01, extras):
        b = pos.shape[0]
        eng.reserve(b)
        dpos = torch.from_numpy(pos).cuda()
        dw = torch.from_numpy(w01).cuda()
        dll = torch.zeros(b, dtype=torch.float64, device="cuda")
        dcs = torch.zeros((b, e), dtype=torch.float64, device="cuda") if extras else None
        dow = torch.zeros((b, s + 1, e), dtype=torch.float64, device="cuda") if extras else None
        _lib.check(lib.nemo_score_dev(eng._ctx, b, dpos.data_ptr(), dw.data_ptr(), 0, dll.data_ptr(),
                                      dcs.data_ptr() if extras else None, None,
                                      dow.data_ptr() if extras else None, st))
        torch.cuda.synchronize()
        return dll.cpu().numpy(), (dcs.cpu().numpy() if extras else None), (dow.cpu().numpy() if extras else None)

    pos = np.array([np.argsort(p) for p in z["perm"]], dtype=np.int32)
    w01 = expit(z["W"])
    ll, cs, ow = run(pos, w01, True)
    assert _bits_equal(ll, z["ll"]) and _bits_equal(cs, z["cs"]) and _bits_equal(ow[0], z["ow0"])
    rng = np.random.default_rng(9)
    pos = np.array([rng.permutation(s) for _ in range(300)], dtype=np.int32)
    w01 = expit(rng.uniform(-6, 6, (300, s, s)))
    ll, _, _ = run(pos, w01, False)
    assert _bits_equal(ll, eng.score(pos, w01))
    # the cells alone (d_cells), against the host-pointer exact path's cells
    b = 5
    dpos = torch.from_numpy(pos[:b]).cuda()
    dw = torch.from_numpy(w01[:b]).cuda()
    dll = torch.zeros(b, dtype=torch.float64, device="cuda")
    dcells = torch.zeros((b, s + 1, e), dtype=torch.float64, device="cuda")
    _lib.check(lib.nemo_score_dev(eng._ctx, b, dpos.data_ptr(), dw.data_ptr(), 0, dll.data_ptr(), None,
                                  dcells.data_ptr(), None, st))
    torch.cuda.synchronize()
    host = eng.score(pos[:b], w01[:b], want_cells=True)
    assert _bits_equal(dcells.cpu().numpy(), host["cells"]) and _bits_equal(dll.cpu().numpy(), host["ll"])
    # cells and order weights share the exact path's one buffer: refused
    with pytest.raises(RuntimeError):
        _lib.check(lib.nemo_score_dev(eng._ctx, b, dpos.data_ptr(), dw.data_ptr(), 0, dll.data_ptr(), None,
                                      dcells.data_ptr(), dcells.data_ptr(), st))
    eng.set_option("exact_dev", 0)   # the fast kernels again: within 1e-6, not the same bits
    ll_fast, _, _ = run(pos, w01, False)
    assert np.max(np.abs(ll_fast - ll)) <= 1e-6
    eng.close()


def test_exact_fused_step_equals_oracle_c3():
    """One get_optimal_weights at 64 x 2000 (2016 local optima) against the
    oracle, i.e. numpy and scipy: every weight, ll and dag_ll to the bit."""
    from nemo.nem_order_mcmc import NEMOrderMCMC
    m = generator.synthetic_nem(64, 2000, 0)
    eng = Engine.for_nem(m)
    t = m.get_score_tensor()
    rng = np.random.default_rng(12)
    perm = rng.permutation(m.num_s)
    smp = NEMOrderMCMC(m, perm, engine=eng)
    w_raw = rng.uniform(-3, 3, (m.num_s, m.num_s))
    smp.parent_weights = w_raw.copy()
    ora = no.OracleSampler(m.U, t, perm)
    ora.w = w_raw.copy()
    ref_dag = ora.optimal_weights()
    got_dag = smp.get_optimal_weights(init=True)
    assert smp.ll == ora.ll1
    assert _bits_equal(smp.parent_weights, ora.w)
    assert got_dag == ref_dag
    eng.close()


@pytest.mark.parametrize("e", [2600, 3900, 4096, 4097, 5000, 9000, 16384, 16392, 40000])
def test_exact_fused_step_equals_oracle_more_slots(e):
    """E past 2048 (more than 16 leaf blocks of numpy's pairwise sum: 3 to 8
    slots of the wave plan; 3900 and 4097 split into 33 leaves, 5000 into 64;
    from 8193 numpy's np.sum adds buffers of 8192 terms, one wave plan each:
    9000 and 16384 in two, 16392 in three, 40000 in five): one
    fused step in the throughput,
    pair and slot forms, with c stored and recomputed, against the oracle, to
    the bit (several plans always take the throughput form, c recomputed)."""
    from nemo.nem_order_mcmc import NEMOrderMCMC
    m = generator.synthetic_nem(12, e, 3)
    eng = Engine.for_nem(m)
    assert eng.get_option("exact_ok") == 1
    t = m.get_score_tensor()
    rng = np.random.default_rng(e)
    perm = rng.permutation(m.num_s)
    w_raw = rng.uniform(-3, 3, (m.num_s, m.num_s))
    ora = no.OracleSampler(m.U, t, perm)
    ora.w = w_raw.copy()
    ref_dag = ora.optimal_weights()
    try:
        for form in (2, 3, 7):
            for cform in (0, 1):
                eng.set_option("exact_form", form)
                eng.set_option("exact_cform", cform)
                smp = NEMOrderMCMC(m, perm, engine=eng)
                smp.parent_weights = w_raw.copy()
                got_dag = smp.get_optimal_weights(init=True)
                assert smp.ll == ora.ll1 and got_dag == ref_dag, (form, cform)
                assert _bits_equal(smp.parent_weights, ora.w), (form, cform)
    finally:
        eng.set_option("exact_form", 0)
        eng.set_option("exact_cform", 1)
        eng.close()


def test_exact_capped_fused_step_equals_oracle_c5():
    """C5's shape, 128 x 5000 with parent cap 6 (the build-defined cap: every
    parent list the last <= 6 predecessors): one fused step against the oracle
    with the same capped lists -- eval #1's ll, every weight and dag_ll to the
    bit -- in both c forms."""
    from nemo.nem_order_mcmc import NEMOrderMCMC
    m = generator.config_nem("C5")
    eng = Engine.for_nem(m)
    assert eng.get_option("exact_ok") == 1
    t = m.get_score_tensor()
    rng = np.random.default_rng(55)
    perm = rng.permutation(m.num_s)
    w_raw = rng.uniform(-3, 3, (m.num_s, m.num_s))
    ora = no.OracleSampler(m.U, t, perm, cap=6)
    ora.w = w_raw.copy()
    ref_dag = ora.optimal_weights()
    try:
        for cform in (1, 0):
            eng.set_option("exact_cform", cform)
            smp = NEMOrderMCMC(m, perm, engine=eng, cap=6)
            smp.parent_weights = w_raw.copy()
            got_dag = smp.get_optimal_weights(init=True)
            assert smp.ll == ora.ll1 and got_dag == ref_dag, cform
            assert _bits_equal(smp.parent_weights, ora.w), cform
    finally:
        eng.set_option("exact_cform", 1)
        eng.close()


def test_exact_capped_step_equals_reference_capture():
    """The capped step pinned to the reference itself (not only to the
    oracle): tests/golden/step_C5cap_40x333.npz holds three
    get_optimal_weights(init=True) steps of the reference with its
    parents_list cut to the last 6 predecessors (the C5 shape on a 40 x 333
    model; nem_order_mcmc.py:172-208, :186-189).  The sampler's fused step
    from W (W~ and ancestor_x on the device) gives the same ll, dag_ll,
    ancestor_x and new weights, and every local optimum the reference's nit
    and nfev, to the bit."""
    from nemo.nem_order_mcmc import NEMOrderMCMC, SIG0, SIG1
    z = golden("step_C5cap_40x333.npz")
    s, e, cap = int(z["S"]), int(z["E"]), int(z["cap"])
    m = generator.synthetic_nem(s, e, int(z["seed"]))
    d = np.unpackbits(z["D_packed"])[: s * e].reshape(s, e)
    assert np.array_equal(m.observed_knockdown_mat, d)
    eng = Engine.for_nem(m)
    assert eng.get_option("exact_ok") == 1
    try:
        for c in range(int(z["n_cases"])):
            perm = z[f"c{c}_perm"]
            smp = NEMOrderMCMC(m, perm, engine=eng, cap=cap)
            smp.parent_weights = np.array(z[f"c{c}_W"], copy=True)
            got_dag = smp.get_optimal_weights(init=True)
            assert smp.ll == z[f"c{c}_ll"] and got_dag == z[f"c{c}_dag_ll"], c
            assert _bits_equal(smp.parent_weights, z[f"c{c}_W_new"]), c
            assert _bits_equal(smp.ancestor_x, z[f"c{c}_anc"]), c
            # the optimiser's own counts, pair by pair
            pos = np.empty(s, dtype=np.int32)
            pos[perm] = np.arange(s)
            *_, info = eng.optimal_weights_w(pos[None], z[f"c{c}_W"][None], SIG0, SIG1, cap=cap,
                                             raise_on_fail=False)
            ik, n = z[f"c{c}_local"], z[f"c{c}_local_n"]
            inf = info[0][ik[:, 0], ik[:, 1]]
            assert np.array_equal((inf >> 4) & 0xfff, n[:, 0]) and np.array_equal(inf >> 16, n[:, 1]), c
            assert ((info[0] != -1).sum()) == len(ik)
    finally:
        eng.close()


def test_exact_capped_scores_equal_golden_c5():
    """The capped order scores of the C5 golden (the reference's own
    calculate_ll with parents_list cut to the last 6 predecessors,
    tests/golden/make_goldens.py): ll and cs to the bit, through the
    sampler's host path and the batched device entry (option exact_dev)."""
    import torch
    z = golden("eval_C5cap.npz")
    m = generator.synthetic_nem(int(z["S"]), int(z["E"]), int(z["seed"]))
    cap = int(z["cap"])
    eng = Engine.for_nem(m)
    pos = np.array([np.argsort(p) for p in z["perm"]], dtype=np.int32)
    w01 = expit(z["W"])
    r = eng.score(pos, w01, cap=cap, want_cs=True)
    assert _bits_equal(r["ll"], z["ll"]) and _bits_equal(r["cs"], z["cs"])
    eng.set_option("exact_dev", 1)
    try:
        b = pos.shape[0]
        eng.reserve(b)
        dpos, dw = torch.from_numpy(pos).cuda(), torch.from_numpy(w01).cuda()
        dll = torch.zeros(b, dtype=torch.float64, device="cuda")
        eng.score_dev(b, dpos.data_ptr(), dw.data_ptr(), dll.data_ptr(), cap=cap,
                      stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert _bits_equal(dll.cpu().numpy(), z["ll"])
    finally:
        eng.set_option("exact_dev", 0)
        eng.close()


def test_exact_score_cells_and_order_weights_together():
    """nemo_score asked for the cells AND the order weights in the exact
    arithmetic (both through one call): the cells of a cells-only call and
    the order weights of an ow-only call, to the bit; with option exact_dev
    set too (the host path never routes through the device entry's
    one-buffer refusal)."""
    m = generator.synthetic_nem(16, 500, 0)
    eng = Engine.for_nem(m)
    rng = np.random.default_rng(21)
    pos = np.array([rng.permutation(16) for _ in range(3)], dtype=np.int32)
    w01 = expit(rng.uniform(-4, 4, (3, 16, 16)))
    cells = eng.score(pos, w01, want_cells=True)["cells"]
    ow = eng.score(pos, w01, want_ow=True)["ow"]
    for dev in (0, 1):
        eng.set_option("exact_dev", dev)
        r = eng.score(pos, w01, want_cells=True, want_ow=True)
        assert _bits_equal(r["cells"], cells) and _bits_equal(r["ow"], ow), dev
    eng.set_option("exact_dev", 0)
    eng.close()


def test_exact_kernel_forms_give_the_same_bits():
    """The local-optimum kernel's latency, throughput, pair, cached
    throughput, dual and slot forms (option exact_form 1 / 2 / 3 / 4 / 5 / 7), c stored or recomputed (exact_cform 0 /
    1), in
    launch order or XCD-contiguous order (exact_xcd): the same weights, dag
    weights and lls, to the bit, for one chain and for three."""
    from nemo.nem_order_mcmc import SIG0, SIG1
    m = generator.synthetic_nem(64, 2000, 0)
    eng = Engine.for_nem(m)
    rng = np.random.default_rng(4)
    for n in (1, 3):
        pos = np.array([rng.permutation(64) for _ in range(n)], dtype=np.int32)
        w = rng.uniform(-3, 3, (n, 64, 64))
        anc = np.clip(rng.random((n, 64, 64)) - 0.5, 0, 1)
        outs = []
        try:
            for form in (1, 2, 3, 4, 5, 7):
                for cform in (0, 1):
                    for xcd in (0, 1):
                        eng.set_option("exact_form", form)
                        eng.set_option("exact_cform", cform)
                        eng.set_option("exact_xcd", xcd)
                        r = eng.optimal_weights(pos, expit(w), anc, w, SIG0, SIG1, raise_on_fail=False)
                        outs.append([np.array(x, copy=True) for x in r])
        finally:
            eng.set_option("exact_form", 0)
            eng.set_option("exact_cform", 1)
            eng.set_option("exact_xcd", 1)
        for o in outs[1:]:
            assert len(o) == len(outs[0])
            for a, b in zip(outs[0], o):
                assert _bits_equal(a, b)
    eng.close()


def test_exact_chain_batch_equals_single_chains():
    """Batched chains (one fused call per step for all) give every chain the
    bits of its own single-chain run, in the exact arithmetic too."""
    from nemo.chains import ChainBatch
    from nemo.nem_order_mcmc import NEMOrderMCMC
    m = generator.synthetic_nem(16, 500, 0)
    eng = Engine.for_nem(m)
    order = np.arange(16)
    cb = ChainBatch(m, [order] * 5, seeds=list(range(5)), engine=eng, on_fail="continue")
    best, _ = cb.run(6)
    for c in (0, 3):
        smp = NEMOrderMCMC(m, order, engine=eng)
        smp.rng = random.Random(c)
        b1, _ = smp.method(n_iterations=6, gamma=2.0 * 16 / 500, swap_prob=0.95, verbose=False)
        assert b1 == best[c]
        assert _bits_equal(smp.parent_weights, cb.chains[c].parent_weights)
    eng.close()


def test_exact_fallback_is_loud():
    """A model outside the exact kernels (generic, non-factored tables)
    reports exact_ok 0, and the sampler says so: a warning, or with
    strict=True an error.  A covered model constructs silently -- E past 8192
    included (numpy's buffers, one plan each)."""
    import warnings
    from nemo.engine import ExactArithmeticWarning
    from nemo.nem_order_mcmc import NEMOrderMCMC
    big = Engine.for_nem(generator.synthetic_nem(3, 9000, 1))
    assert big.get_option("exact_ok") == 1 and big.exact_status() == (True, "")
    big.close()
    m = generator.synthetic_nem(6, 300, 1)
    perm = np.arange(6)
    rng = np.random.default_rng(2)
    gen_eng = Engine(m.U, rng.normal(0, 1, (6, 6, 300)))   # not the factored form
    assert gen_eng.get_option("exact_ok") == 0
    with pytest.warns(ExactArithmeticWarning, match="factored"):
        NEMOrderMCMC(m, perm, engine=gen_eng)
    with pytest.raises(RuntimeError, match="factored"):
        NEMOrderMCMC(m, perm, engine=gen_eng, strict=True)
    gen_eng.close()
    ok_eng = Engine.for_nem(m)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        NEMOrderMCMC(m, perm, engine=ok_eng, strict=True)
    ok_eng.set_option("exact", 0)          # chosen on purpose: not checked
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        NEMOrderMCMC(m, perm, engine=ok_eng, strict=True)
    ok_eng.close()
