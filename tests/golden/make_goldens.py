"""Capture golden vectors from the reference implementation.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference (it never travels to the GPU box).  It imports the reference
modules flat (its __init__.py is broken), with a no-op ``wandb`` stub and the
documented ``opt_weights`` pass-through, and writes small
``.npz`` fixtures next to this script.  The fixtures are data (inputs and the
reference's outputs); no reference source is stored.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py [--only-replica | --only-methods | --only-networks | --only-evals | --only-traj-c3 N | --only-traj-nem
                                                          | --only-c3-extra | --only-capped-step]

Versions at capture: see ``meta.json`` written alongside.
"""
from __future__ import annotations

import hashlib
import json
import os
import platform
import random
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def load_reference():
    if not os.path.isdir(REF):
        raise SystemExit(f"{REF} not present: goldens can only be captured in the build container")
    stub = types.ModuleType("wandb")
    for name in ("init", "log", "login", "finish"):
        setattr(stub, name, lambda *a, **k: None)
    sys.modules.setdefault("wandb", stub)
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import nem as ref_nem
    import nem_order_mcmc as ref_mcmc
    import utils as ref_utils

    def opt_weights_passthrough(self):
        return ref_utils.compute_ll(self.compute_cell_ratios(
            self.create_dag(self.parent_weights)[1], self.score_tables))

    ref_mcmc.NEMOrderMCMC.opt_weights = opt_weights_passthrough
    return ref_nem, ref_mcmc, ref_utils


def quiet(fn, *a, **k):
    """The reference prints every weight pass; silence it."""
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def repo_generator():
    sys.path.insert(0, os.path.join(REPO, "nem-mcmc-optimization_amd"))
    from nemo import generator
    return generator


def ref_nem_without_diagnostics(ref_nem, ref_utils, adj, end_nodes, errors, s, e, seed=42):
    """NEM.__init__ minus compute_real_score (nem.py:21-22, diagnostic only and
    very slow at S>=16): same RNG consumption, same tables."""
    m = ref_nem.NEM.__new__(ref_nem.NEM)
    m.num_s, m.num_e, m.adj_matrix = s, e, adj
    alpha, beta = errors
    m.real_knockdown_mat = ref_utils.create_real_knockdown_mat(adj, end_nodes)
    random.seed(seed)
    m.A = np.log(alpha / (1.0 - beta))
    m.B = np.log(beta / (1.0 - alpha))
    m.observed_knockdown_mat = ref_utils.create_observed_knockdown_mat(m.real_knockdown_mat, alpha, beta)
    m.U = m.get_node_lr_table(m.get_score_tables(m.observed_knockdown_mat))
    return m


def ref_eval(ref_mcmc, m, tables, perm, w_raw, cap=0):
    """compute_cell_ratios + calculate_ll of the reference on (perm, raw W).
    With a cap, parents_list is overridden by the last <= cap predecessors."""
    mc = ref_mcmc.NEMOrderMCMC.__new__(ref_mcmc.NEMOrderMCMC)
    mc.num_s, mc.num_e, mc.U = m.num_s, m.num_e, m.U.copy()
    mc.parent_weights = np.zeros((m.num_s, m.num_s))
    mc.get_permissible_parents(perm, init=True, init_value=1.0)
    if cap:
        capped = np.empty(m.num_s, dtype=object)
        for i, pl in enumerate(mc.parents_list):
            capped[i] = pl[max(0, len(pl) - cap):]
        mc.parents_list = capped
    mc.cell_ratios = mc.compute_cell_ratios(w_raw, tables)
    ow, ll = mc.calculate_ll()
    cs = np.logaddexp.reduce(mc.cell_ratios, axis=0)
    return ll, cs, ow


def capture_evals(ref_nem, ref_mcmc, ref_utils, gen, name, s, e, seed, cap, n_eval, keep_ow):
    """n_eval evaluations with the inputs of tests/golden/eval_inputs.py
    (k < 20: random orders and W ~ U(-3, 3); then saturated, all-0, all-1,
    all-1/2 and mixed 0/1 weights, the identity and reversed orders)."""
    sys.path.insert(0, HERE)
    from eval_inputs import KINDS, eval_inputs
    net = gen.synthetic_network(s, e, seed)
    m = ref_nem_without_diagnostics(ref_nem, ref_utils, net.adj.copy(), net.end_nodes, net.errors, s, e)
    tables = m.get_score_tables(m.observed_knockdown_mat)
    perms, ws, lls, css = [], [], [], []
    ow0 = None
    for c in range(n_eval):
        perm, w = eval_inputs(s, c)
        ll, cs, ow = ref_eval(ref_mcmc, m, tables, perm, w, cap)
        perms.append(perm)
        ws.append(w)
        lls.append(ll)
        css.append(cs)
        if keep_ow and c == 0:
            ow0 = ow
    d = m.observed_knockdown_mat.astype(np.uint8)
    out = dict(S=s, E=e, seed=seed, cap=cap, A=m.A, B=m.B,
               D_packed=np.packbits(d, axis=None),
               U_sha256=hashlib.sha256(np.ascontiguousarray(m.U, dtype=np.float64).tobytes()).hexdigest(),
               perm=np.array(perms), W=np.array(ws), ll=np.array(lls), cs=np.array(css),
               kind=np.array(KINDS[:n_eval]))
    if ow0 is not None:
        out["ow0"] = ow0
    if s <= 16:
        out["U"] = m.U
    np.savez_compressed(os.path.join(HERE, f"eval_{name}.npz"), **out)
    print(f"eval_{name}: S={s} E={e} cap={cap} ll={lls}")


def capture_traj(ref_mcmc, m, order, gamma, swap_prob, n_iter, name, record_local_every=0, use_nem=False):
    """Run the patched reference sampler, recording every proposal and
    decision (and a sample of local optimisations).  ``use_nem``: the
    transitive-closure DAG path of method() (nem_order_mcmc.py:203-204,
    283-284; utils.py:37-54)."""
    rec = {"perm": [], "i1": [], "i2": [], "acc": []}
    local = []
    cls = ref_mcmc.NEMOrderMCMC
    orig_new, orig_acc, orig_loc = cls.get_new_order, cls.accepting, cls.calculate_local_optimum
    counter = {"n": 0}

    def new_order(self, curr, swap_prob=0.95):
        p, i1, i2 = orig_new(self, curr, swap_prob=swap_prob)
        rec["perm"].append(p.copy())
        rec["i1"].append(i1)
        rec["i2"].append(i2)
        return p, i1, i2

    def accepting(self, *a):
        r = orig_acc(self, *a)
        rec["acc"].append(bool(r[0]))
        return r

    def local_opt(self, i, k):
        from scipy.optimize import minimize
        from scipy.special import expit
        counter["n"] += 1
        if record_local_every and counter["n"] % record_local_every == 0:
            lv = np.exp(self.score_tables[i][k])
            a = (lv - 1.0) * self.order_weights[k]
            s = expit(self.parent_weights[i][k])
            b = 1.0 - s * a + s * (lv - 1.0)
            c = a / b
            x0 = expit(self.parent_weights[i][k])
            res = minimize(ref_mcmc.local_ll_sum_penalized, x0=x0, bounds=[(-float("inf"), float("inf"))],
                           args=(c, self.ancestor_x[i][k]), method="L-BFGS-B", tol=0.01)
            out = orig_loc(self, i, k)
            assert out[0] == expit(res.x)[0]
            local.append((c, self.ancestor_x[i][k], x0, res.x[0], res.nit, res.nfev, res.fun))
            return out
        return orig_loc(self, i, k)

    orig_gow = cls.get_optimal_weights
    scores = []

    def gow(self, *a, **k):
        r = orig_gow(self, *a, **k)
        scores.append(r)
        return r

    cls.get_new_order, cls.accepting, cls.calculate_local_optimum = new_order, accepting, local_opt
    cls.get_optimal_weights = gow
    raised = None
    try:
        mc = cls(m, order)
        try:
            best, best_dag = quiet(mc.method, n_iterations=n_iter, gamma=gamma, swap_prob=swap_prob,
                                   use_nem=use_nem)
        except Exception as exc:  # the reference's own failure (nem_order_mcmc.py:168-169)
            if not str(exc).startswith("Minimization not successful"):
                raise
            raised = str(exc)
    finally:
        cls.get_new_order, cls.accepting, cls.calculate_local_optimum = orig_new, orig_acc, orig_loc
        cls.get_optimal_weights = orig_gow
    if raised is not None:
        # method() raised inside step len(rec["perm"]) (1-based: proposals made);
        # keep what was decided before it: every proposal, every accept, the
        # scores of the completed steps (scores[0] is the initial pass, whose
        # value opt_weights then replaces), the random state at the raise
        steps = len(rec["acc"])
        out = dict(order0=np.asarray(order), gamma=gamma, swap_prob=swap_prob, n_iter=n_iter, use_nem=use_nem,
                   raised=raised, raised_in_step=len(rec["perm"]), steps_completed=steps,
                   perm=np.array(rec["perm"]), i1=np.array(rec["i1"]), i2=np.array(rec["i2"]),
                   acc=np.array(rec["acc"]), step_scores=np.array(scores[1:1 + steps]),
                   W_at_raise=mc.parent_weights, rng_state_at_raise=np.array(random.getstate()[1], dtype=np.int64))
        np.savez_compressed(os.path.join(HERE, f"traj_{name}.npz"), **out)
        print(f"traj_{name}: raised in step {len(rec['perm'])} after {steps} completed steps: {raised}")
        return
    out = dict(order0=np.asarray(order), gamma=gamma, swap_prob=swap_prob, n_iter=n_iter,
               perm=np.array(rec["perm"]), i1=np.array(rec["i1"]), i2=np.array(rec["i2"]),
               acc=np.array(rec["acc"]), all_scores=np.array(mc.all_score_list),
               curr_scores=np.array(mc.curr_score_list), best_scores=np.array(mc.best_score_list),
               best_score=best, best_order=np.asarray(mc.best_order), final_W=mc.parent_weights,
               best_dag=np.asarray(best_dag), use_nem=use_nem,
               rng_state_after=np.array(random.getstate()[1], dtype=np.int64))
    np.savez_compressed(os.path.join(HERE, f"traj_{name}.npz"), **out)
    print(f"traj_{name}: best={best} accepts={int(np.sum(rec['acc']))}")
    if local:
        e = len(local[0][0])
        np.savez_compressed(
            os.path.join(HERE, f"localopt_{name}.npz"),
            c=np.array([r[0] for r in local]).reshape(-1, e), anc=np.array([r[1] for r in local]),
            x0=np.array([r[2] for r in local]), xstar=np.array([r[3] for r in local]),
            nit=np.array([r[4] for r in local]), nfev=np.array([r[5] for r in local]),
            fun=np.array([r[6] for r in local]))
        print(f"localopt_{name}: {len(local)} records")


def capture_capped_step(ref_nem, ref_mcmc, ref_utils, gen, s=40, e=333, cap=6, n_cases=3, seed=0):
    """The capped fused step (the build-defined C5 shape):
    one get_optimal_weights(init=True) (nem_order_mcmc.py:172-208) per case on
    a reference sampler whose parents_list is cut to the last <= cap
    predecessors, as ``ref_eval`` cuts it for eval_C5cap -- the cell ratios,
    expit_parent_weights (ancestor_x), the local optima (:186-189) and the
    dag's score all read that list.  Recorded per case: the inputs (perm, raw
    W), the step's ll, dag_ll, ancestor_x, the new weights and, per local
    optimum in the reference's loop order, (i, k, x0, anc, x*, nit, nfev, f*)."""
    from scipy.optimize import minimize
    from scipy.special import expit
    net = gen.synthetic_network(s, e, seed)
    m = ref_nem_without_diagnostics(ref_nem, ref_utils, net.adj.copy(), net.end_nodes, net.errors, s, e)
    tables = m.get_score_tables(m.observed_knockdown_mat)
    rng = np.random.default_rng(4242)
    out = dict(S=s, E=e, seed=seed, cap=cap, A=m.A, B=m.B,
               D_packed=np.packbits(m.observed_knockdown_mat.astype(np.uint8), axis=None))
    for case in range(n_cases):
        perm = rng.permutation(s)
        w_raw = rng.uniform(-3, 3, (s, s))
        mc = ref_mcmc.NEMOrderMCMC.__new__(ref_mcmc.NEMOrderMCMC)
        mc.num_s, mc.num_e, mc.U = s, e, m.U.copy()
        mc.score_tables = tables
        mc.I = np.identity(s)
        mc.parent_weights = np.zeros((s, s))
        mc.get_permissible_parents(perm, init=True, init_value=1.0)
        capped = np.empty(s, dtype=object)
        for i, pl in enumerate(mc.parents_list):
            capped[i] = pl[max(0, len(pl) - cap):]
        mc.parents_list = capped
        mc.parent_weights = w_raw.copy()
        recs = []
        orig = mc.calculate_local_optimum

        def local_opt(i, k, mc=mc, orig=orig, recs=recs):
            lv = np.exp(mc.score_tables[i][k])
            a = (lv - 1.0) * mc.order_weights[k]
            sg = expit(mc.parent_weights[i][k])
            c = a / (1.0 - sg * a + sg * (lv - 1.0))
            res = minimize(ref_mcmc.local_ll_sum_penalized, x0=sg, bounds=[(-float("inf"), float("inf"))],
                           args=(c, mc.ancestor_x[i][k]), method="L-BFGS-B", tol=0.01)
            got = orig(i, k)
            assert got[0] == expit(res.x)[0]
            recs.append((i, k, sg, mc.ancestor_x[i][k], res.x[0], res.nit, res.nfev, res.fun))
            return got
        mc.calculate_local_optimum = local_opt
        dag_ll = quiet(mc.get_optimal_weights, init=True)
        out[f"c{case}_perm"] = perm
        out[f"c{case}_W"] = w_raw
        out[f"c{case}_ll"] = mc.ll
        out[f"c{case}_dag_ll"] = dag_ll
        out[f"c{case}_anc"] = mc.ancestor_x
        out[f"c{case}_W_new"] = mc.parent_weights
        out[f"c{case}_local"] = np.array([r[:2] for r in recs], dtype=np.int64)
        out[f"c{case}_local_f"] = np.array([r[2:5] + (r[7],) for r in recs], dtype=np.float64)
        out[f"c{case}_local_n"] = np.array([r[5:7] for r in recs], dtype=np.int64)
        print(f"capped step case {case}: ll={mc.ll} dag_ll={dag_ll} optima={len(recs)}")
    np.savez_compressed(os.path.join(HERE, f"step_C5cap_{s}x{e}.npz"), n_cases=n_cases, **out)


def capture_replica_exchange(ref_nem, ref_mcmc, ref_utils, n_exchange=3, n_iter=4, seed=2024, model=None,
                             name="net2"):
    """replica_exchange_method (nem_order_mcmc.py:344-363) on net2 (or on the
    given (model, order)): 10 replicas, gamma_r = (1 + 0.2 r) S / E,
    `n_exchange` rounds of `n_iter` steps.  Each round's replica_exchange_step
    result is recorded through a wrapper of the module-level function (the
    reference itself runs unchanged)."""
    if model is None:
        adj, end, err, s, e = ref_utils.read_csv_to_adj(os.path.join(REF, "DAGs/networks/network2/network2.csv"))
        m = quiet(ref_nem.NEM, adj, end, err, s, e)
        order = ref_utils.initial_order_guess(m.observed_knockdown_mat)
    else:
        m, order = model
    rounds = []
    orig = ref_mcmc.replica_exchange_step

    def recording_step(replicas, gammas, n_replicas, n_iters, scores, upwards):
        out = orig(replicas, gammas, n_replicas, n_iters, scores, upwards)
        best_score, best_nem, reps, sc, nex = out
        rounds.append(dict(scores=np.array(sc, dtype=float), n_ex=nex, best=best_score,
                           orders=np.array([np.asarray(r.perm_order) for r in reps]),
                           best_orders=np.array([np.asarray(r.best_order) for r in reps])))
        return out

    random.seed(seed)
    ref_mcmc.replica_exchange_step = recording_step
    try:
        best_score, best_nem = quiet(ref_mcmc.replica_exchange_method, m, n_exchange, n_iter, order)
    finally:
        ref_mcmc.replica_exchange_step = orig
    np.savez_compressed(
        os.path.join(HERE, f"replica_{name}.npz"), seed=seed, n_exchange=n_exchange, n_iter=n_iter,
        order0=order, best_score=best_score, best_dag=np.asarray(best_nem.best_dag),
        best_order=np.asarray(best_nem.best_order),
        round_scores=np.array([r["scores"] for r in rounds]), round_nex=np.array([r["n_ex"] for r in rounds]),
        round_best=np.array([r["best"] for r in rounds]), round_orders=np.array([r["orders"] for r in rounds]),
        round_best_orders=np.array([r["best_orders"] for r in rounds]),
        rng_state_after=np.array(random.getstate()[1], dtype=np.int64))
    print("replica exchange:", best_score, [r["n_ex"] for r in rounds])


def capture_methods(ref_nem, ref_utils, gen):
    """The fixed-order optimizers of methods.py:
    ``Method.optimize`` (methods.py:407-436) and ``InverseMethod.optimize``
    (:131-172) on net2 and C2 from the initial order guess.  Recorded per
    weight sweep (opt_gamma :397-405 / opt_b :117-129): the sweep's ll and
    the weights it returns; and the optimizers' outputs."""
    import methods as ref_methods
    out = {}
    adj, end, err, s, e = ref_utils.read_csv_to_adj(os.path.join(REF, "DAGs/networks/network2/network2.csv"))
    m2 = quiet(ref_nem.NEM, adj, end, err, s, e)
    net = gen.synthetic_network(16, 500, 0)
    mc2 = ref_nem_without_diagnostics(ref_nem, ref_utils, net.adj.copy(), net.end_nodes, net.errors, 16, 500)
    for name, m, iters in (("net2", m2, {"gamma": 1000, "inverse": 1000}),
                           ("C2", mc2, {"gamma": 60, "inverse": 1000})):
        tables = m.get_score_tables(m.observed_knockdown_mat)
        order = ref_utils.initial_order_guess(m.observed_knockdown_mat)
        for kind, cls, sweep in (("gamma", ref_methods.Method, "opt_γ"),
                                 ("inverse", ref_methods.InverseMethod, "opt_b")):
            meth = cls(order, m.num_s, m.num_e, m.U, tables)
            lls, ws = [], []
            orig = getattr(meth, sweep)

            def rec(weights, bounds, orig=orig, lls=lls, ws=ws):
                ll, w = orig(weights, bounds)
                lls.append(ll)
                ws.append(np.array(w, dtype=np.float64))
                return ll, w
            setattr(meth, sweep, rec)
            dag, real_ll = quiet(meth.optimize, max_iter=iters[kind])
            keep = min(len(ws), 40)
            np.savez_compressed(
                os.path.join(HERE, f"methods_{kind}_{name}.npz"), S=m.num_s, E=m.num_e, order=order,
                D=m.observed_knockdown_mat.astype(np.uint8), A=m.A, B=m.B, max_iter=iters[kind],
                sweep_ll=np.array(lls), sweep_w=np.array(ws[:keep]), last_w=ws[-1],
                dag=np.asarray(dag), real_ll=real_ll)
            out[(name, kind)] = (len(lls), real_ll)
            print(name, kind, "sweeps", len(lls), "real_ll", real_ll, flush=True)
    return out


def capture_networks(ref_nem, ref_mcmc, ref_utils, n_iter=10):
    """The bundled networks 0-19 (DAGs/networks).
    Copies each network's data files (closure CSV, reduced CSV and the DOT
    files the reference's DAGs/dot.py:4-26 made from them) into
    ``networks/``, and records per network a short run of main.py's MCMC
    configuration (initial_order_guess, gamma = 2S/E, swap_prob 0.90,
    main.py:62-70) with the DOT text output_handling (main.py:44-53) writes
    for the best DAG (DAGs/dot.py:28-42)."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(REF, "DAGs"))
    import dot as ref_dot
    dst = os.path.join(HERE, "networks")
    os.makedirs(dst, exist_ok=True)
    out = {}
    for i in range(20):
        base = os.path.join(REF, f"DAGs/networks/network{i}/network{i}")
        for suffix in (".csv", ".dot", "_red.csv", "_red.dot"):
            shutil.copyfile(base + suffix, os.path.join(dst, f"network{i}{suffix}"))
        adj, end, err, s, e = ref_utils.read_csv_to_adj(base + ".csv")
        m = ref_nem_without_diagnostics(ref_nem, ref_utils, adj, end, err, s, e)
        order = ref_utils.initial_order_guess(m.observed_knockdown_mat)
        acc = []
        cls = ref_mcmc.NEMOrderMCMC
        orig_acc = cls.accepting

        def accepting(self, *a, orig_acc=orig_acc, acc=acc):
            r = orig_acc(self, *a)
            acc.append(bool(r[0]))
            return r
        cls.accepting = accepting
        try:
            mc = cls(m, order)
            best, best_dag = quiet(mc.method, n_iterations=n_iter, gamma=2.0 * s / e, swap_prob=0.90)
        finally:
            cls.accepting = orig_acc
        texts = []
        cwd = os.getcwd()
        with tempfile.TemporaryDirectory() as td:
            os.makedirs(os.path.join(td, "x"))
            for k, mat in enumerate((ref_utils.ancestor(best_dag), ref_utils.transitive_reduction(best_dag))):
                os.chdir(os.path.join(td, "x"))  # generate_dot_from_matrix changes directory to '../'
                path = os.path.join(td, f"o{k}.dot")
                quiet(ref_dot.generate_dot_from_matrix, mat, path)
                with open(path) as fh:
                    texts.append(fh.read())
        os.chdir(cwd)
        out.update({f"n{i}_order0": np.asarray(order), f"n{i}_all_scores": np.array(mc.all_score_list),
                    f"n{i}_acc": np.array(acc), f"n{i}_best_score": best,
                    f"n{i}_best_order": np.asarray(mc.best_order), f"n{i}_best_dag": np.asarray(best_dag),
                    f"n{i}_closed_dot": np.array(texts[0]), f"n{i}_red_dot": np.array(texts[1]),
                    f"n{i}_D_packed": np.packbits(m.observed_knockdown_mat.astype(np.uint8), axis=None)})
        print(f"network{i}: S={s} E={e} best={best} accepts={sum(acc)}", flush=True)
    np.savez_compressed(os.path.join(HERE, "networks_mcmc.npz"), n_iter=n_iter, **out)


def main():
    import scipy
    ref_nem, ref_mcmc, ref_utils = load_reference()
    if "--only-networks" in sys.argv:
        capture_networks(ref_nem, ref_mcmc, ref_utils)
        return
    if "--only-replica" in sys.argv:
        capture_replica_exchange(ref_nem, ref_mcmc, ref_utils)
        return
    gen = repo_generator()
    if "--only-methods" in sys.argv:
        capture_methods(ref_nem, ref_utils, gen)
        return
    if "--only-traj-c3" in sys.argv:
        # C3 trajectory (the headline model, 64 x 2000): default swap_prob 0.95,
        # gamma = 2S/E, as the C2 one
        n_iter = int(sys.argv[sys.argv.index("--only-traj-c3") + 1])
        net = gen.synthetic_network(64, 2000, 0)
        mc3 = ref_nem_without_diagnostics(ref_nem, ref_utils, net.adj.copy(), net.end_nodes, net.errors, 64, 2000)
        order3 = ref_utils.initial_order_guess(mc3.observed_knockdown_mat)
        capture_traj(ref_mcmc, mc3, order3, 2.0 * 64 / 2000, 0.95, n_iter, f"C3_{n_iter}")
        return
    if "--only-traj-nem" in sys.argv:
        # C1's model and stream (net2, full constructor, post-NEM state as in
        # main()), method(use_nem=True), main.py's swap_prob 0.90 and gamma 2S/E
        adj, end, err, s, e = ref_utils.read_csv_to_adj(os.path.join(REF, "DAGs/networks/network2/network2.csv"))
        m = quiet(ref_nem.NEM, adj, end, err, s, e)
        order = ref_utils.initial_order_guess(m.observed_knockdown_mat)
        capture_traj(ref_mcmc, m, order, 2.0 * s / e, 0.90, 50, "net2_nem_50", use_nem=True)
        return
    if "--only-c3-extra" in sys.argv:
        # the headline model (C3, 64 x 2000): replica_exchange_method with 10
        # replicas, 2 exchange rounds of 3 steps, and a 20-step
        # method(use_nem=True) trajectory (default swap_prob 0.95, gamma 2S/E)
        net = gen.synthetic_network(64, 2000, 0)
        mc3 = ref_nem_without_diagnostics(ref_nem, ref_utils, net.adj.copy(), net.end_nodes, net.errors, 64, 2000)
        order3 = ref_utils.initial_order_guess(mc3.observed_knockdown_mat)
        capture_replica_exchange(ref_nem, ref_mcmc, ref_utils, n_exchange=2, n_iter=3, seed=2025,
                                 model=(mc3, order3), name="C3")
        random.seed(77)
        capture_traj(ref_mcmc, mc3, order3, 2.0 * 64 / 2000, 0.95, 20, "C3_nem_20", use_nem=True)
        return
    if "--only-capped-step" in sys.argv:
        capture_capped_step(ref_nem, ref_mcmc, ref_utils, gen)
        return
    if "--only-evals" in sys.argv:
        capture_evals(ref_nem, ref_mcmc, ref_utils, gen, "C3", 64, 2000, 0, 0, 32, True)
        capture_evals(ref_nem, ref_mcmc, ref_utils, gen, "C5cap", 128, 5000, 0, 6, 32, False)
        return

    # KAT from the reference's own test (tests/utils.tests.py:11-27): data only.
    s_mat = np.array([[0, 1, 1, 0, 1, 0], [0, 0, 1, 0, 1, 0], [0, 0, 0, 0, 1, 0],
                      [0, 0, 1, 0, 1, 0], [0, 0, 0, 0, 0, 0], [0, 0, 0, 0, 1, 0]])
    e_arr = np.array([0, 1, 2, 3, 4, 5, 0])
    got = ref_utils.create_real_knockdown_mat(s_mat.tolist(), e_arr.tolist())
    np.savez_compressed(os.path.join(HERE, "kat_knockdown.npz"), s_mat=s_mat, e_arr=e_arr, expected=got)

    # net2 (C1): full reference constructor
    adj, end, err, s, e = ref_utils.read_csv_to_adj(os.path.join(REF, "DAGs/networks/network2/network2.csv"))
    adj_in = adj.copy()
    m = quiet(ref_nem.NEM, adj, end, err, s, e)
    tables = np.array(m.get_score_tables(m.observed_knockdown_mat))
    order = ref_utils.initial_order_guess(m.observed_knockdown_mat)
    np.savez_compressed(
        os.path.join(HERE, "net2_tables.npz"), adj_in=adj_in, adj_after=adj, end_nodes=end, errors=err,
        S=s, E=e, D=m.observed_knockdown_mat.astype(np.uint8), D_real=m.real_knockdown_mat.astype(np.uint8),
        A=m.A, B=m.B, U=m.U, T=tables, order0=order,
        rng_state_after_nem=np.array(random.getstate()[1], dtype=np.int64),
        real_order_ll=m.real_order_ll, real_ll=m.real_ll, obs_order_ll=m.obs_order_ll, obs_ll=m.obs_ll)
    # eval fixtures on net2
    perms, ws, lls, css = [], [], [], []
    for c in range(8):
        perm, _pos, w = gen.random_chain_inputs(s, c)
        ll, cs, ow = ref_eval(ref_mcmc, m, list(tables), perm, w)
        perms.append(perm), ws.append(w), lls.append(ll), css.append(cs)
        if c == 0:
            ow0 = ow
    np.savez_compressed(os.path.join(HERE, "eval_net2.npz"), S=s, E=e, cap=0, perm=np.array(perms),
                        W=np.array(ws), ll=np.array(lls), cs=np.array(css), ow0=ow0)

    # C1 trajectory: net2, 200 steps, gamma = 2S/E, swap_prob 0.90 (main.py:66-70)
    random.setstate(random.getstate())  # state is the post-NEM state, as in main()
    capture_traj(ref_mcmc, m, order, 2.0 * s / e, 0.90, 200, "net2_200", record_local_every=5)

    # synthetic evals: C2, C3, C5 (cap 6, reference fp64)
    capture_evals(ref_nem, ref_mcmc, ref_utils, gen, "C2", 16, 500, 0, 0, 8, True)
    capture_evals(ref_nem, ref_mcmc, ref_utils, gen, "C3", 64, 2000, 0, 0, 32, True)
    capture_evals(ref_nem, ref_mcmc, ref_utils, gen, "C5cap", 128, 5000, 0, 6, 32, False)

    # C2 trajectory, 20 steps (default swap_prob 0.95, gamma = 2S/E)
    net = gen.synthetic_network(16, 500, 0)
    mc2 = ref_nem_without_diagnostics(ref_nem, ref_utils, net.adj.copy(), net.end_nodes, net.errors, 16, 500)
    order2 = ref_utils.initial_order_guess(mc2.observed_knockdown_mat)
    capture_traj(ref_mcmc, mc2, order2, 2.0 * 16 / 500, 0.95, 20, "C2_20", record_local_every=7)

    capture_replica_exchange(ref_nem, ref_mcmc, ref_utils)
    capture_methods(ref_nem, ref_utils, gen)
    capture_networks(ref_nem, ref_mcmc, ref_utils)

    meta = dict(python=platform.python_version(), numpy=np.__version__, scipy=scipy.__version__,
                machine=platform.machine(), processor=platform.processor(), reference=REF)
    with open(os.path.join(HERE, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    print(meta)


if __name__ == "__main__":
    main()
