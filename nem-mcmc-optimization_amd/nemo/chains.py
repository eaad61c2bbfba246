"""Independent chains: lock-step batching on one GPU, sharding over GPUs.

The reference runs one chain per process and its replicas sequentially
(nem_order_mcmc.py:316-363).  Here every chain keeps the reference's
per-chain state machine (``NEMOrderMCMC``'s proposal / reset / accept logic
with its own ``random.Random`` stream), and the chains of one GPU advance in
lock-step so each MCMC step is ONE batched ``nemo_optimal_weights`` call for
all of them.  Chains shard over GPUs with no data-path collective; the only
exchange is one all-gather of per-chain (best score, best order) at the end
(BASELINE config C4), over RCCL on GPUs or gloo on CPU.
"""
from __future__ import annotations

import random

import numpy as np
from scipy.linalg import inv
from scipy.special import expit

from .engine import Engine
from .nem_order_mcmc import SIG0, SIG1, NEMOrderMCMC, draw_swap, permissible_batch, reset_weights_batch


def shard(n_chains: int, rank: int, world: int) -> range:
    """Contiguous block of global chain ids owned by ``rank``."""
    base, extra = divmod(n_chains, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


_LAPACK = {}


def inv_stack(a):
    """``scipy.linalg.inv`` of every matrix of a stack, bit for bit: the same
    LAPACK getrf + getri calls with scipy's lwork (scipy/linalg/_basic.py
    inv), minus its per-call validation."""
    n = a.shape[-1]
    if n not in _LAPACK:
        from scipy.linalg import get_lapack_funcs
        from scipy.linalg.lapack import _compute_lwork
        getrf, getri, getri_lwork = get_lapack_funcs(("getrf", "getri", "getri_lwork"), (a[0],))
        _LAPACK[n] = (getrf, getri, int(1.01 * _compute_lwork(getri_lwork, n)))
    getrf, getri, lwork = _LAPACK[n]
    out = np.empty_like(a)
    for k in range(a.shape[0]):
        if not np.all(np.isfinite(a[k])):
            out[k] = inv(a[k])  # scipy's own error behaviour
            continue
        lu, piv, info = getrf(a[k])
        if info == 0:
            out[k], info = getri(lu, piv, lwork=lwork, overwrite_lu=1)
        if info != 0:
            out[k] = inv(a[k])  # scipy raises the reference's LinAlgError
    return out


def propose_batch(chains, curr_perms, swap_prob=0.95, w=None):
    """``get_new_order`` then ``reset(perm, i1, i2)`` (nem_order_mcmc.py:
    231-255, :50-77) of every chain of a group: each chain draws from its own
    stream in the reference's order, and the array work (the swap, positions,
    permissible masks, the weight resets) runs once over the group's stacked
    arrays.  Leaves every chain in the state its own calls would (same
    arrays, same bits; its weights, positions and mask are views of the
    group's stacks).  Returns the proposed orders and the stacks
    (pos, weights, mask).  ``w``: a stack whose rows ARE the chains' current
    weights (the last step's output); the reset then updates it in place, as
    the reference updates ``self.parent_weights``."""
    n = len(chains)
    s = chains[0].num_s
    ar = np.arange(n)
    ij = np.array([draw_swap(c.rng, s, swap_prob) for c in chains], dtype=np.int64).reshape(n, 2)
    perm = np.stack(curr_perms)
    # i1, i2: the positions of the LABELS i, j in the current order
    pos_c = np.empty_like(perm, dtype=np.int64)
    pos_c[ar[:, None], perm] = np.arange(s)
    i1, i2 = pos_c[ar, ij[:, 0]], pos_c[ar, ij[:, 1]]
    # ...while the swap exchanges POSITIONS i, j (as written)
    a, b = perm[ar, ij[:, 0]], perm[ar, ij[:, 1]]
    perm[ar, ij[:, 0]], perm[ar, ij[:, 1]] = b, a
    pos = np.empty((n, s), dtype=np.int64)
    pos[ar[:, None], perm] = np.arange(s)
    mask = permissible_batch(pos, chains[0].cap)
    if w is None:
        w = np.stack([c.parent_weights for c in chains])
    reset_weights_batch(w, mask, i1, i2)
    perms = list(perm)
    for k, c in enumerate(chains):
        c.ll = 0.0
        c.parent_weights = w[k]
        c._perm, c._pos, c._mask = perms[k], pos[k], mask[k]
        c._parents = None
    return perms, (pos, w, mask)


def _prepare_start(chains, pool=None, stacks=None):
    """First half of ``_prepare``.  With an ``InvPool`` the per-chain work
    (expit, inversion, clip) starts in its workers.  ``stacks``: the
    group's (pos, weights, mask) stacks when they exist (propose_batch)."""
    if stacks is None:
        stacks = (np.stack([c._pos for c in chains]), np.stack([c.parent_weights for c in chains]),
                  np.stack([c._mask for c in chains]))
    pos, w, mask = stacks
    pos = pos.astype(np.int32)
    if pool is not None:
        pool.start_prepare(w, mask)
        return pos, w, None
    sig = w.copy()
    sig[mask] = expit(w[mask])
    eye = np.identity(chains[0].num_s)
    return pos, w, (sig, np.clip(inv_stack(eye - sig) - eye, 0, 1))


def _prepare_end(chains, part, pool=None):
    pos, w, rest = part
    sig, anc = pool.finish_prepare() if rest is None else rest
    for k, c in enumerate(chains):
        c.ll = 0.0
        c.ancestor_x = anc[k]
    return pos, w, sig, anc


def _prepare(chains, pool=None):
    """Host inputs of ``get_optimal_weights`` for a group of chains: positions,
    weights, expit(weights) and ancestor_x = clip(inv(I - W~) - I, 0, 1) with W~
    the weights under expit on the permissible entries only
    (nem_order_mcmc.py:98-103, :185).  W~ doubles as the device's w01: the
    kernels read it at permissible (child, parent) entries only, where it is
    expit(W); expit runs on those entries alone (scipy's ufunc is elementwise,
    so the bits are those of expit over the whole matrix).  The inversions run
    in ``pool``'s worker processes when one is given (same LAPACK calls, same
    bits: nemo/invpool.py)."""
    return _prepare_end(chains, _prepare_start(chains, pool), pool)


def _device_step(engine: Engine, prep, cap, raise_on_fail):
    pos, w, w01, anc = prep
    return engine.optimal_weights(pos, w01, anc, w, SIG0, SIG1, cap=cap, raise_on_fail=raise_on_fail)


def _finish(chains, engine: Engine, prep, res, use_nem, cap):
    pos, _w, w01, _anc = prep   # w01 None: made from W when the chain's order weights are read
    w_new, ll1, lld, _ = res
    out = np.empty(len(chains))
    for k, c in enumerate(chains):
        c._set_eval1(pos[k], None if w01 is None else w01[k], _w[k])
        c.parent_weights = w_new[k]   # a fresh array per call: the views are private
        c.ll = float(ll1[k])
        if use_nem:
            _, dag = c.create_nem(c.parent_weights)
            out[k] = float(engine.score(c._pos[None, :], expit(dag.astype(float))[None], cap=cap)[0])
        else:
            out[k] = float(lld[k])
    return out


def _device_ancestor(engine: Engine, pool) -> bool:
    """W~ and ancestor_x made on the device (nemo_optimal_weights_w, S <= 64)
    unless an ``InvPool`` is given: then the host makes them in its workers."""
    return pool is None and engine.device_ancestor


def _w_call_end(chains, call, raise_on_fail, drain=None):
    """The result of an ended ``nemo_optimal_weights_w`` call and the prep tuple
    ``_finish`` takes; sets every chain's ancestor_x.  A non-finite value inside
    the device's factorisation (never met on the sampler's matrices) reruns the
    step with the host's ancestor_x, after ``drain()`` has ended every call
    queued behind it."""
    from .engine import AncestorRecompute
    try:
        res = call.result(raise_on_fail)
    except AncestorRecompute:
        if drain is not None:
            drain()
        call.recompute()
        res = call.result(raise_on_fail)
    for k, c in enumerate(chains):
        c.ll = 0.0
        if call.anc is not None:
            c.ancestor_x = call.anc[k]
        else:   # made on the host, same bits, if ever read
            c._set_ancestor_src(call.pos[k], call.w[k])
    return (call.pos, call.w, call.w01, call.anc), res


def optimal_weights_batch(chains, engine: Engine, use_nem=False, cap=0, raise_on_fail=True, pool=None):
    """``get_optimal_weights(init=True)`` (nem_order_mcmc.py:172-208) of every
    chain in ONE fused device call; each chain's state is updated exactly as
    its own call would (same kernels, batch-invariant bits).  A failed local
    optimisation raises the reference's Exception (nem_order_mcmc.py:168-169);
    with ``raise_on_fail=False`` the step keeps the optimiser's last point.
    W~ and ancestor_x come from the device (S <= 64, no ``pool``) or the host."""
    if _device_ancestor(engine, pool):
        pos = np.stack([c._pos for c in chains]).astype(np.int32)
        w = np.stack([c.parent_weights for c in chains])
        call = engine.bind_optimal_weights_w(pos, w, SIG0, SIG1, cap=cap, want_prep=False)
        call.run()
        prep, res = _w_call_end(chains, call, raise_on_fail)
        return _finish(chains, engine, prep, res, use_nem, cap)
    prep = _prepare(chains, pool)
    return _finish(chains, engine, prep, _device_step(engine, prep, cap, raise_on_fail), use_nem, cap)


def opt_weights_batch(chains, engine: Engine, cap=0):
    """The documented ``opt_weights`` pass-through of every
    chain in one batched score call: the score of its binarised weights."""
    pos = np.stack([c._pos for c in chains]).astype(np.int32)
    w01d = np.stack([expit(np.asarray(c.create_dag(c.parent_weights)[1], dtype=np.float64))
                     for c in chains])
    ll = engine.score(pos, w01d, cap=cap)
    for k, c in enumerate(chains):
        c.ll = float(ll[k])
    return np.asarray(ll, dtype=np.float64)


def run_methods(chains, gammas, n_iterations, engine: Engine, swap_prob=0.95, use_nem=False, cap=0,
                raise_on_fail=True, pool=None, state=None, return_state=False, groups=None):
    """``NEMOrderMCMC.method`` (nem_order_mcmc.py:257-310) of every chain, in
    lock-step: each MCMC step is one fused device call per chain group.  Chain k
    draws from ``chains[k].rng`` in the reference's call order, and ends with
    the attributes its own ``method`` call would leave (best_score, best_dag,
    best_order, score lists, parents_list of the best order).  Returns the
    per-chain best scores (and, with ``return_state``, the loop state:
    passed back as ``state`` it continues the same run as if it had not
    stopped -- ``ChainBatch.run(n, resume=True)`` and its checkpoints).  If a local optimisation fails and
    ``raise_on_fail`` is set, the reference's Exception propagates and the
    chains' states are unspecified afterwards (see the pipeline below).
    ``pool`` (an ``InvPool``) runs the ancestor_x inversions in worker
    processes instead of the device (which makes them at S <= 64); the results
    do not change.  ``groups``: the number of chain
    groups in the pipeline below (default 3 from 6 chains, else 2)."""
    n = len(chains)
    s = chains[0].num_s
    if state is None:
        optimal_weights_batch(chains, engine, use_nem=use_nem, cap=cap, raise_on_fail=raise_on_fail, pool=pool)
        curr = list(opt_weights_batch(chains, engine, cap=cap))
        st = []
        for k, c in enumerate(chains):
            dag, _ = c.create_dag(c.parent_weights)
            st.append(dict(best=curr[k], best_dag=dag, curr_perm=c.perm_order, best_order=c.perm_order,
                           best_order_list=[c.perm_order], curr_dag=np.zeros((s, s)),
                           curr_list=[curr[k]], best_list=[curr[k]], all_list=[curr[k]],
                           best_parents=c.parents_list.copy(), best_struct=(c._pos, c._mask), acc=[]))
    else:
        st, curr = state["st"], state["curr"]
    props = [None] * n

    def propose(idx, w=None):
        perms, stacks = propose_batch([chains[k] for k in idx], [st[k]["curr_perm"] for k in idx],
                                      swap_prob, w=w)
        for j, k in enumerate(idx):
            props[k] = perms[j]
        return stacks

    def post(idx, lls):
        for j, k in enumerate(idx):
            c, q = chains[k], st[k]
            ll = float(lls[j])
            q["all_list"].append(ll)
            q["curr_list"].append(curr[k])
            # the proposal's DAG (create_dag / create_nem, nem_order_mcmc.py:
            # 210-221) is kept only when accepted: built after the draw
            acc, curr[k], q["curr_dag"], q["curr_perm"] = c.accepting(
                ll, curr[k], gammas[k], None, q["curr_dag"], props[k], q["curr_perm"])
            q["acc"].append(acc)
            if acc:
                dag = c.create_nem(c.parent_weights)[0] if use_nem else c.create_dag(c.parent_weights)[0]
                q["curr_dag"] = dag
                if curr[k] > q["best"]:
                    q["best"] = curr[k]
                    q["best_dag"] = dag
                    q["best_order"] = q["curr_perm"].copy()
                    q["best_parents"] = None   # parents_list of this order: built at the end
                    q["best_perm"] = c._perm
                    q["best_struct"] = (c._pos, c._mask)
                    q["best_list"].append(q["best"])
                    q["best_order_list"].append(q["best_order"])

    # Chain groups in a software pipeline: the device step of a group runs on
    # the library's step thread (nemo_optimal_weights[_w]_begin / _end) while
    # the host accepts / proposes / resets the others.  Per group: propose,
    # (host ancestor_x only: hand it to the pool's workers, finish the oldest
    # running group while they compute,) then queue this group's step.  With
    # three or more groups one more step stays queued on the device while the
    # host does that, so the device goes from group to group without waiting
    # for the host; with two, the step is queued before the other one is
    # finished instead.
    # Chains are independent and results are batch-invariant, so the bits are
    # those of one batch; use_nem scores on the device in the host phase, so it runs
    # unpipelined.  A failed local optimisation of one group surfaces when
    # that group is finished, after others have already proposed their
    # next order: with raise_on_fail the exception leaves the chains' states
    # (orders, weights, RNG streams) unspecified -- only the results of runs
    # that complete are defined to equal a sequential batched run.
    dev = _device_ancestor(engine, pool)
    # device ancestor_x: one group up to 32 chains -- a group's step carries the
    # inversion's fixed latency, so splitting few chains costs more device time
    # than the host work it hides (16 chains: 2.38 ms per step in one group,
    # 2.94 in two; 32: 4.33 / 4.44) -- two from 64, where the host's share is
    # worth hiding (128: 15.7 / 14.1 / 14.8 ms in 1 / 2 / 3);
    # host ancestor_x: groups hide the pool's inversions
    n_groups = 1 if (use_nem or n < 2) else (groups or ((2 if n >= 64 else 1) if dev else 3 if n >= 6 else 2))
    n_groups = max(1, min(n_groups, n))
    bounds = [n * g // n_groups for g in range(n_groups + 1)]
    glist = [list(range(bounds[g], bounds[g + 1])) for g in range(n_groups)]
    if n_groups == 1:
        for _ in range(n_iterations):
            propose(glist[0])
            post(glist[0], optimal_weights_batch(chains, engine, use_nem=use_nem, cap=cap,
                                                 raise_on_fail=raise_on_fail, pool=pool))
    else:
        from collections import deque
        pending = deque()
        wst = [None] * n_groups     # each group's weights stack (its last step's w_new)
        early = n_groups >= 3       # finish the oldest group before queuing the next

        def drain():
            for p in pending:
                p[3].end()

        def collect():
            g, cs, prep, call = pending.popleft()
            call.end()
            if dev:
                prep, res = _w_call_end(cs, call, raise_on_fail, drain)
            else:
                res = call.result(raise_on_fail)
            wst[g] = res[0]
            post(glist[g], _finish(cs, engine, prep, res, False, cap))

        try:
            for _ in range(n_iterations):
                for g, idx in enumerate(glist):
                    stacks = propose(idx, wst[g])
                    wst[g] = None
                    cs = [chains[k] for k in idx]
                    if dev:
                        while early and len(pending) > n_groups - 2:
                            collect()
                        prep = None
                        call = engine.bind_optimal_weights_w(stacks[0].astype(np.int32), stacks[1], SIG0, SIG1,
                                                             cap=cap, want_prep=False)
                    else:
                        part = _prepare_start(cs, pool, stacks)
                        while early and len(pending) > n_groups - 2:
                            collect()
                        prep = _prepare_end(cs, part, pool)
                        pos, w, w01, anc = prep
                        call = engine.bind_optimal_weights(pos, w01, anc, w, SIG0, SIG1, cap=cap)
                    call.begin()
                    pending.append((g, cs, prep, call))
                    while len(pending) > n_groups - 1:
                        collect()
            while pending:
                collect()
        finally:
            for p in pending:   # an exception left queued steps: wait for them
                p[3].end()

    for k, c in enumerate(chains):
        q = st[k]
        c.best_score, c.best_dag, c.best_order = q["best"], q["best_dag"], q["best_order"]
        c.all_score_list, c.curr_score_list = q["all_list"], q["curr_list"]
        c.best_score_list, c.best_order_list = q["best_list"], q["best_order_list"]
        c.accepted = q["acc"]
        if q["best_parents"] is None:
            bpos = q["best_struct"][0]
            q["best_parents"] = np.empty(s, dtype=object)
            for i in range(s):
                q["best_parents"][i] = c._parents_of(q["best_perm"], bpos, i)
        c.parents_list = q["best_parents"]
        c._pos, c._mask = q["best_struct"]
    best = np.array([q["best"] for q in st])
    return (best, {"st": st, "curr": curr}) if return_state else best


class ChainBatch:
    """``n`` independent order-MCMC chains on one staged model.

    Chain ``c`` uses ``random.Random(seed + c)`` for its proposals and
    acceptances, in exactly the reference's call order, so chain ``c`` of a
    batch reproduces a single ``NEMOrderMCMC.method`` run driven by that
    stream.  ``on_fail="raise"`` (the reference's behaviour) raises when a
    local optimisation terminates abnormally -- at C3 most chains hit one
    within a few dozen steps, in the reference as here; the chains' states
    are unspecified after that exception.  ``"continue"`` keeps the
    optimiser's last point and goes on (an extension for long runs).
    ``inv_pool`` (an ``InvPool``, shareable among batches) runs the per-step
    ancestor_x inversions in worker processes: same bits, less host time."""

    def __init__(self, nem, init_orders, seeds, engine: Engine | None = None, gamma=None,
                 swap_prob=0.95, use_nem=False, cap=0, on_fail="raise", inv_pool=None, groups=None):
        if on_fail not in ("raise", "continue"):
            raise ValueError(f"on_fail={on_fail!r}: 'raise' or 'continue'")
        self.raise_on_fail = on_fail == "raise"
        self.nem = nem
        self.engine = engine if engine is not None else Engine.for_nem(nem)
        self.n = len(init_orders)
        self.gamma = (2.0 * nem.num_s / nem.num_e) if gamma is None else gamma
        self.gammas = np.broadcast_to(np.asarray(self.gamma, dtype=float), (self.n,)).copy()
        self.swap_prob = swap_prob
        self.use_nem = use_nem
        self.cap = cap
        if inv_pool is not None and (inv_pool.s != nem.num_s or inv_pool.maxb < len(init_orders)):
            raise ValueError("inv_pool: matrix size or capacity does not fit this batch")
        self.inv_pool = inv_pool
        self.groups = groups      # pipeline chain groups (run_methods); None: by batch size
        self._state = None
        self.chains = []
        for order, seed in zip(init_orders, seeds):
            c = NEMOrderMCMC(nem, np.asarray(order), engine=self.engine, cap=cap)
            c.rng = random.Random(seed)
            self.chains.append(c)
        self.engine.reserve(self.n, self.n)

    def run(self, n_iterations: int, resume: bool = False):
        """Every chain runs the reference's ``method`` loop
        (nem_order_mcmc.py:257-310) for ``n_iterations`` steps.  Returns
        (best scores [n], best orders [n, S]).  ``resume=True`` continues the
        previous run (or the checkpoint this batch was restored from) for
        ``n_iterations`` more steps, exactly as one longer run would;
        ``accepted`` then covers the whole run."""
        if resume and self._state is None:
            raise ValueError("resume=True: no run or checkpoint to continue")
        self.best_scores, self._state = run_methods(
            self.chains, self.gammas, n_iterations, self.engine, swap_prob=self.swap_prob, use_nem=self.use_nem,
            cap=self.cap, raise_on_fail=self.raise_on_fail, pool=self.inv_pool,
            state=self._state if resume else None, return_state=True, groups=self.groups)
        self.best_orders = [np.asarray(c.best_order).copy() for c in self.chains]
        self.accepted = np.array([c.accepted for c in self.chains]).T.reshape(-1, self.n)
        return self.best_scores, np.stack(self.best_orders)

    # -- checkpoint / resume of the chain states ----------------
    def save_checkpoint(self, path: str):
        """Every chain's state after ``run`` -- weights, order, random stream,
        and the loop state (current / best order and score, the score and
        accept lists) -- to one ``.npz`` of plain arrays (no pickle).
        ``ChainBatch.from_checkpoint`` + ``run(n, resume=True)`` continues
        bit for bit as if the run had not stopped."""
        import json
        if self._state is None:
            raise ValueError("save_checkpoint: run() first")
        st, curr = self._state["st"], self._state["curr"]
        arr = {}
        meta = {"n": self.n, "num_s": self.nem.num_s, "num_e": self.nem.num_e, "gammas": self.gammas.tolist(),
                "swap_prob": self.swap_prob, "use_nem": self.use_nem, "cap": self.cap,
                "raise_on_fail": self.raise_on_fail, "curr": [float(v) for v in curr], "chains": []}
        for k, (c, q) in enumerate(zip(self.chains, st)):
            arr[f"c{k}.w"] = np.asarray(c.parent_weights, dtype=np.float64)
            arr[f"c{k}.perm"] = np.asarray(c._perm)
            version, mt, gauss = c.rng.getstate()
            arr[f"c{k}.rng"] = np.asarray(mt, dtype=np.int64)
            for a in ("best_dag", "curr_perm", "best_order", "curr_dag"):
                arr[f"c{k}.{a}"] = np.asarray(q[a])
            arr[f"c{k}.best_order_list"] = np.stack([np.asarray(o) for o in q["best_order_list"]])
            arr[f"c{k}.best_pos"] = np.asarray(q["best_struct"][0])
            for a in ("curr_list", "best_list", "all_list"):
                arr[f"c{k}.{a}"] = np.asarray(q[a], dtype=np.float64)
            arr[f"c{k}.acc"] = np.asarray(q["acc"], dtype=bool)
            meta["chains"].append({"ll": float(c.ll), "best": float(q["best"]), "rng_version": version,
                                   "rng_gauss": gauss})
        arr["meta"] = np.asarray(json.dumps(meta))
        np.savez_compressed(path, **arr)

    @classmethod
    def from_checkpoint(cls, path: str, nem, engine: Engine | None = None, inv_pool=None):
        """A batch in the state ``save_checkpoint`` wrote; ``nem`` is the same
        model (checked by shape).  Continue it with ``run(n, resume=True)``."""
        import json
        z = np.load(path, allow_pickle=False)
        meta = json.loads(str(z["meta"]))
        if (meta["num_s"], meta["num_e"]) != (nem.num_s, nem.num_e):
            raise ValueError("checkpoint of another model shape")
        n = meta["n"]
        self = cls(nem, [z[f"c{k}.perm"] for k in range(n)], seeds=list(range(n)), engine=engine,
                   gamma=np.asarray(meta["gammas"]), swap_prob=meta["swap_prob"], use_nem=meta["use_nem"],
                   cap=meta["cap"], on_fail="raise" if meta["raise_on_fail"] else "continue", inv_pool=inv_pool)
        st = []
        for k, c in enumerate(self.chains):
            cm = meta["chains"][k]
            perm = np.array(z[f"c{k}.perm"])
            # the structures reset() leaves for this order; W is the saved one
            # (reset's quirks already applied to it)
            c.get_permissible_parents(perm, init=True, init_value=1.0)
            c.parent_weights = np.array(z[f"c{k}.w"], dtype=np.float64)
            c.perm_order = perm
            c.ll = cm["ll"]
            c.rng.setstate((cm["rng_version"], tuple(int(v) for v in z[f"c{k}.rng"]), cm["rng_gauss"]))
            bpos = np.array(z[f"c{k}.best_pos"])
            bperm = np.argsort(bpos)
            best_parents = np.empty(nem.num_s, dtype=object)
            for i in range(nem.num_s):
                best_parents[i] = c._parents_of(bperm, bpos, i)
            st.append(dict(best=cm["best"], best_dag=np.array(z[f"c{k}.best_dag"]),
                           curr_perm=np.array(z[f"c{k}.curr_perm"]), best_order=np.array(z[f"c{k}.best_order"]),
                           best_order_list=list(np.array(z[f"c{k}.best_order_list"])),
                           curr_dag=np.array(z[f"c{k}.curr_dag"]),
                           curr_list=z[f"c{k}.curr_list"].tolist(), best_list=z[f"c{k}.best_list"].tolist(),
                           all_list=z[f"c{k}.all_list"].tolist(), best_parents=best_parents,
                           best_struct=(bpos, c._permissible(bpos)), acc=z[f"c{k}.acc"].tolist()))
        self._state = {"st": st, "curr": list(meta["curr"])}
        return self


def gather_best(best_scores, best_orders, device=None):
    """All-gather per-chain (best score, best order) from every rank.

    Uses the default ``torch.distributed`` process group (RCCL on GPUs, gloo on
    CPU).  Ranks may own different numbers of chains.  Returns
    (scores [n_total], orders [n_total, S]) ordered by rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    scores = torch.as_tensor(np.asarray(best_scores, dtype=np.float64))
    orders = torch.as_tensor(np.asarray(best_orders, dtype=np.int32))
    if device is not None:
        scores, orders = scores.to(device), orders.to(device)
    n = torch.tensor([scores.numel()], dtype=torch.int64, device=scores.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    m = max(counts)
    s = orders.shape[1]
    pad_s = torch.full((m,), float("-inf"), dtype=torch.float64, device=scores.device)
    pad_o = torch.zeros((m, s), dtype=torch.int32, device=scores.device)
    pad_s[: scores.numel()] = scores
    pad_o[: orders.shape[0]] = orders
    all_s = [torch.empty_like(pad_s) for _ in range(world)]
    all_o = [torch.empty_like(pad_o) for _ in range(world)]
    dist.all_gather(all_s, pad_s)
    dist.all_gather(all_o, pad_o)
    out_s = np.concatenate([a[:c].cpu().numpy() for a, c in zip(all_s, counts)])
    out_o = np.concatenate([a[:c].cpu().numpy() for a, c in zip(all_o, counts)])
    return out_s, out_o


def run_c4(nem, engine: Engine, n_chains: int = 128, steps: int = 10, warmup_steps: int = 2, inv_workers=None,
           device=None, cap: int = 0, repeats: int = 1):
    """BASELINE config C4 on the default process group (or alone without one):
    ``n_chains`` independent chains of ``nem`` sharded over the ranks
    (``shard``; chain c keeps seed 1234 + c and the reference's initial order
    whatever the rank count), each rank's share run as ONE ``ChainBatch``
    (the reference's per-chain state machines, nem_order_mcmc.py:257-310, one
    fused device step per MCMC step), then ONE all-gather of every chain's
    (best score, best order) -- the only collective.  The
    ranks run ``warmup_steps`` untimed steps on a throw-away batch first.

    Returns, on every rank, a dict: wall seconds of the timed run (max over
    ranks, barrier before; with ``repeats`` > 1 the run is repeated from the
    same seeds -- the same results -- and the median of the runs' walls is
    reported, the host side being noisy run to run), chain-steps/s, the
    gathered scores and orders and the global best."""
    import hashlib
    import time

    from . import utils
    from .invpool import InvPool, default_workers

    world, rank, pg = 1, 0, False
    try:
        import torch.distributed as dist
        pg = dist.is_available() and dist.is_initialized()
        if pg:
            world, rank = dist.get_world_size(), dist.get_rank()
    except ImportError:
        dist = None
    mine = shard(n_chains, rank, world)
    order = utils.initial_order_guess(nem.observed_knockdown_mat)
    seeds = [1234 + c for c in mine]
    # ancestor_x: on the device at S <= 64 (no worker processes), else in an InvPool
    nw = (0 if engine.device_ancestor else default_workers()) if inv_workers is None else int(inv_workers)
    pool = InvPool(nem.num_s, len(mine), nw) if nw > 0 and len(mine) > 0 else None
    try:
        if warmup_steps > 0 and len(mine):
            ChainBatch(nem, [order] * len(mine), seeds=seeds, engine=engine, on_fail="continue", cap=cap,
                       inv_pool=pool).run(warmup_steps)
        walls = []
        for _ in range(max(1, int(repeats))):
            cb = ChainBatch(nem, [order] * len(mine), seeds=seeds, engine=engine, on_fail="continue", cap=cap,
                            inv_pool=pool) if len(mine) else None
            if pg:
                dist.barrier()
            t0 = time.perf_counter()
            if cb is not None:
                best, orders = cb.run(steps)
            else:
                best, orders = np.zeros(0), np.zeros((0, nem.num_s), dtype=np.int32)
            if pg:  # a process group (even of one rank): the collective runs
                all_s, all_o = gather_best(best, orders, device=device)
            else:
                all_s, all_o = np.asarray(best, dtype=np.float64), np.asarray(orders)
            wall = time.perf_counter() - t0
            if pg:
                import torch
                t = torch.tensor([wall], dtype=torch.float64, device=device if device is not None else "cpu")
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                wall = float(t.item())
            walls.append(wall)
    finally:
        if pool is not None:
            pool.close()
    wall = float(np.median(walls))
    g = int(np.argmax(all_s))
    return {"wall_s": wall, "chain_steps_per_s": n_chains * steps / wall, "ms_per_step": 1e3 * wall / steps,
            "ms_per_step_runs": [1e3 * w / steps for w in walls],
            "n_ranks": world, "chains_per_rank": len(mine), "inv_workers_per_rank": nw if pool else 0,
            "n_gathered": int(len(all_s)), "best_score": float(all_s[g]), "best_chain": g,
            "gathered_over": dist.get_backend() if pg else None,
            "accepted": None if cb is None else cb.accepted,
            "best_order": [int(v) for v in all_o[g]],
            "scores_sha256": hashlib.sha256(np.ascontiguousarray(all_s, dtype=np.float64).tobytes()).hexdigest()[:16],
            "scores": all_s, "orders": all_o}
