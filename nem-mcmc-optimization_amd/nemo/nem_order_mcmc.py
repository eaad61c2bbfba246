"""Order MCMC for Nested Effects Models with the per-step scorer on the GPU.

Drop-in for the reference's ``nem_order_mcmc.NEMOrderMCMC`` (nem_order_mcmc.py:
28-313): same constructor, method names, argument meaning, attributes and
random-number stream.  The host keeps the sampler state machine (proposals,
parent-set bookkeeping, acceptance -- all Python ``random`` calls in the
reference's order); every numerical routine of the hot path runs on the GPU
through ``libnemo`` (include/nemo.h):

* ``compute_cell_ratios`` + ``calculate_ll`` (nem_order_mcmc.py:79-93)
  -> ``nemo_score`` / ``nemo_lse``;
* ``get_optimal_weights`` (nem_order_mcmc.py:172-208): eval #1, the L-BFGS-B
  local optimum of every permissible pair, eval #2 on the binarised weights
  -> one ``nemo_optimal_weights`` call (three kernels, one host sync);
* ``calculate_local_optimum`` (nem_order_mcmc.py:160-170) -> ``nemo_local_opt``.

The reference's entry point crashes (``opt_weights`` calls an undefined
``modified_logistic``, nem_order_mcmc.py:140).  ``opt_weights`` here is the
documented pass-through: it returns the score of the current
weights, which equals the score ``get_optimal_weights`` just produced.
"""
from __future__ import annotations

import random
import warnings
from itertools import cycle

import numpy as np
from scipy.linalg import inv
from scipy.special import expit

from . import utils
from .engine import Engine, ExactArithmeticWarning, lse_full
from ._lib import LBFGSB_ABNORMAL

SIG0 = float(expit(0.0))   # expit of a binarised "no edge" weight
SIG1 = float(expit(1.0))   # expit of a binarised "edge" weight


def draw_swap(rng, s, swap_prob=0.95):
    """The draws of get_new_order (nem_order_mcmc.py:236-241): one random(),
    then a sample of two positions or one randint (adjacent swap)."""
    if rng.random() < swap_prob:
        i, j = rng.sample(range(s), 2)
    else:
        i = rng.randint(0, s - 2)
        j = i + 1
    return i, j


def permissible_batch(pos, cap=0):
    """mask[c, i, j]: j is a permissible parent of i in order c (it comes
    before i, within ``cap`` places when a cap is set)."""
    p = pos.astype(np.int16)            # S <= 32767: the gaps fit
    m = p[:, :, None] > p[:, None, :]
    if cap:
        m &= (p[:, :, None] - p[:, None, :]) <= cap
    return m


def reset_weights_batch(w, mask, i1, i2, init_value=0.5):
    """``get_permissible_parents(init=False)``'s in-place weight updates
    (nem_order_mcmc.py:67-77; the per-chain form is
    NEMOrderMCMC.get_permissible_parents) on a stack of chains at once:
    w[c], mask[c] of chain c with its own i1[c], i2[c] (i1 != i2).  Rows and
    columns i1, i2 are zeroed; then column i1 holds ``init_value`` at the
    children with i1 as a permissible parent, column i2 at the remaining
    children with i2 as one, and column i (i in {i1, i2}) additionally at
    i's own parents when i is in neither set.  Every write stores one of two
    constants, so the order of the reference's writes fixes the result."""
    n = w.shape[0]
    ar = np.arange(n)
    w[ar, i1] = 0
    w[ar, i2] = 0
    to1 = mask[ar, :, i1]                 # (n, S): mask[c, :, i1[c]]
    to2 = mask[ar, :, i2] & ~to1
    for i, col in ((i1, to1), (i2, to2)):
        quirk = ~to1[ar, i] & ~to2[ar, i]
        col = col | (mask[ar, i, :] & quirk[:, None])
        w[ar, :, i] = np.where(col, init_value, 0.0)


class NEMOrderMCMC:
    # proposal / acceptance stream: the global ``random`` module, as in the
    # reference; nemo.chains gives each batched chain its own random.Random
    rng = random

    def __init__(self, nem, perm_order, device: int = 0, dtype: str = "f64", cap: int = 0,
                 engine: Engine | None = None, strict: bool = False):
        """Reference: nem_order_mcmc.py:29-48.

        Extra keyword arguments (build-defined): ``device`` (GPU index),
        ``dtype`` ('f64' or the fp32 'f32' table path), ``cap`` (parent-set cap,
        0 = every predecessor, as in the reference), ``engine`` (share a staged
        model between samplers), ``strict`` (raise instead of warning when the
        staged model is outside the reference-arithmetic kernels; an engine
        whose option ``exact`` was set to 0 on purpose is not checked)."""
        self.nem = nem
        self.num_s = nem.num_s
        self.num_e = nem.num_e
        self.U = nem.U.copy()
        self.perm_orders = [perm_order]
        self.parent_weights = np.zeros((self.num_s, self.num_s))
        self.score_tables = nem.get_score_tables(nem.observed_knockdown_mat)
        self.cap = int(cap)
        self.engine = engine if engine is not None else Engine.for_nem(nem, device=device, dtype=dtype)
        if self.engine.get_option("exact"):
            ok, why = self.engine.exact_status()
            if not ok:
                msg = (f"NEMOrderMCMC: {why}; the step runs the fast kernels (log-scores within 1e-6 of "
                       "the reference's, not its bits)")
                if strict:
                    raise RuntimeError(msg)
                warnings.warn(msg, ExactArithmeticWarning, stacklevel=2)
        self.get_permissible_parents(perm_order, init=True, init_value=1.0)
        self.cell_ratios = self.compute_cell_ratios(self.parent_weights, self.score_tables)
        self.perm_order = perm_order
        self.I = np.identity(self.num_s)
        self._eval1 = None      # (pos, W~ or None, W) of the last eval #1
        self._anc = None        # ancestor_x (or where to make it: _anc_src)
        self._anc_src = None
        self._ow = None         # its order weights, computed on first access

    # -- A3 / A7: parent sets and the reset quirks ---------------------------
    def reset(self, perm_order, i1=None, i2=None, init=False):
        """Reference: nem_order_mcmc.py:50-52."""
        self.ll = 0.0
        self.get_permissible_parents(perm_order, i1, i2, init=init)

    def get_permissible_parents(self, perm_order, i1=None, i2=None, init=False, init_value=0.5):
        """Reference: nem_order_mcmc.py:54-77, including its in-place weight
        updates on reset: rows/columns i1, i2 zeroed; then per child i, the
        weight to i1 (else to i2) reset if that node is a permissible parent;
        else, for i in {i1, i2}, the *transposed* entries W[j][i] of its parents
        set -- exactly as written there.  Every write stores ``init_value``, so
        the reference's per-child loop is applied as whole-array assignments.
        ``parents_list`` / ``n_parents`` are built on first access."""
        perm = np.asarray(perm_order)
        s = self.num_s
        pos = np.empty(s, dtype=np.int64)
        pos[perm] = np.arange(s)
        mask = self._permissible(pos)   # mask[i, j]: j in parents_list[i]
        w = self.parent_weights
        if init:
            w[mask] = init_value
        else:
            w[i1] = 0
            w[i2] = 0
            w[:, i1] = 0
            w[:, i2] = 0
            to_i1 = mask[:, i1]
            to_i2 = mask[:, i2] & ~to_i1
            w[to_i1, i1] = init_value
            w[to_i2, i2] = init_value
            for i in (i1, i2):
                if not to_i1[i] and not to_i2[i]:
                    w[self._parents_of(perm, pos, i), i] = init_value
        self._perm, self._pos, self._mask = perm, pos, mask
        self._parents = None

    def _parents_of(self, perm, pos, i):
        lo = max(0, pos[i] - self.cap) if self.cap else 0
        return perm[lo:pos[i]]

    @property
    def parents_list(self):
        """parents_list[i] = the order prefix before i (within the cap), an
        object array as in the reference (nem_order_mcmc.py:62-65)."""
        if self._parents is None:
            pl = np.empty(self.num_s, dtype=object)
            for i in range(self.num_s):
                pl[i] = self._parents_of(self._perm, self._pos, i)
            self._parents = pl
        return self._parents

    @parents_list.setter
    def parents_list(self, value):
        self._parents = value

    @property
    def n_parents(self):
        """nem_order_mcmc.py:65-66: the parent counts of the last
        get_permissible_parents call (stale after ``method`` restores the best
        order's parents_list, as in the reference)."""
        return np.minimum(self._pos, self.cap).astype(int) if self.cap else self._pos.astype(int)

    def _permissible(self, pos):
        gap = pos[:, None] - pos[None, :]
        m = gap > 0
        if self.cap:
            m &= gap <= self.cap
        return m

    def _pos_of(self, perm):
        pos = np.empty(self.num_s, dtype=np.int64)
        pos[np.asarray(perm)] = np.arange(self.num_s)
        return pos

    # -- A4 + A5 -----------------------------------------------------------------
    def compute_cell_ratios(self, weights, score_tables):
        """Reference: nem_order_mcmc.py:79-87 (expit applied to the weights
        of the permissible parents).  Evaluated by the score kernel."""
        eng = self._engine_for(score_tables)
        w01 = expit(np.asarray(weights, dtype=np.float64))
        out = eng.score(self._pos[None, :], w01[None], cap=self.cap, want_cells=True)
        return out["cells"][0]

    def calculate_ll(self):
        """Reference: nem_order_mcmc.py:89-93 -> (order_weights, ll), from
        ``self.cell_ratios``, on the GPU."""
        ll, _cs, ow = lse_full(self.cell_ratios, device=self.engine.device)
        return ow, ll

    def _engine_for(self, score_tables):
        if score_tables is self.score_tables:
            return self.engine
        t = np.asarray(score_tables, dtype=np.float64)
        return Engine(self.U, t, device=self.engine.device, dtype=self.engine.dtype)

    def expit_parent_weights(self, weights):
        """Reference: nem_order_mcmc.py:98-103 / 152-157: expit on the
        permissible entries only, the other (stale) entries kept raw."""
        out = np.array(weights, dtype=np.float64, copy=True)
        out[self._mask] = expit(out[self._mask])
        return out

    # -- A6 -------------------------------------------------------------------------
    def get_optimal_weights(self, abs_diff=1e-6, max_iter=1, use_nem=False, i1=None, i2=None,
                            init=False, ultra_verbose=False):
        """Reference: nem_order_mcmc.py:172-208.  Each weight pass is one fused
        device call: eval #1 with order weights, the local optimum of every
        permissible (i, k) pair, eval #2 of the binarised weights."""
        old_ll = -float("inf")
        ll_diff = float("inf")
        iter_count = 1
        self.ll = 0.0
        dag_ll = None
        pos = self._pos
        while iter_count <= max_iter and ll_diff > abs_diff:
            self.ratio = iter_count / max_iter
            w = self.parent_weights
            # init=False re-optimises only the pairs that touch i1 / i2
            # (nem_order_mcmc.py:190-194): the fused call optimises every
            # permissible pair, so a failure raises only on a re-optimised one
            if self.engine.device_ancestor:
                # W~ = expit on the permissible entries and ancestor_x (:98-103,
                # :185) made on the device, in scipy's bits
                try:
                    w01, anc, w_new, ll1, lld, info = self.engine.optimal_weights_w(
                        pos[None, :], w[None], SIG0, SIG1, cap=self.cap, raise_on_fail=init)
                except Exception as e:
                    # the reference sets order_weights (:182) before inv can
                    # raise and ancestor_x (:185) before a local optimum can:
                    # both follow this step's W (made from it when read); an
                    # error of inv itself (LinAlgError / ValueError) leaves the
                    # previous ancestor_x, as the reference's assignment never ran
                    wc = np.array(w, dtype=np.float64, copy=True)
                    if not isinstance(e, (np.linalg.LinAlgError, ValueError)):
                        self._set_ancestor_src(pos.copy(), wc)
                    self._set_eval1(pos.copy(), None, wc)
                    raise
                w01, self.ancestor_x = w01[0], anc[0]
            else:
                w01 = expit(w)
                mapped = self.expit_parent_weights(w)
                self.ancestor_x = np.clip(inv(self.I - mapped) - self.I, 0, 1)
                w_new, ll1, lld, info = self.engine.optimal_weights(
                    pos[None, :], w01[None], self.ancestor_x[None], w[None], SIG0, SIG1, cap=self.cap,
                    raise_on_fail=init)
            self._set_eval1(pos.copy(), w01.copy())
            w_new = w_new[0]
            if not init:
                keep = np.zeros_like(self._mask)
                for a in range(self.num_s):
                    for k in self.parents_list[a]:
                        if not (i1 == k or i2 == k or a == i1 or a == i2):
                            keep[a, k] = True
                redo = self._mask & ~keep
                failed = redo & (info[0] != -1) & ((info[0] & 15) >= LBFGSB_ABNORMAL)
                if failed.any():
                    # the reference's first failing pair: child i ascending, parents in order
                    a, k = min(zip(*np.nonzero(failed)), key=lambda ak: (ak[0], self._pos[ak[1]]))
                    reason = ("ABNORMAL_TERMINATION_IN_LNSRCH" if (info[0][a, k] & 15) == LBFGSB_ABNORMAL
                              else "STOP: TOTAL NO. of ITERATIONS REACHED LIMIT")
                    raise Exception(f"Minimization not successful, Reason: {reason}")
                w_new[keep] = w[keep]
                lld = None
            self.ll = float(ll1[0])
            ll_diff = np.abs(self.ll - old_ll)
            old_ll = self.ll
            if ultra_verbose:
                print(f"LL: {self.ll}")
                print(f"Iteration of weight optimization: {iter_count + 1}")
            iter_count += 1
            self.parent_weights = w_new.copy()
            dag_ll = None if lld is None else float(lld[0])
        if use_nem or dag_ll is None:
            if use_nem:
                _, dag_weights = self.create_nem(self.parent_weights)
            else:
                _, dag_weights = self.create_dag(self.parent_weights)
            w01d = expit(np.asarray(dag_weights, dtype=np.float64))
            dag_ll = float(self.engine.score(pos[None, :], w01d[None], cap=self.cap)[0])
        return dag_ll

    def _set_eval1(self, pos, w01, w=None):
        """The last eval #1's (pos, W~); W~ None: made from W when needed
        (expit of W -- the score reads the permissible entries only)."""
        self._eval1 = (pos, w01, w)
        self._ow = None

    @property
    def ancestor_x(self):
        """clip(inv(I - W~) - I, 0, 1) of the last step (nem_order_mcmc.py:185).
        A chain batch whose device made it leaves where it came from: the
        host makes the same bits (scipy's expit and inv) on first access."""
        if self._anc is None and self._anc_src is not None:
            pos, w = self._anc_src
            mask = self._permissible(pos)
            sig = np.array(w, dtype=np.float64, copy=True)
            sig[mask] = expit(sig[mask])
            self._anc = np.clip(inv(self.I - sig) - self.I, 0, 1)
            self._anc_src = None
        return self._anc

    @ancestor_x.setter
    def ancestor_x(self, value):
        self._anc = value
        self._anc_src = None

    def _set_ancestor_src(self, pos, w):
        self._anc, self._anc_src = None, (pos, w)

    @property
    def order_weights(self):
        """Order weights of this sampler's last eval #1 (the attribute
        get_optimal_weights sets in the reference, nem_order_mcmc.py:182).
        Computed from that evaluation's own (pos, expit(W)) on first access --
        not read from the engine, which other samplers share."""
        if self._ow is None:
            if self._eval1 is None:
                raise AttributeError("'NEMOrderMCMC' object has no attribute 'order_weights' "
                                     "(set by get_optimal_weights)")
            pos, w01, w = self._eval1
            if w01 is None:
                w01 = expit(np.asarray(w, dtype=np.float64))
            self._ow = self.engine.score(pos[None, :], w01[None], cap=self.cap, want_ow=True)["ow"][0]
        return self._ow

    @order_weights.setter
    def order_weights(self, value):
        self._ow = np.asarray(value, dtype=np.float64)

    # -- A8 (single pair, API compatibility) ---------------------------------------
    def calculate_local_optimum(self, i, k):
        """Reference: nem_order_mcmc.py:160-170.  The c vector is assembled on
        the host from the staged inputs; the L-BFGS-B solve runs on the GPU."""
        ow = self.order_weights
        lv = np.exp(self.score_tables[i][k])
        a = (lv - 1.0) * ow[k]
        s = expit(self.parent_weights[i][k])
        b = 1.0 - s * a + s * (lv - 1.0)
        c = a / b
        xs, _f, _nit, _nfev, st = self.engine.local_opt(c[None], self.ancestor_x[i][k], s)
        if st[0] >= 2:
            raise Exception("Minimization not successful, Reason: ABNORMAL_TERMINATION_IN_LNSRCH")
        return expit(xs[:1])

    def opt_weights(self, max_iter=50):
        """The reference's global optimiser crashes (nem_order_mcmc.py:140,
        undefined ``modified_logistic``).  Documented pass-through: the score of
        the current binarised weights."""
        _, dag_weights = self.create_dag(self.parent_weights)
        w01d = expit(np.asarray(dag_weights, dtype=np.float64))
        self.ll = float(self.engine.score(self._pos[None, :], w01d[None], cap=self.cap)[0])
        return self.ll

    # -- A9 ---------------------------------------------------------------------------
    def create_dag(self, weights):
        """Reference: nem_order_mcmc.py:210-214."""
        dag_weights = 1 * (weights > 0.5)
        return dag_weights.T, dag_weights

    def create_nem(self, weights):
        """Reference: nem_order_mcmc.py:216-221."""
        nem_weights = utils.ancestor(1 * (weights > 0.5))
        return nem_weights.T, nem_weights

    # -- A7 ---------------------------------------------------------------------------
    def accepting(self, score, curr_score, gamma, net, curr_net, perm_order, curr_perm_order):
        """Reference: nem_order_mcmc.py:224-229 (one random() draw)."""
        acceptance_rate = np.exp(gamma * (score - curr_score))
        if self.rng.random() < acceptance_rate:
            return True, score, net, perm_order
        return False, curr_score, curr_net, curr_perm_order

    def get_new_order(self, curr_perm_order, swap_prob=0.95):
        """Reference: nem_order_mcmc.py:231-255.  i1, i2 are the positions of
        the node LABELS i, j; the swap exchanges POSITIONS i, j (as written)."""
        perm_order = curr_perm_order.copy()
        i, j = draw_swap(self.rng, self.num_s, swap_prob)
        i1 = np.where(perm_order == i)[0][0]
        i2 = np.where(perm_order == j)[0][0]
        perm_order[i], perm_order[j] = perm_order[j], perm_order[i]
        return perm_order, i1, i2

    def method(self, swap_prob=0.95, gamma=1, seed=1234, n_iterations=500, verbose=True,
               ultra_verbose=False, use_nem=False):
        """Reference: nem_order_mcmc.py:257-310 (``seed`` unused there too)."""
        curr_score = self.get_optimal_weights(init=True, ultra_verbose=ultra_verbose, use_nem=use_nem)
        curr_score = self.opt_weights()
        best_score = curr_score
        dag, _ = self.create_dag(self.parent_weights)
        best_dag = dag
        curr_perm_order = self.perm_order
        perm_order = curr_perm_order
        best_order = perm_order
        best_order_list = [best_order]
        curr_dag = np.zeros((self.num_s, self.num_s))
        curr_score_list = [curr_score]
        best_score_list = [best_score]
        all_score_list = [curr_score]
        best_parents_list = self.parents_list.copy()
        best_struct = (self._pos, self._mask)   # the device mask behind parents_list
        accepted = []
        for it in range(n_iterations):
            if verbose and it % 50 == 0:
                print(f"{it}-th iteration")
            perm_order, i1, i2 = self.get_new_order(curr_perm_order, swap_prob=swap_prob)
            self.reset(perm_order=perm_order, i1=i1, i2=i2)
            ll = self.get_optimal_weights(init=True, use_nem=use_nem, ultra_verbose=ultra_verbose)
            all_score_list.append(ll)
            if use_nem:
                dag, _ = self.create_nem(self.parent_weights)
            else:
                dag, _ = self.create_dag(self.parent_weights)
            curr_score_list.append(curr_score)
            acc, curr_score, curr_dag, curr_perm_order = self.accepting(
                ll, curr_score, gamma, dag, curr_dag, perm_order, curr_perm_order)
            perm_order = curr_perm_order
            accepted.append(acc)
            if acc and curr_score > best_score:
                best_score = curr_score
                best_dag = dag
                best_order = curr_perm_order.copy()
                best_parents_list = self.parents_list.copy()
                best_struct = (self._pos, self._mask)
                best_score_list.append(best_score)
                best_order_list.append(best_order)
        self.best_score = best_score
        self.best_dag = best_dag
        self.best_order = best_order
        self.all_score_list = all_score_list
        self.curr_score_list = curr_score_list
        self.best_score_list = best_score_list
        self.best_order_list = best_order_list
        self.accepted = accepted
        # the reference leaves parents_list at the best order's parent sets
        # (n_parents stays stale, as there); the next method() call -- replica
        # exchange rounds -- scores with them
        self.parents_list = best_parents_list
        self._pos, self._mask = best_struct
        return best_score, best_dag

    def condition(self, i, j):
        """Reference: nem_order_mcmc.py:312-313."""
        return i in self.parents_list[j]


# -- replica exchange (nem_order_mcmc.py:316-363) ------------------------------------
def replica_exchange_step(replicas, gammas, n_replicas, n_iters, scores, upwards_cylce):
    """Reference: nem_order_mcmc.py:316-342.  Replicas run in turn (the
    reference's order, so the shared random stream matches); each replica's
    steps use the GPU scorer."""
    n_exchanges = 0
    for i in range(n_replicas):
        replicas[i].method(n_iterations=n_iters, gamma=gammas[i], verbose=True)
        replicas[i].perm_orders = [replicas[i].perm_orders[-1]]
        scores[i] = replicas[i].best_score
    best_score = np.max(scores)
    best_nem = replicas[np.argmax(scores)]
    if upwards_cylce:
        partners = [(j - 1, j) for j in range(1, n_replicas, 2)]
    else:
        partners = [(j - 1, j) for j in range(2, n_replicas, 2)]
    for (i, j) in partners:
        delta = gammas[i] * scores[j] - gammas[i] * scores[i] + gammas[j] * scores[i] - gammas[j] * scores[j]
        if random.random() < np.exp(-delta):
            replicas[i], replicas[j] = replicas[j], replicas[i]
            scores[i], scores[j] = scores[j], scores[i]
            n_exchanges += 1
            if scores[i] > best_score:
                best_score = scores[i]
                best_nem = replicas[i]
    return best_score, best_nem, replicas, scores, n_exchanges


def replica_exchange_method(nem, n_exchange, n_iter, init_order_guess, n_replicas=10, **kw):
    """Reference: nem_order_mcmc.py:344-363 (10 replicas, gamma_r =
    (1 + 0.2 r) S / E).  All replicas share one staged model on the GPU."""
    gammas, replicas = [], []
    engine = Engine.for_nem(nem, **kw)
    for i in range(n_replicas):
        gammas.append((1.0 + i * 0.2) * nem.num_s / nem.num_e)
        replicas.append(NEMOrderMCMC(nem, init_order_guess, engine=engine))
    scores = np.zeros(n_replicas)
    n_exchanges = 0
    cycler = cycle([True, False])
    best_score, best_nem = None, None
    for _ in range(n_exchange):
        best_score, best_nem, replicas, scores, exchanges = replica_exchange_step(
            replicas, gammas, n_replicas, n_iter, scores, next(cycler))
        n_exchanges += exchanges
    return best_score, best_nem
