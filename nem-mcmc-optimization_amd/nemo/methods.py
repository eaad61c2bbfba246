"""The fixed-order weight optimizers of the reference's methods.py on the GPU.

Mirrors ``InverseMethod`` (methods.py:21-172, the optimizer ``main()`` runs,
main.py:115-116) and ``Method`` (methods.py:342-436) with the reference's
constructor, attributes and ``optimize`` loop; the weight sweep of each
(``opt_b`` / ``opt_γ``) is one C-ABI call that evaluates the order score and
runs every pair's bounded L-BFGS-B on the device (``nemo_inverse_sweep`` /
``nemo_gamma_sweep``).  The host keeps only the loop
of ``optimize``: the ll bookkeeping, the best sweep and the final rounding.

``ExpitMethod`` / ``ExpMethod`` are not mirrored: the first has no
``optimize``; the second feeds exp(6.0) = 403 as a weight into
log(1 - w + w e^T), which is NaN for every table nem.py builds (e^B < 1),
so it has no meaningful output to match.
"""
from __future__ import annotations

import numpy as np

from .engine import Engine

INVERSE_BOUNDS = [(-5000, 500)]   # methods.py:132
GAMMA_BOUNDS = [(0, 1)]           # methods.py:408


def _positions(order):
    order = np.asarray(order)
    pos = np.empty(len(order), dtype=np.int32)
    pos[order] = np.arange(len(order))
    return pos


class _Base:
    def __init__(self, order, num_s, num_e, U, score_tables, engine: Engine | None = None,
                 device: int = 0, dtype: str = "f64"):
        self.order = order
        self.num_s = num_s
        self.num_e = num_e
        self.U = U
        self.score_tables = score_tables
        self.eye = np.eye(self.num_s)
        self.mask = np.zeros((self.num_s, self.num_s))
        self.get_permissible_parents(order, self.mask, init_val=1.0)
        self.engine = engine if engine is not None else Engine.for_tables(U, score_tables, device, dtype)
        self.engine.reserve(1, 1)
        self._pos = _positions(order)

    def get_permissible_parents(self, perm_order, weights, init_val=0.5, i1=None, i2=None):
        """methods.py:34-42: parents_list[i] = the order prefix before i; sets
        weights[i][j] = init_val on it (in place) and returns weights."""
        perm_order = np.asarray(perm_order)
        parents_list = np.empty(self.num_s, dtype=object)
        for i in range(self.num_s):
            index = int(np.where(perm_order == i)[0][0])
            parents_list[i] = perm_order[:index]
            for j in parents_list[i]:
                weights[i][j] = init_val
        self.parents_list = parents_list
        return weights

    def create_dag(self, weights):
        """methods.py:44-47."""
        return 1 * (weights > 0.5)

    def compute_cell_ratios(self, weights, score_tables):
        """methods.py:49-58 (raw weights, no expit) on the GPU."""
        eng = self.engine if score_tables is self.score_tables else Engine.for_tables(self.U, score_tables)
        out = eng.score(self._pos[None, :], np.asarray(weights, dtype=np.float64)[None], want_cells=True)
        return out["cells"][0]

    def calculate_ll(self, cell_ratios):
        """methods.py:60-64 -> (order_weights, ll)."""
        ll, _cs, ow = self.engine.lse(cell_ratios, want_ow=True)
        return ow, ll

    def _ll_of(self, weights):
        return float(self.engine.score(self._pos[None, :], np.asarray(weights, dtype=np.float64)[None])[0])

    @staticmethod
    def _loop(sweep, weights, max_iter, rel_diff):
        """The common loop of optimize (methods.py:150-164 / :418-429): stop
        when |ll - ll_old| <= rel_diff; best = the sweep whose evaluated ll
        is highest, its returned weights are kept."""
        ll_diff = float("inf")
        ll_old = -float("inf")
        ll_list, weight_list = [], []
        best_ll = -float("inf")
        best_index = 0
        iter_count = 0
        while iter_count < max_iter and ll_diff > rel_diff:
            ll, weights = sweep(weights)
            ll_list.append(ll)
            if ll > best_ll:
                best_ll = ll
                best_index = iter_count
            weight_list.append(weights)
            ll_diff = np.abs(ll - ll_old)
            ll_old = ll
            iter_count += 1
        return ll_list, weight_list, best_ll, best_index


class InverseMethod(_Base):
    """Reference: methods.py:21-172."""

    def exp_parent_weights(self, weights):
        """methods.py:66-71."""
        new_weights = np.array(weights, dtype=np.float64, copy=True)
        for i in range(self.num_s):
            for j in self.parents_list[i]:
                new_weights[i][j] = np.exp(new_weights[i][j])
        return new_weights

    def opt_b(self, weights, bounds):
        """methods.py:117-129: the evaluation on B/(1+B) and every pair's
        local optimum in the reference's loop order, in one device call."""
        if [tuple(b) for b in bounds] != [tuple(b) for b in INVERSE_BOUNDS]:
            raise NotImplementedError(f"opt_b runs with the reference's bounds {INVERSE_BOUNDS}")
        w_out, ll, _info = self.engine.inverse_sweep(self._pos[None, :], weights)
        return float(ll[0]), w_out[0]

    def ancestral(self, weights):
        """unorder_arr(order, B/(1+B)) of methods.py:118-121 / 160-163."""
        return self.engine.inverse_ancestral(self._pos[None, :], weights)[0]

    def optimize(self, max_iter=1000, rel_diff=1e-8, weights=None, init_weight=-5000.0, init_val=0.0,
                 use_wandb=False):
        """methods.py:131-172 -> (B_tilde.T, rounded ll).  ``use_wandb`` is
        accepted and ignored (no wandb here)."""
        bounds = INVERSE_BOUNDS
        if weights is None:
            weights = np.full((self.num_s, self.num_s), init_weight, dtype=np.float64)
            weights = self.get_permissible_parents(perm_order=self.order, weights=weights, init_val=init_val)
        else:
            weights = np.where(np.asarray(weights) == 0.0, init_weight, init_val).astype(np.float64)
        ll_list, weight_list, best_ll, best_index = self._loop(
            lambda w: self.opt_b(w, bounds), weights, max_iter, rel_diff)
        self.ll_list = ll_list
        weights = weight_list[best_index]
        print(f"Best ll: {best_ll}")
        b_tilde = 1 * (self.ancestral(weights) > 0.5)
        real_ll = self._ll_of(b_tilde)
        print(f"Rounded LL: {real_ll}")
        return b_tilde.T, real_ll


class Method(_Base):
    """Reference: methods.py:342-436 (the weights are probabilities in [0, 1])."""

    def opt_γ(self, weights, bounds):
        """methods.py:397-405."""
        if [tuple(b) for b in bounds] != [tuple(b) for b in GAMMA_BOUNDS]:
            raise NotImplementedError(f"opt_γ runs with the reference's bounds {GAMMA_BOUNDS}")
        w_out, ll, _info = self.engine.gamma_sweep(self._pos[None, :], weights)
        return float(ll[0]), w_out[0]

    def optimize(self, max_iter=1000, rel_diff=1e-8, use_wandb=False):
        """methods.py:407-436 -> (rounded weights.T, rounded ll)."""
        bounds = GAMMA_BOUNDS
        weights = np.zeros((self.num_s, self.num_s))
        weights = self.get_permissible_parents(perm_order=self.order, weights=weights, init_val=0.5)
        ll_list, weight_list, best_ll, best_index = self._loop(
            lambda w: self.opt_γ(w, bounds), weights, max_iter, rel_diff)
        self.ll_list = ll_list
        weights = 1 * (weight_list[best_index] > 0.5)
        print(f"Best ll: {best_ll}")
        real_ll = self._ll_of(weights)
        print(f"Rounded LL: {real_ll}")
        return weights.T, real_ll


__all__ = ["InverseMethod", "Method", "INVERSE_BOUNDS", "GAMMA_BOUNDS"]
