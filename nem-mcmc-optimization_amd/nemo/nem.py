"""Nested Effects Model: observed knockdown data and the effect score tables.

Mirrors the reference ``nem.NEM`` (nem.py:8-144).  The class builds, on the
host and once per model, the two inputs of the hot path:

* the score tables ``T`` (nem.py:25-54): for child S-gene ``i`` and candidate
  parent ``j``, ``T[i][j][e]`` is the log-likelihood increment of effect ``e``;
* the node LR table ``U`` (nem.py:56-64), shape (S+1, E); row ``S`` is the
  "effect attached to nothing" row.

Both are reproduced bit for bit: the reference builds row ``i`` of ``T[i]`` and
row ``S`` of ``U`` by *sequential* float additions of ``A`` (nem.py:30-32,
nem.py:62), which differ from ``A * count`` in the last bits; we replay the
same addition chain through a lookup table instead of an S*S*E Python loop.

The tables are staged to HBM once by :class:`nemo.engine.Engine`; nothing in
this file is on the per-step path.
"""
from __future__ import annotations

import random

import numpy as np

from . import utils


def _addition_chain(start: float, step: float, count: int) -> np.ndarray:
    """chain[k] = (((start + step) + step) ... + step), k additions (float64)."""
    chain = np.empty(count + 1, dtype=np.float64)
    acc = float(start)
    chain[0] = acc
    for k in range(1, count + 1):
        acc = acc + step
        chain[k] = acc
    return chain


class ScoreTables:
    """Lazy stand-in for the reference's list of S score tables (nem.py:49-54):
    indexable, iterable, sized; T[i] is built on access."""

    def __init__(self, nem, knockdown_mat):
        self._nem = nem
        self._d = knockdown_mat

    def __len__(self):
        return self._nem.num_s

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        i = int(i)
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        return self._nem.build_score_table(i, self._d)

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    def __array__(self, dtype=None, copy=None):
        t = self._nem.get_score_tensor(self._d)
        return t if dtype is None else t.astype(dtype, copy=False)

    @property
    def knockdown_mat(self):
        return self._d


class NEM:
    """Reference: nem.py:8-22.

    ``adj_matrix[a][b] = 1`` is an edge a->b (closure form, as the bundled CSVs
    store it); ``end_nodes[k]`` is the S-gene effect ``k`` hangs off;
    ``errors = (alpha, beta)`` are the false-positive / false-negative rates.

    Construction consumes the global Python ``random`` stream exactly like the
    reference (``random.seed(seed)`` then ``create_observed_knockdown_mat``
    re-seeds with 42 and draws S*E numbers, utils.py:25-35), so a sampler
    started afterwards sees the same proposal stream.

    The reference also runs ``compute_real_score`` twice at construction
    (nem.py:21-22), a diagnostic L-BFGS-B fit of the *true* graph that does not
    feed the sampler.  It is out of scope here; its only
    side effect on shared state -- zeroing the caller's adjacency diagonal in
    place (nem.py:90-91) -- is reproduced, and the diagnostic attributes are
    left as ``None``.
    """

    def __init__(self, adj_matrix, end_nodes, errors, num_s, num_e, seed=42):
        self.num_s = int(num_s)
        self.num_e = int(num_e)
        self.adj_matrix = adj_matrix
        alpha, beta = float(errors[0]), float(errors[1])
        self.real_knockdown_mat = utils.create_real_knockdown_mat(adj_matrix, end_nodes)
        random.seed(seed)
        self.A = np.log(alpha / (1.0 - beta))
        self.B = np.log(beta / (1.0 - alpha))
        self.observed_knockdown_mat = utils.create_observed_knockdown_mat(
            self.real_knockdown_mat, alpha, beta)
        self._tensor_cache = None
        # U without the S*S*E table: the diagonal rows by their closed form
        # (bit-identical to get_node_lr_table(get_score_tables(D)), tested)
        self.U = self._node_lr_table_direct()
        # compute_real_score side effect (nem.py:90-91): diagonal of the
        # caller's adjacency zeroed in place.
        for i in range(self.num_s):
            adj_matrix[i][i] = 0
        self.real_order_ll = self.real_ll = self.real_parent_order = None
        self.obs_order_ll = self.obs_ll = self.obs_parent_order = None

    # -- A1: score tables -------------------------------------------------
    def _chains(self):
        """Addition chains of A from bases 0.0 and B (see module docstring)."""
        return (_addition_chain(0.0, self.A, self.num_s),
                _addition_chain(self.B, self.A, self.num_s))

    def compute_scores(self, node, knockdown_mat):
        """Base row of ``T[node]``: where(D[node]==1, 0, B) + sum_{m != node}
        where(D[m]==1, A, 0), summed in ascending m.  Reference: nem.py:25-34."""
        d = np.asarray(knockdown_mat)
        ones_elsewhere = (d == 1).sum(axis=0) - (d[node] == 1)
        chain0, chainb = self._chains()
        return np.where(d[node] == 1, chain0[ones_elsewhere], chainb[ones_elsewhere])

    def build_score_table(self, node, knockdown_mat):
        """``T[node]``, shape (S, E).  Row ``node`` is :meth:`compute_scores`;
        every other row m is where(D[m]==0, B, -A).  Reference: nem.py:36-47."""
        d = np.asarray(knockdown_mat)
        table = np.where(d == 0, self.B, -self.A).astype(np.float64)
        table[node, :] = self.compute_scores(node, d)
        return table

    def get_score_tables(self, knockdown_mat):
        """The S tables (S, E).  Reference: nem.py:49-54 (a list of arrays).

        Returned as a lazy sequence: ``tables[i]`` builds T[i] on access and
        ``np.asarray(tables)`` the whole tensor, so a sampler that only hands
        the model to the GPU (which builds its tables from D itself,
        ``nemo_stage_knockdown``) never holds the S*S*E table on the host."""
        return ScoreTables(self, knockdown_mat)

    def get_score_tensor(self, knockdown_mat=None) -> np.ndarray:
        """The score tables as one C-contiguous (S, S, E) float64 tensor
        ``T[i, j, e]`` (child i, parent j) -- the layout staged to HBM."""
        d = self.observed_knockdown_mat if knockdown_mat is None else np.asarray(knockdown_mat)
        if (self._tensor_cache is not None and self._tensor_cache[0] is d):
            return self._tensor_cache[1]
        s, e = self.num_s, self.num_e
        off_diag = np.where(d == 0, self.B, -self.A).astype(np.float64)
        ones_total = (d == 1).sum(axis=0)
        chain0, chainb = self._chains()
        tensor = np.empty((s, s, e), dtype=np.float64)
        tensor[:] = off_diag[None, :, :]
        for i in range(s):
            k = ones_total - (d[i] == 1)
            tensor[i, i] = np.where(d[i] == 1, chain0[k], chainb[k])
        self._tensor_cache = (d, tensor)
        return tensor

    # -- A2: node LR table --------------------------------------------------
    def _node_lr_table_direct(self):
        d = np.asarray(self.observed_knockdown_mat)
        chain0, chainb = self._chains()
        k = ((d == 1).sum(axis=0)[None, :] - (d == 1)).astype(np.int64)
        rows = np.where(d == 1, chain0[k], chainb[k])
        null_row = chain0[(d != 0).sum(axis=0)]
        return np.vstack([rows, null_row[None, :]])

    def get_node_lr_table(self, all_score_tables):
        """Rows 0..S-1: diagonal rows ``T[i][i]``; row S: sum over S-genes of
        where(D==0, 0, A), added row by row.  Reference: nem.py:56-64."""
        s = self.num_s
        rows = [np.asarray(all_score_tables[i])[i] for i in range(s)]
        chain0, _ = self._chains()
        null_row = chain0[(self.observed_knockdown_mat != 0).sum(axis=0)]
        return np.vstack(rows + [null_row])
