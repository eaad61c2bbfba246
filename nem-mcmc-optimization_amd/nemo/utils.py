"""Host-side NEM utilities: knockdown data, DAG helpers, network CSV I/O.

Mirrors the reference module ``utils.py`` (MrGreyPanda/NEM-MCMC-optimization) so a
user of the reference finds the same names, argument meaning and results.
Everything here is O(S*E) host bookkeeping that *feeds* the hot path; the one
numerical routine of ``utils.py`` that sits on the hot path, ``compute_ll``
(utils.py:84-94), runs on the GPU through the C-ABI (``nemo.engine``).

Random-number parity: ``create_observed_knockdown_mat`` consumes Python's global
``random`` stream exactly as the reference does (utils.py:25-35), because the
sampler's proposals continue from that state.
"""
from __future__ import annotations

import os
import random

import numpy as np


def create_connection_mat(s_mat) -> np.ndarray:
    """conn[b, a] = 1 for every edge a->b of ``s_mat``, plus the diagonal.

    Reference: utils.py:5-13.  Returned as float64, like the reference.
    """
    adj = np.asarray(s_mat)
    dim = adj.shape[1]
    conn = (adj[:dim, :dim] == 1).T.astype(np.float64)
    conn[np.diag_indices(dim)] = 1.0
    return conn


def create_real_knockdown_mat(s_mat, e_arr) -> np.ndarray:
    """Noise-free knockdown matrix: knock[i, k] = 1 iff S-gene i is e_arr[k] or
    one of its (closure) parents.  Reference: utils.py:15-23.
    """
    conn = create_connection_mat(s_mat)
    ends = np.asarray(e_arr, dtype=np.int64)
    # row s_gene of conn marks every i with conn[s_gene][i] == 1
    return np.ascontiguousarray(conn[ends, :].T).astype(np.float64)


def create_observed_knockdown_mat(knockdown_mat, alpha, beta, seed=42) -> np.ndarray:
    """Flip 0->1 with prob. alpha and 1->0 with prob. beta, row-major, one
    ``random.random()`` draw per cell after ``random.seed(seed)``.

    Reference: utils.py:25-35.  The draws are taken from the *global* Python
    RNG in the same order, so the RNG state afterwards is identical.
    """
    random.seed(seed)
    real = np.asarray(knockdown_mat, dtype=np.float64)
    rows, cols = real.shape
    draws = np.fromiter((random.random() for _ in range(rows * cols)),
                        dtype=np.float64, count=rows * cols).reshape(rows, cols)
    obs = real.copy()
    obs[(real == 0) & (draws < alpha)] = 1.0
    obs[(real == 1) & (draws < beta)] = 0.0
    return obs


def ancestor(incidence) -> np.ndarray:
    """Ancestor (reachability) matrix by summing integer matrix powers.

    Reference: utils.py:37-54.  The reference accumulates A + A^2 + ... + A^S
    in the input's integer dtype; path counts can wrap around int64 for dense
    graphs (S >= 63), which changes ``> 0``.  We keep that arithmetic so the
    result is identical, wrap-around included.
    """
    inc = np.asarray(incidence)
    n = inc.shape[0]
    power = inc.copy()
    total = inc.copy()
    with np.errstate(over="ignore"):
        for _ in range(1, n):
            power = power.dot(inc)
            total += power
    return (total > 0).astype(int)


def initial_order_guess(observed_knockdown_mat) -> np.ndarray:
    """Order S-genes by decreasing number of observed effects.

    Reference: utils.py:56-64 (numpy's default argsort kind, so ties break the
    same way).
    """
    row_sums = np.sum(observed_knockdown_mat, axis=1)
    return np.argsort(-row_sums)


def compute_ll(cell_ratios) -> float:
    """sum_e logsumexp_i cell_ratios[i, e] -- evaluated on the GPU.

    Reference: utils.py:84-94.  Runs the device LSE kernel through the C-ABI
    (``nemo_lse``); there is no host fallback.
    """
    from .engine import lse_ll
    return lse_ll(np.asarray(cell_ratios, dtype=np.float64))


def read_csv_to_adj(pathname):
    """Parse a bundled network CSV.

    Format (reference utils.py:96-118): ``S,E`` header; one ``a,b`` line per
    (closure) edge a->b; one line of E end-node indices; one ``alpha,beta``
    line.  Relative paths resolve against the current directory, as in the
    reference.  Returns (adj int (S,S), end_nodes, errors, S, E).
    """
    path = os.path.join(os.getcwd(), pathname)
    with open(path, "r") as fh:
        lines = fh.read().splitlines()
    num_s, num_e = (int(v) for v in lines[0].strip().split(","))
    adj = np.zeros((num_s, num_s), dtype=int)
    idx = 1
    end_line = None
    while idx < len(lines):
        fields = [int(v) for v in lines[idx].strip().split(",")]
        idx += 1
        if len(fields) != 2:
            end_line = fields
            break
        adj[fields[0], fields[1]] = 1
    if end_line is None:
        raise ValueError(f"{pathname}: no end-node line")
    end_nodes = np.array(end_line)
    errors = np.array([float(v) for v in lines[idx].strip().split(",")])
    return adj, end_nodes, errors, num_s, num_e


def write_adj_to_csv(pathname, adj, end_nodes, errors) -> None:
    """Inverse of :func:`read_csv_to_adj` (the bundled-network format)."""
    adj = np.asarray(adj)
    with open(pathname, "w") as fh:
        fh.write(f"{adj.shape[0]},{len(end_nodes)}\n")
        for a, b in zip(*np.nonzero(adj)):
            fh.write(f"{a},{b}\n")
        fh.write(",".join(str(int(v)) for v in end_nodes) + "\n")
        fh.write(",".join(repr(float(v)) for v in errors) + "\n")


def transitive_reduction(adj_matrix) -> np.ndarray:
    """Remove edges implied by longer paths.  Reference: utils.py:120-129."""
    red = np.array(adj_matrix, copy=True)
    n = red.shape[0]
    for k in range(n):
        for i in range(n):
            if not red[i, k]:
                continue
            # the reference scans j in order and updates in place: once j == k
            # with a self-loop on k clears red[i, k], later j see no path
            stop = k + 1 if (i != k and red[k, k]) else n
            cols = np.nonzero(red[k, :stop])[0]
            cols = cols[cols != i]
            red[i, cols] = 0
    return red


def hamming_distance(mat_a, mat_b):
    """Reference: utils.py:148-149."""
    return np.sum(np.abs(np.asarray(mat_a) - np.asarray(mat_b)))


def order_arr(order, unsorted_array) -> np.ndarray:
    """Permute every axis of ``unsorted_array`` by argsort(order).
    Reference: utils.py:173-188."""
    idx = np.argsort(order)
    out = np.asarray(unsorted_array)
    return out[np.ix_(*([idx] * out.ndim))]


def unorder_arr(perm_order, sorted_array) -> np.ndarray:
    """Inverse of :func:`order_arr`.  Reference: utils.py:190-216."""
    inv = np.argsort(np.argsort(perm_order))
    out = np.asarray(sorted_array)
    return out[np.ix_(*([inv] * out.ndim))]
