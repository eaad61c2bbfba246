"""Synthetic NEM generator for the benchmark configurations.

The reference's own DAG generator (DAGs/rnd_dag_gen.py:47-103) is rank-based and
cannot target a given number of S-genes, so the synthetic configurations
C2/C3/C5 of BASELINE.json use this build-defined generator:

* a random topological order ``rng.permutation(S)``; an edge a->b for every
  pair with a before b, independently with probability ``edge_p``;
* the transitive closure of that DAG (the bundled CSVs store closures);
* ``end_nodes = rng.integers(0, S, E)``;
* errors (alpha, beta) = (0.05, 0.10), as in networks 10-19;
* D from :class:`nemo.nem.NEM`, i.e. the reference's knockdown semantics with
  Python ``random.seed(42)`` (utils.py:25-35).

``rng = numpy.random.default_rng(seed)`` drives everything except D.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .nem import NEM

# name -> (S, E, seed, parent cap, table dtype)
CONFIGS = {
    "C2": (16, 500, 0, 0, "f64"),
    "C3": (64, 2000, 0, 0, "f64"),
    "C5": (128, 5000, 0, 6, "f32"),
    # uncapped 64 < S <= 128 (the int8 log2 kernel for wide models,
    # score_i8w_kernel; not a BASELINE config)
    "W128": (128, 2000, 0, 0, "f64"),
}


@dataclass
class SyntheticNetwork:
    adj: np.ndarray          # (S, S) int closure adjacency, adj[a, b] = edge a->b
    end_nodes: np.ndarray    # (E,) int
    errors: tuple            # (alpha, beta)
    num_s: int
    num_e: int


def transitive_closure(adj: np.ndarray) -> np.ndarray:
    """Boolean reachability (Warshall), returned as int adjacency."""
    reach = np.asarray(adj).astype(bool).copy()
    for k in range(reach.shape[0]):
        reach |= reach[:, k:k + 1] & reach[k:k + 1, :]
    np.fill_diagonal(reach, False)
    return reach.astype(int)


def synthetic_network(num_s: int, num_e: int, seed: int = 0, edge_p: float = 0.1,
                      errors=(0.05, 0.10)) -> SyntheticNetwork:
    rng = np.random.default_rng(seed)
    topo = rng.permutation(num_s)
    draws = rng.random((num_s, num_s))
    adj = np.zeros((num_s, num_s), dtype=int)
    a_pos, b_pos = np.triu_indices(num_s, k=1)
    keep = draws[a_pos, b_pos] < edge_p
    adj[topo[a_pos[keep]], topo[b_pos[keep]]] = 1
    adj = transitive_closure(adj)
    end_nodes = rng.integers(0, num_s, num_e)
    return SyntheticNetwork(adj, end_nodes, tuple(errors), num_s, num_e)


def synthetic_nem(num_s: int, num_e: int, seed: int = 0, **kw) -> NEM:
    net = synthetic_network(num_s, num_e, seed, **kw)
    return NEM(net.adj.copy(), net.end_nodes, net.errors, num_s, num_e)


def config_nem(name: str) -> NEM:
    s, e, seed, _cap, _dtype = CONFIGS[name]
    return synthetic_nem(s, e, seed)


def random_chain_inputs(num_s: int, chain: int, wscale: float = 3.0):
    """One evaluation input (pos, raw W) as SURVEY.md 8(d) specifies:
    a random order (seed 1234 + chain) and W ~ U(-wscale, wscale) pre-sigmoid.

    Returns (perm, pos, W): perm[p] = node at position p, pos = inverse.
    """
    rng = np.random.default_rng(1234 + chain)
    perm = rng.permutation(num_s)
    pos = np.empty(num_s, dtype=np.int64)
    pos[perm] = np.arange(num_s)
    w = rng.uniform(-wscale, wscale, size=(num_s, num_s))
    return perm, pos, w


def permissible_mask(pos: np.ndarray, cap: int = 0) -> np.ndarray:
    """mask[i, j] = j is a permissible parent of i: pos[j] < pos[i], and with a
    parent cap, one of the ``cap`` nearest predecessors of i in the order."""
    pos = np.asarray(pos)
    gap = pos[:, None] - pos[None, :]
    mask = gap > 0
    if cap:
        mask &= gap <= cap
    return mask
