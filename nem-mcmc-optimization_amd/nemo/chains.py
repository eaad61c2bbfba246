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
from .nem_order_mcmc import SIG0, SIG1, NEMOrderMCMC


def shard(n_chains: int, rank: int, world: int) -> range:
    """Contiguous block of global chain ids owned by ``rank``."""
    base, extra = divmod(n_chains, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


class ChainBatch:
    """``n`` independent order-MCMC chains on one staged model.

    Chain ``c`` uses ``random.Random(seed + c)`` for its proposals and
    acceptances, in exactly the reference's call order, so chain ``c`` of a
    batch reproduces a single ``NEMOrderMCMC.method`` run driven by that
    stream."""

    def __init__(self, nem, init_orders, seeds, engine: Engine | None = None, gamma=None,
                 swap_prob=0.95, use_nem=False, cap=0):
        self.nem = nem
        self.engine = engine if engine is not None else Engine.for_nem(nem)
        self.n = len(init_orders)
        self.gamma = (2.0 * nem.num_s / nem.num_e) if gamma is None else gamma
        self.gammas = np.broadcast_to(np.asarray(self.gamma, dtype=float), (self.n,)).copy()
        self.swap_prob = swap_prob
        self.use_nem = use_nem
        self.cap = cap
        self.chains = []
        for order, seed in zip(init_orders, seeds):
            c = NEMOrderMCMC(nem, np.asarray(order), engine=self.engine, cap=cap)
            c.rng = random.Random(seed)
            self.chains.append(c)
        self.engine.reserve(self.n, self.n)

    # one batched get_optimal_weights(init=True) over all chains
    def _optimal_weights(self):
        s = self.nem.num_s
        pos = np.stack([c._pos for c in self.chains]).astype(np.int32)
        w = np.stack([c.parent_weights for c in self.chains])
        w01 = expit(w)
        anc = np.empty_like(w)
        eye = np.identity(s)
        for k, c in enumerate(self.chains):
            c.ancestor_x = np.clip(inv(eye - c.expit_parent_weights(w[k])) - eye, 0, 1)
            anc[k] = c.ancestor_x
        w_new, ll1, lld, _ = self.engine.optimal_weights(pos, w01, anc, w, SIG0, SIG1, cap=self.cap)
        out = np.empty(self.n)
        for k, c in enumerate(self.chains):
            c.parent_weights = w_new[k].copy()
            c.ll = float(ll1[k])
            if self.use_nem:
                _, dag = c.create_nem(c.parent_weights)
                out[k] = float(self.engine.score(c._pos[None, :], expit(dag.astype(float))[None],
                                                 cap=self.cap)[0])
            else:
                out[k] = float(lld[k])
        return out

    def run(self, n_iterations: int):
        """Every chain runs the reference's ``method`` loop
        (nem_order_mcmc.py:257-310) for ``n_iterations`` steps."""
        curr = self._optimal_weights()
        self.curr_scores = curr.copy()
        self.best_scores = curr.copy()
        self.curr_orders = [c.perm_order for c in self.chains]
        self.best_orders = [np.asarray(o).copy() for o in self.curr_orders]
        self.accepted = np.zeros((n_iterations, self.n), dtype=bool)
        for it in range(n_iterations):
            props = []
            for k, c in enumerate(self.chains):
                perm, i1, i2 = c.get_new_order(self.curr_orders[k], swap_prob=self.swap_prob)
                c.reset(perm_order=perm, i1=i1, i2=i2)
                props.append(perm)
            lls = self._optimal_weights()
            for k, c in enumerate(self.chains):
                acc, self.curr_scores[k], _, self.curr_orders[k] = c.accepting(
                    lls[k], self.curr_scores[k], self.gammas[k], None, None, props[k], self.curr_orders[k])
                self.accepted[it, k] = acc
                if acc and self.curr_scores[k] > self.best_scores[k]:
                    self.best_scores[k] = self.curr_scores[k]
                    self.best_orders[k] = np.asarray(self.curr_orders[k]).copy()
        return self.best_scores, np.stack(self.best_orders)


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
