"""Replica exchange (parallel tempering) over the batched scorer.

Reference: ``replica_exchange_step`` / ``replica_exchange_method``,
nem_order_mcmc.py:316-363 -- 10 replicas at gamma_r = (1 + 0.2 r) S / E, each
round every replica runs ``method(n_iter)`` in turn, then neighbouring
positions (0,1),(2,3),... or (1,2),(3,4),... swap replicas with probability
exp(-delta), all from the one global ``random`` stream.

Built the MI355X way, with the same trajectory:

* The random draws of a round do not depend on any score: per step
  ``get_new_order`` draws (random, then sample or randint) and ``accepting``
  one random, whatever the outcome; the exchange draws one random per
  partner pair.  So a round's stream is drawn up front, in the reference's
  order (position 0's steps, position 1's, ..., then the exchange draws),
  into one replay queue per replica, and all replicas then advance in
  lock-step -- ONE fused ``optimal_weights`` call per MCMC step for all of a
  GPU's replicas (``chains.run_methods``).
* Over GPUs, replica objects stay where they were created (object r on rank
  r % world).  An exchange swaps which object sits at which position (and so
  its gamma and its slice of the stream), never the object's state; every
  rank draws the whole stream from the shared seed and makes the same
  exchange decisions after one all-gather of the objects' best scores
  (SURVEY.md 8(e)).
"""
from __future__ import annotations

import collections
import random
from itertools import cycle

import numpy as np

from .chains import run_methods
from .engine import Engine
from .nem_order_mcmc import NEMOrderMCMC


class _Replay:
    """Random-stream facade replaying pre-drawn values in call order (the
    three calls ``get_new_order`` and ``accepting`` make)."""

    def __init__(self):
        self.q = collections.deque()

    def random(self):
        return self.q.popleft()

    def sample(self, population, k):
        return self.q.popleft()

    def randint(self, a, b):
        return self.q.popleft()


def _predraw_steps(rng, replay: _Replay, n_steps: int, s: int, swap_prob: float):
    for _ in range(n_steps):
        u = rng.random()                       # is_swap (nem_order_mcmc.py:237)
        replay.q.append(u)
        if u < swap_prob:
            replay.q.append(rng.sample(range(s), 2))   # :240
        else:
            replay.q.append(rng.randint(0, s - 2))     # :246
        replay.q.append(rng.random())          # accepting (:226)


def partners(n_replicas: int, upwards: bool):
    """nem_order_mcmc.py:328-333."""
    start = 1 if upwards else 2
    return [(j - 1, j) for j in range(start, n_replicas, 2)]


def exchange(scores, gammas, obj_at_pos, pairs, us):
    """The exchange loop of nem_order_mcmc.py:334-341 on positions, given the
    pre-drawn uniforms ``us`` (one per pair).  Mutates ``scores`` and
    ``obj_at_pos``; returns (n_exchanges, best_score, best object id) -- the
    best is taken before the swaps, as there (:326-327)."""
    best_pos = int(np.argmax(scores))
    best_score = float(scores[best_pos])
    best_obj = obj_at_pos[best_pos]
    n_ex = 0
    for (i, j), u in zip(pairs, us):
        delta = gammas[i] * scores[j] - gammas[i] * scores[i] + gammas[j] * scores[i] - gammas[j] * scores[j]
        if u < np.exp(-delta):
            obj_at_pos[i], obj_at_pos[j] = obj_at_pos[j], obj_at_pos[i]
            scores[i], scores[j] = scores[j], scores[i]
            n_ex += 1
            if scores[i] > best_score:
                best_score = float(scores[i])
                best_obj = obj_at_pos[i]
    return n_ex, best_score, best_obj


class ReplicaExchange:
    """``n_replicas`` tempered replicas of ``NEMOrderMCMC`` on the GPU(s).

    ``rng`` is the shared stream (default: the global ``random`` module, as the
    reference uses); with ``world > 1`` every rank must pass an identically
    seeded ``random.Random``."""

    def __init__(self, nem, init_order, n_replicas=10, engine: Engine | None = None, rng=None,
                 swap_prob=0.95, use_nem=False, cap=0, rank=0, world=1, device=None,
                 make_replica=None, runner=None):
        self.nem = nem
        self.n = n_replicas
        self.s = nem.num_s
        self.rng = random if rng is None else rng
        self.swap_prob, self.use_nem, self.cap = swap_prob, use_nem, cap
        self.rank, self.world, self.device = rank, world, device
        self.gammas = [(1.0 + i * 0.2) * nem.num_s / nem.num_e for i in range(n_replicas)]
        self.local = [r for r in range(n_replicas) if r % world == rank]
        # make_replica / runner: injection points for host-logic tests only
        self.runner = run_methods if runner is None else runner
        if make_replica is None:
            self.engine = engine if engine is not None else Engine.for_nem(nem)
            self.engine.reserve(max(1, len(self.local)), max(1, len(self.local)))

            def make_replica(order):
                return NEMOrderMCMC(nem, np.asarray(order), engine=self.engine, cap=cap)
        else:
            self.engine = engine
        self.objs = {}
        for r in self.local:
            c = make_replica(init_order)
            c.rng = _Replay()
            self.objs[r] = c
        self.obj_at_pos = list(range(n_replicas))
        self.scores = np.zeros(n_replicas)
        self.n_exchanges = 0
        self._cycler = cycle([True, False])

    def _gather_scores(self, local_best):
        """Best score of every replica object (all-gather over ranks)."""
        out = np.full(self.n, np.nan)
        for r, v in local_best.items():
            out[r] = v
        if self.world == 1:
            return out
        import torch
        import torch.distributed as dist
        t = torch.as_tensor(np.nan_to_num(out, nan=-np.inf), dtype=torch.float64)
        if self.device is not None:
            t = t.to(self.device)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t)
        allv = np.stack([p.cpu().numpy() for p in parts])
        for r in range(self.n):
            out[r] = allv[r % self.world][r]
        return out

    def step(self, n_iters: int, upwards: bool):
        """One ``replica_exchange_step`` (nem_order_mcmc.py:316-342).  Returns
        (best_score, best replica object id, n_exchanges)."""
        pos_of = {r: p for p, r in enumerate(self.obj_at_pos)}
        for p in range(self.n):                     # the stream, in the reference's order
            r = self.obj_at_pos[p]
            _predraw_steps(self.rng, self.objs[r].rng if r in self.objs else _Replay(),
                           n_iters, self.s, self.swap_prob)
        pairs = partners(self.n, upwards)
        us = [self.rng.random() for _ in pairs]
        chains = [self.objs[r] for r in self.local]
        gam = [self.gammas[pos_of[r]] for r in self.local]
        best = self.runner(chains, gam, n_iters, self.engine, swap_prob=self.swap_prob,
                           use_nem=self.use_nem, cap=self.cap) if chains else []
        for c in chains:
            c.perm_orders = [c.perm_orders[-1]]     # nem_order_mcmc.py:324
        obj_best = self._gather_scores(dict(zip(self.local, best)))
        self.scores = np.array([obj_best[self.obj_at_pos[p]] for p in range(self.n)])
        n_ex, best_score, best_obj = exchange(self.scores, self.gammas, self.obj_at_pos, pairs, us)
        self.n_exchanges += n_ex
        return best_score, best_obj, n_ex

    def run(self, n_exchange: int, n_iter: int):
        """``replica_exchange_method``'s loop (nem_order_mcmc.py:354-363): the
        best score and replica id of the LAST round, as the reference returns."""
        best_score, best_obj = None, None
        for _ in range(n_exchange):
            best_score, best_obj, _ = self.step(n_iter, next(self._cycler))
        self.best_score, self.best_obj = best_score, best_obj
        return best_score, best_obj


def replica_exchange_batched(nem, n_exchange, n_iter, init_order_guess, n_replicas=10, **kw):
    """Drop-in for ``replica_exchange_method`` (nem_order_mcmc.py:344-363)
    with all replicas batched on the GPU.  Returns (best_score, best_nem) with
    best_nem the winning replica's ``NEMOrderMCMC`` (single process)."""
    rx = ReplicaExchange(nem, init_order_guess, n_replicas=n_replicas, **kw)
    best_score, best_obj = rx.run(n_exchange, n_iter)
    return best_score, rx.objs.get(best_obj)
