"""Replica exchange host logic (nem_order_mcmc.py:316-363) on CPU: the
pre-drawn shared random stream, the exchange decisions, and the gloo
world-size-2 path, with a stand-in scorer.  The GPU run against the
reference's own replica_exchange_method golden is in test_gpu_parity.py."""
import os
import random
import socket
import types

import numpy as np
import pytest
import torch.multiprocessing as mp

from nemo import replicas
from nemo.nem_order_mcmc import NEMOrderMCMC


def _fake_chain(s, order):
    c = types.SimpleNamespace(num_s=s, perm_order=np.asarray(order), perm_orders=[np.asarray(order)])
    c.get_new_order = types.MethodType(NEMOrderMCMC.get_new_order, c)
    c.accepting = types.MethodType(NEMOrderMCMC.accepting, c)
    return c


def _fake_ll(order):
    """Deterministic stand-in score of an order."""
    o = np.asarray(order)
    return -float(np.sum(np.abs(o - np.arange(len(o))) * (1 + np.arange(len(o)) % 3)))


def fake_method(c, gamma, n_iters, swap_prob=0.95):
    """method()'s random-call sequence and accept logic with the stand-in score."""
    curr = _fake_ll(c.perm_order)
    best = curr
    curr_perm = c.perm_order
    for _ in range(n_iters):
        perm, _i1, _i2 = c.get_new_order(curr_perm, swap_prob=swap_prob)
        ll = _fake_ll(perm)
        acc, curr, _, curr_perm = c.accepting(ll, curr, gamma, None, None, perm, curr_perm)
        if acc and curr > best:
            best = curr
    c.best_score = best
    return best


def fake_runner(chains, gammas, n_iters, engine, swap_prob=0.95, use_nem=False, cap=0):
    return np.array([fake_method(c, g, n_iters, swap_prob) for c, g in zip(chains, gammas)])


def sequential_reference(s, e, order, n_rep, n_exchange, n_iter, seed):
    """nem_order_mcmc.py:316-363 transcribed, with the stand-in method."""
    rng = random.Random(seed)
    gammas = [(1.0 + i * 0.2) * s / e for i in range(n_rep)]
    reps = []
    for _ in range(n_rep):
        c = _fake_chain(s, order)
        c.rng = rng
        reps.append(c)
    ids = list(range(n_rep))
    scores = np.zeros(n_rep)
    up = True
    hist = []
    for _ in range(n_exchange):
        for i in range(n_rep):
            fake_method(reps[i], gammas[i], n_iter)
            scores[i] = reps[i].best_score
        best_score = np.max(scores)
        best_id = ids[int(np.argmax(scores))]
        pairs = [(j - 1, j) for j in range(1 if up else 2, n_rep, 2)]
        n_ex = 0
        for (i, j) in pairs:
            delta = gammas[i] * scores[j] - gammas[i] * scores[i] + gammas[j] * scores[i] - gammas[j] * scores[j]
            if rng.random() < np.exp(-delta):
                reps[i], reps[j] = reps[j], reps[i]
                ids[i], ids[j] = ids[j], ids[i]
                scores[i], scores[j] = scores[j], scores[i]
                n_ex += 1
                if scores[i] > best_score:
                    best_score, best_id = scores[i], ids[i]
        hist.append((scores.copy(), list(ids), n_ex, best_score, best_id))
        up = not up
    return hist, rng.getstate()


def _nem(s, e):
    return types.SimpleNamespace(num_s=s, num_e=e)


def _run_batched(s, e, order, n_rep, n_exchange, n_iter, seed, rank=0, world=1):
    rng = random.Random(seed)
    rx = replicas.ReplicaExchange(_nem(s, e), order, n_replicas=n_rep, rng=rng, rank=rank, world=world,
                                  make_replica=lambda o: _fake_chain(s, o), runner=fake_runner)
    hist = []
    for _ in range(n_exchange):
        best_score, best_obj, n_ex = rx.step(n_iter, next(rx._cycler))
        hist.append((rx.scores.copy(), list(rx.obj_at_pos), n_ex, best_score, best_obj))
    return hist, rng.getstate()


def test_replay_reproduces_direct_calls():
    s = 9
    rng_a, rng_b = random.Random(5), random.Random(5)
    direct = _fake_chain(s, np.arange(s))
    direct.rng = rng_a
    replayed = _fake_chain(s, np.arange(s))
    replayed.rng = replicas._Replay()
    replicas._predraw_steps(rng_b, replayed.rng, 50, s, 0.7)
    curr_a = curr_b = np.arange(s)
    for _ in range(50):
        pa = direct.get_new_order(curr_a, swap_prob=0.7)
        pb = replayed.get_new_order(curr_b, swap_prob=0.7)
        assert all(np.array_equal(x, y) for x, y in zip(pa, pb))
        assert direct.accepting(-1.0, -0.5, 1.0, None, None, pa[0], curr_a)[0] == \
            replayed.accepting(-1.0, -0.5, 1.0, None, None, pb[0], curr_b)[0]
        curr_a, curr_b = pa[0], pb[0]
    assert not replayed.rng.q and rng_a.getstate() == rng_b.getstate()


@pytest.mark.parametrize("n_rep", [10, 5])
def test_batched_replica_exchange_matches_sequential(n_rep):
    s, e = 8, 40
    order = np.random.default_rng(1).permutation(s)
    want, state_w = sequential_reference(s, e, order, n_rep, 4, 6, 99)
    got, state_g = _run_batched(s, e, order, n_rep, 4, 6, 99)
    assert state_w == state_g
    for (sw, iw, nw, bw, bidw), (sg, ig, ng, bg, bidg) in zip(want, got):
        assert np.array_equal(sw, sg) and iw == ig and nw == ng and bw == bg and bidw == bidg


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    order = np.random.default_rng(1).permutation(8)
    hist, _ = _run_batched(8, 40, order, 10, 4, 6, 99, rank=rank, world=world)
    out.put((rank, [(h[0].tolist(), h[1], h[2], h[3], h[4]) for h in hist]))
    dist.destroy_process_group()


def test_replica_exchange_gloo_world2():
    """Objects split over two ranks (object r on rank r % 2); one all-gather of
    best scores per round; both ranks reach the single-process result."""
    want, _ = sequential_reference(8, 40, np.random.default_rng(1).permutation(8), 10, 4, 6, 99)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        for (sw, iw, nw, bw, bidw), (sg, ig, ng, bg, bidg) in zip(want, res[rank]):
            assert np.array_equal(sw, np.array(sg)) and iw == ig and nw == ng and bw == bg and bidw == bidg
