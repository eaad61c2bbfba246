"""GPU: the multi-rank paths rehearsed on one MI355X -- two ``gloo`` ranks
sharing cuda:0, each with its own staged engine, against the same work done by
one process.  The C4 path (``nemo.chains.run_c4``: chains sharded over the
ranks, one all-gather of every chain's best score and order) and the replica
exchange (``nemo.replicas.ReplicaExchange``: replicas owned round-robin by the
ranks, one all-gather of the scores per round, the shared stream drawn
identically on every rank) must give the world-1 run's results bit for bit.
The 8-GPU run itself is the driver's (the same code, ``nccl`` = RCCL)."""
import hashlib
import os
import random
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()[:16]


def _rank_main(rank, world, port, q):
    """One rank: a gloo group, its own engine on cuda:0, run_c4 (32 chains of C3,
    3 steps) and 2 rounds of a 6-replica exchange on C2."""
    import torch.distributed as dist

    from nemo import generator, utils
    from nemo.chains import run_c4
    from nemo.engine import Engine
    from nemo.replicas import ReplicaExchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = generator.config_nem("C3")
        eng = Engine.for_nem(m)
        r = run_c4(m, eng, n_chains=32, steps=3, warmup_steps=0, inv_workers=1)
        m2 = generator.config_nem("C2")
        rx = ReplicaExchange(m2, utils.initial_order_guess(m2.observed_knockdown_mat), n_replicas=6,
                             rng=random.Random(2025), rank=rank, world=world)
        rounds = []
        for k in range(2):
            best, best_obj, nx = rx.step(2, k % 2 == 0)
            rounds.append((rx.scores.copy(), nx, best, best_obj, list(rx.obj_at_pos)))
        if rank == 0:
            q.put(dict(c4=dict(n_gathered=r["n_gathered"], n_ranks=r["n_ranks"], chains_per_rank=r["chains_per_rank"],
                               sha=r["scores_sha256"], scores=r["scores"], orders=r["orders"],
                               backend=r["gathered_over"]),
                       rx=rounds))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_gloo_ranks_on_one_gpu_equal_world1():
    import torch.multiprocessing as mp

    from nemo import generator, utils
    from nemo.chains import run_c4
    from nemo.engine import Engine
    from nemo.replicas import ReplicaExchange
    # world 1, this process, no process group
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    r1 = run_c4(m, eng, n_chains=32, steps=3, warmup_steps=0, inv_workers=1)
    assert r1["n_gathered"] == 32 and r1["n_ranks"] == 1
    m2 = generator.config_nem("C2")
    rx = ReplicaExchange(m2, utils.initial_order_guess(m2.observed_knockdown_mat), n_replicas=6,
                         rng=random.Random(2025))
    rounds1 = []
    for k in range(2):
        best, best_obj, nx = rx.step(2, k % 2 == 0)
        rounds1.append((rx.scores.copy(), nx, best, best_obj, list(rx.obj_at_pos)))
    # world 2: two spawned ranks sharing cuda:0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    c4 = got["c4"]
    assert c4["backend"] == "gloo" and c4["n_ranks"] == 2 and c4["chains_per_rank"] == 16
    assert c4["n_gathered"] == 32
    assert c4["sha"] == r1["scores_sha256"] == _sha(c4["scores"])
    assert np.array_equal(c4["orders"], r1["orders"])
    for (s2, nx2, b2, o2, pos2), (s1, nx1, b1, o1, pos1) in zip(got["rx"], rounds1):
        assert np.array_equal(s2, s1) and nx2 == nx1 and b2 == b1 and o2 == o1 and pos2 == pos1
    eng.close()

