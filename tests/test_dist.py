"""Multi-rank path on CPU (gloo, world_size 2): chain sharding and the
all-gather of per-chain best scores/orders that closes a C4 run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from nemo import chains


def test_shard_partitions_chains():
    for n, world in ((128, 8), (10, 3), (5, 8), (0, 2)):
        got = [list(chains.shard(n, r, world)) for r in range(world)]
        assert sum(got, []) == list(range(n))
        sizes = [len(g) for g in got]
        assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_chains, s, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = chains.shard(n_chains, rank, world)
    rng = np.random.default_rng(100 + rank)
    scores = np.array([-1000.0 - c for c in mine])
    orders = np.array([np.roll(np.arange(s), c) for c in mine], dtype=np.int32).reshape(len(mine), s)
    gs, go = chains.gather_best(scores, orders)
    if rank == 0:
        out.put((gs, go))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_chains", [7, 16])
def test_gather_best_gloo_world2(n_chains):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = 6
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_chains, s, q)) for r in range(2)]
    for p in procs:
        p.start()
    gs, go = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(gs, np.array([-1000.0 - c for c in range(n_chains)]))
    assert np.array_equal(go, np.array([np.roll(np.arange(s), c) for c in range(n_chains)]))
