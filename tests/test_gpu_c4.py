"""BASELINE config C4 on the GPU: 128 chains of the C3 model (64 x 2000), the
per-rank share as one ChainBatch, and the one collective -- an all-gather of
every chain's (best score, best order) as device tensors over RCCL
(``nemo.chains.gather_best``; the reference runs its chains one after the
other in one process, nem_order_mcmc.py:316-363).  A world-size-1 ``nccl``
process group on cuda:0 executes the same RCCL call sites the 8-GPU run uses
(``nemo/chains.py`` gather_best / run_c4, ``bench.py`` timed_steps), and the
gathered results are checked against independent single-chain samplers."""
import hashlib
import os
import random
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_world1():
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        yield dist
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def c3():
    from nemo import generator
    from nemo.engine import Engine
    m = generator.config_nem("C3")
    return m, Engine.for_nem(m)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()[:16]


def test_c4_128_chains_rccl_gather(rccl_world1, c3):
    """run_c4 at C3 with 128 chains for 3 steps, gathered over RCCL: every chain
    gathered; chains 0, 91 and 127 equal independent NEMOrderMCMC runs with
    their seeds (accepts, best score and order); the gathered scores equal a
    one-group ChainBatch run bit for bit."""
    import torch
    from nemo import utils
    from nemo.chains import ChainBatch, run_c4
    from nemo.nem_order_mcmc import NEMOrderMCMC
    dist = rccl_world1
    m, eng = c3
    steps = 3
    r = run_c4(m, eng, n_chains=128, steps=steps, warmup_steps=0, device=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and r["gathered_over"] == "nccl"
    assert r["n_gathered"] == 128 and r["n_ranks"] == 1 and r["chains_per_rank"] == 128
    scores, orders = r["scores"], r["orders"]
    assert scores.dtype == np.float64 and orders.shape == (128, m.num_s)
    acc = np.asarray(r["accepted"])
    assert acc.shape == (steps, 128)
    order0 = utils.initial_order_guess(m.observed_knockdown_mat)
    gamma = 2.0 * m.num_s / m.num_e
    for c in (0, 91, 127):
        smp = NEMOrderMCMC(m, np.asarray(order0), engine=eng)
        smp.rng = random.Random(1234 + c)
        best, _dag = smp.method(n_iterations=steps, gamma=gamma, swap_prob=0.95, verbose=False)
        assert np.array_equal(np.array(smp.accepted), acc[:, c]), c
        assert best == scores[c], c
        assert np.array_equal(np.asarray(smp.best_order), orders[c]), c
    cb = ChainBatch(m, [order0] * 128, seeds=[1234 + c for c in range(128)], engine=eng, on_fail="continue",
                    groups=1)
    best, best_orders = cb.run(steps)
    assert _sha(best) == r["scores_sha256"] == _sha(scores)
    assert np.array_equal(best_orders, orders)


def test_bench_timed_region_gathers_over_rccl(rccl_world1, c3):
    """bench.py's timed region with its collective on: the barrier and the
    all-gather of the batch's best score as a device tensor over RCCL."""
    import torch
    from scipy.special import expit
    sys.path.insert(0, REPO)
    import bench
    dist = rccl_world1
    m, eng = c3
    b = 64
    rng = np.random.default_rng(5)
    pos = np.array([rng.permutation(m.num_s) for _ in range(b)], dtype=np.int32)
    w01 = expit(rng.uniform(-3, 3, (b, m.num_s, m.num_s)))
    eng.reserve(b)
    d_pos, d_w01 = torch.from_numpy(pos).cuda(), torch.from_numpy(w01).cuda()
    d_ll = torch.zeros(b, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    wall, kern_ms, _ = bench.timed_steps(eng, torch, b, 0, 3, 1, d_pos, d_w01, d_ll, stream, 1, dist,
                                         collective=True)
    assert wall > 0 and kern_ms > 0
    # the timed region runs the batched fixed-point kernel: the host call with
    # the fast kernels gives its bits (the exact arithmetic is within 1e-6)
    eng.set_option("exact", 0)
    try:
        assert np.array_equal(d_ll.cpu().numpy(), eng.score(pos, w01))
    finally:
        eng.set_option("exact", 1)
    assert np.max(np.abs(d_ll.cpu().numpy() - eng.score(pos, w01))) <= 1e-6
