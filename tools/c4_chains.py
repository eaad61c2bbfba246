"""BASELINE config C4: N_CHAINS independent order-MCMC chains of the C3 model
sharded over the ranks (one process per GPU), each rank running its share as
one ChainBatch (the reference's per-chain state machines, one fused device
step per MCMC step for all of them), then ONE all-gather of every chain's
(best score, best order) -- the only collective.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P tools/c4_chains.py [--chains 128] [--steps 50]

NEMO_BENCH_BACKEND=gloo rehearses N > 1 with several ranks on one GPU (device
= local rank modulo the visible GPUs); RCCL ("nccl") is the default.  Rank 0
prints one JSON line: aggregate chain-steps/s (max wall over ranks) and the
global best.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--inv-workers", type=int, default=8)
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("NEMO_BENCH_BACKEND", "nccl")
    local = local % max(torch.cuda.device_count(), 1) if backend != "nccl" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from nemo import generator, utils
    from nemo.chains import ChainBatch, gather_best, shard
    from nemo.engine import Engine
    from nemo.invpool import InvPool

    m = generator.config_nem(a.config)
    eng = Engine.for_nem(m, device=local)
    mine = shard(a.chains, rank, world)
    order = utils.initial_order_guess(m.observed_knockdown_mat)
    seeds = [1234 + c for c in mine]  # chain c's stream whatever the rank count
    pool = InvPool(m.num_s, len(mine), a.inv_workers) if a.inv_workers and len(mine) else None
    try:
        ChainBatch(m, [order] * len(mine), seeds=seeds, engine=eng, on_fail="continue", inv_pool=pool).run(2)
        cb = ChainBatch(m, [order] * len(mine), seeds=seeds, engine=eng, on_fail="continue", inv_pool=pool)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        best, orders = cb.run(a.steps)
        dev = torch.device("cuda", local) if backend == "nccl" else None
        if world > 1:
            all_s, all_o = gather_best(best, orders, device=dev)
        else:
            all_s, all_o = np.asarray(best), np.asarray(orders)
        wall = time.perf_counter() - t0
    finally:
        if pool is not None:
            pool.close()
    t = torch.tensor([wall], dtype=torch.float64, device=dev if dev is not None else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    if rank == 0:
        g = int(np.argmax(all_s))
        print(json.dumps({
            "workload": f"C4: {a.chains} chains of the {a.config} model over {world} rank(s), "
                        f"{a.steps} MCMC steps, one all-gather of (best score, best order)",
            "chain_steps_per_s": a.chains * a.steps / wall, "ms_per_step": 1e3 * wall / a.steps,
            "n_ranks": world, "chains_per_rank": len(mine), "backend": backend if world > 1 else None,
            "best_score": float(all_s[g]), "best_chain": g, "n_gathered": int(len(all_s))}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
