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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--inv-workers", type=int, default=None,
                    help="InvPool workers per rank (default: the rank's share of the affinity set - 1, <= 8)")
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

    from nemo import generator
    from nemo.chains import run_c4
    from nemo.engine import Engine

    m = generator.config_nem(a.config)
    eng = Engine.for_nem(m, device=local)
    dev = torch.device("cuda", local) if backend == "nccl" and world > 1 else None
    r = run_c4(m, eng, n_chains=a.chains, steps=a.steps, inv_workers=a.inv_workers, device=dev)
    if rank == 0:
        out = {k: v for k, v in r.items() if k not in ("scores", "orders")}
        out["workload"] = (f"C4: {a.chains} chains of the {a.config} model over {world} rank(s), "
                           f"{a.steps} MCMC steps, one all-gather of (best score, best order)")
        out["backend"] = backend if world > 1 else None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
