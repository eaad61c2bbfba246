"""Benchmark: order-score evaluations/s on the synthetic 64 S-gene x 2000
effect NEM (BASELINE.json metric, config C3; C4 = the same per GPU at N > 1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--group G]

A step is one batched pass of the hot path over B (pos, W) evaluations whose
inputs are already resident in HBM: prep (parent lists) + score kernel +
finalize, enqueued on torch's current stream through the C-ABI.  With N > 1
(torchrun, one rank per GPU) every rank evaluates its own B evaluations of
its own chains (weak scaling, no data-path collective); the only collective
is one RCCL all-gather of per-chain best scores at the end of the timed
region (C4).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def algorithmic_bytes_per_eval(S, E, cap, b):
    """P*E*b (table rows) + (S+1)*E*b (U) + S^2*b (W) + 4S (pos) + b (ll)."""
    P = sum(min(q, cap) if cap else q for q in range(S))
    return P * E * b + (S + 1) * E * b + S * S * b + 4 * S + b


def cpu_baseline(m, seconds=10.0):
    """The oracle (numpy restatement of the reference's compute_cell_ratios +
    calculate_ll, nem_order_mcmc.py:79-93) timed on this host, 1 thread."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import nemo_oracle as no
    from scipy.special import expit
    t = m.get_score_tensor()
    rng = np.random.default_rng(77)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        perm = rng.permutation(m.num_s)
        w01 = expit(rng.uniform(-3, 3, (m.num_s, m.num_s)))
        no.order_score(m.U, t, perm, w01)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": f"{n} order-score evals of the 64x2000 C3 model in {dt:.1f} s, "
                      "oracle numpy loop form (reference operation order), OMP_NUM_THREADS=1"}


def load_traffic(workload):
    p = os.path.join(HERE, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        d = json.load(fh)
    return d.get(workload)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("NEMO_BENCH_BATCH", 128)))
    ap.add_argument("--group", type=int, default=int(os.environ.get("NEMO_BENCH_GROUP", 1)))
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine

    S, E, seed, cap, dtype = generator.CONFIGS[args.config]
    m = generator.config_nem(args.config)
    eng = Engine.for_nem(m, device=local, dtype=dtype)
    B = args.batch
    eng.reserve(B)
    rng = np.random.default_rng(1000 + rank)
    pos = np.array([rng.permutation(S) for _ in range(B)], dtype=np.int32)
    w01 = expit(rng.uniform(-3, 3, (B, S, S)))
    d_pos = torch.from_numpy(pos).cuda()
    d_w01 = torch.from_numpy(w01).cuda()
    d_ll = torch.zeros(B, dtype=torch.float64, device="cuda")
    side = torch.cuda.Stream()          # the stream every kernel is launched on
    torch.cuda.set_stream(side)
    stream = side.cuda_stream

    def step():
        eng.score_dev(B, d_pos.data_ptr(), d_w01.data_ptr(), d_ll.data_ptr(), cap=cap,
                      stream=stream, group=args.group)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.timing(True)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(side)
    for _ in range(args.steps):
        step()
    if world > 1:
        # C4: gather every chain's best score (tiny, latency-bound)
        best = d_ll.max().reshape(1)
        allb = [torch.empty_like(best) for _ in range(world)]
        dist.all_gather(allb, best)
    ev1.record(side)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms, launches = eng.timing_read()
    eng.timing(False)
    t_max = torch.tensor([wall], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    t_max = float(t_max.item())

    # parity spot check of the timed results (outside the timed region)
    ll = d_ll.cpu().numpy()
    sys.path.insert(0, os.path.join(HERE, "oracle"))

    if rank == 0:
        b = 8 if dtype == "f64" else 4
        bpe = algorithmic_bytes_per_eval(S, E, cap, b)
        avg_kernel_s = (kern_ms / max(launches, 1)) / 1e3
        achieved = B * bpe / avg_kernel_s / 1e9
        workload = f"{args.config} synthetic S={S} E={E} cap={cap} {dtype}, batch={B}, group={args.group}"
        rec = {
            "metric": "order-score evals/sec (64 S-genes x 2000 effects); HBM GB/s fraction",
            "value": world * B * args.steps / t_max,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * t_max / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if dtype == "f64" else "f32",
            "data": "synthetic (build-defined generator, SURVEY.md 8(d)); random orders and W~U(-3,3)",
            "config": {"workload": workload, "S": S, "E": E, "cap": cap, "batch_per_gpu": B,
                       "group": args.group, "evals_per_step": world * B,
                       "parallelism": f"chains sharded, {world} GPU(s), RCCL all-gather of best scores"},
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": load_traffic(f"{args.config}:b{B}:g{args.group}"),
                "kernel": "score_kernel" if args.group == 1 else "score_group_kernel",
                "kernel_avg_ms": avg_kernel_s * 1e3,
                "bytes_per_eval": bpe,
            },
            "wall_check_ms_per_step": 1e3 * ev0.elapsed_time(ev1) / args.steps,
            "ll_sample": float(ll[0]),
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(m, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
