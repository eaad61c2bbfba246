"""Benchmark: order-score evaluations/s on the synthetic 64 S-gene x 2000
effect NEM (BASELINE.json metric, config C3; C4 = the same per GPU at N > 1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--path auto|stream|factored]

A step is one batched pass of the hot path over B = 2048 (pos, W)
evaluations whose inputs are already resident in HBM, enqueued on one HIP
stream through the C-ABI: for the default path (the staged C3 model has the
NEM structure) that is ONE kernel, score_i8l_kernel: per evaluation the
fixed-point digits of Delta in LDS, the int8 MFMA contraction and the fp64
log-sum-exp, with the effect sum finalized in-kernel.
With N > 1 (torchrun, one rank per GPU) every rank evaluates its own B
evaluations (weak scaling, no data-path collective); the only collective is
one RCCL all-gather of per-chain best scores at the end of the timed region
(C4).  Rank 0 prints one JSON line.
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

HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
F64_MFMA_PEAK_TF = 78.6  # v_mfma_f64_16x16x4_f64: 2048 FLOP / 64 busy cycles / SIMD (PMC-checked)
I8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA (MI355X_MICROARCH.md: 2x the ~2.5 PF BF16 rate)
PATHS = {"auto": 0, "stream": 1, "factored": 2}


def n_pairs(S, cap):
    return sum(min(q, cap) if cap else q for q in range(S))


def algorithmic_bytes_per_eval(S, E, cap, b):
    """P*E*b (table rows) + (S+1)*E*b (U) + S^2*b (W) + 4S (pos) + b (ll)."""
    return n_pairs(S, cap) * E * b + (S + 1) * E * b + S * S * b + 4 * S + b


def algorithmic_flops_per_eval(S, E, cap):
    """Factored form: cell = U + G + Delta.D1 over the permissible (i, j):
    2 FLOP per (pair, effect)."""
    return 2 * n_pairs(S, cap) * E


def cpu_baseline(m, seconds=10.0, config="C3"):
    """The oracle (numpy restatement of the reference's compute_cell_ratios +
    calculate_ll, nem_order_mcmc.py:79-93, same operation order) timed on
    this host, one thread."""
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
            "sample": f"{n} order-score evals of the {m.num_s}x{m.num_e} {config} model in {dt:.1f} s: oracle numpy "
                      "loop form (reference operation order), one thread, this host"}


_CPU_CHILD = r"""
import sys, time
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import nemo_oracle as no
from scipy.special import expit
from nemo import generator
m = generator.config_nem(sys.argv[3]); t = m.get_score_tensor()
rng = np.random.default_rng(int(sys.argv[5]))
sys.stdout.write("ready\n"); sys.stdout.flush()
sys.stdin.readline()
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < float(sys.argv[4]):
    no.order_score(m.U, t, rng.permutation(m.num_s), expit(rng.uniform(-3, 3, (m.num_s, m.num_s))))
    n += 1
print(n, time.perf_counter() - t0)
"""


def cpu_baseline_procs(config, nproc=8, seconds=10.0):
    """the same oracle loop in nproc independent processes
    (one thread each, independent chains), started together; the rate is the
    sum of the processes' own rates.  Children are plain subprocesses that
    never touch the GPU."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    args = [os.path.join(HERE, "oracle"), os.path.join(HERE, "nem-mcmc-optimization_amd"), config, str(seconds)]
    procs = [subprocess.Popen([sys.executable, "-c", _CPU_CHILD] + args + [str(100 + k)], stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, text=True, env=env) for k in range(nproc)]
    try:
        for p in procs:  # every child has built its model before any starts timing
            if p.stdout.readline().strip() != "ready":
                raise RuntimeError("cpu baseline child failed to start")
        for p in procs:
            p.stdin.write("go\n")
            p.stdin.flush()
        res = [p.communicate(timeout=seconds + 120)[0].split() for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    rates = [int(n) / float(dt) for n, dt in res]
    n = sum(int(r[0]) for r in res)
    return {"value": sum(rates), "unit": "evals/s", "cores": nproc, "kind": "port",
            "sample": f"{n} order-score evals of the {config} model by {nproc} independent one-thread "
                      f"processes in ~{seconds:.0f} s each: oracle numpy loop form (reference operation "
                      "order), this host"}


def load_valu_bound(key):
    """PMC-derived VALU utilisation of the score kernel (profiles/valu.json,
    tools/make_valu.py): VALU-busy cycles over SIMD cycles."""
    p = os.path.join(HERE, "profiles", "valu.json")
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        return json.load(fh).get(key)


def load_traffic(key):
    p = os.path.join(HERE, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        return json.load(fh).get(key)


def timed_steps(eng, torch, B, cap, steps, warmup, d_pos, d_w01, d_ll, stream, world, dist,
                warmup_s=0.0):
    def step():
        eng.score_dev(B, d_pos.data_ptr(), d_w01.data_ptr(), d_ll.data_ptr(), cap=cap, stream=stream)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # the engine clock ramps up over the first tens of ms of load (a 20-step
    # run measures ~10% slower per launch than a 200-step one): untimed steps
    # until warmup_s of load have passed, so the K timed steps see the
    # sustained clock whatever W is
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warmup_s:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # kernel time = HIP events recorded on the launch stream around the K
    # back-to-back launches, divided by K (an upper bound on the kernel's own
    # duration: it includes any gap between launches).  The library's
    # per-launch events would add ~6 us of stream work per step inside the
    # timed region, so they run after it, on 20 more launches, as a cross-check
    ts = torch.cuda.current_stream()  # the stream every kernel is launched on
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(ts)
    for _ in range(steps):
        step()
    ev1.record(ts)
    if world > 1:
        # C4: gather every rank's per-chain best score (tiny, latency-bound)
        best = d_ll.max().reshape(1)
        if dist.get_backend() != "nccl":
            best = best.cpu()
        allb = [torch.empty_like(best) for _ in range(world)]
        dist.all_gather(allb, best)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps
    eng.timing(True)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    lt_ms, launches = eng.timing_read()
    eng.timing(False)
    return wall, kern_ms, lt_ms / max(launches, 1)


def c5_capped(torch, dist, stream, batch=2048, steps=10, warmup_s=0.3):
    """BASELINE config C5 (S=128, E=5000, parent cap 6): evals/s of the capped
    lookup-table kernel (fact_kernel 9, what auto takes for capped calls), of
    its round-1 form (fact_kernel 15) and of the fp64 MFMA factored kernel
    (fact_kernel 1) on the same resident inputs; kernel time per launch from
    the library's HIP events."""
    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine
    S, E, _seed, cap, dtype = generator.CONFIGS["C5"]
    eng = Engine.for_nem(generator.config_nem("C5"), dtype=dtype)
    eng.reserve(batch)
    rng = np.random.default_rng(78)
    d_pos = torch.from_numpy(np.array([rng.permutation(S) for _ in range(batch)], dtype=np.int32)).cuda()
    d_w01 = torch.from_numpy(expit(rng.uniform(-3, 3, (batch, S, S)))).cuda()
    d_ll = torch.zeros(batch, dtype=torch.float64, device="cuda")
    staged = bool(eng.get_option("win"))
    out = {"workload": f"C5: S={S} E={E} cap={cap} {dtype} tables, {batch} evaluations per launch",
           "lookup_table_staged": staged}
    lls = {}
    runs = ((("lookup_table_kernel", 9), ("lookup_table_kernel_r1", 15)) if staged else ()) + \
        (("f64_mfma_factored_kernel", 1),)
    for name, fk in runs:
        eng.set_option("fact_kernel", fk)
        wall, kms, _ = timed_steps(eng, torch, batch, cap, steps, 2, d_pos, d_w01, d_ll, stream, 1, dist,
                                   warmup_s=warmup_s)
        lls[name] = d_ll.cpu().numpy()
        out[name] = {"evals_per_s": batch * steps / wall, "kernel_avg_ms": kms,
                     "cells_per_s": batch * S * E / (kms / 1e3)}
    if staged:
        out["lookup_table_kernel"]["kernel"] = (
            "score_window2_kernel (row bits transposed into registers, 7-bit window per row by one "
            "funnel shift; two table reads + one FMA per cell)")
        out["lookup_table_kernel_r1"]["kernel"] = "score_window_kernel (round 1: row bits re-read from LDS)"
        # the walk reads two f64 table entries per cell from LDS: priced
        # against the chip's ds_read_b64 rate (MI355X_MICROARCH.md, LDS table:
        # 256 B/clk/CU, ~150 TB/s with every CU streaming)
        kms = out["lookup_table_kernel"]["kernel_avg_ms"]
        lds_tbs = batch * S * E * 16 / (kms / 1e3) / 1e12
        out["lookup_table_kernel"]["roofline"] = {
            "bound": "lds", "achieved": lds_tbs, "peak": 150.0, "unit": "TB/s", "frac": lds_tbs / 150.0,
            "bytes_per_eval": S * E * 16, "note": "2 x 8 B of LDS reads per cell (S*E cells per evaluation)"}
        out["max_abs_ll_diff"] = float(np.max(np.abs(lls["lookup_table_kernel"] -
                                                     lls["f64_mfma_factored_kernel"])))
        out["max_abs_ll_diff_r1"] = float(np.max(np.abs(lls["lookup_table_kernel"] -
                                                        lls["lookup_table_kernel_r1"])))
    eng.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-seconds", type=float, default=0.5,
                    help="untimed load after the W warmup steps (clock ramp); 0: W steps only")
    ap.add_argument("--batch", type=int, default=int(os.environ.get("NEMO_BENCH_BATCH", 2048)))
    ap.add_argument("--path", default=os.environ.get("NEMO_BENCH_PATH", "auto"), choices=list(PATHS))
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the stream-kernel and MCMC lines")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=8,
                    help="processes of the multi-process CPU baseline (1: off)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NEMO_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on
    # one GPU (device = local rank modulo the visible GPUs); the driver's
    # multi-GPU runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("NEMO_BENCH_BACKEND", "nccl")
    local = local % max(torch.cuda.device_count(), 1) if backend != "nccl" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine

    S, E, seed, cap, dtype = generator.CONFIGS[args.config]
    m = generator.config_nem(args.config)
    eng = Engine.for_nem(m, device=local, dtype=dtype)
    eng.set_option("score_path", PATHS[args.path])
    factored = eng.factored and args.path != "stream"
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

    wall, kern_ms, launch_ev_ms = timed_steps(eng, torch, B, cap, args.steps, args.warmup, d_pos, d_w01,
                                              d_ll, stream, world, dist, warmup_s=args.warmup_seconds)
    t_max = torch.tensor([wall], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    t_max = float(t_max.item())
    ll = d_ll.cpu().numpy()

    extras = {}
    if rank == 0 and not args.no_extras:
        # the generic streaming kernel on the same model (HBM-priced roofline)
        eng.set_option("score_path", 1)
        Bs = min(B, 128)
        w_s, k_s, _ = timed_steps(eng, torch, Bs, cap, 10, 2, d_pos, d_w01, d_ll, stream, 1, dist,
                                  warmup_s=min(args.warmup_seconds, 0.3))
        bpe = algorithmic_bytes_per_eval(S, E, cap, 8 if dtype == "f64" else 4)
        ach = Bs * bpe / (k_s / 1e3) / 1e9
        extras["stream_kernel"] = {
            "evals_per_s": Bs * 10 / w_s, "batch": Bs, "kernel_avg_ms": k_s,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "bytes_per_eval": bpe,
                         "traffic": load_traffic(f"{args.config}:stream:b{Bs}"),
                         "note": "the 65.5 MB exp(T) table is Infinity-Cache resident at C3, so "
                                 "algorithmic bytes exceed HBM bytes (traffic = PMC bytes)"}}
        eng.set_option("score_path", PATHS[args.path])
        # fused per-step scorer of the sampler: 16 chains (C4 share of one GPU)
        from nemo.nem_order_mcmc import SIG0, SIG1
        nch = 16
        pos_h = pos[:nch]
        w_h = rng.uniform(-3, 3, (nch, S, S))
        anc = np.clip(rng.random((nch, S, S)) - 0.5, 0, 1)
        eng.optimal_weights(pos_h, expit(w_h), anc, w_h, SIG0, SIG1, cap=cap, raise_on_fail=False)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            eng.optimal_weights(pos_h, expit(w_h), anc, w_h, SIG0, SIG1, cap=cap, raise_on_fail=False)
            ts.append(time.perf_counter() - t0)
        fs = float(np.median(ts))
        extras["mcmc_fused_step"] = {
            "chains": nch, "ms_per_step": 1e3 * fs, "chain_steps_per_s": nch / fs,
            "includes": "H2D of pos/W/anc, eval#1 with order weights, 2016 L-BFGS-B local optima "
                        "per chain, eval#2 on binarised weights, D2H"}
        # BASELINE C3 names ONE chain: what one chain sees per call -- a
        # synchronous host-pointer order score (B = 1: the calculate_ll path of
        # one sampler, H2D + kernel + D2H) and the fused step of one chain
        lat = []
        for _ in range(50):
            t0 = time.perf_counter()
            eng.score(pos[:1], w01[:1], cap=cap)
            lat.append(time.perf_counter() - t0)
        ts1 = []
        for _ in range(10):
            t0 = time.perf_counter()
            eng.optimal_weights(pos_h[:1], expit(w_h[:1]), anc[:1], w_h[:1], SIG0, SIG1, cap=cap,
                                raise_on_fail=False)
            ts1.append(time.perf_counter() - t0)
        extras["single_chain"] = {
            "score_call_us": 1e6 * float(np.median(lat)), "evals_per_s_sequential": 1.0 / float(np.median(lat)),
            "fused_step_ms": 1e3 * float(np.median(ts1)), "chain_steps_per_s": 1.0 / float(np.median(ts1)),
            "reference_cpu_s_per_chain_step": 1.2,
            "includes": "score_call_us: one synchronous nemo_score call for one (pos, W) from host "
                        "arrays; fused_step_ms: nemo_optimal_weights for one chain (eval#1 with order "
                        "weights, 2016 local optima, eval#2, transfers)"}
        # the whole sampler: 16 chains' host state machines (reference call order,
        # Python random) + one fused device call per step
        from nemo import utils as nutils
        from nemo.chains import ChainBatch
        order0 = nutils.initial_order_guess(m.observed_knockdown_mat)
        seeds = [1234 + c for c in range(nch)]
        from nemo.invpool import InvPool
        pool = InvPool(S, nch, n_workers=4)
        n_it = 20
        e2e = {}
        for tag, pl in (("pool", pool), ("serial", None)):
            ChainBatch(m, [order0] * nch, seeds=seeds, engine=eng, on_fail="continue", inv_pool=pl).run(2)
            cb = ChainBatch(m, [order0] * nch, seeds=seeds, engine=eng, on_fail="continue", inv_pool=pl)
            t0 = time.perf_counter()
            cb.run(n_it)
            e2e[tag] = (time.perf_counter() - t0, cb.best_scores)
        pool.close()
        dt = e2e["pool"][0]
        extras["mcmc_end_to_end"] = {
            "chains": nch, "steps": n_it, "ms_per_step": 1e3 * dt / n_it,
            "chain_steps_per_s": nch * n_it / dt,
            "includes": "ChainBatch.run: proposals, reset quirks, ancestor_x (scipy getrf/getri in 4 "
                        "InvPool worker processes) and accept per chain on the host + the fused device step",
            "ms_per_step_serial_inv": 1e3 * e2e["serial"][0] / n_it,
            "pool_bits_equal_serial": bool(np.array_equal(e2e["pool"][1], e2e["serial"][1])),
            "reference_cpu_s_per_chain_step": 1.2}
        if args.config == "C3":
            # BASELINE config C5 (128 x 5000, parent cap 6): the capped
            # lookup-table kernel next to the fp64 MFMA factored kernel
            extras["c5_capped"] = c5_capped(torch, dist, stream, warmup_s=min(args.warmup_seconds, 0.3))

    if rank == 0:
        if factored:
            fpe = algorithmic_flops_per_eval(S, E, cap)
            ach = B * fpe / (kern_ms / 1e3) / 1e12
            fk = eng.get_option("fact_kernel")
            i8l = S <= 64 and eng.get_option("i8l") > 0 and fk in (0, 10, 11, 12, 13, 14, 16)
            i8o = not i8l and S <= 64 and eng.get_option("i8o") > 0 and fk in (0, 7, 8)
            i8 = S <= 64 and (i8l or i8o or fk in (4, 5, 6))
            kname = ("score_i8l_kernel (x / ln 2 = Delta.D1 + U' + G exact in int8 fixed point on "
                     "v_mfma_i32_16x16x64_i8, 7 digit slices; e^x assembled from the integer "
                     "accumulators + table + degree-2 series; log-sum-exp offset by the null row; "
                     "two 16-effect tiles per iteration share the A fragments)"
                     if i8l else
                     "score_i8o_kernel (Delta.D1 + U - U[S] exact in int8 fixed point on "
                     "v_mfma_i32_16x16x64_i8, fp64 cells, log-sum-exp offset by the null row)" if i8o else
                     "score_i8_kernel (Delta.D1 exact in int8 fixed point on v_mfma_i32_16x16x64_i8, "
                     "fp64 cells + fused log-sum-exp)" if i8 else
                     "score_factored_kernel (fp64 MFMA 16x16x4 + fused log-sum-exp)")
            tkey = "i8l" if i8l else ("i8o" if i8o else ("i8" if i8 else "factored"))
            roof = {"bound": "mfma", "achieved": ach, "peak": F64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                    "frac": ach / F64_MFMA_PEAK_TF,
                    "traffic": load_traffic(f"{args.config}:{tkey}:b{B}"),
                    "kernel": kname, "kernel_avg_ms": kern_ms, "flops_per_eval": fpe,
                    "kernel_avg_ms_launch_events": launch_ev_ms,
                    "note": "achieved = the algorithmic fp64 contraction Delta.D1 over the permissible "
                            "pairs (2*P*E FLOP/eval) per kernel second (kernel_avg_ms: HIP events on the "
                            "launch stream around the K timed launches / K; kernel_avg_ms_launch_events: "
                            "the library's per-launch events on 20 more launches), priced against the dense fp64 "
                            "MFMA peak (the arithmetic type of the path). The int8 kernels compute that "
                            "contraction exactly in fixed point on the int8 matrix cores (score_i8l: 7 "
                            "digit slices, 2^-38 / ln 2 per entry) and assemble e^x from the integer "
                            "accumulators, so they can run faster than an fp64 MFMA contraction: frac "
                            "> 1 means the reformulation beats the fp64 matrix roofline, not a "
                            "measurement artefact. What binds is the SIMD issue of the VALU epilogue "
                            "(S*E exps/eval) beside the MFMAs: valu_bound (PMC, profiles/valu.json; "
                            "DESIGN.md 3.1e)",
                    "valu_bound": load_valu_bound(f"{args.config}:{tkey}:b{B}")}
            if roof["traffic"]:
                # the metric's HBM GB/s fraction: the kernel's PMC HBM bytes per
                # launch (its only HBM stream is the w01 input) over this run's
                # launch time -- far from 8 TB/s: the kernel is not memory-bound
                hbm = roof["traffic"]["bytes_per_launch"] / (kern_ms / 1e3) / 1e9
                roof["hbm_measured"] = {"achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                        "frac": hbm / HBM_PEAK_GBS,
                                        "note": "PMC traffic per launch / HIP-event launch time"}
            if i8l:
                # what the matrix cores actually execute: 7 v_mfma_i32_16x16x64_i8
                # (2*16*16*64 ops each) per 16-child row block per 16-effect tile,
                # against the dense int8 peak (2x BF16 per clock, ~5 POPS)
                ops = ((E + 15) // 16) * (4 if S > 32 else 2 if S > 16 else 1) * 7 * 32768
                roof["int8_mfma_executed"] = {
                    "achieved": B * ops / (kern_ms / 1e3) / 1e12, "peak": I8_MFMA_PEAK_TOPS, "unit": "TOPS",
                    "frac": B * ops / (kern_ms / 1e3) / 1e12 / I8_MFMA_PEAK_TOPS, "ops_per_eval": ops,
                    "note": "the matrix pipe is ~30% busy (PMC mfma_busy, valu_bound); the epilogue VALU issue binds"}
        else:
            bpe = algorithmic_bytes_per_eval(S, E, cap, 8 if dtype == "f64" else 4)
            ach = B * bpe / (kern_ms / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ach / HBM_PEAK_GBS, "traffic": load_traffic(f"{args.config}:stream:b{B}"),
                    "kernel": "score_kernel (streams exp(T) rows)", "kernel_avg_ms": kern_ms,
                    "kernel_avg_ms_launch_events": launch_ev_ms,
                    "bytes_per_eval": bpe}
        path = "factored" if factored else "stream"
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
            "data": "synthetic (build-defined generator, SURVEY.md 8(d)); random orders, W~U(-3,3)",
            "config": {"workload": f"{args.config}: S={S} E={E} cap={cap} {dtype}, {B} order-score "
                                   f"evaluations per step per GPU, {path} kernel",
                       "S": S, "E": E, "cap": cap, "batch_per_gpu": B, "path": path,
                       "parallelism": f"independent evaluations/chains sharded over {world} GPU(s); "
                                      "one RCCL all-gather of best scores"},
            "roofline": roof,
            "ll_sample": float(ll[0]),
        }
        rec.update(extras)
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(m, args.cpu_seconds, args.config)
            if args.cpu_procs > 1:  # also all the host cores the round budget allows
                rec["cpu_baseline_procs"] = cpu_baseline_procs(args.config, args.cpu_procs, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
