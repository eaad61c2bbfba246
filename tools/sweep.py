"""Interleaved A/B sweep of score-kernel variants in ONE process
(cdna_hip_programming.md 5.4 rule 24): N rounds x every variant, median and
min of the per-launch kernel time from the library's HIP-event timing.

    python tools/sweep.py [--rounds 5] [--steps 20]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--configs", default="C3,C5")
    ap.add_argument("--batches", default="32,128,512")
    ap.add_argument("--fks", default="1,2,4,6,7,8")
    ap.add_argument("--out", default=os.path.join(HERE, "gpurun_out", "sweep.json"))
    ap.add_argument("--no-fused", action="store_true", help="skip the fused-step timings")
    ap.add_argument("--no-stream", action="store_true", help="skip the streaming-kernel variants")
    args = ap.parse_args()
    import torch
    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine

    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    results = {}
    for cfg in args.configs.split(","):
        S, E, seed, cap, dtype = generator.CONFIGS[cfg]
        m = generator.config_nem(cfg)
        eng = Engine.for_nem(m, dtype=dtype)
        # (batch, group, xcd_remap, path): path 1 = stream, 2 + 10 * fact_kernel = factored
        variants = []
        for batch in [int(v) for v in args.batches.split(",")]:
            for group in (() if args.no_stream else ((1, 8) if cap == 0 else (1,))):
                variants.append((batch, group, 1, 1))
            for fk in [int(v) for v in args.fks.split(",")]:  # 1 chunked, 2 f64 pipelined, 4/6 int8 x4/x8 waves, 7/8 offset int8 x4/x8
                variants.append((batch, 1, 1, 2 + 10 * fk))
        maxb = max(v[0] for v in variants)
        eng.reserve(maxb)
        rng = np.random.default_rng(5)
        pos = torch.from_numpy(np.array([rng.permutation(S) for _ in range(maxb)], dtype=np.int32)).cuda()
        w01 = torch.from_numpy(expit(rng.uniform(-3, 3, (maxb, S, S)))).cuda()
        ll = torch.zeros(maxb, dtype=torch.float64, device="cuda")
        times = {v: [] for v in variants}
        with torch.cuda.stream(stream):
            st = stream.cuda_stream
            for v in variants:  # warm-up / first-use allocations
                batch, group, remap, path = v
                eng.set_option("xcd_remap", remap)
                eng.set_option("score_path", path % 10)
                eng.set_option("fact_kernel", path // 10)
                eng.score_dev(batch, pos.data_ptr(), w01.data_ptr(), ll.data_ptr(), cap=cap, stream=st, group=group)
            torch.cuda.synchronize()
            for _ in range(args.rounds):
                for v in variants:
                    batch, group, remap, path = v
                    eng.set_option("xcd_remap", remap)
                    eng.set_option("score_path", path % 10)
                    eng.set_option("fact_kernel", path // 10)
                    eng.timing(True)
                    for _ in range(args.steps):
                        eng.score_dev(batch, pos.data_ptr(), w01.data_ptr(), ll.data_ptr(), cap=cap,
                                      stream=st, group=group)
                    torch.cuda.synchronize()
                    ms, n = eng.timing_read()
                    eng.timing(False)
                    times[v].append(ms / n)
        for v, ts in times.items():
            batch, group, remap, path = v
            med = float(np.median(ts))
            name = f"factored fk={path // 10}" if path % 10 == 2 else "stream"
            results[f"{cfg} b={batch} g={group} remap={remap} path={name}"] = {
                "median_ms": med, "min_ms": float(np.min(ts)),
                "evals_per_s_kernel": batch / (med / 1e3)}
        eng.set_option("score_path", 0)
        eng.set_option("fact_kernel", 0)
        eng.set_option("xcd_remap", 1)
        # fused per-step scorer (eval #1 + local optima + eval #2)
        from nemo.nem_order_mcmc import SIG0, SIG1
        for nch in (() if args.no_fused else (1, 16)):
            pos_h = np.array([rng.permutation(S) for _ in range(nch)], dtype=np.int32)
            w_h = rng.uniform(-3, 3, (nch, S, S))
            anc = np.clip(rng.random((nch, S, S)) - 0.5, 0, 1)
            eng.optimal_weights(pos_h, expit(w_h), anc, w_h, SIG0, SIG1, cap=cap, raise_on_fail=False)
            ts = []
            for _ in range(args.rounds):
                t0 = time.perf_counter()
                eng.optimal_weights(pos_h, expit(w_h), anc, w_h, SIG0, SIG1, cap=cap, raise_on_fail=False)
                ts.append(time.perf_counter() - t0)
            results[f"{cfg} fused_step chains={nch}"] = {"median_ms": 1e3 * float(np.median(ts)),
                                                         "min_ms": 1e3 * float(np.min(ts))}
        eng.close()
        del m
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(results, fh, indent=1)
    for k, v in results.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()
