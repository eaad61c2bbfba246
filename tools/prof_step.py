"""Profiling target for the fused per-step scorer (nemo_optimal_weights):
a few calls for N chains at C3.   python tools/prof_step.py [--chains 16] [--reps 5]"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--config", default="C3")
    args = ap.parse_args()
    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine
    from nemo.nem_order_mcmc import SIG0, SIG1
    S, E, seed, cap, dtype = generator.CONFIGS[args.config]
    m = generator.config_nem(args.config)
    eng = Engine.for_nem(m, dtype=dtype)
    rng = np.random.default_rng(3)
    n = args.chains
    pos = np.array([rng.permutation(S) for _ in range(n)], dtype=np.int32)
    w = rng.uniform(-3, 3, (n, S, S))
    anc = np.clip(rng.random((n, S, S)) - 0.5, 0, 1)
    eng.optimal_weights(pos, expit(w), anc, w, SIG0, SIG1, cap=cap, raise_on_fail=False)
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        eng.optimal_weights(pos, expit(w), anc, w, SIG0, SIG1, cap=cap, raise_on_fail=False)
        ts.append(time.perf_counter() - t0)
    print(f"chains={n} median {1e3 * np.median(ts):.3f} ms")


if __name__ == "__main__":
    main()
