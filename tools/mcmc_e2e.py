"""End-to-end MCMC throughput: ChainBatch (host state machines + one fused
device call per step) at C3, chain-steps per second, with a cProfile of the
host side.   python tools/mcmc_e2e.py [--chains 16] [--steps 20] [--profile]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=16)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--local-prod", type=int, default=1)
    ap.add_argument("--seed-base", type=int, default=1234)
    ap.add_argument("--on-fail", default="continue", choices=["raise", "continue"])
    a = ap.parse_args()
    from nemo import generator, utils
    from nemo.chains import ChainBatch
    m = generator.config_nem(a.config)
    order = utils.initial_order_guess(m.observed_knockdown_mat)
    cb = ChainBatch(m, [order] * a.chains, seeds=[a.seed_base + c for c in range(a.chains)],
                    on_fail=a.on_fail)
    cb.engine.set_option("local_prod", a.local_prod)
    cb.run(2)  # warm-up
    cb = ChainBatch(m, [order] * a.chains, seeds=[a.seed_base + c for c in range(a.chains)], engine=cb.engine,
                    on_fail=a.on_fail)
    prof = cProfile.Profile() if a.profile else None
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    best, _ = cb.run(a.steps)
    if prof:
        prof.disable()
    dt = time.perf_counter() - t0
    print(f"{a.config}: {a.chains} chains x {a.steps} steps in {dt:.3f} s: "
          f"{1e3 * dt / a.steps:.2f} ms/step, {a.chains * a.steps / dt:.0f} chain-steps/s; best {best.max():.3f}")
    if prof:
        pstats.Stats(prof).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
