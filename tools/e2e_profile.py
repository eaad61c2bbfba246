"""cProfile of ChainBatch.run at C3 (16 chains, device ancestor_x, one
group): where the host's share of an MCMC step goes.
    python tools/e2e_profile.py [chains=16] [steps=30] [groups=1]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
from nemo import generator, utils  # noqa: E402
from nemo.chains import ChainBatch  # noqa: E402
from nemo.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    g = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    order = utils.initial_order_guess(m.observed_knockdown_mat)
    seeds = [1234 + c for c in range(n)]
    ChainBatch(m, [order] * n, seeds=seeds, engine=eng, on_fail="continue", groups=g).run(2)
    cb = ChainBatch(m, [order] * n, seeds=seeds, engine=eng, on_fail="continue", groups=g)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    cb.run(steps)
    pr.disable()
    print(f"{1e3 * (time.perf_counter() - t0) / steps:.3f} ms/step (profiled)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
