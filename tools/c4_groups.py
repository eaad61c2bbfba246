"""C4's 128 chains on one GPU as one ChainBatch with 1..4 chain groups
(nemo/chains.py run_methods' software pipeline): ms per MCMC step, interleaved
repeats, the same chains and seeds as run_c4.

    python tools/c4_groups.py [chains] [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402

from nemo import generator, utils  # noqa: E402
from nemo.chains import ChainBatch  # noqa: E402
from nemo.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    order = utils.initial_order_guess(m.observed_knockdown_mat)
    seeds = [1234 + c for c in range(n)]
    ChainBatch(m, [order] * n, seeds=seeds, engine=eng, on_fail="continue").run(2)
    res = {g: [] for g in (1, 2, 3, 4)}
    for _ in range(3):
        for g in res:
            cb = ChainBatch(m, [order] * n, seeds=seeds, engine=eng, on_fail="continue", groups=g)
            t0 = time.perf_counter()
            cb.run(steps)
            res[g].append(1e3 * (time.perf_counter() - t0) / steps)
    for g, v in res.items():
        print(f"groups {g}: {np.median(v):.3f} ms per step ({n * 1e3 / np.median(v):.0f} chain-steps/s), runs "
              f"{[round(x, 3) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
