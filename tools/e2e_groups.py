"""ChainBatch end to end at C3 (16 chains, device ancestor_x) by pipeline
group count and option anc_overlap, ms per MCMC step (median of 3 runs):
    python tools/e2e_groups.py [chains=16] [steps=30]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
from nemo import generator, utils  # noqa: E402
from nemo.chains import ChainBatch  # noqa: E402
from nemo.engine import Engine  # noqa: E402
from nemo.nem_order_mcmc import SIG0, SIG1  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    order = utils.initial_order_guess(m.observed_knockdown_mat)
    seeds = [1234 + c for c in range(n)]
    rng = np.random.default_rng(3)
    pos = np.array([rng.permutation(64) for _ in range(n)], dtype=np.int32)
    w = np.where(pos[:, None, :] < pos[:, :, None], rng.uniform(-3, 3, (n, 64, 64)), 0.0)
    for ov in (1,):
        eng.set_option("anc_overlap", ov)
        eng.optimal_weights_w(pos, w, SIG0, SIG1, raise_on_fail=False)
        ts = []
        for _ in range(10):
            t0 = time.perf_counter()
            eng.optimal_weights_w(pos, w, SIG0, SIG1, raise_on_fail=False)
            ts.append(time.perf_counter() - t0)
        print(f"anc_overlap {ov}: fused step from W {1e3 * np.median(ts):.3f} ms", flush=True)
        for g in (1, 2, 3):
            ChainBatch(m, [order] * n, seeds=seeds, engine=eng, on_fail="continue", groups=g).run(2)
            walls = []
            for _ in range(3):
                cb = ChainBatch(m, [order] * n, seeds=seeds, engine=eng, on_fail="continue", groups=g)
                t0 = time.perf_counter()
                cb.run(steps)
                walls.append(time.perf_counter() - t0)
            print(f"  groups {g}: {1e3 * np.median(walls) / steps:.3f} ms/step", flush=True)
    eng.set_option("anc_overlap", 1)


if __name__ == "__main__":
    main()
