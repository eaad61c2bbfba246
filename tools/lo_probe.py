"""What sets the local-optimum kernel's time for one chain: the slowest
problem's serial line search, or the work of all of them?  Builds the 2016
(c, anc, x0) problems of one fused step at C3 on the host (the oracle's
local_c over the order weights of eval #1), then times nemo_local_opt (the
same objective and L-BFGS-B code as the fused step's kernel) on: all 2016,
the slowest alone, 2016 copies of the slowest, 2016 copies of a median one.

    python tools/lo_probe.py      (GPU box; kernel times from HIP events)
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "nem-mcmc-optimization_amd"), os.path.join(HERE, "oracle")]
import numpy as np  # noqa: E402
from scipy.special import expit  # noqa: E402

import nemo_oracle as no  # noqa: E402
from nemo import generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402


def main():
    m = generator.config_nem("C3")
    t = m.get_score_tensor()
    rng = np.random.default_rng(3)
    perm = rng.permutation(64)
    w_raw = rng.uniform(-3, 3, (64, 64))
    w = expit(w_raw)
    ow, _, _ = no.calculate_ll(no.cell_ratios(m.U, t, no.parents_of(perm), w))
    pos = np.argsort(perm)
    cs, x0s = [], []
    for i in range(64):
        for k in range(64):
            if pos[k] < pos[i]:
                cs.append(no.local_c(t[i][k], ow[k], w_raw[i][k]))
                x0s.append(w[i][k])
    c = np.array(cs)
    x0 = np.array(x0s)
    anc = np.clip(rng.random(len(c)) - 0.5, 0, 1)
    eng = Engine(m.U, t)
    xs, fs, nit, nfev, st = eng.local_opt(c, anc, x0)
    slow = int(np.argmax(nfev))
    med = int(np.argsort(nfev)[len(nfev) // 2])
    print(f"problems {len(c)}: nfev mean {nfev.mean():.1f} max {nfev.max()} (#{slow}), median #{med} {nfev[med]}")

    def timed(cc, aa, xx, reps=20):
        eng.local_opt(cc, aa, xx)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            eng.local_opt(cc, aa, xx)
            ts.append(time.perf_counter() - t0)
        return 1e3 * np.median(ts)

    n = len(c)
    print("all", timed(c, anc, x0))
    print("slowest alone", timed(c[slow:slow + 1], anc[slow:slow + 1], x0[slow:slow + 1]))
    print("median alone", timed(c[med:med + 1], anc[med:med + 1], x0[med:med + 1]))
    print("slowest x n", timed(np.repeat(c[slow:slow + 1], n, 0), np.repeat(anc[slow:slow + 1], n), np.repeat(x0[slow:slow + 1], n)))
    print("median x n", timed(np.repeat(c[med:med + 1], n, 0), np.repeat(anc[med:med + 1], n), np.repeat(x0[med:med + 1], n)))


if __name__ == "__main__":
    main()
