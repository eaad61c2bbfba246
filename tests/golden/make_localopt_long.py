"""localopt_C3_long.npz: scipy's L-BFGS-B (the library call of
nem_order_mcmc.py:167, restated by oracle.nemo_oracle.local_optimum) on the
C3 local optima that run longest -- six steps' worth of (child, parent) pairs
of the synthetic 64 x 2000 model under random weights, kept when nit >= 6
(the reference's own records stop at nit = 5; these reach nit = 11, where the
optimiser's memory of m = 10 pairs is full and the oldest is dropped).

Only the pair indices and scipy's results are stored; the tests rebuild each
c vector from the model (long_cases() below), so the fixture stays small.
python tests/golden/make_localopt_long.py"""
import os
import sys

import numpy as np
from scipy.special import expit

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "nem-mcmc-optimization_amd")]

import nemo_oracle as no  # noqa: E402

SEEDS = tuple(range(100, 106))
MIN_NIT = 6


def step_inputs(m, t, seed):
    """The c / anc / x0 inputs of one step's local optima (oracle
    optimal_weights up to the minimize calls)."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(m.num_s)
    o = no.OracleSampler(m.U, t, perm)
    o.w = rng.uniform(-6, 6, (m.num_s, m.num_s))
    mapped = o._mapped(o.w)
    ow, _, _ = no.calculate_ll(no.cell_ratios(o.u, o.t, o.parents, mapped))
    anc = np.clip(np.linalg.inv(np.identity(o.s) - mapped) - np.identity(o.s), 0, 1)
    pairs = [(i, int(k)) for i in range(o.s) for k in o.parents[i]]
    return o, ow, anc, pairs


def long_cases(path=os.path.join(HERE, "localopt_C3_long.npz")):
    """(c [n][E], anc, x0, and the record) for the stored pairs."""
    from nemo import generator
    z = np.load(path)
    m = generator.synthetic_nem(64, 2000, 0)
    t = m.get_score_tensor()
    cs, ancs, x0s = [], [], []
    for seed in SEEDS:
        sel = np.nonzero(z["seed"] == seed)[0]
        if len(sel) == 0:
            continue
        o, ow, anc, _ = step_inputs(m, t, seed)
        for r in sel:
            i, k = int(z["i"][r]), int(z["k"][r])
            cs.append(no.local_c(o.t[i][k], ow[k], o.w[i][k]))
            ancs.append(anc[i][k])
            x0s.append(expit(o.w[i][k]))
    order = np.concatenate([np.nonzero(z["seed"] == s)[0] for s in SEEDS])
    rec = {f: z[f][order] for f in ("xstar", "fun", "nit", "nfev")}
    return np.array(cs), np.array(ancs), np.array(x0s), rec


def main():
    from nemo import generator
    m = generator.synthetic_nem(64, 2000, 0)
    t = m.get_score_tensor()
    out = {f: [] for f in ("seed", "i", "k", "xstar", "fun", "nit", "nfev")}
    for seed in SEEDS:
        o, ow, anc, pairs = step_inputs(m, t, seed)
        for i, k in pairs:
            c = no.local_c(o.t[i][k], ow[k], o.w[i][k])
            res = no.local_optimum(c, anc[i][k], expit(o.w[i][k]))
            if res.nit >= MIN_NIT:
                for f, v in (("seed", seed), ("i", i), ("k", k), ("xstar", res.x[0]), ("fun", res.fun),
                             ("nit", res.nit), ("nfev", res.nfev)):
                    out[f].append(v)
    arr = {f: np.array(v) for f, v in out.items()}
    np.savez_compressed(os.path.join(HERE, "localopt_C3_long.npz"), **arr)
    print(len(arr["nit"]), "records; nit", np.bincount(arr["nit"]))


if __name__ == "__main__":
    main()
