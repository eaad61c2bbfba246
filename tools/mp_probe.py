"""Two-part pairwise plans (E > 8192): nemo_local_opt (the generic kernel,
c from the caller) against scipy on random c, and the fused step's weights
against the oracle: python tools/mp_probe.py [E]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import numpy as np

import nemo_oracle as no
from nemo import generator
from nemo.engine import Engine

E = int(sys.argv[1]) if len(sys.argv) > 1 else 9000
m = generator.synthetic_nem(12, E, 3)
eng = Engine.for_nem(m)
print("exact_ok", eng.get_option("exact_ok"))
rng = np.random.default_rng(1)
n = 8
c = rng.uniform(-0.3, 1.5, (n, E))
anc = rng.uniform(0, 0.5, n)
x0 = rng.uniform(-2, 2, n)
xs, fs, nit, nfev, st = eng.local_opt(c, anc, x0)
for k in range(n):
    r = no.local_optimum(c[k], anc[k], x0[k])
    print(k, "x*", xs[k] == r.x[0], xs[k] - r.x[0], "nfev", nfev[k], r.nfev, "f", fs[k] - r.fun)
