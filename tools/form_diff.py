"""Compare the exact local-optimum forms pair by pair (w_new bits, status,
nit, nfev) on one random C3 step: python tools/form_diff.py [chains] [formA] [formB]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
import numpy as np
from scipy.special import expit

from nemo import generator
from nemo.engine import Engine
from nemo.nem_order_mcmc import SIG0, SIG1

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
fa = int(sys.argv[2]) if len(sys.argv) > 2 else 1
fb = int(sys.argv[3]) if len(sys.argv) > 3 else 5
S = int(os.environ.get("S", 64))
E = int(os.environ.get("E", 2000))
m = generator.synthetic_nem(S, E, 0)
eng = Engine.for_nem(m)
rng = np.random.default_rng(4)
pos = np.array([rng.permutation(S) for _ in range(n)], dtype=np.int32)
w = rng.uniform(-3, 3, (n, S, S))
anc = np.clip(rng.random((n, S, S)) - 0.5, 0, 1)
if os.environ.get("DUAL_DBG"):
    eng.set_option("exact_dual_dbg", int(os.environ["DUAL_DBG"]))
out = {}
for f in (fa, fb):
    eng.set_option("exact_form", f)
    out[f] = [np.array(x, copy=True) for x in eng.optimal_weights(pos, expit(w), anc, w, SIG0, SIG1, raise_on_fail=False)]
(wa, l1a, lda, ia), (wb, l1b, ldb, ib) = out[fa], out[fb]
mask = ia != -1
print("pairs", mask.sum(), "ll1 equal", np.array_equal(l1a, l1b), "lld equal", np.array_equal(lda, ldb))
dw = (wa.view(np.uint64) != wb.view(np.uint64)) & mask
di = (ia != ib) & mask
print("w_new differ", dw.sum(), "info differ", di.sum())
for b, i, k in list(zip(*np.nonzero(dw | di)))[:12]:
    print(f"  chain {b} pair {i}<-{k}: A w {wa[b, i, k]!r} st {ia[b, i, k] & 15} nit {(ia[b, i, k] >> 4) & 4095} nfev {ia[b, i, k] >> 16}"
          f" | B w {wb[b, i, k]!r} st {ib[b, i, k] & 15} nit {(ib[b, i, k] >> 4) & 4095} nfev {ib[b, i, k] >> 16}")
