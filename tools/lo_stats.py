"""Per-pair L-BFGS-B statistics of one fused step (nit, nfev from the info
field) for n chains at C3: the local-optimum kernel's time is set by its
slowest waves.

    python tools/lo_stats.py [n_chains]      (GPU box)
"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402
from scipy.special import expit  # noqa: E402

from nemo import generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402
from nemo.nem_order_mcmc import SIG0, SIG1  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
m = generator.config_nem("C3")
eng = Engine.for_nem(m)
S = 64
rng = np.random.default_rng(3)
pos = np.array([rng.permutation(S) for _ in range(n)], dtype=np.int32)
w = rng.uniform(-3, 3, (n, S, S))
anc = np.clip(rng.random((n, S, S)) - 0.5, 0, 1)
w_new, ll1, lld, info = eng.optimal_weights(pos, expit(w), anc, w, SIG0, SIG1, raise_on_fail=False)
import hashlib  # noqa: E402
print("sha256(w_new, ll1, lld, info)", hashlib.sha256(b"".join(np.ascontiguousarray(a).tobytes()
                                                         for a in (w_new, ll1, lld, info))).hexdigest()[:16])
inf = info[info != -1]
nit, nfev, st = (inf >> 4) & 4095, (inf >> 16) & 32767, inf & 15
for name, v in (("nit", nit), ("nfev", nfev)):
    q = np.percentile(v, [50, 90, 99, 100])
    print(f"{name}: mean {v.mean():.2f} p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} max {q[3]:.0f}")
print("status counts", np.bincount(st, minlength=4).tolist(), "pairs", inf.size, "sum nfev", int(nfev.sum()))
# repeated launches of the same step for a counter pass (rocprofv3 --pmc)
for _ in range(int(os.environ.get("LO_REPEAT", "0"))):
    eng.optimal_weights(pos, expit(w), anc, w, SIG0, SIG1, raise_on_fail=False)
