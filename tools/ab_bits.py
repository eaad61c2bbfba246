"""Bits of fact_kernel variants that must agree exactly with the default on
random C3 inputs (python tools/ab_bits.py [fk ...]); odd batch sizes, so
the tail tiles and the block split are exercised."""
import sys
sys.path.insert(0, "nem-mcmc-optimization_amd")
import numpy as np  # noqa: E402
from scipy.special import expit  # noqa: E402

from nemo import generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402

fks = [int(v) for v in sys.argv[1:]] or [10, 14, 16]
for cfg in ("C3", "C2"):
    m = generator.config_nem(cfg)
    eng = Engine.for_nem(m)
    S = m.num_s
    rng = np.random.default_rng(1)
    for B in (1, 7, 300):
        pos = np.array([rng.permutation(S) for _ in range(B)], dtype=np.int32)
        w = expit(rng.uniform(-3, 3, (B, S, S)))
        eng.set_option("fact_kernel", 0)
        ref = eng.score(pos, w)
        for fk in fks:
            eng.set_option("fact_kernel", fk)
            out = eng.score(pos, w)
            print(cfg, "B", B, "fk", fk, "bits equal to auto:", bool(np.array_equal(out, ref)))
    eng.close()
