"""ll bits of two builds of the library on the same random inputs (run once
per build: python tools/ab_bits_libs.py <out.npy>; NEMO_LIBRARY picks the
build), for changes that must not move a bit."""
import sys
sys.path.insert(0, "nem-mcmc-optimization_amd")
import numpy as np  # noqa: E402
from scipy.special import expit  # noqa: E402

from nemo import generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402

out = []
for cfg, fks in (("C3", (0, 8, 7, 13, 16)), ("C2", (0, 8))):
    m = generator.config_nem(cfg)
    eng = Engine.for_nem(m)
    S = m.num_s
    rng = np.random.default_rng(11)
    pos = np.array([rng.permutation(S) for _ in range(257)], dtype=np.int32)
    w = expit(rng.uniform(-3, 3, (257, S, S)))
    for fk in fks:
        eng.set_option("fact_kernel", fk)
        out.append(eng.score(pos, w))
    eng.close()
np.save(sys.argv[1], np.concatenate(out))
