"""Single-evaluation (B = 1) launches of the score kernels at C3, for a
kernel trace: the fused step's eval #1 (chunked fp64 with order weights), the
same kernel without outputs beyond ll, and eval #2's int8 log2 kernel.

    rocprofv3 --kernel-trace --stats -- python tools/b1_probe.py   (GPU box)
"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402
from scipy.special import expit  # noqa: E402

from nemo import generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402

m = generator.config_nem("C3")
eng = Engine.for_nem(m)
rng = np.random.default_rng(1)
pos = np.array([rng.permutation(64)], dtype=np.int32)
w01 = expit(rng.uniform(-3, 3, (1, 64, 64)))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
for _ in range(n):
    eng.score(pos, w01, want_ow=True)          # chunked fp64 + order weights (eval #1)
eng.set_option("fact_kernel", 1)
for _ in range(n):
    eng.score(pos, w01)                        # chunked fp64, ll only
eng.set_option("fact_kernel", 0)
for _ in range(n):
    eng.score(pos, w01)                        # auto: int8 log2 (eval #2)
print("done")
