"""Inter-launch gap of the headline step: wall time per step of K back-to-back
score_dev launches (C3, B = 2048) with the library's per-launch HIP-event
timing on and off, after a 0.5 s warm-up.

    python tools/gap_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from scipy.special import expit  # noqa: E402

from nemo import generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402

m = generator.config_nem("C3")
eng = Engine.for_nem(m)
B, S, K = 2048, m.num_s, 200
eng.reserve(B)
rng = np.random.default_rng(3)
d_pos = torch.from_numpy(np.array([rng.permutation(S) for _ in range(B)], dtype=np.int32)).cuda()
d_w = torch.from_numpy(expit(rng.uniform(-3, 3, (B, S, S)))).cuda()
d_ll = torch.zeros(B, dtype=torch.float64, device="cuda")
side = torch.cuda.Stream()
torch.cuda.set_stream(side)
st = side.cuda_stream


def run(n):
    for _ in range(n):
        eng.score_dev(B, d_pos.data_ptr(), d_w.data_ptr(), d_ll.data_ptr(), stream=st)


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    run(10)
    torch.cuda.synchronize()
for rnd in range(3):
    for timing in (False, True):
        eng.timing(timing)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(K)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / K
        kern = eng.timing_read() if timing else None
        eng.timing(False)
        print(f"round {rnd} timing={timing}: {1e3 * wall:.4f} ms/step"
              + (f", kernel {kern[0] / kern[1]:.4f} ms" if kern else ""), flush=True)
