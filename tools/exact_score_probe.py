"""Batched order scores in the reference's arithmetic (option exact_dev) on
device-resident C3 inputs: ms per call by HIP events on the launch stream at
several batch sizes, and the bits of the first evaluations against the
host-pointer exact path.

    python tools/exact_score_probe.py [B ...]          (default 16 128 2048)"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nem-mcmc-optimization_amd"))


def main():
    import torch
    from scipy.special import expit

    from nemo import generator
    from nemo.engine import Engine
    sizes = [int(a) for a in sys.argv[1:]] or [16, 128, 2048]
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    S, E = m.num_s, m.num_e
    eng.reserve(max(sizes))
    rng = np.random.default_rng(5)
    nb = max(sizes)
    pos = np.array([rng.permutation(S) for _ in range(nb)], dtype=np.int32)
    w01 = expit(rng.uniform(-3, 3, (nb, S, S)))
    d_pos = torch.from_numpy(pos).cuda()
    d_w = torch.from_numpy(w01).cuda()
    d_ll = torch.zeros(nb, dtype=torch.float64, device="cuda")
    side = torch.cuda.Stream()
    torch.cuda.set_stream(side)
    st = side.cuda_stream
    eng.set_option("exact_dev", 1)
    for b in sizes:
        reps = max(3, min(200, int(20000 / b)))
        for _ in range(3):
            eng.score_dev(b, d_pos.data_ptr(), d_w.data_ptr(), d_ll.data_ptr(), stream=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(side)
        for _ in range(reps):
            eng.score_dev(b, d_pos.data_ptr(), d_w.data_ptr(), d_ll.data_ptr(), stream=st)
        e1.record(side)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ms = e0.elapsed_time(e1) / reps
        got = d_ll[:min(b, 8)].cpu().numpy()
        eng.set_option("exact_dev", 0)
        host = eng.score(pos[:len(got)], w01[:len(got)])
        eng.set_option("exact_dev", 1)
        same = np.array_equal(got.view(np.uint64), host.view(np.uint64))
        print(f"B={b} ms_per_call {ms:.4f} evals_per_s {b / (ms / 1e3):.4g} wall_evals_per_s "
              f"{b * reps / wall:.4g} bits_equal_host_exact {same}", flush=True)
        if not same:
            sys.exit(1)
    eng.close()


if __name__ == "__main__":
    main()
