"""Host-side profile of ChainBatch with a mock engine (no GPU): the device
step returns immediately with plausible outputs."""
import cProfile, pstats, sys, time
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
import numpy as np
from nemo import generator
from nemo.chains import ChainBatch
from nemo import utils

class Call:
    def __init__(self, pos, w01, anc, w):
        n, s = pos.shape[0], pos.shape[1]
        self.w_new = w.copy(); self.w_new[w01 > 0.6] = 0.7
        self.ll1 = np.full(n, -36500.0); self.lld = -36500.0 + np.random.rand(n) * 50
        self.info = np.zeros((n, s, s), dtype=np.int32)
    def begin(self): pass
    def end(self): pass
    def run(self): pass
    def result(self, raise_on_fail=True): return self.w_new, self.ll1, self.lld, self.info

class Mock:
    S = 64
    def reserve(self, *a): pass
    def bind_optimal_weights(self, pos, w01, anc, w, s0, s1, cap=0): return Call(pos, w01, anc, w)
    def optimal_weights(self, pos, w01, anc, w, s0, s1, cap=0, raise_on_fail=True): return Call(pos, w01, anc, w).result()
    def score(self, pos, w01, cap=0, want_cs=False, want_cells=False, want_ow=False):
        ll = -36500.0 + np.random.rand(len(pos)) * 50
        if want_cells or want_cs or want_ow:
            return {"ll": ll, "cells": np.zeros((len(pos), 65, 2000)), "cs": np.zeros((len(pos), 2000)),
                    "ow": np.zeros((len(pos), 65, 2000))}
        return ll

def main():
    m = generator.config_nem("C3")
    order = utils.initial_order_guess(m.observed_knockdown_mat)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    pool = None
    if len(sys.argv) > 2 and int(sys.argv[2]) > 0:
        from nemo.invpool import InvPool
        pool = InvPool(64, n, int(sys.argv[2]))
    cb = ChainBatch(m, [order] * n, seeds=[1234 + c for c in range(n)], engine=Mock(), on_fail="continue", inv_pool=pool)
    cb.run(2)
    cb = ChainBatch(m, [order] * n, seeds=[1234 + c for c in range(n)], engine=Mock(), on_fail="continue", inv_pool=pool)
    t0 = time.perf_counter()
    pr = cProfile.Profile(); pr.enable()
    cb.run(30)
    pr.disable()
    dt = time.perf_counter() - t0
    print(f"{n} chains: {1e3*dt/30:.3f} ms per step host-only (profiled)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
    if pool: pool.close()

if __name__ == "__main__":
    main()
