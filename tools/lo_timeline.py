"""Timeline of the exact local optima of one fused step (option exact_trace):
when each optimum starts and ends (wall_clock64, 10 ns ticks), how many run at
once, how much of the launch is the tail, and how an optimum's duration
follows its evaluation count.

    python tools/lo_timeline.py [chains=16] [options as NAME=VALUE ...]
"""
import ctypes as C
import os
import sys

import numpy as np
from scipy.special import expit

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
from nemo import _lib, generator  # noqa: E402
from nemo.engine import Engine  # noqa: E402
from nemo.nem_order_mcmc import SIG0, SIG1  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    m = generator.config_nem("C3")
    eng = Engine.for_nem(m)
    for kv in sys.argv[2:]:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    eng.set_option("exact_trace", 1)
    S = 64
    rng = np.random.default_rng(3)
    pos = np.array([rng.permutation(S) for _ in range(n)], dtype=np.int32)
    w = rng.uniform(-3, 3, (n, S, S))
    anc = np.clip(rng.random((n, S, S)) - 0.5, 0, 1)
    for _ in range(3):
        _wn, _l1, _ld, info = eng.optimal_weights(pos, expit(w), anc, w, SIG0, SIG1, raise_on_fail=False)
    lib = _lib.load()
    cnt = C.c_int(0)
    _lib.check(lib.nemo_fetch_exact_trace(eng._ctx, C.byref(cnt), None))
    tr = np.zeros((cnt.value, 4), dtype=np.int64)
    _lib.check(lib.nemo_fetch_exact_trace(eng._ctx, C.byref(cnt), tr.ctypes.data_as(C.c_void_p)))
    # launch order: chain-major; a chain's pairs child-major (node 0..S-1),
    # parents in the order's prefix (the step prep's pair list)
    nfev = []
    for b in range(n):
        perm = np.argsort(pos[b])
        for i in range(S):
            for q in range(pos[b][i]):
                nfev.append((int(info[b, i, perm[q]]) >> 16) & 32767)
    nfev = np.array(nfev)
    assert len(nfev) == len(tr), (len(nfev), len(tr))
    t0 = tr[:, 0].min()
    st, en = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0   # us
    dur = en - st
    span = en.max()
    print(f"chains {n}: {len(tr)} optima, span {span:.1f} us (first start to last end)")
    print(f"  duration us: mean {dur.mean():.1f} median {np.median(dur):.1f} p99 {np.percentile(dur, 99):.1f} "
          f"max {dur.max():.1f}")
    print(f"  nfev: mean {nfev.mean():.2f} median {np.median(nfev):.0f} p99 {np.percentile(nfev, 99):.0f} "
          f"max {nfev.max()}; us per evaluation pair (dur / (nfev/2)): {np.median(dur / np.maximum(nfev / 2, 1)):.2f}")
    edges = np.linspace(0, span, 101)
    active = np.array([np.sum((st < edges[j + 1]) & (en > edges[j])) for j in range(100)])
    peak = active.max()
    print(f"  concurrent optima per 1% of the span (peak {peak}):")
    print("   ", " ".join(str(a) for a in active[::5]))
    half = np.where(active < 0.5 * peak)[0]
    tail = (100 - half[0]) if len(half) and half[0] > 50 else 0
    print(f"  tail below half the peak: the last {tail}% of the span")
    last = np.argsort(en)[-5:]
    for g in last[::-1]:
        print(f"  ends last: optimum {g} start {st[g]:.1f} end {en[g]:.1f} dur {dur[g]:.1f} nfev {nfev[g]}")
    print(f"  work / (peak x span): {dur.sum() / (peak * span):.3f}")
    c = np.corrcoef(nfev, dur)[0, 1]
    print(f"  corr(nfev, duration) {c:.3f}")
    ev = np.maximum(nfev / 2, 1)
    print(f"  shader cycles per evaluation pair: objective {np.median(tr[:, 2] / ev):.0f}, control "
          f"{np.median(tr[:, 3] / ev):.0f} (medians); control share of the optima's cycles "
          f"{tr[:, 3].sum() / max(tr[:, 2].sum() + tr[:, 3].sum(), 1):.3f}")
    print(f"  average concurrent optima (sum of durations / span): {dur.sum() / span:.0f}")


if __name__ == "__main__":
    main()
