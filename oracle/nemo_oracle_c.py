"""ORACLE -- test infrastructure only.  ctypes binding of the C restatement
(oracle/nemo_oracle_c.c, the CPU twin of the order-score kernels).  Only
``tests/`` and ``bench.py``'s cpu_baseline leg import it; the product path
never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libnemo_oracle_c.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile libnemo_oracle_c.so with gcc (oracle/Makefile)."""
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(
            os.path.join(HERE, "nemo_oracle_c.c")):
        subprocess.run(["make", "-s", "-B", "-C", HERE, "libnemo_oracle_c.so"], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        lib = ctypes.CDLL(build())
        f = lib.nemo_oracle_order_scores
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 5 + [ctypes.c_void_p] * 2
        _lib = lib
    return _lib


def order_scores(u, t, pos, w01, cap: int = 0, threads: int = 1, want_cs: bool = False):
    """ll of each (pos[b], w01[b]) -- and the column log-sum-exps cs when
    ``want_cs`` -- with T as an (S, S, E) array (nemo_oracle.score_tensor)."""
    u = np.ascontiguousarray(u, dtype=np.float64)
    t = np.ascontiguousarray(t, dtype=np.float64)
    pos = np.ascontiguousarray(pos, dtype=np.int32)
    w01 = np.ascontiguousarray(w01, dtype=np.float64)
    s, e = t.shape[0], t.shape[2]
    if u.shape != (s + 1, e) or t.shape != (s, s, e) or pos.ndim != 2 or pos.shape[1] != s \
            or w01.shape != (pos.shape[0], s, s):
        raise ValueError("order_scores: inconsistent shapes")
    n = pos.shape[0]
    ll = np.empty(n)
    cs = np.empty((n, e)) if want_cs else None
    rc = load().nemo_oracle_order_scores(
        u.ctypes.data, t.ctypes.data, pos.ctypes.data, w01.ctypes.data, s, e, n, cap, threads,
        ll.ctypes.data, cs.ctypes.data if want_cs else None)
    if rc != 0:
        raise ValueError("nemo_oracle_order_scores: bad argument (a pos row is not a permutation?)")
    return (ll, cs) if want_cs else ll
