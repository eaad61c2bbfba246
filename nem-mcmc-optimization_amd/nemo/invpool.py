"""The per-step host preparation of ``get_optimal_weights`` in worker processes.

Every MCMC step computes, per chain, W~ = expit(W) on the permissible entries
and ancestor_x = clip(inv(I - W~) - I, 0, 1) (nem_order_mcmc.py:98-103,
:185), with scipy's ``expit`` and LAPACK getrf + getri (scipy.linalg.inv).
Those calls hold the GIL or do not run faster from threads on the GPU box
host (tools/lapack_threads.py), so ``InvPool`` spreads a group's chains over
a few spawned worker processes that make the SAME calls (same ufunc, same
library, same lwork; every step is per chain and elementwise or per matrix,
so the split changes no bit: equal to ``chains._prepare``) on shared memory.
A matrix that is not finite or singular is handed back and inverted by
``scipy.linalg.inv`` in the caller, which raises the reference's error.

The workers are plain child processes (spawn: fork + exec of a fresh
interpreter); they never touch the GPU.
"""
from __future__ import annotations

import os

import numpy as np


def default_workers(local_world: int | None = None, cap: int = 8) -> int:
    """Worker processes per rank so that the ranks of one node do not
    oversubscribe its cores: the cores this process may run on, shared by
    the node's ranks (LOCAL_WORLD_SIZE), minus one for the rank itself;
    at least 1, at most ``cap`` (8 measured best for 128 chains on one GPU,
    DESIGN.md 6)."""
    if local_world is None:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    try:
        cores = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cores = os.cpu_count() or 1
    return max(1, min(cap, cores // max(1, local_world) - 1))


def _worker(conn, names, maxb, s):
    from multiprocessing import shared_memory
    from scipy.linalg import get_lapack_funcs
    from scipy.linalg.lapack import _compute_lwork
    from scipy.special import expit

    shms = [shared_memory.SharedMemory(name=nm) for nm in names]
    f8 = [np.ndarray((maxb, s, s), dtype=np.float64, buffer=m.buf) for m in shms[:3]]
    a_all, sig_all, o_all = f8              # input W (or I - W~), W~, output
    m_all = np.ndarray((maxb, s, s), dtype=np.bool_, buffer=shms[3].buf)
    getrf, getri, getri_lwork = get_lapack_funcs(("getrf", "getri", "getri_lwork"), (a_all[0],))
    lwork = int(1.01 * _compute_lwork(getri_lwork, s))
    eye = np.identity(s)
    try:
        while True:
            msg = conn.recv()
            if msg is None:
                break
            kind, lo, hi = msg
            bad = []
            for k in range(lo, hi):
                if kind == "prep":
                    w, mask = a_all[k], m_all[k]
                    sig = w.copy()
                    sig[mask] = expit(w[mask])
                    sig_all[k] = sig
                    a = eye - sig
                else:
                    a = a_all[k]
                if not np.all(np.isfinite(a)):
                    bad.append(k)
                    continue
                lu, piv, info = getrf(a)
                if info == 0:
                    inv, info = getri(lu, piv, lwork=lwork, overwrite_lu=1)
                if info != 0:
                    bad.append(k)
                    continue
                o_all[k] = np.clip(inv - eye, 0, 1) if kind == "prep" else inv
            conn.send(bad)
    finally:
        del a_all, sig_all, o_all, m_all, f8
        for m in shms:
            m.close()


class InvPool:
    """``n_workers`` processes serving up to ``maxb`` S x S matrices per call.

    ``start(mats)`` / ``finish()``: the inverses of ``mats`` (bit-identical to
    ``chains.inv_stack``).  ``start_prepare(ws, masks)`` / ``finish_prepare()``:
    (W~, ancestor_x) of each chain (bit-identical to ``chains._prepare``).
    ``start*`` hands the work out and returns at once."""

    def __init__(self, s: int, maxb: int = 64, n_workers: int = 4):
        import multiprocessing as mp
        from multiprocessing import shared_memory
        self.s, self.maxb = s, maxb
        n = maxb * s * s
        self._shm = [shared_memory.SharedMemory(create=True, size=n * 8) for _ in range(3)]
        self._shm.append(shared_memory.SharedMemory(create=True, size=n))
        self._a, self._sig, self._o = [np.ndarray((maxb, s, s), dtype=np.float64, buffer=m.buf)
                                       for m in self._shm[:3]]
        self._m = np.ndarray((maxb, s, s), dtype=np.bool_, buffer=self._shm[3].buf)
        ctx = mp.get_context("spawn")
        self._conns, self._procs = [], []
        saved = {k: os.environ.get(k) for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS")}
        os.environ["OPENBLAS_NUM_THREADS"] = "1"   # one thread per worker (bits do not depend on it)
        os.environ["OMP_NUM_THREADS"] = "1"
        try:
            for _ in range(n_workers):
                parent, child = ctx.Pipe()
                p = ctx.Process(target=_worker, args=(child, [m.name for m in self._shm], maxb, s),
                                daemon=True)
                p.start()
                child.close()
                self._conns.append(parent)
                self._procs.append(p)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        self._busy = None

    def _send(self, kind, n):
        nw = min(len(self._conns), n)
        bounds = [n * w // nw for w in range(nw + 1)]
        for w in range(nw):
            self._conns[w].send((kind, bounds[w], bounds[w + 1]))
        self._busy = (kind, n, nw)

    def _check(self, n):
        if self._busy is not None:   # a caller that raised between start and finish
            self._drain()
        if n > self.maxb:
            raise ValueError(f"InvPool: {n} matrices > capacity {self.maxb}")

    def start(self, mats):
        n = len(mats)
        self._check(n)
        self._a[:n] = mats
        self._send("inv", n)

    def start_prepare(self, ws, masks):
        n = len(ws)
        self._check(n)
        self._a[:n] = ws
        self._m[:n] = masks
        self._send("prep", n)

    def _drain(self):
        _kind, _n, nw = self._busy
        self._busy = None
        for w in range(nw):
            self._conns[w].recv()

    def _collect(self, kind):
        from scipy.linalg import inv
        k_, n, nw = self._busy
        if k_ != kind:
            raise RuntimeError(f"InvPool: finish of {kind!r} after start of {k_!r}")
        self._busy = None
        bad = []
        for w in range(nw):
            bad += self._conns[w].recv()
        out = np.array(self._o[:n])
        for k in bad:   # scipy's own error (or result) for that matrix
            if kind == "prep":
                eye = np.identity(self.s)
                out[k] = np.clip(inv(eye - self._sig[k]) - eye, 0, 1)
            else:
                out[k] = inv(self._a[k])
        return n, out

    def finish(self):
        return self._collect("inv")[1]

    def finish_prepare(self):
        n, anc = self._collect("prep")
        return np.array(self._sig[:n]), anc

    def close(self):
        for c in self._conns:
            try:
                c.send(None)
            except (BrokenPipeError, OSError):
                pass
        for p in self._procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
        self._conns, self._procs = [], []
        del self._a, self._sig, self._o, self._m
        for m in self._shm:
            m.close()
            m.unlink()
        self._shm = []

    def __del__(self):
        if getattr(self, "_procs", None):
            try:
                self.close()
            except Exception:
                pass

