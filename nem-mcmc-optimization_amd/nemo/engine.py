"""Python face of the C-ABI: one :class:`Engine` per (model, device).

An Engine owns a ``nemo_ctx``: the staged tables exp(T) and U in HBM plus the
per-batch scratch.  Host-array methods mirror the reference's numerical
routines batch-wise; ``*_dev`` methods take raw device pointers (e.g. from
``torch.Tensor.data_ptr()``) for callers that keep inputs resident in HBM.
"""
from __future__ import annotations

import ctypes as C
import weakref

import numpy as np

from . import _lib
from ._lib import check, f64, i32, ptr

_DTYPES = {"f64": _lib.NEMO_F64, "f32": _lib.NEMO_F32}


class ExactArithmeticWarning(UserWarning):
    """The staged model is outside what the reference-arithmetic kernels
    cover, so the sampler's step runs the fast kernels: log-scores within
    1e-6 of the reference's, not its bits."""


class Engine:
    """Staged model on one GPU.

    ``U`` (S+1, E) and ``T`` (S, S, E) are the reference's node LR table and
    score tables (nem.py:49-64).  ``dtype='f32'`` stores exp(T) and U in fp32
    and runs the per-element products in fp32 (the C5 configuration); logs,
    log-sum-exp and the effect sum stay fp64.
    """

    def __init__(self, U, T, device: int = 0, dtype: str = "f64"):
        U = f64(U)
        T = f64(T)
        if T.ndim != 3 or T.shape[0] != T.shape[1]:
            raise ValueError(f"T must be (S, S, E), got {T.shape}")
        S, _, E = T.shape
        if U.shape != (S + 1, E):
            raise ValueError(f"U must be ({S + 1}, {E}), got {U.shape}")
        self._create(S, E, device, dtype)
        check(_lib.load().nemo_stage_tables(self._ctx, ptr(U), ptr(T)))

    def _create(self, S, E, device, dtype):
        lib = _lib.load()
        self.S, self.E, self.device, self.dtype = S, E, device, dtype
        self._ctx = C.c_void_p()
        check(lib.nemo_ctx_create(device, S, E, _DTYPES[dtype], C.byref(self._ctx)))
        self._fin = weakref.finalize(self, lib.nemo_ctx_destroy, self._ctx)

    @classmethod
    def from_knockdown(cls, D, A, B, device: int = 0, dtype: str = "f64") -> "Engine":
        """The model built on the GPU from the observed knockdown matrix D
        (S, E) with entries 0/1 and the NEM's A, B (nem.py:17-18, 25-64):
        the same staged tables as ``Engine(U, T)`` with the reference's U and
        T, without the S*S*E host table."""
        D = np.asarray(D)
        if D.ndim != 2:
            raise ValueError(f"D must be (S, E), got {D.shape}")
        if not np.isin(D, (0, 1)).all():
            raise ValueError("D must hold only 0 and 1")
        d8 = np.ascontiguousarray(D, dtype=np.uint8)
        self = cls.__new__(cls)
        self._create(d8.shape[0], d8.shape[1], device, dtype)
        check(_lib.load().nemo_stage_knockdown(self._ctx, d8.ctypes.data_as(_lib._u8p),
                                               float(A), float(B)))
        return self

    # -- cached engines per model -----------------------------------------
    @classmethod
    def for_nem(cls, nem, device: int = 0, dtype: str = "f64") -> "Engine":
        """The model's engine (one per device and dtype), staged from its
        knockdown matrix on the GPU (``from_knockdown``)."""
        cache = nem.__dict__.setdefault("_nemo_engines", {})
        key = (device, dtype)
        eng = cache.get(key)
        if eng is None:
            eng = cls.from_knockdown(nem.observed_knockdown_mat, nem.A, nem.B, device=device,
                                     dtype=dtype)
            cache[key] = eng
        return eng

    @classmethod
    def for_tables(cls, U, score_tables, device: int = 0, dtype: str = "f64") -> "Engine":
        """Engine for the (U, score_tables) pair a caller of methods.py holds:
        the model's cached engine, staged from D, when the tables are a NEM's
        lazy tables and U is its U; else a new engine on the given tables."""
        from .nem import ScoreTables
        if isinstance(score_tables, ScoreTables):
            nem = score_tables._nem
            if score_tables.knockdown_mat is nem.observed_knockdown_mat and np.array_equal(U, nem.U):
                return cls.for_nem(nem, device=device, dtype=dtype)
        return cls(U, np.asarray(score_tables, dtype=np.float64), device=device, dtype=dtype)

    @property
    def handle(self):
        return self._ctx

    def close(self):
        self._fin()

    def reserve(self, max_batch: int, max_chains: int = 0):
        check(_lib.load().nemo_reserve(self._ctx, int(max_batch), int(max_chains)))

    # -- A4 + A5 -----------------------------------------------------------
    def score(self, pos, w01, cap: int = 0, want_cs=False, want_cells=False, want_ow=False):
        """Batched order scores.  pos (B, S) int, w01 (B, S, S) mapped weights.
        Returns ll (B,) or a dict with the requested extras."""
        pos = i32(np.atleast_2d(pos))
        b = pos.shape[0]
        w01 = f64(w01).reshape(b, self.S, self.S)
        ll = np.empty(b)
        cs = np.empty((b, self.E)) if want_cs else None
        cells = np.empty((b, self.S + 1, self.E)) if want_cells else None
        ow = np.empty((b, self.S + 1, self.E)) if want_ow else None
        a = _lib.addr  # plain addresses (~0.4 us each against ~4 for ctypes.data_as)
        check(_lib.load().nemo_score(self._ctx, b, a(pos), a(w01), int(cap), a(ll),
                                     None if cs is None else a(cs), None if cells is None else a(cells),
                                     None if ow is None else a(ow)))
        if not (want_cs or want_cells or want_ow):
            return ll
        return {"ll": ll, "cs": cs, "cells": cells, "ow": ow}

    def score_dev(self, batch, d_pos, d_w01, d_ll, cap=0, stream=None, group=1):
        """Enqueue a batched evaluation on device pointers (no sync)."""
        lib = _lib.load()
        if group == 1:
            check(lib.nemo_score_dev(self._ctx, int(batch), d_pos, d_w01, int(cap), d_ll,
                                     None, None, None, stream))
        else:
            check(lib.nemo_score_group_dev(self._ctx, int(batch), int(group), d_pos, d_w01,
                                           int(cap), d_ll, stream))

    # -- utils.compute_ll / calculate_ll on a given cell matrix ------------
    def lse(self, cells, want_ow=False):
        cells = f64(cells)
        rows = cells.shape[0]
        ll = np.empty(1)
        cs = np.empty(self.E)
        ow = np.empty_like(cells) if want_ow else None
        check(_lib.load().nemo_lse(self._ctx, rows, ptr(cells), ptr(ll), ptr(cs), ptr(ow)))
        return float(ll[0]), cs, ow

    # -- A8 core -------------------------------------------------------------
    def local_opt(self, c, anc, x0):
        c = f64(np.atleast_2d(c))
        n = c.shape[0]
        anc = f64(np.broadcast_to(anc, (n,)))
        x0 = f64(np.broadcast_to(x0, (n,)))
        xs, fs = np.empty(n), np.empty(n)
        nit, nfev, st = (np.empty(n, dtype=np.int32) for _ in range(3))
        check(_lib.load().nemo_local_opt(self._ctx, n, ptr(c), ptr(anc), ptr(x0), ptr(xs), ptr(fs),
                                         ptr(nit, _lib._i32p), ptr(nfev, _lib._i32p),
                                         ptr(st, _lib._i32p)))
        return xs, fs, nit, nfev, st

    # -- A6 fused step -------------------------------------------------------
    def optimal_weights(self, pos, w01, anc, w_prev, sig0, sig1, cap: int = 0, raise_on_fail=True):
        """One get_optimal_weights(init=True, max_iter=1) per chain.

        Returns (w_new, ll1, ll_dag, info): w_new is ``w_prev`` with every
        permissible entry replaced by expit(x*)."""
        call = self.bind_optimal_weights(pos, w01, anc, w_prev, sig0, sig1, cap=cap)
        call.run()
        return call.result(raise_on_fail)

    def bind_optimal_weights(self, pos, w01, anc, w_prev, sig0, sig1, cap: int = 0):
        """``optimal_weights`` in parts: the arguments are converted here;
        ``run()`` is the library call, or ``begin()`` queues it on the library's
        own step thread and ``end()`` waits for it (no Python thread, so no GIL
        hand-over); ``result(raise_on_fail)`` returns what ``optimal_weights``
        returns."""
        return _OptimalWeightsCall(self, pos, w01, anc, w_prev, sig0, sig1, cap)

    @property
    def device_ancestor(self) -> bool:
        """True when the fused step can start from W itself: W~ and
        ancestor_x made on the device in scipy's bits (S <= 64).  The device
        restates scipy's OpenBLAS with its SkylakeX kernels:
        on a host whose scipy selects other kernels, its own inv gives other
        bits, so the sampler inverts on the host there (with a warning)."""
        return self.S <= 64 and host_blas_is_restated()

    def optimal_weights_w(self, pos, w, sig0, sig1, cap: int = 0, raise_on_fail=True, want_prep=True):
        """``optimal_weights`` from the weights themselves: the device makes
        W~ and ancestor_x (nem_order_mcmc.py:98-103, :185) as scipy does.
        Returns (w01, anc, w_new, ll1, ll_dag, info); w01 / anc None with
        ``want_prep=False`` (they stay on the device)."""
        call = self.bind_optimal_weights_w(pos, w, sig0, sig1, cap=cap, want_prep=want_prep)
        call.run()
        try:
            res = call.result(raise_on_fail)
        except AncestorRecompute:
            call.recompute()
            res = call.result(raise_on_fail)
        return (call.w01, call.anc) + res

    def bind_optimal_weights_w(self, pos, w, sig0, sig1, cap: int = 0, want_prep=True):
        """``optimal_weights_w`` in parts, as ``bind_optimal_weights``; the
        call's ``w01`` / ``anc`` hold W~ and ancestor_x once it has ended
        (``want_prep=False``: None, neither leaves the device)."""
        return _OptimalWeightsWCall(self, pos, w, sig0, sig1, cap, want_prep)

    # -- fixed-order optimizers (methods.py) --------------------------------
    def _sweep(self, fn, pos, w, *extra, raise_on_fail=True):
        pos = i32(np.atleast_2d(pos))
        n = pos.shape[0]
        w = f64(w).reshape(n, self.S, self.S)
        w_out = np.empty_like(w)
        ll = np.empty(n)
        info = np.empty((n, self.S, self.S), dtype=np.int32)
        rc = fn(self._ctx, n, ptr(pos, _lib._i32p), ptr(w), *extra, ptr(w_out), ptr(ll),
                ptr(info, _lib._i32p))
        if rc == _lib.NEMO_ERR_OPT and raise_on_fail:
            # the reference raises a plain Exception (methods.py:115, :394)
            raise Exception(_lib.load().nemo_last_error().decode())
        if rc != _lib.NEMO_ERR_OPT:
            check(rc)
        return w_out, ll, info

    def gamma_sweep(self, pos, w, cap: int = 0, raise_on_fail=True):
        """``Method.opt_γ`` (methods.py:397-405) per problem: (w_out, ll, info)."""
        return self._sweep(_lib.load().nemo_gamma_sweep, pos, w, int(cap), raise_on_fail=raise_on_fail)

    def inverse_sweep(self, pos, w, raise_on_fail=True):
        """``InverseMethod.opt_b`` (methods.py:117-129) per problem: (w_out, ll, info)."""
        return self._sweep(_lib.load().nemo_inverse_sweep, pos, w, raise_on_fail=raise_on_fail)

    def inverse_ancestral(self, pos, w):
        """unorder_arr(order, B/(1+B)), B = (I - order_arr(order, exp(w)))^-1 lower
        (methods.py:118-121, :160-164), per problem."""
        pos = i32(np.atleast_2d(pos))
        n = pos.shape[0]
        w = f64(w).reshape(n, self.S, self.S)
        out = np.empty_like(w)
        check(_lib.load().nemo_inverse_ancestral(self._ctx, n, ptr(pos, _lib._i32p), ptr(w), ptr(out)))
        return out

    def order_weights(self, chain: int = 0) -> np.ndarray:
        out = np.empty((self.S + 1, self.E))
        check(_lib.load().nemo_fetch_order_weights(self._ctx, int(chain), ptr(out)))
        return out

    def set_option(self, name: str, value: int):
        check(_lib.load().nemo_set_option(self._ctx, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = C.c_int32(0)
        check(_lib.load().nemo_get_option(self._ctx, name.encode(), C.byref(v)))
        return v.value

    def set_option_f64(self, name: str, value: float):
        check(_lib.load().nemo_set_option_f64(self._ctx, name.encode(), float(value)))

    def get_option_f64(self, name: str) -> float:
        v = C.c_double(0.0)
        check(_lib.load().nemo_get_option_f64(self._ctx, name.encode(), C.byref(v)))
        return v.value

    def score_kernel(self, cap: int = 0, ll_only: bool = True):
        """(fact_kernel, worst-case |ll error| bound) a factored score call
        with this cap takes; fact_kernel -1 = the streaming kernel."""
        fk = C.c_int32(0)
        b = C.c_double(0.0)
        check(_lib.load().nemo_score_kernel(self._ctx, int(cap), 1 if ll_only else 0, C.byref(fk),
                                            C.byref(b)))
        return fk.value, b.value

    def exact_limits(self, cap: int = 0):
        """The reference-arithmetic path's limits for this model
        (``nemo.limits``: one row per limit, the model's value, whether it is
        covered and what the sampler does outside it)."""
        from .limits import exact_limits
        return exact_limits(self.S, self.E, self.factored, cap, host_blas_arch(),
                            exact_option=bool(self.get_option("exact")))

    def exact_status(self, cap: int = 0):
        """(True, "") when the fused step and the sampler's score calls run in
        the reference's own arithmetic (option ``exact``, the default, on a
        model the exact kernels cover); else (False, the limit that breaks it
        and what runs instead) -- the rows of ``exact_limits``."""
        from .limits import exact_status_from
        ok, why = exact_status_from(self.exact_limits(cap))
        # the library's own verdict on the staging (the wave plan it built)
        if ok and not self.get_option("exact_ok"):
            return False, f"E={self.E}: the staging found no wave plan for numpy's pairwise sum; the fast kernels"
        return ok, why

    @property
    def factored(self) -> bool:
        """True when the staged table has the NEM structure the MFMA kernel uses."""
        return bool(self.get_option("factored"))

    # -- timing of the score kernel ------------------------------------------
    def timing(self, enable: bool):
        check(_lib.load().nemo_timing_enable(self._ctx, 1 if enable else 0))

    def timing_read(self):
        ms = C.c_double(0.0)
        n = C.c_int32(0)
        check(_lib.load().nemo_timing_read(self._ctx, C.byref(ms), C.byref(n)))
        return ms.value, n.value


_HOST_BLAS = None


def host_blas_arch():
    """The architecture of the OpenBLAS kernels scipy.linalg runs on this
    host (threadpoolctl), or None when it cannot be told."""
    global _HOST_BLAS
    if _HOST_BLAS is None:
        arch = ""
        try:
            import scipy.linalg  # noqa: F401  (loads its OpenBLAS)
            from threadpoolctl import threadpool_info
            for p in threadpool_info():
                if p.get("internal_api") == "openblas" and "scipy" in p.get("filepath", ""):
                    arch = p.get("architecture") or ""
                    break
        except Exception:  # threadpoolctl absent: cannot tell
            arch = ""
        _HOST_BLAS = arch
    return _HOST_BLAS or None


def host_blas_is_restated() -> bool:
    """True when scipy's OpenBLAS on this host runs the SkylakeX kernels the
    device's getrf / getri restate (csrc/nemo_ancestor.hip), or when the host
    cannot be told (then with a warning: the device's bits are SkylakeX's)."""
    import warnings
    arch = host_blas_arch()
    if arch == "SkylakeX":
        return True
    if arch is None:
        warnings.warn("cannot tell which OpenBLAS kernels scipy runs on this host (threadpoolctl): the device's "
                      "ancestor_x has the bits of scipy's SkylakeX kernels", ExactArithmeticWarning, stacklevel=3)
        return True
    warnings.warn(f"scipy's OpenBLAS runs {arch} kernels on this host, not the SkylakeX kernels the device's "
                  "ancestor_x restates: ancestor_x is made on the host (scipy.linalg.inv)",
                  ExactArithmeticWarning, stacklevel=3)
    return False


_LSE_ENGINES = {}


def lse_ll(cells: np.ndarray, device: int = 0) -> float:
    """sum_e logsumexp over rows, on the GPU (utils.compute_ll)."""
    cells = f64(cells)
    rows, e = cells.shape
    eng = _LSE_ENGINES.get((e, device))
    if eng is None:
        eng = _LseEngine(e, device)
        _LSE_ENGINES[(e, device)] = eng
    return eng.ll(cells)


class _LseEngine:
    """A table-less context used only for the LSE kernel."""

    def __init__(self, E, device):
        lib = _lib.load()
        self.E = E
        self._ctx = C.c_void_p()
        check(lib.nemo_ctx_create(device, 2, E, _lib.NEMO_F64, C.byref(self._ctx)))
        self._fin = weakref.finalize(self, lib.nemo_ctx_destroy, self._ctx)

    def ll(self, cells, want=False):
        rows = cells.shape[0]
        ll = np.empty(1)
        cs = np.empty(self.E)
        ow = np.empty_like(cells) if want else None
        check(_lib.load().nemo_lse(self._ctx, rows, ptr(cells), ptr(ll), ptr(cs), ptr(ow)))
        if want:
            return float(ll[0]), cs, ow
        return float(ll[0])


def lse_full(cells: np.ndarray, device: int = 0):
    """(ll, cs, order_weights) of a given cell matrix, on the GPU."""
    cells = f64(cells)
    e = cells.shape[1]
    eng = _LSE_ENGINES.get((e, device))
    if eng is None:
        eng = _LseEngine(e, device)
        _LSE_ENGINES[(e, device)] = eng
    return eng.ll(cells, want=True)


class _OptimalWeightsCall:
    __slots__ = ("w_new", "ll1", "lld", "info", "_keep", "_fn", "_args", "rc")

    def __init__(self, eng: Engine, pos, w01, anc, w_prev, sig0, sig1, cap):
        pos = i32(np.atleast_2d(pos))
        n, s = pos.shape[0], eng.S
        w01 = f64(w01).reshape(n, s, s)
        anc = f64(anc).reshape(n, s, s)
        self.w_new = np.array(w_prev, dtype=np.float64, copy=True).reshape(n, s, s)
        self.ll1, self.lld = np.empty(n), np.empty(n)
        self.info = np.empty((n, s, s), dtype=np.int32)
        self._keep = (pos, w01, anc)
        self._fn = _lib.load().nemo_optimal_weights
        # (the arrays stay referenced by this object for the call's lifetime)
        a = _lib.addr
        self._args = (eng._ctx, n, a(pos), a(w01), a(anc), float(sig0), float(sig1),
                      int(cap), a(self.w_new), a(self.ll1), a(self.lld), a(self.info))
        self.rc = None

    def run(self):
        self.rc = self._fn(*self._args)

    def begin(self):
        """Queue the call on the library's step thread and return at once."""
        check(_lib.load().nemo_optimal_weights_begin(*self._args))

    def end(self):
        """Wait for the oldest queued call (this one, when begun and ended in order)."""
        self.rc = _lib.load().nemo_optimal_weights_end(self._args[0])

    def result(self, raise_on_fail=True):
        rc = self.rc
        if rc == _lib.NEMO_ERR_OPT and not raise_on_fail:
            return self.w_new, self.ll1, self.lld, self.info
        if rc == _lib.NEMO_ERR_OPT:
            # the reference raises a plain Exception (nem_order_mcmc.py:168-169)
            raise Exception(_lib.load().nemo_last_error().decode())
        check(rc)
        return self.w_new, self.ll1, self.lld, self.info


class AncestorRecompute(_lib.NemoError):
    """The device's ancestor_x met a non-finite intermediate value, where its
    restatement is not held to scipy's bits: the step is to be recomputed with
    the host's W~ / ancestor_x (``_OptimalWeightsWCall.recompute``)."""


class _OptimalWeightsWCall:
    """``nemo_optimal_weights_w``: W in; W~, ancestor_x and the step out."""
    __slots__ = ("eng", "pos", "w", "w01", "anc", "flag", "w_new", "ll1", "lld", "info", "cap", "sig",
                 "_args", "rc", "ended")

    def __init__(self, eng: Engine, pos, w, sig0, sig1, cap, want_prep=True):
        self.eng = eng
        self.pos = i32(np.atleast_2d(pos))
        n, s = self.pos.shape[0], eng.S
        self.w = f64(w).reshape(n, s, s)
        self.w_new = np.array(self.w, copy=True)
        self.w01, self.anc = (np.empty((n, s, s)), np.empty((n, s, s))) if want_prep else (None, None)
        self.flag = np.zeros(n, dtype=np.int32)
        self.ll1, self.lld = np.empty(n), np.empty(n)
        self.info = np.empty((n, s, s), dtype=np.int32)
        self.cap, self.sig = int(cap), (float(sig0), float(sig1))
        a = _lib.addr
        self._args = (eng._ctx, n, a(self.pos), a(self.w), float(sig0), float(sig1), int(cap),
                      None if self.w01 is None else a(self.w01), None if self.anc is None else a(self.anc),
                      a(self.w_new), a(self.ll1), a(self.lld), a(self.info), a(self.flag))
        self.rc, self.ended = None, False

    def run(self):
        self.rc = _lib.load().nemo_optimal_weights_w(*self._args)
        self.ended = True

    def begin(self):
        check(_lib.load().nemo_optimal_weights_w_begin(*self._args))

    def end(self):
        if not self.ended:
            self.rc = _lib.load().nemo_optimal_weights_end(self._args[0])
            self.ended = True

    def recompute(self):
        """The step again with W~ and ancestor_x made on the host (scipy's
        expit and inv: chains.inv_stack), synchronously -- no other call may
        be queued on the engine."""
        from .chains import inv_stack
        sig = self.host_w01()
        eye = np.identity(self.eng.S)
        self.w01 = sig
        self.anc = np.clip(inv_stack(eye - sig) - eye, 0, 1)
        self.flag[:] = 0
        call = _OptimalWeightsCall(self.eng, self.pos, self.w01, self.anc, self.w, *self.sig, self.cap)
        call.run()
        self.w_new, self.ll1, self.lld, self.info, self.rc = call.w_new, call.ll1, call.lld, call.info, call.rc

    def host_w01(self):
        """W~ as the host makes it (scipy's expit on the permissible entries)."""
        from scipy.special import expit

        from .nem_order_mcmc import permissible_batch
        mask = permissible_batch(self.pos, self.cap)
        sig = self.w.copy()
        sig[mask] = expit(self.w[mask])
        return sig

    def result(self, raise_on_fail=True):
        if self.rc == _lib.NEMO_ERR_LINALG:
            from scipy.linalg import inv
            eye = np.identity(self.eng.S)
            w01 = self.w01 if self.w01 is not None else self.host_w01()
            for k in np.nonzero(self.flag)[0]:
                if self.flag[k] & 3:   # scipy.linalg.inv's own error (LinAlgError / ValueError)
                    inv(eye - w01[k])
            raise AncestorRecompute(self.rc, _lib.load().nemo_last_error().decode())
        rc = self.rc
        if rc == _lib.NEMO_ERR_OPT and not raise_on_fail:
            return self.w_new, self.ll1, self.lld, self.info
        if rc == _lib.NEMO_ERR_OPT:
            raise Exception(_lib.load().nemo_last_error().decode())
        check(rc)
        return self.w_new, self.ll1, self.lld, self.info
