"""ctypes binding of ``libnemo.so`` (the C-ABI declared in include/nemo.h).

Loading order matters on ROCm: PyTorch ships its own ``libamdhip64.so`` and
links it by the unversioned name, so when torch is importable it is imported
first and our library (NEEDED libamdhip64.so.7) resolves to the runtime already
in the process instead of pulling in a second copy.

There is no CPU fallback: if the library or a GPU is missing, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_LIB = None
# NEMO_LIBRARY: load another build of the same C-ABI (tools/ablate.sh's
# instrumented variants); the product path is the in-tree libnemo.so
_PATH = os.environ.get("NEMO_LIBRARY") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                       "libnemo.so")

NEMO_F64, NEMO_F32 = 0, 1
NEMO_OK, NEMO_ERR_ARG, NEMO_ERR_HIP, NEMO_ERR_STATE, NEMO_ERR_OPT, NEMO_ERR_LINALG = 0, -1, -2, -3, -5, -6
# per-pair L-BFGS-B status in the low 4 bits of ``info`` (include/nemo.h)
LBFGSB_CONV_PGTOL, LBFGSB_CONV_REL, LBFGSB_ABNORMAL, LBFGSB_MAXITER = 0, 1, 2, 3

_i32p = C.POINTER(C.c_int32)
_f64p = C.POINTER(C.c_double)
_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p

# (name, restype, argtypes) -- one line per symbol of include/nemo.h
SIGNATURES = [
    ("nemo_last_error", C.c_char_p, []),
    ("nemo_version", C.c_int, []),
    ("nemo_build_id", C.c_char_p, []),
    ("nemo_device_count", C.c_int, [_i32p]),
    ("nemo_ctx_create", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_vp)]),
    ("nemo_ctx_destroy", None, [_vp]),
    ("nemo_reserve", C.c_int, [_vp, C.c_int, C.c_int]),
    ("nemo_stage_tables", C.c_int, [_vp, _f64p, _f64p]),
    ("nemo_stage_knockdown", C.c_int, [_vp, _u8p, C.c_double, C.c_double]),
    ("nemo_score", C.c_int, [_vp, C.c_int, _vp, _vp, C.c_int, _vp, _vp, _vp, _vp]),  # addr()
    ("nemo_score_dev", C.c_int, [_vp, C.c_int, _vp, _vp, C.c_int, _vp, _vp, _vp, _vp, _vp]),
    ("nemo_score_group_dev", C.c_int, [_vp, C.c_int, C.c_int, _vp, _vp, C.c_int, _vp, _vp]),
    ("nemo_lse", C.c_int, [_vp, C.c_int, _f64p, _f64p, _f64p, _f64p]),
    ("nemo_local_opt", C.c_int, [_vp, C.c_int, _f64p, _f64p, _f64p, _f64p, _f64p, _i32p, _i32p, _i32p]),
    # the fused step's host buffers go as plain addresses (addr(): ~0.4 us each
    # against ~4 for ndarray.ctypes.data_as; the call is on every MCMC step)
    ("nemo_optimal_weights", C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_double, C.c_double,
                                        C.c_int, _vp, _vp, _vp, _vp]),
    ("nemo_optimal_weights_dev", C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_double, C.c_double,
                                            C.c_int, _vp, _vp, _vp, _vp, _vp]),
    ("nemo_optimal_weights_begin", C.c_int, [_vp, C.c_int, _vp, _vp, _vp, C.c_double, C.c_double,
                                              C.c_int, _vp, _vp, _vp, _vp]),
    ("nemo_optimal_weights_end", C.c_int, [_vp]),
    ("nemo_optimal_weights_w", C.c_int, [_vp, C.c_int, _vp, _vp, C.c_double, C.c_double, C.c_int,
                                          _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("nemo_optimal_weights_w_begin", C.c_int, [_vp, C.c_int, _vp, _vp, C.c_double, C.c_double, C.c_int,
                                                _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("nemo_ancestor_dev", C.c_int, [_vp, C.c_int, _vp, _vp, C.c_int, _vp, _vp, _vp, _vp]),
    ("nemo_fetch_order_weights", C.c_int, [_vp, C.c_int, _f64p]),
    ("nemo_fetch_exact_trace", C.c_int, [_vp, C.POINTER(C.c_int), C.c_void_p]),
    ("nemo_gamma_sweep", C.c_int, [_vp, C.c_int, _i32p, _f64p, C.c_int, _f64p, _f64p, _i32p]),
    ("nemo_inverse_ancestral", C.c_int, [_vp, C.c_int, _i32p, _f64p, _f64p]),
    ("nemo_inverse_sweep", C.c_int, [_vp, C.c_int, _i32p, _f64p, _f64p, _f64p, _i32p]),
    ("nemo_set_option", C.c_int, [_vp, C.c_char_p, C.c_int]),
    ("nemo_get_option", C.c_int, [_vp, C.c_char_p, _i32p]),
    ("nemo_set_option_f64", C.c_int, [_vp, C.c_char_p, C.c_double]),
    ("nemo_get_option_f64", C.c_int, [_vp, C.c_char_p, _f64p]),
    ("nemo_score_kernel", C.c_int, [_vp, C.c_int, C.c_int, _i32p, _f64p]),
    ("nemo_timing_enable", C.c_int, [_vp, C.c_int]),
    ("nemo_timing_read", C.c_int, [_vp, _f64p, _i32p]),
    ("nemo_refmath_probe", C.c_int, [C.c_int, C.c_int, _f64p, _f64p, _f64p]),
]


class NemoError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


def lib_path() -> str:
    return _PATH


def load():
    """Load (once) and return the ctypes library handle."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(_PATH):
        raise NemoError(NEMO_ERR_STATE, f"{_PATH} not built: run `python -m nemo.build` "
                                        "(or __graft_entry__.build()); there is no CPU fallback")
    try:  # share torch's HIP runtime if torch is present (see module docstring)
        import torch  # noqa: F401
    except Exception:
        pass
    lib = C.CDLL(_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int):
    if rc != NEMO_OK:
        msg = load().nemo_last_error().decode(errors="replace")
        raise NemoError(rc, msg)


def f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def ptr(a, kind=_f64p):
    if a is None:
        return None
    return a.ctypes.data_as(kind)


def addr(a: np.ndarray) -> int:
    """Address of a C-contiguous array's data, for c_void_p arguments: a
    writable array through a ctypes buffer view, a read-only one through its
    array interface."""
    if a.flags.writeable:
        return C.addressof(C.c_char.from_buffer(a)) if a.nbytes else a.ctypes.data
    return a.__array_interface__["data"][0]


def build_id() -> str:
    """The loaded library's build id (a hash of its sources and flags)."""
    return load().nemo_build_id().decode()


def device_count() -> int:
    n = C.c_int32(0)
    check(load().nemo_device_count(C.byref(n)))
    return n.value


REFMATH_FNS = {"log": 0, "exp": 1, "expit": 2, "logaddexp": 3, "glibc_exp": 4, "glibc_log1p": 5,
               "sqrt": 6, "div": 7, "log1p_unit": 8}


def refmath_probe(fn: str, x, y=None) -> np.ndarray:
    """csrc/refmath.h's restatement ``fn`` evaluated on the device (test hook:
    numpy's np.log / np.exp, scipy's expit, np.logaddexp, glibc's exp and
    log1p, bit for bit)."""
    x = f64(x).ravel()
    y = None if y is None else f64(y).ravel()
    out = np.empty_like(x)
    check(load().nemo_refmath_probe(REFMATH_FNS[fn], x.size, ptr(x), ptr(y), ptr(out)))
    return out
