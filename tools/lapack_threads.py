"""Can the host's ancestor_x inversions run in parallel threads?  The same
LAPACK getrf / getri scipy.linalg.inv calls, through scipy.linalg.cython_lapack's
function pointers with ctypes (which releases the GIL): bits against
nemo.chains.inv_stack, time serial vs a thread pool.  python tools/lapack_threads.py"""
import ctypes as C
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nem-mcmc-optimization_amd"))
import numpy as np  # noqa: E402
from scipy.linalg import cython_lapack  # noqa: E402

from nemo.chains import _LAPACK, inv_stack  # noqa: E402

C.pythonapi.PyCapsule_GetPointer.restype = C.c_void_p
C.pythonapi.PyCapsule_GetPointer.argtypes = [C.py_object, C.c_char_p]
C.pythonapi.PyCapsule_GetName.restype = C.c_char_p
C.pythonapi.PyCapsule_GetName.argtypes = [C.py_object]


def fptr(name):
    c = cython_lapack.__pyx_capi__[name]
    return C.pythonapi.PyCapsule_GetPointer(c, C.pythonapi.PyCapsule_GetName(c))


IP, DP = C.POINTER(C.c_int), C.POINTER(C.c_double)
getrf = C.CFUNCTYPE(None, IP, IP, DP, IP, IP, IP)(fptr("dgetrf"))
getri = C.CFUNCTYPE(None, IP, DP, IP, IP, DP, IP, IP)(fptr("dgetri"))


def inv_ct(a, lwork):
    n = a.shape[0]
    f = np.array(a, order="F")
    piv = np.zeros(n, dtype=np.int32)
    info, nn, lw = C.c_int(0), C.c_int(n), C.c_int(lwork)
    getrf(C.byref(nn), C.byref(nn), f.ctypes.data_as(DP), C.byref(nn), piv.ctypes.data_as(IP), C.byref(info))
    work = np.empty(lwork)
    getri(C.byref(nn), f.ctypes.data_as(DP), C.byref(nn), piv.ctypes.data_as(IP), work.ctypes.data_as(DP),
          C.byref(lw), C.byref(info))
    return np.ascontiguousarray(f)


rng = np.random.default_rng(0)
S, n = 64, 16
a = []
for k in range(n):
    p = rng.permutation(S)
    sig = rng.uniform(-3, 3, (S, S)) * (rng.random((S, S)) < 0.2)
    m = p[:, None] < p[None, :]
    sig[m] = rng.random(m.sum())
    a.append(np.eye(S) - sig)
a = np.array(a)
ref = inv_stack(a)
lwork = _LAPACK[S][2]
print("cpus", os.cpu_count(), len(os.sched_getaffinity(0)))
print("bits equal:", np.array_equal(np.array([inv_ct(x, lwork) for x in a]), ref))


def T(f, k=20):
    ts = []
    for _ in range(k):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return np.median(ts) * 1e3


for nt in (2, 4, 8):
    ex = ThreadPoolExecutor(nt)
    print(f"16 inversions: inv_stack {T(lambda: inv_stack(a)):.3f} ms, ctypes serial "
          f"{T(lambda: [inv_ct(x, lwork) for x in a]):.3f} ms, ctypes {nt} threads "
          f"{T(lambda: list(ex.map(lambda x: inv_ct(x, lwork), a))):.3f} ms")
