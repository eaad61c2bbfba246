"""CPU: the reference's own arithmetic as the device path restates it
(csrc/refmath.h, csrc/lbfgsb_exact.h, the wave plan of numpy's pairwise sum
in csrc/nemo_host.h), compiled for the host from the SAME headers and checked
bit for bit against numpy, scipy, glibc and the reference's recorded outputs.
(The device builds of the same headers: tests/test_gpu_exact.py.)"""
import ctypes
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest
from conftest import REPO, golden
from scipy.special import expit

CSRC = os.path.join(REPO, "nem-mcmc-optimization_amd", "csrc")
HOST = os.path.join(REPO, "tests", "host")
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


def _p(a):
    return a.ctypes.data_as(_dp)


@pytest.fixture(scope="module")
def spec(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("spec") / "libexact_spec.so")
    subprocess.run([hipcc, "-O2", "-fPIC", "-shared", "-ffp-contract=off", f"-I{CSRC}",
                    os.path.join(HOST, "exact_spec.cpp"), "-o", out], check=True)
    lib = ctypes.CDLL(out)
    lib.spec_objective.restype = ctypes.c_double
    lib.spec_objective.argtypes = [ctypes.c_int, _dp, ctypes.c_double, ctypes.c_double]
    lib.spec_eval.restype = ctypes.c_double
    lib.spec_plan_sum.restype = ctypes.c_double
    lib.spec_parts_sum.restype = ctypes.c_double
    lib.spec_pairwise_sum.restype = ctypes.c_double
    return lib


def _f_ref(x, c, anc):
    ex = expit(x)
    return -np.sum(np.log(c * ex + 1.0)) + np.abs(ex - anc) + ex * (1.0 - ex)


def test_refmath_host_check_against_the_libraries(tmp_path):
    """tests/host/refmath_check.cpp: every refmath.h function against glibc and
    numpy's own SVML kernels (dlopen'ed), 2 * 10^5 inputs per range."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    if "avx512f" not in open("/proc/cpuinfo").read():
        pytest.skip("SVML's AVX-512 kernels need an AVX-512 CPU")
    import numpy._core._multiarray_umath as um
    exe = str(tmp_path / "rc")
    pyver = f"python{sys.version_info.major}.{sys.version_info.minor}"
    subprocess.run([gxx, "-O2", "-std=c++17", "-mavx512f", "-mfma", "-ffp-contract=off", "-fno-builtin",
                    f"-I{CSRC}", os.path.join(HOST, "refmath_check.cpp"), "-ldl", "-Wl,--no-as-needed",
                    f"-l{pyver}", "-o", exe], check=True)
    r = subprocess.run([exe, um.__file__, "200000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def _scipy_openblas():
    """(path, architecture) of the OpenBLAS scipy.linalg calls."""
    import scipy.linalg  # noqa: F401  (loads it)
    from threadpoolctl import threadpool_info
    for p in threadpool_info():
        if p.get("internal_api") == "openblas" and "scipy.libs" in p.get("filepath", ""):
            return p["filepath"], p.get("architecture")
    return None, None


def test_lapack_inverse_restatement_against_scipys_openblas(tmp_path):
    """tests/host/lapack_check.c: getrf (n = 1..128) and getri (n <= 64) as
    csrc/nemo_ancestor.hip restates them, against scipy's own LAPACK calls
    (scipy_dgetrf_ / scipy_dgetri_, dlopen'ed), to the bit."""
    gcc = shutil.which("gcc")
    path, arch = _scipy_openblas()
    if gcc is None or path is None:
        pytest.skip("gcc or scipy's OpenBLAS not found")
    if arch != "SkylakeX":
        pytest.skip(f"the restatement is of OpenBLAS's SkylakeX kernels (this host: {arch})")
    exe = str(tmp_path / "lc")
    subprocess.run([gcc, "-O2", "-ffp-contract=off", os.path.join(HOST, "lapack_check.c"), "-ldl", "-lm",
                    "-o", exe], check=True)
    r = subprocess.run([exe, path, "6"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


def test_rcp14_step_function_bucketed_form_is_the_same():
    """svml_log's reduction point r = RNE_1/32(vrcp14pd(m)): the device's
    bucketed lookup (kRcp14Base / kRcp14InBucket) gives the threshold count
    of kRcp14Switch for every one of the 2^22 mantissa prefixes."""
    import re
    text = open(os.path.join(CSRC, "refmath_tables.h")).read()

    def arr(name):
        body = re.search(name + r"\[\d+\] = \{([^}]*)\}", text).group(1)
        return np.array([int(v.strip().rstrip("u"), 0) for v in body.split(",") if v.strip()], dtype=np.int64)
    th, base, inb = arr("kRcp14Switch"), arr("kRcp14Base"), arr("kRcp14InBucket")
    p = np.arange(1 << 22, dtype=np.int64)
    n_loop = np.searchsorted(th, p, side="right")
    n_bucket = base[p >> 16] + (p >= inb[p >> 16])
    assert np.array_equal(n_loop, n_bucket)


def test_elementwise_functions_equal_numpy_scipy(spec):
    rng = np.random.default_rng(3)
    n = 200000
    for name, fn, ref, x in (
            ("spec_svml_log", None, np.log, np.exp(rng.uniform(-7, 14, n))),
            ("spec_svml_exp", None, np.exp, rng.uniform(-707, 707, n)),
            ("spec_expit", None, expit, rng.normal(0, 8, n))):
        out = np.empty(n)
        getattr(spec, name)(ctypes.c_long(n), _p(x), _p(out))
        assert np.array_equal(out.view(np.uint64), ref(x).view(np.uint64)), name
    a, b = rng.normal(-60, 25, n), rng.normal(-60, 25, n)
    out = np.empty(n)
    spec.spec_logaddexp(ctypes.c_long(n), _p(a), _p(b), _p(out))
    assert np.array_equal(out, np.logaddexp(a, b))


def test_pairwise_sum_and_its_wave_plan(spec):
    """numpy's np.sum (pairwise) and the device's wave layout of it
    (host::build_pairwise_plan, run lane by lane on the host) for every E up
    to 700 and the configs' E."""
    rng = np.random.default_rng(5)
    for e in list(range(1, 700)) + [1999, 2000, 2001, 4096]:
        a = rng.normal(size=e) * np.exp(rng.normal(size=e) * 4)
        ref = np.sum(a)
        assert spec.spec_pairwise_sum(ctypes.c_long(e), _p(a)) == ref, e
        assert spec.spec_plan_sum(e, _p(a)) == ref, e


def test_np_sum_past_one_buffer_in_plan_parts(spec):
    """np.sum of more than 8192 terms adds numpy's buffer-sized chunks (8192,
    np.getbufsize()) in order, each summed pairwise -- not the pairwise
    recursion over all E: the device's
    parts (host::build_pairwise_parts, one wave plan per buffer) give numpy's
    bits for E past 8192, up to 64 buffers."""
    assert np.getbufsize() == 8192
    rng = np.random.default_rng(6)
    for e in (8192, 8193, 9000, 12345, 16384, 16385, 20000, 40000, 65536, 100001):
        a = rng.normal(size=e) * np.exp(rng.normal(size=e) * 4)
        assert spec.spec_parts_sum(e, _p(a)) == np.sum(a), e
        assert spec.spec_parts_sum(e, _p(a)) == np.add.reduce(a), e


@pytest.mark.parametrize("name", ["net2_200", "C2_20"])
def test_local_optima_equal_scipy_records_bit_for_bit(spec, name):
    """The objective at recorded points equals numpy's, and every recorded
    scipy optimisation (x*, f*, nit, nfev) is reproduced to the bit."""
    z = golden(f"localopt_{name}.npz")
    c = np.ascontiguousarray(z["c"])
    n, e = c.shape
    for k in range(0, n, 11):
        for x in (z["x0"][k], z["xstar"][k], z["xstar"][k] + 1e-8):
            assert spec.spec_objective(e, _p(c[k]), float(z["anc"][k]), float(x)) == \
                float(_f_ref(np.array([x]), c[k], z["anc"][k])[0])
    xs, fs = np.zeros(n), np.zeros(n)
    nit, nfev, st = (np.zeros(n, np.int32) for _ in range(3))
    spec.spec_local_opt(n, e, _p(c), _p(np.ascontiguousarray(z["anc"], dtype=np.float64)),
                        _p(np.ascontiguousarray(z["x0"], dtype=np.float64)), _p(xs), _p(fs),
                        nit.ctypes.data_as(_ip), nfev.ctypes.data_as(_ip), st.ctypes.data_as(_ip))
    assert np.array_equal(nit, z["nit"]) and np.array_equal(nfev, z["nfev"])
    assert np.array_equal(xs, z["xstar"]) and np.array_equal(fs, z["fun"])


def test_long_local_optima_equal_scipy_bit_for_bit(spec):
    """The C3 optima that run longest (nit 6..11: the memory of m = 10 pairs
    full and its oldest pair dropped; tests/golden/make_localopt_long.py)."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from make_localopt_long import long_cases
    c, anc, x0, rec = long_cases()
    c = np.ascontiguousarray(c)
    n, e = c.shape
    xs, fs = np.zeros(n), np.zeros(n)
    nit, nfev, st = (np.zeros(n, np.int32) for _ in range(3))
    spec.spec_local_opt(n, e, _p(c), _p(np.ascontiguousarray(anc)), _p(np.ascontiguousarray(x0)), _p(xs), _p(fs),
                        nit.ctypes.data_as(_ip), nfev.ctypes.data_as(_ip), st.ctypes.data_as(_ip))
    assert rec["nit"].max() == 11
    assert np.array_equal(nit, rec["nit"]) and np.array_equal(nfev, rec["nfev"])
    assert np.array_equal(xs, rec["xstar"]) and np.array_equal(fs, rec["fun"])


@pytest.mark.parametrize("name,s,e,k", [("C2", 16, 500, 8), ("C3", 64, 2000, 3)])
def test_order_scores_equal_reference_goldens_bit_for_bit(spec, name, s, e, k):
    """compute_cell_ratios + calculate_ll in the reference's order: ll, cs and
    the order weights of the golden evaluations, to the bit."""
    sys.path.insert(0, os.path.join(REPO, "nem-mcmc-optimization_amd"))
    from nemo import generator
    z = golden(f"eval_{name}.npz")
    m = generator.synthetic_nem(s, e, 0)
    t = np.ascontiguousarray(m.get_score_tensor(), dtype=np.float64)
    u = np.ascontiguousarray(m.U)
    cells, cs, ow = np.zeros((s + 1, e)), np.zeros(e), np.zeros((s + 1, e))
    for j in range(k):
        perm = np.ascontiguousarray(z["perm"][j], dtype=np.int32)
        ll = spec.spec_eval(s, e, _p(u), _p(t), perm.ctypes.data_as(_ip), _p(np.ascontiguousarray(z["W"][j])),
                            _p(cells), _p(cs), _p(ow))
        assert ll == z["ll"][j] and np.array_equal(cs, z["cs"][j])
        if j == 0:
            assert np.array_equal(ow, z["ow0"])
