"""Pin the C restatement of the order score (oracle/nemo_oracle_c.c, the CPU
twin of the score kernels; test infrastructure like the numpy oracle) to the
reference's golden vectors and to oracle/nemo_oracle.py, and run it under
AddressSanitizer + UndefinedBehaviorSanitizer.

Tolerance: the operation order is the numpy oracle's, but exp / log / log1p
are the C library's (numpy has SIMD loops of its own), so ll agrees with the
reference's goldens within 1e-9 absolute (observed: bit-equal on net2 and C2,
<= 7.3e-12 on C3, 30 of 32 bit-equal) and every column log-sum-exp within
1e-12.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest
from conftest import REPO, golden
from scipy.special import expit

import nemo_oracle as no
import nemo_oracle_c as oc
from nemo import generator

LL_TOL, CS_TOL = 1e-9, 1e-12


def _tables(z, name):
    if name == "net2":
        t = golden("net2_tables.npz")
        return t["U"], t["T"]
    s, e = int(z["S"]), int(z["E"])
    d = np.unpackbits(z["D_packed"])[: s * e].reshape(s, e).astype(np.float64)
    tt = no.score_tensor(d, float(z["A"]), float(z["B"]))
    return no.node_lr_table(tt, d, float(z["A"])), tt


@pytest.mark.parametrize("name,count", [("net2", None), ("C2", None), ("C3", None), ("C5cap", 8)])
def test_c_oracle_matches_reference_goldens(name, count):
    z = golden(f"eval_{name}.npz")
    u, tt = _tables(z, name)
    n = len(z["ll"]) if count is None else count
    pos = np.argsort(z["perm"][:n], axis=1).astype(np.int32)
    cap = int(z["cap"]) if "cap" in z.files else 0
    ll, cs = oc.order_scores(u, tt, pos, expit(z["W"][:n]), cap=cap, threads=4, want_cs=True)
    assert np.max(np.abs(ll - z["ll"][:n])) <= LL_TOL
    assert np.max(np.abs(cs - z["cs"][:n])) <= CS_TOL
    if name in ("net2", "C2"):
        assert np.array_equal(ll, z["ll"][:n])   # observed bit-equal here


@pytest.mark.parametrize("s,e,cap", [(1, 1, 0), (2, 1, 0), (3, 65, 0), (5, 130, 2), (9, 40, 1), (12, 77, 11)])
def test_c_oracle_matches_numpy_oracle(s, e, cap):
    m = generator.synthetic_nem(s, e, s + e)
    t = m.get_score_tensor()
    rng = np.random.default_rng(s * 1000 + e)
    perms = [rng.permutation(s) for _ in range(5)]
    w01 = expit(rng.uniform(-3, 3, (5, s, s)))
    pos = np.array([np.argsort(p) for p in perms], dtype=np.int32)
    ll = oc.order_scores(m.U, t, pos, w01, cap=cap)
    ref = np.array([no.order_score(m.U, t, perms[c], w01[c], cap) for c in range(5)])
    assert np.max(np.abs(ll - ref)) <= LL_TOL
    # thread count, batch split and cap >= S - 1 (no cap) change no bit
    assert np.array_equal(oc.order_scores(m.U, t, pos, w01, cap=cap, threads=3), ll)
    assert np.array_equal(np.concatenate([oc.order_scores(m.U, t, pos[c:c + 1], w01[c:c + 1], cap=cap)
                                          for c in range(5)]), ll)
    if cap == 0:
        assert np.array_equal(oc.order_scores(m.U, t, pos, w01, cap=max(s - 1, 1)), ll)


def test_c_oracle_edges():
    m = generator.synthetic_nem(4, 10, 0)
    t = m.get_score_tensor()
    assert oc.order_scores(m.U, t, np.zeros((0, 4), np.int32), np.zeros((0, 4, 4))).shape == (0,)
    with pytest.raises(ValueError, match="permutation"):
        oc.order_scores(m.U, t, np.array([[0, 0, 1, 2]], np.int32), np.zeros((1, 4, 4)))
    with pytest.raises(ValueError, match="shapes"):
        oc.order_scores(m.U, t, np.zeros((1, 3), np.int32), np.zeros((1, 4, 4)))


def test_c_oracle_clean_under_asan_ubsan(tmp_path):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not available")
    exe = tmp_path / "oracle_c_check"
    cmd = [gcc, "-std=c11", "-O1", "-g", "-Wall", "-Wextra", "-Werror", "-fopenmp", "-ffp-contract=off",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
           os.path.join(REPO, "oracle", "nemo_oracle_c.c"), os.path.join(REPO, "tests", "host", "oracle_c_check.c"),
           "-lm", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    res = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.startswith("ok "), res.stdout
    assert "runtime error" not in res.stderr, res.stderr
