"""The fixed-order optimizers of methods.py on the
CPU: the oracle's restatement against the goldens captured from the
reference, and the bounded / analytic-gradient L-BFGS-B specification
(oracle/lbfgsb1.py, which the HIP kernels follow) against scipy on every
local problem of those sweeps."""
import numpy as np
import pytest
from conftest import golden

import lbfgsb1
import nemo_oracle as no
from nemo import generator


def _model(name):
    if name == "net2":
        t = golden("net2_tables.npz")
        return t["U"], t["T"]
    m = generator.synthetic_nem(16, 500, 0)
    return m.U, m.get_score_tensor()


def _init(kind, order, s):
    parents = no.parents_of(order)
    w = np.zeros((s, s)) if kind == "gamma" else np.full((s, s), -5000.0)
    for i in range(s):
        for j in parents[i]:
            w[i][j] = 0.5 if kind == "gamma" else 0.0
    return w


@pytest.mark.parametrize("kind", ["gamma", "inverse"])
@pytest.mark.parametrize("name", ["net2", "C2"])
def test_oracle_sweeps_match_reference(kind, name):
    z = golden(f"methods_{kind}_{name}.npz")
    u, t = _model(name)
    order, s = z["order"], int(z["S"])
    w = _init(kind, order, s)
    f = no.opt_gamma if kind == "gamma" else no.opt_b
    for sweep in range(2):
        ll, w = f(u, t, order, w)
        assert ll == z["sweep_ll"][sweep]
        assert np.array_equal(w, z["sweep_w"][sweep])


@pytest.mark.parametrize("kind", ["gamma", "inverse"])
def test_bounded_spec_matches_scipy(kind, monkeypatch):
    """Every local problem of two net2 sweeps and one C2 sweep: the spec's
    x*, nit and nfev equal scipy's (all but a few, which differ in the last
    bits of x*: the spec's Cauchy step is x - g s/y, L-BFGS-B's the compact
    form of the same number)."""
    rec = []
    real = no.minimize

    def spy(fun, x0, args=(), **kw):
        snap = tuple(a.copy() if isinstance(a, np.ndarray) else a for a in args)
        r = real(fun, x0, args=args, **kw)
        rec.append((fun, float(np.asarray(x0).ravel()[0]), snap, kw, r))
        return r

    monkeypatch.setattr(no, "minimize", spy)
    for name, sweeps in (("net2", 2), ("C2", 1)):
        z = golden(f"methods_{kind}_{name}.npz")
        u, t = _model(name)
        w = _init(kind, z["order"], int(z["S"]))
        for _ in range(sweeps):
            _, w = (no.opt_gamma if kind == "gamma" else no.opt_b)(u, t, z["order"], w)
    assert len(rec) > 100
    same = 0
    for fun, x0, args, kw, r in rec:
        (lo, hi), = kw["bounds"]
        if kind == "gamma":
            c = args[0]
            x, f, nit, nfev, st = lbfgsb1.minimize_1d(
                lambda v: tuple(float(q) for q in fun(v, c)), x0, ftol=kw["tol"], gtol=kw["tol"],
                lo=lo, hi=hi, jac=True)
        else:
            w0 = args[0].copy()
            x, f, nit, nfev, st = lbfgsb1.minimize_1d(
                lambda v: float(fun(np.array([v]), w0, *args[1:])), x0, ftol=kw["tol"], gtol=kw["tol"],
                eps=kw["options"]["eps"], lo=lo, hi=hi)
        assert st in (lbfgsb1.CONV_PGTOL, lbfgsb1.CONV_REL) and r.success
        assert abs(x - r.x[0]) <= 1e-9 * max(1.0, abs(x))
        same += (x == r.x[0] and nit == r.nit and nfev == r.nfev)
    assert same >= 0.9 * len(rec)
