"""Prototype: scipy 1.15's L-BFGS-B (the C translation of L-BFGS-B 3.0) for
ONE unbounded variable with its compact-form arithmetic kept as written
(matupd / formt / formk / cmprlb / subsm / bmv, m = 10), calling the same
BLAS / LAPACK routines through scipy.linalg.blas / lapack (the same
scipy_openblas library scipy's _lbfgsb links), or -- with ``scalar=True`` --
the scalar restatements of those routines (tools/openblas_small.py) that the
device port follows.  Used to find where the simplified secant form
(oracle/lbfgsb1.py) departs from scipy's bits; see DESIGN.md 3.5b.
"""
from __future__ import annotations

import math

import numpy as np

EPSMCH = 2.220446049250313e-16
SQRT_EPS = 1.4901161193847656e-08


class Blas:
    """The library's own routines (column-major, upper triangles)."""

    def __init__(self):
        from scipy.linalg import blas, lapack
        self.b, self.l = blas, lapack

    def ddot(self, x, y):
        n = len(x)
        return float(self.b.ddot(np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64))) if n else 0.0

    def potrf_u(self, a):
        """dpotrf('U') of the leading n x n block; returns (factor, info)."""
        c, info = self.l.dpotrf(np.asfortranarray(a), lower=0, clean=0)
        return c, info

    def trtrs(self, a, b, trans):
        """dtrtrs('U', trans, 'N')."""
        x, info = self.l.dtrtrs(np.asfortranarray(a), np.asarray(b, dtype=np.float64), lower=0, trans=trans)
        return x, info


def minimize_1d(fun, x0, blas=None, m=10, ftol=0.01, pgtol=0.01, eps=1e-8, maxls=20, maxiter=15000,
                trace=None):
    import sys
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/oracle")
    import lbfgsb1 as spec
    B = blas or Blas()
    nfev = 0
    cache = [None, 0.0, 0.0]

    def f_and_g(x):
        nonlocal nfev
        if cache[0] is not None and x == cache[0]:
            return cache[1], cache[2]
        f0 = fun(x)
        h = eps
        if (x + h) - x == 0.0:
            h = SQRT_EPS * (1.0 if x >= 0.0 else -1.0) * max(1.0, abs(x))
        x1 = x + h
        g = (fun(x1) - f0) / (x1 - x)
        nfev += 2
        cache[:] = [x, f0, g]
        return f0, g

    factr = ftol / EPSMCH
    tol = factr * EPSMCH
    x = float(x0)
    f, g = f_and_g(x)
    if abs(g) <= pgtol:
        return x, f, 0, nfev, spec.CONV_PGTOL
    # state (0-based pointers)
    ws = np.zeros(m)
    wy = np.zeros(m)
    sy = np.zeros((m, m))
    ss = np.zeros((m, m))
    wt = np.zeros((m, m))
    wn1 = np.zeros((2 * m, 2 * m))
    col, head, itail, iupdat, theta, updatd = 0, 0, 0, 0, 1.0, False
    nit = 0
    wn = None
    while True:
        # ---- search for the GCP (cauchy) or skip it (unconstrained, col > 0)
        if col > 0:
            z = x
            wrk = updatd
        else:
            # cauchy with col = 0: d = -g, f1 = -g*g, f2 = -theta*f1, dtm = -f1/f2
            neggi = -g
            f1 = 0.0 - neggi * neggi
            f2 = -theta * f1
            dtm = -f1 / f2
            if dtm <= 0.0:
                dtm = 0.0
            tsum = 0.0 + dtm
            z = x + tsum * neggi     # daxpy, n = 1
            wrk = False
        if col > 0:
            if wrk:
                wn = formk(B, m, ws, wy, sy, wn1, theta, col, head, updatd, iupdat)
                if wn is None:
                    raise RuntimeError("formk: not positive definite (restart not restated)")
            r = -g                  # cmprlb, unconstrained with col > 0
            z = subsm(B, m, ws, wy, theta, col, head, wn, r, z, x, g)
        # ---- lnsrlb
        d = z - x
        dtd = B.ddot([d], [d])
        dnorm = math.sqrt(dtd)
        stpmx = 1e10
        stp = min(1.0 / dnorm, stpmx) if nit == 0 else 1.0
        xk, fold, gold = x, f, g
        gd = B.ddot([g], [d])
        task = "FAIL"
        if gd < 0.0:
            ls = spec.Dcsrch(0.0, stpmx)
            stp, task = ls.start(stp, f, gd)
            gdold = gd
            ifun = 0
            while True:
                ifun += 1
                if ifun - 1 >= maxls:
                    task = "FAIL"
                    break
                x = z if stp == 1.0 else stp * d + xk
                f, g = f_and_g(x)
                gd = B.ddot([g], [d])
                stp, task = ls.step(stp, f, gd)
                if task != "FG":
                    break
        if task in ("FAIL", "ERROR"):
            x, f, g = xk, fold, gold
            if col == 0:
                return x, f, nit, nfev, spec.ABNORMAL
            col, head, itail, iupdat, theta, updatd = 0, 0, 0, 0, 1.0, False
            continue
        nit += 1
        if abs(g) <= pgtol:
            return x, f, nit, nfev, spec.CONV_PGTOL
        ddum = max(abs(fold), abs(f), 1.0)
        if (fold - f) <= tol * ddum:
            return x, f, nit, nfev, spec.CONV_REL
        if nit >= maxiter:
            return x, f, nit, nfev, spec.MAXITER
        # ---- update
        r = g - gold
        rr = B.ddot([r], [r])
        if stp == 1.0:
            dr = gd - gdold
            ddum = -gdold
        else:
            dr = (gd - gdold) * stp
            d = d * stp             # dscal
            ddum = -gdold * stp
        if dr <= EPSMCH * ddum:
            updatd = False
            continue
        updatd = True
        iupdat += 1
        # matupd
        if iupdat <= m:
            col = iupdat
            itail = (head + iupdat - 1) % m
        else:
            itail = (itail + 1) % m
            head = (head + 1) % m
        ws[itail] = d
        wy[itail] = r
        theta = rr / dr
        if iupdat > m:
            for j in range(col - 1):
                ss[0:j + 1, j] = ss[1:j + 2, j + 1]
                sy[j:col - 1, j] = sy[j + 1:col, j + 1]
        p = head
        for j in range(col - 1):
            sy[col - 1, j] = B.ddot([d], [wy[p]])
            ss[j, col - 1] = B.ddot([ws[p]], [d])
            p = (p + 1) % m
        ss[col - 1, col - 1] = dtd if stp == 1.0 else stp * stp * dtd
        sy[col - 1, col - 1] = dr
        # formt
        for j in range(col):
            wt[0, j] = theta * ss[0, j]
        for i in range(1, col):
            for j in range(i, col):
                k1 = min(i, j)
                ddum = 0.0
                for k in range(k1):
                    ddum = ddum + sy[i, k] * sy[j, k] / sy[k, k]
                wt[i, j] = ddum + theta * ss[i, j]
        c, info = B.potrf_u(wt[:col, :col])
        if info != 0:
            raise RuntimeError("formt: not positive definite (restart not restated)")
        wt[:col, :col] = np.triu(c) + np.tril(wt[:col, :col], -1)
        if trace is not None:
            trace.append((nit, col, theta))


def formk(B, m, ws, wy, sy, wn1, theta, col, head, updatd, iupdat):
    """formk for n = nsub = 1, every variable free and staying free
    (nenter = 0, ileave = n + 1): WN1's new row / column, then WN and its
    two Cholesky factorisations (None when one fails)."""
    if updatd:
        if iupdat > m:
            for jy in range(m - 1):
                js = m + jy
                wn1[jy:m - 1, jy] = wn1[jy + 1:m, jy + 1]
                wn1[js:js + m - jy - 1, js] = wn1[js + 1:js + m - jy, js + 1]
                wn1[m:2 * m - 1, jy] = wn1[m + 1:2 * m, jy + 1]
        iy = col - 1
        is_ = m + col - 1
        ipntr = (head + col - 1) % m
        jpntr = head
        for jy in range(col):
            js = m + jy
            temp1 = 0.0 + wy[ipntr] * wy[jpntr]
            wn1[iy, jy] = temp1
            wn1[is_, js] = 0.0
            wn1[is_, jy] = 0.0
            jpntr = (jpntr + 1) % m
        jy = col - 1
        jpntr = (head + col - 1) % m
        ipntr = head
        for i in range(col):
            is2 = m + i
            temp3 = 0.0 + ws[ipntr] * wy[jpntr]
            ipntr = (ipntr + 1) % m
            wn1[is2, jy] = temp3
        upcl = col - 1
    else:
        upcl = col
    for iy in range(upcl):
        is_ = m + iy
        for jy in range(iy + 1):
            js = m + jy
            wn1[iy, jy] = wn1[iy, jy] + 0.0 - 0.0
            wn1[is_, js] = wn1[is_, js] - 0.0 + 0.0
    for is_ in range(m, m + upcl):
        for jy in range(upcl):
            if is_ <= jy + m:
                wn1[is_, jy] = wn1[is_, jy] + 0.0 - 0.0
            else:
                wn1[is_, jy] = wn1[is_, jy] - 0.0 + 0.0
    c2 = 2 * col
    wn = np.zeros((c2, c2))
    for iy in range(col):
        is_ = col + iy
        is1 = m + iy
        for jy in range(iy + 1):
            js = col + jy
            js1 = m + jy
            wn[jy, iy] = wn1[iy, jy] / theta
            wn[js, is_] = wn1[is1, js1] * theta
        for jy in range(iy):
            wn[jy, is_] = -wn1[is1, jy]
        for jy in range(iy, col):
            wn[jy, is_] = wn1[is1, jy]
        wn[iy, iy] = wn[iy, iy] + sy[iy, iy]
    c, info = B.potrf_u(wn[:col, :col])
    if info != 0:
        return None
    wn[:col, :col] = np.triu(c) + np.tril(wn[:col, :col], -1)
    # one dtrtrs('U', 'T', 'N') with nrhs = col (the C translation's single
    # call for the whole (1,2) block, not one solve per column)
    xblk, info = B.trtrs(wn[:col, :col], np.asfortranarray(wn[:col, col:c2]), 1)
    if info != 0:
        return None
    wn[:col, col:c2] = xblk
    for is_ in range(col, c2):
        for js in range(is_, c2):
            wn[is_, js] = wn[is_, js] + B.ddot(wn[:col, is_], wn[:col, js])
    c, info = B.potrf_u(wn[col:, col:])
    if info != 0:
        return None
    wn[col:, col:] = np.triu(c) + np.tril(wn[col:, col:], -1)
    return wn


def subsm(B, m, ws, wy, theta, col, head, wn, d, z, xx, gg):
    """subsm for nsub = 1 (unbounded): the Newton step from z = x; returns
    the new z (the projection's descent check kept)."""
    c2 = 2 * col
    wv = np.zeros(c2)
    p = head
    for i in range(col):
        temp1 = 0.0 + wy[p] * d
        temp2 = 0.0 + ws[p] * d
        wv[i] = temp1
        wv[col + i] = theta * temp2
        p = (p + 1) % m
    up = np.triu(wn)
    wv, info = B.trtrs(up, wv, 1)
    if info != 0:
        raise RuntimeError("subsm: singular")
    wv[:col] = -wv[:col]
    wv, info = B.trtrs(up, wv, 0)
    if info != 0:
        raise RuntimeError("subsm: singular")
    p = head
    for jy in range(col):
        js = col + jy
        d = d + wy[p] * wv[jy] / theta + ws[p] * wv[js]
        p = (p + 1) % m
    d = d * (1.0 / theta)
    xk = z
    znew = xk + d
    dd_p = 0.0 + (znew - xx) * gg
    if dd_p > 0.0:
        raise RuntimeError("subsm: positive directional derivative (backtracking not restated)")
    return znew
