"""ORACLE -- test infrastructure only.

Restatement of scipy 1.15's L-BFGS-B (``scipy.optimize.minimize(method=
'L-BFGS-B')``, C translation of L-BFGS-B 3.0: mainlb/cauchy/subsm/lnsrlb/
dcsrch/dcstep) specialised to what the reference calls it with at
nem_order_mcmc.py:167:

* one variable, bounds (-inf, inf)   -> no projection, every variable free;
* tol=0.01                           -> ftol = gtol (pgtol) = 0.01;
* jac=None                           -> forward difference, absolute step
  eps=1e-8, dx recomputed as (x+h)-x (scipy optimize/_numdiff.py);
* defaults m=10, maxls=20, maxiter=maxfun=15000.

With n = 1 the compact L-BFGS matrix after any update reduces to the secant
slope of the latest accepted pair, B = y/s, so the subspace step is the
secant-Newton step -g*s/y (the generalised Cauchy point before the first
update is x - g/theta, theta = 1).  The line search is More-Thuente dcsrch
with ftol=1e-3, gtol=0.9, xtol=0.1, stpmin=0, stpmax=1e10; the first trial
step of iteration 0 is 1/|d|.

This module is the *specification* the HIP ``local_opt`` kernel implements;
tests/test_lbfgsb1.py checks it against scipy itself on the golden local-
optimum inputs captured from the reference run.
"""
from __future__ import annotations

import math

EPSMCH = 2.220446049250313e-16
SQRT_EPS = 1.4901161193847656e-08

# status codes shared with the HIP kernel (include/nemo.h)
CONV_PGTOL = 0      # CONVERGENCE: NORM_OF_PROJECTED_GRADIENT_<=_PGTOL
CONV_REL = 1        # CONVERGENCE: REL_REDUCTION_OF_F_<=_FACTR*EPSMCH
ABNORMAL = 2        # ABNORMAL_TERMINATION_IN_LNSRCH
MAXITER = 3


def dcstep(stx, fx, dx, sty, fy, dy, stp, fp, dp, brackt, stpmin, stpmax):
    """MINPACK-2 dcstep (safeguarded cubic/quadratic step)."""
    sgnd = dp * (dx / abs(dx))
    if fp > fx:
        theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * math.sqrt((theta / s) ** 2 - (dx / s) * (dp / s))
        if stp < stx:
            gamma = -gamma
        p = (gamma - dx) + theta
        q = ((gamma - dx) + gamma) + dp
        r = p / q
        stpc = stx + r * (stp - stx)
        stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx)
        stpf = stpc if abs(stpc - stx) < abs(stpq - stx) else stpc + (stpq - stpc) / 2.0
        brackt = True
    elif sgnd < 0.0:
        theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * math.sqrt((theta / s) ** 2 - (dx / s) * (dp / s))
        if stp > stx:
            gamma = -gamma
        p = (gamma - dp) + theta
        q = ((gamma - dp) + gamma) + dx
        r = p / q
        stpc = stp + r * (stx - stp)
        stpq = stp + (dp / (dp - dx)) * (stx - stp)
        stpf = stpc if abs(stpc - stp) > abs(stpq - stp) else stpq
        brackt = True
    elif abs(dp) < abs(dx):
        theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * math.sqrt(max(0.0, (theta / s) ** 2 - (dx / s) * (dp / s)))
        if stp > stx:
            gamma = -gamma
        p = (gamma - dp) + theta
        q = (gamma + (dx - dp)) + gamma
        r = p / q
        if r < 0.0 and gamma != 0.0:
            stpc = stp + r * (stx - stp)
        elif stp > stx:
            stpc = stpmax
        else:
            stpc = stpmin
        stpq = stp + (dp / (dp - dx)) * (stx - stp)
        if brackt:
            stpf = stpc if abs(stpc - stp) < abs(stpq - stp) else stpq
            if stp > stx:
                stpf = min(stp + 0.66 * (sty - stp), stpf)
            else:
                stpf = max(stp + 0.66 * (sty - stp), stpf)
        else:
            stpf = stpc if abs(stpc - stp) > abs(stpq - stp) else stpq
            stpf = min(stpmax, stpf)
            stpf = max(stpmin, stpf)
    else:
        if brackt:
            theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp
            s = max(abs(theta), abs(dy), abs(dp))
            gamma = s * math.sqrt((theta / s) ** 2 - (dy / s) * (dp / s))
            if stp > sty:
                gamma = -gamma
            p = (gamma - dp) + theta
            q = ((gamma - dp) + gamma) + dy
            r = p / q
            stpc = stp + r * (sty - stp)
            stpf = stpc
        elif stp > stx:
            stpf = stpmax
        else:
            stpf = stpmin
    if fp > fx:
        sty, fy, dy = stp, fp, dp
    else:
        if sgnd < 0.0:
            sty, fy, dy = stx, fx, dx
        stx, fx, dx = stp, fp, dp
    return stx, fx, dx, sty, fy, dy, stpf, brackt


class Dcsrch:
    """MINPACK-2 dcsrch as a resumable state machine (task 'FG' = evaluate)."""
    FTOL, GTOL, XTOL = 1e-3, 0.9, 0.1

    def __init__(self, stpmin, stpmax):
        self.stpmin, self.stpmax = stpmin, stpmax

    def start(self, stp, f, g):
        if g >= 0.0:
            return stp, "ERROR"
        self.brackt = False
        self.stage = 1
        self.finit, self.ginit = f, g
        self.gtest = self.FTOL * g
        self.width = self.stpmax - self.stpmin
        self.width1 = self.width / 0.5
        self.stx, self.fx, self.gx = 0.0, f, g
        self.sty, self.fy, self.gy = 0.0, f, g
        self.stmin = 0.0
        self.stmax = stp + 4.0 * stp
        return stp, "FG"

    def step(self, stp, f, g):
        ftest = self.finit + stp * self.gtest
        if self.stage == 1 and f <= ftest and g >= 0.0:
            self.stage = 2
        task = None
        if self.brackt and (stp <= self.stmin or stp >= self.stmax):
            task = "WARN"
        if self.brackt and self.stmax - self.stmin <= self.XTOL * self.stmax:
            task = "WARN"
        if stp == self.stpmax and f <= ftest and g <= self.gtest:
            task = "WARN"
        if stp == self.stpmin and (f > ftest or g >= self.gtest):
            task = "WARN"
        if f <= ftest and abs(g) <= self.GTOL * (-self.ginit):
            task = "CONV"
        if task is not None:
            return stp, task
        if self.stage == 1 and f <= self.fx and f > ftest:
            fm = f - stp * self.gtest
            fxm = self.fx - self.stx * self.gtest
            fym = self.fy - self.sty * self.gtest
            gm = g - self.gtest
            gxm = self.gx - self.gtest
            gym = self.gy - self.gtest
            (self.stx, fxm, gxm, self.sty, fym, gym, stp, self.brackt) = dcstep(
                self.stx, fxm, gxm, self.sty, fym, gym, stp, fm, gm, self.brackt, self.stmin, self.stmax)
            self.fx = fxm + self.stx * self.gtest
            self.fy = fym + self.sty * self.gtest
            self.gx = gxm + self.gtest
            self.gy = gym + self.gtest
        else:
            (self.stx, self.fx, self.gx, self.sty, self.fy, self.gy, stp, self.brackt) = dcstep(
                self.stx, self.fx, self.gx, self.sty, self.fy, self.gy, stp, f, g, self.brackt,
                self.stmin, self.stmax)
        if self.brackt:
            if abs(self.sty - self.stx) >= 0.66 * self.width1:
                stp = self.stx + 0.5 * (self.sty - self.stx)
            self.width1 = self.width
            self.width = abs(self.sty - self.stx)
            self.stmin = min(self.stx, self.sty)
            self.stmax = max(self.stx, self.sty)
        else:
            self.stmin = stp + 1.1 * (stp - self.stx)
            self.stmax = stp + 4.0 * (stp - self.stx)
        stp = max(stp, self.stpmin)
        stp = min(stp, self.stpmax)
        if (self.brackt and (stp <= self.stmin or stp >= self.stmax)) or \
           (self.brackt and self.stmax - self.stmin <= self.XTOL * self.stmax):
            stp = self.stx
        return stp, "FG"


def minimize_1d(fun, x0, ftol=0.01, gtol=0.01, eps=1e-8, maxls=20, maxiter=15000, maxfun=15000,
                lo=-math.inf, hi=math.inf, jac=False):
    """Returns (x*, f*, nit, nfev, status).

    ``lo``/``hi``: the bounds (scipy ``bounds=[(lo, hi)]``); ``jac=True``:
    ``fun`` returns (f, g) (scipy ``jac=True``), else forward differences with
    absolute step ``eps``.  With both bounds finite (the fixed-order methods,
    methods.py:95, :238, :384) L-BFGS-B 3.0 runs its constrained branch:
    x0 clipped, projected gradient, generalised Cauchy point with the bound
    as breakpoint, unit first step and stpmax from the bounds."""
    nfev = 0
    cache = [None, 0.0, 0.0]   # scipy's ScalarFunction memoises the last (x, f, g)
    cnstnd = lo > -math.inf or hi < math.inf
    boxed = lo > -math.inf and hi < math.inf

    def f_and_g(x):
        nonlocal nfev
        if cache[0] is not None and x == cache[0]:
            return cache[1], cache[2]
        if jac:
            f0, g = fun(x)
            nfev += 1
        else:
            f0 = fun(x)
            h = eps
            if (x + h) - x == 0.0:
                h = SQRT_EPS * (1.0 if x >= 0.0 else -1.0) * max(1.0, abs(x))
            if cnstnd:     # scipy optimize/_numdiff.py _adjust_scheme_to_bounds('1-sided')
                ldist, udist = x - lo, hi - x
                xt = x + h
                fitting = abs(h) <= max(ldist, udist)
                if (xt < lo or xt > hi) and fitting:
                    h = -h
                elif not fitting:
                    h = udist if udist >= ldist else -ldist
            x1 = x + h
            g = (fun(x1) - f0) / (x1 - x)
            nfev += 2
        cache[:] = [x, f0, g]
        return f0, g

    def projg(x, g):           # projgr
        if g < 0.0:
            return max(x - hi, g) if hi < math.inf else g
        return min(x - lo, g) if lo > -math.inf else g

    tol = (ftol / EPSMCH) * EPSMCH
    x = min(max(float(x0), lo), hi)
    f, g = f_and_g(x)
    if abs(projg(x, g)) <= gtol:
        return x, f, 0, nfev, CONV_PGTOL
    nit = 0
    have_pair = False   # col > 0
    s_last = y_last = 0.0
    theta = 1.0
    while True:
        # search direction d = z - x, z the subspace minimiser (lnsrlb works
        # with the rounded d, and evaluates the unit step at z itself):
        # Cauchy point x - g/theta before the first update (theta = 1 then),
        # secant-Newton step -g*s/y afterwards; with bounds, the GCP stops at
        # the bound when the model's minimiser lies beyond it (cauchy: the
        # breakpoint tl/g or tu/-g against dtm)
        if have_pair:
            dtm = s_last / y_last
            z = x + (-g) * dtm
        else:
            dtm = 1.0 / theta
            z = x + dtm * (-g)
        if cnstnd and g != 0.0:
            if g > 0.0 and lo > -math.inf:
                dt, zb = (x - lo) / g, lo
            elif g < 0.0 and hi < math.inf:
                dt, zb = (hi - x) / (-g), hi
            else:
                dt = None
            if dt is not None and not (dtm < dt):
                z = zb
        d = z - x
        # lnsrlb
        dnorm = abs(d)  # scipy: dnrm2 (OpenBLAS, extended precision): |d| exactly for n = 1
        stpmx = 1e10
        if cnstnd:
            if nit == 0:
                stpmx = 1.0
            elif d < 0.0 and lo > -math.inf:
                a2 = lo - x
                if a2 >= 0.0:
                    stpmx = 0.0
                elif d * stpmx < a2:
                    stpmx = a2 / d
            elif d > 0.0 and hi < math.inf:
                a2 = hi - x
                if a2 <= 0.0:
                    stpmx = 0.0
                elif d * stpmx > a2:
                    stpmx = a2 / d
        stp = min(1.0 / dnorm, stpmx) if (nit == 0 and not boxed) else 1.0
        xk, fold, gold = x, f, g
        gd = g * d
        task = "FAIL"
        if gd < 0.0:
            ls = Dcsrch(0.0, stpmx)
            stp, task = ls.start(stp, f, gd)
            gdold = gd
            ifun = 0
            while True:
                ifun += 1
                if ifun - 1 >= maxls:       # iback >= maxls
                    task = "FAIL"
                    break
                x = z if stp == 1.0 else stp * d + xk
                f, g = f_and_g(x)
                gd = g * d
                stp, task = ls.step(stp, f, gd)
                if task != "FG":
                    break
        if task == "FAIL" or task == "ERROR":
            # restore the previous iterate; with no pairs stored this is fatal,
            # otherwise the memory is dropped and the iteration restarts
            x, f, g = xk, fold, gold
            if not have_pair:
                return x, f, nit, nfev, ABNORMAL
            have_pair = False
            theta = 1.0
            continue
        nit += 1
        if abs(projg(x, g)) <= gtol:
            return x, f, nit, nfev, CONV_PGTOL
        if (fold - f) <= tol * max(abs(fold), abs(f), 1.0):
            return x, f, nit, nfev, CONV_REL
        if nit >= maxiter or nfev > maxfun:
            return x, f, nit, nfev, MAXITER
        # L-BFGS update (skipped on non-positive curvature)
        r = g - gold
        rr = r * r
        if stp == 1.0:
            dr = gd - gdold
            ddum = -gdold
            s = d
        else:
            dr = (gd - gdold) * stp
            s = d * stp
            ddum = -gdold * stp
        if dr <= EPSMCH * ddum:
            continue
        have_pair = True
        s_last, y_last = s, r
        theta = rr / dr
