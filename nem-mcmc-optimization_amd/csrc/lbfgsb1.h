// lbfgsb1.h -- L-BFGS-B (v3.0 logic, as scipy 1.15 runs it) for ONE unbounded
// variable, as a wave-uniform device routine.
//
// This is the optimiser the reference calls once per permissible (child,
// parent) pair and MCMC step: scipy.optimize.minimize(..., method='L-BFGS-B',
// bounds=[(-inf, inf)], tol=0.01) at nem_order_mcmc.py:167.  For n = 1:
//   * every variable is free, the projected gradient is |g|;
//   * before the first BFGS update the generalised Cauchy point is
//     x - g/theta (theta = 1); after it, the compact L-BFGS matrix reduces to
//     the secant slope y/s of the latest accepted pair, so the subspace step is
//     -g*s/y;
//   * lnsrlb: d = z - x (rounded), first trial step 1/|d| at iteration 0 and 1
//     afterwards, x = z at stp == 1; More-Thuente dcsrch (ftol 1e-3, gtol 0.9,
//     xtol 0.1, stpmin 0, stpmax 1e10), at most maxls = 20 trials, then restart
//     (memory dropped) or abnormal termination when no pair is stored;
//   * stopping: |g| <= pgtol (0.01), (fold - f) <= ftol * max(|fold|,|f|,1),
//     update skipped when s'y <= eps * (-g0'd * stp).
// The gradient is scipy's forward difference with absolute step 1e-8
// (scipy optimize/_numdiff.py): h = 1e-8 unless (x+h)-x == 0, then
// sqrt(eps)*sign(x)*max(1,|x|); g = (f(x+h) - f(x)) / ((x+h) - x).
//
// The objective is supplied by the caller as a functor
//   void fg(double x, double x1, double& f0, double& f1)
// that returns f(x) and f(x1) identically in every lane of the wave.
// Python specification: oracle/lbfgsb1.py (checked against scipy).
#pragma once

#include <hip/hip_runtime.h>

// the control code is also compiled for the host (tests/host: the exact
// compact form of lbfgsb_exact.h checked against scipy on the CPU)
#define NEMO_LB __host__ __device__ __forceinline__

namespace nemo {

struct LbfgsResult {
  double x, f;
  int nit, nfev, status;
};

namespace lb {

constexpr double kEpsMch = 2.220446049250313e-16;
constexpr double kSqrtEps = 1.4901161193847656e-08;
constexpr double kStpMax = 1e10;
constexpr double kFtolLs = 1e-3, kGtolLs = 0.9, kXtolLs = 0.1;

NEMO_LB double dmax(double a, double b) { return a > b ? a : b; }

// A branch of the optimiser's control flow: its condition is wave-uniform
// (every lane holds the same f, g and state), so the first lane decides and
// the compiler emits a scalar branch -- no exec-mask save / restore and no
// divergent-merge copies of the ~30 state values per branch.
NEMO_LB bool uni(bool b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane((int)b) != 0;
#else
  return b;
#endif
}
// H (the dual form, nemo_exact.hip): the condition is uniform within each
// half of the wave -- two optima's controls share the wave -- so it is a
// divergent branch (exec masks), not the first lane's decision
template <bool H>
NEMO_LB bool uniH(bool b) {
  return H ? b : uni(b);
}
NEMO_LB double dmin(double a, double b) { return a < b ? a : b; }

// MINPACK-2 dcstep: safeguarded step and interval update.
template <bool H = false>
NEMO_LB void dcstep(double& stx, double& fx, double& dx, double& sty, double& fy,
                              double& dy, double& stp, double fp, double dp, bool& brackt,
                              double stpmin, double stpmax) {
#pragma clang fp contract(off)
  // dp * (dx / |dx|) without the division (it heads the case selection's
  // dependent chain): dx / |dx| is exactly +-1 for a finite non-zero dx, so
  // the product is +-dp bit for bit; 0 / 0 and inf / inf give NaN, so does
  // this (and every test of sgnd is then false, as with the quotient)
  const double sgnd = (dx != 0.0 && fabs(dx) < __builtin_inf()) ? (dx > 0.0 ? dp : -dp) : __builtin_nan("");
  double stpf;
  if (uniH<H>(fp > fx)) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = dmax(dmax(fabs(theta), fabs(dx)), fabs(dp));
    const double ts = theta / s;
    double gamma = s * sqrt(ts * ts - (dx / s) * (dp / s));
    if (stp < stx) gamma = -gamma;
    const double p = (gamma - dx) + theta;
    const double q = ((gamma - dx) + gamma) + dp;
    const double r = p / q;
    const double stpc = stx + r * (stp - stx);
    const double stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
    stpf = (fabs(stpc - stx) < fabs(stpq - stx)) ? stpc : stpc + (stpq - stpc) / 2.0;
    brackt = true;
  } else if (uniH<H>(sgnd < 0.0)) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = dmax(dmax(fabs(theta), fabs(dx)), fabs(dp));
    const double ts = theta / s;
    double gamma = s * sqrt(ts * ts - (dx / s) * (dp / s));
    if (stp > stx) gamma = -gamma;
    const double p = (gamma - dp) + theta;
    const double q = ((gamma - dp) + gamma) + dx;
    const double r = p / q;
    const double stpc = stp + r * (stx - stp);
    const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
    stpf = (fabs(stpc - stp) > fabs(stpq - stp)) ? stpc : stpq;
    brackt = true;
  } else if (uniH<H>(fabs(dp) < fabs(dx))) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = dmax(dmax(fabs(theta), fabs(dx)), fabs(dp));
    const double ts = theta / s;
    double gamma = s * sqrt(dmax(0.0, ts * ts - (dx / s) * (dp / s)));
    if (stp > stx) gamma = -gamma;
    const double p = (gamma - dp) + theta;
    const double q = (gamma + (dx - dp)) + gamma;
    const double r = p / q;
    double stpc;
    if (r < 0.0 && gamma != 0.0) stpc = stp + r * (stx - stp);
    else if (stp > stx) stpc = stpmax;
    else stpc = stpmin;
    const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
    if (uniH<H>(brackt)) {
      stpf = (fabs(stpc - stp) < fabs(stpq - stp)) ? stpc : stpq;
      if (stp > stx) stpf = dmin(stp + 0.66 * (sty - stp), stpf);
      else stpf = dmax(stp + 0.66 * (sty - stp), stpf);
    } else {
      stpf = (fabs(stpc - stp) > fabs(stpq - stp)) ? stpc : stpq;
      stpf = dmin(stpmax, stpf);
      stpf = dmax(stpmin, stpf);
    }
  } else {
    if (uniH<H>(brackt)) {
      const double theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
      const double s = dmax(dmax(fabs(theta), fabs(dy)), fabs(dp));
      const double ts = theta / s;
      double gamma = s * sqrt(ts * ts - (dy / s) * (dp / s));
      if (stp > sty) gamma = -gamma;
      const double p = (gamma - dp) + theta;
      const double q = ((gamma - dp) + gamma) + dy;
      const double r = p / q;
      stpf = stp + r * (sty - stp);
    } else if (stp > stx) {
      stpf = stpmax;
    } else {
      stpf = stpmin;
    }
  }
  // the interval update as value selects: written as branches that assign
  // either end, the compiler kept (stx, fx, dx, sty, fy, dy) in a scratch
  // array with computed store addresses -- a chain of scratch round trips in
  // every line-search step, most of a lone wave's time per f-evaluation
  const bool upper = fp > fx;
  const bool swap = !upper && sgnd < 0.0;
  const double nsty = upper ? stp : (swap ? stx : sty);
  const double nfy = upper ? fp : (swap ? fx : fy);
  const double ndy = upper ? dp : (swap ? dx : dy);
  const double nstx = upper ? stx : stp;
  const double nfx = upper ? fx : fp;
  const double ndx = upper ? dx : dp;
  sty = nsty; fy = nfy; dy = ndy;
  stx = nstx; fx = nfx; dx = ndx;
  stp = stpf;
}

// MINPACK-2 dcsrch as a resumable state machine.
struct Dcsrch {
  bool brackt;
  int stage;
  double finit, ginit, gtest, width, width1;
  double stx, fx, gx, sty, fy, gy, stmin, stmax;
  double stpmax = kStpMax;  // lnsrlb's stpmx (1e10 unbounded; from the bounds otherwise)

  // returns false on ERROR (initial derivative not negative)
  template <bool H = false>
  NEMO_LB bool start(double stp, double f, double g) {
#pragma clang fp contract(off)
    if (uniH<H>(!(g < 0.0))) return false;
    brackt = false;
    stage = 1;
    finit = f;
    ginit = g;
    gtest = kFtolLs * g;
    width = stpmax - 0.0;
    width1 = width / 0.5;
    stx = 0.0; fx = f; gx = g;
    sty = 0.0; fy = f; gy = g;
    stmin = 0.0;
    stmax = stp + 4.0 * stp;
    return true;
  }

  // one dcsrch call with (f, g) at stp; returns 0 = FG (evaluate new stp),
  // 1 = CONV, 2 = WARN
  template <bool H = false>
  NEMO_LB int step(double& stp, double f, double g) {
#pragma clang fp contract(off)
    const double stpmin = 0.0;
    const double ftest = finit + stp * gtest;
    if (stage == 1 && f <= ftest && g >= 0.0) stage = 2;
    int task = 0;
    if (brackt && (stp <= stmin || stp >= stmax)) task = 2;
    if (brackt && stmax - stmin <= kXtolLs * stmax) task = 2;
    if (stp == stpmax && f <= ftest && g <= gtest) task = 2;
    if (stp == stpmin && (f > ftest || g >= gtest)) task = 2;
    if (f <= ftest && fabs(g) <= kGtolLs * (-ginit)) task = 1;
    if (uniH<H>(task != 0)) return task;
    // one dcstep call site on locals (keeps the state in registers): the
    // modified function psi is used in stage 1 when f fell but not enough
    const bool modified = stage == 1 && f <= fx && f > ftest;
    double sx = stx, sy = sty, fxl = fx, gxl = gx, fyl = fy, gyl = gy, fp = f, gp = g;
    if (uniH<H>(modified)) {
      fp = f - stp * gtest;
      fxl = fx - stx * gtest;
      fyl = fy - sty * gtest;
      gp = g - gtest;
      gxl = gx - gtest;
      gyl = gy - gtest;
    }
    dcstep<H>(sx, fxl, gxl, sy, fyl, gyl, stp, fp, gp, brackt, stmin, stmax);
    stx = sx;
    sty = sy;
    if (uniH<H>(modified)) {
      fx = fxl + stx * gtest;
      fy = fyl + sty * gtest;
      gx = gxl + gtest;
      gy = gyl + gtest;
    } else {
      fx = fxl; fy = fyl; gx = gxl; gy = gyl;
    }
    if (uniH<H>(brackt)) {
      if (fabs(sty - stx) >= 0.66 * width1) stp = stx + 0.5 * (sty - stx);
      width1 = width;
      width = fabs(sty - stx);
      stmin = dmin(stx, sty);
      stmax = dmax(stx, sty);
    } else {
      stmin = stp + 1.1 * (stp - stx);
      stmax = stp + 4.0 * (stp - stx);
    }
    stp = dmax(stp, stpmin);
    stp = dmin(stp, stpmax);
    if ((brackt && (stp <= stmin || stp >= stmax)) ||
        (brackt && stmax - stmin <= kXtolLs * stmax))
      stp = stx;
    return 0;
  }
};

// projgr: the projected gradient of one variable
template <bool BOUNDED>
__device__ __forceinline__ double projg(double x, double g, bool has_lo, double lo, bool has_hi, double hi) {
  if (!BOUNDED) return g;
  if (g < 0.0) return has_hi ? dmax(x - hi, g) : g;
  return has_lo ? dmin(x - lo, g) : g;
}

#ifdef NEMO_LO_TRACE
// cycle probe (instrumented builds only): the line-search step's share,
// accumulated into objectives that carry a cy_ls counter
template <class F>
__device__ __forceinline__ auto trace_ls(F& f, long long c, int) -> decltype(f.cy_ls += c, void()) { f.cy_ls += c; }
template <class F>
__device__ __forceinline__ void trace_ls(F&, long long, long) {}
#endif

}  // namespace lb

// Options of the bounded / analytic-gradient variant (the fixed-order
// optimizers of methods.py: bounds [(0, 1)] with jac=True at :393,
// [(-5000, 500)] with eps=1e-3 and tol=0.1 at :110).
struct LbOpts {
  double ftol = 0.01, gtol = 0.01, eps = 1e-8;
  double lo = -__builtin_inf(), hi = __builtin_inf();
  int maxls = 20, maxiter = 15000, maxfun = 15000;
};

// Minimise a 1-D objective from x0.  Without gradient (ANALYTIC = false)
// `fg(x, x1, f0, f1)` must return the objective at x and at x1; with it,
// `fg(x, f, g)` returns the objective and its derivative at x (identical in
// all lanes).  BOUNDED runs L-BFGS-B 3.0's constrained branch (cnstnd, and
// boxed when both bounds are finite, as in every bounded call the reference
// makes): x0 clipped, projected gradient, the generalised Cauchy point stops
// at the bound when the model minimiser lies beyond it, unit first trial
// step, stpmax from the bounds, forward differences flipped inside the box
// (scipy _numdiff._adjust_scheme_to_bounds).  Written as a state machine
// with ONE evaluation site so the (large, fully unrolled) objective body is
// instantiated once.  Python specification: oracle/lbfgsb1.py minimize_1d.
template <bool BOUNDED, bool ANALYTIC, class FG>
__device__ __forceinline__ LbfgsResult lbfgsb1_minimize_opts(FG& fg, double x0, const LbOpts o) {
#pragma clang fp contract(off)
  using namespace lb;
  const double tol = (o.ftol / kEpsMch) * kEpsMch;
  const double lo = o.lo, hi = o.hi;
  const bool has_lo = BOUNDED && lo > -__builtin_inf();
  const bool has_hi = BOUNDED && hi < __builtin_inf();
  const bool boxed = has_lo && has_hi;
  int nfev = 0, nit = 0, ifun = 0;
  bool have_pair = false, in_ls = false;
  double s_last = 0.0, y_last = 0.0, theta = 1.0;
  if (BOUNDED) x0 = dmin(dmax(x0, lo), hi);
  double x = x0, f = 0.0, g = 0.0;
  double z = 0.0, d = 0.0, stp = 0.0, xk = 0.0, fold = 0.0, gold = 0.0, gdold = 0.0;
  double x_eval = x0;
  bool have_last = false;
  double x_last = 0.0, f_last = 0.0, g_last = 0.0;
  Dcsrch ls;
  for (;;) {
    // ---- the single evaluation site: f and g at x_eval.  scipy's
    // ScalarFunction memoises the last point: a repeated x costs no
    // evaluation (and no nfev).
    if (uni(!(have_last && x_eval == x_last))) {
      if constexpr (ANALYTIC) {
        double f0, g0;
        fg(x_eval, f0, g0);
        nfev += 1;
        f_last = f0;
        g_last = g0;
      } else {
        double h = o.eps;
        if (uni((x_eval + h) - x_eval == 0.0))
          h = kSqrtEps * (x_eval >= 0.0 ? 1.0 : -1.0) * dmax(1.0, fabs(x_eval));
        if (BOUNDED) {
          const double ld = x_eval - lo, ud = hi - x_eval;
          const double xt = x_eval + h;
          const bool fitting = fabs(h) <= dmax(ld, ud);
          if ((xt < lo || xt > hi) && fitting) h = -h;
          else if (!fitting) h = (ud >= ld) ? ud : -ld;
        }
        const double x1 = x_eval + h;
        double f0, f1;
        fg(x_eval, x1, f0, f1);
        nfev += 2;
        f_last = f0;
        g_last = (f1 - f0) / (x1 - x_eval);
      }
      have_last = true;
      x_last = x_eval;
    }
    x = x_eval;
    f = f_last;
    g = g_last;

    if (uni(!in_ls)) {
      if (uni(fabs(lb::projg<BOUNDED>(x, g, has_lo, lo, has_hi, hi)) <= o.gtol)) return LbfgsResult{x, f, 0, nfev, 0};
    } else {
#ifdef NEMO_LO_TRACE
      const long long tl0 = clock64();
#endif
      int task = ls.step(stp, f, g * d);
#ifdef NEMO_LO_TRACE
      { const double keep = stp; asm volatile("" :: "v"(keep)); }
      lb::trace_ls(fg, clock64() - tl0, 0);
#endif
      if (uni(task == 0)) {
        ++ifun;
        if (uni(ifun - 1 < o.maxls)) {
          x_eval = (stp == 1.0) ? z : stp * d + xk;
          continue;
        }
        task = -1;  // iback >= maxls
      }
      if (uni(task < 0)) {
        x = xk; f = fold; g = gold;
        if (uni(!have_pair)) return LbfgsResult{x, f, nit, nfev, 2};
        have_pair = false;
        theta = 1.0;
      } else {
        ++nit;
        if (uni(fabs(lb::projg<BOUNDED>(x, g, has_lo, lo, has_hi, hi)) <= o.gtol)) return LbfgsResult{x, f, nit, nfev, 0};
        if (uni((fold - f) <= tol * dmax(dmax(fabs(fold), fabs(f)), 1.0)))
          return LbfgsResult{x, f, nit, nfev, 1};
        if (uni(nit >= o.maxiter || nfev > o.maxfun)) return LbfgsResult{x, f, nit, nfev, 3};
        const double gd = g * d;
        const double r = g - gold;
        const double rr = r * r;
        double dr, ddum, s;
        if (stp == 1.0) { dr = gd - gdold; ddum = -gdold; s = d; }
        else { dr = (gd - gdold) * stp; s = d * stp; ddum = -gdold * stp; }
        if (uni(!(dr <= kEpsMch * ddum))) {
          have_pair = true;
          s_last = s;
          y_last = r;
          theta = rr / dr;
        }
      }
    }
    // ---- next search direction and line-search start (restarts loop here)
    for (;;) {
      double dtm;
      if (have_pair) { dtm = s_last / y_last; z = x + (-g) * dtm; }
      else { dtm = 1.0 / theta; z = x + dtm * (-g); }
      if (BOUNDED && g != 0.0) {
        // cauchy: the bound is the one breakpoint along -g
        if (g > 0.0 && has_lo) { if (!(dtm < (x - lo) / g)) z = lo; }
        else if (g < 0.0 && has_hi) { if (!(dtm < (hi - x) / (-g))) z = hi; }
      }
      d = z - x;
      const double dnorm = sqrt(d * d);
      double stpmx = kStpMax;
      if (BOUNDED) {
        if (nit == 0) {
          stpmx = 1.0;
        } else if (d < 0.0 && has_lo) {
          const double a2 = lo - x;
          if (a2 >= 0.0) stpmx = 0.0;
          else if (d * stpmx < a2) stpmx = a2 / d;
        } else if (d > 0.0 && has_hi) {
          const double a2 = hi - x;
          if (a2 <= 0.0) stpmx = 0.0;
          else if (d * stpmx > a2) stpmx = a2 / d;
        }
      }
      stp = (nit == 0 && !boxed) ? dmin(1.0 / dnorm, stpmx) : 1.0;
      xk = x; fold = f; gold = g;
      gdold = g * d;
      if (uni(gdold < 0.0)) {
        ls.stpmax = stpmx;
        ls.start(stp, f, gdold);
        ifun = 1;
        in_ls = true;
        x_eval = (stp == 1.0) ? z : stp * d + xk;
        break;
      }
      if (uni(!have_pair)) return LbfgsResult{x, f, nit, nfev, 2};
      have_pair = false;
      theta = 1.0;
    }
  }
}

// the reference's unbounded call (nem_order_mcmc.py:167)
template <class FG>
__device__ __forceinline__ LbfgsResult lbfgsb1_minimize(FG& fg, double x0) {
  return lbfgsb1_minimize_opts<false, false>(fg, x0, LbOpts{});
}

}  // namespace nemo
