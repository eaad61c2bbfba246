// lbfgsb_exact.h -- scipy 1.15's L-BFGS-B for ONE unbounded variable with
// the compact-form arithmetic it actually runs, bit for bit.
//
// lbfgsb1.h reduces the compact L-BFGS matrix to its 1-D value y/s: the same
// iteration path, but not the same bits (1538 of 2211 net2 optima bit-equal
// even with numpy's own objective).  This is the other form: mainlb / matupd
// / formt / formk / cmprlb / subsm of the C translation in scipy 1.15
// (__lbfgsb.c, L-BFGS-B 3.0, m = 10), specialised to n = 1 with every
// variable free, and the OpenBLAS 0.3.28 kernels it calls (SkylakeX, the
// kernels the build container's and the GPU box host's scipy select:
// tools/host_blas_probe.py) restated operation for operation:
//   * ddot: a fused multiply-add chain from 0 for n < 16, the 4 x 4-lane
//     AVX kernel for the first 16 (dot_compute, ddot_k_SKYLAKEX);
//   * dpotrf('U'), n <= 16: potf2_U -- ajj = a_jj - ddot, sqrt, then the row
//     by dgemv_t (dgemv_t_4.c: 4-row blocks in FMA lanes summed (0+2)+(1+3),
//     unfused 2-lane kernels for the odd columns, the 1-3 remainder rows with
//     alpha folded into x) and a scale by 1/ajj;
//   * dtrtrs('U', 'T' | 'N', 'N') with one right-hand side: trsv (divisions;
//     'T' by ddot, 'N' by fused axpy); with several ('T', formk's one call
//     for the (1,2) block): trsm with the inverted diagonal, rows in blocks of
//     the 16-row unroll and its power-of-two remainders, a fused dot of the
//     solved rows ahead of each block;
//   * dnrm2 (x87): |d| for n = 1.
// Every product of the 1-D compact form that the library stores (S'Y, S'S,
// Y'Y, R_z) is one rounded product of two stored scalars, so only the
// diagonals (s's, s'y), the s / y rings and the factored WN are kept: 540
// doubles in `mem` (LDS per wave on the device), with subsm's work vector.
// Host check: tools/lbfgsb_proto.py found the form (the library's own
// routines, 2571 / 2571 reference optima bit-equal); tests/test_exact_spec.py
// runs THIS header on the CPU against the same records.
#pragma once

#include "lbfgsb1.h"

namespace nemo {
namespace lbx {

using lb::dmax;
using lb::dmin;
using lb::uni;

constexpr int kM = 10;          // scipy's default memory
constexpr int kLdN = 2 * kM;    // WN's leading dimension (m2)
constexpr int kLdT = kM;        // WT's
constexpr int kMemDoubles = 4 * kM + kLdN * kLdN + kLdT * kLdT + 2 * kM;

// mem layout (doubles): ws[m] wy[m] ssd[m] syd[m] wn[2m x 2m] wt[m x m] wv[2m]
struct Mem {
  double* p;
  NEMO_LB double& ws(int i) { return p[i]; }
  NEMO_LB double& wy(int i) { return p[kM + i]; }
  NEMO_LB double& ssd(int i) { return p[2 * kM + i]; }
  NEMO_LB double& syd(int i) { return p[3 * kM + i]; }
  NEMO_LB double* wn() { return p + 4 * kM; }
  NEMO_LB double* wt() { return p + 4 * kM + kLdN * kLdN; }
  NEMO_LB double* wv() { return p + 4 * kM + kLdN * kLdN + kLdT * kLdT; }
};

NEMO_LB double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

// OpenBLAS ddot_k_SKYLAKEX, unit strides, n < 32
NEMO_LB double ob_ddot(int n, const double* x, const double* y) {
#pragma clang fp contract(off)
  double dot = 0.0;
  int i = 0;
  if (n >= 16) {
    double a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0}, a2[4] = {0, 0, 0, 0}, a3[4] = {0, 0, 0, 0};
    for (int l = 0; l < 4; ++l) {
      a0[l] = fma_(x[l], y[l], a0[l]);
      a1[l] = fma_(x[4 + l], y[4 + l], a1[l]);
      a2[l] = fma_(x[8 + l], y[8 + l], a2[l]);
      a3[l] = fma_(x[12 + l], y[12 + l], a3[l]);
    }
    double t[4];
    for (int l = 0; l < 4; ++l) t[l] = ((a0[l] + a1[l]) + a2[l]) + a3[l];
    dot = (t[0] + t[2]) + (t[1] + t[3]);
    i = 16;
  }
  for (; i < n; ++i) dot = fma_(y[i], x[i], dot);
  return dot;
}

// OpenBLAS dgemv_t_SKYLAKEX with alpha = -1: y[k * incy] += -(A(:, k)' x),
// A m x n column-major (lda), m < 2048
NEMO_LB void ob_gemv_t_m1(int m, int n, const double* a, int lda, const double* x, double* y, int incy) {
#pragma clang fp contract(off)
  const int m3 = m & 3, nb = m - m3;
  int c = 0;
  if (nb > 0) {
    const int n1 = n >> 2, n2 = n & 3;
    for (int g = 0; g < n1 * 4; ++g, ++c) {  // dgemv_kernel_4x4: per-column FMA lanes
      const double* col = a + (long)c * lda;
      double acc[4] = {0, 0, 0, 0};
      int i = 0;
      if (nb & 4) {
        for (int l = 0; l < 4; ++l) acc[l] = fma_(x[l], col[l], acc[l]);
        i = 4;
      }
      for (; i < nb; i += 8) {
        for (int l = 0; l < 4; ++l) acc[l] = fma_(x[i + l], col[i + l], acc[l]);
        for (int l = 0; l < 4; ++l) acc[l] = fma_(x[i + 4 + l], col[i + 4 + l], acc[l]);
      }
      const double t = (acc[0] + acc[2]) + (acc[1] + acc[3]);
      y[c * incy] = fma_(t, -1.0, y[c * incy]);  // add_y (exact for alpha = -1 either way)
    }
    if (n2 & 2) {  // dgemv_kernel_4x2: unfused 2-lane sums
      for (int q = 0; q < 2; ++q, ++c) {
        const double* col = a + (long)c * lda;
        double acc0 = 0.0, acc1 = 0.0;
        for (int i = 0; i < nb; i += 4) {
          acc0 = acc0 + x[i] * col[i];
          acc1 = acc1 + x[i + 1] * col[i + 1];
          acc0 = acc0 + x[i + 2] * col[i + 2];
          acc1 = acc1 + x[i + 3] * col[i + 3];
        }
        y[c * incy] = fma_(acc0 + acc1, -1.0, y[c * incy]);
      }
    }
    if (n2 & 1) {  // dgemv_kernel_4x1: two 2-lane accumulators
      const double* col = a + (long)c * lda;
      double p0 = 0.0, p1 = 0.0, q0 = 0.0, q1 = 0.0;
      for (int i = 0; i < nb; i += 4) {
        p0 = p0 + col[i] * x[i];
        p1 = p1 + col[i + 1] * x[i + 1];
        q0 = q0 + col[i + 2] * x[i + 2];
        q1 = q1 + col[i + 3] * x[i + 3];
      }
      y[c * incy] = fma_((p0 + q0) + (p1 + q1), -1.0, y[c * incy]);
      ++c;
    }
  }
  if (m3) {  // the last m3 rows, x pre-scaled by alpha
    const int r = nb;
    const double xt0 = -x[r], xt1 = m3 > 1 ? -x[r + 1] : 0.0, xt2 = m3 > 2 ? -x[r + 2] : 0.0;
    for (int k = 0; k < n; ++k) {
      const double* col = a + (long)k * lda + r;
      if (m3 == 1) {
        y[k * incy] = fma_(col[0], xt0, y[k * incy]);
      } else {
        double t = fma_(col[0], xt0, col[1] * xt1);
        if (m3 == 3) t = fma_(col[2], xt2, t);
        y[k * incy] = t + y[k * incy];
      }
    }
  }
}

// OpenBLAS dpotrf('U') for n <= 16 (potf2_U); returns info (0 or j + 1)
NEMO_LB int ob_potrf_u(int n, double* a, int lda) {
#pragma clang fp contract(off)
  for (int j = 0; j < n; ++j) {
    double* cj = a + (long)j * lda;
    double ajj = cj[j] - ob_ddot(j, cj, cj);
    if (uni(ajj <= 0.0)) {   // potf2: a NaN goes on to the square root
      cj[j] = ajj;
      return j + 1;
    }
    ajj = __builtin_sqrt(ajj);
    cj[j] = ajj;
    const int i = n - j - 1;
    if (i > 0) {
      if (j > 0) ob_gemv_t_m1(j, i, a + (long)(j + 1) * lda, lda, cj, cj + j + lda, lda);
      const double inv = 1.0 / ajj;
      for (int k = 0; k < i; ++k) cj[j + (long)(k + 1) * lda] = cj[j + (long)(k + 1) * lda] * inv;
    }
  }
  return 0;
}

// dtrtrs('U', 'T', 'N') with one right-hand side (trsv_TUN); 0 or the index
// + 1 of a zero diagonal (checked first, as dtrtrs does)
NEMO_LB int ob_trsv_tun(int n, const double* u, int ldu, double* b) {
#pragma clang fp contract(off)
  for (int i = 0; i < n; ++i)
    if (uni(u[i + (long)i * ldu] == 0.0)) return i + 1;
  for (int i = 0; i < n; ++i) {
    const double* ci = u + (long)i * ldu;
    if (i > 0) b[i] = b[i] - ob_ddot(i, ci, b);
    b[i] = b[i] / ci[i];
  }
  return 0;
}

// dtrtrs('U', 'N', 'N') with one right-hand side (trsv_NUN)
NEMO_LB int ob_trsv_nun(int n, const double* u, int ldu, double* b) {
#pragma clang fp contract(off)
  for (int i = 0; i < n; ++i)
    if (uni(u[i + (long)i * ldu] == 0.0)) return i + 1;
  for (int j = n - 1; j >= 0; --j) {
    const double* cj = u + (long)j * ldu;
    b[j] = b[j] / cj[j];
    const double nb = -b[j];
    for (int k = 0; k < j; ++k) b[k] = fma_(nb, cj[k], b[k]);
  }
  return 0;
}

// dtrtrs('U', 'T', 'N') with nrhs >= 2 (trsm_LTUN: the inverted diagonal,
// row blocks of 16 then 8, 4, 2, 1), n <= 16, B n x nrhs (ldb)
NEMO_LB int ob_trsm_lt(int n, int nrhs, const double* u, int ldu, double* b, int ldb) {
#pragma clang fp contract(off)
  for (int i = 0; i < n; ++i)
    if (uni(u[i + (long)i * ldu] == 0.0)) return i + 1;
  for (int j = 0; j < nrhs; ++j) {
    double* x = b + (long)j * ldb;
    int r0 = 0;
    for (int sz = 16; sz >= 1; sz >>= 1) {
      if (sz == 16 ? n < 16 : !(n & sz)) continue;
      if (r0 > 0)
        for (int r = r0; r < r0 + sz; ++r) {
          const double* cr = u + (long)r * ldu;
          double acc = 0.0;
          for (int k = 0; k < r0; ++k) acc = fma_(cr[k], x[k], acc);
          x[r] = x[r] - acc;
        }
      for (int i = r0; i < r0 + sz; ++i) {
        const double bb = x[i] * (1.0 / u[i + (long)i * ldu]);
        x[i] = bb;
        for (int k = i + 1; k < r0 + sz; ++k) x[k] = fma_(-bb, u[i + (long)k * ldu], x[k]);
      }
      r0 += sz;
    }
  }
  return 0;
}

// the stored products of the compact form (see the header)
NEMO_LB double prod0(double a, double b) { return fma_(a, b, 0.0); }   // ddot, n = 1
NEMO_LB double sum0(double a, double b) { return 0.0 + a * b; }        // C loop from zero

struct Ring {
  int col = 0, head = 0, itail = 0, iupdat = 0;
  NEMO_LB int p(int i) const { return (head + i) % kM; }   // logical i (0 = oldest) -> slot
};

// formt: T = theta SS + L D^-1 L' and its Cholesky factor; returns info
NEMO_LB int formt(Mem& mem, const Ring& rg, double theta) {
#pragma clang fp contract(off)
  const int col = rg.col;
  double* wt = mem.wt();
  auto sy = [&](int i, int k) { return i == k ? mem.syd(rg.p(i)) : prod0(mem.ws(rg.p(i)), mem.wy(rg.p(k))); };
  auto ss = [&](int i, int k) { return i == k ? mem.ssd(rg.p(i)) : prod0(mem.ws(rg.p(i)), mem.ws(rg.p(k))); };
  for (int j = 0; j < col; ++j) wt[(long)j * kLdT] = theta * ss(0, j);
  for (int i = 1; i < col; ++i)
    for (int j = i; j < col; ++j) {
      const int k1 = i < j ? i : j;
      double ddum = 0.0;
      for (int k = 0; k < k1; ++k) ddum = ddum + sy(i, k) * sy(j, k) / sy(k, k);
      wt[i + (long)j * kLdT] = ddum + theta * ss(i, j);
    }
  return ob_potrf_u(col, wt, kLdT);
}

// formk for n = nsub = 1, the variable free and staying free: WN (upper,
// 2col x 2col, ld 2m) and its two Cholesky factorisations; info 0, -1, -2
NEMO_LB int formk(Mem& mem, const Ring& rg, double theta) {
#pragma clang fp contract(off)
  const int col = rg.col;
  double* wn = mem.wn();
  auto at = [&](int r, int c) -> double& { return wn[r + (long)c * kLdN]; };
  for (int iy = 0; iy < col; ++iy) {
    const int is = col + iy;
    const double yi = mem.wy(rg.p(iy)), si = mem.ws(rg.p(iy));
    for (int jy = 0; jy <= iy; ++jy) {
      at(jy, iy) = sum0(yi, mem.wy(rg.p(jy))) / theta;   // Y'ZZ'Y / theta
      at(col + jy, is) = 0.0 * theta;                     // S'AA'S theta (no active set)
    }
    for (int jy = 0; jy < iy; ++jy) at(jy, is) = -0.0;   // -L_a
    for (int jy = iy; jy < col; ++jy) at(jy, is) = sum0(si, mem.wy(rg.p(jy)));   // R_z
    at(iy, iy) = at(iy, iy) + mem.syd(rg.p(iy));
  }
  if (ob_potrf_u(col, wn, kLdN) != 0) return -1;
  // L^-1 (-L_a' + R_z') in the (1,2) block: one dtrtrs call with nrhs = col
  double* b12 = wn + (long)col * kLdN;
  const int info = col == 1 ? ob_trsv_tun(1, wn, kLdN, b12) : ob_trsm_lt(col, col, wn, kLdN, b12, kLdN);
  if (info != 0) return -1;
  for (int is = col; is < 2 * col; ++is)
    for (int js = is; js < 2 * col; ++js)
      at(is, js) = at(is, js) + ob_ddot(col, wn + (long)is * kLdN, wn + (long)js * kLdN);
  if (ob_potrf_u(col, wn + col + (long)col * kLdN, kLdN) != 0) return -2;
  return 0;
}

// subsm from z = x with r = -g (cmprlb, unconstrained): the Newton step;
// false when a triangular solve is singular (the caller restarts)
NEMO_LB bool subsm(Mem& mem, const Ring& rg, double theta, double r, double x, double& z) {
#pragma clang fp contract(off)
  const int col = rg.col, c2 = 2 * col;
  double* wv = mem.wv();   // (a local array would live in per-lane scratch on the device)
  for (int i = 0; i < col; ++i) {
    wv[i] = sum0(mem.wy(rg.p(i)), r);
    wv[col + i] = theta * sum0(mem.ws(rg.p(i)), r);
  }
  const double* wn = mem.wn();
  if (ob_trsv_tun(c2, wn, kLdN, wv) != 0) return false;
  for (int i = 0; i < col; ++i) wv[i] = -wv[i];
  if (ob_trsv_nun(c2, wn, kLdN, wv) != 0) return false;
  double d = r;
  for (int jy = 0; jy < col; ++jy) {
    const int p = rg.p(jy);
    d = d + mem.wy(p) * wv[jy] / theta + mem.ws(p) * wv[col + jy];
  }
  d = d * (1.0 / theta);
  z = x + d;   // the projection step of L-BFGS-B 3.0 (no bounds: alpha = 1, same bits)
  return true;
}

}  // namespace lbx

// Minimise the reference's unbounded 1-D objective from x0 with scipy's
// exact arithmetic (header); fg as lbfgsb1_minimize.  Status as there.
template <class FG>
NEMO_LB LbfgsResult lbfgsb1_minimize_exact(FG& fg, double x0, lbx::Mem mem) {
#pragma clang fp contract(off)
  using namespace lb;
  using lbx::fma_;
  const double tol = (0.01 / kEpsMch) * kEpsMch;
  const double pgtol = 0.01;
  const int maxls = 20, maxiter = 15000, maxfun = 15000;
  int nfev = 0, nit = 0, ifun = 0;
  bool in_ls = false, updatd = false;
  lbx::Ring rg;
  double theta = 1.0;
  double x = x0, f = 0.0, g = 0.0;
  double z = 0.0, d = 0.0, stp = 0.0, xk = 0.0, fold = 0.0, gold = 0.0, gdold = 0.0, dtd = 0.0;
  double x_eval = x0;
  bool have_last = false;
  double x_last = 0.0, f_last = 0.0, g_last = 0.0;
  Dcsrch ls;
  auto restart = [&]() {
    rg = lbx::Ring{};
    theta = 1.0;
    updatd = false;
  };
  for (;;) {
    // ---- the single evaluation site (scipy's ScalarFunction memoises the
    // last point: a repeated x costs no evaluation)
    if (uni(!(have_last && x_eval == x_last))) {
      double h = 1e-8;
      if (uni((x_eval + h) - x_eval == 0.0))
        h = kSqrtEps * (x_eval >= 0.0 ? 1.0 : -1.0) * dmax(1.0, fabs(x_eval));
      const double x1 = x_eval + h;
      double f0, f1;
      fg(x_eval, x1, f0, f1);
      nfev += 2;
      f_last = f0;
      g_last = (f1 - f0) / (x1 - x_eval);
      have_last = true;
      x_last = x_eval;
    }
    x = x_eval;
    f = f_last;
    g = g_last;
    if (uni(!in_ls)) {
      if (uni(fabs(g) <= pgtol)) return LbfgsResult{x, f, 0, nfev, 0};
    } else {
      int task = ls.step(stp, f, lbx::prod0(g, d));
      if (uni(task == 0)) {
        ++ifun;
        if (uni(ifun - 1 < maxls)) {
          x_eval = (stp == 1.0) ? z : stp * d + xk;
          continue;
        }
        task = -1;
      }
      if (uni(task < 0)) {  // line search failed: previous iterate, restart or give up
        x = xk; f = fold; g = gold;
        if (uni(rg.col == 0)) return LbfgsResult{x, f, nit, nfev, 2};
        restart();
      } else {
        ++nit;
        if (uni(fabs(g) <= pgtol)) return LbfgsResult{x, f, nit, nfev, 0};
        if (uni((fold - f) <= tol * dmax(dmax(fabs(fold), fabs(f)), 1.0))) return LbfgsResult{x, f, nit, nfev, 1};
        if (uni(nit >= maxiter || nfev > maxfun)) return LbfgsResult{x, f, nit, nfev, 3};
        const double gd = lbx::prod0(g, d);
        const double r = g - gold;
        const double rr = lbx::prod0(r, r);
        double dr, ddum;
        if (stp == 1.0) { dr = gd - gdold; ddum = -gdold; }
        else { dr = (gd - gdold) * stp; d = d * stp; ddum = -gdold * stp; }
        if (uni(dr <= kEpsMch * ddum)) {
          updatd = false;
        } else {
          updatd = true;
          rg.iupdat += 1;
          if (rg.iupdat <= lbx::kM) {   // matupd
            rg.col = rg.iupdat;
            rg.itail = (rg.head + rg.iupdat - 1) % lbx::kM;
          } else {
            rg.itail = (rg.itail + 1) % lbx::kM;
            rg.head = (rg.head + 1) % lbx::kM;
          }
          mem.ws(rg.itail) = d;
          mem.wy(rg.itail) = r;
          theta = rr / dr;
          mem.ssd(rg.itail) = (stp == 1.0) ? dtd : stp * stp * dtd;
          mem.syd(rg.itail) = dr;
          if (uni(lbx::formt(mem, rg, theta) != 0)) restart();
        }
      }
    }
    // ---- the next search direction (cauchy at col = 0; else formk + subsm)
    for (;;) {
      if (uni(rg.col == 0)) {
        const double neggi = -g;
        const double f1 = 0.0 - neggi * neggi;
        const double f2 = -theta * f1;
        double dtm = -f1 / f2;
        if (dtm <= 0.0) dtm = 0.0;
        z = fma_(0.0 + dtm, neggi, x);   // daxpy
      } else {
        if (uni(updatd) && uni(lbx::formk(mem, rg, theta) != 0)) {
          restart();
          continue;
        }
        double zz = x;
        if (uni(!lbx::subsm(mem, rg, theta, -g, x, zz))) {
          restart();
          continue;
        }
        z = zz;
      }
      d = z - x;
      dtd = lbx::prod0(d, d);
      const double dnorm = fabs(d);    // dnrm2, n = 1
      stp = (nit == 0) ? dmin(1.0 / dnorm, kStpMax) : 1.0;
      xk = x; fold = f; gold = g;
      gdold = lbx::prod0(g, d);
      if (uni(gdold < 0.0)) {
        ls.stpmax = kStpMax;
        ls.start(stp, f, gdold);
        ifun = 1;
        in_ls = true;
        x_eval = (stp == 1.0) ? z : stp * d + xk;
        break;
      }
      // lnsrlb: the directional derivative is not negative (info = -4)
      if (uni(rg.col == 0)) return LbfgsResult{x, f, nit, nfev, 2};
      restart();
    }
  }
}

}  // namespace nemo
