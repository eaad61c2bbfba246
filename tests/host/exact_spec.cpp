// The bit-exact local optimum of the reference (refmath.h objective +
// lbfgsb_exact.h control) compiled for the HOST, as a ctypes library for
// tests/test_exact_spec.py: the same source the device kernels instantiate,
// checked against scipy's records and the reference's trajectories on the CPU.
//   hipcc -O2 -fPIC -shared -ffp-contract=off -I<csrc> exact_spec.cpp -o libexact_spec.so
#include <stdint.h>

#include "lbfgsb_exact.h"
#include "refmath.h"

using namespace nemo;

// numpy's pairwise summation (DOUBLE_pairwise_sum, PW_BLOCKSIZE 128)
static double pairwise_sum(const double* a, long n) {
#pragma clang fp contract(off)
  if (n < 8) {
    double res = 0.0;
    for (long i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128) {
    double r[8];
    for (int k = 0; k < 8; ++k) r[k] = a[k];
    long i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int k = 0; k < 8; ++k) r[k] += a[i + k];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  long n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

// local_ll_sum_penalized (nem_order_mcmc.py:18-23) as numpy evaluates it
static double objective(const double* c, int E, double anc, double x, double* buf) {
#pragma clang fp contract(off)
  const double ex = refmath::expit(x);
  for (int e = 0; e < E; ++e) buf[e] = refmath::svml_log(c[e] * ex + 1.0);
  const double temp1 = -pairwise_sum(buf, E);
  const double temp2 = __builtin_fabs(ex - anc);
  return (temp1 + temp2) + ex * (1.0 - ex);
}

struct HostFG {
  const double* c;
  int E;
  double anc;
  double* buf;
  void operator()(double x, double x1, double& f0, double& f1) {
    f0 = objective(c, E, anc, x, buf);
    f1 = objective(c, E, anc, x1, buf);
  }
};

extern "C" {

int spec_local_opt(int n, int E, const double* c, const double* anc, const double* x0, double* xstar,
                   double* fstar, int32_t* nit, int32_t* nfev, int32_t* status) {
  double* buf = new double[E];
  double mem[lbx::kMemDoubles];
  for (int k = 0; k < n; ++k) {
    HostFG fg{c + (long)k * E, E, anc[k], buf};
    const LbfgsResult r = lbfgsb1_minimize_exact(fg, x0[k], lbx::Mem{mem});
    xstar[k] = r.x;
    fstar[k] = r.f;
    nit[k] = r.nit;
    nfev[k] = r.nfev;
    status[k] = r.status;
  }
  delete[] buf;
  return 0;
}

double spec_objective(int E, const double* c, double anc, double x) {
  double* buf = new double[E];
  const double f = objective(c, E, anc, x, buf);
  delete[] buf;
  return f;
}

void spec_svml_log(long n, const double* x, double* y) {
  for (long i = 0; i < n; ++i) y[i] = refmath::svml_log(x[i]);
}
void spec_svml_exp(long n, const double* x, double* y) {
  for (long i = 0; i < n; ++i) y[i] = refmath::svml_exp(x[i]);
}
void spec_expit(long n, const double* x, double* y) {
  for (long i = 0; i < n; ++i) y[i] = refmath::expit(x[i]);
}
void spec_logaddexp(long n, const double* x, const double* y, double* z) {
  for (long i = 0; i < n; ++i) z[i] = refmath::logaddexp(x[i], y[i]);
}
double spec_pairwise_sum(long n, const double* a) { return pairwise_sum(a, n); }

}  // extern "C"
