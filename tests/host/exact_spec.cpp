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

extern "C" {

// compute_cell_ratios + calculate_ll (nem_order_mcmc.py:79-93) as numpy runs
// them, for one order: cells (S+1) x E, cs = logaddexp.reduce over the rows,
// ow = exp(cell - cs), ll = sum(cs) (Python's left fold); T is S x S x E,
// perm the order, w_raw S x S (expit applied here, as the reference does)
double spec_eval(int S, int E, const double* U, const double* T, const int32_t* perm, const double* w_raw,
                 double* cells, double* cs, double* ow) {
#pragma clang fp contract(off)
  int* pos = new int[S];
  for (int q = 0; q < S; ++q) pos[perm[q]] = q;
  for (long k = 0; k < (long)(S + 1) * E; ++k) cells[k] = U[k];
  for (int i = 0; i < S; ++i)
    for (int q = 0; q < pos[i]; ++q) {
      const int j = perm[q];
      const double s = refmath::expit(w_raw[(long)i * S + j]);
      const double oms = 1.0 - s;
      const double* t = T + ((long)i * S + j) * E;
      double* c = cells + (long)i * E;
      for (int e = 0; e < E; ++e) c[e] += refmath::svml_log(oms + s * refmath::svml_exp(t[e]));
    }
  double ll = 0.0;
  for (int e = 0; e < E; ++e) {
    double acc = cells[e];
    for (int r = 1; r <= S; ++r) acc = refmath::logaddexp(acc, cells[(long)r * E + e]);
    cs[e] = acc;
    ll = ll + acc;
  }
  for (int r = 0; r <= S; ++r)
    for (int e = 0; e < E; ++e) ow[(long)r * E + e] = refmath::svml_exp(cells[(long)r * E + e] - cs[e]);
  delete[] pos;
  return ll;
}

}  // extern "C"

#include "nemo_host.h"

extern "C" {

// host::build_pairwise_plan run as the device runs it (nemo_exact.hip's
// ExactObjective::sum_logs, lanes as arrays): numpy's pairwise sum of a[E]?
// Returns the sum, or NaN when the plan does not fit.
static double plan_sum(const nemo::host::PairwisePlan& pl, const double* a);

double spec_plan_sum(int E, const double* a) {
  nemo::host::PairwisePlan pl;
  if (!nemo::host::build_pairwise_plan(E, pl)) return __builtin_nan("");
  return plan_sum(pl, a);
}

// np.sum past one numpy buffer (E > 8192): the parts' plans, each run as the
// wave runs it, added in order (host::build_pairwise_parts)
double spec_parts_sum(int E, const double* a) {
#pragma clang fp contract(off)
  std::vector<nemo::host::PairwisePlan> parts;
  if (!nemo::host::build_pairwise_parts(E, parts)) return __builtin_nan("");
  double s = 0.0;
  for (size_t p = 0; p < parts.size(); ++p) {
    const double v = plan_sum(parts[p], a);
    s = p == 0 ? v : s + v;
  }
  return s;
}

static double plan_sum(const nemo::host::PairwisePlan& pl, const double* a) {
#pragma clang fp contract(off)
  const int NS = pl.ns;
  std::vector<double> res((size_t)NS * 64);
  for (int u = 0; u < NS; ++u) {
    double acc[64], tr[64];
    for (int l = 0; l < 64; ++l) {
      const size_t q = (size_t)u * 64 + l;
      const int st = pl.start[q], ct = pl.cnt[q];
      double v = ct > 0 ? a[st] : 0.0;
      for (int m = 1; m < ct; ++m) v = v + a[st + 8 * m];
      acc[l] = v;
      tr[l] = pl.rem[q] >= 0 ? a[pl.rem[q]] : 0.0;
    }
    for (int d : {1, 2, 4}) {
      double nx[64];
      for (int l = 0; l < 64; ++l) nx[l] = acc[l] + acc[l ^ d];
      for (int l = 0; l < 64; ++l) acc[l] = nx[l];
    }
    for (int l = 0; l < 64; ++l) {
      const int nr = pl.nrem[(size_t)u * 64 + l];
      for (int r = 0; r < nr; ++r) acc[l] = acc[l] + tr[(l & ~7) + r];
      res[(size_t)u * 64 + l] = acc[l];
    }
  }
  double v[64];
  for (int l = 0; l < 64; ++l) v[l] = (l >> 3) < NS ? res[(size_t)(l >> 3) * 64 + 8 * (l & 7)] : 0.0;
  for (int h = 0; h < pl.nh; ++h) {
    double nx[64];
    for (int l = 0; l < 64; ++l) {
      const int p = pl.partner[(size_t)h * 64 + l];
      nx[l] = p >= 0 ? v[l] + v[p] : v[l];
    }
    for (int l = 0; l < 64; ++l) v[l] = nx[l];
  }
  return v[0];
}

int spec_plan_shape(int E, int32_t* out4) {
  nemo::host::PairwisePlan pl;
  if (!nemo::host::build_pairwise_plan(E, pl)) return -1;
  out4[0] = pl.nleaf;
  out4[1] = pl.ns;
  out4[2] = pl.nh;
  out4[3] = pl.maxrem;
  return 0;
}

}  // extern "C"
