// Host check of refmath.h against the libraries it restates, bit for bit:
// glibc's exp / log1p (called directly), and numpy's bundled SVML
// __svml_log8_ha / __svml_exp8_ha (dlopen'ed from numpy's _multiarray_umath,
// AVX-512 vector ABI).  N inputs per range (argv[2], default 10^6), each range
// drawn from where the path's arguments live.  Exit status 0 iff every value
// is bit-identical.
//
//   g++ -O2 -mavx512f -mfma -ffp-contract=off -fno-builtin -I<csrc> refmath_check.cpp -ldl -o rc
//   ./rc <path of _multiarray_umath.so> [N]
#include <dlfcn.h>
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "refmath.h"

using namespace nemo::refmath;
typedef __m512d (*svml_fn)(__m512d);

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64() {
  s_state ^= s_state << 13;
  s_state ^= s_state >> 7;
  s_state ^= s_state << 17;
  return s_state;
}
static double uni(double lo, double hi) { return lo + (hi - lo) * ((next_u64() >> 11) * 0x1p-53); }
static double loguni(double lo, double hi) { return exp(uni(log(lo), log(hi))); }

struct Stat {
  long n = 0, bad = 0;
  double first = 0;
};

static void report(const char* name, const Stat& s, int& fails) {
  printf("%-34s %10ld inputs  %ld differ%s", name, s.n, s.bad, s.bad ? "" : "\n");
  if (s.bad) printf("  (first at %.17g)\n", s.first);
  if (s.bad) fails++;
}

template <class Gen>
static Stat check_scalar(double (*ref)(double), double (*mine)(double), Gen gen, long n) {
  Stat s;
  for (long i = 0; i < n; ++i) {
    const double x = gen();
    const double a = ref(x), b = mine(x);
    if (memcmp(&a, &b, 8) != 0 && !(a != a && b != b)) {
      if (!s.bad) s.first = x;
      s.bad++;
    }
    s.n++;
  }
  return s;
}

template <class Gen>
static Stat check_svml(svml_fn f, double (*mine)(double), Gen gen, long n) {
  Stat s;
  double in[8], out[8];
  for (long i = 0; i < n; i += 8) {
    for (int l = 0; l < 8; ++l) in[l] = gen();
    _mm512_storeu_pd(out, f(_mm512_loadu_pd(in)));
    for (int l = 0; l < 8; ++l) {
      const double b = mine(in[l]);
      if (memcmp(&out[l], &b, 8) != 0) {
        if (!s.bad) s.first = in[l];
        s.bad++;
      }
      s.n++;
    }
  }
  return s;
}

static double libm_exp(double x) { return exp(x); }
static double libm_log1p(double x) { return log1p(x); }
static double my_exp(double x) { return glibc_exp(x); }
static double my_log1p(double x) { return glibc_log1p(x); }
static double my_log1p_unit(double x) { return log1p_unit(x); }
// npymath's npy_logaddexp over libm's exp / log1p
static double npy_logaddexp(double x, double y) {
  if (x == y) return x + 0.693147180559945309417232121458176568;
  const double tmp = x - y;
  if (tmp > 0) return x + log1p(exp(-tmp));
  if (tmp <= 0) return y + log1p(exp(tmp));
  return tmp;
}
static Stat check_lae(long n, double lo, double hi, double spread) {
  Stat s;
  for (long i = 0; i < n; ++i) {
    const double x = uni(lo, hi);
    double y = x + uni(-spread, spread);
    if ((next_u64() & 15) == 0) y = x;
    const double a = npy_logaddexp(x, y), b = logaddexp(x, y);
    if (memcmp(&a, &b, 8) != 0) {
      if (!s.bad) s.first = x;
      s.bad++;
    }
    s.n++;
  }
  return s;
}
static double my_slog(double x) { return svml_log(x); }
static double my_sexp(double x) { return svml_exp(x); }

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <_multiarray_umath.so> [N]\n", argv[0]);
    return 2;
  }
  const long n = argc > 2 ? atol(argv[2]) : 1000000;
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  svml_fn slog = (svml_fn)dlsym(h, "__svml_log8_ha"), sexp = (svml_fn)dlsym(h, "__svml_exp8_ha");
  if (!slog || !sexp) {
    fprintf(stderr, "SVML symbols not found\n");
    return 2;
  }
  int fails = 0;
  report("glibc exp  [-745, 710]", check_scalar(libm_exp, my_exp, [] { return uni(-745, 710); }, n), fails);
  report("glibc exp  [-40, 40] (expit)", check_scalar(libm_exp, my_exp, [] { return uni(-40, 40); }, n), fails);
  report("glibc exp  |x| in [1e-20, 1]", check_scalar(libm_exp, my_exp, [] {
           return (next_u64() & 1 ? 1 : -1) * loguni(1e-20, 1); }, n), fails);
  report("glibc log1p (0, 1] (logaddexp)", check_scalar(libm_log1p, my_log1p, [] { return loguni(1e-300, 1); }, n), fails);
  report("glibc log1p (-1, 100]", check_scalar(libm_log1p, my_log1p, [] { return uni(-0.999999, 100); }, n), fails);
  report("log1p_unit (0, 1]", check_scalar(libm_log1p, my_log1p_unit, [] { return loguni(1e-300, 1); }, n), fails);
  report("log1p_unit [0.4, 1]", check_scalar(libm_log1p, my_log1p_unit, [] { return uni(0.4, 1.0); }, n), fails);
  report("log1p_unit sqrt(2) - 1 +- 1e-5", check_scalar(libm_log1p, my_log1p_unit, [] { return uni(0.41420, 0.41424); }, n), fails);
  report("log1p_unit 1 - [0, 1e-15]", check_scalar(libm_log1p, my_log1p_unit, [] { return 1.0 - uni(0, 1e-15); }, n), fails);
  report("logaddexp spread 5", check_lae(n, -3000, 0, 5), fails);
  report("logaddexp spread 800", check_lae(n, -3000, 0, 800), fails);
  report("logaddexp spread 1e-14", check_lae(n, -100, 100, 1e-14), fails);
  report("svml log  [1, 1e6] (1 + c e)", check_svml(slog, my_slog, [] { return loguni(1, 1e6); }, n), fails);
  report("svml log  [1e-3, 10]", check_svml(slog, my_slog, [] { return loguni(1e-3, 10); }, n), fails);
  report("svml log  1 + [1e-12, 1e-2]", check_svml(slog, my_slog, [] { return 1.0 + loguni(1e-12, 1e-2); }, n), fails);
  report("svml log  [1e-300, 1e300]", check_svml(slog, my_slog, [] { return loguni(1e-300, 1e300); }, n), fails);
  report("svml exp  [-707, 707]", check_svml(sexp, my_sexp, [] { return uni(-707, 707); }, n), fails);
  report("svml exp  [-50, 0] (order weights)", check_svml(sexp, my_sexp, [] { return uni(-50, 0); }, n), fails);
  report("svml exp  |x| in [1e-20, 1]", check_svml(sexp, my_sexp, [] {
           return (next_u64() & 1 ? 1 : -1) * loguni(1e-20, 1); }, n), fails);
  return fails ? 1 : 0;
}
