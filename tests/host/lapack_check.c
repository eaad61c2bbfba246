// scipy.linalg.inv's LAPACK calls (getrf + getri of scipy's OpenBLAS 0.3.28,
// SkylakeX kernels) as csrc/nemo_ancestor.hip restates them, run sequentially
// on the host and compared bit for bit with the library itself (dlopen'ed):
// the LU factors and pivots for n = 1..128, the inverse for n = 1..64 (the
// device path's range).  Build with -ffp-contract=off: every fused operation
// is an explicit fma().
//   lapack_check <path to libscipy_openblas*.so> [trials]
#include <dlfcn.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { LD = 128 };
static double at_buf[LD * LD];
#define A(r, c) a[(r) + (c) * (long)lda]

// ddot_k, x strided (a panel row), y unit
static double ddot_row(int n, const double* x, int incx, const double* y) {
  double t1 = 0, t2 = 0;
  int i = 0, n1 = n & -4;
  for (; i < n1; i += 4) {
    double m3 = y[i + 2] * x[(i + 2) * incx], m4 = y[i + 3] * x[(i + 3) * incx];
    t1 = t1 + fma(y[i], x[i * incx], m3);
    t2 = t2 + fma(y[i + 1], x[(i + 1) * incx], m4);
  }
  for (; i < n; ++i) t1 = fma(y[i], x[i * incx], t1);
  return t1 + t2;
}

// dgemv_n, alpha -1, beta 1, unit strides
static void gemv_n_m1(int m, int n, const double* a, int lda, const double* x, double* y) {
  int mb = m - (m & 3);
  for (int i = 0; i < m; ++i) {
    double yi = y[i];
    int c = 0;
    if (i < mb) {
      for (; c + 4 <= n; c += 4) {
        double t = A(i, c + 1) * x[c + 1];
        t = fma(A(i, c), x[c], t);
        t = fma(A(i, c + 2), x[c + 2], t);
        t = fma(A(i, c + 3), x[c + 3], t);
        yi = fma(t, -1.0, yi);
      }
      if (n - c >= 2) {
        double t = A(i, c + 1) * x[c + 1];
        t = fma(A(i, c), x[c], t);
        yi = fma(t, -1.0, yi);
        c += 2;
      }
      for (; c < n; ++c) {
        double xa = x[c] * -1.0;
        yi = yi + A(i, c) * xa;
      }
    } else {
      double t = 0;
      for (; c < n; ++c) t = fma(A(i, c), x[c], t);
      yi = fma(t, -1.0, yi);
    }
    y[i] = yi;
  }
}

static void getf2(int S, double* a, int lda, int* piv, int off, int n) {
  int m = S - off;
  for (int jl = 0; jl < n; ++jl) {
    double* b = &A(off, off + jl);
    int jm = jl < m ? jl : m;
    for (int i = 0; i < jm; ++i) {
      int ip = piv[off + i] - 1 - off;
      if (ip != i) { double t = b[i]; b[i] = b[ip]; b[ip] = t; }
    }
    for (int i = 1; i < jm; ++i) b[i] = b[i] - ddot_row(i, &A(off + i, off), lda, b);
    if (jl < m) {
      gemv_n_m1(m - jl, jl, &A(off + jl, off), lda, b, b + jl);
      int jp = jl;
      double mx = fabs(b[jl]);
      for (int i = jl + 1; i < m; ++i)
        if (fabs(b[i]) > mx) { mx = fabs(b[i]); jp = i; }
      piv[off + jl] = off + jp + 1;
      double t1 = b[jp];
      if (t1 != 0.0) {
        if (jp != jl)
          for (int k = 0; k <= jl; ++k) { double t = A(off + jl, off + k); A(off + jl, off + k) = A(off + jp, off + k); A(off + jp, off + k) = t; }
        double r = 1.0 / t1;
        for (int i = jl + 1; i < m; ++i) b[i] *= r;
      }
    }
  }
}

static void laswp(double* a, int lda, const int* piv, int r0, int r1, int c0, int c1) {
  for (int c = c0; c < c1; ++c)
    for (int r = r0; r < r1; ++r) {
      int ip = piv[r] - 1;
      if (ip != r) { double t = A(r, c); A(r, c) = A(ip, c); A(ip, c) = t; }
    }
}

static void trsm(double* a, int lda, int d, int jb, int c0, int c1) {
  for (int col = c0; col < c1; ++col) {
    double* x = &A(d, col);
    for (int r0 = 0; r0 < jb;) {
      int rest = jb - r0, mb = rest >= 16 ? 16 : (rest & 8) ? 8 : (rest & 4) ? 4 : (rest & 2) ? 2 : 1;
      if (r0 > 0)
        for (int r = r0; r < r0 + mb; ++r) {
          double acc = 0;
          for (int k = 0; k < r0; ++k) acc = fma(A(d + r, d + k), x[k], acc);
          x[r] = x[r] - acc;
        }
      for (int i = r0; i < r0 + mb; ++i) {
        double bb = x[i];
        for (int k = i + 1; k < r0 + mb; ++k) x[k] = fma(-bb, A(d + k, d + i), x[k]);
      }
      r0 += mb;
    }
  }
}

static void gemm(int S, double* a, int lda, int d, int jb, int R0, int C0, int C1) {
  int M = S - R0, N = C1 - C0;
  if (M <= 0 || N <= 0) return;
  int r8 = (M & ~15) + (M & 8), r4 = r8 + (M & 4), n12 = N - N % 12;
  for (int jc = 0; jc < N; ++jc)
    for (int ii = 0; ii < M; ++ii) {
      int split = (jc >= n12 || ii < r8) ? 1 : ii < r4 ? 2 : 4;
      double p[4] = {0, 0, 0, 0};
      int k = 0, kk = jb - jb % split;
      for (; k < kk; ++k) p[k % split] = fma(A(R0 + ii, d + k), A(d + k, C0 + jc), p[k % split]);
      double acc = split == 1 ? p[0] : split == 2 ? p[0] + p[1] : (p[0] + p[1]) + (p[2] + p[3]);
      for (; k < jb; ++k) acc = fma(A(R0 + ii, d + k), A(d + k, C0 + jc), acc);
      A(R0 + ii, C0 + jc) = fma(acc, -1.0, A(R0 + ii, C0 + jc));
    }
}

static void getrf(int S, double* a, int lda, int* piv, int off, int nn) {
  int m = S - off, mn = m < nn ? m : nn;
  if (m <= 0 || nn <= 0) return;
  int blocking = ((mn / 2 + 1) / 2) * 2;
  if (blocking <= 4) { getf2(S, a, lda, piv, off, nn); return; }
  for (int j = 0; j < mn; j += blocking) {
    int jb = mn - j < blocking ? mn - j : blocking;
    getrf(S, a, lda, piv, off + j, jb);
    if (j + jb < nn) {
      laswp(a, lda, piv, off + j, off + j + jb, off + j + jb, off + nn);
      trsm(a, lda, off + j, jb, off + j + jb, off + nn);
      gemm(S, a, lda, off + j, jb, off + j + jb, off + j + jb, off + nn);
    }
  }
  for (int j = 0; j < mn; j += blocking) {
    int jb = mn - j < blocking ? mn - j : blocking;
    laswp(a, lda, piv, off + j + jb, off + mn, off + j, off + j + jb);
  }
}

static void getri(int n, double* a, int lda, const int* piv) {
  double work[LD];
  for (int j = 0; j < n; ++j) {   // trti2_UN
    double ajj = 1.0 / A(j, j), v[LD];
    for (int r = 0; r < j; ++r) {
      double acc = A(r, j) * A(r, r);
      for (int i = r + 1; i < j; ++i) acc = fma(A(i, j), A(r, i), acc);
      v[r] = acc * -ajj;
    }
    for (int r = 0; r < j; ++r) A(r, j) = v[r];
    A(j, j) = ajj;
  }
  for (int j = n - 1; j >= 0; --j) {
    for (int i = j + 1; i < n; ++i) { work[i] = A(i, j); A(i, j) = 0.0; }
    if (j < n - 1) gemv_n_m1(n, n - 1 - j, &A(0, j + 1), lda, work + j + 1, &A(0, j));
  }
  for (int j = n - 2; j >= 0; --j) {
    int jp = piv[j] - 1;
    if (jp != j)
      for (int i = 0; i < n; ++i) { double t = A(i, j); A(i, j) = A(i, jp); A(i, jp) = t; }
  }
}

static double rnd(void) { return (double)rand() / RAND_MAX * 2 - 1; }

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: lapack_check <libscipy_openblas.so> [trials]\n"); return 2; }
  void* L = dlopen(argv[1], RTLD_NOW);
  if (!L) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
  void (*dgetrf)(int*, int*, double*, int*, int*, int*) = (void (*)(int*, int*, double*, int*, int*, int*))dlsym(L, "scipy_dgetrf_");
  void (*dgetri)(int*, double*, int*, int*, double*, int*, int*) = (void (*)(int*, double*, int*, int*, double*, int*, int*))dlsym(L, "scipy_dgetri_");
  if (!dgetrf || !dgetri) { fprintf(stderr, "no scipy_dgetrf_ / scipy_dgetri_\n"); return 2; }
  int trials = argc > 2 ? atoi(argv[2]) : 20, bad = 0;
  static double X[LD * LD], Y[LD * LD], W[LD * 80];
  static int p1[LD], p2[LD];
  (void)at_buf;
  srand(12345);
  for (int n = 1; n <= LD; ++n)
    for (int t = 0; t < trials; ++t) {
      // I - W~ of a random order (a DAG's strict triangle under a permutation),
      // with stale entries elsewhere on odd trials
      for (int i = 0; i < n * n; ++i) X[i] = 0.0;
      for (int i = 0; i < n; ++i)
        for (int k = 0; k < n; ++k) {
          if (i == k) continue;
          int pi = (i * 37 + t) % n, pk = (k * 37 + t) % n;   // a permutation when gcd(37, n) = 1
          if (pk < pi || ((t & 1) && rand() % 7 == 0)) X[i + k * n] = -1.0 / (1.0 + exp(-4 * rnd()));
        }
      for (int i = 0; i < n; ++i) X[i + i * n] = 1.0;
      memcpy(Y, X, sizeof(double) * n * n);
      int info;
      dgetrf(&n, &n, X, &n, p1, &info);
      getrf(n, Y, n, p2, 0, n);
      for (int i = 0; i < n * n; ++i) bad += memcmp(&X[i], &Y[i], 8) != 0;
      for (int i = 0; i < n; ++i) bad += p1[i] != p2[i];
      if (n <= 64 && info == 0) {
        int lwork = (int)(1.01 * 64 * n);
        dgetri(&n, X, &n, p1, W, &lwork, &info);
        getri(n, Y, n, p2);
        for (int i = 0; i < n * n; ++i) bad += memcmp(&X[i], &Y[i], 8) != 0;
      }
      if (bad) { printf("n=%d trial %d: %d differing values\n", n, t, bad); return 1; }
    }
  printf("ok\n");
  return 0;
}
