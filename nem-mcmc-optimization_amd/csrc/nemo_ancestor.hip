// nemo_ancestor.hip -- the step's ancestor_x on the device, in the reference's bits.
//
// get_optimal_weights(init=True) (nem_order_mcmc.py:172-208) starts every step with
//   W~ = expit_parent_weights(W)                  (:98-103, :152-157: expit on the
//                                                   permissible entries, the rest raw)
//   ancestor_x = clip(inv(I - W~) - I, 0, 1)      (:185)
// where inv is scipy.linalg.inv: LAPACK getrf + getri (scipy 1.15, lwork =
// 1.01 x getri's optimum) as built into scipy's OpenBLAS 0.3.28, SkylakeX kernels
// on this image and on the GPU box's host (tools/host_blas_probe.py).  One wave per
// chain restates, operation for operation, what those calls compute for S <= 64:
//  * getrf: OpenBLAS's recursive getrf_single (lapack/getrf/getrf_single.c): panel
//    width ((mn / 2 + 1) / 2) * 2, the unblocked getf2 (lapack/getf2/getf2.c) once
//    that width is <= 4 -- pivots of earlier columns, the strided ddot of the U part,
//    dgemv_n of the rest, idamax (first largest |.|), the row swap and the scale by
//    the pivot's reciprocal -- then per panel the row swaps (laswp), the unit lower
//    triangular solve (dtrsm_kernel_LT: row blocks of 16, then 8 / 4 / 2 / 1, each
//    the GEMM chain of the solved rows above it, then in-block fma(-b, l, x)) and the
//    trailing update (dgemm_kernel, alpha -1: rows in blocks of 16, 8, 4, 2, 1 and
//    columns in groups of 12; a 16- or 8-row block and the last n % 12 columns chain k,
//    a 4-row block accumulates even and odd k apart, a 2- or 1-row block the four
//    classes of k mod 4, the remainder of k chaining on the combined sum, C =
//    fma(acc, -1, C)); at the end the later panels' row swaps on the earlier columns.
//  * getri: reference LAPACK dgetri, unblocked because NB = 64 >= N: dtrtri ->
//    OpenBLAS trti2_UN (column j: 1 / u_jj, trmv_NUN as axpy's fma chain over the
//    inverted columns, scal by -1 / u_jj), then per column from the right the L
//    column into WORK, zeros, dgemv_n (alpha -1, beta 1), and the column swaps
//    j = N-2 .. 0.
//  * np.clip (numpy 2.2's SIMD loop: x < lo ? lo : x, then > hi ? hi : x, so
//    -0.0 stays -0.0) of inv - I.
// The restatement was derived against the library's own kernels on the host
// (tools/lapack_restate_check.c: 0 differing bits for n = 1..128 getrf and
// n = 1..64 getri) and the device build is compared with scipy.linalg.inv by
// tests/test_gpu_ancestor.py.
//
// Flags per chain (d_flag): 1 a zero pivot (scipy raises LinAlgError "singular
// matrix"), 2 a non-finite entry of I - W~ (scipy's check_finite raises
// ValueError), 4 a non-finite value in the factors or the inverse (the
// restatement is not held to the library's bits there: the host recomputes).
#include "nemo_internal.h"
#include "refmath.h"

namespace nemo {
namespace {

constexpr int kAncS = 64;   // one lane per row
constexpr int kLd = 65;     // LDS column stride in doubles: a lane per column, distinct banks

__device__ __forceinline__ double& at(double* a, int r, int c) { return a[r + c * kLd]; }

__device__ __forceinline__ double wave_fmax(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ int wave_imin(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

// ddot_k (SkylakeX, x strided): products of elements 2 and 3 of each group of
// four feed the fmas of elements 0 and 1 into two sums; the tail chains on the
// first; the sums add at the end.  x: a row of the panel (stride kLd), y: a column.
__device__ double ob_ddot_row(int n, const double* x, const double* y) {
  NEMO_RM_NOCONTRACT
  double t1 = 0.0, t2 = 0.0;
  int i = 0;
  const int n1 = n & -4;
  for (; i < n1; i += 4) {
    const double m3 = y[i + 2] * x[(i + 2) * kLd], m4 = y[i + 3] * x[(i + 3) * kLd];
    t1 = t1 + __builtin_fma(y[i], x[i * kLd], m3);
    t2 = t2 + __builtin_fma(y[i + 1], x[(i + 1) * kLd], m4);
  }
  for (; i < n; ++i) t1 = __builtin_fma(y[i], x[i * kLd], t1);
  return t1 + t2;
}

// row i of dgemv_n (SkylakeX, unit strides, alpha -1, beta 1) over `rows` rows and
// ncol columns: y + (-1) * sum_c A[i][c] x[c].  Rows below rows & ~3 take the
// 4-column kernel (t = a1 x1, fma a0 x0, a2 x2, a3 x3; y = fma(t, alpha, y)), a
// 2-column step when ncol % 4 >= 2 and unfused y + a (x alpha) for the last
// column; the rows & 3 last rows one fma chain then y = fma(t, alpha, y).
// arow: A[i][0] (stride kLd), x: the vector (LDS, uniform reads)
__device__ double ob_gemv_n_row(int i, int rows, int ncol, const double* arow, const double* x, double y) {
  NEMO_RM_NOCONTRACT
  const int mb = rows - (rows & 3);
  int c = 0;
  if (i < mb) {
    for (; c + 4 <= ncol; c += 4) {
      double t = arow[(c + 1) * kLd] * x[c + 1];
      t = __builtin_fma(arow[c * kLd], x[c], t);
      t = __builtin_fma(arow[(c + 2) * kLd], x[c + 2], t);
      t = __builtin_fma(arow[(c + 3) * kLd], x[c + 3], t);
      y = __builtin_fma(t, -1.0, y);
    }
    if (ncol - c >= 2) {
      double t = arow[(c + 1) * kLd] * x[c + 1];
      t = __builtin_fma(arow[c * kLd], x[c], t);
      y = __builtin_fma(t, -1.0, y);
      c += 2;
    }
    for (; c < ncol; ++c) {
      const double xa = x[c] * -1.0;
      y = y + arow[c * kLd] * xa;
    }
  } else {
    double t = 0.0;
    for (; c < ncol; ++c) t = __builtin_fma(arow[c * kLd], x[c], t);
    y = __builtin_fma(t, -1.0, y);
  }
  return y;
}

struct Lu {
  double* a;  // LDS, column-major, stride kLd
  int* piv;   // LDS, 1-based global pivots
  int S, lane;
  int flag;   // per-wave uniform
};

// getf2 on the panel rows off..S-1 x columns off..off+n-1
__device__ void lu_getf2(Lu& L, int off, int n) {
  NEMO_RM_NOCONTRACT
  double* a = L.a;
  const int m = L.S - off, lane = L.lane;
  for (int jl = 0; jl < n; ++jl) {
    double* b = &at(a, off, off + jl);   // b[i]: row off + i of column off + jl
    const int jm = jl < m ? jl : m;
    if (lane == 0) {
      for (int i = 0; i < jm; ++i) {
        const int ip = L.piv[off + i] - 1 - off;
        if (ip != i) {
          const double t = b[i];
          b[i] = b[ip];
          b[ip] = t;
        }
      }
      for (int i = 1; i < jm; ++i) b[i] = b[i] - ob_ddot_row(i, &at(a, off + i, off), b);
    }
    __syncthreads();
    if (jl < m) {
      const int rows = m - jl, i = lane - (off + jl);
      if (i >= 0 && i < rows) b[jl + i] = ob_gemv_n_row(i, rows, jl, &at(a, lane, off), b, b[jl + i]);
      __syncthreads();
      // idamax: the first of the largest |b|
      const double v = (i >= 0 && i < rows) ? fabs(b[jl + i]) : -1.0;
      const double mx = wave_fmax(v);
      const int jpl = wave_imin((i >= 0 && i < rows && v == mx) ? i : kAncS);
      const int jp = off + jl + (jpl < kAncS ? jpl : 0);   // global row
      const double t1 = b[jp - off];
      __syncthreads();
      if (lane == 0) L.piv[off + jl] = jp + 1;
      if (t1 != 0.0) {
        if (jp != off + jl && lane <= jl) {   // rows off+jl <-> jp over the panel's columns 0..jl
          double& p = at(a, off + jl, off + lane);
          double& q = at(a, jp, off + lane);
          const double t = p;
          p = q;
          q = t;
        }
        __syncthreads();
        const double r = 1.0 / t1;
        if (lane > off + jl && lane < L.S) b[lane - off] *= r;
      } else {
        L.flag |= 1;
      }
      __syncthreads();
    }
  }
}

// the rows r0..r1-1's pivots on columns c0..c1-1 (one lane per column)
__device__ void lu_laswp(Lu& L, int r0, int r1, int c0, int c1) {
  for (int col = c0 + L.lane; col < c1; col += kAncS)
    for (int r = r0; r < r1; ++r) {
      const int ip = L.piv[r] - 1;
      if (ip != r) {
        const double t = at(L.a, r, col);
        at(L.a, r, col) = at(L.a, ip, col);
        at(L.a, ip, col) = t;
      }
    }
}

// dtrsm_kernel_LT with the unit lower block at (d, d), jb rows, on columns c0..c1-1
__device__ void lu_trsm(Lu& L, int d, int jb, int c0, int c1) {
  NEMO_RM_NOCONTRACT
  double* a = L.a;
  for (int col = c0 + L.lane; col < c1; col += kAncS) {
    double* x = &at(a, d, col);
    int r0 = 0;
    while (r0 < jb) {
      const int rest = jb - r0;
      const int mb = rest >= 16 ? 16 : (rest & 8) ? 8 : (rest & 4) ? 4 : (rest & 2) ? 2 : 1;
      if (r0 > 0)
        for (int r = r0; r < r0 + mb; ++r) {
          double acc = 0.0;
          for (int k = 0; k < r0; ++k) acc = __builtin_fma(at(a, d + r, d + k), x[k], acc);
          x[r] = x[r] - acc;
        }
      for (int i = r0; i < r0 + mb; ++i) {
        const double bb = x[i];
        for (int k = i + 1; k < r0 + mb; ++k) x[k] = __builtin_fma(-bb, at(a, d + k, d + i), x[k]);
      }
      r0 += mb;
    }
  }
}

// dgemm_kernel, alpha -1: A[R][C] -= A[R][d..d+jb) A[d..d+jb)[C] over rows
// R0..S-1 and columns C0..C1-1
__device__ void lu_gemm(Lu& L, int d, int jb, int R0, int C0, int C1) {
  NEMO_RM_NOCONTRACT
  double* a = L.a;
  const int M = L.S - R0, N = C1 - C0;
  if (M <= 0 || N <= 0) return;
  const int r8 = (M & ~15) + (M & 8), r4 = r8 + (M & 4), n12 = N - N % 12;
  for (int e = L.lane; e < M * N; e += kAncS) {
    const int ii = e % M, jc = e / M;
    const int split = (jc >= n12 || ii < r8) ? 1 : ii < r4 ? 2 : 4;
    const double* ar = &at(a, R0 + ii, d);
    const double* bc = &at(a, d, C0 + jc);
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0, acc;
    int k = 0;
    if (split == 1) {
      for (; k < jb; ++k) p0 = __builtin_fma(ar[k * kLd], bc[k], p0);
      acc = p0;
    } else if (split == 2) {
      for (; k + 2 <= jb; k += 2) {
        p0 = __builtin_fma(ar[k * kLd], bc[k], p0);
        p1 = __builtin_fma(ar[(k + 1) * kLd], bc[k + 1], p1);
      }
      acc = p0 + p1;
    } else {
      for (; k + 4 <= jb; k += 4) {
        p0 = __builtin_fma(ar[k * kLd], bc[k], p0);
        p1 = __builtin_fma(ar[(k + 1) * kLd], bc[k + 1], p1);
        p2 = __builtin_fma(ar[(k + 2) * kLd], bc[k + 2], p2);
        p3 = __builtin_fma(ar[(k + 3) * kLd], bc[k + 3], p3);
      }
      acc = (p0 + p1) + (p2 + p3);
    }
    for (; k < jb; ++k) acc = __builtin_fma(ar[k * kLd], bc[k], acc);
    double& cc = at(a, R0 + ii, C0 + jc);
    cc = __builtin_fma(acc, -1.0, cc);
  }
}

// getrf_single on the panel starting at (off, off), rows off..S-1, nn columns.
// Depth: S <= 64 halves the panel width 32 -> 16 -> 8, whose panels go to getf2.
template <int D>
__device__ void lu_getrf(Lu& L, int off, int nn) {
  const int m = L.S - off, mn = m < nn ? m : nn;
  if (m <= 0 || nn <= 0) return;
  const int blocking = ((mn / 2 + 1) / 2) * 2;
  if (blocking <= 4 || D >= 4) {
    if (blocking > 4) L.flag |= 4;   // never at S <= 64: the host recomputes
    lu_getf2(L, off, nn);
    return;
  }
  for (int j = 0; j < mn; j += blocking) {
    const int jb = mn - j < blocking ? mn - j : blocking;
    lu_getrf<D + 1>(L, off + j, jb);
    __syncthreads();
    if (j + jb < nn) {
      lu_laswp(L, off + j, off + j + jb, off + j + jb, off + nn);
      lu_trsm(L, off + j, jb, off + j + jb, off + nn);
      __syncthreads();
      lu_gemm(L, off + j, jb, off + j + jb, off + j + jb, off + nn);
      __syncthreads();
    }
  }
  for (int j = 0; j < mn; j += blocking) {
    const int jb = mn - j < blocking ? mn - j : blocking;
    lu_laswp(L, off + j + jb, off + mn, off + j, off + j + jb);
  }
  __syncthreads();
}

template <>
__device__ void lu_getrf<5>(Lu&, int, int) {}

__global__ __launch_bounds__(kAncS) void ancestor_kernel(int S, int cap, const int32_t* __restrict__ pos,
                                                         const double* __restrict__ w, double* __restrict__ w01,
                                                         double* __restrict__ anc, int32_t* __restrict__ flag) {
  NEMO_RM_NOCONTRACT
  __shared__ double a[kAncS * kLd];
  __shared__ double work[kAncS];
  __shared__ int piv[kAncS];
  __shared__ int spos[kAncS];
  const int b = blockIdx.x, lane = threadIdx.x;
  const size_t base = (size_t)b * S * S;
  if (lane < S) spos[lane] = pos[(size_t)b * S + lane];
  __syncthreads();
  // W~ (w01 out) and I - W~ (column-major in LDS); lane = parent k
  bool finite = true;
  if (lane < S) {
    const int pk = spos[lane];
    for (int i = 0; i < S; ++i) {
      const int pi = spos[i];
      const double wv = w[base + (size_t)i * S + lane];
      const bool perm = pk < pi && (cap == 0 || pi - pk <= cap);
      const double sv = perm ? refmath::expit(wv) : wv;
      w01[base + (size_t)i * S + lane] = sv;
      const double mv = (i == lane ? 1.0 : 0.0) - sv;
      finite &= __builtin_isfinite(mv);
      at(a, i, lane) = mv;
    }
  }
  Lu L{a, piv, S, lane, 0};
  const bool all_finite = __all(finite);
  if (!all_finite) L.flag |= 2;
  __syncthreads();
  if (all_finite) {
    lu_getrf<0>(L, 0, S);
    // dtrtri -> trti2_UN: column j of inv(U) from the inverted columns 0..j-1
    for (int j = 0; j < S && !(L.flag & 1); ++j) {
      const double ajj = 1.0 / at(a, j, j);
      double v = 0.0;
      if (lane < j) {
        v = at(a, lane, j) * at(a, lane, lane);
        for (int i = lane + 1; i < j; ++i) v = __builtin_fma(at(a, i, j), at(a, lane, i), v);
        v = v * -ajj;
      }
      __syncthreads();
      if (lane < j) at(a, lane, j) = v;
      if (lane == j) at(a, j, j) = ajj;
      __syncthreads();
    }
    // dgetri's unblocked loop: inv(A) L = inv(U), column j from the right
    for (int j = S - 1; j >= 0 && !(L.flag & 1); --j) {
      if (lane > j && lane < S) {
        work[lane] = at(a, lane, j);
        at(a, lane, j) = 0.0;
      }
      __syncthreads();
      if (j < S - 1 && lane < S)
        at(a, lane, j) = ob_gemv_n_row(lane, S, S - 1 - j, &at(a, lane, j + 1), &work[j + 1], at(a, lane, j));
      __syncthreads();
    }
    // column swaps j = S-2 .. 0 (a lane per row: no cross-lane order)
    if (lane < S)
      for (int j = S - 2; j >= 0; --j) {
        const int jp = piv[j] - 1;
        if (jp != j) {
          const double t = at(a, lane, j);
          at(a, lane, j) = at(a, lane, jp);
          at(a, lane, jp) = t;
        }
      }
    __syncthreads();
  }
  // clip(inv - I, 0, 1); lane = column k
  bool ok = true;
  if (lane < S)
    for (int i = 0; i < S; ++i) {
      const double x = at(a, i, lane);
      ok &= __builtin_isfinite(x);
      double v = i == lane ? x - 1.0 : x;
      v = v < 0.0 ? 0.0 : v;
      v = v > 1.0 ? 1.0 : v;
      anc[base + (size_t)i * S + lane] = v;
    }
  if (!__all(ok) && all_finite) L.flag |= 4;
  if (lane == 0) flag[b] = L.flag;
}

}  // namespace

bool ancestor_supported(const Ctx& c) { return c.S <= kAncS; }

hipError_t launch_ancestor(Ctx& c, int nchains, int cap, const int32_t* d_pos, const double* d_w, double* d_w01,
                           double* d_anc, int32_t* d_flag, hipStream_t st) {
  if (c.S > kAncS) return hipErrorInvalidValue;
  if (nchains <= 0) return hipSuccess;
  ancestor_kernel<<<nchains, kAncS, 0, st>>>(c.S, cap >= c.S - 1 ? 0 : cap, d_pos, d_w, d_w01, d_anc, d_flag);
  return hipGetLastError();
}

}  // namespace nemo
