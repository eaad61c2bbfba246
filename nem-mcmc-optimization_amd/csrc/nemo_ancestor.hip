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
// (tests/host/lapack_check.c: 0 differing bits for n = 1..128 getrf and
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
constexpr int kJb = 32;     // the widest panel of a getrf at S <= 64

// One wave per chain; every phase is written for latency: the matrix lives in
// LDS, but a phase's operands are loaded in batches ahead of its dependent
// chain, a column or a row being solved sits in registers (static indices,
// loops unrolled over the largest size with uniform predicates), and the
// cross-lane steps are DPP / permlane moves and readlanes, not LDS round trips.

__device__ __forceinline__ double& at(double* a, int r, int c) { return a[r + c * kLd]; }

__device__ __forceinline__ double readlane_d(double v, int l) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}

// (v, i) <- the larger v, the smaller i on a tie (idamax: the first largest)
__device__ __forceinline__ void amax_take(double& v, int& i, double ov, int oi) {
  const bool take = ov > v || (ov == v && oi < i);
  v = take ? ov : v;
  i = take ? oi : i;
}

// idamax over the wave, the result in every lane
__device__ __forceinline__ void wave_argmax(double& v, int& i) {
  amax_take(v, i, dpp_d<0xB1>(v), dpp_i<0xB1>(i));    // quad_perm [1,0,3,2]
  amax_take(v, i, dpp_d<0x4E>(v), dpp_i<0x4E>(i));    // quad_perm [2,3,0,1]
  amax_take(v, i, dpp_d<0x141>(v), dpp_i<0x141>(i));  // row_half_mirror
  amax_take(v, i, dpp_d<0x140>(v), dpp_i<0x140>(i));  // row_mirror
  {  // row pairs (0,1), (2,3): both outputs of a permlane16 swap
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)b, (uint32_t)b, false, false);
    auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    auto ix = __builtin_amdgcn_permlane16_swap((uint32_t)i, (uint32_t)i, false, false);
    double v0 = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
    int i0 = (int)ix[0];
    amax_take(v0, i0, __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]), (int)ix[1]);
    v = v0;
    i = i0;
  }
  {  // halves
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
    auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    auto ix = __builtin_amdgcn_permlane32_swap((uint32_t)i, (uint32_t)i, false, false);
    double v0 = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
    int i0 = (int)ix[0];
    amax_take(v0, i0, __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]), (int)ix[1]);
    v = v0;
    i = i0;
  }
}

#ifndef NEMO_ANC_PROFILE
#define NEMO_ANC_PROFILE 0
#endif

struct Lu {
  double* a;  // LDS, column-major, stride kLd
  int* piv;   // LDS, 1-based global pivots
  int S, lane;
  int flag;   // wave-uniform
#if NEMO_ANC_PROFILE  // instrumented build (tools/anc_phases.py): shader cycles per phase
  long long cyc[4] = {0, 0, 0, 0};   // getf2, laswp, trsm, gemm
#endif
};

#if NEMO_ANC_PROFILE
#define ANC_T0() const long long t0_ = clock64()
#define ANC_T1(L, k) (L).cyc[k] += clock64() - t0_
#else
#define ANC_T0()
#define ANC_T1(L, k)
#endif

// getf2 (lapack/getf2/getf2.c) on the panel rows off..S-1 x columns
// off..off+n-1, n <= NM.  Per column, in registers (lane = row): the earlier
// pivots of the panel composed into one gather; the U part (ddot_k, x strided:
// products of elements 2 and 3 of each group of four feed the fmas of elements
// 0 and 1 into two sums, the tail chains on the first, the sums add at the end)
// on wave-uniform values; dgemv_n of the rows below (alpha -1: rows below
// rows & ~3 the 4-column kernel t = a1 x1, fma a0 x0, a2 x2, a3 x3, y = fma(t,
// -1, y), a 2-column step, unfused y + a (x * -1) for the last column; the last
// rows & 3 rows one fma chain, y = fma(t, -1, y)); idamax; the row swap and the
// scale by the pivot's reciprocal.  Branch-free: every unrolled step computes
// and a uniform select keeps it or not, so the loads issue ahead of the chains.
template <int NM>
__device__ __forceinline__ void lu_getf2(Lu& L, int off, int n) {
  NEMO_RM_NOCONTRACT
  double* a = L.a;
  const int S = L.S, lane = L.lane, m = S - off;
  for (int jl = 0; jl < n; ++jl) {   // m >= n > jl: every column has its pivot search
    const int col = off + jl;
    int pv[NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) pv[i] = L.piv[off + (i < jl ? i : 0)] - 1;
    int src = lane;
#pragma unroll
    for (int i = NM - 1; i >= 0; --i) {
      const int r = off + i, ip = pv[i];
      const int s1 = src == r ? ip : src == ip ? r : src;
      src = i < jl ? s1 : src;
    }
    double bv = at(a, src, col);
    double lrow[NM];
#pragma unroll
    for (int c = 0; c < NM; ++c) lrow[c] = at(a, lane, off + (c < jl ? c : 0));
    double bu[NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const int li = (off + i) & (kAncS - 1);
      double v = readlane_d(bv, li);
      if (i >= 1) {
        double t1 = 0.0, t2 = 0.0;
        int k = 0;
#pragma unroll
        for (; k + 4 <= i; k += 4) {
          const double m3 = bu[k + 2] * readlane_d(lrow[k + 2], li);
          const double m4 = bu[k + 3] * readlane_d(lrow[k + 3], li);
          t1 = t1 + __builtin_fma(bu[k], readlane_d(lrow[k], li), m3);
          t2 = t2 + __builtin_fma(bu[k + 1], readlane_d(lrow[k + 1], li), m4);
        }
#pragma unroll
        for (; k < i; ++k) t1 = __builtin_fma(bu[k], readlane_d(lrow[k], li), t1);
        v = v - (t1 + t2);
        bv = (i < jl && lane == off + i) ? v : bv;
      }
      bu[i] = i < jl ? v : 0.0;
    }
    const int rows = m - jl, i = lane - col;
    const bool act = i >= 0 && i < rows;
    const int mb = rows - (rows & 3);
    double yb = bv;
#pragma unroll
    for (int c = 0; c + 4 <= NM; c += 4) {
      double t = lrow[c + 1] * bu[c + 1];
      t = __builtin_fma(lrow[c], bu[c], t);
      t = __builtin_fma(lrow[c + 2], bu[c + 2], t);
      t = __builtin_fma(lrow[c + 3], bu[c + 3], t);
      yb = c + 4 <= jl ? __builtin_fma(t, -1.0, yb) : yb;
    }
    const int c4 = jl & ~3;
#pragma unroll
    for (int c = 0; c + 2 <= NM; c += 4) {
      double t = lrow[c + 1] * bu[c + 1];
      t = __builtin_fma(lrow[c], bu[c], t);
      yb = (c == c4 && jl - c4 >= 2) ? __builtin_fma(t, -1.0, yb) : yb;
    }
    const int c1 = c4 + ((jl - c4) & 2);
#pragma unroll
    for (int c = 0; c < NM; ++c) {
      const double xa = bu[c] * -1.0;
      yb = (c >= c1 && c < jl) ? yb + lrow[c] * xa : yb;
    }
    double tc = 0.0;
#pragma unroll
    for (int c = 0; c < NM; ++c) tc = c < jl ? __builtin_fma(lrow[c], bu[c], tc) : tc;
    const double yc = __builtin_fma(tc, -1.0, bv);
    bv = act ? (i < mb ? yb : yc) : bv;
    double v = act ? fabs(bv) : -1.0;
    int ix = act ? i : kAncS;
    wave_argmax(v, ix);
    const int jp = col + (ix < kAncS ? ix : 0);
    const double t1 = readlane_d(bv, jp);
    if (lane == 0) L.piv[col] = jp + 1;
    if (t1 != 0.0) {
      if (jp != col) {
        const double vc = readlane_d(bv, col);
        bv = lane == col ? t1 : lane == jp ? vc : bv;
        if (lane < jl) {  // the panel's earlier columns: rows col <-> jp
          double& p = at(a, col, off + lane);
          double& q = at(a, jp, off + lane);
          const double t = p;
          p = q;
          q = t;
        }
      }
      const double r = 1.0 / t1;
      bv = (lane > col && lane < S) ? bv * r : bv;
    } else {
      L.flag |= 1;
    }
    if (lane >= off && lane < S) at(a, lane, col) = bv;
    __syncthreads();
  }
}

// the rows r0..r1-1's pivots on columns c0..c1-1 (one lane per column)
__device__ __forceinline__ void lu_laswp(Lu& L, int r0, int r1, int c0, int c1) {
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

// the start of row k's block in dtrsm_kernel_LT's row blocking of jb rows:
// 16 while 16 remain, then 8, 4, 2, 1 by the bits of the remainder (selects)
__device__ __forceinline__ int trsm_block_start(int k, int jb) {
  const int q16 = jb & ~15, rest = jb - q16;
  int base = q16, res = -1;
#pragma unroll
  for (int w = 8; w >= 1; w >>= 1) {
    const bool has = (rest & w) != 0;
    res = (has && res < 0 && k < base + w) ? base : res;
    base = has ? base + w : base;
  }
  return k < q16 ? (k & ~15) : res < 0 ? base : res;
}

// dtrsm_kernel_LT with the unit lower block at (d, d), jb <= K rows, on
// columns c0..c1-1, a lane per column, the column in registers.  Row k: minus
// the GEMM chain over the solved rows above its block (fma from 0, k
// ascending), then fma(-x_i, l_ki, x_k) over the rows of its block above it --
// each element's operations in the kernel's own order.
template <int K>
__device__ __forceinline__ void lu_trsm(Lu& L, int d, int jb, int c0, int c1) {
  NEMO_RM_NOCONTRACT
  double* a = L.a;
  const int col = c0 + L.lane;
  const bool act = col < c1;
  const int cc = act ? col : c0;
  double x[K];
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = at(a, d + (k < jb ? k : 0), cc);
#pragma unroll
  for (int k = 1; k < K; ++k) {
    const int r0 = trsm_block_start(k, jb), kr = k < jb ? k : 0;
    double acc = 0.0;
#pragma unroll
    for (int m = 0; m < k; ++m) acc = m < r0 ? __builtin_fma(at(a, d + kr, d + m), x[m], acc) : acc;
    double v = r0 > 0 ? x[k] - acc : x[k];
#pragma unroll
    for (int m = 0; m < k; ++m) v = m >= r0 ? __builtin_fma(-x[m], at(a, d + kr, d + m), v) : v;
    x[k] = v;
  }
  if (act)
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < jb) at(a, d + k, col) = x[k];
}

// dgemm_kernel, alpha -1: A[R][C] -= A[R][d..d+jb) A[d..d+jb)[C] over rows
// R0..S-1 (a lane per row, its jb <= K multipliers in registers, zero beyond
// jb: fma(0, b, p) leaves p, which is never -0) and columns C0..C1-1, four at
// a time.  Rows in blocks of 16, 8, 4, 2, 1 and columns in groups of 12: a 16-
// or 8-row block and the last N % 12 columns chain k; a 4-row block sums even
// and odd k apart, a 2- or 1-row block the classes of k mod 4, the rest of k
// chaining on the combined sum; C = fma(acc, -1, C).
template <int K>
__device__ __forceinline__ void lu_gemm(Lu& L, int d, int jb, int R0, int C0, int C1) {
  NEMO_RM_NOCONTRACT
  double* a = L.a;
  const int M = L.S - R0, N = C1 - C0, ii = L.lane;
  if (M <= 0 || N <= 0) return;
  const bool act = ii < M;
  const int row = R0 + (act ? ii : 0);
  const int r8 = (M & ~15) + (M & 8), r4 = r8 + (M & 4), n12 = N - N % 12;
  const int split = ii < r8 ? 1 : ii < r4 ? 2 : 4;
  double ar[K];
#pragma unroll
  for (int k = 0; k < K; ++k) ar[k] = k < jb ? at(a, row, d + k) : 0.0;
  for (int j0 = 0; j0 < N; j0 += 4) {
    int cq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cq[q] = C0 + (j0 + q < N ? j0 + q : 0);
    double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int kk = d + (k < jb ? k : 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) p[q] = __builtin_fma(ar[k], at(a, kk, cq[q]), p[q]);
    }
    if (split != 1 && act) {  // the tail rows' split sums on the first n12 columns
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (j0 + q < n12) {
          const double* bc = &at(a, d, C0 + j0 + q);
          const double* ra = &at(a, row, d);
          double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, acc;
          int k = 0;
          if (split == 2) {
            for (; k + 2 <= jb; k += 2) {
              s0 = __builtin_fma(ra[k * kLd], bc[k], s0);
              s1 = __builtin_fma(ra[(k + 1) * kLd], bc[k + 1], s1);
            }
            acc = s0 + s1;
          } else {
            for (; k + 4 <= jb; k += 4) {
              s0 = __builtin_fma(ra[k * kLd], bc[k], s0);
              s1 = __builtin_fma(ra[(k + 1) * kLd], bc[k + 1], s1);
              s2 = __builtin_fma(ra[(k + 2) * kLd], bc[k + 2], s2);
              s3 = __builtin_fma(ra[(k + 3) * kLd], bc[k + 3], s3);
            }
            acc = (s0 + s1) + (s2 + s3);
          }
          for (; k < jb; ++k) acc = __builtin_fma(ra[k * kLd], bc[k], acc);
          p[q] = acc;
        }
    }
    if (act)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (j0 + q < N) {
          double& c = at(a, row, C0 + j0 + q);
          c = __builtin_fma(p[q], -1.0, c);
        }
  }
}

// getrf_single on the panel starting at (off, off), rows off..S-1, nn columns.
// Depth: S <= 64 halves the panel width 32 -> 16 -> 8, whose panels go to getf2.
template <int D>
__device__ __forceinline__ void lu_getrf(Lu& L, int off, int nn) {
  const int m = L.S - off, mn = m < nn ? m : nn;
  if (m <= 0 || nn <= 0) return;
  const int blocking = ((mn / 2 + 1) / 2) * 2;
  if (blocking <= 4 || D >= 4) {
    if (blocking > 4) L.flag |= 4;   // never at S <= 64: the host recomputes
    ANC_T0();
    if (nn <= 8)
      lu_getf2<8>(L, off, nn);
    else if (nn <= 16)
      lu_getf2<16>(L, off, nn);
    else
      L.flag |= 4;
    ANC_T1(L, 0);
    return;
  }
  if (blocking > kJb) {
    L.flag |= 4;
    return;
  }
  for (int j = 0; j < mn; j += blocking) {
    const int jb = mn - j < blocking ? mn - j : blocking;
    lu_getrf<D + 1>(L, off + j, jb);
    __syncthreads();
    if (j + jb < nn) {
      {
        ANC_T0();
        lu_laswp(L, off + j, off + j + jb, off + j + jb, off + nn);
        ANC_T1(L, 1);
      }
      {
        ANC_T0();
        if (jb <= 8)
          lu_trsm<8>(L, off + j, jb, off + j + jb, off + nn);
        else if (jb <= 16)
          lu_trsm<16>(L, off + j, jb, off + j + jb, off + nn);
        else
          lu_trsm<32>(L, off + j, jb, off + j + jb, off + nn);
        __syncthreads();
        ANC_T1(L, 2);
      }
      ANC_T0();
      if (jb <= 8)
        lu_gemm<8>(L, off + j, jb, off + j + jb, off + j + jb, off + nn);
      else if (jb <= 16)
        lu_gemm<16>(L, off + j, jb, off + j + jb, off + j + jb, off + nn);
      else
        lu_gemm<32>(L, off + j, jb, off + j + jb, off + j + jb, off + nn);
      __syncthreads();
      ANC_T1(L, 3);
    }
  }
  ANC_T0();
  for (int j = 0; j < mn; j += blocking) {
    const int jb = mn - j < blocking ? mn - j : blocking;
    lu_laswp(L, off + j + jb, off + mn, off + j, off + j + jb);
  }
  __syncthreads();
  ANC_T1(L, 1);
}

template <>
__device__ __forceinline__ void lu_getrf<5>(Lu&, int, int) {}

// dtrtri (trti2_UN) + dgetri's unblocked loop + its column swaps for S fixed
// at compile time: a lane per row, the rows of the inverse in a second LDS
// matrix ib (each lane reads back only what it wrote), every operand address a
// constant.  Row r of inv(U), column j: x_r * inv_rr, then fma(x_i, inv_ri, .)
// for i = r+1..j-1, times -1 / u_jj (trmv_NUN's axpy chain, scal); then from
// the right y = row[j] (0 below the diagonal) minus dgemv_n's 4-column sums of
// row[c] L[c][j] over c > j; the column swaps composed into one permutation,
// applied as the rows go back to the matrix.
template <int S>
__device__ __forceinline__ void inv_rows_static(Lu& L, double* ib) {
  NEMO_RM_NOCONTRACT
  static_assert(S % 4 == 0 && S <= kAncS, "rows below rows & ~3 only");
  double* a = L.a;
  const int lane = L.lane;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const double ajj = 1.0 / at(a, j, j);
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < j; ++i) {
      const double x = at(a, i, j), u = at(ib, lane, i);
      const double pr = x * u, f = __builtin_fma(x, u, v);
      v = i == lane ? pr : f;   // before i == lane: discarded there
    }
    at(ib, lane, j) = j > lane ? v * -ajj : j == lane ? ajj : 0.0;
  }
#pragma unroll
  for (int j = S - 2; j >= 0; --j) {
    const int ncol = S - 1 - j;
    double y = at(ib, lane, j);
    int c = 0;
#pragma unroll
    for (; c + 4 <= ncol; c += 4) {
      const int b = j + 1 + c;
      double t = at(ib, lane, b + 1) * at(a, b + 1, j);
      t = __builtin_fma(at(ib, lane, b), at(a, b, j), t);
      t = __builtin_fma(at(ib, lane, b + 2), at(a, b + 2, j), t);
      t = __builtin_fma(at(ib, lane, b + 3), at(a, b + 3, j), t);
      y = __builtin_fma(t, -1.0, y);
    }
    if (ncol - c >= 2) {
      const int b = j + 1 + c;
      double t = at(ib, lane, b + 1) * at(a, b + 1, j);
      t = __builtin_fma(at(ib, lane, b), at(a, b, j), t);
      y = __builtin_fma(t, -1.0, y);
      c += 2;
    }
#pragma unroll
    for (; c < ncol; ++c) {
      const int b = j + 1 + c;
      const double xa = at(a, b, j) * -1.0;
      y = y + at(ib, lane, b) * xa;
    }
    at(ib, lane, j) = y;
  }
  // where column c ends up after the swaps j = S-2 .. 0 (lane c tracks it)
  int dst = lane;
#pragma unroll
  for (int j = S - 2; j >= 0; --j) {
    const int jp = L.piv[j] - 1;
    dst = dst == j ? jp : dst == jp ? j : dst;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < S; ++c) at(a, lane, __builtin_amdgcn_readlane(dst, c)) = at(ib, lane, c);
  __syncthreads();
}

// SS > 0: S fixed at compile time (the configs' S = 64: every loop bound and
// panel offset a constant), 0: S from the argument
// w01 null: W~ not written (w01_kernel writes it, on the main stream)
template <int SS>
__global__ __launch_bounds__(kAncS) void ancestor_kernel(int S_arg, int cap, const int32_t* __restrict__ pos,
                                                         const double* __restrict__ w, double* __restrict__ w01,
                                                         double* __restrict__ anc, int32_t* __restrict__ flag) {
  NEMO_RM_NOCONTRACT
  const int S = SS > 0 ? SS : S_arg;
  __shared__ double a[kAncS * kLd];
  __shared__ double ib[SS > 0 ? kAncS * kLd : 1];   // inv_rows_static's rows
  __shared__ double work[kAncS];
  __shared__ int piv[kAncS];
  __shared__ int spos[kAncS];
  const int b = blockIdx.x, lane = threadIdx.x;
  const size_t base = (size_t)b * S * S;
  // every entry finite (the branch-free steps read, and multiply by zero,
  // entries outside the S x S matrix)
  for (int k = lane; k < kAncS * kLd; k += kAncS) a[k] = 0.0;
  if (lane < S) spos[lane] = pos[(size_t)b * S + lane];
  __syncthreads();
  // W~ (w01 out) and I - W~ (column-major in LDS); lane = parent k
  bool finite = true;
  if (lane < S) {
    const int pk = spos[lane];
#pragma unroll 4
    for (int i = 0; i < S; ++i) {
      const int pi = spos[i];
      const double wv = w[base + (size_t)i * S + lane];
      const bool perm = pk < pi && (cap == 0 || pi - pk <= cap);
      const double sv = perm ? refmath::expit(wv) : wv;
      if (w01) w01[base + (size_t)i * S + lane] = sv;
      const double mv = (i == lane ? 1.0 : 0.0) - sv;
      finite &= __builtin_isfinite(mv);
      at(a, i, lane) = mv;
    }
  }
  Lu L{a, piv, S, lane, 0};
  const bool all_finite = __all(finite);
  if (!all_finite) L.flag |= 2;
  __syncthreads();
#if NEMO_ANC_PROFILE
  long long tp[6];
  tp[0] = clock64();
#endif
  if (all_finite) {
    lu_getrf<0>(L, 0, S);
#if NEMO_ANC_PROFILE
    tp[1] = clock64();
#endif
    if constexpr (SS > 0) {
      if (!(L.flag & 1)) inv_rows_static<SS>(L, ib);
#if NEMO_ANC_PROFILE
      tp[2] = tp[3] = clock64();
#endif
    } else {
    // dtrtri -> trti2_UN: column j of inv(U) from the inverted columns 0..j-1;
    // lane r: x_r * inv_rr, then fma(x_i, inv_ri, .) for i = r+1..j-1, times -1 / u_jj
    for (int j = 0; j < S && !(L.flag & 1); ++j) {
      const double ajj = 1.0 / at(a, j, j);
      double v = 0.0;
      int i = 0;
      for (; i + 8 <= j; i += 8) {
        double xs[8], us[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          xs[q] = at(a, i + q, j);
          us[q] = at(a, lane, i + q);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const double pr = xs[q] * us[q], f = __builtin_fma(xs[q], us[q], v);
          v = i + q == lane ? pr : i + q > lane ? f : v;
        }
      }
      for (; i < j; ++i) {
        const double xs = at(a, i, j), us = at(a, lane, i);
        const double pr = xs * us, f = __builtin_fma(xs, us, v);
        v = i == lane ? pr : i > lane ? f : v;
      }
      v = v * -ajj;
      __syncthreads();
      if (lane < j) at(a, lane, j) = v;
      if (lane == j) at(a, j, j) = ajj;
      __syncthreads();
    }
#if NEMO_ANC_PROFILE
    tp[2] = clock64();
#endif
    // dgetri's unblocked loop: inv(A) L = inv(U), column j from the right; lane
    // = row g: dgemv_n (alpha -1) of the columns right of j against WORK
    const int mb = S - (S & 3);
    for (int j = S - 1; j >= 0 && !(L.flag & 1); --j) {
      if (lane > j && lane < S) {
        work[lane] = at(a, lane, j);
        at(a, lane, j) = 0.0;
      }
      __syncthreads();
      if (j < S - 1 && lane < S) {
        const int ncol = S - 1 - j;
        const double* arow = &at(a, lane, j + 1);
        const double* x = &work[j + 1];
        double y = at(a, lane, j);
        int c = 0;
        if (lane < mb) {
          for (; c + 16 <= ncol; c += 16) {
            double av[16], xv[16], t[4];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              av[q] = arow[(c + q) * kLd];
              xv[q] = x[c + q];
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              t[g] = av[4 * g + 1] * xv[4 * g + 1];
              t[g] = __builtin_fma(av[4 * g], xv[4 * g], t[g]);
              t[g] = __builtin_fma(av[4 * g + 2], xv[4 * g + 2], t[g]);
              t[g] = __builtin_fma(av[4 * g + 3], xv[4 * g + 3], t[g]);
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) y = __builtin_fma(t[g], -1.0, y);
          }
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
          for (; c + 8 <= ncol; c += 8) {
            double av[8], xv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              av[q] = arow[(c + q) * kLd];
              xv[q] = x[c + q];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) t = __builtin_fma(av[q], xv[q], t);
          }
          for (; c < ncol; ++c) t = __builtin_fma(arow[c * kLd], x[c], t);
          y = __builtin_fma(t, -1.0, y);
        }
        at(a, lane, j) = y;
      }
      __syncthreads();
    }
#if NEMO_ANC_PROFILE
    tp[3] = clock64();
#endif
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
  }
  // clip(inv - I, 0, 1) as numpy's loop (x < 0 ? 0 : x, then > 1 ? 1 : x); lane = column k
  bool ok = true;
  if (lane < S)
#pragma unroll 4
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
#if NEMO_ANC_PROFILE
  // the last chain's first ancestor_x row: the phases' shader cycles
  // (getrf, trti2, getri, swaps + clip; getf2, laswp, trsm, gemm inside getrf)
  tp[4] = clock64();
  __syncthreads();
  if (lane == 0 && b == (int)gridDim.x - 1) {
    double* o = anc + base;
    o[0] = (double)(tp[1] - tp[0]);
    o[1] = (double)(tp[2] - tp[1]);
    o[2] = (double)(tp[3] - tp[2]);
    o[3] = (double)(tp[4] - tp[3]);
    for (int k = 0; k < 4; ++k) o[4 + k] = (double)L.cyc[k];
  }
#endif
}

// W~ alone (expit on the permissible entries, the rest W's own): what eval #1
// needs, while ancestor_kernel runs beside it on a second stream
__global__ __launch_bounds__(256) void w01_kernel(int S, int cap, const int32_t* __restrict__ pos,
                                                  const double* __restrict__ w, double* __restrict__ w01) {
  const int b = blockIdx.x;
  const int32_t* p = pos + (size_t)b * S;
  const size_t base = (size_t)b * S * S;
  for (int idx = threadIdx.x; idx < S * S; idx += blockDim.x) {
    const int i = idx / S, k = idx - i * S;
    const int pi = p[i], pk = p[k];
    const double wv = w[base + idx];
    w01[base + idx] = (pk < pi && (cap == 0 || pi - pk <= cap)) ? refmath::expit(wv) : wv;
  }
}

}  // namespace

bool ancestor_supported(const Ctx& c) { return c.S <= kAncS; }

hipError_t launch_w01(Ctx& c, int nchains, int cap, const int32_t* d_pos, const double* d_w, double* d_w01,
                      hipStream_t st) {
  if (nchains <= 0) return hipSuccess;
  w01_kernel<<<nchains, 256, 0, st>>>(c.S, cap >= c.S - 1 ? 0 : cap, d_pos, d_w, d_w01);
  return hipGetLastError();
}

hipError_t launch_ancestor(Ctx& c, int nchains, int cap, const int32_t* d_pos, const double* d_w, double* d_w01,
                           double* d_anc, int32_t* d_flag, hipStream_t st) {
  if (c.S > kAncS) return hipErrorInvalidValue;
  if (nchains <= 0) return hipSuccess;
  const int cp = cap >= c.S - 1 ? 0 : cap;
  if (c.S == kAncS)
    ancestor_kernel<kAncS><<<nchains, kAncS, 0, st>>>(c.S, cp, d_pos, d_w, d_w01, d_anc, d_flag);
  else
    ancestor_kernel<0><<<nchains, kAncS, 0, st>>>(c.S, cp, d_pos, d_w, d_w01, d_anc, d_flag);
  return hipGetLastError();
}

}  // namespace nemo
