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
using lb::uniH;

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

// The control's wave: every lane runs the optimiser (uniform values, scalar
// branches); the independent entries of its small matrices are spread over
// the lanes -- each entry computed by one lane, in the library's order -- and
// written to `mem` (LDS), and the wave syncs before they are read.  On the
// host: one lane, the loops in sequence.
struct Lanes {
  int id, n;
};
// H: the dual form's half wave (lanes 32 h .. 32 h + 31 run optimum h)
template <bool H = false>
NEMO_LB Lanes lanes() {
#if defined(__HIP_DEVICE_COMPILE__)
  return H ? Lanes{(int)__lane_id() & 31, 32} : Lanes{(int)__lane_id(), 64};
#else
  return Lanes{0, 1};
#endif
}
NEMO_LB void lanes_sync() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}
#if defined(__HIP_DEVICE_COMPILE__)
// lane l's value, to every lane
__device__ __forceinline__ double readlane_d(double v, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// lane l of this lane's group (H: of its half) to every lane of the group.
// H: l is uniform within each half but may differ between them (a loop from
// 2 col - 1 down, col + j), so each half's l is read from the half's first
// lane and each half's value from its own lane (readlane takes a uniform
// lane number: one for both halves would serve the first active half only)
template <bool H>
__device__ __forceinline__ double bcast(double v, int l) {
  if (!H) return readlane_d(v, l);
  const int la = __builtin_amdgcn_readlane(l, 0) & 31, lb = __builtin_amdgcn_readlane(l, 32) & 31;
  const double a = readlane_d(v, la), b = readlane_d(v, 32 + lb);
  return (__lane_id() & 32) ? b : a;
}
#endif

// One output of OpenBLAS dgemv_t_SKYLAKEX with alpha = -1 (A m x n
// column-major, lda, m < 2048): y - A(:, c)' x for column c, in the order of
// the kernel that column falls to -- dgemv_kernel_4x4 (per-column FMA lanes
// summed (0+2)+(1+3)) for the first 4 (n / 4) columns, then the unfused
// 2-lane dgemv_kernel_4x2, then dgemv_kernel_4x1 -- and the m % 4 tail rows
// last with x pre-scaled by alpha.
NEMO_LB double ob_gemv_t_m1_col(int m, int n, int c, const double* a, int lda, const double* x, double y) {
#pragma clang fp contract(off)
  const int m3 = m & 3, nb = m - m3;
  const double* col = a + (long)c * lda;
  if (nb > 0) {
    const int n4 = (n >> 2) * 4, n2 = n & 3;
    if (c < n4) {
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
      y = fma_(t, -1.0, y);  // add_y (exact for alpha = -1 either way)
    } else if ((n2 & 2) && c < n4 + 2) {
      double acc0 = 0.0, acc1 = 0.0;
      for (int i = 0; i < nb; i += 4) {
        acc0 = acc0 + x[i] * col[i];
        acc1 = acc1 + x[i + 1] * col[i + 1];
        acc0 = acc0 + x[i + 2] * col[i + 2];
        acc1 = acc1 + x[i + 3] * col[i + 3];
      }
      y = fma_(acc0 + acc1, -1.0, y);
    } else {
      double p0 = 0.0, p1 = 0.0, q0 = 0.0, q1 = 0.0;
      for (int i = 0; i < nb; i += 4) {
        p0 = p0 + col[i] * x[i];
        p1 = p1 + col[i + 1] * x[i + 1];
        q0 = q0 + col[i + 2] * x[i + 2];
        q1 = q1 + col[i + 3] * x[i + 3];
      }
      y = fma_((p0 + q0) + (p1 + q1), -1.0, y);
    }
  }
  if (m3) {  // the last m3 rows, x pre-scaled by alpha
    const int r = nb;
    const double xt0 = -x[r], xt1 = m3 > 1 ? -x[r + 1] : 0.0, xt2 = m3 > 2 ? -x[r + 2] : 0.0;
    const double* cr = col + r;
    if (m3 == 1) {
      y = fma_(cr[0], xt0, y);
    } else {
      double t = fma_(cr[0], xt0, cr[1] * xt1);
      if (m3 == 3) t = fma_(cr[2], xt2, t);
      y = t + y;
    }
  }
  return y;
}

// OpenBLAS dpotrf('U') for n <= 16 (potf2_U); returns info (0 or j + 1).
// Row j's update (dgemv_t) and scaling by 1 / ajj: one column per lane.
#if !defined(__HIP_DEVICE_COMPILE__)
template <bool H = false>
NEMO_LB int ob_potrf_u(int n, double* a, int lda, Lanes L) {
#pragma clang fp contract(off)
  for (int j = 0; j < n; ++j) {
    double* cj = a + (long)j * lda;
    double ajj = cj[j] - ob_ddot(j, cj, cj);
    if (uniH<H>(ajj <= 0.0)) {   // potf2: a NaN goes on to the square root
      cj[j] = ajj;
      return j + 1;
    }
    ajj = __builtin_sqrt(ajj);
    cj[j] = ajj;
    const int i = n - j - 1;
    if (i > 0) {
      const double inv = 1.0 / ajj;
      for (int k = L.id; k < i; k += L.n) {
        double* y = cj + j + (long)(k + 1) * lda;
        double v = *y;
        if (j > 0) v = ob_gemv_t_m1_col(j, i, k, a + (long)(j + 1) * lda, lda, cj, v);
        *y = v * inv;
      }
      lanes_sync();
    }
  }
  return 0;
}
#else
// On the wave lane c owns column c (n <= 16): it also accumulates ddot(c,
// A(:, c), A(:, c)) -- for n < 16 a chain in row order -- as the rows of its
// column become final, so step j starts from its diagonal at once.
template <bool H = false>
__device__ __forceinline__ int ob_potrf_u(int n, double* a, int lda, Lanes L) {
#pragma clang fp contract(off)
  const int ln = L.id;
  double* mine = a + (long)(ln < n ? ln : 0) * lda;
  double sd = 0.0;
  for (int j = 0; j < n; ++j) {
    double* cj = a + (long)j * lda;
    double ajj = ln == j ? cj[j] - sd : 0.0;
    ajj = bcast<H>(ajj, j);
    if (uniH<H>(ajj <= 0.0)) {   // potf2: a NaN goes on to the square root
      if (ln == j) cj[j] = ajj;
      lanes_sync();
      return j + 1;
    }
    ajj = __builtin_sqrt(ajj);
    if (ln == j) cj[j] = ajj;
    const int i = n - j - 1;
    if (i > 0) {
      const double inv = 1.0 / ajj;
      if (ln > j && ln < n) {
        double v = mine[j];
        if (j > 0) v = ob_gemv_t_m1_col(j, i, ln - j - 1, a + (long)(j + 1) * lda, lda, cj, v);
        v = v * inv;
        mine[j] = v;
        sd = fma_(v, v, sd);
      }
    }
    lanes_sync();
  }
  return 0;
}
#endif

// dtrtrs('U', 'T', 'N') with one right-hand side (trsv_TUN); 0 or the index
// + 1 of a zero diagonal (checked first, as dtrtrs does)
template <bool H = false>
NEMO_LB int ob_trsv_tun(int n, const double* u, int ldu, double* b) {
#pragma clang fp contract(off)
  for (int i = 0; i < n; ++i)
    if (uniH<H>(u[i + (long)i * ldu] == 0.0)) return i + 1;
  for (int i = 0; i < n; ++i) {
    const double* ci = u + (long)i * ldu;
    if (i > 0) b[i] = b[i] - ob_ddot(i, ci, b);
    b[i] = b[i] / ci[i];
  }
  return 0;
}

// dtrtrs('U', 'N', 'N') with one right-hand side (trsv_NUN)
template <bool H = false>
NEMO_LB int ob_trsv_nun(int n, const double* u, int ldu, double* b) {
#pragma clang fp contract(off)
  for (int i = 0; i < n; ++i)
    if (uniH<H>(u[i + (long)i * ldu] == 0.0)) return i + 1;
  for (int j = n - 1; j >= 0; --j) {
    const double* cj = u + (long)j * ldu;
    b[j] = b[j] / cj[j];
    const double nb = -b[j];
    for (int k = 0; k < j; ++k) b[k] = fma_(nb, cj[k], b[k]);
  }
  return 0;
}

// dtrtrs('U', 'T', 'N') with nrhs >= 2 (trsm_LTUN: the inverted diagonal,
// row blocks of 16 then 8, 4, 2, 1), n <= 16, B n x nrhs (ldb); one
// right-hand side per lane
template <bool H = false>
NEMO_LB int ob_trsm_lt(int n, int nrhs, const double* u, int ldu, double* b, int ldb, Lanes L) {
#pragma clang fp contract(off)
  for (int i = 0; i < n; ++i)
    if (uniH<H>(u[i + (long)i * ldu] == 0.0)) return i + 1;
  for (int j = L.id; j < nrhs; j += L.n) {
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
  lanes_sync();
  return 0;
}

// the stored products of the compact form (see the header)
NEMO_LB double prod0(double a, double b) { return fma_(a, b, 0.0); }   // ddot, n = 1
NEMO_LB double sum0(double a, double b) { return 0.0 + a * b; }        // C loop from zero

// The s / y memory in logical order (0 = the oldest pair): the library's
// circular buffer (head, itail) holds the same pairs, and every product reads
// them by logical index, so the bits do not depend on where they are stored.
// When the memory is full the oldest pair is dropped by shifting.
struct Ring {
  int col = 0, iupdat = 0;
};

// matupd: the new pair (s, y, s's, s'y) as the newest
NEMO_LB void matupd(Mem& mem, Ring& rg, double s, double y, double ssd, double syd) {
  rg.iupdat += 1;
  if (rg.iupdat <= kM) {
    rg.col = rg.iupdat;
  } else {
    for (int i = 0; i + 1 < kM; ++i) {
      mem.ws(i) = mem.ws(i + 1);
      mem.wy(i) = mem.wy(i + 1);
      mem.ssd(i) = mem.ssd(i + 1);
      mem.syd(i) = mem.syd(i + 1);
    }
  }
  const int t = rg.col - 1;
  mem.ws(t) = s;
  mem.wy(t) = y;
  mem.ssd(t) = ssd;
  mem.syd(t) = syd;
}

// formt: T = theta SS + L D^-1 L' and its Cholesky factor; returns info.
// T's upper triangle: one entry per lane.
template <bool H = false>
NEMO_LB int formt(Mem& mem, const Ring& rg, double theta, Lanes L) {
#pragma clang fp contract(off)
  const int col = rg.col;
  double* wt = mem.wt();
  auto sy = [&](int i, int k) { return i == k ? mem.syd(i) : prod0(mem.ws(i), mem.wy(k)); };
  auto ss = [&](int i, int k) { return i == k ? mem.ssd(i) : prod0(mem.ws(i), mem.ws(k)); };
  for (int t = L.id; t < kM * col; t += L.n) {
    const int i = t % kM, j = t / kM;
    if (i > j) continue;
    if (i == 0) {
      wt[(long)j * kLdT] = theta * ss(0, j);
    } else {
      double ddum = 0.0;
      for (int k = 0; k < i; ++k) ddum = ddum + sy(i, k) * sy(j, k) / sy(k, k);
      wt[i + (long)j * kLdT] = ddum + theta * ss(i, j);
    }
  }
  lanes_sync();
  return ob_potrf_u<H>(col, wt, kLdT, L);
}

// formk for n = nsub = 1, the variable free and staying free: WN (upper,
// 2col x 2col, ld 2m) and its two Cholesky factorisations; info 0, -1, -2.
// WN's entries, the solve's right-hand sides and the (2,2) block's updates:
// one per lane.
template <bool H = false>
NEMO_LB int formk(Mem& mem, const Ring& rg, double theta, Lanes L) {
#pragma clang fp contract(off)
  const int col = rg.col, c2 = 2 * col;
  double* wn = mem.wn();
  auto at = [&](int r, int c) -> double& { return wn[r + (long)c * kLdN]; };
  for (int t = L.id; t < kLdN * c2; t += L.n) {
    const int r = t % kLdN, c = t / kLdN;
    if (r > c) continue;
    double v;
    if (c < col) {            // Y'ZZ'Y / theta, + s'y on the diagonal
      v = sum0(mem.wy(c), mem.wy(r)) / theta;
      if (r == c) v = v + mem.syd(c);
    } else if (r < col) {     // -L_a (zero: no active set) and R_z
      const int iy = c - col;
      v = r < iy ? -0.0 : sum0(mem.ws(iy), mem.wy(r));
    } else {                  // S'AA'S theta (no active set)
      v = 0.0 * theta;
    }
    at(r, c) = v;
  }
  lanes_sync();
  if (ob_potrf_u<H>(col, wn, kLdN, L) != 0) return -1;
  // L^-1 (-L_a' + R_z') in the (1,2) block: one dtrtrs call with nrhs = col
  double* b12 = wn + (long)col * kLdN;
  const int info = col == 1 ? ob_trsv_tun<H>(1, wn, kLdN, b12) : ob_trsm_lt<H>(col, col, wn, kLdN, b12, kLdN, L);
  if (info != 0) return -1;
  for (int t = L.id; t < kM * col; t += L.n) {
    const int a = t % kM, b = t / kM;
    if (a > b) continue;
    const int is = col + a, js = col + b;
    at(is, js) = at(is, js) + ob_ddot(col, wn + (long)is * kLdN, wn + (long)js * kLdN);
  }
  lanes_sync();
  if (ob_potrf_u<H>(col, wn + col + (long)col * kLdN, kLdN, L) != 0) return -2;
  return 0;
}

// subsm from z = x with r = -g (cmprlb, unconstrained): the Newton step;
// false when a triangular solve is singular (the caller restarts)
#if !defined(__HIP_DEVICE_COMPILE__)
template <bool H = false>
NEMO_LB bool subsm(Mem& mem, const Ring& rg, double theta, double r, double x, double& z, Lanes) {
#pragma clang fp contract(off)
  const int col = rg.col, c2 = 2 * col;
  double* wv = mem.wv();
  for (int i = 0; i < col; ++i) {
    wv[i] = sum0(mem.wy(i), r);
    wv[col + i] = theta * sum0(mem.ws(i), r);
  }
  const double* wn = mem.wn();
  if (ob_trsv_tun<H>(c2, wn, kLdN, wv) != 0) return false;
  for (int i = 0; i < col; ++i) wv[i] = -wv[i];
  if (ob_trsv_nun<H>(c2, wn, kLdN, wv) != 0) return false;
  double d = r;
  for (int jy = 0; jy < col; ++jy) d = d + mem.wy(jy) * wv[jy] / theta + mem.ws(jy) * wv[col + jy];
  d = d * (1.0 / theta);
  z = x + d;   // the projection step of L-BFGS-B 3.0 (no bounds: alpha = 1, same bits)
  return true;
}
#else
// The same on the wave, the work vector in registers (lane i holds wv[i]):
// the two triangular solves as pipelines over the lanes -- trsv_TUN's dot of
// row i accumulated on lane i as each earlier entry becomes final (the chain
// of ddot's order; rows >= 16 take ddot's 16-term block sum at step 16), and
// trsv_NUN's axpy updates applied by each lane to its own entry -- so a step
// costs one operation, not a dot product.
template <bool H = false>
__device__ __forceinline__ bool subsm(Mem& mem, const Ring& rg, double theta, double r, double x, double& z,
                                      Lanes L) {
#pragma clang fp contract(off)
  const int col = rg.col, c2 = 2 * col;
  const int ln = L.id;
  const double* wn = mem.wn();
  for (int i = 0; i < c2; ++i)   // dtrtrs checks the diagonal first (both solves: the same diagonal)
    if (uniH<H>(wn[i + (long)i * kLdN] == 0.0)) return false;
  double b = 0.0;
  if (ln < col) b = sum0(mem.wy(ln), r);
  else if (ln < c2) b = theta * sum0(mem.ws(ln - col), r);
  // trsv_TUN: b_i = (b_i - ddot(i, U(:, i), b)) / u_ii
  const double* ucol = wn + (long)(ln < c2 ? ln : 0) * kLdN;   // this lane's column of U
  double dot = 0.0;
  for (int k = 0; k < c2; ++k) {
    if (k == 16 && ln >= 16 && ln < c2) {   // ddot_k, n >= 16: 4 x 4 lanes over the first 16
      double t[4];
      for (int l = 0; l < 4; ++l) {
        const double a0 = fma_(ucol[l], bcast<H>(b, l), 0.0);
        const double a1 = fma_(ucol[4 + l], bcast<H>(b, 4 + l), 0.0);
        const double a2 = fma_(ucol[8 + l], bcast<H>(b, 8 + l), 0.0);
        const double a3 = fma_(ucol[12 + l], bcast<H>(b, 12 + l), 0.0);
        t[l] = ((a0 + a1) + a2) + a3;
      }
      dot = (t[0] + t[2]) + (t[1] + t[3]);
    }
    if (ln == k) {
      if (k > 0) b = b - dot;
      b = b / ucol[k];
    }
    const double bk = bcast<H>(b, k);
    if (ln > k && ln < c2 && (ln < 16 || k >= 16)) dot = fma_(bk, ucol[k], dot);
  }
  if (ln < col) b = -b;
  // trsv_NUN: b_j /= u_jj, then b_k -= b_j u_kj for k < j
  for (int j = c2 - 1; j >= 0; --j) {
    if (ln == j) b = b / wn[j + (long)j * kLdN];
    const double nb = -bcast<H>(b, j);
    if (ln < j) b = fma_(nb, wn[ln + (long)j * kLdN], b);
  }
  double d = r;
  for (int jy = 0; jy < col; ++jy)
    d = d + mem.wy(jy) * bcast<H>(b, jy) / theta + mem.ws(jy) * bcast<H>(b, col + jy);
  d = d * (1.0 / theta);
  z = x + d;   // the projection step of L-BFGS-B 3.0 (no bounds: alpha = 1, same bits)
  return true;
}
#endif

}  // namespace lbx

// (tools/ubench/exact_obj.hip times the parts of the control through this
// hook; in the library it is the statement itself)
#ifndef NEMO_LBX_T
#define NEMO_LBX_T(k, stmt) stmt
#endif

// The optimiser as a resumable machine ("reverse communication", as the
// Fortran original): lbx_run advances to the next evaluation the library
// would make (or to the end), the caller evaluates the objective at the two
// points of the forward difference and hands the values to lbx_feed.  On the
// device the whole state lives in LDS next to `mem`, so the objective's
// registers and the optimiser's never overlap.
struct LbxState {
  double theta, x, f, g, z, d, stp, xk, fold, gold, gdold, dtd;
  double x_eval, x1, x_last, f_last, g_last;
  lb::Dcsrch ls;
  lbx::Ring rg;
  int nfev, nit, ifun, status;
  bool in_ls, updatd, have_last;
};

NEMO_LB void lbx_init(LbxState& S, double x0) {
  S.theta = 1.0;
  S.x = x0; S.f = 0.0; S.g = 0.0;
  S.z = S.d = S.stp = S.xk = S.fold = S.gold = S.gdold = S.dtd = 0.0;
  S.x_eval = x0; S.x1 = x0;
  S.x_last = S.f_last = S.g_last = 0.0;
  S.ls = lb::Dcsrch{};
  S.rg = lbx::Ring{};
  S.nfev = S.nit = S.ifun = 0;
  S.status = -1;
  S.in_ls = S.updatd = S.have_last = false;
}

// scipy's ScalarFunction: f at x_eval and the forward difference at x1
NEMO_LB void lbx_feed(LbxState& S, double f0, double f1) {
#pragma clang fp contract(off)
  S.nfev += 2;
  S.f_last = f0;
  S.g_last = (f1 - f0) / (S.x1 - S.x_eval);
  S.have_last = true;
  S.x_last = S.x_eval;
}

// true: evaluate at (S.x_eval, S.x1) and lbx_feed; false: done, the result
// in S.x, S.f, S.nit, S.nfev, S.status
template <bool H = false>
NEMO_LB bool lbx_run(LbxState& S, lbx::Mem mem) {
#pragma clang fp contract(off)
  using namespace lb;
  using lbx::fma_;
  const double tol = (0.01 / kEpsMch) * kEpsMch;
  const double pgtol = 0.01;
  const int maxls = 20, maxiter = 15000, maxfun = 15000;
  const lbx::Lanes L = lbx::lanes<H>();
  auto restart = [&]() {
    S.rg = lbx::Ring{};
    S.theta = 1.0;
    S.updatd = false;
  };
  auto done = [&](double x, double f, int status) {
    S.x = x; S.f = f; S.status = status;
    return false;
  };
  for (;;) {
    // ---- the single evaluation site (the ScalarFunction memoises the last
    // point: a repeated x costs no evaluation)
    if (uniH<H>(!(S.have_last && S.x_eval == S.x_last))) {
      const double xe = S.x_eval;
      double h = 1e-8;
      if (uniH<H>((xe + h) - xe == 0.0)) h = kSqrtEps * (xe >= 0.0 ? 1.0 : -1.0) * dmax(1.0, fabs(xe));
      S.x1 = xe + h;
      return true;
    }
    double x = S.x_eval, f = S.f_last, g = S.g_last;
    if (uniH<H>(!S.in_ls)) {
      if (uniH<H>(fabs(g) <= pgtol)) { S.nit = 0; return done(x, f, 0); }
    } else {
      double stp = S.stp;
      int task;
      NEMO_LBX_T(0, task = S.ls.template step<H>(stp, f, lbx::prod0(g, S.d)));
      S.stp = stp;
      if (uniH<H>(task == 0)) {
        ++S.ifun;
        if (uniH<H>(S.ifun - 1 < maxls)) {
          S.x_eval = (stp == 1.0) ? S.z : stp * S.d + S.xk;
          continue;
        }
        task = -1;
      }
      if (uniH<H>(task < 0)) {  // line search failed: previous iterate, restart or give up
        x = S.xk; f = S.fold; g = S.gold;
        if (uniH<H>(S.rg.col == 0)) return done(x, f, 2);
        restart();
      } else {
        ++S.nit;
        if (uniH<H>(fabs(g) <= pgtol)) return done(x, f, 0);
        const double fold = S.fold;
        if (uniH<H>((fold - f) <= tol * dmax(dmax(fabs(fold), fabs(f)), 1.0))) return done(x, f, 1);
        if (uniH<H>(S.nit >= maxiter || S.nfev > maxfun)) return done(x, f, 3);
        double d = S.d;
        const double gdold = S.gdold;
        const double gd = lbx::prod0(g, d);
        const double r = g - S.gold;
        const double rr = lbx::prod0(r, r);
        double dr, ddum;
        if (stp == 1.0) { dr = gd - gdold; ddum = -gdold; }
        else { dr = (gd - gdold) * stp; d = d * stp; ddum = -gdold * stp; }
        S.d = d;
        if (uniH<H>(dr <= kEpsMch * ddum)) {
          S.updatd = false;
        } else {
          S.updatd = true;
          lbx::Ring rg = S.rg;
          S.theta = rr / dr;
          lbx::matupd(mem, rg, d, r, (stp == 1.0) ? S.dtd : stp * stp * S.dtd, dr);
          S.rg = rg;
          int ft;
          NEMO_LBX_T(1, ft = lbx::formt<H>(mem, rg, S.theta, L));
          if (uniH<H>(ft != 0)) restart();
        }
      }
    }
    // ---- the next search direction (cauchy at col = 0; else formk + subsm)
    for (;;) {
      double z;
      const double theta = S.theta;
      if (uniH<H>(S.rg.col == 0)) {
        const double neggi = -g;
        const double f1 = 0.0 - neggi * neggi;
        const double f2 = -theta * f1;
        double dtm = -f1 / f2;
        if (dtm <= 0.0) dtm = 0.0;
        z = fma_(0.0 + dtm, neggi, x);   // daxpy
      } else {
        const lbx::Ring rg = S.rg;
        int fk = 0;
        if (uniH<H>(S.updatd)) NEMO_LBX_T(2, fk = lbx::formk<H>(mem, rg, theta, L));
        if (uniH<H>(fk != 0)) {
          restart();
          continue;
        }
        double zz = x;
        bool ok;
        NEMO_LBX_T(3, ok = lbx::subsm<H>(mem, rg, theta, -g, x, zz, L));
        if (uniH<H>(!ok)) {
          restart();
          continue;
        }
        z = zz;
      }
      const double d = z - x;
      S.z = z;
      S.d = d;
      S.dtd = lbx::prod0(d, d);
      const double dnorm = fabs(d);    // dnrm2, n = 1
      const double stp = (S.nit == 0) ? dmin(1.0 / dnorm, kStpMax) : 1.0;
      S.stp = stp;
      S.xk = x; S.fold = f; S.gold = g;
      const double gdold = lbx::prod0(g, d);
      S.gdold = gdold;
      if (uniH<H>(gdold < 0.0)) {
        S.ls.stpmax = kStpMax;
        S.ls.template start<H>(stp, f, gdold);
        S.ifun = 1;
        S.in_ls = true;
        S.x_eval = (stp == 1.0) ? z : stp * d + x;
        break;
      }
      // lnsrlb: the directional derivative is not negative (info = -4)
      if (uniH<H>(S.rg.col == 0)) return done(x, f, 2);
      restart();
    }
  }
}

// Minimise the reference's unbounded 1-D objective from x0 with scipy's
// exact arithmetic (header); fg as lbfgsb1_minimize.  Status as there.
template <class FG>
NEMO_LB LbfgsResult lbfgsb1_minimize_exact(FG& fg, double x0, lbx::Mem mem) {
  LbxState S;
  lbx_init(S, x0);
  while (lbx_run(S, mem)) {
    double f0, f1;
    fg(S.x_eval, S.x1, f0, f1);
    lbx_feed(S, f0, f1);
  }
  return LbfgsResult{S.x, S.f, S.nit, S.nfev, S.status};
}

}  // namespace nemo
