// nemo_methods.hip -- the fixed-order weight optimizers of methods.py on the
// GPU.  Both reuse the order-score kernels for their
// evaluation and run the per-pair 1-D L-BFGS-B of lbfgsb1.h in its bounded
// form, one wave per (problem, pair).
//
//   Method.opt_gamma (methods.py:397-405): evaluation on the raw weights,
//     then every permissible pair minimises -sum_e log(g c_e + 1) with its
//     analytic gradient, bounds [0, 1], tol 0.01 (:385-395, local_ll_sum at
//     :8-9).  The pairs are independent.
//   InverseMethod.opt_b (methods.py:117-129): the weights are log-weights of
//     a DAG, M = order_arr(order, exp(W)) (utils.py:173: row/column a of M is
//     node pos[a]), the evaluation weights are B/(1+B) of B =
//     solve_triangular(I - M, I, lower=True); every pair minimises
//     -sum_e log(b c_e(b) + 1) in x = W[i][k] with b = B[a][b]/(1+B[a][b])
//     (:73-82), bounds [-5000, 500], forward differences with step 1e-3,
//     tol 0.1 (:106-115).  The loop updates W in place, so a pair sees the
//     optima of the pairs before it that lie on its paths; the host groups
//     the pairs into levels that respect exactly those reads (nemo_abi.cpp)
//     and every level is one launch plus a commit.
#include "nemo_internal.h"
#include "lbfgsb1.h"

#include <math.h>

namespace nemo {

namespace {

// wave sum on the line searches' serial path: DPP + permlane swaps (VALU),
// not a ds_bpermute tree (nemo_internal.h)
__device__ __forceinline__ double wsum_m(double v) { return wsum_dpp(v); }

// log for the objectives: the table log where it is defined, else the
// library log (0 -> -inf, negative -> NaN, as numpy gives)
__device__ __forceinline__ double log_obj(double t, const double2* ltab) {
  return (t >= 2.2250738585072014e-308 && t < __builtin_inf()) ? log_fast(t, ltab) : log(t);
}

__device__ __forceinline__ int32_t pack_info_m(const LbfgsResult& r) {
  const int nit = r.nit < 4095 ? r.nit : 4095;
  const int nfev = r.nfev < 32767 ? r.nfev : 32767;
  return (int32_t)(r.status | (nit << 4) | (nfev << 16));
}

// ---------------------------------------------------------------------------
// Method: f(g) = -sum log(g c + 1), f'(g) = -sum c / (g c + 1)
// ---------------------------------------------------------------------------
template <int NPL>
struct GammaObjective {
  double c[NPL];
  const double2* ltab;
  __device__ __forceinline__ void operator()(double x, double& f, double& g) const {
#pragma clang fp contract(off)
    double p = 0.0, q = 0.0;
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const double t = x * c[j] + 1.0;
      p += log_obj(t, ltab);
      q += c[j] / t;
    }
    f = -wsum_m(p);
    g = -wsum_m(q);
  }
};

template <typename TT, int NPL>
__global__ __launch_bounds__(256) void gamma_pairs_kernel(
    int S, int E, int npairs, int nprob, const TT* __restrict__ eT, const int32_t* __restrict__ pairs,
    const int32_t* __restrict__ rows, const double* __restrict__ w, const double* __restrict__ ow,
    double* __restrict__ wout, int32_t* __restrict__ info) {
  __shared__ double2 ltab[128];
  fill_log_table(ltab, threadIdx.x, blockDim.x);
  __syncthreads();
  const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (gw >= nprob * npairs) return;  // uniform per wave
  const int b = gw / npairs;
  const int n = gw - b * npairs;
  const int pk = pairs[(size_t)b * S * S + n];
  const int i = pk >> 16;
  const int k = pk & 0xffff;  // the parent node (prep_child_list)
  const size_t idx = ((size_t)b * S + i) * S + k;
  const double s = w[idx];
  const TT* tv = eT + ((size_t)i * S + k) * E;
  const double* owk = ow + ((size_t)b * (S + 1) + k) * E;  // order weights row k (:388)
  GammaObjective<NPL> obj;
  obj.ltab = ltab;
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    // branch-free setup (a clamped index past E, padding selected away), so
    // the loads and divisions of all elements overlap
    const int e = q * kWave + lane;
    const int ec = e < E ? e : E - 1;
    double cv;
    {
#pragma clang fp contract(off)
      const double lv = (double)tv[ec];
      const double a = (lv - 1.0) * owk[ec];
      const double bb = (1.0 - s * a) + s * (lv - 1.0);
      cv = a / bb;
    }
    obj.c[q] = e < E ? cv : 0.0;  // padding: log(1) = 0, c/(1) = 0
  }
  LbOpts o;
  o.lo = 0.0;
  o.hi = 1.0;
  const LbfgsResult r = lbfgsb1_minimize_opts<true, true>(obj, s, o);
  if (lane == 0) {
    wout[idx] = r.x;
    if (info) info[idx] = pack_info_m(r);
  }
}

// ---------------------------------------------------------------------------
// InverseMethod
// ---------------------------------------------------------------------------
// M[a][d] = exp(W[pos a][pos d]) of problem b (order_arr: index a is node pos[a])
__device__ __forceinline__ double mval(const double* __restrict__ wb, const int32_t* __restrict__ pb, int S,
                                       int a, int d) {
  return exp(wb[(size_t)pb[a] * S + pb[d]]);
}

// column `col` of B = (I - M)^-1 (lower triangle), rows col..last, by
// forward substitution with one wave: X_c = (sum_{col <= d < c} M[c][d] X_d)
// / (1 - M[c][c]).  X_d lives in lane (d - col) & 63, slot (d - col) >> 6.
template <int NS>
__device__ __forceinline__ void column_solve(const double* __restrict__ wb, const int32_t* __restrict__ pb, int S,
                                             int col, int last, int lane, double (&X)[NS]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int q = 0; q < NS; ++q) X[q] = 0.0;
  const double x0 = 1.0 / (1.0 - mval(wb, pb, S, col, col));
  if (lane == 0) X[0] = x0;
  for (int c = col + 1; c <= last; ++c) {
    double p = 0.0;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const int d = col + q * kWave + lane;
      if (d < c) p += mval(wb, pb, S, c, d) * X[q];
    }
    const double xc = wsum_m(p) / (1.0 - mval(wb, pb, S, c, c));
    const int off = c - col;
    if ((off & (kWave - 1)) == lane) {
#pragma unroll
      for (int q = 0; q < NS; ++q)
        if (q == (off >> 6)) X[q] = xc;
    }
  }
}

// out[b][pos c][pos col] = X_c / (1 + X_c): the evaluation weights of opt_b
// (methods.py:119-121) and the rounding of optimize (:160-164).  Entries of
// the upper triangle are 0.  One wave per column.
template <int NS>
__global__ __launch_bounds__(256) void ancestral_kernel(int S, int nprob, const int32_t* __restrict__ pos,
                                                        const double* __restrict__ w, double* __restrict__ out) {
  const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (gw >= nprob * S) return;
  const int b = gw / S;
  const int col = gw - b * S;
  const int32_t* pb = pos + (size_t)b * S;
  const double* wb = w + (size_t)b * S * S;
  double* ob = out + (size_t)b * S * S;
  double X[NS];
  column_solve<NS>(wb, pb, S, col, S - 1, lane, X);
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    // row c's X sits in lane off & 63, slot off >> 6 (shuffled with every
    // lane active; rows above the column read slot -1, i.e. 0)
    const int c = q * kWave + lane;
    const int off = c - col;
    double xv = 0.0;
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      const double t = __shfl(X[r], off & (kWave - 1), kWave);
      if (r == (off >> 6)) xv = t;
    }
    if (c < S) ob[(size_t)pb[c] * S + pb[col]] = (c >= col) ? xv / (1.0 + xv) : 0.0;
  }
}

// a_e = (lv_e - 1) ow[i][e] in registers; l1_e = lv_e - 1 in registers too
// when it fits (L1REG), else re-read from the table row every evaluation
template <typename TT, int NPL, bool L1REG>
struct InverseObjective {
  double a[NPL];
  double l1[L1REG ? NPL : 1];
  const TT* tv;            // exp(T[i][k]) row (L1REG = false)
  int lane, E;
  double xb, r, da;        // B[a][b](x) = (e^x X_b + R) / (1 - M[a][a])
  const double2* ltab;
  __device__ __forceinline__ double beta(double x) const {
#pragma clang fp contract(off)
    const double bv = (exp(x) * xb + r) / da;
    return bv / (1.0 + bv);
  }
  __device__ __forceinline__ double lm1(int j) const {
    if constexpr (L1REG) {
      return l1[j];
    } else {
      const int e = j * kWave + lane;
      return e < E ? (double)tv[e] - 1.0 : 0.0;
    }
  }
  __device__ __forceinline__ void operator()(double x0, double x1, double& f0, double& f1) const {
#pragma clang fp contract(off)
    const double b0 = beta(x0), b1 = beta(x1);
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const double l = lm1(j);
      const double c0 = a[j] / ((1.0 - b0 * a[j]) + b0 * l);
      const double c1 = a[j] / ((1.0 - b1 * a[j]) + b1 * l);
      p0 += log_obj(b0 * c0 + 1.0, ltab);
      p1 += log_obj(b1 * c1 + 1.0, ltab);
    }
    f0 = -wsum_m(p0);
    f1 = -wsum_m(p1);
  }
};

// one level of opt_b's pair loop: list entries (problem << 16 | i << 8 | k)
template <typename TT, int NPL, int NS>
__global__ __launch_bounds__(256) void inverse_pairs_kernel(
    int S, int E, int n, const int32_t* __restrict__ list, const int32_t* __restrict__ pos,
    const double* __restrict__ w, const TT* __restrict__ eT, const double* __restrict__ ow,
    double* __restrict__ xout, int32_t* __restrict__ info) {
  __shared__ double2 ltab[128];
  fill_log_table(ltab, threadIdx.x, blockDim.x);
  __syncthreads();
  const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (gw >= n) return;
  const int ent = list[gw];
  const int b = ent >> 16;
  const int i = (ent >> 8) & 0xff;
  const int k = ent & 0xff;
  const int32_t* pb = pos + (size_t)b * S;
  const double* wb = w + (size_t)b * S * S;
  // a, c: the indices of i and k in order_arr's arrangement (pos[a] = i)
  int ra = -1, rb = -1;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int d = q * kWave + lane;
    if (d < S) {
      const int nd = pb[d];
      if (nd == i) ra = d;
      if (nd == k) rb = d;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    ra = max(ra, __shfl_xor(ra, o, kWave));
    rb = max(rb, __shfl_xor(rb, o, kWave));
  }
  double X[NS];
  column_solve<NS>(wb, pb, S, rb, ra - 1, lane, X);
  // R = sum_{rb < d < ra} M[ra][d] X_d;  X_b in lane 0 slot 0
  double p = 0.0;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int d = rb + q * kWave + lane;
    if (d > rb && d < ra) p += mval(wb, pb, S, ra, d) * X[q];
  }
  InverseObjective<TT, NPL, (NPL <= 32)> obj;
  obj.ltab = ltab;
  obj.lane = lane;
  obj.E = E;
  obj.r = wsum_m(p);
  obj.xb = __shfl(X[0], 0, kWave);
  obj.da = 1.0 - mval(wb, pb, S, ra, ra);
  const TT* tv = eT + ((size_t)i * S + k) * E;
  obj.tv = tv;
  const double* owi = ow + ((size_t)b * (S + 1) + i) * E;  // order weights row i (:108)
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int e = q * kWave + lane;
    double av = 0.0, lv1 = 0.0;
    if (e < E) {
      lv1 = (double)tv[e] - 1.0;
      av = lv1 * owi[e];
    }
    obj.a[q] = av;
    if constexpr (NPL <= 32) obj.l1[q] = lv1;
  }
  LbOpts o;
  o.ftol = o.gtol = 0.1;
  o.eps = 1e-3;
  o.lo = -5000.0;
  o.hi = 500.0;
  const size_t idx = ((size_t)b * S + i) * S + k;
  const LbfgsResult r = lbfgsb1_minimize_opts<true, false>(obj, wb[(size_t)i * S + k], o);
  if (lane == 0) {
    xout[idx] = r.x;
    if (info) info[idx] = pack_info_m(r);
  }
}

__global__ void commit_kernel(int S, int n, const int32_t* __restrict__ list, const double* __restrict__ xout,
                              double* __restrict__ w) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int ent = list[t];
  const size_t idx = ((size_t)(ent >> 16) * S + ((ent >> 8) & 0xff)) * S + (ent & 0xff);
  w[idx] = xout[idx];
}

int npl_m(int E) {
  const int need = (E + kWave - 1) / kWave;
  const int sizes[] = {4, 8, 16, 32, 48, 64, 80};
  for (int v : sizes)
    if (need <= v) return v;
  return -1;
}

#define NEMO_NPL_SWITCH(E, MACRO) \
  switch (npl_m(E)) {             \
    case 4: MACRO(4); break;      \
    case 8: MACRO(8); break;      \
    case 16: MACRO(16); break;    \
    case 32: MACRO(32); break;    \
    case 48: MACRO(48); break;    \
    case 64: MACRO(64); break;    \
    case 80: MACRO(80); break;    \
    default: return hipErrorInvalidValue; \
  }

template <typename TT>
hipError_t gamma_t(Ctx& c, int nprob, int npairs, const int32_t* d_pairs, const int32_t* d_rows,
                   const double* d_w, const double* d_ow, double* d_wout, int32_t* d_info, hipStream_t st) {
  const int blocks = (int)(((size_t)nprob * npairs + 3) / 4);
  const TT* eT = (const TT*)c.d_eT;
#define NEMO_G(NPL) \
  gamma_pairs_kernel<TT, NPL><<<blocks, 256, 0, st>>>(c.S, c.E, npairs, nprob, eT, d_pairs, d_rows, d_w, d_ow, d_wout, d_info)
  NEMO_NPL_SWITCH(c.E, NEMO_G)
#undef NEMO_G
  return hipGetLastError();
}

template <typename TT, int NS>
hipError_t inverse_t(Ctx& c, int n, const int32_t* d_list, const int32_t* d_pos, const double* d_w,
                     const double* d_ow, double* d_xout, int32_t* d_info, hipStream_t st) {
  const int blocks = (n + 3) / 4;
  const TT* eT = (const TT*)c.d_eT;
#define NEMO_I(NPL) \
  inverse_pairs_kernel<TT, NPL, NS><<<blocks, 256, 0, st>>>(c.S, c.E, n, d_list, d_pos, d_w, eT, d_ow, d_xout, d_info)
  NEMO_NPL_SWITCH(c.E, NEMO_I)
#undef NEMO_I
  return hipGetLastError();
}

}  // namespace

hipError_t launch_gamma_pairs(Ctx& c, int nprob, int npairs, const int32_t* d_pairs, const int32_t* d_rows,
                              const double* d_w, const double* d_ow, double* d_wout, int32_t* d_info,
                              hipStream_t st) {
  if ((size_t)nprob * npairs == 0) return hipSuccess;
  if (c.dtype == 0) return gamma_t<double>(c, nprob, npairs, d_pairs, d_rows, d_w, d_ow, d_wout, d_info, st);
  return gamma_t<float>(c, nprob, npairs, d_pairs, d_rows, d_w, d_ow, d_wout, d_info, st);
}

hipError_t launch_ancestral(Ctx& c, int nprob, const int32_t* d_pos, const double* d_w, double* d_out,
                            hipStream_t st) {
  if (nprob == 0) return hipSuccess;
  const int blocks = (int)(((size_t)nprob * c.S + 3) / 4);
  if (c.S <= 64) ancestral_kernel<1><<<blocks, 256, 0, st>>>(c.S, nprob, d_pos, d_w, d_out);
  else if (c.S <= 128) ancestral_kernel<2><<<blocks, 256, 0, st>>>(c.S, nprob, d_pos, d_w, d_out);
  else ancestral_kernel<4><<<blocks, 256, 0, st>>>(c.S, nprob, d_pos, d_w, d_out);
  return hipGetLastError();
}

hipError_t launch_inverse_level(Ctx& c, int n, const int32_t* d_list, const int32_t* d_pos, double* d_w,
                                const double* d_ow, double* d_xout, int32_t* d_info, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipError_t e;
  if (c.dtype == 0) {
    if (c.S <= 64) e = inverse_t<double, 1>(c, n, d_list, d_pos, d_w, d_ow, d_xout, d_info, st);
    else if (c.S <= 128) e = inverse_t<double, 2>(c, n, d_list, d_pos, d_w, d_ow, d_xout, d_info, st);
    else e = inverse_t<double, 4>(c, n, d_list, d_pos, d_w, d_ow, d_xout, d_info, st);
  } else {
    if (c.S <= 64) e = inverse_t<float, 1>(c, n, d_list, d_pos, d_w, d_ow, d_xout, d_info, st);
    else if (c.S <= 128) e = inverse_t<float, 2>(c, n, d_list, d_pos, d_w, d_ow, d_xout, d_info, st);
    else e = inverse_t<float, 4>(c, n, d_list, d_pos, d_w, d_ow, d_xout, d_info, st);
  }
  if (e != hipSuccess) return e;
  commit_kernel<<<(n + 255) / 256, 256, 0, st>>>(c.S, n, d_list, d_xout, d_w);
  return hipGetLastError();
}

}  // namespace nemo
