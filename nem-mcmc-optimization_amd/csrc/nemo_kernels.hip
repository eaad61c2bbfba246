// nemo_kernels.hip -- gfx950 kernels of the NEM order-score engine.
//
// Hot path:
//   A4+A5  order score  : cell[i][e] = U[i][e] + sum_{j in pa(i)} log(1 - w_ij + w_ij*exp(T[i][j][e]))
//                          cs[e] = logsumexp_i cell[i][e];  ll = sum_e cs[e]
//                          (nem_order_mcmc.py:79-93, utils.py:84-94)
//   A8     local optimum: one L-BFGS-B 1-D solve per permissible (i, k) pair
//                          (nem_order_mcmc.py:18-23, 160-170)
//
// Layout in HBM (all row-major): eT = exp(T) [S][S][E] in the table dtype,
// U [S+1][E] in the table dtype, per-evaluation parent lists built by
// prep_kernel.  A score block owns 64 effects (one per lane) of one
// evaluation and splits the S children over its 4 waves; every wave streams
// the table rows of its children's permissible parents (one coalesced
// 64-lane row segment per parent) and keeps the per-child sum of logs as a
// running PRODUCT (one multiply per element, one log per child), then the
// waves merge online log-sum-exp states through LDS.
#include "nemo_internal.h"
#include "lbfgsb1.h"

#include <math.h>

namespace nemo {

namespace {

constexpr double kLn2 = 0.69314718055994530942;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// online log-sum-exp state (m = running max, l = sum of exp(c - m))
__device__ __forceinline__ void lse_push(double& m, double& l, double c) {
  if (c == -INFINITY) return;
  if (c > m) {
    l = l * exp(m - c) + 1.0;
    m = c;
  } else {
    l += exp(c - m);
  }
}

__device__ __forceinline__ void lse_merge(double& m, double& l, double m2, double l2) {
  if (l2 == 0.0) return;
  if (l == 0.0) { m = m2; l = l2; return; }
  const double mx = m > m2 ? m : m2;
  l = l * exp(m - mx) + l2 * exp(m2 - mx);
  m = mx;
}

// XCD-aware block order (MI355X_MICROARCH.md: blocks are dealt round-robin to
// the 8 XCDs, so block L runs on XCD L % 8).  Remap the 1-D block index to a
// work index so that each XCD receives a CONTIGUOUS range of the tile-major
// work list: the blocks in flight on one XCD then share the same 64-effect
// table columns, which stay in that XCD's 4 MB L2.  Bijective for any N;
// placement only changes speed, never results.
__device__ __forceinline__ int xcd_work_index(int L, int N, int remap) {
  if (!remap) return L;
  const int x = L & 7, k = L >> 3;
  const int q = N >> 3, r = N & 7;
  return x * q + (x < r ? x : r) + k;
}

template <typename TT> struct Acc;
template <> struct Acc<double> {
  using T = double;
  __device__ static T term(double s, double v) { return fma(s, v - 1.0, 1.0); }
  __device__ static T renorm(T p, int& ex) { int e; T r = frexp(p, &e); ex += e; return r; }
};
template <> struct Acc<float> {
  using T = float;
  __device__ static T term(float s, float v) { return fmaf(s, v - 1.0f, 1.0f); }
  __device__ static T renorm(T p, int& ex) { int e; T r = frexpf(p, &e); ex += e; return r; }
};

// ---------------------------------------------------------------------------
// exp of the staged table (once per model)
// ---------------------------------------------------------------------------
template <typename TT>
__global__ void exp_table_kernel(size_t n, const double* __restrict__ t64, TT* __restrict__ out) {
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n;
       k += (size_t)gridDim.x * blockDim.x)
    out[k] = (TT)exp(t64[k]);
}

// ---------------------------------------------------------------------------
// prep: per evaluation, per child i, the permissible parents in pi order
// (nem_order_mcmc.py:62-65; with cap, the last `cap` of them) and their
// weights; plus the flat (child, list index) pair list for the local optima.
// grid = batch * ceil(S / 4), block = 256: one wave per child, one lane per
// list slot (so a chain's prep is ceil(S / 4) blocks, not one serial loop per
// child); every block rebuilds the evaluation's order and the prefix sums of
// the list lengths in LDS (S <= 256).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prep_kernel(int S, int cap, const int32_t* __restrict__ pos,
                                                   const double* __restrict__ w01, int32_t* __restrict__ rows,
                                                   double* __restrict__ sw, int32_t* __restrict__ cnt,
                                                   int32_t* __restrict__ pairs, int32_t* __restrict__ info) {
  __shared__ int perm[kMaxS];
  __shared__ int scan[kMaxS];
  const int nblk = (S + 3) / 4;
  const int b = blockIdx.x / nblk;
  const int i = (blockIdx.x - b * nblk) * 4 + (int)(threadIdx.x / kWave);  // this wave's child
  const int32_t* pb = pos + (size_t)b * S;
  prep_order_lds(S, cap, pb, perm, scan, pairs != nullptr);
  if (i >= S) return;  // uniform per wave
  prep_child_list(S, cap, pb, w01, rows, sw, cnt, pairs, info, b, i, perm, scan, threadIdx.x & (kWave - 1));
}

// ---------------------------------------------------------------------------
// score: one evaluation x 64 effects per block, children split over waves.
// grid = ntiles * batch (1-D, XCD-remapped), block = kScoreWaves * 64.
// ---------------------------------------------------------------------------
template <typename TT, bool RENORM>
__global__ __launch_bounds__(kScoreWaves * kWave) void score_kernel(
    int S, int E, int ntiles, const TT* __restrict__ eT, const TT* __restrict__ U,
    const int32_t* __restrict__ rows, const double* __restrict__ sw,
    const int32_t* __restrict__ cnt, double* __restrict__ partial, double* __restrict__ cs_out,
    double* __restrict__ cells, double* __restrict__ ow, int remap) {
  using A = Acc<TT>;
  using PT = typename A::T;
  __shared__ double sm_m[kScoreWaves][kWave];
  __shared__ double sm_l[kScoreWaves][kWave];
  __shared__ double sm_cs[kWave];
  const int batch = (int)gridDim.x / ntiles;
  const int work = xcd_work_index((int)blockIdx.x, (int)gridDim.x, remap);
  const int tile = work / batch;       // tile-major: consecutive work shares columns
  const int b = work - tile * batch;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int e = tile * kTileCols + lane;
  const bool valid = e < E;
  const int ec = valid ? e : E - 1;
  double* park = cells ? cells : ow;  // where cell values wait for the ow pass

  double m = -INFINITY, l = 0.0;
  for (int i = w; i < S; i += kScoreWaves) {
    const int n = __builtin_amdgcn_readfirstlane(cnt[(size_t)b * S + i]);
    const int32_t* rp = rows + ((size_t)b * S + i) * S;
    const double* wp = sw + ((size_t)b * S + i) * S;
    const TT* base = eT + (size_t)i * S * E + ec;
    PT prod = (PT)1;
    int expo = 0;
    int t = 0;
    for (; t + 8 <= n; t += 8) {
      int jj[8];
      double ss[8];
      TT vv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        jj[k] = rp[t + k];
        ss[k] = wp[t + k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) vv[k] = base[(size_t)jj[k] * E];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        prod *= A::term((PT)ss[k], vv[k]);
        if (RENORM && (k & 3) == 3) prod = A::renorm(prod, expo);
      }
    }
    for (; t < n; ++t) {
      const int j = rp[t];
      prod *= A::term((PT)wp[t], base[(size_t)j * E]);
      if (RENORM) prod = A::renorm(prod, expo);
    }
    double cell = (double)U[(size_t)i * E + ec] + log((double)prod);
    if (RENORM) cell += (double)expo * kLn2;
    if (park && valid) park[((size_t)b * (S + 1) + i) * E + e] = cell;
    lse_push(m, l, cell);
  }
  sm_m[w][lane] = m;
  sm_l[w][lane] = l;
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int k = 1; k < kScoreWaves; ++k) lse_merge(m, l, sm_m[k][lane], sm_l[k][lane]);
    const double cnull = (double)U[(size_t)S * E + ec];  // row S: attached to nothing
    if (park && valid) park[((size_t)b * (S + 1) + S) * E + e] = cnull;
    lse_push(m, l, cnull);
    const double cs = m + log(l);
    sm_cs[lane] = cs;
    if (cs_out && valid) cs_out[(size_t)b * E + e] = cs;
    const double part = wave_sum(valid ? cs : 0.0);
    if (lane == 0) partial[(size_t)b * ntiles + tile] = part;
  }
  if (ow == nullptr) return;
  __syncthreads();
  const double cs = sm_cs[lane];
  if (!valid) return;
  for (int i = w; i <= S; i += kScoreWaves) {
    const size_t k = ((size_t)b * (S + 1) + i) * E + e;
    ow[k] = exp(park[k] - cs);
  }
}

// ll[b] = sum over tiles (fixed order: bitwise reproducible)
__global__ void finalize_kernel(int batch, int ntiles, const double* __restrict__ partial,
                                double* __restrict__ ll) {
  // one wave per evaluation: strided lane sums then a fixed xor tree
  // (bitwise reproducible)
  const int b = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  if (b >= batch) return;
  double s = 0.0;
  for (int t = lane; t < ntiles; t += kWave) s += partial[(size_t)b * ntiles + t];
  s = wave_sum(s);
  if (lane == 0) ll[b] = s;
}

// ---------------------------------------------------------------------------
// grouped (reuse) score: CB evaluations share every table row a block reads.
// prep_group: for group g and child i, the parents any member needs (ascending
// j) and a [t][CB] weight block (0 where the member has no such parent).
// ---------------------------------------------------------------------------
template <int CB>
__global__ void prep_group_kernel(int S, int batch, int cap, const int32_t* __restrict__ pos,
                                  const double* __restrict__ w01, int32_t* __restrict__ rows,
                                  double* __restrict__ sw, int32_t* __restrict__ cnt) {
  __shared__ int sp[CB][kMaxS];
  const int g = blockIdx.x;
  const int i = threadIdx.x;
  const int b0 = g * CB;
  for (int q = 0; q < CB; ++q)
    if (i < S) sp[q][i] = (b0 + q < batch) ? pos[(size_t)(b0 + q) * S + i] : 0;
  __syncthreads();
  if (i >= S) return;
  int32_t* r = rows + ((size_t)g * S + i) * S;
  double* w = sw + ((size_t)g * S + i) * S * CB;
  int t = 0;
  for (int j = 0; j < S; ++j) {
    if (j == i) continue;
    bool any = false;
    double wt[CB];
#pragma unroll
    for (int q = 0; q < CB; ++q) {
      const int gap = sp[q][i] - sp[q][j];
      const bool ok = (b0 + q < batch) && gap > 0 && (cap == 0 || gap <= cap);
      wt[q] = ok ? w01[((size_t)(b0 + q) * S + i) * S + j] : 0.0;
      any |= ok;
    }
    if (!any) continue;
    r[t] = j;
#pragma unroll
    for (int q = 0; q < CB; ++q) w[(size_t)t * CB + q] = wt[q];
    ++t;
  }
  cnt[(size_t)g * S + i] = t;
}

// grid = (ntiles, ngroups), block = GW waves; dynamic LDS: GW * (S-1) * CB
// doubles of weights (wave-private), reused for the LSE merge.
template <typename TT, int CB, int GW>
__global__ __launch_bounds__(GW * kWave) void score_group_kernel(
    int S, int E, int ntiles, int batch, const TT* __restrict__ eT, const TT* __restrict__ U,
    const int32_t* __restrict__ rows, const double* __restrict__ sw,
    const int32_t* __restrict__ cnt, double* __restrict__ partial, int remap) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int ngroups = (int)gridDim.x / ntiles;
  const int work = xcd_work_index((int)blockIdx.x, (int)gridDim.x, remap);
  const int tile = work / ngroups;
  const int g = work - tile * ngroups;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int e = tile * kTileCols + lane;
  const bool valid = e < E;
  const int ec = valid ? e : E - 1;
  double* wl = lds + (size_t)w * (S - 1) * CB;
  double m[CB], l[CB];
#pragma unroll
  for (int q = 0; q < CB; ++q) { m[q] = -INFINITY; l[q] = 0.0; }
  for (int i = w; i < S; i += GW) {
    const int n = __builtin_amdgcn_readfirstlane(cnt[(size_t)g * S + i]);
    const int32_t* rp = rows + ((size_t)g * S + i) * S;
    const double* wp = sw + ((size_t)g * S + i) * S * CB;
    for (int k = lane; k < n * CB; k += kWave) wl[k] = wp[k];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const TT* base = eT + (size_t)i * S * E + ec;
    double prod[CB];
#pragma unroll
    for (int q = 0; q < CB; ++q) prod[q] = 1.0;
    int t = 0;
    for (; t + 4 <= n; t += 4) {
      double vv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) vv[k] = (double)base[(size_t)rp[t + k] * E];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double wv = vv[k] - 1.0;
#pragma unroll
        for (int q = 0; q < CB; ++q) prod[q] *= fma(wl[(t + k) * CB + q], wv, 1.0);
      }
    }
    for (; t < n; ++t) {
      const double wv = (double)base[(size_t)rp[t] * E] - 1.0;
#pragma unroll
      for (int q = 0; q < CB; ++q) prod[q] *= fma(wl[t * CB + q], wv, 1.0);
    }
    const double u = (double)U[(size_t)i * E + ec];
#pragma unroll
    for (int q = 0; q < CB; ++q) lse_push(m[q], l[q], u + log(prod[q]));
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // merge: waves write states over the (now free) weight region
  double* mm = lds;                       // [GW][CB][64]
  double* ll = lds + (size_t)GW * CB * kWave;
#pragma unroll
  for (int q = 0; q < CB; ++q) {
    mm[((size_t)w * CB + q) * kWave + lane] = m[q];
    ll[((size_t)w * CB + q) * kWave + lane] = l[q];
  }
  __syncthreads();
  if (w != 0) return;
  const double unull = (double)U[(size_t)S * E + ec];
#pragma unroll
  for (int q = 0; q < CB; ++q) {
    for (int k = 1; k < GW; ++k)
      lse_merge(m[q], l[q], mm[((size_t)k * CB + q) * kWave + lane],
                ll[((size_t)k * CB + q) * kWave + lane]);
    lse_push(m[q], l[q], unull);
    const double cs = m[q] + log(l[q]);
    const double part = wave_sum(valid ? cs : 0.0);
    const int b = g * CB + q;
    if (lane == 0 && b < batch) partial[(size_t)b * ntiles + tile] = part;
  }
}

// ---------------------------------------------------------------------------
// LSE over a given cell matrix (utils.compute_ll / calculate_ll)
// ---------------------------------------------------------------------------
__global__ void lse_kernel(int rows, int E, int ntiles, const double* __restrict__ cells,
                           double* __restrict__ partial, double* __restrict__ cs_out,
                           double* __restrict__ ow) {
  const int e = blockIdx.x * kWave + threadIdx.x;
  const bool valid = e < E;
  const int ec = valid ? e : E - 1;
  double m = -INFINITY, l = 0.0;
  for (int i = 0; i < rows; ++i) lse_push(m, l, cells[(size_t)i * E + ec]);
  const double cs = m + log(l);
  if (valid && cs_out) cs_out[e] = cs;
  const double part = wave_sum(valid ? cs : 0.0);
  if (threadIdx.x == 0) partial[blockIdx.x] = part;
  if (ow && valid)
    for (int i = 0; i < rows; ++i) ow[(size_t)i * E + e] = exp(cells[(size_t)i * E + e] - cs);
}

// ---------------------------------------------------------------------------
// local optimum: one wave per problem, c kept in registers (NPL per lane)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double expit_d(double x) { return 1.0 / (1.0 + exp(-x)); }

// One row of exp(T) (TT = double or float) or of the order weights, read
// through a buffer resource bounded to the row: element q * 64 + lane is the
// lane's byte offset (one VGPR, fixed) plus a scalar offset, and a read past
// the row's E elements returns 0 instead of faulting -- no per-element clamp
// or address arithmetic in the setup of a local optimum.
struct RowRsrc {
  __amdgpu_buffer_rsrc_t r;
  template <typename T>
  __device__ __forceinline__ RowRsrc(const T* row, int E)
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)row, (short)0, E * (int)sizeof(T), 0x00020000)) {}
  template <typename T>
  __device__ __forceinline__ double at(int lane, int q) const {  // element q * 64 + lane
    if constexpr (sizeof(T) == 8)
      return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)lane * 8u, q * 64 * 8, 0));
    else
      return (double)__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)lane * 4u, q * 64 * 4, 0));
  }
};

// c = a / b with a = (lv - 1)*ow_k, b = 1 - s*a + s*(lv - 1)
// (nem_order_mcmc.py:161-164), operation order kept, no contraction.
__device__ __forceinline__ double local_c(double lv, double owk, double s) {
#pragma clang fp contract(off)
  const double a = (lv - 1.0) * owk;
  const double b = (1.0 - s * a) + s * (lv - 1.0);
  return a / b;
}

// PROD: sum_e log(c_e e + 1) as the log of a product -- per lane, chains of
// 4 factors renormalised by frexp and combined in a fixed tree (the caller
// guarantees the factors stay in range: |T| <= 40 makes each factor lie in
// [e^-80, e^80]) and ONE log per lane, instead of a log per element.  Every
// factor is > 0 for weights in [0, 1] (1 + e a / b = (b + e a) / b with b =
// 1 + s (lv - 1)(1 - ow) > 0), as the reference's log needs too.
template <int NPL, bool PROD>
struct LocalObjective {
  double c[NPL];  // this lane's share of the c vector, kept in registers
  double anc;
  const double2* ltab;  // log_fast table (LDS)
#ifdef NEMO_LO_TRACE
  // cycle probe: a build with -DNEMO_LO_TRACE=<nfev> prints, for every pair
  // needing at least that many f-evaluations, the cycles of its minimisation
  // and of the objective's parts (expit, products, log + wave sums); run
  // tools/lo_stats.py with NEMO_LIBRARY pointing at that build
  mutable long long cy_exp = 0, cy_prod = 0, cy_tail = 0, cy_calls = 0, cy_ls = 0;
#endif
  __device__ __forceinline__ void operator()(double x0, double x1, double& f0, double& f1) const {
#pragma clang fp contract(off)
#ifdef NEMO_LO_TRACE
    const long long t0 = clock64();
#endif
    const double e0 = expit_d(x0);
    const double e1 = expit_d(x1);
#ifdef NEMO_LO_TRACE
    const long long te = clock64();
    long long tp = te;
#endif
    double p0 = 0.0, p1 = 0.0;
    if constexpr (PROD) {
      constexpr double kLn2Hi = 0x1.62e42fefa3800p-1;
      constexpr double kLn2Lo = 5.4956039718945254e-14;
      // NC independent chains of 4 factors (chain u: elements 4u .. 4u + 3 of
      // the lane) multiplied in a fixed pairwise tree, renormalised by frexp
      // after its first level: the dependent chain of an f-evaluation (the
      // line search's serial path) is 4 + log2(NC) products instead of NPL.
      // A factor lies in [e^-80, e^80] for |T| <= 40, so 8 of them stay
      // normal, and a product of <= 16 mantissas in [0.5, 1) too.
      constexpr int NC = NPL / 4;
      double m0[NC], m1[NC];
      int k0 = 0, k1 = 0;
#pragma unroll
      for (int u = 0; u < NC; ++u) {
        // one FMA per factor (the reference rounds c e and + 1 separately;
        // the product form already departs from its sum of logs)
        double a0 = fma(c[4 * u], e0, 1.0), a1 = fma(c[4 * u], e1, 1.0);
#pragma unroll
        for (int v = 1; v < 4; ++v) {
          a0 *= fma(c[4 * u + v], e0, 1.0);
          a1 *= fma(c[4 * u + v], e1, 1.0);
        }
        m0[u] = a0;
        m1[u] = a1;
      }
      // the tree's first level multiplies two chains' raw products (8 factors
      // in [e^-640, e^640]: normal, so the rounding is that of their mantissas'
      // product), then renormalises: half the frexps of renormalising every
      // chain, and the same bits (an exact power of 2 never changes a
      // product's rounding); deeper levels multiply mantissas in [0.5, 1)
      if constexpr (NC == 1) {
        k0 += __builtin_amdgcn_frexp_exp(m0[0]);
        m0[0] = __builtin_amdgcn_frexp_mant(m0[0]);
        k1 += __builtin_amdgcn_frexp_exp(m1[0]);
        m1[0] = __builtin_amdgcn_frexp_mant(m1[0]);
      }
#pragma unroll
      for (int u = 0; u + 1 < NC; u += 2) {
        m0[u] *= m0[u + 1];
        m1[u] *= m1[u + 1];
        k0 += __builtin_amdgcn_frexp_exp(m0[u]);
        m0[u] = __builtin_amdgcn_frexp_mant(m0[u]);
        k1 += __builtin_amdgcn_frexp_exp(m1[u]);
        m1[u] = __builtin_amdgcn_frexp_mant(m1[u]);
      }
#pragma unroll
      for (int wd = 2; wd < NC; wd *= 2)
#pragma unroll
        for (int u = 0; u + wd < NC; u += 2 * wd) {
          m0[u] *= m0[u + wd];
          m1[u] *= m1[u + wd];
        }
      k0 += __builtin_amdgcn_frexp_exp(m0[0]);
      k1 += __builtin_amdgcn_frexp_exp(m1[0]);
      const double r0 = __builtin_amdgcn_frexp_mant(m0[0]), r1 = __builtin_amdgcn_frexp_mant(m1[0]);
#ifdef NEMO_LO_TRACE
      __builtin_amdgcn_s_waitcnt(0);
      tp = clock64();
#endif
      p0 = fma((double)k0, kLn2Hi, log_fast(r0, ltab)) + (double)k0 * kLn2Lo;
      p1 = fma((double)k1, kLn2Hi, log_fast(r1, ltab)) + (double)k1 * kLn2Lo;
    } else {
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        p0 += log_fast(c[q] * e0 + 1.0, ltab);
        p1 += log_fast(c[q] * e1 + 1.0, ltab);
      }
    }
    // wave sums by DPP + permlane swaps (VALU): the f-evaluation is on the
    // serial critical path of the line search, and a ds_bpermute tree adds
    // six LDS round trips to it
    p0 = wsum_dpp(p0);
    p1 = wsum_dpp(p1);
    // nem_order_mcmc.py:20-22: (-sum + |ex - anc|) + ex*(1 - ex)
    f0 = (-p0 + fabs(e0 - anc)) + e0 * (1.0 - e0);
    f1 = (-p1 + fabs(e1 - anc)) + e1 * (1.0 - e1);
#ifdef NEMO_LO_TRACE
    const long long t3 = clock64();
    cy_exp += te - t0;
    cy_prod += tp - te;
    cy_tail += t3 - tp;
    cy_calls += 1;
#endif
  }
};

__device__ __forceinline__ int32_t pack_info(const LbfgsResult& r) {
  const int nit = r.nit < 4095 ? r.nit : 4095;
  const int nfev = r.nfev < 32767 ? r.nfev : 32767;
  return (int32_t)(r.status | (nit << 4) | (nfev << 16));
}

// occupancy target of the local-optimum kernel: 3 waves per SIMD (168
// VGPRs) hide more of the serial line-search latency than 2
#ifndef NEMO_LOCAL_OPT_WAVES
#define NEMO_LOCAL_OPT_WAVES 3
#endif
constexpr int kLocalOptWavesPerSimd = NEMO_LOCAL_OPT_WAVES;
// at most this many (chain, pair) problems take the 4-wave split form under
// auto.  0: measured slower for one chain at C3 (84 against 75-79 us per
// launch, tools/step_probe.py): a lone wave's f-evaluation is bound by its
// dependent chain (expit, log, wave sums, the line-search logic), not by the
// products the split divides, and the split adds a barrier and an LDS round
// trip per f-evaluation.  Kept for A/B (option local_split = 2; same bits).
#ifndef NEMO_LOCAL_SPLIT_MAX
#define NEMO_LOCAL_SPLIT_MAX 0
#endif
constexpr int kLocalSplitMax = NEMO_LOCAL_SPLIT_MAX;

// eval #1's partial sums alone (the split local-optimum path and steps with
// no pair): finalize_factored_kernel's work
__global__ void finalize_factored_sums(FinalizeArgs fin) {
  const int e = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  if (e >= fin.batch) return;
  const double v = sum_partials(fin.partial + (size_t)e * fin.n, fin.n, lane);
  if (lane == 0) fin.ll[e] = v;
}

// pairs of the fused per-step scorer.  grid covers nchains * npairs waves
// (lo_blocks blocks of 4), then the appended finalize blocks of `fin`.
template <typename TT, int NPL, bool PROD>
__global__ __launch_bounds__(256, kLocalOptWavesPerSimd) void local_opt_pairs_kernel(
    int S, int E, int npairs, int nchains, const TT* __restrict__ eT,
    const int32_t* __restrict__ pairs, const int32_t* __restrict__ rows,
    const double* __restrict__ w01, const double* __restrict__ anc, const double* __restrict__ ow,
    double sig0, double sig1, double* __restrict__ wnew, double* __restrict__ wdag,
    int32_t* __restrict__ info, int lo_blocks, FinalizeArgs fin) {
  if ((int)blockIdx.x >= lo_blocks) {  // appended blocks: eval #1's partial sums, one wave per evaluation
    const int e = ((int)blockIdx.x - lo_blocks) * 4 + (int)(threadIdx.x / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    if (e < fin.batch) {
      const double v = sum_partials(fin.partial + (size_t)e * fin.n, fin.n, lane);
      if (lane == 0) fin.ll[e] = v;
    }
    return;
  }
  __shared__ double2 ltab[128];
  fill_log_table(ltab, threadIdx.x, blockDim.x);
  __syncthreads();
  const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (gw >= nchains * npairs) return;  // uniform per wave
  const int b = gw / npairs;
  const int n = gw - b * npairs;
  const int pk = pairs[(size_t)b * S * S + n];
  const int i = pk >> 16;
  const int k = pk & 0xffff;  // the parent node (prep_child_list)
  const size_t idx = ((size_t)b * S + i) * S + k;
  const double s = w01[idx];
  const TT* tv = eT + ((size_t)i * S + k) * E;
  const double* owk = ow + ((size_t)b * (S + 1) + k) * E;
  LocalObjective<NPL, PROD> obj;
  obj.ltab = ltab;
  // every lane loads (bounded rows: 0 past E) and divides, then padding is
  // selected away: no branch per element, so the 2 NPL loads and the NPL
  // divisions of the setup overlap instead of running one after another
  const RowRsrc rt(tv, E), ro(owk, E);
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const double v = local_c(rt.at<TT>(lane, q), ro.at<double>(lane, q), s);
    obj.c[q] = (lane < E - q * kWave) ? v : 0.0;  // padding: log(1) = 0
  }
  obj.anc = anc[idx];
#ifdef NEMO_LO_TRACE
  const long long ts = clock64();
#endif
  const LbfgsResult r = lbfgsb1_minimize(obj, s);
#ifdef NEMO_LO_TRACE
  const long long tend = clock64();
  if (lane == 0 && r.nfev >= NEMO_LO_TRACE)
    printf("lo_trace b %d i %d k %d nfev %d nit %d min %lld calls %lld exp %lld prod %lld tail %lld ls %lld\n", b, i,
           k, r.nfev, r.nit, tend - ts, obj.cy_calls, obj.cy_exp, obj.cy_prod, obj.cy_tail, obj.cy_ls);
#endif
  if (lane == 0) {
    const double wx = expit_d(r.x);
    wnew[idx] = wx;
    wdag[idx] = (wx > 0.5) ? sig1 : sig0;
    if (info) info[idx] = pack_info(r);
  }
}

// The same objective with one problem's effects split over the 4 waves of a
// block (wave w: the lane's elements 8w .. 8w + 7 of LocalObjective's NPL =
// 32, i.e. its chains 2w, 2w + 1; NPL = 16 / 64: one / four chains per
// wave).  Each wave multiplies its chains and the first tree levels, posts
// the product and exponent sum per lane to LDS, and after ONE barrier every
// wave finishes the tree over the four posts in LocalObjective's order
// ((w0 w1)(w2 w3)), then the log and the wave sum: every bit of f equals
// LocalObjective's, in all four waves, so the four run the same L-BFGS-B
// control flow.  For few problems (one chain's step) the serial line search
// of the slowest pair sets the kernel's time, and a wave issues the whole
// objective (~430 instructions per f-evaluation at NPL = 32) alone: split,
// each wave issues a quarter of the products.  Posts are double-buffered, so
// one barrier per f-evaluation suffices.
// NW = 2 (option local_split 3): two waves per problem, each multiplying half
// the chains, and the last tree level over the two posts -- the same tree, so
// the same bits -- at half the waves of the 4-wave form (4032 for one C3
// chain, which fit the chip at once; the 4-wave form's 8064 do not).
template <int NPL, int NW = 4>
struct SplitObjective {
  static constexpr int NC = NPL / 4;  // chains of LocalObjective
  static constexpr int L = NC / NW;   // chains per wave (a power of 2)
  static_assert((NW == 4 || NW == 2) && (L == 1 || L == 2 || L == 4 || L == 8),
                "split objective: NPL in {16, 32, 64}, 2 or 4 waves");
  double c[4 * L];                    // this lane's elements 4 L w .. 4 L w + 4 L - 1
  double anc;
  const double2* ltab;
  double2* post;                      // LDS [2 buffers][NW waves][64 lanes] (m(x0), m(x1))
  int2* kpost;                        // LDS [2][NW][64] (k(x0), k(x1))
  int w, lane;
  mutable int par = 0;
  __device__ __forceinline__ void operator()(double x0, double x1, double& f0, double& f1) const {
#pragma clang fp contract(off)
    constexpr double kLn2Hi = 0x1.62e42fefa3800p-1;
    constexpr double kLn2Lo = 5.4956039718945254e-14;
    const double e0 = expit_d(x0);
    const double e1 = expit_d(x1);
    double m0[L], m1[L];
    int k0 = 0, k1 = 0;
#pragma unroll
    for (int u = 0; u < L; ++u) {
      double a0 = fma(c[4 * u], e0, 1.0), a1 = fma(c[4 * u], e1, 1.0);
#pragma unroll
      for (int v = 1; v < 4; ++v) {
        a0 *= fma(c[4 * u + v], e0, 1.0);
        a1 *= fma(c[4 * u + v], e1, 1.0);
      }
      k0 += __builtin_amdgcn_frexp_exp(a0);
      m0[u] = __builtin_amdgcn_frexp_mant(a0);
      k1 += __builtin_amdgcn_frexp_exp(a1);
      m1[u] = __builtin_amdgcn_frexp_mant(a1);
    }
#pragma unroll
    for (int wd = 1; wd < L; wd *= 2)
#pragma unroll
      for (int u = 0; u + wd < L; u += 2 * wd) {
        m0[u] *= m0[u + wd];
        m1[u] *= m1[u + wd];
      }
    const int slot = (par * NW + w) * kWave + lane;
    post[slot] = double2{m0[0], m1[0]};
    kpost[slot] = int2{k0, k1};
    __syncthreads();
    const int base = par * NW * kWave + lane;
    double r0, r1;
    int kk0, kk1;
    if constexpr (NW == 4) {
      const double2 q0 = post[base], q1 = post[base + kWave], q2 = post[base + 2 * kWave],
                    q3 = post[base + 3 * kWave];
      const int2 j0 = kpost[base], j1 = kpost[base + kWave], j2 = kpost[base + 2 * kWave],
                 j3 = kpost[base + 3 * kWave];
      r0 = (q0.x * q1.x) * (q2.x * q3.x);
      r1 = (q0.y * q1.y) * (q2.y * q3.y);
      kk0 = j0.x + j1.x + j2.x + j3.x;
      kk1 = j0.y + j1.y + j2.y + j3.y;
    } else {
      const double2 q0 = post[base], q1 = post[base + kWave];
      const int2 j0 = kpost[base], j1 = kpost[base + kWave];
      r0 = q0.x * q1.x;
      r1 = q0.y * q1.y;
      kk0 = j0.x + j1.x;
      kk1 = j0.y + j1.y;
    }
    par ^= 1;
    kk0 += __builtin_amdgcn_frexp_exp(r0);
    kk1 += __builtin_amdgcn_frexp_exp(r1);
    r0 = __builtin_amdgcn_frexp_mant(r0);
    r1 = __builtin_amdgcn_frexp_mant(r1);
    double p0 = fma((double)kk0, kLn2Hi, log_fast(r0, ltab)) + (double)kk0 * kLn2Lo;
    double p1 = fma((double)kk1, kLn2Hi, log_fast(r1, ltab)) + (double)kk1 * kLn2Lo;
    p0 = wsum_dpp(p0);
    p1 = wsum_dpp(p1);
    f0 = (-p0 + fabs(e0 - anc)) + e0 * (1.0 - e0);
    f1 = (-p1 + fabs(e1 - anc)) + e1 * (1.0 - e1);
  }
};

// local_opt_pairs_kernel with one (chain, pair) per 4-wave block
// (SplitObjective): the same results bit for bit.  grid = nchains * npairs.
template <typename TT, int NPL, int NW = 4>
__global__ __launch_bounds__(NW * kWave) void local_opt_pairs_split_kernel(
    int S, int E, int npairs, int nchains, const TT* __restrict__ eT,
    const int32_t* __restrict__ pairs, const int32_t* __restrict__ rows,
    const double* __restrict__ w01, const double* __restrict__ anc, const double* __restrict__ ow,
    double sig0, double sig1, double* __restrict__ wnew, double* __restrict__ wdag,
    int32_t* __restrict__ info) {
  __shared__ double2 ltab[128];
  __shared__ double2 post[2 * NW * kWave];
  __shared__ int2 kpost[2 * NW * kWave];
  fill_log_table(ltab, threadIdx.x, blockDim.x);
  __syncthreads();
  const int gp = blockIdx.x;  // one problem per block
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  const int b = gp / npairs;
  const int n = gp - b * npairs;
  const int pk = pairs[(size_t)b * S * S + n];
  const int i = pk >> 16;
  const int k = pk & 0xffff;  // the parent node (prep_child_list)
  const size_t idx = ((size_t)b * S + i) * S + k;
  const double s = w01[idx];
  const TT* tv = eT + ((size_t)i * S + k) * E;
  const double* owk = ow + ((size_t)b * (S + 1) + k) * E;
  using Obj = SplitObjective<NPL, NW>;
  Obj obj;
  obj.ltab = ltab;
  obj.post = post;
  obj.kpost = kpost;
  obj.w = w;
  obj.lane = lane;
  const RowRsrc rt(tv, E), ro(owk, E);
#pragma unroll
  for (int q = 0; q < 4 * Obj::L; ++q) {  // (branch-free setup as in local_opt_pairs_kernel)
    const int qq = 4 * Obj::L * w + q;
    const double v = local_c(rt.at<TT>(lane, qq), ro.at<double>(lane, qq), s);
    obj.c[q] = (lane < E - qq * kWave) ? v : 0.0;  // padding: log(1) = 0
  }
  obj.anc = anc[idx];
  const LbfgsResult r = lbfgsb1_minimize(obj, s);
  if (w == 0 && lane == 0) {
    const double wx = expit_d(r.x);
    wnew[idx] = wx;
    wdag[idx] = (wx > 0.5) ? sig1 : sig0;
    if (info) info[idx] = pack_info(r);
  }
}

// generic batch of problems with caller-given c vectors
template <int NPL, bool PROD>
__global__ __launch_bounds__(256) void local_opt_generic_kernel(
    int n, int E, const double* __restrict__ cvec, const double* __restrict__ anc,
    const double* __restrict__ x0, double* __restrict__ out) {
  __shared__ double2 ltab[128];
  fill_log_table(ltab, threadIdx.x, blockDim.x);
  __syncthreads();
  const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (gw >= n) return;
  LocalObjective<NPL, PROD> obj;
  obj.ltab = ltab;
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    const int e = q * kWave + lane;
    const double v = cvec[(size_t)gw * E + (e < E ? e : E - 1)];  // branch-free: clamped, then selected
    obj.c[q] = (e < E) ? v : 0.0;
  }
  obj.anc = anc[gw];
  const LbfgsResult r = lbfgsb1_minimize(obj, x0[gw]);
  if (lane == 0) {
    out[(size_t)gw * 3 + 0] = r.x;
    out[(size_t)gw * 3 + 1] = r.f;
    out[(size_t)gw * 3 + 2] = (double)pack_info(r);
  }
}

int npl_for(int E) {
  const int need = (E + kWave - 1) / kWave;
  const int sizes[] = {4, 8, 16, 32, 48, 64, 80};
  for (int v : sizes)
    if (need <= v) return v;
  return -1;
}

}  // namespace

int pairs_per_chain(int S, int cap) {
  int p = 0;
  for (int q = 0; q < S; ++q) p += (cap > 0 && q > cap) ? cap : q;
  return p;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_exp_table(Ctx& c, const double* d_T64, hipStream_t st) {
  const size_t n = (size_t)c.S * c.S * c.E;
  const int blocks = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  if (c.dtype == 0)
    exp_table_kernel<double><<<blocks, 256, 0, st>>>(n, d_T64, (double*)c.d_eT);
  else
    exp_table_kernel<float><<<blocks, 256, 0, st>>>(n, d_T64, (float*)c.d_eT);
  return hipGetLastError();
}

hipError_t launch_prep(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                       int32_t* d_rows, double* d_sw, int32_t* d_cnt, int32_t* d_pairs,
                       hipStream_t st, int32_t* d_info) {
  prep_kernel<<<batch * ((c.S + 3) / 4), 256, 0, st>>>(c.S, cap, d_pos, d_w01, d_rows, d_sw, d_cnt, d_pairs,
                                                        d_info);
  return hipGetLastError();
}

static bool needs_renorm(const Ctx& c) {
  // products of up to S-1 factors in [min(1,e^T), max(1,e^T)]
  const double bound = c.table_absmax * (double)(c.S - 1);
  return c.dtype == 0 ? bound > 600.0 : bound > 80.0;
}

hipError_t launch_score(Ctx& c, int batch, const int32_t* d_rows, const double* d_sw,
                        const int32_t* d_cnt, double* d_ll, double* d_cs, double* d_cells,
                        double* d_ow, hipStream_t st) {
  const int nt = c.ntiles();
  dim3 grid(nt * batch);
  const bool rn = needs_renorm(c);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c.timing && c.timing_kernel == 0 && c.ev_used + 2 <= c.ev_pool.size()) {
    e0 = c.ev_pool[c.ev_used++];
    e1 = c.ev_pool[c.ev_used++];
    { hipError_t re = hipEventRecord(e0, st); if (re != hipSuccess) return re; }
  }
#define NEMO_SC(TT, RN)                                                                      \
  score_kernel<TT, RN><<<grid, kScoreWaves * kWave, 0, st>>>(                                \
      c.S, c.E, nt, (const TT*)c.d_eT, (const TT*)c.d_U, d_rows, d_sw, d_cnt, c.d_partial,   \
      d_cs, d_cells, d_ow, c.xcd_remap)
  if (c.dtype == 0) {
    if (rn) NEMO_SC(double, true); else NEMO_SC(double, false);
  } else {
    if (rn) NEMO_SC(float, true); else NEMO_SC(float, false);
  }
#undef NEMO_SC
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  if (e1) {
    { hipError_t re = hipEventRecord(e1, st); if (re != hipSuccess) return re; }
    c.launches++;
  }
  finalize_kernel<<<(batch + 3) / 4, 256, 0, st>>>(batch, nt, c.d_partial, d_ll);
  return hipGetLastError();
}

hipError_t launch_prep_group(Ctx& c, int batch, int group, int cap, const int32_t* d_pos,
                             const double* d_w01, hipStream_t st) {
  const int threads = ((c.S + kWave - 1) / kWave) * kWave;
  const int ng = (batch + group - 1) / group;
  switch (group) {
    case 4:
      prep_group_kernel<4><<<ng, threads, 0, st>>>(c.S, batch, cap, d_pos, d_w01, c.d_grows,
                                                    c.d_gsw, c.d_gcnt);
      break;
    case 8:
      prep_group_kernel<8><<<ng, threads, 0, st>>>(c.S, batch, cap, d_pos, d_w01, c.d_grows,
                                                    c.d_gsw, c.d_gcnt);
      break;
    case 16:
      prep_group_kernel<16><<<ng, threads, 0, st>>>(c.S, batch, cap, d_pos, d_w01, c.d_grows,
                                                     c.d_gsw, c.d_gcnt);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int CB, int GW>
static hipError_t launch_group_t(Ctx& c, int batch, hipStream_t st) {
  const int nt = c.ntiles();
  const int ng = (batch + CB - 1) / CB;
  const size_t wbytes = (size_t)GW * (c.S - 1) * CB * sizeof(double);
  const size_t mbytes = (size_t)2 * GW * CB * kWave * sizeof(double);
  const size_t lds = wbytes > mbytes ? wbytes : mbytes;
  dim3 grid(nt * ng);
  if (c.dtype == 0)
    score_group_kernel<double, CB, GW><<<grid, GW * kWave, lds, st>>>(
        c.S, c.E, nt, batch, (const double*)c.d_eT, (const double*)c.d_U, c.d_grows, c.d_gsw,
        c.d_gcnt, c.d_partial, c.xcd_remap);
  else
    score_group_kernel<float, CB, GW><<<grid, GW * kWave, lds, st>>>(
        c.S, c.E, nt, batch, (const float*)c.d_eT, (const float*)c.d_U, c.d_grows, c.d_gsw,
        c.d_gcnt, c.d_partial, c.xcd_remap);
  return hipGetLastError();
}

hipError_t launch_score_group(Ctx& c, int batch, int group, double* d_ll, hipStream_t st) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c.timing && c.timing_kernel == 0 && c.ev_used + 2 <= c.ev_pool.size()) {
    e0 = c.ev_pool[c.ev_used++];
    e1 = c.ev_pool[c.ev_used++];
    { hipError_t re = hipEventRecord(e0, st); if (re != hipSuccess) return re; }
  }
  hipError_t err;
  switch (group) {
    case 4: err = launch_group_t<4, 4>(c, batch, st); break;
    case 8: err = launch_group_t<8, 4>(c, batch, st); break;
    case 16: err = launch_group_t<16, 2>(c, batch, st); break;
    default: return hipErrorInvalidValue;
  }
  if (err != hipSuccess) return err;
  if (e1) {
    { hipError_t re = hipEventRecord(e1, st); if (re != hipSuccess) return re; }
    c.launches++;
  }
  finalize_kernel<<<(batch + 3) / 4, 256, 0, st>>>(batch, c.ntiles(), c.d_partial, d_ll);
  return hipGetLastError();
}

hipError_t launch_lse(Ctx& c, int rows, const double* d_cells, double* d_ll, double* d_cs,
                      double* d_ow, hipStream_t st) {
  const int nt = c.ntiles();
  lse_kernel<<<nt, kWave, 0, st>>>(rows, c.E, nt, d_cells, c.d_partial, d_cs, d_ow);
  finalize_kernel<<<1, 64, 0, st>>>(1, nt, c.d_partial, d_ll);
  return hipGetLastError();
}

template <typename TT>
static hipError_t local_pairs_t(Ctx& c, int nchains, int npairs, const int32_t* d_pairs,
                                const int32_t* d_rows, const double* d_w01, const double* d_anc,
                                const double* d_ow, double sig0, double sig1, double* d_wnew,
                                double* d_wdag, int32_t* d_info, hipStream_t st, FinalizeArgs fin) {
  const size_t waves = (size_t)nchains * npairs;
  const int lo_blocks = (int)((waves + 3) / 4);
  const int blocks = lo_blocks + (fin.ll ? (fin.batch + 3) / 4 : 0);
  const TT* eT = (const TT*)c.d_eT;
  // the product form needs every 4 factors in range (LocalObjective)
  const bool prod = c.local_prod && c.table_absmax <= 40.0;
  // few problems: one block of 4 waves per problem (SplitObjective, same
  // bits); option "local_split": 0 auto, 1 never, 2 always (where it applies)
  const int npl = npl_for(c.E);
  const bool splittable = prod && (npl == 16 || npl == 32 || npl == 64);
  const bool split = splittable && (c.local_split >= 2 || (c.local_split == 0 && waves <= (size_t)kLocalSplitMax));
  if (split) {
    if (fin.ll)
      finalize_factored_sums<<<(fin.batch + 3) / 4, 256, 0, st>>>(fin);
    const int nb = (int)waves;
    if (c.local_split == 3) {  // two waves per problem
      if (npl == 16)
        local_opt_pairs_split_kernel<TT, 16, 2><<<nb, 128, 0, st>>>(c.S, c.E, npairs, nchains, eT, d_pairs, d_rows,
                                                                   d_w01, d_anc, d_ow, sig0, sig1, d_wnew, d_wdag, d_info);
      else if (npl == 32)
        local_opt_pairs_split_kernel<TT, 32, 2><<<nb, 128, 0, st>>>(c.S, c.E, npairs, nchains, eT, d_pairs, d_rows,
                                                                   d_w01, d_anc, d_ow, sig0, sig1, d_wnew, d_wdag, d_info);
      else
        local_opt_pairs_split_kernel<TT, 64, 2><<<nb, 128, 0, st>>>(c.S, c.E, npairs, nchains, eT, d_pairs, d_rows,
                                                                   d_w01, d_anc, d_ow, sig0, sig1, d_wnew, d_wdag, d_info);
      return hipGetLastError();
    }
    if (npl == 16)
      local_opt_pairs_split_kernel<TT, 16><<<nb, 256, 0, st>>>(c.S, c.E, npairs, nchains, eT, d_pairs, d_rows,
                                                              d_w01, d_anc, d_ow, sig0, sig1, d_wnew, d_wdag, d_info);
    else if (npl == 32)
      local_opt_pairs_split_kernel<TT, 32><<<nb, 256, 0, st>>>(c.S, c.E, npairs, nchains, eT, d_pairs, d_rows,
                                                              d_w01, d_anc, d_ow, sig0, sig1, d_wnew, d_wdag, d_info);
    else
      local_opt_pairs_split_kernel<TT, 64><<<nb, 256, 0, st>>>(c.S, c.E, npairs, nchains, eT, d_pairs, d_rows,
                                                              d_w01, d_anc, d_ow, sig0, sig1, d_wnew, d_wdag, d_info);
    return hipGetLastError();
  }
#define NEMO_LP(NPL)                                                                            \
  if (prod)                                                                                     \
    local_opt_pairs_kernel<TT, NPL, true><<<blocks, 256, 0, st>>>(c.S, c.E, npairs, nchains, eT, \
        d_pairs, d_rows, d_w01, d_anc, d_ow, sig0, sig1, d_wnew, d_wdag, d_info, lo_blocks, fin); \
  else                                                                                          \
    local_opt_pairs_kernel<TT, NPL, false><<<blocks, 256, 0, st>>>(c.S, c.E, npairs, nchains, eT, \
        d_pairs, d_rows, d_w01, d_anc, d_ow, sig0, sig1, d_wnew, d_wdag, d_info, lo_blocks, fin)
  switch (npl_for(c.E)) {
    case 4: NEMO_LP(4); break;
    case 8: NEMO_LP(8); break;
    case 16: NEMO_LP(16); break;
    case 32: NEMO_LP(32); break;
    case 48: NEMO_LP(48); break;
    case 64: NEMO_LP(64); break;
    case 80: NEMO_LP(80); break;
    default: return hipErrorInvalidValue;
  }
#undef NEMO_LP
  return hipGetLastError();
}

hipError_t launch_local_opt_pairs(Ctx& c, int nchains, int npairs, const int32_t* d_pairs,
                                  const int32_t* d_rows, const double* d_w01, const double* d_anc,
                                  const double* d_ow, double sig0, double sig1, double* d_wnew,
                                  double* d_wdag, int32_t* d_info, hipStream_t st, FinalizeArgs fin) {
  if (nchains * npairs == 0) {
    if (fin.ll) finalize_factored_sums<<<(fin.batch + 3) / 4, 256, 0, st>>>(fin);
    return hipGetLastError();
  }
  if (c.dtype == 0)
    return local_pairs_t<double>(c, nchains, npairs, d_pairs, d_rows, d_w01, d_anc, d_ow, sig0,
                                 sig1, d_wnew, d_wdag, d_info, st, fin);
  return local_pairs_t<float>(c, nchains, npairs, d_pairs, d_rows, d_w01, d_anc, d_ow, sig0, sig1,
                              d_wnew, d_wdag, d_info, st, fin);
}

hipError_t launch_local_opt_generic(Ctx& c, int n, const double* d_c, const double* d_anc,
                                    const double* d_x0, double* d_out, bool prod, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const int blocks = (n + 3) / 4;
#define NEMO_LG(NPL)                                                                               \
  if (prod) local_opt_generic_kernel<NPL, true><<<blocks, 256, 0, st>>>(n, c.E, d_c, d_anc, d_x0, d_out); \
  else local_opt_generic_kernel<NPL, false><<<blocks, 256, 0, st>>>(n, c.E, d_c, d_anc, d_x0, d_out)
  switch (npl_for(c.E)) {
    case 4: NEMO_LG(4); break;
    case 8: NEMO_LG(8); break;
    case 16: NEMO_LG(16); break;
    case 32: NEMO_LG(32); break;
    case 48: NEMO_LG(48); break;
    case 64: NEMO_LG(64); break;
    case 80: NEMO_LG(80); break;
    default: return hipErrorInvalidValue;
  }
#undef NEMO_LG
  return hipGetLastError();
}

}  // namespace nemo
