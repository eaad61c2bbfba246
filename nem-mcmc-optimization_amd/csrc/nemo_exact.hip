// nemo_exact.hip -- the fused MCMC step in the reference's own arithmetic.
//
// The default kernels of the step (nemo_factored*.hip, local_opt_pairs_kernel)
// are fast restatements: order scores within ~1e-9 of numpy's and a local
// objective that agrees with numpy's to the last bits.  The forward-difference
// gradient of L-BFGS-B (h = 1e-8) amplifies those last bits, so a few of a C3
// step's 2016 optima follow another line search.  The kernels
// here compute what the reference computes, operation for operation:
//   * eval #1 / #2 (nem_order_mcmc.py:79-93, utils.py:84-94): cells U[i] +
//     log((1 - s) + s exp(T)) summed in the parent order of pi (numpy's SVML
//     log and exp, refmath.h), cs = logaddexp.reduce over the rows in order
//     (glibc exp / log1p), order weights exp(cell - cs), ll = Python's left
//     fold of cs;
//   * the local optimum (nem_order_mcmc.py:160-170): c = a / b as written,
//     the objective (:18-23) with numpy's pairwise sum of the SVML logs and
//     scipy's expit, and scipy's compact-form L-BFGS-B with OpenBLAS's small
//     kernels (lbfgsb_exact.h).
// Every kernel keeps the reference's order of operations, so the bits do not
// depend on the batch or the launch shape.  Host restatement and checks:
// tests/host/exact_spec.cpp, tests/test_exact_spec.py; GPU: test_gpu_exact.py.
#include "lbfgsb_exact.h"
#include "nemo_internal.h"
#include "refmath.h"

// no multiply-add is fused in this file but the explicit fma() calls (HIP's
// default contraction would fuse them; the functions repeat the pragma)
#pragma clang fp contract(off)

namespace nemo {
namespace {

using refmath::LdsTabs;

// the SVML / glibc tables in LDS (per-lane indices)
struct TabsLds {
  double log_hi[16], log_lo[16], exp_hi[16], exp_lo[16];
  uint64_t gexp[256];
  uint32_t rbase[64], rin[64];
  __device__ void fill(int t, int nt) {
    for (int q = t; q < 64; q += nt) {
      rbase[q] = refmath::kRcp14Base[q];
      rin[q] = refmath::kRcp14InBucket[q];
    }
    for (int q = t; q < 16; q += nt) {
      log_hi[q] = refmath::as_double(refmath::kSvmlLogHi[q]);
      log_lo[q] = refmath::as_double(refmath::kSvmlLogLo[q]);
      exp_hi[q] = refmath::as_double(refmath::kSvmlExpHi[q]);
      exp_lo[q] = refmath::as_double(refmath::kSvmlExpLo[q]);
    }
    for (int q = t; q < 256; q += nt) gexp[q] = refmath::kGlibcExpTab[q];
  }
  __device__ LdsTabs view() const { return LdsTabs{log_hi, log_lo, exp_hi, exp_lo, gexp, rbase, rin}; }
};

__device__ __forceinline__ int d1bit(const uint64_t* __restrict__ d1w, int nwords, int j, int e) {
  return (int)((d1w[(size_t)j * nwords + (e >> 6)] >> (e & 63)) & 1ull);
}

// ---------------------------------------------------------------------------
// cells: one block per (evaluation, child i, 256 effects).  The block first
// evaluates the child's two log factors per parent, log((1 - s) + s x) for x =
// exp(lo_j), exp(hi_j) (numpy: `1.0 - expit(w) + expit(w) * np.exp(T)`, then
// np.log), then each thread adds them to U[i][e] in pi's parent order.  Row S
// (attached to nothing) is U[S].  Cells go to `cells` [b][S+1][E].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void exact_cells_kernel(int S, int E, int etiles, const int32_t* __restrict__ pos,
                                                          const double* __restrict__ w01,
                                                          const double* __restrict__ xlo,
                                                          const double* __restrict__ xhi,
                                                          const uint64_t* __restrict__ d1w, int nwords,
                                                          const double* __restrict__ U, double* __restrict__ cells) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  __shared__ int perm[kMaxS];
  __shared__ double v[kMaxS][2];
  const int et = blockIdx.x % etiles;
  const int i = (blockIdx.x / etiles) % (S + 1);
  const int b = blockIdx.x / (etiles * (S + 1));
  const int t = threadIdx.x;
  const int e = et * 256 + t;
  tabs.fill(t, blockDim.x);
  const int32_t* pb = pos + (size_t)b * S;
  for (int q = t; q < S; q += blockDim.x) perm[pb[q]] = q;
  __syncthreads();
  const LdsTabs tb = tabs.view();
  const int pi = i < S ? pb[i] : 0;
  for (int q = t; q < pi; q += blockDim.x) {
    const int j = perm[q];
    const double s = w01[((size_t)b * S + i) * S + j];
    const double oms = 1.0 - s;
    v[q][0] = refmath::svml_log(oms + s * xlo[j], tb);
    v[q][1] = refmath::svml_log(oms + s * xhi[j], tb);
  }
  __syncthreads();
  if (e >= E) return;
  double cell = U[(size_t)i * E + e];
  for (int q = 0; q < pi; ++q) cell = cell + v[q][d1bit(d1w, nwords, perm[q], e)];
  cells[((size_t)b * (S + 1) + i) * E + e] = cell;
}

// ---------------------------------------------------------------------------
// fold: one thread per (evaluation, effect): cs = logaddexp.reduce over the
// S + 1 rows in order (numpy's reduction of axis 0), then, with OW, the order
// weights exp(cell - cs) in place of the cells.
// ---------------------------------------------------------------------------
template <bool OW>
__global__ __launch_bounds__(256) void exact_fold_kernel(int S, int E, int batch, double* __restrict__ cells,
                                                         double* __restrict__ cs) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  tabs.fill(threadIdx.x, blockDim.x);
  __syncthreads();
  const LdsTabs tb = tabs.view();
  const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (g >= (size_t)batch * E) return;
  const int b = (int)(g / E), e = (int)(g % E);
  double* col = cells + (size_t)b * (S + 1) * E + e;
  double acc = col[0];
  for (int r = 1; r <= S; ++r) acc = refmath::logaddexp(acc, col[(size_t)r * E], tb);
  cs[(size_t)b * E + e] = acc;
  if (OW)
    for (int r = 0; r <= S; ++r) col[(size_t)r * E] = refmath::svml_exp(col[(size_t)r * E] - acc, tb);
}

// ll = sum(cs): Python's built-in sum, a left fold over the effects (one lane
// per evaluation)
__device__ __forceinline__ void seq_sum(const double* __restrict__ cs, int E, double* __restrict__ ll) {
#pragma clang fp contract(off)
  double acc = 0.0;
  for (int e = 0; e < E; ++e) acc = acc + cs[e];
  *ll = acc;
}

__global__ void exact_seq_sum_kernel(int E, int batch, const double* __restrict__ cs, double* __restrict__ ll) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < batch) seq_sum(cs + (size_t)b * E, E, ll + b);
}

// ---------------------------------------------------------------------------
// the local objective, nem_order_mcmc.py:18-23 as numpy evaluates it:
//   -np.sum(np.log(c * ex + 1.0)) + |ex - anc| + ex (1 - ex)
// c * ex and + 1.0 rounded separately, SVML log, and numpy's pairwise sum
// over the wave as laid out by host::build_pairwise_plan.
// ---------------------------------------------------------------------------
template <int NS>
struct ExactObjective {
  static constexpr int kChain = 16;  // a leaf block of <= 128 elements: <= 16 per chain
  double c[NS][kChain];
  double crem[NS];
  int cnt[NS], nrem[NS];
  bool hasrem[NS];
  int partner[8];
  int nh, maxrem, lane;
  double anc;
  LdsTabs tb;

  __device__ __forceinline__ double sum_logs(double ex) const {
#pragma clang fp contract(off)
    double res[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      double acc = cnt[u] > 0 ? refmath::svml_log(c[u][0] * ex + 1.0, tb) : 0.0;
#pragma unroll
      for (int m = 1; m < kChain; ++m) {
        const double tm = refmath::svml_log(c[u][m] * ex + 1.0, tb);
        acc = m < cnt[u] ? acc + tm : acc;
      }
      // the block's 8 accumulators: ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))
      acc = acc + __shfl_xor(acc, 1);
      acc = acc + __shfl_xor(acc, 2);
      acc = acc + __shfl_xor(acc, 4);
      if (lb::uni(maxrem > 0)) {  // the block's n % 8 trailing elements, in order
        const double tr = hasrem[u] ? refmath::svml_log(crem[u] * ex + 1.0, tb) : 0.0;
        for (int r = 0; r < 7; ++r) {
          const double y = __shfl(tr, (lane & ~7) + r);
          acc = r < nrem[u] ? acc + y : acc;
        }
      }
      res[u] = acc;
    }
    // leaf L (slot L / 8, lanes 8 (L % 8) ..) to lane L
    double v = 0.0;
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const double x = __shfl(res[u], 8 * (lane & 7));
      v = (lane >> 3) == u ? x : v;
    }
    // the recursion's additions, one height at a time
    for (int h = 0; h < nh; ++h) {
      const int p = partner[h];
      const double y = __shfl(v, p < 0 ? lane : p);
      v = p >= 0 ? v + y : v;
    }
    return __shfl(v, 0);  // the root: its first leaf is leaf 0
  }

  __device__ __forceinline__ void operator()(double x0, double x1, double& f0, double& f1) const {
#pragma clang fp contract(off)
    const double e0 = refmath::expit(x0, tb);
    const double e1 = refmath::expit(x1, tb);
    const double p0 = sum_logs(e0);
    const double p1 = sum_logs(e1);
    f0 = (-p0 + fabs(e0 - anc)) + e0 * (1.0 - e0);
    f1 = (-p1 + fabs(e1 - anc)) + e1 * (1.0 - e1);
  }
};

struct SeqSumArgs {
  const double* cs = nullptr;
  int E = 0, batch = 0;
  double* ll = nullptr;
};

constexpr int kExactWaves = 4;

// one wave per (chain, permissible pair), kExactWaves per block; then the
// appended blocks of `fin` (eval #1's ll, one lane per chain)
template <int NS>
__global__ __launch_bounds__(kExactWaves * kWave) void local_opt_exact_kernel(
    int S, int E, int npairs, int nchains, const int32_t* __restrict__ pairs, const double* __restrict__ w01,
    const double* __restrict__ anc, const double* __restrict__ ow, const double* __restrict__ xlo,
    const double* __restrict__ xhi, const uint64_t* __restrict__ d1w, int nwords, const int32_t* __restrict__ plan,
    int nh, int maxrem, double sig0, double sig1, double* __restrict__ wnew, double* __restrict__ wdag,
    int32_t* __restrict__ info, int lo_blocks, SeqSumArgs fin) {
#pragma clang fp contract(off)
  if ((int)blockIdx.x >= lo_blocks) {
    const int bb = ((int)blockIdx.x - lo_blocks) * (int)blockDim.x + (int)threadIdx.x;
    if (bb < fin.batch) seq_sum(fin.cs + (size_t)bb * fin.E, fin.E, fin.ll + bb);
    return;
  }
  __shared__ TabsLds tabs;
  __shared__ double mem[kExactWaves][lbx::kMemDoubles];
  tabs.fill(threadIdx.x, blockDim.x);
  __syncthreads();
  const int wv = threadIdx.x / kWave;
  const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (gw >= nchains * npairs) return;  // uniform per wave
  const int b = gw / npairs;
  const int n = gw - b * npairs;
  const int pk = pairs[(size_t)b * S * S + n];
  const int i = pk >> 16;
  const int k = pk & 0xffff;
  const size_t idx = ((size_t)b * S + i) * S + k;
  const double s = w01[idx];
  const double lvlo = xlo[k], lvhi = xhi[k];
  const double* owk = ow + ((size_t)b * (S + 1) + k) * E;
  ExactObjective<NS> obj;
  obj.tb = tabs.view();
  obj.lane = lane;
  obj.nh = nh;
  obj.maxrem = maxrem;
  obj.anc = anc[idx];
  // c = a / b, nem_order_mcmc.py:161-164 (local_vec = np.exp(T[i][k]))
  auto cval = [&](int e) {
#pragma clang fp contract(off)
    const double lv = d1bit(d1w, nwords, k, e) ? lvhi : lvlo;
    const double a = (lv - 1.0) * owk[e];
    const double bd = (1.0 - s * a) + s * (lv - 1.0);
    return a / bd;
  };
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int q = u * kWave + lane;
    const int st = plan[q], ct = plan[NS * kWave + q], re = plan[2 * NS * kWave + q];
    obj.cnt[u] = ct;
    obj.nrem[u] = plan[3 * NS * kWave + q];
#pragma unroll
    for (int m = 0; m < ExactObjective<NS>::kChain; ++m) obj.c[u][m] = m < ct ? cval(st + 8 * m) : 0.0;
    obj.hasrem[u] = re >= 0;
    obj.crem[u] = re >= 0 ? cval(re) : 0.0;
  }
#pragma unroll
  for (int h = 0; h < 8; ++h) obj.partner[h] = h < nh ? plan[4 * NS * kWave + h * kWave + lane] : -1;
  const LbfgsResult r = lbfgsb1_minimize_exact(obj, s, lbx::Mem{mem[wv]});
  if (lane == 0) {
    const double wx = refmath::expit(r.x, obj.tb);
    wnew[idx] = wx;
    wdag[idx] = (wx > 0.5) ? sig1 : sig0;
    if (info) {
      const int nit = r.nit < 4095 ? r.nit : 4095;
      const int nfev = r.nfev < 32767 ? r.nfev : 32767;
      info[idx] = (int32_t)(r.status | (nit << 4) | (nfev << 16));
    }
  }
}

// the same optimiser on caller-supplied c vectors [n][E] (nemo_local_opt:
// calculate_local_optimum of one pair, and the scipy records of the tests);
// out [n][3] = x*, f*, packed info
template <int NS>
__global__ __launch_bounds__(kExactWaves * kWave) void local_opt_exact_generic_kernel(
    int E, int n, const double* __restrict__ cvec, const double* __restrict__ anc, const double* __restrict__ x0,
    const int32_t* __restrict__ plan, int nh, int maxrem, double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  __shared__ double mem[kExactWaves][lbx::kMemDoubles];
  tabs.fill(threadIdx.x, blockDim.x);
  __syncthreads();
  const int wv = threadIdx.x / kWave;
  const int p = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (p >= n) return;
  const double* cp = cvec + (size_t)p * E;
  ExactObjective<NS> obj;
  obj.tb = tabs.view();
  obj.lane = lane;
  obj.nh = nh;
  obj.maxrem = maxrem;
  obj.anc = anc[p];
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const int q = u * kWave + lane;
    const int st = plan[q], ct = plan[NS * kWave + q], re = plan[2 * NS * kWave + q];
    obj.cnt[u] = ct;
    obj.nrem[u] = plan[3 * NS * kWave + q];
#pragma unroll
    for (int m = 0; m < ExactObjective<NS>::kChain; ++m) obj.c[u][m] = m < ct ? cp[st + 8 * m] : 0.0;
    obj.hasrem[u] = re >= 0;
    obj.crem[u] = re >= 0 ? cp[re] : 0.0;
  }
#pragma unroll
  for (int h = 0; h < 8; ++h) obj.partner[h] = h < nh ? plan[4 * NS * kWave + h * kWave + lane] : -1;
  const LbfgsResult r = lbfgsb1_minimize_exact(obj, x0[p], lbx::Mem{mem[wv]});
  if (lane == 0) {
    const int nit = r.nit < 4095 ? r.nit : 4095;
    const int nfev = r.nfev < 32767 ? r.nfev : 32767;
    out[(size_t)p * 3] = r.x;
    out[(size_t)p * 3 + 1] = r.f;
    out[(size_t)p * 3 + 2] = (double)(r.status | (nit << 4) | (nfev << 16));
  }
}

// device evaluations of refmath.h for the tests (fn: 0 svml_log, 1 svml_exp,
// 2 expit, 3 logaddexp(x, y), 4 glibc_exp, 5 glibc_log1p, 6 sqrt, 7 x / y)
__global__ void refmath_probe_kernel(int fn, int n, const double* __restrict__ x, const double* __restrict__ y,
                                     double* __restrict__ out) {
  __shared__ TabsLds tabs;
  tabs.fill(threadIdx.x, blockDim.x);
  __syncthreads();
  const LdsTabs tb = tabs.view();
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const double v = x[g];
  double r = 0.0;
  switch (fn) {
    case 0: r = refmath::svml_log(v, tb); break;
    case 1: r = refmath::svml_exp(v, tb); break;
    case 2: r = refmath::expit(v, tb); break;
    case 3: r = refmath::logaddexp(v, y[g], tb); break;
    case 4: r = refmath::glibc_exp(v, tb); break;
    case 5: r = refmath::glibc_log1p(v); break;
    case 6: r = __builtin_sqrt(v); break;  // the optimiser's square roots and divisions
    default: r = v / y[g]; break;
  }
  out[g] = r;
}

}  // namespace

hipError_t launch_local_opt_exact_generic(Ctx& c, int n, const double* d_c, const double* d_anc, const double* d_x0,
                                          double* d_out, hipStream_t st) {
  const dim3 grid((n + kExactWaves - 1) / kExactWaves);
  switch (c.pw_ns) {
#define NEMO_EXACT_NS(NSV)                                                                                   \
  case NSV:                                                                                                  \
    local_opt_exact_generic_kernel<NSV><<<grid, kExactWaves * kWave, 0, st>>>(c.E, n, d_c, d_anc, d_x0,       \
                                                                              c.d_pwplan, c.pw_nh,            \
                                                                              c.pw_maxrem, d_out);            \
    break;
    NEMO_EXACT_NS(1)
    NEMO_EXACT_NS(2)
    NEMO_EXACT_NS(3)
    NEMO_EXACT_NS(4)
#undef NEMO_EXACT_NS
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_refmath_probe(int fn, int n, const double* d_x, const double* d_y, double* d_out, hipStream_t st) {
  refmath_probe_kernel<<<(n + 255) / 256, 256, 0, st>>>(fn, n, d_x, d_y, d_out);
  return hipGetLastError();
}

bool exact_supported(const Ctx& c) { return c.factored && c.exact_ok && c.d_xlo && c.d_pwplan; }

hipError_t launch_exact_eval(Ctx& c, int batch, const int32_t* d_pos, const double* d_w01, double* d_cells,
                             double* d_cs, double* d_ll, bool want_ow, hipStream_t st) {
  const int S = c.S, E = c.E;
  const int etiles = (E + 255) / 256;
  exact_cells_kernel<<<dim3(batch * (S + 1) * etiles), 256, 0, st>>>(S, E, etiles, d_pos, d_w01, c.d_xlo, c.d_xhi,
                                                                     c.d_D1w, c.nwords, c.d_U64, d_cells);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  const size_t nthr = (size_t)batch * E;
  const int fb = (int)((nthr + 255) / 256);
  if (want_ow) exact_fold_kernel<true><<<fb, 256, 0, st>>>(S, E, batch, d_cells, d_cs);
  else exact_fold_kernel<false><<<fb, 256, 0, st>>>(S, E, batch, d_cells, d_cs);
  err = hipGetLastError();
  if (err != hipSuccess || !d_ll) return err;
  exact_seq_sum_kernel<<<(batch + 63) / 64, 64, 0, st>>>(E, batch, d_cs, d_ll);
  return hipGetLastError();
}

hipError_t launch_local_opt_exact(Ctx& c, int nchains, int npairs, const int32_t* d_pairs, const double* d_w01,
                                  const double* d_anc, const double* d_ow, double sig0, double sig1, double* d_wnew,
                                  double* d_wdag, int32_t* d_info, const double* d_cs1, double* d_ll1,
                                  hipStream_t st) {
  const int nw = nchains * npairs;
  const int lo_blocks = (nw + kExactWaves - 1) / kExactWaves;
  SeqSumArgs fin{d_cs1, c.E, nchains, d_ll1};
  const int fin_blocks = d_ll1 ? (nchains + kExactWaves * kWave - 1) / (kExactWaves * kWave) : 0;
  const dim3 grid(lo_blocks + fin_blocks);
  switch (c.pw_ns) {
#define NEMO_EXACT_NS(NSV)                                                                                         \
  case NSV:                                                                                                        \
    local_opt_exact_kernel<NSV><<<grid, kExactWaves * kWave, 0, st>>>(                                            \
        c.S, c.E, npairs, nchains, d_pairs, d_w01, d_anc, d_ow, c.d_xlo, c.d_xhi, c.d_D1w, c.nwords, c.d_pwplan, \
        c.pw_nh, c.pw_maxrem, sig0, sig1, d_wnew, d_wdag, d_info, lo_blocks, fin);                                 \
    break;
    NEMO_EXACT_NS(1)
    NEMO_EXACT_NS(2)
    NEMO_EXACT_NS(3)
    NEMO_EXACT_NS(4)
#undef NEMO_EXACT_NS
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace nemo
