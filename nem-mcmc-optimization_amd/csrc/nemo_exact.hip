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

#include <type_traits>

// no multiply-add is fused in this file but the explicit fma() calls (HIP's
// default contraction would fuse them; the functions repeat the pragma)
#pragma clang fp contract(off)

#ifndef NEMO_EXACT_LOGPAIR
// ExactObjective::log_pair shares the two points' log row when set; off: the
// extra registers cost more than the lookups they save (C3, 16 chains: 1.75 vs
// 1.50 ms per fused step; 1 chain 0.50 vs 0.46 ms; profiles/r5/r5h_logpair_ab.txt)
#define NEMO_EXACT_LOGPAIR 0
#endif
#ifndef NEMO_EXACT_TPUT_WAVES
#define NEMO_EXACT_TPUT_WAVES 4   // the throughput form's waves per SIMD (its register budget)
#endif
#ifndef NEMO_EXACT_TPUT_UNROLL
#define NEMO_EXACT_TPUT_UNROLL 4   // the throughput forms' chain loop unroll
#endif
#ifndef NEMO_EXACT_SLOT_PAIRS
#define NEMO_EXACT_SLOT_PAIRS 1   // the slot form's row set in element pairs (ExactObjective::kPairs)
#endif
#ifndef NEMO_EXACT_SLOT_GROUP
#define NEMO_EXACT_SLOT_GROUP 4   // the slot form's pair loads in flight together (2, 4 or 8)
#endif
#ifndef NEMO_EXACT_SLOT_WAVES
#define NEMO_EXACT_SLOT_WAVES 4   // the slot form's waves per SIMD (3 measured slower, profiles/r6/r6j_forms_ab.txt)
#endif
#ifndef NEMO_EXACT_CT_WAVES
#define NEMO_EXACT_CT_WAVES 3   // the cached throughput form's waves per SIMD (form 4)
#endif
#ifndef NEMO_EXACT_CCACHE
#define NEMO_EXACT_CCACHE 1   // the latency form holds its c values in registers (ExactObjective::kCache)
#endif

namespace nemo {
namespace {

using refmath::LdsTabs;

// the SVML / glibc tables in LDS (per-lane indices)
struct TabsLds {
  alignas(16) double lrow[128][4];
  alignas(16) double erow[16][2];
  uint64_t gexp[256];
  uint32_t rthr[64];
  __device__ void fill(int t, int nt) {
    for (int q = t; q < 128; q += nt) refmath::svml_log_row((int)refmath::kRcp14Base[q >> 1] + (q & 1), lrow[q]);
    for (int q = t; q < 64; q += nt) rthr[q] = refmath::kRcp14InBucket[q];
    for (int q = t; q < 16; q += nt) {
      erow[q][0] = refmath::as_double(refmath::kSvmlExpHi[q]);
      erow[q][1] = refmath::as_double(refmath::kSvmlExpLo[q]);
    }
    for (int q = t; q < 256; q += nt) gexp[q] = refmath::kGlibcExpTab[q];
  }
  // only what svml_log reads
  __device__ void fill_log(int t, int nt) {
    for (int q = t; q < 128; q += nt) refmath::svml_log_row((int)refmath::kRcp14Base[q >> 1] + (q & 1), lrow[q]);
    for (int q = t; q < 64; q += nt) rthr[q] = refmath::kRcp14InBucket[q];
  }
  // only what glibc_exp reads (logaddexp)
  __device__ void fill_gexp(int t, int nt) {
    for (int q = t; q < 256; q += nt) gexp[q] = refmath::kGlibcExpTab[q];
  }
  // only what svml_exp reads
  __device__ void fill_exp(int t, int nt) {
    for (int q = t; q < 16; q += nt) {
      erow[q][0] = refmath::as_double(refmath::kSvmlExpHi[q]);
      erow[q][1] = refmath::as_double(refmath::kSvmlExpLo[q]);
    }
  }
  __device__ LdsTabs view() const { return LdsTabs{rthr, &lrow[0][0], &erow[0][0], gexp}; }
};

__device__ __forceinline__ int d1bit(const uint64_t* __restrict__ d1w, int nwords, int j, int e) {
  return (int)((d1w[(size_t)j * nwords + (e >> 6)] >> (e & 63)) & 1ull);
}

// XCD-contiguous block order (blocks are dealt round-robin to the 8 XCDs, so
// physical block P runs on XCD P % 8): XCD x takes the x-th contiguous range of
// the n logical blocks, so the optima in flight on one XCD share few chains
// and their parents' a rows stay in that XCD's L2.  Bijective on [0, n);
// blocks >= n (appended work) keep their index.
__device__ __forceinline__ int xcd_block(int on, int P, int n) {
  if (!on || P >= n) return P;
  const int x = P & 7, k = P >> 3, q = n >> 3, r = n & 7;
  return x * q + (x < r ? x : r) + k;
}

// ---------------------------------------------------------------------------
// cells: one block per (evaluation, `rows` consecutive children i).  The block
// first evaluates each child's two log factors per parent, log((1 - s) + s x)
// for x = exp(lo_j), exp(hi_j) (numpy: `1.0 - expit(w) + expit(w) *
// np.exp(T)`, then np.log), then each thread adds them to U[i][e] in pi's
// parent order.  Row S (attached to nothing) is U[S].  Cells go to `cells`
// [b][S+1][E].  A wave takes kGW consecutive D1 words at a time: per parent
// one scalar load of the words (their bits are the wave's lane masks, inverse
// ballot) and one broadcast read of the factor pair serve kGW cells per lane.
// Several children per block share the block's table fill and permutation
// (large batches); one child per block keeps small batches wide.
// ---------------------------------------------------------------------------
constexpr int kCellsThreads = 512, kCellsRows = 8, kCellsSlots = 512;

__global__ __launch_bounds__(kCellsThreads) void exact_cells_kernel(int S, int E, int rows, int cap,
                                                                    const int32_t* __restrict__ pos,
                                                                    const double* __restrict__ w01,
                                                                    const double* __restrict__ xlo,
                                                                    const double* __restrict__ xhi,
                                                                    const uint64_t* __restrict__ d1w, int nwords,
                                                                    const double* __restrict__ U,
                                                                    double* __restrict__ cells) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  __shared__ int perm[kMaxS];
  __shared__ double v[kCellsSlots][2];   // [rows][S] factor pairs, rows * S <= kCellsSlots
  const int nchunk = (S + rows) / rows;   // ceil((S + 1) / rows)
  const int i0 = (blockIdx.x % nchunk) * rows;
  const int b = blockIdx.x / nchunk;
  const int nr = min(rows, S + 1 - i0);
  const int t = threadIdx.x;
  const int32_t* pb = pos + (size_t)b * S;
  if (i0 < S) tabs.fill_log(t, blockDim.x);
  for (int q = t; q < S; q += blockDim.x) perm[pb[q]] = q;
  __syncthreads();
  const LdsTabs tb = tabs.view();
  for (int r = 0; r < nr; ++r) {
    const int i = i0 + r;
    const int pi = i < S ? pb[i] : 0;
    const int lo = (cap > 0 && pi > cap) ? pi - cap : 0;   // with a cap: the last `cap` parents
    for (int q = t; q < 2 * (pi - lo); q += blockDim.x) {   // lo and hi factors on separate lanes
      const int j = perm[lo + (q >> 1)];
      const double s = w01[((size_t)b * S + i) * S + j];
      v[r * S + (q >> 1)][q & 1] = refmath::svml_log((1.0 - s) + s * ((q & 1) ? xhi[j] : xlo[j]), tb);
    }
  }
  __syncthreads();
  const int lane = t & (kWave - 1);
  const int nwaves = __builtin_amdgcn_readfirstlane(blockDim.x / kWave);
  const int w0 = __builtin_amdgcn_readfirstlane(t / kWave);
  constexpr int kGW = 4, kU = 4;
  const int ngroups = nwords / kGW;
  for (int r = 0; r < nr; ++r) {
    const int i = i0 + r;
    const int p0 = i < S ? pb[i] : 0;
    const int lo = (cap > 0 && p0 > cap) ? p0 - cap : 0;
    const int pi = p0 - lo;       // the parents perm[lo ..], in pi's order
    const int* pp = perm + lo;
    const double* urow = U + (size_t)i * E;
    double* crow = cells + ((size_t)b * (S + 1) + i) * E;
    const double2* v2 = reinterpret_cast<const double2*>(&v[r * S][0]);
    int g = w0;
    for (; g < ngroups; g += nwaves) {
      double cell[kGW];
#pragma unroll
      for (int w = 0; w < kGW; ++w) {
        const int e = (g * kGW + w) * kWave + lane;
        cell[w] = e < E ? urow[e] : 0.0;
      }
      const uint64_t* dw = d1w + g * kGW;
      int q = 0;
      for (; q + kU <= pi; q += kU) {
        uint64_t wd[kU][kGW];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const uint64_t* p = dw + (size_t)__builtin_amdgcn_readfirstlane(pp[q + u]) * nwords;
#pragma unroll
          for (int w = 0; w < kGW; ++w) wd[u][w] = p[w];
        }
        double2 f[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) f[u] = v2[q + u];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
#pragma unroll
          for (int w = 0; w < kGW; ++w)
            cell[w] = cell[w] + (__builtin_amdgcn_inverse_ballot_w64(wd[u][w]) ? f[u].y : f[u].x);
        }
      }
      for (; q < pi; ++q) {
        const uint64_t* p = dw + (size_t)__builtin_amdgcn_readfirstlane(pp[q]) * nwords;
        const double2 f = v2[q];
#pragma unroll
        for (int w = 0; w < kGW; ++w) cell[w] = cell[w] + (__builtin_amdgcn_inverse_ballot_w64(p[w]) ? f.y : f.x);
      }
#pragma unroll
      for (int w = 0; w < kGW; ++w) {
        const int e = (g * kGW + w) * kWave + lane;
        if (e < E) crow[e] = cell[w];
      }
    }
    // the words past the last whole group, one at a time
    for (int word = ngroups * kGW + (g - ngroups); word < nwords; word += nwaves) {
      const int e = word * kWave + lane;
      double cell = e < E ? urow[e] : 0.0;
      const uint64_t* dw = d1w + word;
      for (int q = 0; q < pi; ++q) {
        const uint64_t wd = dw[(size_t)__builtin_amdgcn_readfirstlane(pp[q]) * nwords];
        const double2 f = v2[q];
        cell = cell + (__builtin_amdgcn_inverse_ballot_w64(wd) ? f.y : f.x);
      }
      if (e < E) crow[e] = cell;
    }
  }
}

// ---------------------------------------------------------------------------
// fold: one thread per (evaluation, effect): cs = logaddexp.reduce over the
// S + 1 rows in order (numpy's reduction of axis 0).  The chain of S
// logaddexps is the step's serial latency at one chain, so the rows come in
// register blocks of 16, the next block's loads in flight during the fold of
// the current one.  The order weights exp(cell - cs) follow in a separate,
// fully parallel launch.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void exact_fold_kernel(int S, int E, int batch, const double* __restrict__ cells,
                                                         double* __restrict__ cs) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  tabs.fill_gexp(threadIdx.x, blockDim.x);
  __syncthreads();
  const LdsTabs tb = tabs.view();
  const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (g >= (size_t)batch * E) return;
  const int b = (int)(g / E), e = (int)(g % E);
  const double* col = cells + (size_t)b * (S + 1) * E + e;
  const int R = S + 1;
  constexpr int kC = 16;
  double nxt[kC];
#pragma unroll
  for (int q = 0; q < kC; ++q) nxt[q] = q < R ? col[(size_t)q * E] : 0.0;
  double acc = 0.0;
  for (int r0 = 0; r0 < R; r0 += kC) {
    double cur[kC];
#pragma unroll
    for (int q = 0; q < kC; ++q) cur[q] = nxt[q];
    if (r0 + kC < R) {
#pragma unroll
      for (int q = 0; q < kC; ++q) nxt[q] = r0 + kC + q < R ? col[(size_t)(r0 + kC + q) * E] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kC; ++q) {
      const int r = r0 + q;
      if (r < R) acc = r == 0 ? cur[q] : refmath::logaddexp(acc, cur[q], tb);
    }
  }
  cs[(size_t)b * E + e] = acc;
}

// order weights in place: cell = exp(cell - cs) (nem_order_mcmc.py:92), one
// thread per cell.  With xa (the fused step's recompute form): also the local
// optima's a = (lv - 1) * ow (nem_order_mcmc.py:161-162, lv = np.exp(T[i][k])
// of parent row k) at the element's plan position, [batch][S][plan]
__global__ __launch_bounds__(256) void exact_ow_kernel(int S, int E, int batch, double* __restrict__ cells,
                                                       const double* __restrict__ cs, double* __restrict__ xa,
                                                       const int32_t* __restrict__ pwpos, int plan_doubles,
                                                       const double* __restrict__ xlo, const double* __restrict__ xhi,
                                                       const uint64_t* __restrict__ d1w, int nwords) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  tabs.fill_exp(threadIdx.x, blockDim.x);
  __syncthreads();
  const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t n = (size_t)batch * (S + 1) * E;
  if (g >= n) return;
  const int e = (int)(g % E);
  const size_t rb = g / E;   // b * (S + 1) + row
  const size_t b = rb / (S + 1);
  const int row = (int)(rb - b * (S + 1));
  const double ow = refmath::svml_exp(cells[g] - cs[b * E + e], tabs.view());
  cells[g] = ow;
  if (xa && row < S) {
    const double lv = d1bit(d1w, nwords, row, e) ? xhi[row] : xlo[row];
    xa[(b * S + row) * (size_t)plan_doubles + pwpos[e]] = (lv - 1.0) * ow;
  }
}

// ll = sum(cs): Python's built-in sum, a left fold over the effects, by one
// wave: 64 values per coalesced load (the next one in flight), staged in the
// wave's LDS row and added in order from broadcast reads, which issue ahead
// of the chain of additions; every lane holds the sum
__device__ __forceinline__ double wave_seq_sum(const double* __restrict__ cs, int E, int lane, double* row) {
#pragma clang fp contract(off)
  double acc = 0.0;
  double nxt = lane < E ? cs[lane] : 0.0;
  for (int base = 0; base < E; base += kWave) {
    const double v = nxt;
    if (base + kWave < E) nxt = base + kWave + lane < E ? cs[base + kWave + lane] : 0.0;
    row[lane] = v;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int n = E - base < kWave ? E - base : kWave;
    if (n == kWave) {
      // 32 values read before their 32 adds: the chain waits on one read latency
      // per half row, not on one per pair of adds
#pragma unroll
      for (int h = 0; h < kWave; h += 32) {
        double vals[32];
#pragma unroll
        for (int l = 0; l < 32; ++l) vals[l] = row[h + l];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int l = 0; l < 32; ++l) acc = acc + vals[l];
      }
    } else {
      for (int l = 0; l < n; ++l) acc = acc + row[l];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  return acc;
}

// one wave per evaluation
__global__ __launch_bounds__(256) void exact_seq_sum_kernel(int E, int batch, const double* __restrict__ cs,
                                                            double* __restrict__ ll) {
  __shared__ double rows[4][kWave];
  const int b = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (b >= batch) return;
  const double v = wave_seq_sum(cs + (size_t)b * E, E, lane, rows[threadIdx.x / kWave]);
  if (lane == 0) ll[b] = v;
}

// ---------------------------------------------------------------------------
// the local objective, nem_order_mcmc.py:18-23 as numpy evaluates it:
//   -np.sum(np.log(c * ex + 1.0)) + |ex - anc| + ex (1 - ex)
// c * ex and + 1.0 rounded separately, SVML log, and numpy's pairwise sum
// over the wave as laid out by host::build_pairwise_plan.
// ---------------------------------------------------------------------------
// c is read from memory at every evaluation, so no register holds it while
// the optimiser runs: kPlan, the plan-ordered copy the fused kernel writes
// ([NS][17][64]: chain element m of slot u at row u * 17 + m, the remainder
// at row 16, one coalesced row per element); else the caller's [E] vector at
// the plan's indices.  kRc (with kPlan): c recomputed at every evaluation from
// the parent's plan-ordered a = (lv - 1) ow (the order weights' launch writes
// them, one row set per (chain, parent k), shared by the S - 1 children of k)
// and lv's bit -- c = a / ((1 - s a) + s (lv - 1)), nem_order_mcmc.py:161-164,
// the same rounded operations -- so the objective reads 1.1 MB per chain
// instead of one 17 KB row set per optimum.  The plan itself (per lane: chain
// starts, counts, remainders, tree partners) is the block's LDS copy.
// kPairs (the slot form): the row set's 16 chain rows stored as 8 rows of
// element pairs (lane l's elements 2p and 2p + 1 side by side), so one 16-byte
// load brings two c values; the remainder row as before
template <int NS, bool kPlan, bool kLat, bool kPair = false, bool kRc = false, bool kCache = false, bool kMP = false,
          bool kPairs = false>
struct ExactObjective {
  static constexpr int kChain = 16;  // a leaf block of <= 128 elements: <= 16 per chain
  static constexpr int kRows = kChain + 1;
  static constexpr bool kPairsLayout = kPairs;
  const double* cp;
  // kCache (the latency form's recompute rows, 2 waves per SIMD): the lane's
  // c values made once per optimum (fill_cache) and held in registers through
  // the optimiser, instead of recomputed from the a rows every evaluation --
  // the same rc_c values, so the same bits
  double cc[kCache ? NS : 1][kCache ? kRows : 1];
  // kRc: this lane's lv bits per slot (bit m: chain element m, bit 16: the
  // remainder), s and s (lv - 1) of both values; pad_guard: a padding
  // element's 1 + s (lo - 1) is 0 (s = 1, exp(lo) = 0), so its 0 / 0 is
  // replaced by the 0 a stored row holds there
  uint32_t rbits[kRc ? NS : 1];
  double rs = 0.0, rslo = 0.0, rshi = 0.0;
  bool pad_guard = false;
  const int32_t* pl;   // host::PairwisePlan rows in LDS: start, cnt, rem, nrem [NS][64], partner [8][64]
  int nh, maxrem, lane;
  // numpy's pairwise sum in two wave plans (E > 8192, CArgs::nparts): each
  // part's rows in global memory (plg), its height and trailing count (pmeta),
  // kRc: the parent's lv bits of all parts' slots (xbk)
  int nparts = 1;
  const int32_t* plg = nullptr;
  const int32_t* pmeta = nullptr;
  const uint32_t* xbk = nullptr;
  double anc;
  LdsTabs tb;

  // kLat: the plan's per-lane values also in registers (load_plan), off the
  // evaluation's critical path; else read from LDS where used
  static constexpr bool kRegs = kLat || kPair;
  int r_cnt[kRegs ? NS : 1], r_rem[kRegs ? NS : 1], r_nrem[kRegs ? NS : 1], r_partner[kRegs ? 8 : 1];

  __device__ __forceinline__ void load_plan() {
    if (kRegs) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        r_cnt[u] = pl[(NS + u) * kWave + lane];
        r_rem[u] = pl[(2 * NS + u) * kWave + lane];
        r_nrem[u] = pl[(3 * NS + u) * kWave + lane];
      }
#pragma unroll
      for (int h = 0; h < 8; ++h) r_partner[h] = pl[(4 * NS + h) * kWave + lane];
    }
  }
  __device__ __forceinline__ int start(int u) const { return pl[u * kWave + lane]; }
  __device__ __forceinline__ int cnt(int u) const { return kRegs ? r_cnt[kRegs ? u : 0] : pl[(NS + u) * kWave + lane]; }
  __device__ __forceinline__ int rem(int u) const {
    return kRegs ? r_rem[kRegs ? u : 0] : pl[(2 * NS + u) * kWave + lane];
  }
  __device__ __forceinline__ int nrem(int u) const {
    return kRegs ? r_nrem[kRegs ? u : 0] : pl[(3 * NS + u) * kWave + lane];
  }
  __device__ __forceinline__ int partner(int h) const {
    return kRegs ? r_partner[kRegs ? h : 0] : pl[(4 * NS + h) * kWave + lane];
  }

  __device__ __forceinline__ double rc_c(int u, int m, bool real) const {
#pragma clang fp contract(off)
    const double a = cp[(u * kRows + m) * kWave + lane];
    const double sl = ((rbits[kRc ? u : 0] >> m) & 1u) ? rshi : rslo;
    const double bd = (1.0 - rs * a) + sl;
    const double c = a / bd;
    return lb::uni(pad_guard) ? (real ? c : 0.0) : c;
  }
  __device__ __forceinline__ void fill_cache() {
    if (!kCache) return;
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int cu = cnt(u);
#pragma unroll
      for (int m = 0; m < kChain; ++m) cc[kCache ? u : 0][kCache ? m : 0] = rc_c(u, m, m < cu);
      cc[kCache ? u : 0][kCache ? kChain : 0] = rc_c(u, kChain, rem(u) >= 0);
    }
  }
  __device__ __forceinline__ double cval(int u, int m, int cu) const {
    if (kCache) return cc[kCache ? u : 0][kCache ? m : 0];
    if (kRc) return rc_c(u, m, m < cu);
    if (kPlan) return cp[(u * kRows + m) * kWave + lane];
    return m < cu ? cp[start(u) + 8 * m] : 0.0;
  }
  __device__ __forceinline__ double crem(int u, int ru) const {
    if (kPairs) return cp[(u * kRows + kChain) * kWave + lane];
    if (kCache) return cc[kCache ? u : 0][kCache ? kChain : 0];
    if (kRc) return rc_c(u, kChain, ru >= 0);
    if (kPlan) return cp[(u * kRows + kChain) * kWave + lane];
    return ru >= 0 ? cp[ru] : 0.0;
  }

  // svml_log of the forward difference's two arguments (x and x + h: almost
  // always one reduction row and one exponent): the second log reuses the
  // first's row and k ln2 terms H, L when its argument shares them -- the
  // values its own lookup would give, so the same bits -- and does its own
  // lookup in the lanes where it crossed a switch point (a branch that is
  // skipped when no lane did)
  __device__ __forceinline__ void log_pair(double x0, double x1, double& y0, double& y1) const {
#pragma clang fp contract(off)
    if (!NEMO_EXACT_LOGPAIR) {
      y0 = refmath::svml_log(x0, tb);
      y1 = refmath::svml_log(x1, tb);
      return;
    }
    const uint64_t b0 = refmath::as_u64(x0), b1 = refmath::as_u64(x1);
    const uint32_t p0 = (uint32_t)(b0 >> 30) & 0x3fffff, p1 = (uint32_t)(b1 >> 30) & 0x3fffff;
    const uint32_t bk = p0 >> 16;
    const uint32_t thr = tb.rthr_p[bk];
    const bool a0 = p0 >= thr;
    const double* row = tb.lrow_p + 4 * (2 * bk + (a0 ? 1 : 0));
    const double k = (double)(int)((b0 >> 52) & 0x7ff) + row[1];
    const double H = refmath::fma_(k, refmath::kSvmlLn2Hi, row[2]);
    const double L = refmath::fma_(refmath::kSvmlLn2Lo, k, row[3]);
    y0 = refmath::svml_log_core(refmath::svml_mant(b0), row[0], H, L);
    // exponent and bucket (bits 46..62) equal and the same side of the bucket's switch point
    const bool same = (b0 >> 46) == (b1 >> 46) && (p1 >= thr) == a0;
    if (__builtin_expect(same, 1))
      y1 = refmath::svml_log_core(refmath::svml_mant(b1), row[0], H, L);
    else
      y1 = refmath::svml_log(x1, tb);
  }

  // both points of the forward difference in one pass over c (each point's
  // own order of operations).  kLat (few optima per SIMD: the step's time is
  // one optimum's latency): a slot's 16 c values loaded at once, the logs in
  // pairs of elements; else (many per SIMD: throughput) the chain loop
  // unrolled by 4 with c read as it goes -- fewer registers, more waves.
  // one slot's chain sums of both points after the 8-accumulator combine and
  // the block's tail elements (the leaf values of its 8 blocks, on lanes 8 L)
  __device__ __forceinline__ void slot_sums(int u, double ex0, double ex1, double& a0, double& a1) const {
#pragma clang fp contract(off)
    const int cu = cnt(u);
    // the chain starts from -0.0: -0.0 + t is t for every t, so the first term
    // is added like the rest -- the same bits as starting from it, without a
    // select per term where the loop index is not a constant (the throughput
    // form's unroll by 4)
    a0 = -0.0;
    a1 = -0.0;
    // past the chain's count c is 0 (the rows are written so; cval gives 0),
    // so its term is log(0 ex + 1) = +0 and a + 0 = a: a is never -0 (a log is
    // never -0, and a sum of nonzero terms rounds to +0), so no select is needed
    auto step = [&](int, double cm) {
      double t0, t1;
      log_pair(cm * ex0 + 1.0, cm * ex1 + 1.0, t0, t1);
      a0 = a0 + t0;
      a1 = a1 + t1;
    };
    // (the cached throughput form keeps the unroll by 4: its cache then lives
    // in scratch, which measured faster than registers at its 3-wave budget --
    // 1.61 against 1.84 ms per 16-chain step, profiles/r6/r6f_forms_sweep.txt)
    if (kPairs) {
      // a group's pairs all requested before the first one's logs (the
      // scheduling barrier keeps the later loads from sinking to their use)
      constexpr int kG = NEMO_EXACT_SLOT_GROUP;
      const double2* pr = reinterpret_cast<const double2*>(cp + (size_t)u * kRows * kWave) + lane;
#pragma unroll 1
      for (int p = 0; p < kChain / 2; p += kG) {
        double2 cg[kG];
#pragma unroll
        for (int g = 0; g < kG; ++g) cg[g] = pr[(p + g) * kWave];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < kG; ++g) {
          step(2 * (p + g), cg[g].x);
          step(2 * (p + g) + 1, cg[g].y);
        }
      }
    } else if (kLat) {
      double c[kChain];
#pragma unroll
      for (int m = 0; m < kChain; ++m) c[m] = cval(u, m, cu);
#pragma unroll
      for (int m = 0; m < kChain; ++m) {
        step(m, c[m]);
        if (m & 1) __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll NEMO_EXACT_TPUT_UNROLL
      for (int m = 0; m < kChain; ++m) step(m, cval(u, m, cu));
    }
    // the block's 8 accumulators: ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))
    a0 = a0 + __shfl_xor(a0, 1);
    a1 = a1 + __shfl_xor(a1, 1);
    a0 = a0 + __shfl_xor(a0, 2);
    a1 = a1 + __shfl_xor(a1, 2);
    a0 = a0 + __shfl_xor(a0, 4);
    a1 = a1 + __shfl_xor(a1, 4);
    if (lb::uni(maxrem > 0)) {  // the block's n % 8 trailing elements, in order
      const int ru = rem(u), nr = nrem(u);
      const double cr = crem(u, ru);
      const double tr0 = ru >= 0 ? refmath::svml_log(cr * ex0 + 1.0, tb) : 0.0;
      const double tr1 = ru >= 0 ? refmath::svml_log(cr * ex1 + 1.0, tb) : 0.0;
      for (int r = 0; r < 7; ++r) {
        const double y0 = __shfl(tr0, (lane & ~7) + r);
        const double y1 = __shfl(tr1, (lane & ~7) + r);
        a0 = r < nr ? a0 + y0 : a0;
        a1 = r < nr ? a1 + y1 : a1;
      }
    }
  }

  // the leaves to the root: leaf L (slot L / 8, lanes 8 (L % 8) ..) to lane
  // L, then the recursion's additions one height at a time
  __device__ __forceinline__ void tree(const double (&res0)[NS], const double (&res1)[NS], double& s0,
                                       double& s1) const {
#pragma clang fp contract(off)
    double v0 = 0.0, v1 = 0.0;
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const double x0 = __shfl(res0[u], 8 * (lane & 7));
      const double x1 = __shfl(res1[u], 8 * (lane & 7));
      v0 = (lane >> 3) == u ? x0 : v0;
      v1 = (lane >> 3) == u ? x1 : v1;
    }
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      if (!lb::uni(h < nh)) break;
      const int p = partner(h);
      const double y0 = __shfl(v0, p < 0 ? lane : p);
      const double y1 = __shfl(v1, p < 0 ? lane : p);
      v0 = p >= 0 ? v0 + y0 : v0;
      v1 = p >= 0 ? v1 + y1 : v1;
    }
    s0 = __shfl(v0, 0);  // the root: its first leaf is leaf 0
    s1 = __shfl(v1, 0);
  }

  // the pair form (kPair: two waves per optimum, the slots split between
  // them, u % 2 == half): each wave's slot sums meet in LDS (double-buffered
  // by evaluation parity), then both waves form the same root
  double* xres = nullptr;   // [2][NS][64][2] in LDS
  int half = 0, par = 0;

  __device__ __forceinline__ void sum_logs2(double ex0, double ex1, double& s0, double& s1) {
#pragma clang fp contract(off)
    // c is memory the compiler must read here, not values it carries over
    // from the writes (that would hold them in registers through the optimiser)
    __asm__ volatile("" ::: "memory");
    double res0[NS], res1[NS];
    if (kPair) {
      double* xr = xres + (size_t)par * NS * kWave * 2;
      par ^= 1;
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        if ((u & 1) != half) continue;
        if (u > 1) __asm__ volatile("" ::: "memory");
        double a0, a1;
        slot_sums(u, ex0, ex1, a0, a1);
        xr[(u * kWave + lane) * 2] = a0;
        xr[(u * kWave + lane) * 2 + 1] = a1;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        res0[u] = xr[(u * kWave + lane) * 2];
        res1[u] = xr[(u * kWave + lane) * 2 + 1];
      }
    } else if (!kMP) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        if (kLat && u > 0) __asm__ volatile("" ::: "memory");   // one slot's c loaded at a time
        slot_sums(u, ex0, ex1, res0[u], res1[u]);
      }
    } else {
      // numpy's buffers of 8192 terms (E > 8192), each summed pairwise on
      // its own wave plan and added to the running sum in order
      const int32_t* pl0 = pl;
      const double* cp0 = cp;
      const int nh0 = nh, mr0 = maxrem;
      double q0 = 0.0, q1 = 0.0;
      for (int p = 0; p < nparts; ++p) {
        pl = plg + (size_t)p * (4 * NS + 8) * kWave;
        nh = pmeta[2 * p];
        maxrem = pmeta[2 * p + 1];
        if (kPlan) cp = cp0 + (size_t)p * NS * kRows * kWave;
        if (kRc) {
#pragma unroll
          for (int u = 0; u < NS; ++u) rbits[kRc ? u : 0] = xbk[((size_t)p * NS + u) * kWave + lane];
        }
#pragma unroll
        for (int u = 0; u < NS; ++u) {
          __asm__ volatile("" ::: "memory");
          slot_sums(u, ex0, ex1, res0[u], res1[u]);
        }
        double p0, p1;
        tree(res0, res1, p0, p1);
        q0 = p == 0 ? p0 : q0 + p0;
        q1 = p == 0 ? p1 : q1 + p1;
      }
      pl = pl0;
      cp = cp0;
      nh = nh0;
      maxrem = mr0;
      s0 = q0;
      s1 = q1;
      return;
    }
    tree(res0, res1, s0, s1);
  }

  __device__ __forceinline__ void operator()(double x0, double x1, double& f0, double& f1) {
#pragma clang fp contract(off)
    const double e0 = refmath::expit(x0, tb);
    const double e1 = refmath::expit(x1, tb);
    double p0, p1;
    sum_logs2(e0, e1, p0, p1);
    f0 = (-p0 + fabs(e0 - anc)) + e0 * (1.0 - e0);
    f1 = (-p1 + fabs(e1 - anc)) + e1 * (1.0 - e1);
  }
};

// the plan's rows to LDS (every thread of the block)
template <int NS>
__device__ __forceinline__ void plan_to_lds(const int32_t* __restrict__ plan, int nh, int32_t* lds) {
  const int n = (4 * NS + nh) * kWave;
  for (int q = threadIdx.x; q < (4 * NS + 8) * kWave; q += blockDim.x) lds[q] = q < n ? plan[q] : -1;
}

struct SeqSumArgs {
  const double* cs = nullptr;
  int E = 0, batch = 0;
  double* ll = nullptr;
};

constexpr int kExactWaves = 4;
constexpr int kStateDoubles = (int)((sizeof(LbxState) + 7) / 8);

// The local optima's c rows (both forms): the stored form writes c = a / b,
// nem_order_mcmc.py:161-164 (local_vec = np.exp(T[i][k])), once, into this
// optimum's plan-ordered rows `rows` (`slots`: the slots this wave writes,
// bit u); the recompute form instead points the objective at the parent's a
// rows (xa, written by eval #1's order-weight launch) with s, s (lv - 1) and
// the lane's lv bits
struct CArgs {
  const double* xa = nullptr;        // kRc: [chains][S][plan doubles]
  const uint32_t* xbits = nullptr;   // kRc: [S][NS][64]
  double* cbuf = nullptr;            // stored: [optima][plan doubles]
  int xcd = 0;                       // XCD-contiguous optimum ranges (option exact_xcd)
  long long* trace = nullptr;        // option exact_trace: [optima][4] start / end (wall_clock64), objective /
                                     // control shader cycles
  int* queue = nullptr;              // option exact_persist: the work counter (zeroed before the launch)
  const int32_t* order = nullptr;    // the optima in the order they are handed out (null: launch order)
  int32_t* cost = nullptr;           // option exact_sched: [chains][S][S] each pair's last evaluation count
  // numpy's pairwise sum in nparts wave plans (two: the halves of its top
  // split, E > 8192): the plans' rows in global memory, [part][2] (tree
  // height, largest trailing count), and the doubles of one plan-ordered row
  // set over all parts
  int nparts = 1;
  const int32_t* plan = nullptr;
  const int32_t* pmeta = nullptr;
  size_t pd = 0;
  // kSlot (form 7): one plan-ordered c row set per resident wave, [waves][pd]
  double* sbuf = nullptr;
};

// The persistent form (option exact_persist): resident blocks whose waves take
// optima from a counter until none is left, so a wave's slot is refilled the
// moment its optimum ends (in one-optimum-per-wave blocks a block's slots free
// only when its slowest optimum ends: 0.56 of the slots busy on average at 16
// C3 chains, tools/lo_timeline.py).  Every wave ends when the counter passes
// the last optimum.  Lane 0 takes the item, the wave reads it uniformly.
__device__ __forceinline__ int next_item(int* q, int lane) {
  int v = 0;
  if (lane == 0) v = atomicAdd(q, 1);
  return __builtin_amdgcn_readfirstlane(v);
}
template <class Obj, int NS, bool kRc>
__device__ __forceinline__ void setup_c(Obj& obj, const CArgs& ca, int S, int E, int b, int k, size_t gw, double s,
                                        double lvlo, double lvhi, const double* __restrict__ owk,
                                        const uint64_t* __restrict__ d1w, int nwords, int lane, unsigned slots) {
#pragma clang fp contract(off)
  constexpr size_t kPlanD = (size_t)NS * Obj::kRows * kWave;   // (one part: the stored form)
  if (kRc) {
    obj.cp = ca.xa + ((size_t)b * S + k) * ca.pd;
    obj.xbk = ca.xbits + (size_t)k * NS * ca.nparts * kWave;
#pragma unroll
    for (int u = 0; u < NS; ++u) obj.rbits[kRc ? u : 0] = obj.xbk[(size_t)u * kWave + lane];
    obj.rs = s;
    obj.rslo = s * (lvlo - 1.0);
    obj.rshi = s * (lvhi - 1.0);
    obj.pad_guard = 1.0 + obj.rslo == 0.0;
    return;
  }
  auto cval = [&](int e) {
#pragma clang fp contract(off)
    const double lv = d1bit(d1w, nwords, k, e) ? lvhi : lvlo;
    const double a = (lv - 1.0) * owk[e];
    const double bd = (1.0 - s * a) + s * (lv - 1.0);
    return a / bd;
  };
  double* rows = ca.cbuf + gw * kPlanD;
  obj.cp = rows;
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    if (!((slots >> u) & 1u)) continue;
    const int st = obj.start(u), ct = obj.cnt(u), re = obj.rem(u);
    double* row = rows + u * Obj::kRows * kWave + lane;
#pragma unroll 4
    for (int m = 0; m < Obj::kChain; ++m) row[m * kWave] = m < ct ? cval(st + 8 * m) : 0.0;
    row[Obj::kChain * kWave] = re >= 0 ? cval(re) : 0.0;
  }
  __threadfence_block();   // the rows are read back by the same lanes
}

// The slot form (form 7): the recompute form's c values -- rc_c's operations
// on the parent's a rows and lv bits, so the same bits -- made once per
// optimum into this resident wave's own row set `rows` (plan order, one
// coalesced row per element), which the objective then reads like a stored
// row set: no division, select or bit test per element and evaluation.  The
// same lanes write and read the rows.
template <class Obj, int NS>
__device__ __forceinline__ void setup_slot(Obj& obj, const CArgs& ca, int S, int b, int k, double s, double lvlo,
                                           double lvhi, int lane, double* __restrict__ rows) {
#pragma clang fp contract(off)
  const double* xa = ca.xa + ((size_t)b * S + k) * ca.pd;
  const uint32_t* xb = ca.xbits + (size_t)k * NS * kWave;
  const double rslo = s * (lvlo - 1.0), rshi = s * (lvhi - 1.0);
  const bool pad_guard = lb::uni(1.0 + rslo == 0.0);
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    const uint32_t bits = xb[(size_t)u * kWave + lane];
    const int cu = obj.cnt(u), ru = obj.rem(u);
#pragma unroll 4
    for (int m = 0; m <= Obj::kChain; ++m) {
      const size_t at = (size_t)(u * Obj::kRows + m) * kWave + lane;
      // (kPairs: chain rows as pairs, element m of pair m / 2 at its m % 2)
      const size_t to = Obj::kPairsLayout && m < Obj::kChain
                            ? (size_t)u * Obj::kRows * kWave + ((size_t)(m >> 1) * kWave + lane) * 2 + (m & 1)
                            : at;
      const double a = xa[at];
      const double sl = ((bits >> m) & 1u) ? rshi : rslo;
      const double bd = (1.0 - s * a) + sl;
      const double c = a / bd;
      const bool real = m < Obj::kChain ? m < cu : ru >= 0;
      rows[to] = pad_guard ? (real ? c : 0.0) : c;
    }
  }
  obj.cp = rows;
  __threadfence_block();   // the rows are read back by the same lanes
}

// one wave per (chain, permissible pair), kExactWaves per block; then the
// appended blocks of `fin` (eval #1's ll, one lane per chain)
// kCt (form 4, the cached throughput form): the throughput form's objective
// loop on the latency form's register c cache, at NEMO_EXACT_CT_WAVES per SIMD
// kSlot (form 7, the slot form): the throughput form reading c from the
// resident wave's row set made by setup_slot (persistent launches only)
template <int NS, bool kLat, bool kRc, bool kCt = false, bool kMP = false, bool kSlot = false>
__global__ __launch_bounds__(kExactWaves * kWave)
__attribute__((amdgpu_waves_per_eu(kSlot ? NEMO_EXACT_SLOT_WAVES : kCt ? NEMO_EXACT_CT_WAVES : kLat ? 2 : NEMO_EXACT_TPUT_WAVES,
                                   kSlot ? NEMO_EXACT_SLOT_WAVES : kCt ? NEMO_EXACT_CT_WAVES : kLat ? 2 : NEMO_EXACT_TPUT_WAVES))) void local_opt_exact_kernel(
    int S, int E, int npairs, int nchains, const int32_t* __restrict__ pairs, const double* __restrict__ w01,
    const double* __restrict__ anc, const double* __restrict__ ow, const double* __restrict__ xlo,
    const double* __restrict__ xhi, const uint64_t* __restrict__ d1w, int nwords, const int32_t* __restrict__ plan,
    int nh, int maxrem, double sig0, double sig1, double* __restrict__ wnew, double* __restrict__ wdag,
    int32_t* __restrict__ info, CArgs ca, int lo_blocks, SeqSumArgs fin) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  __shared__ double mem[kExactWaves][lbx::kMemDoubles];
  __shared__ double lst_raw[kExactWaves][kStateDoubles];   // LbxState (not trivially constructible)
  __shared__ int32_t pl[(4 * NS + 8) * kWave];
  if ((int)blockIdx.x >= lo_blocks) {   // one wave per chain
    const int bb = __builtin_amdgcn_readfirstlane(((int)blockIdx.x - lo_blocks) * kExactWaves +
                                                  (int)threadIdx.x / kWave);
    const int ln = threadIdx.x & (kWave - 1);
    if (bb < fin.batch) {
      const double v = wave_seq_sum(fin.cs + (size_t)bb * fin.E, fin.E, ln, &mem[threadIdx.x / kWave][0]);
      if (ln == 0) fin.ll[bb] = v;
    }
    return;
  }
  tabs.fill(threadIdx.x, blockDim.x);
  plan_to_lds<NS>(plan, nh, pl);
  __syncthreads();
  const int wv = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int total = nchains * npairs;
  int item = ca.queue ? next_item(ca.queue, lane)
                      : __builtin_amdgcn_readfirstlane(xcd_block(ca.xcd, (int)blockIdx.x, lo_blocks) * kExactWaves + wv);
  for (; item < total; item = ca.queue ? next_item(ca.queue, lane) : total) {   // uniform per wave
  const int gw = ca.order ? __builtin_amdgcn_readfirstlane(ca.order[item]) : item;
  const int b = gw / npairs;
  const int n = gw - b * npairs;
  const int pk = pairs[(size_t)b * S * S + n];
  const int i = pk >> 16;
  const int k = pk & 0xffff;
  const size_t idx = ((size_t)b * S + i) * S + k;
  const double s = w01[idx];
  const double* owk = ow + ((size_t)b * (S + 1) + k) * E;
  const long long t_start = ca.trace ? (long long)wall_clock64() : 0;
  using Obj = ExactObjective<NS, true, kLat, false, kRc && !kSlot, (kLat || kCt) && kRc && NEMO_EXACT_CCACHE, kMP,
                             kSlot && NEMO_EXACT_SLOT_PAIRS>;
  Obj obj;
  obj.tb = tabs.view();
  obj.pl = pl;
  obj.lane = lane;
  obj.nh = nh;
  obj.maxrem = maxrem;
  obj.anc = anc[idx];
  obj.load_plan();
  if constexpr (kSlot)
    setup_slot<Obj, NS>(obj, ca, S, b, k, s, xlo[k], xhi[k], lane,
                        ca.sbuf + ((size_t)blockIdx.x * kExactWaves + wv) * ca.pd);
  else
    setup_c<Obj, NS, kRc>(obj, ca, S, E, b, k, (size_t)gw, s, xlo[k], xhi[k], owk, d1w, nwords, lane, ~0u);
  obj.nparts = ca.nparts;
  obj.plg = ca.plan;
  obj.pmeta = ca.pmeta;
  obj.fill_cache();
  LbxState& st = *reinterpret_cast<LbxState*>(lst_raw[wv]);
  lbx_init(st, s);
  long long c_obj = 0, c_ctl = 0, tc = ca.trace ? (long long)clock64() : 0;   // (trace: shader cycles)
  while (lbx_run(st, lbx::Mem{mem[wv]})) {
    double f0, f1;
    const long long t1 = ca.trace ? (long long)clock64() : 0;
    obj(st.x_eval, st.x1, f0, f1);
    if (ca.trace) {
      const long long t2 = (long long)clock64();
      c_ctl += t1 - tc;
      c_obj += t2 - t1;
      tc = t2;
    }
    lbx_feed(st, f0, f1);
  }
  if (ca.trace) c_ctl += (long long)clock64() - tc;
  const LbfgsResult r{st.x, st.f, st.nit, st.nfev, st.status};
  if (lane == 0) {
    const double wx = refmath::expit(r.x, obj.tb);
    wnew[idx] = wx;
    wdag[idx] = (wx > 0.5) ? sig1 : sig0;
    if (info) {
      const int nit = r.nit < 4095 ? r.nit : 4095;
      const int nfev = r.nfev < 32767 ? r.nfev : 32767;
      info[idx] = (int32_t)(r.status | (nit << 4) | (nfev << 16));
    }
    if (ca.cost) ca.cost[idx] = r.nfev;
    if (ca.trace) {
      ca.trace[4 * (size_t)gw] = t_start;
      ca.trace[4 * (size_t)gw + 1] = (long long)wall_clock64();
      ca.trace[4 * (size_t)gw + 2] = c_obj;
      ca.trace[4 * (size_t)gw + 3] = c_ctl;
    }
  }
  }
}

// The pair form (few optima: a step's time is its slowest optimum): two waves
// per (chain, pair), one block each, the objective's slots split between
// them (u % 2 == the wave) and met in LDS per evaluation; both waves run the
// same optimiser on their own copy of its state, so they take the same path
// and the same number of barriers.  Appended blocks as above (two chains per
// block).
template <int NS, bool kRc>
__global__ __launch_bounds__(2 * kWave) __attribute__((amdgpu_waves_per_eu(4, 4))) void local_opt_exact_pair_kernel(
    int S, int E, int npairs, int nchains, const int32_t* __restrict__ pairs, const double* __restrict__ w01,
    const double* __restrict__ anc, const double* __restrict__ ow, const double* __restrict__ xlo,
    const double* __restrict__ xhi, const uint64_t* __restrict__ d1w, int nwords, const int32_t* __restrict__ plan,
    int nh, int maxrem, double sig0, double sig1, double* __restrict__ wnew, double* __restrict__ wdag,
    int32_t* __restrict__ info, CArgs ca, int lo_blocks, SeqSumArgs fin) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  __shared__ double mem[2][lbx::kMemDoubles];
  __shared__ double lst_raw[2][kStateDoubles];
  __shared__ double xres[2 * NS * kWave * 2];
  const int wv = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  if ((int)blockIdx.x >= lo_blocks) {   // one wave per chain
    const int bb = __builtin_amdgcn_readfirstlane(((int)blockIdx.x - lo_blocks) * 2 + wv);
    if (bb < fin.batch) {
      const double v = wave_seq_sum(fin.cs + (size_t)bb * fin.E, fin.E, lane, &mem[wv][0]);
      if (lane == 0) fin.ll[bb] = v;
    }
    return;
  }
  __shared__ int s_item;
  tabs.fill(threadIdx.x, blockDim.x);
  const int total = nchains * npairs;
  // the optimum, uniform over the block: taken by thread 0 and handed to both
  // waves through LDS (the barriers sit in straight-line code, executed the
  // same number of times by both waves)
  auto fetch = [&]() {
    if (threadIdx.x == 0) s_item = atomicAdd(ca.queue, 1);
    __syncthreads();
    const int v = __builtin_amdgcn_readfirstlane(s_item);
    __syncthreads();   // both waves hold it before thread 0 may take the next
    return v;
  };
  __syncthreads();
  int item = ca.queue ? fetch() : xcd_block(ca.xcd, (int)blockIdx.x, lo_blocks);
  while (item < total) {
  const int gw = ca.order ? __builtin_amdgcn_readfirstlane(ca.order[item]) : item;
  const int b = gw / npairs;
  const int n = gw - b * npairs;
  const int pk = pairs[(size_t)b * S * S + n];
  const int i = pk >> 16;
  const int k = pk & 0xffff;
  const size_t idx = ((size_t)b * S + i) * S + k;
  const double s = w01[idx];
  const double* owk = ow + ((size_t)b * (S + 1) + k) * E;
  const long long t_start = ca.trace ? (long long)wall_clock64() : 0;
  // the throughput form's objective (few registers: four waves per SIMD
  // hold the 2 x 2016 waves of one chain's step), its plan in registers
  // (read once from global memory: no LDS copy, so eight blocks fit a CU)
  using Obj = ExactObjective<NS, true, false, true, kRc>;
  Obj obj;
  obj.tb = tabs.view();
  obj.pl = plan;
  obj.lane = lane;
  obj.nh = nh;
  obj.maxrem = maxrem;
  obj.anc = anc[idx];
  obj.xres = xres;
  obj.half = wv;
  obj.load_plan();
  // this wave's slots' rows (it alone reads them)
  setup_c<Obj, NS, kRc>(obj, ca, S, E, b, k, (size_t)gw, s, xlo[k], xhi[k], owk, d1w, nwords, lane,
                        wv ? 0xaaaaaaaau : 0x55555555u);
  LbxState& st = *reinterpret_cast<LbxState*>(lst_raw[wv]);
  lbx_init(st, s);
  long long c_obj = 0, c_ctl = 0, tc = ca.trace ? (long long)clock64() : 0;   // (trace: shader cycles)
  while (lbx_run(st, lbx::Mem{mem[wv]})) {
    double f0, f1;
    const long long t1 = ca.trace ? (long long)clock64() : 0;
    obj(st.x_eval, st.x1, f0, f1);
    if (ca.trace) {
      const long long t2 = (long long)clock64();
      c_ctl += t1 - tc;
      c_obj += t2 - t1;
      tc = t2;
    }
    lbx_feed(st, f0, f1);
  }
  if (ca.trace) c_ctl += (long long)clock64() - tc;
  if (wv == 0 && lane == 0) {
    const double wx = refmath::expit(st.x, obj.tb);
    wnew[idx] = wx;
    wdag[idx] = (wx > 0.5) ? sig1 : sig0;
    if (info) {
      const int nit = st.nit < 4095 ? st.nit : 4095;
      const int nfev = st.nfev < 32767 ? st.nfev : 32767;
      info[idx] = (int32_t)(st.status | (nit << 4) | (nfev << 16));
    }
    if (ca.cost) ca.cost[idx] = st.nfev;
    if (ca.trace) {
      ca.trace[4 * (size_t)gw] = t_start;
      ca.trace[4 * (size_t)gw + 1] = (long long)wall_clock64();
      ca.trace[4 * (size_t)gw + 2] = c_obj;
      ca.trace[4 * (size_t)gw + 3] = c_ctl;
    }
  }
  item = ca.queue ? fetch() : total;
  }
}

// The dual form (option exact_form 5): two optima per wave.  Half h of the
// wave (lanes 32 h .. 32 h + 31) runs optimum h's control -- lbfgsb_exact.h
// with H = true: the same operations spread over 32 lanes instead of 64, its
// branches divergent by half -- and every lane holds BOTH optima's c values
// at its plan positions (the latency form's register cache, twice), so one
// pass of the objective makes both optima's forward differences.  Two optima
// share each control instruction the halves take together, and each pass of
// the objective carries twice the independent logs.  Each optimum's rounded
// operations are those of the one-wave forms, so the bits are the same.
template <int NS>
struct DualObjective {
  static constexpr int kChain = 16;
  static constexpr int kRows = kChain + 1;
  double cc[2][NS][kRows];   // optimum o's c values at this lane's plan positions
  const int32_t* pl;         // host::PairwisePlan rows in LDS (ExactObjective)
  int nh, maxrem, lane;
  LdsTabs tb;

  __device__ __forceinline__ int cnt(int u) const { return pl[(NS + u) * kWave + lane]; }
  __device__ __forceinline__ int rem(int u) const { return pl[(2 * NS + u) * kWave + lane]; }
  __device__ __forceinline__ int nrem(int u) const { return pl[(3 * NS + u) * kWave + lane]; }
  __device__ __forceinline__ int partner(int h) const { return pl[(4 * NS + h) * kWave + lane]; }

  // optimum o's c = a / ((1 - s a) + s (lv - 1)) from its parent's
  // plan-ordered a rows (ExactObjective::rc_c, fill_cache)
  template <int o>
  __device__ __forceinline__ void fill(const double* __restrict__ cp, const uint32_t* rbits, double rs, double rslo,
                                       double rshi, bool pad_guard) {
#pragma clang fp contract(off)
    auto cv = [&](int u, int m, bool real) {
      const double a = cp[(u * kRows + m) * kWave + lane];
      const double sl = ((rbits[u] >> m) & 1u) ? rshi : rslo;
      const double bd = (1.0 - rs * a) + sl;
      const double c = a / bd;
      return pad_guard ? (real ? c : 0.0) : c;
    };
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int cu = cnt(u);
#pragma unroll
      for (int m = 0; m < kChain; ++m) cc[o][u][m] = cv(u, m, m < cu);
      cc[o][u][kChain] = cv(u, kChain, rem(u) >= 0);
    }
  }

  // slot u's chain sums of the four points (optimum o, point p: a[2 o + p]),
  // each as ExactObjective::slot_sums makes it
  __device__ __forceinline__ void slot_sums(int u, const double (&ex)[4], double (&a)[4]) const {
#pragma clang fp contract(off)
    // fully unrolled: the cache is registers only while every index is a
    // constant (a loop index would put it in scratch); one element's four
    // logs at a time in the schedule
#pragma unroll
    for (int m = 0; m < kChain; ++m) {
      double t[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = refmath::svml_log(cc[q >> 1][u][m] * ex[q] + 1.0, tb);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = m == 0 ? t[q] : a[q] + t[q];
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int d = 1; d <= 4; d <<= 1)
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = a[q] + __shfl_xor(a[q], d);
    if (lb::uni(maxrem > 0)) {
      const int ru = rem(u), nr = nrem(u);
      double tr[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) tr[q] = ru >= 0 ? refmath::svml_log(cc[q >> 1][u][kChain] * ex[q] + 1.0, tb) : 0.0;
      for (int r = 0; r < 7; ++r) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double y = __shfl(tr[q], (lane & ~7) + r);
          a[q] = r < nr ? a[q] + y : a[q];
        }
      }
    }
  }

  // ExactObjective::tree for the four sums
  __device__ __forceinline__ void tree(const double (&res)[NS][4], double (&s)[4]) const {
#pragma clang fp contract(off)
    double v[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < NS; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double x = __shfl(res[u][q], 8 * (lane & 7));
        v[q] = (lane >> 3) == u ? x : v[q];
      }
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      if (!lb::uni(h < nh)) break;
      const int p = partner(h);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double y = __shfl(v[q], p < 0 ? lane : p);
        v[q] = p >= 0 ? v[q] + y : v[q];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] = __shfl(v[q], 0);
  }

  // f at x[q] (optimum q >> 1, point q & 1), local_ll_sum_penalized (:18-23)
  __device__ __forceinline__ void operator()(const double (&x)[4], double anc0, double anc1, double (&f)[4]) const {
#pragma clang fp contract(off)
    double e[4], res[NS][4], p[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) e[q] = refmath::expit(x[q], tb);
#pragma unroll
    for (int u = 0; u < NS; ++u) slot_sums(u, e, res[u]);
    tree(res, p);
#pragma unroll
    for (int q = 0; q < 4; ++q) f[q] = (-p[q] + fabs(e[q] - (q < 2 ? anc0 : anc1))) + e[q] * (1.0 - e[q]);
  }
};

template <int NS>
__global__ __launch_bounds__(kExactWaves * kWave) __attribute__((amdgpu_waves_per_eu(2, 2))) void local_opt_exact_dual_kernel(
    int S, int E, int npairs, int nchains, const int32_t* __restrict__ pairs, const double* __restrict__ w01,
    const double* __restrict__ anc, const double* __restrict__ xlo, const double* __restrict__ xhi,
    const int32_t* __restrict__ plan, int nh, int maxrem, double sig0, double sig1, double* __restrict__ wnew,
    double* __restrict__ wdag, int32_t* __restrict__ info, CArgs ca, int lo_blocks, SeqSumArgs fin) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  __shared__ double mem[kExactWaves][2][lbx::kMemDoubles];
  __shared__ double lst_raw[kExactWaves][2][kStateDoubles];
  __shared__ int32_t pl[(4 * NS + 8) * kWave];
  const int wv = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  if ((int)blockIdx.x >= lo_blocks) {   // one wave per chain: eval #1's ll
    const int bb = __builtin_amdgcn_readfirstlane(((int)blockIdx.x - lo_blocks) * kExactWaves + wv);
    if (bb < fin.batch) {
      const double v = wave_seq_sum(fin.cs + (size_t)bb * fin.E, fin.E, lane, &mem[wv][0][0]);
      if (lane == 0) fin.ll[bb] = v;
    }
    return;
  }
  tabs.fill(threadIdx.x, blockDim.x);
  plan_to_lds<NS>(plan, nh, pl);
  __syncthreads();
  const int hf = lane >> 5;
  const int total = nchains * npairs;
  const size_t kPlanD = ca.pd;   // (one part: the dual form is not taken for two)
  DualObjective<NS> obj;
  obj.tb = tabs.view();
  obj.pl = pl;
  obj.lane = lane;
  obj.nh = nh;
  obj.maxrem = maxrem;
  LbxState& st = *reinterpret_cast<LbxState*>(lst_raw[wv][hf]);   // this half's optimum's state
  const lbx::Mem mm{mem[wv][hf]};
  // per slot (uniform): the optimum's (chain, child, parent) index and anc
  size_t idx0 = 0, idx1 = 0;
  double anc0 = 0.0, anc1 = 0.0;
  // take the next optimum into slot o: its c values (every lane) and its
  // control's start (half o); false when the queue is drained
  auto take = [&](auto oc) -> bool {
    constexpr int o = decltype(oc)::value;
    const int item = next_item(ca.queue, lane);
    if (item >= total) return false;
    const int gw = ca.order ? __builtin_amdgcn_readfirstlane(ca.order[item]) : item;
    const int b = gw / npairs;
    const int n = gw - b * npairs;
    const int pk = pairs[(size_t)b * S * S + n];
    const int i = pk >> 16;
    const int k = pk & 0xffff;
    const size_t idx = ((size_t)b * S + i) * S + k;
    const double s = w01[idx];
    uint32_t rb[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) rb[u] = ca.xbits[((size_t)k * NS + u) * kWave + lane];
    const double rslo = s * (xlo[k] - 1.0), rshi = s * (xhi[k] - 1.0);
    obj.template fill<o>(ca.xa + ((size_t)b * S + k) * kPlanD, rb, s, rslo, rshi,
                         __builtin_amdgcn_readfirstlane((int)(1.0 + rslo == 0.0)) != 0);
    if (o == 0) idx0 = idx, anc0 = anc[idx];
    else idx1 = idx, anc1 = anc[idx];
    if (hf == o) lbx_init(st, s);
    return true;
  };
  // One call site of the control (every inlined copy costs registers next to
  // the two caches): passes over the halves that need their next point --
  // after an evaluation, or a fresh optimum its first -- until both have one
  // or are drained; an optimum that ends hands its slot to the next one,
  // which then needs a pass of its own
  bool act0 = false, act1 = false;
  bool need0 = false, need1 = false;
  uint64_t ended = ~0ull;   // both slots take their first optimum
  for (;;) {
    for (;;) {
      if (ended & 1ull) need0 = act0 = take(std::integral_constant<int, 0>{});
      if (ended >> 32) need1 = act1 = take(std::integral_constant<int, 1>{});
      const bool run = hf ? need1 : need0;
      if (__ballot(run) == 0ull) break;
      const bool more = run ? lbx_run<true>(st, mm) : false;
      const bool done = run && !more;
      if (done && (lane & 31) == 0) {   // optimum hf ended: its outputs (as local_opt_exact_kernel)
        const size_t idx = hf ? idx1 : idx0;
        const double wx = refmath::expit(st.x, obj.tb);
        wnew[idx] = wx;
        wdag[idx] = (wx > 0.5) ? sig1 : sig0;
        if (info) {
          const int nit = st.nit < 4095 ? st.nit : 4095;
          const int nfev = st.nfev < 32767 ? st.nfev : 32767;
          info[idx] = (int32_t)(st.status | (nit << 4) | (nfev << 16));
        }
        if (ca.cost) ca.cost[idx] = st.nfev;
      }
      ended = __ballot(done);
      need0 = need1 = false;
    }
    if (!act0 && !act1) break;
    // both points of both optima (a drained slot's stale points are evaluated
    // and ignored)
    lbx::lanes_sync();
    const LbxState& s0 = *reinterpret_cast<const LbxState*>(lst_raw[wv][0]);
    const LbxState& s1 = *reinterpret_cast<const LbxState*>(lst_raw[wv][1]);
    const double x[4] = {act0 ? s0.x_eval : 0.0, act0 ? s0.x1 : 0.0, act1 ? s1.x_eval : 0.0, act1 ? s1.x1 : 0.0};
    double f[4];
    obj(x, anc0, anc1, f);
    if (hf ? act1 : act0) lbx_feed(st, hf ? f[2] : f[0], hf ? f[3] : f[1]);
    need0 = act0;
    need1 = act1;
    ended = 0ull;
  }
}

// the same optimiser on caller-supplied c vectors [n][E] (nemo_local_opt:
// calculate_local_optimum of one pair, and the scipy records of the tests);
// out [n][3] = x*, f*, packed info
// (kMP: numpy's pairwise sum in two wave plans, E > 8192 -- the objective
// reads each part's plan from global memory, nparts / pmeta as CArgs)
template <int NS, bool kMP = false>
__global__ __launch_bounds__(kExactWaves * kWave)
__attribute__((amdgpu_waves_per_eu(2, 2))) void local_opt_exact_generic_kernel(
    int E, int n, const double* __restrict__ cvec, const double* __restrict__ anc, const double* __restrict__ x0,
    const int32_t* __restrict__ plan, int nh, int maxrem, double* __restrict__ out, int nparts,
    const int32_t* __restrict__ pmeta) {
#pragma clang fp contract(off)
  __shared__ TabsLds tabs;
  __shared__ double mem[kExactWaves][lbx::kMemDoubles];
  __shared__ double lst_raw[kExactWaves][kStateDoubles];   // LbxState (not trivially constructible)
  __shared__ int32_t pl[(4 * NS + 8) * kWave];
  tabs.fill(threadIdx.x, blockDim.x);
  plan_to_lds<NS>(plan, nh, pl);
  __syncthreads();
  const int wv = threadIdx.x / kWave;
  const int p = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (p >= n) return;
  ExactObjective<NS, false, !kMP, false, false, false, kMP> obj;
  obj.tb = tabs.view();
  obj.pl = pl;
  obj.lane = lane;
  obj.nh = nh;
  obj.maxrem = maxrem;
  obj.anc = anc[p];
  obj.cp = cvec + (size_t)p * E;
  obj.nparts = kMP ? nparts : 1;
  obj.plg = plan;
  obj.pmeta = pmeta;
  obj.load_plan();
  LbxState& st = *reinterpret_cast<LbxState*>(lst_raw[wv]);
  lbx_init(st, x0[p]);
  while (lbx_run(st, lbx::Mem{mem[wv]})) {
    double f0, f1;
    obj(st.x_eval, st.x1, f0, f1);
    lbx_feed(st, f0, f1);
  }
  const LbfgsResult r{st.x, st.f, st.nit, st.nfev, st.status};
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
    case 7: r = v / y[g]; break;
    case 8: r = refmath::log1p_unit(v); break;
    default: r = v; break;
  }
  out[g] = r;
}

// The hand-out order of the persistent form (option exact_sched 1): the
// optima by their pair's evaluation count in the chain's previous step, most
// first -- longest-processing-time first, so the long optimisations do not
// start last and leave the end of the launch to a few waves
// (tools/lo_timeline.py: at 16 C3 chains the last 27% of the launch ran below
// half the resident waves).  Within one count the chains stay in launch order
// (a chain's optima share the parent rows the recompute form reads, so the
// waves in flight read few chains' rows at a time).  A counting sort in two
// launches of one block per chain: the chain's histogram over kSchedBuckets
// counts, then every block places its (count, chain) segment after all larger
// counts and all earlier chains of its count.  The order within a segment is
// whatever the LDS atomics give: it changes which wave takes which optimum,
// never a bit.
constexpr int kSchedBuckets = 64, kSchedThreads = 256;
__device__ __forceinline__ int sched_bucket(const int32_t* __restrict__ pairs, const int32_t* __restrict__ cost,
                                            int S, int b, int n) {
  const int pk = pairs[(size_t)b * S * S + n];
  const int c = cost[((size_t)b * S + (pk >> 16)) * S + (pk & 0xffff)] >> 1;   // evaluation pairs
  return kSchedBuckets - 1 - (c < kSchedBuckets - 1 ? c : kSchedBuckets - 1);   // most work: bucket 0
}

__global__ __launch_bounds__(kSchedThreads) void exact_sched_hist_kernel(int S, int npairs,
                                                                          const int32_t* __restrict__ pairs,
                                                                          const int32_t* __restrict__ cost,
                                                                          int* __restrict__ hist) {
  __shared__ int h[kSchedBuckets];
  const int b = blockIdx.x;
  for (int q = threadIdx.x; q < kSchedBuckets; q += blockDim.x) h[q] = 0;
  __syncthreads();
  for (int n = threadIdx.x; n < npairs; n += blockDim.x) atomicAdd(&h[sched_bucket(pairs, cost, S, b, n)], 1);
  __syncthreads();
  for (int q = threadIdx.x; q < kSchedBuckets; q += blockDim.x) hist[(size_t)b * kSchedBuckets + q] = h[q];
}

__global__ __launch_bounds__(kSchedThreads) void exact_sched_place_kernel(int S, int npairs, int nchains,
                                                                           const int32_t* __restrict__ pairs,
                                                                           const int32_t* __restrict__ cost,
                                                                           const int* __restrict__ hist,
                                                                           int32_t* __restrict__ order) {
  __shared__ int pos[kSchedBuckets];
  __shared__ int col[kSchedBuckets];
  const int b = blockIdx.x;
  // segment (q, b) starts after every optimum of buckets < q and those of
  // chains < b in bucket q: one thread per bucket sums its histogram column
  for (int q = threadIdx.x; q < kSchedBuckets; q += blockDim.x) {
    int tot = 0, before = 0;
    for (int c = 0; c < nchains; ++c) {
      const int v = hist[(size_t)c * kSchedBuckets + q];
      tot += v;
      before += c < b ? v : 0;
    }
    col[q] = tot;
    pos[q] = before;
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // the buckets before q (64 additions)
    int acc = 0;
    for (int q = 0; q < kSchedBuckets; ++q) {
      pos[q] += acc;
      acc += col[q];
    }
  }
  __syncthreads();
  for (int n = threadIdx.x; n < npairs; n += blockDim.x)
    order[atomicAdd(&pos[sched_bucket(pairs, cost, S, b, n)], 1)] = b * npairs + n;
}

}  // namespace

#ifndef NEMO_EXACT_KERNELS_ONLY   // (tools/ubench: the kernels alone, for their register reports)
hipError_t launch_local_opt_exact_generic(Ctx& c, int n, const double* d_c, const double* d_anc, const double* d_x0,
                                          double* d_out, hipStream_t st) {
  const dim3 grid((n + kExactWaves - 1) / kExactWaves);
  switch (c.pw_ns) {
#define NEMO_EXACT_NS(NSV)                                                                                  \
  case NSV:                                                                                                 \
    if (c.pw_parts > 1)                                                                                     \
      local_opt_exact_generic_kernel<NSV, true><<<grid, kExactWaves * kWave, 0, st>>>(                      \
          c.E, n, d_c, d_anc, d_x0, c.d_pwplan, c.pw_nh, c.pw_maxrem, d_out, c.pw_parts, c.d_pwmeta);       \
    else                                                                                                    \
      local_opt_exact_generic_kernel<NSV><<<grid, kExactWaves * kWave, 0, st>>>(                            \
          c.E, n, d_c, d_anc, d_x0, c.d_pwplan, c.pw_nh, c.pw_maxrem, d_out, 1, c.d_pwmeta);                \
    break;
    NEMO_EXACT_NS(1)
    NEMO_EXACT_NS(2)
    NEMO_EXACT_NS(3)
    NEMO_EXACT_NS(4)
    NEMO_EXACT_NS(5)
    NEMO_EXACT_NS(6)
    NEMO_EXACT_NS(7)
    NEMO_EXACT_NS(8)
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

size_t exact_plan_doubles(const Ctx& c) {
  return (size_t)c.pw_parts * c.pw_ns * (ExactObjective<1, true, true>::kRows * kWave);
}

hipError_t launch_exact_eval(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01, double* d_cells,
                             double* d_cs, double* d_ll, bool want_ow, hipStream_t st, double* d_xa) {
  const int S = c.S, E = c.E;
  // one wave per group of 4 D1 words, at most kCellsThreads / 64 waves; 8
  // children per block once the batch alone fills the chip
  const int cw = std::min(kCellsThreads / kWave, std::max(1, (c.nwords + 3) / 4));
  const int rows = batch >= 512 ? std::min(kCellsRows, kCellsSlots / S) : 1;
  const int nchunk = (S + rows) / rows;
  exact_cells_kernel<<<dim3(batch * nchunk), cw * kWave, 0, st>>>(S, E, rows, cap >= S - 1 ? 0 : cap, d_pos, d_w01,
                                                                  c.d_xlo, c.d_xhi,
                                                                  c.d_D1w, c.nwords, c.d_U64, d_cells);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  const size_t nthr = (size_t)batch * E;
  const int fb = (int)((nthr + 255) / 256);
  exact_fold_kernel<<<fb, 256, 0, st>>>(S, E, batch, d_cells, d_cs);
  err = hipGetLastError();
  if (err == hipSuccess && want_ow) {
    const size_t ncell = (size_t)batch * (S + 1) * E;
    exact_ow_kernel<<<(unsigned)((ncell + 255) / 256), 256, 0, st>>>(
        S, E, batch, d_cells, d_cs, d_xa, c.d_pwpos, (int)exact_plan_doubles(c), c.d_xlo, c.d_xhi, c.d_D1w,
        c.nwords);
    err = hipGetLastError();
  }
  if (err != hipSuccess || !d_ll) return err;
  exact_seq_sum_kernel<<<(batch + 3) / 4, 256, 0, st>>>(E, batch, d_cs, d_ll);
  return hipGetLastError();
}

namespace {

struct LoArgs {
  int S, E, npairs, nchains;
  const int32_t* pairs;
  const double *w01, *anc, *ow, *xlo, *xhi;
  const uint64_t* d1w;
  int nwords;
  const int32_t* plan;
  int nh, maxrem;
  double sig0, sig1;
  double *wnew, *wdag;
  int32_t* info;
  CArgs ca;
  int lo_blocks;
  SeqSumArgs fin;
};

// resident blocks of one kernel on the device at its block size (cached per kernel)
template <auto K>
int resident_blocks(int threads) {
  static int n = -1;
  if (n < 0) {
    int per_cu = 0, dev = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, K, threads, 0) != hipSuccess || per_cu < 1)
      per_cu = 1;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || ncu < 1)
      ncu = 256;
    n = per_cu * ncu;
  }
  return n;
}

template <int NS, bool kRc>
int lo_resident(int form) {
  if (form == 3) return resident_blocks<local_opt_exact_pair_kernel<NS, kRc>>(2 * kWave);
  if (form == 1) return resident_blocks<local_opt_exact_kernel<NS, true, kRc>>(kExactWaves * kWave);
  if (form == 4) return resident_blocks<local_opt_exact_kernel<NS, false, kRc, true>>(kExactWaves * kWave);
  if (form == 6) return resident_blocks<local_opt_exact_kernel<NS, false, true, false, true>>(kExactWaves * kWave);
  if (form == 7)
    return resident_blocks<local_opt_exact_kernel<NS, false, true, false, false, true>>(kExactWaves * kWave);
  return resident_blocks<local_opt_exact_kernel<NS, false, kRc>>(kExactWaves * kWave);
}

template <int NS>
int lo_resident_ns(int form, bool rc) {
  if (form == 5) {
    if constexpr (NS <= 2) return resident_blocks<local_opt_exact_dual_kernel<NS>>(kExactWaves * kWave);
    return 0;
  }
  return rc ? lo_resident<NS, true>(form) : lo_resident<NS, false>(form);
}

template <int NS, bool kRc>
void launch_lo(const LoArgs& a, int form, dim3 grid, hipStream_t st) {
  if (form == 3)
    local_opt_exact_pair_kernel<NS, kRc><<<grid, 2 * kWave, 0, st>>>(
        a.S, a.E, a.npairs, a.nchains, a.pairs, a.w01, a.anc, a.ow, a.xlo, a.xhi, a.d1w, a.nwords, a.plan, a.nh,
        a.maxrem, a.sig0, a.sig1, a.wnew, a.wdag, a.info, a.ca, a.lo_blocks, a.fin);
  else if (form == 1)
    local_opt_exact_kernel<NS, true, kRc><<<grid, kExactWaves * kWave, 0, st>>>(
        a.S, a.E, a.npairs, a.nchains, a.pairs, a.w01, a.anc, a.ow, a.xlo, a.xhi, a.d1w, a.nwords, a.plan, a.nh,
        a.maxrem, a.sig0, a.sig1, a.wnew, a.wdag, a.info, a.ca, a.lo_blocks, a.fin);
  else if (form == 6)   // (internal: the throughput form on two plan parts)
    local_opt_exact_kernel<NS, false, true, false, true><<<grid, kExactWaves * kWave, 0, st>>>(
        a.S, a.E, a.npairs, a.nchains, a.pairs, a.w01, a.anc, a.ow, a.xlo, a.xhi, a.d1w, a.nwords, a.plan, a.nh,
        a.maxrem, a.sig0, a.sig1, a.wnew, a.wdag, a.info, a.ca, a.lo_blocks, a.fin);
  else if (form == 7)   // (the slot form: recompute rows in, kRc)
    local_opt_exact_kernel<NS, false, true, false, false, true><<<grid, kExactWaves * kWave, 0, st>>>(
        a.S, a.E, a.npairs, a.nchains, a.pairs, a.w01, a.anc, a.ow, a.xlo, a.xhi, a.d1w, a.nwords, a.plan, a.nh,
        a.maxrem, a.sig0, a.sig1, a.wnew, a.wdag, a.info, a.ca, a.lo_blocks, a.fin);
  else if (form == 4)
    local_opt_exact_kernel<NS, false, kRc, true><<<grid, kExactWaves * kWave, 0, st>>>(
        a.S, a.E, a.npairs, a.nchains, a.pairs, a.w01, a.anc, a.ow, a.xlo, a.xhi, a.d1w, a.nwords, a.plan, a.nh,
        a.maxrem, a.sig0, a.sig1, a.wnew, a.wdag, a.info, a.ca, a.lo_blocks, a.fin);
  else
    local_opt_exact_kernel<NS, false, kRc><<<grid, kExactWaves * kWave, 0, st>>>(
        a.S, a.E, a.npairs, a.nchains, a.pairs, a.w01, a.anc, a.ow, a.xlo, a.xhi, a.d1w, a.nwords, a.plan, a.nh,
        a.maxrem, a.sig0, a.sig1, a.wnew, a.wdag, a.info, a.ca, a.lo_blocks, a.fin);
}

template <int NS>
void launch_lo_ns(const LoArgs& a, int form, bool rc, dim3 grid, hipStream_t st) {
  if (form == 5) {
    if constexpr (NS <= 2)
      local_opt_exact_dual_kernel<NS><<<grid, kExactWaves * kWave, 0, st>>>(
          a.S, a.E, a.npairs, a.nchains, a.pairs, a.w01, a.anc, a.xlo, a.xhi, a.plan, a.nh, a.maxrem, a.sig0, a.sig1,
          a.wnew, a.wdag, a.info, a.ca, a.lo_blocks, a.fin);
    return;
  }
  if (rc) launch_lo<NS, true>(a, form, grid, st);
  else launch_lo<NS, false>(a, form, grid, st);
}

}  // namespace

size_t exact_slot_doubles(const Ctx& c) {
  int res = 0;
  switch (c.pw_ns) {
    case 1: res = lo_resident_ns<1>(7, true); break;
    case 2: res = lo_resident_ns<2>(7, true); break;
    case 3: res = lo_resident_ns<3>(7, true); break;
    case 4: res = lo_resident_ns<4>(7, true); break;
    case 5: res = lo_resident_ns<5>(7, true); break;
    case 6: res = lo_resident_ns<6>(7, true); break;
    case 7: res = lo_resident_ns<7>(7, true); break;
    case 8: res = lo_resident_ns<8>(7, true); break;
    default: return 0;
  }
  return (size_t)std::max(res, 1) * kExactWaves * exact_plan_doubles(c);
}

hipError_t launch_local_opt_exact(Ctx& c, int nchains, int npairs, const int32_t* d_pairs, const double* d_w01,
                                  const double* d_anc, const double* d_ow, double sig0, double sig1, double* d_wnew,
                                  double* d_wdag, int32_t* d_info, const double* d_cs1, double* d_ll1,
                                  hipStream_t st) {
  const int nw = nchains * npairs;
  const bool rc = exact_rc(c);
  if (rc ? (size_t)nchains * c.S * exact_plan_doubles(c) > c.cap_xa
         : (size_t)nw * exact_plan_doubles(c) > c.cap_xcbuf)
    return hipErrorInvalidValue;
  // the latency form up to exact_lat_waves optima (~10 C3 chains), the slot
  // form (four waves per SIMD, c made once per optimum) beyond -- measured
  // crossover between 8 and 12 chains, profiles/r6/r6j_forms_ab.txt -- or the
  // throughput form where the slot form does not apply; the pair form for few
  // optima with two slots or more
  int form = c.exact_form;
  if (form == 0) form = nw <= c.exact_lat_waves ? 1 : 7;
  // (auto: the pair form up to 3 slots; from 4 its LDS and registers hold it
  // to 1-2 waves per SIMD)
  if (c.pw_ns >= 2 && (c.exact_form == 3 || (c.exact_form == 0 && nw <= c.exact_pair_waves && c.pw_ns <= 3)))
    form = 3;
  if (c.pw_ns < 2 && form == 3) form = 2;
  // two plan parts (E > 8192): the throughput form, whose objective reads
  // each part's plan from global memory and recomputes c per evaluation
  if (c.pw_parts > 1) form = 6;
  // the persistent form: at most the resident blocks, the work counter zeroed
  const bool persist = c.exact_persist && c.d_xqueue;
  // the slot form: one row set per resident wave, so persistent launches only
  if (form == 7 && !(rc && persist && c.pw_parts == 1 && c.d_xsbuf)) form = 2;
  // the dual form (two optima per wave) needs the register cache's recompute
  // rows, the work queue and at most two slots; else the latency form
  if (form == 5 && !(rc && persist && c.pw_ns <= 2)) form = 1;
  const int per_block = form == 3 ? 1 : form == 5 ? 2 * kExactWaves : kExactWaves;   // optima a block holds at once
  int lo_blocks = (nw + per_block - 1) / per_block;
  if (persist) {
    int res = 0;
    switch (c.pw_ns) {
      case 1: res = lo_resident_ns<1>(form, rc); break;
      case 2: res = lo_resident_ns<2>(form, rc); break;
      case 3: res = lo_resident_ns<3>(form, rc); break;
      case 4: res = lo_resident_ns<4>(form, rc); break;
      case 5: res = lo_resident_ns<5>(form, rc); break;
      case 6: res = lo_resident_ns<6>(form, rc); break;
      case 7: res = lo_resident_ns<7>(form, rc); break;
      case 8: res = lo_resident_ns<8>(form, rc); break;
      default: return hipErrorInvalidValue;
    }
    lo_blocks = std::min(lo_blocks, std::max(res, 1));
    if (form == 7 && (size_t)lo_blocks * kExactWaves * exact_plan_doubles(c) > c.cap_xsbuf) return hipErrorInvalidValue;
    const hipError_t me = hipMemsetAsync(c.d_xqueue, 0, sizeof(int), st);
    if (me != hipSuccess) return me;
  }
  const int per_fin = form == 3 ? 2 : kExactWaves;   // waves per appended block
  const int fin_blocks = d_ll1 ? (nchains + per_fin - 1) / per_fin : 0;
  LoArgs a{c.S,     c.E,      npairs,  nchains,  d_pairs,  d_w01,    d_anc,    d_ow,     c.d_xlo,
           c.d_xhi, c.d_D1w,  c.nwords, c.d_pwplan, c.pw_nh, c.pw_maxrem, sig0,  sig1,     d_wnew,
           d_wdag,  d_info,   CArgs{c.d_xa, c.d_xbits, c.d_xcbuf, c.exact_xcd,
                                    c.exact_trace && c.cap_xtrace >= (size_t)nw ? c.d_xtrace : nullptr,
                                    persist ? c.d_xqueue : nullptr, nullptr,
                                    c.exact_sched && c.d_xcost ? c.d_xcost : nullptr},
           lo_blocks, SeqSumArgs{d_cs1, c.E, nchains, d_ll1}};
  // only when the optima outnumber the resident waves (else all start at once)
  // and make at most 16 rounds of them: past that the last optimum's share of
  // the launch is small and the chains' interleaving costs more (C3, 128
  // chains: 11.99 against 11.84 ms per step, tools/step_probe.py)
  if (persist && c.exact_sched && c.d_xcost && c.d_xorder && c.cap_xorder >= (size_t)nw &&
      nw > lo_blocks * per_block && nw <= 16 * lo_blocks * per_block) {
    exact_sched_hist_kernel<<<nchains, kSchedThreads, 0, st>>>(c.S, npairs, d_pairs, c.d_xcost, c.d_xhist);
    hipError_t se = hipGetLastError();
    if (se != hipSuccess) return se;
    exact_sched_place_kernel<<<nchains, kSchedThreads, 0, st>>>(c.S, npairs, nchains, d_pairs, c.d_xcost, c.d_xhist,
                                                                c.d_xorder);
    se = hipGetLastError();
    if (se != hipSuccess) return se;
    a.ca.order = c.d_xorder;
  }
  const dim3 grid(lo_blocks + fin_blocks);
  hipEvent_t e0 = nullptr, e1 = nullptr;   // (option timing_kernel 1: bench.py's local-optimum roofline)
  if (c.timing && c.timing_kernel == 1 && c.ev_used + 2 <= c.ev_pool.size()) {
    e0 = c.ev_pool[c.ev_used++];
    e1 = c.ev_pool[c.ev_used++];
    const hipError_t re = hipEventRecord(e0, st);
    if (re != hipSuccess) return re;
  }
  if (form == 5) a.ca.trace = nullptr;   // (the dual form keeps no timeline)
  a.ca.nparts = c.pw_parts;
  a.ca.plan = c.d_pwplan;
  a.ca.pmeta = c.d_pwmeta;
  a.ca.pd = exact_plan_doubles(c);
  a.ca.sbuf = c.d_xsbuf;
  c.xtrace_n = a.ca.trace ? nw : 0;
  switch (c.pw_ns) {
    case 1: launch_lo_ns<1>(a, form, rc, grid, st); break;
    case 2: launch_lo_ns<2>(a, form, rc, grid, st); break;
    case 3: launch_lo_ns<3>(a, form, rc, grid, st); break;
    case 4: launch_lo_ns<4>(a, form, rc, grid, st); break;
    case 5: launch_lo_ns<5>(a, form, rc, grid, st); break;
    case 6: launch_lo_ns<6>(a, form, rc, grid, st); break;
    case 7: launch_lo_ns<7>(a, form, rc, grid, st); break;
    case 8: launch_lo_ns<8>(a, form, rc, grid, st); break;
    default: return hipErrorInvalidValue;
  }
  if (e1) {
    const hipError_t re = hipEventRecord(e1, st);
    if (re != hipSuccess) return re;
    ++c.launches;
  }
  return hipGetLastError();
}

#endif  // NEMO_EXACT_KERNELS_ONLY

}  // namespace nemo
