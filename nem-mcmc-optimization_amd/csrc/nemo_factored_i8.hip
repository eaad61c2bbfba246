// nemo_factored_i8.hip -- the factored order score with the contraction on
// the int8 matrix cores, exactly (S <= 64).
//
// The factored form (nemo_factored.hip) is
//     cell[i][e] = U[i][e] + G[i] + sum_j Delta[i][j] * D1[j][e],   D1 in {0, 1}.
// On gfx950 the f64 MFMA (64 cycles per 16x16x4) and the VALU do not overlap
// (tools/ubench/overlap.hip), so the fp64 contraction costs ~2560 SIMD cycles
// per 16-effect tile on top of the log-sum-exp epilogue.  Here Delta is
// written in fixed point against one per-model scale 2^c >= 2 max|hi - lo|
// (|Delta(i,j)| <= |hi_j - lo_j| for every weight):
//     Delta = 2^(c-6) * sum_{s<2NP} d_s * 64^-s,   d_s integers in [-32, 32],
// error <= 2^(c-6) 64^-(2NP-1) / 2 per entry (NP = 4: 2^(c-49), 2^-45 at c = 4).  Each pair of
// digit slices is one integer accumulation on v_mfma_i32_16x16x64_i8 (K = 64
// parents in one instruction): the first MFMA takes d_2t against B = 64*D1,
// the second d_2t+1 against B = D1 into the same accumulator, so
//     acc_t = sum_j (64 d_2t + d_2t+1)[i][j] * D1[j][e]      (exact, |acc_t| < 2^18)
// and two pairs combine exactly in int32: T = acc_2u * 2^12 + acc_2u+1.  The
// cell is then U + G + T_0 2^(c-24) + T_1 2^(c-48) [+ acc_4 2^(c-60)]: two
// (three) int->f64 conversions and fmas -- the f64 work left is the epilogue.
//
// Rows and parents are in NODE order (the order only decides which Delta are
// non-zero), so D1 is a per-model constant: its B fragments are expanded to
// bytes once at staging (nemo_abi.cpp) and each tile reads them with one
// 16-byte load per lane; the U rows need no permutation either.
#include "nemo_internal.h"

#include <math.h>

#ifndef NEMO_I8_ABLATE
#define NEMO_I8_ABLATE 0
#endif
// register budget: waves per SIMD the int8 score kernel is compiled for
#ifndef NEMO_I8_WAVES_PER_SIMD
#define NEMO_I8_WAVES_PER_SIMD 2
#endif

namespace nemo {

namespace {

using i32x4 = __attribute__((ext_vector_type(4))) int;

constexpr double kPadG8 = -1.0e6;    // G of padding rows: exp underflows to 0
// A rows in LDS: 6 chunks of 16 B (96 B).  tools/ubench/lds_pattern.hip: the
// lane pattern (row = lane & 15, chunk = lane >> 4) of ds_read_b128 costs 4
// conflict cycles per read at 64- or 80-B rows, 0 at 96 B.
constexpr int kARow = 6;

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// see exp_lse in nemo_factored.hip: 256-entry table, degree 4, one-constant
// reduction, exact-integer k from the 1.5*2^52 shift
__device__ __forceinline__ double exp_lse8(double x, const double* __restrict__ tab) {
  constexpr double kInvLn2x256 = 369.32993046757462707;
  constexpr double kLn2d256 = 2.7076061740622862e-03;
  constexpr double kMagic = 6755399441055744.0;
  const double t = fma(x, kInvLn2x256, kMagic);
  const double kf = t - kMagic;
  const int k = (int)(uint32_t)__builtin_bit_cast(uint64_t, t);
  const double r = fma(-kf, kLn2d256, x);
  double p = fma(r, 1.0 / 24.0, 1.0 / 6.0);
  p = fma(r, p, 0.5);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
  return ldexp(p * tab[k & 255], k >> 8);
}

__device__ __forceinline__ double vmax8(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ int xcd_index8(int L, int N, int remap) {
  if (!remap) return L;
  const int x = L & 7, k = L >> 3;
  const int q = N >> 3, r = N & 7;
  return x * q + (x < r ? x : r) + k;
}

// ---------------------------------------------------------------------------
// Shared pieces of the two int8 kernels.
//
// Per evaluation the LDS holds its Delta digits A[NSL][SPAD][kARow] (16-B
// chunks, 96-B rows), G[SPAD] and perm[SPAD] (node at each order position).
// ---------------------------------------------------------------------------
struct EvalLds {
  i32x4* A;
  double* G;
  int* perm;
};

// perm from pos, G preset (0 / kPadG8 on padding rows), digits zeroed
template <int SPAD, int NSL>
__device__ __forceinline__ void i8_init_eval(EvalLds e, const int32_t* __restrict__ pb, int S, int tid,
                                             int nthreads) {
  for (int j = tid; j < S; j += nthreads) {
    int pj = pb[j];
    pj = pj < 0 ? 0 : (pj >= S ? S - 1 : pj);  // malformed input must not fault
    e.perm[pj] = j;
  }
  for (int i = tid; i < SPAD; i += nthreads) e.G[i] = i < S ? 0.0 : kPadG8;
  for (int k = tid; k < NSL * SPAD * kARow; k += nthreads) e.A[k] = i32x4{0, 0, 0, 0};
}

// Delta digits and G of one evaluation, passes [k0, k0 + KB) of this wave
// (pass index k: q = w + k * WAVES).  Work runs in ORDER positions: the child
// at position q has the parents at positions < q (within `cap`), so a pass
// packs the children at positions q and S-1-q into one wave -- lane p < q:
// (q, p); lane p >= q: (S-1-q, p-q) -- every lane one (child, parent) pair:
//     lo = log(1 - w + w e^lo_j), Delta = log(1 - w + w e^hi_j) - lo
// (nem_order_mcmc.py:83-86 per factor).  The weights of the KB passes are
// fetched first and their G sums reduced together (independent butterflies).
template <int SPAD, int NSL, int WAVES, int KB>
__device__ __forceinline__ void i8_prep_passes(EvalLds e, int k0, int w, int lane, int S, int cap,
                                               int cexp, const double* __restrict__ w01b,
                                               const double* __restrict__ elo_s,
                                               const double* __restrict__ ehi_s,
                                               const double2* __restrict__ ltab) {
  const bool packed = cap == 0 || cap >= S - 1;
  const int npass = packed ? (S + 1) / 2 : S;
  const int p = lane;
  int8_t* A8 = (int8_t*)e.A;
  int ii[KB], jj[KB];
  double sw[KB], ga[KB], gb[KB];
#pragma unroll
  for (int kk = 0; kk < KB; ++kk) {
    const int q = w + (k0 + kk) * WAVES;
    int qr = 0, pp = 0;
    bool act = false;
    if (q < npass) {
      if (packed) {
        const int q2 = S - 1 - q;
        if (p < q) { qr = q; pp = p; act = true; }
        else { qr = q2; pp = p - q; act = q2 != q && pp < q2; }
      } else {
        const int np = q < cap ? q : cap;
        qr = q; pp = q - 1 - p; act = p < np;
      }
    }
    ii[kk] = act ? e.perm[qr] : -1;
    jj[kk] = act ? e.perm[pp] : 0;
    sw[kk] = act ? w01b[ii[kk] * S + jj[kk]] : 0.0;
  }
#pragma unroll
  for (int kk = 0; kk < KB; ++kk) {
    const int q = w + (k0 + kk) * WAVES;
    const bool act = ii[kk] >= 0;
    double lo = 0.0;
    if (act && !(NEMO_I8_ABLATE & 8)) {  // (8: instrumented build, no digits)
      const int i = ii[kk], j = jj[kk];
      lo = log_fast(fma(sw[kk], elo_s[j] - 1.0, 1.0), ltab);
      const double d = log_fast(fma(sw[kk], ehi_s[j] - 1.0, 1.0), ltab) - lo;
      // fixed point: x = Delta * 2^(6-c) in [-32, 32]; every step is exact
      double x = ldexp(d, 6 - cexp);
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl) {
        const double qd = rint(x);
        A8[(sl * SPAD + i) * (16 * kARow) + j] = (int8_t)(int)qd;
        x = (x - qd) * 64.0;
      }
    }
    ga[kk] = (act && p < q) || !packed ? lo : 0.0;
    gb[kk] = packed && act && p >= q ? lo : 0.0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      ga[kk] += __shfl_xor(ga[kk], o, kWave);
      gb[kk] += __shfl_xor(gb[kk], o, kWave);
    }
  if (lane == 0) {
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      const int q = w + (k0 + kk) * WAVES;
      if (q >= npass) continue;
      if (packed && S - 1 - q != q) e.G[e.perm[S - 1 - q]] = gb[kk];
      e.G[e.perm[q]] = ga[kk];
    }
  }
}

__device__ __forceinline__ int i8_npass(int S, int cap) {
  return (cap == 0 || cap >= S - 1) ? (S + 1) / 2 : S;
}

// One 16-effect tile, part 1: NP pairs of i8 MFMAs per row block and the
// exact integer recombination into f64 cells (U + G + T_0 2^(c-24) +
// T_1 2^(c-48)).  After this the U registers are free for the next tile.
template <int NR, int NP>
__device__ __forceinline__ void i8_cells(const i32x4* __restrict__ Al, const double* __restrict__ Gs,
                                         const i32x4 b1, const double (&uc)[NR][4], int rg, double sA,
                                         double sB, double sC, double (&cell)[NR][4]) {
  constexpr int SPAD = NR * 16;
  const i32x4 b64 = b1 << 6;  // bytes 0/1 -> 0/64
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    i32x4 acc[NP];
#pragma unroll
    for (int pr = 0; pr < NP; ++pr) {
      const i32x4 a0 = Al[((2 * pr) * SPAD + 16 * r) * kARow];
      const i32x4 a1 = Al[((2 * pr + 1) * SPAD + 16 * r) * kARow];
#if NEMO_I8_ABLATE & 2  // instrumented build (tools/ablate.sh): no MFMA
      acc[pr] = a0 + b64 + a1;
#else
      acc[pr] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b64, i32x4{0, 0, 0, 0}, 0, 0, 0);
      acc[pr] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b1, acc[pr], 0, 0, 0);
#endif
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ta = (acc[0][g] << 12) + acc[1][g];
      const int tb = (acc[2][g] << 12) + acc[3][g];
      double v = Gs[16 * r + 4 * rg + g];
      if constexpr (NP == 5) v = fma((double)acc[4][g], sC, v);
      v = fma((double)tb, sB, v);
      v = fma((double)ta, sA, v);
      cell[r][g] = v + uc[r][g];
    }
  }
}

// part 2: the column log-sum-exp over the SPAD rows and the null row, folded
// into (msum, lprod * 2^lexp).  Max and sum run as pairwise trees (depth
// log2(4 NR) instead of 4 NR: the tile is latency-bound at 2 waves/SIMD).
template <int NR>
__device__ __forceinline__ void i8_lse(double (&cell)[NR][4], double unull, bool valid,
                                       const double* __restrict__ etab, double& msum,
                                       double& lprod, int& lexp) {
  constexpr int NC = 4 * NR;
  double* c = &cell[0][0];
  double mx[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) mx[k] = c[k];
#pragma unroll
  for (int h = NC / 2; h >= 1; h /= 2)
#pragma unroll
    for (int k = 0; k < h; ++k) mx[k] = vmax8(mx[k], mx[k + h]);
  double m = vmax8(mx[0], unull);
  m = vmax8(m, __shfl_xor(m, 16, kWave));
  m = vmax8(m, __shfl_xor(m, 32, kWave));
  double ex[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
#if NEMO_I8_ABLATE & 1  // instrumented build (tools/ablate.sh): no exp
    ex[k] = c[k] - m;
#else
    ex[k] = exp_lse8(c[k] - m, etab);
#endif
  }
#pragma unroll
  for (int h = NC / 2; h >= 1; h /= 2)
#pragma unroll
    for (int k = 0; k < h; ++k) ex[k] += ex[k + h];
  double l = ex[0];
  l += __shfl_xor(l, 16, kWave);
  l += __shfl_xor(l, 32, kWave);
  l += exp_lse8(unull - m, etab);
  // prod(l) kept as mantissa * 2^lexp: branch-free, no overflow
  msum += valid ? m : 0.0;
  lprod *= valid ? l : 1.0;
  lexp += __builtin_amdgcn_frexp_exp(lprod);
  lprod = __builtin_amdgcn_frexp_mant(lprod);
}

__device__ __forceinline__ double i8_set_value(double msum, double lprod, int lexp, int lane) {
  double v = msum + (log(lprod) + (double)lexp * 0.69314718055994530942);
  v = lane < 16 ? v : 0.0;
  return wsum(v);
}

// block-wide tables: 2^(j/256) for exp_lse8, the log_fast table, e^lo / e^hi
__device__ __forceinline__ void i8_tables(double* etab, double2* ltab, double* elo_s, double* ehi_s,
                                          const double* __restrict__ e_lo, const double* __restrict__ e_hi,
                                          int S, int SPAD, int tid, int nthreads) {
  for (int k = tid; k < 256; k += nthreads) etab[k] = exp2((double)k * (1.0 / 256.0));
  fill_log_table(ltab, tid, nthreads);
  for (int i = tid; i < SPAD; i += nthreads) {
    elo_s[i] = i < S ? e_lo[i] : 1.0;
    ehi_s[i] = i < S ? e_hi[i] : 1.0;
  }
}

// ---------------------------------------------------------------------------
// block = (evaluation b, a range of "sets"; set s = the 8
// consecutive 16-effect tiles [8s, 8s + 8)).  The block first builds its
// evaluation's digits and G in LDS, then every wave takes sets round-robin,
// one partial per set.  Partials are indexed by set, so the bits of ll do not
// depend on how many blocks an evaluation is split into (split = f(batch),
// for occupancy).  (A persistent variant that overlapped the next
// evaluation's digit prep with the tiles, double-buffering A in LDS, ran
// 1.5x slower at one block per CU and was dropped.)
// ---------------------------------------------------------------------------
template <int NR, int WAVES, int NP>
__global__ __launch_bounds__(WAVES * kWave, NEMO_I8_WAVES_PER_SIMD) void score_i8_kernel(
    int S, int E, int ntiles, int nsets, int split, int cap, int cexp,
    const int32_t* __restrict__ pos, const double* __restrict__ w01,
    const double* __restrict__ e_lo, const double* __restrict__ e_hi,
    const uint8_t* __restrict__ B8, const double* __restrict__ U, double sA, double sB,
    double sC, double* __restrict__ partial, double* __restrict__ ll_out, int remap) {
  constexpr int SPAD = NR * 16;
  constexpr int NSL = 2 * NP;
  extern __shared__ __attribute__((aligned(16))) double lds8[];
  double* etab = lds8;                                   // [256] 2^(j/256)
  double2* ltab = (double2*)(etab + 256);                // [128] log table
  double* elo_s = (double*)(ltab + 128);                 // [SPAD] e^lo_j
  double* ehi_s = elo_s + SPAD;                          // [SPAD] e^hi_j
  EvalLds ev;
  ev.G = ehi_s + SPAD;                                   // [SPAD]
  ev.perm = (int*)(ev.G + SPAD);                         // [SPAD]
  ev.A = (i32x4*)(ev.perm + SPAD);                       // [NSL][SPAD][kARow]

  const int work = xcd_index8((int)blockIdx.x, (int)gridDim.x, remap);
  const int b = work / split;
  const int part = work - b * split;
  const int spb = (nsets + split - 1) / split;
  const int s_begin = part * spb;
  const int s_end = min(nsets, s_begin + spb);
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int col = lane & 15, rg = lane >> 4;

  i8_tables(etab, ltab, elo_s, ehi_s, e_lo, e_hi, S, SPAD, tid, blockDim.x);
  i8_init_eval<SPAD, NSL>(ev, pos + (size_t)b * S, S, tid, blockDim.x);
  __syncthreads();
  {
    constexpr int KB = 4;
    const int npass = i8_npass(S, cap);
    const int my = npass > w ? (npass - w + WAVES - 1) / WAVES : 0;
    for (int k0 = 0; k0 < my; k0 += KB)
      i8_prep_passes<SPAD, NSL, WAVES, KB>(ev, k0, w, lane, S, cap, cexp, w01 + (size_t)b * S * S,
                                           elo_s, ehi_s, ltab);
  }
  // U rows of this lane's cells: 16r + 4rg + g (i8 C layout).  The staged U
  // has >= SPAD rows (rows S+1.. are zero; their G is kPadG8), so a cell's
  // address is a uniform part ((16r + g) E) + one per-lane offset (4 rg E + col).
  const uint32_t uln = (uint32_t)(4 * rg * E + col);
  __syncthreads();

  const i32x4* Bt = (const i32x4*)B8;
  const uint32_t a_lane = (uint32_t)(col * kARow + rg);  // A chunk of this lane, row block 0, slice 0
  // one flat stream of (set, tile) per wave, so the next tile's U rows and
  // D1 bytes are always in flight -- across set boundaries too
  int set = s_begin + w;
  if (set < s_end) {
    double msum = 0.0, lprod = 1.0;
    int lexp = 0;
    double uc[NR][4], unc;
    i32x4 bc;
    auto load_tile = [&](int tt) {
      const double* base = U + (size_t)tt * 16;
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int g = 0; g < 4; ++g) uc[r][g] = (base + (size_t)(16 * r + g) * E)[uln];
      unc = (base + (size_t)S * E)[col];
      bc = Bt[(size_t)tt * kWave + lane];
    };
    int t = 8 * set;
    load_tile(t);
    for (;;) {
      // launder the A offset each tile: keeps the loop-invariant A fragments
      // (2NP * NR * 16 B per lane) in LDS instead of hoisted into registers
      uint32_t ao = a_lane;
      asm volatile("" : "+v"(ao));
      double cell[NR][4];
      i8_cells<NR, NP>(ev.A + ao, ev.G, bc, uc, rg, sA, sB, sC, cell);
      const double unull = unc;
      int tn = t + 1, setn = set;
      if (tn >= min(ntiles, 8 * set + 8)) {
        setn = set + WAVES;
        tn = 8 * setn;
      }
      const bool more = setn < s_end;
      if (more) load_tile(tn);  // into the registers the cells just freed
      i8_lse<NR>(cell, unull, t * 16 + col < E, etab, msum, lprod, lexp);
      if (setn != set) {  // set complete: one partial
        const double v = i8_set_value(msum, lprod, lexp, lane);
        if (lane == 0) partial[(size_t)b * nsets + set] = v;
        msum = 0.0;
        lprod = 1.0;
        lexp = 0;
      }
      if (!more) break;
      t = tn;
      set = setn;
    }
  }
  // one block per evaluation: it sums its own partials (same order as
  // finalize_factored_kernel, so the bits match the split > 1 path)
  if (split == 1) {
    __syncthreads();  // the block's partial stores are visible to the block
    if (w == 0) {
      const double v = sum_partials(partial + (size_t)b * nsets, nsets, lane);
      if (lane == 0) ll_out[b] = v;
    }
  }
}

template <int NR, int WAVES, int NP>
hipError_t launch_i8_t(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                       double* d_ll, hipStream_t st, int* nparts, bool* finalized) {
  constexpr int SPAD = NR * 16;
  const int ntiles = (c.E + 15) / 16;
  const int nsets = (ntiles + 7) / 8;
  // blocks per evaluation: fill 2 waves per SIMD on 256 CUs; each split
  // re-derives its evaluation's digits (cheap next to its tiles)
  const int slots = 256 * (8 / WAVES);
  int split = (slots + batch - 1) / batch;
  split = split < 1 ? 1 : (split > nsets ? nsets : split);
  const size_t lds = 256 * 8 + 128 * 16 + 4 * SPAD * 8 + SPAD * 4 + (size_t)2 * NP * SPAD * 16 * kARow;
  const double sA = ldexp(1.0, c.i8_cexp - 24), sB = ldexp(1.0, c.i8_cexp - 48),
               sC = ldexp(1.0, c.i8_cexp - 60);
  score_i8_kernel<NR, WAVES, NP><<<dim3(batch * split), WAVES * kWave, lds, st>>>(
      c.S, c.E, ntiles, nsets, split, cap, c.i8_cexp, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_B8,
      (const double*)c.d_U64, sA, sB, sC, c.d_fpartial, d_ll, c.xcd_remap);
  *nparts = nsets;
  *finalized = split == 1;
  return hipGetLastError();
}

}  // namespace

hipError_t launch_score_i8(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                           double* d_ll, int np, int waves, hipStream_t st, int* nparts,
                           bool* finalized) {
  const int nr = c.fspad / 16;
  if (c.fspad > 64 || !c.d_B8) return hipErrorInvalidValue;
#define NEMO_I8(NRV, WV, NPV)                \
  if (nr == NRV && waves == WV && np == NPV) \
    return launch_i8_t<NRV, WV, NPV>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized);
  NEMO_I8(1, 4, 4) NEMO_I8(2, 4, 4) NEMO_I8(4, 4, 4)
  NEMO_I8(1, 4, 5) NEMO_I8(2, 4, 5) NEMO_I8(4, 4, 5)
  NEMO_I8(1, 8, 4) NEMO_I8(2, 8, 4) NEMO_I8(4, 8, 4)
#undef NEMO_I8
  return hipErrorInvalidValue;
}

}  // namespace nemo
