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

namespace nemo {

namespace {

using i32x4 = __attribute__((ext_vector_type(4))) int;

constexpr double kPadG8 = -1.0e6;    // G of padding rows: exp underflows to 0

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
// One kernel per batch: block = (evaluation b, a range of "sets"), where set
// s = the 8 consecutive 16-effect tiles [8s, 8s + 8).  The block first builds
// its evaluation's Delta digits and G in LDS (node order; wave = row i, lane
// = parent j):
//     lo = log(1 - w + w e^lo_j), Delta = log(1 - w + w e^hi_j) - lo
// (nem_order_mcmc.py:83-86 per factor), then every wave takes sets
// round-robin: per tile NP pairs of i8 MFMAs per row block, exact integer
// recombination, f64 cells, column log-sum-exp; one partial per set.
// Partials are indexed by set, so the bits of ll do not depend on how many
// blocks an evaluation is split into (split = f(batch), for occupancy).
// ---------------------------------------------------------------------------
template <int NR, int WAVES, int NP>
__global__ __launch_bounds__(WAVES * kWave, 2) void score_i8_kernel(
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
  double* Gs = (double*)(ltab + 128);                    // [SPAD]
  double* elo_s = Gs + SPAD;                             // [SPAD] e^lo_j
  double* ehi_s = elo_s + SPAD;                          // [SPAD] e^hi_j
  int* perm_s = (int*)(ehi_s + SPAD);                    // [SPAD] node at each position
  i32x4* A = (i32x4*)(perm_s + SPAD);                    // [NSL][SPAD][5] 16-byte chunks
  int8_t* A8 = (int8_t*)A;                               // (80-B rows: conflict-free b128)

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

  for (int k = tid; k < 256; k += blockDim.x) etab[k] = exp2((double)k * (1.0 / 256.0));
  fill_log_table(ltab, tid, blockDim.x);
  {
    const int32_t* pb = pos + (size_t)b * S;
    for (int j = tid; j < S; j += blockDim.x) {
      int pj = pb[j];
      pj = pj < 0 ? 0 : (pj >= S ? S - 1 : pj);  // malformed input must not fault
      perm_s[pj] = j;
    }
    for (int i = tid; i < SPAD; i += blockDim.x) {
      Gs[i] = i < S ? 0.0 : kPadG8;
      elo_s[i] = i < S ? e_lo[i] : 1.0;
      ehi_s[i] = i < S ? e_hi[i] : 1.0;
    }
    i32x4* a4 = A;
    for (int k = tid; k < NSL * SPAD * 5; k += blockDim.x) a4[k] = i32x4{0, 0, 0, 0};
  }
  __syncthreads();
  // ---- Delta digits and G of evaluation b.  Work runs in ORDER positions:
  // the child at position q has the parents at positions < q (within `cap`),
  // so pass q packs the children at positions q and S-1-q into one wave --
  // lane p < q: (q, p); lane p >= q: (S-1-q, p-q) -- every lane one
  // (child, parent) pair.  Digits land at [child node][parent node].
  {
    const bool packed = cap == 0 || cap >= S - 1;
    const int npass = packed ? (S + 1) / 2 : S;
    const int p = lane;
    // this wave's passes q = w, w + WAVES, ... (at most kMaxPass): the
    // (child, parent) pair of every lane and its weight are fetched first,
    // so the global loads of all passes are in flight together
    constexpr int kMaxPass = (SPAD / 2 + WAVES - 1) / WAVES + (SPAD % 2);
    constexpr int kMaxPassAll = (SPAD + WAVES - 1) / WAVES;
    int ii[kMaxPassAll], jj[kMaxPassAll];
    double sw[kMaxPassAll];
#pragma unroll
    for (int k = 0; k < kMaxPassAll; ++k) {
      const int q = w + k * WAVES;
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
      ii[k] = act ? perm_s[qr] : -1;
      jj[k] = act ? perm_s[pp] : 0;
      sw[k] = act ? w01[((size_t)b * S + ii[k]) * S + jj[k]] : 0.0;
    }
    (void)kMaxPass;
#pragma unroll
    for (int k = 0; k < kMaxPassAll; ++k) {
      const int q = w + k * WAVES;
      if (q >= npass) break;
      const bool act = ii[k] >= 0;
      double lo = 0.0;
      if (act) {
        const int i = ii[k], j = jj[k];
        lo = log_fast(fma(sw[k], elo_s[j] - 1.0, 1.0), ltab);
        const double d = log_fast(fma(sw[k], ehi_s[j] - 1.0, 1.0), ltab) - lo;
        // fixed point: x = Delta * 2^(6-c) in [-32, 32]; every step is exact
        double x = ldexp(d, 6 - cexp);
#pragma unroll
        for (int sl = 0; sl < NSL; ++sl) {
          const double qd = rint(x);
          A8[(sl * SPAD + i) * 80 + j] = (int8_t)(int)qd;
          x = (x - qd) * 64.0;
        }
      }
      // G of the one or two children of this pass (segmented wave sums)
      const double ga = wsum((act && p < q) || !packed ? lo : 0.0);
      if (packed) {
        const double gb = wsum(act && p >= q ? lo : 0.0);
        if (lane == 0 && S - 1 - q != q) Gs[perm_s[S - 1 - q]] = gb;
      }
      if (lane == 0) Gs[perm_s[q]] = ga;
    }
  }
  // U rows of this lane's cells: 16r + 4rg + g (i8 C layout).  The staged U
  // has >= SPAD rows (rows S+1.. are zero; their G is kPadG8), so a cell's
  // address is a uniform part ((16r + g) E) + one per-lane offset (4 rg E + col).
  const uint32_t uln = (uint32_t)(4 * rg * E + col);
  __syncthreads();

  const i32x4* Bt = (const i32x4*)B8;
  const uint32_t a_lane = (uint32_t)(col * 5 + rg);  // A chunk of this lane, row block 0, slice 0
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
    const i32x4* Al = A + ao;
    const i32x4 b1 = bc;
    const i32x4 b64 = b1 << 6;  // bytes 0/1 -> 0/64
    double cell[NR][4];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      i32x4 acc[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const i32x4 a0 = Al[((2 * p) * SPAD + 16 * r) * 5];
        const i32x4 a1 = Al[((2 * p + 1) * SPAD + 16 * r) * 5];
        acc[p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b64, i32x4{0, 0, 0, 0}, 0, 0, 0);
        acc[p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b1, acc[p], 0, 0, 0);
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
    const double unull = unc;
    // next (set, tile) of this wave
    int tn = t + 1, setn = set;
    if (tn >= min(ntiles, 8 * set + 8)) {
      setn = set + WAVES;
      tn = 8 * setn;
    }
    const bool more = setn < s_end;
    if (more) load_tile(tn);
    // column log-sum-exp over the SPAD rows and the null row
    const bool valid = t * 16 + col < E;
    double m = unull;
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g) m = vmax8(m, cell[r][g]);
    m = vmax8(m, __shfl_xor(m, 16, kWave));
    m = vmax8(m, __shfl_xor(m, 32, kWave));
    double l = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g) l += exp_lse8(cell[r][g] - m, etab);
    l += __shfl_xor(l, 16, kWave);
    l += __shfl_xor(l, 32, kWave);
    l += exp_lse8(unull - m, etab);
    // prod(l) kept as mantissa * 2^lexp: branch-free, no overflow
    msum += valid ? m : 0.0;
    lprod *= valid ? l : 1.0;
    lexp += __builtin_amdgcn_frexp_exp(lprod);
    lprod = __builtin_amdgcn_frexp_mant(lprod);
    if (setn != set) {  // set complete: one partial
      double v = msum + (log(lprod) + (double)lexp * 0.69314718055994530942);
      v = lane < 16 ? v : 0.0;
      v = wsum(v);
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
  // ---- one block per evaluation: it sums its own partials (same order as
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
  const size_t lds = 256 * 8 + 128 * 16 + 3 * SPAD * 8 + SPAD * 4 + (size_t)2 * NP * SPAD * 80;
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
#define NEMO_I8(NRV, WV, NPV) \
  if (nr == NRV && waves == WV && np == NPV) \
    return launch_i8_t<NRV, WV, NPV>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized);
  NEMO_I8(1, 4, 4) NEMO_I8(2, 4, 4) NEMO_I8(4, 4, 4)
  NEMO_I8(1, 4, 5) NEMO_I8(2, 4, 5) NEMO_I8(4, 4, 5)
  NEMO_I8(1, 8, 4) NEMO_I8(2, 8, 4) NEMO_I8(4, 8, 4)
#undef NEMO_I8
  return hipErrorInvalidValue;
}

}  // namespace nemo
