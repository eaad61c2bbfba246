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

#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

#ifndef NEMO_I8_ABLATE
#define NEMO_I8_ABLATE 0
#endif
// score_i8l_kernel's two-tile walk: the remainder R through slice 4's C-init
// (1) or formed after the MFMAs (0; the round-2 form, same bits)
#ifndef NEMO_I8L_RINIT
#define NEMO_I8L_RINIT 1
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
// The offset kernel's A rows: 4 chunks (64 B) with chunk c of row i stored at
// chunk (c + 2 ((i >> 2) & 3)) & 3 -- every 16-lane group of the
// A-fragment ds_read_b128 (row = lane & 15, chunk = lane >> 4) then hits 16
// distinct 16-B bank quads, and A takes 2/3 of the 96-B rows' LDS.
template <int ROWC>
__device__ __forceinline__ int a_byte(int i, int j) {
  if constexpr (ROWC == 4) return i * 64 + (((j >> 4) + 2 * ((i >> 2) & 3)) & 3) * 16 + (j & 15);
  else return i * (16 * ROWC) + j;
}

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
template <int SPAD, int NSL, int ROWC = kARow>
__device__ __forceinline__ void i8_init_eval(EvalLds e, const int32_t* __restrict__ pb, int S, int tid,
                                             int nthreads, double padg = kPadG8) {
  for (int j = tid; j < S; j += nthreads) {
    int pj = pb[j];
    pj = pj < 0 ? 0 : (pj >= S ? S - 1 : pj);  // malformed input must not fault
    e.perm[pj] = j;
  }
  for (int i = tid; i < SPAD; i += nthreads) e.G[i] = i < S ? 0.0 : padg;
  for (int k = tid; k < NSL * SPAD * ROWC; k += nthreads) e.A[k] = i32x4{0, 0, 0, 0};
}

// Delta digits and G of one evaluation, passes [k0, k0 + KB) of this wave
// (pass index k: q = w + k * WAVES).  Work runs in ORDER positions: the child
// at position q has the parents at positions < q (within `cap`), so a pass
// packs the children at positions q and S-1-q into one wave -- lane p < q:
// (q, p); lane p >= q: (S-1-q, p-q) -- every lane one (child, parent) pair:
//     lo = log(1 - w + w e^lo_j), Delta = log(1 - w + w e^hi_j) - lo
// (nem_order_mcmc.py:83-86 per factor).  The weights of the KB passes are
// fetched first and their G sums reduced together (independent butterflies).
template <int SPAD, int NSL, int WAVES, int KB, int ROWC = kARow>
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
        A8[sl * SPAD * 16 * ROWC + a_byte<ROWC>(i, j)] = (int8_t)(int)qd;
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

// --- the offset kernel's prep: the same passes, cheaper arithmetic --------
// (dpp_d, rowsum4, wsum_dpp and rowsum16: nemo_internal.h)

// Delta digits of one pair in integers: x = Delta 2^(6-c) in (-32, 32),
// h = rint(x 2^18), l = rint((x 2^18 - h) 2^24) (both |.| <= 2^23, the first
// difference exact by fma), x = h 2^-18 + l 2^-42 + <= 2^-43; then four
// balanced base-64 digits of each: d_k = ((v + 32 (1 + 64 + 64^2)) >> 6k & 63)
// - 32 for k < 3 and the top one (v + ...) >> 18 (in [-32, 32]).  Slices 0-3
// hold h's digits (most significant first), 4-7 l's: the MFMA pairs then
// rebuild T_0 = h and T_1 = l exactly.
template <int SPAD, int ROWC>
__device__ __forceinline__ void i8o_digits(int8_t* A8, int i, int j, double d, int cexp) {
  const double x = ldexp(d, 6 - cexp);
  const double hd = rint(x * 262144.0);
  const int h = (int)hd;
  const int l = (int)rint(fma(x, 262144.0, -hd) * 16777216.0);
  const int off = a_byte<ROWC>(i, j);
  constexpr int kBias = 32 * (1 + 64 + 4096);
  const int hb = h + kBias, lb = l + kBias;
  constexpr int SL = SPAD * 16 * ROWC;  // bytes per slice
  A8[0 * SL + off] = (int8_t)(hb >> 18);
  A8[1 * SL + off] = (int8_t)(((hb >> 12) & 63) - 32);
  A8[2 * SL + off] = (int8_t)(((hb >> 6) & 63) - 32);
  A8[3 * SL + off] = (int8_t)((hb & 63) - 32);
  A8[4 * SL + off] = (int8_t)(lb >> 18);
  A8[5 * SL + off] = (int8_t)(((lb >> 12) & 63) - 32);
  A8[6 * SL + off] = (int8_t)(((lb >> 6) & 63) - 32);
  A8[7 * SL + off] = (int8_t)((lb & 63) - 32);
}

// The log2 fixed-point kernel (score_i8l_kernel) writes 7 slices of
// v = d 2^20 / ln 2: h = rint(v) as above (|h| < 2^25 - 2^17: top digit in
// [-128, 127]) in slices 0-3, and l = rint((v - h) 2^18) (|l| <= 2^17) as
// three balanced base-64 digits in slices 4-6, so T_0 counts units of 2^-20
// and T_1 units of 2^-38 of y = x / ln 2 (per-entry error <= 2^-39).
constexpr double kL2Scale = 1512775.3951951857;   // 2^20 / ln 2

template <int SPAD, int ROWC>
__device__ __forceinline__ void i8l_digits(int8_t* A8, int i, int j, double d) {
  const double hd = rint(d * kL2Scale);
  const int h = (int)hd;
  const int l = (int)rint(fma(d, kL2Scale, -hd) * 262144.0);
  const int off = a_byte<ROWC>(i, j);
  const int hb = h + 32 * (1 + 64 + 4096), lb = l + 32 * (1 + 64);
  constexpr int SL = SPAD * 16 * ROWC;  // bytes per slice
  A8[0 * SL + off] = (int8_t)(hb >> 18);
  A8[1 * SL + off] = (int8_t)(((hb >> 12) & 63) - 32);
  A8[2 * SL + off] = (int8_t)(((hb >> 6) & 63) - 32);
  A8[3 * SL + off] = (int8_t)((hb & 63) - 32);
  A8[4 * SL + off] = (int8_t)(lb >> 12);
  A8[5 * SL + off] = (int8_t)(((lb >> 6) & 63) - 32);
  A8[6 * SL + off] = (int8_t)((lb & 63) - 32);
}

// Pairwise lane swaps of a double (both dwords): dswap32 returns a's lanes
// 0-31 next to b's lanes 0-31 (out_b: a's and b's lanes 32-63), dswap16 the
// same per pair of 16-lane rows (v_permlane32_swap / v_permlane16_swap).
// i8o_prep_passes builds its 8 G sums from them as a reduce-scatter.
__device__ __forceinline__ double dswap32(double a, double b, double& out_b) {
  const uint64_t x = __builtin_bit_cast(uint64_t, a), y = __builtin_bit_cast(uint64_t, b);
  auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)x, (uint32_t)y, false, false);
  auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(x >> 32), (uint32_t)(y >> 32), false, false);
  out_b = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
  return __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
}
__device__ __forceinline__ double dswap16(double a, double b, double& out_b) {
  const uint64_t x = __builtin_bit_cast(uint64_t, a), y = __builtin_bit_cast(uint64_t, b);
  auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)x, (uint32_t)y, false, false);
  auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(x >> 32), (uint32_t)(y >> 32), false, false);
  out_b = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
  return __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
}

template <int SPAD, int WAVES, int KB, int ROWC, bool L2 = false>
__device__ __forceinline__ void i8o_prep_passes(EvalLds e, int k0, int w, int lane, int S, int cap,
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
      if constexpr (L2) i8l_digits<SPAD, ROWC>(A8, i, j, d);
      else i8o_digits<SPAD, ROWC>(A8, i, j, d, cexp);
    }
    ga[kk] = (act && p < q) || !packed ? lo : 0.0;
    gb[kk] = packed && act && p >= q ? lo : 0.0;
  }
  if constexpr (KB == 4) {
    // reduce-scatter of the 8 sums: after the permlane32 step lanes 0-31
    // hold pair sums of (ga[k], gb[k]) for k = 0, 1 and lanes 32-63 for
    // k = 2, 3; after the permlane16 step row r (16 lanes) holds those of
    // pass kk = (0, 2, 1, 3)[r] ... rows 0 / 1 / 2 / 3 -> kk 0 / 1 / 2 / 3
    // with the operand order below; DPP folds each row.
    double u0b, u1b, x0, x1, y0, y1;
    double u0 = dswap32(ga[0], ga[2], u0b);   // lanes 0-31: ga0 halves, 32-63: ga2 halves
    u0 += u0b;
    double u1 = dswap32(gb[0], gb[2], u1b);
    u1 += u1b;
    double v0b, v1b;
    double v0 = dswap32(ga[1], ga[3], v0b);
    v0 += v0b;
    double v1 = dswap32(gb[1], gb[3], v1b);
    v1 += v1b;
    // rows: u* hold kk 0 (rows 0, 1) / kk 2 (rows 2, 3); v* kk 1 / kk 3
    x0 = dswap16(u0, v0, y0);   // row 0, 2: u0 rows (0|2) + (1|3);  row 1, 3: v0 ...
    x0 += y0;
    x1 = dswap16(u1, v1, y1);
    x1 += y1;
    // row 0: kk 0, row 1: kk 1, row 2: kk 2, row 3: kk 3 -- a and b sums
    x0 += dpp_d<0xB1>(x0);
    x1 += dpp_d<0xB1>(x1);
    x0 += dpp_d<0x4E>(x0);
    x1 += dpp_d<0x4E>(x1);
    x0 += dpp_d<0x141>(x0);
    x1 += dpp_d<0x141>(x1);
    x0 += dpp_d<0x140>(x0);
    x1 += dpp_d<0x140>(x1);
    if ((lane & 15) == 0) {
      const int kk = lane >> 4;
      const int q = w + (k0 + kk) * WAVES;
      if (q < npass) {
        if (packed && S - 1 - q != q) e.G[e.perm[S - 1 - q]] = x1;
        e.G[e.perm[q]] = x0;
      }
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      ga[kk] = wsum_dpp(ga[kk]);
      gb[kk] = wsum_dpp(gb[kk]);
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
      (const double*)c.d_U64, sA, sB, sC, fpartial(c), d_ll, c.xcd_remap);
  *nparts = nsets;
  *finalized = split == 1;
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// score_i8o_kernel: the same contraction with an offset log-sum-exp.
//
// The column log-sum-exp needs SOME offset, not the maximum: with the null
// row as the offset,
//     cs[e] = U[S][e] + log(1 + sum_{i<S} exp(x[i][e])),
//     x[i][e] = cell[i][e] - U[S][e] = U'[i][e] + G[i] + (Delta.D1)[i][e],
// where U' = U - U[S] is staged once (stage_i8o).  Staging bounds |x| <= 690
// for every order and weight in [0, 1] (each log factor lies between 0 and
// T), so no exp overflows, the sum stays finite and no term is subnormal:
// the exponent of 2^(k/256) goes straight into the table entry's exponent
// field.  Against score_i8_kernel this drops the max pass and its two
// cross-lane steps, the "- m" per cell, the ldexp and the null row's exp, and
// each cell's exp is accumulated as soon as the cell exists, so no cell is
// held (fewer registers, more waves per SIMD).  G rides in the integer
// accumulators: G = g0 2^(c-24) + g1 2^(c-48) (+ <= 2^(c-49)), g0 / g1 the C
// init of the pair-1 / pair-3 accumulators, so a cell is two cvt + two fma.
// The column sum over the four row groups uses the gfx950 permlane swaps
// (VALU, no LDS round trip).  Sums per set: sum_e U[S][e] is a staged
// constant per 8-tile set (fixed order), the logs run once per set on
// prod(l) kept as mantissa * 2^lexp.
// ---------------------------------------------------------------------------
#ifndef NEMO_I8O_WAVES_PER_SIMD
#define NEMO_I8O_WAVES_PER_SIMD 4
#endif
#ifndef NEMO_I8L2_OCC  // waves per SIMD the two-tile log2 kernel is compiled for
#define NEMO_I8L2_OCC 4
#endif

// acc + e^x for |x| <= 700: 2^(k/2048) e^r, k = rint(x 2048/ln2), |r| <=
// ln2/4096, degree-3 series (error r^4/24 < 4e-17).  The rounding constant is
// 1.5 2^52 + kBias, kBias = 1023 * 2048, so the low dword of t is k + kBias
// (> 0 for x > -709): its low 11 bits are the table index j = k & 2047 and
// (lo << 9) = ((k >> 11) + 1023) << 20 + (j << 9).  The table entry's high
// dword is stored as hi(2^(j/2048)) with its exponent field cleared, XOR
// (j << 9), so one shift-xor makes the exponent field 1023 + (k >> 11) (no
// ldexp; |x| <= 700 keeps it normal).  Table: kExpTabN entries, 16 KB.
constexpr int kExpTabN = 2048;
constexpr double kExpMagicB = 6755399441055744.0 + 1023.0 * 2048.0;

__device__ __forceinline__ double exp_acc(double x, const uint2* __restrict__ tab, double acc) {
  constexpr double kInvLn2x2048 = 2954.6394437405970166;
  constexpr double kLn2d2048 = 3.3845077175778578e-04;
  const double t = fma(x, kInvLn2x2048, kExpMagicB);
  const double kf = t - kExpMagicB;
  const uint32_t lo = (uint32_t)__builtin_bit_cast(uint64_t, t);
  const double r = fma(-kf, kLn2d2048, x);
  double p = fma(r, 1.0 / 6.0, 0.5);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
#if NEMO_I8_ABLATE & 64  // instrumented build: every lane reads entry 0 (no bank conflicts)
  const uint2 e = tab[lo & 0u];
#else
  const uint2 e = tab[lo & (kExpTabN - 1)];
#endif
  const uint32_t hi = (lo << 9) ^ e.y;
  return fma(p, __builtin_bit_cast(double, ((uint64_t)hi << 32) | e.x), acc);
}

// acc + 2^y for score_i8l_kernel, y = (T_0 2^-20 + T_1 2^-38) - 1023: T_0
// carries the exponent bias (G's C-init), so bits 20..30 of T_0 are the
// biased exponent 1023 + floor(y) and bits 9..19 the index j of 2^(j/2048).
// The table's high dword is stored with its exponent field cleared, XOR
// (j << 9) (exp_acc's table), so (T_0 & ~511) ^ e.y is the high dword of
// 2^(floor(y) + j/2048): no range reduction in f64.  The remainder
// R = (T_0 & 511) 2^18 + T_1 (units of 2^-38, |R| < 2^28: one shift-add and
// one conversion, exact) gives f = R 2^-38 ln 2 in (-2.2e-5, 3.6e-4), where
// a degree-2 polynomial in R interpolating e^f at the three Chebyshev nodes
// of that interval is within 2.9e-13 (relative, alternating sign) -- below
// the fixed-point truncation of the cell (~2^-38 per entry).  Per cell: ~8
// integer + 1 cvt + 3 f64 VALU and one LDS read, against 4 + 2 + 9 for
// exp_acc on an f64 cell.  Coefficients: Newton form through the nodes in
// 50-digit decimal arithmetic, rounded to double.
constexpr double kL2C0 = 1.0000000000000377;
constexpr double kL2C1 = 2.521654728528023e-12;
constexpr double kL2C2 = 3.179908378901339e-24;

// split in three so a caller can keep several table reads in flight
__device__ __forceinline__ uint64_t exp2_fx_load(uint32_t t0) {
#if NEMO_I8_ABLATE & 64  // instrumented build: every lane reads entry 0 (no bank conflicts)
  const uint32_t addr = 0u;
#else
  const uint32_t addr = (t0 >> 6) & 0x3ff8u;
#endif
  // the table sits at LDS address 0 (the kernel's dynamic LDS starts there:
  // it has no static LDS); an LDS-space pointer from the integer address
  // avoids the base add of a generic pointer
  return *(const __attribute__((address_space(3))) uint64_t*)(size_t)addr;
}
__device__ __forceinline__ double exp2_fx_series(uint32_t t0, int t1) {
  // R = (T_0 & 511) 2^18 + T_1 as one v_lshl_add_u32 after the mask (the
  // compiler's own form is two shifts, an AND and an add3)
  uint32_t rr;
  asm("v_lshl_add_u32 %0, %1, 18, %2" : "=v"(rr) : "v"(t0 & 511u), "v"((uint32_t)t1));
  const double r = (double)(int)rr;
  return fma(r, fma(r, kL2C2, kL2C1), kL2C0);
}
// the same series from R itself (score_i8l_kernel's two-tile walk forms R
// through slice 4's C-init)
__device__ __forceinline__ double exp2_fx_series_r(int rr) {
  const double r = (double)rr;
  return fma(r, fma(r, kL2C2, kL2C1), kL2C0);
}
__device__ __forceinline__ double exp2_fx_apply(uint32_t t0, uint64_t ev, double p, double acc) {
  // (one v_bitop3: bits 9-19 of T_0 cancel the index the entry carries)
  const uint32_t hi = (t0 & ~511u) ^ (uint32_t)(ev >> 32);
  return fma(__builtin_bit_cast(double, ((uint64_t)hi << 32) | (uint32_t)ev), p, acc);
}

template <int NR, int WAVES, bool DIAG>
__global__ __launch_bounds__(WAVES * kWave, NEMO_I8O_WAVES_PER_SIMD) void score_i8o_kernel(
    int S, int E, int ntiles, int nsets, int split, int cap, int cexp, double padg,
    const int32_t* __restrict__ pos, const double* __restrict__ w01,
    const double* __restrict__ e_lo, const double* __restrict__ e_hi,
    const uint8_t* __restrict__ B8, const double* __restrict__ Uoff,
    const int8_t* __restrict__ udig, const double* __restrict__ u0,
    const double* __restrict__ nullsum, const void* __restrict__ tabs, double sA, double sB,
    double* __restrict__ partial, double* __restrict__ ll_out, int remap) {
  constexpr int SPAD = NR * 16;
  constexpr int NP = 4;
  constexpr int NSL = 2 * NP;
  extern __shared__ __attribute__((aligned(16))) double lds8[];
  uint2* etab_o = (uint2*)lds8;                          // [kExpTabN] exp_acc's table
  double2* ltab = (double2*)(etab_o + kExpTabN);         // [128] log table
  double* elo_s = (double*)(ltab + 128);                 // [SPAD] e^lo_j
  double* ehi_s = elo_s + SPAD;                          // [SPAD] e^hi_j
  EvalLds ev;
  ev.G = ehi_s + SPAD;                                   // [SPAD]
  int* gi = (int*)(ev.G + SPAD);                         // [2][SPAD] g0, g1
  ev.perm = gi + 2 * SPAD;                               // [SPAD]
  ev.A = (i32x4*)(ev.perm + SPAD);                       // [NSL][SPAD][4] swizzled (a_byte)

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

  {  // both tables (precomputed per context) in one contiguous 18 KB copy
    const int4* src = (const int4*)tabs;
    int4* dst = (int4*)lds8;
    for (int k = tid; k < (kExpTabN * 8 + 128 * 16) / 16; k += blockDim.x) dst[k] = src[k];
    for (int i = tid; i < SPAD; i += blockDim.x) {
      elo_s[i] = i < S ? e_lo[i] : 1.0;
      ehi_s[i] = i < S ? e_hi[i] : 1.0;
    }
  }
  i8_init_eval<SPAD, NSL, 4>(ev, pos + (size_t)b * S, S, tid, blockDim.x, padg);
  __syncthreads();
  if constexpr (DIAG) {  // U' as the free diagonal "parent" i of child i (stage_i8o)
    int8_t* A8 = (int8_t*)ev.A;
    for (int k = tid; k < S * NSL; k += blockDim.x) {
      const int i = k / NSL, sl = k - i * NSL;
      A8[sl * SPAD * 64 + a_byte<4>(i, i)] = udig[k];
    }
  }
  {
    constexpr int KB = 4;
    const int npass = i8_npass(S, cap);
    const int my = npass > w ? (npass - w + WAVES - 1) / WAVES : 0;
    for (int k0 = 0; k0 < my; k0 += KB)
      i8o_prep_passes<SPAD, WAVES, KB, 4>(ev, k0, w, lane, S, cap, cexp, w01 + (size_t)b * S * S,
                                          elo_s, ehi_s, ltab);
  }
  __syncthreads();
  // G in fixed point: g0 = rint(G 2^(24-c)), g1 = rint((G - g0 2^(c-24)) 2^(48-c))
  for (int i = tid; i < SPAD; i += blockDim.x) {
    const double g = DIAG && i < S ? ev.G[i] + u0[i] : ev.G[i];
    const double g0 = rint(ldexp(g, 24 - cexp));
    const double rho = fma(-g0, ldexp(1.0, cexp - 24), g);  // exact
    gi[i] = (int)g0;
    gi[SPAD + i] = (int)rint(ldexp(rho, 48 - cexp));
  }
  const uint32_t uln8 = (uint32_t)(4 * rg * E + col) * 8u;  // byte offset of this lane's U' cells
  __syncthreads();
#if NEMO_I8_ABLATE & 32  // instrumented build (tools/ablate.sh): prep only, no tiles
  if (s_end > 0) return;
#endif

  const i32x4* Bt = (const i32x4*)B8;
  const i32x4* Gi = (const i32x4*)gi;
  const uint32_t a_lane = (uint32_t)(col * 4 + ((rg + 2 * (col >> 2)) & 3));  // swizzled chunk
  int set = s_begin + w;
  if (set < s_end) {
    double lprod = 1.0;
    int lexp = 0;
    double uc[NR][4];
    int t = 8 * set;
    // U' through a buffer resource: the lane offset stays in one VGPR, the
    // tile and row offsets are scalar (no per-load address arithmetic)
    const __amdgpu_buffer_rsrc_t urs =
        __builtin_amdgcn_make_buffer_rsrc((void*)Uoff, (short)0, (int)((SPAD + 1) * E + 16) * 8, 0x00020000);
    auto uload = [&](int tt, int row) {
      return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                            urs, uln8, (tt * 16 + row * E) * 8, 0));
    };
    if constexpr (!DIAG)
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int g = 0; g < 4; ++g) uc[r][g] = uload(t, 16 * r + g);
    i32x4 bc = Bt[(size_t)t * kWave + lane];
    for (;;) {
      uint32_t ao = a_lane;
      asm volatile("" : "+v"(ao));
      const i32x4* Al = ev.A + ao;
      int tn = t + 1, setn = set;
      if (tn >= min(ntiles, 8 * set + 8)) {
        setn = set + WAVES;
        tn = 8 * setn;
      }
      const bool more = setn < s_end;
      const int tl = more ? tn : t;  // prefetch target (the current tile again at the end)
      const i32x4 b1 = bc;
      const i32x4 b64 = b1 << 6;
      bc = Bt[(size_t)tl * kWave + lane];
      double ls0 = 0.0, ls1 = 0.0;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        i32x4 acc[NP];
        const i32x4 c0 = Gi[(16 * r) / 4 + rg];
        const i32x4 c1 = Gi[(SPAD + 16 * r) / 4 + rg];
#pragma unroll
        for (int pr = 0; pr < NP; ++pr) {
          const i32x4 a0 = Al[((2 * pr) * SPAD + 16 * r) * 4];
          const i32x4 a1 = Al[((2 * pr + 1) * SPAD + 16 * r) * 4];
          const i32x4 ci = pr == 1 ? c0 : (pr == 3 ? c1 : i32x4{0, 0, 0, 0});
          acc[pr] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b64, ci, 0, 0, 0);
          acc[pr] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b1, acc[pr], 0, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ta = (acc[0][g] << 12) + acc[1][g];
          const int tb = (acc[2][g] << 12) + acc[3][g];
          double x;
          if constexpr (DIAG) {
            x = fma((double)ta, sA, (double)tb * sB);
          } else {
            x = fma((double)ta, sA, fma((double)tb, sB, uc[r][g]));
            uc[r][g] = uload(tl, 16 * r + g);
          }
#if NEMO_I8_ABLATE & 1  // instrumented build: no exp
          if (g & 1) ls1 += x;
          else ls0 += x;
#else
          if (g & 1) ls1 = exp_acc(x, etab_o, ls1);
          else ls0 = exp_acc(x, etab_o, ls0);
#endif
        }
      }
      double l = rowsum4(ls0 + ls1) + 1.0;  // + e^0 of the null row
      lprod *= t * 16 + col < E ? l : 1.0;
      lexp += __builtin_amdgcn_frexp_exp(lprod);
      lprod = __builtin_amdgcn_frexp_mant(lprod);
      if (setn != set) {  // set complete: one partial
        double v = log(lprod) + (double)lexp * 0.69314718055994530942;
        v = wsum(lane < 16 ? v : 0.0);
        if (lane == 0) partial[(size_t)b * nsets + set] = nullsum[set] + v;
        lprod = 1.0;
        lexp = 0;
      }
      if (!more) break;
      t = tn;
      set = setn;
    }
  }
  if (split == 1) {
    __syncthreads();
    if (w == 0) {
      const double v = sum_partials(partial + (size_t)b * nsets, nsets, lane);
      if (lane == 0) ll_out[b] = v;
    }
  }
}

template <int NR, int WAVES, bool DIAG>
hipError_t launch_i8o_t(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                        double* d_ll, hipStream_t st, int* nparts, bool* finalized) {
  constexpr int SPAD = NR * 16;
  const int ntiles = (c.E + 15) / 16;
  const int nsets = (ntiles + 7) / 8;
  const int slots = 256 * (NEMO_I8O_WAVES_PER_SIMD * 4 / WAVES);
  int split = (slots + batch - 1) / batch;
  split = split < 1 ? 1 : (split > nsets ? nsets : split);
  const size_t lds = kExpTabN * 8 + 128 * 16 + 3 * SPAD * 8 + 3 * SPAD * 4 + (size_t)8 * SPAD * 64;
  const double sA = ldexp(1.0, c.i8_cexp - 24), sB = ldexp(1.0, c.i8_cexp - 48);
  score_i8o_kernel<NR, WAVES, DIAG><<<dim3(batch * split), WAVES * kWave, lds, st>>>(
      c.S, c.E, ntiles, nsets, split, cap, c.i8_cexp, c.i8o_padg, d_pos, d_w01, c.d_elo, c.d_ehi,
      c.d_B8, c.d_Uoff, c.d_udig, c.d_u0, c.d_nullsum, c.d_i8o_tabs, sA, sB, fpartial(c), d_ll,
      c.xcd_remap);
  *nparts = nsets;
  *finalized = split == 1;
  return hipGetLastError();
}

// The two-tile walk of score_i8l_kernel over sets [set, s_end) step WAVES of
// one evaluation (A fragments Al, G C-inits Gi, partials of evaluation b).
// hook(it) runs between iterations it and it + 1 (it = 0, 1, ...) and returns
// nothing the walk reads: score_i8p_kernel runs the next evaluation's digit
// prep there.  Returns the number of iterations walked.
template <int NR, int WAVES, class Hook>
__device__ __forceinline__ int i8l_walk2(const i32x4* __restrict__ Al0, const i32x4* __restrict__ Gi,
                                        const i32x4* __restrict__ Bt, const i32x4* __restrict__ Bt64,
                                        int set, int s_end, int ntiles, int E, int col, int lane,
                                        uint32_t a_lane, const double* __restrict__ nullsum,
                                        double* __restrict__ partial, size_t b, int nsets,
                                        const double2* __restrict__ ltab, Hook hook) {
  constexpr int SPAD = NR * 16;
  const int rg = lane >> 4;
  int it = 0;
  if (set < s_end) {
    double lprod = 1.0;
    int lexp = 0;
    int t = 8 * set;
    auto tend = [&](int st) { return min(ntiles, 8 * st + 8); };
    int t2 = t + 1 < tend(set) ? t + 1 : t;
    // the B fragments through a buffer resource: the lane's byte offset stays
    // in one VGPR and the tile offset is scalar, so a prefetch is one
    // buffer_load with no per-load address arithmetic (Bt64 follows Bt)
    const __amdgpu_buffer_rsrc_t brs =
        __builtin_amdgcn_make_buffer_rsrc((void*)Bt, (short)0, 2 * ntiles * kWave * 16, 0x00020000);
    const uint32_t bln = (uint32_t)lane * 16u;
    auto bload = [&](int tile, int x64) {
      return __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           brs, bln, (x64 * ntiles + tile) * kWave * 16, 0));
    };
    i32x4 bca = bload(t, 0), bca64 = bload(t, 1);
    i32x4 bcb = bload(t2, 0), bcb64 = bload(t2, 1);
    for (;;) {
      uint32_t ao = a_lane;
      asm volatile("" : "+v"(ao));
      const i32x4* Al = Al0 + ao;
      const bool two = t2 != t;
      int tn = t + 2, setn = set;
      if (tn >= tend(set)) {
        setn = set + WAVES;
        tn = 8 * setn;
      }
      const bool more = setn < s_end;
      const int tla = __builtin_amdgcn_readfirstlane(more ? tn : t);
      const int tlb = __builtin_amdgcn_readfirstlane(more ? (tn + 1 < tend(setn) ? tn + 1 : tn) : t);
      const i32x4 b1a = bca, b64a = bca64, b1b = bcb, b64b = bcb64;
      bca = bload(tla, 0);
      bca64 = bload(tla, 1);
      bcb = bload(tlb, 0);
      bcb64 = bload(tlb, 1);
      double la0 = 0.0, la1 = 0.0, lb0 = 0.0, lb1 = 0.0;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const i32x4 c0 = Gi[(16 * r) / 4 + rg];
        const i32x4 c1 = Gi[(SPAD + 16 * r) / 4 + rg];
        auto A = [&](int sl) { return Al[(sl * SPAD + 16 * r) * 4]; };
        // slice by slice for both tiles: each A fragment dies after its two MFMAs
        i32x4 h0a, h0b, h1a, h1b, l0a, l0b, l1a, l1b;
        {
          const i32x4 a = A(0);
          h0a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64a, i32x4{0, 0, 0, 0}, 0, 0, 0);
          h0b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64b, i32x4{0, 0, 0, 0}, 0, 0, 0);
        }
        {
          const i32x4 a = A(1);
          h0a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a, h0a, 0, 0, 0);
          h0b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b, h0b, 0, 0, 0);
        }
        {
          const i32x4 a = A(2);
          h1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64a, c0, 0, 0, 0);
          h1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64b, c0, 0, 0, 0);
        }
        {
          const i32x4 a = A(3);
          h1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a, h1a, 0, 0, 0);
          h1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b, h1b, 0, 0, 0);
        }
#if NEMO_I8L_RINIT
        // slices 5-6 first; then T_0 of both tiles and their table reads, and
        // the remainder's upper part (T_0 & 511) 2^6 becomes the C-init of
        // slice 4, so R = l0 2^12 + l1 is one shift-add (the same integer R
        // as exp2_fx_series forms, so the same bits; one VOP3 less per cell)
        {
          const i32x4 a = A(5);
          l1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64a, c1, 0, 0, 0);
          l1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64b, c1, 0, 0, 0);
        }
        {
          const i32x4 a = A(6);
          l1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a, l1a, 0, 0, 0);
          l1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b, l1b, 0, 0, 0);
        }
        uint32_t t0a[4], t0b[4];
        uint64_t eva[4], evb[4];
        i32x4 ma, mb;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          t0a[g] = ((uint32_t)h0a[g] << 12) + (uint32_t)h1a[g];
          eva[g] = exp2_fx_load(t0a[g]);
          ma[g] = (int)((t0a[g] & 511u) << 6);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          t0b[g] = ((uint32_t)h0b[g] << 12) + (uint32_t)h1b[g];
          evb[g] = exp2_fx_load(t0b[g]);
          mb[g] = (int)((t0b[g] & 511u) << 6);
        }
        {
          const i32x4 a = A(4);
          l0a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a, ma, 0, 0, 0);
          l0b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b, mb, 0, 0, 0);
        }
        auto epi = [&](const uint32_t (&t0)[4], const uint64_t (&evv)[4], const i32x4 l0, const i32x4 l1,
                       double& ls0, double& ls1) {
          double pr[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) pr[g] = exp2_fx_series_r((int)(((uint32_t)l0[g] << 12) + (uint32_t)l1[g]));
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if (g & 1) ls1 = exp2_fx_apply(t0[g], evv[g], pr[g], ls1);
            else ls0 = exp2_fx_apply(t0[g], evv[g], pr[g], ls0);
          }
        };
        epi(t0a, eva, l0a, l1a, la0, la1);
        epi(t0b, evb, l0b, l1b, lb0, lb1);
#else
        {
          const i32x4 a = A(4);
          l0a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a, i32x4{0, 0, 0, 0}, 0, 0, 0);
          l0b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b, i32x4{0, 0, 0, 0}, 0, 0, 0);
        }
        {
          const i32x4 a = A(5);
          l1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64a, c1, 0, 0, 0);
          l1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64b, c1, 0, 0, 0);
        }
        {
          const i32x4 a = A(6);
          l1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a, l1a, 0, 0, 0);
          l1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b, l1b, 0, 0, 0);
        }
        auto epi = [&](const i32x4 h0, const i32x4 h1, const i32x4 l0, const i32x4 l1, double& ls0,
                       double& ls1) {
          uint32_t t0[4];
          uint64_t evv[4];
          double pr[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            t0[g] = ((uint32_t)h0[g] << 12) + (uint32_t)h1[g];
            evv[g] = exp2_fx_load(t0[g]);
          }
#pragma unroll
          for (int g = 0; g < 4; ++g)
            pr[g] = exp2_fx_series(t0[g], (int)(((uint32_t)l0[g] << 12) + (uint32_t)l1[g]));
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if (g & 1) ls1 = exp2_fx_apply(t0[g], evv[g], pr[g], ls1);
            else ls0 = exp2_fx_apply(t0[g], evv[g], pr[g], ls0);
          }
        };
        epi(h0a, h1a, l0a, l1a, la0, la1);
        epi(h0b, h1b, l0b, l1b, lb0, lb1);
#endif
      }
      // both tiles' column sums in one pass (rowsum_pair): rows 0 / 2 of the
      // wave then hold tile a's, rows 1 / 3 tile b's, and each lane keeps the
      // product of its own tile's columns
      const double l = rowsum_pair(la0 + la1, lb0 + lb1) + 1.0;  // + e^0 of the null row
      const bool tb = (lane & 16) != 0;
      const bool ok = (((tb ? t2 : t) * 16 + col) < E) & (two | !tb);  // branch-free (bitwise)
      lprod *= ok ? l : 1.0;
      lexp += __builtin_amdgcn_frexp_exp(lprod);
      lprod = __builtin_amdgcn_frexp_mant(lprod);
      if (setn != set) {  // set complete: one partial
        // row 0 holds the 16 column products of the set's a tiles, row 1 those
        // of its b tiles: log_fast (lprod is a mantissa in [0.5, 1)), a DPP sum
        // within each row, then row 0's sum + row 1's
        double v = log_fast(lprod, ltab) + (double)lexp * 0.69314718055994530942;
        v = rowsum16(v);
        v += __shfl_down(v, 16, kWave);
        if (lane == 0) partial[(size_t)b * nsets + set] = nullsum[set] + v;
        lprod = 1.0;
        lexp = 0;
      }
      hook(it++);
      if (!more) break;
      t = tn;
      t2 = tlb;
      set = setn;
    }
  }
  return it;
}

// ---------------------------------------------------------------------------
// score_i8l_kernel: score_i8o_kernel's contraction and offset log-sum-exp
// with every table quantity in units of 1 / ln 2 (digits of Delta / ln 2,
// U' / ln 2 on the diagonal, G / ln 2), so the contraction yields
// y = x / ln 2 in fixed point and 2^y = e^x is assembled from the integer
// accumulators (exp2_fx_acc).  T_0 = acc_0 2^12 + acc_1 (slices 0-3, units
// 2^-20, G's high part and the exponent bias 1023 << 20 in acc_1's C-init);
// T_1 = acc_2 2^12 + acc_3 (slice 4; slices 5-6 with G's low part as C-init,
// units 2^-38): 7 MFMAs per row block against 8.  Requires the diagonal form
// (stage_i8o).
// ---------------------------------------------------------------------------
// MODE (fact_kernel 20, an experiment): 0 = prep and walk in one block (the
// default); 1 = prep only, the evaluation's LDS image (G split, perm, digits)
// copied out to img; 2 = walk only, the image copied in from img
template <int NR, int WAVES, int OCC, int TT = 1, int MODE = 0>
__global__ __launch_bounds__(WAVES * kWave, OCC) void score_i8l_kernel(
    int S, int E, int ntiles, int nsets, int split, int cap, double padg,
    const int32_t* __restrict__ pos, const double* __restrict__ w01,
    const double* __restrict__ e_lo, const double* __restrict__ e_hi,
    const uint8_t* __restrict__ B8, const int8_t* __restrict__ udig, const double* __restrict__ u0,
    const double* __restrict__ nullsum, const void* __restrict__ tabs,
    double* __restrict__ partial, double* __restrict__ ll_out, int remap,
    int4* __restrict__ img = nullptr) {
  constexpr int SPAD = NR * 16;
  constexpr int NSL = 7;
  extern __shared__ __attribute__((aligned(16))) double lds8[];
  uint2* etab_o = (uint2*)lds8;                          // [kExpTabN] at LDS address 0
  double2* ltab = (double2*)(etab_o + kExpTabN);         // [128] log table
  double* elo_s = (double*)(ltab + 128);                 // [SPAD] e^lo_j
  double* ehi_s = elo_s + SPAD;                          // [SPAD] e^hi_j
  EvalLds ev;
  ev.G = ehi_s + SPAD;                                   // [SPAD]
  int* gi = (int*)(ev.G + SPAD);                         // [2][SPAD] g0, g1
  ev.perm = gi + 2 * SPAD;                               // [SPAD]
  ev.A = (i32x4*)(ev.perm + SPAD);                       // [NSL][SPAD][4] swizzled (a_byte)

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

  constexpr int kImg4 = SPAD * 460 / 16;  // the image in int4: gi, perm, digits (i8img_bytes)
  {  // both tables (precomputed per context) in one contiguous 18 KB copy
    // (the prep-only launch needs the log table alone)
    const int4* src = (const int4*)tabs;
    int4* dst = (int4*)lds8;
    for (int k = tid + (MODE == 1 ? kExpTabN * 8 / 16 : 0); k < (kExpTabN * 8 + 128 * 16) / 16;
         k += blockDim.x)
      dst[k] = src[k];
    if constexpr (MODE != 2)
      for (int i = tid; i < SPAD; i += blockDim.x) {
        elo_s[i] = i < S ? e_lo[i] : 1.0;
        ehi_s[i] = i < S ? e_hi[i] : 1.0;
      }
  }
  if constexpr (MODE == 2) {
    const int4* src = img + (size_t)b * kImg4;
    int4* dst = (int4*)gi;
    for (int k = tid; k < kImg4; k += blockDim.x) dst[k] = src[k];
    __syncthreads();
  } else {
  i8_init_eval<SPAD, NSL, 4>(ev, pos + (size_t)b * S, S, tid, blockDim.x, padg);
  __syncthreads();
  {  // U' / ln 2 as the free diagonal "parent" i of child i
    int8_t* A8 = (int8_t*)ev.A;
    for (int k = tid; k < S * NSL; k += blockDim.x) {
      const int i = k / NSL, sl = k - i * NSL;
      A8[sl * SPAD * 64 + a_byte<4>(i, i)] = udig[i * 8 + sl];
    }
  }
  {
    constexpr int KB = 4;
    const int npass = i8_npass(S, cap);
    const int my = npass > w ? (npass - w + WAVES - 1) / WAVES : 0;
    for (int k0 = 0; k0 < my; k0 += KB)
      i8o_prep_passes<SPAD, WAVES, KB, 4, true>(ev, k0, w, lane, S, cap, 0, w01 + (size_t)b * S * S,
                                                elo_s, ehi_s, ltab);
  }
  __syncthreads();
  // G + u0 in units of 2^-20 / ln 2: g0 = rint(.) + (1023 << 20) (the exponent
  // bias of exp2_fx_acc), g1 = the remainder in units of 2^-38 / ln 2 (the
  // C-init of slices 5-6); |g1| <= 2^17.  G is one value per row, so its
  // rounding is systematic over the effects: it gets T_1's full resolution.
  for (int i = tid; i < SPAD; i += blockDim.x) {
    const double g = i < S ? ev.G[i] + u0[i] : ev.G[i];
    const double g0 = rint(g * kL2Scale);
    gi[i] = (int)g0 + (1023 << 20);
    gi[SPAD + i] = (int)rint(fma(g, kL2Scale, -g0) * 262144.0);
  }
  __syncthreads();
  if constexpr (MODE == 1) {
    const int4* src = (const int4*)gi;
    int4* dst = img + (size_t)b * kImg4;
    for (int k = tid; k < kImg4; k += blockDim.x) dst[k] = src[k];
    return;
  }
  }  // MODE != 2
#if NEMO_I8_ABLATE & 32  // instrumented build (tools/ablate.sh): prep only, no tiles
  if (s_end > 0) return;
#endif

  const i32x4* Bt = (const i32x4*)B8;
  const i32x4* Bt64 = Bt + (size_t)ntiles * kWave;  // the staged D1 bytes x 64
  const i32x4* Gi = (const i32x4*)gi;
  const uint32_t a_lane = (uint32_t)(col * 4 + ((rg + 2 * (col >> 2)) & 3));  // swizzled chunk
  int set = s_begin + w;
  if constexpr (TT == 1) {
    int set = s_begin + w;
    if (set < s_end) {
      double lprod = 1.0;
      int lexp = 0;
      int t = 8 * set;
      i32x4 bc = Bt[(size_t)t * kWave + lane];
      i32x4 bc64 = Bt64[(size_t)t * kWave + lane];
      for (;;) {
        uint32_t ao = a_lane;
        asm volatile("" : "+v"(ao));
        const i32x4* Al = ev.A + ao;
        int tn = t + 1, setn = set;
        if (tn >= min(ntiles, 8 * set + 8)) {
          setn = set + WAVES;
          tn = 8 * setn;
        }
        const bool more = setn < s_end;
        const int tl = more ? tn : t;  // prefetch target (the current tile again at the end)
        const i32x4 b1 = bc, b64 = bc64;
        bc = Bt[(size_t)tl * kWave + lane];
        bc64 = Bt64[(size_t)tl * kWave + lane];
        double ls0 = 0.0, ls1 = 0.0;
  #pragma unroll
        for (int r = 0; r < NR; ++r) {
          const i32x4 c0 = Gi[(16 * r) / 4 + rg];
          const i32x4 c1 = Gi[(SPAD + 16 * r) / 4 + rg];
  #if NEMO_I8_ABLATE & 128  // instrumented build: half the A-fragment reads (wrong values)
          auto A = [&](int sl) { return Al[((sl & ~1) * SPAD + 16 * r) * 4]; };
  #else
          auto A = [&](int sl) { return Al[(sl * SPAD + 16 * r) * 4]; };
  #endif
  #if NEMO_I8_ABLATE & 2  // instrumented build: no MFMA (one add per pair; wrong values)
          const i32x4 h0 = A(0) + A(1) + b64, h1 = A(2) + A(3) + c0, l0 = A(4) + b1,
                      l1 = A(5) + A(6) + c1;
  #else
          i32x4 h0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(0), b64, i32x4{0, 0, 0, 0}, 0, 0, 0);
          h0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(1), b1, h0, 0, 0, 0);
          i32x4 h1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(2), b64, c0, 0, 0, 0);
          h1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(3), b1, h1, 0, 0, 0);
          const i32x4 l0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(4), b1, i32x4{0, 0, 0, 0}, 0, 0, 0);
          i32x4 l1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(5), b64, c1, 0, 0, 0);
          l1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(6), b1, l1, 0, 0, 0);
  #endif
          // the row block's 4 cells per lane in three phases, so the 4 table
          // reads (random entries: ~3.5-way bank conflicts) are in flight
          // while the series runs: addresses + reads, series, then assembly
          uint32_t t0[4];
          uint64_t ev[4];
          double pr[4];
  #pragma unroll
          for (int g = 0; g < 4; ++g) {
            // T_0 wraps mod 2^32 only transiently (its true value is in (0, 2^31))
            t0[g] = ((uint32_t)h0[g] << 12) + (uint32_t)h1[g];
            ev[g] = exp2_fx_load(t0[g]);
          }
  #pragma unroll
          for (int g = 0; g < 4; ++g)
            pr[g] = exp2_fx_series(t0[g], (int)(((uint32_t)l0[g] << 12) + (uint32_t)l1[g]));
  #pragma unroll
          for (int g = 0; g < 4; ++g) {
            if (g & 1) ls1 = exp2_fx_apply(t0[g], ev[g], pr[g], ls1);
            else ls0 = exp2_fx_apply(t0[g], ev[g], pr[g], ls0);
          }
        }
        double l = rowsum4(ls0 + ls1) + 1.0;  // + e^0 of the null row
        lprod *= t * 16 + col < E ? l : 1.0;
        lexp += __builtin_amdgcn_frexp_exp(lprod);
        lprod = __builtin_amdgcn_frexp_mant(lprod);
        if (setn != set) {  // set complete: one partial
          // every 16-lane row holds the 16 column products (rowsum4): log_fast
          // (lprod is a mantissa in [0.5, 1)) and a DPP sum within the row
          double v = log_fast(lprod, ltab) + (double)lexp * 0.69314718055994530942;
          v = rowsum16(v);
          if (lane == 0) partial[(size_t)b * nsets + set] = nullsum[set] + v;
          lprod = 1.0;
          lexp = 0;
        }
        if (!more) break;
        t = tn;
        set = setn;
      }
    }
  } else {
    // TT = 2: two 16-effect tiles per iteration share each row block's A
    // fragments and G C-inits (half the A-fragment LDS reads); the same
    // arithmetic per cell and the same order of the column products as TT = 1,
    // so the same bits.  The second tile of a set's odd tail repeats the first
    // and is not multiplied in.
    i8l_walk2<NR, WAVES>(ev.A, Gi, Bt, Bt64, set, s_end, ntiles, E, col, lane, a_lane, nullsum, partial, b,
                         nsets, ltab, [](int) {});
  }
  if (split == 1) {
    __syncthreads();
    if (w == 0) {
      const double v = sum_partials(partial + (size_t)b * nsets, nsets, lane);
      if (lane == 0) ll_out[b] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// score_i8s_kernel: score_i8l_kernel with the Delta digits stationary in
// registers.  In score_i8l_kernel every wave walks all row blocks of its
// tiles, re-reading the 7 x NR A fragments from LDS per tile (28 KB of LDS
// reads per 16-effect tile at S = 64, next to the table reads): the LDS, not
// the SIMDs, sets the pace.  Here wave w owns row block rb = w % NR for every
// tile of its group of sets (grp = w / NR, NG = 8 / NR groups): its 7 A
// fragments and G C-inits are loaded into registers once, after the prep.
// Per tile a wave sums its 16 rows per effect column (4 cells per lane +
// the row-group swaps) and posts the sums to LDS; after a block barrier per
// set, one wave of the group (rotating) adds the NR row-block sums, forms
// l = 1 + sum and the set's partial (product per lane over two tiles, one
// log).  Partials are per set, as in score_i8l_kernel, so ll bits do not
// depend on the batch size or the block split.
// ---------------------------------------------------------------------------
template <int NR>
__global__ __launch_bounds__(8 * kWave, NEMO_I8O_WAVES_PER_SIMD) void score_i8s_kernel(
    int S, int E, int ntiles, int nsets, int split, int cap, double padg,
    const int32_t* __restrict__ pos, const double* __restrict__ w01,
    const double* __restrict__ e_lo, const double* __restrict__ e_hi,
    const uint8_t* __restrict__ B8, const int8_t* __restrict__ udig, const double* __restrict__ u0,
    const double* __restrict__ nullsum, const void* __restrict__ tabs,
    double* __restrict__ partial, double* __restrict__ ll_out, int remap) {
  constexpr int WAVES = 8;
  constexpr int SPAD = NR * 16;
  constexpr int NSL = 7;
  constexpr int NG = WAVES / NR;                          // groups of row-block waves
  extern __shared__ __attribute__((aligned(16))) double lds8[];
  uint2* etab_o = (uint2*)lds8;                          // [kExpTabN] at LDS address 0
  double2* ltab = (double2*)(etab_o + kExpTabN);         // [128] log table
  double* elo_s = (double*)(ltab + 128);                 // [SPAD] e^lo_j
  double* ehi_s = elo_s + SPAD;                          // [SPAD] e^hi_j
  EvalLds ev;
  ev.G = ehi_s + SPAD;                                   // [SPAD]
  int* gi = (int*)(ev.G + SPAD);                         // [2][SPAD] g0, g1
  ev.perm = gi + 2 * SPAD;                               // [SPAD]
  ev.A = (i32x4*)(ev.perm + SPAD);                       // [NSL][SPAD][4] swizzled (a_byte)
  // after the A fragments are in registers the same region holds the
  // row-block column sums: [NG][2 (parity)][8 tiles][NR][16] doubles (16 KB)
  double* colsum = (double*)ev.A;

  const int work = xcd_index8((int)blockIdx.x, (int)gridDim.x, remap);
  const int b = work / split;
  const int part = work - b * split;
  const int spb = (nsets + split - 1) / split;
  const int s_begin = part * spb;
  const int s_end = min(nsets, s_begin + spb);
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int rb = w % NR, grp = w / NR;
  const int col = lane & 15, rg = lane >> 4;

  {  // both tables (precomputed per context) in one contiguous 18 KB copy
    const int4* src = (const int4*)tabs;
    int4* dst = (int4*)lds8;
    for (int k = tid; k < (kExpTabN * 8 + 128 * 16) / 16; k += blockDim.x) dst[k] = src[k];
    for (int i = tid; i < SPAD; i += blockDim.x) {
      elo_s[i] = i < S ? e_lo[i] : 1.0;
      ehi_s[i] = i < S ? e_hi[i] : 1.0;
    }
  }
  i8_init_eval<SPAD, NSL, 4>(ev, pos + (size_t)b * S, S, tid, blockDim.x, padg);
  __syncthreads();
  {  // U' / ln 2 as the free diagonal "parent" i of child i
    int8_t* A8 = (int8_t*)ev.A;
    for (int k = tid; k < S * NSL; k += blockDim.x) {
      const int i = k / NSL, sl = k - i * NSL;
      A8[sl * SPAD * 64 + a_byte<4>(i, i)] = udig[i * 8 + sl];
    }
  }
  {
    constexpr int KB = 4;
    const int npass = i8_npass(S, cap);
    const int my = npass > w ? (npass - w + WAVES - 1) / WAVES : 0;
    for (int k0 = 0; k0 < my; k0 += KB)
      i8o_prep_passes<SPAD, WAVES, KB, 4, true>(ev, k0, w, lane, S, cap, 0, w01 + (size_t)b * S * S,
                                                elo_s, ehi_s, ltab);
  }
  __syncthreads();
  for (int i = tid; i < SPAD; i += blockDim.x) {  // G + u0 as in score_i8l_kernel
    const double g = i < S ? ev.G[i] + u0[i] : ev.G[i];
    const double g0 = rint(g * kL2Scale);
    gi[i] = (int)g0 + (1023 << 20);
    gi[SPAD + i] = (int)rint(fma(g, kL2Scale, -g0) * 262144.0);
  }
  __syncthreads();
  // this wave's row block: A fragments and G C-inits into registers
  i32x4 af[NSL];
  {
    const i32x4* Al = ev.A + (uint32_t)(col * 4 + ((rg + 2 * (col >> 2)) & 3));  // swizzled chunk
#pragma unroll
    for (int sl = 0; sl < NSL; ++sl) af[sl] = Al[(sl * SPAD + 16 * rb) * 4];
  }
  const i32x4 c0 = ((const i32x4*)gi)[(16 * rb) / 4 + rg];
  const i32x4 c1 = ((const i32x4*)gi)[(SPAD + 16 * rb) / 4 + rg];
  __syncthreads();  // the A region becomes the column-sum buffer
#if NEMO_I8_ABLATE & 32  // instrumented build (tools/ablate.sh): prep only, no tiles
  if (s_end > 0) return;
#endif

  const i32x4* Bt = (const i32x4*)B8;
  const int nsb = s_end > s_begin ? s_end - s_begin : 0;
  const int niter = (nsb + NG - 1) / NG;  // uniform over the block
  int tpre = 8 * (s_begin + grp);
  i32x4 bc = Bt[(size_t)min(tpre, ntiles - 1) * kWave + lane];
  for (int k = 0; k < niter; ++k) {
    const int set = s_begin + k * NG + grp;
    double* cs = colsum + (size_t)((grp * 2 + (k & 1)) * 8) * NR * 16;
    if (set < s_end) {
      const int t_end = min(ntiles, 8 * set + 8);
      for (int t = 8 * set; t < t_end; ++t) {
        // next tile of this wave (next set of the group after the last one)
        const int tn = t + 1 < t_end ? t + 1 : 8 * (set + NG);
        const i32x4 b1 = bc;
        const i32x4 b64 = b1 << 6;
        bc = Bt[(size_t)min(tn, ntiles - 1) * kWave + lane];
        const i32x4 h0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(
            af[1], b1, __builtin_amdgcn_mfma_i32_16x16x64_i8(af[0], b64, i32x4{0, 0, 0, 0}, 0, 0, 0), 0, 0, 0);
        const i32x4 h1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(
            af[3], b1, __builtin_amdgcn_mfma_i32_16x16x64_i8(af[2], b64, c0, 0, 0, 0), 0, 0, 0);
        const i32x4 l0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[4], b1, i32x4{0, 0, 0, 0}, 0, 0, 0);
        const i32x4 l1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(
            af[6], b1, __builtin_amdgcn_mfma_i32_16x16x64_i8(af[5], b64, c1, 0, 0, 0), 0, 0, 0);
        uint32_t t0[4];
        uint64_t evt[4];
        double pr[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          t0[g] = ((uint32_t)h0[g] << 12) + (uint32_t)h1[g];
          evt[g] = exp2_fx_load(t0[g]);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g)
          pr[g] = exp2_fx_series(t0[g], (int)(((uint32_t)l0[g] << 12) + (uint32_t)l1[g]));
        double ls0 = 0.0, ls1 = 0.0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (g & 1) ls1 = exp2_fx_apply(t0[g], evt[g], pr[g], ls1);
          else ls0 = exp2_fx_apply(t0[g], evt[g], pr[g], ls0);
        }
        const double v = rowsum4(ls0 + ls1);  // the row block's 16 rows, per column
        if (lane < 16) cs[((t - 8 * set) * NR + rb) * 16 + col] = v;
      }
    }
    __syncthreads();
    if (set < s_end && rb == k % NR) {  // this set's partial: 8 tiles x 16 columns
      double lp = 1.0;
      int le = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tt = (lane >> 4) + 4 * h;
        const int t = 8 * set + tt;
        double l = 1.0;  // + e^0 of the null row
#pragma unroll
        for (int q = 0; q < NR; ++q) l += cs[(tt * NR + q) * 16 + col];
        lp *= t < ntiles && t * 16 + col < E ? l : 1.0;
        le += __builtin_amdgcn_frexp_exp(lp);
        lp = __builtin_amdgcn_frexp_mant(lp);
      }
      const double v = wsum(log(lp) + (double)le * 0.69314718055994530942);
      if (lane == 0) partial[(size_t)b * nsets + set] = nullsum[set] + v;
    }
  }
  if (split == 1) {
    __syncthreads();
    if (w == 0) {
      const double v = sum_partials(partial + (size_t)b * nsets, nsets, lane);
      if (lane == 0) ll_out[b] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// score_i8p_kernel (fact_kernel 17; an experiment, not auto): score_i8l_kernel's
// two-tile walk in a persistent block that pipelines its evaluations.  In
// score_i8l_kernel a block preps one evaluation's digits (global weight loads,
// two log_fast and the digit split per pair; 19% of the launch on its own)
// before it walks its tiles.  Here each block owns evaluations b, b + grid, ...
// with two digit buffers: while the waves walk evaluation n from one buffer,
// each wave preps its passes of evaluation n + 1 into the other after its first
// walk iteration, so the prep's loads and logs interleave with the tiles; no
// per-evaluation table copy.  Two block barriers per evaluation.  The per-set
// arithmetic, the digits, G and the partial sum are score_i8l_kernel's own
// code, so the bits are too.  Measured 7-13% SLOWER than score_i8l_kernel at
// C3 whatever the prep point: one evaluation per block lets
// the dispatcher backfill retiring blocks, which overlaps the preps already.
// ---------------------------------------------------------------------------
template <int NR, int WAVES>
__global__ __launch_bounds__(WAVES * kWave, NEMO_I8L2_OCC) void score_i8p_kernel(
    int S, int E, int ntiles, int nsets, int batch, int cap, double padg,
    const int32_t* __restrict__ pos, const double* __restrict__ w01,
    const double* __restrict__ e_lo, const double* __restrict__ e_hi,
    const uint8_t* __restrict__ B8, const int8_t* __restrict__ udig, const double* __restrict__ u0,
    const double* __restrict__ nullsum, const void* __restrict__ tabs,
    double* __restrict__ partial, double* __restrict__ ll_out) {
  constexpr int SPAD = NR * 16;
  constexpr int NSL = 7;
  // one evaluation buffer: G [SPAD] f64, gi [2][SPAD], perm [SPAD], A [NSL][SPAD][4] x 16 B
  constexpr int kBufG = 0, kBufGi = SPAD * 8, kBufPerm = kBufGi + 2 * SPAD * 4, kBufA = kBufPerm + SPAD * 4;
  constexpr int kBuf = kBufA + NSL * SPAD * 64;
  static_assert(kBufA % 16 == 0 && kBuf % 16 == 0, "16-B alignment of the A fragments");
  extern __shared__ __attribute__((aligned(16))) double lds8[];
  uint2* etab_o = (uint2*)lds8;                          // [kExpTabN] at LDS address 0
  double2* ltab = (double2*)(etab_o + kExpTabN);         // [128] log table
  double* elo_s = (double*)(ltab + 128);                 // [SPAD] e^lo_j
  double* ehi_s = elo_s + SPAD;                          // [SPAD] e^hi_j
  char* bufs = (char*)(ehi_s + SPAD);                    // [2][kBuf]
  auto evb = [&](int k) {
    EvalLds e;
    char* p = bufs + k * kBuf;
    e.G = (double*)(p + kBufG);
    e.perm = (int*)(p + kBufPerm);
    e.A = (i32x4*)(p + kBufA);
    return e;
  };
  auto gib = [&](int k) { return (int*)(bufs + k * kBuf + kBufGi); };

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int col = lane & 15, rg = lane >> 4;
  const int nb = gridDim.x;
  const int b0 = blockIdx.x;
  if (b0 >= batch) return;  // (the launch never makes more blocks than evaluations)

  auto set_perm = [&](int k, int e) {
    int* perm = evb(k).perm;
    for (int j = tid; j < S; j += blockDim.x) {
      int pj = pos[(size_t)e * S + j];
      pj = pj < 0 ? 0 : (pj >= S ? S - 1 : pj);  // malformed input must not fault
      perm[pj] = j;
    }
  };
  auto zero_a = [&](int k) {
    i32x4* A = evb(k).A;
    for (int q = tid; q < NSL * SPAD * 4; q += blockDim.x) A[q] = i32x4{0, 0, 0, 0};
  };
  auto diag = [&](int k) {  // U' / ln 2 as the free diagonal "parent" i of child i
    int8_t* A8 = (int8_t*)evb(k).A;
    for (int q = tid; q < S * NSL; q += blockDim.x) {
      const int i = q / NSL, sl = q - i * NSL;
      A8[sl * SPAD * 64 + a_byte<4>(i, i)] = udig[i * 8 + sl];
    }
  };
  auto prep = [&](int k, int e) {  // this wave's passes of evaluation e into buffer k
    constexpr int KB = 4;
    const int npass = i8_npass(S, cap);
    const int my = npass > w ? (npass - w + WAVES - 1) / WAVES : 0;
    for (int k0 = 0; k0 < my; k0 += KB)
      i8o_prep_passes<SPAD, WAVES, KB, 4, true>(evb(k), k0, w, lane, S, cap, 0, w01 + (size_t)e * S * S,
                                                elo_s, ehi_s, ltab);
  };
  auto finalize_g = [&](int k) {  // score_i8l_kernel's G + u0 split (see there)
    const EvalLds ev = evb(k);
    int* gi = gib(k);
    for (int i = tid; i < SPAD; i += blockDim.x) {
      const double g = i < S ? ev.G[i] + u0[i] : ev.G[i];
      const double g0 = rint(g * kL2Scale);
      gi[i] = (int)g0 + (1023 << 20);
      gi[SPAD + i] = (int)rint(fma(g, kL2Scale, -g0) * 262144.0);
    }
  };

  {  // both tables (precomputed per context) in one contiguous 18 KB copy
    const int4* src = (const int4*)tabs;
    int4* dst = (int4*)lds8;
    for (int k = tid; k < (kExpTabN * 8 + 128 * 16) / 16; k += blockDim.x) dst[k] = src[k];
    for (int i = tid; i < SPAD; i += blockDim.x) {
      elo_s[i] = i < S ? e_lo[i] : 1.0;
      ehi_s[i] = i < S ? e_hi[i] : 1.0;
    }
  }
  for (int k = 0; k < 2; ++k) {
    for (int i = tid; i < SPAD; i += blockDim.x) evb(k).G[i] = i < S ? 0.0 : padg;
    zero_a(k);
  }
  set_perm(0, b0);
  if (b0 + nb < batch) set_perm(1, b0 + nb);
  __syncthreads();
  diag(0);
  diag(1);
  __syncthreads();
  prep(0, b0);
  __syncthreads();
  finalize_g(0);
  __syncthreads();

  const i32x4* Bt = (const i32x4*)B8;
  const i32x4* Bt64 = Bt + (size_t)ntiles * kWave;  // the staged D1 bytes x 64
  const uint32_t a_lane = (uint32_t)(col * 4 + ((rg + 2 * (col >> 2)) & 3));  // swizzled chunk
  int k = 0;
  for (int e = b0; e < batch; e += nb, k ^= 1) {
    const int en = e + nb;
    bool pending = en < batch;
    i8l_walk2<NR, WAVES>(evb(k).A, (const i32x4*)gib(k), Bt, Bt64, w, nsets, ntiles, E, col, lane, a_lane,
                         nullsum, partial, (size_t)e, nsets, ltab, [&](int it) {
                           if (pending && it == 0) {
                             prep(k ^ 1, en);
                             pending = false;
                           }
                         });
    if (pending) prep(k ^ 1, en);  // a wave with no set to walk (nsets < 8)
    __syncthreads();  // evaluation e walked (its partials written), en prepped
    if (w == 0) {
      const double v = sum_partials(partial + (size_t)e * nsets, nsets, lane);
      if (lane == 0) ll_out[e] = v;
    }
    if (en < batch) finalize_g(k ^ 1);
    const bool again = en + nb < batch;  // buffer k is refilled with evaluation en + nb
    if (again) {
      zero_a(k);
      set_perm(k, en + nb);
    }
    __syncthreads();
    if (again) diag(k);  // other bytes than the prep's, which may already run (next walk)
  }
}

template <int NR>
hipError_t launch_i8s_t(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                        double* d_ll, hipStream_t st, int* nparts, bool* finalized) {
  constexpr int SPAD = NR * 16;
  const int ntiles = (c.E + 15) / 16;
  const int nsets = (ntiles + 7) / 8;
  const int slots = 256 * (NEMO_I8O_WAVES_PER_SIMD * 4 / 8);
  int split = (slots + batch - 1) / batch;
  split = split < 1 ? 1 : (split > nsets ? nsets : split);
  const size_t region = std::max((size_t)7 * SPAD * 64, (size_t)16384);
  const size_t lds = kExpTabN * 8 + 128 * 16 + 3 * SPAD * 8 + 3 * SPAD * 4 + region;
  score_i8s_kernel<NR><<<dim3(batch * split), 8 * kWave, lds, st>>>(
      c.S, c.E, ntiles, nsets, split, cap, c.i8o_padg, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_B8,
      c.d_udig2, c.d_u0, c.d_nullsum, c.d_i8o_tabs, fpartial(c), d_ll, c.xcd_remap);
  *nparts = nsets;
  *finalized = split == 1;
  return hipGetLastError();
}

template <int NR>
hipError_t launch_i8p_t(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                        double* d_ll, hipStream_t st, int* nparts, bool* finalized) {
  constexpr int SPAD = NR * 16;
  const int ntiles = (c.E + 15) / 16;
  const int nsets = (ntiles + 7) / 8;
  const size_t lds = kExpTabN * 8 + 128 * 16 + 2 * SPAD * 8 + 2 * ((size_t)SPAD * 20 + (size_t)7 * SPAD * 64);
  int dev = 0, ncu = 0;
  hipError_t ge = hipGetDevice(&dev);
  if (ge == hipSuccess) ge = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (ge != hipSuccess) return ge;
  if (ncu <= 0) ncu = 256;
  if (lds > 65536) {  // past the default 64 KB of dynamic LDS (gfx950 has 160 KB per CU)
    hipError_t ae = hipFuncSetAttribute((const void*)score_i8p_kernel<NR, 8>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (ae != hipSuccess) return ae;
  }
  // two resident blocks per CU (LDS: 2 x 77.5 KB at S = 64; VGPRs: 4 waves per SIMD)
  // three blocks per CU in the grid (two are resident: LDS 2 x 77.5 KB at S =
  // 64), so the third set of blocks starts as the first ones retire and the
  // CU's blocks drift out of phase (1 / 2 / 3 per CU: 0.202 / 0.172 / 0.167 ms
  // at C3, B = 2048); every wave preps at the start of its walk (staggered
  // points measured the same or slower)
  const int grid = std::min(batch, 3 * ncu);
  score_i8p_kernel<NR, 8><<<dim3(grid), 8 * kWave, lds, st>>>(
      c.S, c.E, ntiles, nsets, batch, cap, c.i8o_padg, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_B8,
      c.d_udig2, c.d_u0, c.d_nullsum, c.d_i8o_tabs, fpartial(c), d_ll);
  *nparts = nsets;
  *finalized = true;
  return hipGetLastError();
}

template <int NR, int WAVES, int OCC = NEMO_I8O_WAVES_PER_SIMD, int TT = 1, bool SPLIT = false>
hipError_t launch_i8l_t(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                        double* d_ll, hipStream_t st, int* nparts, bool* finalized) {
  constexpr int SPAD = NR * 16;
  const int ntiles = (c.E + 15) / 16;
  const int nsets = (ntiles + 7) / 8;
  const int slots = 256 * (OCC * 4 / WAVES);
  int split = (slots + batch - 1) / batch;
  split = split < 1 ? 1 : (split > nsets ? nsets : split);
  const size_t lds = kExpTabN * 8 + 128 * 16 + 3 * SPAD * 8 + 3 * SPAD * 4 + (size_t)7 * SPAD * 64;
  if (SPLIT) {  // fact_kernel 20: a prep-only launch (one block per evaluation), then the walks
    if (!c.d_i8img || c.i8img_cap < batch || (size_t)SPAD * 460 != i8img_bytes(c.fspad))
      return hipErrorInvalidValue;
    score_i8l_kernel<NR, WAVES, OCC, TT, 1><<<dim3(batch), WAVES * kWave, lds, st>>>(
        c.S, c.E, ntiles, nsets, 1, cap, c.i8o_padg, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_B8,
        c.d_udig2, c.d_u0, c.d_nullsum, c.d_i8o_tabs, fpartial(c), d_ll, c.xcd_remap, (int4*)c.d_i8img);
    score_i8l_kernel<NR, WAVES, OCC, TT, 2><<<dim3(batch * split), WAVES * kWave, lds, st>>>(
        c.S, c.E, ntiles, nsets, split, cap, c.i8o_padg, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_B8,
        c.d_udig2, c.d_u0, c.d_nullsum, c.d_i8o_tabs, fpartial(c), d_ll, c.xcd_remap, (int4*)c.d_i8img);
  } else {
    score_i8l_kernel<NR, WAVES, OCC, TT><<<dim3(batch * split), WAVES * kWave, lds, st>>>(
        c.S, c.E, ntiles, nsets, split, cap, c.i8o_padg, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_B8,
        c.d_udig2, c.d_u0, c.d_nullsum, c.d_i8o_tabs, fpartial(c), d_ll, c.xcd_remap);
  }
  *nparts = nsets;
  *finalized = split == 1;
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// score_i8w_kernel (fact_kernel 18): score_i8l_kernel for 64 < S <= 128.
//
// The contraction runs over K = 128 parents as two K = 64 halves per row
// block, accumulated into the same int32 accumulators (|acc| < 2^20 for 128
// parents: T_0 = acc_0 2^12 + acc_1 wraps mod 2^32 only transiently, its
// true value is in (0, 2^31) by stage_i8o's |x| <= 690, as at S <= 64).  The
// digits, G in the C-inits, the exp assembly from the integer accumulators
// and the offset log-sum-exp are score_i8l_kernel's (7 slices, 2^-38 / ln 2
// per entry).  Per evaluation the LDS holds A[7][2][128][64 B] = 112 KB, so
// one 16-wave block runs per CU (4 waves per SIMD).  The walk takes one
// 16-effect tile per iteration; partials are per pair of tiles (32 effects),
// so even E = 700 gives the 16 waves 22 partials to share, and ll bits do
// not depend on the batch size (one block per evaluation, in-kernel sum).
// ---------------------------------------------------------------------------
constexpr int kWideKH = 2;    // K halves
// kWideSetT (nemo_internal.h): tiles per partial

// i8l_digits into the two-half layout: slice sl, half j >> 6
__device__ __forceinline__ void i8w_digits(int8_t* A8, int i, int j, double d) {
  constexpr int SPAD = 128, SL = SPAD * 64;  // bytes per (slice, half)
  const double hd = rint(d * kL2Scale);
  const int h = (int)hd;
  const int l = (int)rint(fma(d, kL2Scale, -hd) * 262144.0);
  const int off = (j >> 6) * SL + a_byte<4>(i, j & 63);
  const int hb = h + 32 * (1 + 64 + 4096), lb = l + 32 * (1 + 64);
  A8[(0 * kWideKH) * SL + off] = (int8_t)(hb >> 18);
  A8[(1 * kWideKH) * SL + off] = (int8_t)(((hb >> 12) & 63) - 32);
  A8[(2 * kWideKH) * SL + off] = (int8_t)(((hb >> 6) & 63) - 32);
  A8[(3 * kWideKH) * SL + off] = (int8_t)((hb & 63) - 32);
  A8[(4 * kWideKH) * SL + off] = (int8_t)(lb >> 12);
  A8[(5 * kWideKH) * SL + off] = (int8_t)(((lb >> 6) & 63) - 32);
  A8[(6 * kWideKH) * SL + off] = (int8_t)((lb & 63) - 32);
}

// the prep passes of i8o_prep_passes with up to 127 parents per pair of
// children: each pass covers its (child, parent) slots in kWideKH rounds of
// 64 lanes; a lane's G terms of the pass are summed over the rounds, then
// over the wave
template <int WAVES, int KB>
__device__ __forceinline__ void i8w_prep_passes(EvalLds e, int k0, int w, int lane, int S, int cap,
                                                const double* __restrict__ w01b,
                                                const double* __restrict__ elo_s,
                                                const double* __restrict__ ehi_s,
                                                const double2* __restrict__ ltab) {
  const bool packed = cap == 0 || cap >= S - 1;
  const int npass = packed ? (S + 1) / 2 : S;
  int8_t* A8 = (int8_t*)e.A;
  double ga[KB], gb[KB];
#pragma unroll
  for (int kk = 0; kk < KB; ++kk) {
    ga[kk] = 0.0;
    gb[kk] = 0.0;
    const int q = w + (k0 + kk) * WAVES;
#pragma unroll
    for (int hr = 0; hr < kWideKH; ++hr) {
      const int p = lane + 64 * hr;
      int qr = 0, pp = 0;
      bool act = false, side_a = true;
      if (q < npass) {
        if (packed) {
          const int q2 = S - 1 - q;
          if (p < q) { qr = q; pp = p; act = true; }
          else { qr = q2; pp = p - q; act = q2 != q && pp < q2; side_a = false; }
        } else {
          const int np = q < cap ? q : cap;
          qr = q; pp = q - 1 - p; act = p < np;
        }
      }
      if (act) {
        const int i = e.perm[qr], j = e.perm[pp];
        const double sw = w01b[i * S + j];
        const double lo = log_fast(fma(sw, elo_s[j] - 1.0, 1.0), ltab);
        const double d = log_fast(fma(sw, ehi_s[j] - 1.0, 1.0), ltab) - lo;
        i8w_digits(A8, i, j, d);
        if (side_a) ga[kk] += lo;
        else gb[kk] += lo;
      }
    }
  }
#pragma unroll
  for (int kk = 0; kk < KB; ++kk) {
    ga[kk] = wsum_dpp(ga[kk]);
    gb[kk] = wsum_dpp(gb[kk]);
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

template <int WAVES, int OCC, bool TWO>
__global__ __launch_bounds__(WAVES * kWave, OCC) void score_i8w_kernel(
    int S, int E, int ntiles, int nsets, int cap, double padg,
    const int32_t* __restrict__ pos, const double* __restrict__ w01,
    const double* __restrict__ e_lo, const double* __restrict__ e_hi,
    const uint8_t* __restrict__ B8, const int8_t* __restrict__ udig, const double* __restrict__ u0,
    const double* __restrict__ nullsum, const void* __restrict__ tabs,
    double* __restrict__ partial, double* __restrict__ ll_out, int remap) {
  constexpr int NR = 8, SPAD = NR * 16;
  constexpr int NSL = 7;
  extern __shared__ __attribute__((aligned(16))) double lds8[];
  uint2* etab_o = (uint2*)lds8;                          // [kExpTabN] at LDS address 0
  double2* ltab = (double2*)(etab_o + kExpTabN);         // [128] log table
  double* elo_s = (double*)(ltab + 128);                 // [SPAD] e^lo_j
  double* ehi_s = elo_s + SPAD;                          // [SPAD] e^hi_j
  EvalLds ev;
  ev.G = ehi_s + SPAD;                                   // [SPAD]
  int* gi = (int*)(ev.G + SPAD);                         // [2][SPAD] g0, g1
  ev.perm = gi + 2 * SPAD;                               // [SPAD]
  ev.A = (i32x4*)(ev.perm + SPAD);                       // [NSL][KH][SPAD][4] swizzled (a_byte)

  const int b = xcd_index8((int)blockIdx.x, (int)gridDim.x, remap);
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int col = lane & 15, rg = lane >> 4;

  {  // both tables (precomputed per context) in one contiguous 18 KB copy
    const int4* src = (const int4*)tabs;
    int4* dst = (int4*)lds8;
    for (int k = tid; k < (kExpTabN * 8 + 128 * 16) / 16; k += blockDim.x) dst[k] = src[k];
    for (int i = tid; i < SPAD; i += blockDim.x) {
      elo_s[i] = i < S ? e_lo[i] : 1.0;
      ehi_s[i] = i < S ? e_hi[i] : 1.0;
    }
  }
  i8_init_eval<SPAD, NSL * kWideKH, 4>(ev, pos + (size_t)b * S, S, tid, blockDim.x, padg);
  __syncthreads();
  {  // U' / ln 2 as the free diagonal "parent" i of child i
    int8_t* A8 = (int8_t*)ev.A;
    for (int k = tid; k < S * NSL; k += blockDim.x) {
      const int i = k / NSL, sl = k - i * NSL;
      A8[(sl * kWideKH + (i >> 6)) * SPAD * 64 + a_byte<4>(i, i & 63)] = udig[i * 8 + sl];
    }
  }
  {
    constexpr int KB = 2;
    const int npass = i8_npass(S, cap);
    const int my = npass > w ? (npass - w + WAVES - 1) / WAVES : 0;
    for (int k0 = 0; k0 < my; k0 += KB)
      i8w_prep_passes<WAVES, KB>(ev, k0, w, lane, S, cap, w01 + (size_t)b * S * S, elo_s, ehi_s, ltab);
  }
  __syncthreads();
  // G + u0 in units of 2^-20 / ln 2 (score_i8l_kernel)
  for (int i = tid; i < SPAD; i += blockDim.x) {
    const double g = i < S ? ev.G[i] + u0[i] : ev.G[i];
    const double g0 = rint(g * kL2Scale);
    gi[i] = (int)g0 + (1023 << 20);
    gi[SPAD + i] = (int)rint(fma(g, kL2Scale, -g0) * 262144.0);
  }
  __syncthreads();

  const i32x4* Gi = (const i32x4*)gi;
  const uint32_t a_lane = (uint32_t)(col * 4 + ((rg + 2 * (col >> 2)) & 3));  // swizzled chunk
  // B fragments [x64][half][tile][lane] through a buffer resource
  const __amdgpu_buffer_rsrc_t brs =
      __builtin_amdgcn_make_buffer_rsrc((void*)B8, (short)0, 2 * kWideKH * ntiles * kWave * 16, 0x00020000);
  const uint32_t bln = (uint32_t)lane * 16u;
  auto bload = [&](int tile, int x64, int h) {
    return __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         brs, bln, ((x64 * kWideKH + h) * ntiles + tile) * kWave * 16, 0));
  };
  if constexpr (TWO) {
    // the set's two tiles a, b in one iteration: each A fragment is read once
    // for both (half the LDS A traffic); rowsum_pair leaves tile a's column
    // sums in rows 0 / 2 and tile b's in rows 1 / 3 (as score_i8l_kernel's
    // two-tile walk).  A set of one tile (odd ntiles) repeats it and does not
    // multiply the copy in.
    for (int set = w; set < nsets; set += WAVES) {
      const int ta = kWideSetT * set;
      const bool two = ta + 1 < ntiles;
      const int tb = two ? ta + 1 : ta;
      const i32x4 b1a[2] = {bload(ta, 0, 0), bload(ta, 0, 1)}, b64a[2] = {bload(ta, 1, 0), bload(ta, 1, 1)};
      const i32x4 b1b[2] = {bload(tb, 0, 0), bload(tb, 0, 1)}, b64b[2] = {bload(tb, 1, 0), bload(tb, 1, 1)};
      uint32_t ao = a_lane;
      asm volatile("" : "+v"(ao));
      const i32x4* Al = ev.A + ao;
      double la0 = 0.0, la1 = 0.0, lb0 = 0.0, lb1 = 0.0;
#pragma unroll 1
      for (int r = 0; r < NR; ++r) {
        const i32x4 c0 = Gi[(16 * r) / 4 + rg];
        const i32x4 c1 = Gi[(SPAD + 16 * r) / 4 + rg];
        auto A = [&](int sl, int h) { return Al[((sl * kWideKH + h) * SPAD + 16 * r) * 4]; };
        i32x4 h0a = i32x4{0, 0, 0, 0}, h0b = i32x4{0, 0, 0, 0}, h1a = c0, h1b = c0;
        i32x4 l0a = i32x4{0, 0, 0, 0}, l0b = i32x4{0, 0, 0, 0}, l1a = c1, l1b = c1;
#pragma unroll
        for (int h = 0; h < kWideKH; ++h) {
          {
            const i32x4 a = A(0, h);
            h0a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64a[h], h0a, 0, 0, 0);
            h0b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64b[h], h0b, 0, 0, 0);
          }
          {
            const i32x4 a = A(1, h);
            h0a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a[h], h0a, 0, 0, 0);
            h0b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b[h], h0b, 0, 0, 0);
          }
          {
            const i32x4 a = A(2, h);
            h1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64a[h], h1a, 0, 0, 0);
            h1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64b[h], h1b, 0, 0, 0);
          }
          {
            const i32x4 a = A(3, h);
            h1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a[h], h1a, 0, 0, 0);
            h1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b[h], h1b, 0, 0, 0);
          }
          {
            const i32x4 a = A(4, h);
            l0a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a[h], l0a, 0, 0, 0);
            l0b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b[h], l0b, 0, 0, 0);
          }
          {
            const i32x4 a = A(5, h);
            l1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64a[h], l1a, 0, 0, 0);
            l1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b64b[h], l1b, 0, 0, 0);
          }
          {
            const i32x4 a = A(6, h);
            l1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1a[h], l1a, 0, 0, 0);
            l1b = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b1b[h], l1b, 0, 0, 0);
          }
        }
        auto epi = [&](const i32x4 h0, const i32x4 h1, const i32x4 l0, const i32x4 l1, double& ls0,
                       double& ls1) {
          uint32_t t0[4];
          uint64_t evv[4];
          double pr[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            t0[g] = ((uint32_t)h0[g] << 12) + (uint32_t)h1[g];
            evv[g] = exp2_fx_load(t0[g]);
          }
#pragma unroll
          for (int g = 0; g < 4; ++g)
            pr[g] = exp2_fx_series(t0[g], (int)(((uint32_t)l0[g] << 12) + (uint32_t)l1[g]));
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if (g & 1) ls1 = exp2_fx_apply(t0[g], evv[g], pr[g], ls1);
            else ls0 = exp2_fx_apply(t0[g], evv[g], pr[g], ls0);
          }
        };
        epi(h0a, h1a, l0a, l1a, la0, la1);
        epi(h0b, h1b, l0b, l1b, lb0, lb1);
      }
      const double l = rowsum_pair(la0 + la1, lb0 + lb1) + 1.0;  // + e^0 of the null row
      const bool tile_b = (lane & 16) != 0;
      const bool ok = (((tile_b ? tb : ta) * 16 + col) < E) & (two | !tile_b);
      const double lprod = ok ? l : 1.0;  // one factor per lane: no renormalisation
      // rows 0 / 1 hold tile a's / tile b's 16 column values
      double v = log_fast(lprod, ltab);
      v = rowsum16(v);
      v += __shfl_down(v, 16, kWave);
      if (lane == 0) partial[(size_t)b * nsets + set] = nullsum[set] + v;
    }
  } else {
    for (int set = w; set < nsets; set += WAVES) {
      double lprod = 1.0;
      int lexp = 0;
      const int t_end = min(ntiles, kWideSetT * set + kWideSetT);
      for (int t = kWideSetT * set; t < t_end; ++t) {
        const i32x4 b1[2] = {bload(t, 0, 0), bload(t, 0, 1)};
        const i32x4 b64[2] = {bload(t, 1, 0), bload(t, 1, 1)};
        uint32_t ao = a_lane;
        asm volatile("" : "+v"(ao));
        const i32x4* Al = ev.A + ao;
        double ls0 = 0.0, ls1 = 0.0;
  #pragma unroll 2
        for (int r = 0; r < NR; ++r) {
          const i32x4 c0 = Gi[(16 * r) / 4 + rg];
          const i32x4 c1 = Gi[(SPAD + 16 * r) / 4 + rg];
          auto A = [&](int sl, int h) { return Al[((sl * kWideKH + h) * SPAD + 16 * r) * 4]; };
          i32x4 h0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(0, 0), b64[0], i32x4{0, 0, 0, 0}, 0, 0, 0);
          h0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(0, 1), b64[1], h0, 0, 0, 0);
          h0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(1, 0), b1[0], h0, 0, 0, 0);
          h0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(1, 1), b1[1], h0, 0, 0, 0);
          i32x4 h1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(2, 0), b64[0], c0, 0, 0, 0);
          h1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(2, 1), b64[1], h1, 0, 0, 0);
          h1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(3, 0), b1[0], h1, 0, 0, 0);
          h1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(3, 1), b1[1], h1, 0, 0, 0);
          i32x4 l0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(4, 0), b1[0], i32x4{0, 0, 0, 0}, 0, 0, 0);
          l0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(4, 1), b1[1], l0, 0, 0, 0);
          i32x4 l1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(5, 0), b64[0], c1, 0, 0, 0);
          l1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(5, 1), b64[1], l1, 0, 0, 0);
          l1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(6, 0), b1[0], l1, 0, 0, 0);
          l1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A(6, 1), b1[1], l1, 0, 0, 0);
          uint32_t t0[4];
          uint64_t evv[4];
          double pr[4];
  #pragma unroll
          for (int g = 0; g < 4; ++g) {
            t0[g] = ((uint32_t)h0[g] << 12) + (uint32_t)h1[g];
            evv[g] = exp2_fx_load(t0[g]);
          }
  #pragma unroll
          for (int g = 0; g < 4; ++g)
            pr[g] = exp2_fx_series(t0[g], (int)(((uint32_t)l0[g] << 12) + (uint32_t)l1[g]));
  #pragma unroll
          for (int g = 0; g < 4; ++g) {
            if (g & 1) ls1 = exp2_fx_apply(t0[g], evv[g], pr[g], ls1);
            else ls0 = exp2_fx_apply(t0[g], evv[g], pr[g], ls0);
          }
        }
        const double l = rowsum4(ls0 + ls1) + 1.0;  // + e^0 of the null row
        lprod *= t * 16 + col < E ? l : 1.0;
        lexp += __builtin_amdgcn_frexp_exp(lprod);
        lprod = __builtin_amdgcn_frexp_mant(lprod);
      }
      // every 16-lane row holds the 16 column products (rowsum4)
      double v = log_fast(lprod, ltab) + (double)lexp * 0.69314718055994530942;
      v = rowsum16(v);
      if (lane == 0) partial[(size_t)b * nsets + set] = nullsum[set] + v;
    }
  }
  __syncthreads();
  if (w == 0) {
    const double v = sum_partials(partial + (size_t)b * nsets, nsets, lane);
    if (lane == 0) ll_out[b] = v;
  }
}

}  // namespace

hipError_t i8img_reserve(Ctx& c) {
  const int nb = std::max(c.cap_batch, 1);
  if (c.d_i8img && c.i8img_cap >= nb) return hipSuccess;
  hipError_t e = hipStreamSynchronize(c.stream);
  if (e != hipSuccess) return e;
  ++c.graph_epoch;
  if (c.d_i8img) (void)hipFree(c.d_i8img);
  c.d_i8img = nullptr;
  c.i8img_cap = 0;
  e = hipMalloc((void**)&c.d_i8img, (size_t)nb * i8img_bytes(std::max(c.fspad, 16)));
  if (e == hipSuccess) c.i8img_cap = nb;
  return e;
}

hipError_t launch_score_i8o(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                            double* d_ll, int waves, bool l2, hipStream_t st, int* nparts,
                            bool* finalized) {
  if (!c.i8o_ok || !c.d_Uoff || !c.d_nullsum || !c.d_B8 || !c.d_i8o_tabs) return hipErrorInvalidValue;
  if (l2 && (!c.i8l_ok || !c.d_udig2)) return hipErrorInvalidValue;
  switch (c.fspad / 16) {
#define NEMO_I8O(NRV)                                                                          \
  case NRV:                                                                                    \
    if (l2)                                                                                    \
      return waves == 0 ? launch_i8s_t<NRV>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized) \
           : waves == 16 ? launch_i8l_t<NRV, 16>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized) \
           : waves == -3 ? launch_i8p_t<NRV>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized) \
           : waves == 8  ? launch_i8l_t<NRV, 8>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized)  \
           : waves == -8 ? launch_i8l_t<NRV, 8, 6>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized) \
           : waves == -2 ? launch_i8l_t<NRV, 8, NEMO_I8L2_OCC, 2>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized) \
           : waves == -20 ? launch_i8l_t<NRV, 8, NEMO_I8L2_OCC, 2, true>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized) \
                         : launch_i8l_t<NRV, 4>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized); \
    if (c.i8o_diag && !c.i8o_nodiag)                                                           \
      return waves == 8 ? launch_i8o_t<NRV, 8, true>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized) \
                        : launch_i8o_t<NRV, 4, true>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized); \
    return waves == 8 ? launch_i8o_t<NRV, 8, false>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized) \
                      : launch_i8o_t<NRV, 4, false>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized);
    NEMO_I8O(1)
    NEMO_I8O(2)
    NEMO_I8O(4)
#undef NEMO_I8O
    default: return hipErrorInvalidValue;
  }
}

template <bool TWO>
hipError_t launch_i8w_t(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                        double* d_ll, hipStream_t st, int* nparts, bool* finalized) {
  if (!c.i8w_ok || c.fspad != 128 || !c.d_nullsum_w || !c.d_B8 || !c.d_udig2 || !c.d_i8o_tabs)
    return hipErrorInvalidValue;
  constexpr int SPAD = 128, WAVES = 16, NSL = 7;
  const int ntiles = (c.E + 15) / 16;
  const int nsets = (ntiles + kWideSetT - 1) / kWideSetT;
  const size_t lds = kExpTabN * 8 + 128 * 16 + 3 * SPAD * 8 + 3 * SPAD * 4 + (size_t)NSL * kWideKH * SPAD * 64;
  hipError_t ae = hipFuncSetAttribute((const void*)score_i8w_kernel<WAVES, 4, TWO>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (ae != hipSuccess) return ae;
  score_i8w_kernel<WAVES, 4, TWO><<<dim3(batch), WAVES * kWave, lds, st>>>(
      c.S, c.E, ntiles, nsets, cap, c.i8o_padg, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_B8, c.d_udig2, c.d_u0,
      c.d_nullsum_w, c.d_i8o_tabs, fpartial(c), d_ll, c.xcd_remap);
  *nparts = nsets;
  *finalized = true;
  return hipGetLastError();
}

// fact_kernel 18: two tiles per iteration (auto); 19: one
hipError_t launch_score_i8w(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                            double* d_ll, bool two, hipStream_t st, int* nparts, bool* finalized) {
  return two ? launch_i8w_t<true>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized)
             : launch_i8w_t<false>(c, batch, cap, d_pos, d_w01, d_ll, st, nparts, finalized);
}

// staging for score_i8o_kernel (after d_U64, e^lo / e^hi and the int8 scale):
// U' = U - U[S] ((fspad + 1) rows, zero past S), sum_e U[S][e] per 8-tile set
// (left fold), and the range checks that make the offset exp safe.
hipError_t stage_i8o(Ctx& c, const std::vector<double>& elo, const std::vector<double>& ehi,
                     const std::vector<uint64_t>& d1) {
  c.i8o_ok = false;
  c.i8o_diag = false;
  c.i8l_ok = false;
  c.i8w_ok = false;
  for (void** p : {(void**)&c.d_Uoff, (void**)&c.d_nullsum, (void**)&c.d_udig, (void**)&c.d_u0,
                   (void**)&c.d_udig2, (void**)&c.d_nullsum_w})
    if (*p) {
      hipError_t fe = hipFree(*p);
      *p = nullptr;
      if (fe != hipSuccess) return fe;
    }
  const int S = c.S, E = c.E, SPAD = c.fspad;
  // S <= 64: the int8 offset kernels; 64 < S <= 128: score_i8w_kernel (the
  // same checks, the log2 form only)
  if (!c.d_B8 || SPAD > 128 || SPAD < S) return hipSuccess;
  hipError_t err = hipStreamSynchronize(c.stream);
  if (err != hipSuccess) return err;
  std::vector<double> U((size_t)(S + 1) * E);
  if ((err = copy_sync(c, U.data(), c.d_U64, U.size() * 8, hipMemcpyDeviceToHost)) != hipSuccess) return err;
  const double* un = U.data() + (size_t)S * E;
  std::vector<double> uo((size_t)(SPAD + 1) * E + 16, 0.0);
  double umin = 0.0, umax = 0.0;
  for (int i = 0; i < S; ++i)
    for (int e = 0; e < E; ++e) {
      const double v = U[(size_t)i * E + e] - un[e];
      uo[(size_t)i * E + e] = v;
      umin = std::min(umin, v);
      umax = std::max(umax, v);
    }
  // each parent's log factor lies between 0 and its table value (lo_j or hi_j)
  double fmin = 0.0, fmax = 0.0, gabs = 0.0;
  for (int j = 0; j < S; ++j) {
    const double lo = log(elo[j]), hi = log(ehi[j]);
    fmin += std::min(0.0, std::min(lo, hi));
    fmax += std::max(0.0, std::max(lo, hi));
    gabs += fabs(lo);
  }
  // |g0| must leave the int32 room of T_0 = (acc0 << 12) + acc1 (|acc| < 2^19)
  const double glim = 0.9 * (ldexp(1.0, 30) - ldexp(1.0, 20)) * ldexp(1.0, c.i8_cexp - 24);
  const double padg = -std::min(500.0, glim);
  const bool ok = std::isfinite(umin) && std::isfinite(umax) && umin + fmin >= -690.0 &&
                  umax + fmax <= 690.0 && gabs <= glim && padg <= -40.0;
  if (!ok) return hipSuccess;
  const int ntiles = (E + 15) / 16, nsets = (ntiles + 7) / 8;
  std::vector<double> ns(nsets, 0.0);
  for (int s = 0; s < nsets; ++s) {
    double acc = 0.0;
    for (int e = 128 * s; e < std::min(E, 128 * s + 128); ++e) acc += un[e];
    ns[s] = acc;
  }
  if (!c.d_i8o_tabs) {
    // exp_acc's table (2^(j/2048), high dword adjusted) then log_fast's, as
    // fill_log_table computes it; long double for correctly rounded entries
    std::vector<uint32_t> tb(kExpTabN * 2 + 128 * 4);
    for (int j = 0; j < kExpTabN; ++j) {
      const double v = (double)exp2l((long double)j / kExpTabN);
      uint64_t b;
      memcpy(&b, &v, 8);
      tb[2 * j] = (uint32_t)b;
      tb[2 * j + 1] = ((uint32_t)(b >> 32) & 0x800fffffu) ^ ((uint32_t)j << 9);
    }
    double* lt = (double*)(tb.data() + kExpTabN * 2);
    for (int k = 0; k < 128; ++k) {
      const double inv = 1.0 / (1.0 + ((double)k + 0.5) * (1.0 / 128.0));
      lt[2 * k] = inv;
      lt[2 * k + 1] = (double)-logl((long double)inv);
    }
    if ((err = hipMalloc(&c.d_i8o_tabs, tb.size() * 4)) != hipSuccess) return err;
    if ((err = copy_sync(c, c.d_i8o_tabs, tb.data(), tb.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
      return err;
  }
  // diagonal form: U'[i][e] = u0_i + (u1_i - u0_i) D1[i][e] (within 1e-11; every U
  // nem.py builds: U' = D ? -A : B up to the rounding of its addition chains),
  // then U' is the free diagonal entry of the contraction (digits of u1 - u0
  // at A[i][i], u0 in G) and the kernel reads no U at all
  {
    const int nwords = (E + 63) / 64;
    bool diag = true;
    std::vector<double> u0(S, 0.0), du(S, 0.0);
    const double half = ldexp(1.0, c.i8_cexp - 1) * (1.0 - 1e-9);
    for (int i = 0; i < S && diag; ++i) {
      double ub[2] = {0.0, 0.0};
      bool have[2] = {false, false};
      for (int e = 0; e < E && diag; ++e) {
        const int bit = (int)((d1[(size_t)i * nwords + e / 64] >> (e % 64)) & 1ull);
        const double v = uo[(size_t)i * E + e];
        if (!have[bit]) {
          ub[bit] = v;
          have[bit] = true;
        } else if (fabs(v - ub[bit]) > 1e-11) {
          diag = false;
        }
      }
      u0[i] = have[0] ? ub[0] : ub[1];
      du[i] = have[0] && have[1] ? ub[1] - ub[0] : 0.0;
      if (!(fabs(du[i]) < half)) diag = false;
    }
    if (diag) {
      // the device's digit expansion (i8o_digits, i8l_digits)
      auto expand = [&](bool l2, std::vector<int8_t>& dig) {
        dig.assign((size_t)S * 8, 0);
        for (int i = 0; i < S; ++i) {
          double hd, lr;
          if (l2) {
            hd = nearbyint(du[i] * kL2Scale);
            lr = fma(du[i], kL2Scale, -hd);
          } else {
            const double x = ldexp(du[i], 6 - c.i8_cexp);
            hd = nearbyint(x * 262144.0);
            lr = fma(x, 262144.0, -hd);
          }
          const int h = (int)hd;
          const int kb = 32 * (1 + 64 + 4096);
          int8_t* o = dig.data() + (size_t)i * 8;
          const int hb = h + kb;
          o[0] = (int8_t)(hb >> 18);
          o[1] = (int8_t)(((hb >> 12) & 63) - 32);
          o[2] = (int8_t)(((hb >> 6) & 63) - 32);
          o[3] = (int8_t)((hb & 63) - 32);
          if (l2) {  // i8l_digits: l in units of 2^-38, three digits, slice 7 unused
            const int lb = (int)nearbyint(lr * 262144.0) + 32 * (1 + 64);
            o[4] = (int8_t)(lb >> 12);
            o[5] = (int8_t)(((lb >> 6) & 63) - 32);
            o[6] = (int8_t)((lb & 63) - 32);
          } else {
            const int lb = (int)nearbyint(lr * 16777216.0) + kb;
            o[4] = (int8_t)(lb >> 18);
            o[5] = (int8_t)(((lb >> 12) & 63) - 32);
            o[6] = (int8_t)(((lb >> 6) & 63) - 32);
            o[7] = (int8_t)((lb & 63) - 32);
          }
        }
      };
      std::vector<int8_t> dig, dig2;
      expand(false, dig);
      if ((err = hipMalloc((void**)&c.d_udig, dig.size())) != hipSuccess) return err;
      if ((err = hipMalloc((void**)&c.d_u0, S * 8)) != hipSuccess) return err;
      if ((err = copy_sync(c, c.d_udig, dig.data(), dig.size(), hipMemcpyHostToDevice)) != hipSuccess) return err;
      if ((err = copy_sync(c, c.d_u0, u0.data(), S * 8, hipMemcpyHostToDevice)) != hipSuccess) return err;
      c.i8o_diag = true;
      // log2 fixed point: every entry v = delta 2^20 / ln 2 needs |rint(v)| <
      // 2^25 - 2^17 - 2^6 (top digit in [-128, 127] after the balancing bias),
      // and T_0 = (x / ln 2 + 1023) 2^20 must stay in (0, 2^31): |x| <= 690
      // (checked above) gives 27 < x / ln 2 + 1023 < 2019, and G + u0 rides
      // in T_0's C-init, so |G + u0| / ln 2 + 1023 < 2047
      constexpr double kLn2 = 0.69314718055994530942;
      const double vmax = ldexp(1.0, 25) - ldexp(1.0, 17) - 128.0;
      double dmax = 0.0, umax0 = 0.0;
      for (int j = 0; j < S; ++j) dmax = std::max(dmax, fabs(log(ehi[j]) - log(elo[j])));
      for (int i = 0; i < S; ++i) {
        dmax = std::max(dmax, fabs(du[i]));
        umax0 = std::max(umax0, fabs(u0[i]));
      }
      if (dmax * kL2Scale < vmax && (gabs + umax0) / kLn2 + 1023.0 < 2000.0 && -padg / kLn2 < 1000.0) {
        expand(true, dig2);
        if ((err = hipMalloc((void**)&c.d_udig2, dig2.size())) != hipSuccess) return err;
        if ((err = copy_sync(c, c.d_udig2, dig2.data(), dig2.size(), hipMemcpyHostToDevice)) != hipSuccess)
          return err;
        c.i8l_ok = true;
      }
    }
  }
  if (SPAD == 128 && c.i8l_ok) {
    // score_i8w_kernel's partials cover 2 tiles (32 effects): sum_e U[S][e]
    // per 32 effects, left fold
    const int nsw = (ntiles + kWideSetT - 1) / kWideSetT;
    std::vector<double> nw(nsw, 0.0);
    for (int s2 = 0; s2 < nsw; ++s2) {
      double acc = 0.0;
      for (int e = 32 * s2; e < std::min(E, 32 * s2 + 32); ++e) acc += un[e];
      nw[s2] = acc;
    }
    if ((err = hipMalloc((void**)&c.d_nullsum_w, nw.size() * 8)) != hipSuccess) return err;
    if ((err = copy_sync(c, c.d_nullsum_w, nw.data(), nw.size() * 8, hipMemcpyHostToDevice)) != hipSuccess)
      return err;
    c.i8w_ok = true;
  }
  if ((err = hipMalloc((void**)&c.d_Uoff, uo.size() * 8)) != hipSuccess) return err;
  if ((err = hipMalloc((void**)&c.d_nullsum, ns.size() * 8)) != hipSuccess) return err;
  if ((err = copy_sync(c, c.d_Uoff, uo.data(), uo.size() * 8, hipMemcpyHostToDevice)) != hipSuccess) return err;
  if ((err = copy_sync(c, c.d_nullsum, ns.data(), ns.size() * 8, hipMemcpyHostToDevice)) != hipSuccess) return err;
  c.i8o_padg = padg;
  c.i8o_ok = true;
  return hipSuccess;
}

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
