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
// error <= 2^(c-6-6*2NP-1) per entry (NP = 4: 2^-45 at c = 4).  Each pair of
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
constexpr int kI8TilesPerWave = 8;   // fixed: ll bits independent of batch
constexpr int kI8WavesPerSimd = 2;   // occupancy target of the register budget

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
// prep: Delta digits and G in node order.  grid = batch * (SPAD / 16),
// block = 256 (4 waves x 4 rows); lane = parent node j (SPAD <= 64).
//   D8 [b][2NP][SPAD][64] int8,  G [b][SPAD]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prep_i8_kernel(int S, int SPAD, int cap, int nsl, int cexp,
                                                      const int32_t* __restrict__ pos,
                                                      const double* __restrict__ w01,
                                                      const double* __restrict__ e_lo,
                                                      const double* __restrict__ e_hi,
                                                      int8_t* __restrict__ D8, double* __restrict__ G) {
  const int ngroups = SPAD / 16;
  const int b = blockIdx.x / ngroups;
  const int grp = blockIdx.x - b * ngroups;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = threadIdx.x / kWave;
  const int j = lane;
  const int* pb = pos + (size_t)b * S;
  const int pj = j < S ? pb[j] : 0;
  const double elo = j < S ? e_lo[j] : 1.0, ehi = j < S ? e_hi[j] : 1.0;
  for (int i = 16 * grp + w; i < 16 * grp + 16; i += 4) {
    double d = 0.0, lo = 0.0;
    if (i < S && j < S) {
      const int pi = pb[i];
      if (pj < pi && (cap == 0 || pi - pj <= cap)) {
        const double s = w01[((size_t)b * S + i) * S + j];
        lo = log(fma(s, elo - 1.0, 1.0));
        d = log(fma(s, ehi - 1.0, 1.0)) - lo;
      }
    }
    const double g = wsum(lo);
    if (lane == 0) G[(size_t)b * SPAD + i] = i < S ? g : kPadG8;
    // fixed-point digits: x = Delta * 2^(6-c) in [-32, 32]; each step is exact
    double x = ldexp(d, 6 - cexp);
    int8_t* out = D8 + (((size_t)b * nsl) * SPAD + i) * 64 + j;
    for (int s = 0; s < nsl; ++s) {
      const double q = rint(x);
      out[(size_t)s * SPAD * 64] = (int8_t)(int)q;
      x = (x - q) * 64.0;
    }
  }
}

// ---------------------------------------------------------------------------
// score: block = (evaluation b, WAVES * 8 consecutive 16-effect tiles),
// wave = tiles t_begin + w, + WAVES, ...; grid = batch * split (XCD remap,
// evaluation-major).  Every wave: per tile, NP pairs of i8 MFMAs per row
// block, exact integer recombination, f64 cells, column log-sum-exp.
// ---------------------------------------------------------------------------
template <int NR, int WAVES, int NP, bool AREG>
__global__ __launch_bounds__(WAVES * kWave, AREG ? 1 : kI8WavesPerSimd) void score_i8_kernel(
    int S, int E, int ntiles, int split, const int8_t* __restrict__ D8,
    const double* __restrict__ Gd, const uint8_t* __restrict__ B8, const double* __restrict__ U,
    double sA, double sB, double sC, double* __restrict__ partial, int remap) {
  constexpr int SPAD = NR * 16;
  constexpr int NSL = 2 * NP;
  extern __shared__ __attribute__((aligned(16))) double lds8[];
  double* etab = lds8;                                   // [256]
  double* Gs = etab + 256;                               // [SPAD]
  i32x4* A = (i32x4*)(Gs + SPAD);                        // [NSL][SPAD][5] 16-byte chunks
                                                         // (80-B rows: conflict-free b128)

  const int work = xcd_index8((int)blockIdx.x, (int)gridDim.x, remap);
  const int b = work / split;
  const int part = work - b * split;
  const int t_begin = part * kI8TilesPerWave * WAVES;
  const int t_end = min(ntiles, t_begin + kI8TilesPerWave * WAVES);
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int col = lane & 15, rg = lane >> 4;

  for (int k = tid; k < 256; k += blockDim.x) etab[k] = exp2((double)k * (1.0 / 256.0));
  for (int k = tid; k < SPAD; k += blockDim.x) Gs[k] = Gd[(size_t)b * SPAD + k];
  const i32x4* Ag = (const i32x4*)(D8 + (size_t)b * NSL * SPAD * 64);
  for (int k = tid; k < NSL * SPAD * 4; k += blockDim.x) A[(k >> 2) * 5 + (k & 3)] = Ag[k];
  // U rows of this lane's cells: 16r + 4rg + g (i8 C layout).  The staged U
  // has >= SPAD rows (rows S+1.. are zero; their G is kPadG8), so a cell's
  // address is a uniform part ((16r + g) E, an SGPR base) + one per-lane
  // offset (4 rg E + col): no per-load VALU.
  const uint32_t uln = (uint32_t)(4 * rg * E + col);
  __syncthreads();

  double* part_out = partial + (size_t)b * split * WAVES + part * WAVES + w;
  int t = t_begin + w;
  if (t >= t_end) {
    if (lane == 0) *part_out = 0.0;
    return;
  }
  const i32x4* Bt = (const i32x4*)B8;

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
  load_tile(t);
  const uint32_t a_lane = (uint32_t)(col * 5 + rg);  // A chunk of this lane, row block 0, slice 0
  for (; t < t_end; t += WAVES) {
    // launder the A offset each tile: keeps the loop-invariant A fragments
    // (2NP * NR * 16 B per lane) in LDS instead of hoisted into registers
    uint32_t ao = a_lane;
    if constexpr (!AREG) asm volatile("" : "+v"(ao));
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
    if (t + WAVES < t_end) load_tile(t + WAVES);
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
    msum += valid ? m : 0.0;
    lprod *= valid ? l : 1.0;
    lexp += __builtin_amdgcn_frexp_exp(lprod);
    lprod = __builtin_amdgcn_frexp_mant(lprod);
  }
  double v = msum + (log(lprod) + (double)lexp * 0.69314718055994530942);
  v = lane < 16 ? v : 0.0;
  v = wsum(v);
  if (lane == 0) *part_out = v;
}

template <int NR, int WAVES, int NP, bool AREG>
hipError_t launch_i8_t(Ctx& c, int batch, hipStream_t st, int* nparts) {
  constexpr int SPAD = NR * 16;
  const int ntiles = (c.E + 15) / 16;
  const int tpb = kI8TilesPerWave * WAVES;
  const int split = (ntiles + tpb - 1) / tpb;
  const size_t lds = 256 * 8 + SPAD * 8 + (size_t)2 * NP * SPAD * 80;
  const double sA = ldexp(1.0, c.i8_cexp - 24), sB = ldexp(1.0, c.i8_cexp - 48),
               sC = ldexp(1.0, c.i8_cexp - 60);
  score_i8_kernel<NR, WAVES, NP, AREG><<<dim3(batch * split), WAVES * kWave, lds, st>>>(
      c.S, c.E, ntiles, split, c.d_fD8, c.d_fG, c.d_B8, (const double*)c.d_U64, sA, sB, sC,
      c.d_fpartial, c.xcd_remap);
  *nparts = split * WAVES;
  return hipGetLastError();
}

}  // namespace

hipError_t launch_prep_i8(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01, int np,
                          hipStream_t st) {
  const int spad = c.fspad;
  if (spad > 64 || np < 4 || np > kI8MaxPairs) return hipErrorInvalidValue;
  prep_i8_kernel<<<batch * (spad / 16), 256, 0, st>>>(c.S, spad, cap, 2 * np, c.i8_cexp, d_pos, d_w01,
                                                     c.d_elo, c.d_ehi, c.d_fD8, c.d_fG);
  return hipGetLastError();
}

hipError_t launch_score_i8(Ctx& c, int batch, int np, int waves, bool areg, hipStream_t st,
                           int* nparts) {
  const int nr = c.fspad / 16;
#define NEMO_I8(NRV, WV, NPV, AR)                           \
  if (nr == NRV && waves == WV && np == NPV && areg == AR) \
    return launch_i8_t<NRV, WV, NPV, AR>(c, batch, st, nparts);
  NEMO_I8(1, 4, 4, false) NEMO_I8(2, 4, 4, false) NEMO_I8(4, 4, 4, false)
  NEMO_I8(1, 4, 5, false) NEMO_I8(2, 4, 5, false) NEMO_I8(4, 4, 5, false)
  NEMO_I8(1, 8, 4, false) NEMO_I8(2, 8, 4, false) NEMO_I8(4, 8, 4, false)
  NEMO_I8(1, 4, 4, true) NEMO_I8(2, 4, 4, true) NEMO_I8(4, 4, 4, true)
#undef NEMO_I8
  return hipErrorInvalidValue;
}

}  // namespace nemo
