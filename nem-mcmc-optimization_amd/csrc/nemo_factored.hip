// nemo_factored.hip -- order score as a dense fp64 MFMA contraction.
//
// Every score table the reference builds (nem.py:36-47) has, for a parent
// j != child i, T[i][j][e] = L[j][e] independent of i, and L[j][e] takes two
// values (B where D[j][e] == 0, -A where D[j][e] == 1).  So each log factor of
// compute_cell_ratios (nem_order_mcmc.py:83-86) is one of two numbers per
// (i, j):  g_lo(i,j) = log(1 - w + w e^{lo_j}),  g_hi(i,j) = log(1 - w + w e^{hi_j}),
// and the cell ratios become
//     cell[i][e] = U[i][e] + G[i] + sum_j Delta[i][j] * D1[j][e],
//     G[i] = sum_{j in pa(i)} g_lo(i,j),   Delta = g_hi - g_lo (0 off pa(i)),
// a (S x S) . (S x E) product with K = S.  Staging detects the structure and
// keeps D1 as a bit matrix; the product runs on v_mfma_f64_16x16x4_f64 and
// the column log-sum-exp is fused into the epilogue.
//
// Children and parents are taken in ORDER position (pi), so Delta is strictly
// lower triangular (a band of width `cap` with a parent cap) and the MFMA
// k-loop of row block r stops at the diagonal: ~half the square's work.
//
// Geometry: one block = one evaluation x (WAVES*16) effects; each wave owns
// 16 effects and ALL children (NR row blocks of 16), so the log-sum-exp over
// children stays inside the wave (two xor-shuffles).  Delta is staged
// through LDS per 64-parent chunk (row stride 66 doubles: conflict-free
// ds_read_b64 A-fragments); the B fragments are bits of D1, expanded in
// registers once per chunk.
#include "nemo_internal.h"

#include <math.h>

#include <algorithm>

namespace nemo {

namespace {

using f64x4 = __attribute__((ext_vector_type(4))) double;

__device__ __forceinline__ double fwave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// exp(x) for x <= ~0 in fp64 from a 64-entry table of 2^(j/64) and a
// degree-5 polynomial on |r| <= ln2/128 (truncation < 4e-17): ~12 VALU ops
// instead of the ~25 of the general exp; relative error a few ulp.
__device__ __forceinline__ double exp_tab(double x, const double* __restrict__ tab) {
  constexpr double kInvLn2x64 = 92.332482616893656768;     // 64 / ln 2
  constexpr double kLn2d64Hi = 1.0830424696223417e-02;     // ln2/64, high part
  constexpr double kLn2d64Lo = 2.5728046223276690e-14;     // ln2/64 - high part
  x = fmax(x, -1000.0);
  const double kf = rint(x * kInvLn2x64);
  const int k = (int)kf;
  double r = fma(-kf, kLn2d64Hi, x);
  r = fma(-kf, kLn2d64Lo, r);
  double p = fma(r, 1.0 / 120.0, 1.0 / 24.0);
  p = fma(r, p, 1.0 / 6.0);
  p = fma(r, p, 0.5);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
  return ldexp(p * tab[k & 63], k >> 6);
}

// exp(x) for finite x in [-1e12, ~0] (the log-sum-exp terms): 256-entry
// table of 2^(j/256) and a degree-4 polynomial on |r| <= ln2/512 (truncation
// < 4e-17).  k = round(x * 256/ln2) comes from the low word of
// fma(x, 256/ln2, 1.5*2^52) (no clamp, rint or cvt), and the reduction uses
// one constant: its error, |x| * 1.6e-16 relative, is weighted by e^x in the
// sum (< 1e-16 of it).  9 f64 VALU + 3 integer.
__device__ __forceinline__ double exp_lse(double x, const double* __restrict__ tab) {
  constexpr double kInvLn2x256 = 369.32993046757462707;  // 256 / ln 2
  constexpr double kLn2d256 = 2.7076061740622862e-03;    // ln 2 / 256
  constexpr double kMagic = 6755399441055744.0;          // 1.5 * 2^52
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

// v_max_f64 without the sNaN canonicalisation hipcc wraps around fmax: the
// operands here are MFMA results and loads of finite tables
__device__ __forceinline__ double vmax(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// value of the G column on padding rows (q >= S): cells of padding rows are
// U[S][e] + kPadG, whose exp underflows to exactly 0 next to any real row
constexpr double kPadG = -1.0e6;

// tiles per wave of the pipelined kernel: fixed, so the tile -> wave ->
// partial assignment (hence every bit of ll) does not depend on the batch
constexpr int kPipeTilesPerWave = 8;

__device__ __forceinline__ int fxcd_work_index(int L, int N, int remap) {
  if (!remap) return L;
  const int x = L & 7, k = L >> 3;
  const int q = N >> 3, r = N & 7;
  return x * q + (x < r ? x : r) + k;
}

// ---------------------------------------------------------------------------
// prep: Delta, G and pi of every evaluation.  grid = batch, block = 256.
// Dp [b][SPAD][SPAD] (row = child position q, col = parent position p),
// G  [b][SPAD], permo [b][SPAD] (node at position q; S for padding rows).
// ---------------------------------------------------------------------------
// one wave: row q (child position q) of Delta and its G, for the order in
// perm (LDS); padding rows (q >= S) carry zeros and a finite "no row" G
__device__ __forceinline__ void delta_row(int S, int SPAD, int cap, int b, int q, const int* perm,
                                          const double* __restrict__ w01, const double* __restrict__ e_lo,
                                          const double* __restrict__ e_hi, double* __restrict__ Dp,
                                          double* __restrict__ G, int lane) {
  const int i = q < S ? perm[q] : 0;
  const double* wrow = w01 + ((size_t)b * S + i) * S;
  double* drow = Dp + ((size_t)b * SPAD + q) * SPAD;
  double gsum = 0.0;
  for (int p0 = 0; p0 < SPAD; p0 += kWave) {
    const int p = p0 + lane;
    double d = 0.0, glo = 0.0;
    const bool ok = q < S && p < q && (cap == 0 || q - p <= cap);
    if (ok) {
      const int j = perm[p];
      const double s = wrow[j];
      const double lo = log(fma(s, e_lo[j] - 1.0, 1.0));
      const double hi = log(fma(s, e_hi[j] - 1.0, 1.0));
      d = hi - lo;
      glo = lo;
    }
    if (p < SPAD && p != (q | 15)) drow[p] = d;
    gsum += fwave_sum(glo);
  }
  if (lane == 0) {
    G[(size_t)b * SPAD + q] = gsum;
    // column 16r+15 of row block r is never a parent of rows 16r..16r+15:
    // it carries G (the score kernels multiply it by 1), and a finite
    // "no row" value on padding rows
    drow[q | 15] = q < S ? gsum : kPadG;
  }
}

__global__ __launch_bounds__(256) void prep_factored_kernel(
    int S, int SPAD, int cap, const int32_t* __restrict__ pos, const double* __restrict__ w01,
    const double* __restrict__ e_lo, const double* __restrict__ e_hi, double* __restrict__ Dp,
    double* __restrict__ G, int32_t* __restrict__ permo) {
  __shared__ int perm[kMaxS];
  __shared__ int scan[kMaxS];
  // block = (evaluation, group of 4 child positions); one row per wave (the
  // rows of one evaluation spread over SPAD / 4 blocks: a lone evaluation's
  // prep is a quarter of the serial work per wave it was with 16-row blocks)
  const int ngroups = SPAD / 4;
  const int b = blockIdx.x / ngroups;
  const int grp = blockIdx.x - b * ngroups;
  const int tid = threadIdx.x;
  prep_order_lds(S, cap, pos + (size_t)b * S, perm, scan, false);
  if (grp == 0)
    for (int k = tid; k < SPAD; k += blockDim.x) permo[(size_t)b * SPAD + k] = k < S ? perm[k] : S;
  const int q = 4 * grp + tid / kWave;
  delta_row(S, SPAD, cap, b, q, perm, w01, e_lo, e_hi, Dp, G, tid & (kWave - 1));
}

// the fused step's prep (nemo_optimal_weights_dev): prep_kernel's work for
// children 4 g .. 4 g + 3 and prep_factored_kernel's for positions 4 g ..
// 4 g + 3 in one block g of the evaluation -- the same arithmetic, one
// launch (a graph node costs ~5 us however small its kernel)
__global__ __launch_bounds__(256) void step_prep_kernel(
    int S, int SPAD, int cap, const int32_t* __restrict__ pos, const double* __restrict__ w01,
    const double* __restrict__ e_lo, const double* __restrict__ e_hi, int32_t* __restrict__ rows,
    double* __restrict__ sw, int32_t* __restrict__ cnt, int32_t* __restrict__ pairs, int32_t* __restrict__ info,
    double* __restrict__ Dp, double* __restrict__ G, int32_t* __restrict__ permo) {
  __shared__ int perm[kMaxS];
  __shared__ int scan[kMaxS];
  const int ngroups = max((S + 3) / 4, SPAD / 4);
  const int b = blockIdx.x / ngroups;
  const int grp = blockIdx.x - b * ngroups;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int32_t* pb = pos + (size_t)b * S;
  prep_order_lds(S, cap, pb, perm, scan, true);
  if (grp == 0)
    for (int k = tid; k < SPAD; k += blockDim.x) permo[(size_t)b * SPAD + k] = k < S ? perm[k] : S;
  const int r = 4 * grp + tid / kWave;  // this wave's child and position
  if (r < S) prep_child_list(S, cap, pb, w01, rows, sw, cnt, pairs, info, b, r, perm, scan, lane);
  if (r < SPAD) delta_row(S, SPAD, cap, b, r, perm, w01, e_lo, e_hi, Dp, G, lane);
}

// ---------------------------------------------------------------------------
// score: grid = batch * ntiles (1-D, XCD remap, evaluation-major so the
// blocks of one evaluation share its Delta in L2), block = WAVES waves.
// ---------------------------------------------------------------------------
template <int NR, int WAVES>
__global__ __launch_bounds__(WAVES * kWave) void score_factored_kernel(
    int S, int E, int ntiles, int cap, const double* __restrict__ Dp,
    const int32_t* __restrict__ permo,
    const uint64_t* __restrict__ D1w, int nwords, const double* __restrict__ U,
    double* __restrict__ partial, double* __restrict__ cs_out, double* __restrict__ cells,
    double* __restrict__ ow, int remap) {
  constexpr int SPAD = NR * 16;
  constexpr int KC = SPAD < 64 ? SPAD : 64;  // parents per LDS chunk
  constexpr int LDA = KC + 1;                // odd row stride: conflict-free A reads
  constexpr int NS = KC / 4;                 // k-steps per chunk
  constexpr int COLS = WAVES * 16;
  constexpr int WPR = (COLS + 63) / 64 + 1;  // D1 words per parent row a block can touch
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* A = lds;                                       // [SPAD][LDA]
  uint64_t* words = (uint64_t*)(A + SPAD * LDA);         // [SPAD][WPR]
  double* etab = (double*)(words + SPAD * WPR);          // [64] 2^(j/64)
  int* perm_s = (int*)(etab + 64);                       // [SPAD]

  const int work = fxcd_work_index((int)blockIdx.x, (int)gridDim.x, remap);
  const int b = work / ntiles;  // evaluation-major
  const int tile = work - b * ntiles;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int e_blk = tile * COLS;
  const int e_w0 = e_blk + w * 16;
  const int col = lane & 15;
  const int e = e_w0 + col;
  const bool valid = e < E;
  const int ec = valid ? e : E - 1;
  const int word0 = e_blk >> 6;
  const int shift = (e_w0 >> 6) - word0;  // which of the block's words this wave reads
  const int bitpos = (e_w0 & 63) + col;
  const uint32_t diag = lane >= 48 ? 1u : 0u;

  if (tid < 64) etab[tid] = exp2((double)tid * (1.0 / 64.0));
  for (int k = tid; k < SPAD; k += blockDim.x) {
    const int node = permo[(size_t)b * SPAD + k];
    perm_s[k] = node;
    for (int u = 0; u < WPR; ++u) {
      const int wi = word0 + u;
      words[k * WPR + u] = (node < S && wi < nwords) ? D1w[(size_t)node * nwords + wi] : 0ull;
    }
  }

  f64x4 acc[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) acc[r] = f64x4{0.0, 0.0, 0.0, 0.0};

  const double* Db = Dp + (size_t)b * SPAD * SPAD;
  constexpr int NCH = SPAD / KC;
  // the epilogue's U values, loaded once perm_s is visible (the first chunk's
  // barrier) so their latency hides behind the staging and the MFMAs instead
  // of following them (a lone evaluation's launch is a chain of such waits)
  double uv[NR][4];
  double unull = 0.0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int c0 = c * KC;
    __syncthreads();
    if (c == 0) {
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int q = 16 * r + (lane >> 4) + 4 * g;
          uv[r][g] = q < S ? U[(size_t)perm_s[q] * E + ec] : 0.0;
        }
      unull = U[(size_t)S * E + ec];
    }
    // stage Delta[:, c0 .. c0+KC) (coalesced rows); only rows that have
    // parents in this chunk (row q needs p < q, i.e. q > c0)
    for (int k = tid; k < SPAD * KC; k += blockDim.x) {
      const int row = k / KC, kk = k - row * KC;
      if (c0 + kk <= (row | 15))  // only the k range row's block reads
        A[row * LDA + kk] = Db[(size_t)row * SPAD + c0 + kk];
    }
    __syncthreads();
    // B fragments of this chunk: lane holds D1[parent at 4s + lane/16][its effect]
    uint32_t bits[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int p = c0 + 4 * s + (lane >> 4);
      const uint64_t wd = words[p * WPR + shift];
      bits[s] = (uint32_t)((wd >> bitpos) & 1ull);
    }
    // lower-triangular k-loop, fully static: row block r (positions
    // 16r..16r+15) has parents only at positions <= 16r+14, and column
    // 16r+15 holds G (B = 1 there: lanes 48..63 of the diagonal k-step).
    // k-steps outer, row blocks inner: consecutive MFMAs use independent
    // accumulators.
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if (c0 + 4 * s <= 16 * r + 12) {
          const uint32_t bv = (c0 + 4 * s == 16 * r + 12) ? (bits[s] | diag) : bits[s];
          const double a = A[(16 * r + (lane & 15)) * LDA + 4 * s + (lane >> 4)];
          acc[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, (double)bv, acc[r], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: cells, column log-sum-exp, order weights --------------
  // f64 16x16x4 C layout: col = lane & 15, row = (lane >> 4) + 4 * reg
  double cell[NR][4];
  double m = -INFINITY;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int q = 16 * r + (lane >> 4) + 4 * g;
      double v = -INFINITY;
      if (q < S) v = uv[r][g] + acc[r][g];
      cell[r][g] = v;
      m = v > m ? v : m;
    }
  }
  m = m > unull ? m : unull;
  m = fmax(m, __shfl_xor(m, 16, kWave));
  m = fmax(m, __shfl_xor(m, 32, kWave));
  double l = 0.0;
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int g = 0; g < 4; ++g) l += exp_tab(cell[r][g] - m, etab);
  l += __shfl_xor(l, 16, kWave);
  l += __shfl_xor(l, 32, kWave);
  l += exp_tab(unull - m, etab);
  const double cs = m + log(l);
  if (valid && lane < 16 && cs_out) cs_out[(size_t)b * E + e] = cs;
  // per-wave partial over its 16 effects (lanes 0..15 hold one copy each)
  double part = (valid && lane < 16) ? cs : 0.0;
  part = fwave_sum(part);
  const int ntw = ntiles * WAVES;
  if (lane == 0) partial[(size_t)b * ntw + tile * WAVES + w] = part;
  if ((cells || ow) && valid) {
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int q = 16 * r + (lane >> 4) + 4 * g;
        if (q < S) {
          const size_t k = ((size_t)b * (S + 1) + perm_s[q]) * E + e;
          if (cells) cells[k] = cell[r][g];
          if (ow) ow[k] = exp_tab(cell[r][g] - cs, etab);
        }
      }
    if (lane < 16) {
      const size_t k = ((size_t)b * (S + 1) + S) * E + e;
      if (cells) cells[k] = unull;
      if (ow) ow[k] = exp_tab(unull - cs, etab);
    }
  }
}

__global__ void finalize_factored_kernel(int batch, int n, const double* __restrict__ partial,
                                         double* __restrict__ ll) {
  // one wave per evaluation: strided lane sums, then a fixed xor tree --
  // bitwise reproducible, and ~n/64 dependent adds instead of n
  const int b = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  if (b >= batch) return;
  const double s = sum_partials(partial + (size_t)b * n, n, lane);
  if (lane == 0) ll[b] = s;
}

// ---------------------------------------------------------------------------
// pipelined kernel (SPAD <= 64, the C1-C3 shapes): a block owns one
// evaluation x a contiguous range of 16-effect tiles and stages that
// evaluation's Delta (+ G column) and the D1 words of its range ONCE; each
// wave then walks its tiles (t_begin + w, + WAVES, ...) with no further
// barrier; the U rows of the next tile are prefetched.  (On gfx950 the f64
// MFMA pipe and the VALU do not overlap -- tools/ubench/overlap.hip -- so
// the cost is MFMA cycles + VALU cycles, and the epilogue is kept lean.)
// The MFMA accumulators start at U[perm[q]][e] (the C operand), and the G
// column rides in the diagonal k-step, so a cell leaves the MFMA complete.
// Per tile the epilogue keeps sum(m) and prod(l) per column (l in [1, S+1],
// the product as mantissa x 2^exp), so the log of the log-sum-exp runs once
// per wave, not per tile.  ll only: calls that want cs / cells / order
// weights take the chunked kernel.
// ---------------------------------------------------------------------------
template <int NR, int WAVES>
__global__ __launch_bounds__(WAVES * kWave, 2) void score_factored_pipe_kernel(
    int S, int E, int ntiles, int split, const double* __restrict__ Dp,
    const int32_t* __restrict__ permo, const uint64_t* __restrict__ D1w, int nwords,
    const double* __restrict__ U, double* __restrict__ partial, int remap) {
  // block = (evaluation b, tile range [t_begin, t_begin + WAVES * 8))
  constexpr int SPAD = NR * 16;
  constexpr int LDA = SPAD + 2;  // == 2 mod 32: conflict-free b64 A fragments
  constexpr int NS = SPAD / 4;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* etab = lds;                            // [256] 2^(j/256)
  double* A = etab + 256;                        // [SPAD][LDA]
  uint64_t* words = (uint64_t*)(A + SPAD * LDA); // [nwb][SPAD] D1 words, word-major

  const int work = fxcd_work_index((int)blockIdx.x, (int)gridDim.x, remap);
  const int b = work / split;
  const int part = work - b * split;
  const int tpb = kPipeTilesPerWave * WAVES;
  const int t_begin = part * tpb;
  const int t_end = min(ntiles, t_begin + tpb);
  const int w_lo = (t_begin * 16) >> 6;
  const int nwb = t_end > t_begin ? (((t_end * 16 - 1) >> 6) - w_lo + 1) : 0;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int col = lane & 15, rg = lane >> 4;

  const int32_t* pm = permo + (size_t)b * SPAD;
  for (int k = tid; k < 256; k += blockDim.x) etab[k] = exp2((double)k * (1.0 / 256.0));
  for (int k = tid; k < SPAD * nwb; k += blockDim.x) {
    const int u = k / SPAD, p = k - u * SPAD;
    const int node = pm[p];
    const int wi = w_lo + u;
    words[k] = (node < S && wi < nwords) ? D1w[(size_t)node * nwords + wi] : 0ull;
  }
  const double* Db = Dp + (size_t)b * SPAD * SPAD;
  for (int k = tid; k < SPAD * SPAD; k += blockDim.x) {
    const int row = k / SPAD, kk = k - row * SPAD;
    if (kk <= (row | 15)) A[row * LDA + kk] = Db[k];
  }
  // byte offsets of this lane's 16 cells in U: row perm[q] (S = the
  // "attached to nothing" row for padding), column = its effect in the tile
  uint32_t uoff[NR][4];
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      uoff[r][g] = ((uint32_t)pm[16 * r + rg + 4 * g] * (uint32_t)E + col) * 8u;
  const uint32_t unoff = ((uint32_t)S * E + col) * 8u;
  __syncthreads();

  const int ntw = split * WAVES;
  double* part_out = partial + (size_t)b * ntw + part * WAVES + w;
  int t = t_begin + w;
  if (t >= t_end) {
    if (lane == 0) *part_out = 0.0;
    return;
  }

  const uint32_t diag = lane >= 48 ? 1u : 0u;
  const int arow = col * LDA + rg;
  const uint32_t* w32 = (const uint32_t*)words;
  const char* Ub = (const char*)U;

  // U rows of tile tt: the MFMA chain's C-init (prefetched one tile ahead)
  auto load_u = [&](int tt, double (&u)[NR][4], double& un) {
    const char* base = Ub + (size_t)tt * 128;  // 16 effects x 8 B (uniform)
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g) u[r][g] = *(const double*)(base + uoff[r][g]);
    un = *(const double*)(base + unoff);
  };

  double msum = 0.0, lprod = 1.0;
  int lexp = 0;
  double uc[NR][4], unc;
  load_u(t, uc, unc);
  for (; t < t_end; t += WAVES) {
    // ---- cells of tile t: U + G + Delta . D1 on the MFMA (G rides in the
    // diagonal k-step: column 16r+15 of row block r, B = 1 in lanes 48..63)
    f64x4 acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = f64x4{uc[r][0], uc[r][1], uc[r][2], uc[r][3]};
    const double unull = unc;
    {
      const int uidx = ((t * 16) >> 6) - w_lo;
      const int half = (t >> 1) & 1;
      const uint32_t bit = ((t & 1) << 4) + col;
      const uint32_t* wp = w32 + ((size_t)uidx * SPAD + rg) * 2 + half;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint32_t bv = __builtin_amdgcn_ubfe(wp[8 * s], bit, 1);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          if (4 * s <= 16 * r + 12) {
            const uint32_t bb = (4 * s == 16 * r + 12) ? (bv | diag) : bv;
            const double a = A[arow + 16 * r * LDA + 4 * s];
            acc[r] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, (double)bb, acc[r], 0, 0, 0);
          }
        }
      }
    }
    if (t + WAVES < t_end) load_u(t + WAVES, uc, unc);
    // ---- column log-sum-exp (over the NR*16 rows and the null row)
    const bool valid = t * 16 + col < E;
    double m = unull;
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g) m = vmax(m, acc[r][g]);
    m = vmax(m, __shfl_xor(m, 16, kWave));
    m = vmax(m, __shfl_xor(m, 32, kWave));
    double l = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int g = 0; g < 4; ++g) l += exp_lse(acc[r][g] - m, etab);
    l += __shfl_xor(l, 16, kWave);
    l += __shfl_xor(l, 32, kWave);
    l += exp_lse(unull - m, etab);
    // prod(l) kept as mantissa * 2^lexp: branch-free, no overflow
    msum += valid ? m : 0.0;
    lprod *= valid ? l : 1.0;
    lexp += __builtin_amdgcn_frexp_exp(lprod);
    lprod = __builtin_amdgcn_frexp_mant(lprod);
  }
  double v = msum + (log(lprod) + (double)lexp * 0.69314718055994530942);
  v = lane < 16 ? v : 0.0;
  v = fwave_sum(v);
  if (lane == 0) *part_out = v;
}

template <int NR, int WAVES>
hipError_t launch_fact_w(Ctx& c, int batch, int cap, double* d_cs, double* d_cells,
                         double* d_ow, hipStream_t st, int* nparts) {
  constexpr int SPAD = NR * 16;
  constexpr int KC = SPAD < 64 ? SPAD : 64;
  constexpr int COLS = WAVES * 16;
  constexpr int WPR = (COLS + 63) / 64 + 1;
  const int nt = (c.E + COLS - 1) / COLS;
  const size_t lds = (size_t)SPAD * (KC + 1) * 8 + (size_t)SPAD * WPR * 8 + 64 * 8 + SPAD * 4;
  score_factored_kernel<NR, WAVES><<<dim3(nt * batch), WAVES * kWave, lds, st>>>(
      c.S, c.E, nt, cap, c.d_fDp, c.d_fperm, c.d_D1w, c.nwords, (const double*)c.d_U64,
      fpartial(c), d_cs, d_cells, d_ow, c.xcd_remap);
  *nparts = nt * WAVES;
  return hipGetLastError();
}

// partial t of an evaluation is its 16-effect tile t's sum whatever WAVES
// is (sum_partials adds the zero padding of the last block exactly), so any
// WAVES gives the same bits.  Tried: 2 waves (32 effects) per block for the
// fused step of one chain (63 blocks instead of 16): 23 against 18 us per
// launch -- each block stages the whole Delta (32 KB) with a quarter of the
// threads -- so every batch takes 8 waves per block.
template <int NR>
hipError_t launch_fact_t(Ctx& c, int batch, int cap, double* d_cs, double* d_cells,
                         double* d_ow, hipStream_t st, int* nparts) {
  return launch_fact_w<NR, kFactWaves>(c, batch, cap, d_cs, d_cells, d_ow, st, nparts);
}

template <int NR, int WAVES>
hipError_t launch_pipe_t(Ctx& c, int batch, hipStream_t st, int* nparts) {
  constexpr int SPAD = NR * 16;
  const int ntiles = (c.E + 15) / 16;
  const int tpb = kPipeTilesPerWave * WAVES;
  const int split = (ntiles + tpb - 1) / tpb;
  const int nwb_max = (tpb * 16 + 63) / 64 + 1;
  const size_t lds = 256 * 8 + (size_t)SPAD * (SPAD + 2) * 8 + (size_t)nwb_max * SPAD * 8;
  score_factored_pipe_kernel<NR, WAVES><<<dim3(batch * split), WAVES * kWave, lds, st>>>(
      c.S, c.E, ntiles, split, c.d_fDp, c.d_fperm, c.d_D1w, c.nwords, (const double*)c.d_U64,
      fpartial(c), c.xcd_remap);
  *nparts = split * WAVES;
  return hipGetLastError();
}

}  // namespace

int factored_spad(int S) {
  const int nr = (S + 15) / 16;
  const int sizes[] = {1, 2, 4, 8, 16};
  for (int v : sizes)
    if (nr <= v) return v * 16;
  return -1;
}

int factored_partials(const Ctx& c) {
  // chunked: one per wave slot of the 128-effect blocks; pipelined: one per
  // wave of ceil(tiles / (8 * waves)) blocks, waves in {4, 8}
  const int cols = kFactWaves * 16;
  const int nt = (c.E + 15) / 16;
  int n = ((c.E + cols - 1) / cols) * kFactWaves;
  for (int wv : {4, 8}) n = std::max(n, ((nt + kPipeTilesPerWave * wv - 1) / (kPipeTilesPerWave * wv)) * wv);
  return std::max(n, (c.E + 63) / 64);  // the lookup-table kernel: one per word
}

int score_partials(const Ctx& c, int fk) {
  const int nt = (c.E + 15) / 16;
  if (fk == 9 || fk == 15) return c.nwords;                        // launch_score_window
  if (fk == 18 || fk == 19) return (nt + kWideSetT - 1) / kWideSetT;  // launch_i8w_t
  if (fk >= 4) return (nt + 7) / 8;                                 // launch_i8_t / i8o_t / i8l_t / i8s / i8p
  if (fk == 2 || fk == 3) {                                         // launch_pipe_t
    const int wv = fk == 3 ? 8 : 4, tpb = kPipeTilesPerWave * wv;
    return ((nt + tpb - 1) / tpb) * wv;
  }
  const int cols = kFactWaves * 16;                                 // launch_fact_w
  return ((c.E + cols - 1) / cols) * kFactWaves;
}

int resolve_fact_kernel(const Ctx& c, int cap, bool ll_only, double* bound) {
  if (bound) *bound = 0.0;
  if (!c.factored) return -1;
  if (cap >= c.S - 1) cap = 0;  // every predecessor is within the cap: no cap (same bits)
  // the int8 kernels: S <= 64, ll only (they write no cs / cells / order weights)
  const bool i8cap = c.fspad <= 64 && c.d_B8 && ll_only;
  const bool wincap = ll_only && c.win_ok && cap >= 1 && cap <= kWinMaxCap;
  auto bnd = [&](int kind) { return host::fixed_point_bound(kind, c.i8_cexp, c.fx_colsum, c.S, c.E, cap); };
  // the log2 kernel for 64 < S <= 128 (score_i8w_kernel)
  const bool i8wcap = c.fspad == 128 && c.i8w_ok && c.d_B8 && ll_only;
  int fk = c.fact_kernel;
  if (fk == 0) {
    // auto: the capped lookup-table kernel for capped calls; else the fastest
    // int8 kernel whose worst-case ll error (nemo_host.h) stays within
    // err_budget -- log2 fixed point (10; 18 for S > 64), natural units (8),
    // max offset (4) -- else the fp64 MFMA kernels
    if (wincap) fk = 9;
    else if (i8wcap && bnd(host::kFxLog2) <= c.err_budget) fk = 18;
    else if (!i8cap) fk = 1;
    else if (c.i8o_ok && c.i8l_ok && bnd(host::kFxLog2) <= c.err_budget) fk = 10;
    else if (c.i8o_ok && bnd(host::kFxNatural) <= c.err_budget) fk = 8;
    else if (!c.i8o_ok && bnd(host::kFxNatural) <= c.err_budget) fk = 4;
    else fk = 2;
  } else if (fk == 18 || fk == 19) {
    if (!ll_only || c.fspad != 128) fk = 1;
    else if (!i8wcap) return -1;
  } else if (fk == 9 || fk == 15) {
    if (!wincap) return -1;
  } else if (fk == 2 || fk == 3) {
    if (!(ll_only && c.fspad <= 64)) fk = 1;
  } else if (fk >= 4) {
    if (!i8cap) fk = 1;  // an int8 kernel asked for a call it cannot serve: chunked fp64
    else if ((fk == 7 || fk == 8) && !c.i8o_ok) return -1;
    else if (fk >= 10 && !(c.i8o_ok && c.i8l_ok)) return -1;
  }
  if (bound) {
    const bool l2 = fk >= 10 && fk != 15, nat = fk >= 4 && fk <= 8;  // (18: log2, S > 64)
    *bound = l2 ? bnd(host::kFxLog2) : nat ? bnd(host::kFxNatural) : 0.0;
  }
  return fk;
}

hipError_t launch_score_factored(Ctx& c, int batch, int cap, const int32_t* d_pos,
                                 const double* d_w01, double* d_ll, double* d_cs, double* d_cells,
                                 double* d_ow, hipStream_t st, bool prepped, int* defer_np) {
  const int spad = c.fspad;
  if (cap >= c.S - 1) cap = 0;  // every predecessor is within the cap: no cap (same bits)
  const bool ll_only = !d_cs && !d_cells && !d_ow;
  // option fact_kernel: 0 auto (resolve_fact_kernel), 1 chunked, 2 / 3 f64
  // pipelined with 4 / 8 waves per block, 4 / 5 int8 with 4 / 5 digit pairs,
  // 6 int8 (4 pairs) with 8 waves, 7 / 8 int8 with the offset log-sum-exp
  // (4 / 8 waves), 9 / 15 the capped lookup-table kernel (15: its round-1
  // form), 10 / 11 the offset kernel in log2 fixed point (8 / 4 waves; 12: 16
  // waves; 13: register-stationary; 14: 8 waves compiled for 6 waves per
  // SIMD; 10 walks two effect tiles per iteration, 16 is the same kernel with
  // one; 17: 10's walk in persistent blocks that prep the next evaluation
  // during the walk; 18 / 19 the log2 kernel for 64 < S <= 128 with two / one
  // tiles per iteration; 20: 10 as a prep-only and a walk-only launch)
  const int fk = resolve_fact_kernel(c, cap, ll_only, nullptr);
  if (fk < 0) return hipErrorInvalidValue;  // asked for a kernel the staged model does not support
  // every partial buffer (d_fpartial, a redirected part_out) holds
  // factored_partials per evaluation: checked before anything is launched
  const int np_pred = score_partials(c, fk);
  if (np_pred > factored_partials(c)) return hipErrorInvalidValue;
  const bool is_auto = c.fact_kernel == 0;
  const bool win = fk == 9 || fk == 15;
  const bool wide = fk == 18 || fk == 19;
  const bool l2 = fk >= 10 && fk != 15 && !wide;
  const bool i8o = fk == 7 || fk == 8 || l2;
  const bool i8 = fk >= 4 && fk <= 6;
  const bool pipe = fk == 2 || fk == 3;
  hipError_t err = hipSuccess;
  if (!i8 && !i8o && !win && !wide && !prepped) {  // the int8 and lookup-table kernels derive their inputs themselves
    prep_factored_kernel<<<batch * (spad / 4), 256, 0, st>>>(c.S, spad, cap, d_pos, d_w01, c.d_elo,
                                                             c.d_ehi, c.d_fDp, c.d_fG, c.d_fperm);
    err = hipGetLastError();
  }
  if (err != hipSuccess) return err;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c.timing && c.timing_kernel == 0 && c.ev_used + 2 <= c.ev_pool.size()) {
    e0 = c.ev_pool[c.ev_used++];
    e1 = c.ev_pool[c.ev_used++];
    { hipError_t re = hipEventRecord(e0, st); if (re != hipSuccess) return re; }
  }
  int np = 0;
  bool finalized = false;
  if (win) {
    err = launch_score_window(c, batch, cap, d_pos, d_w01, d_ll, st, &np, &finalized, fk == 15);
  } else if (wide) {
    err = launch_score_i8w(c, batch, cap, d_pos, d_w01, d_ll, fk == 18, st, &np, &finalized);
  } else if (i8o) {
    // 7 / 8: offset log-sum-exp with 4 / 8 waves per block; 10 (auto's l2
    // choice): 8 waves, two effect tiles per iteration; 11: 4 waves; 12: 16;
    // 16: 8 waves, one tile per iteration
    const int waves = fk == 20 ? -20 : fk == 17 ? -3 : fk == 13 ? 0 : fk == 14 ? -8 : fk == 16 ? 8 : fk == 12 ? 16
                    : (fk == 7 || fk == 11) ? 4 : fk == 10 ? -2 : 8;
    err = launch_score_i8o(c, batch, cap, d_pos, d_w01, d_ll, waves, l2, st, &np, &finalized);
  } else if (i8) {
    // auto: 4 waves per block for large batches, 8 (fewer splits) below
    const int waves = fk == 6 ? 8 : (fk == 4 && is_auto && batch < 384 ? 8 : 4);
    err = launch_score_i8(c, batch, cap, d_pos, d_w01, d_ll, fk == 5 ? 5 : 4, waves, st, &np,
                          &finalized);
  } else if (pipe) {
    const bool w8 = fk == 3;
    switch (spad / 16) {
#define NEMO_PIPE(NRV)                                                               \
  case NRV:                                                                          \
    err = w8 ? launch_pipe_t<NRV, 8>(c, batch, st, &np)                              \
             : launch_pipe_t<NRV, 4>(c, batch, st, &np);                             \
    break;
      NEMO_PIPE(1)
      NEMO_PIPE(2)
      NEMO_PIPE(4)
#undef NEMO_PIPE
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (spad / 16) {
      case 1: err = launch_fact_t<1>(c, batch, cap, d_cs, d_cells, d_ow, st, &np); break;
      case 2: err = launch_fact_t<2>(c, batch, cap, d_cs, d_cells, d_ow, st, &np); break;
      case 4: err = launch_fact_t<4>(c, batch, cap, d_cs, d_cells, d_ow, st, &np); break;
      case 8: err = launch_fact_t<8>(c, batch, cap, d_cs, d_cells, d_ow, st, &np); break;
      case 16: err = launch_fact_t<16>(c, batch, cap, d_cs, d_cells, d_ow, st, &np); break;
      default: return hipErrorInvalidValue;
    }
  }
  if (err != hipSuccess) return err;
  if (np != np_pred) return hipErrorUnknown;  // score_partials out of step with a launcher: a build bug
  if (e1) {
    (void)hipEventRecord(e1, st);
    c.launches++;
  }
  // per-evaluation partials, summed in a fixed order
  if (defer_np) *defer_np = finalized ? 0 : np;
  else if (!finalized)
    finalize_factored_kernel<<<(batch + 3) / 4, 256, 0, st>>>(batch, np, fpartial(c), d_ll);
  return hipGetLastError();
}

hipError_t launch_step_prep(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                            int32_t* d_info, hipStream_t st) {
  const int spad = c.fspad;
  if (cap >= c.S - 1) cap = 0;  // as launch_score_factored (same lists: a cap >= S - 1 cuts nothing)
  const int ngroups = std::max((c.S + 3) / 4, spad / 4);
  step_prep_kernel<<<batch * ngroups, 256, 0, st>>>(c.S, spad, cap, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_rows,
                                                    c.d_sw, c.d_cnt, c.d_pairs, d_info, c.d_fDp, c.d_fG,
                                                    c.d_fperm);
  return hipGetLastError();
}

}  // namespace nemo
