// nemo_window.hip -- order scores under a parent-set cap (BASELINE config C5:
// S = 128, E = 5000, cap 6): a banded lookup-table kernel.
//
// With a cap, child q (in ORDER position) has parents q-1 .. q-cap only
// (the build-defined cap: the last <= cap entries of the
// order prefix).  For every table nem.py builds, parent j's log factor
// log(1 - w + w e^{T[i][j][e]}) takes one of two values per (i, j), picked by
// the bit D1[j][e], and U[i][e] - U[S][e] takes one of two values picked by
// D1[i][e] (stage_window checks both).  So x = cell[q][e] - U[S][e] is a
// function of 7 bits: node pi(q)'s own bit and those of the rows at
// q-1 .. q-6, and so is exp(x).  Per evaluation the block tabulates it in LDS
// as a product of two tables per row,
//     A[q][m] = exp(U'(bit 0) + sum_{d=1..3} f_d(bit d))   (16 entries),
//     B[q][m] = exp(sum_{d=4..6} f_d(bit d))                (8 entries),
// and a lane (one effect) walks the rows in order with a shift register of
// bits h: s += A[q][h & 15] * B[q][(h >> 4) & 7] -- two LDS reads and one FMA
// per cell, no exp, instead of a K = S contraction of which only cap terms
// are nonzero.  The column log-sum-exp is offset by the null row (as in
// score_i8o_kernel): cs[e] = U[S][e] + log(1 + sum_q exp(x_q)); staging bounds
// every partial sum of a cell by 690, so no entry overflows or is subnormal.
//
// Reference: compute_cell_ratios + calculate_ll, nem_order_mcmc.py:79-93;
// utils.compute_ll, utils.py:84-94.
#include <math.h>

#include <algorithm>
#include <cmath>
#include <functional>

#include "nemo_internal.h"

namespace nemo {
namespace {

constexpr int kWinWaves = 8;
constexpr int kWinLo = 16;             // entries over (self, parents 1..3)
constexpr int kWinRow = kWinLo + 8;    // + entries over parents 4..6

// LDS layout: [S][6] double2 factor scratch; [S][kWinRow] tables; per wave
// the current word of every row as two dword arrays of odd stride (S | 1);
// [S] int perm
__host__ __device__ __forceinline__ size_t win_lds_bytes(int S, int waves) {
  return ((size_t)12 * S + (size_t)kWinRow * S) * 8 + (size_t)waves * 8 * (S | 1) + (size_t)S * 4;
}

// block = (evaluation b, part of its 64-effect words); each wave walks whole
// words (all S rows of 64 effects) and writes one partial per word
template <int WAVES>
__global__ __launch_bounds__(WAVES * kWave) void score_window_kernel(
    int S, int E, int nwords, int cap, int split, const int32_t* __restrict__ pos,
    const double* __restrict__ w01, const double* __restrict__ e_lo, const double* __restrict__ e_hi,
    const uint64_t* __restrict__ D1w, const double* __restrict__ uw, const double* __restrict__ nullw,
    double* __restrict__ partial, double* __restrict__ ll_out) {
  extern __shared__ __attribute__((aligned(16))) double ldsw[];
  const int rs = S | 1;
  double2* fac = (double2*)ldsw;                               // [S][6] (f at lo, f at hi)
  double* lut = ldsw + (size_t)12 * S;                         // [S][kWinRow]
  uint32_t* rowbits = (uint32_t*)(lut + (size_t)S * kWinRow);  // [WAVES][2][rs]
  int* perm = (int*)(rowbits + (size_t)WAVES * 2 * rs);        // [S]

  const int b = blockIdx.x / split;
  const int part = blockIdx.x - b * split;
  const int wpb = (nwords + split - 1) / split;
  const int wbeg = part * wpb, wend = min(nwords, wbeg + wpb);
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int nt = blockDim.x;

  for (int k = tid; k < S; k += nt) perm[k] = 0;
  __syncthreads();
  for (int i = tid; i < S; i += nt) {
    int p = pos[(size_t)b * S + i];
    p = p < 0 ? 0 : (p >= S ? S - 1 : p);  // malformed input must not fault (the ABI validates)
    perm[p] = i;
  }
  __syncthreads();
  // the two log factors of parent q-d of child q (0 past the cap / the order start)
  const double* wb = w01 + (size_t)b * S * S;
  for (int k = tid; k < 6 * S; k += nt) {
    const int q = k / 6, d = k - 6 * q + 1;
    double flo = 0.0, fhi = 0.0;
    if (d <= cap && q >= d) {
      const int i = perm[q], j = perm[q - d];
      const double s = wb[(size_t)i * S + j];
      flo = log(fma(s, e_lo[j] - 1.0, 1.0));
      fhi = log(fma(s, e_hi[j] - 1.0, 1.0));
    }
    fac[k] = double2{flo, fhi};
  }
  __syncthreads();
  for (int k = tid; k < kWinRow * S; k += nt) {
    const int q = k / kWinRow, m = k - kWinRow * q;
    const double2* f = fac + 6 * q;
    double v;
    if (m < kWinLo) {
      v = uw[2 * perm[q] + (m & 1)];
#pragma unroll
      for (int d = 1; d <= 3; ++d) v += (m >> d) & 1 ? f[d - 1].y : f[d - 1].x;
    } else {
      const int mm = m - kWinLo;
      v = mm & 1 ? f[3].y : f[3].x;
      v += (mm >> 1) & 1 ? f[4].y : f[4].x;
      v += (mm >> 2) & 1 ? f[5].y : f[5].x;
    }
    lut[k] = exp(v);
  }
  __syncthreads();

  // lanes 0-31 read the low dwords of the row words, lanes 32-63 the high
  // ones: two broadcast addresses per read, in different banks (odd stride)
  uint32_t* mine = rowbits + (size_t)w * 2 * rs;
  const uint32_t* half = mine + (lane >> 5) * rs;
  const uint32_t bit = lane & 31;
  for (int word = wbeg + w; word < wend; word += WAVES) {
    // this word of every row, in order position; the wave reads back what it
    // wrote (LDS operations of one wave complete in order)
    for (int q = lane; q < S; q += kWave) {
      const uint64_t v = D1w[(size_t)perm[q] * nwords + word];
      mine[q] = (uint32_t)v;
      mine[rs + q] = (uint32_t)(v >> 32);
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t h = 0;
    double s = 0.0;
    const double* lq = lut;
#pragma unroll 4
    for (int q = 0; q < S; ++q, lq += kWinRow) {
      h = (h << 1) | ((half[q] >> bit) & 1u);
      s = fma(lq[h & 15], lq[kWinLo + ((h >> 4) & 7)], s);
    }
    double v = 64 * word + lane < E ? log1p(s) : 0.0;  // 1 = e^0 of the null row
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
    if (lane == 0) partial[(size_t)b * nwords + word] = nullw[word] + v;
    __builtin_amdgcn_wave_barrier();
  }
  if (split == 1) {
    __syncthreads();
    if (w == 0) {
      const double v = sum_partials(partial + (size_t)b * nwords, nwords, lane);
      if (lane == 0) ll_out[b] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// score_window2_kernel: the same tables, walked from registers.
//
// Per 64-effect word a wave loads the D1 words of its rows in ORDER position
// (lane r: row r, r + 64, ...) and transposes each 64 x 64 bit block across
// the lanes (one v_permlane32_swap, then five butterfly stages of a partner
// fetch, a rotate and a bit select), so lane e holds R = the bits of effect e
// over the order positions, 32 rows per dword.  The window of row q -- the
// bits of rows q-6 .. q -- is then one funnel shift of two of those dwords:
//     X_q = (R >> (q - 6)) (32 bits),  bits 3..6 = rows q-3 .. q,
// so X_q & 0x78 is directly the byte offset of row q's A entry (own bit and
// parents 1-3, 16 entries).  Parents 4-6 of row q are rows q-6 .. q-4, the
// low three bits of row q-3's A index: row q's second table B' is stored with
// 16 entries (B'[m] = B[m & 7]) and read at row q-3's A offset.  Row q's A
// sits at 128 q, its B' at kB0 + 128 q; the rows run in 32-row groups,
// unrolled, so every row offset is an instruction immediate and a cell costs
// one shift, one bit select (group base), two LDS reads and one FMA (against
// ~9 VALU and three LDS reads in score_window_kernel, which re-extracts each
// row's bit from an LDS word).
// Tables are products of the per-parent factors 1 - w + w e^{T} (the terms
// whose logs the cell sums) and e^{U'}: no log or exp per entry.
// ---------------------------------------------------------------------------
constexpr int kWin2Row = 256;  // bytes of tables per row: A[16] and B'[16], in two regions
#ifndef NEMO_WIN2_OCC
#define NEMO_WIN2_OCC 6
#endif

__host__ __device__ __forceinline__ size_t win2_lds_bytes(int S) {
  const int rows = 64 * ((S + 63) / 64);
  return (size_t)rows * kWin2Row + 64 + 128 * 16 + (size_t)S * 4;
}

__device__ __forceinline__ double lds_f64(uint32_t addr) {
  return *(const __attribute__((address_space(3))) double*)(size_t)addr;
}

// value of lane ^ D (D < 32) within 32-lane halves
template <int D>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
  if constexpr (D == 1) return __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  else if constexpr (D == 2) return __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
  else if constexpr (D == 8) return __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  else return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (D << 10));  // bit mode, xor D
}

// one butterfly stage of the 32 x 32 transpose (lane = row, bit = column):
// the lane with bit D clear keeps its columns with bit D clear and takes the
// partner's (shifted up by D), the other one the reverse (tests/test_numerics.py
// restates it)
template <int D>
__device__ __forceinline__ uint32_t tr_stage(uint32_t x, uint32_t sh, uint32_t m) {
  const uint32_t p = lane_xor<D>(x);
  const uint32_t rot = __builtin_amdgcn_alignbit(p, p, sh);
  return (x & m) | (rot & ~m);
}

template <int NB, int WAVES>
__global__ __launch_bounds__(WAVES * kWave, NEMO_WIN2_OCC) void score_window2_kernel(
    int S, int E, int nwords, int cap, int split, const int32_t* __restrict__ pos,
    const double* __restrict__ w01, const double* __restrict__ e_lo, const double* __restrict__ e_hi,
    const uint64_t* __restrict__ D1w, const double* __restrict__ uw, const double* __restrict__ nullw,
    double* __restrict__ partial, double* __restrict__ ll_out) {
  constexpr int ROWS = 64 * NB;
  // B' region: 64 B past the A rows, so no A / B' read pair is a multiple of
  // 512 B apart (the compiler would fuse it into ds_read2st64_b64, which moves
  // 128 B/clk against 256 for two ds_read_b64)
  constexpr int kB0 = ROWS * 128 + 64;
  extern __shared__ __attribute__((aligned(16))) double ldsw[];
  double* lut = ldsw;  // at LDS address 0: A [ROWS][16], then B' [ROWS][16] from kB0
  double2* ltab = (double2*)(ldsw + (size_t)ROWS * 32 + 8);  // log_fast's table
  int* perm = (int*)(ltab + 128);                            // [S] node at each order position

  const int b = blockIdx.x / split;
  const int part = blockIdx.x - b * split;
  const int wpb = (nwords + split - 1) / split;
  const int wbeg = part * wpb, wend = min(nwords, wbeg + wpb);
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int nt = blockDim.x;

  for (int k = tid; k < S; k += nt) perm[k] = 0;
  fill_log_table(ltab, tid, nt);
  __syncthreads();
  for (int i = tid; i < S; i += nt) {
    int p = pos[(size_t)b * S + i];
    p = p < 0 ? 0 : (p >= S ? S - 1 : p);  // malformed input must not fault (the ABI validates)
    perm[p] = i;
  }
  __syncthreads();
  // the factors of every row: y[q][d] = (1 - w + w e^{lo}, 1 - w + w e^{hi})
  // of parent q-d (d = 1..6; (1, 1) past the cap / the order start), y[q][0]
  // = e^{U'} at the row's own bit 0 / 1; one thread per (row, d).  They are
  // staged in row q's B' slot (112 of its 128 bytes), which is written last.
  double2* ysc = (double2*)(lut + kB0 / 8);
  const double* wb = w01 + (size_t)b * S * S;
  for (int k = tid; k < 7 * S; k += nt) {
    const int q = k / 7, d = k - 7 * q;
    const int i = perm[q];
    double2 f = double2{1.0, 1.0};
    if (d == 0) {
      f = double2{exp(uw[2 * i]), exp(uw[2 * i + 1])};
    } else if (d <= cap && q >= d) {
      const int j = perm[q - d];
      const double sw = wb[(size_t)i * S + j];
      f = double2{fma(sw, e_lo[j] - 1.0, 1.0), fma(sw, e_hi[j] - 1.0, 1.0)};
    }
    ysc[8 * q + d] = f;
  }
  __syncthreads();
  // the tables, one thread per entry (consecutive lanes, consecutive entries):
  // A index bits 0..3 = rows q-3, q-2, q-1, q; B' index bits 0..2 = rows
  // q-6, q-5, q-4 (bit 3 ignored); padding rows 0 (A = 0 adds nothing).  The
  // B' entries wait in registers until every thread has read its factors.
  constexpr int kEpt = 32 * ROWS / (WAVES * kWave);  // entries per thread
  double bv[kEpt];
#pragma unroll
  for (int e = 0; e < kEpt; ++e) {
    const int k = tid + e * WAVES * kWave;
    const int q = k >> 5, m = k & 15;
    const bool isb = (k & 16) != 0;
    double v = 0.0;
    if (q < S) {
      const double2* y = ysc + 8 * q;
      auto pick = [&](int d, int bit) { return bit ? y[d].y : y[d].x; };
      v = isb ? (pick(4, (m >> 2) & 1) * pick(5, (m >> 1) & 1)) * pick(6, m & 1)
              : ((pick(0, (m >> 3) & 1) * pick(1, (m >> 2) & 1)) * pick(2, (m >> 1) & 1)) * pick(3, m & 1);
    }
    if (!isb) lut[16 * q + m] = v;
    bv[e] = v;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kEpt; ++e) {
    const int k = tid + e * WAVES * kWave;
    if (k & 16) lut[kB0 / 8 + 16 * (k >> 5) + (k & 15)] = bv[e];
  }
  __syncthreads();

  // per-lane constants of the five butterfly stages (D = 16 .. 1)
  constexpr uint32_t kMlo[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
  uint32_t tsh[5], tm[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int d = 16 >> k;
    const bool up = (lane & d) != 0;
    tsh[k] = up ? (uint32_t)d : (uint32_t)(32 - d);
    tm[k] = up ? ~kMlo[k] : kMlo[k];
  }
  for (int word = wbeg + w; word < wend; word += WAVES) {
    uint32_t R[2 * NB];
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
      const int r = 64 * blk + lane;
      const uint64_t v = r < S ? D1w[(size_t)perm[r] * nwords + word] : 0ull;
      uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
      // lanes 0-31: high dwords <-> lanes 32-63: low dwords (the off-diagonal 32 x 32 blocks)
      const auto sw = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
      lo = sw[0];
      hi = sw[1];
      lo = tr_stage<16>(lo, tsh[0], tm[0]);
      hi = tr_stage<16>(hi, tsh[0], tm[0]);
      lo = tr_stage<8>(lo, tsh[1], tm[1]);
      hi = tr_stage<8>(hi, tsh[1], tm[1]);
      lo = tr_stage<4>(lo, tsh[2], tm[2]);
      hi = tr_stage<4>(hi, tsh[2], tm[2]);
      lo = tr_stage<2>(lo, tsh[3], tm[3]);
      hi = tr_stage<2>(hi, tsh[3], tm[3]);
      lo = tr_stage<1>(lo, tsh[4], tm[4]);
      hi = tr_stage<1>(hi, tsh[4], tm[4]);
      R[2 * blk] = lo;      // rows 64 blk + 0..31 of effect 64 word + lane
      R[2 * blk + 1] = hi;  // rows 64 blk + 32..63
    }
    // rows in 32-row groups (a runtime loop, so the scheduler sees one group
    // at a time); av = (X & 0x78) | 4096 g, so A(q) is at av + 128 t and
    // B'(q) at av(q-3) + kB0 + 128 t(q-3) + 384 (t = row within its group)
    double s0 = 0.0, s1 = 0.0;
    uint32_t ap0 = (uint32_t)-4096, ap1 = ap0, ap2 = ap0;  // rows -3..-1: group -1, index 0
    uint32_t Rp = 0u, Rc = R[0];
#pragma unroll 1
    for (int g = 0; g < 2 * NB; ++g) {
      // the group base in a VGPR (opaque), so each row's offset is one bit
      // select (X & 0x78) | (gv & ~0x78) instead of an AND and an add
      uint32_t gv = (uint32_t)g << 12;
      asm volatile("" : "+v"(gv));
      uint32_t av[32];
      // 8 rows at a time: 16 reads in flight, then the FMAs
#pragma unroll
      for (int t0 = 0; t0 < 32; t0 += 8) {
        double A[8], B[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int t = t0 + u;
          const uint32_t X = t >= 6 ? Rc >> (t - 6) : __builtin_amdgcn_alignbit(Rc, Rp, t + 26);
          av[t] = (X & 0x78u) | (gv & ~0x78u);
          const uint32_t aq3 = t >= 3 ? av[t >= 3 ? t - 3 : 0] : (t == 0 ? ap0 : (t == 1 ? ap1 : ap2));
          A[u] = lds_f64(av[t] + (uint32_t)(t * 128));
          // aq3 holds row q-3's group base and index only: add its row within
          // that group (t - 3, or t + 29 for the previous group) and 3 rows
          B[u] = lds_f64(aq3 + (uint32_t)(kB0 + 128 * (t >= 3 ? t - 3 : t + 29) + 384));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (u & 1) s1 = fma(A[u], B[u], s1);
          else s0 = fma(A[u], B[u], s0);
        }
      }
      ap0 = av[29];
      ap1 = av[30];
      ap2 = av[31];
      Rp = Rc;
      // next group's dword (R shifts down one: a compile-time rotation)
#pragma unroll
      for (int k = 0; k + 1 < 2 * NB; ++k) R[k] = R[k + 1];
      Rc = R[0];
    }
    double v = 64 * word + lane < E ? log_fast(1.0 + (s0 + s1), ltab) : 0.0;  // 1 = e^0 of the null row
    v = wsum_dpp(v);  // DPP + permlane swaps: no ds_bpermute on the LDS this kernel is bound by
    if (lane == 0) partial[(size_t)b * nwords + word] = nullw[word] + v;
  }
  if (split == 1) {
    __syncthreads();
    if (w == 0) {
      const double v = sum_partials(partial + (size_t)b * nwords, nwords, lane);
      if (lane == 0) ll_out[b] = v;
    }
  }
}

template <int NB>
hipError_t launch_window2_t(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                            double* d_ll, hipStream_t st, int split) {
  const size_t lds = win2_lds_bytes(c.S);
  if (lds > 65536) {  // S > 128: past the default 64 KB of dynamic LDS (gfx950 has 160 KB)
    hipError_t ae = hipFuncSetAttribute((const void*)score_window2_kernel<NB, kWinWaves>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (ae != hipSuccess) return ae;
  }
  score_window2_kernel<NB, kWinWaves><<<dim3(batch * split), kWinWaves * kWave, lds, st>>>(
      c.S, c.E, c.nwords, cap, split, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_D1w, c.d_wuw, c.d_wnull,
      fpartial(c), d_ll);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_score_window(Ctx& c, int batch, int cap, const int32_t* d_pos, const double* d_w01,
                               double* d_ll, hipStream_t st, int* nparts, bool* finalized, bool walk_lds) {
  if (!c.win_ok || cap < 1 || cap > kWinMaxCap || c.S > kWinMaxS) return hipErrorInvalidValue;
  const int nwords = c.nwords;
  if (!walk_lds) {
    // 3 blocks per CU (LDS at S = 128, 80 VGPRs)
    int split = (768 + batch - 1) / batch;
    split = std::max(1, std::min(split, (nwords + kWinWaves - 1) / kWinWaves));
    hipError_t err;
    switch ((c.S + 63) / 64) {
      case 1: err = launch_window2_t<1>(c, batch, cap, d_pos, d_w01, d_ll, st, split); break;
      case 2: err = launch_window2_t<2>(c, batch, cap, d_pos, d_w01, d_ll, st, split); break;
      case 3: err = launch_window2_t<3>(c, batch, cap, d_pos, d_w01, d_ll, st, split); break;
      case 4: err = launch_window2_t<4>(c, batch, cap, d_pos, d_w01, d_ll, st, split); break;
      default: return hipErrorInvalidValue;
    }
    *nparts = nwords;
    *finalized = split == 1;
    return err;
  }
  // enough blocks to fill 256 CUs (LDS allows 3 per CU at S = 128); every
  // word's partial is the same whatever the split, so bits do not depend on it
  const int slots = 768;
  int split = (slots + batch - 1) / batch;
  split = std::max(1, std::min(split, (nwords + kWinWaves - 1) / kWinWaves));
  const size_t lds1 = win_lds_bytes(c.S, kWinWaves);
  if (lds1 > 65536) {  // past the default 64 KB of dynamic LDS
    hipError_t ae = hipFuncSetAttribute((const void*)score_window_kernel<kWinWaves>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1);
    if (ae != hipSuccess) return ae;
  }
  score_window_kernel<kWinWaves><<<dim3(batch * split), kWinWaves * kWave, lds1, st>>>(
      c.S, c.E, nwords, cap, split, d_pos, d_w01, c.d_elo, c.d_ehi, c.d_D1w, c.d_wuw, c.d_wnull,
      fpartial(c), d_ll);
  *nparts = nwords;
  *finalized = split == 1;
  return hipGetLastError();
}

// staging of score_window_kernel (after the factored form): U' = U - U[S]
// two-valued per row, picked by the row's own D1 bit (within 1e-11, as
// stage_i8o's diagonal form), the per-word sums of U[S] (left fold), and the
// range check that keeps every table entry and the column sums finite and
// normal for any order, any cap <= 6 and any weights in [0, 1]
hipError_t stage_window(Ctx& c, const std::vector<double>& elo, const std::vector<double>& ehi,
                        const std::vector<uint64_t>& d1) {
  c.win_ok = false;
  for (void** p : {(void**)&c.d_wuw, (void**)&c.d_wnull})
    if (*p) {
      hipError_t fe = hipFree(*p);
      *p = nullptr;
      if (fe != hipSuccess) return fe;
    }
  const int S = c.S, E = c.E, nwords = c.nwords;
  if (S > kWinMaxS || S < 1 || !c.d_D1w) return hipSuccess;
  hipError_t err = hipStreamSynchronize(c.stream);
  if (err != hipSuccess) return err;
  std::vector<double> U((size_t)(S + 1) * E);
  if ((err = copy_sync(c, U.data(), c.d_U64, U.size() * 8, hipMemcpyDeviceToHost)) != hipSuccess) return err;
  const double* un = U.data() + (size_t)S * E;
  std::vector<double> uw(2 * (size_t)S, 0.0);
  double umin = 0.0, umax = 0.0;
  for (int i = 0; i < S; ++i) {
    bool have[2] = {false, false};
    for (int e = 0; e < E; ++e) {
      const int bit = (int)((d1[(size_t)i * nwords + e / 64] >> (e % 64)) & 1ull);
      const double v = U[(size_t)i * E + e] - un[e];
      if (!std::isfinite(v)) return hipSuccess;
      if (!have[bit]) {
        uw[2 * i + bit] = v;
        have[bit] = true;
      } else if (fabs(v - uw[2 * i + bit]) > 1e-11) {
        return hipSuccess;  // not two-valued: the general kernels only
      }
    }
    if (!have[0]) uw[2 * i] = uw[2 * i + 1];
    if (!have[1]) uw[2 * i + 1] = uw[2 * i];
    umin = std::min({umin, uw[2 * i], uw[2 * i + 1]});
    umax = std::max({umax, uw[2 * i], uw[2 * i + 1]});
  }
  // each parent's log factor lies between 0 and its table value; at most
  // kWinMaxCap parents per child, so every partial sum of a cell is bounded too
  std::vector<double> neg(S), posv(S);
  for (int j = 0; j < S; ++j) {
    const double lo = log(elo[j]), hi = log(ehi[j]);
    neg[j] = std::min(0.0, std::min(lo, hi));
    posv[j] = std::max(0.0, std::max(lo, hi));
  }
  std::sort(neg.begin(), neg.end());
  std::sort(posv.begin(), posv.end(), std::greater<double>());
  double fmin = 0.0, fmax = 0.0;
  for (int k = 0; k < std::min(S, kWinMaxCap); ++k) {
    fmin += neg[k];
    fmax += posv[k];
  }
  if (!(std::isfinite(fmin) && std::isfinite(fmax) && umin + fmin >= -690.0 && umax + fmax <= 690.0))
    return hipSuccess;
  std::vector<double> nw(nwords, 0.0);
  for (int k = 0; k < nwords; ++k) {
    double acc = 0.0;
    for (int e = 64 * k; e < std::min(E, 64 * k + 64); ++e) acc += un[e];
    nw[k] = acc;
  }
  if ((err = hipMalloc((void**)&c.d_wuw, uw.size() * 8)) != hipSuccess) return err;
  if ((err = hipMalloc((void**)&c.d_wnull, nw.size() * 8)) != hipSuccess) return err;
  if ((err = copy_sync(c, c.d_wuw, uw.data(), uw.size() * 8, hipMemcpyHostToDevice)) != hipSuccess) return err;
  if ((err = copy_sync(c, c.d_wnull, nw.data(), nw.size() * 8, hipMemcpyHostToDevice)) != hipSuccess) return err;
  c.win_ok = true;
  return hipSuccess;
}

}  // namespace nemo
