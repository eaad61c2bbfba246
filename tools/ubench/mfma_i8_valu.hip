// mfma_i8_valu.hip -- VERDICT r5 item 5: do score_i8l_kernel's matrix pipe and its VALU
// epilogue overlap on one SIMD?  i8 MFMAs (v_mfma_i32_16x16x64_i8, the headline's
// contraction) against the epilogue's per-cell VALU mix (integer field work, a cvt, three
// fp64 FMAs: DESIGN.md 3.1h's 11 per cell), in one wave or in separate waves of one SIMD,
// with and without s_setprio.  SIMD cycles per iteration against each side alone.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench/mfma_i8_valu.hip -o tools/ubench/mfma_i8_valu
#include <hip/hip_runtime.h>
#include <stdio.h>

using i32x4 = __attribute__((ext_vector_type(4))) int;

// one cell of the epilogue: T0, the table address, slice 4's C-init, R, cvt, the degree-2
// series, an exponent insert, the accumulation
__device__ __forceinline__ void cell(int a0, int a1, int l0, int l1, double& acc, int& addr_acc) {
#pragma clang fp contract(off)
  const int t0 = (a0 << 12) + a1;
  const int addr = (t0 >> 6) & 0x3ff8;
  const int c4 = (t0 & 511) << 6;
  const int r = (l0 << 12) + l1 + c4;
  const double f = (double)r;
  double p = __builtin_fma(f, 1.0e-22, 0.5);
  p = __builtin_fma(p, f, 1.0);
  const unsigned hi = (unsigned)(t0 & ~511) ^ (unsigned)addr;
  acc = __builtin_fma(p, (double)(hi & 0xff), acc);
  addr_acc ^= addr;
}

// MODE 1 MFMA only; 2 VALU only; 3 both in every wave; 4 half the waves MFMA, half VALU, one
// of each per SIMD (a block's waves w and w + 4 share a SIMD); 5 = 4 with s_setprio 3 in the
// MFMA waves; 6 = 4 with s_setprio 3 in the VALU waves.  Each role runs its own loop, so no
// wave carries the other role's registers (round 6's first cut kept both live and spilled).
template <int NM>
__device__ __forceinline__ void mfma_loop(int iters, int lane, int seed, double& s) {
  i32x4 a = {lane + seed, lane * 3, lane ^ 7, 1}, b = {seed, 2, lane, 5};
  i32x4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < NM; ++k) acc[k & 3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[k & 3], 0, 0, 0);
  }
  s += acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
}

template <int NC>
__device__ __forceinline__ void valu_loop(int iters, int lane, int seed, double& s) {
  // independent cells (each its own accumulators): the VALU side is issue-bound, as the
  // headline's epilogue over its 64-lane row blocks, not a dependent chain
  int x[NC], ia[NC];
  double da[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) x[c] = lane * (c + 1) + seed, ia[c] = 0, da[c] = 0.0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < NC; ++c) cell(x[c], x[c] ^ 5, it, x[c] + it, da[c], ia[c]);
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) s += da[c] + ia[c];
}

template <int NM, int NC>
__device__ __forceinline__ void both_loop(int iters, int lane, int seed, double& s) {
  i32x4 a = {lane + seed, lane * 3, lane ^ 7, 1}, b = {seed, 2, lane, 5};
  i32x4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  int x[NC], ia[NC];
  double da[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) x[c] = lane * (c + 1) + seed, ia[c] = 0, da[c] = 0.0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < NM; ++k) acc[k & 3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[k & 3], 0, 0, 0);
#pragma unroll
    for (int c = 0; c < NC; ++c) cell(x[c], x[c] ^ 5, it, x[c] + it, da[c], ia[c]);
  }
  s += acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
#pragma unroll
  for (int c = 0; c < NC; ++c) s += da[c] + ia[c];
}

template <int MODE, int NM, int NC>
__global__ __launch_bounds__(512) void kern(int iters, int seed, double* out) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / 64);
  const int lane = threadIdx.x & 63;
  const bool mfma_wave = ((w >> 2) & 1) == 0;
  double s = 0.0;
  if (MODE == 1) mfma_loop<NM>(iters, lane, seed, s);
  else if (MODE == 2) valu_loop<NC>(iters, lane, seed, s);
  else if (MODE == 3) both_loop<NM, NC>(iters, lane, seed, s);
  else if (mfma_wave) {
    if (MODE == 5) __builtin_amdgcn_s_setprio(3);
    mfma_loop<NM>(2 * iters, lane, seed, s);
  } else {
    if (MODE == 6) __builtin_amdgcn_s_setprio(3);
    valu_loop<NC>(2 * iters, lane, seed, s);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int NM, int NC>
double run(const char* name, int threads) {
  double* out;
  const int blocks = 256;
  (void)hipMalloc(&out, (size_t)blocks * threads * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 2000;
  kern<MODE, NM, NC><<<blocks, threads>>>(iters, 1, out);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) kern<MODE, NM, NC><<<blocks, threads>>>(iters, r, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  // one block per CU: threads / 256 waves per SIMD
  const double cyc = ms * 1e-3 * 2.4e9 / iters;
  printf("%-44s waves/SIMD %d: %7.3f ms  %7.1f SIMD-cycles/iter\n", name, threads / 256, ms, cyc);
  (void)hipFree(out);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return cyc;
}

template <int NM, int NC>
void suite() {
  printf("-- %d MFMA and %d epilogue cells per wave-iteration (the headline walk: ~8 cells per MFMA)\n", NM, NC);
  // 2 waves per SIMD throughout: the split modes give each SIMD one MFMA wave and one VALU wave
  const double m = run<1, NM, NC>("MFMA only (2 MFMA waves)", 512);
  const double v = run<2, NM, NC>("VALU only (2 VALU waves)", 512);
  const double b = run<3, NM, NC>("both in every wave (2 waves)", 512);
  const double s = run<4, NM, NC>("1 MFMA wave + 1 VALU wave", 512);
  const double sm = run<5, NM, NC>("  + s_setprio 3 on the MFMA wave", 512);
  const double sv = run<6, NM, NC>("  + s_setprio 3 on the VALU wave", 512);
  printf("   both-in-every-wave / (MFMA only + VALU only) = %.3f (1 = no overlap, 0.5 = full)\n", b / (m + v));
  // split: each wave does its role for 2 x iters, so the SIMD's total work equals 'both'
  printf("   split (same total work as 'both'): no overlap = %.1f, full overlap = %.1f; measured %.1f / "
         "%.1f / %.1f (ratio %.3f / %.3f / %.3f)\n", m + v, (m > v ? m : v), s, sm, sv, s / (m + v), sm / (m + v),
         sv / (m + v));
}

int main() {
  suite<8, 16>();
  suite<8, 32>();
  suite<16, 32>();
  suite<4, 32>();
  return 0;
}
