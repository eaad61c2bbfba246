// Which VALU classes overlap with which MFMA classes on one SIMD?
// Each kernel: waves of the first half run MFMAs of type MT, waves of the
// second half run VALU work of type VT (2 waves per SIMD), or one wave does
// both (mode "same").  Prints SIMD-cycles per iteration.
//   hipcc --offload-arch=gfx950 -O3 overlap.hip -o overlap && ./overlap
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

using f64x4 = __attribute__((ext_vector_type(4))) double;
using i32x4 = __attribute__((ext_vector_type(4))) int;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;

enum { M_NONE, M_F64, M_I8, M_BF16 };
enum { V_NONE, V_F64, V_F32, V_I32 };

template <int MT, int VT, bool SAME>
__global__ __launch_bounds__(512) void kern(int iters, double* out) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const bool first = w < (int)(blockDim.x / 128);
  const bool do_m = SAME || first, do_v = SAME || !first;
  const double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  f64x4 d0 = {0, 0, 0, 0}, d1 = d0, d2 = d0, d3 = d0;
  i32x4 i0 = {0, 0, 0, 0}, i1 = i0, i2 = i0, i3 = i0;
  f32x4 f0 = {0, 0, 0, 0}, f1 = f0, f2 = f0, f3 = f0;
  const i32x4 ia = {(int)threadIdx.x, 3, 5, 7}, ib = {1, (int)threadIdx.x, 2, 9};
  bf16x8 ba, bb;
  for (int i = 0; i < 8; ++i) { ba[i] = (__bf16)(float)(threadIdx.x + i); bb[i] = (__bf16)(float)(i + 1); }
  double v[8];
  float vf[8];
  uint32_t vi[8];
  for (int i = 0; i < 8; ++i) { v[i] = a * (i + 1); vf[i] = (float)v[i]; vi[i] = threadIdx.x * (i + 3); }
  for (int it = 0; it < iters; ++it) {
    if (MT != M_NONE && do_m) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {  // 32 MFMAs
        if (MT == M_F64) {
          d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d0, 0, 0, 0);
          d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d1, 0, 0, 0);
          d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d2, 0, 0, 0);
          d3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d3, 0, 0, 0);
        } else if (MT == M_I8) {
          i0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ia, ib, i0, 0, 0, 0);
          i1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ia, ib, i1, 0, 0, 0);
          i2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ia, ib, i2, 0, 0, 0);
          i3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ia, ib, i3, 0, 0, 0);
        } else {
          f0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba, bb, f0, 0, 0, 0);
          f1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba, bb, f1, 0, 0, 0);
          f2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba, bb, f2, 0, 0, 0);
          f3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba, bb, f3, 0, 0, 0);
        }
      }
    }
    if (VT != V_NONE && do_v) {
#pragma unroll
      for (int k = 0; k < 32; ++k)  // 256 VALU
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (VT == V_F64) v[i] = fma(v[i], b, a);
          else if (VT == V_F32) vf[i] = fmaf(vf[i], 1.0001f, 0.5f);
          else vi[i] = (vi[i] ^ (vi[i] >> 3)) + 0x9e3779b9u;  // 2 int ops
        }
    }
  }
  double s = d0[0] + d1[1] + d2[2] + d3[3] + i0[0] + i1[1] + i2[2] + i3[3] + f0[0] + f1[1] + f2[2] + f3[3];
  for (int i = 0; i < 8; ++i) s += v[i] + vf[i] + vi[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MT, int VT, bool SAME>
double run(int threads) {
  double* out;
  (void)hipMalloc(&out, (size_t)256 * threads * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 400;
  kern<MT, VT, SAME><<<256, threads>>>(iters, out);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) kern<MT, VT, SAME><<<256, threads>>>(iters, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(out);
  return ms / 5 * 1e-3 * 2.4e9 / iters;
}

int main() {
  const char* mn[] = {"none", "f64 16x16x4", "i8 16x16x64", "bf16 16x16x32"};
  const char* vn[] = {"none", "f64 fma", "f32 fma", "int xor/shift/add"};
  printf("cycles per iteration (32 MFMAs and/or 256 VALU ops per wave)\n");
#define ROW(MT, VT)                                                                          \
  printf("%-14s + %-18s  alone-M %6.0f  alone-V %6.0f  split-waves %6.0f  same-wave %6.0f\n", \
         mn[MT], vn[VT], run<MT, V_NONE, false>(256), run<M_NONE, VT, false>(256),         \
         run<MT, VT, false>(512), run<MT, VT, true>(256));
  ROW(M_F64, V_F64)
  ROW(M_F64, V_F32)
  ROW(M_F64, V_I32)
  ROW(M_I8, V_F64)
  ROW(M_I8, V_I32)
  ROW(M_BF16, V_F64)
  ROW(M_BF16, V_F32)
  return 0;
}
