// Micro-benchmark: issue cost on gfx950 of the integer / conversion VALU
// instructions a fixed-point exp epilogue can use (cycles per wave-instruction
// per SIMD, 8 independent chains per lane, 4 waves per SIMD on every CU;
// "cycles" assume 2.4 GHz, so compare rows with each other and with fma_f32,
// the 2-cycle reference).
//   hipcc --offload-arch=gfx950 -O3 valu_rate2.hip -o valu_rate2 && ./valu_rate2
#include <hip/hip_runtime.h>
#include <stdio.h>

#define OP_KERNEL(NAME, DECL, INIT, ASM, CONS)                                 \
  __global__ __launch_bounds__(256) void NAME(int iters, double* out) {       \
    DECL v[8];                                                                \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) v[i] = INIT;                \
    for (int it = 0; it < iters; ++it) {                                      \
      _Pragma("unroll") for (int k = 0; k < 8; ++k) {                         \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) ASM;                    \
      }                                                                       \
    }                                                                         \
    double s = 0;                                                             \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s += CONS;                  \
    if (s == 1.2345) out[threadIdx.x] = s;                                    \
  }

#define IOP(NAME, TXT) \
  OP_KERNEL(NAME, int, (int)threadIdx.x + i, asm volatile(TXT : "+v"(v[i])), (double)v[i])

IOP(k_and, "v_and_b32 %0, 0x3ff8, %0")
IOP(k_lshr, "v_lshrrev_b32 %0, 6, %0")
IOP(k_ashr, "v_ashrrev_i32 %0, 3, %0")
IOP(k_add, "v_add_u32 %0, %0, %0")
IOP(k_sub, "v_sub_u32 %0, %0, %0")
IOP(k_xor, "v_xor_b32 %0, %0, %0")
IOP(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %0")
IOP(k_xad, "v_xad_u32 %0, %0, %0, %0")
IOP(k_add3, "v_add3_u32 %0, %0, %0, %0")
IOP(k_bfe, "v_bfe_u32 %0, %0, 9, 11")
IOP(k_lshl_or, "v_lshl_or_b32 %0, %0, 3, %0")
IOP(k_and_or, "v_and_or_b32 %0, %0, 63, %0")
IOP(k_mad24, "v_mad_u32_u24 %0, %0, %0, %0")
IOP(k_mullo, "v_mul_lo_u32 %0, %0, %0")
IOP(k_perm, "v_perm_b32 %0, %0, %0, %0")
IOP(k_cvt_f32, "v_cvt_f32_i32 %0, %0")
OP_KERNEL(k_cvt64u, int, (int)threadIdx.x + i,
          asm volatile("v_cvt_f64_u32 v[40:41], %0\n v_mov_b32 %0, v41" : "+v"(v[i]) :: "v40", "v41"), (double)v[i])
OP_KERNEL(k_cvt64i, int, (int)threadIdx.x + i,
          asm volatile("v_cvt_f64_i32 v[40:41], %0\n v_mov_b32 %0, v41" : "+v"(v[i]) :: "v40", "v41"), (double)v[i])
OP_KERNEL(k_mov, int, (int)threadIdx.x + i, asm volatile("v_mov_b32 %0, %0" : "+v"(v[i])), (double)v[i])
OP_KERNEL(k_fma32, float, threadIdx.x * 1e-3f + i,
          asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(v[i])), (double)v[i])
OP_KERNEL(k_fma64, double, threadIdx.x * 1e-3 + i,
          asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(v[i])), v[i])
OP_KERNEL(k_add64, double, threadIdx.x * 1e-3 + i,
          asm volatile("v_add_f64 %0, %0, %0" : "+v"(v[i])), v[i])
typedef float f2 __attribute__((ext_vector_type(2)));
#define F2INIT ((f2){threadIdx.x * 1e-3f + i, 1.0f})
OP_KERNEL(k_pkfma, f2, F2INIT,
          asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(v[i])), (double)v[i].x)
OP_KERNEL(k_pkmul, f2, F2INIT,
          asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(v[i])), (double)v[i].x)

template <typename K>
static void run(const char* name, K k, int extra_per_op) {
  double* d;
  hipMalloc(&d, 4096 * 8);
  const int blocks = 256 * 4;  // 4 blocks of 256 threads per CU = 4 waves per SIMD
  const int iters = 2000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, 10, d);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, iters, d);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double waves = blocks * 4.0;
  const double insts = waves * iters * 64.0 * (1 + extra_per_op);
  const double cyc = ms * 1e-3 * 2.4e9 * 1024 / insts;
  printf("%-10s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (2.4 GHz)\n", name, ms, cyc);
  hipFree(d);
}

int main() {
  run("fma_f32", k_fma32, 0);
  run("mov_b32", k_mov, 0);
  run("fma_f64", k_fma64, 0);
  run("add_f64", k_add64, 0);
  run("pk_fma_f32", k_pkfma, 0);
  run("pk_mul_f32", k_pkmul, 0);
  run("and_b32", k_and, 0);
  run("lshrrev", k_lshr, 0);
  run("ashrrev", k_ashr, 0);
  run("add_u32", k_add, 0);
  run("sub_u32", k_sub, 0);
  run("xor_b32", k_xor, 0);
  run("lshl_add", k_lshl_add, 0);
  run("xad_u32", k_xad, 0);
  run("add3_u32", k_add3, 0);
  run("bfe_u32", k_bfe, 0);
  run("lshl_or", k_lshl_or, 0);
  run("and_or", k_and_or, 0);
  run("mad_u24", k_mad24, 0);
  run("mul_lo", k_mullo, 0);
  run("perm_b32", k_perm, 0);
  run("cvt_f32_i32", k_cvt_f32, 0);
  run("cvt_f64_u32+mov", k_cvt64u, 1);
  run("cvt_f64_i32+mov", k_cvt64i, 1);
  return 0;
}
