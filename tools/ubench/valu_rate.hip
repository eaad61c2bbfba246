// Micro-benchmark: issue cost of the VALU instructions of the int8 score
// kernel's cell + exp chain on gfx950 (cycles per wave-instruction per SIMD,
// 8 independent chains per lane, 4 waves per SIMD on every CU).
//   hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate && ./valu_rate
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

OP_KERNEL(k_fma64, double, threadIdx.x * 1e-3 + i,
          asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(v[i])), v[i])
OP_KERNEL(k_add64, double, threadIdx.x * 1e-3 + i,
          asm volatile("v_add_f64 %0, %0, %0" : "+v"(v[i])), v[i])
OP_KERNEL(k_mul64, double, threadIdx.x * 1e-3 + i,
          asm volatile("v_mul_f64 %0, %0, %0" : "+v"(v[i])), v[i])
OP_KERNEL(k_cvt64, int, (int)threadIdx.x + i,
          asm volatile("v_cvt_f64_i32 v[40:41], %0\n v_mov_b32 %0, v40" : "+v"(v[i]) :: "v40", "v41"), (double)v[i])
OP_KERNEL(k_ldexp64, double, threadIdx.x * 1e-3 + i,
          asm volatile("v_ldexp_f64 %0, %0, 1" : "+v"(v[i])), v[i])
OP_KERNEL(k_rnd64, double, threadIdx.x * 1e-3 + i,
          asm volatile("v_rndne_f64 %0, %0" : "+v"(v[i])), v[i])
OP_KERNEL(k_lshladd, int, (int)threadIdx.x + i,
          asm volatile("v_lshl_add_u32 %0, %0, 3, %0" : "+v"(v[i])), (double)v[i])
OP_KERNEL(k_fma32, float, threadIdx.x * 1e-3f + i,
          asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(v[i])), (double)v[i])
OP_KERNEL(k_mov32, int, (int)threadIdx.x + i,
          asm volatile("v_mov_b32 %0, %0" : "+v"(v[i])), (double)v[i])

template <typename K>
static void run(const char* name, K k, int extra_per_op) {
  double* d;
  hipMalloc(&d, 4096 * 8);
  const int blocks = 256 * 4;  // 4 waves of 256 threads per CU... 16 waves/CU = 4 per SIMD
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
  // cycles per wave-instruction per SIMD at 2.4 GHz, 1024 SIMDs
  const double cyc = ms * 1e-3 * 2.4e9 * 1024 / insts;
  printf("%-10s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (2.4 GHz)\n", name, ms, cyc);
  hipFree(d);
}

int main() {
  run("fma_f64", k_fma64, 0);
  run("add_f64", k_add64, 0);
  run("mul_f64", k_mul64, 0);
  run("cvt_f64", k_cvt64, 1);
  run("ldexp_f64", k_ldexp64, 0);
  run("rndne_f64", k_rnd64, 0);
  run("lshl_add", k_lshladd, 0);
  run("fma_f32", k_fma32, 0);
  run("mov_b32", k_mov32, 0);
  return 0;
}
