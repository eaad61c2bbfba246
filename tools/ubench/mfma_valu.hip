// Micro-benchmark: can v_mfma_f64_16x16x4_f64 and f64 VALU work overlap on
// one SIMD (same wave / different waves)?
//   hipcc --offload-arch=gfx950 -O3 mfma_valu.hip -o mfma_valu && ./mfma_valu
#include <hip/hip_runtime.h>
#include <stdio.h>

using f64x4 = __attribute__((ext_vector_type(4))) double;

// MODE 1: MFMA only; 2: VALU only; 3: both interleaved (sched_group_barrier);
// 4: both, sched_barrier between (no interleave); 5: waves of the first half
// of the block run the MFMAs, the second half the VALU
template <int MODE, int NM, int NV>
__global__ __launch_bounds__(512) void kern(int iters, double* out) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  f64x4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  double v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = a * (i + 1);
  const bool do_m = MODE == 1 || MODE == 3 || MODE == 4 || (MODE == 5 && w < (int)(blockDim.x / 128));
  const bool do_v = MODE == 2 || MODE == 3 || MODE == 4 || (MODE == 5 && w >= (int)(blockDim.x / 128));
  for (int it = 0; it < iters; ++it) {
    if (MODE == 5) {
      if (do_m) {
#pragma unroll
        for (int k = 0; k < NM / 4; ++k) {
          acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc1, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2, 0, 0, 0);
          acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc3, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int k = 0; k < NV / 8; ++k)
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = fma(v[i], b, a);
      }
      continue;
    }
    if (do_m) {
#pragma unroll
      for (int k = 0; k < NM / 4; ++k) {
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc3, 0, 0, 0);
      }
    }
    if (MODE == 4) __builtin_amdgcn_sched_barrier(0);
    if (do_v) {
#pragma unroll
      for (int k = 0; k < NV / 8; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fma(v[i], b, a);
    }
    if (MODE == 3) {
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV / NM, 0);
      }
    }
  }
  double s = acc0[0] + acc1[1] + acc2[2] + acc3[3];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int NM, int NV>
void run(const char* name, int threads, int blocks) {
  double* out;
  (void)hipMalloc(&out, (size_t)blocks * threads * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 400;
  kern<MODE, NM, NV><<<blocks, threads>>>(iters, out);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) kern<MODE, NM, NV><<<blocks, threads>>>(iters, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double cyc = ms * 1e-3 * 2.4e9 / iters;
  printf("%-36s NM=%2d NV=%3d threads=%3d: %8.4f ms  %6.0f SIMD-cyc/iter  (MFMA-only floor %d, waves/SIMD %d)\n",
         name, NM, NV, threads, ms, cyc, 64 * NM * (MODE == 5 ? 1 : threads / 256), threads / 256);
  (void)hipFree(out);
}

template <int NM, int NV>
void suite() {
  for (int t : {256, 512}) {
    run<1, NM, NV>("MFMA only", t, 256);
    run<2, NM, NV>("VALU only", t, 256);
    run<3, NM, NV>("both, one wave, interleaved", t, 256);
    run<4, NM, NV>("both, one wave, sequential", t, 256);
  }
  run<5, NM, NV>("MFMA waves + VALU waves (2/SIMD)", 512, 256);
}

int main() {
  suite<32, 256>();
  suite<32, 512>();
  return 0;
}
