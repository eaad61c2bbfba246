// LDS bank-conflict probe for the int8 kernel's access patterns: each kernel
// issues one pattern many times; run under rocprofv3 --pmc SQ_LDS_BANK_CONFLICT
// SQ_INSTS_LDS and compare per-kernel counts.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

using i32x4 = __attribute__((ext_vector_type(4))) int;

// b128 reads: lane (col = l & 15, rg = l >> 4) reads chunk col * STRIDE16 + rg
template <int STRIDE16>
__global__ void b128_rows(int iters, int* out) {
  __shared__ i32x4 buf[64 * 8];
  for (int k = threadIdx.x; k < 64 * 8; k += blockDim.x) buf[k] = i32x4{k, k + 1, k + 2, k + 3};
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t off = (uint32_t)((lane & 15) * STRIDE16 + (lane >> 4));
  i32x4 acc = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    asm volatile("" : "+v"(off));
    acc += buf[off];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

// b64 reads from a table of N doubles at a pseudo-random index per lane
template <int N>
__global__ void b64_random(int iters, double* out) {
  __shared__ double tab[256];
  for (int k = threadIdx.x; k < 256; k += blockDim.x) tab[k] = k;
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  double acc = 0;
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    acc += tab[(x >> 13) & (N - 1)];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  int* oi;
  double* od;
  (void)hipMalloc(&oi, 1 << 20);
  (void)hipMalloc(&od, 1 << 21);
  const int iters = 1000;
  b128_rows<4><<<256, 256>>>(iters, oi);
  b128_rows<5><<<256, 256>>>(iters, oi);
  b128_rows<6><<<256, 256>>>(iters, oi);
  b128_rows<8><<<256, 256>>>(iters, oi);
  b64_random<16><<<256, 256>>>(iters, od);
  b64_random<32><<<256, 256>>>(iters, od);
  b64_random<64><<<256, 256>>>(iters, od);
  b64_random<256><<<256, 256>>>(iters, od);
  (void)hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
