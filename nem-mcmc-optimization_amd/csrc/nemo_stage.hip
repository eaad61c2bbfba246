// nemo_stage.hip -- building the staged model on the device from the
// observed knockdown matrix D (nem.py:25-64), so the
// host never materialises the S x S x E score table (655 MB at C5 in fp64).
//
// The reference's tables, restated (nem.py):
//   off-diagonal rows  T[i][j] = where(D[j] == 0, B, -A)               (:44-46)
//   diagonal rows      T[i][i] = where(D[i] == 1, 0, B)
//                                + sum_{m != i} where(D[m] == 1, A, 0)   (:25-34)
//   node LR table      U[i] = T[i][i];  U[S] = sum_m where(D[m] == 0, 0, A) (:56-64)
// The A's of a diagonal row are added one at a time onto the base 0 or B;
// adding the zeros in between is exact, so the value is the k-th element of
// an addition chain (k = number of other ones in the column).  The host
// computes the two chains (0 + A + A ..., B + A + A ...) sequentially, as the
// reference's loop does, and the kernels only index them: U is bit-identical
// to the reference's and exp(T) to what nemo_stage_tables stages.
#include "nemo_internal.h"

#include <math.h>

#include <algorithm>

namespace nemo {

namespace {

// one thread per effect: the column count k of D, then every U row of it
__global__ void knockdown_u_kernel(int S, int E, const uint8_t* __restrict__ D,
                                   const double* __restrict__ chains, double* __restrict__ U64) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const double* c0 = chains;          // 0 + k A
  const double* cb = chains + S + 1;  // B + k A
  int k = 0;
  for (int i = 0; i < S; ++i) k += D[(size_t)i * E + e];
  for (int i = 0; i < S; ++i) {
    const int d = D[(size_t)i * E + e];
    U64[(size_t)i * E + e] = d ? c0[k - 1] : cb[k];
  }
  U64[(size_t)S * E + e] = c0[k];
}

// exp(T) in the table dtype: one block per row (i, j), threads over effects;
// the same exp() as exp_table_kernel, so the bits match the host-T staging
template <class TT>
__global__ void knockdown_exp_kernel(int S, int E, const uint8_t* __restrict__ D,
                                     const double* __restrict__ U64, double negA, double B,
                                     TT* __restrict__ eT) {
  const int i = blockIdx.x / S;
  const int j = blockIdx.x - i * S;
  TT* out = eT + ((size_t)i * S + j) * E;
  if (i == j) {
    const double* u = U64 + (size_t)i * E;
    for (int e = threadIdx.x; e < E; e += blockDim.x) out[e] = (TT)exp(u[e]);
  } else {
    const uint8_t* d = D + (size_t)j * E;
    for (int e = threadIdx.x; e < E; e += blockDim.x) out[e] = (TT)exp(d[e] ? negA : B);
  }
}

__global__ void cast_f32_kernel(size_t n, const double* __restrict__ in, float* __restrict__ out) {
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n;
       k += (size_t)gridDim.x * blockDim.x)
    out[k] = (float)in[k];
}

}  // namespace

hipError_t launch_knockdown_tables(Ctx& c, const uint8_t* d_D, const double* d_chains, double A,
                                   double B, hipStream_t st) {
  const int S = c.S, E = c.E;
  knockdown_u_kernel<<<(E + 255) / 256, 256, 0, st>>>(S, E, d_D, d_chains, c.d_U64);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int threads = E >= 256 ? 256 : ((E + kWave - 1) / kWave) * kWave;
  if (c.dtype == 0)
    knockdown_exp_kernel<double><<<S * S, threads, 0, st>>>(S, E, d_D, c.d_U64, -A, B, (double*)c.d_eT);
  else
    knockdown_exp_kernel<float><<<S * S, threads, 0, st>>>(S, E, d_D, c.d_U64, -A, B, (float*)c.d_eT);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t nu = (size_t)(S + 1) * E;
  if (c.dtype == 0) return hipMemcpyAsync(c.d_U, c.d_U64, nu * 8, hipMemcpyDeviceToDevice, st);
  const int blocks = (int)std::min<size_t>((nu + 255) / 256, 4096);
  cast_f32_kernel<<<blocks, 256, 0, st>>>(nu, c.d_U64, (float*)c.d_U);
  return hipGetLastError();
}

}  // namespace nemo
