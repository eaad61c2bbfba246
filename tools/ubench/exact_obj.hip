// exact_obj.hip -- the exact local objective alone (nemo_exact.hip's
// ExactObjective, plan-ordered c rows), K forward-difference evaluations per
// wave, W waves: how much of local_opt_exact_kernel's time the objective is.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I nem-mcmc-optimization_amd/csrc \
//         tools/ubench/exact_obj.hip -o tools/ubench/exact_obj
//   tools/ubench/exact_obj [W=32256] [K=5] [E=2000]
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include <hip/hip_runtime.h>
// per-part cycle totals of the control (lane 0 of every wave adds its own;
// -DNEMO_UB_NOHOOK: the plain control, for its time)
__device__ unsigned long long g_lbx_t[8];
#ifndef NEMO_UB_NOHOOK
// per-wave totals in LDS (lane 0 adds; one global atomic per wave at the end)
__shared__ unsigned long long ub_t[4][8];
#define NEMO_LBX_T(k, stmt)                                                              \
  do {                                                                                   \
    const long long t0_ = wall_clock64();                                                \
    stmt;                                                                                \
    if ((threadIdx.x & 63) == 0) ub_t[threadIdx.x >> 6][k] += (unsigned long long)(wall_clock64() - t0_); \
  } while (0)
#endif
#include "nemo_exact.hip"

namespace nemo {
namespace {

template <int NS>
__global__ __launch_bounds__(kExactWaves * kWave) void obj_bench_kernel(int W, int K, const double* __restrict__ cbuf,
                                                                         const int32_t* __restrict__ plan, int nh,
                                                                         int maxrem, double* __restrict__ out) {
  __shared__ TabsLds tabs;
  __shared__ int32_t pl[(4 * NS + 8) * kWave];
  tabs.fill(threadIdx.x, blockDim.x);
  plan_to_lds<NS>(plan, nh, pl);
  __syncthreads();
  const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  const int lane = threadIdx.x & (kWave - 1);
  if (gw >= W) return;
  using Obj = ExactObjective<NS, true, false>;
  Obj obj;
  obj.tb = tabs.view();
  obj.pl = pl;
  obj.lane = lane;
  obj.nh = nh;
  obj.maxrem = maxrem;
  obj.anc = 0.25;
  obj.cp = cbuf + (size_t)gw * NS * Obj::kRows * kWave;
  double acc = 0.0;
  for (int k = 0; k < K; ++k) {
    const double x = 0.3 * k - 0.6;
    double f0, f1;
    obj(x, x + 1e-8, f0, f1);
    acc = acc + f0 + f1;
  }
  if (lane == 0) out[gw] = acc;
}

// the optimiser's control alone: a 1-D objective of the reference's shape at
// the cost of a few logs, the LbxState in LDS (kLds) or in registers
struct CheapObjective {
  double c, anc, wgt;
  LdsTabs tb;
  __device__ __forceinline__ void operator()(double x0, double x1, double& f0, double& f1) const {
#pragma clang fp contract(off)
    const double e0 = refmath::expit(x0, tb), e1 = refmath::expit(x1, tb);
    f0 = (-wgt * refmath::svml_log(c * e0 + 1.0, tb) + fabs(e0 - anc)) + e0 * (1.0 - e0);
    f1 = (-wgt * refmath::svml_log(c * e1 + 1.0, tb) + fabs(e1 - anc)) + e1 * (1.0 - e1);
  }
};

template <bool kLds>
__global__ __launch_bounds__(kExactWaves * kWave) void ctrl_bench_kernel(int W, const double* __restrict__ prm,
                                                                          double* __restrict__ out) {
  __shared__ TabsLds tabs;
  __shared__ double mem[kExactWaves][lbx::kMemDoubles];
  __shared__ double lst_raw[kExactWaves][kStateDoubles];
  tabs.fill(threadIdx.x, blockDim.x);
  __syncthreads();
  const int wv = threadIdx.x / kWave;
  const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave));
  if (gw >= W) return;
  CheapObjective obj{prm[3 * gw], prm[3 * gw + 1], 40.0, tabs.view()};
#ifndef NEMO_UB_NOHOOK
  if ((threadIdx.x & 63) < 8) ub_t[wv][threadIdx.x & 63] = 0;
#endif
  LbxState reg;
  LbxState& st = kLds ? *reinterpret_cast<LbxState*>(lst_raw[wv]) : reg;
  lbx_init(st, prm[3 * gw + 2]);
  for (;;) {
    bool more;
    NEMO_LBX_T(4, more = lbx_run(st, lbx::Mem{mem[wv]}));
    if (!more) break;
    double f0, f1;
    NEMO_LBX_T(5, obj(st.x_eval, st.x1, f0, f1));
    lbx_feed(st, f0, f1);
  }
  if ((threadIdx.x & (kWave - 1)) == 0) {
    out[2 * gw] = st.x;
    out[2 * gw + 1] = st.nfev;
#ifndef NEMO_UB_NOHOOK
    for (int q = 0; q < 8; ++q) atomicAdd(&g_lbx_t[q], ub_t[wv][q]);
#endif
  }
}

}  // namespace
}  // namespace nemo

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                      \
    }                                                                \
  } while (0)

int main(int argc, char** argv) {
  using namespace nemo;
  const int W = argc > 1 ? atoi(argv[1]) : 32256;
  const int K = argc > 2 ? atoi(argv[2]) : 5;
  const int E = argc > 3 ? atoi(argv[3]) : 2000;
  host::PairwisePlan pl;
  if (!host::build_pairwise_plan(E, pl) || pl.ns != 2) {
    fprintf(stderr, "plan: E=%d ns=%d (this bench instantiates ns = 2)\n", E, pl.ns);
    return 1;
  }
  std::vector<int32_t> dev;
  dev.insert(dev.end(), pl.start.begin(), pl.start.end());
  dev.insert(dev.end(), pl.cnt.begin(), pl.cnt.end());
  dev.insert(dev.end(), pl.rem.begin(), pl.rem.end());
  dev.insert(dev.end(), pl.nrem.begin(), pl.nrem.end());
  dev.insert(dev.end(), pl.partner.begin(), pl.partner.end());
  const size_t per = (size_t)pl.ns * 17 * 64;
  std::vector<double> c(per * W);
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-0.5, 2.0);
  for (auto& v : c) v = U(rng);
  double *d_c, *d_out;
  int32_t* d_plan;
  CK(hipMalloc(&d_c, c.size() * 8));
  CK(hipMalloc(&d_out, W * 8));
  CK(hipMalloc(&d_plan, dev.size() * 4));
  CK(hipMemcpy(d_c, c.data(), c.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_plan, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const dim3 grid((W + kExactWaves - 1) / kExactWaves);
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(a));
    obj_bench_kernel<2><<<grid, kExactWaves * kWave>>>(W, K, d_c, d_plan, pl.nh, pl.maxrem, d_out);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double logs = 2.0 * W * (double)K * E;
    printf("W=%d K=%d E=%d: %.3f ms, %.2f G logs/s, %.1f ns per wave-evaluation-pair\n", W, K, E, ms,
           logs / ms / 1e6, ms * 1e6 / ((double)W * K));
  }
  // the control alone
  std::vector<double> prm(3 * W);
  std::uniform_real_distribution<double> A(0.0, 0.5), X(-3.0, 3.0), C(-0.3, 1.5);
  for (int w = 0; w < W; ++w) prm[3 * w] = C(rng), prm[3 * w + 1] = A(rng), prm[3 * w + 2] = X(rng);
  double *d_prm, *d_res;
  CK(hipMalloc(&d_prm, prm.size() * 8));
  CK(hipMalloc(&d_res, 2 * (size_t)W * 8));
  CK(hipMemcpy(d_prm, prm.data(), prm.size() * 8, hipMemcpyHostToDevice));
  for (int lds = 0; lds < 2; ++lds)
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      if (lds) ctrl_bench_kernel<true><<<grid, kExactWaves * kWave>>>(W, d_prm, d_res);
      else ctrl_bench_kernel<false><<<grid, kExactWaves * kWave>>>(W, d_prm, d_res);
      CK(hipGetLastError());
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      std::vector<double> res(2 * (size_t)W);
      CK(hipMemcpy(res.data(), d_res, res.size() * 8, hipMemcpyDeviceToHost));
      double nf = 0, mx = 0;
      for (int w = 0; w < W; ++w) nf += res[2 * w + 1], mx = res[2 * w + 1] > mx ? res[2 * w + 1] : mx;
      printf("control (state in %s) W=%d: %.3f ms, nfev mean %.2f max %.0f\n", lds ? "LDS" : "registers", W, ms,
             nf / W, mx);
      unsigned long long t[8];
      CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_lbx_t), sizeof(t)));
      const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_lbx_t), z, sizeof(z)));
      const char* nm[6] = {"dcsrch", "formt", "formk", "subsm", "lbx_run", "objective"};
      printf("   wall-clock (100 MHz) ticks per wave:");
      for (int k = 0; k < 6; ++k) printf(" %s %.0f", nm[k], (double)t[k] / W);
      printf("\n");
    }
  return 0;
}
