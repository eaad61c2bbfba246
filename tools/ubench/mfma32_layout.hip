// Layout check of v_mfma_i32_32x32x32_i8 (gfx950) as score_i8l32 uses it:
// lane l holds A[m = l % 32][k = 16 (l / 32) + 0..15], B[k = 16 (l / 32) + 0..15][n = l % 32],
// and D element v of lane l is D[8 (v / 4) + 4 (l / 32) + v % 4][l % 32].
// Random int8 A, B; D checked against a host product.  hipcc --offload-arch=gfx950 -O2 -o mfma32 mfma32_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <random>

typedef int v4 __attribute__((ext_vector_type(4)));
typedef int v16 __attribute__((ext_vector_type(16)));

__global__ void probe(const int8_t* a, const int8_t* b, int* d) {
  const int l = threadIdx.x;
  v4 av, bv;
  int8_t* pa = (int8_t*)&av;
  int8_t* pb = (int8_t*)&bv;
  for (int j = 0; j < 16; ++j) {
    pa[j] = a[(l % 32) * 32 + 16 * (l / 32) + j];      // A row-major 32 x 32 (m, k)
    pb[j] = b[(16 * (l / 32) + j) * 32 + l % 32];      // B row-major 32 x 32 (k, n)
  }
  v16 c = {};
  v16 r = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int v = 0; v < 16; ++v) d[(8 * (v / 4) + 4 * (l / 32) + v % 4) * 32 + l % 32] = r[v];
}

int main() {
  std::mt19937 g(7);
  std::uniform_int_distribution<int> u(-128, 127);
  int8_t ha[1024], hb[1024];
  for (int i = 0; i < 1024; ++i) { ha[i] = (int8_t)u(g); hb[i] = (int8_t)u(g); }
  int8_t *da, *db; int* dd;
  if (hipMalloc(&da, 1024) || hipMalloc(&db, 1024) || hipMalloc(&dd, 4096)) return 2;
  hipMemcpy(da, ha, 1024, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, 1024, hipMemcpyHostToDevice);
  hipMemset(dd, 0, 4096);
  probe<<<1, 64>>>(da, db, dd);
  int hd[1024];
  if (hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost)) return 3;
  int bad = 0;
  for (int m = 0; m < 32; ++m)
    for (int n = 0; n < 32; ++n) {
      int s = 0;
      for (int k = 0; k < 32; ++k) s += ha[m * 32 + k] * hb[k * 32 + n];
      if (s != hd[m * 32 + n]) ++bad;
    }
  printf("mfma_i32_32x32x32_i8 layout %s (%d mismatches of 1024)\n", bad ? "WRONG" : "ok", bad);
  return bad ? 1 : 0;
}
