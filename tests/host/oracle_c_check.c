/* Drives oracle/nemo_oracle_c.c (the C restatement of the order score) for
 * tests/test_oracle_c.py under AddressSanitizer + UndefinedBehaviorSanitizer:
 * seeded synthetic tables, every cap, 1 and 3 OpenMP threads, with and without
 * the column output, the empty batch and the argument errors.  Prints "ok ..."
 * on success. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int nemo_oracle_order_scores(const double* U, const double* T, const int32_t* pos, const double* w01, int S,
                             int E, int batch, int cap, int threads, double* ll, double* cs);

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static double unif(void) { /* xorshift64*, [0, 1) */
  rng ^= rng >> 12; rng ^= rng << 25; rng ^= rng >> 27;
  return (double)((rng * 0x2545f4914f6cdd1dull) >> 11) * (1.0 / 9007199254740992.0);
}

static int check(int S, int E, int batch) {
  const size_t ne = (size_t)E;
  double* U = malloc(sizeof(double) * (S + 1) * ne);
  double* T = malloc(sizeof(double) * S * S * ne);
  int32_t* pos = malloc(sizeof(int32_t) * S * batch);
  double* w = malloc(sizeof(double) * S * S * batch);
  double *ll1 = malloc(sizeof(double) * batch), *ll3 = malloc(sizeof(double) * batch);
  double* cs = malloc(sizeof(double) * batch * ne);
  for (size_t k = 0; k < (S + 1) * ne; ++k) U[k] = -4.0 * unif();
  for (size_t k = 0; k < (size_t)S * S * ne; ++k) T[k] = 6.0 * unif() - 3.0;
  for (int b = 0; b < batch; ++b) {
    int32_t* p = pos + (size_t)b * S;
    for (int i = 0; i < S; ++i) p[i] = i;
    for (int i = S - 1; i > 0; --i) { /* Fisher-Yates */
      const int j = (int)(unif() * (i + 1));
      const int32_t t = p[i]; p[i] = p[j]; p[j] = t;
    }
  }
  for (size_t k = 0; k < (size_t)S * S * batch; ++k) w[k] = unif();
  int fails = 0;
  for (int cap = 0; cap <= S; ++cap) {
    if (nemo_oracle_order_scores(U, T, pos, w, S, E, batch, cap, 1, ll1, NULL) != 0) ++fails;
    if (nemo_oracle_order_scores(U, T, pos, w, S, E, batch, cap, 3, ll3, cs) != 0) ++fails;
    for (int b = 0; b < batch; ++b) {
      if (memcmp(&ll1[b], &ll3[b], sizeof(double)) != 0 || !isfinite(ll1[b])) ++fails;
      double sum = 0.0; /* ll is the left fold of cs */
      for (int e = 0; e < E; ++e) sum += cs[(size_t)b * E + e];
      if (memcmp(&sum, &ll1[b], sizeof(double)) != 0) ++fails;
    }
  }
  /* the empty batch; a repeated position; a position out of range; bad sizes */
  if (nemo_oracle_order_scores(U, T, NULL, NULL, S, E, 0, 0, 2, NULL, NULL) != 0) ++fails;
  if (S > 1) {
    const int32_t keep = pos[1];
    pos[1] = pos[0];
    if (nemo_oracle_order_scores(U, T, pos, w, S, E, batch, 0, 1, ll1, NULL) != -1) ++fails;
    pos[1] = S;
    if (nemo_oracle_order_scores(U, T, pos, w, S, E, batch, 0, 1, ll1, NULL) != -1) ++fails;
    pos[1] = keep;
  }
  if (nemo_oracle_order_scores(U, T, pos, w, 0, E, batch, 0, 1, ll1, NULL) != -1) ++fails;
  if (nemo_oracle_order_scores(U, T, pos, w, S, E, batch, -1, 1, ll1, NULL) != -1) ++fails;
  free(U); free(T); free(pos); free(w); free(ll1); free(ll3); free(cs);
  return fails;
}

int main(void) {
  int fails = 0, cases = 0;
  const int shapes[][3] = {{1, 1, 1}, {2, 1, 3}, {3, 65, 4}, {7, 130, 5}, {16, 33, 6}};
  for (size_t k = 0; k < sizeof(shapes) / sizeof(shapes[0]); ++k, ++cases)
    fails += check(shapes[k][0], shapes[k][1], shapes[k][2]);
  if (fails) {
    printf("FAIL %d\n", fails);
    return 1;
  }
  printf("ok %d shapes\n", cases);
  return 0;
}
