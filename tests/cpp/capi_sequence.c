/* C client of include/nngp.h (the call sequence the R shim's drop-in makes,
 * rpkg/R/mcmc_nngp_update_Gaussian.R): order -> NN -> colouring -> create a
 * 2-chain context -> factor -> field / mu -> log-likelihood -> sweep_chains
 * -> get_field -> destroy.  Prints the log-likelihood and both chains' fields
 * (%a, exact) for tests/test_gpu_capi_sequence.py, which repeats the same
 * sequence through the Python binding and requires identical output.
 * Usage: capi_sequence [n] [m] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "nngp.h"

#define CHECK(call, ctx)                                                                            \
  do {                                                                                              \
    int st_ = (call);                                                                               \
    if (st_ != NNGP_OK) {                                                                           \
      fprintf(stderr, "%s failed: %s (%s)\n", #call, nngp_status_string(st_),                       \
              (ctx) ? nngp_ctx_last_error(ctx) : "");                                               \
      if (ctx) nngp_ctx_destroy(ctx);                                                               \
      return 1;                                                                                     \
    }                                                                                               \
  } while (0)

/* deterministic inputs: a jittered grid and smooth observations */
static double jit(int i, int k) {
  uint32_t h = (uint32_t)i * 2654435761u ^ (uint32_t)(k + 1) * 40503u;
  h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
  return (h & 0xFFFFFF) / (double)0x1000000 - 0.5;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 3000, m = argc > 2 ? atoi(argv[2]) : 10, d = 2, b = m + 1;
  const int side = (int)ceil(sqrt((double)n));
  double* raw = malloc(sizeof(double) * n * d);
  double* locs = malloc(sizeof(double) * n * d);
  int* order = malloc(sizeof(int) * n);
  int* NN = malloc(sizeof(int) * n * b);
  int* col = malloc(sizeof(int) * n);
  int* lm = malloc(sizeof(int) * n);
  double *y = malloc(sizeof(double) * n), *f = malloc(sizeof(double) * n);
  for (int i = 0; i < n; ++i) {
    raw[i] = (i % side + 0.3 * jit(i, 0)) / side;
    raw[i + n] = (i / side + 0.3 * jit(i, 1)) / side;
  }
  nngp_ctx* ctx = NULL;
  CHECK(nngp_order_maxmin(raw, n, d, order), ctx);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < d; ++k) locs[i + (size_t)k * n] = raw[order[i] - 1 + (size_t)k * n];
  CHECK(nngp_find_ordered_nn(locs, n, d, m, NN), ctx);
  int K = 0;
  CHECK(nngp_greedy_coloring(NN, n, b, col, &K), ctx);
  for (int i = 0; i < n; ++i) {
    lm[i] = i + 1;
    y[i] = sin(6 * locs[i]) + cos(4 * locs[i + n]) + 0.3 * jit(i, 2);
    f[i] = y[i] + 0.1 * jit(i, 3);
  }
  CHECK(nngp_ctx_create(locs, n, d, NN, b, col, lm, y, n, 2, 0, &ctx), ctx);
  const double cp[2][3] = {{1.0, 0.1, 0.0}, {0.8, 0.15, 0.0}};
  const double b0[2] = {0.1, -0.2}, ls[2] = {0.0, 0.3}, lnv[2] = {-1.0, -0.7};
  const uint64_t seed[2] = {101, 202}, cb[2] = {0, 50};
  double ll = 0;
  for (int k = 0; k < 2; ++k) {
    CHECK(nngp_set_chain(ctx, k), ctx);
    CHECK(nngp_factor(ctx, 0, NNGP_EXPONENTIAL_ISOTROPIC, cp[k], 3), ctx);
    CHECK(nngp_set_field(ctx, f), ctx);
    CHECK(nngp_set_mu(ctx, NULL, b0[k]), ctx);
  }
  CHECK(nngp_set_chain(ctx, 1), ctx);
  CHECK(nngp_loglik(ctx, 0, b0[1], ls[1], &ll), ctx);
  CHECK(nngp_sweep_chains(ctx, 3, b0, ls, lnv, seed, cb), ctx);
  printf("colours %d\nloglik %a\n", K, ll);
  for (int k = 0; k < 2; ++k) {
    CHECK(nngp_set_chain(ctx, k), ctx);
    CHECK(nngp_get_field(ctx, f), ctx);
    printf("chain %d", k);
    for (int i = 0; i < n; ++i) printf(" %a", f[i]);
    printf("\n");
  }
  nngp_ctx_destroy(ctx);
  free(raw); free(locs); free(order); free(NN); free(col); free(lm); free(y); free(f);
  return 0;
}
