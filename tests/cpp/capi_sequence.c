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

/* The call sequence of the R drop-in's lockstep iteration
 * (rpkg/R/mcmc_nngp_update_Gaussian.R, update_Gaussian.R:113-311) over 3
 * chains of one context, 2 iterations, n_chromatic = 2, with the R side's
 * random draws replaced by fixed numbers and its accept decisions by fixed
 * log-uniforms (chain 0 always accepts, chain 1 never, chain 2 by the device
 * value): every device result the host sees is printed in hex (the Python
 * binding replays the same sequence, tests/test_gpu_capi_sequence.py). */
static void pr3(const char* tag, int it, const double* v) {
  printf("%s %d %a %a %a\n", tag, it, v[0], v[1], v[2]);
}

static int lockstep(nngp_ctx* ctx, int n, double* f) {
  const int C = 3, all = 7, NC = 2, NIT = 2;
  double ls[3] = {0.0, 0.2, -0.1}, shape[3] = {-2.3, -2.0, -2.6}, b0[3] = {0.1, -0.2, 0.0};
  double lnv[3] = {-1.0, -0.7, -1.2};
  const double lu_anc[3] = {-1e300, 1e300, -0.7}, lu_suf[3] = {1e300, -1e300, -0.3};
  /* chains 1 and 2 stream their records into host arrays as the R drop-in
     does; chain 0 keeps them on the device until get_records */
  double* rb[3] = {NULL, malloc(sizeof(double) * (size_t)NIT * n), malloc(sizeof(double) * (size_t)NIT * n)};
  for (int k = 0; k < C; ++k) {
    const double cp[3] = {1.0, exp(shape[k]), 0.0};
    for (int i = 0; i < n; ++i) f[i] = 0.05 * k + sin(3.0 * i / n + k);
    CHECK(nngp_set_chain(ctx, k), ctx);
    CHECK(nngp_records_reserve(ctx, NIT), ctx);
    if (rb[k]) CHECK(nngp_records_stream(ctx, rb[k], NIT), ctx);
    CHECK(nngp_factor(ctx, 0, NNGP_EXPONENTIAL_ISOTROPIC, cp, 3), ctx);
    CHECK(nngp_set_field(ctx, f), ctx);
    CHECK(nngp_set_mu(ctx, NULL, b0[k]), ctx);
  }
  for (int it = 1; it <= NIT; ++it) {
    double nls[3], nsh[3], cps[9], dls[3], v[3], l1[3], l0[3], ssr[3];
    int st[3];
    /* ancillary covariance update (:113-157) */
    for (int k = 0; k < C; ++k) {
      nls[k] = ls[k] + 0.05 * (k + 1) * (it % 2 ? 1.0 : -1.0);
      nsh[k] = shape[k] + 0.02 * (k - 1);
      cps[3 * k] = 1.0; cps[3 * k + 1] = exp(nsh[k]); cps[3 * k + 2] = 0.0;
      dls[k] = nls[k] - ls[k];
    }
    /* the R drop-in's one-sync step: factor, proposal field and ratio */
    CHECK(nngp_ancillary_step_chains(ctx, all, NNGP_EXPONENTIAL_ISOTROPIC, cps, 3, b0, dls, lnv, st, v), ctx);
    pr3("ratio", it, v);
    for (int k = 0; k < C; ++k)
      if (st[k] == 0 && v[k] > lu_anc[k]) {
        shape[k] = nsh[k]; ls[k] = nls[k];
        CHECK(nngp_set_chain(ctx, k), ctx);
        CHECK(nngp_accept_field(ctx), ctx);
        CHECK(nngp_accept_factor(ctx), ctx);
      }
    /* sufficient covariance update (:165-213) */
    for (int k = 0; k < C; ++k) {
      nls[k] = ls[k] - 0.03 * (k + 1);
      nsh[k] = shape[k] + 0.01 * (2 - k);
      cps[3 * k] = 1.0; cps[3 * k + 1] = exp(nsh[k]); cps[3 * k + 2] = 0.0;
    }
    CHECK(nngp_sufficient_step_chains(ctx, all, NNGP_EXPONENTIAL_ISOTROPIC, cps, 3, b0, nls, ls, st, l1, l0), ctx);
    pr3("l1", it, l1);
    pr3("l0", it, l0);
    for (int k = 0; k < C; ++k) {
      if (st[k] == 0 && l1[k] - l0[k] > lu_suf[k]) {
        shape[k] = nsh[k]; ls[k] = nls[k];
        CHECK(nngp_set_chain(ctx, k), ctx);
        CHECK(nngp_accept_factor(ctx), ctx);
      }
      /* field mean (:219-224) */
      double oqo = 0, oqf = 0;
      CHECK(nngp_set_chain(ctx, k), ctx);
      CHECK(nngp_beta0_stats(ctx, &oqo, &oqf), ctx);
      printf("beta0_stats %d %d %a %a\n", it, k, oqo, oqf);
      b0[k] = 0.5 * oqf / oqo + 0.1 * k;
      CHECK(nngp_set_mu(ctx, NULL, b0[k]), ctx);
    }
    /* chromatic sweeps of every chain, one call (:257-275) */
    const uint64_t seed[3] = {11, 12, 13};
    const uint64_t cb[3] = {(uint64_t)(it - 1) * NC, (uint64_t)(it - 1) * NC, (uint64_t)(it - 1) * NC};
    CHECK(nngp_sweep_chains(ctx, NC, b0, ls, lnv, seed, cb), ctx);
    /* noise variance (:281-293) */
    CHECK(nngp_sum_squared_residuals_chains(ctx, all, b0, ssr), ctx);
    pr3("ssr", it, ssr);
    for (int k = 0; k < C; ++k) lnv[k] += ssr[k] > n * exp(lnv[k]) ? 0.01 : -0.01;
    /* records (:305-311) */
    for (int k = 0; k < C; ++k) {
      CHECK(nngp_set_chain(ctx, k), ctx);
      CHECK(nngp_record_field(ctx, it - 1), ctx);
    }
  }
  double* rec = malloc(sizeof(double) * (size_t)NIT * n);
  for (int k = 0; k < C; ++k) {
    CHECK(nngp_set_chain(ctx, k), ctx);
    const double* rk = rb[k] ? rb[k] : rec;
    CHECK(nngp_get_records(ctx, 0, NIT, rb[k] ? rb[k] : rec), ctx);
    for (int r = 0; r < NIT; ++r) {
      printf("record %d %d", k, r);
      for (int i = 0; i < n; ++i) printf(" %a", rk[(size_t)r * n + i]);
      printf("\n");
    }
    CHECK(nngp_get_field(ctx, f), ctx);
    printf("field %d", k);
    for (int i = 0; i < n; ++i) printf(" %a", f[i]);
    printf("\n");
    if (rb[k]) {
      CHECK(nngp_records_stream(ctx, NULL, 0), ctx);
      free(rb[k]);
    }
  }
  free(rec);
  return 0;
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
  if (argc > 3) {  /* "lockstep": the R drop-in's 3-chain iteration */
    CHECK(nngp_ctx_create(locs, n, d, NN, b, col, lm, y, n, 3, 0, &ctx), ctx);
    printf("colours %d\n", K);
    if (lockstep(ctx, n, f)) return 1;  /* (CHECK destroyed the context) */
    nngp_ctx_destroy(ctx);
    free(raw); free(locs); free(order); free(NN); free(col); free(lm); free(y); free(f);
    return 0;
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
