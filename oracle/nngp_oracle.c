/*
 * nngp_oracle.c -- CPU ORACLE (test infrastructure ONLY).
 *
 * This file is a plain-C restatement of the reference's NNGP chromatic-Gibbs
 * hot path.  It is the CHECKER for the HIP product path: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product (libnngp.so) never links, calls or falls back to it.
 *
 * Reference followed (R scripts + the un-vendored CRAN packages they call):
 *   - ll_compressed_sparse_chol ........ Scripts/mcmc_nngp_update_Gaussian.R:8-12
 *   - GpGp::Linv_mult .................. (called at update_Gaussian.R:10)
 *   - GpGp::vecchia_Linv ............... (called at update_Gaussian.R:72,123,179;
 *                                         mcmc_nngp_initialize.R:201)
 *   - precision_diag ................... update_Gaussian.R:74,142,197
 *   - residuals_sum .................... update_Gaussian.R:90,260
 *   - chromatic sweep (masked form) .... update_Gaussian.R:257-275
 *   - GpGp::find_ordered_nn ............ mcmc_nngp_initialize.R:93
 *   - moral graph + greedy coloring .... mcmc_nngp_initialize.R:97-110,
 *                                         Scripts/Coloring.R:2-20
 *   - sparse triangular solve .......... update_Gaussian.R:127, initialize.R:208
 *
 * GpGp / Matrix / FNN are NOT present in this image: the
 * GpGp functions are restated from their published algorithm (GpGp ~0.3/0.4,
 * inferred from the 2021-06-14 vignette render; version unpinned).  Pinning:
 * NNarray rows, the moral-graph block and (implicitly) the first colours are
 * pinned by the golden values printed in Vignette.md (tests/golden); the
 * numerical kernels (vecchia_Linv, Linv_mult, sweep) are pinned by
 * mathematical known-answer tests (dense inverse Cholesky, dense MVN density,
 * dense Gaussian conditionals) -- see DESIGN.md "Parity".
 *
 * Conventions (same as R): matrices are column-major; NNarray is n x (m+1),
 * 1-based, with NA encoded as INT_MIN (R's NA_INTEGER); coloring is 1-based.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <limits.h>

#define OR_NA INT_MIN

/* ------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al. 2011, Random123).  Counter-based RNG used */
/* by the product for the per-location normals of the chromatic sweep.   */
/* ------------------------------------------------------------------ */
static void or_philox_round(uint32_t c[4], const uint32_t k[2]) {
  uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  uint32_t n0 = hi1 ^ c[1] ^ k[0];
  uint32_t n2 = hi0 ^ c[3] ^ k[1];
  c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  uint32_t k[2] = {key[0], key[1]};
  for (int r = 0; r < 10; ++r) {
    if (r) { k[0] += 0x9E3779B9u; k[1] += 0xBB67AE85u; }
    or_philox_round(c, k);
  }
  out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
}

/* Standard normal by inversion, Wichura's AS241 (PPND16) -- the algorithm of
 * R's qnorm, which R's default norm_rand (INVERSION) applies to a uniform. */
double or_qnorm(double p) {
  double q = p - 0.5, r, val;
  if (fabs(q) <= 0.425) {
    r = 0.180625 - q * q;
    return q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r +
                    45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
                  133.14166789178437745) * r + 3.387132872796366608) /
           (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r +
                 21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
             42.313330701600911252) * r + 1.);
  }
  r = q < 0 ? p : 1.0 - p;
  r = sqrt(-log(r));
  if (r <= 5.) {
    r -= 1.6;
    val = (((((((r * 7.7454501427834140764e-4 + .0227238449892691845833) * r + .24178072517745061177) * r +
               1.27045825245236838258) * r + 3.64784832476320460504) * r + 5.7694972214606914055) * r +
             4.6303378461565452959) * r + 1.42343711074968357734) /
          (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r + .0151986665636164571966) * r +
               .14810397642748007459) * r + .68976733498510000455) * r + 1.6763848301838038494) * r +
             2.05319162663775882187) * r + 1.);
  } else {
    r -= 5.;
    val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r + .0012426609473880784386) * r +
               .026532189526576123093) * r + .29656057182850489123) * r + 1.7848265399172913358) * r +
             5.4637849111641143699) * r + 6.6579046435011037772) /
          (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r + 1.8463183175100546818e-5) * r +
               7.868691311456132591e-4) * r + .0148753612908506148525) * r + .13692988092273580531) * r +
             .59983220655588793769) * r + 1.);
  }
  return q < 0.0 ? -val : val;
}

/* Standard normal for location `loc` (0-based) in global sweep `sweep` with
 * 64-bit `seed`: one Philox call per location, counter = (loc, sweep_lo,
 * sweep_hi, 0x5EEDu), key = seed; its first 53 bits give u in (0,1) and the
 * normal is qnorm(u). */
double or_normal(uint64_t seed, uint64_t sweep, uint32_t loc) {
  uint32_t ctr[4] = {loc, (uint32_t)sweep, (uint32_t)(sweep >> 32), 0x5EEDu};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  or_philox4x32_10(ctr, key, o);
  uint64_t a = (((uint64_t)o[1] << 32) | o[0]) >> 11;
  return or_qnorm(((double)a + 0.5) * 0x1.0p-53);   /* u in (0,1) */
}

void or_normals(uint64_t seed, uint64_t sweep, int n, double *z) {
  for (int i = 0; i < n; ++i) z[i] = or_normal(seed, sweep, (uint32_t)i);
}

/* ------------------------------------------------------------------ */
/* GpGp covariance functions (unit-free restatement).                  */
/* ids: 0 exponential_isotropic, 1 exponential_sphere,                 */
/*      2 exponential_scaledim, 3 exponential_spacetime,               */
/*      4 matern_isotropic, 5 matern_sphere, 6 matern_scaledim,        */
/*      7 matern_spacetime, 8 matern15_isotropic (extension)           */
/* ------------------------------------------------------------------ */

/* K_nu(x) by the integral representation K_nu(x) = int_0^inf exp(-x cosh t)
 * cosh(nu t) dt, trapezoid rule (spectrally accurate for this integrand).
 * Deliberately a different algorithm from the product's Temme/Steed code. */
double or_bessel_k(double nu, double x) {
  double h = 0.01;
  double T = log(2.0 * 800.0 / x) + 2.0;
  if (T < 5.0) T = 5.0;
  int nt = (int)(T / h) + 1;
  double s = 0.5 * exp(-x);
  for (int i = 1; i <= nt; ++i) {
    double t = i * h;
    double e = x * cosh(t);
    if (e > 745.0) break;
    s += exp(-e) * cosh(nu * t);
  }
  return s * h;
}

static double or_matern_corr(double nu, double d) {
  if (d == 0.0) return 1.0;
  double lg = lgamma(nu);
  double norm = exp((1.0 - nu) * log(2.0) - lg);
  return norm * pow(d, nu) * or_bessel_k(nu, d);
}

/* number of covariance parameters for a covfun id and dimension d */
int or_ncovparms(int covfun, int d) {
  switch (covfun) {
    case 0: case 1: case 8: return 3;
    case 2: return d + 2;
    case 3: return 4;
    case 4: case 5: return 4;
    case 6: return d + 3;
    case 7: return 5;
  }
  return -1;
}

/* transform raw coordinates into the space where the covariance is isotropic
 * with unit range; writes up to 3 coords to out, returns dimension. */
static int or_scaled_coords(int covfun, const double *cp, const double *x, int d, double *out) {
  switch (covfun) {
    case 0: case 4: case 8:
      for (int k = 0; k < d; ++k) out[k] = x[k] / cp[1];
      return d;
    case 1: case 5: {
      double lon = x[0] * 3.14159265358979323846 / 180.0;
      double lat = x[1] * 3.14159265358979323846 / 180.0;
      out[0] = cos(lat) * cos(lon) / cp[1];
      out[1] = cos(lat) * sin(lon) / cp[1];
      out[2] = sin(lat) / cp[1];
      return 3;
    }
    case 2: case 6:
      for (int k = 0; k < d; ++k) out[k] = x[k] / cp[1 + k];
      return d;
    case 3: case 7:
      for (int k = 0; k < d - 1; ++k) out[k] = x[k] / cp[1];
      out[d - 1] = x[d - 1] / cp[2];
      return d;
  }
  return 0;
}

static double or_cov_of_dist(int covfun, const double *cp, int d, double dist) {
  double var = cp[0];
  switch (covfun) {
    case 0: case 1: case 2: case 3:
      return var * exp(-dist);
    case 8:
      return var * (1.0 + dist) * exp(-dist);
    case 4: case 5: return var * or_matern_corr(cp[2], dist);
    case 6: return var * or_matern_corr(cp[1 + d], dist);
    case 7: return var * or_matern_corr(cp[3], dist);
  }
  return NAN;
}

static double or_nugget(int covfun, const double *cp, int d) {
  return cp[or_ncovparms(covfun, d) - 1];
}

/* Dense covariance matrix (column-major nloc x nloc) of locs (nloc x d,
 * column-major, leading dimension ld). */
void or_covmat(int covfun, const double *cp, const double *locs, int nloc, int d, int ld, double *C) {
  double a[3], b[3], xa[8], xb[8];
  for (int i = 0; i < nloc; ++i) {
    for (int k = 0; k < d; ++k) xa[k] = locs[i + (size_t)k * ld];
    int dd = or_scaled_coords(covfun, cp, xa, d, a);
    for (int j = 0; j <= i; ++j) {
      for (int k = 0; k < d; ++k) xb[k] = locs[j + (size_t)k * ld];
      or_scaled_coords(covfun, cp, xb, d, b);
      double s = 0;
      for (int k = 0; k < dd; ++k) s += (a[k] - b[k]) * (a[k] - b[k]);
      double c = or_cov_of_dist(covfun, cp, d, sqrt(s));
      if (i == j) c += cp[0] * or_nugget(covfun, cp, d);
      C[i + (size_t)j * nloc] = c;
      C[j + (size_t)i * nloc] = c;
    }
  }
}

/* textbook (Cholesky-Banachiewicz) lower Cholesky, in place, col-major.
 * returns 0 on success, (row+1) of the failing pivot otherwise */
int or_chol_lower(double *A, int nn) {
  for (int j = 0; j < nn; ++j) {
    double s = A[j + (size_t)j * nn];
    for (int p = 0; p < j; ++p) s -= A[j + (size_t)p * nn] * A[j + (size_t)p * nn];
    if (!(s > 0.0)) return j + 1;
    double ljj = sqrt(s);
    A[j + (size_t)j * nn] = ljj;
    for (int i = j + 1; i < nn; ++i) {
      double t = A[i + (size_t)j * nn];
      for (int p = 0; p < j; ++p) t -= A[i + (size_t)p * nn] * A[j + (size_t)p * nn];
      A[i + (size_t)j * nn] = t / ljj;
    }
    for (int i = 0; i < j; ++i) A[i + (size_t)j * nn] = 0.0;
  }
  return 0;
}

/* GpGp::vecchia_Linv restated: for row i, bsize = min(i+1, b); locsub =
 * locs[rev(NNarray[i, 1:bsize])] (self last); L = chol(covmat(locsub));
 * choli2 = solve(t(L), e_last); Linv[i, j] = choli2[bsize-1-j].
 * Linv: n x b column-major, unfilled entries 0.  Returns 0 or (i+1) of the
 * first row whose local covariance is not positive definite. */
int or_vecchia_linv(int covfun, const double *cp, const double *locs, int n, int d,
                    const int *NN, int b, double *Linv) {
  double *sub = (double *)malloc(sizeof(double) * (size_t)b * d);
  double *C = (double *)malloc(sizeof(double) * (size_t)b * b);
  double *x = (double *)malloc(sizeof(double) * (size_t)b);
  int fail = 0;
  memset(Linv, 0, sizeof(double) * (size_t)n * b);
  for (int i = 0; i < n && !fail; ++i) {
    int bs = i + 1 < b ? i + 1 : b;
    for (int r = 0; r < bs; ++r) {
      int idx = NN[i + (size_t)(bs - 1 - r) * n] - 1;
      for (int k = 0; k < d; ++k) sub[r + (size_t)k * bs] = locs[idx + (size_t)k * n];
    }
    or_covmat(covfun, cp, sub, bs, d, bs, C);
    if (or_chol_lower(C, bs)) { fail = i + 1; break; }
    /* back substitution L^T x = e_last */
    for (int r = bs - 1; r >= 0; --r) {
      double s = (r == bs - 1) ? 1.0 : 0.0;
      for (int q = r + 1; q < bs; ++q) s -= C[q + (size_t)r * bs] * x[q];
      x[r] = s / C[r + (size_t)r * bs];
    }
    for (int j = 0; j < bs; ++j) Linv[i + (size_t)j * n] = x[bs - 1 - j];
  }
  free(sub); free(C); free(x);
  return fail;
}

/* GpGp::Linv_mult: u_i = sum_j Linv[i,j] z[NNarray[i,j]] over non-NA j */
void or_linv_mult(const double *Linv, const double *z, const int *NN, int n, int b, double *u) {
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int j = 0; j < b; ++j) {
      int idx = NN[i + (size_t)j * n];
      if (idx == OR_NA) continue;
      s += Linv[i + (size_t)j * n] * z[idx - 1];
    }
    u[i] = s;
  }
}

/* ll_compressed_sparse_chol (update_Gaussian.R:8-12) */
double or_loglik(const double *Linv, const double *z, const int *NN, int n, int b, double log_scale) {
  double *u = (double *)malloc(sizeof(double) * (size_t)n);
  or_linv_mult(Linv, z, NN, n, b, u);
  double slog = 0, sq = 0;
  for (int i = 0; i < n; ++i) { slog += log(Linv[i]); sq += u[i] * u[i]; }
  free(u);
  return slog - n * 0.5 * log_scale - 0.5 * sq / exp(log_scale);
}

/* precision_diag = colSums(B o B) (update_Gaussian.R:74) */
void or_precision_diag(const double *Linv, const int *NN, int n, int b, double *D) {
  memset(D, 0, sizeof(double) * (size_t)n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < b; ++j) {
      int idx = NN[i + (size_t)j * n];
      if (idx == OR_NA) continue;
      double v = Linv[i + (size_t)j * n];
      D[idx - 1] += v * v;
    }
}

/* residuals_sum = residuals_sum_matrix %*% (y - mu)  (update_Gaussian.R:90,260) */
void or_residuals_sum(const double *y, const double *mu, const int *locs_match, int n_obs, int n, double *R) {
  memset(R, 0, sizeof(double) * (size_t)n);
  for (int o = 0; o < n_obs; ++o) R[locs_match[o] - 1] += y[o] - mu[o];
}

/* ------------------------------------------------------------------ */
/* Chromatic sweep, reference-faithful MASKED form                     */
/* (update_Gaussian.R:257-275): per colour, a full SpMV of B on the     */
/* masked field and a column-subset crossprod.                          */
/* z: n_sweeps x n, z[s*n + i] is the normal used for location i in     */
/* sweep s (the reference draws rnorm(length(selected_locs)) in the     */
/* order of `which`; here the normal is addressed by location).         */
/* ------------------------------------------------------------------ */
void or_sweep_masked(int n_sweeps, const double *Linv, const int *NN, int n, int b,
                     const int *coloring, const double *D, const int *obs_per_loc,
                     const double *y, const double *mu, const int *locs_match, int n_obs,
                     double beta0, double log_scale, double log_noise_var,
                     const double *z, double *field) {
  int K = 0;
  for (int i = 0; i < n; ++i) if (coloring[i] > K) K = coloring[i];
  double *R = (double *)malloc(sizeof(double) * (size_t)n);
  double *w = (double *)malloc(sizeof(double) * (size_t)n);
  double *v = (double *)malloc(sizeof(double) * (size_t)n);
  double *t = (double *)malloc(sizeof(double) * (size_t)n);
  double is2 = exp(-log_scale), it2 = exp(-log_noise_var);
  for (int s = 0; s < n_sweeps; ++s) {
    or_residuals_sum(y, mu, locs_match, n_obs, n, R);
    for (int c = 1; c <= K; ++c) {  /* unique(coloring) == 1..K for first-fit */
      for (int i = 0; i < n; ++i) w[i] = (coloring[i] != c) ? field[i] - beta0 : 0.0;
      or_linv_mult(Linv, w, NN, n, b, v);          /* B %*% (masked field) */
      for (int i = 0; i < n; ++i) t[i] = 0.0;
      for (int k = 0; k < n; ++k)                   /* crossprod(B[,sel], v) */
        for (int j = 0; j < b; ++j) {
          int idx = NN[k + (size_t)j * n];
          if (idx == OR_NA) continue;
          if (coloring[idx - 1] == c) t[idx - 1] += Linv[k + (size_t)j * n] * v[k];
        }
      for (int i = 0; i < n; ++i) {
        if (coloring[i] != c) continue;
        double P = is2 * D[i] + it2 * obs_per_loc[i];
        double cm = beta0 - (1.0 / P) * (t[i] * is2 - it2 * R[i]);
        field[i] = cm + z[(size_t)s * n + i] / sqrt(P);
      }
    }
  }
  free(R); free(w); free(v); free(t);
}

/* ------------------------------------------------------------------ */
/* Chromatic sweep, LOCAL form: r = B w is formed once per call, then    */
/* (B^T B w_{!c})_i = sum_{k: B[k,i]!=0} B[k,i] r_k - D_i w_i and        */
/* r_k += B[k,i] dw_i after each location update (conflict-free within a */
/* colour: every Vecchia row is a clique of the moral graph).            */
/* ------------------------------------------------------------------ */
void or_sweep_local(int n_sweeps, const double *Linv, const int *NN, int n, int b,
                    const int *coloring, const double *D, const int *obs_per_loc,
                    const double *y, const double *mu, const int *locs_match, int n_obs,
                    double beta0, double log_scale, double log_noise_var,
                    const double *z, double *field) {
  int K = 0;
  for (int i = 0; i < n; ++i) if (coloring[i] > K) K = coloring[i];
  /* CSC of B: column i -> (row k, value) */
  int *cnt = (int *)calloc((size_t)n + 1, sizeof(int));
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < b; ++j) {
      int idx = NN[k + (size_t)j * n];
      if (idx != OR_NA) cnt[idx]++;
    }
  for (int i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
  int nnz = cnt[n];
  int *crow = (int *)malloc(sizeof(int) * (size_t)nnz);
  double *cval = (double *)malloc(sizeof(double) * (size_t)nnz);
  int *fill = (int *)malloc(sizeof(int) * (size_t)n);
  memcpy(fill, cnt, sizeof(int) * (size_t)n);
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < b; ++j) {
      int idx = NN[k + (size_t)j * n];
      if (idx == OR_NA) continue;
      int p = fill[idx - 1]++;
      crow[p] = k; cval[p] = Linv[k + (size_t)j * n];
    }
  /* colour lists in index order */
  int *cptr = (int *)calloc((size_t)K + 2, sizeof(int));
  for (int i = 0; i < n; ++i) cptr[coloring[i] + 1]++;
  for (int c = 0; c <= K; ++c) cptr[c + 1] += cptr[c];
  int *clist = (int *)malloc(sizeof(int) * (size_t)n);
  int *cfill = (int *)malloc(sizeof(int) * ((size_t)K + 1));
  memcpy(cfill, cptr, sizeof(int) * ((size_t)K + 1));
  for (int i = 0; i < n; ++i) clist[cfill[coloring[i]]++] = i;

  double *R = (double *)malloc(sizeof(double) * (size_t)n);
  double *w = (double *)malloc(sizeof(double) * (size_t)n);
  double *r = (double *)malloc(sizeof(double) * (size_t)n);
  double is2 = exp(-log_scale), it2 = exp(-log_noise_var);
  or_residuals_sum(y, mu, locs_match, n_obs, n, R);
  for (int i = 0; i < n; ++i) w[i] = field[i] - beta0;
  or_linv_mult(Linv, w, NN, n, b, r);
  for (int s = 0; s < n_sweeps; ++s) {
    for (int c = 1; c <= K; ++c) {
      for (int q = cptr[c]; q < cptr[c + 1]; ++q) {
        int i = clist[q];
        double acc = 0;
        for (int p = cnt[i]; p < cnt[i + 1]; ++p) acc += cval[p] * r[crow[p]];
        acc -= D[i] * w[i];
        double P = is2 * D[i] + it2 * obs_per_loc[i];
        double wn = (it2 * R[i] - is2 * acc) / P + z[(size_t)s * n + i] / sqrt(P);
        double dw = wn - w[i];
        w[i] = wn;
        for (int p = cnt[i]; p < cnt[i + 1]; ++p) r[crow[p]] += cval[p] * dw;
      }
    }
  }
  for (int i = 0; i < n; ++i) field[i] = w[i] + beta0;
  free(cnt); free(crow); free(cval); free(fill); free(cptr); free(clist); free(cfill);
  free(R); free(w); free(r);
}

/* ------------------------------------------------------------------ */
/* Multi-threaded forms (OpenMP) of the two sweeps above, for the CPU     */
/* baseline "one chain on all host cores" (BASELINE.md).  Bitwise equal   */
/* to the serial forms: every output element is summed by one thread in   */
/* the serial order (columns of B are walked with rows ascending, as the  */
/* serial crossprod adds them), and within a colour the local form's     */
/* row updates are disjoint (each Vecchia row is a moral clique).         */
/* ------------------------------------------------------------------ */
static void or_csc(const double *Linv, const int *NN, int n, int b, int **cnt_o, int **crow_o, double **cval_o) {
  int *cnt = (int *)calloc((size_t)n + 1, sizeof(int));
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < b; ++j) {
      int idx = NN[k + (size_t)j * n];
      if (idx != OR_NA) cnt[idx]++;
    }
  for (int i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
  int *crow = (int *)malloc(sizeof(int) * (size_t)cnt[n]);
  double *cval = (double *)malloc(sizeof(double) * (size_t)cnt[n]);
  int *fill = (int *)malloc(sizeof(int) * (size_t)n);
  memcpy(fill, cnt, sizeof(int) * (size_t)n);
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < b; ++j) {
      int idx = NN[k + (size_t)j * n];
      if (idx == OR_NA) continue;
      int p = fill[idx - 1]++;
      crow[p] = k; cval[p] = Linv[k + (size_t)j * n];
    }
  free(fill);
  *cnt_o = cnt; *crow_o = crow; *cval_o = cval;
}

static void or_colour_lists(const int *coloring, int n, int *K_o, int **cptr_o, int **clist_o) {
  int K = 0;
  for (int i = 0; i < n; ++i) if (coloring[i] > K) K = coloring[i];
  int *cptr = (int *)calloc((size_t)K + 2, sizeof(int));
  for (int i = 0; i < n; ++i) cptr[coloring[i] + 1]++;
  for (int c = 0; c <= K; ++c) cptr[c + 1] += cptr[c];
  int *clist = (int *)malloc(sizeof(int) * (size_t)n);
  int *cfill = (int *)malloc(sizeof(int) * ((size_t)K + 1));
  memcpy(cfill, cptr, sizeof(int) * ((size_t)K + 1));
  for (int i = 0; i < n; ++i) clist[cfill[coloring[i]]++] = i;
  free(cfill);
  *K_o = K; *cptr_o = cptr; *clist_o = clist;
}

void or_sweep_masked_mt(int nthreads, int n_sweeps, const double *Linv, const int *NN, int n, int b,
                        const int *coloring, const double *D, const int *obs_per_loc,
                        const double *y, const double *mu, const int *locs_match, int n_obs,
                        double beta0, double log_scale, double log_noise_var,
                        const double *z, double *field) {
  int K, *cptr, *clist, *cnt, *crow;
  double *cval;
  or_colour_lists(coloring, n, &K, &cptr, &clist);
  or_csc(Linv, NN, n, b, &cnt, &crow, &cval);
  double *R = (double *)malloc(sizeof(double) * (size_t)n);
  double *w = (double *)malloc(sizeof(double) * (size_t)n);
  double *v = (double *)malloc(sizeof(double) * (size_t)n);
  double is2 = exp(-log_scale), it2 = exp(-log_noise_var);
  for (int s = 0; s < n_sweeps; ++s) {
    or_residuals_sum(y, mu, locs_match, n_obs, n, R);
    for (int c = 1; c <= K; ++c) {
#pragma omp parallel num_threads(nthreads)
      {
#pragma omp for schedule(static)
        for (int i = 0; i < n; ++i) w[i] = (coloring[i] != c) ? field[i] - beta0 : 0.0;
#pragma omp for schedule(static)
        for (int k = 0; k < n; ++k) {       /* B %*% (masked field), row k as or_linv_mult */
          double u = 0.0;
          for (int j = 0; j < b; ++j) {
            int idx = NN[k + (size_t)j * n];
            if (idx == OR_NA) continue;
            u += Linv[k + (size_t)j * n] * w[idx - 1];
          }
          v[k] = u;
        }
#pragma omp for schedule(dynamic, 256)
        for (int q = cptr[c]; q < cptr[c + 1]; ++q) {  /* crossprod(B[,sel], v), rows ascending */
          int i = clist[q];
          double t = 0.0;
          for (int p = cnt[i]; p < cnt[i + 1]; ++p) t += cval[p] * v[crow[p]];
          double P = is2 * D[i] + it2 * obs_per_loc[i];
          double cm = beta0 - (1.0 / P) * (t * is2 - it2 * R[i]);
          field[i] = cm + z[(size_t)s * n + i] / sqrt(P);
        }
      }
    }
  }
  free(R); free(w); free(v); free(cptr); free(clist); free(cnt); free(crow); free(cval);
}

void or_sweep_local_mt(int nthreads, int n_sweeps, const double *Linv, const int *NN, int n, int b,
                       const int *coloring, const double *D, const int *obs_per_loc,
                       const double *y, const double *mu, const int *locs_match, int n_obs,
                       double beta0, double log_scale, double log_noise_var,
                       const double *z, double *field) {
  int K, *cptr, *clist, *cnt, *crow;
  double *cval;
  or_colour_lists(coloring, n, &K, &cptr, &clist);
  or_csc(Linv, NN, n, b, &cnt, &crow, &cval);
  double *R = (double *)malloc(sizeof(double) * (size_t)n);
  double *w = (double *)malloc(sizeof(double) * (size_t)n);
  double *r = (double *)malloc(sizeof(double) * (size_t)n);
  double is2 = exp(-log_scale), it2 = exp(-log_noise_var);
  or_residuals_sum(y, mu, locs_match, n_obs, n, R);
  for (int i = 0; i < n; ++i) w[i] = field[i] - beta0;
  or_linv_mult(Linv, w, NN, n, b, r);
  for (int s = 0; s < n_sweeps; ++s)
    for (int c = 1; c <= K; ++c) {
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 256)
      for (int q = cptr[c]; q < cptr[c + 1]; ++q) {
        int i = clist[q];
        double acc = 0;
        for (int p = cnt[i]; p < cnt[i + 1]; ++p) acc += cval[p] * r[crow[p]];
        acc -= D[i] * w[i];
        double P = is2 * D[i] + it2 * obs_per_loc[i];
        double wn = (it2 * R[i] - is2 * acc) / P + z[(size_t)s * n + i] / sqrt(P);
        double dw = wn - w[i];
        w[i] = wn;
        for (int p = cnt[i]; p < cnt[i + 1]; ++p) r[crow[p]] += cval[p] * dw;
      }
    }
  for (int i = 0; i < n; ++i) field[i] = w[i] + beta0;
  free(R); free(w); free(r); free(cptr); free(clist); free(cnt); free(crow); free(cval);
}

/* ------------------------------------------------------------------ */
/* GpGp::find_ordered_nn restated (exact, no jitter): row i = [i, the m  */
/* nearest j < i by ascending Euclidean distance on the raw coordinates, */
/* ties broken by smaller index], NA-padded.  Brute force O(n^2 m).      */
/* ------------------------------------------------------------------ */
void or_find_ordered_nn(const double *locs, int n, int d, int m, int *NN) {
  int b = m + 1;
  double *bd = (double *)malloc(sizeof(double) * (size_t)b);
  int *bi = (int *)malloc(sizeof(int) * (size_t)b);
  for (int i = 0; i < n; ++i) {
    int cnt = 0;
    for (int j = 0; j < i; ++j) {
      double s = 0;
      for (int k = 0; k < d; ++k) {
        double t = locs[i + (size_t)k * n] - locs[j + (size_t)k * n];
        s += t * t;
      }
      /* insert (s, j) into sorted list of size <= m (stable: j increasing) */
      if (cnt < m || s < bd[cnt - 1]) {
        int p = cnt < m ? cnt++ : cnt - 1;
        while (p > 0 && bd[p - 1] > s) { bd[p] = bd[p - 1]; bi[p] = bi[p - 1]; --p; }
        bd[p] = s; bi[p] = j;
      }
    }
    NN[i] = i + 1;
    for (int j = 1; j < b; ++j) NN[i + (size_t)j * n] = (j - 1 < cnt) ? bi[j - 1] + 1 : OR_NA;
  }
  free(bd); free(bi);
}

/* ------------------------------------------------------------------ */
/* Moral graph (initialize.R:103-109) + naive_greedy_coloring           */
/* (Coloring.R:2-20), restated with the reference's data flow: build     */
/* M = pattern(crossprod(B)) with full columns incl. the diagonal, the   */
/* degree vector, the (n+1) x max(degree) incompatibility matrix, then   */
/* cols[i] = match(0, incompat[i,]); incompat[adj(i), cols[i]] = 1.      */
/* Returns K, or -1 on allocation failure.                               */
/* ------------------------------------------------------------------ */
int or_moral_graph(const int *NN, int n, int b, int **colptr_out, int **rowidx_out) {
  /* rows of B: members of row k */
  /* adjacency sets via sort-unique per column */
  int *deg = (int *)calloc((size_t)n + 1, sizeof(int));
  for (int k = 0; k < n; ++k) {
    int cntk = 0;
    for (int j = 0; j < b; ++j) if (NN[k + (size_t)j * n] != OR_NA) cntk++;
    for (int j = 0; j < b; ++j) {
      int a = NN[k + (size_t)j * n];
      if (a == OR_NA) continue;
      deg[a] += cntk;  /* upper bound incl. duplicates */
    }
  }
  for (int i = 0; i < n; ++i) deg[i + 1] += deg[i];
  int tot = deg[n];
  int *tmp = (int *)malloc(sizeof(int) * (size_t)(tot > 0 ? tot : 1));
  int *fill = (int *)malloc(sizeof(int) * (size_t)n);
  memcpy(fill, deg, sizeof(int) * (size_t)n);
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < b; ++j) {
      int a = NN[k + (size_t)j * n];
      if (a == OR_NA) continue;
      for (int q = 0; q < b; ++q) {
        int c = NN[k + (size_t)q * n];
        if (c == OR_NA) continue;
        tmp[fill[a - 1]++] = c - 1;
      }
    }
  /* sort + unique each column (insertion sort: columns are short) */
  int *colptr = (int *)malloc(sizeof(int) * ((size_t)n + 1));
  int *rowidx = (int *)malloc(sizeof(int) * (size_t)(tot > 0 ? tot : 1));
  int nz = 0;
  colptr[0] = 0;
  for (int i = 0; i < n; ++i) {
    int lo = deg[i], hi = fill[i];
    for (int p = lo + 1; p < hi; ++p) {
      int v = tmp[p], q = p;
      while (q > lo && tmp[q - 1] > v) { tmp[q] = tmp[q - 1]; --q; }
      tmp[q] = v;
    }
    for (int p = lo; p < hi; ++p)
      if (p == lo || tmp[p] != tmp[p - 1]) rowidx[nz++] = tmp[p];
    colptr[i + 1] = nz;
  }
  free(deg); free(tmp); free(fill);
  *colptr_out = colptr; *rowidx_out = rowidx;
  return nz;
}

void or_free(void *p) { free(p); }

int or_greedy_coloring(const int *NN, int n, int b, int *cols) {
  int *colptr, *rowidx;
  or_moral_graph(NN, n, b, &colptr, &rowidx);
  int maxdeg = 0;
  for (int i = 0; i < n; ++i) {
    int dg = colptr[i + 1] - colptr[i];
    if (dg > maxdeg) maxdeg = dg;
  }
  unsigned char *inc = (unsigned char *)calloc(((size_t)n + 1) * (size_t)maxdeg, 1);
  if (!inc) { free(colptr); free(rowidx); return -1; }
  int K = 0;
  for (int i = 0; i < n; ++i) {
    int c = 0;
    while (c < maxdeg && inc[(size_t)i * maxdeg + c]) ++c;
    cols[i] = c + 1;  /* match(0, incompat[i,]) */
    if (c + 1 > K) K = c + 1;
    for (int p = colptr[i]; p < colptr[i + 1]; ++p) inc[(size_t)rowidx[p] * maxdeg + c] = 1;
  }
  free(inc); free(colptr); free(rowidx);
  return K;
}

/* ------------------------------------------------------------------ */
/* Sparse lower-triangular solve B x = u (Matrix::solve(sparse_chol, .), */
/* update_Gaussian.R:127, initialize.R:208): forward substitution.      */
/* ------------------------------------------------------------------ */
void or_tri_solve(const double *Linv, const int *NN, int n, int b, const double *u, double *x) {
  for (int i = 0; i < n; ++i) {
    double s = u[i];
    for (int j = 1; j < b; ++j) {
      int idx = NN[i + (size_t)j * n];
      if (idx == OR_NA) continue;
      s -= Linv[i + (size_t)j * n] * x[idx - 1];
    }
    x[i] = s / Linv[i];
  }
}

/* exact max-min ordering, O(n^2): first point closest to the centroid,
 * then repeatedly the point with the largest distance to the selected set
 * (ties: smaller index).  order: 1-based permutation. */
void or_order_maxmin_exact(const double *locs, int n, int d, int *order) {
  double *dist = (double *)malloc(sizeof(double) * (size_t)n);
  char *used = (char *)calloc((size_t)n, 1);
  double cen[8] = {0};
  for (int k = 0; k < d; ++k) {
    for (int i = 0; i < n; ++i) cen[k] += locs[i + (size_t)k * n];
    cen[k] /= n;
  }
  int first = 0; double best = INFINITY;
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int k = 0; k < d; ++k) { double t = locs[i + (size_t)k * n] - cen[k]; s += t * t; }
    if (s < best) { best = s; first = i; }
  }
  for (int i = 0; i < n; ++i) dist[i] = INFINITY;
  int cur = first;
  for (int q = 0; q < n; ++q) {
    order[q] = cur + 1;
    used[cur] = 1;
    int nxt = -1; double bd = -1;
    for (int i = 0; i < n; ++i) {
      if (used[i]) continue;
      double s = 0;
      for (int k = 0; k < d; ++k) { double t = locs[i + (size_t)k * n] - locs[cur + (size_t)k * n]; s += t * t; }
      if (s < dist[i]) dist[i] = s;
      if (dist[i] > bd) { bd = dist[i]; nxt = i; }
    }
    cur = nxt;
  }
  free(dist); free(used);
}
