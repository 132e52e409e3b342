/*
 * nngp_shim.c -- R .Call shim over the C ABI of include/nngp.h.
 *
 * One .Call entry point per nngp.h function (R_registerRoutines below), so
 * the R host code of the reference (Scripts/mcmc_nngp_*.R) can drive the
 * MI355X hot path.  Conventions:
 *  - a context is an external pointer with a finalizer (nngp_ctx_destroy);
 *  - R's own arrays cross unchanged (column-major, 1-based, NA_integer_ ==
 *    INT_MIN), integers as INTSXP, reals as REALSXP; uint64 seeds / counters
 *    arrive as doubles (exact below 2^53);
 *  - a non-zero nngp_status becomes Rf_error with the context's message.
 *    The library is C/C++ behind a C ABI and has returned before Rf_error
 *    runs, so no longjmp crosses a C++ frame; temporaries are R-allocated.
 *  - HIP must not be initialised before a fork(): the R side replaces
 *    parallel::mclapply over chains (update_Gaussian.R:25-26) by contexts
 *    holding up to 4 chains each.
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <stdint.h>
#include <string.h>

#include "nngp.h"
#include "nngp_rows.h"

static SEXP ctx_tag(void) { return Rf_install("nngp_ctx"); }

/* The external pointer's protected slot: a list of kKeep + 1 entries, [k] =
 * the numeric vector bound to chain k by C_nngp_records_stream (kept alive
 * while the library may stream rows into it, whatever happens to the R
 * variables that referenced it), [kKeep] = the selected chain (INTSXP). */
#define kKeep 4

static void ctx_finalizer(SEXP p) {
  nngp_ctx* c = (nngp_ctx*)R_ExternalPtrAddr(p);
  if (c) {
    nngp_ctx_destroy(c);
    R_ClearExternalPtr(p);
  }
}

static SEXP wrap_ctx(nngp_ctx* c) {
  SEXP keep = PROTECT(Rf_allocVector(VECSXP, kKeep + 1));
  SET_VECTOR_ELT(keep, kKeep, Rf_ScalarInteger(0));  /* a new context selects chain 0 */
  SEXP p = PROTECT(R_MakeExternalPtr(c, ctx_tag(), keep));
  R_RegisterCFinalizerEx(p, ctx_finalizer, TRUE);
  UNPROTECT(2);
  return p;
}

/* the bound records vector of the selected chain (R_NilValue: none) */
static void keep_bound(SEXP p, SEXP buf) {
  SEXP keep = R_ExternalPtrProtected(p);
  if (TYPEOF(keep) != VECSXP) return;
  const int k = INTEGER(VECTOR_ELT(keep, kKeep))[0];
  if (k >= 0 && k < kKeep) SET_VECTOR_ELT(keep, k, buf);
}

static nngp_ctx* get_ctx(SEXP p) {
  if (TYPEOF(p) != EXTPTRSXP || R_ExternalPtrTag(p) != ctx_tag()) Rf_error("nngp: not a context");
  nngp_ctx* c = (nngp_ctx*)R_ExternalPtrAddr(p);
  if (!c) Rf_error("nngp: the context was destroyed");
  return c;
}

/* status -> R error (message copied first: the context may be gone after) */
static void check(int st, const nngp_ctx* c) {
  if (st == NNGP_OK) return;
  char msg[512];
  const char* m = c ? nngp_ctx_last_error(c) : NULL;
  snprintf(msg, sizeof msg, "nngp: %s%s%s", nngp_status_string(st), (m && m[0]) ? ": " : "", m ? m : "");
  Rf_error("%s (status %d)", msg, st);
}

static int as_int(SEXP x) { return Rf_asInteger(x); }
static double as_real(SEXP x) { return Rf_asReal(x); }
static const double* rptr(SEXP x) { return TYPEOF(x) == NILSXP ? NULL : REAL(x); }

static void to_u64(SEXP x, uint64_t* out, int n) {
  if (TYPEOF(x) != REALSXP || XLENGTH(x) != n) Rf_error("nngp: need %d seeds / counters (double)", n);
  for (int k = 0; k < n; ++k) out[k] = (uint64_t)REAL(x)[k];
}

/* chains of the context */
static int ctx_chains(nngp_ctx* c) {
  nngp_info inf;
  check(nngp_ctx_info(c, &inf), c);
  return inf.n_chains;
}

/* a per-chain argument: a double vector with one entry per chain of the
 * context (the library reads every chain's entry; R's recycling does not
 * apply across the boundary) */
static const double* per_chain(SEXP x, int k, const char* what) {
  if (TYPEOF(x) != REALSXP || XLENGTH(x) != k)
    Rf_error("nngp: %s must be a double vector with one entry per chain (%d)", what, k);
  return REAL(x);
}

/* ---------- library ---------- */
SEXP C_nngp_abi_version(void) { return Rf_ScalarInteger(nngp_abi_version()); }
SEXP C_nngp_status_string(SEXP st) { return Rf_mkString(nngp_status_string(as_int(st))); }

/* ---------- graph preparation ---------- */
SEXP C_nngp_order_maxmin(SEXP locs) {
  int n = Rf_nrows(locs), d = Rf_ncols(locs);
  SEXP o = PROTECT(Rf_allocVector(INTSXP, n));
  check(nngp_order_maxmin(REAL(locs), n, d, INTEGER(o)), NULL);
  UNPROTECT(1);
  return o;
}

SEXP C_nngp_find_ordered_nn(SEXP locs, SEXP m) {
  int n = Rf_nrows(locs), d = Rf_ncols(locs), mm = as_int(m);
  SEXP nn = PROTECT(Rf_allocMatrix(INTSXP, n, mm + 1));
  check(nngp_find_ordered_nn(REAL(locs), n, d, mm, INTEGER(nn)), NULL);
  UNPROTECT(1);
  return nn;
}

SEXP C_nngp_greedy_coloring(SEXP NNarray) {
  int n = Rf_nrows(NNarray), b = Rf_ncols(NNarray), K = 0;
  SEXP col = PROTECT(Rf_allocVector(INTSXP, n));
  check(nngp_greedy_coloring(INTEGER(NNarray), n, b, INTEGER(col), &K), NULL);
  UNPROTECT(1);
  return col;
}

/* ---------- contexts ---------- */
SEXP C_nngp_ctx_create(SEXP locs, SEXP NNarray, SEXP coloring, SEXP locs_match, SEXP y, SEXP n_chains,
                       SEXP device) {
  nngp_ctx* c = NULL;
  check(nngp_ctx_create(REAL(locs), Rf_nrows(locs), Rf_ncols(locs), INTEGER(NNarray), Rf_ncols(NNarray),
                        INTEGER(coloring), INTEGER(locs_match), REAL(y), (int)XLENGTH(y), as_int(n_chains),
                        as_int(device), &c),
        NULL);
  return wrap_ctx(c);
}

SEXP C_nngp_ctx_create_shard(SEXP locs, SEXP NNarray, SEXP coloring, SEXP locs_match, SEXP y, SEXP n_chains,
                             SEXP device, SEXP n_ranks, SEXP rank) {
  nngp_ctx* c = NULL;
  check(nngp_ctx_create_shard(REAL(locs), Rf_nrows(locs), Rf_ncols(locs), INTEGER(NNarray), Rf_ncols(NNarray),
                              INTEGER(coloring), INTEGER(locs_match), REAL(y), (int)XLENGTH(y),
                              as_int(n_chains), as_int(device), as_int(n_ranks), as_int(rank), &c),
        NULL);
  return wrap_ctx(c);
}

SEXP C_nngp_ctx_destroy(SEXP p) {
  ctx_finalizer(p);
  return R_NilValue;
}

SEXP C_nngp_ctx_last_error(SEXP p) { return Rf_mkString(nngp_ctx_last_error(get_ctx(p))); }

SEXP C_nngp_set_chain(SEXP p, SEXP chain) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_set_chain(c, as_int(chain)), c);
  SEXP keep = R_ExternalPtrProtected(p);
  if (TYPEOF(keep) == VECSXP) INTEGER(VECTOR_ELT(keep, kKeep))[0] = as_int(chain);
  return R_NilValue;
}

SEXP C_nngp_ctx_engine_note(SEXP p) { return Rf_mkString(nngp_ctx_engine_note(get_ctx(p))); }

SEXP C_nngp_ctx_info(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  nngp_info inf;
  check(nngp_ctx_info(c, &inf), c);
  const char* nm[] = {"n", "b", "d", "n_obs", "n_colors", "n_levels", "nnz", "n_entries", "max_collen", "device",
                      "n_chains", "lanes_per_chain", "n_chunks", "sweep_engine", "n_tiles", "tile_rows_max",
                      "n_ghost_cells", "n_ranks", "rank", "shard_owned", "shard_needed_rows",
                      "shard_exchange_slots", "tile_ghost_pass", "tile_ghost_cells_max", "tile_r_global",
                      "tile_chain_split", "tile_resident_per_cu", "engine_fallback", "tile_exchange_wave",
                      "device_cus"};
  const double v[] = {inf.n, inf.b, inf.d, inf.n_obs, inf.n_colors, inf.n_levels, (double)inf.nnz,
                      (double)inf.n_entries, inf.max_collen, inf.device, inf.n_chains, inf.lanes_per_chain,
                      inf.n_chunks, inf.sweep_engine, inf.n_tiles, inf.tile_rows_max, (double)inf.n_ghost_cells,
                      inf.n_ranks, inf.rank, (double)inf.shard_owned, (double)inf.shard_needed_rows,
                      (double)inf.shard_exchange_slots, inf.tile_ghost_pass, inf.tile_ghost_cells_max,
                      inf.tile_r_global, inf.tile_chain_split, inf.tile_resident_per_cu, inf.engine_fallback,
                      inf.tile_exchange_wave, inf.device_cus};
  const int k = (int)(sizeof v / sizeof v[0]);
  SEXP out = PROTECT(Rf_allocVector(REALSXP, k)), names = PROTECT(Rf_allocVector(STRSXP, k));
  for (int i = 0; i < k; ++i) {
    REAL(out)[i] = v[i];
    SET_STRING_ELT(names, i, Rf_mkChar(nm[i]));
  }
  Rf_setAttrib(out, R_NamesSymbol, names);
  UNPROTECT(2);
  return out;
}

/* ---------- factor (A4/A5) ---------- */
SEXP C_nngp_factor(SEXP p, SEXP which, SEXP covfun, SEXP covparms) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_factor(c, as_int(which), as_int(covfun), REAL(covparms), (int)XLENGTH(covparms)), c);
  return R_NilValue;
}

SEXP C_nngp_get_linv(SEXP p, SEXP which) {
  nngp_ctx* c = get_ctx(p);
  nngp_info inf;
  check(nngp_ctx_info(c, &inf), c);
  SEXP L = PROTECT(Rf_allocMatrix(REALSXP, inf.n, inf.b));
  check(nngp_get_linv(c, as_int(which), REAL(L)), c);
  UNPROTECT(1);
  return L;
}

SEXP C_nngp_set_linv(SEXP p, SEXP which, SEXP Linv) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_set_linv(c, as_int(which), REAL(Linv)), c);
  return R_NilValue;
}

SEXP C_nngp_accept_factor(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_accept_factor(c), c);
  return R_NilValue;
}

static int ctx_n(nngp_ctx* c) {
  nngp_info inf;
  check(nngp_ctx_info(c, &inf), c);
  return inf.n;
}

SEXP C_nngp_get_precision_diag(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  SEXP D = PROTECT(Rf_allocVector(REALSXP, ctx_n(c)));
  check(nngp_get_precision_diag(c, REAL(D)), c);
  UNPROTECT(1);
  return D;
}

/* ---------- state ---------- */
SEXP C_nngp_set_field(SEXP p, SEXP field) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_set_field(c, REAL(field)), c);
  return R_NilValue;
}

SEXP C_nngp_get_field(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  SEXP f = PROTECT(Rf_allocVector(REALSXP, ctx_n(c)));
  check(nngp_get_field(c, REAL(f)), c);
  UNPROTECT(1);
  return f;
}

SEXP C_nngp_set_mu(SEXP p, SEXP mu, SEXP beta0) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_set_mu(c, rptr(mu), as_real(beta0)), c);
  return R_NilValue;
}

SEXP C_nngp_records_reserve(SEXP p, SEXP n_rows) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_records_reserve(c, as_int(n_rows)), c);
  keep_bound(p, R_NilValue);  /* a reserve ends the binding */
  return R_NilValue;
}

SEXP C_nngp_record_field(SEXP p, SEXP row) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_record_field(c, as_int(row)), c);
  return R_NilValue;
}

/* binds (or, for NULL, releases) a numeric vector of rows x n as the
 * selected chain's streamed records (row-major); the context keeps the vector
 * alive until the binding ends (R objects do not move).  A failed call
 * leaves the binding as it was (nngp.h), so does the kept reference. */
SEXP C_nngp_records_stream(SEXP p, SEXP buf) {
  nngp_ctx* c = get_ctx(p);
  if (buf == R_NilValue) {
    check(nngp_records_stream(c, NULL, 0), c);
    keep_bound(p, R_NilValue);
    return R_NilValue;
  }
  if (TYPEOF(buf) != REALSXP || XLENGTH(buf) % ctx_n(c) != 0) Rf_error("nngp: records buffer must be a numeric vector of rows x n");
  check(nngp_records_stream(c, REAL(buf), (int)(XLENGTH(buf) / ctx_n(c))), c);
  keep_bound(p, buf);
  return R_NilValue;
}

/* rows [row0, row0 + n_rows) as an n_rows x n matrix (records$field layout).
 * buf: the vector bound by C_nngp_records_stream -- the rows are already
 * there (the call waits for them and ends the binding) and are transposed
 * straight out of it; NULL: the rows come from the device in blocks of
 * kRowBlock into one small temporary, each block transposed in turn. */
#define kRowBlock 16
SEXP C_nngp_get_records(SEXP p, SEXP row0, SEXP n_rows, SEXP buf) {
  nngp_ctx* c = get_ctx(p);
  const int n = ctx_n(c), r = as_int(n_rows), r0 = as_int(row0);
  if (r < 0 || r0 < 0) Rf_error("nngp: negative record rows");
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, r, n));
  if (buf != R_NilValue) {
    if (TYPEOF(buf) != REALSXP || XLENGTH(buf) < (R_xlen_t)(r0 + r) * n) Rf_error("nngp: records buffer too short");
    check(nngp_get_records(c, r0, r, REAL(buf) + (R_xlen_t)r0 * n), c);
    keep_bound(p, R_NilValue);
    nngp_rows_to_colmajor(REAL(buf) + (R_xlen_t)r0 * n, REAL(out), r, r, n);
  } else {
    const int blk = r < kRowBlock ? r : kRowBlock;
    SEXP tmp = PROTECT(Rf_allocVector(REALSXP, (R_xlen_t)blk * n));
    for (int i = 0; i < r; i += blk) {
      const int k = r - i < blk ? r - i : blk;
      check(nngp_get_records(c, r0 + i, k, REAL(tmp)), c);
      nngp_rows_to_colmajor(REAL(tmp), REAL(out) + i, r, k, n);
    }
    UNPROTECT(1);
  }
  UNPROTECT(1);
  return out;
}

/* ---------- kernels ---------- */
SEXP C_nngp_loglik(SEXP p, SEXP which, SEXP beta0, SEXP log_scale) {
  nngp_ctx* c = get_ctx(p);
  double ll = 0;
  check(nngp_loglik(c, as_int(which), as_real(beta0), as_real(log_scale), &ll), c);
  return Rf_ScalarReal(ll);
}

SEXP C_nngp_sweep(SEXP p, SEXP n_sweeps, SEXP beta0, SEXP log_scale, SEXP lnv, SEXP seed, SEXP counter_base,
                  SEXP z) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_sweep(c, as_int(n_sweeps), as_real(beta0), as_real(log_scale), as_real(lnv),
                   (uint64_t)as_real(seed), (uint64_t)as_real(counter_base), rptr(z)),
        c);
  return R_NilValue;
}

SEXP C_nngp_sweep_chains(SEXP p, SEXP n_sweeps, SEXP beta0, SEXP log_scale, SEXP lnv, SEXP seed,
                         SEXP counter_base) {
  nngp_ctx* c = get_ctx(p);
  uint64_t s[4], cb[4];
  const int k = ctx_chains(c);
  const double *b0 = per_chain(beta0, k, "beta0"), *ls = per_chain(log_scale, k, "log_scale"),
               *nv = per_chain(lnv, k, "log_noise_variance");
  to_u64(seed, s, k);
  to_u64(counter_base, cb, k);
  check(nngp_sweep_chains(c, as_int(n_sweeps), b0, ls, nv, s, cb), c);
  return R_NilValue;
}

SEXP C_nngp_sweep_timed(SEXP p, SEXP n_sweeps, SEXP beta0, SEXP log_scale, SEXP lnv, SEXP seed,
                        SEXP counter_base) {
  nngp_ctx* c = get_ctx(p);
  uint64_t s[4], cb[4];
  const int k = ctx_chains(c);
  const double *b0 = per_chain(beta0, k, "beta0"), *ls = per_chain(log_scale, k, "log_scale"),
               *nv = per_chain(lnv, k, "log_noise_variance");
  to_u64(seed, s, k);
  to_u64(counter_base, cb, k);
  double ms = 0, kms = 0;
  check(nngp_sweep_timed(c, as_int(n_sweeps), b0, ls, nv, s, cb, &ms, &kms), c);
  SEXP out = PROTECT(Rf_allocVector(REALSXP, 2));
  REAL(out)[0] = ms;
  REAL(out)[1] = kms;
  UNPROTECT(1);
  return out;
}

SEXP C_nngp_ancillary_propose(SEXP p, SEXP beta0, SEXP dlog_scale) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_ancillary_propose(c, as_real(beta0), as_real(dlog_scale)), c);
  return R_NilValue;
}

SEXP C_nngp_ancillary_propose_chains(SEXP p, SEXP chain_mask, SEXP beta0, SEXP dlog_scale) {
  nngp_ctx* c = get_ctx(p);
  const int k = ctx_chains(c);
  check(nngp_ancillary_propose_chains(c, as_int(chain_mask), per_chain(beta0, k, "beta0"),
                                      per_chain(dlog_scale, k, "dlog_scale")),
        c);
  return R_NilValue;
}

SEXP C_nngp_field_response_ratio(SEXP p, SEXP beta0, SEXP lnv) {
  nngp_ctx* c = get_ctx(p);
  double r = 0;
  check(nngp_field_response_ratio(c, as_real(beta0), as_real(lnv), &r), c);
  return Rf_ScalarReal(r);
}

SEXP C_nngp_accept_field(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_accept_field(c), c);
  return R_NilValue;
}

SEXP C_nngp_beta0_stats(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  SEXP out = PROTECT(Rf_allocVector(REALSXP, 2));
  check(nngp_beta0_stats(c, REAL(out), REAL(out) + 1), c);
  UNPROTECT(1);
  return out;
}

SEXP C_nngp_sum_squared_residuals(SEXP p, SEXP beta0) {
  nngp_ctx* c = get_ctx(p);
  double ssr = 0;
  check(nngp_sum_squared_residuals(c, as_real(beta0), &ssr), c);
  return Rf_ScalarReal(ssr);
}

SEXP C_nngp_spmv(SEXP p, SEXP which, SEXP X) {
  nngp_ctx* c = get_ctx(p);
  const int n = ctx_n(c);
  const int ncols = Rf_isMatrix(X) ? Rf_ncols(X) : 1;
  if ((Rf_isMatrix(X) ? Rf_nrows(X) : (int)XLENGTH(X)) != n) Rf_error("nngp_spmv: X must have n rows");
  SEXP Y = PROTECT(Rf_isMatrix(X) ? Rf_allocMatrix(REALSXP, n, ncols) : Rf_allocVector(REALSXP, n));
  check(nngp_spmv(c, as_int(which), REAL(X), ncols, REAL(Y)), c);
  UNPROTECT(1);
  return Y;
}

SEXP C_nngp_tri_solve(SEXP p, SEXP which, SEXP u) {
  nngp_ctx* c = get_ctx(p);
  SEXP x = PROTECT(Rf_allocVector(REALSXP, ctx_n(c)));
  check(nngp_tri_solve(c, as_int(which), REAL(u), REAL(x)), c);
  UNPROTECT(1);
  return x;
}

SEXP C_nngp_tri_rescues(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  long long k = 0;
  check(nngp_tri_rescues(c, &k), c);
  return Rf_ScalarReal((double)k);
}

SEXP C_nngp_device_normals(SEXP device, SEXP seed, SEXP sweep, SEXP n) {
  SEXP z = PROTECT(Rf_allocVector(REALSXP, as_int(n)));
  check(nngp_device_normals(as_int(device), (uint64_t)as_real(seed), (uint64_t)as_real(sweep), as_int(n), REAL(z)),
        NULL);
  UNPROTECT(1);
  return z;
}

SEXP C_nngp_get_sweep_r(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  SEXP r = PROTECT(Rf_allocVector(REALSXP, ctx_n(c)));
  check(nngp_get_sweep_r(c, REAL(r)), c);
  UNPROTECT(1);
  return r;
}

/* ---------- sharded sweep (colour shard / tile shard) ---------- */
SEXP C_nngp_shard_unique_id(void) {
  SEXP id = PROTECT(Rf_allocVector(RAWSXP, NNGP_SHARD_ID_BYTES));
  check(nngp_shard_unique_id(RAW(id), NNGP_SHARD_ID_BYTES), NULL);
  UNPROTECT(1);
  return id;
}

SEXP C_nngp_shard_comm_init(SEXP p, SEXP id) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_shard_comm_init(c, RAW(id), (int)XLENGTH(id)), c);
  return R_NilValue;
}

SEXP C_nngp_sweep_chains_group(SEXP ctxs, SEXP n_sweeps, SEXP beta0, SEXP log_scale, SEXP lnv, SEXP seed,
                               SEXP counter_base) {
  const int G = (int)XLENGTH(ctxs);
  if (G < 1 || G > 64) Rf_error("nngp: 1..64 ranks");
  nngp_ctx* cs[64];
  for (int g = 0; g < G; ++g) cs[g] = get_ctx(VECTOR_ELT(ctxs, g));
  uint64_t s[4], cb[4];
  const int k = ctx_chains(cs[0]);
  const double *b0 = per_chain(beta0, k, "beta0"), *ls = per_chain(log_scale, k, "log_scale"),
               *nv = per_chain(lnv, k, "log_noise_variance");
  to_u64(seed, s, k);
  to_u64(counter_base, cb, k);
  check(nngp_sweep_chains_group(cs, G, as_int(n_sweeps), b0, ls, nv, s, cb), cs[0]);
  return R_NilValue;
}

/* tile shard: HIP IPC handle of this rank's granule buffer (a raw vector the
   ranks exchange out of band), and the mapping of the others' (list of raws) */
SEXP C_nngp_shard_ipc_handle(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  SEXP h = PROTECT(Rf_allocVector(RAWSXP, NNGP_IPC_HANDLE_BYTES));
  check(nngp_shard_ipc_handle(c, RAW(h), NNGP_IPC_HANDLE_BYTES), c);
  UNPROTECT(1);
  return h;
}

SEXP C_nngp_shard_sync(SEXP p) {
  nngp_ctx* c = get_ctx(p);
  check(nngp_shard_sync(c), c);
  return R_NilValue;
}

SEXP C_nngp_shard_ipc_open(SEXP p, SEXP handles) {
  nngp_ctx* c = get_ctx(p);
  const int G = (int)XLENGTH(handles);
  if (G < 1 || G > 16) Rf_error("nngp: 1..16 ranks in a tile shard");
  unsigned char buf[16 * NNGP_IPC_HANDLE_BYTES];
  for (int g = 0; g < G; ++g) {
    SEXP h = VECTOR_ELT(handles, g);
    if (TYPEOF(h) != RAWSXP || XLENGTH(h) != NNGP_IPC_HANDLE_BYTES) Rf_error("nngp: IPC handles must be raw(%d)", NNGP_IPC_HANDLE_BYTES);
    memcpy(buf + (size_t)g * NNGP_IPC_HANDLE_BYTES, RAW(h), NNGP_IPC_HANDLE_BYTES);
  }
  check(nngp_shard_ipc_open(c, buf, NNGP_IPC_HANDLE_BYTES), c);
  return R_NilValue;
}

/* ---------- batched per-chain forms (one host sync for all chains) ---------- */
SEXP C_nngp_factor_chains(SEXP p, SEXP which, SEXP mask, SEXP covfun, SEXP covparms) {
  nngp_ctx* c = get_ctx(p);
  nngp_info inf;
  check(nngp_ctx_info(c, &inf), c);
  /* covparms: n_chains x ncovparms matrix (row k = chain k), column-major in R */
  const int k = inf.n_chains, ncp = Rf_ncols(covparms);
  if (Rf_nrows(covparms) != k) Rf_error("nngp: covparms needs one row per chain");
  double rm[4 * 16];
  if (ncp > 16) Rf_error("nngp: at most 16 covariance parameters");
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < ncp; ++j) rm[i * ncp + j] = REAL(covparms)[i + (size_t)j * k];
  SEXP st = PROTECT(Rf_allocVector(INTSXP, k));
  for (int i = 0; i < k; ++i) INTEGER(st)[i] = 0;
  const int rc = nngp_factor_chains(c, as_int(which), as_int(mask), as_int(covfun), rm, ncp, INTEGER(st));
  UNPROTECT(1);
  check(rc, c);
  return st;
}

/* covparms: n_chains x ncovparms matrix (row k = chain k) -> row-major rm */
static int covparms_rows(nngp_ctx* c, SEXP covparms, double* rm) {
  nngp_info inf;
  check(nngp_ctx_info(c, &inf), c);
  const int k = inf.n_chains, ncp = Rf_ncols(covparms);
  if (Rf_nrows(covparms) != k) Rf_error("nngp: covparms needs one row per chain");
  if (ncp > 16) Rf_error("nngp: at most 16 covariance parameters");
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < ncp; ++j) rm[i * ncp + j] = REAL(covparms)[i + (size_t)j * k];
  return ncp;
}

static SEXP named_list(int n, SEXP* v, const char** names) {
  SEXP out = PROTECT(Rf_allocVector(VECSXP, n));
  SEXP nm = PROTECT(Rf_allocVector(STRSXP, n));
  for (int i = 0; i < n; ++i) {
    SET_VECTOR_ELT(out, i, v[i]);
    SET_STRING_ELT(nm, i, Rf_mkChar(names[i]));
  }
  Rf_setAttrib(out, R_NamesSymbol, nm);
  UNPROTECT(2);
  return out;
}

static SEXP chains_out(nngp_ctx* c) {
  nngp_info inf;
  check(nngp_ctx_info(c, &inf), c);
  return Rf_allocVector(REALSXP, inf.n_chains);
}

SEXP C_nngp_loglik_chains(SEXP p, SEXP which, SEXP mask, SEXP beta0, SEXP log_scale) {
  nngp_ctx* c = get_ctx(p);
  const int k = ctx_chains(c);
  const double *b0 = per_chain(beta0, k, "beta0"), *ls = per_chain(log_scale, k, "log_scale");
  SEXP out = PROTECT(chains_out(c));
  const int rc = nngp_loglik_chains(c, as_int(which), as_int(mask), b0, ls, REAL(out));
  UNPROTECT(1);
  check(rc, c);
  return out;
}

SEXP C_nngp_loglik_pair_chains(SEXP p, SEXP mask, SEXP beta0, SEXP ls_prop, SEXP ls_cur) {
  nngp_ctx* c = get_ctx(p);
  const int k = ctx_chains(c);
  const double *b0 = per_chain(beta0, k, "beta0"), *lp = per_chain(ls_prop, k, "log_scale_prop"),
               *lc = per_chain(ls_cur, k, "log_scale_cur");
  SEXP prop = PROTECT(chains_out(c));
  SEXP cur = PROTECT(chains_out(c));
  const int rc = nngp_loglik_pair_chains(c, as_int(mask), b0, lp, lc, REAL(prop), REAL(cur));
  if (rc) {
    UNPROTECT(2);
    check(rc, c);
  }
  SEXP out = PROTECT(Rf_allocVector(VECSXP, 2));
  SEXP nm = PROTECT(Rf_allocVector(STRSXP, 2));
  SET_VECTOR_ELT(out, 0, prop);
  SET_VECTOR_ELT(out, 1, cur);
  SET_STRING_ELT(nm, 0, Rf_mkChar("proposal"));
  SET_STRING_ELT(nm, 1, Rf_mkChar("current"));
  Rf_setAttrib(out, R_NamesSymbol, nm);
  UNPROTECT(4);
  return out;
}

SEXP C_nngp_field_response_ratio_chains(SEXP p, SEXP mask, SEXP beta0, SEXP lnv) {
  nngp_ctx* c = get_ctx(p);
  const int k = ctx_chains(c);
  const double *b0 = per_chain(beta0, k, "beta0"), *nv = per_chain(lnv, k, "log_noise_variance");
  SEXP out = PROTECT(chains_out(c));
  const int rc = nngp_field_response_ratio_chains(c, as_int(mask), b0, nv, REAL(out));
  UNPROTECT(1);
  check(rc, c);
  return out;
}

SEXP C_nngp_sum_squared_residuals_chains(SEXP p, SEXP mask, SEXP beta0) {
  nngp_ctx* c = get_ctx(p);
  const double* b0 = per_chain(beta0, ctx_chains(c), "beta0");
  SEXP out = PROTECT(chains_out(c));
  const int rc = nngp_sum_squared_residuals_chains(c, as_int(mask), b0, REAL(out));
  UNPROTECT(1);
  check(rc, c);
  return out;
}

/* ---------- registration ---------- */
#define E(name, n) {#name, (DL_FUNC)&name, n}
SEXP C_nngp_ancillary_step_chains(SEXP p, SEXP mask, SEXP covfun, SEXP covparms, SEXP beta0, SEXP dls, SEXP lnv) {
  nngp_ctx* c = get_ctx(p);
  const int k = ctx_chains(c);
  double rm[4 * 16];
  const int ncp = covparms_rows(c, covparms, rm);
  const double *b0 = per_chain(beta0, k, "beta0"), *dl = per_chain(dls, k, "dlog_scale"),
               *lv = per_chain(lnv, k, "log_noise_variance");
  SEXP st = PROTECT(Rf_allocVector(INTSXP, k));
  SEXP ratio = PROTECT(chains_out(c));
  for (int i = 0; i < k; ++i) INTEGER(st)[i] = 0;
  const int rc = nngp_ancillary_step_chains(c, as_int(mask), as_int(covfun), rm, ncp, b0, dl, lv, INTEGER(st),
                                            REAL(ratio));
  if (rc) {
    UNPROTECT(2);
    check(rc, c);
  }
  SEXP v[2] = {st, ratio};
  const char* nm[2] = {"status", "ratio"};
  SEXP out = named_list(2, v, nm);
  UNPROTECT(2);
  return out;
}

SEXP C_nngp_sufficient_step_chains(SEXP p, SEXP mask, SEXP covfun, SEXP covparms, SEXP beta0, SEXP ls_prop,
                                   SEXP ls_cur) {
  nngp_ctx* c = get_ctx(p);
  const int k = ctx_chains(c);
  double rm[4 * 16];
  const int ncp = covparms_rows(c, covparms, rm);
  const double *b0 = per_chain(beta0, k, "beta0"), *lp = per_chain(ls_prop, k, "log_scale_prop"),
               *lc = per_chain(ls_cur, k, "log_scale_cur");
  SEXP st = PROTECT(Rf_allocVector(INTSXP, k));
  SEXP prop = PROTECT(chains_out(c));
  SEXP cur = PROTECT(chains_out(c));
  for (int i = 0; i < k; ++i) INTEGER(st)[i] = 0;
  const int rc = nngp_sufficient_step_chains(c, as_int(mask), as_int(covfun), rm, ncp, b0, lp, lc, INTEGER(st),
                                             REAL(prop), REAL(cur));
  if (rc) {
    UNPROTECT(3);
    check(rc, c);
  }
  SEXP v[3] = {st, prop, cur};
  const char* nm[3] = {"status", "proposal", "current"};
  SEXP out = named_list(3, v, nm);
  UNPROTECT(3);
  return out;
}

static const R_CallMethodDef call_methods[] = {
    E(C_nngp_abi_version, 0),
    E(C_nngp_status_string, 1),
    E(C_nngp_order_maxmin, 1),
    E(C_nngp_find_ordered_nn, 2),
    E(C_nngp_greedy_coloring, 1),
    E(C_nngp_ctx_create, 7),
    E(C_nngp_ctx_create_shard, 9),
    E(C_nngp_ctx_destroy, 1),
    E(C_nngp_ctx_last_error, 1),
    E(C_nngp_set_chain, 2),
    E(C_nngp_ctx_info, 1),
    E(C_nngp_ctx_engine_note, 1),
    E(C_nngp_shard_sync, 1),
    E(C_nngp_factor, 4),
    E(C_nngp_get_linv, 2),
    E(C_nngp_set_linv, 3),
    E(C_nngp_accept_factor, 1),
    E(C_nngp_get_precision_diag, 1),
    E(C_nngp_set_field, 2),
    E(C_nngp_get_field, 1),
    E(C_nngp_set_mu, 3),
    E(C_nngp_records_reserve, 2),
    E(C_nngp_record_field, 2),
    E(C_nngp_get_records, 4),
    E(C_nngp_records_stream, 2),
    E(C_nngp_loglik, 4),
    E(C_nngp_sweep, 8),
    E(C_nngp_sweep_chains, 7),
    E(C_nngp_sweep_timed, 7),
    E(C_nngp_ancillary_propose, 3),
    E(C_nngp_ancillary_propose_chains, 4),
    E(C_nngp_field_response_ratio, 3),
    E(C_nngp_accept_field, 1),
    E(C_nngp_beta0_stats, 1),
    E(C_nngp_sum_squared_residuals, 2),
    E(C_nngp_spmv, 3),
    E(C_nngp_tri_solve, 3),
    E(C_nngp_tri_rescues, 1),
    E(C_nngp_device_normals, 4),
    E(C_nngp_get_sweep_r, 1),
    E(C_nngp_shard_unique_id, 0),
    E(C_nngp_shard_comm_init, 2),
    E(C_nngp_sweep_chains_group, 7),
    E(C_nngp_shard_ipc_handle, 1),
    E(C_nngp_shard_ipc_open, 2),
    E(C_nngp_factor_chains, 5),
    E(C_nngp_loglik_chains, 5),
    E(C_nngp_loglik_pair_chains, 5),
    E(C_nngp_ancillary_step_chains, 7),
    E(C_nngp_sufficient_step_chains, 7),
    E(C_nngp_field_response_ratio_chains, 4),
    E(C_nngp_sum_squared_residuals_chains, 3),
    {NULL, NULL, 0}};
#undef E

void R_init_nngpamd(DllInfo* dll) {
  R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}
