# Drop-in for mcmc_nngp_predict_field (Scripts/mcmc_nngp_predict.R:1-60) on
# the MI355X path.  Same arguments and returned list.  The array work moves to
# libnngp.so:
#   GpGp::find_ordered_nn(rbind(locs, predicted_locs), m) (:5)  -> nngp_find_ordered_nn (bit-exact)
#   GpGp::vecchia_Linv + sparseMatrix (:39-40)                  -> nngp_factor (device factor of the stacked locations)
#   sparse_chol[1:n, 1:n] %*% (field - beta_0) (:48)            -> nngp_spmv (B is lower triangular: the first
#                                                                  n rows of B c(w, 0))
#   Matrix::solve(sparse_chol, .) (:46-52)                      -> nngp_tri_solve (level-scheduled on the device)
# parallel::mclapply over chains (:16) becomes a loop over the chains on one
# device context (HIP is not fork-safe).  Kept from the reference: the factor
# is rebuilt only where !duplicated(shape) marks a sample (:21) -- so a shape
# that comes back after another one reuses the LAST factor built, as there --
# and the 1.5 * plogis smoothness transform of predict (:37).
# mcmc_nngp_predict_fixed_effects (:67-104) has no array work on the path and
# stays the reference's.

mcmc_nngp_predict_field <- function(mcmc_nngp_list, predicted_locs, burn_in = .5, n_cores = 1, m = 10,
                                    device = -1L) {
  locs <- rbind(mcmc_nngp_list$locs, predicted_locs)
  n <- mcmc_nngp_list$vecchia_approx$n_locs
  N <- nrow(locs)
  n_new <- N - n
  NNarray <- nngp_find_ordered_nn(locs, m)
  ctx <- nngp_context(locs, NNarray, nngp_greedy_coloring(NNarray), seq_len(N), numeric(N), 1L, device)
  on.exit(nngp_destroy(ctx), add = TRUE)
  covfun <- mcmc_nngp_list$space_time_model$covfun$stationary_covfun
  shape_params <- mcmc_nngp_list$space_time_model$covfun$shape_params
  stored_idx <- mcmc_nngp_list$records$chain_1$saved_field
  stored_idx <- stored_idx[stored_idx > burn_in * max(stored_idx)]
  n_samples <- length(stored_idx)
  own <- seq_len(n)
  samples <- lapply(mcmc_nngp_list$records, function(chain) {
    out <- matrix(0, n_samples, n_new)
    refactor <- !duplicated(chain$params$shape[stored_idx, , drop = FALSE])
    for (k in seq_len(n_samples)) {
      i_chain <- stored_idx[k]
      i_field <- match(i_chain, chain$saved_field)
      if (refactor[k])
        nngp_factor(ctx, 0L, covfun, nngp_covparms(shape_params, chain$params$shape[i_chain, ], lo = 0, span = 1.5))
      sd <- exp(.5 * chain$params$log_scale[i_chain])
      w <- chain$params$field[i_field, ] - chain$params$beta_0[i_chain]
      u <- as.vector(nngp_spmv(ctx, 0L, matrix(c(w, numeric(n_new)), ncol = 1)))[own]
      x <- nngp_tri_solve(ctx, 0L, c(u / sd, rnorm(n_new)))
      out[k, ] <- sd * x[-own]
    }
    out
  })
  list(predicted_locs = predicted_locs, predicted_field_samples = samples,
       predicted_field_summary = get_summary(do.call(rbind, samples)))
}
