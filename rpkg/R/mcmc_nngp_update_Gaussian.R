# Drop-in for Scripts/mcmc_nngp_update_Gaussian.R:14-317 on the MI355X path.
#
# Same arguments and the same returned list (one list(state, records) per
# chain).  The scalar Metropolis-Hastings / Gibbs logic stays in R; every
# O(n) / O(nnz) step is a .Call into libnngp.so:
#   vecchia_Linv + sparseMatrix (:72-73,123-124,179-180)  -> nngp_factor
#   precision_diag (:74,142,197)                          -> nngp_factor / nngp_accept_factor
#   solve(new_B, B (field - beta_0)) (:127)                -> nngp_ancillary_propose
#   dnorm ratio (:129-131)                                 -> nngp_field_response_ratio
#   ll_compressed_sparse_chol (:8-12,184-186)              -> nngp_loglik
#   crossprod(B 1), (B field, B 1) (:221-222)              -> nngp_beta0_stats
#   chromatic sampling (:257-275)                          -> nngp_sweep (Philox normals on the device)
#   SSR (:281)                                             -> nngp_sum_squared_residuals
#   sparse_chol %*% X (:79,82,147,241)                     -> nngp_spmv
#   records$field (:305-311)                               -> nngp_record_field / nngp_get_records
# parallel::mclapply over chains (:25-26) is replaced by ONE device context
# holding the chains (HIP must not be initialised before a fork()); the
# chains are advanced one after another through nngp_set_chain.  The host
# draws keep R's RNG with set.seed(iter_start + i) as the reference does (:36);
# the sweep's normals come from the device Philox stream keyed by that seed.

.nngp_is_chol_error <- function(e) grepl("(status 3)", conditionMessage(e), fixed = TRUE)

.nngp_interweave <- function(ctx, X, vecchia_approx) {
  Xl <- X$X[vecchia_approx$hctam_scol_1, X$locs, drop = FALSE]
  SX <- nngp_spmv(ctx, 0L, cbind(1, Xl))
  cov_mat <- solve(crossprod(SX))
  list(Xl = Xl, SX = SX, covmat = cov_mat, covmat_chol = chol(cov_mat))
}

mcmc_nngp_update_Gaussian <- function(locs, X, observed_field, space_time_model, vecchia_approx, states,
                                      n_iterations_update = 400, n_cores = NULL, field_thinning = .1,
                                      ancillary = TRUE, n_chromatic = 5, iterations = NULL,
                                      contexts = NULL, device = -1L, on_chol_error = c("error", "reject")) {
  on_chol_error <- match.arg(on_chol_error)
  iter_start <- if (is.null(iterations)) 0 else iterations[nrow(iterations), 1]
  n_chains <- length(states)
  if (n_chains > 4) stop("nngp: at most 4 chains per device context")
  own_ctx <- is.null(contexts)
  ctx <- if (own_ctx) nngp_context(locs, vecchia_approx$NNarray, vecchia_approx$coloring,
                                   vecchia_approx$locs_match, observed_field, n_chains, device) else contexts
  if (own_ctx) on.exit(nngp_destroy(ctx), add = TRUE)
  covfun <- space_time_model$covfun$stationary_covfun
  sp <- space_time_model$covfun$shape_params
  n_shape <- length(sp)
  n_obs <- vecchia_approx$n_obs
  var_y <- var(observed_field)
  has_X <- !is.null(X$X)
  has_locs <- has_X && length(X$locs) > 0
  n_saved <- round(n_iterations_update * field_thinning)

  run_one <- function(i) {
    nngp_set_chain(ctx, i - 1L)
    set.seed(iter_start + i)
    key <- iter_start + i
    params <- states[[i]]$params
    tk <- states[[i]]$transition_kernels
    rec <- list(beta_0 = matrix(0, n_iterations_update, 1), log_scale = matrix(0, n_iterations_update, 1),
                log_noise_variance = matrix(0, n_iterations_update, 1),
                shape = matrix(0, n_iterations_update, n_shape))
    if (has_X) rec$beta <- matrix(0, n_iterations_update, ncol(X$X))
    acc_anc <- acc_suf <- rep(0, n_iterations_update)
    if (n_saved > 0) nngp_records_reserve(ctx, n_saved)
    nngp_factor(ctx, 0L, covfun, nngp_covparms(sp, params$shape))
    nngp_set_field(ctx, params$field)
    iw <- if (has_locs) .nngp_interweave(ctx, X, vecchia_approx) else NULL
    mu_of <- function() if (has_X) params$beta_0 + X$X %*% params$beta else NULL
    nngp_set_mu(ctx, mu_of(), params$beta_0)
    adapt <- iter_start >= 0 && iter_start <= 2000
    try_factor <- function(new_shape) {
      tryCatch({
        nngp_factor(ctx, 1L, covfun, nngp_covparms(sp, new_shape))
        TRUE
      }, error = function(e) {
        if (on_chol_error == "reject" && .nngp_is_chol_error(e)) return(FALSE)
        stop(e)
      })
    }
    for (it in seq(n_iterations_update)) {
      if (ancillary) {  # :113-157
        innov <- rnorm(n_shape + 1, 0, exp(.5 * tk$covariance_params_ancillary$logvar))
        new_ls <- params$log_scale + innov[1]
        new_shape <- params$shape + innov[-1]
        if (try_factor(new_shape)) {
          nngp_ancillary_propose(ctx, params$beta_0, new_ls - params$log_scale)
          ratio <- nngp_field_response_ratio(ctx, params$beta_0, params$log_noise_variance)
          if (ratio > log(runif(1))) {
            params$shape <- new_shape
            params$log_scale <- new_ls
            nngp_accept_field(ctx)
            nngp_accept_factor(ctx)
            acc_anc[it] <- 1
            if (has_locs) iw <- .nngp_interweave(ctx, X, vecchia_approx)
          }
        }
        if (adapt && it %% 25 == 0) {
          a <- mean(acc_anc[(it - 24):it])
          if (a < .05) tk$covariance_params_ancillary$logvar <- tk$covariance_params_ancillary$logvar - rnorm(1, .4, .05)
          if (a > .15) tk$covariance_params_ancillary$logvar <- tk$covariance_params_ancillary$logvar + rnorm(1, .4, .05)
        }
      }
      innov <- rnorm(n_shape + 1, 0, exp(.5 * tk$covariance_params_sufficient$logvar))  # :165-213
      new_ls <- params$log_scale + innov[1]
      if (exp(new_ls) < var_y) {
        new_shape <- params$shape + innov[-1]
        if (try_factor(new_shape)) {
          gp_ratio <- nngp_loglik(ctx, 1L, params$beta_0, new_ls) -
            nngp_loglik(ctx, 0L, params$beta_0, params$log_scale)
          if (gp_ratio > log(runif(1))) {
            params$shape <- new_shape
            params$log_scale <- new_ls
            nngp_accept_factor(ctx)
            acc_suf[it] <- 1
            if (has_locs) iw <- .nngp_interweave(ctx, X, vecchia_approx)
          }
        }
      }
      if (adapt && it %% 25 == 0) {
        a <- mean(acc_suf[(it - 24):it])
        if (a < .05) tk$covariance_params_sufficient$logvar <- tk$covariance_params_sufficient$logvar - rnorm(1, .2, .05)
        if (a > .15) tk$covariance_params_sufficient$logvar <- tk$covariance_params_sufficient$logvar + rnorm(1, .2, .05)
      }
      if (!has_locs || !has_X) {  # :219-224
        st <- nngp_beta0_stats(ctx)
        beta_cov <- exp(params$log_scale) / st[1]
        beta_mean <- exp(-params$log_scale) * st[2] * beta_cov
        params$beta_0 <- beta_mean + sqrt(beta_cov) * rnorm(1)
      }
      if (has_X) {  # :226-247
        field <- nngp_get_field(ctx)
        X1 <- cbind(1, X$X)
        resid <- observed_field - field[vecchia_approx$locs_match] + params$beta_0
        innov <- as.vector(crossprod(X1, resid)) %*% X$solve_1XT1X +
          exp(.5 * params$log_noise_variance) * t(X$chol_solve_1XT1X) %*% rnorm(ncol(X1))
        innov <- as.vector(innov)
        field <- field - params$beta_0 + innov[1]
        params$beta_0 <- innov[1]
        params$beta <- innov[-1]
        if (has_locs) {
          other <- field + as.vector(iw$Xl %*% params$beta[X$locs])
          Bo <- nngp_spmv(ctx, 0L, other)
          bm <- iw$covmat %*% crossprod(iw$SX, Bo)
          innov <- as.vector(bm + exp(.5 * params$log_scale) * t(iw$covmat_chol) %*% rnorm(length(X$locs) + 1))
          params$beta_0 <- innov[1]
          params$beta[X$locs] <- innov[-1]
          field <- other - as.vector(iw$Xl %*% params$beta[X$locs])
        }
        nngp_set_field(ctx, field)
      }
      nngp_set_mu(ctx, mu_of(), params$beta_0)
      nngp_sweep(ctx, n_chromatic, params$beta_0, params$log_scale, params$log_noise_variance,
                 key, (iter_start + it - 1) * n_chromatic)  # :257-275
      ssr <- nngp_sum_squared_residuals(ctx, params$beta_0)  # :281-293
      for (k in 1:10) {
        innov <- rnorm(1, 0, .01)
        if (exp(params$log_noise_variance + innov) < var_y) {
          lnv <- params$log_noise_variance
          if (-.5 * n_obs * innov - .5 * ssr * (exp(-lnv - innov) - exp(-lnv)) > log(runif(1)))
            params$log_noise_variance <- lnv + innov
        }
      }
      if (has_X) rec$beta[it, ] <- params$beta  # :305-311
      rec$beta_0[it, ] <- params$beta_0
      rec$log_noise_variance[it, ] <- params$log_noise_variance
      rec$log_scale[it, ] <- params$log_scale
      rec$shape[it, ] <- params$shape
      if (round(it * field_thinning) == it * field_thinning) nngp_record_field(ctx, it * field_thinning - 1)
    }
    rec$field <- if (n_saved > 0) nngp_get_records(ctx, 0L, n_saved) else matrix(0, 0, length(params$field))
    if (n_saved > 0) nngp_records_reserve(ctx, 0L)
    params$field <- nngp_get_field(ctx)
    list(state = list(params = params, transition_kernels = tk), records = rec)
  }
  lapply(seq(n_chains), run_one)
}
