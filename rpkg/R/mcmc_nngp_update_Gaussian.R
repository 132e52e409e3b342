# Drop-in for Scripts/mcmc_nngp_update_Gaussian.R:14-317 on the MI355X path.
#
# Same arguments and the same returned list (one list(state, records) per
# chain).  The scalar Metropolis-Hastings / Gibbs logic stays in R; every
# O(n) / O(nnz) step is a .Call into libnngp.so:
#   vecchia_Linv + sparseMatrix (:72-73)                   -> nngp_factor
#   precision_diag (:74,142,197)                          -> inside nngp_factor / nngp_accept_factor
#   ancillary step: vecchia_Linv (:123-124), solve(new_B, B (field - beta_0)) (:127),
#     dnorm ratio (:129-131)                               -> nngp_ancillary_step_chains (one host sync)
#   sufficient step: vecchia_Linv (:179-180), ll_compressed_sparse_chol of both
#     factors (:8-12,184-186)                              -> nngp_sufficient_step_chains (one host sync)
#   crossprod(B 1), (B field, B 1) (:221-222)              -> nngp_beta0_stats
#   chromatic sampling (:257-275)                          -> nngp_sweep_chains (Philox normals on the device)
#   SSR (:281)                                             -> nngp_sum_squared_residuals_chains
#   sparse_chol %*% X (:79,82,147,241)                     -> nngp_spmv
#   records$field (:305-311)                               -> nngp_record_field / nngp_get_records
# parallel::mclapply over chains (:25-26) is replaced by ONE device context
# holding the chains (HIP must not be initialised before a fork()), advanced in
# lockstep: every step of an iteration is one batched call for all chains of
# the context (one kernel pass, one host synchronisation), in the order of the
# Python host mirror (update_gaussian.py): per iteration ancillary_step_chains,
# chain by chain the acceptances, sufficient_step_chains, chain by chain
# the acceptances, beta_0 and mu, sweep_chains, sum_squared_residuals_chains,
# chain by chain the field records -- the sequence the C client
# tests/cpp/capi_sequence.c replays against the Python binding.  Each chain
# keeps its own R RNG stream, set.seed(iter_start + i) as the reference does
# (:36), swapped in around that chain's draws, so the lockstep order draws
# exactly what running the chains one after another would; the sweep's
# normals come from the device Philox stream keyed by iter_start + i.

.nngp_is_chol_error <- function(e) grepl("(status 3)", conditionMessage(e), fixed = TRUE)

.nngp_interweave <- function(ctx, X, vecchia_approx) {  # :77-83,145-151
  Xl <- X$X[vecchia_approx$hctam_scol_1, X$locs, drop = FALSE]
  SX <- nngp_spmv(ctx, 0L, cbind(1, Xl))
  prec <- crossprod(SX)
  cov_mat <- solve(prec, tol = min(rcond(prec), .Machine$double.eps))
  list(Xl = Xl, SX = SX, covmat = cov_mat, covmat_chol = chol(cov_mat))
}

# bit mask of the chains (1-based indices) for the *_chains entry points
.nngp_mask <- function(idx) as.integer(sum(2^(idx - 1)))

mcmc_nngp_update_Gaussian <- function(locs, X, observed_field, space_time_model, vecchia_approx, states,
                                      n_iterations_update, n_cores = NULL, field_thinning = 1,
                                      ancillary = TRUE, n_chromatic = 10, iterations = NULL,
                                      contexts = NULL, device = -1L, on_chol_error = c("error", "reject")) {
  on_chol_error <- match.arg(on_chol_error)
  iter_start <- if (is.null(iterations)) 0 else iterations[nrow(iterations), 1]
  C <- length(states)
  if (C > 4) stop("nngp: at most 4 chains per device context")
  own_ctx <- is.null(contexts)
  ctx <- if (own_ctx) nngp_context(locs, vecchia_approx$NNarray, vecchia_approx$coloring,
                                   vecchia_approx$locs_match, observed_field, C, device) else contexts
  if (own_ctx) on.exit(nngp_destroy(ctx), add = TRUE)
  covfun <- space_time_model$covfun$stationary_covfun
  sp <- space_time_model$covfun$shape_params
  n_shape <- length(sp)
  n_obs <- vecchia_approx$n_obs
  var_y <- var(observed_field)
  has_X <- !is.null(X$X)
  has_locs <- has_X && length(X$locs) > 0
  n_saved <- round(n_iterations_update * field_thinning)
  all_chains <- .nngp_mask(seq_len(C))
  adapt <- iter_start >= 0 && iter_start <= 2000

  # one R RNG stream per chain, swapped in around that chain's draws; the
  # caller's stream is restored on exit
  had_seed <- exists(".Random.seed", envir = .GlobalEnv, inherits = FALSE)
  if (had_seed) caller_seed <- get(".Random.seed", envir = .GlobalEnv)
  on.exit(if (had_seed) assign(".Random.seed", caller_seed, envir = .GlobalEnv)
          else if (exists(".Random.seed", envir = .GlobalEnv, inherits = FALSE))
            rm(".Random.seed", envir = .GlobalEnv), add = TRUE)
  rng <- vector("list", C)
  for (i in seq_len(C)) {
    set.seed(iter_start + i)
    rng[[i]] <- get(".Random.seed", envir = .GlobalEnv)
  }
  draw <- function(i, f) {
    assign(".Random.seed", rng[[i]], envir = .GlobalEnv)
    v <- f()
    rng[[i]] <<- get(".Random.seed", envir = .GlobalEnv)
    v
  }
  # a proposal's factor statuses (:123,179): GpGp raises on a non positive
  # definite local covariance, which ends the call (on_chol_error = "error");
  # "reject" treats the proposal as rejected
  proposal_ok <- function(st, idx) {
    ok <- rep(FALSE, C)
    ok[idx] <- st[idx] == 0L
    if (on_chol_error == "error" && any(st[idx] == 3L))
      stop("nngp: vecchia factor: a local covariance of the proposal is not positive definite (status 3)")
    ok
  }
  set_mu <- function(i) {
    nngp_set_chain(ctx, i - 1L)
    mu <- if (has_X) P[[i]]$beta_0 + X$X %*% P[[i]]$beta else NULL
    nngp_set_mu(ctx, mu, P[[i]]$beta_0)
  }

  P <- lapply(states, function(s) s$params)
  TK <- lapply(states, function(s) s$transition_kernels)
  REC <- lapply(seq_len(C), function(i) {
    r <- list(beta_0 = matrix(0, n_iterations_update, 1), log_scale = matrix(0, n_iterations_update, 1),
              log_noise_variance = matrix(0, n_iterations_update, 1),
              shape = matrix(0, n_iterations_update, n_shape))
    if (has_X) r$beta <- matrix(0, n_iterations_update, ncol(X$X))
    r
  })
  acc_anc <- acc_suf <- matrix(0, n_iterations_update, C)
  IW <- vector("list", C)
  RB <- vector("list", C)  # host vectors the field records stream into while the chains run
  # a binding ends before its vector can go: on any exit (an error, an
  # interrupt) the chains of a caller's context are unbound (the shim also
  # keeps each bound vector alive; an own context ends them by nngp_destroy)
  if (!own_ctx) on.exit(for (i in seq_len(C)) if (!is.null(RB[[i]])) try({
    nngp_set_chain(ctx, i - 1L)
    nngp_records_stream(ctx, NULL)
  }, silent = TRUE), add = TRUE)
  for (i in seq_len(C)) {  # :67-90
    nngp_set_chain(ctx, i - 1L)
    if (n_saved > 0) {
      nngp_records_reserve(ctx, n_saved)
      RB[[i]] <- numeric(n_saved * length(P[[i]]$field))
      nngp_records_stream(ctx, RB[[i]])
    }
    nngp_factor(ctx, 0L, covfun, nngp_covparms(sp, P[[i]]$shape))
    nngp_set_field(ctx, P[[i]]$field)
    if (has_locs) IW[[i]] <- .nngp_interweave(ctx, X, vecchia_approx)
    set_mu(i)
  }
  cp_rows <- function(shapes, idx) {
    cp <- matrix(0, C, n_shape + 2)
    for (i in idx) cp[i, ] <- nngp_covparms(sp, shapes[[i]])
    cp
  }
  vec <- function(name) vapply(P, function(p) p[[name]], 0)

  for (it in seq_len(n_iterations_update)) {
    # ---- ancillary covariance update (:113-157)
    if (ancillary) {
      new_ls <- numeric(C)
      new_shape <- vector("list", C)
      for (i in seq_len(C)) {
        innov <- draw(i, function() rnorm(n_shape + 1, 0, exp(.5 * TK[[i]]$covariance_params_ancillary$logvar)))
        new_ls[i] <- P[[i]]$log_scale + innov[1]
        new_shape[[i]] <- P[[i]]$shape + innov[-1]
      }
      # the proposals' factors, fields and dnorm ratios behind one host sync
      stp <- nngp_ancillary_step_chains(ctx, all_chains, covfun, cp_rows(new_shape, seq_len(C)), vec("beta_0"),
                                        new_ls - vec("log_scale"), vec("log_noise_variance"))
      ok <- proposal_ok(stp$status, seq_len(C))
      ratio <- stp$ratio
      for (i in seq_len(C)) {
        if (ok[i] && ratio[i] > log(draw(i, function() runif(1)))) {
          P[[i]]$shape <- new_shape[[i]]
          P[[i]]$log_scale <- new_ls[i]
          nngp_set_chain(ctx, i - 1L)
          nngp_accept_field(ctx)
          nngp_accept_factor(ctx)
          acc_anc[it, i] <- 1
          if (has_locs) IW[[i]] <- .nngp_interweave(ctx, X, vecchia_approx)
        }
        if (adapt && it %% 25 == 0) {
          a <- mean(acc_anc[(it - 24):it, i])
          lv <- TK[[i]]$covariance_params_ancillary$logvar
          if (a < .05) lv <- lv - draw(i, function() rnorm(1, .4, .05))
          if (a > .15) lv <- lv + draw(i, function() rnorm(1, .4, .05))
          TK[[i]]$covariance_params_ancillary$logvar <- lv
        }
      }
    }
    # ---- sufficient covariance update (:165-213)
    new_ls <- numeric(C)
    new_shape <- vector("list", C)
    for (i in seq_len(C)) {
      innov <- draw(i, function() rnorm(n_shape + 1, 0, exp(.5 * TK[[i]]$covariance_params_sufficient$logvar)))
      new_ls[i] <- P[[i]]$log_scale + innov[1]
      new_shape[[i]] <- P[[i]]$shape + innov[-1]
    }
    prop <- which(exp(new_ls) < var_y)
    ok <- rep(FALSE, C)
    if (length(prop)) {
      # the proposals' factors and both log-likelihoods behind one host sync
      stp <- nngp_sufficient_step_chains(ctx, .nngp_mask(prop), covfun, cp_rows(new_shape, prop), vec("beta_0"),
                                         new_ls, vec("log_scale"))
      ok <- proposal_ok(stp$status, prop)
      l1 <- stp$proposal
      l0 <- stp$current
    }
    for (i in seq_len(C)) {
      if (ok[i] && l1[i] - l0[i] > log(draw(i, function() runif(1)))) {
        P[[i]]$shape <- new_shape[[i]]
        P[[i]]$log_scale <- new_ls[i]
        nngp_set_chain(ctx, i - 1L)
        nngp_accept_factor(ctx)
        acc_suf[it, i] <- 1
        if (has_locs) IW[[i]] <- .nngp_interweave(ctx, X, vecchia_approx)
      }
      if (adapt && it %% 25 == 0) {
        a <- mean(acc_suf[(it - 24):it, i])
        lv <- TK[[i]]$covariance_params_sufficient$logvar
        if (a < .05) lv <- lv - draw(i, function() rnorm(1, .2, .05))
        if (a > .15) lv <- lv + draw(i, function() rnorm(1, .2, .05))
        TK[[i]]$covariance_params_sufficient$logvar <- lv
      }
      # ---- field mean (:219-247)
      nngp_set_chain(ctx, i - 1L)
      if (!has_locs || !has_X) {  # :219-224
        st0 <- nngp_beta0_stats(ctx)
        beta_cov <- exp(P[[i]]$log_scale) / st0[1]
        beta_mean <- exp(-P[[i]]$log_scale) * st0[2] * beta_cov
        P[[i]]$beta_0 <- beta_mean + sqrt(beta_cov) * draw(i, function() rnorm(1))
      }
      if (has_X) {  # :226-247
        field <- nngp_get_field(ctx)
        X1 <- cbind(1, X$X)
        resid <- observed_field - field[vecchia_approx$locs_match] + P[[i]]$beta_0
        z <- draw(i, function() rnorm(ncol(X1)))
        innov <- as.vector(as.vector(crossprod(X1, resid)) %*% X$solve_1XT1X +
                             exp(.5 * P[[i]]$log_noise_variance) * t(X$chol_solve_1XT1X) %*% z)
        field <- field - P[[i]]$beta_0 + innov[1]
        P[[i]]$beta_0 <- innov[1]
        P[[i]]$beta <- innov[-1]
        if (has_locs) {
          iw <- IW[[i]]
          other <- field + as.vector(iw$Xl %*% P[[i]]$beta[X$locs])
          Bo <- nngp_spmv(ctx, 0L, other)
          bm <- iw$covmat %*% crossprod(iw$SX, Bo)
          z <- draw(i, function() rnorm(length(X$locs) + 1))
          innov <- as.vector(bm + exp(.5 * P[[i]]$log_scale) * t(iw$covmat_chol) %*% z)
          P[[i]]$beta_0 <- innov[1]
          P[[i]]$beta[X$locs] <- innov[-1]
          field <- other - as.vector(iw$Xl %*% P[[i]]$beta[X$locs])
        }
        nngp_set_field(ctx, field)
      }
      set_mu(i)
    }
    # ---- chromatic sampling of every chain's field, one call (:257-275)
    nngp_sweep_chains(ctx, n_chromatic, vec("beta_0"), vec("log_scale"), vec("log_noise_variance"),
                      iter_start + seq_len(C), rep((iter_start + it - 1) * n_chromatic, C))
    # a tile-shard context without a communicator (the same script run on
    # every rank, one GPU each) has only its halo exchanged after the sweep:
    # the full exchange of the field replicas is this explicit collective,
    # at the same point on every rank, before anything below reads the field
    # (a no-op on every other context)
    nngp_shard_sync(ctx)
    # ---- noise variance (:281-293)
    ssr <- nngp_sum_squared_residuals_chains(ctx, all_chains, vec("beta_0"))
    for (i in seq_len(C)) {
      for (k in 1:10) {
        innov <- draw(i, function() rnorm(1, 0, .01))
        if (exp(P[[i]]$log_noise_variance + innov) < var_y) {
          lnv <- P[[i]]$log_noise_variance
          if (-.5 * n_obs * innov - .5 * ssr[i] * (exp(-lnv - innov) - exp(-lnv)) > log(draw(i, function() runif(1))))
            P[[i]]$log_noise_variance <- lnv + innov
        }
      }
    }
    # ---- records (:305-311); records$field[0, ] is a no-op in R
    for (i in seq_len(C)) {
      if (has_X) REC[[i]]$beta[it, ] <- P[[i]]$beta
      REC[[i]]$beta_0[it, ] <- P[[i]]$beta_0
      REC[[i]]$log_noise_variance[it, ] <- P[[i]]$log_noise_variance
      REC[[i]]$log_scale[it, ] <- P[[i]]$log_scale
      REC[[i]]$shape[it, ] <- P[[i]]$shape
      if (round(it * field_thinning) == it * field_thinning && it * field_thinning >= 1) {
        nngp_set_chain(ctx, i - 1L)
        nngp_record_field(ctx, it * field_thinning - 1)
      }
    }
  }
  lapply(seq_len(C), function(i) {
    nngp_set_chain(ctx, i - 1L)
    rec <- REC[[i]]
    rec$field <- if (n_saved > 0) nngp_get_records(ctx, 0L, n_saved, RB[[i]]) else matrix(0, 0, length(P[[i]]$field))
    if (n_saved > 0) nngp_records_reserve(ctx, 0L)
    params <- P[[i]]
    params$field <- nngp_get_field(ctx)
    list(state = list(params = params, transition_kernels = TK[[i]]), records = rec)
  })
}
