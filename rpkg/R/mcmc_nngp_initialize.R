# Drop-in for mcmc_nngp_initialize (Scripts/mcmc_nngp_initialize.R:1-240) on
# the MI355X path.  Same arguments and the same returned list.  The steps on
# the hot path's inputs move to libnngp.so:
#   GpGp::find_ordered_nn(locs, m) (:93)                       -> nngp_find_ordered_nn (bit-exact, ties by the
#                                                                  smaller index; raw coordinates as GpGp here)
#   crossprod(sparseMatrix(row, col)) + naive_greedy_coloring  -> nngp_greedy_coloring (the moral graph's greedy
#     (:103-110, Scripts/Coloring.R:2-20)                          first-fit colouring, bit-exact, without the
#                                                                  (n+1) x max_degree dense matrix of Coloring.R)
#   GpGp::vecchia_Linv + Matrix::solve(Linv, rnorm(n)) (:201-208) -> nngp_factor + nngp_tri_solve (device)
# The ordering (:29-33) stays GpGp's -- it is an input of the hot path
# (RNG-jittered, SURVEY §0.1-4) -- when GpGp is installed; without it the
# "maxmin" ordering is nngp_order_maxmin (exact max-min).  The moral graph
# itself is not kept (vecchia_approx$MRF_adjacency_mat: nothing downstream
# reads it).  The regressors, the OLS starting points and the records
# skeleton are host R as in the reference.

mcmc_nngp_initialize <- function(observed_locs, observed_field, X_obs = NULL, X_locs = NULL, m = 10,
                                 reordering = "maxmin", stationary_covfun = "exponential_isotropic",
                                 response_model = "Gaussian", n_chains = 3, seed = 1, device = -1L) {
  t_begin <- Sys.time()
  set.seed(seed)
  sphere <- grepl("sphere", stationary_covfun)
  have_gpgp <- requireNamespace("GpGp", quietly = TRUE)

  # ---- unique locations in the chosen order (:26-36)
  locs <- observed_locs[!duplicated(observed_locs), , drop = FALSE]
  ord <- switch(reordering[1],
    maxmin = if (have_gpgp) GpGp::order_maxmin(locs, lonlat = sphere) else nngp_order_maxmin(locs),
    random = sample(seq(nrow(locs))),
    coord = GpGp::order_coordinate(locs = locs, coordinate = as.numeric(reordering[2])),
    dist_to_point = GpGp::order_dist_to_point(locs, loc0 = as.numeric(reordering[2]), lonlat = sphere),
    middleout = GpGp::order_middleout(locs, lonlat = sphere),
    stop("unknown reordering ", reordering[1]))
  locs <- locs[ord, , drop = FALSE]
  n <- nrow(locs)

  # ---- space-time model (:43-79)
  d <- ncol(locs)
  shape_params <- switch(stationary_covfun,
    exponential_isotropic = "log_range",
    exponential_sphere = "log_range",
    exponential_scaledim = paste("log_range", seq(d), sep = "_"),
    exponential_spacetime = c("log_range_1", "log_range_2"),
    matern_isotropic = c("log_range", "qlogis_smoothness"),
    matern_sphere = c("log_range", "qlogis_smoothness"),
    matern_scaledim = c(paste("log_range", seq(d), sep = "_"), "qlogis_smoothness"),
    matern_spacetime = c("log_range_1", "log_range_2", "qlogis_smoothness"),
    matern15_isotropic = "log_range",
    stop("unknown covariance function ", stationary_covfun))
  space_time_model <- list(response_model = response_model,
                           covfun = list(stationary_covfun = stationary_covfun, shape_params = shape_params))

  # ---- Vecchia approximation (:81-110)
  va <- list(n_locs = n, n_obs = length(observed_field))
  va$locs_match <- match(split(observed_locs, row(observed_locs)), split(locs, row(locs)))  # exact rows
  va$hctam_scol <- split(seq(va$n_obs), va$locs_match)
  va$hctam_scol_1 <- vapply(va$hctam_scol, function(x) x[1], 0L)
  va$obs_per_loc <- lengths(va$hctam_scol)
  va$NNarray <- nngp_find_ordered_nn(locs, m)
  va$NNarray_non_NA <- !is.na(va$NNarray)
  va$sparse_chol_column_idx <- va$NNarray[va$NNarray_non_NA]
  va$sparse_chol_row_idx <- row(va$NNarray)[va$NNarray_non_NA]
  va$coloring <- nngp_greedy_coloring(va$NNarray)

  # ---- regressors (:116-137): model matrix without intercept, centred
  X <- list(arg = list(X_locs = X_locs, X_obs = X_obs))
  parts <- Filter(Negate(is.null), list(X_locs, X_obs))
  X$X <- if (length(parts)) do.call(cbind, parts) else NULL
  if (!is.null(X$X)) {
    mm <- model.matrix(~., X$X)
    cn <- colnames(mm)[-1]
    X$X <- matrix(mm[, -1], nrow = nrow(mm))
    colnames(X$X) <- cn
    X$locs <- seq(ncol(X_locs))
    X$X_mean <- colMeans(X$X)
    X$X <- sweep(X$X, 2, X$X_mean)
    X$solve_XTX <- solve(crossprod(X$X))
    X$chol_solve_XTX <- chol(X$solve_XTX)
    X$solve_1XT1X <- solve(crossprod(cbind(1, X$X)))
    X$chol_solve_1XT1X <- chol(X$solve_1XT1X)
  }

  # ---- chain states (:143-209)
  span <- function(cols) log(max(dist(locs[1:100, cols, drop = FALSE]))) - log(seq(20, 200, 1))
  start_shape <- function() {
    r1 <- function(cols) sample(span(cols), 1)
    switch(stationary_covfun,
      exponential_scaledim = vapply(seq(d), function(j) r1(j), 0),
      exponential_spacetime = c(r1(-d), r1(d)),
      matern_isotropic = , matern_sphere = c(r1(seq(d)), rnorm(1)),
      matern_scaledim = c(vapply(seq(d), function(j) r1(j), 0), rnorm(1)),
      matern_spacetime = c(r1(-d), r1(d), rnorm(1)),
      r1(seq(d)))
  }
  states <- setNames(lapply(seq(n_chains), function(i) list(params = list(shape = start_shape()))),
                     paste("chain", seq(n_chains), sep = "_"))
  if (response_model == "Gaussian") {
    ols <- if (!is.null(X$X)) lm(observed_field ~ X$X) else lm(observed_field ~ NULL)
    ctx <- nngp_context(locs, va$NNarray, va$coloring, va$locs_match, observed_field, 1L, device)
    on.exit(nngp_destroy(ctx), add = TRUE)
    for (i in seq(n_chains)) {
      states[[i]]$transition_kernels <- list(covariance_params_sufficient = list(logvar = -2),
                                             covariance_params_ancillary = list(logvar = -2),
                                             log_noise_variance = list(logvar = -1))
      perturb <- t(chol(vcov(ols))) %*% rnorm(length(ols$coefficients))
      states[[i]]$params$beta_0 <- ols$coefficients[1] + perturb[1]
      if (!is.null(X$X)) states[[i]]$params$beta <- ols$coefficients[-1] + perturb[-1]
      states[[i]]$params$log_scale <- log(rbeta(1, 10, 10) * var(ols$residuals))
      states[[i]]$params$log_noise_variance <- log(rbeta(1, 10, 10) * var(ols$residuals))
      # initial field: beta_0 + sigma B^{-1} z with the .4 + .7 plogis smoothness of :199
      nngp_factor(ctx, 0L, stationary_covfun, nngp_covparms(shape_params, states[[i]]$params$shape, lo = .4, span = .7))
      states[[i]]$params$field <- states[[i]]$params$beta_0 +
        sqrt(exp(states[[i]]$params$log_scale)) * nngp_tri_solve(ctx, 0L, rnorm(n))
    }
  }

  # ---- records skeleton (:215-229)
  records <- setNames(lapply(seq(n_chains), function(i) {
    it <- matrix(c(0, Sys.time() - t_begin), ncol = 2)
    colnames(it) <- c("iteration", "time")
    list(iterations = it, params = list())
  }), paste("chain", seq(n_chains), sep = "_"))
  print(paste("Setup done,", as.numeric(Sys.time() - t_begin, units = "secs"), "s elapsed"))
  list(locs = locs, X = X, observed_field = observed_field, observed_locs = observed_locs,
       space_time_model = space_time_model, vecchia_approx = va, states = states, records = records,
       diagnostics = list(Gelman_Rubin_Brooks = list()), t_begin = t_begin, seed = seed)
}
