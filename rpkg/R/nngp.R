# Thin R wrappers of the .Call entry points of src/nngp_shim.c (one per
# function of include/nngp.h).  Arrays follow R's own conventions
# (column-major, 1-based, NA_integer_), so GpGp / Matrix outputs of the
# reference pass through unchanged.

.covfun_ids <- c(exponential_isotropic = 0L, exponential_sphere = 1L, exponential_scaledim = 2L,
                 exponential_spacetime = 3L, matern_isotropic = 4L, matern_sphere = 5L,
                 matern_scaledim = 6L, matern_spacetime = 7L, matern15_isotropic = 8L)

nngp_covfun_id <- function(covfun_name) {
  id <- .covfun_ids[covfun_name]
  if (is.na(id)) stop("nngp: unknown covariance function ", covfun_name)
  unname(id)
}

# c(1, shape, 0) with the MCMC's transforms (update_Gaussian.R:67-72):
# exp() for log_* parameters, lo + span * plogis() for qlogis_* ones
nngp_covparms <- function(shape_params, shape, lo = .5, span = .5) {
  tr <- vapply(seq_along(shape_params), function(j) {
    if (substr(shape_params[j], 1, 3) == "log") exp(shape[j])
    else lo + span * stats::plogis(shape[j])
  }, 0)
  c(1, tr, 0)
}

nngp_abi_version <- function() .Call(C_nngp_abi_version)
nngp_status_string <- function(status) .Call(C_nngp_status_string, as.integer(status))
nngp_last_error <- function(ctx) .Call(C_nngp_ctx_last_error, ctx)
nngp_order_maxmin <- function(locs) .Call(C_nngp_order_maxmin, as.matrix(locs) + 0)
nngp_find_ordered_nn <- function(locs, m) .Call(C_nngp_find_ordered_nn, as.matrix(locs) + 0, as.integer(m))
nngp_greedy_coloring <- function(NNarray) .Call(C_nngp_greedy_coloring, NNarray)

nngp_context <- function(locs, NNarray, coloring, locs_match, observed_field, n_chains = 1L, device = -1L) {
  storage.mode(NNarray) <- "integer"
  .Call(C_nngp_ctx_create, as.matrix(locs) + 0, NNarray, as.integer(coloring), as.integer(locs_match),
        as.double(observed_field), as.integer(n_chains), as.integer(device))
}
nngp_context_shard <- function(locs, NNarray, coloring, locs_match, observed_field, n_ranks, rank,
                               n_chains = 1L, device = -1L) {
  storage.mode(NNarray) <- "integer"
  .Call(C_nngp_ctx_create_shard, as.matrix(locs) + 0, NNarray, as.integer(coloring), as.integer(locs_match),
        as.double(observed_field), as.integer(n_chains), as.integer(device), as.integer(n_ranks),
        as.integer(rank))
}
nngp_destroy <- function(ctx) invisible(.Call(C_nngp_ctx_destroy, ctx))
nngp_info <- function(ctx) .Call(C_nngp_ctx_info, ctx)
# the sweep engine chosen at creation and why (tile residency / LDS fallbacks)
nngp_engine_note <- function(ctx) .Call(C_nngp_ctx_engine_note, ctx)
nngp_set_chain <- function(ctx, chain) invisible(.Call(C_nngp_set_chain, ctx, as.integer(chain)))

nngp_factor <- function(ctx, which, covfun_name, covparms)
  invisible(.Call(C_nngp_factor, ctx, as.integer(which), nngp_covfun_id(covfun_name), as.double(covparms)))
nngp_get_linv <- function(ctx, which = 0L) .Call(C_nngp_get_linv, ctx, as.integer(which))
nngp_set_linv <- function(ctx, which, Linv) invisible(.Call(C_nngp_set_linv, ctx, as.integer(which), Linv + 0))
nngp_accept_factor <- function(ctx) invisible(.Call(C_nngp_accept_factor, ctx))
nngp_precision_diag <- function(ctx) .Call(C_nngp_get_precision_diag, ctx)

nngp_set_field <- function(ctx, field) invisible(.Call(C_nngp_set_field, ctx, as.double(field)))
nngp_get_field <- function(ctx) .Call(C_nngp_get_field, ctx)
nngp_set_mu <- function(ctx, mu, beta_0)
  invisible(.Call(C_nngp_set_mu, ctx, if (is.null(mu)) NULL else as.double(mu), as.double(beta_0)))
nngp_records_reserve <- function(ctx, n_rows) invisible(.Call(C_nngp_records_reserve, ctx, as.integer(n_rows)))
nngp_record_field <- function(ctx, row) invisible(.Call(C_nngp_record_field, ctx, as.integer(row)))
nngp_get_records <- function(ctx, row0, n_rows, buf = NULL) .Call(C_nngp_get_records, ctx, as.integer(row0), as.integer(n_rows), buf)
# rows x n numeric vector the selected chain's records stream into while it runs (NULL: release)
nngp_records_stream <- function(ctx, buf) invisible(.Call(C_nngp_records_stream, ctx, buf))

nngp_loglik <- function(ctx, which, beta_0, log_scale)
  .Call(C_nngp_loglik, ctx, as.integer(which), as.double(beta_0), as.double(log_scale))
# ll_compressed_sparse_chol (update_Gaussian.R:8-12) on the device factor `which`
ll_compressed_sparse_chol <- function(ctx, which, beta_0, log_scale) nngp_loglik(ctx, which, beta_0, log_scale)

nngp_sweep <- function(ctx, n_sweeps, beta_0, log_scale, log_noise_variance, seed, counter_base, z = NULL)
  invisible(.Call(C_nngp_sweep, ctx, as.integer(n_sweeps), as.double(beta_0), as.double(log_scale),
                  as.double(log_noise_variance), as.double(seed), as.double(counter_base),
                  if (is.null(z)) NULL else as.double(z)))
nngp_sweep_chains <- function(ctx, n_sweeps, beta_0, log_scale, log_noise_variance, seed, counter_base)
  invisible(.Call(C_nngp_sweep_chains, ctx, as.integer(n_sweeps), as.double(beta_0), as.double(log_scale),
                  as.double(log_noise_variance), as.double(seed), as.double(counter_base)))
nngp_sweep_timed <- function(ctx, n_sweeps, beta_0, log_scale, log_noise_variance, seed, counter_base)
  .Call(C_nngp_sweep_timed, ctx, as.integer(n_sweeps), as.double(beta_0), as.double(log_scale),
        as.double(log_noise_variance), as.double(seed), as.double(counter_base))
nngp_ancillary_propose <- function(ctx, beta_0, dlog_scale)
  invisible(.Call(C_nngp_ancillary_propose, ctx, as.double(beta_0), as.double(dlog_scale)))
nngp_ancillary_propose_chains <- function(ctx, chain_mask, beta_0, dlog_scale)
  invisible(.Call(C_nngp_ancillary_propose_chains, ctx, as.integer(chain_mask), as.double(beta_0),
                  as.double(dlog_scale)))
nngp_field_response_ratio <- function(ctx, beta_0, log_noise_variance)
  .Call(C_nngp_field_response_ratio, ctx, as.double(beta_0), as.double(log_noise_variance))
nngp_accept_field <- function(ctx) invisible(.Call(C_nngp_accept_field, ctx))
nngp_beta0_stats <- function(ctx) .Call(C_nngp_beta0_stats, ctx)
nngp_sum_squared_residuals <- function(ctx, beta_0) .Call(C_nngp_sum_squared_residuals, ctx, as.double(beta_0))
nngp_spmv <- function(ctx, which, X) .Call(C_nngp_spmv, ctx, as.integer(which), X + 0)
nngp_tri_solve <- function(ctx, which, u) .Call(C_nngp_tri_solve, ctx, as.integer(which), as.double(u))
# solves that finished in the rescue's ticket order (diagnostic)
nngp_tri_rescues <- function(ctx) .Call(C_nngp_tri_rescues, ctx)
nngp_device_normals <- function(device, seed, sweep, n)
  .Call(C_nngp_device_normals, as.integer(device), as.double(seed), as.double(sweep), as.integer(n))
# r = B (field - beta0) of the selected chain as the last sweep call left it (warm-call state)
nngp_get_sweep_r <- function(ctx) .Call(C_nngp_get_sweep_r, ctx)

nngp_shard_unique_id <- function() .Call(C_nngp_shard_unique_id)
nngp_shard_comm_init <- function(ctx, id) invisible(.Call(C_nngp_shard_comm_init, ctx, id))
nngp_factor_chains <- function(ctx, which, chain_mask, covfun, covparms)
  .Call(C_nngp_factor_chains, ctx, as.integer(which), as.integer(chain_mask), nngp_covfun_id(covfun),
        as.matrix(covparms) + 0)
nngp_loglik_chains <- function(ctx, which, chain_mask, beta_0, log_scale)
  .Call(C_nngp_loglik_chains, ctx, as.integer(which), as.integer(chain_mask), as.double(beta_0), as.double(log_scale))
# list(proposal = loglik_chains(1, ...), current = loglik_chains(0, ...)) in one pass over the rows
nngp_loglik_pair_chains <- function(ctx, chain_mask, beta_0, log_scale_prop, log_scale_cur)
  .Call(C_nngp_loglik_pair_chains, ctx, as.integer(chain_mask), as.double(beta_0), as.double(log_scale_prop),
        as.double(log_scale_cur))
# one host sync for a proposal's factor and its MH step (update_Gaussian.R:123-131 / :179-186):
# list(status, ratio) / list(status, proposal, current); a failed factor (status 3): NaN values
nngp_ancillary_step_chains <- function(ctx, chain_mask, covfun, covparms, beta_0, dlog_scale, log_noise_variance)
  .Call(C_nngp_ancillary_step_chains, ctx, as.integer(chain_mask), nngp_covfun_id(covfun), as.matrix(covparms) + 0,
        as.double(beta_0), as.double(dlog_scale), as.double(log_noise_variance))
nngp_sufficient_step_chains <- function(ctx, chain_mask, covfun, covparms, beta_0, log_scale_prop, log_scale_cur)
  .Call(C_nngp_sufficient_step_chains, ctx, as.integer(chain_mask), nngp_covfun_id(covfun), as.matrix(covparms) + 0,
        as.double(beta_0), as.double(log_scale_prop), as.double(log_scale_cur))
nngp_field_response_ratio_chains <- function(ctx, chain_mask, beta_0, log_noise_variance)
  .Call(C_nngp_field_response_ratio_chains, ctx, as.integer(chain_mask), as.double(beta_0),
        as.double(log_noise_variance))
nngp_sum_squared_residuals_chains <- function(ctx, chain_mask, beta_0)
  .Call(C_nngp_sum_squared_residuals_chains, ctx, as.integer(chain_mask), as.double(beta_0))
nngp_shard_ipc_handle <- function(ctx) .Call(C_nngp_shard_ipc_handle, ctx)
nngp_shard_ipc_open <- function(ctx, handles) invisible(.Call(C_nngp_shard_ipc_open, ctx, handles))
# collective over the ranks of a tile shard: full exchange of the replicas
# (the readers of the field refuse a stale replica)
nngp_shard_sync <- function(ctx) invisible(.Call(C_nngp_shard_sync, ctx))
nngp_sweep_chains_group <- function(ctxs, n_sweeps, beta_0, log_scale, log_noise_variance, seed, counter_base)
  invisible(.Call(C_nngp_sweep_chains_group, ctxs, as.integer(n_sweeps), as.double(beta_0), as.double(log_scale),
                  as.double(log_noise_variance), as.double(seed), as.double(counter_base)))
