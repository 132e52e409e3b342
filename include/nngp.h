/*
 * nngp.h -- C ABI of the MI355X-native NNGP chromatic-Gibbs hot path.
 *
 * Drop-in boundary for the reference's L1/L0 calls on the hot path (SURVEY.md
 * §8b).  Plain pointers and sizes only; no torch / C++ types cross it.  All
 * host arrays use R's conventions: matrices column-major, indices 1-based,
 * NA_integer_ == INT_MIN.  Every entry point returns 0 (NNGP_OK) or an
 * nngp_status; a context keeps the message of its last error
 * (nngp_ctx_last_error).  Host inputs are read-only for the call; outputs are
 * caller-allocated.  Device state is owned by the context and freed only by
 * nngp_ctx_destroy.  Calls on one context are serialised by the caller;
 * distinct contexts may live on distinct devices.  HIP is initialised lazily
 * by nngp_ctx_create: never fork() after it.  A context holds 1..4 MCMC chains
 * over the same locations / NNarray / colouring (replaces the per-chain
 * workers of parallel::mclapply, Scripts/mcmc_nngp_update_Gaussian.R:25-26):
 * per-chain entry points act on the chain chosen by nngp_set_chain, and
 * nngp_sweep_chains sweeps all chains of the context in the same kernels.
 *
 * Reference interface each entry point replaces (path:line under the
 * reference tree):
 *   nngp_order_maxmin ........ GpGp::order_maxmin, Scripts/mcmc_nngp_initialize.R:29
 *   nngp_find_ordered_nn ..... GpGp::find_ordered_nn, Scripts/mcmc_nngp_initialize.R:93
 *   nngp_greedy_coloring ..... moral graph Scripts/mcmc_nngp_initialize.R:97-109 +
 *                              naive_greedy_coloring Scripts/Coloring.R:2-20
 *   nngp_factor .............. GpGp::vecchia_Linv + Matrix::sparseMatrix,
 *                              Scripts/mcmc_nngp_update_Gaussian.R:72-73,123-124,179-180
 *   nngp_accept_factor ....... precision_diag refresh, update_Gaussian.R:140-142,195-197
 *   nngp_loglik .............. ll_compressed_sparse_chol (+GpGp::Linv_mult),
 *                              Scripts/mcmc_nngp_update_Gaussian.R:8-12,184-186
 *   nngp_set_mu .............. mu + residuals_sum, update_Gaussian.R:85-90,249-250,260
 *   nngp_sweep ............... chromatic sampling, update_Gaussian.R:257-275
 *   nngp_sweep_chains ........ the same for every chain (mclapply over chains,
 *                              update_Gaussian.R:25-26, around :257-275)
 *   nngp_ancillary_propose ... new_field, update_Gaussian.R:127 (SpMV + sparse
 *                              triangular solve); _chains: every chain at once
 *   nngp_field_response_ratio  dnorm ratio, update_Gaussian.R:129-131
 *   nngp_beta0_stats ......... beta_0 Gibbs block, update_Gaussian.R:221-222
 *   nngp_sum_squared_residuals update_Gaussian.R:281
 *   nngp_record_field ........ records$field[i, ] = field, update_Gaussian.R:305-311
 *   nngp_records_stream ...... records$field in host memory while the chain runs (same lines)
 *   nngp_spmv / nngp_tri_solve sparse_chol %*% X (update_Gaussian.R:79,147) /
 *                              Matrix::solve (initialize.R:208, predict.R:46)
 */
#ifndef NNGP_H_
#define NNGP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NNGP_ABI_VERSION 14  /* 14: nngp_tri_rescues; 13: nngp_records_stream; 12: nngp_info gained tile_rows_needed, device_lds */
#define NNGP_SHARD_ID_BYTES 128 /* RCCL unique id */
#define NNGP_IPC_HANDLE_BYTES 192 /* HIP IPC handles of a tile shard's granule buffer, w replica, flags */

typedef enum {
  NNGP_OK = 0,
  NNGP_ERR_ARG = 1,     /* invalid argument / shape */
  NNGP_ERR_HIP = 2,     /* HIP runtime error (message in the context) */
  NNGP_ERR_CHOL = 3,    /* local covariance not positive definite */
  NNGP_ERR_STATE = 4,   /* call out of order (e.g. sweep before factor) */
  NNGP_ERR_NOMEM = 5,   /* host or device allocation failed */
  NNGP_ERR_NODEV = 6,   /* no HIP device available */
  NNGP_ERR_COMM = 7     /* RCCL error */
} nngp_status;

/* Covariance functions (GpGp names; covparms = c(variance, shape..., nugget)). */
typedef enum {
  NNGP_EXPONENTIAL_ISOTROPIC = 0, /* (var, range, nugget)                */
  NNGP_EXPONENTIAL_SPHERE = 1,    /* (var, range[Earth radii], nugget)   */
  NNGP_EXPONENTIAL_SCALEDIM = 2,  /* (var, range_1..range_d, nugget)     */
  NNGP_EXPONENTIAL_SPACETIME = 3, /* (var, range_space, range_time, nug) */
  NNGP_MATERN_ISOTROPIC = 4,      /* (var, range, smoothness, nugget)    */
  NNGP_MATERN_SPHERE = 5,         /* (var, range, smoothness, nugget)    */
  NNGP_MATERN_SCALEDIM = 6,       /* (var, range_1..range_d, smooth, nug)*/
  NNGP_MATERN_SPACETIME = 7,      /* (var, r_space, r_time, smooth, nug) */
  NNGP_MATERN15_ISOTROPIC = 8     /* (var, range, nugget); extension     */
} nngp_covfun;

typedef struct nngp_ctx nngp_ctx;

typedef struct {
  int n;           /* locations */
  int b;           /* m + 1 */
  int d;           /* coordinate dimension */
  int n_obs;       /* observations */
  int n_colors;    /* K */
  int n_levels;    /* depth of the Vecchia DAG (triangular solve) */
  long long nnz;   /* nonzeros of B */
  long long n_entries; /* sliced-ELL entries incl. padding */
  int max_collen;  /* longest column of B */
  int device;      /* HIP device ordinal */
  int n_chains;    /* chains held by the context */
  int lanes_per_chain; /* sweep lanes of one chain in a wavefront (64/32/16) */
  int n_chunks;    /* sweep chunks (wavefront tasks per chain and sweep) */
  int sweep_engine;  /* 0: one launch per colour, 1: tile-resident persistent sweep */
  int n_tiles;       /* tiles (persistent workgroups) of the tile engine */
  int tile_rows_max; /* max local rows (own + foreign) of a tile: its resident r */
  long long n_ghost_cells; /* foreign-member cells the tiles (or shard ranks) apply after a hand-off */
  int n_ranks;       /* shard contexts: ranks of the sharded sweep (0: not sharded);
                        sweep_engine 0: colour shard, 1: tile shard */
  int rank;          /* shard contexts: this context's rank */
  long long shard_owned;          /* locations swept by this rank */
  long long shard_needed_rows;    /* rows of B its columns touch (its r halo included) */
  long long shard_exchange_slots; /* colour shard: slots of all colours' exchange regions (padded);
                                     tile shard: locations whose draws other ranks read */
  int tile_ghost_pass;       /* tile engine: ghost cells a (tile, colour) applies per register pass */
  int tile_ghost_cells_max;  /* tile engine: most ghost cells of one (tile, colour) */
  int tile_r_global;         /* tile engine: 1 = the tiles' r in global memory (layout beyond the LDS) */
  int tile_chain_split;      /* tile engine: 1 = one workgroup per (chain, tile), the chains of a tile on one CU */
  int tile_resident_per_cu;  /* tile engine: workgroups of its kernel resident per CU at once (occupancy query);
                                the persistent launch needs tiles <= this x CUs, else the colour engine runs */
  int engine_fallback;       /* why not the tile engine: 0 = it runs, 1 = layout unsuitable (LDS, shape),
                                2 = residency (more tile workgroups than fit the device at once),
                                3 = NNGP_ENGINE=colors / more ranks than the tile shard takes */
  int tile_exchange_wave;    /* tile engine: 1 = the last wave of each tile polls the hand-offs (NT - 64 cell threads) */
  int device_cus;            /* compute units of the context's device */
  int tile_rows_needed;      /* largest local-row count of a tile in the tile layout built for this context
                                (also when the tile engine was not used or keeps r in global memory; 0: none built) */
  int device_lds;            /* LDS bytes per CU of the context's device */
} nngp_info;

/* ---------- library ---------- */
int nngp_abi_version(void);
const char* nngp_status_string(int status);

/* ---------- host-side graph preparation (init-time, C++) ---------- */
/* locs: n x d column-major.  order: 1-based permutation (length n). */
int nngp_order_maxmin(const double* locs, int n, int d, int* order);
/* NNarray: n x (m+1) column-major, 1-based, NA = INT_MIN. Exact NN on the raw
 * coordinates, ties broken by the smaller index. */
int nngp_find_ordered_nn(const double* locs, int n, int d, int m, int* NNarray);
/* coloring: length n, 1-based colours; *n_colors = K. */
int nngp_greedy_coloring(const int* NNarray, int n, int b, int* coloring, int* n_colors);

/* ---------- device context ---------- */
/* locs n x d col-major (ordered); NNarray n x b col-major 1-based (NA=INT_MIN);
 * coloring 1-based (length n); locs_match 1-based (length n_obs);
 * observed_field length n_obs; n_chains 1..4 (chain 0 selected).
 * device: HIP ordinal (-1: current). */
int nngp_ctx_create(const double* locs, int n, int d, const int* NNarray, int b,
                    const int* coloring, const int* locs_match,
                    const double* observed_field, int n_obs, int n_chains, int device,
                    nngp_ctx** out);
/* select the chain (0-based) the per-chain entry points below act on */
int nngp_set_chain(nngp_ctx* ctx, int chain);
void nngp_ctx_destroy(nngp_ctx* ctx);
const char* nngp_ctx_last_error(const nngp_ctx* ctx);
int nngp_ctx_info(const nngp_ctx* ctx, nngp_info* info);
/* one line: the sweep engine chosen at creation and why (e.g. the residency
 * or LDS reason the tile engine was not used); owned by the context */
const char* nngp_ctx_engine_note(const nngp_ctx* ctx);

/* Vecchia factor (A4).  which: 0 = current factor, 1 = proposal. */
int nngp_factor(nngp_ctx* ctx, int which, int covfun, const double* covparms, int ncovparms);
/* copy a factor out as GpGp's Linv (n x b column-major, unfilled entries 0) */
int nngp_get_linv(nngp_ctx* ctx, int which, double* Linv);
/* upload an externally computed Linv (n x b col-major) into `which` */
int nngp_set_linv(nngp_ctx* ctx, int which, const double* Linv);
/* proposal factor becomes current; refreshes the sweep values + precision_diag (A5) */
int nngp_accept_factor(nngp_ctx* ctx);
/* precision_diag = colSums(B o B) of the current factor (length n) */
int nngp_get_precision_diag(nngp_ctx* ctx, double* D);

/* latent field (length n, location order) */
int nngp_set_field(nngp_ctx* ctx, const double* field);
int nngp_get_field(nngp_ctx* ctx, double* field);
/* mu (length n_obs): beta_0 + X beta; recomputes residuals_sum (A7).
 * mu == NULL means mu = beta0 for every observation. */
int nngp_set_mu(nngp_ctx* ctx, const double* mu, double beta0);

/* On-device field records (records$field, update_Gaussian.R:56,305-311 with
 * field_thinning): the selected chain's device buffer of n_rows
 * x n (location order); record_field copies the current field into row `row`
 * without a host round trip; get_records copies rows [row0, row0+n_rows) out
 * (row-major n_rows x n).  reserve(0) frees the buffer. */
int nngp_records_reserve(nngp_ctx* ctx, int n_rows);
int nngp_record_field(nngp_ctx* ctx, int row);
int nngp_get_records(nngp_ctx* ctx, int row0, int n_rows, double* out);
/* Streams the selected chain's recorded rows into a caller-owned host array
 * (n_rows x n row-major, n_rows = the reserved rows) as they are recorded: a
 * worker thread copies each row behind the stream while the chain runs, and
 * nngp_get_records(ctx, row0, k, host + row0 * n) only waits for them (rows
 * not recorded since the binding are copied from the device there).  The
 * array must stay valid until that get_records, the next records_reserve,
 * nngp_records_stream(ctx, NULL, 0) or nngp_ctx_destroy, which all end the
 * binding (after the rows in flight have landed).  A call that fails leaves
 * an existing binding in place. */
int nngp_records_stream(nngp_ctx* ctx, double* host, int n_rows);

/* Vecchia log-likelihood (A6) of z = field - beta0 under factor `which` */
int nngp_loglik(nngp_ctx* ctx, int which, double beta0, double log_scale, double* ll);

/* n_sweeps chromatic sweeps (A1).  Normals: Philox4x32-10 with key = seed,
 * counter = (location, counter_base + sweep, 0x5EED) unless z != NULL, in which
 * case z (n_sweeps x n row-major, z[s*n + i]) supplies them.  Stream-ordered:
 * the call may return before the sweeps have run (the only tile context of a
 * device; NNGP_SWEEP_SYNC=1 waits); every entry point that hands results to
 * the host waits for them, and reports a tile timeout of an earlier sweep. */
int nngp_sweep(nngp_ctx* ctx, int n_sweeps, double beta0, double log_scale,
               double log_noise_variance, uint64_t seed, uint64_t counter_base,
               const double* z);

/* n_sweeps sweeps of EVERY chain of the context in the same kernels; arrays
 * of length n_chains.  Chain k's result is bitwise identical to nngp_sweep on
 * chain k alone with the same arguments. */
int nngp_sweep_chains(nngp_ctx* ctx, int n_sweeps, const double* beta0, const double* log_scale,
                      const double* log_noise_variance, const uint64_t* seed,
                      const uint64_t* counter_base);

/* Ancillary proposal: proposal field = beta0 + exp(0.5*dlog_scale) *
 * B_prop^{-1} (B_cur (field - beta0)) (update_Gaussian.R:127). */
int nngp_ancillary_propose(nngp_ctx* ctx, double beta0, double dlog_scale);
/* nngp_ancillary_propose for the chains in chain_mask (bit k = chain k) in
 * the same kernels (one triangular-solve schedule for all of them); beta0 and
 * dlog_scale have n_chains entries (others ignored).  Chain k's proposal is
 * bitwise identical to nngp_ancillary_propose on chain k alone. */
int nngp_ancillary_propose_chains(nngp_ctx* ctx, int chain_mask, const double* beta0,
                                  const double* dlog_scale);
/* sum dnorm(y | proposal) - sum dnorm(y | field), sd = exp(lnv/2) (A8) */
int nngp_field_response_ratio(nngp_ctx* ctx, double beta0, double log_noise_variance,
                              double* ratio);
/* proposal field becomes current */
int nngp_accept_field(nngp_ctx* ctx);
/* 1'B'B1 and 1'B'B field (current factor) -- beta_0 Gibbs (update_Gaussian.R:221-222) */
int nngp_beta0_stats(nngp_ctx* ctx, double* ones_Q_ones, double* ones_Q_field);
/* sum (y - field[loc] - mu + beta0)^2 (update_Gaussian.R:281) */
int nngp_sum_squared_residuals(nngp_ctx* ctx, double beta0, double* ssr);
/* Batched forms for the chains in chain_mask (bit k = chain k), one host
 * synchronisation per call: parameter and result arrays have n_chains
 * entries (entries of other chains ignored).  factor_chains: covparms is
 * n_chains x ncovparms (row k = chain k); status[k] = NNGP_OK or
 * NNGP_ERR_CHOL per chain (the call itself returns NNGP_OK then).  Each
 * chain's result is bitwise the single-chain entry point's. */
int nngp_factor_chains(nngp_ctx* ctx, int which, int chain_mask, int covfun, const double* covparms,
                       int ncovparms, int* status);
int nngp_loglik_chains(nngp_ctx* ctx, int which, int chain_mask, const double* beta0,
                       const double* log_scale, double* ll);
int nngp_field_response_ratio_chains(nngp_ctx* ctx, int chain_mask, const double* beta0,
                                     const double* log_noise_variance, double* ratio);
int nngp_sum_squared_residuals_chains(nngp_ctx* ctx, int chain_mask, const double* beta0, double* ssr);
/* The sufficient MH step's two log-likelihoods (update_Gaussian.R:184-186:
 * ll_compressed_sparse_chol of the proposal minus that of the current factor)
 * for the chains in chain_mask in ONE pass over the rows: ll_prop[k] =
 * nngp_loglik_chains(1, ...) with log_scale_prop, ll_cur[k] =
 * nngp_loglik_chains(0, ...) with log_scale_cur, bitwise. */
int nngp_loglik_pair_chains(nngp_ctx* ctx, int chain_mask, const double* beta0, const double* log_scale_prop,
                            const double* log_scale_cur, double* ll_prop, double* ll_cur);
/* One Metropolis-Hastings covariance step behind ONE host sync (the separate
 * calls take two or three).  covparms, status as nngp_factor_chains (factor 1
 * = the proposal of each chain in chain_mask); then, enqueued before any
 * factor's outcome is known:
 *   ancillary_step_chains  (update_Gaussian.R:123-131): nngp_ancillary_propose_chains
 *     with beta0 / dlog_scale and nngp_field_response_ratio_chains with beta0 / lnv
 *     -> ratio[k];
 *   sufficient_step_chains (update_Gaussian.R:179-186): nngp_loglik_pair_chains
 *     -> ll_prop[k], ll_cur[k].
 * A chain whose proposal factor is not positive definite reports
 * status NNGP_ERR_CHOL and NaN results; every other chain's results are
 * bitwise those of the separate calls. */
int nngp_ancillary_step_chains(nngp_ctx* ctx, int chain_mask, int covfun, const double* covparms, int ncovparms,
                               const double* beta0, const double* dlog_scale, const double* log_noise_variance,
                               int* status, double* ratio);
int nngp_sufficient_step_chains(nngp_ctx* ctx, int chain_mask, int covfun, const double* covparms, int ncovparms,
                                const double* beta0, const double* log_scale_prop, const double* log_scale_cur,
                                int* status, double* ll_prop, double* ll_cur);
/* Y = B X for X n x ncols column-major (host buffers) */
int nngp_spmv(nngp_ctx* ctx, int which, const double* X, int ncols, double* Y);
/* x = B^{-1} u (host buffers, length n) */
int nngp_tri_solve(nngp_ctx* ctx, int which, const double* u, double* x);
/* Diagnostics of the sync-free solve (update_Gaussian.R:127): the solves of
 * this context so far whose static order stalled (a wave waited 20 ms on one
 * group, e.g. its inputs' waves were not resident) and finished in the
 * ticket order of the rescue; forced ticket orders (NNGP_TRI_RESCUE=1) do not
 * count.  Waits for the context's stream. */
int nngp_tri_rescues(nngp_ctx* ctx, long long* out);

/* ---------- colour-sharded sweep (multi-GPU) ----------
 * The chromatic sweep of ONE set of chains split over n_ranks contexts (one
 * per GPU, one process per GPU): rank g sweeps its spatial block of every
 * colour class, and after each colour the ranks all-gather {dw, w_new} of the
 * colour's locations (RCCL over xGMI) and apply the updates that cross their
 * block boundary.  Results are bitwise identical to n_ranks = 1.  A shard
 * context supports every entry point above (factor, loglik, field, ... are
 * computed redundantly on every rank) except nngp_sweep with injected
 * normals and nngp_sweep_timed; nngp_sweep / nngp_sweep_chains run the sharded
 * sweep (n_ranks > 1: after nngp_shard_comm_init).  Replaces the per-colour
 * masked update of update_Gaussian.R:261-275 across devices. */
int nngp_ctx_create_shard(const double* locs, int n, int d, const int* NNarray, int b,
                          const int* coloring, const int* locs_match,
                          const double* observed_field, int n_obs, int n_chains, int device,
                          int n_ranks, int rank, nngp_ctx** out);
/* rank 0 creates the id (len >= NNGP_SHARD_ID_BYTES) and sends it to the
 * other ranks out of band (e.g. torch.distributed broadcast) */
int nngp_shard_unique_id(unsigned char* id, int len);
/* collective over the n_ranks contexts: RCCL communicator of the shard */
int nngp_shard_comm_init(nngp_ctx* ctx, const unsigned char* id, int len);
/* all n_ranks shard contexts in ONE process (ctxs[g] = rank g; any devices):
 * nngp_sweep_chains with the exchange done by device copies between them.
 * Tile shards: the ranks of one device run in one launch (their tiles must fit
 * the device's CUs together), ranks on one device contiguous. */
int nngp_sweep_chains_group(nngp_ctx** ctxs, int n_ranks, int n_sweeps, const double* beta0,
                            const double* log_scale, const double* log_noise_variance,
                            const uint64_t* seed, const uint64_t* counter_base);

/* Tile shard (sweep_engine 1 on a shard context, the default when the tile
 * layout fits): the tile-resident sweep with its tiles split over the ranks
 * (rank g runs tiles [g*T/G, (g+1)*T/G) on its GPU).  A draw read by a tile
 * of another rank is written into that rank's granule buffer (peer memory
 * over xGMI) by the producing tile, so the hand-offs stay inside the one
 * persistent launch per call.  After the launch the ranks' replicas of the
 * field are brought up to date: with a communicator (nngp_shard_comm_init),
 * one grouped RCCL broadcast of every rank's slots; without one (the
 * default), each rank stores only its halo -- its slots that other ranks'
 * rows contain -- into the peers' replicas (peer stores + device flags), and
 * the other foreign slots of each replica fall behind until nngp_shard_sync.
 * Setup, every rank: export this rank's handles (nngp_shard_ipc_handle),
 * exchange them out of band (all-gather), open the others'
 * (nngp_shard_ipc_open).  NNGP_ENGINE=colors at creation selects the colour
 * shard instead. */
int nngp_shard_ipc_handle(nngp_ctx* ctx, unsigned char* handle, int len);
/* handles: n_ranks x len_each bytes, rank order (this rank's entry ignored).
 * Without a communicator (no nngp_shard_comm_init) a call exchanges w by
 * peer copies into the mapped replicas and device flags instead of RCCL. */
int nngp_shard_ipc_open(nngp_ctx* ctx, const unsigned char* handles, int len_each);
/* Collective over the ranks of a tile shard without a communicator (every
 * rank calls it, in the same order relative to its sweeps): the full
 * exchange of the field replicas.  After sweeps without it, the entry points
 * that read the field (nngp_get_field, nngp_record_field, nngp_loglik*,
 * nngp_beta0_stats, nngp_field_response_ratio*, nngp_sum_squared_residuals*,
 * nngp_ancillary_propose*, nngp_accept_field) return NNGP_ERR_STATE -- a
 * reader never performs a hidden collective.  A no-op on every other
 * context and on an up-to-date replica. */
int nngp_shard_sync(nngp_ctx* ctx);

/* ---------- measurement ---------- */
/* nngp_sweep_chains bracketed by HIP events on the context's stream;
 * *ms = elapsed for the whole call; *kernel_ms (if not NULL) = elapsed for the
 * n_sweeps x n_colors sweep-kernel launches alone (a graph of only those
 * launches between two events: mean launch time = kernel_ms / launches). */
int nngp_sweep_timed(nngp_ctx* ctx, int n_sweeps, const double* beta0, const double* log_scale,
                     const double* log_noise_variance, const uint64_t* seed,
                     const uint64_t* counter_base, double* ms, double* kernel_ms);
/* Philox normals generated by the device code path (test hook). */
int nngp_device_normals(int device, uint64_t seed, uint64_t sweep, int n, double* z);
/* r = B (field - beta0) of the selected chain as the last sweep call left it
 * (location order, length n): the state a warm tile call starts from (the
 * tile kernel writes its r back).  Introspection for the
 * warm-call drift tests -- nngp_spmv gives the fresh product to compare. */
int nngp_get_sweep_r(nngp_ctx* ctx, double* r);

#ifdef __cplusplus
}
#endif
#endif /* NNGP_H_ */
