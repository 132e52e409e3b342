// Launch wrappers for the NNGP HIP kernels (gfx950).  Internal C++ header.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

namespace nngp {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kRedBlocks = 4096;  // max partial blocks of a reduction

// per-chain scalars read by the sweep kernels from device memory (graph-replay safe)
struct SweepScalars {
  double inv_s2;     // exp(-log_scale)
  double inv_t2;     // exp(-log_noise_variance)
  double beta0;
  double dshift;     // warm tile call after a beta_0-only change: w -= dshift, r -= dshift B 1 (else 0)
  uint64_t seed;
  uint64_t counter_base;
};

constexpr int kSweepRows = 16;  // == kRowsMax of the layout planner
constexpr int kMaxChains = 4;

constexpr int kPkRowBits = 25;                    // ent_pk = rowpos | q << 25
constexpr int kPkPadRow = (1 << kPkRowBits) - 1;  // padding rowpos

// device pointers of the merge-path sweep layout (graph_prep.h); per-chain
// arrays interleave the chains (slot*C + chain, row*C + chain) so the chains of
// one entry share cache lines; ent_val is chain-planar (chain*n_entries + e).
// Per-slot arrays are in compact order (graph_prep.h): slot q of chunk ch is
// compact index chunk_first[ch] + q.
struct SweepDev {
  const int2* sinfo;          // n: {obs_per_loc, f0 | collen << 16}
  const int* compact_loc;     // n: location of each compact index
  double2* dr;                // n x C: {precision_diag, residuals_sum}
  const double* ent_val;      // C x n_entries
  const int* ent_pk;          // n_entries
  const uint16_t* ent_pos;    // n_entries: stream position of each (row-sorted) cell
  const uint16_t* start_mask; // nchunks x LW: bit j = stream cell lane*16+j begins a slot
  double* w_slot;             // n x C
  double* r;                  // n x C, Morton rows
  const SweepScalars* scal;   // C
  long long n_entries;
  int C;                      // chains in the context
  int LW;                     // lanes per chain (64, 32, 16, 16 for 1..4 chains); <= 2*LW-1 slots per chunk
  const int* chunk_first;     // nchunks+1: compact index of each chunk's first slot
  const int* loc_rank;        // n: compact index of each location (device row order independent)
  unsigned long long* dbg;    // diagnostic timestamps (NNGP_PROBE=9 builds only), else null
};

// one colour launch of the sweep (+ the next sweep's normals of the colour)
struct ColorLaunch {
  int chunk0, nch;            // chunks of the colour
  int chain_mask;
  int sweep_local;            // sweep index inside the call
  const double* z_cur;        // this sweep's normals, compact order x C
  double* z_next;             // next sweep's normals (nullptr: none generated)
  const int* pairs;           // pair ids whose normals this colour generates
  int npairs;
  int n;
  double2* xsend = nullptr;   // sharded sweep: {dw, w_new} of compact slot x at xsend[(x - xs0)*C + chain]
  int xs0 = 0;                //   (nullptr: single rank)
};

// colour-sharded sweep (graph_prep.h ShardPlan): after the exchange of colour
// c, apply the ghost cells r[row] += B[k,j] dw_j and the replica updates
// w_slot[x] = w_new of the foreign slots of the colour, for the chains in mask
struct ShardGhostLaunch {
  const int* grow;            // ghost cells of the colour (g0 .. g0+ng)
  const int* grecv;
  const double* gval;         // C x ng_total, chain-planar
  long long ng_total;
  int g0, ng;
  const double2* xbuf;        // exchange region of the colour: slot*C + chain
  int G, rank, cnt;
  int seg0[65];               // compact boundaries of the ranks inside the colour
  int chain_mask;
};
hipError_t launch_shard_ghosts(hipStream_t st, const SweepDev& L, const ShardGhostLaunch& a);

// coordinate transform into the isotropic unit-range space (per covfun)
hipError_t launch_scale_coords(hipStream_t st, int covfun, const double* cp, int ncp,
                               const double* locs_rm, int n, int d, double* sc, int ds_stride);

// Vecchia factor: Linv (row-major n x b) from scaled coords.  fail: device int
// (0 = ok, else 1 + first failing row; atomicMin semantics).
hipError_t launch_factor(hipStream_t st, int family, double var, double nugget, double nu,
                         const double* sc, int ds, const int* nn, int n, int b, double* linv,
                         int* fail);

// the factors of up to kMaxChains chains (one covariance family) in ONE
// launch of each of the two kernels: scaled coordinates of every job (and its
// failure flag reset to INT_MAX), then the factor rows of all jobs as one
// grid-stride range (one tail instead of one per chain).  Rows bitwise those
// of launch_scale_coords + launch_factor per job.
struct ScaleArgs {
  double c[8];  // covariance parameters
  int covfun;
};
struct FactorJobs {
  int n_jobs = 0;
  ScaleArgs sa[kMaxChains];
  double var[kMaxChains], nugget[kMaxChains];
  double* sc[kMaxChains];                   // per-job scaled coordinates (n x ds)
  double* linv[kMaxChains];
  int* fail[kMaxChains];
};
hipError_t launch_factor_jobs(hipStream_t st, int family, double nu, const FactorJobs& J,
                              const double* locs_rm, int n, int d, int ds, const int* nn, int b);

// per-row statistics of B x (x shifted): partial sums of
// {log L[k][0], u_k^2, a_k^2, a_k*u_k} with u = B (x - shift), a = B 1.
// If out != nullptr, out[k] = u_k.  All arrays in device row order.
// Returns #blocks used.
int launch_row_stats(hipStream_t st, const double* linv, const int* nn, int n, int b,
                     const double* x, double shift, double* out,
                     double* partials /* kRedBlocks x 4 */,
                     const double* shift_dev = nullptr /* overrides shift when set */,
                     const double* const* linv_dev = nullptr /* overrides linv when set */,
                     int out_stride = 1);
// row statistics of up to kRowJobsMax (factor, field) jobs in ONE pass over
// the rows: the NNarray entries are read once for all jobs; per job exactly
// row_stats_kernel's products, butterfly and accumulation order (bitwise the
// same partials), partials of job j at partials + j * kRedBlocks * 4, its
// totals at res[4 * res_slot[j]] after launch_reduce4_jobs.  Returns #blocks.
constexpr int kRowJobsMax = 8;  // e.g. 4 chains x (proposal, current factor)
struct RowJobs {
  const double* linv[kRowJobsMax];
  const double* x[kRowJobsMax];
  double shift[kRowJobsMax];
  double* out[kRowJobsMax];   // nullptr: no per-row output
  int res_slot[kRowJobsMax];
  // 0: per-row output only (no partials); 1: statistics incl. sum log L[k][0];
  // 2: statistics without the log term (the caller has it: it depends on the
  // factor only)
  int mode[kRowJobsMax];
  int M = 0;
  int out_stride = 1;
};
int launch_row_stats_jobs(hipStream_t st, const RowJobs& J, const int* nn, int n, int b,
                          double* partials /* kRowJobsMax x kRedBlocks x 4 */);
hipError_t launch_reduce4_jobs(hipStream_t st, const RowJobs& J, const double* partials, int nblocks, double* res);
// r = B (field_chain - beta0_chain) for every chain in mask: out[k*C + chain]
// (factor of chain k: *linv_dev[k]; the row's NNarray read once)
// field pointer of each chain (device row order)
struct FieldPtrs { double* p[kMaxChains]; };
hipError_t launch_spmv_chains(hipStream_t st, const double* const* linv_dev, const int* nn, int n, int b,
                              const FieldPtrs& f, const SweepScalars* sc, double* out, int C, int mask);
// reduce `nblocks` x 4 partials into res[4] (deterministic order)
hipError_t launch_reduce4(hipStream_t st, const double* partials, int nblocks, double* res);
// dst[k] = p in stream order
hipError_t launch_set_ptr(hipStream_t st, const double** dst, int k, const double* p);

// chain `chain`: ent_val[chain] from Linv (device order) and
// dr[s*C+chain].x = precision_diag, for chunks [0, nchunks)
hipError_t launch_sell_refresh(hipStream_t st, const SweepDev& L, int nchunks, const int* ent_src,
                               const double* linv, int chain);

// residual sums of up to kMaxChains chains in one pass (chain J.chain[j]:
// mu J.mu[j], or beta0 J.beta0[j] when null)
struct ResJobs {
  const double* mu[kMaxChains] = {};
  double beta0[kMaxChains] = {};
  int chain[kMaxChains] = {};
  int M = 0;
};
hipError_t launch_residual_sums_jobs(hipStream_t st, int n, const SweepDev& L, const ResJobs& J,
                                     const int* obs_ptr, const int* obs_idx, const double* y,
                                     const double* ysum = nullptr, const int2* sinfo = nullptr);
// obs reductions (as launch_obs_reduce) of up to kMaxChains chains in one
// pass; partials of job j at partials + j * kRedBlocks * 4.  Returns #blocks.
struct ObsJobs {
  const double* mu[kMaxChains] = {};
  double beta0[kMaxChains] = {};
  const double* f[kMaxChains] = {};
  const double* fnew[kMaxChains] = {};
  double inv_2var[kMaxChains] = {};
  int M = 0;
};
int launch_obs_reduce_jobs(hipStream_t st, int mode, int n_obs, const double* y, const int* lm, const ObsJobs& J,
                           double* partials);
// dr[x*C+chain].y = residuals_sum of the observations of compact slot x
hipError_t launch_residual_sums(hipStream_t st, int n, const SweepDev& L, int chain, const int* obs_ptr,
                                const int* obs_idx, const double* y, const double* mu, double beta0);

// w[x*C+chain] = field_chain[dpos[x]] - beta0 (and back), x compact, for
// every chain in mask in one pass (field of chain k: f.p[k])
hipError_t launch_field_to_slots_multi(hipStream_t st, int n, const int* slot_dpos, const FieldPtrs& f,
                                       const SweepScalars* sc, double* w_slot, int C, int mask);
hipError_t launch_slots_to_field_multi(hipStream_t st, int n, const int* slot_dpos, const FieldPtrs& f,
                                       const SweepScalars* sc, const double* w_slot, int C, int mask);

// one colour of the chromatic sweep for the chains in a.chain_mask
hipError_t launch_sweep_color(hipStream_t st, const SweepDev& L, const ColorLaunch& a);

// normals of sweep (counter_base + sweep_off) for every location, compact order
hipError_t launch_normals_compact(hipStream_t st, const SweepDev& L, int chain_mask, int sweep_off, int n,
                                  double* z);

// ---- tile-resident sweep (graph_prep.h TileLayout): one persistent launch
// runs every sweep of a call; r of each tile's local rows stays in its LDS;
// colour c's dw of exported slots is handed to the neighbour tiles through
// dwx (sc1 stores / loads) behind a per-tile progress flag.
struct TileDev {
  const int4* batch;          // own batches {off, R, nslots, slot0}
  const int* batch_ptr;       // T*K+1
  const uint32_t* cell_pk;    // n_cells
  const double* cell_val;     // C x n_cells
  long long n_cells;
  const int2* gcell;          // n_gcells: {local row, index of its foreign slot in the (tile, colour)}
  const double* gval;         // C x n_gcells
  long long n_gcells;
  const int* gptr;            // T*K+1
  const int* gslot;           // foreign slots of each (tile, colour): slot index
  const int* gslot_ptr;       // T*K+1
  const int* batch_split;     // T*K: split layouts, first boundary batch of (tile, colour); else null
  const int* nb_ptr;          // T*K+1
  const int* nb;
  const int* erow_ptr;        // T+1
  const int* erow;            // local row -> device row
  const int2* sinfo;          // per slot {obs_per_loc, f0 | exported}
  const int* slot_loc;        // per slot: location (normals)
  const uint32_t* rmask;      // tile shard: per slot, ranks (other than the owner's) reading its dw, else null
  double2* dr;                // per slot x C {precision_diag, residuals_sum}
  double* w_slot;             // per slot x C
  double* dwx;                // per slot x C: 16-byte granules {dw, epoch, call id}
  const double* r;            // device rows x C (r = B w at call start)
  double* rg;                 // tiles with r in global memory: local rows x C (null: r in LDS)
  const SweepScalars* scal;   // C
  const double* const* b1;    // C: B 1 of each chain's current factor (device rows; read when scal.dshift != 0)
  unsigned* ctl;              // [0] call id (bumped on the device before every launch), [1] timeout word
  unsigned long long* dbg;    // NNGP_PROBE=9 / 2: per-tile phase times / per-phase timeline, else null
  int K, C, T, n;
  int max_gslots;             // max foreign slots of a (tile, colour): LDS of their dw
  int probe = 0;              // dbg layout: 1 = per-tile segment sums (T x 8), 2 = timeline (T x 512 phases x 8)
  int xw = 0;                 // exchange-wave tiles: the last wave polls the hand-offs, the
                              // layout's batches are cut for NT - 64 cell threads
};

struct TileLaunch {
  int n_sweeps;
  int chain_mask;
  const double* z_in;         // injected normals, per sweep: slot x C (nullptr: Philox inline)
  int stagger = 0;            // chain-split: chain k starts k x stagger ticks (100 MHz) late
  int variant = 0;            // NNGP_TILE_VARIANT: experiment bits (probe builds only)
};

// cells per thread of an own batch (the layout's RMAX): two batches of C
// chains stay in registers (C >= 3: fewer cells per batch)
// double-buffered batch registers (the next colour's loads in flight during
// this colour's work) where two batches fit in registers
// (256-thread tiles at 3 chains, one wave per SIMD with 512 registers, double
// buffered: 7.7k vs 10.7k chain-sweeps/s -- the own work needs the waves)
constexpr int tile_double_buffer(int C, int NT) { return C <= 2 ? 1 : 0; }
constexpr int tile_rmax(int C, int NT) { return 4096 / NT; }
// chain-split launches (one chain per workgroup, 3 waves per SIMD): 2048-cell
// batches keep the kernel within its 168 registers
constexpr int tile_rmax_cs(int NT) { return 2048 / NT; }
// ghost-cell registers per thread: NT * GMAX ghost cells of a (tile, colour) per pass
constexpr int tile_gmax(int NT) { return NT == 256 ? 4 : (NT == 512 ? 3 : 1); }
// Tile-sharded sweep: the T tiles of the layout are split
// over G ranks (rank h runs tiles [h*Tl, (h+1)*Tl)); a launch runs the tiles
// [tile0, tile0 + grid) -- one rank's (a process per GPU) or every rank's
// (the ranks of a group on one device).  A draw read by tiles of other ranks
// is also stored into those ranks' granule buffers (peer memory over xGMI),
// so every tile polls its own rank's buffer only.
constexpr int kTileRanksMax = 16;
struct TileShard {
  int G = 1, Tl = 0, tile0 = 0, rank0 = 0;
  const TileDev* devs = nullptr;     // device array: the TileDev of ranks rank0, rank0 + 1, ... of this launch
  const unsigned* call = nullptr;    // call-id word of the launch (every rank tags with the same id)
  double* gx[kTileRanksMax] = {};    // granule buffer of every rank (this process's mapping)
};
// occ != nullptr: no launch; *occ = workgroups of the instantiation this call
// would launch that are resident on one CU at once (occupancy query)
hipError_t launch_sweep_tiles(hipStream_t st, const TileDev& D, const TileLaunch& a, int max_rows, int NT,
                              int max_batches, int max_gslots, const TileShard* sh = nullptr, int grid = 0,
                              int* occ = nullptr);
// chain-split launch: D.C one-chain workgroups per tile (256-thread layouts,
// one GPU), the chains' phases interleaved on each CU
hipError_t launch_sweep_tiles_cs(hipStream_t st, const TileDev& D, const TileLaunch& a, int max_rows, int NT,
                                 int max_batches, int max_gslots, int* occ = nullptr);
// ctl[0] += 1 (call id), ctl[1] = 0 (timeout word): before every launch of a rank
hipError_t launch_tile_call_bump(hipStream_t st, unsigned* ctl);
// tests: the control words a launch whose tiles timed out leaves behind
hipError_t launch_tile_inject_timeout(hipStream_t st, unsigned* ctl);
// tile shard, w exchange by peer copies instead of RCCL: signal the peers
// (flag word `rank` of every other rank := call id), wait for theirs
struct TilePeerFlags { unsigned* f[kTileRanksMax] = {}; };
// (flag words carry the exchange sequence number, the same on every rank)
hipError_t launch_tile_xsignal(hipStream_t st, const TilePeerFlags& pf, unsigned seq, int G, int rank);
hipError_t launch_tile_xwait(hipStream_t st, const unsigned* xflag, unsigned* ctl, unsigned seq, int G, int rank);
// halo slots of w into the peers' replicas: hptr[h] .. hptr[h+1] = peer h's
// entries of `halo` (hptr[kTileRanksMax] = all entries)
struct TilePeerW { double* w[kTileRanksMax] = {}; int hptr[kTileRanksMax + 1] = {}; };
hipError_t launch_tile_halo_put(hipStream_t st, const TilePeerW& pw, const int* halo, const double* w, int C);
// chain `chain`: cell/ghost values from Linv (device order) and precision_diag
// work items of the refresh, dealt to kRefreshLists (= XCDs) lists by tile;
// olen = the longest list
struct TileBatch;  // graph_prep.h
constexpr int kRefreshLists = 8;
constexpr int kRefreshCells = 4096;  // cells of one work item (a run of batches): its LDS
std::vector<int4> tile_refresh_order(const std::vector<int>& batch_ptr, const std::vector<int>& gptr,
                                     const std::vector<TileBatch>& batch, int NT, int T, int K, int& olen);
hipError_t launch_tile_refresh(hipStream_t st, const TileDev& D, const int4* order, int olen, int NT,
                               const int* cell_src, const int* gsrc, const double* linv, int chain);

// obs reductions: mode 0 -> partial[0] += (y - f[loc] - mu + beta0)^2
//                 mode 1 -> partial[0] += ((y-b)^2 - (y-a)^2) / (2 sd^2),
//                           a = fnew[loc]+mu-beta0, b = f[loc]+mu-beta0
int launch_obs_reduce(hipStream_t st, int mode, int n_obs, const double* y, const double* mu,
                      double beta0, const int* locs_match0, const double* field,
                      const double* field_new, double inv_2var, double* partials);

// triangular solve over up to kMaxChains chains: factor of chain slot kk =
// linv[kk], vector element (row d, chain kidx[kk]) at d*stride + kidx[kk]
struct TriArgs {
  const double* linv[kMaxChains];
  int kidx[kMaxChains];
  int nc;
  int stride;
};
hipError_t launch_tri_level(hipStream_t st, const TriArgs& a, const int* rows, int nrows, const int* nn, int b,
                            const double* u, double* x);
// levels [lv0, lv1) of the DAG (small ones) in one 1024-thread workgroup
hipError_t launch_tri_levels_block(hipStream_t st, const TriArgs& a, const int* rows, const int* lptr, int lv0,
                                   int lv1, const int* nn, int b, const double* u, double* x);
// the whole DAG in one sync-free launch (rows = all levels back to back,
// nrows of them); x (x_len doubles) is overwritten with a pending sentinel
// first; ctl: 4 words -- [0] set if a wait timed out (sticky until the host
// clears it), [1] the rescue word, [2..3] the rescue ticket counter (both
// reset by the launch; kernels.hip tri_dag_kernel); rescue: every wave takes
// the ticket order from the start (tests)
// B 1 (row sums of a factor): the warm tile call after a beta_0-only change
hipError_t launch_linv_rowsum(hipStream_t st, const double* linv, int n, int b, double* out);
hipError_t launch_tri_dag(hipStream_t st, const TriArgs& a, const int* rows, int nrows, const int* nn, int b,
                          const double* u, double* x, long long x_len, unsigned* ctl, bool rescue = false,
                          int oversub = 1);
// y[i] = shift + scale * x[i*xstride]
// dst[i] = src[idx[i]] (gather) / dst[idx[i]] = src[i] (scatter), i < n:
// R order <-> device row order of a field-sized vector
hipError_t launch_permute_gather(hipStream_t st, int n, const int* idx, const double* src, double* dst);
hipError_t launch_permute_scatter(hipStream_t st, int n, const int* idx, const double* src, double* dst);
hipError_t launch_axpby_shift(hipStream_t st, int n, const double* x, int xstride, double scale, double shift,
                              double* y);

// busy-wait on the device for `seconds` (bounded; measurement helper)
hipError_t launch_spin(hipStream_t st, double seconds);

hipError_t launch_normals(hipStream_t st, uint64_t seed, uint64_t sweep, int n, double* z);

}  // namespace nngp
