// C ABI (include/nngp.h) of the MI355X-native NNGP chromatic-Gibbs hot path.
// One nngp_ctx per group of <= 4 MCMC chains: device buffers, the sweep layout planned on the
// host (graph_prep.cpp), one HIP stream, and cached hipGraphs of the sweep.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <atomic>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/nngp.h"
#include "graph_prep.h"
#include "kernels.h"
#include "rec_stream.h"

using namespace nngp;

// Device row order: every row-indexed device array (locations, NNarray,
// Linv, field, r) is stored in Morton order ("dpos" = lay.rpos[loc]) so the
// neighbour gathers of the factor build, the SpMV and the sweep hit nearby
// lines; the host boundary converts to and from the Vecchia (location) order.
//
// A context holds C <= 4 chains over the same locations / NNarray / colouring
// (the reference's n_chains, each with its own covariance parameters, factor,
// field and mean).  Per-chain entry points act on the chain selected by
// nngp_set_chain; nngp_sweep_chains sweeps every chain in the same kernels.
struct ChainState {
  double* linv_d[2] = {nullptr, nullptr};
  double* field_d = nullptr;
  double* field_prop_d = nullptr;
  double* mu_d = nullptr;
  double* rec_d = nullptr;  // on-device field records: rec_rows x n, location order
  int rec_rows = 0;
  double* rec_host = nullptr;  // caller's host array the rows are streamed into (nngp_records_stream)
  std::vector<uint8_t> rec_pushed;  // rows handed to the streamer since the binding (the others: copied at get_records)
  bool have_factor[2] = {false, false};
  bool have_field = false, have_mu = false, mu_is_const = true;
  double mu_beta0 = 0.0;
  // generations of the field and of the two factor slots (bumped on every
  // write) and the last row-statistics passes (nngp_loglik) they produced:
  // nngp_beta0_stats reuses a pass over the current factor and field
  uint64_t fgen = 1, lgen[2] = {1, 1};
  struct RowStats { uint64_t lg = 0, fg = 0; double shift = 0.0, r[4] = {0, 0, 0, 0}; } rs[2];
  // sum_k log Linv[k][0] of the last two factors seen by a log-likelihood
  // pass (keyed by the factor generation): later passes over the same factor
  // skip the n logs
  struct LogDet { uint64_t lg = 0; double v = 0.0; } ld[2];
  int ld_next = 0;
  // warm sweep calls (tile engine, one GPU): the last call left w in slot
  // order and r = B w (the tile kernel writes its r back) for this field,
  // factor and beta0 -- the next call with all three unchanged skips its
  // prologue (field -> slots, r = B w)
  bool warm = false;
  uint64_t warm_fgen = 0, warm_lgen = 0;
  double warm_beta0 = 0.0;
  // B 1 of the current factor (device rows; generation b1_lgen): a call whose
  // field and factor are unchanged but beta_0 moved (the no-X beta_0 Gibbs
  // step, update_Gaussian.R:219-224) stays warm -- w -= d, r -= d B 1
  double* b1_d = nullptr;
  uint64_t b1_lgen = 0;
  int rs_next = 0;
  // the sweep's copy of the current factor (tile cells / colour entries and
  // precision_diag) is behind it: refreshed before the next reader (a sweep,
  // nngp_get_precision_diag), so a chain that accepts two proposals in one
  // MCMC iteration refreshes once
  bool vals_stale = false;
  // the residual sums (SweepDev::dr .y) are behind mu / beta_0: recomputed for
  // every such chain in one pass before the next sweep (flush_sweep_values)
  bool res_stale = false;
};

// res_d / res_h: 4 x kRowJobsMax reduction results, then the kMaxChains
// failure flags of the factors (fail_d / fail_h)
constexpr int kResFailOff = 4 * kRowJobsMax;
constexpr size_t kResBytes = kResFailOff * sizeof(double) + kMaxChains * sizeof(int);
static_assert(kResBytes % sizeof(double) == 0, "res_d holds whole doubles");

// tile-engine contexts per device (persistent launches of two contexts on one
// device must not overlap: see tile_lock)
std::atomic<int>& tile_ctx_count(int device) {
  static std::atomic<int> counts[64];
  return counts[device & 63];
}

struct nngp_ctx {
  ~nngp_ctx() {
    if (tile_counted) tile_ctx_count(device)--;
  }
  bool tile_counted = false;  // counted in tile_ctx_count(device)
  RecordStreamer* recs = nullptr;  // record rows -> host arrays (nngp_records_stream), lazily started
  // a sweep returned without a host sync: its tile timeout word is checked
  // after the next one (sync_stream)
  bool tile_pending = false;
  uint64_t gen = 1;  // generation counter of ChainState::fgen / lgen
  int device = 0;
  hipStream_t st = nullptr;
  int n = 0, d = 0, b = 0, n_obs = 0, ds = 2;
  int C = 1, cur = 0;
  std::string err;
  SweepLayout lay;
  std::vector<int> dpos;   // loc -> device row (== lay.rpos)
  std::vector<int> level_ptr, level_rows;
  ChainState ch[kMaxChains];
  // device buffers
  double* locs_d = nullptr;  // n x d row-major
  double* sc_d = nullptr;    // n x ds scaled coordinates
  double* scm_d = nullptr;   // per-chain scaled coordinates of a multi-chain factor launch
  size_t scm_cap = 0;        // its capacity in doubles
  int* nn_d = nullptr;       // n x b row-major, 0-based, -1 = NA
  const double** linv_cur_d = nullptr;  // C pointers: current factor of each chain
  const double** linv_cur_h = nullptr;  // pinned mirror
  const double** b1_tab_d = nullptr;    // C pointers: each chain's B 1 buffer (ChainState::b1_d; TileDev::b1)
  int* fail_d = nullptr;         // inside res_d (kResFailOff)
  int2* sinfo_d = nullptr;       // n compact: {obs_per_loc, f0 | collen << 16}
  int* compact_loc_d = nullptr;  // n
  double2* dr_d = nullptr;
  int* slot_dpos_d = nullptr;
  int* dpos_d = nullptr;          // loc -> device row, on the device
  double* stage_h = nullptr;      // pinned n-double staging for field-sized copies
  double* mu_stage_h = nullptr;   // pinned n_obs-double staging of set_mu
  hipEvent_t mu_stage_ev = nullptr;
  double* perm_d = nullptr;       // device n-double scratch of those copies (R order)
  int* chunk_first_d = nullptr;  // nchunks+1
  int* loc_rank_d = nullptr;     // n: compact index of each location (Vecchia order)
  int* pairs_d = nullptr;        // normal pairs grouped by the colour of their even member
  std::vector<int> pair_ptr;     // K+1
  std::vector<int> loc_rank;     // host copy
  double* zbuf_d = nullptr;      // 2 x n x C: normals of the current / next sweep
  int* ent_pk_d = nullptr;
  uint16_t* ent_pos_d = nullptr;
  uint16_t* start_mask_d = nullptr;
  int* ent_src_d = nullptr;
  double* ent_val_d = nullptr;   // C x n_entries
  double* w_slot_d = nullptr;    // n x C
  double* r_d = nullptr;         // n x C
  int* level_rows_d = nullptr;
  int* level_ptr_d = nullptr;    // DAG level offsets (device copy)
  std::vector<int> tri_seg;      // solve plan: (lv0, lv1, kind) triples, kind 1 = one-workgroup run
  bool tri_dag = false;          // NNGP_TRI=dag: one sync-free launch for the whole DAG
  bool tri_rescue = false;       // NNGP_TRI_RESCUE=1: its ticket order from the start (tests)
  unsigned* tri_tmo_d = nullptr; // its control words: [0] timeout, [1] rescue, [2..3] rescue tickets, [4] rescues raised
  int tri_oversub = 1;            // NNGP_TRI_OVERSUB=k: k x the resident grid (tests: the static order cannot finish)
  unsigned* tri_tmo_h = nullptr; // pinned copy, read at the next host sync
  int* obs_ptr_d = nullptr;
  double* ysum_d = nullptr;       // per slot (compact order): the sum of its observations' y (residual sums, mu = beta_0)
  int* obs_idx_d = nullptr;
  int* lm_d = nullptr;  // locs_match, 0-based
  double* y_d = nullptr;
  double* tmp_d = nullptr;
  double* tmp2_d = nullptr;
  double* partials_d = nullptr;
  double* res_d = nullptr;
  double* z_d = nullptr;
  size_t z_cap = 0;
  SweepScalars* scal_d = nullptr;  // C
  SweepScalars* scal_h = nullptr;  // pinned, C: the next call's scalars (sweep_prepare)
  // staging ring of the scalar uploads: a sweep call returns before its
  // upload has run, so the next call stages into another slot (a slot is
  // reused once its previous copy has run: its event)
  static constexpr int kScalRing = 8;
  SweepScalars* scal_ring_h = nullptr;  // pinned, kScalRing x C
  hipEvent_t scal_ev[kScalRing] = {};
  int scal_next = 0;
  double* res_h = nullptr;         // pinned, 4 x kRowJobsMax doubles, then fail_h
  int* fail_h = nullptr;           // pinned, kMaxChains failure rows of the factors (inside res_h)
  unsigned long long* dbg_d = nullptr;  // NNGP_PROBE=9: per-chunk timestamps
  // tile-resident sweep engine (engine == 1; graph_prep.h TileLayout)
  int engine = 0;                 // 0: colour launches, 1: tiles
  TileLayout tl;
  int4* tb_d = nullptr;           // own batches
  int* tb_ptr_d = nullptr;
  uint32_t* cell_pk_d = nullptr;
  int* cell_src_d = nullptr;
  double* cell_val_d = nullptr;   // C x cells
  int2* gcell_d = nullptr;
  int* gsrc_d = nullptr;
  int4* rorder_d = nullptr;       // tile_refresh work items (kRefreshLists x rorder_len)
  int rorder_len = 0;
  double* gval_d = nullptr;       // C x ghost cells
  int* gptr_d = nullptr;
  int* gslot_d = nullptr;
  int* gslot_ptr_d = nullptr;
  int* bsplit_d = nullptr;        // split tile layouts: first boundary batch of (tile, colour)
  int* nb_ptr_d = nullptr;
  int* nb_d = nullptr;
  int* erow_ptr_d = nullptr;
  int* erow_d = nullptr;
  double* dwx_d = nullptr;        // n x C granules of 16 B
  bool rglobal = false;           // tiles keep r in global memory (rg_d) instead of LDS
  bool warm_on = false;           // warm sweep calls allowed (tile engine, not a shard; NNGP_SWEEP_WARM=0: off)
  bool tcs = false;               // chain-split tile launches (one chain per workgroup, kernels.hip sweep_tiles_cs_kernel)
  int txw = 0;                    // exchange-wave tiles (tiles.hip tile_phase_xw): layout cut for NT - 64 cell threads
  int cus = 0;                    // compute units of the device
  int tresident = 0;              // tile workgroups resident per CU (occupancy query of the instantiation)
  int engine_fallback = 0;        // 0: none, 1: tile layout unsuitable (LDS, shape), 2: residency, 3: forced colours
  std::string engine_note;        // why this sweep engine (nngp_ctx_engine_note)
  int tstagger = 0;               // chain-split: start offset per chain (NNGP_TILE_STAGGER, 100 MHz ticks)
  int tvariant = 0;               // NNGP_TILE_VARIANT (probe builds): experiment bits
  int tile_rows_needed = 0;       // largest local rows of a tile of the layout built here (nngp_info)
  int lds_max = 0;                // LDS bytes per CU of the device
  double* rg_d = nullptr;         // sum of the tiles' local rows x C
  unsigned* ctl_d = nullptr;      // [0] call id, [1] timeout word of a launch, [2] sticky timeout (tiles.hip)
  unsigned* tmo_h = nullptr;      // pinned copy of the sticky timeout word after each launch
  int inject_tmo = 0;             // tests (NNGP_TILE_INJECT_TIMEOUT=k): the first k sweep calls report a timeout
  unsigned long long* tdbg_d = nullptr;  // NNGP_PROBE=9: per-tile phase times, =2: per-phase timeline
  size_t tdbg_n = 0;
  int tprobe = 0;
  // colour-sharded sweep (nngp_ctx_create_shard; graph_prep.h ShardPlan):
  // this context is rank sp.rank of sp.G; it sweeps its own chunks of every
  // colour and exchanges {dw, w_new} of the colour's slots through xbuf_d
  // (RCCL all-gather, or device copies between the contexts of a group)
  bool shard = false;
  ShardPlan sp;
  int* sg_row_d = nullptr;        // ghost cells: device row
  int* sg_recv_d = nullptr;       //              exchange index
  int* sg_src_d = nullptr;        //              Linv index
  double* sg_val_d = nullptr;     //              B value, C x cells
  double2* xbuf_d = nullptr;      // exchange regions of all colours: slot x C
  int* sp_pairs_d = nullptr;      // normal pairs of the rank
  ncclComm_t comm = nullptr;
  // tile shard (engine 1 on a shard context): rank trank of tG runs tiles
  // [trank*tTl, (trank+1)*tTl) of the layout (graph_prep.h TileLayout::G)
  int tG = 0, trank = 0, tTl = 0;
  uint32_t* rmask_d = nullptr;     // per slot: remote reader ranks
  TileDev* tdev_d = nullptr;       // kTileRanksMax entries: this rank's TileDev, or a group's
  double* peer_gx[kTileRanksMax] = {};  // the other ranks' granule buffers (IPC mappings)
  double* peer_w[kTileRanksMax] = {};   // ... their w replicas (exchange without RCCL)
  unsigned* peer_xf[kTileRanksMax] = {};  // ... their exchange flag words
  unsigned* xflag_d = nullptr;          // kTileRanksMax flag words the peers write (exchange numbers)
  bool peers_open = false;
  // exchange without RCCL: after a call only the halo (this rank's slots read
  // by other ranks' rows) goes out; the chains in stale_mask then have a
  // replica whose other foreign slots are behind, brought up to date by a
  // full exchange before anything reads the field (SPMD: every rank does it
  // at the same entry point)
  int* halo_d = nullptr;
  int halo_ptr[kTileRanksMax + 1] = {};
  unsigned xseq = 0;
  int stale_mask = 0;
  std::map<long long, hipGraphExec_t> graphs;  // key: n_sweeps << 8 | chain mask
  std::vector<hipGraph_t> graph_objs;
};

namespace {

constexpr int kTileNT = 512;       // threads per tile workgroup (NNGP_TILE_NT: 256, 512, 1024)
constexpr int kTileTarget = 2048;  // locations per tile (default tile count: n / this, <= CUs)

thread_local std::string g_err;

int fail_hip(nngp_ctx* c, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  if (c) c->err = m;
  g_err = m;
  return NNGP_ERR_HIP;
}
int fail_msg(nngp_ctx* c, int code, const std::string& m) {
  if (c) c->err = m;
  g_err = m;
  return code;
}

#define HIPCHK(c, x)                                       \
  do {                                                     \
    hipError_t e_ = (x);                                   \
    if (e_ != hipSuccess) return fail_hip((c), e_, #x);    \
  } while (0)

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  return hipMalloc((void**)p, sizeof(T) * count);
}
// the buffers other ranks of a tile shard store into over xGMI while this
// rank's kernels read them (granules, the w replica, the exchange flags):
// fine-grained device memory, coherent with the peers' stores (a coarse-
// grained line of them held in this GPU's L2 could be read stale)
template <typename T>
hipError_t shared_alloc(T** p, size_t count, bool fine) {
  if (count == 0) count = 1;
  if (!fine) return hipMalloc((void**)p, sizeof(T) * count);
  return hipExtMallocWithFlags((void**)p, sizeof(T) * count, hipDeviceMallocFinegrained);
}
template <typename T>
hipError_t upload(T* dst, const T* src, size_t count, hipStream_t st) {
  if (count == 0) return hipSuccess;
  return hipMemcpyAsync(dst, src, sizeof(T) * count, hipMemcpyHostToDevice, st);
}

// (after a host sync) the sticky timeout word of the launches since the last
// check: reported once, then cleared on the device too
static int tile_timeout_check(nngp_ctx* c) {
  if (c->engine == 1 && c->tmo_h && *c->tmo_h != 0) {
    *c->tmo_h = 0;
    HIPCHK(c, hipMemsetAsync(c->ctl_d + 2, 0, sizeof(unsigned), c->st));
    return fail_msg(c, NNGP_ERR_HIP, "tile sweep: neighbour wait timed out (tiles not co-resident?)");
  }
  return NNGP_OK;
}

// host sync of the context's stream; then the timeout word of a sweep that
// returned without one
int sync_stream(nngp_ctx* c) {
  HIPCHK(c, hipStreamSynchronize(c->st));
  if (c->tile_pending) {
    c->tile_pending = false;
    return tile_timeout_check(c);
  }
  return NNGP_OK;
}

int set_device(nngp_ctx* c) {
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return fail_hip(c, e, "hipSetDevice");
  return NNGP_OK;
}

// sweep-layout pointers
SweepDev sweep_dev(nngp_ctx* c) {
  SweepDev L;
  L.sinfo = c->sinfo_d;
  L.compact_loc = c->compact_loc_d;
  L.dr = c->dr_d;
  L.ent_val = c->ent_val_d;
  L.ent_pk = c->ent_pk_d;
  L.ent_pos = c->ent_pos_d;
  L.start_mask = c->start_mask_d;
  L.w_slot = c->w_slot_d;
  L.r = c->r_d;
  L.scal = c->scal_d;
  L.n_entries = c->lay.n_entries;
  L.C = c->C;
  L.LW = c->lay.LW;
  L.chunk_first = c->chunk_first_d;
  L.loc_rank = c->loc_rank_d;
  L.dbg = c->dbg_d;
  return L;
}

TileDev tile_dev(nngp_ctx* c) {
  TileDev D;
  D.batch = c->tb_d;
  D.batch_ptr = c->tb_ptr_d;
  D.cell_pk = c->cell_pk_d;
  D.cell_val = c->cell_val_d;
  D.n_cells = (long long)c->tl.cell_pk.size();
  D.gcell = c->gcell_d;
  D.gval = c->gval_d;
  D.n_gcells = (long long)c->tl.gsrc.size();
  D.gptr = c->gptr_d;
  D.gslot = c->gslot_d;
  D.gslot_ptr = c->gslot_ptr_d;
  D.batch_split = c->tl.split ? c->bsplit_d : nullptr;
  D.max_gslots = c->tl.max_gslots;
  D.nb_ptr = c->nb_ptr_d;
  D.nb = c->nb_d;
  D.erow_ptr = c->erow_ptr_d;
  D.erow = c->erow_d;
  D.sinfo = c->sinfo_d;
  D.slot_loc = c->compact_loc_d;
  D.rmask = c->rmask_d;
  D.dr = c->dr_d;
  D.w_slot = c->w_slot_d;
  D.dwx = c->dwx_d;
  D.r = c->r_d;
  D.rg = c->rg_d;
  D.scal = c->scal_d;
  D.ctl = c->ctl_d;
  D.dbg = c->tdbg_d;
  D.probe = c->tprobe;
  D.xw = c->txw;
  D.b1 = c->b1_tab_d;
  D.K = c->tl.K;
  D.C = c->C;
  D.T = c->tl.T;
  D.n = c->n;
  return D;
}

int flush_one(nngp_ctx* c, int k);

// chain k's current factor changed: the pointer table of captured graphs and
// the sweep values, now (stream order, no host buffer).  NNGP_REFRESH=deferred
// refreshes the values at their next reader instead (flush_sweep_values: a
// chain accepting two proposals refreshes once) -- measured slower in the
// MCMC iteration, 1.5 refreshes of 334 us against 1.7 of 208 us: right after
// the factor its Linv is still in the Infinity Cache.
int refresh_sweep_values(nngp_ctx* c, int k) {
  c->linv_cur_h[k] = c->ch[k].linv_d[0];
  HIPCHK(c, launch_set_ptr(c->st, c->linv_cur_d, k, c->ch[k].linv_d[0]));
  c->ch[k].vals_stale = true;
  static const bool deferred = [] {
    const char* e = std::getenv("NNGP_REFRESH");
    return e && std::string(e) == "deferred";
  }();
  return deferred ? NNGP_OK : flush_one(c, k);
}

// sweep values of B + precision_diag of chain k from its current factor
int flush_one(nngp_ctx* c, int k) {
  if (c->engine == 1)
    HIPCHK(c, launch_tile_refresh(c->st, tile_dev(c), c->rorder_d, c->rorder_len, c->tl.NT, c->cell_src_d,
                                  c->gsrc_d, c->ch[k].linv_d[0], k));
  else
    HIPCHK(c, launch_sell_refresh(c->st, sweep_dev(c), c->lay.nchunks, c->ent_src_d, c->ch[k].linv_d[0], k));
  if (c->shard && !c->sp.grow.empty()) {
    const int ng = (int)c->sp.grow.size();
    HIPCHK(c, launch_permute_gather(c->st, ng, c->sg_src_d, c->ch[k].linv_d[0], c->sg_val_d + (size_t)k * ng));
  }
  c->ch[k].vals_stale = false;
  return NNGP_OK;
}

// the sweep values of the chains in mask, where behind their current factor,
// and their residual sums, where behind mu / beta_0 (one pass for all chains)
int flush_sweep_values(nngp_ctx* c, int mask) {
  ResJobs J;
  for (int k = 0; k < c->C; ++k) {
    ChainState& S = c->ch[k];
    if (!((mask >> k) & 1) || !S.res_stale) continue;
    J.mu[J.M] = S.mu_is_const ? nullptr : S.mu_d;
    J.beta0[J.M] = S.mu_beta0;
    J.chain[J.M] = k;
    ++J.M;
  }
  if (J.M) {
    HIPCHK(c, launch_residual_sums_jobs(c->st, c->n, sweep_dev(c), J, c->obs_ptr_d, c->obs_idx_d, c->y_d, c->ysum_d,
                                        c->sinfo_d));
    // up to date only once the pass is enqueued (a failed launch leaves them stale)
    for (int q = 0; q < J.M; ++q) c->ch[J.chain[q]].res_stale = false;
  }
  for (int k = 0; k < c->C; ++k)
    if (((mask >> k) & 1) && c->ch[k].vals_stale) {
      int rc = flush_one(c, k);
      if (rc) return rc;
    }
  return NNGP_OK;
}

// Persistent tile launches: every workgroup spins on its neighbours'
// granules, so all workgroups of a launch must be resident at once.  Two such
// launches on one device at the same time -- two contexts swept from two host
// threads, each on its own stream -- could each hold part of the CUs and wait
// for the rest forever.  A call of this process that launches tiles on a
// device holds that device's lock from before the launch to the host sync
// after it: one persistent tile launch per device at a time.  (Other work --
// factor, solves -- is not held back: it does not wait on other workgroups of
// another launch and drains by itself.)
std::mutex& tile_lock(int device) {
  static std::mutex locks[64];
  return locks[device & 63];
}

// With several tile contexts on a device, their persistent launches are
// chained on the GPU instead of drained on the host: under the device's tile
// lock a launch first waits (on its stream) for the event recorded after the
// device's previous tile launch, then records its own -- no two persistent
// launches overlap, and a sweep call returns without a host sync.
static hipEvent_t& tile_chain_event(int device) {
  static hipEvent_t evs[64] = {};
  return evs[device & 63];
}

static int tile_chain_wait(nngp_ctx* c) {
  hipEvent_t& ev = tile_chain_event(c->device);
  if (ev) HIPCHK(c, hipStreamWaitEvent(c->st, ev, 0));
  return NNGP_OK;
}

static int tile_chain_record(nngp_ctx* c) {
  hipEvent_t& ev = tile_chain_event(c->device);
  if (!ev) HIPCHK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPCHK(c, hipEventRecord(ev, c->st));
  return NNGP_OK;
}

// reduce partials to res_d and copy 4 doubles to the host (synchronises)
int fetch4(nngp_ctx* c, int nblocks, double out[4]) {
  HIPCHK(c, launch_reduce4(c->st, c->partials_d, nblocks, c->res_d));
  HIPCHK(c, hipMemcpyAsync(c->res_h, c->res_d, 4 * sizeof(double), hipMemcpyDeviceToHost, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  for (int k = 0; k < 4; ++k) out[k] = c->res_h[k];
  return NNGP_OK;
}

}  // namespace

// tile shard without RCCL (defined with the sharded sweep below)
static int tile_ipc_exchange(nngp_ctx* c, bool full);
static int replica_sync(nngp_ctx* c);
// entry points that read the field of a tile-shard rank whose replica is
// behind (halo-only exchanges since the last nngp_shard_sync) refuse: the
// full exchange is a collective over the ranks, so it is the caller's
// explicit nngp_shard_sync on every rank, never a hidden one inside a reader
static int replica_fresh(nngp_ctx* c) {
  if (!c->stale_mask) return NNGP_OK;
  return fail_msg(c, NNGP_ERR_STATE, "tile shard: this rank's replica of the field is behind after sweeps without a "
                                     "communicator -- call nngp_shard_sync on every rank first");
}

// ====================================================================== ABI
extern "C" {

int nngp_abi_version(void) { return NNGP_ABI_VERSION; }

const char* nngp_status_string(int s) {
  switch (s) {
    case NNGP_OK: return "ok";
    case NNGP_ERR_ARG: return "invalid argument";
    case NNGP_ERR_HIP: return "HIP runtime error";
    case NNGP_ERR_CHOL: return "local covariance not positive definite";
    case NNGP_ERR_STATE: return "call out of order";
    case NNGP_ERR_NOMEM: return "allocation failed";
    case NNGP_ERR_NODEV: return "no HIP device";
    case NNGP_ERR_COMM: return "RCCL error";
  }
  return "unknown status";
}

// ---------------------------------------------------------------- host prep
int nngp_order_maxmin(const double* locs, int n, int d, int* order) {
  if (!locs || !order || n < 1 || d < 1) return fail_msg(nullptr, NNGP_ERR_ARG, "order_maxmin: bad args");
  std::vector<int> o;
  try { order_maxmin(locs, n, d, o); } catch (std::bad_alloc&) { return NNGP_ERR_NOMEM; }
  for (int i = 0; i < n; ++i) order[i] = o[i] + 1;
  return NNGP_OK;
}

int nngp_find_ordered_nn(const double* locs, int n, int d, int m, int* NNarray) {
  if (!locs || !NNarray || n < 1 || d < 1 || m < 0) return fail_msg(nullptr, NNGP_ERR_ARG, "find_ordered_nn: bad args");
  std::vector<int> nn;
  try { find_ordered_nn(locs, n, d, m, nn); } catch (std::bad_alloc&) { return NNGP_ERR_NOMEM; }
  const int b = m + 1;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < b; ++j) {
      int v = nn[(size_t)i * b + j];
      NNarray[i + (size_t)j * n] = v < 0 ? INT_MIN : v + 1;
    }
  return NNGP_OK;
}

static bool nn_to_rowmajor(const int* NNarray, int n, int b, std::vector<int>& nn, std::string& err) {
  nn.resize((size_t)n * b);
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < b; ++j) {
      int v = NNarray[i + (size_t)j * n];
      if (v == INT_MIN) { nn[(size_t)i * b + j] = -1; continue; }
      if (v < 1 || v > n) { err = "NNarray entry out of range"; return false; }
      if (j == 0 && v != i + 1) { err = "NNarray[, 1] must be 1..n"; return false; }
      if (j > 0 && v - 1 >= i) { err = "NNarray neighbours must precede the row (ordered NN)"; return false; }
      nn[(size_t)i * b + j] = v - 1;
    }
  }
  return true;
}

int nngp_greedy_coloring(const int* NNarray, int n, int b, int* coloring, int* n_colors) {
  if (!NNarray || !coloring || n < 1 || b < 1) return fail_msg(nullptr, NNGP_ERR_ARG, "greedy_coloring: bad args");
  std::vector<int> nn, col;
  std::string err;
  if (!nn_to_rowmajor(NNarray, n, b, nn, err)) return fail_msg(nullptr, NNGP_ERR_ARG, err);
  int K = greedy_coloring(nn.data(), n, b, col);
  std::memcpy(coloring, col.data(), sizeof(int) * n);
  if (n_colors) *n_colors = K;
  return NNGP_OK;
}

// ---------------------------------------------------------------- context
void nngp_ctx_destroy(nngp_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->st) hipStreamSynchronize(c->st);
  if (c->recs) {
    c->recs->stop();
    delete c->recs;
  }
  for (auto& kv : c->graphs) hipGraphExecDestroy(kv.second);
  for (auto g : c->graph_objs) hipGraphDestroy(g);
  std::vector<void*> ptrs = {c->locs_d, c->sc_d, c->scm_d, c->nn_d, c->linv_cur_d, c->b1_tab_d, c->sinfo_d, c->compact_loc_d,
                             c->dr_d, c->slot_dpos_d, c->ent_pk_d, c->ent_src_d, c->ent_val_d, c->w_slot_d,
                             c->r_d, c->level_rows_d, c->obs_ptr_d, c->obs_idx_d, c->ysum_d, c->lm_d, c->y_d, c->tmp_d,
                             c->tmp2_d, c->partials_d, c->res_d, c->z_d, c->scal_d, c->dbg_d,
                             c->chunk_first_d, c->loc_rank_d, c->pairs_d, c->level_ptr_d, c->zbuf_d, c->ent_pos_d, c->start_mask_d,
                             c->dpos_d, c->perm_d, c->tb_d, c->tb_ptr_d, c->cell_pk_d, c->cell_src_d,
                             c->cell_val_d, c->gcell_d, c->gsrc_d, c->gval_d, c->gptr_d, c->rorder_d, c->gslot_d, c->gslot_ptr_d, c->nb_ptr_d, c->nb_d,
                             c->erow_ptr_d, c->erow_d, c->dwx_d, c->ctl_d, c->tdbg_d, c->sg_row_d,
                             c->sg_recv_d, c->sg_src_d, c->sg_val_d, c->xbuf_d, c->sp_pairs_d, c->tri_tmo_d};
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->peers_open)
    for (int h = 0; h < c->tG; ++h) {
      if (h == c->trank) continue;
      for (void* q : {(void*)c->peer_gx[h], (void*)c->peer_w[h], (void*)c->peer_xf[h]})
        if (q) hipIpcCloseMemHandle(q);
    }
  ptrs.push_back(c->xflag_d);
  ptrs.push_back(c->halo_d);
  ptrs.push_back(c->rmask_d);
  ptrs.push_back(c->rg_d);
  ptrs.push_back(c->bsplit_d);
  ptrs.push_back(c->tdev_d);
  for (int k = 0; k < kMaxChains; ++k) {
    ChainState& s = c->ch[k];
    ptrs.insert(ptrs.end(), {s.linv_d[0], s.linv_d[1], s.field_d, s.field_prop_d, s.mu_d, s.rec_d, s.b1_d});
  }
  for (void* p : ptrs) if (p) hipFree(p);
  if (c->scal_h) hipHostFree(c->scal_h);
  if (c->scal_ring_h) hipHostFree(c->scal_ring_h);
  for (hipEvent_t& e : c->scal_ev)
    if (e) hipEventDestroy(e);
  if (c->res_h) hipHostFree(c->res_h);
  if (c->linv_cur_h) hipHostFree(c->linv_cur_h);
  if (c->stage_h) hipHostFree(c->stage_h);
  if (c->mu_stage_h) hipHostFree(c->mu_stage_h);
  if (c->mu_stage_ev) hipEventDestroy(c->mu_stage_ev);
  if (c->tmo_h) hipHostFree(c->tmo_h);
  if (c->tri_tmo_h) hipHostFree(c->tri_tmo_h);
  if (c->st) hipStreamDestroy(c->st);
  delete c;
}

const char* nngp_ctx_last_error(const nngp_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }

// shard_G > 0: a rank of the colour-sharded sweep (colour-launch engine)
// the longest column of B (entries of a location in the NNarray rows)
static int max_column_length(const int* nn, int n, int b) {
  std::vector<int> cl(n, 0);
  int mx = 0;
  for (long long e = 0; e < (long long)n * b; ++e)
    if (nn[e] >= 0) mx = std::max(mx, ++cl[nn[e]]);
  return mx;
}

// lanes per chain of the colour engine's chunks (a column must fit one chunk
// of LW x kRowsMax entries): 3 chains use the 4-chain shape (measured faster
// than 21 lanes) unless a column is longer than its 256 entries (m = 20:
// up to 275), then 21 lanes (336 entries)
static int colour_lanes(int C, int max_col) {
  if (const char* e = std::getenv("NNGP_COLOUR_LANES"))  // tests: 21 lanes at 3 chains
    if (C == 3 && std::atoi(e) == 21) return 21;
  if (C == 1) return 64;
  if (C == 2) return 32;
  if (C == 3 && max_col > 16 * kRowsMax) return 21;
  return 16;
}

static int ctx_create(const double* locs, int n, int d, const int* NNarray, int b, const int* coloring,
                      const int* locs_match, const double* observed_field, int n_obs, int n_chains,
                      int device, int shard_G, int shard_rank, nngp_ctx** out) {
  if (!out) return fail_msg(nullptr, NNGP_ERR_ARG, "ctx_create: out == NULL");
  *out = nullptr;
  if (!locs || !NNarray || !coloring || !locs_match || !observed_field || n < 1 || d < 1 || d > 4 ||
      b < 1 || b > 32 || n_obs < 1 || n_chains < 1 || n_chains > kMaxChains)
    return fail_msg(nullptr, NNGP_ERR_ARG,
                    "ctx_create: bad arguments (need n>=1, 1<=d<=4, 1<=b<=32, n_obs>=1, 1<=n_chains<=4)");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail_msg(nullptr, NNGP_ERR_NODEV, "no HIP device");
  nngp_ctx* c = new (std::nothrow) nngp_ctx();
  if (!c) return NNGP_ERR_NOMEM;
  if (device < 0) { if (hipGetDevice(&device) != hipSuccess) device = 0; }
  if (device >= ndev) { delete c; return fail_msg(nullptr, NNGP_ERR_ARG, "device ordinal out of range"); }
  c->device = device;
  c->n = n; c->d = d; c->b = b; c->n_obs = n_obs; c->C = n_chains;
  c->ds = d <= 2 ? 2 : (d == 3 ? 3 : 4);
  int rc;
  std::vector<int> nn;
  std::string err;
  if (!nn_to_rowmajor(NNarray, n, b, nn, err)) { int e = fail_msg(nullptr, NNGP_ERR_ARG, err); delete c; return e; }
  for (int i = 0; i < n; ++i)
    if (coloring[i] < 1) { delete c; return fail_msg(nullptr, NNGP_ERR_ARG, "coloring must be >= 1"); }
  // validate colouring: no two members of a Vecchia row share a colour
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < b; ++j) {
      int a = nn[(size_t)k * b + j];
      if (a < 0) continue;
      for (int q = j + 1; q < b; ++q) {
        int e2 = nn[(size_t)k * b + q];
        if (e2 >= 0 && coloring[a] == coloring[e2]) {
          delete c;
          return fail_msg(nullptr, NNGP_ERR_ARG, "coloring is not a proper colouring of the moral graph");
        }
      }
    }
  std::vector<int> lm0(n_obs), obs_cnt(n + 1, 0);
  for (int o = 0; o < n_obs; ++o) {
    if (locs_match[o] < 1 || locs_match[o] > n) { delete c; return fail_msg(nullptr, NNGP_ERR_ARG, "locs_match out of range"); }
    lm0[o] = locs_match[o] - 1;
    obs_cnt[lm0[o] + 1]++;
  }
  for (int i = 0; i < n; ++i) obs_cnt[i + 1] += obs_cnt[i];
  std::vector<int> obs_idx(n_obs);
  {
    std::vector<int> f(obs_cnt.begin(), obs_cnt.end() - 1);
    for (int o = 0; o < n_obs; ++o) obs_idx[f[lm0[o]]++] = o;
  }
  // the longest column of B, once (a scan of the n x b NNarray: 2e8 entries at
  // configs[4]): the engine choice and the colour chunks' lanes use it
  const int max_col = max_column_length(nn.data(), n, b);
  // sweep engine: tiles (one persistent launch per call, r resident in LDS)
  // when the tile layout fits a CU's LDS, else one launch per colour.
  // NNGP_ENGINE=colors|tiles forces one; NNGP_TILES=T sets the tile count.
  {
    const char* eng = std::getenv("NNGP_ENGINE");
    const std::string es = eng ? eng : "";
    if (es != "" && es != "colors" && es != "tiles") {
      delete c;
      return fail_msg(nullptr, NNGP_ERR_ARG, "NNGP_ENGINE must be colors or tiles");
    }
    // shards: the tile shard when it fits (G ranks x up to one tile per CU;
    // NNGP_TILES = the total), else the colour shard
    const int G = shard_G > 0 ? shard_G : 1;
    if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) c->cus = 0;
    if (es != "colors" && G <= kTileRanksMax) {
      int cus = 0, lds_max = 0;
      cus = c->cus;
      if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeSharedMemPerBlockOptin, device) != hipSuccess) lds_max = 0;
      c->lds_max = lds_max;
      int T = std::max(1, std::min(G * cus, (n + kTileTarget - 1) / kTileTarget));
      // NNGP_TILES may ask for more tiles than CUs: the residency check below
      // then falls back to the colour engine (the tiles spin on each other, so
      // every workgroup of the launch must be resident at once)
      if (const char* te = std::getenv("NNGP_TILES")) T = std::max(1, std::atoi(te));
      T = std::min(T, n);
      T = std::max(G, T / G * G);  // a multiple of the ranks
      std::string terr;
      int NT = kTileNT;
      // NNGP_TILE_CHAINS=split (2-4 chains, one GPU): one workgroup per
      // (chain, tile), 256-thread tiles, the chains' workgroups of a tile
      // interleaved on its CU (kernels.hip sweep_tiles_cs_kernel)
      const char* tch = std::getenv("NNGP_TILE_CHAINS");
      const std::string tcs = tch ? tch : "";
      if (tcs != "" && tcs != "split" && tcs != "joint") {
        delete c;
        return fail_msg(nullptr, NNGP_ERR_ARG, "NNGP_TILE_CHAINS must be split or joint");
      }
      const bool csplit = tcs == "split" && shard_G == 0 && n_chains >= 2;
      if (csplit) NT = 256;
      if (const char* te = std::getenv("NNGP_TILE_NT")) NT = std::atoi(te);
      if (NT != 256 && NT != 512 && NT != 1024) {
        delete c;
        return fail_msg(nullptr, NNGP_ERR_ARG, "NNGP_TILE_NT must be 256, 512 or 1024");
      }
      // NNGP_TILE_SPLIT=1 (3-4 chains): interior-first layouts (kernels.hip
      // tile_phase_ib).  Opt-in: measured 3,607 vs 2,564 us per 10-sweep
      // launch at the headline (two batches per colour, and the next colour's
      // stream no longer overlaps the hand-off with one register set)
      const char* tsp = std::getenv("NNGP_TILE_SPLIT");
      const bool split = !csplit && tile_double_buffer(n_chains, NT) == 0 && tsp && std::string(tsp) == "1";
      // a tile's own rows alone beyond the LDS: no layout to build (n = 8e6 on
      // one GPU would spend ~30 s building one that cannot run)
      // The colour engine refuses a column of B longer than its sweep chunk
      // (LW x kRowsMax entries, 256 at 3-4 chains: configs[4]'s m = 20 graph
      // at 3 chains); tiles whose r does not fit the LDS then run with r in
      // global memory rather than fail
      const bool colours_refuse = max_col > colour_lanes(n_chains, max_col) * kRowsMax;
      const bool rows_beyond_lds = (long long)(n / std::max(T, 1)) * n_chains * 8 > (long long)lds_max;
      const bool rg_forced = (std::getenv("NNGP_TILE_R") && std::string(std::getenv("NNGP_TILE_R")) == "global") ||
                             (rows_beyond_lds && colours_refuse && NT == 512);
      const bool hopeless = !rg_forced && rows_beyond_lds;
      if (hopeless) terr = "tile layout: a tile's own rows exceed the LDS";
      // cells per own batch: NT x RMAX of the kernel; NNGP_TILE_BATCH_CELLS
      // may lower it (e.g. joint tiles cut like chain-split ones, for bitwise
      // comparisons)
      int rmax_l = csplit ? tile_rmax_cs(NT) : tile_rmax(n_chains, NT);
      // exchange-wave tiles (default for 512-thread LDS tiles; NNGP_TILE_XW=0
      // turns them off): the last wave of the workgroup polls the hand-offs,
      // the batches are cut for the other NT - 64 threads.  Measured at the
      // headline: 11.16k vs 11.02k chain-sweeps/s at 3 chains, 6.34k vs 5.71k
      // at 1 chain (tiles.hip tile_phase_xw)
      const char* txe = std::getenv("NNGP_TILE_XW");
      const int xwm = txe ? std::atoi(txe) : 1;
      // wave-local batches (exchange-wave tiles): one wave per batch, the
      // layout cut for 64-lane batches in rounds of the NT/64 - 1 cell waves
      // (tiles.hip tile_phase_wl); with r in global memory too.  Default at 3+
      // chains (NNGP_TILE_WL=0 turns them off, =1 asks for them at any chain
      // count).  Measured at the headline: 12.96k vs 12.47k chain-sweeps/s at
      // 3 chains (2,218 vs 2,275 us per 10-sweep launch), 5.76k vs 7.09k at 1
      // chain
      // Not by default with r in global memory: at configs[4]'s per-GPU share
      // (n = 1.25e6, m = 20, 3 chains) 2,702 vs 2,819 chain-sweeps/s, at
      // n = 1e7 one chain 284 vs 364.
      const char* twl = std::getenv("NNGP_TILE_WL");
      const bool wl_env = twl ? std::string(twl) == "1" : (n_chains >= 3 && !rg_forced);
      // interior-first layouts run on wave-local batches (tiles.hip
      // tile_phase_wlib) or, without the exchange wave, on workgroup batches
      const bool xw = !csplit && (!split || wl_env) && (!rg_forced || wl_env) && NT == 512 && xwm == 1;
      const bool wl = xw && wl_env;
      const int NTL = wl ? 64 : (xw ? NT - 64 : NT);  // the layout's cell threads of a batch
      if (const char* bc = std::getenv("NNGP_TILE_BATCH_CELLS"))
        rmax_l = std::max(1, std::min(rmax_l, std::atoi(bc) / NTL));
      bool ok = cus > 0 && T <= n && !hopeless &&
                build_tile_layout(nn.data(), n, b, coloring, locs, d, T, NTL, rmax_l, c->tl, terr, G,
                                  split, wl ? NT / 64 - 1 : 0);
      c->tl.NTK = NT;
      c->txw = xw ? (wl ? 2 : 1) : 0;
      if (ok && csplit) {
        // n_chains workgroups of one chain per CU
        const int need1 = tile_lds_bytes(c->tl.max_rows, 1, NT, c->tl.K, c->tl.max_batches, c->tl.max_gslots);
        if (NT != 256 || (long long)need1 * n_chains > lds_max) {
          ok = false;
          terr = "chain-split tiles need 256 threads and " + std::to_string(need1) + " B of LDS per chain x " +
                 std::to_string(n_chains) + " chains per CU (device: " + std::to_string(lds_max) + ")";
        } else {
          c->tcs = true;
          if (const char* sg = std::getenv("NNGP_TILE_STAGGER")) c->tstagger = std::max(0, std::atoi(sg));
        }
      }
      const int need = ok && !csplit ? tile_lds_bytes(c->tl.max_rows, n_chains, NT, c->tl.K, c->tl.max_batches, c->tl.max_gslots) : 0;
      // NNGP_TILE_R=global: the tiles' r in global memory (tiles.hip RG; one
      // GPU, or a tile shard with 512-thread tiles),
      // one GPU, for layouts beyond the LDS.  Opt-in: at n = 1e7, m = 20 (one
      // chain) it measured 362 chain-sweeps/s (26.4 ms per 10-sweep launch,
      // 1024 threads: 341) against the colour engine's 449 -- five serial
      // batches per phase, each behind dependent global round trips -- so the
      // colour engine stays the default there
      bool force_rg = rg_forced;
      int need_now = need;
      // a tile shard (G > 1) whose LDS tiles do not fit runs tiles with r in
      // global memory instead of the colour shard (configs[4]: n = 1e7, m = 20,
      // 3 chains over 8 GPUs, tests/test_capi_and_graph.py
      // test_configs4_tile_shard_geometry): the layout is rebuilt
      // for the RG kernel's 512 cell threads
      // One GPU takes the same route when the colour engine cannot either
      if (ok && (shard_G > 1 || colours_refuse) && !force_rg && need > lds_max && NT == 512 && !csplit && !split) {
        ok = build_tile_layout(nn.data(), n, b, coloring, locs, d, T, NT, tile_rmax(n_chains, NT), c->tl, terr, G,
                               false, 0);
        c->tl.NTK = NT;
        c->txw = 0;
        force_rg = true;
        need_now = ok ? tile_lds_bytes(c->tl.max_rows, n_chains, NT, c->tl.K, c->tl.max_batches, c->tl.max_gslots) : 0;
      }
      if (ok && c->txw && !force_rg && need_now > lds_max) { ok = false; terr = "exchange-wave tiles exceed the LDS"; }
      if (ok && (need_now > lds_max || force_rg)) {
        const int need_rg = tile_lds_bytes(0, n_chains, NT, c->tl.K, c->tl.max_batches, c->tl.max_gslots);
        if (force_rg && (NT == 512 || (NT == 1024 && shard_G == 0)) && need_rg <= lds_max) {
          c->rglobal = true;
        } else {
          ok = false;
          terr = "tile layout needs " + std::to_string(need_now) +
                 " B of LDS per tile (device: " + std::to_string(lds_max) + ")";
        }
      }
      // residency: the persistent launch needs all its workgroups on the device
      // at once (tiles poll each other's granules); the occupancy of exactly
      // the instantiation that will run, at its LDS, times the CUs must cover
      // the launch's grid (one rank's tiles per process; every chain's tiles
      // of a chain-split launch)
      if (ok) {
        TileDev Dq;
        Dq.C = n_chains;
        Dq.K = c->tl.K;
        Dq.rg = c->rglobal ? reinterpret_cast<double*>(16) : nullptr;
        Dq.batch_split = c->tl.split ? reinterpret_cast<const int*>(16) : nullptr;
        Dq.xw = c->txw;
        if (const char* pr = std::getenv("NNGP_PROBE"))
          if ((std::atoi(pr) == 9 || std::atoi(pr) == 2) && (n_chains == 1 || n_chains == 3)) {
            Dq.dbg = reinterpret_cast<unsigned long long*>(16);
            Dq.probe = std::atoi(pr) == 9 ? 1 : 2;
          }
        TileShard shq;
        int per_cu = 0;
        hipError_t oe;
        if (csplit) {
          // by construction: the kernel's register budget is pinned to C
          // workgroups per CU (amdgpu_waves_per_eu) and its LDS floor allows
          // no more than C (the occupancy query rejects this kernel)
          oe = hipSuccess;
          per_cu = n_chains;
        } else
          oe = launch_sweep_tiles(nullptr, Dq, TileLaunch(), c->tl.max_rows, NT, c->tl.max_batches, c->tl.max_gslots,
                                  shard_G > 0 ? &shq : nullptr, 0, &per_cu);
        (void)hipGetLastError();
        const long long grid = csplit ? (long long)T * n_chains : (long long)(T / G);
        c->tresident = oe == hipSuccess ? per_cu : 0;
        if (oe != hipSuccess || (long long)per_cu * cus < grid) {
          ok = false;
          c->engine_fallback = 2;
          terr = "residency: " + std::to_string(grid) + " tile workgroups per device > " + std::to_string(per_cu) +
                 " resident per CU x " + std::to_string(cus) + " CUs" +
                 (oe != hipSuccess ? std::string(" (occupancy query: ") + hipGetErrorString(oe) + ")" : "");
        }
      }
      if (ok) {
        c->engine = 1;
        c->tile_rows_needed = c->tl.max_rows;
        {
          // a sweep of another tile context of this device may still be in
          // flight (it returned without a sync while it was the only one):
          // drain it before two contexts can launch
          std::lock_guard<std::mutex> lk(tile_lock(device));
          if (tile_ctx_count(device)++ > 0) (void)hipDeviceSynchronize();
        }
        c->tile_counted = true;
        {
          const char* sw = std::getenv("NNGP_SWEEP_WARM");
          c->warm_on = shard_G == 0 && !(sw && std::string(sw) == "0");
        }
        c->engine_note = "tiles: " + std::to_string(T) + " tiles of " + std::to_string(NT) + " threads, " +
                         std::to_string(c->tresident) + " resident per CU x " + std::to_string(cus) + " CUs" +
                         (c->rglobal ? ", r in global memory" : "") + (c->txw == 2 ? ", exchange wave, wave-local batches" : c->txw ? ", exchange wave" : "") +
                         (c->tl.split ? ", interior first" : "") +
                         (c->tcs ? ", chain-split" : "");
        if (shard_G > 0) {
          c->shard = true;
          c->tG = G;
          c->trank = shard_rank;
          c->tTl = T / G;
        }
      } else {
        c->tile_rows_needed = c->tl.max_rows;
        c->tl = TileLayout();
        c->txw = 0;
        c->tcs = false;
        c->rglobal = false;
        if (c->engine_fallback == 0) c->engine_fallback = 1;
        c->engine_note = "colours (tile engine not used: " + terr + ")";
        if (es == "tiles") { delete c; return fail_msg(nullptr, NNGP_ERR_ARG, "tile engine: " + terr); }
      }
    } else {
      c->engine_fallback = 3;
      c->engine_note = es == "colors" ? "colours (NNGP_ENGINE=colors)" : "colours (more ranks than the tile shard takes)";
    }
  }
  if (c->engine == 1) {
    // the tile layout defines the device row and slot orders
    SweepLayout& Lw = c->lay;
    Lw.n = n; Lw.b = b; Lw.K = c->tl.K; Lw.nnz = c->tl.nnz; Lw.max_collen = c->tl.max_collen;
    Lw.rpos = c->tl.rpos;
    Lw.compact_loc = c->tl.compact_loc;
    Lw.LW = 0; Lw.nchunks = 0;
    Lw.n_entries = (long long)c->tl.cell_pk.size() + (long long)c->tl.gsrc.size();
  } else {
    const int LW = colour_lanes(n_chains, max_col);
    if (!build_sweep_layout(nn.data(), n, b, coloring, locs, d, LW, c->lay, err)) {
      delete c;
      return fail_msg(nullptr, NNGP_ERR_ARG, err);
    }
    if (shard_G > 0 && shard_G > kMaxRanks) {
      delete c;
      return fail_msg(nullptr, NNGP_ERR_ARG, "colour shard: too many ranks");
    }
    if (shard_G > 0) {
      if (!build_shard_plan(nn.data(), n, b, coloring, c->lay, shard_G, shard_rank, c->sp, err)) {
        delete c;
        return fail_msg(nullptr, NNGP_ERR_ARG, err);
      }
      c->shard = true;
    }
  }
  const SweepLayout& L = c->lay;
  static_assert(kPkRowBits == kRowBits && kPkPadRow == kPadRow, "packed entry format");
  dag_levels(nn.data(), n, b, c->level_ptr, c->level_rows);
  c->dpos = L.rpos;
  const std::vector<int>& dp = c->dpos;
  for (auto& r : c->level_rows) r = dp[r];
  // rows of a level in device (Morton) order: coalesced row loads, local x gathers
  for (size_t l = 0; l + 1 < c->level_ptr.size(); ++l)
    std::sort(c->level_rows.begin() + c->level_ptr[l], c->level_rows.begin() + c->level_ptr[l + 1]);
  // device-order copies
  std::vector<double> locs_rm((size_t)n * d);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < d; ++k) locs_rm[(size_t)dp[i] * d + k] = locs[i + (size_t)k * n];
  std::vector<int> nn_dev((size_t)n * b);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < b; ++j) {
      int a = nn[(size_t)i * b + j];
      nn_dev[(size_t)dp[i] * b + j] = a < 0 ? -1 : dp[a];
    }
  const size_t NS = (size_t)n;
  std::vector<int> lm_dev(n_obs), slot_dpos(NS);
  for (int o = 0; o < n_obs; ++o) lm_dev[o] = dp[lm0[o]];
  for (size_t x = 0; x < NS; ++x) slot_dpos[x] = dp[L.compact_loc[x]];

  if ((rc = set_device(c))) { delete c; return rc; }
#define CK(x)                                                     \
  do {                                                            \
    hipError_t e_ = (x);                                          \
    if (e_ != hipSuccess) {                                       \
      int r_ = fail_hip(nullptr, e_, #x);                         \
      nngp_ctx_destroy(c);                                        \
      return r_;                                                  \
    }                                                             \
  } while (0)
  const int C = n_chains;
  CK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
  CK(dalloc(&c->locs_d, (size_t)n * d));
  CK(dalloc(&c->sc_d, (size_t)n * c->ds));
  CK(dalloc(&c->nn_d, (size_t)n * b));
  for (int k = 0; k < C; ++k) {
    ChainState& s = c->ch[k];
    CK(dalloc(&s.linv_d[0], (size_t)n * b));
    CK(dalloc(&s.linv_d[1], (size_t)n * b));
    CK(dalloc(&s.field_d, n));
    CK(dalloc(&s.field_prop_d, n));
    CK(dalloc(&s.mu_d, n_obs));
    CK(dalloc(&s.b1_d, n));
  }
  CK(dalloc(&c->linv_cur_d, C));
  CK(dalloc(&c->b1_tab_d, C));
  CK(hipHostMalloc((void**)&c->linv_cur_h, sizeof(double*) * C, hipHostMallocDefault));
  for (int k = 0; k < C; ++k) c->linv_cur_h[k] = c->ch[k].linv_d[0];
  CK(dalloc(&c->sinfo_d, NS));
  CK(dalloc(&c->compact_loc_d, NS));
  CK(dalloc(&c->dr_d, NS * C));
  CK(dalloc(&c->slot_dpos_d, NS));
  CK(dalloc(&c->dpos_d, n));
  CK(dalloc(&c->perm_d, n));
  CK(hipHostMalloc((void**)&c->stage_h, sizeof(double) * n, hipHostMallocDefault));
  CK(dalloc(&c->loc_rank_d, n));
  if (c->engine == 0) {
    CK(dalloc(&c->chunk_first_d, L.chunk_first.size()));
    CK(dalloc(&c->pairs_d, (n + 1) / 2));
    CK(dalloc(&c->zbuf_d, (size_t)2 * n * C));
    CK(dalloc(&c->ent_pk_d, (size_t)L.n_entries));
    CK(dalloc(&c->ent_pos_d, (size_t)L.n_entries));
    CK(dalloc(&c->start_mask_d, L.start_mask.size()));
    CK(dalloc(&c->ent_src_d, (size_t)L.n_entries));
    CK(dalloc(&c->ent_val_d, (size_t)L.n_entries * C));
  } else {
    const TileLayout& TL = c->tl;
    const size_t nb = TL.batch.size(), ncell = TL.cell_pk.size(), ng = TL.gsrc.size();
    CK(dalloc(&c->tb_d, nb));
    CK(dalloc(&c->tb_ptr_d, TL.batch_ptr.size()));
    CK(dalloc(&c->cell_pk_d, ncell));
    CK(dalloc(&c->cell_src_d, ncell));
    CK(dalloc(&c->cell_val_d, ncell * C));
    CK(dalloc(&c->gcell_d, ng));
    CK(dalloc(&c->gsrc_d, ng));
    CK(dalloc(&c->gval_d, ng * C));
    CK(dalloc(&c->gptr_d, TL.gptr.size()));
    CK(dalloc(&c->gslot_d, TL.gslot.size()));
    CK(dalloc(&c->gslot_ptr_d, TL.gslot_ptr.size()));
    CK(upload(c->gslot_d, TL.gslot.data(), TL.gslot.size(), c->st));
    CK(upload(c->gslot_ptr_d, TL.gslot_ptr.data(), TL.gslot_ptr.size(), c->st));
    if (TL.split) {
      CK(dalloc(&c->bsplit_d, TL.batch_split.size()));
      CK(upload(c->bsplit_d, TL.batch_split.data(), TL.batch_split.size(), c->st));
    }
    CK(dalloc(&c->nb_ptr_d, TL.nb_ptr.size()));
    CK(dalloc(&c->nb_d, TL.nb.size()));
    CK(dalloc(&c->erow_ptr_d, TL.erow_ptr.size()));
    CK(dalloc(&c->erow_d, TL.erow.size()));
    CK(shared_alloc(&c->dwx_d, (size_t)n * C * 2, c->tG > 1));
    if (c->rglobal) CK(dalloc(&c->rg_d, TL.erow.size() * C));
    CK(dalloc(&c->ctl_d, 4));
    CK(hipHostMalloc((void**)&c->tmo_h, sizeof(unsigned), hipHostMallocDefault));
    *c->tmo_h = 0;
    if (const char* e = std::getenv("NNGP_TILE_INJECT_TIMEOUT")) c->inject_tmo = std::atoi(e);
    // device batch record {off, R | nthr << 16, nslots, slot0}
    std::vector<int4> tb(nb);
    for (size_t q = 0; q < nb; ++q) {
      const TileBatch& B = TL.batch[q];
      tb[q] = make_int4(B.off, B.R | (B.nthr << 16), B.nslots, B.slot0);
    }
    CK(hipMemcpy(c->tb_d, tb.data(), sizeof(int4) * nb, hipMemcpyHostToDevice));
    CK(upload(c->tb_ptr_d, TL.batch_ptr.data(), TL.batch_ptr.size(), c->st));
    {
      // device encoding (tiles.hip tile_lr): the local-row field XOR its
      // padding value, so padding -- and an out-of-range buffer load -- is 0
      std::vector<uint32_t> pk(TL.cell_pk);
      for (uint32_t& v : pk) v ^= kTilePadRow;
      CK(hipMemcpy(c->cell_pk_d, pk.data(), sizeof(uint32_t) * ncell, hipMemcpyHostToDevice));
    }
    CK(upload(c->cell_src_d, TL.cell_src.data(), ncell, c->st));
    CK(hipMemsetAsync(c->cell_val_d, 0, sizeof(double) * std::max<size_t>(1, ncell * C), c->st));
    CK(upload(c->gcell_d, reinterpret_cast<const int2*>(TL.gcell.data()), ng, c->st));
    CK(upload(c->gsrc_d, TL.gsrc.data(), ng, c->st));
    CK(hipMemsetAsync(c->gval_d, 0, sizeof(double) * std::max<size_t>(1, ng * C), c->st));
    CK(upload(c->gptr_d, TL.gptr.data(), TL.gptr.size(), c->st));
    {
      const std::vector<int4> ro = tile_refresh_order(TL.batch_ptr, TL.gptr, TL.batch, TL.NT, TL.T, TL.K, c->rorder_len);
      CK(dalloc(&c->rorder_d, ro.size()));
      CK(upload(c->rorder_d, ro.data(), ro.size(), c->st));
    }
    CK(upload(c->nb_ptr_d, TL.nb_ptr.data(), TL.nb_ptr.size(), c->st));
    CK(upload(c->nb_d, TL.nb.data(), TL.nb.size(), c->st));
    CK(upload(c->erow_ptr_d, TL.erow_ptr.data(), TL.erow_ptr.size(), c->st));
    CK(upload(c->erow_d, TL.erow.data(), TL.erow.size(), c->st));
    CK(hipMemsetAsync(c->dwx_d, 0, sizeof(double) * (size_t)n * C * 2, c->st));
    CK(hipMemsetAsync(c->ctl_d, 0, sizeof(unsigned) * 4, c->st));
    if (c->tG > 1) {
      CK(dalloc(&c->rmask_d, TL.rmask.size()));
      CK(upload(c->rmask_d, TL.rmask.data(), TL.rmask.size(), c->st));
      // the halo of this rank per peer: its slots with a reader on that peer
      std::vector<int> halo;
      for (int h = 0; h < kTileRanksMax; ++h) {
        c->halo_ptr[h] = (int)halo.size();
        if (h < c->tG && h != c->trank)
          for (int x = TL.rank_slot0[c->trank]; x < TL.rank_slot0[c->trank + 1]; ++x)
            if ((TL.rmask[x] >> h) & 1u) halo.push_back(x);
      }
      c->halo_ptr[kTileRanksMax] = (int)halo.size();
      CK(dalloc(&c->halo_d, halo.size()));
      CK(upload(c->halo_d, halo.data(), halo.size(), c->st));
      CK(hipStreamSynchronize(c->st));
    }
    if (c->tG > 0) {
      CK(dalloc(&c->tdev_d, kTileRanksMax));
      CK(shared_alloc(&c->xflag_d, kTileRanksMax, c->tG > 1));
      CK(hipMemsetAsync(c->xflag_d, 0, sizeof(unsigned) * kTileRanksMax, c->st));
    }
    if (const char* pr = std::getenv("NNGP_PROBE"))
      if ((std::atoi(pr) == 9 || std::atoi(pr) == 2) && (C == 1 || C == 3)) {
        c->tprobe = std::atoi(pr) == 9 ? 1 : 2;
        c->tdbg_n = (size_t)TL.T * (c->tprobe == 1 ? 8 : 512 * 16);  // tiles.hip kTimelinePhases x kTimelineSlots
        if (const char* v = std::getenv("NNGP_TILE_VARIANT")) c->tvariant = std::atoi(v);
        CK(dalloc(&c->tdbg_d, c->tdbg_n));
        CK(hipMemsetAsync(c->tdbg_d, 0, sizeof(unsigned long long) * c->tdbg_n, c->st));
      }
  }
  CK(shared_alloc(&c->w_slot_d, NS * C, c->tG > 1));
  CK(dalloc(&c->r_d, (size_t)n * C));
  CK(dalloc(&c->level_rows_d, n));
  CK(dalloc(&c->level_ptr_d, c->level_ptr.size()));
  CK(upload(c->level_ptr_d, c->level_ptr.data(), c->level_ptr.size(), c->st));
  {
    // triangular-solve plan: runs of levels with <= kSmallLevel rows go to one
    // workgroup (a barrier per level; one CU streams ~10 B/cycle, so only
    // small levels are cheaper there than behind a launch), larger levels get
    // a launch each
    // (NNGP_TRI=level: one launch per level, the reference plan of the tests;
    // NNGP_TRI=levels: this plan; default: the sync-free one-launch solve,
    // tri_dag_kernel)
    const char* e = std::getenv("NNGP_TRI");
    const bool per_level = e && std::string(e) == "level";
    c->tri_dag = !per_level && !(e && std::string(e) == "levels");
    const char* er = std::getenv("NNGP_TRI_RESCUE");
    c->tri_rescue = er && std::string(er) == "1";
    const char* eo = std::getenv("NNGP_TRI_OVERSUB");
    c->tri_oversub = eo ? std::max(1, std::min(16, std::atoi(eo))) : 1;
    CK(dalloc(&c->tri_tmo_d, 6));
    CK(hipMemset(c->tri_tmo_d, 0, 6 * sizeof(unsigned)));
    CK(hipHostMalloc((void**)&c->tri_tmo_h, sizeof(unsigned), hipHostMallocDefault));
    *c->tri_tmo_h = 0;
    const int L = (int)c->level_ptr.size() - 1;
    for (int lv = 0; lv < L;) {
      const int sz = c->level_ptr[lv + 1] - c->level_ptr[lv];
      constexpr int kSmallLevel = 128;
      if (per_level || sz > kSmallLevel) {
        c->tri_seg.insert(c->tri_seg.end(), {lv, lv + 1, 0});
        ++lv;
        continue;
      }
      int lv1 = lv;
      while (lv1 < L && c->level_ptr[lv1 + 1] - c->level_ptr[lv1] <= kSmallLevel) ++lv1;
      c->tri_seg.insert(c->tri_seg.end(), {lv, lv1, 1});
      lv = lv1;
    }
  }
  CK(dalloc(&c->obs_ptr_d, (size_t)n + 1));
  CK(dalloc(&c->obs_idx_d, n_obs));
  CK(dalloc(&c->lm_d, n_obs));
  CK(dalloc(&c->y_d, n_obs));
  CK(dalloc(&c->tmp_d, (size_t)n * C));   // scratch vectors, chain-strided for batched solves
  CK(dalloc(&c->tmp2_d, (size_t)n * C));
  CK(dalloc(&c->partials_d, 4 * kRedBlocks * kRowJobsMax));
  // the factors' failure flags sit right after the reductions' results, so
  // one copy brings both to the host (kResFailOff doubles in)
  CK(dalloc(&c->res_d, kResBytes / sizeof(double)));
  c->fail_d = reinterpret_cast<int*>(c->res_d + kResFailOff);
  CK(dalloc(&c->scal_d, C));
  CK(hipHostMalloc((void**)&c->scal_h, sizeof(SweepScalars) * C, hipHostMallocDefault));
  std::memset(c->scal_h, 0, sizeof(SweepScalars) * C);
  CK(hipHostMalloc((void**)&c->scal_ring_h, sizeof(SweepScalars) * C * nngp_ctx::kScalRing, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&c->res_h, kResBytes, hipHostMallocDefault));
  c->fail_h = reinterpret_cast<int*>(c->res_h + kResFailOff);
  CK(upload(c->locs_d, locs_rm.data(), locs_rm.size(), c->st));
  CK(upload(c->nn_d, nn_dev.data(), nn_dev.size(), c->st));
  {
    std::vector<int2> sd(NS);
    for (size_t x = 0; x < NS; ++x) {
      const int i = L.compact_loc[x];
      sd[x].x = obs_cnt[i + 1] - obs_cnt[i];
      sd[x].y = c->engine == 1 ? c->tl.slot_f0[x] : (L.slot_f0[x] | (L.collen[x] << 16));
    }
    CK(hipMemcpy(c->sinfo_d, sd.data(), sizeof(int2) * sd.size(), hipMemcpyHostToDevice));
    std::vector<double> ys(NS, 0.0);
    for (size_t x = 0; x < NS; ++x) {
      const int i = L.compact_loc[x];
      for (int p = obs_cnt[i]; p < obs_cnt[i + 1]; ++p) ys[x] += observed_field[obs_idx[p]];
    }
    CK(dalloc(&c->ysum_d, NS));
    CK(hipMemcpy(c->ysum_d, ys.data(), sizeof(double) * NS, hipMemcpyHostToDevice));
    CK(hipMemcpy(c->compact_loc_d, L.compact_loc.data(), sizeof(int) * NS, hipMemcpyHostToDevice));
  }
  CK(hipMemsetAsync(c->dr_d, 0, sizeof(double2) * NS * C, c->st));
  CK(hipMemsetAsync(c->w_slot_d, 0, sizeof(double) * NS * C, c->st));
  CK(upload(c->slot_dpos_d, slot_dpos.data(), NS, c->st));
  CK(upload(c->dpos_d, dp.data(), n, c->st));
  {
    // normals: compact rank of each location; pair p = (2p, 2p+1) is generated
    // by the colour of 2p, pairs ordered by the compact rank of 2p
    c->loc_rank.assign(n, 0);
    for (int x = 0; x < n; ++x) c->loc_rank[L.compact_loc[x]] = x;
    CK(upload(c->loc_rank_d, c->loc_rank.data(), n, c->st));
    if (c->engine == 0) {
      std::vector<int> pairs;
      pairs.reserve((n + 1) / 2);
      c->pair_ptr.assign(L.K + 1, 0);
      for (int col = 0; col < L.K; ++col) {
        for (int x = L.color_loc_ptr[col]; x < L.color_loc_ptr[col + 1]; ++x)
          if ((L.compact_loc[x] & 1) == 0) pairs.push_back(L.compact_loc[x] >> 1);
        c->pair_ptr[col + 1] = (int)pairs.size();
      }
      CK(upload(c->chunk_first_d, L.chunk_first.data(), L.chunk_first.size(), c->st));
      CK(upload(c->pairs_d, pairs.data(), pairs.size(), c->st));
    }
    CK(hipStreamSynchronize(c->st));
  }
  if (c->engine == 0) {
    CK(upload(c->ent_pk_d, L.ent_pk.data(), (size_t)L.n_entries, c->st));
    CK(upload(c->ent_pos_d, L.ent_pos.data(), (size_t)L.n_entries, c->st));
    CK(upload(c->start_mask_d, L.start_mask.data(), L.start_mask.size(), c->st));
    CK(upload(c->ent_src_d, L.ent_src.data(), (size_t)L.n_entries, c->st));
    CK(hipMemsetAsync(c->ent_val_d, 0, sizeof(double) * std::max<long long>(1, L.n_entries * C), c->st));
  }
  if (c->shard && c->engine == 0) {
    const ShardPlan& SP = c->sp;
    const size_t ng = SP.grow.size();
    CK(dalloc(&c->sg_row_d, ng));
    CK(dalloc(&c->sg_recv_d, ng));
    CK(dalloc(&c->sg_src_d, ng));
    CK(dalloc(&c->sg_val_d, ng * C));
    CK(dalloc(&c->xbuf_d, (size_t)SP.xoff[SP.K] * C));
    CK(dalloc(&c->sp_pairs_d, SP.pairs.size()));
    CK(upload(c->sg_row_d, SP.grow.data(), ng, c->st));
    CK(upload(c->sg_recv_d, SP.grecv.data(), ng, c->st));
    CK(upload(c->sg_src_d, SP.gsrc.data(), ng, c->st));
    CK(hipMemsetAsync(c->sg_val_d, 0, sizeof(double) * std::max<size_t>(1, ng * C), c->st));
    CK(hipMemsetAsync(c->xbuf_d, 0, sizeof(double2) * std::max<size_t>(1, (size_t)SP.xoff[SP.K] * C), c->st));
    CK(upload(c->sp_pairs_d, SP.pairs.data(), SP.pairs.size(), c->st));
  }
  CK(hipMemcpyAsync(c->linv_cur_d, c->linv_cur_h, sizeof(double*) * C, hipMemcpyHostToDevice, c->st));
  {
    std::vector<const double*> b1p(C);
    for (int k = 0; k < C; ++k) b1p[k] = c->ch[k].b1_d;
    CK(upload(c->b1_tab_d, b1p.data(), (size_t)C, c->st));
  }
  CK(upload(c->level_rows_d, c->level_rows.data(), n, c->st));
  CK(upload(c->obs_ptr_d, obs_cnt.data(), (size_t)n + 1, c->st));
  CK(upload(c->obs_idx_d, obs_idx.data(), n_obs, c->st));
  CK(upload(c->lm_d, lm_dev.data(), n_obs, c->st));
  CK(upload(c->y_d, observed_field, n_obs, c->st));
  if (const char* pr = std::getenv("NNGP_PROBE"))
    if (std::atoi(pr) == 9 && c->engine == 0) {
      CK(dalloc(&c->dbg_d, (size_t)L.nchunks * 8));
      CK(hipMemset(c->dbg_d, 0, sizeof(unsigned long long) * L.nchunks * 8));
    }
  if (c->tG > 0) {
    const TileDev D = tile_dev(c);
    CK(hipMemcpy(c->tdev_d, &D, sizeof(TileDev), hipMemcpyHostToDevice));
  }
  CK(hipStreamSynchronize(c->st));
#undef CK
  *out = c;
  return NNGP_OK;
}

int nngp_ctx_create(const double* locs, int n, int d, const int* NNarray, int b, const int* coloring,
                    const int* locs_match, const double* observed_field, int n_obs, int n_chains,
                    int device, nngp_ctx** out) {
  return ctx_create(locs, n, d, NNarray, b, coloring, locs_match, observed_field, n_obs, n_chains, device, 0, 0,
                    out);
}

int nngp_ctx_create_shard(const double* locs, int n, int d, const int* NNarray, int b, const int* coloring,
                          const int* locs_match, const double* observed_field, int n_obs, int n_chains,
                          int device, int n_ranks, int rank, nngp_ctx** out) {
  if (n_ranks < 1 || n_ranks > kMaxRanks || rank < 0 || rank >= n_ranks) {
    if (out) *out = nullptr;
    return fail_msg(nullptr, NNGP_ERR_ARG, "ctx_create_shard: need 1 <= n_ranks <= 64 and 0 <= rank < n_ranks");
  }
  return ctx_create(locs, n, d, NNarray, b, coloring, locs_match, observed_field, n_obs, n_chains, device,
                    n_ranks, rank, out);
}

int nngp_set_chain(nngp_ctx* c, int chain) {
  if (!c) return NNGP_ERR_ARG;
  if (chain < 0 || chain >= c->C) return fail_msg(c, NNGP_ERR_ARG, "set_chain: chain out of range");
  c->cur = chain;
  return NNGP_OK;
}

const char* nngp_ctx_engine_note(const nngp_ctx* c) { return c ? c->engine_note.c_str() : ""; }

int nngp_ctx_info(const nngp_ctx* c, nngp_info* info) {
  if (!c || !info) return NNGP_ERR_ARG;
  info->n = c->n; info->b = c->b; info->d = c->d; info->n_obs = c->n_obs;
  info->n_colors = c->lay.K;
  info->n_levels = (int)c->level_ptr.size() - 1;
  info->nnz = c->lay.nnz;
  info->n_entries = c->lay.n_entries;
  info->max_collen = c->lay.max_collen;
  info->device = c->device;
  info->n_chains = c->C;
  info->lanes_per_chain = c->lay.LW;
  info->n_chunks = c->lay.nchunks;
  info->sweep_engine = c->engine;
  info->n_tiles = c->engine == 1 ? c->tl.T : 0;
  info->tile_rows_max = c->engine == 1 ? c->tl.max_rows : 0;
  info->n_ghost_cells = c->engine == 1 ? (long long)c->tl.gsrc.size() : (long long)c->sp.grow.size();
  if (c->tG > 0) {
    const TileLayout& TL = c->tl;
    const int r = c->trank;
    info->n_ranks = c->tG;
    info->rank = r;
    info->shard_owned = TL.rank_slot0[r + 1] - TL.rank_slot0[r];
    info->shard_needed_rows = TL.erow_ptr[(size_t)(r + 1) * c->tTl] - TL.erow_ptr[(size_t)r * c->tTl];
    long long x = 0;
    for (uint32_t m : TL.rmask) x += m != 0;
    info->shard_exchange_slots = x;
  } else {
    info->n_ranks = c->shard ? c->sp.G : 0;
    info->rank = c->shard ? c->sp.rank : 0;
    info->shard_owned = c->shard ? c->sp.owned : 0;
    info->shard_needed_rows = c->shard ? c->sp.needed_rows : 0;
    info->shard_exchange_slots = c->shard ? c->sp.xoff[c->sp.K] : 0;
  }
  info->tile_ghost_pass = c->engine == 1 ? c->tl.NTK * tile_gmax(c->tl.NTK) : 0;
  info->tile_ghost_cells_max = 0;
  info->tile_r_global = c->rglobal ? 1 : 0;
  info->tile_chain_split = c->tcs ? 1 : 0;
  info->tile_resident_per_cu = c->engine == 1 ? c->tresident : 0;
  info->engine_fallback = c->engine_fallback;
  info->tile_exchange_wave = c->txw ? 1 : 0;
  info->device_cus = c->cus;
  info->tile_rows_needed = c->tile_rows_needed;
  info->device_lds = c->lds_max;
  if (c->engine == 1)
    for (size_t i = 0; i + 1 < c->tl.gptr.size(); ++i)
      info->tile_ghost_cells_max = std::max(info->tile_ghost_cells_max, c->tl.gptr[i + 1] - c->tl.gptr[i]);
  return NNGP_OK;
}

// ---------------------------------------------------------------- factor
static int covfun_family(int covfun, int d, const double* cp, int ncp, double* var, double* nug,
                         double* nu, std::string& err) {
  int need = 0, fam = 0;
  switch (covfun) {
    case NNGP_EXPONENTIAL_ISOTROPIC: case NNGP_EXPONENTIAL_SPHERE: need = 3; fam = 0; break;
    case NNGP_MATERN15_ISOTROPIC: need = 3; fam = 1; break;
    case NNGP_EXPONENTIAL_SCALEDIM: need = d + 2; fam = 0; break;
    case NNGP_EXPONENTIAL_SPACETIME: need = 4; fam = 0; break;
    case NNGP_MATERN_ISOTROPIC: case NNGP_MATERN_SPHERE: need = 4; fam = 2; break;
    case NNGP_MATERN_SCALEDIM: need = d + 3; fam = 2; break;
    case NNGP_MATERN_SPACETIME: need = 5; fam = 2; break;
    default: err = "unknown covfun"; return -1;
  }
  if (ncp != need) { err = "covparms has the wrong length for this covfun"; return -1; }
  if ((covfun == NNGP_EXPONENTIAL_SPHERE || covfun == NNGP_MATERN_SPHERE) && d != 2) { err = "sphere covfuns need d == 2 (lon, lat)"; return -1; }
  if ((covfun == NNGP_EXPONENTIAL_SPACETIME || covfun == NNGP_MATERN_SPACETIME) && d < 2) { err = "spacetime covfuns need d >= 2"; return -1; }
  for (int k = 0; k < ncp; ++k)
    if (!std::isfinite(cp[k])) { err = "non-finite covparms"; return -1; }
  *var = cp[0];
  *nug = cp[ncp - 1];
  *nu = 0.0;
  if (fam == 2) *nu = cp[ncp - 2];
  if (!(*var > 0)) { err = "variance must be > 0"; return -1; }
  for (int k = 1; k < ncp - 1 - (fam == 2 ? 1 : 0); ++k)
    if (!(cp[k] > 0)) { err = "ranges must be > 0"; return -1; }
  if (fam == 2 && !(*nu > 0)) { err = "smoothness must be > 0"; return -1; }
  return fam;
}

// the factor of chain k into slot `which`; its failure row (or INT_MAX)
// lands in fail_d[k] (the caller copies the flags once for all chains)
static int factor_enqueue(nngp_ctx* c, int k, int which, int covfun, const double* cp, int ncp) {
  double var, nug, nu;
  std::string err;
  int fam = covfun_family(covfun, c->d, cp, ncp, &var, &nug, &nu, err);
  if (fam < 0) return fail_msg(c, NNGP_ERR_ARG, err);
  ChainState& S = c->ch[k];
  const bool sphere = covfun == NNGP_EXPONENTIAL_SPHERE || covfun == NNGP_MATERN_SPHERE;
  if (sphere && c->ds < 3) {
    // sphere on d == 2: scaled coordinates are 3-D; grow the buffer once
    { int ss_ = sync_stream(c); if (ss_) return ss_; }
    hipFree(c->sc_d);
    c->sc_d = nullptr;
    HIPCHK(c, dalloc(&c->sc_d, (size_t)c->n * 4));
    c->ds = 4;  // capacity marker
  }
  const int use_ds = sphere ? 3 : (c->d <= 2 ? 2 : (c->d == 3 ? 3 : 4));
  // the scaled coordinates are shared scratch: the chains' factors run one
  // after another in stream order
  HIPCHK(c, launch_scale_coords(c->st, covfun, cp, ncp, c->locs_d, c->n, c->d, c->sc_d, use_ds));
  HIPCHK(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->fail_d + k), INT_MAX, 1, c->st));
  S.lgen[which] = ++c->gen;
  HIPCHK(c, launch_factor(c->st, fam, var, nug, nu, c->sc_d, use_ds, c->nn_d, c->n, c->b, S.linv_d[which],
                          c->fail_d + k));
  return NNGP_OK;
}

// the factors of the chains in mask into slot `which` (covparms: C x ncp,
// row k for chain k): one scaled-coordinate launch and one factor launch for
// all of them (launch_factor_jobs; rows bitwise those of factor_enqueue per
// chain); NNGP_FACTOR_JOBS=0, the sphere covariances and chains of different
// Matern smoothness go chain by chain
static int factor_enqueue_chains(nngp_ctx* c, int mask, int which, int covfun, const double* covparms, int ncp) {
  const char* fj = std::getenv("NNGP_FACTOR_JOBS");  // per call (A/B in one process)
  const bool off = fj && fj[0] == '0';
  const bool sphere = covfun == NNGP_EXPONENTIAL_SPHERE || covfun == NNGP_MATERN_SPHERE;
  int cnt = 0;
  for (int k = 0; k < c->C; ++k) cnt += (mask >> k) & 1;
  FactorJobs J;
  int fam0 = -1;
  double nu0 = 0.0;
  bool same = true;
  for (int k = 0; k < c->C && cnt >= 2 && !off && !sphere; ++k) {
    if (!((mask >> k) & 1)) continue;
    const double* cp = covparms + (size_t)k * ncp;
    double var, nug, nu;
    std::string err;
    const int fam = covfun_family(covfun, c->d, cp, ncp, &var, &nug, &nu, err);
    if (fam < 0) return fail_msg(c, NNGP_ERR_ARG, err);
    if (J.n_jobs == 0) {
      fam0 = fam;
      nu0 = nu;
    } else if (fam != fam0 || !(nu == nu0)) {
      same = false;
    }
    const int j = J.n_jobs++;
    for (int q = 0; q < 8; ++q) J.sa[j].c[q] = q < ncp ? cp[q] : 0.0;
    J.sa[j].covfun = covfun;
    J.var[j] = var;
    J.nugget[j] = nug;
    J.linv[j] = c->ch[k].linv_d[which];
    J.fail[j] = c->fail_d + k;
  }
  if (cnt < 2 || off || sphere || !same) {
    for (int k = 0; k < c->C; ++k)
      if ((mask >> k) & 1) {
        int rc = factor_enqueue(c, k, which, covfun, covparms + (size_t)k * ncp, ncp);
        if (rc) return rc;
      }
    return NNGP_OK;
  }
  const int use_ds = c->d <= 2 ? 2 : (c->d == 3 ? 3 : 4);
  const size_t need = (size_t)c->n * use_ds * J.n_jobs;
  if (need > c->scm_cap) {
    { int ss_ = sync_stream(c); if (ss_) return ss_; }
    if (c->scm_d) hipFree(c->scm_d);
    c->scm_d = nullptr;
    c->scm_cap = 0;
    HIPCHK(c, dalloc(&c->scm_d, need));
    c->scm_cap = need;
  }
  for (int j = 0; j < J.n_jobs; ++j) J.sc[j] = c->scm_d + (size_t)j * c->n * use_ds;
  for (int k = 0; k < c->C; ++k)
    if ((mask >> k) & 1) c->ch[k].lgen[which] = ++c->gen;
  HIPCHK(c, launch_factor_jobs(c->st, fam0, nu0, J, c->locs_d, c->n, c->d, use_ds, c->nn_d, c->b));
  return NNGP_OK;
}

// after factor_enqueue of the chains in mask and a host sync that followed
// the copy of the flags into fail_h: per-chain outcomes
static int factor_outcomes(nngp_ctx* c, int which, int mask, int* status) {
  int rc = NNGP_OK;
  for (int k = 0; k < c->C; ++k) {
    if (!((mask >> k) & 1)) continue;
    ChainState& S = c->ch[k];
    if (c->fail_h[k] != INT_MAX) {
      S.have_factor[which] = false;
      char buf[160];
      std::snprintf(buf, sizeof buf, "vecchia factor: local covariance of row %d is not positive definite",
                    c->fail_h[k]);
      fail_msg(c, NNGP_ERR_CHOL, buf);
      if (status) status[k] = NNGP_ERR_CHOL;
      rc = NNGP_ERR_CHOL;
      continue;
    }
    S.have_factor[which] = true;
    if (status) status[k] = NNGP_OK;
    if (which == 0) {
      int r2 = refresh_sweep_values(c, k);
      if (r2) return r2;
    }
  }
  return rc;
}

// after factor_enqueue of the chains in mask: one copy of the flags, one sync
static int factor_collect(nngp_ctx* c, int which, int mask, int* status) {
  HIPCHK(c, hipMemcpyAsync(c->fail_h, c->fail_d, sizeof(int) * c->C, hipMemcpyDeviceToHost, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  return factor_outcomes(c, which, mask, status);
}

int nngp_factor(nngp_ctx* c, int which, int covfun, const double* cp, int ncp) {
  if (!c || (which != 0 && which != 1) || !cp) return fail_msg(c, NNGP_ERR_ARG, "factor: bad args");
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = factor_enqueue(c, c->cur, which, covfun, cp, ncp))) return rc;
  return factor_collect(c, which, 1 << c->cur, nullptr);
}

int nngp_factor_chains(nngp_ctx* c, int which, int chain_mask, int covfun, const double* covparms, int ncp,
                       int* status) {
  if (!c || (which != 0 && which != 1) || !covparms || !status || chain_mask <= 0 || chain_mask >= (1 << c->C))
    return fail_msg(c, NNGP_ERR_ARG, "factor_chains: bad args");
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = factor_enqueue_chains(c, chain_mask, which, covfun, covparms, ncp))) return rc;
  rc = factor_collect(c, which, chain_mask, status);
  return rc == NNGP_ERR_CHOL ? NNGP_OK : rc;  // per-chain outcomes in status
}

int nngp_get_linv(nngp_ctx* c, int which, double* Linv) {
  if (!c || !Linv || (which != 0 && which != 1)) return NNGP_ERR_ARG;
  ChainState& S = c->ch[c->cur];
  if (!S.have_factor[which]) return fail_msg(c, NNGP_ERR_STATE, "get_linv: factor not computed");
  int rc;
  if ((rc = set_device(c))) return rc;
  std::vector<double> rm((size_t)c->n * c->b);
  HIPCHK(c, hipMemcpyAsync(rm.data(), S.linv_d[which], rm.size() * sizeof(double), hipMemcpyDeviceToHost, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  for (int i = 0; i < c->n; ++i)
    for (int j = 0; j < c->b; ++j) Linv[i + (size_t)j * c->n] = rm[(size_t)c->dpos[i] * c->b + j];
  return NNGP_OK;
}

int nngp_set_linv(nngp_ctx* c, int which, const double* Linv) {
  if (!c || !Linv || (which != 0 && which != 1)) return NNGP_ERR_ARG;
  int rc;
  if ((rc = set_device(c))) return rc;
  ChainState& S = c->ch[c->cur];
  std::vector<double> rm((size_t)c->n * c->b);
  for (int i = 0; i < c->n; ++i)
    for (int j = 0; j < c->b; ++j) rm[(size_t)c->dpos[i] * c->b + j] = Linv[i + (size_t)j * c->n];
  S.lgen[which] = ++c->gen;
  HIPCHK(c, hipMemcpyAsync(S.linv_d[which], rm.data(), rm.size() * sizeof(double), hipMemcpyHostToDevice, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  S.have_factor[which] = true;
  if (which == 0) return refresh_sweep_values(c, c->cur);
  return NNGP_OK;
}

int nngp_accept_factor(nngp_ctx* c) {
  if (!c) return NNGP_ERR_ARG;
  ChainState& S = c->ch[c->cur];
  if (!S.have_factor[1]) return fail_msg(c, NNGP_ERR_STATE, "accept_factor: no proposal factor");
  int rc;
  if ((rc = set_device(c))) return rc;
  std::swap(S.linv_d[0], S.linv_d[1]);
  std::swap(S.have_factor[0], S.have_factor[1]);
  std::swap(S.lgen[0], S.lgen[1]);
  // captured sweep graphs read the current factor through linv_cur_d: they stay valid
  return refresh_sweep_values(c, c->cur);
}

int nngp_get_precision_diag(nngp_ctx* c, double* D) {
  if (!c || !D) return NNGP_ERR_ARG;
  if (!c->ch[c->cur].have_factor[0]) return fail_msg(c, NNGP_ERR_STATE, "precision_diag: no factor");
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = flush_sweep_values(c, 1 << c->cur))) return rc;
  std::vector<double2> dr((size_t)c->n * c->C);
  HIPCHK(c, hipMemcpyAsync(dr.data(), c->dr_d, dr.size() * sizeof(double2), hipMemcpyDeviceToHost, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  for (int x = 0; x < c->n; ++x) D[c->lay.compact_loc[x]] = dr[(size_t)x * c->C + c->cur].x;
  return NNGP_OK;
}

// ---------------------------------------------------------------- state
// field-sized host <-> device copies through the pinned stage, permuted
// between R order and device row order on the device
static int upload_field(nngp_ctx* c, const double* host, double* dev) {
  std::memcpy(c->stage_h, host, sizeof(double) * c->n);
  HIPCHK(c, hipMemcpyAsync(c->perm_d, c->stage_h, c->n * sizeof(double), hipMemcpyHostToDevice, c->st));
  HIPCHK(c, launch_permute_scatter(c->st, c->n, c->dpos_d, c->perm_d, dev));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  return NNGP_OK;
}

static int download_field(nngp_ctx* c, const double* dev, double* host) {
  HIPCHK(c, launch_permute_gather(c->st, c->n, c->dpos_d, dev, c->perm_d));
  HIPCHK(c, hipMemcpyAsync(c->stage_h, c->perm_d, c->n * sizeof(double), hipMemcpyDeviceToHost, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  std::memcpy(host, c->stage_h, sizeof(double) * c->n);
  return NNGP_OK;
}

int nngp_set_field(nngp_ctx* c, const double* field) {
  if (!c || !field) return NNGP_ERR_ARG;
  int rc;
  if ((rc = set_device(c))) return rc;
  c->stale_mask &= ~(1 << c->cur);  // the whole replica of this chain is rewritten
  ChainState& S = c->ch[c->cur];
  S.fgen = ++c->gen;
  if ((rc = upload_field(c, field, S.field_d))) return rc;
  S.have_field = true;
  return NNGP_OK;
}

int nngp_get_field(nngp_ctx* c, double* field) {
  if (!c || !field) return NNGP_ERR_ARG;
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  ChainState& S = c->ch[c->cur];
  if (!S.have_field) return fail_msg(c, NNGP_ERR_STATE, "get_field: no field");
  int rc;
  if ((rc = set_device(c))) return rc;
  return download_field(c, S.field_d, field);
}

// ---------------------------------------------------------------- records
int nngp_records_reserve(nngp_ctx* c, int n_rows) {
  if (!c || n_rows < 0) return NNGP_ERR_ARG;
  int rc;
  if ((rc = set_device(c))) return rc;
  ChainState& S = c->ch[c->cur];
  if (S.rec_host) {  // a reserve ends the binding of a host array
    S.rec_host = nullptr;
    HIPCHK(c, c->recs->drain());
  }
  if (n_rows == S.rec_rows && (S.rec_d || n_rows == 0)) return NNGP_OK;
  if (S.rec_d) {
    { int ss_ = sync_stream(c); if (ss_) return ss_; }
    hipFree(S.rec_d);
  }
  S.rec_d = nullptr;
  S.rec_rows = 0;
  if (n_rows == 0) return NNGP_OK;
  if (dalloc(&S.rec_d, (size_t)n_rows * c->n) != hipSuccess) {
    hipGetLastError();
    S.rec_d = nullptr;
    return fail_msg(c, NNGP_ERR_NOMEM, "records_reserve: device allocation failed");
  }
  S.rec_rows = n_rows;
  return NNGP_OK;
}

int nngp_record_field(nngp_ctx* c, int row) {
  if (!c) return NNGP_ERR_ARG;
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  ChainState& S = c->ch[c->cur];
  if (!S.rec_d || row < 0 || row >= S.rec_rows) return fail_msg(c, NNGP_ERR_ARG, "record_field: row out of the reserved records");
  if (!S.have_field) return fail_msg(c, NNGP_ERR_STATE, "record_field: no field");
  int rc;
  if ((rc = set_device(c))) return rc;
  // device row order -> location order, stays on the device (no host sync)
  HIPCHK(c, launch_permute_gather(c->st, c->n, c->dpos_d, S.field_d, S.rec_d + (size_t)row * c->n));
  if (S.rec_host) {  // and on to the bound host array behind the stream (rec_stream.h)
    hipEvent_t ev = nullptr;
    HIPCHK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipError_t e = hipEventRecord(ev, c->st);
    if (e != hipSuccess) hipEventDestroy(ev);
    HIPCHK(c, e);
    c->recs->push({ev, S.rec_d + (size_t)row * c->n, S.rec_host + (size_t)row * c->n, (size_t)c->n});
    S.rec_pushed[row] = 1;
  }
  return NNGP_OK;
}

int nngp_records_stream(nngp_ctx* c, double* host, int n_rows) {
  if (!c) return NNGP_ERR_ARG;
  ChainState& S = c->ch[c->cur];
  int rc;
  if ((rc = set_device(c))) return rc;
  // a call that fails leaves an existing binding as it was
  if (host && (!S.rec_d || n_rows != S.rec_rows))
    return fail_msg(c, NNGP_ERR_ARG, "records_stream: the host array must have the reserved rows (records_reserve first)");
  if (host && !c->recs) c->recs = new (std::nothrow) RecordStreamer();
  if (host && (!c->recs || !c->recs->start(c->device))) {
    hipGetLastError();
    return fail_msg(c, NNGP_ERR_NOMEM, "records_stream: staging buffers or worker could not be set up");
  }
  if (S.rec_host) {
    S.rec_host = nullptr;
    HIPCHK(c, c->recs->drain());
  }
  if (!host) return NNGP_OK;
  // rows recorded before the binding are not streamed: get_records copies them
  S.rec_pushed.assign((size_t)S.rec_rows, 0);
  S.rec_host = host;
  return NNGP_OK;
}

int nngp_get_records(nngp_ctx* c, int row0, int n_rows, double* out) {
  if (!c || !out || n_rows < 0) return NNGP_ERR_ARG;
  ChainState& S = c->ch[c->cur];
  if (row0 < 0 || row0 + n_rows > S.rec_rows) return fail_msg(c, NNGP_ERR_ARG, "get_records: rows out of the reserved records");
  if (n_rows == 0) return NNGP_OK;
  int rc;
  if ((rc = set_device(c))) return rc;
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  if (S.rec_host && out == S.rec_host + (size_t)row0 * c->n) {
    // the bound array: its rows were streamed as they were recorded; rows
    // never handed to the streamer (recorded before the binding, or never
    // recorded) are copied from the device as on the unbound path.  The call
    // ends the binding (nngp.h): later record_field calls stay on the device.
    S.rec_host = nullptr;
    HIPCHK(c, c->recs->drain());
    for (int r = row0; r < row0 + n_rows;) {
      if (S.rec_pushed[r]) { ++r; continue; }
      int e = r;
      while (e < row0 + n_rows && !S.rec_pushed[e]) ++e;
      HIPCHK(c, hipMemcpy(out + (size_t)(r - row0) * c->n, S.rec_d + (size_t)r * c->n, sizeof(double) * (size_t)(e - r) * c->n,
                          hipMemcpyDeviceToHost));
      r = e;
    }
    return NNGP_OK;
  }
  HIPCHK(c, hipMemcpy(out, S.rec_d + (size_t)row0 * c->n, sizeof(double) * (size_t)n_rows * c->n, hipMemcpyDeviceToHost));
  return NNGP_OK;
}

int nngp_set_mu(nngp_ctx* c, const double* mu, double beta0) {
  if (!c) return NNGP_ERR_ARG;
  int rc;
  if ((rc = set_device(c))) return rc;
  ChainState& S = c->ch[c->cur];
  if (mu) {
    // through pinned staging: the call returns before the copy runs (the
    // previous copy out of the stage is waited for first -- normally long done)
    if (!c->mu_stage_h) {
      HIPCHK(c, hipHostMalloc((void**)&c->mu_stage_h, sizeof(double) * c->n_obs, hipHostMallocDefault));
      HIPCHK(c, hipEventCreateWithFlags(&c->mu_stage_ev, hipEventDisableTiming));
    } else {
      HIPCHK(c, hipEventSynchronize(c->mu_stage_ev));
    }
    std::memcpy(c->mu_stage_h, mu, sizeof(double) * c->n_obs);
    HIPCHK(c, hipMemcpyAsync(S.mu_d, c->mu_stage_h, c->n_obs * sizeof(double), hipMemcpyHostToDevice, c->st));
    HIPCHK(c, hipEventRecord(c->mu_stage_ev, c->st));
  }
  S.mu_is_const = (mu == nullptr);
  S.mu_beta0 = beta0;
  S.res_stale = true;
  S.have_mu = true;
  return NNGP_OK;
}

// ---------------------------------------------------------------- loglik
static void rowstats_store(nngp_ctx* c, int k, int which, double beta0, const double* r) {
  ChainState& S = c->ch[k];
  ChainState::RowStats& e = S.rs[S.rs_next];
  S.rs_next ^= 1;
  e.lg = S.lgen[which];
  e.fg = S.fgen;
  e.shift = beta0;
  for (int q = 0; q < 4; ++q) e.r[q] = r[q];
}

int nngp_loglik(nngp_ctx* c, int which, double beta0, double log_scale, double* ll) {
  if (!c || !ll || (which != 0 && which != 1)) return NNGP_ERR_ARG;
  double b0[kMaxChains], ls[kMaxChains], out[kMaxChains];
  b0[c->cur] = beta0;
  ls[c->cur] = log_scale;
  int rc = nngp_loglik_chains(c, which, 1 << c->cur, b0, ls, out);
  if (!rc) *ll = out[c->cur];
  return rc;
}

// log-likelihood jobs (chain k, factor `which`) in ONE pass over the rows
// (NNarray read once): per job exactly the single-job arithmetic, so any
// grouping of jobs gives the same bits.  The factors' log-determinant and
// row-statistics caches are updated in job order.
struct LLJob {
  int k, which;
  double beta0, log_scale;
  double* out;
  bool cached = false;  // set at enqueue: the factor's log-determinant was cached (the pass skips the logs)
  double ld = 0.0;
};

static int loglik_jobs_enqueue(nngp_ctx* c, LLJob* jobs, int nj, bool copy = true) {
  if (nj < 1 || nj > kRowJobsMax) return fail_msg(c, NNGP_ERR_ARG, "loglik: too many jobs");
  for (int j = 0; j < nj; ++j) {
    const ChainState& S = c->ch[jobs[j].k];
    if (!S.have_factor[jobs[j].which] || !S.have_field)
      return fail_msg(c, NNGP_ERR_STATE, "loglik: need factor and field");
  }
  // passes of at most kPassJobs jobs: the row-statistics kernel's registers
  // grow with the jobs (3: 127 VGPRs, 4 waves per SIMD; 6: 227, 2 waves) and
  // two 3-job passes (2 x 225 us at n = 1e6, b = 16) beat one 6-job pass
  // (774 us).  Each job's arithmetic is the one-job kernel's in any grouping.
  constexpr int kPassJobs = 3;
  for (int j0 = 0; j0 < nj; j0 += kPassJobs) {
    RowJobs J;
    for (int j = j0; j < nj && j < j0 + kPassJobs; ++j) {
      ChainState& S = c->ch[jobs[j].k];
      const int which = jobs[j].which;
      J.linv[J.M] = S.linv_d[which];
      J.x[J.M] = S.field_d;
      J.shift[J.M] = jobs[j].beta0;
      J.out[J.M] = nullptr;
      J.res_slot[J.M] = j;
      J.mode[J.M] = 1;
      jobs[j].cached = false;
      for (const ChainState::LogDet& e : S.ld)
        if (e.lg == S.lgen[which]) {
          J.mode[J.M] = 2;
          jobs[j].cached = true;
          jobs[j].ld = e.v;
        }
      ++J.M;
    }
    const int nb = launch_row_stats_jobs(c->st, J, c->nn_d, c->n, c->b, c->partials_d);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, launch_reduce4_jobs(c->st, J, c->partials_d, nb, c->res_d));
  }
  if (copy) HIPCHK(c, hipMemcpyAsync(c->res_h, c->res_d, 4 * nj * sizeof(double), hipMemcpyDeviceToHost, c->st));
  return NNGP_OK;
}

// after the sync: the jobs' values and the caches (jobs of chains in `skip`
// -- a proposal factor that failed -- neither answer nor touch the caches)
static void loglik_jobs_finish(nngp_ctx* c, const LLJob* jobs, int nj, int skip = 0) {
  for (int j = 0; j < nj; ++j) {
    const int k = jobs[j].k, which = jobs[j].which;
    if ((skip >> k) & 1) {
      *jobs[j].out = std::nan("");
      continue;
    }
    ChainState& S = c->ch[k];
    double* r = c->res_h + 4 * j;
    // the cache as the pass saw it at enqueue (an earlier job of this pass may
    // have evicted the entry since)
    if (jobs[j].cached) r[0] = jobs[j].ld;
    bool present = false;
    for (const ChainState::LogDet& e : S.ld) present |= e.lg == S.lgen[which];
    if (!present) {  // (re-)insert: the cache ends as after one call per job
      S.ld[S.ld_next] = {S.lgen[which], r[0]};
      S.ld_next ^= 1;
    }
    *jobs[j].out = r[0] - c->n * 0.5 * jobs[j].log_scale - 0.5 * r[1] / std::exp(jobs[j].log_scale);
    rowstats_store(c, k, which, jobs[j].beta0, r);
  }
}

static int loglik_jobs(nngp_ctx* c, LLJob* jobs, int nj) {
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = loglik_jobs_enqueue(c, jobs, nj))) return rc;
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  loglik_jobs_finish(c, jobs, nj);
  return NNGP_OK;
}

int nngp_loglik_chains(nngp_ctx* c, int which, int chain_mask, const double* beta0, const double* log_scale,
                       double* ll) {
  if (!c || !ll || !beta0 || !log_scale || (which != 0 && which != 1) || chain_mask <= 0 ||
      chain_mask >= (1 << c->C))
    return NNGP_ERR_ARG;
  LLJob jobs[kRowJobsMax];
  int nj = 0;
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) jobs[nj++] = {k, which, beta0[k], log_scale[k], ll + k};
  return loglik_jobs(c, jobs, nj);
}

int nngp_loglik_pair_chains(nngp_ctx* c, int chain_mask, const double* beta0, const double* log_scale_prop,
                            const double* log_scale_cur, double* ll_prop, double* ll_cur) {
  if (!c || !beta0 || !log_scale_prop || !log_scale_cur || !ll_prop || !ll_cur || chain_mask <= 0 ||
      chain_mask >= (1 << c->C))
    return NNGP_ERR_ARG;
  // the proposal's jobs first, then the current factor's: the cache updates of
  // nngp_loglik_chains(1, ...) followed by nngp_loglik_chains(0, ...)
  LLJob jobs[kRowJobsMax];
  int nj = 0;
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) jobs[nj++] = {k, 1, beta0[k], log_scale_prop[k], ll_prop + k};
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) jobs[nj++] = {k, 0, beta0[k], log_scale_cur[k], ll_cur + k};
  return loglik_jobs(c, jobs, nj);
}

// ---------------------------------------------------------------- sweep
static int sweep_prepare(nngp_ctx* c, int k, double beta0, double log_scale, double lnv, uint64_t seed,
                         uint64_t counter_base) {
  ChainState& S = c->ch[k];
  if (!S.have_factor[0] || !S.have_field || !S.have_mu) {
    char buf[96];
    std::snprintf(buf, sizeof buf, "sweep: chain %d needs factor, field and mu", k);
    return fail_msg(c, NNGP_ERR_STATE, buf);
  }
  if (S.mu_is_const && S.mu_beta0 != beta0) {  // residual sums depend on beta0 when mu = beta0
    S.mu_beta0 = beta0;
    S.res_stale = true;
  }
  SweepScalars& sc = c->scal_h[k];
  sc.inv_s2 = std::exp(-log_scale);
  sc.inv_t2 = std::exp(-lnv);
  sc.beta0 = beta0;
  sc.dshift = 0.0;
  sc.seed = seed;
  sc.counter_base = counter_base;
  return NNGP_OK;
}

// a sweep call rewrites the fields of the chains in mask (row-statistics cache)
static void fields_written(nngp_ctx* c, int mask) {
  for (int k = 0; k < c->C; ++k)
    if ((mask >> k) & 1) c->ch[k].fgen = ++c->gen;
}

// the tile engine's bounded spins set a timeout word instead of hanging


static int upload_scalars(nngp_ctx* c) {
  const int r = c->scal_next;
  c->scal_next = (r + 1) % nngp_ctx::kScalRing;
  if (c->scal_ev[r]) HIPCHK(c, hipEventSynchronize(c->scal_ev[r]));  // that slot's last copy has run
  else HIPCHK(c, hipEventCreateWithFlags(&c->scal_ev[r], hipEventDisableTiming));
  SweepScalars* slot = c->scal_ring_h + (size_t)r * c->C;
  std::memcpy(slot, c->scal_h, sizeof(SweepScalars) * c->C);
  HIPCHK(c, hipMemcpyAsync(c->scal_d, slot, sizeof(SweepScalars) * c->C, hipMemcpyHostToDevice, c->st));
  HIPCHK(c, hipEventRecord(c->scal_ev[r], c->st));
  return NNGP_OK;
}

// A sweep call = prologue (per chain in mask: w = field - beta0 in compact
// slot order, r = B w at Morton rows; the normals of sweep 0), the colour
// launches of every sweep, epilogue (field = w + beta0).
enum SweepPart { kPrologue = 1, kColours = 2, kEpilogue = 4, kAll = 7 };

static int enqueue_sweep_body(nngp_ctx* c, int n_sweeps, int mask, const double* z_dev, int parts = kAll) {
  const int n = c->n;
  SweepDev L = sweep_dev(c);
  FieldPtrs fp;
  for (int k = 0; k < kMaxChains; ++k) fp.p[k] = k < c->C ? c->ch[k].field_d : nullptr;
  if (parts & kPrologue) {
    HIPCHK(c, launch_field_to_slots_multi(c->st, c->n, c->slot_dpos_d, fp, c->scal_d, c->w_slot_d, c->C, mask));
    // r = B w of every chain in one pass; factor pointers and beta0 read from
    // device memory so a replayed graph sees the current factor and beta0
    HIPCHK(c, launch_spmv_chains(c->st, c->linv_cur_d, c->nn_d, n, c->b, fp, c->scal_d, c->r_d, c->C, mask));
    // normals of sweep 0 (later sweeps' normals are generated inside the
    // previous sweep's colour launches; the tile engine draws them inline)
    if (!z_dev && c->engine == 0) HIPCHK(c, launch_normals_compact(c->st, L, mask, 0, n, c->zbuf_d));
  }
  if ((parts & kColours) && c->engine == 1) {
    TileLaunch a;
    a.n_sweeps = n_sweeps;
    a.chain_mask = mask;
    a.z_in = z_dev;
    a.variant = c->tvariant;
    if (c->tcs) {
      a.stagger = c->tstagger;
      HIPCHK(c, launch_sweep_tiles_cs(c->st, tile_dev(c), a, c->tl.max_rows, c->tl.NTK, c->tl.max_batches,
                                      c->tl.max_gslots));
    } else {
      HIPCHK(c, launch_sweep_tiles(c->st, tile_dev(c), a, c->tl.max_rows, c->tl.NTK, c->tl.max_batches,
                                    c->tl.max_gslots));
    }
    HIPCHK(c, hipMemcpyAsync(c->tmo_h, c->ctl_d + 2, sizeof(unsigned), hipMemcpyDeviceToHost, c->st));
  }
  if ((parts & kColours) && c->engine == 0) {
    const size_t zn = (size_t)n * c->C;
    for (int s = 0; s < n_sweeps; ++s) {
      for (int col = 0; col < c->lay.K; ++col) {
        ColorLaunch a;
        a.chunk0 = c->lay.color_chunk_ptr[col];
        a.nch = c->lay.color_chunk_ptr[col + 1] - a.chunk0;
        a.chain_mask = mask;
        a.sweep_local = s;
        a.z_cur = z_dev ? z_dev + (size_t)s * zn : c->zbuf_d + (size_t)(s & 1) * zn;
        a.z_next = (!z_dev && s + 1 < n_sweeps) ? c->zbuf_d + (size_t)((s + 1) & 1) * zn : nullptr;
        a.pairs = c->pairs_d + c->pair_ptr[col];
        a.npairs = c->pair_ptr[col + 1] - c->pair_ptr[col];
        a.n = n;
        HIPCHK(c, launch_sweep_color(c->st, L, a));
      }
    }
  }
  if (parts & kEpilogue)
    HIPCHK(c, launch_slots_to_field_multi(c->st, c->n, c->slot_dpos_d, fp, c->scal_d, c->w_slot_d, c->C, mask));
  return NNGP_OK;
}

static int graph_for(nngp_ctx* c, int n_sweeps, int mask, hipGraphExec_t* out, int parts = kAll) {
  const long long key = ((long long)n_sweeps << 12) | ((long long)parts << 8) | mask;
  auto it = c->graphs.find(key);
  if (it == c->graphs.end()) {
    hipGraph_t g;
    HIPCHK(c, hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    int rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, parts);
    hipError_t e = hipStreamEndCapture(c->st, &g);
    if (rc) return rc;
    if (e != hipSuccess) return fail_hip(c, e, "hipStreamEndCapture");
    hipGraphExec_t ex;
    HIPCHK(c, hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    c->graph_objs.push_back(g);
    it = c->graphs.emplace(key, ex).first;
  }
  *out = it->second;
  return NNGP_OK;
}

static int shard_call(nngp_ctx* c, int n_sweeps, int mask);
// a call that needs the other ranks (a 1-rank tile shard is a plain tile context)
static bool sharded_call(const nngp_ctx* c) { return c->shard && !(c->engine == 1 && c->tG == 1); }
static int shard_ranks(const nngp_ctx* c) { return c->tG > 0 ? c->tG : c->sp.G; }
static int shard_rank(const nngp_ctx* c) { return c->tG > 0 ? c->trank : c->sp.rank; }

// the chains of mask can start from the slot-order w and r the last call
// left (call BEFORE fields_written): *cold = the chains that need the
// prologue (field -> slots, r = B w), *shift = warm chains whose beta_0 moved
// since (their field and factor unchanged): w -= d, r -= d B 1 instead.
// NNGP_SWEEP_WARM=0 (warm_on false): every chain cold; NNGP_SWEEP_SHIFT=0:
// a moved beta_0 makes the chain cold (the round-5 behaviour)
static void warm_kinds(const nngp_ctx* c, int mask, const double* beta0, int* cold, int* shift) {
  static const bool shift_on = [] {
    const char* e = std::getenv("NNGP_SWEEP_SHIFT");
    return !(e && std::string(e) == "0");
  }();
  *cold = 0;
  *shift = 0;
  const bool on = c->warm_on && c->engine == 1 && !c->shard;
  for (int k = 0; k < c->C; ++k) {
    if (!((mask >> k) & 1)) continue;
    const ChainState& S = c->ch[k];
    if (!on || !S.warm || S.fgen != S.warm_fgen || S.lgen[0] != S.warm_lgen) *cold |= 1 << k;
    else if (beta0[k] != S.warm_beta0) *(shift_on ? shift : cold) |= 1 << k;
  }
}

// the chains of shift start from w - d and r - d B 1 (the tile kernel's
// prologue and first draws, SweepScalars::dshift; B 1 computed once per
// factor generation, stream-ordered before the launch).  Call after
// sweep_prepare (which zeroes dshift) and before upload_scalars.
static int stage_warm_shift(nngp_ctx* c, int shift, const double* beta0) {
  for (int k = 0; k < c->C; ++k) {
    if (!((shift >> k) & 1)) continue;
    ChainState& S = c->ch[k];
    if (S.b1_lgen != S.lgen[0]) {
      HIPCHK(c, launch_linv_rowsum(c->st, S.linv_d[0], c->n, c->b, S.b1_d));
      S.b1_lgen = S.lgen[0];
    }
    c->scal_h[k].dshift = beta0[k] - S.warm_beta0;
  }
  return NNGP_OK;
}

// the call's launches: one captured graph of the whole call when every chain
// is cold; else the prologue graph of the cold chains and the graph of the
// colours + epilogue (warm and shifted chains start from the last call's w, r)
static int enqueue_call(nngp_ctx* c, int n_sweeps, int mask, int cold) {
  hipGraphExec_t ex;
  int rc;
  if (cold == mask) {
    if ((rc = graph_for(c, n_sweeps, mask, &ex, kAll))) return rc;
    HIPCHK(c, hipGraphLaunch(ex, c->st));
    return NNGP_OK;
  }
  if (cold) {
    if ((rc = graph_for(c, n_sweeps, cold, &ex, kPrologue))) return rc;
    HIPCHK(c, hipGraphLaunch(ex, c->st));
  }
  if ((rc = graph_for(c, n_sweeps, mask, &ex, kColours | kEpilogue))) return rc;
  HIPCHK(c, hipGraphLaunch(ex, c->st));
  return NNGP_OK;
}

// after a completed tile call (AFTER fields_written): slot-order w and r
// match the chains' new fields
static void warm_set(nngp_ctx* c, int mask, const double* beta0) {
  for (int k = 0; k < c->C; ++k) {
    if (!((mask >> k) & 1)) continue;
    ChainState& S = c->ch[k];
    S.warm = c->warm_on && c->engine == 1 && !c->shard;
    S.warm_fgen = S.fgen;
    S.warm_lgen = S.lgen[0];
    S.warm_beta0 = beta0[k];
  }
}

// A sweep call returns without a host sync (stream-ordered, like the other
// calls; its tile timeout word is checked after the next sync) unless a probe
// buffer is read.  Tile launches of several contexts on one device are
// chained by an event under the device's tile lock (tile_chain_event).
static bool sweep_async(const nngp_ctx* c) {
  static const bool force_sync = [] {  // NNGP_SWEEP_SYNC=1: every sweep call ends with a host sync
    const char* e = std::getenv("NNGP_SWEEP_SYNC");
    return e && std::string(e) == "1";
  }();
  return !force_sync && !c->tdbg_d && !c->dbg_d;
}

int nngp_sweep(nngp_ctx* c, int n_sweeps, double beta0, double log_scale, double lnv, uint64_t seed,
               uint64_t counter_base, const double* z) {
  if (!c || n_sweeps < 0) return NNGP_ERR_ARG;
  if (n_sweeps == 0) return NNGP_OK;
  int rc;
  if ((rc = set_device(c))) return rc;
  const int k = c->cur, mask = 1 << k;
  double b0v[kMaxChains] = {0, 0, 0, 0};
  b0v[k] = beta0;
  int cold = mask, shift = 0;
  if (!z) warm_kinds(c, mask, b0v, &cold, &shift);
  fields_written(c, mask);
  if ((rc = sweep_prepare(c, k, beta0, log_scale, lnv, seed, counter_base))) return rc;
  if (shift && (rc = stage_warm_shift(c, shift, b0v))) return rc;
  if ((rc = flush_sweep_values(c, mask))) return rc;
  if ((rc = upload_scalars(c))) return rc;
  if (sharded_call(c)) {
    if (z) return fail_msg(c, NNGP_ERR_ARG, "sweep: injected normals are not supported on shard contexts");
    return shard_call(c, n_sweeps, mask);
  }
  // the device's tile lock around the launch (and, unless the call returns
  // without a sync, until it has drained)
  std::unique_lock<std::mutex> tlk;
  if (c->engine == 1) tlk = std::unique_lock<std::mutex>(tile_lock(c->device));
  const bool async = sweep_async(c) && !z;
  if (z) {
    // injected normals -> compact order, chain-interleaved
    const size_t need = (size_t)n_sweeps * c->C * c->n;
    if (need > c->z_cap) {
      if (c->z_d) hipFree(c->z_d);
      c->z_d = nullptr;
      c->z_cap = 0;
      HIPCHK(c, dalloc(&c->z_d, need));
      c->z_cap = need;
    }
    std::vector<double> zc(need, 0.0);
    for (int s = 0; s < n_sweeps; ++s)
      for (int i = 0; i < c->n; ++i)
        zc[((size_t)s * c->n + c->loc_rank[i]) * c->C + k] = z[(size_t)s * c->n + i];
    HIPCHK(c, hipMemcpyAsync(c->z_d, zc.data(), need * sizeof(double), hipMemcpyHostToDevice, c->st));
    { int ss_ = sync_stream(c); if (ss_) return ss_; }
    if (c->engine == 1 && (rc = tile_chain_wait(c))) return rc;
    if ((rc = enqueue_sweep_body(c, n_sweeps, mask, c->z_d))) return rc;
    if (c->engine == 1 && (rc = tile_chain_record(c))) return rc;
  } else {
    // replay captured graphs of the call (launch-bound at small n)
    if (c->engine == 1 && (rc = tile_chain_wait(c))) return rc;
    if ((rc = enqueue_call(c, n_sweeps, mask, cold))) return rc;
    if (c->inject_tmo > 0 && c->engine == 1) {
      --c->inject_tmo;
      HIPCHK(c, launch_tile_inject_timeout(c->st, c->ctl_d));
    }
    if (c->engine == 1 && (rc = tile_chain_record(c))) return rc;
  }
  if (async) {
    c->tile_pending = c->engine == 1;
    if (tlk.owns_lock()) tlk.unlock();
  } else {
    { int ss_ = sync_stream(c); if (ss_) return ss_; }
    if ((rc = tile_timeout_check(c))) return rc;
  }
  warm_set(c, mask, b0v);
  return NNGP_OK;
}

int nngp_sweep_chains(nngp_ctx* c, int n_sweeps, const double* beta0, const double* log_scale,
                      const double* lnv, const uint64_t* seed, const uint64_t* counter_base) {
  if (!c || n_sweeps < 0 || !beta0 || !log_scale || !lnv || !seed || !counter_base) return NNGP_ERR_ARG;
  if (n_sweeps == 0) return NNGP_OK;
  int rc;
  if ((rc = set_device(c))) return rc;
  const int all = (1 << c->C) - 1;
  int cold = all, shift = 0;
  warm_kinds(c, all, beta0, &cold, &shift);
  fields_written(c, all);
  for (int k = 0; k < c->C; ++k)
    if ((rc = sweep_prepare(c, k, beta0[k], log_scale[k], lnv[k], seed[k], counter_base[k]))) return rc;
  if (shift && (rc = stage_warm_shift(c, shift, beta0))) return rc;
  if ((rc = flush_sweep_values(c, all))) return rc;
  if ((rc = upload_scalars(c))) return rc;
  if (sharded_call(c)) return shard_call(c, n_sweeps, all);
  // the device's tile lock around the launch (and, unless the call returns
  // without a sync, until it has drained)
  std::unique_lock<std::mutex> tlk;
  if (c->engine == 1) tlk = std::unique_lock<std::mutex>(tile_lock(c->device));
  const bool async = sweep_async(c);
  if (c->engine == 1 && (rc = tile_chain_wait(c))) return rc;
  if ((rc = enqueue_call(c, n_sweeps, all, cold))) return rc;
  if (c->inject_tmo > 0 && c->engine == 1) {
    --c->inject_tmo;
    HIPCHK(c, launch_tile_inject_timeout(c->st, c->ctl_d));
  }
  if (c->engine == 1 && (rc = tile_chain_record(c))) return rc;
  if (async) {
    c->tile_pending = c->engine == 1;
    if (tlk.owns_lock()) tlk.unlock();
  } else {
    { int ss_ = sync_stream(c); if (ss_) return ss_; }
    tlk = std::unique_lock<std::mutex>();
    if ((rc = tile_timeout_check(c))) return rc;
  }
  warm_set(c, all, beta0);
  if (c->tdbg_d) {
    if (const char* path = std::getenv("NNGP_DBG_OUT")) {
      std::vector<unsigned long long> h(c->tdbg_n);
      HIPCHK(c, hipMemcpy(h.data(), c->tdbg_d, h.size() * 8, hipMemcpyDeviceToHost));
      if (FILE* f = std::fopen(path, "wb")) {
        std::fwrite(h.data(), 8, h.size(), f);
        // then the neighbour tiles of each (tile, colour) (timeline.py: skew vs transit)
        std::fwrite(c->tl.nb_ptr.data(), sizeof(int), c->tl.nb_ptr.size(), f);
        std::fwrite(c->tl.nb.data(), sizeof(int), c->tl.nb.size(), f);
        std::fclose(f);
      }
    }
  }
  if (c->dbg_d) {
    if (const char* path = std::getenv("NNGP_DBG_OUT")) {
      std::vector<unsigned long long> h((size_t)c->lay.nchunks * 8);
      HIPCHK(c, hipMemcpy(h.data(), c->dbg_d, h.size() * 8, hipMemcpyDeviceToHost));
      if (FILE* f = std::fopen(path, "wb")) {
        std::fwrite(c->lay.color_chunk_ptr.data(), sizeof(int), c->lay.K + 1, f);
        std::fwrite(h.data(), 8, h.size(), f);
        std::fclose(f);
      }
    }
  }
  return NNGP_OK;
}

// ---------------------------------------------------------------- sharded sweep
// A call of the colour-sharded sweep on rank sp.rank: the
// prologue/epilogue of the single-rank call (every rank keeps a full replica
// of w, so r = B w and field = w + beta0 need no exchange), and per colour:
//   own    -- the rank's chunks of the colour; the kernel also writes {dw, w_new}
//             of its slots into the rank's segment of the colour's exchange region;
//   xchg   -- all-gather of the region (RCCL, in place) or, in a group of
//             contexts in one process, device copies of the other segments;
//   ghosts -- r_k += B[k,j] dw_j for the foreign members j of the colour in
//             rows the rank's columns touch; w replica of foreign slots = w_new.
static int enqueue_shard_own(nngp_ctx* c, int s, int col, int mask, int n_sweeps) {
  const ShardPlan& P = c->sp;
  const int G = P.G, rk = P.rank;
  const size_t zn = (size_t)c->n * c->C;
  ColorLaunch a;
  a.chunk0 = P.cb[(size_t)col * (G + 1) + rk];
  a.nch = P.cb[(size_t)col * (G + 1) + rk + 1] - a.chunk0;
  a.chain_mask = mask;
  a.sweep_local = s;
  a.z_cur = c->zbuf_d + (size_t)(s & 1) * zn;
  a.z_next = s + 1 < n_sweeps ? c->zbuf_d + (size_t)((s + 1) & 1) * zn : nullptr;
  a.pairs = c->sp_pairs_d + P.pair_ptr[col];
  a.npairs = P.pair_ptr[col + 1] - P.pair_ptr[col];
  a.n = c->n;
  a.xsend = c->xbuf_d + (size_t)(P.xoff[col] + (long long)rk * P.cnt[col]) * c->C;
  a.xs0 = P.seg0[(size_t)col * (G + 1) + rk];
  HIPCHK(c, launch_sweep_color(c->st, sweep_dev(c), a));
  return NNGP_OK;
}

static int enqueue_shard_ghosts(nngp_ctx* c, int col, int mask) {
  const ShardPlan& P = c->sp;
  ShardGhostLaunch g;
  g.grow = c->sg_row_d;
  g.grecv = c->sg_recv_d;
  g.gval = c->sg_val_d;
  g.ng_total = (long long)P.grow.size();
  g.g0 = P.gptr[col];
  g.ng = P.gptr[col + 1] - g.g0;
  g.xbuf = c->xbuf_d + (size_t)P.xoff[col] * c->C;
  g.G = P.G;
  g.rank = P.rank;
  g.cnt = P.cnt[col];
  for (int h = 0; h <= P.G; ++h) g.seg0[h] = P.seg0[(size_t)col * (P.G + 1) + h];
  g.chain_mask = mask;
  HIPCHK(c, launch_shard_ghosts(c->st, sweep_dev(c), g));
  return NNGP_OK;
}

static int enqueue_shard_allgather(nngp_ctx* c, int col) {
  const ShardPlan& P = c->sp;
  if (P.G == 1) return NNGP_OK;
  const size_t cnt = (size_t)P.cnt[col] * c->C * 2;  // doubles per rank
  double* base = reinterpret_cast<double*>(c->xbuf_d + (size_t)P.xoff[col] * c->C);
  ncclResult_t e = ncclAllGather(base + (size_t)P.rank * cnt, base, cnt, ncclDouble, c->comm, c->st);
  if (e != ncclSuccess) return fail_msg(c, NNGP_ERR_COMM, std::string("ncclAllGather: ") + ncclGetErrorString(e));
  return NNGP_OK;
}

// Host checks of everything the per-colour loop reads, so that a failure can
// only happen before the first collective is enqueued or after the last one
// (a rank leaving the loop half way would leave its peers waiting in the next
// all-gather).
static int shard_plan_check(const nngp_ctx* c) {
  const ShardPlan& P = c->sp;
  const int G = P.G, K = P.K;
  if (G < 1 || G > 64 || P.rank < 0 || P.rank >= G || K < 1) return NNGP_ERR_ARG;
  if ((int)P.cb.size() != K * (G + 1) || (int)P.seg0.size() != K * (G + 1) || (int)P.cnt.size() != K ||
      (int)P.xoff.size() != K + 1 || (int)P.gptr.size() != K + 1 || (int)P.pair_ptr.size() != K + 1)
    return NNGP_ERR_ARG;
  for (int col = 0; col < K; ++col) {
    if (P.cnt[col] < 0 || P.xoff[col + 1] - P.xoff[col] != (long long)G * P.cnt[col]) return NNGP_ERR_ARG;
    if (P.gptr[col] > P.gptr[col + 1] || P.gptr[col + 1] > (int)P.grow.size()) return NNGP_ERR_ARG;
    if (P.pair_ptr[col] > P.pair_ptr[col + 1]) return NNGP_ERR_ARG;
    for (int h = 0; h < G; ++h) {
      const size_t i = (size_t)col * (G + 1) + h;
      if (P.cb[i] > P.cb[i + 1] || P.seg0[i] > P.seg0[i + 1] || P.seg0[i + 1] - P.seg0[i] > P.cnt[col])
        return NNGP_ERR_ARG;
    }
  }
  return NNGP_OK;
}

// ---------------------------------------------------------------- tile shard
// Exchange without RCCL: full -- this rank's slots into every
// peer's replica (peer copies over xGMI); else only the halo (its slots read
// by other ranks' rows: what their next prologue needs), stored straight into
// the peers' replicas.  Then the flags: every rank stores the exchange number
// into every peer's flag word and waits for all of its own.  A peer writes
// only this rank's foreign slots, and only after the rendezvous that orders
// it behind this rank's reads of them.
static int tile_ipc_exchange(nngp_ctx* c, bool full) {
  const TileLayout& TL = c->tl;
  c->xseq++;
  TilePeerFlags pf;
  for (int h = 0; h < c->tG; ++h)
    if (h != c->trank) pf.f[h] = c->peer_xf[h];
  if (full) {
    const size_t s0 = (size_t)TL.rank_slot0[c->trank] * c->C;
    const size_t cnt = (size_t)(TL.rank_slot0[c->trank + 1] - TL.rank_slot0[c->trank]) * c->C;
    for (int h = 0; h < c->tG; ++h)
      if (h != c->trank)
        HIPCHK(c, hipMemcpyAsync(c->peer_w[h] + s0, c->w_slot_d + s0, cnt * sizeof(double), hipMemcpyDeviceToDevice,
                                 c->st));
  } else {
    TilePeerW pw;
    for (int h = 0; h < c->tG; ++h)
      if (h != c->trank) pw.w[h] = c->peer_w[h];
    for (int h = 0; h <= kTileRanksMax; ++h) pw.hptr[h] = c->halo_ptr[h];
    HIPCHK(c, launch_tile_halo_put(c->st, pw, c->halo_d, c->w_slot_d, c->C));
  }
  HIPCHK(c, launch_tile_xsignal(c->st, pf, c->xseq, c->tG, c->trank));
  HIPCHK(c, launch_tile_xwait(c->st, c->xflag_d, c->ctl_d, c->xseq, c->tG, c->trank));
  HIPCHK(c, hipMemcpyAsync(c->tmo_h, c->ctl_d + 2, sizeof(unsigned), hipMemcpyDeviceToHost, c->st));
  return NNGP_OK;
}

// before an entry point reads the field of a tile-shard rank whose last
// calls exchanged only the halo: a full exchange, then field = w + beta0 of
// every slot of those chains again
static int replica_sync(nngp_ctx* c) {
  if (!c->stale_mask) return NNGP_OK;
  int rc;
  if ((rc = set_device(c))) return rc;
  const int mask = c->stale_mask;
  if ((rc = tile_ipc_exchange(c, true))) return rc;
  if ((rc = enqueue_sweep_body(c, 1, mask, nullptr, 4))) return rc;  // kEpilogue
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  c->stale_mask = 0;
  return tile_timeout_check(c);
}

int nngp_shard_sync(nngp_ctx* c) {
  if (!c) return NNGP_ERR_ARG;
  return replica_sync(c);
}

// A call of the tile-sharded sweep on rank trank: prologue
// (full replica: r = B w of every row), one persistent launch of the rank's
// tiles (draws read by other ranks' tiles go into their granule buffers over
// xGMI), then every rank's own slots of w to the others (one RCCL broadcast
// per rank, in place) and the epilogue (field = w + beta0 of every slot).
// The next call's launch starts after every rank's broadcast, i.e. after
// every rank's tiles have stopped polling: granules of consecutive calls
// never mix (and carry the call id besides).
static int tile_shard_exchange(nngp_ctx* c) {
  const TileLayout& TL = c->tl;
  if (!c->comm) return tile_ipc_exchange(c, false);
  ncclResult_t e = ncclGroupStart();
  for (int h = 0; h < c->tG && e == ncclSuccess; ++h) {
    const size_t s0 = (size_t)TL.rank_slot0[h] * c->C, cnt = (size_t)(TL.rank_slot0[h + 1] - TL.rank_slot0[h]) * c->C;
    e = ncclBroadcast(c->w_slot_d + s0, c->w_slot_d + s0, cnt, ncclDouble, h, c->comm, c->st);
  }
  ncclResult_t e2 = ncclGroupEnd();
  if (e == ncclSuccess) e = e2;
  if (e != ncclSuccess) return fail_msg(c, NNGP_ERR_COMM, std::string("tile shard broadcast: ") + ncclGetErrorString(e));
  return NNGP_OK;
}

static TileShard tile_shard_args(nngp_ctx* const* ranks, int G, int g0, int Tl) {
  TileShard sh;
  sh.G = G;
  sh.Tl = Tl;
  sh.tile0 = g0 * Tl;
  sh.rank0 = g0;
  sh.devs = ranks[g0]->tdev_d;
  sh.call = ranks[g0]->ctl_d;
  for (int h = 0; h < G; ++h) sh.gx[h] = ranks[h]->dwx_d;
  return sh;
}

static int tile_shard_call(nngp_ctx* c, int n_sweeps, int mask) {
  if (!c->comm && !c->peers_open)
    return fail_msg(c, NNGP_ERR_STATE, "tile shard: no communicator (nngp_shard_comm_init) -- or use nngp_sweep_chains_group");
  if (!c->peers_open)
    return fail_msg(c, NNGP_ERR_STATE, "tile shard: the other ranks' granule buffers are not open (nngp_shard_ipc_open)");
  if (!c->rmask_d || c->tG < 2) return fail_msg(c, NNGP_ERR_STATE, "tile shard: no remote-reader plan");
  int rc;
  std::lock_guard<std::mutex> tlk(tile_lock(c->device));
  if ((rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, kPrologue))) return rc;
  HIPCHK(c, launch_tile_call_bump(c->st, c->ctl_d));
  TileShard sh;
  sh.G = c->tG;
  sh.Tl = c->tTl;
  sh.tile0 = c->trank * c->tTl;
  sh.rank0 = c->trank;
  sh.devs = c->tdev_d;
  sh.call = c->ctl_d;
  for (int h = 0; h < c->tG; ++h) sh.gx[h] = h == c->trank ? c->dwx_d : c->peer_gx[h];
  TileLaunch a;
  a.n_sweeps = n_sweeps;
  a.chain_mask = mask;
  a.z_in = nullptr;
  int wrc = tile_chain_wait(c);
  hipError_t e = wrc ? hipErrorUnknown
                     : launch_sweep_tiles(c->st, tile_dev(c), a, c->tl.max_rows, c->tl.NTK, c->tl.max_batches,
                                          c->tl.max_gslots, &sh, c->tTl);
  if (e == hipSuccess && tile_chain_record(c)) e = hipErrorUnknown;
  if (e == hipSuccess) e = hipMemcpyAsync(c->tmo_h, c->ctl_d + 2, sizeof(unsigned), hipMemcpyDeviceToHost, c->st);
  // the broadcasts go out even after a failed launch: the peers wait in them
  rc = tile_shard_exchange(c);
  if (e != hipSuccess || rc) {
    if (c->comm) {
      ncclCommAbort(c->comm);
      c->comm = nullptr;
    }
    return e != hipSuccess ? fail_hip(c, e, "tile shard launch") : rc;
  }
  if ((rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, kEpilogue))) return rc;
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  if (!c->comm) c->stale_mask |= mask;
  return tile_timeout_check(c);
}

// the three buffers the other ranks map: granules, w replica, exchange flags
static_assert(NNGP_IPC_HANDLE_BYTES >= 3 * (int)sizeof(hipIpcMemHandle_t), "IPC handle record");
int nngp_shard_ipc_handle(nngp_ctx* c, unsigned char* handle, int len) {
  if (!c || !handle || len < NNGP_IPC_HANDLE_BYTES) return NNGP_ERR_ARG;
  if (c->tG < 1) return fail_msg(c, NNGP_ERR_STATE, "shard_ipc_handle: not a tile shard context");
  int rc;
  if ((rc = set_device(c))) return rc;
  void* bufs[3] = {c->dwx_d, c->w_slot_d, c->xflag_d};
  for (int k = 0; k < 3; ++k) {
    hipIpcMemHandle_t h;
    HIPCHK(c, hipIpcGetMemHandle(&h, bufs[k]));
    std::memcpy(handle + k * sizeof h, &h, sizeof h);
  }
  return NNGP_OK;
}

int nngp_shard_ipc_open(nngp_ctx* c, const unsigned char* handles, int len_each) {
  if (!c || !handles || len_each < NNGP_IPC_HANDLE_BYTES) return NNGP_ERR_ARG;
  if (c->tG < 1) return fail_msg(c, NNGP_ERR_STATE, "shard_ipc_open: not a tile shard context");
  if (c->peers_open) return fail_msg(c, NNGP_ERR_STATE, "shard_ipc_open: already open");
  int rc;
  if ((rc = set_device(c))) return rc;
  auto close_all = [&] {
    for (int q = 0; q < c->tG; ++q) {
      if (q == c->trank) continue;
      for (void** pp : {(void**)&c->peer_gx[q], (void**)&c->peer_w[q], (void**)&c->peer_xf[q]})
        if (*pp) { hipIpcCloseMemHandle(*pp); *pp = nullptr; }
    }
  };
  for (int h = 0; h < c->tG; ++h) {
    if (h == c->trank) continue;
    void* got[3] = {nullptr, nullptr, nullptr};
    for (int k = 0; k < 3; ++k) {
      hipIpcMemHandle_t hh;
      std::memcpy(&hh, handles + (size_t)h * len_each + k * sizeof hh, sizeof hh);
      hipError_t e = hipIpcOpenMemHandle(&got[k], hh, hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) {
        for (int q = 0; q < k; ++q) hipIpcCloseMemHandle(got[q]);
        close_all();
        return fail_hip(c, e, "hipIpcOpenMemHandle (a buffer of another rank)");
      }
    }
    c->peer_gx[h] = static_cast<double*>(got[0]);
    c->peer_w[h] = static_cast<double*>(got[1]);
    c->peer_xf[h] = static_cast<unsigned*>(got[2]);
  }
  c->peers_open = true;
  return NNGP_OK;
}

static int shard_call(nngp_ctx* c, int n_sweeps, int mask) {
  if (c->engine == 1) return tile_shard_call(c, n_sweeps, mask);
  if (c->sp.G > 1 && !c->comm)
    return fail_msg(c, NNGP_ERR_STATE, "sharded sweep: no communicator (nngp_shard_comm_init) -- or use nngp_sweep_chains_group");
  if (shard_plan_check(c)) return fail_msg(c, NNGP_ERR_ARG, "sharded sweep: inconsistent shard plan");
  int rc;
  if ((rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, kPrologue))) return rc;
  for (int s = 0; s < n_sweeps; ++s)
    for (int col = 0; col < c->sp.K; ++col) {
      if (!(rc = enqueue_shard_own(c, s, col, mask, n_sweeps)) && !(rc = enqueue_shard_allgather(c, col)))
        rc = enqueue_shard_ghosts(c, col, mask);
      if (rc) {
        // a launch or RCCL failure half way (the checks above exclude the
        // argument errors): abort the communicator so this rank does not
        // leave queued collectives its peers wait on; the shard is unusable
        // until the contexts are recreated
        if (c->comm) {
          ncclCommAbort(c->comm);
          c->comm = nullptr;
        }
        return rc;
      }
    }
  if ((rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, kEpilogue))) return rc;
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  return NNGP_OK;
}

int nngp_shard_unique_id(unsigned char* id, int len) {
  if (!id || len < (int)sizeof(ncclUniqueId))
    return fail_msg(nullptr, NNGP_ERR_ARG, "shard_unique_id: need a buffer of NNGP_SHARD_ID_BYTES");
  ncclUniqueId u;
  ncclResult_t e = ncclGetUniqueId(&u);
  if (e != ncclSuccess) return fail_msg(nullptr, NNGP_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(e));
  std::memcpy(id, &u, sizeof u);
  return NNGP_OK;
}

int nngp_shard_comm_init(nngp_ctx* c, const unsigned char* id, int len) {
  if (!c || !id || len < (int)sizeof(ncclUniqueId)) return NNGP_ERR_ARG;
  if (!c->shard) return fail_msg(c, NNGP_ERR_STATE, "shard_comm_init: not a shard context (nngp_ctx_create_shard)");
  if (c->comm) return fail_msg(c, NNGP_ERR_STATE, "shard_comm_init: communicator already initialised");
  int rc;
  if ((rc = set_device(c))) return rc;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclResult_t e = ncclCommInitRank(&c->comm, shard_ranks(c), u, shard_rank(c));
  if (e != ncclSuccess) {
    c->comm = nullptr;
    return fail_msg(c, NNGP_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(e));
  }
  return NNGP_OK;
}

// All ranks of a tile shard in one process: the ranks of each device run in
// one launch (tiles [g0*Tl, g1*Tl)), the granules of ranks on other devices
// go to their buffers through peer access; w of every rank's slots reaches the
// others by device copies.
static int tile_group_call(nngp_ctx** ctxs, int G, int n_sweeps, const double* beta0, const double* log_scale,
                           const double* lnv, const uint64_t* seed, const uint64_t* counter_base) {
  nngp_ctx* c0 = ctxs[0];
  for (int g = 0; g < G; ++g) {
    nngp_ctx* c = ctxs[g];
    if (!c || c->engine != 1 || c->tG != G || c->trank != g || c->tTl != c0->tTl || c->n != c0->n || c->C != c0->C ||
        c->tl.K != c0->tl.K || c->tl.T != c0->tl.T || !c->rmask_d)
      return fail_msg(c, NNGP_ERR_ARG, "sweep_chains_group: ctxs[g] must be rank g of a G-rank tile shard of one graph");
    for (int h = 0; h + 1 < g; ++h)
      if (ctxs[h]->device == c->device && ctxs[g - 1]->device != c->device)
        return fail_msg(c, NNGP_ERR_ARG, "sweep_chains_group: the ranks of one device must be contiguous");
  }
  if (n_sweeps == 0) return NNGP_OK;
  const int Tl = c0->tTl, mask = (1 << c0->C) - 1;
  int rc;
  // every device of the group, in device order (no lock-order inversion)
  std::vector<int> devs_used;
  for (int g = 0; g < G; ++g) devs_used.push_back(ctxs[g]->device);
  std::sort(devs_used.begin(), devs_used.end());
  devs_used.erase(std::unique(devs_used.begin(), devs_used.end()), devs_used.end());
  std::vector<std::unique_lock<std::mutex>> tlks;
  for (int dv : devs_used) tlks.emplace_back(tile_lock(dv));
  std::vector<hipEvent_t> ev(2 * G, nullptr);  // [g]: prologue of rank g done; [G + g]: launch of rank g's device done
  auto cleanup = [&] {
    for (auto e : ev) if (e) hipEventDestroy(e);
  };
#define GCHK(c, x)                                                     \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) { cleanup(); return fail_hip((c), e_, #x); } \
  } while (0)
  for (int g = 0; g < G; ++g) {
    nngp_ctx* c = ctxs[g];
    if ((rc = set_device(c))) { cleanup(); return rc; }
    GCHK(c, hipEventCreateWithFlags(&ev[g], hipEventDisableTiming));
    GCHK(c, hipEventCreateWithFlags(&ev[G + g], hipEventDisableTiming));
    for (int k = 0; k < c->C; ++k)
      if ((rc = sweep_prepare(c, k, beta0[k], log_scale[k], lnv[k], seed[k], counter_base[k]))) { cleanup(); return rc; }
    if ((rc = flush_sweep_values(c, mask))) { cleanup(); return rc; }
    if ((rc = upload_scalars(c))) { cleanup(); return rc; }
    if ((rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, kPrologue))) { cleanup(); return rc; }
    GCHK(c, launch_tile_call_bump(c->st, c->ctl_d));  // every rank's call id and timeout word
    GCHK(c, hipEventRecord(ev[g], c->st));
  }
  std::vector<TileDev> devs(G);
  for (int g = 0; g < G; ++g) devs[g] = tile_dev(ctxs[g]);
  for (int g0 = 0; g0 < G;) {
    int g1 = g0 + 1;
    while (g1 < G && ctxs[g1]->device == ctxs[g0]->device) ++g1;
    nngp_ctx* L = ctxs[g0];
    set_device(L);
    int cus = 0;
    GCHK(L, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, L->device));
    if ((long long)(g1 - g0) * Tl > (long long)std::max(L->tresident, 1) * cus) {
      cleanup();
      return fail_msg(L, NNGP_ERR_ARG, "sweep_chains_group: the tiles of the ranks on one device exceed what is "
                                       "resident at once (occupancy x CUs; fewer tiles: NNGP_TILES)");
    }
    for (int h = 0; h < G; ++h)
      if (ctxs[h]->device != L->device) {
        hipError_t pe = hipDeviceEnablePeerAccess(ctxs[h]->device, 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) GCHK(L, pe);
        (void)hipGetLastError();
      }
    for (int h = g0; h < g1; ++h) GCHK(L, hipStreamWaitEvent(L->st, ev[h], 0));
    GCHK(L, hipMemcpyAsync(L->tdev_d, devs.data() + g0, sizeof(TileDev) * (g1 - g0), hipMemcpyHostToDevice, L->st));
    TileShard sh = tile_shard_args(ctxs, G, g0, Tl);
    TileLaunch a;
    a.n_sweeps = n_sweeps;
    a.chain_mask = mask;
    a.z_in = nullptr;
    if ((rc = tile_chain_wait(L))) { cleanup(); return rc; }
    GCHK(L, launch_sweep_tiles(L->st, devs[g0], a, L->tl.max_rows, L->tl.NTK, L->tl.max_batches, L->tl.max_gslots, &sh,
                               (g1 - g0) * Tl));
    if ((rc = tile_chain_record(L))) { cleanup(); return rc; }
    for (int h = g0; h < g1; ++h)
      GCHK(L, hipMemcpyAsync(ctxs[h]->tmo_h, ctxs[h]->ctl_d + 2, sizeof(unsigned), hipMemcpyDeviceToHost, L->st));
    for (int h = g0; h < g1; ++h) GCHK(L, hipEventRecord(ev[G + h], L->st));
    g0 = g1;
  }
  // every rank's own slots of w to the others, then the epilogues
  const TileLayout& TL = c0->tl;
  for (int g = 0; g < G; ++g) {
    nngp_ctx* c = ctxs[g];
    set_device(c);
    for (int h = 0; h < G; ++h) GCHK(c, hipStreamWaitEvent(c->st, ev[G + h], 0));
    for (int h = 0; h < G; ++h) {
      if (h == g) continue;
      const size_t s0 = (size_t)TL.rank_slot0[h] * c->C, cnt = (size_t)(TL.rank_slot0[h + 1] - TL.rank_slot0[h]) * c->C;
      GCHK(c, hipMemcpyAsync(c->w_slot_d + s0, ctxs[h]->w_slot_d + s0, cnt * sizeof(double), hipMemcpyDefault, c->st));
    }
    if ((rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, kEpilogue))) { cleanup(); return rc; }
  }
  for (int g = 0; g < G; ++g) {
    set_device(ctxs[g]);
    GCHK(ctxs[g], hipStreamSynchronize(ctxs[g]->st));
  }
#undef GCHK
  cleanup();
  for (int g = 0; g < G; ++g)
    if ((rc = tile_timeout_check(ctxs[g]))) return rc;
  return NNGP_OK;
}

int nngp_sweep_chains_group(nngp_ctx** ctxs, int G, int n_sweeps, const double* beta0, const double* log_scale,
                            const double* lnv, const uint64_t* seed, const uint64_t* counter_base) {
  if (!ctxs || G < 1 || n_sweeps < 0 || !beta0 || !log_scale || !lnv || !seed || !counter_base) return NNGP_ERR_ARG;
  for (int g = 0; g < G; ++g)
    if (ctxs[g] && n_sweeps > 0) fields_written(ctxs[g], (1 << ctxs[g]->C) - 1);
  if (ctxs[0] && ctxs[0]->engine == 1) {
    if (G > kTileRanksMax) return fail_msg(ctxs[0], NNGP_ERR_ARG, "sweep_chains_group: too many ranks");
    // one rank: the plain tile sweep (no remote readers, no plan masks)
    if (G == 1 && ctxs[0]->tG == 1)
      return nngp_sweep_chains(ctxs[0], n_sweeps, beta0, log_scale, lnv, seed, counter_base);
    return tile_group_call(ctxs, G, n_sweeps, beta0, log_scale, lnv, seed, counter_base);
  }
  for (int g = 0; g < G; ++g) {
    nngp_ctx* c = ctxs[g];
    if (!c || !c->shard || c->sp.G != G || c->sp.rank != g || c->n != ctxs[0]->n || c->C != ctxs[0]->C ||
        c->sp.K != ctxs[0]->sp.K)
      return fail_msg(c, NNGP_ERR_ARG, "sweep_chains_group: ctxs[g] must be rank g of a G-rank shard of one graph");
  }
  if (n_sweeps == 0) return NNGP_OK;
  int rc;
  const int mask = (1 << ctxs[0]->C) - 1;
  for (int g = 0; g < G; ++g) {
    nngp_ctx* c = ctxs[g];
    if ((rc = set_device(c))) return rc;
    for (int k = 0; k < c->C; ++k)
      if ((rc = sweep_prepare(c, k, beta0[k], log_scale[k], lnv[k], seed[k], counter_base[k]))) return rc;
    if ((rc = flush_sweep_values(c, mask))) return rc;
    if ((rc = upload_scalars(c))) return rc;
    if ((rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, kPrologue))) return rc;
  }
  // ev_own[g]: rank g's segment of the colour is written; ev_done[g]: rank g
  // has copied the others' segments (nobody rewrites a segment before every
  // rank has read it)
  std::vector<hipEvent_t> ev_own(G), ev_done(G);
  auto cleanup = [&] {
    for (auto e : ev_own) if (e) hipEventDestroy(e);
    for (auto e : ev_done) if (e) hipEventDestroy(e);
  };
  for (int g = 0; g < G; ++g) {
    set_device(ctxs[g]);
    if (hipEventCreateWithFlags(&ev_own[g], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev_done[g], hipEventDisableTiming) != hipSuccess) {
      cleanup();
      return fail_msg(ctxs[g], NNGP_ERR_HIP, "sweep_chains_group: hipEventCreate");
    }
  }
#define GCHK(c, x)                                                   \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) { cleanup(); return fail_hip((c), e_, #x); } \
  } while (0)
  const ShardPlan& P0 = ctxs[0]->sp;
  for (int s = 0; s < n_sweeps; ++s)
    for (int col = 0; col < P0.K; ++col) {
      for (int g = 0; g < G; ++g) {
        nngp_ctx* c = ctxs[g];
        set_device(c);
        if (s + col > 0)
          for (int h = 0; h < G; ++h) GCHK(c, hipStreamWaitEvent(c->st, ev_done[h], 0));
        if ((rc = enqueue_shard_own(c, s, col, mask, n_sweeps))) { cleanup(); return rc; }
        GCHK(c, hipEventRecord(ev_own[g], c->st));
      }
      const size_t seg = (size_t)P0.cnt[col] * ctxs[0]->C;
      for (int g = 0; g < G; ++g) {
        nngp_ctx* c = ctxs[g];
        set_device(c);
        for (int h = 0; h < G; ++h) {
          if (h == g) continue;
          GCHK(c, hipStreamWaitEvent(c->st, ev_own[h], 0));
          const size_t off = (size_t)P0.xoff[col] * c->C + (size_t)h * seg;
          GCHK(c, hipMemcpyAsync(c->xbuf_d + off, ctxs[h]->xbuf_d + off, seg * sizeof(double2), hipMemcpyDefault,
                                 c->st));
        }
        GCHK(c, hipEventRecord(ev_done[g], c->st));
        if ((rc = enqueue_shard_ghosts(c, col, mask))) { cleanup(); return rc; }
      }
    }
#undef GCHK
  for (int g = 0; g < G; ++g) {
    nngp_ctx* c = ctxs[g];
    set_device(c);
    if ((rc = enqueue_sweep_body(c, n_sweeps, mask, nullptr, kEpilogue))) { cleanup(); return rc; }
  }
  for (int g = 0; g < G; ++g) {
    set_device(ctxs[g]);
    hipError_t e = hipStreamSynchronize(ctxs[g]->st);
    if (e != hipSuccess) { cleanup(); return fail_hip(ctxs[g], e, "hipStreamSynchronize"); }
  }
  cleanup();
  return NNGP_OK;
}

int nngp_sweep_timed(nngp_ctx* c, int n_sweeps, const double* beta0, const double* log_scale,
                     const double* lnv, const uint64_t* seed, const uint64_t* counter_base, double* ms,
                     double* kernel_ms) {
  if (!c || n_sweeps < 1 || !ms || !beta0 || !log_scale || !lnv || !seed || !counter_base) return NNGP_ERR_ARG;
  if (sharded_call(c)) return fail_msg(c, NNGP_ERR_STATE, "sweep_timed: not available on shard contexts");
  int rc;
  if ((rc = set_device(c))) return rc;
  fields_written(c, (1 << c->C) - 1);
  for (int k = 0; k < c->C; ++k)
    if ((rc = sweep_prepare(c, k, beta0[k], log_scale[k], lnv[k], seed[k], counter_base[k]))) return rc;
  if ((rc = flush_sweep_values(c, (1 << c->C) - 1))) return rc;
  if ((rc = upload_scalars(c))) return rc;
  const int mask = (1 << c->C) - 1;
  std::unique_lock<std::mutex> tlk;
  if (c->engine == 1) tlk = std::unique_lock<std::mutex>(tile_lock(c->device));
  hipGraphExec_t pro, col, epi;
  if ((rc = graph_for(c, n_sweeps, mask, &pro, kPrologue))) return rc;
  if ((rc = graph_for(c, n_sweeps, mask, &col, kColours))) return rc;
  if ((rc = graph_for(c, n_sweeps, mask, &epi, kEpilogue))) return rc;
  if (c->engine == 1 && (rc = tile_chain_wait(c))) return rc;
  hipEvent_t e[4];
  for (auto& x : e) HIPCHK(c, hipEventCreate(&x));
  // the colour launches alone are bracketed by e[1], e[2]: their mean
  // duration (including the dependent-launch gaps, as in a rocprofv3 trace
  // of the same graph) is the sweep kernel's launch time
  HIPCHK(c, hipEventRecord(e[0], c->st));
  HIPCHK(c, hipGraphLaunch(pro, c->st));
  HIPCHK(c, hipEventRecord(e[1], c->st));
  HIPCHK(c, hipGraphLaunch(col, c->st));
  HIPCHK(c, hipEventRecord(e[2], c->st));
  HIPCHK(c, hipGraphLaunch(epi, c->st));
  HIPCHK(c, hipEventRecord(e[3], c->st));
  if (c->engine == 1 && (rc = tile_chain_record(c))) return rc;
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  float f = 0, g = 0;
  HIPCHK(c, hipEventElapsedTime(&f, e[0], e[3]));
  HIPCHK(c, hipEventElapsedTime(&g, e[1], e[2]));
  *ms = f;
  if (kernel_ms) *kernel_ms = g;
  for (auto& x : e) hipEventDestroy(x);
  if ((rc = tile_timeout_check(c))) return rc;
  warm_set(c, mask, beta0);
  return NNGP_OK;
}

int nngp_get_sweep_r(nngp_ctx* c, double* r) {
  if (!c || !r) return NNGP_ERR_ARG;
  int rc;
  if ((rc = set_device(c))) return rc;
  std::vector<double> h((size_t)c->n * c->C);
  HIPCHK(c, hipMemcpyAsync(h.data(), c->r_d, h.size() * sizeof(double), hipMemcpyDeviceToHost, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  for (int i = 0; i < c->n; ++i) r[i] = h[(size_t)c->dpos[i] * c->C + c->cur];
  return NNGP_OK;
}

// ---------------------------------------------------------------- MH helpers
static int tri_solve_dev(nngp_ctx* c, const TriArgs& ta, const double* u, double* x) {
  if (c->tri_dag) {
    HIPCHK(c, launch_tri_dag(c->st, ta, c->level_rows_d, c->n, c->nn_d, c->b, u, x, (long long)c->n * ta.stride,
                             c->tri_tmo_d, c->tri_rescue, c->tri_oversub));
    HIPCHK(c, hipMemcpyAsync(c->tri_tmo_h, c->tri_tmo_d, sizeof(unsigned), hipMemcpyDeviceToHost, c->st));
    return NNGP_OK;
  }
  for (size_t k = 0; k + 2 < c->tri_seg.size(); k += 3) {
    const int lv0 = c->tri_seg[k], lv1 = c->tri_seg[k + 1];
    if (c->tri_seg[k + 2]) {
      HIPCHK(c, launch_tri_levels_block(c->st, ta, c->level_rows_d, c->level_ptr_d, lv0, lv1, c->nn_d, c->b, u, x));
    } else {
      const int a = c->level_ptr[lv0], e = c->level_ptr[lv1];
      if (e > a) HIPCHK(c, launch_tri_level(c->st, ta, c->level_rows_d + a, e - a, c->nn_d, c->b, u, x));
    }
  }
  return NNGP_OK;
}

// after a host sync: did a sync-free solve since the last check time out?
// (its unfinished entries are NaN)
static int tri_timeout_check(nngp_ctx* c) {
  if (c->tri_tmo_h && *c->tri_tmo_h) {
    *c->tri_tmo_h = 0;
    HIPCHK(c, hipMemsetAsync(c->tri_tmo_d, 0, sizeof(unsigned), c->st));
    return fail_msg(c, NNGP_ERR_HIP, "triangular solve: a dependency wait timed out (waves not co-resident?)");
  }
  return NNGP_OK;
}

int nngp_tri_rescues(nngp_ctx* c, long long* out) {
  if (!c || !out) return NNGP_ERR_ARG;
  *out = 0;
  if (!c->tri_tmo_d) return NNGP_OK;
  int rc;
  if ((rc = set_device(c))) return rc;
  unsigned w[6];
  HIPCHK(c, hipMemcpyAsync(w, c->tri_tmo_d, sizeof w, hipMemcpyDeviceToHost, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  *out = (long long)w[4] + (w[1] == 1u ? 1 : 0);
  return NNGP_OK;
}

static TriArgs tri_one(const double* linv) {
  TriArgs ta;
  std::memset(&ta, 0, sizeof ta);
  ta.linv[0] = linv;
  ta.kidx[0] = 0;
  ta.nc = 1;
  ta.stride = 1;
  return ta;
}

int nngp_ancillary_propose(nngp_ctx* c, double beta0, double dlog_scale) {
  if (!c) return NNGP_ERR_ARG;
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  ChainState& S = c->ch[c->cur];
  if (!S.have_factor[0] || !S.have_factor[1] || !S.have_field)
    return fail_msg(c, NNGP_ERR_STATE, "ancillary_propose: need both factors and the field");
  int rc;
  if ((rc = set_device(c))) return rc;
  // tmp = B_cur (field - beta0)
  launch_row_stats(c->st, S.linv_d[0], c->nn_d, c->n, c->b, S.field_d, beta0, c->tmp_d, c->partials_d);
  HIPCHK(c, hipGetLastError());
  if ((rc = tri_solve_dev(c, tri_one(S.linv_d[1]), c->tmp_d, c->tmp2_d))) return rc;
  HIPCHK(c, launch_axpby_shift(c->st, c->n, c->tmp2_d, 1, std::exp(0.5 * dlog_scale), beta0, S.field_prop_d));
  return NNGP_OK;  // stream-ordered: the proposal is read by the next call on this context
}

int nngp_ancillary_propose_chains(nngp_ctx* c, int chain_mask, const double* beta0, const double* dlog_scale) {
  if (!c || !beta0 || !dlog_scale || chain_mask <= 0 || chain_mask >= (1 << c->C)) return NNGP_ERR_ARG;
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  int rc;
  if ((rc = set_device(c))) return rc;
  TriArgs ta;
  std::memset(&ta, 0, sizeof ta);
  ta.stride = c->C;
  RowJobs J;
  J.out_stride = c->C;
  for (int k = 0; k < c->C; ++k) {
    if (!((chain_mask >> k) & 1)) continue;
    ChainState& S = c->ch[k];
    if (!S.have_factor[0] || !S.have_factor[1] || !S.have_field) {
      char buf[96];
      std::snprintf(buf, sizeof buf, "ancillary_propose_chains: chain %d needs both factors and the field", k);
      return fail_msg(c, NNGP_ERR_STATE, buf);
    }
    // tmp[d*C + k] = B_cur (field - beta0): every chain in one pass
    J.linv[J.M] = S.linv_d[0];
    J.x[J.M] = S.field_d;
    J.shift[J.M] = beta0[k];
    J.out[J.M] = c->tmp_d + k;
    J.res_slot[J.M] = k;
    J.mode[J.M] = 0;
    ++J.M;
    ta.linv[ta.nc] = S.linv_d[1];
    ta.kidx[ta.nc] = k;
    ++ta.nc;
  }
  launch_row_stats_jobs(c->st, J, c->nn_d, c->n, c->b, c->partials_d);
  HIPCHK(c, hipGetLastError());
  if ((rc = tri_solve_dev(c, ta, c->tmp_d, c->tmp2_d))) return rc;
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1)
      HIPCHK(c, launch_axpby_shift(c->st, c->n, c->tmp2_d + k, c->C, std::exp(0.5 * dlog_scale[k]), beta0[k],
                                   c->ch[k].field_prop_d));
  return NNGP_OK;  // stream-ordered
}

// data-term reductions (mode 1: the dnorm ratio of the proposal, mode 0:
// the sum of squared residuals) of the chains in mask into res_d[4k..]
static int obs_chains_enqueue(nngp_ctx* c, int mode, int chain_mask, const double* beta0, const double* lnv,
                              bool copy = true) {
  // every chain in one pass (per chain obs_enqueue's bits), totals at res_d[4k]
  ObsJobs J;
  RowJobs R;
  for (int k = 0; k < c->C; ++k) {
    if (!((chain_mask >> k) & 1)) continue;
    ChainState& S = c->ch[k];
    if (!S.have_field || !S.have_mu) return fail_msg(c, NNGP_ERR_STATE, "data term: need field and mu");
    J.mu[J.M] = S.mu_is_const ? nullptr : S.mu_d;
    J.beta0[J.M] = beta0[k];
    J.f[J.M] = S.field_d;
    J.fnew[J.M] = mode == 1 ? S.field_prop_d : nullptr;
    J.inv_2var[J.M] = mode == 1 ? 0.5 * std::exp(-lnv[k]) : 0.0;
    ++J.M;
    R.res_slot[R.M++] = k;
  }
  const int nb = launch_obs_reduce_jobs(c->st, mode, c->n_obs, c->y_d, c->lm_d, J, c->partials_d);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, launch_reduce4_jobs(c->st, R, c->partials_d, nb, c->res_d));
  if (copy) HIPCHK(c, hipMemcpyAsync(c->res_h, c->res_d, 4 * c->C * sizeof(double), hipMemcpyDeviceToHost, c->st));
  return NNGP_OK;
}

static int obs_chains(nngp_ctx* c, int mode, int chain_mask, const double* beta0, const double* lnv, double* out) {
  if (!c || !out || !beta0 || (mode == 1 && !lnv) || chain_mask <= 0 || chain_mask >= (1 << c->C))
    return NNGP_ERR_ARG;
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = obs_chains_enqueue(c, mode, chain_mask, beta0, lnv))) return rc;
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  if ((rc = tri_timeout_check(c))) return rc;  // the proposal field of a ratio comes from the solve
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) out[k] = c->res_h[4 * k];
  return NNGP_OK;
}

int nngp_field_response_ratio(nngp_ctx* c, double beta0, double lnv, double* ratio) {
  if (!c || !ratio) return NNGP_ERR_ARG;
  double b0[kMaxChains], l[kMaxChains], out[kMaxChains];
  b0[c->cur] = beta0;
  l[c->cur] = lnv;
  int rc = obs_chains(c, 1, 1 << c->cur, b0, l, out);
  if (!rc) *ratio = out[c->cur];
  return rc;
}

int nngp_field_response_ratio_chains(nngp_ctx* c, int chain_mask, const double* beta0, const double* lnv,
                                     double* ratio) {
  return obs_chains(c, 1, chain_mask, beta0, lnv, ratio);
}

// ---------------------------------------------------------------- MH steps
// A covariance proposal's factor and what its Metropolis-Hastings step
// computes with it, behind ONE host sync (the separate calls take two or
// three): the factors, then the step's reductions, are enqueued for every
// chain in the mask before the outcome of any factor is known; one copy
// brings the failure flags and the results back.  A chain whose proposal
// factor fails reports NNGP_ERR_CHOL and NaN results (what its step computed
// from that factor is discarded, and the caches do not see it); every other
// chain gets exactly the bits of the separate calls.

static int step_common(nngp_ctx* c, int chain_mask, int covfun, const double* covparms, int ncp, bool need_mu,
                       const char* what) {
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  int rc;
  if ((rc = set_device(c))) return rc;
  for (int k = 0; k < c->C; ++k) {
    if (!((chain_mask >> k) & 1)) continue;
    const ChainState& S = c->ch[k];
    if (!S.have_factor[0] || !S.have_field || (need_mu && !S.have_mu)) {
      char buf[128];
      std::snprintf(buf, sizeof buf, "%s: chain %d needs its current factor, the field%s", what, k,
                    need_mu ? " and mu" : "");
      return fail_msg(c, NNGP_ERR_STATE, buf);
    }
  }
  if ((rc = factor_enqueue_chains(c, chain_mask, 1, covfun, covparms, ncp))) return rc;
  // provisional until the flags are back (factor_outcomes settles it)
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) c->ch[k].have_factor[1] = true;
  return NNGP_OK;
}

// an error after step_common's provisional marking: no masked chain keeps a
// proposal factor whose outcome was never settled (accept_factor refuses it)
static int step_abort(nngp_ctx* c, int chain_mask, int rc) {
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) c->ch[k].have_factor[1] = false;
  return rc;
}

static int step_collect(nngp_ctx* c, int chain_mask, int* status, int* failed) {
  HIPCHK(c, hipMemcpyAsync(c->res_h, c->res_d, kResBytes, hipMemcpyDeviceToHost, c->st));
  { int ss_ = sync_stream(c); if (ss_) return ss_; }
  int rc;
  if ((rc = tri_timeout_check(c))) return rc;
  rc = factor_outcomes(c, 1, chain_mask, status);
  if (rc && rc != NNGP_ERR_CHOL) return rc;
  *failed = 0;
  for (int k = 0; k < c->C; ++k)
    if (((chain_mask >> k) & 1) && status[k] != NNGP_OK) *failed |= 1 << k;
  return NNGP_OK;
}

int nngp_ancillary_step_chains(nngp_ctx* c, int chain_mask, int covfun, const double* covparms, int ncp,
                               const double* beta0, const double* dlog_scale, const double* lnv, int* status,
                               double* ratio) {
  if (!c || !covparms || !beta0 || !dlog_scale || !lnv || !status || !ratio || chain_mask <= 0 ||
      chain_mask >= (1 << c->C))
    return fail_msg(c, NNGP_ERR_ARG, "ancillary_step_chains: bad args");
  int rc, failed = 0;
  if ((rc = step_common(c, chain_mask, covfun, covparms, ncp, true, "ancillary_step_chains"))) return rc;
  if ((rc = nngp_ancillary_propose_chains(c, chain_mask, beta0, dlog_scale))) return step_abort(c, chain_mask, rc);
  if ((rc = obs_chains_enqueue(c, 1, chain_mask, beta0, lnv, false))) return step_abort(c, chain_mask, rc);
  if ((rc = step_collect(c, chain_mask, status, &failed))) return step_abort(c, chain_mask, rc);
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) ratio[k] = ((failed >> k) & 1) ? std::nan("") : c->res_h[4 * k];
  return NNGP_OK;
}

int nngp_sufficient_step_chains(nngp_ctx* c, int chain_mask, int covfun, const double* covparms, int ncp,
                                const double* beta0, const double* log_scale_prop, const double* log_scale_cur,
                                int* status, double* ll_prop, double* ll_cur) {
  if (!c || !covparms || !beta0 || !log_scale_prop || !log_scale_cur || !status || !ll_prop || !ll_cur ||
      chain_mask <= 0 || chain_mask >= (1 << c->C))
    return fail_msg(c, NNGP_ERR_ARG, "sufficient_step_chains: bad args");
  int rc, failed = 0;
  if ((rc = step_common(c, chain_mask, covfun, covparms, ncp, false, "sufficient_step_chains"))) return rc;
  // nngp_loglik_pair_chains' jobs: the proposals first, then the current factors
  LLJob jobs[kRowJobsMax];
  int nj = 0;
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) jobs[nj++] = {k, 1, beta0[k], log_scale_prop[k], ll_prop + k};
  for (int k = 0; k < c->C; ++k)
    if ((chain_mask >> k) & 1) jobs[nj++] = {k, 0, beta0[k], log_scale_cur[k], ll_cur + k};
  if ((rc = loglik_jobs_enqueue(c, jobs, nj, false))) return step_abort(c, chain_mask, rc);
  if ((rc = step_collect(c, chain_mask, status, &failed))) return step_abort(c, chain_mask, rc);
  loglik_jobs_finish(c, jobs, nj, failed);
  return NNGP_OK;
}

int nngp_accept_field(nngp_ctx* c) {
  if (!c) return NNGP_ERR_ARG;
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  int rc;
  if ((rc = set_device(c))) return rc;
  ChainState& S = c->ch[c->cur];
  S.fgen = ++c->gen;
  HIPCHK(c, hipMemcpyAsync(S.field_d, S.field_prop_d, c->n * sizeof(double), hipMemcpyDeviceToDevice, c->st));
  return NNGP_OK;  // stream-ordered: no host sync
}

int nngp_beta0_stats(nngp_ctx* c, double* oqo, double* oqf) {
  if (!c || !oqo || !oqf) return NNGP_ERR_ARG;
  { int rs_ = replica_fresh(c); if (rs_) return rs_; }
  ChainState& S = c->ch[c->cur];
  if (!S.have_factor[0] || !S.have_field) return fail_msg(c, NNGP_ERR_STATE, "beta0_stats: need factor and field");
  // a log-likelihood pass over the current factor and field already has
  // sum (B1)^2 and sum (B1)(B(f - shift)): (B1)'(Bf) = that + shift (B1)'(B1)
  for (const ChainState::RowStats& e : S.rs)
    if (e.lg == S.lgen[0] && e.fg == S.fgen) {
      *oqo = e.r[2];
      *oqf = e.r[3] + e.shift * e.r[2];
      return NNGP_OK;
    }
  int rc;
  if ((rc = set_device(c))) return rc;
  int nb = launch_row_stats(c->st, S.linv_d[0], c->nn_d, c->n, c->b, S.field_d, 0.0, nullptr, c->partials_d);
  HIPCHK(c, hipGetLastError());
  double r[4];
  if ((rc = fetch4(c, nb, r))) return rc;
  *oqo = r[2];
  *oqf = r[3];
  return NNGP_OK;
}

int nngp_sum_squared_residuals(nngp_ctx* c, double beta0, double* ssr) {
  if (!c || !ssr) return NNGP_ERR_ARG;
  double b0[kMaxChains], out[kMaxChains];
  b0[c->cur] = beta0;
  int rc = obs_chains(c, 0, 1 << c->cur, b0, nullptr, out);
  if (!rc) *ssr = out[c->cur];
  return rc;
}

int nngp_sum_squared_residuals_chains(nngp_ctx* c, int chain_mask, const double* beta0, double* ssr) {
  return obs_chains(c, 0, chain_mask, beta0, nullptr, ssr);
}

int nngp_spmv(nngp_ctx* c, int which, const double* X, int ncols, double* Y) {
  if (!c || !X || !Y || ncols < 0 || (which != 0 && which != 1)) return NNGP_ERR_ARG;
  ChainState& S = c->ch[c->cur];
  if (!S.have_factor[which]) return fail_msg(c, NNGP_ERR_STATE, "spmv: no factor");
  int rc;
  if ((rc = set_device(c))) return rc;
  std::vector<double> in(c->n), outv(c->n);
  for (int col = 0; col < ncols; ++col) {
    for (int i = 0; i < c->n; ++i) in[c->dpos[i]] = X[(size_t)col * c->n + i];
    HIPCHK(c, hipMemcpyAsync(c->tmp2_d, in.data(), c->n * sizeof(double), hipMemcpyHostToDevice, c->st));
    launch_row_stats(c->st, S.linv_d[which], c->nn_d, c->n, c->b, c->tmp2_d, 0.0, c->tmp_d, c->partials_d);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(outv.data(), c->tmp_d, c->n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    { int ss_ = sync_stream(c); if (ss_) return ss_; }
    for (int i = 0; i < c->n; ++i) Y[(size_t)col * c->n + i] = outv[c->dpos[i]];
  }
  return NNGP_OK;
}

int nngp_tri_solve(nngp_ctx* c, int which, const double* u, double* x) {
  if (!c || !u || !x || (which != 0 && which != 1)) return NNGP_ERR_ARG;
  ChainState& S = c->ch[c->cur];
  if (!S.have_factor[which]) return fail_msg(c, NNGP_ERR_STATE, "tri_solve: no factor");
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = upload_field(c, u, c->tmp_d))) return rc;
  if ((rc = tri_solve_dev(c, tri_one(S.linv_d[which]), c->tmp_d, c->tmp2_d))) return rc;
  if ((rc = download_field(c, c->tmp2_d, x))) return rc;
  return tri_timeout_check(c);
}

int nngp_device_normals(int device, uint64_t seed, uint64_t sweep, int n, double* z) {
  if (!z || n < 1) return NNGP_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail_msg(nullptr, NNGP_ERR_NODEV, "no HIP device");
  if (device < 0) device = 0;
  if (hipSetDevice(device) != hipSuccess) return NNGP_ERR_HIP;
  double* d = nullptr;
  if (hipMalloc((void**)&d, sizeof(double) * n) != hipSuccess) return NNGP_ERR_NOMEM;
  hipError_t e = launch_normals(nullptr, seed, sweep, n, d);
  if (e == hipSuccess) e = hipMemcpy(z, d, sizeof(double) * n, hipMemcpyDeviceToHost);
  hipFree(d);
  return e == hipSuccess ? NNGP_OK : fail_hip(nullptr, e, "device_normals");
}

}  // extern "C"
