// Tile-resident chromatic sweep (update_Gaussian.R:257-275):
// the persistent sweep_tiles_kernel, its launch wrappers, the tile shard's
// exchange kernels and the tile-layout value refresh (A5).  gfx950.
#include "kernels.h"
#include "device_common.h"
#include "graph_prep.h"

namespace nngp {

// ------------------------------------------------------------------ A1 (tiles)
// Tile-resident chromatic sweep: ONE persistent launch per call runs every
// sweep; workgroup t owns tile t (graph_prep.h TileLayout).  r of the tile's
// local rows (its own rows plus the foreign rows its columns touch) lives in
// LDS for the whole call, so the per-colour r traffic of the colour-launch
// engine (every launch re-reads / writes back almost every line of r) is gone;
// HBM carries only the B values, the per-slot records and the halo dw.
// Per colour c (epoch = sweep*K + c + 1):
//  1. own batches: cells (coalesced, non-temporal; the colour's first batch
//     was prefetched during the previous colour's hand-off) -> products
//     B[k,i] r_k with r_k from LDS -> running sums along each thread's
//     contiguous cells (restart at slot starts) -> per-thread tails in LDS ->
//     the thread holding a slot's last cell adds the tails of the threads the
//     slot spans (thread order: deterministic) -> the slot's thread draws w_i'
//     -> dw_i in LDS, and for a slot other tiles read, one 16-byte write-through
//     granule {dw_i, tag} (tag = call id << 32 | epoch) -> every cell scatters
//     r_k += B[k,i] dw_i in LDS (the rows of one colour are distinct);
//  2. the next colour's first batch is prefetched;
//  3. ghosts: every ghost cell (local row k, foreign slot j of colour c) reads
//     j's granule (sc1) until its tag is this call's epoch, then adds B[k,j]
//     dw_j to its local row.  The data is its own flag (MI355X_MICROARCH
//     "R2" granules): no drain, no flag store, no barrier before the read.
// Each row of B has at most one member of colour c, so steps 1 and 3 never
// update a row twice within a colour.  j's granule is rewritten one sweep
// later, after its owner has read granules of every tile reading j (they
// share the row, so each is the other's neighbour at its own colour), so no
// reader sees a later value; the call id (bumped on the device before every
// launch) keeps granules of earlier calls from matching.  Spins are bounded: a
// timeout sets ctl[1] and the launch drains (the host reports an error).
// the cell / slot encoding of the host layout (graph_prep.h), one definition
constexpr uint32_t kTPad = kTilePadRow;
constexpr uint32_t kTStart = kCellStart, kTEnd = kCellEnd;
constexpr int kTExported = kSlotExported;
constexpr int kTSlots = kTileSlotsMax;  // slots per own batch
static_assert(kTileQShift == kTileRowBits && kTileQMask + 1 >= (uint32_t)kTSlots && kTileRowBits + 11 <= 30,
              "cell_pk fields: local row | slot << kTileQShift | start << 30 | end << 31");
constexpr int kTSpreadLds = 82 * 1024;  // LDS floor: at most one tile per CU


typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// cell_pk on the device: the local-row field is stored XOR kTPad, so padding
// is 0 -- also what an out-of-range buffer load returns (capi.hip uploads it
// so).  Decoded at each use: a decode at the load would wait for the load.
__device__ __forceinline__ uint32_t tile_lr(uint32_t pk) { return (pk & kTPad) ^ kTPad; }



// dst[k] = p, in stream order (the current-factor table of captured graphs:
// the value travels as a kernel argument, no host buffer to keep alive)
__global__ void set_ptr_kernel(const double** dst, int k, const double* p) {
  if (threadIdx.x == 0) dst[k] = p;
}

hipError_t launch_set_ptr(hipStream_t st, const double** dst, int k, const double* p) {
  hipLaunchKernelGGL(set_ptr_kernel, dim3(1), dim3(64), 0, st, dst, k, p);
  return hipGetLastError();
}

// ctl: [0] call id, [1] the launch's timeout word (its tiles stop waiting once
// it is set), [2] the sticky copy the host reads: a timeout stays reported
// until the host has seen it (capi.hip tile_timeout_check clears it), however
// many launches follow before the next host sync
__global__ void tile_call_bump_kernel(unsigned* ctl) {
  ctl[0] += 1u;  // call id (never 0 inside a launch)
  ctl[1] = 0u;   // timeout word of this launch
}

__device__ __forceinline__ void tile_timeout_raise(unsigned* tmo) {
  __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(tmo + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tests (NNGP_TILE_INJECT_TIMEOUT=k: after each of the first k sweep calls of
// a context): what a launch whose tiles timed out leaves in ctl
__global__ void tile_inject_timeout_kernel(unsigned* ctl) { tile_timeout_raise(ctl + 1); }

hipError_t launch_tile_inject_timeout(hipStream_t st, unsigned* ctl) {
  hipLaunchKernelGGL(tile_inject_timeout_kernel, dim3(1), dim3(1), 0, st, ctl);
  return hipGetLastError();
}

hipError_t launch_tile_call_bump(hipStream_t st, unsigned* ctl) {
  hipLaunchKernelGGL(tile_call_bump_kernel, dim3(1), dim3(1), 0, st, ctl);
  return hipGetLastError();
}

// tile shard without RCCL: once this rank's own slots of w are in every
// peer's replica (peer copies ahead on the stream), lane h stores the call id
// into rank h's flag word `rank`; the wait polls this rank's flag words
// until every peer's carries the call id (bounded: the timeout word)
__global__ void tile_xsignal_kernel(TilePeerFlags pf, unsigned seq, int G, int rank) {
  const int h = threadIdx.x;
  __threadfence_system();
  if (h < G && h != rank) __hip_atomic_store(pf.f[h] + rank, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void tile_xwait_kernel(const unsigned* __restrict__ xflag, unsigned* ctl, unsigned seq, int G, int rank) {
  const int h = threadIdx.x;
  const unsigned call = seq;
  if (h < G && h != rank) {
    for (unsigned spins = 0;; ++spins) {
      if (__hip_atomic_load(xflag + h, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == call) break;
      if (spins > (1u << 22)) {
        tile_timeout_raise(ctl + 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
}

hipError_t launch_tile_xsignal(hipStream_t st, const TilePeerFlags& pf, unsigned seq, int G, int rank) {
  hipLaunchKernelGGL(tile_xsignal_kernel, dim3(1), dim3(64), 0, st, pf, seq, G, rank);
  return hipGetLastError();
}

hipError_t launch_tile_xwait(hipStream_t st, const unsigned* xflag, unsigned* ctl, unsigned seq, int G, int rank) {
  hipLaunchKernelGGL(tile_xwait_kernel, dim3(1), dim3(64), 0, st, xflag, ctl, seq, G, rank);
  return hipGetLastError();
}

// the rank's halo slots (read by other ranks' rows) into those ranks' w
// replicas: entry e of peer h's list (hptr[h] <= e < hptr[h+1]) is a slot
__global__ void tile_halo_put_kernel(TilePeerW pw, const int* __restrict__ halo, const double* __restrict__ w,
                                     int C) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= pw.hptr[kTileRanksMax]) return;
  int h = 0;
  while (e >= pw.hptr[h + 1]) ++h;
  const int x = halo[e];
  for (int ch = 0; ch < C; ++ch) pw.w[h][(size_t)x * C + ch] = w[(size_t)x * C + ch];
}

hipError_t launch_tile_halo_put(hipStream_t st, const TilePeerW& pw, const int* halo, const double* w, int C) {
  const int ne = pw.hptr[kTileRanksMax];
  if (ne == 0) return hipSuccess;
  hipLaunchKernelGGL(tile_halo_put_kernel, dim3((ne + 255) / 256), dim3(256), 0, st, pw, halo, w, C);
  return hipGetLastError();
}

// granule cache policy: sc1 (device scope: the producer's write-through store,
// the consumer's L2-bypassing poll, coherent across the XCDs); tile shard:
// sc0|sc1 (system scope) for the stores into other ranks' buffers and the
// polls, which see draws arriving from peer GPUs over xGMI
constexpr int kGranAux = 16, kGranAuxSys = 17;

// registers of one own batch: this thread's cells (f = t*R + j) and its draw
// items u = t + k*NT < nslots*C (slot q = u / C, chain u % C: per-slot
// records of consecutive items are consecutive, the loads coalesce).  Item
// fields hold the raw records after tile_load_batch and the draw scalars
// after tile_prep_items (in place: two batches stay in registers).
template <int C, int NT, int RMAX>
struct TileBatchRegs {
  // slots of a batch: NT == 64 is a wave-local batch (TileLayout::W), at most
  // kWaveSlotsMax slots; otherwise a workgroup's, at most kTSlots
  static constexpr int SMAX = NT == 64 ? kWaveSlotsMax : kTSlots;
  static constexpr int IMAX = (SMAX * C + NT - 1) / NT;
  int R, ns, x0;
  uint32_t rm[IMAX];          // tile shard: remote readers of the slot
  uint32_t pk[RMAX];
  double v[RMAX][C];
  int nobs[IMAX], flag[IMAX], loc[IMAX];
  double a0[IMAX], a1[IMAX];  // raw: precision_diag, residuals_sum; prepped: cR, 1/P
  double w[IMAX], zs[IMAX];   // w; prepped: z / sqrt(P)
};

// index of item u (= slot-in-batch q x C + chain) of the batch at slot x0 in
// the per-slot x chain arrays (dr, w_slot, granules).  CS = their chain
// stride: C, or (chain-split launches: one chain per workgroup, C = 1) the
// context's chain count, the chain's offset folded into the pointers
template <int C, int CS>
__device__ __forceinline__ size_t tile_xu(int x0, int u) {
  if constexpr (CS == C) {
    return (size_t)x0 * C + u;
  } else {
    const int q = u / C;
    return (size_t)(x0 + q) * CS + (u - q * C);
  }
}

// the batch's per-slot records (the draw preparation waits for them)
template <int C, int NT, int RMAX, int SH, int CS = C>
__device__ __forceinline__ void tile_load_items(const TileDev& D, const int4 B, TileBatchRegs<C, NT, RMAX>& b, int t) {
  b.ns = B.z; b.x0 = B.w;
#pragma unroll
  for (int k = 0; k < TileBatchRegs<C, NT, RMAX>::IMAX; ++k) {
    const int u = t + k * NT;
    if (u < b.ns * C) {
      const int q = u / C;
      const size_t xu = tile_xu<C, CS>(b.x0, u);  // = (x0 + q) * CS + chain
      const int2 si = D.sinfo[b.x0 + q];
      b.nobs[k] = si.x;
      b.flag[k] = si.y;
      b.loc[k] = D.slot_loc[b.x0 + q];
      if (SH) b.rm[k] = D.rmask[b.x0 + q];
      const double2 dr = D.dr[xu];
      b.a0[k] = dr.x;
      b.a1[k] = dr.y;
      b.w[k] = D.w_slot[xu];
    }
  }
}

// the batch's cells: thread t's run f = t*R + j sits at off + j*NT + t
template <int C, int NT, int RMAX>
__device__ __forceinline__ void tile_load_cells(const TileDev& D, const int4 B, TileBatchRegs<C, NT, RMAX>& b, int t) {
  b.R = B.y & 0xFFFF;
  const bool live = t < (B.y >> 16);  // threads past nthr hold padding only: no load
#pragma unroll
  for (int j = 0; j < RMAX; ++j) {
    if (j < b.R && live) {
      const long long e = B.x + (long long)j * NT + t;
      b.pk[j] = __builtin_nontemporal_load(D.cell_pk + e);
#pragma unroll
      for (int ch = 0; ch < C; ++ch) b.v[j][ch] = __builtin_nontemporal_load(D.cell_val + ch * D.n_cells + e);
    } else {
      // padding (device encoding, tile_lr); where the products run whole
      // groups of cells (tile_products: wave-local batches) with a
      // zero value, so that a cell past R is a no-op there (the tile's last
      // row times 0)
      b.pk[j] = 0u;
      if constexpr (NT == 64) {
#pragma unroll
        for (int ch = 0; ch < C; ++ch) b.v[j][ch] = 0.0;
      }
    }
  }
}

template <int C, int NT, int RMAX, int SH, int CS = C>
__device__ __forceinline__ void tile_load_batch(const TileDev& D, const int4 B, TileBatchRegs<C, NT, RMAX>& b, int t) {
  tile_load_items<C, NT, RMAX, SH, CS>(D, B, b, t);
  tile_load_cells<C, NT, RMAX>(D, B, b, t);
}

// everything of the Gibbs draw but acc: P = D/s2 + n/t2, w' = (cR - acc/s2)/P
// + z/sqrt(P) with cR = R/t2 + D w/s2 (w of an own slot is constant until its
// colour, so this runs a colour ahead, during the previous hand-off)
template <int C, int NT, int RMAX, int CS = C>
__device__ __forceinline__ void tile_prep_items(const TileDev& D, const TileLaunch& a, const double* sc_s,
                                                const unsigned long long* seed_s, int s,
                                                TileBatchRegs<C, NT, RMAX>& b, int t, int var = 0) {
#pragma unroll
  for (int k = 0; k < TileBatchRegs<C, NT, RMAX>::IMAX; ++k) {
    const int u = t + k * NT;
    if (u < b.ns * C) {
      const int q = u / C, ch = u - q * C;
      const double inv_s2 = sc_s[2 * ch], inv_t2 = sc_s[2 * ch + 1];
      double z = 0.0;
      // var (NNGP_TILE_VARIANT, probe timing experiments only, wrong results):
      // 2 = no normals, 4 = no records
      if (var & 2) z = 0.0;
      else if (a.z_in) z = a.z_in[((size_t)s * D.n + b.x0 + q) * CS + ch];
      else z = normal_loc(seed_s[2 * ch], seed_s[2 * ch + 1] + s, (uint32_t)b.loc[k]);
      const double a0 = (var & 4) ? 1.0 : b.a0[k], a1 = (var & 4) ? 0.5 : b.a1[k], wk = (var & 4) ? 0.0 : b.w[k];
      const double P = a0 * inv_s2 + (double)((var & 4) ? 1 : b.nobs[k]) * inv_t2;
      const double cR = inv_t2 * a1 + inv_s2 * (a0 * wk);
      // 1/sqrt(P) once (hardware rsq + Newton) for both 1/P and z/sqrt(P):
      // a few instructions instead of a square root and two divisions on the
      // cell waves' path (within ~2 ulp of them)
      const double rs = rsqrt_pos(P);
      b.a0[k] = cR;
      b.a1[k] = rs * rs;
      b.zs[k] = z * rs;
    }
  }
}

// ghost cells of one chunk: local row, foreign slot, B values
template <int C, int GMAX>
struct TileGhostRegs {
  int lr[GMAX], gx[GMAX];
  double gv[GMAX][C];
};

template <int C, int NT, int GMAX>
__device__ __forceinline__ void tile_load_ghosts(const TileDev& D, int gb, int g1, TileGhostRegs<C, GMAX>& g, int t) {
#pragma unroll
  for (int k = 0; k < GMAX; ++k) {
    const int e = gb + k * NT + t;
    g.lr[k] = -1;
    if (e < g1) {
      const long long raw = __builtin_nontemporal_load(reinterpret_cast<const long long*>(D.gcell) + e);
      g.lr[k] = (int)(raw & 0xFFFFFFFFll);
      g.gx[k] = (int)(raw >> 32);
#pragma unroll
      for (int ch = 0; ch < C; ++ch) g.gv[k][ch] = __builtin_nontemporal_load(D.gval + ch * D.n_gcells + e);
    }
  }
}

// ghost adds of one register pass: r_k += B[k,j] dw_j.  The rows are
// distinct (one foreign member per colour per row), so every read goes out
// before any write (see tile_own_scatter)
struct TileState;
template <int C, int GMAX>
__device__ __forceinline__ void tile_ghost_adds(TileState& S, const TileGhostRegs<C, GMAX>& gr);

// per-workgroup state of the persistent sweep
struct TileState {
  double* r_s;
  double* acc_s;
  double* wsum;
  double* sc_s;   // C x {inv_s2, inv_t2}
  unsigned long long* seed_s;  // C x {seed, counter_base}
  double* dsh_s;  // C: the call's beta_0 shift of each chain (SweepScalars::dshift; sweep 0's w)
  int4* batch_s;  // this tile's own batches
  int* bptr_s;    // K+1: batches of colour c = batch_s[bptr_s[c] .. bptr_s[c+1])
  int* gptr_s;    // K+1: ghost cells of colour c (global indices)
  int* gsp_s;     // K+1: foreign slots of colour c (global indices into gslot)
  int* bsp_s;     // K: split layouts, first boundary batch of colour c (as bptr_s)
  double* gdw_s;  // foreign slots x C: their dw of the current colour
  int* wflag;
  unsigned* spin_s;
  int* pub_s;     // wave-local tiles: the last phase whose first own batch has drawn (wave 0; hand-off poll gate)
  __amdgpu_buffer_rsrc_t gran;
  unsigned call;
  int gsl;                          // this phase's first foreign slot index of the thread (loaded a phase ahead)
  unsigned* tmo;
  int G;                            // tile shard: ranks (1: single GPU)
  bool timed_out;
  int T, t, lane, wv, K, nph, ph;
  uint32_t lrmax;                   // the tile's last local row (padding cells read it, times a zero value)
  unsigned long long tp[8], t_prev;
};

template <int C, int GMAX>
__device__ __forceinline__ void tile_ghost_adds(TileState& S, const TileGhostRegs<C, GMAX>& gr) {
  double rv[GMAX][C], dv[GMAX][C];
#pragma unroll
  for (int k = 0; k < GMAX; ++k) {
    const bool ok = gr.lr[k] >= 0;
    const int row = ok ? gr.lr[k] : 0, x = ok ? gr.gx[k] : 0;
#pragma unroll
    for (int ch = 0; ch < C; ++ch) {
      rv[k][ch] = S.r_s[row * C + ch];
      dv[k][ch] = S.gdw_s[x * C + ch];
    }
  }
#pragma unroll
  for (int k = 0; k < GMAX; ++k)
    if (gr.lr[k] >= 0)
#pragma unroll
      for (int ch = 0; ch < C; ++ch) S.r_s[gr.lr[k] * C + ch] = rv[k][ch] + gr.gv[k][ch] * dv[k][ch];
}

#define TSTAMP(S, k)                                                      \
  do {                                                                    \
    if (PROBE == 1) {                                                          \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");         \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();   \
      if ((k) >= 0) (S).tp[(k) < 0 ? 0 : (k)] += now_ - (S).t_prev;       \
      (S).t_prev = now_;                                                  \
    }                                                                     \
  } while (0)

// NNGP_PROBE=2 timeline: thread 0 of every tile stores the 100 MHz clock at
// points k of phase S.ph (no waits added besides the clock read's own)
constexpr int kTimelinePhases = 512;
constexpr int kTimelineSlots = 16;  // stamps per phase (capi.hip allocates T x phases x slots)
#define TLSTAMP(S, k)                                                                         \
  do {                                                                                        \
    if (PROBE == 2 && (S).t == 0 && (S).ph < kTimelinePhases)                                 \
      D.dbg[((size_t)(S).T * kTimelinePhases + (S).ph) * kTimelineSlots + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// (wave-local tiles: slot 9 + w = wave w's last publish of the phase, so the
// host can tell the neighbours' skew from the hand-off's transit; the dump
// appends the neighbour lists, scripts/timeline.py)


// one step of a segmented inclusive scan (flag f = "a segment starts here or
// in an earlier lane of my partial"): (f_e, v_e) (+) (f, v) = (f_e | f, f ? v : v_e + v)
// (v = fma(e, keep, v) with keep = f ? 0 : 1 is bitwise the select of
// e + v and v -- round(e * 1 + v) = round(e + v), e * 0 + v = v for the
// finite e of a scan -- in one instruction instead of an add and two
// 32-bit selects per chain)
template <int CTRL, int RM, bool BC, int C>
__device__ __forceinline__ void seg_scan_step(double (&v)[C], int& f) {
  double e[C];
#pragma unroll
  for (int ch = 0; ch < C; ++ch) e[ch] = dpp_f64<CTRL, RM, BC>(v[ch]);
  const int fe = __builtin_amdgcn_update_dpp(0, f, CTRL, RM, 0xF, BC);
  const double keep = f ? 0.0 : 1.0;
#pragma unroll
  for (int ch = 0; ch < C; ++ch) v[ch] = __builtin_fma(e[ch], keep, v[ch]);
  f |= fe;
}

// one own batch of colour c (epoch): products -> slot totals -> draws ->
// scatter.  LDS and registers only, plus the draws' stores: no global load
// (a load here would wait behind the next batch's prefetch, vmcnt is in order).
// Workgroup barriers inside it: kOwnDrawBarriers -- the exchange wave, which
// holds no cells, passes exactly as many per batch (tile_phase_xw); a barrier
// added or removed here must change this count.
constexpr int kOwnDrawBarriers = 3;
// the products of one own batch: running sums over a thread's cells,
// restarted at slot starts (run * keep + p, keep in {0, 1}: see
// seg_scan_step), every slot end stored into acc_s; cont_q = the slot this
// thread continues from earlier threads (completed after the scan).  The r
// reads of a group of GRP cells go out together, before any of its
// arithmetic: one LDS round trip per group instead of one or two per cell
// (the per-cell `j < R` blocks kept each cell's reads behind the previous
// cell's).  Cells past R are padding with a zero value (tile_load_cells), so
// the last group runs whole; padding reads the tile's last row.  Wave-local
// batches only (tile_own_wl); tile_own_draw keeps its cell-by-cell loop (the
// group's registers spill its 2-chain instantiation)
template <int C, int RMAX, int GRP, class TB>
__device__ __forceinline__ void tile_products(const TB& b, int R, const double* __restrict__ r_s,
                                              double* __restrict__ acc_s, uint32_t lrmax, double (&run)[C],
                                              int& cont_q, bool& seen_start) {
#pragma unroll
  for (int ch = 0; ch < C; ++ch) run[ch] = 0.0;
#pragma unroll
  for (int j0 = 0; j0 < RMAX; j0 += GRP) {
    if (j0 >= R) break;
    double rv[GRP][C];
#pragma unroll
    for (int jj = 0; jj < GRP; ++jj) {
      if (j0 + jj < RMAX) {
        const uint32_t lr = min(tile_lr(b.pk[j0 + jj]), lrmax);
#pragma unroll
        for (int ch = 0; ch < C; ++ch) rv[jj][ch] = r_s[lr * C + ch];
      }
    }
#pragma unroll
    for (int jj = 0; jj < GRP; ++jj) {
      const int j = j0 + jj;
      if (j < RMAX) {
        const uint32_t pk = b.pk[j];
        const bool st = (pk & kTStart) != 0;
        const double keep = st ? 0.0 : 1.0;
#pragma unroll
        for (int ch = 0; ch < C; ++ch) run[ch] = __builtin_fma(run[ch], keep, b.v[j][ch] * rv[jj][ch]);
        const int q = (int)((pk >> kTileQShift) & kTileQMask);
        if (pk & kTEnd) {
#pragma unroll
          for (int ch = 0; ch < C; ++ch) acc_s[q * C + ch] = run[ch];
        }
        seen_start |= st;  // (before the end test: a slot may start and end at this cell)
        cont_q = ((pk & kTEnd) && !seen_start && cont_q < 0) ? q : cont_q;
      }
    }
  }
}

template <int C, int NT, int RMAX, int PROBE, int SH, int CS = C>
__device__ __forceinline__ void tile_own_draw(const TileDev& D, const TileLaunch& a, const TileShard& sh, TileState& S,
                                              TileBatchRegs<C, NT, RMAX>& b, unsigned epoch) {
  constexpr int IMAX = TileBatchRegs<C, NT, RMAX>::IMAX;
  const int t = S.t, lane = S.lane, wv = S.wv;
  // r (the tile's rows) and acc_s (slot totals, then dw) are disjoint LDS
  // regions: restrict lets the products' r reads go out ahead of the slot
  // totals written between them
  const double* __restrict__ r_s = S.r_s;
  double* __restrict__ acc_s = S.acc_s;
  const int R = b.R, nit = b.ns * C;
  // products, running sums restarted at slot starts.  A slot that began in
  // this thread is complete at its last cell (-> acc_s); the thread's first
  // cells may continue a slot of earlier threads: its end (if here) waits for
  // the carry of those threads.
  tile_cells_landed(b);
  // straight-line products as tile_own_wl's (padding reads the tile's last
  // row times a zero value; every slot end stores its run, the continued
  // slot of earlier threads completed after the scan)
  double run[C];
  int cont_q = -1;
  bool seen_start = false;
#pragma unroll
  for (int ch = 0; ch < C; ++ch) run[ch] = 0.0;
#pragma unroll
  for (int j = 0; j < RMAX; ++j) {
    if (j < R) {
      const uint32_t pk = b.pk[j];
      const uint32_t lr = min(tile_lr(pk), S.lrmax);
      const bool st = (pk & kTStart) != 0;
      const double keep = st ? 0.0 : 1.0;  // restart at a slot start: run * 0 + p (see seg_scan_step)
#pragma unroll
      for (int ch = 0; ch < C; ++ch) run[ch] = __builtin_fma(run[ch], keep, b.v[j][ch] * r_s[lr * C + ch]);
      const int q = (int)((pk >> kTileQShift) & kTileQMask);
      if (pk & kTEnd) {
#pragma unroll
        for (int ch = 0; ch < C; ++ch) acc_s[q * C + ch] = run[ch];
      }
      seen_start |= st;  // (before the end test: a slot may start and end at this cell)
      cont_q = ((pk & kTEnd) && !seen_start && cont_q < 0) ? q : cont_q;
    }
  }
  TSTAMP(S, 1);
  // segmented inclusive scan of the thread tails (restart at threads holding
  // a slot start): in the wave by shuffles, across waves through LDS
  // (DPP: row shifts 1, 2, 4, 8 inside each row of 16 lanes, then the row
  // broadcasts 15 and 31 -- no LDS round trips)
  double v[C];
  int f = seen_start ? 1 : 0;
#pragma unroll
  for (int ch = 0; ch < C; ++ch) v[ch] = run[ch];
  seg_scan_step<0x111, 0xF, true, C>(v, f);  // row_shr:1
  seg_scan_step<0x112, 0xF, true, C>(v, f);  // row_shr:2
  seg_scan_step<0x114, 0xF, true, C>(v, f);  // row_shr:4
  seg_scan_step<0x118, 0xF, true, C>(v, f);  // row_shr:8
  seg_scan_step<0x142, 0xA, false, C>(v, f); // row_bcast:15 -> rows 1, 3
  seg_scan_step<0x143, 0xC, false, C>(v, f); // row_bcast:31 -> rows 2, 3
  if (lane == 63) {
#pragma unroll
    for (int ch = 0; ch < C; ++ch) S.wsum[wv * C + ch] = v[ch];
    S.wflag[wv] = f;
  }
  __syncthreads();
  double in[C];
#pragma unroll
  for (int ch = 0; ch < C; ++ch) in[ch] = 0.0;
  for (int p = wv - 1; p >= 0; --p) {
#pragma unroll
    for (int ch = 0; ch < C; ++ch) in[ch] = S.wsum[p * C + ch] + in[ch];
    if (S.wflag[p]) break;
  }
#pragma unroll
  for (int ch = 0; ch < C; ++ch) {
    const double Sv = f ? v[ch] : v[ch] + in[ch];
    const double up = dpp_f64<0x138, 0xF, true>(Sv);  // wave_shr:1
    const double cp = lane ? up : in[ch];
    if (cont_q >= 0) acc_s[cont_q * C + ch] = acc_s[cont_q * C + ch] + cp;
  }
  __syncthreads();
  TSTAMP(S, 2);
#pragma unroll
  for (int k = 0; k < IMAX; ++k) {
    const int u = t + k * NT;
    if (u < nit) {
      const int ch = u % C;
      double dw = 0.0;
      const size_t xu = tile_xu<C, CS>(b.x0, u);
      if ((a.chain_mask >> ch) & 1) {
        const double wn = (b.a0[k] - S.sc_s[2 * ch] * acc_s[u]) * b.a1[k] + b.zs[k];
        dw = wn - b.w[k];
        D.w_slot[xu] = wn;
      }
      acc_s[u] = dw;
      if (b.flag[k] & kTExported) {
        const unsigned long long uu = __builtin_bit_cast(unsigned long long, dw);
        u32x4_t g;
        // {dw, epoch, call ^ dw_lo ^ dw_hi}: one 16-B write-through store.  The
        // tag word also checks the payload, so a torn read (new tag, old dw --
        // not observed on gfx950, not architecturally excluded) is not taken
        g.x = (unsigned)uu; g.y = (unsigned)(uu >> 32); g.z = epoch; g.w = S.call ^ g.x ^ g.y;
        __builtin_amdgcn_raw_buffer_store_b128(g, S.gran, (int)(xu * 16), 0, SH ? kGranAuxSys : kGranAux);
        if (SH) {
          // the same granule into the buffer of every other rank with a reader
#pragma unroll
          for (int h = 0; h < kTileRanksMax; ++h)
            if (h < S.G && ((b.rm[k] >> h) & 1u))
              __builtin_amdgcn_raw_buffer_store_b128(
                  g, __builtin_amdgcn_make_buffer_rsrc(sh.gx[h], 0, 0x7FFFFFFF, 0x00020000), (int)(xu * 16), 0,
                  kGranAuxSys);
        }
      }
    }
  }
  __syncthreads();
  TSTAMP(S, 3);
  TLSTAMP(S, 1);
}

// ... and its scatter r_k += B[k,i] dw_i (dw in acc_s).  Needs only the
// batch's cells: its per-slot records may be overwritten by then.
// The rows of a batch's cells are distinct (one member per colour per row),
// so the reads of r and dw of a group of rows all go out before any write:
// one LDS round trip per group instead of one per cell (the compiler cannot
// see the distinctness and would order every read after the previous write)
template <int C, int NT, int RMAX, int PROBE>
__device__ __forceinline__ void tile_own_scatter(TileState& S, const TileBatchRegs<C, NT, RMAX>& b, int R,
                                                 const double* acc_base = nullptr) {
  constexpr int GRP = RMAX < 4 ? RMAX : 4;  // rows per group (registers: 2 x GRP x C doubles)
  double* r_s = S.r_s;
  const double* acc_s = acc_base ? acc_base : S.acc_s;
#pragma unroll
  for (int j0 = 0; j0 < RMAX; j0 += GRP) {
    if (j0 >= R) break;
    double rv[GRP][C], dv[GRP][C];
#pragma unroll
    for (int jj = 0; jj < GRP; ++jj) {
      const int j = j0 + jj;
      const uint32_t lr = tile_lr(b.pk[j]);
      const bool ok = j < R && lr != kTPad;
      const int row = ok ? (int)lr : 0, q = ok ? (int)((b.pk[j] >> kTileQShift) & kTileQMask) : 0;
#pragma unroll
      for (int ch = 0; ch < C; ++ch) {
        rv[jj][ch] = r_s[row * C + ch];
        dv[jj][ch] = acc_s[q * C + ch];
      }
    }
#pragma unroll
    for (int jj = 0; jj < GRP; ++jj) {
      const int j = j0 + jj;
      const uint32_t lr = tile_lr(b.pk[j]);
      if (j < R && lr != kTPad) {
#pragma unroll
        for (int ch = 0; ch < C; ++ch) r_s[lr * C + ch] = rv[jj][ch] + b.v[j][ch] * dv[jj][ch];
      }
    }
  }
  TSTAMP(S, 4);
}

// every cell register of the batch in place: the one wait for the batch's
// loads goes here, where they have landed, instead of wherever a later
// conditional use makes the compiler wait conservatively (vmcnt counts a
// wave's loads in order: such a wait would cover every load issued since)
template <int C, int NT, int RMAX>
__device__ __forceinline__ void tile_cells_landed(const TileBatchRegs<C, NT, RMAX>& b) {
#pragma unroll
  for (int j = 0; j < RMAX; ++j) {
    asm volatile("" ::"v"(b.pk[j]));
#pragma unroll
    for (int ch = 0; ch < C; ++ch) asm volatile("" ::"v"(b.v[j][ch]));
  }
}

// one colour phase ph = sweep*K + c with `cur` holding its prepared first
// batch.  Double-buffered (DB): the next phase's first batch is loaded into
// `nxt` at the start (its HBM stream overlaps this colour's work); otherwise
// after the own work, before the hand-off.  (Measured and dropped, see
// the normals pregenerated by a separate kernel -- no Philox here,
// 132 instead of 255 VGPRs at 1 chain --, double buffering at 3 chains, an L2
// prefetch of the next stream during the own work, other load orders.)
template <int C, int NT, int RMAX, int GMAX, int DB, int PROBE, int SH, int CS = C>
__device__ __forceinline__ void tile_phase(const TileDev& D, const TileLaunch& a, const TileShard& sh, TileState& S, int ph,
                                           TileBatchRegs<C, NT, RMAX>& cur, TileBatchRegs<C, NT, RMAX>& nxt,
                                           TileGhostRegs<C, GMAX>& gr, TileGhostRegs<C, GMAX>& grn) {
  const int K = S.K, t = S.t;
  const int s = ph / K, c = ph - s * K;
  const unsigned epoch = (unsigned)ph + 1;
  S.ph = ph;
  TLSTAMP(S, 0);
  const int phn = ph + 1;
  const int cn = phn % K, sn = phn / K;
  const bool has_next = phn < S.nph;
  const bool more = has_next && S.bptr_s[cn] < S.bptr_s[cn + 1];
  const int bfirst = S.bptr_s[c], bend = S.bptr_s[c + 1];
  const int g0 = S.gptr_s[c], g1 = S.gptr_s[c + 1];
  const int gn0 = S.gptr_s[cn], gn1 = S.gptr_s[cn + 1];
  // this colour's foreign slots (one granule per slot and chain): the first
  // NT items' slot indices load now, behind the own work
  const int gs0 = S.gsp_s[c], nfi = (S.gsp_s[c + 1] - gs0) * C;
  // loaded during the previous phase's hand-off: a load issued here would be
  // waited for behind the draw's (conditional) stores before the first poll
  // (double-buffered: at the phase start, measured faster at 1 chain)
  const int gsl_pref = DB ? (t < nfi ? D.gslot[gs0 + t / C] : 0) : S.gsl;
  if (DB) {
    // the next colour's first batch (and ghost chunk): their HBM stream
    // overlaps this colour's work (two register sets)
    if (more) tile_load_batch<C, NT, RMAX, SH, CS>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
    if (has_next && gn1 > gn0) tile_load_ghosts<C, NT, GMAX>(D, gn0, gn1, grn, t);
  }
  // ---- 1. own batches.  One register set (!DB): after the draw of the last
  // batch, the next colour's per-slot records, this colour's ghost cells and
  // the first poll of its granules go out before the scatter (the draw's
  // records are dead, the scatter needs only the cells), the next cells
  // after it
  const bool pol = t < nfi;
  u32x4_t gfirst;
  for (int bi = bfirst; bi < bend; ++bi) {
    if (bi != bfirst) {  // rare: a colour with more than one batch in this tile
      __syncthreads();   // acc_s is indexed by slot-in-batch: every wave is done with the last batch
      tile_load_batch<C, NT, RMAX, SH, CS>(D, S.batch_s[bi], cur, t);
      tile_prep_items<C, NT, RMAX, CS>(D, a, S.sc_s, S.seed_s, s, cur, t);
    }
    tile_own_draw<C, NT, RMAX, PROBE, SH, CS>(D, a, sh, S, cur, epoch);
    const int R = cur.R;
    if (!DB && bi + 1 == bend) {
      if (more) tile_load_items<C, NT, RMAX, SH, CS>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
      if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
      if (pol) gfirst = __builtin_amdgcn_raw_buffer_load_b128(S.gran, (int)(((size_t)gsl_pref * CS + t % C) * 16), 0, SH ? kGranAuxSys : kGranAux);
    }
    tile_own_scatter<C, NT, RMAX, PROBE>(S, cur, R);
  }
  TLSTAMP(S, 6);
  // ---- 2. the next colour's cells (one register set), the next batch's
  // draw scalars, then (two register sets) the first poll
  if (!DB) {
    if (bend == bfirst) {  // no own batch of this colour in the tile
      if (more) tile_load_items<C, NT, RMAX, SH, CS>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
      if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
      if (pol) gfirst = __builtin_amdgcn_raw_buffer_load_b128(S.gran, (int)(((size_t)gsl_pref * CS + t % C) * 16), 0, SH ? kGranAuxSys : kGranAux);
    }
    // the next batch's draw scalars before its cells go out: the cells' loads
    // are conditional (rows past R), so a wait for the records issued before
    // them would also wait for every cell
    if (more) tile_prep_items<C, NT, RMAX, CS>(D, a, S.sc_s, S.seed_s, sn, nxt, t);
    if (more) tile_load_cells<C, NT, RMAX>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
  } else if (more) {
    tile_prep_items<C, NT, RMAX, CS>(D, a, S.sc_s, S.seed_s, sn, nxt, t);
  }
  if (DB && pol) gfirst = __builtin_amdgcn_raw_buffer_load_b128(S.gran, (int)(((size_t)gsl_pref * CS + t % C) * 16), 0, SH ? kGranAuxSys : kGranAux);
  TSTAMP(S, 5);
  TLSTAMP(S, 4);
  if (!DB) {  // the next phase's first foreign slot indices (complete once the polls below have waited)
    const int gn = S.gsp_s[cn], nfn = has_next ? (S.gsp_s[cn + 1] - gn) * C : 0;
    S.gsl = t < nfn ? D.gslot[gn + t / C] : 0;
  }
  // ---- 3. hand-off: the granule of each (foreign slot, chain) of this colour
  // until it carries this epoch -> gdw_s; then every ghost cell adds B[k,j]
  // dw_j to its local row (a slot read by several rows of the tile is fetched
  // once)
  for (int u0 = 0; u0 < nfi; u0 += NT) {
    const int u = u0 + t;
    if (u < nfi) {
      const int x = u0 == 0 ? gsl_pref : D.gslot[gs0 + u / C];
      const int ch = u % C;
      const int off = (int)(((size_t)x * CS + ch) * 16);
      u32x4_t g = u0 == 0 ? gfirst : __builtin_amdgcn_raw_buffer_load_b128(S.gran, off, 0, SH ? kGranAuxSys : kGranAux);
      double dw = 0.0;
      for (unsigned spins = 0;; ++spins) {
        if (g.z == epoch && (g.w ^ g.x ^ g.y) == S.call) {
          dw = __builtin_bit_cast(double, (unsigned long long)g.x | ((unsigned long long)g.y << 32));
          if (PROBE == 2) atomicMax(S.spin_s, spins);
          break;
        }
        // bounded wait (about a second per poll); once any tile of the launch
        // has given up (timeout word), the others stop waiting within ~1k polls
        if (S.timed_out || spins > (1u << 20) ||
            ((spins & 1023u) == 1023u && __hip_atomic_load(S.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          if (!S.timed_out) tile_timeout_raise(S.tmo);
          S.timed_out = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        g = __builtin_amdgcn_raw_buffer_load_b128(S.gran, off, 0, SH ? kGranAuxSys : kGranAux);
      }
      S.gdw_s[u] = dw;
    }
  }
  __syncthreads();
  TLSTAMP(S, 2);
  if (PROBE == 2 && t == 0 && S.ph < kTimelinePhases) {
    D.dbg[((size_t)S.T * kTimelinePhases + S.ph) * kTimelineSlots + 5] = *S.spin_s;
    *S.spin_s = 0;
  }
  for (int gb = g0; gb < g1; gb += NT * GMAX) {
    if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, gr, t);
    tile_ghost_adds<C, GMAX>(S, gr);
  }
  // ---- 4. the next batch's draw scalars (registers only: no barrier needed
  // before them; the barrier below orders the ghost adds before the products)
  __syncthreads();
  TSTAMP(S, 6);
  TLSTAMP(S, 3);
}

// One colour phase of a SPLIT layout (one register set, C >= 3): the
// interior batches of colour c -- slots whose rows have no member of colour
// c-1 owned by another tile -- go first, while the granules of colour c-1
// are still in flight; then that hand-off (poll, ghost cells of c-1); then
// the boundary batches of c.  The chain from a neighbour's draw to this
// tile's next draw runs through the few boundary slots only; the interior
// work covers the hand-off latency.  Per row the updates of c and c-1 may
// land in the other order than in the colour-by-colour schedule (rounding
// only: an interior slot never reads a row waiting for its c-1 update).
template <int C, int NT, int RMAX, int GMAX, int PROBE, int SH>
__device__ __forceinline__ void tile_phase_ib(const TileDev& D, const TileLaunch& a, const TileShard& sh, TileState& S,
                                              int ph, TileBatchRegs<C, NT, RMAX>& cur, TileGhostRegs<C, GMAX>& gr) {
  const int K = S.K, t = S.t;
  const int s = ph / K, c = ph - s * K;
  const unsigned epoch = (unsigned)ph + 1;
  S.ph = ph;
  TLSTAMP(S, 0);
  const int phn = ph + 1;
  const int cn = phn % K, sn = phn / K;
  const bool has_next = phn < S.nph;
  const bool more = has_next && S.bptr_s[cn] < S.bptr_s[cn + 1];
  const int bfirst = S.bptr_s[c], bsplit = S.bsp_s[c], bend = S.bptr_s[c + 1];
  const bool had_int = bsplit > bfirst, had_bnd = bend > bsplit;
  // the hand-off of the previous colour (none at the first phase of a call)
  const bool hp = ph > 0;
  const int cp = hp ? (ph - 1) % K : 0;
  const int g0 = S.gptr_s[cp], g1 = hp ? S.gptr_s[cp + 1] : g0;
  const int gs0 = S.gsp_s[cp], nfi = hp ? (S.gsp_s[cp + 1] - gs0) * C : 0;
  const int gsl_pref = t < nfi ? D.gslot[gs0 + t / C] : 0;
  const bool pol = t < nfi;
  u32x4_t gfirst;
  // ---- 1. interior batches; after the last draw (records dead) the next
  // batch's records, the hand-off's ghost cells and first poll go out
  for (int bi = bfirst; bi < bsplit; ++bi) {
    if (bi != bfirst) {
      __syncthreads();
      tile_load_batch<C, NT, RMAX, SH>(D, S.batch_s[bi], cur, t);
      tile_prep_items<C, NT, RMAX>(D, a, S.sc_s, S.seed_s, s, cur, t);
    }
    tile_own_draw<C, NT, RMAX, PROBE, SH>(D, a, sh, S, cur, epoch);
    const int R = cur.R;
    if (bi + 1 == bsplit) {
      if (had_bnd) tile_load_items<C, NT, RMAX, SH>(D, S.batch_s[bsplit], cur, t);
      else if (more) tile_load_items<C, NT, RMAX, SH>(D, S.batch_s[S.bptr_s[cn]], cur, t);
      if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
      if (pol) gfirst = __builtin_amdgcn_raw_buffer_load_b128(S.gran, (int)(((size_t)gsl_pref * C + t % C) * 16), 0,
                                                              SH ? kGranAuxSys : kGranAux);
    }
    tile_own_scatter<C, NT, RMAX, PROBE>(S, cur, R);
  }
  if (!had_int) {
    if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
    if (pol) gfirst = __builtin_amdgcn_raw_buffer_load_b128(S.gran, (int)(((size_t)gsl_pref * C + t % C) * 16), 0,
                                                            SH ? kGranAuxSys : kGranAux);
  } else {
    if (had_bnd) tile_load_cells<C, NT, RMAX>(D, S.batch_s[bsplit], cur, t);
    else if (more) tile_load_cells<C, NT, RMAX>(D, S.batch_s[S.bptr_s[cn]], cur, t);
  }
  TLSTAMP(S, 6);
  // ---- 2. hand-off of colour c-1: the granule of each (foreign slot, chain)
  // until it carries epoch ph -> gdw_s; then its ghost cells
  if (hp) {
    const unsigned ep = (unsigned)ph;
    for (int u0 = 0; u0 < nfi; u0 += NT) {
      const int u = u0 + t;
      if (u < nfi) {
        const int x = u0 == 0 ? gsl_pref : D.gslot[gs0 + u / C];
        const int ch = u % C;
        const int off = (int)(((size_t)x * C + ch) * 16);
        u32x4_t g = u0 == 0 ? gfirst
                            : __builtin_amdgcn_raw_buffer_load_b128(S.gran, off, 0, SH ? kGranAuxSys : kGranAux);
        double dw = 0.0;
        for (unsigned spins = 0;; ++spins) {
          if (g.z == ep && (g.w ^ g.x ^ g.y) == S.call) {
            dw = __builtin_bit_cast(double, (unsigned long long)g.x | ((unsigned long long)g.y << 32));
            if (PROBE == 2) atomicMax(S.spin_s, spins);
            break;
          }
          if (S.timed_out || spins > (1u << 20) ||
              ((spins & 1023u) == 1023u && __hip_atomic_load(S.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            if (!S.timed_out) tile_timeout_raise(S.tmo);
            S.timed_out = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          g = __builtin_amdgcn_raw_buffer_load_b128(S.gran, off, 0, SH ? kGranAuxSys : kGranAux);
        }
        S.gdw_s[u] = dw;
      }
    }
    __syncthreads();
    if (PROBE == 2 && t == 0 && S.ph < kTimelinePhases) {
      D.dbg[((size_t)S.T * kTimelinePhases + S.ph) * kTimelineSlots + 5] = *S.spin_s;
      *S.spin_s = 0;
    }
    for (int gb = g0; gb < g1; gb += NT * GMAX) {
      if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, gr, t);
      tile_ghost_adds<C, GMAX>(S, gr);
    }
    __syncthreads();
  } else if (had_int && had_bnd) {
    __syncthreads();  // acc_s: every wave is done with the interior batch
  }
  TLSTAMP(S, 2);
  // ---- 3. boundary batches; after the last draw the next phase's records
  for (int bi = bsplit; bi < bend; ++bi) {
    if (bi != bsplit) {
      __syncthreads();
      tile_load_batch<C, NT, RMAX, SH>(D, S.batch_s[bi], cur, t);
    }
    if (bi != bsplit || had_int) tile_prep_items<C, NT, RMAX>(D, a, S.sc_s, S.seed_s, s, cur, t);
    tile_own_draw<C, NT, RMAX, PROBE, SH>(D, a, sh, S, cur, epoch);
    const int R = cur.R;
    if (bi + 1 == bend && more) tile_load_items<C, NT, RMAX, SH>(D, S.batch_s[S.bptr_s[cn]], cur, t);
    tile_own_scatter<C, NT, RMAX, PROBE>(S, cur, R);
  }
  // ---- 4. the next phase's first batch: its cells, then its draw scalars
  if (more) {
    if (had_bnd) tile_load_cells<C, NT, RMAX>(D, S.batch_s[S.bptr_s[cn]], cur, t);
    else if (!had_int) tile_load_batch<C, NT, RMAX, SH>(D, S.batch_s[S.bptr_s[cn]], cur, t);
    tile_prep_items<C, NT, RMAX>(D, a, S.sc_s, S.seed_s, sn, cur, t);
  }
  __syncthreads();
  TLSTAMP(S, 3);
}

// ---- wave-local batches (XW == 2; TileLayout::W): every own batch is ONE
// wave's -- whole slots, 64 lanes x R cells, at most kWaveSlotsMax slots --
// and the W cell waves run the batches of a colour side by side, wave w the
// batches first + w, first + w + W, ...  A wave's slots start at its lane 0
// and end inside the wave, so the slot totals need no cross-wave carry and
// the draw and the scatter read only what this wave wrote into its own part
// of acc_s: no workgroup barrier inside a colour (the batches of one colour
// touch disjoint rows of B: a row has at most one member per colour), two per
// colour phase (the hand-off, the ghost adds).  LDS accesses of one wave
// complete in issue order; wave_lds_order keeps the compiler from moving them.
__device__ __forceinline__ void wave_lds_order() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int C, int RMAX, int PROBE, int SH>
__device__ __forceinline__ void tile_own_wl(const TileDev& D, const TileLaunch& a, const TileShard& sh, TileState& S,
                                            TileBatchRegs<C, 64, RMAX>& b, unsigned epoch, double* acc_w,
                                            bool first = false) {
  constexpr int IMAX = TileBatchRegs<C, 64, RMAX>::IMAX;
  const int lane = S.lane;
  const double* __restrict__ r_s = S.r_s;
  double* __restrict__ acc_s = acc_w;
  const int R = b.R, nit = b.ns * C;
  tile_cells_landed(b);
  // Straight-line products: every live cell's r read goes out unmasked (a
  // padding cell reads the tile's last row, times its zero value; lanes past
  // the batch's live ones compute garbage that only flows to higher lanes and
  // is never stored), the running sum restarts by a 0/1 multiplier (see
  // seg_scan_step), and every slot end stores its run into acc_s -- also the
  // one that continues a slot of earlier lanes, completed after the scan
  // (acc_s[cont_q] += carry: the same operands as cont + carry).  No branch
  // per cell beyond the end stores.
  double run[C];
  int cont_q = -1;
  bool seen_start = false;
  tile_products<C, RMAX, 4>(b, R, r_s, acc_s, S.lrmax, run, cont_q, seen_start);
  // segmented inclusive scan of the lane tails inside the wave (as
  // tile_own_draw's); lane 0 holds the first cell of the wave's first slot,
  // so nothing is carried in from another wave
  double v[C];
  int f = seen_start ? 1 : 0;
#pragma unroll
  for (int ch = 0; ch < C; ++ch) v[ch] = run[ch];
  seg_scan_step<0x111, 0xF, true, C>(v, f);  // row_shr:1
  seg_scan_step<0x112, 0xF, true, C>(v, f);  // row_shr:2
  seg_scan_step<0x114, 0xF, true, C>(v, f);  // row_shr:4
  seg_scan_step<0x118, 0xF, true, C>(v, f);  // row_shr:8
  seg_scan_step<0x142, 0xA, false, C>(v, f); // row_bcast:15 -> rows 1, 3
  seg_scan_step<0x143, 0xC, false, C>(v, f); // row_bcast:31 -> rows 2, 3
#pragma unroll
  for (int ch = 0; ch < C; ++ch) {
    const double up = dpp_f64<0x138, 0xF, true>(v[ch]);  // wave_shr:1
    const double cp = lane ? up : 0.0;
    if (cont_q >= 0) acc_s[cont_q * C + ch] = acc_s[cont_q * C + ch] + cp;
  }
  wave_lds_order();
#pragma unroll
  for (int k = 0; k < IMAX; ++k) {
    const int u = lane + k * 64;
    if (u < nit) {
      const int ch = u % C;
      double dw = 0.0;
      const size_t xu = tile_xu<C, C>(b.x0, u);
      if ((a.chain_mask >> ch) & 1) {
        const double wn = (b.a0[k] - S.sc_s[2 * ch] * acc_s[u]) * b.a1[k] + b.zs[k];
        dw = wn - b.w[k];
        D.w_slot[xu] = wn;
      }
      acc_s[u] = dw;
      if (b.flag[k] & kTExported) {
        const unsigned long long uu = __builtin_bit_cast(unsigned long long, dw);
        u32x4_t g;
        g.x = (unsigned)uu; g.y = (unsigned)(uu >> 32); g.z = epoch; g.w = S.call ^ g.x ^ g.y;
        __builtin_amdgcn_raw_buffer_store_b128(g, S.gran, (int)(xu * 16), 0, SH ? kGranAuxSys : kGranAux);
        if (SH) {
#pragma unroll
          for (int h = 0; h < kTileRanksMax; ++h)
            if (h < S.G && ((b.rm[k] >> h) & 1u))
              __builtin_amdgcn_raw_buffer_store_b128(
                  g, __builtin_amdgcn_make_buffer_rsrc(sh.gx[h], 0, 0x7FFFFFFF, 0x00020000), (int)(xu * 16), 0,
                  kGranAuxSys);
        }
      }
    }
  }
  wave_lds_order();
  TLSTAMP(S, 1);
  if (PROBE == 2 && lane == 0 && S.ph < kTimelinePhases && S.wv < 7)
    D.dbg[((size_t)S.T * kTimelinePhases + S.ph) * kTimelineSlots + 9 + S.wv] = __builtin_amdgcn_s_memrealtime();
}

// the cell waves' colour phase on wave-local batches.  DB (<= 2 chains, two
// register sets): the wave's next batch loads at the phase start, its HBM
// stream overlapping this colour's work; otherwise its records after the
// draw and its cells after the scatter and the draw preparation.
template <int C, int NT, int RMAX, int GMAX, int PROBE, int SH, int DB>
__device__ __forceinline__ void tile_phase_wl(const TileDev& D, const TileLaunch& a, const TileShard& sh,
                                              TileState& S, int ph, TileBatchRegs<C, 64, RMAX>& cur,
                                              TileBatchRegs<C, 64, RMAX>& nxt, TileGhostRegs<C, GMAX>& gr) {
  constexpr int W = NT / 64 - 1;  // cell waves
  const int K = S.K, t = S.t, lane = S.lane;
  const int s = ph / K, c = ph - s * K;
  const unsigned epoch = (unsigned)ph + 1;
  S.ph = ph;
  TLSTAMP(S, 0);
  const int phn = ph + 1;
  const int cn = phn % K, sn = phn / K;
  const bool has_next = phn < S.nph;
  const int bnext = S.bptr_s[cn] + S.wv;
  const bool more = has_next && bnext < S.bptr_s[cn + 1];
  const int bfirst = S.bptr_s[c] + S.wv, bend = S.bptr_s[c + 1];
  const int g0 = S.gptr_s[c], g1 = S.gptr_s[c + 1];
  double* acc_w = S.acc_s + S.wv * (kWaveSlotsMax * C);
  if (DB && more) tile_load_batch<C, 64, RMAX, SH>(D, S.batch_s[bnext], nxt, lane);
  for (int bi = bfirst; bi < bend; bi += W) {
    if (bi != bfirst) {  // a later round of this colour (large colours only): independent rows, no barrier
      tile_load_batch<C, 64, RMAX, SH>(D, S.batch_s[bi], cur, lane);
      tile_prep_items<C, 64, RMAX>(D, a, S.sc_s, S.seed_s, s, cur, lane);
    }
    tile_own_wl<C, RMAX, PROBE, SH>(D, a, sh, S, cur, epoch, acc_w, bi == bfirst);
    if (bi == bfirst && S.wv == 0 && lane == 0)  // the exchange wave's poll gate (tile_phase_xw)
      __hip_atomic_store(S.pub_s, ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int R = cur.R;
    if (bi + W >= bend) {  // this wave's last batch of the colour: its records are dead
      if (!DB && more) tile_load_items<C, 64, RMAX, SH>(D, S.batch_s[bnext], nxt, lane);
      if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
    }
    tile_own_scatter<C, 64, RMAX, PROBE>(S, cur, R, acc_w);
  }
  if (bfirst >= bend) {  // no batch of this colour for this wave
    if (!DB && more) tile_load_items<C, 64, RMAX, SH>(D, S.batch_s[bnext], nxt, lane);
    if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
  }
  TLSTAMP(S, 6);
  if (more) tile_prep_items<C, 64, RMAX>(D, a, S.sc_s, S.seed_s, sn, nxt, lane, PROBE == 2 ? a.variant : 0);
  if (!DB && more) tile_load_cells<C, 64, RMAX>(D, S.batch_s[bnext], nxt, lane);
  TLSTAMP(S, 4);
  __syncthreads();  // the exchange wave has every dw of the colour in gdw_s
  TLSTAMP(S, 2);
  for (int gb = g0; gb < g1; gb += NT * GMAX) {
    if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, gr, t);
    tile_ghost_adds<C, GMAX>(S, gr);
  }
  __syncthreads();
  TLSTAMP(S, 3);
}

// Wave-local batches on an interior-first layout (IB with XW == 2;
// TileLayout::split): per colour c, each cell wave first runs its batches of
// c's interior slots -- no row of their columns waits for a draw of colour
// c-1 in another tile -- while the exchange wave is still polling colour
// c-1's granules; then (barrier A) colour c-1's ghost adds (barrier B); then
// its batches of c's boundary slots.  The chain from a neighbour's draw to
// this tile's next draw runs through the boundary batches only; the interior
// work overlaps the hand-off.  The rows of an interior column take no ghost
// add of c-1, so every row sees its updates in the colour-by-colour order.
// `cur` holds this wave's first batch of the phase (interior, else boundary),
// prepared; the hand-off of the last colour of the call is the epilogue's.
// Three workgroup barriers per phase: A (the hand-off is in), B (the ghost
// adds are done), C (the boundary batches are done).
template <int C, int NT, int RMAX, int GMAX, int PROBE, int SH>
__device__ __forceinline__ int tile_wlib_first(const TileState& S, int c) {
  const int fi = S.bptr_s[c] + S.wv, fb = S.bsp_s[c] + S.wv;
  return fi < S.bsp_s[c] ? fi : (fb < S.bptr_s[c + 1] ? fb : -1);
}

template <int C, int NT, int RMAX, int GMAX, int PROBE, int SH>
__device__ __forceinline__ void tile_phase_wlib(const TileDev& D, const TileLaunch& a, const TileShard& sh,
                                                TileState& S, int ph, TileBatchRegs<C, 64, RMAX>& cur,
                                                TileGhostRegs<C, GMAX>& gr) {
  constexpr int W = NT / 64 - 1;  // cell waves
  const int K = S.K, t = S.t, lane = S.lane;
  const int s = ph / K, c = ph - s * K;
  const unsigned epoch = (unsigned)ph + 1;
  S.ph = ph;
  TLSTAMP(S, 0);
  const int phn = ph + 1;
  const int cn = phn % K, sn = phn / K;
  const int nxt_b = phn < S.nph ? tile_wlib_first<C, NT, RMAX, GMAX, PROBE, SH>(S, cn) : -1;
  const int bsp = S.bsp_s[c], b1 = S.bptr_s[c + 1];
  const int ifirst = S.bptr_s[c] + S.wv, bfirst = bsp + S.wv;
  // the hand-off of the previous colour (none at the first phase of a call)
  const bool hp = ph > 0;
  const int cp = hp ? (ph - 1) % K : 0;
  const int g0 = S.gptr_s[cp], g1 = hp ? S.gptr_s[cp + 1] : g0;
  double* acc_w = S.acc_s + S.wv * (kWaveSlotsMax * C);
  bool nx_items = false;  // the next phase's first batch: records in flight
  // ---- interior batches
  for (int bi = ifirst; bi < bsp; bi += W) {
    if (bi != ifirst) {
      tile_load_batch<C, 64, RMAX, SH>(D, S.batch_s[bi], cur, lane);
      tile_prep_items<C, 64, RMAX>(D, a, S.sc_s, S.seed_s, s, cur, lane);
    }
    tile_own_wl<C, RMAX, PROBE, SH>(D, a, sh, S, cur, epoch, acc_w);
    const int R = cur.R;
    if (bi + W >= bsp) {  // the last interior batch: its records are dead
      if (bfirst < b1) {
        tile_load_items<C, 64, RMAX, SH>(D, S.batch_s[bfirst], cur, lane);
      } else if (nxt_b >= 0) {
        tile_load_items<C, 64, RMAX, SH>(D, S.batch_s[nxt_b], cur, lane);
        nx_items = true;
      }
      if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
    }
    tile_own_scatter<C, 64, RMAX, PROBE>(S, cur, R, acc_w);
  }
  if (ifirst >= bsp) {  // no interior batch: cur already holds the first boundary batch, if any
    if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
  } else if (bfirst < b1) {
    tile_prep_items<C, 64, RMAX>(D, a, S.sc_s, S.seed_s, s, cur, lane);
    tile_load_cells<C, 64, RMAX>(D, S.batch_s[bfirst], cur, lane);
  }
  TLSTAMP(S, 6);
  __syncthreads();  // A: the exchange wave has every dw of colour c-1 in gdw_s
  TLSTAMP(S, 4);
  for (int gb = g0; gb < g1; gb += NT * GMAX) {
    if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, gr, t);
    tile_ghost_adds<C, GMAX>(S, gr);
  }
  __syncthreads();  // B
  TLSTAMP(S, 2);
  // ---- boundary batches
  for (int bi = bfirst; bi < b1; bi += W) {
    if (bi != bfirst) {
      tile_load_batch<C, 64, RMAX, SH>(D, S.batch_s[bi], cur, lane);
      tile_prep_items<C, 64, RMAX>(D, a, S.sc_s, S.seed_s, s, cur, lane);
    }
    tile_own_wl<C, RMAX, PROBE, SH>(D, a, sh, S, cur, epoch, acc_w);
    const int R = cur.R;
    if (bi + W >= b1 && nxt_b >= 0) {
      tile_load_items<C, 64, RMAX, SH>(D, S.batch_s[nxt_b], cur, lane);
      nx_items = true;
    }
    tile_own_scatter<C, 64, RMAX, PROBE>(S, cur, R, acc_w);
  }
  if (nxt_b >= 0) {
    if (!nx_items) tile_load_items<C, 64, RMAX, SH>(D, S.batch_s[nxt_b], cur, lane);
    tile_prep_items<C, 64, RMAX>(D, a, S.sc_s, S.seed_s, sn, cur, lane);
    tile_load_cells<C, 64, RMAX>(D, S.batch_s[nxt_b], cur, lane);
  }
  // C: every wave's boundary batches of c are done before any wave's interior
  // batches of c+1 (a row may have an own member of c in one wave's boundary
  // batch and one of c+1 in another wave's interior batch)
  __syncthreads();
  TLSTAMP(S, 3);
}

// ---- exchange-wave tiles (XW; TileDev::xw).  vmcnt counts a wave's
// vector-memory operations in issue order, loads and stores together, so in
// a wave that streams the next batch's cells every poll of a granule -- and
// every retry -- waits for that whole stream first (and the conditional loads
// leave the compiler no count but vmcnt(0)).  Here the last wave of the
// workgroup owns no cells and no draw items: it loads its share of this
// colour's ghost cells at the phase start (static data), passes the own
// batches' barriers, and after the last draw polls the colour's foreign
// granules with only its own polls in its queue, while the other NT - 64
// threads ("cell waves") scatter, prepare the next batch and stream its cells.
// The layout's batches are cut for NT - 64 cell threads.

// the exchange wave's phase: its share of the colour's ghost cells (static
// data: loaded at the phase start, long in registers when the hand-off
// ends), the own batches' barriers, then the hand-off polls -> gdw_s, and its
// share of the ghost adds
// LAG (interior-first wave-local tiles): phase ph hands off colour ph - 1
// between its interior and boundary batches (none at ph = 0; ph = nph: the
// launch's epilogue)
template <int C, int NT, int GMAX, int PROBE, int SH, int WL = 0, int LAG = 0>
__device__ __forceinline__ void tile_phase_xw(const TileDev& D, TileState& S, int ph, TileGhostRegs<C, GMAX>& gr) {
  constexpr int PB = 4;  // granule polls in flight per lane
  const int K = S.K, t = S.t, lane = S.lane;
  S.ph = ph;
  if (LAG && ph == 0) {  // the cell waves' barriers A, B and C
    __syncthreads();
    __syncthreads();
    __syncthreads();
    return;
  }
  const int phx = ph - LAG;
  const int c = phx % K;
  const unsigned epoch = (unsigned)phx + 1;
  const int bfirst = S.bptr_s[c], bend = S.bptr_s[c + 1];
  const int g0 = S.gptr_s[c], g1 = S.gptr_s[c + 1];
  const int gs0 = S.gsp_s[c], nfi = (S.gsp_s[c + 1] - gs0) * C;
  const int aux = SH ? kGranAuxSys : kGranAux;
  if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
  int gx[PB];  // the first round's foreign slot indices
#pragma unroll
  for (int k = 0; k < PB; ++k) {
    const int u = k * 64 + lane;
    gx[k] = u < nfi ? D.gslot[gs0 + u / C] : 0;
  }
  // the own batches' barriers (tile_own_draw: kOwnDrawBarriers each, + 1
  // before a later batch, as tile_phase_cells; wave-local batches have none)
  for (int bi = bfirst; bi < (WL ? bfirst : bend); ++bi) {
    if (bi != bfirst) __syncthreads();
#pragma unroll
    for (int q = 0; q < kOwnDrawBarriers; ++q) __syncthreads();
  }
  // (Measured and dropped: an L2 prefetch of the next batch's records and
  // cells and the colour's ghost cells by this wave at the phase start, one
  // 4-B load per 64-B segment: 3,160-3,400 vs 2,275 us per 10-sweep launch at
  // the headline -- the polls wait behind the prefetch.)
  // Wave-local tiles: the first poll round waits until this tile's wave 0 has
  // drawn its first batch of the colour -- the neighbours draw theirs at about
  // the same time, so earlier rounds would only find old granules (each poll
  // is an L2-bypassing request: they were most of the traffic above the
  // layout's bytes).  Wave 0 has a batch whenever the colour has one here.
  if (WL && !LAG && S.bptr_s[c] < S.bptr_s[c + 1])
    while (__hip_atomic_load(S.pub_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < ph) __builtin_amdgcn_s_sleep(1);
  // hand-off: every (foreign slot, chain) of colour c until its granule
  // carries this epoch -> gdw_s (polls in flight per lane; a retry waits for
  // this wave's own polls only).  (Measured and dropped: a train of 3 poll
  // rounds in flight per item, 11.65k -> 10.5k chain-sweeps/s: the extra
  // polls queue in the memory system in front of everyone's stream.)
  for (int u0 = 0; u0 < nfi; u0 += 64 * PB) {
    u32x4_t g[PB];
    int off[PB];
    unsigned pend = 0;
#pragma unroll
    for (int k = 0; k < PB; ++k) {
      const int u = u0 + k * 64 + lane;
      if (u < nfi) {
        const int x = u0 == 0 ? gx[k] : D.gslot[gs0 + u / C];
        off[k] = (int)(((size_t)x * C + u % C) * 16);
        g[k] = __builtin_amdgcn_raw_buffer_load_b128(S.gran, off[k], 0, aux);
        pend |= 1u << k;
      }
    }
    for (unsigned spins = 0; pend; ++spins) {
#pragma unroll
      for (int k = 0; k < PB; ++k) {
        if (((pend >> k) & 1u) && g[k].z == epoch && (g[k].w ^ g[k].x ^ g[k].y) == S.call) {
          S.gdw_s[u0 + k * 64 + lane] =
              __builtin_bit_cast(double, (unsigned long long)g[k].x | ((unsigned long long)g[k].y << 32));
          pend &= ~(1u << k);
        }
      }
      if (!pend) break;
      if (PROBE == 2) atomicMax(S.spin_s, spins + 1);
      // bounded wait (about a second per poll); once any tile of the launch
      // has given up (timeout word), the others stop waiting within ~1k polls
      if (S.timed_out || spins > (1u << 20) ||
          ((spins & 1023u) == 1023u && __hip_atomic_load(S.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        if (!S.timed_out) tile_timeout_raise(S.tmo);
        S.timed_out = true;
#pragma unroll
        for (int k = 0; k < PB; ++k)
          if ((pend >> k) & 1u) S.gdw_s[u0 + k * 64 + lane] = 0.0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int k = 0; k < PB; ++k)
        if ((pend >> k) & 1u) g[k] = __builtin_amdgcn_raw_buffer_load_b128(S.gran, off[k], 0, aux);
    }
  }
  if (PROBE == 2 && lane == 0 && S.ph < kTimelinePhases) {
    D.dbg[((size_t)S.T * kTimelinePhases + S.ph) * kTimelineSlots + 7] = __builtin_amdgcn_s_memrealtime();
    D.dbg[((size_t)S.T * kTimelinePhases + S.ph) * kTimelineSlots + 5] = *S.spin_s;
    *S.spin_s = 0;
  }
  __syncthreads();
  for (int gb = g0; gb < g1; gb += NT * GMAX) {
    if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, gr, t);
    tile_ghost_adds<C, GMAX>(S, gr);
  }
  __syncthreads();
  if (LAG && ph < S.nph) __syncthreads();  // C: the cell waves' boundary batches are done
}

// the cell waves' phase (threads t < NTC = NT - 64): own batches (their
// granule stores in the draw, ahead of any load of the phase), the next
// batch -- records after the draw, then (one register set) its cells after
// the scatter and the draw preparation, or (DB) its cells with the records --
// and their share of the ghost cells after the hand-off
template <int C, int NT, int NTC, int RMAX, int GMAX, int DB, int PROBE, int SH>
__device__ __forceinline__ void tile_phase_cells(const TileDev& D, const TileLaunch& a, const TileShard& sh,
                                                 TileState& S, int ph, TileBatchRegs<C, NTC, RMAX>& cur,
                                                 TileBatchRegs<C, NTC, RMAX>& nxt, TileGhostRegs<C, GMAX>& gr) {
  const int K = S.K, t = S.t;
  const int s = ph / K, c = ph - s * K;
  const unsigned epoch = (unsigned)ph + 1;
  S.ph = ph;
  TLSTAMP(S, 0);
  const int phn = ph + 1;
  const int cn = phn % K, sn = phn / K;
  const bool has_next = phn < S.nph;
  const bool more = has_next && S.bptr_s[cn] < S.bptr_s[cn + 1];
  const int bfirst = S.bptr_s[c], bend = S.bptr_s[c + 1];
  const int g0 = S.gptr_s[c], g1 = S.gptr_s[c + 1];
  for (int bi = bfirst; bi < bend; ++bi) {
    if (bi != bfirst) {  // rare: a colour with more than one batch in this tile
      __syncthreads();
      tile_load_batch<C, NTC, RMAX, SH>(D, S.batch_s[bi], cur, t);
      tile_prep_items<C, NTC, RMAX>(D, a, S.sc_s, S.seed_s, s, cur, t);
    }
    tile_own_draw<C, NTC, RMAX, PROBE, SH>(D, a, sh, S, cur, epoch);
    const int R = cur.R;
    if (bi + 1 == bend) {
      if (more) {
        if (DB) tile_load_batch<C, NTC, RMAX, SH>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
        else tile_load_items<C, NTC, RMAX, SH>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
      }
      if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
    }
    tile_own_scatter<C, NTC, RMAX, PROBE>(S, cur, R);
  }
  if (bend == bfirst) {
    if (more) {
      if (DB) tile_load_batch<C, NTC, RMAX, SH>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
      else tile_load_items<C, NTC, RMAX, SH>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
    }
    if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, gr, t);
  }
  TLSTAMP(S, 6);
  // the next batch's draw scalars, then (one register set) its cells: they
  // stream while the exchange wave waits for the neighbours.  (Measured and
  // dropped: the draw's w stores deferred behind the next records, 11.65k ->
  // 10.5k chain-sweeps/s.)
  if (more) tile_prep_items<C, NTC, RMAX>(D, a, S.sc_s, S.seed_s, sn, nxt, t);
  if (!DB && more) tile_load_cells<C, NTC, RMAX>(D, S.batch_s[S.bptr_s[cn]], nxt, t);
  TLSTAMP(S, 4);
  __syncthreads();  // the exchange wave has every dw of the colour in gdw_s
  TLSTAMP(S, 2);
  for (int gb = g0; gb < g1; gb += NT * GMAX) {
    if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, gr, t);
    tile_ghost_adds<C, GMAX>(S, gr);
  }
  __syncthreads();
  TLSTAMP(S, 3);
}

// RG: the tile's r in global memory (D.rg, the tile's local rows at
// erow_ptr[tile] x C) instead of LDS -- layouts whose tiles do not fit a CU's
// LDS (n = 1e7 on one GPU).  A row takes at most one update per colour (one
// member per colour), so the scatter and the ghost adds stay plain
// read-modify-writes; the phase barriers order them for the workgroup.
// CS: chain stride of the per-slot arrays.  CS == C: the workgroup runs every
// chain of the context (one workgroup per tile).  CS > C = 1 (chain-split,
// sweep_tiles_cs_kernel): workgroup b runs chain b / T of tile b % T -- the
// chains are independent Markov chains, so the CS workgroups of a tile share
// its CU and each one's stream and hand-off waits overlap the others' work.
// Chain-major numbering: the dispatcher places chain 0's tiles first, so a
// chain never waits on a tile of its own that is not resident.
template <int C, int NT, int RMAX, int GMAX, int DB, int PROBE, int SH, int RG, int IB, int CS, int XW = 0>
__device__ __forceinline__ void sweep_tiles_body(const TileDev& D0, TileLaunch a, const TileShard& sh) {
  static_assert(!XW || ((!RG || XW == 2) && (!IB || XW == 2) && CS == C),
                "exchange-wave tiles: joint chains; split layouts and r in global memory only with wave-local batches");
  constexpr int NTC = XW ? NT - 64 : NT;  // cell threads
  using BR = TileBatchRegs<C, NTC, RMAX>;
  constexpr int NW = NT / 64;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  // tile shard: global tile index, its rank, that rank's buffers
  int Tg = SH ? sh.tile0 + (int)blockIdx.x : (int)blockIdx.x;
  const int rk = SH ? Tg / sh.Tl : 0;
  TileDev D = SH ? sh.devs[rk - sh.rank0] : D0;
  int ch0 = 0;
  if constexpr (CS != C) {
    static_assert(C == 1 && !SH && !RG && !IB && !PROBE, "chain-split: one chain per workgroup, single GPU");
    ch0 = Tg / D.T;
    Tg -= ch0 * D.T;
    D.cell_val += (size_t)ch0 * D.n_cells;
    D.gval += (size_t)ch0 * D.n_gcells;
    D.dr += ch0;
    D.w_slot += ch0;
    D.dwx += 2 * ch0;  // 16-B granules
    D.r += ch0;
    D.scal += ch0;
    D.b1 += ch0;
    a.chain_mask >>= ch0;
    if (a.z_in) a.z_in += ch0;
  }
  TileState S;
  S.G = SH ? sh.G : 1;
  S.T = Tg; S.t = threadIdx.x; S.lane = S.t & 63; S.wv = S.t >> 6; S.K = D.K;
  S.nph = a.n_sweeps * D.K;
  S.timed_out = false;
  for (int k = 0; k < 8; ++k) S.tp[k] = 0;
  S.t_prev = 0;
  const int T = S.T, t = S.t, K = D.K;
  const int row0 = D.erow_ptr[T], nrows = D.erow_ptr[T + 1] - row0;
  S.lrmax = nrows > 0 ? (uint32_t)(nrows - 1) : 0u;
  const int b_lo = D.batch_ptr[T * K], nbt = D.batch_ptr[T * K + K] - b_lo;
  S.r_s = RG ? D.rg + (size_t)row0 * C : smem;
  S.acc_s = RG ? smem : smem + ((nrows * C + 1) / 2) * 2;  // kAccSlots x C: slot totals, then dw
  S.wsum = S.acc_s + kAccSlots * C;              // NW x C: segmented wave totals
  S.sc_s = S.wsum + NW * C;                      // C x {inv_s2, inv_t2}
  S.seed_s = reinterpret_cast<unsigned long long*>(S.sc_s + 2 * C);
  S.dsh_s = reinterpret_cast<double*>(S.seed_s + 2 * C);  // C
  S.gdw_s = S.dsh_s + C;                         // max foreign slots x C (even count)
  S.batch_s = reinterpret_cast<int4*>(S.gdw_s + ((D.max_gslots * C + 1) / 2) * 2);
  S.bptr_s = reinterpret_cast<int*>(S.batch_s + nbt);
  S.gptr_s = S.bptr_s + K + 1;
  S.gsp_s = S.gptr_s + K + 1;
  S.bsp_s = S.gsp_s + K + 1;                     // K+1 (split layouts)
  S.wflag = S.bsp_s + K + 1;                     // NW: the wave holds a slot start
  S.spin_s = reinterpret_cast<unsigned*>(S.wflag + NW);  // NNGP_PROBE=2: max poll spins of the phase
  if (PROBE == 2 && t == 0) *S.spin_s = 0;
  S.pub_s = reinterpret_cast<int*>(S.spin_s + 1);        // (tile_lds_bytes' 64-byte tail)
  if (t == 0) *S.pub_s = -1;
  TSTAMP(S, -1);
  // r of the local rows as the last call left it; a warm call after a
  // beta_0-only change (capi.hip warm_kinds) starts from r - d B 1, and its
  // own slots' w from w - d (below)
  double dsh[C];
#pragma unroll
  for (int ch = 0; ch < C; ++ch) dsh[ch] = D.scal[ch].dshift;
  for (int lr = t; lr < nrows; lr += NT) {
    const int row = D.erow[row0 + lr];
    const size_t g = (size_t)row * CS;
#pragma unroll
    for (int ch = 0; ch < C; ++ch) {
      const double v = D.r[g + ch];
      S.r_s[lr * C + ch] = dsh[ch] != 0.0 ? __builtin_fma(-dsh[ch], D.b1[ch][row], v) : v;
    }
  }
  // per-tile metadata in LDS: no dependent scalar loads in the phase loop
  for (int i = t; i < nbt; i += NT) S.batch_s[i] = D.batch[b_lo + i];
  for (int i = t; i <= K; i += NT) {
    S.bptr_s[i] = D.batch_ptr[T * K + i] - b_lo;
    S.gptr_s[i] = D.gptr[T * K + i];
    S.gsp_s[i] = D.gslot_ptr[T * K + i];
    if (IB) S.bsp_s[i] = i < K ? D.batch_split[T * K + i] - b_lo : 0;
  }
  if (t < C) {
    S.dsh_s[t] = D.scal[t].dshift;
    S.sc_s[2 * t] = D.scal[t].inv_s2;
    S.sc_s[2 * t + 1] = D.scal[t].inv_t2;
    S.seed_s[2 * t] = D.scal[t].seed;
    S.seed_s[2 * t + 1] = D.scal[t].counter_base;
  }
  S.call = SH ? *sh.call : D.ctl[0];
  S.gsl = 0;
  S.tmo = D.ctl + 1;
  S.gran = __builtin_amdgcn_make_buffer_rsrc(SH ? sh.gx[rk] : D.dwx, 0, 0x7FFFFFFF, 0x00020000);
  __syncthreads();
  bool shifted = false;
#pragma unroll
  for (int ch = 0; ch < C; ++ch) shifted |= dsh[ch] != 0.0;
  if (shifted && nbt > 0) {
    // w = field - beta_0 of the own slots (one contiguous range: slot order
    // is tile-major, the batches cover it in order) moved by -d before any
    // batch loads it; the stores are this workgroup's, ordered by the barrier
    const int x0 = S.batch_s[0].w, x1 = S.batch_s[nbt - 1].w + S.batch_s[nbt - 1].z;
    for (int u = t; u < (x1 - x0) * C; u += NT) D.w_slot[tile_xu<C, CS>(x0, u)] -= S.dsh_s[u % C];
    __syncthreads();
  }
  if constexpr (XW) {
    if (S.wv == NW - 1) {  // the exchange wave
      TileGhostRegs<C, GMAX> GX;
      __syncthreads();
      if constexpr (IB) {
        for (int ph = 0; ph <= S.nph; ++ph) tile_phase_xw<C, NT, GMAX, PROBE, SH, 1, 1>(D, S, ph, GX);
      } else {
        for (int ph = 0; ph < S.nph; ++ph) tile_phase_xw<C, NT, GMAX, PROBE, SH, XW == 2>(D, S, ph, GX);
      }
    } else if constexpr (XW == 2 && IB) {  // interior-first wave-local batches
      TileBatchRegs<C, 64, RMAX> A;
      TileGhostRegs<C, GMAX> GA;
      const int f0 = S.nph > 0 ? tile_wlib_first<C, NT, RMAX, GMAX, PROBE, SH>(S, 0) : -1;
      if (f0 >= 0) {
        tile_load_batch<C, 64, RMAX, SH>(D, S.batch_s[f0], A, S.lane);
        tile_prep_items<C, 64, RMAX>(D, a, S.sc_s, S.seed_s, 0, A, S.lane);
      }
      __syncthreads();
      for (int ph = 0; ph < S.nph; ++ph) tile_phase_wlib<C, NT, RMAX, GMAX, PROBE, SH>(D, a, sh, S, ph, A, GA);
      // epilogue: the hand-off of the call's last colour (the exchange wave's ph = nph)
      const int cp = S.nph > 0 ? (S.nph - 1) % K : 0;
      const int g0 = S.gptr_s[cp], g1 = S.nph > 0 ? S.gptr_s[cp + 1] : g0;
      if (g1 > g0) tile_load_ghosts<C, NT, GMAX>(D, g0, g1, GA, t);
      if (S.nph > 0) {
        __syncthreads();
        for (int gb = g0; gb < g1; gb += NT * GMAX) {
          if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, GA, t);
          tile_ghost_adds<C, GMAX>(S, GA);
        }
        __syncthreads();
      } else {
        __syncthreads();
        __syncthreads();
      }
    } else if constexpr (XW == 2) {  // wave-local batches: wave w runs batches first + w, + W, ...
      TileBatchRegs<C, 64, RMAX> A, B;
      TileGhostRegs<C, GMAX> GA;
      if (S.nph > 0 && S.bptr_s[0] + S.wv < S.bptr_s[1]) {
        tile_load_batch<C, 64, RMAX, SH>(D, S.batch_s[S.bptr_s[0] + S.wv], A, S.lane);
        tile_prep_items<C, 64, RMAX>(D, a, S.sc_s, S.seed_s, 0, A, S.lane);
      }
      __syncthreads();
      if (DB) {
        for (int ph = 0; ph < S.nph; ph += 2) {
          tile_phase_wl<C, NT, RMAX, GMAX, PROBE, SH, DB>(D, a, sh, S, ph, A, B, GA);
          if (ph + 1 < S.nph) tile_phase_wl<C, NT, RMAX, GMAX, PROBE, SH, DB>(D, a, sh, S, ph + 1, B, A, GA);
        }
      } else {
        for (int ph = 0; ph < S.nph; ++ph) tile_phase_wl<C, NT, RMAX, GMAX, PROBE, SH, DB>(D, a, sh, S, ph, A, A, GA);
      }
    } else {
      BR A, B;
      TileGhostRegs<C, GMAX> GA;
      if (S.nph > 0 && S.bptr_s[0] < S.bptr_s[1]) {
        tile_load_batch<C, NTC, RMAX, SH>(D, S.batch_s[S.bptr_s[0]], A, t);
        tile_prep_items<C, NTC, RMAX>(D, a, S.sc_s, S.seed_s, 0, A, t);
      }
      __syncthreads();
      if (DB) {
        for (int ph = 0; ph < S.nph; ph += 2) {
          tile_phase_cells<C, NT, NTC, RMAX, GMAX, DB, PROBE, SH>(D, a, sh, S, ph, A, B, GA);
          if (ph + 1 < S.nph) tile_phase_cells<C, NT, NTC, RMAX, GMAX, DB, PROBE, SH>(D, a, sh, S, ph + 1, B, A, GA);
        }
      } else {
        for (int ph = 0; ph < S.nph; ++ph) tile_phase_cells<C, NT, NTC, RMAX, GMAX, DB, PROBE, SH>(D, a, sh, S, ph, A, A, GA);
      }
    }
  } else {
  BR A, B;  // batch register sets: the current colour's and (DB) the next one's
  TileGhostRegs<C, GMAX> GA, GB;
  if (S.nph > 0 && S.bptr_s[0] < S.bptr_s[1]) {
    tile_load_batch<C, NT, RMAX, SH, CS>(D, S.batch_s[S.bptr_s[0]], A, t);
    tile_prep_items<C, NT, RMAX, CS>(D, a, S.sc_s, S.seed_s, 0, A, t);
  }
  if (DB && S.nph > 0 && S.gptr_s[0] < S.gptr_s[1]) tile_load_ghosts<C, NT, GMAX>(D, S.gptr_s[0], S.gptr_s[1], GA, t);
  if (S.nph > 0 && t < (S.gsp_s[1] - S.gsp_s[0]) * C) S.gsl = D.gslot[S.gsp_s[0] + t / C];
  __syncthreads();
  TSTAMP(S, 7);
  if (CS != C && ch0 > 0 && a.stagger > 0) {
    // chain-split: the chains' phases out of step (identical work per phase
    // would keep them in lockstep, contending for the CU at the same time)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ch0 * (unsigned)a.stagger) __builtin_amdgcn_s_sleep(4);
  }
  if (DB) {
    for (int ph = 0; ph < S.nph; ph += 2) {
      tile_phase<C, NT, RMAX, GMAX, DB, PROBE, SH, CS>(D, a, sh, S, ph, A, B, GA, GB);
      if (ph + 1 < S.nph) tile_phase<C, NT, RMAX, GMAX, DB, PROBE, SH, CS>(D, a, sh, S, ph + 1, B, A, GB, GA);
    }
  } else if (IB) {
    for (int ph = 0; ph < S.nph; ++ph) tile_phase_ib<C, NT, RMAX, GMAX, PROBE, SH>(D, a, sh, S, ph, A, GA);
  } else {
    for (int ph = 0; ph < S.nph; ++ph) tile_phase<C, NT, RMAX, GMAX, DB, PROBE, SH, CS>(D, a, sh, S, ph, A, A, GA, GA);
  }
  }  // !XW
  // r of the tile's local rows back to global memory: the next call can start
  // from it instead of recomputing r = B w (capi.hip "warm" calls).  Every
  // tile holding row k applied the same updates to it in the same (colour)
  // order from the same start, so the copies written by different tiles are
  // bitwise equal.
  __syncthreads();
  for (int lr = t; lr < nrows; lr += NT) {
    double* rg = const_cast<double*>(D.r) + (size_t)D.erow[row0 + lr] * CS;
#pragma unroll
    for (int ch = 0; ch < C; ++ch) rg[ch] = S.r_s[lr * C + ch];
  }
  if (PROBE == 1 && t == 0) {
    unsigned long long* o = D.dbg + (size_t)T * 8;
    for (int k = 0; k < 8; ++k) o[k] = S.tp[k];
  }
}

template <int C, int NT, int RMAX, int GMAX, int DB, int PROBE, int SH, int RG, int IB, int XW>
__global__ __launch_bounds__(NT) void sweep_tiles_kernel(TileDev D0, TileLaunch a, TileShard sh) {
  sweep_tiles_body<C, NT, RMAX, GMAX, DB, PROBE, SH, RG, IB, C, XW>(D0, a, sh);
}

// chain-split: CS one-chain workgroups per tile, CS per CU (CS waves of
// NT / 64 per SIMD: the register budget of that occupancy)
template <int CS, int NT, int RMAX, int GMAX>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(CS * NT / 256, CS * NT / 256)))
void sweep_tiles_cs_kernel(TileDev D0, TileLaunch a) {
  sweep_tiles_body<1, NT, RMAX, GMAX, 0, 0, 0, 0, 0, CS>(D0, a, TileShard());
}
#undef TSTAMP

// sh == nullptr: one GPU, the call-id bump and the whole grid of tiles here;
// else the caller bumped the call ids and `grid` tiles from sh->tile0 run
// occ != nullptr: no launch -- *occ = the workgroups of exactly this
// instantiation (and LDS) that fit one CU at once (the residency check of
// the persistent launch: every tile must be resident, tiles spin on each other)
template <int C, int NT, int PROBE, int SH, int RG = 0, int IB0 = -1>
static hipError_t launch_tiles_c(hipStream_t st, const TileDev& D, const TileLaunch& a, int lds, const TileShard* sh,
                                 int grid, int* occ = nullptr) {
  constexpr int RMAX = tile_rmax(C, NT);
  constexpr int DB = tile_double_buffer(C, NT);
  constexpr int GMAX = tile_gmax(NT);
  // split layouts (interior first) at one register set; IB0 >= 0 pins it
  if constexpr (IB0 < 0 && DB == 0) {
    if (D.batch_split) return launch_tiles_c<C, NT, PROBE, SH, RG, 1>(st, D, a, lds, sh, grid, occ);
    return launch_tiles_c<C, NT, PROBE, SH, RG, 0>(st, D, a, lds, sh, grid, occ);
  }
  constexpr int IB = IB0 > 0 ? 1 : 0;
  if (D.batch_split && !IB) return hipErrorInvalidValue;  // split layout: double-buffered path not for it
  auto k = sweep_tiles_kernel<C, NT, RMAX, GMAX, DB, PROBE, SH, RG, IB, 0>;
  if constexpr (NT == 512 && !RG && !IB) {
    if (D.xw == 1) k = sweep_tiles_kernel<C, NT, RMAX, GMAX, DB, PROBE, SH, RG, IB, 1>;
  }
  // wave-local batches: r in LDS or (no probes) in global memory, plain or
  // interior-first layouts
  if constexpr (NT == 512 && (!RG || !PROBE)) {
    if (D.xw == 2) k = sweep_tiles_kernel<C, NT, RMAX, GMAX, DB, PROBE, SH, RG, IB, 2>;
  }
  if (D.xw && (NT != 512 || ((RG || IB) && D.xw != 2))) return hipErrorInvalidValue;
  lds = lds < kTSpreadLds ? kTSpreadLds : lds;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  if (occ) return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, reinterpret_cast<const void*>(k), NT, lds);
  if constexpr (SH) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, st, D, a, *sh);
  } else {
    hipLaunchKernelGGL(tile_call_bump_kernel, dim3(1), dim3(1), 0, st, D.ctl);
    hipLaunchKernelGGL(k, dim3(D.T), dim3(NT), lds, st, D, a, TileShard());
  }
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_tiles_nt(hipStream_t st, const TileDev& D, const TileLaunch& a, int lds, const TileShard* sh,
                                  int grid, int* occ) {
  if (D.rg) {  // r in global memory: 512- or 1024-thread tiles; tile shards 512
    if constexpr (NT == 512) {
      if (sh) {
        switch (D.C) {
          case 1: return launch_tiles_c<1, NT, 0, 1, 1>(st, D, a, lds, sh, grid, occ);
          case 2: return launch_tiles_c<2, NT, 0, 1, 1>(st, D, a, lds, sh, grid, occ);
          case 3: return launch_tiles_c<3, NT, 0, 1, 1>(st, D, a, lds, sh, grid, occ);
          case 4: return launch_tiles_c<4, NT, 0, 1, 1>(st, D, a, lds, sh, grid, occ);
          default: return hipErrorInvalidValue;
        }
      }
    }
    if constexpr (NT == 512 || NT == 1024) {
      if (sh) return hipErrorInvalidValue;
      switch (D.C) {
        case 1: return launch_tiles_c<1, NT, 0, 0, 1>(st, D, a, lds, nullptr, 0, occ);
        case 2: return launch_tiles_c<2, NT, 0, 0, 1>(st, D, a, lds, nullptr, 0, occ);
        case 3: return launch_tiles_c<3, NT, 0, 0, 1>(st, D, a, lds, nullptr, 0, occ);
        case 4: return launch_tiles_c<4, NT, 0, 0, 1>(st, D, a, lds, nullptr, 0, occ);
        default: return hipErrorInvalidValue;
      }
    }
    return hipErrorInvalidValue;
  }
  if (sh) {
    switch (D.C) {
      case 1: return launch_tiles_c<1, NT, 0, 1>(st, D, a, lds, sh, grid, occ);
      case 2: return launch_tiles_c<2, NT, 0, 1>(st, D, a, lds, sh, grid, occ);
      case 3: return launch_tiles_c<3, NT, 0, 1>(st, D, a, lds, sh, grid, occ);
      case 4: return launch_tiles_c<4, NT, 0, 1>(st, D, a, lds, sh, grid, occ);
      default: return hipErrorInvalidValue;
    }
  }
  if (D.dbg && D.probe == 1) {
    switch (D.C) {
      case 1: return launch_tiles_c<1, NT, 1, 0>(st, D, a, lds, nullptr, 0, occ);
      case 3: return launch_tiles_c<3, NT, 1, 0>(st, D, a, lds, nullptr, 0, occ);
      default: break;
    }
  }
  if (D.dbg && D.probe == 2) {
    switch (D.C) {
      case 1: return launch_tiles_c<1, NT, 2, 0>(st, D, a, lds, nullptr, 0, occ);
      case 3: return launch_tiles_c<3, NT, 2, 0>(st, D, a, lds, nullptr, 0, occ);
      default: break;
    }
  }
  switch (D.C) {
    case 1: return launch_tiles_c<1, NT, 0, 0>(st, D, a, lds, nullptr, 0, occ);
    case 2: return launch_tiles_c<2, NT, 0, 0>(st, D, a, lds, nullptr, 0, occ);
    case 3: return launch_tiles_c<3, NT, 0, 0>(st, D, a, lds, nullptr, 0, occ);
    case 4: return launch_tiles_c<4, NT, 0, 0>(st, D, a, lds, nullptr, 0, occ);
    default: return hipErrorInvalidValue;
  }
}

// chain-split launch (256-thread tiles, one chain per workgroup, D.C per CU)
template <int CS>
static hipError_t launch_tiles_cs(hipStream_t st, const TileDev& D, const TileLaunch& a, int lds, int* occ) {
  constexpr int NT = 256;
  auto k = sweep_tiles_cs_kernel<CS, NT, tile_rmax_cs(NT), tile_gmax(NT)>;
  // LDS floor: at most CS workgroups per CU
  const int floor = kTileCuLds / (CS + 1) + 64;
  lds = lds < floor ? floor : lds;
  if (lds * CS > kTileCuLds) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  if (occ) return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, reinterpret_cast<const void*>(k), NT, lds);
  hipLaunchKernelGGL(tile_call_bump_kernel, dim3(1), dim3(1), 0, st, D.ctl);
  hipLaunchKernelGGL(k, dim3(D.T * CS), dim3(NT), lds, st, D, a);
  return hipGetLastError();
}

hipError_t launch_sweep_tiles_cs(hipStream_t st, const TileDev& D, const TileLaunch& a, int max_rows, int NT,
                                 int max_batches, int max_gslots, int* occ) {
  if (NT != 256 || D.rg || D.batch_split || D.dbg) return hipErrorInvalidValue;
  const int lds = tile_lds_bytes(max_rows, 1, NT, D.K, max_batches, max_gslots);
  switch (D.C) {
    case 2: return launch_tiles_cs<2>(st, D, a, lds, occ);
    case 3: return launch_tiles_cs<3>(st, D, a, lds, occ);
    case 4: return launch_tiles_cs<4>(st, D, a, lds, occ);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_sweep_tiles(hipStream_t st, const TileDev& D, const TileLaunch& a, int max_rows, int NT,
                              int max_batches, int max_gslots, const TileShard* sh, int grid, int* occ) {
  const int lds = tile_lds_bytes(D.rg ? 0 : max_rows, D.C, NT, D.K, max_batches, max_gslots);
  switch (NT) {
    case 256: return launch_tiles_nt<256>(st, D, a, lds, sh, grid, occ);
    case 512: return launch_tiles_nt<512>(st, D, a, lds, sh, grid, occ);
    case 1024: return launch_tiles_nt<1024>(st, D, a, lds, sh, grid, occ);
    default: return hipErrorInvalidValue;
  }
}

// B values of chain `chain` into the tile layout + precision_diag (column
// sums of squares in stream = row order, as sell_refresh).  Work items
// (order[], built with the layout): an own batch (cell f of the batch at
// off + (f % R)*NT + f / R; NT = the layout's threads per tile) or a run of
// <= 2048 ghost cells.  The items of a tile read Linv rows of that tile (a
// contiguous device-row range), so the items are dealt to the XCDs by tile:
// block b runs item b / 8 of list b % 8 (the dispatcher's round robin over
// the 8 XCDs; speed only), and each list holds whole tiles of a contiguous
// tile range -- a tile's rows are fetched into ONE L2 and every Linv line is
// read from HBM about once instead of once per cell
__global__ __launch_bounds__(256) void tile_refresh_kernel(TileDev D, const int4* __restrict__ order, int olen,
                                                           int NT, const int* __restrict__ cell_src,
                                                           const int* __restrict__ gsrc,
                                                           const double* __restrict__ linv, int chain) {
  __shared__ double sq[kRefreshCells];
  __shared__ unsigned char endf[kRefreshCells];
  __shared__ int4 bsh[kRefreshCells / 64];
  // U independent gathers in flight per thread
  constexpr int U = 8;
  const int t = threadIdx.x;
  const int4 o = order[(size_t)(blockIdx.x % kRefreshLists) * olen + blockIdx.x / kRefreshLists];
  if (o.x == 2) return;
  if (o.x == 1) {  // ghost cells [o.y, o.z)
    double* gv = const_cast<double*>(D.gval) + (size_t)chain * D.n_gcells;
    for (int g0 = o.y + t; g0 < o.z; g0 += U * 256) {
      int src[U];
      double v[U];
#pragma unroll
      for (int q = 0; q < U; ++q) src[q] = g0 + q * 256 < o.z ? __builtin_nontemporal_load(gsrc + g0 + q * 256) : -1;
#pragma unroll
      for (int q = 0; q < U; ++q) v[q] = src[q] >= 0 ? linv[src[q]] : 0.0;
#pragma unroll
      for (int q = 0; q < U; ++q)
        if (g0 + q * 256 < o.z) gv[g0 + q * 256] = v[q];
    }
    return;
  }
  // a run of o.z consecutive batches of one tile (wave-local batches are small:
  // several per item), their cells one contiguous range of the stream
  const int4 B0 = D.batch[o.y], BL = D.batch[o.y + o.z - 1];
  double* cv = const_cast<double*>(D.cell_val) + (size_t)chain * D.n_cells;
  const int ncell = BL.x + (BL.y & 0xFFFF) * NT - B0.x;
  for (int e00 = t; e00 < ncell; e00 += U * 256) {
    int src[U];
    unsigned pk[U];
    double v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e0 = e00 + q * 256;
      src[q] = e0 < ncell ? __builtin_nontemporal_load(cell_src + B0.x + e0) : -1;
      pk[q] = e0 < ncell ? __builtin_nontemporal_load(D.cell_pk + B0.x + e0) : 0u;
    }
#pragma unroll
    for (int q = 0; q < U; ++q) v[q] = src[q] >= 0 ? linv[src[q]] : 0.0;
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int e0 = e00 + q * 256;
      if (e0 < ncell) {
        cv[B0.x + e0] = v[q];
        sq[e0] = v[q] * v[q];
        endf[e0] = (pk[q] & kTEnd) ? 1 : 0;
      }
    }
  }
  // the item's batch descriptors in LDS (a run of <= kRefreshCells / 64
  // wave-local batches): each slot finds its batch by a binary search there
  // instead of a chain of dependent global loads
  for (int i = t; i < o.z; i += 256) bsh[i] = D.batch[o.y + i];
  __syncthreads();
  // per slot: the sum of squares of its cells in stream order f (cell f of a
  // batch at (f % R) * NT + f / R, stepped incrementally)
  const int nslots = BL.w + BL.z - B0.w;
  for (int u = t; u < nslots; u += 256) {
    const int x = B0.w + u;
    int lo = 0, hi = o.z - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (bsh[mid].w <= x) lo = mid;
      else hi = mid - 1;
    }
    const int4 B = bsh[lo];
    const int R = B.y & 0xFFFF, rel = B.x - B0.x;
    const int f0 = D.sinfo[x].y & 0xFFFFF;
    int fj = f0 % R, ft = f0 / R;
    double s = 0.0;
    for (;;) {
      const int e = rel + fj * NT + ft;
      s += sq[e];
      if (endf[e]) break;
      if (++fj == R) { fj = 0; ++ft; }
    }
    D.dr[(size_t)x * D.C + chain].x = s;
  }
}

std::vector<int4> tile_refresh_order(const std::vector<int>& batch_ptr, const std::vector<int>& gptr,
                                     const std::vector<TileBatch>& batch, int NT, int T, int K, int& olen) {
  std::vector<std::vector<int4>> lists(kRefreshLists);
  for (int t = 0; t < T; ++t) {
    std::vector<int4>& l = lists[(size_t)t * kRefreshLists / T];
    // runs of consecutive batches of the tile with at most kRefreshCells cells
    const int q1 = batch_ptr[(size_t)(t + 1) * K];
    for (int q = batch_ptr[(size_t)t * K]; q < q1;) {
      int nb = 0, cells = 0;
      while (q + nb < q1 && (nb == 0 || cells + batch[q + nb].R * NT <= kRefreshCells)) cells += batch[q + nb++].R * NT;
      l.push_back(make_int4(0, q, nb, 0));
      q += nb;
    }
    const int g1 = gptr[(size_t)(t + 1) * K];
    for (int g = gptr[(size_t)t * K]; g < g1; g += 2048) l.push_back(make_int4(1, g, std::min(g + 2048, g1), 0));
  }
  olen = 0;
  for (const auto& l : lists) olen = std::max(olen, (int)l.size());
  std::vector<int4> order((size_t)kRefreshLists * std::max(olen, 1), make_int4(2, 0, 0, 0));
  for (int x = 0; x < kRefreshLists; ++x)
    for (size_t j = 0; j < lists[x].size(); ++j) order[(size_t)x * olen + j] = lists[x][j];
  return order;
}

hipError_t launch_tile_refresh(hipStream_t st, const TileDev& D, const int4* order, int olen, int NT,
                               const int* cell_src, const int* gsrc, const double* linv, int chain) {
  if (olen == 0) return hipSuccess;
  hipLaunchKernelGGL(tile_refresh_kernel, dim3(kRefreshLists * olen), dim3(256), 0, st, D, order, olen, NT, cell_src,
                     gsrc, linv, chain);
  return hipGetLastError();
}

}  // namespace nngp
