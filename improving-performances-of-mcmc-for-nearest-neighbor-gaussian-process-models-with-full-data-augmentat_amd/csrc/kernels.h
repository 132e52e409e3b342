// Launch wrappers for the NNGP HIP kernels (gfx950).  Internal C++ header.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace nngp {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kRedBlocks = 1024;  // max partial blocks of a reduction

// scalars read by the sweep kernels from device memory (graph-replay safe)
struct SweepScalars {
  double inv_s2;     // exp(-log_scale)
  double inv_t2;     // exp(-log_noise_variance)
  double beta0;
  double pad;
  uint64_t seed;
  uint64_t counter_base;
};

constexpr int kSweepRows = 16;  // == kRowsMax of the layout planner

// one wavefront's chunk of the sweep layout, loaded with one 16-byte scalar load
struct __attribute__((aligned(16))) ChunkMeta {
  int slot0;       // first slot (a valid slot of the chunk)
  int packed;      // rows | min(nslot,255) << 8 | max_lk << 16
  long long off;   // first entry
};
// per-slot constants of the sweep, one 32-byte record per slot
struct __attribute__((aligned(32))) SlotData {
  double D;        // precision_diag
  double R;        // residuals_sum
  int nobs;        // obs_per_loc
  int loc;         // location index (0-based, Vecchia order)
  int collen;      // length of column loc of B
  int dpos;        // device row of the location (Morton rank)
};

struct SweepDev {  // device pointers of the sliced-ELL layout
  const ChunkMeta* meta;
  const int* lane_tab;      // nchunks x 64: (slot + 1) | lk << 28, 0 = idle
  SlotData* slots;
  const double* ent_val;
  const int* ent_rowpos;
  double* w_slot;
  double* r;
};

// coordinate transform into the isotropic unit-range space (per covfun)
hipError_t launch_scale_coords(hipStream_t st, int covfun, const double* cp, int ncp,
                               const double* locs_rm, int n, int d, double* sc, int ds_stride);

// Vecchia factor: Linv (row-major n x b) from scaled coords.  fail: device int
// (0 = ok, else 1 + first failing row; atomicMin semantics).
hipError_t launch_factor(hipStream_t st, int family, double var, double nugget, double nu,
                         const double* sc, int ds, const int* nn, int n, int b, double* linv,
                         int* fail);

// per-row statistics of B x (x shifted): partial sums of
// {log L[k][0], u_k^2, a_k^2, a_k*u_k} with u = B (x - shift), a = B 1.
// If out != nullptr, out[k] = u_k.  All arrays in device row order.
// Returns #blocks used.
int launch_row_stats(hipStream_t st, const double* linv, const int* nn, int n, int b,
                     const double* x, double shift, double* out,
                     double* partials /* kRedBlocks x 4 */,
                     const double* shift_dev = nullptr /* overrides shift when set */);
// reduce `nblocks` x 4 partials into res[4] (deterministic order)
hipError_t launch_reduce4(hipStream_t st, const double* partials, int nblocks, double* res);

hipError_t launch_sell_refresh(hipStream_t st, const SweepDev& L, int nchunks, const int* ent_src,
                               const double* linv, double* ent_val);

hipError_t launch_residual_sums(hipStream_t st, int n, SlotData* slots, const int* obs_ptr,
                                const int* obs_idx, const double* y, const double* mu, double beta0);

hipError_t launch_field_to_slots(hipStream_t st, int n, const int* slot_dpos, const double* field,
                                 const SweepScalars* sc, double* w_slot);
hipError_t launch_slots_to_field(hipStream_t st, int n, const int* slot_dpos, const double* w_slot,
                                 const SweepScalars* sc, double* field);

hipError_t launch_sweep_color(hipStream_t st, const SweepDev& L, int chunk_begin, int nchunks_color,
                              const SweepScalars* sc, int sweep_local, const double* z, int n);

// all colours of n_sweeps sweeps in one persistent launch (grid = T tiles,
// T <= #CUs); progress[T] must be zero and *err zero before the launch.
hipError_t launch_sweep_persistent(hipStream_t st, const SweepDev& L, const int* tile_chunks, int T, int K,
                                   int n_sweeps, const int* nbr_ptr, const int* nbr_idx, int* progress,
                                   int* err, const SweepScalars* sc, const double* z, int n);

// obs reductions: mode 0 -> partial[0] += (y - f[loc] - mu + beta0)^2
//                 mode 1 -> partial[0] += ((y-b)^2 - (y-a)^2) / (2 sd^2),
//                           a = fnew[loc]+mu-beta0, b = f[loc]+mu-beta0
int launch_obs_reduce(hipStream_t st, int mode, int n_obs, const double* y, const double* mu,
                      double beta0, const int* locs_match0, const double* field,
                      const double* field_new, double inv_2var, double* partials);

hipError_t launch_tri_level(hipStream_t st, const int* rows, int nrows, const double* linv,
                            const int* nn, int b, const double* u, double* x);
hipError_t launch_axpby_shift(hipStream_t st, int n, const double* x, double scale, double shift,
                              double* y);

// x[0..n) = v (a kernel node, replayed with the graph)
hipError_t launch_fill_int(hipStream_t st, int* x, int n, int v);

// busy-wait on the device for `seconds` (bounded; measurement helper)
hipError_t launch_spin(hipStream_t st, double seconds);

hipError_t launch_normals(hipStream_t st, uint64_t seed, uint64_t sweep, int n, double* z);

}  // namespace nngp
