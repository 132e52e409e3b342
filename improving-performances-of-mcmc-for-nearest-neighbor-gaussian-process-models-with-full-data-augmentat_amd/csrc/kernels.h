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

struct SweepDev {  // device pointers of the sliced-ELL layout
  const int* chunk_slot0;
  const int* chunk_len;
  const long long* chunk_off;
  const int* collen;
  const int* slot_loc;
  const double* ent_val;
  const int* ent_rowpos;
  const double* D_slot;
  const double* R_slot;
  const int* nobs_slot;
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
// If out != nullptr, out[perm ? perm[k] : k] = u_k.  Returns #blocks used.
int launch_row_stats(hipStream_t st, const double* linv, const int* nn, int n, int b,
                     const double* x, double shift, double* out, const int* perm,
                     double* partials /* kRedBlocks x 4 */,
                     const double* shift_dev = nullptr /* overrides shift when set */);
// reduce `nblocks` x 4 partials into res[4] (deterministic order)
hipError_t launch_reduce4(hipStream_t st, const double* partials, int nblocks, double* res);

hipError_t launch_sell_refresh(hipStream_t st, const int* chunk_slot0, const long long* chunk_off,
                               int nchunks, const int* slot_chunk_end_unused, const int* collen,
                               int n, const int* ent_src, const double* linv, double* ent_val,
                               double* D_slot);

hipError_t launch_residual_sums(hipStream_t st, int n, const int* slot_loc, const int* obs_ptr,
                                const int* obs_idx, const double* y, const double* mu,
                                double beta0, double* R_slot);

hipError_t launch_field_to_slots(hipStream_t st, int n, const int* slot_loc, const double* field,
                                 const SweepScalars* sc, double* w_slot);
hipError_t launch_slots_to_field(hipStream_t st, int n, const int* slot_loc, const double* w_slot,
                                 const SweepScalars* sc, double* field);

hipError_t launch_sweep_color(hipStream_t st, const SweepDev& L, int chunk_begin, int nchunks_color,
                              int slot_end, const SweepScalars* sc, int sweep_local,
                              const double* z, int n);

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

hipError_t launch_normals(hipStream_t st, uint64_t seed, uint64_t sweep, int n, double* z);

}  // namespace nngp
