// HIP kernels of the NNGP chromatic-Gibbs hot path, written for gfx950
// (MI355X, CDNA4: wave64, 256 CUs in 8 XCDs).  fp64 throughout.
//
// Kernel map (SURVEY.md §8a ids):
//   scale_coords_kernel / factor_kernel  A4  GpGp::vecchia_Linv
//   row_stats_kernel + reduce4_kernel    A6  ll_compressed_sparse_chol, B x, beta_0 stats
//   spmv_chains_kernel                   A1  r = B w of every chain at the start of a sweep call
//   sell_refresh_kernel / tile_refresh   A5  B values in sweep layout + precision_diag
//   residual_sums_kernel                 A7  residuals_sum
//   sweep_tiles_kernel                   A1  the chromatic sweep, one persistent launch per call (default)
//   sweep_color_kernel                   A1  one colour of the chromatic sweep (fallback)
//   shard_ghost_kernel                   A1  colour-sharded sweep: halo updates after the exchange
//   field/slots_to_*_multi_kernel        A1  field <-> compact slot order, every chain
//   obs_reduce_kernel                    A8  SSR, dnorm ratio
//   tri_level_kernel / _levels_block     (next) Matrix::solve by DAG level
#include "kernels.h"
#include "device_common.h"
#include <climits>
#include <cstdlib>

#include <cmath>

namespace nngp {


__global__ void normals_kernel(uint64_t seed, uint64_t sweep, int n, double* z) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) z[i] = normal_loc(seed, sweep, (uint32_t)i);
}

// ------------------------------------------------------------------ Bessel K
// K_nu(x) for the general Matern correlation (x > 0, nu >= 0; relative error
// <= 1e-14 against 40-digit mpmath over nu in [0, 2.5], x in [1e-8, 690]).
// nu = l + mu, |mu| <= 1/2; K_mu and K_{mu+1} from
//  * x <= 1.5: Temme's series (N. M. Temme, J. Comput. Phys. 19 (1975)
//    324-337): with c_k = (x^2/4)^k / k!, K_mu = sum_k c_k f_k and
//    K_{mu+1} = (2/x) sum_k c_k (p_k - k f_k), where
//    f_k = (k f_{k-1} + p_{k-1} + q_{k-1}) / (k^2 - mu^2), p_k = p_{k-1}/(k - mu),
//    q_k = q_{k-1}/(k + mu), p_0 = (x/2)^-mu Gamma(1+mu)/2,
//    q_0 = (x/2)^mu Gamma(1-mu)/2, f_0 = (mu pi / sin mu pi)
//    [G1(mu) cosh s + G2(mu) ln(2/x) sinh(s)/s], s = mu ln(2/x),
//    G1 = (1/Gamma(1-mu) - 1/Gamma(1+mu)) / (2 mu), G2 = (1/Gamma(1-mu) + 1/Gamma(1+mu)) / 2;
//  * x > 1.5: K_mu(x) = sqrt(pi) (2x)^mu e^-x u_0 with u_k = U(mu+1/2+k, 2mu+1, 2x)
//    (Temme 1975, Sec. 3).  u_k is the minimal solution of
//    u_{k-1} = 2(k+x) u_k - ((k+1/2)^2 - mu^2) u_{k+1} (Abramowitz & Stegun
//    13.4.15), taken by backward (Miller) recurrence from k = N; it is
//    normalised by sum_k C_k u_k = (2x)^-(mu+1/2) with C_0 = 1,
//    C_k = C_{k-1} ((k-1/2)^2 - mu^2) / k (from the integral form of U), so
//    K_mu = sqrt(pi/(2x)) e^-x u_0 / sum_k C_k u_k, and
//    K_{mu+1} = K_mu (mu + 1/2 + x + (mu^2 - 1/4) u_1/u_0) / x;
// then K_{k+1} = K_{k-1} + (2k/x) K_k upwards to nu (stable for K).
__device__ void temme_g1g2(double mu, double& g1, double& g2, double& rg_p, double& rg_m) {
  rg_p = 1.0 / tgamma(1.0 + mu);  // 1/Gamma(1+mu)
  rg_m = 1.0 / tgamma(1.0 - mu);  // 1/Gamma(1-mu)
  g2 = 0.5 * (rg_m + rg_p);
  if (fabs(mu) < 0.05) {
    // G1 = -(even part of 1/Gamma(1+z))/... from the Taylor coefficients of
    // 1/Gamma(z) (Abramowitz & Stegun 6.1.34): G1(mu) = -sum_j c_{2j+2} mu^{2j}
    const double m2 = mu * mu;
    g1 = -(0.5772156649015329 +
           m2 * (-0.0420026350340952 +
                 m2 * (-0.0421977345555443 +
                       m2 * (0.0072189432466630 + m2 * (-0.0002152416741149 + m2 * -0.0000201348547807)))));
  } else {
    g1 = (rg_m - rg_p) / (2.0 * mu);
  }
}

__device__ void bessel_k_mu_series(double mu, double x, double& k0, double& k1) {
  const double PI = 3.141592653589793238462643383;
  const double lg = log(2.0 / x), sg = mu * lg;
  double g1, g2, rg_p, rg_m;
  temme_g1g2(mu, g1, g2, rg_p, rg_m);
  const double pm = PI * mu;
  const double fac = pm == 0.0 ? 1.0 : pm / sin(pm);
  const double shs = sg == 0.0 ? 1.0 : sinh(sg) / sg;
  double f = fac * (g1 * cosh(sg) + g2 * lg * shs);
  const double es = exp(sg);
  double p = 0.5 * es / rg_p, q = 0.5 / (es * rg_m);
  const double y = 0.25 * x * x;
  double c = 1.0, s0 = f, s1 = p;
  for (int k = 1; k < 80; ++k) {
    const double dk = (double)k;
    f = (dk * f + p + q) / (dk * dk - mu * mu);
    p /= dk - mu;
    q /= dk + mu;
    c *= y / dk;
    s0 += c * f;
    s1 += c * (p - dk * f);
    if (fabs(c * f) < 1e-17 * fabs(s0)) break;
  }
  k0 = s0;
  k1 = 2.0 * s1 / x;
}

__device__ void bessel_k_mu_miller(double mu, double x, double& k0, double& k1) {
  const double PI = 3.141592653589793238462643383;
  const int N = min(100, 12 + (int)(160.0 / x));
  const double m2 = mu * mu;
  double un = 0.0, u = 1e-200, acc = 1e-200, u1 = 0.0;  // u_{k+1}, u_k, sum_{j>=k} (C_j/C_k) u_j
  for (int k = N; k >= 1; --k) {
    const double dk = (double)k;
    const double um = 2.0 * (dk + x) * u - ((dk + 0.5) * (dk + 0.5) - m2) * un;
    acc = um + ((dk - 0.5) * (dk - 0.5) - m2) / dk * acc;
    un = u;
    u = um;
    if (fabs(u) > 1e200) { u *= 1e-200; un *= 1e-200; acc *= 1e-200; }
  }
  u1 = un;
  k0 = sqrt(PI / (2.0 * x)) * exp(-x) * (u / acc);
  k1 = k0 * (mu + 0.5 + x + (m2 - 0.25) * (u1 / u)) / x;
}

__device__ double bessel_k(double nu, double x) {
  const int l = (int)(nu + 0.5);
  const double mu = nu - l;
  double k0, k1;
  if (x <= 1.5) bessel_k_mu_series(mu, x, k0, k1);
  else bessel_k_mu_miller(mu, x, k0, k1);
  for (int k = 1; k <= l; ++k) {
    const double t = k0 + 2.0 * (mu + k) / x * k1;
    k0 = k1;
    k1 = t;
  }
  return k0;
}

// 2^(j/64), j = 0..63, correctly rounded (staged into LDS by the factor kernel)
__constant__ double kExp2Tab[64] = {
    1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951};

// exp(x) for x <= 0 (the factor's correlations): x = (64 m + j) ln2/64 + r,
// |r| <= ln2/128, exp(x) = 2^m 2^(j/64) e^r with e^r - 1 by a degree-6
// Taylor polynomial of degree 5 (truncation r^6/720 <= 3.5e-17 for
// |r| <= ln2/128, below half an ulp); within 1 ulp of the correctly rounded
// exp (measured, scripts/micro/dmath.hip).  Very negative x (including the
// padding distances of ~1e30) gives exactly 0.
__device__ __forceinline__ double exp_nonpos(double x, const double* tab) {
  const double k = __builtin_rint(x * 92.33248261689366);  // 64/ln2
  double r = __builtin_fma(-k, 0.010830424696249145, x);    // ln2/64, high part
  r = __builtin_fma(-k, 3.623510646634843e-19, r);          // low part
  const int ki = (int)k;                                      // saturates for huge |x|
  double p = 8.3333333333333332e-03;
  p = __builtin_fma(p, r, 4.1666666666666664e-02);
  p = __builtin_fma(p, r, 1.6666666666666666e-01);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  const double t = tab[ki & 63];
  return __builtin_ldexp(__builtin_fma(p * r, t, t), ki >> 6);
}

// sqrt(s) for s >= 0 (squared distances): hardware rsq (~2^-24) and two
// residual corrections; correctly rounded on every sample measured.  The
// rsq argument is floored at 1e-300 so that coinciding points (s = 0, whose
// correlation is 1: a PD local covariance with a nugget) give exactly 0
// instead of 0 x inf.
__device__ __forceinline__ double sqrt_pos(double s) {
  const double y = __builtin_amdgcn_rsq(__builtin_fmax(s, 1e-300));
  const double h = 0.5 * y;
  double g = s * y;
  double e = __builtin_fma(-g, g, s);
  g = __builtin_fma(e, h, g);
  e = __builtin_fma(-g, g, s);
  return __builtin_fma(e, h, g);
}


// correlation at unit-range distance dist.  FAM 0: exponential, 1: Matern 3/2,
// 2: general Matern with norm = 2^(1-nu)/Gamma(nu)
template <int FAM>
__device__ __forceinline__ double corr(double dist, double nu, double norm) {
  if (FAM == 0) return exp(-dist);
  if (FAM == 1) return (1.0 + dist) * exp(-dist);
  if (dist == 0.0) return 1.0;
  return norm * pow(dist, nu) * bessel_k(nu, dist);
}

// ------------------------------------------------------------------ A4
__device__ __forceinline__ void scale_point(const ScaleArgs& a, const double* __restrict__ locs, int i, int d,
                                            double* __restrict__ sc, int ds) {
  double x[4] = {0, 0, 0, 0}, o[4] = {0, 0, 0, 0};
  for (int k = 0; k < d && k < 4; ++k) x[k] = locs[(size_t)i * d + k];
  switch (a.covfun) {
    case 1:
    case 5: {  // lon/lat degrees -> unit sphere, chordal distance, range in radii
      const double deg = 3.14159265358979323846 / 180.0;
      double lon = x[0] * deg, lat = x[1] * deg;
      o[0] = cos(lat) * cos(lon) / a.c[1];
      o[1] = cos(lat) * sin(lon) / a.c[1];
      o[2] = sin(lat) / a.c[1];
      break;
    }
    case 2:
    case 6:
      for (int k = 0; k < d; ++k) o[k] = x[k] / a.c[1 + k];
      break;
    case 3:
    case 7:
      for (int k = 0; k < d - 1; ++k) o[k] = x[k] / a.c[1];
      o[d - 1] = x[d - 1] / a.c[2];
      break;
    default:
      for (int k = 0; k < d; ++k) o[k] = x[k] / a.c[1];
  }
  for (int k = 0; k < ds; ++k) sc[(size_t)i * ds + k] = o[k];
}

__global__ void scale_coords_kernel(ScaleArgs a, const double* __restrict__ locs, int n, int d,
                                    double* __restrict__ sc, int ds) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  scale_point(a, locs, i, d, sc, ds);
}

// every job's scaled coordinates (blockIdx.y = job) and its failure flag reset
__global__ void scale_coords_jobs_kernel(FactorJobs J, const double* __restrict__ locs, int n, int d, int ds) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  switch (blockIdx.y) {  // constant indices into the kernel argument
#define NNGP_SCALE_JOB(k)                                  \
    case k:                                                \
      if (i == 0) *J.fail[k] = INT_MAX;                    \
      scale_point(J.sa[k], locs, i, d, J.sc[k], ds);       \
      break;
    NNGP_SCALE_JOB(0)
    NNGP_SCALE_JOB(1)
    NNGP_SCALE_JOB(2)
    NNGP_SCALE_JOB(3)
#undef NNGP_SCALE_JOB
  }
}

hipError_t launch_scale_coords(hipStream_t st, int covfun, const double* cp, int ncp,
                               const double* locs_rm, int n, int d, double* sc, int ds) {
  ScaleArgs a;
  for (int k = 0; k < 8; ++k) a.c[k] = k < ncp ? cp[k] : 0.0;
  a.covfun = covfun;
  int g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(scale_coords_kernel, dim3(g), dim3(kBlock), 0, st, a, locs_rm, n, d, sc, ds);
  return hipGetLastError();
}

// One lane per Vecchia row i (GpGp::vecchia_Linv semantics): the local
// covariance of locsub = locs[rev(NNarray[i,1:bs])] (self last) is factored
// by an up-looking Cholesky held entirely in registers (compile-time indices);
// rows of a short neighbourhood (bs < BM) are padded IN FRONT with identity
// rows, which leaves the real block's factor and solution unchanged.
// Linv[i, j] = x[BM-1-j] with L^T x = e_last.
// One row of the factor from its neighbour coordinates xa(r, k) (locsub
// order: the point itself last) and its count of valid neighbours bs.
// The Cholesky runs on the correlation scale (K = C / var: off-diagonal
// correlations, diagonal 1 + nugget) and the solution is scaled by
// rsv = 1/sqrt(var) at the end (chol(var K) = sqrt(var) chol(K)): one multiply
// per output instead of one per covariance entry.
template <int BM, int FAM, int DS, int V, class XA>
__device__ __forceinline__ void factor_row(const XA& xa, int bs, int i, double rsv, double nugget, int b,
                                           const double* __restrict__ tab, double* __restrict__ linv,
                                           int* __restrict__ fail) {
  constexpr int T = BM * (BM + 1) / 2;
  double L[T];
  double inv[BM];
  bool bad = false;
  // row t of the local covariance, then row t of its Cholesky factor
  // (left-looking).  No masks: padded rows sit ~1e30 away from everything
  // (gather_coords), so their correlations come out exactly 0.
#pragma unroll
  for (int t = 0; t < BM; ++t) {
    const bool dt = (BM - 1 - t) >= bs;
#pragma unroll
    for (int q = 0; q < t; ++q) {
      double s2 = 0.0;
#pragma unroll
      for (int k = 0; k < DS; ++k) {
        const double u = xa(t, k) - xa(q, k);
        s2 = __builtin_fma(u, u, s2);
      }
      const double dist = sqrt_pos(s2);
      const double e = exp_nonpos(-dist, tab);
      L[t * (t + 1) / 2 + q] = FAM == 1 ? __builtin_fma(dist, e, e) : e;
    }
#pragma unroll
    for (int q = 0; q <= t; ++q) {
      double s = q == t ? (dt ? 1.0 : 1.0 + nugget) : L[t * (t + 1) / 2 + q];
      if (V & 1) {  // two partial sums: half the dependent chain
        double s1 = 0.0;
#pragma unroll
        for (int p = 0; p < q; ++p) {
          if (p & 1) s1 -= L[t * (t + 1) / 2 + p] * L[q * (q + 1) / 2 + p];
          else s -= L[t * (t + 1) / 2 + p] * L[q * (q + 1) / 2 + p];
        }
        s += s1;
      } else {
#pragma unroll
        for (int p = 0; p < q; ++p) s -= L[t * (t + 1) / 2 + p] * L[q * (q + 1) / 2 + p];
      }
      if (q < t) {
        L[t * (t + 1) / 2 + q] = s * inv[q];
      } else {
        if (!(s > 0.0)) { bad = true; s = 1.0; }
        const double ri = rsqrt_pos(s);
        L[t * (t + 1) / 2 + t] = s * ri;
        inv[t] = ri;
      }
    }
  }
  double x[BM];
  x[BM - 1] = inv[BM - 1];
#pragma unroll
  for (int r = BM - 2; r >= 0; --r) {
    double s = 0.0;
#pragma unroll
    for (int q = r + 1; q < BM; ++q) s -= L[q * (q + 1) / 2 + r] * x[q];
    x[r] = s * inv[r];
  }
  if (bad) atomicMin(fail, i + 1);
#pragma unroll
  for (int j = 0; j < BM; ++j)
    if (j < b) linv[(size_t)i * b + j] = (j < bs) ? x[BM - 1 - j] * rsv : 0.0;
}

// neighbour indices of row i (clamped to n-1; entries j >= b read as -1)
template <int BM>
__device__ __forceinline__ void load_nn_row(int (&nc)[BM], const int* __restrict__ nn, int i, int n, int b) {
  const int r = i < n ? i : n - 1;
#pragma unroll
  for (int j = 0; j < BM; ++j) nc[j] = j < b ? __builtin_nontemporal_load(nn + (size_t)r * b + j) : -1;
}

// coordinates feeding locsub row r = NNarray column BM-1-r (missing
// neighbours: distinct points ~1e30 away); returns the valid count bs
template <int BM, int DS>
__device__ __forceinline__ int gather_coords(double (&X)[BM][DS], const int (&nc)[BM],
                                             const double* __restrict__ sc, int i, int n) {
  const int self = i < n ? i : n - 1;
  int bs = 1;
#pragma unroll
  for (int j = 1; j < BM; ++j)
    if (nc[j] >= 0) bs = j + 1;
#pragma unroll
  for (int r = 0; r < BM; ++r) {
    const int j = BM - 1 - r;
    const int idx = (j < bs) ? nc[j] : self;
#pragma unroll
    for (int k = 0; k < DS; ++k) {
      const double v = sc[(size_t)idx * DS + k];
      X[r][k] = (j < bs) ? v : (k == 0 ? 1e30 * (r + 1) : 0.0);  // padding: far apart from all
    }
  }
  return bs;
}

// the job's entry of a per-job kernel-argument array (wave-uniform j; a
// select chain keeps the argument in scalar registers instead of a private copy)
template <class T>
__device__ __forceinline__ T job_pick(const T (&v)[kMaxChains], int j) {
  return j == 0 ? v[0] : j == 1 ? v[1] : j == 2 ? v[2] : v[3];
}

// Grid-stride over groups of 64 rows with a two-deep software pipeline: the
// next group's coordinate gathers and the group after's neighbour indices
// are in flight while this group's covariance/Cholesky runs (one wave per
// SIMD fits the register footprint, so no other wave hides that latency).
// The groups of all jobs (chains) form one range: group g is rows
// (g mod G) * 64 + lane of job g / G, G = ceil(n / 64).
template <int BM, int FAM, int DS, int V>
__global__ __launch_bounds__(64) void factor_kernel(FactorJobs J, double nu, double norm,
                                                   const int* __restrict__ nn, int n, int b) {
  __shared__ double tab[64];
  tab[threadIdx.x] = kExp2Tab[threadIdx.x];
  __syncthreads();
  const int G = (n + 63) / 64, total = G * J.n_jobs;
  const int stride = gridDim.x;
  auto row_of = [&](int g, int& jb) {  // past the last group: row n (no work), last job
    if (g >= total) {
      jb = J.n_jobs - 1;
      return n;
    }
    jb = g / G;
    return (g - jb * G) * 64 + (int)threadIdx.x;
  };
  int nc[BM], nx[BM];
  double X[BM][DS];
  int g = blockIdx.x, jc, jn;
  int i = row_of(g, jc);
  load_nn_row<BM>(nc, nn, i, n, b);
  int bs = gather_coords<BM, DS>(X, nc, job_pick(J.sc, jc), i, n);
  int i1 = row_of(g + stride, jn);
  load_nn_row<BM>(nx, nn, i1, n, b);
  for (; g < total; g += stride) {
    int j2;
    const int i2 = row_of(g + 2 * stride, j2);
    double Xn[BM][DS];
    const int bsn = gather_coords<BM, DS>(Xn, nx, job_pick(J.sc, jn), i1, n);
    load_nn_row<BM>(nx, nn, i2, n, b);
    if (i < n)
      factor_row<BM, FAM, DS, V>([&](int r, int k) { return X[r][k]; }, bs, i, rsqrt_pos(job_pick(J.var, jc)),
                                 job_pick(J.nugget, jc), b, tab, job_pick(J.linv, jc), job_pick(J.fail, jc));
#pragma unroll
    for (int r = 0; r < BM; ++r)
#pragma unroll
      for (int k = 0; k < DS; ++k) X[r][k] = Xn[r][k];
    bs = bsn;
    i = i1;
    jc = jn;
    i1 = i2;
    jn = j2;
  }
}

// Lane pairs (north star's "a lane group per location"): two lanes per row,
// lane j = 0, 1 of a pair owns the local block's points r = 2k + j (their
// coordinates, 8 of 16 at BM = 16) and the columns p = 2k + j of the
// Cholesky factor L -- half of the register footprint of one lane per row,
// so two waves fit a SIMD instead of one (the one-lane kernel is issue-bound
// at one wave per SIMD, ~60 % issue efficiency).  Same left-looking Cholesky
// on the correlation scale as factor_row: each lane computes the covariance
// entries (t, q) of its columns q, the dot products
// sum_{p < q} L[t][p] L[q][p] are split by the parity of p and the two halves
// added with one DPP swap (IEEE addition commutes: both lanes hold the same
// bits); the owner of column q keeps L[t][q].  The back substitution
// x = L^-T e_last needs no reduction (column r of L lives in one lane); each
// x[r] is swapped to the partner.  The dot products' summation order differs
// from factor_row's (even and odd p separately), so rows differ from the
// one-lane kernel in the last bits, within the factor tolerance.
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true); }
// a cross-lane value stays where it is computed (with every lane of the
// wave active): the compiler would otherwise sink the DPP move into the
// lane-dependent select that uses it, where the partner lane is masked off
// and the move reads 0
__device__ __forceinline__ void pin_full_exec(double& v) { asm volatile("" : "+v"(v)); }

template <int BM, int FAM, int DS>
__global__ __launch_bounds__(64) void factor_pair_kernel(double var, double nugget, double nu, double norm,
                                                        const double* __restrict__ sc,
                                                        const int* __restrict__ nn, int n, int b,
                                                        double* __restrict__ linv, int* __restrict__ fail) {
  static_assert(BM % 2 == 0, "lane pairs: even block size");
  constexpr int H = BM / 2;            // points / columns per lane
  constexpr int TH = H * (H + 1);      // owned entries of the packed lower triangle: sum_t ceil((t+1)/2)
  constexpr int SWAP = 0xB1;           // quad_perm [1,0,3,2]: the pair partner
  __shared__ double tab[64];
  tab[threadIdx.x] = kExp2Tab[threadIdx.x];
  __syncthreads();
  const double rsv = rsqrt_pos(var);
  const int j = threadIdx.x & 1;
  const int stride = gridDim.x * 32;
  for (int base = blockIdx.x * 32; base < n; base += stride) {
    const int i = base + (threadIdx.x >> 1);
    const int row = i < n ? i : n - 1;
    // this lane's points r = 2k + j: NNarray column BM-1-r (self at r = BM-1)
    int nc[H];
#pragma clang loop unroll(full)
    for (int k = 0; k < H; ++k) {
      const int c = BM - 1 - (2 * k + j);
      nc[k] = c < b ? __builtin_nontemporal_load(nn + (size_t)row * b + c) : -1;
    }
    // valid count bs: 1 + the last valid column over both lanes
    int last = 0;
#pragma clang loop unroll(full)
    for (int k = 0; k < H; ++k) {
      const int c = BM - 1 - (2 * k + j);
      if (c >= 1 && nc[k] >= 0 && c > last) last = c;
    }
    int lo = dpp_i32<SWAP>(last);
    asm volatile("" : "+v"(lo));
    const int bs = (last > lo ? last : lo) + 1;
    double Xo[H][DS];
#pragma clang loop unroll(full)
    for (int k = 0; k < H; ++k) {
      const int r = 2 * k + j, c = BM - 1 - r;
      const bool valid = c < bs;
      const int idx = valid ? nc[k] : row;
#pragma clang loop unroll(full)
      for (int d = 0; d < DS; ++d) {
        const double v = sc[(size_t)idx * DS + d];
        Xo[k][d] = valid ? v : (d == 0 ? 1e30 * (r + 1) : 0.0);
      }
    }
    // L[t][2k + j] at off(t) + k, off(t) = sum_{s<t} ceil((s+1)/2); slots a
    // lane does not own in a row (and inv of columns not reached yet) are
    // read only into discarded selects -- zeroed so they are defined
    double L[TH];
    double inv[H];
#pragma clang loop unroll(full)
    for (int e = 0; e < TH; ++e) L[e] = 0.0;
#pragma clang loop unroll(full)
    for (int e = 0; e < H; ++e) inv[e] = 0.0;
    bool bad = false;
#pragma clang loop unroll(full)
    for (int t = 0; t < BM; ++t) {
      const int ot = (t / 2) * (t / 2 + 1) + ((t & 1) ? t / 2 + 1 : 0);  // off(t)
      const bool dt = (BM - 1 - t) >= bs;
      // point t's coordinates in both lanes
      double xt[DS];
#pragma clang loop unroll(full)
      for (int d = 0; d < DS; ++d) {
        const double mine = Xo[t / 2][d];
        double other = dpp_f64<SWAP, 0xF, true>(mine);
        pin_full_exec(other);
        xt[d] = (j == (t & 1)) ? mine : other;
      }
      // covariance entries (t, q), q = 2k + j < t
      double K[H];
#pragma clang loop unroll(full)
      for (int k = 0; k < (t + 1) / 2; ++k) {
        double s2 = 0.0;
#pragma clang loop unroll(full)
        for (int d = 0; d < DS; ++d) {
          const double u = xt[d] - Xo[k][d];
          s2 = __builtin_fma(u, u, s2);
        }
        const double dist = sqrt_pos(s2);
        const double e = exp_nonpos(-dist, tab);
        K[k] = FAM == 1 ? __builtin_fma(dist, e, e) : e;
      }
#pragma clang loop unroll(full)
      for (int q = 0; q <= t; ++q) {
        const int oq = (q / 2) * (q / 2 + 1) + ((q & 1) ? q / 2 + 1 : 0);
        // this lane's half of sum_{p<q} L[t][p] L[q][p]: p = 2k + j < q
        double sp = 0.0;
#pragma clang loop unroll(full)
        for (int k = 0; k < (q + 1) / 2; ++k) {
          const double term = L[ot + k] * L[oq + k];
          // q odd: lane 1's last slot is column q itself (not yet a term)
          sp = (2 * k + 1 >= q && (q & 1) && j == 1) ? sp : sp + term;
        }
        double sw = dpp_f64<SWAP, 0xF, true>(sp);
        pin_full_exec(sw);
        const double s = sp + sw;
        const bool own = (q & 1) == j;
        if (q < t) {
          const double v = (K[q / 2] - s) * inv[q / 2];
          // q even: lane 1's slot q/2 is column q+1 of row t, written at q+1
          if (!(q & 1) || own) L[ot + q / 2] = v;
        } else {
          double dd = (dt ? 1.0 : 1.0 + nugget) - s;
          if (!(dd > 0.0)) { bad = true; dd = 1.0; }
          const double ri = rsqrt_pos(dd);
          if (!(q & 1) || own) {
            L[ot + q / 2] = dd * ri;
            inv[q / 2] = ri;
          }
        }
      }
    }
    // x = L^-T e_last; x[r] lives in both lanes after its owner computes it
    double x[BM];
    {
      const double own = inv[H - 1];  // column BM-1 is odd: lane 1's
      double other = dpp_f64<SWAP, 0xF, true>(own);
      pin_full_exec(other);
      x[BM - 1] = j == 1 ? own : other;
    }
#pragma clang loop unroll(full)
    for (int r = BM - 2; r >= 0; --r) {
      double sacc = 0.0;
#pragma clang loop unroll(full)
      for (int q = r + 1; q < BM; ++q) {
        const int oq = (q / 2) * (q / 2 + 1) + ((q & 1) ? q / 2 + 1 : 0);
        sacc -= L[oq + r / 2] * x[q];  // L[q][r]: column r's owner holds it
      }
      const double mine = sacc * inv[r / 2];
      double other = dpp_f64<SWAP, 0xF, true>(mine);
      pin_full_exec(other);
      x[r] = ((r & 1) == j) ? mine : other;
    }
    if (i < n) {
      if (bad) atomicMin(fail, i + 1);
#pragma clang loop unroll(full)
      for (int k = 0; k < H; ++k) {
        const int c = 2 * k + j;  // output column
        if (c < b) linv[(size_t)i * b + c] = (c < bs) ? x[BM - 1 - c] * rsv : 0.0;
      }
    }
  }
}

// Lane groups (north star's "one wavefront per location" at the DPP-row
// grain, NNGP_FACTOR_LANES=16, b <= 16): the 16 lanes of a DPP row own one
// location's local block, lane q its point q (locsub order, self last) and
// column q of the block.  Each lane computes its whole covariance column from
// the 16 points broadcast across the row (row_newbcast), so the block is
// symmetric bitwise (the squared differences are the same both ways); the
// Cholesky runs right-looking: at step k lane k's column is broadcast,
// scaled by 1/sqrt of its diagonal into L[.][k], and every lane j > k updates
// its column with L[t][k] L[j][k] -- the Schur complement stays in the
// lanes' own registers (L[j][k] is lane j's own entry k by symmetry).  The
// back substitution x = L^-T e_last is sequential in 16 broadcasts: x[r] is
// final in lane r once every x[q > r] has been folded into its running sum.
// Registers: the column (16 doubles), the point (DS), a few scalars -- many
// waves per SIMD where the one-lane-per-row kernel has one.  Rows differ
// from factor_kernel's in the last bits (another operation order), within
// the factor tolerance of the parity tests.
template <int K>
__device__ __forceinline__ double row_bcast(double v) {  // lane K of each row of 16, to the whole row
  return dpp_f64<0x150 + K, 0xF, false>(v);
}

template <int FAM, int DS>
__global__ __launch_bounds__(256) void factor_lanes_kernel(FactorJobs J, const int* __restrict__ nn, int n, int b) {
  constexpr int BM = 16;
  __shared__ double tab[64];
  if (threadIdx.x < 64) tab[threadIdx.x] = kExp2Tab[threadIdx.x];
  __syncthreads();
  const int q = threadIdx.x & 15;
  const long long total = (long long)n * J.n_jobs;
  const long long gstride = (long long)gridDim.x * (blockDim.x >> 4);
  for (long long u = (long long)blockIdx.x * (blockDim.x >> 4) + (threadIdx.x >> 4); u < total; u += gstride) {
    const int jb = (int)(u / n), i = (int)(u - (long long)jb * n);
    const double* sc = job_pick(J.sc, jb);
    // point q = NNarray column c = BM-1-q (column 0: the location itself)
    const int c = BM - 1 - q;
    const int nc = (c < b) ? __builtin_nontemporal_load(nn + (size_t)i * b + c) : -1;
    // bs = 1 + the last valid column (max over the row's lanes)
    int last = (c >= 1 && nc >= 0) ? c : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) last = max(last, __shfl_xor(last, o, 16));
    const int bs = last + 1;
    const bool valid = c < bs;
    double xq[DS];
#pragma unroll
    for (int k = 0; k < DS; ++k) {
      const double v = sc[(size_t)(valid ? nc : i) * DS + k];
      xq[k] = valid ? v : (k == 0 ? 1e30 * (q + 1) : 0.0);  // padding: far apart from all
    }
    // column q of the correlation block (the diagonal 1 + nugget; padded
    // points: an identity row and column)
    const double nug = job_pick(J.nugget, jb);
    double a[BM];
#pragma unroll
    for (int t = 0; t < BM; ++t) {
      double s2 = 0.0;
#pragma unroll
      for (int k = 0; k < DS; ++k) {
        double xt = 0.0;
        switch (t) {  // compile-time lane of the broadcast
#define NNGP_BC(T) case T: xt = row_bcast<T>(xq[k]); break;
          NNGP_BC(0) NNGP_BC(1) NNGP_BC(2) NNGP_BC(3) NNGP_BC(4) NNGP_BC(5) NNGP_BC(6) NNGP_BC(7)
          NNGP_BC(8) NNGP_BC(9) NNGP_BC(10) NNGP_BC(11) NNGP_BC(12) NNGP_BC(13) NNGP_BC(14) NNGP_BC(15)
#undef NNGP_BC
        }
        pin_full_exec(xt);
        const double d = xt - xq[k];
        s2 = __builtin_fma(d, d, s2);
      }
      const double dist = sqrt_pos(s2);
      const double e = exp_nonpos(-dist, tab);
      const double cr = FAM == 1 ? __builtin_fma(dist, e, e) : e;
      a[t] = (t == q) ? (valid ? 1.0 + nug : 1.0) : cr;
    }
    // right-looking Cholesky, lane k's column broadcast at step k
    bool bad = false;
    double inv = 0.0;
#pragma unroll
    for (int k = 0; k < BM; ++k) {
      double dk = 0.0;
      switch (k) {
#define NNGP_BC(T) case T: dk = row_bcast<T>(a[T]); break;
        NNGP_BC(0) NNGP_BC(1) NNGP_BC(2) NNGP_BC(3) NNGP_BC(4) NNGP_BC(5) NNGP_BC(6) NNGP_BC(7)
        NNGP_BC(8) NNGP_BC(9) NNGP_BC(10) NNGP_BC(11) NNGP_BC(12) NNGP_BC(13) NNGP_BC(14) NNGP_BC(15)
#undef NNGP_BC
      }
      pin_full_exec(dk);
      if (!(dk > 0.0)) { bad = true; dk = 1.0; }
      const double rk = rsqrt_pos(dk);
      const double ljk = a[k] * rk;  // L[q][k] (lanes q > k)
#pragma unroll
      for (int t = k + 1; t < BM; ++t) {
        double vt = 0.0;
        switch (k) {
#define NNGP_BC(T) case T: vt = row_bcast<T>(a[t]); break;
          NNGP_BC(0) NNGP_BC(1) NNGP_BC(2) NNGP_BC(3) NNGP_BC(4) NNGP_BC(5) NNGP_BC(6) NNGP_BC(7)
          NNGP_BC(8) NNGP_BC(9) NNGP_BC(10) NNGP_BC(11) NNGP_BC(12) NNGP_BC(13) NNGP_BC(14) NNGP_BC(15)
#undef NNGP_BC
        }
        pin_full_exec(vt);
        const double ltk = vt * rk;  // L[t][k]
        a[t] = q > k ? __builtin_fma(-ltk, ljk, a[t]) : (q == k ? ltk : a[t]);
      }
      if (q == k) {
        a[k] = dk * rk;
        inv = rk;
      }
    }
    // x = L^-T e_last: lane r holds column r of L (a[t], t >= r); running
    // sums s_r += L[q][r] x[q] as each x[q] is broadcast, q = BM-1 .. 0
    double s = 0.0, xr = 0.0;
#pragma unroll
    for (int k = BM - 1; k >= 0; --k) {
      const double mine = k == BM - 1 ? inv : -s * inv;  // x[k] in lane k
      double xk = 0.0;
      switch (k) {
#define NNGP_BC(T) case T: xk = row_bcast<T>(mine); break;
        NNGP_BC(0) NNGP_BC(1) NNGP_BC(2) NNGP_BC(3) NNGP_BC(4) NNGP_BC(5) NNGP_BC(6) NNGP_BC(7)
        NNGP_BC(8) NNGP_BC(9) NNGP_BC(10) NNGP_BC(11) NNGP_BC(12) NNGP_BC(13) NNGP_BC(14) NNGP_BC(15)
#undef NNGP_BC
      }
      pin_full_exec(xk);
      if (q == k) xr = xk;
      s = __builtin_fma(a[k], xk, s);  // lanes q < k: L[k][q] x[k]
    }
    // reduce the failure flag of the row (any lane's pivot) -- every lane
    // saw the same broadcast pivots, so lane 15's flag is the row's
    if (bad && q == BM - 1) atomicMin(job_pick(J.fail, jb), i + 1);
    if (c < b) job_pick(J.linv, jb)[(size_t)i * b + c] = valid ? xr * rsqrt_pos(job_pick(J.var, jb)) : 0.0;
  }
}

// Runtime-b variant (b <= 32, and the general Matern family whose Bessel
// evaluation defeats full unrolling): same algorithm, private arrays indexed
// at run time (held in scratch; correct for every b, slower than the
// register-resident templates above).
constexpr int kBMaxRt = 32;
template <int FAM, int DS>
__global__ __launch_bounds__(64) void factor_kernel_rt(double var, double nugget, double nu, double norm,
                                                      const double* __restrict__ sc,
                                                      const int* __restrict__ nn, int n, int b,
                                                      double* __restrict__ linv, int* __restrict__ fail) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  int bs = b;
  while (bs > 1 && nn[(size_t)i * b + bs - 1] < 0) --bs;
  double X[kBMaxRt][DS];
  double L[kBMaxRt * (kBMaxRt + 1) / 2];
  double inv[kBMaxRt], x[kBMaxRt];
  for (int r = 0; r < bs; ++r) {
    const int idx = nn[(size_t)i * b + (bs - 1 - r)];
    for (int k = 0; k < DS; ++k) X[r][k] = sc[(size_t)idx * DS + k];
  }
  bool bad = false;
  for (int t = 0; t < bs; ++t) {
    for (int q = 0; q <= t; ++q) {
      double c;
      if (q == t) {
        c = var * (1.0 + nugget);
      } else {
        double s2 = 0.0;
        for (int k = 0; k < DS; ++k) {
          double u = X[t][k] - X[q][k];
          s2 += u * u;
        }
        c = var * corr<FAM>(sqrt(s2), nu, norm);
      }
      double s = c;
      for (int p = 0; p < q; ++p) s -= L[t * (t + 1) / 2 + p] * L[q * (q + 1) / 2 + p];
      if (q < t) {
        L[t * (t + 1) / 2 + q] = s * inv[q];
      } else {
        if (!(s > 0.0)) { bad = true; s = 1.0; }
        double l = sqrt(s);
        L[t * (t + 1) / 2 + t] = l;
        inv[t] = 1.0 / l;
      }
    }
  }
  x[bs - 1] = inv[bs - 1];
  for (int r = bs - 2; r >= 0; --r) {
    double s = 0.0;
    for (int q = r + 1; q < bs; ++q) s -= L[q * (q + 1) / 2 + r] * x[q];
    x[r] = s * inv[r];
  }
  if (bad) atomicMin(fail, i + 1);
  for (int j = 0; j < b; ++j) linv[(size_t)i * b + j] = (j < bs) ? x[bs - 1 - j] : 0.0;
}

#define NNGP_FACTOR_ARGS var, nugget, nu, norm, sc, nn, n, b, linv, fail
// workgroups of a grid-stride kernel: NNGP_FACTOR_GRID (default 2) x the
// resident one-wave workgroups of the current device, at most the row
// groups.  Twice resident measured best at n = 1e6 (0.350 vs 0.354 ms at 1x,
// 0.373 at 4x): a shorter last round without giving up the pipeline.
static int resident_grid(const void* kern, int groups, int block = 64) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cus <= 0)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, 0) != hipSuccess || per_cu <= 0) per_cu = 4;
  static const int mult = [] {
    const char* e = std::getenv("NNGP_FACTOR_GRID");
    int v = e ? std::atoi(e) : 2;
    return v >= 1 && v <= 64 ? v : 2;
  }();
  const long long g = (long long)cus * per_cu * mult;
  return (int)(g < groups ? g : groups);
}

static bool factor_lanes_on() {  // read at every launch (tests switch it per context)
  const char* e = std::getenv("NNGP_FACTOR_LANES");
  return e && std::atoi(e) == 16;
}

static hipError_t launch_factor_lanes(hipStream_t st, int family, int ds, const FactorJobs& J, const int* nn, int n,
                                      int b) {
  auto go = [&](auto kern) {
    const long long units = (long long)n * J.n_jobs;
    const int g = resident_grid(reinterpret_cast<const void*>(kern), (int)std::min<long long>((units + 15) / 16, 1 << 30),
                                256);
    hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, st, J, nn, n, b);
    return hipGetLastError();
  };
  if (family == 0) {
    switch (ds) {
      case 2: return go(factor_lanes_kernel<0, 2>);
      case 3: return go(factor_lanes_kernel<0, 3>);
      case 4: return go(factor_lanes_kernel<0, 4>);
    }
  } else {
    switch (ds) {
      case 2: return go(factor_lanes_kernel<1, 2>);
      case 3: return go(factor_lanes_kernel<1, 3>);
      case 4: return go(factor_lanes_kernel<1, 4>);
    }
  }
  return hipErrorInvalidValue;
}

template <int BM, int FAM, int DS>
static hipError_t launch_factor_one(hipStream_t st, double var, double nugget, double nu, double norm,
                                    const double* sc, const int* nn, int n, int b, double* linv, int* fail) {
  if (BM <= 16 && factor_lanes_on()) {
    FactorJobs J;
    J.n_jobs = 1;
    J.var[0] = var;
    J.nugget[0] = nugget;
    J.sc[0] = const_cast<double*>(sc);
    J.linv[0] = linv;
    J.fail[0] = fail;
    return launch_factor_lanes(st, FAM, DS, J, nn, n, b);
  }
  // NNGP_FACTOR_PAIR=1: the lane-pair kernel (opt-in: measured slower)
  if constexpr (BM == 16) {
    const char* pe = std::getenv("NNGP_FACTOR_PAIR");
    if (pe && pe[0] == '1') {
      const auto kp = factor_pair_kernel<BM, FAM, DS>;
      const int g = resident_grid(reinterpret_cast<const void*>(kp), (n + 31) / 32);
      hipLaunchKernelGGL(kp, dim3(g), dim3(64), 0, st, NNGP_FACTOR_ARGS);
      return hipGetLastError();
    }
  }
  FactorJobs J;
  J.n_jobs = 1;
  J.var[0] = var;
  J.nugget[0] = nugget;
  J.sc[0] = const_cast<double*>(sc);
  J.linv[0] = linv;
  J.fail[0] = fail;
  const auto kern = factor_kernel<BM, FAM, DS, 0>;
  const int g = resident_grid(reinterpret_cast<const void*>(kern), (n + 63) / 64);
  hipLaunchKernelGGL(kern, dim3(g), dim3(64), 0, st, J, nu, norm, nn, n, b);
  return hipGetLastError();
}

// all jobs in one factor_kernel launch (the register-resident block sizes)
template <int BM, int FAM>
static hipError_t launch_factor_jobs_bm(hipStream_t st, int ds, double nu, const FactorJobs& J, const int* nn,
                                        int n, int b) {
  const long long groups = (long long)((n + 63) / 64) * J.n_jobs;
  if (groups > INT_MAX / 2) return hipErrorInvalidValue;  // group index arithmetic stays in int
  auto go = [&](auto kern) {
    const int g = resident_grid(reinterpret_cast<const void*>(kern), (int)groups);
    hipLaunchKernelGGL(kern, dim3(g), dim3(64), 0, st, J, nu, 0.0, nn, n, b);
    return hipGetLastError();
  };
  switch (ds) {
    case 2: return go(factor_kernel<BM, FAM, 2, 0>);
    case 3: return go(factor_kernel<BM, FAM, 3, 0>);
    case 4: return go(factor_kernel<BM, FAM, 4, 0>);
    default: return hipErrorInvalidValue;
  }
}

template <int BM, int FAM>
static hipError_t launch_factor_ds(hipStream_t st, int ds, double var, double nugget, double nu,
                                   double norm, const double* sc, const int* nn, int n, int b,
                                   double* linv, int* fail) {
  switch (ds) {
    case 2: return launch_factor_one<BM, FAM, 2>(st, NNGP_FACTOR_ARGS);
    case 3: return launch_factor_one<BM, FAM, 3>(st, NNGP_FACTOR_ARGS);
    case 4: return launch_factor_one<BM, FAM, 4>(st, NNGP_FACTOR_ARGS);
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int FAM>
static hipError_t launch_factor_rt(hipStream_t st, int ds, double var, double nugget, double nu,
                                   double norm, const double* sc, const int* nn, int n, int b,
                                   double* linv, int* fail) {
  int g = (n + 63) / 64;
  switch (ds) {
    case 2: hipLaunchKernelGGL((factor_kernel_rt<FAM, 2>), dim3(g), dim3(64), 0, st, NNGP_FACTOR_ARGS); break;
    case 3: hipLaunchKernelGGL((factor_kernel_rt<FAM, 3>), dim3(g), dim3(64), 0, st, NNGP_FACTOR_ARGS); break;
    case 4: hipLaunchKernelGGL((factor_kernel_rt<FAM, 4>), dim3(g), dim3(64), 0, st, NNGP_FACTOR_ARGS); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_factor(hipStream_t st, int family, double var, double nugget, double nu,
                         const double* sc, int ds, const int* nn, int n, int b, double* linv,
                         int* fail) {
  double norm = 0.0;
  if (b > kBMaxRt || b < 1) return hipErrorInvalidValue;
  if (family == 2) {
    norm = exp((1.0 - nu) * log(2.0) - lgamma(nu));
    return launch_factor_rt<2>(st, ds, NNGP_FACTOR_ARGS);
  }
  if (b <= 16) {
    if (family == 0) {
      if (b <= 8) return launch_factor_ds<8, 0>(st, ds, NNGP_FACTOR_ARGS);
      if (b <= 12) return launch_factor_ds<12, 0>(st, ds, NNGP_FACTOR_ARGS);
      return launch_factor_ds<16, 0>(st, ds, NNGP_FACTOR_ARGS);
    }
    if (b <= 8) return launch_factor_ds<8, 1>(st, ds, NNGP_FACTOR_ARGS);
    if (b <= 12) return launch_factor_ds<12, 1>(st, ds, NNGP_FACTOR_ARGS);
    return launch_factor_ds<16, 1>(st, ds, NNGP_FACTOR_ARGS);
  }
  if (b <= 21) {  // m = 20 (configs[4]): the local block in registers, part of L spilled
    if (family == 0) return launch_factor_ds<21, 0>(st, ds, NNGP_FACTOR_ARGS);
    return launch_factor_ds<21, 1>(st, ds, NNGP_FACTOR_ARGS);
  }
  if (family == 0) return launch_factor_rt<0>(st, ds, NNGP_FACTOR_ARGS);
  return launch_factor_rt<1>(st, ds, NNGP_FACTOR_ARGS);
}
#undef NNGP_FACTOR_ARGS

hipError_t launch_factor_jobs(hipStream_t st, int family, double nu, const FactorJobs& J,
                              const double* locs_rm, int n, int d, int ds, const int* nn, int b) {
  if (J.n_jobs < 1 || J.n_jobs > kMaxChains || b < 1 || b > kBMaxRt) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scale_coords_jobs_kernel, dim3((n + kBlock - 1) / kBlock, J.n_jobs), dim3(kBlock), 0, st, J,
                     locs_rm, n, d, ds);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // NNGP_FACTOR_LANES=16: the 16-lane-group kernel (b <= 16, opt-in)
  if (factor_lanes_on() && b <= 16 && family != 2) return launch_factor_lanes(st, family, ds, J, nn, n, b);
  // one launch for the register-resident kernels; the others (general
  // Matern, b > 21, the lane-pair opt-in) run job after job as launch_factor
  const char* pe = std::getenv("NNGP_FACTOR_PAIR");
  const bool pair = b > 12 && b <= 16 && family != 2 && pe && pe[0] == '1';
  if (family != 2 && !pair) {
    if (b <= 8) return family == 0 ? launch_factor_jobs_bm<8, 0>(st, ds, nu, J, nn, n, b)
                                   : launch_factor_jobs_bm<8, 1>(st, ds, nu, J, nn, n, b);
    if (b <= 12) return family == 0 ? launch_factor_jobs_bm<12, 0>(st, ds, nu, J, nn, n, b)
                                    : launch_factor_jobs_bm<12, 1>(st, ds, nu, J, nn, n, b);
    if (b <= 16) return family == 0 ? launch_factor_jobs_bm<16, 0>(st, ds, nu, J, nn, n, b)
                                    : launch_factor_jobs_bm<16, 1>(st, ds, nu, J, nn, n, b);
    if (b <= 21) return family == 0 ? launch_factor_jobs_bm<21, 0>(st, ds, nu, J, nn, n, b)
                                    : launch_factor_jobs_bm<21, 1>(st, ds, nu, J, nn, n, b);
  }
  for (int j = 0; j < J.n_jobs; ++j)
    if ((e = launch_factor(st, family, J.var[j], J.nugget[j], nu, J.sc[j], ds, nn, n, b, J.linv[j], J.fail[j])) !=
        hipSuccess)
      return e;
  return hipSuccess;
}

// ------------------------------------------------------------------ reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// block of 256 threads: sum 4 values per thread into out[0..3] (thread 0)
__device__ __forceinline__ void block_sum4(double v[4], double* out) {
  __shared__ double sm[4][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double s = wave_sum(v[k]);
    if (lane == 0) sm[w][k] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = ((sm[0][k] + sm[1][k]) + sm[2][k]) + sm[3][k];
  }
}

// sum over each aligned group of G lanes (G = 4, 8, 16, 32), every lane gets
// it.  DPP inside a row of 16 lanes (quad_perm [1,0,3,2] and [2,3,0,1], then
// row_half_mirror and row_mirror: the partner of every step holds a partial
// over the same lane set as in the xor butterfly, and IEEE addition is
// commutative, so the result is bitwise the butterfly's), one shuffle across
// rows for G = 32.  The xor butterfly with __shfl_xor costs a ds_bpermute
// (an LDS round trip) per 32-bit half and step; DPP moves are VALU.
template <int G>
__device__ __forceinline__ double group_sum(double v) {
  v += dpp_f64<0xB1, 0xF, true>(v);
  v += dpp_f64<0x4E, 0xF, true>(v);
  if (G >= 8) v += dpp_f64<0x141, 0xF, true>(v);
  if (G >= 16) v += dpp_f64<0x140, 0xF, true>(v);
  if (G >= 32) v += __shfl_xor(v, 16, 64);
  return v;
}

// G lanes per row (G >= b, power of two): lane g of a row reads entry g, so a
// wave reads G*8 contiguous bytes of Linv per row; a G-lane butterfly sums it.
template <int G>
__global__ __launch_bounds__(256) void row_stats_kernel(const double* __restrict__ linv,
                                                        const int* __restrict__ nn, int n, int b,
                                                        const double* __restrict__ x, double shift,
                                                        double* __restrict__ out,
                                                        double* __restrict__ partials,
                                                        const double* __restrict__ shift_dev,
                                                        const double* const* __restrict__ linv_dev,
                                                        int out_stride) {
  if (shift_dev) shift = *shift_dev;
  if (linv_dev) linv = *linv_dev;
  double acc[4] = {0, 0, 0, 0};
  const int g = threadIdx.x & (G - 1);
  const int rows_per_grid = gridDim.x * (blockDim.x / G);
  // two rows per group and trip (k, k + rows_per_grid): their loads are in
  // flight together; the row sums and their accumulation order are those of
  // one row per trip (bitwise the same results)
  for (int k = blockIdx.x * (blockDim.x / G) + threadIdx.x / G; k < n; k += 2 * rows_per_grid) {
    const int k2 = k + rows_per_grid;
    const bool two = k2 < n;
    int idx = -1, idx2 = -1;
    if (g < b) {
      idx = __builtin_nontemporal_load(nn + (size_t)k * b + g);
      if (two) idx2 = __builtin_nontemporal_load(nn + (size_t)k2 * b + g);
    }
    double l = 0.0, xv = 0.0, l2 = 0.0, xv2 = 0.0;
    if (idx >= 0) {
      l = __builtin_nontemporal_load(linv + (size_t)k * b + g);
      xv = x[idx] - shift;
    }
    if (idx2 >= 0) {
      l2 = __builtin_nontemporal_load(linv + (size_t)k2 * b + g);
      xv2 = x[idx2] - shift;
    }
    double u = l * xv, a = l, u2 = l2 * xv2, a2 = l2;
    u = group_sum<G>(u);
    a = group_sum<G>(a);
    u2 = group_sum<G>(u2);
    a2 = group_sum<G>(a2);
    if (g == 0) {  // (acc[0] stays 0: no caller reads this kernel's log term)
      acc[1] += u * u;
      acc[2] += a * a;
      acc[3] += a * u;
      if (out) out[(size_t)k * out_stride] = u;
      if (two) {
        acc[1] += u2 * u2;
        acc[2] += a2 * a2;
        acc[3] += a2 * u2;
        if (out) out[(size_t)k2 * out_stride] = u2;
      }
    }
  }
  block_sum4(acc, partials + 4 * blockIdx.x);
}

int launch_row_stats(hipStream_t st, const double* linv, const int* nn, int n, int b,
                     const double* x, double shift, double* out, double* partials,
                     const double* shift_dev, const double* const* linv_dev, int out_stride) {
  const int G = b <= 4 ? 4 : b <= 8 ? 8 : b <= 16 ? 16 : 32;
  long long rows_per_block = kBlock / G;
  int g = (int)((n + rows_per_block - 1) / rows_per_block);
  if (g > kRedBlocks) g = kRedBlocks;
  if (g < 1) g = 1;
  switch (G) {
    case 4: hipLaunchKernelGGL(row_stats_kernel<4>, dim3(g), dim3(kBlock), 0, st, linv, nn, n, b, x, shift, out, partials, shift_dev, linv_dev, out_stride); break;
    case 8: hipLaunchKernelGGL(row_stats_kernel<8>, dim3(g), dim3(kBlock), 0, st, linv, nn, n, b, x, shift, out, partials, shift_dev, linv_dev, out_stride); break;
    case 16: hipLaunchKernelGGL(row_stats_kernel<16>, dim3(g), dim3(kBlock), 0, st, linv, nn, n, b, x, shift, out, partials, shift_dev, linv_dev, out_stride); break;
    default: hipLaunchKernelGGL(row_stats_kernel<32>, dim3(g), dim3(kBlock), 0, st, linv, nn, n, b, x, shift, out, partials, shift_dev, linv_dev, out_stride); break;
  }
  return g;
}

// row_stats_kernel for several (factor, field) jobs in one pass: the row's
// NNarray entries load once; per job the same loads, butterfly and
// accumulation order as row_stats_kernel (so the same partials, bitwise).
// Two rows per trip as there, i.e. 2 x M independent gathers in flight.
// Mode 1's log determinant sum_k log L[k][0]: a running product of the row
// diagonals kept as mantissa x 2^exponent (frexp after every factor: no
// overflow or underflow), one log per thread at the end -- a log per row in
// the one lane of its group cost ~45 % of the pass (303 vs 159 us for three
// jobs at n = 1e6, b = 16).  The product's rounding (~n ulp relative) is far
// below the log-likelihood tolerance.
constexpr double kLn2Hi = 0.6931471803691238;       // 28 significant bits: pe * kLn2Hi is exact
constexpr double kLn2Lo = 1.9082149292705877e-10;   // ln 2 - kLn2Hi
template <int G, int MJ>
__global__ __launch_bounds__(256) void row_stats_jobs_kernel(RowJobs J, const int* __restrict__ nn, int n, int b,
                                                             double* __restrict__ partials) {
  double acc[MJ][4];
  double pm[MJ];  // mode 1: product of the diagonals seen = pm x 2^pe
  int pe[MJ];
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    pm[j] = 1.0;
    pe[j] = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[j][q] = 0.0;
  }
  const int g = threadIdx.x & (G - 1);
  const int rows_per_grid = gridDim.x * (blockDim.x / G);
  for (int k = blockIdx.x * (blockDim.x / G) + threadIdx.x / G; k < n; k += 2 * rows_per_grid) {
    const int k2 = k + rows_per_grid;
    const bool two = k2 < n;
    int idx = -1, idx2 = -1;
    if (g < b) {
      idx = __builtin_nontemporal_load(nn + (size_t)k * b + g);
      if (two) idx2 = __builtin_nontemporal_load(nn + (size_t)k2 * b + g);
    }
    double u[MJ], a[MJ], u2[MJ], a2[MJ];
    double dg[MJ], dg2[MJ];  // lane g = 0: the row's diagonal L[k][0] (its own entry, NNarray column 0)
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      double l = 0.0, xv = 0.0, l2 = 0.0, xv2 = 0.0;
      if (j < J.M) {
        if (idx >= 0) {
          l = __builtin_nontemporal_load(J.linv[j] + (size_t)k * b + g);
          xv = J.x[j][idx] - J.shift[j];
        }
        if (idx2 >= 0) {
          l2 = __builtin_nontemporal_load(J.linv[j] + (size_t)k2 * b + g);
          xv2 = J.x[j][idx2] - J.shift[j];
        }
      }
      u[j] = l * xv; a[j] = l; u2[j] = l2 * xv2; a2[j] = l2;
      dg[j] = l; dg2[j] = l2;
    }
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      u[j] = group_sum<G>(u[j]);
      a[j] = group_sum<G>(a[j]);
      u2[j] = group_sum<G>(u2[j]);
      a2[j] = group_sum<G>(a2[j]);
    }
    if (g == 0) {
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        if (j >= J.M) continue;
        if (J.out[j]) J.out[j][(size_t)k * J.out_stride] = u[j];
        if (two && J.out[j]) J.out[j][(size_t)k2 * J.out_stride] = u2[j];
        if (J.mode[j] == 0) continue;
        if (J.mode[j] == 1) {
          int e;
          pm[j] = __builtin_frexp(pm[j] * dg[j], &e);
          pe[j] += e;
          if (two) {
            pm[j] = __builtin_frexp(pm[j] * dg2[j], &e);
            pe[j] += e;
          }
        }
        acc[j][1] += u[j] * u[j];
        acc[j][2] += a[j] * a[j];
        acc[j][3] += a[j] * u[j];
        if (two) {
          acc[j][1] += u2[j] * u2[j];
          acc[j][2] += a2[j] * a2[j];
          acc[j][3] += a2[j] * u2[j];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MJ; ++j)
    if (j < J.M && J.mode[j] == 1 && g == 0) acc[j][0] = log(pm[j]) + ((double)pe[j] * kLn2Hi + (double)pe[j] * kLn2Lo);
#pragma unroll
  for (int j = 0; j < MJ; ++j)
    if (j < J.M && J.mode[j] != 0) {
      block_sum4(acc[j], partials + (size_t)j * kRedBlocks * 4 + 4 * blockIdx.x);
      __syncthreads();  // block_sum4's LDS is reused by the next job
    }
}

int launch_row_stats_jobs(hipStream_t st, const RowJobs& J, const int* nn, int n, int b, double* partials) {
  const int G = b <= 4 ? 4 : b <= 8 ? 8 : b <= 16 ? 16 : 32;
  long long rows_per_block = kBlock / G;
  int g = (int)((n + rows_per_block - 1) / rows_per_block);
  if (g > kRedBlocks) g = kRedBlocks;
  if (g < 1) g = 1;
  if (J.M < 1 || J.M > kRowJobsMax) return -1;
#define NNGP_RSJ(GG)                                                                                         \
  switch (J.M) {                                                                                           \
    case 1: hipLaunchKernelGGL((row_stats_jobs_kernel<GG, 1>), dim3(g), dim3(kBlock), 0, st, J, nn, n, b, partials); break; \
    case 2: hipLaunchKernelGGL((row_stats_jobs_kernel<GG, 2>), dim3(g), dim3(kBlock), 0, st, J, nn, n, b, partials); break; \
    case 3: hipLaunchKernelGGL((row_stats_jobs_kernel<GG, 3>), dim3(g), dim3(kBlock), 0, st, J, nn, n, b, partials); break; \
    case 4: hipLaunchKernelGGL((row_stats_jobs_kernel<GG, 4>), dim3(g), dim3(kBlock), 0, st, J, nn, n, b, partials); break; \
    case 5: hipLaunchKernelGGL((row_stats_jobs_kernel<GG, 5>), dim3(g), dim3(kBlock), 0, st, J, nn, n, b, partials); break; \
    case 6: hipLaunchKernelGGL((row_stats_jobs_kernel<GG, 6>), dim3(g), dim3(kBlock), 0, st, J, nn, n, b, partials); break; \
    default: hipLaunchKernelGGL((row_stats_jobs_kernel<GG, 8>), dim3(g), dim3(kBlock), 0, st, J, nn, n, b, partials); break; \
  }
  switch (G) {
    case 4: NNGP_RSJ(4) break;
    case 8: NNGP_RSJ(8) break;
    case 16: NNGP_RSJ(16) break;
    default: NNGP_RSJ(32) break;
  }
#undef NNGP_RSJ
  return g;
}

// one block per job: the job's partials in reduce4_kernel's order
__global__ __launch_bounds__(256) void reduce4_jobs_kernel(RowJobs J, const double* __restrict__ partials,
                                                           int nblocks, double* __restrict__ res) {
  const int j = blockIdx.x;
  const double* pj = partials + (size_t)j * kRedBlocks * 4;
  double acc[4] = {0, 0, 0, 0};
  for (int p = threadIdx.x; p < nblocks; p += blockDim.x)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += pj[4 * p + k];
  block_sum4(acc, res + 4 * J.res_slot[j]);
}

hipError_t launch_reduce4_jobs(hipStream_t st, const RowJobs& J, const double* partials, int nblocks, double* res) {
  hipLaunchKernelGGL(reduce4_jobs_kernel, dim3(J.M), dim3(kBlock), 0, st, J, partials, nblocks, res);
  return hipGetLastError();
}

// r = B (field - beta0) for every chain in mask in one pass: the row's
// NNarray entries are read once for all chains; per chain the same products
// and butterfly as row_stats_kernel (bitwise the same r).  Factor pointers
// and beta0 are read from device memory (graph-replay safe).
template <int G>
__global__ __launch_bounds__(256) void spmv_chains_kernel(const double* const* __restrict__ linv_dev,
                                                          const int* __restrict__ nn, int n, int b, FieldPtrs f,
                                                          const SweepScalars* __restrict__ sc,
                                                          double* __restrict__ out, int C, int mask) {
  const int g = threadIdx.x & (G - 1);
  const int rows_per_grid = gridDim.x * (blockDim.x / G);
  for (int k = blockIdx.x * (blockDim.x / G) + threadIdx.x / G; k < n; k += rows_per_grid) {
    const int idx = g < b ? nn[(size_t)k * b + g] : -1;
#pragma unroll
    for (int ch = 0; ch < kMaxChains; ++ch) {
      if (ch >= C || !((mask >> ch) & 1)) continue;
      double l = 0.0, xv = 0.0;
      if (idx >= 0) {
        l = linv_dev[ch][(size_t)k * b + g];
        xv = f.p[ch][idx] - sc[ch].beta0;
      }
      // (shuffle butterfly: the DPP group_sum measured 134 vs 125 us here --
      // one reduction per row and chain, latency-bound on the gathers)
      double u = l * xv;
#pragma unroll
      for (int off = 1; off < G; off <<= 1) u += __shfl_xor(u, off, 64);
      if (g == 0) out[(size_t)k * C + ch] = u;
    }
  }
}

hipError_t launch_spmv_chains(hipStream_t st, const double* const* linv_dev, const int* nn, int n, int b,
                              const FieldPtrs& f, const SweepScalars* sc, double* out, int C, int mask) {
  const int G = b <= 4 ? 4 : b <= 8 ? 8 : b <= 16 ? 16 : 32;
  const long long rows_per_block = kBlock / G;
  int g = (int)((n + rows_per_block - 1) / rows_per_block);
  if (g > kRedBlocks) g = kRedBlocks;
  if (g < 1) g = 1;
  switch (G) {
    case 4: hipLaunchKernelGGL(spmv_chains_kernel<4>, dim3(g), dim3(kBlock), 0, st, linv_dev, nn, n, b, f, sc, out, C, mask); break;
    case 8: hipLaunchKernelGGL(spmv_chains_kernel<8>, dim3(g), dim3(kBlock), 0, st, linv_dev, nn, n, b, f, sc, out, C, mask); break;
    case 16: hipLaunchKernelGGL(spmv_chains_kernel<16>, dim3(g), dim3(kBlock), 0, st, linv_dev, nn, n, b, f, sc, out, C, mask); break;
    default: hipLaunchKernelGGL(spmv_chains_kernel<32>, dim3(g), dim3(kBlock), 0, st, linv_dev, nn, n, b, f, sc, out, C, mask); break;
  }
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void reduce4_kernel(const double* __restrict__ partials,
                                                      int nblocks, double* __restrict__ res) {
  double acc[4] = {0, 0, 0, 0};
  for (int p = threadIdx.x; p < nblocks; p += blockDim.x)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += partials[4 * p + k];
  block_sum4(acc, res);
}

hipError_t launch_reduce4(hipStream_t st, const double* partials, int nblocks, double* res) {
  hipLaunchKernelGGL(reduce4_kernel, dim3(1), dim3(kBlock), 0, st, partials, nblocks, res);
  return hipGetLastError();
}

// ------------------------------------------------------------------ A5
// Merge-path sweep layout (graph_prep.h): chunk ch of one chain is LW*16
// cells, sorted by row of B; cell k is entry ch*LW*16 + k and sits at stream
// position ent_pos (slot q of the chunk covers stream [f0_q, f0_q + len_q)).

// refresh chain `chain`'s B values in the sweep layout and precision_diag
// (entries of a column summed in stream = row order); one wavefront per chunk
template <int LW>
__global__ __launch_bounds__(256) void sell_refresh_kernel(SweepDev L, int nchunks,
                                                           const int* __restrict__ ent_src,
                                                           const double* __restrict__ linv, int chain) {
  constexpr int CAP = LW * kSweepRows;
  __shared__ double sq_s[4][CAP];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int chk = blockIdx.x * 4 + wv;
  if (chk >= nchunks) return;
  double* sq = sq_s[wv];
  const long long base = (long long)chk * CAP;
  double* val = const_cast<double*>(L.ent_val) + (size_t)chain * L.n_entries;
  for (int k = lane; k < CAP; k += 64) {
    const long long e = base + k;
    const int src = ent_src[e];
    const double v = src >= 0 ? linv[src] : 0.0;
    val[e] = v;
    sq[L.ent_pos[e]] = v * v;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int x0 = L.chunk_first[chk], nsl = L.chunk_first[chk + 1] - x0;
  for (int t = lane; t < nsl; t += 64) {
    const int2 si = L.sinfo[x0 + t];
    const int f0 = si.y & 0xFFFF, len = si.y >> 16;
    double D = 0.0;
    for (int f = f0; f < f0 + len; ++f) D += sq[f];
    L.dr[(size_t)(x0 + t) * L.C + chain].x = D;
  }
}

hipError_t launch_sell_refresh(hipStream_t st, const SweepDev& L, int nchunks, const int* ent_src,
                               const double* linv, int chain) {
  const int g = (nchunks + 3) / 4;
  if (g == 0) return hipSuccess;
  switch (L.LW) {
    case 64: hipLaunchKernelGGL(sell_refresh_kernel<64>, dim3(g), dim3(kBlock), 0, st, L, nchunks, ent_src, linv, chain); break;
    case 32: hipLaunchKernelGGL(sell_refresh_kernel<32>, dim3(g), dim3(kBlock), 0, st, L, nchunks, ent_src, linv, chain); break;
    case 16: hipLaunchKernelGGL(sell_refresh_kernel<16>, dim3(g), dim3(kBlock), 0, st, L, nchunks, ent_src, linv, chain); break;
    case 21: hipLaunchKernelGGL(sell_refresh_kernel<21>, dim3(g), dim3(kBlock), 0, st, L, nchunks, ent_src, linv, chain); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------ A7
__global__ void residual_sums_kernel(int n, SweepDev L, int chain,
                                     const int* __restrict__ obs_ptr, const int* __restrict__ obs_idx,
                                     const double* __restrict__ y, const double* __restrict__ mu,
                                     double beta0) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  int loc = L.compact_loc[s];
  double R = 0.0;
  for (int p = obs_ptr[loc]; p < obs_ptr[loc + 1]; ++p) {
    int o = obs_idx[p];
    R += y[o] - (mu ? mu[o] : beta0);
  }
  L.dr[(size_t)s * L.C + chain].y = R;
}

// residual sums of several chains in one pass: the location's observation
// list and y read once, per chain exactly residual_sums_kernel's sum
__global__ void residual_sums_jobs_kernel(int n, SweepDev L, ResJobs J, const int* __restrict__ obs_ptr,
                                          const int* __restrict__ obs_idx, const double* __restrict__ y) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  int loc = L.compact_loc[s];
  double R[kMaxChains] = {0.0, 0.0, 0.0, 0.0};
  for (int p = obs_ptr[loc]; p < obs_ptr[loc + 1]; ++p) {
    int o = obs_idx[p];
    const double yo = y[o];
#pragma unroll
    for (int j = 0; j < kMaxChains; ++j)
      if (j < J.M) R[j] += yo - (J.mu[j] ? J.mu[j][o] : J.beta0[j]);
  }
#pragma unroll
  for (int j = 0; j < kMaxChains; ++j)
    if (j < J.M) L.dr[(size_t)s * L.C + J.chain[j]].y = R[j];
}

// every job with mu = beta_0 (no X, update_Gaussian.R:85-90): R = sum y -
// n_obs beta_0 per slot from the per-slot sums of y (ysum, compact order,
// fixed per context) -- a streaming pass instead of the gathers over the
// observations (the data term moves with every beta_0 draw)
__global__ void residual_sums_const_kernel(int n, SweepDev L, ResJobs J, const double* __restrict__ ysum,
                                           const int2* __restrict__ sinfo) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const double ys = ysum[s], no = (double)sinfo[s].x;
#pragma unroll
  for (int j = 0; j < kMaxChains; ++j)
    if (j < J.M) L.dr[(size_t)s * L.C + J.chain[j]].y = __builtin_fma(-no, J.beta0[j], ys);
}

hipError_t launch_residual_sums_jobs(hipStream_t st, int n, const SweepDev& L, const ResJobs& J,
                                     const int* obs_ptr, const int* obs_idx, const double* y, const double* ysum,
                                     const int2* sinfo) {
  if (J.M < 1 || J.M > kMaxChains) return hipErrorInvalidValue;
  bool all_const = ysum && sinfo;
  for (int j = 0; j < J.M; ++j) all_const &= J.mu[j] == nullptr;
  if (all_const) {
    hipLaunchKernelGGL(residual_sums_const_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, n, L, J, ysum,
                       sinfo);
    return hipGetLastError();
  }
  int g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(residual_sums_jobs_kernel, dim3(g), dim3(kBlock), 0, st, n, L, J, obs_ptr, obs_idx, y);
  return hipGetLastError();
}

hipError_t launch_residual_sums(hipStream_t st, int n, const SweepDev& L, int chain, const int* obs_ptr,
                                const int* obs_idx, const double* y, const double* mu, double beta0) {
  int g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(residual_sums_kernel, dim3(g), dim3(kBlock), 0, st, n, L, chain, obs_ptr, obs_idx,
                     y, mu, beta0);
  return hipGetLastError();
}

// every chain in `mask` at once: slot_dpos read once, w written as whole
// slot records (slot*C + chain)
__global__ void field_to_slots_multi_kernel(int n, const int* __restrict__ slot_dpos, FieldPtrs f,
                                            const SweepScalars* __restrict__ sc, double* __restrict__ w, int C,
                                            int mask) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const int d = slot_dpos[s];
#pragma unroll
  for (int k = 0; k < kMaxChains; ++k)
    if (k < C && ((mask >> k) & 1)) w[(size_t)s * C + k] = f.p[k][d] - sc[k].beta0;
}
__global__ void slots_to_field_multi_kernel(int n, const int* __restrict__ slot_dpos, FieldPtrs f,
                                            const SweepScalars* __restrict__ sc, const double* __restrict__ w,
                                            int C, int mask) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const int d = slot_dpos[s];
#pragma unroll
  for (int k = 0; k < kMaxChains; ++k)
    if (k < C && ((mask >> k) & 1)) f.p[k][d] = w[(size_t)s * C + k] + sc[k].beta0;
}

hipError_t launch_field_to_slots_multi(hipStream_t st, int n, const int* slot_dpos, const FieldPtrs& f,
                                       const SweepScalars* sc, double* w_slot, int C, int mask) {
  int g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(field_to_slots_multi_kernel, dim3(g), dim3(kBlock), 0, st, n, slot_dpos, f, sc, w_slot, C, mask);
  return hipGetLastError();
}
hipError_t launch_slots_to_field_multi(hipStream_t st, int n, const int* slot_dpos, const FieldPtrs& f,
                                       const SweepScalars* sc, const double* w_slot, int C, int mask) {
  int g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(slots_to_field_multi_kernel, dim3(g), dim3(kBlock), 0, st, n, slot_dpos, f, sc, w_slot, C, mask);
  return hipGetLastError();
}

// ------------------------------------------------------------------ A1
// Normals of one sweep in compact order, chain-interleaved:
// z[(rank[loc]) * C + chain].  Work item = (pair p of a pair list, chain);
// chains outside chain_mask are skipped.
__device__ __forceinline__ void gen_normals(int item, const int* __restrict__ pairs, int npairs,
                                            const SweepScalars* __restrict__ scal, int C, int chain_mask,
                                            uint64_t sweep_off, const int* __restrict__ loc_rank, int n,
                                            double* __restrict__ z) {
  if (item >= npairs * C) return;
  const int chain = item % C;
  if (!((chain_mask >> chain) & 1)) return;
  const int p = pairs ? pairs[item / C] : item / C;
  const uint64_t sw = scal[chain].counter_base + sweep_off;
  __builtin_nontemporal_store(normal_loc(scal[chain].seed, sw, (uint32_t)(2 * p)),
                              z + (size_t)loc_rank[2 * p] * C + chain);
  if (2 * p + 1 < n)
    __builtin_nontemporal_store(normal_loc(scal[chain].seed, sw, (uint32_t)(2 * p + 1)),
                                z + (size_t)loc_rank[2 * p + 1] * C + chain);
}

__global__ __launch_bounds__(256) void normals_compact_kernel(SweepDev L, int chain_mask, int sweep_off,
                                                              int n, double* z) {
  gen_normals(blockIdx.x * blockDim.x + threadIdx.x, nullptr, (n + 1) / 2, L.scal, L.C, chain_mask,
              (uint64_t)sweep_off, L.loc_rank, n, z);
}

hipError_t launch_normals_compact(hipStream_t st, const SweepDev& L, int chain_mask, int sweep_off, int n,
                                  double* z) {
  const long long items = (long long)((n + 1) / 2) * L.C;
  const int g = (int)((items + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(normals_compact_kernel, dim3(g), dim3(kBlock), 0, st, L, chain_mask, sweep_off, n, z);
  return hipGetLastError();
}

// One colour of the chromatic sweep, local form, for up to 4 chains at once:
//   acc  = sum_{k in col(i)} B[k,i] r_k - D_i w_i      (= (B^T B w_{!c})_i)
//   P    = D_i/s2 + n_i/t2
//   w_i' = (R_i/t2 - acc/s2)/P + z_i/sqrt(P)
//   r_k += B[k,i] (w_i' - w_i)
// Workgroups [0, gs) sweep: one wavefront per chunk; its 64/LW chain groups
// run the same chunk for different chains (same entry cells,
// chain-interleaved r / w / {D,R} / z).
//  1. round trip 1: the lane's 16 cells (row-sorted: one instruction's
//     lanes cover consecutive rows), the records of the two slots it owns
//     (q = lane, lane + LW) and the chunk's first compact index -- all
//     addressed by the chunk index alone;
//  2. round trip 2: r gathered at the cells' rows (a few lines per
//     instruction); the owned slots' normals;
//  3. products B[k,i] r_k regrouped by stream position in LDS; lane l then
//     runs along stream cells l*16 .. l*16+15, restarting where a new slot
//     begins (start_mask), and stores every running sum (LDS rows padded
//     against bank conflicts);
//  4. owner of slot q: acc = its run ending in its last cell, plus the lane
//     totals of the lanes it spans before that (in lane order: deterministic);
//     the draw; dw[q] -> LDS;
//  5. every cell scatters r_k += B[k,i] dw[q] (again a few lines per
//     instruction).
// Workgroups [gs, gs + gz) generate the NEXT sweep's normals of this
// colour's pairs (z_next) on the SIMD time the latency-bound sweep waves
// leave idle; the next sweep reads them >= K launches later.
// Slots of one colour share no row of B, so the scatter is conflict-free.
// Sweep blocks are remapped so that consecutive (spatially adjacent) chunks
// run on the same XCD and share its L2 for the r gathers.
// PROBE 9 (diagnostic build, NNGP_PROBE=9): per-phase s_memtime stamps.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kCellStride = kSweepRows + 1;  // LDS row pitch (doubles): lanes hit distinct banks

template <int LW, int PROBE = 0>
__global__ __launch_bounds__(256) void sweep_color_kernel(SweepDev L, ColorLaunch a) {
  constexpr int CG = 64 / LW;  // chain groups per wavefront
  constexpr int SPC = 2 * LW;  // slots per chunk (bound)
  __shared__ double cells_s[4][CG][LW * kCellStride];
  __shared__ double dw_s[4][CG][SPC];
  const int gs = (a.nch + 3) / 4;
  if ((int)blockIdx.x >= gs) {
    gen_normals(((int)blockIdx.x - gs) * 256 + threadIdx.x, a.pairs, a.npairs, L.scal, L.C, a.chain_mask,
                (uint64_t)a.sweep_local + 1, L.loc_rank, a.n, a.z_next);
    return;
  }
  unsigned long long stamp[8];
#define STAMP(k)                                                      \
  do {                                                                \
    if (PROBE == 9) {                                                 \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");     \
      stamp[k] = __builtin_amdgcn_s_memtime();                        \
    }                                                                 \
  } while (0)
  if (PROBE == 9) stamp[7] = __builtin_amdgcn_s_memrealtime();
  STAMP(0);
  const int bid = blockIdx.x;
  const int xcd = bid & 7, qq = gs >> 3, rm = gs & 7;
  const int lb = (xcd < rm ? xcd * (qq + 1) : rm * (qq + 1) + (xcd - rm) * qq) + (bid >> 3);
  const int wv = threadIdx.x >> 6;
  const int lch = lb * 4 + wv;
  if (lch >= a.nch) return;
  const int lane = threadIdx.x & 63;
  const int cg = lane / LW, l = lane % LW;
  const int C = L.C;
  if (cg >= C || !((a.chain_mask >> cg) & 1)) return;
  const int chain = cg;
  double* cells = cells_s[wv][cg];
  double* dws = dw_s[wv][cg];
  const int ch = a.chunk0 + lch;
  const long long base = (long long)ch * LW * kSweepRows;
  const double* val = L.ent_val + (size_t)chain * L.n_entries;
  double* r = L.r;  // gathered then scattered: no __restrict__
  // round trip 1
  double v[kSweepRows], rv[kSweepRows];
  int pk[kSweepRows], ps[kSweepRows];
#pragma unroll
  for (int j = 0; j < kSweepRows; ++j) {
    // read once per sweep: non-temporal, so the XCD's L2 keeps r
    const long long e = base + (long long)j * LW + l;
    v[j] = __builtin_nontemporal_load(val + e);
    pk[j] = __builtin_nontemporal_load(L.ent_pk + e);
    ps[j] = __builtin_nontemporal_load(L.ent_pos + e);
  }
  const int x0 = L.chunk_first[ch];
  const int nsl = L.chunk_first[ch + 1] - x0;
  const unsigned smask = L.start_mask[(size_t)ch * LW + l];
  const SweepScalars* scal = L.scal + chain;
  const double inv_s2 = scal->inv_s2, inv_t2 = scal->inv_t2;
  if (PROBE == 9) { double x = x0 + nsl; for (int j = 0; j < kSweepRows; ++j) x += v[j] + pk[j] + ps[j]; if (x == 12345.678) stamp[0] = 0; }
  STAMP(1);
  // round trip 2: gathers + the owned slots' records and normals
#pragma unroll
  for (int j = 0; j < kSweepRows; ++j) {
    const int p = pk[j] & kPkPadRow;
    rv[j] = (p != kPkPadRow) ? r[(size_t)p * C + chain] : 0.0;
  }
  int2 si[2];
  double2 dr[2];
  double w[2], zz[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = l + u * LW;
    const size_t x = (size_t)x0 + min(t, nsl - 1);
    // per-slot data is touched once per sweep: non-temporal like the cells
    {
      const long long raw = __builtin_nontemporal_load(reinterpret_cast<const long long*>(L.sinfo + x));
      si[u].x = (int)(raw & 0xFFFFFFFFll);
      si[u].y = (int)(raw >> 32);
    }
    dr[u].x = __builtin_nontemporal_load(&L.dr[x * C + chain].x);
    dr[u].y = __builtin_nontemporal_load(&L.dr[x * C + chain].y);
    w[u] = __builtin_nontemporal_load(L.w_slot + x * C + chain);
    zz[u] = __builtin_nontemporal_load(a.z_cur + x * C + chain);
  }
  // w' = (R/t2 - (acc - D w)/s2) / P + z / sqrt(P): everything but acc
  double cR[2], invP[2], zs[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const double P = dr[u].x * inv_s2 + (double)si[u].x * inv_t2;
    invP[u] = 1.0 / P;
    zs[u] = zz[u] / sqrt(P);
    cR[u] = inv_t2 * dr[u].y + inv_s2 * (dr[u].x * w[u]);
  }
  if (PROBE == 9) { double x = zs[0] + zs[1] + cR[0] + invP[0]; for (int j = 0; j < kSweepRows; ++j) x += rv[j]; if (x == 12345.678) stamp[0] = 0; }
  STAMP(2);
  // products regrouped by stream position, then running sums along the
  // lane's stream cells, restarted at every slot start (start_mask bit j:
  // stream cell l*16 + j begins a slot)
  int q[kSweepRows];
#pragma unroll
  for (int j = 0; j < kSweepRows; ++j) {
    q[j] = (int)((unsigned)pk[j] >> kPkRowBits);
    cells[(ps[j] / kSweepRows) * kCellStride + ps[j] % kSweepRows] = v[j] * rv[j];
  }
  wave_lds_sync();
  {
    double x[kSweepRows];
#pragma unroll
    for (int j = 0; j < kSweepRows; ++j) x[j] = cells[l * kCellStride + j];
    double run = 0.0;
#pragma unroll
    for (int j = 0; j < kSweepRows; ++j) {
      run = ((smask >> j) & 1u) ? x[j] : run + x[j];
      cells[l * kCellStride + j] = run;
    }
  }
  wave_lds_sync();
  STAMP(3);
  // owners: the Gibbs draw of slots q = l and q = l + LW
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = l + u * LW;
    if (t < nsl) {
      const int f0 = si[u].y & 0xFFFF, fe = f0 + (si[u].y >> 16) - 1;
      const int l0 = f0 / kSweepRows, l1 = fe / kSweepRows;
      // its run ending in its last cell, after the totals of the lanes it
      // spans before (lane order)
      double acc;
      if (l0 == l1) {
        acc = cells[l1 * kCellStride + fe % kSweepRows];
      } else {
        acc = cells[l0 * kCellStride + kSweepRows - 1];
        for (int ll = l0 + 1; ll < l1; ++ll) acc += cells[ll * kCellStride + kSweepRows - 1];
        acc += cells[l1 * kCellStride + fe % kSweepRows];
      }
      const double wn = (cR[u] - inv_s2 * acc) * invP[u] + zs[u];
      const double dw = wn - w[u];
      dws[t] = dw;
      __builtin_nontemporal_store(wn, L.w_slot + ((size_t)x0 + t) * C + chain);
      // sharded sweep: publish {dw, w_new} into this rank's exchange segment
      if (a.xsend) a.xsend[((size_t)x0 + t - a.xs0) * C + chain] = make_double2(dw, wn);
    }
  }
  wave_lds_sync();
  STAMP(4);
#pragma unroll
  for (int j = 0; j < kSweepRows; ++j) {
    const int p = pk[j] & kPkPadRow;
    // explicit fma: the ghost cells of the sharded sweep round identically
    if (p != kPkPadRow) r[(size_t)p * C + chain] = __builtin_fma(v[j], dws[q[j]], rv[j]);
  }
  STAMP(5);
  if (PROBE == 9 && l == 0 && chain == 0) {
    unsigned long long* o = L.dbg + (size_t)ch * 8;
    for (int k = 0; k < 6; ++k) o[k] = stamp[k];
    o[6] = 0;
    o[7] = stamp[7];
  }
#undef STAMP
}

hipError_t launch_sweep_color(hipStream_t st, const SweepDev& L, const ColorLaunch& a) {
  const int gs = (a.nch + 3) / 4;
  const int gz = a.z_next ? (int)(((long long)a.npairs * L.C + 255) / 256) : 0;
  if (gs + gz == 0) return hipSuccess;
  static const int probe = [] { const char* e = std::getenv("NNGP_PROBE"); return e ? std::atoi(e) : 0; }();
  if (probe == 9 && L.LW == 64 && L.dbg) {
    hipLaunchKernelGGL((sweep_color_kernel<64, 9>), dim3(gs + gz), dim3(kBlock), 0, st, L, a);
    return hipGetLastError();
  }
  switch (L.LW) {
    case 64: hipLaunchKernelGGL((sweep_color_kernel<64>), dim3(gs + gz), dim3(kBlock), 0, st, L, a); break;
    case 32: hipLaunchKernelGGL((sweep_color_kernel<32>), dim3(gs + gz), dim3(kBlock), 0, st, L, a); break;
    case 16: hipLaunchKernelGGL((sweep_color_kernel<16>), dim3(gs + gz), dim3(kBlock), 0, st, L, a); break;
    case 21: hipLaunchKernelGGL((sweep_color_kernel<21>), dim3(gs + gz), dim3(kBlock), 0, st, L, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------ A1 (sharded)
// After colour c's exchange: workgroups [0, gb) apply the ghost cells (one
// thread per (cell, chain): r[row] += B[k,j] dw_j; rows are distinct inside a
// colour, so no atomics), workgroups [gb, ...) copy w_new of the other ranks'
// slots into the w replica.  Both read the exchange region only.
__global__ __launch_bounds__(256) void shard_ghost_kernel(SweepDev L, ShardGhostLaunch a, int gb) {
  const int C = L.C;
  if ((int)blockIdx.x < gb) {
    const long long it = (long long)blockIdx.x * 256 + threadIdx.x;
    if (it >= (long long)a.ng * C) return;
    const int e = a.g0 + (int)(it / C), chain = (int)(it % C);
    if (!((a.chain_mask >> chain) & 1)) return;
    const double v = __builtin_nontemporal_load(a.gval + (size_t)chain * a.ng_total + e);
    const double dw = a.xbuf[(size_t)__builtin_nontemporal_load(a.grecv + e) * C + chain].x;
    double* rp = L.r + (size_t)__builtin_nontemporal_load(a.grow + e) * C + chain;
    *rp = __builtin_fma(v, dw, *rp);
    return;
  }
  const long long it = (long long)(blockIdx.x - gb) * 256 + threadIdx.x;
  if (it >= (long long)a.G * a.cnt * C) return;
  const int s = (int)(it / C), chain = (int)(it % C);
  const int h = s / a.cnt, off = s % a.cnt;
  if (h == a.rank || !((a.chain_mask >> chain) & 1)) return;
  const int x = a.seg0[h] + off;
  if (x >= a.seg0[h + 1]) return;
  L.w_slot[(size_t)x * C + chain] = a.xbuf[(size_t)s * C + chain].y;
}

hipError_t launch_shard_ghosts(hipStream_t st, const SweepDev& L, const ShardGhostLaunch& a) {
  const int gb = (int)(((long long)a.ng * L.C + 255) / 256);
  const int wb = a.G > 1 ? (int)(((long long)a.G * a.cnt * L.C + 255) / 256) : 0;
  if (gb + wb == 0) return hipSuccess;
  hipLaunchKernelGGL(shard_ghost_kernel, dim3(gb + wb), dim3(kBlock), 0, st, L, a, gb);
  return hipGetLastError();
}


// ------------------------------------------------------------------ A8
__global__ __launch_bounds__(256) void obs_reduce_kernel(int mode, int n_obs, const double* __restrict__ y,
                                                         const double* __restrict__ mu, double beta0,
                                                         const int* __restrict__ lm,
                                                         const double* __restrict__ f,
                                                         const double* __restrict__ fnew,
                                                         double inv_2var, double* __restrict__ partials) {
  double acc[4] = {0, 0, 0, 0};
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < n_obs; o += gridDim.x * blockDim.x) {
    double m = mu ? mu[o] : beta0;
    int loc = lm[o];
    if (mode == 0) {
      double e = y[o] - f[loc] - m + beta0;
      acc[0] += e * e;
    } else {
      double ea = y[o] - (fnew[loc] + m - beta0);
      double eb = y[o] - (f[loc] + m - beta0);
      acc[0] += (eb * eb - ea * ea) * inv_2var;
    }
  }
  block_sum4(acc, partials + 4 * blockIdx.x);
}

// obs reductions of several chains in one pass (y and the location map read
// once): per chain exactly obs_reduce_kernel's terms, accumulation order and
// block partials (the same grid), partials of chain job j at j x kRedBlocks x 4
template <int MJ>
__global__ __launch_bounds__(256) void obs_reduce_jobs_kernel(int mode, int n_obs, const double* __restrict__ y,
                                                              const int* __restrict__ lm, ObsJobs J,
                                                              double* __restrict__ partials) {
  double acc[MJ][4];
#pragma unroll
  for (int j = 0; j < MJ; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[j][q] = 0.0;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < n_obs; o += gridDim.x * blockDim.x) {
    const double yo = y[o];
    const int loc = lm[o];
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      if (j >= J.M) continue;
      const double m = J.mu[j] ? J.mu[j][o] : J.beta0[j];
      if (mode == 0) {
        double e = yo - J.f[j][loc] - m + J.beta0[j];
        acc[j][0] += e * e;
      } else {
        double ea = yo - (J.fnew[j][loc] + m - J.beta0[j]);
        double eb = yo - (J.f[j][loc] + m - J.beta0[j]);
        acc[j][0] += (eb * eb - ea * ea) * J.inv_2var[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MJ; ++j)
    if (j < J.M) {
      block_sum4(acc[j], partials + (size_t)j * kRedBlocks * 4 + 4 * blockIdx.x);
      __syncthreads();  // block_sum4's LDS is reused by the next chain
    }
}

int launch_obs_reduce_jobs(hipStream_t st, int mode, int n_obs, const double* y, const int* lm, const ObsJobs& J,
                           double* partials) {
  int g = (n_obs + kBlock - 1) / kBlock;
  if (g > kRedBlocks) g = kRedBlocks;
  if (g < 1) g = 1;
  switch (J.M) {
    case 1: hipLaunchKernelGGL(obs_reduce_jobs_kernel<1>, dim3(g), dim3(kBlock), 0, st, mode, n_obs, y, lm, J, partials); break;
    case 2: hipLaunchKernelGGL(obs_reduce_jobs_kernel<2>, dim3(g), dim3(kBlock), 0, st, mode, n_obs, y, lm, J, partials); break;
    case 3: hipLaunchKernelGGL(obs_reduce_jobs_kernel<3>, dim3(g), dim3(kBlock), 0, st, mode, n_obs, y, lm, J, partials); break;
    case 4: hipLaunchKernelGGL(obs_reduce_jobs_kernel<4>, dim3(g), dim3(kBlock), 0, st, mode, n_obs, y, lm, J, partials); break;
    default: return -1;
  }
  return g;
}

int launch_obs_reduce(hipStream_t st, int mode, int n_obs, const double* y, const double* mu,
                      double beta0, const int* lm, const double* field, const double* field_new,
                      double inv_2var, double* partials) {
  int g = (n_obs + kBlock - 1) / kBlock;
  if (g > kRedBlocks) g = kRedBlocks;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(obs_reduce_kernel, dim3(g), dim3(kBlock), 0, st, mode, n_obs, y, mu, beta0, lm,
                     field, field_new, inv_2var, partials);
  return g;
}

// ------------------------------------------------------------------ tri solve
// Sparse triangular solve B x = u for up to 4 chains at once (same DAG, per
// chain factor): work item = (row of the level, chain slot kk); u and x are
// chain-strided (element d*stride + kidx[kk]).  One chain: stride 1.
// b <= BMAX (ctx_create caps b at 32).
// 16 lanes per (row, chain) -- one DPP row: lane l takes neighbours j = l and
// l + 16 (b <= 32), so a row's NNarray / Linv entries load as one or two
// coalesced lines instead of b scattered ones; the products reduce by DPP
// row shifts and lane 15 of the row writes x_i = (u_i - sum_j B[i,j] x_j) / B[i,i].
// Every lane of a 16-lane row runs the same path (`active` is row-uniform).
template <int BMAX>
__device__ __forceinline__ void tri_row16(const TriArgs& a, int i, int kk, int l, bool active,
                                          const int* __restrict__ nn, int b, const double* __restrict__ u,
                                          double* __restrict__ x) {
  double p = 0.0;
  const int k = active ? a.kidx[kk] : 0, S = a.stride;
  const double* lr = active ? a.linv[kk] + (size_t)i * b : nullptr;
  if (active) {
    const int* nr = nn + (size_t)i * b;
#pragma unroll
    for (int j = l; j < BMAX; j += 16) {
      if (j >= 1 && j < b) {
        const int idx = __builtin_nontemporal_load(nr + j);
        if (idx >= 0) p = __builtin_fma(__builtin_nontemporal_load(lr + j), x[(size_t)idx * S + k], p);
      }
    }
  }
  p += dpp_f64<0x111, 0xF, true>(p);  // row_shr:1
  p += dpp_f64<0x112, 0xF, true>(p);  // row_shr:2
  p += dpp_f64<0x114, 0xF, true>(p);  // row_shr:4
  p += dpp_f64<0x118, 0xF, true>(p);  // row_shr:8 -> lane 15 holds the row sum
  if (active && l == 15) x[(size_t)i * S + k] = (u[(size_t)i * S + k] - p) / lr[0];
}

template <int BMAX>
__global__ __launch_bounds__(256) void tri_level_kernel(TriArgs a, const int* __restrict__ rows, int nrows,
                                                        const int* __restrict__ nn, int b,
                                                        const double* __restrict__ u, double* __restrict__ x) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long item = t >> 4;
  const bool active = item < (long long)nrows * a.nc;
  const int i = active ? rows[item / a.nc] : 0;
  tri_row16<BMAX>(a, i, active ? (int)(item % a.nc) : 0, (int)(t & 15), active, nn, b, u, x);
}

hipError_t launch_tri_level(hipStream_t st, const TriArgs& a, const int* rows, int nrows, const int* nn, int b,
                            const double* u, double* x) {
  const long long threads = (long long)nrows * a.nc * 16;
  const int g = (int)((threads + kBlock - 1) / kBlock);
  if (b <= 16)
    hipLaunchKernelGGL(tri_level_kernel<16>, dim3(g), dim3(kBlock), 0, st, a, rows, nrows, nn, b, u, x);
  else
    hipLaunchKernelGGL(tri_level_kernel<32>, dim3(g), dim3(kBlock), 0, st, a, rows, nrows, nn, b, u, x);
  return hipGetLastError();
}

// A run of consecutive SMALL levels of the Vecchia DAG in one workgroup:
// the rows of level lv are rows[lptr[lv] .. lptr[lv+1]); the workgroup
// barrier between levels replaces a kernel launch (same arithmetic as
// tri_level_kernel: 16 lanes per (row, chain), 64 at a time).
template <int BMAX>
__global__ __launch_bounds__(1024) void tri_levels_block_kernel(TriArgs a, const int* __restrict__ rows,
                                                                const int* __restrict__ lptr, int lv0, int lv1,
                                                                const int* __restrict__ nn, int b,
                                                                const double* __restrict__ u, double* x) {
  const int l = threadIdx.x & 15, grp = threadIdx.x >> 4, ngrp = blockDim.x >> 4;
  for (int lv = lv0; lv < lv1; ++lv) {
    const int r0 = lptr[lv], cnt = (lptr[lv + 1] - r0) * a.nc;
    for (int it = grp; it < cnt; it += ngrp) tri_row16<BMAX>(a, rows[r0 + it / a.nc], it % a.nc, l, true, nn, b, u, x);
    __syncthreads();
  }
}

hipError_t launch_tri_levels_block(hipStream_t st, const TriArgs& a, const int* rows, const int* lptr, int lv0,
                                   int lv1, const int* nn, int b, const double* u, double* x) {
  if (b <= 16)
    hipLaunchKernelGGL(tri_levels_block_kernel<16>, dim3(1), dim3(1024), 0, st, a, rows, lptr, lv0, lv1, nn, b, u,
                       x);
  else
    hipLaunchKernelGGL(tri_levels_block_kernel<32>, dim3(1), dim3(1024), 0, st, a, rows, lptr, lv0, lv1, nn, b, u,
                       x);
  return hipGetLastError();
}

// Sync-free variant: the whole DAG in ONE persistent launch, no level
// barriers.  x starts as a NaN sentinel (kTriPending, never produced by
// arithmetic); a (row, chain) item is ready when none of the x values it
// reads is the sentinel any more, and its result is stored with device scope
// (sc1, write-through) so items on other CUs / XCDs see it.  Item order =
// level order (rows[] holds the levels back to back, chains interleaved);
// wave w takes items 4w.., 4(w+W).., ... (16 lanes per item, as tri_row16:
// the same products, the same DPP row reduction, so x is bitwise the level
// kernels' x).  Inside a wave the 4 items are retried until all are done (an
// item may read one of the same wave), and every wave's waits are bounded: on
// a timeout the word ctl[0] is set, the unfinished entries stay NaN and the
// waves leave.
// Progress does not rest on residency or dispatch order.  The static striding
// is fast when every wave of the grid runs, but a wave that is not resident
// (another launch holds CUs -- e.g. a persistent tile sweep of another
// context, which in turn waits for CUs this launch holds) would leave its
// items undone and the running waves waiting on them.  So a wave that has
// waited on one group for kTriRescueTicks raises the rescue word ctl[1]; from
// then on every running wave (and every wave that starts later) takes groups
// in increasing order from ONE ticket counter (ctl[2..3], a returning device
// atomic per group), skipping groups already done.  The claimed groups are
// always a prefix of the item order, so the lowest unfinished item is held by
// a running wave whose inputs (lower items) are all done: it completes, at any
// residency.  An item computed twice (a static wave and a rescuer) stores the
// same bits.
constexpr unsigned long long kTriPending = 0x7FF4A5A5DEAD5A5Aull;
constexpr unsigned long long kTriRescueTicks = 2000000;  // 20 ms of the 100 MHz clock on one group

__device__ __forceinline__ double tri_load_dev(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// one group of 4 items (16 lanes each) from item `base`.  Returns 0 when all
// four are done, 1 on a timeout (ctl[0] set), 2 when the group was left
// undone because a rescue is on (watch: the static pass).  skip: items whose
// x is already stored count as done (rescue mode: another wave computed them)
template <int BMAX>
__device__ __forceinline__ int tri_dag_group(const TriArgs& a, const int* __restrict__ rows, long long nitems,
                                             const int* __restrict__ nn, int b, const double* __restrict__ u,
                                             double* x, unsigned* ctl, long long base, bool watch, bool skip) {
  constexpr int J = BMAX / 16;
  const int l = threadIdx.x & 15, sub = (threadIdx.x >> 4) & 3;
  const int S = a.stride;
  const long long it = base + sub;
  const bool active = it < nitems;
  const int i = active ? rows[it / a.nc] : 0;
  const int kk = active ? (int)(it % a.nc) : 0;
  const int k = a.kidx[kk];
  const double* lr = a.linv[kk] + (size_t)i * b;
  bool done = !active;
  if (skip && active) {
    const double v = tri_load_dev(x + (size_t)i * S + k);
    done = __builtin_bit_cast(unsigned long long, v) != kTriPending;
  }
  if (__ballot(!done) == 0) return 0;
  int idx[J];
  double lv[J], xv[J];
  bool have[J];
#pragma unroll
  for (int q = 0; q < J; ++q) {
    const int j = l + 16 * q;
    idx[q] = (active && j >= 1 && j < b) ? __builtin_nontemporal_load(nn + (size_t)i * b + j) : -1;
    lv[q] = idx[q] >= 0 ? __builtin_nontemporal_load(lr + j) : 0.0;
    xv[q] = 0.0;
    have[q] = idx[q] < 0;
  }
  const double ui = (active && l == 15) ? u[(size_t)i * S + k] : 0.0;
  const double d0 = (active && l == 15) ? lr[0] : 1.0;
  const unsigned long long t0 = watch ? wall_clock64() : 0ull;
  for (unsigned spins = 0;; ++spins) {
    bool ready = true;
#pragma unroll
    for (int q = 0; q < J; ++q) {
      if (!have[q]) {
        const double v = tri_load_dev(x + (size_t)idx[q] * S + k);
        if (__builtin_bit_cast(unsigned long long, v) != kTriPending) {
          xv[q] = v;
          have[q] = true;
        } else {
          ready = false;
        }
      }
    }
    const unsigned long long bal = __ballot(ready);
    const bool grp = ((bal >> (16 * sub)) & 0xFFFFull) == 0xFFFFull;
    double p = 0.0;
#pragma unroll
    for (int q = 0; q < J; ++q) p = __builtin_fma(lv[q], xv[q], p);
    p += dpp_f64<0x111, 0xF, true>(p);  // row_shr:1
    p += dpp_f64<0x112, 0xF, true>(p);  // row_shr:2
    p += dpp_f64<0x114, 0xF, true>(p);  // row_shr:4
    p += dpp_f64<0x118, 0xF, true>(p);  // row_shr:8 -> lane 15 holds the row sum
    if (!done && grp) {
      if (l == 15)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(x + (size_t)i * S + k),
                           __builtin_bit_cast(unsigned long long, (ui - p) / d0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      done = true;
    }
    if (__ballot(!done) == 0) return 0;
    // (wave-uniform: the control words are read by the first lane only)
    if ((spins & 255u) == 255u) {
      if (spins > (1u << 22) ||
          __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 1;
      }
      if (watch) {
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
          return 2;
        if (wall_clock64() - t0 > kTriRescueTicks) {
          __hip_atomic_store(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return 2;
        }
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

template <int BMAX>
__global__ __launch_bounds__(256) void tri_dag_kernel(TriArgs a, const int* __restrict__ rows, long long nitems,
                                                      const int* __restrict__ nn, int b,
                                                      const double* __restrict__ u, double* x,
                                                      unsigned* __restrict__ ctl) {
  const long long W = (long long)gridDim.x * (blockDim.x >> 6);
  const long long w = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  bool rescue = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  for (long long base = 4 * w; base < nitems && !rescue; base += 4 * W) {
    const int r = tri_dag_group<BMAX>(a, rows, nitems, nn, b, u, x, ctl, base, true, false);
    if (r == 1) return;
    rescue = r == 2;
  }
  // a rescue raised while this wave was in its static pass (or after it):
  // help, in ticket order
  if (!rescue) rescue = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (!rescue) return;
  unsigned long long* head = reinterpret_cast<unsigned long long*>(ctl + 2);
  for (;;) {
    unsigned long long g = 0;
    if ((threadIdx.x & 63) == 0) g = __hip_atomic_fetch_add(head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g = __shfl(g, 0);
    if ((long long)g * 4 >= nitems) return;
    if (tri_dag_group<BMAX>(a, rows, nitems, nn, b, u, x, ctl, (long long)g * 4, false, true) == 1) return;
  }
}

__global__ void fill_u64_kernel(long long n, unsigned long long v, unsigned long long* __restrict__ p) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    p[e] = v;
}

// x := the pending sentinel; the rescue word (:= 2 when forced: every wave
// goes straight to the ticket order -- NNGP_TRI_RESCUE=1, the tests' way to
// check that order; a wave that raises it stores 1) and the ticket counter of
// the tri_dag launch that follows := 0 (the timeout word ctl[0] stays set
// until the host has read it).  ctl[4] counts the solves whose rescue was
// raised (not forced), the previous solve's added here (nngp_tri_rescues).
__global__ void tri_dag_init_kernel(long long n, double* __restrict__ x, unsigned* __restrict__ ctl, unsigned rescue) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctl[4] += ctl[1] == 1u ? 1u : 0u;
    ctl[1] = rescue;
    *reinterpret_cast<unsigned long long*>(ctl + 2) = 0ull;
  }
  unsigned long long* p = reinterpret_cast<unsigned long long*>(x);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    p[e] = kTriPending;
}

hipError_t launch_tri_dag(hipStream_t st, const TriArgs& a, const int* rows, int nrows, const int* nn, int b,
                          const double* u, double* x, long long x_len, unsigned* ctl, bool rescue, int oversub) {
  const auto kern = b <= 16 ? tri_dag_kernel<16> : tri_dag_kernel<32>;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cus <= 0)
    return hipErrorInvalidDevice;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), 256, 0);
  if (e != hipSuccess) return e;
  if (per_cu <= 0) return hipErrorInvalidConfiguration;
  const long long nitems = (long long)nrows * a.nc;
  // oversub > 1 (tests, NNGP_TRI_OVERSUB): a grid of oversub x the resident
  // workgroups, so that the static order waits on waves that are not
  // resident and only the rescue completes the solve
  long long g = std::min<long long>((long long)cus * per_cu * (oversub > 1 ? oversub : 1), (nitems + 15) / 16);
  if (g < 1) g = 1;
  const int gf = (int)std::min<long long>((x_len + 255) / 256, 4096);
  hipLaunchKernelGGL(tri_dag_init_kernel, dim3(gf > 0 ? gf : 1), dim3(256), 0, st, x_len, x, ctl, rescue ? 2u : 0u);
  hipLaunchKernelGGL(kern, dim3((int)g), dim3(256), 0, st, a, rows, nitems, nn, b, u, x, ctl);
  return hipGetLastError();
}

// B 1 (row sums of the factor, device row order): a warm sweep call after a
// beta_0-only change (update_Gaussian.R:219-224) starts from r - d B 1
// instead of recomputing r = B w (capi.hip warm_kinds, tiles.hip prologue)
__global__ void linv_rowsum_kernel(const double* __restrict__ linv, int n, int b, double* __restrict__ out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int j = 0; j < b; ++j) s += linv[(size_t)i * b + j];
    out[i] = s;
  }
}

hipError_t launch_linv_rowsum(hipStream_t st, const double* linv, int n, int b, double* out) {
  const int g = std::min((n + 255) / 256, 4096);
  hipLaunchKernelGGL(linv_rowsum_kernel, dim3(g > 0 ? g : 1), dim3(256), 0, st, linv, n, b, out);
  return hipGetLastError();
}

__global__ void permute_gather_kernel(int n, const int* __restrict__ idx, const double* __restrict__ src,
                                      double* __restrict__ dst) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

__global__ void permute_scatter_kernel(int n, const int* __restrict__ idx, const double* __restrict__ src,
                                       double* __restrict__ dst) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[idx[i]] = src[i];
}

hipError_t launch_permute_gather(hipStream_t st, int n, const int* idx, const double* src, double* dst) {
  hipLaunchKernelGGL(permute_gather_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, n, idx, src, dst);
  return hipGetLastError();
}

hipError_t launch_permute_scatter(hipStream_t st, int n, const int* idx, const double* src, double* dst) {
  hipLaunchKernelGGL(permute_scatter_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, n, idx, src,
                     dst);
  return hipGetLastError();
}

__global__ void axpby_shift_kernel(int n, const double* __restrict__ x, int xstride, double scale, double shift,
                                   double* __restrict__ y) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = shift + scale * x[(size_t)i * xstride];
}

hipError_t launch_axpby_shift(hipStream_t st, int n, const double* x, int xstride, double scale, double shift,
                              double* y) {
  int g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(axpby_shift_kernel, dim3(g), dim3(kBlock), 0, st, n, x, xstride, scale, shift, y);
  return hipGetLastError();
}

__global__ void spin_kernel(unsigned long long ticks) {
  // wall_clock64(): constant 100 MHz counter on gfx950
  unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

hipError_t launch_spin(hipStream_t st, double seconds) {
  if (seconds > 1.0) seconds = 1.0;
  int rate = 0;
  if (hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0) != hipSuccess || rate <= 0) rate = 100000;
  unsigned long long ticks = (unsigned long long)(seconds * rate * 1e3);  // rate in kHz
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, st, ticks);
  return hipGetLastError();
}

hipError_t launch_normals(hipStream_t st, uint64_t seed, uint64_t sweep, int n, double* z) {
  int g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(normals_kernel, dim3(g), dim3(kBlock), 0, st, seed, sweep, n, z);
  return hipGetLastError();
}

}  // namespace nngp
