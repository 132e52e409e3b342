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
#include <cstdlib>

#include <cmath>

namespace nngp {

// DPP move of a double (both halves; lanes without a source read +0.0)
template <int CTRL, int RM, bool BC>
__device__ __forceinline__ double dpp_f64(double x) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, RM, 0xF, BC);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, RM, 0xF, BC);
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}

// ------------------------------------------------------------------ RNG
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
  }
}

// Standard normal by inversion (R's own default, norm_rand INVERSION ->
// qnorm): Wichura's AS241 (PPND16) at p in (0, 1).
__device__ __forceinline__ double qnorm_as241(double p) {
  const double q = p - 0.5;
  double r, val;
  if (fabs(q) <= 0.425) {
    r = 0.180625 - q * q;
    return q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r +
                    45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
                  133.14166789178437745) * r + 3.387132872796366608) /
           (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r +
                 21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
             42.313330701600911252) * r + 1.);
  }
  r = q < 0 ? p : 1.0 - p;
  r = sqrt(-log(r));
  if (r <= 5.) {
    r -= 1.6;
    val = (((((((r * 7.7454501427834140764e-4 + .0227238449892691845833) * r + .24178072517745061177) * r +
               1.27045825245236838258) * r + 3.64784832476320460504) * r + 5.7694972214606914055) * r +
             4.6303378461565452959) * r + 1.42343711074968357734) /
          (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r + .0151986665636164571966) * r +
               .14810397642748007459) * r + .68976733498510000455) * r + 1.6763848301838038494) * r +
             2.05319162663775882187) * r + 1.);
  } else {
    r -= 5.;
    val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r + .0012426609473880784386) * r +
               .026532189526576123093) * r + .29656057182850489123) * r + 1.7848265399172913358) * r +
             5.4637849111641143699) * r + 6.6579046435011037772) /
          (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r + 1.8463183175100546818e-5) * r +
               7.868691311456132591e-4) * r + .0148753612908506148525) * r + .13692988092273580531) * r +
             .59983220655588793769) * r + 1.);
  }
  return q < 0.0 ? -val : val;
}

// N(0,1) for location `loc` of global sweep `sweep`: one Philox4x32-10 call,
// counter (loc, sweep_lo, sweep_hi, 0x5EED), key = seed; its first 53 bits
// give u in (0,1); z = qnorm(u) (AS241).  Every location draws alone, so any
// subset of locations (a colour class, a tile) generates exactly its own.
__device__ __forceinline__ double normal_loc(uint64_t seed, uint64_t sweep, uint32_t loc) {
  uint32_t c[4] = {loc, (uint32_t)sweep, (uint32_t)(sweep >> 32), 0x5EEDu};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint64_t a = ((((uint64_t)c[1]) << 32) | c[0]) >> 11;
  return qnorm_as241(((double)a + 0.5) * 0x1.0p-53);
}

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
// Taylor polynomial; within 1 ulp of the correctly rounded exp (measured,
// scripts/micro/dmath.hip).  Very negative x (including the padding
// distances of ~1e30) gives exactly 0.
__device__ __forceinline__ double exp_nonpos(double x, const double* tab) {
  const double k = __builtin_rint(x * 92.33248261689366);  // 64/ln2
  double r = __builtin_fma(-k, 0.010830424696249145, x);    // ln2/64, high part
  r = __builtin_fma(-k, 3.623510646634843e-19, r);          // low part
  const int ki = (int)k;                                      // saturates for huge |x|
  double p = 1.3888888888888889e-03;
  p = __builtin_fma(p, r, 8.3333333333333332e-03);
  p = __builtin_fma(p, r, 4.1666666666666664e-02);
  p = __builtin_fma(p, r, 1.6666666666666666e-01);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  const double t = tab[ki & 63];
  return __builtin_ldexp(__builtin_fma(p * r, t, t), ki >> 6);
}

// sqrt(s) for normal s > 0 (squared distances): hardware rsq (~2^-24) and
// two residual corrections; correctly rounded on every sample measured.
__device__ __forceinline__ double sqrt_pos(double s) {
  const double y = __builtin_amdgcn_rsq(s);
  const double h = 0.5 * y;
  double g = s * y;
  double e = __builtin_fma(-g, g, s);
  g = __builtin_fma(e, h, g);
  e = __builtin_fma(-g, g, s);
  return __builtin_fma(e, h, g);
}

// 1/sqrt(s) for normal s > 0: hardware rsq + two Newton-Raphson steps
// (within ~1 ulp).
__device__ __forceinline__ double rsqrt_pos(double s) {
  double y = __builtin_amdgcn_rsq(s);
  const double hs = 0.5 * s;
  y = y * __builtin_fma(-hs * y, y, 1.5);
  y = y * __builtin_fma(-hs * y, y, 1.5);
  return y;
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
struct ScaleArgs {
  double c[8];
  int covfun;
};

__global__ void scale_coords_kernel(ScaleArgs a, const double* __restrict__ locs, int n, int d,
                                    double* __restrict__ sc, int ds) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
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
template <int BM, int FAM, int DS, class XA>
__device__ __forceinline__ void factor_row(const XA& xa, int bs, int i, double var, double nugget, int b,
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
      L[t * (t + 1) / 2 + q] = FAM == 1 ? var * ((1.0 + dist) * e) : var * e;
    }
#pragma unroll
    for (int q = 0; q <= t; ++q) {
      double s = q == t ? (dt ? 1.0 : var * (1.0 + nugget)) : L[t * (t + 1) / 2 + q];
#pragma unroll
      for (int p = 0; p < q; ++p) s -= L[t * (t + 1) / 2 + p] * L[q * (q + 1) / 2 + p];
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
    if (j < b) linv[(size_t)i * b + j] = (j < bs) ? x[BM - 1 - j] : 0.0;
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

// Grid-stride over groups of 64 rows with a two-deep software pipeline: the
// next group's coordinate gathers and the group after's neighbour indices
// are in flight while this group's covariance/Cholesky runs (one wave per
// SIMD fits the register footprint, so no other wave hides that latency).
template <int BM, int FAM, int DS>
__global__ __launch_bounds__(64) void factor_kernel(double var, double nugget, double nu, double norm,
                                                   const double* __restrict__ sc,
                                                   const int* __restrict__ nn, int n, int b,
                                                   double* __restrict__ linv, int* __restrict__ fail) {
  __shared__ double tab[64];
  tab[threadIdx.x] = kExp2Tab[threadIdx.x];
  __syncthreads();
  const int stride = gridDim.x * 64;
  int i = blockIdx.x * 64 + threadIdx.x;
  int nc[BM], nx[BM];
  double X[BM][DS];
  load_nn_row<BM>(nc, nn, i, n, b);
  int bs = gather_coords<BM, DS>(X, nc, sc, i, n);
  load_nn_row<BM>(nx, nn, i + stride, n, b);
  for (int base = blockIdx.x * 64; base < n; base += stride, i += stride) {
    double Xn[BM][DS];
    const int bsn = gather_coords<BM, DS>(Xn, nx, sc, i + stride, n);
    load_nn_row<BM>(nx, nn, i + 2 * stride, n, b);
    if (i < n)
      factor_row<BM, FAM, DS>([&](int r, int k) { return X[r][k]; }, bs, i, var, nugget, b, tab, linv, fail);
#pragma unroll
    for (int r = 0; r < BM; ++r)
#pragma unroll
      for (int k = 0; k < DS; ++k) X[r][k] = Xn[r][k];
    bs = bsn;
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

// Planar coordinates (DS = 2): the coordinates of the next group of 64 rows
// are DMA'd global -> LDS (global_load_lds_dwordx4, one 16-byte point per
// lane and neighbour) into the second of two stages while this group
// computes, so the in-flight coordinates occupy no VGPRs (the factor's L
// needs nearly all of them).  Stage layout [r][lane] x 16 B; 32 KB per
// one-wave workgroup at BM = 16.  Missing neighbours load the point itself
// and read back as the far-away padding of gather_coords.
#define NNGP_FACTOR_ARGS var, nugget, nu, norm, sc, nn, n, b, linv, fail
// workgroups of a grid-stride kernel: NNGP_FACTOR_GRID (default 2) x the
// resident one-wave workgroups of the current device, at most the row
// groups.  Twice resident measured best at n = 1e6 (0.350 vs 0.354 ms at 1x,
// 0.373 at 4x): a shorter last round without giving up the pipeline.
static int resident_grid(const void* kern, int groups) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cus <= 0)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0) != hipSuccess || per_cu <= 0) per_cu = 4;
  static const int mult = [] {
    const char* e = std::getenv("NNGP_FACTOR_GRID");
    int v = e ? std::atoi(e) : 2;
    return v >= 1 && v <= 64 ? v : 2;
  }();
  const long long g = (long long)cus * per_cu * mult;
  return (int)(g < groups ? g : groups);
}

template <int BM, int FAM, int DS>
static hipError_t launch_factor_one(hipStream_t st, double var, double nugget, double nu, double norm,
                                    const double* sc, const int* nn, int n, int b, double* linv, int* fail) {
  const auto kern = factor_kernel<BM, FAM, DS>;
  const int g = resident_grid(reinterpret_cast<const void*>(kern), (n + 63) / 64);
  hipLaunchKernelGGL(kern, dim3(g), dim3(64), 0, st, NNGP_FACTOR_ARGS);
  return hipGetLastError();
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
  if (family == 0) return launch_factor_rt<0>(st, ds, NNGP_FACTOR_ARGS);
  return launch_factor_rt<1>(st, ds, NNGP_FACTOR_ARGS);
}
#undef NNGP_FACTOR_ARGS

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
  for (int k = blockIdx.x * (blockDim.x / G) + threadIdx.x / G; k < n; k += rows_per_grid) {
    double l = 0.0, xv = 0.0;
    if (g < b) {
      const int idx = nn[(size_t)k * b + g];
      if (idx >= 0) {
        l = linv[(size_t)k * b + g];
        xv = x[idx] - shift;
      }
    }
    double u = l * xv, a = l;
#pragma unroll
    for (int off = 1; off < G; off <<= 1) {
      u += __shfl_xor(u, off, 64);
      a += __shfl_xor(a, off, 64);
    }
    if (g == 0) {
      acc[0] += log(linv[(size_t)k * b]);
      acc[1] += u * u;
      acc[2] += a * a;
      acc[3] += a * u;
      if (out) out[(size_t)k * out_stride] = u;
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
constexpr uint32_t kTPad = (1u << 17) - 1;
constexpr uint32_t kTStart = 1u << 30, kTEnd = 1u << 31;
constexpr int kTExported = 1 << 30;
constexpr int kTSlots = 256;       // slots per own batch (graph_prep.h kTileSlotsMax)
constexpr int kTSpreadLds = 82 * 1024;  // LDS floor: at most one tile per CU
constexpr int kTCuLds = 160 * 1024;     // LDS per CU

int tile_lds_bytes(int max_rows, int C, int NT, int K, int max_batches, int max_gslots) {
  const int rbytes = ((max_rows * C * 8 + 15) / 16) * 16;
  return rbytes + kTSlots * C * 8 + (NT / 64) * C * 8 + 4 * C * 8 + ((max_gslots * C + 1) / 2) * 16 +
         max_batches * 16 + 4 * (K + 1) * 4 + (NT / 64) * 4 + 64;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// dst[k] = p, in stream order (the current-factor table of captured graphs:
// the value travels as a kernel argument, no host buffer to keep alive)
__global__ void set_ptr_kernel(const double** dst, int k, const double* p) {
  if (threadIdx.x == 0) dst[k] = p;
}

hipError_t launch_set_ptr(hipStream_t st, const double** dst, int k, const double* p) {
  hipLaunchKernelGGL(set_ptr_kernel, dim3(1), dim3(64), 0, st, dst, k, p);
  return hipGetLastError();
}

__global__ void tile_call_bump_kernel(unsigned* ctl) {
  ctl[0] += 1u;  // call id (never 0 inside a launch)
  ctl[1] = 0u;   // timeout word
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
        __hip_atomic_store(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  static constexpr int IMAX = (kTSlots * C + NT - 1) / NT;
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
      b.pk[j] = kTPad;
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
                                                TileBatchRegs<C, NT, RMAX>& b, int t) {
#pragma unroll
  for (int k = 0; k < TileBatchRegs<C, NT, RMAX>::IMAX; ++k) {
    const int u = t + k * NT;
    if (u < b.ns * C) {
      const int q = u / C, ch = u - q * C;
      const double inv_s2 = sc_s[2 * ch], inv_t2 = sc_s[2 * ch + 1];
      double z = 0.0;
      if (a.z_in) z = a.z_in[((size_t)s * D.n + b.x0 + q) * CS + ch];
      else z = normal_loc(seed_s[2 * ch], seed_s[2 * ch + 1] + s, (uint32_t)b.loc[k]);
      const double P = b.a0[k] * inv_s2 + (double)b.nobs[k] * inv_t2;
      const double cR = inv_t2 * b.a1[k] + inv_s2 * (b.a0[k] * b.w[k]);
      b.a0[k] = cR;
      b.a1[k] = 1.0 / P;
      b.zs[k] = z / sqrt(P);
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

// per-workgroup state of the persistent sweep
struct TileState {
  double* r_s;
  double* acc_s;
  double* wsum;
  double* sc_s;   // C x {inv_s2, inv_t2}
  unsigned long long* seed_s;  // C x {seed, counter_base}
  int4* batch_s;  // this tile's own batches
  int* bptr_s;    // K+1: batches of colour c = batch_s[bptr_s[c] .. bptr_s[c+1])
  int* gptr_s;    // K+1: ghost cells of colour c (global indices)
  int* gsp_s;     // K+1: foreign slots of colour c (global indices into gslot)
  int* bsp_s;     // K: split layouts, first boundary batch of colour c (as bptr_s)
  double* gdw_s;  // foreign slots x C: their dw of the current colour
  int* wflag;
  unsigned* spin_s;
  __amdgpu_buffer_rsrc_t gran;
  unsigned call;
  int gsl;                          // this phase's first foreign slot index of the thread (loaded a phase ahead)
  unsigned* tmo;
  int G;                            // tile shard: ranks (1: single GPU)
  bool timed_out;
  int T, t, lane, wv, K, nph, ph;
  unsigned long long tp[8], t_prev;
};

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
#define TLSTAMP(S, k)                                                                         \
  do {                                                                                        \
    if (PROBE == 2 && (S).t == 0 && (S).ph < kTimelinePhases)                                 \
      D.dbg[((size_t)(S).T * kTimelinePhases + (S).ph) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)


// one step of a segmented inclusive scan (flag f = "a segment starts here or
// in an earlier lane of my partial"): (f_e, v_e) (+) (f, v) = (f_e | f, f ? v : v_e + v)
template <int CTRL, int RM, bool BC, int C>
__device__ __forceinline__ void seg_scan_step(double (&v)[C], int& f) {
  double e[C];
#pragma unroll
  for (int ch = 0; ch < C; ++ch) e[ch] = dpp_f64<CTRL, RM, BC>(v[ch]);
  const int fe = __builtin_amdgcn_update_dpp(0, f, CTRL, RM, 0xF, BC);
  if (!f) {
#pragma unroll
    for (int ch = 0; ch < C; ++ch) v[ch] = e[ch] + v[ch];
  }
  f |= fe;
}

// one own batch of colour c (epoch): products -> slot totals -> draws ->
// scatter.  LDS and registers only, plus the draws' stores: no global load
// (a load here would wait behind the next batch's prefetch, vmcnt is in order)
template <int C, int NT, int RMAX, int PROBE, int SH, int CS = C>
__device__ __forceinline__ void tile_own_draw(const TileDev& D, const TileLaunch& a, const TileShard& sh, TileState& S,
                                              TileBatchRegs<C, NT, RMAX>& b, unsigned epoch) {
  constexpr int IMAX = TileBatchRegs<C, NT, RMAX>::IMAX;
  const int t = S.t, lane = S.lane, wv = S.wv;
  double* r_s = S.r_s;
  double* acc_s = S.acc_s;
  const int R = b.R, nit = b.ns * C;
  // products, running sums restarted at slot starts.  A slot that began in
  // this thread is complete at its last cell (-> acc_s); the thread's first
  // cells may continue a slot of earlier threads: its end (if here) waits for
  // the carry of those threads.
  double run[C], cont[C];
  int cont_q = -1;
  bool seen_start = false;
#pragma unroll
  for (int ch = 0; ch < C; ++ch) { run[ch] = 0.0; cont[ch] = 0.0; }
#pragma unroll
  for (int j = 0; j < RMAX; ++j) {
    if (j < R) {
      const uint32_t lr = b.pk[j] & kTPad;
      const bool st = (b.pk[j] & kTStart) != 0;
#pragma unroll
      for (int ch = 0; ch < C; ++ch) {
        const double p = (lr != kTPad) ? b.v[j][ch] * r_s[lr * C + ch] : 0.0;
        run[ch] = st ? p : run[ch] + p;
      }
      seen_start |= st;
      if (b.pk[j] & kTEnd) {
        const int q = (int)((b.pk[j] >> 17) & 0x7FF);
        if (seen_start) {
#pragma unroll
          for (int ch = 0; ch < C; ++ch) acc_s[q * C + ch] = run[ch];
        } else {
          cont_q = q;
#pragma unroll
          for (int ch = 0; ch < C; ++ch) cont[ch] = run[ch];
        }
      }
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
    if (cont_q >= 0) acc_s[cont_q * C + ch] = cont[ch] + cp;
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
template <int C, int NT, int RMAX, int PROBE>
__device__ __forceinline__ void tile_own_scatter(TileState& S, const TileBatchRegs<C, NT, RMAX>& b, int R) {
  double* r_s = S.r_s;
  const double* acc_s = S.acc_s;
#pragma unroll
  for (int j = 0; j < RMAX; ++j) {
    if (j < R) {
      const uint32_t lr = b.pk[j] & kTPad;
      if (lr != kTPad) {
        const int q = (int)((b.pk[j] >> 17) & 0x7FF);
#pragma unroll
        for (int ch = 0; ch < C; ++ch) r_s[lr * C + ch] += b.v[j][ch] * acc_s[q * C + ch];
      }
    }
  }
  TSTAMP(S, 4);
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
          if (!S.timed_out) __hip_atomic_store(S.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    D.dbg[((size_t)S.T * kTimelinePhases + S.ph) * 8 + 5] = *S.spin_s;
    *S.spin_s = 0;
  }
  for (int gb = g0; gb < g1; gb += NT * GMAX) {
    if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, gr, t);
#pragma unroll
    for (int k = 0; k < GMAX; ++k)
      if (gr.lr[k] >= 0)
#pragma unroll
        for (int ch = 0; ch < C; ++ch) S.r_s[gr.lr[k] * C + ch] += gr.gv[k][ch] * S.gdw_s[gr.gx[k] * C + ch];
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
            if (!S.timed_out) __hip_atomic_store(S.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
      D.dbg[((size_t)S.T * kTimelinePhases + S.ph) * 8 + 5] = *S.spin_s;
      *S.spin_s = 0;
    }
    for (int gb = g0; gb < g1; gb += NT * GMAX) {
      if (gb != g0) tile_load_ghosts<C, NT, GMAX>(D, gb, g1, gr, t);
#pragma unroll
      for (int k = 0; k < GMAX; ++k)
        if (gr.lr[k] >= 0)
#pragma unroll
          for (int ch = 0; ch < C; ++ch) S.r_s[gr.lr[k] * C + ch] += gr.gv[k][ch] * S.gdw_s[gr.gx[k] * C + ch];
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
template <int C, int NT, int RMAX, int GMAX, int DB, int PROBE, int SH, int RG, int IB, int CS>
__device__ __forceinline__ void sweep_tiles_body(const TileDev& D0, TileLaunch a, const TileShard& sh) {
  using BR = TileBatchRegs<C, NT, RMAX>;
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
  const int b_lo = D.batch_ptr[T * K], nbt = D.batch_ptr[T * K + K] - b_lo;
  S.r_s = RG ? D.rg + (size_t)row0 * C : smem;
  S.acc_s = RG ? smem : smem + ((nrows * C + 1) / 2) * 2;  // kTSlots x C: slot totals, then dw
  S.wsum = S.acc_s + kTSlots * C;                // NW x C: segmented wave totals
  S.sc_s = S.wsum + NW * C;                      // C x {inv_s2, inv_t2}
  S.seed_s = reinterpret_cast<unsigned long long*>(S.sc_s + 2 * C);
  S.gdw_s = reinterpret_cast<double*>(S.seed_s + 2 * C);  // max foreign slots x C (even count)
  S.batch_s = reinterpret_cast<int4*>(S.gdw_s + ((D.max_gslots * C + 1) / 2) * 2);
  S.bptr_s = reinterpret_cast<int*>(S.batch_s + nbt);
  S.gptr_s = S.bptr_s + K + 1;
  S.gsp_s = S.gptr_s + K + 1;
  S.bsp_s = S.gsp_s + K + 1;                     // K+1 (split layouts)
  S.wflag = S.bsp_s + K + 1;                     // NW: the wave holds a slot start
  S.spin_s = reinterpret_cast<unsigned*>(S.wflag + NW);  // NNGP_PROBE=2: max poll spins of the phase
  if (PROBE == 2 && t == 0) *S.spin_s = 0;
  TSTAMP(S, -1);
  for (int lr = t; lr < nrows; lr += NT) {
    const size_t g = (size_t)D.erow[row0 + lr] * CS;
#pragma unroll
    for (int ch = 0; ch < C; ++ch) S.r_s[lr * C + ch] = D.r[g + ch];
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
  if (PROBE == 1 && t == 0) {
    unsigned long long* o = D.dbg + (size_t)T * 8;
    for (int k = 0; k < 8; ++k) o[k] = S.tp[k];
  }
}

template <int C, int NT, int RMAX, int GMAX, int DB, int PROBE, int SH, int RG, int IB>
__global__ __launch_bounds__(NT) void sweep_tiles_kernel(TileDev D0, TileLaunch a, TileShard sh) {
  sweep_tiles_body<C, NT, RMAX, GMAX, DB, PROBE, SH, RG, IB, C>(D0, a, sh);
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
template <int C, int NT, int PROBE, int SH, int RG = 0, int IB0 = -1>
static hipError_t launch_tiles_c(hipStream_t st, const TileDev& D, const TileLaunch& a, int lds, const TileShard* sh,
                                 int grid) {
  constexpr int RMAX = tile_rmax(C, NT);
  constexpr int DB = tile_double_buffer(C, NT);
  constexpr int GMAX = tile_gmax(NT);
  // split layouts (interior first) at one register set; IB0 >= 0 pins it
  if constexpr (IB0 < 0 && DB == 0) {
    if (D.batch_split) return launch_tiles_c<C, NT, PROBE, SH, RG, 1>(st, D, a, lds, sh, grid);
    return launch_tiles_c<C, NT, PROBE, SH, RG, 0>(st, D, a, lds, sh, grid);
  }
  constexpr int IB = IB0 > 0 ? 1 : 0;
  if (D.batch_split && !IB) return hipErrorInvalidValue;  // split layout: double-buffered path not for it
  auto k = sweep_tiles_kernel<C, NT, RMAX, GMAX, DB, PROBE, SH, RG, IB>;
  lds = lds < kTSpreadLds ? kTSpreadLds : lds;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
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
                                  int grid) {
  if (D.rg) {  // r in global memory: 512- or 1024-thread tiles, one GPU
    if constexpr (NT == 512 || NT == 1024) {
      if (sh) return hipErrorInvalidValue;
      switch (D.C) {
        case 1: return launch_tiles_c<1, NT, 0, 0, 1>(st, D, a, lds, nullptr, 0);
        case 2: return launch_tiles_c<2, NT, 0, 0, 1>(st, D, a, lds, nullptr, 0);
        case 3: return launch_tiles_c<3, NT, 0, 0, 1>(st, D, a, lds, nullptr, 0);
        case 4: return launch_tiles_c<4, NT, 0, 0, 1>(st, D, a, lds, nullptr, 0);
        default: return hipErrorInvalidValue;
      }
    }
    return hipErrorInvalidValue;
  }
  if (sh) {
    switch (D.C) {
      case 1: return launch_tiles_c<1, NT, 0, 1>(st, D, a, lds, sh, grid);
      case 2: return launch_tiles_c<2, NT, 0, 1>(st, D, a, lds, sh, grid);
      case 3: return launch_tiles_c<3, NT, 0, 1>(st, D, a, lds, sh, grid);
      case 4: return launch_tiles_c<4, NT, 0, 1>(st, D, a, lds, sh, grid);
      default: return hipErrorInvalidValue;
    }
  }
  if (D.dbg && D.probe == 1) {
    switch (D.C) {
      case 1: return launch_tiles_c<1, NT, 1, 0>(st, D, a, lds, nullptr, 0);
      case 3: return launch_tiles_c<3, NT, 1, 0>(st, D, a, lds, nullptr, 0);
      default: break;
    }
  }
  if (D.dbg && D.probe == 2) {
    switch (D.C) {
      case 1: return launch_tiles_c<1, NT, 2, 0>(st, D, a, lds, nullptr, 0);
      case 3: return launch_tiles_c<3, NT, 2, 0>(st, D, a, lds, nullptr, 0);
      default: break;
    }
  }
  switch (D.C) {
    case 1: return launch_tiles_c<1, NT, 0, 0>(st, D, a, lds, nullptr, 0);
    case 2: return launch_tiles_c<2, NT, 0, 0>(st, D, a, lds, nullptr, 0);
    case 3: return launch_tiles_c<3, NT, 0, 0>(st, D, a, lds, nullptr, 0);
    case 4: return launch_tiles_c<4, NT, 0, 0>(st, D, a, lds, nullptr, 0);
    default: return hipErrorInvalidValue;
  }
}

// chain-split launch (256-thread tiles, one chain per workgroup, D.C per CU)
template <int CS>
static hipError_t launch_tiles_cs(hipStream_t st, const TileDev& D, const TileLaunch& a, int lds) {
  constexpr int NT = 256;
  auto k = sweep_tiles_cs_kernel<CS, NT, tile_rmax_cs(NT), tile_gmax(NT)>;
  // LDS floor: at most CS workgroups per CU
  const int floor = kTCuLds / (CS + 1) + 64;
  lds = lds < floor ? floor : lds;
  if (lds * CS > kTCuLds) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tile_call_bump_kernel, dim3(1), dim3(1), 0, st, D.ctl);
  hipLaunchKernelGGL(k, dim3(D.T * CS), dim3(NT), lds, st, D, a);
  return hipGetLastError();
}

hipError_t launch_sweep_tiles_cs(hipStream_t st, const TileDev& D, const TileLaunch& a, int max_rows, int NT,
                                 int max_batches, int max_gslots) {
  if (NT != 256 || D.rg || D.batch_split || D.dbg) return hipErrorInvalidValue;
  const int lds = tile_lds_bytes(max_rows, 1, NT, D.K, max_batches, max_gslots);
  switch (D.C) {
    case 2: return launch_tiles_cs<2>(st, D, a, lds);
    case 3: return launch_tiles_cs<3>(st, D, a, lds);
    case 4: return launch_tiles_cs<4>(st, D, a, lds);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_sweep_tiles(hipStream_t st, const TileDev& D, const TileLaunch& a, int max_rows, int NT,
                              int max_batches, int max_gslots, const TileShard* sh, int grid) {
  const int lds = tile_lds_bytes(D.rg ? 0 : max_rows, D.C, NT, D.K, max_batches, max_gslots);
  switch (NT) {
    case 256: return launch_tiles_nt<256>(st, D, a, lds, sh, grid);
    case 512: return launch_tiles_nt<512>(st, D, a, lds, sh, grid);
    case 1024: return launch_tiles_nt<1024>(st, D, a, lds, sh, grid);
    default: return hipErrorInvalidValue;
  }
}

// B values of chain `chain` into the tile layout + precision_diag (column
// sums of squares in stream = row order, as sell_refresh); workgroups
// [0, nbatches) take one own batch each (NT = the layout's threads per tile,
// cell f of the batch at off + (f % R)*NT + f / R), the rest copy ghost values
__global__ __launch_bounds__(256) void tile_refresh_kernel(TileDev D, int nbatches, int NT,
                                                           const int* __restrict__ cell_src,
                                                           const int* __restrict__ gsrc,
                                                           const double* __restrict__ linv, int chain) {
  __shared__ double sq[4096];
  __shared__ unsigned char endf[4096];
  const int t = threadIdx.x;
  if ((int)blockIdx.x >= nbatches) {
    double* gv = const_cast<double*>(D.gval) + (size_t)chain * D.n_gcells;
    for (long long g = (long long)(blockIdx.x - nbatches) * 256 + t; g < D.n_gcells;
         g += (long long)(gridDim.x - nbatches) * 256)
      gv[g] = linv[gsrc[g]];
    return;
  }
  const int4 B = D.batch[blockIdx.x];  // refresh kernel: one batch per workgroup
  double* cv = const_cast<double*>(D.cell_val) + (size_t)chain * D.n_cells;
  const int R = B.y & 0xFFFF;
  for (int e0 = t; e0 < R * NT; e0 += 256) {
    const long long e = B.x + e0;
    const int src = cell_src[e];
    const double v = src >= 0 ? linv[src] : 0.0;
    cv[e] = v;
    const int f = (e0 % NT) * R + e0 / NT;  // e0 = j*NT + thread
    sq[f] = v * v;
    endf[f] = (D.cell_pk[e] & kTEnd) ? 1 : 0;
  }
  __syncthreads();
  if (t < B.z) {
    const int x = B.w + t;
    const int f0 = D.sinfo[x].y & 0xFFFFF;
    double s = 0.0;
    for (int f = f0;; ++f) {
      s += sq[f];
      if (endf[f]) break;
    }
    D.dr[(size_t)x * D.C + chain].x = s;
  }
}

hipError_t launch_tile_refresh(hipStream_t st, const TileDev& D, int nbatches, int NT, const int* cell_src,
                               const int* gsrc, const double* linv, int chain) {
  const int gx = D.n_gcells > 0 ? 256 : 0;
  if (nbatches + gx == 0) return hipSuccess;
  hipLaunchKernelGGL(tile_refresh_kernel, dim3(nbatches + gx), dim3(256), 0, st, D, nbatches, NT, cell_src, gsrc,
                     linv, chain);
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
