// Device helpers shared by the NNGP kernel translation units (gfx950):
// DPP moves, the Philox4x32-10 counter RNG and the AS241 normal inversion.
#pragma once
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

namespace nngp {

// DPP move of a double (both halves; lanes without a source read +0.0)
template <int CTRL, int RM, bool BC>
__device__ __forceinline__ double dpp_f64(double x) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, RM, 0xF, BC);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, RM, 0xF, BC);
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
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

// log x for x in (0, 1] (AS241's tail, x = min(p, 1 - p) < 0.075): x = m 2^e
// with m in [sqrt(1/2), sqrt(2)), log x = e ln2 + 2 atanh(s), s = (m-1)/(m+1),
// |s| <= 0.1716, the atanh series to s^21 (truncation < 2^-55 relative);
// s by a hardware reciprocal, two Newton steps and one residual correction.
// Within 2 ulp of the correctly rounded log (tests: test_log_unit_accuracy,
// CPU; device normals vs the oracle's libm-based ones to 1e-14), about a
// third of the instructions of the library log on the sweep's critical path.
__host__ __device__ __forceinline__ double log_unit(double x) {
  int e;
  double m = frexp(x, &e);
  if (m < 0.70710678118654752440) {
    m += m;
    --e;
  }
  const double f = m - 1.0, d = m + 1.0;
#ifdef __HIP_DEVICE_COMPILE__
  double y = __builtin_amdgcn_rcp(d);
#else
  double y = 1.0 / d;
#endif
  y = fma(fma(-d, y, 1.0), y, y);
  y = fma(fma(-d, y, 1.0), y, y);
  double s = f * y;
  s = fma(fma(-d, s, f), y, s);
  const double z = s * s;
  double q = 2.0 / 21.0;
  q = fma(q, z, 2.0 / 19.0);
  q = fma(q, z, 2.0 / 17.0);
  q = fma(q, z, 2.0 / 15.0);
  q = fma(q, z, 2.0 / 13.0);
  q = fma(q, z, 2.0 / 11.0);
  q = fma(q, z, 2.0 / 9.0);
  q = fma(q, z, 2.0 / 7.0);
  q = fma(q, z, 2.0 / 5.0);
  q = fma(q, z, 2.0 / 3.0);
  // 2 atanh(s) = 2 s + s z q; e ln2 with ln2 split (the high part has 11
  // trailing zero bits: e ln2_hi is exact for |e| < 2^11)
  const double ed = (double)e;
  const double lo = fma(ed, 1.90821492927058770002e-10, s * z * q);
  return fma(ed, 6.93147180369123816490e-01, fma(2.0, s, lo));
}

// Standard normal by inversion (R's own default, norm_rand INVERSION ->
// qnorm): Wichura's AS241 (PPND16) at p in (0, 1); the tail's log by
// log_unit (the oracle uses libm's: the normals agree to ~1e-16).
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
  r = sqrt(-log_unit(r));
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

}  // namespace nngp
