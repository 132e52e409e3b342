// Microbenchmark (diagnostic): cost of fp64 normal generators on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1; c[3] = (uint32_t)p0; c[0] = n0; c[2] = n2;
  }
}
__device__ __forceinline__ void uniforms(uint32_t loc, double& u1, double& u2) {
  uint32_t c[4] = {loc, 7u, 0u, 0x5EEDu};
  philox(c, 12345u, 0u);
  uint64_t a = ((((uint64_t)c[1]) << 32) | c[0]) >> 11, b = ((((uint64_t)c[3]) << 32) | c[2]) >> 11;
  u1 = ((double)a + 0.5) * 0x1.0p-53; u2 = (double)b * 0x1.0p-53;
}
// Wichura AS241 PPND16
__device__ __forceinline__ double qnorm_as241(double p) {
  double q = p - 0.5, r, val;
  if (fabs(q) <= 0.425) {
    r = 0.180625 - q * q;
    val = q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r +
                   45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
                 133.14166789178437745) * r + 3.387132872796366608) /
          (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r +
                21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
            42.313330701600911252) * r + 1.);
    return val;
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

template <int M>
__global__ void k_lat(double* out, unsigned long long* t, int salt) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double u1, u2;
  uniforms(threadIdx.x * 977 + salt, u1, u2);
  asm volatile("" :: "v"(u1), "v"(u2));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double z;
  if (M == 0) z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  else if (M == 1) z = log(u1);
  else if (M == 2) z = cos(6.283185307179586 * u2);
  else if (M == 3) z = qnorm_as241(u1);
  else { double s, c; sincos(6.283185307179586 * u2, &s, &c); z = sqrt(-2.0 * log(u1)) * (c + s); }
  asm volatile("" :: "v"(z));
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = z;
  if (threadIdx.x == 0) { t[0] = t1 - t0; t[1] = t2 - t1; }
}

template <int M>
__global__ void k_bulk(double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double u1, u2;
  uniforms(i, u1, u2);
  double z;
  if (M == 0) z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  else if (M == 3) z = qnorm_as241(u1);
  else z = u1 + u2;  // philox only
  out[i] = z;
}

int main() {
  double* d; unsigned long long* t; CHK(hipMalloc(&d, sizeof(double) * 10000000)); CHK(hipMalloc(&t, 16));
  unsigned long long h[2];
  const char* names[] = {"box-muller", "log", "cos", "as241", "box-muller sincos"};
#define LAT(M) for (int r = 0; r < 3; ++r) { hipLaunchKernelGGL(k_lat<M>, dim3(1), dim3(64), 0, 0, d, t, r); CHK(hipDeviceSynchronize()); CHK(hipMemcpy(h, t, 16, hipMemcpyDeviceToHost)); if (r == 2) printf("%-18s philox %llu cyc, transform %llu cyc (one wave)\n", names[M], h[0], h[1]); }
  LAT(0) LAT(1) LAT(2) LAT(3) LAT(4)
  hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  const int n = 10000000;
#define BULK(M, name) for (int r = 0; r < 3; ++r) { CHK(hipEventRecord(a)); hipLaunchKernelGGL(k_bulk<M>, dim3((n + 255) / 256), dim3(256), 0, 0, d, n); CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b)); float ms; CHK(hipEventElapsedTime(&ms, a, b)); if (r == 2) printf("bulk %-12s 1e7 normals %.1f us\n", name, ms * 1e3); }
  BULK(0, "box-muller") BULK(3, "as241") BULK(9, "philox-only")
  return 0;
}
