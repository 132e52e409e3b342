// Accuracy of the factor kernel's device math on gfx950, in ulp against the
// host's libm: hardware rsq + Newton sqrt variants, the Taylor exp and a
// 64-entry-table exp for non-positive arguments.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

__device__ double sqrt2c(double s) {  // rsq + two residual corrections
  const double y = __builtin_amdgcn_rsq(s);
  double g = s * y;
  const double h = 0.5 * y;
  double e = __builtin_fma(-g, g, s);
  g = __builtin_fma(e, h, g);
  e = __builtin_fma(-g, g, s);
  return __builtin_fma(e, h, g);
}
__device__ double sqrt1c(double s) {
  const double y = __builtin_amdgcn_rsq(s);
  const double g = s * y;
  const double e = __builtin_fma(-g, g, s);
  return __builtin_fma(e, 0.5 * y, g);
}
__device__ double rsq_raw(double s) { return __builtin_amdgcn_rsq(s); }

__device__ double exp_taylor(double x) {
  const double k = __builtin_rint(x * 1.4426950408889634);
  double r = __builtin_fma(-k, 6.93147180559945286227e-01, x);
  r = __builtin_fma(-k, 2.31904681384629955842e-17, r);
  double p = 1.6059043836821614599e-10;
  p = __builtin_fma(p, r, 2.0876756987868098979e-09);
  p = __builtin_fma(p, r, 2.5052108385441718775e-08);
  p = __builtin_fma(p, r, 2.7557319223985890653e-07);
  p = __builtin_fma(p, r, 2.7557319223985890653e-06);
  p = __builtin_fma(p, r, 2.4801587301587301566e-05);
  p = __builtin_fma(p, r, 1.9841269841269841253e-04);
  p = __builtin_fma(p, r, 1.3888888888888889419e-03);
  p = __builtin_fma(p, r, 8.3333333333333332177e-03);
  p = __builtin_fma(p, r, 4.1666666666666664354e-02);
  p = __builtin_fma(p, r, 1.6666666666666665741e-01);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_ldexp(p, (int)k);
}

// exp(x) = 2^(k/64) e^r: k = rint(64 x / ln2), |r| <= ln2/128
__device__ double exp_table(double x, const double* __restrict__ tab) {
  const double k = __builtin_rint(x * 92.332482616893656);  // 64/ln2
  double r = __builtin_fma(-k, 1.0830424696249145e-02, x);   // ln2/64 hi
  r = __builtin_fma(-k, 3.6235106472610935e-19, r);          // ln2/64 lo
  const int ki = (int)k;
  double p = 1.3888888888888889e-03;  // 1/720 (degree 6)
  p = __builtin_fma(p, r, 8.3333333333333332e-03);
  p = __builtin_fma(p, r, 4.1666666666666664e-02);
  p = __builtin_fma(p, r, 1.6666666666666666e-01);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  const double t = tab[ki & 63];
  p = __builtin_fma(p * r, t, t);
  return __builtin_ldexp(p, ki >> 6);
}

__global__ void run(int n, const double* in, const double* xin, const double* tab, double* o) {
  __shared__ double st[64];
  if (threadIdx.x < 64) st[threadIdx.x] = tab[threadIdx.x];
  __syncthreads();
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o[0 * n + i] = sqrt2c(in[i]);
  o[1 * n + i] = sqrt1c(in[i]);
  o[2 * n + i] = rsq_raw(in[i]);
  o[3 * n + i] = exp_taylor(xin[i]);
  o[4 * n + i] = exp_table(xin[i], st);
}

static double ulp_err(double got, double ref) {
  if (got == ref) return 0.0;
  if (!std::isfinite(got)) return 1e300;
  double u = std::nextafter(std::fabs(ref), INFINITY) - std::fabs(ref);
  if (ref == 0.0) u = 4.9e-324;
  return std::fabs(got - ref) / u;
}

int main() {
  const int n = 1 << 22;
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> U(0, 1);
  std::vector<double> s(n), x(n), tab(64), o(5 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    s[i] = std::pow(10.0, -300 + 600 * U(g));            // any normal positive
    x[i] = i % 2 ? -40.0 * U(g) : -std::pow(10.0, -8 + 10.5 * U(g));  // [-3e2, 0)
    if (x[i] < -744) x[i] = -744;
  }
  for (int j = 0; j < 64; ++j) tab[j] = std::exp2(j / 64.0);
  double *ds, *dx, *dt, *dout;
  hipMalloc(&ds, n * 8); hipMalloc(&dx, n * 8); hipMalloc(&dt, 64 * 8); hipMalloc(&dout, 5 * (size_t)n * 8);
  hipMemcpy(ds, s.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dt, tab.data(), 64 * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(run, dim3((n + 255) / 256), dim3(256), 0, 0, n, ds, dx, dt, dout);
  hipMemcpy(o.data(), dout, 5 * (size_t)n * 8, hipMemcpyDeviceToHost);
  const char* names[5] = {"sqrt rsq+2 corrections", "sqrt rsq+1 correction", "rsq raw (vs 1/sqrt)",
                          "exp Taylor-13", "exp table-64 deg6"};
  for (int v = 0; v < 5; ++v) {
    double mx = 0, sum = 0;
    for (int i = 0; i < n; ++i) {
      double ref = v < 2 ? std::sqrt(s[i]) : v == 2 ? 1.0 / std::sqrt(s[i]) : std::exp(x[i]);
      double e = ulp_err(o[(size_t)v * n + i], ref);
      mx = std::max(mx, e);
      sum += e;
    }
    std::printf("%-26s max %.3g ulp  mean %.3g ulp\n", names[v], mx, sum / n);
  }
  return 0;
}
