// CPU check of nngp::log_unit (device_common.h, the AS241 tail's log of the
// sweep's normals): max ulp distance to libm's log over the uniforms the
// sweep draws and their powers-of-two scalings.  Test infrastructure
// (tests/test_capi_and_graph.py builds and runs it with hipcc, host only).
#include "device_common.h"
#include <cstdio>
#include <cstring>
#include <random>
static long long ulp(double a, double b) {
  long long x, y;
  std::memcpy(&x, &a, 8);
  std::memcpy(&y, &b, 8);
  return x > y ? x - y : y - x;
}
int main() {
  std::mt19937_64 g(1);
  long long worst = 0;
  double wx = 0;
  for (int i = 0; i < 4000000; ++i) {
    const double u = std::ldexp((double)(g() >> 11) + 0.5, -53);
    const double x = (i & 1) ? u : std::ldexp(u, -(int)(g() % 60));
    const long long d = ulp(nngp::log_unit(x), std::log(x));
    if (d > worst) { worst = d; wx = x; }
  }
  const double edge[] = {1.0, 0.5, 0.70710678118654752440, 0.7071067811865475, 0x1.0p-53, 1e-300, 0.075, 0.925};
  for (double x : edge) {
    const long long d = ulp(nngp::log_unit(x), std::log(x));
    if (d > worst) { worst = d; wx = x; }
  }
  std::printf("max_ulp %lld at %.17g\n", worst, wx);
  return worst <= 2 ? 0 : 1;
}
