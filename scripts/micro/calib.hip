// PMC calibration (diagnostic): known-byte kernels with the sweep kernel's
// access widths; compare rocprofv3 FETCH_SIZE / WRITE_SIZE with the bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
constexpr size_t N = (size_t)512 << 20;  // bytes per buffer (beyond the 256 MiB Infinity Cache)
__global__ void rd8(const double* a, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  if (s == 1.2345) out[0] = s;
}
__global__ void rd4(const int* a, size_t n, int* out) {
  int s = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  if (s == 12345) out[0] = s;
}
__global__ void rd2(const unsigned short* a, size_t n, int* out) {
  int s = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  if (s == 12345) out[0] = s;
}
__global__ void wr8(double* a, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = (double)i;
}
int main() {
  char *a, *b; double* o;
  CHK(hipMalloc(&a, N)); CHK(hipMalloc(&b, N)); CHK(hipMalloc(&o, 64));
  CHK(hipMemset(a, 1, N)); CHK(hipMemset(b, 1, N));
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(rd8, dim3(4096), dim3(256), 0, 0, (const double*)a, N / 8, o);
    hipLaunchKernelGGL(rd4, dim3(4096), dim3(256), 0, 0, (const int*)b, N / 4, (int*)o);
    hipLaunchKernelGGL(rd2, dim3(4096), dim3(256), 0, 0, (const unsigned short*)a, N / 2, (int*)o);
    hipLaunchKernelGGL(wr8, dim3(4096), dim3(256), 0, 0, (double*)b, N / 8);
  }
  CHK(hipDeviceSynchronize());
  printf("calibration kernels: each moves %zu bytes\n", N);
  return 0;
}
