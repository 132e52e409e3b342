// Microbenchmark (diagnostic): does data written by kernel A stay in the XCD
// L2 for kernel B on the same stream, and is a cross-XCD re-read ever stale?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NB = 256, PER = 4096;  // 256 blocks x 4096 doubles (32 KB) = 8 MB
__global__ void k_write(double* x, double v) {
  const size_t b = blockIdx.x;
  for (int i = threadIdx.x; i < PER; i += 256) x[b * PER + i] = v + i;
}
// block b reads region (b + shift) % NB; counts mismatches vs v
__global__ void k_read(const double* x, double v, int shift, int* bad, unsigned long long* cyc) {
  const size_t b = (blockIdx.x + shift) % NB;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int nb = 0;
  for (int i = threadIdx.x; i < PER; i += 256) nb += (x[b * PER + i] != v + i);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (nb) atomicAdd(bad, nb);
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
__global__ void k_xcc(int* id) {
  if (threadIdx.x == 0) {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    id[blockIdx.x] = v & 0xf;
  }
}

int main() {
  double* x; int* bad; unsigned long long* cyc; int* ids;
  CHK(hipMalloc(&x, sizeof(double) * NB * PER)); CHK(hipMalloc(&bad, 4)); CHK(hipMalloc(&cyc, 8 * NB));
  CHK(hipMalloc(&ids, 4 * NB));
  std::vector<int> hid(NB);
  hipLaunchKernelGGL(k_xcc, dim3(NB), dim3(64), 0, 0, ids);
  CHK(hipMemcpy(hid.data(), ids, 4 * NB, hipMemcpyDeviceToHost));
  printf("xcc of blocks 0..15:"); for (int i = 0; i < 16; ++i) printf(" %d", hid[i]); printf("\n");
  std::vector<unsigned long long> h(NB);
  auto med = [&](void) { std::vector<unsigned long long> v(h); std::sort(v.begin(), v.end()); return v[NB / 2]; };
  int hbad = 0;
  for (int it = 0; it < 6; ++it) {
    double v = 1000.0 * (it + 1);
    hipLaunchKernelGGL(k_write, dim3(NB), dim3(256), 0, 0, x, v);
    for (int shift : {0, 8, 1, 0}) {
      CHK(hipMemset(bad, 0, 4));
      hipLaunchKernelGGL(k_read, dim3(NB), dim3(256), 0, 0, x, v, shift, bad, cyc);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(h.data(), cyc, 8 * NB, hipMemcpyDeviceToHost));
      CHK(hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost));
      if (it >= 4) printf("iter %d read shift %d (same XCD if shift %% 8 == 0): median %llu cyc, stale %d\n", it, shift, med(), hbad);
    }
  }
  return 0;
}
