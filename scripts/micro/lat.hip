// Microbenchmarks (diagnostic, not part of the product): latencies seen by one
// wavefront on an otherwise idle MI355X.  Prints cycles (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
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
__device__ double normal_at(uint64_t seed, uint64_t sweep, uint32_t loc) {
  uint32_t c[4] = {loc, (uint32_t)sweep, (uint32_t)(sweep >> 32), 0x5EEDu};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  uint64_t a = ((((uint64_t)c[1]) << 32) | c[0]) >> 11, b = ((((uint64_t)c[3]) << 32) | c[2]) >> 11;
  double u1 = ((double)a + 0.5) * 0x1.0p-53, u2 = (double)b * 0x1.0p-53;
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586476925286766559 * u2);
}

struct Args { const int* chase; const double* arr; const int* idx; double* out; unsigned long long* t; int hops; };

__global__ void k_chase(Args a) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int p = threadIdx.x;
  for (int h = 0; h < a.hops; ++h) p = a.chase[p];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { a.t[0] = t1 - t0; a.out[0] = p; }
}

// 16 independent gathers per lane (random indices), then 16 coalesced loads
__global__ void k_gather(Args a) {
  const int l = threadIdx.x;
  int ix[16];
  for (int j = 0; j < 16; ++j) ix[j] = a.idx[j * 64 + l];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double s = 0;
  double v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = a.arr[ix[j]];
#pragma unroll
  for (int j = 0; j < 16; ++j) s += v[j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = a.arr[(size_t)(blockIdx.x + 1) * 4096 * 64 + j * 64 + l];
#pragma unroll
  for (int j = 0; j < 16; ++j) s += v[j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  a.out[l] = s;
  if (l == 0) { a.t[0] = t1 - t0; a.t[1] = t2 - t1; }
}

__global__ void k_normal(Args a) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double z = normal_at(12345, threadIdx.x, threadIdx.x * 7 + a.hops);
  double z2 = normal_at(12345, threadIdx.x + 1, threadIdx.x * 7 + a.hops);
  asm volatile("" :: "v"(z), "v"(z2));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double q = 1.0 / (z + 3.0) + sqrt(z2 + 5.0);
  asm volatile("" :: "v"(q));
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  a.out[threadIdx.x] = z + z2 + q;
  if (threadIdx.x == 0) { a.t[0] = t1 - t0; a.t[1] = t2 - t1; }
}

// time from kernel entry to the first kernarg-dependent global load landing
__global__ void k_kernarg(Args a) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  asm volatile("" ::: "memory");
  double x = a.arr[threadIdx.x];
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  a.out[threadIdx.x] = x;
  if (threadIdx.x == 0) { a.t[0] = t1 - t0; }
}

int main() {
  const size_t N = 1 << 24;  // 16M doubles = 128 MB
  std::mt19937 g(1);
  std::vector<int> chase(N), idx(64 * 16);
  // random cyclic permutation for the chase (within 32 MB of ints)
  std::vector<int> perm(N);
  for (size_t i = 0; i < N; ++i) perm[i] = (int)i;
  std::shuffle(perm.begin(), perm.end(), g);
  for (size_t i = 0; i < N; ++i) chase[perm[i]] = perm[(i + 1) % N];
  for (auto& x : idx) x = g() % N;
  int *dchase, *didx; double *darr, *dout; unsigned long long* dt;
  CHK(hipMalloc(&dchase, N * 4)); CHK(hipMalloc(&didx, idx.size() * 4));
  CHK(hipMalloc(&darr, N * 8)); CHK(hipMalloc(&dout, 4096 * 8)); CHK(hipMalloc(&dt, 64));
  CHK(hipMemcpy(dchase, chase.data(), N * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(didx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemset(darr, 0, N * 8));
  Args a{dchase, darr, didx, dout, dt, 64};
  unsigned long long t[8];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, a);
    CHK(hipDeviceSynchronize()); CHK(hipMemcpy(t, dt, 16, hipMemcpyDeviceToHost));
    printf("chase (HBM/MALL random, 64 hops): %.0f cyc/hop\n", (double)t[0] / 64);
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_gather, dim3(1), dim3(64), 0, 0, a);
    CHK(hipDeviceSynchronize()); CHK(hipMemcpy(t, dt, 16, hipMemcpyDeviceToHost));
    printf("one wave: 16 random gathers/lane %llu cyc; 16 coalesced rows %llu cyc\n", t[0], t[1]);
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_normal, dim3(1), dim3(64), 0, 0, a);
    CHK(hipDeviceSynchronize()); CHK(hipMemcpy(t, dt, 16, hipMemcpyDeviceToHost));
    printf("two fp64 Box-Muller normals %llu cyc; div+sqrt %llu cyc\n", t[0], t[1]);
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_kernarg, dim3(1), dim3(64), 0, 0, a);
    CHK(hipDeviceSynchronize()); CHK(hipMemcpy(t, dt, 16, hipMemcpyDeviceToHost));
    printf("kernel entry -> kernarg-addressed load landed: %llu cyc\n", t[0]);
  }
  // clock calibration: memtime vs memrealtime
  return 0;
}
