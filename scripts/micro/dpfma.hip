// fp64 VALU issue rate on gfx950 (diagnostic for the factor kernel): cycles
// per v_fma_f64 of one wave (A independent accumulators) at 1 or 2 waves per
// SIMD, and the same for v_fma_f32.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

template <int A, class T>
__global__ __launch_bounds__(64) void chains(T* out, int iters, unsigned long long* cyc) {
  T acc[A];
  for (int a = 0; a < A; ++a) acc[a] = (T)(threadIdx.x + a);
  const T m = (T)0.999999, c = (T)1e-7;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int a = 0; a < A; ++a) acc[a] = __builtin_fma(acc[a], m, c);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  T s = 0;
  for (int a = 0; a < A; ++a) s += acc[a];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int A, class T>
void run(const char* name, int blocks, int iters) {
  T* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(T) * blocks * 64);
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks);
  hipLaunchKernelGGL((chains<A, T>), dim3(blocks), dim3(64), 0, 0, out, 10, cyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((chains<A, T>), dim3(blocks), dim3(64), 0, 0, out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[8];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  const double ninst = (double)iters * 16 * A;
  // s_memtime ticks at the shader clock on gfx950 (MI355X guide)
  printf("%-8s A=%2d blocks=%5d  %.3f ms  wave cycles/inst %.2f  (chip: %.2f ns/inst/wave)\n", name, A, blocks, ms,
         h[0] / ninst, ms * 1e6 / ninst);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  const int it = 4000;
  for (int blocks : {1024, 2048, 4096}) {
    run<1, double>("f64", blocks, it);
    run<8, double>("f64", blocks, it);
    run<16, double>("f64", blocks, it);
    run<8, float>("f32", blocks, it);
  }
  return 0;
}
