// fp64 VALU issue probe (diagnostic): cycles per wave64 v_fma_f64 with C independent chains per lane and W waves per
// SIMD (one workgroup of 4 W waves per CU, 256 workgroups), and the same for a Horner-shaped dependent chain.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/fma_probe tools/fma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int C>
__global__ void k_fma(double* out, double a, double b, int iters, unsigned long long* cyc) {
  double x[C];
#pragma unroll
  for (int c = 0; c < C; ++c) x[c] = threadIdx.x * 1e-3 + c;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int c = 0; c < C; ++c) x[c] = fma(x[c], a, b);
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

template <int C>
void run(int W, double* d, unsigned long long* dc) {
  const int iters = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_fma<C>, dim3(256), dim3(256 * W), 0, 0, d, 0.999, 1e-3, iters, dc);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_fma<C>, dim3(256), dim3(256 * W), 0, 0, d, 0.999, 1e-3, iters, dc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long cyc = 0;
  (void)hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
  const double per_wave_fma = (double)iters * 16 * C;
  const double flops = per_wave_fma * 64 * 2 * 4 * W * 256;
  printf("chains %2d waves/SIMD %d: %.4f ms  %.1f TF/s  cycles per FMA per SIMD %.2f  (wave 0: %.2f per own FMA)  clock %.2f GHz\n",
         C, W, ms, flops / ms / 1e9, (double)cyc / (per_wave_fma * W), (double)cyc / per_wave_fma,
         cyc / (ms * 1e6));
}

int main() {
  double* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, 256 * 1024 * 8 * 4);
  (void)hipMalloc(&dc, 8);
  for (int W = 1; W <= 4; W *= 2) {
    run<1>(W, d, dc);
    run<2>(W, d, dc);
    run<4>(W, d, dc);
    run<8>(W, d, dc);
  }
  return 0;
}
