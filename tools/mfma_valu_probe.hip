// Does the fp64 matrix pipe run beside the fp64 VALU?  (diagnostic)  Kernel time of a loop body with NV independent
// v_fma_f64 chains only, NM independent v_mfma_f64_4x4x4_4b accumulators only, and both, at W waves per SIMD over
// 256 workgroups.  If both ≈ max(alone), the pipes overlap; if both ≈ sum, they share the issue or the datapath.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mfma_valu_probe tools/mfma_valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NV, int NM>
__global__ void k_mix(double* out, double a, double b, int iters) {
  double x[NV > 0 ? NV : 1], acc[NM > 0 ? NM : 1];
#pragma unroll
  for (int c = 0; c < NV; ++c) x[c] = threadIdx.x * 1e-3 + c;
#pragma unroll
  for (int c = 0; c < NM; ++c) acc[c] = 0.0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int c = 0; c < NM; ++c) acc[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[c], 0, 0, 0);
#pragma unroll
      for (int c = 0; c < NV; ++c) x[c] = fma(x[c], a, b);
    }
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < NV; ++c) s += x[c];
#pragma unroll
  for (int c = 0; c < NM; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NV, int NM>
float run(int W, double* d, const char* tag) {
  const int iters = 512;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k_mix<NV, NM>), dim3(256), dim3(256 * W), 0, 0, d, 0.999, 1e-3, iters);
  float best = 1e9;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_mix<NV, NM>), dim3(256), dim3(256 * W), 0, 0, d, 0.999, 1e-3, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  const double vflop = (double)iters * 4 * NV * 64 * 2, mflop = (double)iters * 4 * NM * 512;
  const double flops = (vflop + mflop) * 4 * W * 256;
  printf("W=%d %-6s NV=%2d NM=%2d: %.4f ms  %.1f TF/s\n", W, tag, NV, NM, best, flops / best / 1e9);
  return best;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 256 * 1024 * 8);
  for (int W = 1; W <= 2; ++W) {
    run<8, 0>(W, d, "valu");
    run<0, 2>(W, d, "mfma");
    run<8, 2>(W, d, "both");
    run<16, 0>(W, d, "valu");
    run<0, 4>(W, d, "mfma");
    run<16, 4>(W, d, "both");
    run<8, 4>(W, d, "both");
  }
  return 0;
}
