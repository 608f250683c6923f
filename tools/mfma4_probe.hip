// Issue-rate probe: v_mfma_f64_16x16x4_f64 vs v_mfma_f64_4x4x4_4b_f64 (independent accumulators).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma4_probe tools/mfma4_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ void k16(double* out, long long* cyc, double a, double b) {
  v4d acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = v4d{0, 0, 0, 0};
  long long t0 = clock64();
  for (int it = 0; it < 256; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k4(double* out, long long* cyc, double a, double b) {
  double acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = 0;
  long long t0 = clock64();
  for (int it = 0; it < 256; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
  double* o;
  long long* c;
  (void)hipMalloc(&o, 64 * 8);
  (void)hipMalloc(&c, 8);
  long long h;
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, o, c, 1.0, 1e-3);
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("16x16x4 f64: %.1f cycles per instruction (2048 in flight groups of 8)\n", (double)h / 2048);
    hipLaunchKernelGGL(k4, dim3(1), dim3(64), 0, 0, o, c, 1.0, 1e-3);
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("4x4x4_4b f64: %.1f cycles per instruction\n", (double)h / 2048);
  }
  return 0;
}
