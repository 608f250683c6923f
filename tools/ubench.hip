// Microbenchmarks of the instruction costs the GRAPE kernels depend on (gfx950, s_memtime cycles).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ unsigned long long g_t[16];
#define STAMP(v) do { __builtin_amdgcn_sched_barrier(0); asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); __builtin_amdgcn_sched_barrier(0);} while(0)

__global__ void k_mfma(double* out, int iters) {
  d4 a0 = {0,0,0,0}, a1 = a0, a2 = a0, a3 = a0;
  double x = threadIdx.x * 1e-3, y = 1.0 + threadIdx.x * 1e-4;
  unsigned long long t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a3, 0, 0, 0);
  }
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[0] = t1 - t0;
  out[threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3];
}
__global__ void k_mfma_dep(double* out, int iters) {
  d4 a0 = {0,0,0,0};
  double x = threadIdx.x * 1e-3, y = 1.0 + threadIdx.x * 1e-4;
  unsigned long long t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i) a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[1] = t1 - t0;
  out[threadIdx.x] = a0[0];
}
__global__ void k_fma(double* out, int iters) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const double m = 0.999999, c = 1e-7;
  unsigned long long t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i) {
    a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
    a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
  }
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[2] = t1 - t0;
  out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ void k_lds(double* out, int iters) {
  __shared__ double s[1024];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  int idx = threadIdx.x;
  double acc = 0;
  unsigned long long t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i) {  // dependent LDS chain
    double v = s[idx & 1023];
    acc += v;
    idx = (int)v + 1;
  }
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[3] = t1 - t0;
  out[threadIdx.x] = acc;
}
__global__ void k_bar(double* out, int iters) {
  unsigned long long t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i) __syncthreads();
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[4] = t1 - t0;
}
__global__ void k_div(double* out, int iters) {
  double a = 1.0 + threadIdx.x;
  unsigned long long t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i) a = 1.0 / (a + 1.0);
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[5] = t1 - t0;
  out[threadIdx.x] = a;
}

__global__ void k_mfma_valu(double* out, int iters, int nf) {
  d4 a0 = {0,0,0,0}, a1 = a0, a2 = a0, a3 = a0;
  double x = threadIdx.x * 1e-3, y = 1.0 + threadIdx.x * 1e-4;
  double b0 = threadIdx.x, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3, b4 = b0 + 4, b5 = b0 + 5, b6 = b0 + 6, b7 = b0 + 7;
  const double m = 0.999999, c = 1e-7;
  unsigned long long t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
    b0 = fma(b0, m, c); b1 = fma(b1, m, c); b2 = fma(b2, m, c); b3 = fma(b3, m, c);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a1, 0, 0, 0);
    b4 = fma(b4, m, c); b5 = fma(b5, m, c); b6 = fma(b6, m, c); b7 = fma(b7, m, c);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a2, 0, 0, 0);
    b0 = fma(b0, m, c); b1 = fma(b1, m, c); b2 = fma(b2, m, c); b3 = fma(b3, m, c);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a3, 0, 0, 0);
    b4 = fma(b4, m, c); b5 = fma(b5, m, c); b6 = fma(b6, m, c); b7 = fma(b7, m, c);
  }
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[6] = t1 - t0;
  out[threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3] + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7;
}
__global__ void k_mfma_multi(double* out, int iters, int slot) {
  d4 a0 = {0,0,0,0}, a1 = a0, a2 = a0, a3 = a0;
  double x = threadIdx.x * 1e-3, y = 1.0 + threadIdx.x * 1e-4;
  unsigned long long t0, t1;
  __syncthreads();
  STAMP(t0);
  for (int i = 0; i < iters; ++i) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a3, 0, 0, 0);
  }
  __syncthreads();
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[slot] = t1 - t0;
  out[threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3];
}
__global__ void k_mfma44(double* out, int iters) {
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  double x = threadIdx.x * 1e-3, y = 1.0 + threadIdx.x * 1e-4;
  unsigned long long t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i) {
    a0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, a3, 0, 0, 0);
  }
  STAMP(t1);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_t[10] = t1 - t0;
  out[threadIdx.x] = a0 + a1 + a2 + a3;
}
__global__ void k_rt(double* out) {
  unsigned long long t0, t1, r0, r1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r0)::"memory");
  STAMP(t0);
  double a = threadIdx.x;
  for (int i = 0; i < 200000; ++i) a = fma(a, 0.9999, 1e-7);
  STAMP(t1);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
  if (threadIdx.x == 0) { g_t[11] = t1 - t0; g_t[12] = r1 - r0; }
  out[threadIdx.x] = a;
}
int main() {
  double* d; (void)hipMalloc(&d, 1 << 20);
  const int it = 1000;
  hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, d, it);
  hipLaunchKernelGGL(k_mfma_dep, dim3(1), dim3(64), 0, 0, d, it);
  hipLaunchKernelGGL(k_fma, dim3(1), dim3(64), 0, 0, d, it);
  hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, d, it);
  hipLaunchKernelGGL(k_bar, dim3(1), dim3(256), 0, 0, d, it);
  hipLaunchKernelGGL(k_div, dim3(1), dim3(64), 0, 0, d, it);
  (void)hipDeviceSynchronize();
  unsigned long long t[16]; (void)hipMemcpyFromSymbol(t, HIP_SYMBOL(g_t), sizeof(t));
  printf("mfma_f64_16x16x4 independent x4: %.1f cycles/instr\n", t[0] / (4.0 * it));
  printf("mfma_f64_16x16x4 dependent:      %.1f cycles/instr\n", t[1] / (1.0 * it));
  printf("v_fma_f64 independent x8 (1 wave): %.1f cycles/instr\n", t[2] / (8.0 * it));
  printf("ds_read_b64 dependent chain:     %.1f cycles/iter\n", t[3] / (1.0 * it));
  printf("__syncthreads (4 waves):         %.1f cycles\n", t[4] / (1.0 * it));
  printf("f64 reciprocal dependent chain:  %.1f cycles/iter\n", t[5] / (1.0 * it));
  hipLaunchKernelGGL(k_mfma_valu, dim3(1), dim3(64), 0, 0, d, it, 0);
  hipLaunchKernelGGL(k_mfma_multi, dim3(1), dim3(256), 0, 0, d, it, 7);
  hipLaunchKernelGGL(k_mfma_multi, dim3(1), dim3(512), 0, 0, d, it, 8);
  hipLaunchKernelGGL(k_mfma_multi, dim3(1), dim3(1024), 0, 0, d, it, 9);
  hipLaunchKernelGGL(k_mfma44, dim3(1), dim3(64), 0, 0, d, it);
  hipLaunchKernelGGL(k_rt, dim3(1), dim3(64), 0, 0, d);
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(t, HIP_SYMBOL(g_t), sizeof(t));
  printf("mfma x4 + 16 v_fma_f64 interleaved (1 wave): %.1f cycles/iter (mfma-only x4 = %.1f)\n", t[6] / (1.0 * it), t[0] / (1.0 * it));
  printf("mfma x4, 4 waves: %.1f cycles/iter; 8 waves %.1f; 16 waves %.1f\n", t[7] / (1.0 * it), t[8] / (1.0 * it), t[9] / (1.0 * it));
  printf("mfma_f64_4x4x4 independent x4: %.1f cycles/instr\n", t[10] / (4.0 * it));
  printf("memtime vs realtime: %llu memtime ticks, %llu realtime (100MHz) ticks -> %.3f GHz\n", t[11], t[12], t[11] / (t[12] * 0.01) / 1e3);
  return 0;
}
