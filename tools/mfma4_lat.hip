// Dependent-latency probe of v_mfma_f64_4x4x4_4b_f64 (the Taylor-action chains' matvec instruction): 2048 MFMAs
// in NCH interleaved accumulation chains, one wave; cycles per instruction vs NCH.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma4_lat tools/mfma4_lat.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NCH>
__global__ void kc(double* out, long long* cyc, double a, double b) {
  double acc[NCH];
  for (int i = 0; i < NCH; ++i) acc[i] = 0;
  long long t0 = clock64();
  for (int it = 0; it < 2048 / NCH; ++it)
#pragma unroll
    for (int i = 0; i < NCH; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < NCH; ++i) s += acc[i];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// LDS round trip of the chain's term exchange: write one double per lane, wait, barrier, read it back (3 waves)
__global__ void klds(double* out, long long* cyc, int iters) {
  __shared__ double buf[2][4 * 64 * 4];
  double v = threadIdx.x;
  __syncthreads();
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    buf[it & 1][threadIdx.x * 4] = v;
    __syncthreads();
    v += buf[it & 1][((threadIdx.x + 64) % blockDim.x) * 4];
  }
  long long t1 = clock64();
  out[threadIdx.x] = v;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  double* o;
  long long* c;
  (void)hipMalloc(&o, 256 * 8);
  (void)hipMalloc(&c, 8);
  long long h;
  for (int r = 0; r < 2; ++r) {
#define RUN(N)                                                                              \
    hipLaunchKernelGGL(kc<N>, dim3(1), dim3(64), 0, 0, o, c, 1.0, 1e-3);                    \
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);                                       \
    printf("4x4x4_4b f64, %d chains: %.1f cycles per instruction\n", N, (double)h / 2048);
    RUN(1) RUN(2) RUN(3) RUN(4) RUN(8)
    for (int w : {1, 3, 4}) {
      hipLaunchKernelGGL(klds, dim3(1), dim3(64 * w), 0, 0, o, c, 1024);
      (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
      printf("LDS write + barrier + read, %d waves: %.1f cycles per round\n", w, (double)h / 1024);
    }
  }
  return 0;
}
