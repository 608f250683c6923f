// Microbenchmark of ExpmRR::rmul (the register-resident GEMM step of k_expm_rr): cycles per GEMM.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/rmul_bench tools/rmul_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_expm_rr.hpp"
using namespace qoc;
__device__ unsigned long long g_cyc[4];

template <int NT, int MODE>
__global__ __launch_bounds__(64 * NT, 2) void k_rmul(int N, int iters, double* out) {
  using M = MF<double>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using E = ExpmRR<double, NT>;
  double* Br = (double*)smem;
  double* Bi = Br + E::plane(N);
  for (int e = threadIdx.x; e < E::plane(N); e += blockDim.x) {
    const int r = e / E::ldp(N), c = e % E::ldp(N);
    Br[e] = (r < N && c < N) ? 0.01 * ((e * 7) % 13) / N : 0.0;
    Bi[e] = (r < N && c < N) ? 0.01 * ((e * 5) % 11) / N : 0.0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, row = 16 * wave + (lane & 15);
  typename E::Own V, Z;
  E::zero(Z);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = 16 * t + M::drow(lane, e);
      V.r[t][e] = (row < N && col < N) ? (row == col ? 1.0 : 0.001) : 0.0;
      V.i[t][e] = 0.0;
    }
  unsigned long long t0, t1;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  for (int it = 0; it < iters; ++it) E::template rmul<10>(N, V, Br, Bi, V, Z, lane);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  if (threadIdx.x == 0 && blockIdx.x == 0) g_cyc[MODE] = t1 - t0;
  double s = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) s += V.r[t][0] + V.i[t][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 1 << 24);
  const int N = 40, it = 200;
  const size_t lds = ExpmRR<double, 3>::lds_bytes(N);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  int grids[] = {1, 256, 512, 768};
  for (int g : grids) {
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL((k_rmul<3, 0>), dim3(g), dim3(192), lds, 0, N, it, d);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      (void)hipEventElapsedTime(&ms, a, b);
    }
    unsigned long long c[4];
    (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(g_cyc), sizeof(c));
    const double mfma_cyc = 10.0 * 9 * 64;  // ksteps x MFMAs x cycles
    printf("N=%d grid %d: %.0f cycles/GEMM (wave 0 of block 0), MFMA-bound %.0f; wall %.3f ms -> %.0f cycles/GEMM/CU-slot\n", N, g,
           (double)c[0] / it, mfma_cyc, ms, ms * 1e-3 * 2.388e9 / it / ((g + 255) / 256.0));
  }
  return 0;
}
