// Issue-rate probe of the register-state chain term (TChainRot<2>): 32 v_mfma_f64_4x4x4_4b per "term" in 4
// accumulation chains with distinct A operands, alone / with the term's fp64 VALU work / with its DPP moves, one
// wave.  Cycles per term (s_memtime).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma4_mix tools/mfma4_mix.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ double mv(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u, CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// MODE 0: MFMAs only (B fixed); 1: + per-term recurrence VALU (dependent on D); 2: + DPP rotations of the new state
// (B operands depend on the previous term: the real chain)
template <int MODE>
__global__ void kterm(double* out, long long* cyc, const double* a, int terms) {
  double ar[16], ai[16];
  for (int x = 0; x < 16; ++x) {
    ar[x] = a[x * 64 + threadIdx.x];
    ai[x] = a[(16 + x) * 64 + threadIdx.x];
  }
  double y[2] = {a[threadIdx.x] * 1e-3, a[64 + threadIdx.x] * 1e-3}, ym2[2] = {0, 0}, acc[2] = {0, 0};
  double bv[2][4];
  for (int g = 0; g < 2; ++g) {
    bv[g][0] = y[g];
    bv[g][1] = mv<0x124>(y[g]);
    bv[g][2] = mv<0x128>(y[g]);
    bv[g][3] = mv<0x12C>(y[g]);
  }
  const int n = threadIdx.x & 3;
  long long t0 = clock64();
  for (int t = 0; t < terms; ++t) {
    double d0[2], d1[2];
#pragma unroll
    for (int gi = 0; gi < 2; ++gi)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int go = 0; go < 2; ++go) {
          const int x = (go * 2 + gi) * 4 + j;
          d0[go] = __builtin_amdgcn_mfma_f64_4x4x4f64(ar[x], bv[gi][j], gi || j ? d0[go] : 0.0, 0, 0, 0);
          d1[go] = __builtin_amdgcn_mfma_f64_4x4x4f64(ai[x], bv[gi][j], gi || j ? d1[go] : 0.0, 0, 0, 0);
        }
    if constexpr (MODE == 0) {
      acc[0] += d0[0] + d1[0];
      acc[1] += d0[1] + d1[1];
    } else {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const double o = mv<0xB1>(d1[g]);
        const double D = (n & 1) ? d0[g] + o : d0[g] - o;
        const double z = D + ym2[g];
        ym2[g] = y[g];
        acc[g] += 0.37 * z;
        y[g] = z * 1e-3;
        if constexpr (MODE == 2) {
          bv[g][0] = y[g];
          bv[g][1] = mv<0x124>(y[g]);
          bv[g][2] = mv<0x128>(y[g]);
          bv[g][3] = mv<0x12C>(y[g]);
        }
      }
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc[0] + acc[1] + y[0] + y[1];
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// G = 1 (zz): 8 MFMAs per term in 2 chains, the recurrence and the rotations of the new state
template <int MODE>
__global__ void kterm1(double* out, long long* cyc, const double* a, const double* cw, int terms) {
  double ar[4], ai[4];
  for (int x = 0; x < 4; ++x) {
    ar[x] = a[x * 64 + threadIdx.x];
    ai[x] = a[(16 + x) * 64 + threadIdx.x];
  }
  double y = a[threadIdx.x] * 1e-3, ym2 = 0, acc = 0;
  double bv[4] = {y, mv<0x124>(y), mv<0x128>(y), mv<0x12C>(y)};
  const int n = threadIdx.x & 3;
  __shared__ double cws[64];
  cws[threadIdx.x] = cw[threadIdx.x];
  __syncthreads();
  long long t0 = clock64();
  for (int t = 0; t < terms; ++t) {
    const double ct = MODE >= 3 ? cws[t & 63] : 0.37;
    double d0 = 0.0, d1 = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      d0 = __builtin_amdgcn_mfma_f64_4x4x4f64(ar[j], bv[j], d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f64_4x4x4f64(ai[j], bv[j], d1, 0, 0, 0);
    }
    const double o = mv<0xB1>(d1);
    const double D = (n & 1) ? d0 + o : d0 - o;
    const double z = D + ym2;
    ym2 = y;
    acc += ct * z;
    y = z * 1e-3;
    if constexpr (MODE >= 2) {
      bv[0] = y;
      bv[1] = mv<0x124>(y);
      bv[2] = mv<0x128>(y);
      bv[3] = mv<0x12C>(y);
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc + y;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  double *o, *a;
  long long* c;
  (void)hipMalloc(&o, 64 * 8);
  (void)hipMalloc(&a, 32 * 64 * 8);
  (void)hipMemset(a, 0, 32 * 64 * 8);
  (void)hipMalloc(&c, 8);
  long long h;
  const int terms = 4096;
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(kterm<0>, dim3(1), dim3(64), 0, 0, o, c, a, terms);
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("32 MFMA per term, 4 chains, B fixed:            %.1f cycles per term\n", (double)h / terms);
    hipLaunchKernelGGL(kterm<1>, dim3(1), dim3(64), 0, 0, o, c, a, terms);
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("  + recurrence VALU (B fixed):                  %.1f cycles per term\n", (double)h / terms);
    hipLaunchKernelGGL(kterm<2>, dim3(1), dim3(64), 0, 0, o, c, a, terms);
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("  + DPP rotations (B from the previous term):   %.1f cycles per term\n", (double)h / terms);
  }
  double* cwd;
  (void)hipMalloc(&cwd, 64 * 8);
  (void)hipMemset(cwd, 0, 64 * 8);
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(kterm1<1>, dim3(1), dim3(64), 0, 0, o, c, a, cwd, terms);
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("G=1: 8 MFMA + recurrence (B fixed):            %.1f cycles per term\n", (double)h / terms);
    hipLaunchKernelGGL(kterm1<2>, dim3(1), dim3(64), 0, 0, o, c, a, cwd, terms);
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("G=1:  + DPP rotations:                          %.1f cycles per term\n", (double)h / terms);
    hipLaunchKernelGGL(kterm1<3>, dim3(1), dim3(64), 0, 0, o, c, a, cwd, terms);
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("G=1:  + coefficient from LDS per term:          %.1f cycles per term\n", (double)h / terms);
  }
  return 0;
}
