// qoc_common.hpp — device helpers shared by the GRAPE kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qoc {

constexpr int WAVE = 64;
// executed-terms counter: partial sums in TERM_SLOTS words (workgroup b adds to word b % TERM_SLOTS), summed by
// qoc_chain_terms -- one shared word serialised thousands of atomics per launch on one L2 address
constexpr int TERM_SLOTS = 256;

template <typename T>
struct alignas(2 * sizeof(T)) cx {
  T r, i;
};

template <typename T>
__device__ __forceinline__ cx<T> cmul(cx<T> a, cx<T> b) {
  return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r};
}
// a + b*c
template <typename T>
__device__ __forceinline__ cx<T> cfma(cx<T> a, cx<T> b, cx<T> c) {
  return {a.r + b.r * c.r - b.i * c.i, a.i + b.r * c.i + b.i * c.r};
}
// a + conj(b)*c
template <typename T>
__device__ __forceinline__ cx<T> cfmaconj(cx<T> a, cx<T> b, cx<T> c) {
  return {a.r + b.r * c.r + b.i * c.i, a.i + b.r * c.i - b.i * c.r};
}
template <typename T>
__device__ __forceinline__ cx<T> cinv(cx<T> d) {
  T s = T(1) / (d.r * d.r + d.i * d.i);
  return {d.r * s, -d.i * s};
}

// ---------------------------------------------------------------------------
// MFMA wrappers.  A operand: lane l holds A[l&15][k=l>>4]; B operand: B[k=l>>4][l&15].
// D layout differs by dtype (cdna_hip_programming.md §3):
//   f64 16x16x4: reg i -> row (l>>4) + 4 i, col l&15
//   f32 16x16x4: reg i -> row 4 (l>>4) + i, col l&15
// ---------------------------------------------------------------------------
template <typename T>
struct MF;

template <>
struct MF<double> {
  typedef double v4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ v4 mma(double a, double b, v4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int drow(int lane, int i) { return (lane >> 4) + 4 * i; }
  // v_mfma_f64_4x4x4_4b (16 cycles, the same FMA rate as 16x16x4): block b = (l >> 2) & 3; A[m][k] at lane
  // m + 4b + 16k, B[k][n] at n + 4b + 16k, D[m][n] at n + 4b + 16m (measured, tools/mfma4_layout.hip).  With
  // the blocks side by side along n, B is the 16x16x4 B fragment and D is one register (m-quad) of the
  // 16x16x4 D layout; A carries rows 4q + (l & 3) of that quad.
  static __device__ __forceinline__ double mma4(double a, double b, double c) {
    return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
  }
};

template <>
struct MF<float> {
  typedef float v4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ v4 mma(float a, float b, v4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int drow(int lane, int i) { return ((lane >> 4) << 2) + i; }
  // fp32 tiles never take the 4x4x4 path (its k order interleaves the lane groups); present so that the
  // constant-false branches compile
  static __device__ __forceinline__ float mma4(float, float, float c) { return c; }
};

// Uniform-lane broadcast (v_readlane -> SGPR).
__device__ __forceinline__ float bcast(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double bcast(double v, int l) {
  unsigned long long u = (unsigned long long)__double_as_longlong(v);
  unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ int bcast(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations, not for its
// outstanding global loads/stores (a __syncthreads() fence would drain vmcnt every step and
// serialise the HBM prefetch of the next propagators behind the barrier).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Block-wide sum of a double over blockDim.x threads (<= 1024); result valid in all threads.
__device__ __forceinline__ double block_sum(double v, double* scratch) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  double s = 0.0;
  const int nw = (blockDim.x + 63) >> 6;
  for (int i = 0; i < nw; ++i) s += scratch[i];
  __syncthreads();
  return s;
}

}  // namespace qoc
