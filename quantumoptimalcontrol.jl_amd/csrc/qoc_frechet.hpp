// qoc_frechet.hpp — opt-in exact gradient (dUkdp_order = QOC_DUKDP_EXACT).
//
// The Taylor series of expm_jacobian! (src/gradient_computations.jl:177-213) is replaced by the
// Fréchet derivative of the propagator.  With L(A, E) = int_0^1 e^{sA} E e^{(1-s)A} ds,
//   dJ/du_j[k] = Re <λ_{k+1}, L(A_k, A_j) x_k> = Re tr(A_j L(A_k, Z_k)),   Z_k = x_k λ_{k+1}^H,
// so ONE Fréchet derivative per slice serves every control.  It is the top-right block of
// exp([[A_k, αZ_k], [0, A_k]]) / α (α a power of two that makes αZ_k tiny next to A_k, so the Padé
// degree / squarings of the block match those of A_k and the result is exactly linear in Z).
#pragma once
#include "qoc_common.hpp"

namespace qoc {

// blocks[it] (2N x 2N, column-major) = [[A_k, α Z_k], [0, A_k]], alpha[it] = α; unit = u0 + it = b*Nt + k.
template <typename T>
__global__ __launch_bounds__(256) void k_frechet_build(int N, int m, int nu, int Nt, long long u0,
                                                       const cx<T>* __restrict__ Agen, const double* __restrict__ u,
                                                       const cx<T>* __restrict__ X, const cx<T>* __restrict__ Lam,
                                                       cx<T>* __restrict__ blocks, double* __restrict__ alpha) {
  __shared__ double red[8];
  const int it = blockIdx.x;
  const long long unit = u0 + it;
  const long long b = unit / Nt, k = unit - b * Nt;
  const size_t NN = (size_t)N * N, Nm = (size_t)N * m, n2 = 2 * (size_t)N;
  const cx<T>* xk = X + ((size_t)b * (Nt + 1) + k) * Nm;
  const cx<T>* lk = Lam + ((size_t)b * (Nt + 1) + k + 1) * Nm;
  cx<T>* M = blocks + (size_t)it * n2 * n2;
  double uj[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) uj[j] = j < nu ? u[unit * nu + j] : 0.0;
  double amax = 0.0, zmax = 0.0;
  for (size_t e = threadIdx.x; e < NN; e += blockDim.x) {
    const int r = (int)(e % N), cc = (int)(e / N);
    cx<T> a = Agen[e];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < nu) {
        const cx<T> v = Agen[(size_t)(j + 1) * NN + e];
        a.r += (T)uj[j] * v.r;
        a.i += (T)uj[j] * v.i;
      }
    }
    M[r + n2 * cc] = a;                     // top-left
    M[(N + r) + n2 * (N + cc)] = a;         // bottom-right
    M[(N + r) + n2 * cc] = cx<T>{0, 0};     // bottom-left
    cx<double> z = {0, 0};                  // Z[r, cc] = sum_i x[r, i] conj(λ[cc, i])
    for (int i = 0; i < m; ++i) {
      const cx<T> xv = xk[r + (size_t)N * i], lv = lk[cc + (size_t)N * i];
      z.r += (double)xv.r * lv.r + (double)xv.i * lv.i;
      z.i += (double)xv.i * lv.r - (double)xv.r * lv.i;
    }
    M[r + n2 * (N + cc)] = cx<T>{(T)z.r, (T)z.i};  // top-right, rescaled below
    amax = fmax(amax, fabs((double)a.r) + fabs((double)a.i));
    zmax = fmax(zmax, fabs(z.r) + fabs(z.i));
  }
  // block max of amax / zmax
  for (int off = 32; off > 0; off >>= 1) {
    amax = fmax(amax, __shfl_xor(amax, off));
    zmax = fmax(zmax, __shfl_xor(zmax, off));
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) {
    red[w] = amax;
    red[4 + w] = zmax;
  }
  __syncthreads();
  amax = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  zmax = fmax(fmax(red[4], red[5]), fmax(red[6], red[7]));
  double al = 1.0;
  if (zmax > 0.0) al = ldexp(1.0, (int)floor(log2(fmax(amax, 1e-300) / zmax)) - 20);
  if (threadIdx.x == 0) alpha[it] = al;
  for (size_t e = threadIdx.x; e < NN; e += blockDim.x) {  // each thread rescales what it wrote
    const int r = (int)(e % N), cc = (int)(e / N);
    cx<T> z = M[r + n2 * (N + cc)];
    z.r = (T)(z.r * al);
    z.i = (T)(z.i * al);
    M[r + n2 * (N + cc)] = z;
  }
}

// dJdu[unit*nu + j] = Re sum_{p,q} A_j[p,q] L[q,p] / α,  L[q,p] = E[q + 2N (N + p)].
// At holds the transposed generators (At_j[q + N p] = A_j[p, q]) so both reads are coalesced.
template <typename T>
__global__ __launch_bounds__(256) void k_frechet_contract(int N, int nu, long long u0, const cx<T>* __restrict__ At,
                                                          const cx<T>* __restrict__ E, const double* __restrict__ alpha,
                                                          double* __restrict__ dJdu) {
  __shared__ double red[8];
  const int it = blockIdx.x;
  const size_t NN = (size_t)N * N, n2 = 2 * (size_t)N;
  const cx<T>* Eb = E + (size_t)it * n2 * n2;
  double acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.0;
  for (size_t e = threadIdx.x; e < NN; e += blockDim.x) {
    const int q = (int)(e % N), p = (int)(e / N);
    const cx<T> L = Eb[q + n2 * (N + p)];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < nu) {
        const cx<T> a = At[(size_t)j * NN + e];
        acc[j] += (double)a.r * L.r - (double)a.i * L.i;
      }
    }
  }
  const double inv = 1.0 / alpha[it];
  const long long unit = u0 + it;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j < nu) {
      const double s = block_sum(acc[j], red);
      if (threadIdx.x == 0) dJdu[unit * nu + j] = s * inv;
    }
  }
}

// At_j[q + N p] = A_j[p, q] for the nu control generators (Agen + NN).
template <typename T>
__global__ void k_transpose_gens(int N, int nu, const cx<T>* __restrict__ Agen, cx<T>* __restrict__ At) {
  const size_t NN = (size_t)N * N;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < NN * nu; g += (size_t)gridDim.x * blockDim.x) {
    const size_t j = g / NN, e = g - j * NN;
    const size_t q = e % N, p = e / N;
    At[g] = Agen[(j + 1) * NN + p + N * q];
  }
}

// max over items of the 1-norm (max column sum of |a_ij|) of explicit n x n matrices.
template <typename T>
__global__ __launch_bounds__(256) void k_norm1_max(int n, const cx<T>* __restrict__ A, unsigned long long* __restrict__ nmax) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const cx<T>* Ab = A + (size_t)blockIdx.x * n * n;
  double best = 0.0;
  for (int c = wave; c < n; c += 4) {
    double s = 0.0;
    for (int r = lane; r < n; r += 64) {
      const cx<T> a = Ab[r + (size_t)n * c];
      s += sqrt((double)a.r * a.r + (double)a.i * a.i);
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    best = fmax(best, s);
  }
  if (lane == 0) atomicMax(nmax, (unsigned long long)__double_as_longlong(best));
}

}  // namespace qoc
