// qoc_ode.hpp — the ODE path: fixed-step Tsit5 on the batched layout.
//
//   k_ode_pwc:      propagate_pwc (src/gradient_computations.jl:108-128) — slice k integrates
//                   dx/dτ = A_k x over τ ∈ [k, k+1] with nsub Tsit5 steps (reference dt = 0.1Δt ->
//                   nsub = 10) and stores the slice-boundary states; with adjoint != 0 it runs the
//                   co-state sweep of compute_pwc_gradient (:130-150) backwards, dλ/dτ = -A_k^H λ.
//   k_ode_envelope: continuous controls c_j(t) from a parameterised pulse (wrap_envelope,
//                   src/QuantumOptimalControl.jl:43-54; examples/two_qubit_tunable_bus.jl:10-60).
//
// Layout: one workgroup per seed, one wave per state column (lane = row, N <= 64); the slice's A_k
// (or A_k^H) lives in LDS, the state and the seven Tsit5 stages live in registers, and the mat-vec
// broadcasts x_j with v_readlane (no LDS traffic for the state, no barriers inside a step).
#pragma once
#include "qoc_common.hpp"

namespace qoc {

// Tsitouras (2011) 5(4) tableau as in OrdinaryDiffEq's Tsit5 (row 7 = b, first-same-as-last).
__constant__ double kTsitC[7] = {0.0, 0.161, 0.327, 0.9, 0.9800255409045097, 1.0, 1.0};
__constant__ double kTsitA[7][6] = {
    {0, 0, 0, 0, 0, 0},
    {0.161, 0, 0, 0, 0, 0},
    {-0.008480655492356989, 0.335480655492357, 0, 0, 0, 0},
    {2.897153057105493, -6.359448489975075, 4.3622954328695815, 0, 0, 0},
    {5.325864828439257, -11.748883564062828, 7.4955393428898365, -0.09249506636175525, 0, 0},
    {5.86145544294642, -12.92096931784711, 8.159367898576159, -0.071584973281401, -0.028269050394068383, 0},
    {0.09646076681806523, 0.01, 0.4798896504144996, 1.379008574103742, -3.290069515436081, 2.324710524099774}};

// y_lane = sum_j M[lane + N j] x_j  (M column-major N x N in LDS, x distributed one element per lane).
// Eight LDS loads are issued ahead of their FMAs and two accumulators break the FMA dependency chain.
template <typename T>
__device__ __forceinline__ cx<T> ode_matvec(int N, const cx<T>* __restrict__ M, cx<T> x, int lane) {
  cx<T> y0 = {0, 0}, y1 = {0, 0};
  const int row = lane < N ? lane : 0;
  int j = 0;
  for (; j + 8 <= N; j += 8) {
    cx<T> a[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) a[t] = M[row + N * (j + t)];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const T xr = bcast(x.r, j + t), xi = bcast(x.i, j + t);
      cx<T>& y = (t & 1) ? y1 : y0;
      y.r += a[t].r * xr - a[t].i * xi;
      y.i += a[t].r * xi + a[t].i * xr;
    }
  }
  for (; j < N; ++j) {
    const T xr = bcast(x.r, j), xi = bcast(x.i, j);
    const cx<T> a = M[row + N * j];
    y0.r += a.r * xr - a.i * xi;
    y0.i += a.r * xi + a.i * xr;
  }
  return cx<T>{y0.r + y1.r, y0.i + y1.i};
}

// Same product with the lane's row of M held in registers (arow[j] = M[lane, j], zero-padded to NB
// and zero rows for lanes >= N, so those lanes stay at x = 0).  x goes through a wave-private LDS
// slot and comes back as broadcast ds_reads (no SGPR traffic), eight at a time; the uniform guard
// skips whole blocks of eight beyond N.
template <typename T, int NB>
__device__ __forceinline__ cx<T> ode_matvec_reg(int N, const cx<T> (&arow)[NB], cx<T> x, cx<T>* __restrict__ xs,
                                                int lane) {
  xs[lane] = x;  // LDS operations of one wave complete in order: the reads below see this write
  cx<T> y0 = {0, 0}, y1 = {0, 0};
#pragma unroll
  for (int jb = 0; jb < NB; jb += 8) {
    if (jb < N) {
      cx<T> xv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) xv[t] = xs[jb + t];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const cx<T> a = arow[jb + t];
        cx<T>& y = (t & 1) ? y1 : y0;
        y.r = fma(a.r, xv[t].r, y.r);
        y.r = fma(-a.i, xv[t].i, y.r);
        y.i = fma(a.r, xv[t].i, y.i);
        y.i = fma(a.i, xv[t].r, y.i);
      }
    }
  }
  return cx<T>{y0.r + y1.r, y0.i + y1.i};
}

// One Tsit5 step of size h for dx/dt = F(x, stage time), F given as a functor (mat-vec(s)).
template <typename T, typename RHS>
__device__ __forceinline__ void tsit5_step(cx<T>& x, cx<T>& k1, T h, double t, RHS rhs) {
  cx<T> k[7];
  k[0] = k1;
#pragma unroll
  for (int i = 1; i < 7; ++i) {
    cx<T> xi = x;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      if (j < i) {
        const T a = (T)kTsitA[i][j] * h;
        xi.r += a * k[j].r;
        xi.i += a * k[j].i;
      }
    }
    k[i] = rhs(xi, t + kTsitC[i] * (double)h);
  }
  // x_{n+1} = x + h sum_j b_j k_j  (b = row 7); the 7th stage was evaluated there (FSAL)
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const T b = (T)kTsitA[6][j] * h;
    x.r += b * k[j].r;
    x.i += b * k[j].i;
  }
  k1 = k[6];
}

// Slice-by-slice PWC propagation.  Forward (adjoint = 0): S[b][0] = x0, S[b][k+1] from S[b][k].
// Adjoint: S = Lam holds λ_Nt already (cost gradient + penalty); λ_k from λ_{k+1} under A_k^H, then
// += 2 mu mask .* x_k (the exp path's dL/dx convention).  Block = 64 * W threads, wave w owns
// columns w, w + W, ...  NB > 0: each lane keeps its row of A_k (N <= NB) in registers for the
// slice's nsub * 6 stage products; NB = 0: the rows are read from LDS.
template <typename T, int NB>
__global__ __launch_bounds__(256) void k_ode_pwc(int N, int m, int nu, int Nt, int nsub, int adjoint,
                                                 const cx<T>* __restrict__ Agen, const double* __restrict__ u,
                                                 const cx<T>* __restrict__ x0, int x0_per_seed, cx<T>* __restrict__ S,
                                                 const cx<T>* __restrict__ X, const unsigned char* __restrict__ pmask,
                                                 double two_mu) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cx<T>* Ak = reinterpret_cast<cx<T>*>(smem);
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, W = blockDim.x >> 6;
  const size_t NN = (size_t)N * N, Nm = (size_t)N * m;
  cx<T>* Sb = S + (size_t)b * (Nt + 1) * Nm;
  const cx<T>* Xb = X + (size_t)b * (Nt + 1) * Nm;
  const T h = (T)(1.0 / nsub);
  if (!adjoint) {
    const cx<T>* x0b = x0 + (x0_per_seed ? (size_t)b * Nm : 0);
    for (size_t o = tid; o < Nm; o += blockDim.x) Sb[o] = x0b[o];
  }
  for (int kk = 0; kk < Nt; ++kk) {
    const int k = adjoint ? Nt - 1 - kk : kk;
    __syncthreads();
    // A_k (forward) or A_k^H (adjoint) into LDS
    const double* uk = u + ((size_t)b * Nt + k) * nu;
    for (size_t e = tid; e < NN; e += blockDim.x) {
      const size_t r = e % N, c = e / N;
      const size_t src = adjoint ? c + N * r : e;
      cx<T> a = Agen[src];
      for (int j = 0; j < nu; ++j) {
        const cx<T> v = Agen[(size_t)(j + 1) * NN + src];
        a.r += (T)uk[j] * v.r;
        a.i += (T)uk[j] * v.i;
      }
      if (adjoint) a.i = -a.i;
      Ak[e] = a;
    }
    __syncthreads();
    if constexpr (NB > 0) {
      static_assert(NB % 8 == 0, "row blocks of eight");
      cx<T>* xs = reinterpret_cast<cx<T>*>(smem + ((NN * sizeof(cx<T>) + 15) & ~(size_t)15)) + 64 * wave;
      cx<T> arow[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) arow[j] = (lane < N && j < N) ? Ak[lane + N * j] : cx<T>{0, 0};
      for (int col = wave; col < m; col += W) {
        const size_t in = (size_t)(adjoint ? k + 1 : k) * Nm + (size_t)N * col;
        const size_t outo = (size_t)(adjoint ? k : k + 1) * Nm + (size_t)N * col;
        cx<T> x = lane < N ? Sb[in + lane] : cx<T>{0, 0};
        auto rhs = [&](cx<T> y, double) __attribute__((always_inline)) {
          return ode_matvec_reg<T, NB>(N, arow, y, xs, lane);
        };
        cx<T> k1 = rhs(x, 0.0);
        for (int s = 0; s < nsub; ++s) tsit5_step<T>(x, k1, h, 0.0, rhs);
        if (lane < N) {
          if (adjoint && pmask && pmask[(size_t)N * col + lane]) {
            const cx<T> xv = Xb[outo + lane];
            x.r += (T)two_mu * xv.r;
            x.i += (T)two_mu * xv.i;
          }
          Sb[outo + lane] = x;
        }
      }
    } else {
      for (int col = wave; col < m; col += W) {
        const size_t in = (size_t)(adjoint ? k + 1 : k) * Nm + (size_t)N * col;
        const size_t outo = (size_t)(adjoint ? k : k + 1) * Nm + (size_t)N * col;
        cx<T> x = lane < N ? Sb[in + lane] : cx<T>{0, 0};
        auto rhs = [&](cx<T> y, double) __attribute__((always_inline)) { return ode_matvec<T>(N, Ak, y, lane); };
        cx<T> k1 = rhs(x, 0.0);
        for (int s = 0; s < nsub; ++s) tsit5_step<T>(x, k1, h, 0.0, rhs);
        if (lane < N) {
          if (adjoint && pmask && pmask[(size_t)N * col + lane]) {
            const cx<T> xv = Xb[outo + lane];
            x.r += (T)two_mu * xv.r;
            x.i += (T)two_mu * xv.i;
          }
          Sb[outo + lane] = x;
        }
      }
    }
  }
}

// Parameterised pulses (src/parameterized_pulses.jl) evaluated on the device.
enum { ENV_TUNABLE_BUS = 0, ENV_DRAG = 1, ENV_SINEBASIS = 2 };

__device__ __forceinline__ double cos_envelope_dev(double t_plateau, double t_rise_fall, double t) {
  if (t > t_rise_fall / 2 && t <= t_rise_fall / 2 + t_plateau) return 1.0;
  if (t <= t_rise_fall / 2) return 0.5 * (1 - cos(2 * M_PI * t / t_rise_fall));
  return 0.5 * (1 - cos(2 * M_PI * (t - t_plateau) / t_rise_fall));
}

// c[0..nu) at time t for envelope `kind` with parameters p
__device__ __forceinline__ void envelope_dev(int kind, const double* __restrict__ p, int np, double t, double (&c)[2]) {
  if (kind == ENV_TUNABLE_BUS) {  // examples/two_qubit_tunable_bus.jl:10-18
    const double d = cos_envelope_dev(p[0], p[1], t);
    c[0] = sqrt(fabs(cos(M_PI * (p[2] + p[4] * d * cos(p[3] * t)))));
  } else if (kind == ENV_DRAG) {  // u_drag: (tgate, sigma, A, xi) -> (Re, Im)
    const double x = t - p[0] / 2, s2 = p[1] * p[1];
    const double tmp = exp(-x * x / (2 * s2));
    c[0] = p[2] * (tmp - exp(-p[0] * p[0] / (8 * s2)));
    c[1] = p[2] * (-p[3] * x / s2 * tmp);
  } else {  // u_sinebasis: (Tgate, p_1x, p_1y, p_2x, ...) -> (Re, Im)
    double ox = 0, oy = 0;
    for (int k = 1; 2 * k + 1 <= np; ++k) {
      const double bk = sin(M_PI * k * t / p[0]);
      ox += p[2 * k - 1] * bk;
      oy += p[2 * k] * bk;
    }
    c[0] = ox;
    c[1] = oy;
  }
}

// dx/dt = (A0 + sum_j c_j(t) A_j) x from t = 0 to nsteps * dt; S[b][0] = x0, S[b][Nt] = x(tgate).
template <typename T>
__global__ __launch_bounds__(256) void k_ode_envelope(int N, int m, int nu, int Nt, int kind, const double* __restrict__ P,
                                                      int np, double dt, long long nsteps, const cx<T>* __restrict__ Agen,
                                                      const cx<T>* __restrict__ x0, int x0_per_seed,
                                                      cx<T>* __restrict__ S) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cx<T>* G = reinterpret_cast<cx<T>*>(smem);  // (nu + 1) generators
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, W = blockDim.x >> 6;
  const size_t NN = (size_t)N * N, Nm = (size_t)N * m;
  for (size_t e = tid; e < (size_t)(nu + 1) * NN; e += blockDim.x) G[e] = Agen[e];
  cx<T>* Sb = S + (size_t)b * (Nt + 1) * Nm;
  const cx<T>* x0b = x0 + (x0_per_seed ? (size_t)b * Nm : 0);
  for (size_t o = tid; o < Nm; o += blockDim.x) Sb[o] = x0b[o];
  const double* p = P + (size_t)b * np;
  __syncthreads();
  for (int col = wave; col < m; col += W) {
    cx<T> x = lane < N ? x0b[(size_t)N * col + lane] : cx<T>{0, 0};
    auto rhs = [&](cx<T> y, double t) __attribute__((always_inline)) {
      double cc[2] = {0, 0};
      envelope_dev(kind, p, np, t, cc);
      cx<T> r = ode_matvec<T>(N, G, y, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (j < nu) {
          const cx<T> v = ode_matvec<T>(N, G + (size_t)(j + 1) * NN, y, lane);
          r.r += (T)cc[j] * v.r;
          r.i += (T)cc[j] * v.i;
        }
      }
      return r;
    };
    cx<T> k1 = rhs(x, 0.0);
    for (long long s = 0; s < nsteps; ++s) tsit5_step<T>(x, k1, (T)dt, (double)s * dt, rhs);
    if (lane < N) Sb[(size_t)Nt * Nm + (size_t)N * col + lane] = x;
  }
}

}  // namespace qoc
