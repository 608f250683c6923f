// qoc_grad_rr.hpp — fused order-3 GRAPE gradient, register-resident (N <= 48, 16 % m == 0, nu <= 2).
//
// Replaces expm_jacobian!(dUkdp_order = 3) + _compute_u_sensitivity at
// src/gradient_computations.jl:61-74,177-223 for every (seed, slice) unit:
//   dJdu[k, j] = Re sum_cols [ <W0, A_j x> + <W1, A_j P1> + <λ/6, A_j P2> ],
//   P1 = X x, P2 = X P1, Q1 = X^H λ, Q2 = X^H Q1, W0 = λ + Q1/2 + Q2/6, W1 = λ/2 + Q1/6,
// with X = A_k = A0 + sum_j u_jk A_j, x = x_k, λ = λ_{k+1} (the same contraction as k_grad and the
// GEMM path), in ONE kernel:
//   * persistent workgroups of 4 waves keep the nu+1 generators in LDS (column-major, odd pitch) and
//     every wave loops over 16-column tiles: 16/m units side by side, one column per lane (l & 15);
//   * a tile's vectors (λ, Q1, W1, W0, x, P1, P2) live in registers in the MFMA D layout, which is
//     also the B-operand layout of the next product (k-step (t, e) = register (t, e)), so
//     X v = [A0 | A1 | ...] [v; u_1 v; ...] runs straight from registers with the generator as the
//     A operand (K-concatenated over the generators, u scaling per column);
//   * the contraction with A_j runs one row tile at a time and reduces in registers; one lane per
//     unit writes dJdu.  No intermediate touches HBM: per unit only x_k, λ_{k+1}, u_k in, dJdu out.
#pragma once
#include <type_traits>

#include "qoc_common.hpp"

namespace qoc {

template <typename T, int NT>
struct GradRR {
  static constexpr int NMAX = 16 * NT;
  static constexpr int NW = 4;  // waves per workgroup
  using M = MF<T>;
  using v4 = typename M::v4;
  struct Own {  // V[16t + drow(l, e)][tile column l & 15]
    v4 r[NT], i[NT];
  };
  // Generator pitch (column-major): odd for f64 (the A^H reads stride by it), multiple of 4 for f32.
  static __host__ __device__ int ldp(int N) { return sizeof(T) == 8 ? (N | 1) : ((N + 3) & ~3); }
  static __host__ __device__ size_t lds_bytes(int N, int nu) {  // the nu+1 generators
    return (size_t)2 * (nu + 1) * N * ldp(N) * sizeof(T);
  }
  static __device__ __forceinline__ int kidx(int s, int lane) { return 16 * (s >> 2) + M::drow(lane, s & 3); }
  // fp64: valid row quads of the last row tile (KS = ceil(N / 4)); < 4 runs it on 4x4x4 blocks
  template <int KS>
  static constexpr int last_quads() {
    return sizeof(T) == 8 ? KS - 4 * (NT - 1) : 4;
  }

  static __device__ __forceinline__ void mask_rows(int N, Own& X, int lane) {  // rows >= N -> 0 (last tile)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool ok = 16 * (NT - 1) + M::drow(lane, e) < N;
      X.r[NT - 1][e] = ok ? X.r[NT - 1][e] : T(0);
      X.i[NT - 1][e] = ok ? X.i[NT - 1][e] : T(0);
    }
  }

  // out = A_k V (HERM = false) or A_k^H V (HERM = true), A_k = sum_j c_j A_j with c_0 = 1, c_j = u_j of
  // this lane's unit (K-concatenation over the generators: B operand = c_j V).  One row tile at a time
  // (3 accumulators), so out must not alias V.
  template <int KS, int NU, bool HERM>
  static __device__ __forceinline__ void xmul(int N, const T* __restrict__ Gr, const T* __restrict__ Gi,
                                              const double* uj, const Own& V, Own& out, int lane) {
    const int ld = ldp(N), PL = N * ld;
    int li = lane & 15, l3 = lane & 3;
    asm volatile("" : "+v"(li), "+v"(l3));  // opaque: keeps the operand addresses from being hoisted out of the tile loop
    // the last row tile with LQ < 4 valid row quads runs as LQ v_mfma_f64_4x4x4_4b (MF<double>::mma4)
    constexpr int LQ = last_quads<KS>();
    constexpr bool Q4 = LQ < 4;
    auto tile = [&](int t, auto quads) __attribute__((always_inline)) {
      constexpr int QN = decltype(quads)::value;  // 0: one 16x16x4 per k-step; else QN 4x4x4 blocks
      constexpr int NQ = QN ? QN : 1;
      const int pc = min(16 * t + li, N - 1);  // clamped row of the A operand
      v4 rr = v4{0, 0, 0, 0}, ii = v4{0, 0, 0, 0}, S = v4{0, 0, 0, 0};
      T qrr[NQ], qii[NQ], qS[NQ];  // 4x4x4 accumulators (one register of the 16x16 D layout each)
#pragma unroll
      for (int q = 0; q < NQ; ++q) qrr[q] = qii[q] = qS[q] = T(0);
#pragma unroll
      for (int j = 0; j <= NU; ++j) {
        T cj = j == 0 ? T(1) : (T)uj[j - 1];
        asm volatile("" : "+v"(cj));  // opaque per row tile: c_j V is recomputed, not kept for every tile
        const T* gr = Gr + (size_t)j * PL;
        const T* gi = Gi + (size_t)j * PL;
        T pr[KS][NQ], pi[KS][NQ];
        auto load = [&](int s) __attribute__((always_inline)) {
          const int k = min(kidx(s, lane), N - 1);
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int pq = QN ? min(16 * t + 4 * q + l3, N - 1) : pc;
            const int a = HERM ? pq * ld + k : k * ld + pq;
            pr[s][q] = gr[a];
            pi[s][q] = gi[a];
          }
        };
        load(0);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          __builtin_amdgcn_sched_barrier(0);  // one k-step of look-ahead (register pressure)
          if (s + 1 < KS) load(s + 1);
          const T qr = cj * V.r[s >> 2][s & 3], qi = cj * V.i[s >> 2][s & 3];
          if constexpr (QN == 0) {
            rr = M::mma(pr[s][0], qr, rr);
            ii = M::mma(pi[s][0], qi, ii);
            S = M::mma(HERM ? pr[s][0] - pi[s][0] : pr[s][0] + pi[s][0], qr + qi, S);
          } else {
#pragma unroll
            for (int q = 0; q < QN; ++q) {
              qrr[q] = M::mma4(pr[s][q], qr, qrr[q]);
              qii[q] = M::mma4(pi[s][q], qi, qii[q]);
              qS[q] = M::mma4(HERM ? pr[s][q] - pi[s][q] : pr[s][q] + pi[s][q], qr + qi, qS[q]);
            }
          }
        }
      }
      if constexpr (QN > 0) {
#pragma unroll
        for (int q = 0; q < QN; ++q) {
          rr[q] = qrr[q];
          ii[q] = qii[q];
          S[q] = qS[q];
        }
      }
      if (HERM) {  // conj(a) q: Re = rr + ii, Im = S - rr + ii with S = (ar - ai)(qr + qi)
        out.r[t] = rr + ii;
        out.i[t] = S - rr + ii;
      } else {
        out.r[t] = rr - ii;
        out.i[t] = S - rr - ii;
      }
    };
#pragma unroll
    for (int t = 0; t < (Q4 ? NT - 1 : NT); ++t) tile(t, std::integral_constant<int, 0>());
    if constexpr (Q4) tile(NT - 1, std::integral_constant<int, Q4 ? LQ : 0>());
    mask_rows(N, out, lane);
  }

  // s_j += Re <W, A_j V> over this lane's entries, j = 1..nu (one row tile at a time: 3 accumulators).
  template <int KS, int NU>
  static __device__ __forceinline__ void contract(int N, const T* __restrict__ Gr, const T* __restrict__ Gi,
                                                  const Own& V, const Own& W, double* sj, int lane) {
    const int ld = ldp(N), PL = N * ld;
    int li = lane & 15, l3 = lane & 3;
    asm volatile("" : "+v"(li), "+v"(l3));  // see xmul
#pragma unroll
    for (int j = 1; j <= NU; ++j) {
      const T* gr = Gr + (size_t)j * PL;
      const T* gi = Gi + (size_t)j * PL;
      double acc = 0.0;
      constexpr int LQ = last_quads<KS>();
      constexpr bool Q4 = LQ < 4;
      auto tile = [&](int t, auto quads) __attribute__((always_inline)) {
        constexpr int QN = decltype(quads)::value;  // 0: 16x16x4; else QN 4x4x4 blocks (partial last tile)
        constexpr int NQ = QN ? QN : 1;
        const int pc = min(16 * t + li, N - 1);
        v4 rr = v4{0, 0, 0, 0}, ii = v4{0, 0, 0, 0}, S = v4{0, 0, 0, 0};
        T qrr[NQ], qii[NQ], qS[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) qrr[q] = qii[q] = qS[q] = T(0);
        T pr[KS][NQ], pi[KS][NQ];
        auto load = [&](int s) __attribute__((always_inline)) {
          const int k = min(kidx(s, lane), N - 1);
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int a = k * ld + (QN ? min(16 * t + 4 * q + l3, N - 1) : pc);
            pr[s][q] = gr[a];
            pi[s][q] = gi[a];
          }
        };
        load(0);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          __builtin_amdgcn_sched_barrier(0);
          if (s + 1 < KS) load(s + 1);
          const T qr = V.r[s >> 2][s & 3], qi = V.i[s >> 2][s & 3];
          if constexpr (QN == 0) {
            rr = M::mma(pr[s][0], qr, rr);
            ii = M::mma(pi[s][0], qi, ii);
            S = M::mma(pr[s][0] + pi[s][0], qr + qi, S);
          } else {
#pragma unroll
            for (int q = 0; q < QN; ++q) {
              qrr[q] = M::mma4(pr[s][q], qr, qrr[q]);
              qii[q] = M::mma4(pi[s][q], qi, qii[q]);
              qS[q] = M::mma4(pr[s][q] + pi[s][q], qr + qi, qS[q]);
            }
          }
        }
        if constexpr (QN > 0) {
#pragma unroll
          for (int q = 0; q < QN; ++q) {
            rr[q] = qrr[q];
            ii[q] = qii[q];
            S[q] = qS[q];
          }
        }
        // W is zero outside N, so the junk rows >= N of this tile contribute nothing
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double dr = (double)(rr[e] - ii[e]), di = (double)(S[e] - rr[e] - ii[e]);
          acc += (double)W.r[t][e] * dr + (double)W.i[t][e] * di;
        }
        asm volatile("" : "+v"(acc));  // materialise now: otherwise the tile's products are kept (spilled) to the end
      };
#pragma unroll
      for (int t = 0; t < (Q4 ? NT - 1 : NT); ++t) tile(t, std::integral_constant<int, 0>());
      if constexpr (Q4) tile(NT - 1, std::integral_constant<int, Q4 ? LQ : 0>());
      sj[j - 1] += acc;
    }
  }
};

// Tile geometry shared by the two gradient kernels: wave w of workgroup g takes tiles
// g*NW + w, + gridDim*NW, ...; a tile is 16/m units side by side, lane column c = l & 15.
struct GradTile {
  long long unit;
  bool ok;
  size_t bx, bl;  // x_k and λ_{k+1} column (c % m) offsets in the (Nt+1)-block state layout
};
// The units are the slices k0 .. k0+nk-1 of every seed (units = B nk); `unit` is the global b Nt + k.
__device__ __forceinline__ GradTile grad_tile(long long tile, int lane, int N, int m, int Nt, int k0, int nk,
                                              long long units) {
  GradTile g;
  const int c = lane & 15, upt = 16 / m;
  const long long ul = tile * upt + c / m;
  g.ok = ul < units;
  const long long un = g.ok ? ul : 0, b = un / nk, k = k0 + un % nk;
  g.unit = b * Nt + k;
  g.bx = ((size_t)(b * (Nt + 1) + k) * m + c % m) * N;
  g.bl = g.bx + (size_t)m * N;
  return g;
}

template <typename T, int NT>
__device__ __forceinline__ void grad_gens_to_lds(int N, int nu, const cx<T>* __restrict__ Agen, T* Gr, T* Gi) {
  using G = GradRR<T, NT>;
  const int ld = G::ldp(N), PL = N * ld, NN = N * N;
  for (int e = threadIdx.x; e < (nu + 1) * NN; e += blockDim.x) {  // column-major, pitch ld
    const int j = e / NN, r = e % NN;
    const cx<T> g = Agen[e];
    Gr[j * PL + (r / N) * ld + r % N] = g.r;
    Gi[j * PL + (r / N) * ld + r % N] = g.i;
  }
  __syncthreads();
}

template <typename T, int NT>
__device__ __forceinline__ void grad_load(const cx<T>* __restrict__ src, size_t base, bool ok, int N,
                                          typename GradRR<T, NT>::Own& V, int lane) {
  using M = MF<T>;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 16 * t + M::drow(lane, e);
      const bool v_ok = ok && row < N;
      const cx<T> v = src[base + (size_t)min(row, N - 1)];
      V.r[t][e] = v_ok ? v.r : T(0);
      V.i[t][e] = v_ok ? v.i : T(0);
    }
}
template <typename T, int NT>
__device__ __forceinline__ void grad_store(cx<T>* __restrict__ dst, size_t base, bool ok, int N,
                                           const typename GradRR<T, NT>::Own& V, int lane) {
  using M = MF<T>;
  if (!ok) return;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 16 * t + M::drow(lane, e);
      if (row < N) dst[base + row] = cx<T>{V.r[t][e], V.i[t][e]};
    }
}

// Co-state side: Q1 = X^H λ, Q2 = X^H Q1 -> W0 = λ + Q1/2 + Q2/6, W1 = λ/2 + Q1/6, written in the
// state layout (W0, W1 buffers shaped like X).
template <typename T, int NT, int KS, int NU>
__global__ __launch_bounds__(256, 2) void k_grad_rr_q(int N, int m, int Nt, int B, int k0, int nk, const cx<T>* __restrict__ Agen,
                                                      const double* __restrict__ u, const cx<T>* __restrict__ L,
                                                      cx<T>* __restrict__ W0, cx<T>* __restrict__ W1) {
  using G = GradRR<T, NT>;
  using Own = typename G::Own;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  T* Gr = reinterpret_cast<T*>(smem);
  T* Gi = Gr + (size_t)(NU + 1) * N * G::ldp(N);
  grad_gens_to_lds<T, NT>(N, NU, Agen, Gr, Gi);
  const long long units = (long long)B * nk, ntiles = (units + 16 / m - 1) / (16 / m);
  for (long long tile = (long long)blockIdx.x * nw + wave; tile < ntiles; tile += (long long)gridDim.x * nw) {
    const GradTile g = grad_tile(tile, lane, N, m, Nt, k0, nk, units);
    double uj[NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) uj[j] = u[g.unit * NU + j];
    Own Lam, Q1, Q2;
    grad_load<T, NT>(L, g.bl, g.ok, N, Lam, lane);
    G::template xmul<KS, NU, true>(N, Gr, Gi, uj, Lam, Q1, lane);
    G::template xmul<KS, NU, true>(N, Gr, Gi, uj, Q1, Q2, lane);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      Q2.r[t] = Lam.r[t] + Q1.r[t] * T(0.5) + Q2.r[t] * T(1.0 / 6.0);  // W0
      Q2.i[t] = Lam.i[t] + Q1.i[t] * T(0.5) + Q2.i[t] * T(1.0 / 6.0);
      Q1.r[t] = Lam.r[t] * T(0.5) + Q1.r[t] * T(1.0 / 6.0);  // W1
      Q1.i[t] = Lam.i[t] * T(0.5) + Q1.i[t] * T(1.0 / 6.0);
    }
    grad_store<T, NT>(W0, g.bx, g.ok, N, Q2, lane);
    grad_store<T, NT>(W1, g.bx, g.ok, N, Q1, lane);
  }
}

// State side and contraction: dJdu = Re[<W0, A_j x> + <W1, A_j P1> + <λ/6, A_j P2>], P1 = X x, P2 = X P1.
// PRE: P1 and P2 were computed beforehand by k_grad_rr_s (next to the first backward range) and are read here.
template <typename T, int NT, int KS, int NU, bool PRE = false>
__global__ __launch_bounds__(256, 2) void k_grad_rr_p(int N, int m, int Nt, int B, int k0, int nk, const cx<T>* __restrict__ Agen,
                                                      const double* __restrict__ u, const cx<T>* __restrict__ X,
                                                      const cx<T>* __restrict__ L, const cx<T>* __restrict__ W0,
                                                      const cx<T>* __restrict__ W1, double* __restrict__ dJdu,
                                                      const cx<T>* __restrict__ P1in = nullptr,
                                                      const cx<T>* __restrict__ P2in = nullptr) {
  using G = GradRR<T, NT>;
  using Own = typename G::Own;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  T* Gr = reinterpret_cast<T*>(smem);
  T* Gi = Gr + (size_t)(NU + 1) * N * G::ldp(N);
  grad_gens_to_lds<T, NT>(N, NU, Agen, Gr, Gi);
  const long long units = (long long)B * nk, ntiles = (units + 16 / m - 1) / (16 / m);
  for (long long tile = (long long)blockIdx.x * nw + wave; tile < ntiles; tile += (long long)gridDim.x * nw) {
    const GradTile g = grad_tile(tile, lane, N, m, Nt, k0, nk, units);
    double uj[NU], sj[NU], s2[NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) {
      uj[j] = u[g.unit * NU + j];
      sj[j] = 0.0;
      s2[j] = 0.0;
    }
    Own P, Pn, W;
    grad_load<T, NT>(X, g.bx, g.ok, N, P, lane);
    grad_load<T, NT>(W0, g.bx, g.ok, N, W, lane);
    G::template contract<KS, NU>(N, Gr, Gi, P, W, sj, lane);
    if constexpr (PRE) grad_load<T, NT>(P1in, g.bx, g.ok, N, Pn, lane);
    else G::template xmul<KS, NU, false>(N, Gr, Gi, uj, P, Pn, lane);  // P1
    asm volatile("" ::: "memory");  // keep the W loads here: hoisted above a product they add 48 live VGPRs
    grad_load<T, NT>(W1, g.bx, g.ok, N, W, lane);
    G::template contract<KS, NU>(N, Gr, Gi, Pn, W, sj, lane);
    if constexpr (PRE) grad_load<T, NT>(P2in, g.bx, g.ok, N, P, lane);
    else G::template xmul<KS, NU, false>(N, Gr, Gi, uj, Pn, P, lane);  // P2
    asm volatile("" ::: "memory");
    grad_load<T, NT>(L, g.bl, g.ok, N, W, lane);
    G::template contract<KS, NU>(N, Gr, Gi, P, W, s2, lane);
    // reduce over the unit's lanes: the 4 row groups (l >> 4) and its m columns
    const int c = lane & 15;
#pragma unroll
    for (int j = 0; j < NU; ++j) {
      double v = sj[j] + s2[j] * (1.0 / 6.0);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      for (int o = 1; o < m; o <<= 1) v += __shfl_xor(v, o);
      if (g.ok && lane < 16 && c % m == 0) dJdu[g.unit * NU + j] = v;
    }
  }
}

// State side alone: P1 = X x, P2 = X P1 for the units of slices k0 .. k0+nk-1, written in the state layout.  It
// needs only the forward's states, so it runs on the second stream beside the first backward range (which
// otherwise has nothing beside it); k_grad_rr_p<PRE = true> then reads P1, P2 instead of forming them.
template <typename T, int NT, int KS, int NU>
__global__ __launch_bounds__(256, 2) void k_grad_rr_s(int N, int m, int Nt, int B, int k0, int nk, const cx<T>* __restrict__ Agen,
                                                      const double* __restrict__ u, const cx<T>* __restrict__ X,
                                                      cx<T>* __restrict__ P1out, cx<T>* __restrict__ P2out) {
  using G = GradRR<T, NT>;
  using Own = typename G::Own;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  T* Gr = reinterpret_cast<T*>(smem);
  T* Gi = Gr + (size_t)(NU + 1) * N * G::ldp(N);
  grad_gens_to_lds<T, NT>(N, NU, Agen, Gr, Gi);
  const long long units = (long long)B * nk, ntiles = (units + 16 / m - 1) / (16 / m);
  for (long long tile = (long long)blockIdx.x * nw + wave; tile < ntiles; tile += (long long)gridDim.x * nw) {
    const GradTile g = grad_tile(tile, lane, N, m, Nt, k0, nk, units);
    double uj[NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) uj[j] = u[g.unit * NU + j];
    Own P, Pn;
    grad_load<T, NT>(X, g.bx, g.ok, N, P, lane);
    G::template xmul<KS, NU, false>(N, Gr, Gi, uj, P, Pn, lane);
    grad_store<T, NT>(P1out, g.bx, g.ok, N, Pn, lane);
    G::template xmul<KS, NU, false>(N, Gr, Gi, uj, Pn, P, lane);
    grad_store<T, NT>(P2out, g.bx, g.ok, N, P, lane);
  }
}

// ---------------------------------------------------------------------------------------------------------
// Contraction from the chains' captured products (k_grad_rr_c).  The register-resident MFMA chains write, per slice,
// their first two products D1 = Â v, D2 = Â y_1 with Â = scale · Ã_k (Ã_k = A_k − μ_k I, the exact scalar shift) and
// y_1 = D1 / κ' (κ' = 2 Chebyshev, 1 Taylor): Ã v = r D1 and Ã² v = κ r² D2 with r = 1 / scale, κ = κ'.  So, with
// A_k = Ã_k + μ_k I (src/gradient_computations.jl:18-22) and the products of the reference's order-3 Jacobian
// (:177-213, contracted as in k_grad_rr_q / _p):
//   P1 = A x = μ x + r F1,   P2 = A² x = μ² x + 2 μ r F1 + κ r² F2            (F: forward captures, v = x_k)
//   Q1 = A^H λ = μ̄ λ + r G1, Q2 = μ̄² λ + 2 μ̄ r G1 + κ r² G2                  (G: backward captures, v = λ_{k+1})
//   W0 = λ + Q1/2 + Q2/6,    W1 = λ/2 + Q1/6
//   dJdu[k, j] = Re[<W0, A_j x> + <W1, A_j P1> + <λ/6, A_j P2>]
// i.e. only the 3 nu contractions are generator products.  μ mode (coef != nullptr): the backward chain ran from
// X_target (μ_k = U_k^H .. U_{Nt-1}^H X_target) and λ = coef ⊙ μ element-wise (lam_coef: per row sector and column),
// which commutes with every product above, so W0, W1 and λ are scaled by the coefficient on load.
struct GradCapArgs {
  int N, m, Nt, B, k0, nk;
  const void* Agen;          // generators A_j (unshifted), column-major
  const double* u;           // B x Nt x nu
  const void* X;             // states (B x (Nt+1) x N x m)
  const void* L;             // co-states λ, or μ in μ mode
  const void* F1;            // forward captures D1, D2 at slice k
  const void* F2;
  const void* G1;            // backward captures D1, D2 at slice k
  const void* G2;
  const double* steps;       // TStep records, 4 doubles each (scale at [3]); nullptr: scale 1 (qoc_blkp.hpp)
  double mur[3], mui[3];     // shifts μ_j: μ_k = μ_0 + Σ_j u_jk μ_j
  double kappa;              // 2 Chebyshev, 1 Taylor
  const cx<double>* coef;    // μ mode: λ_N coefficients (B x 2m, chain_costs); nullptr: L holds λ
  unsigned long long rsec_mask;  // packed states: bit r = row sector of row r (N <= 64), else 0
  double* dJdu;
};

template <int NT, int KS, int NU>
__global__ __launch_bounds__(256, 2) void k_grad_rr_c(const GradCapArgs a) {
  using G = GradRR<double, NT>;
  using Own = typename G::Own;
  using M = MF<double>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.N, m = a.m, Nt = a.Nt;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  double* Gr = reinterpret_cast<double*>(smem);
  double* Gi = Gr + (size_t)(NU + 1) * N * G::ldp(N);
  grad_gens_to_lds<double, NT>(N, NU, (const cx<double>*)a.Agen, Gr, Gi);
  const long long units = (long long)a.B * a.nk, ntiles = (units + 16 / m - 1) / (16 / m);
  const int col = (lane & 15) % m;
  // V = c * src (ACC: V += c * src) over this lane's entries; rows >= N read the last row (masked later)
  // the lane index is made opaque per call: otherwise every row offset / mask of every call is hoisted out of the
  // tile loop (loop-invariant) and spilled
  auto ld = [&](Own& V, const void* srcv, size_t base, cx<double> c, bool accum) __attribute__((always_inline)) {
    const cx<double>* src = (const cx<double>*)srcv + base;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const cx<double> x = src[min(16 * t + M::drow(ln, e), N - 1)];
        const double vr = c.r * x.r - c.i * x.i, vi = c.r * x.i + c.i * x.r;
        V.r[t][e] = accum ? V.r[t][e] + vr : vr;
        V.i[t][e] = accum ? V.i[t][e] + vi : vi;
      }
    asm volatile("" ::: "memory");  // one source at a time
  };
  // rows >= N (and tiles past the last unit) -> 0; μ mode: × λ_N coefficient of (row sector, column)
  auto fin = [&](Own& V, bool ok, bool scl, cx<double> f0, cx<double> f1) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * t + M::drow(ln, e);
        const bool in = ok && row < N;
        double vr = V.r[t][e], vi = V.i[t][e];
        if (scl) {
          const cx<double> f = ((a.rsec_mask >> min(row, 63)) & 1ull) ? f1 : f0;
          const double wr = f.r * vr - f.i * vi;
          vi = f.r * vi + f.i * vr;
          vr = wr;
        }
        V.r[t][e] = in ? vr : 0.0;
        V.i[t][e] = in ? vi : 0.0;
      }
  };
  for (long long tile = (long long)blockIdx.x * nw + wave; tile < ntiles; tile += (long long)gridDim.x * nw) {
    const GradTile g = grad_tile(tile, lane, N, m, Nt, a.k0, a.nk, units);
    double sj[NU], s2[NU];
    double mr = a.mur[0], mi = a.mui[0];
#pragma unroll
    for (int j = 0; j < NU; ++j) {
      const double uj = a.u[g.unit * NU + j];
      mr += uj * a.mur[j + 1];
      mi += uj * a.mui[j + 1];
      sj[j] = 0.0;
      s2[j] = 0.0;
    }
    const double r = a.steps ? 1.0 / a.steps[4 * g.unit + 3] : 1.0, kr2 = a.kappa * r * r;
    const bool scl = a.coef != nullptr;
    cx<double> f0 = {1.0, 0.0}, f1 = {1.0, 0.0};
    if (scl) {
      const cx<double>* cb = a.coef + (size_t)(g.unit / Nt) * 2 * m;
      f0 = cb[col];
      f1 = cb[m + col];
    }
    const double br = mr, bi = -mi;                                  // conj(μ_k)
    const double b2r = mr * mr - mi * mi, b2i = -2.0 * mr * mi;      // conj(μ_k)^2
    Own V, W;
    // <W0, A_j x>,  W0 = (1 + μ̄/2 + μ̄²/6) λ + r (1/2 + μ̄/3) G1 + κ r²/6 G2
    ld(W, a.L, g.bl, cx<double>{1.0 + br / 2 + b2r / 6, bi / 2 + b2i / 6}, false);
    ld(W, a.G1, g.bx, cx<double>{r * (0.5 + br / 3), r * bi / 3}, true);
    ld(W, a.G2, g.bx, cx<double>{kr2 / 6, 0.0}, true);
    fin(W, g.ok, scl, f0, f1);
    ld(V, a.X, g.bx, cx<double>{1.0, 0.0}, false);
    fin(V, g.ok, false, f0, f1);
    G::template contract<KS, NU>(N, Gr, Gi, V, W, sj, lane);
    asm volatile("" ::: "memory");
    // <W1, A_j P1>,  P1 = μ x + r F1,  W1 = (1/2 + μ̄/6) λ + r/6 G1
    ld(V, a.X, g.bx, cx<double>{mr, mi}, false);
    ld(V, a.F1, g.bx, cx<double>{r, 0.0}, true);
    fin(V, g.ok, false, f0, f1);
    ld(W, a.L, g.bl, cx<double>{0.5 + br / 6, bi / 6}, false);
    ld(W, a.G1, g.bx, cx<double>{r / 6, 0.0}, true);
    fin(W, g.ok, scl, f0, f1);
    G::template contract<KS, NU>(N, Gr, Gi, V, W, sj, lane);
    asm volatile("" ::: "memory");
    // <λ, A_j P2> / 6,  P2 = μ² x + 2 μ r F1 + κ r² F2
    ld(V, a.X, g.bx, cx<double>{b2r, -b2i}, false);
    ld(V, a.F1, g.bx, cx<double>{2.0 * r * mr, 2.0 * r * mi}, true);
    ld(V, a.F2, g.bx, cx<double>{kr2, 0.0}, true);
    fin(V, g.ok, false, f0, f1);
    ld(W, a.L, g.bl, cx<double>{1.0, 0.0}, false);
    fin(W, g.ok, scl, f0, f1);
    G::template contract<KS, NU>(N, Gr, Gi, V, W, s2, lane);
    const int c = lane & 15;
#pragma unroll
    for (int j = 0; j < NU; ++j) {
      double v = sj[j] + s2[j] * (1.0 / 6.0);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      for (int o = 1; o < m; o <<= 1) v += __shfl_xor(v, o);
      if (g.ok && lane < 16 && c % m == 0) a.dJdu[g.unit * NU + j] = v;
    }
  }
}

}  // namespace qoc
