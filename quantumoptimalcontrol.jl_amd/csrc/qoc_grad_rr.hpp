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

}  // namespace qoc
