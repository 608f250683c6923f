// qoc_expm_rr.hpp — register-resident Taylor exponential (the default GRAPE exponential).
//
// Replaces ExponentialUtilities.exponential!(Ak, ExpMethodHigham2005(), cache) at
// src/gradient_computations.jl:24 (A_k formation :18-22) with the degree m = 3r+2 Taylor polynomial
// evaluated by Paterson-Stockmeyer (see qoc_expm.hpp: taylor_select, kTaylorTheta), re-organised so
// that the running matrix never leaves the registers:
//
//   * one workgroup of NT waves per (seed, slice) unit; wave w OWNS rows [16w, 16w+16) of every
//     matrix.  Its registers hold X^T tiles (t, w) in the MFMA D layout, i.e. lane l holds
//     X[16w + (l&15)][16t + drow(l, e)] for t < NT, e < 4;
//   * the product of an owned matrix X with a shared matrix B (row-major in LDS) is computed as
//     (X B)^T = B^T X^T: the MFMA A operand is B^T, read from LDS, and the B operand is X^T, whose
//     fragment for k-step (t, e) is exactly register (t, e) of the D layout — no data movement;
//   * polynomials in A commute, so the Horner step V <- A3 V + B_i is computed as V A3 + B_i with
//     A3 shared in LDS and V in registers: the r Horner GEMMs need no barrier and no LDS store;
//   * B_i = c_{3i} I + c_{3i+1} A + c_{3i+2} A2 is folded into the accumulator initialisation;
//   * LDS holds A, A2 (for the B_i) and the current right operand (A3, then the squaring operand),
//     row-major with row pitch ldp(N) (odd for f64); operand reads are unmasked (columns >= N read the next row or the
//     slack, which only reaches result columns >= N, and those are zeroed after every product), so
//     the loads of k-step s+1 stay in flight under the MFMAs of k-step s;
//   * squarings store the owned rows (ping-pong between two LDS buffers, one barrier each);
//   * U_k goes straight from registers to HBM (column-major, 16 consecutive rows per lane group).
//
// The Padé + solve kernel (k_expm ALG 0, the reference algorithm) stays in qoc_expm.hpp.
#pragma once
#include "qoc_expm.hpp"

namespace qoc {

// Sum over the 16 lanes of a DPP row (xor 1, xor 2, half mirror, mirror); result in every lane.
__device__ __forceinline__ float dpp_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xf, 0xf, false));  // row_mirror
  return v;
}

template <typename T, int NT>
struct ExpmRR {
  static constexpr int NMAX = 16 * NT;
  using M = MF<T>;
  using v4 = typename M::v4;

  struct Own {  // X[16w + (l&15)][16t + drow(l, e)], re / im; zero outside N x N
    v4 r[NT], i[NT];
  };

  // Rows of an LDS operand that the k-steps touch (rows N..R-1 are kept zero): f64 executes
  // ceil(N/4) k-steps (k < 4 ceil(N/4)), f32 all 4 NT (its k order interleaves the lane groups).
  static __host__ __device__ int rows(int N) { return sizeof(T) == 8 ? 4 * ((N + 3) / 4) : NMAX; }
  // Row pitch.  f64: odd, so the 16 rows one store_own / make_B instruction touches fall on distinct
  // banks.  f32: a multiple of 4 — the 4 consecutive columns a lane owns (drow = 4 (l>>4) + e) are
  // merged into 16-byte LDS accesses, which must stay 16-byte aligned.
  static __host__ __device__ int ldp(int N) { return sizeof(T) == 8 ? (N | 1) : ((N + 3) & ~3); }
  static __host__ __device__ int plane(int N) { return rows(N) * ldp(N); }
  // 3 matrices (A, A2, operand) x re/im planes, read slack past the last row, fp32 column partial sums.
  static __host__ __device__ size_t lds_bytes(int N) {
    return ((size_t)6 * plane(N) + 16) * sizeof(T) + (size_t)NT * NMAX * sizeof(float) + 16;
  }

  // k index of k-step s = 4 tk + e for this lane (f64: 16tk + 4e + (l>>4); f32: 16tk + 4(l>>4) + e).
  static __device__ __forceinline__ int kidx(int s, int lane) { return 16 * (s >> 2) + M::drow(lane, s & 3); }

  // Zero the entries of result columns >= N (they may hold products of the unmasked reads).
  static __device__ __forceinline__ void mask_cols(int N, Own& X, int lane) {
    // tiles t < NT-1 lie inside N (NT = ceil(N / 16))
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool ok = 16 * (NT - 1) + M::drow(lane, e) < N;
      X.r[NT - 1][e] = ok ? X.r[NT - 1][e] : T(0);
      X.i[NT - 1][e] = ok ? X.i[NT - 1][e] : T(0);
    }
  }

  // out = X B + init, with X owned (registers, zero outside N) and B shared (row-major LDS, pitch ldp(N)).
  // KS k-steps (compile time, branch-free); one k-step of look-ahead on the operand loads.
  // fp64: the last row tile holds LQ = KS - 4 (NT - 1) valid row quads (KS = ceil(N / 4)); when LQ < 4 it
  // runs as LQ v_mfma_f64_4x4x4_4b per component (16 cycles each) instead of one 16x16x4 (64 cycles).
  template <int KS>
  static constexpr int last_quads() {
    return sizeof(T) == 8 ? KS - 4 * (NT - 1) : 4;
  }
  template <int KS>
  static __device__ __forceinline__ void rmul(int N, const Own& X, const T* __restrict__ Br,
                                              const T* __restrict__ Bi, Own& out, const Own& init, int lane) {
    constexpr int LQ = last_quads<KS>();
    constexpr bool Q4 = LQ < 4;
    constexpr int NF = Q4 ? NT - 1 : NT;  // full 16-row tiles
    v4 rr[NT], ii[NT], S[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      rr[t] = init.r[t];
      ii[t] = v4{0, 0, 0, 0};
      S[t] = init.r[t] + init.i[t];
    }
    const int base = lane & 15;
    T pr[KS][NT], pi[KS][NT];
    T qpr[KS][Q4 ? LQ : 1], qpi[KS][Q4 ? LQ : 1];
    auto load = [&](int s) __attribute__((always_inline)) {
      const int a = kidx(s, lane) * ldp(N) + base;
#pragma unroll
      for (int t = 0; t < NF; ++t) {
        pr[s][t] = Br[a + 16 * t];
        pi[s][t] = Bi[a + 16 * t];
      }
      if constexpr (Q4) {
        const int a4 = kidx(s, lane) * ldp(N) + 16 * (NT - 1) + (lane & 3);
#pragma unroll
        for (int q = 0; q < LQ; ++q) {
          qpr[s][q] = Br[a4 + 4 * q];
          qpi[s][q] = Bi[a4 + 4 * q];
        }
      }
    };
    load(0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      __builtin_amdgcn_sched_barrier(0);  // keep the look-ahead at one k-step (register pressure)
      if (s + 1 < KS) load(s + 1);
      const T qr = X.r[s >> 2][s & 3], qi = X.i[s >> 2][s & 3], qs = qr + qi;
#pragma unroll
      for (int t = 0; t < NF; ++t) {
        rr[t] = M::mma(pr[s][t], qr, rr[t]);
        ii[t] = M::mma(pi[s][t], qi, ii[t]);
        S[t] = M::mma(pr[s][t] + pi[s][t], qs, S[t]);
      }
      if constexpr (Q4) {
#pragma unroll
        for (int q = 0; q < LQ; ++q) {
          rr[NT - 1][q] = M::mma4(qpr[s][q], qr, rr[NT - 1][q]);
          ii[NT - 1][q] = M::mma4(qpi[s][q], qi, ii[NT - 1][q]);
          S[NT - 1][q] = M::mma4(qpr[s][q] + qpi[s][q], qs, S[NT - 1][q]);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      out.r[t] = rr[t] - ii[t];
      out.i[t] = S[t] - rr[t] - ii[t];
    }
    mask_cols(N, out, lane);
  }

  static __device__ __forceinline__ void zero(Own& X) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      X.r[t] = v4{0, 0, 0, 0};
      X.i[t] = v4{0, 0, 0, 0};
    }
  }
  static __device__ __forceinline__ void scale(Own& X, T a) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      X.r[t] *= a;
      X.i[t] *= a;
    }
  }

  // Owned rows -> row-major LDS (pitch ldp(N)).  Rows N..rows(N)-1 are written too (zeros), which keeps
  // every row a k-step reads finite.
  static __device__ __forceinline__ void store_own(int N, const Own& X, T* Br, T* Bi, int row, int lane) {
    if (row >= rows(N)) return;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = 16 * t + M::drow(lane, e);
        if (t < NT - 1 || col < N) {  // tiles t < NT-1 lie inside N
          Br[row * ldp(N) + col] = X.r[t][e];
          Bi[row * ldp(N) + col] = X.i[t][e];
        }
      }
  }
};

// ALG 1 (Taylor) kernel.  unit = blockIdx.x.  Either generators (Agen, u) or explicit matrices (Ain).
// hist receives the Padé (d, s) the reference would select (reference-equivalent accounting), thist the
// executed Taylor (r, s).  KS: k-steps per product (see ExpmRR::rows).
template <typename T, int NT, int KS, int MODE>
__device__ __forceinline__ void expm_rr_unit(int unit, int N, int nu, const cx<T>* __restrict__ Agen,
                                             const double* __restrict__ u, const cx<T>* __restrict__ Ain,
                                             cx<T>* __restrict__ Uout, unsigned long long* __restrict__ hist,
                                             unsigned long long* __restrict__ thist, int* __restrict__ ps_list,
                                             int* __restrict__ ps_count) {
  using E = ExpmRR<T, NT>;
  using Own = typename E::Own;
  using M = typename E::M;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // opaque: in the persistent pass nothing derived is hoisted out of the unit loop
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NN = N * N, PL = E::plane(N);
  const int row = 16 * wave + (lane & 15);
  const bool rok = row < N;
  T* Ar = reinterpret_cast<T*>(smem);  // A_k (unscaled)
  T* Ai = Ar + PL;
  T* Br = Ai + PL;  // A2 (scaled)
  T* Bi = Br + PL;
  T* Xr = Bi + PL;  // A3 (scaled), then the squaring operand (ping-pong with A)
  T* Xi = Xr + PL;
  float* colf = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(Xi + PL + 16));

  auto mask_own = [&](Own& X) __attribute__((always_inline)) { E::mask_cols(N, X, lane); };
  QOC_STAMP(0);
  QOC_RTSTAMP(60);
  QOC_LIFE(0);
  // ---- own rows of A_k (src/gradient_computations.jl:18-22), straight from HBM/L2 ----
  Own V;
  {
    // all loads of one generator in flight together (generator-major order)
    const size_t r0 = (size_t)min(row, N - 1);
    const cx<T>* src = Agen ? Agen : Ain + (size_t)unit * NN;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const cx<T> a = src[r0 + (size_t)N * min(16 * t + M::drow(lane, e), N - 1)];
        V.r[t][e] = a.r;
        V.i[t][e] = a.i;
      }
    if (Agen) {
      const double* uu = u + (size_t)unit * nu;
      for (int j = 0; j < nu; ++j) {
        const T uj = (T)uu[j];
        const cx<T>* G = Agen + (size_t)(j + 1) * NN;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const cx<T> g = G[r0 + (size_t)N * min(16 * t + M::drow(lane, e), N - 1)];
            V.r[t][e] += uj * g.r;
            V.i[t][e] += uj * g.i;
          }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = rok && 16 * t + M::drow(lane, e) < N;
        V.r[t][e] = ok ? V.r[t][e] : T(0);
        V.i[t][e] = ok ? V.i[t][e] : T(0);
      }
  }
  QOC_STAMP(1);
  E::store_own(N, V, Ar, Ai, row, lane);

  // ---- ||A_k||_1 (selects (r, s) only): an fp32 upper bound, column sums over this wave's 16 rows
  // by DPP, then over waves through LDS; every wave reduces redundantly (one barrier) ----
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xr = (float)V.r[t][e], xi = (float)V.i[t][e];
      const float cs = dpp_sum16(sqrtf(xr * xr + xi * xi));
      if ((lane & 15) == 0) colf[wave * E::NMAX + 16 * t + M::drow(lane, e)] = cs;
    }
  __syncthreads();
  double nA;
  {
    float c = 0.f;
    if (lane < N) {
#pragma unroll
      for (int w = 0; w < NT; ++w) c += colf[w * E::NMAX + lane];
    }
    // the fp32 sqrt / sums are within 2^-17 relative for N <= 64: the scaled value bounds ||A||_1
    nA = (double)__uint_as_float(wave_max_u32(__float_as_uint(c))) * (1.0 + 1.0 / 65536.0);
  }

  QOC_STAMP(2);
  // ---- T12 = Taylor degree 12 in 4 products (kT12, qoc_expm.hpp) with s squarings; when T12 would
  // need >= 3 squarings (||A||_1 > 4 theta_12), Paterson-Stockmeyer degree 3r+2 instead (taylor_select:
  // about the same GEMM count, fewer squarings, so 2^s times less rounding growth) ----
  int ts = 0;
  if (nA > kTheta12) ts = (int)ceil(log2(nA / kTheta12));
  int tr = 0;  // 0: T12; 2..8: Paterson-Stockmeyer r
  // MODE 0: T12 only (A2 / A3 from registers), larger norms listed for the Paterson-Stockmeyer pass;
  // MODE 1: Paterson-Stockmeyer only (the listed units); MODE 2: both inline (T12 reading A2 / A3 back
  // from LDS, so that no register state crosses the algorithm branch).
  if (MODE == 0) {
    if (ts >= 3) {
      if (tid == 0) ps_list[atomicAdd(ps_count, 1)] = unit;
      return;
    }
  } else if (MODE == 1 || ts >= 3) {
    taylor_select(nA, tr, ts);
  }
  tr = __builtin_amdgcn_readfirstlane(tr);
  ts = __builtin_amdgcn_readfirstlane(ts);
  if (tid == 0) {
    int d, sq = 0;
    if (nA <= 2.1) {
      d = nA > 0.95 ? 9 : nA > 0.25 ? 7 : nA > 0.015 ? 5 : 3;
    } else {
      d = 13;
      const double s = log2(nA / 5.4);
      sq = s > 0 ? (int)ceil(s) : 0;
    }
    if (hist) atomicAdd(&hist[degree_index(d) * 64 + (sq < 63 ? sq : 63)], 1ULL);
    if (thist) atomicAdd(&thist[(tr ? tr - 2 : kT12Row) * 64 + (ts < 63 ? ts : 63)], 1ULL);
  }
  const T sc = (T)ldexp(1.0, -ts);  // exact power-of-two scaling

  // As = 2^-s A (owned); A2 = As As = 2^-s (As A); A3 = A2 As = 2^-s (A2 A)   [products 1, 2]
  Own Z, W, V3;
  E::zero(Z);
  E::scale(V, sc);
  E::template rmul<KS>(N, V, Ar, Ai, W, Z, lane);
  E::scale(W, sc);
  E::template rmul<KS>(N, W, Ar, Ai, V3, Z, lane);
  E::scale(V3, sc);

  // Paterson-Stockmeyer pass: A3 -> buffer 3 (row-major, its operand), A2 -> buffer 2 at the owned
  // rows (read back by make_Bps).  The T12 pass uses A2 / A3 from registers.
  if constexpr (MODE != 0) {
    E::store_own(N, V3, Xr, Xi, row, lane);
    E::store_own(N, W, Br, Bi, row, lane);
  }
  const int ra = min(row, N - 1) * E::ldp(N);  // owned row; columns >= N read junk that reaches only
                                                // result columns >= N (masked by rmul)
  // Park / fetch an owned matrix at its own (row-major) positions; only the writing lane reads it back.
  auto get = [&](Own& X, const T* Pr, const T* Pi) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = 16 * t + M::drow(lane, e);
        const bool ok = rok && (t < NT - 1 || col < N);
        const int a = ra + min(col, N - 1);
        const T xr = Pr[a], xi = Pi[a];
        X.r[t][e] = ok ? xr : T(0);
        X.i[t][e] = ok ? xi : T(0);
      }
  };
  QOC_STAMP(3);
  if constexpr (MODE == 0) {
    // ---- T12: B_j = x_j0 I + x_j1 As + x_j2 A2 + x_j3 A3 at the owned positions (As from buffer 1,
    // A2 / A3 from registers); B4 -> buffer 2 and B2 -> buffer 3 over this lane's own rows ----
    auto make_B = [&](const double* x, Own& B) __attribute__((always_inline)) {
      const T x0 = (T)x[0], x1 = (T)x[1] * sc, x2 = (T)x[2], x3 = (T)x[3];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = 16 * t + M::drow(lane, e);
          const int a = ra + col;
          const T br = x1 * Ar[a] + x2 * W.r[t][e] + x3 * V3.r[t][e] + (row == col ? x0 : T(0));
          const T bi = x1 * Ai[a] + x2 * W.i[t][e] + x3 * V3.i[t][e];
          B.r[t][e] = rok ? br : T(0);
          B.i[t][e] = rok ? bi : T(0);
        }
    };
    Own B4, B3;
    make_B(kT12[3], B4);
    mask_own(B4);
    E::store_own(N, B4, Br, Bi, row, lane);  // B4 -> buffer 2 (operand of product 3)
    {
      Own B2;
      make_B(kT12[1], B2);
      E::store_own(N, B2, Xr, Xi, row, lane);  // B2 -> buffer 3 (own positions)
    }
    make_B(kT12[2], B3);
    Own B1;
    make_B(kT12[0], B1);
    QOC_STAMP(10);
    __syncthreads();                                    // A (buffer 1) readers done, buffer 2 = B4 complete
    QOC_STAMP(11);
    E::store_own(N, B1, Ar, Ai, row, lane);             // B1 -> buffer 1 (own positions)
    E::template rmul<KS>(N, B4, Br, Bi, V, B3, lane);  // A6 = B3 + B4 B4   [product 3]
    QOC_STAMP(12);
    // A6 -> buffer 3 over this wave's B2 rows (read back first; other waves only touch their own rows
    // of buffer 3 until the barrier), so buffer 2 (B4, still read by product 3 elsewhere) stays intact
    get(W, Xr, Xi);                                     // B2
    E::store_own(N, V, Xr, Xi, row, lane);              // A6 -> buffer 3
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      W.r[t] += V.r[t];
      W.i[t] += V.i[t];
    }
    get(B1, Ar, Ai);
    QOC_STAMP(14);
    __syncthreads();                                    // buffer 3 = A6 complete
    QOC_STAMP(15);
    E::template rmul<KS>(N, W, Xr, Xi, V, B1, lane);  // T12 = B1 + (B2 + A6) A6   [product 4]
    QOC_STAMP(16);
  } else if (MODE == 2 && !tr) {
    // ---- T12 with A2 / A3 read back from LDS: one pass over the owned positions, B4 -> buffer 2 and
    // B2 -> buffer 3 in place of this lane's A2 / A3, B3 and B1 in registers ----
    Own B4, B3, B1;
    {
      const double* x1 = kT12[0];
      const double* x2 = kT12[1];
      const double* x3 = kT12[2];
      const double* x4 = kT12[3];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = 16 * t + M::drow(lane, e);
          const int a = ra + col;
          const T pr = Ar[a] * sc, pi = Ai[a] * sc, qr = Br[a], qi = Bi[a], wr = Xr[a], wi = Xi[a];
          const bool dg = row == col;
          auto comb = [&](const double* x, T& br, T& bi) __attribute__((always_inline)) {
            br = (T)x[1] * pr + (T)x[2] * qr + (T)x[3] * wr + (dg ? (T)x[0] : T(0));
            bi = (T)x[1] * pi + (T)x[2] * qi + (T)x[3] * wi;
            br = rok ? br : T(0);
            bi = rok ? bi : T(0);
          };
          T r4, i4, r2, i2, r3, i3, r1, i1;
          comb(x4, r4, i4);
          comb(x2, r2, i2);
          comb(x3, r3, i3);
          comb(x1, r1, i1);
          B4.r[t][e] = r4;
          B4.i[t][e] = i4;
          B3.r[t][e] = r3;
          B3.i[t][e] = i3;
          B1.r[t][e] = r1;
          B1.i[t][e] = i1;
          if (rok && (t < NT - 1 || col < N)) {  // same positions this lane just read
            Br[a] = r4;
            Bi[a] = i4;
            Xr[a] = r2;
            Xi[a] = i2;
          }
        }
    }
    mask_own(B4);
    mask_own(B3);
    mask_own(B1);
    __syncthreads();                                    // A (buffer 1) readers done, buffer 2 = B4 complete
    E::store_own(N, B1, Ar, Ai, row, lane);             // B1 -> buffer 1 (own positions)
    E::template rmul<KS>(N, B4, Br, Bi, V, B3, lane);  // A6 = B3 + B4 B4   [product 3]
    __syncthreads();                                    // buffer 2 (B4) readers are done
    E::store_own(N, V, Br, Bi, row, lane);              // A6 -> buffer 2
    get(W, Xr, Xi);                                     // B2
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      W.r[t] += V.r[t];
      W.i[t] += V.i[t];
    }
    get(B1, Ar, Ai);
    __syncthreads();
    E::template rmul<KS>(N, W, Br, Bi, V, B1, lane);  // T12 = B1 + (B2 + A6) A6   [product 4]
  } else {
    // ---- Paterson-Stockmeyer: V <- V A3 + B_i, B_i = c_3i I + c_3i+1 As + c_3i+2 A2 (A3 the LDS operand,
    // As / A2 read back at the owned positions), barrier-free Horner ----
    __syncthreads();  // buffer 3 complete
    auto make_Bps = [&](int i, Own& B) __attribute__((always_inline)) {
      const T c0 = (T)kInvFact[3 * i], c1 = (T)kInvFact[3 * i + 1] * sc, c2 = (T)kInvFact[3 * i + 2];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = 16 * t + M::drow(lane, e);
          const int a = ra + col;
          const T br = c1 * Ar[a] + c2 * Br[a] + (row == col ? c0 : T(0));
          const T bi = c1 * Ai[a] + c2 * Bi[a];
          B.r[t][e] = rok ? br : T(0);
          B.i[t][e] = rok ? bi : T(0);
        }
    };
    Own Bx;
    make_Bps(tr, V);
    for (int i = tr - 1; i >= 0; --i) {
      make_Bps(i, Bx);
      E::template rmul<KS>(N, V, Xr, Xi, V, Bx, lane);  // = A3 V + B_i (polynomials in A commute)
    }
  }
  // ---- squarings: ping-pong buffers 3 / 1, one barrier each, plus one first (the last product may still
  // be reading buffer 3 in other waves) ----

  QOC_STAMP(4);
  if (ts > 0) __syncthreads();
  for (int q = 0; q < ts; ++q) {
    T* Sr = (q & 1) ? Ar : Xr;
    T* Si = (q & 1) ? Ai : Xi;
    E::store_own(N, V, Sr, Si, row, lane);
    __syncthreads();
    E::template rmul<KS>(N, V, Sr, Si, V, Z, lane);
  }

  QOC_STAMP(5);
  // ---- U_k -> HBM, column-major (Julia layout) ----
  if (rok) {
    cx<T>* out = Uout + (size_t)unit * NN;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = 16 * t + M::drow(lane, e);
        if (col < N) out[row + (size_t)N * col] = cx<T>{V.r[t][e], V.i[t][e]};
      }
  }
  QOC_STAMP(6);
  QOC_RTSTAMP(61);
  QOC_LIFE(1);
}


// ALG 1 (Taylor), two passes.  Pass 0 (MODE 0): one workgroup per unit; slices with ||A_k||_1 <= 4 theta_12
// run T12 (+ <= 2 squarings), the others are appended to ps_list.  Pass 1 (MODE 1): one workgroup per
// listed slice runs Paterson-Stockmeyer (taylor_select).  k_expm_rr_mix does both inline in one pass
// (T12 reading A2 / A3 back from LDS); the engine launches it when the norms are large anyway
// (||A_0||_1 > 4 theta_12), saving pass 0's A_k loads and norms on every slice.  Units are either generators
// (Agen, u) or explicit matrices (Ain).  hist: the Padé (d, s) the reference would select; thist: the
// executed Taylor (r, s) / T12 s.  KS: k-steps per product (see ExpmRR::rows).
template <typename T, int NT, int KS>
__global__ __launch_bounds__(64 * NT, 2) void k_expm_rr(int N, int nu, int nunits, const cx<T>* __restrict__ Agen,
                                                        const double* __restrict__ u, const cx<T>* __restrict__ Ain,
                                                        cx<T>* __restrict__ Uout, unsigned long long* __restrict__ hist,
                                                        unsigned long long* __restrict__ thist, int* __restrict__ ps_list,
                                                        int* __restrict__ ps_count) {
  const int unit = blockIdx.x;
  if (unit >= nunits) return;
  expm_rr_unit<T, NT, KS, 0>(unit, N, nu, Agen, u, Ain, Uout, hist, thist, ps_list, ps_count);
}
template <typename T, int NT, int KS>
__global__ __launch_bounds__(64 * NT, 2) void k_expm_rr_mix(int N, int nu, int nunits, const cx<T>* __restrict__ Agen,
                                                            const double* __restrict__ u, const cx<T>* __restrict__ Ain,
                                                            cx<T>* __restrict__ Uout, unsigned long long* __restrict__ hist,
                                                            unsigned long long* __restrict__ thist) {
  const int unit = blockIdx.x;
  if (unit >= nunits) return;
  expm_rr_unit<T, NT, KS, 2>(unit, N, nu, Agen, u, Ain, Uout, hist, thist, nullptr, nullptr);
}
template <typename T, int NT, int KS>
__global__ __launch_bounds__(64 * NT, 2) void k_expm_rr_ps(int N, int nu, const cx<T>* __restrict__ Agen,
                                                           const double* __restrict__ u, const cx<T>* __restrict__ Ain,
                                                           cx<T>* __restrict__ Uout, unsigned long long* __restrict__ hist,
                                                           unsigned long long* __restrict__ thist,
                                                           const int* __restrict__ ps_list, const int* __restrict__ ps_count) {
  // one workgroup per listed unit (grid = nunits; workgroups past the count exit at once — cheaper than a
  // persistent loop, which serialises the phases of consecutive units)
  const int i = blockIdx.x;
  if (i >= *ps_count) return;
  expm_rr_unit<T, NT, KS, 1>(ps_list[i], N, nu, Agen, u, Ain, Uout, hist, thist, nullptr, nullptr);
}

}  // namespace qoc
