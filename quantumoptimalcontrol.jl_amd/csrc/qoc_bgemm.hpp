// qoc_bgemm.hpp — kernels of the large-N (HBM-resident) path: batched complex GEMM on MFMA with a
// fused multi-term epilogue, plus the element-wise and reduction kernels around it.
//
// Used when N exceeds the LDS-resident envelope of k_expm / k_chain_* (e.g. the synthetic N = 256
// fp32 configuration).  Everything is a batch of independent complex
// matrices in the engine's HBM layout (column-major, interleaved re/im).  A batch item locates
// each operand through an affine "unit map" (Opd), so the same GEMM serves
//   - per-slice Padé products   (item = slice in a chunk, workspace stride),
//   - chain steps               (item = seed b at fixed slice k: U[b,k], x[b,k]),
//   - gradient products         (item = slice unit b*Nt+k: x_k, λ_{k+1} live at (Nt+1)-strided slots).
#pragma once
#include "qoc_common.hpp"

namespace qoc {

// Operand address: base + (v / per) * outer + (v % per) * inner, v = item + u0 (per <= 0: v * inner).
struct Opd {
  const void* p = nullptr;
  long long outer = 0, inner = 0;
  int per = 0, u0 = 0;
};

template <typename T>
__device__ __forceinline__ const cx<T>* opd_ptr(const Opd& o, int item) {
  const long long v = (long long)item + o.u0;
  long long off;
  if (o.per > 0) {
    const long long q = v / o.per;
    off = q * o.outer + (v - q * o.per) * o.inner;
  } else {
    off = v * o.inner;
  }
  return reinterpret_cast<const cx<T>*>(o.p) + off;
}

constexpr int BG_BM = 64, BG_BN = 64, BG_BK = 16, BG_THREADS = 256;

// C1 = alpha1 * op(A) op(B) + sum_t w1[t] Y_t + gamma1 I
// C2 = alpha2 * op(A) op(B) + sum_t w2[t] Y_t + gamma2 I          (optional)
// sumsq (optional): sumsq[item] += ||C1||_F^2 (Newton-Schulz residual bound, ||R||_2 <= ||R||_F).
struct GemmArgs {
  Opd A, B, C1, C2, Y[3];
  int nY;
  int M, K, Ncol;  // op(A): M x K, op(B): K x Ncol
  int nitems, tiles_m, tiles;
  double alpha1, alpha2, gamma1, gamma2;
  double w1[3], w2[3];
  double* sumsq;
};

// LDS operand layouts: "k-major" [k][row] when the global operand is contiguous along rows,
// "row-major" [row][k] when it is contiguous along k.  Padding spreads MFMA fragment reads over banks.
template <bool KMAJOR>
struct LdsLay;
template <>
struct LdsLay<true> {
  static constexpr int SIZE = BG_BK * (BG_BM + 4);
  static __device__ __forceinline__ int at(int k, int r) { return k * (BG_BM + 4) + r; }
};
template <>
struct LdsLay<false> {
  static constexpr int SIZE = BG_BM * (BG_BK + 1);
  static __device__ __forceinline__ int at(int k, int r) { return r * (BG_BK + 1) + k; }
};

// OPA: 0 -> op(A) = A (stored M x K, contiguous along rows); 1 -> A^H (stored K x M, contiguous along k)
// OPB: 0 -> op(B) = B (stored K x Ncol, contiguous along k); 1 -> B^H (stored Ncol x K, contiguous along cols)
template <typename T, int OPA, int OPB>
__global__ __launch_bounds__(BG_THREADS) void k_bgemm(GemmArgs g) {
  using MFT = MF<T>;
  using v4 = typename MFT::v4;
  using LA = LdsLay<OPA == 0>;
  using LB = LdsLay<OPB == 1>;
  __shared__ T As[2][2][LA::SIZE];
  __shared__ T Bs[2][2][LB::SIZE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // XCD-aware order: consecutive workgroups are dispatched round-robin over the 8 XCDs; give each
  // XCD a contiguous range of (item, tile) so that one item's tiles share an L2.
  const int L = blockIdx.x;
  const int total = g.nitems * g.tiles;
  const int lin = (total & 7) == 0 ? (L & 7) * (total >> 3) + (L >> 3) : L;
  const int item = lin / g.tiles, tile = lin - item * g.tiles;
  const int tm = tile % g.tiles_m, tn = tile / g.tiles_m;
  const int row0 = tm * BG_BM, col0 = tn * BG_BN;
  const cx<T>* Ab = opd_ptr<T>(g.A, item);
  const cx<T>* Bb = opd_ptr<T>(g.B, item);
  const int M = g.M, K = g.K, NC = g.Ncol;

  cx<T> ra[4], rb[4];
#define QOC_BG_LOAD(K0)                                                                      \
  do {                                                                                       \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                          \
      const int e = tid + BG_THREADS * r;                                                    \
      const int ka = OPA ? (e & 15) : (e >> 6), ia = OPA ? (e >> 4) : (e & 63);              \
      const int gr = row0 + ia, gk = (K0) + ka;                                              \
      const bool oka = gr < M && gk < K;                                                     \
      const size_t oa = OPA ? (size_t)(oka ? gk : 0) + (size_t)K * (oka ? gr : 0)            \
                            : (size_t)(oka ? gr : 0) + (size_t)M * (oka ? gk : 0);           \
      cx<T> va = Ab[oa];                                                                     \
      if (OPA) va.i = -va.i;                                                                 \
      ra[r] = oka ? va : cx<T>{0, 0};                                                        \
      const int kb = OPB ? (e >> 6) : (e & 15), jb = OPB ? (e & 63) : (e >> 4);              \
      const int gc = col0 + jb, gkb = (K0) + kb;                                             \
      const bool okb = gc < NC && gkb < K;                                                   \
      const size_t ob = OPB ? (size_t)(okb ? gc : 0) + (size_t)NC * (okb ? gkb : 0)          \
                            : (size_t)(okb ? gkb : 0) + (size_t)K * (okb ? gc : 0);          \
      cx<T> vb = Bb[ob];                                                                     \
      if (OPB) vb.i = -vb.i;                                                                 \
      rb[r] = okb ? vb : cx<T>{0, 0};                                                        \
    }                                                                                        \
  } while (0)
#define QOC_BG_STORE(BUF)                                                                    \
  do {                                                                                       \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                          \
      const int e = tid + BG_THREADS * r;                                                    \
      const int ka = OPA ? (e & 15) : (e >> 6), ia = OPA ? (e >> 4) : (e & 63);              \
      As[BUF][0][LA::at(ka, ia)] = ra[r].r;                                                  \
      As[BUF][1][LA::at(ka, ia)] = ra[r].i;                                                  \
      const int kb = OPB ? (e >> 6) : (e & 15), jb = OPB ? (e & 63) : (e >> 4);              \
      Bs[BUF][0][LB::at(kb, jb)] = rb[r].r;                                                  \
      Bs[BUF][1][LB::at(kb, jb)] = rb[r].i;                                                  \
    }                                                                                        \
  } while (0)

  v4 cr[2][2], ci[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      cr[x][y] = v4{0, 0, 0, 0};
      ci[x][y] = v4{0, 0, 0, 0};
    }
  const int wr = (wave & 1) * 32, wc = (wave >> 1) * 32;
  const int li = lane & 15, kq = lane >> 4;
  const int nslab = (K + BG_BK - 1) / BG_BK;
  QOC_BG_LOAD(0);
  QOC_BG_STORE(0);
  __syncthreads();
  for (int s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    if (s + 1 < nslab) QOC_BG_LOAD((s + 1) * BG_BK);
#pragma unroll
    for (int kk = 0; kk < BG_BK; kk += 4) {
      T ar[2], ai[2], br[2], bi[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        ar[x] = As[buf][0][LA::at(kk + kq, wr + 16 * x + li)];
        ai[x] = As[buf][1][LA::at(kk + kq, wr + 16 * x + li)];
      }
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        br[y] = Bs[buf][0][LB::at(kk + kq, wc + 16 * y + li)];
        bi[y] = Bs[buf][1][LB::at(kk + kq, wc + 16 * y + li)];
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          cr[x][y] = MFT::mma(ar[x], br[y], cr[x][y]);
          ci[x][y] = MFT::mma(ar[x], bi[y], ci[x][y]);
        }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          cr[x][y] = MFT::mma(-ai[x], bi[y], cr[x][y]);
          ci[x][y] = MFT::mma(ai[x], br[y], ci[x][y]);
        }
    }
    if (s + 1 < nslab) QOC_BG_STORE(buf ^ 1);
    __syncthreads();
  }
#undef QOC_BG_LOAD
#undef QOC_BG_STORE

  // ---- fused epilogue ----
  cx<T>* C1 = const_cast<cx<T>*>(opd_ptr<T>(g.C1, item));
  cx<T>* C2 = g.C2.p ? const_cast<cx<T>*>(opd_ptr<T>(g.C2, item)) : nullptr;
  const cx<T>* Y0 = g.nY > 0 ? opd_ptr<T>(g.Y[0], item) : nullptr;
  const cx<T>* Y1 = g.nY > 1 ? opd_ptr<T>(g.Y[1], item) : nullptr;
  const cx<T>* Y2 = g.nY > 2 ? opd_ptr<T>(g.Y[2], item) : nullptr;
  double mx = 0.0;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int col = col0 + wc + 16 * y + li;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = row0 + wr + 16 * x + MFT::drow(lane, i);
        if (row < M && col < NC) {
          const size_t o = row + (size_t)M * col;
          const double pr = cr[x][y][i], pi = ci[x][y][i];
          double r1 = g.alpha1 * pr, i1 = g.alpha1 * pi;
          double r2 = g.alpha2 * pr, i2 = g.alpha2 * pi;
          if (Y0) { const cx<T> v = Y0[o]; r1 += g.w1[0] * v.r; i1 += g.w1[0] * v.i; r2 += g.w2[0] * v.r; i2 += g.w2[0] * v.i; }
          if (Y1) { const cx<T> v = Y1[o]; r1 += g.w1[1] * v.r; i1 += g.w1[1] * v.i; r2 += g.w2[1] * v.r; i2 += g.w2[1] * v.i; }
          if (Y2) { const cx<T> v = Y2[o]; r1 += g.w1[2] * v.r; i1 += g.w1[2] * v.i; r2 += g.w2[2] * v.r; i2 += g.w2[2] * v.i; }
          if (row == col) {
            r1 += g.gamma1;
            r2 += g.gamma2;
          }
          C1[o] = cx<T>{(T)r1, (T)i1};
          if (C2) C2[o] = cx<T>{(T)r2, (T)i2};
          mx += r1 * r1 + i1 * i1;
        }
      }
    }
  if (g.sumsq) {
    for (int off = 32; off > 0; off >>= 1) mx += __shfl_xor(mx, off);
    if (lane == 0) atomicAdd(g.sumsq + item, mx);
  }
}

// ---------------------------------------------------------------------------------------------
// Element-wise kernels
// ---------------------------------------------------------------------------------------------

// Out_item = sum_{t < nt} w_t Y_t,item + dI * I   (rows x cols per item, leading dimension rows).
struct LinArgs {
  Opd out, Y[4];
  double w[4];
  int nt, rows, cols, nitems;
  double dI;
};

template <typename T>
__global__ void k_lincomb(LinArgs a) {
  const size_t per = (size_t)a.rows * a.cols;
  const size_t total = per * a.nitems;
  for (size_t gi = blockIdx.x * (size_t)blockDim.x + threadIdx.x; gi < total; gi += (size_t)gridDim.x * blockDim.x) {
    const int it = (int)(gi / per);
    const size_t e = gi - (size_t)it * per;
    double r = 0, im = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < a.nt) {
        const cx<T> v = opd_ptr<T>(a.Y[t], it)[e];
        r += a.w[t] * v.r;
        im += a.w[t] * v.i;
      }
    }
    if (a.dI != 0.0 && (int)(e % a.rows) == (int)(e / a.rows)) r += a.dI;
    const_cast<cx<T>*>(opd_ptr<T>(a.out, it))[e] = cx<T>{(T)r, (T)im};
  }
}

// A_unit = A0 + sum_j u[unit, j] A_j for units [unit0, unit0 + count) -> out (count x N x N), and the
// 1-norm (max column sum of |a_ij|) of each, max-reduced into *nmax.  One workgroup per slice;
// each wave owns whole columns (coalesced column reads, shuffle reduction).
template <typename T>
__global__ __launch_bounds__(256) void k_form_norm(int N, int nu, long long unit0, const cx<T>* __restrict__ Agen,
                                                   const double* __restrict__ u, cx<T>* __restrict__ out,
                                                   unsigned long long* __restrict__ nmax) {
  const int it = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t NN = (size_t)N * N;
  const long long unit = unit0 + it;
  T uj[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) uj[j] = j < nu ? (T)u[unit * nu + j] : T(0);
  cx<T>* ob = out + (size_t)it * NN;
  double best = 0.0;
  for (int c = wave; c < N; c += 4) {
    double s = 0.0;
    for (int r = lane; r < N; r += 64) {
      const size_t e = r + (size_t)N * c;
      cx<T> a = Agen[e];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j < nu) {
          const cx<T> v = Agen[(size_t)(j + 1) * NN + e];
          a.r += uj[j] * v.r;
          a.i += uj[j] * v.i;
        }
      }
      ob[e] = a;
      s += sqrt((double)a.r * a.r + (double)a.i * a.i);
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    best = fmax(best, s);
  }
  if (lane == 0 && nmax) atomicMax(nmax, (unsigned long long)__double_as_longlong(best));
}

// λ_N = coef_b * Xt (trace cost) written to Lam[b][Nt] for all seeds.
template <typename T>
__global__ void k_lambda_final(int N, int m, int Nt, int B, const cx<T>* __restrict__ Xt,
                               const cx<double>* __restrict__ coef, cx<T>* __restrict__ Lam) {
  const size_t Nm = (size_t)N * m;
  for (size_t gi = blockIdx.x * (size_t)blockDim.x + threadIdx.x; gi < Nm * B; gi += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(gi / Nm);
    const size_t o = gi - (size_t)b * Nm;
    const cx<double> cf = coef[(size_t)b * m + o / N];
    const cx<T> t = Xt[o];
    Lam[((size_t)b * (Nt + 1) + Nt) * Nm + o] =
        cx<T>{(T)(cf.r * t.r - cf.i * t.i), (T)(cf.r * t.i + cf.i * t.r)};
  }
}

// Trace cost on x_N for every seed (one workgroup per seed): J = 1 - |tr(Xt' x_N)|^2 / n^2, added to
// J[b] when accumulate != 0 (penalty already stored there); coef = -2 tr(Xt' x_N) / n^2 per column.
template <typename T>
__global__ void k_trace_cost(int N, int m, int Nt, const cx<T>* __restrict__ X, const cx<T>* __restrict__ Xt,
                             double n_norm, int accumulate, double* __restrict__ J, cx<double>* __restrict__ coef) {
  __shared__ double red[8];
  const int b = blockIdx.x;
  const size_t Nm = (size_t)N * m;
  const cx<T>* xN = X + ((size_t)b * (Nt + 1) + Nt) * Nm;
  double orr = 0, oii = 0;
  for (size_t o = threadIdx.x; o < Nm; o += blockDim.x) {
    const cx<T> t = Xt[o], v = xN[o];
    orr += (double)t.r * v.r + (double)t.i * v.i;
    oii += (double)t.r * v.i - (double)t.i * v.r;
  }
  orr = block_sum(orr, red);
  oii = block_sum(oii, red);
  if (threadIdx.x == 0) {
    const double n2 = n_norm * n_norm;
    const double j = 1.0 - (orr * orr + oii * oii) / n2;
    J[b] = accumulate ? J[b] + j : j;
    for (int c = 0; c < m; ++c) coef[(size_t)b * m + c] = cx<double>{-2.0 * orr / n2, -2.0 * oii / n2};
  }
}

// Guard-state penalty over all stored states: J[b] = mu * sum_{k, masked} |x_k|^2 (one WG per seed).
template <typename T>
__global__ void k_penalty_sum(int N, int m, int Nt, const cx<T>* __restrict__ X, const unsigned char* __restrict__ pmask,
                              double mu, double* __restrict__ J) {
  __shared__ double red[8];
  const int b = blockIdx.x;
  const size_t Nm = (size_t)N * m;
  const cx<T>* Xb = X + (size_t)b * (Nt + 1) * Nm;
  double s = 0.0;
  for (size_t gi = threadIdx.x; gi < (size_t)(Nt + 1) * Nm; gi += blockDim.x) {
    if (pmask[gi % Nm]) {
      const cx<T> v = Xb[gi];
      s += (double)v.r * v.r + (double)v.i * v.i;
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) J[b] = mu * s;
}

// λ_k[b] += 2 mu mask .* x_k[b] for one slice index k, all seeds.
template <typename T>
__global__ void k_penalty_grad(int N, int m, int Nt, int B, int k, const cx<T>* __restrict__ X,
                               const unsigned char* __restrict__ pmask, double two_mu, cx<T>* __restrict__ Lam) {
  const size_t Nm = (size_t)N * m;
  for (size_t gi = blockIdx.x * (size_t)blockDim.x + threadIdx.x; gi < Nm * B; gi += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(gi / Nm);
    const size_t o = gi - (size_t)b * Nm;
    if (!pmask[o]) continue;
    const size_t at = ((size_t)b * (Nt + 1) + k) * Nm + o;
    const cx<T> x = X[at];
    cx<T> l = Lam[at];
    l.r += (T)two_mu * x.r;
    l.i += (T)two_mu * x.i;
    Lam[at] = l;
  }
}

// dJdu[unit, j] = sum_{p,q} Re(A_j[p,q] conj(M'[p,q])) with M' = W P^H (one WG per slice in the chunk).
// This is Re tr(A_j P W^H) = sum_{a+b<=o-1} Re<(X^H)^b λ, A_j X^a x>/(a+b+1)!.
template <typename T>
__global__ __launch_bounds__(256) void k_gen_contract(int N, int nu, long long unit0, const cx<T>* __restrict__ Agen,
                                                      const cx<T>* __restrict__ Mp, double* __restrict__ dJdu) {
  __shared__ double red[8];
  const int it = blockIdx.x;
  const size_t NN = (size_t)N * N;
  const cx<T>* Mb = Mp + (size_t)it * NN;
  double acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.0;
  for (size_t e = threadIdx.x; e < NN; e += blockDim.x) {
    const cx<T> mv = Mb[e];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < nu) {
        const cx<T> a = Agen[(size_t)(j + 1) * NN + e];
        acc[j] += (double)a.r * mv.r + (double)a.i * mv.i;
      }
    }
  }
  const long long unit = unit0 + it;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j < nu) {
      const double s = block_sum(acc[j], red);
      if (threadIdx.x == 0) dJdu[unit * nu + j] = s;  // u layout: b*nu*Nt + k*nu + j == unit*nu + j
    }
  }
}

}  // namespace qoc
