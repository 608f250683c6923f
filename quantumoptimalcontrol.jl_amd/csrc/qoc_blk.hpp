// qoc_blk.hpp — generators with small invariant blocks: the chains and the order-o gradient block by block.
//
// When A_0, A_1, ..., A_nu share one block-diagonal pattern up to a permutation of the basis (the connected
// components of the graph with an edge {i, k} whenever some A_j[i, k] != 0), every slice generator
// A_k = A_0 + Σ_j u_jk A_j has that pattern, and so do exp(A_k) (a power series in A_k) and every term of
// expm_jacobian! (products of A_k and A_j, src/gradient_computations.jl:177-213).  The reference's dense steps
//   x_{k+1} = exp(A_k) x_k                          (:17-29)
//   λ_k = exp(A_k)^H λ_{k+1} (+ dL/dx(x_k))          (:52-58)
//   dJdu[k, j] = Re Σ_cols λ_{k+1}^H dU_kj x_k       (:65-74, 217-223)
// therefore split exactly into independent products on each block: the entries outside the blocks are zero in
// every factor, so they add exact zeros.  The cavity-qubit system (qubit drive ⊗ cavity, dispersive H_0) has
// 20 blocks of 2, the zz-coupling system (a drive on one transmon) 3 blocks of 3.
//
// The chains keep the Taylor-action scheme of qoc_tchain.hpp unchanged — the same step records (P, s, e^{μ_k},
// operand scale, Chebyshev coefficients) from k_tchain_prep / k_tchain_prep_cheb and the same shifted
// generators Ã_j = A_j - μ_j I (a multiple of the identity shifts every block alike) — so the polynomial in
// Ã_k applied to each block is the dense chains' polynomial restricted to the block.  Each lane owns one
// (block, state column) pair: its NB-element slice of the state and the NB x NB block of every generator sit
// in registers, and a Chebyshev / Taylor term is an NB x NB complex matvec in VALU registers with no exchange
// between lanes.  One workgroup per seed (per seed and direction in the dual launch).  The serial chain per
// seed drops from Σ P_k dense N x N x m products to Σ P_k products of NB x NB, and the states go to HBM in the
// caller's layout, so the costs, qoc_get_states / qoc_get_costates and every other gradient kernel read them
// unchanged.
#pragma once
#include "qoc_tchain.hpp"

namespace qoc {

constexpr int BLK_NBMAX = 4;  // largest block the register-resident lanes take
constexpr int BLK_MAXT = 256;  // lanes (blocks x columns) per workgroup
constexpr int BLK_ORDMAX = 4;  // expm_jacobian! orders 1..4

struct BlkArgs {
  const int* brow;         // nblk x NB: rows (= columns) of each block in increasing order, -1 padding
  const void* A;           // (nu+1) x N x N unshifted generators (the gradient's A_k and A_j)
  int nblk;
  const int* wrow;         // MFMA block waves: nwb x 16 rows of each wave's state (-1 padding)
  int nwb;
};

// This lane's (block, column) pair: lane l < nblk m owns block l % nblk of column l / nblk, so that the lanes of
// one column read consecutive rows of every block.
template <int NB>
struct BlkLane {
  int r[NB];  // rows of the block (-1: padding)
  int c;      // state column
  __device__ __forceinline__ void setup(const BlkArgs& bk, int m, int l) {
    const bool act = l < bk.nblk * m;
    const int beta = act ? l % bk.nblk : 0;
    c = act ? l / bk.nblk : 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) r[i] = act ? bk.brow[beta * NB + i] : -1;
  }
};

// The block of Ã_j (j <= nu <= 2; HERM: of Ã_j^H, the backward chain's) at this lane's rows, zero outside.
template <int NB, bool HERM>
__device__ __forceinline__ void blk_load_gen(const cx<double>* __restrict__ At, int N, int nu, const int (&r)[NB],
                                             double (&gr)[3][NB][NB], double (&gi)[3][NB][NB]) {
  const size_t NN = (size_t)N * N;
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const bool ok = j <= nu && r[i] >= 0 && r[k] >= 0;
        const int ri = max(r[i], 0), rk = max(r[k], 0);
        const cx<double> v = At[(size_t)min(j, nu) * NN + (HERM ? rk + (size_t)N * ri : ri + (size_t)N * rk)];
        gr[j][i][k] = ok ? v.r : 0.0;
        gi[j][i][k] = ok ? (HERM ? -v.i : v.i) : 0.0;
      }
}

// d = a y (NB x NB complex by NB complex)
template <int NB>
__device__ __forceinline__ void blk_mv(const double (&ar)[NB][NB], const double (&ai)[NB][NB], const double (&yr)[NB],
                                       const double (&yi)[NB], double (&dr)[NB], double (&di)[NB]) {
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    double sr = ar[i][0] * yr[0], si = ar[i][0] * yi[0];
    sr = fma(-ai[i][0], yi[0], sr);
    si = fma(ai[i][0], yr[0], si);
#pragma unroll
    for (int k = 1; k < NB; ++k) {
      sr = fma(ar[i][k], yr[k], sr);
      si = fma(ar[i][k], yi[k], si);
      sr = fma(-ai[i][k], yi[k], sr);
      si = fma(ai[i][k], yr[k], si);
    }
    dr[i] = sr;
    di[i] = si;
  }
}

// One slice on this lane's block: y <- e^{μ} (p(Â))^s y with the dense chains' polynomial (TChainMF::step):
// Chebyshev y_1 = Â y_0 / 2, y_{t+1} = Â y_t + y_{t-1}, Σ c_t y_t (c_t = lane t of cl); Taylor z_t = Â z_{t-1} / t.
template <int NB, bool CHEB>
__device__ __forceinline__ void blk_slice(const double (&ar)[NB][NB], const double (&ai)[NB][NB], double (&yr)[NB],
                                          double (&yi)[NB], int P, int s, double phr, double phi, double cl,
                                          const double* __restrict__ invt) {
  for (int sub = 0; sub < s; ++sub) {
    double accr[NB], acci[NB], m1r[NB], m1i[NB], m2r[NB], m2i[NB];
    const double c0 = CHEB ? bcast(cl, 0) : 1.0;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      accr[i] = c0 * yr[i];
      acci[i] = c0 * yi[i];
      m1r[i] = yr[i];
      m1i[i] = yi[i];
      m2r[i] = m2i[i] = 0.0;
    }
    for (int t = 1; t <= P; ++t) {
      const double ct = CHEB ? bcast(cl, t) : invt[t];
      double dr[NB], di[NB];
      blk_mv<NB>(ar, ai, m1r, m1i, dr, di);
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        double zr, zi;
        if constexpr (CHEB) {
          zr = t == 1 ? 0.5 * dr[i] : dr[i] + m2r[i];
          zi = t == 1 ? 0.5 * di[i] : di[i] + m2i[i];
          m2r[i] = m1r[i];
          m2i[i] = m1i[i];
          accr[i] = fma(ct, zr, accr[i]);
          acci[i] = fma(ct, zi, acci[i]);
        } else {
          zr = dr[i] * ct;
          zi = di[i] * ct;
          accr[i] += zr;
          acci[i] += zi;
        }
        m1r[i] = zr;
        m1i[i] = zi;
      }
    }
    const bool last = sub == s - 1;
    const double pr = last ? phr : 1.0, pi = last ? phi : 0.0;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      yr[i] = pr * accr[i] - pi * acci[i];
      yi[i] = pr * acci[i] + pi * accr[i];
    }
  }
}

// Â = scale (Ã_0 + u_1 Ã_1 + u_2 Ã_2) on the block (u[j >= nu] multiplies zero generator registers)
template <int NB>
__device__ __forceinline__ void blk_form(const double (&gr)[3][NB][NB], const double (&gi)[3][NB][NB],
                                         const double (&u)[2], double scale, double (&ar)[NB][NB],
                                         double (&ai)[NB][NB]) {
  const double u1 = u[0] * scale, u2 = u[1] * scale;
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      ar[i][k] = fma(u2, gr[2][i][k], fma(u1, gr[1][i][k], scale * gr[0][i][k]));
      ai[i][k] = fma(u2, gi[2][i][k], fma(u1, gi[1][i][k], scale * gi[0][i][k]));
    }
}

// LDS of the block chains: 1/t (64) | reduction (16) | x_N in the caller's layout (2 N m)
__host__ __device__ inline size_t blk_lds(int N, int m) { return (size_t)(80 + 2 * N * m) * sizeof(double); }

template <int NB, bool CHEB>
__device__ __forceinline__ void blk_fwd_body(const TChainArgs& g, const BlkArgs& bk, const int b) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* invt = reinterpret_cast<double*>(smem);
  double* red = invt + 64;
  double* xN = red + 16;
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, tid = threadIdx.x, nthr = blockDim.x;
  const size_t Nm = (size_t)N * m;
  for (int e = tid; e < 64; e += nthr) invt[e] = e ? 1.0 / e : 0.0;
  BlkLane<NB> ln;
  ln.setup(bk, m, tid);
  double gr[3][NB][NB], gi[3][NB][NB];
  blk_load_gen<NB, false>((const cx<double>*)g.At, N, nu, ln.r, gr, gi);
  const cx<double>* x0b = (const cx<double>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0);
  double* Xb = reinterpret_cast<double*>((cx<double>*)g.X + (size_t)b * (Nt + 1) * Nm);
  double* const sink = tchain_sink(g);
  double yr[NB], yi[NB];
  size_t off[NB];
  bool pm[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const bool ok = ln.r[i] >= 0;
    const size_t o = (size_t)ln.c * N + max(ln.r[i], 0);
    off[i] = 2 * o;
    const cx<double> v = ok ? x0b[o] : cx<double>{0.0, 0.0};
    yr[i] = v.r;
    yi[i] = v.i;
    pm[i] = ok && g.pmask && g.pmask[o];
  }
  double pen = 0.0;
  // x_k to HBM in the caller's layout; padding elements go to the sink (no branch around the stores)
  auto store = [&](int k) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      double* p = ln.r[i] >= 0 ? Xb + (size_t)k * 2 * Nm + off[i] : sink;
      *reinterpret_cast<double2*>(p) = make_double2(yr[i], yi[i]);
      pen += pm[i] ? yr[i] * yr[i] + yi[i] * yi[i] : 0.0;
    }
  };
  __syncthreads();
  store(0);
  const double* ceb = CHEB ? g.tcoef + (size_t)b * Nt * TCHEB_STRIDE : nullptr;
  const TStep* stb = g.steps + (size_t)b * Nt;
  const double* ub = g.u + (size_t)b * Nt * nu;
  constexpr int PD = 2;  // slices of step data in flight
  TPreN<2> nx[PD];
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int ki = min(i, Nt - 1);
    tpre_load<2, CHEB, false>(stb + ki, ub + (size_t)ki * nu, nu, nx[i], CHEB ? ceb + (size_t)ki * TCHEB_STRIDE : nullptr);
  }
  for (int k0 = 0; k0 < Nt; k0 += PD)
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int k = k0 + i;
      if (k >= Nt) break;
      const TPreN<2>& st = nx[i];
      const int P = __builtin_amdgcn_readfirstlane(st.P), s = __builtin_amdgcn_readfirstlane(st.s);
      double ar[NB][NB], ai[NB][NB];
      blk_form<NB>(gr, gi, st.u, st.scale, ar, ai);
      blk_slice<NB, CHEB>(ar, ai, yr, yi, P, s, st.pr, st.pi, st.cl, invt);
      const int kn = min(k + PD, Nt - 1);
      tpre_load<2, CHEB, false>(stb + kn, ub + (size_t)kn * nu, nu, nx[i], CHEB ? ceb + (size_t)kn * TCHEB_STRIDE : nullptr);
      store(k + 1);
    }
#pragma unroll
  for (int i = 0; i < NB; ++i)
    if (ln.r[i] >= 0) {
      xN[off[i]] = yr[i];
      xN[off[i] + 1] = yi[i];
    }
  __syncthreads();
  chain_costs<double>(N, m, (const cx<double>*)g.Xt, [&](int o) { return cx<double>{xN[2 * o], xN[2 * o + 1]}; },
                      g.cost_kind, g.n_norm, block_sum(pen, red) * g.mu, red, g.J + b, g.coef + (size_t)b * 2 * m, g.sc);
}

// λ_N = dJ/dx(x_N) (+ 2μ x_N on the penalty mask + the caller's dL/dx(x_N)), then λ_k = exp(A_k)^H λ_{k+1} (+ the
// same at x_k) down to k = 0.  μ mode: μ_N = X_target and no additions (λ = coef ⊙ μ, applied by the gradient).
template <int NB, bool CHEB>
__device__ __forceinline__ void blk_bwd_body(const TChainArgs& g, const BlkArgs& bk, const int b) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* invt = reinterpret_cast<double*>(smem);
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, tid = threadIdx.x, nthr = blockDim.x;
  const size_t Nm = (size_t)N * m;
  for (int e = tid; e < 64; e += nthr) invt[e] = e ? 1.0 / e : 0.0;
  BlkLane<NB> ln;
  ln.setup(bk, m, tid);
  double gr[3][NB][NB], gi[3][NB][NB];
  blk_load_gen<NB, true>((const cx<double>*)g.At, N, nu, ln.r, gr, gi);
  const double* Xb = reinterpret_cast<const double*>((const cx<double>*)g.X + (size_t)b * (Nt + 1) * Nm);
  double* Lb = reinterpret_cast<double*>((cx<double>*)g.L + (size_t)b * (Nt + 1) * Nm);
  const double* srcb =
      (g.src && !g.mu_mode) ? reinterpret_cast<const double*>((const cx<double>*)g.src + (size_t)b * (Nt + 1) * Nm) : nullptr;
  const unsigned char* pmask = g.mu_mode ? nullptr : g.pmask;
  const cx<double>* Xt = (const cx<double>*)g.Xt;
  const double tmu = 2.0 * g.mu;
  double* const sink = tchain_sink(g);
  double yr[NB], yi[NB];
  size_t off[NB];
  bool pm[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const bool ok = ln.r[i] >= 0;
    const size_t o = (size_t)ln.c * N + max(ln.r[i], 0);
    off[i] = 2 * o;
    pm[i] = ok && pmask && pmask[o];
    cx<double> v = {0.0, 0.0};
    if (ok) {
      if (g.mu_mode) {
        v = Xt[o];
      } else if (g.cost_kind == COST_EXTERNAL) {
        v = reinterpret_cast<const cx<double>*>(Lb)[(size_t)Nt * Nm + o];
      } else {
        const cx<double> cf = g.coef[(size_t)b * 2 * m + ln.c], t = Xt[o];
        v = cx<double>{cf.r * t.r - cf.i * t.i, cf.r * t.i + cf.i * t.r};
      }
      if (pm[i]) {
        v.r += tmu * Xb[(size_t)Nt * 2 * Nm + 2 * o];
        v.i += tmu * Xb[(size_t)Nt * 2 * Nm + 2 * o + 1];
      }
      if (srcb) {
        v.r += srcb[(size_t)Nt * 2 * Nm + 2 * o];
        v.i += srcb[(size_t)Nt * 2 * Nm + 2 * o + 1];
      }
    }
    yr[i] = v.r;
    yi[i] = v.i;
  }
  auto store = [&](int k) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      double* p = ln.r[i] >= 0 ? Lb + (size_t)k * 2 * Nm + off[i] : sink;
      *reinterpret_cast<double2*>(p) = make_double2(yr[i], yi[i]);
    }
  };
  __syncthreads();
  store(Nt);
  const double* ceb = CHEB ? g.tcoef + (size_t)b * Nt * TCHEB_STRIDE : nullptr;
  const TStep* stb = g.steps + (size_t)b * Nt;
  const double* ub = g.u + (size_t)b * Nt * nu;
  const bool add = pmask || srcb;
  constexpr int PD = 2;
  TPreN<2> nx[PD];
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int ki = max(Nt - 1 - i, 0);
    tpre_load<2, CHEB, false>(stb + ki, ub + (size_t)ki * nu, nu, nx[i], CHEB ? ceb + (size_t)ki * TCHEB_STRIDE : nullptr);
  }
  for (int k0 = Nt - 1; k0 >= 0; k0 -= PD)
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int k = k0 - i;
      if (k < 0) break;
      const TPreN<2>& st = nx[i];
      const int P = __builtin_amdgcn_readfirstlane(st.P), s = __builtin_amdgcn_readfirstlane(st.s);
      double xr[NB], xi[NB];
      if (add) {  // 2μ x_k on the mask + the caller's dL/dx(x_k), added after the slice
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2) {
          const size_t o = (size_t)k * 2 * Nm + off[i2];
          const bool ok = ln.r[i2] >= 0;
          xr[i2] = pm[i2] ? tmu * Xb[o] : 0.0;
          xi[i2] = pm[i2] ? tmu * Xb[o + 1] : 0.0;
          if (srcb && ok) {
            xr[i2] += srcb[o];
            xi[i2] += srcb[o + 1];
          }
        }
      }
      double ar[NB][NB], ai[NB][NB];
      blk_form<NB>(gr, gi, st.u, st.scale, ar, ai);
      blk_slice<NB, CHEB>(ar, ai, yr, yi, P, s, st.pr, -st.pi, st.cl, invt);
      const int kp = max(k - PD, 0);
      tpre_load<2, CHEB, false>(stb + kp, ub + (size_t)kp * nu, nu, nx[i], CHEB ? ceb + (size_t)kp * TCHEB_STRIDE : nullptr);
      if (add) {
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2) {
          yr[i2] += xr[i2];
          yi[i2] += xi[i2];
        }
      }
      store(k);
    }
}

template <int NB, bool CHEB>
__global__ __launch_bounds__(BLK_MAXT) void k_blk_fwd(const TChainArgs g, const BlkArgs bk) {
  blk_fwd_body<NB, CHEB>(g, bk, blockIdx.x);
}
template <int NB, bool CHEB>
__global__ __launch_bounds__(BLK_MAXT) void k_blk_bwd(const TChainArgs g, const BlkArgs bk) {
  blk_bwd_body<NB, CHEB>(g, bk, blockIdx.x);
}
// Forward chain and μ recurrence of every seed in one launch of 2B workgroups (as k_tchain_mf_dual)
template <int NB, bool CHEB>
__global__ __launch_bounds__(BLK_MAXT) void k_blk_dual(const TChainArgs gf, const TChainArgs gb, const BlkArgs bk) {
  const int i = blockIdx.x, B = gridDim.x >> 1;
  const bool by8 = (B & 7) == 0;
  const int dir = by8 ? (i >> 3) & 1 : i & 1;
  const int seed = by8 ? ((i >> 4) << 3) | (i & 7) : i >> 1;
  if (dir == 0) blk_fwd_body<NB, CHEB>(gf, bk, seed);
  else blk_bwd_body<NB, CHEB>(gb, bk, seed);
}

// ---------------------------------------------------------------------------------------------------------
// MFMA block waves: each wave owns a 16-row state ("wave block", wrow: 16 global rows, -1 padding) and one state
// column pair, and runs TChainRot<1>'s v_mfma_f64_4x4x4_4b term (qoc_tchain.hpp) on it.  In the 4x4x4_4b layout a
// lane's D element (local row 4b + hi, column lo) is block b's B operand for k = hi of a k-quad, and a DPP row_ror by
// 4j hands block b the k-quad q_j(b) of the state; the A operands hold Ã[r(4b + lo)][r(4 q_j(b) + hi)].
//  * JR = 4: one invariant block of 5..16 rows per wave (the tunable bus: two parity blocks of 14 and 13 rows at
//    N = 27): 8 MFMAs per term per block wave instead of the dense two-group chain's 32 in one wave.
//  * JR = 1: invariant blocks of <= 4 rows packed into the wave's four aligned 4-row slots (cavity: two 2-row blocks
//    per slot, zz: one 3-row block per slot).  No block couples two slots, so only the unrotated k-quad (j = 0)
//    carries entries: a term is 2 MFMAs (Ar, Ai) on the state as it sits in the D layout (D = B layout at K = 4),
//    no rotation, and 4 slots x 2 columns of blocks per instruction.
// No cross-wave exchange per term.  With captures (D1 = Â v, D2 = Â y_1 of each slice, the layout TChainArgs::cap1 /
// cap2 documents) the concurrent eval's contraction is k_grad_rr_c; the blocks of <= 4 rows use k_blk_grad instead.
struct BlkRotLane {
  int n, cp, beta;
  int rowE;     // global row of this lane's D element (-1: padding, or no block)
  int pe;       // the D element's part: 0 real, 1 imaginary
  int colD;     // state column of the D element
  bool act;     // rowE >= 0 && colD < m
  int rowA;     // global row of the lane's A-operand entries (JR = 0: row * 2 + part)
  int colA[4];  // global column of the A-operand entry of rotation j (JR = 0: column * 2 + part)
  // JR = 0 (real embedding): wrow entries are row * 2 + part, a wave holds 4 complex state columns (n)
  template <int JR>
  __device__ __forceinline__ void setup(const BlkArgs& bk, int m) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int b = (l >> 2) & 3, kl = l >> 4, lo = l & 3;
    const int CPW = JR == 0 ? (m + 3) / 4 : (m + 1) / 2;
    const bool wok = w < bk.nwb * CPW;
    beta = wok ? w % bk.nwb : 0;
    cp = wok ? w / bk.nwb : 0;
    n = lo;
    const int* rb = bk.wrow + beta * 16;
    const int e = wok ? rb[4 * b + kl] : -1;
    if constexpr (JR == 0) {
      colD = 4 * cp + n;
      rowE = e >= 0 ? e >> 1 : -1;
      pe = e >= 0 ? e & 1 : 0;
      rowA = wok ? rb[4 * b + lo] : -1;
      colA[0] = e;
      colA[1] = colA[2] = colA[3] = -1;
    } else {
      colD = 2 * cp + (n >> 1);
      rowE = e;
      pe = n & 1;
      rowA = wok ? rb[4 * b + lo] : -1;
      const int q[4] = {b, __builtin_amdgcn_update_dpp(0, b, 0x124, 0xf, 0xf, false),   // row_ror:4
                        __builtin_amdgcn_update_dpp(0, b, 0x128, 0xf, 0xf, false),      // row_ror:8
                        __builtin_amdgcn_update_dpp(0, b, 0x12C, 0xf, 0xf, false)};     // row_ror:12
#pragma unroll
      for (int j = 0; j < 4; ++j) colA[j] = wok ? rb[4 * q[j] + kl] : -1;
    }
    act = rowE >= 0 && colD < m;
  }
  // the A-operand entries of Ã_0..Ã_2 (HERM: of Ã_j^H), zero outside the block and for j > nu.  JR = 0: the real
  // embedding [[Re, -Im], [Im, Re]] of the complex entry (rows / columns carry their part), in gr (gi unused)
  template <bool HERM, int JR, int JA>
  __device__ __forceinline__ void load_gen(const cx<double>* __restrict__ At, int N, int nu, double (&gr)[3][JA],
                                           double (&gi)[3][JA]) const {
    const size_t NN = (size_t)N * N;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int x = 0; x < JA; ++x) {
        if constexpr (JR == 0) {
          const bool ok = j <= nu && rowA >= 0 && colA[0] >= 0;
          const int rr = max(rowA, 0) >> 1, cc = max(colA[0], 0) >> 1, p1 = rowA & 1, p2 = colA[0] & 1;
          const cx<double> v = At[(size_t)min(j, nu) * NN + (HERM ? cc + (size_t)N * rr : rr + (size_t)N * cc)];
          const double a = v.r, bi = HERM ? -v.i : v.i;
          gr[j][x] = ok ? (p1 == p2 ? a : (p1 == 0 ? -bi : bi)) : 0.0;
          gi[j][x] = 0.0;
        } else {
          const bool ok = j <= nu && rowA >= 0 && colA[x] >= 0;
          const int rr = max(rowA, 0), cc = max(colA[x], 0);
          const cx<double> v = At[(size_t)min(j, nu) * NN + (HERM ? cc + (size_t)N * rr : rr + (size_t)N * cc)];
          gr[j][x] = ok ? v.r : 0.0;
          gi[j][x] = ok ? (HERM ? -v.i : v.i) : 0.0;
        }
      }
  }
};

// one slice on the wave's 16-row block state (one element per lane, TChainRot<1>::step without the LDS mirror);
// D1, D2 of the first substep go to cd1, cd2 (the captures).  sg = +1 on imaginary lanes, -1 on real ones: the Ai
// products enter through the n <-> n^1 swap with that sign, as one FMA.  Chebyshev terms carry y_{t-2} in the Ar
// MFMA's accumulator input (y_t = Â y_{t-1} + y_{t-2} in one chain), and the term loop runs two terms per
// iteration with the roles of the two state registers swapped, so no register copies are left in it.
// cof: the slice's staged Chebyshev coefficients in LDS (c_t at cof[t], read as broadcasts: one ds_read2 per two
// terms instead of two v_readlane per term on the VALU)
template <int JR, bool CHEB, int JA = (JR ? JR : 1)>
__device__ __forceinline__ void blkrot_slice(const double (&ar)[JA], const double (&ai)[JA], double& acc, bool act,
                                             double sg, int P, int s, double phr, double phi,
                                             const double* __restrict__ cof, const double* __restrict__ invt,
                                             double& cd1, double& cd2) {
  using R = TChainRot<1>;
  // Ar y + c + sg (Ai y)[n ^ 1]
  auto prod = [&](double y, double c) __attribute__((always_inline)) {
    if constexpr (JR == 0) return MF<double>::mma4(ar[0], y, c);  // real embedding: one real 4x4 per slot
    double bv[4];
    bv[0] = y;
    if constexpr (JR > 1) {
      bv[1] = R::mv<0x124>(y);  // row_ror:4
      bv[2] = R::mv<0x128>(y);  // row_ror:8
      bv[3] = R::mv<0x12C>(y);  // row_ror:12
    }
    double d1 = 0.0, d0 = c;
#pragma unroll
    for (int j = 0; j < JR; ++j) d1 = MF<double>::mma4(ai[j], bv[j], d1);
#pragma unroll
    for (int j = 0; j < JR; ++j) d0 = MF<double>::mma4(ar[j], bv[j], d0);
    return fma(sg, R::mv<0xB1>(d1), d0);  // quad_perm [1,0,3,2]
  };
  for (int sub = 0; sub < s; ++sub) {
    const double y0 = act ? acc : 0.0;
    if constexpr (CHEB) {
      const double c0 = cof[0], c1 = cof[1], c2 = cof[2];
      acc = c0 * y0;
      double a = y0, b;
      {  // t = 1: y_1 = Â y_0 / 2
        const double D = prod(y0, 0.0);
        if (sub == 0) cd1 = D;
        b = 0.5 * D;
        acc = fma(c1, b, acc);
      }
      if (P >= 2) {  // t = 2: the plain product is the second capture
        const double D = prod(b, 0.0);
        if (sub == 0) cd2 = D;
        a = D + a;
        acc = fma(c2, a, acc);
      } else {
        a = b;  // y_{t-1} in a for the (empty) loop below
      }
      // here a = y_{t-1}, b = y_{t-2} for t = 3
      int t = 3;
      for (; t + 1 <= P; t += 2) {
        const double ca = cof[t], cb = cof[t + 1];
        b = prod(a, b);
        acc = fma(ca, b, acc);
        a = prod(b, a);
        acc = fma(cb, a, acc);
      }
      if (t <= P) {
        const double ca = cof[t];
        b = prod(a, b);
        acc = fma(ca, b, acc);
      }
    } else {
      acc = y0;
      double z = y0;
      for (int t = 1; t <= P; ++t) {
        const double D = prod(z, 0.0);
        if (sub == 0 && t == 1) cd1 = D;
        if (sub == 0 && t == 2) cd2 = D;
        z = D * invt[t];
        acc += z;
      }
    }
    if (sub == s - 1) {  // e^{μ}: the partner part of the element is lane n ^ 1 (complex slots) or l ^ 32 (real)
      const double o = JR == 0 ? __shfl_xor(acc, 32) : R::mv<0xB1>(acc);
      acc = fma(sg * phi, o, phr * acc);
    }
  }
}

template <int JA>
__device__ __forceinline__ void blkrot_form(const double (&gr)[3][JA], const double (&gi)[3][JA], const double (&u)[2],
                                            double scale, double (&ar)[JA], double (&ai)[JA]) {
  const double u1 = u[0] * scale, u2 = u[1] * scale;
#pragma unroll
  for (int x = 0; x < JA; ++x) {
    ar[x] = fma(u2, gr[2][x], fma(u1, gr[1][x], scale * gr[0][x]));
    ai[x] = fma(u2, gi[2][x], fma(u1, gi[1][x], scale * gi[0][x]));
  }
}

// Step records of the MFMA block waves, staged through a per-wave LDS slot in chunks of BLK_CH slices.  A slice
// of packed blocks is short (~9 terms of a few dozen cycles), shorter than an HBM round trip; with per-slice
// register prefetches the compiler's vmcnt waits at the loop head also covered the newest prefetches, so every
// slice waited for memory (~0.75 us per slice measured).  Here the loads of chunk c + 1 are issued at the start of
// chunk c into registers and written to LDS at the start of chunk c + 1 (one wait per chunk); the slices read
// their record (broadcast) and this lane's Chebyshev coefficient from LDS.
constexpr int BLK_CH = 8;
constexpr int BLK_STAGE = BLK_CH * (8 + 64);  // doubles per wave: [CH][8] records + [CH][64] coefficients
struct BlkStage {
  double* rec;  // this wave's [CH][8]: pr, pi, (P | s << 32), scale, u_1, u_2
  double* cof;  // this wave's [CH][64]
  double4 t4;
  double u0, u1;
  double rc[BLK_CH];
};
// loads of the chunk whose slice j is k = kfirst + dir j (clamped: the same loads on every path)
template <bool CHEB>
__device__ __forceinline__ void blk_stage_issue(BlkStage& S, const TStep* __restrict__ stb, const double* __restrict__ ub,
                                                const double* __restrict__ ceb, int nu, int Nt, int kfirst, int dir) {
  const int l = threadIdx.x & 63;
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));  // per-lane (VGPR) address: vector loads, not s_load (see tpre_load)
  const int kl = min(max(kfirst + dir * (l & (BLK_CH - 1)), 0), Nt - 1);
  S.t4 = *reinterpret_cast<const double4*>(reinterpret_cast<const double*>(stb + kl) + z);
  S.u0 = ub[(size_t)kl * nu + z];
  S.u1 = ub[(size_t)kl * nu + min(1, nu - 1) + z];
  if constexpr (CHEB) {
#pragma unroll
    for (int j = 0; j < BLK_CH; ++j) {
      const int kj = min(max(kfirst + dir * j, 0), Nt - 1);
      S.rc[j] = ceb[(size_t)kj * TCHEB_STRIDE + l + z];
    }
  }
}
template <bool CHEB>
__device__ __forceinline__ void blk_stage_commit(BlkStage& S) {
  const int l = threadIdx.x & 63;
  if (l < BLK_CH) {
    double* r = S.rec + 8 * l;
    r[0] = S.t4.x;
    r[1] = S.t4.y;
    r[2] = S.t4.z;
    r[3] = S.t4.w;
    r[4] = S.u0;
    r[5] = S.u1;
  }
  if constexpr (CHEB) {
#pragma unroll
    for (int j = 0; j < BLK_CH; ++j) S.cof[64 * j + l] = S.rc[j];
  }
}
// slice j of the staged chunk
struct BlkRec {
  double pr, pi, scale, u[2], cl;
  int P, s;
};
template <bool CHEB>
__device__ __forceinline__ BlkRec blk_stage_read(const BlkStage& S, int j) {
  const double* r = S.rec + 8 * j;
  BlkRec q;
  q.pr = r[0];
  q.pi = r[1];
  const long long ps = __double_as_longlong(r[2]);
  q.P = __builtin_amdgcn_readfirstlane((int)(ps & 0xffffffff));
  q.s = __builtin_amdgcn_readfirstlane((int)(ps >> 32));
  q.scale = r[3];
  q.u[0] = r[4];
  q.u[1] = r[5];
  q.cl = 0.0;
  return q;
}
// LDS of the MFMA block waves: blk_lds + one staging slot per wave
__host__ __device__ inline size_t blkrot_lds(int N, int m, int waves) {
  return blk_lds(N, m) + (size_t)waves * BLK_STAGE * sizeof(double);
}
// after_xN: 80 + 2 N m doubles into the dynamic LDS, 16-byte aligned.  No integer round trip on the pointer: the
// compiler must still see an LDS address (a generic one becomes flat_load, whose waitcnt drains vmcnt as well)
__device__ __forceinline__ BlkStage blk_stage_slot(double* after_xN) {
  double* base = after_xN;
  BlkStage S;
  S.rec = base + (size_t)(threadIdx.x >> 6) * BLK_STAGE;
  S.cof = S.rec + 8 * BLK_CH;
  return S;
}

template <int JR, bool CHEB>
__device__ __forceinline__ void blkrot_fwd_body(const TChainArgs& g, const BlkArgs& bk, const int b) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* invt = reinterpret_cast<double*>(smem);
  double* red = invt + 64;
  double* xN = red + 16;
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, tid = threadIdx.x, nthr = blockDim.x;
  const size_t Nm = (size_t)N * m;
  for (int e = tid; e < 64; e += nthr) invt[e] = e ? 1.0 / e : 0.0;
  constexpr int JA = JR ? JR : 1;
  BlkRotLane ln;
  ln.setup<JR>(bk, m);
  const double sg = ln.pe ? 1.0 : -1.0;
  double gr[3][JA], gi[3][JA];
  ln.load_gen<false, JR, JA>((const cx<double>*)g.At, N, nu, gr, gi);
  const cx<double>* x0b = (const cx<double>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0);
  double* Xb = reinterpret_cast<double*>((cx<double>*)g.X + (size_t)b * (Nt + 1) * Nm);
  double* const sink = tchain_sink(g);
  const size_t o = (size_t)ln.colD * N + max(ln.rowE, 0), oe = 2 * o + ln.pe;
  double acc = 0.0;
  if (ln.act) {
    const cx<double> v = x0b[o];
    acc = ln.pe ? v.i : v.r;
  }
  const bool pm = ln.act && g.pmask && g.pmask[o];
  const bool cap = g.cap1 != nullptr;
  double* c1b = cap ? reinterpret_cast<double*>((cx<double>*)g.cap1 + (size_t)b * (Nt + 1) * Nm) : nullptr;
  double* c2b = cap ? reinterpret_cast<double*>((cx<double>*)g.cap2 + (size_t)b * (Nt + 1) * Nm) : nullptr;
  double pen = 0.0;
  for (size_t e = tid; e < 2 * Nm; e += nthr) xN[e] = 0.0;  // the rows of blocks without a wave (blk_live) stay 0
  __syncthreads();
  *(ln.act ? Xb + oe : sink) = acc;
  pen += pm ? acc * acc : 0.0;
  const double* ceb = CHEB ? g.tcoef + (size_t)b * Nt * TCHEB_STRIDE : nullptr;
  const TStep* stb = g.steps + (size_t)b * Nt;
  const double* ub = g.u + (size_t)b * Nt * nu;
  BlkStage S = blk_stage_slot(xN + 2 * Nm);
  blk_stage_issue<CHEB>(S, stb, ub, ceb, nu, Nt, 0, 1);
  for (int c0 = 0; c0 < Nt; c0 += BLK_CH) {
    blk_stage_commit<CHEB>(S);
    if (c0 + BLK_CH < Nt) blk_stage_issue<CHEB>(S, stb, ub, ceb, nu, Nt, c0 + BLK_CH, 1);
    for (int j = 0; j < BLK_CH; ++j) {
      const int k = c0 + j;
      if (k >= Nt) break;
      const BlkRec st = blk_stage_read<CHEB>(S, j);
      double ar[JA], ai[JA], cd1 = 0.0, cd2 = 0.0;
      blkrot_form<JA>(gr, gi, st.u, st.scale, ar, ai);
      blkrot_slice<JR, CHEB>(ar, ai, acc, ln.act, sg, st.P, st.s, st.pr, st.pi, S.cof + 64 * j, invt, cd1, cd2);
      *(ln.act ? Xb + (size_t)(k + 1) * 2 * Nm + oe : sink) = acc;
      pen += pm ? acc * acc : 0.0;
      if constexpr (JR > 1) {  // packed blocks (JR = 1) feed k_blk_grad, which forms its own products
        const bool to = cap && ln.act;
        *(to ? c1b + (size_t)k * 2 * Nm + oe : sink) = cd1;
        *(to ? c2b + (size_t)k * 2 * Nm + oe : sink + 1) = cd2;
      }
    }
  }
  if (ln.act) xN[oe] = acc;
  __syncthreads();
  chain_costs<double>(N, m, (const cx<double>*)g.Xt, [&](int q) { return cx<double>{xN[2 * q], xN[2 * q + 1]}; },
                      g.cost_kind, g.n_norm, block_sum(pen, red) * g.mu, red, g.J + b, g.coef + (size_t)b * 2 * m, g.sc);
}

template <int JR, bool CHEB>
__device__ __forceinline__ void blkrot_bwd_body(const TChainArgs& g, const BlkArgs& bk, const int b) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* invt = reinterpret_cast<double*>(smem);
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, tid = threadIdx.x, nthr = blockDim.x;
  const size_t Nm = (size_t)N * m;
  for (int e = tid; e < 64; e += nthr) invt[e] = e ? 1.0 / e : 0.0;
  constexpr int JA = JR ? JR : 1;
  BlkRotLane ln;
  ln.setup<JR>(bk, m);
  const double sg = ln.pe ? 1.0 : -1.0;
  double gr[3][JA], gi[3][JA];
  ln.load_gen<true, JR, JA>((const cx<double>*)g.At, N, nu, gr, gi);
  const double* Xb = reinterpret_cast<const double*>((const cx<double>*)g.X + (size_t)b * (Nt + 1) * Nm);
  double* Lb = reinterpret_cast<double*>((cx<double>*)g.L + (size_t)b * (Nt + 1) * Nm);
  const double* srcb =
      (g.src && !g.mu_mode) ? reinterpret_cast<const double*>((const cx<double>*)g.src + (size_t)b * (Nt + 1) * Nm) : nullptr;
  const unsigned char* pmask = g.mu_mode ? nullptr : g.pmask;
  const double tmu = 2.0 * g.mu;
  double* const sink = tchain_sink(g);
  const size_t o = (size_t)ln.colD * N + max(ln.rowE, 0), oe = 2 * o + ln.pe;
  const bool pm = ln.act && pmask && pmask[o];
  const bool srcl = ln.act && srcb;
  double acc = 0.0;
  if (ln.act) {
    cx<double> v;
    if (g.mu_mode) {
      v = ((const cx<double>*)g.Xt)[o];
    } else if (g.cost_kind == COST_EXTERNAL) {
      v = reinterpret_cast<const cx<double>*>(Lb)[(size_t)Nt * Nm + o];
    } else {
      const cx<double> cf = g.coef[(size_t)b * 2 * m + ln.colD], t = ((const cx<double>*)g.Xt)[o];
      v = cx<double>{cf.r * t.r - cf.i * t.i, cf.r * t.i + cf.i * t.r};
    }
    acc = ln.pe ? v.i : v.r;
    if (pm) acc += tmu * Xb[(size_t)Nt * 2 * Nm + oe];
    if (srcl) acc += srcb[(size_t)Nt * 2 * Nm + oe];
  }
  const bool cap = g.cap1 != nullptr;
  double* c1b = cap ? reinterpret_cast<double*>((cx<double>*)g.cap1 + (size_t)b * (Nt + 1) * Nm) : nullptr;
  double* c2b = cap ? reinterpret_cast<double*>((cx<double>*)g.cap2 + (size_t)b * (Nt + 1) * Nm) : nullptr;
  __syncthreads();
  *(ln.act ? Lb + (size_t)Nt * 2 * Nm + oe : sink) = acc;
  const double* ceb = CHEB ? g.tcoef + (size_t)b * Nt * TCHEB_STRIDE : nullptr;
  const TStep* stb = g.steps + (size_t)b * Nt;
  const double* ub = g.u + (size_t)b * Nt * nu;
  BlkStage S = blk_stage_slot(reinterpret_cast<double*>(smem) + 80 + 2 * Nm);
  blk_stage_issue<CHEB>(S, stb, ub, ceb, nu, Nt, Nt - 1, -1);
  for (int c0 = 0; c0 < Nt; c0 += BLK_CH) {
    blk_stage_commit<CHEB>(S);
    if (c0 + BLK_CH < Nt) blk_stage_issue<CHEB>(S, stb, ub, ceb, nu, Nt, Nt - 1 - (c0 + BLK_CH), -1);
    for (int j = 0; j < BLK_CH; ++j) {
      const int k = Nt - 1 - (c0 + j);
      if (k < 0) break;
      const BlkRec st = blk_stage_read<CHEB>(S, j);
      const size_t ok_ = (size_t)k * 2 * Nm + oe;
      double xa = pm ? tmu * Xb[ok_] : 0.0;  // 2μ x_k on the mask + the caller's dL/dx(x_k), after the slice
      if (srcl) xa += srcb[ok_];
      double ar[JA], ai[JA], cd1 = 0.0, cd2 = 0.0;
      blkrot_form<JA>(gr, gi, st.u, st.scale, ar, ai);
      blkrot_slice<JR, CHEB>(ar, ai, acc, ln.act, sg, st.P, st.s, st.pr, -st.pi, S.cof + 64 * j, invt, cd1, cd2);
      acc += xa;
      *(ln.act ? Lb + ok_ : sink) = acc;
      if constexpr (JR > 1) {
        const bool to = cap && ln.act;
        *(to ? c1b + ok_ : sink) = cd1;
        *(to ? c2b + ok_ : sink + 1) = cd2;
      }
    }
  }
}

// Zeros on the rows of the blocks that carry no state (qoc_run_blk.hip blk_live): rows[0..nrow) of each of the
// `cols` N-row columns of up to six state-shaped buffers (x_k, μ_k and the chains' captured products)
struct ZeroRows {
  double2* buf[6];
  int nbuf;
};
static __global__ void k_zero_rows(const ZeroRows z, long long cols, int N, const int* __restrict__ rows, int nrow) {
  const long long total = cols * nrow;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long q = e / nrow;
    const size_t o = (size_t)q * N + rows[e - q * nrow];
    for (int i = 0; i < z.nbuf; ++i) z.buf[i][o] = make_double2(0.0, 0.0);
  }
}

template <int JR, bool CHEB>
__global__ __launch_bounds__(512) void k_blkrot_fwd(const TChainArgs g, const BlkArgs bk) {
  blkrot_fwd_body<JR, CHEB>(g, bk, blockIdx.x);
}
template <int JR, bool CHEB>
__global__ __launch_bounds__(512) void k_blkrot_bwd(const TChainArgs g, const BlkArgs bk) {
  blkrot_bwd_body<JR, CHEB>(g, bk, blockIdx.x);
}
template <int JR, bool CHEB>
__global__ __launch_bounds__(512) void k_blkrot_dual(const TChainArgs gf, const TChainArgs gb, const BlkArgs bk) {
  const int i = blockIdx.x, B = gridDim.x >> 1;
  const bool by8 = (B & 7) == 0;
  const int dir = by8 ? (i >> 3) & 1 : i & 1;
  const int seed = by8 ? ((i >> 4) << 3) | (i & 7) : i >> 1;
  if (dir == 0) blkrot_fwd_body<JR, CHEB>(gf, bk, seed);
  else blkrot_bwd_body<JR, CHEB>(gb, bk, seed);
}

// The order-ORD gradient per block (expm_jacobian! + _compute_u_sensitivity, src/gradient_computations.jl:177-223):
// with X = A_k on the block, P_b = X^b x_k and Q_a = (X^H)^a λ_{k+1},
//   λ^H dU_j x = Σ_{a+b < ORD} <Q_a, A_j P_b> / (a+b+1)! = Σ_b <W_b, A_j P_b>,  W_b = Σ_{a < ORD-b} Q_a / (a+b+1)!
// (order 3: W_0 = λ + Q_1/2 + Q_2/6, W_1 = λ/2 + Q_1/6, W_2 = λ/6).  One thread per (seed, slice, block) over the
// state columns; the blocks of a unit are adjacent threads of one workgroup and reduce through LDS in a fixed
// order (no atomics: the result does not depend on scheduling).  μ mode: L holds μ and λ = coef ⊙ μ per column.
template <int NB, int ORD>
__global__ __launch_bounds__(256) void k_blk_grad(const TChainArgs g, const BlkArgs bk, long long units, int mu_mode,
                                                   double* __restrict__ dJdu) {
  __shared__ double red[256 * 2];
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, nblk = bk.nblk, UPW = 256 / nblk;
  const size_t Nm = (size_t)N * m, NN = (size_t)N * N;
  const int t = threadIdx.x, ul = t / nblk, beta = t - ul * nblk;
  const long long unit = (long long)blockIdx.x * UPW + ul;
  const bool act = ul < UPW && unit < units;
  const long long uu = act ? unit : 0;
  const int b = (int)(uu / Nt), k = (int)(uu - (long long)b * Nt);
  int r[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) r[i] = act ? bk.brow[beta * NB + i] : -1;
  const cx<double>* A = (const cx<double>*)bk.A;
  double ur[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) ur[j] = j < nu ? g.u[(size_t)uu * nu + j] : 0.0;
  // X = A_0 + Σ_j u_j A_j and A_j on the block
  double xr_[NB][NB], xi_[NB][NB], ajr[2][NB][NB], aji[2][NB][NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int kk = 0; kk < NB; ++kk) {
      const bool ok = r[i] >= 0 && r[kk] >= 0;
      const size_t o = (size_t)max(r[i], 0) + (size_t)N * max(r[kk], 0);
      const cx<double> a0 = ok ? A[o] : cx<double>{0.0, 0.0};
      xr_[i][kk] = a0.r;
      xi_[i][kk] = a0.i;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const cx<double> v = ok && j < nu ? A[(size_t)(j + 1) * NN + o] : cx<double>{0.0, 0.0};
        ajr[j][i][kk] = v.r;
        aji[j][i][kk] = v.i;
        xr_[i][kk] = fma(ur[j], v.r, xr_[i][kk]);
        xi_[i][kk] = fma(ur[j], v.i, xi_[i][kk]);
      }
    }
  // X^H on the block
  double hr[NB][NB], hi[NB][NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int kk = 0; kk < NB; ++kk) {
      hr[i][kk] = xr_[kk][i];
      hi[i][kk] = -xi_[kk][i];
    }
  constexpr double invf[8] = {1.0, 1.0, 0.5, 1.0 / 6, 1.0 / 24, 1.0 / 120, 1.0 / 720, 1.0 / 5040};
  const double* Xs = reinterpret_cast<const double*>((const cx<double>*)g.X + ((size_t)b * (Nt + 1) + k) * Nm);
  const double* Ls = reinterpret_cast<const double*>((const cx<double>*)g.L + ((size_t)b * (Nt + 1) + k + 1) * Nm);
  double acc[2] = {0.0, 0.0};
  for (int c = 0; c < m; ++c) {
    cx<double> cf = {1.0, 0.0};
    if (mu_mode) cf = g.coef[(size_t)b * 2 * m + c];
    double pr[ORD][NB], pi[ORD][NB], qr[ORD][NB], qi[ORD][NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const bool ok = r[i] >= 0;
      const size_t o = 2 * ((size_t)c * N + max(r[i], 0));
      const double2 xv = ok ? *reinterpret_cast<const double2*>(Xs + o) : make_double2(0.0, 0.0);
      const double2 lv = ok ? *reinterpret_cast<const double2*>(Ls + o) : make_double2(0.0, 0.0);
      pr[0][i] = xv.x;
      pi[0][i] = xv.y;
      qr[0][i] = cf.r * lv.x - cf.i * lv.y;
      qi[0][i] = cf.r * lv.y + cf.i * lv.x;
    }
#pragma unroll
    for (int p = 1; p < ORD; ++p) {
      blk_mv<NB>(xr_, xi_, pr[p - 1], pi[p - 1], pr[p], pi[p]);
      blk_mv<NB>(hr, hi, qr[p - 1], qi[p - 1], qr[p], qi[p]);
    }
#pragma unroll
    for (int p = 0; p < ORD; ++p) {
      double wr[NB], wi[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        wr[i] = 0.0;
        wi[i] = 0.0;
#pragma unroll
        for (int a = 0; a + p < ORD; ++a) {
          wr[i] = fma(invf[a + p + 1], qr[a][i], wr[i]);
          wi[i] = fma(invf[a + p + 1], qi[a][i], wi[i]);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (j >= nu) break;
        double yr[NB], yi[NB];
        blk_mv<NB>(ajr[j], aji[j], pr[p], pi[p], yr, yi);
        double sacc = 0.0;
#pragma unroll
        for (int i = 0; i < NB; ++i) sacc = fma(wr[i], yr[i], fma(wi[i], yi[i], sacc));  // Re conj(w) y
        acc[j] += sacc;
      }
    }
  }
  red[2 * t] = act ? acc[0] : 0.0;
  red[2 * t + 1] = act ? acc[1] : 0.0;
  __syncthreads();
  if (t < UPW * nu) {
    const int u2 = t / nu, j = t - u2 * nu;
    const long long un = (long long)blockIdx.x * UPW + u2;
    double s = 0.0;
    for (int q = 0; q < nblk; ++q) s += red[2 * (u2 * nblk + q) + j];
    if (un < units) dJdu[(size_t)un * nu + j] = s;
  }
}

}  // namespace qoc
