// qoc_blkp.hpp — stored propagators for invariant blocks of 5..16 rows (the tunable bus' parity blocks).
//
// The reference forms every slice propagator U_k = exp(A_k) (src/gradient_computations.jl:17-24) and then runs one
// matvec per slice in the chains (:27-29 forward, :52-58 backward).  The MFMA block waves (k_blkrot_*, qoc_blk.hpp)
// instead apply the slice polynomial to the state inside the serial chain: on the tunable bus (‖A_k‖ ≈ 30) that is
// ~42 Chebyshev terms per slice, one wave per (seed, block, direction) and one wave per SIMD, so the serial term
// latency bounds the whole eval.  Here the exponentials leave the chain:
//   * k_blkp_exp: U_k on each live 16-row wave block (BlkArgs::wrow, -1 padding), one wave per (seed, slice, block),
//     every matrix in registers in the v_mfma_f64_16x16x4 D layout ("C layout": lane j + 16 g, register e holds
//     M[g + 4e][j]).  A product L R takes L as its transpose's C layout (register e of L^T is the A operand of k-step e)
//     and R as is (register e is the B operand), so a product needs no data movement; transposes go through a
//     wave-private LDS tile.  Complex products run as three real ones (12 MFMAs).  U_k = e^{μ_k} T_{4r}(2^-s Ã_k)^{2^s}
//     with the degree-4r Taylor polynomial by Paterson-Stockmeyer (X², X³, X⁴, then r - 1 Horner products in X⁴)
//     and s squarings; (r, s) per unit from Σ_{k>4r} ρ^k / k! <= 2^-53 at ρ = 2^-s ρ̂, ρ̂ = sqrt(‖Ã_k‖_1 ‖Ã_k‖_∞) >= ‖Ã_k‖_2,
//     the fewest squarings within one product of the fewest products.
//   * k_blkp_dual: the forward chain x_{k+1} = U_k x_k and the μ recurrence μ_k = U_k^H μ_{k+1} (μ_N = X_target,
//     λ_k = coef ⊙ μ_k) from the stored propagators, one wave per (seed, block, column, direction): lane i + 16 q
//     takes row i and the column quarter 4q..4q+3 of U_k, the quarters are summed with permlane swaps and the new
//     state goes to the next slice through a 16-entry LDS row.  k_blkp_chain runs one direction alone (the split
//     call form: the forward chain in propagate, the μ recurrence in grape_sensitivity).
//   * k_blkp_grad: the order-3 gradient from x_k and μ_{k+1}, 16 slices per wave as the columns of 16 x 16 x 16
//     generator GEMMs on MFMA.
// With one control (nu = 1) the propagators are a Chebyshev series in u over the batch's control range instead:
//   * k_blkp_int forms the stored propagators from its coefficients (D + 1 scaled sums of LDS-resident matrices);
//   * k_blkp_ichain / k_blkp_ichain2 (one live wave block, one state column: the tunable bus, the default) let the chain
//     waves form their own propagators in registers and apply them at once, nothing stored (k_blkp_phase precomputes
//     the slices' e^{μ(u_k)}; the forward's cost is k_terminal_cost's).
#pragma once
#include "qoc_blk.hpp"

namespace qoc {

constexpr int BLKP_WG = 256;  // formation: waves of one workgroup
constexpr int BLKP_RMIN = 2, BLKP_RMAX = 8;
constexpr int BLKP_TP = 16 * 17;  // transpose tile per wave (double2, padded rows)
// θ_{4r}: the largest ρ with Σ_{k>4r} ρ^k / k! <= 2^-53 (r = 1..8)
__constant__ double kBlkpTheta[9] = {0.0,
                                     0.0016783942982781048,
                                     0.06993278480782539,
                                     0.33521368782861477,
                                     0.8246031916386087,
                                     1.504147322395163,
                                     2.3324673844012387,
                                     3.2752135590741402,
                                     4.3063288801167054};
__constant__ double kBlkpInvTheta[9] = {0.0,
                                        1.0 / 0.0016783942982781048,
                                        1.0 / 0.06993278480782539,
                                        1.0 / 0.33521368782861477,
                                        1.0 / 0.8246031916386087,
                                        1.0 / 1.504147322395163,
                                        1.0 / 2.3324673844012387,
                                        1.0 / 3.2752135590741402,
                                        1.0 / 4.3063288801167054};
__constant__ double kBlkpInvFact[33] = {1.0,
                                        1.0,
                                        0.5,
                                        1.6666666666666666e-01,
                                        4.1666666666666664e-02,
                                        8.3333333333333332e-03,
                                        1.3888888888888889e-03,
                                        1.9841269841269841e-04,
                                        2.4801587301587302e-05,
                                        2.7557319223985893e-06,
                                        2.7557319223985888e-07,
                                        2.5052108385441720e-08,
                                        2.0876756987868100e-09,
                                        1.6059043836821613e-10,
                                        1.1470745597729725e-11,
                                        7.6471637318198164e-13,
                                        4.7794773323873853e-14,
                                        2.8114572543455206e-15,
                                        1.5619206968586225e-16,
                                        8.2206352466243295e-18,
                                        4.1103176233121648e-19,
                                        1.9572941063391263e-20,
                                        8.8967913924505741e-22,
                                        3.8681701706306835e-23,
                                        1.6117375710961184e-24,
                                        6.4469502843844736e-26,
                                        2.4795962632247972e-27,
                                        9.1836898637955460e-29,
                                        3.2798892370698380e-30,
                                        1.1309962886447717e-31,
                                        3.7699876288159054e-33,
                                        1.2161250415535179e-34,
                                        3.8003907548547434e-36};

// position of U[r][c] (r, c < 16) in a slice's 256 entries: column quarter c & 3 of 64 entries, row group c >> 2 of 16,
// row r swizzled by c.  The forward lane (i, q) reads U[i][4q + t] at 64t + 16q + (i ^ (4q + t)), the backward lane
// reads U[4q + t][i] at 64(i & 3) + 16(i >> 2) + (i ^ (4q + t)): in either, the 16 lanes of a quarter hit 16 distinct
// 16-byte slots modulo 16 (no LDS bank conflicts), and one 1 KB DMA piece holds one column quarter.
__host__ __device__ constexpr int blkp_upos(int r, int c) { return 64 * (c & 3) + 16 * (c >> 2) + (r ^ c); }

struct BlkpArgs {
  int N, nu, nwb;
  int skew;                    // every Ã_j exactly skew-Hermitian (qoc_ctx::skew_exact, imaginary shifts)
  int four;                    // complex products from four real ones (QOC_BLKP_4M)
  int slack;                   // up to this many products more for each squaring fewer (QOC_BLKP_SLACK)
  // the truncation criterion with the squarings counted (tail > 0): s squarings amplify the degree-4r polynomial's
  // truncation R of exp(2^-s X) 2^s times (U = (e^{2^-s X} - R)^{2^s} = e^X - 2^s R + ..., ||e^{2^-s X}|| = 1), and over
  // the chain the slices' truncations add up coherently; so s is the fewest squarings with
  // tail_{4r}(2^-s ρ̂) <= 2^-53 2^-(s + tail), theta[r][s] the largest ρ meeting it (blkp_theta_table, host).
  // tail = 0: the plain bound tail_{4r}(2^-s ρ̂) <= 2^-53 of kBlkpTheta.
  int tail;
  double theta[BLKP_RMAX + 1][16];
  double rcap;                 // > 0: the accurate (r, s) choice, 2^-s ρ̂ <= rcap (QOC_BLKP_RCAP, default 1); 0: the
                               // fewest products (slack / tail)
  // skew-Hermitian blocks, Chebyshev form (k_blkp_exp<.., CM > 0>): the coefficient table (blkp_cheb_table, one row of
  // BLKP_CT_STRIDE doubles per grid point ρ_c(g) = 2^((g - BLKP_CT_G0) / 4), g < cgn <= ρ_c = crmax)
  const double* ctab;
  int cgn;
  double crmax;
  long long unit0, units;      // this launch's units [unit0, units) of B Nt nwb: unit = (b Nt + k) nwb + β
  const int* wrow;             // nwb x 16 rows of the live wave blocks
  const cx<double>* At;        // (nu+1) N x N shifted generators Ã_j, column-major
  const double* u;             // B x Nt x nu
  double mur[3], mui[3];       // μ_k = μ_0 + Σ_j u_j μ_j
  // U_k of the block (e^{μ_k} included), 256 entries per unit from unit ubase on: U[r][c] at blkp_upos(r, c), so that
  // a chain's four DMA pieces per slice read 1 KB contiguous each and both chains read their quarters from LDS without
  // bank conflicts (the eval keeps two seed groups' slabs, the split propagate every seed's)
  double2* UF;
  long long ubase;
  unsigned long long* prods;   // TERM_SLOTS counters: executed 16 x 16 complex products (nullptr: not counted)
};

using BV4 = MF<double>::v4;
struct CMat {  // 16 x 16 complex in the C layout
  BV4 r, i;
};

// Z = L R (+ I0): Lt = C layout of L^T, R and I0 in C layout; 3 real products (Zr = T1 - T2, Zi = T3 - T1 - T2 with
// T3 = (Lr + Li)(Rr + Ri)), the addend folded into the accumulators' start values
template <bool INIT>
__device__ __forceinline__ CMat cm_mul(const CMat& Lt, const CMat& R, const CMat& I0) {
  BV4 t1 = INIT ? I0.r : BV4{0.0, 0.0, 0.0, 0.0};
  BV4 t2 = BV4{0.0, 0.0, 0.0, 0.0};
  BV4 t3 = INIT ? I0.r + I0.i : BV4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const double ar = Lt.r[e], ai = Lt.i[e], br = R.r[e], bi = R.i[e];
    t1 = MF<double>::mma(ar, br, t1);
    t2 = MF<double>::mma(ai, bi, t2);
    t3 = MF<double>::mma(ar + ai, br + bi, t3);
  }
  return CMat{t1 - t2, t3 - t1 - t2};
}

// LDS traffic between the lanes of one wave: LDS operations of a wave complete in order, the fences keep the compiler
// from moving them across the exchange
__device__ __forceinline__ void blkp_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the same product from four real ones (16 MFMAs, no cancellation in the imaginary part)
template <bool INIT>
__device__ __forceinline__ CMat cm_mul4(const CMat& Lt, const CMat& R, const CMat& I0) {
  BV4 tr = INIT ? I0.r : BV4{0.0, 0.0, 0.0, 0.0};
  BV4 ti = INIT ? I0.i : BV4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    tr = MF<double>::mma(Lt.r[e], R.r[e], tr);
    ti = MF<double>::mma(Lt.r[e], R.i[e], ti);
    tr = MF<double>::mma(-Lt.i[e], R.i[e], tr);
    ti = MF<double>::mma(Lt.i[e], R.r[e], ti);
  }
  return CMat{tr, ti};
}
template <bool INIT>
__device__ __forceinline__ CMat cm_mulx(bool four, const CMat& Lt, const CMat& R, const CMat& I0) {
  return four ? cm_mul4<INIT>(Lt, R, I0) : cm_mul<INIT>(Lt, R, I0);
}

// C layout of X^T through the wave's LDS tile (row pitch 17: the transposed reads of a 16-lane row fall on distinct
// banks).  Within a wave LDS operations complete in order; the fences keep the compiler from moving them.
__device__ __forceinline__ CMat cm_transpose(const CMat& X, double2* tile) {
  const int l = threadIdx.x & 63, j = l & 15, g = l >> 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) tile[(g + 4 * e) * 17 + j] = make_double2(X.r[e], X.i[e]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  CMat T;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const double2 v = tile[j * 17 + g + 4 * e];
    T.r[e] = v.x;
    T.i[e] = v.y;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return T;
}

// v + v(lane ^ 16) and v + v(lane ^ 32) with the gfx950 row swaps (VALU, no LDS crossbar): each swap returns the two
// registers with the partner rows exchanged, so the two results hold v and its partner in some order
__device__ __forceinline__ double2 swap16_f64(double v) {
  const unsigned long long q = (unsigned long long)__double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)q, (unsigned)q, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(q >> 32), (unsigned)(q >> 32), false, false);
  return make_double2(__longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0])),
                      __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1])));
}
__device__ __forceinline__ double2 swap32_f64(double v) {
  const unsigned long long q = (unsigned long long)__double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)q, (unsigned)q, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(q >> 32), (unsigned)(q >> 32), false, false);
  return make_double2(__longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0])),
                      __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1])));
}
__device__ __forceinline__ double xsum_rows(double v) {  // over the four lanes i, i + 16, i + 32, i + 48
  double2 a = swap16_f64(v);
  v = a.x + a.y;
  a = swap32_f64(v);
  return a.x + a.y;
}
// both parts of a complex value at once (the two dependency chains interleaved)
__device__ __forceinline__ double2 xsum_rows2(double2 v) {
  double2 a = swap16_f64(v.x), b = swap16_f64(v.y);
  v = make_double2(a.x + a.y, b.x + b.y);
  a = swap32_f64(v.x);
  b = swap32_f64(v.y);
  return make_double2(a.x + a.y, b.x + b.y);
}
__device__ __forceinline__ double xmax_rows(double v) {
  double2 a = swap16_f64(v);
  v = fmax(a.x, a.y);
  a = swap32_f64(v);
  return fmax(a.x, a.y);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long q = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)q, CTRL, 0xf, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(q >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// over the 16 lanes of a DPP row (quad xor 1, quad xor 2, half mirror, mirror); the result in every lane
__device__ __forceinline__ double row_sum16(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  return v + dpp_f64<0x140>(v);
}
__device__ __forceinline__ double row_max16(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  return fmax(v, dpp_f64<0x140>(v));
}
__device__ __forceinline__ double uniform_f64(double v) {
  const unsigned long long q = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)q);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(q >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// B_i = c_{4i} I + c_{4i+1} X + c_{4i+2} X² + c_{4i+3} X³ (c_k = 1/k!)
__device__ __forceinline__ CMat blkp_horner_b(int i, const CMat& X, const CMat& X2, const CMat& X3) {
  const int l = threadIdx.x & 63, j = l & 15, g = l >> 4;
  const double c0 = kBlkpInvFact[4 * i], c1 = kBlkpInvFact[4 * i + 1], c2 = kBlkpInvFact[4 * i + 2],
               c3 = kBlkpInvFact[4 * i + 3];
  CMat B;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    B.r[e] = fma(c3, X3.r[e], fma(c2, X2.r[e], fma(c1, X.r[e], g + 4 * e == j ? c0 : 0.0)));
    B.i[e] = fma(c3, X3.i[e], fma(c2, X2.i[e], c1 * X.i[e]));
  }
  return B;
}

// ---- the Chebyshev form for skew-Hermitian blocks ----
// exp(X) for X = -i H (H Hermitian, ||H||_2 <= ρ̂): with s halvings (2^-s ρ̂ <= crmax) and the grid point ρ_c >= 2^-s ρ̂,
// Y = 2^-s H / ρ_c has its spectrum in [-1, 1], and the Jacobi-Anger series
//   exp(2^-s X) = exp(-i ρ_c Y) = J_0(ρ_c) + 2 Σ_{k>=1} (-i)^k J_k(ρ_c) T_k(Y)
// converges without cancellation (|T_k(Y)| <= 1, the Bessel coefficients decay): no e^ρ growth of the rounding as in
// the Taylor terms, and few or no squarings to amplify it.  Truncated at degree n (tail <= 2^-57, host), evaluated
// by block Clenshaw in Z = T_CM(Y): p = Σ_{q=0}^{Q} A_q(Y) T_q(Z), A_q = Σ_{j<CM} β_{q,j} (-i)^j T_j(Y) (the host's
// exact rewrite of the series, T_j T_{CM q} = (T_{CM q + j} + T_{CM q - j}) / 2; β real since CM is even), so CM - 1
// products for T_2..T_CM and Q for the recurrence b_q = A_q + 2 Z b_{q+1} - b_{q+2}, p = A_0 + Z b_1 - b_2.  Every left
// operand is Hermitian (its transpose is its conjugate): no LDS round trip but the squarings'.
// Table row: [ρ_c, 1 / ρ_c, Q, -, β[q][j] (q = 0..Q, j < CM)]
constexpr int BLKP_CT_STRIDE = 64, BLKP_CT_G0 = 32;

// (2 T)^T for a Hermitian T (the left operand of a product with 2 T)
__device__ __forceinline__ CMat blkp_herm2t(const CMat& T) {
  CMat o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    o.r[e] = 2.0 * T.r[e];
    o.i[e] = -2.0 * T.i[e];
  }
  return o;
}

template <int CM>
__device__ __forceinline__ CMat blkp_cheb(const CMat& X, double rho, const BlkpArgs& a, double2* tile, bool four,
                                          int& nprod) {
  const int l = threadIdx.x & 63, j = l & 15, g = l >> 4;
  int s = 0;
  double q = rho;
  while (s < 15 && q > a.crmax) {
    q *= 0.5;
    ++s;
  }
  // the smallest grid point ρ_c(gi) >= q (a float log2 guess, corrected against the table)
  int gi = q > 0.0 ? (int)ceilf(4.0f * __builtin_amdgcn_logf((float)q)) + BLKP_CT_G0 : 0;
  gi = min(max(gi, 0), a.cgn - 1);
  while (gi < a.cgn - 1 && a.ctab[(size_t)gi * BLKP_CT_STRIDE] < q) ++gi;
  while (gi > 0 && a.ctab[(size_t)(gi - 1) * BLKP_CT_STRIDE] >= q) --gi;
  gi = __builtin_amdgcn_readfirstlane(gi);
  const double* ct = a.ctab + (size_t)gi * BLKP_CT_STRIDE;
  const double sc = ldexp(ct[1], -s);
  const int Q = __builtin_amdgcn_readfirstlane((int)ct[2]);
  // T[1] = Y = i X sc (Hermitian), T[2..CM-1], Z = T_CM
  CMat T[CM];
  CMat mI, Z;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    T[1].r[e] = -X.i[e] * sc;
    T[1].i[e] = X.r[e] * sc;
    mI.r[e] = g + 4 * e == j ? -1.0 : 0.0;
    mI.i[e] = 0.0;
  }
  auto neg = [](const CMat& M) {
    CMat o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o.r[e] = -M.r[e];
      o.i[e] = -M.i[e];
    }
    return o;
  };
  // T_{a+b} = 2 T_a T_b - T_{|a-b|}
  T[2] = cm_mulx<true>(four, blkp_herm2t(T[1]), T[1], mI);
  T[3] = cm_mulx<true>(four, blkp_herm2t(T[1]), T[2], neg(T[1]));
  if constexpr (CM == 4) {
    Z = cm_mulx<true>(four, blkp_herm2t(T[2]), T[2], mI);
  } else {
    static_assert(CM == 6, "block size 4 or 6");
    T[4] = cm_mulx<true>(four, blkp_herm2t(T[2]), T[2], mI);
    T[5] = cm_mulx<true>(four, blkp_herm2t(T[2]), T[3], neg(T[1]));
    Z = cm_mulx<true>(four, blkp_herm2t(T[3]), T[3], mI);
  }
  // A_q = Σ_j β_{q,j} (-i)^j T_j, minus an addend D (the recurrence's b_{q+2})
  auto Aq = [&](int qq, const CMat& D) {
    const double* bq = ct + 4 + qq * CM;
    CMat A;
    const double b0 = bq[0];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      A.r[e] = (g + 4 * e == j ? b0 : 0.0) - D.r[e];
      A.i[e] = -D.i[e];
    }
#pragma unroll
    for (int jj = 1; jj < CM; ++jj) {
      const double b = bq[jj];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double tr = T[jj].r[e], ti = T[jj].i[e];
        switch (jj & 3) {  // (-i)^jj
          case 0: A.r[e] = fma(b, tr, A.r[e]); A.i[e] = fma(b, ti, A.i[e]); break;
          case 1: A.r[e] = fma(b, ti, A.r[e]); A.i[e] = fma(-b, tr, A.i[e]); break;
          case 2: A.r[e] = fma(-b, tr, A.r[e]); A.i[e] = fma(-b, ti, A.i[e]); break;
          default: A.r[e] = fma(-b, ti, A.r[e]); A.i[e] = fma(b, tr, A.i[e]); break;
        }
      }
    }
    return A;
  };
  CMat zero;
#pragma unroll
  for (int e = 0; e < 4; ++e) zero.r[e] = zero.i[e] = 0.0;
  CMat R;
  if (Q == 0) {
    R = Aq(0, zero);
  } else {
    const CMat Z2t = blkp_herm2t(Z);
    CMat b1 = Aq(Q, zero), b2 = zero;
    for (int qq = Q - 1; qq >= 1; --qq) {
      const CMat nb = cm_mulx<true>(four, Z2t, b1, Aq(qq, b2));
      b2 = b1;
      b1 = nb;
    }
    CMat Zt;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      Zt.r[e] = 0.5 * Z2t.r[e];
      Zt.i[e] = 0.5 * Z2t.i[e];
    }
    R = cm_mulx<true>(four, Zt, b1, Aq(0, b2));
  }
  for (int t = 0; t < s; ++t) {
    const CMat Rt = cm_transpose(R, tile);
    R = cm_mulx<false>(four, Rt, R, R);
  }
  nprod = CM - 1 + Q + s;
  return R;
}

// One workgroup of BLKP_WG / 64 waves walks the units wave by wave (persistent grid).  LDS: the generators' blocks in
// C layout ([β][j][e][lane] double2) and one transpose tile per wave.  CM > 0: skew-Hermitian blocks in the Chebyshev
// form (blkp_cheb, block size CM); 0: Taylor / Paterson-Stockmeyer and squarings.
// OCC: workgroups per CU the launch bound asks for (3: 168 VGPRs, 3 spilled; 2: 214 with AGPRs, no spills)
template <int NU, int OCC, int CM = 0>
__global__ __launch_bounds__(BLKP_WG, OCC) void k_blkp_exp(const BlkpArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double2* gen = reinterpret_cast<double2*>(smem);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, j = l & 15, g = l >> 4;
  const int N = a.N, nwb = a.nwb;
  const size_t NN = (size_t)N * N;
  const int ngen = nwb * 3 * 256;
  for (int e = tid; e < ngen; e += blockDim.x) {
    const int ll = e & 63, ee = (e >> 6) & 3, jb = e >> 8, jg = jb % 3, bb = jb / 3;
    const int* rb = a.wrow + 16 * bb;
    const int row = rb[(ll >> 4) + 4 * ee], col = rb[ll & 15];
    double2 v = make_double2(0.0, 0.0);
    if (row >= 0 && col >= 0 && jg <= NU) {
      const cx<double> z = a.At[jg * NN + row + (size_t)N * col];
      v = make_double2(z.r, z.i);
    }
    gen[e] = v;
  }
  double2* tile = gen + ngen + w * BLKP_TP;
  __syncthreads();
  const int WPG = BLKP_WG / 64;
  const long long TW = (long long)gridDim.x * WPG;
  unsigned long long prods = 0;
  const bool four = a.four != 0;
  for (long long unit = a.unit0 + (long long)blockIdx.x * WPG + w; unit < a.units; unit += TW) {
    const long long bk = unit / nwb;
    const int beta = (int)(unit - bk * nwb);
    const double u1 = a.u[bk * NU], u2 = NU > 1 ? a.u[bk * NU + (NU > 1 ? 1 : 0)] : 0.0;
    const double2* gb = gen + (size_t)beta * 768;
    CMat X;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const double2 g0 = gb[64 * e + l], g1 = gb[256 + 64 * e + l];
      const double2 g2 = NU > 1 ? gb[512 + 64 * e + l] : make_double2(0.0, 0.0);
      X.r[e] = fma(u2, g2.x, fma(u1, g1.x, g0.x));
      X.i[e] = fma(u2, g2.y, fma(u1, g1.y, g0.y));
    }
    // ρ̂ = sqrt(‖X‖_1 ‖X‖_∞) >= ‖X‖_2 with |re| + |im| >= |z| in the sums.  On the tunable bus it averages 14.70
    // against a spectral radius of 14.53 and the same products per unit as the exact radius (11.70); the Frobenius
    // norm (26.96) never came out smaller, so it is not formed
    double cs = 0.0, rmax = 0.0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const double az = fabs(X.r[e]) + fabs(X.i[e]);
      cs += az;
      rmax = fmax(rmax, row_sum16(az));  // row g + 4e
    }
    const double n1 = row_max16(xsum_rows(cs)), ninf = xmax_rows(rmax);
    const double rho = uniform_f64(sqrt(n1 * ninf));
    CMat R;
    int nprod = 0;
    if constexpr (CM > 0) {
      R = blkp_cheb<CM>(X, rho, a, tile, four, nprod);
    } else {
    // (the sharper α_p = max(‖X^p‖^{1/p}, ‖X^{p+1}‖^{1/(p+1)}) of Al-Mohy & Higham from the computed powers chose the
    // same (r, s) on the tunable bus -- 10.75 products per unit either way -- and cost three more reductions)
    int r = BLKP_RMAX, s = 0;
    if (a.rcap > 0.0) {
      // the accurate choice (default): halve until 2^-s ρ̂ <= rcap (1), then the smallest degree whose truncation,
      // amplified by the squarings, stays 2^-tail below an ulp (θ[r][s]).  The polynomial's rounding grows like
      // e^{2^-s ρ̂} (its terms cancel on the imaginary axis) and the squarings' like 2^s, so the pieces are kept near
      // norm 1: on the tunable bus (ρ̂ ≈ 14.7: r = 5, s = 4, 11 products) the bias of J over 2000 chained slices
      // against an extended-precision propagation drops ~5x from the fewest-products choice (tools/tb_truth.py)
      double q = rho;
      while (s < 15 && q > a.rcap) {
        q *= 0.5;
        ++s;
      }
      r = 0;
#pragma unroll
      for (int rr = BLKP_RMAX; rr >= BLKP_RMIN; --rr)
        if (q <= a.theta[rr][s]) r = rr;
      while (r == 0 && s < 15) {  // a cap above θ_{4 RMAX}: more halvings at the top degree
        q *= 0.5;
        ++s;
        if (q <= a.theta[BLKP_RMAX][s]) r = BLKP_RMAX;
      }
      if (r == 0) r = BLKP_RMAX;
    } else {
      // the fewest products r + 2 + s with 2^-s ρ̂ <= θ_{4r} (tail > 0: θ[r][s], the squarings counted), or (slack)
      // the fewest squarings within slack of that
      int ssel[BLKP_RMAX + 1];
      int best = 1 << 30;
#pragma unroll
      for (int rr = BLKP_RMIN; rr <= BLKP_RMAX; ++rr) {
        if (a.tail > 0) {  // the fewest s with 2^-s ρ̂ <= θ[r][s] (ρ̂ is wave-uniform: a scalar loop)
          int sq = 0;
          double q = rho;
          while (sq < 15 && q > a.theta[rr][sq]) {
            q *= 0.5;
            ++sq;
          }
          ssel[rr] = sq;
        } else {
          // s = max(0, ceil(log2(ρ̂ / θ))): with ρ̂ / θ = f 2^e, f in [0.5, 1), that is e, or e - 1 when f = 1/2
          const double q = rho * kBlkpInvTheta[rr];  // (a product: ρ̂ θ⁻¹ rounds the same side of 2^s but a few ulps)
          const int e = q > 1.0 ? __builtin_amdgcn_frexp_exp(q) : 0;
          ssel[rr] = q > 1.0 ? (__builtin_amdgcn_frexp_mant(q) == 0.5 ? e - 1 : e) : 0;
        }
        best = min(best, rr + 2 + ssel[rr]);
      }
      s = 1 << 30;
#pragma unroll
      for (int rr = BLKP_RMAX; rr >= BLKP_RMIN; --rr)
        if (rr + 2 + ssel[rr] <= best + a.slack && ssel[rr] < s) {
          s = ssel[rr];
          r = rr;
        }
      if (a.slack == 0) {  // the fewest products, the smaller r on ties
#pragma unroll
        for (int rr = BLKP_RMAX; rr >= BLKP_RMIN; --rr)
          if (rr + 2 + ssel[rr] == best) {
            s = ssel[rr];
            r = rr;
          }
      }
    }
    {
      const double sc = ldexp(1.0, -s);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        X.r[e] *= sc;
        X.i[e] *= sc;
      }
    }
    // X^T: for skew-Hermitian blocks -conj(X) (no LDS round trip), else through the tile
    CMat Xt;
    if (a.skew) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        Xt.r[e] = -X.r[e];
        Xt.i[e] = X.i[e];
      }
    } else {
      Xt = cm_transpose(X, tile);
    }
    const CMat X2 = cm_mulx<false>(four, Xt, X, X);
    const CMat X3 = cm_mulx<false>(four, Xt, X2, X);
    const CMat X4 = cm_mulx<false>(four, Xt, X3, X);
    CMat X4t;  // X^4 of a skew-Hermitian X is Hermitian: its transpose is conj(X^4)
    if (a.skew) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        X4t.r[e] = X4.r[e];
        X4t.i[e] = -X4.i[e];
      }
    } else {
      X4t = cm_transpose(X4, tile);
    }
    R = blkp_horner_b(r - 1, X, X2, X3);
    {
      const double cm = kBlkpInvFact[4 * r];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        R.r[e] = fma(cm, X4.r[e], R.r[e]);
        R.i[e] = fma(cm, X4.i[e], R.i[e]);
      }
    }
    for (int i = r - 2; i >= 0; --i) R = cm_mulx<true>(four, X4t, R, blkp_horner_b(i, X, X2, X3));
    for (int t = 0; t < s; ++t) {
      const CMat Rt = cm_transpose(R, tile);
      R = cm_mulx<false>(four, Rt, R, R);
    }
    nprod = r + 2 + s;
    }  // CM == 0
    const double mr = fma(u2, a.mur[2], fma(u1, a.mur[1], a.mur[0]));
    const double mi = fma(u2, a.mui[2], fma(u1, a.mui[1], a.mui[0]));
    const double em = a.skew ? 1.0 : exp(mr);  // skew-Hermitian blocks: imaginary shifts
    double sn, cn;
    sincos(mi, &sn, &cn);
    const double pr = em * cn, pi = em * sn;
    double2* const uf = a.UF + (unit - a.ubase) * 256;
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // this lane holds U[g + 4e][j]
      const double vr = fma(pr, R.r[e], -pi * R.i[e]), vi = fma(pr, R.i[e], pi * R.r[e]);
      uf[blkp_upos(g + 4 * e, j)] = make_double2(vr, vi);
    }
    prods += (unsigned long long)nprod;
  }
  if (a.prods && l == 0 && prods) atomicAdd(a.prods + (blockIdx.x & (TERM_SLOTS - 1)), prods);
}

// ---- one control: the propagators interpolated in u (k_blkp_int) ----
// With a single control (nu = 1, the tunable bus' flux) every slice propagator lies on one curve,
// U(u) = e^{μ(u)} exp(Ã_0 + u Ã_1), an entire function of the scalar u.  On the batch's control range [lo, hi] its
// Chebyshev expansion in ξ = (2u - lo - hi) / (hi - lo) converges super-exponentially (|c_i| ~ (ρ_1 w / 4)^i / i!,
// w = hi - lo), so a degree D ~ 20 reaches the ulp: exp(Ã_0 + u Ã_1) = Σ_{i<=D} T_i(ξ) M_i.  The host forms the D + 1
// coefficient matrices once per range (exponentials at 40 Chebyshev points in long double, then the discrete cosine
// transform: blkp_interp_setup); a unit is then D + 1 scaled sums of LDS-resident 16 x 16 matrices -- ~200 VALU
// instructions instead of 11 MFMA products -- and its accuracy is that of the interpolant (truncation < 2^-56, no
// squarings: tools/tb_truth.py).
struct BlkpIntArgs {
  int nwb, D;                  // live wave blocks, the largest interpolation degree (the coefficients' stride D + 1)
  int beta0, nb;               // this launch's blocks [beta0, beta0 + nb) (their coefficients fill the LDS)
  int Db[8];                   // each block's own degree (its coefficients alone decide it: a block's propagators do
                               // not depend on which other blocks the launch carries)
  long long slot0, slots;      // this launch's (seed, slice) slots [slot0, slots) of B Nt; unit = slot nwb + β
  long long ubase;             // the unit whose propagator sits at UF[0]
  const double* u;             // B x Nt (nu = 1)
  double xa, xb;               // ξ = xa u + xb
  double mur[2], mui[2];       // μ(u) = μ_0 + u μ_1
  int skew;                    // imaginary shifts: e^{μ} = e^{i Im μ}
  const double2* M;            // [β][i][p]: M_i of block β at the propagator store positions p = blkp_upos(r, c)
                               // (lane l, register e: p = 64 e + l), so that loads and stores are contiguous
  const double2* Msym;         // complex-symmetric generators: [i][slot] the packed upper triangle of block 0's nl
  int nl;                      // live rows (k_blkp_ichain<., true>, blkp_sym_slot), else nullptr / 0
  double2* ph;                 // B x Nt: e^{μ(u_k)} of every (seed, slice) (k_blkp_phase, read by k_blkp_ichain)
  double2* UF;
  unsigned long long* prods;   // counted as 0 products (none run)
};
__host__ __device__ inline size_t blkp_int_lds(int nwb, int D) { return (size_t)nwb * (D + 1) * 256 * sizeof(double2); }

// UPW consecutive slots of one block per wave: each M_i entry read from LDS once serves UPW units
template <int UPW, int WG>
__global__ __launch_bounds__(WG) void k_blkp_int(const BlkpIntArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double2* Ms = reinterpret_cast<double2*>(smem);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int nwb = a.nwb, D = a.D, nb = a.nb;
  for (int e = tid; e < nb * (D + 1) * 256; e += blockDim.x) Ms[e] = a.M[(size_t)a.beta0 * (D + 1) * 256 + e];
  __syncthreads();
  const long long nsg = (a.slots - a.slot0 + UPW - 1) / UPW, items = nsg * nb;
  for (long long it = (long long)blockIdx.x * (blockDim.x >> 6) + w; it < items; it += (long long)gridDim.x * (blockDim.x >> 6)) {
    const long long sg = it / nb;
    const int bl = (int)(it - sg * nb), beta = a.beta0 + bl;
    const long long s0 = a.slot0 + sg * UPW;
    double uu[UPW], xi[UPW], tm[UPW], tc[UPW];
    double ar[UPW][4], ai[UPW][4];
#pragma unroll
    for (int t = 0; t < UPW; ++t) {
      uu[t] = a.u[min(s0 + t, a.slots - 1)];
      xi[t] = fma(a.xa, uu[t], a.xb);
      tm[t] = 1.0;  // T_{i-1}
      tc[t] = 1.0;  // T_i (i = 0)
#pragma unroll
      for (int e = 0; e < 4; ++e) ar[t][e] = ai[t][e] = 0.0;
    }
    const double2* Mb = Ms + (size_t)bl * (D + 1) * 256 + l;
    const int Dq = a.Db[beta];
    for (int i = 0; i <= Dq; ++i) {
      double2 mv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) mv[e] = Mb[(size_t)i * 256 + 64 * e];
#pragma unroll
      for (int t = 0; t < UPW; ++t) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ar[t][e] = fma(tc[t], mv[e].x, ar[t][e]);
          ai[t][e] = fma(tc[t], mv[e].y, ai[t][e]);
        }
        // T_{i+1} = 2 ξ T_i - T_{i-1} (T_1 = ξ)
        const double tn = i == 0 ? xi[t] : fma(2.0 * xi[t], tc[t], -tm[t]);
        tm[t] = tc[t];
        tc[t] = tn;
      }
    }
#pragma unroll
    for (int t = 0; t < UPW; ++t) {
      const long long slot = s0 + t;
      if (slot >= a.slots) break;  // uniform
      const double mr = fma(uu[t], a.mur[1], a.mur[0]), mi = fma(uu[t], a.mui[1], a.mui[0]);
      const double em = a.skew ? 1.0 : exp(mr);
      double sn, cn;
      sincos(mi, &sn, &cn);
      const double pr = em * cn, pi = em * sn;
      double2* const uf = a.UF + (slot * nwb + beta - a.ubase) * 256;
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // store position 64 e + l (1 KB contiguous per store)
        const double vr = fma(pr, ar[t][e], -pi * ai[t][e]), vi = fma(pr, ai[t][e], pi * ar[t][e]);
        uf[64 * e + l] = make_double2(vr, vi);
      }
    }
  }
}

// min / max of n doubles: per block into part[2 blockIdx.x], [2 blockIdx.x + 1] (the host finishes)
static __global__ void k_minmax(const double* __restrict__ v, long long n, double* part) {
  double lo = __builtin_inf(), hi = -__builtin_inf();
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    lo = fmin(lo, v[e]);
    hi = fmax(hi, v[e]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off));
    hi = fmax(hi, __shfl_xor(hi, off));
  }
  __shared__ double sl[16], sh[16];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sl[w] = lo;
    sh[w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
      lo = fmin(lo, sl[i]);
      hi = fmax(hi, sh[i]);
    }
    part[2 * blockIdx.x] = lo;
    part[2 * blockIdx.x + 1] = hi;
  }
}

// ---- chains from the stored propagators ----
// The chains are bound by the propagators they read (4 KB per slice and direction, 8.4 GB per tunable-bus eval).  The
// slices run in chunks of CH: the propagator quarters of chunk c + 1 stream into the wave's LDS by LDS-DMA
// (global_load_lds_dwordx4, two buffers) while chunk c runs, and the new states collect in LDS and are stored at the
// next chunk start, so the slices touch LDS only and the one wait for memory per chunk (vmcnt(0), by hand: the
// compiler does not see the DMA) finds loads and stores a whole chunk old.  (Per-slice register prefetches did not
// work: the compiler's waits at the loop head also covered the newest loads.)  The gradient's products are not formed
// here (k_blkp_grad forms them from x_k and μ_{k+1}, all slices in parallel): with them every slice of the one wave per
// SIMD carried three times the dependent instructions (2.9 ms per tunable-bus eval against 0.9 ms without).
// LDS: [32 doubles scratch][x_N: 2 N m doubles][per wave, double2: exchange row 32 | new states CH x 16 |
// propagators 2 x CH x 4 x 64]
__host__ __device__ constexpr int blkp_wave_lds2(int CH) { return 32 + CH * 16 + 2 * CH * 256; }
__host__ __device__ inline size_t blkp_chain_lds(int N, int m, int waves, int CH) {
  return (size_t)(32 + 2 * N * m) * sizeof(double) + (size_t)waves * blkp_wave_lds2(CH) * sizeof(double2);
}
// slices per chunk (QOC_BLKP_CH overrides: 1, 2, 4, 8): one-wave chains (one live block, one state column: the tunable
// bus) at CH = 8, 69 KB of LDS each (with the trimmed formation beside them 64.25k vs 63.79k evals/s at CH = 4, same
// box, profiles/r05ab7/; before the trims the two measured the same), else the LDS of 4 chain waves per CU
__host__ __device__ inline int blkp_chunk(int waves, int parts = 1) {
  (void)parts;
  return waves <= 1 ? 8 : waves <= 2 ? 4 : waves <= 4 ? 2 : 1;
}
// 16 B per lane from src to LDS byte address lds + 16 lane (lds wave-uniform); M0 set and restored in the statement
__device__ __forceinline__ void blkp_dma(const void* src, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}

// this lane's view of wave block β: row rb[i] (i = lane & 15), quarter q = lane >> 4, state column c
struct BlkpLane {
  int i, q, beta, c, row;
  __device__ __forceinline__ void setup(const BlkArgs& bk) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    i = l & 15;
    q = l >> 4;
    beta = w % bk.nwb;
    c = w / bk.nwb;
    row = bk.wrow[16 * beta + i];
  }
};

// Σ_t a_t b_t (complex) over this lane's quarter, two partial sums per part; every fma spelled out, so that each
// chunk-size instantiation rounds alike (a free a b - c d is contracted either way round)
__device__ __forceinline__ double2 blkp_dot4(const double (&ar)[4], const double (&ai)[4], const double (&br)[4],
                                             const double (&bi)[4]) {
  const double r0 = fma(ar[0], br[0], fma(-ai[0], bi[0], fma(ar[1], br[1], -(ai[1] * bi[1]))));
  const double r1 = fma(ar[2], br[2], fma(-ai[2], bi[2], fma(ar[3], br[3], -(ai[3] * bi[3]))));
  const double i0 = fma(ar[0], bi[0], fma(ai[0], br[0], fma(ar[1], bi[1], ai[1] * br[1])));
  const double i1 = fma(ar[2], bi[2], fma(ai[2], br[2], fma(ar[3], bi[3], ai[3] * br[3])));
  return make_double2(r0 + r1, i0 + i1);
}

// FWD: x_{k+1} = U_k x_k (lane (i, q) reads U_k[i][4q + t]); else μ_k = U_k^H μ_{k+1} (lane (i, q) reads
// (U_k^H)[i][4q + t] = conj(U_k[4q + t][i])), μ_N = X_target (λ_k = coef ⊙ μ_k).  The forward ends with J and the λ_N
// coefficients.
template <bool FWD, int CH>
__device__ __forceinline__ void blkp_chain_body(const TChainArgs& g, const BlkArgs& bk, const double2* __restrict__ U,
                                                const int b, const int useed0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* red = reinterpret_cast<double*>(smem);
  double* xN = red + 32;
  const int N = g.N, m = g.m, Nt = g.Nt, nwb = bk.nwb, tid = threadIdx.x, nthr = blockDim.x, l = tid & 63;
  const size_t Nm = (size_t)N * m;
  BlkpLane ln;
  ln.setup(bk);
  double2* const xs = reinterpret_cast<double2*>(xN + 2 * Nm) + (tid >> 6) * blkp_wave_lds2(CH);
  double2* const Os = xs + 32;        // [jj][i]: x_{k+1} / μ_k of row i
  double2* const Ub2 = Os + CH * 16;  // [buffer][jj][t][lane]: this lane's propagator quarter of chunk slice jj
  const bool act = ln.row >= 0, own = act && ln.q == 0;
  double2* const sink2 = reinterpret_cast<double2*>(tchain_sink(g));
  const size_t oe = (size_t)ln.c * N + max(ln.row, 0);  // element offset (complex) of this lane's row
  double2* const Sb = reinterpret_cast<double2*>((cx<double>*)(FWD ? g.X : g.L) + (size_t)b * (Nt + 1) * Nm);
  if (FWD)
    for (size_t e = tid; e < 2 * Nm; e += nthr) xN[e] = 0.0;
  double2 v0 = make_double2(0.0, 0.0);
  if (act) {
    cx<double> v;
    if (FWD) v = ((const cx<double>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0))[oe];
    else v = ((const cx<double>*)g.Xt)[oe];
    v0 = make_double2(v.r, v.i);
  }
  xs[ln.i] = v0;
  __syncthreads();
  *(own ? Sb + (FWD ? 0 : (size_t)Nt * Nm) + oe : sink2) = v0;
  double xr[4], xi[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const double2 v = xs[4 * ln.q + t];
    xr[t] = v.x;
    xi[t] = v.y;
  }
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));  // per-lane (VGPR) source addresses
  const double2* Ubase = U + (size_t)(b - useed0) * Nt * nwb * 256 + (size_t)ln.beta * 256 + l + z;  // U: seed useed0's
  const size_t ustep = (size_t)nwb * 256;
  const unsigned ub_lds = (unsigned)(size_t)(__attribute__((address_space(3))) double2*)Ub2;
  int uo[4];  // this lane's four propagator entries within a slice's LDS copy
#pragma unroll
  for (int t = 0; t < 4; ++t) uo[t] = FWD ? blkp_upos(ln.i, 4 * ln.q + t) : blkp_upos(4 * ln.q + t, ln.i);
  // chunk cc's propagator quarters by DMA into buffer cc & 1 (1 KB contiguous per piece)
  auto issue = [&](int cc) __attribute__((always_inline)) {
#pragma unroll
    for (int jj = 0; jj < CH; ++jj) {
      const int j = cc * CH + jj;
      const int k = FWD ? min(j, Nt - 1) : max(Nt - 1 - j, 0);
      const double2* p = Ubase + (size_t)k * ustep;
      const unsigned dst =
          (unsigned)__builtin_amdgcn_readfirstlane((int)(ub_lds + (unsigned)((((cc & 1) * CH + jj) * 4) * 1024)));
#pragma unroll
      for (int t = 0; t < 4; ++t) blkp_dma(p + 64 * t, dst + t * 1024);
    }
  };
  typedef double D2V __attribute__((ext_vector_type(2)));
  using G2 = __attribute__((address_space(1))) D2V;
  // chunk cc's new states from LDS to HBM, branch-free (lanes without an element write the sink)
  auto flush = [&](int cc) __attribute__((always_inline)) {
#pragma unroll
    for (int jj = 0; jj < CH; ++jj) {
      const int j = cc * CH + jj;
      const int k = FWD ? j : Nt - 1 - j;
      G2* p = (G2*)(own && j < Nt ? Sb + (size_t)(FWD ? k + 1 : k) * Nm + oe : sink2);
      asm volatile("" : "+v"(p));
      const double2 v = Os[jj * 16 + ln.i];
      *p = D2V{v.x, v.y};
    }
  };
  issue(0);
  int c = 0;
  for (int j0 = 0; j0 < Nt; j0 += CH, ++c) {
    // chunk c's DMA and chunk c - 2's stores were issued a chunk ago
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    blkp_wave_sync();
    issue(c + 1);
    if (c > 0) flush(c - 1);
    blkp_wave_sync();
    const double2* const Us = Ub2 + (c & 1) * CH * 256;
    double ur[4], ui[4];  // slice jj's propagator quarter, read one slice ahead (off the chain's critical path)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const double2 pv = Us[uo[t]];
      ur[t] = pv.x;
      ui[t] = FWD ? pv.y : -pv.y;
    }
    for (int jj = 0; jj < CH; ++jj) {
      if (j0 + jj >= Nt) break;
      double2 y = blkp_dot4(ur, ui, xr, xi);
      const int jn = min(jj + 1, CH - 1);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double2 pv = Us[jn * 256 + uo[t]];
        ur[t] = pv.x;
        ui[t] = FWD ? pv.y : -pv.y;
      }
      y = xsum_rows2(y);
      xs[ln.i] = y;
      blkp_wave_sync();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double2 v = xs[4 * ln.q + t];
        xr[t] = v.x;
        xi[t] = v.y;
      }
      blkp_wave_sync();
      if (ln.q == 0) Os[jj * 16 + ln.i] = y;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) DMA must land before the LDS is reused
  blkp_wave_sync();
  flush(c - 1);
  if (FWD) {
    if (own) {  // x_N: the exchange row holds the last slice's result
      const double2 v = xs[ln.i];
      xN[2 * oe] = v.x;
      xN[2 * oe + 1] = v.y;
    }
    __syncthreads();
    chain_costs<double>(N, m, (const cx<double>*)g.Xt, [&](int o) { return cx<double>{xN[2 * o], xN[2 * o + 1]}; },
                        g.cost_kind, g.n_norm, 0.0, red, g.J + b, g.coef + (size_t)b * 2 * m, g.sc);
  }
}

// forward chain and μ recurrence of every seed in one launch of 2B workgroups (seed-direction interleave as
// k_blkrot_dual), nwb m waves each
// (seeds seed0 .. seed0 + gridDim.x / 2 - 1; U holds the propagators from seed useed0 on)
template <int CH>
__global__ __launch_bounds__(512) void k_blkp_dual(const TChainArgs gf, const TChainArgs gb, const BlkArgs bk,
                                                   const double2* __restrict__ U, int seed0, int useed0, int prio) {
  // beside the formation's MFMA waves the chain's dependent VALU steps would queue behind their MFMAs: the chain wave
  // can take the issue priority (prio, QOC_BLKP_PRIO)
  if (prio) __builtin_amdgcn_s_setprio(3);
  const int i = blockIdx.x, B = gridDim.x >> 1;
  const bool by8 = (B & 7) == 0;
  const int dir = by8 ? (i >> 3) & 1 : i & 1;
  const int seed = seed0 + (by8 ? ((i >> 4) << 3) | (i & 7) : i >> 1);
  if (dir == 0) blkp_chain_body<true, CH>(gf, bk, U, seed, useed0);
  else blkp_chain_body<false, CH>(gb, bk, U, seed, useed0);
}

// one direction alone (the reference's split call form: the forward chain in propagate, the μ recurrence in
// grape_sensitivity), one workgroup per seed seed0 + blockIdx.x; stale: a stale-u flag queued before the launch
// (nonzero: nothing is written)
template <bool FWD, int CH>
__global__ __launch_bounds__(512) void k_blkp_chain(const TChainArgs g, const BlkArgs bk, const double2* __restrict__ U,
                                                    int seed0, int useed0, const int* stale) {
  if (stale && *stale != 0) return;
  blkp_chain_body<FWD, CH>(g, bk, U, seed0 + (int)blockIdx.x, useed0);
}

// ---- one control, fused: the chains interpolate their own propagators (k_blkp_ichain) ----
// With the interpolation a propagator is D + 1 scaled sums of LDS-resident 16 x 16 matrices, which costs a chain wave
// less than storing it (4 KB) and reading it back (twice: forward and μ recurrence), and the four seed groups of the
// stored form left one chain wave per CU beside the formation.  Here one wave per (seed, direction) for one live wave
// block and one state column (the tunable bus): per chunk of SL slices the wave forms the SL propagators' entries in
// registers (each coefficient entry read once from LDS for the SL slices; k_blkp_int's arithmetic term by term), then
// runs the SL chain steps on them (blkp_chain_body's arithmetic), then stores the SL new states.  No propagator reaches
// HBM; all B seeds and both directions run at once (4 waves per workgroup, the coefficients in its LDS).  The
// forward's terminal cost is k_terminal_cost's (one 64-thread workgroup per seed: chain_costs as the chains' one-wave
// workgroups run it).
//   SYM: complex-symmetric generators (A_j^T = A_j: -i H Δt with H real symmetric, the tunable bus) give symmetric
// propagators, so only the nl (nl + 1) / 2 <= 128 entries of the upper triangle of the nl live rows are formed, two
// per lane (half the interpolation's FMAs), from packed coefficients [D + 1][128] (slot k of entry (a, b), a <= b:
// blkp_sym_slot); each slice's 128 entries go through a wave-private LDS slab to the lanes that apply them (lane (i, q)
// the entries (i, 4q + t) forward, their conjugates backward: U^H = conj(U)).  The host symmetrises the coefficients
// of such generators for every form (the stored one too), so both give the same bits.
// LDS: the coefficients [D + 1][256] (at blkp_upos positions) or [D + 1][128] (SYM) double2 | per wave: exchange row
// 32 | new states SL x 16 | SYM: the entry slab SL x 128 (double2)
__host__ __device__ constexpr int blkp_ichain_wave_lds(int SL, bool sym, int D) {
  return 32 + SL * 16 + (sym ? SL * 128 : 0) + (D + 1) * SL / 2;
}
__host__ __device__ inline size_t blkp_ichain_lds(int D, int SL, int waves, bool sym) {
  return ((size_t)(D + 1) * (sym ? 128 : 256) + (size_t)waves * blkp_ichain_wave_lds(SL, sym, D)) * sizeof(double2);
}
// slot of the upper-triangle entry (a, b), a <= b < nl, in the packed layout (row-major triangle)
__host__ __device__ constexpr int blkp_sym_slot(int a, int b, int nl) { return a * nl - a * (a - 1) / 2 + (b - a); }

// the interpolation of SL slices' propagator entries, NE per lane (k_blkp_int's arithmetic, term by term)
template <bool FWD, int SL, int NE>
struct BlkpIAcc {
  double ur[SL][NE], ui[SL][NE];
  // the Chebyshev values of slices j0 .. j0 + SL - 1 of this direction (clamped at the ends) into Ts[i SL + s]: lane
  // s < SL runs slice s's recurrence (k_blkp_int's, the same values), so the other lanes need not
  __device__ __forceinline__ void tvalues(const BlkpIntArgs& ia, const double* ub, int Nt, int j0, int D, double* Ts) {
    const int l = threadIdx.x & 63;
    if (l < SL) {
      const int j = j0 + l;
      const double x = fma(ia.xa, ub[FWD ? min(j, Nt - 1) : max(Nt - 1 - j, 0)], ia.xb);
      double tm = 1.0, tc = 1.0;
      for (int ti = 0; ti <= D; ++ti) {
        Ts[ti * SL + l] = tc;
        const double tn = ti == 0 ? x : fma(2.0 * x, tc, -tm);
        tm = tc;
        tc = tn;
      }
    }
#pragma unroll
    for (int s = 0; s < SL; ++s)
#pragma unroll
      for (int t = 0; t < NE; ++t) ur[s][t] = ui[s][t] = 0.0;
  }
  // terms [t0, t1) of Σ T_i(ξ) M_i: this lane's entries at off[] in each coefficient matrix of `stride` entries, the
  // T_i(ξ_s) read from Ts (one broadcast per two slices)
  __device__ __forceinline__ void terms(const double2* Ms, const int (&off)[NE], int stride, const double* Ts, int t0,
                                        int t1) {
#pragma unroll 2
    for (int ti = t0; ti < t1; ++ti) {
      double2 mv[NE];
#pragma unroll
      for (int t = 0; t < NE; ++t) mv[t] = Ms[ti * stride + off[t]];
      double tv[SL];
#pragma unroll
      for (int s = 0; s < SL; s += 2) {
        const double2 v = *reinterpret_cast<const double2*>(Ts + ti * SL + s);
        tv[s] = v.x;
        tv[s + 1] = v.y;
      }
#pragma unroll
      for (int s = 0; s < SL; ++s)
#pragma unroll
        for (int t = 0; t < NE; ++t) {
          ur[s][t] = fma(tv[s], mv[t].x, ur[s][t]);
          ui[s][t] = fma(tv[s], mv[t].y, ui[s][t]);
        }
    }
  }
  // times e^{μ(u)} (phs[s]: k_blkp_phase's); conj: the conjugates (the μ recurrence's U^H entries)
  __device__ __forceinline__ void finish(const double2 (&phs)[SL], bool conj) {
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      const double pr = phs[s].x, pi = phs[s].y;
#pragma unroll
      for (int t = 0; t < NE; ++t) {
        const double vr = fma(pr, ur[s][t], -pi * ui[s][t]), vi = fma(pr, ui[s][t], pi * ur[s][t]);
        ur[s][t] = vr;
        ui[s][t] = conj ? -vi : vi;
      }
    }
  }
};

constexpr int BLKP_ISLB = 2;  // SYM: slices per pass through the entry slab (its LDS: BLKP_ISLB x 128 double2 per wave)
// One chain wave's view of its (seed, direction): state rows, output and sink pointers, this lane's entries
template <bool FWD, int SL, bool SYM>
struct BlkpIChain {
  static constexpr int NE = SYM ? 2 : 4;
  static constexpr int SLB = SL < BLKP_ISLB ? SL : BLKP_ISLB;  // SYM: slices per pass through the entry slab
  int Nt, l, i, q;
  bool act, own;
  size_t Nm, oe;
  double2 *Sb, *sink2;
  const double* ub;
  const double2* phb;
  int off[NE];  // this lane's entries in a coefficient matrix
  int ks[4];    // SYM: the packed slots of this lane's four entries (i, 4q + t), -1: a padding row or column
  __device__ __forceinline__ void setup(const TChainArgs& g, const BlkArgs& bk, const BlkpIntArgs& ia, int b) {
    Nt = g.Nt;
    l = threadIdx.x & 63;
    i = l & 15;
    q = l >> 4;
    Nm = (size_t)g.N;  // one state column
    const int row = bk.wrow[i];  // wave block 0
    act = row >= 0;
    own = act && q == 0;
    oe = (size_t)max(row, 0);
    Sb = reinterpret_cast<double2*>((cx<double>*)(FWD ? g.X : g.L) + (size_t)b * (Nt + 1) * Nm);
    sink2 = reinterpret_cast<double2*>(tchain_sink(g));
    ub = ia.u + (size_t)b * Nt;
    phb = ia.ph + (size_t)b * Nt;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * q + t, a = min(i, c), bb = max(i, c);
      ks[t] = bb < ia.nl ? blkp_sym_slot(a, bb, ia.nl) : -1;
    }
#pragma unroll
    for (int t = 0; t < NE; ++t) off[t] = SYM ? 64 * t + l : FWD ? blkp_upos(i, 4 * q + t) : blkp_upos(4 * q + t, i);
  }
  // x_0 / μ_N into the exchange row xs and to HBM
  __device__ __forceinline__ void init(const TChainArgs& g, double2* xs, int b) {
    double2 v0 = make_double2(0.0, 0.0);
    if (act) {
      cx<double> v;
      if (FWD) v = ((const cx<double>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0))[oe];
      else v = ((const cx<double>*)g.Xt)[oe];
      v0 = make_double2(v.r, v.i);
    }
    xs[i] = v0;
    *(own ? Sb + (FWD ? 0 : (size_t)Nt * Nm) + oe : sink2) = v0;
  }
  // the propagator entries this lane applies in slices j0 .. j0 + SL - 1 (k_blkp_int's arithmetic term by term; SYM:
  // the packed entries through the slab Es)
  __device__ __forceinline__ void form(const BlkpIntArgs& ia, const double2* Ms, double2* Es, double* Ts, int j0,
                                       double (&ur)[SL][4], double (&ui)[SL][4]) {
    BlkpIAcc<FWD, SL, NE> a;
    double2 phs[SL];  // the slices' e^{μ(u)}, loaded with the controls, used after the terms
#pragma unroll
    for (int s = 0; s < SL; ++s) phs[s] = phb[FWD ? min(j0 + s, Nt - 1) : max(Nt - 1 - j0 - s, 0)];
    a.tvalues(ia, ub, Nt, j0, ia.Db[0], Ts);
    blkp_wave_sync();
    a.terms(Ms, off, SYM ? 128 : 256, Ts, 0, ia.Db[0] + 1);
    blkp_wave_sync();  // Ts is rewritten by the next chunk
    a.finish(phs, !SYM && !FWD);
    if constexpr (SYM) {
#pragma unroll
      for (int s0 = 0; s0 < SL; s0 += SLB) {
#pragma unroll
        for (int s = 0; s < SLB; ++s)
#pragma unroll
          for (int t = 0; t < NE; ++t) Es[s * 128 + 64 * t + l] = make_double2(a.ur[s0 + s][t], a.ui[s0 + s][t]);
        blkp_wave_sync();
#pragma unroll
        for (int s = 0; s < SLB; ++s)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const double2 v = ks[t] >= 0 ? Es[s * 128 + ks[t]] : make_double2(0.0, 0.0);
            ur[s0 + s][t] = v.x;
            ui[s0 + s][t] = FWD ? v.y : -v.y;
          }
        blkp_wave_sync();
      }
    } else {
#pragma unroll
      for (int s = 0; s < SL; ++s)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          ur[s][t] = a.ur[s][t];
          ui[s][t] = a.ui[s][t];
        }
    }
  }
  // the chunk's chain steps from the state in the exchange row xs (blkp_chain_body's arithmetic); the new states to
  // Os, the last one left in xs
  __device__ __forceinline__ void steps(const double (&ur)[SL][4], const double (&ui)[SL][4], double2* xs, double2* Os,
                                        int j0) {
    double xr[4], xi[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const double2 v = xs[4 * q + t];
      xr[t] = v.x;
      xi[t] = v.y;
    }
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      if (j0 + s >= Nt) break;  // uniform
      double2 y = blkp_dot4(ur[s], ui[s], xr, xi);
      y = xsum_rows2(y);
      blkp_wave_sync();  // every lane has read the row
      xs[i] = y;
      blkp_wave_sync();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double2 v = xs[4 * q + t];
        xr[t] = v.x;
        xi[t] = v.y;
      }
      if (q == 0) Os[s * 16 + i] = y;
    }
    blkp_wave_sync();
  }
  // the chunk's new states to HBM, branch-free (lanes without an element write the sink)
  __device__ __forceinline__ void flush(const double2* Os, int j0) {
    typedef double D2V __attribute__((ext_vector_type(2)));
    using G2 = __attribute__((address_space(1))) D2V;
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      const int j = j0 + s;
      const int k = FWD ? j : Nt - 1 - j;
      G2* p = (G2*)(own && j < Nt ? Sb + (size_t)(FWD ? k + 1 : k) * Nm + oe : sink2);
      asm volatile("" : "+v"(p));
      const double2 v = Os[s * 16 + i];
      *p = D2V{v.x, v.y};
    }
  }
};

// one wave per (seed, direction): form, steps, flush, chunk after chunk
template <bool FWD, int SL, bool SYM>
__device__ __forceinline__ void blkp_ichain_body(const TChainArgs& g, const BlkArgs& bk, const BlkpIntArgs& ia,
                                                 const double2* Ms, double2* xs, const int b) {
  BlkpIChain<FWD, SL, SYM> cw;
  cw.setup(g, bk, ia, b);
  double2* const Os = xs + 32;       // [s][i]: x_{k+1} / μ_k of row i
  double2* const Es = Os + SL * 16;  // SYM: [s][slot] the slices' packed entries
  double* const Ts = reinterpret_cast<double*>(Es + (SYM ? SL * 128 : 0));  // [i][s] the chunk's T_i(ξ_s)
  cw.init(g, xs, b);
  blkp_wave_sync();
  for (int j0 = 0; j0 < g.Nt; j0 += SL) {
    double ur[SL][4], ui[SL][4];
    cw.form(ia, Ms, Es, Ts, j0, ur, ui);
    cw.steps(ur, ui, xs, Os, j0);
    cw.flush(Os, j0);
    blkp_wave_sync();  // Os and Es are rewritten by the next chunk
  }
}

// two waves per (seed, direction), on one SIMD (waves w and w + 4 of an 8-wave workgroup): wave role r takes the
// chunks c = r, r + 2, ...; it forms chunk c's propagator entries, waits until its partner has run chunk c - 1 (the
// pair's chunk counter in LDS), runs chunk c's steps from the state the partner left in the pair's exchange row at the
// top issue priority, stores the chunk's states and publishes c + 1.  So one wave's latency-bound chain steps run while
// the other forms the next chunk on the same SIMD.
template <bool FWD, int SL, bool SYM>
__device__ __forceinline__ void blkp_ichain_pair_body(const TChainArgs& g, const BlkArgs& bk, const BlkpIntArgs& ia,
                                                      const double2* Ms, double2* xs, int* flag, double2* wl,
                                                      const int role, const int b) {
  BlkpIChain<FWD, SL, SYM> cw;
  cw.setup(g, bk, ia, b);
  double2* const Os = wl;            // this wave's [s][i]
  double2* const Es = Os + SL * 16;  // SYM: this wave's slab
  double* const Ts = reinterpret_cast<double*>(Es + (SYM ? BLKP_ISLB * 128 : 0));  // [i][s] the chunk's T_i(ξ_s)
  const int Nt = g.Nt, C = (Nt + SL - 1) / SL;
  for (int c = role; c < C; c += 2) {
    const int j0 = c * SL;
    double ur[SL][4], ui[SL][4];
    cw.form(ia, Ms, Es, Ts, j0, ur, ui);
    if (c == 0) {
      cw.init(g, xs, b);
    } else {
      while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < c) __builtin_amdgcn_s_sleep(1);
    }
    blkp_wave_sync();
    __builtin_amdgcn_s_setprio(2);
    cw.steps(ur, ui, xs, Os, j0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the exchange row is written before the counter
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(flag, c + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    cw.flush(Os, j0);
    blkp_wave_sync();
  }
}

// e^{μ(u_k)} of every (seed, slice), as k_blkp_int forms it (the two chain directions of a seed share them)
static __global__ void k_blkp_phase(const BlkpIntArgs ia, long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const double uu = ia.u[e];
    const double mr = fma(uu, ia.mur[1], ia.mur[0]), mi = fma(uu, ia.mui[1], ia.mui[0]);
    const double em = ia.skew ? 1.0 : exp(mr);
    double sn, cn;
    sincos(mi, &sn, &cn);
    ia.ph[e] = make_double2(em * cn, em * sn);
  }
}

// nseeds seeds from seed0 on; dual: both directions (wave pair 2 s + d: seed seed0 + s, d = 0 forward, 1 μ), else
// the direction dir alone; every wave passes the coefficients' barrier before it may leave
template <int SL, bool SYM>
__global__ __launch_bounds__(256) void k_blkp_ichain(const TChainArgs gf, const TChainArgs gb, const BlkArgs bk,
                                                     const BlkpIntArgs ia, int seed0, int nseeds, int dual, int dir,
                                                     const int* stale) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (stale && *stale != 0) return;  // uniform over the grid
  double2* const Ms = reinterpret_cast<double2*>(smem);
  const int D = ia.D, tid = threadIdx.x, w = tid >> 6, msz = (D + 1) * (SYM ? 128 : 256);
  const double2* const src = SYM ? ia.Msym : ia.M;
  for (int e = tid; e < msz; e += blockDim.x) Ms[e] = src[e];
  __syncthreads();
  double2* const xs = Ms + msz + (size_t)w * blkp_ichain_wave_lds(SL, SYM, D);
  const int p = (int)blockIdx.x * (int)(blockDim.x >> 6) + w;
  if (p >= (dual ? 2 : 1) * nseeds) return;
  const int s = dual ? p >> 1 : p, d = dual ? p & 1 : dir;
  if (d == 0) blkp_ichain_body<true, SL, SYM>(gf, bk, ia, Ms, xs, seed0 + s);
  else blkp_ichain_body<false, SL, SYM>(gb, bk, ia, Ms, xs, seed0 + s);
}

// the paired form: npw pairs per workgroup of 2 npw waves (blockDim.x = 128 npw), pair (w, w + npw) = (seed,
// direction) npw blockIdx.x + w % npw (npw = 4: the two waves of a pair on one SIMD; npw = 2 when the pairs would
// fill only half the CUs, the single-direction launches at B = 512); LDS: the coefficients | per pair: exchange row
// 32 + counter | per wave: new states SL x 16 | SYM: slab BLKP_ISLB x 128 (double2)
__host__ __device__ constexpr int blkp_ipair_wave_lds(int SL, bool sym, int D) {
  return SL * 16 + (sym ? BLKP_ISLB * 128 : 0) + (D + 1) * SL / 2;
}
__host__ __device__ inline size_t blkp_ipair_lds(int D, int SL, bool sym, int npw) {
  return ((size_t)(D + 1) * (sym ? 128 : 256) + (size_t)npw * 34 + 2 * (size_t)npw * blkp_ipair_wave_lds(SL, sym, D)) *
         sizeof(double2);
}
template <int SL, bool SYM>
__global__ __launch_bounds__(512) void k_blkp_ichain2(const TChainArgs gf, const TChainArgs gb, const BlkArgs bk,
                                                      const BlkpIntArgs ia, int seed0, int nseeds, int dual, int dir,
                                                      const int* stale) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (stale && *stale != 0) return;  // uniform over the grid
  double2* const Ms = reinterpret_cast<double2*>(smem);
  const int D = ia.D, tid = threadIdx.x, w = tid >> 6, msz = (D + 1) * (SYM ? 128 : 256);
  const double2* const src = SYM ? ia.Msym : ia.M;
  for (int e = tid; e < msz; e += blockDim.x) Ms[e] = src[e];
  const int npw = (int)(blockDim.x >> 7), pw = w % npw;
  double2* const pr = Ms + msz + 34 * pw;  // the pair's exchange row (32) and counter
  int* const flag = reinterpret_cast<int*>(pr + 32);
  if (w < npw && (tid & 63) == 0) *flag = 0;
  __syncthreads();
  double2* const wl = Ms + msz + npw * 34 + (size_t)w * blkp_ipair_wave_lds(SL, SYM, D);
  const int p = (int)blockIdx.x * npw + pw;
  if (p >= (dual ? 2 : 1) * nseeds) return;  // both waves of the pair
  const int s = dual ? p >> 1 : p, d = dual ? p & 1 : dir;
  if (d == 0) blkp_ichain_pair_body<true, SL, SYM>(gf, bk, ia, Ms, pr, flag, wl, w / npw, seed0 + s);
  else blkp_ichain_pair_body<false, SL, SYM>(gb, bk, ia, Ms, pr, flag, wl, w / npw, seed0 + s);
}

// ---- the order-3 gradient on the stored states (the reference's expm_jacobian! + _compute_u_sensitivity,
// src/gradient_computations.jl:177-223): with A_k = Σ_j u_jk A_j (unshifted generators), P_1 = A_k x_k,
// P_2 = A_k P_1, Q_1 = A_k^H λ_{k+1}, Q_2 = A_k^H Q_1, W_0 = λ + Q_1 / 2 + Q_2 / 6, W_1 = λ / 2 + Q_1 / 6:
//   dJ/du_jk = Re[<W_0, A_j x_k> + <W_1, A_j P_1> + <λ / 6, A_j P_2>]
// One wave per (seed, 16 consecutive slices): the 16 slices are the columns of 16 x 16 complex matrices in the C
// layout (lane j + 16 g: slice k0 + j, block rows g + 4e), so every generator product is a 16 x 16 x 16 GEMM on MFMA
// with the generator block as the left operand (from LDS) and the per-slice u_jk a per-lane scale; summed over the
// live blocks and state columns.  λ = coef ⊙ μ (the μ recurrence's coefficients).
struct BlkpGradArgs {
  int N, m, Nt, nwb;
  const int* wrow;           // nwb x 16 rows of the live wave blocks
  const cx<double>* A;       // (nu+1) N x N unshifted generators, column-major
  const double* u;           // B x Nt x nu
  const cx<double>* X;       // B x (Nt+1) x N x m states
  const cx<double>* L;       // μ_k, same layout
  const cx<double>* coef;    // B x 2m λ_N coefficients
  double* dJdu;              // B x Nt x nu
  long long tiles;           // B ceil(Nt / 16)
  const int* stale;          // a stale-u flag queued before the launch (nonzero: nothing is written), or nullptr
  cx<double>* coef_out;      // a copy of coef (qoc_get_costates' λ = coef ⊙ μ), written by workgroup 0, or nullptr
  unsigned diag;             // bit j: A_j (j >= 1) diagonal on the live wave blocks' rows (the tunable bus' flux term):
                             // its products are row scalings on the VALU instead of 12 MFMAs
};
__host__ __device__ inline size_t blkp_grad_lds(int nwb, int nu) { return (size_t)nwb * (nu + 1) * 2 * 256 * sizeof(double2); }

__device__ __forceinline__ double blkp_redot(const CMat& W, const CMat& Y) {  // Re Σ conj(W) Y over this lane's entries
  double a = 0.0;
#pragma unroll
  for (int e = 0; e < 4; ++e) a = fma(W.r[e], Y.r[e], fma(W.i[e], Y.i[e], a));
  return a;
}
__device__ __forceinline__ void blkp_axpy(CMat& Y, double a, const CMat& X) {  // Y += a X
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    Y.r[e] = fma(a, X.r[e], Y.r[e]);
    Y.i[e] = fma(a, X.i[e], Y.i[e]);
  }
}

template <int NU>
__global__ __launch_bounds__(256, 2) void k_blkp_grad(const BlkpGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (a.stale && *a.stale != 0) return;
  double2* gen = reinterpret_cast<double2*>(smem);  // [β][j][form][e][lane]: form 0 A_j, form 1 A_j^H as left operands
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, jl = l & 15, g = l >> 4;
  const int N = a.N, m = a.m, Nt = a.Nt, nwb = a.nwb;
  if (a.coef_out && blockIdx.x == 0) {
    const long long nc = a.tiles / ((Nt + 15) / 16) * 2 * m;  // B 2m
    for (long long e = tid; e < nc; e += blockDim.x) a.coef_out[e] = a.coef[e];
  }
  const size_t NN = (size_t)N * N, Nm = (size_t)N * m;
  const int ngen = nwb * (NU + 1) * 2 * 256;
  for (int e = tid; e < ngen; e += blockDim.x) {
    const int ll = e & 63, ee = (e >> 6) & 3, form = (e >> 8) & 1, jg = (e >> 9) % (NU + 1), bb = (e >> 9) / (NU + 1);
    const int* rb = a.wrow + 16 * bb;
    const int r1 = rb[ll & 15], r2 = rb[(ll >> 4) + 4 * ee];
    double2 v = make_double2(0.0, 0.0);
    if (r1 >= 0 && r2 >= 0) {  // form 0: A[r1][r2]; form 1: conj(A[r2][r1])
      const cx<double> z = form == 0 ? a.A[jg * NN + r1 + (size_t)N * r2] : a.A[jg * NN + r2 + (size_t)N * r1];
      v = make_double2(z.r, form == 0 ? z.i : -z.i);
    }
    gen[e] = v;
  }
  __syncthreads();
  const int T16 = (Nt + 15) >> 4;
  for (long long tile = (long long)blockIdx.x * 4 + w; tile < a.tiles; tile += (long long)gridDim.x * 4) {
    const int b = (int)(tile / T16), k0 = (int)(tile - (long long)b * T16) * 16;
    const int kj = k0 + jl, kc = min(kj, Nt - 1);
    double uj[NU];
#pragma unroll
    for (int q = 0; q < NU; ++q) uj[q] = a.u[((size_t)b * Nt + kc) * NU + q];
    double acc[NU];
#pragma unroll
    for (int q = 0; q < NU; ++q) acc[q] = 0.0;
    for (int beta = 0; beta < nwb; ++beta) {
      const int* rb = a.wrow + 16 * beta;
      int rows[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) rows[e] = rb[g + 4 * e];
      const double2* G = gen + (size_t)beta * (NU + 1) * 512;
      // a generator operand from LDS at each use (an opaque lane index: hoisted out of the loops, the 2 (nu + 1)
      // operands would hold 16 (nu + 1) VGPRs for the whole kernel)
      auto op = [&](int jg, int form) __attribute__((always_inline)) {
        CMat M;
        int ll = l;
        asm volatile("" : "+v"(ll));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double2 v = G[(jg * 2 + form) * 256 + 64 * e + ll];
          M.r[e] = v.x;
          M.i[e] = v.y;
        }
        return M;
      };
      // diagonal A_{q+1}: this lane's rows' entries (A_j^H: the conjugates)
      double dr[NU][4], di[NU][4];
#pragma unroll
      for (int q = 0; q < NU; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const cx<double> z = rows[e] >= 0 && ((a.diag >> (q + 1)) & 1u)
                                   ? a.A[(size_t)(q + 1) * NN + rows[e] + (size_t)N * rows[e]] : cx<double>{0.0, 0.0};
          dr[q][e] = z.r;
          di[q][e] = z.i;
        }
      // A_{q+1} M (form 0) or A_{q+1}^H M (form 1)
      auto mulA = [&](int q, int form, const CMat& M) __attribute__((always_inline)) {
        if ((a.diag >> (q + 1)) & 1u) {  // uniform
          CMat Y;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const double zi = form ? -di[q][e] : di[q][e];
            Y.r[e] = fma(dr[q][e], M.r[e], -(zi * M.i[e]));
            Y.i[e] = fma(dr[q][e], M.i[e], zi * M.r[e]);
          }
          return Y;
        }
        return cm_mul<false>(op(q + 1, form), M, M);
      };
      for (int c = 0; c < m; ++c) {
        const cx<double> cf = a.coef[(size_t)b * 2 * m + c];
        const cx<double>* xb = a.X + ((size_t)b * (Nt + 1) + kc) * Nm + (size_t)c * N;  // x_k
        const cx<double>* lb = a.L + ((size_t)b * (Nt + 1) + kc + 1) * Nm + (size_t)c * N;  // μ_{k+1}
        CMat X, Lm;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = rows[e] >= 0;
          const cx<double> xv = ok ? xb[rows[e]] : cx<double>{0.0, 0.0};
          const cx<double> mv = ok ? lb[rows[e]] : cx<double>{0.0, 0.0};
          X.r[e] = xv.r;
          X.i[e] = xv.i;
          Lm.r[e] = cf.r * mv.r - cf.i * mv.i;
          Lm.i[e] = cf.r * mv.i + cf.i * mv.r;
        }
        // the co-state side: Q_1 = A_k^H λ, Q_2 = A_k^H Q_1
        CMat Q1 = cm_mul<false>(op(0, 1), Lm, Lm);
#pragma unroll
        for (int q = 0; q < NU; ++q) blkp_axpy(Q1, uj[q], mulA(q, 1, Lm));
        CMat Q2 = cm_mul<false>(op(0, 1), Q1, Q1);
#pragma unroll
        for (int q = 0; q < NU; ++q) blkp_axpy(Q2, uj[q], mulA(q, 1, Q1));
        CMat W0, W1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          W0.r[e] = Lm.r[e] + 0.5 * Q1.r[e] + (1.0 / 6.0) * Q2.r[e];
          W0.i[e] = Lm.i[e] + 0.5 * Q1.i[e] + (1.0 / 6.0) * Q2.i[e];
          W1.r[e] = 0.5 * Lm.r[e] + (1.0 / 6.0) * Q1.r[e];
          W1.i[e] = 0.5 * Lm.i[e] + (1.0 / 6.0) * Q1.i[e];
          Lm.r[e] *= 1.0 / 6.0;
          Lm.i[e] *= 1.0 / 6.0;
        }
        // the state side: <W_0, A_j x>, P_1, <W_1, A_j P_1>, P_2, <λ/6, A_j P_2>
        CMat P1 = cm_mul<false>(op(0, 0), X, X);
#pragma unroll
        for (int q = 0; q < NU; ++q) {
          const CMat Y = mulA(q, 0, X);
          acc[q] += blkp_redot(W0, Y);
          blkp_axpy(P1, uj[q], Y);
        }
        CMat P2 = cm_mul<false>(op(0, 0), P1, P1);
#pragma unroll
        for (int q = 0; q < NU; ++q) {
          const CMat Y = mulA(q, 0, P1);
          acc[q] += blkp_redot(W1, Y);
          blkp_axpy(P2, uj[q], Y);
        }
#pragma unroll
        for (int q = 0; q < NU; ++q) acc[q] += blkp_redot(Lm, mulA(q, 0, P2));
      }
    }
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      const double v = xsum_rows(acc[q]);
      if (g == 0 && kj < Nt) a.dJdu[((size_t)b * Nt + kj) * NU + q] = v;
    }
  }
}

}  // namespace qoc
