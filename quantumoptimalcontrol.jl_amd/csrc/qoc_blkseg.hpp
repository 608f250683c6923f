// qoc_blkseg.hpp — one evaluation (propagate + J + grape_sensitivity) on block propagators with the time axis cut
// into segments, so that the serial depth per seed is about 2 Nt / S + log2 S instead of 2 Nt.
//
// The reference's two chains are serial in k (src/gradient_computations.jl:27-29 forward, :52-58 co-states); only
// the exponentials are parallel (:17-25).  With generators whose invariant blocks have <= 3 rows (qoc_blk.hpp: cavity
// 20 blocks of 2, zz 3 blocks of 3) every U_k is block-diagonal, and one block of it costs as much to form as to
// apply.  One workgroup per seed; lane (s, β) owns block β of segment s = slices [s L, s L + L):
//   phase 0  step records of every slice (e^{μ_k}, 2^-J u_k) into LDS, J and the Taylor degree P from the seed's
//            largest ρ_k (one pair for the whole seed: every lane runs the same term loop);
//   phase 1  the segment product P_s = U_{sL+L-1} .. U_{sL} on the block (U_k formed per slice, the k_blku_* block
//            exponential: Taylor polynomial in the Cayley-Hamilton basis with the phase folded in);
//   phase 2  inclusive prefix products Q_s = P_s .. P_0 over the segments (a Hillis-Steele scan inside each wave,
//            then the earlier waves' totals; one workgroup barrier),
//            x_N = Q_{S-1} x_0, the terminal cost J and λ_N (chain_costs, src/penalty_fcns.jl:15-42), then
//            G_N = Σ_c x_N,c λ_N,c^H per block;
//   phase 3  every segment backwards from its end, with G_k = Σ_c x_k,c λ_k,c^H instead of the states: because U_k is
//            unitary (skew-Hermitian generators; the host checks them exactly),
//              K_k = Σ_c x_k λ_{k+1}^H = U_k^H G_{k+1},    G_k = K_k U_k,
//            and G at the segment's end is Q_s G_0 Q_s^H with G_0 = Q_{S-1}^H G_N Q_{S-1}.  The gradient of the slice is
//            the trace form of expm_jacobian! + _compute_u_sensitivity (:177-223, blku_contract) on K_k:
//              dJ/du_jk = Re tr(A_j M_k),  M = Σ_{a+b<ORD} X^b K X^a / (a+b+1)!,  X = A_k,
//            summed over the slice's blocks (a wave-private LDS slot, fixed order: no atomics).
// Neither x_k, λ_k nor U_k go to HBM: the launch reads u and writes J, the λ_N coefficients and dJdu.  qoc_get_states
// and qoc_get_costates rebuild x_k / λ_k on demand with the k_blku_* chains (qoc_run_blk.hip).
//
// The reference's own call form runs the two halves apart: Ipopt's f calls propagate, its f_grad grape_sensitivity
// (examples/ipopt_callbacks_exp.jl:11-31; f alone in every line-search trial).  MODE splits the launch at the end of
// phase 2 (BLKSEG_FWD: phases 0-2, which also write G at every segment's end, Q_s G_0 Q_s^H, to HBM: S nblk NB^2
// complex per seed, 31 KB at cavity size) and BLKSEG_BWD (phase 0's records and (J, P) again -- the same arithmetic on
// the same u, so the same values -- then phase 3 from those G): bitwise the fused launch's J and dJdu.
#pragma once
#include "qoc_blku.hpp"

namespace qoc {

struct BlksegParams {
  double rad[3];               // ρ_k = rad[0] + Σ_j |u_jk| rad[j] (spectral half-widths of the shifted generators)
  double mur[3], mui[3];       // shifts μ_j: Ã_j = A_j - μ_j I, e^{μ_k} = exp(μ_0 + Σ_j u_jk μ_j)
  double theta_cap;            // ρ / 2^J <= theta_cap
  int S;                       // segments per seed
  int L;                       // slices per segment (S L >= Nt; the last segment may be shorter)
  int UPW;                     // segments per wave (64 / nblk)
  int RB;                      // slice-steps per block-sum reduction (blkseg_rb)
  const double* u;             // B x Nt x nu controls (the caller's buffer)
  double* u_copy;              // copies of u written by the launch (the stale check, the lazy rebuilds), or nullptr
  double* u_copy2;
  double* J2;                  // a second copy of J (the caller's), or nullptr
  cx<double>* coef2;           // a second copy of the λ_N coefficients (the lazy co-states), or nullptr
  double* dJdu;                // B x Nt x nu
  unsigned long long* terms;   // Σ P 2^J per pass over the slices (executed Taylor terms), nullptr: not counted
  // the best (J, global seed) of this launch for qoc_allgather_best_dev (the last workgroup to publish its J reduces
  // them; done counts the published ones and is reset by that workgroup), or nullptr
  unsigned int* done;
  double* best;
  long long seed_offset;
  // nothing to exchange (one rank): the final pair also into the context's result slot and the registered output
  // (qoc_set_best_output), or nullptr
  double* best_res;
  double* best_out;
  // the split launches: G at every segment's end, B x [NB^2][S][nblk] complex (written by BLKSEG_FWD, read by
  // BLKSEG_BWD); stale: the stale-u flag of the check queued before BLKSEG_BWD (nonzero: the launch writes nothing)
  double2* gseg;
  const int* stale;
};
enum { BLKSEG_FUSED = 0, BLKSEG_FWD = 1, BLKSEG_BWD = 2 };

// LDS, in doubles: shifted generator blocks [nblk][3][E] complex | step records [Nt][4] | segment products [S][E][nblk]
// complex | G_0 [E][nblk] complex | x_0 then x_N (N m complex) | λ_N coefficients (2 m complex) | scratch (24) |
// per-wave partial sums [W][RB][64][2] | dJdu [Nt][nu]
__host__ __device__ inline size_t blkseg_off_rec(int NB, int nblk) { return (size_t)6 * NB * NB * nblk; }
__host__ __device__ inline size_t blkseg_off_slot(int NB, int nblk, int Nt) { return blkseg_off_rec(NB, nblk) + 4 * (size_t)Nt; }
__host__ __device__ inline size_t blkseg_off_g0(int NB, int nblk, int Nt, int S) {
  return blkseg_off_slot(NB, nblk, Nt) + (size_t)2 * S * NB * NB * nblk;
}
__host__ __device__ inline size_t blkseg_off_xN(int NB, int nblk, int Nt, int S) {
  return blkseg_off_g0(NB, nblk, Nt, S) + (size_t)2 * NB * NB * nblk;
}
__host__ __device__ inline size_t blkseg_off_cf(int N, int m, int NB, int nblk, int Nt, int S) {
  return blkseg_off_xN(NB, nblk, Nt, S) + (size_t)2 * N * m;
}
__host__ __device__ inline size_t blkseg_off_red(int N, int m, int NB, int nblk, int Nt, int S) {
  return blkseg_off_cf(N, m, NB, nblk, Nt, S) + (size_t)4 * m;
}
__host__ __device__ inline size_t blkseg_off_wred(int N, int m, int NB, int nblk, int Nt, int S) {
  return blkseg_off_red(N, m, NB, nblk, Nt, S) + 32;  // red[0..23]: reductions, red[24..31]: wave progress
}
__host__ __device__ inline size_t blkseg_off_dJ(int N, int m, int NB, int nblk, int Nt, int S, int W, int RB) {
  return blkseg_off_wred(N, m, NB, nblk, Nt, S) + (size_t)128 * W * RB;
}
__host__ __device__ inline size_t blkseg_lds(int N, int m, int nu, int NB, int nblk, int Nt, int S, int W, int RB) {
  return (blkseg_off_dJ(N, m, NB, nblk, Nt, S, W, RB) + (size_t)Nt * nu) * sizeof(double);
}
// slice-steps whose block sums are reduced together (phase 3): as many as the reducing lanes of one wave allow
// (RB x segments per wave x controls <= 64), at most 4
__host__ __device__ inline int blkseg_rb(int upw, int nu) {
  const int r = 64 / (upw * (nu > 0 ? nu : 1));
  return r < 1 ? 1 : r > 4 ? 4 : r;
}

// Diagnostic per-wave stamps (tools/blkseg_probe.hip, -DQOC_PROBE): workgroup 7, wave w: phase 1 ends at
// g_segw[w], phase 3 at g_segw[16 + w] (cycles from the workgroup's start)
#ifdef QOC_PROBE
static __device__ unsigned long long g_segw[32];
#define SEGW_SET(slot, v)                                                        \
  do {                                                                           \
    if (blockIdx.x == 7 && (threadIdx.x & 63) == 0) g_segw[slot] = (v);          \
  } while (0)
static __device__ int g_seg_noturn, g_seg_turnmode;
#define SEG_TURNS (!g_seg_noturn)
#define SEG_TURNMODE g_seg_turnmode
#else
#define SEG_TURNS true
#define SEG_TURNMODE 1
#define SEGW_SET(slot, v) \
  do {                    \
  } while (0)
#endif

// launch bounds: WMAX = 8 waves (2 per SIMD, <= 256 VGPRs: the lane's generator blocks in registers) or 12 (3 per
// SIMD, <= 168 VGPRs: generator blocks read from LDS where used)

// c = a b, c = a^H b, c = a b^H on NB x NB complex blocks (row-major)
template <int NB, bool AH, bool BH>
__device__ __forceinline__ void seg_mm(const double (&ar)[NB * NB], const double (&ai)[NB * NB], const double (&br)[NB * NB],
                                       const double (&bi)[NB * NB], double (&cr)[NB * NB], double (&ci)[NB * NB]) {
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      double sr = 0.0, si = 0.0;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int ea = AH ? q * NB + i : i * NB + q, eb = BH ? k * NB + q : q * NB + k;
        const double xr = ar[ea], xi = AH ? -ai[ea] : ai[ea];
        const double yr = br[eb], yi = BH ? -bi[eb] : bi[eb];
        sr = fma(xr, yr, fma(-xi, yi, sr));
        si = fma(xr, yi, fma(xi, yr, si));
      }
      cr[i * NB + k] = sr;
      ci[i * NB + k] = si;
    }
}

// cos x and sin x / x as polynomials in x^2 (Horner, a fixed degree BLKSEG_KMAX = 9: the terms of exp(B) up to
// B^19, whose tail is below 2^-53 for every |x| <= θ_cap ≈ 0.98, so at least the Taylor polynomial's degree P; a
// fixed count keeps the loop free of branches and uniform masks)
constexpr int BLKSEG_KMAX = 9;
struct BlksegTrig {
  double c[BLKSEG_KMAX + 1];  // (-1)^k / (2k)!
  double s[BLKSEG_KMAX + 1];  // (-1)^k / (2k+1)!
};
// The series degree K (terms up to x^(2K+1)) a seed needs: the first omitted term ρ^(2K+2) / (2K+2)! below 2^-53 for
// every |x| <= ρ (both ω and |t| are bounded by the seed's largest ρ_k: the eigenvalues i(t ± ω) of a shifted block lie
// within [-ρ, ρ]).  K = 5 up to ρ = 0.24, 7 up to 0.66, else 9 (covers θ_cap ≈ 0.98); the bounds leave margin
// (exact limits 0.248 / 0.684 / 1.32).
__host__ __device__ constexpr int blkseg_series_k(double rho) { return rho <= 0.24 ? 5 : rho <= 0.66 ? 7 : BLKSEG_KMAX; }
constexpr BlksegTrig blkseg_trig() {
  BlksegTrig t{};
  double f = 1.0;  // 1 / n!
  for (int n = 0; n <= 2 * BLKSEG_KMAX + 1; ++n) {
    if (n > 0) f /= n;
    const double sg = (n / 2) % 2 ? -1.0 : 1.0;
    if (n % 2 == 0) t.c[n / 2] = sg * f;
    else t.s[n / 2] = sg * f;
  }
  return t;
}

// Â = 2^-J Ã_k on the lane's block and U_k = e^{μ_k} (p(Â))^{2^J} for NV slices at once (independent recurrences
// interleaved); rk[v]: the slice's record [Re e^μ, Im e^μ, 2^-J u_1, 2^-J u_2]; gen(j, e): entry e of Ã_j's block.
// P and J are uniform over the workgroup (k_blkseg_eval's phase 0).
template <int NB, int NV, typename GEN>
__device__ __forceinline__ void seg_form(GEN&& gen, const double* const (&rk)[NV], double s0, int P, int J,
                                         double (&ar)[NV][NB * NB], double (&ai)[NV][NB * NB], double (&ur)[NV][NB * NB],
                                         double (&ui)[NV][NB * NB]) {
  constexpr int E = NB * NB;
  double pr[NV], pi[NV], qr[NV], qi[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const double2 ph = *reinterpret_cast<const double2*>(rk[v]);
    const double2 su = *reinterpret_cast<const double2*>(rk[v] + 2);
    qr[v] = ph.x;
    qi[v] = ph.y;
    pr[v] = J ? 1.0 : ph.x;
    pi[v] = J ? 0.0 : ph.y;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 g0 = gen(0, e), g1 = gen(1, e), g2 = gen(2, e);
      ar[v][e] = fma(su.y, g2.x, fma(su.x, g1.x, s0 * g0.x));
      ai[v][e] = fma(su.y, g2.y, fma(su.x, g1.y, s0 * g0.y));
    }
  }
  if constexpr (NB == 2) {
    if (J == 0) {
      // blocks of 2 rows without halvings: the closed form.  Â is exactly skew-Hermitian (the host checks the
      // generators exactly; the scaled sums keep it so): Â = i t I + B with Â_00 = i (t + a), Â_11 = i (t - a),
      // B_01 = Â_01, B_10 = Â_10 = -conj(Â_01), B^2 = -ω^2 I, ω^2 = a^2 + |Â_01|^2, so
      //   exp(Â) = e^{i t} (cos ω I + (sin ω / ω) B)
      // with |t|, ω <= ρ <= θ_cap (the eigenvalues i (t ± ω) of Â lie within ±i ρ_k): both series to degree 19,
      // beyond the Taylor polynomial's P, so U_k agrees with it to rounding
      constexpr BlksegTrig T = blkseg_trig();
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const double t = 0.5 * (ai[v][0] + ai[v][3]), a = 0.5 * (ai[v][0] - ai[v][3]);
        const double w = fma(a, a, fma(ar[v][1], ar[v][1], ai[v][1] * ai[v][1])), t2 = t * t;
        double cw = 0.0, sw = 0.0, ct = 0.0, st = 0.0;
#pragma unroll
        for (int k = BLKSEG_KMAX; k >= 0; --k) {
          cw = fma(cw, w, T.c[k]);
          sw = fma(sw, w, T.s[k]);
          ct = fma(ct, t2, T.c[k]);
          st = fma(st, t2, T.s[k]);
        }
        st *= t;  // sin t
        // z = e^{μ_k} e^{i t};  U = z cos ω I + z sinc ω B
        const double zr = qr[v] * ct - qi[v] * st, zi = fma(qr[v], st, qi[v] * ct);
        const double cr = zr * cw, ci = zi * cw, sr = zr * sw, si = zi * sw;
        ur[v][0] = fma(-si, a, cr);
        ui[v][0] = fma(sr, a, ci);
        ur[v][3] = fma(si, a, cr);
        ui[v][3] = fma(-sr, a, ci);
        ur[v][1] = fma(sr, ar[v][1], -si * ai[v][1]);
        ui[v][1] = fma(sr, ai[v][1], si * ar[v][1]);
        ur[v][2] = fma(sr, ar[v][2], -si * ai[v][2]);
        ui[v][2] = fma(sr, ai[v][2], si * ar[v][2]);
      }
      return;
    }
  }
  blku_taylor<NB, NV>(ar, ai, P, pr, pi, nullptr, ur, ui);
  if (J) {  // squarings on the phase-free polynomial, then the phase
    for (int q = 0; q < J; ++q)
#pragma unroll
      for (int v = 0; v < NV; ++v) blku_square<NB>(ur[v], ui[v]);
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double vr = ur[v][e], vi = ui[v][e];
        ur[v][e] = qr[v] * vr - qi[v] * vi;
        ui[v][e] = qr[v] * vi + qi[v] * vr;
      }
  }
}

// Re tr(A_j M) for j = 1, 2 with M = Σ_{a+b<ORD} X^b K X^a / (a+b+1)! (blku_contract's recurrence: L_0 = R_0 = K,
// R_n = R_{n-1} X, L_n = X L_{n-1} + R_n, M = Σ_n L_n / (n+1)!) from the slice's X = A_k and the shifted generator
// blocks: A_j = Ã_j + μ_j I, so Re tr(A_j M) = Re tr(Ã_j M) + Re(μ_j tr M).  The traces are accumulated order by
// order (Re tr(A_j L_n) / (n+1)!), so that M is never held: three NB x NB matrices live (K -> L, R, X) instead of
// four.  K is overwritten.
template <int NB, typename GEN>
__device__ __forceinline__ void seg_trace(GEN&& gen, const double (&Lr)[NB * NB], const double (&Li)[NB * NB], double f,
                                          double m1r, double m1i, double m2r, double m2i, double& acc1, double& acc2) {
  double a1 = 0.0, a2 = 0.0, tr = 0.0, ti = 0.0;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    tr += Lr[i * NB + i];
    ti += Li[i * NB + i];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const double2 g1 = gen(1, i * NB + q), g2 = gen(2, i * NB + q);
      a1 = fma(g1.x, Lr[q * NB + i], fma(-g1.y, Li[q * NB + i], a1));
      a2 = fma(g2.x, Lr[q * NB + i], fma(-g2.y, Li[q * NB + i], a2));
    }
  }
  acc1 = fma(f, fma(m1r, tr, fma(-m1i, ti, a1)), acc1);
  acc2 = fma(f, fma(m2r, tr, fma(-m2i, ti, a2)), acc2);
}

// MACC: accumulate M = Σ_n L_n / (n+1)! and take the traces once (fewer flops, one more live matrix: blocks of 2
// rows); otherwise the traces order by order (blocks of 3 rows, where the registers are short)
template <int NB, int ORD, bool MACC, typename GEN>
__device__ __forceinline__ void seg_contract(GEN&& gen, const double (&xr_)[NB * NB], const double (&xi_)[NB * NB],
                                             double (&Lr)[NB * NB], double (&Li)[NB * NB], double m1r, double m1i,
                                             double m2r, double m2i, double& acc1, double& acc2) {
  constexpr int E = NB * NB;
  constexpr double invf[6] = {1.0, 1.0, 0.5, 1.0 / 6, 1.0 / 24, 1.0 / 120};
  acc1 = acc2 = 0.0;
  double Mr[MACC ? E : 1], Mi[MACC ? E : 1];
  if constexpr (MACC) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      Mr[e] = Lr[e];
      Mi[e] = Li[e];
    }
  } else {
    seg_trace<NB>(gen, Lr, Li, 1.0, m1r, m1i, m2r, m2i, acc1, acc2);
  }
  if constexpr (ORD > 1) {
    double Rr[E], Ri[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      Rr[e] = Lr[e];
      Ri[e] = Li[e];
    }
#pragma unroll
    for (int n = 1; n < ORD; ++n) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {  // R_n = R_{n-1} X, row by row in place
        double tr[NB], ti[NB];
#pragma unroll
        for (int kk = 0; kk < NB; ++kk) {
          double sr = 0.0, si = 0.0;
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            sr = fma(Rr[i * NB + q], xr_[q * NB + kk], fma(-Ri[i * NB + q], xi_[q * NB + kk], sr));
            si = fma(Rr[i * NB + q], xi_[q * NB + kk], fma(Ri[i * NB + q], xr_[q * NB + kk], si));
          }
          tr[kk] = sr;
          ti[kk] = si;
        }
#pragma unroll
        for (int kk = 0; kk < NB; ++kk) {
          Rr[i * NB + kk] = tr[kk];
          Ri[i * NB + kk] = ti[kk];
        }
      }
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {  // L_n = X L_{n-1} + R_n, column by column in place
        double tr[NB], ti[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          double sr = Rr[i * NB + kk], si = Ri[i * NB + kk];
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            sr = fma(xr_[i * NB + q], Lr[q * NB + kk], fma(-xi_[i * NB + q], Li[q * NB + kk], sr));
            si = fma(xr_[i * NB + q], Li[q * NB + kk], fma(xi_[i * NB + q], Lr[q * NB + kk], si));
          }
          tr[i] = sr;
          ti[i] = si;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          Lr[i * NB + kk] = tr[i];
          Li[i * NB + kk] = ti[i];
          if constexpr (MACC) {
            Mr[i * NB + kk] = fma(invf[n + 1], tr[i], Mr[i * NB + kk]);
            Mi[i * NB + kk] = fma(invf[n + 1], ti[i], Mi[i * NB + kk]);
          }
        }
      }
      if constexpr (!MACC) seg_trace<NB>(gen, Lr, Li, invf[n + 1], m1r, m1i, m2r, m2i, acc1, acc2);
    }
  }
  if constexpr (MACC) seg_trace<NB>(gen, Mr, Mi, 1.0, m1r, m1i, m2r, m2i, acc1, acc2);
}

// ---- blocks of 2 rows, exactly skew-Hermitian: [[i d0, r + i q], [-r + i q, i d1]] (4 reals instead of 8) ----
struct Sk2 {
  double d0, d1, r, q;
};
__device__ __forceinline__ Sk2 sk2_of(const double2 (&e)[4]) { return Sk2{e[0].y, e[3].y, e[1].x, e[1].y}; }

// cos t and sin t of the block's mean diagonal t = (d0 + d1) / 2 (sk2_form's series)
template <int K = BLKSEG_KMAX>
__device__ __forceinline__ void sk2_phase(double d0, double d1, double& ct, double& st) {
  constexpr BlksegTrig T = blkseg_trig();
  const double t = 0.5 * (d0 + d1), t2 = t * t;
  ct = 0.0;
  st = 0.0;
#pragma unroll
  for (int k = K; k >= 0; --k) {
    ct = fma(ct, t2, T.c[k]);
    st = fma(st, t2, T.s[k]);
  }
  st *= t;
}
// ZD with constant shifts: z = e^{μ_0} e^{it} of the lane's block, the same in every slice (rec[0..1]: e^{μ_0})
template <int K = BLKSEG_KMAX>
__device__ __forceinline__ void sk2_z(const Sk2& g0, const double* rec, double& zr, double& zi) {
  double ct, st;
  sk2_phase<K>(g0.d0, g0.d1, ct, st);
  const double2 ph = *reinterpret_cast<const double2*>(rec);
  zr = ph.x * ct - ph.y * st;
  zi = fma(ph.x, st, ph.y * ct);
}
// Â = Ã_0 + u_1 Ã_1 + u_2 Ã_2 (no halvings) and U = e^{μ_k} exp(Â) in the closed form of seg_form (ph = e^{μ_k}).
// ZD: the control generators' blocks have zero diagonals and no shifts, so Â's diagonal is Ã_0's and e^{μ_k} = e^{μ_0}
// in every slice: z = e^{μ_k} e^{it} comes precomputed (ct0, st0: sk2_z, the same value)
template <int K = BLKSEG_KMAX, bool ZD = false>
__device__ __forceinline__ void sk2_form(const Sk2 (&g)[3], double2 ph, double2 u, Sk2& ah, double (&ur)[4],
                                         double (&ui)[4], double ct0 = 1.0, double st0 = 0.0, double a0 = 0.0) {
  constexpr BlksegTrig T = blkseg_trig();
  if constexpr (ZD) {  // the same values (u_j times a zero diagonal adds nothing)
    ah.d0 = g[0].d0;
    ah.d1 = g[0].d1;
  } else {
    ah.d0 = fma(u.y, g[2].d0, fma(u.x, g[1].d0, g[0].d0));
    ah.d1 = fma(u.y, g[2].d1, fma(u.x, g[1].d1, g[0].d1));
  }
  ah.r = fma(u.y, g[2].r, fma(u.x, g[1].r, g[0].r));
  ah.q = fma(u.y, g[2].q, fma(u.x, g[1].q, g[0].q));
  const double a = ZD ? a0 : 0.5 * (ah.d0 - ah.d1);  // (ZD: a0 the same value, once per lane)
  const double w = fma(a, a, fma(ah.r, ah.r, ah.q * ah.q));
  double cw = 0.0, sw = 0.0, ct = ct0, st = st0;
#pragma unroll
  for (int k = K; k >= 0; --k) {
    cw = fma(cw, w, T.c[k]);
    sw = fma(sw, w, T.s[k]);
  }
  if constexpr (!ZD) sk2_phase<K>(ah.d0, ah.d1, ct, st);
  // z = e^{μ_k} e^{it}; ZD (constant shifts too): the same in every slice, (ct0, st0) hold it
  const double zr = ZD ? ct0 : ph.x * ct - ph.y * st, zi = ZD ? st0 : fma(ph.x, st, ph.y * ct);
  const double cr = zr * cw, ci = zi * cw, sr = zr * sw, si = zi * sw;
  ur[0] = fma(-si, a, cr);
  ui[0] = fma(sr, a, ci);
  ur[3] = fma(si, a, cr);
  ui[3] = fma(-sr, a, ci);
  ur[1] = fma(sr, ah.r, -si * ah.q);  // z sinc(ω) (r + i q)
  ui[1] = fma(sr, ah.q, si * ah.r);
  ur[2] = fma(-sr, ah.r, -si * ah.q);  // z sinc(ω) (-r + i q)
  ui[2] = fma(sr, ah.q, -si * ah.r);
}

// R <- R X in place, X skew-Hermitian (x0, x1, yr + i yq): 12 FMAs per row instead of 16
__device__ __forceinline__ void sk2_rx(double (&Rr)[4], double (&Ri)[4], const Sk2& x) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double p0r = Rr[2 * i], p0i = Ri[2 * i], p1r = Rr[2 * i + 1], p1i = Ri[2 * i + 1];
    Rr[2 * i] = fma(-p0i, x.d0, fma(-p1r, x.r, -p1i * x.q));
    Ri[2 * i] = fma(p0r, x.d0, fma(p1r, x.q, -p1i * x.r));
    Rr[2 * i + 1] = fma(p0r, x.r, fma(-p0i, x.q, -p1i * x.d1));
    Ri[2 * i + 1] = fma(p0r, x.q, fma(p0i, x.r, p1r * x.d1));
  }
}
// L <- X L + R in place, X skew-Hermitian
__device__ __forceinline__ void sk2_xlr(double (&Lr)[4], double (&Li)[4], const double (&Rr)[4], const double (&Ri)[4],
                                        const Sk2& x) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const double c0r = Lr[k], c0i = Li[k], c1r = Lr[2 + k], c1i = Li[2 + k];
    Lr[k] = fma(-x.d0, c0i, fma(x.r, c1r, fma(-x.q, c1i, Rr[k])));
    Li[k] = fma(x.d0, c0r, fma(x.r, c1i, fma(x.q, c1r, Ri[k])));
    Lr[2 + k] = fma(-x.r, c0r, fma(-x.q, c0i, fma(-x.d1, c1i, Rr[2 + k])));
    Li[2 + k] = fma(-x.r, c0i, fma(x.q, c0r, fma(x.d1, c1r, Ri[2 + k])));
  }
}
// Re tr(A_j M) for j = 1, 2 with M = Σ_{a+b<ORD} X^b K X^a / (a+b+1)! (seg_contract's recurrence on skew X) and
// A_j = Ã_j + i m_j I: -(d0 + m) Im M00 - (d1 + m) Im M11 + r (Re M10 - Re M01) - q (Im M10 + Im M01); e_j = (d0 + m,
// d1 + m, r, q) of each generator.  K is overwritten.
template <int ORD>
__device__ __forceinline__ void sk2_contract(const Sk2& x, const Sk2& e1, const Sk2& e2, double (&Lr)[4],
                                             double (&Li)[4], double& acc1, double& acc2) {
  constexpr double invf[6] = {1.0, 1.0, 0.5, 1.0 / 6, 1.0 / 24, 1.0 / 120};
  double Mr[4], Mi[4], Rr[4], Ri[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    Mr[e] = Rr[e] = Lr[e];
    Mi[e] = Ri[e] = Li[e];
  }
#pragma unroll
  for (int n = 1; n < ORD; ++n) {
    sk2_rx(Rr, Ri, x);
    sk2_xlr(Lr, Li, Rr, Ri, x);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      Mr[e] = fma(invf[n + 1], Lr[e], Mr[e]);
      Mi[e] = fma(invf[n + 1], Li[e], Mi[e]);
    }
  }
  const double dr = Mr[2] - Mr[1], di = Mi[2] + Mi[1];
  acc1 = fma(-e1.d0, Mi[0], fma(-e1.d1, Mi[3], fma(e1.r, dr, -e1.q * di)));
  acc2 = fma(-e2.d0, Mi[0], fma(-e2.d1, Mi[3], fma(e2.r, dr, -e2.q * di)));
}

// The same traces for ORD <= 3 in the Pauli basis.  With X = i(x0 I + x.σ) (x real: x0 = (d0 + d1)/2, x = (q, r,
// (d0 - d1)/2)), K = k0 I + k.σ (complex) and A_j = i(a0 I + a.σ), Re tr(A_j M) = -2 (a0 Im m0 + a.Im m), and the
// order-ORD M = Σ_{a+b<ORD} X^b K X^a / (a+b+1)! has (d = x.k, ω² = |x|²)
//   ORD 2: Im m0 = Im k0 + x0 Re k0 + Re d,  Im m = Im k + x0 Re k + Re k0 x
//   ORD 3: Im m0 = (1 - (x0² + ω²)/2) Im k0 + x0 (Re k0 - Im d) + Re d,
//          Im m = (1 - x0²/2 - ω²/6) Im k + x0 Re k + (Re k0 - x0 Im k0 - Im d / 3) x
// (the Pauli products (x.σ)(k.σ)(x.σ) = 2 (x.k) x.σ - ω² k.σ etc.; checked against the matrix recurrence in numpy).
// ~73 flops instead of sk2_contract's 224 at order 3.  aj: the generators' Pauli vectors times 2 (pre-scaled so that
// the K components below can stay doubled: 2 k0 = K00 + K11, ...).
// CX: X's diagonal is the same in every slice (zero-diagonal controls, zero control shifts): x0, x3 and x0² come
// precomputed (x0c, x3c, x02c: the same values)
template <int ORD, bool CX = false>
__device__ __forceinline__ void sk2_contract_pauli(const Sk2& x, const double (&a1)[4], const double (&a2)[4],
                                                   const double (&Kr)[4], const double (&Ki)[4], double& acc1,
                                                   double& acc2, double x0c = 0.0, double x3c = 0.0,
                                                   double x02c = 0.0) {
  static_assert(ORD >= 1 && ORD <= 3, "Pauli form for orders 1..3");
  // doubled Pauli components of K: 2k0 = K00 + K11, 2k1 = K01 + K10, 2k2 = i (K01 - K10), 2k3 = K00 - K11
  const double k0i = Ki[0] + Ki[3], k1i = Ki[1] + Ki[2], k2i = Kr[1] - Kr[2], k3i = Ki[0] - Ki[3];
  double m0, m1, m2, m3;  // 2 Im m
  if constexpr (ORD == 1) {
    m0 = k0i;
    m1 = k1i;
    m2 = k2i;
    m3 = k3i;
  } else {
    const double k0r = Kr[0] + Kr[3], k1r = Kr[1] + Kr[2], k2r = Ki[2] - Ki[1], k3r = Kr[0] - Kr[3];
    const double x0 = CX ? x0c : 0.5 * (x.d0 + x.d1), x1 = x.q, x2 = x.r, x3 = CX ? x3c : 0.5 * (x.d0 - x.d1);
    const double dr = fma(x3, k3r, fma(x2, k2r, x1 * k1r)), di = fma(x3, k3i, fma(x2, k2i, x1 * k1i));
    if constexpr (ORD == 2) {
      m0 = fma(x0, k0r, k0i + dr);
      m1 = fma(x0, k1r, fma(k0r, x1, k1i));
      m2 = fma(x0, k2r, fma(k0r, x2, k2i));
      m3 = fma(x0, k3r, fma(k0r, x3, k3i));
    } else {
      const double w = fma(x3, x3, fma(x2, x2, x1 * x1)), x02 = CX ? x02c : x0 * x0;
      const double al0 = fma(-0.5, x02 + w, 1.0), al1 = fma(-0.5, x02, fma(-1.0 / 6.0, w, 1.0));
      m0 = fma(al0, k0i, fma(x0, k0r - di, dr));
      const double c = fma(-x0, k0i, fma(-1.0 / 3.0, di, k0r));
      m1 = fma(al1, k1i, fma(x0, k1r, c * x1));
      m2 = fma(al1, k2i, fma(x0, k2r, c * x2));
      m3 = fma(al1, k3i, fma(x0, k3r, c * x3));
    }
  }
  // -2 a.Im m = -(a/2 ... ): aj holds 2 a, m holds 2 Im m, so the trace is -(aj.m) / 2
  acc1 = -0.5 * fma(a1[3], m3, fma(a1[2], m2, fma(a1[1], m1, a1[0] * m0)));
  acc2 = -0.5 * fma(a2[3], m3, fma(a2[2], m2, fma(a2[1], m1, a2[0] * m0)));
}
// doubled Pauli vector of an Sk2 generator block (sk2_contract_pauli's aj)
__device__ __forceinline__ void sk2_pauli2(const Sk2& e, double (&a)[4]) {
  a[0] = e.d0 + e.d1;
  a[1] = 2.0 * e.q;
  a[2] = 2.0 * e.r;
  a[3] = e.d0 - e.d1;
}

__device__ __forceinline__ double block_max(double v, double* scratch) {
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  double s = scratch[0];
  const int nw = (blockDim.x + 63) >> 6;
  for (int i = 1; i < nw; ++i) s = fmax(s, scratch[i]);
  __syncthreads();
  return s;
}

// wave-private LDS traffic between lanes of one wave: program order is LDS order within a wave; this keeps the
// compiler from moving accesses across the exchange
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Waves w, w + 4, w + 8 of a workgroup share a SIMD, and the oldest one wins the VALU issue arbitration: it would
// finish its segments far ahead and leave its partners alone on the SIMD at the end of each phase.  The partners
// take the priority in turns, one slice-step each.
__device__ __forceinline__ void seg_turn(int grp, int ngrp, int jj) {
  if ((grp + jj) % ngrp == 0) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}
// SIMD partners by progress (QOC_PROBE builds: g_seg_turnmode 1): each wave posts its step count in LDS and runs the
// next step at the higher issue priority when its partner (w ^ 4) is ahead (ties: the younger wave, which loses the
// arbitration otherwise).  The partner's count is read one step early, so the LDS latency hides behind the step.
struct SegProg {
  int* prog;
  int partner, other;
  bool on, young;
  __device__ __forceinline__ void step(int t) {
    if (!on) return;
    if (other > t || (other == t && young)) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    prog[threadIdx.x >> 6] = t;
    other = __builtin_amdgcn_readfirstlane(prog[partner]);
  }
};

// One workgroup per seed (blockIdx.x), W = blockDim / 64 waves, UPW segments of nblk lanes per wave (lanes past
// UPW nblk idle).  Built-in costs only (TRACE / ZCAL), no state penalty, no co-state source, unpacked states,
// skew-Hermitian generators (the host's blkseg_ok).
template <int NB, int ORD, int WMAX, int MODE = BLKSEG_FUSED>
__global__ __launch_bounds__(64 * WMAX) void k_blkseg_eval(const TChainArgs g, const BlkArgs bk, const BlksegParams sp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if constexpr (MODE == BLKSEG_BWD) {  // a stale u (the check queued before this launch): leave every output alone
    if (sp.stale && *sp.stale != 0) return;
  }
  constexpr int E = NB * NB;
  // the lane's generator blocks in registers (blocks of 2 rows at <= 8 waves), else from LDS where used; blocks of 2
  // rows keep Â for X = A_k and accumulate M in the contraction
  constexpr bool GREG = NB == 2 && WMAX <= 8;
  constexpr bool XA = NB == 2;
  constexpr int NV1 = NB == 2 ? 2 : 1;  // slices formed at once in phase 1
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, nblk = bk.nblk, S = sp.S, L = sp.L;
  const int tid = threadIdx.x, nthr = blockDim.x, w = tid >> 6, l = tid & 63, W = nthr >> 6;
  const int b = blockIdx.x;
  const size_t Nm = (size_t)N * m;
  BK_T(t0);
  double* const lds = reinterpret_cast<double*>(smem);
  double2* const gsh = reinterpret_cast<double2*>(lds);
  double* const rec = lds + blkseg_off_rec(NB, nblk);
  double2* const slot = reinterpret_cast<double2*>(lds + blkseg_off_slot(NB, nblk, Nt));
  double2* const g0s = reinterpret_cast<double2*>(lds + blkseg_off_g0(NB, nblk, Nt, S));
  double* const xN = lds + blkseg_off_xN(NB, nblk, Nt, S);
  cx<double>* const cf = reinterpret_cast<cx<double>*>(lds + blkseg_off_cf(N, m, NB, nblk, Nt, S));
  double* const red = lds + blkseg_off_red(N, m, NB, nblk, Nt, S);
  double* const wred = lds + blkseg_off_wred(N, m, NB, nblk, Nt, S);
  const int RB = sp.RB;
  double* const dJ = lds + blkseg_off_dJ(N, m, NB, nblk, Nt, S, W, RB);

  // ---- prologue: generator blocks, x_0, the seed's largest ρ_k ----
  {
    const cx<double>* At = (const cx<double>*)g.At;
    const size_t NN = (size_t)N * N;
    for (int q = tid; q < 3 * E * nblk; q += nthr) {  // block-major [nblk][3][E]: compile-time offsets per block
      const int beta = q / (3 * E), r = q - beta * 3 * E, j = r / E, e = r - j * E;
      const int ri = bk.brow[beta * NB + e / NB], rk = bk.brow[beta * NB + e % NB];
      cx<double> v = {0.0, 0.0};
      if (j <= nu && ri >= 0 && rk >= 0) v = At[(size_t)j * NN + ri + (size_t)N * rk];
      gsh[q] = make_double2(v.r, v.i);
    }
    if constexpr (MODE != BLKSEG_BWD) {
      const cx<double>* x0 = (const cx<double>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0);
      for (size_t o = tid; o < Nm; o += nthr) {
        xN[2 * o] = x0[o].r;
        xN[2 * o + 1] = x0[o].i;
      }
    }
  }
  // one pass over u: ρ_k, the copies of u (the stale check, the lazy rebuilds) and the records
  // [Re e^{μ_k}, Im e^{μ_k}, u_1k, u_2k] (e^{μ_k} does not depend on J; u is scaled by 2^-J below when J > 0)
  const double* ub = sp.u + (size_t)b * Nt * nu;
  double rmax = 0.0;
  // controls without shifts: e^{μ_k} = e^{μ_0} in every slice (the same value), one exp and sincos per thread
  const bool cmu = sp.mur[1] == 0.0 && sp.mur[2] == 0.0 && sp.mui[1] == 0.0 && sp.mui[2] == 0.0;
  double2 emu0 = make_double2(1.0, 0.0);
  if (cmu) {
    const double er = exp(sp.mur[0]);
    double sn, cs;
    sincos(sp.mui[0], &sn, &cs);
    emu0 = make_double2(er * cs, er * sn);
  }
  for (int k = tid; k < Nt; k += nthr) {
    const double u1 = nu > 0 ? ub[(size_t)k * nu] : 0.0, u2 = nu > 1 ? ub[(size_t)k * nu + 1] : 0.0;
    for (int j = 0; j < nu; ++j) {
      const double v = j ? u2 : u1;
      if (sp.u_copy) sp.u_copy[((size_t)b * Nt + k) * nu + j] = v;
      if (sp.u_copy2) sp.u_copy2[((size_t)b * Nt + k) * nu + j] = v;
    }
    rmax = fmax(rmax, fma(fabs(u2), sp.rad[2], fma(fabs(u1), sp.rad[1], sp.rad[0])));
    double2* r = reinterpret_cast<double2*>(rec + 4 * (size_t)k);
    if (cmu) {  // uniform
      r[0] = emu0;
    } else {
      const double mr = fma(u2, sp.mur[2], fma(u1, sp.mur[1], sp.mur[0]));
      const double mi = fma(u2, sp.mui[2], fma(u1, sp.mui[1], sp.mui[0]));
      const double er = exp(mr);
      double sn, cs;
      sincos(mi, &sn, &cs);
      r[0] = make_double2(er * cs, er * sn);
    }
    r[1] = make_double2(u1, u2);
  }
  rmax = block_max(rmax, red);  // (its barriers also publish the records)
  // J: the fewest halvings with ρ / 2^J <= θ_cap; P: the smallest degree whose tail bound
  // b^{P+1} / (P+1)! / (1 - b / (P+2)) is <= 2^-53 (b = ρmax / 2^J; every slice's ρ_k is <= ρmax)
  int J = 0;
  double s0 = 1.0;
  while (rmax * s0 > sp.theta_cap && J < 60) {
    s0 *= 0.5;
    ++J;
  }
  int P = 0;
  {
    const double bb = rmax * s0, tol = 1.1102230246251565e-16;
    constexpr BlkuCoef K = blku_coef();
    double term = bb;
#pragma unroll
    for (int q = 0; q < BLKU_TMAX; ++q) {
      if (!(term > tol * fma(-bb, K.inv[q + 2], 1.0))) break;
      P = q + 1;
      term *= bb * K.inv[q + 2];
    }
  }
  P = __builtin_amdgcn_readfirstlane(P);
  J = __builtin_amdgcn_readfirstlane(J);
  if (tid < 8) reinterpret_cast<int*>(red + 24)[tid] = 0;  // wave progress (SegProg)
  if (J) {  // the records hold 2^-J u (exact scaling)
    for (int k = tid; k < Nt; k += nthr) {
      rec[4 * (size_t)k + 2] *= s0;
      rec[4 * (size_t)k + 3] *= s0;
    }
  }
  __syncthreads();
  BK_T(t1);
  BK_ADD(0, t1 - t0);

  // ---- the lane's unit: segment s, block beta ----
  const int uw = l / nblk;
  const bool lact = uw < sp.UPW;
  const int beta = lact ? l - uw * nblk : 0;
  const int s = w * sp.UPW + uw;
  const bool sact = lact && s < S;
  const int kb = sact ? s * L : 0;
  const int ke = sact ? min(kb + L, Nt) : 0;
  int brw[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) brw[i] = bk.brow[beta * NB + i];
  double2 greg[GREG ? 3 : 1][GREG ? E : 1];
  if constexpr (GREG) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int e = 0; e < E; ++e) greg[j][e] = gsh[(beta * 3 + j) * E + e];
  }
  // the generator blocks (blocks of 3 rows: read from LDS where used, through an opaque copy of the block index made
  // inside each loop, so that the compiler does not hoist all 3 E of them into registers and spill)
  auto gen_at = [&](int bc) {
    return [&, bc](int j, int e) -> double2 {
      if constexpr (GREG) return greg[j][e];
      else return gsh[(bc * 3 + j) * E + e];
    };
  };
  auto opaque = [](int v) {
    asm volatile("" : "+v"(v));
    return v;
  };

  // SIMD partners (w, w + 4) alternate the issue priority (seg_turn); QOC_PROBE builds: g_seg_noturn turns it off
  const int grp = __builtin_amdgcn_readfirstlane(w >> 2), ngrp = (W + 3) >> 2;
  const bool turns = ngrp > 1 && SEG_TURNS && SEG_TURNMODE == 0;
  SegProg sprog;
  sprog.prog = reinterpret_cast<int*>(red + 24);
  sprog.partner = __builtin_amdgcn_readfirstlane(w ^ 4);
  sprog.on = ngrp > 1 && SEG_TURNS && SEG_TURNMODE == 1 && sprog.partner < W;
  sprog.young = grp == 1;
  sprog.other = 0;
  // ---- phase 1: the segment product P_s = U_{ke-1} .. U_{kb} ----
  double qr[E], qi[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    qr[e] = e % (NB + 1) == 0 ? 1.0 : 0.0;
    qi[e] = 0.0;
  }
  // every segment but the last has L slices; below Lf (the last one's length) no lane of a segment is past its end,
  // so those steps need no selects
  const int Lf = Nt - (S - 1) * L;
  // the fast path (blocks of 2 rows, no halvings): skew-Hermitian blocks in 4 reals, the closed-form exponential
  const bool fast = NB == 2 && J == 0;
  Sk2 gk[3];
  if constexpr (NB == 2) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double2 e4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) e4[e] = gsh[(beta * 3 + j) * E + e];
      gk[j] = sk2_of(e4);
    }
  }
  // the control generators' blocks without diagonal (cavity, zz: drives between levels): Â's diagonal is Ã_0's in
  // every slice, so e^{it} of the block's mean diagonal is computed once per lane (uniform over the workgroup)
  const bool zdl = NB != 2 || (gk[1].d0 == 0.0 && gk[1].d1 == 0.0 && gk[2].d0 == 0.0 && gk[2].d1 == 0.0);
  const bool zd = __syncthreads_and(zdl ? 1 : 0) != 0 && cmu;
  const double za0 = NB == 2 ? 0.5 * (gk[0].d0 - gk[0].d1) : 0.0;  // ZD: the blocks' constant half-difference
  auto p1_fast = [&](int jj, auto SEL_, auto K_, auto ZD_, double ct0, double st0) {
    constexpr bool SEL = decltype(SEL_)::value;
    constexpr int KS = decltype(K_)::value;
    constexpr bool ZD = decltype(ZD_)::value;
    if constexpr (NB == 2) {
      double ur[2][4], ui[2][4];
      bool act[2];
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int k = kb + jj + v;
        act[v] = !SEL || (sact && jj + v < L && k < ke);
        const double* r = rec + 4 * (size_t)(act[v] ? k : 0);
        Sk2 ah;
        sk2_form<KS, ZD>(gk, *reinterpret_cast<const double2*>(r), *reinterpret_cast<const double2*>(r + 2), ah, ur[v],
                         ui[v], ct0, st0, za0);
      }
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        double tr[4], ti[4];
        seg_mm<2, false, false>(ur[v], ui[v], qr, qi, tr, ti);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          qr[e] = !SEL || act[v] ? tr[e] : qr[e];
          qi[e] = !SEL || act[v] ? ti[e] : qi[e];
        }
      }
    }
  };
  // the fast path's series degree (uniform per seed: one loop instance per degree class)
  const int ksel = __builtin_amdgcn_readfirstlane(blkseg_series_k(rmax * s0));
  auto loop1z = [&](auto K_, auto ZD_) {
    constexpr int KS = decltype(K_)::value;
    double ct0 = 1.0, st0 = 0.0;
    if constexpr (NB == 2 && decltype(ZD_)::value) sk2_z<KS>(gk[0], rec, ct0, st0);
    for (int jj = 0; jj < L; jj += 2) {
      if (turns) seg_turn(grp, ngrp, jj >> 1);
      sprog.step(jj >> 1);
      if (jj + 1 < Lf) p1_fast(jj, std::false_type(), K_, ZD_, ct0, st0);
      else p1_fast(jj, std::true_type(), K_, ZD_, ct0, st0);
    }
  };
  auto loop1 = [&](auto K_) {
    if (zd) loop1z(K_, std::true_type());
    else loop1z(K_, std::false_type());
  };
  // G at the end of the lane's segment (phase 3's start): formed here, or read back (BLKSEG_BWD)
  double Gr[E], Gi[E];
  auto gseg_at = [&](int e) -> double2& { return sp.gseg[(((size_t)b * E + e) * S + s) * nblk + beta]; };
  if constexpr (MODE == BLKSEG_BWD) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 v = sact ? gseg_at(e) : make_double2(0.0, 0.0);
      Gr[e] = v.x;
      Gi[e] = v.y;
    }
    // the co-states' rebuild source (blku_costates): this u (copied in the prologue) and the forward's λ_N coefficients
    if (sp.coef2 && tid < 2 * m) sp.coef2[(size_t)b * 2 * m + tid] = g.coef[(size_t)b * 2 * m + tid];
  } else {
  if (fast) {
    if (ksel == 5) loop1(std::integral_constant<int, 5>());
    else if (ksel == 7) loop1(std::integral_constant<int, 7>());
    else loop1(std::integral_constant<int, BLKSEG_KMAX>());
  } else {
    for (int jj = 0; jj < L; jj += NV1) {
      if (turns) seg_turn(grp, ngrp, jj / NV1);
      sprog.step(jj / NV1);
      const double* rk[NV1];
      bool act[NV1];
#pragma unroll
      for (int v = 0; v < NV1; ++v) {
        const int k = kb + jj + v;
        act[v] = sact && jj + v < L && k < ke;
        rk[v] = rec + 4 * (size_t)(act[v] ? k : 0);
      }
      double ar[NV1][E], ai[NV1][E], ur[NV1][E], ui[NV1][E];
      seg_form<NB, NV1>(gen_at(GREG ? beta : opaque(beta)), rk, s0, P, J, ar, ai, ur, ui);
#pragma unroll
      for (int v = 0; v < NV1; ++v) {
        double tr[E], ti[E];
        seg_mm<NB, false, false>(ur[v], ui[v], qr, qi, tr, ti);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          qr[e] = act[v] ? tr[e] : qr[e];
          qi[e] = act[v] ? ti[e] : qi[e];
        }
      }
    }
  }

  if (turns || sprog.on) __builtin_amdgcn_s_setprio(0);
  BK_T(t2);
  BK_ADD(1, t2 - t1);
  SEGW_SET(w, t2 - t0);
  // ---- phase 2: prefix products Q_s = P_s .. P_0 ----
  // Two levels: a Hillis-Steele scan over the UPW segments of each wave through its own slot rows (one wave's LDS
  // accesses are ordered, so the rounds need wave syncs only), then every lane multiplies by the product of the
  // earlier waves' totals T_v (the local Q of their last segments), read after the one workgroup barrier.  Lanes of
  // segments past S hold the identity (phase 1 left their P = I), so the last wave's scan needs no masks.  14 of the
  // 15 barriers of the plain scan over 84 segments (zz) are gone.
  auto slot_at = [&](int ss, int e) -> double2& { return slot[((size_t)ss * E + e) * nblk + beta]; };
  const int UPW = sp.UPW, uw0 = lact ? uw : 0;
  if (sact)
#pragma unroll
    for (int e = 0; e < E; ++e) slot_at(s, e) = make_double2(qr[e], qi[e]);
  wave_lds_sync();
  for (int d = 1; d < UPW; d <<= 1) {
    const bool take = sact && uw0 >= d;
    double tr[E], ti[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 v = take ? slot_at(s - d, e) : make_double2(0.0, 0.0);
      tr[e] = v.x;
      ti[e] = v.y;
    }
    wave_lds_sync();
    if (take) {
      double cr[E], ci[E];
      seg_mm<NB, false, false>(qr, qi, tr, ti, cr, ci);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        qr[e] = cr[e];
        qi[e] = ci[e];
        slot_at(s, e) = make_double2(cr[e], ci[e]);
      }
    }
    wave_lds_sync();
  }
  lds_barrier();
  if (sact && w > 0) {  // E_w = T_{w-1} .. T_0, then Q_s = Q_s(local) E_w
    double er[E], ei[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 v = slot_at(UPW - 1, e);
      er[e] = v.x;
      ei[e] = v.y;
    }
    for (int v = 1; v < w; ++v) {
      double tr[E], ti[E], cr[E], ci[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double2 x = slot_at(v * UPW + UPW - 1, e);
        tr[e] = x.x;
        ti[e] = x.y;
      }
      seg_mm<NB, false, false>(tr, ti, er, ei, cr, ci);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        er[e] = cr[e];
        ei[e] = ci[e];
      }
    }
    double cr[E], ci[E];
    seg_mm<NB, false, false>(qr, qi, er, ei, cr, ci);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      qr[e] = cr[e];
      qi[e] = ci[e];
    }
  }
  // x_N = Q_{S-1} x_0 on each block (the last segment's lanes), in place in xN
  const bool last = sact && s == S - 1;
  if (last) {
    for (int c = 0; c < m; ++c) {
      double xr[NB], xi[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const size_t o = 2 * ((size_t)c * N + max(brw[i], 0));
        xr[i] = brw[i] >= 0 ? xN[o] : 0.0;
        xi[i] = brw[i] >= 0 ? xN[o + 1] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        double yr = 0.0, yi = 0.0;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          yr = fma(qr[i * NB + q], xr[q], fma(-qi[i * NB + q], xi[q], yr));
          yi = fma(qr[i * NB + q], xi[q], fma(qi[i * NB + q], xr[q], yi));
        }
        if (brw[i] >= 0) {
          const size_t o = 2 * ((size_t)c * N + brw[i]);
          xN[o] = yr;
          xN[o + 1] = yi;
        }
      }
    }
  }
  __syncthreads();
  // J and the λ_N coefficients (src/penalty_fcns.jl:15-42)
  chain_costs<double>(N, m, (const cx<double>*)g.Xt, [&](int q) { return cx<double>{xN[2 * q], xN[2 * q + 1]}; },
                      g.cost_kind, g.n_norm, 0.0, red, red + 16, cf, g.sc);
  __syncthreads();
  if (tid < 2 * m) {
    g.coef[(size_t)b * 2 * m + tid] = cf[tid];
    if (sp.coef2) sp.coef2[(size_t)b * 2 * m + tid] = cf[tid];
  }
  if (tid == 0) {
    // J is the one value other workgroups read in this launch (publish): stored write-through at agent scope (sc1),
    // so the hand-off needs no release fence (no L2 write-back of everything this XCD holds dirty)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(g.J + b),
                       (unsigned long long)__double_as_longlong(red[16]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sp.J2) sp.J2[b] = red[16];
  }
  // J is published after the cost: before the barrier that precedes G_0 when no waves share a SIMD within the
  // workgroup (early: all waves wait for the fences together), else after the last barrier before phase 3, so that
  // only wave 0 (one of the fast waves, seg_turn) waits for them.  The last workgroup to publish finds the best
  // (J, seed) of the launch (k_argmin_seed's order: NaN never wins, ties go to the lower seed).  The hand-off is the
  // write-through form of the guide's counter recipe (cdna_hip_programming.md, split-K combine / Guideline 16 R1):
  // J stored sc1, vmcnt(0), relaxed agent counter add; the last adder acquires and then reads every J.
  // This hand-off leans on gfx950's memory subsystem (the write-through sc1 store is complete at vmcnt(0), before the
  // counter add), not on a release/acquire pair, which would write back the whole L2 of the XCD; the build targets
  // gfx950 only (the check below keeps another target from compiling it silently).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "k_blkseg_eval's best-(J, seed) hand-off is written for gfx950"
#endif
  const bool early = W <= 4;
  auto publish = [&]() {
    if (w != 0 || !sp.done) return;
    unsigned int prev = 0;
    if (l == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sc1 J store has reached memory
      prev = __hip_atomic_fetch_add(sp.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    prev = __shfl(prev, 0);
    if (prev == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      double bv = __builtin_inf();
      long long bi = -1;
      for (int e = l; e < (int)gridDim.x; e += 64) {
        // agent-scope atomic loads (sc1 on gfx950): the other workgroups' J stores were write-through at agent scope
        const double v = __longlong_as_double((long long)__hip_atomic_load(
            reinterpret_cast<unsigned long long*>(g.J + e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (v < bv || (v == bv && e < bi)) {
          bv = v;
          bi = e;
        }
      }
      for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(bv, off);
        const long long oi = __shfl_xor(bi, off);
        if (ov < bv || (ov == bv && oi >= 0 && (bi < 0 || oi < bi))) {
          bv = ov;
          bi = oi;
        }
      }
      if (l == 0) {
        const double bs = bi >= 0 ? (double)(bi + sp.seed_offset) : -1.0;
        sp.best[0] = bv;
        sp.best[1] = bs;
        if (sp.best_res) {
          sp.best_res[0] = bv;
          sp.best_res[1] = bs;
        }
        if (sp.best_out) {
          sp.best_out[0] = bv;
          sp.best_out[1] = bs;
        }
        *sp.done = 0;  // ready for the next launch (the kernel boundary orders it)
      }
    }
  };
  if (early) publish();
  // G_N = Σ_c x_N λ_N^H on each block, G_0 = Q_{S-1}^H G_N Q_{S-1}
  if (last) {
    const cx<double>* Xt = (const cx<double>*)g.Xt;
    double gr[E], gi[E];
#pragma unroll
    for (int e = 0; e < E; ++e) gr[e] = gi[e] = 0.0;
    for (int c = 0; c < m; ++c) {
      double2 xv[NB], lv[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int r = brw[i];
        const size_t o = (size_t)c * N + max(r, 0);
        const cx<double> f = lam_coef(cf, g.sc, m, max(r, 0), c), t = Xt[o];
        xv[i] = r >= 0 ? make_double2(xN[2 * o], xN[2 * o + 1]) : make_double2(0.0, 0.0);
        lv[i] = r >= 0 ? make_double2(f.r * t.r - f.i * t.i, f.r * t.i + f.i * t.r) : make_double2(0.0, 0.0);
      }
      blku_kacc<NB>(gr, gi, xv, lv);
    }
    double tr[E], ti[E], cr[E], ci[E];
    seg_mm<NB, true, false>(qr, qi, gr, gi, tr, ti);
    seg_mm<NB, false, false>(tr, ti, qr, qi, cr, ci);
#pragma unroll
    for (int e = 0; e < E; ++e) g0s[e * nblk + beta] = make_double2(cr[e], ci[e]);
  }
  __syncthreads();
  // G at the segment's end: Q_s G_0 Q_s^H
  {
    double hr[E], hi[E], tr[E], ti[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 v = g0s[e * nblk + beta];
      hr[e] = v.x;
      hi[e] = v.y;
    }
    seg_mm<NB, false, false>(qr, qi, hr, hi, tr, ti);
    seg_mm<NB, false, true>(tr, ti, qr, qi, Gr, Gi);
  }

  if (!early) publish();
  BK_T(t2e);
  BK_ADD(2, t2e - t2);
  if constexpr (MODE == BLKSEG_FWD) {  // the forward half ends here: G to HBM for the backward launch
    if (sact)
#pragma unroll
      for (int e = 0; e < E; ++e) gseg_at(e) = make_double2(Gr[e], Gi[e]);
    if (sp.terms && tid == 0) atomicAdd(sp.terms + b % TERM_SLOTS, (unsigned long long)Nt * ((unsigned long long)P << J));
    return;
  }
  }  // MODE != BLKSEG_BWD
  BK_T(t3);
  // ---- phase 3: each segment backwards, the gradient of every slice ----
  const double mu1r = sp.mur[1], mu1i = sp.mui[1], mu2r = sp.mur[2], mu2i = sp.mui[2];
  double* const wr = wred + 128 * RB * w;
  // the slices' sums over their blocks: each step's partial sums go to slot (L - 1 - jj) % RB of a wave-private
  // area; every RB steps (and after the last) one lane per (step, segment of the wave, control) adds its nblk
  // entries in a fixed order
  const int nrl = sp.UPW * max(nu, 1);  // reducing lanes per step
  const int rq = l / nrl, rrem = l - rq * nrl, ro = rrem / max(nu, 1), rj = rrem - ro * max(nu, 1);
  int rslot = 0;  // (L - 1 - jj) % RB as a counter (jj runs down from L - 1 by one)
  auto reduce = [&](int jj, double acc1, double acc2) {
    const int r = rslot;
    rslot = r == RB - 1 ? 0 : r + 1;
    *reinterpret_cast<double2*>(wr + 128 * r + 2 * l) = make_double2(acc1, acc2);
    if (r == RB - 1 || jj == 0) {  // uniform
      wave_lds_sync();
      if (rq <= r) {  // slot rq holds step jj + r - rq
        const int ss = w * sp.UPW + ro, kk = ss * L + jj + r - rq;
        if (ss < S && kk < Nt) {
          const double* src = wr + 128 * rq + 2 * ro * nblk + rj;
          double sum = 0.0;
          for (int q = 0; q < nblk; ++q) sum += src[2 * q];
          dJ[(size_t)kk * nu + rj] = sum;
        }
      }
      wave_lds_sync();
    }
  };
  double pa1[4] = {0, 0, 0, 0}, pa2[4] = {0, 0, 0, 0};  // the generators' (A_j = Ã_j + i m_j I) doubled Pauli vectors
  // ZD: X's diagonal in every slice (Ã_0's plus i Im μ_0) and its Pauli components
  const double zxd0 = NB == 2 ? gk[0].d0 + sp.mui[0] : 0.0, zxd1 = NB == 2 ? gk[0].d1 + sp.mui[0] : 0.0;
  const double zx0 = 0.5 * (zxd0 + zxd1), zx3 = 0.5 * (zxd0 - zxd1), zx02 = zx0 * zx0;
  if constexpr (NB == 2) {
    sk2_pauli2(Sk2{gk[1].d0 + mu1i, gk[1].d1 + mu1i, gk[1].r, gk[1].q}, pa1);
    sk2_pauli2(Sk2{gk[2].d0 + mu2i, gk[2].d1 + mu2i, gk[2].r, gk[2].q}, pa2);
  }
  auto p3_fast = [&](int jj, auto SEL_, auto K_, auto ZD_, double ct0, double st0) {
    constexpr bool SEL = decltype(SEL_)::value;
    constexpr int KS = decltype(K_)::value;
    constexpr bool ZD = decltype(ZD_)::value;
    if constexpr (NB == 2) {
      const int k = kb + jj;
      const bool act = !SEL || (sact && k < ke);
      const double* r = rec + 4 * (size_t)(act ? k : 0);
      const double2 u = *reinterpret_cast<const double2*>(r + 2);
      Sk2 ah;
      double ur[4], ui[4];
      sk2_form<KS, ZD>(gk, *reinterpret_cast<const double2*>(r), u, ah, ur, ui, ct0, st0, za0);
      // K_k = U_k^H G_{k+1}, G_k = K_k U_k
      double Kr[4], Ki[4], tr[4], ti[4];
      seg_mm<2, true, false>(ur, ui, Gr, Gi, Kr, Ki);
      seg_mm<2, false, false>(Kr, Ki, ur, ui, tr, ti);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        Gr[e] = !SEL || act ? tr[e] : Gr[e];
        Gi[e] = !SEL || act ? ti[e] : Gi[e];
      }
      // X = A_k = Â + μ_k I (skew: μ_k = i (Im μ_0 + u_1 Im μ_1 + u_2 Im μ_2))
      // (ZD: μ_k = i Im μ_0, the same value)
      const double mki = ZD ? sp.mui[0] : fma(u.y, mu2i, fma(u.x, mu1i, sp.mui[0]));
      const Sk2 x{ah.d0 + mki, ah.d1 + mki, ah.r, ah.q};
      double acc1, acc2;
      if constexpr (ORD <= 3) {
        sk2_contract_pauli<ORD, ZD>(x, pa1, pa2, Kr, Ki, acc1, acc2, zx0, zx3, zx02);
      } else {
        const Sk2 e1{gk[1].d0 + mu1i, gk[1].d1 + mu1i, gk[1].r, gk[1].q};
        const Sk2 e2{gk[2].d0 + mu2i, gk[2].d1 + mu2i, gk[2].r, gk[2].q};
        sk2_contract<ORD>(x, e1, e2, Kr, Ki, acc1, acc2);
      }
      reduce(jj, !SEL || act ? acc1 : 0.0, !SEL || act ? acc2 : 0.0);
    }
  };
  auto loop3z = [&](auto K_, auto ZD_) {
    constexpr int KS = decltype(K_)::value;
    double ct0 = 1.0, st0 = 0.0;
    if constexpr (NB == 2 && decltype(ZD_)::value) sk2_z<KS>(gk[0], rec, ct0, st0);
    for (int jj = L - 1; jj >= 0; --jj) {
      if (turns) seg_turn(grp, ngrp, jj);
      sprog.step(L + (L - 1 - jj));
      if (jj < Lf) p3_fast(jj, std::false_type(), K_, ZD_, ct0, st0);
      else p3_fast(jj, std::true_type(), K_, ZD_, ct0, st0);
    }
  };
  auto loop3 = [&](auto K_) {
    if (zd) loop3z(K_, std::true_type());
    else loop3z(K_, std::false_type());
  };
  if (fast) {
    if (ksel == 5) loop3(std::integral_constant<int, 5>());
    else if (ksel == 7) loop3(std::integral_constant<int, 7>());
    else loop3(std::integral_constant<int, BLKSEG_KMAX>());
  } else {
    for (int jj = L - 1; jj >= 0; --jj) {
      if (turns) seg_turn(grp, ngrp, jj);
      sprog.step(L + (L - 1 - jj));
      const int k = kb + jj;
      const bool act = sact && k < ke;
      const double* rk[1] = {rec + 4 * (size_t)(act ? k : 0)};
      const auto gen = gen_at(GREG ? beta : opaque(beta));
      double ar[1][E], ai[1][E], ur[1][E], ui[1][E];
      seg_form<NB, 1>(gen, rk, s0, P, J, ar, ai, ur, ui);
      // K_k = U_k^H G_{k+1}, G_k = K_k U_k
      double Kr[E], Ki[E], tr[E], ti[E];
      seg_mm<NB, true, false>(ur[0], ui[0], Gr, Gi, Kr, Ki);
      seg_mm<NB, false, false>(Kr, Ki, ur[0], ui[0], tr, ti);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        Gr[e] = act ? tr[e] : Gr[e];
        Gi[e] = act ? ti[e] : Gi[e];
      }
      // X = A_k = 2^J Â + μ_k I, u_j = 2^J (2^-J u_j) exactly
      const double2 su = *reinterpret_cast<const double2*>(rk[0] + 2);
      const double u1 = ldexp(su.x, J), u2 = ldexp(su.y, J);
      const double mkr = fma(u2, sp.mur[2], fma(u1, sp.mur[1], sp.mur[0]));
      const double mki = fma(u2, sp.mui[2], fma(u1, sp.mui[1], sp.mui[0]));
      double xr[E], xi[E];
      if constexpr (XA) {  // from the formation's Â
#pragma unroll
        for (int e = 0; e < E; ++e) {
          xr[e] = (J ? ldexp(ar[0][e], J) : ar[0][e]) + (e % (NB + 1) == 0 ? mkr : 0.0);
          xi[e] = (J ? ldexp(ai[0][e], J) : ai[0][e]) + (e % (NB + 1) == 0 ? mki : 0.0);
        }
      } else {  // re-read (blocks of 3 rows: Â is not kept live across the two products)
        const auto gen2 = gen_at(opaque(beta));
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const double2 g0 = gen2(0, e), g1 = gen2(1, e), g2 = gen2(2, e);
          xr[e] = fma(u2, g2.x, fma(u1, g1.x, g0.x)) + (e % (NB + 1) == 0 ? mkr : 0.0);
          xi[e] = fma(u2, g2.y, fma(u1, g1.y, g0.y)) + (e % (NB + 1) == 0 ? mki : 0.0);
        }
      }
      double acc1, acc2;
      seg_contract<NB, ORD, XA>(gen, xr, xi, Kr, Ki, mu1r, mu1i, mu2r, mu2i, acc1, acc2);
      reduce(jj, act ? acc1 : 0.0, act ? acc2 : 0.0);
    }
  }
  if (turns || sprog.on) __builtin_amdgcn_s_setprio(0);
  BK_T(t4);
  BK_ADD(3, t4 - t3);
  SEGW_SET(16 + w, t4 - t0);
  __syncthreads();
  double* const og = sp.dJdu + (size_t)b * Nt * nu;
  for (int i = tid; i < Nt * nu; i += nthr) og[i] = dJ[i];
  if (MODE == BLKSEG_FUSED && sp.terms && tid == 0)
    atomicAdd(sp.terms + b % TERM_SLOTS, (unsigned long long)Nt * ((unsigned long long)P << J));
  BK_T(t5);
  BK_ADD(4, t5 - t4);
  BK_ADD(5, t5 - t0);
}

}  // namespace qoc
