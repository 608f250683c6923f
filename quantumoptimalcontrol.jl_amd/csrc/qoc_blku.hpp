// qoc_blku.hpp — block propagators: the slice exponential formed per invariant block, apart from the serial chain.
//
// The reference forms every U_k = exponential!(A_k) in a loop that is parallel over k
// (src/gradient_computations.jl:17-25), and only the products x_{k+1} = U_k x_k (:27-29) and
// λ_k = U_k^H λ_{k+1} (:52-58) are serial.  When the generators have small invariant blocks (qoc_blk.hpp: cavity 20
// blocks of 2 rows, zz 3 blocks of 3), U_k is block-diagonal with the same blocks, and one block of it is an NB x NB
// matrix that costs about as much to form as the exponential's action on the m state columns — but it does not
// depend on the state.  These kernels therefore keep the reference's split inside one workgroup per (seed,
// direction):
//   * formation waves form the block propagators U_k^β of the next chunk of C slices, parallel over (slice, block),
//     into LDS (double-buffered), and the step records of the chunk after that (ρ_k, P_k, e^{μ_k});
//   * chain waves advance the state with ONE NB x NB complex matvec per slice and block from LDS, and store x_{k+1}
//     (μ_k / λ_k backward) in the caller's layout.
// The serial depth per seed drops from Σ_k P_k dependent polynomial terms (cavity 9 000) to Nt matvecs.
//
// The block exponential: exp(A_k) = e^{μ_k} exp(Ã_k) with the shifted generators Ã_j = A_j - μ_j I of
// qoc_tchain.hpp (a multiple of the identity shifts every block alike), and exp(Ã_k) on a block is the degree-P
// Taylor polynomial of (Ã_k / 2^J) squared J times.  ρ_k = r_0 + Σ_j |u_jk| r_j bounds ||Ã_k||_2 (skew-Hermitian
// generators: r_j = half the width of H_j's spectral interval, Weyl) or ||Ã_k||_1 (other generators: r_j the
// shifted 1-norms); J is the fewest halvings with ρ_k / 2^J <= θ_cap, and P the smallest degree whose tail
// Σ_{t>P} (ρ_k / 2^J)^t / t! is <= 2^-53 — the backward-error level of the reference's Padé choice
// (ExpMethodHigham2005), so U_k agrees with the reference's to rounding.  For NB = 2 and 3 the polynomial is
// evaluated in the basis {I, Â, Â²} (Cayley-Hamilton: Â^NB is a combination of the lower powers with the
// characteristic polynomial's coefficients), so that a term costs NB complex multiply-adds instead of NB³;
// NB = 4 runs the plain matrix recurrence.  θ_cap = θ_17 ≈ 0.98 keeps the basis' rounding at the level of the
// direct recurrence (numpy: ≤ 8e-16 against mpmath up to norm 1).
#pragma once
#include "qoc_blk.hpp"

namespace qoc {

struct BlkuParams {
  double rad[3];                   // ρ_k = rad[0] + Σ_j |u_jk| rad[j]
  double mur[3], mui[3];           // shifts μ_j (e^{μ_k} = exp(μ_0 + Σ_j u_jk μ_j))
  double theta_cap;                // ρ_k / 2^J <= theta_cap (< 1)
  int C;                           // slices per chunk
  int CW;                          // chain waves (waves >= CW form propagators)
  unsigned long long* terms;       // Σ_k P_k 2^J_k per forward pass (nullptr: not counted)
};

constexpr int BLKU_REC = 8;   // doubles per step record: e^{μ} (2), scale, scale u_1, scale u_2, P, J, -
constexpr int BLKU_INVT = 32; // 1/t table

// LDS of one workgroup, in doubles: 1/t | generator blocks [3][NB^2][nblk] complex | step records [3][C][REC] |
// block propagators [2][C][NB^2][nblk] complex | x_N (2 N m) | reduction (16)
__host__ __device__ inline size_t blku_off_gb() { return BLKU_INVT; }
__host__ __device__ inline size_t blku_off_rec(int NB, int nblk) { return blku_off_gb() + (size_t)6 * NB * NB * nblk; }
__host__ __device__ inline size_t blku_off_U(int NB, int nblk, int C) {
  return blku_off_rec(NB, nblk) + (size_t)3 * BLKU_REC * C;
}
__host__ __device__ inline size_t blku_off_xN(int NB, int nblk, int C) {
  return blku_off_U(NB, nblk, C) + (size_t)4 * C * NB * NB * nblk;
}
__host__ __device__ inline size_t blku_lds(int N, int m, int NB, int nblk, int C) {
  return (blku_off_xN(NB, nblk, C) + 2 * (size_t)N * m + 16) * sizeof(double);
}

// Step record of slice k from u_k (one lane per slice).  cnt += P 2^J (executed Taylor terms).  P is the smallest
// degree whose tail bound b^{P+1} / (P+1)! / (1 - b / (P+2)) >= Σ_{t>P} b^t / t! is <= 2^-53 (b = ρ_k / 2^J < 1).
__device__ __forceinline__ void blku_record(const BlkuParams& bp, double u1, double u2, const double* __restrict__ invt,
                                            double* __restrict__ rec, unsigned long long& cnt) {
  const double rho = fma(fabs(u2), bp.rad[2], fma(fabs(u1), bp.rad[1], bp.rad[0]));
  const double mr = fma(u2, bp.mur[2], fma(u1, bp.mur[1], bp.mur[0]));
  const double mi = fma(u2, bp.mui[2], fma(u1, bp.mui[1], bp.mui[0]));
  int J = 0;
  double sc = 1.0;
  while (rho * sc > bp.theta_cap && J < 60) {
    sc *= 0.5;
    ++J;
  }
  const double b = rho * sc, tol = 1.1102230246251565e-16;
  double term = b;  // b^{P+1} / (P+1)!
  int P = 0;
  while (P < TCHAIN_PMAX && term > tol * fma(-b, invt[P + 2], 1.0)) {
    ++P;
    term *= b * invt[P + 1];
  }
  const double er = exp(mr);
  double sn, cs;
  sincos(mi, &sn, &cs);
  rec[0] = er * cs;
  rec[1] = er * sn;
  rec[2] = sc;
  rec[3] = sc * u1;
  rec[4] = sc * u2;
  rec[5] = (double)P;
  rec[6] = (double)J;
  rec[7] = 0.0;
  cnt += (unsigned long long)P << J;
}

// u <- u u (NB x NB complex, row-major e = i NB + k)
template <int NB>
__device__ __forceinline__ void blku_square(double (&ur)[NB * NB], double (&ui)[NB * NB]) {
  double vr[NB * NB], vi[NB * NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      double sr = 0.0, si = 0.0;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        sr = fma(ur[i * NB + q], ur[q * NB + k], sr);
        sr = fma(-ui[i * NB + q], ui[q * NB + k], sr);
        si = fma(ur[i * NB + q], ui[q * NB + k], si);
        si = fma(ui[i * NB + q], ur[q * NB + k], si);
      }
      vr[i * NB + k] = sr;
      vi[i * NB + k] = si;
    }
#pragma unroll
  for (int e = 0; e < NB * NB; ++e) {
    ur[e] = vr[e];
    ui[e] = vi[e];
  }
}

// Σ_{t<=P} Â^t / t! on the block (Â = ar + i ai, row-major).  invt[t] = 1/t.
template <int NB>
__device__ __forceinline__ void blku_taylor(const double (&ar)[NB * NB], const double (&ai)[NB * NB], int P,
                                            const double* __restrict__ invt, double (&ur)[NB * NB],
                                            double (&ui)[NB * NB]) {
  if constexpr (NB == 2) {
    // Â² = τ Â - δ I: z_t = α_t I + β_t Â with (α, β) <- (-δ β, α + τ β)
    const double tr = ar[0] + ar[3], ti = ai[0] + ai[3];
    const double nr = (ar[1] * ar[2] - ai[1] * ai[2]) - (ar[0] * ar[3] - ai[0] * ai[3]);  // -δ
    const double ni = (ar[1] * ai[2] + ai[1] * ar[2]) - (ar[0] * ai[3] + ai[0] * ar[3]);
    double zar = 1.0, zai = 0.0, zbr = 0.0, zbi = 0.0;
    double aar = 1.0, aai = 0.0, abr = 0.0, abi = 0.0, f = 1.0;
    for (int t = 1; t <= P; ++t) {
      const double yar = fma(nr, zbr, -ni * zbi), yai = fma(nr, zbi, ni * zbr);
      const double ybr = fma(tr, zbr, fma(-ti, zbi, zar)), ybi = fma(tr, zbi, fma(ti, zbr, zai));
      zar = yar;
      zai = yai;
      zbr = ybr;
      zbi = ybi;
      f *= invt[t];
      aar = fma(f, zar, aar);
      aai = fma(f, zai, aai);
      abr = fma(f, zbr, abr);
      abi = fma(f, zbi, abi);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ur[e] = abr * ar[e] - abi * ai[e] + (e == 0 || e == 3 ? aar : 0.0);
      ui[e] = abr * ai[e] + abi * ar[e] + (e == 0 || e == 3 ? aai : 0.0);
    }
  } else if constexpr (NB == 3) {
    // Â³ = c2 Â² + c1 Â + c0 I (c2 = tr, c1 = -(sum of the principal 2x2 minors), c0 = det):
    // z_t = α I + β Â + γ Â² with (α, β, γ) <- (γ c0, α + γ c1, β + γ c2)
    auto mr = [&](int a, int b) { return ar[a] * ar[b] - ai[a] * ai[b]; };
    auto mi = [&](int a, int b) { return ar[a] * ai[b] + ai[a] * ar[b]; };
    // principal minors m01 = a00 a11 - a01 a10, m02 = a00 a22 - a02 a20, m12 = a11 a22 - a12 a21
    const double m01r = mr(0, 4) - mr(1, 3), m01i = mi(0, 4) - mi(1, 3);
    const double m02r = mr(0, 8) - mr(2, 6), m02i = mi(0, 8) - mi(2, 6);
    const double m12r = mr(4, 8) - mr(5, 7), m12i = mi(4, 8) - mi(5, 7);
    const double c2r = ar[0] + ar[4] + ar[8], c2i = ai[0] + ai[4] + ai[8];
    const double c1r = -(m01r + m02r + m12r), c1i = -(m01i + m02i + m12i);
    // det = a00 m12 - a01 (a10 a22 - a12 a20) + a02 (a10 a21 - a11 a20)
    const double q1r = mr(3, 8) - mr(5, 6), q1i = mi(3, 8) - mi(5, 6);
    const double q2r = mr(3, 7) - mr(4, 6), q2i = mi(3, 7) - mi(4, 6);
    const double c0r = (ar[0] * m12r - ai[0] * m12i) - (ar[1] * q1r - ai[1] * q1i) + (ar[2] * q2r - ai[2] * q2i);
    const double c0i = (ar[0] * m12i + ai[0] * m12r) - (ar[1] * q1i + ai[1] * q1r) + (ar[2] * q2i + ai[2] * q2r);
    double zr[3] = {1.0, 0.0, 0.0}, zi[3] = {0.0, 0.0, 0.0};
    double sr[3] = {1.0, 0.0, 0.0}, si[3] = {0.0, 0.0, 0.0}, f = 1.0;
    for (int t = 1; t <= P; ++t) {
      const double gr = zr[2], gi = zi[2];
      const double n0r = fma(gr, c0r, -gi * c0i), n0i = fma(gr, c0i, gi * c0r);
      const double n1r = fma(gr, c1r, fma(-gi, c1i, zr[0])), n1i = fma(gr, c1i, fma(gi, c1r, zi[0]));
      const double n2r = fma(gr, c2r, fma(-gi, c2i, zr[1])), n2i = fma(gr, c2i, fma(gi, c2r, zi[1]));
      zr[0] = n0r;
      zi[0] = n0i;
      zr[1] = n1r;
      zi[1] = n1i;
      zr[2] = n2r;
      zi[2] = n2i;
      f *= invt[t];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        sr[q] = fma(f, zr[q], sr[q]);
        si[q] = fma(f, zi[q], si[q]);
      }
    }
    // U = α I + Â (β I + γ Â)
    double hr[9], hi[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      hr[e] = sr[2] * ar[e] - si[2] * ai[e] + (e % 4 == 0 ? sr[1] : 0.0);
      hi[e] = sr[2] * ai[e] + si[2] * ar[e] + (e % 4 == 0 ? si[1] : 0.0);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        double pr = i == k ? sr[0] : 0.0, pi = i == k ? si[0] : 0.0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          pr = fma(ar[i * 3 + q], hr[q * 3 + k], pr);
          pr = fma(-ai[i * 3 + q], hi[q * 3 + k], pr);
          pi = fma(ar[i * 3 + q], hi[q * 3 + k], pi);
          pi = fma(ai[i * 3 + q], hr[q * 3 + k], pi);
        }
        ur[i * 3 + k] = pr;
        ui[i * 3 + k] = pi;
      }
  } else {
    // plain matrix recurrence Y_t = Â Y_{t-1}
    double yr[NB * NB], yi[NB * NB];
#pragma unroll
    for (int e = 0; e < NB * NB; ++e) {
      yr[e] = ur[e] = (e % (NB + 1) == 0) ? 1.0 : 0.0;
      yi[e] = ui[e] = 0.0;
    }
    double f = 1.0;
    for (int t = 1; t <= P; ++t) {
      double vr[NB * NB], vi[NB * NB];
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double pr = 0.0, pi = 0.0;
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            pr = fma(ar[i * NB + q], yr[q * NB + k], pr);
            pr = fma(-ai[i * NB + q], yi[q * NB + k], pr);
            pi = fma(ar[i * NB + q], yi[q * NB + k], pi);
            pi = fma(ai[i * NB + q], yr[q * NB + k], pi);
          }
          vr[i * NB + k] = pr;
          vi[i * NB + k] = pi;
        }
      f *= invt[t];
#pragma unroll
      for (int e = 0; e < NB * NB; ++e) {
        yr[e] = vr[e];
        yi[e] = vi[e];
        ur[e] = fma(f, vr[e], ur[e]);
        ui[e] = fma(f, vi[e], ui[e]);
      }
    }
  }
}

// One block propagator U_k^β = e^{μ_k} (p(Ã_k / 2^J))^{2^J} from the step record rec; gb: generator blocks
// [3][NB^2][nblk] complex (entries of Ã_j at the block's rows), out: U at entry stride nblk.
template <int NB>
__device__ __forceinline__ void blku_form(const double2* __restrict__ gb, int nblk, int beta,
                                          const double* __restrict__ rec, const double* __restrict__ invt,
                                          double2* __restrict__ out) {
  constexpr int E = NB * NB;
  const double s0 = rec[2], s1 = rec[3], s2 = rec[4];
  const int P = (int)rec[5], J = (int)rec[6];
  double ar[E], ai[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const double2 g0 = gb[(0 * E + e) * nblk + beta], g1 = gb[(1 * E + e) * nblk + beta],
                  g2 = gb[(2 * E + e) * nblk + beta];
    ar[e] = fma(s2, g2.x, fma(s1, g1.x, s0 * g0.x));
    ai[e] = fma(s2, g2.y, fma(s1, g1.y, s0 * g0.y));
  }
  double ur[E], ui[E];
  blku_taylor<NB>(ar, ai, P, invt, ur, ui);
  for (int q = 0; q < J; ++q) blku_square<NB>(ur, ui);
  const double pr = rec[0], pi = rec[1];
#pragma unroll
  for (int e = 0; e < E; ++e) out[e * nblk] = make_double2(pr * ur[e] - pi * ui[e], pr * ui[e] + pi * ur[e]);
}

// y = U x (FWD) or U^H x on one block (U row-major complex from LDS, entries at stride nblk)
template <int NB, bool FWD>
__device__ __forceinline__ void blku_apply(const double2 (&U)[NB * NB], const double (&xr)[NB], const double (&xi)[NB],
                                           double (&yr)[NB], double (&yi)[NB]) {
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    double sr = 0.0, si = 0.0;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const double2 u = FWD ? U[i * NB + k] : U[k * NB + i];
      const double uim = FWD ? u.y : -u.y;  // conj for U^H
      sr = fma(u.x, xr[k], sr);
      sr = fma(-uim, xi[k], sr);
      si = fma(u.x, xi[k], si);
      si = fma(uim, xr[k], si);
    }
    yr[i] = sr;
    yi[i] = si;
  }
}

// One workgroup per (seed, direction): FWD x_0 -> x_Nt (+ costs), else λ_Nt -> λ_0 (μ mode: X_target -> μ_0).
template <int NB, bool FWD>
__device__ __forceinline__ void blku_body(const TChainArgs& g, const BlkArgs& bk, const BlkuParams& bp, const int b,
                                          const int mu_mode) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int E = NB * NB;
  double* lds = reinterpret_cast<double*>(smem);
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, nblk = bk.nblk, C = bp.C;
  const int tid = threadIdx.x, nthr = blockDim.x, w = tid >> 6;
  const size_t Nm = (size_t)N * m;
  double* invt = lds;
  double2* gb = reinterpret_cast<double2*>(lds + blku_off_gb());
  double* recs = lds + blku_off_rec(NB, nblk);
  double2* Ub = reinterpret_cast<double2*>(lds + blku_off_U(NB, nblk, C));
  double* xN = lds + blku_off_xN(NB, nblk, C);
  double* red = xN + 2 * Nm;
  // 1/t and the generator blocks Ã_j at the blocks' rows (zero outside the block and for j > nu)
  for (int e = tid; e < BLKU_INVT; e += nthr) invt[e] = e ? 1.0 / e : 0.0;
  {
    const cx<double>* At = (const cx<double>*)g.At;
    const size_t NN = (size_t)N * N;
    for (int q = tid; q < 3 * E * nblk; q += nthr) {
      const int j = q / (E * nblk), r = q - j * E * nblk, e = r / nblk, beta = r - e * nblk;
      const int ri = bk.brow[beta * NB + e / NB], rk = bk.brow[beta * NB + e % NB];
      cx<double> v = {0.0, 0.0};
      if (j <= nu && ri >= 0 && rk >= 0) v = At[(size_t)j * NN + ri + (size_t)N * rk];
      gb[q] = make_double2(v.r, v.i);
    }
  }
  const int nC = (Nt + C - 1) / C;
  const double* ub = g.u + (size_t)b * Nt * nu;
  const bool chain = w < bp.CW;
  const int fl = tid - 64 * bp.CW, FL = nthr - 64 * bp.CW;  // formation lanes
  unsigned long long cnt = 0;
  // slice of chunk position p (clamped into [0, Nt-1]: the tail of the last chunk repeats slice Nt-1, unused)
  auto slice_of = [&](int p) { return FWD ? min(p, Nt - 1) : max(Nt - 1 - p, 0); };
  // step records of chunk c: one lane per slice, u prefetched one chunk ahead
  double pu1 = 0.0, pu2 = 0.0;
  auto uload = [&](int c) {
    if (!chain && fl < C) {
      const int k = slice_of(c * C + fl);
      pu1 = nu > 0 ? ub[(size_t)k * nu] : 0.0;
      pu2 = nu > 1 ? ub[(size_t)k * nu + 1] : 0.0;
    }
  };
  auto records = [&](int c, double u1, double u2) {
    if (!chain && fl < C) {
      unsigned long long dummy = 0;
      const bool real = c * C + fl < Nt;
      blku_record(bp, u1, u2, invt, recs + ((size_t)(c % 3) * C + fl) * BLKU_REC, FWD && real ? cnt : dummy);
    }
  };
  auto form = [&](int c) {
    if (!chain) {
      const int units = C * nblk;
      const double* rc = recs + (size_t)(c % 3) * C * BLKU_REC;
      double2* Uc = Ub + (size_t)(c & 1) * C * E * nblk;
      for (int q = fl; q < units; q += FL) {
        const int jj = q / nblk, beta = q - jj * nblk;
        blku_form<NB>(gb, nblk, beta, rc + (size_t)jj * BLKU_REC, invt, Uc + (size_t)jj * E * nblk + beta);
      }
    }
  };
  // chain lanes: lane l < nblk m owns block l % nblk of column l / nblk
  BlkLane<NB> ln;
  ln.setup(bk, m, chain ? tid : 1 << 30);
  const int beta = chain && tid < nblk * m ? tid % nblk : 0;
  double* const sink = tchain_sink(g);
  double xr[NB], xi[NB];
  size_t off[NB];
  bool pm[NB];
  double pen = 0.0;
  double* Sb = reinterpret_cast<double*>((cx<double>*)(FWD ? g.X : g.L) + (size_t)b * (Nt + 1) * Nm);
  const double* Xb = reinterpret_cast<const double*>((const cx<double>*)g.X + (size_t)b * (Nt + 1) * Nm);
  const double* srcb =
      (!FWD && g.src && !mu_mode) ? reinterpret_cast<const double*>((const cx<double>*)g.src + (size_t)b * (Nt + 1) * Nm)
                                    : nullptr;
  const unsigned char* pmask = (FWD || !mu_mode) ? g.pmask : nullptr;
  const double tmu = 2.0 * g.mu;
  const bool add = !FWD && (pmask || srcb);
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const bool ok = ln.r[i] >= 0;
    const size_t o = (size_t)ln.c * N + max(ln.r[i], 0);
    off[i] = 2 * o;
    pm[i] = ok && pmask && pmask[o];
    cx<double> v = {0.0, 0.0};
    if (ok) {
      if (FWD) {
        v = ((const cx<double>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0))[o];
      } else if (mu_mode) {
        v = ((const cx<double>*)g.Xt)[o];
      } else {
        if (g.cost_kind == COST_EXTERNAL) {
          v = reinterpret_cast<const cx<double>*>(Sb)[(size_t)Nt * Nm + o];
        } else {
          const cx<double> cf = g.coef[(size_t)b * 2 * m + ln.c], t = ((const cx<double>*)g.Xt)[o];
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
    }
    xr[i] = v.r;
    xi[i] = v.i;
  }
  // the state of slice position k to HBM (padding elements go to the sink: no branch around the stores)
  auto store = [&](int k) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      double* p = ln.r[i] >= 0 ? Sb + (size_t)k * 2 * Nm + off[i] : sink;
      *reinterpret_cast<double2*>(p) = make_double2(xr[i], xi[i]);
      if (FWD) pen += pm[i] ? xr[i] * xr[i] + xi[i] * xi[i] : 0.0;
    }
  };
  if (chain) store(FWD ? 0 : Nt);
  // prologue: records of chunks 0 and 1, propagators of chunk 0
  uload(0);
  records(0, pu1, pu2);
  if (nC > 1) {
    uload(1);
    records(1, pu1, pu2);
  }
  if (nC > 2) uload(2);
  lds_barrier();
  form(0);
  lds_barrier();
  for (int c = 0; c < nC; ++c) {
    if (chain) {
      const double2* Uc = Ub + (size_t)(c & 1) * C * E * nblk + beta;
      double2 U0[E], U1[E];
#pragma unroll
      for (int e = 0; e < E; ++e) U0[e] = Uc[e * nblk];
      const int jn = min(C, Nt - c * C);
      for (int jj = 0; jj < jn; ++jj) {
        const int k = FWD ? c * C + jj : Nt - 1 - (c * C + jj);
        const int jp = min(jj + 1, C - 1);
#pragma unroll
        for (int e = 0; e < E; ++e) U1[e] = Uc[(size_t)jp * E * nblk + e * nblk];
        double ar_[NB], ai_[NB];
        if (add) {  // 2μ x_k on the mask + the caller's dL/dx(x_k), added after the slice
#pragma unroll
          for (int i = 0; i < NB; ++i) {
            const size_t o = (size_t)k * 2 * Nm + off[i];
            ar_[i] = pm[i] ? tmu * Xb[o] : 0.0;
            ai_[i] = pm[i] ? tmu * Xb[o + 1] : 0.0;
            if (srcb && ln.r[i] >= 0) {
              ar_[i] += srcb[o];
              ai_[i] += srcb[o + 1];
            }
          }
        }
        double yr[NB], yi[NB];
        blku_apply<NB, FWD>(U0, xr, xi, yr, yi);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const bool ok = ln.r[i] >= 0;
          xr[i] = ok ? yr[i] : 0.0;
          xi[i] = ok ? yi[i] : 0.0;
          if (add) {
            xr[i] += ar_[i];
            xi[i] += ai_[i];
          }
        }
        store(FWD ? k + 1 : k);
#pragma unroll
        for (int e = 0; e < E; ++e) U0[e] = U1[e];
      }
    } else {
      const double u1 = pu1, u2 = pu2;
      if (c + 3 < nC) uload(c + 3);
      if (c + 1 < nC) form(c + 1);
      if (c + 2 < nC) records(c + 2, u1, u2);
    }
    lds_barrier();
  }
  if (FWD) {
    if (chain) {
#pragma unroll
      for (int i = 0; i < NB; ++i)
        if (ln.r[i] >= 0) {
          xN[off[i]] = xr[i];
          xN[off[i] + 1] = xi[i];
        }
    }
    if (bp.terms) {
      for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
      if ((tid & 63) == 0 && cnt) atomicAdd(bp.terms, cnt);
    }
    __syncthreads();
    chain_costs<double>(N, m, (const cx<double>*)g.Xt, [&](int q) { return cx<double>{xN[2 * q], xN[2 * q + 1]}; },
                        g.cost_kind, g.n_norm, block_sum(pen, red) * g.mu, red, g.J + b, g.coef + (size_t)b * 2 * m,
                        g.sc);
  }
}

template <int NB>
__global__ __launch_bounds__(NB == 4 ? 256 : 512) void k_blku_fwd(const TChainArgs g, const BlkArgs bk, const BlkuParams bp) {
  blku_body<NB, true>(g, bk, bp, blockIdx.x, 0);
}
template <int NB>
__global__ __launch_bounds__(NB == 4 ? 256 : 512) void k_blku_bwd(const TChainArgs g, const BlkArgs bk, const BlkuParams bp) {
  blku_body<NB, false>(g, bk, bp, blockIdx.x, g.mu_mode);
}
// the forward chain and the μ recurrence (mu_mode) of every seed in one launch of 2B workgroups (the direction
// alternating every 8 workgroups, so that each XCD takes both)
template <int NB>
__global__ __launch_bounds__(NB == 4 ? 256 : 512) void k_blku_dual(const TChainArgs g, const BlkArgs bk, const BlkuParams bp) {
  const int i = blockIdx.x, B = gridDim.x >> 1;
  const bool by8 = (B & 7) == 0;
  const int dir = by8 ? (i >> 3) & 1 : i & 1;
  const int seed = by8 ? ((i >> 4) << 3) | (i & 7) : i >> 1;
  if (dir == 0) blku_body<NB, true>(g, bk, bp, seed, 0);
  else blku_body<NB, false>(g, bk, bp, seed, 1);
}

// The order-ORD gradient per block (expm_jacobian! + _compute_u_sensitivity, src/gradient_computations.jl:177-223)
// as one trace per generator: with X = A_k on the block and K = Σ_cols x_k λ_{k+1}^H (NB x NB),
//   Σ_cols λ^H dU_j x = tr(dU_j K) = tr(A_j M),  M = Σ_{a+b<ORD} X^b K X^a / (a+b+1)! = Σ_n L_n / (n+1)!,
//   L_0 = K, L_n = X L_{n-1} + K X^n
// (dU_j = Σ_{a+b<ORD} X^a A_j X^b / (a+b+1)!, the reference's Taylor terms).  Order 3: 4 products of NB x NB
// blocks instead of 4 m matvecs + 3 nu m contractions.  A unit is one (seed, slice); its nblk blocks are adjacent
// lanes of one wave, 64 / nblk units per wave-iteration, and they reduce through a wave-private LDS slot in a fixed
// order (no atomics, no workgroup barrier).  Persistent grid.  μ mode: L holds μ and λ = coef ⊙ μ per column.
__host__ __device__ inline size_t blku_grad_lds(int NB, int nblk) { return (4 * 128 + (size_t)6 * NB * NB * nblk) * 8; }

template <int NB, int ORD>
__global__ __launch_bounds__(256) void k_blku_grad(const TChainArgs g, const BlkArgs bk, long long units, int mu_mode,
                                                   double* __restrict__ dJdu) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int E = NB * NB;
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, nblk = bk.nblk;
  const size_t Nm = (size_t)N * m, NN = (size_t)N * N;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* rw = reinterpret_cast<double*>(smem) + 128 * w;
  // unshifted generator blocks A_0, A_1, A_2 [3][E][nblk] (row-major e), zero outside the block and for j > nu
  double2* gsh = reinterpret_cast<double2*>(reinterpret_cast<double*>(smem) + 4 * 128);
  {
    const cx<double>* A = (const cx<double>*)bk.A;
    for (int q = threadIdx.x; q < 3 * E * nblk; q += blockDim.x) {
      const int j = q / (E * nblk), r = q - j * E * nblk, e = r / nblk, bb = r - e * nblk;
      const int ri = bk.brow[bb * NB + e / NB], rk = bk.brow[bb * NB + e % NB];
      cx<double> v = {0.0, 0.0};
      if (j <= nu && ri >= 0 && rk >= 0) v = A[(size_t)j * NN + ri + (size_t)N * rk];
      gsh[q] = make_double2(v.r, v.i);
    }
  }
  __syncthreads();
  const int UPW = 64 / nblk, ul = l / nblk, beta = l - ul * nblk;
  const bool lact = ul < UPW;
  const double2* G0 = gsh + beta;
  const double2* G1 = gsh + E * nblk + beta;
  const double2* G2 = gsh + 2 * E * nblk + beta;
  int r[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) r[i] = lact ? bk.brow[beta * NB + i] : -1;
  constexpr double invf[6] = {1.0, 1.0, 0.5, 1.0 / 6, 1.0 / 24, 1.0 / 120};
  const long long wpb = blockDim.x >> 6;
  const long long nw = (long long)gridDim.x * wpb, wid = (long long)blockIdx.x * wpb + w;
  for (long long base = wid * UPW; base < units; base += nw * UPW) {
    const long long unit = base + ul;
    const bool act = lact && unit < units;
    const long long uu = act ? unit : 0;
    const int b = (int)(uu / Nt), k = (int)(uu - (long long)b * Nt);
    const double u1 = nu > 0 ? g.u[(size_t)uu * nu] : 0.0, u2 = nu > 1 ? g.u[(size_t)uu * nu + 1] : 0.0;
    const double* Xs = reinterpret_cast<const double*>((const cx<double>*)g.X + ((size_t)b * (Nt + 1) + k) * Nm);
    const double* Ls = reinterpret_cast<const double*>((const cx<double>*)g.L + ((size_t)b * (Nt + 1) + k + 1) * Nm);
    // K = Σ_c x_c λ_c^H : K[p][q] = Σ_c x_c[p] conj(λ_c[q])
    double kr[E], ki[E];
#pragma unroll
    for (int e = 0; e < E; ++e) kr[e] = ki[e] = 0.0;
    for (int c = 0; c < m; ++c) {
      double2 xv[NB], lv[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const size_t o = 2 * ((size_t)c * N + max(r[i], 0));
        xv[i] = r[i] >= 0 ? *reinterpret_cast<const double2*>(Xs + o) : make_double2(0.0, 0.0);
        lv[i] = r[i] >= 0 ? *reinterpret_cast<const double2*>(Ls + o) : make_double2(0.0, 0.0);
      }
      if (mu_mode) {  // λ = coef μ
        const cx<double> cf = g.coef[(size_t)b * 2 * m + c];
#pragma unroll
        for (int i = 0; i < NB; ++i) lv[i] = make_double2(cf.r * lv[i].x - cf.i * lv[i].y, cf.r * lv[i].y + cf.i * lv[i].x);
      }
#pragma unroll
      for (int p = 0; p < NB; ++p)
#pragma unroll
        for (int q = 0; q < NB; ++q) {  // x_p conj(λ_q)
          kr[p * NB + q] = fma(xv[p].x, lv[q].x, fma(xv[p].y, lv[q].y, kr[p * NB + q]));
          ki[p * NB + q] = fma(xv[p].y, lv[q].x, fma(-xv[p].x, lv[q].y, ki[p * NB + q]));
        }
    }
    // X = A_0 + u_1 A_1 + u_2 A_2
    double xr_[E], xi_[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 a0 = G0[e * nblk], a1 = G1[e * nblk], a2 = G2[e * nblk];
      xr_[e] = fma(u2, a2.x, fma(u1, a1.x, a0.x));
      xi_[e] = fma(u2, a2.y, fma(u1, a1.y, a0.y));
    }
    // M = K + Σ_{n>=1} L_n / (n+1)!,  L_n = X L_{n-1} + R_n,  R_n = R_{n-1} X  (L_0 = R_0 = K)
    double Mr[E], Mi[E], Lr[E], Li[E], Rr[E], Ri[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      Mr[e] = Lr[e] = Rr[e] = kr[e];
      Mi[e] = Li[e] = Ri[e] = ki[e];
    }
#pragma unroll
    for (int n = 1; n < ORD; ++n) {
      double tr[E], ti[E];
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int kk = 0; kk < NB; ++kk) {  // R_{n-1} X
          double sr = 0.0, si = 0.0;
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            sr = fma(Rr[i * NB + q], xr_[q * NB + kk], fma(-Ri[i * NB + q], xi_[q * NB + kk], sr));
            si = fma(Rr[i * NB + q], xi_[q * NB + kk], fma(Ri[i * NB + q], xr_[q * NB + kk], si));
          }
          tr[i * NB + kk] = sr;
          ti[i * NB + kk] = si;
        }
      double sr_[E], si_[E];
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int kk = 0; kk < NB; ++kk) {  // X L_{n-1} + R_n
          double sr = tr[i * NB + kk], si = ti[i * NB + kk];
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            sr = fma(xr_[i * NB + q], Lr[q * NB + kk], fma(-xi_[i * NB + q], Li[q * NB + kk], sr));
            si = fma(xr_[i * NB + q], Li[q * NB + kk], fma(xi_[i * NB + q], Lr[q * NB + kk], si));
          }
          sr_[i * NB + kk] = sr;
          si_[i * NB + kk] = si;
        }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        Rr[e] = tr[e];
        Ri[e] = ti[e];
        Lr[e] = sr_[e];
        Li[e] = si_[e];
        Mr[e] = fma(invf[n + 1], Lr[e], Mr[e]);
        Mi[e] = fma(invf[n + 1], Li[e], Mi[e]);
      }
    }
    // Re tr(A_j M) = Re Σ_{i,q} A_j[i][q] M[q][i]
    double acc1 = 0.0, acc2 = 0.0;
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const double2 a1 = G1[(i * NB + q) * nblk], a2 = G2[(i * NB + q) * nblk];
        acc1 = fma(a1.x, Mr[q * NB + i], fma(-a1.y, Mi[q * NB + i], acc1));
        acc2 = fma(a2.x, Mr[q * NB + i], fma(-a2.y, Mi[q * NB + i], acc2));
      }
    rw[2 * l] = act ? acc1 : 0.0;
    rw[2 * l + 1] = act ? acc2 : 0.0;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (l < UPW * nu) {
      const int u2_ = l / nu, j = l - u2_ * nu;
      double s = 0.0;
      for (int q = 0; q < nblk; ++q) s += rw[2 * (u2_ * nblk + q) + j];
      if (base + u2_ < units) dJdu[(size_t)(base + u2_) * nu + j] = s;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

}  // namespace qoc
