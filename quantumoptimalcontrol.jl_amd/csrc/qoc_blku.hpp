// qoc_blku.hpp — block propagators: the slice exponential formed per invariant block, apart from the serial chain.
//
// The reference forms every U_k = exponential!(A_k) in a loop that is parallel over k
// (src/gradient_computations.jl:17-25), and only the products x_{k+1} = U_k x_k (:27-29) and
// λ_k = U_k^H λ_{k+1} (:52-58) are serial.  When the generators have small invariant blocks (qoc_blk.hpp: cavity 20
// blocks of 2 rows, zz 3 blocks of 3), U_k is block-diagonal with the same blocks, and one block of it is an NB x NB
// matrix that costs about as much to form as the exponential's action on the m state columns — but it does not
// depend on the state.  So the work is split the reference's way:
//   * k_blku_rec: one thread per (seed, slice) forms the step record (ρ_k, the Taylor degree P and halvings J,
//     e^{μ_k}, the scaled controls), in parallel over every slice of the batch;
//   * k_blku_fwd / _bwd / _dual: one workgroup per (seed, direction).  Formation waves form the block propagators
//     U_k^β of the next chunk of C slices, parallel over (slice, block), into LDS (double-buffered); chain waves
//     advance the state with ONE NB x NB complex matvec per slice and block from LDS, and store x_{k+1} (μ_k / λ_k
//     backward) in the caller's layout.  The two roles run separate loops with one workgroup barrier per chunk, so
//     the chain's loop issues no global load (its stores are never waited on).
// The serial depth per seed drops from Σ_k P_k dependent polynomial terms (cavity 9 000) to Nt matvecs.
//
// The block exponential: exp(A_k) = e^{μ_k} exp(Ã_k) with the shifted generators Ã_j = A_j - μ_j I of
// qoc_tchain.hpp (a multiple of the identity shifts every block alike), and exp(Ã_k) on a block is the degree-P
// Taylor polynomial of (Ã_k / 2^J) squared J times.  ρ_k = r_0 + Σ_j |u_jk| r_j bounds ||Ã_k||_2 (skew-Hermitian
// generators: r_j = half the width of H_j's spectral interval, Weyl) or ||Ã_k||_1 (other generators: r_j the
// shifted 1-norms); J is the fewest halvings with ρ_k / 2^J <= θ_cap, and P the smallest degree whose tail
// Σ_{t>P} (ρ_k / 2^J)^t / t! is <= 2^-53 — the backward-error level of the reference's Padé choice
// (ExpMethodHigham2005), so U_k agrees with the reference's to rounding.  Slices are grouped in aligned blocks of 64
// that share the largest (J, P) among them (more terms than a slice needs only shrink its truncation error), so
// every propagator of a chunk runs the same term loop.  For NB = 2 and 3 the polynomial is evaluated by Horner's
// rule in the basis {I, Â, Â²} (Cayley-Hamilton: Â^NB is a combination of the lower powers with the characteristic
// polynomial's coefficients), a term costing NB complex multiply-adds instead of NB³; NB = 4 runs the plain matrix
// recurrence.  θ_cap = θ_17 ≈ 0.98 keeps the basis' rounding at the level of the direct recurrence (numpy: ≤ 8e-16
// against mpmath up to norm 1).
#pragma once
#include "qoc_blk.hpp"

namespace qoc {

struct BlkuParams {
  double rad[3];                   // ρ_k = rad[0] + Σ_j |u_jk| rad[j]
  double mur[3], mui[3];           // shifts μ_j (e^{μ_k} = exp(μ_0 + Σ_j u_jk μ_j))
  double theta_cap;                // ρ_k / 2^J <= theta_cap (< 1)
  int C;                           // slices per chunk (<= 64; the fused backward's need not divide 64)
  int CW;                          // chain waves (waves >= CW form propagators)
  int Ntp;                         // slices per seed in the record array: Nt rounded up to 64
  const double* rec;               // B x Ntp x BLKU_REC step records (k_blku_rec)
  unsigned long long* terms;       // Σ_k P_k 2^J_k per forward pass (k_blku_rec; nullptr: not counted)
  double* dJdu;                    // B x Nt x nu: the fused backward's gradient (k_blku_bwdg)
  double2* Uout;                   // k_blku_fwd (S = 1): also store each slice's block propagators, B x Nt x NB^2 x nblk
  const double2* Uin;              // k_blku_bwdg: read them instead of forming (the staging wave copies them to LDS)
  int ustg;                        // with Uin: 1 one staging wave copies the records, x_k and the propagators (small
                                   // chunks), else a second one the propagators
  int probe_mode;                  // QOC_PROBE builds only: 1 skip the formation, 2 the chain, 3 the chain's stores,
                                   // 4 the chain's LDS reads
};

// Diagnostic cycle stamps (tools/blku_probe.hip builds with -DQOC_PROBE; empty otherwise): per-role segment times of
// workgroup 7, summed over its lane-0 threads.
#ifdef QOC_PROBE
static __device__ unsigned long long g_bk[16];
#define BK_T(var) TC_T(var)
#define BK_ADD(slot, v)                                                          \
  do {                                                                           \
    if (blockIdx.x == 7 && (threadIdx.x & 63) == 0) atomicAdd(&g_bk[slot], (v)); \
  } while (0)
#else
#define BK_T(var) \
  do {            \
  } while (0)
#define BK_ADD(slot, v) \
  do {                  \
  } while (0)
#endif

// Propagators formed per lane at a time (independent recurrences interleaved): 2 for blocks of 2 rows; blocks of 3
// and 4 rows take one (two would exceed 256 VGPRs).  Probe builds may override it.
#ifndef QOC_BLKU_NU
#define QOC_BLKU_NU(NB) ((NB) == 2 ? 2 : 1)
#endif

constexpr int BLKU_REC = 8;   // doubles per step record: e^{μ} (2), scale, scale u_1, scale u_2, P, J, -
constexpr int BLKU_INVT = 32; // 1/t table
constexpr int BLKU_RECBLK = 64;  // slices sharing one (J, P)
// Taylor degrees of the block propagators: ρ_k / 2^J <= θ_cap ≈ 0.98 needs P <= 18; the term loops are unrolled to
// BLKU_TMAX with the coefficients 1/t! as compile-time constants
constexpr int BLKU_TMAX = 20;
constexpr int BLKU_XMAX = 20;  // fused backward: x_k elements staged per stager lane and chunk
struct BlkuCoef {
  double inv[BLKU_TMAX + 2];   // 1/t
  double fact[BLKU_TMAX + 1];  // 1/t!
};
constexpr BlkuCoef blku_coef() {
  BlkuCoef c{};
  c.inv[0] = 0.0;
  for (int t = 1; t <= BLKU_TMAX + 1; ++t) c.inv[t] = 1.0 / t;
  c.fact[0] = 1.0;
  for (int t = 1; t <= BLKU_TMAX; ++t) c.fact[t] = c.fact[t - 1] / t;
  return c;
}

// LDS of one workgroup, in doubles: 1/t | generator blocks [3][NB^2][nblk] complex | step records [4][C][REC] |
// block propagators [2][C][NB^2][nblk] complex | x_N (2 N m) | reduction (16)
__host__ __device__ inline size_t blku_off_gb() { return BLKU_INVT; }
__host__ __device__ inline size_t blku_off_rec(int NB, int nblk) { return blku_off_gb() + (size_t)6 * NB * NB * nblk; }
__host__ __device__ inline size_t blku_off_U(int NB, int nblk, int C) {
  return blku_off_rec(NB, nblk) + (size_t)4 * BLKU_REC * C;
}
__host__ __device__ inline size_t blku_off_xN(int NB, int nblk, int C) {
  return blku_off_U(NB, nblk, C) + (size_t)4 * C * NB * NB * nblk;
}
// the fused backward (k_blku_bwdg) adds: the co-state ring [2][C][N m] complex (λ_{k+1} of each slice of the last
// two chunks, written by the chain waves) | unshifted generator blocks [3][NB^2][nblk] complex
__host__ __device__ inline size_t blku_off_lam(int N, int m, int NB, int nblk, int C) {
  return blku_off_xN(NB, nblk, C) + 2 * (size_t)N * m + 16;
}
__host__ __device__ inline size_t blku_off_ga(int N, int m, int NB, int nblk, int C) {
  return blku_off_lam(N, m, NB, nblk, C) + (size_t)4 * C * N * m;
}
__host__ __device__ inline size_t blku_off_xs(int N, int m, int NB, int nblk, int C) {
  return blku_off_ga(N, m, NB, nblk, C) + (size_t)6 * NB * NB * nblk;
}
// | x_k of the last two chunks [2][CNp] complex (CNp = C N m rounded up to 64: whole wave-instructions of LDS-DMA)
__host__ __device__ inline int blku_cnp(int N, int m, int C) { return (C * N * m + 63) / 64 * 64; }
// bytes; gw: worker waves of the fused backward (0: the kernels without the gradient)
__host__ __device__ inline size_t blku_lds(int N, int m, int NB, int nblk, int C, int gw = 0) {
  if (gw > 0) return (blku_off_xs(N, m, NB, nblk, C) + (size_t)4 * blku_cnp(N, m, C)) * sizeof(double);
  return blku_off_lam(N, m, NB, nblk, C) * sizeof(double);
}

// DPP move of a double whose every source lane is valid (quad permutations), or whose invalid-source lanes are never
// read (row shifts in blku_scan): no old value to preserve, so no zero-initialised destination
template <int CTRL>
__device__ __forceinline__ double dpp_any(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// The launch bound of the chain kernels (k_blku_fwd / _bwd / _bwdg): 8 waves, 4 for blocks of 4 rows (their
// formation takes the whole register file).  The host sizes every launch within it (blku_shape).  (12 waves for
// blocks of 2 rows, <= 168 VGPRs, measured no faster: forward 0.17 vs 0.15 ms, fused backward 0.196 vs 0.198 ms.)
__host__ __device__ constexpr int blku_max_threads(int NB) { return NB == 4 ? 256 : 512; }

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// Step records, one thread per (seed, slice) over B x Ntp (a wave = 64 aligned slices of one seed, which share the
// largest J and P among them).  J: the fewest halvings with ρ_k / 2^J <= θ_cap; P: the smallest degree whose tail
// bound b^{P+1} / (P+1)! / (1 - b / (P+2)) >= Σ_{t>P} b^t / t! is <= 2^-53 (b = ρ_k / 2^J < 1).
// rec = [Re e^{μ_k}, Im e^{μ_k}, 2^-J, 2^-J u_1k, 2^-J u_2k, P, J, 0]; terms += Σ P 2^J (executed Taylor terms).
__global__ __launch_bounds__(256) void k_blku_rec(const BlkuParams bp, const double* __restrict__ u, int nu, int Nt,
                                                  long long total, double* __restrict__ rec) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long tt = t < total ? t : 0;
  const int b = (int)(tt / bp.Ntp), k = (int)(tt - (long long)b * bp.Ntp);
  const bool valid = t < total && k < Nt;
  const double* uk = u + ((size_t)b * Nt + min(k, Nt - 1)) * nu;
  const double u1 = valid && nu > 0 ? uk[0] : 0.0, u2 = valid && nu > 1 ? uk[1] : 0.0;
  const double rho = valid ? fma(fabs(u2), bp.rad[2], fma(fabs(u1), bp.rad[1], bp.rad[0])) : 0.0;
  int Jo = 0;
  double so = 1.0;
  while (rho * so > bp.theta_cap && Jo < 60) {
    so *= 0.5;
    ++Jo;
  }
  const int J = wave_max(Jo);
  const double sc = ldexp(1.0, -J);
  const double bb = rho * sc, tol = 1.1102230246251565e-16;
  constexpr BlkuCoef K = blku_coef();
  double term = bb;  // b^{P+1} / (P+1)!
  int Po = 0;
#pragma unroll
  for (int q = 0; q < BLKU_TMAX; ++q) {  // Po == q in iteration q: the 1/t are constants
    if (!(term > tol * fma(-bb, K.inv[q + 2], 1.0))) break;
    Po = q + 1;
    term *= bb * K.inv[q + 2];
  }
  const int P = wave_max(Po);
  unsigned long long cnt = valid ? (unsigned long long)P << J : 0ull;
  if (valid) {
    const double mr = fma(u2, bp.mur[2], fma(u1, bp.mur[1], bp.mur[0]));
    const double mi = fma(u2, bp.mui[2], fma(u1, bp.mui[1], bp.mui[0]));
    const double er = exp(mr);
    double sn, cs;
    sincos(mi, &sn, &cs);
    double2* r = reinterpret_cast<double2*>(rec + (size_t)tt * BLKU_REC);
    r[0] = make_double2(er * cs, er * sn);
    r[1] = make_double2(sc, sc * u1);
    r[2] = make_double2(sc * u2, (double)P);
    r[3] = make_double2((double)J, 0.0);
  }
  if (bp.terms) {  // one atomic per workgroup, into the workgroup's partial-sum word
    __shared__ unsigned long long part[4];
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long tot = part[0] + part[1] + part[2] + part[3];
      if (tot) atomicAdd(bp.terms + blockIdx.x % TERM_SLOTS, tot);
    }
  }
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

// e^{μ} Σ_{t<=P} Â^t / t! for NU independent blocks at once (Â_u = ar[u] + i ai[u], row-major; P uniform over the
// wave, e^{μ} = (pr[u], pi[u])): the NU recurrences interleave instruction by instruction, so that a lane keeps NU
// dependency chains in flight.  NB = 2, 3: Horner's rule h <- Â h + c_t I from t = P down to 0 with c_t = 1/t!
// (compile-time constants) in the Cayley-Hamilton basis, started from h = e^{μ} c_P so that the phase rides along;
// NB = 4: the matrix recurrence (invt[t] = 1/t).
template <int NB, int NU>
__device__ __forceinline__ void blku_taylor(const double (&ar)[NU][NB * NB], const double (&ai)[NU][NB * NB], int P,
                                            const double (&pr)[NU], const double (&pi)[NU],
                                            const double* __restrict__ invt, double (&ur)[NU][NB * NB],
                                            double (&ui)[NU][NB * NB]) {
  constexpr BlkuCoef K = blku_coef();
  if constexpr (NB == 2) {
    // Â² = τ Â - δ I: Â (α I + β Â) = (-δ β) I + (α + τ β) Â
    double tr[NU], ti[NU], nr[NU], ni[NU], hr[NU][2], hi[NU][2];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      tr[u] = ar[u][0] + ar[u][3];
      ti[u] = ai[u][0] + ai[u][3];
      nr[u] = (ar[u][1] * ar[u][2] - ai[u][1] * ai[u][2]) - (ar[u][0] * ar[u][3] - ai[u][0] * ai[u][3]);  // -δ
      ni[u] = (ar[u][1] * ai[u][2] + ai[u][1] * ar[u][2]) - (ar[u][0] * ai[u][3] + ai[u][0] * ar[u][3]);
      hr[u][0] = hi[u][0] = hr[u][1] = hi[u][1] = 0.0;
    }
#pragma unroll
    for (int t = BLKU_TMAX; t >= 0; --t) {
      if (t > P) continue;  // uniform
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const double cr = K.fact[t] * pr[u], ci = K.fact[t] * pi[u];  // e^{μ} c_t
        const double a_r = fma(nr[u], hr[u][1], fma(-ni[u], hi[u][1], cr));
        const double a_i = fma(nr[u], hi[u][1], fma(ni[u], hr[u][1], ci));
        const double b_r = fma(tr[u], hr[u][1], fma(-ti[u], hi[u][1], hr[u][0]));
        const double b_i = fma(tr[u], hi[u][1], fma(ti[u], hr[u][1], hi[u][0]));
        hr[u][0] = a_r;
        hi[u][0] = a_i;
        hr[u][1] = b_r;
        hi[u][1] = b_i;
      }
    }
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ur[u][e] = hr[u][1] * ar[u][e] - hi[u][1] * ai[u][e] + (e == 0 || e == 3 ? hr[u][0] : 0.0);
        ui[u][e] = hr[u][1] * ai[u][e] + hi[u][1] * ar[u][e] + (e == 0 || e == 3 ? hi[u][0] : 0.0);
      }
  } else if constexpr (NB == 3) {
    // Â³ = c2 Â² + c1 Â + c0 I (c2 = tr, c1 = -(sum of the principal 2x2 minors), c0 = det):
    // Â (α I + β Â + γ Â²) = γ c0 I + (α + γ c1) Â + (β + γ c2) Â²
    double c0r[NU], c0i[NU], c1r[NU], c1i[NU], c2r[NU], c2i[NU], hr[NU][3], hi[NU][3];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      auto mr = [&](int a, int b) { return ar[u][a] * ar[u][b] - ai[u][a] * ai[u][b]; };
      auto mi = [&](int a, int b) { return ar[u][a] * ai[u][b] + ai[u][a] * ar[u][b]; };
      // principal minors m01 = a00 a11 - a01 a10, m02 = a00 a22 - a02 a20, m12 = a11 a22 - a12 a21
      const double m01r = mr(0, 4) - mr(1, 3), m01i = mi(0, 4) - mi(1, 3);
      const double m02r = mr(0, 8) - mr(2, 6), m02i = mi(0, 8) - mi(2, 6);
      const double m12r = mr(4, 8) - mr(5, 7), m12i = mi(4, 8) - mi(5, 7);
      c2r[u] = ar[u][0] + ar[u][4] + ar[u][8];
      c2i[u] = ai[u][0] + ai[u][4] + ai[u][8];
      c1r[u] = -(m01r + m02r + m12r);
      c1i[u] = -(m01i + m02i + m12i);
      // det = a00 m12 - a01 (a10 a22 - a12 a20) + a02 (a10 a21 - a11 a20)
      const double q1r = mr(3, 8) - mr(5, 6), q1i = mi(3, 8) - mi(5, 6);
      const double q2r = mr(3, 7) - mr(4, 6), q2i = mi(3, 7) - mi(4, 6);
      c0r[u] = (ar[u][0] * m12r - ai[u][0] * m12i) - (ar[u][1] * q1r - ai[u][1] * q1i) + (ar[u][2] * q2r - ai[u][2] * q2i);
      c0i[u] = (ar[u][0] * m12i + ai[u][0] * m12r) - (ar[u][1] * q1i + ai[u][1] * q1r) + (ar[u][2] * q2i + ai[u][2] * q2r);
#pragma unroll
      for (int q = 0; q < 3; ++q) hr[u][q] = hi[u][q] = 0.0;
    }
#pragma unroll
    for (int t = BLKU_TMAX; t >= 0; --t) {
      if (t > P) continue;  // uniform
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const double gr = hr[u][2], gi = hi[u][2];
        const double cr = K.fact[t] * pr[u], ci = K.fact[t] * pi[u];
        const double n0r = fma(gr, c0r[u], fma(-gi, c0i[u], cr)), n0i = fma(gr, c0i[u], fma(gi, c0r[u], ci));
        const double n1r = fma(gr, c1r[u], fma(-gi, c1i[u], hr[u][0])), n1i = fma(gr, c1i[u], fma(gi, c1r[u], hi[u][0]));
        const double n2r = fma(gr, c2r[u], fma(-gi, c2i[u], hr[u][1])), n2i = fma(gr, c2i[u], fma(gi, c2r[u], hi[u][1]));
        hr[u][0] = n0r;
        hi[u][0] = n0i;
        hr[u][1] = n1r;
        hi[u][1] = n1i;
        hr[u][2] = n2r;
        hi[u][2] = n2i;
      }
    }
    // U = α I + Â (β I + γ Â)
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      double wr[9], wi[9];
#pragma unroll
      for (int e = 0; e < 9; ++e) {
        wr[e] = hr[u][2] * ar[u][e] - hi[u][2] * ai[u][e] + (e % 4 == 0 ? hr[u][1] : 0.0);
        wi[e] = hr[u][2] * ai[u][e] + hi[u][2] * ar[u][e] + (e % 4 == 0 ? hi[u][1] : 0.0);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          double sr = i == k ? hr[u][0] : 0.0, si = i == k ? hi[u][0] : 0.0;
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            sr = fma(ar[u][i * 3 + q], wr[q * 3 + k], sr);
            sr = fma(-ai[u][i * 3 + q], wi[q * 3 + k], sr);
            si = fma(ar[u][i * 3 + q], wi[q * 3 + k], si);
            si = fma(ai[u][i * 3 + q], wr[q * 3 + k], si);
          }
          ur[u][i * 3 + k] = sr;
          ui[u][i * 3 + k] = si;
        }
    }
  } else {
    // plain matrix recurrence Y_t = Â Y_{t-1}, NU = 1 (NB = 4: 64 CMAC per term); the phase multiplies at the end
    static_assert(NU == 1, "NB = 4 forms one block per lane at a time");
    double yr[NB * NB], yi[NB * NB], sr[NB * NB], si[NB * NB];
#pragma unroll
    for (int e = 0; e < NB * NB; ++e) {
      yr[e] = sr[e] = (e % (NB + 1) == 0) ? 1.0 : 0.0;
      yi[e] = si[e] = 0.0;
    }
    double f = 1.0;
    for (int t = 1; t <= P; ++t) {  // not unrolled; the 1/t read is off the critical path
      double vr[NB * NB], vi[NB * NB];
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          double qr = 0.0, qi = 0.0;
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            qr = fma(ar[0][i * NB + q], yr[q * NB + k], qr);
            qr = fma(-ai[0][i * NB + q], yi[q * NB + k], qr);
            qi = fma(ar[0][i * NB + q], yi[q * NB + k], qi);
            qi = fma(ai[0][i * NB + q], yr[q * NB + k], qi);
          }
          vr[i * NB + k] = qr;
          vi[i * NB + k] = qi;
        }
      f *= invt[t];
#pragma unroll
      for (int e = 0; e < NB * NB; ++e) {
        yr[e] = vr[e];
        yi[e] = vi[e];
        sr[e] = fma(f, vr[e], sr[e]);
        si[e] = fma(f, vi[e], si[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < NB * NB; ++e) {
      ur[0][e] = pr[0] * sr[e] - pi[0] * si[e];
      ui[0][e] = pr[0] * si[e] + pi[0] * sr[e];
    }
  }
}

// NU block propagators U_k^β = e^{μ_k} (p(Ã_k / 2^J))^{2^J} at once into registers (unit u: block beta[u] of the
// slice whose step record is rec[u]; the chunk's P and J are uniform); gb: generator blocks [3][NB^2][nblk] complex
// (entries of Ã_j at the block's rows).  With J > 0 the squarings run on the phase-free polynomial and e^{μ} multiplies
// after them.
template <int NB, int NU>
__device__ __forceinline__ void blku_form(const double2* __restrict__ gb, int nblk, const int (&beta)[NU],
                                          const double* const (&rec)[NU], const double* __restrict__ invt,
                                          double (&ur)[NU][NB * NB], double (&ui)[NU][NB * NB]) {
  constexpr int E = NB * NB;
  const int P = __builtin_amdgcn_readfirstlane((int)rec[0][5]), J = __builtin_amdgcn_readfirstlane((int)rec[0][6]);
  double ar[NU][E], ai[NU][E], pr[NU], pi[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const double s0 = rec[u][2], s1 = rec[u][3], s2 = rec[u][4];
    pr[u] = J ? 1.0 : rec[u][0];
    pi[u] = J ? 0.0 : rec[u][1];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 g0 = gb[(0 * E + e) * nblk + beta[u]], g1 = gb[(1 * E + e) * nblk + beta[u]],
                    g2 = gb[(2 * E + e) * nblk + beta[u]];
      ar[u][e] = fma(s2, g2.x, fma(s1, g1.x, s0 * g0.x));
      ai[u][e] = fma(s2, g2.y, fma(s1, g1.y, s0 * g0.y));
    }
  }
  blku_taylor<NB, NU>(ar, ai, P, pr, pi, invt, ur, ui);
  if (J) {
    for (int q = 0; q < J; ++q)
#pragma unroll
      for (int u = 0; u < NU; ++u) blku_square<NB>(ur[u], ui[u]);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const double qr = rec[u][0], qi = rec[u][1];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double vr = ur[u][e], vi = ui[u][e];
        ur[u][e] = qr * vr - qi * vi;
        ui[u][e] = qr * vi + qi * vr;
      }
    }
  }
}

// c = a b (NB x NB complex, row-major)
template <int NB>
__device__ __forceinline__ void blku_mm(const double (&ar)[NB * NB], const double (&ai)[NB * NB],
                                        const double (&br)[NB * NB], const double (&bi)[NB * NB], double (&cr)[NB * NB],
                                        double (&ci)[NB * NB]) {
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      double sr = 0.0, si = 0.0;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        sr = fma(ar[i * NB + q], br[q * NB + k], fma(-ai[i * NB + q], bi[q * NB + k], sr));
        si = fma(ar[i * NB + q], bi[q * NB + k], fma(ai[i * NB + q], br[q * NB + k], si));
      }
      cr[i * NB + k] = sr;
      ci[i * NB + k] = si;
    }
}

// Inclusive prefix products over the S lanes of a group (lane jl of the group holds T_jl on entry, Q_jl after):
// forward Q_j = T_j Q_{j-1}, backward Q_j = Q_{j-1} T_j.  Lane jl takes lane jl - d's product by a DPP row shift.
template <int NB, int S, bool FWD, int D = 1>
__device__ __forceinline__ void blku_scan(double (&ur)[NB * NB], double (&ui)[NB * NB], int jl) {
  if constexpr (D < S) {
    constexpr int E = NB * NB;
    double vr[E], vi[E], cr[E], ci[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      vr[e] = dpp_any<0x110 + D>(ur[e]);  // row_shr:D
      vi[e] = dpp_any<0x110 + D>(ui[e]);
    }
    if (FWD) blku_mm<NB>(ur, ui, vr, vi, cr, ci);
    else blku_mm<NB>(vr, vi, ur, ui, cr, ci);
    const bool take = jl >= D;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      ur[e] = take ? cr[e] : ur[e];
      ui[e] = take ? ci[e] : ui[e];
    }
    blku_scan<NB, S, FWD, 2 * D>(ur, ui, jl);
  }
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

// nblk rounded up to a power of two: a gradient unit's blocks sit on NBP adjacent lanes (lanes >= nblk of the group
// idle), so the sum over blocks is a butterfly within the group
__host__ __device__ inline int blku_nbp(int nblk) {
  int p = 1;
  while (p < nblk) p <<= 1;
  return p;
}
__device__ __forceinline__ double blku_group_sum(double v, int nbp) {
  if (nbp > 1) v += dpp_any<0xB1>(v);   // quad_perm [1,0,3,2]
  if (nbp > 2) v += dpp_any<0x4E>(v);   // quad_perm [2,3,0,1]
  if (nbp > 4) v += dpp_any<0x141>(v);  // row_half_mirror: the other quad of 8
  if (nbp > 8) v += dpp_any<0x140>(v);  // row_mirror: the other 8 of 16
  if (nbp > 16) v = swap_sum<16>(v);    // the other row of 32
  return v;
}

// Gradient of one (slice, block) unit (expm_jacobian! + _compute_u_sensitivity, src/gradient_computations.jl:177-223)
// as one trace per generator: with X = A_k on the block and K = Σ_cols x_k λ_{k+1}^H (NB x NB),
//   Σ_cols λ^H dU_j x = tr(dU_j K) = tr(A_j M),  M = Σ_{a+b<ORD} X^b K X^a / (a+b+1)! = Σ_n L_n / (n+1)!,
//   L_0 = R_0 = K, L_n = X L_{n-1} + R_n, R_n = R_{n-1} X
// (dU_j = Σ_{a+b<ORD} X^a A_j X^b / (a+b+1)!, the reference's Taylor terms).
// K += x λ^H from one column's rows (K[p][q] = Σ_c x_c[p] conj(λ_c[q]))
template <int NB>
__device__ __forceinline__ void blku_kacc(double (&kr)[NB * NB], double (&ki)[NB * NB], const double2 (&xv)[NB],
                                          const double2 (&lv)[NB]) {
#pragma unroll
  for (int p = 0; p < NB; ++p)
#pragma unroll
    for (int q = 0; q < NB; ++q) {  // x_p conj(λ_q)
      kr[p * NB + q] = fma(xv[p].x, lv[q].x, fma(xv[p].y, lv[q].y, kr[p * NB + q]));
      ki[p * NB + q] = fma(xv[p].y, lv[q].x, fma(-xv[p].x, lv[q].y, ki[p * NB + q]));
    }
}
// Re tr(A_j M) for j = 1, 2 from K and u_k; ga(j, e): entry e (row-major) of the unit's block of the unshifted
// generator A_j (from registers or LDS)
template <int NB, int ORD, typename GA>
__device__ __forceinline__ void blku_contract(GA&& ga, const double (&kr)[NB * NB], const double (&ki)[NB * NB],
                                              double u1, double u2, double& acc1, double& acc2) {
  constexpr int E = NB * NB;
  constexpr double invf[6] = {1.0, 1.0, 0.5, 1.0 / 6, 1.0 / 24, 1.0 / 120};
  // X = A_0 + u_1 A_1 + u_2 A_2
  double xr_[E], xi_[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const double2 a0 = ga(0, e), a1 = ga(1, e), a2 = ga(2, e);
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
  // in place: row i of R X needs only row i of R, column k of X L + R only column k of L (the same sums, in the
  // same order, as with separate product matrices: a third fewer live registers)
#pragma unroll
  for (int n = 1; n < ORD; ++n) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {  // R_n = R_{n-1} X
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
    for (int kk = 0; kk < NB; ++kk) {  // L_n = X L_{n-1} + R_n
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
        Mr[i * NB + kk] = fma(invf[n + 1], tr[i], Mr[i * NB + kk]);
        Mi[i * NB + kk] = fma(invf[n + 1], ti[i], Mi[i * NB + kk]);
      }
    }
  }
  // Re tr(A_j M) = Re Σ_{i,q} A_j[i][q] M[q][i]
  acc1 = acc2 = 0.0;
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const double2 a1 = ga(1, i * NB + q), a2 = ga(2, i * NB + q);
      acc1 = fma(a1.x, Mr[q * NB + i], fma(-a1.y, Mi[q * NB + i], acc1));
      acc2 = fma(a2.x, Mr[q * NB + i], fma(-a2.y, Mi[q * NB + i], acc2));
    }
}

// One workgroup per (seed, direction): FWD x_0 -> x_Nt (+ costs), else λ_Nt -> λ_0 (μ mode: X_target -> μ_0).
// ADD (backward, non-μ): 2μ x_k on the penalty mask and the caller's dL/dx(x_k) are added to λ_k after each slice
// (the only variant whose chain loop reads global memory).  Chunks lie on the absolute slice grid [aC, aC + C), the
// forward pass taking a = 0, 1, .., the backward pass a = nC - 1, .., 0 (its first chunk may be partial), so that a
// chunk never straddles two of k_blku_rec's 64-slice (J, P) groups.
// GORD > 0 (backward, non-μ, no additions): the fused gradient of order GORD.  The chain writes λ_{k+1} of every slice
// into an LDS ring instead of HBM, and the worker waves, besides forming the next chunk's propagators, contract the
// previous chunk's slices with x_k from HBM (blku_contract): the co-states never leave the workgroup.
template <int NB, int S, bool FWD, bool ADD, int GORD = 0>
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
  static_assert(GORD == 0 || (!FWD && !ADD), "the fused gradient runs on the plain backward chain");
  double2* const lam = reinterpret_cast<double2*>(lds + blku_off_lam(N, m, NB, nblk, C));
  double2* const ga = reinterpret_cast<double2*>(lds + blku_off_ga(N, m, NB, nblk, C));
  if constexpr (GORD > 0) {  // the unshifted generator blocks A_j for the gradient
    const cx<double>* A = (const cx<double>*)bk.A;
    const size_t NN = (size_t)N * N;
    for (int q = tid; q < 3 * E * nblk; q += nthr) {
      const int j = q / (E * nblk), r = q - j * E * nblk, e = r / nblk, beta = r - e * nblk;
      const int ri = bk.brow[beta * NB + e / NB], rk = bk.brow[beta * NB + e % NB];
      cx<double> v = {0.0, 0.0};
      if (j <= nu && ri >= 0 && rk >= 0) v = A[(size_t)j * NN + ri + (size_t)N * rk];
      ga[q] = make_double2(v.r, v.i);
    }
  }
  const int nC = (Nt + C - 1) / C;
  auto chunk_of = [&](int c) { return FWD ? c : nC - 1 - c; };  // absolute chunk of sequence position c
  const bool chain = w < bp.CW;
  // the fused backward has one staging wave (wave CW) between the chain and the worker waves: it moves the step
  // records and x_k global -> registers -> LDS one iteration apart, so that neither the chain (whose first matvec of a
  // chunk would wait on the loads) nor the workers (whose registers go to the formation and the contraction) wait
  // With stored propagators (bp.Uin) a second staging wave copies them (each stager holds one chunk's worth of
  // registers: two in one wave would spill).
  const int STG = GORD > 0 ? (bp.Uin && bp.ustg != 1 ? 2 : 1) : 0;
  const bool stager = GORD > 0 && w >= bp.CW && w < bp.CW + STG;
  const int stg_i = w - bp.CW;  // 0: step records and x_k, 1: propagators
  const int fl = tid - 64 * (bp.CW + STG), FL = nthr - 64 * (bp.CW + STG);  // formation lanes
  // staging lanes (global -> registers, one iteration later registers -> LDS): a stager, else the worker lanes
  const int sl = GORD > 0 ? (tid & 63) : fl, SLN = GORD > 0 ? 64 : FL;
  // step records of sequence chunk c: C x REC doubles from k_blku_rec (the tail of a partial chunk: clamped reads,
  // never used), through registers into the LDS ring slot c & 3
  constexpr int RMAX = 8;  // loads per lane: 64 x REC doubles / 64 lanes at most
  double rr[RMAX];
  const double* recb = bp.rec + (size_t)b * bp.Ntp * BLKU_REC;
  auto rec_load = [&](int c) {
    const int a = chunk_of(c), n = min(C, Nt - a * C) * BLKU_REC;  // (a C not dividing 64 can pass Ntp)
    const size_t base = (size_t)a * C * BLKU_REC;
#pragma unroll
    for (int i = 0; i < RMAX; ++i)  // unconditional (clamped) loads: the waits before rec_store count them exactly
      rr[i] = recb[base + min(sl + i * SLN, n - 1)];
  };
  auto rec_store = [&](int c) {
    double* dst = recs + (size_t)(c & 3) * C * BLKU_REC;
#pragma unroll
    for (int i = 0; i < RMAX; ++i) {
      const int e = sl + i * SLN;
      if (e < C * BLKU_REC) dst[e] = rr[i];
    }
  };
  // sequence position s_ (0 .. jn-1, the chain's order) -> chunk position: forward s_, backward jn - 1 - s_
  auto posn = [&](int s_, int jn) { return FWD ? s_ : jn - 1 - s_; };
  // the chunk's propagators, folded into prefix products over groups of S consecutive sequence positions:
  // position lo + j of a group holds Q_j = T_{lo+j} .. T_lo (T = U forward; backward Q_j^H = U_{lo+j}^H .. U_lo^H, so
  // Q_j = U_lo .. U_{lo+j}), and the chain applies Q_j to the group's incoming state for every j: S independent
  // matvecs per group instead of S dependent ones.  A unit is one (position, block); the S units of a group sit on S
  // adjacent lanes (S | 16: one DPP row) and scan by row shifts (Hillis-Steele, log2 S block products).  NU units per
  // lane at a time, at stride FL (independent recurrences interleaved).
  constexpr int NU = QOC_BLKU_NU(NB);
  auto form_n = [&](auto NU_, int c, int units, int jn) {
    constexpr int NV = decltype(NU_)::value;
    const double* rc = recs + (size_t)(c & 3) * C * BLKU_REC;
    double2* Uc = Ub + (size_t)(c & 1) * C * E * nblk;
    for (int q = fl; q < units; q += NV * FL) {
      int be[NV], pp[NV], jl[NV];
      const double* rp[NV];
      bool st[NV];
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const int qu = q + u * FL;
        const int qq = qu < units ? qu : q, t = qq / S, gq = t / nblk;
        jl[u] = qq - t * S;
        be[u] = t - gq * nblk;
        const int s_ = gq * S + jl[u];
        st[u] = qu < units && s_ < jn;
        pp[u] = posn(min(s_, jn - 1), jn);
        rp[u] = rc + (size_t)pp[u] * BLKU_REC;
      }
      double ur[NV][E], ui[NV][E];
      blku_form<NB, NV>(gb, nblk, be, rp, invt, ur, ui);
      if (FWD && bp.Uout) {  // the propagators themselves (before any prefix scan) to HBM at the absolute slice
#pragma unroll
        for (int u = 0; u < NV; ++u)
          if (st[u]) {
            double2* og = bp.Uout + ((size_t)b * Nt + (size_t)chunk_of(c) * C + pp[u]) * E * nblk + be[u];
#pragma unroll
            for (int e = 0; e < E; ++e) og[e * nblk] = make_double2(ur[u][e], ui[u][e]);
          }
      }
      if constexpr (S > 1) {
#pragma unroll
        for (int u = 0; u < NV; ++u) blku_scan<NB, S, FWD>(ur[u], ui[u], jl[u]);
      }
#pragma unroll
      for (int u = 0; u < NV; ++u)
        if (st[u]) {
          double2* o = Uc + (size_t)pp[u] * E * nblk + be[u];
#pragma unroll
          for (int e = 0; e < E; ++e) o[e * nblk] = make_double2(ur[u][e], ui[u][e]);
        }
    }
  };
  // NU units per lane only when the chunk has more units than formation lanes (else the second would be idle work)
  auto form = [&](int c) {
    const int a = chunk_of(c), jn = min(C, Nt - a * C), units = (jn + S - 1) / S * S * nblk;
    if (NU > 1 && units > FL) form_n(std::integral_constant<int, NU>(), c, units, jn);
    else form_n(std::integral_constant<int, 1>(), c, units, jn);
  };
  // x_k of sequence chunk cq (GORD > 0) through registers into the x ring slot cq & 1: loaded one iteration before
  // it is stored (like the step records), so the wait falls on loads long landed (LDS-DMA instead would make every
  // LDS access of the formation wait for the copy in flight); the chunk's jn N m complex are contiguous in HBM
  constexpr int XMAX = GORD > 0 ? BLKU_XMAX : 1;  // loads per stager lane (the host keeps C N m <= 64 BLKU_XMAX)
  const int CNp = blku_cnp(N, m, C);
  double2* const xring = reinterpret_cast<double2*>(lds + blku_off_xs(N, m, NB, nblk, C));
  typedef double dv2 __attribute__((ext_vector_type(2)));
  dv2 xreg[XMAX];  // (a clang vector type: an array of HIP's double2 struct is not promoted to registers)
  auto xs_load = [&](int cq) {
    if constexpr (GORD > 0) {
      const int a = chunk_of(cq), n = min(C, Nt - a * C) * (int)Nm;
      const double2* src = reinterpret_cast<const double2*>((const cx<double>*)g.X + ((size_t)b * (Nt + 1) + (size_t)a * C) * Nm);
#pragma unroll
      for (int i = 0; i < XMAX; ++i)  // clamped, unconditional
        xreg[i] = *reinterpret_cast<const dv2*>(src + min(sl + i * SLN, n - 1));
    }
  };
  auto xs_store = [&](int cq) {
    if constexpr (GORD > 0) {
      double2* dst = xring + (size_t)(cq & 1) * CNp;
#pragma unroll
      for (int i = 0; i < XMAX; ++i) {
        const int e = sl + i * SLN;
        if (e < C * (int)Nm) *reinterpret_cast<dv2*>(dst + e) = xreg[i];
      }
    }
  };
  // the stored propagators of sequence chunk cq (GORD > 0 with bp.Uin): global -> stager registers -> the U slot
  // cq & 1, one iteration apart (the chunk's jn NB^2 nblk complex are contiguous in HBM and in LDS)
  constexpr int UMAX = GORD > 0 ? BLKU_XMAX : 1;
  dv2 ureg[UMAX];
  const bool uin = GORD > 0 && bp.Uin != nullptr;
  auto us_load = [&](int cq) {
    if constexpr (GORD > 0) {
      const int a = chunk_of(cq), n = min(C, Nt - a * C) * E * nblk;
      const double2* src = bp.Uin + ((size_t)b * Nt + (size_t)a * C) * E * nblk;
#pragma unroll
      for (int i = 0; i < UMAX; ++i)  // clamped, unconditional
        ureg[i] = *reinterpret_cast<const dv2*>(src + min(sl + i * SLN, n - 1));
    }
  };
  auto us_store = [&](int cq) {
    if constexpr (GORD > 0) {
      double2* dst = Ub + (size_t)(cq & 1) * C * E * nblk;
#pragma unroll
      for (int i = 0; i < UMAX; ++i) {
        const int e = sl + i * SLN;
        if (e < C * E * nblk) *reinterpret_cast<dv2*>(dst + e) = ureg[i];
      }
    }
  };
  // the fused gradient of sequence chunk cq (GORD > 0): UPW = 64 / nblk slices per wave-iteration, a lane per (slice,
  // block), the nblk blocks of a slice on adjacent lanes (lanes past UPW nblk idle); wave-iteration it on worker wave
  // it % NWK (the host picks C so that the iterations come out even over the workers).  K = Σ_c x_k λ_{k+1}^H from the
  // x ring and the λ ring (slots cq & 1), then Re tr(A_j M), summed over the slice's blocks by a segmented lane scan.
  // (Packing the chunk's units densely over all 64 lanes splits slices between wave-iterations: their halves need
  // atomic adds, whose round trips cost more than the idle lanes.)
  const int wk = w - bp.CW - STG, NWK = nthr / 64 - bp.CW - STG;
  const int UPW = 64 / nblk, gl = tid & 63, ul = gl / nblk, be = gl - ul * nblk;
  // the lane's block rows, read once (a global load inside the contraction would expose its latency every chunk)
  int grow[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) grow[i] = GORD > 0 && wk >= 0 && ul < UPW ? bk.brow[be * NB + i] : -1;
  auto grad = [&](int cq) {
    if constexpr (GORD > 0) {
      const int a = chunk_of(cq), jn = min(C, Nt - a * C), nit = (jn + UPW - 1) / UPW;
      const double2* lr = lam + (size_t)(cq & 1) * C * Nm;
      const double2* xq = xring + (size_t)(cq & 1) * CNp;
      const double* rq = recs + (size_t)(cq & 3) * C * BLKU_REC;
      double2 areg[3][NB == 2 ? E : 1];
      if constexpr (NB == 2)  // the lane's block of A_0..A_2 in registers
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int e = 0; e < E; ++e) areg[j][e] = ga[(j * E + e) * nblk + be];
      for (int it = wk; it < nit; it += NWK) {
        const int jj = it * UPW + ul;
        const bool act = ul < UPW && jj < jn;
        int r[NB];  // (opaque copies: nothing derived from them is hoisted out of the loop to sit in registers)
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          r[i] = grow[i];
          if constexpr (NB > 2) asm volatile("" : "+v"(r[i]));
        }
        const int jc = act ? jj : 0;
        // u_k from the step record (2^-J u_j scaled back by 2^J: exact)
        const double* rk = rq + (size_t)jc * BLKU_REC;
        const int Jk = (int)rk[6];
        const double u1 = ldexp(rk[3], Jk), u2 = ldexp(rk[4], Jk);
        double kr[E], ki[E];
#pragma unroll
        for (int e = 0; e < E; ++e) kr[e] = ki[e] = 0.0;
        // K = Σ_c x_c λ_c^H from x_k in the x ring and λ_{k+1} in the λ ring
        constexpr int CB = NB == 2 ? 2 : 1;  // columns whose loads are in flight at once (a missing one: zeros)
        const double2* xs = xq + (size_t)jc * Nm;
        const double2* ls = lr + (size_t)jc * Nm;
        for (int c0 = 0; c0 < m; c0 += CB) {
          double2 xv[CB][NB], lv[CB][NB];
#pragma unroll
          for (int cc = 0; cc < CB; ++cc)
#pragma unroll
            for (int i = 0; i < NB; ++i) {
              const bool v = r[i] >= 0 && c0 + cc < m;
              const int o = v ? (c0 + cc) * N + r[i] : 0;
              xv[cc][i] = v ? xs[o] : make_double2(0.0, 0.0);
              lv[cc][i] = v ? ls[o] : make_double2(0.0, 0.0);
            }
#pragma unroll
          for (int cc = 0; cc < CB; ++cc) blku_kacc<NB>(kr, ki, xv[cc], lv[cc]);
        }
        double acc1, acc2;
        if constexpr (NB == 2)
          blku_contract<NB, GORD>([&](int j, int e) { return areg[j][e]; }, kr, ki, u1, u2, acc1, acc2);
        else {
          // the block's A_j read from LDS where used: an opaque copy of the block index keeps the compiler from
          // hoisting all 3 E of them out of the loop into registers (they spill)
          int bc = be;
          asm volatile("" : "+v"(bc));
          blku_contract<NB, GORD>([&](int j, int e) { return ga[(j * E + e) * nblk + bc]; }, kr, ki, u1, u2, acc1,
                                  acc2);
        }
        double s1 = act ? acc1 : 0.0, s2 = act ? acc2 : 0.0;
        for (int d = 1; d < nblk; d <<= 1) {  // inclusive scan within the slice's lanes
          const double t1 = __shfl_up(s1, d), t2 = __shfl_up(s2, d);
          s1 += be >= d ? t1 : 0.0;
          s2 += be >= d ? t2 : 0.0;
        }
        if (act && be == nblk - 1) {
          double* o = bp.dJdu + ((size_t)b * Nt + a * C + jj) * nu;
          o[0] = s1;
          if (nu > 1) o[1] = s2;
        }
      }
    }
  };
  // chain lanes, one state element each: the SL lanes of group p = l / SL own rows i = l % SL < NB of block p % nblk
  // in column p / nblk (SL = 2 for blocks of 2 rows, else 4: a DPP quad; lanes i >= NB idle).  Each slice a lane
  // gathers its block's column from the group by DPP broadcasts and forms its row of U x (U^H x backward).
  constexpr int SL = NB == 2 ? 2 : 4;
  const int pq = tid / SL, ri = tid - pq * SL;
  const bool cact = chain && pq < nblk * m && ri < NB;
  const int beta = cact ? pq % nblk : 0, col = cact ? pq / nblk : 0, rr_ = min(ri, NB - 1);
  const int row = cact ? bk.brow[beta * NB + ri] : -1;
  const bool ok = row >= 0;
  double* const sink = tchain_sink(g);
  const size_t off = 2 * ((size_t)col * N + max(row, 0));
  double pen = 0.0;
  double* Sb = reinterpret_cast<double*>((cx<double>*)(FWD ? g.X : g.L) + (size_t)b * (Nt + 1) * Nm);
  const double* Xb = reinterpret_cast<const double*>((const cx<double>*)g.X + (size_t)b * (Nt + 1) * Nm);
  const double* srcb =
      (ADD && g.src) ? reinterpret_cast<const double*>((const cx<double>*)g.src + (size_t)b * (Nt + 1) * Nm) : nullptr;
  const unsigned char* pmask = (FWD || !mu_mode) ? g.pmask : nullptr;
  const double tmu = 2.0 * g.mu;
  const bool penon = pmask != nullptr;
  const bool pm = ok && pmask && pmask[off / 2];
  double xr = 0.0, xi = 0.0;
  if (ok) {
    const size_t o = off / 2;
    cx<double> v;
    if (FWD) {
      v = ((const cx<double>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0))[o];
    } else if (mu_mode) {
      v = ((const cx<double>*)g.Xt)[o];
    } else {
      if (g.cost_kind == COST_EXTERNAL) {
        v = reinterpret_cast<const cx<double>*>(Sb)[(size_t)Nt * Nm + o];
      } else {
        const cx<double> cf = g.coef[(size_t)b * 2 * m + col], t = ((const cx<double>*)g.Xt)[o];
        v = cx<double>{cf.r * t.r - cf.i * t.i, cf.r * t.i + cf.i * t.r};
      }
      if (pm) {
        v.r += tmu * Xb[(size_t)Nt * 2 * Nm + off];
        v.i += tmu * Xb[(size_t)Nt * 2 * Nm + off + 1];
      }
      if (srcb) {
        v.r += srcb[(size_t)Nt * 2 * Nm + off];
        v.i += srcb[(size_t)Nt * 2 * Nm + off + 1];
      }
    }
    xr = v.r;
    xi = v.i;
  }
  if (chain && GORD == 0) {  // the first state (x_0 / λ_Nt)
    double* p = ok ? Sb + (size_t)(FWD ? 0 : Nt) * 2 * Nm + off : sink;
    *reinterpret_cast<double2*>(p) = make_double2(xr, xi);
    if (FWD && penon) pen += pm ? xr * xr + xi * xi : 0.0;
  }
  // prologue: records of sequence chunks 0 and 1 in LDS, chunk 2's in flight, propagators of chunk 0.  The fused
  // backward's stagers run their prologue inside their own branch, so that their staging registers are not live
  // across the workers' first formation.
  if (GORD == 0 && !chain) {
    rec_load(0);
    rec_store(0);
    if (nC > 1) {
      rec_load(1);
      rec_store(1);
    }
    if (nC > 2) rec_load(2);
  }
  if (stager && stg_i == 0) {  // GORD: the staging loops (two prologue barriers of their own)
    rec_load(0);
    rec_store(0);
    if (nC > 1) {
      rec_load(1);
      rec_store(1);
    }
    rec_load(min(2, nC - 1));
    xs_load(0);
    const bool su = uin && STG == 1;  // this wave also copies the propagators
    if (su) {
      us_load(0);
      us_store(0);
      us_load(min(1, nC - 1));
    }
    lds_barrier();
    lds_barrier();
    for (int c = 0; c < nC; ++c) {
      BK_T(s0);
      // the copies run unconditionally (past the last chunk: clamped reloads into free slots): no staged register is
      // carried through a whole iteration
      rec_store(c + 2);  // loaded one iteration ago
      xs_store(c);  // read by grad(c) in the next iteration
      if (su) us_store(c + 1);  // read by the chain in the next iteration (past the last chunk: a free slot)
      rec_load(min(c + 3, nC - 1));
      xs_load(min(c + 1, nC - 1));
      if (su) us_load(min(c + 2, nC - 1));
      BK_T(s1);
      lds_barrier();
      BK_T(s2);
      BK_ADD(7, s1 - s0);
      BK_ADD(8, s2 - s1);
    }
  } else if (stager) {
    us_load(0);
    us_store(0);
    us_load(min(1, nC - 1));
    lds_barrier();
    lds_barrier();
    for (int c = 0; c < nC; ++c) {
      BK_T(s0);
      us_store(c + 1);  // read by the chain in the next iteration (past the last chunk: a free slot)
      us_load(min(c + 2, nC - 1));
      BK_T(s1);
      lds_barrier();
      BK_T(s2);
      BK_ADD(9, s1 - s0);
      BK_ADD(10, s2 - s1);
    }
  } else {
  lds_barrier();
  if (!chain && !uin) form(0);
  lds_barrier();
  if (chain) {
    // the state element's running pointer (lanes without one go to the sink with stride 0: no branch around stores)
    double* sp = ok ? Sb + (FWD ? 2 * Nm : (size_t)(Nt - 1) * 2 * Nm) + off : sink;
    const long long sst = ok ? (FWD ? 2 * (long long)Nm : -2 * (long long)Nm) : 0;
    // this lane's row of U (U^H backward: the conjugated column) at entry stride nblk
    int eo[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) eo[q] = (FWD ? rr_ * NB + q : q * NB + rr_) * nblk;
    for (int c = 0; c < nC; ++c) {
      BK_T(t0);
#ifdef QOC_PROBE
      if (bp.probe_mode != 2) {
#else
      {
#endif
        const int a = chunk_of(c), jn = min(C, Nt - a * C), ng = (jn + S - 1) / S;
        const double2* Uc = Ub + (size_t)(c & 1) * C * E * nblk + beta;
        double2* const lr = lam + (size_t)(c & 1) * C * Nm + (off >> 1);  // GORD: this element's ring entries
        // this lane's rows of the group's S prefix products (clamped past the chunk's end: never used)
        auto ldq = [&](double2(&Q)[S][NB], int gq) __attribute__((always_inline)) {
#pragma unroll
          for (int j = 0; j < S; ++j) {
            const size_t o = (size_t)posn(min(gq * S + j, jn - 1), jn) * E * nblk;
#pragma unroll
            for (int q = 0; q < NB; ++q) Q[j][q] = Uc[o + eo[q]];
          }
        };
        // one group (ns <= S positions): gather the block's column of the incoming state, y_j = Q_j x for every j
        // (independent), the additions of the non-μ backward (S = 1), the stores; the state carries on as y_{ns-1}
        auto group = [&](const double2(&Q)[S][NB], int gq) __attribute__((always_inline)) {
          const int ns = min(S, jn - gq * S);
          double ar_ = 0.0, ai_ = 0.0;
          if constexpr (ADD) {  // 2μ x_k on the mask + the caller's dL/dx(x_k), added after the slice
            const size_t o = (size_t)(a * C + posn(gq, jn)) * 2 * Nm + off;
            ar_ = pm ? tmu * Xb[o] : 0.0;
            ai_ = pm ? tmu * Xb[o + 1] : 0.0;
            if (srcb && ok) {
              ar_ += srcb[o];
              ai_ += srcb[o + 1];
            }
          }
          double gr[NB], gi[NB];
          if constexpr (SL == 2) {
            gr[0] = dpp_any<0xA0>(xr);  // quad_perm [0,0,2,2]: row 0 of the pair
            gi[0] = dpp_any<0xA0>(xi);
            gr[1] = dpp_any<0xF5>(xr);  // quad_perm [1,1,3,3]: row 1
            gi[1] = dpp_any<0xF5>(xi);
          } else {
            gr[0] = dpp_any<0x00>(xr);  // quad_perm [q,q,q,q]
            gi[0] = dpp_any<0x00>(xi);
            gr[1] = dpp_any<0x55>(xr);
            gi[1] = dpp_any<0x55>(xi);
            gr[2] = dpp_any<0xAA>(xr);
            gi[2] = dpp_any<0xAA>(xi);
            if constexpr (NB == 4) {
              gr[3] = dpp_any<0xFF>(xr);
              gi[3] = dpp_any<0xFF>(xi);
            }
          }
          double yr[S], yi[S];
#pragma unroll
          for (int j = 0; j < S; ++j) {
            double sr = 0.0, si = 0.0;
#pragma unroll
            for (int q = 0; q < NB; ++q) {
              const double uim = FWD ? Q[j][q].y : -Q[j][q].y;  // conj for Q^H
              sr = fma(Q[j][q].x, gr[q], sr);
              sr = fma(-uim, gi[q], sr);
              si = fma(Q[j][q].x, gi[q], si);
              si = fma(uim, gr[q], si);
            }
            yr[j] = sr;  // padding rows stay 0: Q is diagonal there and x is 0
            yi[j] = si;
          }
          if constexpr (ADD) {
            yr[0] += ar_;
            yi[0] += ai_;
          }
          if constexpr (GORD > 0) {  // λ_{k+1} of each slice k of the group into the ring (the group's incoming state
                                     // for its first slice)
#pragma unroll
            for (int j = 0; j < S; ++j)
              if (j < ns && ok) lr[(size_t)posn(gq * S + j, jn) * Nm] = j ? make_double2(yr[j - 1], yi[j - 1])
                                                                           : make_double2(xr, xi);
          } else {
#pragma unroll
            for (int j = 0; j < S; ++j)
              if (j < ns) {  // uniform
#ifdef QOC_PROBE
                if (bp.probe_mode != 3)
#endif
                  *reinterpret_cast<double2*>(sp) = make_double2(yr[j], yi[j]);
                sp += sst;
                if (FWD && penon) pen += pm ? yr[j] * yr[j] + yi[j] * yi[j] : 0.0;  // uniform branch
              }
          }
          xr = yr[S - 1];
          xi = yi[S - 1];
#pragma unroll
          for (int j = 0; j + 1 < S; ++j)
            if (j == ns - 1) {
              xr = yr[j];
              xi = yi[j];
            }
        };
        // two groups per iteration with the roles of the two Q register sets swapped (no register copies); the next
        // group's rows are read from LDS before this group's matvecs
        double2 Q0[S][NB], Q1[S][NB];
        ldq(Q0, 0);
        for (int gq = 0; gq < ng; gq += 2) {
          ldq(Q1, min(gq + 1, ng - 1));
          group(Q0, gq);
          if (gq + 1 >= ng) break;
          ldq(Q0, min(gq + 2, ng - 1));
          group(Q1, gq + 1);
        }
      }
      BK_T(t1);
      lds_barrier();
      BK_T(t2);
      BK_ADD(0, t1 - t0);
      BK_ADD(1, t2 - t1);
    }
  } else {
    for (int c = 0; c < nC; ++c) {
      BK_T(t0);
      if constexpr (GORD == 0) {
        if (c + 2 < nC) rec_store(c + 2);  // loaded one iteration ago
        if (c + 3 < nC) rec_load(c + 3);
      }
      BK_T(tf);
      BK_ADD(6, tf - t0);
#ifdef QOC_PROBE
      if (c + 1 < nC && bp.probe_mode != 1 && !uin) form(c + 1);
#else
      if (c + 1 < nC && !uin) form(c + 1);
#endif
      BK_T(tg);
#ifdef QOC_PROBE
      if (GORD > 0 && c > 0 && bp.probe_mode != 5) grad(c - 1);
#else
      if (GORD > 0 && c > 0) grad(c - 1);
#endif
      BK_T(t1);
      BK_ADD(5, t1 - tg);
      lds_barrier();
      BK_T(t2);
      BK_ADD(3, t1 - t0);
      BK_ADD(4, t2 - t1);
    }
    grad(nC - 1);  // GORD: the last chunk, after the chain's final barrier
  }
  }  // chain / worker waves
  if (FWD) {
    if (ok) {
      xN[off] = xr;
      xN[off + 1] = xi;
    }
    __syncthreads();
    chain_costs<double>(N, m, (const cx<double>*)g.Xt, [&](int q) { return cx<double>{xN[2 * q], xN[2 * q + 1]}; },
                        g.cost_kind, g.n_norm, block_sum(pen, red) * g.mu, red, g.J + b, g.coef + (size_t)b * 2 * m,
                        g.sc);
  }
}

// S: prefix-product group (1, 2, 4, 8; 1 for the backward with additions)
template <int NB, int S>
__global__ __launch_bounds__(blku_max_threads(NB)) void k_blku_fwd(const TChainArgs g, const BlkArgs bk, const BlkuParams bp) {
  blku_body<NB, S, true, false>(g, bk, bp, blockIdx.x, 0);
}
// backward: ADD = the state penalty or the caller's co-state source (not in μ mode), which enter after every slice
template <int NB, int S, bool ADD>
__global__ __launch_bounds__(blku_max_threads(NB)) void k_blku_bwd(const TChainArgs g, const BlkArgs bk, const BlkuParams bp) {
  static_assert(!ADD || S == 1, "additions after every slice: no prefix groups");
  blku_body<NB, S, false, ADD>(g, bk, bp, blockIdx.x, g.mu_mode);
}
// the backward chain with the fused order-ORD gradient (qoc_eval_dev / grape_sensitivity without additions): λ stays
// in LDS, dJdu -> bp.dJdu.
template <int NB, int S, int ORD>
__global__ __launch_bounds__(blku_max_threads(NB)) void k_blku_bwdg(const TChainArgs g, const BlkArgs bk, const BlkuParams bp) {
  blku_body<NB, S, false, false, ORD>(g, bk, bp, blockIdx.x, 0);
}

// The order-ORD block gradient over every (seed, slice) from the stored x_k and λ_{k+1} (blku_contract).  A unit is
// one (seed, slice); its nblk blocks are adjacent lanes of one wave, 64 / nblk units per wave-iteration, and they
// reduce through a wave-private LDS slot in a fixed order (no atomics, no workgroup barrier).  Persistent grid.
// μ mode: L holds μ and λ = coef ⊙ μ per column.
__host__ __device__ inline size_t blku_grad_lds(int NB, int nblk) { return (size_t)6 * NB * NB * nblk * 8; }

// Loaded operands of one gradient unit (the lane's block rows of x_k and λ_{k+1} for MM columns, u_k, the columns'
// λ_N coefficients in μ mode)
template <int NB, int MM>
struct BlkuGradLd {
  double2 x[MM][NB], l[MM][NB];
  double u1, u2;
};

template <int NB, int ORD, int MM>
__global__ __launch_bounds__(256) void k_blku_grad(const TChainArgs g, const BlkArgs bk, long long units, int mu_mode,
                                                   double* __restrict__ dJdu) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int E = NB * NB;
  const int N = g.N, m = MM ? MM : g.m, nu = g.nu, Nt = g.Nt, nblk = bk.nblk;
  const size_t Nm = (size_t)N * m, NN = (size_t)N * N;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  // unshifted generator blocks A_0, A_1, A_2 [3][E][nblk] (row-major e), zero outside the block and for j > nu
  double2* gsh = reinterpret_cast<double2*>(smem);
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
  const int NBP = blku_nbp(nblk), UPW = 64 / NBP, ul = l / NBP, beta = l - ul * NBP;
  const bool lact = beta < nblk;
  const int bc = min(beta, nblk - 1);
  const double2* G0 = gsh + bc;
  const double2* G1 = gsh + E * nblk + bc;
  const double2* G2 = gsh + 2 * E * nblk + bc;
  int r[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) r[i] = lact ? bk.brow[beta * NB + i] : -1;
  const long long wpb = blockDim.x >> 6;
  const long long nw = (long long)gridDim.x * wpb, wid = (long long)blockIdx.x * wpb + w;
  // K = Σ_c x_c λ_c^H from one column's rows, λ = coef μ in μ mode
  auto kacc = [&](double (&kr)[E], double (&ki)[E], const double2 (&xv)[NB], double2 (&lv)[NB], int b, int c) {
    if (mu_mode) {
      const cx<double> cf = g.coef[(size_t)b * 2 * m + c];
#pragma unroll
      for (int i = 0; i < NB; ++i) lv[i] = make_double2(cf.r * lv[i].x - cf.i * lv[i].y, cf.r * lv[i].y + cf.i * lv[i].x);
    }
    blku_kacc<NB>(kr, ki, xv, lv);
  };
  auto contract = [&](const double (&kr)[E], const double (&ki)[E], double u1, double u2, double& acc1, double& acc2) {
    blku_contract<NB, ORD>([&](int j, int e) { return (j == 0 ? G0 : j == 1 ? G1 : G2)[e * nblk]; }, kr, ki, u1, u2,
                           acc1, acc2);
  };
  // per wave-iteration: the blocks of each unit reduce through the wave's LDS slot in a fixed order
  auto reduce_store = [&](long long base, bool act, double acc1, double acc2) {
    acc1 = blku_group_sum(act ? acc1 : 0.0, NBP);
    acc2 = blku_group_sum(act ? acc2 : 0.0, NBP);
    if (beta == 0 && base + ul < units) {
      dJdu[(size_t)(base + ul) * nu] = acc1;
      if (nu > 1) dJdu[(size_t)(base + ul) * nu + 1] = acc2;
    }
  };
  auto unit_bk = [&](long long base, long long& uu, int& b, int& k) {
    const long long unit = base + ul;
    uu = unit < units ? unit : 0;
    b = (int)(uu / Nt);
    k = (int)(uu - (long long)b * Nt);
  };
  if constexpr (MM > 0) {
    // compile-time column count: the next wave-iteration's operands are loaded before this one's products
    auto load = [&](long long base, BlkuGradLd<NB, MM>& d) {
      long long uu;
      int b, k;
      unit_bk(base, uu, b, k);
      d.u1 = nu > 0 ? g.u[(size_t)uu * nu] : 0.0;
      d.u2 = nu > 1 ? g.u[(size_t)uu * nu + 1] : 0.0;
      const double* Xs = reinterpret_cast<const double*>((const cx<double>*)g.X + ((size_t)b * (Nt + 1) + k) * Nm);
      const double* Ls = reinterpret_cast<const double*>((const cx<double>*)g.L + ((size_t)b * (Nt + 1) + k + 1) * Nm);
#pragma unroll
      for (int c = 0; c < MM; ++c)
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const size_t o = 2 * ((size_t)c * N + max(r[i], 0));
          d.x[c][i] = r[i] >= 0 ? *reinterpret_cast<const double2*>(Xs + o) : make_double2(0.0, 0.0);
          d.l[c][i] = r[i] >= 0 ? *reinterpret_cast<const double2*>(Ls + o) : make_double2(0.0, 0.0);
        }
    };
    BlkuGradLd<NB, MM> cur, nxt;
    long long base = wid * UPW;
    if (base < units) load(base, cur);
    for (; base < units; base += nw * UPW) {
      const long long nb = base + nw * UPW;
      load(nb < units ? nb : base, nxt);
      long long uu;
      int b, k;
      unit_bk(base, uu, b, k);
      double kr[E], ki[E];
#pragma unroll
      for (int e = 0; e < E; ++e) kr[e] = ki[e] = 0.0;
#pragma unroll
      for (int c = 0; c < MM; ++c) kacc(kr, ki, cur.x[c], cur.l[c], b, c);
      double acc1, acc2;
      contract(kr, ki, cur.u1, cur.u2, acc1, acc2);
      reduce_store(base, lact && base + ul < units, acc1, acc2);
      cur = nxt;
    }
  } else {
    for (long long base = wid * UPW; base < units; base += nw * UPW) {
      long long uu;
      int b, k;
      unit_bk(base, uu, b, k);
      const double u1 = nu > 0 ? g.u[(size_t)uu * nu] : 0.0, u2 = nu > 1 ? g.u[(size_t)uu * nu + 1] : 0.0;
      const double* Xs = reinterpret_cast<const double*>((const cx<double>*)g.X + ((size_t)b * (Nt + 1) + k) * Nm);
      const double* Ls = reinterpret_cast<const double*>((const cx<double>*)g.L + ((size_t)b * (Nt + 1) + k + 1) * Nm);
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
        kacc(kr, ki, xv, lv, b, c);
      }
      double acc1, acc2;
      contract(kr, ki, u1, u2, acc1, acc2);
      reduce_store(base, lact && base + ul < units, acc1, acc2);
    }
  }
}

}  // namespace qoc
