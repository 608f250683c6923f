// qoc_tchain.hpp — propagation by the action of the slice exponential ("Taylor-action chains").
//
// The reference forms every propagator U_k = exponential!(A_k) (src/gradient_computations.jl:17-25) and then
// uses it only in the serial chains x_{k+1} = U_k x_k (:27-29) and λ_k = U_k^H λ_{k+1} (:52-58).  With m << N
// state columns (cavity m = 2, zz m = 4) forming U_k costs ~4 N^3 CMAC per slice while its action on the state
// costs P N^2 m (P ~ 10-13 Taylor terms).  These kernels apply the exponential to the state directly:
//
//   exp(A_k) v = e^{μ_k} (exp(Ã_k / s))^s v,   Ã_k = A_k - μ_k I = Ã_0 + Σ_j u_jk Ã_j,
//   exp(Ã/s) v ≈ Σ_{t <= P} (Ã/s)^t v / t!   (Horner-free: z_t = (Ã/s) z_{t-1} / t, acc += z_t)
//
// with Ã_j = A_j - μ_j I (host-chosen scalar shifts that shrink ||Ã_j||_1; e^{μ} is an exact scalar factor)
// and (P, s) from the bound β_k = ||Ã_0||_1 + Σ_j |u_jk| ||Ã_j||_1 >= ||Ã_k||_1: s = ⌈β_k / θ_max⌉ and the
// smallest P whose Taylor tail Σ_{t>P} (β/s)^t / t! is <= 2^-53 (fp64) / 2^-24 (fp32) — the same backward
// error bound the reference's Padé selection meets (ExpMethodHigham2005), so x_k and λ_k agree with the
// reference's U_k products to rounding.  The backward sweep uses exp(A)^H = conj(e^{μ}) exp(Ã^H).
//
// One workgroup per seed (the time axis is a serial recurrence).  Thread layout (as the propagator chains,
// qoc_chain.hpp): a thread owns output row i and part p of the inner index j = p + S q (q < JT); its JT
// elements of Ã_k are formed each step from the generators (LDS) into registers, and each Taylor term is one
// matvec with the state read from LDS (broadcast), a register reduction over the S parts, and one barrier.
// No propagator is ever written: per slice the HBM traffic is the state (and u), not 16 N^2 bytes of U_k.
#pragma once
#include "qoc_chain.hpp"

namespace qoc {

// Diagnostic cycle stamps of the term loop (tools/tchain_probe.hip builds with -DQOC_PROBE; empty otherwise).
#ifdef QOC_PROBE
static __device__ unsigned long long g_tc[16];
#define TC_T(var)                                                                \
  unsigned long long var;                                                        \
  do {                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                           \
  } while (0)
#define TC_ADD(slot, v) \
  do {                  \
    if (blockIdx.x == 7 && threadIdx.x == 0) g_tc[slot] += (v); \
  } while (0)
#else
#define TC_T(var) \
  do {            \
  } while (0)
#define TC_ADD(slot, v) \
  do {                  \
  } while (0)
#endif

// Per-(seed, slice) step data written by k_tchain_prep: e^{μ_k} and the (P, s) choice.
struct TStep {
  double pr, pi;  // e^{μ_k}
  int P, s;       // terms per substep, substeps
  double scale;   // operand scale: Taylor 1/s, Chebyshev 2/β (32-byte records: two 16-byte loads)
};

// Chebyshev coefficients per slice (c_0 = J_0(ρ), c_t = 2 J_t(ρ)), one 64-double record per slice: lane t of the
// chain reads c_t (a register), the term loop takes it with v_readlane.
constexpr int TCHEB_PMAX = 60;
constexpr int TCHEB_STRIDE = 64;

constexpr int TCHAIN_PMAX = 30;  // thresholds θ_P for P = 1..TCHAIN_PMAX
constexpr int TCHAIN_NUMAX = 8;  // controls per slice the Taylor-action chains take

// Per-step inputs of the chains (TStep + u_k), fetched one step ahead through VECTOR loads: scalar loads would
// miss the scalar cache on every new step (an L2 / HBM round trip on the critical path), and an outstanding
// scalar load shares lgkmcnt with the LDS traffic of the Taylor terms, forcing lgkmcnt(0) drains there.
// NUR: control registers (TCHAIN_NUMAX; 2 in the register-resident MFMA chains, which take nu <= 2 — six fewer
// live doubles per copy in a kernel that has to stay within 256 VGPRs).
template <int NUR>
struct TPreN {
  double pr, pi;
  int P, s;
  double scale;
  double cl;  // Chebyshev: c_t of this lane's t = lane (v_readlane'd by the term loop)
  double u[NUR];
};
using TPre = TPreN<TCHAIN_NUMAX>;
// CL: load the Chebyshev coefficient (ce valid) — a compile-time choice, so that the loads are the same on every
// path (a load skipped at run time leaves the waitcnt pass unsure of the count in flight; see TChainArgs::sink)
// ZERO: u[j >= nu] = 0 (the VALU chains read every slot).  The MFMA chains never read u[j >= nu] and pass false:
// the select needs the loaded value, and the compiler put it (with its vmcnt wait for the just-issued prefetch)
// at the loop latch.
template <int NUR, bool CL = false, bool ZERO = true>
__device__ __forceinline__ void tpre_load(const TStep* __restrict__ st, const double* __restrict__ uk, int nu,
                                          TPreN<NUR>& d, const double* __restrict__ ce = nullptr) {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));  // per-lane (VGPR) address: global_load, not s_load
  const double4 v = *reinterpret_cast<const double4*>(reinterpret_cast<const double*>(st) + z);
  d.pr = v.x;
  d.pi = v.y;
  const long long ps = __double_as_longlong(v.z);
  d.P = (int)(ps & 0xffffffff);
  d.s = (int)(ps >> 32);
  d.scale = v.w;
  if constexpr (CL) d.cl = ce[(threadIdx.x & 63) + z];
  else d.cl = ce ? ce[threadIdx.x & 63] : 0.0;
#pragma unroll
  for (int j = 0; j < NUR; ++j) {  // clamped, unconditional loads: no branches around them
    const double v = uk[min(j, nu - 1) + z];
    d.u[j] = !ZERO || j < nu ? v : 0.0;
  }
}

struct TChainParams {
  double nrm[9];              // ||Ã_j||_1, j = 0..nu (Taylor variant)
  double rad[9];              // half-width of H_j's spectral interval, Ã_j = -i (H_j - c_j I) (Chebyshev variant)
  double mur[9], mui[9];      // shifts μ_j
  double theta[TCHAIN_PMAX + 1];  // θ_P: largest β whose degree-P Taylor tail is within tolerance (θ_0 unused)
  double theta_max;           // substep bound (β / s <= theta_max)
  int pmin;                   // fewest terms per substep (2: the chains' first two products are the gradient's
                              // A_k x and A_k^2 x, captured by the register-resident MFMA chains)
};

// (P, s, e^{μ}) per unit, plus Σ P s (executed Taylor terms per direction) for the roofline accounting.
static __global__ void k_tchain_prep(int nu, long long units, const double* __restrict__ u, const TChainParams prm,
                              TStep* __restrict__ steps, unsigned long long* __restrict__ terms) {
  unsigned long long cnt = 0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < units; e += (long long)gridDim.x * blockDim.x) {
    double beta = prm.nrm[0], mr = prm.mur[0], mi = prm.mui[0];
    for (int j = 0; j < nu; ++j) {
      const double uj = u[e * nu + j];
      beta += fabs(uj) * prm.nrm[j + 1];
      mr += uj * prm.mur[j + 1];
      mi += uj * prm.mui[j + 1];
    }
    int s = 1;
    if (beta > prm.theta_max) {
      s = (int)ceil(beta / prm.theta_max);
      beta /= s;
    }
    int P = prm.pmin > 1 ? prm.pmin : 1;
    while (P < TCHAIN_PMAX && prm.theta[P] < beta) ++P;
    const double er = exp(mr);
    steps[e] = TStep{er * cos(mi), er * sin(mi), P, s, 1.0 / s};
    cnt += (unsigned long long)(P * s);
  }
  // one atomic per wave
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(terms + blockIdx.x % TERM_SLOTS, cnt);
}

// Chebyshev variant (skew-Hermitian generators, Ã_k = -i H̃_k with spectrum within [-ρ, ρ], ρ = β_k):
//   exp(Ã) v = J_0(ρ) y_0 + 2 Σ_{t>=1} J_t(ρ) y_t,  y_0 = v, y_1 = Â v / 2, y_{t+1} = Â y_t + y_{t-1},  Â = (2/ρ) Ã
// (the Jacobi-Anger expansion of e^{-iρx} with y_t = (-i)^t T_t(H̃/ρ) v: real coefficients, |y_t| <= |v|, so no
// cancellation and no substeps up to ρ ~ 40); P = the smallest with 2 Σ_{t>P} |J_t(ρ)| <= 2^-53.
__device__ void bessel_j(double rho, int K, double* j) {  // J_0..J_K(ρ)
  if (rho <= 2.0) {  // power series (no cancellation for ρ <= 2); stops once J_k < 1e-40 (k > ρ: decreasing)
    const double h = 0.5 * rho, h2 = -h * h;
    double lead = 1.0;  // (ρ/2)^k / k!
    for (int k = 0; k <= K; ++k) {
      if (k) lead *= h / k;
      if (lead < 1e-40) {
        for (int q = k; q <= K; ++q) j[q] = 0.0;
        return;
      }
      double term = lead, sum = lead;
      for (int m = 1; m < 40 && fabs(term) > 1e-22 * fabs(sum); ++m) {
        term *= h2 / (m * (double)(m + k));
        sum += term;
      }
      j[k] = sum;
    }
    return;
  }
  // Miller's backward recurrence, normalised by J_0 + 2 Σ J_2k = 1
  int K0 = (int)(rho + 4.0 * cbrt(rho)) + 30;  // J_k negligible beyond ρ + O(ρ^(1/3))
  for (int q = K0; q <= K; ++q) j[q] = 0.0;
  K0 += K0 & 1;
  double jp = 0.0, jc = 1e-280, norm = 0.0;
  for (int k = K0; k >= 1; --k) {
    const double jm = (2.0 * k / rho) * jc - jp;
    jp = jc;
    jc = jm;  // J_{k-1} (unnormalised)
    if (k - 1 <= K) j[k - 1] = jc;
    if (((k - 1) & 1) == 0) norm += (k - 1 ? 2.0 : 1.0) * jc;
    if (fabs(jc) > 1e250) {  // rescale to stay finite
      jc *= 1e-250;
      jp *= 1e-250;
      norm *= 1e-250;
      for (int q = k - 1; q <= K && q <= K0; ++q) j[q] *= 1e-250;
    }
  }
  for (int k = 0; k <= K; ++k) j[k] /= norm;
}

// ρ > 2: bessel_j's Miller recurrence in two passes with no array (a per-thread table of J_k lived in scratch):
// pass 1 gets the normalisation and the number of rescalings R; pass 2 repeats the recurrence, which yields
// J_t in descending t, i.e. in the order of the tail sum, so P and the coefficients ce[t] (J_0, 2 J_t) come out
// of the same loop.  Every value goes through the same operations as in bessel_j (the rescalings that would
// have reached the stored entry, then the division by the norm), so the coefficients are bitwise the same.
__device__ int cheb_miller(double rho, double tol, double* __restrict__ ce) {
  constexpr int K = TCHEB_PMAX + 1;
  int K0 = (int)(rho + 4.0 * cbrt(rho)) + 30;
  K0 += K0 & 1;
  double jp = 0.0, jc = 1e-280, norm = 0.0;
  int R = 0;
  for (int k = K0; k >= 1; --k) {
    const double jm = (2.0 * k / rho) * jc - jp;
    jp = jc;
    jc = jm;
    if (((k - 1) & 1) == 0) norm += (k - 1 ? 2.0 : 1.0) * jc;
    if (fabs(jc) > 1e250) {
      jc *= 1e-250;
      jp *= 1e-250;
      norm *= 1e-250;
      ++R;
    }
  }
  for (int t = K0; t <= K; ++t) ce[t] = 0.0;  // J_t negligible
  jp = 0.0;
  jc = 1e-280;
  int r = 0, P = 0;
  bool found = false;
  double tail = 0.0;
  for (int k = K0; k >= 1; --k) {
    const double jm = (2.0 * k / rho) * jc - jp;
    jp = jc;
    jc = jm;  // J_{k-1} (unnormalised)
    const int t = k - 1;
    const bool big = fabs(jc) > 1e250;
    if (t <= K) {
      double v = jc;
      for (int q = r; q < R; ++q) v *= 1e-250;  // the rescalings at this and later iterations
      v /= norm;
      if (!found && t >= 1) {  // smallest P with 2 Σ_{t>P} |J_t| <= tol
        tail += 2.0 * fabs(v);
        if (tail > tol) {
          P = t < TCHEB_PMAX ? t : TCHEB_PMAX;
          found = true;
        }
      }
      ce[t] = t ? 2.0 * v : v;
    }
    if (big) {
      jc *= 1e-250;
      jp *= 1e-250;
      ++r;
    }
  }
  return P;
}

// ρ <= 2: bessel_j's power series, again without a table.  J_k depends only on k, so the tail sum runs over
// descending k with each J_k recomputed (its (ρ/2)^k / k! by the same ascending product), and only the P + 1
// coefficients are written.  Same operations per value as bessel_j, so the same P and coefficients.
__device__ double bessel_series_k(double h, int k) {
  double lead = 1.0;
  for (int q = 1; q <= k; ++q) lead *= h / q;
  const double h2 = -h * h;
  double term = lead, sum = lead;
  for (int m = 1; m < 40 && fabs(term) > 1e-22 * fabs(sum); ++m) {
    term *= h2 / (m * (double)(m + k));
    sum += term;
  }
  return sum;
}

__device__ int cheb_series(double rho, double tol, double* __restrict__ ce, int pmin) {
  constexpr int K = TCHEB_PMAX + 1;
  const double h = 0.5 * rho;
  int kz = K + 1;  // J_k = 0 for k >= kz (bessel_j stops once (ρ/2)^k / k! < 1e-40)
  double lead = 1.0;
  for (int k = 1; k <= K; ++k) {
    lead *= h / k;
    if (lead < 1e-40) {
      kz = k;
      break;
    }
  }
  double tail = 0.0;
  int P = 0;
  for (int k = kz - 1; k >= 1; --k) {  // smallest P with 2 Σ_{t>P} |J_t| <= tol
    tail += 2.0 * fabs(bessel_series_k(h, k));
    if (tail > tol) {
      P = k < TCHEB_PMAX ? k : TCHEB_PMAX;
      break;
    }
  }
  if (P < pmin) P = pmin;  // more terms than the tail needs: the extra coefficients are just as exact
  for (int k = 0; k <= P; ++k) {
    const double v = bessel_series_k(h, k);
    ce[k] = k ? 2.0 * v : v;
  }
  return P;
}

// One wave per workgroup, 64 consecutive (seed, slice) units per wave-iteration.  The coefficients are computed into
// an LDS row per lane (65-double stride: conflict-free columns) and leave the wave as one coalesced block -- rows
// e0 .. e0+63 are contiguous in HBM -- of the first PW = max(P + 1) entries of each row (the chains read 0 .. P).
// Per-lane strided 8-byte stores straight to HBM left partially written lines L2 several times over (4x the
// record bytes on the tunable bus).  Entries P+1 .. PW-1 are zero.
constexpr int TCHEB_LDS_STRIDE = TCHEB_STRIDE + 1;
static __global__ __launch_bounds__(64) void k_tchain_prep_cheb(int nu, long long units, const double* __restrict__ u,
                                                                const TChainParams prm, TStep* __restrict__ steps,
                                                                double* __restrict__ coef,
                                                                unsigned long long* __restrict__ terms, int pwmin) {
  __shared__ double rows[64 * TCHEB_LDS_STRIDE];
  const int l = threadIdx.x;
  double* ce = rows + l * TCHEB_LDS_STRIDE;
  unsigned long long cnt = 0;
  const double tol = 1.1102230246251565e-16;
  for (long long e0 = (long long)blockIdx.x * 64; e0 < units; e0 += (long long)gridDim.x * 64) {
    const long long e = e0 + l;
    const bool valid = e < units;
    for (int t = 0; t < TCHEB_STRIDE; ++t) ce[t] = 0.0;
    int P = -1;
    if (valid) {
      double beta = prm.rad[0], mr = prm.mur[0], mi = prm.mui[0];  // ρ_k >= the spectral radius of H̃_k (Weyl)
      for (int j = 0; j < nu; ++j) {
        const double uj = u[e * nu + j];
        beta += fabs(uj) * prm.rad[j + 1];
        mr += uj * prm.mur[j + 1];
        mi += uj * prm.mui[j + 1];
      }
      beta = fmax(beta, 1e-300);
      int s = 1;
      if (beta > 25.0) s = (int)ceil(beta / 25.0);  // substeps only beyond ρ = 25 (P <= 58 < TCHEB_PMAX)
      const double rho = beta / s;
      if (rho <= 2.0) {
        P = cheb_series(rho, tol, ce, prm.pmin);
      } else {
        P = cheb_miller(rho, tol, ce);  // every coefficient 0..TCHEB_PMAX written
        if (P < prm.pmin) P = prm.pmin;
      }
      const double er = exp(mr);
      steps[e] = TStep{er * cos(mi), er * sin(mi), P, s, 2.0 / beta};
      cnt += (unsigned long long)(P * s);
    }
    int pw = P + 1;
    for (int o = 32; o > 0; o >>= 1) pw = max(pw, __shfl_xor(pw, o));
    pw = min(max((pw + 1) & ~1, pwmin), TCHEB_STRIDE);
    __syncthreads();
    const int nrow = (int)min<long long>(64, units - e0);
    double* dst = coef + (size_t)e0 * TCHEB_STRIDE;
    for (int f = l; f < nrow * pw; f += 64) {
      const int r = f / pw, j = f - r * pw;
      dst[(size_t)r * TCHEB_STRIDE + j] = rows[r * TCHEB_LDS_STRIDE + j];
    }
    __syncthreads();
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if (l == 0 && cnt) atomicAdd(terms + blockIdx.x % TERM_SLOTS, cnt);
}

// The Chebyshev prep's default form (qoc_run_tchain.hip tchain_prep: the A/B against k_tchain_prep_cheb): one thread
// per unit, its coefficient row stored straight to HBM
static __global__ void k_tchain_prep_cheb_strided(int nu, long long units, const double* __restrict__ u,
                                                  const TChainParams prm, TStep* __restrict__ steps,
                                                  double* __restrict__ coef, unsigned long long* __restrict__ terms) {
  unsigned long long cnt = 0;
  const double tol = 1.1102230246251565e-16;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < units; e += (long long)gridDim.x * blockDim.x) {
    double beta = prm.rad[0], mr = prm.mur[0], mi = prm.mui[0];
    for (int j = 0; j < nu; ++j) {
      const double uj = u[e * nu + j];
      beta += fabs(uj) * prm.rad[j + 1];
      mr += uj * prm.mur[j + 1];
      mi += uj * prm.mui[j + 1];
    }
    beta = fmax(beta, 1e-300);
    int s = 1;
    if (beta > 25.0) s = (int)ceil(beta / 25.0);
    const double rho = beta / s;
    double* ce = coef + (size_t)e * TCHEB_STRIDE;
    int P = 0;
    if (rho <= 2.0) {
      P = cheb_series(rho, tol, ce, prm.pmin);
    } else {
      P = cheb_miller(rho, tol, ce);
      if (P < prm.pmin) P = prm.pmin;
    }
    const double er = exp(mr);
    steps[e] = TStep{er * cos(mi), er * sin(mi), P, s, 2.0 / beta};
    cnt += (unsigned long long)(P * s);
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(terms + blockIdx.x % TERM_SLOTS, cnt);
}

struct TChainArgs {
  int N, m, nu, Nt;
  const void* At;          // (nu+1) N x N shifted generators Ã_j, column-major (device precision)
  const double* u;         // B x Nt x nu
  const TStep* steps;      // B x Nt
  const void* x0;          // N x m or B x N x m
  int x0_per_seed;
  void* X;                 // B x (Nt+1) x N x m states
  void* L;                 // B x (Nt+1) x N x m co-states
  const void* Xt;          // N x m target
  int cost_kind;
  double n_norm;
  const unsigned char* pmask;  // N x m state-penalty mask (nullptr: no penalty)
  double mu;
  double* J;               // B
  cx<double>* coef;        // B x 2m λ_N coefficients ([sector][column], chain_costs)
  Sectors sc;              // row sectors of a packed state (compress_states)
  const void* src;         // B x (Nt+1) x N x m caller's dL/dx(x_k) added to λ_k (nullptr: none)
  const double* tcoef;     // B x Nt x TCHEB_STRIDE Chebyshev coefficients (Chebyshev variant)
  int k_lo, k_hi;          // backward MFMA chain: slices k_hi-1 .. k_lo (k_hi < Nt: λ_{k_hi} read from L)
  int prio;                // raise the chain waves' issue priority (gradient waves share the SIMDs)
  // Register-resident MFMA chains: the first two products of every slice, D1 = Â v and D2 = Â y_1 (v = x_k forward,
  // λ_{k+1} backward, Â the scaled shifted generator), written in the state layout at slice k (nullptr: not kept).
  // They are the order-3 gradient's A_k x_k, A_k^2 x_k and A_k^H λ, (A_k^H)^2 λ up to the exact shift / scale
  // (k_grad_rr_c), so the gradient runs no generator products of its own except the contractions.
  void* cap1;
  void* cap2;
  int mu_mode;             // backward: μ_k = U_k^H .. U_{Nt-1}^H X_target (λ_k = coef ⊙ μ_k for the built-in costs),
                           // started from X_target alone: it needs no forward result and can run beside it
  // TCHAIN_SINK doubles that the MFMA chains' lanes without a state element store to, so that the per-slice stores
  // need no branch: with a skipped store on one path the waitcnt pass no longer knows how many memory operations
  // are in flight and waits for all of them (the just-issued stores and prefetches included) before the next use
  // of the step data, an HBM round trip per slice (measured: 550 cycles at N = 9, 1650 at N = 27)
  double* sink;
};
constexpr int TCHAIN_SINK = 1 << 16;
__device__ __forceinline__ double* tchain_sink(const TChainArgs& g) {
  return g.sink + 2 * (((size_t)blockIdx.x * blockDim.x + threadIdx.x) & (TCHAIN_SINK / 2 - 1));
}

// Thread layout of the Taylor-action chains.  Waves split the rows into G blocks of R = 64 / S rows and the
// columns into CGN groups (G = 1: 4 groups, G = 2: 2, else 1); each computing wave walks its columns in
// blocks of CB (NP blocks at most).  Host-side selection: tchain_shape().
struct TShape {
  int S, JT, CB, NP;
};
__host__ __device__ inline TShape tchain_shape(int N, int m, bool fp64) {
  const int S = N <= 16 ? 4 : N <= 32 ? 8 : 4;
  const int R = 64 / S, G = (N + R - 1) / R, CGN = G == 1 ? 4 : G == 2 ? 2 : 1;
  const int JT = N <= 16 ? 4 : N <= 32 ? 4 : N <= 40 ? 10 : N <= 48 ? 12 : (fp64 ? 0 : 16);
  const int cpw = (m + CGN - 1) / CGN;  // columns per computing wave
  const int CB = JT >= 10 ? (cpw >= 2 ? 2 : 1) : (cpw >= 2 ? 2 : 1);
  const int NP = (cpw + CB - 1) / CB;
  return {S, JT, CB, NP <= 1 ? 1 : NP <= 2 ? 2 : NP <= 4 ? 4 : 0};  // NP 0: outside the envelope
}

template <typename T, int S, int JT, int CB, int NP>
struct TChain {
  static constexpr int XS = S * JT;  // LDS state column stride (rows >= N held at zero)
  static constexpr int R = 64 / S;   // rows per wave
  // N <= 16 (S = 4, JT = 4): every row of a column lives in one wave and the columns are split over the
  // waves, so a wave only ever reads back what it wrote itself — LDS operations of one wave complete in
  // order, and no workgroup barrier is needed between Taylor terms.
  static constexpr bool SOLO = S == 4 && JT == 4;
  static __device__ __forceinline__ void sync() {
    if constexpr (SOLO) {
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    } else {
      lds_barrier();
    }
  }
  int i, p, c_begin, c_step;
  bool act, busy;

  __device__ __forceinline__ void setup(int N) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int G = (N + R - 1) / R, CGN = G == 1 ? 4 : G == 2 ? 2 : 1;
    const int rb = w % G, cg = w / G;
    i = rb * R + l % R;
    p = l / R;
    busy = w < G * CGN;
    act = busy && i < N;
    c_begin = busy ? cg * CB : 1 << 20;
    c_step = CGN * CB;
  }
  // sum over the S parts of a row (lane offsets R, 2R, ..): row rotations, then row / half swaps
  __device__ __forceinline__ T psum(T v) const {
    if (R <= 8) v += dpp_mov<0x128>(v);  // row_ror:8
    if (R <= 4) v += dpp_mov<0x124>(v);  // row_ror:4
    return swap_sum<32>(swap_sum<16>(v));
  }
  // a[q] = Ã_k[i, p + S q] (forward) from the generators in LDS (column-major: G_j[r + N c]); the backward
  // kernels keep the conjugate transposes there, so the same read gives Ã_k^H.  Zero outside N x N.
  __device__ __forceinline__ void form(int N, int nu, const cx<T>* __restrict__ gen, const double (&uk)[TCHAIN_NUMAX],
                                       T scale, cx<T> (&a)[JT]) const {
    const int NN = N * N, ic = min(i, N - 1);
#pragma unroll
    for (int q = 0; q < JT; ++q) a[q] = gen[ic + N * min(p + S * q, N - 1)];
#pragma unroll
    for (int j = 0; j < TCHAIN_NUMAX; ++j) {
      if (j >= nu) break;
      const T uj = (T)uk[j];
      const cx<T>* Gj = gen + (size_t)(j + 1) * NN;
#pragma unroll
      for (int q = 0; q < JT; ++q) {
        const cx<T> g = Gj[ic + N * min(p + S * q, N - 1)];
        a[q].r += uj * g.r;
        a[q].i += uj * g.i;
      }
    }
#pragma unroll
    for (int q = 0; q < JT; ++q) {
      const bool ok = act && p + S * q < N;
      a[q].r = ok ? a[q].r * scale : T(0);
      a[q].i = ok ? a[q].i * scale : T(0);
    }
  }
  // z[b] = Σ_j a_j y[j, c0 + b] over all parts (every lane of the row gets the sum)
  __device__ __forceinline__ void matvec(const cx<T> (&a)[JT], const cx<T>* __restrict__ ys, int c0, cx<T> (&z)[CB]) const {
    cx<T> yv[CB][JT];
#pragma unroll
    for (int b = 0; b < CB; ++b)
#pragma unroll
      for (int q = 0; q < JT; ++q) yv[b][q] = ys[XS * (c0 + b) + p + S * q];
    T ar0[CB], ai0[CB], ar1[CB], ai1[CB];
#pragma unroll
    for (int b = 0; b < CB; ++b) ar0[b] = ai0[b] = ar1[b] = ai1[b] = T(0);
#pragma unroll
    for (int q = 0; q < JT; ++q)
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        const cx<T> y = yv[b][q];
        T& ar = (q & 1) ? ar1[b] : ar0[b];
        T& ai = (q & 1) ? ai1[b] : ai0[b];
        ar = fma(a[q].r, y.r, ar);
        ai = fma(a[q].r, y.i, ai);
        ar = fma(-a[q].i, y.i, ar);
        ai = fma(a[q].i, y.r, ai);
      }
#pragma unroll
    for (int b = 0; b < CB; ++b) {
      z[b].r = psum(ar0[b] + ar1[b]);
      z[b].i = psum(ai0[b] + ai1[b]);
    }
  }

  // One slice: state y (LDS buffer `cur`, rows >= N zero) -> e^{μ} exp(Ã/s)^s y, left in buffer `cur` on return
  // and in acc (this lane's rows / columns).  Per substep P barriers.  `ph`: e^{μ} (forward) or its conjugate.
  __device__ __forceinline__ void step(int N, int m, const cx<T> (&a)[JT], cx<T>* __restrict__ yb, int XB, int& cur,
                                       int P, int s, cx<double> ph, cx<T> (&acc)[NP][CB]) const {
    for (int sub = 0; sub < s; ++sub) {
      const cx<T>* y0 = yb + cur * XB;
#pragma unroll
      for (int ps = 0; ps < NP; ++ps) {
        const int c0 = c_begin + c_step * ps;
#pragma unroll
        for (int b = 0; b < CB; ++b) acc[ps][b] = (c0 < m) ? y0[XS * (c0 + b) + min(i, XS - 1)] : cx<T>{0, 0};
      }
      for (int t = 1; t <= P; ++t) {
        TC_T(t0);
        const cx<T>* ys = yb + cur * XB;
        cx<T>* yn = yb + (cur ^ 1) * XB;
        // 1/t in registers: a scalar-memory table read here would share lgkmcnt with the LDS reads and make
        // the compiler drain all of them (lgkmcnt(0)) before the first FMA
        const T inv = T(1) / (T)t;
#pragma unroll
        for (int ps = 0; ps < NP; ++ps) {
          const int c0 = c_begin + c_step * ps;
          if (c0 < m) {
            cx<T> z[CB];
            matvec(a, ys, c0, z);
            TC_T(t1);
            TC_ADD(0, t1 - t0);
#pragma unroll
            for (int b = 0; b < CB; ++b) {
              z[b].r *= inv;
              z[b].i *= inv;
              acc[ps][b].r += z[b].r;
              acc[ps][b].i += z[b].i;
              if (t < P && act && p == 0 && c0 + b < m) yn[XS * (c0 + b) + i] = z[b];
            }
          }
        }
        TC_T(t2);
        if (t < P) {
          sync();
          cur ^= 1;
        }
        TC_T(t3);
        TC_ADD(1, t2 - t0);
        TC_ADD(2, t3 - t2);
        TC_ADD(3, 1);
      }
      // substep result -> the buffer the last term did not read (its readers passed the previous barrier)
      const bool last = sub == s - 1;
      cx<T>* yn = yb + (cur ^ 1) * XB;
#pragma unroll
      for (int ps = 0; ps < NP; ++ps) {
        const int c0 = c_begin + c_step * ps;
#pragma unroll
        for (int b = 0; b < CB; ++b) {
          if (last) {
            const cx<T> v = acc[ps][b];
            acc[ps][b] = cx<T>{(T)(ph.r * v.r - ph.i * v.i), (T)(ph.r * v.i + ph.i * v.r)};
          }
          if (act && p == 0 && c0 < m && c0 + b < m) yn[XS * (c0 + b) + i] = acc[ps][b];
        }
      }
      sync();
      cur ^= 1;
    }
  }
};

// x_{k+1} = exp(A_k) x_k for every slice of one seed (src/gradient_computations.jl:27-29), states -> HBM, then
// the terminal cost (+ state penalty) as k_chain_fwd.
template <typename T, int S, int JT, int CB, int NP>
__global__ __launch_bounds__(CHAIN_THREADS) void k_tchain_fwd(const TChainArgs g) {
  using C = TChain<T, S, JT, CB, NP>;
  constexpr int XS = C::XS;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, b = blockIdx.x, tid = threadIdx.x;
  const int NN = N * N, Nm = N * m, XB = XS * chain_mpad(m, CB);
  cx<T>* gen = reinterpret_cast<cx<T>*>(smem);
  cx<T>* yb = gen + (size_t)(nu + 1) * NN;
  double* red = reinterpret_cast<double*>(yb + 2 * XB);
  const cx<T>* At = (const cx<T>*)g.At;
  const cx<T>* x0b = (const cx<T>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0);
  cx<T>* Xb = (cx<T>*)g.X + (size_t)b * (Nt + 1) * Nm;
  const double* ub = g.u + (size_t)b * Nt * nu;
  const TStep* stb = g.steps + (size_t)b * Nt;
  C rg;
  rg.setup(N);
  for (int e = tid; e < (nu + 1) * NN; e += CHAIN_THREADS) gen[e] = At[e];
  for (int e = tid; e < 2 * XB; e += CHAIN_THREADS) {
    const int c = (e % XB) / XS, r = e % XS;
    yb[e] = e < XB && r < N && c < m ? x0b[r + N * c] : cx<T>{0, 0};
  }
  // this lane's state elements: columns c_begin + c_step ps + bb of row i (written by p == 0 lanes)
  bool own[NP][CB], pen_m[NP][CB];
#pragma unroll
  for (int ps = 0; ps < NP; ++ps)
#pragma unroll
    for (int bb = 0; bb < CB; ++bb) {
      const int c = rg.c_begin + rg.c_step * ps + bb;
      own[ps][bb] = rg.act && rg.p == 0 && c < m;
      pen_m[ps][bb] = own[ps][bb] && g.pmask && g.pmask[rg.i + N * c];
    }
  double pen = 0.0;
  auto store = [&](const cx<T> (&v)[NP][CB], int k_) __attribute__((always_inline)) {
    cx<T>* Xk = Xb + (size_t)k_ * Nm;
#pragma unroll
    for (int ps = 0; ps < NP; ++ps)
#pragma unroll
      for (int bb = 0; bb < CB; ++bb)
        if (own[ps][bb]) {
          Xk[rg.i + N * (rg.c_begin + rg.c_step * ps + bb)] = v[ps][bb];
          if (pen_m[ps][bb]) pen += (double)v[ps][bb].r * v[ps][bb].r + (double)v[ps][bb].i * v[ps][bb].i;
        }
  };
  __syncthreads();
  cx<T> acc[NP][CB];
#pragma unroll
  for (int ps = 0; ps < NP; ++ps)
#pragma unroll
    for (int bb = 0; bb < CB; ++bb) {
      const int c = rg.c_begin + rg.c_step * ps + bb;
      acc[ps][bb] = c < m ? yb[XS * c + min(rg.i, XS - 1)] : cx<T>{0, 0};
    }
  store(acc, 0);
  int cur = 0;
  TPre nx;
  tpre_load(stb, ub, nu, nx);
  for (int k = 0; k < Nt; ++k) {
    if (k > 0) store(acc, k);  // ahead of the prefetch (see k_tchain_mf_fwd)
    const TPre st = nx;
    const int kn = min(k + 1, Nt - 1);
    tpre_load(stb + kn, ub + (size_t)kn * nu, nu, nx);
    const int P = __builtin_amdgcn_readfirstlane(st.P), ns = __builtin_amdgcn_readfirstlane(st.s);
    cx<T> a[JT];
    rg.form(N, nu, gen, st.u, (T)st.scale, a);
    rg.step(N, m, a, yb, XB, cur, P, ns, cx<double>{st.pr, st.pi}, acc);
  }
  store(acc, Nt);
  __syncthreads();  // SOLO shapes skip the per-term barriers: x_N of every wave visible to all
  const cx<T>* xNp = yb + cur * XB;
  chain_costs<T>(N, m, (const cx<T>*)g.Xt, [&](int o) { return xNp[XS * (o / N) + o % N]; }, g.cost_kind, g.n_norm,
                 block_sum(pen, red) * g.mu, red, g.J + b, g.coef + (size_t)b * 2 * m, g.sc);
}

// λ_k = exp(A_k)^H λ_{k+1} + dL/dx(x_k) for every slice of one seed (src/gradient_computations.jl:46-58); the
// generators in LDS are the conjugate transposes Ã_j^H.
template <typename T, int S, int JT, int CB, int NP>
__global__ __launch_bounds__(CHAIN_THREADS) void k_tchain_bwd(const TChainArgs g) {
  using C = TChain<T, S, JT, CB, NP>;
  constexpr int XS = C::XS;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, b = blockIdx.x, tid = threadIdx.x;
  const int NN = N * N, Nm = N * m, XB = XS * chain_mpad(m, CB);
  cx<T>* gen = reinterpret_cast<cx<T>*>(smem);
  cx<T>* yb = gen + (size_t)(nu + 1) * NN;
  const cx<T>* At = (const cx<T>*)g.At;
  const cx<T>* Xb = (const cx<T>*)g.X + (size_t)b * (Nt + 1) * Nm;
  cx<T>* Lb = (cx<T>*)g.L + (size_t)b * (Nt + 1) * Nm;
  const cx<T>* Xt = (const cx<T>*)g.Xt;
  const double* ub = g.u + (size_t)b * Nt * nu;
  const TStep* stb = g.steps + (size_t)b * Nt;
  const T tmu = (T)(2.0 * g.mu);
  const cx<T>* srcb = g.src ? (const cx<T>*)g.src + (size_t)b * (Nt + 1) * Nm : nullptr;
  C rg;
  rg.setup(N);
  for (int e = tid; e < (nu + 1) * NN; e += CHAIN_THREADS) {
    const int j = e / NN, rc = e - j * NN, r = rc % N, c = rc / N;
    const cx<T> v = At[(size_t)j * NN + c + N * r];  // (Ã_j^H)[r, c] = conj(Ã_j[c, r])
    gen[e] = cx<T>{v.r, -v.i};
  }
  // λ_{Nt} = dJfinal/dx(x_N) (+ dL/dx(x_N)) -> buffer 0, also to HBM
  for (int e = tid; e < 2 * XB; e += CHAIN_THREADS) {
    const int c = (e % XB) / XS, r = e % XS, o = r + N * c;
    cx<T> v = {0, 0};
    if (e < XB && r < N && c < m) {
      if (g.cost_kind == COST_EXTERNAL) {
        v = Lb[(size_t)Nt * Nm + o];
      } else {
        const cx<double> cf = lam_coef(g.coef + (size_t)b * 2 * m, g.sc, m, r, c);
        const cx<T> t = Xt[o];
        v.r = (T)(cf.r * t.r - cf.i * t.i);
        v.i = (T)(cf.r * t.i + cf.i * t.r);
      }
      if (g.pmask && g.pmask[o]) {
        const cx<T> xv = Xb[(size_t)Nt * Nm + o];
        v.r += tmu * xv.r;
        v.i += tmu * xv.i;
      }
      if (srcb) {
        const cx<T> sv = srcb[(size_t)Nt * Nm + o];
        v.r += sv.r;
        v.i += sv.i;
      }
      Lb[(size_t)Nt * Nm + o] = v;
    }
    yb[e] = v;
  }
  bool own[NP][CB], pen_m[NP][CB];
#pragma unroll
  for (int ps = 0; ps < NP; ++ps)
#pragma unroll
    for (int bb = 0; bb < CB; ++bb) {
      const int c = rg.c_begin + rg.c_step * ps + bb;
      own[ps][bb] = rg.act && rg.p == 0 && c < m;
      pen_m[ps][bb] = own[ps][bb] && g.pmask && g.pmask[rg.i + N * c];
    }
  __syncthreads();
  int cur = 0;
  cx<T> acc[NP][CB];
  TPre nx;
  tpre_load(stb + Nt - 1, ub + (size_t)(Nt - 1) * nu, nu, nx);
  auto store_lam = [&](int k_) __attribute__((always_inline)) {
    cx<T>* Lk = Lb + (size_t)k_ * Nm;
#pragma unroll
    for (int ps = 0; ps < NP; ++ps)
#pragma unroll
      for (int bb = 0; bb < CB; ++bb)
        if (own[ps][bb]) Lk[rg.i + N * (rg.c_begin + rg.c_step * ps + bb)] = acc[ps][bb];
  };
  for (int k = Nt - 1; k >= 0; --k) {
    if (k < Nt - 1) store_lam(k + 1);  // ahead of the prefetch (see k_tchain_mf_fwd)
    const TPre st = nx;
    const int kp = max(k - 1, 0);
    tpre_load(stb + kp, ub + (size_t)kp * nu, nu, nx);
    const int P = __builtin_amdgcn_readfirstlane(st.P), ns = __builtin_amdgcn_readfirstlane(st.s);
    cx<T> xk[NP][CB];  // 2 mu x_k (penalty) + the caller's dL/dx(x_k), loaded ahead of the Taylor terms
#pragma unroll
    for (int ps = 0; ps < NP; ++ps)
#pragma unroll
      for (int bb = 0; bb < CB; ++bb) {
        const size_t o = (size_t)k * Nm + rg.i + N * (rg.c_begin + rg.c_step * ps + bb);
        cx<T> v = pen_m[ps][bb] ? Xb[o] : cx<T>{0, 0};
        v.r *= tmu;
        v.i *= tmu;
        if (srcb && own[ps][bb]) {
          v.r += srcb[o].r;
          v.i += srcb[o].i;
        }
        xk[ps][bb] = v;
      }
    cx<T> a[JT];
    rg.form(N, nu, gen, st.u, (T)st.scale, a);
    rg.step(N, m, a, yb, XB, cur, P, ns, cx<double>{st.pr, -st.pi}, acc);
    bool any_pen = false;
#pragma unroll
    for (int ps = 0; ps < NP; ++ps)
#pragma unroll
      for (int bb = 0; bb < CB; ++bb) {
        if (pen_m[ps][bb] || (srcb && own[ps][bb])) {
          acc[ps][bb].r += xk[ps][bb].r;
          acc[ps][bb].i += xk[ps][bb].i;
          any_pen = true;
          yb[cur * XB + XS * (rg.c_begin + rg.c_step * ps + bb) + rg.i] = acc[ps][bb];
        }
      }
    if (g.pmask || srcb) {  // the penalised entries of the state changed after the step's last barrier
      (void)any_pen;
      C::sync();
    }
  }
  store_lam(0);
}

// ---------------------------------------------------------------------------------------------------------
// fp64: the Taylor terms on v_mfma_f64_4x4x4_4b.  One wave per (16-row block, column pair): the four blocks of
// the instruction are the wave's four row quads, K runs over the k-quads, so no cross-lane reduction is needed.
// Complex arithmetic as two real products into one accumulator: with B = [yr0, yi0, yr1, yi1] (the column pair,
// one real column per n) and B' = [-yi0, yr0, -yi1, yr1],  Ar B + Ai B' = [Re, Im, Re, Im] of A y.  The state
// lives in LDS twice (y and y') so that both operands are plain ds_read_b64s.  With one wave per SIMD an fp64
// VALU instruction issues every ~8 cycles; a 4x4x4 MFMA does 256 FMAs in 16, so the matvec runs at ~4x the
// VALU formulation's issue rate and the part sums disappear.
// Lane roles (tools/mfma4_layout.hip): A[m][k] at lane m + 4b + 16k, B[k][n] at n + 4b + 16k, D[m][n] at
// n + 4b + 16m (b = (l >> 2) & 3).
// ---------------------------------------------------------------------------------------------------------
__host__ __device__ inline int tchain_mf_kq(int N) {  // k-quads per product, bucketed (zero padding is exact)
  const int q = (N + 3) / 4;
  return q <= 3 ? 3 : q <= 4 ? 4 : q <= 6 ? 6 : q <= 8 ? 8 : q <= 10 ? 10 : q <= 12 ? 12 : 0;
}
__host__ __device__ inline int tchain_mf_waves(int N, int m) { return ((N + 15) / 16) * ((m + 1) / 2); }
// Launch bound of the MFMA chain kernels: a workgroup of <= 8 waves (cavity 3, zz 2) is compiled for 512 threads,
// i.e. 256 VGPRs per wave (the KQ = 12 kernels use <= 241).  The former 1024-thread bound capped the waves at 128
// VGPRs: from KQ = 6 up the formed A rows and the step data spilled to scratch (308 B per lane at KQ = 10), and the
// reload's vmcnt(0) waited for the next step's prefetch in every slice (~3k cycles per slice at N = 40).
// MAXT = 256 (<= 4 waves, nu <= 2) additionally keeps the generators in registers (REGS in the kernels).
__host__ __device__ inline int tchain_mf_maxt(int N, int m, int nu) {
  const int w = tchain_mf_waves(N, m);
  return w <= 4 && nu <= 2 ? 256 : w <= 8 ? 512 : 1024;
}
// LDS of the MFMA chains: the generators (the register-resident variant, MAXT = 256, keeps only Ã_2 there and reads
// its register operands from HBM once), 2 x (y, y') state buffers, 16 reduction doubles + 48 for 1/t + 64 per wave
// (coefficients).  So two chain workgroups fit one CU's 160 KB (forward and backward side by side).
// rot: the TChainRot kernels (16 G-row state, one wave per column pair; G = 3 keeps every generator in LDS).
__host__ inline size_t tchain_mf_lds(int N, int m, int nu, bool rot = false) {
  const int G = (N + 15) / 16, CP = (m + 1) / 2;
  const int KQ = rot ? 4 * G : tchain_mf_kq(N);
  const bool regs = rot ? G <= 2 : tchain_mf_maxt(N, m, nu) == 256;
  // register-resident variant: Ã_0, Ã_1 in registers, Ã_2 (nu = 2) in LDS
  const size_t gen = (size_t)(regs ? (nu >= 2 ? 1 : 0) : nu + 1) * N * N * 16;
  return gen + (size_t)2 * 2 * CP * 4 * KQ * 4 * 8 + (64 + 64 * (rot ? CP : tchain_mf_waves(N, m))) * 8;
}

template <int KQ>
struct TChainMF {
  static constexpr int RP = 4 * KQ;  // padded rows of the LDS state
  static constexpr int E = 1;        // D elements per lane (TChainRot<2>: 2)
  static constexpr int KA = KQ;      // A-operand registers per generator part
  static constexpr int PD = KQ <= 10 ? 2 : 1;  // slices of step data in flight (tchain_mf_fwd_body; KQ = 12 would
                                              // pass 256 VGPRs with a second record)
  static constexpr bool REGS_OK = true;
  static constexpr int NG = 2;  // generators with register-resident A operands (Ã_0, Ã_1; Ã_2 from LDS)
  int rowA, rowD, n, kl, cp, G, CP;
  bool solo;  // one row block (N <= 16): each wave owns its column pair outright, no workgroup barriers
  bool actD;  // this lane's D element is a real state entry (row < N, column < m)
  int colD;   // complex column of the D element

  __device__ __forceinline__ void setup(int N, int m) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    G = (N + 15) / 16;
    CP = (m + 1) / 2;
    solo = G == 1;
    const int rb = w % G;
    cp = w / G;
    const int blk = (l >> 2) & 3;
    rowA = 16 * rb + 4 * blk + (l & 3);
    kl = l >> 4;
    rowD = 16 * rb + 4 * blk + (l >> 4);
    n = l & 3;
    colD = 2 * cp + (n >> 1);
    actD = rowD < N && colD < m;
  }
  __device__ __forceinline__ int rowE(int) const { return rowD; }
  __device__ __forceinline__ bool actE(int) const { return actD; }
  __device__ __forceinline__ void put_e(double* yb, int buf, int, double v) const {
    put(ybuf(yb, CP, buf, 0), ybuf(yb, CP, buf, 1), v);
  }
  // LDS state: [buf][y | y'][cp][RP rows][4]
  static __device__ __forceinline__ double* ybuf(double* yb, int CP, int buf, int prime) {
    return yb + (size_t)((buf * 2 + prime) * CP) * RP * 4;
  }
  // a = Ã_k (or its conjugate transpose, whichever the LDS generators hold) at A-operand positions
  template <int NUR>
  __device__ __forceinline__ void form(int N, int nu, const cx<double>* __restrict__ gen, const double (&uk)[NUR],
                                       double scale, double (&ar)[KQ], double (&ai)[KQ]) const {
    const int NN = N * N, rc = min(rowA, N - 1);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const cx<double> v = gen[rc + N * min(4 * q + kl, N - 1)];
      ar[q] = v.r;
      ai[q] = v.i;
    }
    // each generator's KQ elements are read into their own registers before any of them is used: with one
    // register pair reused per element the compiler waited for every read in turn (lgkmcnt(0) after each
    // ds_read_b128, ~KQ LDS latencies per generator and slice)
#pragma unroll
    for (int j = 0; j < NUR; ++j) {
      if (j >= nu) break;
      const double uj = uk[j];
      const cx<double>* Gj = gen + (size_t)(j + 1) * NN;
      cx<double> v[KQ];
#pragma unroll
      for (int q = 0; q < KQ; ++q) v[q] = Gj[rc + N * min(4 * q + kl, N - 1)];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        ar[q] += uj * v[q].r;
        ai[q] += uj * v[q].i;
      }
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const bool ok = rowA < N && 4 * q + kl < N;
      ar[q] = ok ? ar[q] * scale : 0.0;
      ai[q] = ok ? ai[q] * scale : 0.0;
    }
  }
  // Register-resident generators (nu <= 2, 256-thread launch bound): this lane's A-operand elements of Ã_0 and Ã_1
  // (HERM: of Ã_j^H, the backward chain's), read from HBM once (At: column-major Ã_j, L2-resident); Ã_2 stays in
  // LDS (a third register copy would take the kernel past the 256 VGPRs that let two chain waves share a SIMD).
  // form_regs then builds a slice's rows with KQ LDS reads at most.
  template <bool HERM>
  __device__ __forceinline__ void load_gen(int N, int nu, const cx<double>* __restrict__ At, double (&gr)[2][KQ],
                                           double (&gi)[2][KQ]) const {
    const int NN = N * N, rc = min(rowA, N - 1);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const bool ok = j <= nu && rowA < N && 4 * q + kl < N;
        const int cc = min(4 * q + kl, N - 1);
        const cx<double> v = At[(size_t)min(j, nu) * NN + (HERM ? cc + N * rc : rc + N * cc)];
        gr[j][q] = ok ? v.r : 0.0;
        gi[j][q] = ok ? (HERM ? -v.i : v.i) : 0.0;
      }
  }
  // g2: LDS image of Ã_2 (or Ã_2^H), column-major, used when nu == 2
  template <int NUR>
  __device__ __forceinline__ void form_regs(int N, int nu, const double (&gr)[2][KQ], const double (&gi)[2][KQ],
                                            const cx<double>* __restrict__ g2, const double (&uk)[NUR], double scale,
                                            double (&ar)[KQ], double (&ai)[KQ]) const {
    static_assert(NUR >= 2, "form_regs reads u_1, u_2");
    const double u1 = uk[0] * scale, u2 = uk[1] * scale;  // uk[j >= nu] = 0
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      ar[q] = fma(u1, gr[1][q], scale * gr[0][q]);
      ai[q] = fma(u1, gi[1][q], scale * gi[0][q]);
    }
    if (nu >= 2) {
      const int rc = min(rowA, N - 1);
      cx<double> v[KQ];
#pragma unroll
      for (int q = 0; q < KQ; ++q) v[q] = g2[rc + N * min(4 * q + kl, N - 1)];
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const bool ok = rowA < N && 4 * q + kl < N;
        ar[q] = fma(ok ? u2 : 0.0, v[q].r, ar[q]);
        ai[q] = fma(ok ? u2 : 0.0, v[q].i, ai[q]);
      }
    }
  }
  // D = A y for this wave's rows and column pair (y from buffer `buf`)
  __device__ __forceinline__ double matvec(const double (&ar)[KQ], const double (&ai)[KQ], const double* __restrict__ y,
                                           const double* __restrict__ yp) const {
#ifdef QOC_TCHAIN_DPP_PRIME
    // y' without LDS: B' = S P B with P the n <-> n^1 swap inside each lane quad (DPP quad_perm [1,0,3,2]) and
    // S = diag(-1, +1, -1, +1) on the output columns, so Ai B' = S (Ai (P B)): the Ai products accumulate on
    // their own chain and enter with the column sign.  Half the LDS reads per term, and put() writes y only.
    // Measured slower (tools/tchain_probe.hip, same box: N = 40 Taylor 558 vs 466 ns per term, Chebyshev 666 vs
    // 536; N = 9 equal): the DPP moves put VALU results in front of every second MFMA (VALU -> MFMA operand
    // hazards), which costs more than the LDS reads they replace.  Kept as an option.
    {
      double bv[KQ];
      const int base = (cp * RP + kl) * 4 + n;
#pragma unroll
      for (int q = 0; q < KQ; ++q) bv[q] = y[base + 16 * q];
      double d0 = 0.0, d1 = 0.0;
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        d0 = MF<double>::mma4(ar[q], bv[q], d0);
        d1 = MF<double>::mma4(ai[q], dpp_mov<0xB1>(bv[q]), d1);
      }
      return (n & 1) ? d0 + d1 : d0 - d1;
    }
#endif
    double bv[KQ], bp[KQ];
    const int base = (cp * RP + kl) * 4 + n;
#pragma unroll
    for (int q = 0; q < KQ; ++q) bv[q] = y[base + 16 * q];
#pragma unroll
    for (int q = 0; q < KQ; ++q) bp[q] = yp[base + 16 * q];
    // all operand reads are issued before the first MFMA (left to itself the scheduler keeps one read ahead of the
    // MFMAs, and each MFMA pair then waits out a read's LDS latency).  Same box, tools/tchain_probe.hip: N = 40
    // 445 vs 451 ns per Chebyshev term, N = 9 310 vs 331 (with the register spills of the 1024-thread bound
    // it had measured the other way).  QOC_TCHAIN_LAZY_READS restores the scheduler's order.
#ifndef QOC_TCHAIN_LAZY_READS
    __builtin_amdgcn_sched_barrier(0);
#endif
    // two accumulation chains, alternating, so consecutive MFMAs never depend on each other; the Ar products
    // first (their operands arrive first)
    double d0 = 0.0, d1 = 0.0;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      double& d = (q & 1) ? d1 : d0;
      d = MF<double>::mma4(ar[q], bv[q], d);
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      double& d = ((q + KQ) & 1) ? d1 : d0;
      d = MF<double>::mma4(ai[q], bp[q], d);
    }
    return d0 + d1;
  }
  // write this lane's element v (re or im of its complex entry) into y and its rotated copy into y'
  __device__ __forceinline__ void put(double* y, double* yp, double v) const {
    if (rowD < RP) {
      const int o = (cp * RP + rowD) * 4;
      y[o + n] = v;
#ifndef QOC_TCHAIN_DPP_PRIME
      yp[o + (n ^ 1)] = (n & 1) ? -v : v;  // y' = [-yi, yr]: re (n even) -> slot n+1 as is; im -> slot n-1 negated
#endif
    }
  }
  __device__ __forceinline__ void sync() const {
    if (solo) {  // LDS operations of one wave complete in order
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    } else {
      lds_barrier();
    }
  }

  // One slice (see TChain::step); acc = this lane's D element of the state.  CHEB: the Chebyshev recurrence
  // with this lane's coefficient register cl (lane t holds c_t); else Taylor (1/t from the LDS table invt).
  // CAP: the first substep's first two products D1 = Â y_0 and D2 = Â y_1 go to cd1, cd2 (P >= 2: prm.pmin).
  template <bool CHEB, bool CAP = false>
  __device__ __forceinline__ void step(int N, const double (&ar)[KQ], const double (&ai)[KQ], double* yb,
                                       const double* __restrict__ invt, int& cur, int P, int s, cx<double> ph,
                                       double (&acc_)[1], double cl, double* __restrict__ cw, double (&cd1_)[1],
                                       double (&cd2_)[1]) const {
    double &acc = acc_[0], &cd1 = cd1_[0], &cd2 = cd2_[0];
    if constexpr (CHEB) {  // this step's coefficients -> the wave's own LDS slot (in-order LDS: no barrier)
      cw[threadIdx.x & 63] = cl;
      __builtin_amdgcn_wave_barrier();
    }
    for (int sub = 0; sub < s; ++sub) {
      const double y0 = actD ? ybuf(yb, CP, cur, 0)[(cp * RP + rowD) * 4 + n] : 0.0;
      double ym1 = y0, ym2 = 0.0;  // y_{t-1}, y_{t-2} (Chebyshev)
      acc = CHEB ? cw[0] * y0 : y0;
      for (int t = 1; t <= P; ++t) {
        TC_T(t0);
        // the term's coefficient (1/t or c_t) read first: left to the scheduler it is issued after the last MFMA
        // and its LDS latency lands in front of the state write and the barrier
        const double ct = CHEB ? cw[t] : invt[t];
        __builtin_amdgcn_sched_barrier(0);
        const double D = matvec(ar, ai, ybuf(yb, CP, cur, 0), ybuf(yb, CP, cur, 1));
        if constexpr (CAP) {
          if (sub == 0 && t <= 2) {
            if (t == 1) cd1 = D;
            else cd2 = D;
          }
        }
        double z;
        if constexpr (CHEB) {
          z = t == 1 ? 0.5 * D : D + ym2;
          ym2 = ym1;
          ym1 = z;
          acc += ct * z;
        } else {
          z = D * ct;  // 1/t from LDS (an fp64 division is ~12 dependent VALU ops)
          acc += z;
        }
        TC_T(t1);
        if (t < P) {
          if (actD) put(ybuf(yb, CP, cur ^ 1, 0), ybuf(yb, CP, cur ^ 1, 1), z);
          TC_T(t2);
          sync();
          cur ^= 1;
          TC_T(t3);
          TC_ADD(4, t1 - t0);
          TC_ADD(5, t2 - t1);
          TC_ADD(6, t3 - t2);
          TC_ADD(7, 1);
        }
      }
      if (sub == s - 1) {  // e^{μ} (complex): the partner element (re <-> im) is the neighbouring lane
        const double o = dpp_mov<0xB1>(acc);  // quad_perm [1,0,3,2]
        acc = (n & 1) ? ph.r * acc + ph.i * o : ph.r * acc - ph.i * o;
      }
      if (actD) put(ybuf(yb, CP, cur ^ 1, 0), ybuf(yb, CP, cur ^ 1, 1), acc);
      sync();
      cur ^= 1;
    }
  }
};

// ---------------------------------------------------------------------------------------------------------
// N <= 32 (G = 1 or 2 row groups of 16, the zz and tunable-bus systems): the products without LDS.  One wave per
// column pair owns the whole state, G elements per lane.  In the 4x4x4_4b layout a lane's D element (row
// 16g + 4b + hi, column lo; hi = l >> 4, lo = l & 3) sits in the lane where block b's B operand holds k = hi of a
// k-quad.  Rotating the state by 4j lanes inside each 16-lane DPP row (row_ror) hands block b the k-quad
// q_j(b) = the bank that rotation brings in, and instruction (g_out, g_in, j)'s A operand holds the matching
// entries Ã[16 g_out + 4b + lo][16 g_in + 4 q_j(b) + hi] (arranged once per slice).  4 G^2 instructions per part
// (Ar, Ai) cover K = 16 G, so the state stays in registers from one Taylor term to the next: no LDS write / read
// round trip and no barrier per term (the TChainMF term's critical path: ~750 cycles at N = 9), and for G = 2 one
// wave instead of two per column pair (no cross-wave exchange).  The Ai products accumulate on their own chains
// and enter through the n <-> n^1 swap with the column sign (y' = [-yi, yr] on the output side).  The LDS state
// buffers still receive each substep's result (the cost epilogue and the penalty update read them).  Needs the
// register-resident generators of MAXT = 256 (nu <= 2): 2 x 4G^2 complex A-operand registers per generator.
// ---------------------------------------------------------------------------------------------------------
template <int G>
struct TChainRot {
  static constexpr int RP = 16 * G;     // padded rows of the LDS state
  static constexpr int E = G;           // D elements per lane
  static constexpr int KA = 4 * G * G;  // A-operand registers per generator part: [g_out][g_in][j]
  static constexpr int PD = G == 1 ? 3 : 2;  // step records in flight (PD - 1 slices of latency hidden): G = 1
                                             // slices (~7 terms at N = 9, ~1 us) are shorter than a loaded HBM
                                             // round trip
  // G <= 2: the generators' A-operand entries live in registers (MAXT = 256, nu <= 2); G = 3 (N <= 48): 2 x 36
  // complex per generator would not fit beside the 36 formed ones, so all nu + 1 generators stay in LDS and
  // form() reads each slice's entries there
  static constexpr bool REGS_OK = G <= 2;
  static constexpr int NG = G == 1 ? 3 : 2;  // register-resident generators: G = 1 keeps Ã_2 there too (4 entries)
  int n, kl, cp, CP, b4, lo, colD;
  bool solo = true;
  int qj[4];  // the k-quad rotation j brings to this lane's block
  bool act[G];
  __device__ __forceinline__ void setup(int N, int m) {
    const int l = threadIdx.x & 63;
    cp = threadIdx.x >> 6;
    CP = (m + 1) / 2;
    const int b = (l >> 2) & 3;
    b4 = 4 * b;
    kl = l >> 4;
    lo = l & 3;
    n = lo;
    colD = 2 * cp + (n >> 1);
#pragma unroll
    for (int e = 0; e < G; ++e) act[e] = rowE(e) < N && colD < m;
    qj[0] = b;
    qj[1] = __builtin_amdgcn_update_dpp(0, b, 0x124, 0xf, 0xf, false);  // row_ror:4
    qj[2] = __builtin_amdgcn_update_dpp(0, b, 0x128, 0xf, 0xf, false);  // row_ror:8
    qj[3] = __builtin_amdgcn_update_dpp(0, b, 0x12C, 0xf, 0xf, false);  // row_ror:12
  }
  __device__ __forceinline__ int rowE(int e) const { return 16 * e + b4 + kl; }  // D element e's row
  __device__ __forceinline__ bool actE(int e) const { return act[e]; }
  __device__ __forceinline__ int rowA(int go) const { return 16 * go + b4 + lo; }
  __device__ __forceinline__ int colA(int gi, int j) const { return 16 * gi + 4 * qj[j] + kl; }
  static __device__ __forceinline__ double* ybuf(double* yb, int CP, int buf, int prime) {
    return yb + (size_t)((buf * 2 + prime) * CP) * RP * 4;
  }
  // full-row DPP move with bound_ctrl (every lane has a source, so no old value is materialised first)
  template <int CTRL>
  static __device__ __forceinline__ double mv(double v) {
    const long long u = __double_as_longlong(v);
    const int lo_ = __builtin_amdgcn_update_dpp(0, (int)u, CTRL, 0xf, 0xf, true);
    const int hi_ = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi_ << 32) | (unsigned)lo_);
  }
  template <bool HERM>
  __device__ __forceinline__ void load_gen(int N, int nu, const cx<double>* __restrict__ At, double (&gr)[NG][KA],
                                           double (&gi)[NG][KA]) const {
    const int NN = N * N;
#pragma unroll
    for (int j = 0; j < NG; ++j)
#pragma unroll
      for (int x = 0; x < KA; ++x) {
        const int row = rowA(x / (4 * G)), col = colA((x / 4) % G, x % 4);
        const int rc = min(row, N - 1), cc = min(col, N - 1);
        const bool ok = j <= nu && row < N && col < N;
        const cx<double> v = At[(size_t)min(j, nu) * NN + (HERM ? cc + N * rc : rc + N * cc)];
        gr[j][x] = ok ? v.r : 0.0;
        gi[j][x] = ok ? (HERM ? -v.i : v.i) : 0.0;
      }
  }
  template <int NUR>
  __device__ __forceinline__ void form_regs(int N, int nu, const double (&gr)[NG][KA], const double (&gi)[NG][KA],
                                            const cx<double>* __restrict__ g2, const double (&uk)[NUR], double scale,
                                            double (&ar)[KA], double (&ai)[KA]) const {
    static_assert(NUR >= 2, "form_regs reads u_1, u_2");
    const double u1 = uk[0] * scale, u2 = nu >= 2 ? uk[1] * scale : 0.0;
#pragma unroll
    for (int x = 0; x < KA; ++x) {
      ar[x] = fma(u1, gr[1][x], scale * gr[0][x]);
      ai[x] = fma(u1, gi[1][x], scale * gi[0][x]);
    }
    if constexpr (NG == 3) {  // Ã_2 in registers too (zero when nu < 2)
#pragma unroll
      for (int x = 0; x < KA; ++x) {
        ar[x] = fma(u2, gr[2][x], ar[x]);
        ai[x] = fma(u2, gi[2][x], ai[x]);
      }
    } else if (nu >= 2) {
      cx<double> v[KA];
#pragma unroll
      for (int x = 0; x < KA; ++x) {
        const int row = rowA(x / (4 * G)), col = colA((x / 4) % G, x % 4);
        v[x] = g2[min(row, N - 1) + N * min(col, N - 1)];
      }
#pragma unroll
      for (int x = 0; x < KA; ++x) {
        const int row = rowA(x / (4 * G)), col = colA((x / 4) % G, x % 4);
        const bool ok = row < N && col < N;
        ar[x] = fma(ok ? u2 : 0.0, v[x].r, ar[x]);
        ai[x] = fma(ok ? u2 : 0.0, v[x].i, ai[x]);
      }
    }
  }
  // from the LDS generators (column-major; the backward kernels keep the conjugate transposes there)
  template <int NUR>
  __device__ __forceinline__ void form(int N, int nu, const cx<double>* __restrict__ gen, const double (&uk)[NUR],
                                       double scale, double (&ar)[KA], double (&ai)[KA]) const {
    const int NN = N * N;
    // the lane roles from an opaque lane index: left loop-invariant, the compiler hoists every entry's LDS offset
    // and validity out of the slice loop and runs out of registers (G = 3: 512 VGPRs and scratch)
    int l = threadIdx.x & 63;
    asm volatile("" : "+v"(l));
    const int bq = (l >> 2) & 3, lq = l & 3, kq = l >> 4;
    const int q[4] = {bq, __builtin_amdgcn_update_dpp(0, bq, 0x124, 0xf, 0xf, false),
                      __builtin_amdgcn_update_dpp(0, bq, 0x128, 0xf, 0xf, false),
                      __builtin_amdgcn_update_dpp(0, bq, 0x12C, 0xf, 0xf, false)};
#pragma unroll
    for (int go = 0; go < G; ++go) {  // one output group (4G entries) at a time: bounded transient registers
      constexpr int W = 4 * G;
      const int row = 16 * go + 4 * bq + lq, rc = min(row, N - 1);
      int off[W];
      bool ok[W];
#pragma unroll
      for (int y = 0; y < W; ++y) {
        const int col = 16 * (y / 4) + 4 * q[y % 4] + kq;
        off[y] = rc + N * min(col, N - 1);
        ok[y] = row < N && col < N;
      }
      cx<double> v[W];
#pragma unroll
      for (int y = 0; y < W; ++y) v[y] = gen[off[y]];
#pragma unroll
      for (int y = 0; y < W; ++y) {
        ar[go * W + y] = v[y].r;
        ai[go * W + y] = v[y].i;
      }
#pragma unroll
      for (int j = 0; j < NUR; ++j) {
        if (j >= nu) break;
        const double uj = uk[j];
        const cx<double>* Gj = gen + (size_t)(j + 1) * NN;
#pragma unroll
        for (int y = 0; y < W; ++y) v[y] = Gj[off[y]];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int y = 0; y < W; ++y) {
          ar[go * W + y] = fma(uj, v[y].r, ar[go * W + y]);
          ai[go * W + y] = fma(uj, v[y].i, ai[go * W + y]);
        }
      }
#pragma unroll
      for (int y = 0; y < W; ++y) {
        ar[go * W + y] = ok[y] ? ar[go * W + y] * scale : 0.0;
        ai[go * W + y] = ok[y] ? ai[go * W + y] * scale : 0.0;
      }
    }
  }
  // D = A y with y this wave's state in the D layout (G elements per lane)
  __device__ __forceinline__ void matvec(const double (&ar)[KA], const double (&ai)[KA], const double (&y)[G],
                                         double (&D)[G]) const {
    double bv[G][4];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      bv[g][0] = y[g];
      bv[g][1] = mv<0x124>(y[g]);  // row_ror:4
      bv[g][2] = mv<0x128>(y[g]);  // row_ror:8
      bv[g][3] = mv<0x12C>(y[g]);  // row_ror:12
    }
    double d0[G], d1[G];  // Ar and Ai products of each output group: 2G chains, interleaved
#pragma unroll
    for (int g = 0; g < G; ++g) d0[g] = d1[g] = 0.0;
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int go = 0; go < G; ++go) {
          const int x = (go * G + gi) * 4 + j;
          d0[go] = MF<double>::mma4(ar[x], bv[gi][j], d0[go]);
          d1[go] = MF<double>::mma4(ai[x], bv[gi][j], d1[go]);
        }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const double o = mv<0xB1>(d1[g]);  // quad_perm [1,0,3,2]: (Ai y)[n ^ 1]
      D[g] = (n & 1) ? d0[g] + o : d0[g] - o;
    }
  }
  // this lane's element of row `row` into y and its rotated copy into y' (see TChainMF::put)
  __device__ __forceinline__ void put_row(double* y, double* yp, int row, double v) const {
    const int o = (cp * RP + row) * 4;
    y[o + n] = v;
    yp[o + (n ^ 1)] = (n & 1) ? -v : v;
  }
  __device__ __forceinline__ void put_e(double* yb, int buf, int e, double v) const {
    put_row(ybuf(yb, CP, buf, 0), ybuf(yb, CP, buf, 1), rowE(e), v);
  }
  __device__ __forceinline__ void sync() const {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  __device__ __forceinline__ void put_all(double* yb, int buf, const double (&v)[G]) const {
#pragma unroll
    for (int e = 0; e < G; ++e)
      if (act[e]) put_row(ybuf(yb, CP, buf, 0), ybuf(yb, CP, buf, 1), rowE(e), v[e]);
  }
  // One slice (see TChainMF::step); the slice's start state is acc (this lane's D elements).
  template <bool CHEB, bool CAP = false>
  __device__ __forceinline__ void step(int N, const double (&ar)[KA], const double (&ai)[KA], double* yb,
                                       const double* __restrict__ invt, int& cur, int P, int s, cx<double> ph,
                                       double (&acc)[G], double cl, double* __restrict__ cw, double (&cd1)[G],
                                       double (&cd2)[G]) const {
    // the term coefficients: Chebyshev c_t from lane t of cl (v_readlane, no LDS round trip; they only enter the
    // sum, off the recurrence's critical path), Taylor 1/t from the LDS table
    auto coef = [&](int t) __attribute__((always_inline)) {
      if constexpr (CHEB) {
        const long long u = __double_as_longlong(cl);
        const int lo_ = __builtin_amdgcn_readlane((int)u, t), hi_ = __builtin_amdgcn_readlane((int)(u >> 32), t);
        return __longlong_as_double(((long long)hi_ << 32) | (unsigned)lo_);
      } else {
        return invt[t];
      }
    };
    (void)cw;
    for (int sub = 0; sub < s; ++sub) {
      double y[G], ym2[G];  // y_{t-1}, y_{t-2} (Chebyshev)
      const double c0 = CHEB ? coef(0) : 1.0;
#pragma unroll
      for (int e = 0; e < G; ++e) {
        y[e] = act[e] ? acc[e] : 0.0;
        ym2[e] = 0.0;
        acc[e] = c0 * y[e];
      }
      // group e's product D of term t -> the recurrence (captures, z_t, the sum) and its next B operands
      double bv[G][4];
      auto rot = [&](int e) __attribute__((always_inline)) {
        bv[e][0] = y[e];
        bv[e][1] = mv<0x124>(y[e]);  // row_ror:4
        bv[e][2] = mv<0x128>(y[e]);  // row_ror:8
        bv[e][3] = mv<0x12C>(y[e]);  // row_ror:12
      };
      auto fin = [&](int e, double D, int t, double ct) __attribute__((always_inline)) {
        if constexpr (CAP) {
          if (sub == 0 && t <= 2) {
            if (t == 1) cd1[e] = D;
            else cd2[e] = D;
          }
        }
        double z;
        if constexpr (CHEB) {
          z = t == 1 ? 0.5 * D : D + ym2[e];
          ym2[e] = y[e];
          acc[e] += ct * z;
        } else {
          z = D * ct;
          acc[e] += z;
        }
        y[e] = z;
        rot(e);
      };
      auto dsum = [&](double d0, double d1) __attribute__((always_inline)) {
        const double o = mv<0xB1>(d1);  // quad_perm [1,0,3,2]: (Ai y)[n ^ 1]
        return (n & 1) ? d0 + o : d0 - o;
      };
#pragma unroll
      for (int e = 0; e < G; ++e) rot(e);
      if constexpr (G == 1) {
        for (int t = 1; t <= P; ++t) {
          const double ct = coef(t);
          __builtin_amdgcn_sched_barrier(0);
          double d0 = 0.0, d1 = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            d0 = MF<double>::mma4(ar[j], bv[0][j], d0);
            d1 = MF<double>::mma4(ai[j], bv[0][j], d1);
          }
          fin(0, dsum(d0, d1), t, ct);
        }
      } else {
        // Software-pipelined across terms: the products of input group 0 go first, and the previous term's last
        // output group is finished behind them; the last input group runs output-group-major, so groups
        // 0..G-2 complete early and their recurrence runs behind the remaining products.  The MFMA pipe then
        // never waits for a term's tail (DPP swap, recurrence, rotations) before the next term's products.
        double pd0 = 0.0, pd1 = 0.0, pct = 0.0;  // the previous term's pending group G - 1
        for (int t = 1; t <= P; ++t) {
          const double ct = coef(t);
          double d0[G], d1[G];
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int go = 0; go < G; ++go) {
              const int x = go * G * 4 + j;
              d0[go] = MF<double>::mma4(ar[x], bv[0][j], j ? d0[go] : 0.0);
              d1[go] = MF<double>::mma4(ai[x], bv[0][j], j ? d1[go] : 0.0);
            }
          __builtin_amdgcn_sched_barrier(0);
          if (t > 1) fin(G - 1, dsum(pd0, pd1), t - 1, pct);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int gi = 1; gi < G - 1; ++gi)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int go = 0; go < G; ++go) {
                const int x = (go * G + gi) * 4 + j;
                d0[go] = MF<double>::mma4(ar[x], bv[gi][j], d0[go]);
                d1[go] = MF<double>::mma4(ai[x], bv[gi][j], d1[go]);
              }
#pragma unroll
          for (int go = 0; go < G; ++go)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int x = (go * G + G - 1) * 4 + j;
              d0[go] = MF<double>::mma4(ar[x], bv[G - 1][j], d0[go]);
              d1[go] = MF<double>::mma4(ai[x], bv[G - 1][j], d1[go]);
            }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int e = 0; e < G - 1; ++e) fin(e, dsum(d0[e], d1[e]), t, ct);
          pd0 = d0[G - 1];
          pd1 = d1[G - 1];
          pct = ct;
        }
        fin(G - 1, dsum(pd0, pd1), P, pct);
      }
      if (sub == s - 1) {
#pragma unroll
        for (int e = 0; e < G; ++e) {
          const double o = mv<0xB1>(acc[e]);
          acc[e] = (n & 1) ? ph.r * acc[e] + ph.i * o : ph.r * acc[e] - ph.i * o;
        }
      }
      put_all(yb, cur ^ 1, acc);
      sync();
      cur ^= 1;
    }
  }
};

// the chain struct of a body instantiation: KQ < 0 selects the LDS-free TChainRot<-KQ / 4>
template <int KQ>
struct TChainSel {
  using type = TChainMF<KQ>;
};
template <>
struct TChainSel<-4> {
  using type = TChainRot<1>;
};
template <>
struct TChainSel<-8> {
  using type = TChainRot<2>;
};
template <>
struct TChainSel<-12> {
  using type = TChainRot<3>;
};

// Register-resident variant (MAXT = 256, nu <= 2): the generators live in registers, not in LDS, and the first two
// products of every slice are written to g.cap1 / g.cap2 when those are set (TChainArgs); the writes of slice k
// are issued at the start of slice k + 1, next to the state's, ahead of the step-data prefetch.
template <int KQ, bool CHEB, int MAXT>
__device__ __forceinline__ void tchain_mf_fwd_body(const TChainArgs& g, const int b) {
  using C = typename TChainSel<KQ>::type;
  constexpr int KA = C::KA, E = C::E;
  constexpr int RP = C::RP;
  constexpr bool REGS = MAXT == 256 && C::REGS_OK;  // generators in registers (the dispatch picks MAXT = 256 only for nu <= 2)
  constexpr bool CAPS = REGS || KQ < 0;  // chains that write the gradient's captured products
  constexpr int NUR = REGS ? 2 : TCHAIN_NUMAX;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, tid = threadIdx.x, nthr = blockDim.x;
  const int NN = N * N, Nm = N * m, CP = (m + 1) / 2;
  cx<double>* gen = reinterpret_cast<cx<double>*>(smem);  // REGS: Ã_2 only
  double* yb = reinterpret_cast<double*>(gen + (size_t)(REGS ? (nu >= 2 ? 1 : 0) : nu + 1) * NN);
  double* red = yb + (size_t)2 * 2 * CP * RP * 4;
  double* invt = red + 16;
  double* cw = invt + 48 + 64 * (tid >> 6);  // per-wave Chebyshev coefficient slot
  const cx<double>* At = (const cx<double>*)g.At;
  const cx<double>* x0b = (const cx<double>*)g.x0 + (g.x0_per_seed ? (size_t)b * Nm : 0);
  for (int e = tid; e <= TCHAIN_PMAX; e += nthr) invt[e] = e ? 1.0 / e : 0.0;
  cx<double>* Xb = (cx<double>*)g.X + (size_t)b * (Nt + 1) * Nm;
  const double* ub = g.u + (size_t)b * Nt * nu;
  const TStep* stb = g.steps + (size_t)b * Nt;
  C rg;
  rg.setup(N, m);
  if constexpr (!REGS) {
    for (int e = tid; e < (nu + 1) * NN; e += nthr) gen[e] = At[e];
  } else if (nu >= 2) {
    for (int e = tid; e < NN; e += nthr) gen[e] = At[2 * (size_t)NN + e];
  }
  const int YB = 2 * 2 * CP * RP * 4;
  for (int e = tid; e < YB; e += nthr) yb[e] = 0.0;
  __syncthreads();
  for (int o = tid; o < CP * RP * 4; o += nthr) {  // x0 -> y, y' of buffer 0
    const int c2 = o / (RP * 4), r = (o / 4) % RP, nn = o % 4, col = 2 * c2 + (nn >> 1);
    if (r < N && col < m) {
      const cx<double> v = x0b[r + N * col];
      yb[o] = (nn & 1) ? v.i : v.r;
      yb[CP * RP * 4 + (c2 * RP + r) * 4 + (nn ^ 1)] = (nn & 1) ? -v.i : v.r;
    }
  }
  // this lane's E state elements: rows rg.rowE(e) of column rg.colD (re or im by rg.n)
  bool pen_m[E];
  size_t own[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    own[e] = (size_t)rg.rowE(e) + (size_t)N * rg.colD;
    pen_m[e] = rg.actE(e) && g.pmask && g.pmask[own[e]];
  }
  double pen = 0.0;
  double* const sink = tchain_sink(g);
  // stores without branches (TChainArgs::sink): lanes without an element write to the sink
  // count: the state enters the penalty sum (false for the loop's k = 0 rewrite of x_0)
  auto store = [&](const double (&v)[E], int k_, bool count) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      double* p = rg.actE(e) ? reinterpret_cast<double*>(Xb + (size_t)k_ * Nm + own[e]) + (rg.n & 1) : sink;
      *p = v[e];
      pen += pen_m[e] && count ? v[e] * v[e] : 0.0;
    }
  };
  const bool cap = CAPS && g.cap1 != nullptr;
  double* c1b = cap ? reinterpret_cast<double*>((cx<double>*)g.cap1 + (size_t)b * (Nt + 1) * Nm) : nullptr;
  double* c2b = cap ? reinterpret_cast<double*>((cx<double>*)g.cap2 + (size_t)b * (Nt + 1) * Nm) : nullptr;
  // real = false: the same stores, all to the sink (the loops' first iteration has no previous slice to store)
  auto cap_store = [&](const double (&d1)[E], const double (&d2)[E], int k_, bool real) __attribute__((always_inline)) {
    if constexpr (!CAPS) return;
#pragma unroll
    for (int e = 0; e < E; ++e) {  // without captures (cap1 = nullptr) every lane writes to the sink
      const bool to = cap && real && rg.actE(e);
      const size_t o = 2 * ((size_t)k_ * Nm + own[e]) + (rg.n & 1);
      double* p1 = to ? c1b + o : sink;
      double* p2 = to ? c2b + o : sink + 1;
      *p1 = d1[e];
      *p2 = d2[e];
    }
  };
  __syncthreads();
  double gr[C::NG][KA], gi[C::NG][KA];
  if constexpr (REGS) rg.template load_gen<false>(N, nu, At, gr, gi);
  double acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = rg.actE(e) ? yb[(rg.cp * RP + rg.rowE(e)) * 4 + rg.n] : 0.0;
  store(acc, 0, true);
#ifdef QOC_PROBE
  const unsigned long long c0_ = __builtin_amdgcn_s_memtime(), r0_ = __builtin_amdgcn_s_memrealtime();
#endif
  int cur = 0;
  double cd1[E] = {}, cd2[E] = {};
  const double* ceb = CHEB ? g.tcoef + (size_t)b * Nt * TCHEB_STRIDE : nullptr;
  // step data of PD slices in flight (TChainRot<1>: its slices, ~7 terms at N = 9, ~1 us, are shorter than a
  // loaded HBM round trip, so one slice of prefetch left each slice waiting for the next one's records)
  constexpr int PD = C::PD;
  TPreN<NUR> nx[PD];
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int ki = min(i, Nt - 1);
    tpre_load<NUR, CHEB, false>(stb + ki, ub + (size_t)ki * nu, nu, nx[i], CHEB ? ceb + (size_t)ki * TCHEB_STRIDE : nullptr);
  }
  for (int k0 = 0; k0 < Nt; k0 += PD)
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int k = k0 + i;
    if (k >= Nt) break;
    TC_T(s0);
    // x_k (the previous slice's result) goes to HBM here, ahead of this slice's prefetch.  The same stores in every
    // iteration (k = 0 rewrites x_0, its captures go to the sink): a store skipped on some path leaves the waitcnt
    // pass unsure how many memory operations are in flight, and the next use of the prefetched step data then
    // waited for the just-issued stores as well (an HBM round trip per slice)
    store(acc, k, k > 0);
    cap_store(cd1, cd2, max(k - 1, 0), k > 0);
    // PD = 1: copy the record, then prefetch the next into its registers.  PD > 1: use the record in place and
    // prefetch into its registers after the slice (PD - 1 slices of latency hidden): no copy, which the compiler
    // otherwise made at the loop latch from the just-issued loads, waiting for them there
    const int kn = min(k + PD, Nt - 1);
    TPreN<NUR> st_;
    if constexpr (PD == 1) {
      st_ = nx[i];
      tpre_load<NUR, CHEB, false>(stb + kn, ub + (size_t)kn * nu, nu, nx[i],
                                  CHEB ? ceb + (size_t)kn * TCHEB_STRIDE : nullptr);
    }
    const TPreN<NUR>& st = PD == 1 ? st_ : nx[i];
    const int P = __builtin_amdgcn_readfirstlane(st.P), ns = __builtin_amdgcn_readfirstlane(st.s);
    double ar[KA], ai[KA];
    if constexpr (REGS) rg.form_regs(N, nu, gr, gi, gen, st.u, st.scale, ar, ai);
    else rg.form(N, nu, gen, st.u, st.scale, ar, ai);
    TC_T(s1);
    rg.template step<CHEB, CAPS>(N, ar, ai, yb, invt, cur, P, ns, cx<double>{st.pr, st.pi}, acc, st.cl, cw, cd1, cd2);
    if constexpr (PD > 1)
      tpre_load<NUR, CHEB, false>(stb + kn, ub + (size_t)kn * nu, nu, nx[i],
                                  CHEB ? ceb + (size_t)kn * TCHEB_STRIDE : nullptr);
    TC_T(s2);
    TC_T(s3);
    TC_ADD(10, s1 - s0);
    TC_ADD(11, s2 - s1);
    TC_ADD(12, s3 - s2);
    TC_ADD(13, 1);
  }
  store(acc, Nt, true);
  cap_store(cd1, cd2, Nt - 1, true);
  __syncthreads();
#ifdef QOC_PROBE
  if (blockIdx.x == 7 && threadIdx.x == 0) {
    g_tc[8] = __builtin_amdgcn_s_memtime() - c0_;
    g_tc[9] = __builtin_amdgcn_s_memrealtime() - r0_;
  }
#endif
  const double* yN = C::ybuf(yb, CP, cur, 0);
  chain_costs<double>(N, m, (const cx<double>*)g.Xt,
                      [&](int o) {
                        const int r = o % N, col = o / N, q = ((col >> 1) * RP + r) * 4 + 2 * (col & 1);
                        return cx<double>{yN[q], yN[q + 1]};
                      },
                      g.cost_kind, g.n_norm, block_sum(pen, red) * g.mu, red, g.J + b, g.coef + (size_t)b * 2 * m, g.sc);
}

template <int KQ, bool CHEB, int MAXT>
__device__ __forceinline__ void tchain_mf_bwd_body(const TChainArgs& g, const int b) {
  using C = typename TChainSel<KQ>::type;
  constexpr int KA = C::KA, E = C::E;
  constexpr int RP = C::RP;
  constexpr bool REGS = MAXT == 256 && C::REGS_OK;  // see k_tchain_mf_fwd
  constexpr bool CAPS = REGS || KQ < 0;  // chains that write the gradient's captured products
  constexpr int NUR = REGS ? 2 : TCHAIN_NUMAX;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = g.N, m = g.m, nu = g.nu, Nt = g.Nt, tid = threadIdx.x, nthr = blockDim.x;
  const int NN = N * N, Nm = N * m, CP = (m + 1) / 2;
  cx<double>* gen = reinterpret_cast<cx<double>*>(smem);  // REGS: Ã_2^H only
  double* yb = reinterpret_cast<double*>(gen + (size_t)(REGS ? (nu >= 2 ? 1 : 0) : nu + 1) * NN);
  double* invt = yb + (size_t)2 * 2 * CP * RP * 4 + 16;
  double* cw = invt + 48 + 64 * (tid >> 6);  // per-wave Chebyshev coefficient slot
  for (int e = tid; e <= TCHAIN_PMAX; e += nthr) invt[e] = e ? 1.0 / e : 0.0;
  const cx<double>* At = (const cx<double>*)g.At;
  const cx<double>* Xb = (const cx<double>*)g.X + (size_t)b * (Nt + 1) * Nm;
  cx<double>* Lb = (cx<double>*)g.L + (size_t)b * (Nt + 1) * Nm;
  const cx<double>* Xt = (const cx<double>*)g.Xt;
  const double* ub = g.u + (size_t)b * Nt * nu;
  const TStep* stb = g.steps + (size_t)b * Nt;
  const double tmu = 2.0 * g.mu;
  // μ mode: no penalty and no co-state source (the host selects it only without them)
  const unsigned char* pmask = g.mu_mode ? nullptr : g.pmask;
  const cx<double>* srcb = (g.src && !g.mu_mode) ? (const cx<double>*)g.src + (size_t)b * (Nt + 1) * Nm : nullptr;
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  C rg;
  rg.setup(N, m);
  for (int e = tid; e < (REGS ? (nu >= 2 ? NN : 0) : (nu + 1) * NN); e += nthr) {
    const int j = (REGS ? 2 : 0) + e / NN, rc = e % NN, r = rc % N, c = rc / N;
    const cx<double> v = At[(size_t)j * NN + c + N * r];  // (Ã_j^H)[r, c] = conj(Ã_j[c, r])
    gen[e] = cx<double>{v.r, -v.i};
  }
  const int YB = 2 * 2 * CP * RP * 4;
  for (int e = tid; e < YB; e += nthr) yb[e] = 0.0;
  __syncthreads();
  // λ_{Nt} = dJfinal/dx(x_N) (+ dL/dx(x_N)) -> buffer 0 and HBM (μ mode: μ_{Nt} = X_target); a later range of
  // slices starts from the λ_{k_hi} the previous range stored
  const int k_lo = g.k_lo, k_hi = g.k_hi;
  for (int o = tid; o < Nm; o += nthr) {
    const int r = o % N, col = o / N;
    cx<double> v;
    if (k_hi < Nt) {
      v = Lb[(size_t)k_hi * Nm + o];
    } else if (g.mu_mode) {
      v = Xt[o];
    } else if (g.cost_kind == COST_EXTERNAL) {
      v = Lb[(size_t)Nt * Nm + o];
    } else {
      const cx<double> cf = lam_coef(g.coef + (size_t)b * 2 * m, g.sc, m, r, col), t = Xt[o];
      v = cx<double>{cf.r * t.r - cf.i * t.i, cf.r * t.i + cf.i * t.r};
    }
    if (k_hi == Nt) {
      if (pmask && pmask[o]) {
        const cx<double> xv = Xb[(size_t)Nt * Nm + o];
        v.r += tmu * xv.r;
        v.i += tmu * xv.i;
      }
      if (srcb) {
        v.r += srcb[(size_t)Nt * Nm + o].r;
        v.i += srcb[(size_t)Nt * Nm + o].i;
      }
      Lb[(size_t)Nt * Nm + o] = v;
    }
    const int q = ((col >> 1) * RP + r) * 4 + 2 * (col & 1);
    yb[q] = v.r;
    yb[q + 1] = v.i;
    yb[CP * RP * 4 + q + 1] = v.r;
    yb[CP * RP * 4 + q] = -v.i;
  }
  bool pen_m[E];
  size_t own[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    own[e] = (size_t)rg.rowE(e) + (size_t)N * rg.colD;
    pen_m[e] = rg.actE(e) && pmask && pmask[own[e]];
  }
  const bool cap = CAPS && g.cap1 != nullptr;
  double* c1b = cap ? reinterpret_cast<double*>((cx<double>*)g.cap1 + (size_t)b * (Nt + 1) * Nm) : nullptr;
  double* c2b = cap ? reinterpret_cast<double*>((cx<double>*)g.cap2 + (size_t)b * (Nt + 1) * Nm) : nullptr;
  double* const sink = tchain_sink(g);  // stores without branches (see the forward body)
  // real = false: the same stores, all to the sink (the loops' first iteration has no previous slice to store)
  auto cap_store = [&](const double (&d1)[E], const double (&d2)[E], int k_, bool real) __attribute__((always_inline)) {
    if constexpr (!CAPS) return;
#pragma unroll
    for (int e = 0; e < E; ++e) {  // without captures (cap1 = nullptr) every lane writes to the sink
      const bool to = cap && real && rg.actE(e);
      const size_t o = 2 * ((size_t)k_ * Nm + own[e]) + (rg.n & 1);
      double* p1 = to ? c1b + o : sink;
      double* p2 = to ? c2b + o : sink + 1;
      *p1 = d1[e];
      *p2 = d2[e];
    }
  };
  auto store_lam = [&](const double (&v)[E], int k_) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      double* p = rg.actE(e) ? reinterpret_cast<double*>(Lb + (size_t)k_ * Nm + own[e]) + (rg.n & 1) : sink;
      *p = v[e];
    }
  };
  __syncthreads();
  double gr[C::NG][KA], gi[C::NG][KA];
  if constexpr (REGS) rg.template load_gen<true>(N, nu, At, gr, gi);
  int cur = 0;
  double acc[E];  // λ at k_hi (TChainRot starts from acc)
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = rg.actE(e) ? yb[(rg.cp * RP + rg.rowE(e)) * 4 + rg.n] : 0.0;
  double cd1[E] = {}, cd2[E] = {};
  const double* ceb = CHEB ? g.tcoef + (size_t)b * Nt * TCHEB_STRIDE : nullptr;
  constexpr int PD = C::PD;  // slices of step data in flight (see tchain_mf_fwd_body)
  TPreN<NUR> nx[PD];
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int ki = max(k_hi - 1 - i, 0);
    tpre_load<NUR, CHEB, false>(stb + ki, ub + (size_t)ki * nu, nu, nx[i], CHEB ? ceb + (size_t)ki * TCHEB_STRIDE : nullptr);
  }
  for (int k0 = k_hi - 1; k0 >= k_lo; k0 -= PD)
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    const int k = k0 - i;
    if (k < k_lo) break;
    // λ_{k+1} (the previous slice's result) to HBM ahead of this slice's loads, the same stores in every iteration
    // (see tchain_mf_fwd_body; the first rewrites λ_{k_hi}, its captures go to the sink)
    store_lam(acc, k + 1);
    cap_store(cd1, cd2, k + 1, k < k_hi - 1);
    const int kp = max(k - PD, 0);
    TPreN<NUR> st_;  // see tchain_mf_fwd_body
    if constexpr (PD == 1) {
      st_ = nx[i];
      tpre_load<NUR, CHEB, false>(stb + kp, ub + (size_t)kp * nu, nu, nx[i],
                                  CHEB ? ceb + (size_t)kp * TCHEB_STRIDE : nullptr);
    }
    const TPreN<NUR>& st = PD == 1 ? st_ : nx[i];
    const int P = __builtin_amdgcn_readfirstlane(st.P), ns = __builtin_amdgcn_readfirstlane(st.s);
    double xk[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const size_t ok_ = (size_t)k * Nm + own[e];
      xk[e] = pen_m[e] ? tmu * reinterpret_cast<const double*>(Xb + ok_)[rg.n & 1] : 0.0;
      if (srcb && rg.actE(e)) xk[e] += reinterpret_cast<const double*>(srcb + ok_)[rg.n & 1];
    }
    double ar[KA], ai[KA];
    if constexpr (REGS) rg.form_regs(N, nu, gr, gi, gen, st.u, st.scale, ar, ai);
    else rg.form(N, nu, gen, st.u, st.scale, ar, ai);
    rg.template step<CHEB, CAPS>(N, ar, ai, yb, invt, cur, P, ns, cx<double>{st.pr, -st.pi}, acc, st.cl, cw, cd1, cd2);
    if constexpr (PD > 1)
      tpre_load<NUR, CHEB, false>(stb + kp, ub + (size_t)kp * nu, nu, nx[i],
                                  CHEB ? ceb + (size_t)kp * TCHEB_STRIDE : nullptr);
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (pen_m[e] || (srcb && rg.actE(e))) {
        acc[e] += xk[e];
        rg.put_e(yb, cur, e, acc[e]);
      }
    if (pmask || srcb) rg.sync();  // the penalised entries changed after the step's last barrier
  }
  store_lam(acc, k_lo);  // λ_{k_lo}
  cap_store(cd1, cd2, k_lo, true);
}

template <int KQ, bool CHEB, int MAXT>
__global__ __launch_bounds__(MAXT) void k_tchain_mf_fwd(const TChainArgs g) {
  tchain_mf_fwd_body<KQ, CHEB, MAXT>(g, blockIdx.x);
}
template <int KQ, bool CHEB, int MAXT>
__global__ __launch_bounds__(MAXT) void k_tchain_mf_bwd(const TChainArgs g) {
  tchain_mf_bwd_body<KQ, CHEB, MAXT>(g, blockIdx.x);
}

// Forward chain and μ recurrence of every seed in ONE launch of 2B workgroups (the concurrent eval): every workgroup
// is resident from the start, so each CU carries both directions' chains side by side.  Two launches on two
// streams leave the placement to the dispatcher, which can stack one direction's workgroups on some CUs while
// others idle.  The direction alternates every 8 workgroups, so that each XCD (workgroups round-robin over the
// 8 XCDs) takes both.
template <int KQ, bool CHEB, int MAXT>
__global__ __launch_bounds__(MAXT) void k_tchain_mf_dual(const TChainArgs gf, const TChainArgs gb) {
  const int i = blockIdx.x, B = gridDim.x >> 1;
  const bool by8 = (B & 7) == 0;
  const int dir = by8 ? (i >> 3) & 1 : i & 1;
  const int seed = by8 ? ((i >> 4) << 3) | (i & 7) : i >> 1;
  if (dir == 0) tchain_mf_fwd_body<KQ, CHEB, MAXT>(gf, seed);
  else tchain_mf_bwd_body<KQ, CHEB, MAXT>(gb, seed);
}

// Reference-equivalent accounting (the Taylor-action path forms no A_k norm of its own): the Padé (d, s) that
// ExpMethodHigham2005 would select for ||A_k||_1 (qoc_expm.hpp / k_expm_rr use the same rule), one wave per unit,
// lane = column (N <= 64).
template <typename T>
__global__ void k_pade_units(int N, int nu, long long units, const cx<T>* __restrict__ Agen, const double* __restrict__ u,
                             unsigned long long* __restrict__ hist) {
  const int lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
  const int NN = N * N;
  for (long long e = (long long)blockIdx.x * wpb + (threadIdx.x >> 6); e < units; e += (long long)gridDim.x * wpb) {
    double cs = 0.0;
    if (lane < N) {
      for (int r = 0; r < N; ++r) {
        double ar = Agen[r + N * lane].r, ai = Agen[r + N * lane].i;
        for (int j = 0; j < nu; ++j) {
          const double uj = u[e * nu + j];
          ar += uj * Agen[(size_t)(j + 1) * NN + r + N * lane].r;
          ai += uj * Agen[(size_t)(j + 1) * NN + r + N * lane].i;
        }
        cs += sqrt(ar * ar + ai * ai);
      }
    }
    for (int off = 32; off > 0; off >>= 1) cs = fmax(cs, __shfl_xor(cs, off));
    if (lane == 0) {
      int d, sq = 0;
      if (cs <= 2.1) {
        d = cs > 0.95 ? 9 : cs > 0.25 ? 7 : cs > 0.015 ? 5 : 3;
      } else {
        d = 13;
        const double sl = log2(cs / 5.4);
        sq = sl > 0 ? (int)ceil(sl) : 0;
      }
      atomicAdd(&hist[degree_index(d) * 64 + (sq < 63 ? sq : 63)], 1ULL);
    }
  }
}

}  // namespace qoc
