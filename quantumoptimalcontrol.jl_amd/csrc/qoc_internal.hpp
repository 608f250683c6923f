// qoc_internal.hpp — host-side internals of libqoc_mi355x.so shared by its translation units.
//
// The library is compiled as several translation units in parallel (one per kernel family, __graft_entry__.build):
//   qoc_engine.hip        the C ABI (include/qoc.h), context setup, host math, RCCL epilogue
//   qoc_run.hip           run_forward / run_backward: the propagator chains and the per-slice gradient
//   qoc_run_expm.hip      the exponential kernels (k_expm, k_expm_rr*)
//   qoc_run_tchain.hip    the Taylor-action chains (k_tchain_*)
//   qoc_run_grad.hip      the fused order-3 gradient (k_grad_rr_*)
//   qoc_run_big.hip       the large-N GEMM pipeline, the GEMM-shaped gradient and the Fréchet gradient
//   qoc_run_ode.hip       the Tsit5 path
//   qoc_run_blk.hip       the block chains and block gradient (generators with small invariant blocks)
// Each kernel template is launched from one translation unit only; the context (qoc_ctx) and the entry points
// between the units are declared here.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/qoc.h"
#include "qoc_chain.hpp"
#include "qoc_comm.hpp"
#include "qoc_tchain.hpp"

using namespace qoc;

struct qoc_ctx {
  int dev = 0, N = 0, m = 0, nu = 0, Nt = 0, B = 0, prec = QOC_FP64;
  size_t esz = 16;  // bytes per complex element on device
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;        // gradient ranges overlapped with the backward chain
  std::vector<hipEvent_t> sync_ev;      // cross-stream ordering events (no timing)
  int bwd_chunks = 4;                   // slice ranges of the overlapped backward chain (1: not overlapped)
  double bwd_last_frac = 0.5;           // last range's length relative to the others
  int bwd_prio = 0;                     // bit 0: s_setprio in the chain; bit 1: low-priority gradient stream
  int bwd_prestate = 2;                 // P1, P2 of every slice beside the first backward range (k_grad_rr_s): 0 off, 1 on, 2 auto
  void* d_A = nullptr;    // (nu+1) x N*N
  void* d_x0 = nullptr;   // N*m or B*N*m
  int x0_per_seed = 0;
  void* d_Xt = nullptr;   // N*m target
  int cost_kind = QOC_COST_TRACE;
  double cost_n = 1.0;
  unsigned char* d_pmask = nullptr;
  double mu = 0.0;
  void* d_src = nullptr;   // B x (Nt+1) x N x m caller's dL/dx(x_k) (qoc_set_costate_source), device precision
  bool src_on = false;
  double* d_u = nullptr;     // B*nu*Nt, u of the last propagate
  void* d_U = nullptr;       // B*Nt*N*N
  void* d_X = nullptr;       // B*(Nt+1)*N*m
  void* d_L = nullptr;       // B*(Nt+1)*N*m
  double* d_J = nullptr;     // B
  cx<double>* d_coef = nullptr;  // B*m
  double* d_dJdu = nullptr;  // B*nu*Nt
  int* d_flag = nullptr;
  double* d_sink = nullptr;  // TCHAIN_SINK doubles: the MFMA chains' branch-free stores of lanes without an element
  unsigned long long* d_hist = nullptr;  // 5*64 reference (Padé) selection + 8*64 executed Taylor (r, s) / T12 s
  int chain_cb_fwd = 0, chain_cb_bwd = 0;  // 0: chain_shape's column block; QOC_CHAIN_CB_FWD / _BWD = 1 | 2 (N > 32)
  int expm_alg = 1;  // 1 Taylor: register-resident T12 (default), 2 LDS Paterson-Stockmeyer (QOC_EXPM_LDS=1), 0 Padé (QOC_EXPM_PADE=1)
  int prop_method = 0;                   // QOC_PROP_EXPM / QOC_PROP_TSIT5
  int nsub = 10;                         // Tsit5 steps per slice (reference dt = 0.1 Δt)
  int ode_kernel = 0;                    // 0 register-resident rows when N fits, 1 LDS rows (QOC_ODE_LDS=1)
  double* d_stage = nullptr;             // host->device staging (fp64 complex), max(B*N*m, (nu+1)*N*N)*2
  size_t stage_elems = 0;
  std::vector<double> h_u;
  std::vector<double> h_coef;  // spline coefficients of the last qoc_propagate_spline
  // live per-kernel timing (hipEvents recorded on `stream` around each hot-path launch)
  bool profiling = false;
  struct Mark {
    int phase;
    hipEvent_t a, b;
  };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> event_pool;
  double phase_ms[4] = {0, 0, 0, 0};
  long long phase_n[4] = {0, 0, 0, 0};
  // large-N path: every k_bgemm launch bracketed while profiling (algorithmic FLOPs per launch)
  struct GMark {
    hipEvent_t a, b;
    double flops;
  };
  std::vector<GMark> gmarks;
  double gemm_ms = 0, gemm_flops = 0;
  long long gemm_n = 0;
  // large-N path (N beyond the LDS-resident kernels): chunked batched-GEMM pipeline
  bool big = false;
  int chunk = 0;                // slices per chunk
  void* d_ws = nullptr;         // chunk workspace
  double* d_red = nullptr;      // per-item reductions (chunk + 8 doubles)
  long long big_hist[5 * 64] = {};
  long long big_thist[9 * 64] = {};  // executed Taylor (r, s) on the large-N path; row 8: T8
  long long ns_iters = 0;       // Newton-Schulz iterations executed (all chunks)
  // skew-Hermitian generators: ρ_j = ||A_j||_2 (host tridiagonalisation + bisection at qoc_set_generators); the
  // chunk's Taylor degree / squarings then follow the 2-norm bound Σ_j |c_jk| ρ_j instead of the 1-norm
  double big_rho[9] = {};
  bool big_rho_ok = false;
  size_t dev_bytes = 0;
  // spline parameterisation (examples/ipopt_callbacks_exp.jl:13-14, 28)
  double* d_Bs = nullptr;  // Nt x ns
  int ns = 0;
  double* d_cstage = nullptr;  // host-pointer variants: B x ns x nu coefficients / gradient
  // GEMM-shaped gradient of the LDS-resident path (order 3, N >= 32: below that the 64-row GEMM tiles
  // are mostly padding and the per-slice k_grad is faster): generator layouts + P/Q/W workspace
  void* d_AH = nullptr;    // (nu+1) x N*N: [A0^H | A1^H | ...]
  void* d_Cst = nullptr;   // nu N x N: [A1; A2; ...]
  void* d_gws = nullptr;   // 6 x N x B(Nt+1)m
  void* d_pws = nullptr;   // 2 x N x B(Nt+1)m: P1, P2 of the state-side gradient pass (bwd_prestate)
  size_t pws_bytes = 0;
  bool grad_gemm = true;
  bool grad_rr = false;  // fused register-resident order-3 gradient (qoc_grad_rr.hpp)
  int* d_ps = nullptr;   // k_expm_rr pass-2 counter + list of Paterson-Stockmeyer units
  double a0norm = 0.0;   // ||A0||_1 of the generators (host-side, at qoc_set_generators)
  // exponential that runs: expm_alg, except that when every slice has a large norm (||A0||_1 > 4 theta_12,
  // tunable bus: ||A_k||_1 ~ 30) the default register-resident Taylor hands over to the reference's own Padé-13
  // + solve (k_expm ALG 0): over 2000 chained slices only the same algorithm holds |ΔJ| <= 1e-12 against the
  // reference (Paterson-Stockmeyer: 1.6e-12).  QOC_EXPM_PS=1 keeps Paterson-Stockmeyer there (1.8x faster).
  int expm_run = 1;
  bool expm_ps = false;
  int ncu = 256;         // compute units of the device (persistent-grid sizing)
  // Taylor-action chains (qoc_tchain.hpp): x_{k+1} = exp(A_k) x_k applied to the state, no U_k formed.
  // chain_mode 1 selects them (QOC_CHAIN=taylor / expm overrides the automatic choice at qoc_set_generators)
  int chain_mode = 0;            // 0: propagators (k_expm + k_chain_*), 1: Taylor action (k_tchain_*)
  int chain_req = QOC_CHAIN_AUTO;  // what qoc_set_chain asked for (kept across qoc_set_generators)
  bool tchain_ok = false;        // the shape fits the Taylor-action kernels
  void* d_At = nullptr;          // (nu+1) N x N shifted generators Ã_j = A_j - μ_j I
  TStep* d_steps = nullptr;      // B x Nt (P, s, e^{μ_k})
  unsigned long long* d_terms = nullptr;  // Σ P s per forward (executed Taylor terms per direction)
  TChainParams tprm{};
  bool cheb_ok = false;          // generators skew-Hermitian with imaginary shifts: Chebyshev applies
  bool cheb = false;             // Chebyshev terms (k_tchain_prep_cheb) instead of Taylor (QOC_TCHAIN_POLY=taylor)
  bool cheb_ran = false;         // what the last forward pass used (the backward pass reuses its steps)
  bool steps_stale = false;      // the last eval formed its propagators without step records (blkp): re-prep first
  double* d_tcoef = nullptr;     // B x Nt x TCHEB_STRIDE Chebyshev coefficients (allocated on first use)
  long long props_since_reset = 0;  // forward passes since the last Padé-histogram reset (chain mode 1)
  // Captured products (register-resident MFMA chains, order-3 fused gradient): the chains write their first two
  // products per slice (forward -> d_pws, backward -> d_gws) and the gradient is k_grad_rr_c, contractions only.
  bool cap_ok = false;           // the shape takes it (qoc_set_generators; QOC_CAPTURE=0 turns it off)
  bool fwd_captured = false;     // the last forward pass wrote its captures
  // qoc_eval_dev with a built-in cost and no penalty / co-state source: the backward recurrence runs from X_target
  // (μ_k, λ_k = coef ⊙ μ_k) beside the forward chain: 1 (default) both in one launch (k_tchain_mf_dual), 2 two
  // launches on two streams, 0 off (QOC_CONCURRENT)
  int concurrent = 1;
  // the MFMA chains with the state in registers (TChainRot): 1 (default) for N <= 32 with nu <= 2, 3 also for
  // N <= 48 (generators in LDS), 0 off: TChainMF everywhere (QOC_TCHAIN_ROT)
  int tchain_rot = 1;
  bool L_is_mu = false;          // d_L holds μ_k (qoc_get_costates applies the coefficients d_coef_mu)
  bool L_lazy = false;           // the fused block backward left d_L unwritten: qoc_get_costates rebuilds it
                                 // (blku_costates) from the saved u and λ_N coefficients
  double* d_u_lam = nullptr;     // B x Nt x nu: u of that backward
  void* d_blkU = nullptr;        // B x Nt x NB^2 x nblk complex: block propagators of the eval's forward (fused backward)
  size_t blkU_bytes = 0;         // its allocated size (reallocated when a new block layout needs more)
  // one control: the propagators interpolated in u (qoc_blkp.hpp k_blkp_int): the coefficient matrices of the control
  // range [int_lo, int_hi] for the live-wave layout int_wrow, degree int_D (int_ok: valid for the current generators)
  double2* d_blkp_M = nullptr;
  size_t blkp_M_bytes = 0;
  bool int_ok = false;
  int int_D = 0;
  std::vector<int> int_Db;           // per live wave block
  double int_lo = 0.0, int_hi = 0.0;
  std::vector<int> int_wrow;
  bool int_sym = false;              // complex-symmetric generators on one live wave block: d_blkp_M also holds its
  int int_nl = 0;                    // packed upper triangle of int_nl live rows, from element int_nfull on
  size_t int_nfull = 0;
  bool int_failed = false;           // [int_fail_lo, int_fail_hi] did not converge (a wider range will not either)
  double int_fail_lo = 0.0, int_fail_hi = 0.0;
  double* d_minmax = nullptr;        // k_minmax partials (256 blocks x 2)
  double* h_minmax = nullptr;        // pinned host copy
  int last_int_D = 0;                // the degree the last formation ran with (0: not interpolated; qoc_get_info)
  // the last eval / propagate ran the interpolating chains (k_blkp_ichain: no stored propagators); for the split call
  // form: grape_sensitivity's μ recurrence interpolates from the same coefficients (set by blkp_forward, cleared by
  // every other forward and by new generators)
  double2* d_blkp_ph = nullptr;      // B x Nt: e^{μ(u_k)} for the interpolating chains (k_blkp_phase)
  size_t blkp_ph_n = 0;
  int ichain_last = 0;               // 0: no, 1: every entry, 2: the symmetric propagators' upper triangle
  bool ichain_fwd = false;
  double* d_blkp_ctab = nullptr; // the Chebyshev form's coefficient table (qoc_blkp.hpp blkp_cheb), for ctab_cm / ctab_rmax
  int ctab_cm = 0;
  double ctab_rmax = 0.0;
  // the segmented block eval (qoc_blkseg.hpp) writes neither x_k nor λ_k: qoc_get_states / a later backward rebuild
  // the states on demand (blku_states) from the u in d_u, with J and the coefficients going to scratch
  bool X_lazy = false;
  // what the last propagate left for grape_sensitivity (the reference's split call form,
  // examples/ipopt_callbacks_exp.jl:11-31): 0 states in d_X (every path), 1 the segmented forward's G at every
  // segment end (d_gseg, qoc_blkseg.hpp BLKSEG_FWD), 2 the stored block propagators and states of blocks of 5..16 rows
  // (d_blkU + d_X, qoc_blkp.hpp; or the interpolating chains' states alone, ichain_fwd).  Reset by every other
  // forward or eval.
  int fwd_kind = 0;
  double2* d_gseg = nullptr;         // B x NB^2 x S x nblk complex
  size_t gseg_bytes = 0;
  int* h_flag = nullptr;             // host-mapped stale-u flag of the queued check (k_compare_u_flags)
  int flag_turn = 0;                 // which of the two device flags d_flag[0 / 1] the next queued check writes
  hipEvent_t flag_ev = nullptr;      // recorded after that copy
  double* d_J_scr = nullptr;         // B
  cx<double>* d_coef_scr = nullptr;  // B x 2m
  // every generator exactly skew-Hermitian (|A + A^H| <= 4 eps max|A|): the slice propagators are unitary, which the
  // segmented eval's backward relies on (λ_{k+1} = U_k λ_k)
  bool skew_exact = false;
  cx<double>* d_coef_lam = nullptr;  // B x 2m: its λ_N coefficients
  cx<double>* d_coef_mu = nullptr;  // B x 2m: the λ_N coefficients of the eval that left μ in d_L
  int last_eval_mode = 0;        // 0 other, 1 captured sequential backward, 2 / 3 concurrent μ mode: two streams /
                                 // one dual launch, 4 block chains' concurrent eval (qoc_get_info)
  // generators with small invariant blocks (qoc_blk.hpp, detected at qoc_set_generators; QOC_BLOCKS=0 off): the
  // chains and the gradient run per block
  int blk_nb = 0;                // padded block size 2 / 3 / 4 (VALU lanes), 16 (MFMA block waves), 0: no block path
  int nblk = 0;                  // blocks
  int* d_brow = nullptr;         // nblk x blk_nb rows of each block (-1 padding)
  int blk_jr = 0;                // chain kernels: 0 VALU lanes (k_blk_*), 1 / 4 MFMA block waves (k_blkrot_*<JR>)
  bool blk_real = false;         // MFMA block waves on the real embedding of blocks of <= 2 rows (k_blkrot_*<0>)
  int nwb = 0;                   // MFMA block waves per column pair
  int* d_wrow = nullptr;         // nwb x 16 rows of each wave's state (-1 padding)
  std::vector<int> h_wrow;       // host copy (blocks of 5..16 rows: one wave per block)
  // blocks of 5..16 rows with x_0 and X_target zero on their rows (blk_live): the waves of the others, the dead rows
  std::vector<int> h_wrow_live, h_dead_rows;
  double* d_gc_part = nullptr;   // large-N gradient: per (slice, column block) partial traces (k_gen_contract2)
  size_t gc_part_bytes = 0;
  // the dead rows known to hold zeros in the six state-shaped buffers (blk_zero_dead), and those buffers: a backward
  // with an external λ_N or a co-state source (the only writers of nonzero values into rows whose x0 and target are
  // zero) sets dead_dirty
  std::vector<int> h_dead_zeroed;
  const void* dead_bufs[6] = {};
  bool dead_dirty = true;
  int* d_wrow_live = nullptr;
  int* d_dead_rows = nullptr;
  size_t blk_dev_bytes = 0;      // d_brow + d_wrow (counted in dev_bytes)
  double* d_blkrec = nullptr;    // block propagators: B x Ntp x BLKU_REC step records (k_blku_rec, allocated on first use)
  // multi-GPU epilogue (qoc_comm.hpp): RCCL communicator over the ranks' contexts
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0;
  long long seed_offset = 0;   // global id of this context's seed 0
  double* d_best = nullptr;    // [2 local | 2 x world gathered | 2 result]
  unsigned int* d_done = nullptr;  // the segmented eval's workgroup counter (its last workgroup finds the best pair)
  double* best_out = nullptr;  // qoc_set_best_output's buffer
  bool best_direct = false;     // the last eval also wrote the final pair into the result slot and best_out
  bool best_ready = false;     // the last eval already wrote this rank's best (J, seed) into the gathered slot
  // exact (Fréchet) gradient mode workspace, allocated on first use
  void* d_fws = nullptr;
  size_t fws_bytes = 0;
  // packed states (compress_states, src/utils.jl:96-109): two parity sectors share the kernels' columns, so the
  // chains and the gradient run on m = max(n1, n2) columns instead of the caller's m_user = n1 + n2
  int m_user = 0;                       // columns of the caller's states (qoc_create's m)
  bool packed = false;
  std::vector<unsigned char> h_rsec;    // N row sectors (0 / 1)
  std::vector<int> pk_cols[2];          // original columns of sector s: packed column i holds pk_cols[s][i]
  std::vector<int> pk_pos[2];           // m_user: packed column of original column c in sector s, or -1
  int zmap[4] = {0, 1, 2, 3};           // z-calibrated cost: original column c -> s m + i
  unsigned char* d_rsec = nullptr;
  bool grad_rr_any_m = false;           // the fused gradient fits apart from the column count
  // caller-layout copies, re-packed when the packing changes
  std::vector<double> h_gen, h_x0, h_Xt;
  std::vector<int> h_pen_rows, h_pen_cols;
  bool have_gen = false, have_x0 = false, have_cost = false, have_prop = false;
  std::string err;
};

namespace qoc_host {

extern thread_local std::string g_err;
int fail(qoc_ctx* ctx, int code, const char* fmt, ...);

#define HIPCHK(ctx, expr)                                                                     \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail(ctx, QOC_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

constexpr int kChainMaxN = 64;

// ---- qoc_engine.hip: staging, packed states, timing marks, dispatch ----
int upload(qoc_ctx* ctx, const double* host, void* dev, size_t nelem);
int download(qoc_ctx* ctx, const void* dev, double* host, size_t nelem);
bool grad_rr_cols(int m);
Sectors sectors(const qoc_ctx* c);
int upload_states(qoc_ctx* c, const double* host, void* dev, size_t count, const char* what);
int download_states(qoc_ctx* c, const void* dev, double* host);
hipEvent_t take_event(qoc_ctx* c);
int mark_begin(qoc_ctx* c, int phase, hipStream_t s = nullptr);
void mark_end(qoc_ctx* c, int idx, hipStream_t s = nullptr);
RcclApi& rccl();

// ---- qoc_run_expm.hip ----
bool expm_supported(int N, int prec);
// alg 0: Padé + solve (reference algorithm); alg 1: register-resident Taylor T12; alg 2: LDS Paterson-Stockmeyer.
hipError_t launch_expm(int prec, hipStream_t s, int N, int nu, int nunits, const void* Agen, const double* u,
                       const void* Ain, void* Uout, unsigned long long* hist, int* deg, int* sq, int alg = 0,
                       unsigned long long* thist = nullptr, int* ps = nullptr, bool mix = false);

// ---- qoc_run.hip ----
template <typename T>
int run_forward(qoc_ctx* c);
template <typename T>
int run_backward(qoc_ctx* c, int order, double* d_dJdu);
template <typename T>
int dense_gradient(qoc_ctx* c, int order, double* d_dJdu);

// ---- qoc_run_big.hip ----
size_t big_ws_elems_per_item(int N, int m);
// extreme eigenvalues of the Hermitian H = i A of a skew-Hermitian generator (column-major interleaved N x N):
// Householder tridiagonalisation + Sturm bisection, O(N^3), any N
void herm_extremes(const double* A, int N, double& lmin, double& lmax);
template <typename T>
int big_forward(qoc_ctx* c);
template <typename T>
int big_backward(qoc_ctx* c, int order, double* d_dJdu);
template <typename T>
int grad_gemm_o3(qoc_ctx* c, double* d_dJdu);
template <typename T>
int frechet_grad(qoc_ctx* c, double* d_dJdu);
hipError_t launch_gen_aux(qoc_ctx* c);

// ---- qoc_run_grad.hip ----
template <typename T>
int grad_rr_o3(qoc_ctx* c, double* d_dJdu, hipStream_t st, int k0, int nk, int mode = 0);
// k_grad_rr_c: the order-3 contraction from the chains' captures (mu_mode: L holds μ, λ = coef ⊙ μ)
int grad_rr_cap(qoc_ctx* c, double* d_dJdu, hipStream_t st, int k0, int nk, bool mu_mode);

// ---- qoc_run_ode.hip ----
template <typename T>
int ode_forward(qoc_ctx* c);
template <typename T>
int ode_adjoint(qoc_ctx* c);
hipError_t launch_envelope(qoc_ctx* c, int kind, const double* dP, int np, double dt, long long nsteps);
hipError_t launch_terminal_cost(qoc_ctx* c);

// ---- qoc_run_tchain.hip ----
bool tchain_mf(const qoc_ctx* c);
bool tchain_mf_rot(const qoc_ctx* c);
template <typename T>
int tchain_forward(qoc_ctx* c);
// flags: TB_CAPTURE (write the backward captures), TB_MU (start from X_target: μ mode); st: nullptr = c->stream
enum { TB_CAPTURE = 1, TB_MU = 2 };
template <typename T>
int tchain_backward(qoc_ctx* c, int k_lo = 0, int k_hi = -1, hipStream_t st = nullptr, int flags = 0);
template <typename T>
int tchain_backward_captured(qoc_ctx* c, double* d_dJdu);
template <typename T>
int tchain_eval_concurrent(qoc_ctx* c, double* d_dJdu);
bool tchain_concurrent_ok(const qoc_ctx* c, int order);
bool tchain_cap_ok(const qoc_ctx* c);
int ensure_pws(qoc_ctx* c);
int ensure_stream2(qoc_ctx* c, int nev);
template <typename T>
int tchain_backward_overlapped(qoc_ctx* c, double* d_dJdu);
hipError_t launch_pade_units(qoc_ctx* c, long long units);
TChainArgs tchain_args(qoc_ctx* c);
int tchain_prep(qoc_ctx* c);

// ---- qoc_run_blk.hip ----
int blk_detect(qoc_ctx* c);
bool blk_active(const qoc_ctx* c);
bool blk_rot(const qoc_ctx* c);
bool blku_on(const qoc_ctx* c);
bool blkp_on(const qoc_ctx* c);  // blocks of 5..16 rows: the concurrent eval on stored propagators (qoc_blkp.hpp)
int blku_costates(qoc_ctx* c);  // qoc_get_costates after the fused block backward
int blk_forward(qoc_ctx* c);
int blk_backward(qoc_ctx* c, int order, double* d_dJdu);
bool blk_concurrent_ok(const qoc_ctx* c, int order);
int blk_eval_concurrent(qoc_ctx* c, int order, double* d_dJdu);
// the segmented block eval (qoc_blkseg.hpp): one launch for J and dJdu, x_k / λ_k rebuilt on demand
bool blkseg_ok(const qoc_ctx* c, int order);
int blkseg_eval(qoc_ctx* c, int order, const double* d_u, double* d_J, double* d_dJdu);
int blku_states(qoc_ctx* c);      // rebuild x_k after a segmented eval (no-op unless X_lazy)
// the reference's split call form on the segmented eval: propagate = phases 0-2 (G at the segment ends to HBM),
// grape_sensitivity = phase 3 (stale: the device flag of a stale-u check queued before it, or nullptr)
bool blkseg_split_ok(const qoc_ctx* c);
int blkseg_forward(qoc_ctx* c, const double* d_u, double* d_J);
int blkseg_backward(qoc_ctx* c, int order, double* d_dJdu, const int* stale);
// the same for blocks of 5..16 rows on stored propagators: propagate = formation + forward chain (1: not applicable),
// grape_sensitivity = the μ recurrence + the order-3 gradient
int blkp_forward(qoc_ctx* c);
bool blkp_backward_ok(const qoc_ctx* c, int order);
int blkp_backward(qoc_ctx* c, double* d_dJdu, const int* stale);
int blk_materialize(qoc_ctx* c);  // rebuild every lazily kept x_k / λ_k (before a setter changes what they need)

}  // namespace qoc_host
