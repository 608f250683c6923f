/*
 * qoc.h — C ABI of the MI355X-native GRAPE propagation/gradient engine (libqoc_mi355x.so).
 *
 * Drop-in boundary for the piecewise-constant Schrödinger hot path of
 * olof3/QuantumOptimalControl.jl.  Every entry point names the reference
 * interface it replaces (file:line in the reference repository).
 *
 * Conventions (identical to Julia's memory layout, so a ccall shim passes
 * arrays without conversion):
 *   - complex matrices are column-major, interleaved (re, im) double pairs
 *     (Julia Matrix{ComplexF64});
 *   - controls u are column-major nu x Nt Float64 per seed (Julia Matrix{Float64}),
 *     seeds contiguous: u[b*nu*Nt + k*nu + j] == u_b[j,k];
 *   - dJdu uses the same layout as u;
 *   - every entry point returns QOC_OK (0) or a negative error code; the
 *     message is available from qoc_last_error(ctx) (ctx may be NULL);
 *   - one caller thread per context (the reference is called from Ipopt's
 *     single callback thread, examples/ipopt_callbacks_exp.jl:11-31).
 * Host-side inputs are always fp64; a QOC_FP32 context converts them once.
 */
#ifndef QOC_MI355X_H
#define QOC_MI355X_H

#ifdef __cplusplus
extern "C" {
#endif

#define QOC_OK 0
#define QOC_ERR_ARG (-1)        /* bad argument / dimension mismatch  (src/gradient_computations.jl:84-87) */
#define QOC_ERR_HIP (-2)        /* HIP runtime failure */
#define QOC_ERR_STALE (-3)      /* u differs from the last propagate  (src/gradient_computations.jl:37-39) */
#define QOC_ERR_STATE (-4)      /* call order violated (e.g. sensitivity before propagate) */
#define QOC_ERR_UNSUPPORTED (-5)/* size outside the compiled kernel envelope */

#define QOC_FP64 0
#define QOC_FP32 1

/* dUkdp_order: 1..4 = truncated Taylor series of expm_jacobian! (src/gradient_computations.jl:177-213,
 * the reference's definition; 3 in the Ipopt path); QOC_DUKDP_EXACT = exact Fréchet derivative of the
 * propagator (opt-in, SURVEY.md §8f item 2: one 2N x 2N block exponential per slice). */
#define QOC_DUKDP_EXACT 0

#define QOC_COST_TRACE 0     /* J = 1-|tr(X'x)|^2/n^2            (src/penalty_fcns.jl:15-24) */
#define QOC_COST_ZCAL 1      /* z-calibrated, 4 columns           (src/penalty_fcns.jl:27-42, src/fidelities.jl:48-137) */
#define QOC_COST_EXTERNAL 2  /* caller supplies lambda_final      (any Julia closure dJfinal_dx) */

typedef struct qoc_ctx qoc_ctx;

/* Workspace for B seeds sharing (A0, A_j, x0, target).
 * Replaces setup_grape_cache (src/gradient_computations.jl:79-96): x, λ (B x (Nt+1) x N x m),
 * propagators Uk_vec (B x Nt x N x N), dJdu and the u copy live in HBM. */
int qoc_create(qoc_ctx** out, int device, int N, int m, int nu, int Nt, int B, int precision);
void qoc_destroy(qoc_ctx* ctx);
const char* qoc_last_error(const qoc_ctx* ctx);
/* sha256 of the sources (csrc/ and include/qoc.h) this library was compiled from ("unknown" when built
 * without the hash); the bindings refuse a library whose hash differs from the sources beside it. */
const char* qoc_source_hash(void);
void* qoc_stream(qoc_ctx* ctx);                 /* hipStream_t the engine launches on */
int qoc_synchronize(qoc_ctx* ctx);

/* Δt-prescaled generators A0Δt and A_jΔt (src/utils.jl:86-91), N x N each. */
int qoc_set_generators(qoc_ctx* ctx, const double* A0, const double* const* Aj);
/* x0 (N x m) shared by all seeds (per_seed = 0) or B x N x m (per_seed = 1) — propagate :14. */
int qoc_set_x0(qoc_ctx* ctx, const double* x0, int per_seed);
/* Terminal cost: kind QOC_COST_TRACE (X_target N x m, normalisation n),
 * QOC_COST_ZCAL (m must be 4; every propagation path), QOC_COST_EXTERNAL (X_target may be NULL). */
int qoc_set_cost(qoc_ctx* ctx, int kind, const double* X_target, double n);
/* Guard-state penalty L = mu sum |x[P,C]|^2 (src/penalty_fcns.jl:1-11); 0-based indices; mu = 0 disables. */
int qoc_set_state_penalty(qoc_ctx* ctx, const int* P, int np, const int* C, int nc, double mu);

/* propagate (src/gradient_computations.jl:2-32) for all B seeds, host pointers.
 * u: B x nu x Nt (see layout above).  J_out (B, may be NULL) receives the objective
 * of examples/ipopt_callbacks_exp.jl:18, Jfinal(x[end]) + sum(L, x)
 * (for QOC_COST_EXTERNAL only the penalty part). */
int qoc_propagate(qoc_ctx* ctx, const double* u, double* J_out);
/* grape_sensitivity (src/gradient_computations.jl:35-77), host pointers.
 * Returns QOC_ERR_STALE unless u is bitwise the u of the last propagate.
 * lambda_final (B x N x m) is required for QOC_COST_EXTERNAL and ignored otherwise. */
int qoc_grape_sensitivity(qoc_ctx* ctx, const double* u, int dUkdp_order,
                          const double* lambda_final, double* dJdu_out);

/* A caller's state-penalty gradient that is not a built-in penalty (any Julia closure dL_dx,
 * src/gradient_computations.jl:47-49, 55-57): dLdx holds dL_dx(x_k) for every seed and k = 0..Nt
 * (B x (Nt+1) x N x m, the states' layout), added to λ_k by the following grape_sensitivity calls until cleared
 * with NULL.  The host evaluates the closure on the states (qoc_get_states); J's sum(L, x) stays with the
 * caller.  Not on the Tsit5 path (compute_pwc_gradient has no dL_dx). */
int qoc_set_costate_source(qoc_ctx* ctx, const double* dLdx);

/* compress_states / decompress_states (src/utils.jl:96-109) inside the engine.  When the generators keep the
 * two row blocks rows1 / rows2 (a partition of the N rows) apart, and the state's columns cols1 live only on
 * rows1 and cols2 only on rows2 (a partition of the m columns), the engine packs both blocks into
 * max(nc1, nc2) columns: the chains and the gradient run on the packed states, and every host-side state
 * argument (x0, X_target, lambda_final, dLdx, penalty columns) and result (qoc_get_states / costates) keeps the
 * caller's N x m layout.  J and dJdu equal the unpacked problem's.  0-based indices; nr1 = nr2 = 0 turns packing
 * off.  Errors: QOC_ERR_ARG when the index lists do not partition rows / columns, the generators couple the blocks,
 * or x0 has an entry outside its block.  Re-packs an x0 / target / penalty already set; a co-state source must be
 * set again.  Co-states come back projected on the blocks (the rest never reaches the gradient). */
int qoc_set_compression(qoc_ctx* ctx, const int* rows1, int nr1, const int* cols1, int nc1, const int* rows2,
                        int nr2, const int* cols2, int nc2);

/* Device-pointer variants (inputs already resident in HBM, asynchronous on qoc_stream). */
int qoc_propagate_dev(qoc_ctx* ctx, const double* d_u, double* d_J);
int qoc_grape_sensitivity_dev(qoc_ctx* ctx, const double* d_u, int dUkdp_order, double* d_dJdu);
/* One GRAPE gradient eval = f + f_grad of examples/ipopt_callbacks_exp.jl:11-31 (no spline map). */
int qoc_eval_dev(qoc_ctx* ctx, const double* d_u, int dUkdp_order, double* d_J, double* d_dJdu);

/* Spline parameterisation of the controls, the optimisation variables of the Ipopt callbacks
 * (examples/ipopt_callbacks_exp.jl:13-14, 28): u_b = transpose(Bs * c_b), dJdc_b = Bs' * transpose(dJdu_b).
 * Bs is Nt x ns column-major (Julia Matrix); c_b is ns x nu column-major (reshape(c, nsplines, nu)),
 * seeds contiguous (B x ns x nu). */
int qoc_set_spline_basis(qoc_ctx* ctx, const double* Bs, int ns);
/* f + f_grad of examples/ipopt_callbacks_exp.jl:11-31 in the coefficients, device pointers. */
int qoc_eval_spline_dev(qoc_ctx* ctx, const double* d_c, int dUkdp_order, double* d_J, double* d_dJdc);
/* Host-pointer variant (J_out: B, dJdc_out: B x ns x nu). */
int qoc_eval_spline(qoc_ctx* ctx, const double* c, int dUkdp_order, double* J_out, double* dJdc_out);
/* f alone (examples/ipopt_callbacks_exp.jl:11-19: spline map, propagate, J; no sensitivity), host pointers; and
 * f_grad's sensitivity (:21-31) for the coefficients last passed to qoc_propagate_spline (QOC_ERR_STALE for any
 * other c, the reference's "Cache data from other control signal u"). */
int qoc_propagate_spline(qoc_ctx* ctx, const double* c, double* J_out);
int qoc_sensitivity_spline(qoc_ctx* ctx, const double* c, int dUkdp_order, double* dJdc_out);
/* Constraints g = [norm(c), norm(diff(c, dims=1))] and their Jacobian (examples/ipopt_callbacks_exp.jl:33-51),
 * device pointers: d_g (B x 2), d_gjac (B x 2 x nc, constraint-major = Ipopt's dense triplet order; may be NULL). */
int qoc_spline_constraints_dev(qoc_ctx* ctx, const double* d_c, double* d_g, double* d_gjac);

/* Lazy readback of cache fields (test/test_gradient_computation.jl:84,86 read cache.x / cache.λ). */
int qoc_get_states(qoc_ctx* ctx, int seed, int k, double* x_out);       /* k in [0,Nt], -1 = final */
int qoc_get_costates(qoc_ctx* ctx, int seed, int k, double* lam_out);
int qoc_get_propagator(qoc_ctx* ctx, int seed, int k, double* U_out);   /* Uk_vec[k+1], k in [0,Nt) */
/* Histogram of selected (Padé degree, squarings) since the last reset:
 * hist[di*64 + s], di = index of degree in {3,5,7,9,13}.  Used for the FLOP accounting.  Under
 * QOC_CHAIN_TAYLOR (no exponential is formed) it is evaluated at call time from the last propagated u,
 * counted once per forward pass since the reset. */
int qoc_pade_histogram(qoc_ctx* ctx, long long* hist, int reset);

/* Exponential algorithm actually executed (no linear solve; same result as the reference's Padé to
 * fp rounding; QOC_EXPM_PADE=1 at qoc_create selects the Padé + solve algorithm).  QOC_TAYLOR_HIST_ENTRIES = 9*64 entries:
 *   hist[(r-2)*64 + s], r = 2..8: degree m = 3r+2 Taylor by Paterson-Stockmeyer (2 + r GEMMs) with s
 *     squarings (large-N pipeline; LDS kernel with QOC_EXPM_LDS=1);
 *   hist[7*64 + s]: degree-12 Taylor in 4 GEMMs (Bader-Blanes-Casas form) with s squarings (the
 *     default register-resident kernel);
 *   hist[8*64 + s]: degree-8 Taylor in 3 GEMMs (Bader-Blanes-Casas form) with s squarings (large-N pipeline).
 * The truncation tail is <= 2^-53 in every case.  qoc_pade_histogram keeps reporting the Padé (d, s)
 * the reference would select.  qoc_taylor_histogram_n takes the capacity of hist and fails (QOC_ERR_ARG) when it
 * is below QOC_TAYLOR_HIST_ENTRIES; qoc_taylor_histogram (no capacity) writes QOC_TAYLOR_HIST_ENTRIES entries. */
#define QOC_TAYLOR_HIST_ENTRIES (9 * 64)
int qoc_taylor_histogram(qoc_ctx* ctx, long long* hist /*[QOC_TAYLOR_HIST_ENTRIES]*/, int reset);
int qoc_taylor_histogram_n(qoc_ctx* ctx, long long* hist, int n, int reset);

/* Live per-kernel timing: when enabled, hipEvents are recorded on qoc_stream around each hot-path
 * kernel (phase 0 k_expm, 1 k_chain_fwd, 2 k_chain_bwd, 3 k_grad).  qoc_phase_times synchronises the
 * stream and returns the accumulated milliseconds and launch counts per phase. */
int qoc_set_profiling(qoc_ctx* ctx, int enable);
int qoc_phase_times(qoc_ctx* ctx, double* ms_out /*[4]*/, long long* launches_out /*[4]*/, int reset);

/* Large-N path only: accumulated time, launch count and algorithmic FLOPs (8 M K Ncol per complex
 * GEMM item) of the k_bgemm launches recorded while profiling was enabled. */
int qoc_gemm_stats(qoc_ctx* ctx, double* ms, long long* launches, double* flops, int reset);

/* Propagation method.  QOC_PROP_EXPM (default): U_k = exp(A_k) per slice.
 * QOC_PROP_TSIT5: the reference's ODE path propagate_pwc / compute_pwc_gradient
 * (src/gradient_computations.jl:108-169): nsub fixed Tsit5 steps per slice (the reference's
 * dt = 0.1 Δt is nsub = 10) for the states and, backwards, for the co-states dλ/dτ = -A_k^H λ; the
 * gradient contraction is unchanged.  LDS-resident sizes (N <= 64), trace / external costs. */
#define QOC_PROP_EXPM 0
#define QOC_PROP_TSIT5 1
int qoc_set_propagation(qoc_ctx* ctx, int method, int nsub);

/* Continuous-envelope propagation with fixed-step Tsit5 (wrap_envelope, src/QuantumOptimalControl.jl:43-54;
 * examples/two_qubit_tunable_bus.jl:58-67): dx/dt = (A0 + sum_j c_j(t) A_j) x, t in [0, tgate], step dt,
 * with c(t) from the pulse `kind` and per-seed parameters params[b*np ...] (src/parameterized_pulses.jl).
 * The generators are used as set (not Δt-scaled).  x_out (optional, B x N x m interleaved complex,
 * column-major per seed) receives x(tgate); J_out (optional, B) the trace cost when one is set.  QOC_ENV_TUNABLE_BUS: [t_plateau, t_rise_fall, theta0, omega_Phi, A], nu = 1;
 * QOC_ENV_DRAG (u_drag): [tgate, sigma, A, xi], nu = 2 (Re, Im); QOC_ENV_SINEBASIS: [Tgate, p1x, p1y, ...], nu = 2. */
#define QOC_ENV_TUNABLE_BUS 0
#define QOC_ENV_DRAG 1
#define QOC_ENV_SINEBASIS 2
int qoc_propagate_envelope(qoc_ctx* ctx, int kind, const double* params, int np, double tgate, double dt,
                           double* J_out, double* x_out);

/* Engine facts: info[0] = path (0 = LDS-resident kernels, 1 = large-N chunked GEMM pipeline),
 * info[1] = slices per chunk (large-N), info[2] = Newton-Schulz iterations executed so far (large-N),
 * info[3] = device bytes allocated by the context, info[4] = chain mode (QOC_CHAIN_PROPAGATORS /
 * QOC_CHAIN_TAYLOR), info[5] = exponential the propagators run (0 the reference's Padé + solve, 1 register-
 * resident Taylor / Paterson-Stockmeyer, 2 LDS Paterson-Stockmeyer), info[6] = 1 when the Taylor-action chains
 * use Chebyshev terms (skew-Hermitian generators, fp64; QOC_TCHAIN_POLY=taylor keeps Taylor), info[7] = state columns the kernels run on (m, or max(nc1, nc2) with qoc_set_compression), info[8] = how the
 * last backward ran (0 generic, 1 from the chains' captured products, 2 concurrent μ recurrence of qoc_eval_dev on
 * a second stream, 3 the same in one launch with the forward chain, 4 the block chains' concurrent eval, 5 the block
 * propagators' fused backward: λ kept on chip, the gradient contracted beside the chain; qoc_get_costates then
 * rebuilds λ on demand),
 * info[9] = 1 when the last forward chain wrote its captured products, info[10] = the Taylor-action chain kernels
 * (0 none / the fp32 VALU ones, 1 MFMA with the state in LDS, 2 MFMA with the state in registers: N <= 32, nu <= 2,
 * QOC_TCHAIN_ROT=0 keeps 1; 3 block chains: the generators split into invariant blocks of <= 4 rows, one VALU lane
 * per (block, column); 4 block chains with one MFMA wave per (block of 5..16 rows, column pair), or blocks of <= 4 rows
 * packed into MFMA slots (QOC_BLKU=0); 5 block propagators: blocks of <= 4 rows, U_k formed per (slice, block) apart
 * from the serial chain, one block matvec per slice (the default for blocks of <= 4 rows); QOC_BLOCKS=0 at
 * qoc_set_generators keeps the dense kernels).  QOC_FORCE_LARGE_N=1 in the environment at qoc_create selects the
 * large-N path for any size (testing).  qoc_get_info_n takes the capacity of info and fails (QOC_ERR_ARG) when it is
 * below QOC_INFO_ENTRIES; qoc_get_info (no capacity) writes QOC_INFO_ENTRIES entries.  info[11] = what the last
 * propagate left for grape_sensitivity (the reference's split call form, examples/ipopt_callbacks_exp.jl:11-31):
 * 0 the states x_k, 1 the segmented forward (blocks of 2-3 rows: G at every segment's end, x_k rebuilt on demand;
 * grape_sensitivity then runs the segmented backward alone), 2 the stored propagators of blocks of 5..16 rows
 * (grape_sensitivity: the co-state chain and the gradient on them).  info[12] = the degree of the last stored-propagator
 * formation's interpolation in u (one control: U(u) = Σ_i T_i(ξ) M_i over the batch's control range), 0 when the
 * exponentials were formed per slice.  info[13] = 1 when the last eval / propagate on blocks of 5..16 rows ran the
 * interpolating chains (each chain forms its slice propagators from those coefficients in registers: none stored),
 * 2 when they formed the upper triangle alone (complex-symmetric generators), 0 otherwise. */
#define QOC_INFO_ENTRIES 14
int qoc_get_info(qoc_ctx* ctx, long long* info /*[QOC_INFO_ENTRIES]*/);
int qoc_get_info_n(qoc_ctx* ctx, long long* info, int n);

/* How the chains x_{k+1} = U_k x_k (src/gradient_computations.jl:27-29) and λ_k = U_k^H λ_{k+1} (:52-58)
 * apply the slice exponentials:
 *   QOC_CHAIN_PROPAGATORS: form every U_k = exp(A_k) (register-resident Taylor / Padé on MFMA, the
 *     reference's structure), then the serial products;
 *   QOC_CHAIN_TAYLOR: apply exp(A_k) to the N x m state directly (shifted, truncated Taylor series with the
 *     degree chosen per slice for a tail <= 2^-53 / 2^-24) — no U_k is formed (qoc_get_propagator computes
 *     one on demand).  N <= 48 (fp64) / 64 (fp32), nu <= 8;
 *   QOC_CHAIN_AUTO: Taylor when ||A0 - μ I||_1 <= 1 (few terms per slice), else propagators (the default,
 *     chosen at qoc_set_generators; QOC_CHAIN=taylor|expm in the environment overrides it).
 * The states, co-states, J and dJdu agree to rounding either way. */
#define QOC_CHAIN_AUTO (-1)
#define QOC_CHAIN_PROPAGATORS 0
#define QOC_CHAIN_TAYLOR 1
int qoc_set_chain(qoc_ctx* ctx, int mode);
/* Taylor terms executed per direction (Σ over slices of P s) since the last reset (QOC_CHAIN_TAYLOR). */
int qoc_chain_terms(qoc_ctx* ctx, long long* terms, int reset);

/* Multi-GPU epilogue: seeds are sharded contiguously over ranks, one context per GPU; the
 * only exchange is an all-gather of each rank's best (J, global seed id) over RCCL (xGMI), 16 bytes per rank.
 * qoc_comm_unique_id (one rank) creates the RCCL unique id (QOC_UNIQUE_ID_BYTES opaque bytes) that the caller
 * distributes (MPI / Distributed.jl / torch.distributed); every rank then calls qoc_comm_init with its rank
 * and the global id of its seed 0.  qoc_allgather_best returns the best J of the last propagate over all
 * ranks and its global seed (lowest seed on ties); without qoc_comm_init it covers this context alone.
 * With an id, qoc_comm_init creates a real RCCL communicator for any world size (world = 1 included: a
 * one-rank ncclAllGather on the same path as the multi-GPU run); with id = NULL (world = 1 only) none is made.
 * On any error the context is left without a communicator (world 1, seed offset 0).
 * qoc_comm_ranks returns the communicator's rank count, 0 when the context has none.
 * RCCL is loaded on first use (librccl.so.1); two ranks cannot share one GPU (RCCL rejects duplicate
 * devices).  The _dev variant writes (J_best, seed) as two doubles to device memory on qoc_stream without
 * synchronising. */
#define QOC_UNIQUE_ID_BYTES 128
int qoc_comm_unique_id(void* id_out);
int qoc_comm_init(qoc_ctx* ctx, int world, int rank, const void* id, long long seed_offset);
int qoc_comm_ranks(qoc_ctx* ctx);
int qoc_allgather_best(qoc_ctx* ctx, double* J_best, int* seed_best);
int qoc_allgather_best_dev(qoc_ctx* ctx, double* d_out);
/* Registers a device buffer of two doubles (NULL: none).  With nothing to exchange (no communicator, or one rank) the
 * evals that reduce their own J (the segmented block eval) then also write the best (J, seed) there, and
 * qoc_allgather_best_dev(ctx, that buffer) queues nothing more: the result is the same pair, without the pick kernel
 * after every eval.  The caller keeps the buffer valid while it is registered. */
int qoc_set_best_output(qoc_ctx* ctx, double* d_out);

/* Standalone ops on the same kernels. */
/* exponential!(A, ExpMethodHigham2005()) for `count` independent N x N matrices
 * (src/gradient_computations.jl:24, third-party ExponentialUtilities). */
int qoc_expm_batched(int device, int N, int count, int precision, const double* A, double* X,
                     int* degree_out, int* squarings_out);
/* expm_jacobian! (src/gradient_computations.jl:177-213): dFdp_j for F = exp(dt(A0 + sum p_j A_j)),
 * truncated Taylor order 1..4; dFdp_out is nu x (N x N). */
int qoc_expm_jacobian(int device, int N, int nu, const double* A0, const double* const* Aj,
                      const double* p, int order, double dt, double* dFdp_out);

#ifdef __cplusplus
}
#endif
#endif /* QOC_MI355X_H */
