// qoc_run.hip — run_forward / run_backward: per path (propagators, Taylor action, Tsit5, large N) the launches of
// one propagate and one grape_sensitivity; the propagator chains (k_chain_fwd / k_chain_bwd) and the per-slice
// gradient k_grad live here.
#include "qoc_internal.hpp"

namespace qoc_host {

size_t chain_lds(const qoc_ctx* c) {
  const ChainShape sh = chain_shape(c->N, c->m, c->prec == QOC_FP64);
  // sized for the largest column block either direction may use (chain_dispatch's override: 2 at JT >= 10)
  const int cb = sh.JT >= 10 ? 2 : sh.CB;
  return (size_t)(2 * sh.S * sh.JT * chain_mpad(c->m, cb)) * c->esz + 64 * sizeof(double);
}

// k_chain_fwd / k_chain_bwd instantiated per thread shape (chain_shape): (S, JT, CB) = (4, 4, 1|4),
// (8, 4, 1|4), (4, 10, 1|2), (4, 12, 1|2), fp32 also (4, 16, 1|2).
template <typename T, typename F>
hipError_t chain_dispatch(int N, int m, int cb_override, F&& f) {
  using std::integral_constant;
  ChainShape sh = chain_shape(N, m, sizeof(T) == 8);
  if (cb_override > 0 && sh.JT >= 10) sh.CB = cb_override == 2 ? 2 : 1;  // tuning knob (QOC_CHAIN_CB_*)
  if (sh.JT == 4) {
    if (sh.S == 4)
      return sh.CB == 4 ? f(integral_constant<int, 4>(), integral_constant<int, 4>(), integral_constant<int, 4>())
                        : f(integral_constant<int, 4>(), integral_constant<int, 4>(), integral_constant<int, 1>());
    return sh.CB == 4 ? f(integral_constant<int, 8>(), integral_constant<int, 4>(), integral_constant<int, 4>())
                      : f(integral_constant<int, 8>(), integral_constant<int, 4>(), integral_constant<int, 1>());
  }
  if (sh.JT == 10)
    return sh.CB == 2 ? f(integral_constant<int, 4>(), integral_constant<int, 10>(), integral_constant<int, 2>())
                      : f(integral_constant<int, 4>(), integral_constant<int, 10>(), integral_constant<int, 1>());
  if (sh.JT == 12)
    return sh.CB == 2 ? f(integral_constant<int, 4>(), integral_constant<int, 12>(), integral_constant<int, 2>())
                      : f(integral_constant<int, 4>(), integral_constant<int, 12>(), integral_constant<int, 1>());
  if constexpr (sizeof(T) == 4) {
    if (sh.JT == 16)
      return sh.CB == 2 ? f(integral_constant<int, 4>(), integral_constant<int, 16>(), integral_constant<int, 2>())
                        : f(integral_constant<int, 4>(), integral_constant<int, 16>(), integral_constant<int, 1>());
  }
  return hipErrorInvalidValue;
}

size_t grad_lds(const qoc_ctx* c, int order) {
  return (size_t)(c->N * (c->N + 1) + 2 * order * c->N * c->m) * c->esz + 64 * sizeof(double);
}

template <typename T>
int run_forward(qoc_ctx* c) {
  if (c->prop_method == QOC_PROP_TSIT5) return ode_forward<T>(c);
  if (c->chain_mode == 1) return tchain_forward<T>(c);
  int mk = mark_begin(c, 0);
  hipError_t e = launch_expm(c->prec, c->stream, c->N, c->nu, c->B * c->Nt, c->d_A, c->d_u, nullptr, c->d_U,
                             c->d_hist, nullptr, nullptr, c->expm_run, c->d_hist + 5 * 64, c->d_ps,
                             c->a0norm > 4.0 * kTheta12);
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_expm launch: %s", hipGetErrorString(e));
  const size_t lds = chain_lds(c);
  mk = mark_begin(c, 1);
  e = chain_dispatch<T>(c->N, c->m, c->chain_cb_fwd, [&](auto S_, auto JT_, auto CB_) {
    constexpr int S = decltype(S_)::value, JT = decltype(JT_)::value, CB = decltype(CB_)::value;
    hipError_t r = hipFuncSetAttribute((const void*)k_chain_fwd<T, S, JT, CB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL((k_chain_fwd<T, S, JT, CB>), dim3(c->B), dim3(CHAIN_THREADS), lds, c->stream, c->N, c->m, c->Nt,
                       (const cx<T>*)c->d_U, (const cx<T>*)c->d_x0, c->x0_per_seed, (cx<T>*)c->d_X,
                       (const cx<T>*)c->d_Xt, c->cost_kind, c->cost_n, c->mu != 0.0 ? c->d_pmask : nullptr, c->mu,
                       c->d_J, c->d_coef, sectors(c));
    return hipGetLastError();
  });
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_chain_fwd launch: %s", hipGetErrorString(e));
  return QOC_OK;
}

template <typename T>
int run_backward(qoc_ctx* c, int order, double* d_dJdu) {
  size_t lds = chain_lds(c);
  int mk;
  if (c->prop_method == QOC_PROP_TSIT5) {
    int r = ode_adjoint<T>(c);
    if (r) return r;
  } else if (c->chain_mode == 1) {
    if (order == 3 && c->grad_rr && c->fwd_captured) return tchain_backward_captured<T>(c, d_dJdu);
    if (order == 3 && c->grad_rr && c->bwd_chunks > 1 && c->Nt >= 64 && tchain_mf(c)) return tchain_backward_overlapped<T>(c, d_dJdu);
    int r = tchain_backward<T>(c);
    if (r) return r;
  } else {
    mk = mark_begin(c, 2);
    const hipError_t e = chain_dispatch<T>(c->N, c->m, c->chain_cb_bwd, [&](auto S_, auto JT_, auto CB_) {
      constexpr int S = decltype(S_)::value, JT = decltype(JT_)::value, CB = decltype(CB_)::value;
      hipError_t r = hipFuncSetAttribute((const void*)k_chain_bwd<T, S, JT, CB>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (r != hipSuccess) return r;
      hipLaunchKernelGGL((k_chain_bwd<T, S, JT, CB>), dim3(c->B), dim3(CHAIN_THREADS), lds, c->stream, c->N, c->m, c->Nt,
                         (const cx<T>*)c->d_U, (const cx<T>*)c->d_X, (cx<T>*)c->d_L, (const cx<T>*)c->d_Xt,
                         c->cost_kind, (const cx<double>*)c->d_coef, c->mu != 0.0 ? c->d_pmask : nullptr, c->mu,
                         c->src_on ? (const cx<T>*)c->d_src : nullptr, sectors(c));
      return hipGetLastError();
    });
    mark_end(c, mk);
    if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_chain_bwd launch: %s", hipGetErrorString(e));
  }
  return dense_gradient<T>(c, order, d_dJdu);
}

// the gradient from the stored x_k and λ_k (every chain kind): the exact Fréchet kernel, the fused order-3
// kernels, the GEMM-shaped order-3 path or the per-slice k_grad
template <typename T>
int dense_gradient(qoc_ctx* c, int order, double* d_dJdu) {
  int mk;
  size_t lds;
  if (order == QOC_DUKDP_EXACT) {
    mk = mark_begin(c, 3);
    int r = frechet_grad<T>(c, d_dJdu);
    mark_end(c, mk);
    return r;
  }
  if (order == 3 && c->grad_rr) {
    mk = mark_begin(c, 3);
    int r = grad_rr_o3<T>(c, d_dJdu, c->stream, 0, c->Nt);
    mark_end(c, mk);
    return r;
  }
  if (order == 3 && c->grad_gemm) {
    mk = mark_begin(c, 3);
    int r = grad_gemm_o3<T>(c, d_dJdu);
    mark_end(c, mk);
    return r;
  }
  lds = grad_lds(c, order);
  HIPCHK(c, hipFuncSetAttribute((const void*)k_grad<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  mk = mark_begin(c, 3);
  hipLaunchKernelGGL((k_grad<T>), dim3(c->B * c->Nt), dim3(GRAD_THREADS), lds, c->stream, c->N, c->m, c->nu, c->Nt,
                     order, (const cx<T>*)c->d_A, c->d_u, (const cx<T>*)c->d_X, (const cx<T>*)c->d_L, d_dJdu);
  mark_end(c, mk);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}

template int run_forward<double>(qoc_ctx*);
template int run_forward<float>(qoc_ctx*);
template int run_backward<double>(qoc_ctx*, int, double*);
template int run_backward<float>(qoc_ctx*, int, double*);
template int dense_gradient<double>(qoc_ctx*, int, double*);
template int dense_gradient<float>(qoc_ctx*, int, double*);

}  // namespace qoc_host
