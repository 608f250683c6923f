// qoc_run_ode.hip — the fixed-step Tsit5 path (qoc_ode.hpp: k_ode_pwc, k_ode_envelope) and the terminal-cost
// kernel of the paths without a fused forward epilogue.
#include "qoc_bgemm.hpp"
#include "qoc_internal.hpp"
#include "qoc_ode.hpp"

namespace qoc_host {

// ---- ODE path (fixed-step Tsit5, qoc_ode.hpp) ------------------------------------------------
// k_ode_pwc instantiation by N: register-resident rows up to 48 (fp64) / 64 (fp32), LDS beyond
template <typename T>
void launch_ode_pwc(qoc_ctx* c, int adjoint, cx<T>* S, const unsigned char* pmask, double two_mu) {
  const int N = c->N, W = std::min(c->m, 4);
  const size_t lds = (((size_t)N * N * c->esz + 15) & ~(size_t)15) + (size_t)W * 64 * c->esz;
  auto go = [&](auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(c->B), dim3(64 * W), lds, c->stream, N, c->m, c->nu, c->Nt, c->nsub, adjoint,
                       (const cx<T>*)c->d_A, (const double*)c->d_u, (const cx<T>*)c->d_x0, c->x0_per_seed, S,
                       (const cx<T>*)c->d_X, pmask, two_mu);
  };
  if (c->ode_kernel == 1) go(k_ode_pwc<T, 0>);
  else if (N <= 16) go(k_ode_pwc<T, 16>);
  else if (N <= 32) go(k_ode_pwc<T, 32>);
  else if (N <= 48) go(k_ode_pwc<T, 48>);
  else if (sizeof(T) == 4) go(k_ode_pwc<T, 64>);
  else go(k_ode_pwc<T, 0>);
}

template <typename T>
int ode_forward(qoc_ctx* c) {
  int mk = mark_begin(c, 1);
  launch_ode_pwc<T>(c, 0, (cx<T>*)c->d_X, nullptr, 0.0);
  HIPCHK(c, hipGetLastError());
  const bool pen = c->mu != 0.0;
  if (pen) {
    hipLaunchKernelGGL((k_penalty_sum<T>), dim3(c->B), dim3(256), 0, c->stream, c->N, c->m, c->Nt,
                       (const cx<T>*)c->d_X, c->d_pmask, c->mu, c->d_J);
    HIPCHK(c, hipGetLastError());
  }
  if (c->cost_kind != QOC_COST_EXTERNAL) {
    hipLaunchKernelGGL((k_terminal_cost<T>), dim3(c->B), dim3(256), 0, c->stream, c->N, c->m, c->Nt,
                       (const cx<T>*)c->d_X, (const cx<T>*)c->d_Xt, c->cost_kind, c->cost_n, pen ? 1 : 0, c->d_J,
                       c->d_coef, sectors(c));
    HIPCHK(c, hipGetLastError());
  } else if (!pen) {
    HIPCHK(c, hipMemsetAsync(c->d_J, 0, (size_t)c->B * sizeof(double), c->stream));
  }
  mark_end(c, mk);
  return QOC_OK;
}

template <typename T>
int ode_adjoint(qoc_ctx* c) {
  const int N = c->N, m = c->m, Nt = c->Nt, B = c->B;
  const size_t Nm = (size_t)N * m;
  const bool pen = c->mu != 0.0;
  const unsigned eb = (unsigned)std::min<size_t>((Nm * B + 255) / 256, 8192);
  int mk = mark_begin(c, 2);
  if (c->cost_kind != QOC_COST_EXTERNAL) {
    hipLaunchKernelGGL((k_lambda_final<T>), dim3(eb), dim3(256), 0, c->stream, N, m, Nt, B, (const cx<T>*)c->d_Xt,
                       (const cx<double>*)c->d_coef, (cx<T>*)c->d_L, sectors(c));
    HIPCHK(c, hipGetLastError());
  }
  if (pen) {
    hipLaunchKernelGGL((k_penalty_grad<T>), dim3(eb), dim3(256), 0, c->stream, N, m, Nt, B, Nt,
                       (const cx<T>*)c->d_X, c->d_pmask, 2.0 * c->mu, (cx<T>*)c->d_L);
    HIPCHK(c, hipGetLastError());
  }
  launch_ode_pwc<T>(c, 1, (cx<T>*)c->d_L, pen ? c->d_pmask : nullptr, 2.0 * c->mu);
  HIPCHK(c, hipGetLastError());
  mark_end(c, mk);
  return QOC_OK;
}

hipError_t launch_envelope(qoc_ctx* c, int kind, const double* dP, int np, double dt, long long nsteps) {
  const size_t lds = (size_t)(c->nu + 1) * c->N * c->N * c->esz;
  const int W = std::min(c->m, 4);
  hipError_t e;
  if (c->prec == QOC_FP64) {
    e = hipFuncSetAttribute((const void*)k_ode_envelope<double>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_ode_envelope<double>), dim3(c->B), dim3(64 * W), lds, c->stream, c->N, c->m, c->nu, c->Nt,
                       kind, dP, np, dt, nsteps, (const cx<double>*)c->d_A, (const cx<double>*)c->d_x0,
                       c->x0_per_seed, (cx<double>*)c->d_X);
  } else {
    e = hipFuncSetAttribute((const void*)k_ode_envelope<float>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_ode_envelope<float>), dim3(c->B), dim3(64 * W), lds, c->stream, c->N, c->m, c->nu, c->Nt,
                       kind, dP, np, dt, nsteps, (const cx<float>*)c->d_A, (const cx<float>*)c->d_x0,
                       c->x0_per_seed, (cx<float>*)c->d_X);
  }
  return hipGetLastError();
}

// J and the λ_N coefficients of the stored x_N (no state penalty)
hipError_t launch_terminal_cost(qoc_ctx* c) {
  if (c->prec == QOC_FP64)
    hipLaunchKernelGGL((k_terminal_cost<double>), dim3(c->B), dim3(256), 0, c->stream, c->N, c->m, c->Nt,
                       (const cx<double>*)c->d_X, (const cx<double>*)c->d_Xt, c->cost_kind, c->cost_n, 0, c->d_J,
                       c->d_coef, sectors(c));
  else
    hipLaunchKernelGGL((k_terminal_cost<float>), dim3(c->B), dim3(256), 0, c->stream, c->N, c->m, c->Nt,
                       (const cx<float>*)c->d_X, (const cx<float>*)c->d_Xt, c->cost_kind, c->cost_n, 0, c->d_J,
                       c->d_coef, sectors(c));
  return hipGetLastError();
}

template int ode_forward<double>(qoc_ctx*);
template int ode_forward<float>(qoc_ctx*);
template int ode_adjoint<double>(qoc_ctx*);
template int ode_adjoint<float>(qoc_ctx*);

}  // namespace qoc_host
