// qoc_run_grad.hip — launches of the fused order-3 gradient (qoc_grad_rr.hpp: k_grad_rr_q / _p / _s).
#include "qoc_grad_rr.hpp"
#include "qoc_internal.hpp"

namespace qoc_host {

// Fused order-3 gradient (qoc_grad_rr.hpp): k_grad_rr_q (co-state side -> W0, W1 in the state layout)
// then k_grad_rr_p (state side + contraction -> dJdu).  Persistent grids of 4-wave workgroups.
template <typename T, int NT, int KS, int NU>
int grad_rr_launch(qoc_ctx* c, double* d_dJdu, hipStream_t st, int k0, int nk, int mode) {
  using G = GradRR<T, NT>;
  const int N = c->N, m = c->m, Nt = c->Nt, B = c->B;
  const size_t lds = G::lds_bytes(N, NU);
  const long long units = (long long)B * nk, ntiles = (units + 16 / m - 1) / (16 / m);
  const int per_cu = lds <= 80 * 1024 ? 2 : 1;
  const int grid = (int)std::max<long long>(1, std::min<long long>((ntiles + 3) / 4, (long long)c->ncu * per_cu));
  const size_t bufN = (size_t)N * ((size_t)B * (Nt + 1) * m);
  cx<T>* W0 = (cx<T>*)c->d_gws;
  cx<T>* W1 = W0 + bufN;
  // mode 0: q + p;  1: state side only (k_grad_rr_s -> P1, P2 in d_pws);  2: q + p reading P1, P2
  cx<T>* P1 = (cx<T>*)c->d_pws;
  cx<T>* P2 = P1 ? P1 + bufN : nullptr;
  if (mode == 1) {
    HIPCHK(c, hipFuncSetAttribute((const void*)k_grad_rr_s<T, NT, KS, NU>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_grad_rr_s<T, NT, KS, NU>), dim3(grid), dim3(256), lds, st, N, m, Nt, B, k0, nk,
                       (const cx<T>*)c->d_A, c->d_u, (const cx<T>*)c->d_X, P1, P2);
    HIPCHK(c, hipGetLastError());
    return QOC_OK;
  }
  HIPCHK(c, hipFuncSetAttribute((const void*)k_grad_rr_q<T, NT, KS, NU>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((k_grad_rr_q<T, NT, KS, NU>), dim3(grid), dim3(256), lds, st, N, m, Nt, B, k0, nk,
                     (const cx<T>*)c->d_A, c->d_u, (const cx<T>*)c->d_L, W0, W1);
  HIPCHK(c, hipGetLastError());
  if (mode == 2) {
    HIPCHK(c, hipFuncSetAttribute((const void*)k_grad_rr_p<T, NT, KS, NU, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_grad_rr_p<T, NT, KS, NU, true>), dim3(grid), dim3(256), lds, st, N, m, Nt, B, k0, nk,
                       (const cx<T>*)c->d_A, c->d_u, (const cx<T>*)c->d_X, (const cx<T>*)c->d_L, (const cx<T>*)W0,
                       (const cx<T>*)W1, d_dJdu, (const cx<T>*)P1, (const cx<T>*)P2);
  } else {
    HIPCHK(c, hipFuncSetAttribute((const void*)k_grad_rr_p<T, NT, KS, NU>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_grad_rr_p<T, NT, KS, NU>), dim3(grid), dim3(256), lds, st, N, m, Nt, B, k0, nk,
                       (const cx<T>*)c->d_A, c->d_u, (const cx<T>*)c->d_X, (const cx<T>*)c->d_L, (const cx<T>*)W0,
                       (const cx<T>*)W1, d_dJdu);
  }
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}

template <typename T, int NT, int NU>
int grad_rr_nt(qoc_ctx* c, double* d_dJdu, hipStream_t st, int k0, int nk, int mode) {
  const int ks = sizeof(T) == 8 ? (c->N + 3) / 4 : 4 * NT;
  if constexpr (sizeof(T) == 8) {
    if (ks == 4 * NT - 3) return grad_rr_launch<T, NT, 4 * NT - 3, NU>(c, d_dJdu, st, k0, nk, mode);
    if (ks == 4 * NT - 2) return grad_rr_launch<T, NT, 4 * NT - 2, NU>(c, d_dJdu, st, k0, nk, mode);
    if (ks == 4 * NT - 1) return grad_rr_launch<T, NT, 4 * NT - 1, NU>(c, d_dJdu, st, k0, nk, mode);
  }
  return grad_rr_launch<T, NT, 4 * NT, NU>(c, d_dJdu, st, k0, nk, mode);
}

template <typename T>
int grad_rr_o3(qoc_ctx* c, double* d_dJdu, hipStream_t st, int k0, int nk, int mode) {
  const int NT = (c->N + 15) / 16;
  if (c->nu == 1) {
    if (NT == 1) return grad_rr_nt<T, 1, 1>(c, d_dJdu, st, k0, nk, mode);
    if (NT == 2) return grad_rr_nt<T, 2, 1>(c, d_dJdu, st, k0, nk, mode);
    return grad_rr_nt<T, 3, 1>(c, d_dJdu, st, k0, nk, mode);
  }
  if (NT == 1) return grad_rr_nt<T, 1, 2>(c, d_dJdu, st, k0, nk, mode);
  if (NT == 2) return grad_rr_nt<T, 2, 2>(c, d_dJdu, st, k0, nk, mode);
  return grad_rr_nt<T, 3, 2>(c, d_dJdu, st, k0, nk, mode);
}

// k_grad_rr_c over the units of slices [k0, k0 + nk) (fp64: the captures come from the MFMA chains)
template <int NT, int KS, int NU>
int grad_cap_launch(qoc_ctx* c, double* d_dJdu, hipStream_t st, int k0, int nk, bool mu_mode) {
  using G = GradRR<double, NT>;
  const int N = c->N, m = c->m, Nt = c->Nt, B = c->B;
  const size_t lds = G::lds_bytes(N, NU);
  const long long units = (long long)B * nk, ntiles = (units + 16 / m - 1) / (16 / m);
  // as many resident workgroups as the kernel's registers and LDS allow (N <= 16: 3 per CU; the loads of a tile
  // are waited for before its contractions, so resident waves are the memory-level parallelism)
  HIPCHK(c, hipFuncSetAttribute((const void*)k_grad_rr_c<NT, KS, NU>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  static int occ = 0;  // per instantiation (lds depends on N, fixed by the instantiation up to 3 rows)
  int per_cu = occ;
  if (per_cu < 1) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_grad_rr_c<NT, KS, NU>, 256, lds) !=
            hipSuccess ||
        per_cu < 1)
      per_cu = lds <= 80 * 1024 ? 2 : 1;
    occ = per_cu;
  }
  const int grid = (int)std::max<long long>(1, std::min<long long>((ntiles + 3) / 4, (long long)c->ncu * per_cu));
  const size_t bufN = (size_t)N * ((size_t)B * (Nt + 1) * m);
  GradCapArgs a{};
  a.N = N;
  a.m = m;
  a.Nt = Nt;
  a.B = B;
  a.k0 = k0;
  a.nk = nk;
  a.Agen = c->d_A;
  a.u = c->d_u;
  a.X = c->d_X;
  a.L = c->d_L;
  a.F1 = c->d_pws;
  a.F2 = (const cx<double>*)c->d_pws + bufN;
  a.G1 = c->d_gws;
  a.G2 = (const cx<double>*)c->d_gws + bufN;
  a.steps = (const double*)c->d_steps;
  for (int j = 0; j < 3; ++j) {
    a.mur[j] = j <= c->nu ? c->tprm.mur[j] : 0.0;
    a.mui[j] = j <= c->nu ? c->tprm.mui[j] : 0.0;
  }
  a.kappa = c->cheb_ran ? 2.0 : 1.0;
  a.coef = mu_mode ? c->d_coef : nullptr;
  a.rsec_mask = 0;
  if (c->packed)
    for (int r = 0; r < N && r < 64; ++r) a.rsec_mask |= (unsigned long long)(c->h_rsec[r] & 1) << r;
  a.dJdu = d_dJdu;
  hipLaunchKernelGGL((k_grad_rr_c<NT, KS, NU>), dim3(grid), dim3(256), lds, st, a);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}

template <int NT, int NU>
int grad_cap_nt(qoc_ctx* c, double* d_dJdu, hipStream_t st, int k0, int nk, bool mu_mode) {
  const int ks = (c->N + 3) / 4;
  if (ks == 4 * NT - 3) return grad_cap_launch<NT, 4 * NT - 3, NU>(c, d_dJdu, st, k0, nk, mu_mode);
  if (ks == 4 * NT - 2) return grad_cap_launch<NT, 4 * NT - 2, NU>(c, d_dJdu, st, k0, nk, mu_mode);
  if (ks == 4 * NT - 1) return grad_cap_launch<NT, 4 * NT - 1, NU>(c, d_dJdu, st, k0, nk, mu_mode);
  return grad_cap_launch<NT, 4 * NT, NU>(c, d_dJdu, st, k0, nk, mu_mode);
}

int grad_rr_cap(qoc_ctx* c, double* d_dJdu, hipStream_t st, int k0, int nk, bool mu_mode) {
  if (c->prec != QOC_FP64 || !c->d_pws || !c->d_gws) return fail(c, QOC_ERR_STATE, "captured gradient: no captures");
  const int NT = (c->N + 15) / 16;
  if (c->nu == 1) {
    if (NT == 1) return grad_cap_nt<1, 1>(c, d_dJdu, st, k0, nk, mu_mode);
    if (NT == 2) return grad_cap_nt<2, 1>(c, d_dJdu, st, k0, nk, mu_mode);
    return grad_cap_nt<3, 1>(c, d_dJdu, st, k0, nk, mu_mode);
  }
  if (NT == 1) return grad_cap_nt<1, 2>(c, d_dJdu, st, k0, nk, mu_mode);
  if (NT == 2) return grad_cap_nt<2, 2>(c, d_dJdu, st, k0, nk, mu_mode);
  return grad_cap_nt<3, 2>(c, d_dJdu, st, k0, nk, mu_mode);
}

template int grad_rr_o3<double>(qoc_ctx*, double*, hipStream_t, int, int, int);
template int grad_rr_o3<float>(qoc_ctx*, double*, hipStream_t, int, int, int);

}  // namespace qoc_host
