// Per-term cycle breakdown of the Taylor-action forward chain (diagnostic; built with -DQOC_PROBE).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DQOC_PROBE -o tools/tchain_probe tools/tchain_probe.hip
// g_tc[0] = matvec (LDS reads + FMAs + part sums), g_tc[1] = matvec + z store issue, g_tc[2] = barrier,
// g_tc[3] = terms (block 7, thread 0).
#include <cstdio>
#include <vector>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_tchain.hpp"
using namespace qoc;

template <int S, int JT, int CB, int NP>
void run(int N, int m, int Nt, int B, int P) {
  const int nu = 2;
  const size_t NN = (size_t)N * N;
  std::vector<cx<double>> A((nu + 1) * NN);
  for (size_t e = 0; e < A.size(); ++e) A[e] = {((e * 7919) % 97) / (97.0 * N) - 0.5 / N, ((e * 104729) % 89) / (89.0 * N) - 0.5 / N};
  std::vector<double> u((size_t)B * Nt * nu, 0.01);
  std::vector<TStep> st((size_t)B * Nt, TStep{1.0, 0.0, P, 1, 1.0});
  std::vector<cx<double>> x0((size_t)N * m, cx<double>{1.0 / N, 0});
  cx<double>*dA, *dx0, *dX, *dcoef;
  double *dJ, *du;
  TStep* dst;
  (void)hipMalloc(&dA, A.size() * 16);
  (void)hipMalloc(&du, u.size() * 8);
  (void)hipMalloc(&dst, st.size() * sizeof(TStep));
  (void)hipMalloc(&dx0, x0.size() * 16);
  (void)hipMalloc(&dX, (size_t)B * (Nt + 1) * N * m * 16);
  (void)hipMalloc(&dcoef, (size_t)B * m * 16);
  (void)hipMalloc(&dJ, B * 8);
  (void)hipMemcpy(dA, A.data(), A.size() * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(du, u.data(), u.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dst, st.data(), st.size() * sizeof(TStep), hipMemcpyHostToDevice);
  (void)hipMemcpy(dx0, x0.data(), x0.size() * 16, hipMemcpyHostToDevice);
  TChainArgs g{};
  g.N = N; g.m = m; g.nu = nu; g.Nt = Nt; g.At = dA; g.u = du; g.steps = dst; g.x0 = dx0; g.X = dX; g.L = dX;
  g.Xt = dx0; g.cost_kind = 2; g.n_norm = 1.0; g.J = dJ; g.coef = (cx<double>*)dcoef;
  const size_t lds = (nu + 1) * NN * 16 + (size_t)2 * S * JT * chain_mpad(m, CB) * 16 + 512;
  (void)hipFuncSetAttribute((const void*)k_tchain_fwd<double, S, JT, CB, NP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0;
  for (int it = 0; it < 3; ++it) {
#ifdef QOC_PROBE
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tc), z, sizeof(z));
#endif
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k_tchain_fwd<double, S, JT, CB, NP>), dim3(B), dim3(CHAIN_THREADS), lds, 0, g);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
  }
  printf("N=%d m=%d Nt=%d B=%d P=%d (S=%d JT=%d CB=%d): %.3f ms = %.3f us/step, %.0f ns/term\n", N, m, Nt, B, P, S, JT, CB, ms,
         ms * 1e3 / Nt, ms * 1e6 / Nt / P);
#ifdef QOC_PROBE
  unsigned long long tc[16];
  (void)hipMemcpyFromSymbol(tc, HIP_SYMBOL(g_tc), sizeof(tc));
  const double nt = (double)tc[3];
  printf("   per term (s_memtime units): matvec %.0f  matvec+store %.0f  barrier %.0f  (terms %.0f)\n", tc[0] / nt,
         tc[1] / nt, tc[2] / nt, nt);
#endif
}

template <int KQ, bool CHEB, int MAXT = 256>
void run_mf(int N, int m, int Nt, int B, int P) {
  const int nu = 2;
  const size_t NN = (size_t)N * N;
  std::vector<cx<double>> A((nu + 1) * NN);
  for (size_t e = 0; e < A.size(); ++e) A[e] = {((e * 7919) % 97) / (97.0 * N) - 0.5 / N, ((e * 104729) % 89) / (89.0 * N) - 0.5 / N};
  std::vector<double> u((size_t)B * Nt * nu, 0.01);
  std::vector<TStep> st((size_t)B * Nt, TStep{1.0, 0.0, P, 1, 1.0});
  std::vector<cx<double>> x0((size_t)N * m, cx<double>{1.0 / N, 0});
  cx<double>*dA, *dx0, *dX, *dcoef;
  double *dJ, *du;
  TStep* dst;
  (void)hipMalloc(&dA, A.size() * 16);
  (void)hipMalloc(&du, u.size() * 8);
  (void)hipMalloc(&dst, st.size() * sizeof(TStep));
  (void)hipMalloc(&dx0, x0.size() * 16);
  (void)hipMalloc(&dX, (size_t)B * (Nt + 1) * N * m * 16);
  (void)hipMalloc(&dcoef, (size_t)B * 2 * m * 16);
  (void)hipMalloc(&dJ, B * 8);
  (void)hipMemcpy(dA, A.data(), A.size() * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(du, u.data(), u.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dst, st.data(), st.size() * sizeof(TStep), hipMemcpyHostToDevice);
  (void)hipMemcpy(dx0, x0.data(), x0.size() * 16, hipMemcpyHostToDevice);
  double* dtc = nullptr;  // Chebyshev coefficients (any values: the timing does not depend on them)
  std::vector<double> tc_h((size_t)B * Nt * TCHEB_STRIDE);
  for (size_t e = 0; e < tc_h.size(); ++e) tc_h[e] = 1.0 / (1.0 + (double)(e % TCHEB_STRIDE));
  (void)hipMalloc(&dtc, tc_h.size() * 8);
  (void)hipMemcpy(dtc, tc_h.data(), tc_h.size() * 8, hipMemcpyHostToDevice);
  TChainArgs g{};
  g.N = N; g.m = m; g.nu = nu; g.Nt = Nt; g.At = dA; g.u = du; g.steps = dst; g.x0 = dx0; g.X = dX; g.L = dX;
  g.Xt = dx0; g.cost_kind = 2; g.n_norm = 1.0; g.J = dJ; g.coef = (cx<double>*)dcoef; g.tcoef = dtc;
  (void)hipMalloc(&g.sink, TCHAIN_SINK * sizeof(double));
  const size_t lds = tchain_mf_lds(N, m, nu, KQ < 0);
  const int threads = KQ < 0 ? 64 * ((m + 1) / 2) : 64 * tchain_mf_waves(N, m);
  (void)hipFuncSetAttribute((const void*)k_tchain_mf_fwd<KQ, CHEB, MAXT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0;
  for (int it = 0; it < 3; ++it) {
#ifdef QOC_PROBE
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tc), z, sizeof(z));
#endif
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k_tchain_mf_fwd<KQ, CHEB, MAXT>), dim3(B), dim3(threads), lds, 0, g);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
  }
  std::vector<double> xh((size_t)B * (Nt + 1) * N * m * 2);
  (void)hipMemcpy(xh.data(), dX, xh.size() * 8, hipMemcpyDeviceToHost);
  double cs = 0;
  for (size_t e = 0; e < xh.size(); ++e) cs += xh[e] * (1.0 + (double)(e % 7));
  printf("MFMA%s N=%d m=%d Nt=%d B=%d P=%d (KQ=%d, %d waves): %.3f ms = %.3f us/step, %.0f ns/term  checksum %.15e\n",
         CHEB ? " cheb" : "", N, m, Nt, B, P, KQ, tchain_mf_waves(N, m), ms, ms * 1e3 / Nt, ms * 1e6 / Nt / P, cs);
  (void)hipFree(dtc);
#ifdef QOC_PROBE
  unsigned long long tc[16];
  (void)hipMemcpyFromSymbol(tc, HIP_SYMBOL(g_tc), sizeof(tc));
  const double nt = (double)tc[7];
  printf("   per term (s_memtime): matvec %.0f  put %.0f  barrier %.0f  (terms %.0f); clock %.2f GHz\n", tc[4] / nt, tc[5] / nt,
         tc[6] / nt, nt, (double)tc[8] / ((double)tc[9] * 10.0));
  const double ns_ = (double)tc[13];
  printf("   per slice: prefetch+form %.0f  step %.0f  store %.0f  (slices %.0f)\n", tc[10] / ns_, tc[11] / ns_, tc[12] / ns_, ns_);
#endif
}

int main() {
  // KQ < 0: the register-state chains (TChainRot<-KQ / 4>); B = 2x the bench's seeds mimics the dual launch's waves
  run_mf<3, true>(9, 4, 500, 512, 8);
  run_mf<-4, true>(9, 4, 500, 512, 8);
  run_mf<-4, true>(9, 4, 500, 512, 4);
  run_mf<-4, true>(9, 4, 500, 512, 2);
  run_mf<-4, true>(9, 4, 500, 1024, 8);
  run_mf<8, true>(27, 1, 500, 512, 40);
  run_mf<-8, true>(27, 1, 500, 512, 40);
  run_mf<-8, true>(27, 1, 500, 512, 20);
  run_mf<-8, true>(27, 1, 500, 1024, 40);
  run_mf<10, true>(40, 2, 500, 256, 9);
  run_mf<-12, true>(40, 2, 250, 256, 9);
  return 0;
}
