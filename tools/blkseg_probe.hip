// Phase cycle breakdown of the segmented block eval (diagnostic; built with -DQOC_PROBE):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DQOC_PROBE -o tools/blkseg_probe tools/blkseg_probe.hip
// A cavity-shaped problem (N = 2 n blocks of 2 rows {b, b + n}, m = 2, nu = 2; NB = 3: the zz shape, m = 4) with
// synthetic skew-Hermitian generators of the cavity's norms; prints the launch time of k_blkseg_eval (order 3) per
// waves-per-seed W and segment count S, and for workgroup 7 the cycles per wave of: prologue (generators, records),
// phase 1 (segment products), phase 2 (scan, costs, G), phase 3 (backward + gradient), epilogue.
// Usage: blkseg_probe [NB=2|3] [B] [Nt]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_blkseg.hpp"
using namespace qoc;

template <int NB, int WMAX = 8>
void run(int B, int Nt, int nblk, int m, int W, int Scap, int noturn = 0, int turnmode = 1) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_seg_noturn), &noturn, sizeof(int));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_seg_turnmode), &turnmode, sizeof(int));
  const int nu = 2, N = NB * nblk;
  const size_t NN = (size_t)N * N;
  std::vector<cx<double>> A((nu + 1) * NN, cx<double>{0, 0});
  std::vector<int> brow((size_t)nblk * NB);
  for (int b = 0; b < nblk; ++b)
    for (int i = 0; i < NB; ++i) brow[b * NB + i] = b + i * nblk;
  for (int b = 0; b < nblk; ++b)
    for (int i = 0; i < NB; ++i)
      for (int k = 0; k < NB; ++k) {
        const int r = brow[b * NB + i], c = brow[b * NB + k];
        if (i == k) A[r + (size_t)N * c] = {0.0, -0.016 * (i * b) + 0.15};
        if (i != k) {
          A[NN + r + (size_t)N * c] = {0.0, -0.5};
          A[2 * NN + r + (size_t)N * c] = {i < k ? 0.5 : -0.5, 0.0};
        }
      }
  std::vector<double> u((size_t)B * Nt * nu);
  for (size_t e = 0; e < u.size(); ++e) u[e] = 0.05 * (((e * 7919) % 1000) / 500.0 - 1.0);
  std::vector<cx<double>> x0((size_t)N * m, cx<double>{0, 0});
  for (int c = 0; c < m; ++c)
    for (int r = 0; r < N; ++r) x0[r + (size_t)N * c] = {(r % 2 == c % 2) ? 1.0 / std::sqrt(N / 2.0) : 0.0, 0.0};
  cx<double>*dA, *dx0, *dcoef;
  double *dJ, *du, *ddJ;
  int* dbrow;
  (void)hipMalloc(&dA, A.size() * 16);
  (void)hipMalloc(&du, u.size() * 8);
  (void)hipMalloc(&dx0, x0.size() * 16);
  (void)hipMalloc(&dcoef, (size_t)B * 2 * m * 16);
  (void)hipMalloc(&dJ, B * 8);
  (void)hipMalloc(&ddJ, (size_t)B * Nt * nu * 8);
  (void)hipMalloc(&dbrow, brow.size() * 4);
  (void)hipMemcpy(dA, A.data(), A.size() * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(du, u.data(), u.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dx0, x0.data(), x0.size() * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(dbrow, brow.data(), brow.size() * 4, hipMemcpyHostToDevice);
  TChainArgs g{};
  g.N = N; g.m = m; g.nu = nu; g.Nt = Nt; g.At = dA; g.u = du; g.x0 = dx0;
  g.Xt = dx0; g.cost_kind = COST_TRACE; g.n_norm = m; g.J = dJ; g.coef = dcoef;
  BlkArgs bk{};
  bk.brow = dbrow; bk.A = dA; bk.nblk = nblk;
  BlksegParams sp{};
  sp.rad[0] = 0.154; sp.rad[1] = sp.rad[2] = 0.5;
  sp.theta_cap = 0.978;
  sp.UPW = 64 / nblk;
  int S = std::min(std::min(W * sp.UPW, Nt), Scap);
  sp.L = (Nt + S - 1) / S;
  sp.S = (Nt + sp.L - 1) / sp.L;
  W = (sp.S + sp.UPW - 1) / sp.UPW;
  sp.RB = blkseg_rb(sp.UPW, nu);
  sp.u = du;
  sp.dJdu = ddJ;
  const size_t lds = blkseg_lds(N, m, nu, NB, nblk, Nt, sp.S, W, sp.RB);
  if (lds > 160 * 1024) return;
  (void)hipFuncSetAttribute((const void*)k_blkseg_eval<NB, 3, WMAX>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0, best = 1e9;
  unsigned long long z[16] = {};
  for (int it = 0; it < 5; ++it) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bk), z, sizeof(z));
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k_blkseg_eval<NB, 3, WMAX>), dim3(B), dim3(64 * W), lds, 0, g, bk, sp);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    best = std::min(best, ms);
  }
  if (hipGetLastError() != hipSuccess) {
    printf("launch failed\n");
    exit(1);
  }
  unsigned long long tc[16];
  (void)hipMemcpyFromSymbol(tc, HIP_SYMBOL(g_bk), sizeof(tc));
  printf("%s NB=%d B=%d Nt=%d W=%d S=%3d L=%3d lds=%6zu: %.4f ms (best of 5) | cycles per wave: prologue %6.0f  seg %6.0f"
         "  scan+cost %6.0f  backward %7.0f  epilogue %5.0f  total %7.0f  (per slice-step: seg %.0f, bwd %.0f)\n",
         noturn ? "noturn" : turnmode ? "progr " : "turns ", NB, B, Nt, W, sp.S, sp.L, lds, best, tc[0] / (double)W, tc[1] / (double)W, tc[2] / (double)W,
         tc[3] / (double)W, tc[4] / (double)W, tc[5] / (double)W, tc[1] / (double)W / sp.L,
         tc[3] / (double)W / sp.L);
  unsigned long long sw[32];
  (void)hipMemcpyFromSymbol(sw, HIP_SYMBOL(g_segw), sizeof(sw));
  printf("    per wave: phase-1 end");
  for (int w = 0; w < W; ++w) printf(" %7llu", sw[w]);
  printf(" | phase-3 end");
  for (int w = 0; w < W; ++w) printf(" %7llu", sw[16 + w]);
  printf("\n");
  (void)hipFree(dA); (void)hipFree(du); (void)hipFree(dx0); (void)hipFree(dcoef); (void)hipFree(dJ);
  (void)hipFree(ddJ); (void)hipFree(dbrow);
}

int main(int argc, char** argv) {
  const int NB = argc > 1 ? atoi(argv[1]) : 2;
  const int B = argc > 2 ? atoi(argv[2]) : (NB == 2 ? 256 : 512);
  const int Nt = argc > 3 ? atoi(argv[3]) : (NB == 2 ? 1000 : 500);
  const int nblk = NB == 2 ? 20 : 3, m = NB == 2 ? 2 : 4;
  if (NB == 2) {
    run<2, 8>(B, Nt, nblk, m, 8, 1 << 20, 0, 1);
    run<2, 8>(B, Nt, nblk, m, 8, 1 << 20, 0, 0);
    run<2, 8>(B, Nt, nblk, m, 8, 1 << 20, 1);
    run<2, 8>(B, Nt, nblk, m, 8, 1 << 20, 0, 1);
  } else {
    run<3, 8>(B, Nt, nblk, m, 4, 1 << 20);
    run<3, 8>(B, Nt, nblk, m, 8, 1 << 20, 0, 1);
    run<3, 8>(B, Nt, nblk, m, 8, 1 << 20, 0, 0);
  }
  return 0;
}
