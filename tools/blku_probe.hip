// Segment cycle breakdown of the block-propagator launches (diagnostic; built with -DQOC_PROBE):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DQOC_PROBE -o tools/blku_probe tools/blku_probe.hip
// A cavity-shaped problem (N = 2 n blocks of 2 rows {b, b + n}, m = 2, nu = 2; NB = 3: the zz shape) with
// synthetic skew-Hermitian generators of the cavity's norms; prints the launch time of k_blku_fwd and of the fused
// backward k_blku_bwdg (order 3) per worker-wave count and chunk size, and for workgroup 7 the cycles per chunk
// of: chain compute, chain barrier wait, worker (formation + records + gradient), of which gradient, worker
// barrier wait.  Probe modes: 1 no formation, 2 no chain, 3 no chain stores, 5 no gradient.
// Usage: blku_probe [NB=2|3] [B] [Nt]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_blku.hpp"
using namespace qoc;

template <int NB, int S>
void run(int B, int Nt, int nblk, int m, int W, int C, int mode, bool bwdg) {
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
        if (i == k) A[r + (size_t)N * c] = {0.0, -0.016 * (i * b) + 0.15};  // -i (H0 - centre)
        if (i != k) {
          A[NN + r + (size_t)N * c] = {0.0, -0.5};                     // -i (T + T^H) / 2
          A[2 * NN + r + (size_t)N * c] = {i < k ? 0.5 : -0.5, 0.0};  // -i i (T - T^H) / 2
        }
      }
  std::vector<double> u((size_t)B * Nt * nu);
  for (size_t e = 0; e < u.size(); ++e) u[e] = 0.05 * (((e * 7919) % 1000) / 500.0 - 1.0);
  std::vector<cx<double>> x0((size_t)N * m, cx<double>{0, 0});
  for (int c = 0; c < m; ++c)
    for (int r = 0; r < N; ++r) x0[r + (size_t)N * c] = {(r % 2 == c % 2) ? 1.0 / std::sqrt(N / 2.0) : 0.0, 0.0};
  cx<double>*dA, *dx0, *dX, *dL, *dcoef;
  double *dJ, *du, *dsink;
  int* dbrow;
  unsigned long long* dterms;
  (void)hipMalloc(&dA, A.size() * 16);
  (void)hipMalloc(&du, u.size() * 8);
  (void)hipMalloc(&dx0, x0.size() * 16);
  (void)hipMalloc(&dX, (size_t)B * (Nt + 1) * N * m * 16);
  (void)hipMalloc(&dL, (size_t)B * (Nt + 1) * N * m * 16);
  (void)hipMalloc(&dcoef, (size_t)B * 2 * m * 16);
  (void)hipMalloc(&dJ, B * 8);
  (void)hipMalloc(&dsink, TCHAIN_SINK * 8);
  (void)hipMalloc(&dbrow, brow.size() * 4);
  (void)hipMalloc(&dterms, 256 * 8);  // TERM_SLOTS partial sums
  (void)hipMemcpy(dA, A.data(), A.size() * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(du, u.data(), u.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dx0, x0.data(), x0.size() * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(dbrow, brow.data(), brow.size() * 4, hipMemcpyHostToDevice);
  TChainArgs g{};
  g.N = N; g.m = m; g.nu = nu; g.Nt = Nt; g.At = dA; g.u = du; g.x0 = dx0; g.X = dX; g.L = dL;
  g.Xt = dx0; g.cost_kind = COST_TRACE; g.n_norm = m; g.J = dJ; g.coef = dcoef; g.sink = dsink;
  BlkArgs bk{};
  bk.brow = dbrow; bk.A = dA; bk.nblk = nblk;
  BlkuParams bp{};
  bp.rad[0] = 0.154; bp.rad[1] = bp.rad[2] = 0.5;
  bp.theta_cap = 0.978;
  bp.C = C;
  if (C < S) return;
  bp.CW = (nblk * m * (NB == 2 ? 2 : 4) + 63) / 64;
  bp.Ntp = (Nt + 63) / 64 * 64;
  bp.terms = dterms;
  bp.probe_mode = mode;
  double* ddJ;
  (void)hipMalloc(&ddJ, (size_t)B * Nt * nu * 8);
  bp.dJdu = ddJ;
  double2* dU = nullptr;  // stored propagators for the fused backward (mode >= 10: mode - 10 with bp.Uin)
  if (bwdg && mode >= 10) {
    (void)hipMalloc(&dU, (size_t)B * Nt * NB * NB * nblk * 16);
    (void)hipMemset(dU, 0, (size_t)B * Nt * NB * NB * nblk * 16);
    bp.Uin = dU;
    bp.probe_mode = mode - 10;
  }
  if (!bwdg && mode == 20) {  // the forward storing the propagators (the eval's)
    (void)hipMalloc(&dU, (size_t)B * Nt * NB * NB * nblk * 16);
    bp.Uout = dU;
    bp.probe_mode = 0;
  }
  {
    std::vector<cx<double>> cf((size_t)B * 2 * m, cx<double>{0.3, -0.1});
    (void)hipMemcpy(dcoef, cf.data(), cf.size() * 16, hipMemcpyHostToDevice);
  }
  (void)hipMemset(dX, 0, (size_t)B * (Nt + 1) * N * m * 16);
  double* drec;
  const long long total = (long long)B * bp.Ntp;
  (void)hipMalloc(&drec, total * BLKU_REC * 8);
  bp.rec = drec;
  hipLaunchKernelGGL(k_blku_rec, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, 0, bp, du, nu, Nt, total, drec);
  (void)hipDeviceSynchronize();
  const size_t lds = blku_lds(N, m, NB, nblk, C, bwdg ? 1 : 0);
  if (lds > 160 * 1024) return;  // does not fit one CU
  const void* kf = bwdg ? (const void*)k_blku_bwdg<NB, S, 3> : (const void*)k_blku_fwd<NB, S>;
  (void)hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0;
  unsigned long long z[16] = {};
  for (int it = 0; it < 3; ++it) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bk), z, sizeof(z));
    (void)hipEventRecord(a);
    if (bwdg) hipLaunchKernelGGL((k_blku_bwdg<NB, S, 3>), dim3(B), dim3(64 * W), lds, 0, g, bk, bp);
    else hipLaunchKernelGGL((k_blku_fwd<NB, S>), dim3(B), dim3(64 * W), lds, 0, g, bk, bp);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
  }
  if (hipGetLastError() != hipSuccess) {
    printf("launch failed\n");
    exit(1);
  }
  unsigned long long tc[16];
  (void)hipMemcpyFromSymbol(tc, HIP_SYMBOL(g_bk), sizeof(tc));
  const int nC = (Nt + C - 1) / C, fw = W - bp.CW - (bwdg ? (bp.Uin ? 2 : 1) : 0);  // bwdg: staging waves
  printf("%s NB=%d S=%d B=%d Nt=%d W=%d C=%2d mode=%d lds=%6zu: %.4f ms  per chunk (cycles): chain %6.0f  wait %6.0f"
         " | worker %6.0f  (recs %5.0f  grad %6.0f)  wait %6.0f | stage x %5.0f wait %5.0f  U %5.0f wait %5.0f\n",
         bwdg ? "bwdg" : "fwd ", NB, S, B, Nt, W, C, mode, lds, ms, tc[0] / (double)nC / bp.CW,
         tc[1] / (double)nC / bp.CW, tc[3] / (double)nC / fw, tc[6] / (double)nC / fw, tc[5] / (double)nC / fw,
         tc[4] / (double)nC / fw, tc[7] / (double)nC, tc[8] / (double)nC, tc[9] / (double)nC, tc[10] / (double)nC);
  (void)hipFree(dA); (void)hipFree(du); (void)hipFree(dx0); (void)hipFree(dX); (void)hipFree(dL); (void)hipFree(dcoef);
  (void)hipFree(dJ); (void)hipFree(dsink); (void)hipFree(dbrow); (void)hipFree(dterms); (void)hipFree(drec); (void)hipFree(ddJ); if (dU) (void)hipFree(dU);
}

int main(int argc, char** argv) {
  const int NB = argc > 1 ? atoi(argv[1]) : 2;
  const int B = argc > 2 ? atoi(argv[2]) : (NB == 2 ? 256 : 512);
  const int Nt = argc > 3 ? atoi(argv[3]) : (NB == 2 ? 1000 : 500);
  const int nblk = NB == 2 ? 20 : 3, m = NB == 2 ? 2 : 4;
  const int W0 = NB == 2 ? 2 : 1;  // chain waves
  (void)W0;
  for (int C : {16, 19, 21, 24, 28, 32}) {  // forward storing the propagators, per chunk size
    if (NB == 2) run<2, 1>(B, Nt, nblk, m, 8, C, 20, false);
    else run<3, 1>(B, Nt, nblk, m, 4, C, 20, false);
  }
  // fused backward with stored propagators: all (10), no grad (15), per chunk size (the workgroups a CU holds: 8 waves)
  const int Wb = NB == 2 ? 8 : 4;
  for (int mode : {10, 15})
    for (int C : {8, 12, 15, 16, 20, 21}) {
      if (NB == 2 && C > 16) continue;
      if (mode == 15 && C != 12 && C != 16) continue;
      if (NB == 2) run<2, 1>(B, Nt, nblk, m, Wb, C, mode, true);
      else run<3, 1>(B, Nt, nblk, m, Wb, C, mode, true);
    }
  return 0;
}
