// Diagnostic microbenchmark for k_expm: phase stamps (s_memtime) + wall time per configuration.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DQOC_PROBE -o tools/expm_probe tools/expm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_expm_rr.hpp"
using namespace qoc;
static int* g_ps = nullptr;  // pass-2 counter + list

template <int NT, int ALG = 0>
void run(int N, double scale, int units, std::vector<cx<double>>* keep = nullptr) {
  using E = Expm<double, NT>;
  std::vector<cx<double>> A((size_t)units * N * N);
  srand(1);
  for (int u = 0; u < units; ++u) {
    // random skew-Hermitian with ||A||_1 ~ scale
    std::vector<cx<double>> H((size_t)N * N);
    for (int j = 0; j < N; ++j)
      for (int i = 0; i <= j; ++i) {
        double re = rand() / (double)RAND_MAX - 0.5, im = (i == j) ? 0 : rand() / (double)RAND_MAX - 0.5;
        H[i + N * j] = {re, im};
        H[j + N * i] = {re, -im};
      }
    double nrm = 0;
    for (int j = 0; j < N; ++j) {
      double s = 0;
      for (int i = 0; i < N; ++i) s += std::hypot(H[i + N * j].r, H[i + N * j].i);
      nrm = std::max(nrm, s);
    }
    for (int e = 0; e < N * N; ++e) A[(size_t)u * N * N + e] = {H[e].i * scale / nrm, -H[e].r * scale / nrm};
  }
  cx<double>*dA, *dX;
  (void)hipMalloc(&dA, A.size() * 16);
  (void)hipMalloc(&dX, A.size() * 16);
  (void)hipMemcpy(dA, A.data(), A.size() * 16, hipMemcpyHostToDevice);
  size_t lds = E::lds_bytes(N);
  (void)hipFuncSetAttribute((const void*)k_expm<double, NT, ALG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int it = 0; it < 3; ++it) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k_expm<double, NT, ALG>), dim3(units), dim3(256), lds, 0, N, 0, units, nullptr, nullptr, dA,
                       dX, nullptr, nullptr, nullptr, nullptr);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
  }
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  unsigned long long st[64];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_probe), sizeof(st));
  printf("N=%d scale=%.3g units=%d ALG=%d lds=%zu  wall %.3f ms  (%.3f us/unit/CU-slot)\n", N, scale, units, ALG, lds,
         ms, ms * 1e3 / units * 256);
  if (keep) {
    std::vector<cx<double>> X(A.size());
    (void)hipMemcpy(X.data(), dX, X.size() * 16, hipMemcpyDeviceToHost);
    if (keep->empty()) {
      *keep = X;
    } else {
      double md = 0;
      for (size_t i = 0; i < X.size(); ++i)
        md = std::max(md, std::abs(X[i].r - (*keep)[i].r) + std::abs(X[i].i - (*keep)[i].i));
      printf("   max |Taylor - Pade| = %.3g\n", md);
    }
  }
  if (ALG == 1) {
    printf("   form+norm %llu  A2 %llu  A3 %llu  Horner %llu  squarings %llu  store %llu\n", st[1] - st[0],
           st[50] - st[1], st[51] - st[50], st[5] - st[51], st[6] - st[5], st[7] - st[6]);
    goto done;
  }
  {
  const char* names[] = {"form+norm", "pade gemms", "Q/P store", "LU solve", "squarings", "store"};
  int idx[] = {0, 1, 2, 3, 5, 6, 7};
  for (int i = 0; i < 6; ++i) printf("   %-12s %8llu cycles(memtime)\n", names[i], st[idx[i + 1]] - st[idx[i]]);
  for (int pn = 0; pn < 3; ++pn)
    if (st[10 + 4 * pn])
      printf("   panel %d: factor %llu  U12 %llu  trailing %llu\n", pn, st[11 + 4 * pn] - st[10 + 4 * pn],
             st[12 + 4 * pn] - st[11 + 4 * pn], (pn < 2 && st[14 + 4 * pn] ? st[14 + 4 * pn] : st[30]) - st[12 + 4 * pn]);
  printf("   first GEMM (wave0) %llu   GJ block p0=20: publish %llu  W %llu  mfma %llu\n", st[21] - st[20],
         st[41] - st[40], st[42] - st[41], st[43] - st[42]);
  if (st[44])
    printf("   GJ16 block p0=16: publish %llu  Dinv %llu  W %llu  update %llu\n", st[45] - st[44], st[46] - st[45],
           st[47] - st[46], st[48] - st[47]);
  }
done:
  (void)hipMemset(0, 0, 0);
  {
    unsigned long long z[64] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_probe), z, sizeof(z));
  }
  (void)hipFree(dA);
  (void)hipFree(dX);
}

template <int NT>
void run_rr(int N, double scale, int units, std::vector<cx<double>>* keep) {
  using E = ExpmRR<double, NT>;
  std::vector<cx<double>> A((size_t)units * N * N);
  srand(1);
  for (int u = 0; u < units; ++u) {
    std::vector<cx<double>> H((size_t)N * N);
    for (int j = 0; j < N; ++j)
      for (int i = 0; i <= j; ++i) {
        double re = rand() / (double)RAND_MAX - 0.5, im = (i == j) ? 0 : rand() / (double)RAND_MAX - 0.5;
        H[i + N * j] = {re, im};
        H[j + N * i] = {re, -im};
      }
    double nrm = 0;
    for (int j = 0; j < N; ++j) {
      double s = 0;
      for (int i = 0; i < N; ++i) s += std::hypot(H[i + N * j].r, H[i + N * j].i);
      nrm = std::max(nrm, s);
    }
    for (int e = 0; e < N * N; ++e) A[(size_t)u * N * N + e] = {H[e].i * scale / nrm, -H[e].r * scale / nrm};
  }
  cx<double>*dA, *dX;
  (void)hipMalloc(&dA, A.size() * 16);
  (void)hipMalloc(&dX, A.size() * 16);
  (void)hipMemcpy(dA, A.data(), A.size() * 16, hipMemcpyHostToDevice);
  size_t lds = E::lds_bytes(N);
  (void)hipFuncSetAttribute((const void*)k_expm_rr<double, NT, (NT == 3 ? 10 : NT == 2 ? 7 : 3)>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int it = 0; it < 3; ++it) {
    (void)hipEventRecord(a);
    if (!g_ps) (void)hipMalloc(&g_ps, (1 << 20) * sizeof(int));
    (void)hipMemset(g_ps, 0, 4);
    hipLaunchKernelGGL((k_expm_rr<double, NT, (NT == 3 ? 10 : NT == 2 ? 7 : 3)>), dim3(units), dim3(64 * NT), lds, 0, N, 0, units, nullptr, nullptr, dA,
                       dX, nullptr, nullptr, g_ps + 1, g_ps);
    (void)hipFuncSetAttribute((const void*)k_expm_rr_ps<double, NT, (NT == 3 ? 10 : NT == 2 ? 7 : 3)>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k_expm_rr_ps<double, NT, (NT == 3 ? 10 : NT == 2 ? 7 : 3)>), dim3(units), dim3(64 * NT), lds, 0, N, 0, nullptr, nullptr, dA,
                       dX, nullptr, nullptr, g_ps + 1, g_ps);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
  }
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("RR N=%d scale=%.3g units=%d lds=%zu  wall %.3f ms  (%.3f us/unit/CU)\n", N, scale, units, lds, ms, ms * 1e3 / units * 256);
  std::vector<cx<double>> X(A.size());
  (void)hipMemcpy(X.data(), dX, X.size() * 16, hipMemcpyDeviceToHost);
  double md = 0;
  for (size_t i = 0; i < X.size(); ++i)
    md = std::max(md, std::abs(X[i].r - (*keep)[i].r) + std::abs(X[i].i - (*keep)[i].i));
  printf("   max |RR - Pade| = %.3g\n", md);
  {
    unsigned long long st[64];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_probe), sizeof(st));
    printf("   load A %llu  norm %llu  A2+A3 %llu  B's+products 3,4 %llu  squarings %llu  store %llu\n", st[1] - st[0], st[2] - st[1],
           st[3] - st[2], st[4] - st[3], st[5] - st[4], st[6] - st[5]);
    if (st[16])
      printf("   T12: make_B x4 %llu  bar %llu  B1 store + P3 %llu  A6 store + gets %llu  bar %llu  P4 %llu\n",
             st[10] - st[3], st[11] - st[10], st[12] - st[11], st[14] - st[12], st[15] - st[14], st[16] - st[15]);
    if (units <= 65536) {
      std::vector<unsigned long long> L(3 * (size_t)units);
      (void)hipMemcpyFromSymbol(L.data(), HIP_SYMBOL(g_life), L.size() * 8);
      unsigned long long t0 = ~0ull, t1 = 0;
      double life = 0;
      for (int u = 0; u < units; ++u) {
        t0 = std::min(t0, L[3 * u]);
        t1 = std::max(t1, L[3 * u + 1]);
        life += (double)(L[3 * u + 1] - L[3 * u]);
      }
      // average number of resident WGs = sum of lifetimes / (span x CUs)
      printf("   all WGs: span %.1f us, mean lifetime %.2f us, mean resident WGs per CU %.2f\n", (t1 - t0) / 100.0,
             life / units / 100.0, life / ((double)(t1 - t0) * 256.0));
    }
    printf("   block lifetime %llu memtime ticks, %llu realtime ticks -> %.3f GHz\n", st[6] - st[0], st[61] - st[60],
           (double)(st[6] - st[0]) / (double)(st[61] - st[60]) / 10.0);
  }
  (void)hipFree(dA);
  (void)hipFree(dX);
}

int main(int argc, char** argv) {
  {
    std::vector<cx<double>> k;
    run<1, 0>(9, 0.11, 256 * 64, &k);
    run<1, 1>(9, 0.11, 256 * 64, &k);
    run_rr<1>(9, 0.11, 256 * 64, &k);
  }
  {
    std::vector<cx<double>> k;
    run<2, 0>(27, 30.0, 256 * 64, &k);
    run<2, 1>(27, 30.0, 256 * 64, &k);
    run_rr<2>(27, 30.0, 256 * 64, &k);
  }
  {
    std::vector<cx<double>> k;
    run<3, 0>(40, 0.33, 256 * 64, &k);
    run<3, 1>(40, 0.33, 256 * 64, &k);
    run_rr<3>(40, 0.33, 256 * 64, &k);
    run_rr<3>(40, 0.33, 256, &k);
    run_rr<3>(40, 0.33, 512, &k);
    run_rr<3>(40, 0.33, 768, &k);
    run_rr<3>(40, 0.33, 1024, &k);
  }
  run<3, 1>(40, 0.33, 256);  // one workgroup per CU: uncontended phase costs
  {
    std::vector<cx<double>> k;
    run<3, 0>(40, 4.0, 256 * 16, &k);
    run<3, 1>(40, 4.0, 256 * 16, &k);
    run_rr<3>(40, 4.0, 256 * 16, &k);
  }
  return 0;
}
