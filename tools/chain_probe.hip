// Per-phase cycle counts of the forward chain step (diagnostic; built with -DQOC_PROBE).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DQOC_PROBE -o tools/chain_probe tools/chain_probe.hip
#include <cstdio>
#include <vector>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_chain.hpp"
using namespace qoc;

template <int S, int JT, int CB>
void run(int N, int m, int Nt, int B) {
  const size_t NN = (size_t)N * N;
  std::vector<cx<double>> U(NN * Nt * B);
  for (size_t e = 0; e < U.size(); ++e) U[e] = {((e * 7919) % 97) / (97.0 * N), ((e * 104729) % 89) / (89.0 * N)};
  std::vector<cx<double>> x0((size_t)N * m, cx<double>{1.0 / N, 0});
  cx<double>*dU, *dx0, *dX, *dcoef;
  double* dJ;
  (void)hipMalloc(&dU, U.size() * 16);
  (void)hipMalloc(&dx0, x0.size() * 16);
  (void)hipMalloc(&dX, (size_t)B * (Nt + 1) * N * m * 16);
  (void)hipMalloc(&dcoef, (size_t)B * m * 16);
  (void)hipMalloc(&dJ, B * 8);
  (void)hipMemcpy(dU, U.data(), U.size() * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(dx0, x0.data(), x0.size() * 16, hipMemcpyHostToDevice);
  const size_t lds = (size_t)(2 * S * JT * chain_mpad(m, CB)) * 16 + 64 * 8;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0;
  for (int it = 0; it < 3; ++it) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k_chain_fwd<double, S, JT, CB>), dim3(B), dim3(CHAIN_THREADS), lds, 0, N, m, Nt, dU, dx0, 0, dX,
                       dx0, 2, 1.0, nullptr, 0.0, dJ, dcoef);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
  }
  unsigned long long st[64];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_probe), sizeof(st));
  printf("N=%d m=%d Nt=%d B=%d (S=%d JT=%d D=%d): %.3f ms = %.3f us/step\n", N, m, Nt, B, S, JT, ChainRegs<double, S, JT, CB, true>::D,
         ms, ms * 1e3 / Nt);
  printf("   cycles/step: copy_out %.0f  settle(wait U) %.0f  matvec %.0f  refill issue %.0f  barrier %.0f\n",
         (double)st[33] / Nt, (double)st[34] / Nt, (double)st[35] / Nt, (double)st[36] / Nt, (double)st[37] / Nt);
  (void)hipFree(dU);
  (void)hipFree(dx0);
  (void)hipFree(dX);
  (void)hipFree(dcoef);
  (void)hipFree(dJ);
}

int main() {
  run<4, 4, 4>(9, 4, 500, 512);
  run<4, 4, 4>(9, 4, 500, 8);
  run<8, 4, 1>(27, 1, 2000, 512);
  run<4, 10, 1>(40, 2, 1000, 256);
  run<4, 10, 1>(40, 2, 1000, 8);
  return 0;
}
