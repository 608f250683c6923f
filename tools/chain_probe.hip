// Diagnostic: one step of k_chain_fwd stamped (s_memtime), cavity-sized (N=40, m=2, Nt=1000, B=256).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_chain.hpp"
using namespace qoc;
int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 40, m = 2, Nt = 1000, B = 256;
  const size_t NN = (size_t)N * N, Nm = (size_t)N * m;
  cx<double>*U, *X, *x0, *Xt, *coef;
  double* J;
  (void)hipMalloc(&U, B * Nt * NN * 16);
  (void)hipMalloc(&X, B * (Nt + 1) * Nm * 16);
  (void)hipMalloc(&x0, Nm * 16);
  (void)hipMalloc(&Xt, Nm * 16);
  (void)hipMalloc(&coef, B * m * 16);
  (void)hipMalloc(&J, B * 8);
  (void)hipMemset(U, 0, B * Nt * NN * 16);
  (void)hipMemset(x0, 0, Nm * 16);
  (void)hipMemset(Xt, 0, Nm * 16);
  size_t lds = (2 * N * (N + 1) + 2 * Nm) * 16 + 512;
  (void)hipFuncSetAttribute((const void*)k_chain_fwd<double>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int it = 0; it < 2; ++it) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k_chain_fwd<double>), dim3(B), dim3(256), lds, 0, N, m, Nt, U, x0, 0, X, Xt, 0, 2.0,
                       (const unsigned char*)nullptr, 0.0, J, coef);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
  }
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  unsigned long long st[64];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_probe), sizeof(st));
  printf("N=%d chain_fwd %.3f ms (%.2f us/step)  step500: dot %llu  commit %llu  prefetch-issue %llu  barrier %llu\n",
         N, ms, ms * 1e3 / Nt, st[51] - st[50], st[52] - st[51], st[53] - st[52], st[54] - st[53]);
  return 0;
}
