// Standalone check of k_expm_rr against a host Taylor reference (NaN / accuracy hunt), any N, fp32/fp64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <complex>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_expm_rr.hpp"
using namespace qoc;
static int* g_ps = nullptr;  // pass-2 counter + list
typedef std::complex<double> C;
static std::vector<C> expm_ref(const std::vector<C>& A, int N) {
  // scaling and squaring with a long Taylor series (reference quality for ||A|| ~ 1)
  double nrm = 0;
  for (int j = 0; j < N; ++j) { double s = 0; for (int i = 0; i < N; ++i) s += std::abs(A[i + N * j]); nrm = std::max(nrm, s); }
  int sq = std::max(0, (int)std::ceil(std::log2(nrm / 0.25)));
  std::vector<C> X(N * N), T(N * N), R(N * N, 0.0);
  for (int e = 0; e < N * N; ++e) X[e] = A[e] / std::ldexp(1.0, sq);
  for (int i = 0; i < N; ++i) R[i + N * i] = 1.0;
  std::vector<C> P = R;
  for (int k = 1; k < 30; ++k) {
    for (int i = 0; i < N; ++i) for (int j = 0; j < N; ++j) { C s = 0; for (int l = 0; l < N; ++l) s += P[i + N * l] * X[l + N * j]; T[i + N * j] = s / (double)k; }
    P = T; for (int e = 0; e < N * N; ++e) R[e] += P[e];
  }
  for (int q = 0; q < sq; ++q) { for (int i = 0; i < N; ++i) for (int j = 0; j < N; ++j) { C s = 0; for (int l = 0; l < N; ++l) s += R[i + N * l] * R[l + N * j]; T[i + N * j] = s; } R = T; }
  return R;
}
template <typename T, int NT, int KS>
void check(int N, double scale, int units) {
  std::vector<cx<T>> A((size_t)units * N * N);
  std::vector<std::vector<C>> ref;
  srand(3);
  for (int u = 0; u < units; ++u) {
    std::vector<C> H(N * N);
    for (int j = 0; j < N; ++j) for (int i = 0; i <= j; ++i) {
      double re = rand() / (double)RAND_MAX - 0.5, im = (i == j) ? 0 : rand() / (double)RAND_MAX - 0.5;
      H[i + N * j] = C(re, im); H[j + N * i] = C(re, -im);
    }
    std::vector<C> Ad(N * N);
    for (int e = 0; e < N * N; ++e) { Ad[e] = C(0, -1) * H[e] * (scale / N); A[(size_t)u * N * N + e] = {(T)Ad[e].real(), (T)Ad[e].imag()}; Ad[e] = C((double)(T)Ad[e].real(), (double)(T)Ad[e].imag()); }
    if (u < 4) ref.push_back(expm_ref(Ad, N));
  }
  cx<T>*dA, *dX; (void)hipMalloc(&dA, A.size() * sizeof(cx<T>)); (void)hipMalloc(&dX, A.size() * sizeof(cx<T>));
  (void)hipMemcpy(dA, A.data(), A.size() * sizeof(cx<T>), hipMemcpyHostToDevice);
  (void)hipMemset(dX, 0xff, A.size() * sizeof(cx<T>));
  const size_t lds = ExpmRR<T, NT>::lds_bytes(N);
  (void)hipFuncSetAttribute((const void*)k_expm_rr<T, NT, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (!g_ps) (void)hipMalloc(&g_ps, (1 << 20) * sizeof(int));
    (void)hipMemset(g_ps, 0, 4);
    hipLaunchKernelGGL((k_expm_rr<T, NT, KS>), dim3(units), dim3(64 * NT), lds, 0, N, 0, units, nullptr, nullptr, dA, dX, nullptr, nullptr, g_ps + 1, g_ps);
    (void)hipFuncSetAttribute((const void*)k_expm_rr_ps<T, NT, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k_expm_rr_ps<T, NT, KS>), dim3(units), dim3(64 * NT), lds, 0, N, 0, nullptr, nullptr, dA, dX, nullptr, nullptr, g_ps + 1, g_ps);
  hipError_t e = hipDeviceSynchronize();
  std::vector<cx<T>> X(A.size());
  (void)hipMemcpy(X.data(), dX, X.size() * sizeof(cx<T>), hipMemcpyDeviceToHost);
  double md = 0; int nan = 0, first = -1;
  for (int u = 0; u < units; ++u) for (int i = 0; i < N * N; ++i) {
    const cx<T> x = X[(size_t)u * N * N + i];
    if (!std::isfinite((double)x.r) || !std::isfinite((double)x.i)) { if (first < 0) first = u * N * N + i; ++nan; continue; }
    if (u < 4) md = std::max(md, std::abs(C(x.r, x.i) - ref[u][i]));
  }
  for (int u = 0; u < 4 && nan; ++u) {
    int cnt = 0; printf("   unit %d nonfinite:", u);
    for (int i = 0; i < N * N; ++i) { const cx<T> x = X[(size_t)u * N * N + i]; if (!std::isfinite((double)x.r) || !std::isfinite((double)x.i)) { if (cnt < 12) printf(" (%d,%d)", i % N, i / N); ++cnt; } }
    printf("  total %d\n", cnt);
  }
  printf("%s N=%d NT=%d KS=%d scale=%g: %s  max err %.3g  nonfinite %d (first unit %d elem %d = row %d col %d)\n", sizeof(T) == 8 ? "f64" : "f32", N, NT, KS, scale,
         hipGetErrorString(e), md, nan, first < 0 ? -1 : first / (N * N), first < 0 ? -1 : first % (N * N), first < 0 ? -1 : (first % (N * N)) % N, first < 0 ? -1 : (first % (N * N)) / N);
  (void)hipFree(dA); (void)hipFree(dX);
}
int main() {
  for (int rep = 0; rep < 6; ++rep) {
    check<float, 3, 12>(40, 0.5, 4096);
    check<float, 2, 8>(20, 0.5, 4096);
    check<double, 3, 10>(40, 0.5, 4096);
    check<double, 2, 7>(27, 3.0, 4096);
  }
  return 0;
}
