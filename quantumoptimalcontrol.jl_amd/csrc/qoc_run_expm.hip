// qoc_run_expm.hip — launches of the exponential kernels (qoc_expm.hpp: k_expm, qoc_expm_rr.hpp: k_expm_rr*).
#include "qoc_expm_rr.hpp"
#include "qoc_internal.hpp"

namespace qoc_host {

bool expm_supported(int N, int prec) {
  if (N < 1 || N > 48) return false;
  const int NT = (N + 15) / 16;
  size_t lds = 0;
  if (prec == QOC_FP64) {
    lds = NT == 1 ? Expm<double, 1>::lds_bytes(N) : NT == 2 ? Expm<double, 2>::lds_bytes(N) : Expm<double, 3>::lds_bytes(N);
  } else {
    lds = NT == 1 ? Expm<float, 1>::lds_bytes(N) : NT == 2 ? Expm<float, 2>::lds_bytes(N) : Expm<float, 3>::lds_bytes(N);
  }
  return lds <= 160 * 1024;
}

// Two launches: the T12 pass over every unit, then the Paterson-Stockmeyer pass over the units the
// first one listed (||A_k||_1 > 4 theta_12); ps = {list (>= nunits ints), counter}.
template <typename T, int NT, int KS>
hipError_t launch_expm_rr_k(hipStream_t s, int N, int nu, int nunits, const void* Agen, const double* u,
                            const void* Ain, void* Uout, unsigned long long* hist, unsigned long long* thist,
                            int* ps, bool mix) {
  const size_t lds = ExpmRR<T, NT>::lds_bytes(N);
  if (mix) {  // one pass, T12 or Paterson-Stockmeyer per slice inline
    hipError_t e =
        hipFuncSetAttribute((const void*)k_expm_rr_mix<T, NT, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_expm_rr_mix<T, NT, KS>), dim3(nunits), dim3(64 * NT), lds, s, N, nu, nunits,
                       (const cx<T>*)Agen, u, (const cx<T>*)Ain, (cx<T>*)Uout, hist, thist);
    return hipGetLastError();
  }
  hipError_t e =
      hipFuncSetAttribute((const void*)k_expm_rr<T, NT, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_expm_rr_ps<T, NT, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int* list = ps + 1;
  if ((e = hipMemsetAsync(ps, 0, sizeof(int), s)) != hipSuccess) return e;
  hipLaunchKernelGGL((k_expm_rr<T, NT, KS>), dim3(nunits), dim3(64 * NT), lds, s, N, nu, nunits, (const cx<T>*)Agen, u,
                     (const cx<T>*)Ain, (cx<T>*)Uout, hist, thist, list, ps);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int grid = nunits;  // pass 2 exits at once past the listed count
  hipLaunchKernelGGL((k_expm_rr_ps<T, NT, KS>), dim3(grid), dim3(64 * NT), lds, s, N, nu, (const cx<T>*)Agen, u,
                     (const cx<T>*)Ain, (cx<T>*)Uout, hist, thist, (const int*)list, (const int*)ps);
  return hipGetLastError();
}

// k-steps: f64 ceil(N/4) (compile-time, one of the 4 values for this NT), f32 all 4 NT.
template <typename T, int NT>
hipError_t launch_expm_rr_t(hipStream_t s, int N, int nu, int nunits, const void* Agen, const double* u,
                            const void* Ain, void* Uout, unsigned long long* hist, unsigned long long* thist, int* ps,
                            bool mix) {
  const int ks = sizeof(T) == 8 ? (N + 3) / 4 : 4 * NT;
#define QOC_RRK(K) \
  if (ks == (K)) return launch_expm_rr_k<T, NT, (K)>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, thist, ps, mix)
  if constexpr (sizeof(T) == 8) {
    QOC_RRK(4 * NT - 3);
    QOC_RRK(4 * NT - 2);
    QOC_RRK(4 * NT - 1);
  }
  QOC_RRK(4 * NT);
#undef QOC_RRK
  return hipErrorInvalidValue;
}

template <typename T, int NT, int ALG>
hipError_t launch_expm_t(hipStream_t s, int N, int nu, int nunits, const void* Agen, const double* u,
                         const void* Ain, void* Uout, unsigned long long* hist, int* deg, int* sq,
                         unsigned long long* thist) {
  const size_t lds = Expm<T, NT>::lds_bytes(N);
  hipError_t e =
      hipFuncSetAttribute((const void*)k_expm<T, NT, ALG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_expm<T, NT, ALG>), dim3(nunits), dim3(256), lds, s, N, nu, nunits, (const cx<T>*)Agen, u,
                     (const cx<T>*)Ain, (cx<T>*)Uout, hist, deg, sq, thist);
  return hipGetLastError();
}

hipError_t launch_expm(int prec, hipStream_t s, int N, int nu, int nunits, const void* Agen, const double* u,
                       const void* Ain, void* Uout, unsigned long long* hist, int* deg, int* sq, int alg,
                       unsigned long long* thist, int* ps, bool mix) {
  const int NT = (N + 15) / 16;
  // alg 1: the register-resident T12 kernel (qoc_expm_rr.hpp); alg 2: the LDS Paterson-Stockmeyer one.
  const bool rr = alg == 1 && ps;  // the register-resident kernel needs the pass-2 list (ctx workspace)
#define QOC_LX(TT, NTT)                                                                                   \
  return alg ? (rr ? launch_expm_rr_t<TT, NTT>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, thist, ps, mix) \
                   : launch_expm_t<TT, NTT, 1>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, deg, sq, thist)) \
             : launch_expm_t<TT, NTT, 0>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, deg, sq, thist)
  if (prec == QOC_FP64) {
    if (NT == 1) QOC_LX(double, 1);
    if (NT == 2) QOC_LX(double, 2);
    QOC_LX(double, 3);
  }
  if (NT == 1) QOC_LX(float, 1);
  if (NT == 2) QOC_LX(float, 2);
  QOC_LX(float, 3);
#undef QOC_LX
}

}  // namespace qoc_host
