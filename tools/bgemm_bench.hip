// bgemm_bench.hip — microbenchmark + cross-check of the large-N batched complex GEMM kernels.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bgemm_bench.hip -o tools/bgemm_bench
//   ./tools/bgemm_bench [N] [items] [K]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_bgemm.hpp"

using namespace qoc;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

static Opd opd(const void* p, long long inner) {
  Opd o;
  o.p = p;
  o.inner = inner;
  return o;
}

template <typename KFN>
static float timeit(KFN launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 256;
  const int items = argc > 2 ? atoi(argv[2]) : 1260;
  const int Kd = argc > 3 ? atoi(argv[3]) : N;
  const size_t per = (size_t)N * Kd, perC = (size_t)N * N;
  std::vector<cx<float>> h(per * items);
  srand(1);
  for (auto& v : h) {
    v.r = (float)(rand() / (double)RAND_MAX) - 0.5f;
    v.i = (float)(rand() / (double)RAND_MAX) - 0.5f;
  }
  cx<float>*A, *B, *C0, *C1;
  CK(hipMalloc(&A, per * items * sizeof(cx<float>)));
  CK(hipMalloc(&B, per * items * sizeof(cx<float>)));
  CK(hipMalloc(&C0, perC * items * sizeof(cx<float>)));
  CK(hipMalloc(&C1, perC * items * sizeof(cx<float>)));
  CK(hipMemcpy(A, h.data(), per * items * sizeof(cx<float>), hipMemcpyHostToDevice));
  for (auto& v : h) v.r = -v.r;
  CK(hipMemcpy(B, h.data(), per * items * sizeof(cx<float>), hipMemcpyHostToDevice));
  const double flops = 8.0 * N * (double)N * Kd * items;
  GemmArgs g;
  std::memset(&g, 0, sizeof(g));
  g.A = opd(A, (long long)per);
  g.B = opd(B, (long long)per);
  g.M = N;
  g.K = Kd;
  g.Ncol = N;
  g.nitems = items;
  g.alpha1 = 1.0;
  g.tiles_m = (N + BG_BM - 1) / BG_BM;
  g.tiles = g.tiles_m * ((N + BG_BN - 1) / BG_BN);
  GemmArgs g0 = g;
  g0.C1 = opd(C0, (long long)perC);
  g.C1 = opd(C1, (long long)perC);
  const dim3 grid(g.nitems * g.tiles);
  // reference: 4-product, KS=1, NBUF=2
  auto ref = [&]() { hipLaunchKernelGGL((k_bgemm<float, 0, 0, false, 1, 2>), grid, dim3(256), 0, 0, g0); };
  const float tr = timeit(ref, 5);
  printf("N=%d K=%d items=%d  ref 4M KS1 NBUF2: %.3f ms %.1f TF/s\n", N, Kd, items, tr, flops / tr / 1e9);
  std::vector<cx<float>> r0(perC * items), r1(perC * items);
  CK(hipMemcpy(r0.data(), C0, perC * items * sizeof(cx<float>), hipMemcpyDeviceToHost));
  auto check = [&](const char* name, float t) {
    CK(hipGetLastError());
    CK(hipMemcpy(r1.data(), C1, perC * items * sizeof(cx<float>), hipMemcpyDeviceToHost));
    double md = 0;
    for (size_t i = 0; i < r0.size(); ++i) md = fmax(md, fabs(r0[i].r - r1[i].r) + fabs(r0[i].i - r1[i].i));
    printf("  %-22s %.3f ms %.1f TF/s  maxdiff %.3g\n", name, t, flops / t / 1e9, md);
  };
#define VARIANT(KS, NB)                                                                             \
  {                                                                                                 \
    auto f = [&]() { hipLaunchKernelGGL((k_bgemm<float, 0, 0, true, KS, NB>), grid, dim3(256), 0, 0, g); }; \
    check("3M KS" #KS " NBUF" #NB, timeit(f, 5));                                                   \
  }
  VARIANT(1, 2)
  VARIANT(1, 1)
  VARIANT(2, 1)
  VARIANT(2, 2)
  if (Kd % 16 == 0 && N % 2 == 0) {
    auto f = [&]() { hipLaunchKernelGGL((k_bgemm_glds<0, 0>), grid, dim3(256), 0, 0, g); };
    check("glds 3M", timeit(f, 5));
    auto f2 = [&]() { hipLaunchKernelGGL((k_bgemm_glds<0, 0, 2>), grid, dim3(256), 0, 0, g); };
    check("glds 3M 2 stages", timeit(f2, 5));
    // op variants against their k_bgemm counterparts (A^H: square N = K only)
    auto cmp = [&](const char* name, auto kref, auto kg) {
      kref();
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(r0.data(), C1, perC * items * sizeof(cx<float>), hipMemcpyDeviceToHost));
      const float t = timeit(kg, 5);
      check(name, t);
    };
    if (Kd == N) {
      cmp("glds 3M opA=H", [&]() { hipLaunchKernelGGL((k_bgemm<float, 1, 0, true, 1, 2>), grid, dim3(256), 0, 0, g); },
          [&]() { hipLaunchKernelGGL((k_bgemm_glds<1, 0>), grid, dim3(256), 0, 0, g); });
      cmp("glds 3M opB=H", [&]() { hipLaunchKernelGGL((k_bgemm<float, 0, 1, true, 1, 2>), grid, dim3(256), 0, 0, g); },
          [&]() { hipLaunchKernelGGL((k_bgemm_glds<0, 1>), grid, dim3(256), 0, 0, g); });
      cmp("glds 3M opA=H opB=H", [&]() { hipLaunchKernelGGL((k_bgemm<float, 1, 1, true, 1, 2>), grid, dim3(256), 0, 0, g); },
          [&]() { hipLaunchKernelGGL((k_bgemm_glds<1, 1>), grid, dim3(256), 0, 0, g); });
    }
    // ragged M (rows past M clamped), items not a multiple of 8 (no XCD remap)
    {
      GemmArgs h = g;
      h.M = N - 6;
      h.nitems = items - 3;
      h.tiles_m = (h.M + BG_BM - 1) / BG_BM;
      h.tiles = h.tiles_m * ((N + BG_BN - 1) / BG_BN);
      const dim3 gr2(h.nitems * h.tiles);
      CK(hipMemset(C1, 0, perC * items * sizeof(cx<float>)));
      hipLaunchKernelGGL((k_bgemm<float, 0, 0, true, 1, 2>), gr2, dim3(256), 0, 0, h);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(r0.data(), C1, perC * items * sizeof(cx<float>), hipMemcpyDeviceToHost));
      CK(hipMemset(C1, 0, perC * items * sizeof(cx<float>)));
      const float t = timeit([&]() { hipLaunchKernelGGL((k_bgemm_glds<0, 0>), gr2, dim3(256), 0, 0, h); }, 2);
      check("glds ragged M", t);
    }
  }
  {
    auto f = [&]() { hipLaunchKernelGGL((k_bgemm<float, 1, 0, true, 1, 2>), grid, dim3(256), 0, 0, g); };
    const float t = timeit(f, 5);
    printf("  %-22s %.3f ms %.1f TF/s\n", "3M opA=H KS1 NBUF2", t, flops / t / 1e9);
  }
  {
    auto f = [&]() { hipLaunchKernelGGL((k_bgemm<float, 0, 1, true, 1, 2>), grid, dim3(256), 0, 0, g); };
    const float t = timeit(f, 5);
    printf("  %-22s %.3f ms %.1f TF/s\n", "3M opB=H KS1 NBUF2", t, flops / t / 1e9);
  }
  return 0;
}
