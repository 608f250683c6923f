// LDS-DMA image check for k_bgemm_glds' two operand layouts (diagnostic):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/glds_probe tools/glds_probe.hip
// Fills one 64 x 16 image of a 64 x 64 complex matrix (element (r, k) = (r, k)) through bgg_piece / bgg_dma and reads
// every (r, k) back through bgg_off; prints the number of mismatches per layout.
#include <cstdio>
#include <vector>
#include <cmath>
#include "../quantumoptimalcontrol.jl_amd/csrc/qoc_bgemm.hpp"
using namespace qoc;

template <bool KR>
__global__ __launch_bounds__(256) void k_probe(const cx<float>* M, int ld, float2* out) {
  __shared__ __attribute__((aligned(16))) float lds[4096];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int i = tid; i < 4096; i += 256) lds[i] = -1.0f;
  __syncthreads();
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) float*)lds;
  for (int h = 0; h < 2; ++h) {
    int r, k;
    bgg_piece<KR>(2 * wave + h, lane, r, k);
    const long long src = KR ? r + (long long)ld * k : k + (long long)ld * r;
    const unsigned q = (unsigned)__builtin_amdgcn_readfirstlane(2 * wave + h);
    bgg_dma(M + src, lds0 + q * 1024);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int e = tid; e < 1024; e += 256) {
    const int r = e / 16, k = e % 16;
    out[e] = *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(lds) + bgg_off<KR>(r, k));
  }
}

int main() {
  const int n = 64;
  for (int kr = 0; kr < 2; ++kr) {
    // KR: stored with rows contiguous (element (r, k) at r + n k); RK: k contiguous (at k + n r)
    std::vector<cx<float>> h((size_t)n * n);
    for (int r = 0; r < n; ++r)
      for (int k = 0; k < n; ++k) h[kr ? r + (size_t)n * k : k + (size_t)n * r] = {(float)r, (float)k};
    cx<float>* d;
    float2* o;
    (void)hipMalloc(&d, h.size() * 8);
    (void)hipMalloc(&o, 1024 * 8);
    (void)hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    if (kr) hipLaunchKernelGGL(k_probe<true>, dim3(1), dim3(256), 0, 0, d, n, o);
    else hipLaunchKernelGGL(k_probe<false>, dim3(1), dim3(256), 0, 0, d, n, o);
    std::vector<float2> out(1024);
    (void)hipMemcpy(out.data(), o, 1024 * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int e = 0; e < 1024; ++e) {
      const int r = e / 16, k = e % 16;
      if (out[e].x != r || out[e].y != k) {
        if (bad < 8) printf("  %s (r %d, k %d) read (%g, %g)\n", kr ? "KR" : "RK", r, k, out[e].x, out[e].y);
        ++bad;
      }
    }
    printf("%s: %d mismatches of 1024\n", kr ? "KR" : "RK", bad);
    (void)hipFree(d);
    (void)hipFree(o);
  }
  // the GEMM against k_bgemm on one item per (M, K, N) shape and op pair
  auto gemm_case = [&](int M, int K, int NC, int opa, int opb) {
    const int ra = opa ? K : M, ca = opa ? M : K, rb = opb ? NC : K, cb = opb ? K : NC;
    std::vector<cx<float>> ha((size_t)ra * ca), hb((size_t)rb * cb);
    for (size_t i = 0; i < ha.size(); ++i) ha[i] = {(float)((i * 37) % 17) / 17.0f - 0.5f, (float)((i * 11) % 13) / 13.0f - 0.5f};
    for (size_t i = 0; i < hb.size(); ++i) hb[i] = {(float)((i * 29) % 19) / 19.0f - 0.5f, (float)((i * 7) % 23) / 23.0f - 0.5f};
    cx<float>*A, *B, *C0, *C1;
    (void)hipMalloc(&A, ha.size() * 8);
    (void)hipMalloc(&B, hb.size() * 8);
    (void)hipMalloc(&C0, (size_t)M * NC * 8);
    (void)hipMalloc(&C1, (size_t)M * NC * 8);
    (void)hipMemcpy(A, ha.data(), ha.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(B, hb.data(), hb.size() * 8, hipMemcpyHostToDevice);
    GemmArgs g{};
    g.A.p = A; g.A.inner = (long long)ha.size();
    g.B.p = B; g.B.inner = (long long)hb.size();
    g.M = M; g.K = K; g.Ncol = NC; g.nitems = 1; g.alpha1 = 1.0;
    g.tiles_m = (M + 63) / 64;
    g.tiles = g.tiles_m * ((NC + 63) / 64);
    GemmArgs g0 = g;
    g0.C1.p = C0; g0.C1.inner = (long long)M * NC;
    g.C1.p = C1; g.C1.inner = (long long)M * NC;
    const dim3 grid(g.tiles);
#define QOC_PAIR(OA, OB)                                                                  \
  if (opa == OA && opb == OB) {                                                           \
    hipLaunchKernelGGL((k_bgemm<float, OA, OB, true, 1, 2>), grid, dim3(256), 0, 0, g0);  \
    hipLaunchKernelGGL((k_bgemm_glds<OA, OB>), grid, dim3(256), 0, 0, g);                 \
  }
    QOC_PAIR(0, 0) QOC_PAIR(1, 0) QOC_PAIR(0, 1) QOC_PAIR(1, 1)
#undef QOC_PAIR
    std::vector<cx<float>> c0((size_t)M * NC), c1((size_t)M * NC);
    (void)hipMemcpy(c0.data(), C0, c0.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(c1.data(), C1, c1.size() * 8, hipMemcpyDeviceToHost);
    double md = 0;
    int first = -1;
    for (size_t i = 0; i < c0.size(); ++i) {
      const double d = fabs(c0[i].r - c1[i].r) + fabs(c0[i].i - c1[i].i);
      if (d > 1e-3 && first < 0) first = (int)i;
      md = fmax(md, d);
    }
    printf("gemm M %d K %d N %d op %d%d: maxdiff %.3g", M, K, NC, opa, opb, md);
    if (first >= 0) printf("  first bad (row %d, col %d): ref (%g, %g) glds (%g, %g)", first % M, first / M,
                           c0[first].r, c0[first].i, c1[first].r, c1[first].i);
    printf("\n");
    (void)hipFree(A); (void)hipFree(B); (void)hipFree(C0); (void)hipFree(C1);
  };
  for (int opa = 0; opa < 2; ++opa)
    for (int opb = 0; opb < 2; ++opb)
      for (int K : {16, 32, 48, 64, 256}) gemm_case(64, K, 64, opa, opb);
  gemm_case(256, 256, 256, 0, 0);
  return 0;
}
