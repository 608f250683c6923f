// qoc_spline.hpp — spline parameterisation of the controls and the Ipopt constraint callbacks,
// batched over seeds (examples/ipopt_callbacks_exp.jl:13-14, 28, 33-51).
//
//   u_b    = transpose(Bs * c_b)            Bs: Nt x ns (column-major), c_b: ns x nu (column-major)
//   dJdc_b = Bs' * transpose(dJdu_b)
//   g_b    = [norm(c_b), norm(diff(c_b, dims=1))]  and  dg/dc (2 x nc, constraint-major)
//
// These are tiny (Nt x ns x nu per seed) and HBM/latency-bound; one thread per output element.
#pragma once
#include "qoc_common.hpp"

namespace qoc {

// u[b*nu*Nt + k*nu + j] = sum_s Bs[k + Nt s] c[b*ns*nu + s + ns j]
static __global__ void k_spline_u(int B, int Nt, int ns, int nu, const double* __restrict__ Bs, const double* __restrict__ c,
                           double* __restrict__ u) {
  const long long total = (long long)B * Nt * nu;
  for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < total; g += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(g % nu);
    const long long bk = g / nu;
    const int k = (int)(bk % Nt);
    const int b = (int)(bk / Nt);
    const double* cb = c + (size_t)b * ns * nu + (size_t)ns * j;
    double acc = 0.0;
    for (int s = 0; s < ns; ++s) acc += Bs[k + (size_t)Nt * s] * cb[s];
    u[g] = acc;
  }
}

// dJdc[b*ns*nu + s + ns j] = sum_k Bs[k + Nt s] dJdu[b*nu*Nt + k*nu + j]   (one wave per output)
static __global__ void k_spline_grad(int B, int Nt, int ns, int nu, const double* __restrict__ Bs,
                              const double* __restrict__ dJdu, double* __restrict__ dJdc) {
  const int lane = threadIdx.x & 63;
  const long long total = (long long)B * ns * nu;
  const long long w0 = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long o = w0; o < total; o += nw) {
    const int s = (int)(o % ns);
    const long long bj = o / ns;
    const int j = (int)(bj % nu);
    const int b = (int)(bj / nu);
    const double* gb = dJdu + (size_t)b * nu * Nt;
    double acc = 0.0;
    for (int k = lane; k < Nt; k += 64) acc += Bs[k + (size_t)Nt * s] * gb[(size_t)k * nu + j];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) dJdc[o] = acc;
  }
}

// g[b*2 + 0] = ||c_b||_2, g[b*2 + 1] = ||diff(c_b, dims=1)||_F and the Jacobian
// gjac[b*2*nc + 0*nc + i] = c_i / g0,  gjac[b*2*nc + nc + (s + ns j)] = (d_s - d_{s+1}) / g1
// with d_s = c[s, j] - c[s-1, j] for 1 <= s < ns and d_0 = d_ns = 0.  A zero norm has a zero
// gradient (the subgradient Zygote's norm rrule returns at 0).  One workgroup per seed.
static __global__ void k_spline_constraints(int ns, int nu, const double* __restrict__ c, double* __restrict__ g,
                                     double* __restrict__ gjac) {
  __shared__ double red[8];
  const int b = blockIdx.x, nc = ns * nu;
  const double* cb = c + (size_t)b * nc;
  double s0 = 0.0, s1 = 0.0;
  for (int i = threadIdx.x; i < nc; i += blockDim.x) {
    const int s = i % ns;
    s0 += cb[i] * cb[i];
    if (s > 0) {
      const double d = cb[i] - cb[i - 1];
      s1 += d * d;
    }
  }
  const double g0 = sqrt(block_sum(s0, red));
  const double g1 = sqrt(block_sum(s1, red));
  if (threadIdx.x == 0) {
    g[2 * b] = g0;
    g[2 * b + 1] = g1;
  }
  if (!gjac) return;
  double* jb = gjac + (size_t)b * 2 * nc;
  for (int i = threadIdx.x; i < nc; i += blockDim.x) {
    const int s = i % ns;
    jb[i] = g0 > 0.0 ? cb[i] / g0 : 0.0;
    const double dl = s > 0 ? cb[i] - cb[i - 1] : 0.0;
    const double dr = s + 1 < ns ? cb[i + 1] - cb[i] : 0.0;
    jb[nc + i] = g1 > 0.0 ? (dl - dr) / g1 : 0.0;
  }
}

}  // namespace qoc
