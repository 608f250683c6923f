// Empirical operand layout of v_mfma_f64_4x4x4_4b_f64: lane bits split into three 2-bit fields
// (block b and the two matrix indices) in some order for A (b, m, k), B (b, k, n) and D (b, m, n).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma4_layout tools/mfma4_layout.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void k(const double* a, const double* b, double* d) {
  const int l = threadIdx.x;
  d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 0, 0, 0);
}

static int field(int lane, int pos) { return (lane >> (2 * pos)) & 3; }

int main() {
  double ha[64], hb[64], hd[64];
  for (int l = 0; l < 64; ++l) {
    ha[l] = std::sin(1.0 + 0.37 * l);
    hb[l] = std::cos(2.0 + 0.71 * l);
  }
  double *da, *db, *dd;
  (void)hipMalloc(&da, 512);
  (void)hipMalloc(&db, 512);
  (void)hipMalloc(&dd, 512);
  (void)hipMemcpy(da, ha, 512, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dd);
  (void)hipMemcpy(hd, dd, 512, hipMemcpyDeviceToHost);
  // permutations of 3 fields: perm[p] = bit-field position of (block, first index, second index)
  const int P[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  int found = 0;
  for (int pa = 0; pa < 6; ++pa)
    for (int pb = 0; pb < 6; ++pb)
      for (int pd = 0; pd < 6; ++pd) {
        double A[4][4][4], B[4][4][4];  // [blk][row][col]
        for (int l = 0; l < 64; ++l) {
          A[field(l, P[pa][0])][field(l, P[pa][1])][field(l, P[pa][2])] = ha[l];  // (b, m, k)
          B[field(l, P[pb][0])][field(l, P[pb][1])][field(l, P[pb][2])] = hb[l];  // (b, k, n)
        }
        double err = 0;
        for (int l = 0; l < 64; ++l) {
          const int bl = field(l, P[pd][0]), m = field(l, P[pd][1]), n = field(l, P[pd][2]);
          double s = 0;
          for (int kk = 0; kk < 4; ++kk) s += A[bl][m][kk] * B[bl][kk][n];
          err = std::fmax(err, std::fabs(s - hd[l]));
        }
        if (err < 1e-12) {
          printf("match: A (b,m,k) at lane-bit fields (%d,%d,%d); B (b,k,n) at (%d,%d,%d); D (b,m,n) at (%d,%d,%d)\n",
                 P[pa][0], P[pa][1], P[pa][2], P[pb][0], P[pb][1], P[pb][2], P[pd][0], P[pd][1], P[pd][2]);
          ++found;
        }
      }
  printf("%d layout(s) found (field f = lane bits [2f, 2f+1])\n", found);
  return 0;
}
