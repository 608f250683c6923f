// qoc_bgemm.hpp — kernels of the large-N (HBM-resident) path: batched complex GEMM on MFMA with a
// fused multi-term epilogue, plus the element-wise and reduction kernels around it.
//
// Used when N exceeds the LDS-resident envelope of k_expm / k_chain_* (e.g. the synthetic N = 256
// fp32 configuration).  Everything is a batch of independent complex
// matrices in the engine's HBM layout (column-major, interleaved re/im).  A batch item locates
// each operand through an affine "unit map" (Opd), so the same GEMM serves
//   - per-slice Padé products   (item = slice in a chunk, workspace stride),
//   - chain steps               (item = seed b at fixed slice k: U[b,k], x[b,k]),
//   - gradient products         (item = slice unit b*Nt+k: x_k, λ_{k+1} live at (Nt+1)-strided slots).
#pragma once
#include "qoc_common.hpp"

namespace qoc {

// Operand address: base + (v / per) * outer + (v % per) * inner, v = item + u0 (per <= 0: v * inner).
struct Opd {
  const void* p = nullptr;
  long long outer = 0, inner = 0;
  int per = 0, u0 = 0;
};

template <typename T>
__device__ __forceinline__ const cx<T>* opd_ptr(const Opd& o, int item) {
  const long long v = (long long)item + o.u0;
  long long off;
  if (o.per > 0) {
    const long long q = v / o.per;
    off = q * o.outer + (v - q * o.per) * o.inner;
  } else {
    off = v * o.inner;
  }
  return reinterpret_cast<const cx<T>*>(o.p) + off;
}

constexpr int BG_BM = 64, BG_BN = 64, BG_THREADS = 256;

// C1 = alpha1 * op(A) op(B) + sum_t w1[t] Y_t + gamma1 I
// C2 = alpha2 * op(A) op(B) + sum_t w2[t] Y_t + gamma2 I          (optional)
// C3 = alpha3 * op(A) op(B) + sum_t w3[t] Y_t + gamma3 I          (optional)
// sumsq (optional): sumsq[item] += ||C1||_F^2 (Newton-Schulz residual bound, ||R||_2 <= ||R||_F).
struct GemmArgs {
  Opd A, B, C1, C2, C3, Y[3];
  int nY;
  int M, K, Ncol;  // op(A): M x K, op(B): K x Ncol
  int nitems, tiles_m, tiles;
  double alpha1, alpha2, alpha3, gamma1, gamma2, gamma3;
  double w1[3], w2[3], w3[3];
  double* sumsq;
  // MODE 1 (generator combine, LDS-resident-N gradient): op(B)(k, col) = Bsrc[k mod kb, col] * s(k / kb, col)
  //   with s(0) = 1, s(j) = uc[(b Nt + t) nu + j - 1] for the slice (b, t) of column col (t < Nt, else 0);
  //   Bsrc has leading dimension kb.  Columns map to slices as col = ((b sps) + t) m + i.
  // MODE 2 (fused contraction): C is not stored; instead
  //   dot[(b Nt + t) nu + row / kb] += Re(conj(Wd[row mod kb, col]) C[row, col])   (t < Nt).
  const double* uc;
  int kb, cm, sps, cNt, cnu;
  double* dot;
  Opd Wd;
};

// Both operands are staged in LDS as [row or col][k] planes (re / im) with k contiguous.  K is
// permuted inside each 16-deep sub-slab: at MFMA step t lane l multiplies k = 4 (l >> 4) + t, so a
// lane's four k values are adjacent and one 16-byte LDS read (per 4 floats) fetches its fragment
// for the sub-slab.  A slab is KS sub-slabs (BK = 16 KS); NBUF = 2 double-buffers the
// LDS image (one barrier per slab), NBUF = 1 uses one image and two barriers per slab but a smaller
// LDS footprint (more workgroups per CU).
// Bank layout.  fp32, KS = 1: rows of 16 floats (64 B, no padding) with the four 16-byte chunks of row r
// XOR-swizzled by (r >> 1) & 3.  A ds_read_b128 lane group ({0-3,12-15,20-27}, ... : rows li, chunk kq =
// l >> 4) then touches 16 distinct 16-byte slots of the 256-byte bank window, and the ds_write_b128 groups (8
// contiguous lanes, 128-byte window) of both store layouts do too — conflict-free both ways.  (The previous
// 16-byte row padding left 2-way conflicts in every read group: ~43 % of the LDS-active cycles in PMC.)
// Otherwise rows are padded by 16 bytes.
template <typename T, int KS>
struct BgLay {
  static constexpr int BK = 16 * KS;
  static constexpr bool SWZ = KS == 1 && sizeof(T) == 4;
  static constexpr int LDK = SWZ ? BK : BK + 16 / (int)sizeof(T);  // row stride in elements
  static constexpr int PLANE = BG_BM * LDK;
  // element offset of the 4-element chunk `ch` (k = 4 ch .. 4 ch + 3 of the slab) of row r
  static __device__ __forceinline__ int off(int r, int ch) { return r * LDK + 4 * (SWZ ? (ch ^ ((r >> 1) & 3)) : ch); }
};

template <typename T>
struct Vec4;
template <>
struct Vec4<float> {
  typedef float type __attribute__((ext_vector_type(4)));
};
template <>
struct Vec4<double> {
  typedef double type __attribute__((ext_vector_type(4)));
};

// Stage one 64 x BK slab of an operand into registers; element (r, k) with r < R, k < K.
// KCONT: memory contiguous along k (address k + ld * r), else along r (address r + ld * k).
// Thread t owns one row/col r and, per sub-slab j, the four consecutive k of group kg.
template <typename T, bool KCONT, bool CONJ, int KS>
__device__ __forceinline__ void bg_load(const cx<T>* __restrict__ base, long long ld, int r0, int k0, int R, int K,
                                        int tid, typename Vec4<T>::type (&re)[KS], typename Vec4<T>::type (&im)[KS]) {
  const int r = KCONT ? (tid >> 2) : (tid & 63);
  const int gr = r0 + r;
#pragma unroll
  for (int j = 0; j < KS; ++j) {
    const int kg = (KCONT ? (tid & 3) : (tid >> 6)) + 4 * j;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int gk = k0 + 4 * kg + t;
      const bool ok = gr < R && gk < K;
      const long long off = KCONT ? (long long)(ok ? gk : 0) + ld * (ok ? gr : 0)
                                  : (long long)(ok ? gr : 0) + ld * (ok ? gk : 0);
      const cx<T> v = base[off];
      re[j][t] = ok ? v.r : T(0);
      im[j][t] = ok ? (CONJ ? -v.i : v.i) : T(0);
    }
  }
}

template <typename T, bool KCONT, int KS>
__device__ __forceinline__ void bg_store(T* __restrict__ pre, T* __restrict__ pim, int tid,
                                         const typename Vec4<T>::type (&re)[KS],
                                         const typename Vec4<T>::type (&im)[KS]) {
  using L = BgLay<T, KS>;
  using V = typename Vec4<T>::type;
  const int r = KCONT ? (tid >> 2) : (tid & 63);
#pragma unroll
  for (int j = 0; j < KS; ++j) {
    const int kg = (KCONT ? (tid & 3) : (tid >> 6)) + 4 * j;
    *reinterpret_cast<V*>(pre + L::off(r, kg)) = re[j];
    *reinterpret_cast<V*>(pim + L::off(r, kg)) = im[j];
  }
}

// OPA: 0 -> op(A) = A (stored M x K, contiguous along rows); 1 -> A^H (stored K x M, contiguous along k)
// OPB: 0 -> op(B) = B (stored K x Ncol, contiguous along k); 1 -> B^H (stored Ncol x K, contiguous along cols)
// M3: complex product with 3 real MFMAs (Gauss): P1 = ar br, P2 = ai bi, P3 = (ar+ai)(br+bi);
// Re = P1 - P2, Im = P3 - P1 - P2.  25 % fewer MFMAs than the 4-product form; the imaginary part's
// rounding error grows to ~2 eps |a||b| (cancellation in P3 - P1 - P2), well inside the fp32/fp64
// parity tolerances.
template <typename T, int OPA, int OPB, bool M3 = true, int KS = 1, int NBUF = 2, int MODE = 0>
__global__ __launch_bounds__(BG_THREADS) void k_bgemm(GemmArgs g) {
  using MFT = MF<T>;
  using v4 = typename MFT::v4;
  using V = typename Vec4<T>::type;
  using L = BgLay<T, KS>;
  // [buf][A re, A im, B re, B im][64][LDK]
  __shared__ __attribute__((aligned(16))) T lds[NBUF * 4 * L::PLANE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // XCD-aware order: consecutive workgroups are dispatched round-robin over the 8 XCDs; give each
  // XCD a contiguous range of (item, tile) so that one item's tiles share an L2.
  const int Lb = blockIdx.x;
  const int total = g.nitems * g.tiles;
  const int lin = (total & 7) == 0 ? (Lb & 7) * (total >> 3) + (Lb >> 3) : Lb;
  const int item = lin / g.tiles, tile = lin - item * g.tiles;
  const int tm = tile % g.tiles_m, tn = tile / g.tiles_m;
  const int row0 = tm * BG_BM, col0 = tn * BG_BN;
  const cx<T>* Ab = opd_ptr<T>(g.A, item);
  const cx<T>* Bb = opd_ptr<T>(g.B, item);
  const int M = g.M, K = g.K, NC = g.Ncol;
  const long long ldA = OPA ? K : M, ldB = OPB ? NC : K;
  // MODE 1: the thread's B column (fixed across slabs) and its generator scales
  double us[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) us[q] = q == 0 ? 1.0 : 0.0;
  if (MODE == 1) {
    const int gc = col0 + (tid >> 2);
    if (gc < NC) {
      const int sl = gc / g.cm, b = sl / g.sps, t = sl - b * g.sps;
      if (t < g.cNt) {
        const double* up = g.uc + ((size_t)b * g.cNt + t) * g.cnu;
#pragma unroll
        for (int q = 1; q < 9; ++q) us[q] = q <= g.cnu ? up[q - 1] : 0.0;
      }
    }
  }
  // MODE 1 B operand: like bg_load<KCONT = true> (op0, contiguous along k) with the generator-block
  // scaling s(k / kb, col) (us[0] = 1); written inline so that us[] stays in registers.
#define QOC_BG_LOADB(K0)                                                                  \
  do {                                                                                    \
    if (MODE == 1) {                                                                      \
      const int gr_ = col0 + (tid >> 2);                                                  \
      _Pragma("unroll") for (int j_ = 0; j_ < KS; ++j_) {                                 \
        const int kg_ = (tid & 3) + 4 * j_;                                               \
        _Pragma("unroll") for (int t_ = 0; t_ < 4; ++t_) {                                \
          const int gk_ = (K0) + 4 * kg_ + t_;                                            \
          const bool ok_ = gr_ < NC && gk_ < K;                                           \
          const int blk_ = ok_ ? gk_ / g.kb : 0;                                          \
          const int kr_ = ok_ ? gk_ - blk_ * g.kb : 0;                                    \
          const cx<T> v_ = Bb[(long long)kr_ + (long long)g.kb * (ok_ ? gr_ : 0)];        \
          double sc_ = us[0];                                                             \
          _Pragma("unroll") for (int q_ = 1; q_ < 9; ++q_) sc_ = blk_ == q_ ? us[q_] : sc_; \
          sbr[j_][t_] = ok_ ? (T)(sc_ * v_.r) : T(0);                                     \
          sbi[j_][t_] = ok_ ? (T)(sc_ * v_.i) : T(0);                                     \
        }                                                                                 \
      }                                                                                   \
    } else {                                                                              \
      bg_load<T, OPB == 0, OPB == 1, KS>(Bb, ldB, col0, (K0), NC, K, tid, sbr, sbi);      \
    }                                                                                     \
  } while (0)

  V sar[KS], sai[KS], sbr[KS], sbi[KS];
  v4 cr[2][2], ci[2][2], cs[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      cr[x][y] = v4{0, 0, 0, 0};
      ci[x][y] = v4{0, 0, 0, 0};
      cs[x][y] = v4{0, 0, 0, 0};
    }
  const int wr = (wave & 1) * 32, wc = (wave >> 1) * 32;
  const int li = lane & 15, kq = lane >> 4;
  const int nslab = (K + L::BK - 1) / L::BK;
  bg_load<T, OPA == 1, OPA == 1, KS>(Ab, ldA, row0, 0, M, K, tid, sar, sai);
  QOC_BG_LOADB(0);
  if (NBUF == 2) {
    bg_store<T, OPA == 1, KS>(lds + 0 * L::PLANE, lds + 1 * L::PLANE, tid, sar, sai);
    bg_store<T, OPB == 0, KS>(lds + 2 * L::PLANE, lds + 3 * L::PLANE, tid, sbr, sbi);
    __syncthreads();
  }
  for (int s = 0; s < nslab; ++s) {
    const T* cur = lds + (NBUF == 2 ? (s & 1) : 0) * 4 * L::PLANE;
    if (NBUF == 1) {
      if (s > 0) __syncthreads();  // previous slab's fragment reads are done
      bg_store<T, OPA == 1, KS>(lds + 0 * L::PLANE, lds + 1 * L::PLANE, tid, sar, sai);
      bg_store<T, OPB == 0, KS>(lds + 2 * L::PLANE, lds + 3 * L::PLANE, tid, sbr, sbi);
      __syncthreads();
    }
    if (s + 1 < nslab) {
      bg_load<T, OPA == 1, OPA == 1, KS>(Ab, ldA, row0, (s + 1) * L::BK, M, K, tid, sar, sai);
      QOC_BG_LOADB((s + 1) * L::BK);
    }
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      V ar[2], ai[2], br[2], bi[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int o = L::off(wr + 16 * x + li, 4 * q + kq);
        ar[x] = *reinterpret_cast<const V*>(cur + 0 * L::PLANE + o);
        ai[x] = *reinterpret_cast<const V*>(cur + 1 * L::PLANE + o);
      }
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const int o = L::off(wc + 16 * y + li, 4 * q + kq);
        br[y] = *reinterpret_cast<const V*>(cur + 2 * L::PLANE + o);
        bi[y] = *reinterpret_cast<const V*>(cur + 3 * L::PLANE + o);
      }
      if (M3) {
        V as[2], bs[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) as[x] = ar[x] + ai[x];
#pragma unroll
        for (int y = 0; y < 2; ++y) bs[y] = br[y] + bi[y];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
              cr[x][y] = MFT::mma(ar[x][t], br[y][t], cr[x][y]);
              ci[x][y] = MFT::mma(ai[x][t], bi[y][t], ci[x][y]);
              cs[x][y] = MFT::mma(as[x][t], bs[y][t], cs[x][y]);
            }
        }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
              cr[x][y] = MFT::mma(ar[x][t], br[y][t], cr[x][y]);
              ci[x][y] = MFT::mma(ar[x][t], bi[y][t], ci[x][y]);
            }
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
              cr[x][y] = MFT::mma(-ai[x][t], bi[y][t], cr[x][y]);
              ci[x][y] = MFT::mma(ai[x][t], br[y][t], ci[x][y]);
            }
        }
      }
    }
    if (NBUF == 2) {
      if (s + 1 < nslab) {
        T* nxt = lds + ((s + 1) & 1) * 4 * L::PLANE;
        bg_store<T, OPA == 1, KS>(nxt + 0 * L::PLANE, nxt + 1 * L::PLANE, tid, sar, sai);
        bg_store<T, OPB == 0, KS>(nxt + 2 * L::PLANE, nxt + 3 * L::PLANE, tid, sbr, sbi);
      }
      __syncthreads();
    }
  }

#undef QOC_BG_LOADB
  if (MODE == 2) {
    // fused contraction: per (slice, j) partial sums of Re(conj(W) C) over this tile
    const cx<T>* Wb = opd_ptr<T>(g.Wd, item);
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int rbase = row0 + wr + 16 * x;
      const int jb = rbase / g.kb;
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const int col = col0 + wc + 16 * y + li;
        double acc[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rbase + MFT::drow(lane, i);
          if (row < M && col < NC) {
            double pr, pi;
            if (M3) {
              pr = (double)cr[x][y][i] - (double)ci[x][y][i];
              pi = (double)cs[x][y][i] - (double)cr[x][y][i] - (double)ci[x][y][i];
            } else {
              pr = cr[x][y][i];
              pi = ci[x][y][i];
            }
            const int j = row / g.kb;
            const cx<T> wv = Wb[(row - j * g.kb) + (size_t)g.kb * col];
            const double e = (double)wv.r * pr + (double)wv.i * pi;
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] += (j - jb == q) ? e : 0.0;
          }
        }
        int sl = 0, b = 0, t = 0;
        if (col < NC) {
          sl = col / g.cm;
          b = sl / g.sps;
          t = sl - b * g.sps;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          double v = acc[q];
          v += __shfl_xor(v, 16);
          v += __shfl_xor(v, 32);
          const int j = jb + q;
          if ((lane >> 4) == 0 && col < NC && t < g.cNt && j < g.cnu && j * g.kb < M && v != 0.0)
            atomicAdd(g.dot + ((size_t)b * g.cNt + t) * g.cnu + j, v);
        }
      }
    }
    return;
  }
  // ---- fused epilogue ----
  cx<T>* C1 = const_cast<cx<T>*>(opd_ptr<T>(g.C1, item));
  cx<T>* C2 = g.C2.p ? const_cast<cx<T>*>(opd_ptr<T>(g.C2, item)) : nullptr;
  cx<T>* C3 = g.C3.p ? const_cast<cx<T>*>(opd_ptr<T>(g.C3, item)) : nullptr;
  const cx<T>* Y0 = g.nY > 0 ? opd_ptr<T>(g.Y[0], item) : nullptr;
  const cx<T>* Y1 = g.nY > 1 ? opd_ptr<T>(g.Y[1], item) : nullptr;
  const cx<T>* Y2 = g.nY > 2 ? opd_ptr<T>(g.Y[2], item) : nullptr;
  double mx = 0.0;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int col = col0 + wc + 16 * y + li;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = row0 + wr + 16 * x + MFT::drow(lane, i);
        if (row < M && col < NC) {
          const size_t o = row + (size_t)M * col;
          double pr, pi;
          if (M3) {
            pr = (double)cr[x][y][i] - (double)ci[x][y][i];
            pi = (double)cs[x][y][i] - (double)cr[x][y][i] - (double)ci[x][y][i];
          } else {
            pr = cr[x][y][i];
            pi = ci[x][y][i];
          }
          double r1 = g.alpha1 * pr, i1 = g.alpha1 * pi;
          double r2 = g.alpha2 * pr, i2 = g.alpha2 * pi;
          double r3 = g.alpha3 * pr, i3 = g.alpha3 * pi;
#define QOC_EPI_Y(YP, t)                                        \
  if (YP) {                                                     \
    const cx<T> v = YP[o];                                      \
    r1 += g.w1[t] * v.r; i1 += g.w1[t] * v.i;                   \
    r2 += g.w2[t] * v.r; i2 += g.w2[t] * v.i;                   \
    r3 += g.w3[t] * v.r; i3 += g.w3[t] * v.i;                   \
  }
          QOC_EPI_Y(Y0, 0)
          QOC_EPI_Y(Y1, 1)
          QOC_EPI_Y(Y2, 2)
#undef QOC_EPI_Y
          if (row == col) {
            r1 += g.gamma1;
            r2 += g.gamma2;
            r3 += g.gamma3;
          }
          C1[o] = cx<T>{(T)r1, (T)i1};
          if (C2) C2[o] = cx<T>{(T)r2, (T)i2};
          if (C3) C3[o] = cx<T>{(T)r3, (T)i3};
          mx += r1 * r1 + i1 * i1;
        }
      }
    }
  if (g.sumsq) {
    for (int off = 32; off > 0; off >>= 1) mx += __shfl_xor(mx, off);
    if (lane == 0) atomicAdd(g.sumsq + item, mx);
  }
}

// ---------------------------------------------------------------------------------------------
// k_bgemm_glds: the fp32 MODE-0 product of k_bgemm (same GemmArgs, tiles, XCD order, epilogue) with its operand
// slabs staged by LDS-DMA (global_load_lds_dwordx4) three slabs deep.  k_bgemm stages each 16-deep slab through
// registers one slab ahead; at N = 256 the items a CU works on at once do not fit the XCD's L2, most slab loads come
// from HBM, and the waves waited for them at every slab (the MFMA pipe ~55 % busy by PMC).  Here the slab s + 2 is
// in flight while slab s is multiplied, with no registers held for it, and each wave waits with a counted vmcnt for
// its own DMA pieces of slab s + 1 only, followed by a raw s_barrier (a __syncthreads would drain every DMA).
//
// LDS image per stage: A and B slabs of 64 "rows" (A: rows of op(A); B: columns of op(B)) x 16 k, complex
// interleaved (8 B), 8 KB each.  The DMA writes 16 B per lane at a lane-linear position, so each image takes the
// layout in which 16 B are contiguous in HBM, with the XOR swizzle on the source address:
//   KR (memory contiguous along the row: A, or B^H):  (r, k) at k*512 + ((r/16 ^ k&1) * 128) + (r%16)*8
//   RK (memory contiguous along k: A^H, or B):        (r, k) at r*128 + (((k/2) ^ ((r/2)&7)) * 16) + (k&1)*8
// Fragment reads are ds_read_b64 (one complex): lane (i = l%16, kq = l/16) at MFMA step t reads (row 16x + i,
// k = 4t + kq).  The 32 lanes of one LDS cycle then cover all 64 banks once in both layouts.
// Requirements (bgemm_glds_ok): T = float, K % 16 == 0, M and Ncol even (a 16-byte piece is two elements).
constexpr int BGG_STAGE_FLOATS = 2 * 64 * 16 * 2;  // A + B, complex fp32
template <bool KR>
__device__ __forceinline__ int bgg_off(int r, int k) {  // byte offset of (r, k) in an operand image
  return KR ? k * 512 + (((r >> 4) ^ (k & 1)) << 7) + ((r & 15) << 3)
            : r * 128 + ((((k >> 1) ^ ((r >> 1) & 7))) << 4) + ((k & 1) << 3);
}
// the (row, k) of the first of the two elements lane j of DMA piece q (0..7) writes
template <bool KR>
__device__ __forceinline__ void bgg_piece(int q, int j, int& r, int& k) {
  if (KR) {
    k = 2 * q + (j >> 5);
    r = 16 * (((j >> 3) & 3) ^ (k & 1)) + 2 * (j & 7);
  } else {
    r = 8 * q + (j >> 3);
    k = 2 * ((j & 7) ^ ((r >> 1) & 7));
  }
}
// One DMA piece: 16 B per lane from src (per lane) to LDS byte address lds_base + 16 lane (lds_base wave-uniform).
// Inline asm rather than the builtin: for the builtin hipcc inserts vmcnt(0) before the next ds_read of the (one)
// LDS array, which would drain the slabs kept in flight; the waits are counted by hand (k_bgemm_glds).  M0 is set
// and restored in the same statement.
__device__ __forceinline__ void bgg_dma(const void* src, unsigned lds_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_base)
               : "memory");
}

// NS LDS stages: 2 (the default: slab s + 1 in flight while s is multiplied, 32 KB, four workgroups per CU) or 3
// (s + 2 in flight, 48 KB, three per CU).  Microbench (profiles/bgemm_bench_r05g.txt): 2 stages 1.360 vs 1.389 ms
// at 1260 items, 0.131 vs 0.134 ms at 128 (the chain GEMMs' size).
template <int OPA, int OPB, int NS = 2>
__global__ __launch_bounds__(BG_THREADS) void k_bgemm_glds(GemmArgs g) {
  static_assert(NS == 2 || NS == 3, "two or three stages");
  constexpr int BGG_STAGES = NS;
  using MFT = MF<float>;
  using v4 = typename MFT::v4;
  constexpr bool KRA = OPA == 0, KRB = OPB == 1;  // layouts of the A and B images
  __shared__ __attribute__((aligned(16))) float lds[BGG_STAGES * BGG_STAGE_FLOATS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int Lb = blockIdx.x;
  const int total = g.nitems * g.tiles;
  const int lin = (total & 7) == 0 ? (Lb & 7) * (total >> 3) + (Lb >> 3) : Lb;
  const int item = lin / g.tiles, tile = lin - item * g.tiles;
  const int tm = tile % g.tiles_m, tn = tile / g.tiles_m;
  const int row0 = tm * BG_BM, col0 = tn * BG_BN;
  const cx<float>* Ab = opd_ptr<float>(g.A, item);
  const cx<float>* Bb = opd_ptr<float>(g.B, item);
  const int M = g.M, K = g.K, NC = g.Ncol;
  const long long ldA = OPA ? K : M, ldB = OPB ? NC : K;
  // this wave's two DMA pieces per operand (q = 2 wave + h): per-lane source element at slab 0, and the per-slab step
  long long srcA[2], srcB[2];
  const long long stepA = KRA ? 16 * ldA : 16, stepB = KRB ? 16 * ldB : 16;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    int r, k;
    bgg_piece<KRA>(2 * wave + h, lane, r, k);
    // rows past M: any valid row (their outputs are not stored); KR pieces hold the row pair (r, r + 1), r even
    const int gr = min(row0 + r, KRA ? M - 2 : M - 1);
    srcA[h] = KRA ? gr + ldA * k : k + ldA * gr;
    bgg_piece<KRB>(2 * wave + h, lane, r, k);
    const int gc = min(col0 + r, KRB ? NC - 2 : NC - 1);
    srcB[h] = KRB ? gc + ldB * k : k + ldB * gc;
  }
  const int nslab = K / 16;
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) float*)lds;
  auto issue = [&](int s) __attribute__((always_inline)) {
    const unsigned st = lds0 + (unsigned)((s % BGG_STAGES) * BGG_STAGE_FLOATS * 4);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned q = (unsigned)__builtin_amdgcn_readfirstlane(2 * wave + h);
      bgg_dma(Ab + srcA[h] + s * stepA, st + q * 1024);
      bgg_dma(Bb + srcB[h] + s * stepB, st + 8192 + q * 1024);
    }
  };
  v4 cr[2][2], ci[2][2], cs[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      cr[x][y] = v4{0, 0, 0, 0};
      ci[x][y] = v4{0, 0, 0, 0};
      cs[x][y] = v4{0, 0, 0, 0};
    }
  const int wr = (wave & 1) * 32, wc = (wave >> 1) * 32;
  const int li = lane & 15, kq = lane >> 4;
  // fragment byte offsets in an image at step t = 0 (step t adds 4t to k: KR +2048 B, RK via the slot XOR)
  issue(0);
  if (NS == 3 && nslab > 1) issue(1);
  if (NS == 3 && nslab > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int s = 0; s < nslab; ++s) {
    if (s + NS - 1 < nslab) issue(s + NS - 1);
    const char* cur = reinterpret_cast<const char*>(lds + (s % BGG_STAGES) * BGG_STAGE_FLOATS);
    const char* curB = cur + 8192;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = 4 * t + kq;
      float ar[2], ai[2], br[2], bi[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const float2 v = *reinterpret_cast<const float2*>(cur + bgg_off<KRA>(wr + 16 * x + li, k));
        ar[x] = v.x;
        ai[x] = OPA ? -v.y : v.y;
      }
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const float2 v = *reinterpret_cast<const float2*>(curB + bgg_off<KRB>(wc + 16 * y + li, k));
        br[y] = v.x;
        bi[y] = OPB ? -v.y : v.y;
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          cr[x][y] = MFT::mma(ar[x], br[y], cr[x][y]);
          ci[x][y] = MFT::mma(ai[x], bi[y], ci[x][y]);
          cs[x][y] = MFT::mma(ar[x] + ai[x], br[y] + bi[y], cs[x][y]);
        }
    }
    // slab s + 1 landed (this wave's pieces; slab s + 2's stay in flight), every read of slab s done, then the
    // barrier: after it slab s + 1 is readable and slab s's buffer may be refilled (by slab s + 3)
    if (NS == 3 && s + 2 < nslab) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // ---- epilogue (k_bgemm MODE 0) ----
  cx<float>* C1 = const_cast<cx<float>*>(opd_ptr<float>(g.C1, item));
  cx<float>* C2 = g.C2.p ? const_cast<cx<float>*>(opd_ptr<float>(g.C2, item)) : nullptr;
  cx<float>* C3 = g.C3.p ? const_cast<cx<float>*>(opd_ptr<float>(g.C3, item)) : nullptr;
  const cx<float>* Y0 = g.nY > 0 ? opd_ptr<float>(g.Y[0], item) : nullptr;
  const cx<float>* Y1 = g.nY > 1 ? opd_ptr<float>(g.Y[1], item) : nullptr;
  const cx<float>* Y2 = g.nY > 2 ? opd_ptr<float>(g.Y[2], item) : nullptr;
  double mx = 0.0;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int col = col0 + wc + 16 * y + li;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = row0 + wr + 16 * x + MFT::drow(lane, i);
        if (row < M && col < NC) {
          const size_t o = row + (size_t)M * col;
          const double pr = (double)cr[x][y][i] - (double)ci[x][y][i];
          const double pi = (double)cs[x][y][i] - (double)cr[x][y][i] - (double)ci[x][y][i];
          double r1 = g.alpha1 * pr, i1 = g.alpha1 * pi;
          double r2 = g.alpha2 * pr, i2 = g.alpha2 * pi;
          double r3 = g.alpha3 * pr, i3 = g.alpha3 * pi;
#define QOC_EPI_Y(YP, t)                                        \
  if (YP) {                                                     \
    const cx<float> v = YP[o];                                  \
    r1 += g.w1[t] * v.r; i1 += g.w1[t] * v.i;                   \
    r2 += g.w2[t] * v.r; i2 += g.w2[t] * v.i;                   \
    r3 += g.w3[t] * v.r; i3 += g.w3[t] * v.i;                   \
  }
          QOC_EPI_Y(Y0, 0)
          QOC_EPI_Y(Y1, 1)
          QOC_EPI_Y(Y2, 2)
#undef QOC_EPI_Y
          if (row == col) {
            r1 += g.gamma1;
            r2 += g.gamma2;
            r3 += g.gamma3;
          }
          C1[o] = cx<float>{(float)r1, (float)i1};
          if (C2) C2[o] = cx<float>{(float)r2, (float)i2};
          if (C3) C3[o] = cx<float>{(float)r3, (float)i3};
          mx += r1 * r1 + i1 * i1;
        }
      }
    }
  if (g.sumsq) {
    for (int off = 32; off > 0; off >>= 1) mx += __shfl_xor(mx, off);
    if (lane == 0) atomicAdd(g.sumsq + item, mx);
  }
}

// 2-norm bound of every A_k of a chunk for skew-Hermitian generators: ||A_k||_2 <= Σ_j |c_jk| ρ_j with c_0 = 1,
// c_j = u_jk, ρ_j = ||A_j||_2 (the spectral radius, A_j normal) -> atomic max in bmax (one thread per unit).
struct SpecBound {
  double rho[9];
};
static __global__ void k_spec_bound(int nu, long long unit0, int cnt, const double* __restrict__ u, const SpecBound sb,
                             unsigned long long* __restrict__ bmax) {
  double best = 0.0;
  for (int it = blockIdx.x * blockDim.x + threadIdx.x; it < cnt; it += gridDim.x * blockDim.x) {
    double b = sb.rho[0];
    for (int j = 0; j < nu; ++j) b += fabs(u[(unit0 + it) * nu + j]) * sb.rho[j + 1];
    best = fmax(best, b);
  }
  for (int off = 32; off > 0; off >>= 1) best = fmax(best, __shfl_xor(best, off));
  if ((threadIdx.x & 63) == 0) atomicMax(bmax, (unsigned long long)__double_as_longlong(best));
}

// ---------------------------------------------------------------------------------------------
// Element-wise kernels
// ---------------------------------------------------------------------------------------------

// Out_item = sum_{t < nt} w_t Y_t,item + dI * I   (rows x cols per item, leading dimension rows);
// optionally a second output Out2 = sum_t w2_t Y_t + dI2 * I from the same reads.
struct LinArgs {
  Opd out, out2, Y[4];
  double w[4], w2[4];
  int nt, rows, cols, nitems;
  double dI, dI2;
};

template <typename T>
__global__ void k_lincomb(LinArgs a) {
  const size_t per = (size_t)a.rows * a.cols;
  const size_t total = per * a.nitems;
  for (size_t gi = blockIdx.x * (size_t)blockDim.x + threadIdx.x; gi < total; gi += (size_t)gridDim.x * blockDim.x) {
    const int it = (int)(gi / per);
    const size_t e = gi - (size_t)it * per;
    double r = 0, im = 0, r2 = 0, im2 = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < a.nt) {
        const cx<T> v = opd_ptr<T>(a.Y[t], it)[e];
        r += a.w[t] * v.r;
        im += a.w[t] * v.i;
        r2 += a.w2[t] * v.r;
        im2 += a.w2[t] * v.i;
      }
    }
    const bool diag = (int)(e % a.rows) == (int)(e / a.rows);
    if (diag) {
      r += a.dI;
      r2 += a.dI2;
    }
    const_cast<cx<T>*>(opd_ptr<T>(a.out, it))[e] = cx<T>{(T)r, (T)im};
    if (a.out2.p) const_cast<cx<T>*>(opd_ptr<T>(a.out2, it))[e] = cx<T>{(T)r2, (T)im2};
  }
}

// A_unit = A0 + sum_j u[unit, j] A_j for units [unit0, unit0 + count) -> out (count x N x N), and (nmax set) the
// 1-norm (max column sum of |a_ij|) of each, max-reduced into *nmax.  One workgroup per slice; each wave takes
// batches of FN_C whole columns at a time, FN_R rows per lane per batch, so that FN_C * FN_R independent loads of
// each generator are in flight per lane (one column per wave-iteration left every load's L2 round trip exposed:
// ~0.8 TB/s of writes at N = 256).  The atomic max is skipped when the running value is already larger.
constexpr int FN_C = 4, FN_R = 4;
template <typename T>
__global__ __launch_bounds__(256) void k_form_norm(int N, int nu, long long unit0, const cx<T>* __restrict__ Agen,
                                                   const double* __restrict__ u, cx<T>* __restrict__ out,
                                                   unsigned long long* __restrict__ nmax) {
  const int it = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t NN = (size_t)N * N;
  const long long unit = unit0 + it;
  T uj[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) uj[j] = j < nu ? (T)u[unit * nu + j] : T(0);
  cx<T>* ob = out + (size_t)it * NN;
  double best = 0.0;
  for (int c0 = wave * FN_C; c0 < N; c0 += 4 * FN_C) {
    double s[FN_C];
#pragma unroll
    for (int x = 0; x < FN_C; ++x) s[x] = 0.0;
    for (int r0 = 0; r0 < N; r0 += 64 * FN_R) {
      size_t e[FN_C][FN_R];
      bool ok[FN_C][FN_R];
      cx<T> a[FN_C][FN_R];
#pragma unroll
      for (int x = 0; x < FN_C; ++x)
#pragma unroll
        for (int q = 0; q < FN_R; ++q) {
          const int r = r0 + lane + 64 * q, c = c0 + x;
          ok[x][q] = r < N && c < N;
          e[x][q] = ok[x][q] ? r + (size_t)N * c : 0;
          a[x][q] = Agen[e[x][q]];
        }
      for (int j = 0; j < nu && j < 8; ++j) {
        const cx<T>* Aj = Agen + (size_t)(j + 1) * NN;
        T w = uj[0];
#pragma unroll
        for (int q = 1; q < 8; ++q) w = j == q ? uj[q] : w;
#pragma unroll
        for (int x = 0; x < FN_C; ++x)
#pragma unroll
          for (int q = 0; q < FN_R; ++q) {
            const cx<T> v = Aj[e[x][q]];
            a[x][q].r += w * v.r;
            a[x][q].i += w * v.i;
          }
      }
#pragma unroll
      for (int x = 0; x < FN_C; ++x)
#pragma unroll
        for (int q = 0; q < FN_R; ++q)
          if (ok[x][q]) {
            ob[e[x][q]] = a[x][q];
            if (nmax) s[x] += sqrt((double)a[x][q].r * a[x][q].r + (double)a[x][q].i * a[x][q].i);
          }
    }
    if (nmax) {
#pragma unroll
      for (int x = 0; x < FN_C; ++x) {
        double v = s[x];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        best = fmax(best, v);
      }
    }
  }
  if (nmax && lane == 0) {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(best);
    if (bits > __hip_atomic_load(nmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(nmax, bits);
  }
}

// The same A_k and norm for N <= 64 RQ with the generators held in registers: workgroup (column block, slice group),
// wave w owns column 4 cb + w and keeps its RQ rows of A_0..A_nu in registers (lane rows r = lane + 64 q), then forms
// A_k for the group's slices in turn.  One workgroup per slice (k_form_norm) re-read the generators for every slice
// (3 x 512 KB per slice at N = 256, nu = 2: the kernel ran at ~2.6 TB/s of mostly generator reads); here they are
// read once per workgroup and the launch writes A_k at the store rate.  Column sums complete in the wave (the norm
// is the max column sum), one atomic max per workgroup.
constexpr int FN2_SG = 16;  // slices per workgroup
template <typename T, int RQ>
__global__ __launch_bounds__(256) void k_form_norm2(int N, int nu, long long unit0, int cnt,
                                                    const cx<T>* __restrict__ Agen, const double* __restrict__ u,
                                                    cx<T>* __restrict__ out, unsigned long long* __restrict__ nmax) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = 4 * blockIdx.x + wave, it0 = blockIdx.y * FN2_SG;
  const size_t NN = (size_t)N * N;
  const bool cok = c < N;
  cx<T> g[3][RQ];
  bool ok[RQ];
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int r = lane + 64 * q;
    ok[q] = cok && r < N;
    const size_t e = ok[q] ? r + (size_t)N * c : 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) g[j][q] = j <= nu ? Agen[(size_t)j * NN + e] : cx<T>{T(0), T(0)};
  }
  double best = 0.0;
  const int nit = min(FN2_SG, cnt - it0);
  for (int i = 0; i < nit; ++i) {
    const int it = it0 + i;
    const long long unit = unit0 + it;
    const T u1 = nu > 0 ? (T)u[unit * nu] : T(0), u2 = nu > 1 ? (T)u[unit * nu + 1] : T(0);
    cx<T>* ob = out + (size_t)it * NN + (size_t)N * c;
    double sum = 0.0;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      cx<T> a;
      a.r = g[0][q].r + u1 * g[1][q].r + u2 * g[2][q].r;
      a.i = g[0][q].i + u1 * g[1][q].i + u2 * g[2][q].i;
      if (ok[q]) {
        ob[lane + 64 * q] = a;
        if (nmax) sum += sqrt((double)a.r * a.r + (double)a.i * a.i);
      }
    }
    if (nmax) {
      for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
      best = fmax(best, sum);
    }
  }
  if (nmax) {
    __shared__ double wb[4];
    if (lane == 0) wb[wave] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
      const double bw = fmax(fmax(wb[0], wb[1]), fmax(wb[2], wb[3]));
      const unsigned long long bits = (unsigned long long)__double_as_longlong(bw);
      if (bits > __hip_atomic_load(nmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(nmax, bits);
    }
  }
}

// Guard-state penalty over all stored states: J[b] = mu * sum_{k, masked} |x_k|^2 (one WG per seed).
template <typename T>
__global__ void k_penalty_sum(int N, int m, int Nt, const cx<T>* __restrict__ X, const unsigned char* __restrict__ pmask,
                              double mu, double* __restrict__ J) {
  __shared__ double red[8];
  const int b = blockIdx.x;
  const size_t Nm = (size_t)N * m;
  const cx<T>* Xb = X + (size_t)b * (Nt + 1) * Nm;
  double s = 0.0;
  for (size_t gi = threadIdx.x; gi < (size_t)(Nt + 1) * Nm; gi += blockDim.x) {
    if (pmask[gi % Nm]) {
      const cx<T> v = Xb[gi];
      s += (double)v.r * v.r + (double)v.i * v.i;
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) J[b] = mu * s;
}

// λ_k[b] += 2 mu mask .* x_k[b] for one slice index k, all seeds.
template <typename T>
__global__ void k_add_source(int N, int m, int Nt, int B, int k, const cx<T>* __restrict__ src, cx<T>* __restrict__ Lam) {
  const size_t Nm = (size_t)N * m;
  for (size_t gi = blockIdx.x * (size_t)blockDim.x + threadIdx.x; gi < Nm * B; gi += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(gi / Nm);
    const size_t at = ((size_t)b * (Nt + 1) + k) * Nm + (gi - (size_t)b * Nm);
    cx<T> l = Lam[at];
    l.r += src[at].r;
    l.i += src[at].i;
    Lam[at] = l;
  }
}
template <typename T>
__global__ void k_penalty_grad(int N, int m, int Nt, int B, int k, const cx<T>* __restrict__ X,
                               const unsigned char* __restrict__ pmask, double two_mu, cx<T>* __restrict__ Lam) {
  const size_t Nm = (size_t)N * m;
  for (size_t gi = blockIdx.x * (size_t)blockDim.x + threadIdx.x; gi < Nm * B; gi += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(gi / Nm);
    const size_t o = gi - (size_t)b * Nm;
    if (!pmask[o]) continue;
    const size_t at = ((size_t)b * (Nt + 1) + k) * Nm + o;
    const cx<T> x = X[at];
    cx<T> l = Lam[at];
    l.r += (T)two_mu * x.r;
    l.i += (T)two_mu * x.i;
    Lam[at] = l;
  }
}

// dJdu[unit, j] = sum_{p,q} Re(A_j[p,q] conj(M'[p,q])) with M' = W P^H (one WG per slice in the chunk).
// This is Re tr(A_j P W^H) = sum_{a+b<=o-1} Re<(X^H)^b λ, A_j X^a x>/(a+b+1)!.
template <typename T>
__global__ __launch_bounds__(256) void k_gen_contract(int N, int nu, long long unit0, const cx<T>* __restrict__ Agen,
                                                      const cx<T>* __restrict__ Mp, double* __restrict__ dJdu) {
  __shared__ double red[8];
  const int it = blockIdx.x;
  const size_t NN = (size_t)N * N;
  const cx<T>* Mb = Mp + (size_t)it * NN;
  double acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.0;
  for (size_t e = threadIdx.x; e < NN; e += blockDim.x) {
    const cx<T> mv = Mb[e];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < nu) {
        const cx<T> a = Agen[(size_t)(j + 1) * NN + e];
        acc[j] += (double)a.r * mv.r + (double)a.i * mv.i;
      }
    }
  }
  const long long unit = unit0 + it;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j < nu) {
      const double s = block_sum(acc[j], red);
      if (threadIdx.x == 0) dJdu[unit * nu + j] = s;  // u layout: b*nu*Nt + k*nu + j == unit*nu + j
    }
  }
}

// The same contraction with the generators in registers (k_form_norm2's layout): workgroup (block of 4 columns, group
// of GC2_SG slices), wave w owns column 4 cb + w and keeps its rows of A_1..A_nu (nu <= 2) in registers, so only M'
// streams (k_gen_contract re-read 2 x 512 KB of generators per slice at N = 256).  Each workgroup writes its column
// block's partial sums part[(it * ncb + cb) * nu + j] (the four columns added in a fixed order); k_gen_reduce adds the
// ncb partials of every (slice, j) in a fixed order: the result does not depend on scheduling.
constexpr int GC2_SG = 16;
template <typename T, int RQ>
__global__ __launch_bounds__(256) void k_gen_contract2(int N, int nu, int cnt, const cx<T>* __restrict__ Agen,
                                                       const cx<T>* __restrict__ Mp, double* __restrict__ part) {
  __shared__ double wsum[4][GC2_SG][2];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cb = blockIdx.x, c = 4 * cb + wave, it0 = blockIdx.y * GC2_SG, ncb = gridDim.x;
  const size_t NN = (size_t)N * N;
  const bool cok = c < N;
  cx<T> a[2][RQ];
  bool ok[RQ];
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int r = lane + 64 * q;
    ok[q] = cok && r < N;
    const size_t e = ok[q] ? r + (size_t)N * c : 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) a[j][q] = j < nu && ok[q] ? Agen[(size_t)(j + 1) * NN + e] : cx<T>{T(0), T(0)};
  }
  const int nit = min(GC2_SG, cnt - it0);
  for (int i = 0; i < nit; ++i) {
    const cx<T>* Mb = Mp + (size_t)(it0 + i) * NN + (size_t)N * (cok ? c : 0);
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      if (ok[q]) {
        const cx<T> mv = Mb[lane + 64 * q];
        s0 += (double)a[0][q].r * mv.r + (double)a[0][q].i * mv.i;
        s1 += (double)a[1][q].r * mv.r + (double)a[1][q].i * mv.i;
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      s0 += __shfl_xor(s0, off);
      s1 += __shfl_xor(s1, off);
    }
    if (lane == 0) {
      wsum[wave][i][0] = s0;
      wsum[wave][i][1] = s1;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nit * nu; e += blockDim.x) {
    const int i = e / nu, j = e - i * nu;
    const double v = ((wsum[0][i][j] + wsum[1][i][j]) + wsum[2][i][j]) + wsum[3][i][j];
    part[((size_t)(it0 + i) * ncb + cb) * nu + j] = v;
  }
}
static __global__ void k_gen_reduce(int cnt, int nu, int ncb, long long unit0, const double* __restrict__ part,
                                    double* __restrict__ dJdu) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < cnt * nu; e += gridDim.x * blockDim.x) {
    const int it = e / nu, j = e - it * nu;
    const double* p = part + (size_t)it * ncb * nu + j;
    double s = 0.0;
    for (int q = 0; q < ncb; ++q) s += p[(size_t)q * nu];
    dJdu[(unit0 + it) * nu + j] = s;
  }
}

// Auxiliary generator layouts for the GEMM-shaped gradient of the LDS-resident path:
//   AH  = [A0^H | A1^H | ... | A_nu^H]   (N x (nu+1) N, column blocks)
//   Cst = [A1; A2; ...; A_nu]            (nu N x N, row blocks)
template <typename T>
__global__ void k_gen_aux(int N, int nu, const cx<T>* __restrict__ Agen, cx<T>* __restrict__ AH, cx<T>* __restrict__ Cst) {
  const size_t NN = (size_t)N * N;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < NN * (nu + 1); g += (size_t)gridDim.x * blockDim.x) {
    const size_t gi = g / NN, e = g - gi * NN;
    const size_t r = e % N, c = e / N;
    const cx<T> v = Agen[gi * NN + c + N * r];  // A_gi[c, r]
    AH[gi * NN + e] = cx<T>{v.r, -v.i};          // A_gi^H[r, c]
    if (gi > 0) Cst[(gi - 1) * N + r + (size_t)nu * N * c] = Agen[gi * NN + e];
  }
}

}  // namespace qoc
