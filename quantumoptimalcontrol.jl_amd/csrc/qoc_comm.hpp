// qoc_comm.hpp — multi-GPU epilogue behind the C ABI: the best (J, seed) over every rank's seeds.
//
// Seeds are sharded contiguously over ranks, one process (one context) per GPU; the only exchange on the hot
// path is an all-gather of each rank's best (J, global seed id), 16 bytes per rank, over RCCL
// (xGMI within a node).  The reference has no counterpart (it is single-process); its caller is the multi-start
// driver around examples/ipopt_callbacks_exp.jl:9-31.  RCCL is dlopen'ed on the first qoc_comm_* call, so the
// library loads (and single-GPU use works) without it.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "qoc_common.hpp"

namespace qoc {

// (min J, its global seed id) over J[0..B) -> out[0..1]; one workgroup.
static __global__ void k_argmin_seed(const double* __restrict__ J, int B, long long seed_offset, double* __restrict__ out) {
  __shared__ double sv[16];
  __shared__ long long si[16];
  double best = __builtin_inf();
  long long bi = -1;
  for (int e = threadIdx.x; e < B; e += blockDim.x) {
    const double v = J[e];
    if (v < best || (v == best && e < bi)) {  // NaN never wins; ties go to the lower seed
      best = v;
      bi = e;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(best, off);
    const long long oi = __shfl_xor(bi, off);
    if (ov < best || (ov == best && oi >= 0 && (bi < 0 || oi < bi))) {
      best = ov;
      bi = oi;
    }
  }
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = best;
    si[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < nw; ++i)
      if (sv[i] < best || (sv[i] == best && si[i] >= 0 && (bi < 0 || si[i] < bi))) {
        best = sv[i];
        bi = si[i];
      }
    out[0] = best;
    out[1] = bi >= 0 ? (double)(bi + seed_offset) : -1.0;
  }
}

// Reduce the gathered (J, seed) pairs of `world` ranks to the best one (lowest seed on ties).
static __global__ void k_pick_best(const double* __restrict__ g, int world, double* __restrict__ out,
                                   double* __restrict__ out2) {
  if (threadIdx.x != 0) return;
  double best = g[0], seed = g[1];
  for (int r = 1; r < world; ++r) {
    const double v = g[2 * r], s = g[2 * r + 1];
    if (v < best || (v == best && s >= 0 && (seed < 0 || s < seed))) {
      best = v;
      seed = s;
    }
  }
  out[0] = best;
  out[1] = seed;
  if (out2) {
    out2[0] = best;
    out2[1] = seed;
  }
}

// The RCCL entry points the epilogue uses, resolved from librccl at run time.
struct RcclApi {
  ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  const char* (*getErrorString)(ncclResult_t) = nullptr;
  bool ok = false;
};

}  // namespace qoc
