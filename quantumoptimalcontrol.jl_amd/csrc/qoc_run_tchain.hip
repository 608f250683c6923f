// qoc_run_tchain.hip — launches of the Taylor-action chains (qoc_tchain.hpp) and the overlapped backward.
#include "qoc_internal.hpp"

namespace qoc_host {

// ---- Taylor-action chains (qoc_tchain.hpp) -----------------------------------------------------
size_t tchain_lds(const qoc_ctx* c) {
  const TShape sh = tchain_shape(c->N, c->m, c->prec == QOC_FP64);
  return (size_t)(c->nu + 1) * c->N * c->N * c->esz + (size_t)2 * sh.S * sh.JT * chain_mpad(c->m, sh.CB) * c->esz +
         64 * sizeof(double);
}

// k_tchain_* instantiated per (S, JT) x (CB, NP) in {(1, 1), (2, 1), (2, 2), (2, 4)}.
template <typename T, typename F>
hipError_t tchain_dispatch(int N, int m, F&& f) {
  using std::integral_constant;
  const TShape sh = tchain_shape(N, m, sizeof(T) == 8);
  auto cbnp = [&](auto S_, auto JT_) -> hipError_t {
    if (sh.CB == 1 && sh.NP == 1) return f(S_, JT_, integral_constant<int, 1>(), integral_constant<int, 1>());
    if (sh.CB == 2 && sh.NP == 1) return f(S_, JT_, integral_constant<int, 2>(), integral_constant<int, 1>());
    if (sh.CB == 2 && sh.NP == 2) return f(S_, JT_, integral_constant<int, 2>(), integral_constant<int, 2>());
    if (sh.CB == 2 && sh.NP == 4) return f(S_, JT_, integral_constant<int, 2>(), integral_constant<int, 4>());
    return hipErrorInvalidValue;
  };
  if (sh.JT == 4)
    return sh.S == 4 ? cbnp(integral_constant<int, 4>(), integral_constant<int, 4>())
                     : cbnp(integral_constant<int, 8>(), integral_constant<int, 4>());
  if (sh.JT == 10) return cbnp(integral_constant<int, 4>(), integral_constant<int, 10>());
  if (sh.JT == 12) return cbnp(integral_constant<int, 4>(), integral_constant<int, 12>());
  if constexpr (sizeof(T) == 4) {
    if (sh.JT == 16) return cbnp(integral_constant<int, 4>(), integral_constant<int, 16>());
  }
  return hipErrorInvalidValue;
}

TChainArgs tchain_args(qoc_ctx* c) {
  TChainArgs g{};
  g.N = c->N;
  g.m = c->m;
  g.nu = c->nu;
  g.Nt = c->Nt;
  g.At = c->d_At;
  g.u = c->d_u;
  g.steps = c->d_steps;
  g.x0 = c->d_x0;
  g.x0_per_seed = c->x0_per_seed;
  g.sink = c->d_sink;
  g.X = c->d_X;
  g.L = c->d_L;
  g.Xt = c->d_Xt;
  g.cost_kind = c->cost_kind;
  g.n_norm = c->cost_n;
  g.pmask = c->mu != 0.0 ? c->d_pmask : nullptr;
  g.mu = c->mu;
  g.J = c->d_J;
  g.coef = c->d_coef;
  g.src = c->src_on ? c->d_src : nullptr;
  g.tcoef = c->d_tcoef;
  g.sc = sectors(c);
  g.k_lo = 0;
  g.k_hi = c->Nt;
  return g;
}

// fp64: the MFMA formulation (k_tchain_mf_*), one wave per (16-row block, column pair); fp32: the VALU one.
bool tchain_mf(const qoc_ctx* c) {
  return c->prec == QOC_FP64 && tchain_mf_kq(c->N) > 0 && tchain_mf_waves(c->N, c->m) <= 16 &&
         tchain_mf_lds(c->N, c->m, c->nu) <= 160 * 1024;
}
// TChainRot<G> (KQ = -4 / -8 / -12 select G = 1 / 2 / 3): one wave per column pair with the state in registers, no
// LDS round trip per term.  m <= 8; G <= 2 (N <= 32) with nu <= 2 by default (generators in registers); G = 3
// (N <= 48, generators in LDS) with QOC_TCHAIN_ROT=3
bool tchain_mf_rot(const qoc_ctx* c) {
  if (!c->tchain_rot || !tchain_mf(c) || (c->m + 1) / 2 > 4) return false;
  if (c->N <= 32) return c->nu <= 2;
  return c->tchain_rot >= 3 && c->N <= 48 && tchain_mf_lds(c->N, c->m, c->nu, true) <= 160 * 1024;
}
int tchain_mf_threads(const qoc_ctx* c) {
  return 64 * (tchain_mf_rot(c) ? (c->m + 1) / 2 : tchain_mf_waves(c->N, c->m));
}
template <typename F>
hipError_t tchain_mf_dispatch(const qoc_ctx* c, F&& f) {
  using std::integral_constant;
  if (tchain_mf_rot(c))
    return c->N <= 16 ? f(integral_constant<int, -4>())
           : c->N <= 32 ? f(integral_constant<int, -8>())
                        : f(integral_constant<int, -12>());
  switch (tchain_mf_kq(c->N)) {
    case 3: return f(integral_constant<int, 3>());
    case 4: return f(integral_constant<int, 4>());
    case 6: return f(integral_constant<int, 6>());
    case 8: return f(integral_constant<int, 8>());
    case 10: return f(integral_constant<int, 10>());
    case 12: return f(integral_constant<int, 12>());
  }
  return hipErrorInvalidValue;
}
// the chain kernels of one KQ for a launch bound (TChainRot: 256 only)
template <int KQ>
void (*mf_fwd_kernel(int mt, bool cheb))(TChainArgs) {
  if constexpr (KQ < 0) {
    return cheb ? k_tchain_mf_fwd<KQ, true, 256> : k_tchain_mf_fwd<KQ, false, 256>;
  } else {
    return mt == 256   ? (cheb ? k_tchain_mf_fwd<KQ, true, 256> : k_tchain_mf_fwd<KQ, false, 256>)
           : mt == 512 ? (cheb ? k_tchain_mf_fwd<KQ, true, 512> : k_tchain_mf_fwd<KQ, false, 512>)
                       : (cheb ? k_tchain_mf_fwd<KQ, true, 1024> : k_tchain_mf_fwd<KQ, false, 1024>);
  }
}
template <int KQ>
void (*mf_bwd_kernel(int mt, bool cheb))(TChainArgs) {
  if constexpr (KQ < 0) {
    return cheb ? k_tchain_mf_bwd<KQ, true, 256> : k_tchain_mf_bwd<KQ, false, 256>;
  } else {
    return mt == 256   ? (cheb ? k_tchain_mf_bwd<KQ, true, 256> : k_tchain_mf_bwd<KQ, false, 256>)
           : mt == 512 ? (cheb ? k_tchain_mf_bwd<KQ, true, 512> : k_tchain_mf_bwd<KQ, false, 512>)
                       : (cheb ? k_tchain_mf_bwd<KQ, true, 1024> : k_tchain_mf_bwd<KQ, false, 1024>);
  }
}

bool tchain_cap_ok(const qoc_ctx* c);

// the step records of every (seed, slice): β_k, (P, s), e^{μ_k} and the Chebyshev coefficients
int tchain_prep(qoc_ctx* c) {
  const long long units = (long long)c->B * c->Nt;
  const bool cheb = c->cheb && tchain_mf(c);
  if (cheb && !c->d_tcoef) {
    const size_t bytes = (size_t)units * TCHEB_STRIDE * sizeof(double);
    HIPCHK(c, hipMalloc((void**)&c->d_tcoef, bytes));
    c->dev_bytes += bytes;
  }
  int mk = mark_begin(c, 0);
  const unsigned pb = (unsigned)std::min<long long>((units + 255) / 256, 2048);
  // The Chebyshev prep: one thread per unit storing its coefficient row (default), or QOC_TCHEB_PREP=1 one wave per
  // 64 units with the rows staged in LDS and stored coalesced (round 4).  Same-box A/B on the tunable bus
  // (profiles/bench_r05k_tb_*.json): the staged form writes fewer bytes but its prep is slower (0.41 vs 0.35 ms) and
  // the block chain after it ran 22.0 instead of 18.4 ms (writing full 64-entry rows, QOC_TCHEB_PW=64, did not
  // change that); with dead blocks skipped (blk_live) both give 15.1 ms.
  const char* pk = getenv("QOC_TCHEB_PREP");
  const char* pwe = getenv("QOC_TCHEB_PW");  // smallest coefficient row width the staged form writes
  const int prep_kind = pk ? atoi(pk) : 0, prep_pw = pwe ? atoi(pwe) : 0;
  if (cheb && prep_kind == 0)
    hipLaunchKernelGGL(k_tchain_prep_cheb_strided, dim3(pb), dim3(256), 0, c->stream, c->nu, units,
                       (const double*)c->d_u, c->tprm, c->d_steps, c->d_tcoef, c->d_terms);
  else if (cheb)  // one wave per workgroup (the coefficient rows are staged in its LDS)
    hipLaunchKernelGGL(k_tchain_prep_cheb, dim3((unsigned)std::min<long long>((units + 63) / 64, 8192)), dim3(64), 0,
                       c->stream, c->nu, units, (const double*)c->d_u, c->tprm, c->d_steps, c->d_tcoef, c->d_terms,
                       prep_pw);
  else
    hipLaunchKernelGGL(k_tchain_prep, dim3(pb), dim3(256), 0, c->stream, c->nu, units, (const double*)c->d_u, c->tprm,
                       c->d_steps, c->d_terms);
  mark_end(c, mk);
  HIPCHK(c, hipGetLastError());
  c->cheb_ran = cheb;
  c->steps_stale = false;
  return QOC_OK;
}

template <typename T>
int tchain_forward_chain(qoc_ctx* c);

template <typename T>
int tchain_forward(qoc_ctx* c) {
  const int r = tchain_prep(c);
  return r ? r : tchain_forward_chain<T>(c);
}

// the forward chain over the step records tchain_prep wrote (with its captures when the shape takes them)
template <typename T>
int tchain_forward_chain(qoc_ctx* c) {
  const bool cheb = c->cheb_ran;
  int mk;
  TChainArgs g = tchain_args(c);
  c->fwd_captured = false;
  if (tchain_cap_ok(c) && ensure_pws(c) == QOC_OK) {  // P1 / P2 of the gradient as by-products
    const size_t bufN = (size_t)c->N * ((size_t)c->B * (c->Nt + 1) * c->m);
    g.cap1 = c->d_pws;
    g.cap2 = (cx<double>*)c->d_pws + bufN;
    c->fwd_captured = true;
  }
  if (tchain_mf(c)) {
    const size_t lds = tchain_mf_lds(c->N, c->m, c->nu, tchain_mf_rot(c));
    const int threads = tchain_mf_threads(c);
    mk = mark_begin(c, 1);
    hipError_t e = tchain_mf_dispatch(c, [&](auto KQ_) {
      constexpr int KQ = decltype(KQ_)::value;
      auto kern = mf_fwd_kernel<KQ>(tchain_mf_maxt(c->N, c->m, c->nu), cheb);
      hipError_t r = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (r != hipSuccess) return r;
      hipLaunchKernelGGL(kern, dim3(c->B), dim3(threads), lds, c->stream, g);
      return hipGetLastError();
    });
    mark_end(c, mk);
    if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_tchain_mf_fwd launch: %s", hipGetErrorString(e));
    c->props_since_reset++;
    return QOC_OK;
  }
  const size_t lds = tchain_lds(c);
  mk = mark_begin(c, 1);
  hipError_t e = tchain_dispatch<T>(c->N, c->m, [&](auto S_, auto JT_, auto CB_, auto NP_) {
    constexpr int S = decltype(S_)::value, JT = decltype(JT_)::value, CB = decltype(CB_)::value,
                  NP = decltype(NP_)::value;
    hipError_t r = hipFuncSetAttribute((const void*)k_tchain_fwd<T, S, JT, CB, NP>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL((k_tchain_fwd<T, S, JT, CB, NP>), dim3(c->B), dim3(CHAIN_THREADS), lds, c->stream, g);
    return hipGetLastError();
  });
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_tchain_fwd launch: %s", hipGetErrorString(e));
  c->props_since_reset++;
  return QOC_OK;
}

template <typename T>
int tchain_backward(qoc_ctx* c, int k_lo, int k_hi, hipStream_t st, int flags) {
  TChainArgs g = tchain_args(c);
  if (!st) st = c->stream;
  if (tchain_mf(c)) {
    if (k_hi >= 0) {  // a range of slices (tchain_backward_overlapped)
      g.k_lo = k_lo;
      g.k_hi = k_hi;
      g.prio = c->bwd_prio & 1;
    }
    if (flags & TB_CAPTURE) {  // Q1 / Q2 of the gradient as by-products (d_gws: the W0 / W1 buffers)
      const size_t bufN = (size_t)c->N * ((size_t)c->B * (c->Nt + 1) * c->m);
      g.cap1 = c->d_gws;
      g.cap2 = (cx<double>*)c->d_gws + bufN;
    }
    g.mu_mode = (flags & TB_MU) ? 1 : 0;
    const size_t lds = tchain_mf_lds(c->N, c->m, c->nu, tchain_mf_rot(c));
    const int threads = tchain_mf_threads(c);
    int mk = mark_begin(c, 2, st);
    hipError_t e = tchain_mf_dispatch(c, [&](auto KQ_) {
      constexpr int KQ = decltype(KQ_)::value;
      // the (P, s, coefficients) of the forward pass are reused: the same polynomial as the states'
      auto kern = mf_bwd_kernel<KQ>(tchain_mf_maxt(c->N, c->m, c->nu), c->cheb_ran);
      hipError_t r = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (r != hipSuccess) return r;
      hipLaunchKernelGGL(kern, dim3(c->B), dim3(threads), lds, st, g);
      return hipGetLastError();
    });
    mark_end(c, mk, st);
    if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_tchain_mf_bwd launch: %s", hipGetErrorString(e));
    return QOC_OK;
  }
  if (flags) return fail(c, QOC_ERR_UNSUPPORTED, "captured / μ-mode backward needs the MFMA chains");
  const size_t lds = tchain_lds(c);
  int mk = mark_begin(c, 2);
  hipError_t e = tchain_dispatch<T>(c->N, c->m, [&](auto S_, auto JT_, auto CB_, auto NP_) {
    constexpr int S = decltype(S_)::value, JT = decltype(JT_)::value, CB = decltype(CB_)::value,
                  NP = decltype(NP_)::value;
    hipError_t r = hipFuncSetAttribute((const void*)k_tchain_bwd<T, S, JT, CB, NP>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL((k_tchain_bwd<T, S, JT, CB, NP>), dim3(c->B), dim3(CHAIN_THREADS), lds, c->stream, g);
    return hipGetLastError();
  });
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_tchain_bwd launch: %s", hipGetErrorString(e));
  return QOC_OK;
}

// Backward chain in slice ranges with the gradient of each finished range on a second stream: the order-3
// gradient of slices [k_lo, k_hi) needs only x_k and λ_{k+1}, so it runs while the chain works on the
// next range (lower k).  The chain's workgroup (3 waves, ~84 KB LDS, <= 264 VGPRs at N = 40) leaves room on
// each CU for one gradient workgroup, whose waves take the chain's MFMA idle cycles.  Chunk boundaries are
// uniform in k except the last (exposed) range, bwd_last_frac of a uniform one.
template <typename T>
int tchain_backward_overlapped(qoc_ctx* c, double* d_dJdu) {
  const int Nt = c->Nt, S = std::min(c->bwd_chunks, std::max(1, Nt / 32));  // ranges of >= ~32 slices
  if (!c->stream2) {
    int lo = 0, hi = 0;
    HIPCHK(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPCHK(c, hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, (c->bwd_prio & 2) ? lo : 0));
  }
  while ((int)c->sync_ev.size() < S + 2) {
    hipEvent_t e;
    HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->sync_ev.push_back(e);
  }
  // k boundaries: kb[0] = Nt > kb[1] > ... > kb[S] = 0; the last range is shorter
  std::vector<int> kb(S + 1);
  const double last = std::max(0.05, std::min(1.0, c->bwd_last_frac)), w = Nt / (S - 1 + last);
  for (int i = 0; i <= S; ++i) kb[i] = std::max(0, Nt - (int)std::lround(i * w));
  kb[S] = 0;
  // state side first (QOC_BWD_PRESTATE): P1 = X x_k, P2 = X P1 of every slice need only the forward's states, so
  // they run beside the first range, which otherwise has nothing beside it; each range then runs q + p (PRE).
  const size_t pws = (size_t)2 * c->N * c->B * (Nt + 1) * c->m * c->esz;
  // auto: only when a CU keeps room beside its chain waves (<= 3 per CU, or small N whose chain waves are
  // light); measured: cavity (3 waves/CU) +1.3 %, zz +0.9 %, tunable bus (2 WGs x 2 waves/CU) -2.6 %
  const long long chain_waves = (long long)((c->B + c->ncu - 1) / c->ncu) * tchain_mf_waves(c->N, c->m);
  bool pre = c->bwd_prestate == 1 || (c->bwd_prestate == 2 && (chain_waves <= 3 || c->N <= 16));
  if (pre && c->pws_bytes < pws) {  // grown on first use; without the buffer the ranges run q + p in full
    if (c->d_pws) {
      HIPCHK(c, hipStreamSynchronize(c->stream2));
      HIPCHK(c, hipFree(c->d_pws));
      c->dev_bytes -= c->pws_bytes;
    }
    c->d_pws = nullptr;
    c->pws_bytes = 0;
    if (hipMalloc(&c->d_pws, pws) == hipSuccess) {
      c->pws_bytes = pws;
      c->dev_bytes += pws;
    } else {
      (void)hipGetLastError();
      c->d_pws = nullptr;
      pre = false;
    }
  }
  HIPCHK(c, hipEventRecord(c->sync_ev[S], c->stream));  // stream2 starts after everything queued so far
  HIPCHK(c, hipStreamWaitEvent(c->stream2, c->sync_ev[S], 0));
  // every exit joins stream2 back into the engine stream, so that later work on c->stream (uploads, the next
  // call's kernels) is ordered after the gradients already queued on stream2
  auto join = [&](int r) {
    const hipError_t e1 = hipEventRecord(c->sync_ev[S + 1], c->stream2);
    const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(c->stream, c->sync_ev[S + 1], 0) : e1;
    if (r == QOC_OK && e2 != hipSuccess) return fail(c, QOC_ERR_HIP, "stream join: %s", hipGetErrorString(e2));
    return r;
  };
  if (pre) {
    const int mk = mark_begin(c, 3, c->stream2);
    const int r = grad_rr_o3<T>(c, d_dJdu, c->stream2, 0, Nt, 1);
    mark_end(c, mk, c->stream2);
    if (r) return join(r);
  }
  for (int i = 0; i < S; ++i) {
    if (kb[i + 1] >= kb[i]) continue;
    int r = tchain_backward<T>(c, kb[i + 1], kb[i]);
    if (r) return join(r);
    hipError_t e = hipEventRecord(c->sync_ev[i], c->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->stream2, c->sync_ev[i], 0);
    if (e != hipSuccess) return join(fail(c, QOC_ERR_HIP, "range event: %s", hipGetErrorString(e)));
    const int mk = mark_begin(c, 3, c->stream2);
    r = grad_rr_o3<T>(c, d_dJdu, c->stream2, kb[i + 1], kb[i] - kb[i + 1], pre ? 2 : 0);
    mark_end(c, mk, c->stream2);
    if (r) return join(r);
  }
  return join(QOC_OK);
}

// reference-equivalent Padé (d, s) of every unit of the last propagated u -> c->d_hist (k_pade_units)
hipError_t launch_pade_units(qoc_ctx* c, long long units) {
  const unsigned blocks = (unsigned)std::min<long long>((units + 3) / 4, 8192);
  if (c->prec == QOC_FP64)
    hipLaunchKernelGGL((k_pade_units<double>), dim3(blocks), dim3(256), 0, c->stream, c->N, c->nu, units,
                       (const cx<double>*)c->d_A, (const double*)c->d_u, c->d_hist);
  else
    hipLaunchKernelGGL((k_pade_units<float>), dim3(blocks), dim3(256), 0, c->stream, c->N, c->nu, units,
                       (const cx<float>*)c->d_A, (const double*)c->d_u, c->d_hist);
  return hipGetLastError();
}

// The register-resident MFMA chains (MAXT = 256) can write their first two products per slice; with the fused
// order-3 gradient they then replace its generator products (k_grad_rr_c).
bool tchain_cap_ok(const qoc_ctx* c) {
  return c->cap_ok && tchain_mf(c) && (tchain_mf_rot(c) || tchain_mf_maxt(c->N, c->m, c->nu) == 256) && c->grad_rr &&
         c->nu <= 2;
}

// d_pws: the forward captures (two state-shaped buffers), grown on first use; QOC_ERR_HIP if it cannot be had
int ensure_pws(qoc_ctx* c) {
  const size_t pws = (size_t)2 * c->N * c->B * (c->Nt + 1) * c->m * c->esz;
  if (c->d_pws && c->pws_bytes >= pws) return QOC_OK;
  if (c->d_pws) {
    if (c->stream2) HIPCHK(c, hipStreamSynchronize(c->stream2));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(c->d_pws));
    c->dev_bytes -= c->pws_bytes;
  }
  c->d_pws = nullptr;
  c->pws_bytes = 0;
  if (hipMalloc(&c->d_pws, pws) != hipSuccess) {
    (void)hipGetLastError();
    c->d_pws = nullptr;
    return fail(c, QOC_ERR_HIP, "capture buffers (%zu bytes) not available", pws);
  }
  c->pws_bytes = pws;
  c->dev_bytes += pws;
  return QOC_OK;
}

int ensure_stream2(qoc_ctx* c, int nev) {
  if (!c->stream2) {
    int lo = 0, hi = 0;
    HIPCHK(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPCHK(c, hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, (c->bwd_prio & 2) ? lo : 0));
  }
  while ((int)c->sync_ev.size() < nev) {
    hipEvent_t e;
    HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->sync_ev.push_back(e);
  }
  return QOC_OK;
}

// grape_sensitivity after a captured forward: the backward chain writes its captures, range by range (as
// tchain_backward_overlapped), and each finished range's contraction (k_grad_rr_c) runs on the second stream.
template <typename T>
int tchain_backward_captured(qoc_ctx* c, double* d_dJdu) {
  const int Nt = c->Nt;
  const int S = c->bwd_chunks > 1 && Nt >= 64 ? std::min(c->bwd_chunks, std::max(1, Nt / 32)) : 1;
  int r = ensure_stream2(c, S + 2);
  if (r) return r;
  std::vector<int> kb(S + 1);
  const double last = std::max(0.05, std::min(1.0, c->bwd_last_frac)), w = Nt / (S - 1 + last);
  for (int i = 0; i <= S; ++i) kb[i] = std::max(0, Nt - (int)std::lround(i * w));
  kb[S] = 0;
  kb[0] = Nt;
  HIPCHK(c, hipEventRecord(c->sync_ev[S], c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->stream2, c->sync_ev[S], 0));
  auto join = [&](int rc) {
    const hipError_t e1 = hipEventRecord(c->sync_ev[S + 1], c->stream2);
    const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(c->stream, c->sync_ev[S + 1], 0) : e1;
    if (rc == QOC_OK && e2 != hipSuccess) return fail(c, QOC_ERR_HIP, "stream join: %s", hipGetErrorString(e2));
    return rc;
  };
  for (int i = 0; i < S; ++i) {
    if (kb[i + 1] >= kb[i]) continue;
    r = tchain_backward<T>(c, kb[i + 1], kb[i], c->stream, TB_CAPTURE);
    if (r) return join(r);
    hipError_t e = hipEventRecord(c->sync_ev[i], c->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->stream2, c->sync_ev[i], 0);
    if (e != hipSuccess) return join(fail(c, QOC_ERR_HIP, "range event: %s", hipGetErrorString(e)));
    const int mk = mark_begin(c, 3, c->stream2);
    r = grad_rr_cap(c, d_dJdu, c->stream2, kb[i + 1], kb[i] - kb[i + 1], false);
    mark_end(c, mk, c->stream2);
    if (r) return join(r);
  }
  c->last_eval_mode = 1;
  return join(QOC_OK);
}

// One eval (propagate + order-3 sensitivity) with a built-in cost and no penalty / co-state source: for those costs
// λ_{Nt} = coef ⊙ X_target (src/penalty_fcns.jl:19-22, 35-40), and every later λ_k = U_k^H λ_{k+1} is linear, so
// λ_k = coef ⊙ μ_k with μ_k = U_k^H .. U_{Nt-1}^H X_target, which needs only the step records.  The μ recurrence
// (k_tchain_mf_bwd in μ mode) therefore runs on the second stream beside the forward chain, whose coefficients are
// not known until its end; the contraction (k_grad_rr_c) then applies coef on load.  d_L holds μ afterwards.
bool tchain_concurrent_ok(const qoc_ctx* c, int order) {
  return c->concurrent && order == 3 && tchain_cap_ok(c) && c->chain_mode == 1 && c->prop_method == QOC_PROP_EXPM &&
         !c->big && (c->cost_kind == QOC_COST_TRACE || c->cost_kind == QOC_COST_ZCAL) && c->mu == 0.0 && !c->src_on;
}

template <typename T>
int tchain_eval_concurrent(qoc_ctx* c, double* d_dJdu) {
  int r = ensure_stream2(c, 4);
  if (r) return r;
  if ((r = ensure_pws(c))) return r;
  if (!c->d_coef_mu) {
    HIPCHK(c, hipMalloc((void**)&c->d_coef_mu, (size_t)c->B * 2 * c->m_user * sizeof(cx<double>)));
    c->dev_bytes += (size_t)c->B * 2 * c->m_user * sizeof(cx<double>);
  }
  // the step records first (both chains read them)
  if ((r = tchain_prep(c))) return r;
  HIPCHK(c, hipEventRecord(c->sync_ev[0], c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->stream2, c->sync_ev[0], 0));
  if (c->concurrent == 2) {
    // μ recurrence beside the forward chain: two launches on two streams
    r = tchain_backward<T>(c, 0, c->Nt, c->stream2, TB_CAPTURE | TB_MU);
    if (r == QOC_OK) r = tchain_forward_chain<T>(c);
    if (r == QOC_OK && !c->fwd_captured) r = fail(c, QOC_ERR_STATE, "concurrent eval: forward captures missing");
    const hipError_t e1 = hipEventRecord(c->sync_ev[1], c->stream2);
    const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(c->stream, c->sync_ev[1], 0) : e1;
    if (r) return r;
    if (e2 != hipSuccess) return fail(c, QOC_ERR_HIP, "stream join: %s", hipGetErrorString(e2));
  } else {
    // one launch of 2B workgroups: k_tchain_mf_dual (forward chain and μ recurrence of every seed)
    const size_t bufN = (size_t)c->N * ((size_t)c->B * (c->Nt + 1) * c->m);
    TChainArgs gf = tchain_args(c), gb = tchain_args(c);
    gf.cap1 = c->d_pws;
    gf.cap2 = (cx<double>*)c->d_pws + bufN;
    gb.cap1 = c->d_gws;
    gb.cap2 = (cx<double>*)c->d_gws + bufN;
    gb.mu_mode = 1;
    const size_t lds = tchain_mf_lds(c->N, c->m, c->nu, tchain_mf_rot(c));
    const int threads = tchain_mf_threads(c);
    const int mk = mark_begin(c, 1);
    hipError_t e = tchain_mf_dispatch(c, [&](auto KQ_) {
      constexpr int KQ = decltype(KQ_)::value;
      auto kern = c->cheb_ran ? k_tchain_mf_dual<KQ, true, 256> : k_tchain_mf_dual<KQ, false, 256>;
      hipError_t q = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (q != hipSuccess) return q;
      hipLaunchKernelGGL(kern, dim3(2 * c->B), dim3(threads), lds, c->stream, gf, gb);
      return hipGetLastError();
    });
    mark_end(c, mk);
    if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_tchain_mf_dual launch: %s", hipGetErrorString(e));
    c->fwd_captured = true;
    c->props_since_reset++;
  }
  const int mk = mark_begin(c, 3);
  r = grad_rr_cap(c, d_dJdu, c->stream, 0, c->Nt, true);
  mark_end(c, mk);
  if (r) return r;
  // the coefficients that turn μ into λ, kept for qoc_get_costates (a later forward rewrites d_coef)
  HIPCHK(c, hipMemcpyAsync(c->d_coef_mu, c->d_coef, (size_t)c->B * 2 * c->m * sizeof(cx<double>),
                           hipMemcpyDeviceToDevice, c->stream));
  c->L_is_mu = true;
  c->last_eval_mode = c->concurrent == 2 ? 2 : 3;
  return QOC_OK;
}

template int tchain_forward<double>(qoc_ctx*);
template int tchain_forward<float>(qoc_ctx*);
template int tchain_backward<double>(qoc_ctx*, int, int, hipStream_t, int);
template int tchain_backward<float>(qoc_ctx*, int, int, hipStream_t, int);
template int tchain_backward_overlapped<double>(qoc_ctx*, double*);
template int tchain_backward_overlapped<float>(qoc_ctx*, double*);
template int tchain_backward_captured<double>(qoc_ctx*, double*);
template int tchain_backward_captured<float>(qoc_ctx*, double*);
template int tchain_eval_concurrent<double>(qoc_ctx*, double*);
template int tchain_eval_concurrent<float>(qoc_ctx*, double*);

}  // namespace qoc_host
