// qoc_engine.hip — host side of libqoc_mi355x.so: the C ABI declared in include/qoc.h.
//
// The context replaces the reference's GRAPE cache (src/gradient_computations.jl:79-96):
// all per-slice propagators, states and co-states live in HBM for the whole batch of
// seeds, and the hot path (propagate + grape_sensitivity) is four kernel launches on
// one HIP stream:  k_expm -> k_chain_fwd  |  k_chain_bwd -> k_grad.
//
// The kernel launches live in the qoc_run*.hip translation units (see qoc_internal.hpp).
#include <dlfcn.h>

#include "qoc_internal.hpp"
#include "qoc_spline.hpp"

namespace qoc_host {

thread_local std::string g_err;

int fail(qoc_ctx* ctx, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  if (ctx) ctx->err = buf;
  return code;
}

template <typename T>
int upload_complex(qoc_ctx* ctx, const double* host, void* dev, size_t nelem) {
  if (sizeof(T) == sizeof(double)) {
    HIPCHK(ctx, hipMemcpyAsync(dev, host, nelem * 16, hipMemcpyHostToDevice, ctx->stream));
    return QOC_OK;
  }
  if (nelem > ctx->stage_elems) {
    if (ctx->d_stage) hipFree(ctx->d_stage);
    HIPCHK(ctx, hipMalloc(&ctx->d_stage, nelem * 16));
    ctx->stage_elems = nelem;
  }
  HIPCHK(ctx, hipMemcpyAsync(ctx->d_stage, host, nelem * 16, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL((k_cvt_in<T>), dim3(256), dim3(256), 0, ctx->stream, (const cx<double>*)ctx->d_stage,
                     (cx<T>*)dev, nelem);
  HIPCHK(ctx, hipGetLastError());
  return QOC_OK;
}

int upload(qoc_ctx* ctx, const double* host, void* dev, size_t nelem) {
  return ctx->prec == QOC_FP64 ? upload_complex<double>(ctx, host, dev, nelem)
                               : upload_complex<float>(ctx, host, dev, nelem);
}

int download(qoc_ctx* ctx, const void* dev, double* host, size_t nelem) {
  if (ctx->prec == QOC_FP64) {
    HIPCHK(ctx, hipMemcpyAsync(host, dev, nelem * 16, hipMemcpyDeviceToHost, ctx->stream));
  } else {
    if (nelem > ctx->stage_elems) {
      if (ctx->d_stage) hipFree(ctx->d_stage);
      HIPCHK(ctx, hipMalloc(&ctx->d_stage, nelem * 16));
      ctx->stage_elems = nelem;
    }
    hipLaunchKernelGGL((k_cvt_out<float>), dim3(256), dim3(256), 0, ctx->stream, (const cx<float>*)dev,
                       (cx<double>*)ctx->d_stage, nelem);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(host, ctx->d_stage, nelem * 16, hipMemcpyDeviceToHost, ctx->stream));
  }
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return QOC_OK;
}

// ---- packed states (compress_states / decompress_states, src/utils.jl:96-109) ----------------------------
// The caller's N x m_user states hold two parity sectors: rows with h_rsec[r] = s are nonzero only in the
// original columns pk_cols[s].  With generators that keep the two row sets apart (block-diagonal), packed
// column i = (rows of sector 0 from column pk_cols[0][i]) + (rows of sector 1 from pk_cols[1][i]) propagates
// exactly like the two original columns, so every kernel runs on m = max(n1, n2) columns.
bool grad_rr_cols(int m) { return m == 1 || m == 2 || m == 4 || m == 8 || m == 16; }

Sectors sectors(const qoc_ctx* c) {
  Sectors s;
  if (c->packed) {
    s.rsec = c->d_rsec;
    for (int q = 0; q < 4; ++q) s.zmap[q] = c->zmap[q];
  }
  return s;
}

// caller layout (N x m_user, interleaved complex, column-major) -> the kernels' N x m layout.  Entries outside
// the two blocks are dropped; `what` != nullptr makes a nonzero one an error (initial states: dropping one would
// change the result; targets and co-state inputs only ever meet zeros there, see qoc_set_compression).
int pack_states(qoc_ctx* c, const double* in, double* out, const char* what) {
  const int N = c->N, m = c->m;
  if (!c->packed) {
    std::memcpy(out, in, (size_t)2 * N * m * sizeof(double));
    return QOC_OK;
  }
  std::fill(out, out + (size_t)2 * N * m, 0.0);
  for (int r = 0; r < N; ++r) {
    const int s = c->h_rsec[r];
    for (int oc = 0; oc < c->m_user; ++oc) {
      const double* v = in + 2 * (r + (size_t)N * oc);
      const int i = c->pk_pos[s][oc];
      if (i >= 0) {
        out[2 * (r + (size_t)N * i)] = v[0];
        out[2 * (r + (size_t)N * i) + 1] = v[1];
      } else if (what && (v[0] != 0.0 || v[1] != 0.0)) {
        return fail(c, QOC_ERR_ARG, "%s has a nonzero entry (row %d, column %d) outside the compress_states blocks",
                    what, r, oc);
      }
    }
  }
  return QOC_OK;
}

void unpack_states(const qoc_ctx* c, const double* in, double* out) {
  const int N = c->N;
  std::fill(out, out + (size_t)2 * N * c->m_user, 0.0);
  for (int r = 0; r < N; ++r) {
    const auto& cols = c->pk_cols[c->h_rsec[r]];
    for (size_t i = 0; i < cols.size(); ++i) {
      out[2 * (r + (size_t)N * cols[i])] = in[2 * (r + N * i)];
      out[2 * (r + (size_t)N * cols[i]) + 1] = in[2 * (r + N * i) + 1];
    }
  }
}

// `count` consecutive N x m_user blocks -> packed device blocks (N x m each)
int upload_states(qoc_ctx* c, const double* host, void* dev, size_t count, const char* what) {
  const size_t Nm = (size_t)c->N * c->m, Nmu = (size_t)c->N * c->m_user;
  if (!c->packed) return upload(c, host, dev, count * Nm);
  std::vector<double> buf(2 * Nm * count);
  for (size_t q = 0; q < count; ++q) {
    int r = pack_states(c, host + 2 * Nmu * q, buf.data() + 2 * Nm * q, what);
    if (r) return r;
  }
  int r = upload(c, buf.data(), dev, count * Nm);
  if (r) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // buf is released on return
  return QOC_OK;
}

// one packed device block -> N x m_user host block
int download_states(qoc_ctx* c, const void* dev, double* host) {
  const size_t Nm = (size_t)c->N * c->m;
  if (!c->packed) return download(c, dev, host, Nm);
  std::vector<double> buf(2 * Nm);
  int r = download(c, dev, buf.data(), Nm);
  if (r) return r;
  unpack_states(c, buf.data(), host);
  return QOC_OK;
}

// the generators keep the two row sectors apart (compress_states applies)
bool gens_block_diagonal(const qoc_ctx* c) {
  const int N = c->N;
  const size_t NN = (size_t)N * N;
  for (int j = 0; j <= c->nu; ++j)
    for (int col = 0; col < N; ++col)
      for (int row = 0; row < N; ++row)
        if (c->h_rsec[row] != c->h_rsec[col]) {
          const double* v = c->h_gen.data() + 2 * (j * NN + row + (size_t)N * col);
          if (v[0] != 0.0 || v[1] != 0.0) return false;
        }
  return true;
}

hipEvent_t take_event(qoc_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// RAII-less bracket: mark_begin returns the index of the pending mark, mark_end records its stop event.
int mark_begin(qoc_ctx* c, int phase, hipStream_t s) {
  if (!c->profiling) return -1;
  qoc_ctx::Mark m{phase, take_event(c), take_event(c)};
  (void)hipEventRecord(m.a, s ? s : c->stream);
  c->marks.push_back(m);
  return (int)c->marks.size() - 1;
}
void mark_end(qoc_ctx* c, int idx, hipStream_t s) {
  if (idx >= 0) (void)hipEventRecord(c->marks[idx].b, s ? s : c->stream);
}

// Taylor-tail thresholds: θ_P = largest β with Σ_{t>P} β^t / t! <= tol.
double taylor_tail(double b, int P) {
  double term = 1.0, sum = 0.0;
  for (int t = 1; t <= P + 60; ++t) {
    term *= b / t;
    if (t > P) sum += term;
  }
  return sum;
}
void tchain_thresholds(TChainParams& prm, int prec) {
  const double tol = prec == QOC_FP64 ? std::ldexp(1.0, -53) : std::ldexp(1.0, -24);
  for (int P = 1; P <= TCHAIN_PMAX; ++P) {
    double lo = 0.0, hi = 64.0;
    for (int it = 0; it < 200; ++it) {
      const double mid = 0.5 * (lo + hi);
      (taylor_tail(mid, P) <= tol ? lo : hi) = mid;
    }
    prm.theta[P] = lo;
  }
  prm.theta[0] = 0.0;
  prm.theta_max = prm.theta[prec == QOC_FP64 ? 24 : 12];
}

// Scalar shift μ of a generator (column-major interleaved complex, N x N) that minimises ||A - μ I||_1 over a few
// candidates (0, trace / N, the centre of the diagonal's bounding box); returns the shifted norm.
double choose_shift(const double* A, int N, double& mr, double& mi) {
  std::vector<double> off(N, 0.0);
  double tr_r = 0, tr_i = 0, rmin = 1e300, rmax = -1e300, imin = 1e300, imax = -1e300;
  for (int col = 0; col < N; ++col) {
    for (int row = 0; row < N; ++row) {
      const double re = A[2 * (row + (size_t)N * col)], im = A[2 * (row + (size_t)N * col) + 1];
      if (row == col) {
        tr_r += re;
        tr_i += im;
        rmin = std::min(rmin, re);
        rmax = std::max(rmax, re);
        imin = std::min(imin, im);
        imax = std::max(imax, im);
      } else {
        off[col] += std::hypot(re, im);
      }
    }
  }
  auto norm = [&](double sr, double si) {
    double n = 0.0;
    for (int col = 0; col < N; ++col) {
      const double re = A[2 * (col + (size_t)N * col)], im = A[2 * (col + (size_t)N * col) + 1];
      n = std::max(n, off[col] + std::hypot(re - sr, im - si));
    }
    return n;
  };
  const double cand[3][2] = {{0.0, 0.0}, {tr_r / N, tr_i / N}, {0.5 * (rmin + rmax), 0.5 * (imin + imax)}};
  double best = 1e300;
  for (auto& cd : cand) {
    const double n = norm(cd[0], cd[1]);
    if (n < best) {
      best = n;
      mr = cd[0];
      mi = cd[1];
    }
  }
  return best;
}

// Spectral interval of the Hermitian H = i A for a skew-Hermitian generator A (column-major interleaved N x N):
// cyclic Jacobi on the real symmetric embedding [[Re H, -Im H], [Im H, Re H]], whose eigenvalues are H's, twice.
// Host-side, once per qoc_set_generators (N <= 64).
void herm_interval(const double* A, int N, double& lmin, double& lmax) {
  const int n = 2 * N;
  std::vector<double> S((size_t)n * n);
  auto at = [&](int r, int c) -> double& { return S[(size_t)r * n + c]; };
  for (int col = 0; col < N; ++col)
    for (int row = 0; row < N; ++row) {
      const double ar = A[2 * (row + (size_t)N * col)], ai = A[2 * (row + (size_t)N * col) + 1];
      const double hr = -ai, hi = ar;  // H = i A
      at(row, col) = hr;
      at(row + N, col + N) = hr;
      at(row + N, col) = hi;
      at(row, col + N) = -hi;
    }
  for (int r = 0; r < n; ++r)  // exact symmetry (A is skew-Hermitian to rounding)
    for (int c = r + 1; c < n; ++c) at(r, c) = at(c, r) = 0.5 * (at(r, c) + at(c, r));
  double fro = 0.0;
  for (double v : S) fro += v * v;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) off += at(p, q) * at(p, q);
    if (off <= 1e-32 * fro) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = at(p, q);
        if (std::fabs(apq) < 1e-300) continue;
        const double theta = (at(q, q) - at(p, p)) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double cs = 1.0 / std::sqrt(t * t + 1.0), sn = t * cs;
        for (int k = 0; k < n; ++k) {  // rows/columns p, q of the rotation J^T S J
          const double skp = at(k, p), skq = at(k, q);
          at(k, p) = cs * skp - sn * skq;
          at(k, q) = sn * skp + cs * skq;
        }
        for (int k = 0; k < n; ++k) {
          const double spk = at(p, k), sqk = at(q, k);
          at(p, k) = cs * spk - sn * sqk;
          at(q, k) = sn * spk + cs * sqk;
        }
      }
  }
  lmin = 1e300;
  lmax = -1e300;
  for (int k = 0; k < n; ++k) {
    lmin = std::min(lmin, at(k, k));
    lmax = std::max(lmax, at(k, k));
  }
}

// RCCL, resolved on first use (librccl.so.1 of the ROCm install).
RcclApi& rccl() {
  static RcclApi api;
  static bool tried = false;
  if (!tried) {
    tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (h) {
      api.getUniqueId = (decltype(api.getUniqueId))dlsym(h, "ncclGetUniqueId");
      api.commInitRank = (decltype(api.commInitRank))dlsym(h, "ncclCommInitRank");
      api.allGather = (decltype(api.allGather))dlsym(h, "ncclAllGather");
      api.commDestroy = (decltype(api.commDestroy))dlsym(h, "ncclCommDestroy");
      api.getErrorString = (decltype(api.getErrorString))dlsym(h, "ncclGetErrorString");
      api.ok = api.getUniqueId && api.commInitRank && api.allGather && api.commDestroy && api.getErrorString;
    }
  }
  return api;
}

// d_src: the caller's device u when it is not yet in d_u (the segmented forward copies it itself), d_J: the caller's J
// buffer (written by that launch; the other paths leave J in d_J)
int forward(qoc_ctx* c, const double* d_src = nullptr, double* d_J = nullptr) {
  c->X_lazy = false;  // every forward path but the segmented one writes x_k
  c->best_ready = false;
  c->fwd_kind = 0;
  if (blkseg_split_ok(c)) return blkseg_forward(c, d_src ? d_src : c->d_u, d_J);
  if (d_src && d_src != c->d_u)
    HIPCHK(c, hipMemcpyAsync(c->d_u, d_src, (size_t)c->B * c->nu * c->Nt * sizeof(double), hipMemcpyDeviceToDevice,
                             c->stream));
  int r = QOC_OK;
  if (blk_active(c)) r = blk_forward(c);
  else if (c->big) r = c->prec == QOC_FP64 ? big_forward<double>(c) : big_forward<float>(c);
  else r = c->prec == QOC_FP64 ? run_forward<double>(c) : run_forward<float>(c);
  if (r == QOC_OK && d_J && d_J != c->d_J)
    HIPCHK(c, hipMemcpyAsync(d_J, c->d_J, c->B * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  return r;
}
// stale: a device stale-u flag the segmented backward checks itself (queue_stale_check), or nullptr
int backward(qoc_ctx* c, int order, double* d_dJdu, const int* stale = nullptr) {
  // the segmented forward left G at every segment's end: the backward half only (x_k never formed); the stored block
  // propagators: the μ recurrence and the gradient on them
  if (c->fwd_kind == 1 && blkseg_ok(c, order)) return blkseg_backward(c, order, d_dJdu, stale);
  if (blkp_backward_ok(c, order)) return blkp_backward(c, d_dJdu, stale);
  if (c->cost_kind == QOC_COST_EXTERNAL || c->src_on) c->dead_dirty = true;  // λ may be nonzero on dead rows
  if (c->X_lazy) {  // after a segmented eval: the backward paths read x_k
    const int r = blku_states(c);
    if (r) return r;
  }
  c->L_is_mu = false;  // every backward path below writes λ itself (the fused block backward: on demand)
  c->L_lazy = false;
  c->last_eval_mode = 0;
  if (c->src_on && c->prop_method == QOC_PROP_TSIT5)
    return fail(c, QOC_ERR_UNSUPPORTED, "a co-state source (dL_dx) is not part of the Tsit5 path (compute_pwc_gradient)");
  if (blk_active(c)) return blk_backward(c, order, d_dJdu);
  if (c->big)
    return c->prec == QOC_FP64 ? big_backward<double>(c, order, d_dJdu) : big_backward<float>(c, order, d_dJdu);
  return c->prec == QOC_FP64 ? run_backward<double>(c, order, d_dJdu) : run_backward<float>(c, order, d_dJdu);
}

// the bitwise comparison of d_u with the u of the last propagate (src/gradient_computations.jl:37-39) on the stream,
// one launch: its device flag (returned in *dflag, for launches queued behind it) and the host-mapped flag c->h_flag,
// read at c->flag_ev (wait_stale_check).  The two device flags take turns, each check zeroing the next one's.
int queue_stale_check(qoc_ctx* c, const double* d_u, const int** dflag) {
  if (!c->h_flag) HIPCHK(c, hipHostMalloc((void**)&c->h_flag, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  if (!c->flag_ev) HIPCHK(c, hipEventCreateWithFlags(&c->flag_ev, hipEventDisableTiming));
  int* hdev = nullptr;
  HIPCHK(c, hipHostGetDevicePointer((void**)&hdev, c->h_flag, 0));
  const size_t nu_t = (size_t)c->B * c->nu * c->Nt;
  const int cur = c->flag_turn, nxt = cur ^ 1;
  c->flag_turn = nxt;
  *(volatile int*)c->h_flag = 0;  // no launch that writes it is pending: the last one's event was waited for
  const unsigned grid = (unsigned)std::max<size_t>(1, std::min<size_t>((nu_t + 255) / 256, 1024));
  hipLaunchKernelGGL(k_compare_u_flags, dim3(grid), dim3(256), 0, c->stream, d_u, c->d_u, nu_t, c->d_flag + cur,
                     c->d_flag + nxt, hdev);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->flag_ev, c->stream));
  if (dflag) *dflag = c->d_flag + cur;
  return QOC_OK;
}
int wait_stale_check(qoc_ctx* c) {
  HIPCHK(c, hipEventSynchronize(c->flag_ev));
  if (*(volatile int*)c->h_flag) return fail(c, QOC_ERR_STALE, "Cache data from other control signal u");
  return QOC_OK;
}

int check_ready(qoc_ctx* c) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (!c->have_gen) return fail(c, QOC_ERR_STATE, "generators not set (qoc_set_generators)");
  if (!c->have_x0) return fail(c, QOC_ERR_STATE, "x0 not set (qoc_set_x0)");
  if (!c->have_cost) return fail(c, QOC_ERR_STATE, "cost not set (qoc_set_cost)");
  HIPCHK(c, hipSetDevice(c->dev));
  return QOC_OK;
}

}  // namespace qoc_host

using namespace qoc_host;


extern "C" {

const char* qoc_last_error(const qoc_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int qoc_create(qoc_ctx** out, int device, int N, int m, int nu, int Nt, int B, int precision) {
  if (!out) return fail(nullptr, QOC_ERR_ARG, "out is null");
  *out = nullptr;
  if (N < 1 || m < 1 || nu < 1 || Nt < 1 || B < 1)
    return fail(nullptr, QOC_ERR_ARG, "invalid dimensions N=%d m=%d nu=%d Nt=%d B=%d", N, m, nu, Nt, B);
  if (precision != QOC_FP64 && precision != QOC_FP32) return fail(nullptr, QOC_ERR_ARG, "invalid precision");
  // LDS-resident kernels when the problem fits them, the chunked GEMM pipeline otherwise
  const bool small = expm_supported(N, precision) && N <= kChainMaxN &&
                     N <= (precision == QOC_FP64 ? chain_max_n<double>() : chain_max_n<float>()) && N * m <= 4 * CHAIN_THREADS;
  const bool force_big = getenv("QOC_FORCE_LARGE_N") && atoi(getenv("QOC_FORCE_LARGE_N")) != 0;
  if ((!small || force_big) && nu > 8)
    return fail(nullptr, QOC_ERR_UNSUPPORTED, "large-N path supports nu <= 8 (got %d)", nu);
  qoc_ctx* c = new qoc_ctx();
  c->big = !small || force_big;
  c->dev = device;
  c->N = N;
  c->m = m;
  c->m_user = m;
  c->nu = nu;
  c->Nt = Nt;
  c->B = B;
  c->prec = precision;
  c->esz = precision == QOC_FP64 ? 16 : 8;
  auto bail = [&](hipError_t e, const char* what) {
    fail(nullptr, QOC_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    qoc_destroy(c);
    return QOC_ERR_HIP;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess) return bail(e, "hipSetDevice");
  if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bail(e, "stream");
  const size_t NN = (size_t)N * N, Nm = (size_t)N * m;
  struct {
    void** p;
    size_t bytes;
  } allocs[] = {
      {&c->d_A, (nu + 1) * NN * c->esz},
      {&c->d_x0, (size_t)B * Nm * c->esz},
      {&c->d_Xt, Nm * c->esz},
      {(void**)&c->d_pmask, Nm},
      {(void**)&c->d_u, (size_t)B * nu * Nt * sizeof(double) + 16},  // + 16: slack past the last control
      {&c->d_U, (size_t)B * Nt * NN * c->esz},
      {&c->d_X, (size_t)B * (Nt + 1) * Nm * c->esz},
      {&c->d_L, (size_t)B * (Nt + 1) * Nm * c->esz},
      {(void**)&c->d_J, (size_t)B * sizeof(double)},
      {(void**)&c->d_coef, (size_t)B * 2 * m * sizeof(cx<double>)},
      {(void**)&c->d_rsec, (size_t)N},
      {(void**)&c->d_dJdu, (size_t)B * nu * Nt * sizeof(double)},
      {(void**)&c->d_flag, 2 * sizeof(int)},  // [0] the synchronous checks, [0] / [1] in turns the queued ones
      {(void**)&c->d_hist, 13 * 64 * sizeof(unsigned long long)},
      {(void**)&c->d_sink, TCHAIN_SINK * sizeof(double)},
      {(void**)&c->d_ps, ((size_t)std::max<long long>((long long)B * Nt, 16384) + 1) * sizeof(int)},
  };
  for (auto& a : allocs) {
    if ((e = hipMalloc(a.p, a.bytes)) != hipSuccess) return bail(e, "hipMalloc");
    c->dev_bytes += a.bytes;
  }
  if ((e = hipMemset(c->d_flag, 0, 2 * sizeof(int))) != hipSuccess) return bail(e, "hipMemset");
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0) c->ncu = ncu;
  }
  const bool env_kernel = getenv("QOC_GRAD_KERNEL") && atoi(getenv("QOC_GRAD_KERNEL")) != 0;
  const bool env_gemm = getenv("QOC_GRAD_GEMM") && atoi(getenv("QOC_GRAD_GEMM")) != 0;
  const size_t grr_lds = (size_t)2 * (nu + 1) * N * (precision == QOC_FP64 ? (N | 1) : ((N + 3) & ~3)) *
                         (precision == QOC_FP64 ? 8 : 4);
  c->grad_rr_any_m = !c->big && N <= 48 && (nu == 1 || nu == 2) && grr_lds <= 160 * 1024 && !env_kernel && !env_gemm;
  c->grad_rr = c->grad_rr_any_m && grad_rr_cols(m);
  c->grad_gemm = !c->grad_rr && !c->big && N >= 32 && nu <= 8 && !env_kernel;
  if (c->grad_rr) {
    const size_t cols = (size_t)B * (Nt + 1) * m;
    if ((e = hipMalloc(&c->d_gws, 2 * (size_t)N * cols * c->esz)) != hipSuccess) return bail(e, "hipMalloc");
    c->dev_bytes += 2 * (size_t)N * cols * c->esz;
  }
  if (c->grad_gemm) {
    const size_t cols = (size_t)B * (Nt + 1) * m;
    if ((e = hipMalloc(&c->d_AH, (nu + 1) * NN * c->esz)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&c->d_Cst, nu * NN * c->esz)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&c->d_gws, 6 * (size_t)N * cols * c->esz)) != hipSuccess) return bail(e, "hipMalloc");
    c->dev_bytes += (2 * nu + 1) * NN * c->esz + 6 * (size_t)N * cols * c->esz;
  }
  {
    const TShape sh = tchain_shape(N, m, precision == QOC_FP64);
    const size_t tl = (size_t)(nu + 1) * NN * c->esz + (size_t)2 * sh.S * sh.JT * chain_mpad(m, sh.CB) * c->esz + 512;
    const bool valu_ok = sh.JT > 0 && sh.NP > 0 && tl <= 160 * 1024;
    const bool mf_ok = precision == QOC_FP64 && tchain_mf_kq(N) > 0 && tchain_mf_waves(N, m) <= 16 &&
                       tchain_mf_lds(N, m, nu) <= 160 * 1024;
    c->tchain_ok = !c->big && nu <= TCHAIN_NUMAX && (precision == QOC_FP64 ? mf_ok || valu_ok : valu_ok);
    if (c->tchain_ok) {
      const size_t bytes[3] = {(nu + 1) * NN * c->esz, (size_t)B * Nt * sizeof(TStep),
                               TERM_SLOTS * sizeof(unsigned long long)};
      void** ptrs[3] = {&c->d_At, (void**)&c->d_steps, (void**)&c->d_terms};
      for (int i = 0; i < 3; ++i) {
        if ((e = hipMalloc(ptrs[i], bytes[i])) != hipSuccess) return bail(e, "hipMalloc");
        c->dev_bytes += bytes[i];
      }
      hipMemset(c->d_terms, 0, TERM_SLOTS * sizeof(unsigned long long));
    }
  }
  if (c->big) {
    // chunk of slices sized to a workspace of <= 8 GiB (and <= 1/8 of what is free)
    size_t freeb = 0, totalb = 0;
    (void)hipMemGetInfo(&freeb, &totalb);
    const size_t per_item = big_ws_elems_per_item(N, m) * c->esz;
    size_t budget = std::min<size_t>(8ull << 30, freeb / 8);
    const long long units = (long long)B * Nt;
    long long ch = std::max<long long>(1, (long long)(budget / per_item));
    ch = std::min<long long>(ch, units);
    ch = std::min<long long>(ch, 16384);
    if (getenv("QOC_CHUNK")) ch = std::max(1, std::min<int>(atoi(getenv("QOC_CHUNK")), (int)std::min<long long>(units, 16384)));
    c->chunk = (int)ch;
    if ((e = hipMalloc(&c->d_ws, (size_t)ch * per_item)) != hipSuccess) return bail(e, "hipMalloc (workspace)");
    if ((e = hipMalloc((void**)&c->d_red, ((size_t)ch + 8) * sizeof(double))) != hipSuccess)
      return bail(e, "hipMalloc");
    c->dev_bytes += (size_t)ch * per_item + ((size_t)ch + 8) * sizeof(double);
  }
  hipMemset(c->d_pmask, 0, Nm);
  hipMemset(c->d_hist, 0, 13 * 64 * sizeof(unsigned long long));
  c->chain_cb_fwd = getenv("QOC_CHAIN_CB_FWD") ? atoi(getenv("QOC_CHAIN_CB_FWD")) : 0;
  c->chain_cb_bwd = getenv("QOC_CHAIN_CB_BWD") ? atoi(getenv("QOC_CHAIN_CB_BWD")) : 0;
  c->expm_ps = getenv("QOC_EXPM_PS") && atoi(getenv("QOC_EXPM_PS")) != 0;
  c->expm_alg = (getenv("QOC_EXPM_PADE") && atoi(getenv("QOC_EXPM_PADE")) != 0) ? 0
                : (getenv("QOC_EXPM_LDS") && atoi(getenv("QOC_EXPM_LDS")) != 0)   ? 2
                                                                                   : 1;
  c->ode_kernel = (getenv("QOC_ODE_LDS") && atoi(getenv("QOC_ODE_LDS")) != 0) ? 1 : 0;
  if (getenv("QOC_BWD_CHUNKS")) c->bwd_chunks = std::max(1, atoi(getenv("QOC_BWD_CHUNKS")));
  if (getenv("QOC_BWD_LAST")) c->bwd_last_frac = atof(getenv("QOC_BWD_LAST"));
  if (getenv("QOC_BWD_PRIO")) c->bwd_prio = atoi(getenv("QOC_BWD_PRIO"));
  if (getenv("QOC_BWD_PRESTATE")) c->bwd_prestate = atoi(getenv("QOC_BWD_PRESTATE"));
  if (getenv("QOC_CONCURRENT")) c->concurrent = std::max(0, std::min(2, atoi(getenv("QOC_CONCURRENT"))));
  if (getenv("QOC_TCHAIN_ROT")) c->tchain_rot = atoi(getenv("QOC_TCHAIN_ROT"));
  hipMemset(c->d_L, 0, (size_t)B * (Nt + 1) * Nm * c->esz);
  *out = c;
  return QOC_OK;
}

void qoc_destroy(qoc_ctx* c) {
  if (!c) return;
  hipSetDevice(c->dev);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->comm && rccl().commDestroy) rccl().commDestroy(c->comm);
  if (c->d_best) hipFree(c->d_best);
  if (c->d_done) hipFree(c->d_done);
  if (c->d_tcoef) hipFree(c->d_tcoef);
  if (c->d_coef_mu) hipFree(c->d_coef_mu);
  if (c->d_brow) hipFree(c->d_brow);
  if (c->d_wrow) hipFree(c->d_wrow);
  if (c->d_wrow_live) hipFree(c->d_wrow_live);
  if (c->d_dead_rows) hipFree(c->d_dead_rows);
  if (c->d_gc_part) hipFree(c->d_gc_part);
  if (c->d_gseg) hipFree(c->d_gseg);
  if (c->d_blkp_ctab) hipFree(c->d_blkp_ctab);
  if (c->d_blkp_M) hipFree(c->d_blkp_M);
  if (c->d_blkp_ph) hipFree(c->d_blkp_ph);
  if (c->d_minmax) hipFree(c->d_minmax);
  if (c->h_minmax) hipHostFree(c->h_minmax);
  if (c->h_flag) hipHostFree(c->h_flag);
  if (c->flag_ev) hipEventDestroy(c->flag_ev);
  void* ptrs[] = {c->d_A, c->d_x0, c->d_Xt, c->d_pmask, c->d_u,    c->d_U,    c->d_X, c->d_L, c->d_u_lam, c->d_coef_lam, c->d_blkU, c->d_J_scr, c->d_coef_scr,
                  c->d_J, c->d_coef, c->d_dJdu, c->d_flag, c->d_hist, c->d_stage, c->d_ws, c->d_red, c->d_Bs, c->d_cstage, c->d_fws, c->d_AH, c->d_Cst, c->d_gws, c->d_pws, c->d_ps, c->d_At, c->d_steps, c->d_terms, c->d_src, c->d_rsec, c->d_sink, c->d_blkrec};
  for (void* p : ptrs)
    if (p) hipFree(p);
  for (auto& m : c->marks) {
    hipEventDestroy(m.a);
    hipEventDestroy(m.b);
  }
  for (auto& m : c->gmarks) {
    hipEventDestroy(m.a);
    hipEventDestroy(m.b);
  }
  for (auto e : c->event_pool) hipEventDestroy(e);
  for (auto e : c->sync_ev) hipEventDestroy(e);
  if (c->stream2) {
    hipStreamSynchronize(c->stream2);
    hipStreamDestroy(c->stream2);
  }
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

void* qoc_stream(qoc_ctx* c) { return c ? (void*)c->stream : nullptr; }

int qoc_synchronize(qoc_ctx* c) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return QOC_OK;
}

int qoc_set_generators(qoc_ctx* c, const double* A0, const double* const* Aj) {
  if (!c || !A0 || !Aj) return fail(c, QOC_ERR_ARG, "null argument");
  HIPCHK(c, hipSetDevice(c->dev));
  if (int r0 = blk_materialize(c)) return r0;  // x_k / λ_k kept lazily need the current system
  const size_t NN = (size_t)c->N * c->N;
  {  // host copy (compress_states needs block-diagonal generators; checked here and at qoc_set_compression)
    std::vector<double> g((size_t)(c->nu + 1) * 2 * NN);
    std::memcpy(g.data(), A0, 2 * NN * sizeof(double));
    for (int j = 0; j < c->nu; ++j) {
      if (!Aj[j]) return fail(c, QOC_ERR_ARG, "A[%d] is null", j);
      std::memcpy(g.data() + (j + 1) * 2 * NN, Aj[j], 2 * NN * sizeof(double));
    }
    g.swap(c->h_gen);
    if (c->packed && !gens_block_diagonal(c)) {
      g.swap(c->h_gen);
      return fail(c, QOC_ERR_ARG, "generators couple the two compress_states row blocks");
    }
  }
  int r = upload(c, A0, c->d_A, NN);
  for (int j = 0; j < c->nu && r == QOC_OK; ++j) {
    if (!Aj[j]) return fail(c, QOC_ERR_ARG, "A[%d] is null", j);
    r = upload(c, Aj[j], (char*)c->d_A + (j + 1) * NN * c->esz, NN);
  }
  if (r != QOC_OK) return r;
  if (c->d_AH) HIPCHK(c, launch_gen_aux(c));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  {  // ||A0||_1 (host copy): selects the one-pass k_expm_rr_mix when every slice has large norm anyway
    double nrm = 0.0;
    for (int col = 0; col < c->N; ++col) {
      double sum = 0.0;
      for (int row = 0; row < c->N; ++row) sum += std::hypot(A0[2 * (row + (size_t)c->N * col)], A0[2 * (row + (size_t)c->N * col) + 1]);
      nrm = std::max(nrm, sum);
    }
    c->a0norm = nrm;
    c->expm_run = (c->expm_alg == 1 && nrm > 4.0 * kTheta12 && !c->expm_ps) ? 0 : c->expm_alg;
  }
  c->big_rho_ok = false;
  if (c->big && !(getenv("QOC_BIG_NORM1") && atoi(getenv("QOC_BIG_NORM1")) != 0)) {
    // large-N path: 2-norm bounds of skew-Hermitian generators (ρ_j = ||A_j||_2) for the Taylor degree choice
    bool skew = true;
    for (int j = 0; j <= c->nu && skew; ++j) {
      const double* G = j == 0 ? A0 : Aj[j - 1];
      double amax = 0.0, dev = 0.0;
      for (int col = 0; col < c->N; ++col)
        for (int row = 0; row < c->N; ++row) {
          const size_t a = 2 * (row + (size_t)c->N * col), b = 2 * (col + (size_t)c->N * row);
          amax = std::max(amax, std::hypot(G[a], G[a + 1]));
          dev = std::max(dev, std::hypot(G[a] + G[b], G[a + 1] - G[b + 1]));
        }
      skew = dev <= 1e-13 * std::max(amax, 1e-300);
    }
    if (skew && c->nu < 9) {
      for (int j = 0; j <= c->nu; ++j) {
        double lmin, lmax;
        herm_extremes(j == 0 ? A0 : Aj[j - 1], c->N, lmin, lmax);
        const double rho = std::max(std::fabs(lmin), std::fabs(lmax));
        c->big_rho[j] = rho * (1.0 + 1e-12) + 4.0 * c->N * 2.3e-16 * rho + 1e-300;  // backward-error margin
      }
      c->big_rho_ok = true;
    }
  }
  if (c->tchain_ok) {  // shifted generators Ã_j = A_j - μ_j I and their norms for the Taylor-action chains
    tchain_thresholds(c->tprm, c->prec);
    const char* capenv = getenv("QOC_CAPTURE");
    c->cap_ok = c->prec == QOC_FP64 && !(capenv && atoi(capenv) == 0);
    c->tprm.pmin = c->cap_ok ? 2 : 1;  // the captured products are the first two of every slice
    // Chebyshev needs every Ã_j skew-Hermitian (A_j^H = -A_j, Schrödinger generators -i H Δt), so that
    // Ã_k = -i H̃_k has its spectrum on the imaginary axis within the bound ρ_k
    bool skew = true, exact = true;
    for (int j = 0; j <= c->nu && skew; ++j) {
      const double* G = j == 0 ? A0 : Aj[j - 1];
      double amax = 0.0, dev = 0.0;
      for (int col = 0; col < c->N; ++col)
        for (int row = 0; row < c->N; ++row) {
          const size_t a = 2 * (row + (size_t)c->N * col), b = 2 * (col + (size_t)c->N * row);
          amax = std::max(amax, std::hypot(G[a], G[a + 1]));
          dev = std::max(dev, std::hypot(G[a] + G[b], G[a + 1] - G[b + 1]));  // |A + A^H|
        }
      skew = dev <= 1e-13 * std::max(amax, 1e-300);
      exact = exact && dev <= 4.0 * 2.220446049250313e-16 * amax;  // -i H dt of an exactly Hermitian H: dev = 0
    }
    c->skew_exact = skew && exact;
    std::vector<double> sh(2 * NN);
    for (int j = 0; j <= c->nu && r == QOC_OK; ++j) {
      const double* G = j == 0 ? A0 : Aj[j - 1];
      double mr = 0, mi = 0;
      if (skew) {
        // the centre of H_j's spectral interval [λmin, λmax] (H_j = i A_j): Ã_j = -i (H_j - c_j I), and by Weyl's
        // inequality every H̃_k = Σ_j u_jk (H_j - c_j I) has its spectrum within ±(r_0 + Σ_j |u_jk| r_j),
        // r_j = (λmax - λmin) / 2 — the Chebyshev interval, tighter than the 1-norm (tunable bus: ρ 14.2 vs 19.5)
        double lmin, lmax;
        herm_interval(G, c->N, lmin, lmax);
        const double cen = 0.5 * (lmin + lmax), scale = std::max(std::fabs(lmin), std::fabs(lmax));
        mr = 0.0;
        mi = -cen;
        c->tprm.rad[j] = 0.5 * (lmax - lmin) + 1e-13 * scale + 1e-300;  // Jacobi's error is ~N eps |H|
      }
      std::memcpy(sh.data(), G, 2 * NN * sizeof(double));
      if (!skew) {
        c->tprm.nrm[j] = choose_shift(G, c->N, mr, mi);
      }
      for (int d = 0; d < c->N; ++d) {
        sh[2 * (d + (size_t)c->N * d)] -= mr;
        sh[2 * (d + (size_t)c->N * d) + 1] -= mi;
      }
      if (skew) {  // 1-norm of the shifted generator (the Taylor variant's bound)
        double nrm = 0.0;
        for (int col = 0; col < c->N; ++col) {
          double sum = 0.0;
          for (int row = 0; row < c->N; ++row)
            sum += std::hypot(sh[2 * (row + (size_t)c->N * col)], sh[2 * (row + (size_t)c->N * col) + 1]);
          nrm = std::max(nrm, sum);
        }
        c->tprm.nrm[j] = nrm;
      } else {
        c->tprm.rad[j] = c->tprm.nrm[j];
      }
      c->tprm.mur[j] = mr;
      c->tprm.mui[j] = mi;
      r = upload(c, sh.data(), (char*)c->d_At + j * NN * c->esz, NN);
      if (r == QOC_OK) HIPCHK(c, hipStreamSynchronize(c->stream));  // sh is reused
    }
    if (r != QOC_OK) return r;
    c->cheb_ok = skew;
    const char* poly = getenv("QOC_TCHAIN_POLY");
    c->cheb = skew && !(poly && !std::strcmp(poly, "taylor"));
    // Taylor action by default while the slices need moderately many terms: Chebyshev (fp64, skew-Hermitian)
    // up to ρ_0 = 25 without substeps (cavity 0.15, zz 0.05, tunable bus 9.1: measured faster than Padé-13
    // propagators there too), the Taylor variant while ||Ã_0||_1 <= 1; larger norms form propagators on MFMA
    const bool cheb_run = c->cheb && tchain_mf(c);
    const char* env = getenv("QOC_CHAIN");
    if (c->chain_req != QOC_CHAIN_AUTO) c->chain_mode = c->chain_req;
    else if (env && !std::strcmp(env, "taylor")) c->chain_mode = 1;
    else if (env && !std::strcmp(env, "expm")) c->chain_mode = 0;
    else c->chain_mode = (cheb_run ? c->tprm.rad[0] <= 25.0 : c->tprm.nrm[0] <= 1.0) ? 1 : 0;
  } else {
    c->chain_mode = 0;
    c->skew_exact = false;
  }
  if (c->tchain_ok) {  // invariant blocks of the generators (qoc_blk.hpp)
    c->int_ok = c->int_failed = false;  // the interpolated propagators belong to the old generators
    c->ichain_fwd = false;
    c->fwd_kind = 0;  // a split forward's propagators or coefficients belong to the old generators
    r = blk_detect(c);
    if (r) return r;
  } else {
    c->blk_nb = 0;
  }
  c->have_gen = true;
  c->have_prop = false;
  return QOC_OK;
}

int qoc_set_x0(qoc_ctx* c, const double* x0, int per_seed) {
  if (!c || !x0) return fail(c, QOC_ERR_ARG, "null argument");
  HIPCHK(c, hipSetDevice(c->dev));
  if (int r0 = blk_materialize(c)) return r0;  // x_k / λ_k kept lazily need the current system
  const size_t Nmu = (size_t)c->N * c->m_user, cnt = per_seed ? (size_t)c->B : 1;
  int r = upload_states(c, x0, c->d_x0, cnt, "x0");
  if (r != QOC_OK) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->h_x0.assign(x0, x0 + 2 * Nmu * cnt);
  c->x0_per_seed = per_seed ? 1 : 0;
  c->dead_dirty = true;  // rows live under the previous x0 may hold nonzero states
  c->have_x0 = true;
  c->have_prop = false;
  return QOC_OK;
}

int qoc_set_cost(qoc_ctx* c, int kind, const double* X_target, double n) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (kind != QOC_COST_TRACE && kind != QOC_COST_ZCAL && kind != QOC_COST_EXTERNAL)
    return fail(c, QOC_ERR_ARG, "unknown cost kind %d", kind);
  if (kind == QOC_COST_ZCAL && c->m_user != 4)
    return fail(c, QOC_ERR_ARG, "Only works for two-qubit gates, x_target must have four columns");
  if (kind != QOC_COST_EXTERNAL && !X_target) return fail(c, QOC_ERR_ARG, "X_target is null");
  if (kind == QOC_COST_TRACE && !(n != 0.0)) return fail(c, QOC_ERR_ARG, "normalisation n must be nonzero");
  HIPCHK(c, hipSetDevice(c->dev));
  if (int r0 = blk_materialize(c)) return r0;  // λ_k kept lazily needs the current target
  if (X_target) {
    int r = upload_states(c, X_target, c->d_Xt, 1, nullptr);
    if (r != QOC_OK) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->h_Xt.assign(X_target, X_target + (size_t)2 * c->N * c->m_user);
  } else {
    c->h_Xt.clear();
  }
  c->cost_kind = kind;
  c->cost_n = n;
  c->dead_dirty = true;  // rows live under the previous target may hold nonzero co-states
  c->have_cost = true;
  c->have_prop = false;
  return QOC_OK;
}

int qoc_set_state_penalty(qoc_ctx* c, const int* P, int np, const int* C, int nc, double mu) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if ((np > 0 && !P) || (nc > 0 && !C)) return fail(c, QOC_ERR_ARG, "null index list");
  std::vector<unsigned char> mask((size_t)c->N * c->m, 0);
  for (int a = 0; a < np; ++a) {
    if (P[a] < 0 || P[a] >= c->N) return fail(c, QOC_ERR_ARG, "penalty row %d out of range", P[a]);
    for (int bb = 0; bb < nc; ++bb) {
      if (C[bb] < 0 || C[bb] >= c->m_user) return fail(c, QOC_ERR_ARG, "penalty column %d out of range", C[bb]);
      // packed: an entry outside the two blocks is identically zero (no penalty, no gradient)
      const int col = c->packed ? c->pk_pos[c->h_rsec[P[a]]][C[bb]] : C[bb];
      if (col >= 0) mask[P[a] + (size_t)c->N * col] = 1;
    }
  }
  c->h_pen_rows.assign(P, P + np);
  c->h_pen_cols.assign(C, C + nc);
  HIPCHK(c, hipSetDevice(c->dev));
  // kernels queued by the asynchronous entry points may still read the mask: finish them first (the engine
  // stream is non-blocking, a null-stream copy would not wait for it)
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(c->d_pmask, mask.data(), mask.size(), hipMemcpyHostToDevice));
  c->mu = mu;  // affects J of the next propagate and dL/dx of the next sensitivity
  return QOC_OK;
}

int qoc_set_costate_source(qoc_ctx* c, const double* dLdx) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  HIPCHK(c, hipSetDevice(c->dev));
  HIPCHK(c, hipStreamSynchronize(c->stream));  // queued backward kernels may still read the old source
  if (!dLdx) {
    c->src_on = false;
    return QOC_OK;
  }
  const size_t cnt = (size_t)c->B * (c->Nt + 1), n = cnt * c->N * c->m_user;  // allocated for m_user >= m
  if (!c->d_src) {
    HIPCHK(c, hipMalloc(&c->d_src, n * c->esz));
    c->dev_bytes += n * c->esz;
  }
  int r = upload_states(c, dLdx, c->d_src, cnt, nullptr);
  if (r) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->src_on = true;
  return QOC_OK;
}

int qoc_set_compression(qoc_ctx* c, const int* rows1, int nr1, const int* cols1, int nc1, const int* rows2, int nr2,
                        const int* cols2, int nc2) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  HIPCHK(c, hipSetDevice(c->dev));
  if (int r0 = blk_materialize(c)) return r0;  // x_k / λ_k kept lazily are in the current layout
  HIPCHK(c, hipStreamSynchronize(c->stream));  // queued kernels may still read the packed buffers
  c->dead_dirty = true;
  const int N = c->N, mu_ = c->m_user;
  std::vector<unsigned char> rsec;
  std::vector<int> cols[2], pos[2];
  const bool on = nr1 > 0 || nr2 > 0;
  if (on) {
    if (!rows1 || !cols1 || !rows2 || !cols2 || nr1 < 0 || nr2 < 0 || nc1 < 0 || nc2 < 0)
      return fail(c, QOC_ERR_ARG, "null or negative index list");
    if (nr1 + nr2 != N) return fail(c, QOC_ERR_ARG, "the two row blocks must partition the %d rows (got %d + %d)", N, nr1, nr2);
    if (nc1 + nc2 != mu_)
      return fail(c, QOC_ERR_ARG, "the two column sets must partition the %d columns (got %d + %d)", mu_, nc1, nc2);
    rsec.assign(N, 255);
    for (int s = 0; s < 2; ++s)
      for (int a = 0; a < (s ? nr2 : nr1); ++a) {
        const int r = (s ? rows2 : rows1)[a];
        if (r < 0 || r >= N || rsec[r] != 255) return fail(c, QOC_ERR_ARG, "row %d out of range or in both blocks", r);
        rsec[r] = (unsigned char)s;
      }
    for (int s = 0; s < 2; ++s) pos[s].assign(mu_, -1);
    std::vector<char> seen(mu_, 0);
    for (int s = 0; s < 2; ++s)
      for (int a = 0; a < (s ? nc2 : nc1); ++a) {
        const int oc = (s ? cols2 : cols1)[a];
        if (oc < 0 || oc >= mu_ || seen[oc]) return fail(c, QOC_ERR_ARG, "column %d out of range or in both sets", oc);
        seen[oc] = 1;
        pos[s][oc] = (int)cols[s].size();
        cols[s].push_back(oc);
      }
  }
  // install, validate against the generators and x0 already set, roll back on error
  auto old_rsec = c->h_rsec;
  std::vector<int> old_cols[2] = {c->pk_cols[0], c->pk_cols[1]}, old_pos[2] = {c->pk_pos[0], c->pk_pos[1]};
  const bool old_packed = c->packed;
  const int old_m = c->m;
  auto restore = [&]() {
    c->h_rsec = old_rsec;
    for (int s = 0; s < 2; ++s) {
      c->pk_cols[s] = old_cols[s];
      c->pk_pos[s] = old_pos[s];
    }
    c->packed = old_packed;
    c->m = old_m;
  };
  c->packed = on;
  c->m = on ? std::max<int>(std::max<int>((int)cols[0].size(), (int)cols[1].size()), 1) : mu_;
  c->h_rsec = rsec;
  for (int s = 0; s < 2; ++s) {
    c->pk_cols[s] = cols[s];
    c->pk_pos[s] = pos[s];
  }
  if (on && c->have_gen && !gens_block_diagonal(c)) {
    restore();
    return fail(c, QOC_ERR_ARG, "generators couple the two compress_states row blocks");
  }
  int old_zmap[4];
  std::memcpy(old_zmap, c->zmap, sizeof(old_zmap));
  if (on && mu_ == 4)
    for (int oc = 0; oc < 4; ++oc) c->zmap[oc] = pos[0][oc] >= 0 ? pos[0][oc] : c->m + pos[1][oc];
  std::string saved_err = c->err;
  int r = QOC_OK;
  // packing on the host (pack_states reads h_rsec), validated before any device state changes
  if (c->have_x0) r = upload_states(c, c->h_x0.data(), c->d_x0, c->x0_per_seed ? (size_t)c->B : 1, "x0");
  if (r == QOC_OK && c->have_cost && !c->h_Xt.empty()) r = upload_states(c, c->h_Xt.data(), c->d_Xt, 1, nullptr);
  if (r == QOC_OK && on) {
    const hipError_t e = hipMemcpy(c->d_rsec, rsec.data(), N, hipMemcpyHostToDevice);
    if (e != hipSuccess) r = fail(c, QOC_ERR_HIP, "row sectors upload: %s", hipGetErrorString(e));
  }
  if (r != QOC_OK) {
    saved_err = c->err;
    restore();
    std::memcpy(c->zmap, old_zmap, sizeof(old_zmap));
    if (c->have_x0) upload_states(c, c->h_x0.data(), c->d_x0, c->x0_per_seed ? (size_t)c->B : 1, nullptr);
    if (c->have_cost && !c->h_Xt.empty()) upload_states(c, c->h_Xt.data(), c->d_Xt, 1, nullptr);
    if (!old_rsec.empty()) (void)hipMemcpy(c->d_rsec, old_rsec.data(), N, hipMemcpyHostToDevice);
    c->err = saved_err;
    return r;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (!c->h_pen_rows.empty() || c->mu != 0.0) {
    const std::vector<int> P = c->h_pen_rows, C = c->h_pen_cols;
    r = qoc_set_state_penalty(c, P.data(), (int)P.size(), C.data(), (int)C.size(), c->mu);
    if (r) return r;
  }
  c->src_on = false;  // a co-state source must be set again in the new layout
  c->grad_rr = c->grad_rr_any_m && grad_rr_cols(c->m);
  if (c->grad_rr && !c->d_gws) {  // the fused gradient's W0/W1 workspace (qoc_create sized none for m_user)
    const size_t bytes = 2 * (size_t)N * c->B * (c->Nt + 1) * mu_ * c->esz;
    HIPCHK(c, hipMalloc(&c->d_gws, bytes));
    c->dev_bytes += bytes;
  }
  c->have_prop = false;
  return QOC_OK;
}

int qoc_propagate_dev(qoc_ctx* c, const double* d_u, double* d_J) {
  int r = check_ready(c);
  if (r) return r;
  if (!d_u) return fail(c, QOC_ERR_ARG, "d_u is null");
  r = forward(c, d_u, d_J);  // u into d_u (kept for the stale check), J into d_J and the caller's buffer
  if (r) return r;
  c->have_prop = true;
  c->h_u.clear();  // host copy unknown for device-side u
  c->h_coef.clear();
  return QOC_OK;
}

int qoc_grape_sensitivity_dev(qoc_ctx* c, const double* d_u, int order, double* d_dJdu) {
  int r = check_ready(c);
  if (r) return r;
  if (!c->have_prop) return fail(c, QOC_ERR_STATE, "grape_sensitivity called before propagate");
  if (order < 0 || order > 4) return fail(c, QOC_ERR_ARG, "dUkdp_order must be 1..4 or QOC_DUKDP_EXACT (got %d)", order);
  if (c->cost_kind == QOC_COST_EXTERNAL)
    return fail(c, QOC_ERR_STATE, "QOC_COST_EXTERNAL needs qoc_grape_sensitivity (host lambda_final)");
  double* const out = d_dJdu ? d_dJdu : c->d_dJdu;
  if (!d_u || d_u == c->d_u) return backward(c, order, out);  // the cache's own u (the reference passes cache.u)
  const int* dflag = nullptr;
  if ((r = queue_stale_check(c, d_u, &dflag))) return r;
  if ((c->fwd_kind == 1 && blkseg_ok(c, order)) || blkp_backward_ok(c, order)) {
    // the split backward's launches read the flag themselves and write nothing on a stale u: they are queued behind
    // the check, and the host waits for the check alone, not for them (the stream never idles between the calls)
    const bool lmu = c->L_is_mu, llazy = c->L_lazy;
    const int lmode = c->last_eval_mode;
    r = backward(c, order, out, dflag);
    const int w = wait_stale_check(c);
    if (w) {  // nothing was written: the co-states are still the last grape_sensitivity's
      c->L_is_mu = lmu;
      c->L_lazy = llazy;
      c->last_eval_mode = lmode;
    }
    return w ? w : r;
  }
  if ((r = wait_stale_check(c))) return r;
  return backward(c, order, out);
}

int qoc_eval_dev(qoc_ctx* c, const double* d_u, int order, double* d_J, double* d_dJdu) {
  if (c && c->cost_kind == QOC_COST_EXTERNAL)
    return fail(c, QOC_ERR_STATE, "qoc_eval_dev needs a device-side cost (TRACE or ZCAL)");
  if (c) c->fwd_kind = 0;  // whatever runs below leaves no split forward behind
  if (c && c->have_gen && c->concurrent && blkseg_ok(c, order)) {
    // block propagators with the time axis in segments: one launch reads u (and copies it to d_u) and writes J and
    // dJdu; x_k and λ_k are rebuilt on demand (qoc_blkseg.hpp)
    int r = check_ready(c);
    if (r) return r;
    if (!d_u) return fail(c, QOC_ERR_ARG, "d_u is null");
    c->have_prop = false;
    r = blkseg_eval(c, order, d_u, d_J, d_dJdu ? d_dJdu : c->d_dJdu);
    if (r) return r;
    c->props_since_reset++;
    c->have_prop = true;
    c->h_u.clear();
    c->h_coef.clear();
    return QOC_OK;
  }
  if (c) {
    c->X_lazy = false;  // the other eval paths write x_k
    c->best_ready = false;
  }
  if (c && c->have_gen && (blk_concurrent_ok(c, order) || tchain_concurrent_ok(c, order))) {
    // forward chain and the μ recurrence side by side (tchain_eval_concurrent)
    int r = check_ready(c);
    if (r) return r;
    if (!d_u) return fail(c, QOC_ERR_ARG, "d_u is null");
    const size_t nu_t = (size_t)c->B * c->nu * c->Nt;
    if (d_u != c->d_u) HIPCHK(c, hipMemcpyAsync(c->d_u, d_u, nu_t * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    c->have_prop = false;
    c->L_lazy = false;
    r = blk_concurrent_ok(c, order)  ? blk_eval_concurrent(c, order, d_dJdu ? d_dJdu : c->d_dJdu)
        : c->prec == QOC_FP64 ? tchain_eval_concurrent<double>(c, d_dJdu ? d_dJdu : c->d_dJdu)
                              : tchain_eval_concurrent<float>(c, d_dJdu ? d_dJdu : c->d_dJdu);
    if (r) return r;
    c->props_since_reset++;
    if (d_J && d_J != c->d_J)
      HIPCHK(c, hipMemcpyAsync(d_J, c->d_J, c->B * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    c->have_prop = true;
    c->h_u.clear();
    c->h_coef.clear();
    return QOC_OK;
  }
  int r = qoc_propagate_dev(c, d_u, d_J);
  if (r) return r;
  if (order < 0 || order > 4) return fail(c, QOC_ERR_ARG, "dUkdp_order must be 1..4 or QOC_DUKDP_EXACT (got %d)", order);
  return backward(c, order, d_dJdu ? d_dJdu : c->d_dJdu);
}

int qoc_propagate(qoc_ctx* c, const double* u, double* J_out) {
  int r = check_ready(c);
  if (r) return r;
  if (!u) return fail(c, QOC_ERR_ARG, "u is null");
  const size_t nu_t = (size_t)c->B * c->nu * c->Nt;
  HIPCHK(c, hipMemcpyAsync(c->d_u, u, nu_t * sizeof(double), hipMemcpyHostToDevice, c->stream));
  r = forward(c);
  if (r) return r;
  if (J_out) HIPCHK(c, hipMemcpyAsync(J_out, c->d_J, c->B * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->h_u.assign(u, u + nu_t);
  c->h_coef.clear();
  c->have_prop = true;
  return QOC_OK;
}

int qoc_grape_sensitivity(qoc_ctx* c, const double* u, int order, const double* lambda_final, double* dJdu_out) {
  int r = check_ready(c);
  if (r) return r;
  if (!c->have_prop) return fail(c, QOC_ERR_STATE, "grape_sensitivity called before propagate");
  if (order < 0 || order > 4) return fail(c, QOC_ERR_ARG, "dUkdp_order must be 1..4 or QOC_DUKDP_EXACT (got %d)", order);
  const size_t nu_t = (size_t)c->B * c->nu * c->Nt;
  if (!u) return fail(c, QOC_ERR_ARG, "u is null");
  if (c->h_u.size() == nu_t) {
    if (std::memcmp(u, c->h_u.data(), nu_t * sizeof(double)) != 0)
      return fail(c, QOC_ERR_STALE, "Cache data from other control signal u");
  } else {
    // last propagate came from device memory: compare on the device
    HIPCHK(c, hipMemcpyAsync(c->d_dJdu, u, nu_t * sizeof(double), hipMemcpyHostToDevice, c->stream));
    if ((r = queue_stale_check(c, c->d_dJdu, nullptr))) return r;
    if ((r = wait_stale_check(c))) return r;
  }
  if (c->cost_kind == QOC_COST_EXTERNAL) {
    if (!lambda_final) return fail(c, QOC_ERR_ARG, "lambda_final is required for QOC_COST_EXTERNAL");
    // λ_{Nt+1} for every seed lives at Lam[b][Nt]
    const size_t Nm = (size_t)c->N * c->m, Nmu = (size_t)c->N * c->m_user;
    for (int b = 0; b < c->B; ++b) {
      r = upload_states(c, lambda_final + 2 * Nmu * b, (char*)c->d_L + ((size_t)b * (c->Nt + 1) + c->Nt) * Nm * c->esz,
                        1, nullptr);
      if (r) return r;
    }
  }
  r = backward(c, order, c->d_dJdu);
  if (r) return r;
  if (dJdu_out)
    HIPCHK(c, hipMemcpyAsync(dJdu_out, c->d_dJdu, nu_t * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return QOC_OK;
}

int qoc_get_states(qoc_ctx* c, int seed, int k, double* x_out) {
  if (!c || !x_out) return fail(c, QOC_ERR_ARG, "null argument");
  if (!c->have_prop) return fail(c, QOC_ERR_STATE, "no propagated states");
  if (k == -1) k = c->Nt;
  if (seed < 0 || seed >= c->B || k < 0 || k > c->Nt) return fail(c, QOC_ERR_ARG, "index out of range");
  HIPCHK(c, hipSetDevice(c->dev));
  if (c->X_lazy) {  // after a segmented eval: the states are rebuilt on demand
    const int r = blku_states(c);
    if (r) return r;
  }
  const size_t Nm = (size_t)c->N * c->m;
  return download_states(c, (char*)c->d_X + ((size_t)seed * (c->Nt + 1) + k) * Nm * c->esz, x_out);
}

int qoc_get_costates(qoc_ctx* c, int seed, int k, double* lam_out) {
  if (!c || !lam_out) return fail(c, QOC_ERR_ARG, "null argument");
  if (k == -1) k = c->Nt;
  if (seed < 0 || seed >= c->B || k < 0 || k > c->Nt) return fail(c, QOC_ERR_ARG, "index out of range");
  HIPCHK(c, hipSetDevice(c->dev));
  const size_t Nm = (size_t)c->N * c->m;
  const void* src = (char*)c->d_L + ((size_t)seed * (c->Nt + 1) + k) * Nm * c->esz;
  if (c->L_lazy) {
    const int r = blku_costates(c);
    if (r) return r;
  }
  if (!c->L_is_mu) return download_states(c, src, lam_out);
  // the concurrent eval left μ_k: λ_k = coef ⊙ μ_k (per row sector and packed column, lam_coef)
  std::vector<double> mu(2 * Nm), cf(4 * (size_t)c->m);
  int r = download(c, src, mu.data(), Nm);
  if (r) return r;
  HIPCHK(c, hipMemcpy(cf.data(), c->d_coef_mu + (size_t)seed * 2 * c->m, 2 * (size_t)c->m * sizeof(cx<double>),
                      hipMemcpyDeviceToHost));
  for (int col = 0; col < c->m; ++col)
    for (int row = 0; row < c->N; ++row) {
      const int sct = c->packed ? c->h_rsec[row] : 0;
      const double fr = cf[2 * (sct * c->m + col)], fi = cf[2 * (sct * c->m + col) + 1];
      double* v = mu.data() + 2 * (row + (size_t)c->N * col);
      const double vr = v[0], vi = v[1];
      v[0] = fr * vr - fi * vi;
      v[1] = fr * vi + fi * vr;
    }
  if (!c->packed) {
    std::memcpy(lam_out, mu.data(), 2 * Nm * sizeof(double));
    return QOC_OK;
  }
  unpack_states(c, mu.data(), lam_out);
  return QOC_OK;
}

int qoc_get_propagator(qoc_ctx* c, int seed, int k, double* U_out) {
  if (!c || !U_out) return fail(c, QOC_ERR_ARG, "null argument");
  if (!c->have_prop) return fail(c, QOC_ERR_STATE, "no propagators");
  if (c->prop_method == QOC_PROP_TSIT5) return fail(c, QOC_ERR_STATE, "the Tsit5 path does not form propagators");
  if (seed < 0 || seed >= c->B || k < 0 || k >= c->Nt) return fail(c, QOC_ERR_ARG, "index out of range");
  HIPCHK(c, hipSetDevice(c->dev));
  const size_t NN = (size_t)c->N * c->N, unit = (size_t)seed * c->Nt + k;
  if (c->chain_mode == 1) {  // the Taylor-action chains form no propagators: exp(A_k) of this slice on demand
    hipError_t e = launch_expm(c->prec, c->stream, c->N, c->nu, 1, c->d_A, c->d_u + unit * c->nu, nullptr,
                               (char*)c->d_U + unit * NN * c->esz, nullptr, nullptr, nullptr, c->expm_run,
                               c->d_hist + 5 * 64, c->d_ps, c->a0norm > 4.0 * kTheta12);
    if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_expm (propagator on demand): %s", hipGetErrorString(e));
  }
  return download(c, (char*)c->d_U + unit * NN * c->esz, U_out, NN);
}

int qoc_set_profiling(qoc_ctx* c, int enable) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  c->profiling = enable != 0;
  return QOC_OK;
}

int qoc_phase_times(qoc_ctx* c, double* ms_out, long long* launches_out, int reset) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (auto& m : c->marks) {
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, m.a, m.b));
    c->phase_ms[m.phase] += ms;
    c->phase_n[m.phase] += 1;
    c->event_pool.push_back(m.a);
    c->event_pool.push_back(m.b);
  }
  c->marks.clear();
  for (auto& m : c->gmarks) {
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, m.a, m.b));
    c->gemm_ms += ms;
    c->gemm_n += 1;
    c->gemm_flops += m.flops;
    c->event_pool.push_back(m.a);
    c->event_pool.push_back(m.b);
  }
  c->gmarks.clear();
  for (int p = 0; p < 4; ++p) {
    if (ms_out) ms_out[p] = c->phase_ms[p];
    if (launches_out) launches_out[p] = c->phase_n[p];
    if (reset) {
      c->phase_ms[p] = 0;
      c->phase_n[p] = 0;
    }
  }
  return QOC_OK;
}

int qoc_gemm_stats(qoc_ctx* c, double* ms, long long* launches, double* flops, int reset) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  int r = qoc_phase_times(c, nullptr, nullptr, 0);  // drains pending marks
  if (r) return r;
  if (ms) *ms = c->gemm_ms;
  if (launches) *launches = c->gemm_n;
  if (flops) *flops = c->gemm_flops;
  if (reset) {
    c->gemm_ms = 0;
    c->gemm_flops = 0;
    c->gemm_n = 0;
  }
  return QOC_OK;
}

int qoc_set_spline_basis(qoc_ctx* c, const double* Bs, int ns) {
  if (!c || !Bs) return fail(c, QOC_ERR_ARG, "null argument");
  if (ns < 1) return fail(c, QOC_ERR_ARG, "nsplines must be >= 1 (got %d)", ns);
  HIPCHK(c, hipSetDevice(c->dev));
  HIPCHK(c, hipStreamSynchronize(c->stream));  // queued spline kernels may still read the old basis
  if (c->d_Bs) HIPCHK(c, hipFree(c->d_Bs));
  if (c->d_cstage) HIPCHK(c, hipFree(c->d_cstage));
  c->d_Bs = nullptr;
  c->d_cstage = nullptr;
  HIPCHK(c, hipMalloc((void**)&c->d_Bs, (size_t)c->Nt * ns * sizeof(double)));
  HIPCHK(c, hipMalloc((void**)&c->d_cstage, (size_t)2 * c->B * ns * c->nu * sizeof(double)));
  HIPCHK(c, hipMemcpy(c->d_Bs, Bs, (size_t)c->Nt * ns * sizeof(double), hipMemcpyHostToDevice));
  c->ns = ns;
  // states and co-states of a spline propagate belong to the old basis' u: qoc_sensitivity_spline must now see
  // them as stale (QOC_ERR_STALE), even for the same coefficients
  c->h_coef.clear();
  return QOC_OK;
}

int qoc_eval_spline_dev(qoc_ctx* c, const double* d_c, int order, double* d_J, double* d_dJdc) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (!c->ns) return fail(c, QOC_ERR_STATE, "spline basis not set (qoc_set_spline_basis)");
  if (!d_c) return fail(c, QOC_ERR_ARG, "d_c is null");
  HIPCHK(c, hipSetDevice(c->dev));
  const long long nuT = (long long)c->B * c->Nt * c->nu;
  const unsigned blocks = (unsigned)std::min<long long>((nuT + 255) / 256, 4096);
  hipLaunchKernelGGL(k_spline_u, dim3(blocks), dim3(256), 0, c->stream, c->B, c->Nt, c->ns, c->nu, c->d_Bs, d_c,
                     c->d_u);
  HIPCHK(c, hipGetLastError());
  int r = qoc_eval_dev(c, c->d_u, order, d_J, c->d_dJdu);
  if (r) return r;
  if (d_dJdc) {
    const long long outs = (long long)c->B * c->ns * c->nu;
    const unsigned gb = (unsigned)std::min<long long>((outs * 64 + 255) / 256, 4096);
    hipLaunchKernelGGL(k_spline_grad, dim3(gb), dim3(256), 0, c->stream, c->B, c->Nt, c->ns, c->nu, c->d_Bs,
                       c->d_dJdu, d_dJdc);
    HIPCHK(c, hipGetLastError());
  }
  return QOC_OK;
}

int qoc_eval_spline(qoc_ctx* c, const double* coef, int order, double* J_out, double* dJdc_out) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (!c->ns) return fail(c, QOC_ERR_STATE, "spline basis not set (qoc_set_spline_basis)");
  if (!coef) return fail(c, QOC_ERR_ARG, "c is null");
  HIPCHK(c, hipSetDevice(c->dev));
  const size_t nc = (size_t)c->B * c->ns * c->nu;
  HIPCHK(c, hipMemcpyAsync(c->d_cstage, coef, nc * sizeof(double), hipMemcpyHostToDevice, c->stream));
  int r = qoc_eval_spline_dev(c, c->d_cstage, order, c->d_J, dJdc_out ? c->d_cstage + nc : nullptr);
  if (r) return r;
  if (J_out) HIPCHK(c, hipMemcpyAsync(J_out, c->d_J, c->B * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (dJdc_out)
    HIPCHK(c, hipMemcpyAsync(dJdc_out, c->d_cstage + nc, nc * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return QOC_OK;
}

int qoc_propagate_spline(qoc_ctx* c, const double* coef, double* J_out) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (!c->ns) return fail(c, QOC_ERR_STATE, "spline basis not set (qoc_set_spline_basis)");
  if (!coef) return fail(c, QOC_ERR_ARG, "c is null");
  HIPCHK(c, hipSetDevice(c->dev));
  const size_t nc = (size_t)c->B * c->ns * c->nu;
  HIPCHK(c, hipMemcpyAsync(c->d_cstage, coef, nc * sizeof(double), hipMemcpyHostToDevice, c->stream));
  const long long nuT = (long long)c->B * c->Nt * c->nu;
  const unsigned blocks = (unsigned)std::min<long long>((nuT + 255) / 256, 4096);
  hipLaunchKernelGGL(k_spline_u, dim3(blocks), dim3(256), 0, c->stream, c->B, c->Nt, c->ns, c->nu, c->d_Bs,
                     c->d_cstage, c->d_u);
  HIPCHK(c, hipGetLastError());
  c->h_coef.clear();
  int r = qoc_propagate_dev(c, c->d_u, nullptr);
  if (r) return r;
  if (J_out) HIPCHK(c, hipMemcpyAsync(J_out, c->d_J, c->B * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->h_coef.assign(coef, coef + nc);
  return QOC_OK;
}

int qoc_sensitivity_spline(qoc_ctx* c, const double* coef, int order, double* dJdc_out) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (!c->ns) return fail(c, QOC_ERR_STATE, "spline basis not set (qoc_set_spline_basis)");
  if (!coef) return fail(c, QOC_ERR_ARG, "c is null");
  int r = check_ready(c);
  if (r) return r;
  const size_t nc = (size_t)c->B * c->ns * c->nu;
  if (!c->have_prop || c->h_coef.size() != nc || std::memcmp(coef, c->h_coef.data(), nc * sizeof(double)) != 0)
    return fail(c, QOC_ERR_STALE, "Cache data from other control signal u");
  if (order < 0 || order > 4) return fail(c, QOC_ERR_ARG, "dUkdp_order must be 1..4 or QOC_DUKDP_EXACT (got %d)", order);
  if (c->cost_kind == QOC_COST_EXTERNAL)
    return fail(c, QOC_ERR_STATE, "qoc_sensitivity_spline needs a device-side cost (TRACE or ZCAL)");
  r = backward(c, order, c->d_dJdu);
  if (r) return r;
  if (dJdc_out) {
    const long long outs = (long long)c->B * c->ns * c->nu;
    const unsigned gb = (unsigned)std::min<long long>((outs * 64 + 255) / 256, 4096);
    hipLaunchKernelGGL(k_spline_grad, dim3(gb), dim3(256), 0, c->stream, c->B, c->Nt, c->ns, c->nu, c->d_Bs,
                       c->d_dJdu, c->d_cstage + nc);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(dJdc_out, c->d_cstage + nc, nc * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return QOC_OK;
}

int qoc_spline_constraints_dev(qoc_ctx* c, const double* d_c, double* d_g, double* d_gjac) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (!c->ns) return fail(c, QOC_ERR_STATE, "spline basis not set (qoc_set_spline_basis)");
  if (!d_c || !d_g) return fail(c, QOC_ERR_ARG, "null argument");
  HIPCHK(c, hipSetDevice(c->dev));
  hipLaunchKernelGGL(k_spline_constraints, dim3(c->B), dim3(256), 0, c->stream, c->ns, c->nu, d_c, d_g, d_gjac);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}

int qoc_set_propagation(qoc_ctx* c, int method, int nsub) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (int r0 = blk_materialize(c)) return r0;  // x_k / λ_k kept lazily are rebuilt by the current path
  if (method != QOC_PROP_EXPM && method != QOC_PROP_TSIT5) return fail(c, QOC_ERR_ARG, "unknown method %d", method);
  if (method == QOC_PROP_TSIT5) {
    if (nsub < 1) return fail(c, QOC_ERR_ARG, "nsub must be >= 1 (got %d)", nsub);
    if (c->big || c->N > 64)
      return fail(c, QOC_ERR_UNSUPPORTED, "the Tsit5 path runs on the LDS-resident sizes (N <= 64)");
    c->nsub = nsub;
  }
  c->prop_method = method;
  c->have_prop = false;
  return QOC_OK;
}

int qoc_propagate_envelope(qoc_ctx* c, int kind, const double* params, int np, double tgate, double dt, double* J_out,
                           double* x_out) {
  int r = check_ready(c);
  if (r) return r;
  if (!params || np < 1 || np > 64) return fail(c, QOC_ERR_ARG, "bad parameter array");
  if (kind < QOC_ENV_TUNABLE_BUS || kind > QOC_ENV_SINEBASIS) return fail(c, QOC_ERR_ARG, "unknown envelope %d", kind);
  const int need_nu = kind == QOC_ENV_TUNABLE_BUS ? 1 : 2;
  if (c->nu != need_nu) return fail(c, QOC_ERR_ARG, "envelope %d drives %d controls, context has nu=%d", kind, need_nu, c->nu);
  if (c->big || c->N > 64) return fail(c, QOC_ERR_UNSUPPORTED, "the Tsit5 path runs on the LDS-resident sizes (N <= 64)");
  if (!(dt > 0) || !(tgate > 0)) return fail(c, QOC_ERR_ARG, "tgate and dt must be positive");
  const long long nsteps = (long long)std::llround(tgate / dt);
  const size_t env_lds = (size_t)(c->nu + 1) * c->N * c->N * c->esz;
  if (env_lds > 160 * 1024) return fail(c, QOC_ERR_UNSUPPORTED, "generators (%zu B) exceed the 160 KiB LDS", env_lds);
  double* dP = nullptr;
  HIPCHK(c, hipMalloc((void**)&dP, (size_t)c->B * np * sizeof(double)));
  hipError_t e = hipMemcpy(dP, params, (size_t)c->B * np * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_envelope(c, kind, dP, np, dt, nsteps);
  c->best_ready = false;  // J is rewritten below
  if (e == hipSuccess && c->cost_kind != QOC_COST_EXTERNAL) e = launch_terminal_cost(c);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess && J_out && c->cost_kind != QOC_COST_EXTERNAL)
    e = hipMemcpy(J_out, c->d_J, c->B * sizeof(double), hipMemcpyDeviceToHost);
  hipFree(dP);
  if (e == hipSuccess && x_out) {
    const size_t Nm = (size_t)c->N * c->m, Nmu = (size_t)c->N * c->m_user;
    for (int b = 0; b < c->B; ++b) {
      int r2 = download_states(c, (char*)c->d_X + ((size_t)b * (c->Nt + 1) + c->Nt) * Nm * c->esz, x_out + 2 * Nmu * b);
      if (r2) return r2;
    }
  }
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "qoc_propagate_envelope: %s", hipGetErrorString(e));
  c->have_prop = false;  // states other than x(tgate) are not stored
  return QOC_OK;
}

int qoc_get_info_n(qoc_ctx* c, long long* info, int n) {
  if (n < QOC_INFO_ENTRIES)
    return fail(c, QOC_ERR_ARG, "info buffer holds %d entries, QOC_INFO_ENTRIES = %d", n, QOC_INFO_ENTRIES);
  return qoc_get_info(c, info);
}

int qoc_get_info(qoc_ctx* c, long long* info) {
  if (!c || !info) return fail(c, QOC_ERR_ARG, "null argument");
  info[0] = c->big ? 1 : 0;
  info[1] = c->chunk;
  info[2] = c->ns_iters;
  info[3] = (long long)c->dev_bytes;
  info[4] = c->chain_mode;
  info[5] = c->big ? c->expm_alg : c->expm_run;  // the large-N pipeline keeps its own (Taylor / Padé) choice
  info[6] = c->chain_mode == 1 && c->cheb && tchain_mf(c) ? 1 : 0;  // Taylor-action chains: Chebyshev terms
  info[7] = c->m;  // state columns the kernels run on (< the caller's m when compress_states packing is on)
  info[8] = c->last_eval_mode;  // last backward: 0 other, 1 captured products, 2 / 3 / 4 concurrent μ recurrence, 5 fused block gradient, 6 segmented block eval, 7 stored propagators of blocks of 5..16 rows
  info[9] = c->fwd_captured ? 1 : 0;
  // 6: the last eval ran the stored-propagator chains of blocks of 5..16 rows (propagate / grape_sensitivity: 4)
  info[11] = c->fwd_kind;
  info[13] = c->ichain_last;  // the last eval / propagate on blocks of 5..16 rows: interpolating chains (2: triangle)
  info[12] = c->last_int_D;  // the stored block propagators' last formation: interpolation degree in u (0: exponentials)
  info[10] = blk_active(c) ? (blku_on(c) ? 5 : blkp_on(c) && c->last_eval_mode == 7 ? 6 : blk_rot(c) ? 4 : 3) : c->big || c->chain_mode != 1 || !tchain_mf(c) ? 0 : tchain_mf_rot(c) ? 2 : 1;
  return QOC_OK;
}

int qoc_set_chain(qoc_ctx* c, int mode) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (int r0 = blk_materialize(c)) return r0;  // x_k / λ_k kept lazily are rebuilt by the current path
  if (mode != QOC_CHAIN_AUTO && mode != QOC_CHAIN_PROPAGATORS && mode != QOC_CHAIN_TAYLOR)
    return fail(c, QOC_ERR_ARG, "unknown chain mode %d", mode);
  if (mode == QOC_CHAIN_TAYLOR && !c->tchain_ok)
    return fail(c, QOC_ERR_UNSUPPORTED, "Taylor-action chains need N <= 48 (fp64) / 64 (fp32), nu <= 8 and the "
                                        "generators within the 160 KiB LDS");
  c->chain_req = mode;
  if (mode == QOC_CHAIN_AUTO)
    mode = c->tchain_ok && c->have_gen &&
                   (c->cheb && tchain_mf(c) ? c->tprm.rad[0] <= 25.0 : c->tprm.nrm[0] <= 1.0) ? 1 : 0;
  c->chain_mode = mode;
  c->have_prop = false;
  return QOC_OK;
}

int qoc_comm_unique_id(void* id_out) {
  if (!id_out) return fail(nullptr, QOC_ERR_ARG, "id_out is null");
  RcclApi& r = rccl();
  if (!r.ok) return fail(nullptr, QOC_ERR_UNSUPPORTED, "RCCL (librccl.so.1) not available");
  ncclUniqueId id;
  const ncclResult_t e = r.getUniqueId(&id);
  if (e != ncclSuccess) return fail(nullptr, QOC_ERR_HIP, "ncclGetUniqueId: %s", r.getErrorString(e));
  std::memcpy(id_out, &id, sizeof(id));
  return QOC_OK;
}

int qoc_comm_init(qoc_ctx* c, int world, int rank, const void* id, long long seed_offset) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (world < 1 || rank < 0 || rank >= world) return fail(c, QOC_ERR_ARG, "invalid rank %d of %d", rank, world);
  if (world > 1 && !id) return fail(c, QOC_ERR_ARG, "unique id is null");
  HIPCHK(c, hipSetDevice(c->dev));
  RcclApi& r = rccl();
  // any previous communicator is dropped first; until the new one exists the context covers its own seeds
  if (c->comm) {
    r.commDestroy(c->comm);
    c->comm = nullptr;
  }
  if (c->d_best) HIPCHK(c, hipFree(c->d_best));
  c->d_best = nullptr;
  c->best_ready = false;
  c->world = 1;
  c->rank = 0;
  c->seed_offset = 0;
  double* best = nullptr;
  HIPCHK(c, hipMalloc((void**)&best, (size_t)(4 + 2 * world) * sizeof(double)));
  // With a unique id a real RCCL communicator is created, also for world = 1 (a one-rank all-gather through the
  // same code path as the multi-GPU run); without one (world = 1 only) the context covers its own seeds.
  ncclComm_t comm = nullptr;
  if (id) {
    if (!r.ok) {
      hipFree(best);
      return fail(c, QOC_ERR_UNSUPPORTED, "RCCL (librccl.so.1) not available");
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const ncclResult_t e = r.commInitRank(&comm, world, uid, rank);
    if (e != ncclSuccess || !comm) {
      hipFree(best);
      return fail(c, QOC_ERR_HIP, "ncclCommInitRank (rank %d of %d): %s", rank, world, r.getErrorString(e));
    }
  }
  c->comm = comm;
  c->d_best = best;
  c->world = world;
  c->rank = rank;
  c->seed_offset = seed_offset;
  return QOC_OK;
}

int qoc_comm_ranks(qoc_ctx* c) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  return c->comm ? c->world : 0;
}

int qoc_allgather_best_dev(qoc_ctx* c, double* d_out) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  HIPCHK(c, hipSetDevice(c->dev));
  if (!c->d_best) {  // no communicator: this context alone (world 1, seed offset 0)
    HIPCHK(c, hipMalloc((void**)&c->d_best, 6 * sizeof(double)));
    c->world = 1;
    c->rank = 0;
  }
  double* res = c->d_best + 2 + 2 * c->world;
  double* slot = c->d_best + 2 + 2 * c->rank;  // this rank's pair in the gathered array (in-place all-gather)
  // one rank, and the eval already wrote the final pair into res and the registered output: nothing to queue
  if (c->best_ready && c->best_direct && c->world == 1 && (d_out == nullptr || d_out == c->best_out)) return QOC_OK;
  // the segmented eval already reduced its J in its last workgroup (best_ready); otherwise k_argmin_seed
  if (!c->best_ready) {
    hipLaunchKernelGGL(k_argmin_seed, dim3(1), dim3(256), 0, c->stream, (const double*)c->d_J, c->B, c->seed_offset,
                       slot);
    HIPCHK(c, hipGetLastError());
  }
  if (c->comm && rccl().ok) {
    const ncclResult_t e = rccl().allGather(slot, c->d_best + 2, 2, ncclFloat64, c->comm, c->stream);
    if (e != ncclSuccess) return fail(c, QOC_ERR_HIP, "ncclAllGather: %s", rccl().getErrorString(e));
  }
  // the best over the gathered pairs, into the context's result and the caller's buffer
  hipLaunchKernelGGL(k_pick_best, dim3(1), dim3(64), 0, c->stream, (const double*)(c->d_best + 2),
                     c->comm && rccl().ok ? c->world : 1, res, d_out);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}

int qoc_set_best_output(qoc_ctx* c, double* d_out) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  c->best_out = d_out;
  c->best_direct = false;  // the next eval decides
  return QOC_OK;
}

int qoc_allgather_best(qoc_ctx* c, double* J_best, int* seed_best) {
  int r = qoc_allgather_best_dev(c, nullptr);
  if (r) return r;
  double h[2];
  HIPCHK(c, hipMemcpyAsync(h, c->d_best + 2 + 2 * c->world, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (J_best) *J_best = h[0];
  if (seed_best) *seed_best = (int)h[1];
  return QOC_OK;
}

int qoc_chain_terms(qoc_ctx* c, long long* terms, int reset) {
  if (!c || !terms) return fail(c, QOC_ERR_ARG, "null argument");
  *terms = 0;
  if (!c->d_terms) return QOC_OK;
  HIPCHK(c, hipSetDevice(c->dev));
  unsigned long long part[TERM_SLOTS];
  HIPCHK(c, hipMemcpyAsync(part, c->d_terms, sizeof(part), hipMemcpyDeviceToHost, c->stream));
  if (reset) HIPCHK(c, hipMemsetAsync(c->d_terms, 0, sizeof(part), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  unsigned long long t = 0;
  for (int i = 0; i < TERM_SLOTS; ++i) t += part[i];
  *terms = (long long)t;
  return QOC_OK;
}

int qoc_taylor_histogram_n(qoc_ctx* c, long long* hist, int n, int reset) {
  if (n < QOC_TAYLOR_HIST_ENTRIES)
    return fail(c, QOC_ERR_ARG, "histogram buffer holds %d entries, QOC_TAYLOR_HIST_ENTRIES = %d", n,
                QOC_TAYLOR_HIST_ENTRIES);
  return qoc_taylor_histogram(c, hist, reset);
}

int qoc_taylor_histogram(qoc_ctx* c, long long* hist, int reset) {
  if (!c || !hist) return fail(c, QOC_ERR_ARG, "null argument");
  HIPCHK(c, hipSetDevice(c->dev));
  HIPCHK(c, hipMemcpyAsync(hist, c->d_hist + 5 * 64, 8 * 64 * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
  if (reset) HIPCHK(c, hipMemsetAsync(c->d_hist + 5 * 64, 0, 8 * 64 * sizeof(long long), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int i = 8 * 64; i < 9 * 64; ++i) hist[i] = 0;
  for (int i = 0; i < 9 * 64; ++i) hist[i] += c->big_thist[i];
  if (reset) std::memset(c->big_thist, 0, sizeof(c->big_thist));
  return QOC_OK;
}

int qoc_pade_histogram(qoc_ctx* c, long long* hist, int reset) {
  if (!c || !hist) return fail(c, QOC_ERR_ARG, "null argument");
  HIPCHK(c, hipSetDevice(c->dev));
  if (c->chain_mode == 1 && c->prop_method == QOC_PROP_EXPM) {
    // no exponentials ran: the Padé choice for the last propagated u, once per forward pass since the last reset
    std::memset(hist, 0, 5 * 64 * sizeof(long long));
    if (c->props_since_reset > 0 && c->have_gen) {
      HIPCHK(c, hipMemsetAsync(c->d_hist, 0, 5 * 64 * sizeof(long long), c->stream));
      const long long units = (long long)c->B * c->Nt;
      HIPCHK(c, launch_pade_units(c, units));
      HIPCHK(c, hipMemcpyAsync(hist, c->d_hist, 5 * 64 * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipMemsetAsync(c->d_hist, 0, 5 * 64 * sizeof(long long), c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      for (int i = 0; i < 5 * 64; ++i) hist[i] *= c->props_since_reset;
    }
    if (reset) c->props_since_reset = 0;
    return QOC_OK;
  }
  HIPCHK(c, hipMemcpyAsync(hist, c->d_hist, 5 * 64 * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
  if (reset) HIPCHK(c, hipMemsetAsync(c->d_hist, 0, 5 * 64 * sizeof(long long), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int i = 0; i < 5 * 64; ++i) hist[i] += c->big_hist[i];
  if (reset) std::memset(c->big_hist, 0, sizeof(c->big_hist));
  return QOC_OK;
}

int qoc_expm_batched(int device, int N, int count, int precision, const double* A, double* X, int* degree_out,
                     int* squarings_out) {
  if (!A || !X || count < 1) return fail(nullptr, QOC_ERR_ARG, "bad argument");
  if (precision != QOC_FP64 && precision != QOC_FP32) return fail(nullptr, QOC_ERR_ARG, "bad precision");
  if (!expm_supported(N, precision)) return fail(nullptr, QOC_ERR_UNSUPPORTED, "N=%d unsupported", N);
  // Reuse the context machinery for staging/conversion.
  qoc_ctx tmp;
  tmp.dev = device;
  tmp.N = N;
  tmp.prec = precision;
  tmp.esz = precision == QOC_FP64 ? 16 : 8;
  qoc_ctx* c = &tmp;
  HIPCHK(c, hipSetDevice(device));
  HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  const size_t n = (size_t)count * N * N;
  void *dA = nullptr, *dX = nullptr;
  int *dd = nullptr, *ds = nullptr;
  int r = QOC_OK;
  hipError_t e = hipMalloc(&dA, n * c->esz);
  if (e == hipSuccess) e = hipMalloc(&dX, n * c->esz);
  if (e == hipSuccess) e = hipMalloc(&dd, count * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&ds, count * sizeof(int));
  if (e != hipSuccess) r = fail(nullptr, QOC_ERR_HIP, "hipMalloc: %s", hipGetErrorString(e));
  if (!r) r = upload(c, A, dA, n);
  if (!r) {
    e = launch_expm(precision, c->stream, N, 0, count, nullptr, nullptr, dA, dX, nullptr, dd, ds);
    if (e != hipSuccess) r = fail(nullptr, QOC_ERR_HIP, "k_expm: %s", hipGetErrorString(e));
  }
  if (!r) r = download(c, dX, X, n);
  if (!r && degree_out) hipMemcpy(degree_out, dd, count * sizeof(int), hipMemcpyDeviceToHost);
  if (!r && squarings_out) hipMemcpy(squarings_out, ds, count * sizeof(int), hipMemcpyDeviceToHost);
  hipFree(dA);
  hipFree(dX);
  hipFree(dd);
  hipFree(ds);
  if (c->d_stage) hipFree(c->d_stage);
  c->d_stage = nullptr;
  hipStreamDestroy(c->stream);
  c->stream = nullptr;
  if (r) g_err = tmp.err.empty() ? g_err : tmp.err;
  return r;
}

int qoc_expm_jacobian(int device, int N, int nu, const double* A0, const double* const* Aj, const double* p,
                      int order, double dt, double* dFdp_out) {
  if (!A0 || !Aj || !p || !dFdp_out || N < 1 || nu < 1) return fail(nullptr, QOC_ERR_ARG, "bad argument");
  if (order < 1 || order > 4) return fail(nullptr, QOC_ERR_ARG, "order must be 1..4");
  if (hipSetDevice(device) != hipSuccess) return fail(nullptr, QOC_ERR_HIP, "hipSetDevice");
  const size_t NN = (size_t)N * N, bytes = NN * 16;
  // buffers: A0, Aj[nu], X, AjX, XAj, X2, out[nu]
  std::vector<void*> bufs(2 * nu + 5, nullptr);
  for (auto& b : bufs)
    if (hipMalloc(&b, bytes) != hipSuccess) return fail(nullptr, QOC_ERR_HIP, "hipMalloc");
  auto A0d = (cx<double>*)bufs[0];
  auto Xd = (cx<double>*)bufs[nu + 1];
  auto AjXd = (cx<double>*)bufs[nu + 2];
  auto XAjd = (cx<double>*)bufs[nu + 3];
  auto X2d = (cx<double>*)bufs[nu + 4];
  hipMemcpy(A0d, A0, bytes, hipMemcpyHostToDevice);
  for (int j = 0; j < nu; ++j) hipMemcpy(bufs[1 + j], Aj[j], bytes, hipMemcpyHostToDevice);
  const dim3 g((unsigned)((NN + 255) / 256)), t(256);
  // X = A0 + sum p_j A_j   (src/gradient_computations.jl:188-191)
  hipLaunchKernelGGL(k_axpby, g, t, 0, 0, (int)NN, Xd, 1.0, A0d, 0.0, (const cx<double>*)nullptr);
  for (int j = 0; j < nu; ++j)
    hipLaunchKernelGGL(k_axpby, g, t, 0, 0, (int)NN, Xd, 1.0, Xd, p[j], (const cx<double>*)bufs[1 + j]);
  for (int j = 0; j < nu; ++j) {
    auto Aj_d = (const cx<double>*)bufs[1 + j];
    auto out = (cx<double>*)bufs[nu + 5 + j];
    hipLaunchKernelGGL(k_axpby, g, t, 0, 0, (int)NN, out, dt, Aj_d, 0.0, (const cx<double>*)nullptr);  // :179-181
    if (order >= 2) {  // :194-197
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, Aj_d, (const cx<double>*)Xd, AjXd, 1.0, 0.0);
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)Xd, Aj_d, XAjd, 1.0, 0.0);
      hipLaunchKernelGGL(k_axpby, g, t, 0, 0, (int)NN, out, 1.0, out, dt * dt / 2, (const cx<double>*)AjXd);
      hipLaunchKernelGGL(k_axpby, g, t, 0, 0, (int)NN, out, 1.0, out, dt * dt / 2, (const cx<double>*)XAjd);
    }
    if (order >= 3) {  // :199-202
      const double c3 = dt * dt * dt / 6;
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)AjXd, (const cx<double>*)Xd, out, c3, 1.0);
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)XAjd, (const cx<double>*)Xd, out, c3, 1.0);
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)Xd, (const cx<double>*)XAjd, out, c3, 1.0);
    }
    if (order >= 4) {  // :204-210
      const double c4 = dt * dt * dt * dt / 24;
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)Xd, (const cx<double>*)Xd, X2d, 1.0, 0.0);
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)AjXd, (const cx<double>*)X2d, out, c4, 1.0);
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)XAjd, (const cx<double>*)X2d, out, c4, 1.0);
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)X2d, (const cx<double>*)AjXd, out, c4, 1.0);
      hipLaunchKernelGGL(k_cgemm_naive, g, t, 0, 0, N, (const cx<double>*)X2d, (const cx<double>*)XAjd, out, c4, 1.0);
    }
  }
  int r = QOC_OK;
  if (hipDeviceSynchronize() != hipSuccess) r = fail(nullptr, QOC_ERR_HIP, "expm_jacobian kernels failed");
  for (int j = 0; j < nu && !r; ++j) hipMemcpy(dFdp_out + 2 * NN * j, bufs[nu + 5 + j], bytes, hipMemcpyDeviceToHost);
  for (auto b : bufs) hipFree(b);
  return r;
}

}  // extern "C"
