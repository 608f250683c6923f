// qoc_engine.hip — host side of libqoc_mi355x.so: the C ABI declared in include/qoc.h.
//
// The context replaces the reference's GRAPE cache (src/gradient_computations.jl:79-96):
// all per-slice propagators, states and co-states live in HBM for the whole batch of
// seeds, and the hot path (propagate + grape_sensitivity) is four kernel launches on
// one HIP stream:  k_expm -> k_chain_fwd  |  k_chain_bwd -> k_grad.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/qoc.h"
#include "qoc_chain.hpp"
#include "qoc_expm.hpp"

using namespace qoc;

namespace {

thread_local std::string g_err;

int fail(qoc_ctx* ctx, int code, const char* fmt, ...);

}  // namespace

struct qoc_ctx {
  int dev = 0, N = 0, m = 0, nu = 0, Nt = 0, B = 0, prec = QOC_FP64;
  size_t esz = 16;  // bytes per complex element on device
  hipStream_t stream = nullptr;
  void* d_A = nullptr;    // (nu+1) x N*N
  void* d_x0 = nullptr;   // N*m or B*N*m
  int x0_per_seed = 0;
  void* d_Xt = nullptr;   // N*m target
  int cost_kind = QOC_COST_TRACE;
  double cost_n = 1.0;
  unsigned char* d_pmask = nullptr;
  double mu = 0.0;
  double* d_u = nullptr;     // B*nu*Nt, u of the last propagate
  void* d_U = nullptr;       // B*Nt*N*N
  void* d_X = nullptr;       // B*(Nt+1)*N*m
  void* d_L = nullptr;       // B*(Nt+1)*N*m
  double* d_J = nullptr;     // B
  cx<double>* d_coef = nullptr;  // B*m
  double* d_dJdu = nullptr;  // B*nu*Nt
  int* d_flag = nullptr;
  unsigned long long* d_hist = nullptr;  // 5*64
  double* d_stage = nullptr;             // host->device staging (fp64 complex), max(B*N*m, (nu+1)*N*N)*2
  size_t stage_elems = 0;
  std::vector<double> h_u;
  // live per-kernel timing (hipEvents recorded on `stream` around each hot-path launch)
  bool profiling = false;
  struct Mark {
    int phase;
    hipEvent_t a, b;
  };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> event_pool;
  double phase_ms[4] = {0, 0, 0, 0};
  long long phase_n[4] = {0, 0, 0, 0};
  bool have_gen = false, have_x0 = false, have_cost = false, have_prop = false;
  std::string err;
};

namespace {

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

#define HIPCHK(ctx, expr)                                                                     \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail(ctx, QOC_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

constexpr int kChainMaxN = 64;

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

template <typename T, int NT>
hipError_t launch_expm_t(hipStream_t s, int N, int nu, int nunits, const void* Agen, const double* u,
                         const void* Ain, void* Uout, unsigned long long* hist, int* deg, int* sq) {
  const size_t lds = Expm<T, NT>::lds_bytes(N);
  hipError_t e = hipFuncSetAttribute((const void*)k_expm<T, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_expm<T, NT>), dim3(nunits), dim3(256), lds, s, N, nu, nunits, (const cx<T>*)Agen, u,
                     (const cx<T>*)Ain, (cx<T>*)Uout, hist, deg, sq);
  return hipGetLastError();
}

hipError_t launch_expm(int prec, hipStream_t s, int N, int nu, int nunits, const void* Agen, const double* u,
                       const void* Ain, void* Uout, unsigned long long* hist, int* deg, int* sq) {
  const int NT = (N + 15) / 16;
  if (prec == QOC_FP64) {
    if (NT == 1) return launch_expm_t<double, 1>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, deg, sq);
    if (NT == 2) return launch_expm_t<double, 2>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, deg, sq);
    return launch_expm_t<double, 3>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, deg, sq);
  }
  if (NT == 1) return launch_expm_t<float, 1>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, deg, sq);
  if (NT == 2) return launch_expm_t<float, 2>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, deg, sq);
  return launch_expm_t<float, 3>(s, N, nu, nunits, Agen, u, Ain, Uout, hist, deg, sq);
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

size_t chain_lds(const qoc_ctx* c) {
  return (size_t)(2 * c->N * (c->N + 1) + 2 * c->N * c->m) * c->esz + 64 * sizeof(double);
}
size_t grad_lds(const qoc_ctx* c, int order) {
  return (size_t)(c->N * (c->N + 1) + 2 * order * c->N * c->m) * c->esz + 64 * sizeof(double);
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
int mark_begin(qoc_ctx* c, int phase) {
  if (!c->profiling) return -1;
  qoc_ctx::Mark m{phase, take_event(c), take_event(c)};
  (void)hipEventRecord(m.a, c->stream);
  c->marks.push_back(m);
  return (int)c->marks.size() - 1;
}
void mark_end(qoc_ctx* c, int idx) {
  if (idx >= 0) (void)hipEventRecord(c->marks[idx].b, c->stream);
}

template <typename T>
int run_forward(qoc_ctx* c) {
  int mk = mark_begin(c, 0);
  hipError_t e = launch_expm(c->prec, c->stream, c->N, c->nu, c->B * c->Nt, c->d_A, c->d_u, nullptr, c->d_U,
                             c->d_hist, nullptr, nullptr);
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_expm launch: %s", hipGetErrorString(e));
  const size_t lds = chain_lds(c);
  HIPCHK(c, hipFuncSetAttribute((const void*)k_chain_fwd<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  mk = mark_begin(c, 1);
  hipLaunchKernelGGL((k_chain_fwd<T>), dim3(c->B), dim3(CHAIN_THREADS), lds, c->stream, c->N, c->m, c->Nt,
                     (const cx<T>*)c->d_U, (const cx<T>*)c->d_x0, c->x0_per_seed, (cx<T>*)c->d_X,
                     (const cx<T>*)c->d_Xt, c->cost_kind, c->cost_n, c->mu != 0.0 ? c->d_pmask : nullptr, c->mu,
                     c->d_J, c->d_coef);
  mark_end(c, mk);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}

template <typename T>
int run_backward(qoc_ctx* c, int order, double* d_dJdu) {
  size_t lds = chain_lds(c);
  HIPCHK(c, hipFuncSetAttribute((const void*)k_chain_bwd<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int mk = mark_begin(c, 2);
  hipLaunchKernelGGL((k_chain_bwd<T>), dim3(c->B), dim3(CHAIN_THREADS), lds, c->stream, c->N, c->m, c->Nt,
                     (const cx<T>*)c->d_U, (const cx<T>*)c->d_X, (cx<T>*)c->d_L, (const cx<T>*)c->d_Xt, c->cost_kind,
                     (const cx<double>*)c->d_coef, c->mu != 0.0 ? c->d_pmask : nullptr, c->mu);
  mark_end(c, mk);
  HIPCHK(c, hipGetLastError());
  lds = grad_lds(c, order);
  HIPCHK(c, hipFuncSetAttribute((const void*)k_grad<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  mk = mark_begin(c, 3);
  hipLaunchKernelGGL((k_grad<T>), dim3(c->B * c->Nt), dim3(GRAD_THREADS), lds, c->stream, c->N, c->m, c->nu, c->Nt,
                     order, (const cx<T>*)c->d_A, c->d_u, (const cx<T>*)c->d_X, (const cx<T>*)c->d_L, d_dJdu);
  mark_end(c, mk);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}

int forward(qoc_ctx* c) { return c->prec == QOC_FP64 ? run_forward<double>(c) : run_forward<float>(c); }
int backward(qoc_ctx* c, int order, double* d_dJdu) {
  return c->prec == QOC_FP64 ? run_backward<double>(c, order, d_dJdu) : run_backward<float>(c, order, d_dJdu);
}

int check_ready(qoc_ctx* c) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (!c->have_gen) return fail(c, QOC_ERR_STATE, "generators not set (qoc_set_generators)");
  if (!c->have_x0) return fail(c, QOC_ERR_STATE, "x0 not set (qoc_set_x0)");
  if (!c->have_cost) return fail(c, QOC_ERR_STATE, "cost not set (qoc_set_cost)");
  HIPCHK(c, hipSetDevice(c->dev));
  return QOC_OK;
}

}  // namespace

extern "C" {

const char* qoc_last_error(const qoc_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int qoc_create(qoc_ctx** out, int device, int N, int m, int nu, int Nt, int B, int precision) {
  if (!out) return fail(nullptr, QOC_ERR_ARG, "out is null");
  *out = nullptr;
  if (N < 1 || m < 1 || nu < 1 || Nt < 1 || B < 1)
    return fail(nullptr, QOC_ERR_ARG, "invalid dimensions N=%d m=%d nu=%d Nt=%d B=%d", N, m, nu, Nt, B);
  if (precision != QOC_FP64 && precision != QOC_FP32) return fail(nullptr, QOC_ERR_ARG, "invalid precision");
  if (!expm_supported(N, precision) || N > kChainMaxN || N * N > CHAIN_THREADS * (precision == QOC_FP64 ? 8 : 16) ||
      N * m > 4 * CHAIN_THREADS)
    return fail(nullptr, QOC_ERR_UNSUPPORTED, "N=%d m=%d outside the LDS-resident kernel envelope", N, m);
  qoc_ctx* c = new qoc_ctx();
  c->dev = device;
  c->N = N;
  c->m = m;
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
      {(void**)&c->d_u, (size_t)B * nu * Nt * sizeof(double)},
      {&c->d_U, (size_t)B * Nt * NN * c->esz},
      {&c->d_X, (size_t)B * (Nt + 1) * Nm * c->esz},
      {&c->d_L, (size_t)B * (Nt + 1) * Nm * c->esz},
      {(void**)&c->d_J, (size_t)B * sizeof(double)},
      {(void**)&c->d_coef, (size_t)B * m * sizeof(cx<double>)},
      {(void**)&c->d_dJdu, (size_t)B * nu * Nt * sizeof(double)},
      {(void**)&c->d_flag, sizeof(int)},
      {(void**)&c->d_hist, 5 * 64 * sizeof(unsigned long long)},
  };
  for (auto& a : allocs) {
    if ((e = hipMalloc(a.p, a.bytes)) != hipSuccess) return bail(e, "hipMalloc");
  }
  hipMemset(c->d_pmask, 0, Nm);
  hipMemset(c->d_hist, 0, 5 * 64 * sizeof(unsigned long long));
  hipMemset(c->d_L, 0, (size_t)B * (Nt + 1) * Nm * c->esz);
  *out = c;
  return QOC_OK;
}

void qoc_destroy(qoc_ctx* c) {
  if (!c) return;
  hipSetDevice(c->dev);
  if (c->stream) hipStreamSynchronize(c->stream);
  void* ptrs[] = {c->d_A, c->d_x0, c->d_Xt, c->d_pmask, c->d_u,    c->d_U,    c->d_X, c->d_L,
                  c->d_J, c->d_coef, c->d_dJdu, c->d_flag, c->d_hist, c->d_stage};
  for (void* p : ptrs)
    if (p) hipFree(p);
  for (auto& m : c->marks) {
    hipEventDestroy(m.a);
    hipEventDestroy(m.b);
  }
  for (auto e : c->event_pool) hipEventDestroy(e);
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
  const size_t NN = (size_t)c->N * c->N;
  int r = upload(c, A0, c->d_A, NN);
  for (int j = 0; j < c->nu && r == QOC_OK; ++j) {
    if (!Aj[j]) return fail(c, QOC_ERR_ARG, "A[%d] is null", j);
    r = upload(c, Aj[j], (char*)c->d_A + (j + 1) * NN * c->esz, NN);
  }
  if (r != QOC_OK) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->have_gen = true;
  c->have_prop = false;
  return QOC_OK;
}

int qoc_set_x0(qoc_ctx* c, const double* x0, int per_seed) {
  if (!c || !x0) return fail(c, QOC_ERR_ARG, "null argument");
  HIPCHK(c, hipSetDevice(c->dev));
  const size_t Nm = (size_t)c->N * c->m;
  int r = upload(c, x0, c->d_x0, per_seed ? (size_t)c->B * Nm : Nm);
  if (r != QOC_OK) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->x0_per_seed = per_seed ? 1 : 0;
  c->have_x0 = true;
  c->have_prop = false;
  return QOC_OK;
}

int qoc_set_cost(qoc_ctx* c, int kind, const double* X_target, double n) {
  if (!c) return fail(nullptr, QOC_ERR_ARG, "null context");
  if (kind != QOC_COST_TRACE && kind != QOC_COST_ZCAL && kind != QOC_COST_EXTERNAL)
    return fail(c, QOC_ERR_ARG, "unknown cost kind %d", kind);
  if (kind == QOC_COST_ZCAL && c->m != 4)
    return fail(c, QOC_ERR_ARG, "Only works for two-qubit gates, x_target must have four columns");
  if (kind != QOC_COST_EXTERNAL && !X_target) return fail(c, QOC_ERR_ARG, "X_target is null");
  if (kind == QOC_COST_TRACE && !(n != 0.0)) return fail(c, QOC_ERR_ARG, "normalisation n must be nonzero");
  HIPCHK(c, hipSetDevice(c->dev));
  if (X_target) {
    int r = upload(c, X_target, c->d_Xt, (size_t)c->N * c->m);
    if (r != QOC_OK) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  c->cost_kind = kind;
  c->cost_n = n;
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
      if (C[bb] < 0 || C[bb] >= c->m) return fail(c, QOC_ERR_ARG, "penalty column %d out of range", C[bb]);
      mask[P[a] + (size_t)c->N * C[bb]] = 1;
    }
  }
  HIPCHK(c, hipSetDevice(c->dev));
  HIPCHK(c, hipMemcpy(c->d_pmask, mask.data(), mask.size(), hipMemcpyHostToDevice));
  c->mu = mu;  // affects J of the next propagate and dL/dx of the next sensitivity
  return QOC_OK;
}

int qoc_propagate_dev(qoc_ctx* c, const double* d_u, double* d_J) {
  int r = check_ready(c);
  if (r) return r;
  if (!d_u) return fail(c, QOC_ERR_ARG, "d_u is null");
  const size_t nu_t = (size_t)c->B * c->nu * c->Nt;
  if (d_u != c->d_u) HIPCHK(c, hipMemcpyAsync(c->d_u, d_u, nu_t * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  r = forward(c);
  if (r) return r;
  if (d_J && d_J != c->d_J)
    HIPCHK(c, hipMemcpyAsync(d_J, c->d_J, c->B * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  c->have_prop = true;
  c->h_u.clear();  // host copy unknown for device-side u
  return QOC_OK;
}

int qoc_grape_sensitivity_dev(qoc_ctx* c, const double* d_u, int order, double* d_dJdu) {
  int r = check_ready(c);
  if (r) return r;
  if (!c->have_prop) return fail(c, QOC_ERR_STATE, "grape_sensitivity called before propagate");
  if (order < 1 || order > 4) return fail(c, QOC_ERR_ARG, "dUkdp_order must be 1..4 (got %d)", order);
  if (c->cost_kind == QOC_COST_EXTERNAL)
    return fail(c, QOC_ERR_STATE, "QOC_COST_EXTERNAL needs qoc_grape_sensitivity (host lambda_final)");
  const size_t nu_t = (size_t)c->B * c->nu * c->Nt;
  if (d_u && d_u != c->d_u) {
    HIPCHK(c, hipMemsetAsync(c->d_flag, 0, sizeof(int), c->stream));
    hipLaunchKernelGGL(k_compare_u, dim3(256), dim3(256), 0, c->stream, d_u, c->d_u, nu_t, c->d_flag);
    HIPCHK(c, hipGetLastError());
    int flag = 0;
    HIPCHK(c, hipMemcpyAsync(&flag, c->d_flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (flag) return fail(c, QOC_ERR_STALE, "Cache data from other control signal u");
  }
  return backward(c, order, d_dJdu ? d_dJdu : c->d_dJdu);
}

int qoc_eval_dev(qoc_ctx* c, const double* d_u, int order, double* d_J, double* d_dJdu) {
  if (c && c->cost_kind == QOC_COST_EXTERNAL)
    return fail(c, QOC_ERR_STATE, "qoc_eval_dev needs a device-side cost (TRACE or ZCAL)");
  int r = qoc_propagate_dev(c, d_u, d_J);
  if (r) return r;
  if (order < 1 || order > 4) return fail(c, QOC_ERR_ARG, "dUkdp_order must be 1..4 (got %d)", order);
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
  c->have_prop = true;
  return QOC_OK;
}

int qoc_grape_sensitivity(qoc_ctx* c, const double* u, int order, const double* lambda_final, double* dJdu_out) {
  int r = check_ready(c);
  if (r) return r;
  if (!c->have_prop) return fail(c, QOC_ERR_STATE, "grape_sensitivity called before propagate");
  if (order < 1 || order > 4) return fail(c, QOC_ERR_ARG, "dUkdp_order must be 1..4 (got %d)", order);
  const size_t nu_t = (size_t)c->B * c->nu * c->Nt;
  if (!u) return fail(c, QOC_ERR_ARG, "u is null");
  if (c->h_u.size() == nu_t) {
    if (std::memcmp(u, c->h_u.data(), nu_t * sizeof(double)) != 0)
      return fail(c, QOC_ERR_STALE, "Cache data from other control signal u");
  } else {
    // last propagate came from device memory: compare on the device
    HIPCHK(c, hipMemcpyAsync(c->d_dJdu, u, nu_t * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_flag, 0, sizeof(int), c->stream));
    hipLaunchKernelGGL(k_compare_u, dim3(256), dim3(256), 0, c->stream, c->d_dJdu, c->d_u, nu_t, c->d_flag);
    int flag = 0;
    HIPCHK(c, hipMemcpyAsync(&flag, c->d_flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (flag) return fail(c, QOC_ERR_STALE, "Cache data from other control signal u");
  }
  if (c->cost_kind == QOC_COST_EXTERNAL) {
    if (!lambda_final) return fail(c, QOC_ERR_ARG, "lambda_final is required for QOC_COST_EXTERNAL");
    // λ_{Nt+1} for every seed lives at Lam[b][Nt]
    const size_t Nm = (size_t)c->N * c->m;
    for (int b = 0; b < c->B; ++b) {
      r = upload(c, lambda_final + 2 * Nm * b, (char*)c->d_L + ((size_t)b * (c->Nt + 1) + c->Nt) * Nm * c->esz, Nm);
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
  const size_t Nm = (size_t)c->N * c->m;
  return download(c, (char*)c->d_X + ((size_t)seed * (c->Nt + 1) + k) * Nm * c->esz, x_out, Nm);
}

int qoc_get_costates(qoc_ctx* c, int seed, int k, double* lam_out) {
  if (!c || !lam_out) return fail(c, QOC_ERR_ARG, "null argument");
  if (k == -1) k = c->Nt;
  if (seed < 0 || seed >= c->B || k < 0 || k > c->Nt) return fail(c, QOC_ERR_ARG, "index out of range");
  HIPCHK(c, hipSetDevice(c->dev));
  const size_t Nm = (size_t)c->N * c->m;
  return download(c, (char*)c->d_L + ((size_t)seed * (c->Nt + 1) + k) * Nm * c->esz, lam_out, Nm);
}

int qoc_get_propagator(qoc_ctx* c, int seed, int k, double* U_out) {
  if (!c || !U_out) return fail(c, QOC_ERR_ARG, "null argument");
  if (!c->have_prop) return fail(c, QOC_ERR_STATE, "no propagators");
  if (seed < 0 || seed >= c->B || k < 0 || k >= c->Nt) return fail(c, QOC_ERR_ARG, "index out of range");
  HIPCHK(c, hipSetDevice(c->dev));
  const size_t NN = (size_t)c->N * c->N;
  return download(c, (char*)c->d_U + ((size_t)seed * c->Nt + k) * NN * c->esz, U_out, NN);
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

int qoc_pade_histogram(qoc_ctx* c, long long* hist, int reset) {
  if (!c || !hist) return fail(c, QOC_ERR_ARG, "null argument");
  HIPCHK(c, hipSetDevice(c->dev));
  HIPCHK(c, hipMemcpyAsync(hist, c->d_hist, 5 * 64 * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
  if (reset) HIPCHK(c, hipMemsetAsync(c->d_hist, 0, 5 * 64 * sizeof(long long), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
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
