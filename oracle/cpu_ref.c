/*
 * cpu_ref.c — C restatement of the reference GRAPE hot path, used as the CPU baseline.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/qoc_oracle.py header): called by tests/ and by
 * bench.py's cpu_baseline leg, never by the product path.
 *
 * Follows olof3/QuantumOptimalControl.jl line by line in algorithm (not in language):
 *   propagate            src/gradient_computations.jl:2-32   (A_k formation :18-22, chain :27-29)
 *   exponential!         ExponentialUtilities ExpMethodHigham2005 (called at :24): Padé 3/5/7/9/13,
 *                        scaling & squaring, LU with partial pivoting (LAPACK gesv)
 *   grape_sensitivity    src/gradient_computations.jl:35-77  (λ sweep :52-58, gradient loop :65-74)
 *   expm_jacobian!       src/gradient_computations.jl:177-213 (dense Taylor terms, 5 nu GEMMs at order 3)
 *   _compute_u_sensitivity src/gradient_computations.jl:217-223
 *   setup_infidelity     src/penalty_fcns.jl:15-24
 * Complex matrices: column-major, interleaved (Julia ComplexF64 layout).
 *
 * Two timing modes: mode 0 = seed-parallel (one seed per thread),
 * mode 1 = reference-faithful (exponentials OpenMP-parallel over k, like Threads.@threads at :17).
 *
 * BLAS/LAPACK: the reference calls zgemm (mul!) and zgesv (exponential!'s solve) of MKL
 * (examples/zz_coupling_ipopt_exp.jl:2).  qocref_set_blas(path) dlopens an OpenBLAS (the one scipy ships in
 * this image) and routes every N x N product and the Padé solve through its zgemm_ / zgesv_ (one BLAS thread
 * per call, the parallelism is OpenMP over seeds or slices); without it the loops below are used.
 */
#include <complex.h>
#include <dlfcn.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef double complex cd;

typedef void (*zgemm_fn)(const char*, const char*, const int*, const int*, const int*, const cd*, const cd*,
                         const int*, const cd*, const int*, const cd*, cd*, const int*);
typedef void (*zgesv_fn)(const int*, const int*, cd*, const int*, int*, cd*, const int*, int*);
static zgemm_fn blas_zgemm = NULL;
static zgesv_fn blas_zgesv = NULL;

/* Returns 0 when zgemm and zgesv were found (symbol prefix: "" or "scipy_"). */
int qocref_set_blas(const char* path) {
  blas_zgemm = NULL;
  blas_zgesv = NULL;
  if (!path || !*path) return 0;
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return -1;
  const char* pre[2] = {"scipy_", ""};
  for (int i = 0; i < 2 && !blas_zgemm; ++i) {
    char nm[64];
    strcpy(nm, pre[i]);
    strcat(nm, "zgemm_");
    blas_zgemm = (zgemm_fn)dlsym(h, nm);
    strcpy(nm, pre[i]);
    strcat(nm, "zgesv_");
    blas_zgesv = (zgesv_fn)dlsym(h, nm);
    void (*nt)(int) = NULL;
    strcpy(nm, pre[i]);
    strcat(nm, "openblas_set_num_threads");
    nt = (void (*)(int))dlsym(h, nm);
    if (nt) nt(1);
  }
  if (!blas_zgemm || !blas_zgesv) {
    blas_zgemm = NULL;
    blas_zgesv = NULL;
    return -2;
  }
  return 0;
}
int qocref_have_blas(void) { return blas_zgemm != NULL; }

static const double P3[4] = {120.0, 60.0, 12.0, 1.0};
static const double P5[6] = {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0};
static const double P7[8] = {17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0};
static const double P9[10] = {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
                              2162160.0, 110880.0, 3960.0, 90.0, 1.0};
static const double P13[14] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                               1187353796428800.0, 129060195264000.0, 10559470521600.0, 670442572800.0,
                               33522128640.0, 1323241920.0, 40840800.0, 960960.0, 16380.0, 182.0, 1.0};

/* C = alpha*A*B + beta*C, column-major N x N (zgemm-shaped loop order j,l,i). */
static void gemm(int N, const cd* A, const cd* B, cd* C, cd alpha, cd beta) {
  if (blas_zgemm) {
    blas_zgemm("N", "N", &N, &N, &N, &alpha, A, &N, B, &N, &beta, C, &N);
    return;
  }
  for (int j = 0; j < N; ++j) {
    cd* c = C + (size_t)N * j;
    if (beta == 0.0)
      memset(c, 0, sizeof(cd) * N);
    else if (beta != 1.0)
      for (int i = 0; i < N; ++i) c[i] *= beta;
    for (int l = 0; l < N; ++l) {
      const cd b = alpha * B[l + (size_t)N * j];
      const cd* a = A + (size_t)N * l;
      for (int i = 0; i < N; ++i) c[i] += a[i] * b;
    }
  }
}

/* y = A x  (N x N times N x m) */
static void gemm_nm(int N, int m, const cd* A, const cd* X, cd* Y) {
  if (blas_zgemm) {
    const cd one = 1.0, zero = 0.0;
    blas_zgemm("N", "N", &N, &m, &N, &one, A, &N, X, &N, &zero, Y, &N);
    return;
  }
  for (int c = 0; c < m; ++c) {
    cd* y = Y + (size_t)N * c;
    memset(y, 0, sizeof(cd) * N);
    for (int l = 0; l < N; ++l) {
      const cd b = X[l + (size_t)N * c];
      const cd* a = A + (size_t)N * l;
      for (int i = 0; i < N; ++i) y[i] += a[i] * b;
    }
  }
}

/* y = A^H x */
static void gemm_h_nm(int N, int m, const cd* A, const cd* X, cd* Y) {
  if (blas_zgemm) {
    const cd one = 1.0, zero = 0.0;
    blas_zgemm("C", "N", &N, &m, &N, &one, A, &N, X, &N, &zero, Y, &N);
    return;
  }
  for (int c = 0; c < m; ++c)
    for (int i = 0; i < N; ++i) {
      cd s = 0;
      const cd* a = A + (size_t)N * i;
      const cd* x = X + (size_t)N * c;
      for (int l = 0; l < N; ++l) s += conj(a[l]) * x[l];
      Y[i + (size_t)N * c] = s;
    }
}

/* Solve Q X = P in place (X overwrites P); LU with partial pivoting, izamax rule (|re|+|im|). */
static void gesv(int N, cd* Q, cd* P) {
  int* piv = (int*)malloc(sizeof(int) * N);
  if (blas_zgesv) {
    int info = 0;
    blas_zgesv(&N, &N, Q, &N, piv, P, &N, &info);
    free(piv);
    return;
  }
  for (int p = 0; p < N; ++p) {
    int r = p;
    double best = -1.0;
    for (int i = p; i < N; ++i) {
      const double a = fabs(creal(Q[i + (size_t)N * p])) + fabs(cimag(Q[i + (size_t)N * p]));
      if (a > best) {
        best = a;
        r = i;
      }
    }
    piv[p] = r;
    if (r != p) {
      for (int j = 0; j < N; ++j) {
        cd t = Q[p + (size_t)N * j];
        Q[p + (size_t)N * j] = Q[r + (size_t)N * j];
        Q[r + (size_t)N * j] = t;
        t = P[p + (size_t)N * j];
        P[p + (size_t)N * j] = P[r + (size_t)N * j];
        P[r + (size_t)N * j] = t;
      }
    }
    const cd inv = 1.0 / Q[p + (size_t)N * p];
    for (int i = p + 1; i < N; ++i) Q[i + (size_t)N * p] *= inv;
    for (int j = p + 1; j < N; ++j) {
      const cd b = Q[p + (size_t)N * j];
      for (int i = p + 1; i < N; ++i) Q[i + (size_t)N * j] -= Q[i + (size_t)N * p] * b;
    }
    for (int j = 0; j < N; ++j) {
      const cd b = P[p + (size_t)N * j];
      for (int i = p + 1; i < N; ++i) P[i + (size_t)N * j] -= Q[i + (size_t)N * p] * b;
    }
  }
  for (int j = 0; j < N; ++j)
    for (int p = N - 1; p >= 0; --p) {
      cd s = P[p + (size_t)N * j];
      for (int l = p + 1; l < N; ++l) s -= Q[p + (size_t)N * l] * P[l + (size_t)N * j];
      P[p + (size_t)N * j] = s / Q[p + (size_t)N * p];
    }
  free(piv);
}

/* exp(A) in place of X; ws = 6 N x N scratch.  Returns degree*64 + squarings. */
static int expm(int N, const cd* Ain, cd* X, cd* ws) {
  const size_t NN = (size_t)N * N;
  cd *A = ws, *A2 = ws + NN, *A4 = ws + 2 * NN, *A6 = ws + 3 * NN, *U = ws + 4 * NN, *V = ws + 5 * NN;
  memcpy(A, Ain, sizeof(cd) * NN);
  double nA = 0;
  for (int j = 0; j < N; ++j) {
    double s = 0;
    for (int i = 0; i < N; ++i) s += cabs(A[i + (size_t)N * j]);
    if (s > nA) nA = s;
  }
  int d, sq = 0;
  if (nA <= 2.1) {
    const double* C = nA > 0.95 ? P9 : nA > 0.25 ? P7 : nA > 0.015 ? P5 : P3;
    d = nA > 0.95 ? 9 : nA > 0.25 ? 7 : nA > 0.015 ? 5 : 3;
    gemm(N, A, A, A2, 1.0, 0.0);
    /* U' = b1 I + b3 A2 + ..., V = b0 I + b2 A2 + ...; P = current power (A4 buffer) */
    for (size_t e = 0; e < NN; ++e) {
      U[e] = C[3] * A2[e];
      V[e] = C[2] * A2[e];
    }
    for (int i = 0; i < N; ++i) {
      U[i + (size_t)N * i] += C[1];
      V[i + (size_t)N * i] += C[0];
    }
    cd* P = A2;
    for (int k = 2; 2 * k < d + 1; ++k) {
      cd* Pn = (P == A4) ? A6 : A4;
      gemm(N, P, A2, Pn, 1.0, 0.0);
      for (size_t e = 0; e < NN; ++e) {
        U[e] += C[2 * k + 1] * Pn[e];
        V[e] += C[2 * k] * Pn[e];
      }
      P = Pn;
    }
    gemm(N, A, U, A4, 1.0, 0.0); /* A4 <- A U' */
    memcpy(U, A4, sizeof(cd) * NN);
  } else {
    const double* C = P13;
    d = 13;
    const double s = log2(nA / 5.4);
    sq = s > 0 ? (int)ceil(s) : 0;
    if (sq > 0) {
      const double sc = ldexp(1.0, -sq);
      for (size_t e = 0; e < NN; ++e) A[e] *= sc;
    }
    gemm(N, A, A, A2, 1.0, 0.0);
    gemm(N, A2, A2, A4, 1.0, 0.0);
    gemm(N, A2, A4, A6, 1.0, 0.0);
    for (size_t e = 0; e < NN; ++e) {
      U[e] = C[13] * A6[e] + C[11] * A4[e] + C[9] * A2[e];
      V[e] = C[12] * A6[e] + C[10] * A4[e] + C[8] * A2[e];
    }
    gemm(N, A6, U, X, 1.0, 0.0); /* X used as scratch */
    for (size_t e = 0; e < NN; ++e) U[e] = X[e] + C[7] * A6[e] + C[5] * A4[e] + C[3] * A2[e];
    gemm(N, A6, V, X, 1.0, 0.0);
    for (size_t e = 0; e < NN; ++e) V[e] = X[e] + C[6] * A6[e] + C[4] * A4[e] + C[2] * A2[e];
    for (int i = 0; i < N; ++i) {
      U[i + (size_t)N * i] += C[1];
      V[i + (size_t)N * i] += C[0];
    }
    gemm(N, A, U, A2, 1.0, 0.0);
    memcpy(U, A2, sizeof(cd) * NN);
  }
  for (size_t e = 0; e < NN; ++e) {
    X[e] = V[e] + U[e];
    V[e] = V[e] - U[e];
  }
  gesv(N, V, X);
  for (int t = 0; t < sq; ++t) {
    gemm(N, X, X, A, 1.0, 0.0);
    memcpy(X, A, sizeof(cd) * NN);
  }
  return d * 64 + sq;
}

/* expm_jacobian! (src/gradient_computations.jl:177-213); ws = 4 N x N, out = nu N x N. */
static void expm_jacobian(int N, int nu, const cd* A0, const cd* Aj, const double* p, int order, double dt,
                          cd* out, cd* ws) {
  const size_t NN = (size_t)N * N;
  cd *X = ws, *AjX = ws + NN, *XAj = ws + 2 * NN, *X2 = ws + 3 * NN;
  for (int j = 0; j < nu; ++j)
    for (size_t e = 0; e < NN; ++e) out[j * NN + e] = dt * Aj[j * NN + e];
  if (order <= 1) return;
  memcpy(X, A0, sizeof(cd) * NN);
  for (int j = 0; j < nu; ++j)
    for (size_t e = 0; e < NN; ++e) X[e] += p[j] * Aj[j * NN + e];
  for (int j = 0; j < nu; ++j) {
    const cd* A = Aj + j * NN;
    cd* o = out + j * NN;
    gemm(N, A, X, AjX, 1.0, 0.0);
    gemm(N, X, A, XAj, 1.0, 0.0);
    const double c2 = dt * dt / 2;
    for (size_t e = 0; e < NN; ++e) o[e] += c2 * (AjX[e] + XAj[e]);
    if (order >= 3) {
      const double c3 = dt * dt * dt / 6;
      gemm(N, AjX, X, o, c3, 1.0);
      gemm(N, XAj, X, o, c3, 1.0);
      gemm(N, X, XAj, o, c3, 1.0);
    }
    if (order >= 4) {
      const double c4 = dt * dt * dt * dt / 24;
      gemm(N, X, X, X2, 1.0, 0.0);
      gemm(N, AjX, X2, o, c4, 1.0);
      gemm(N, XAj, X2, o, c4, 1.0);
      gemm(N, X2, AjX, o, c4, 1.0);
      gemm(N, X2, XAj, o, c4, 1.0);
    }
  }
}

int qocref_expm(int N, const double* A, double* X, int* deg, int* sq) {
  cd* ws = (cd*)malloc(sizeof(cd) * 6 * (size_t)N * N);
  const int r = expm(N, (const cd*)A, (cd*)X, ws);
  free(ws);
  if (deg) *deg = r / 64;
  if (sq) *sq = r % 64;
  return 0;
}

int qocref_expm_jacobian(int N, int nu, const double* A0, const double* Aj, const double* p, int order, double dt,
                         double* out) {
  cd* ws = (cd*)malloc(sizeof(cd) * 4 * (size_t)N * N);
  expm_jacobian(N, nu, (const cd*)A0, (const cd*)Aj, p, order, dt, (cd*)out, ws);
  free(ws);
  return 0;
}

/* One GRAPE eval (propagate + J + grape_sensitivity) for one seed.
 * par_k: parallelise the exponentials over k (reference-faithful mode). */
static int grape_eval1(int N, int m, int nu, int Nt, const cd* A0, const cd* Aj, const double* u, const cd* x0,
                       const cd* Xt, double n, int order, double* J, double* dJdu, int* degs, int par_k) {
  const size_t NN = (size_t)N * N, Nm = (size_t)N * m;
  cd* Uk = (cd*)malloc(sizeof(cd) * NN * Nt);
  cd* x = (cd*)malloc(sizeof(cd) * Nm * (Nt + 1));
  cd* lam = (cd*)malloc(sizeof(cd) * Nm * (Nt + 1));
  if (!Uk || !x || !lam) {
    free(Uk);
    free(x);
    free(lam);
    return -1;
  }
#pragma omp parallel if (par_k)
  {
    cd* ws = (cd*)malloc(sizeof(cd) * 7 * NN);
    cd* Ak = ws + 6 * NN;
#pragma omp for schedule(static)
    for (int k = 0; k < Nt; ++k) { /* :17-25 */
      memcpy(Ak, A0, sizeof(cd) * NN);
      for (int j = 0; j < nu; ++j) {
        const double uj = u[(size_t)k * nu + j];
        for (size_t e = 0; e < NN; ++e) Ak[e] += uj * Aj[j * NN + e];
      }
      const int r = expm(N, Ak, Uk + NN * k, ws);
      if (degs) {
        degs[2 * k] = r / 64;
        degs[2 * k + 1] = r % 64;
      }
    }
    free(ws);
  }
  memcpy(x, x0, sizeof(cd) * Nm);
  for (int k = 0; k < Nt; ++k) gemm_nm(N, m, Uk + NN * k, x + Nm * k, x + Nm * (k + 1)); /* :27-29 */
  /* J = 1 - |tr(X'x)|^2/n^2, λ_N = -(2Ω/n^2) X  (src/penalty_fcns.jl:15-24) */
  cd om = 0;
  const cd* xN = x + Nm * Nt;
  for (size_t e = 0; e < Nm; ++e) om += conj(Xt[e]) * xN[e];
  *J = 1.0 - (creal(om) * creal(om) + cimag(om) * cimag(om)) / (n * n);
  cd* lN = lam + Nm * Nt;
  for (size_t e = 0; e < Nm; ++e) lN[e] = (-2.0 * om / (n * n)) * Xt[e];
  for (int k = Nt - 1; k >= 0; --k) gemm_h_nm(N, m, Uk + NN * k, lam + Nm * (k + 1), lam + Nm * k); /* :52-58 */
  cd* dU = (cd*)malloc(sizeof(cd) * NN * nu);
  cd* ws = (cd*)malloc(sizeof(cd) * 4 * NN);
  cd* tmp = (cd*)malloc(sizeof(cd) * Nm);
  for (int k = Nt - 1; k >= 0; --k) { /* :65-74 */
    expm_jacobian(N, nu, A0, Aj, u + (size_t)k * nu, order, 1.0, dU, ws);
    for (int j = 0; j < nu; ++j) {
      gemm_nm(N, m, dU + NN * j, x + Nm * k, tmp);
      double s = 0;
      const cd* l = lam + Nm * (k + 1);
      for (size_t e = 0; e < Nm; ++e) s += creal(conj(l[e]) * tmp[e]);
      dJdu[(size_t)k * nu + j] = s;
    }
  }
  free(dU);
  free(ws);
  free(tmp);
  free(Uk);
  free(x);
  free(lam);
  return 0;
}

int qocref_grape_eval(int N, int m, int nu, int Nt, const double* A0, const double* Aj, const double* u,
                      const double* x0, const double* Xt, double n, int order, double* J, double* dJdu, int* degs) {
  return grape_eval1(N, m, nu, Nt, (const cd*)A0, (const cd*)Aj, u, (const cd*)x0, (const cd*)Xt, n, order, J, dJdu,
                     degs, 0);
}

/* B seeds; mode 0 = seed-parallel, 1 = reference-faithful (k-parallel expm, seeds serial). */
int qocref_grape_eval_batch(int N, int m, int nu, int Nt, int B, const double* A0, const double* Aj, const double* u,
                            const double* x0, const double* Xt, double n, int order, double* J, double* dJdu, int mode,
                            int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  int err = 0;
  if (mode == 0) {
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
    for (int b = 0; b < B; ++b)
      err |= grape_eval1(N, m, nu, Nt, (const cd*)A0, (const cd*)Aj, u + (size_t)b * nu * Nt, (const cd*)x0,
                         (const cd*)Xt, n, order, J + b, dJdu + (size_t)b * nu * Nt, NULL, 0);
  } else {
    for (int b = 0; b < B; ++b)
      err |= grape_eval1(N, m, nu, Nt, (const cd*)A0, (const cd*)Aj, u + (size_t)b * nu * Nt, (const cd*)x0,
                         (const cd*)Xt, n, order, J + b, dJdu + (size_t)b * nu * Nt, NULL, 1);
  }
  return err;
}

int qocref_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
