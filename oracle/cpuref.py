"""ctypes wrapper of oracle/build/libqoc_cpuref.so (TEST INFRASTRUCTURE ONLY: tests/ and bench cpu_baseline)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# QOC_CPUREF_LIB: another build of cpu_ref.c (the sanitizer build of `make -C oracle asan`, tools/asan_oracle.sh)
LIB = os.environ.get("QOC_CPUREF_LIB") or os.path.join(HERE, "build", "libqoc_cpuref.so")
_dp = C.POINTER(C.c_double)
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        _lib = C.CDLL(LIB)
        _lib.qocref_grape_eval_batch.argtypes = [C.c_int] * 5 + [_dp] * 5 + [C.c_double, C.c_int, _dp, _dp,
                                                                              C.c_int, C.c_int]
        _lib.qocref_grape_eval.argtypes = [C.c_int] * 4 + [_dp] * 5 + [C.c_double, C.c_int, _dp, _dp,
                                                                       C.POINTER(C.c_int)]
        _lib.qocref_expm.argtypes = [C.c_int, _dp, _dp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        _lib.qocref_expm_jacobian.argtypes = [C.c_int, C.c_int, _dp, _dp, _dp, C.c_int, C.c_double, _dp]
        _lib.qocref_max_threads.restype = C.c_int
        _lib.qocref_set_blas.argtypes = [C.c_char_p]
        _lib.qocref_have_blas.restype = C.c_int
    return _lib


def find_openblas():
    """The OpenBLAS that scipy/numpy ship in this image (LP64 first: its zgemm_ takes 32-bit ints)."""
    import glob
    for pkg in ("scipy", "numpy"):
        try:
            mod = __import__(pkg)
        except Exception:
            continue
        libdir = os.path.join(os.path.dirname(os.path.dirname(mod.__file__)), pkg + ".libs")
        for f in sorted(glob.glob(os.path.join(libdir, "libscipy_openblas-*.so")) +
                        glob.glob(os.path.join(libdir, "libopenblas*.so*"))):
            return f
    return None


def use_blas(enable=True):
    """Route the C port's zgemm / zgesv through the bundled OpenBLAS; returns its path or None."""
    lib = load()
    path = find_openblas() if enable else None
    if path and lib.qocref_set_blas(path.encode()) == 0:
        return path
    lib.qocref_set_blas(None)
    return None


def _cm(a):
    a = np.asarray(a, dtype=np.complex128)
    if a.ndim == 1:
        a = a[:, None]
    return np.ascontiguousarray(a.T).ravel().view(np.float64)


def _p(a):
    return a.ctypes.data_as(_dp)


def expm(A):
    lib = load()
    N = A.shape[0]
    a = _cm(A)
    out = np.zeros_like(a)
    d, s = C.c_int(), C.c_int()
    lib.qocref_expm(N, _p(a), _p(out), C.byref(d), C.byref(s))
    return out.view(np.complex128).reshape(N, N).T.copy(), d.value, s.value


def grape_eval_batch(prob, u, order=3, mode=0, nthreads=0):
    """u: (B, nu, Nt).  Returns J (B,), dJdu (B, nu, Nt)."""
    lib = load()
    B, nu, Nt = u.shape
    N, m = prob.x0.shape
    a0 = _cm(prob.A0)
    aj = np.concatenate([_cm(a) for a in prob.A])
    ub = np.ascontiguousarray(np.transpose(u, (0, 2, 1)))
    x0 = _cm(prob.x0)
    xt = _cm(prob.x_target)
    J = np.zeros(B)
    g = np.zeros((B, Nt, nu))
    rc = lib.qocref_grape_eval_batch(N, m, nu, Nt, B, _p(a0), _p(aj), _p(ub), _p(x0), _p(xt), float(prob.n),
                                     order, _p(J), _p(g), mode, nthreads)
    if rc:
        raise RuntimeError("cpu_ref failed")
    return J, np.transpose(g, (0, 2, 1)).copy()


def max_threads():
    return load().qocref_max_threads()
