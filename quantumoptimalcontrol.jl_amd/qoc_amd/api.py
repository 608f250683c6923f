"""Reference-shaped host API: the functions the Ipopt callbacks call, backed by the MI355X engine.

Mirrors (same names, argument meaning and error behaviour):
  * ``setup_grape_cache(A0, x0, u_size)``                 src/gradient_computations.jl:79-96
  * ``propagate(A0, A, u, x0, cache)``                     src/gradient_computations.jl:2-32
  * ``grape_sensitivity(A0, A, dJfinal_dx, u, x0, cache; dUkdp_order=3, dL_dx)``  :35-77
  * ``propagate_pwc``, ``compute_pwc_gradient`` (the ODE/Tsit5 path)  :108-169
  * ``setup_infidelity``, ``setup_infidelity_zcalibrated``, ``setup_state_penalty``
                                                          src/penalty_fcns.jl:1-42
so ``examples/ipopt_callbacks_exp.jl`` reads the same with this module in place of
``QuantumOptimalControl``.  The returned cost closures are ordinary callables on numpy
arrays (as in the reference) and carry a ``kind`` tag that lets the engine evaluate them
on the GPU; an untagged ``dJfinal_dx`` closure is evaluated on the host at x[end] and its
value handed to the device as λ_{Nt+1} (QOC_COST_EXTERNAL), exactly the reference's data flow.
"""
from __future__ import annotations

import math

import numpy as np

from .engine import GrapeEngine, expm, expm_jacobian  # noqa: F401  (re-exported)
from .systems import setup_bilinear_matrices  # noqa: F401
from ._lib import StaleCacheError  # noqa: F401


# ---------------------------------------------------------------------------
# Tagged cost closures (src/penalty_fcns.jl)
# ---------------------------------------------------------------------------
class _Tagged:
    def __init__(self, fn, kind, **meta):
        self._fn = fn
        self.kind = kind
        self.meta = meta

    def __call__(self, x):
        return self._fn(np.asarray(x))


def setup_infidelity(x_target, n=None):
    """(J, dJ_dx): J = 1 - |tr(X'x)|^2/n^2, dJ/dx = -(2Ω/n^2) X (src/penalty_fcns.jl:15-24)."""
    X = np.asarray(x_target, dtype=np.complex128)
    if X.ndim == 1:
        X = X[:, None]
    n = X.shape[1] if n is None else n

    def J(x):
        return float(1 - abs(np.trace(X.conj().T @ x)) ** 2 / n ** 2)

    def dJ(x):
        return (-2 * np.trace(X.conj().T @ x) / n ** 2) * X
    return _Tagged(J, "trace", X=X, n=n), _Tagged(dJ, "trace", X=X, n=n)


def _optimal_calibration(m, tol=1e-9):
    """Host copy of the golden-section calibration (src/fidelities.jl:81-137) for J(x) only."""
    ab = [abs(complex(v)) for v in m]
    ang = [math.atan2(complex(v).imag, complex(v).real) for v in m]
    a1, b1 = ab[0] ** 2 + ab[1] ** 2, 2 * ab[0] * ab[1]
    a2, b2 = ab[2] ** 2 + ab[3] ** 2, 2 * ab[2] * ab[3]
    p1 = (ang[0] - ang[1]) % (2 * math.pi)
    p2 = (ang[2] - ang[3]) % (2 * math.pi)
    if abs(p2 - p1) <= math.pi:
        pm, D, al = (p1 + p2) / 2, abs(p2 - p1) / 2, (1 if p1 < p2 else -1)
    else:
        pm, D, al = (2 * math.pi + p1 + p2) / 2, math.pi - abs(p2 - p1) / 2, (-1 if p1 < p2 else 1)
    f = lambda d: -(math.sqrt(a1 + b1 * math.cos(d + D)) + math.sqrt(a2 + b2 * math.cos(d - D)))  # noqa: E731
    lo, hi = -D, D
    gr = 0.5 * (3.0 - math.sqrt(5.0))
    xm = lo + gr * (hi - lo)
    fm = f(xm)
    while hi - lo >= tol:
        if hi - xm > xm - lo:
            xn = xm + gr * (hi - xm)
            fn = f(xn)
            if fn < fm:
                lo, xm, fm = xm, xn, fn
            else:
                hi = xn
        else:
            xn = xm - gr * (xm - lo)
            fn = f(xn)
            if fn < fm:
                hi, xm, fm = xm, xn, fn
            else:
                lo = xn
    return -fm, pm + al * xm


def setup_infidelity_zcalibrated(x_target):
    """Z-calibrated infidelity (src/penalty_fcns.jl:27-42); x_target must have 4 columns."""
    X = np.asarray(x_target, dtype=np.complex128)
    if X.shape[1] != 4:
        raise ValueError("Only works for two-qubit gates, x_target must have four columns")

    def J(x):
        F, _ = _optimal_calibration(np.diag(X.conj().T @ x))
        return float(1 - F ** 2 / 16)

    def dJ(x):
        m = np.diag(X.conj().T @ x)
        F, th = _optimal_calibration(m)
        e = complex(math.cos(th), math.sin(th))
        v1, v2 = m[0] + e * m[1], m[2] + e * m[3]
        g = np.array([v1 / abs(v1), v1 / abs(v1) / e, v2 / abs(v2), v2 / abs(v2) / e])
        return (-2 * F / 16) * (X * g[None, :])
    return _Tagged(J, "zcal", X=X), _Tagged(dJ, "zcal", X=X)


def setup_state_penalty(inds_penalty, inds_css, mu):
    """(L, dL_dx) guard-state penalty (src/penalty_fcns.jl:1-11); 0-based indices."""
    P = np.asarray(inds_penalty, dtype=np.int64)
    Cc = np.asarray(inds_css, dtype=np.int64)

    def L(x):
        return float(mu * np.sum(np.abs(np.asarray(x)[np.ix_(P, Cc)]) ** 2))

    def dL(x):
        x = np.asarray(x, dtype=np.complex128)
        g = np.zeros_like(x)
        g[np.ix_(P, Cc)] = 2 * mu * x[np.ix_(P, Cc)]
        return g
    meta = dict(P=P, C=Cc, mu=float(mu))
    return _Tagged(L, "penalty", **meta), _Tagged(dL, "penalty", **meta)


# ---------------------------------------------------------------------------
# Cache + hot path
# ---------------------------------------------------------------------------
class _LazySeries:
    """Read-only, lazily fetched list of the Nt+1 states (or co-states) of one seed."""

    def __init__(self, cache, which, seed=0):
        self._c, self._w, self._s = cache, which, seed

    def __len__(self):
        return self._c.engine.Nt + 1

    def __getitem__(self, k):
        n = len(self)
        if isinstance(k, slice):
            return [self[i] for i in range(*k.indices(n))]
        if k < 0:
            k += n
        if not 0 <= k < n:
            raise IndexError(k)
        e = self._c.engine
        return e.state(k, self._s) if self._w == "x" else e.costate(k, self._s)

    def __iter__(self):
        for k in range(len(self)):
            yield self[k]


class MI355XCache:
    """GPU-resident replacement of the tuple returned by ``setup_grape_cache``.

    Fields read by callers in the reference — ``.u``, ``.x``, ``.λ`` (here ``.lam``),
    ``.dJdu`` — are exposed; ``x``/``lam`` fetch lazily from HBM.
    """

    def __init__(self, A0, x0, u_size, B=1, precision="fp64", device=0, compress=None):
        nu, Nt = u_size
        x0 = np.asarray(x0, dtype=np.complex128)
        if x0.ndim == 1:
            x0 = x0[:, None]
        placeholder = [np.zeros_like(np.asarray(A0, dtype=np.complex128)) for _ in range(nu)]
        self.engine = GrapeEngine(A0, placeholder, x0, Nt, B, precision, device)
        self.engine.set_cost_external()
        if compress is not None:
            self.engine.set_compression(compress)
        self.u = np.zeros((nu, Nt)) if B == 1 else np.zeros((B, nu, Nt))
        self.dJdu = None
        self._penalty = None
        self._propagated = False

    @property
    def x(self):
        return _LazySeries(self, "x")

    @property
    def lam(self):
        return _LazySeries(self, "lam")

    def series(self, which, seed):
        return _LazySeries(self, which, seed)


def setup_grape_cache(A0, x0, u_size, B=1, precision="fp64", device=0, compress=None) -> MI355XCache:
    """Workspace on the GPU (src/gradient_computations.jl:79-96); errors on a dimension mismatch.
    compress = ((rows1, cols1), (rows2, cols2)) (0-based, compress_states' v, src/utils.jl:96-109) runs the
    kernels on the packed columns; x, λ, dL_dx and dJfinal_dx keep the caller's layout."""
    return MI355XCache(A0, x0, u_size, B, precision, device, compress)


def propagate(A0, A, u, x0, cache: MI355XCache | None = None):
    """Forward PWC propagation (src/gradient_computations.jl:2-32), U_k = exp(A_k); returns the lazy x series.
    A cache last used by propagate_pwc (Tsit5) is switched back to the exponential."""
    u = np.asarray(u, dtype=np.float64)
    if cache is None:
        cache = setup_grape_cache(A0, x0, u.shape[-2:], B=1 if u.ndim == 2 else u.shape[0])
    if getattr(cache.engine, "prop_method", "expm") != "expm":
        cache.engine.set_propagation("expm")
    return _propagate(A0, A, u, x0, cache)


def _propagate(A0, A, u, x0, cache: MI355XCache):
    e = cache.engine
    e.set_generators(A0, A)
    x0 = np.asarray(x0, dtype=np.complex128)
    if x0.ndim == 1:
        x0 = x0[:, None]
    if not np.array_equal(x0, e.x0):
        e.set_x0(x0)
    e.propagate(u)
    cache.u = u.copy()        # :12 (kept for the stale check)
    cache._propagated = True
    return cache.x


def grape_sensitivity(A0, A, dJfinal_dx, u, x0, cache: MI355XCache, dUkdp_order=3, dL_dx=None):
    """Co-states + gradient (src/gradient_computations.jl:35-77); returns dJdu (nu x Nt, or B x nu x Nt)."""
    u = np.asarray(u, dtype=np.float64)
    if not cache._propagated or u.shape != cache.u.shape or not np.array_equal(u, cache.u):
        raise StaleCacheError(-3, "Cache data from other control signal u")          # :37-39
    e = cache.engine
    B = e.B
    src = None
    if dL_dx is not None and getattr(dL_dx, "kind", None) == "penalty":
        m = dL_dx.meta
        e.set_state_penalty(m["P"], m["C"], m["mu"])  # applied on the GPU at every slice
    else:
        e.set_state_penalty([], [], 0.0)
        if dL_dx is not None:  # any other closure: evaluated here on every state, added to λ_k on the GPU
            src = np.stack([[np.asarray(dL_dx(e.state(k, b)), dtype=np.complex128) for k in range(e.Nt + 1)]
                            for b in range(B)])
    e.set_costate_source(src)
    lam = np.stack([np.asarray(dJfinal_dx(e.state(-1, b)), dtype=np.complex128) for b in range(B)])  # :46
    dJdu = e.grape_sensitivity(u, dUkdp_order, lambda_final=lam)
    if src is not None:
        e.set_costate_source(None)
    cache.dJdu = dJdu[0] if u.ndim == 2 else dJdu
    return cache.dJdu


# ---------------------------------------------------------------------------
# ODE path (src/gradient_computations.jl:108-169): fixed-step Tsit5 on the GPU
# ---------------------------------------------------------------------------
def _nsub(Δt, dt):
    nsub = 10 if dt is None else int(round(Δt / dt))
    if nsub < 1 or (dt is not None and abs(nsub * dt - Δt) > 1e-9 * Δt):
        raise ValueError(f"dt = {dt} must divide Δt = {Δt}")
    return nsub


def propagate_pwc(A0, A, x0, u, Δt, cache: MI355XCache | None = None, dt=None):
    """propagate_pwc (src/gradient_computations.jl:108-128): dx/dt = (A0 + sum_j u_jk A_j) x on
    [kΔt, (k+1)Δt) with fixed Tsit5 steps dt (default 0.1Δt).  A0, A are the physical generators
    (-iH, not Δt-scaled) in place of the reference's `f` closure; returns the slice-boundary states."""
    u = np.asarray(u, dtype=np.float64)
    if cache is None:
        cache = setup_grape_cache(A0, x0, u.shape[-2:], B=1 if u.ndim == 2 else u.shape[0])
    e = cache.engine
    e.set_propagation("tsit5", _nsub(Δt, dt))
    return _propagate(Δt * np.asarray(A0, dtype=np.complex128), [Δt * np.asarray(a, dtype=np.complex128) for a in A],
                      u, x0, cache)


def compute_pwc_gradient(dJfinal_dx, u, Δt, A0, A, cache: MI355XCache, dUkdp_order=2, dt=None, x0=None):
    """compute_pwc_gradient (src/gradient_computations.jl:130-169): co-states by the adjoint ODE
    dλ/dt = -A_k^H λ with the same fixed steps, then dJdu[j, k] from expm_jacobian! of order
    dUkdp_order.  dUkdp_order = 0 returns after the co-state sweep, as the reference does (:152).
    Call after propagate_pwc with the same u (the stale-u check of grape_sensitivity applies)."""
    e = cache.engine
    nsub = _nsub(Δt, dt)
    if (getattr(e, "prop_method", "expm"), getattr(e, "nsub", None)) != ("tsit5", nsub):
        raise ValueError("compute_pwc_gradient needs the states of propagate_pwc with the same dt")
    A0s = Δt * np.asarray(A0, dtype=np.complex128)
    As = [Δt * np.asarray(a, dtype=np.complex128) for a in A]
    x0 = e.x0 if x0 is None else x0
    if dUkdp_order == 0:  # :152
        return cache.dJdu if cache.dJdu is not None else np.zeros_like(np.asarray(u, dtype=np.float64))
    return grape_sensitivity(A0s, As, dJfinal_dx, u, x0, cache, dUkdp_order=dUkdp_order)
