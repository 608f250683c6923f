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
        v = e.state(k, self._s) if self._w == "x" else e.costate(k, self._s)
        return c2r(v) if self._c.real_layout else v

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
        x0 = np.asarray(x0)
        if x0.ndim == 1:
            x0 = x0[:, None]
        n = np.shape(A0)[0]
        # src/gradient_computations.jl:84-87: a real x0 is the complex2real layout (2N rows, re/im interleaved,
        # src/utils.jl:8-13) of the ODE path; the states are then handed out in that layout too
        self.real_layout = not np.iscomplexobj(x0)
        if (self.real_layout and x0.shape[0] != 2 * n) or (not self.real_layout and x0.shape[0] != n):
            raise ValueError("Error when creating cache, A0 and x0 have incompatiable dimensions")
        x0 = r2c(x0) if self.real_layout else x0.astype(np.complex128)
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

    def __getitem__(self, i):
        """The reference's positional fields (Julia cache[1] = x, cache[2] = λ, cache[3] = dJdu), 0-based here."""
        return (self.x, self.lam, self.dJdu)[i]


def c2r(x):
    """complex2real (src/utils.jl:8-13): re / im interleaved along the rows, 2N x m."""
    x = np.asarray(x)
    out = np.empty((2 * x.shape[0],) + x.shape[1:], dtype=np.float64)
    out[0::2] = x.real
    out[1::2] = x.imag
    return out


def r2c(x):
    """real2complex (src/utils.jl:14-19)."""
    x = np.asarray(x, dtype=np.float64)
    if x.shape[0] % 2:
        raise ValueError("A must have an even number of rows")
    return x[0::2] + 1j * x[1::2]


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
        # the reference converts x0 to complex before building its cache (src/gradient_computations.jl:4-8), so
        # a real N-row x0 is a complex state; only a 2N-row real x0 is the complex2real layout
        x0c = np.asarray(x0)
        if not np.iscomplexobj(x0c) and x0c.shape[0] != 2 * np.shape(A0)[0]:
            x0c = x0c.astype(np.complex128)
        cache = setup_grape_cache(A0, x0c, u.shape[-2:], B=1 if u.ndim == 2 else u.shape[0])
    if getattr(cache.engine, "prop_method", "expm") != "expm":
        cache.engine.set_propagation("expm")
    return _propagate(A0, A, u, x0, cache)


def _propagate(A0, A, u, x0, cache: MI355XCache):
    e = cache.engine
    e.set_generators(A0, A)
    x0 = np.asarray(x0)
    if x0.ndim == 1:
        x0 = x0[:, None]
    x0 = r2c(x0) if not np.iscomplexobj(x0) and x0.shape[0] == 2 * e.N else x0.astype(np.complex128)
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
    lam = np.stack([np.asarray(dJfinal_dx(e.state(-1, b)), dtype=np.complex128).reshape(e.N, -1)
                    for b in range(B)])  # :46
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


def generators_from_rhs(f, n, nu):
    """The complex generators behind a reference right-hand side f(dx, x, p, t) (the examples' setup_dxdt: dx/dt
    of one state column in the complex2real layout, p = u_k): sampled on the 2n basis vectors at p = 0 and
    p = e_j.  Raises ValueError unless f is x -> (M0 + sum_j p_j M_j) x for complex matrices M (what
    wrap_pwc's ODE is on the GRAPE path); the GPU then integrates that ODE."""
    def call(dx, x, p):  # wrap_pwc passes (dx, x, p, t); Symbolics' in-place builds take (dx, x, p)
        try:
            f(dx, x, p, 0.0)
        except TypeError:
            f(dx, x, p)

    def real_matrix(p):
        R = np.zeros((2 * n, 2 * n))
        for i in range(2 * n):
            x = np.zeros(2 * n)
            x[i] = 1.0
            dx = np.zeros(2 * n)
            call(dx, x, p)
            R[:, i] = dx
        return R

    def to_complex(R):
        M = R[0::2, 0::2] + 1j * R[1::2, 0::2]
        if not (np.allclose(R[1::2, 1::2], M.real, rtol=0, atol=1e-14 * max(1.0, np.abs(R).max())) and
                np.allclose(R[0::2, 1::2], -M.imag, rtol=0, atol=1e-14 * max(1.0, np.abs(R).max()))):
            raise ValueError("the right-hand side is not a complex-linear map in the complex2real layout")
        return M
    R0 = real_matrix(np.zeros(nu))
    M0 = to_complex(R0)
    Ms = [to_complex(real_matrix(np.eye(nu)[j]) - R0) for j in range(nu)]
    rng = np.random.default_rng(0)  # affine in p, linear in x: one random check
    p, x = rng.standard_normal(nu), rng.standard_normal(2 * n)
    dx = np.zeros(2 * n)
    call(dx, x, p)
    want = c2r((M0 + sum(p[j] * Ms[j] for j in range(nu))) @ r2c(x))
    if not np.allclose(dx, want, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(want).max())):
        raise ValueError("the right-hand side is not x -> (A0 + sum_j p_j A_j) x")
    return M0, Ms


class PwcSolution:
    """What the reference's propagate_pwc returns (an ODESolution saved at [0, tgate]): .t and .u."""

    def __init__(self, t, u):
        self.t, self.u = t, u


def propagate_pwc(*args, **kw):
    """propagate_pwc (src/gradient_computations.jl:108-128) on the GPU, in both call forms:

    * the reference's, propagate_pwc(f, x0, u, Δt, cache=None; dt): f(dx, x, p, t) the right-hand side on one
      column in the complex2real layout (examples/models/setup_diffeq_rhs.jl), x0 real 2N x m.  The generators
      are recovered from f (generators_from_rhs) and the result is the reference's solution object (.u =
      [x(0), x(tgate)], real layout); the states of every slice are in cache.x;
    * propagate_pwc(A0, A, x0, u, Δt, cache=None, dt=None) with the physical generators (-iH, not Δt-scaled).
    dx/dt = (A0 + sum_j u_jk A_j) x on [kΔt, (k+1)Δt) with fixed Tsit5 steps dt (default 0.1Δt)."""
    if callable(args[0]):
        f, x0, u, Δt = args[:4]
        cache = args[4] if len(args) > 4 else kw.pop("cache", None)
        dt = kw.pop("dt", None)
        u = np.asarray(u, dtype=np.float64)
        x0 = np.asarray(x0)
        if x0.ndim == 1:
            x0 = x0[:, None]
        if np.iscomplexobj(x0) or x0.shape[0] % 2:
            raise ValueError("propagate_pwc(f, x0, ...) takes x0 in the complex2real layout (real, 2N rows)")
        n = x0.shape[0] // 2
        A0, A = generators_from_rhs(f, n, u.shape[-2])
        if cache is None:
            cache = setup_grape_cache(A0, x0, u.shape[-2:], B=1 if u.ndim == 2 else u.shape[0])
        xs = _propagate_pwc(A0, A, x0, u, Δt, cache, dt)
        return PwcSolution([0.0, Δt * u.shape[-1]], [xs[0], xs[-1]])
    return _propagate_pwc(*args, **kw)


def _propagate_pwc(A0, A, x0, u, Δt, cache: MI355XCache | None = None, dt=None):
    u = np.asarray(u, dtype=np.float64)
    if cache is None:
        cache = setup_grape_cache(A0, x0, u.shape[-2:], B=1 if u.ndim == 2 else u.shape[0])
    e = cache.engine
    e.set_propagation("tsit5", _nsub(Δt, dt))
    return _propagate(Δt * np.asarray(A0, dtype=np.complex128), [Δt * np.asarray(a, dtype=np.complex128) for a in A],
                      u, x0, cache)


def compute_pwc_gradient(*args, dUkdp_order=2, dt=None, x0=None, **kw):
    """compute_pwc_gradient (src/gradient_computations.jl:130-169): co-states by the adjoint ODE
    dλ/dt = -A_k^H λ with the same fixed steps, then dJdu[j, k] from expm_jacobian! of order
    dUkdp_order.  dUkdp_order = 0 returns after the co-state sweep, as the reference does (:152).
    Call after propagate_pwc with the same u (the stale-u check of grape_sensitivity applies).

    Call forms: the reference's compute_pwc_gradient(dλdt, dJfinal_dx, u, Δt, A0, A, cache; dUkdp_order, dt),
    where dλdt(dλ, λ, p, t) is the adjoint right-hand side in the complex2real layout (checked against -A^H
    of the generators), and compute_pwc_gradient(dJfinal_dx, u, Δt, A0, A, cache, ...)."""
    if len(args) >= 7 and callable(args[0]) and callable(args[1]):
        dldt, dJfinal_dx, u, Δt, A0, A, cache = args[:7]
        n = np.shape(A0)[0]
        M0, Ms = generators_from_rhs(dldt, n, len(A))
        tol = 1e-12 * max(1.0, np.abs(np.asarray(A0)).max())
        if not (np.allclose(M0, -np.asarray(A0).conj().T, atol=tol) and
                all(np.allclose(Mj, -np.asarray(a).conj().T, atol=tol) for Mj, a in zip(Ms, A))):
            raise ValueError("dλdt is not the adjoint of the generators A0, A (dλ/dt = -A(u)^H λ)")
    else:
        dJfinal_dx, u, Δt, A0, A, cache = args[:6]
    return _compute_pwc_gradient(dJfinal_dx, u, Δt, A0, A, cache, dUkdp_order, dt, x0)


def _compute_pwc_gradient(dJfinal_dx, u, Δt, A0, A, cache: MI355XCache, dUkdp_order=2, dt=None, x0=None):
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
