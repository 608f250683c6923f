"""Host-side problem construction for the GRAPE hot path (numpy, one-time setup).

Restates the reference's operator helpers (``src/utils.jl``) and the model
files under ``examples/models/`` so that the bench and the parity tests can
build the BASELINE.json configurations.  Nothing here runs per iteration; it
only produces the Δt-prescaled generators, x0, targets and synthetic controls
that are handed to the MI355X engine.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


# ---------------------------------------------------------------------------
# Operators (src/utils.jl:35-91)
# ---------------------------------------------------------------------------
def annihilation_op(dim: int) -> np.ndarray:
    """diagm(1 => sqrt.(1:dim-1)) (src/utils.jl:66)."""
    return np.diag(np.sqrt(np.arange(1, dim, dtype=np.float64)), k=1)


def annihilation_ops(*dims: int) -> list[np.ndarray]:
    """Embedded annihilation operators, first subsystem outermost (src/utils.jl:67-71)."""
    out = []
    for j in range(len(dims)):
        op = np.ones((1, 1))
        for k, n in enumerate(dims):
            op = np.kron(op, annihilation_op(n) if k == j else np.eye(n))
        out.append(op)
    return out


def qubit_hamiltonian(wr: float, alpha: float, n: int) -> np.ndarray:
    """diagm([k wr + alpha (k-1) k / 2]) (src/utils.jl:74)."""
    return np.diag([k * wr + alpha * (k - 1) * k / 2 for k in range(n)])


class QuantumBasis:
    """Labelled product basis (src/utils.jl:35-63); labels are digit strings, first subsystem first."""

    def __init__(self, dims):
        self.dims = list(dims)
        labels = [""]
        for n in self.dims:
            labels = [a + str(d) for a in labels for d in range(n)]
        self.state_dict = {s: i for i, s in enumerate(labels)}  # 0-based
        self.Ntot = int(np.prod(self.dims))

    def __call__(self, s):
        if isinstance(s, str):
            return self.state_dict[s]
        return [self.state_dict[x] for x in s]

    def columns(self, labels) -> np.ndarray:
        """qb[:, labels] = columns of the identity (src/utils.jl:47-51)."""
        eye = np.eye(self.Ntot)
        return eye[:, [self.state_dict[s] for s in labels]]


def setup_bilinear_matrices(H0, Tc, dt=1.0):
    """A0Δt = -i H0 Δt, A1Δt = -i (Tc+Tc') Δt, A2Δt = -i (i (Tc-Tc')) Δt (src/utils.jl:86-91)."""
    H0 = np.asarray(H0, dtype=np.complex128)
    Tc = np.asarray(Tc, dtype=np.complex128)
    return (-1j * H0 * dt,
            -1j * (Tc + Tc.conj().T) * dt,
            -1j * (1j * (Tc - Tc.conj().T)) * dt)


def gate_unitary(gatetype: str) -> np.ndarray:
    """CNOT / iSwap / CZ (src/utils.jl:112-133)."""
    U = np.zeros((4, 4))
    if gatetype == "CNOT":
        U[0, 0] = U[1, 1] = U[2, 3] = U[3, 2] = 1
    elif gatetype == "iSwap":
        U[0, 0] = U[2, 1] = U[1, 2] = U[3, 3] = 1
    elif gatetype == "CZ":
        U[0, 0] = U[1, 1] = U[2, 2] = 1
        U[3, 3] = -1
    else:
        raise ValueError("Unknown gate type")
    return U


# ---------------------------------------------------------------------------
# Spline control parameterisation (examples/zz_coupling_ipopt_exp.jl:27-37)
# ---------------------------------------------------------------------------
def _bspline_basis(knots: np.ndarray, order: int, t: float) -> np.ndarray:
    """Cox-de Boor evaluation of all B-splines of `order` at t (right-continuous, last knot closed)."""
    nb = len(knots) - order
    # order-1 indicator functions
    B = np.zeros(len(knots) - 1)
    last = len(knots) - 1
    for i in range(len(knots) - 1):
        if knots[i] <= t < knots[i + 1] or (t == knots[last] and knots[i] < t == knots[i + 1]):
            B[i] = 1.0
    for k in range(2, order + 1):
        Bn = np.zeros(len(knots) - k)
        for i in range(len(knots) - k):
            a = 0.0
            d1 = knots[i + k - 1] - knots[i]
            if d1 > 0:
                a += (t - knots[i]) / d1 * B[i]
            d2 = knots[i + k] - knots[i + 1]
            if d2 > 0:
                a += (knots[i + k] - t) / d2 * B[i + 1]
            Bn[i] = a
        B = Bn
    return B[:nb]


def spline_matrix(tgate: float, Nt: int, nsplines: int) -> np.ndarray:
    """B (Nt x nsplines): cubic B-splines at slice midpoints, interior columns 4:end-3.

    Mirrors ``BSplineBasis(4, LinRange(0,tgate,nsplines+4))`` evaluated at
    ``t_midpoints`` and ``B = Bpre[:, 4:end-3]`` (examples/zz_coupling_ipopt_exp.jl:27-37).
    """
    order = 4
    bp = np.linspace(0.0, tgate, nsplines + 4)
    knots = np.concatenate([[bp[0]] * (order - 1), bp, [bp[-1]] * (order - 1)])
    dt = tgate / Nt
    tm = np.arange(Nt) * dt + dt / 2
    Bpre = np.stack([_bspline_basis(knots, order, t) for t in tm])
    return Bpre[:, 3:-3]


# ---------------------------------------------------------------------------
# Column packing for parity-structured problems (src/utils.jl:96-109)
# ---------------------------------------------------------------------------
def compress_states(x, v):
    """Pack the two disjoint (rows, cols) blocks of x into max(n1, n2) columns (src/utils.jl:96-102).

    v = ((rows1, cols1), (rows2, cols2)) with 0-based index sequences.
    """
    (r1, c1), (r2, c2) = v
    x = np.asarray(x)
    n1, n2 = len(c1), len(c2)
    out = np.zeros((x.shape[0], max(n1, n2)), dtype=x.dtype)
    out[np.ix_(list(r1), range(n1))] = x[np.ix_(list(r1), list(c1))]
    out[np.ix_(list(r2), range(n2))] = x[np.ix_(list(r2), list(c2))]
    return out


def decompress_states(xc, v):
    """Inverse of compress_states (src/utils.jl:103-109)."""
    (r1, c1), (r2, c2) = v
    xc = np.asarray(xc)
    n1, n2 = len(c1), len(c2)
    out = np.zeros((xc.shape[0], n1 + n2), dtype=xc.dtype)
    out[np.ix_(list(r1), list(c1))] = xc[np.ix_(list(r1), range(n1))]
    out[np.ix_(list(r2), list(c2))] = xc[np.ix_(list(r2), range(n2))]
    return out


def compress_problem(prob, v):
    """Problem with x0 / x_target packed by compress_states: m drops to max(n1, n2).

    Valid when every generator maps span(rows1) and span(rows2) into themselves (block-diagonal in
    the row partition), so U_k commutes with the packing and the chains, the trace cost (entries outside
    the blocks are zero in x) and the gradient are unchanged.  Raises ValueError otherwise.
    """
    (r1, _), (r2, _) = v
    r1, r2 = list(r1), list(r2)
    for G in [prob.A0] + list(prob.A):
        G = np.asarray(G)
        if np.abs(G[np.ix_(r1, r2)]).max(initial=0.0) > 0 or np.abs(G[np.ix_(r2, r1)]).max(initial=0.0) > 0:
            raise ValueError("generators couple the two row blocks; compress_states does not apply")
    return Problem(prob.name + "_compressed", prob.A0, list(prob.A), compress_states(prob.x0, v),
                   compress_states(prob.x_target, v), prob.n, prob.Nt, prob.precision)


# ---------------------------------------------------------------------------
# Problem container
# ---------------------------------------------------------------------------
@dataclass
class Problem:
    name: str
    A0: np.ndarray            # N x N complex, Δt-prescaled
    A: list                   # nu matrices N x N complex
    x0: np.ndarray            # N x m complex
    x_target: np.ndarray      # N x m complex
    n: float                  # infidelity normalisation (src/penalty_fcns.jl:15)
    Nt: int
    precision: str            # "fp64" | "fp32"

    @property
    def N(self):
        return self.A0.shape[0]

    @property
    def m(self):
        return self.x0.shape[1]

    @property
    def nu(self):
        return len(self.A)


# ---------------------------------------------------------------------------
# BASELINE.json configurations
# ---------------------------------------------------------------------------
def zz_coupling_model():
    """examples/models/zz_coupling.jl:6-24 (dim 9)."""
    dimq = dims = 3
    aq = annihilation_op(dimq)
    as_ = annihilation_op(dims)
    al_q = 2 * math.pi * 0.2
    al_s = 2 * math.pi * 0.2
    X = 2 * math.pi * 1e-4
    Hq = -al_q / 2 * np.kron(aq.T @ aq.T @ aq @ aq, np.eye(dims))
    Hs = -al_s / 2 * np.kron(np.eye(dimq), as_.T @ as_.T @ as_ @ as_)
    Hint = -X * np.kron(aq.T @ aq, as_.T @ as_)
    Tc = np.kron(aq.T, np.eye(dims))
    qb = QuantumBasis([dimq, dims])
    return Hq + Hs + Hint, Tc, qb


def zz_problem(Nt=100, tgate=None) -> Problem:
    """Config 1/2: NOT gate on the computational subspace (examples/zz_coupling_ipopt_exp.jl:8-23)."""
    H0, Tc, qb = zz_coupling_model()
    if tgate is None:
        tgate = 10.0 if Nt == 100 else 20.0 * Nt / 500
    dt = tgate / Nt
    A0, A1, A2 = setup_bilinear_matrices(H0, Tc, dt)
    Q = qb.columns(["00", "01", "10", "11"])
    css_target = np.kron(np.array([[0, 1], [1, 0]]), np.eye(2))
    return Problem("zz_coupling", A0, [A1, A2], Q.astype(np.complex128),
                   (Q @ css_target).astype(np.complex128), 4.0, Nt, "fp64")


def zz_controls(B: int, Nt: int, tgate: float, seed=0, nsplines=10) -> np.ndarray:
    """u[b] = (Bspl c_b)^T, c_b ~ U(-2pi*0.06, 2pi*0.06) (Ipopt box, examples/zz_coupling_ipopt_exp.jl:54-56)."""
    rng = np.random.default_rng(seed)
    Bs = spline_matrix(tgate, Nt, nsplines)
    cmax = 2 * math.pi * 0.060
    c = rng.uniform(-cmax, cmax, size=(B, nsplines, 2))
    return np.einsum("tn,bnj->bjt", Bs, c)  # B x nu x Nt


def cavity_model(N_cavity=12, N_qubit=2):
    """examples/models/cavity_qubit.jl:6-49 (qubit first in the tensor product)."""
    xi = 2 * math.pi * (-2.574749e-3)
    a = annihilation_op(N_cavity)
    b = annihilation_op(N_qubit)
    H0 = xi * np.kron(b.T @ b, a.T @ a)  # K = alpha = xip = wt = wc = 0
    Tc = np.kron(b.T, np.eye(N_cavity))
    theta = np.zeros(N_cavity)
    th = [3.6348672, 1.1435776, 0.0, 1.7441809, -0.4598031, -0.37506938, -0.27870846]
    theta[:min(len(th), N_cavity)] = th[:N_cavity]
    return H0, Tc, theta


def cavity_problem(N_cavity=20, Nt=1000, dt=1.0) -> Problem:
    """Config 3 (test/test_gradient_computation.jl:16-22 with N_cavity=20): Tc/2 drive, m=2."""
    H0, Tc, theta = cavity_model(N_cavity)
    A0, A1, A2 = setup_bilinear_matrices(H0, Tc / 2, dt)
    nc = N_cavity
    c0 = np.concatenate([np.ones(nc), np.zeros(nc)])
    c1 = np.concatenate([np.zeros(nc), np.ones(nc)])
    x0 = np.stack([c0 / np.linalg.norm(c0), c1 / np.linalg.norm(c1)], axis=1)
    t0 = np.kron([1, 1], np.exp(1j * theta))
    xt = np.stack([t0 / np.linalg.norm(t0), c1 / np.linalg.norm(c1)], axis=1)
    return Problem("cavity_qubit", A0, [A1, A2], x0.astype(np.complex128),
                   xt.astype(np.complex128), 2.0, Nt, "fp64")


def cavity_dense_problem(N_cavity=20, Nt=1000, dt=1.0) -> Problem:
    """Config 3 with a drive that also displaces the cavity: Tc = b^dag (x) I + I (x) a^dag (one drive line coupled to
    both modes), so that the generators no longer split into the 2 x 2 invariant blocks of the qubit-only drive
    (examples/models/cavity_qubit.jl:27, Tc = kron(b', I)) and the dense Taylor-action chains and fused gradient
    run.  Same H0, x0, target and controls as cavity_problem."""
    H0, Tc, theta = cavity_model(N_cavity)
    a = annihilation_op(N_cavity)
    Tc = Tc + np.kron(np.eye(2), a.T)
    A0, A1, A2 = setup_bilinear_matrices(H0, Tc / 2, dt)
    base = cavity_problem(N_cavity, Nt, dt)
    return Problem("cavity_qubit_dense", A0, [A1, A2], base.x0, base.x_target, base.n, Nt, "fp64")


def cavity_controls(B, Nt, seed=0, umax=0.05) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.uniform(-umax, umax, size=(B, 2, Nt))


def tunable_bus_model():
    """examples/models/two_qubit_tunable_bus.jl:7-28 (dim 27)."""
    w1, w2, wc0 = 4.5 * 2 * math.pi, 4.2 * 2 * math.pi, 7.5 * 2 * math.pi
    al1 = al2 = -0.2 * 2 * math.pi
    g1 = g2 = 0.04 * 2 * math.pi
    qb = QuantumBasis([3, 3, 3])
    a1, a2, ac = annihilation_ops(*qb.dims)
    I = np.eye(qb.Ntot)
    n1, n2 = a1.T @ a1, a2.T @ a2
    Hq1 = w1 * n1 + al1 * n1 @ (n1 - I)
    Hq2 = w2 * n2 + al2 * n2 @ (n2 - I)
    Hi1 = g1 * (a1.T + a1) @ (ac.T + ac)
    Hi2 = g2 * (a2.T + a2) @ (ac.T + ac)
    Hc = wc0 * ac.T @ ac
    return Hq1 + Hq2 + Hi1 + Hi2, Hc, qb


def tunable_bus_problem(Nt=2000, tgate=350.0) -> Problem:
    """Config 4: |110> -> |200> population transfer, single flux control (examples/two_qubit_tunable_bus.jl:42-51)."""
    H0, Hc, qb = tunable_bus_model()
    dt = tgate / Nt
    A0 = -1j * H0 * dt
    A1 = -1j * Hc * dt
    x0 = qb.columns(["110"]).astype(np.complex128)
    xt = qb.columns(["200"]).astype(np.complex128)
    return Problem("two_qubit_tunable_bus", A0, [A1], x0, xt, 1.0, Nt, "fp64")


def tunable_bus_cz_problem(Nt=2000, tgate=350.0) -> Problem:
    """The tunable-bus model driven as a CZ gate on the four computational states |q1 c q2> = |000>, |001>,
    |100>, |101> (coupler in 0; m = 4, the z-calibrated cost's two-qubit case).  The Hamiltonian conserves
    excitation number, so it is block-diagonal in the parity of the basis index: TUNABLE_BUS_PARITY is the
    compress_states spec of test/test_utils.jl:23 (rows 1:2:27 with columns [1, 4], rows 2:2:26 with [2, 3],
    here 0-based)."""
    H0, Hc, qb = tunable_bus_model()
    dt = tgate / Nt
    x0 = qb.columns(["000", "001", "100", "101"]).astype(np.complex128)
    xt = x0 @ gate_unitary("CZ").astype(np.complex128)
    return Problem("two_qubit_tunable_bus_cz", -1j * H0 * dt, [-1j * Hc * dt], x0, xt, 4.0, Nt, "fp64")


TUNABLE_BUS_PARITY = ((list(range(0, 27, 2)), [0, 3]), (list(range(1, 27, 2)), [1, 2]))


def tunable_bus_controls(B, Nt, seed=0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.uniform(0.3, 1.0, size=(B, 1, Nt))


def _gue(rng, N):
    G = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    return (G + G.conj().T) / 2


def synthetic_problem(N=256, Nt=1000, nu=2, seed=0, precision="fp32") -> Problem:
    """Config 5: GUE H0/H_j rescaled to ||dt H0||_1 = 3.5, ||dt H_j||_1 = 0.5; x0 = I; Haar target."""
    rng = np.random.default_rng(seed)

    def scaled(H, norm):
        return H * (norm / np.abs(H).sum(axis=0).max())
    A0 = -1j * scaled(_gue(rng, N), 3.5)
    A = [-1j * scaled(_gue(rng, N), 0.5) for _ in range(nu)]
    Z = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    Q, R = np.linalg.qr(Z)
    Q = Q * (np.diag(R) / np.abs(np.diag(R)))[None, :]
    return Problem("synthetic", A0, A, np.eye(N, dtype=np.complex128), Q, float(N), Nt, precision)


def synthetic_controls(B, Nt, nu=2, seed=0) -> np.ndarray:
    rng = np.random.default_rng(seed + 1)
    return rng.uniform(-1.0, 1.0, size=(B, nu, Nt))


CONFIGS = {
    # name: (problem builder, controls builder, B per GPU)
    "zz_plumbing": (lambda: zz_problem(100), lambda B, s=0: zz_controls(B, 100, 10.0, s), 1),
    "zz_batch": (lambda: zz_problem(500), lambda B, s=0: zz_controls(B, 500, 20.0, s), 512),
    "cavity": (lambda: cavity_problem(20, 1000), lambda B, s=0: cavity_controls(B, 1000, s), 256),
    "cavity_dense": (lambda: cavity_dense_problem(20, 1000), lambda B, s=0: cavity_controls(B, 1000, s), 256),
    "tunable_bus": (lambda: tunable_bus_problem(2000), lambda B, s=0: tunable_bus_controls(B, 2000, s), 512),
    "synthetic": (lambda: synthetic_problem(256, 1000), lambda B, s=0: synthetic_controls(B, 1000, 2, s), 128),
}
