"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle on identical inputs.

Tolerances (fp64 GPU vs fp64 restatement): |ΔJ| <= 1e-12 and
||ΔdJdu||_F / ||dJdu||_F <= 1e-10 per seed; fp32: |ΔJ| <= 1e-4, rel 1e-3.
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


def _engine(prob, B, precision="fp64"):
    from qoc_amd import GrapeEngine
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B, precision=precision)
    e.set_cost_trace(prob.x_target, prob.n)
    return e


def _check(prob, u, order=3, precision="fp64", penalty=None):
    B = u.shape[0]
    e = _engine(prob, B, precision)
    if penalty is not None:
        e.set_state_penalty(*penalty)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, order)
    tolJ, tolg = (1e-12, 1e-10) if precision == "fp64" else (1e-4, 1e-3)
    for b in range(B):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=order,
                                 penalty=penalty)
        assert abs(J[b] - Jr) <= tolJ, (b, J[b], Jr)
        rel = np.linalg.norm(g[b] - gr) / max(np.linalg.norm(gr), 1e-300)
        assert rel <= tolg, (b, rel)
    e.close()


def test_expm_matches_oracle_all_degrees(built_lib):
    from qoc_amd import expm, systems
    rng = np.random.default_rng(1)
    for N in (3, 9, 16, 17, 27, 40):
        As, want_deg = [], []
        for sc in (0.005, 0.1, 0.5, 1.5, 4.0, 30.0):
            H = systems._gue(rng, N)
            As.append(-1j * H * sc / np.abs(H).sum(0).max())
        X, deg, sq = expm(np.stack(As), return_degrees=True)
        for a, x, d, s in zip(As, X, deg, sq):
            Xr, dr, sr = O.expm_higham2005(a)
            assert (d, s) == (dr, sr)
            assert np.abs(x - Xr).max() < 1e-13, (N, d, s, np.abs(x - Xr).max())


def test_expm_general_matrix(built_lib):
    from qoc_amd import expm
    rng = np.random.default_rng(2)
    A = rng.standard_normal((4, 11, 11)) * 0.3 + 1j * rng.standard_normal((4, 11, 11)) * 0.3
    X = expm(A)
    for a, x in zip(A, X):
        Xr, _, _ = O.expm_higham2005(a)
        assert np.abs(x - Xr).max() < 1e-12


def test_cavity_small_parity(built_lib):
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=6, Nt=30)
    _check(prob, systems.cavity_controls(3, prob.Nt, seed=0))


def test_zz_parity(built_lib):
    from qoc_amd import systems
    prob = systems.zz_problem(100)
    _check(prob, systems.zz_controls(2, 100, 10.0, seed=0))


def test_cavity40_parity(built_lib):
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=20, Nt=40)
    _check(prob, systems.cavity_controls(2, prob.Nt, seed=5))


def test_tunable_bus_parity(built_lib):
    from qoc_amd import systems
    prob = systems.tunable_bus_problem(Nt=60, tgate=350.0 * 60 / 2000)
    _check(prob, systems.tunable_bus_controls(2, prob.Nt, seed=0))


@pytest.mark.parametrize("order", [1, 2, 3, 4])
def test_orders(built_lib, order):
    from qoc_amd import systems
    prob = systems.zz_problem(50, tgate=5.0)
    _check(prob, systems.zz_controls(2, 50, 5.0, seed=order), order=order)


def test_state_penalty(built_lib):
    from qoc_amd import systems
    prob = systems.zz_problem(40, tgate=4.0)
    qb = systems.QuantumBasis([3, 3])
    pen = (qb(["20", "21", "22"]), [0, 1, 2, 3], 0.37)
    _check(prob, systems.zz_controls(2, 40, 4.0, seed=9), penalty=pen)
