"""The CPU oracle pinned against the reference's own known answers and tolerance contracts.

The reference is Julia (not runnable here); its tests hold no golden arrays, only the values
and thresholds restated below with their file:line.  Tolerances follow Julia's `≈`
(rtol = sqrt(eps)) unless the reference states one.
"""
import math

import numpy as np
import pytest
import scipy.linalg as sl

import qoc_oracle as O
from qoc_amd import systems as S

RTOL = math.sqrt(np.finfo(float).eps)  # Julia isapprox default


def approx(a, b, atol=0.0, rtol=RTOL):
    return abs(a - b) <= max(atol, rtol * max(abs(a), abs(b)))


def Jtheta(m, th):
    """test/test_fidelities.jl:3 (J of both phases)."""
    return abs(m[0] + m[1] * np.exp(1j * th[0]) + m[2] * np.exp(1j * th[1]) + m[3] * np.exp(1j * (th[0] + th[1])))


# ---------------------------------------------------------------------------
# test/test_fidelities.jl
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("m,opt,basic,grid,grid_atol", [
    ([1, 1j, 1j, 1], 2.8284271, 2.0, 2.8284271, 0.0),                       # :17-24
    ([1, 0.1j, 0.1j, 1], 2.0099751, 0.2, 2.0099751, 0.0),                   # :28-35
    (list(np.exp(1j * np.array([1, 2, 3, 4]))), 4.0, 4.0, 4.0, 1e-3),       # :39-46
    (list(np.exp(1j * np.array([1, 2, -2.5, -1.7]))), 3.995001, None, 3.995001, 1e-3),  # :51-56
])
def test_known_answers(m, opt, basic, grid, grid_atol):
    assert approx(O.abs_sum_phase_calibrated(m), opt)
    if basic is not None:
        assert approx(O.abs_sum_phase_calibrated(m, "basic"), basic)
    assert approx(O.abs_sum_phase_calibrated(m, "grid"), grid, atol=grid_atol)
    th = O.optimal_calibration(m)[1]
    assert abs(Jtheta(m, th) - O.abs_sum_phase_calibrated(m)) <= 1e-8   # :25, :59 (atol 1e-12 / 1e-8)


def test_basic_atol_and_theta_opt():
    m = np.exp(1j * np.array([1, 2, -2.5, -1.7]))
    assert approx(O.abs_sum_phase_calibrated(m, "basic"), 3.995001, atol=0.01)  # :54
    th = O.optimal_calibration(m)[1]
    assert np.allclose(th, [5.383258515112539, 3.6000220820575084], atol=1e-4, rtol=0)  # :61


def test_known_answers_exact_values():
    m = np.exp(1j * np.array([2.5, 2.5, 1.5, -2.5]))                   # :66-74
    J, th = O.optimal_calibration(m)
    assert approx(J, 3.365883939061934)
    assert approx(Jtheta(m, th), 3.365883939061934)
    assert approx(O.abs_sum_phase_calibrated(m), 3.365883939061934)
    m = [0.65 - 0.75j, -0.4 + 0.8j, -0.4 + 0.1j, 0.7 - 0.0j]            # :78-84
    assert approx(O.abs_sum_phase_calibrated(m), 2.9787244710195484)
    J, th = O.optimal_calibration(m, 1e-15)
    assert approx(J, 2.9787244710195484)
    assert approx(Jtheta(m, th), 2.9787244710195484)


def test_unmatched_calibration_returns_none():
    assert O.abs_sum_phase_calibrated([1, 1, 1, 1], "lms_phase_semiold") is None   # :44 returns `nothing`


def test_optimal_beats_grid():
    """test/test_fidelities.jl:106-119 (500 random draws, numpy-seeded)."""
    rng = np.random.default_rng(0)
    for _ in range(500):
        m = rng.random(4) * np.exp(2j * np.pi * rng.random(4))
        Fo = 1 - O.abs_sum_phase_calibrated(m, "optimal") / 4
        Fg = 1 - O.abs_sum_phase_calibrated(m, "grid") / 4
        assert Fg - Fo > -np.finfo(float).eps
        assert Fg - Fo < 1e-3


def test_fd_gradient_of_F2():
    """test/test_fidelities.jl:130-148: analytic gradient of F^2 vs central differences, rtol 1e-6."""
    rng = np.random.default_rng(100)
    h = 1e-6
    for _ in range(200):
        m = rng.random(4) * np.exp(2j * np.pi * rng.random(4))
        F, th = O.optimal_calibration(m, 1e-12)
        assert abs(Jtheta(m, O.optimal_calibration(m, 1e-12)[1]) - F) < 1e-10
        g = O.abs_sum_phase_calibrated_grad(m, th[0])
        fd = np.zeros(4, dtype=complex)
        f = lambda mm: O.optimal_calibration(mm, 1e-13)[0] ** 2  # noqa: E731
        for k in range(4):
            for part, unit in ((0, 1.0), (1, 1j)):
                e = np.zeros(4, dtype=complex)
                e[k] = unit * h
                d = (f(m + e) - f(m - e)) / (2 * h)
                fd[k] += d if part == 0 else 1j * d
        assert np.allclose(g, fd, rtol=1e-6, atol=1e-7)


# ---------------------------------------------------------------------------
# exponential! (third-party ExpMethodHigham2005) — no reference test pins it; scipy does.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("N", [1, 3, 9, 27, 40])
def test_expm_vs_scipy_all_degrees(N):
    rng = np.random.default_rng(N)
    seen = set()
    for sc in (0.0, 0.01, 0.1, 0.5, 1.5, 4.0, 30.0, 200.0):
        H = S._gue(rng, N)
        A = -1j * H * (sc / max(np.abs(H).sum(0).max(), 1e-300))
        X, d, s = O.expm_higham2005(A)
        seen.add(d)
        assert np.abs(X - sl.expm(A)).max() <= 1e-13 * max(1.0, np.abs(X).max()) * (1 + s)
        assert np.abs(X.conj().T @ X - np.eye(N)).max() < 1e-12 * (1 + s)  # unitary
    assert seen >= {3, 5, 7, 9, 13}


def test_expm_general_matrix():
    rng = np.random.default_rng(3)
    A = rng.standard_normal((12, 12)) * 0.4 + 1j * rng.standard_normal((12, 12)) * 0.4
    X, _, _ = O.expm_higham2005(A)
    assert np.abs(X - sl.expm(A)).max() < 1e-12 * np.abs(X).max()


def test_pade_degree_thresholds():
    assert O.pade_degree(0.0) == (3, 0)
    assert O.pade_degree(0.015) == (3, 0) and O.pade_degree(0.0150001) == (5, 0)
    assert O.pade_degree(0.25) == (5, 0) and O.pade_degree(0.2500001) == (7, 0)
    assert O.pade_degree(0.95) == (7, 0) and O.pade_degree(0.9500001) == (9, 0)
    assert O.pade_degree(2.1) == (9, 0) and O.pade_degree(2.1000001) == (13, 0)
    assert O.pade_degree(5.4) == (13, 0) and O.pade_degree(5.41) == (13, 1)
    assert O.pade_degree(30.0) == (13, 3)


# ---------------------------------------------------------------------------
# expm_jacobian! finite-difference contract (test/test_expm_jacobian.jl:13-35)
# ---------------------------------------------------------------------------
def _fd_jac(A0, A, u, dt, h=1e-6):
    cols = []
    for j in range(len(u)):
        up, um = u.copy(), u.copy()
        up[j] += h
        um[j] -= h
        Fp = sl.expm(dt * (A0 + sum(up[k] * A[k] for k in range(len(A)))))
        Fm = sl.expm(dt * (A0 + sum(um[k] * A[k] for k in range(len(A)))))
        cols.append(((Fp - Fm) / (2 * h)).ravel(order="F"))
    return np.stack(cols, 1)


def _jac_err(seed, order, dt):
    rng = np.random.default_rng(seed)
    A0, A1, A2 = [0.05 * rng.standard_normal((3, 3)) for _ in range(3)]
    u = np.array([1.0, 2.0])
    d = O.expm_jacobian(A0, [A1, A2], u, order, dt)
    return np.linalg.norm(np.stack([x.ravel(order="F") for x in d], 1) - _fd_jac(A0, [A1, A2], u, dt))


@pytest.mark.parametrize("order,dt,thr", [(3, 1.0, 4e-4), (4, 1.0, 3e-5), (3, 0.25, 2e-6), (4, 0.25, 3e-8)])
def test_expm_jacobian_fd_thresholds(order, dt, thr):
    # The reference thresholds were set on Julia's Random.seed!(0) draw; numpy seed 0 is used here
    # (the Julia RNG stream cannot be reproduced).  Draw-independent checks follow below.
    assert _jac_err(0, order, dt) < thr


def test_expm_jacobian_truncation_scaling():
    for seed in range(10):
        e3, e4 = _jac_err(seed, 3, 1.0), _jac_err(seed, 4, 1.0)
        e3s, e4s = _jac_err(seed, 3, 0.25), _jac_err(seed, 4, 0.25)
        assert e4 < e3 and e4s < e3s
        assert e3s < e3 / 30 and e4s < e4 / 100  # O(dt^4) and O(dt^5) truncation


def test_expm_jacobian_order1_is_dtA():
    rng = np.random.default_rng(1)
    A = [rng.standard_normal((4, 4)) for _ in range(3)]
    d = O.expm_jacobian(A[0], A[1:], [0.3, -0.2], order=1, dt=0.5)
    assert np.array_equal(d[0], 0.5 * A[1]) and np.array_equal(d[1], 0.5 * A[2])


# ---------------------------------------------------------------------------
# Costs (test/test_penalty_fcns.jl) — Wirtinger convention: grad = dJ/dRe x + i dJ/dIm x
# ---------------------------------------------------------------------------
def _wirtinger_fd(f, x, h=1e-6):
    g = np.zeros_like(x, dtype=complex)
    for idx in np.ndindex(x.shape):
        for unit, part in ((1.0, 1.0), (1j, 1j)):
            e = np.zeros_like(x, dtype=complex)
            e[idx] = unit * h
            g[idx] += part * (f(x + e) - f(x - e)) / (2 * h)
    return g


def test_state_penalty_matches_reference_formula():
    inds_css, inds_pen = [0, 1, 4, 5], [6, 7, 8]    # 1-based [1,2,5,6], [7,8,9] at :3-4
    L, dL = O.setup_state_penalty(inds_pen, inds_css, 0.22)
    x0 = np.arange(1.0, 82.0).reshape(9, 9, order="F")
    assert L(x0) == 0.22 * np.linalg.norm(x0[np.ix_(inds_pen, inds_css)]) ** 2       # :9
    assert np.allclose(dL(x0), _wirtinger_fd(lambda x: L(x), x0.astype(complex)), rtol=1e-8, atol=1e-5)


def test_infidelity_gradient():
    rng = np.random.default_rng(4)
    Q, _ = np.linalg.qr(rng.standard_normal((9, 8)) + 1j * rng.standard_normal((9, 8)))
    xt = Q[:, :4]
    x = rng.standard_normal((9, 4)) + 1j * rng.standard_normal((9, 4))
    J, dJ = O.setup_infidelity(xt)
    assert np.allclose(dJ(x), _wirtinger_fd(J, x), rtol=1e-6, atol=1e-8)
    Jz, dJz = O.setup_infidelity_zcalibrated(xt)
    assert np.allclose(dJz(x), _wirtinger_fd(Jz, x, 1e-7), rtol=1e-5, atol=1e-7)
    with pytest.raises(ValueError):
        O.setup_infidelity_zcalibrated(Q[:, :3])


# ---------------------------------------------------------------------------
# Forward known answer: examples/cavity_qubit.jl:80-81 (|<target|x_551>| ≈ 0.999979)
# ---------------------------------------------------------------------------
def test_cavity_known_answer(golden_dir):
    iq = np.load(golden_dir / "cavity_qubit_pulse_marina.npy") * 1e-9
    H0, Tc, theta = S.cavity_model(12)
    A0, A1, A2 = S.setup_bilinear_matrices(H0, Tc / 2, 1.0)
    x0 = np.kron([1, 0], np.ones(12) / np.sqrt(12))[:, None]
    x = O.propagate(A0, [A1, A2], iq.T, x0)
    tgt = np.kron([1, 0], np.exp(1j * theta))
    tgt /= np.linalg.norm(tgt)
    assert abs(abs(np.vdot(x[-1][:, 0], tgt)) - 0.999979) < 1e-6


# ---------------------------------------------------------------------------
# GRAPE gradient: order 4 vs finite differences of the exact propagation
# (test/test_gradient_computation.jl:90-99 displays this comparison; asserted here)
# ---------------------------------------------------------------------------
def test_grape_gradient_vs_fd():
    prob = S.zz_problem(20, tgate=1.0)
    u = S.zz_controls(1, 20, 1.0, seed=5)[0]
    Jf, dJf = O.setup_infidelity(prob.x_target, prob.n)
    cache = O.setup_grape_cache(prob.A0, prob.x0, u.shape)
    O.propagate(prob.A0, prob.A, u, prob.x0, cache)
    g = O.grape_sensitivity(prob.A0, prob.A, dJf, cache.u, prob.x0, cache, dUkdp_order=4).copy()
    h = 1e-6
    fd = np.zeros_like(u)
    for j in range(u.shape[0]):
        for k in range(u.shape[1]):
            up, um = u.copy(), u.copy()
            up[j, k] += h
            um[j, k] -= h
            fd[j, k] = (Jf(O.propagate(prob.A0, prob.A, up, prob.x0)[-1]) -
                        Jf(O.propagate(prob.A0, prob.A, um, prob.x0)[-1])) / (2 * h)
    assert np.linalg.norm(g - fd) / np.linalg.norm(fd) < 1e-4


def test_stale_cache_raises():
    prob = S.zz_problem(10, tgate=1.0)
    u = S.zz_controls(1, 10, 1.0, seed=1)[0]
    Jf, dJf = O.setup_infidelity(prob.x_target, prob.n)
    cache = O.setup_grape_cache(prob.A0, prob.x0, u.shape)
    O.propagate(prob.A0, prob.A, u, prob.x0, cache)
    with pytest.raises(ValueError, match="Cache data from other control signal u"):
        O.grape_sensitivity(prob.A0, prob.A, dJf, u + 1e-3, prob.x0, cache)
    with pytest.raises(ValueError, match="incompatiable dimensions"):
        O.setup_grape_cache(prob.A0, np.ones((4, 2)), u.shape)


# ---------------------------------------------------------------------------
# Oracle self-consistency: golden fixtures and the C restatement
# ---------------------------------------------------------------------------
def test_golden_fixtures_reproduce(golden_dir):
    g = np.load(golden_dir / "golden_evals.npz")
    cases = {"zz": S.zz_problem(60, tgate=6.0), "cavity": S.cavity_problem(N_cavity=8, Nt=40),
             "bus": S.tunable_bus_problem(Nt=40, tgate=7.0)}
    for key, prob in cases.items():
        u = g[f"{key}_u"]
        J, d, _ = O.grape_eval(prob.A0, prob.A, u[0], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J - g[f"{key}_J_o3"][0]) < 1e-13
        assert np.abs(d - g[f"{key}_dJdu_o3"][0]).max() < 1e-12 * max(1, np.abs(d).max())


def test_c_restatement_matches_numpy():
    import cpuref
    for prob, u in ((S.cavity_problem(N_cavity=6, Nt=25), S.cavity_controls(3, 25, seed=2)),
                    (S.tunable_bus_problem(Nt=20, tgate=3.5), S.tunable_bus_controls(2, 20, seed=3))):
        J, g = cpuref.grape_eval_batch(prob, u)
        for b in range(u.shape[0]):
            Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n)
            assert abs(J[b] - Jr) < 1e-13
            assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) < 1e-12
    rng = np.random.default_rng(8)
    for sc in (0.01, 0.3, 1.2, 4.0, 40.0):
        H = S._gue(rng, 11)
        A = -1j * H * sc / np.abs(H).sum(0).max()
        X, d, s = cpuref.expm(A)
        Xr, dr, sr = O.expm_higham2005(A)
        assert (d, s) == (dr, sr) and np.abs(X - Xr).max() < 1e-13 * (1 + s)


# ---- exact (Fréchet) gradient mode, SURVEY.md §8f item 2 ------------------------------------
def test_frechet_block_matches_scipy_expm_frechet():
    from scipy.linalg import expm_frechet
    rng = np.random.default_rng(11)
    for n, sc in ((4, 0.1), (9, 1.0), (7, 6.0)):
        H = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        A = -1j * sc * (H + H.conj().T) / 2 / n
        E = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        X, L = O.expm_frechet_block(A, E)
        Xs, Ls = expm_frechet(A, E)
        assert np.abs(X - Xs).max() < 1e-13
        assert np.abs(L - Ls).max() / np.abs(Ls).max() < 1e-12


def test_exact_gradient_matches_finite_differences_and_adjoint_identity():
    prob = S.zz_problem(12, tgate=3.0)
    rng = np.random.default_rng(4)
    u = rng.uniform(-1.5, 1.5, size=(2, prob.Nt))
    J, g, cache = O.grape_eval(prob.A0, prob.A, u, prob.x0, prob.x_target, prob.n, order="exact")
    eps = 1e-6
    for (j, k) in ((0, 0), (1, 5), (0, 11)):
        up, um = u.copy(), u.copy()
        up[j, k] += eps
        um[j, k] -= eps
        fd = (O.grape_eval(prob.A0, prob.A, up, prob.x0, prob.x_target, prob.n)[0] -
              O.grape_eval(prob.A0, prob.A, um, prob.x0, prob.x_target, prob.n)[0]) / (2 * eps)
        assert abs(g[j, k] - fd) <= 1e-7 * max(1.0, abs(fd)), (j, k, g[j, k], fd)
    # one Fréchet derivative per slice: Re tr(A_j L(A_k, x_k lam_{k+1}^H)) == Re<lam, L(A_k, A_j) x_k>
    k = 4
    Ak = prob.A0 + sum(u[j, k] * prob.A[j] for j in range(2))
    Z = cache.x[k] @ cache.lam[k + 1].conj().T
    _, Lz = O.expm_frechet_block(Ak, Z)
    for j in range(2):
        assert abs(np.real(np.trace(prob.A[j] @ Lz)) - g[j, k]) < 1e-12


# ---- ODE path (fixed-step Tsit5), SURVEY.md §8f item 3 ----------------------------------------
def test_tsit5_tunable_bus_known_answer():
    """examples/two_qubit_tunable_bus.jl:58-67: |<200|x(350)>|^2 'should be something like 0.937218'."""
    H0, Hc, qb = S.tunable_bus_model()
    x0 = qb.columns(["110"])[:, 0].astype(complex)
    xt = qb.columns(["200"])[:, 0].astype(complex)
    i1, i2 = int(np.argmax(np.abs(x0))), int(np.argmax(np.abs(xt)))
    w_phi = abs(H0[i1, i1] - H0[i2, i2]) + (-0.002) * 2 * math.pi
    p0 = [300.0, 50.0, 0.25, w_phi, 0.13]
    x = O.propagate_envelope(-1j * H0, [-1j * Hc], O.tunable_bus_envelope, p0, x0, 350.0, 1e-3)
    assert abs(abs(np.vdot(x, xt)) ** 2 - 0.937218) < 5e-7


def test_tsit5_order_and_pwc_ode_matches_expm_path():
    # 5th order: halving the step reduces the error by ~32
    rng = np.random.default_rng(3)
    H = rng.standard_normal((6, 6)) + 1j * rng.standard_normal((6, 6))
    A = -1j * (H + H.conj().T) / 4
    x0 = rng.standard_normal(6) + 1j * rng.standard_normal(6)
    ex = sl.expm(A) @ x0
    e1 = np.abs(O.tsit5_fixed(lambda y, t: A @ y, x0, 0.0, 1 / 8, 8) - ex).max()
    e2 = np.abs(O.tsit5_fixed(lambda y, t: A @ y, x0, 0.0, 1 / 16, 16) - ex).max()
    assert 20 < e1 / e2 < 50
    # PWC ODE gradient (nsub = 10) agrees with the expm path to the integrator's accuracy
    prob = S.zz_problem(30, tgate=3.0)
    u = S.zz_controls(1, 30, 3.0, seed=2)[0]
    J1, g1, _ = O.grape_eval(prob.A0, prob.A, u, prob.x0, prob.x_target, prob.n, order=3)
    J2, g2 = O.grape_eval_ode(prob.A0, prob.A, u, prob.x0, prob.x_target, prob.n, order=3, nsub=10)
    assert abs(J1 - J2) < 1e-9
    assert np.linalg.norm(g1 - g2) / np.linalg.norm(g1) < 1e-7


def test_zcal_gradient_match_recovers_a_phase_shift():
    """qoc_oracle.zcal_gradient_match (the z-cal GPU check): a gradient taken at a calibration phase 3e-9 away
    from the golden-section optimum is recognised (Δθ recovered, residual at rounding level)."""
    from qoc_amd import systems
    prob = systems.tunable_bus_cz_problem(Nt=20, tgate=3.5)
    u = systems.tunable_bus_controls(1, 20, seed=3)[0]
    g = O.grape_eval(prob.A0, prob.A, u, prob.x0, prob.x_target, order=3,
                     cost=O.setup_infidelity_zcalibrated_shifted(prob.x_target, 3e-9))[1]
    res, dth = O.zcal_gradient_match(g, prob.A0, prob.A, u, prob.x0, prob.x_target, order=3)
    assert res < 1e-12 and abs(dth - 3e-9) < 1e-12, (res, dth)
    g0 = O.grape_eval(prob.A0, prob.A, u, prob.x0, prob.x_target, order=3,
                      cost=O.setup_infidelity_zcalibrated(prob.x_target))[1]
    assert np.linalg.norm(g - g0) / np.linalg.norm(g0) > 1e-10  # the shift is visible at the 1e-10 bar


def test_zcal_dtheta_bound_covers_the_golden_section():
    """qoc_oracle.zcal_dtheta_bound (the z-cal GPU tests' |Δθ| bar): the golden-section phase lies within half the
    bound of the true maximiser (Newton on the analytic dJ/dθ), on random overlaps and on the zz test cases."""
    rng = np.random.default_rng(5)
    cases = [rng.standard_normal(4) + 1j * rng.standard_normal(4) for _ in range(200)]
    cases = [c / np.abs(c).max() for c in cases]
    for m in cases:
        F, th = O.optimal_calibration(m)
        t = th[0]

        def d(t, k):  # k-th derivative of |m0 + m1 e^{it}| + |m2 + m3 e^{it}| by central differences of dJ
            def J1(t):
                s = 0.0
                for a, b in ((m[0], m[1]), (m[2], m[3])):
                    v = a + b * np.exp(1j * t)
                    s += (np.conj(v) * 1j * b * np.exp(1j * t)).real / abs(v)
                return s
            return J1(t) if k == 1 else (J1(t + 1e-6) - J1(t - 1e-6)) / 2e-6
        for _ in range(6):
            t -= d(t, 1) / d(t, 2)
        X = np.eye(4, dtype=complex)
        bound = O.zcal_dtheta_bound(X, np.diag(m))
        dd = abs((th[0] - t + np.pi) % (2 * np.pi) - np.pi)
        assert dd <= bound / 2, (m, dd, bound)


def test_oracle_reproduces_zz_pulse_fixture(golden_dir):
    """tests/golden/zz_pulse_fixture.npz (examples/zz_coupling_simulation.jl's forward run) is the oracle's output."""
    from qoc_amd import systems
    fx = np.load(golden_dir / "zz_pulse_fixture.npz")
    prob = systems.zz_problem(500)
    iq = np.load(golden_dir / "zz_coupling_pulse_tahereh210823.npy") * 1e-9
    assert np.array_equal(np.ascontiguousarray(iq.T), fx["u"])
    xs = O.propagate(prob.A0, prob.A, fx["u"], prob.x0)
    assert np.abs(xs[-1] - fx["x_final"]).max() <= 1e-14
    # unitary propagation of an orthonormal x0
    assert np.abs(fx["x_final"].conj().T @ fx["x_final"] - np.eye(4)).max() <= 1e-13
