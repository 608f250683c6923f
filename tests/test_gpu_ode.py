"""GPU parity of the ODE path against the CPU oracle.

* PWC Tsit5 (qoc_set_propagation(QOC_PROP_TSIT5)): the reference's propagate_pwc /
  compute_pwc_gradient (src/gradient_computations.jl:108-169) with nsub fixed steps per slice;
  oracle = qoc_oracle.grape_eval_ode (pinned by test_oracle.py: 5th-order convergence and agreement
  with the expm path).  fp64: |ΔJ| <= 1e-12, rel ||ΔdJdu|| <= 1e-10; fp32: 1e-4 / 1e-3.
* Continuous envelopes (qoc_propagate_envelope): the tunable-bus example's known answer
  |<200|x(350)>|^2 = 0.937218 (examples/two_qubit_tunable_bus.jl:58-67, dt = 1e-3) and DRAG /
  sine-basis pulses (src/parameterized_pulses.jl) vs qoc_oracle.propagate_envelope.
"""
import math

import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


def _problem(which):
    from qoc_amd import systems as S
    if which == "zz":
        prob = S.zz_problem(20, tgate=2.0)
        u = S.zz_controls(3, 20, 2.0, seed=5)
    elif which == "cavity":
        prob = S.cavity_problem(N_cavity=6, Nt=16)
        u = S.cavity_controls(2, prob.Nt, seed=2)
    else:
        prob = S.tunable_bus_problem(12, tgate=350.0 * 12 / 2000)
        u = S.tunable_bus_controls(2, 12, seed=1)
    return prob, u


def _engine(prob, B, precision="fp64", nsub=10):
    from qoc_amd import GrapeEngine
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B, precision=precision)
    e.set_propagation("tsit5", nsub)
    e.set_cost_trace(prob.x_target, prob.n)
    return e


@pytest.mark.parametrize("which", ["zz", "cavity", "tunable_bus"])
def test_pwc_tsit5_matches_oracle(built_lib, which):
    prob, u = _problem(which)
    # tunable bus: ||A_k||_1 ~ 25-35 per slice (lab-frame energies), so nsub = 10 leaves Tsit5's
    # stability region (h ||A|| ~ 3) and both sides blow up identically; 40 steps keep h ||A|| < 1
    nsub = 40 if which == "tunable_bus" else 10
    e = _engine(prob, u.shape[0], nsub=nsub)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    for b in range(u.shape[0]):
        Jr, gr = O.grape_eval_ode(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, nsub=nsub)
        assert abs(J[b] - Jr) <= 1e-12, (b, J[b], Jr)
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10
    xs = O.propagate_pwc_ode(prob.A0, prob.A, u[0], prob.x0, nsub=nsub)
    for k in (1, prob.Nt // 2, prob.Nt):
        assert np.abs(e.state(k, seed=0) - xs[k]).max() < 1e-13
    e.close()


def test_pwc_tsit5_penalty_orders_nsub_and_fp32(built_lib):
    from qoc_amd import QOCError
    prob, u = _problem("cavity")
    pen = (list(range(prob.A0.shape[0] - 3, prob.A0.shape[0])), list(range(prob.x0.shape[1])), 0.4)
    for order, nsub in ((1, 4), (2, 7), (4, 10)):
        e = _engine(prob, u.shape[0], nsub=nsub)
        e.set_state_penalty(*pen)
        J = e.propagate(u)
        g = e.grape_sensitivity(u, order)
        for b in range(u.shape[0]):
            Jr, gr = O.grape_eval_ode(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=order,
                                      nsub=nsub, penalty=pen)
            assert abs(J[b] - Jr) <= 1e-12
            assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10
        with pytest.raises(QOCError):
            e.propagator(0)  # no propagators are formed on the ODE path
        e.close()
    e = _engine(prob, u.shape[0], precision="fp32")
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    for b in range(u.shape[0]):
        Jr, gr = O.grape_eval_ode(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, nsub=10)
        assert abs(J[b] - Jr) <= 1e-4
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-3
    e.close()


def test_pwc_tsit5_switch_back_to_expm(built_lib):
    prob, u = _problem("zz")
    e = _engine(prob, u.shape[0])
    J_ode = e.propagate(u)
    e.set_propagation("expm")
    J_exp = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    for b in range(u.shape[0]):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J_exp[b] - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10
        assert abs(J_ode[b] - J_exp[b]) < 1e-9  # nsub = 10 Tsit5 vs exp at these step sizes
    e.close()


def test_reference_shaped_propagate_pwc_and_gradient(built_lib):
    """Q.propagate_pwc / Q.compute_pwc_gradient called like the reference (physical generators, Δt,
    dt = 0.1Δt, dJfinal_dx closure) == oracle on the Δt-prescaled problem."""
    import qoc_amd as Q
    from qoc_amd import systems as S
    Δt = 0.1
    prob = S.zz_problem(20, tgate=2.0)
    A0 = prob.A0 / Δt
    A = [a / Δt for a in prob.A]
    u = S.zz_controls(1, 20, 2.0, seed=7)[0]
    cache = Q.setup_grape_cache(A0, prob.x0, u.shape)
    x = Q.propagate_pwc(A0, A, prob.x0, u, Δt, cache)
    _, dJf = Q.setup_infidelity(prob.x_target, prob.n)
    g = Q.compute_pwc_gradient(dJf, u, Δt, A0, A, cache, dUkdp_order=2)
    _, gr = O.grape_eval_ode(prob.A0, prob.A, u, prob.x0, prob.x_target, prob.n, order=2, nsub=10)
    xs = O.propagate_pwc_ode(prob.A0, prob.A, u, prob.x0, nsub=10)
    assert np.abs(x[-1] - xs[-1]).max() < 1e-12
    assert np.linalg.norm(g - gr) / np.linalg.norm(gr) <= 1e-10
    with pytest.raises(Q.StaleCacheError):
        Q.compute_pwc_gradient(dJf, u + 0.01, Δt, A0, A, cache)
    with pytest.raises(ValueError):
        Q.propagate_pwc(A0, A, prob.x0, u, Δt, cache, dt=0.03)


def test_reference_call_form_with_rhs_closures_and_real_layout(built_lib):
    """test/test_gradient_computation.jl:44-51 and examples/zz_coupling_ipopt_diffeq.jl:34-52, as written there:
    cache = setup_grape_cache(A0, c2r(x0), (2, Nt)); sol = propagate_pwc(dxdt, c2r(x0), u, Δt, cache; dt);
    compute_pwc_gradient(dλdt, dJfinal_dx, u, Δt, A0, [A1, A2], cache; dUkdp_order=3, dt), with dxdt / dλdt the
    right-hand-side closures of examples/models/setup_diffeq_rhs.jl in the complex2real layout.  Against the
    oracle on the same problem; states come back in the real layout (cache[0] is the reference's cache[1])."""
    import qoc_amd as Q
    from qoc_amd import systems as S
    Δt = 0.1
    prob = S.zz_problem(20, tgate=2.0)
    A0 = prob.A0 / Δt
    A = [a / Δt for a in prob.A]
    u = S.zz_controls(1, 20, 2.0, seed=8)[0]

    def dxdt(dx, x, p, t):
        dx[:] = Q.c2r((A0 + p[0] * A[0] + p[1] * A[1]) @ Q.r2c(x))

    def dldt(dl, l, p, t):
        dl[:] = Q.c2r(-(A0 + p[0] * A[0] + p[1] * A[1]).conj().T @ Q.r2c(l))
    x0r = Q.c2r(prob.x0)
    cache = Q.setup_grape_cache(A0, x0r, u.shape)
    sol = Q.propagate_pwc(dxdt, x0r, u, Δt, cache, dt=0.2 * Δt)
    _, dJf = Q.setup_infidelity(prob.x_target, prob.n)
    g = Q.compute_pwc_gradient(dldt, dJf, u, Δt, A0, A, cache, dUkdp_order=3, dt=0.2 * Δt)
    _, gr = O.grape_eval_ode(prob.A0, prob.A, u, prob.x0, prob.x_target, prob.n, order=3, nsub=5)
    xs = O.propagate_pwc_ode(prob.A0, prob.A, u, prob.x0, nsub=5)
    assert sol.u[-1].shape == x0r.shape and not np.iscomplexobj(sol.u[-1])
    assert np.abs(Q.r2c(sol.u[-1]) - xs[-1]).max() < 1e-12
    assert np.abs(Q.r2c(cache[0][7]) - xs[7]).max() < 1e-12
    assert np.linalg.norm(g - gr) / np.linalg.norm(gr) <= 1e-10
    def wrong(dl, l, p, t):  # +A(u)^H: the adjoint equation with the sign flipped (for skew-Hermitian
        dl[:] = Q.c2r((A0 + p[0] * A[0] + p[1] * A[1]).conj().T @ Q.r2c(l))  # generators dxdt itself is right)
    with pytest.raises(ValueError, match="adjoint"):
        Q.compute_pwc_gradient(wrong, dJf, u, Δt, A0, A, cache, dUkdp_order=3, dt=0.2 * Δt)
    with pytest.raises(ValueError, match="incompatiable"):  # real x0 must have 2N rows (:84-87)
        Q.setup_grape_cache(A0, np.ones((prob.N, 4)), u.shape)


def test_tsit5_unsupported_configurations(built_lib, monkeypatch):
    from qoc_amd import GrapeEngine, QOCError, systems
    prob = systems.zz_problem(10)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=1)
    with pytest.raises(QOCError):
        e.set_propagation("tsit5", 0)
    e.set_propagation("tsit5", 5)
    e.set_cost_zcalibrated(prob.x_target)  # supported on every path (test_gpu_parity.test_zcalibrated_cost)
    e.close()
    monkeypatch.setenv("QOC_FORCE_LARGE_N", "1")
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=1)
    with pytest.raises(QOCError):
        e.set_propagation("tsit5", 10)
    e.close()


def _tunable_bus_setup():
    from qoc_amd import systems as S
    H0, Hc, qb = S.tunable_bus_model()
    x0 = qb.columns(["110"])[:, 0].astype(complex)
    xt = qb.columns(["200"])[:, 0].astype(complex)
    i1, i2 = int(np.argmax(np.abs(x0))), int(np.argmax(np.abs(xt)))
    w_phi = abs(H0[i1, i1] - H0[i2, i2]) + (-0.002) * 2 * math.pi
    return H0, Hc, x0, xt, w_phi


def test_envelope_tunable_bus_known_answer(built_lib):
    """examples/two_qubit_tunable_bus.jl:58-67 — 'should be something like 0.937218'."""
    from qoc_amd import GrapeEngine
    H0, Hc, x0, xt, w_phi = _tunable_bus_setup()
    p0 = [300.0, 50.0, 0.25, w_phi, 0.13]
    e = GrapeEngine(-1j * H0, [-1j * Hc], x0, 1, B=1)
    e.set_cost_trace(xt, 1)
    J, x = e.propagate_envelope("tunable_bus", np.array([p0]), 350.0, 1e-3)
    pop = abs(np.vdot(xt, x[0][:, 0])) ** 2
    assert abs(pop - 0.937218) < 5e-7, pop
    assert abs((1 - J[0]) - pop) < 1e-12
    e.close()


def test_envelope_tunable_bus_batch_matches_oracle(built_lib):
    from qoc_amd import GrapeEngine
    H0, Hc, x0, xt, w_phi = _tunable_bus_setup()
    P = np.array([[300.0, 50.0, 0.25, w_phi, 0.13],
                  [280.0, 60.0, 0.22, w_phi * 1.01, 0.15],
                  [320.0, 20.0, 0.27, w_phi * 0.99, 0.10]])
    e = GrapeEngine(-1j * H0, [-1j * Hc], x0, 1, B=3)
    e.set_cost_external()
    # lab-frame energies reach ~125 rad/ns, so fixed-step Tsit5 needs dt ~ 1e-3 (the example's value);
    # dt = 2e-3 over a 40 ns window keeps the oracle quick
    J, x = e.propagate_envelope("tunable_bus", P, 40.0, 2e-3)
    assert J is None
    for b in range(3):
        xr = O.propagate_envelope(-1j * H0, [-1j * Hc], O.tunable_bus_envelope, P[b], x0, 40.0, 2e-3)
        assert abs(np.linalg.norm(xr) - 1) < 1e-4  # stable integration (Tsit5 damps slightly)
        # 20000 steps through ~5000 rad of phase: summation-order round-off grows ~ steps * eps * ||H|| dt
        assert np.abs(x[b][:, 0] - xr).max() < 1e-10, b
    e.close()


def _transmon(N=4, anh=-0.3):
    from qoc_amd import systems as S
    a = S.annihilation_op(N)
    H0 = anh / 2 * (a.conj().T @ a.conj().T @ a @ a)
    return -1j * H0, [-1j * (a + a.conj().T) / 2, -1j * (1j * (a.conj().T - a)) / 2]


@pytest.mark.parametrize("kind", ["drag", "sinebasis"])
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_envelope_drag_sinebasis_match_oracle(built_lib, kind, precision):
    from qoc_amd import GrapeEngine
    A0, A = _transmon()
    x0 = np.eye(4, dtype=complex)[:, :2]
    if kind == "drag":
        P = np.array([[20.0, 5.0, 0.16, 0.4], [24.0, 4.0, 0.13, -0.2]])
        env = O.drag_envelope
        tg = P[:, 0]
    else:
        P = np.array([[20.0, 0.05, 0.01, -0.02, 0.03, 0.004, 0.0],
                      [20.0, 0.07, -0.01, 0.01, 0.0, -0.01, 0.02]])
        env = O.sinebasis_envelope
        tg = P[:, 0]
    e = GrapeEngine(A0, A, x0, 1, B=2, precision=precision)
    e.set_cost_trace(np.eye(4, dtype=complex)[:, [1, 0]], 2)
    tol = 1e-12 if precision == "fp64" else 2e-5
    for b in range(2):
        # one gate time per call (tgate is shared by the batch)
        _, x = e.propagate_envelope(kind, P, float(tg[b]), 0.01)
        xr = O.propagate_envelope(A0, A, env, P[b], x0, float(tg[b]), 0.01)
        assert np.abs(x[b] - xr).max() < tol, (b, np.abs(x[b] - xr).max())
    e.close()
