"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle on identical inputs.

Tolerances (fp64 GPU vs fp64 restatement): |ΔJ| <= 1e-12 and
||ΔdJdu||_F / ||dJdu||_F <= 1e-10 per seed; fp32: |ΔJ| <= 1e-4, rel 1e-3.

Both chain modes run the hot-path cases: 'propagators' (every U_k = exp(A_k) formed on MFMA, then the serial
products — the reference's structure) and 'taylor' (the exponential applied to the state, no U_k).
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


# "taylor" takes the block chains where the generators have small invariant blocks (zz, cavity: qoc_blk.hpp);
# "taylor_dense" keeps the dense Taylor-action kernels there (QOC_BLOCKS=0 at qoc_set_generators)
CHAINS = ["propagators", "taylor", "taylor_dense"]


def _engine(prob, B, precision="fp64", chain=None, cost=True):
    import os
    from qoc_amd import GrapeEngine
    dense = chain == "taylor_dense"
    old = os.environ.get("QOC_BLOCKS")
    if dense:
        os.environ["QOC_BLOCKS"] = "0"
    try:
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B, precision=precision)
    finally:
        if dense:
            if old is None:
                os.environ.pop("QOC_BLOCKS")
            else:
                os.environ["QOC_BLOCKS"] = old
    if cost:
        e.set_cost_trace(prob.x_target, prob.n)
    if chain is not None:
        chain = "taylor" if dense else chain
        e.set_chain(chain)
        assert e.info()["chain"] == chain
        if dense:
            assert e.info()["chain_kernel"] != "blocks"
    return e


def _check(prob, u, order=3, precision="fp64", penalty=None, chain=None):
    B = u.shape[0]
    e = _engine(prob, B, precision, chain)
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


@pytest.mark.parametrize("chain", CHAINS)
def test_cavity_small_parity(built_lib, chain):
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=6, Nt=30)
    _check(prob, systems.cavity_controls(3, prob.Nt, seed=0), chain=chain)


@pytest.mark.parametrize("chain", CHAINS)
def test_zz_parity(built_lib, chain):
    from qoc_amd import systems
    prob = systems.zz_problem(100)
    _check(prob, systems.zz_controls(2, 100, 10.0, seed=0), chain=chain)


@pytest.mark.parametrize("chain", CHAINS)
def test_cavity40_parity(built_lib, chain):
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=20, Nt=40)
    _check(prob, systems.cavity_controls(2, prob.Nt, seed=5), chain=chain)


@pytest.mark.parametrize("chain", CHAINS)
def test_tunable_bus_parity(built_lib, chain):
    from qoc_amd import systems
    prob = systems.tunable_bus_problem(Nt=60, tgate=350.0 * 60 / 2000)
    _check(prob, systems.tunable_bus_controls(2, prob.Nt, seed=0), chain=chain)


@pytest.mark.parametrize("chain", CHAINS)
@pytest.mark.parametrize("order", [1, 2, 3, 4])
def test_orders(built_lib, order, chain):
    from qoc_amd import systems
    prob = systems.zz_problem(50, tgate=5.0)
    _check(prob, systems.zz_controls(2, 50, 5.0, seed=order), order=order, chain=chain)


@pytest.mark.parametrize("chain", CHAINS)
def test_state_penalty(built_lib, chain):
    from qoc_amd import systems
    prob = systems.zz_problem(40, tgate=4.0)
    qb = systems.QuantumBasis([3, 3])
    pen = (qb(["20", "21", "22"]), [0, 1, 2, 3], 0.37)
    _check(prob, systems.zz_controls(2, 40, 4.0, seed=9), penalty=pen, chain=chain)


# z-calibrated cost: the calibration phase θ comes from a golden-section search over a flat maximum
# (src/fidelities.jl:81-137).  Its iterates branch on comparisons of objective values that agree to ~1e-16 near
# the optimum, so θ is fixed only to ~sqrt(eps) and two correct implementations (GPU, oracle) stop at phases a
# few 1e-9..1e-8 apart.  J is stationary in θ (held to the 1e-12 bar); the gradient carries e^{iθ} linearly, so
# it is compared with the oracle's gradient family g(Δθ) (qoc_oracle.zcal_gradient_match): the GPU gradient
# must equal g(Δθ) to the 1e-10 bar for some |Δθ| within the per-seed bound qoc_oracle.zcal_dtheta_bound derives
# from the curvature of the calibration objective at its maximum (≈ 2.5e-7 for these cases).


@pytest.mark.parametrize("path", ["propagators", "taylor", "large_n", "tsit5"])
def test_zcalibrated_cost(built_lib, path, monkeypatch):
    """setup_infidelity_zcalibrated on the device, on every propagation path (src/penalty_fcns.jl:27-42 works
    for any propagation): fused in the chain epilogues, or k_terminal_cost after the large-N / Tsit5 forward."""
    from qoc_amd import GrapeEngine, systems
    if path == "large_n":
        monkeypatch.setenv("QOC_FORCE_LARGE_N", "1")
    prob = systems.zz_problem(40, tgate=4.0)
    u = systems.zz_controls(3, 40, 4.0, seed=21)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=3)
    if path in ("propagators", "taylor"):
        e.set_chain(path)
    if path == "tsit5":
        e.set_propagation("tsit5", 8)
    assert (e.info()["path"] == "large_n") == (path == "large_n")
    e.set_cost_zcalibrated(prob.x_target)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    Jz, _ = O.setup_infidelity_zcalibrated(prob.x_target)
    nsub = 8 if path == "tsit5" else None
    for b in range(3):
        xN = (O.propagate_pwc_ode(prob.A0, prob.A, u[b], prob.x0, nsub=8) if nsub else
              O.propagate(prob.A0, prob.A, u[b], prob.x0))[-1]
        assert abs(J[b] - Jz(xN)) <= 1e-12, (b, J[b] - Jz(xN))
        res, dth = O.zcal_gradient_match(g[b], prob.A0, prob.A, u[b], prob.x0, prob.x_target, order=3, nsub=nsub)
        bound = O.zcal_dtheta_bound(prob.x_target, xN)
        print(f"zcal {path} seed {b}: |dtheta| = {abs(dth):.3e} (bound {bound:.3e}), residual {res:.2e}")
        assert res <= 1e-10 and abs(dth) <= bound, (b, res, dth, bound)
    e.close()


def test_expm_jacobian_kernel_matches_oracle_and_fd_contract(built_lib):
    from qoc_amd import expm_jacobian
    rng = np.random.default_rng(0)
    A0, A1, A2 = [0.05 * rng.standard_normal((3, 3)) for _ in range(3)]
    u = np.array([1.0, 2.0])
    for order in (1, 2, 3, 4):
        for dt in (1.0, 0.25):
            got = expm_jacobian(A0, [A1, A2], u, order, dt)
            ref = O.expm_jacobian(A0, [A1, A2], u, order, dt)
            for a, b in zip(got, ref):
                assert np.abs(a - b).max() < 1e-15
    from test_oracle import _fd_jac
    for order, dt, thr in ((3, 1.0, 4e-4), (4, 1.0, 3e-5), (3, 0.25, 2e-6), (4, 0.25, 3e-8)):
        got = expm_jacobian(A0, [A1, A2], u, order, dt)
        err = np.linalg.norm(np.stack([x.ravel(order="F") for x in got], 1) - _fd_jac(A0, [A1, A2], u, dt))
        assert err < thr


def test_device_pointer_eval_matches_host_path(built_lib):
    import torch
    from qoc_amd import GrapeEngine, systems
    prob = systems.cavity_problem(N_cavity=10, Nt=30)
    u = systems.cavity_controls(4, 30, seed=3)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=4)
    e.set_cost_trace(prob.x_target, prob.n)
    Jh = e.propagate(u)
    gh = e.grape_sensitivity(u, 3)
    ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
    Jd = torch.empty(4, dtype=torch.float64, device="cuda")
    gd = torch.empty(4, 30, 2, dtype=torch.float64, device="cuda")
    e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
    e.synchronize()
    # the device eval runs the segmented block eval (csrc/qoc_blkseg.hpp: segment products and a prefix scan, the
    # closed-form block exponential) where the host path runs the sequential chains: the same J and gradient to
    # rounding, not bit for bit
    assert np.abs(Jd.cpu().numpy() - Jh).max() <= 1e-13
    gdh = np.transpose(gd.cpu().numpy(), (0, 2, 1))
    for b in range(4):
        assert np.linalg.norm(gdh[b] - gh[b]) / np.linalg.norm(gh[b]) <= 1e-12
    # stale check on the device path
    e.propagate_device(ud.data_ptr(), Jd.data_ptr())
    u2 = ud.clone()
    u2[0, 0, 0] += 1e-3
    from qoc_amd import StaleCacheError
    with pytest.raises(StaleCacheError):
        e.grape_sensitivity_device(u2.data_ptr(), 3, gd.data_ptr())
    e.close()


def test_reference_shaped_api(built_lib):
    """propagate / grape_sensitivity mirror (closure dJfinal_dx evaluated on x[end], stale-u error)."""
    import qoc_amd as Q
    from qoc_amd import systems
    prob = systems.zz_problem(30, tgate=3.0)
    u = systems.zz_controls(1, 30, 3.0, seed=4)[0]
    cache = Q.setup_grape_cache(prob.A0, prob.x0, u.shape)
    x = Q.propagate(prob.A0, prob.A, u, prob.x0, cache)
    assert len(x) == 31
    Jf, dJf = Q.setup_infidelity(prob.x_target, 4)
    user_closure = lambda xN: dJf(xN)  # noqa: E731  (untagged: goes through QOC_COST_EXTERNAL)
    g = Q.grape_sensitivity(prob.A0, prob.A, user_closure, cache.u, prob.x0, cache, dUkdp_order=3)
    Jr, gr, cr = O.grape_eval(prob.A0, prob.A, u, prob.x0, prob.x_target, 4, order=3)
    assert abs(Jf(x[-1]) - Jr) < 1e-12
    assert np.linalg.norm(g - gr) / np.linalg.norm(gr) < 1e-10
    assert np.abs(x[7] - cr.x[7]).max() < 1e-13
    assert np.abs(cache.lam[3] - cr.lam[3]).max() < 1e-12
    with pytest.raises(Q.StaleCacheError, match="Cache data from other control signal u"):
        Q.grape_sensitivity(prob.A0, prob.A, dJf, u * 1.01, prob.x0, cache)
    L, dL = Q.setup_state_penalty([6, 7, 8], [0, 1, 2, 3], 0.3)
    g2 = Q.grape_sensitivity(prob.A0, prob.A, dJf, cache.u, prob.x0, cache, dUkdp_order=3, dL_dx=dL)
    Lo, dLo = O.setup_state_penalty([6, 7, 8], [0, 1, 2, 3], 0.3)
    c2 = O.setup_grape_cache(prob.A0, prob.x0, u.shape)
    O.propagate(prob.A0, prob.A, u, prob.x0, c2)
    gr2 = O.grape_sensitivity(prob.A0, prob.A, O.setup_infidelity(prob.x_target, 4)[1], c2.u, prob.x0, c2,
                              dUkdp_order=3, dL_dx=dLo)
    assert np.linalg.norm(g2 - gr2) / np.linalg.norm(gr2) < 1e-10


def test_propagate_without_cache_real_x0(built_lib):
    """propagate(A0, A, u, x0) with no cache and a real N x m x0 (np.eye(N)[:, :m]): the reference converts x0 to
    complex before building the cache (src/gradient_computations.jl:4-8), so it is a complex state, not the
    2N-row complex2real layout."""
    import qoc_amd as Q
    from qoc_amd import systems
    prob = systems.zz_problem(20, tgate=2.0)
    u = systems.zz_controls(1, 20, 2.0, seed=6)[0]
    x0 = np.eye(prob.N)[:, :4]
    x = Q.propagate(prob.A0, prob.A, u, x0)
    c = O.setup_grape_cache(prob.A0, x0.astype(complex), u.shape)
    xr = O.propagate(prob.A0, prob.A, u, x0.astype(complex), c)
    assert len(x) == 21
    assert np.abs(x[20] - xr[20]).max() < 1e-13


@pytest.mark.parametrize("chain", CHAINS)
def test_fp32_small(built_lib, chain):
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=10, Nt=40)
    _check(prob, systems.cavity_controls(2, 40, seed=8), precision="fp32", chain=chain)


@pytest.mark.parametrize("chain", CHAINS)
def test_per_seed_x0(built_lib, chain):
    from qoc_amd import GrapeEngine, systems
    prob = systems.zz_problem(20, tgate=2.0)
    u = systems.zz_controls(2, 20, 2.0, seed=2)
    rng = np.random.default_rng(5)
    x0s = np.stack([np.linalg.qr(rng.standard_normal((9, 4)) + 1j * rng.standard_normal((9, 4)))[0] for _ in range(2)])
    e = _engine(prob, 2, chain=chain, cost=False)
    e.set_x0(x0s, per_seed=True)
    e.set_cost_trace(prob.x_target, 4)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    for b in range(2):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], x0s[b], prob.x_target, 4, order=3)
        assert abs(J[b] - Jr) < 1e-12 and np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) < 1e-10
    e.close()


def test_non_dominant_q_uses_pivoted_lu(built_lib):
    """Dense random generators with ||A||_1 ~ 4-5: Q = V-U is not diagonally dominant."""
    from qoc_amd import expm, systems
    rng = np.random.default_rng(9)
    for N in (17, 33, 40):
        A = []
        for _ in range(3):
            H = systems._gue(rng, N)
            A.append(-1j * H * 4.5 / np.abs(H).sum(0).max())
        X = expm(np.stack(A))
        for a, x in zip(A, X):
            Xr, d, s = O.expm_higham2005(a)
            assert np.abs(x - Xr).max() < 1e-13


@pytest.mark.parametrize("which", ["zz", "tunable_bus_small"])
def test_exact_frechet_gradient_matches_oracle(built_lib, which):
    """QOC_DUKDP_EXACT: zz (2N = 18 -> k_expm block exponentials) and tunable bus (2N = 54 -> the GEMM
    pipeline); oracle = per-control block exponentials (pinned to scipy expm_frechet and FD)."""
    from qoc_amd import systems
    if which == "zz":
        prob = systems.zz_problem(20, tgate=2.0)
        u = systems.zz_controls(2, 20, 2.0, seed=3)
    else:
        prob = systems.tunable_bus_problem(12, tgate=350.0 * 12 / 2000)
        u = systems.tunable_bus_controls(2, 12, seed=1)
    e = _engine(prob, u.shape[0])
    J = e.propagate(u)
    g = e.grape_sensitivity(u, "exact")
    for b in range(u.shape[0]):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order="exact")
        assert abs(J[b] - Jr) <= 1e-12
        rel = np.linalg.norm(g[b] - gr) / np.linalg.norm(gr)
        assert rel <= 1e-10, (b, rel)
    e.close()


def test_exact_gradient_large_n_path(built_lib, monkeypatch):
    from qoc_amd import systems
    monkeypatch.setenv("QOC_FORCE_LARGE_N", "1")
    prob = systems.zz_problem(10, tgate=2.0)
    u = systems.zz_controls(2, 10, 2.0, seed=4)
    e = _engine(prob, 2)
    assert e.info()["path"] == "large_n"
    e.propagate(u)
    g = e.grape_sensitivity(u, "exact")
    for b in range(2):
        _, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order="exact")
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10
    e.close()


def test_taylor_default_and_pade_option_agree(built_lib, monkeypatch):
    """The default exponential is the register-resident degree-12 Taylor in 4 GEMMs (+ squarings when
    ||A||_1 > 0.335); QOC_EXPM_LDS=1 selects the LDS Paterson-Stockmeyer kernel and QOC_EXPM_PADE=1 the
    reference's Padé + solve.  All match the oracle; the histograms record what ran."""
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=20, Nt=12)
    u = systems.cavity_controls(2, prob.Nt, seed=2)
    out = {}
    for mode, env in (("t12", {}), ("ps", {"QOC_EXPM_LDS": "1"}), ("pade", {"QOC_EXPM_PADE": "1"})):
        for k in ("QOC_EXPM_LDS", "QOC_EXPM_PADE"):
            monkeypatch.setenv(k, env.get(k, "0"))
        e = _engine(prob, 2, chain="propagators")
        J = e.propagate(u)
        g = e.grape_sensitivity(u, 3)
        out[mode] = (J, g, e.pade_histogram(), e.taylor_histogram())
        e.close()
    J0, g0, ph0, th0 = out["t12"]
    assert set(th0) <= {(12, 0), (12, 1)} and sum(th0.values()) == 24
    assert out["ps"][3] == {(14, 0): 24} and out["pade"][3] == {}
    for mode in ("t12", "ps", "pade"):
        assert out[mode][2] == {(7, 0): 24}
        np.testing.assert_allclose(out[mode][0], J0, rtol=0, atol=1e-13)
        np.testing.assert_allclose(out[mode][1], g0, rtol=1e-11, atol=1e-15)
    for b in range(2):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J0[b] - Jr) <= 1e-12
        assert np.linalg.norm(g0[b] - gr) / np.linalg.norm(gr) <= 1e-10


@pytest.mark.parametrize("path", ["fused", "gemm"])
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_gemm_gradient_n40_penalty_and_precision(built_lib, monkeypatch, precision, path):
    """The order-3 gradient at N = 40: the fused register-resident kernels (default) and the GEMM-shaped
    path (QOC_GRAD_GEMM=1: generator-combine + fused contraction), with the guard-state penalty (λ
    carries dL/dx), in both precisions, against the oracle."""
    from qoc_amd import systems
    monkeypatch.setenv("QOC_GRAD_GEMM", "1" if path == "gemm" else "0")
    prob = systems.cavity_problem(N_cavity=20, Nt=16)
    u = systems.cavity_controls(3, prob.Nt, seed=11)
    pen = (list(range(30, 40)), [0, 1], 0.23)
    _check(prob, u, precision=precision, penalty=pen)


@pytest.mark.parametrize("which", ["cavity40", "zz", "tunable_bus", "ragged"])
def test_fused_gradient_equals_per_slice_kernel(built_lib, monkeypatch, which):
    """Fused gradient (default), GEMM path and per-slice k_grad agree to rounding: m = 2, 4, 1, nu = 2, 1,
    and a ragged tile count (B * Nt not a multiple of the 16/m units per tile) with N = 23."""
    from qoc_amd import systems
    if which == "cavity40":
        prob = systems.cavity_problem(N_cavity=20, Nt=10)
        u = systems.cavity_controls(2, prob.Nt, seed=12)
    elif which == "zz":
        prob = systems.zz_problem(Nt=30)
        u = systems.zz_controls(3, prob.Nt, tgate=1.2, seed=4)
    elif which == "tunable_bus":
        prob = systems.tunable_bus_problem(Nt=21)
        u = systems.tunable_bus_controls(3, prob.Nt, seed=5)
    else:
        import dataclasses
        p0 = systems.synthetic_problem(N=23, nu=2, Nt=7, seed=3, precision="fp64")
        prob = dataclasses.replace(p0, x0=p0.x0[:, :2].copy(), x_target=p0.x_target[:, :2].copy(), n=2.0)
        u = systems.synthetic_controls(3, prob.Nt, nu=2, seed=3) * 0.2
    res = []
    for env in ({}, {"QOC_GRAD_GEMM": "1"}, {"QOC_GRAD_KERNEL": "1"}):
        for k in ("QOC_GRAD_GEMM", "QOC_GRAD_KERNEL"):
            monkeypatch.setenv(k, env.get(k, "0"))
        e = _engine(prob, u.shape[0])
        e.propagate(u)
        res.append(e.grape_sensitivity(u, 3))
        e.close()
    scale = np.abs(res[2]).max()
    np.testing.assert_allclose(res[0], res[2], rtol=0, atol=1e-12 * scale)
    np.testing.assert_allclose(res[1], res[2], rtol=0, atol=1e-12 * scale)
    for b in range(u.shape[0]):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert np.linalg.norm(res[0][b] - gr) / np.linalg.norm(gr) <= 1e-10


@pytest.mark.parametrize("which", ["two_pass", "mix"])
def test_t12_and_paterson_stockmeyer_passes(built_lib, monkeypatch, which):
    """Slices with ||A_k||_1 > 4 theta_12 run Paterson-Stockmeyer (fewer squarings than T12): through the
    second pass over the listed units when ||A0||_1 is small (cavity with a few large controls), or in the
    one-pass mixed kernel when ||A0||_1 is large (tunable bus).  Both match the oracle; the executed
    histogram shows which scheme ran."""
    from qoc_amd import systems
    if which == "two_pass":
        prob = systems.cavity_problem(N_cavity=12, Nt=24)
        u = systems.cavity_controls(3, prob.Nt, seed=21)
        u[:, :, ::3] *= 60.0  # every third slice: ||A_k||_1 of a few units
    else:
        monkeypatch.setenv("QOC_EXPM_PS", "1")  # large norms default to the reference's Padé-13 otherwise
        prob = systems.tunable_bus_problem(Nt=200)
        u = systems.tunable_bus_controls(2, prob.Nt, seed=22)
    e = _engine(prob, u.shape[0], chain="propagators")
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    th = e.taylor_histogram()
    e.close()
    t12 = sum(v for (mm, _), v in th.items() if mm == 12)
    ps = sum(v for (mm, _), v in th.items() if mm != 12)
    assert t12 + ps == u.shape[0] * prob.Nt
    assert ps > 0 and (t12 > 0 if which == "two_pass" else t12 == 0)
    for b in range(u.shape[0]):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J[b] - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10


def test_taylor_chain_accounting_and_propagator_on_demand(built_lib):
    """Taylor-action chains: the executed-term counter, the reference-equivalent Padé histogram (evaluated
    from the propagated u) and qoc_get_propagator (formed on demand) against the oracle."""
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=20, Nt=12)
    u = systems.cavity_controls(2, prob.Nt, seed=2)
    e = _engine(prob, 2)
    assert e.info()["chain"] == "taylor"  # auto: ||A0 - mu I||_1 ~ 0.15
    e.chain_terms(reset=True)
    e.pade_histogram(reset=True)
    e.propagate(u)
    e.grape_sensitivity(u, 3)
    terms = e.chain_terms()
    assert 9 * 24 <= terms <= 14 * 24, terms  # P = 10..13 per slice at these norms
    assert e.pade_histogram() == {(7, 0): 24}
    for b, k in ((0, 0), (1, 11), (1, 5)):
        U = e.propagator(k, seed=b)
        Ak = prob.A0 + sum(u[b, j, k] * prob.A[j] for j in range(2))
        Ur, _, _ = O.expm_higham2005(Ak)
        assert np.abs(U - Ur).max() < 1e-13
    e.close()


@pytest.mark.parametrize("chain", CHAINS)
def test_external_cost_and_costates(built_lib, chain):
    """QOC_COST_EXTERNAL (caller's λ_N) and the stored co-states / states through both chain modes."""
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=8, Nt=25)
    u = systems.cavity_controls(2, prob.Nt, seed=31)
    e = _engine(prob, 2, chain=chain, cost=False)
    e.set_cost_external()
    e.propagate(u)
    rng = np.random.default_rng(3)
    lam = rng.standard_normal((2, prob.N, prob.m)) + 1j * rng.standard_normal((2, prob.N, prob.m))
    g = e.grape_sensitivity(u, 3, lambda_final=lam)
    for b in range(2):
        cache = O.setup_grape_cache(prob.A0, prob.x0, u[b].shape)
        O.propagate(prob.A0, prob.A, u[b], prob.x0, cache)
        gr = O.grape_sensitivity(prob.A0, prob.A, lambda x, lb=lam[b]: lb, cache.u, prob.x0, cache, dUkdp_order=3)
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10
        for k in (0, 9, prob.Nt):
            assert np.abs(e.state(k, seed=b) - cache.x[k]).max() < 1e-13
            assert np.abs(e.costate(k, seed=b) - cache.lam[k]).max() < 1e-12
    e.close()


def test_large_norm_slices_default_to_the_reference_pade(built_lib):
    """||A0||_1 > 4 theta_12 (tunable bus): in propagator mode the exponentials run the reference's Padé-13 +
    solve by default (no Taylor scheme in the executed histogram) and match the oracle."""
    from qoc_amd import systems
    prob = systems.tunable_bus_problem(Nt=120)
    u = systems.tunable_bus_controls(2, prob.Nt, seed=23)
    e = _engine(prob, 2, chain="propagators")
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    assert e.taylor_histogram() == {}
    assert sum(v for (d, _), v in e.pade_histogram().items() if d == 13) == 2 * prob.Nt
    e.close()
    for b in range(2):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J[b] - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10


@pytest.mark.parametrize("path", ["propagators", "taylor", "large_n"])
def test_arbitrary_dL_dx_closure(built_lib, monkeypatch, path):
    """A penalty gradient that is not setup_state_penalty's (src/gradient_computations.jl:47-49, 55-57 accept
    any closure): the host evaluates it on every state, the GPU adds dL_dx(x_k) to λ_k in the backward chain
    (qoc_set_costate_source).  Against the oracle with the same closure, through the reference-shaped API."""
    import qoc_amd as Q
    from qoc_amd import systems
    if path == "large_n":
        monkeypatch.setenv("QOC_FORCE_LARGE_N", "1")
    prob = systems.zz_problem(24, tgate=2.4)
    u = systems.zz_controls(1, 24, 2.4, seed=6)[0]
    rng = np.random.default_rng(2)
    W = rng.uniform(0.0, 0.4, size=(prob.N, prob.m))
    dL = lambda x: W * x + 0.05 * np.conj(x) ** 0 * x[0, 0]  # noqa: E731  (not a tagged penalty)
    cache = Q.setup_grape_cache(prob.A0, prob.x0, u.shape)
    if path != "large_n":
        cache.engine.set_chain(path)
    Q.propagate(prob.A0, prob.A, u, prob.x0, cache)
    Jf, dJf = O.setup_infidelity(prob.x_target, 4)
    g = Q.grape_sensitivity(prob.A0, prob.A, dJf, cache.u, prob.x0, cache, dUkdp_order=3, dL_dx=dL)
    c2 = O.setup_grape_cache(prob.A0, prob.x0, u.shape)
    O.propagate(prob.A0, prob.A, u, prob.x0, c2)
    gr = O.grape_sensitivity(prob.A0, prob.A, dJf, c2.u, prob.x0, c2, dUkdp_order=3, dL_dx=dL)
    assert np.linalg.norm(g - gr) / np.linalg.norm(gr) < 1e-10
    for k in (0, 11, 24):
        assert np.abs(cache.lam[k] - c2.lam[k]).max() < 1e-12
    # the source is cleared afterwards: an unpenalised call matches the oracle without dL_dx
    g0 = Q.grape_sensitivity(prob.A0, prob.A, dJf, cache.u, prob.x0, cache, dUkdp_order=3)
    gr0 = O.grape_sensitivity(prob.A0, prob.A, dJf, c2.u, prob.x0, c2, dUkdp_order=3)
    assert np.linalg.norm(g0 - gr0) / np.linalg.norm(gr0) < 1e-10


@pytest.mark.parametrize("poly", ["chebyshev", "taylor"])
@pytest.mark.parametrize("which", ["cavity40", "synthetic_large_norm"])
def test_taylor_action_polynomials(built_lib, monkeypatch, poly, which):
    """The Taylor-action chains' two polynomials: Chebyshev (default for skew-Hermitian generators; ||A||_1 up to
    ~4 here without substeps) and Taylor (QOC_TCHAIN_POLY=taylor; substeps at large norms), both vs the oracle."""
    import dataclasses
    from qoc_amd import systems
    if poly == "taylor":
        monkeypatch.setenv("QOC_TCHAIN_POLY", "taylor")
    if which == "cavity40":
        prob = systems.cavity_problem(N_cavity=20, Nt=30)
        u = systems.cavity_controls(2, prob.Nt, seed=41)
    else:
        p0 = systems.synthetic_problem(N=33, nu=2, Nt=9, seed=4, precision="fp64")
        prob = dataclasses.replace(p0, x0=p0.x0[:, :3].copy(), x_target=p0.x_target[:, :3].copy(), n=3.0)
        u = systems.synthetic_controls(2, prob.Nt, nu=2, seed=4)
    e = _engine(prob, 2, chain="taylor")
    assert e.info()["chain_poly"] == poly
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    e.close()
    for b in range(2):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J[b] - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10


def test_taylor_action_non_skew_hermitian_generators(built_lib):
    """Damped generators (A0 = -i H dt - gamma I, not skew-Hermitian): the Taylor polynomial runs (Chebyshev
    needs a spectrum on the imaginary axis), states no longer unitary; against the oracle."""
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=10, Nt=20)
    import dataclasses
    prob = dataclasses.replace(prob, A0=prob.A0 - 0.01 * np.eye(prob.N))
    u = systems.cavity_controls(2, prob.Nt, seed=42)
    e = _engine(prob, 2, chain="taylor")
    assert e.info()["chain_poly"] == "taylor"
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    e.close()
    for b in range(2):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J[b] - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10


@pytest.mark.parametrize("ranges", [("4", "0.5", "0"), ("3", "0.3", "0"), ("4", "0.5", "1"), ("3", "0.3", "1")])
def test_overlapped_backward_ranges_are_bit_identical(built_lib, monkeypatch, ranges):
    """The backward chain in slice ranges with each range's gradient on a second stream (default for the
    MFMA chains, Nt >= 64) gives bit-identical J, dJ/du and co-states to the single-launch backward
    (QOC_BWD_CHUNKS=1), with a state penalty and a ragged Nt, and matches the oracle.  QOC_BWD_PRESTATE=1: the
    state side (P1, P2) of every slice first, beside the first range (k_grad_rr_s), then q + p reading them."""
    monkeypatch.setenv("QOC_BWD_PRESTATE", ranges[2])
    monkeypatch.setenv("QOC_BLOCKS", "0")  # the dense chains' ranges (the block chains run one backward launch)
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=10, Nt=131)
    u = systems.cavity_controls(3, prob.Nt, seed=17)
    pen = ([3, 7], [0], 0.2)
    out = []
    for chunks in ("1",) + (ranges[0],):
        monkeypatch.setenv("QOC_BWD_CHUNKS", chunks)
        monkeypatch.setenv("QOC_BWD_LAST", ranges[1])
        e = _engine(prob, 3, chain="taylor")
        e.set_state_penalty(*pen)
        e.set_profiling(True)
        J = e.propagate(u)
        g = e.grape_sensitivity(u, 3)
        launches = e.phase_times()["k_chain_bwd"][1]
        lam = [e.costate(k, seed=b) for b in range(3) for k in range(prob.Nt + 1)]
        g2 = e.grape_sensitivity(u, 3)  # a second call on the same propagate: the same result
        assert np.array_equal(g, g2)
        e.close()
        out.append((J, g, np.array(lam), launches))
    assert out[0][3] == 1 and out[1][3] == int(ranges[0])
    for a, b in zip(out[0][:3], out[1][:3]):
        assert np.array_equal(a, b)
    for b in range(3):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, penalty=pen)
        assert abs(out[1][0][b] - Jr) <= 1e-12
        assert np.linalg.norm(out[1][1][b] - gr) / np.linalg.norm(gr) <= 1e-10


def test_overlapped_backward_with_costate_source_repeated(built_lib, monkeypatch):
    """The overlapped backward (ranges + gradient on the second stream) with the caller's co-state source, twice in a
    row on one engine and once more after a new propagate: every call matches the single-launch backward bitwise
    and the oracle's gradient with the same dL/dx closure."""
    from qoc_amd import systems
    monkeypatch.setenv("QOC_BLOCKS", "0")  # the dense chains' ranges
    prob = systems.cavity_problem(N_cavity=10, Nt=96)
    u = systems.cavity_controls(2, prob.Nt, seed=23)
    Lo, dLo = O.setup_state_penalty([1, 4], [0, 1], 0.15)
    res = []
    for chunks in ("1", "4"):
        monkeypatch.setenv("QOC_BWD_CHUNKS", chunks)
        e = _engine(prob, 2, chain="taylor")
        out = []
        for uu in (u, u, u * 0.9):
            e.propagate(uu)
            src = np.stack([np.stack([dLo(e.state(k, seed=b)) for k in range(prob.Nt + 1)]) for b in range(2)])
            e.set_costate_source(src)
            out.append(e.grape_sensitivity(uu, 3))
        e.close()
        res.append(out)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)
    for i, uu in enumerate((u, u, u * 0.9)):
        for b in range(2):
            c = O.setup_grape_cache(prob.A0, prob.x0, uu[b].shape)
            O.propagate(prob.A0, prob.A, uu[b], prob.x0, c)
            gr = O.grape_sensitivity(prob.A0, prob.A, O.setup_infidelity(prob.x_target, prob.n)[1], c.u, prob.x0, c,
                                     dUkdp_order=3, dL_dx=dLo)
            assert np.linalg.norm(res[1][i][b] - gr) / np.linalg.norm(gr) <= 1e-10
