"""GPU parity of the large-N path (chunked batched-GEMM pipeline, Newton-Schulz Padé solve) vs the
CPU oracle.  The path is selected automatically above the LDS-resident envelope (N > 48) and can be
forced for any N with QOC_FORCE_LARGE_N=1, which lets the fp64 cases reuse the small physics
configurations at the oracle's fp64 tolerances (|ΔJ| <= 1e-12, rel ||ΔdJdu|| <= 1e-10).
fp32 (synthetic N = 256, config 5): |ΔJ| <= 1e-4, rel ||ΔdJdu|| <= 1e-3.
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


def _run(prob, u, order=3, precision="fp64", penalty=None, x0=None):
    from qoc_amd import GrapeEngine
    B = u.shape[0]
    e = GrapeEngine(prob.A0, prob.A, prob.x0 if x0 is None else x0, prob.Nt, B=B, precision=precision)
    e.set_cost_trace(prob.x_target, prob.n)
    if penalty is not None:
        e.set_state_penalty(*penalty)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, order)
    info = e.info()
    hist = e.pade_histogram()
    e.close()
    return J, g, info, hist


def _compare(prob, u, J, g, order=3, tol=(1e-12, 1e-10), penalty=None, x0s=None):
    for b in range(u.shape[0]):
        x0 = prob.x0 if x0s is None else x0s[b]
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], x0, prob.x_target, prob.n, order=order, penalty=penalty)
        assert abs(J[b] - Jr) <= tol[0], (b, J[b], Jr)
        rel = np.linalg.norm(g[b] - gr) / max(np.linalg.norm(gr), 1e-300)
        assert rel <= tol[1], (b, rel)


def test_forced_large_n_cavity_fp64(built_lib, monkeypatch):
    from qoc_amd import systems
    monkeypatch.setenv("QOC_FORCE_LARGE_N", "1")
    monkeypatch.setenv("QOC_CHUNK", "7")  # 90 slices -> 13 chunks, ragged last chunk
    prob = systems.cavity_problem(N_cavity=6, Nt=30)
    u = systems.cavity_controls(3, prob.Nt, seed=0)
    J, g, info, hist = _run(prob, u)
    assert info["path"] == "large_n" and info["chunk"] == 7
    assert sum(hist.values()) == 3 * prob.Nt
    _compare(prob, u, J, g)
    # the Padé + Newton-Schulz variant of the pipeline (QOC_EXPM_PADE=1) gives the same results
    monkeypatch.setenv("QOC_EXPM_PADE", "1")
    J2, g2, info2, _ = _run(prob, u)
    assert info2["ns_iters"] > 0
    _compare(prob, u, J2, g2)


@pytest.mark.parametrize("order", [1, 2, 4])
def test_forced_large_n_orders(built_lib, monkeypatch, order):
    from qoc_amd import systems
    monkeypatch.setenv("QOC_FORCE_LARGE_N", "1")
    prob = systems.zz_problem(40)
    u = systems.zz_controls(2, 40, 10.0, seed=1)
    J, g, info, _ = _run(prob, u, order=order)
    assert info["path"] == "large_n"
    _compare(prob, u, J, g, order=order)


def test_forced_large_n_penalty_and_per_seed_x0(built_lib, monkeypatch):
    from qoc_amd import GrapeEngine, systems
    monkeypatch.setenv("QOC_FORCE_LARGE_N", "1")
    prob = systems.cavity_problem(N_cavity=6, Nt=20)
    u = systems.cavity_controls(2, prob.Nt, seed=3)
    pen = (list(range(prob.A0.shape[0] - 3, prob.A0.shape[0])), list(range(prob.x0.shape[1])), 0.7)
    J, g, _, _ = _run(prob, u, penalty=pen)
    _compare(prob, u, J, g, penalty=pen)
    # per-seed x0
    rng = np.random.default_rng(9)
    x0s = []
    for _ in range(2):
        Z = rng.standard_normal(prob.x0.shape) + 1j * rng.standard_normal(prob.x0.shape)
        x0s.append(np.linalg.qr(Z)[0])
    x0s = np.stack(x0s)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2)
    assert e.info()["path"] == "large_n"
    e.set_x0(x0s, per_seed=True)
    e.set_cost_trace(prob.x_target, prob.n)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    e.close()
    _compare(prob, u, J, g, x0s=x0s)


def _gue_problem(N, m, Nt, norm0, normj, nu=2, seed=0):
    from qoc_amd import systems
    rng = np.random.default_rng(seed)

    def scaled(H, s):
        return H * (s / np.abs(H).sum(axis=0).max())
    A0 = -1j * scaled(systems._gue(rng, N), norm0)
    A = [-1j * scaled(systems._gue(rng, N), normj) for _ in range(nu)]
    x0 = np.eye(N, dtype=np.complex128)[:, :m]
    Z = rng.standard_normal((N, m)) + 1j * rng.standard_normal((N, m))
    Xt = np.linalg.qr(Z)[0]
    return systems.Problem("gue", A0, A, x0, Xt, float(m), Nt, "fp64")


def test_auto_large_n_ragged_fp64_with_squarings(built_lib, monkeypatch):
    """N = 70 (not a multiple of the 64-wide GEMM tile), m = 3, norms that select d = 13 with
    squarings in some chunks and lower degrees in others."""
    monkeypatch.setenv("QOC_CHUNK", "3")
    prob = _gue_problem(70, 3, 5, norm0=9.0, normj=2.0, seed=4)
    rng = np.random.default_rng(5)
    u = rng.uniform(-1, 1, size=(2, 2, prob.Nt))
    u[1] *= 0.0  # seed 1: A_k = A0 only
    J, g, info, hist = _run(prob, u)
    assert info["path"] == "large_n"
    assert any(s > 0 for (d, s) in hist), hist
    _compare(prob, u, J, g)
    # low-norm problem -> degrees < 13 on the same path
    prob = _gue_problem(70, 3, 4, norm0=0.6, normj=0.1, seed=6)
    u = rng.uniform(-1, 1, size=(2, 2, prob.Nt))
    J, g, info, hist = _run(prob, u)
    assert all(d < 13 for (d, s) in hist), hist
    _compare(prob, u, J, g)


def test_synthetic_n256_fp32(built_lib):
    from qoc_amd import systems
    prob = systems.synthetic_problem(256, Nt=3)
    u = systems.synthetic_controls(2, 3, 2, seed=0)
    J, g, info, hist = _run(prob, u, precision="fp32")
    assert info["path"] == "large_n"
    assert set(hist) == {(13, 0)}, hist
    _compare(prob, u, J, g, tol=(1e-4, 1e-3))
    # J ~ 1 for a Haar target, so also compare the propagated states themselves
    from qoc_amd import GrapeEngine
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2, precision="fp32")
    e.set_cost_trace(prob.x_target, prob.n)
    e.propagate(u)
    for b in range(2):
        xr = O.propagate(prob.A0, prob.A, u[b], prob.x0)
        for k in (1, prob.Nt):
            x = e.state(k, seed=b)
            assert np.linalg.norm(x - xr[k]) / np.linalg.norm(xr[k]) < 2e-5, (b, k)
        U = e.propagator(0, seed=b)
        Ur = O.expm_higham2005(prob.A0 + sum(u[b, j, 0] * prob.A[j] for j in range(2)))[0]
        assert np.abs(U - Ur).max() < 2e-5
    e.close()


def test_synthetic_n256_fp64(built_lib):
    from qoc_amd import systems
    prob = systems.synthetic_problem(256, Nt=2)
    u = systems.synthetic_controls(1, 2, 2, seed=1)
    J, g, info, _ = _run(prob, u, precision="fp64")
    _compare(prob, u, J, g, tol=(1e-11, 1e-9))


@pytest.mark.parametrize("sandwich", ["0", "1"])
def test_order3_gradient_forms(built_lib, monkeypatch, sandwich):
    """The large-N order-3 gradient in both forms: seven N^2 m-GEMMs through P_a = X^a x and W_a (default for
    m <= 2N/3), and five products of G = λ x^H (default for m > 2N/3; QOC_GRAD_SANDWICH forces either).
    fp64, ragged N = 70 with m = 3 and m = N (chunk of 3 slices, ragged last chunk), penalty on."""
    monkeypatch.setenv("QOC_CHUNK", "3")
    monkeypatch.setenv("QOC_GRAD_SANDWICH", sandwich)
    rng = np.random.default_rng(11)
    for m in (3, 70):
        prob = _gue_problem(70, m, 5, norm0=1.5, normj=0.5, seed=12 + m)
        u = rng.uniform(-1, 1, size=(2, 2, prob.Nt))
        pen = (list(range(60, 70)), list(range(min(m, 4))), 0.3)
        J, g, info, _ = _run(prob, u, penalty=pen)
        assert info["path"] == "large_n"
        _compare(prob, u, J, g, penalty=pen)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_large_n_t12_and_paterson_stockmeyer(built_lib, monkeypatch, precision):
    """The large-N exponential picks the 4-product degree-12 Taylor scheme (histogram row m = 12) whenever it needs
    fewer GEMMs than Paterson-Stockmeyer (m = 3r+2); QOC_BIG_NO_T12=1 keeps Paterson-Stockmeyer.  Both match the
    oracle (fp64 bar, or the fp32 tolerance) on norms that need squarings."""
    from qoc_amd import GrapeEngine
    monkeypatch.setenv("QOC_CHUNK", "4")
    monkeypatch.setenv("QOC_BIG_NORM1", "1")  # the 1-norm choice without the 3-product T8 (next test)
    monkeypatch.setenv("QOC_BIG_NO_T8", "1")
    rng = np.random.default_rng(31)
    prob = _gue_problem(72, 4, 6, norm0=2.4, normj=0.6, seed=32)
    u = rng.uniform(-1, 1, size=(2, 2, prob.Nt))
    tol = (1e-12, 1e-10) if precision == "fp64" else (1e-4, 1e-3)
    hists = {}
    for off in ("0", "1"):
        if off == "1":
            monkeypatch.setenv("QOC_BIG_NO_T12", "1")
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2, precision=precision)
        assert e.info()["path"] == "large_n"
        e.set_cost_trace(prob.x_target, prob.n)
        J = e.propagate(u)
        g = e.grape_sensitivity(u, 3)
        hists[off] = e.taylor_histogram()
        e.close()
        _compare(prob, u, J, g, tol=tol)
    assert hists["0"] and all(m == 12 for (m, _) in hists["0"]), hists
    assert hists["1"] and all(m != 12 for (m, _) in hists["1"]), hists


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_large_n_t8_with_spectral_bound(built_lib, monkeypatch, precision):
    """Skew-Hermitian generators: the chunk's Taylor choice follows the 2-norm bound Σ_j |c_jk| ρ_j (ρ_j = ||A_j||_2
    from the host tridiagonalisation), and degrees <= 8 run in 3 products (T8, histogram row m = 8; fp32: no
    squaring at the GUE norms, fp64 with squarings).  QOC_BIG_NO_T8=1 falls back to T12 / Paterson-Stockmeyer and
    QOC_BIG_NORM1=1 to the 1-norm choice; every variant matches the oracle."""
    from qoc_amd import GrapeEngine
    monkeypatch.setenv("QOC_CHUNK", "4")
    rng = np.random.default_rng(33)
    # 1-norms; the spectral radii of these GUE generators are ~0.3 of them (fp32: bound ~0.5 <= θ8 = 0.648; fp64:
    # bound ~0.04 <= θ8 = 0.0699)
    norms = (1.2, 0.3) if precision == "fp32" else (0.1, 0.03)
    prob = _gue_problem(72, 4, 6, norm0=norms[0], normj=norms[1], seed=34)
    u = rng.uniform(-1, 1, size=(2, 2, prob.Nt))
    tol = (1e-12, 1e-10) if precision == "fp64" else (1e-4, 1e-3)
    hists = {}
    for mode in ("t8", "no_t8", "norm1"):
        if mode == "no_t8":
            monkeypatch.setenv("QOC_BIG_NO_T8", "1")
        if mode == "norm1":
            monkeypatch.delenv("QOC_BIG_NO_T8")
            monkeypatch.setenv("QOC_BIG_NORM1", "1")
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2, precision=precision)
        e.set_cost_trace(prob.x_target, prob.n)
        J = e.propagate(u)
        g = e.grape_sensitivity(u, 3)
        hists[mode] = e.taylor_histogram()
        e.close()
        _compare(prob, u, J, g, tol=tol)
    assert hists["t8"] and all(m == "8t" and s == 0 for (m, s) in hists["t8"]), hists
    assert all(m != "8t" for (m, _) in hists["no_t8"]), hists

    def gemms(h):  # T8 3 + s, T12 4 + s, Paterson-Stockmeyer m = 3r + 2: 2 + r + s
        return sum(c * ((3 if m == "8t" else 4 if m == 12 else 2 + (m - 2) // 3) + s) for (m, s), c in h.items())
    assert gemms(hists["no_t8"]) > gemms(hists["t8"]), hists
    assert gemms(hists["norm1"]) > gemms(hists["t8"]), hists  # the 1-norm bound costs products
