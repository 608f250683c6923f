"""The register-resident MFMA chains (csrc/qoc_tchain.hpp TChainRot<G>: N <= 16 G for G = 1, 2, nu <= 2; one wave
per column pair holds the whole state in registers and the B operands come from DPP row rotations) against the
oracle and against the LDS-state kernels (TChainMF, QOC_TCHAIN_ROT=0), at the fp64 bar of SURVEY.md §8c: |ΔJ| <= 1e-12, ||ΔdJdu|| / ||dJdu|| <= 1e-10 per seed,
co-states 1e-12 relative to max|λ|.  The forward chain follows src/gradient_computations.jl:27-29, the backward
:52-58, the gradient :61-74 (order 3, the default of the Ipopt callbacks).
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _dense_chains(monkeypatch):
    """These kernels are the dense Taylor-action chains: the block path (qoc_blk.hpp) stays off."""
    monkeypatch.setenv("QOC_BLOCKS", "0")


def _cases():
    from qoc_amd import systems
    out = {}
    p = systems.zz_problem(60, tgate=6.0)  # N = 9, m = 4, nu = 2
    out["zz"] = (p, systems.zz_controls(3, 60, 6.0, seed=51))
    p = systems.cavity_problem(N_cavity=8, Nt=50)  # N = 16, m = 2
    out["cavity16"] = (p, systems.cavity_controls(3, p.Nt, seed=52))
    p = systems.cavity_problem(N_cavity=5, Nt=40)  # N = 10
    out["cavity10"] = (p, systems.cavity_controls(2, p.Nt, seed=53))
    # G = 2
    p = systems.tunable_bus_problem(Nt=64, tgate=350.0 * 64 / 2000)  # N = 27, m = 1, nu = 1
    out["tunable_bus"] = (p, systems.tunable_bus_controls(3, p.Nt, seed=56))
    p = systems.cavity_problem(N_cavity=12, Nt=40)  # N = 24
    out["cavity24"] = (p, systems.cavity_controls(2, p.Nt, seed=57))
    p = systems.cavity_problem(N_cavity=16, Nt=30)  # N = 32
    out["cavity32"] = (p, systems.cavity_controls(2, p.Nt, seed=58))
    return out


def _run(prob, u, rot, chain="taylor", device=False, penalty=None, monkeypatch=None):
    from qoc_amd import GrapeEngine
    monkeypatch.setenv("QOC_TCHAIN_ROT", "1" if rot else "0")
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=u.shape[0])
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_chain(chain)
    if penalty is not None:
        e.set_state_penalty(*penalty)
    if device:
        import torch
        B, nu, Nt = u.shape
        ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
        Jd = torch.empty(B, dtype=torch.float64, device="cuda")
        gd = torch.empty(B, Nt, nu, dtype=torch.float64, device="cuda")
        e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
        e.synchronize()
        J, g = Jd.cpu().numpy(), np.transpose(gd.cpu().numpy(), (0, 2, 1))
    else:
        J = e.propagate(u)
        g = e.grape_sensitivity(u, 3)
    info = e.info()
    lam = [e.costate(k, seed=0) for k in (0, prob.Nt // 2, prob.Nt)]
    e.close()
    return J, g, info, lam


@pytest.mark.parametrize("name", ["zz", "cavity16", "cavity10", "tunable_bus", "cavity24", "cavity32"])
@pytest.mark.parametrize("device", [False, True])
def test_rot_chains_match_oracle_and_lds_kernels(built_lib, monkeypatch, name, device):
    prob, u = _cases()[name]
    Jr_, gr_, ir, lr = _run(prob, u, True, device=device, monkeypatch=monkeypatch)
    Jl, gl, il, ll = _run(prob, u, False, device=device, monkeypatch=monkeypatch)
    assert ir["chain_kernel"] == "mfma_regs" and il["chain_kernel"] == "mfma_lds"
    assert ir["backward"] == il["backward"]
    for b in range(u.shape[0]):
        J0, g0, c0 = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(Jr_[b] - J0) <= 1e-12, (name, b, Jr_[b] - J0)
        rel = np.linalg.norm(gr_[b] - g0) / np.linalg.norm(g0)
        assert rel <= 1e-10, (name, b, rel)
        assert abs(Jr_[b] - Jl[b]) <= 1e-12
        assert np.linalg.norm(gr_[b] - gl[b]) / np.linalg.norm(gl[b]) <= 1e-11
    scale = max(np.abs(c0.lam[k]).max() for k in range(prob.Nt + 1))
    _, _, c00 = O.grape_eval(prob.A0, prob.A, u[0], prob.x0, prob.x_target, prob.n, order=3)
    for lam, k in zip(lr, (0, prob.Nt // 2, prob.Nt)):
        assert np.abs(lam - c00.lam[k]).max() <= 1e-12 * scale, k


@pytest.mark.parametrize("poly", ["taylor", "chebyshev"])
def test_rot_chains_polynomials_and_penalty(built_lib, monkeypatch, poly):
    """Taylor and Chebyshev terms (QOC_TCHAIN_POLY), with a state penalty (the backward adds 2 mu x_k after each
    slice: the register state and the LDS mirror must both see it)."""
    from qoc_amd import systems
    monkeypatch.setenv("QOC_TCHAIN_POLY", poly)
    prob = systems.zz_problem(40, tgate=4.0)
    u = systems.zz_controls(2, 40, 4.0, seed=54)
    qb = systems.QuantumBasis([3, 3])
    pen = (qb(["20", "21", "22"]), [0, 1, 2, 3], 0.37)
    J, g, info, _ = _run(prob, u, True, penalty=pen, monkeypatch=monkeypatch)
    assert info["chain_kernel"] == "mfma_regs"
    assert info["chain_poly"] == poly
    for b in range(2):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, penalty=pen)
        assert abs(J[b] - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10


def test_rot_chains_odd_columns_and_one_control(built_lib, monkeypatch):
    """m = 3 (a half-empty column pair) and nu = 1 (no Ã_2 in LDS) on the register-resident chains."""
    from qoc_amd import GrapeEngine, systems
    monkeypatch.setenv("QOC_TCHAIN_ROT", "1")
    p = systems.zz_problem(50, tgate=5.0)
    A = p.A[:1]
    x0 = p.x0[:, :3]
    xt = p.x_target[:, :3]
    u = systems.zz_controls(2, 50, 5.0, seed=55)[:, :1, :]
    e = GrapeEngine(p.A0, A, x0, p.Nt, B=2)
    e.set_cost_trace(xt, 3)
    e.set_chain("taylor")
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    assert e.info()["chain_kernel"] == "mfma_regs"
    e.close()
    for b in range(2):
        Jr, gr, _ = O.grape_eval(p.A0, A, u[b], x0, xt, 3, order=3)
        assert abs(J[b] - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10


@pytest.mark.parametrize("ncav", [20, 17])
def test_rot3_chains_cavity(built_lib, monkeypatch, ncav):
    """G = 3 (N = 40 and 34, generators in LDS; QOC_TCHAIN_ROT=3) against the oracle and the LDS-state kernels, through
    propagate + grape_sensitivity and the concurrent device eval."""
    from qoc_amd import GrapeEngine, systems
    prob = systems.cavity_problem(N_cavity=ncav, Nt=40)
    u = systems.cavity_controls(2, prob.Nt, seed=59)
    res = {}
    for rot in ("3", "0"):
        monkeypatch.setenv("QOC_TCHAIN_ROT", rot)
        for device in (False, True):
            e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2)
            e.set_cost_trace(prob.x_target, prob.n)
            e.set_chain("taylor")
            if device:
                import torch
                ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
                Jd = torch.empty(2, dtype=torch.float64, device="cuda")
                gd = torch.empty(2, prob.Nt, 2, dtype=torch.float64, device="cuda")
                e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
                e.synchronize()
                J, g = Jd.cpu().numpy(), np.transpose(gd.cpu().numpy(), (0, 2, 1))
            else:
                J = e.propagate(u)
                g = e.grape_sensitivity(u, 3)
            res[rot, device] = (J, g, e.info()["chain_kernel"])
            e.close()
    assert res["3", False][2] == "mfma_regs" and res["0", False][2] == "mfma_lds"
    for b in range(2):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        for key, (J, g, _) in res.items():
            assert abs(J[b] - J0) <= 1e-12, (key, b)
            assert np.linalg.norm(g[b] - g0) / np.linalg.norm(g0) <= 1e-10, (key, b)
