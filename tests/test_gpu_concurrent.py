"""The captured-product gradient and the concurrent μ recurrence (csrc/qoc_tchain.hpp, csrc/qoc_grad_rr.hpp
k_grad_rr_c) against the oracle at the fp64 bar.

* Captured products: the register-resident MFMA chains write their first two products of every slice, which are the
  order-3 gradient's A_k x_k, A_k^2 x_k (forward) and A_k^H λ_{k+1}, (A_k^H)^2 λ_{k+1} (backward) up to the exact
  scalar shift and scale; the gradient then runs only the 3 nu contractions (the reference's expm_jacobian! +
  _compute_u_sensitivity, src/gradient_computations.jl:61-74,177-223).  Default for propagate + grape_sensitivity.
* Concurrent eval (qoc_eval_dev, built-in cost, no penalty / co-state source): λ_{Nt} = coef ⊙ X_target
  (src/penalty_fcns.jl:19-22, 35-40), so λ_k = coef ⊙ μ_k with μ_k = U_k^H .. U_{Nt-1}^H X_target; the μ recurrence
  runs beside the forward chain and the contraction applies coef.

Tolerances: |ΔJ| <= 1e-12, ||ΔdJdu|| / ||dJdu|| <= 1e-10 per seed; co-states 1e-12 relative to max|λ|.
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _dense_chains(monkeypatch):
    """These kernels are the dense Taylor-action chains: the block path (qoc_blk.hpp) stays off."""
    monkeypatch.setenv("QOC_BLOCKS", "0")

def _problems():
    from qoc_amd import systems
    out = {}
    p = systems.cavity_problem(N_cavity=20, Nt=96)
    out["cavity40"] = (p, systems.cavity_controls(3, p.Nt, seed=41))
    p = systems.cavity_problem(N_cavity=8, Nt=70)
    out["cavity16"] = (p, systems.cavity_controls(5, p.Nt, seed=42))
    p = systems.zz_problem(80, tgate=8.0)
    out["zz"] = (p, systems.zz_controls(4, 80, 8.0, seed=43))
    p = systems.tunable_bus_problem(Nt=64, tgate=350.0 * 64 / 2000)
    out["tunable_bus"] = (p, systems.tunable_bus_controls(3, p.Nt, seed=44))
    return out


def _device_eval(e, u):
    import torch
    B, nu, Nt = u.shape
    ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
    Jd = torch.empty(B, dtype=torch.float64, device="cuda")
    gd = torch.empty(B, Nt, nu, dtype=torch.float64, device="cuda")
    e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
    e.synchronize()
    return Jd.cpu().numpy(), np.transpose(gd.cpu().numpy(), (0, 2, 1))


@pytest.mark.parametrize("name", ["cavity40", "cavity16", "zz", "tunable_bus"])
def test_concurrent_eval_matches_oracle(built_lib, name):
    from qoc_amd import GrapeEngine
    prob, u = _problems()[name]
    B = u.shape[0]
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_chain("taylor")
    J, g = _device_eval(e, u)
    assert e.info()["backward"] == "concurrent"
    for b in range(B):
        Jr, gr, cr = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J[b] - Jr) <= 1e-12, (b, J[b], Jr)
        rel = np.linalg.norm(g[b] - gr) / np.linalg.norm(gr)
        assert rel <= 1e-10, (name, b, rel)
        scale = max(np.abs(cr.lam[k]).max() for k in range(prob.Nt + 1))
        for k in (0, 1, prob.Nt // 2, prob.Nt):  # co-states: coef applied to μ on the way out
            assert np.abs(e.costate(k, seed=b) - cr.lam[k]).max() <= 1e-12 * scale, (b, k)
    e.close()


@pytest.mark.parametrize("name", ["cavity40", "zz", "tunable_bus"])
def test_captured_products_equal_generic_gradient(built_lib, monkeypatch, name):
    """propagate + grape_sensitivity: the captured-product gradient (default) against QOC_CAPTURE=0 (k_grad_rr_q/p)
    and the concurrent eval against the sequential one, all at the fp64 bar; forward results bitwise equal."""
    from qoc_amd import GrapeEngine
    prob, u = _problems()[name]
    B = u.shape[0]
    res = {}
    for cap in ("1", "0"):
        monkeypatch.setenv("QOC_CAPTURE", cap)
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
        e.set_cost_trace(prob.x_target, prob.n)
        e.set_chain("taylor")
        J = e.propagate(u)
        g = e.grape_sensitivity(u, 3)
        res[cap] = (J, g, e.info()["backward"], e.info()["fwd_captured"])
        Jd, gd = _device_eval(e, u)
        res[cap + "d"] = (Jd, gd, e.info()["backward"])
        e.close()
    assert res["1"][2] == "captured" and res["1"][3]
    assert res["0"][2] == "generic" and not res["0"][3]
    assert res["1d"][2] == "concurrent" and res["0d"][2] == "generic"
    # P >= 2 per slice with captures (prm.pmin): a slice whose tail bound chose P = 1 gets one more exact term, so the
    # forward results agree to rounding rather than bitwise across the two settings
    np.testing.assert_allclose(res["1"][0], res["0"][0], rtol=0, atol=1e-14)
    assert np.array_equal(res["1"][0], res["1d"][0])
    for key in ("1", "1d", "0d"):
        for b in range(B):
            rel = np.linalg.norm(res[key][1][b] - res["0"][1][b]) / np.linalg.norm(res["0"][1][b])
            assert rel <= 1e-11, (key, b, rel)


def test_concurrent_eval_zcalibrated(built_lib):
    """z-calibrated cost (m = 4): per-column coefficients coef_l = -2F/16 g_l (src/penalty_fcns.jl:35-40)."""
    from qoc_amd import GrapeEngine, systems
    prob = systems.zz_problem(60, tgate=6.0)
    u = systems.zz_controls(3, 60, 6.0, seed=45)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=3)
    e.set_cost_zcalibrated(prob.x_target)
    e.set_chain("taylor")
    J, g = _device_eval(e, u)
    assert e.info()["backward"] == "concurrent"
    Jz, _ = O.setup_infidelity_zcalibrated(prob.x_target)
    for b in range(3):
        xN = O.propagate(prob.A0, prob.A, u[b], prob.x0)[-1]
        assert abs(J[b] - Jz(xN)) <= 1e-12
        res, dth = O.zcal_gradient_match(g[b], prob.A0, prob.A, u[b], prob.x0, prob.x_target, order=3)
        bound = O.zcal_dtheta_bound(prob.x_target, xN)  # see test_gpu_parity.test_zcalibrated_cost
        assert res <= 1e-10 and abs(dth) <= bound, (b, res, dth, bound)
    e.close()


def test_concurrent_eval_falls_back_with_penalty_and_source(built_lib):
    """A state penalty or a co-state source makes λ_k depend on the states: the sequential captured backward runs."""
    from qoc_amd import GrapeEngine, systems
    prob = systems.zz_problem(50, tgate=5.0)
    u = systems.zz_controls(2, 50, 5.0, seed=46)
    qb = systems.QuantumBasis([3, 3])
    pen = (qb(["20", "21", "22"]), [0, 1, 2, 3], 0.37)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_chain("taylor")
    e.set_state_penalty(*pen)
    J, g = _device_eval(e, u)
    assert e.info()["backward"] == "captured"
    for b in range(2):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, penalty=pen)
        assert abs(J[b] - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10
    e.close()


def test_concurrent_eval_packed_states(built_lib):
    """compress_states packing (src/utils.jl:96-109): per-row-sector coefficients in the μ mode."""
    from test_gpu_compress import _block_problem
    from qoc_amd import GrapeEngine
    prob, v, u = _block_problem(N=16, Nt=90, seed=47)
    for zcal in (False, True):
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=u.shape[0])
        e.set_compression(v)
        if zcal:
            e.set_cost_zcalibrated(prob.x_target)
        else:
            e.set_cost_trace(prob.x_target, prob.n)
        e.set_chain("taylor")
        J, g = _device_eval(e, u)
        assert e.info()["backward"] == "concurrent" and e.info()["kernel_m"] == 2
        cost = O.setup_infidelity_zcalibrated(prob.x_target) if zcal else None
        for b in range(u.shape[0]):
            Jr, gr, cr = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, cost=cost)
            assert abs(J[b] - Jr) <= 1e-12
            if zcal:
                res, dth = O.zcal_gradient_match(g[b], prob.A0, prob.A, u[b], prob.x0, prob.x_target, order=3)
                bound = O.zcal_dtheta_bound(prob.x_target, O.propagate(prob.A0, prob.A, u[b], prob.x0)[-1])
                assert res <= 1e-10 and abs(dth) <= bound, (b, res, dth, bound)
            else:
                assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10
                scale = np.abs(cr.lam[prob.Nt]).max()
                assert np.abs(e.costate(3, seed=b) - cr.lam[3]).max() <= 1e-12 * scale
        e.close()
