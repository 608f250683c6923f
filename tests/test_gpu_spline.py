"""GPU: spline-parameterised callbacks (examples/ipopt_callbacks_exp.jl:11-51) through the C ABI vs the
oracle restatement, and the batched multi-start optimiser driving the engine vs the same optimiser
driven by the oracle (parity of the iterates, fp64 tolerances)."""
import numpy as np
import pytest
import torch

import qoc_oracle as O

pytestmark = pytest.mark.gpu


def _zz(Nt=100, ns=10):
    from qoc_amd import systems
    prob = systems.zz_problem(Nt)
    Bs = systems.spline_matrix(10.0, Nt, ns)
    return prob, Bs


def test_eval_spline_matches_oracle(built_lib):
    from qoc_amd import GrapeEngine
    prob, Bs = _zz()
    ns = Bs.shape[1]
    rng = np.random.default_rng(0)
    c = 0.2 * rng.standard_normal((3, ns * 2))
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=3)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_spline_basis(Bs)
    J, g = e.eval_spline(c.reshape(3, 2, ns).transpose(0, 2, 1))
    for b in range(3):
        Jr, gr = O.spline_eval(prob.A0, prob.A, Bs, c[b], prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J[b] - Jr) < 1e-12
        gb = g[b].ravel(order="F")
        assert np.linalg.norm(gb - gr) / np.linalg.norm(gr) < 1e-10
    # device path + constraints
    dev = torch.device("cuda", 0)
    cd = torch.from_numpy(c).to(dev)
    Jd = torch.empty(3, dtype=torch.float64, device=dev)
    gd = torch.empty(3, ns * 2, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    e.eval_spline_device(cd.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
    gv = torch.empty(3, 2, dtype=torch.float64, device=dev)
    gj = torch.empty(3, 2, ns * 2, dtype=torch.float64, device=dev)
    e.spline_constraints_device(cd.data_ptr(), gv.data_ptr(), gj.data_ptr())
    e.synchronize()
    np.testing.assert_allclose(Jd.cpu().numpy(), J, rtol=0, atol=1e-14)
    for b in range(3):
        np.testing.assert_allclose(gd[b].cpu().numpy(), g[b].ravel(order="F"), rtol=1e-12, atol=1e-16)
        gr, Jr = O.spline_constraints(c[b], ns)
        np.testing.assert_allclose(gv[b].cpu().numpy(), gr, rtol=1e-14)
        np.testing.assert_allclose(gj[b].cpu().numpy(), Jr, rtol=1e-13, atol=1e-16)
    e.close()


def test_f_alone_then_f_grad_like_the_reference_callbacks(built_lib):
    """Ipopt's f only propagates (examples/ipopt_callbacks_exp.jl:11-19) and f_grad runs the sensitivity for the
    coefficients f last saw (:21-31): qoc_propagate_spline + qoc_sensitivity_spline give the fused eval's J and dJdc
    (to rounding); the sensitivity refuses other coefficients (the reference's stale-u error)."""
    from qoc_amd import GrapeEngine, StaleCacheError
    prob, Bs = _zz()
    ns = Bs.shape[1]
    rng = np.random.default_rng(3)
    c = (0.2 * rng.standard_normal((2, ns * 2))).reshape(2, 2, ns).transpose(0, 2, 1)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_spline_basis(Bs)
    J0, g0 = e.eval_spline(c)
    J1 = e.propagate_spline(c)
    # the fused eval (the segmented block eval: segment products, prefix scan) and the sequential forward chain of
    # propagate: the same J to rounding
    assert np.abs(J0 - J1).max() <= 1e-13
    g1 = e.sensitivity_spline(c)
    # the fused eval runs the co-state recurrence beside the forward chain (λ = coef ⊙ μ), the split calls after it:
    # the same gradient to rounding
    for b in range(2):
        assert np.linalg.norm(g1[b] - g0[b]) / np.linalg.norm(g0[b]) <= 1e-12
    with pytest.raises(StaleCacheError, match="Cache data from other control signal u"):
        e.sensitivity_spline(c * 1.001)
    e.propagate_spline(c * 1.001)  # a line-search f: no sensitivity
    e.sensitivity_spline(c * 1.001)
    # a new basis with the same number of splines: the states belong to the old basis' u, so the sensitivity for the
    # same coefficients is stale too
    e.propagate_spline(c)
    e.set_spline_basis(Bs * 0.5)
    with pytest.raises(StaleCacheError, match="Cache data from other control signal u"):
        e.sensitivity_spline(c)
    e.close()


def test_multistart_optimiser_parity_with_oracle_driven_run(built_lib):
    from qoc_amd import GrapeEngine
    from qoc_amd.optimize import SplineGrape, minimize_batched, spline_constraints_torch
    prob, Bs = _zz(Nt=60, ns=8)
    ns, B = Bs.shape[1], 3
    rng = np.random.default_rng(1)
    c0 = np.concatenate([0.01 * np.ones((B, ns)), np.zeros((B, ns))], 1) + 0.01 * rng.standard_normal((B, 2 * ns))
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    sg = SplineGrape(e, Bs)
    bound = 2 * np.pi * 0.060
    kw = dict(lower=-bound, upper=bound, g_upper=[2.0, 1.0], max_iter=12, outer_iters=1)
    r_gpu = minimize_batched(sg.fg, torch.from_numpy(c0).cuda(), cons=sg.cons, **kw)

    def fg_cpu(c):
        out = [O.spline_eval(prob.A0, prob.A, Bs, ci, prob.x0, prob.x_target, prob.n) for ci in c.numpy()]
        return torch.tensor([o[0] for o in out], dtype=torch.float64), torch.from_numpy(np.stack([o[1] for o in out]))
    r_cpu = minimize_batched(fg_cpu, torch.from_numpy(c0), cons=lambda c: spline_constraints_torch(c, ns, 2), **kw)
    assert r_gpu.n_evals == r_cpu.n_evals
    np.testing.assert_allclose(r_gpu.c.cpu().numpy(), r_cpu.c.numpy(), rtol=0, atol=1e-8)
    np.testing.assert_allclose(r_gpu.f.cpu().numpy(), r_cpu.f.numpy(), rtol=0, atol=1e-10)
    assert float(r_gpu.f.max()) < float(r_gpu.history[0].min())
    e.close()


def test_reference_example_settings_converge(built_lib):
    """examples/zz_coupling_ipopt_exp.jl settings (NOT gate, 100 slices, 10 splines, |c| <= 2pi*0.06,
    g_U = [2, 1]) from 8 perturbed starts: every seed improves and the constraints hold."""
    from qoc_amd import GrapeEngine
    from qoc_amd.optimize import SplineGrape, minimize_batched
    prob, Bs = _zz()
    ns, B = Bs.shape[1], 8
    rng = np.random.default_rng(2)
    c0 = np.concatenate([0.01 * np.ones((B, ns)), np.zeros((B, ns))], 1) + 0.02 * rng.standard_normal((B, 2 * ns))
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    sg = SplineGrape(e, Bs)
    bound = 2 * np.pi * 0.060
    r = minimize_batched(sg.fg, torch.from_numpy(c0).cuda(), lower=-bound, upper=bound, cons=sg.cons,
                         g_upper=[2.0, 1.0], max_iter=60, outer_iters=2)
    f0 = r.history[0]
    assert np.all(r.f.cpu().numpy() < f0)
    assert float(r.f.min()) < 0.1 * float(f0.min())
    assert float(r.c.abs().max()) <= bound + 1e-12
    assert float((r.g - torch.tensor([2.0, 1.0], device=r.g.device)).max()) < 1e-3
    e.close()
