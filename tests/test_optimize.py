"""Batched multi-start optimiser (qoc_amd.optimize) on analytic problems, and the spline
constraint callbacks against the oracle restatement (examples/ipopt_callbacks_exp.jl:33-51).
CPU only: the optimiser is generic over fg / cons callables."""
import numpy as np
import pytest
import torch

import qoc_oracle as O
from qoc_amd.optimize import minimize_batched, spline_constraints_torch

torch.set_default_dtype(torch.float64)


def test_bounded_quadratic_reaches_kkt_point():
    torch.manual_seed(0)
    B, n = 6, 5
    Q = torch.randn(B, n, n)
    Q = Q @ Q.transpose(1, 2) + n * torch.eye(n)
    b = torch.randn(B, n) * 3

    def fg(x):
        r = torch.einsum("bij,bj->bi", Q, x)
        return 0.5 * (x * r).sum(1) - (b * x).sum(1), r - b
    res = minimize_batched(fg, torch.zeros(B, n), -0.5, 0.5, max_iter=200)
    assert bool(res.converged.all())
    f, g = fg(res.c)
    x = res.c
    free = ~(((x <= -0.5) & (g > 0)) | ((x >= 0.5) & (g < 0)))
    assert float((g * free).abs().max()) < 1e-8
    assert float(x.abs().max()) <= 0.5


def test_rosenbrock_multistart_lockstep():
    def rosen(x):
        a, c = x[:, 0], x[:, 1]
        f = (1 - a) ** 2 + 100 * (c - a * a) ** 2
        return f, torch.stack([-2 * (1 - a) - 400 * a * (c - a * a), 200 * (c - a * a)], 1)
    x0 = torch.tensor([[-1.2, 1.0], [0.0, 0.0], [2.0, 2.0], [-0.5, 2.5]])
    r = minimize_batched(rosen, x0, max_iter=300)
    assert torch.allclose(r.c, torch.ones_like(r.c), atol=1e-6)
    assert len(r.history) >= 1 and r.history[-1].shape == (4,)


def test_norm_constraint_augmented_lagrangian():
    cc = torch.tensor([[3.0, 4.0, 0.0], [0.1, 0.2, 0.3]])

    def fq(x):
        return ((x - cc) ** 2).sum(1), 2 * (x - cc)

    def cons(x):
        nrm = x.norm(dim=1, keepdim=True)
        return nrm, (x / nrm.clamp_min(1e-300))[:, None, :]
    r = minimize_batched(fq, torch.zeros_like(cc), cons=cons, g_upper=[1.0], max_iter=100, outer_iters=8)
    assert torch.allclose(r.c[0], torch.tensor([0.6, 0.8, 0.0]), atol=1e-5)   # active: on the sphere
    assert torch.allclose(r.c[1], cc[1], atol=1e-6)                          # inactive
    assert abs(float(r.lam[0, 0]) - 8.0) < 1e-3 and float(r.lam[1, 0]) == 0.0


@pytest.mark.parametrize("ns,nu", [(10, 2), (7, 1), (1, 3)])
def test_spline_constraints_match_oracle(ns, nu):
    rng = np.random.default_rng(ns + nu)
    c = rng.standard_normal((4, ns * nu))
    g, J = spline_constraints_torch(torch.from_numpy(c), ns, nu)
    for b in range(4):
        gr, Jr = O.spline_constraints(c[b], ns)
        np.testing.assert_allclose(g[b].numpy(), gr, rtol=1e-14, atol=1e-15)
        np.testing.assert_allclose(J[b].numpy(), Jr, rtol=1e-13, atol=1e-15)
    # zero vector: zero rows, no NaN
    g0, J0 = spline_constraints_torch(torch.zeros(1, ns * nu), ns, nu)
    assert float(g0.abs().max()) == 0.0 and bool(torch.isfinite(J0).all())


def test_oracle_spline_gradient_matches_finite_differences():
    from qoc_amd import systems
    prob = systems.zz_problem(20, tgate=2.0)
    Bs = systems.spline_matrix(2.0, 20, 5)
    rng = np.random.default_rng(3)
    c = 0.3 * rng.standard_normal(10)
    J, g = O.spline_eval(prob.A0, prob.A, Bs, c, prob.x0, prob.x_target, prob.n, order=4)
    # the Taylor order-4 gradient is close to the true derivative at this small slice norm
    eps = 1e-6
    fd = np.array([(O.spline_eval(prob.A0, prob.A, Bs, c + eps * e, prob.x0, prob.x_target, prob.n)[0] -
                    O.spline_eval(prob.A0, prob.A, Bs, c - eps * e, prob.x0, prob.x_target, prob.n)[0]) / (2 * eps)
                   for e in np.eye(10)])
    assert np.linalg.norm(g - fd) / np.linalg.norm(fd) < 1e-3
