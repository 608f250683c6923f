"""Batched multi-start optimiser over the spline coefficients — the caller of the batch axis
 and the stand-in for Ipopt in examples/zz_coupling_ipopt_exp.jl:56-80
(Ipopt itself is not available in this image).

B independent problems

    min_c  f(c)    s.t.   c_L <= c <= c_U,    g(c) <= g_U,     g(c) = [||c||, ||diff(c, dims=1)||]

advance in lock-step: every line-search trial is ONE batched f + grad evaluation of all seeds on
the GPU (``GrapeEngine.eval_spline_device``: u = transpose(Bs c), propagate, grape_sensitivity,
dJdc = Bs' dJdu').  Bounds are handled by projection (projected L-BFGS, Ipopt's
"hessian_approximation = limited-memory" analogue); the two norm constraints by an augmented
Lagrangian outer loop.  All vector work is batched torch on the engine's device; the optimiser
itself is generic over ``fg`` / ``cons`` callables, so the CPU tests drive it with analytic functions.

Variable layout: c is (B, nc) with nc = ns * nu in Julia's ``c[:]`` order of ``reshape(c, ns, nu)``
(index s + ns * j), which is also the engine's device layout.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


# ---------------------------------------------------------------------------------------------
# Objective / constraints on the engine
# ---------------------------------------------------------------------------------------------
class SplineGrape:
    """f + grad and the norm constraints of the Ipopt callbacks for B seeds on one GPU.

    Mirrors ``setup_ipopt_callbacks`` (examples/ipopt_callbacks_exp.jl:1-54): f(c) = Jfinal(x[end]) +
    sum(L, x) with u = transpose(B c); f_grad = B' transpose(dJdu); g = [norm(c), norm(diff(c))].
    """

    def __init__(self, engine, Bs, order: int = 3):
        import torch
        self.eng = engine
        self.order = order
        engine.set_spline_basis(Bs)
        self.ns, self.nu, self.B = engine.ns, engine.nu, engine.B
        self.nc = self.ns * self.nu
        self.device = torch.device("cuda", engine.device)
        self._J = torch.empty(self.B, dtype=torch.float64, device=self.device)
        self._G = torch.empty(self.B, self.nc, dtype=torch.float64, device=self.device)
        self._g = torch.empty(self.B, 2, dtype=torch.float64, device=self.device)
        self._gj = torch.empty(self.B, 2, self.nc, dtype=torch.float64, device=self.device)
        self.n_evals = 0

    def fg(self, c):
        import torch
        c = c.contiguous()
        torch.cuda.current_stream(self.device).synchronize()  # c produced on torch's stream
        self.eng.eval_spline_device(c.data_ptr(), self.order, self._J.data_ptr(), self._G.data_ptr())
        self.eng.synchronize()
        self.n_evals += 1
        return self._J.clone(), self._G.clone()

    def cons(self, c):
        import torch
        c = c.contiguous()
        torch.cuda.current_stream(self.device).synchronize()
        self.eng.spline_constraints_device(c.data_ptr(), self._g.data_ptr(), self._gj.data_ptr())
        self.eng.synchronize()
        return self._g.clone(), self._gj.clone()


def spline_constraints_torch(c, ns: int, nu: int):
    """Reference (torch) form of g = [norm(c), norm(diff(c, dims=1))] and its Jacobian (B, 2, nc)."""
    import torch
    B = c.shape[0]
    C = c.reshape(B, nu, ns).transpose(1, 2)  # (B, ns, nu) column-major per seed
    g0 = torch.linalg.vector_norm(c, dim=1)
    D = C[:, 1:, :] - C[:, :-1, :]
    g1 = torch.linalg.vector_norm(D.reshape(B, -1), dim=1)
    j0 = torch.where(g0[:, None] > 0, c / g0.clamp_min(1e-300)[:, None], torch.zeros_like(c))
    Dp = torch.zeros(B, ns + 1, nu, dtype=c.dtype, device=c.device)
    Dp[:, 1:ns, :] = D
    J1 = (Dp[:, :ns, :] - Dp[:, 1:, :])  # d_s - d_{s+1}
    j1 = J1.transpose(1, 2).reshape(B, -1)
    j1 = torch.where(g1[:, None] > 0, j1 / g1.clamp_min(1e-300)[:, None], torch.zeros_like(j1))
    return torch.stack([g0, g1], 1), torch.stack([j0, j1], 1)


# ---------------------------------------------------------------------------------------------
# Batched projected L-BFGS with an augmented-Lagrangian outer loop
# ---------------------------------------------------------------------------------------------
@dataclass
class BatchResult:
    c: object                 # (B, n) final iterates
    f: object                 # (B,) objective f (without constraint terms)
    g: object | None          # (B, ng) constraint values
    lam: object | None        # (B, ng) multipliers
    history: list = field(default_factory=list)   # per outer/inner iteration: f (B,) as numpy
    n_evals: int = 0
    converged: object = None  # (B,) bool


def _two_loop(q, S, Y, rho, valid, head, m):
    """H q for every seed from its L-BFGS pairs; S, Y (B, m, n), rho (B, m), valid (B, m) bool."""
    import torch
    B = q.shape[0]
    alpha = torch.zeros(B, m, dtype=q.dtype, device=q.device)
    q = q.clone()
    order = [(head - 1 - i) % m for i in range(m)]  # newest first
    for i in order:
        a = rho[:, i] * (S[:, i] * q).sum(1)
        a = torch.where(valid[:, i], a, torch.zeros_like(a))
        alpha[:, i] = a
        q = q - a[:, None] * Y[:, i]
    newest = order[0]
    sy = (S[:, newest] * Y[:, newest]).sum(1)
    yy = (Y[:, newest] * Y[:, newest]).sum(1)
    gamma = torch.where(valid[:, newest] & (yy > 0), sy / yy.clamp_min(1e-300), torch.ones_like(sy))
    r = gamma[:, None] * q
    for i in reversed(order):
        b = rho[:, i] * (Y[:, i] * r).sum(1)
        b = torch.where(valid[:, i], b, torch.zeros_like(b))
        r = r + (alpha[:, i] - b)[:, None] * S[:, i]
    return r


def minimize_batched(fg, c0, lower=None, upper=None, cons=None, g_upper=None, max_iter: int = 100,
                     memory: int = 10, outer_iters: int = 4, rho0: float = 10.0, gtol: float = 1e-9,
                     max_ls: int = 12, callback=None) -> BatchResult:
    """Minimise B independent problems in lock-step.

    fg(c) -> (f (B,), grad (B, n)); cons(c) -> (g (B, ng), jac (B, ng, n)) with constraints g <= g_upper.
    lower / upper: scalars or (n,) / (B, n) bounds.  max_iter counts inner iterations per outer round.
    """
    import torch
    x = c0.clone().to(torch.float64)
    B, n = x.shape
    dev = x.device
    lo = torch.full_like(x, -np.inf) if lower is None else torch.as_tensor(lower, dtype=x.dtype, device=dev).expand(B, n)
    hi = torch.full_like(x, np.inf) if upper is None else torch.as_tensor(upper, dtype=x.dtype, device=dev).expand(B, n)
    x = torch.minimum(torch.maximum(x, lo), hi)
    ng = 0
    if cons is not None:
        gu = torch.as_tensor(g_upper, dtype=x.dtype, device=dev).expand(B, -1)
        ng = gu.shape[1]
        lam = torch.zeros(B, ng, dtype=x.dtype, device=dev)
        rho = torch.full((B,), rho0, dtype=x.dtype, device=dev)
    evals = 0
    history = []

    def phi(xc):
        nonlocal evals
        f, gr = fg(xc)
        evals += 1
        if cons is None:
            return f, gr, f, None
        gv, gj = cons(xc)
        t = gv - gu
        a = torch.clamp(lam + rho[:, None] * t, min=0.0)
        pen = ((a * a) - lam * lam).sum(1) / (2 * rho)
        return f + pen, gr + torch.einsum("bi,bin->bn", a, gj), f, gv

    converged = torch.zeros(B, dtype=torch.bool, device=dev)
    fx = gxv = None
    for it_outer in range(max(1, outer_iters if cons is not None else 1)):
        fx, gx, f_true, gval = phi(x)
        S = torch.zeros(B, memory, n, dtype=x.dtype, device=dev)
        Y = torch.zeros_like(S)
        rh = torch.zeros(B, memory, dtype=x.dtype, device=dev)
        valid = torch.zeros(B, memory, dtype=torch.bool, device=dev)
        head = 0
        for it in range(max_iter):
            free = ~(((x <= lo) & (gx > 0)) | ((x >= hi) & (gx < 0)))
            q = gx * free
            pgn = q.abs().amax(1)
            converged = pgn <= gtol
            if bool(converged.all()):
                break
            d = -_two_loop(q, S, Y, rh, valid, head, memory) * free
            desc = (d * gx).sum(1)
            bad = ~(desc < 0)
            d = torch.where(bad[:, None], -q, d)
            valid = valid & ~bad[:, None]
            # first step of a fresh history: scaled steepest descent
            fresh = ~valid.any(1)
            step0 = torch.where(fresh, 1.0 / q.abs().amax(1).clamp_min(1e-12), torch.ones_like(pgn)).clamp(max=1.0)
            alpha = step0.clone()
            acc = converged.clone()
            x_new, f_new, g_new, ft_new, gv_new = x.clone(), fx.clone(), gx.clone(), f_true.clone(), gval
            for _ in range(max_ls):
                xt = torch.minimum(torch.maximum(x + alpha[:, None] * d, lo), hi)
                ft, gt, ftt, gvt = phi(xt)
                ok = (ft <= fx + 1e-4 * (gx * (xt - x)).sum(1)) & torch.isfinite(ft) & ~acc
                x_new = torch.where(ok[:, None], xt, x_new)
                f_new = torch.where(ok, ft, f_new)
                g_new = torch.where(ok[:, None], gt, g_new)
                ft_new = torch.where(ok, ftt, ft_new)
                if gvt is not None:
                    gv_new = torch.where(ok[:, None], gvt, gv_new)
                acc = acc | ok
                if bool(acc.all()):
                    break
                alpha = torch.where(acc, alpha, alpha * 0.5)
            s = x_new - x
            yv = g_new - gx
            sy = (s * yv).sum(1)
            upd = acc & ~converged & (sy > 1e-12 * s.norm(dim=1) * yv.norm(dim=1))
            S[:, head] = torch.where(upd[:, None], s, S[:, head])
            Y[:, head] = torch.where(upd[:, None], yv, Y[:, head])
            rh[:, head] = torch.where(upd, 1.0 / sy.where(upd, torch.ones_like(sy)), rh[:, head])
            valid[:, head] = torch.where(upd, torch.ones_like(upd), valid[:, head] & ~acc)
            head = (head + 1) % memory
            # seeds whose line search failed restart from steepest descent
            valid = valid & acc[:, None]
            x, fx, gx, f_true, gval = x_new, f_new, g_new, ft_new, gv_new
            history.append(f_true.detach().cpu().numpy().copy())
            if callback is not None:
                callback(it_outer, it, x, f_true)
        if cons is None:
            break
        t = gval - gu
        viol = t.clamp(min=0).amax(1)
        lam = torch.clamp(lam + rho[:, None] * t, min=0.0)
        if it_outer > 0:
            rho = torch.where(viol > 0.25 * prev_viol, rho * 10.0, rho)
        prev_viol = viol
    return BatchResult(c=x, f=f_true, g=gval, lam=lam if cons is not None else None, history=history,
                       n_evals=evals, converged=converged)
