"""numpy emulation of k_blkp_exp's exponential (csrc/qoc_blkp.hpp) on the tunable bus' live 14-row block, to study
the bias of the stored-propagator path against an extended-precision propagation (tools/tb_truth.py) for different
(degree, squarings) policies and product forms, without a GPU.

  python tools/blkp_emulate.py [seeds]
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "quantumoptimalcontrol.jl_amd"))
sys.path.insert(0, HERE)
from qoc_amd import systems  # noqa: E402

INVF = np.array([1.0 / math.factorial(k) for k in range(40)])


def tailsum(rho, m):
    t = math.exp((m + 1) * math.log(rho) - math.lgamma(m + 2))
    s = 0.0
    for k in range(m + 1, m + 41):
        s += t
        t *= rho / (k + 1)
    return s


def theta(m, tol):
    lo, hi = 0.0, 16.0
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if tailsum(mid, m) <= tol:
            lo = mid
        else:
            hi = mid
    return lo


def cmul(L, R, four=False):
    if four:
        return (L.real @ R.real - L.imag @ R.imag) + 1j * (L.real @ R.imag + L.imag @ R.real)
    t1 = L.real @ R.real
    t2 = L.imag @ R.imag
    t3 = (L.real + L.imag) @ (R.real + R.imag)
    return (t1 - t2) + 1j * (t3 - t1 - t2)


def expm_ps(X, r, s, four=False):
    n = X.shape[0]
    X = X * 2.0 ** -s
    X2 = cmul(X, X, four)
    X3 = cmul(X, X2, four)
    X4 = cmul(X, X3, four)
    I = np.eye(n)

    def Bi(i):
        return INVF[4 * i] * I + INVF[4 * i + 1] * X + INVF[4 * i + 2] * X2 + INVF[4 * i + 3] * X3
    R = Bi(r - 1) + INVF[4 * r] * X4
    for i in range(r - 2, -1, -1):
        R = cmul(X4, R, four) + Bi(i)
    for _ in range(s):
        R = cmul(R, R, four)
    return R


def choose(rho, policy):
    rmin, rmax = 2, 8
    kind, slack, tail = policy
    ssel = {}
    for r in range(rmin, rmax + 1):
        if tail is None:
            th = theta(4 * r, 2.0 ** -53)
            sq = max(0, math.ceil(math.log2(rho / th))) if rho > th else 0
        else:
            sq = 0
            q = rho
            while sq < 15 and q > theta(4 * r, 2.0 ** (-53 - sq - tail)):
                q *= 0.5
                sq += 1
        ssel[r] = sq
    best = min(r + 2 + ssel[r] for r in ssel)
    if kind == "fixed_s":
        # `slack` squarings (at least), the smallest degree that meets the tail criterion there
        for r in range(rmin, rmax + 1):
            if ssel[r] <= slack:
                return r, slack
        return rmax, ssel[rmax]
    rs, ss = 8, 99
    for r in range(rmax, rmin - 1, -1):
        if r + 2 + ssel[r] <= best + slack and ssel[r] < ss:
            ss, rs = ssel[r], r
    return rs, ss


def shift(A):
    """the engine's shift (qoc_engine.hip choose_shift): 0, the trace mean or the diagonal's midrange, whichever
    gives the smallest shifted 1-norm"""
    d = A.diagonal()
    off = np.abs(A).sum(axis=0) - np.abs(d)
    cands = [0.0, d.mean(), 0.5 * (d.real.min() + d.real.max()) + 0.5j * (d.imag.min() + d.imag.max())]
    return min(cands, key=lambda c: np.max(off + np.abs(d - c)))


def live_block(prob):
    M = np.abs(prob.A0) > 0
    for a in prob.A:
        M |= np.abs(a) > 0
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import connected_components
    _, lab = connected_components(csr_matrix(M), directed=False)
    live = lab[np.flatnonzero(np.abs(prob.x0[:, 0]) > 0)[0]]
    return np.flatnonzero(lab == live)


def J_emul(prob, u, policy, four=False, cache=None):
    rows = live_block(prob)
    A0 = prob.A0[np.ix_(rows, rows)]
    A1 = prob.A[0][np.ix_(rows, rows)]
    mu0, mu1 = shift(prob.A0), shift(prob.A[0])
    At0 = A0 - mu0 * np.eye(len(rows))
    At1 = A1 - mu1 * np.eye(len(rows))
    x = prob.x0[rows, 0].astype(complex)
    prods = 0
    for k in range(prob.Nt):
        X = At0 + u[0, k] * At1
        az = np.abs(X.real) + np.abs(X.imag)
        rho = math.sqrt(az.sum(axis=0).max() * az.sum(axis=1).max())
        r, s = choose(rho, policy)
        prods += r + 2 + s
        U = expm_ps(X, r, s, four) * np.exp(mu0 + u[0, k] * mu1)
        x = U @ x
    ov = np.vdot(prob.x_target[rows, 0], x)
    return 1.0 - abs(ov) ** 2 / prob.n ** 2, prods / prob.Nt


def main():
    import tb_truth as T
    nseeds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    mk_prob, mk_u, B = systems.CONFIGS["tunable_bus"]
    prob = mk_prob()
    us = [mk_u(B, 1)[b] for b in range(nseeds // 2)] + [mk_u(B, 3)[b] for b in range(nseeds - nseeds // 2)]
    from concurrent.futures import ProcessPoolExecutor
    with ProcessPoolExecutor(8) as ex:
        truth = list(ex.map(T.J_ld, [prob] * nseeds, us))
    policies = {
        "default(slack1)": (("prod", 1, None), False),
        "s2": (("fixed_s", 2, 3), False),
        "s3": (("fixed_s", 3, 3), False),
        "s4": (("fixed_s", 4, 3), False),
        "s5": (("fixed_s", 5, 3), False),
        "s6": (("fixed_s", 6, 3), False),
        "s3_4m": (("fixed_s", 3, 3), True),
        "s4_4m": (("fixed_s", 4, 3), True),
        "s5_4m": (("fixed_s", 5, 3), True),
    }
    for name, (pol, four) in policies.items():
        with ProcessPoolExecutor(8) as ex:
            res = list(ex.map(J_emul, [prob] * nseeds, us, [pol] * nseeds, [four] * nseeds))
        errs = np.array([float(np.float64(J - t)) for (J, _), t in zip(res, truth)])
        print(f"{name:18s} products {res[0][1]:.3f}  err {' '.join(f'{e:+.2e}' for e in errs)}", flush=True)


if __name__ == "__main__":
    main()
