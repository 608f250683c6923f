"""The segmented block eval (csrc/qoc_blkseg.hpp, qoc_eval_dev's default for generators with invariant blocks of <= 3
rows): one launch per evaluation, the time axis cut into S segments (segment products, a prefix scan over segments,
then every segment backwards with G_k = Σ_c x_k λ_k^H), against the oracle (the reference's sequential chains:
src/gradient_computations.jl:17-29 forward, :52-58 co-states, :65-74 + :177-223 the gradient) at the fp64 bar of
SURVEY.md §8c: |ΔJ| <= 1e-12, ||ΔdJdu|| / ||dJdu|| <= 1e-10 per seed; states and co-states (rebuilt on demand)
1e-12 relative to their largest entry.
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


def _engine(prob, B, monkeypatch, seg="1", S=None, W=None):
    from qoc_amd import GrapeEngine
    monkeypatch.setenv("QOC_BLOCKS", "1")
    monkeypatch.setenv("QOC_BLKU", "1")
    monkeypatch.setenv("QOC_BLKSEG", seg)
    for k, v in (("QOC_BLKSEG_S", S), ("QOC_BLKSEG_W", W)):
        if v is None:
            monkeypatch.delenv(k, raising=False)
        else:
            monkeypatch.setenv(k, str(v))
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_chain("taylor")
    return e


def _eval_dev(e, u, order=3):
    import torch
    B, nu, Nt = u.shape
    ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
    Jd = torch.empty(B, dtype=torch.float64, device="cuda")
    gd = torch.empty(B, Nt, nu, dtype=torch.float64, device="cuda")
    e.eval_device(ud.data_ptr(), order, Jd.data_ptr(), gd.data_ptr())
    e.synchronize()
    return Jd.cpu().numpy(), np.transpose(gd.cpu().numpy(), (0, 2, 1))


def _assert_seed(J, g, Jr, gr, tag):
    assert abs(J - Jr) <= 1e-12, (tag, J - Jr)
    rel = np.linalg.norm(g - gr) / np.linalg.norm(gr)
    assert rel <= 1e-10, (tag, rel)


def _cases():
    from qoc_amd import systems
    out = {}
    p = systems.zz_problem(60, tgate=6.0)  # N = 9, 3 blocks of 3, m = 4, nu = 2
    out["zz"] = (p, systems.zz_controls(3, 60, 6.0, seed=81))
    p = systems.cavity_problem(N_cavity=10, Nt=50)  # N = 20, 10 blocks of 2, m = 2
    out["cavity20"] = (p, systems.cavity_controls(3, p.Nt, seed=82))
    p = systems.cavity_problem(N_cavity=20, Nt=77)  # N = 40 (the BASELINE system), 20 blocks of 2
    out["cavity40"] = (p, systems.cavity_controls(2, p.Nt, seed=83))
    return out


def _block_problem(NB, nblk, nu, m, Nt, seed):
    """Random skew-Hermitian generators (exactly: -i H dt with H = (G + G^H) / 2) with nblk blocks of NB rows under a
    random permutation, the last block one row short (padding)."""
    from qoc_amd import systems
    rng = np.random.default_rng(seed)
    sizes = [NB] * (nblk - 1) + [NB - 1]
    N = sum(sizes)
    perm = rng.permutation(N)
    gens = []
    for j in range(nu + 1):
        H = np.zeros((N, N), complex)
        o = 0
        for s in sizes:
            G = rng.standard_normal((s, s)) + 1j * rng.standard_normal((s, s))
            H[o:o + s, o:o + s] = (G + G.conj().T) / 2
            o += s
        H = H[np.ix_(perm, perm)]
        gens.append(-1j * H * (0.08 if j == 0 else 0.05))
    x0 = np.linalg.qr(rng.standard_normal((N, m)) + 1j * rng.standard_normal((N, m)))[0]
    xt = np.linalg.qr(rng.standard_normal((N, m)) + 1j * rng.standard_normal((N, m)))[0]
    prob = systems.Problem("blocks", gens[0], gens[1:], x0, xt, float(m), Nt, "fp64")
    u = rng.uniform(-1, 1, size=(2, nu, Nt))
    return prob, u


@pytest.mark.parametrize("name", ["zz", "cavity20", "cavity40"])
def test_segmented_eval_matches_oracle_states_costates(built_lib, monkeypatch, name):
    """J and dJdu against the oracle; the states and co-states, which the launch never writes, rebuilt on demand
    (qoc_get_states / qoc_get_costates) and against the oracle's trajectories."""
    prob, u = _cases()[name]
    B = u.shape[0]
    e = _engine(prob, B, monkeypatch)
    J, g = _eval_dev(e, u)
    info = e.info()
    assert info["backward"] == "segmented" and info["chain_kernel"] == "blocks_prop", info
    ks = (0, 1, prob.Nt // 2, prob.Nt - 1, prob.Nt)
    xs = [e.state(k, seed=B - 1) for k in ks]
    lams = [e.costate(k, seed=B - 1) for k in ks]
    e.close()
    for b in range(B):
        J0, g0, c0 = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (name, b))
    xsc = max(np.abs(x).max() for x in c0.x)
    lsc = max(np.abs(lam).max() for lam in c0.lam)
    for k, x, lam in zip(ks, xs, lams):
        assert np.abs(x - c0.x[k]).max() <= 1e-12 * xsc, ("x", k)
        assert np.abs(lam - c0.lam[k]).max() <= 1e-12 * lsc, ("lambda", k)


@pytest.mark.parametrize("S", [1, 2, 3, 7, 13, 50])
@pytest.mark.parametrize("name", ["zz", "cavity20"])
def test_segment_counts_not_dividing_nt(built_lib, monkeypatch, name, S):
    """Segment counts that do not divide Nt (the last segment shorter), a single segment (no scan), and one slice
    per segment (Nt = 50 / 60 slices)."""
    prob, u = _cases()[name]
    e = _engine(prob, u.shape[0], monkeypatch, S=S)
    J, g = _eval_dev(e, u)
    assert e.info()["backward"] == "segmented"
    e.close()
    for b in range(u.shape[0]):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (name, S, b))


@pytest.mark.parametrize("W", [1, 3, 8])
def test_segmented_waves_per_seed(built_lib, monkeypatch, W):
    """1, 3 or 8 waves per seed (the segment count follows: UPW = 64 / nblk segments per wave)."""
    prob, u = _cases()["cavity40"]
    e = _engine(prob, u.shape[0], monkeypatch, W=W)
    J, g = _eval_dev(e, u)
    e.close()
    for b in range(u.shape[0]):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (W, b))


@pytest.mark.parametrize("order", [1, 2, 3, 4])
@pytest.mark.parametrize("name", ["zz", "cavity20"])
def test_segmented_gradient_orders(built_lib, monkeypatch, name, order):
    """expm_jacobian! orders 1..4 (src/gradient_computations.jl:177-213) in the segmented eval."""
    prob, u = _cases()[name]
    e = _engine(prob, u.shape[0], monkeypatch)
    J, g = _eval_dev(e, u, order)
    assert e.info()["backward"] == "segmented"
    e.close()
    for b in range(u.shape[0]):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=order)
        _assert_seed(J[b], g[b], J0, g0, (name, order, b))


@pytest.mark.parametrize("NB,nblk,nu,m", [(2, 7, 1, 3), (2, 24, 2, 1), (3, 5, 2, 2), (3, 9, 1, 4), (2, 4, 2, 8)])
def test_segmented_random_permuted_blocks(built_lib, monkeypatch, NB, nblk, nu, m):
    """Random permuted blocks of 2 / 3 rows (a short last block: padding rows), one or two controls, 1..8 columns,
    24 blocks (two segments per wave)."""
    prob, u = _block_problem(NB, nblk, nu, m, Nt=45, seed=NB * 100 + nblk + nu + m)
    e = _engine(prob, 2, monkeypatch)
    J, g = _eval_dev(e, u)
    assert e.info()["backward"] == "segmented", e.info()
    x = e.state(prob.Nt, seed=1)
    e.close()
    for b in range(2):
        J0, g0, c0 = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (NB, nblk, nu, m, b))
    assert np.abs(x - c0.x[-1]).max() <= 1e-12


def test_segmented_zcalibrated_cost(built_lib, monkeypatch):
    """The z-calibrated cost (src/penalty_fcns.jl:27-42, src/fidelities.jl:81-137) on the segmented eval: J against
    the oracle's cost of its own x_N, the gradient against the oracle's gradient family g(Δθ) within the calibration
    phase's golden-section bound (tests/test_gpu_parity.py)."""
    from qoc_amd import systems
    prob = systems.zz_problem(40, tgate=4.0)
    u = systems.zz_controls(2, 40, 4.0, seed=86)
    Jz, _ = O.setup_infidelity_zcalibrated(prob.x_target)
    e = _engine(prob, 2, monkeypatch)
    e.set_cost_zcalibrated(prob.x_target)
    J, g = _eval_dev(e, u)
    assert e.info()["backward"] == "segmented"
    e.close()
    for b in range(2):
        xN = O.propagate(prob.A0, prob.A, u[b], prob.x0)[-1]
        assert abs(J[b] - Jz(xN)) <= 1e-12
        res, dth = O.zcal_gradient_match(g[b], prob.A0, prob.A, u[b], prob.x0, prob.x_target, order=3)
        assert res <= 1e-10 and abs(dth) <= O.zcal_dtheta_bound(prob.x_target, xN), (b, res, dth)


def test_segmented_matches_fused_backward(built_lib, monkeypatch):
    """The segmented eval against the forward + fused backward of k_blku_* (QOC_BLKSEG=0) on the same inputs."""
    prob, u = _cases()["cavity40"]
    out = {}
    for seg in ("1", "0"):
        e = _engine(prob, u.shape[0], monkeypatch, seg=seg)
        out[seg] = _eval_dev(e, u)
        out[seg + "i"] = e.info()["backward"]
        e.close()
    assert out["1i"] == "segmented" and out["0i"] == "fused"
    for b in range(u.shape[0]):
        _assert_seed(out["1"][0][b], out["1"][1][b], out["0"][0][b], out["0"][1][b], b)


def test_lazy_states_survive_setters_and_later_calls(built_lib, monkeypatch):
    """x_k / λ_k of a segmented eval are rebuilt on demand from the u and λ_N it left behind: before a setter
    changes the system (here: new generators and a new target) they are materialised, a later grape_sensitivity
    (which reads x_k) rebuilds the states first, and a later propagate leaves the eval's co-states as they were."""
    from qoc_amd import systems
    prob, u = _cases()["cavity20"]
    e = _engine(prob, 3, monkeypatch)
    J, g = _eval_dev(e, u)
    J0, g0, c0 = O.grape_eval(prob.A0, prob.A, u[1], prob.x0, prob.x_target, prob.n, order=3)
    # grape_sensitivity right after the eval: the states are rebuilt, λ recomputed
    g2 = e.grape_sensitivity(u, 3)
    assert np.linalg.norm(g2[1] - g0) / np.linalg.norm(g0) <= 1e-10
    _eval_dev(e, u)
    # a different system: the co-states the eval left must come from the old one (the states are invalidated by the
    # setters, as in qoc_set_generators / qoc_set_cost: "no propagated states")
    p2 = systems.cavity_problem(N_cavity=10, Nt=50, dt=0.7)
    e.set_generators(p2.A0, p2.A)
    e.set_cost_trace(-prob.x_target, prob.n)
    lk = e.costate(prob.Nt // 3, seed=1)
    e.close()
    lsc = max(np.abs(lam).max() for lam in c0.lam)
    assert np.abs(lk - c0.lam[prob.Nt // 3]).max() <= 1e-12 * lsc
    # propagate after the eval: new states, the eval's co-states
    e = _engine(prob, 3, monkeypatch)
    _eval_dev(e, u)
    u2 = u * 0.5
    e.propagate(u2)
    lk = e.costate(5, seed=1)
    xk = e.state(5, seed=1)
    e.close()
    assert np.abs(lk - c0.lam[5]).max() <= 1e-12 * lsc
    x2 = O.propagate(prob.A0, prob.A, u2[1], prob.x0)[5]
    assert np.abs(xk - x2).max() <= 1e-12


def test_segmented_off_for_inexact_skew_hermitian(built_lib, monkeypatch):
    """Generators skew-Hermitian only to ~1e-14 (within the Chebyshev check, outside the exact one) keep the forward +
    fused backward: the segmented backward relies on exactly unitary slices."""
    import dataclasses
    prob, u = _cases()["cavity20"]
    A0 = prob.A0 + 1e-14 * np.abs(prob.A0).max() * np.eye(prob.N)
    p2 = dataclasses.replace(prob, A0=A0)
    e = _engine(p2, u.shape[0], monkeypatch)
    J, g = _eval_dev(e, u)
    assert e.info()["backward"] == "fused"
    e.close()
    for b in range(u.shape[0]):
        J0, g0, _ = O.grape_eval(p2.A0, p2.A, u[b], p2.x0, p2.x_target, p2.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, b)


@pytest.mark.parametrize("name,B", [("cavity", 256), ("zz_batch", 512)])
def test_segmented_full_size(built_lib, monkeypatch, name, B):
    """BASELINE configs 3 (cavity N=40, Nt=1000, B=256) and 2 (zz N=9, Nt=500, B=512) through qoc_eval_dev, 16 seeds
    against the C port of the reference (oracle/cpu_ref.c, its Padé + solve)."""
    import cpuref
    from qoc_amd import systems
    mk_prob, mk_u, Bd = systems.CONFIGS[name]
    assert Bd == B
    prob = mk_prob()
    u = mk_u(B, 0)
    e = _engine(prob, B, monkeypatch)
    J, g = _eval_dev(e, u)
    assert e.info()["backward"] == "segmented"
    e.close()
    assert np.all(np.isfinite(J)) and np.all(np.isfinite(g))
    idx = np.asarray(list(range(8)) + list(range(B - 8, B)))
    cpuref.use_blas(True)
    Jc, gc = cpuref.grape_eval_batch(prob, u[idx], order=3, mode=0)
    for i, b in enumerate(idx):
        _assert_seed(J[b], g[b], Jc[i], gc[i], (name, b))


def test_segmented_eval_best_pair_for_the_all_gather(built_lib, monkeypatch):
    """The launch's last workgroup reduces the batch's J to the best (J, global seed) for qoc_allgather_best (no
    k_argmin_seed launch): more seeds than CUs (several workgroups per CU), with and without a seed offset, and a later
    propagate (whose J the epilogue reduces again)."""
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=10, Nt=24)
    B = 300
    u = systems.cavity_controls(B, prob.Nt, seed=91) * 6.0  # spread the fidelities
    e = _engine(prob, B, monkeypatch)
    J, _ = _eval_dev(e, u)
    assert e.info()["backward"] == "segmented"
    assert e.allgather_best() == (J.min(), int(np.argmin(J)))
    e.comm_init(1, 0, None, 1000)  # no communicator, seed offset 1000
    J, _ = _eval_dev(e, u[::-1].copy())
    assert e.allgather_best() == (J.min(), 1000 + int(np.argmin(J)))
    J2 = e.propagate(u * 0.5)
    assert e.allgather_best() == (J2.min(), 1000 + int(np.argmin(J2)))
    J, _ = _eval_dev(e, u)
    assert e.allgather_best() == (J.min(), 1000 + int(np.argmin(J)))
    e.close()


@pytest.mark.parametrize("amp", [1.0, 8.0, 14.0, 22.0])
def test_segmented_series_degree_classes(built_lib, monkeypatch, amp):
    """Blocks of 2 rows: the closed-form exponential's series degree is chosen per seed from its largest ρ_k (K = 5 /
    7 / 9 for ρ <= 0.24 / 0.66 / θ_cap; beyond θ_cap the halving path).  The cavity's controls scaled by amp move ρ
    through every class (ρ = 0.154 + 0.05 amp at |u| = 0.05 amp per control); each seed against the oracle."""
    from qoc_amd import systems
    p = systems.cavity_problem(N_cavity=10, Nt=40)
    u = systems.cavity_controls(3, p.Nt, seed=91) * amp
    e = _engine(p, 3, monkeypatch)
    J, g = _eval_dev(e, u)
    assert e.info()["backward"] == "segmented"
    e.close()
    for b in range(3):
        J0, g0, _ = O.grape_eval(p.A0, p.A, u[b], p.x0, p.x_target, p.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (amp, b))
