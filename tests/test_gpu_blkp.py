"""Stored propagators for invariant blocks of 5..16 rows (csrc/qoc_blkp.hpp: k_blkp_exp, k_blkp_dual + k_grad_rr_c),
the concurrent eval of the tunable bus' parity blocks: U_k = exp(A_k) per (seed, slice, live block) on MFMA, then one
matvec per slice in the chains (the reference's structure, src/gradient_computations.jl:17-29 forward, :52-58
co-states, :65-74 + :177-223 the order-3 gradient).  Against the oracle and the Chebyshev-action block chains
(QOC_BLKP=0) at the fp64 bar of SURVEY.md §8c: |ΔJ| <= 1e-12, ||ΔdJdu|| / ||dJdu|| <= 1e-10 per seed, states and
co-states 1e-12 relative to their largest entry.
"""
import numpy as np
import pytest

import qoc_oracle as O
from test_gpu_blk import _assert_seed, _block_problem, _eval

pytestmark = pytest.mark.gpu


def _engine(prob, B, monkeypatch, blkp=True):
    from qoc_amd import GrapeEngine
    monkeypatch.setenv("QOC_BLOCKS", "1")
    monkeypatch.setenv("QOC_BLKP", "1" if blkp else "0")
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_chain("taylor")
    return e


def _check_states(e, prob, u, b, ks):
    _, _, c0 = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
    xsc = max(np.abs(x).max() for x in c0.x)
    lsc = max(np.abs(lam).max() for lam in c0.lam)
    for k in ks:
        assert np.abs(e.state(k, seed=b) - c0.x[k]).max() <= 1e-12 * xsc, ("x", b, k)
        assert np.abs(e.costate(k, seed=b) - c0.lam[k]).max() <= 1e-12 * lsc, ("lambda", b, k)


@pytest.mark.parametrize("which", ["tunable_bus", "tunable_bus_cz"])
def test_blkp_tunable_bus_matches_oracle(built_lib, monkeypatch, which):
    """The tunable bus (m = 1: the 14-row even block alone is live) and its CZ variant (m = 4, x0 columns in both
    blocks: two live wave blocks, 8 chain waves per seed and direction)."""
    from qoc_amd import systems
    Nt = 48
    mk = systems.tunable_bus_problem if which == "tunable_bus" else systems.tunable_bus_cz_problem
    prob = mk(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(3, Nt, seed=81)
    e = _engine(prob, 3, monkeypatch)
    J, g = _eval(e, u, True)
    info = e.info()
    assert info["chain_kernel"] == "blocks_prop16" and info["backward"] == "blocks_prop16", info
    for b in range(3):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (which, b))
    _check_states(e, prob, u, 1, (0, 1, Nt // 2, Nt))
    e.close()
    ep = _engine(prob, 3, monkeypatch, blkp=False)
    Jp, gp = _eval(ep, u, True)
    assert ep.info()["chain_kernel"] == "blocks_mfma"
    ep.close()
    for b in range(3):
        _assert_seed(J[b], g[b], Jp[b], gp[b], (which, b, "chebyshev chains"))


@pytest.mark.parametrize("NB,nblk,nu,m", [(10, 3, 2, 2), (16, 2, 1, 1), (7, 4, 2, 2), (12, 3, 1, 2), (5, 6, 2, 1)])
def test_blkp_random_permuted_blocks(built_lib, monkeypatch, NB, nblk, nu, m):
    """Random skew-Hermitian generators with permuted blocks of 5..16 rows (a short last block: padding rows and
    columns in the propagator tiles), nu = 1 and 2, up to 8 chain waves."""
    prob, u = _block_problem(NB=NB, nblk=nblk, nu=nu, m=m, Nt=40, seed=NB * 7 + nblk + nu + m)
    e = _engine(prob, 2, monkeypatch)
    J, g = _eval(e, u, True)
    assert e.info()["backward"] == "blocks_prop16", e.info()
    for b in range(2):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (NB, nblk, nu, m, b))
    _check_states(e, prob, u, 0, (0, 1, 20, 40))
    e.close()


@pytest.mark.parametrize("scale", [1e-3, 0.3, 8.0, 40.0])
def test_blkp_norm_range(built_lib, monkeypatch, scale):
    """Slice norms from ~1e-3 (Taylor degree 8, no squaring) to ~100 (degree 24 and 5+ squarings): the per-unit
    (degree, squarings) choice holds the fp64 bar over the whole range."""
    from qoc_amd import systems
    prob, u = _block_problem(NB=14, nblk=2, nu=2, m=1, Nt=24, seed=5)
    prob = systems.Problem("blocks", prob.A0 * scale, [a * scale for a in prob.A], prob.x0, prob.x_target, prob.n,
                           prob.Nt, "fp64")
    e = _engine(prob, 2, monkeypatch)
    e.chain_terms(reset=True)
    J, g = _eval(e, u, True)
    prods = e.chain_terms()
    assert e.info()["backward"] == "blocks_prop16"
    e.close()
    for b in range(2):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (scale, b))
    # executed 16 x 16 products per (seed, slice, block): r + 2 + s with r >= 2
    assert prods >= 4 * 2 * 24 * 2, prods


def test_blkp_eval_then_host_backward(built_lib, monkeypatch):
    """A device eval (stored propagators, no step records) followed by grape_sensitivity on the same u: the block
    backward prepares its step records first (steps_stale) and gives the oracle's gradient for every order."""
    from qoc_amd import systems
    Nt = 40
    prob = systems.tunable_bus_problem(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(2, Nt, seed=82)
    e = _engine(prob, 2, monkeypatch)
    J, g = _eval(e, u, True)
    assert e.info()["backward"] == "blocks_prop16"
    gs = {o: e.grape_sensitivity(u, o) for o in (3, 1, 2)}
    e.close()
    for b in range(2):
        for o, go in gs.items():
            J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=o)
            _assert_seed(J[b], go[b], J0, g0, ("host", o, b))


def test_blkp_dead_block_rows_zero(built_lib, monkeypatch):
    """The tunable bus at m = 1 with the odd block live first (nonzero odd rows in every state buffer), then the even
    block: the stored-propagator eval zeroes the dead rows, so states, co-states, J and dJ/du equal the all-blocks
    launch (QOC_BLK_DEAD=0)."""
    from qoc_amd import systems
    Nt = 32
    prob = systems.tunable_bus_problem(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(2, Nt, seed=83)
    qb = systems.QuantumBasis([3, 3, 3])
    x_odd, t_odd = qb.columns(["100"]).astype(complex), qb.columns(["001"]).astype(complex)
    out = {}
    for dead in ("1", "0"):
        monkeypatch.setenv("QOC_BLK_DEAD", dead)
        e = _engine(prob, 2, monkeypatch)
        e.set_x0(x_odd)
        e.set_cost_trace(t_odd, prob.n)
        _eval(e, u, True)
        e.set_x0(prob.x0)
        e.set_cost_trace(prob.x_target, prob.n)
        J, g = _eval(e, u, True)
        assert e.info()["backward"] == "blocks_prop16"
        xs = [e.state(k, seed=b) for k in (0, 1, Nt) for b in (0, 1)]
        ls = [e.costate(k, seed=b) for k in (0, 1, Nt) for b in (0, 1)]
        e.close()
        out[dead] = (J, g, xs, ls)
    J, g, xs, ls = out["1"]
    assert np.array_equal(J, out["0"][0]) and np.array_equal(g, out["0"][1])
    for a, b in zip(xs + ls, out["0"][2] + out["0"][3]):
        assert np.array_equal(a, b)
    for b in range(2):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, ("dead", b))


def test_blkp_interpolated_propagators(built_lib, monkeypatch):
    """One control (nu = 1): the propagators interpolated in u (k_blkp_int, U(u) = Σ T_i(ξ) M_i over the batch's control
    range, coefficients from long-double exponentials at Chebyshev points) against the oracle and against the
    per-slice exponentials (QOC_BLKP_INTERP=0); a later batch outside the range recomputes the coefficients; a range too
    wide for the series falls back to the exponentials."""
    from qoc_amd import systems
    Nt = 40
    prob = systems.tunable_bus_problem(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(3, Nt, seed=86)
    e = _engine(prob, 3, monkeypatch)
    J, g = _eval(e, u, True)
    info = e.info()
    assert info["interp_degree"] > 0 and info["backward"] == "blocks_prop16", info
    for b in range(3):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, ("interp", b))
    # controls beyond the first range (0.3..1.0 -> up to 1.6): new coefficients
    u2 = u * 1.6
    J2, g2 = _eval(e, u2, True)
    assert e.info()["interp_degree"] > 0
    for b in range(3):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u2[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J2[b], g2[b], J0, g0, ("interp wider", b))
    # a range the 40-point series cannot resolve: the per-slice exponentials
    u3 = u.copy()
    u3[0, 0, 0] = -40.0
    J3, g3 = _eval(e, u3, True)
    assert e.info()["interp_degree"] == 0
    for b in range(3):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u3[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J3[b], g3[b], J0, g0, ("fallback", b))
    e.close()
    monkeypatch.setenv("QOC_BLKP_INTERP", "0")
    ep = _engine(prob, 3, monkeypatch)
    Jp, gp = _eval(ep, u, True)
    assert ep.info()["interp_degree"] == 0
    ep.close()
    for b in range(3):
        _assert_seed(J[b], g[b], Jp[b], gp[b], ("interp vs exponentials", b))


@pytest.mark.parametrize("ch", ["2", "4", "8"])
def test_blkp_tail_chunk(built_lib, monkeypatch, ch):
    """Nt = 37, not a multiple of any chain chunk: the chains' last chunk is partial (the j0 + jj >= Nt exit, the state
    sinks flushed at the end, the clamped DMA slices), for every chunk size the chain kernels instantiate
    (QOC_BLKP_CH), in the device eval (k_blkp_dual) and in the split call form (k_blkp_chain in propagate and in
    grape_sensitivity): the oracle's J, dJ/du and states."""
    from qoc_amd import systems
    Nt = 37
    monkeypatch.setenv("QOC_BLKP_CH", ch)
    monkeypatch.setenv("QOC_BLKP_ICHAIN", "0")  # the stored form (test_blkp_interpolating_chains: the fused one)
    prob = systems.tunable_bus_problem(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(3, Nt, seed=91)
    e = _engine(prob, 3, monkeypatch)
    J, g = _eval(e, u, True)
    assert e.info()["backward"] == "blocks_prop16" and e.info()["interp_chain"] == 0, e.info()
    Js = e.propagate(u)
    gs = e.grape_sensitivity(u, 3)
    assert e.info()["backward"] == "blocks_prop16", e.info()
    for b in range(3):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, ("eval", ch, b))
        _assert_seed(Js[b], gs[b], J0, g0, ("split", ch, b))
    _check_states(e, prob, u, 2, (0, 1, 31, 32, 33, 36, Nt))
    e.close()


def test_blkp_interpolating_chains(built_lib, monkeypatch):
    """The interpolating chains (k_blkp_ichain: each chain wave forms its slices' propagators from the interpolation
    coefficients in registers, nothing stored), on the symmetric propagators' upper triangle (the tunable bus' H is
    real) and on every entry (QOC_BLKP_ISYM=0), two waves per chain taking alternate chunks (2 or 4 pairs per workgroup)
    and one (QOC_BLKP_IPAIR=0):
    the oracle's J, dJ/du, states and co-states, and bit for bit the stored
    form (k_blkp_int + k_blkp_dual / k_blkp_chain, QOC_BLKP_ICHAIN=0) in the device eval and in the split call form.
    Nt = 37 (a partial last chunk of 8 slices), B = 5 (a last workgroup with two of its four waves idle)."""
    from qoc_amd import systems
    Nt, B = 37, 5
    prob = systems.tunable_bus_problem(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(B, Nt, seed=93)
    out = {}
    for ich, isym, ipair, want in (("1", "1", "1", 2), ("1", "1", "4", 2), ("1", "1", "0", 2), ("1", "0", "1", 1),
                                   ("1", "0", "0", 1), ("0", "1", "1", 0)):
        monkeypatch.setenv("QOC_BLKP_ICHAIN", ich)
        monkeypatch.setenv("QOC_BLKP_ISYM", isym)
        monkeypatch.setenv("QOC_BLKP_IPAIR", "0" if ipair == "0" else "1")
        monkeypatch.setenv("QOC_BLKP_IPW", "4" if ipair == "4" else "2")  # pairs per workgroup
        e = _engine(prob, B, monkeypatch)
        J, g = _eval(e, u, True)
        info = e.info()
        assert info["backward"] == "blocks_prop16" and info["interp_degree"] > 0, info
        assert info["interp_chain"] == want, info
        xs = [e.state(k, seed=b) for k in (0, 1, 8, 9, 36, Nt) for b in (0, 4)]
        ls = [e.costate(k, seed=b) for k in (0, 1, 8, 9, 36, Nt) for b in (0, 4)]
        Js = e.propagate(u)
        gs = e.grape_sensitivity(u, 3)
        assert e.info()["interp_chain"] == want
        xs2 = [e.state(k, seed=3) for k in (0, 17, Nt)]
        e.close()
        out[(want, ipair)] = (J, g, xs, ls, Js, gs, xs2)
    ref = out[(0, "1")]
    for form in ((2, "1"), (2, "4"), (2, "0"), (1, "1"), (1, "0")):
        J, g, xs, ls, Js, gs, xs2 = out[form]
        for b in range(B):
            J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
            _assert_seed(J[b], g[b], J0, g0, ("ichain eval", form, b))
            _assert_seed(Js[b], gs[b], J0, g0, ("ichain split", form, b))
        _check_states(_Reader(xs, ls, (0, 1, 8, 9, 36, Nt), (0, 4)), prob, u, 4, (0, 1, 8, 9, 36, Nt))
        for a, r, what in zip((J, g, Js, gs), (ref[0], ref[1], ref[4], ref[5]), ("J", "dJdu", "split J", "split dJdu")):
            assert np.array_equal(a, r), (form, what)
        for a, r in zip(xs + ls + xs2, ref[2] + ref[3] + ref[6]):
            assert np.array_equal(a, r), form


class _Reader:
    """states / co-states read back before the engine closed, served as e.state / e.costate"""

    def __init__(self, xs, ls, ks, seeds):
        self.x = {(k, b): xs[i * len(seeds) + j] for i, k in enumerate(ks) for j, b in enumerate(seeds)}
        self.l = {(k, b): ls[i * len(seeds) + j] for i, k in enumerate(ks) for j, b in enumerate(seeds)}

    def state(self, k, seed=0):
        return self.x[(k, seed)]

    def costate(self, k, seed=0):
        return self.l[(k, seed)]
