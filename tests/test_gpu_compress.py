"""compress_states inside the engine (src/utils.jl:96-109; include/qoc.h qoc_set_compression).

A parity-structured problem has generators that are block-diagonal in two row sets, and each state column
lives in one of the two sets. The engine packs the two blocks into max(n1, n2) columns, so the chains and the
gradient run on those packed columns, while the caller passes and receives the unpacked (N, m) states. Every
result here is checked against the ORACLE evaluated on the UNPACKED problem (oracle/qoc_oracle.py with all m
columns), at the fp64 bar: |ΔJ| <= 1e-12, rel ||ΔdJdu|| <= 1e-10, states to 1e-13.

* The reference's own compress layout (test/test_utils.jl:23: rows 1:2:27 with columns [1, 4], rows 2:2:26 with
  [2, 3]) on the tunable-bus model driven as a CZ gate. Its Hamiltonian conserves excitation number, so it is
  block-diagonal in the parity of the basis index. Costs: trace and z-calibrated.
* A random block-diagonal problem with small norms (Taylor-action chains), with and without the state
  penalty. It runs both chain kinds, the large-N GEMM pipeline (QOC_FORCE_LARGE_N) and the Tsit5 path.
* The second reference vector (test/test_utils.jl:32: columns [1, 4, 5] / [2, 3]), i.e. 3 packed columns of m = 5.
* Errors: coupling generators, x0 outside its block, index lists that do not partition.
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


def _block_problem(N=12, Nt=15, cols=((0, 3), (1, 2)), seed=8, scale=0.2):
    from qoc_amd import systems
    rng = np.random.default_rng(seed)
    r1, r2 = list(range(0, N, 2)), list(range(1, N, 2))

    def block_gen(sc):
        H = np.zeros((N, N), complex)
        for r in (r1, r2):
            G = rng.standard_normal((len(r), len(r))) + 1j * rng.standard_normal((len(r), len(r)))
            H[np.ix_(r, r)] = (G + G.conj().T) / 2
        return -1j * sc * H / np.abs(H).sum(0).max()

    m = len(cols[0]) + len(cols[1])
    x0 = np.zeros((N, m), complex)
    xt = np.zeros((N, m), complex)
    for rows, cs in ((r1, cols[0]), (r2, cols[1])):
        for c in cs:
            for M in (x0, xt):
                v = rng.standard_normal(len(rows)) + 1j * rng.standard_normal(len(rows))
                M[rows, c] = v / np.linalg.norm(v)
    prob = systems.Problem("parity", block_gen(scale), [block_gen(0.05), block_gen(0.05)], x0, xt, float(m), Nt,
                           "fp64")
    v = ((r1, list(cols[0])), (r2, list(cols[1])))
    u = rng.uniform(-1, 1, size=(2, 2, Nt))
    return prob, v, u


def _engine(prob, v, B, chain=None, zcal=False, tsit5=None, penalty=None):
    from qoc_amd import GrapeEngine
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_compression(v)
    if zcal:
        e.set_cost_zcalibrated(prob.x_target)
    else:
        e.set_cost_trace(prob.x_target, prob.n)
    if chain is not None:
        e.set_chain(chain)
    if tsit5:
        e.set_propagation("tsit5", tsit5)
    if penalty is not None:
        e.set_state_penalty(*penalty)
    return e


def _check(prob, v, u, *, chain=None, zcal=False, tsit5=None, penalty=None):
    e = _engine(prob, v, u.shape[0], chain, zcal, tsit5, penalty)
    assert e.info()["kernel_m"] == max(len(v[0][1]), len(v[1][1])) < prob.x0.shape[1]
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    cost = O.setup_infidelity_zcalibrated(prob.x_target) if zcal else None
    for b in range(u.shape[0]):
        if tsit5:
            Jr, gr = O.grape_eval_ode(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, nsub=tsit5,
                                      penalty=penalty, cost=cost)
            xs = O.propagate_pwc_ode(prob.A0, prob.A, u[b], prob.x0, nsub=tsit5)
        else:
            Jr, gr, cache = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3,
                                         penalty=penalty, cost=cost)
            xs = cache.x
        assert abs(J[b] - Jr) <= 1e-12, (b, J[b], Jr)
        if zcal:  # the calibration phase is fixed only to ~sqrt(eps): see test_gpu_parity.test_zcalibrated_cost
            res, dth = O.zcal_gradient_match(g[b], prob.A0, prob.A, u[b], prob.x0, prob.x_target, order=3,
                                             nsub=tsit5)
            assert res <= 1e-10 and abs(dth) <= 1e-6, (b, res, dth)
        else:
            rel = np.linalg.norm(g[b] - gr) / np.linalg.norm(gr)
            assert rel <= 1e-10, (b, rel)
        for k in (0, prob.Nt // 2, prob.Nt):
            assert np.abs(e.state(k, seed=b) - xs[k]).max() < 1e-13  # unpacked layout on the way out
    e.close()
    return J, g


@pytest.mark.parametrize("zcal", [False, True])
def test_reference_layout_on_tunable_bus_cz(built_lib, zcal):
    """test/test_utils.jl:23's layout on the physical model: 4 columns -> 2 packed columns, propagators (Padé)."""
    from qoc_amd import systems
    prob = systems.tunable_bus_cz_problem(Nt=40, tgate=350.0 * 40 / 2000)
    u = systems.tunable_bus_controls(2, prob.Nt, seed=3)
    _check(prob, systems.TUNABLE_BUS_PARITY, u, zcal=zcal)


@pytest.mark.parametrize("chain", ["taylor", "propagators"])
@pytest.mark.parametrize("penalty", [False, True])
def test_block_problem_chains(built_lib, chain, penalty):
    prob, v, u = _block_problem()
    pen = ([0, 1, 10, 11], [0, 1, 2, 3], 0.3) if penalty else None
    _check(prob, v, u, chain=chain, penalty=pen)


def test_block_problem_zcal_taylor_chains(built_lib):
    prob, v, u = _block_problem(seed=11)
    _check(prob, v, u, chain="taylor", zcal=True)


def test_block_problem_large_n_pipeline(built_lib, monkeypatch):
    monkeypatch.setenv("QOC_FORCE_LARGE_N", "1")
    prob, v, u = _block_problem(seed=5)
    _check(prob, v, u)


def test_block_problem_tsit5(built_lib):
    prob, v, u = _block_problem(seed=6)
    _check(prob, v, u, tsit5=6, penalty=([2, 3], [1, 3], 0.2))


def test_second_reference_vector_three_packed_columns(built_lib):
    """test/test_utils.jl:32: columns [1, 4, 5] on the odd rows and [2, 3] on the even rows (1-based) -> m = 5
    packed into 3 columns."""
    prob, v, u = _block_problem(N=27, cols=((0, 3, 4), (1, 2)), seed=9)
    _check(prob, v, u)


def test_api_cache_with_compression_matches_oracle(built_lib):
    """The reference-shaped API: setup_grape_cache(..., compress=v), propagate, grape_sensitivity with closures."""
    import qoc_amd as Q
    prob, v, u = _block_problem(seed=12)
    cache = Q.setup_grape_cache(prob.A0, prob.x0, u.shape[1:], compress=v)
    x = Q.propagate(prob.A0, prob.A, u[0], prob.x0, cache)
    Jf, dJf = Q.setup_infidelity(prob.x_target, prob.n)
    g = Q.grape_sensitivity(prob.A0, prob.A, dJf, cache.u, prob.x0, cache, dUkdp_order=3)
    Jr, gr, c2 = O.grape_eval(prob.A0, prob.A, u[0], prob.x0, prob.x_target, prob.n, order=3)
    assert abs(Jf(x[-1]) - Jr) <= 1e-12
    assert np.linalg.norm(g - gr) / np.linalg.norm(gr) <= 1e-10
    assert np.abs(x[prob.Nt] - c2.x[prob.Nt]).max() < 1e-13


def test_packing_can_be_turned_off_again(built_lib):
    prob, v, u = _block_problem(seed=13)
    e = _engine(prob, v, 2)
    J1 = e.propagate(u)
    e.set_compression(None)
    assert e.info()["kernel_m"] == prob.x0.shape[1]
    J0 = e.propagate(u)
    e.close()
    np.testing.assert_allclose(J1, J0, rtol=0, atol=1e-13)


def test_errors(built_lib):
    from qoc_amd import GrapeEngine, QOCError
    prob, v, u = _block_problem(seed=14)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=1)
    (r1, c1), (r2, c2) = v
    with pytest.raises(QOCError, match="partition"):
        e.set_compression(((r1[:-1], c1), (r2, c2)))
    with pytest.raises(QOCError, match="partition"):
        e.set_compression(((r1, c1[:1]), (r2, c2)))
    # x0 with an entry outside its block
    x0 = prob.x0.copy()
    x0[r2[0], c1[0]] = 0.5
    e.set_x0(x0)
    with pytest.raises(QOCError, match="outside the compress_states blocks"):
        e.set_compression(v)
    assert e.info()["kernel_m"] == prob.x0.shape[1]  # rolled back
    e.set_x0(prob.x0)
    e.set_compression(v)
    # generators that couple the blocks
    A0 = prob.A0.copy()
    A0[r1[0], r2[0]] = 0.01
    with pytest.raises(QOCError, match="couple"):
        e.set_generators(A0, prob.A)
    e.close()


@pytest.mark.parametrize("zcal", [False, True])
def test_failed_repack_leaves_the_packing_intact(built_lib, zcal):
    """A re-pack that x0 fails (entries outside the new blocks) leaves the previous packing fully in place: the host
    layout, the device row sectors and the z-calibrated column map; J and dJ/du still match the oracle."""
    from qoc_amd import QOCError
    prob, v, u = _block_problem(seed=21)
    e = _engine(prob, v, u.shape[0], chain="taylor", zcal=zcal)
    (r1, c1), (r2, c2) = v
    with pytest.raises(QOCError, match="outside the compress_states blocks"):
        e.set_compression(((r1, c2), (r2, c1)))  # x0's columns c1 live on r1: outside the swapped blocks
    assert e.info()["kernel_m"] == 2
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    cost = O.setup_infidelity_zcalibrated(prob.x_target) if zcal else None
    for b in range(u.shape[0]):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, cost=cost)
        assert abs(J[b] - Jr) <= 1e-12, (b, J[b], Jr)
        if zcal:
            res, dth = O.zcal_gradient_match(g[b], prob.A0, prob.A, u[b], prob.x0, prob.x_target, order=3)
            assert res <= 1e-10 and abs(dth) <= 1e-6, (b, res, dth)
        else:
            assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10
    e.close()
