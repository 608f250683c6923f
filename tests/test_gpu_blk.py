"""The block path (csrc/qoc_blk.hpp): generators whose union sparsity pattern splits into small invariant blocks
(cavity-qubit: 2 x 2 blocks, zz coupling: 3 x 3) run the chains and the gradient block by block.  Checked through
the C ABI against the oracle (the reference's dense algorithm: src/gradient_computations.jl:17-29 forward, :52-58
co-states, :65-74 + :177-223 the gradient) and against the dense Taylor-action kernels (QOC_BLOCKS=0), at the
fp64 bar of SURVEY.md §8c: |ΔJ| <= 1e-12, ||ΔdJdu|| / ||dJdu|| <= 1e-10 per seed, states and co-states 1e-12
relative to their largest entry.
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


def _cases():
    from qoc_amd import systems
    out = {}
    p = systems.zz_problem(60, tgate=6.0)  # N = 9, 3 blocks of 3, m = 4, nu = 2
    out["zz"] = (p, systems.zz_controls(3, 60, 6.0, seed=61))
    p = systems.cavity_problem(N_cavity=10, Nt=50)  # N = 20, 10 blocks of 2, m = 2
    out["cavity20"] = (p, systems.cavity_controls(3, p.Nt, seed=62))
    p = systems.cavity_problem(N_cavity=20, Nt=40)  # N = 40 (the BASELINE system), 20 blocks of 2
    out["cavity40"] = (p, systems.cavity_controls(2, p.Nt, seed=63))
    return out


def _block_problem(NB=4, nblk=5, nu=2, m=3, Nt=30, seed=0):
    """Random skew-Hermitian generators with nblk blocks of NB rows under a random permutation (a block of
    NB - 1 rows too, so that padding is exercised)."""
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


BLK = ("blocks", "blocks_mfma", "blocks_prop")
# chain kernel of each block variant: block propagators formed apart from the chain (qoc_blku.hpp, the default for
# blocks of <= 4 rows), the polynomial inside the recurrence on MFMA block waves (QOC_BLKU=0), on the real embedding
# (QOC_BLOCKS=real), on VALU lanes (QOC_BLOCKS=valu)
KIND_KERNEL = {"prop": "blocks_prop", "propsplit": "blocks_prop", "props2": "blocks_prop", "mfma": "blocks_mfma",
               "real": "blocks_mfma", "valu": "blocks"}


def _engine(prob, B, blocks, monkeypatch, penalty=None, chain="taylor"):
    """blocks: True / "prop" (default kernels: block propagators, fused backward), "propsplit" (block propagators,
    plain backward chain + separate gradient), "props2" (block propagators with prefix-product groups of 2 slices),
    "mfma" (MFMA block waves, complex slots), "real" (blocks of <= 2 rows on their real embedding), "valu" (blocks
    of <= 4 rows on VALU lanes), False (dense)."""
    from qoc_amd import GrapeEngine
    monkeypatch.setenv("QOC_BLOCKS", blocks if blocks in ("valu", "real") else "1" if blocks else "0")
    monkeypatch.setenv("QOC_BLKU", "0" if blocks == "mfma" else "1")
    monkeypatch.setenv("QOC_BLKU_FUSED", "0" if blocks == "propsplit" else "1")
    monkeypatch.setenv("QOC_BLKU_S", "2" if blocks == "props2" else "1")
    # the forward + fused backward of k_blku_* on device evals too (the segmented eval: tests/test_gpu_blkseg.py)
    monkeypatch.setenv("QOC_BLKSEG", "0")
    # blocks of 5..16 rows: the Chebyshev-action block chains on device evals too (the stored-propagator eval:
    # tests/test_gpu_blkp.py)
    monkeypatch.setenv("QOC_BLKP", "0")
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_chain(chain)
    if penalty is not None:
        e.set_state_penalty(*penalty)
    return e


def _eval(e, u, device, order=3):
    if not device:
        J = e.propagate(u)
        return J, e.grape_sensitivity(u, order)
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


@pytest.mark.parametrize("name", ["zz", "cavity20", "cavity40"])
@pytest.mark.parametrize("device", [False, True])
@pytest.mark.parametrize("kind", ["prop", "propsplit", "props2", "mfma", "real", "valu"])
def test_blocks_match_oracle_and_dense_chains(built_lib, monkeypatch, name, device, kind):
    """Blocks of <= 4 rows: block propagators formed apart from the chain (default), or the polynomial inside the
    recurrence: packed into the 4-row slots of MFMA block waves, or one VALU lane per (block, column)
    (QOC_BLOCKS=valu); the block gradient either way."""
    prob, u = _cases()[name]
    B = u.shape[0]
    e = _engine(prob, B, kind, monkeypatch)
    J, g = _eval(e, u, device)
    info = e.info()
    assert info["chain_kernel"] == KIND_KERNEL[kind], info
    # block propagators: the backward contracts the gradient itself (k_blku_bwdg) on both the fused eval and
    # grape_sensitivity; the polynomial-in-the-chain kernels: the block chains' concurrent eval or the generic split
    assert info["backward"] == ("fused" if kind in ("prop", "props2") else "blocks" if device else "generic"), info
    xs = [e.state(k, seed=0) for k in (1, prob.Nt // 2, prob.Nt)]
    lams = [e.costate(k, seed=0) for k in (0, prob.Nt // 2, prob.Nt)]
    e.close()
    ed = _engine(prob, B, False, monkeypatch)
    Jd, gd = _eval(ed, u, device)
    assert ed.info()["chain_kernel"] in ("mfma_regs", "mfma_lds")
    ed.close()
    for b in range(B):
        J0, g0, c0 = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (name, b))
        _assert_seed(J[b], g[b], Jd[b], gd[b], (name, b, "dense"))
        if b == 0:
            xsc = max(np.abs(x).max() for x in c0.x)
            for x, k in zip(xs, (1, prob.Nt // 2, prob.Nt)):
                assert np.abs(x - c0.x[k]).max() <= 1e-12 * xsc, ("x", k)
            lsc = max(np.abs(lam).max() for lam in c0.lam)
            for lam, k in zip(lams, (0, prob.Nt // 2, prob.Nt)):
                assert np.abs(lam - c0.lam[k]).max() <= 1e-12 * lsc, ("lambda", k)


@pytest.mark.parametrize("order", [1, 2, 3, 4, "exact"])
@pytest.mark.parametrize("device", [False, True])
@pytest.mark.parametrize("kind", ["prop", "propsplit", "mfma"])
def test_blocks_gradient_orders(built_lib, monkeypatch, order, device, kind):
    """expm_jacobian! orders 1..4 (src/gradient_computations.jl:177-213) in the block gradient; the exact Fréchet
    gradient (opt-in) runs its dense kernel on the block chains' states and co-states."""
    from qoc_amd import systems
    prob = systems.zz_problem(50, tgate=5.0)
    u = systems.zz_controls(2, 50, 5.0, seed=64)
    e = _engine(prob, 2, kind, monkeypatch)
    J, g = _eval(e, u, device and order != "exact", order)
    assert e.info()["chain_kernel"] == KIND_KERNEL[kind]
    e.close()
    for b in range(2):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=order)
        _assert_seed(J[b], g[b], J0, g0, (order, b))


@pytest.mark.parametrize("gc", [13, 21])
@pytest.mark.parametrize("ustg", ["1", "2"])
@pytest.mark.parametrize("name", ["zz", "cavity20"])
def test_blocks_fused_chunk_sizes(built_lib, monkeypatch, gc, ustg, name):
    """The fused backward's chunk size need not divide 64 (the host picks the one that spreads the contraction
    evenly over the workers): Nt = 64 with C = 13 / 21 ends in a partial chunk past the padded record array, with
    one staging wave for records, x_k and stored propagators (QOC_BLKU_USTG=1) or two."""
    from qoc_amd import systems
    if name == "zz":
        prob = systems.zz_problem(64, tgate=6.0)
        u = systems.zz_controls(3, 64, 6.0, seed=71)
    else:
        prob = systems.cavity_problem(N_cavity=10, Nt=64)
        u = systems.cavity_controls(3, 64, seed=72)
    monkeypatch.setenv("QOC_BLKU_GC", str(gc))
    monkeypatch.setenv("QOC_BLKU_USTG", ustg)
    e = _engine(prob, 3, "prop", monkeypatch)
    J, g = _eval(e, u, True)
    assert e.info()["backward"] == "fused"
    e.close()
    for b in range(3):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (name, gc, ustg, b))


@pytest.mark.parametrize("poly", ["taylor", "chebyshev"])
@pytest.mark.parametrize("kind", ["prop", "mfma"])
def test_blocks_penalty_and_costate_source(built_lib, monkeypatch, poly, kind):
    """The state penalty (src/penalty_fcns.jl:1-11: L in the forward, 2 mu x_k added to λ_k in the backward) and a
    caller's dL/dx closure (qoc_set_costate_source) on the block chains, Taylor and Chebyshev terms."""
    from qoc_amd import systems
    monkeypatch.setenv("QOC_TCHAIN_POLY", poly)
    prob = systems.zz_problem(40, tgate=4.0)
    u = systems.zz_controls(2, 40, 4.0, seed=65)
    qb = systems.QuantumBasis([3, 3])
    pen = (qb(["20", "21", "22"]), [0, 1, 2, 3], 0.37)
    e = _engine(prob, 2, kind, monkeypatch, penalty=pen)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    info = e.info()
    assert info["chain_kernel"] == KIND_KERNEL[kind] and info["chain_poly"] == poly
    e.close()
    for b in range(2):
        Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, penalty=pen)
        _assert_seed(J[b], g[b], Jr, gr, ("penalty", b))
    # the same penalty as a co-state source: dL/dx(x_k) from the oracle's states, the cost's L added by hand
    Lf, dLf = O.setup_state_penalty(*pen)
    e = _engine(prob, 2, kind, monkeypatch)
    J = e.propagate(u)
    src = np.stack([np.stack([dLf(e.state(k, seed=b)) for k in range(prob.Nt + 1)]) for b in range(2)])
    e.set_costate_source(src)
    g = e.grape_sensitivity(u, 3)
    e.close()
    for b in range(2):
        Jr, gr, c = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3, penalty=pen)
        assert abs(J[b] + sum(Lf(x) for x in c.x) - Jr) <= 1e-12
        assert np.linalg.norm(g[b] - gr) / np.linalg.norm(gr) <= 1e-10


@pytest.mark.parametrize("NB,nu,m", [(4, 2, 3), (4, 1, 1), (3, 2, 2), (2, 1, 5), (2, 2, 8)])
@pytest.mark.parametrize("poly", ["taylor", "chebyshev"])
@pytest.mark.parametrize("kind", ["prop", "propsplit", "props2", "mfma", "real", "valu"])
def test_blocks_random_permuted_blocks(built_lib, monkeypatch, NB, nu, m, poly, kind):
    """Random block-diagonal skew-Hermitian generators hidden by a permutation (the detection works on the pattern,
    not on contiguous rows), a short last block (padding lanes), one or two controls, odd column counts."""
    monkeypatch.setenv("QOC_TCHAIN_POLY", poly)
    prob, u = _block_problem(NB=NB, nblk=5, nu=nu, m=m, seed=NB * 10 + nu + m)
    for device in (False, True):
        e = _engine(prob, 2, kind, monkeypatch)
        J, g = _eval(e, u, device)
        assert e.info()["chain_kernel"] == KIND_KERNEL[kind]
        e.close()
        for b in range(2):
            J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
            _assert_seed(J[b], g[b], J0, g0, (NB, nu, m, device, b))


def test_blocks_external_cost_and_zcalibrated(built_lib, monkeypatch):
    """An external λ_N (qoc_grape_sensitivity's lambda_final: the caller's dJfinal_dx closure) and the z-calibrated
    cost (src/penalty_fcns.jl:27-42) on the block path; the z-calibrated gradient is held to the oracle's gradient
    family g(Δθ) within the per-seed calibration-phase bound (see tests/test_gpu_parity.py)."""
    from qoc_amd import GrapeEngine, systems
    monkeypatch.setenv("QOC_BLOCKS", "1")
    prob = systems.zz_problem(40, tgate=4.0)
    u = systems.zz_controls(2, 40, 4.0, seed=66)
    Jf, dJf = O.setup_infidelity(prob.x_target, prob.n)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2)
    e.set_cost_external()
    e.set_chain("taylor")
    e.propagate(u)
    lam = np.stack([dJf(e.state(prob.Nt, seed=b)) for b in range(2)])
    g = e.grape_sensitivity(u, 3, lambda_final=lam)
    assert e.info()["chain_kernel"] in BLK
    e.close()
    for b in range(2):
        _, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        assert np.linalg.norm(g[b] - g0) / np.linalg.norm(g0) <= 1e-10
    Jz, _ = O.setup_infidelity_zcalibrated(prob.x_target)
    for device in (False, True):
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2)
        e.set_cost_zcalibrated(prob.x_target)
        e.set_chain("taylor")
        J, g = _eval(e, u, device)
        assert e.info()["chain_kernel"] in BLK
        e.close()
        for b in range(2):
            xN = O.propagate(prob.A0, prob.A, u[b], prob.x0)[-1]
            assert abs(J[b] - Jz(xN)) <= 1e-12
            res, dth = O.zcal_gradient_match(g[b], prob.A0, prob.A, u[b], prob.x0, prob.x_target, order=3)
            assert res <= 1e-10 and abs(dth) <= O.zcal_dtheta_bound(prob.x_target, xN), (device, b, res, dth)


def test_blocks_off_for_dense_generators(built_lib, monkeypatch):
    """Generators coupling every row (one block of 20 rows) keep the dense chains; so do blocks of 5..16 rows at
    N <= 16, where the dense register chain already runs one wave per column pair."""
    prob, _ = _block_problem(NB=4, nblk=2, nu=2, m=2, seed=3)
    import dataclasses
    from qoc_amd import systems
    rng = np.random.default_rng(7)
    H = systems._gue(rng, 20)
    dense = dataclasses.replace(prob, A0=-0.05j * H, A=[-0.03j * systems._gue(rng, 20), -0.02j * systems._gue(rng, 20)],
                                x0=np.eye(20, 2, dtype=complex), x_target=np.eye(20, 2, dtype=complex))
    e = _engine(dense, 1, True, monkeypatch)
    assert e.info()["chain_kernel"] not in BLK
    e.close()
    p16, _ = _block_problem(NB=8, nblk=2, nu=1, m=1, seed=4)  # N = 15
    e = _engine(p16, 1, True, monkeypatch)
    assert e.info()["chain_kernel"] not in BLK
    e.close()


@pytest.mark.parametrize("which", ["tunable_bus", "tunable_bus_cz"])
@pytest.mark.parametrize("device", [False, True])
def test_blocks_mfma_tunable_bus(built_lib, monkeypatch, which, device):
    """The tunable bus (two parity blocks of 14 and 13 rows at N = 27): one MFMA wave per (block, column pair)
    instead of the dense two-group register chain; against the oracle and the dense chains.  The CZ variant
    (m = 4: two column pairs, x0 columns in both blocks)."""
    from qoc_amd import systems
    Nt = 48
    mk = systems.tunable_bus_problem if which == "tunable_bus" else systems.tunable_bus_cz_problem
    prob = mk(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(2, Nt, seed=67)
    e = _engine(prob, 2, True, monkeypatch)
    J, g = _eval(e, u, device)
    info = e.info()
    assert info["chain_kernel"] == "blocks_mfma", info
    lams = [e.costate(k, seed=1) for k in (0, Nt // 2, Nt)]
    xs = [e.state(k, seed=1) for k in (1, Nt // 2, Nt)]
    e.close()
    ed = _engine(prob, 2, False, monkeypatch)
    Jd, gd = _eval(ed, u, device)
    assert ed.info()["chain_kernel"] == "mfma_regs"
    ed.close()
    for b in range(2):
        J0, g0, c0 = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (which, b))
        _assert_seed(J[b], g[b], Jd[b], gd[b], (which, b, "dense"))
    xsc = max(np.abs(x).max() for x in c0.x)
    for x, k in zip(xs, (1, Nt // 2, Nt)):
        assert np.abs(x - c0.x[k]).max() <= 1e-12 * xsc, ("x", k)
    lsc = max(np.abs(lam).max() for lam in c0.lam)
    for lam, k in zip(lams, (0, Nt // 2, Nt)):
        assert np.abs(lam - c0.lam[k]).max() <= 1e-12 * lsc, ("lambda", k)


@pytest.mark.parametrize("NB,nblk,nu,m", [(10, 3, 2, 3), (16, 2, 1, 1), (7, 4, 2, 2), (12, 3, 1, 4)])
@pytest.mark.parametrize("poly", ["taylor", "chebyshev"])
def test_blocks_mfma_random_permuted_blocks(built_lib, monkeypatch, NB, nblk, nu, m, poly):
    """Random permuted blocks of 5..16 rows (a short last block for padding lanes), both polynomials, host and device
    evals, a state penalty and the orders 1, 2, 4 (the dense gradient kernels on the block chains' states)."""
    monkeypatch.setenv("QOC_TCHAIN_POLY", poly)
    prob, u = _block_problem(NB=NB, nblk=nblk, nu=nu, m=m, seed=NB * 10 + nblk + nu + m)
    for device in (False, True):
        e = _engine(prob, 2, True, monkeypatch)
        J, g = _eval(e, u, device)
        assert e.info()["chain_kernel"] == "blocks_mfma"
        e.close()
        for b in range(2):
            J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
            _assert_seed(J[b], g[b], J0, g0, (NB, nu, m, device, b))
    pen = ([0, 3, 5], [0], 0.3)
    e = _engine(prob, 2, True, monkeypatch, penalty=pen)
    J = e.propagate(u)
    gs = {o: e.grape_sensitivity(u, o) for o in (1, 2, 4)}
    e.close()
    for b in range(2):
        for o, g in gs.items():
            J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=o, penalty=pen)
            _assert_seed(J[b], g[b], J0, g0, ("penalty", o, b))


def test_fused_backward_blocks_of_4_rows_two_chain_waves(built_lib, monkeypatch):
    """Blocks of 4 rows with nblk m = 20 (two chain waves inside the 4-wave launch bound of blocks of 4 rows): the
    fused backward keeps a worker wave (one staging wave copies the stored propagators as well), so dJdu is the
    contraction's, not whatever the buffer held."""
    prob, u = _block_problem(NB=4, nblk=5, nu=2, m=4, Nt=40, seed=11)
    e = _engine(prob, 2, "prop", monkeypatch)
    J, g = _eval(e, u, True)
    assert e.info()["backward"] == "fused", e.info()
    e.close()
    for b in range(2):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, b)


def test_new_block_layout_reallocates_stored_propagators(built_lib, monkeypatch):
    """qoc_set_generators with a block layout whose propagators need more room (blocks of 2 rows, then of 4 rows at
    the same N = 11): the fused eval's stored-propagator buffer grows with it; co-states that the fused eval left to be
    rebuilt on demand come from the system they were computed for, also after the generators changed."""
    p2, u2 = _block_problem(NB=2, nblk=6, nu=2, m=2, Nt=30, seed=12)
    p4, u4 = _block_problem(NB=4, nblk=3, nu=2, m=2, Nt=30, seed=13)
    assert p2.N == p4.N
    e = _engine(p2, 2, "prop", monkeypatch)
    J, g = _eval(e, u2, True)
    assert e.info()["backward"] == "fused"
    _, _, c0 = O.grape_eval(p2.A0, p2.A, u2[1], p2.x0, p2.x_target, p2.n, order=3)
    e.set_generators(p4.A0, p4.A)
    lam = e.costate(7, seed=1)  # the first system's co-state (rebuilt before the generators changed)
    lsc = max(np.abs(x).max() for x in c0.lam)
    assert np.abs(lam - c0.lam[7]).max() <= 1e-12 * lsc
    e.set_x0(p4.x0)
    e.set_cost_trace(p4.x_target, p4.n)
    J, g = _eval(e, u4, True)
    assert e.info()["backward"] == "fused"
    e.close()
    for b in range(2):
        J0, g0, _ = O.grape_eval(p4.A0, p4.A, u4[b], p4.x0, p4.x_target, p4.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, b)


def test_blocks_mfma_dead_blocks_skipped(built_lib, monkeypatch):
    """Blocks of 5..16 rows whose x0 and target rows are all zero (the tunable bus at m = 1: |110> -> |200> lives in
    the 14-row even-parity block) get no waves in the concurrent eval; their rows of x_k and λ_k are written as zeros.
    J, dJ/du, states and co-states equal the all-blocks launch (QOC_BLK_DEAD=0) exactly, also after an eval whose
    live block was the other one left nonzero rows behind, and match the oracle."""
    from qoc_amd import systems
    Nt = 48
    prob = systems.tunable_bus_problem(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(2, Nt, seed=71)
    qb = systems.QuantumBasis([3, 3, 3])
    x_odd, t_odd = qb.columns(["100"]).astype(complex), qb.columns(["001"]).astype(complex)
    assert np.abs(x_odd[0::2]).max() == 0 and np.abs(prob.x0[1::2]).max() == 0
    ks = (0, 1, Nt // 2, Nt)
    out = {}
    for dead in ("1", "0"):
        monkeypatch.setenv("QOC_BLK_DEAD", dead)
        e = _engine(prob, 2, True, monkeypatch)
        e.set_x0(x_odd)
        e.set_cost_trace(t_odd, prob.n)
        _eval(e, u, True)  # the odd block live: nonzero odd rows in every buffer
        e.set_x0(prob.x0)
        e.set_cost_trace(prob.x_target, prob.n)
        _eval(e, u, True)  # odd rows zeroed
        e.set_x0(prob.x0 + x_odd)  # both blocks live: nonzero odd rows again
        _eval(e, u, True)
        e.set_x0(prob.x0)
        _eval(e, u, True)  # the same dead rows as two evals ago: must be zeroed again
        J, g = _eval(e, u, True)  # and this one may skip the zeroing
        assert e.info()["chain_kernel"] == "blocks_mfma"
        xs = [e.state(k, seed=b) for k in ks for b in (0, 1)]
        ls = [e.costate(k, seed=b) for k in ks for b in (0, 1)]
        e.close()
        out[dead] = (J, g, xs, ls)
    J, g, xs, ls = out["1"]
    assert np.array_equal(J, out["0"][0]) and np.array_equal(g, out["0"][1])
    for a, b in zip(xs + ls, out["0"][2] + out["0"][3]):
        assert np.array_equal(a, b)
        assert np.abs(a[1::2]).max() == 0.0  # the dead odd rows
    for b in range(2):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, b)
