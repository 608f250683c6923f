"""Parity at the BASELINE.json configurations' stated sizes (per GPU), on the GPU, through the C ABI.

configs 2-4 (fp64): every seed of the batch runs on the GPU; a seed subset is checked against the C port
(oracle/cpu_ref.c: the reference's Padé + solve, zgemm, order-3 Taylor Jacobian; OpenBLAS zgemm/zgesv) at the
SURVEY.md §8c bar |ΔJ| <= 1e-12, ||ΔdJdu|| / ||dJdu|| <= 1e-10 per seed.
config 5 (synthetic N = 256, fp32, large-N pipeline): the full batch runs; a bounded slice prefix of seed 0 is
checked against the numpy oracle in fp64 at the fp32 bar (|ΔJ| <= 1e-4, rel 1e-3) and the full-size states
against size-independent properties (x_N unitary, J recomputed from x_N).
The cavity known answer |<target|x_551>| = 0.999979 (examples/cavity_qubit.jl:75-81, the reference's own pulse
CSV, dim 24, 550 slices) is reproduced on the GPU.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHECK_SEEDS = 16


def _cpu(prob, u):
    import cpuref
    cpuref.use_blas(True)
    return cpuref.grape_eval_batch(prob, u, order=3, mode=0)


def _gpu(prob, u, chain=None):
    from qoc_amd import GrapeEngine
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=u.shape[0], precision=prob.precision)
    e.set_cost_trace(prob.x_target, prob.n)
    if chain:
        e.set_chain(chain)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    info = e.info()
    e.close()
    return J, g, info


def _check_config(name, seeds, chain=None, monkeypatch=None):
    from qoc_amd import systems
    if chain == "dense":  # the dense Taylor-action kernels (no block chains; qoc_blk.hpp)
        monkeypatch.setenv("QOC_BLOCKS", "0")
        chain = None
    if chain == "blkpoly":  # the block chains with the polynomial inside the recurrence (QOC_BLKU=0)
        monkeypatch.setenv("QOC_BLKU", "0")
        chain = None
    mk_prob, mk_u, B = systems.CONFIGS[name]
    prob = mk_prob()
    u = mk_u(B, 0)
    J, g, info = _gpu(prob, u, chain)
    assert np.all(np.isfinite(J)) and np.all(np.isfinite(g))
    idx = np.asarray(seeds)
    Jc, gc = _cpu(prob, u[idx])
    dJ = np.abs(J[idx] - Jc)
    rel = np.array([np.linalg.norm(g[b] - gc[i]) / np.linalg.norm(gc[i]) for i, b in enumerate(idx)])
    assert dJ.max() <= 1e-12, (name, info, dJ.max())
    assert rel.max() <= 1e-10, (name, info, rel.max())
    return info


# the chain kernels each variant must select: block propagators (qoc_blku.hpp, the default), the block chains with
# the polynomial inside the recurrence (qoc_blk.hpp), the dense Taylor-action chains, the reference's propagators
BLOCK_KERNEL = {"auto": "blocks_prop", "blkpoly": "blocks_mfma"}


@pytest.mark.parametrize("chain", ["auto", "blkpoly", "dense", "propagators"])
def test_zz_batch_full_size(built_lib, chain, monkeypatch):
    """config 2: zz_coupling N=9, m=4, Nt=500, B=512 (first and last seeds of the batch checked)."""
    seeds = list(range(CHECK_SEEDS // 2)) + list(range(512 - CHECK_SEEDS // 2, 512))
    info = _check_config("zz_batch", seeds, None if chain == "auto" else chain, monkeypatch)
    assert info["chain_kernel"] == BLOCK_KERNEL.get(chain, info["chain_kernel"]), info
    assert (info["chain_kernel"] in BLOCK_KERNEL.values()) == (chain in BLOCK_KERNEL), info


@pytest.mark.parametrize("chain", ["auto", "blkpoly", "dense", "propagators"])
def test_cavity_full_size(built_lib, chain, monkeypatch):
    """config 3: cavity(20) x qubit N=40, m=2, Nt=1000, B=256."""
    seeds = list(range(0, 256, 256 // CHECK_SEEDS))
    info = _check_config("cavity", seeds, None if chain == "auto" else chain, monkeypatch)
    assert info["chain_kernel"] == BLOCK_KERNEL.get(chain, info["chain_kernel"]), info
    assert (info["chain_kernel"] in BLOCK_KERNEL.values()) == (chain in BLOCK_KERNEL), info


@pytest.mark.parametrize("chain", ["auto", "propagators"])
def test_cavity_dense_full_size(built_lib, chain, monkeypatch):
    """config 3 with a drive that also displaces the cavity (systems.cavity_dense_problem: no invariant blocks): the
    dense Taylor-action chains on v_mfma_f64_4x4x4 and the fused order-3 gradient, N=40, Nt=1000, B=256, against
    the C port."""
    seeds = list(range(0, 256, 256 // CHECK_SEEDS))
    info = _check_config("cavity_dense", seeds, None if chain == "auto" else chain, monkeypatch)
    assert info["chain_kernel"] not in BLOCK_KERNEL.values() and info["chain_kernel"] != "blocks", info
    assert info["chain"] == ("propagators" if chain == "propagators" else "taylor"), info


@pytest.mark.parametrize("chain", ["auto", "dense", "propagators"])
def test_tunable_bus_full_size(built_lib, chain, monkeypatch):
    """config 4: two_qubit_tunable_bus N=27, m=1, Nt=2000, B=512 per GPU, ||A_k||_1 ~ 30: every seed against
    the C port, over 2000 chained slices: the default stored block propagators (propagate: k_blkp_exp + the forward
    chain, grape_sensitivity: the μ recurrence + k_blkp_grad), the dense Chebyshev Taylor-action chains (spectral
    radius ~14 per slice) and the propagators (the reference's Padé-13)."""
    info = _check_config("tunable_bus", list(range(512)), None if chain == "auto" else chain, monkeypatch)
    assert info["chain"] == ("propagators" if chain == "propagators" else "taylor")
    assert (info["chain_kernel"] == "blocks_prop16") == (chain == "auto"), info
    assert (info["backward"] == "blocks_prop16") == (chain == "auto"), info


def test_tunable_bus_full_size_device_eval(built_lib):
    """config 4 through the bench's entry point (qoc_eval_dev): the stored block propagators of the live 14-row block
    (k_blkp_exp / k_blkp_dual / k_blkp_grad, seed groups pipelined over two streams), every seed of B = 512 over
    Nt = 2000 slices against the C port."""
    import torch
    from qoc_amd import GrapeEngine, systems
    mk_prob, mk_u, B = systems.CONFIGS["tunable_bus"]
    prob = mk_prob()
    u = mk_u(B, 0)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
    Jd = torch.empty(B, dtype=torch.float64, device="cuda")
    gd = torch.empty(B, prob.Nt, prob.nu, dtype=torch.float64, device="cuda")
    e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
    e.synchronize()
    info = e.info()
    e.close()
    assert info["chain_kernel"] == "blocks_prop16" and info["backward"] == "blocks_prop16", info
    J = Jd.cpu().numpy()
    g = np.transpose(gd.cpu().numpy(), (0, 2, 1))
    Jc, gc = _cpu(prob, u)
    assert np.abs(J - Jc).max() <= 1e-12, np.abs(J - Jc).max()
    rel = max(np.linalg.norm(g[b] - gc[b]) / np.linalg.norm(gc[b]) for b in range(B))
    assert rel <= 1e-10, rel


def test_tunable_bus_every_rank_seeds(built_lib):
    """config 4 is 4096 seeds over 8 ranks, each rank's u seeded by its rank (bench.py mk_u(B, rank)): ranks 1..7 on
    this GPU (the stored block propagators through qoc_eval_dev), 64 seeds of each against the C port at the fp64 bar
    (rank 0's 512: test_tunable_bus_full_size_device_eval)."""
    import torch
    from qoc_amd import GrapeEngine, systems
    mk_prob, mk_u, B = systems.CONFIGS["tunable_bus"]
    prob = mk_prob()
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    worst = (0.0, 0.0)
    for rank in range(1, 8):
        u = mk_u(B, rank)
        ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
        Jd = torch.empty(B, dtype=torch.float64, device="cuda")
        gd = torch.empty(B, prob.Nt, prob.nu, dtype=torch.float64, device="cuda")
        e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
        e.synchronize()
        assert e.info()["backward"] == "blocks_prop16"
        idx = np.arange(0, B, B // 64)
        J = Jd.cpu().numpy()[idx]
        g = np.transpose(gd.cpu().numpy(), (0, 2, 1))[idx]
        Jc, gc = _cpu(prob, u[idx])
        dJ = np.abs(J - Jc).max()
        rel = max(np.linalg.norm(g[i] - gc[i]) / np.linalg.norm(gc[i]) for i in range(len(idx)))
        worst = (max(worst[0], dJ), max(worst[1], rel))
        assert dJ <= 1e-12, (rank, dJ)
        assert rel <= 1e-10, (rank, rel)
    e.close()
    print("tunable bus ranks 1..7, 64 seeds each: max |dJ|", worst[0], "max rel dJdu", worst[1])


def test_synthetic_full_size_fp32(built_lib, golden_dir):
    """config 5: synthetic GUE N=256, m=256 (x0 = I), nu=2, Nt=1000, B=128, fp32 on the large-N pipeline."""
    import qoc_oracle as O
    from qoc_amd import GrapeEngine, systems
    mk_prob, mk_u, B = systems.CONFIGS["synthetic"]
    prob = mk_prob()
    u = mk_u(B, 0)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B, precision="fp32")
    e.set_cost_trace(prob.x_target, prob.n)
    assert e.info()["path"] == "large_n"
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    assert np.all(np.isfinite(J)) and np.all(np.isfinite(g))
    for b in (0, B - 1):
        xN = e.state(prob.Nt, seed=b)
        # x0 = I: x_N is the product of 1000 unitaries; fp32 drift stays small
        assert np.abs(xN.conj().T @ xN - np.eye(prob.N)).max() < 5e-3
        Jr = 1 - abs(np.trace(prob.x_target.conj().T @ xN)) ** 2 / prob.n ** 2
        assert abs(J[b] - Jr) < 1e-4
    # all 1000 slices against the fp64 oracle's committed fixture (tests/golden/make_fullsize.py): seeds 0 and 127,
    # J, dJdu and x_N of seed 0, at the fp32 bar
    fx = np.load(golden_dir / "synthetic_full.npz")
    for i, b in enumerate(fx["seeds"]):
        assert abs(J[b] - fx["J"][i]) <= 1e-4, (b, J[b], fx["J"][i])
        rel = np.linalg.norm(g[b] - fx["dJdu"][i]) / np.linalg.norm(fx["dJdu"][i])
        assert rel <= 1e-3, (b, rel)
    xN0 = e.state(prob.Nt, seed=0)
    assert np.abs(xN0 - fx["x_final_seed0"]).max() <= 2e-4
    e.close()
    # bounded prefix of seed 0 against the fp64 numpy oracle
    n2 = 12
    e2 = GrapeEngine(prob.A0, prob.A, prob.x0, n2, B=1, precision="fp32")
    e2.set_cost_trace(prob.x_target, prob.n)
    u2 = np.ascontiguousarray(u[:1, :, :n2])
    Jg = e2.propagate(u2)
    gg = e2.grape_sensitivity(u2, 3)
    e2.close()
    Jr, gr, _ = O.grape_eval(prob.A0, prob.A, u2[0], prob.x0, prob.x_target, prob.n, order=3)
    assert abs(Jg[0] - Jr) <= 1e-4
    assert np.linalg.norm(gg[0] - gr) / np.linalg.norm(gr) <= 1e-3


@pytest.mark.parametrize("chain", ["auto", "propagators"])
def test_cavity_known_answer_on_gpu(built_lib, golden_dir, chain):
    """examples/cavity_qubit.jl:75-81: the reference's measured pulse (cavity_qubit_pulse_marina.csv x 1e-9,
    550 slices, dt = 1, generators setup_bilinear_matrices(H0, Tc/2, 1)), dim 24: |<target|x_551>| = 0.999979
    (printed to 6 digits by the reference; the oracle reproduces it to 3.4e-7)."""
    from qoc_amd import GrapeEngine, systems
    H0, Tc, theta = systems.cavity_model(12)
    A0, A1, A2 = systems.setup_bilinear_matrices(H0, Tc / 2, 1.0)
    iq = np.load(golden_dir / "cavity_qubit_pulse_marina.npy") * 1e-9
    u = np.ascontiguousarray(iq.T)[None]  # 1 x 2 x 550
    x0 = np.kron([1.0, 0.0], np.ones(12) / np.sqrt(12))[:, None].astype(complex)
    e = GrapeEngine(A0, [A1, A2], x0, u.shape[2], B=1)
    if chain != "auto":
        e.set_chain(chain)
    e.set_cost_external()
    e.propagate(u)
    xN = e.state(-1)[:, 0]
    e.close()
    tgt = np.kron([1.0, 0.0], np.exp(1j * theta))
    tgt = tgt / np.linalg.norm(tgt)
    assert abs(abs(np.vdot(tgt, xN)) - 0.999979) < 1e-6


@pytest.mark.parametrize("chain", ["auto", "propagators"])
def test_zz_measured_pulse_fixture(built_lib, golden_dir, chain):
    """examples/zz_coupling_simulation.jl:3-13: the reference's measured zz pulse (CSV x 1e-9, 500 slices,
    Δt = 20/500, x0 = Q_css) propagated on the GPU; x_501 against the fp64 oracle's fixture at 1e-13, and the
    NOT-gate cost / order-3 gradient of that pulse at the fp64 bar."""
    from qoc_amd import GrapeEngine, systems
    fx = np.load(golden_dir / "zz_pulse_fixture.npz")
    prob = systems.zz_problem(500)
    u = fx["u"][None]
    e = GrapeEngine(prob.A0, prob.A, prob.x0, 500, B=1)
    if chain != "auto":
        e.set_chain(chain)
    e.set_cost_trace(prob.x_target, prob.n)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    assert np.abs(e.state(500) - fx["x_final"]).max() <= 1e-13
    assert abs(J[0] - fx["J"]) <= 1e-12
    assert np.linalg.norm(g[0] - fx["dJdu"]) / np.linalg.norm(fx["dJdu"]) <= 1e-10
    e.close()
