"""The reference's own call form on the fast kernels: Ipopt's f calls propagate, its f_grad grape_sensitivity
(examples/ipopt_callbacks_exp.jl:11-31; src/gradient_computations.jl:2-32 and :35-77), as two C-ABI calls.

* generators with invariant blocks of 2-3 rows (cavity, zz): propagate runs the segmented eval's phases 0-2
  (csrc/qoc_blkseg.hpp BLKSEG_FWD: J, the λ_N coefficients and G at every segment's end), grape_sensitivity its phase 3
  (BLKSEG_BWD); J and dJdu are bitwise those of the one-launch eval (qoc_eval_dev);
* blocks of 5..16 rows (tunable bus): propagate forms every U_k on MFMA and runs the forward chain (k_blkp_exp +
  k_blkp_chain), grape_sensitivity the μ recurrence and the order-3 gradient on the stored propagators.

Against the oracle / the C port at the fp64 bar of SURVEY.md §8c (|ΔJ| <= 1e-12, ||ΔdJdu|| / ||dJdu|| <= 1e-10 per
seed), plus the stale-u contract (src/gradient_computations.jl:37-39) on both the host and the device entry points.
"""
import numpy as np
import pytest

import qoc_oracle as O

pytestmark = pytest.mark.gpu


def _env(monkeypatch, **kv):
    for k, v in kv.items():
        if v is None:
            monkeypatch.delenv(k, raising=False)
        else:
            monkeypatch.setenv(k, str(v))


def _engine(prob, B, monkeypatch, split="1"):
    from qoc_amd import GrapeEngine
    _env(monkeypatch, QOC_BLOCKS="1", QOC_BLKU="1", QOC_BLKSEG="1", QOC_BLKP="1", QOC_BLKSEG_SPLIT=split,
         QOC_BLKP_SPLIT=split)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_chain("taylor")
    return e


def _dev(u):
    import torch
    return torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()


def _bufs(B, Nt, nu):
    import torch
    return (torch.full((B,), np.nan, dtype=torch.float64, device="cuda"),
            torch.full((B, Nt, nu), np.nan, dtype=torch.float64, device="cuda"))


def _host(t, kind):
    a = t.cpu().numpy()
    return a if kind == "J" else np.transpose(a, (0, 2, 1))


def _split_dev(e, u, order=3):
    B, nu, Nt = u.shape
    ud = _dev(u)
    Jd, gd = _bufs(B, Nt, nu)
    e.propagate_device(ud.data_ptr(), Jd.data_ptr())
    e.grape_sensitivity_device(ud.data_ptr(), order, gd.data_ptr())
    e.synchronize()
    return _host(Jd, "J"), _host(gd, "g")


def _fused_dev(e, u, order=3):
    B, nu, Nt = u.shape
    ud = _dev(u)
    Jd, gd = _bufs(B, Nt, nu)
    e.eval_device(ud.data_ptr(), order, Jd.data_ptr(), gd.data_ptr())
    e.synchronize()
    return _host(Jd, "J"), _host(gd, "g")


def _assert_seed(J, g, Jr, gr, tag):
    assert abs(J - Jr) <= 1e-12, (tag, J - Jr)
    rel = np.linalg.norm(g - gr) / np.linalg.norm(gr)
    assert rel <= 1e-10, (tag, rel)


def _small_cases():
    from qoc_amd import systems
    out = {}
    p = systems.zz_problem(60, tgate=6.0)  # N = 9, 3 blocks of 3, m = 4
    out["zz"] = (p, systems.zz_controls(3, 60, 6.0, seed=181))
    p = systems.cavity_problem(N_cavity=10, Nt=50)  # N = 20, 10 blocks of 2
    out["cavity20"] = (p, systems.cavity_controls(3, p.Nt, seed=182))
    p = systems.cavity_problem(N_cavity=20, Nt=77)  # N = 40, 20 blocks of 2
    out["cavity40"] = (p, systems.cavity_controls(2, p.Nt, seed=183))
    p = systems.tunable_bus_problem(Nt=37, tgate=350.0 * 37 / 2000)  # one live 14-row block, Nt not a chunk multiple
    out["tunable_bus"] = (p, systems.tunable_bus_controls(3, 37, seed=184))
    return out


SPLIT_KIND = {"zz": "segmented", "cavity20": "segmented", "cavity40": "segmented", "tunable_bus": "blocks_prop16"}


@pytest.mark.parametrize("name", ["zz", "cavity20", "cavity40", "tunable_bus"])
def test_split_call_matches_oracle_and_fused_eval(built_lib, monkeypatch, name):
    """propagate + grape_sensitivity (host arrays: the Julia shim's calls) against the oracle, and bitwise against the
    one-launch device eval; then the device entry points (qoc_propagate_dev + qoc_grape_sensitivity_dev) alike."""
    prob, u = _small_cases()[name]
    B = u.shape[0]
    e = _engine(prob, B, monkeypatch)
    J = e.propagate(u)
    assert e.info()["split_forward"] == SPLIT_KIND[name], e.info()
    g = e.grape_sensitivity(u, 3)
    info = e.info()
    assert info["backward"] == SPLIT_KIND[name], info
    Jd, gd = _split_dev(e, u)
    Jf, gf = _fused_dev(e, u)
    assert e.info()["split_forward"] == "states"  # the eval leaves no split forward behind
    e.close()
    for b in range(B):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (name, b))
    assert np.array_equal(J, Jd) and np.array_equal(g, gd)
    assert np.array_equal(J, Jf) and np.array_equal(g, gf), (np.abs(J - Jf).max(), np.abs(g - gf).max())


@pytest.mark.parametrize("name", ["zz", "cavity20"])
def test_split_every_order_after_one_propagate(built_lib, monkeypatch, name):
    """One propagate, then grape_sensitivity at orders 4, 1, 3, 2 (src/gradient_computations.jl:177-213): each from
    the same stored segment ends."""
    prob, u = _small_cases()[name]
    e = _engine(prob, u.shape[0], monkeypatch)
    e.propagate(u)
    gs = {o: e.grape_sensitivity(u, o) for o in (4, 1, 3, 2)}
    assert e.info()["backward"] == "segmented"
    e.close()
    for b in range(u.shape[0]):
        for o, go in gs.items():
            J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=o)
            _assert_seed(J0, go[b], J0, g0, (name, o, b))


def test_split_tunable_bus_other_orders_fall_back(built_lib, monkeypatch):
    """Stored block propagators: order 3 on them; orders 1, 2 and 4 from the forward's states by the block chains."""
    prob, u = _small_cases()["tunable_bus"]
    e = _engine(prob, u.shape[0], monkeypatch)
    e.propagate(u)
    gs = {}
    for o in (1, 3, 4, 2):
        gs[o] = e.grape_sensitivity(u, o)
        assert (e.info()["backward"] == "blocks_prop16") == (o == 3), (o, e.info())
    e.close()
    for b in range(u.shape[0]):
        for o, go in gs.items():
            J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=o)
            _assert_seed(J0, go[b], J0, g0, (o, b))


@pytest.mark.parametrize("name", ["zz", "cavity40", "tunable_bus"])
def test_split_states_and_costates(built_lib, monkeypatch, name):
    """After propagate the states (rebuilt on demand for the segmented forward) are the oracle's; after
    grape_sensitivity the co-states are."""
    prob, u = _small_cases()[name]
    B = u.shape[0]
    e = _engine(prob, B, monkeypatch)
    e.propagate(u)
    ks = (0, 1, prob.Nt // 2, prob.Nt)
    xs = [e.state(k, seed=B - 1) for k in ks]
    e.grape_sensitivity(u, 3)
    lams = [e.costate(k, seed=B - 1) for k in ks]
    e.close()
    _, _, c0 = O.grape_eval(prob.A0, prob.A, u[B - 1], prob.x0, prob.x_target, prob.n, order=3)
    xsc = max(np.abs(x).max() for x in c0.x)
    lsc = max(np.abs(lam).max() for lam in c0.lam)
    for k, x, lam in zip(ks, xs, lams):
        assert np.abs(x - c0.x[k]).max() <= 1e-12 * xsc, ("x", k)
        assert np.abs(lam - c0.lam[k]).max() <= 1e-12 * lsc, ("lambda", k)


@pytest.mark.parametrize("name", ["cavity20", "tunable_bus"])
def test_split_stale_u_device_and_host(built_lib, monkeypatch, name):
    """src/gradient_computations.jl:37-39: a u other than the propagated one raises "Cache data from other control
    signal u" -- on the device entry point the split backward is queued behind the comparison and writes nothing (the
    caller's dJdu buffer keeps its contents, the co-states stay the last sensitivity's); the same u then works."""
    from qoc_amd import StaleCacheError
    prob, u = _small_cases()[name]
    B, nu, Nt = u.shape
    e = _engine(prob, B, monkeypatch)
    J1, g1 = _split_dev(e, u)  # a first sensitivity: its co-states must survive the stale call
    lam1 = e.costate(Nt // 2, seed=1)
    u2 = u.copy()
    u2[1, 0, Nt // 3] += 1e-9
    ud, ud2 = _dev(u), _dev(u2)
    Jd, gd = _bufs(B, Nt, nu)
    e.propagate_device(ud.data_ptr(), Jd.data_ptr())
    with pytest.raises(StaleCacheError):
        e.grape_sensitivity_device(ud2.data_ptr(), 3, gd.data_ptr())
    e.synchronize()
    assert np.all(np.isnan(gd.cpu().numpy()))
    assert np.array_equal(e.costate(Nt // 2, seed=1), lam1)
    e.grape_sensitivity_device(ud.data_ptr(), 3, gd.data_ptr())
    e.synchronize()
    assert np.array_equal(_host(gd, "g"), g1)
    # host entry points
    e.propagate(u)
    with pytest.raises(StaleCacheError):
        e.grape_sensitivity(u2, 3)
    assert np.array_equal(e.grape_sensitivity(u, 3), g1)
    e.close()


def test_split_then_setters_invalidate(built_lib, monkeypatch):
    """A setter between propagate and grape_sensitivity invalidates the stored forward ("called before propagate"),
    and a propagate after an eval, or an eval after a propagate, never mixes their buffers."""
    from qoc_amd import QOCError
    prob, u = _small_cases()["cavity20"]
    e = _engine(prob, u.shape[0], monkeypatch)
    e.propagate(u)
    e.set_cost_trace(prob.x_target, prob.n)
    with pytest.raises(QOCError):
        e.grape_sensitivity(u, 3)
    # propagate(u) -> eval(u2) -> grape_sensitivity(u2) must be the gradient at u2
    u2 = u[::-1].copy()
    e.propagate(u)
    _fused_dev(e, u2)
    g2 = e.grape_sensitivity(u2, 3)
    e.close()
    for b in range(u.shape[0]):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u2[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J0, g2[b], J0, g0, b)


def test_split_spline_callbacks_match_eval(built_lib, monkeypatch):
    """The Julia shim's Ipopt callbacks (propagate_spline -> sensitivity_spline, examples/ipopt_callbacks_exp.jl:11-31)
    on the split kernels: bitwise the one-call spline eval."""
    from qoc_amd import systems
    prob = systems.zz_problem(100)
    Bs = systems.spline_matrix(10.0, 100, 10)
    rng = np.random.default_rng(7)
    c = rng.uniform(-0.3, 0.3, size=(4, 10, 2))
    e = _engine(prob, 4, monkeypatch)
    e.set_spline_basis(Bs)
    J = e.propagate_spline(c)
    g = e.sensitivity_spline(c, 3)
    assert e.info()["backward"] == "segmented"
    Je, ge = e.eval_spline(c, 3)
    e.close()
    assert np.array_equal(J, Je) and np.array_equal(g, ge)
    for b in range(4):
        u = (Bs @ c[b]).T
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u, prob.x0, prob.x_target, prob.n, order=3)
        assert abs(J[b] - J0) <= 1e-12
        g0c = Bs.T @ g0.T
        assert np.linalg.norm(g[b] - g0c) / np.linalg.norm(g0c) <= 1e-10


def test_split_zz_plumbing_single_seed(built_lib, monkeypatch):
    """BASELINE config 1 (examples/zz_coupling_ipopt_exp.jl: N = 9, Nt = 100, B = 1) in the reference's call form."""
    from qoc_amd import systems
    mk_prob, mk_u, B = systems.CONFIGS["zz_plumbing"]
    prob, u = mk_prob(), mk_u(1, 0)
    e = _engine(prob, 1, monkeypatch)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    assert e.info()["backward"] == "segmented"
    e.close()
    J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[0], prob.x0, prob.x_target, prob.n, order=3)
    _assert_seed(J[0], g[0], J0, g0, "zz_plumbing")


@pytest.mark.parametrize("name,B", [("cavity", 256), ("zz_batch", 512)])
def test_split_full_size(built_lib, monkeypatch, name, B):
    """BASELINE configs 3 and 2 at full size in the reference's call form: 16 seeds against the C port of the
    reference, every seed bitwise against the one-launch eval."""
    import cpuref
    from qoc_amd import systems
    mk_prob, mk_u, Bd = systems.CONFIGS[name]
    assert Bd == B
    prob = mk_prob()
    u = mk_u(B, 0)
    e = _engine(prob, B, monkeypatch)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    info = e.info()
    assert info["backward"] == "segmented" and info["split_forward"] == "segmented", info
    Jf, gf = _fused_dev(e, u)
    e.close()
    assert np.array_equal(J, Jf) and np.array_equal(g, gf)
    idx = np.asarray(list(range(8)) + list(range(B - 8, B)))
    cpuref.use_blas(True)
    Jc, gc = cpuref.grape_eval_batch(prob, u[idx], order=3, mode=0)
    for i, b in enumerate(idx):
        _assert_seed(J[b], g[b], Jc[i], gc[i], (name, b))


def test_split_tunable_bus_full_size(built_lib, monkeypatch):
    """BASELINE config 4 per GPU (N = 27, Nt = 2000, B = 512) in the reference's call form on the stored block
    propagators: every seed against the C port, and bitwise against the device eval."""
    import cpuref
    from qoc_amd import systems
    mk_prob, mk_u, B = systems.CONFIGS["tunable_bus"]
    prob = mk_prob()
    u = mk_u(B, 0)
    e = _engine(prob, B, monkeypatch)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    info = e.info()
    assert info["backward"] == "blocks_prop16" and info["split_forward"] == "blocks_prop16", info
    Jf, gf = _fused_dev(e, u)
    e.close()
    assert np.array_equal(J, Jf) and np.array_equal(g, gf)
    cpuref.use_blas(True)
    Jc, gc = cpuref.grape_eval_batch(prob, u, order=3, mode=0)
    assert np.abs(J - Jc).max() <= 1e-12, np.abs(J - Jc).max()
    rel = max(np.linalg.norm(g[b] - gc[b]) / np.linalg.norm(gc[b]) for b in range(B))
    assert rel <= 1e-10, rel


@pytest.mark.parametrize("ch", [1, 2, 4, 8])
@pytest.mark.parametrize("parts", [1, 3, 5])
def test_blkp_chunk_tails_and_slab_ring(built_lib, monkeypatch, ch, parts):
    """The stored-propagator chains at every chunk size with Nt = 37 (a partial last chunk: the early break, the
    clamped DMA slices, the sink flushes), and the eval's two-slab ring over 1, 3 and 5 seed groups (the formation of
    group p + 2 waits for the chains of group p): eval and split call against the oracle."""
    _env(monkeypatch, QOC_BLKP_CH=ch, QOC_BLKP_PARTS=parts)
    prob, u = _small_cases()["tunable_bus"]
    u = np.concatenate([u, u[:, :, ::-1] * 0.9, u * 0.8])[:7]
    e = _engine(prob, u.shape[0], monkeypatch)
    Jf, gf = _fused_dev(e, u)
    assert e.info()["backward"] == "blocks_prop16"
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    e.close()
    assert np.array_equal(J, Jf) and np.array_equal(g, gf)
    for b in range(u.shape[0]):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, (ch, parts, b))


def test_blkp_cz_two_live_blocks_split(built_lib, monkeypatch):
    """The tunable bus' CZ variant (m = 4: both parity blocks live, 8 chain waves, the 2-slice chunk) in the split
    call form."""
    from qoc_amd import systems
    Nt = 29
    prob = systems.tunable_bus_cz_problem(Nt=Nt, tgate=350.0 * Nt / 2000)
    u = systems.tunable_bus_controls(2, Nt, seed=185)
    e = _engine(prob, 2, monkeypatch)
    J = e.propagate(u)
    g = e.grape_sensitivity(u, 3)
    assert e.info()["backward"] == "blocks_prop16"
    e.close()
    for b in range(2):
        J0, g0, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=3)
        _assert_seed(J[b], g[b], J0, g0, b)
