"""CPU tests of the boundary and host logic (no GPU compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from qoc_amd import systems as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "qoc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(qoc_[a-z0-9_]+)\s*\(", txt)))


def test_library_builds_loads_and_exports_every_declared_symbol(built_lib):
    syms = _declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(built_lib, s), f"{s} declared in include/qoc.h but not exported"
    from qoc_amd import _lib
    assert set(_lib.SIGNATURES) == set(syms)


def test_library_is_built_from_the_sources_in_the_tree(built_lib, tmp_path, monkeypatch):
    """The library carries the sha256 of csrc/ + include/qoc.h; load() refuses one built from other sources."""
    from qoc_amd import _lib, _srchash
    assert built_lib.qoc_source_hash().decode() == "qoc-src-" + _srchash.source_hash()
    # a tree whose sources differ by one byte no longer matches the library
    src = tmp_path / "pkg" / "csrc"
    src.mkdir(parents=True)
    for f in _srchash.source_files()[:-1]:
        (src / os.path.basename(f)).write_bytes(open(f, "rb").read())
    hdr = tmp_path / "include"
    hdr.mkdir()
    (hdr / "qoc.h").write_bytes(open(_srchash.HEADER, "rb").read() + b"\n")
    monkeypatch.setattr(_srchash, "CSRC", str(src))
    monkeypatch.setattr(_srchash, "HEADER", str(hdr / "qoc.h"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.QOCError, match="built from other sources"):
        _lib.load()
    monkeypatch.setattr(_lib, "_lib", built_lib)


def test_last_error_without_context(built_lib):
    msg = built_lib.qoc_last_error(None)
    assert isinstance(msg, bytes)


def test_create_rejects_bad_dimensions_before_touching_the_gpu(built_lib):
    h = ctypes.c_void_p()
    rc = built_lib.qoc_create(ctypes.byref(h), 0, 0, 1, 1, 1, 1, 0)
    assert rc == -1 and not h.value
    assert b"invalid dimensions" in built_lib.qoc_last_error(None)
    rc = built_lib.qoc_create(ctypes.byref(h), 0, 200, 1, 9, 1, 1, 0)
    assert rc == -5  # beyond the LDS-resident kernels -> large-N path, which takes nu <= 8
    assert b"nu <= 8" in built_lib.qoc_last_error(None)


def test_engine_dimension_mismatch_message(built_lib):
    from qoc_amd import GrapeEngine
    with pytest.raises(ValueError, match="incompatiable dimensions"):
        GrapeEngine(np.eye(4), [np.eye(4)], np.ones((3, 1)), 10)


def test_layout_helpers_are_julia_layout():
    from qoc_amd.engine import _cm_complex, _from_cm, _u_layout
    a = np.arange(6).reshape(2, 3) + 1j * np.arange(6).reshape(2, 3)
    flat = _cm_complex(a)
    assert np.array_equal(flat, a.ravel(order="F"))
    assert np.array_equal(_from_cm(flat, 2, 3), a)
    u = np.arange(2 * 2 * 5, dtype=float).reshape(2, 2, 5)  # B, nu, Nt
    ub = _u_layout(u, 2, 2, 5)
    assert ub.ravel()[1 * 10 + 3 * 2 + 1] == u[1, 1, 3]  # u[b*nu*Nt + k*nu + j]


def test_quantum_basis_and_operators():
    qb = S.QuantumBasis([3, 3])
    assert qb("00") == 0 and qb("01") == 1 and qb("10") == 3 and qb("22") == 8
    a = S.annihilation_op(4)
    assert np.allclose(np.diag(a.T @ a), np.arange(4)) and np.allclose(a @ a.T - a.T @ a, np.diag([1, 1, 1, -3]))
    a1, a2 = S.annihilation_ops(2, 3)
    assert np.allclose(a1 @ a2, a2 @ a1)
    assert np.allclose(S.qubit_hamiltonian(1, 0, 5), np.diag(np.arange(5)))
    assert np.allclose(S.qubit_hamiltonian(0, 1, 5), np.diag([(k - 1) * k / 2 for k in range(5)]))


def test_bilinear_matrices_are_skew_hermitian():
    H0, Tc, _ = S.cavity_model(5)
    for A in S.setup_bilinear_matrices(H0, Tc, 0.3):
        assert np.allclose(A, -A.conj().T)


def test_spline_matrix():
    Bs = S.spline_matrix(10.0, 100, 10)
    assert Bs.shape == (100, 10) and (Bs >= 0).all()
    # interior cubic B-splines on a uniform grid: each has the same integral
    assert np.allclose(Bs.sum(0), Bs.sum(0)[0], rtol=1e-2)


def test_configs_match_baseline_shapes():
    for name, (N, m, nu, Nt, B) in {"zz_batch": (9, 4, 2, 500, 512), "cavity": (40, 2, 2, 1000, 256),
                                    "tunable_bus": (27, 1, 1, 2000, 512)}.items():
        mk, mu, Bd = S.CONFIGS[name]
        p = mk()
        assert (p.N, p.m, p.nu, p.Nt, Bd) == (N, m, nu, Nt, B)
        assert mu(2).shape == (2, nu, Nt)


def test_gate_unitaries():
    for g in ("CNOT", "iSwap", "CZ"):
        U = S.gate_unitary(g)
        assert np.allclose(U @ U.T, np.eye(4))
    with pytest.raises(ValueError):
        S.gate_unitary("T")


def test_compress_states_reference_vectors():
    """test/test_utils.jl:22-37 (1-based ranges shifted to 0-based)."""
    from qoc_amd import systems as S
    v = ((range(0, 27, 2), [0, 3]), (range(1, 26, 2), [1, 2]))
    x0 = np.arange(1, 27 * 4 + 1).reshape(4, 27).T.copy()   # collect(reshape(1:27*4, 27, 4))
    x0[np.ix_(range(0, 27, 2), [1, 2])] = 0
    x0[np.ix_(range(1, 26, 2), [0, 3])] = 0
    x1 = S.compress_states(x0, v)
    assert x1.shape[1] == 2
    assert np.array_equal(S.decompress_states(x1, v), x0)
    v = ((range(0, 27, 2), [0, 3, 4]), (range(1, 26, 2), [1, 2]))
    x0 = np.arange(1, 27 * 5 + 1).reshape(5, 27).T.copy()
    x0[np.ix_(range(0, 27, 2), [1, 2])] = 0
    x0[np.ix_(range(1, 26, 2), [0, 3, 4])] = 0
    x1 = S.compress_states(x0, v)
    assert x1.shape[1] == 3
    assert np.array_equal(S.decompress_states(x1, v), x0)


def test_compress_problem_rejects_coupling_generators():
    from qoc_amd import systems as S
    prob = S.zz_problem(10)
    v = ((range(0, 9, 2), [0, 3]), (range(1, 9, 2), [1, 2]))
    with pytest.raises(ValueError, match="couple"):
        S.compress_problem(prob, v)


def test_generators_recovered_from_reference_rhs_closures():
    """propagate_pwc(f, ...) takes the reference's right-hand side closure (examples/models/setup_diffeq_rhs.jl:
    rhs = (A0 + sum u_k A_k) x in the complex2real layout); the generators are recovered exactly, and
    anything that is not such a map is refused."""
    from qoc_amd import c2r, generators_from_rhs, r2c
    rng = np.random.default_rng(3)
    n = 5
    A0 = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
    A = [rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n)) for _ in range(2)]

    def dxdt(dx, x, p, t):
        dx[:] = c2r((A0 + p[0] * A[0] + p[1] * A[1]) @ r2c(x))
    M0, Ms = generators_from_rhs(dxdt, n, 2)
    assert np.abs(M0 - A0).max() < 1e-14 and all(np.abs(Mj - Aj).max() < 1e-14 for Mj, Aj in zip(Ms, A))

    def dldt3(dl, l, p):  # Symbolics' in-place signature, adjoint equation
        dl[:] = c2r(-(A0 + p[0] * A[0] + p[1] * A[1]).conj().T @ r2c(l))
    M0, _ = generators_from_rhs(dldt3, n, 2)
    assert np.abs(M0 + A0.conj().T).max() < 1e-14
    x = rng.standard_normal((2 * n, 3))
    assert np.array_equal(c2r(r2c(x)), x)

    def conj_rhs(dx, x, p, t):  # x -> conj(x): real-linear, not complex-linear
        dx[:] = c2r(np.conj(r2c(x)))
    with pytest.raises(ValueError):
        generators_from_rhs(conj_rhs, n, 2)

    def quad(dx, x, p, t):  # not affine in p
        dx[:] = c2r((A0 + p[0] ** 2 * A[0]) @ r2c(x))
    with pytest.raises(ValueError):
        generators_from_rhs(quad, n, 2)
