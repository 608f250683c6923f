"""Batched GRAPE engine on one MI355X (thin owner of a ``qoc_ctx``).

All heavy state (per-slice propagators U_k, states x_k, co-states λ_k) stays in HBM;
numpy arrays cross the boundary only for inputs and results, in Julia's memory layout
(column-major, interleaved complex).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

_dp = C.POINTER(C.c_double)


def _cm_complex(a: np.ndarray) -> np.ndarray:
    """Column-major interleaved complex128 copy (Julia ComplexF64 layout) as a flat array."""
    a = np.asarray(a, dtype=np.complex128)
    return np.ascontiguousarray(a.reshape(a.shape[0], -1).T).ravel()


def _from_cm(flat: np.ndarray, rows: int, cols: int) -> np.ndarray:
    return flat.reshape(cols, rows).T.copy()


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def _order(order) -> int:
    """dUkdp_order: 1..4 (Taylor, the reference's definition) or "exact" (Fréchet, QOC_DUKDP_EXACT = 0)."""
    if isinstance(order, str):
        if order != "exact":
            raise ValueError(f"dUkdp_order must be 1..4 or 'exact' (got {order!r})")
        return L.QOC_DUKDP_EXACT
    return int(order)


def _u_layout(u: np.ndarray, B: int, nu: int, Nt: int) -> np.ndarray:
    """(B, nu, Nt) or (nu, Nt) float64 -> contiguous B x (nu x Nt column-major)."""
    u = np.asarray(u, dtype=np.float64)
    if u.ndim == 2:
        u = u[None]
    if u.shape != (B, nu, Nt):
        raise ValueError(f"u has shape {u.shape}, expected {(B, nu, Nt)}")
    return np.ascontiguousarray(np.transpose(u, (0, 2, 1)))


class GrapeEngine:
    """B seeds sharing (A0, A_j, x0, target) on ``device`` (precision 'fp64' | 'fp32')."""

    def __init__(self, A0, A, x0, Nt: int, B: int = 1, precision: str = "fp64", device: int = 0):
        lib = L.load()
        A0 = np.asarray(A0, dtype=np.complex128)
        x0 = np.asarray(x0, dtype=np.complex128)
        if x0.ndim == 1:
            x0 = x0[:, None]
        self.N = A0.shape[0]
        if x0.shape[0] != self.N:
            raise ValueError("Error when creating cache, A0 and x0 have incompatiable dimensions")
        self.m = x0.shape[1]
        self.nu = len(A)
        self.Nt = int(Nt)
        self.B = int(B)
        self.precision = precision
        self.device = device
        prec = {"fp64": L.QOC_FP64, "fp32": L.QOC_FP32}[precision]
        h = C.c_void_p()
        L.check(lib.qoc_create(C.byref(h), device, self.N, self.m, self.nu, self.Nt, self.B, prec))
        self._h = h
        self._lib = lib
        self._gen_key = None
        self.set_generators(A0, A)
        self.set_x0(x0)
        self.cost_kind = None

    # ---- lifetime ----------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.qoc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        L.check(rc, self._h)

    # ---- configuration -----------------------------------------------------------
    def set_generators(self, A0, A):
        A0 = np.asarray(A0, dtype=np.complex128)
        key = (A0.tobytes(), tuple(np.asarray(a, dtype=np.complex128).tobytes() for a in A))
        if key == self._gen_key:
            return
        if len(A) != self.nu:
            raise ValueError(f"expected {self.nu} control generators, got {len(A)}")
        a0 = _cm_complex(A0).view(np.float64)
        aj = [_cm_complex(a).view(np.float64) for a in A]
        arr = (_dp * self.nu)(*[_ptr(a) for a in aj])
        self._chk(self._lib.qoc_set_generators(self._h, _ptr(a0), arr))
        self._gen_key = key

    def set_x0(self, x0, per_seed: bool = False):
        x0 = np.asarray(x0, dtype=np.complex128)
        if per_seed:
            flat = np.concatenate([_cm_complex(x) for x in x0]).view(np.float64)
        else:
            if x0.ndim == 1:
                x0 = x0[:, None]
            flat = _cm_complex(x0).view(np.float64)
        self._chk(self._lib.qoc_set_x0(self._h, _ptr(flat), int(per_seed)))
        self.x0 = x0

    def set_cost_trace(self, x_target, n=None):
        xt = np.asarray(x_target, dtype=np.complex128)
        if xt.ndim == 1:
            xt = xt[:, None]
        n = xt.shape[1] if n is None else n
        flat = _cm_complex(xt).view(np.float64)
        self._chk(self._lib.qoc_set_cost(self._h, L.QOC_COST_TRACE, _ptr(flat), float(n)))
        self.cost_kind = "trace"

    def set_cost_zcalibrated(self, x_target):
        flat = _cm_complex(x_target).view(np.float64)
        self._chk(self._lib.qoc_set_cost(self._h, L.QOC_COST_ZCAL, _ptr(flat), 4.0))
        self.cost_kind = "zcal"

    def set_cost_external(self):
        self._chk(self._lib.qoc_set_cost(self._h, L.QOC_COST_EXTERNAL, None, 1.0))
        self.cost_kind = "external"

    def set_state_penalty(self, inds_penalty, inds_css, mu):
        P = np.ascontiguousarray(inds_penalty, dtype=np.int32)
        Cc = np.ascontiguousarray(inds_css, dtype=np.int32)
        ip = C.POINTER(C.c_int)
        self._chk(self._lib.qoc_set_state_penalty(self._h, P.ctypes.data_as(ip), len(P), Cc.ctypes.data_as(ip),
                                                  len(Cc), float(mu)))

    def set_costate_source(self, dLdx):
        """dL_dx(x_k) of a caller's penalty closure for every seed and k = 0..Nt ((B, Nt+1, N, m) complex, or
        (Nt+1, N, m) for B = 1), added to λ_k by the following grape_sensitivity calls; None clears it."""
        if dLdx is None:
            self._chk(self._lib.qoc_set_costate_source(self._h, None))
            return
        d = np.asarray(dLdx, dtype=np.complex128)
        if d.ndim == 3:
            d = d[None]
        if d.shape != (self.B, self.Nt + 1, self.N, self.m):
            raise ValueError(f"dL_dx values must be (B, Nt+1, N, m) = {(self.B, self.Nt + 1, self.N, self.m)}")
        flat = np.ascontiguousarray(np.transpose(d, (0, 1, 3, 2))).ravel().view(np.float64)
        self._chk(self._lib.qoc_set_costate_source(self._h, _ptr(flat)))

    def set_compression(self, v):
        """compress_states inside the engine (src/utils.jl:96-109, include/qoc.h qoc_set_compression):
        v = ((rows1, cols1), (rows2, cols2)) with 0-based index sequences, as systems.compress_states takes
        it; the chains and the gradient then run on max(n1, n2) packed columns while every argument and
        result keeps the (N, m) layout.  None turns packing off."""
        ip = C.POINTER(C.c_int)
        if v is None:
            self._chk(self._lib.qoc_set_compression(self._h, None, 0, None, 0, None, 0, None, 0))
            return
        (r1, c1), (r2, c2) = v
        arrs = [np.ascontiguousarray(list(a), dtype=np.int32) for a in (r1, c1, r2, c2)]
        self._keep_cmp = arrs
        args = []
        for a in arrs:
            args += [a.ctypes.data_as(ip), len(a)]
        self._chk(self._lib.qoc_set_compression(self._h, *args))

    def set_propagation(self, method: str = "expm", nsub: int = 10):
        """'expm' (U_k = exp(A_k), default) or 'tsit5': the reference's ODE path (propagate_pwc /
        compute_pwc_gradient, src/gradient_computations.jl:108-169) with nsub fixed Tsit5 steps per
        slice (the reference's dt = 0.1 Δt is nsub = 10)."""
        m = {"expm": L.QOC_PROP_EXPM, "tsit5": L.QOC_PROP_TSIT5}[method]
        self._chk(self._lib.qoc_set_propagation(self._h, m, int(nsub)))
        self.prop_method, self.nsub = method, int(nsub)

    def propagate_envelope(self, kind: str, params, tgate: float, dt: float):
        """Continuous pulse c(t) (wrap_envelope, src/QuantumOptimalControl.jl:43-54) integrated with
        fixed-step Tsit5 on [0, tgate]: params (B, np) per seed -> (J (B,) or None, x(tgate) (B, N, m))."""
        P = np.ascontiguousarray(params, dtype=np.float64)
        if P.ndim == 1:
            P = P[None]
        if P.shape[0] != self.B:
            raise ValueError(f"params must be (B={self.B}, np), got {P.shape}")
        J = np.zeros(self.B)
        X = np.zeros(2 * self.B * self.N * self.m)
        self._chk(self._lib.qoc_propagate_envelope(self._h, L.QOC_ENV[kind], _ptr(P), P.shape[1], float(tgate),
                                                   float(dt), _ptr(J), _ptr(X)))
        Xc = X.view(np.complex128).reshape(self.B, self.N * self.m)
        xs = np.stack([_from_cm(x, self.N, self.m) for x in Xc])
        return (J if self.cost_kind == "trace" else None), xs

    # ---- hot path (host arrays) ---------------------------------------------------
    def propagate(self, u) -> np.ndarray:
        """Forward pass for all seeds; returns J (B,) = Jfinal(x_N) + sum_k L(x_k)."""
        ub = _u_layout(u, self.B, self.nu, self.Nt)
        J = np.zeros(self.B)
        self._chk(self._lib.qoc_propagate(self._h, _ptr(ub), _ptr(J)))
        return J

    def grape_sensitivity(self, u, order: int = 3, lambda_final=None) -> np.ndarray:
        """dJdu (B, nu, Nt); raises StaleCacheError unless u is the last propagated u."""
        ub = _u_layout(u, self.B, self.nu, self.Nt)
        lam = None
        if lambda_final is not None:
            lf = np.asarray(lambda_final, dtype=np.complex128)
            if lf.ndim == 2:
                lf = lf[None]
            lam = np.concatenate([_cm_complex(x) for x in lf]).view(np.float64)
        out = np.zeros((self.B, self.Nt, self.nu))
        self._chk(self._lib.qoc_grape_sensitivity(self._h, _ptr(ub), _order(order),
                                                  _ptr(lam) if lam is not None else None, _ptr(out)))
        return np.transpose(out, (0, 2, 1)).copy()

    # ---- hot path (device pointers, e.g. torch tensors on cuda) ---------------------
    def eval_device(self, d_u: int, order: int, d_J: int, d_dJdu: int):
        """f + f_grad on device-resident buffers (B x Nt x nu doubles in, B / B x Nt x nu out)."""
        self._chk(self._lib.qoc_eval_dev(self._h, C.c_void_p(d_u), _order(order), C.c_void_p(d_J),
                                         C.c_void_p(d_dJdu)))

    def propagate_device(self, d_u: int, d_J: int):
        self._chk(self._lib.qoc_propagate_dev(self._h, C.c_void_p(d_u), C.c_void_p(d_J)))

    def grape_sensitivity_device(self, d_u: int, order: int, d_dJdu: int):
        self._chk(self._lib.qoc_grape_sensitivity_dev(self._h, C.c_void_p(d_u), _order(order), C.c_void_p(d_dJdu)))

    # ---- spline parameterisation (examples/ipopt_callbacks_exp.jl:13-14, 28, 33-51) --------
    def set_spline_basis(self, Bs):
        """Bs: Nt x ns basis matrix (u_b = transpose(Bs c_b))."""
        Bs = np.asarray(Bs, dtype=np.float64)
        if Bs.ndim != 2 or Bs.shape[0] != self.Nt:
            raise ValueError(f"spline basis must be Nt x ns with Nt={self.Nt}, got {Bs.shape}")
        self.ns = Bs.shape[1]
        self._chk(self._lib.qoc_set_spline_basis(self._h, _ptr(np.asfortranarray(Bs).ravel(order="F")), self.ns))

    def eval_spline(self, c, order: int = 3):
        """c: (B, ns, nu) coefficients (Julia reshape(c, nsplines, nu) per seed) -> J (B,), dJdc (B, ns, nu)."""
        c = np.asarray(c, dtype=np.float64).reshape(self.B, self.ns, self.nu)
        cf = np.ascontiguousarray(np.transpose(c, (0, 2, 1)))  # column-major per seed
        J = np.zeros(self.B)
        g = np.zeros_like(cf)
        self._chk(self._lib.qoc_eval_spline(self._h, _ptr(cf), _order(order), _ptr(J), _ptr(g)))
        return J, np.transpose(g, (0, 2, 1)).copy()

    def propagate_spline(self, c):
        """Ipopt's f alone (examples/ipopt_callbacks_exp.jl:11-19): spline map + propagate + J, no sensitivity."""
        c = np.asarray(c, dtype=np.float64).reshape(self.B, self.ns, self.nu)
        cf = np.ascontiguousarray(np.transpose(c, (0, 2, 1)))
        J = np.zeros(self.B)
        self._chk(self._lib.qoc_propagate_spline(self._h, _ptr(cf), _ptr(J)))
        return J

    def sensitivity_spline(self, c, order: int = 3):
        """Ipopt's f_grad sensitivity (:21-31) for the coefficients of the last propagate_spline -> dJdc."""
        c = np.asarray(c, dtype=np.float64).reshape(self.B, self.ns, self.nu)
        cf = np.ascontiguousarray(np.transpose(c, (0, 2, 1)))
        g = np.zeros_like(cf)
        self._chk(self._lib.qoc_sensitivity_spline(self._h, _ptr(cf), _order(order), _ptr(g)))
        return np.transpose(g, (0, 2, 1)).copy()

    def eval_spline_device(self, d_c: int, order: int, d_J: int, d_dJdc: int):
        """Device pointers: c and dJdc are B x nu x ns doubles (column-major ns x nu per seed)."""
        self._chk(self._lib.qoc_eval_spline_dev(self._h, C.c_void_p(d_c), _order(order), C.c_void_p(d_J),
                                                C.c_void_p(d_dJdc)))

    def spline_constraints_device(self, d_c: int, d_g: int, d_gjac: int = 0):
        self._chk(self._lib.qoc_spline_constraints_dev(self._h, C.c_void_p(d_c), C.c_void_p(d_g),
                                                       C.c_void_p(d_gjac) if d_gjac else None))

    def stream(self) -> int:
        return self._lib.qoc_stream(self._h)

    def synchronize(self):
        self._chk(self._lib.qoc_synchronize(self._h))

    # ---- readback -------------------------------------------------------------------
    def state(self, k: int, seed: int = 0) -> np.ndarray:
        buf = np.zeros(2 * self.N * self.m)
        self._chk(self._lib.qoc_get_states(self._h, seed, k, _ptr(buf)))
        return _from_cm(buf.view(np.complex128), self.N, self.m)

    def costate(self, k: int, seed: int = 0) -> np.ndarray:
        buf = np.zeros(2 * self.N * self.m)
        self._chk(self._lib.qoc_get_costates(self._h, seed, k, _ptr(buf)))
        return _from_cm(buf.view(np.complex128), self.N, self.m)

    def propagator(self, k: int, seed: int = 0) -> np.ndarray:
        buf = np.zeros(2 * self.N * self.N)
        self._chk(self._lib.qoc_get_propagator(self._h, seed, k, _ptr(buf)))
        return _from_cm(buf.view(np.complex128), self.N, self.N)

    PHASES = ("k_expm", "k_chain_fwd", "k_chain_bwd", "k_grad")

    def set_profiling(self, enable: bool = True):
        self._chk(self._lib.qoc_set_profiling(self._h, int(enable)))

    def phase_times(self, reset: bool = False) -> dict:
        """{kernel: (total_ms, launches)} from hipEvents recorded on the engine stream."""
        ms = np.zeros(4)
        n = np.zeros(4, dtype=np.int64)
        self._chk(self._lib.qoc_phase_times(self._h, _ptr(ms), n.ctypes.data_as(C.POINTER(C.c_longlong)),
                                            int(reset)))
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.PHASES)}

    def info(self) -> dict:
        """Which pipeline the context runs (qoc_get_info): 'lds' kernels or the 'large_n' GEMM path."""
        v = np.zeros(14, dtype=np.int64)
        self._chk(self._lib.qoc_get_info_n(self._h, v.ctypes.data_as(C.POINTER(C.c_longlong)), v.size))
        return {"path": "large_n" if v[0] else "lds", "chunk": int(v[1]), "ns_iters": int(v[2]),
                "device_bytes": int(v[3]), "chain": "taylor" if v[4] == 1 else "propagators",
                "expm": {0: "pade", 1: "taylor_rr", 2: "ps_lds"}.get(int(v[5]), "?"),
                "chain_poly": "chebyshev" if v[6] else "taylor", "kernel_m": int(v[7]),
                "backward": {0: "generic", 1: "captured", 2: "concurrent", 3: "concurrent", 4: "blocks",
                             5: "fused", 6: "segmented", 7: "blocks_prop16"}.get(int(v[8]), "?"),
                "concurrent_launch": {2: "two_streams", 3: "dual", 4: "dual", 5: "fused",
                                      6: "segmented", 7: "dual"}.get(int(v[8])),
                "fwd_captured": bool(v[9]),
                "chain_kernel": {0: None, 1: "mfma_lds", 2: "mfma_regs", 3: "blocks", 4: "blocks_mfma", 5: "blocks_prop",
                                 6: "blocks_prop16"}.get(int(v[10])),
                "split_forward": {0: "states", 1: "segmented", 2: "blocks_prop16"}.get(int(v[11])),
                "interp_degree": int(v[12]), "interp_chain": int(v[13])}

    def set_chain(self, mode: str = "auto"):
        """How the chains apply exp(A_k) (include/qoc.h qoc_set_chain): 'propagators' forms every U_k (the
        reference's structure), 'taylor' applies the exponential to the state directly, 'auto' chooses by
        the generator norms."""
        self._chk(self._lib.qoc_set_chain(self._h, L.QOC_CHAIN[mode]))

    # ---- multi-GPU epilogue (include/qoc.h qoc_comm_* / qoc_allgather_best) -------------
    def comm_init(self, world: int, rank: int, unique_id: bytes | None, seed_offset: int):
        """Join the RCCL communicator of `world` ranks (unique_id: the QOC_UNIQUE_ID_BYTES bytes one rank made
        with comm_unique_id(); with world = 1 it makes a one-rank communicator, None makes none).
        seed_offset: global id of this context's seed 0."""
        buf = C.create_string_buffer(bytes(unique_id), 128) if unique_id is not None else None
        self._chk(self._lib.qoc_comm_init(self._h, int(world), int(rank), buf, int(seed_offset)))

    def comm_ranks(self) -> int:
        """Ranks of the engine's RCCL communicator (0: none; the epilogue then covers this engine alone)."""
        r = self._lib.qoc_comm_ranks(self._h)
        self._chk(min(r, 0))
        return int(r)

    def allgather_best(self):
        """(J_best, global seed) of the last propagate over every rank of the communicator."""
        J = C.c_double()
        s = C.c_int()
        self._chk(self._lib.qoc_allgather_best(self._h, C.byref(J), C.byref(s)))
        return J.value, s.value

    def allgather_best_device(self, d_out: int):
        """Same, written as two doubles to device memory on the engine stream (no host synchronisation)."""
        self._chk(self._lib.qoc_allgather_best_dev(self._h, C.c_void_p(d_out)))

    def set_best_output(self, d_out: int):
        """Register a device buffer of two doubles (0: none): with one rank, the segmented eval writes the best
        (J, seed) there itself and allgather_best_device(d_out) queues nothing more (qoc_set_best_output)."""
        self._chk(self._lib.qoc_set_best_output(self._h, C.c_void_p(d_out or None)))

    def chain_terms(self, reset: bool = False) -> int:
        """Taylor terms executed per direction since the last reset (Taylor-action chains)."""
        v = C.c_longlong()
        self._chk(self._lib.qoc_chain_terms(self._h, C.byref(v), int(reset)))
        return int(v.value)

    def gemm_stats(self, reset: bool = False) -> dict:
        """Large-N path: live HIP-event time / launches / algorithmic FLOPs of the k_bgemm launches."""
        ms, fl = C.c_double(), C.c_double()
        n = C.c_longlong()
        self._chk(self._lib.qoc_gemm_stats(self._h, C.byref(ms), C.byref(n), C.byref(fl), int(reset)))
        return {"ms": ms.value, "launches": n.value, "flops": fl.value}

    def taylor_histogram(self, reset: bool = False) -> dict:
        """Executed Taylor counts {(m, s): count}: degree m = 3r+2 by Paterson-Stockmeyer (2 + r GEMMs),
        m = 12 by the 4-GEMM scheme, m = "8t" by the 3-GEMM degree-8 scheme (large-N path), with s squarings
        (include/qoc.h: qoc_taylor_histogram)."""
        h = np.zeros(9 * 64, dtype=np.int64)
        self._chk(self._lib.qoc_taylor_histogram_n(self._h, h.ctypes.data_as(C.POINTER(C.c_longlong)), h.size,
                                                   int(reset)))
        # row 8: the 3-product degree-8 scheme (large-N path), reported as m = "8t" to keep it apart from
        # Paterson-Stockmeyer's degree 8 (row 0, 4 GEMMs)
        return {("8t" if i // 64 == 8 else 12 if i // 64 == 7 else 3 * (i // 64 + 2) + 2, i % 64): int(v)
                for i, v in enumerate(h) if v}

    def pade_histogram(self, reset: bool = False) -> dict:
        h = np.zeros(5 * 64, dtype=np.int64)
        self._chk(self._lib.qoc_pade_histogram(self._h, h.ctypes.data_as(C.POINTER(C.c_longlong)), int(reset)))
        out = {}
        for di, d in enumerate((3, 5, 7, 9, 13)):
            for s in range(64):
                if h[di * 64 + s]:
                    out[(d, s)] = int(h[di * 64 + s])
        return out


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (128 bytes) for qoc_comm_init; made on one rank and sent to the others."""
    lib = L.load()
    buf = C.create_string_buffer(128)
    L.check(lib.qoc_comm_unique_id(buf))
    return buf.raw


def expm(A, precision: str = "fp64", device: int = 0, return_degrees: bool = False):
    """Batched exponential!(A, ExpMethodHigham2005()) on the GPU; A is (N,N) or (count,N,N)."""
    lib = L.load()
    A = np.asarray(A, dtype=np.complex128)
    single = A.ndim == 2
    if single:
        A = A[None]
    cnt, N, _ = A.shape
    flat = np.concatenate([_cm_complex(a) for a in A]).view(np.float64)
    out = np.zeros_like(flat)
    deg = np.zeros(cnt, dtype=np.int32)
    sq = np.zeros(cnt, dtype=np.int32)
    ip = C.POINTER(C.c_int)
    L.check(lib.qoc_expm_batched(device, N, cnt, {"fp64": L.QOC_FP64, "fp32": L.QOC_FP32}[precision],
                                 _ptr(flat), _ptr(out), deg.ctypes.data_as(ip), sq.ctypes.data_as(ip)))
    X = np.stack([_from_cm(x, N, N) for x in out.view(np.complex128).reshape(cnt, N * N)])
    X = X[0] if single else X
    return (X, deg, sq) if return_degrees else X


def expm_jacobian(A0, A, p, order=2, dt=1.0, device: int = 0) -> list:
    """expm_jacobian! (src/gradient_computations.jl:177-213) on the GPU; returns nu N x N matrices."""
    lib = L.load()
    A0 = np.asarray(A0, dtype=np.complex128)
    N = A0.shape[0]
    nu = len(A)
    a0 = _cm_complex(A0).view(np.float64)
    aj = [_cm_complex(a).view(np.float64) for a in A]
    arr = (_dp * nu)(*[_ptr(a) for a in aj])
    pp = np.ascontiguousarray(p, dtype=np.float64)
    out = np.zeros(2 * N * N * nu)
    L.check(lib.qoc_expm_jacobian(device, N, nu, _ptr(a0), arr, _ptr(pp), int(order), float(dt), _ptr(out)))
    return [_from_cm(x, N, N) for x in out.view(np.complex128).reshape(nu, N * N)]
