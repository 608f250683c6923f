"""ctypes binding of libqoc_mi355x.so (the C ABI in include/qoc.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).  There is
no CPU fallback: if the library is missing or cannot be loaded every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# QOC_LIB_PATH: another build of the same library (same-box A/B comparisons of kernel variants)
LIB_PATH = os.environ.get("QOC_LIB_PATH") or os.path.join(_HERE, "libqoc_mi355x.so")

QOC_OK = 0
QOC_ERR_ARG = -1
QOC_ERR_HIP = -2
QOC_ERR_STALE = -3
QOC_ERR_STATE = -4
QOC_ERR_UNSUPPORTED = -5
QOC_FP64 = 0
QOC_FP32 = 1
QOC_DUKDP_EXACT = 0
QOC_COST_TRACE = 0
QOC_COST_ZCAL = 1
QOC_COST_EXTERNAL = 2
QOC_PROP_EXPM = 0
QOC_PROP_TSIT5 = 1
QOC_ENV = {"tunable_bus": 0, "drag": 1, "sinebasis": 2}
QOC_CHAIN = {"auto": -1, "propagators": 0, "taylor": 1}

# Every symbol include/qoc.h declares, with (restype, argtypes).
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
_vp = C.c_void_p
SIGNATURES = {
    "qoc_create": (C.c_int, [C.POINTER(_vp), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "qoc_destroy": (None, [_vp]),
    "qoc_last_error": (C.c_char_p, [_vp]),
    "qoc_source_hash": (C.c_char_p, []),
    "qoc_stream": (_vp, [_vp]),
    "qoc_synchronize": (C.c_int, [_vp]),
    "qoc_set_generators": (C.c_int, [_vp, _dp, C.POINTER(_dp)]),
    "qoc_set_x0": (C.c_int, [_vp, _dp, C.c_int]),
    "qoc_set_cost": (C.c_int, [_vp, C.c_int, _dp, C.c_double]),
    "qoc_set_state_penalty": (C.c_int, [_vp, _ip, C.c_int, _ip, C.c_int, C.c_double]),
    "qoc_set_costate_source": (C.c_int, [_vp, _dp]),
    "qoc_set_compression": (C.c_int, [_vp, _ip, C.c_int, _ip, C.c_int, _ip, C.c_int, _ip, C.c_int]),
    "qoc_propagate": (C.c_int, [_vp, _dp, _dp]),
    "qoc_grape_sensitivity": (C.c_int, [_vp, _dp, C.c_int, _dp, _dp]),
    "qoc_propagate_dev": (C.c_int, [_vp, _vp, _vp]),
    "qoc_grape_sensitivity_dev": (C.c_int, [_vp, _vp, C.c_int, _vp]),
    "qoc_eval_dev": (C.c_int, [_vp, _vp, C.c_int, _vp, _vp]),
    "qoc_get_states": (C.c_int, [_vp, C.c_int, C.c_int, _dp]),
    "qoc_get_costates": (C.c_int, [_vp, C.c_int, C.c_int, _dp]),
    "qoc_get_propagator": (C.c_int, [_vp, C.c_int, C.c_int, _dp]),
    "qoc_set_profiling": (C.c_int, [_vp, C.c_int]),
    "qoc_phase_times": (C.c_int, [_vp, _dp, C.POINTER(C.c_longlong), C.c_int]),
    "qoc_pade_histogram": (C.c_int, [_vp, C.POINTER(C.c_longlong), C.c_int]),
    "qoc_taylor_histogram": (C.c_int, [_vp, C.POINTER(C.c_longlong), C.c_int]),
    "qoc_taylor_histogram_n": (C.c_int, [_vp, C.POINTER(C.c_longlong), C.c_int, C.c_int]),
    "qoc_set_propagation": (C.c_int, [_vp, C.c_int, C.c_int]),
    "qoc_propagate_envelope": (C.c_int, [_vp, C.c_int, _dp, C.c_int, C.c_double, C.c_double, _dp, _dp]),
    "qoc_get_info": (C.c_int, [_vp, C.POINTER(C.c_longlong)]),
    "qoc_get_info_n": (C.c_int, [_vp, C.POINTER(C.c_longlong), C.c_int]),
    "qoc_set_chain": (C.c_int, [_vp, C.c_int]),
    "qoc_comm_unique_id": (C.c_int, [_vp]),
    "qoc_comm_init": (C.c_int, [_vp, C.c_int, C.c_int, _vp, C.c_longlong]),
    "qoc_comm_ranks": (C.c_int, [_vp]),
    "qoc_allgather_best": (C.c_int, [_vp, _dp, _ip]),
    "qoc_allgather_best_dev": (C.c_int, [_vp, _vp]),
    "qoc_set_best_output": (C.c_int, [_vp, _vp]),
    "qoc_chain_terms": (C.c_int, [_vp, C.POINTER(C.c_longlong), C.c_int]),
    "qoc_set_spline_basis": (C.c_int, [_vp, _dp, C.c_int]),
    "qoc_eval_spline_dev": (C.c_int, [_vp, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "qoc_eval_spline": (C.c_int, [_vp, _dp, C.c_int, _dp, _dp]),
    "qoc_propagate_spline": (C.c_int, [_vp, _dp, _dp]),
    "qoc_sensitivity_spline": (C.c_int, [_vp, _dp, C.c_int, _dp]),
    "qoc_spline_constraints_dev": (C.c_int, [_vp, C.c_void_p, C.c_void_p, C.c_void_p]),
    "qoc_gemm_stats": (C.c_int, [_vp, _dp, C.POINTER(C.c_longlong), _dp, C.c_int]),
    "qoc_expm_batched": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _ip, _ip]),
    "qoc_expm_jacobian": (C.c_int, [C.c_int, C.c_int, C.c_int, _dp, C.POINTER(_dp), _dp, C.c_int, C.c_double, _dp]),
}


class QOCError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[qoc {code}] {msg}")
        self.code = code


class StaleCacheError(QOCError, ValueError):
    """Raised like the reference's ``error("Cache data from other control signal u")``."""


_lib = None


def load() -> C.CDLL:
    """Load the HIP library (raises if it was not built — there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise QOCError(QOC_ERR_STATE, f"{LIB_PATH} not built; run __graft_entry__.build()")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if not os.environ.get("QOC_LIB_PATH"):  # variant builds for A/B runs carry no hash
        from ._srchash import source_hash
        want = source_hash()
        have = lib.qoc_source_hash().decode().removeprefix("qoc-src-")
        if want is not None and have != want:
            raise QOCError(QOC_ERR_STATE, f"{LIB_PATH} was built from other sources (hash {have[:12]}, tree "
                                          f"{want[:12]}); run __graft_entry__.build()")
    _lib = lib
    return lib


def check(rc: int, ctx=None) -> None:
    if rc == QOC_OK:
        return
    msg = load().qoc_last_error(ctx).decode(errors="replace")
    if rc == QOC_ERR_STALE:
        raise StaleCacheError(rc, msg)
    raise QOCError(rc, msg)
