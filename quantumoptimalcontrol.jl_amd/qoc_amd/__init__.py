"""qoc_amd — MI355X-native GRAPE propagation/gradient engine (host side).

The hot path (per-slice exponentials, forward/backward propagator chains, the
Taylor expm-Jacobian contraction and the trace-fidelity costs of
olof3/QuantumOptimalControl.jl) runs in hand-written HIP kernels for gfx950 in
``libqoc_mi355x.so`` (C ABI: include/qoc.h).  This package is the host mirror of the
reference's interface for that path; it has no CPU fallback.
"""
from . import systems  # noqa: F401
from ._lib import QOCError, StaleCacheError  # noqa: F401
from .api import (  # noqa: F401
    MI355XCache,
    c2r,
    generators_from_rhs,
    r2c,
    compute_pwc_gradient,
    grape_sensitivity,
    propagate,
    propagate_pwc,
    setup_bilinear_matrices,
    setup_grape_cache,
    setup_infidelity,
    setup_infidelity_zcalibrated,
    setup_state_penalty,
)
from .engine import GrapeEngine, comm_unique_id, expm, expm_jacobian  # noqa: F401
from .optimize import SplineGrape, minimize_batched  # noqa: F401

__all__ = [
    "GrapeEngine", "MI355XCache", "comm_unique_id", "QOCError", "StaleCacheError", "expm", "expm_jacobian",
    "grape_sensitivity", "propagate", "setup_bilinear_matrices", "setup_grape_cache",
    "setup_infidelity", "setup_infidelity_zcalibrated", "setup_state_penalty", "systems",
    "SplineGrape", "minimize_batched", "propagate_pwc", "compute_pwc_gradient",
]
