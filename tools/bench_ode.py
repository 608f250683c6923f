"""ODE path throughput: batched f + grad with fixed-step Tsit5 vs the expm path,
on the bench configurations.  One JSON line per config.

    python tools/bench_ode.py [--configs zz_batch,cavity,tunable_bus] [--steps 5]

Work model of the ODE kernel (k_ode_pwc, one workgroup per seed): per slice nsub Tsit5 steps of 6 new
stage evaluations (FSAL), each a complex N x N by N x m product = 8 N^2 m flops (fp64 VALU, peak 78.6 TF/s);
the adjoint sweep does the same work with A_k^H.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quantumoptimalcontrol.jl_amd"))

PEAK_FP64 = 78.6  # TF/s, MI355X fp64 vector / matrix (spec)
NSUB = {"zz_batch": 10, "cavity": 10, "tunable_bus": 40}


def run(name, steps, warmup, seeds):
    import numpy as np
    import torch
    from qoc_amd import GrapeEngine, systems
    mk_prob, mk_u, B = systems.CONFIGS[name]
    B = seeds or B
    prob = mk_prob()
    u = mk_u(B, 0)
    dev = torch.device("cuda", 0)
    u_d = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).to(dev)
    J_d = torch.empty(B, dtype=torch.float64, device=dev)
    g_d = torch.empty(B, prob.Nt, prob.nu, dtype=torch.float64, device=dev)
    out = {"config": name, "N": prob.N, "m": prob.m, "Nt": prob.Nt, "B": B, "nsub": NSUB[name]}
    for method in ("tsit5", "expm"):
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B, precision=prob.precision)
        e.set_cost_trace(prob.x_target, prob.n)
        e.set_propagation(method, NSUB[name])
        for _ in range(warmup):
            e.eval_device(u_d.data_ptr(), 3, J_d.data_ptr(), g_d.data_ptr())
        e.synchronize()
        e.phase_times(reset=True)
        e.set_profiling(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            e.eval_device(u_d.data_ptr(), 3, J_d.data_ptr(), g_d.data_ptr())
        e.synchronize()
        dt = time.perf_counter() - t0
        e.set_profiling(False)
        ph = e.phase_times()
        r = {"evals_per_s": B * steps / dt, "ms_per_step": dt / steps * 1e3,
             "phase_ms_per_step": {k: v[0] / steps for k, v in ph.items()}}
        if method == "tsit5":
            fl = 8.0 * prob.N ** 2 * prob.m * 6 * NSUB[name] * prob.Nt * B
            t_f = ph["k_chain_fwd"][0] / steps / 1e3
            t_b = ph["k_chain_bwd"][0] / steps / 1e3
            r["k_ode_pwc_fwd"] = {"tflops": fl / t_f / 1e12, "frac_fp64_peak": fl / t_f / 1e12 / PEAK_FP64}
            r["k_ode_pwc_adj"] = {"tflops": fl / t_b / 1e12, "frac_fp64_peak": fl / t_b / 1e12 / PEAK_FP64}
        out[method] = r
        e.close()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="zz_batch,cavity,tunable_bus")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seeds", type=int, default=0)
    a = ap.parse_args()
    for name in a.configs.split(","):
        run(name, a.steps, a.warmup, a.seeds)


if __name__ == "__main__":
    main()
