"""Block propagators on the tunable bus (VERDICT round 4 ask #4): the live 14-row even-parity block as its
own system (rows 0, 2, .., 26: x0 = |110> and the target |200> live there, the generators keep the block invariant),
evaluated with every U_k formed (set_chain('propagators'): Padé-13 / Taylor on MFMA per (seed, slice), then one
matvec chain per direction) and with the Chebyshev-action chain, against the full N = 27 engine (dead block skipped).
Same u, B = 512, Nt = 2000; prints one JSON line per variant (ms per eval, phase times, max |ΔJ| to the full engine).
Usage: python tools/tb_blockprop.py [steps]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "quantumoptimalcontrol.jl_amd"))
from qoc_amd import GrapeEngine, systems  # noqa: E402


def run(prob, u, chain, steps):
    B, nu, Nt = u.shape
    e = GrapeEngine(prob.A0, prob.A, prob.x0, Nt, B=B)
    e.set_cost_trace(prob.x_target, prob.n)
    e.set_chain(chain)
    ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
    Jd = torch.empty(B, dtype=torch.float64, device="cuda")
    gd = torch.empty(B, Nt, nu, dtype=torch.float64, device="cuda")
    for _ in range(2):
        e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
    e.synchronize()
    e.phase_times(reset=True)
    e.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
    e.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    ph = e.phase_times(reset=True)
    info = e.info()
    e.close()
    return ms, ph, info, Jd.cpu().numpy(), gd.cpu().numpy()


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    full = systems.tunable_bus_problem(2000)
    u = systems.tunable_bus_controls(512, 2000, seed=0)
    rows = np.arange(0, 27, 2)
    blk = systems.Problem("tunable_bus_even_block", full.A0[np.ix_(rows, rows)], [a[np.ix_(rows, rows)] for a in full.A],
                          full.x0[rows], full.x_target[rows], full.n, full.Nt, "fp64")
    for j, a in enumerate([full.A0] + list(full.A)):  # the block is invariant: nothing couples it to the odd rows
        assert np.abs(a[np.ix_(rows, np.arange(1, 27, 2))]).max() == 0.0, j
    ms_f, ph_f, info_f, J_f, g_f = run(full, u, "auto", steps)
    print(json.dumps({"variant": "full N=27, auto (dead block skipped)", "ms_per_eval": ms_f, "evals_per_s": 512e3 / ms_f,
                      "phases_ms": ph_f, "chain_kernel": info_f.get("chain_kernel")}))
    for chain in ("propagators", "taylor"):
        ms, ph, info, J, g = run(blk, u, chain, steps)
        print(json.dumps({"variant": f"even block N=14, chain={chain}", "ms_per_eval": ms, "evals_per_s": 512e3 / ms,
                          "phases_ms": ph, "chain_kernel": info.get("chain_kernel"),
                          "max_dJ_vs_full": float(np.abs(J - J_f).max()),
                          "max_rel_dJdu_vs_full": float(np.abs(g - g_f).max() / np.abs(g_f).max())}))


if __name__ == "__main__":
    main()
