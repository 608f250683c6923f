"""Accuracy / cost of the stored block propagators' exponential settings on the full tunable bus (B = 512, Nt = 2000)
against the C port (oracle/cpu_ref.c, the reference's Padé-13): max |ΔJ|, max ||ΔdJdu|| / ||dJdu|| over every seed, and
the formation / chain time per eval, for QOC_BLKP_4M / QOC_BLKP_SLACK variants and the Chebyshev-action chains
(QOC_BLKP=0).  Usage: python tools/blkp_accuracy.py"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "quantumoptimalcontrol.jl_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
from qoc_amd import GrapeEngine, systems  # noqa: E402


def main():
    import cpuref
    mk_prob, mk_u, B = systems.CONFIGS["tunable_bus"]
    prob = mk_prob()
    u = mk_u(B, 0)
    cpuref.use_blas(True)
    t0 = time.time()
    Jc, gc = cpuref.grape_eval_batch(prob, u, order=3, mode=0)
    print(json.dumps({"cpu_port_s": time.time() - t0}), flush=True)
    ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
    variants = [("default", {}), ("slack1", {"QOC_BLKP_SLACK": "1"}), ("slack2", {"QOC_BLKP_SLACK": "2"}),
                ("4m", {"QOC_BLKP_4M": "1"}), ("4m_slack1", {"QOC_BLKP_4M": "1", "QOC_BLKP_SLACK": "1"}),
                ("chebyshev_chain", {"QOC_BLKP": "0"})]
    keys = ("QOC_BLKP_4M", "QOC_BLKP_SLACK", "QOC_BLKP")
    for name, env in variants:
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(env)
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
        e.set_cost_trace(prob.x_target, prob.n)
        Jd = torch.empty(B, dtype=torch.float64, device="cuda")
        gd = torch.empty(B, prob.Nt, prob.nu, dtype=torch.float64, device="cuda")
        e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
        e.synchronize()
        e.phase_times(reset=True)
        e.chain_terms(reset=True)
        e.set_profiling(True)
        t0 = time.perf_counter()
        for _ in range(3):
            e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
        e.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / 3
        ph = e.phase_times(reset=True)
        prods = e.chain_terms() / 3
        info = e.info()
        e.close()
        J = Jd.cpu().numpy()
        g = np.transpose(gd.cpu().numpy(), (0, 2, 1))
        rel = max(np.linalg.norm(g[b] - gc[b]) / np.linalg.norm(gc[b]) for b in range(B))
        print(json.dumps({"variant": name, "ms_per_eval": ms, "phases_ms": {k: v[0] / 3 for k, v in ph.items()},
                          "products_per_unit": prods / (B * prob.Nt) if info.get("chain_kernel") == "blocks_prop16" else None,
                          "max_dJ": float(np.abs(J - Jc).max()), "max_rel_dJdu": float(rel),
                          "chain_kernel": info.get("chain_kernel")}), flush=True)


if __name__ == "__main__":
    main()
