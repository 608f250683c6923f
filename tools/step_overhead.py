"""Where the per-step time beyond the eval kernel goes (diagnostic): the segmented eval alone, with the phase
events (qoc_set_profiling), with the best-pair epilogue, and with both, K steps each on the cavity config."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quantumoptimalcontrol.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from qoc_amd import GrapeEngine, systems  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cavity"
comm = len(sys.argv) > 2 and sys.argv[2] == "comm"  # a one-rank RCCL communicator (bench.py at N = 1)
K = 50
mk_prob, mk_u, B = systems.CONFIGS[cfg]
prob = mk_prob()
u = mk_u(B, 0)
torch.cuda.set_device(0)
eng = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
eng.set_cost_trace(prob.x_target, prob.n)
ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
Jd = torch.empty(B, dtype=torch.float64, device="cuda")
gd = torch.empty(B, prob.Nt, prob.nu, dtype=torch.float64, device="cuda")
bd = torch.empty(2, dtype=torch.float64, device="cuda")
if comm:
    from qoc_amd import multi
    print("transport", multi.init_engine_comm(eng, 0), flush=True)
for prof in (False, True):
    for epi in (False, True):
        eng.set_profiling(prof)
        for _ in range(5):
            eng.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
        eng.synchronize()
        t = time.perf_counter()
        for _ in range(K):
            eng.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
            if epi:
                eng.allgather_best_device(bd.data_ptr())
        eng.synchronize()
        dt = (time.perf_counter() - t) / K * 1e3
        print(f"{cfg} comm={comm} profiling={prof} epilogue={epi}: {dt:.4f} ms per step, {B / dt * 1e3:.0f} evals/s", flush=True)
eng.close()
