"""Fixed cost of a timed region (diagnostic): bench.py's step (eval + best-pair epilogue, phase events on) timed over
K = 5, 10, 20, 50, 200 steps between synchronisations; per-step time = slope, fixed cost = intercept."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quantumoptimalcontrol.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from qoc_amd import GrapeEngine, multi, systems  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cavity"
mk_prob, mk_u, B = systems.CONFIGS[cfg]
prob = mk_prob()
u = mk_u(B, 0)
torch.cuda.set_device(0)
eng = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
eng.set_cost_trace(prob.x_target, prob.n)
multi.init_engine_comm(eng, 0)
ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
Jd = torch.empty(B, dtype=torch.float64, device="cuda")
gd = torch.empty(B, prob.Nt, prob.nu, dtype=torch.float64, device="cuda")
bd = torch.empty(2, dtype=torch.float64, device="cuda")
eng.set_profiling(True)


def step():
    eng.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
    eng.allgather_best_device(bd.data_ptr())


for _ in range(3):
    step()
res = []
for K in (5, 10, 20, 50, 200, 20, 10):
    eng.synchronize()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(K):
        step()
    eng.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    res.append((K, dt))
    print(f"{cfg} K={K}: {dt * 1e3:.3f} ms, {dt / K * 1e3:.4f} ms per step", flush=True)
k = np.array([r[0] for r in res], float)
d = np.array([r[1] for r in res]) * 1e3
A = np.vstack([k, np.ones_like(k)]).T
slope, icpt = np.linalg.lstsq(A, d, rcond=None)[0]
print(f"{cfg}: {slope:.4f} ms per step + {icpt:.3f} ms per timed region", flush=True)
eng.close()
