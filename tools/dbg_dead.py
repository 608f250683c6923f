import os, sys, numpy as np
import torch
torch.cuda.init()
sys.path.insert(0, 'quantumoptimalcontrol.jl_amd'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
from qoc_amd import GrapeEngine, systems
from test_gpu_blk import _eval
Nt = 32
prob = systems.tunable_bus_problem(Nt=Nt, tgate=350.0 * Nt / 2000)
u = systems.tunable_bus_controls(2, Nt, seed=83)
qb = systems.QuantumBasis([3, 3, 3])
x_odd, t_odd = qb.columns(["100"]).astype(complex), qb.columns(["001"]).astype(complex)
os.environ["QOC_BLOCKS"] = "1"; os.environ["QOC_BLKP"] = "1"
res = {}
for interp in ("1", "0"):
    os.environ["QOC_BLKP_INTERP"] = interp
    for dead in ("1", "0"):
        for first in (True, False):
            os.environ["QOC_BLK_DEAD"] = dead
            e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=2)
            e.set_cost_trace(prob.x_target, prob.n); e.set_chain("taylor")
            if first:
                e.set_x0(x_odd); e.set_cost_trace(t_odd, prob.n); _eval(e, u, True)
                e.set_x0(prob.x0); e.set_cost_trace(prob.x_target, prob.n)
            J, g = _eval(e, u, True)
            res[(interp, dead, first)] = (J, g, e.info()["interp_degree"])
            e.close()
for k, (J, g, d) in res.items():
    r = res[(k[0], "1", True)]
    print(k, "deg", d, "dJ vs dead1/first", np.abs(J - r[0]).max(), "dg", np.abs(g - r[1]).max(), J)
