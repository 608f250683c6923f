"""Full-length fixtures (run in the build container; writes tests/golden/*.npz, data only):

* zz_pulse_fixture.npz — the reference's zz forward simulation (examples/zz_coupling_simulation.jl:3-13): the
  measured pulse zz_coupling_pulse_tahereh210823 x 1e-9 (2 x 500), Δt = 20/500, generators
  setup_bilinear_matrices(H0, Tc, Δt) of examples/models/zz_coupling.jl, x0 = Q_css; x_501 by the fp64 oracle
  (oracle/qoc_oracle.py: the reference's propagate with ExpMethodHigham2005), and J / dJdu of the NOT-gate trace
  cost (n = 4, examples/zz_coupling_ipopt_exp.jl:16) at order 3.
* synthetic_full.npz — config 5 (synthetic GUE N = 256, m = 256, nu = 2, Nt = 1000; systems.CONFIGS["synthetic"])
  for seeds 0 and 127 of the rank-0 batch: J and dJdu (order 3) over ALL 1000 slices by the fp64 oracle, and x_N of
  seed 0 (stored as complex64: the fp32 GPU result is compared at ~1e-4).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "quantumoptimalcontrol.jl_amd")]
import qoc_oracle as O  # noqa: E402
from qoc_amd import systems as S  # noqa: E402


def zz_pulse():
    prob = S.zz_problem(500)  # tgate 20, Δt = 0.04
    iq = np.load(os.path.join(HERE, "zz_coupling_pulse_tahereh210823.npy")) * 1e-9
    u = np.ascontiguousarray(iq.T)  # 2 x 500
    xs = O.propagate(prob.A0, prob.A, u, prob.x0)
    J, g, _ = O.grape_eval(prob.A0, prob.A, u, prob.x0, prob.x_target, prob.n, order=3)
    np.savez_compressed(os.path.join(HERE, "zz_pulse_fixture.npz"), u=u, x_final=xs[-1], J=J, dJdu=g)
    print("zz pulse: J", J, "|x_501|", np.linalg.norm(xs[-1]))


def synthetic(seeds=(0, 127)):
    mk_prob, mk_u, B = S.CONFIGS["synthetic"]
    prob = mk_prob()
    u = mk_u(B, 0)
    Js, gs, xN = [], [], None
    for s in seeds:
        t = time.time()
        J, g, cache = O.grape_eval(prob.A0, prob.A, u[s], prob.x0, prob.x_target, prob.n, order=3)
        Js.append(J)
        gs.append(g)
        if xN is None:
            xN = np.asarray(cache.x[-1]).astype(np.complex64)
        print(f"synthetic seed {s}: J {J:.12f} ({time.time() - t:.0f} s)", flush=True)
    np.savez_compressed(os.path.join(HERE, "synthetic_full.npz"), seeds=np.array(seeds), J=np.array(Js),
                        dJdu=np.stack(gs), x_final_seed0=xN)


if __name__ == "__main__":
    what = sys.argv[1:] or ["zz", "synthetic"]
    if "zz" in what:
        zz_pulse()
    if "synthetic" in what:
        synthetic()
