"""Regenerate the committed fixtures in tests/golden/ (run in the build container, where
/root/reference exists).  Fixtures are data only:

* cavity_qubit_pulse_marina.npy, zz_coupling_pulse_tahereh210823.npy — the reference's own
  measured I/Q pulses (examples/*.csv), converted to float64 .npy (no scaling applied);
* golden_evals.npz — small GRAPE evals (u, J, dJdu at orders 1-4) computed by the CPU oracle
  (oracle/qoc_oracle.py, pinned against the reference's known answers in tests/test_oracle.py).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "quantumoptimalcontrol.jl_amd")]
import qoc_oracle as O  # noqa: E402
from qoc_amd import systems as S  # noqa: E402

REF = "/root/reference/examples"


def main():
    for name in ("cavity_qubit_pulse_marina", "zz_coupling_pulse_tahereh210823"):
        src = os.path.join(REF, name + ".csv")
        if os.path.exists(src):
            np.save(os.path.join(HERE, name + ".npy"), np.loadtxt(src))
    out = {}
    cases = {
        "zz": (S.zz_problem(60, tgate=6.0), S.zz_controls(2, 60, 6.0, seed=11)),
        "cavity": (S.cavity_problem(N_cavity=8, Nt=40), S.cavity_controls(2, 40, seed=12)),
        "bus": (S.tunable_bus_problem(Nt=40, tgate=7.0), S.tunable_bus_controls(2, 40, seed=13)),
    }
    for key, (prob, u) in cases.items():
        out[f"{key}_u"] = u
        for order in (1, 2, 3, 4):
            Js, gs = [], []
            for b in range(u.shape[0]):
                J, g, _ = O.grape_eval(prob.A0, prob.A, u[b], prob.x0, prob.x_target, prob.n, order=order)
                Js.append(J)
                gs.append(g)
            out[f"{key}_J_o{order}"] = np.array(Js)
            out[f"{key}_dJdu_o{order}"] = np.stack(gs)
    np.savez_compressed(os.path.join(HERE, "golden_evals.npz"), **out)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
