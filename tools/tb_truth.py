"""Where does the tunable bus' |ΔJ| between the GPU and the C port come from?  Both are fp64 approximations with a
per-slice backward error of ~u ||A_k|| (||A_k||_2 ~ 14.5 here), over 2000 chained slices.  This compares each against
an extended-precision propagation (numpy clongdouble: 64-bit mantissas; Taylor degree 30 after scaling to ||X|| <= 1/2,
then the squarings), whose own error is ~1e-17.

  python tools/tb_truth.py dump [tag]    (GPU box) J / dJdu of the first SEEDS seeds of ranks 0..7 for the GPU paths
                                         into gpurun_out/<tag>_tb_dump.npz
  python tools/tb_truth.py truth [tag]   (anywhere) the extended-precision J of those seeds, the C port's, and the
                                         errors of every path against it
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")
sys.path.insert(0, os.path.join(ROOT, "quantumoptimalcontrol.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from qoc_amd import systems  # noqa: E402

SEEDS = int(os.environ.get("TB_SEEDS", "8"))
RANKS = range(8)
VARIANTS = [("blkp", {}), ("taylor", {"QOC_BLKP_INTERP": "0"}),
            ("cheb6", {"QOC_BLKP_INTERP": "0", "QOC_BLKP_CHEB": "6"}), ("chebyshev_chain", {"QOC_BLKP": "0"})]
ENV_KEYS = ("QOC_BLKP", "QOC_BLKP_TAIL", "QOC_BLKP_RCAP", "QOC_BLKP_CHEB", "QOC_BLKP_CRMAX", "QOC_BLKP_INTERP")


def dump(tag):
    import torch
    from qoc_amd import GrapeEngine
    mk_prob, mk_u, B = systems.CONFIGS["tunable_bus"]
    prob = mk_prob()
    out = {}
    for name, env in VARIANTS:
        for k in ENV_KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        e = GrapeEngine(prob.A0, prob.A, prob.x0, prob.Nt, B=B)
        e.set_cost_trace(prob.x_target, prob.n)
        for r in RANKS:
            u = mk_u(B, r)
            ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
            Jd = torch.empty(B, dtype=torch.float64, device="cuda")
            gd = torch.empty(B, prob.Nt, prob.nu, dtype=torch.float64, device="cuda")
            e.chain_terms(reset=True)
            e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
            e.synchronize()
            out[f"{name}_prods_{r}"] = np.array(e.chain_terms() / (B * prob.Nt))
            out[f"{name}_J_{r}"] = Jd.cpu().numpy()
            out[f"{name}_g_{r}"] = np.transpose(gd.cpu().numpy(), (0, 2, 1))[:SEEDS]
        out[f"{name}_info"] = np.array(str(e.info()))
        e.close()
        print(name, "done", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"{tag}_tb_dump.npz"), **out)


def expm_ld(X):
    """exp(X) in clongdouble: scaling to ||X||_1 <= 1/2, Taylor degree 30 (tail < 1e-40), squarings."""
    n1 = float(np.abs(X).sum(axis=0).max())
    s = max(0, int(np.ceil(np.log2(max(n1, 1e-300) / 0.5))))
    Y = X / np.longdouble(2.0) ** s
    E = np.eye(X.shape[0], dtype=np.clongdouble)
    T = np.eye(X.shape[0], dtype=np.clongdouble)
    for k in range(1, 31):
        T = T @ Y / np.longdouble(k)
        E = E + T
    for _ in range(s):
        E = E @ E
    return E


def J_ld(prob, u):
    A0 = prob.A0.astype(np.clongdouble)
    A1 = prob.A[0].astype(np.clongdouble)
    x = prob.x0.astype(np.clongdouble)
    for k in range(prob.Nt):
        x = expm_ld(A0 + np.longdouble(u[0, k]) * A1) @ x
    ov = np.sum(np.conj(prob.x_target.astype(np.clongdouble)) * x)
    return np.longdouble(1.0) - np.abs(ov) ** 2 / np.longdouble(prob.n) ** 2


def truth(tag):
    import cpuref
    from concurrent.futures import ProcessPoolExecutor
    mk_prob, mk_u, B = systems.CONFIGS["tunable_bus"]
    prob = mk_prob()
    d = np.load(os.path.join(ROOT, "gpurun_out", f"{tag}_tb_dump.npz"))
    cpuref.use_blas(True)
    jobs = [(r, b) for r in RANKS for b in range(SEEDS)]
    us = {r: mk_u(B, r)[:SEEDS] for r in RANKS}
    cache = os.path.join(ROOT, "gpurun_out", "tb_truth_cache.npz")  # the extended-precision and C-port J (slow)
    if os.path.exists(cache) and int(np.load(cache)["seeds"]) == SEEDS:
        cz = np.load(cache)
        Jt = {rb: cz["Jt"][i] for i, rb in enumerate(jobs)}
        Jc_full = {r: cz["Jc"][r] for r in RANKS}
    else:
        with ProcessPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
            Jt = list(ex.map(_J_job, [(r, b) for r, b in jobs]))
        Jt = {rb: v for rb, v in zip(jobs, Jt)}
        Jc_full = {r: cpuref.grape_eval_batch(prob, mk_u(B, r), order=3, mode=0)[0] for r in RANKS}
        np.savez(cache, seeds=SEEDS, Jt=np.array([Jt[rb] for rb in jobs], dtype=np.longdouble),
                 Jc=np.stack([Jc_full[r] for r in RANKS]))
    Jc = {r: Jc_full[r][:SEEDS] for r in RANKS}
    rows = []
    for r, b in jobs:
        t = Jt[(r, b)]
        row = {"rank": r, "seed": b, "cport": float(np.float64(Jc[r][b] - t))}
        for name, _ in VARIANTS:
            key = f"{name}_J_{r}"
            if key in d:
                row[name] = float(np.float64(d[key][b] - t))
        rows.append(row)
    names = ["cport"] + [n for n, _ in VARIANTS if f"{n}_J_0" in d]
    print("error against the extended-precision J over", len(rows), "seeds (max |err|, rms):")
    for n in names:
        v = np.array([row[n] for row in rows])
        print(f"  {n:16s} max {np.abs(v).max():.3e}  rms {np.sqrt(np.mean(v * v)):.3e}  mean {v.mean():+.3e}")
    for n in names[1:]:
        v = np.array([row[n] - row["cport"] for row in rows])
        full = max(float(np.abs(d[f"{n}_J_{r}"] - Jc_full[r]).max()) for r in RANKS)
        print(f"  {n:16s} - cport: max {np.abs(v).max():.3e} (these seeds), {full:.3e} (all {B} seeds of every rank);"
              f" products per unit {float(d[f'{n}_prods_0']):.3f}")


def _J_job(rb):
    r, b = rb
    mk_prob, mk_u, B = systems.CONFIGS["tunable_bus"]
    return J_ld(mk_prob(), mk_u(B, r)[b])


if __name__ == "__main__":
    mode = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else "r06"
    dump(tag) if mode == "dump" else truth(tag)
