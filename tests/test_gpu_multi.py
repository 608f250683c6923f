"""Multi-GPU epilogue on the one-GPU box.

* qoc_allgather_best through the C ABI: without a communicator, and with a real one-rank RCCL communicator
  (qoc_comm_unique_id -> ncclCommInitRank(nranks = 1) -> ncclAllGather) created next to torch's own "nccl"
  process group in the same process; the best (J, global seed) of the last propagate equals the argmin.
* Two ranks sharing the one device, each propagating its contiguous shard of the seeds through its own engine:
  the gathered best equals the single-process argmin over the full batch.  RCCL rejects two ranks on one GPU
  ("Duplicate GPU detected"), so these two ranks exchange over gloo (qoc_amd.multi.gather_best); the RCCL
  all-gather itself runs in the driver's multi-GPU bench (bench.py, transport "rccl-libqoc").
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B_TOTAL, NT = 12, 40


def _problem():
    from qoc_amd import systems
    prob = systems.cavity_problem(N_cavity=8, Nt=NT)
    u = systems.cavity_controls(B_TOTAL, NT, seed=17) * 4.0  # spread the fidelities
    return prob, u


def test_allgather_best_world1_c_abi(built_lib):
    from qoc_amd import GrapeEngine
    prob, u = _problem()
    e = GrapeEngine(prob.A0, prob.A, prob.x0, NT, B=B_TOTAL)
    e.set_cost_trace(prob.x_target, prob.n)
    J = e.propagate(u)
    assert e.allgather_best() == (J.min(), int(np.argmin(J)))  # no communicator: this context alone
    e.comm_init(1, 0, None, 1000)
    Jb, sb = e.allgather_best()
    assert Jb == J.min() and sb == 1000 + int(np.argmin(J))
    e.close()


def _rccl_world1(port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "quantumoptimalcontrol.jl_amd"))
    import torch
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        t = torch.ones(4, device="cuda")
        dist.all_reduce(t)  # torch's RCCL communicator is up
        from qoc_amd import GrapeEngine, multi
        prob, u = _problem()
        e = GrapeEngine(prob.A0, prob.A, prob.x0, NT, B=B_TOTAL)
        e.set_cost_trace(prob.x_target, prob.n)
        J = e.propagate(u)
        transport = multi.init_engine_comm(e, 1000)  # libqoc's own one-rank RCCL communicator
        ranks = e.comm_ranks()
        Jb, sb = e.allgather_best()  # ncclAllGather inside libqoc_mi355x.so
        d = torch.empty(2, dtype=torch.float64, device="cuda")
        e.allgather_best_device(d.data_ptr())
        e.synchronize()
        dev = d.cpu().tolist()
        dist.all_reduce(t)  # torch's communicator still works next to libqoc's
        torch.cuda.synchronize()
        ok_t = float(t[0].item()) == 1.0
        e.close()
        dist.destroy_process_group()
        q.put(("ok", transport, ranks, (Jb, sb), dev, J.min(), int(np.argmin(J)), ok_t))
    except Exception as ex:  # reported to the parent
        q.put(("error", repr(ex)))


def test_rccl_world1_communicator_next_to_torch_nccl(built_lib):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_world1, args=(_port(), q))
    p.start()
    res = q.get(timeout=100)
    p.join(timeout=60)
    assert res[0] == "ok", res
    _, transport, ranks, (Jb, sb), dev, Jmin, amin, ok_t = res
    assert transport == "rccl-libqoc" and ranks == 1
    assert Jb == Jmin and sb == 1000 + amin
    assert dev == [Jmin, float(1000 + amin)]
    assert ok_t
    assert p.exitcode == 0


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "quantumoptimalcontrol.jl_amd"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qoc_amd import GrapeEngine, multi
    prob, u = _problem()
    start, stop = multi.shard(B_TOTAL, rank, world)
    e = GrapeEngine(prob.A0, prob.A, prob.x0, NT, B=stop - start)
    e.set_cost_trace(prob.x_target, prob.n)
    J = e.propagate(u[start:stop])
    res = multi.gather_best(torch.from_numpy(J), start)
    e.close()
    q.put((rank, res))
    dist.destroy_process_group()


def test_two_ranks_share_the_gpu_and_gather_the_global_best(built_lib):
    import torch.multiprocessing as mp
    from qoc_amd import GrapeEngine
    prob, u = _problem()
    e = GrapeEngine(prob.A0, prob.A, prob.x0, NT, B=B_TOTAL)
    e.set_cost_trace(prob.x_target, prob.n)
    J = e.propagate(u)
    e.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, (Jb, sb) in out:
        assert sb == int(np.argmin(J))
        assert abs(Jb - J.min()) <= 1e-13


def test_best_output_registered_world1(built_lib):
    """qoc_set_best_output: with one rank the segmented eval writes the best (J, seed) into the registered buffer itself
    and allgather_best_device(that buffer) queues nothing; the pair equals the argmin (and what the pick kernel writes
    into another buffer); after unregistering the pick kernel runs again."""
    import torch
    from qoc_amd import GrapeEngine
    prob, u = _problem()
    e = GrapeEngine(prob.A0, prob.A, prob.x0, NT, B=B_TOTAL)
    e.set_cost_trace(prob.x_target, prob.n)
    e.comm_init(1, 0, None, 500)
    ud = torch.from_numpy(np.ascontiguousarray(np.transpose(u, (0, 2, 1)))).cuda()
    Jd = torch.empty(B_TOTAL, dtype=torch.float64, device="cuda")
    gd = torch.empty(B_TOTAL, NT, prob.nu, dtype=torch.float64, device="cuda")
    reg = torch.full((2,), -7.0, dtype=torch.float64, device="cuda")
    other = torch.full((2,), -7.0, dtype=torch.float64, device="cuda")
    e.set_best_output(reg.data_ptr())
    for u_scale in (1.0, 0.5):
        ud2 = ud * u_scale
        e.eval_device(ud2.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
        assert e.info()["backward"] == "segmented", e.info()
        e.allgather_best_device(reg.data_ptr())
        e.synchronize()
        J = Jd.cpu().numpy()
        assert reg.cpu().tolist() == [J.min(), float(500 + int(np.argmin(J)))]
        assert e.allgather_best() == (J.min(), 500 + int(np.argmin(J)))
        e.allgather_best_device(other.data_ptr())  # another buffer: the pick kernel
        e.synchronize()
        assert other.cpu().tolist() == reg.cpu().tolist()
    e.set_best_output(0)
    reg.fill_(-7.0)
    e.eval_device(ud.data_ptr(), 3, Jd.data_ptr(), gd.data_ptr())
    e.allgather_best_device(reg.data_ptr())
    e.synchronize()
    J = Jd.cpu().numpy()
    assert reg.cpu().tolist() == [J.min(), float(500 + int(np.argmin(J)))]
    e.close()
