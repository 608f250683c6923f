"""World-size-2 gloo test of the seed sharding + best-fidelity all-gather (CPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from qoc_amd.multi import gather_best, shard


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 10
    start, stop = shard(B * world, rank, world)
    torch.manual_seed(rank)
    J = torch.rand(stop - start, dtype=torch.float64) + 0.5
    if rank == 1:
        J[3] = 0.01  # global best lives on rank 1
    res = gather_best(J, start)
    q.put((rank, res))
    dist.destroy_process_group()


def test_shard_partitions():
    for total, world in ((10, 3), (4096, 8), (7, 8)):
        spans = [shard(total, r, world) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == total
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_gather_best_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, (J, seed) in out:
        assert J == pytest.approx(0.01) and seed == 10 + 3


def test_bench_launcher_starts_two_ranks_cpu():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts its own two ranks (torch.distributed.run) and rank 0
    reports n_gpus 2; --cpu-plumbing runs the ranks' best-(J, seed) exchange over gloo without a GPU."""
    import json
    import subprocess
    import sys

    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu-plumbing",
                          "--steps", "3", "--warmup", "1", "--seeds", "8"], capture_output=True, text=True,
                         timeout=240, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["config"]["global_seeds"] == 16
    J = np.concatenate([np.random.default_rng(r).uniform(0.1, 1.0, 8) for r in range(2)])
    assert rec["best_over_ranks"]["seed"] == int(np.argmin(J))
    assert rec["best_over_ranks"]["J"] == J.min()


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu-plumbing"],
                         capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr
