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
