"""Multi-GPU epilogue: seeds are sharded contiguously over ranks (one process per GPU); the
only exchange on the path is an all-gather of each rank's best (J, global seed id)
(SURVEY.md §8e).

Two transports with the same result:
  * ``init_engine_comm`` + ``GrapeEngine.allgather_best[_device]``: RCCL inside libqoc_mi355x.so
    (include/qoc.h qoc_comm_init / qoc_allgather_best) — what a Julia caller binds; torch.distributed only
    carries the 128-byte unique id;
  * ``gather_best``: torch.distributed (RCCL on ROCm's "nccl" backend, or "gloo" for CPU tests).
"""
from __future__ import annotations


def shard(B_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of seeds [start, stop) owned by `rank`."""
    base, rem = divmod(B_total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_best(J_local, seed_offset: int, out=None):
    """All-gather (min J, its global seed) over the default process group.

    J_local: 1-D torch tensor of this rank's objectives (any device the backend supports).
    Returns (J_best, seed_best) as Python numbers; `out` (2*world doubles) may be preallocated.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size() if dist.is_initialized() else 1
    jm, idx = torch.min(J_local, 0)
    mine = torch.stack([jm.to(torch.float64), (idx + seed_offset).to(torch.float64)])
    if world == 1:
        return float(mine[0]), int(mine[1])
    if out is None:
        out = torch.empty(2 * world, dtype=torch.float64, device=J_local.device)
    dist.all_gather_into_tensor(out, mine)
    allv = out.view(world, 2)
    r = int(torch.argmin(allv[:, 0]))
    return float(allv[r, 0]), int(allv[r, 1])


def init_engine_comm(engine, seed_offset: int) -> str:
    """Join the engine's RCCL communicator over the default process group: rank 0 makes the unique id and
    torch.distributed broadcasts it (a one-rank communicator at world 1, through the same ncclAllGather path).
    Returns the transport of the epilogue: "rccl-libqoc" when every rank joined a communicator of `world`
    ranks, else "torch.distributed" (world > 1, RCCL missing on some rank) or "local" (world 1 without RCCL).

    ncclCommInitRank is collective: a rank that fails inside it leaves the others blocked there.  So the ranks
    first agree that every one of them can load RCCL (each makes a unique id of its own, which needs only the
    library), and only then join; a failure of the join itself is an error on every rank, not a fallback."""
    import torch.distributed as dist

    from . import _lib
    from .engine import comm_unique_id

    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    try:
        own_id = comm_unique_id()
    except _lib.QOCError:
        own_id = b""
    ok = bool(own_id)
    if world > 1:  # every rank must take the same transport
        import torch
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        if dist.get_backend() == "nccl":
            flag = flag.cuda()
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item())
    if not ok:
        engine.comm_init(1, 0, None, seed_offset)  # no communicator: the epilogue covers this engine alone
        return "torch.distributed" if world > 1 else "local"
    box = [own_id if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(box, src=0)
    err = None
    try:
        engine.comm_init(world, rank, box[0], seed_offset)  # collective
        if engine.comm_ranks() != world:
            err = f"RCCL communicator has {engine.comm_ranks()} ranks, expected {world}"
    except _lib.QOCError as ex:
        err = str(ex)
    if world > 1:
        # a join that failed on one rank (after the collective part, or with the others already through it) becomes
        # an error on every rank instead of a rank that later waits alone in an all-gather
        import torch
        flag = torch.tensor([0 if err else 1], dtype=torch.int32)
        if dist.get_backend() == "nccl":
            flag = flag.cuda()
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not bool(flag.item()) and err is None:
            err = "RCCL communicator: the join failed on another rank"
    if err:
        raise _lib.QOCError(_lib.QOC_ERR_STATE, err)
    return "rccl-libqoc"
