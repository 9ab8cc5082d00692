"""Multi-GPU sharding of an rx batch.

Frames are independent, so a batch is split into contiguous index ranges,
one per rank (one process per GPU), with no data-path collective.  The one
exchange step the north star asks for is an all-gather of the per-frame
flow hashes (u64) so every rank sees the whole batch's hashes; over RCCL
(backend "nccl") it runs on xGMI and bench.py overlaps it with the next
batch's kernel.  The same code runs on gloo for the CPU tests.
"""


def shard_range(n_total, world, rank):
    """Contiguous [first, first + count) of frames owned by `rank`."""
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def allgather_flow_hash(local, out=None, group=None, async_op=False):
    """All-gather equal-sized per-rank u64 flow-hash shards (torch int64
    tensors) into `out` (world * len(local)), rank-major = global order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    work = dist.all_gather_into_tensor(out, local, group=group, async_op=async_op)
    return (out, work) if async_op else out
