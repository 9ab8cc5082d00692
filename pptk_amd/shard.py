"""Multi-GPU sharding of an rx batch -- the host-side
mirror of the C-ABI's multi-GPU part (include/pptk_rx.h, "Multi-GPU";
pptk_amd/csrc/rx_comm.hip).

Frames are independent, so a batch of n frames is split into contiguous
ranges, one per GPU (one process per GPU here; one thread per GPU in
examples/rx_multigpu.c), with no data-path collective.  The one exchange
step is the all-gather of the per-frame flow hashes (u64): RCCL's
ncclAllGather over xGMI on the communicator each rank's pptk_rx_ctx owns.
Shards are equal (pptk_rx_shard_range: ceil(n / world) frames, the last
ones padded), so the gathered array holds global frame i's hash at index i.

The kernel writes each rank's hashes straight into its own slice of the
gather buffer (pptk_rx_dev_batch.d_hash = out + rank * per) and the
all-gather runs in place: no staging copy, no extra HBM pass.

The uid of the communicator is made on rank 0 and handed to the others over
the job's host control plane (a torch.distributed gloo group here; a file,
socket or MPI in a C application).
"""
from .rx import comm_uid, shard_range  # noqa: F401  (re-exported)


def join(ctx, world, rank, group=None):
    """Join RxContext `ctx` to a new `world`-rank RCCL communicator as
    `rank`; rank 0 makes the uid and broadcasts it over the (gloo)
    torch.distributed `group` (default: the world group)."""
    import torch.distributed as dist
    obj = [comm_uid() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(obj, src=0, group=group)
    ctx.comm_create(world, rank, obj[0])


class GatherBuffer:
    """The all-gather destination of one rank: world * per u64 hashes on
    `device`, and `local`, this rank's slice, which the rx kernel fills
    (d_hash) before the in-place all-gather."""

    def __init__(self, n_total, world, rank, device, inplace=True, out=None):
        import torch
        self.first, self.count, self.per = shard_range(n_total, world, rank)
        self.n_total, self.world, self.rank = n_total, world, rank
        if out is None:
            out = torch.zeros(world * self.per, dtype=torch.int64, device=device)
        # (a caller-placed buffer: bench.placed_gather)
        self.out = out.view(torch.int64)[:world * self.per]
        if inplace:
            self.local = self.out[rank * self.per: rank * self.per + self.per]
        else:   # (experiments: a separate send buffer, so even one rank copies)
            self.local = torch.zeros(self.per, dtype=torch.int64, device=device)

    def gather(self, ctx, stream=None):
        """pptk_rx_allgather_hash of `per` hashes per rank, in place."""
        ctx.allgather_hash(self.local, self.per, self.out, stream=stream)
        return self.out[:self.n_total]
