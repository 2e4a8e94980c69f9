"""Multi-GPU sharding of a codec batch.

Every batch element is compressed independently with its own statistics
and archive (reference README.md:110; ans/GpuANSEncode.cuh:686-711), so a
batch shards by contiguous element ranges with no data-path collective:
one process per GPU runs the full codec on its local HBM.  The only
exchange is an all-gather of the per-element compressed sizes -- RCCL over
xGMI on MI355X (backend "nccl"), gloo in the CPU tests -- from which every
rank derives the global packing offsets of the archives.
"""
import torch
import torch.distributed as dist


def shard_range(nb, rank, world):
    """Contiguous [start, stop) of ceil(nb / world) elements for `rank`."""
    per = -(-nb // world)
    start = min(nb, rank * per)
    return start, min(nb, start + per)


def gather_sizes(local_sizes, nb, group=None):
    """All-gather per-element compressed sizes (int32, one per local element)
    into the global [nb] vector (int64).  Shards are padded to the common
    per-rank length so a single all_gather_into_tensor suffices."""
    world = dist.get_world_size(group)
    per = -(-nb // world)
    buf = torch.zeros(per, dtype=torch.int32, device=local_sizes.device)
    buf[: local_sizes.numel()] = local_sizes.to(torch.int32)
    out = torch.empty(per * world, dtype=torch.int32, device=local_sizes.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    return out[:nb].to(torch.int64)


def archive_offsets(sizes, align=16):
    """Exclusive prefix of roundUp(size, align): where each element's archive
    lands when the batch is packed back to back (archives are 16 B aligned,
    SURVEY 8(b))."""
    r = (sizes + (align - 1)) // align * align
    return torch.cumsum(r, 0) - r
