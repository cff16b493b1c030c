"""Multi-GPU slicing of a block batch.

Blocks are independent, so a batch partitions into contiguous slices, one per
GPU (one process per GPU, torch.distributed over RCCL for the control plane
only). There is no collective on the data path: every rank checksums its
slice from its own HBM. `gather_slices` is a result-collection helper for
verification and for callers that want the whole CRC array on every rank; it
moves 4 B per block.
"""
from __future__ import annotations

from typing import List, Tuple


def shard_range(nblocks: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous slice [start, start+count) of rank `rank`: N // G blocks per
    rank, the remainder spread over the first ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    per, extra = divmod(nblocks, world)
    start = rank * per + min(rank, extra)
    return start, per + (1 if rank < extra else 0)


def all_ranges(nblocks: int, world: int) -> List[Tuple[int, int]]:
    return [shard_range(nblocks, r, world) for r in range(world)]


def gather_slices(local, nblocks: int, group=None):
    """All-gather every rank's slice result (1-D tensor of its `count`
    entries) into the full nblocks-long array, in block order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    ranges = all_ranges(nblocks, world)
    width = max(c for _, c in ranges) if ranges else 0
    padded = torch.zeros(width, dtype=local.dtype, device=local.device)
    padded[: local.numel()] = local
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    return torch.cat([p[:c] for p, (_, c) in zip(parts, ranges)])
