"""Packet sharding across ranks and the gather of 32-bit results.

Packets are independent (crc32 carries no state across calls, Crc32.hpp:92-96), so a
batch of N packets is split into contiguous blocks, one per rank (one process per GPU,
torch.distributed over RCCL).  The only exchange step is a gather of each rank's
32-bit CRCs to rank 0 — nothing is reduced, so there is no all-reduce.
"""
from __future__ import annotations


def shard_range(rank: int, world: int, n: int) -> tuple[int, int]:
    """Packets [lo, hi) owned by `rank` for a batch of n packets (block partition)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return n * rank // world, n * (rank + 1) // world


def shard_byte_range(rank: int, world: int, n: int, stride: int) -> tuple[int, int]:
    lo, hi = shard_range(rank, world, n)
    return lo * stride, hi * stride


def gather_crcs(local, world: int, rank: int, dst: int = 0, group=None):
    """Gather every rank's int32 CRC tensor (equal lengths) to `dst`.

    Returns the concatenated tensor on `dst` (rank order = packet order for the block
    partition) and None elsewhere.  With the "nccl" backend this is an RCCL gather over
    xGMI; with "gloo" it runs on CPU tensors (tests).
    """
    import torch
    import torch.distributed as dist

    if world == 1:
        return local
    if rank == dst:
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.gather(local, gather_list=parts, dst=dst, group=group)
        return torch.cat(parts)
    dist.gather(local, gather_list=None, dst=dst, group=group)
    return None
