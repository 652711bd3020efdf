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
    """Byte range of `rank`'s block of a fixed-stride batch."""
    lo, hi = shard_range(rank, world, n)
    return lo * stride, hi * stride


def shard_by_bytes(rank: int, world: int, lengths) -> tuple[int, int]:
    """Packets [lo, hi) of `rank` for a mixed-length batch, balanced by payload bytes
    rather than by count: rank r starts at the first packet whose
    exclusive byte prefix reaches r/world of the total.  Contiguous, disjoint, covering;
    every rank's byte share is within one packet (<= 4096 B) of total/world."""
    import numpy as np

    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    lens = np.asarray(lengths, dtype=np.uint64)
    excl = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]) if lens.size else np.zeros(0, np.uint64)
    total = int(lens.sum()) if lens.size else 0

    def start(r: int) -> int:
        if r >= world:
            return int(lens.size)
        return int(np.searchsorted(excl, (total * r + world - 1) // world, side="left"))

    return start(rank), start(rank + 1)


def gather_crcs(local, world: int, rank: int, dst: int = 0, group=None, out=None, n_total: int | None = None):
    """Gather every rank's int32 CRC tensor to `dst` in packet order.

    Returns the concatenated tensor on `dst` (rank order = packet order for the block
    partition) and None elsewhere.  `out` (on `dst`: world * local.numel() elements)
    receives the result in place, with no allocation per call.  With the "nccl"
    backend this is an RCCL gather over xGMI.  With "gloo" (CPU tests, or several ranks
    sharing one GPU) device tensors travel through host memory and the result is a
    CPU tensor.

    Equal shard sizes are the fast path.  Pass `n_total` (the batch size every rank
    partitioned with shard_range) and ragged block partitions (n % world != 0) go
    through gather_crcs_var; without it a shard whose size is not n_total / world is an
    error rather than a hang inside the collective.
    """
    import torch.distributed as dist

    if world == 1:
        return local
    if n_total is not None:
        counts = [hi - lo for lo, hi in (shard_range(r, world, n_total) for r in range(world))]
        if local.numel() != counts[rank]:
            raise ValueError(f"rank {rank}: local shard has {local.numel()} CRCs, shard_range gives {counts[rank]}")
        if len(set(counts)) > 1:
            return gather_crcs_var(local, counts, rank, dst=dst, group=group)
    if out is not None and rank == dst and out.numel() != world * local.numel():
        raise ValueError(f"out has {out.numel()} elements, expected {world} x {local.numel()}")
    on_host = local.is_cuda and dist.get_backend(group) == "gloo"
    if on_host:
        local = local.cpu()
        out = None
    if rank == dst:
        import torch
        full = out if out is not None else torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
        parts = list(full.view(world, -1).unbind(0))
        dist.gather(local, gather_list=parts, dst=dst, group=group)
        return full
    dist.gather(local, gather_list=None, dst=dst, group=group)
    return None


def gather_crcs_async(local, world: int, rank: int, out=None, dst: int = 0, group=None):
    """gather_crcs for equal shards without waiting: returns the collective's work handle
    (None when world == 1).  With "nccl" the gather runs on the collective's stream after
    the work already queued on the current stream; `work.wait()` makes the current
    stream wait for it, so `local` may be overwritten and `out` (required on `dst`, in
    the tensors' device memory) read after that.  A caller can so overlap the gather of
    one batch's results with the next batch's CRC launch.  With "gloo" the tensors must
    be host tensors.  A one-rank world gathers to itself (same code path)."""
    import torch.distributed as dist

    if rank == dst:
        if out is None or out.numel() != world * local.numel():
            raise ValueError(f"dst needs out with {world} x {local.numel()} elements")
        return dist.gather(local, gather_list=list(out.view(world, -1).unbind(0)), dst=dst, group=group, async_op=True)
    return dist.gather(local, gather_list=None, dst=dst, group=group, async_op=True)


def gather_crcs_var(local, counts, rank: int, dst: int = 0, group=None):
    """Gather per-rank CRC tensors of different lengths (the byte-balanced partition of
    a mixed-length batch, shard_by_bytes) to `dst`.  `counts[r]` = rank r's packet
    count, known to every rank (each computes the partition itself), so no extra
    exchange is needed: every rank pads to max(counts), one gather moves the data, and
    `dst` trims.  Returns the packet-ordered tensor on `dst`, None elsewhere."""
    import torch
    import torch.distributed as dist

    world = len(counts)
    if world == 1:
        return local
    m = max(counts)
    if local.is_cuda and dist.get_backend(group) == "gloo":
        local = local.cpu()
    padded = torch.zeros(m, dtype=local.dtype, device=local.device)
    padded[:local.numel()] = local
    if rank == dst:
        full = torch.empty(world * m, dtype=local.dtype, device=local.device)
        dist.gather(padded, gather_list=list(full.view(world, m).unbind(0)), dst=dst, group=group)
        return torch.cat([full[r * m:r * m + counts[r]] for r in range(world)])
    dist.gather(padded, gather_list=None, dst=dst, group=group)
    return None
