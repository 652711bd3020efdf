"""N > 1 path on CPU: block partition of packets across ranks + gather of the 32-bit
results to rank 0 (a3-reliable-transport_amd/shard.py), world_size 2 and 4 with gloo.
Each rank checksums its own contiguous shard of the global synthetic stream (the same
global byte offsets bench.py uses) — here with the CPU oracle, on the GPU box with the
HIP kernel (tests/test_gpu_shard.py) — and rank 0 compares the gathered vector with
the single-process result."""
import os
import socket
import sys

import numpy as np
import pytest

import shard

PAYLOAD = 1456


def test_shard_ranges_cover_disjoint():
    for n in (0, 1, 7, 1000, 1 << 20, 16_777_216):
        for world in (1, 2, 3, 4, 8):
            got = [shard.shard_range(r, world, n) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            for (a, b), (c, d) in zip(got, got[1:]):
                assert b == c and a <= b
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(2, 2, 10)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q, use_gpu=False):
    """One rank: checksum packets shard_range(rank) of the global synthetic stream (CPU
    oracle, or the HIP kernel on cuda:0 when use_gpu), then gather to rank 0."""
    import sys
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "a3-reliable-transport_amd"), os.path.join(here, "..", "oracle")):
        sys.path.insert(0, p)
    import shard as S
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = S.shard_range(rank, world, n_total)
    if use_gpu:
        import wtp_crc32 as W
        torch.cuda.set_device(0)
        buf = torch.empty((hi - lo) * PAYLOAD + 16, dtype=torch.uint8, device="cuda")
        W.synth_fill(buf, start_byte=lo * PAYLOAD, nbytes=(hi - lo) * PAYLOAD)
        t = torch.empty(hi - lo, dtype=torch.int32, device="cuda")
        W.crc32_batch_fixed(buf, PAYLOAD, PAYLOAD, hi - lo, t)
        torch.cuda.synchronize()
    else:
        import oracle as O
        shard_bytes = O.synth_fill_np((hi - lo) * PAYLOAD, start_byte=lo * PAYLOAD)
        local = O.batch_fixed(shard_bytes, PAYLOAD, PAYLOAD, hi - lo)
        t = torch.from_numpy(local.view(np.int32).copy())
    full = S.gather_crcs(t, world, rank, n_total=n_total)
    if rank == 0:
        q.put(full.cpu().numpy().view(np.uint32).copy())
    dist.barrier()
    dist.destroy_process_group()


def run_ranks(world, n_total, use_gpu=False):
    """Spawn `world` ranks (gloo), return rank 0's gathered vector."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q, use_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world,n_total", [(2, 1024), (4, 2048), (3, 1001), (4, 4099), (8, 8 * 2048 + 5)])
def test_gather_matches_single_process(world, n_total):
    """Equal shards (fast gather) and ragged block partitions (n % world != 0: padded
    gather through gather_crcs_var) both return the single-process vector."""
    got = run_ranks(world, n_total)
    import oracle as O
    want = O.batch_fixed(O.synth_fill_np(n_total * PAYLOAD), PAYLOAD, PAYLOAD, n_total)
    assert np.array_equal(got, want)


def test_gather_rejects_wrong_shard_size():
    import torch
    with pytest.raises(ValueError):
        shard.gather_crcs(torch.zeros(5, dtype=torch.int32), 2, 0, n_total=12)


def test_shard_by_bytes_balanced():
    import oracle as O
    for lens in (O.zipf_lengths(100_000, s=1.1), O.zipf_lengths(5000, s=1.0), np.full(7, 1456), np.array([4096] * 3),
                 np.array([], dtype=np.uint32), np.array([0, 0, 5, 0])):
        total = int(np.sum(lens, dtype=np.uint64))
        for world in (1, 2, 3, 4, 8):
            rs = [shard.shard_by_bytes(r, world, lens) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == len(lens)
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c and a <= b
            for a, b in rs:
                share = int(np.sum(lens[a:b], dtype=np.uint64))
                assert abs(share - total / world) <= 4096 + 1, (world, share, total / world)


def _worker_var(rank, world, port, q):
    import sys
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "a3-reliable-transport_amd"), os.path.join(here, "..", "oracle")):
        sys.path.insert(0, p)
    import oracle as O
    import shard as S
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lens = O.zipf_lengths(3000, s=1.1)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    data = O.synth_fill_np(int(lens.sum()), start_byte=77)
    ranges = [S.shard_by_bytes(r, world, lens) for r in range(world)]
    lo, hi = ranges[rank]
    local = O.batch_var(data, offs[lo:hi], lens[lo:hi])
    t = torch.from_numpy(local.view(np.int32).copy())
    full = S.gather_crcs_var(t, [b - a for a, b in ranges], rank)
    if rank == 0:
        q.put(full.numpy().view(np.uint32).copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_mixed_length_byte_shards_gather(world):
    """C5-style batch: byte-balanced shards (unequal packet counts) + padded gather."""
    import torch.multiprocessing as mp
    import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_var, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    lens = O.zipf_lengths(3000, s=1.1)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    data = O.synth_fill_np(int(lens.sum()), start_byte=77)
    assert np.array_equal(got, O.batch_var(data, offs, lens))


def _async_worker(rank, world, port, steps, q):
    """Pipelined gather as bench.py runs it: step i writes slot i % 2, the gather of
    step i is in flight while step i+1 is computed, a slot is rewritten only after its
    gather was waited for.  Rank r's step-i values are r * 1000 + i * 7 + lane."""
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "a3-reliable-transport_amd"))
    import shard as S
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 257
    outs = [torch.empty(n, dtype=torch.int32) for _ in range(2)]
    works = [None, None]
    gathered = [torch.empty(world * n, dtype=torch.int32) for _ in range(steps)] if rank == 0 else [None] * steps
    for i in range(steps):
        b = i % 2
        if works[b] is not None:
            works[b].wait()
        outs[b].copy_(torch.arange(n, dtype=torch.int32) + rank * 1000 + i * 7)
        works[b] = S.gather_crcs_async(outs[b], world, rank, out=gathered[i])
    for w in works:
        if w is not None:
            w.wait()
    if rank == 0:
        q.put([g.numpy().copy() for g in gathered])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_gather_async_pipelined(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    steps = 5
    procs = [ctx.Process(target=_async_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n = 257
    for i, g in enumerate(got):
        want = np.concatenate([np.arange(n) + r * 1000 + i * 7 for r in range(world)]).astype(np.int32)
        assert np.array_equal(g, want), i


def test_gather_async_requires_out_on_dst():
    """The asynchronous gather has no allocation path: dst must pass `out` of world x n."""
    import torch
    with pytest.raises(ValueError):
        shard.gather_crcs_async(torch.zeros(4, dtype=torch.int32), 2, 0, out=None)
    with pytest.raises(ValueError):
        shard.gather_crcs_async(torch.zeros(4, dtype=torch.int32), 2, 0, out=torch.zeros(7, dtype=torch.int32))


def _bench_pipe_worker(rank, world, port, every, steps, q, groups=2, host_hop=False):
    """bench.py's own Pipe (results gathered in groups of `every` steps, two groups in
    flight, a partial group flushed at the end) over gloo, with a stand-in launch that
    writes rank * 1000 + step * 7 + lane into the step's result slot."""
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "a3-reliable-transport_amd")):
        sys.path.insert(0, p)
    import bench
    import shard as S
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 257

    class FakeW:
        calls = 0

        def crc32_batch_fixed(self, buf, stride, length, nn, out, stream=None):
            out.copy_(torch.arange(nn, dtype=torch.int32) + rank * 1000 + FakeW.calls * 7)
            FakeW.calls += 1

    gathered = torch.empty(groups * world * every * n, dtype=torch.int32) if rank == 0 else None
    pipe = bench.Pipe(FakeW(), S, [None], n, "stream", True, world, rank, gathered, "cpu", every=every, groups=groups,
                      host_hop=host_hop)
    seen = []
    real = S.gather_crcs_async

    def spy(local, w, r, out=None, **kw):
        seen.append(local.numel() // n)
        return real(local, w, r, out=out, **kw)

    S.gather_crcs_async = spy
    for _ in range(steps):
        pipe.step()
    pipe.drain()
    if rank == 0:
        q.put((pipe.gathered_vector().numpy().copy(), seen))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,every,steps,groups,host_hop", [(2, 1, 3, 2, False), (2, 2, 5, 2, False),
                                                               (3, 4, 6, 2, False), (8, 2, 5, 2, False),
                                                               (2, 2, 9, 3, False), (3, 1, 7, 8, False),
                                                               (2, 2, 5, 2, True), (3, 1, 4, 2, True)])
def test_bench_pipe_grouped_gather(world, every, steps, groups, host_hop):
    """host_hop: the --rehearse-one-gpu form of the pipe (each group copied to a host
    tensor, then a gloo gather), same vector and collectives."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_pipe_worker, args=(r, world, port, every, steps, q, groups, host_hop))
             for r in range(world)]
    for p in procs:
        p.start()
    got, seen = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n = 257
    want = np.concatenate([np.arange(n) + r * 1000 + (steps - 1) * 7 for r in range(world)]).astype(np.uint32)
    assert np.array_equal(got.view(np.uint32), want)
    # full groups of `every` results, then the partial group the drain flushes
    assert seen == [every] * (steps // every) + ([steps % every] if steps % every else [])


class _WallEvent:
    """Host-clock stand-in for bench.TimingEvent (no GPU here)."""

    def record(self, stream):
        import time
        self.t = time.perf_counter()

    def elapsed_time(self, end):
        return (end.t - self.t) * 1e3


def _rank_fields_worker(rank, world, port, every, steps, q):
    """bench.py's N > 1 timed region (time_steps over its Pipe, gathers every `every`
    steps) and its per-rank fields (rank_fields) over gloo, with a stand-in launch."""
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "a3-reliable-transport_amd")):
        sys.path.insert(0, p)
    import bench
    import shard as S
    bench.TimingEvent = _WallEvent
    torch.cuda.synchronize = lambda *a: None
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 4099

    class FakeW:
        def crc32_batch_fixed(self, buf, stride, length, nn, out, stream=None):
            out.copy_(torch.arange(nn, dtype=torch.int32) + rank)

    gathered = torch.empty(2 * world * every * n, dtype=torch.int32) if rank == 0 else None
    pipe = bench.Pipe(FakeW(), S, [None], n, "stream", True, world, rank, gathered, "cpu", every=every)
    for _ in range(3):  # untimed warmup: its gathers are not counted
        pipe.step()
    pipe.drain()
    _, region, el = bench.time_steps(pipe, steps, world)  # the timed pass
    gms = pipe.gather_ms()
    kern, _, _ = bench.time_steps(pipe, steps, world, per_launch=True)  # the instrumented pass
    assert kern is not None and len(kern) == steps and region > 0
    el_max, f = bench.rank_fields(kern, gms, el, steps, world, "cpu", region_ms=region)
    if rank == 0:
        q.put((f, el_max, el))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,every,steps", [(8, 2, 5), (2, 1, 4)])
def test_bench_rank_fields_gather_and_overlap(world, every, steps):
    """The N > 1 line's overlap fields: per-rank gather time, gathers
    per rank (the timed region's collectives only: full groups plus the flushed partial
    one), overlap = step_ms - max(per_rank_region_ms) (both timed pass),
    maxima consistent with the lists."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_fields_worker, args=(r, world, port, every, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    f, el_max, el0 = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(f["per_rank_kernel_ms"]) == len(f["per_rank_gather_ms"]) == world
    assert f["gathers_per_rank"] == [-(-steps // every)] * world
    assert all(g > 0 for g in f["per_rank_gather_ms"]) and all(k > 0 for k in f["per_rank_kernel_ms"])
    assert f["kernel_ms_max_over_ranks"] == max(f["per_rank_kernel_ms"])
    assert f["gather_ms_max_over_ranks"] == max(f["per_rank_gather_ms"])
    assert el_max >= el0 and f["step_ms"] == round(el_max / steps * 1e3, 4)
    assert len(f["per_rank_region_ms"]) == world and all(r > 0 for r in f["per_rank_region_ms"])
    assert abs(f["overlap"] - (f["step_ms"] - max(f["per_rank_region_ms"]))) < 1e-4


def _settle_worker(rank, world, port, q):
    """bench.settle over gloo with rank-dependent launch times: rank 0's settle within
    three blocks, rank 1's never (noisy) until the cap.  The stop decision must be
    collective, or the ranks' Pipes issue different gathers (r06a: a partial group on
    one rank, a whole one on the other -> gloo size mismatch; RCCL would hang)."""
    import random
    import time as _t

    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "a3-reliable-transport_amd")):
        sys.path.insert(0, p)
    import bench
    import shard as S
    bench.TimingEvent = _WallEvent
    torch.cuda.synchronize = lambda *a: None
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 64

    class FakeW:
        def crc32_batch_fixed(self, buf, stride, length, nn, out, stream=None):
            _t.sleep(0.001 if rank == 0 else random.choice((0.0005, 0.003)))
            out.copy_(torch.arange(nn, dtype=torch.int32) + rank)

    gathered = torch.empty(2 * world * 2 * n, dtype=torch.int32) if rank == 0 else None
    pipe = bench.Pipe(FakeW(), S, [None], n, "stream", True, world, rank, gathered, "cpu", every=2)
    done, _ = bench.settle(pipe.step, "stream", 5, block=5, floor=10, cap_s=0.6, world=world, flag_dev="cpu")
    pipe.drain()
    _, _, el = bench.time_steps(pipe, 3, world)
    alld = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(alld, torch.tensor([done]))
    if rank == 0:
        q.put(([int(x) for x in alld], pipe.gathered_vector().numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_settle_is_collective_with_uneven_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_settle_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    dones, vec = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert dones[0] == dones[1]  # one step count on every rank, so the same gathers
    assert np.array_equal(vec, np.concatenate([np.arange(64) + r for r in range(2)]).astype(np.int32))
