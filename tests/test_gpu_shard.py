"""Multi-GPU path on the GPU box, through the HIP kernel.

- Two / three gloo ranks share the one GPU: each runs wtp_crc32_batch_fixed on its
  block shard of the global synthetic stream and shard.gather_crcs collects the u32
  results on rank 0 (equal and ragged partitions), compared element-wise with the
  oracle.
- One full C4 per-rank shard (2,097,152 x 1456 B = 3.05 GB, the first > 2 GB braided
  launch) synthesised at rank 7's global byte offset, element-wise vs the oracle.
- The RCCL gather itself (nccl backend) on a one-rank group over the HIP results.

Packets are independent (crc32 keeps no state across calls, Crc32.hpp:92-96), so a
block partition is exact.
"""
import os
import socket

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
PAYLOAD = 1456
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def W():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import wtp_crc32 as W
    assert W.LIB.wtp_init(0) == 0, W.LIB.wtp_last_error()
    return W


@pytest.mark.parametrize("world,n_total", [(2, 65536), (3, 100_003)])
def test_ranks_share_gpu_hip_shards_gather(W, world, n_total):
    from test_dist import run_ranks
    got = run_ranks(world, n_total, use_gpu=True)
    want = O.batch_fixed(O.synth_fill_np(n_total * PAYLOAD), PAYLOAD, PAYLOAD, n_total, threads=THREADS)
    bad = np.nonzero(got != want)[0]
    assert got.size == n_total and bad.size == 0, (bad.size, bad[:5])


def test_c4_rank7_shard_3gb_elementwise(W):
    """Config C4: 16 M packets over 8 GPUs = 2,097,152 per rank.  Rank 7's shard starts
    at global byte 7 * 2,097,152 * 1456 (21.4 GB into the stream)."""
    n = 2_097_152
    start = 7 * n * PAYLOAD
    nbytes = n * PAYLOAD
    buf = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf, start_byte=start, nbytes=nbytes)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    W.crc32_batch_fixed(buf, PAYLOAD, PAYLOAD, n, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    host = buf[:nbytes].cpu().numpy()
    # the device bytes are the generator's bytes at that global offset (three 1 MiB windows)
    for off in (0, nbytes // 2 - (1 << 19), nbytes - (1 << 20)):
        assert np.array_equal(host[off:off + (1 << 20)], O.synth_fill_np(1 << 20, start_byte=start + off)), off
    want = O.batch_fixed(host, PAYLOAD, PAYLOAD, n, threads=THREADS)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad.size, bad[:5])
    del buf, host


def _rccl_worker(port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "a3-reliable-transport_amd")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import wtp_crc32 as W
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    n = 4096
    buf = torch.empty(n * PAYLOAD, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    W.crc32_batch_fixed(buf, PAYLOAD, PAYLOAD, n, t)
    full = torch.empty(n, dtype=torch.int32, device="cuda")
    dist.gather(t, gather_list=[full], dst=0)  # RCCL gather (one rank: the collective path, no peer)
    torch.cuda.synchronize()
    q.put((dist.get_backend(), full.cpu().numpy().view(np.uint32).copy()))
    dist.destroy_process_group()


def test_rccl_gather_one_rank(W):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = ctx.Process(target=_rccl_worker, args=(port, q))
    p.start()
    backend, got = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl"
    want = O.batch_fixed(O.synth_fill_np(4096 * PAYLOAD), PAYLOAD, PAYLOAD, 4096)
    assert np.array_equal(got, want)


def _group_run(tmp_path, devs, n_per, root):
    import subprocess
    import sys
    out = str(tmp_path / "g.npy")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "group_worker.py"),
                        out, ",".join(map(str, devs)), ",".join(map(str, n_per)), str(root)],
                       capture_output=True, text=True, timeout=120)
    return r, (np.load(out) if r.returncode == 0 else None)


@pytest.mark.parametrize("n", [1, 100_003, 1 << 20])
def test_group_gather_one_device(W, tmp_path, n):
    """libwtp_group.so (one process, RCCL communicator from ncclCommInitAll): the
    braided kernel on the shard, then ncclGather of the u32 results to the root."""
    r, got = _group_run(tmp_path, [0], [n], 0)
    assert r.returncode == 0, r.stdout + r.stderr
    want = O.batch_fixed(O.synth_fill_np(n * PAYLOAD), PAYLOAD, PAYLOAD, n, threads=THREADS)
    assert np.array_equal(got, want)


def test_group_gather_all_devices(W, tmp_path):
    """Every visible device one rank, ragged shards (grouped send/recv); on a one-GPU
    box this is the single-rank ragged-capable path."""
    nd = torch.cuda.device_count()
    n_per = [4099 + 7 * r for r in range(nd)]
    r, got = _group_run(tmp_path, list(range(nd)), n_per, nd - 1)
    assert r.returncode == 0, r.stdout + r.stderr
    total = sum(n_per)
    want = O.batch_fixed(O.synth_fill_np(total * PAYLOAD), PAYLOAD, PAYLOAD, total, threads=THREADS)
    assert np.array_equal(got, want)


def test_bench_pipelined_gather_one_rank(W):
    """bench.py's N > 1 step (CRC on its own stream, asynchronous RCCL gather of the
    results double-buffered behind the next launch, 8 reserved CUs) in a one-rank RCCL
    world: the gathered vector's sha256 equals the reference digest for 1 M packets."""
    import json
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gather-n1", "--steps", "5", "--warmup", "5",
                        "--no-cpu-baseline", "--no-probe"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["config"]["gather"] and line["config"]["reserved_cus"] == 8
    assert line["parity"]["match"] is True, line["parity"]
    # the N > 1 line's per-rank fields, here from RCCL collectives in a one-rank world
    assert line["per_rank_kernel_ms"] == [line["kernel_ms_max_over_ranks"]] and line["kernel_ms_max_over_ranks"] > 0
    every = line["config"]["gather_every"]
    assert line["gathers_per_rank"] == [-(-5 // every)] and line["per_rank_gather_ms"][0] > 0  # full groups + the flushed one
    assert abs(line["overlap"] - (line["step_ms"] - max(line["per_rank_region_ms"]))) < 1e-4


def test_bench_c4_shard_gather_one_rank(W):
    """The per-rank work of the driver's `bench.py --gpus 8` (config C4: 2,097,152 x
    1456 B per rank) through the pipelined RCCL gather in a one-rank world: the gathered
    vector's sha256 equals the reference digest for 2 M packets (bench_digests.json)."""
    import json
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gather-n1", "--packets-per-rank", "2097152",
                        "--steps", "5", "--warmup", "5", "--no-cpu-baseline", "--no-probe"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["config"]["packets_per_rank"] == 2097152 and line["config"]["gather"]
    assert line["parity"]["packets"] == 2097152 and line["parity"]["match"] is True, line["parity"]


def test_bench_n1_line_carries_equal_work_c4_leg(W):
    """The default N = 1 line (the driver's invocation, shortened): the metric's 1 M
    packets, plus c4_shard_1gpu — rank 0's 2 M-packet C4 shard through the N > 1 pipelined
    step with a one-rank RCCL gather, its gathered vector equal to the reference's 2 M
    digest — and alt_buffer."""
    import json
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "5", "--warmup", "5",
                        "--no-cpu-baseline", "--no-probe"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["config"]["packets_per_rank"] == 1 << 20 and line["parity"]["match"] is True
    # the configs leg: every other BASELINE config, each row with its
    # back-to-back and graph times, frac, and parity of the whole result vs a reference digest
    cf = line["configs"]
    assert cf["parity_all"] is True, json.dumps(cf)[:3000]
    rows = {r["config"].split(":")[0]: r for r in cf["rows"]}
    assert not any("error" in r for r in cf["rows"]), [r for r in cf["rows"] if "error" in r]
    for name in ("C2", "C5", "verify", "build"):
        dev_rows = [r for r in cf["rows"] if r["config"].startswith(name)]
        assert dev_rows, name
        for r in dev_rows:
            assert r["b2b_ms"] > 0 and r["graph_ms"] > 0 and 0 < r["graph_frac"] <= 1.0, r
            assert r["parity"]["match"] is True, r
    assert sum(r["config"].startswith("C5") for r in cf["rows"]) == 3  # Zipf 1.1, 1.0, and k_stream forced
    for name, legs in (("C3", ("pinned", "pageable")), ("hostbuild", ("pinned", "pinned_staged", "pageable"))):
        for leg in legs:
            assert rows[name][leg]["parity"]["match"] is True and rows[name][leg]["seconds"] > 0, (name, leg)
    c4 = line["c4_shard_1gpu"]
    assert c4["packets"] == 2097152 and c4["parity_match"] is True, c4
    assert c4["steps"] == 5 and 0 < c4["kernel_ms_mean"] <= c4["step_ms"] * 1.5
    assert line["alt_buffer_kernel_ms"] == line["alt_buffer"]["kernel_ms_mean"] > 0
    assert c4["gathers"] >= 1 and c4["gather_ms"] > 0 and "overlap" in c4
    # roofline.traffic depends on the committed PMC record, not on this run's results:
    # tests/test_bench.py::test_pmc_record_matches_shipped_kernel checks the record
    assert "traffic_check" in line["roofline"]


@pytest.mark.parametrize("gpus", [2, 4])
def test_bench_rehearse_gpus2_end_to_end(W, gpus):
    """the driver's one-shot `bench.py --gpus N` entry, rehearsed with
    N = 2 and 4 on this one-GPU box: self-launch through torch.distributed.run, the WORLD_SIZE
    check, per-rank synth_fill at rank * nbytes, reserve_cus, the real braided launches,
    rank_fields' collectives and the gathered N x 2 M vector against the reference's
    4 M / 8 M-packet digest.  Only the device map (both ranks on device 0), the backend
    (gloo) and the gather's host hop differ from production."""
    import json
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(gpus), "--rehearse-one-gpu",
                        "--steps", "3"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == gpus and line["rehearsal"]["backend"] == "gloo"
    assert line["config"]["packets_per_rank"] == 2097152 and line["config"]["global_packets"] == gpus * 2097152
    assert line["config"]["reserved_cus"] == 8
    assert line["parity"]["packets"] == gpus * 2097152 and line["parity"]["match"] is True, line["parity"]
    for k in ("per_rank_kernel_ms", "per_rank_region_ms", "per_rank_gather_ms", "gathers_per_rank"):
        assert len(line[k]) == gpus, k
    assert all(v > 0 for v in line["per_rank_kernel_ms"]) and all(v > 0 for v in line["per_rank_gather_ms"])
    assert abs(line["overlap"] - (line["step_ms"] - max(line["per_rank_region_ms"]))) < 1e-4
    assert line["value"] > 0 and line["steps"] == 3
