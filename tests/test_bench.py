"""bench.py host logic without a GPU: the N > 1 self-launch, the world-size check and the
parity digest lookup (the GPU legs run on the box)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_gpus_n_self_launches_n_ranks(monkeypatch):
    import bench
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 0

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_parity_digest_lookup():
    import bench
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        d = json.load(f)["sha256_by_packets"]
    assert set(d) >= {str(k << 20) for k in (1, 2, 4, 8, 16)}
    p = bench.parity_digest(np.zeros(5, np.uint32))
    assert p["match"] is None
    p = bench.parity_digest(np.zeros(1 << 20, np.uint32))
    assert p["match"] is False


def test_default_shard_sizes_make_gpus8_config_c4(monkeypatch):
    """The driver runs `bench.py --gpus N` with no other size flag; the self-launched
    ranks re-parse the same argv.  N = 1 must be the metric's 1 M x 1456 B, N = 8 must be
    config C4 (16 M x 1456 B = 2 M per rank), N = 2, 4 the same per-rank work."""
    import bench
    for gpus, ppr in ((1, 1 << 20), (2, 2 << 20), (4, 2 << 20), (8, 2 << 20)):
        monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", str(gpus), "--steps", "5", "--warmup", "5"])
        a = bench.parse()
        assert a.packets_per_rank == ppr == bench.default_packets_per_rank(gpus)
    assert 8 * bench.default_packets_per_rank(8) == 16777216
    assert bench.workload_name(8, 2 << 20).startswith("C4: 16 M")
    assert bench.workload_name(1, 1 << 20).startswith("target")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--packets-per-rank", "1000"])
    assert bench.parse().packets_per_rank == 1000
    # the reference digest for the gathered C4 vector exists
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        assert str(16777216) in json.load(f)["sha256_by_packets"]


def test_host_cores_reports_affinity_and_model():
    import bench
    hc = bench.host_cores()
    assert 1 <= hc["threads"] <= hc["affinity_cpus"] == len(os.sched_getaffinity(0))
    assert "model" in hc


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeW:
    """CPU stand-in for the binding (the oracle computes the CRCs): runs bench.py's legs
    through their real control flow without a GPU.  Test infrastructure only."""

    def __init__(self, O):
        self.O, self.reserved, self.launches = O, [], 0

    def synth_fill(self, out, start_byte=0, seed=0x5EED, nbytes=None, stream=None):
        import torch
        out[:nbytes] = torch.from_numpy(self.O.synth_fill_np(nbytes, start_byte=start_byte))

    def crc32_batch_fixed(self, buf, stride, length, n, out, stream=None):
        import torch
        self.launches += 1
        v = self.O.batch_fixed(buf.numpy()[:n * stride], stride, length, n)
        out.copy_(torch.from_numpy(v.view(np.int32)))

    def reserve_cus(self, k, device=0):
        self.reserved.append(k)


class _FakeEvent:
    def record(self, stream):
        import time
        self.t = time.perf_counter()

    def elapsed_time(self, end):
        return (end.t - self.t) * 1e3


def _fake_settle(step, stream, w_req, **kw):
    for _ in range(3):
        step()
    return 3, []


def _no_gpu(monkeypatch, bench):
    import torch
    monkeypatch.setattr(bench, "TimingEvent", _FakeEvent)
    monkeypatch.setattr(bench, "settle", _fake_settle)
    monkeypatch.setattr(torch.cuda, "Stream", lambda: "crc-stream")
    monkeypatch.setattr(torch.cuda, "current_stream", lambda: "default-stream")
    monkeypatch.setattr(torch.cuda, "set_stream", lambda s: None)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)


@pytest.mark.parametrize("every", [1, 3])
def test_n1_extra_legs_fields_on_cpu(monkeypatch, every):
    """The two legs the N = 1 line carries after its timed region: alt_buffer (two 1 M
    buffers in turn) and c4_shard_1gpu (the N > 1 pipelined step with a one-rank gather,
    here over gloo): fields, sizes, the CU reservation restored, and the gathered vector
    equal to the oracle's over the same packets (small n: the real leg runs 2 M)."""
    import hashlib

    import torch
    import torch.distributed as dist

    import bench
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
    import oracle as O
    import shard
    _no_gpu(monkeypatch, bench)
    W = _FakeW(O)
    n = 3000
    nbytes = n * bench.PAYLOAD
    buf = torch.zeros(nbytes + 64, dtype=torch.uint8)
    W.synth_fill(buf, nbytes=nbytes)
    alt = bench.alt_buffer_leg(W, buf, nbytes, n, "cpu", "default-stream", steps=4, warmup=5)
    assert alt["steps"] == 4 and alt["alt_buffer_kernel_ms"] == alt["kernel_ms_mean"] > 0
    assert {"GBs", "frac", "kernel_ms_median", "step_ms"} <= set(alt)

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        W.launches = 0
        c4 = bench.c4_shard_leg(W, shard, "cpu", 0, steps=4, warmup=5, n=n, every=every)
    finally:
        dist.destroy_process_group()
    assert c4["packets"] == n and c4["bytes_per_launch"] == nbytes and c4["steps"] == 4
    assert c4["gather_every"] == every  # every = 3 over 4 steps: one full group, one partial
    assert W.reserved == [8, 0]  # 8 CUs for the gather while the leg runs, then restored
    assert W.launches == 3 + 4 + 4  # settle, the timed steps, the instrumented pass: one launch each
    want = O.batch_fixed(O.synth_fill_np(nbytes), bench.PAYLOAD, bench.PAYLOAD, n)
    assert c4["sha256"] == hashlib.sha256(want.astype("<u4").tobytes()).hexdigest()[:16]
    assert c4["parity_match"] is None  # no reference digest at this size; the real leg has one
    assert {"kernel_ms_mean", "GBs", "frac", "step_ms", "value_GiBs"} <= set(c4)
    # the timed gathers (full groups + the flushed partial one) and the step time beyond the kernel
    assert c4["gathers"] == -(-4 // every) and c4["gather_ms"] > 0
    assert abs(c4["overlap"] - (c4["step_ms"] - c4["region_ms_per_step"])) < 1e-4  # one pass


def test_default_c4_leg_is_the_two_million_packet_shard():
    import inspect

    import bench
    sig = inspect.signature(bench.c4_shard_leg)
    assert sig.parameters["n"].default == 2097152 == bench.C4_PACKETS // 8


def test_pmc_record_matches_shipped_kernel():
    """profiles/pmc_traffic.json (the PMC pass behind roofline.traffic) was measured on the
    shipped k_fixed_braid<6>'s machine code.  This is the only test that fails on a stale
    record: refresh it with tools/gpu_round.sh (its `pmcnew` step runs first whenever
    tools/codeobj.py's hash differs) after a kernel change."""
    import bench
    sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
    import wtp_crc32 as W
    rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    v, info = bench.pmc_traffic(1 << 20, W.LIB_PATH)
    assert v == rec["hbm_bytes_per_launch"] and info["status"].startswith("measured"), info


def test_traffic_null_unless_kernel_code_matches(tmp_path):
    """roofline.traffic is a PMC record's number only while the shipped k_fixed_braid<6>
    has the code that record names: a record stamped with the shipped hash is reported,
    the same record with one flipped hex digit is null, another batch size is null.  (Built
    on a copy stamped with the shipped hash, so it holds whether or not the committed
    record is current: test_pmc_record_matches_shipped_kernel checks that.)"""
    import bench
    sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import codeobj
    import wtp_crc32 as W
    rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    h = codeobj.kernel_code_sha256(W.LIB_PATH, codeobj.HEADLINE_KERNEL)["sha256"]
    rec["kernel_code"]["sha256"] = h
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(rec))
    v, info = bench.pmc_traffic(1 << 20, W.LIB_PATH, str(p))
    assert v == rec["hbm_bytes_per_launch"] and info["status"].startswith("measured"), info
    rec["kernel_code"]["sha256"] = ("0" if h[0] != "0" else "1") + h[1:]
    p.write_text(json.dumps(rec))
    v, info = bench.pmc_traffic(1 << 20, W.LIB_PATH, str(p))
    assert v is None and info["status"].startswith("stale"), info
    v, info = bench.pmc_traffic(2 << 20, W.LIB_PATH, str(p))
    assert v is None


def test_extra_leg_failure_is_reported_not_fatal(monkeypatch):
    """A leg that cannot run (here the C4 leg's RCCL init raises) is recorded in the line
    and the other leg still runs; a leg with a wrong result vector fails the parity."""
    from types import SimpleNamespace

    import bench
    calls = []

    def alt(*a, **k):
        calls.append("alt")
        return {"kernel_ms_mean": 0.2}

    def c4_fail(*a, **k):
        raise RuntimeError("ProcessGroupNCCL is only supported with GPUs")

    monkeypatch.setattr(bench, "alt_buffer_leg", alt)
    monkeypatch.setattr(bench, "c4_shard_leg", c4_fail)
    args = SimpleNamespace(steps=3, warmup=1, gather_every=2)
    line, parity = {}, {"match": True}
    bench.run_extra_legs(line, parity, None, None, None, 0, 0, "cpu", 0, None, args)
    assert calls == ["alt"] and line["alt_buffer_kernel_ms"] == 0.2
    assert "RCCL" in line["c4_shard_1gpu"]["error"] or "NCCL" in line["c4_shard_1gpu"]["error"]
    assert parity == {"match": True}
    monkeypatch.setattr(bench, "c4_shard_leg", lambda *a, **k: {"parity_match": False})
    bench.run_extra_legs(line, parity, None, None, None, 0, 0, "cpu", 0, None, args)
    assert parity["c4_shard_1gpu"] is False


def test_rehearse_needs_more_than_one_gpu(monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--rehearse-one-gpu"])
    with pytest.raises(SystemExit):
        bench.parse()
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--rehearse-one-gpu", "--steps", "3"])
    a = bench.parse()
    assert a.rehearse_one_gpu and a.packets_per_rank == 2 << 20  # the production per-rank shard


def test_rehearsal_self_launch_keeps_the_flag(monkeypatch):
    """The rehearsal goes through the production self-launch: the ranks re-parse the same
    argv, flag included (read before any GPU call)."""
    import bench
    seen = {}
    monkeypatch.setattr(subprocess, "call", lambda cmd: seen.setdefault("cmd", cmd) and 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--rehearse-one-gpu", "--steps", "3"])
    with pytest.raises(SystemExit):
        bench.main()
    assert "--nproc-per-node=2" in seen["cmd"]
    assert seen["cmd"][-5:] == ["--gpus", "2", "--rehearse-one-gpu", "--steps", "3"]


def test_config_legs_zipf_is_the_oracle_generator():
    """The configs leg restates oracle.zipf_lengths (it may not import the oracle); the
    reference digests were made from the oracle's, so the two must agree bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import oracle as O
    import config_legs
    for n, s in ((1, 1.1), (1000, 1.0), (1 << 20, 1.1), (1 << 20, 1.0), (12345, 1.2)):
        assert np.array_equal(config_legs.zipf_lengths(n, s=s), O.zipf_lengths(n, s=s)), (n, s)


def test_config_digests_cover_every_row():
    """Every configs-leg parity key has a reference digest (tests/golden/config_digests.json
    from make_config_digests.py, bench_digests.json for the 1 M prefix)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import config_legs
    D = config_legs.digests()
    src = open(os.path.join(ROOT, "tools", "config_legs.py")).read()
    for k in ("c2", "c3_1gib", "hostbuild_1gib", "build_1m", "1048576", "verify_fixup_1m"):
        assert f'"{k}"' in src and len(D.get(k, "")) == 64, k
    assert 'f"c5_zipf{s}"' in src
    for k in ("c5_zipf1.1", "c5_zipf1.0"):
        assert len(D.get(k, "")) == 64, k


def test_config_digests_pinned_by_reference_on_small_prefix():
    """Spot check of the digest recipe: the C2 digest is the 64 K prefix of the same
    stream bench_digests.json's prefixes hash, recomputed here with the compiled reference
    (or the oracle when oracle/_ref is absent)."""
    import ctypes as C
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import oracle as O
    import config_legs
    n = 65536
    buf = O.synth_fill_np(n * 1456)
    ref = O.ref_lib()
    out = np.zeros(n, np.uint32)
    if ref is not None:
        ref.ref_crc32_batch_fixed(buf.ctypes.data, 1456, 1456, n, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    else:
        out = O.batch_fixed(buf, 1456, 1456, n)
    assert hashlib.sha256(out.astype("<u4").tobytes()).hexdigest() == config_legs.digests()["c2"]


def test_bench_product_legs_do_not_import_the_oracle():
    """Only bench.py's cpu_baseline leg (and its no-digest spot check) may touch oracle/;
    the configs leg checks parity against committed digests only."""
    src = open(os.path.join(ROOT, "tools", "config_legs.py")).read()
    assert "import oracle" not in src and "oracle/" not in src.replace("oracle/_ref", "")


def test_config_legs_parity_aggregation(monkeypatch):
    """configs leg bookkeeping on the CPU (row functions stubbed): every row's parity and
    the host rows' per-route parities are collected; one mismatch makes parity_all False
    (bench.py then exits non-zero), a row that raises is reported and leaves parity_all
    None unless a mismatch was also seen."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import config_legs as CL
    monkeypatch.setattr(CL, "Timer", lambda TE: None)
    monkeypatch.setattr(CL.torch.cuda, "empty_cache", lambda: None)
    ok = {"match": True}
    monkeypatch.setattr(CL, "c2", lambda W, T, D: {"config": "C2", "parity": ok})
    monkeypatch.setattr(CL, "c5", lambda W, T, D, s, stream_kernel=False: {"config": "C5", "parity": ok})
    monkeypatch.setattr(CL, "verify_and_build", lambda W, T, D: [{"config": "verify", "parity": ok}])
    host = [{"config": "C3", "pinned": {"parity": ok}, "pageable": {"parity": ok}}]
    monkeypatch.setattr(CL, "host_rows", lambda W, D: host)
    r = CL.run(None, None)
    assert r["parity_all"] is True and r["parity_checks"] == 7
    host[0]["pageable"]["parity"] = {"match": False}
    assert CL.run(None, None)["parity_all"] is False

    def boom(W, D):
        raise RuntimeError("no pinned memory")
    monkeypatch.setattr(CL, "host_rows", boom)
    r = CL.run(None, None)
    assert r["parity_all"] is None and any("error" in x for x in r["rows"])
    assert CL.run(None, None, only="c2")["parity_checks"] == 1
