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
