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
