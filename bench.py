#!/usr/bin/env python3
"""bench.py — WTP CRC-32 hot path on MI355X (BASELINE.json metric).

One "step" = one pass of the hot path over one batch of synthetic, device-resident
1456-byte DATA payloads: the braided CRC kernel over this rank's shard, plus (N > 1)
the RCCL gather of the 32-bit results to rank 0.  Default shard sizes
(default_packets_per_rank): N = 1 runs the metric's own workload, 1 M x 1456 B; N > 1
runs config C4's per-GPU shard, 2 M x 1456 B per rank, so that N = 8 is exactly C4
(16 M packets over 8 GPUs) and N = 2, 4 are the same per-rank work (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N` (N > 1) without torchrun starts N rank processes itself (one per GPU).

Rank 0 prints ONE JSON line.  value = GiB/s of payload over all ranks (whole job, max
time over ranks); the timed region holds nothing between the launches but the work, one
HIP event pair on the CRC stream around it; roofline = the CRC kernel's algorithmic read
bytes per launch / (that region's event time / K) vs the 8 TB/s HBM peak, next to the same
box's streaming-read probe (a plain nt read kernel timed in the same process: a reference
point, not a bound); roofline.traffic = the PMC pass's HBM bytes, reported only while the
shipped kernel's code hash matches the one measured; roofline.instrumented_pass and
kernel_us_instrumented_pass = the same K steps run again with an event pair around every
launch (untimed: those events cost ~5 us per step); parity = sha256 of the whole result vector vs
the reference's digest; cpu_baseline = the reference's own crc32 (oracle/_ref, compiled
from cpp/src/common/Crc32.hpp) timed on this host's cores over a bounded sample.
N = 1 adds legs after the timed region (--no-extras skips them): alt_buffer (the
kernel alternating between two 1 M buffers, as a streaming sender would),
c4_shard_1gpu (rank 0's 2 M-packet C4 shard through the N > 1 pipelined step with a
one-rank RCCL gather: the equal-work reference for the N > 1 lines) and configs (every
other BASELINE config: C2, C3, C5 Zipf 1.1 / 1.0, receiver verify, the builders; each row
with back-to-back and graph times, its roofline fraction and parity of its whole result
against a reference-computed digest; tools/config_legs.py, --no-configs skips it).  N > 1
lines add per-rank kernel, region and gather times, step_ms and overlap (rank_fields).
--rehearse-one-gpu runs the N > 1 entry with every rank on device 0 over gloo (a
rehearsal of the driver's one-shot --gpus N run on a one-GPU box, not a measurement).
Warmup: see settle() — untimed launches until the clock transient has passed.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "a3-reliable-transport_amd")
sys.path.insert(0, PKG)

PAYLOAD = 1456
SEED = 0x5EED
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "GiB/s CRC-32 over device-resident 1456-B payloads; % of HBM read roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5, help="minimum untimed launches (see settle())")
    ap.add_argument("--packets-per-rank", type=int, default=None,
                    help="default: 1 M at N = 1 (the metric), 2 M at N > 1 (config C4's shard; N = 8 is C4)")
    ap.add_argument("--cpu-seconds", type=float, default=3.0,
                    help="target wall seconds of the 1-thread CPU-baseline leg (the all-thread leg runs 1/3 of it)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every core this job may run on (sched_getaffinity, capped by a cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the RCCL gather inside the step")
    ap.add_argument("--reserve-cus", type=int, default=None,
                    help="CUs the CRC kernel leaves free (wtp_reserve_cus); default 8 with the gather "
                         "(for the overlapped RCCL gather's workgroups), else 0")
    ap.add_argument("--gather-every", type=int, default=2,
                    help="with the gather: gather the results of this many steps in one collective (the step's "
                         "stream-event hops are paid once per group; 2: 0.480 -> 0.468 ms per C4 step, "
                         "profiles/r04e)")
    ap.add_argument("--result-groups", type=int, default=2,
                    help="with the gather: result-slot groups in rotation (a group is rewritten only after its "
                         "previous gather is done; more groups push that wait further behind)")
    ap.add_argument("--gather-helper", action="store_true",
                    help="A/B: issue the gathers from a helper stream joined to the CRC stream by fence-free events")
    ap.add_argument("--gather-n1", action="store_true",
                    help="N=1: run the pipelined RCCL gather in a one-rank world (exercises the N>1 step on one GPU)")
    ap.add_argument("--no-probe", action="store_true", help="skip the same-box streaming-read probe")
    ap.add_argument("--no-extras", action="store_true",
                    help="N = 1: skip the alternating-buffer and equal-work C4-shard legs (run after the timed region)")
    ap.add_argument("--no-configs", action="store_true",
                    help="N = 1: skip the configs leg (every other BASELINE config, tools/config_legs.py)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="REHEARSAL ONLY (N > 1 on a one-GPU box): every rank on device 0, a gloo process group, "
                         "the gathers hop through host tensors; everything else is the production --gpus N path")
    a = ap.parse_args()
    if a.rehearse_one_gpu and a.gpus < 2:
        ap.error("--rehearse-one-gpu rehearses the N > 1 path: it needs --gpus >= 2")
    if a.packets_per_rank is None:
        a.packets_per_rank = default_packets_per_rank(a.gpus)
    return a


C4_PACKETS = 16 << 20  # BASELINE.json configs[3]: 16 M x 1456 B over 8 GPUs


def default_packets_per_rank(gpus: int) -> int:
    """N = 1: the metric's 1 M x 1456 B.  N > 1: C4's per-GPU shard (16 M / 8 = 2 M), so
    the driver's plain `--gpus 8` run is config C4 and N = 2, 4 keep the same per-rank work."""
    return 1 << 20 if gpus <= 1 else C4_PACKETS // 8


def workload_name(world: int, n: int) -> str:
    if world == 1 and n == 1 << 20:
        return "target: 1 M x 1456 B on 1 GPU (BASELINE metric)"
    if world * n == C4_PACKETS and world == 8:
        return "C4: 16 M x 1456 B sharded over 8 GPUs + RCCL gather of the u32 results"
    if n == C4_PACKETS // 8:
        return f"C4 per-GPU shard (2 M x 1456 B) on {world} GPU(s)"
    return f"{n} x 1456 B per GPU on {world} GPU(s)"


def host_cores() -> dict:
    """Cores this job may run on: the affinity mask, capped by a cgroup v2 CPU quota if
    one is set (a 16-CPU share of a 256-core host shows all 256 in os.cpu_count()), and
    the CPU model from /proc/cpuinfo."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    use = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    return {"threads": use, "affinity_cpus": aff, "cgroup_cpu_quota": quota, "os_cpu_count": os.cpu_count(),
            "model": model}


def cpu_baseline(n_sample: int, seconds: float, threads: int, hc: dict | None = None) -> dict:
    """Reference crc32 (oracle/_ref) or, if it was not built, the oracle port."""
    import ctypes as C

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    ref = O.ref_lib()
    kind = "reference" if ref is not None else "port"
    buf = O.synth_fill_np(n_sample * PAYLOAD)
    out = np.zeros(n_sample, dtype=np.uint32)
    outp = out.ctypes.data_as(C.POINTER(C.c_uint32))

    def run(nthreads: int) -> float:
        if ref is not None:
            if nthreads == 1:
                ref.ref_crc32_batch_fixed(buf.ctypes.data, PAYLOAD, PAYLOAD, n_sample, outp)
            else:
                ref.ref_crc32_batch_fixed_mt(buf.ctypes.data, PAYLOAD, PAYLOAD, n_sample, outp, nthreads)
        else:
            O.lib().oracle_crc32_batch_fixed_mt(buf.ctypes.data, PAYLOAD, PAYLOAD, n_sample, outp, nthreads)
        return float(n_sample * PAYLOAD)

    res = {}
    for nt in (1, threads):
        run(nt)  # warm
        done, t0 = 0.0, time.perf_counter()
        budget = seconds if nt == 1 else seconds / 3
        while True:
            done += run(nt)
            el = time.perf_counter() - t0
            if el >= budget:
                break
        res[nt] = (done / el / 2**30, done, el)
    # sanity: the baseline computes the same CRCs as the oracle
    assert out[0] == O.crc32(buf[:PAYLOAD]) and out[-1] == O.crc32(buf[-PAYLOAD:])
    v1, vn = res[1], res[threads]
    # optional "optimised CPU" line: zlib's crc32 (Python's zlib module,
    # same polynomial/init/xorout), one thread over the same packets, ~1 s
    import zlib
    mv = memoryview(buf)
    zdone, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < min(1.0, seconds / 3):
        for i in range(0, n_sample * PAYLOAD, PAYLOAD):
            zlib.crc32(mv[i:i + PAYLOAD])
        zdone += n_sample * PAYLOAD
    zel = time.perf_counter() - t0
    assert zlib.crc32(mv[:PAYLOAD]) == int(out[0])
    return {
        "value": round(vn[0], 4), "unit": "GiB/s", "cores": threads, "kind": kind,
        "cpu_model": (hc or {}).get("model"),
        "cores_rule": "every CPU in this job's affinity mask, capped by its cgroup CPU quota" if hc else "--cpu-threads",
        "host": hc,
        "sample": f"{n_sample} x {PAYLOAD} B synthetic packets (seed 0x5EED), looped ~{seconds:.0f} s on 1 thread and ~{seconds/3:.0f} s on {threads}; "
                  f"{kind} = {'cpp/src/common/Crc32.hpp:91-102 compiled -O2 (oracle/_ref)' if ref else 'oracle/crc32_oracle.c'}",
        "value_1core": round(v1[0], 4),
        "cpu_seconds": round(v1[2] + vn[2] * threads + zel, 1),
        "optimised_cpu_1core": {"value": round(zdone / zel / 2**30, 4), "unit": "GiB/s", "impl": f"zlib {zlib.ZLIB_RUNTIME_VERSION} crc32 (not the reference)"},
    }


def pmc_traffic(n_packets: int, lib_path: str, path: str | None = None):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/pmc_traffic.json),
    and why it is or is not reported.  The record is stamped with the sha256 of the measured
    kernel's machine code (tools/pmc_traffic.py, tools/codeobj.py); if the shipped library's
    k_fixed_braid<6> differs, the number describes another kernel and traffic is null."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import codeobj

    p = path or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError) as e:
        return None, {"status": f"no PMC record ({e.__class__.__name__})"}
    if int(d.get("packets", -1)) != n_packets:
        return None, {"status": f"PMC record is for {d.get('packets')} packets, not {n_packets}"}
    want = (d.get("kernel_code") or {}).get("sha256")
    try:
        have = codeobj.kernel_code_sha256(lib_path, codeobj.HEADLINE_KERNEL)["sha256"]
    except Exception as e:  # noqa: BLE001 — diagnostics only: any ELF-parse failure is reported, never fatal
        return None, {"status": f"cannot hash the shipped kernel ({e.__class__.__name__}: {e})"}
    if want != have:
        return None, {"status": "stale: the shipped k_fixed_braid<6> code differs from the one the PMC pass measured",
                      "record_sha256": (want or "")[:16], "shipped_sha256": have[:16]}
    return d.get("hbm_bytes_per_launch"), {"status": "measured on this kernel code", "sha256": have[:16],
                                           "source": d.get("source"), "ratio_to_algorithmic": d.get("ratio_to_algorithmic")}


def self_launch(args) -> None:
    """--gpus N > 1 without a launcher: start N rank processes (torch.distributed.run,
    one per GPU) and exit with their status.  Runs before anything touches the GPU, so
    this process never initialises HIP."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    sys.exit(subprocess.call(cmd))


def settle(step, stream, w_req: int, block: int = 25, tol: float = 0.01, floor: int = 100, cap_s: float = 3.0,
           world: int = 1, flag_dev=None):
    """Untimed warmup: at least max(w_req, floor) launches, then until the mean launch
    time of three consecutive blocks of `block` launches agrees within `tol` (cap
    cap_s seconds).  A cold MI355X runs this kernel fast for ~5 launches, then the
    power controller pulls the clock down for launches ~5-50 (262 us vs 219 us steady,
    profiles/r02a/transient.json); a fixed 5-launch warmup times exactly that dip.
    world > 1: the stop decision is collective (all_reduce MAX of "keep going" on
    flag_dev after every block), so every rank runs the same number of steps.  With the
    gather, steps decide the collectives each rank issues: a rank-local count let rank 0
    flush a partial result group that rank 1 gathered whole, a mismatched gather
    (found by the --rehearse-one-gpu run, profiles/r06a)."""
    import torch

    means, done, t0 = [], 0, time.perf_counter()
    while True:
        s, e = TimingEvent(), TimingEvent()
        s.record(stream)
        for _ in range(block):
            step()
        e.record(stream)
        torch.cuda.synchronize()
        done += block
        means.append(s.elapsed_time(e) / block * 1e3)
        stop = (done >= max(w_req, floor) and len(means) >= 3 and max(means[-3:]) <= (1 + tol) * min(means[-3:])) \
            or (time.perf_counter() - t0 > cap_s and done >= w_req)
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([0 if stop else 1], dtype=torch.int32, device=flag_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            stop = int(t.item()) == 0
        if stop:
            break
    return done, [round(m, 1) for m in means]


_DIAG = None


def diag():
    """lib/libwtp_diag.so (include/wtp_diag.h): the read probe and timing-only events."""
    global _DIAG
    if _DIAG is None:
        import ctypes as C
        D = C.CDLL(os.path.join(PKG, "lib", "libwtp_diag.so"))
        D.wtp_diag_read_xor.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint, C.c_uint, C.c_void_p]
        D.wtp_diag_event_create.argtypes = [C.POINTER(C.c_void_p)]
        D.wtp_diag_event_record.argtypes = [C.c_void_p, C.c_void_p]
        D.wtp_diag_event_elapsed_ms.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_float)]
        D.wtp_diag_event_destroy.argtypes = [C.c_void_p]
        D.wtp_diag_stream_wait.argtypes = [C.c_void_p, C.c_void_p]
        _DIAG = D
    return _DIAG


class TimingEvent:
    """A HIP event for timing only (hipEventDisableSystemFence, via libwtp_diag): recording
    it does no system-scope cache writeback/invalidate, which the default event does and
    which both pads the measured interval and slows the next launch."""

    def __init__(self):
        import ctypes as C
        self._C = C
        self.e = C.c_void_p()
        if diag().wtp_diag_event_create(C.byref(self.e)) != 0:
            raise RuntimeError("wtp_diag_event_create failed")

    def record(self, stream):
        if diag().wtp_diag_event_record(self.e, self._C.c_void_p(stream.cuda_stream)) != 0:
            raise RuntimeError("wtp_diag_event_record failed")

    def elapsed_time(self, end) -> float:
        ms = self._C.c_float()
        if diag().wtp_diag_event_elapsed_ms(self.e, end.e, self._C.byref(ms)) != 0:
            raise RuntimeError("wtp_diag_event_elapsed_ms failed")
        return ms.value

    def __del__(self):
        try:
            diag().wtp_diag_event_destroy(self.e)
        except Exception:
            pass


def read_probe(buf, nbytes: int, crc_step, stream, cus: int, reps: int = 10) -> dict:
    """Same-box streaming-read probe: a plain nt dwordx4 read + XOR over the same bytes
    (lib/libwtp_diag.so), 10 launches interleaved with the CRC kernel after the timed
    region, medians of both.  A reference point for this box's HBM, not a bound: the CRC
    kernel has matched it or run up to ~1% faster (its waves keep more rows in flight)."""
    import torch

    D = diag()
    sink = torch.zeros(4, dtype=torch.int32, device=buf.device)
    pe, ce = [], []

    def ev():
        return TimingEvent(), TimingEvent()

    for i in range(reps + 2):
        s, e = ev()
        s.record(stream)
        if D.wtp_diag_read_xor(buf.data_ptr(), nbytes, sink.data_ptr(), cus, 512, stream.cuda_stream) != 0:
            raise RuntimeError("wtp_diag_read_xor failed")
        e.record(stream)
        s2, e2 = ev()
        s2.record(stream)
        crc_step()
        e2.record(stream)
        if i >= 2:
            pe.append((s, e))
            ce.append((s2, e2))
    torch.cuda.synchronize()
    p = sorted(s.elapsed_time(e) for s, e in pe)[len(pe) // 2]
    c = sorted(s.elapsed_time(e) for s, e in ce)[len(ce) // 2]
    return {"probe": f"nt buffer dwordx4 read + XOR, {cus}x512 threads, same {nbytes} B",
            "median_us": round(p * 1e3, 1), "GBs": round(nbytes / (p * 1e-3) / 1e9, 1),
            "crc_interleaved_median_us": round(c * 1e3, 1)}


def parity_digest(vec_u32) -> dict:
    """sha256 of the whole result vector vs the reference's digest for that many packets
    (tests/golden/bench_digests.json, tests/golden/make_bench_digests.py)."""
    import hashlib

    import numpy as np

    got = hashlib.sha256(np.ascontiguousarray(vec_u32).astype("<u4").tobytes()).hexdigest()
    try:
        with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
            want = json.load(f)["sha256_by_packets"].get(str(len(vec_u32)))
    except OSError:
        want = None
    return {"packets": len(vec_u32), "sha256": got[:16],
            "match": None if want is None else got == want,
            "vs": "reference crc32 over the same packets (tests/golden/bench_digests.json)" if want else "no digest"}


def init_one_rank_group(local: int) -> None:
    """A one-rank RCCL world on this process's GPU (the --gather-n1 step, and the equal-work
    C4 shard leg of the N = 1 line): the N > 1 step's code path on one GPU."""
    import socket

    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        s.close()
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")  # the gathers' own durations (Pipe.gather_ms)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))


class Pipe:
    """Step i: the CRC of this rank's shard into a result slot on `stream`, then (with the
    gather) the RCCL gather of the results to rank 0, asynchronous: it runs on the
    collective's stream, on the CUs the CRC kernel leaves free (wtp_reserve_cus), while
    the next steps' CRCs run.  Result slots come in `groups` groups (default 2) of `every` slots; a group is
    gathered in one collective when it is full (every = 1: each step's results right
    after its launch), and rewritten only after that gather is done.  `bufs` may hold
    several shards of equal size: step i reads bufs[i % len(bufs)] (the alternating-buffer
    leg).  `gathered` (rank 0) holds 2 x world x every x n results: one half per group."""

    def __init__(self, W, shard, bufs, n, stream, do_gather, world, rank, gathered, dev, every=1, groups=2,
                 helper=False, host_hop=False):
        import torch
        self.W, self.shard, self.bufs, self.n, self.stream = W, shard, bufs, n, stream
        # --rehearse-one-gpu (gloo): each group's results go to a host tensor before the
        # gather (gloo gathers host tensors); `gathered` is then a host tensor on rank 0
        self.host_hop = host_hop
        self._hop_src = {}
        self.do_gather, self.world, self.rank, self.gathered = do_gather, world, rank, gathered
        self.K = max(1, int(every)) if do_gather else 1
        ng = max(2, int(groups)) if do_gather else 1
        self.groups = [torch.empty(self.K * n, dtype=torch.int32, device=dev) for _ in range(ng)]
        self.works = [None] * len(self.groups)
        self.i = 0       # steps launched
        self.pos = 0     # result slots used (a flush skips to the next group)
        self.last_m, self.last_g = 0, 0  # slots and group of the last gather
        self.last_pos = 0
        self.timed = False  # time_steps sets it: the gathers issued meanwhile are timed
        self.gather_rec = []
        # --gather-helper (A/B option): the collectives are issued from a helper stream that
        # meets the CRC stream only through fence-free events, so torch's own cross-stream
        # events are recorded on the helper, not between the CRC launches
        self.helper = None
        if helper and do_gather and hasattr(stream, "cuda_stream"):
            self.helper = torch.cuda.Stream()
        self._keep = []  # events of the current step pair (alive until their waits are queued)

    def _hop(self, src, dst):
        """dst waits for everything queued on src so far (a fence-free event)."""
        ev = TimingEvent()
        ev.record(src)
        if diag().wtp_diag_stream_wait(dst.cuda_stream, ev.e) != 0:
            raise RuntimeError("wtp_diag_stream_wait failed")
        self._keep.append(ev)

    def _time_gather(self, work):
        """Record one gather for gather_ms().  RCCL: the collective's own duration on its
        stream, from ProcessGroupNCCL's start/end events (TORCH_NCCL_ENABLE_TIMING=1, which
        main() sets before the process group exists; no extra stream or event of ours, so
        nothing is queued beside the CRC stream's hardware queue).  gloo (CPU tests): the
        host clock from the issue to the work's future completing."""
        rec = self.gather_rec[-1]
        rec["work"] = work
        if not hasattr(self.stream, "cuda_stream") or self.host_hop:
            rec["t0"] = time.perf_counter()
            work.get_future().then(lambda f, rec=rec: rec.__setitem__("t1", time.perf_counter()))

    def gather_ms(self) -> list:
        """Durations (ms) of the gathers issued while `timed` (call after drain())."""
        out = []
        for r in self.gather_rec:
            d = None
            if "t1" in r:
                d = (r["t1"] - r["t0"]) * 1e3
            elif "work" in r:
                try:
                    d = float(r["work"]._get_duration())
                except Exception:  # noqa: BLE001 — timing not enabled / backend without it: not reported
                    d = None
            if d is not None:
                out.append(d)
        return out

    def _group(self, pos):
        return (pos // self.K) % len(self.groups)

    def wait_slot(self):
        if self.pos % self.K == 0:  # first slot of a group: its previous gather must be done
            g = self._group(self.pos)
            if self.works[g] is not None:
                if self.helper is not None:
                    import torch
                    with torch.cuda.stream(self.helper):
                        self.works[g].wait()
                    self._hop(self.helper, self.stream)
                else:
                    self.works[g].wait()
                self.works[g] = None

    def launch(self):
        k = self.pos % self.K
        out = self.groups[self._group(self.pos)][k * self.n:(k + 1) * self.n]
        self.W.crc32_batch_fixed(self.bufs[self.i % len(self.bufs)], PAYLOAD, PAYLOAD, self.n, out, self.stream)
        self.last_pos = self.pos

    def _gather(self, m):
        # each group gathers into its own half of `gathered`: two gathers may be in flight
        # at once, and a process group need not complete them in order (gloo does not)
        g = self._group(self.pos - 1)
        out = None
        if self.gathered is not None:
            half = self.world * self.K * self.n
            out = self.gathered[g * half:g * half + self.world * m * self.n]
        if self.timed:
            self.gather_rec.append({"steps": m})
        if self.host_hop:  # rehearsal: device results -> host (waits for the CRC stream), gloo gather
            with torch_stream(self.stream):
                src = self.groups[g][:m * self.n].cpu()
            self._hop_src[g] = src  # alive until the gather is waited for
            self.works[g] = self.shard.gather_crcs_async(src, self.world, self.rank, out=out)
        elif self.helper is not None:
            import torch
            self._hop(self.stream, self.helper)
            with torch.cuda.stream(self.helper):
                self.works[g] = self.shard.gather_crcs_async(self.groups[g][:m * self.n], self.world, self.rank,
                                                             out=out)
            if len(self._keep) > 64:
                self._keep = self._keep[-8:]
        else:
            self.works[g] = self.shard.gather_crcs_async(self.groups[g][:m * self.n], self.world, self.rank, out=out)
        if self.timed and self.works[g] is not None:
            self._time_gather(self.works[g])
        self.last_m, self.last_g = m, g

    def finish(self):
        self.i += 1
        self.pos += 1
        if self.do_gather and self.pos % self.K == 0:
            self._gather(self.K)

    def step(self):
        self.wait_slot()
        self.launch()
        self.finish()

    def flush(self):
        """Gather a partly filled group (the end of a timed region), then start a new group."""
        m = self.pos % self.K
        if self.do_gather and m:
            self._gather(m)
            self.pos += self.K - m

    def drain(self):
        self.flush()
        for b, w in enumerate(self.works):
            if w is not None:
                if self.helper is not None:
                    import torch
                    with torch.cuda.stream(self.helper):
                        w.wait()
                    self._hop(self.helper, self.stream)
                else:
                    w.wait()
                self.works[b] = None

    def last_out(self):
        g, k = self._group(self.last_pos), self.last_pos % self.K
        return self.groups[g][k * self.n:(k + 1) * self.n]

    def gathered_vector(self):
        """Rank 0 after drain(): the gathered u32 results of the last step of every rank, in
        rank order (each rank's block of the last gather holds last_m result vectors)."""
        m, half = self.last_m, self.world * self.K * self.n
        g = self.gathered[self.last_g * half:self.last_g * half + self.world * m * self.n]
        return g.view(self.world, m * self.n)[:, (m - 1) * self.n:].reshape(-1)


def torch_stream(stream):
    """torch.cuda.stream(stream) for a HIP stream; no-op for the CPU tests' stand-in."""
    import contextlib

    import torch
    return torch.cuda.stream(stream) if hasattr(stream, "cuda_stream") else contextlib.nullcontext()


def time_steps(pipe: Pipe, steps: int, world: int, per_launch: bool = False):
    """Exactly `steps` steps, barrier + synchronize on both sides.  One HIP event pair on
    the CRC stream brackets the whole run (the gather runs on the collective's stream).
    per_launch=False is the timed region: nothing between the launches but the work (an
    event pair around every launch cost ~5 us per 215 us step, 2.5%: profiles/r05v).
    per_launch=True adds that pair around every launch: the instrumented pass that gives
    the per-launch kernel times.  Returns (per-launch kernel ms or None, ms between the
    two region events, wall seconds; this rank only)."""
    import torch
    import torch.distributed as dist

    starts = [TimingEvent() for _ in range(steps)] if per_launch else None
    ends = [TimingEvent() for _ in range(steps)] if per_launch else None
    r0, r1 = TimingEvent(), TimingEvent()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    pipe.gather_rec, pipe.timed = [], True  # the gathers of these steps are timed (Pipe.gather_ms)
    t0 = time.perf_counter()
    r0.record(pipe.stream)
    for i in range(steps):
        pipe.wait_slot()  # (stream-side) before the start event: it times the kernel alone
        if per_launch:
            starts[i].record(pipe.stream)
        pipe.launch()
        if per_launch:
            ends[i].record(pipe.stream)
        pipe.finish()
    r1.record(pipe.stream)
    pipe.drain()  # gathers a partly filled group, waits for every gather
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    pipe.timed = False
    kern = [s.elapsed_time(e) for s, e in zip(starts, ends)] if per_launch else None
    return kern, r0.elapsed_time(r1), el


def rank_fields(kern_ms: list, gather_ms: list, el: float, steps: int, world: int, dev,
                region_ms: float | None = None) -> tuple[float, dict]:
    """The N > 1 line's per-rank fields (collectives: every rank must call this).  el =
    this rank's wall seconds and region_ms its CRC-stream event time, both from the timed
    pass; kern_ms = per-launch times from the instrumented pass.  Returns (max over ranks
    of el, fields):
      per_rank_kernel_ms, kernel_ms_max_over_ranks — mean CRC launch time per rank
        (instrumented pass);
      per_rank_region_ms — the timed pass's CRC-stream time per step (its two events / K:
        the launches plus any stream wait for a result slot);
      per_rank_gather_ms, gather_ms_max_over_ranks — mean duration of a gather collective
        on its own stream (ProcessGroupNCCL's timing events, Pipe._time_gather; gloo: host
        clock); gathers_per_rank = collectives timed in the timed region;
      step_ms — wall time per step (max over ranks);
      overlap — step_ms - max(per_rank_region_ms), both from the timed pass: the step time
        the CRC stream does not explain.  About 0 when the gather hides behind the next
        CRC launches; about gather_ms / gather_every when it serialises with them.
    The collectives run on `dev` with RCCL and on host tensors with gloo."""
    import torch
    import torch.distributed as dist

    if dist.get_backend() == "gloo":
        dev = torch.device("cpu")
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    km = sum(kern_ms) / len(kern_ms)
    gm = sum(gather_ms) / len(gather_ms) if gather_ms else 0.0
    rm = region_ms / steps if region_ms is not None else km
    mine = torch.tensor([km, gm, float(len(gather_ms)), rm], dtype=torch.float64, device=dev)
    allr = [torch.zeros(4, dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(allr, mine)
    rows = [[float(v) for v in x.tolist()] for x in allr]
    per_k = [round(r[0], 5) for r in rows]
    per_g = [round(r[1], 5) for r in rows]
    per_r = [round(r[3], 5) for r in rows]
    step_ms = round(el / steps * 1e3, 4)
    return el, {"per_rank_kernel_ms": per_k, "kernel_ms_max_over_ranks": max(per_k),
                "per_rank_region_ms": per_r,
                "per_rank_gather_ms": per_g, "gather_ms_max_over_ranks": max(per_g),
                "gathers_per_rank": [int(r[2]) for r in rows],
                "step_ms": step_ms, "overlap": round(step_ms - max(per_r), 5),
                "overlap_rule": "step_ms - max(per_rank_region_ms), both from the timed pass: ~0 = gather hidden "
                                "behind the CRC launches, ~gather_ms / gather_every = serialised"}


def kstats(kern: list, nbytes: int) -> dict:
    ks = sorted(kern)
    mean = sum(ks) / len(ks)
    gbs = nbytes / (mean * 1e-3) / 1e9
    return {"kernel_ms_mean": round(mean, 5), "kernel_ms_median": round(ks[len(ks) // 2], 5),
            "GBs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


def c4_shard_leg(W, shard, dev, local: int, steps: int, warmup: int, n: int = C4_PACKETS // 8, every: int = 1,
                 groups: int = 2) -> dict:
    """Equal-work reference for the N > 1 lines, in the N = 1 process: rank 0's C4 shard
    (2 M x 1456 B = 3.05 GB, the first 2 M packets of the global stream) through the SAME
    pipelined step the N > 1 ranks run (own stream, 8 reserved CUs, the asynchronous RCCL
    gather of the u32 results, here in a one-rank world), checked against the reference's
    2 M digest.  N = 1 times 1 M packets and N > 1 2 M per rank, and the 2 M launch is a few
    percent slower per byte, so scaling efficiency on equal work is
    value(N) / (N x this leg's GiB/s)."""
    import torch
    import torch.distributed as dist

    nbytes = n * PAYLOAD
    fresh = not dist.is_initialized()
    if fresh:
        init_one_rank_group(local)
    buf = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
    W.synth_fill(buf, start_byte=0, seed=SEED, nbytes=nbytes)
    stream = torch.cuda.Stream()
    prev = torch.cuda.current_stream()
    torch.cuda.set_stream(stream)
    W.reserve_cus(8, torch.cuda.current_device())
    try:
        gathered = torch.empty(max(2, groups) * every * n, dtype=torch.int32, device=dev)
        pipe = Pipe(W, shard, [buf], n, stream, True, 1, 0, gathered, dev, every=every, groups=groups)
        settle(pipe.step, stream, warmup)
        pipe.drain()
        torch.cuda.synchronize()
        _, region_ms, el = time_steps(pipe, steps, 1)  # timed: step_ms, value_GiBs
        gms = pipe.gather_ms()
        kern, _, _ = time_steps(pipe, steps, 1, per_launch=True)  # instrumented: kernel time
        import numpy as np
        par = parity_digest(pipe.gathered_vector().cpu().numpy().view(np.uint32))
    finally:
        W.reserve_cus(0, torch.cuda.current_device())
        torch.cuda.set_stream(prev)
        if fresh:
            dist.destroy_process_group()
    out = {"what": "rank 0's C4 shard (2 M x 1456 B) through the N > 1 step on this GPU: own stream, "
                   "8 reserved CUs, asynchronous one-rank RCCL gather of the u32 results",
           "packets": n, "bytes_per_launch": nbytes, "steps": steps,
           "gather_every": pipe.K,
           "step_ms": round(el / steps * 1e3, 4), "value_GiBs": round(nbytes * steps / el / 2**30, 2),
           "region_ms_per_step": round(region_ms / steps, 5),
           "parity_match": par["match"], "sha256": par["sha256"],
           "timing": "step_ms / value_GiBs: a timed pass with no events between launches; kernel_ms_*: a "
                     "second pass of as many steps with an event pair around every launch"}
    out.update(kstats(kern, nbytes))
    out["gather_ms"] = round(sum(gms) / len(gms), 5) if gms else None
    out["gathers"] = len(gms)
    out["overlap"] = round(out["step_ms"] - out["region_ms_per_step"], 5)
    out["overlap_rule"] = "step_ms - region_ms_per_step, both from the timed pass"
    del buf
    return out


def alt_buffer_leg(W, buf, nbytes: int, n: int, dev, stream, steps: int, warmup: int) -> dict:
    """The headline kernel over two different 1 M-packet buffers in turn: no launch re-reads
    what the previous launch read, as in a streaming sender or receiver.  The headline
    `value` re-reads one buffer every step (the metric's workload); DESIGN 7.11 measured
    ~5% between the two."""
    import torch

    buf2 = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
    W.synth_fill(buf2, start_byte=nbytes, seed=SEED, nbytes=nbytes)
    pipe = Pipe(W, None, [buf, buf2], n, stream, False, 1, 0, None, dev)
    settle(pipe.step, stream, warmup)
    torch.cuda.synchronize()
    if pipe.i % 2:
        pipe.step()
    _, region_ms, el = time_steps(pipe, steps, 1)
    if pipe.i % 2:
        pipe.step()
    kern, _, _ = time_steps(pipe, steps, 1, per_launch=True)
    out = {"what": "k_fixed_braid<6> alternating between two 1 M x 1456 B buffers (the next 1 M packets "
                   "of the stream), current stream, no gather",
           "steps": steps, "step_ms": round(el / steps * 1e3, 4), "region_ms_per_step": round(region_ms / steps, 5),
           "timing": "step_ms: a timed pass with no events between launches; kernel_ms_*: a second pass with an "
                     "event pair around every launch"}
    out.update(kstats(kern, nbytes))
    out["alt_buffer_kernel_ms"] = out["kernel_ms_mean"]
    del buf2
    return out


def run_extra_legs(line: dict, parity: dict, W, shard, buf, nbytes: int, n: int, dev, local: int, stream, args) -> None:
    """The N = 1 line's alt_buffer and c4_shard_1gpu legs.  A leg that cannot run (e.g. no
    RCCL on the box) is reported in the line instead of failing the run; a leg whose
    results differ from the reference's digest marks the parity as failed."""
    try:
        line["alt_buffer"] = alt_buffer_leg(W, buf, nbytes, n, dev, stream, args.steps, args.warmup)
        line["alt_buffer_kernel_ms"] = line["alt_buffer"]["kernel_ms_mean"]
    except (RuntimeError, OSError) as e:  # WtpError is a RuntimeError
        line["alt_buffer"] = {"error": f"{e.__class__.__name__}: {e}"[:300]}
    try:
        line["c4_shard_1gpu"] = c4_shard_leg(W, shard, dev, local, args.steps, args.warmup, every=args.gather_every,
                                             groups=getattr(args, "result_groups", 2))
        if line["c4_shard_1gpu"]["parity_match"] is False:
            parity["c4_shard_1gpu"] = False
    except (RuntimeError, OSError) as e:
        line["c4_shard_1gpu"] = {"error": f"{e.__class__.__name__}: {e}"[:300]}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        self_launch(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rehearse = args.rehearse_one_gpu  # every rank on device 0, gloo, gathers through host tensors
    if world > 1 or args.gather_n1:
        torch.cuda.set_device(0 if rehearse else local)
        if world == 1:
            init_one_rank_group(local)
        elif rehearse:
            dist.init_process_group("gloo")
        else:
            os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")  # the gathers' own durations (Pipe.gather_ms)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    import shard
    import wtp_crc32 as W

    n = args.packets_per_rank
    nbytes = n * PAYLOAD
    dev = torch.device("cuda", torch.cuda.current_device())
    if W.LIB.wtp_init(torch.cuda.current_device()) != 0:
        raise W.WtpError(W.LIB.wtp_last_error().decode())
    cus = torch.cuda.get_device_properties(dev).multi_processor_count

    # this rank's contiguous shard of the global packet stream, generated on-device
    buf = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
    W.synth_fill(buf, start_byte=rank * nbytes, seed=SEED, nbytes=nbytes)
    do_gather = (world > 1 or args.gather_n1) and not args.no_gather
    # with the gather, the CRC launches get a stream of their own (the collective's stream
    # then syncs with it, not with the legacy default stream)
    stream = torch.cuda.Stream() if do_gather else torch.cuda.current_stream()
    torch.cuda.set_stream(stream)
    reserve = args.reserve_cus if args.reserve_cus is not None else (8 if do_gather else 0)
    if reserve:
        W.reserve_cus(reserve, torch.cuda.current_device())
    every = args.gather_every if do_gather else 1
    ngroups = max(2, args.result_groups) if do_gather else 1
    gdev = torch.device("cpu") if rehearse else dev
    gathered = torch.empty(ngroups * world * every * n, dtype=torch.int32, device=gdev) if do_gather and rank == 0 else None
    pipe = Pipe(W, shard, [buf], n, stream, do_gather, world, rank, gathered, dev, every=every, groups=ngroups,
                helper=args.gather_helper and not rehearse, host_hop=rehearse and do_gather)
    out = torch.empty(n, dtype=torch.int32, device=dev)  # the read-probe leg's CRC launches

    def crc():
        W.crc32_batch_fixed(buf, PAYLOAD, PAYLOAD, n, out, stream)

    warm_done, warm_means = settle(pipe.step, stream, args.warmup, world=world,
                                   flag_dev=torch.device("cpu") if rehearse else dev)
    pipe.drain()
    torch.cuda.synchronize()

    # the timed region: exactly K steps, nothing between the launches but the work
    _, region_ms, el = time_steps(pipe, args.steps, world)
    kernel_name = W.LIB.wtp_last_kernel().decode()  # the instantiation the timed launches used
    gms = pipe.gather_ms()
    kmean = region_ms / args.steps  # average launch duration over the timed region (its two events)
    # then as many steps again with an event pair around every launch (untimed diagnostics:
    # the per-launch distribution, and the kernel time the N > 1 `overlap` is read against)
    kern, _, _ = time_steps(pipe, args.steps, world, per_launch=True)
    kern_ms = sorted(kern)
    kmean_pl = sum(kern_ms) / len(kern_ms)

    per_rank = None
    if world > 1 or args.gather_n1:  # --gather-n1: the same fields from a one-rank RCCL world
        el, per_rank = rank_fields(kern, gms, el, args.steps, world, dev, region_ms=region_ms)

    # parity of the WHOLE result vector (rank 0: the gathered vector when N > 1)
    parity = None
    if rank == 0:
        import numpy as np
        vec = (pipe.gathered_vector() if gathered is not None else pipe.last_out()).cpu().numpy().view(np.uint32)
        parity = parity_digest(vec)
        if parity["match"] is None:  # no reference digest for this size: oracle spot check
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            parity["spot_check_vs_oracle"] = all(
                int(vec[i]) == O.crc32(O.synth_fill_np(PAYLOAD, start_byte=i * PAYLOAD))
                for i in (0, 1, len(vec) // 2, len(vec) - 1))
    probe = read_probe(buf, nbytes, crc, stream, cus) if not args.no_probe else None

    total_bytes = float(nbytes) * world * args.steps
    value = total_bytes / el / 2**30
    achieved = nbytes / (kmean * 1e-3) / 1e9  # GB/s, algorithmic read bytes per launch
    traffic, traffic_info = pmc_traffic(n, W.LIB_PATH)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 seed 0x5EED, generated on-device per rank shard)",
        "config": {"workload": workload_name(world, n),
                   "step": f"crc32 of {n} x {PAYLOAD}-B DATA payloads per GPU, device-resident"
                           + (" + RCCL gather of u32 results to rank 0" if do_gather else ""),
                   "packets_per_rank": n, "payload_bytes": PAYLOAD, "global_packets": n * world,
                   "parallelism": f"packet shards x{world}" if world > 1 else "single GPU",
                   "gather": (("REHEARSAL: gloo gather of host copies to rank 0" if rehearse else
                               "RCCL gather to rank 0, overlapped with the next step's CRC") if do_gather else None),
                   "gather_every": every if do_gather else None,
                   "result_groups": ngroups if do_gather else None,
                   "gather_helper_stream": bool(args.gather_helper) if do_gather else None,
                   "reserved_cus": reserve},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_check": traffic_info,
                     "kernel": kernel_name, "kernel_ms_mean": round(kmean, 5),
                     "kernel_ms_rule": "HIP events on the CRC stream around the timed region's K launches, / K"
                                       + (" (with the gather this is the CRC stream's time per step: the launch "
                                          "plus any wait for a free result slot)" if do_gather else ""),
                     "instrumented_pass": {"what": "the same K steps again, an event pair around every launch "
                                                   "(not part of value: ~5 us per step, profiles/r05v)",
                                           "kernel_ms_mean": round(kmean_pl, 5),
                                           "kernel_ms_median": round(kern_ms[len(kern_ms) // 2], 5),
                                           "kernel_ms_p10": round(kern_ms[len(kern_ms) // 10], 5),
                                           "kernel_ms_p90": round(kern_ms[(9 * len(kern_ms)) // 10], 5)},
                     "bytes_per_launch": nbytes,
                     "frac_of_same_box_read_probe": round(achieved / probe["GBs"], 4) if probe else None},
        "kernel_us_instrumented_pass": [round(k * 1e3, 1) for k in kern],
        "warmup_run": warm_done,
        "warmup_rule": "max(--warmup, 100) launches, then until 3 consecutive 25-launch block means agree "
                       "within 1% (cap 3 s); untimed",
        "warmup_block_mean_us": warm_means,
        "same_box_read_probe": probe,
        "pct_hbm_read_roofline": round(100 * achieved / HBM_PEAK_GBS, 2),
        "parity": parity,
    }
    if per_rank is not None:
        line.update(per_rank)
    if rehearse:
        line["rehearsal"] = {"what": f"--rehearse-one-gpu: {world} ranks share device 0 over gloo; gathers hop "
                                     "through host tensors. Exercises the --gpus N entry end to end; its timings "
                                     "are NOT a scaling measurement",
                             "backend": dist.get_backend()}
    extras = rank == 0 and world == 1 and not args.gather_n1 and n == 1 << 20 and not args.no_extras
    if extras:  # after the timed region and the probe: neither leg touches the headline numbers
        run_extra_legs(line, parity, W, shard, buf, nbytes, n, dev, local, stream, args)
    if extras and not args.no_configs:  # every other BASELINE config, parity vs reference digests
        torch.cuda.empty_cache()
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import config_legs
        line["configs"] = config_legs.run(W, TimingEvent)
        if line["configs"]["parity_all"] is False:
            parity["configs"] = False
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        hc = host_cores()
        threads = args.cpu_threads or hc["threads"]
        line["cpu_baseline"] = cpu_baseline(65536, args.cpu_seconds, threads, hc)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    if parity is not None and (parity["match"] is False or parity.get("c4_shard_1gpu") is False
                               or parity.get("configs") is False):
        sys.exit("bench.py: result vector differs from the reference digest")


if __name__ == "__main__":
    main()
