#!/usr/bin/env python3
"""Interleaved A/B of the C4 per-rank leg: why BENCH_r04 -> r05 moved
the c4_shard_1gpu kernel from 0.43736 to 0.44832 ms.  One process, one GPU, `--rounds`
rounds; each round runs every variant once in turn (order rotated per round), each over
the same 2 M x 1456 B shard (rank 0's C4 shard), `--steps` steps like the driver's run:

  head        bench.c4_shard_leg as shipped: TORCH_NCCL_ENABLE_TIMING=1, timed pass with no
              events, then an instrumented pass (an event pair per launch) for kernel_ms
  head_notime the same with TORCH_NCCL_ENABLE_TIMING=0 (no ProcessGroupNCCL timing events)
  r04pipe     round 4's leg: timing off, ONE pass with an event pair around every launch
              giving both kernel_ms and step_ms (bench.time_steps(per_launch=True))
  plain       no gather, no Pipe: 2 M launches on a side stream with 8 reserved CUs, an
              event pair per launch (kernel_ms) and one pair around the run (region)
  pipe_nogather  bench.Pipe without the gather (side stream, 8 reserved CUs): the Pipe's own
              cost, so plain vs pipe_nogather vs head splits the gap into Pipe and gather
  head_every4 head with the results of 4 steps per gather (half the collectives)

Every variant with a process group makes its own one-rank RCCL group (fresh port) and
destroys it.  Prints one JSON line per run and a summary (medians over rounds).
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
import shard  # noqa: E402
import wtp_crc32 as W  # noqa: E402

P, N = 1456, 2 * 1048576


def fresh_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    os.environ["MASTER_PORT"] = str(p)


def head(steps, timing, every=2):
    os.environ["TORCH_NCCL_ENABLE_TIMING"] = "1" if timing else "0"
    fresh_port()
    r = bench.c4_shard_leg(W, shard, torch.device("cuda", 0), 0, steps, 5, every=every, groups=2)
    return {"kernel_ms": r["kernel_ms_mean"], "kernel_median_ms": r["kernel_ms_median"], "step_ms": r["step_ms"],
            "region_ms": r["region_ms_per_step"], "parity": r["parity_match"]}


def r04pipe(steps, buf):
    """Round 4's c4_shard_leg: one timed pass, event pair per launch, timing off."""
    os.environ["TORCH_NCCL_ENABLE_TIMING"] = "0"
    fresh_port()
    bench.init_one_rank_group(0)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    prev = torch.cuda.current_stream()
    torch.cuda.set_stream(st)
    W.reserve_cus(8, 0)
    try:
        gathered = torch.empty(2 * 2 * N, dtype=torch.int32, device=dev)
        pipe = bench.Pipe(W, shard, [buf], N, st, True, 1, 0, gathered, dev, every=2, groups=2)
        bench.settle(pipe.step, st, 5)
        pipe.drain()
        torch.cuda.synchronize()
        kern, region, el = bench.time_steps(pipe, steps, 1, per_launch=True)
        par = bench.parity_digest(pipe.gathered_vector().cpu().numpy().view(np.uint32))["match"]
    finally:
        W.reserve_cus(0, 0)
        torch.cuda.set_stream(prev)
        dist.destroy_process_group()
    ks = sorted(kern)
    return {"kernel_ms": sum(ks) / len(ks), "kernel_median_ms": ks[len(ks) // 2], "step_ms": el / steps * 1e3,
            "region_ms": region / steps, "parity": par}


def pipe_nogather(steps, buf):
    """bench.Pipe without the gather on a side stream, 8 reserved CUs: the pipe's own cost."""
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    W.reserve_cus(8, 0)
    try:
        pipe = bench.Pipe(W, None, [buf], N, st, False, 1, 0, None, dev)
        bench.settle(pipe.step, st, 5)
        torch.cuda.synchronize()
        _, region, el = bench.time_steps(pipe, steps, 1)
        kern, _, _ = bench.time_steps(pipe, steps, 1, per_launch=True)
        par = bench.parity_digest(pipe.last_out().cpu().numpy().view(np.uint32))["match"]
    finally:
        W.reserve_cus(0, 0)
    ks = sorted(kern)
    return {"kernel_ms": sum(ks) / len(ks), "kernel_median_ms": ks[len(ks) // 2], "step_ms": el / steps * 1e3,
            "region_ms": region / steps, "parity": par}


def plain(steps, buf):
    st = torch.cuda.Stream()
    out = torch.empty(N, dtype=torch.int32, device="cuda")
    W.reserve_cus(8, 0)
    try:
        f = lambda: W.crc32_batch_fixed(buf, P, P, N, out, st)  # noqa: E731
        bench.settle(f, st, 5)
        torch.cuda.synchronize()
        ev = [(bench.TimingEvent(), bench.TimingEvent()) for _ in range(steps)]
        for a, b in ev:
            a.record(st)
            f()
            b.record(st)
        torch.cuda.synchronize()
        kern = sorted(a.elapsed_time(b) for a, b in ev)
        r0, r1 = bench.TimingEvent(), bench.TimingEvent()
        t0 = time.perf_counter()
        r0.record(st)
        for _ in range(steps):
            f()
        r1.record(st)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    finally:
        W.reserve_cus(0, 0)
    par = bench.parity_digest(out.cpu().numpy().view(np.uint32))["match"]
    return {"kernel_ms": sum(kern) / len(kern), "kernel_median_ms": kern[len(kern) // 2],
            "step_ms": el / steps * 1e3, "region_ms": r0.elapsed_time(r1) / steps, "parity": par}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default="c4_leg_ab.json")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    assert W.LIB.wtp_init(0) == 0
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["RANK"], os.environ["WORLD_SIZE"] = "0", "1"
    buf = torch.empty(N * P + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf, nbytes=N * P)
    variants = {"head": lambda: head(a.steps, True), "head_notime": lambda: head(a.steps, False),
                "r04pipe": lambda: r04pipe(a.steps, buf), "plain": lambda: plain(a.steps, buf),
                "pipe_nogather": lambda: pipe_nogather(a.steps, buf), "head_every4": lambda: head(a.steps, True, 4)}
    names = list(variants)
    runs = []
    for r in range(a.rounds):
        order = names[r % len(names):] + names[:r % len(names)]
        for v in order:
            res = variants[v]()
            res.update({"variant": v, "round": r})
            runs.append(res)
            print(json.dumps(res), flush=True)
    summ = {}
    for v in names:
        rs = [x for x in runs if x["variant"] == v]
        summ[v] = {k: round(float(np.median([x[k] for x in rs])), 5)
                   for k in ("kernel_ms", "kernel_median_ms", "step_ms", "region_ms")}
        summ[v]["kernel_frac"] = round(N * P / (summ[v]["kernel_ms"] * 1e-3) / 8e12, 4)
        summ[v]["parity_all"] = all(x["parity"] for x in rs)
        summ[v]["runs"] = len(rs)
    base = summ["plain"]["kernel_ms"]
    for v in names:
        summ[v]["kernel_vs_plain"] = round(summ[v]["kernel_ms"] / base, 4)
    doc = {"what": __doc__.strip().splitlines()[0], "device": torch.cuda.get_device_name(0), "steps": a.steps,
           "rounds": a.rounds, "summary_medians": summ, "runs": runs}
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({"summary_medians": summ}), flush=True)


if __name__ == "__main__":
    main()
