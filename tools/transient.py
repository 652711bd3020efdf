#!/usr/bin/env python3
"""Per-launch timeline of the headline kernel from a cold start (diagnostics).

Reproduces bench.py's start (on-device synth fill of 1 M x 1456 B, then back-to-back
CRC launches) and records every launch's HIP-event time, so the warmup transient the
driver's `--warmup 5 --steps 20` window falls into can be characterised.  Then times
the same-box HBM read ceiling (lib/libwtp_diag.so) interleaved with the CRC kernel,
and samples the shader clock between launches.

    python tools/transient.py [--launches 3000] [--out gpurun_out/transient.json]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=3000)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="idle before the run (cold start)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch
    import wtp_crc32 as W

    torch.cuda.set_device(0)
    D = C.CDLL(os.path.join(ROOT, "a3-reliable-transport_amd", "lib", "libwtp_diag.so"))
    D.wtp_diag_read_xor.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint, C.c_uint, C.c_void_p]
    D.wtp_diag_clock.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    n = 1 << 20
    nb = n * 1456
    buf = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    clk = torch.zeros(3, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    W.synth_fill(buf, nbytes=nb)

    def clock_mhz():
        D.wtp_diag_clock(clk.data_ptr(), 20000, st.cuda_stream)
        c = clk.cpu().numpy()
        return float(c[0]) / float(c[1]) * 100.0 if c[1] else 0.0

    if a.idle_ms:
        time.sleep(a.idle_ms / 1e3)
    res = {}
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.launches)]
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(st)
        W.crc32_batch_fixed(buf, 1456, 1456, n, out, st)
        e.record(st)
    torch.cuda.synchronize()
    t = np.array([s.elapsed_time(e) for s, e in ev]) * 1e3  # us
    res["launch_us"] = [round(float(x), 2) for x in t]
    win = {}
    for lo, hi in ((0, 5), (5, 25), (25, 50), (50, 100), (100, 200), (200, 400), (400, 800), (800, 1600),
                   (1600, 3000)):
        if hi <= t.size:
            win[f"{lo}-{hi}"] = round(float(np.median(t[lo:hi])), 2)
    res["median_us_by_window"] = win
    print("CRC median us by launch window:", win, flush=True)
    res["clock_after_MHz"] = round(clock_mhz(), 1)

    # same-box read ceiling, interleaved with the CRC kernel, several grid shapes
    shapes = [(256, 512), (1024, 512), (2048, 256), (4096, 256)]
    pe = {sh: [] for sh in shapes}
    ce = []
    for rep in range(20):
        for sh in shapes:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(st)
            assert D.wtp_diag_read_xor(buf.data_ptr(), nb, sink.data_ptr(), sh[0], sh[1], st.cuda_stream) == 0
            e.record(st)
            pe[sh].append((s, e))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        W.crc32_batch_fixed(buf, 1456, 1456, n, out, st)
        e.record(st)
        ce.append((s, e))
    torch.cuda.synchronize()
    probe = {}
    for sh, lst in pe.items():
        m = float(np.median([s.elapsed_time(e) for s, e in lst]))
        probe[f"{sh[0]}x{sh[1]}"] = {"median_us": round(m * 1e3, 2), "GBs": round(nb / (m * 1e-3) / 1e9, 1)}
    cm = float(np.median([s.elapsed_time(e) for s, e in ce]))
    res["read_probe"] = probe
    res["crc_interleaved"] = {"median_us": round(cm * 1e3, 2), "GBs": round(nb / (cm * 1e-3) / 1e9, 1)}
    print("read probe:", probe, flush=True)
    print("crc interleaved:", res["crc_interleaved"], flush=True)
    res["clock_end_MHz"] = round(clock_mhz(), 1)
    # idle 1 s, then a short burst: how fast does it fall back into the transient?
    time.sleep(1.0)
    ev2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(60)]
    for s, e in ev2:
        s.record(st)
        W.crc32_batch_fixed(buf, 1456, 1456, n, out, st)
        e.record(st)
    torch.cuda.synchronize()
    res["after_idle_1s_us"] = [round(s.elapsed_time(e) * 1e3, 1) for s, e in ev2]
    print("after 1 s idle:", res["after_idle_1s_us"][:30], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
