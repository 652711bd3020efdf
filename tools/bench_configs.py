#!/usr/bin/env python3
"""Measure the non-headline configs of BASELINE.json on one MI355X (writes JSON).

  C2  64K x 1456 B device-resident: single-launch time (launch-bound), sustained rate
      from Python, and the same launches replayed from a captured HIP graph
  C3  1 GiB host file chunked at 1456 B: wtp_crc32_host_chunked end to end, pinned and
      pageable source (PCIe-bound), plus torch's raw H2D copy rate for reference
  C5  1 M mixed-length payloads, Zipf(s) on [1,1456] (s = 1.1, 1.0), packed, per-packet
      offsets/lengths: the general kernel; read bytes = sum(len) + 12 B metadata/packet
  verify   1 M wire datagrams (stride 1472, and in wReceiver's 1504-B slots) through the
           receiver-verify kernel
  build    fused DATA packet builder over a 1.4 GiB payload buffer
Every line carries a spot parity check against the CPU oracle.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "a3-reliable-transport_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import wtp_crc32 as W  # noqa: E402

sys.path.insert(0, ROOT)
from bench import TimingEvent  # noqa: E402

GB = 1e9
GIB = float(1 << 30)
PEAK = 8000.0


def timed(fn, reps, warm=3):
    """(median per-call ms with an event between calls, mean ms per call back to back).
    Events are timing-only (hipEventDisableSystemFence, bench.TimingEvent): a default
    event's system-scope cache flush pads every interval and slows the next launch.  The
    back-to-back figure has no event between the calls at all: one pair around `reps`."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ev = [TimingEvent() for _ in range(reps + 1)]
    ev[0].record(st)
    for i in range(reps):
        fn()
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))
    a, b = TimingEvent(), TimingEvent()
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return ts[len(ts) // 2], a.elapsed_time(b) / reps


def graph_time(fn, G=50, reps=7, per=10):
    """Per-launch ms of fn replayed from a captured HIP graph of G launches (no host work
    between kernels): median over `reps` timings of `per` consecutive replays (timing each
    replay on its own adds the graph-launch gap, ~1.7 us per launch at G = 50)."""
    graph = torch.cuda.CUDAGraph()
    # capture on a stream that ran fn once first: library state keyed by stream (the
    # verify fix-up list) exists before the capture, which never allocates
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        fn()
    cs.synchronize()
    with torch.cuda.graph(graph, stream=cs):
        for _ in range(G):
            fn()
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(per):
            graph.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / (per * G))
    return float(np.median(ts)), graph


def c2():
    n = 65536
    buf = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    f = lambda: W.crc32_batch_fixed(buf, 1456, 1456, n, out)  # noqa: E731
    # single launch from an idle stream
    singles = []
    for _ in range(20):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        singles.append(a.elapsed_time(b))
    med, mean = timed(f, 500)
    # the same launches replayed from a HIP graph (captured through torch): no per-launch
    # host work, so back-to-back kernels are limited by the GPU alone
    gl, graph = graph_time(f)
    out.zero_()
    graph.replay()
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    ok = all(int(got[i]) == O.crc32(O.synth_fill_np(1456, start_byte=i * 1456)) for i in (0, n // 3, n - 1))
    by = n * 1456
    return {"config": "C2 64K x 1456 B device-resident", "packets": n, "bytes": by,
            "single_launch_ms_median": round(float(np.median(singles)), 4),
            "single_launch_GiBps": round(by / (np.median(singles) * 1e-3) / GIB, 1),
            "sustained_ms_per_launch": round(mean, 4), "sustained_GiBps": round(by / (mean * 1e-3) / GIB, 1),
            "sustained_frac_hbm": round(by / (mean * 1e-3) / GB / PEAK, 4),
            "graph_ms_per_launch": round(gl, 4), "graph_GiBps": round(by / (gl * 1e-3) / GIB, 1),
            "graph_frac_hbm": round(by / (gl * 1e-3) / GB / PEAK, 4), "parity_spot": ok}


def c3():
    nbytes = 1 << 30
    res = {"config": "C3 1 GiB host file -> 1456-B chunks, pinned H2D -> CRC -> D2H, 2 streams", "bytes": nbytes,
           "chunks": (nbytes + 1455) // 1456}
    pb = W.PinnedBuffer(nbytes)
    host = pb.array
    # fill with the synthetic stream in 64 MiB pieces
    step = 64 << 20
    for o in range(0, nbytes, step):
        host[o:o + step] = O.synth_fill_np(min(step, nbytes - o), start_byte=o)
    for label, src in (("pinned", host), ("pageable", None)):
        if src is None:
            src = np.empty(nbytes, dtype=np.uint8)
            src[:] = host
        W.host_chunked(src, 1456)  # warm (allocates the library pipeline)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            crcs = W.host_chunked(src, 1456)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        n = crcs.size
        ok = all(int(crcs[i]) == O.crc32(host[i * 1456:min((i + 1) * 1456, nbytes)]) for i in (0, n // 2, n - 1))
        res[label] = {"seconds": round(t, 4), "GiBps": round(nbytes / t / GIB, 2), "GBps": round(nbytes / t / GB, 2),
                      "parity_spot": ok, "last_chunk_bytes": int(nbytes - (n - 1) * 1456)}
        del src
    # raw H2D rate of the link for context
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    ht = torch.from_numpy(host)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.copy_(ht, non_blocking=True)
    torch.cuda.synchronize()
    res["raw_h2d_pinned_GBps"] = round(nbytes / (time.perf_counter() - t0) / GB, 2)
    pb.free()
    return res


def hostbuild():
    """wSender --crc gpu: a 1 GiB host file -> every DATA datagram (header + CRC + payload)
    in a host wire buffer through wtp_host_build_data_packets (H2D -> fused builder -> D2H)."""
    nbytes = 1 << 30
    n = (nbytes + 1455) // 1456
    res = {"config": "host builder: 1 GiB host file -> 1472-B DATA datagrams in host memory", "bytes": nbytes,
           "datagrams": n}
    pb = W.PinnedBuffer(nbytes)
    host = pb.array
    step = 64 << 20
    for o in range(0, nbytes, step):
        host[o:o + step] = O.synth_fill_np(min(step, nbytes - o), start_byte=o)
    pw = W.PinnedBuffer(n * 1472)
    for label in ("pinned", "pinned_staged", "pageable"):
        # pinned: the builder reads/writes host memory across the link (zero copy);
        # pinned_staged: the same buffers through the device slabs (WTP_HOST_BUILD_ZEROCOPY=0)
        os.environ["WTP_HOST_BUILD_ZEROCOPY"] = "0" if label == "pinned_staged" else "1"
        src, wire = (host, pw.array) if label != "pageable" else (np.array(host), np.empty(n * 1472, np.uint8))
        W.host_build_data_packets(src, 0, 1472, wire=wire)  # warm (allocates the wire slabs)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            W.host_build_data_packets(src, 0, 1472, wire=wire)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        ok = all(wire[i * 1472:i * 1472 + 16 + min(1456, nbytes - i * 1456)].tobytes() ==
                 O.build_datagram(i, host[i * 1456:(i + 1) * 1456].tobytes()) for i in (0, n // 2, n - 1))
        res[label] = {"seconds": round(t, 4), "payload_GBps": round(nbytes / t / GB, 2),
                      "moved_GBps": round((nbytes + n * 1472) / t / GB, 2), "parity_spot": ok}
        del src, wire
    del os.environ["WTP_HOST_BUILD_ZEROCOPY"]
    pw.free()
    pb.free()
    return res


def c5(s, entry="var"):
    """entry "var": wtp_crc32_batch_var (k_pieces, any offsets); "packed":
    wtp_crc32_batch_packed (the C5 layout, payloads back to back: the same k_pieces route
    below 2 GiB); "stream": wtp_crc32_batch_packed with WTP_STREAM_KERNEL=1 (k_stream)."""
    n = 1 << 20
    lens = O.zipf_lengths(n, s=s)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(d, nbytes=total)
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    if entry == "stream":  # the stream kernel, forced (wtp_crc32_batch_packed picks k_pieces below 2 GiB)
        os.environ["WTP_STREAM_KERNEL"] = "1"
    fn = W.crc32_batch_packed if entry in ("packed", "stream") else W.crc32_batch_var
    f = lambda: fn(d, total, do, dl, n, out)  # noqa: E731
    med, mean = timed(f, 200)
    gl, _ = graph_time(f)
    got = out.cpu().numpy().view(np.uint32)
    host = d[:total].cpu().numpy()
    ok = bool(np.array_equal(got, O.batch_var(host, offs, lens)))
    rb = total + 12 * n
    os.environ.pop("WTP_STREAM_KERNEL", None)
    kern = {"stream": "k_stream (wtp_crc32_batch_packed, WTP_STREAM_KERNEL=1)",
            "packed": "wtp_crc32_batch_packed (k_pieces below 2 GiB)"}.get(entry, "k_pieces (wtp_crc32_batch_var)")
    return {"config": f"C5 1M mixed lengths Zipf(s={s}) on [1,1456], {kern}", "packets": n,
            "payload_bytes": total, "mean_len": round(total / n, 1), "read_bytes_incl_meta": rb,
            "ms_per_launch": round(mean, 4), "payload_GiBps": round(total / (mean * 1e-3) / GIB, 1),
            "read_GBps": round(rb / (mean * 1e-3) / GB, 1), "frac_hbm": round(rb / (mean * 1e-3) / GB / PEAK, 4),
            "graph_ms_per_launch": round(gl, 4), "graph_frac_hbm": round(rb / (gl * 1e-3) / GB / PEAK, 4),
            "parity_all": ok}


def c5big(s=1.1, n=17_000_000):
    """C5's distribution in a packed buffer past 2 GiB (17 M payloads, ~2.3 GB): the piece
    kernel in device-cut < 2 GiB sub-launches (wtp_crc32_batch_packed, and
    wtp_crc32_batch_var, which takes the same route there) against k_stream (forced, the
    route of both before round 5).  The routes' vectors must be equal; a sample of 4000
    payloads is checked against the oracle."""
    lens = O.zipf_lengths(n, s=s)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(d, nbytes=total)
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    rb = total + 12 * n
    rows, vecs = [], {}
    for entry in ("packed", "var", "stream"):
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        if entry == "stream":  # the stream kernel, forced (the route both entries took before round 5)
            os.environ["WTP_STREAM_KERNEL"] = "1"
        fn = W.crc32_batch_var if entry == "var" else W.crc32_batch_packed
        f = lambda: fn(d, total, do, dl, n, out)  # noqa: E731
        med, mean = timed(f, 20)
        try:  # the packed route allocates its descriptors from a stream-ordered pool
            gl, _ = graph_time(f, G=5, reps=5, per=4)
        except Exception as e:  # noqa: BLE001 — reported, not fatal
            gl, gerr = float("nan"), f"{e.__class__.__name__}: {e}"[:200]
        else:
            gerr = None
        kern = W.LIB.wtp_last_kernel().decode()
        os.environ.pop("WTP_STREAM_KERNEL", None)
        vecs[entry] = out.cpu().numpy().view(np.uint32).copy()
        rows.append({"config": f"C5 distribution past 2 GiB: {n} packed payloads Zipf(s={s}), "
                               f"wtp_crc32_batch_{entry} -> {kern}", "packets": n, "payload_bytes": total,
                     "read_bytes_incl_meta": rb, "ms_per_launch": round(mean, 4),
                     "read_GBps": round(rb / (mean * 1e-3) / GB, 1), "frac_hbm": round(rb / (mean * 1e-3) / GB / PEAK, 4),
                     "graph_ms_per_launch": round(gl, 4), "graph_frac_hbm": round(rb / (gl * 1e-3) / GB / PEAK, 4),
                     "graph_error": gerr})
    idx = np.random.default_rng(5).integers(0, n, 4000)
    host = d.cpu().numpy()
    del d
    ok = bool(np.array_equal(vecs["packed"], vecs["var"])) and bool(np.array_equal(vecs["packed"], vecs["stream"])) and bool(
        np.array_equal(vecs["packed"][idx], O.batch_var(host, offs[idx], lens[idx])))
    for r in rows:
        r["parity_routes_equal_and_sample"] = ok
    return rows


def verify():
    n, stride = 1 << 20, 1472
    wire = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    payload = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(payload)
    wl = torch.empty(n, dtype=torch.int32, device="cuda")
    W.build_data_packets(payload, n * 1456, 0, wire, stride, wl)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    f = lambda: W.verify_batch(wire, stride, wl, n, ok)  # noqa: E731
    med, mean = timed(f, 100)
    gv, _ = graph_time(f)
    good = int(ok.sum().item())
    fb = lambda: W.build_data_packets(payload, n * 1456, 0, wire, stride, wl)  # noqa: E731
    bmed, bmean = timed(fb, 50)
    # copy ceiling for the same traffic shape: a device-to-device copy of the payloads
    # into the wire buffer (torch / HIP runtime copy kernel)
    wv = wire[:n * 1456]
    fc = lambda: wv.copy_(payload)  # noqa: E731
    cmed, cmean = timed(fc, 50)
    W.build_data_packets(payload, n * 1456, 0, wire, stride, wl)
    h = wire[:2 * stride].cpu().numpy().tobytes()
    want = O.build_datagram(0, O.synth_fill_np(1456).tobytes()) + b"\0" * 0
    # wReceiver's ring: the same 1472-B datagrams in 1504-B slots (1500-B receive buffer)
    del wl
    w2 = torch.zeros(n * 1504, dtype=torch.uint8, device="cuda")
    w2.view(n, 1504)[:, :stride].copy_(wire.view(n, stride))
    rl2 = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    f2 = lambda: W.verify_batch(w2, 1504, rl2, n, ok)  # noqa: E731
    med2, mean2 = timed(f2, 100)
    gv2, _ = graph_time(f2)
    good2 = int(ok.sum().item())
    del w2, rl2
    # the same 1472-B ring with three short datagrams (START/END-like 16-B ones and a
    # short last chunk): their workgroups run the in-kernel fix-up phase
    wl = torch.empty(n, dtype=torch.int32, device="cuda")
    W.build_data_packets(payload, n * 1456, 0, wire, stride, wl)
    wl3 = wl.clone()
    wl3[0], wl3[n // 2], wl3[n - 1] = 16, 16, 1016
    f3 = lambda: W.verify_batch(wire, stride, wl3, n, ok)  # noqa: E731
    med3, mean3 = timed(f3, 100)
    gv3, _ = graph_time(f3)
    torch.cuda.synchronize()
    okh = ok.cpu().numpy()
    want3 = okh.sum() == n - 3 and okh[0] == 0 and okh[n - 1] == 0  # short datagrams fail their checksum
    del wl3
    return [{"config": "receiver verify, 1M x 1472-B datagrams device-resident", "packets": n,
             "ms_per_launch": round(mean, 4), "per_call_ms_median_with_events": round(med, 4),
             "payload_GiBps": round(n * 1456 / (mean * 1e-3) / GIB, 1),
             "read_GBps": round(n * (stride + 4) / (mean * 1e-3) / GB, 1), "graph_ms_per_launch": round(gv, 4),
             "graph_frac_hbm": round(n * (stride + 4) / (gv * 1e-3) / GB / PEAK, 4), "all_ok": good == n},
            {"config": "receiver verify, 1M x 1472-B datagrams in 1504-B slots (wReceiver ring)", "packets": n,
             "ms_per_launch": round(mean2, 4), "per_call_ms_median_with_events": round(med2, 4),
             "payload_GiBps": round(n * 1456 / (mean2 * 1e-3) / GIB, 1),
             "read_GBps": round(n * (stride + 4) / (mean2 * 1e-3) / GB, 1), "graph_ms_per_launch": round(gv2, 4),
             "graph_frac_hbm": round(n * (stride + 4) / (gv2 * 1e-3) / GB / PEAK, 4), "all_ok": good2 == n},
            {"config": "receiver verify, 1M x 1472-B ring with 3 short datagrams (in-kernel fix-up)", "packets": n,
             "ms_per_launch": round(mean3, 4), "per_call_ms_median_with_events": round(med3, 4),
             "graph_ms_per_launch": round(gv3, 4), "graph_frac_hbm": round(n * (stride + 4) / (gv3 * 1e-3) / GB / PEAK, 4),
             "ok_pattern_as_expected": bool(want3)},
            {"config": "fused DATA packet builder, 1M x 1456 B -> 1472-B wire slots", "packets": n,
             "ms_per_launch": round(bmean, 4), "GBps_read_plus_write": round(n * (1456 + 1472) / (bmean * 1e-3) / GB, 1),
             "d2d_copy_same_bytes_GBps_read_plus_write": round(2 * n * 1456 / (cmean * 1e-3) / GB, 1),
             "first_datagram_matches_oracle": h[:1472] == want}]


def hostverify():
    """Receiver side end to end (north_star: the path ends in host memory): wReceiver's
    ring of 1504-B slots in pinned memory (wtp_host_alloc, as its recvmmsg ring) with a
    pinned recv_len array -> wtp_crc32_host_verify (H2D of the ring + lengths, the braided
    verify, D2H of ok + crc) at window-size batches and a 1 GiB ring; and the same from a
    pageable numpy ring (staged through the library's pinned slabs).  All datagrams are
    full 1472-B WTP DATA datagrams except the last of each batch (short)."""
    stride = 1504
    out = {"config": "receiver end to end: host ring of 1504-B slots -> wtp_crc32_host_verify -> host ok/crc",
           "stride": stride, "rows": []}
    nmax = (1 << 30) // stride
    ring = W.PinnedBuffer(nmax * stride)
    lens = W.PinnedBuffer(nmax * 4)
    la = lens.array.view(np.uint32)
    # build nmax datagrams on the device, copy into the pinned ring
    payload = torch.empty(nmax * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(payload, start_byte=7)
    wire = torch.zeros(nmax * stride, dtype=torch.uint8, device="cuda")
    wl = torch.empty(nmax, dtype=torch.int32, device="cuda")
    W.build_data_packets(payload, nmax * 1456, 0, wire, stride, wl)
    ring.array[:] = wire.cpu().numpy()
    la[:] = wl.cpu().numpy().view(np.uint32)
    del payload, wire, wl
    torch.cuda.empty_cache()
    okb = np.zeros(nmax, np.uint8)
    crcb = np.zeros(nmax, np.uint32)
    import ctypes as C

    def call(buf_ptr, lens_ptr, n):
        rc = W.LIB.wtp_crc32_host_verify(buf_ptr, stride, lens_ptr, n, okb.ctypes.data, crcb.ctypes.data)
        assert rc == 0, W.LIB.wtp_last_error()

    pageable = np.empty(nmax * stride, np.uint8)
    pageable[:] = ring.array
    plens = la.copy()
    for n in (10, 64, 1024, 2560, 16384, nmax):
        for kind, bp, lp in (("pinned", ring.ptr, lens.ptr), ("pageable", pageable.ctypes.data, plens.ctypes.data)):
            # last datagram of the batch short: the fix-up phase runs, as with a file's tail
            save_p, save_l = la[n - 1], plens[n - 1]
            la[n - 1] = plens[n - 1] = 16 + 100
            reps = 5 if n == nmax else (200 if n <= 1024 else 50)
            call(bp, lp, n)
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                call(bp, lp, n)
                ts.append(time.perf_counter() - t0)
            t = float(np.median(ts))
            good = int(okb[:n].sum())
            la[n - 1], plens[n - 1] = save_p, save_l
            by = n * stride
            out["rows"].append({"n": n, "source": kind, "ring_bytes": by, "median_ms": round(t * 1e3, 4),
                                "ring_GBps": round(by / t / GB, 2), "payload_GiBps": round(n * 1456 / t / GIB, 2),
                                "datagrams_per_s": round(n / t), "ok_all_but_last": bool(good == n - 1 and okb[n - 1] == 0)})
            print(json.dumps(out["rows"][-1]), flush=True)
    # the link itself: pinned H2D of the 1 GiB ring
    d = torch.empty(nmax * stride, dtype=torch.uint8, device="cuda")
    ht = torch.from_numpy(ring.array)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.copy_(ht, non_blocking=True)
    torch.cuda.synchronize()
    out["raw_h2d_pinned_GBps"] = round(nmax * stride / (time.perf_counter() - t0) / GB, 2)
    ring.free()
    lens.free()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="configs.json")
    ap.add_argument("--only", default="c2,c3,c5,verify,hostverify,hostbuild")
    a = ap.parse_args()
    assert W.LIB.wtp_init(0) == 0
    res = {"device": torch.cuda.get_device_name(0), "host_cpus": os.cpu_count(), "results": []}
    sel = a.only.split(",")
    def add(*rs):
        for r in rs:
            res["results"].append(r)
            print(json.dumps(r), flush=True)
            with open(a.out, "w") as f:  # after every result: a later failure keeps the earlier ones
                json.dump(res, f, indent=1)

    if "c2" in sel:
        add(c2())
    if "c5" in sel:
        for entry in ("stream", "var", "packed"):
            add(c5(1.1, entry), c5(1.0, entry))
    if "c5big" in sel:
        add(*c5big())
    if "verify" in sel:
        add(*verify())
    if "c3" in sel:
        add(c3())
    if "hostverify" in sel:
        add(hostverify())
    if "hostbuild" in sel:
        add(hostbuild())


if __name__ == "__main__":
    main()
