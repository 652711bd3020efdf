"""config_legs.py — bench.py's `configs` leg: the BASELINE.json configs other than the
headline, measured in the driver's own bench run (N = 1), each row with its timings, its
fraction of the bound that applies, and parity of its WHOLE result against a digest the
reference computed (tests/golden/config_digests.json, tests/golden/make_config_digests.py;
tests/golden/bench_digests.json for the 1 M prefix).

  c2        configs[1]: 64 K x 1456 B device-resident, wtp_crc32_batch_fixed (braided)
  c5        configs[4]: 1 M packed Zipf(s) payloads on [1, 1456], s = 1.1 and 1.0, through
            wtp_crc32_batch_packed (k_pieces) and, for s = 1.1, the forced k_stream route
  verify    the receiver-verify call site (Receiver.cpp:25-35, 203-206): 1 M x 1472-B DATA
            datagrams at stride 1472 and in wReceiver's 1504-B slots, and a ring with three
            short datagrams (the in-kernel fix-up)
  build     the sender-build call site (Packet.cpp:9-14, 36-47): fused DATA builder,
            1 M x 1456 B -> 1472-B datagrams
  c3        configs[2]: 1 GiB host file chunked at 1456 B, wtp_crc32_host_chunked (pinned
            H2D -> CRC -> D2H on the library's streams), pinned and pageable source
  hostbuild wSender --crc gpu: the same 1 GiB -> every DATA datagram in host memory
            (wtp_host_build_data_packets), pinned zero-copy, pinned staged, pageable

Device rows: `b2b_ms` = one timing-event pair around `reps` back-to-back calls / reps;
`graph_ms` = the calls replayed from a captured HIP graph (no host work between kernels);
`frac` = algorithmic HBM bytes / time / 8 TB/s (bytes per row in `bytes_rule`).  Host rows:
wall seconds (best of 3) and their fraction of this box's raw pinned H2D rate (the bound:
the path moves every byte over PCIe once).

No oracle here: inputs come from the device generator (wtp_synth_fill, the same stream the
digests were made from) and zipf_lengths below; parity is sha256 vs the reference digests.
"""
from __future__ import annotations

import hashlib
import json
import os
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 1456
SEED = 0x5EED
PEAK_GBS = 8000.0
GB = 1e9
GIB = float(1 << 30)


def zipf_lengths(n: int, s: float = 1.1, seed: int = SEED, max_len: int = P) -> np.ndarray:
    """Zipf(s) on [1, max_len] by inverse CDF over splitmix64 uniforms.
    The same function as oracle.zipf_lengths (test_bench.py checks they agree), restated
    here so the bench leg needs no oracle import."""
    k = np.arange(1, max_len + 1, dtype=np.float64)
    cdf = np.cumsum(k ** (-s))
    cdf /= cdf[-1]
    w = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed ^ 0x21F) + (w + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    return np.minimum(np.searchsorted(cdf, u, side="right") + 1, max_len).astype(np.uint32)


def digests() -> dict:
    d = {}
    for name, key in (("config_digests.json", "sha256"), ("bench_digests.json", "sha256_by_packets")):
        try:
            with open(os.path.join(ROOT, "tests", "golden", name)) as f:
                d.update(json.load(f)[key])
        except OSError:
            pass
    return d


def sha_u32(t) -> str:
    a = t.cpu().numpy() if hasattr(t, "cpu") else t
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint32).astype("<u4").tobytes()).hexdigest()


def parity(got: str, key: str, D: dict) -> dict:
    want = D.get(key)
    return {"match": None if want is None else got == want, "sha256": got[:16], "digest": key,
            "vs": "reference crc32 (oracle/_ref) over the same inputs" if want else "no digest"}


class Timer:
    """Back-to-back and graph-replay per-call times of fn on the current stream."""

    def __init__(self, TimingEvent):
        self.TE = TimingEvent

    def b2b(self, fn, reps: int, warm: int = 3) -> float:
        st = torch.cuda.current_stream()
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        a, b = self.TE(), self.TE()
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    def singles(self, fn, reps: int = 20) -> float:
        """Median of single calls from an idle stream (an event pair around each)."""
        st = torch.cuda.current_stream()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            a, b = self.TE(), self.TE()
            a.record(st)
            fn()
            b.record(st)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts))

    def graph(self, fn, G: int = 50, reps: int = 5, per: int = 10) -> float:
        """Per-call ms of fn replayed from a graph of G captured calls: median over `reps`
        timings of `per` consecutive replays."""
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            fn()  # library state keyed by stream is made outside the capture
        cs.synchronize()
        with torch.cuda.graph(g, stream=cs):
            for _ in range(G):
                fn()
        g.replay()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        ts = []
        for _ in range(reps):
            a, b = self.TE(), self.TE()
            a.record(st)
            for _ in range(per):
                g.replay()
            b.record(st)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / (per * G))
        del g
        return float(np.median(ts))


def _dev_row(name, by, rule, b2b, gr, extra=None) -> dict:
    r = {"config": name, "bytes": by, "bytes_rule": rule,
         "b2b_ms": round(b2b, 5), "b2b_frac": round(by / (b2b * 1e-3) / GB / PEAK_GBS, 4),
         "graph_ms": round(gr, 5), "graph_frac": round(by / (gr * 1e-3) / GB / PEAK_GBS, 4),
         "graph_GBs": round(by / (gr * 1e-3) / GB, 1)}
    if extra:
        r.update(extra)
    return r


def c2(W, T, D) -> dict:
    n = 65536
    buf = torch.empty(n * P, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    f = lambda: W.crc32_batch_fixed(buf, P, P, n, out)  # noqa: E731
    single = T.singles(f)
    b2b = T.b2b(f, 500)
    gr = T.graph(f)
    out.zero_()
    f()
    r = _dev_row("C2: 64 K x 1456 B device-resident, wtp_crc32_batch_fixed", n * P, "payload bytes read",
                 b2b, gr, {"packets": n, "kernel": W.LIB.wtp_last_kernel().decode(),
                           "single_launch_ms": round(single, 5),
                           "single_launch_frac": round(n * P / (single * 1e-3) / GB / PEAK_GBS, 4)})
    r["parity"] = parity(sha_u32(out), "c2", D)
    return r


def c5(W, T, D, s: float, stream_kernel: bool = False) -> dict:
    n = 1 << 20
    lens = zipf_lengths(n, s=s)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(d, nbytes=total)
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    if stream_kernel:
        os.environ["WTP_STREAM_KERNEL"] = "1"
    try:
        f = lambda: W.crc32_batch_packed(d, total, do, dl, n, out)  # noqa: E731
        b2b = T.b2b(f, 100)
        gr = T.graph(f)
        out.zero_()
        f()
        kern = W.LIB.wtp_last_kernel().decode()
    finally:
        os.environ.pop("WTP_STREAM_KERNEL", None)
    rb = total + 12 * n
    r = _dev_row(f"C5: 1 M packed payloads, Zipf(s={s}) lengths on [1,1456], wtp_crc32_batch_packed"
                 + (" forced to k_stream (WTP_STREAM_KERNEL=1)" if stream_kernel else ""),
                 rb, "payload bytes + 12 B metadata (u64 offset, u32 length) per packet", b2b, gr,
                 {"packets": n, "payload_bytes": total, "mean_len": round(total / n, 1), "kernel": kern})
    r["parity"] = parity(sha_u32(out), f"c5_zipf{s}", D)
    return r


def verify_and_build(W, T, D) -> list:
    n, stride = 1 << 20, 16 + P
    payload = torch.empty(n * P, dtype=torch.uint8, device="cuda")
    W.synth_fill(payload)
    wire = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    wl = torch.empty(n, dtype=torch.int32, device="cuda")
    fb = lambda: W.build_data_packets(payload, n * P, 0, wire, stride, wl)  # noqa: E731
    bb = T.b2b(fb, 50)
    bg = T.graph(fb, G=20)
    wire.zero_()
    fb()
    bk = W.LIB.wtp_last_kernel().decode()
    h = hashlib.sha256(wire.cpu().numpy().tobytes()).hexdigest()
    rows = [_dev_row("build: fused DATA builder, 1 M x 1456 B -> 1472-B datagrams (seq 0..)", n * (P + stride + 4),
                     "payload read + datagram write + u32 length write per packet", bb, bg,
                     {"packets": n, "kernel": bk, "parity": parity(h, "build_1m", D)})]
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    crc = torch.empty(n, dtype=torch.int32, device="cuda")

    def vrow(name, buf, st, lens, key, want_ok):
        f = lambda: W.verify_batch(buf, st, lens, n, ok)  # noqa: E731
        b2b = T.b2b(f, 100)
        gr = T.graph(f)
        ok.zero_()
        crc.zero_()
        W.verify_batch(buf, st, lens, n, ok, crc)
        kern = W.LIB.wtp_last_kernel().decode()
        par = parity(sha_u32(crc), key, D)
        okh = ok.cpu().numpy()
        par["ok_pattern"] = bool(np.array_equal(okh, want_ok))
        if par["match"] is not None:
            par["match"] = par["match"] and par["ok_pattern"]
        return _dev_row(name, n * (stride + 4) + n, "datagram read + u32 recv_len read + u8 ok write per datagram",
                        b2b, gr, {"packets": n, "stride": st, "kernel": kern, "parity": par})

    ones = np.ones(n, np.uint8)
    rows.append(vrow("verify: receiver verify, 1 M x 1472-B DATA datagrams, stride 1472", wire, stride, wl, "1048576",
                     ones))
    w2 = torch.zeros(n * 1504, dtype=torch.uint8, device="cuda")
    w2.view(n, 1504)[:, :stride].copy_(wire.view(n, stride))
    rl2 = torch.full((n,), stride, dtype=torch.int32, device="cuda")
    rows.append(vrow("verify: the same datagrams in wReceiver's 1504-B ring slots", w2, 1504, rl2, "1048576", ones))
    del w2, rl2
    wl3 = wl.clone()
    wl3[0], wl3[n // 2], wl3[n - 1] = 16, 16, 1016
    want = ones.copy()
    want[[0, n // 2, n - 1]] = 0
    rows.append(vrow("verify: stride-1472 ring with 3 short datagrams (16, 16, 1016 B: in-kernel fix-up)", wire,
                     stride, wl3, "verify_fixup_1m", want))
    return rows


def _h2d_rate(host: np.ndarray) -> float:
    d = torch.empty(host.nbytes, dtype=torch.uint8, device="cuda")
    ht = torch.from_numpy(host)
    best = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(ht, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, host.nbytes / (time.perf_counter() - t0) / GB)
    del d
    return best


def host_rows(W, D) -> list:
    """C3 and the host builder over one 1 GiB pinned file buffer (filled from the device
    generator: the bytes make_config_digests.py hashes)."""
    nb = 1 << 30
    pb = W.PinnedBuffer(nb)
    try:
        d = torch.empty(nb, dtype=torch.uint8, device="cuda")
        W.synth_fill(d)
        torch.from_numpy(pb.array).copy_(d)
        del d
        h2d = _h2d_rate(pb.array)
        rows = []

        def best(fn, k=3):
            fn()  # warm (library pipeline buffers)
            ts = []
            for _ in range(k):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            return min(ts)

        pageable = np.empty(nb, np.uint8)
        pageable[:] = pb.array
        c3 = {"config": "C3: 1 GiB host file chunked at 1456 B -> wtp_crc32_host_chunked (pinned H2D -> CRC -> D2H)",
              "bytes": nb, "chunks": (nb + P - 1) // P, "raw_h2d_pinned_GBs": round(h2d, 2),
              "bound": "PCIe H2D (every byte crosses once): frac = rate / this box's raw pinned H2D rate"}
        for label, src in (("pinned", pb.array), ("pageable", pageable)):
            res = {}
            t = best(lambda: res.__setitem__("c", W.host_chunked(src, P)))
            c3[label] = {"seconds": round(t, 4), "GiBs": round(nb / t / GIB, 2), "GBs": round(nb / t / GB, 2),
                         "frac_of_raw_h2d": round(nb / t / GB / h2d, 4),
                         "parity": parity(hashlib.sha256(res["c"].astype("<u4").tobytes()).hexdigest(), "c3_1gib", D)}
        rows.append(c3)
        n = (nb + P - 1) // P
        pw = W.PinnedBuffer(n * (16 + P))
        try:
            hb = {"config": "hostbuild: 1 GiB host file -> every 1472-B DATA datagram in host memory "
                            "(wtp_host_build_data_packets)", "bytes": nb, "datagrams": n,
                  "raw_h2d_pinned_GBs": round(h2d, 2),
                  "bound": "PCIe: payload H2D + datagram D2H; frac = payload rate / raw pinned H2D rate"}
            for label in ("pinned", "pinned_staged", "pageable"):
                os.environ["WTP_HOST_BUILD_ZEROCOPY"] = "0" if label == "pinned_staged" else "1"
                src, wire = (pb.array, pw.array) if label != "pageable" else (pageable, np.empty(n * (16 + P), np.uint8))
                t = best(lambda: W.host_build_data_packets(src, 0, 16 + P, wire=wire))
                h = hashlib.sha256(wire[:(n - 1) * (16 + P)].tobytes())
                h.update(wire[(n - 1) * (16 + P):(n - 1) * (16 + P) + 16 + nb - (n - 1) * P].tobytes())
                hb[label] = {"seconds": round(t, 4), "payload_GBs": round(nb / t / GB, 2),
                             "moved_GBs": round((nb + n * (16 + P)) / t / GB, 2),
                             "frac_of_raw_h2d": round(nb / t / GB / h2d, 4),
                             "parity": parity(h.hexdigest(), "hostbuild_1gib", D)}
                del wire
            rows.append(hb)
        finally:
            os.environ.pop("WTP_HOST_BUILD_ZEROCOPY", None)
            pw.free()
        del pageable
        return rows
    finally:
        pb.free()


def run(W, TimingEvent, only: str | None = None) -> dict:
    """Every row; a row that raises is reported as an error, not fatal.  Returns
    {"rows": [...], "parity_all": bool or None, "seconds": wall}."""
    T = Timer(TimingEvent)
    D = digests()
    t0 = time.perf_counter()
    rows = []
    legs = [("c2", lambda: [c2(W, T, D)]),
            ("c5", lambda: [c5(W, T, D, 1.1), c5(W, T, D, 1.0), c5(W, T, D, 1.1, stream_kernel=True)]),
            ("verify", lambda: verify_and_build(W, T, D)),
            ("host", lambda: host_rows(W, D))]
    for name, fn in legs:
        if only and name not in only.split(","):
            continue
        try:
            rows.extend(fn())
        except (RuntimeError, OSError, AssertionError) as e:  # WtpError is a RuntimeError
            rows.append({"config": name, "error": f"{e.__class__.__name__}: {e}"[:300]})
        torch.cuda.empty_cache()
    pars = []
    for r in rows:
        for v in [r] + [r[k] for k in ("pinned", "pinned_staged", "pageable") if k in r]:
            if "parity" in v:
                pars.append(v["parity"]["match"])
    ok = None if not pars or any(p is None for p in pars) else all(pars)
    if any("error" in r for r in rows):
        ok = False if ok is False else None
    return {"rows": rows, "parity_all": ok, "parity_checks": len(pars), "seconds": round(time.perf_counter() - t0, 1),
            "rule": "device rows: b2b_ms = event pair around back-to-back calls / reps, graph_ms = replay of a "
                    "captured graph / calls; frac = bytes / time / 8 TB/s; host rows: best of 3 wall; parity = "
                    "sha256 of the whole result vs tests/golden/{config,bench}_digests.json (reference crc32)"}
