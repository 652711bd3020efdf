"""GPU parity: every HIP entry point vs the CPU oracle, bit-exact, through the C-ABI.

Everything is compared element-wise with the oracle, including the full 1 M x 1456
headline batch and the 1 GiB C3 host file (the oracle runs multi-threaded over the
bytes the device holds; those bytes are checked against the generator in windows).
"""
import hashlib
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def W():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import wtp_crc32 as W
    assert W.LIB.wtp_init(0) == 0, W.LIB.wtp_last_error()
    return W


def dev_u8(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).cuda()


def u32_out(n):
    return torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")


def to_u32(t, n):
    torch.cuda.synchronize()
    return t[:n].cpu().numpy().view(np.uint32)


# ---- fixed length, braided fast path ---------------------------------------------------
def test_c2_64k_x_1456_bit_exact(W):
    n = 65536
    buf = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    out = u32_out(n)
    W.crc32_batch_fixed(buf, 1456, 1456, n, out)
    got = to_u32(out, n)
    host = O.synth_fill_np(n * 1456)
    assert np.array_equal(buf.cpu().numpy(), host), "device synth fill != oracle generator"
    want = O.batch_fixed(host, 1456, 1456, n, threads=8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


def test_golden_batch_digest(W, golden):
    g = golden["batch_4096x1456"]
    buf = torch.empty(4096 * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    out = u32_out(4096)
    W.crc32_batch_fixed(buf, 1456, 1456, 4096, out)
    got = to_u32(out, 4096)
    assert [f"0x{c:08X}" for c in got[:8]] == g["first8"]
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == g["sha256_le_u32"]


def test_long_batch_into_unaligned_out(W):
    """A long batch (1 M x 1456 B: >= 64 rounds per wave, the held-results rule) whose
    result buffer is only 4-B aligned (out[1:] of a torch tensor): the held form stores
    16-B bursts, so the launcher must take the direct-store kernel here.  The whole vector
    equals the reference's 1 M digest, the guard word before it is untouched, and the
    aligned call of the same batch takes the held kernel (wtp_last_kernel)."""
    import json
    n = 1 << 20
    want = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_digests.json")))
    want = want["sha256_by_packets"][str(n)]
    buf = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    base = torch.full((n + 4,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    for shift, kern in ((1, "CrcBEpi"), (2, "CrcBEpi"), (3, "CrcBEpi"), (0, "CrcHoldBEpi"), (4, "CrcHoldBEpi")):
        base.fill_(0x5A5A5A5A)
        out = base[shift:shift + n]
        assert (out.data_ptr() % 16 == 0) == (kern == "CrcHoldBEpi")
        W.crc32_batch_fixed(buf, 1456, 1456, n, out)
        assert W.LIB.wtp_last_kernel().decode() == f"k_fixed_braid<6, 0, {kern}>"
        got = to_u32(out, n)
        assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == want, shift
        guard = base.cpu().numpy().view(np.uint32)
        assert (guard[:shift] == 0x5A5A5A5A).all() and (guard[shift + n:] == 0x5A5A5A5A).all(), shift


def test_last_kernel_names_every_route(W):
    """wtp_last_kernel() (bench.py's roofline.kernel) names the instantiation each route
    launched: braided direct / held, the general kernel for odd shapes and mixed lengths,
    the stream kernel when forced, the verify and builder epilogues."""
    name = lambda: W.LIB.wtp_last_kernel().decode()  # noqa: E731
    buf = torch.empty(4096 * 1472 + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    out = u32_out(4096)
    W.crc32_batch_fixed(buf, 1456, 1456, 4096, out)
    assert name() == "k_fixed_braid<6, 0, CrcBEpi>"
    W.crc32_batch_fixed(buf, 1457, 1000, 3000, out)
    assert name() == "k_pieces<FixedProvL, CrcEpi>"
    offs = torch.arange(0, 4096 * 100, 100, dtype=torch.int64, device="cuda")
    lens = torch.full((4096,), 100, dtype=torch.int32, device="cuda")
    W.crc32_batch_var(buf, 4096 * 1472, offs, lens, 4096, out)
    assert name() == "k_pieces<ArrayProvL, CrcEpi>"
    _forced_stream(W)(buf, 4096 * 1472, offs, lens, 4096, out)
    assert name() == "k_stream"
    wire = torch.empty(4096 * 1472 + 64, dtype=torch.uint8, device="cuda")
    wl = torch.empty(4096, dtype=torch.int32, device="cuda")
    W.build_data_packets(buf, 4096 * 1456, 0, wire, 1472, wl)
    assert name() == "k_fixed_braid<6, 0, BuildBEpi>"
    ok = torch.empty(4096, dtype=torch.uint8, device="cuda")
    W.verify_batch(wire, 1472, wl, 4096, ok)
    assert name() == "k_fixed_braid<6, 0, VerifyBEpi>"
    torch.cuda.synchronize()
    assert bool(ok.all())


def test_fixed_held_results_past_2g_result_bytes(W):
    """Held results (CrcHoldBEpi, long batches) past 2^29 packets: 16-B payloads, n =
    2^29 + 1237 (8.6 GB of payloads, 2.1 GB of results), so result byte offsets pass 2^31
    and the last dump ends mid-segment.  Spot checks against the oracle around the 2^29
    boundary, at the tail and at random packets."""
    n = (1 << 29) + 1237
    buf = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    W.crc32_batch_fixed(buf, 16, 16, n, out)
    torch.cuda.synchronize()
    rng = np.random.default_rng(29)
    idx = np.unique(np.concatenate([rng.integers(0, n, 1500), np.arange(n - 600, n),
                                    np.arange((1 << 29) - 300, (1 << 29) + 300), np.arange(0, 64)]))
    got = out[torch.from_numpy(idx).cuda()].cpu().numpy().view(np.uint32)
    want = np.array([O.crc32(O.synth_fill_np(16, start_byte=int(i) * 16)) for i in idx], dtype=np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at packets {idx[bad[:5]]}"
    del buf, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("length,stride", [(16, 16), (256, 256), (528, 544), (1024, 1024), (1296, 1312), (1536, 1536)])
def test_fixed_held_results_every_row_count(W, length, stride):
    """Long batches (>= 64 rounds per wave: the held-results epilogue) at every braided row
    count 1-6, odd n (a partial last round and a partial last dump), strides above the
    payload length: every packet of a sampled set and the whole tail against the oracle."""
    n = 600_001
    buf = torch.empty(n * stride + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    W.crc32_batch_fixed(buf, stride, length, n, out)
    torch.cuda.synchronize()
    rng = np.random.default_rng(length)
    idx = np.unique(np.concatenate([rng.integers(0, n, 400), np.arange(n - 300, n), np.arange(0, 40)]))
    got = out[torch.from_numpy(idx).cuda()].cpu().numpy().view(np.uint32)
    want = np.array([O.crc32(O.synth_fill_np(length, start_byte=int(i) * stride)) for i in idx], dtype=np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at packets {idx[bad[:5]]}"


def test_fixed_held_results_fuzz(W):
    """Seeded fuzz of long fixed batches (the held-results epilogue): random 16-B multiple
    lengths 16-1536, strides up to 1 KiB above them, n from 508 K to 1.2 M (odd counts,
    partial last rounds and dumps), a buffer offset that keeps 16-B alignment; sampled and
    tail packets against the oracle."""
    rng = np.random.default_rng(20261017)
    for case in range(6):
        length = 16 * int(rng.integers(1, 97))
        stride = length + 16 * int(rng.integers(0, 65))
        n = int(rng.integers(508_000, 1_200_000)) | 1
        lead = 16 * int(rng.integers(0, 8))
        buf = torch.empty(lead + n * stride + 64, dtype=torch.uint8, device="cuda")
        W.synth_fill(buf)
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        W.crc32_batch_fixed(buf[lead:], stride, length, n, out)
        torch.cuda.synchronize()
        idx = np.unique(np.concatenate([rng.integers(0, n, 200), np.arange(n - 130, n)]))
        got = out[torch.from_numpy(idx).cuda()].cpu().numpy().view(np.uint32)
        want = np.array([O.crc32(O.synth_fill_np(length, start_byte=lead + int(i) * stride)) for i in idx],
                        dtype=np.uint32)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (case, length, stride, n, lead, idx[bad[:5]])
        del buf, out


def test_reserve_cus_keeps_results(W, golden):
    """wtp_reserve_cus shrinks the persistent grids; results stay bit-exact (golden
    4096 x 1456 digest, a long batch past the 64-rounds-per-wave grid rule, and a mixed
    batch through the general kernel), and out-of-range counts are rejected."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    g = golden["batch_4096x1456"]
    buf = torch.empty(4096 * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    n2 = 600_000
    big = torch.empty(n2 * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(big)
    ref2 = None
    lens = O.zipf_lengths(20_000, s=1.1)
    try:
        for r in (0, 8, cus // 2, cus - 1):
            W.reserve_cus(r)
            out = u32_out(4096)
            W.crc32_batch_fixed(buf, 1456, 1456, 4096, out)
            got = to_u32(out, 4096)
            assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == g["sha256_le_u32"], r
            o2 = u32_out(n2)
            W.crc32_batch_fixed(big, 1456, 1456, n2, o2)
            v2 = to_u32(o2, n2).copy()
            if ref2 is None:
                ref2 = v2
                idx = np.random.default_rng(5).choice(n2, 300, replace=False)
                host = big.cpu().numpy()
                for i in idx:
                    assert v2[i] == O.crc32(host[i * 1456:(i + 1) * 1456]), i
            assert np.array_equal(v2, ref2), r
            _var_check(W.crc32_batch_var, lens, seed=r)
        for bad in (-1, cus, cus + 5):
            with pytest.raises(W.WtpError):
                W.reserve_cus(bad)
    finally:
        W.reserve_cus(0)


@pytest.mark.parametrize("L", [16, 240, 256, 272, 512, 1024, 1280, 1296, 1440, 1456, 1536])
@pytest.mark.parametrize("n", [1, 3, 4, 5, 63, 257, 4099])
def test_fast_path_lengths_and_tails(W, L, n):
    stride = ((L + 15) // 16) * 16 + 32 * (n % 2)  # stride > len on odd n
    host = O.synth_fill_np(n * stride, start_byte=L * 7 + n)
    d = dev_u8(host)
    out = u32_out(n)
    W.crc32_batch_fixed(d, stride, L, n, out)
    assert np.array_equal(to_u32(out, n), O.batch_fixed(host, stride, L, n))


# Horner flush groups: with the full 256-workgroup grid every wave runs 8-round groups;
# these sizes give each wave several full groups plus a partial one (9 or 10 rounds),
# exercising the group flush, the end-of-batch partial flush and the last round's
# packets past n, against the oracle on every packet.
@pytest.mark.parametrize("L", [1456, 1280, 1296, 528])
@pytest.mark.parametrize("n", [4 * (4096 * 9 + 1234) + 3, 4 * 4096 * 16 + 1])
def test_fast_path_full_groups_and_partial_tail(W, L, n):
    stride = ((L + 15) // 16) * 16
    host = O.synth_fill_np(n * stride, start_byte=L * 11 + n)
    d = dev_u8(host)
    out = u32_out(n)
    W.crc32_batch_fixed(d, stride, L, n, out)
    assert np.array_equal(to_u32(out, n), O.batch_fixed(host, stride, L, n))


def test_input_files_through_device(W, golden, golden_dir):
    for name, f in golden["files"].items():
        data = np.frombuffer(open(os.path.join(golden_dir, name), "rb").read(), dtype=np.uint8)
        n = len(f["chunk_lens"])
        full = data.size // 1456
        d = dev_u8(np.concatenate([data, np.zeros(16, np.uint8)]))
        out = u32_out(n)
        if full:
            W.crc32_batch_fixed(d, 1456, 1456, full, out)
        if n > full:
            W.crc32_batch_fixed(d[full * 1456:], 0, data.size - full * 1456, 1, out[full:])
        assert [f"0x{c:08X}" for c in to_u32(out, n)] == f["crc"], name


# ---- general kernel: every length, odd strides/alignments ------------------------------
def test_every_length_0_to_1456_var(W, golden):
    pl = golden["per_length"]["crc"]
    lens = np.arange(1457, dtype=np.uint32)
    offs = (1000 * lens).astype(np.uint64)
    total = int(offs[-1] + lens[-1]) + 16
    host = O.synth_fill_np(total)
    d = dev_u8(host)
    out = u32_out(1457)
    W.crc32_batch_var(d, total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), 1457, out)
    got = to_u32(out, 1457)
    assert list(got) == pl


def test_every_length_fixed_entry(W, golden):
    pl = golden["per_length"]["crc"]
    host = O.synth_fill_np(1457 * 1000 + 1460)
    d = dev_u8(host)
    out = u32_out(1)
    for L in range(0, 1457):
        W.crc32_batch_fixed(d[1000 * L:], 0, L, 1, out)
        got = to_u32(out, 1)[0]
        assert got == pl[L], L


@pytest.mark.parametrize("L,stride,lead", [(1455, 1455, 0), (1456, 1457, 3), (1456, 1456, 5), (100, 101, 1),
                                           (1, 1, 0), (0, 7, 0), (64, 64, 9), (65, 80, 15), (4096, 4100, 2),
                                           (1456, 1472, 8), (1484, 1500, 0)])
def test_general_strides_and_alignment(W, L, stride, lead):
    n = 777
    host = O.synth_fill_np(lead + n * stride + L + 16, start_byte=L + stride)
    d = dev_u8(host)
    out = u32_out(n)
    W.crc32_batch_fixed(d[lead:], stride, L, n, out)
    want = O.batch_fixed(host[lead:], stride, L, n)
    assert np.array_equal(to_u32(out, n), want)


# Mixed-length tests run through every mixed-length route: wtp_crc32_batch_var
# (k_pieces, any offsets), wtp_crc32_batch_packed (the same kernel below 2 GiB) and
# wtp_crc32_batch_packed with WTP_STREAM_KERNEL=1 (k_stream; payloads that break the
# packing take its lane-per-payload path, so every case must still be exact).
def _forced_stream(W):
    def call(*a, **k):
        os.environ["WTP_STREAM_KERNEL"] = "1"
        try:
            return W.crc32_batch_packed(*a, **k)
        finally:
            del os.environ["WTP_STREAM_KERNEL"]
    return call


@pytest.fixture(params=["var", "packed", "stream"])
def VAR(W, request):
    return {"var": W.crc32_batch_var, "packed": W.crc32_batch_packed, "stream": _forced_stream(W)}[request.param]


@pytest.mark.parametrize("n,s", [(200_000, 1.1), (1 << 20, 1.1), (1 << 20, 1.0), (1 << 20, 1.2)])
def test_zipf_mixed_lengths(W, VAR, n, s):
    """C5 itself at full size (1 M packets, Zipf 1.1 and 1.0; 1.2, mean ~96 B, as SURVEY §8a
    lists), every packet vs the oracle."""
    lens = O.zipf_lengths(n, s=s)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    host = O.synth_fill_np(total)
    d = dev_u8(host)
    out = u32_out(n)
    VAR(d, total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    assert np.array_equal(to_u32(out, n), O.batch_var(host, offs, lens))


def _var_check(VAR, lens, seed=0):
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    n = int(lens.size)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = max(int(lens.sum()), 1)
    host = O.synth_fill_np(total, start_byte=seed)
    d = dev_u8(host)
    out = u32_out(n)
    VAR(d, total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    assert np.array_equal(to_u32(out, n), O.batch_var(host, offs, lens))


def test_var_wave_split_long_subranges(W, VAR):
    """> 8 packets per thread in a workgroup's wave split (3 M packets: ~11.5 per thread),
    so the split's non-register fallback loops run; empty packets included."""
    rng = np.random.default_rng(11)
    _var_check(VAR, rng.integers(0, 4, 3 << 20), seed=3)


@pytest.mark.parametrize("n", [1, 2, 17, 1000, 1025, 70_000])
def test_var_wave_split_skewed(W, VAR, n):
    """Piece-balanced wave split with a few 4096-B packets (64 pieces) among 1-B ones:
    several waves' targets land in one packet (empty waves), and workgroups with fewer
    packets than threads."""
    lens = np.ones(n, dtype=np.uint32)
    lens[:: max(1, n // 7)] = 4096
    lens[-1] = 4096
    _var_check(VAR, lens, seed=n)


def test_var_all_tiny_workgroups(W, VAR):
    """Every workgroup's packets are 0 or 1 B (70 K packets, ~270 per workgroup): the
    case that faulted a round-3 development build (a split that counted such
    packets as 0 pieces left the wave ranges to stale LDS).  In the shipped split every
    packet is >= 1 piece and the wave ranges are clamped to the workgroup's packets."""
    rng = np.random.default_rng(70_000)
    _var_check(VAR, rng.integers(0, 2, 70_000).astype(np.uint32), seed=7)


def test_mixed_golden_digest(W, VAR, golden):
    lens = np.array([1 + (i * 7919) % 1456 for i in range(2048)], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    W.synth_fill(d)
    out = u32_out(2048)
    VAR(d, total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), 2048, out)
    got = to_u32(out, 2048)
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == golden["mixed_2048"]["sha256_le_u32"]


def test_var_shuffled_offsets_and_empty(W, VAR):
    rng = np.random.default_rng(5)
    n = 5000
    lens = rng.integers(0, 1485, n).astype(np.uint32)
    lens[::17] = 0
    total = 3_000_000
    offs = rng.integers(0, total - 1500, n).astype(np.uint64)  # overlapping, unordered
    host = O.synth_fill_np(total, start_byte=99)
    d = dev_u8(host)
    out = u32_out(n)
    VAR(d, total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    assert np.array_equal(to_u32(out, n), O.batch_var(host, offs, lens))


# Mixed-length batches: large batches, lengths around the piece boundaries up to the
# 4096-B limit, unordered/overlapping offsets, empty payloads, an unaligned base.
@pytest.mark.parametrize("case", ["uniform_shuffled", "all_long_packed", "all_short", "boundary_lengths", "zipf1.0_lead",
                                  "multi_segment", "row_boundaries", "small_runs"])
def test_var_mixed_cases(W, VAR, case):
    rng = np.random.default_rng(11)
    n = {"uniform_shuffled": 100_000, "multi_segment": 1_300_000}.get(case, 70_000)
    lead = 0
    if case == "uniform_shuffled":
        lens = rng.integers(0, 1600, n).astype(np.uint32)
        total = 40_000_000
        offs = rng.integers(0, total - 1600, n).astype(np.uint64)  # overlapping, unordered
    else:
        if case == "all_long_packed":
            lens = rng.integers(192, 1457, n).astype(np.uint32)
        elif case == "all_short":
            lens = rng.integers(0, 192, n).astype(np.uint32)
        elif case == "boundary_lengths":  # around chunk-count boundaries, up to the 4096-B limit
            lens = np.array([1, 2, 15, 16, 17, 191, 192, 193, 255, 256, 257, 1505, 1520, 1521, 1536, 1537, 4095,
                             4096], np.uint32)[rng.integers(0, 18, n)]
        elif case == "row_boundaries":  # lengths around 64 B pieces and 256 B rows, to 2000 B
            lens = np.array([1, 16, 17, 63, 64, 65, 66, 255, 256, 257, 258, 259, 260, 511, 512, 513, 514, 515, 767,
                             769, 1025, 1027, 1281, 1283, 1455, 1456, 1535, 1536, 1537, 2000], np.uint32)[
                rng.integers(0, 30, n)]
        elif case == "small_runs":  # long runs of <= 64-B packets with rare long ones
            lens = rng.integers(0, 65, n).astype(np.uint32)
            lens[rng.integers(0, n, n // 500)] = 700
        elif case == "multi_segment":  # > 1 segment per workgroup: the next segment's prefetch
            lens = O.zipf_lengths(n, s=1.1)
            lead = 9
        else:
            lens = O.zipf_lengths(n, s=1.0)
            lead = 7
        offs = (np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]) + np.uint64(3)).astype(np.uint64)
        total = int(offs[-1] + lens[-1]) + 16
    host = O.synth_fill_np(lead + total, start_byte=n + lead)
    d = dev_u8(host)
    out = u32_out(n)
    VAR(d[lead:], total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    assert np.array_equal(to_u32(out, n), O.batch_var(host[lead:], offs, lens)), case


# Packets starting in the view's first bytes (their head windows begin before the
# caller's base, which must read as zeros); every base alignment, short and long
# lengths, one packet per lane position.
@pytest.mark.parametrize("lead", [0, 1, 7, 15])
def test_var_packets_at_view_start(W, VAR, lead):
    lens_set = [1, 5, 15, 16, 17, 100, 127, 128, 129, 255, 256, 257, 300, 1456, 4095, 4096]
    offs, lens = [], []
    for L in lens_set:
        for o in range(0, 20):
            offs.append(o)
            lens.append(L)
    offs = np.array(offs, np.uint64)
    lens = np.array(lens, np.uint32)
    n = lens.size
    total = 4200
    host = O.synth_fill_np(lead + total, start_byte=lead * 3 + 1)
    d = dev_u8(host)
    out = u32_out(n)
    VAR(d[lead:], total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    assert np.array_equal(to_u32(out, n), O.batch_var(host[lead:], offs, lens))


def _fuzz_layout(rng):
    """One random mixed-length batch: a length distribution, a layout (packed, packed with
    gaps, unordered and overlapping, or runs of equal offsets) and a view lead."""
    n = int(rng.integers(1, 6000))
    kind = rng.choice(["uniform", "zipf", "tiny", "bimodal", "long", "rows"])
    if kind == "uniform":
        lens = rng.integers(0, 1457, n)
    elif kind == "zipf":
        lens = O.zipf_lengths(n, s=float(rng.choice([1.0, 1.1, 1.3])), seed=int(rng.integers(1 << 30)))
    elif kind == "tiny":
        lens = rng.integers(0, 17, n)
    elif kind == "bimodal":
        lens = np.where(rng.random(n) < 0.6, rng.integers(0, 33, n), rng.integers(1000, 1457, n))
    elif kind == "long":
        lens = rng.integers(1400, 4097, n)
    else:  # lengths at and around 64-B piece and 256-B row boundaries
        lens = rng.choice([1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1455, 1456], n)
    lens = np.asarray(lens, dtype=np.uint32)
    layout = rng.choice(["packed", "gaps", "unordered", "runs"])
    if layout in ("packed", "gaps"):
        gap = rng.integers(0, 40, n) if layout == "gaps" else np.zeros(n, np.int64)
        ends = np.cumsum(lens.astype(np.uint64) + gap.astype(np.uint64))
        offs = (ends - lens).astype(np.uint64)
        total = int(ends[-1]) if n else 1
    else:
        total = int(lens.sum()) + 5000
        offs = rng.integers(0, max(1, total - 4097), n).astype(np.uint64)
        if layout == "runs":
            offs = np.repeat(offs[::7], 7)[:n]
        total = max(total, int((offs + lens).max()))
    return lens, offs, max(total, 1), int(rng.integers(0, 64)), str(kind), str(layout)


@pytest.mark.parametrize("seed", range(12))
def test_var_fuzz_random_layouts(W, VAR, seed):
    """Seeded random batches through every route (piece kernel with LDS-DMA staging, its
    span-miss reloads, the packed and stream routes) vs the oracle, element-wise."""
    rng = np.random.default_rng(1000 + seed)
    for _ in range(4):
        lens, offs, total, lead, kind, layout = _fuzz_layout(rng)
        host = O.synth_fill_np(lead + total, start_byte=int(rng.integers(1 << 20)))
        d = dev_u8(host)
        n = lens.size
        out = u32_out(n)
        VAR(d[lead:], total, torch.from_numpy(offs.view(np.int64)).cuda(),
            torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
        want = O.batch_var(host[lead:], offs, lens)
        got = to_u32(out, n)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (kind, layout, n, lead, bad[:5])


@pytest.mark.parametrize("seed", range(6))
def test_verify_fuzz_random_rings(W, seed):
    """Seeded random datagram rings (stride a multiple of 16 or not, any recv_len including
    runts, oversize and full slots, bit flips in payload and header) vs the oracle."""
    rng = np.random.default_rng(2000 + seed)
    for _ in range(3):
        stride = int(rng.choice([1472, 1488, 1504, 1500, 1473, 64, 1024, 2048]))
        n = int(rng.integers(1, 5000))
        buf = O.synth_fill_np(n * stride, start_byte=int(rng.integers(1 << 20))).copy()
        rl = np.empty(n, np.uint32)
        for i in range(n):
            r = rng.random()
            L = stride if r < 0.5 else (int(rng.integers(0, 16)) if r < 0.6 else
                                       (stride + int(rng.integers(1, 40)) if r < 0.65 else int(rng.integers(16, stride + 1))))
            rl[i] = L
            if 16 <= L <= stride and rng.random() < 0.8:  # a valid checksum for its bytes
                crc = O.crc32(buf[i * stride + 16:i * stride + L])
                buf[i * stride + 12:i * stride + 16] = np.frombuffer(int(crc).to_bytes(4, "big"), np.uint8)
            if L > 16 and rng.random() < 0.1:
                buf[i * stride + 16 + int(rng.integers(0, min(L, stride) - 16))] ^= np.uint8(0x40)
        want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
        d = dev_u8(buf)
        r = torch.from_numpy(rl.view(np.int32)).cuda()
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        crc = u32_out(n)
        W.verify_batch(d, stride, r, n, ok, crc)
        torch.cuda.synchronize()
        assert np.array_equal(ok.cpu().numpy(), want_ok), (stride, n)
        assert np.array_equal(to_u32(crc, n), want_crc), (stride, n)


def test_var_bad_length_large_batch_sets_status(W, VAR):
    W.device_status(0, clear=True)
    n = 70_000
    lens = np.full(n, 700, np.uint32)
    lens[12345] = 5000
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(701)).astype(np.uint64)
    total = int(offs[-1]) + 5001
    host = O.synth_fill_np(total, start_byte=1)
    d = dev_u8(host)
    out = u32_out(n)
    VAR(d, total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    got = to_u32(out, n)
    want = O.batch_var(host, offs, np.where(lens > 4096, 0, lens).astype(np.uint32))
    want[12345] = 0
    assert np.array_equal(got, want)
    assert W.device_status(0, clear=True) & 1


def test_var_bad_length_sets_status(W, VAR):
    W.device_status(0, clear=True)
    host = O.synth_fill_np(10000)
    d = dev_u8(host)
    offs = torch.tensor([0, 10], dtype=torch.int64, device="cuda")
    lens = torch.tensor([5000, 20], dtype=torch.int32, device="cuda")
    out = u32_out(2)
    VAR(d, 10000, offs, lens, 2, out)
    got = to_u32(out, 2)
    assert got[0] == 0 and got[1] == O.crc32(host[10:30])
    assert W.device_status(0, clear=True) & 1


def _packed(lens, first=0):
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    offs = (np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]) + np.uint64(first)).astype(np.uint64)
    return offs, lens


def _run_packed(W, host, lead, offs, lens, total):
    n = int(lens.size)
    d = dev_u8(host)
    out = u32_out(n)
    W.crc32_batch_packed(d[lead:], total, torch.from_numpy(offs.view(np.int64)).cuda(),
                         torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    return to_u32(out, n)


@pytest.mark.parametrize("case", ["gaps", "overlaps", "swapped", "long_4096", "tiny_runs", "max_fast_4095"])
def test_packed_breaks_and_edges(W, case):
    """wtp_crc32_batch_packed on batches that break the packing at a few places (a gap,
    an overlap, two swapped payloads, 4096-B payloads beyond the fast path's 4095):
    the waves hand the rest of their range to the lane-per-payload path; runs of
    0-3-B payloads (many group rotations per 8 KiB round) and 4095-B payloads (the
    largest the length shift covers)."""
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    n = 300_000
    lens = O.zipf_lengths(n, s=1.1).astype(np.uint32)
    if case == "tiny_runs":
        lens = rng.integers(0, 4, n).astype(np.uint32)
        lens[rng.integers(0, n, 50)] = 1456
    if case == "max_fast_4095":
        lens = np.where(rng.random(n) < 0.3, 4095, lens).astype(np.uint32)
    offs, lens = _packed(lens, first=5)
    bad = np.sort(rng.choice(n - 2, 40, replace=False)) + 1
    if case == "gaps":
        offs[bad[0]:] += np.uint64(3)
        for b in bad[1:]:
            offs[b:] += np.uint64(int(rng.integers(1, 200)))
    elif case == "overlaps":
        for b in bad:
            offs[b] -= np.uint64(min(int(lens[b - 1]), 7))
    elif case == "swapped":
        for b in bad:
            offs[[b, b + 1]] = offs[[b + 1, b]]
            lens[[b, b + 1]] = lens[[b + 1, b]]
    elif case == "long_4096":
        lens[bad] = 4096
        offs, lens = _packed(lens, first=5)
    lead = 11
    total = int((offs + lens).max()) + 16
    host = O.synth_fill_np(lead + total, start_byte=n)
    got = _run_packed(W, host, lead, offs, lens, total)
    want = O.batch_var(host[lead:], offs, lens)
    assert np.array_equal(got, want), case
    # the stream kernel on the same batch: exact, and its per-payload path (status bit 3)
    # runs exactly when the batch breaks the packing or holds payloads >= 4096 B
    W.device_status(0, clear=True)
    out = u32_out(n)
    _forced_stream(W)(dev_u8(host)[lead:], total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    assert np.array_equal(to_u32(out, n), want), case
    slow = bool(W.device_status(0, clear=True) & 8)
    assert slow == (case in ("gaps", "overlaps", "swapped", "long_4096")), case


@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 127, 129, 511, 513, 4097])
def test_packed_small_batches(W, n):
    """Small packed batches (fewer payloads than lanes, waves or workgroups), every base
    alignment and a first offset that is not 0."""
    rng = np.random.default_rng(n)
    for lead in (0, 5, 15):
        lens = rng.integers(0, 1500, n).astype(np.uint32)
        offs, lens = _packed(lens, first=int(rng.integers(0, 300)))
        total = int(offs[-1] + lens[-1]) + int(rng.integers(0, 40))
        host = O.synth_fill_np(lead + total, start_byte=n + lead)
        got = _run_packed(W, host, lead, offs, lens, total)
        assert np.array_equal(got, O.batch_var(host[lead:], offs, lens)), (n, lead)


def test_packed_view_over_4gib(W, VAR):
    """A packed batch whose buffer is > 4 GiB (payloads at offsets past 2^32; the general
    kernel's views stop at 2 GiB, so wtp_crc32_batch_var hands it to the stream kernel):
    3.2 M x 1456-B payloads generated on the device, every CRC equal to the braided
    fixed-length kernel's, and sampled payloads vs the oracle (regenerated from the
    generator at their global offsets)."""
    n, L = 3_200_000, 1456
    total = n * L
    assert total > (1 << 32)
    W.device_status(0, clear=True)
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    W.synth_fill(d)
    lens = np.full(n, L, np.uint32)
    offs, lens = _packed(lens)
    out = u32_out(n)
    VAR(d, total, torch.from_numpy(offs.view(np.int64)).cuda(), torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    ref = u32_out(n)
    W.crc32_batch_fixed(d, L, L, n, ref)
    got = to_u32(out, n)
    assert np.array_equal(got, to_u32(ref, n))
    for i in (0, 1, 2949840, 2949841, n - 1):  # payload 2949840 straddles 2^32, 2949841 starts past it
        assert int(got[i]) == O.crc32(O.synth_fill_np(L, start_byte=i * L)), i
    # packed: every wave stays on the fast path, including waves starting between 2 and
    # 4 GiB (a sign-extended wave base sent those to the per-payload path until round 5)
    assert not (W.device_status(0, clear=True) & 8)
    del d


@pytest.mark.parametrize("broken", [False, True])
def test_packed_zipf_over_2gib_piece_ranges(W, broken):
    """wtp_crc32_batch_packed on 17 M Zipf(1.1) payloads (2.3 GB, past 2 GiB): the piece
    kernel in device-cut < 2 GiB sub-launches (launch_packed_ranges), not k_stream.  Every
    CRC equals the stream kernel's over the same batch (WTP_STREAM_KERNEL=1) and the oracle
    on the payloads around each 2 GiB - 64 KiB cut and a random sample.  broken: 40 pairs of
    adjacent payloads swapped (these stay inside their sub-launch's view: computed there)
    and one payload just before the first cut swapped with one ~5000 payloads past it,
    which puts it outside its view (offsets not packed) -> that sub-launch flags it and the
    gated k_stream recomputes the batch (status bit 3: its per-payload path ran); still
    exact.  packed: no flag, k_stream returns at once (bit 3 clear)."""
    n = 17_000_000
    lens = O.zipf_lengths(n, s=1.1).astype(np.uint32)
    offs, lens = _packed(lens, first=3)
    rng = np.random.default_rng(17)
    G = (1 << 31) - (1 << 16)
    cut = int(np.searchsorted(offs, np.uint64(G - 3)))
    if broken:
        for b in np.sort(rng.choice(n - 2, 40, replace=False)):
            offs[[b, b + 1]] = offs[[b + 1, b]]
            lens[[b, b + 1]] = lens[[b + 1, b]]
        a, b = cut - 5, cut + 5000
        assert int(offs[b]) - G > (1 << 16)  # past the first sub-launch's < 2 GiB view
        offs[[a, b]] = offs[[b, a]]
        lens[[a, b]] = lens[[b, a]]
    total = int((offs + lens).max()) + 8
    assert total > (1 << 31)
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    W.synth_fill(d)
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out = u32_out(n)
    W.device_status(0, clear=True)
    W.crc32_batch_packed(d, total, do, dl, n, out)
    assert W.LIB.wtp_last_kernel().decode().startswith("k_pieces<RangeArrayProvL, CrcEpi>")
    assert bool(W.device_status(0, clear=True) & 8) == broken  # the gated k_stream's per-payload path
    got = to_u32(out, n)
    ref = u32_out(n)
    _forced_stream(W)(d, total, do, dl, n, ref)
    assert np.array_equal(got, to_u32(ref, n))
    idx = np.unique(np.concatenate([np.arange(cut - 6, cut + 3), [0, n - 1, cut + 5000], rng.integers(0, n, 3000)]))
    host = d.cpu().numpy()
    del d
    want = O.batch_var(host, offs[idx], lens[idx])
    assert np.array_equal(got[idx], want)


def test_packed_over_2gib_edges_at_the_cut(W):
    """The >= 2 GiB piece route's edges: a 4-B-misaligned base (d[5:]), a first offset
    that is not 0, empty payloads and over-long (5000 B: crc 0, status flag) payloads right
    at the 2 GiB - 64 KiB cut, a payload straddling it, and a short last range.  Every CRC
    equal to the stream kernel's (forced) and the oracle around the cut."""
    W.device_status(0, clear=True)
    G = (1 << 31) - (1 << 16)
    n = 1_650_000
    rng = np.random.default_rng(11)
    lens = rng.integers(0, 2800, n).astype(np.uint32)
    offs, lens = _packed(lens, first=7)
    cut = int(np.searchsorted(offs + np.uint64(5), np.uint64(G)))  # view offsets include the base's lead
    assert 100 < cut < n - 100
    lens[cut - 3:cut - 1] = 0
    lens[cut + 1] = 5000
    lens[cut - 6] = 4096
    offs, lens = _packed(lens, first=7)
    total = int(offs[-1] + lens[-1]) + 3
    assert total + 5 > (1 << 31) + (1 << 20)
    d = torch.empty(total + 5, dtype=torch.uint8, device="cuda")
    W.synth_fill(d)
    dv = d[5:]
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    out, ref = u32_out(n), u32_out(n)
    W.crc32_batch_packed(dv, total, do, dl, n, out)
    assert W.LIB.wtp_last_kernel().decode().startswith("k_pieces<RangeArrayProvL")
    assert W.device_status(0, clear=True) & 1  # the 5000-B payload
    _forced_stream(W)(dv, total, do, dl, n, ref)
    got = to_u32(out, n)
    assert np.array_equal(got, to_u32(ref, n))
    idx = np.arange(cut - 40, cut + 40)
    host = d[5:].cpu().numpy()
    del d, dv
    want = O.batch_var(host, offs[idx], np.where(lens[idx] > 4096, 0, lens[idx]).astype(np.uint32))
    assert np.array_equal(got[idx], want)
    assert got[cut + 1] == 0 and got[cut - 3] == 0 and got[cut - 2] == 0


def _graph_of(calls):
    """One HIP graph holding `calls` in order, captured on a side stream after one eager
    run of each there (library state keyed by stream is made outside the capture)."""
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        for c in calls:
            c()
    cs.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cs):
        for c in calls:
            c()
    return g


def test_packed_over_2gib_graph_of_three_calls(W):
    """Three packed >= 2 GiB calls (device-cut piece sub-launches) captured in ONE graph,
    each into its own output: after clearing, a replay rewrites all three, equal to the
    eager results, and a copy queued behind the replay sees them (stream order).  With
    descriptors from a stream-ordered pool, such a graph replayed as no-ops (r05b)."""
    n = 17_000_000
    lens = O.zipf_lengths(n, s=1.1).astype(np.uint32)
    offs, lens = _packed(lens)
    total = int(offs[-1] + lens[-1])
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    W.synth_fill(d)
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    outs = [u32_out(n) for _ in range(3)]
    calls = [lambda o=o: W.crc32_batch_packed(d, total, do, dl, n, o) for o in outs]
    calls[0]()
    want = outs[0].clone()
    g = _graph_of(calls)
    torch.cuda.synchronize()
    for o in outs:
        o.zero_()
    g.replay()
    snap = torch.stack(outs).clone()  # queued behind the replay, no host sync in between
    torch.cuda.synchronize()
    for i in range(3):
        assert torch.equal(snap[i], want), i
    idx = np.random.default_rng(3).integers(0, n, 500)
    host_idx = np.unique(idx)
    got = to_u32(outs[2], n)
    for i in host_idx[:50]:
        i = int(i)
        assert int(got[i]) == O.crc32(d[int(offs[i]):int(offs[i]) + int(lens[i])].cpu().numpy()), i


def test_packed_over_2gib_captured_on_torch_capture_stream(W):
    """a packed >= 2 GiB call captured with torch.cuda.graph(g) and no
    stream= (torch's shared default capture stream, never used eagerly) must capture, not
    fail; and two such graphs, each over its own batch, replayed at once on two streams
    must each give their own exact results (each captured call owns its descriptor slot)."""
    n = 17_000_000
    lens = O.zipf_lengths(n, s=1.1).astype(np.uint32)
    offs, lens = _packed(lens)
    total = int(offs[-1] + lens[-1])
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    ds = [torch.empty(total, dtype=torch.uint8, device="cuda") for _ in range(2)]
    for k, d in enumerate(ds):
        W.synth_fill(d, start_byte=k * 977)
    outs = [u32_out(n) for _ in range(2)]
    wants = []
    for d in ds:
        w = u32_out(n)
        W.crc32_batch_packed(d, total, do, dl, n, w)
        wants.append(w)
    torch.cuda.synchronize()
    assert not torch.equal(wants[0], wants[1])
    graphs = []
    for d, o in zip(ds, outs):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            W.crc32_batch_packed(d, total, do, dl, n, o)
        graphs.append(g)
    assert W.LIB.wtp_last_kernel().decode().startswith("k_pieces<RangeArrayProvL")
    torch.cuda.synchronize()
    for o in outs:
        o.zero_()
    torch.cuda.synchronize()
    ss = [torch.cuda.Stream() for _ in range(2)]
    for rep in range(3):
        for g, s in zip(graphs, ss):
            with torch.cuda.stream(s):
                g.replay()
        torch.cuda.synchronize()
        for k in range(2):
            assert torch.equal(outs[k], wants[k]), (rep, k)
    i = int(n // 2)
    assert int(to_u32(outs[1], n)[i]) == O.crc32(ds[1][int(offs[i]):int(offs[i]) + int(lens[i])].cpu().numpy())


def test_builder_slow_path_graph_of_three_calls(W):
    """The fused builder's three-step path (unaligned payloads, no length array: its CRCs
    go through stream-ordered scratch) three times in ONE graph, each into its own wire
    buffer: a replay after clearing rebuilds all three exactly as the eager calls did."""
    m = 20_001
    pay = torch.empty(m * 1456 + 64, dtype=torch.uint8, device="cuda")
    W.synth_fill(pay)
    wires = [torch.zeros(m * 1472 + 64, dtype=torch.uint8, device="cuda") for _ in range(3)]
    calls = [lambda w=w, k=k: W.build_data_packets(pay[3 + k:], m * 1456 - 100, 7, w, 1472, None)
             for k, w in enumerate(wires)]
    for c in calls:
        c()
    torch.cuda.synchronize()
    want = [w.clone() for w in wires]
    g = _graph_of(calls)
    torch.cuda.synchronize()
    for w in wires:
        w.zero_()
    g.replay()
    torch.cuda.synchronize()
    for k in range(3):
        assert torch.equal(wires[k], want[k]), k


def test_var_unordered_view_over_2gib(W):
    """wtp_crc32_batch_var on a 2.3 GB buffer (no longer EINVAL): 100 K payloads at
    unordered, overlapping offsets across the whole buffer, lengths 0..1500 and a few
    over-long ones -> the stream kernel's lane-per-payload path, every CRC vs the oracle."""
    W.device_status(0, clear=True)
    total = 2_300_000_000
    rng = np.random.default_rng(23)
    n = 100_000
    lens = rng.integers(0, 1501, n).astype(np.uint32)
    lens[::9973] = 5000
    offs = rng.integers(0, total - 6000, n).astype(np.uint64)
    offs[:50] = np.arange(50, dtype=np.uint64) * np.uint64(3)  # some near the start, overlapping
    offs[50:100] = np.uint64(total - 1600) + np.arange(50, dtype=np.uint64)  # some ending near the end
    lens[50:100] = np.minimum(lens[50:100], 1500)
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    W.synth_fill(d)
    out = u32_out(n)
    W.crc32_batch_var(d, total, torch.from_numpy(offs.view(np.int64)).cuda(),
                      torch.from_numpy(lens.view(np.int32)).cuda(), n, out)
    got = to_u32(out, n)
    host = d.cpu().numpy()
    del d
    want = O.batch_var(host, offs, np.where(lens > 4096, 0, lens).astype(np.uint32))
    assert np.array_equal(got, want)
    assert W.device_status(0, clear=True) & 1


# ---- receiver verify, packet builder, host pipelines -----------------------------------
def _datagrams(n, stride, rng):
    buf = np.zeros(n * stride, dtype=np.uint8)
    rl = np.zeros(n, dtype=np.uint32)
    payloads = []
    for i in range(n):
        L = int(rng.integers(0, min(stride - 16, 1484) + 1))
        p = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        dg = O.build_datagram(i, p)
        buf[i * stride:i * stride + len(dg)] = np.frombuffer(dg, dtype=np.uint8)
        rl[i] = len(dg)
        payloads.append(p)
    return buf, rl


def test_verify_batch(W):
    rng = np.random.default_rng(3)
    n, stride = 3000, 1500
    buf, rl = _datagrams(n, stride, rng)
    # corrupt: payload bit flips, header checksum flips, runts, recv_len > stride
    flip = rng.choice(n, 300, replace=False)
    for i in flip[:200]:
        if rl[i] > 16:
            buf[i * stride + 16 + int(rng.integers(0, rl[i] - 16))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    for i in flip[200:250]:
        buf[i * stride + 12] ^= 0x80
    rl[flip[250:270]] = rng.integers(0, 16, 20).astype(np.uint32)
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    d = dev_u8(buf)
    r = torch.from_numpy(rl.view(np.int32)).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    crc = u32_out(n)
    W.verify_batch(d, stride, r, n, ok, crc)
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), want_ok)
    assert np.array_equal(to_u32(crc, n), want_crc)
    assert want_ok.sum() < n - 200  # the corruptions were caught


def _full_ring(n, stride, rng, frac_full=0.9):
    """A receive ring as the braided verify path sees it: mostly full datagrams
    (recv_len == stride), the rest short, empty, runt or oversize."""
    L = stride - 16
    buf = np.zeros(n * stride, dtype=np.uint8)
    rl = np.zeros(n, dtype=np.uint32)
    body = O.synth_fill_np(n * L, start_byte=stride)
    for i in range(n):
        u = rng.random()
        if u < frac_full:
            p = body[i * L:(i + 1) * L].tobytes()
        else:
            p = body[i * L:i * L + int(rng.integers(0, L))].tobytes()
        dg = O.build_datagram(i, p)
        buf[i * stride:i * stride + len(dg)] = np.frombuffer(dg, dtype=np.uint8)
        rl[i] = len(dg)
    k = max(1, n // 50)
    idx = rng.choice(n, 4 * k, replace=False)
    for i in idx[:k]:  # payload bit flips
        if rl[i] > 16:
            buf[i * stride + 16 + int(rng.integers(0, rl[i] - 16))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    for i in idx[k:2 * k]:  # header checksum flips
        buf[i * stride + 12 + int(rng.integers(0, 4))] ^= 0x10
    rl[idx[2 * k:3 * k]] = rng.integers(0, 16, k).astype(np.uint32)  # runts
    rl[idx[3 * k:]] = stride + rng.integers(1, 40, k).astype(np.uint32)  # oversize (truncated)
    return buf, rl


def _verify_dev(W, buf, stride, rl, n, with_crc=True, offset=0):
    raw = np.zeros(len(buf) + offset, dtype=np.uint8)
    raw[offset:] = buf
    d = dev_u8(raw)[offset:]
    r = torch.from_numpy(rl.view(np.int32)).cuda()
    ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    crc = u32_out(n) if with_crc else None
    W.verify_batch(d, stride, r, n, ok, crc)
    torch.cuda.synchronize()
    return ok.cpu().numpy(), (to_u32(crc, n) if with_crc else None)


@pytest.mark.parametrize("n,stride,frac,with_crc", [
    (3001, 1472, 0.9, True),    # braided fast path + in-kernel fix-up phase
    (3001, 1472, 0.9, False),   # no crc output
    (517, 1472, 1.0, True),     # every datagram full
    (400, 1488, 0.0, True),     # 16-B stride, no datagram full: all through the fix-up
    (999, 32, 0.7, True),       # smallest fast-path stride (16-B payloads)
    (777, 1104, 0.8, True),     # 4-row braid frames
])
def test_verify_fast_path(W, n, stride, frac, with_crc):
    rng = np.random.default_rng(n + stride)
    buf, rl = _full_ring(n, stride, rng, frac)
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    ok, crc = _verify_dev(W, buf, stride, rl, n, with_crc)
    assert np.array_equal(ok, want_ok), np.nonzero(ok != want_ok)[0][:10]
    if with_crc:
        assert np.array_equal(crc, want_crc), np.nonzero(crc != want_crc)[0][:10]
    assert 0 < want_ok.sum() < n or frac == 1.0 or frac == 0.0


def _long_ring(n, stride, rng):
    """A long receive ring built with numpy (n in the hundreds of thousands): full WTP
    datagrams with 16 + (stride - 16)-B lengths and, on a few percent, short receive
    lengths, runts, oversize lengths, payload and header-checksum bit flips."""
    L = stride - 16
    body = O.synth_fill_np(n * L, start_byte=11)
    crcs = O.batch_fixed(body, L, L, n, threads=8)
    buf = np.zeros((n, stride), dtype=np.uint8)
    buf[:, 16:] = body.reshape(n, L)
    hdr = np.stack([np.full(n, 2, np.uint32), np.arange(n, dtype=np.uint32), np.full(n, L, np.uint32), crcs], axis=1)
    buf[:, :16] = hdr.astype(">u4").view(np.uint8).reshape(n, 16)
    rl = np.full(n, stride, dtype=np.uint32)
    k = n // 100
    idx = rng.choice(n, 5 * k, replace=False)
    rl[idx[:k]] = 16 + rng.integers(0, L, k).astype(np.uint32)        # short: the fix-up phase
    rl[idx[k:2 * k]] = rng.integers(0, 16, k).astype(np.uint32)       # runts
    rl[idx[2 * k:3 * k]] = stride + rng.integers(1, 40, k).astype(np.uint32)  # oversize
    for i in idx[3 * k:4 * k]:
        buf[i, 16 + int(rng.integers(0, L))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    buf[idx[4 * k:], 12] ^= 0x10
    return buf.reshape(-1), rl


@pytest.mark.parametrize("stride", [1472, 1504])
def test_verify_long_ring_with_fixups(W, stride):
    """Rings long enough for the long-batch rules (>= 64 rounds per wave), with listed
    datagrams spread over every workgroup: every ok and crc against the oracle (the fix-up
    phase rewrites entries the braided pass wrote first)."""
    n = 600_003
    rng = np.random.default_rng(stride)
    buf, rl = _long_ring(n, stride, rng)
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    ok, crc = _verify_dev(W, buf, stride, rl, n, True)
    assert np.array_equal(ok, want_ok), np.nonzero(ok != want_ok)[0][:10]
    assert np.array_equal(crc, want_crc), np.nonzero(crc != want_crc)[0][:10]
    ok2, _ = _verify_dev(W, buf, stride, rl, n, False)
    assert np.array_equal(ok2, want_ok)
    assert 0 < want_ok.sum() < n


def _wtp_ring(n, stride, rng):
    """wReceiver's ring: 1504-B slots holding up to 1500 received bytes.  Mostly full
    WTP DATA datagrams (1472 B), some 1473-1500 B (non-WTP senders; the reference CRCs
    them like any other, Receiver.cpp:123-125,32-33), short ones, runts, corruptions."""
    buf = np.zeros(n * stride, dtype=np.uint8)
    rl = np.zeros(n, dtype=np.uint32)
    body = O.synth_fill_np(n * 1484, start_byte=stride + n)
    kinds = rng.random(n)
    for i in range(n):
        L = 1456 if kinds[i] < 0.75 else (int(rng.integers(1457, 1485)) if kinds[i] < 0.9 else int(rng.integers(0, 1456)))
        dg = O.build_datagram(i, body[i * 1484:i * 1484 + L].tobytes())
        buf[i * stride:i * stride + len(dg)] = np.frombuffer(dg, dtype=np.uint8)
        rl[i] = len(dg)
    k = n // 40
    idx = rng.choice(n, 3 * k, replace=False)
    for i in idx[:k]:
        buf[i * stride + 16 + int(rng.integers(0, rl[i] - 16 if rl[i] > 16 else 1))] ^= 0x04
    for i in idx[k:2 * k]:
        buf[i * stride + 13] ^= 0x01
    rl[idx[2 * k:]] = rng.integers(0, 16, k).astype(np.uint32)
    return buf, rl


@pytest.mark.parametrize("n", [1, 97, 4099])
def test_verify_wreceiver_1504_slots(W, n):
    """1473-1500-B datagrams are verified with the reference's semantics (CRC over
    [16, recv_len)) at wReceiver's 1504-B stride; full 1472-B WTP datagrams take the
    braided fast path inside the wider slots."""
    rng = np.random.default_rng(n)
    buf, rl = _wtp_ring(n, 1504, rng)
    assert (rl > 1472).any() or n < 10
    want_ok, want_crc = O.verify_datagrams(buf, 1504, rl)
    ok, crc = _verify_dev(W, buf, 1504, rl, n, True)
    assert np.array_equal(ok, want_ok), np.nonzero(ok != want_ok)[0][:10]
    assert np.array_equal(crc, want_crc), np.nonzero(crc != want_crc)[0][:10]
    ok2, crc2 = W.host_verify(buf, 1504, rl)
    assert np.array_equal(ok2, want_ok) and np.array_equal(crc2, want_crc)


def test_verify_calls_are_independent(W):
    """The braided verify keeps no state between calls (each workgroup finishes its own
    short/odd datagrams in its fix-up phase): back-to-back calls on one stream (growing
    and shrinking batches), calls on a second stream, an all-full ring (no fix-up work)
    between them, hipStreamPerThread from two threads, and CUDA-graph captures on a fresh
    stream and on a stream that verified before, each replayed twice, all bit-exact."""
    rng = np.random.default_rng(2024)
    stride = 1504
    rings = {}
    for n in (64, 3001, 97, 20000, 1):
        buf, rl = _wtp_ring(n, stride, rng)
        want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
        rings[n] = (dev_u8(buf), torch.from_numpy(rl.view(np.int32)).cuda(), want_ok, want_crc)
    full_n = 500
    full = torch.empty(full_n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(full)
    fwire = torch.zeros(full_n * stride, dtype=torch.uint8, device="cuda")
    fwl = torch.empty(full_n, dtype=torch.int32, device="cuda")
    W.build_data_packets(full, full_n * 1456, 0, fwire, stride, fwl)

    def run(n, stream=None):
        d, r, _, _ = rings[n]
        ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        crc = u32_out(n)
        W.verify_batch(d, stride, r, n, ok, crc, stream=stream)
        return ok, crc

    def check(n, ok, crc):
        _, _, want_ok, want_crc = rings[n]
        assert np.array_equal(ok.cpu().numpy(), want_ok), n
        assert np.array_equal(to_u32(crc, n), want_crc), n

    outs = []
    for rep in range(3):
        for n in (64, 3001, 97, 20000, 1):
            outs.append((n, *run(n)))
            fok = torch.zeros(full_n, dtype=torch.uint8, device="cuda")
            W.verify_batch(fwire, stride, fwl, full_n, fok)
            outs.append((None, fok, None))
    s2 = torch.cuda.Stream()
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s2):
        for n in (3001, 64):
            outs.append((n, *run(n)))
    torch.cuda.synchronize()
    # hipStreamPerThread (handle 2): a different stream in every host thread; two threads
    # at once
    import threading
    res = {}

    def per_thread(tag, n):
        res[tag] = (n, *run(n, stream=2))

    ths = [threading.Thread(target=per_thread, args=(t, n)) for t, n in (("a", 3001), ("b", 20000))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    outs.extend(res.values())
    torch.cuda.synchronize()
    for n, ok, crc in outs:
        if n is None:
            assert bool(ok.all())
        else:
            check(n, ok, crc)
    # graph capture: the captured call is one kernel node whose only memory is the
    # caller's buffers
    d, r, _, _ = rings[3001]
    for warm in (False, True):
        gok = torch.full((3001,), 7, dtype=torch.uint8, device="cuda")
        gcrc = u32_out(3001)
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            if warm:
                run(3001, stream=cs)
                cs.synchronize()
            g.capture_begin()
            W.verify_batch(d, stride, r, 3001, gok, gcrc)
            g.capture_end()
        torch.cuda.current_stream().wait_stream(cs)
        for _ in range(2):
            gok.fill_(7)
            with torch.cuda.stream(cs):
                g.replay()
            torch.cuda.synchronize()
            check(3001, gok, gcrc)
            check(97, *run(97))  # calls on the default stream between replays


def test_verify_many_streams(W):
    """300 streams, one verify each, all in flight together (round 2 kept a fix-up slot
    per stream and had to drop them past 256; now nothing is kept): every call on every
    stream is bit-exact."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    rng = np.random.default_rng(77)
    n, stride = 97, 1504
    buf, rl = _wtp_ring(n, stride, rng)
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    d = dev_u8(buf)
    r = torch.from_numpy(rl.view(np.int32)).cuda()
    torch.cuda.synchronize()
    streams, outs = [], []
    try:
        for _ in range(300):
            h = C.c_void_p()
            assert hip.hipStreamCreate(C.byref(h)) == 0
            streams.append(h)
            ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
            crc = u32_out(n)
            W.verify_batch(d, stride, r, n, ok, crc, stream=h.value)
            outs.append((ok, crc))
        torch.cuda.synchronize()
        for ok, crc in outs:
            assert np.array_equal(ok.cpu().numpy(), want_ok)
            assert np.array_equal(to_u32(crc, n), want_crc)
    finally:
        torch.cuda.synchronize()
        for h in streams:
            hip.hipStreamDestroy(h)


def test_verify_sub_batches(W):
    """A ring longer than one fast-path launch takes (stride 16384: 131,071 datagrams per
    sub-batch, each launch's ring view < 2 GiB): two launches, each with short and
    corrupt datagrams of its own, including both sides of the boundary."""
    stride, n = 16384, 140_000
    per = ((1 << 31) - 4096) // stride
    assert n > per
    payload = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(payload, start_byte=99)
    wire = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    wl = torch.empty(n, dtype=torch.int32, device="cuda")
    W.build_data_packets(payload, n * 1456, 0, wire, stride, wl)
    del payload
    rng = np.random.default_rng(140)
    short = np.concatenate([rng.choice(per, 300, replace=False), per + rng.choice(n - per, 300, replace=False),
                            [per - 1, per, per + 1]])
    rl = wl.cpu().numpy().view(np.uint32).copy()
    rl[short] = rng.integers(0, 1470, short.size).astype(np.uint32)
    flip = np.concatenate([rng.choice(per, 50, replace=False), per + rng.choice(n - per, 50, replace=False)])
    wv = wire.view(n, stride)
    for i in flip:
        wv[int(i), 100] ^= 0x20
    r = torch.from_numpy(rl.view(np.int32)).cuda()
    ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    crc = u32_out(n)
    W.verify_batch(wire, stride, r, n, ok, crc)
    got_ok = ok.cpu().numpy()
    got_crc = to_u32(crc, n)
    check = np.unique(np.concatenate([short, flip, rng.choice(n, 2000, replace=False), [0, n - 1]]))
    for i in check:
        i = int(i)
        dg = wv[i].cpu().numpy()
        want_ok, want_crc = O.verify_datagrams(dg, stride, rl[i:i + 1])
        assert got_ok[i] == want_ok[0] and got_crc[i] == want_crc[0], i
    # everything not shortened or flipped is a full, valid datagram
    intact = np.ones(n, bool)
    intact[short] = False
    intact[flip] = False
    assert got_ok[intact].all()


def test_verify_graph_replay_after_larger_call_on_its_stream(W):
    """a graph captured on a stream, then a larger verify on that stream (round
    2 then freed the stream's fix-up slot that the graph had baked in), then the graph
    replayed: bit-exact, and so is the larger call."""
    rng = np.random.default_rng(55)
    stride = 1504
    small, big = 3001, 20000
    rings = {}
    for n in (small, big):
        buf, rl = _wtp_ring(n, stride, rng)
        want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
        rings[n] = (dev_u8(buf), torch.from_numpy(rl.view(np.int32)).cuda(), want_ok, want_crc)
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    d, r, want_ok, want_crc = rings[small]
    gok = torch.full((small,), 7, dtype=torch.uint8, device="cuda")
    gcrc = u32_out(small)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cs):
        W.verify_batch(d, stride, r, small, gok, gcrc, stream=cs)
        cs.synchronize()
        g.capture_begin()
        W.verify_batch(d, stride, r, small, gok, gcrc)
        g.capture_end()
        d2, r2, want_ok2, want_crc2 = rings[big]
        ok2 = torch.full((big,), 7, dtype=torch.uint8, device="cuda")
        crc2 = u32_out(big)
        W.verify_batch(d2, stride, r2, big, ok2, crc2)
        for _ in range(2):
            gok.fill_(7)
            gcrc.fill_(-1)
            g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(gok.cpu().numpy(), want_ok) and np.array_equal(to_u32(gcrc, small), want_crc)
    assert np.array_equal(ok2.cpu().numpy(), want_ok2) and np.array_equal(to_u32(crc2, big), want_crc2)


@pytest.mark.parametrize("stride,frac_full", [(1472, 0.0), (1504, 0.3)])
def test_verify_fixup_multi_pass(W, stride, frac_full):
    """More fix-up datagrams per workgroup than one rescan pass covers (4096 packets):
    with all but 6 CUs reserved, 6 workgroups own 30,000 datagrams (~5,000 each), so
    every workgroup's fix-up phase runs two passes; every ok/crc is written (prefilled
    with 7 / 0xFFFFFFFF) and equals the oracle."""
    rng = np.random.default_rng(stride)
    n = 30000
    buf = np.zeros(n * stride, dtype=np.uint8)
    rl = np.zeros(n, dtype=np.uint32)
    body = O.synth_fill_np(n * 1456, start_byte=17)
    for i in range(n):
        L = 1456 if rng.random() < frac_full else int(rng.integers(0, min(stride - 16, 1484) + 1))
        if L == 1456 and stride > 1472 and rng.random() < 0.5:
            L = int(rng.integers(1457, stride - 15))
        dg = O.build_datagram(i, body[i * 1456:i * 1456 + min(L, 1456)].tobytes() + bytes(max(0, L - 1456)))
        buf[i * stride:i * stride + len(dg)] = np.frombuffer(dg, dtype=np.uint8)
        rl[i] = len(dg)
    bad = rng.choice(n, 300, replace=False)
    for i in bad:
        if rl[i] > 16:
            buf[i * stride + 16 + int(rng.integers(0, rl[i] - 16))] ^= 0x08
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    W.reserve_cus(cus - 6, 0)
    try:
        d = dev_u8(buf)
        r = torch.from_numpy(rl.view(np.int32)).cuda()
        ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        crc = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        W.verify_batch(d, stride, r, n, ok, crc)
        torch.cuda.synchronize()
    finally:
        W.reserve_cus(0, 0)
    assert np.array_equal(ok.cpu().numpy(), want_ok), np.nonzero(ok.cpu().numpy() != want_ok)[0][:10]
    assert np.array_equal(to_u32(crc, n), want_crc)
    assert W.device_status(0, clear=True) == 0


def test_verify_misaligned_ring_takes_general_path(W):
    rng = np.random.default_rng(11)
    n, stride = 700, 1472
    buf, rl = _full_ring(n, stride, rng)
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    ok, crc = _verify_dev(W, buf, stride, rl, n, True, offset=4)
    assert np.array_equal(ok, want_ok) and np.array_equal(crc, want_crc)


def test_verify_large_ring_properties(W, golden_dir):
    """1M full 1472-B datagrams built on the device: every one verifies; one flipped
    payload bit per 4099 datagrams is caught exactly there; the whole CRC vector vs the
    reference's digest of the same payloads (bench_digests.json)."""
    import hashlib
    import json
    n, stride = 1 << 20, 1472
    payload = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(payload)
    wire = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    wl = torch.empty(n, dtype=torch.int32, device="cuda")
    W.build_data_packets(payload, n * 1456, 0, wire, stride, wl)
    del payload
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    crc = u32_out(n)
    W.verify_batch(wire, stride, wl, n, ok, crc)
    torch.cuda.synchronize()
    assert int(ok.sum().item()) == n
    got = to_u32(crc, n)
    for i in (0, 1, 2, 3, 4, 65535, n // 2 + 1, n - 2, n - 1):
        assert int(got[i]) == O.crc32(O.synth_fill_np(1456, start_byte=i * 1456)), i
    with open(os.path.join(golden_dir, "bench_digests.json")) as f:
        ref = json.load(f)["sha256_by_packets"][str(n)]
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == ref
    bad = torch.arange(0, n, 4099, device="cuda")
    pos = bad * stride + 16 + (bad % 1456)
    wire[pos] = wire[pos] ^ 1
    ok.zero_()
    W.verify_batch(wire, stride, wl, n, ok, None)
    torch.cuda.synchronize()
    okh = ok.cpu().numpy()
    assert set(np.nonzero(okh == 0)[0].tolist()) == set(bad.cpu().numpy().tolist())


def test_host_verify(W):
    rng = np.random.default_rng(4)
    n, stride = 500, 1472
    buf, rl = _datagrams(n, stride, rng)
    buf[5 * stride + 30] ^= 4
    ok, crc = W.host_verify(buf, stride, rl)
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    assert np.array_equal(ok, want_ok) and np.array_equal(crc, want_crc)


def test_host_verify_pinned_ring(W):
    """wReceiver's path: a pinned (wtp_host_alloc) 1472-B ring is copied to the device
    directly and verified by the braided kernel + fix-up; the recv_len array is pinned
    too.  Includes runts, short, oversize and corrupted datagrams."""
    rng = np.random.default_rng(21)
    n, stride = 2500, 1472
    buf, rl = _full_ring(n, stride, rng, 0.85)
    ring = W.PinnedBuffer(n * stride)
    ring.array[:] = buf
    lens = W.PinnedBuffer(n * 4)
    la = lens.array.view(np.uint32)
    la[:] = rl
    ok, crc = W.host_verify(ring.array, stride, la)
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    assert np.array_equal(ok, want_ok) and np.array_equal(crc, want_crc)
    ring.free()
    lens.free()


@pytest.mark.parametrize("zero_copy", ["1", "0"])
@pytest.mark.parametrize("n,stride,skip", [(10, 1504, 0), (64, 1472, 3), (700, 1472, 17), (2800, 1472, 1), (300, 1500, 5)])
def test_host_verify_pinned_small_batches(W, zero_copy, n, stride, skip):
    """Window-size batches from a pinned ring: rings up to 1 MiB are read by the kernel in
    place (zero copy, WTP_HOST_ZEROCOPY unset) or through the copy pipeline (=0); the
    ring and the lengths start `skip` slots into their pinned allocations (wReceiver hands
    the library a batch inside its ring); a 1500-B stride takes the general kernel."""
    rng = np.random.default_rng(n + stride)
    buf, rl = _full_ring(n, stride, rng, 0.85)
    ring = W.PinnedBuffer((n + skip) * stride)
    ring.array[skip * stride:] = buf
    lens = W.PinnedBuffer((n + skip) * 4)
    la = lens.array.view(np.uint32)
    la[skip:] = rl
    os.environ["WTP_HOST_ZEROCOPY"] = zero_copy
    try:
        ok, crc = W.host_verify(ring.array[skip * stride:], stride, la[skip:])
    finally:
        del os.environ["WTP_HOST_ZEROCOPY"]
    want_ok, want_crc = O.verify_datagrams(buf, stride, rl)
    assert np.array_equal(ok, want_ok) and np.array_equal(crc, want_crc)
    ring.free()
    lens.free()


def test_build_data_packets(W):
    for total in (64, 1456, 2216, 10202, 1456 * 300 + 17):
        host = O.synth_fill_np(total, start_byte=total)
        d = dev_u8(np.concatenate([host, np.zeros(16, np.uint8)]))
        nch = (total + 1455) // 1456
        wire = torch.zeros(nch * 1472, dtype=torch.uint8, device="cuda")
        wl = u32_out(nch)
        W.build_data_packets(d, total, 7, wire, 1472, wl)
        torch.cuda.synchronize()
        w = wire.cpu().numpy()
        lens = to_u32(wl, nch)
        for i in range(nch):
            p = host[i * 1456:(i + 1) * 1456].tobytes()
            want = O.build_datagram(7 + i, p)
            assert lens[i] == len(want)
            assert w[i * 1472:i * 1472 + len(want)].tobytes() == want, (total, i)


@pytest.mark.parametrize("total,stride,pay_off,wire_off,with_len,seq0", [
    (1456 * 5000 + 333, 1472, 0, 0, True, 0),          # fused path + short tail
    (1456 * 4099, 1472, 0, 0, False, 0xFFFFFFF0),      # fused, no tail, no lengths, seq wraps
    (1456 * 777 + 1, 1488, 0, 0, True, 3),             # fused, wider 16-B slots
    (1456 * 513 + 1000, 1500, 0, 0, True, 9),          # slot stride % 16 != 0: three-step path
    (1456 * 300 + 17, 1472, 4, 0, True, 1),            # unaligned payloads: three-step path
    (1456 * 300, 1472, 0, 8, False, 2),                # unaligned wire: three-step path
])
def test_build_data_packets_paths(W, total, stride, pay_off, wire_off, with_len, seq0):
    host = O.synth_fill_np(total, start_byte=total + stride)
    raw = np.zeros(total + pay_off + 16, np.uint8)
    raw[pay_off:pay_off + total] = host
    d = dev_u8(raw)[pay_off:]
    nch = (total + 1455) // 1456
    wraw = torch.full((nch * stride + wire_off,), 0xA5, dtype=torch.uint8, device="cuda")
    wire = wraw[wire_off:]
    wl = u32_out(nch) if with_len else None
    W.build_data_packets(d, total, seq0, wire, stride, wl)
    torch.cuda.synchronize()
    w = wire.cpu().numpy()
    lens = to_u32(wl, nch) if with_len else None
    for i in list(range(min(nch, 40))) + list(range(max(40, nch - 40), nch)):
        p = host[i * 1456:(i + 1) * 1456].tobytes()
        want = O.build_datagram((seq0 + i) & 0xFFFFFFFF, p)
        if with_len:
            assert lens[i] == len(want)
        got = w[i * stride:i * stride + len(want)].tobytes()
        assert got == want, (i, got[:16].hex(), want[:16].hex())
        assert (w[i * stride + len(want):(i + 1) * stride] == 0xA5).all()  # slot tail untouched
    # every header's checksum vs an independent device CRC of the payload buffer
    full = total // 1456
    crcs = u32_out(full)
    W.crc32_batch_fixed(d, 1456, 1456, full, crcs)
    c = to_u32(crcs, full)
    hdr = w[:full * stride].reshape(full, stride)[:, 12:16]
    assert np.array_equal(hdr.copy().view(">u4").ravel(), c)


@pytest.mark.parametrize("total,stride,pin_src,pin_wire,with_len,seq0", [
    (1456 * 50000 + 333, 1472, False, False, True, 5),   # two slabs, pageable both ways, short tail
    (1456 * 50000 + 333, 1472, True, True, True, 5),     # two slabs, pinned both ways (DMA in place)
    (1456 * 1000, 1488, True, False, False, 0xFFFFFFF0),  # wider slots, no lengths, seq wraps
    (1456 * 10 + 1, 1500, False, True, True, 1),         # stride % 16 != 0: the three-step path
    (100, 1472, True, True, True, 0),                    # one short datagram
    (1456 * 100 + 5, 1500, True, True, True, 7),         # zero copy into 1500-B slots: the three-step path over host memory
])
@pytest.mark.parametrize("zero_copy", ["1", "0"])
def test_host_build_data_packets(W, total, stride, pin_src, pin_wire, with_len, seq0, zero_copy):
    """wtp_host_build_data_packets (wSender --crc gpu) against the device builder on the same
    payloads (itself checked against the oracle above) and the oracle on sampled chunks.
    Pinned both ways the builder works on host memory in place unless
    WTP_HOST_BUILD_ZEROCOPY=0, which sends it through the device slabs."""
    if zero_copy == "0" and not (pin_src and pin_wire):
        pytest.skip("the zero-copy switch only matters when both buffers are pinned")
    host = O.synth_fill_np(total, start_byte=total ^ stride)
    nch = (total + 1455) // 1456
    bufs = []
    if pin_src:
        pb = W.PinnedBuffer(total)
        pb.array[:] = host
        src = pb.array
        bufs.append(pb)
    else:
        src = host
    wire = wl = None
    if pin_wire:
        pw = W.PinnedBuffer(nch * stride)
        pl = W.PinnedBuffer(nch * 4)
        wire, wl = pw.array, pl.array.view(np.uint32)
        bufs += [pw, pl]
    if not with_len:
        wl = None
    os.environ["WTP_HOST_BUILD_ZEROCOPY"] = zero_copy
    try:
        got, got_len = W.host_build_data_packets(src, seq0, stride, wire=wire, wire_len=wl) if with_len else (
            W.host_build_data_packets(src, seq0, stride, wire=wire)[0], None)
    finally:
        del os.environ["WTP_HOST_BUILD_ZEROCOPY"]
    got = got[:nch * stride].reshape(nch, stride)
    d = dev_u8(host)
    dw = torch.zeros(nch * stride, dtype=torch.uint8, device="cuda")
    dl = u32_out(nch)
    W.build_data_packets(d, total, seq0, dw, stride, dl)
    torch.cuda.synchronize()
    want = dw.cpu().numpy().reshape(nch, stride)
    want_len = to_u32(dl, nch)
    last = int(want_len[-1])
    assert np.array_equal(got[:-1, :1472], want[:-1, :1472])
    assert np.array_equal(got[-1, :last], want[-1, :last])
    if with_len:
        assert np.array_equal(np.asarray(got_len[:nch]), want_len)
    for i in sorted({0, min(1, nch - 1), nch // 2, nch - 1}):
        p = host[i * 1456:(i + 1) * 1456].tobytes()
        dg = O.build_datagram((seq0 + i) & 0xFFFFFFFF, p)
        assert got[i, :len(dg)].tobytes() == dg, i
    for b in bufs:
        b.free()


def test_host_chunked_pageable_and_pinned(W):
    nbytes = 40 * (1 << 20) + 64  # crosses slab boundaries? (64 MiB slabs) keep moderate
    host = O.synth_fill_np(nbytes, start_byte=5)
    got = W.host_chunked(host, 1456)
    want = O.batch_fixed(np.concatenate([host, np.zeros(1456, np.uint8)]), 1456, 1456, got.size - 1, threads=8)
    assert np.array_equal(got[:-1], want)
    assert got[-1] == O.crc32(host[(got.size - 1) * 1456:])
    pb = W.PinnedBuffer(nbytes)
    pb.array[:] = host
    got2 = W.host_chunked(pb.array, 1456)
    assert np.array_equal(got2, got)
    pb.free()


@pytest.mark.parametrize("parts", [2, 3, 4, 5, 6])
def test_host_chunked_pageable_staging_split(W, parts):
    """Pageable sources are staged into the pinned slab by up to 6 threads, one part each
    (kMinPart = 8 MiB).  Sizes parts * 8 MiB + r (0 < r < parts) make floor(bytes / parts)
    page-aligned while bytes % parts != 0: the last r bytes, i.e. the tail of the last
    chunk, must still be copied (they were left stale)."""
    for r in sorted({1, parts - 1}):
        nbytes = parts * (8 << 20) + r
        host = O.synth_fill_np(nbytes, start_byte=parts * 131 + r)
        # run twice with different tails in between: stale slab bytes would show up
        for rep in range(2):
            host[-1] ^= np.uint8(0x5A * (rep + 1))
            got = W.host_chunked(host, 1456)
            n = got.size
            assert got[-1] == O.crc32(host[(n - 1) * 1456:]), (parts, r, rep)
            assert got[0] == O.crc32(host[:1456])
        idx = np.arange(0, n - 1, 997)
        want = [O.crc32(host[i * 1456:(i + 1) * 1456]) for i in idx]
        assert np.array_equal(got[idx], np.array(want, np.uint32))


def test_c3_1gib_host_chunked_elementwise(W):
    """Config C3 at full size: a 1 GiB host file (2^30 B -> 737,461 chunks, the last one
    64 B) through the pinned H2D -> CRC -> D2H pipeline, pageable and pinned sources,
    every chunk vs the oracle (Sender.cpp:89-92 chunking, Crc32.hpp:91-102)."""
    nbytes = 1 << 30
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    W.synth_fill(dev, start_byte=3)
    host = dev.cpu().numpy()
    del dev
    assert np.array_equal(host[-4096:], O.synth_fill_np(4096, start_byte=3 + nbytes - 4096))
    n = (nbytes + 1455) // 1456
    assert n == 737_461 and nbytes - (n - 1) * 1456 == 64
    want = np.empty(n, np.uint32)
    want[:-1] = O.batch_fixed(host, 1456, 1456, n - 1, threads=THREADS)
    want[-1] = O.crc32(host[(n - 1) * 1456:])
    got = W.host_chunked(host, 1456)
    bad = np.nonzero(got != want)[0]
    assert got.size == n and bad.size == 0, (bad.size, bad[:5])
    pb = W.PinnedBuffer(nbytes)
    pb.array[:] = host
    got2 = W.host_chunked(pb.array, 1456)
    pb.free()
    assert np.array_equal(got2, want)


@pytest.mark.parametrize("devices", [None, [0], [0, 0, 0]])
def test_host_chunked_multi(W, devices):
    """wtp_crc32_host_chunked_multi: chunks split over devices (one pipeline thread per
    entry; [0, 0, 0] runs three range threads through device 0's pipeline), the last
    chunk short, vs the oracle element-wise."""
    nbytes = 200 * (1 << 20) + 777  # > 3 slabs
    host = O.synth_fill_np(nbytes, start_byte=11)
    got = W.host_chunked_multi(host, 1456, devices=devices)
    n = (nbytes + 1455) // 1456
    want = np.empty(n, np.uint32)
    want[:-1] = O.batch_fixed(host, 1456, 1456, n - 1, threads=THREADS)
    want[-1] = O.crc32(host[(n - 1) * 1456:])
    assert np.array_equal(got, want)
    dev = torch.cuda.current_device()
    assert dev == 0  # the caller's device is unchanged


def test_host_error_mid_call_then_correct_call(W):
    """A host wrapper that fails after its first H2D was queued waits for its copies
    before returning (the next call reuses the same pinned slabs); the next call is
    exact element-wise."""
    host = O.synth_fill_np(5000 * 300, start_byte=9)
    with pytest.raises(W.WtpError):
        W.host_batch_fixed(host, 5000, 4500, 300)  # len > 4096: fails after the first slab's H2D
    with pytest.raises(W.WtpError):
        W.host_chunked_multi(host, 4500, devices=[0, 0])
    big = O.synth_fill_np(100 * (1 << 20), start_byte=1)
    got = W.host_chunked(big, 1456)
    n = got.size
    want = np.empty(n, np.uint32)
    want[:-1] = O.batch_fixed(big, 1456, 1456, n - 1, threads=THREADS)
    want[-1] = O.crc32(big[(n - 1) * 1456:])
    assert np.array_equal(got, want)


def test_host_batch_fixed_odd_stride(W):
    host = O.synth_fill_np(1001 * 999 + 10)
    got = W.host_batch_fixed(host, 1001, 999, 999)
    assert np.array_equal(got, O.batch_fixed(host, 1001, 999, 999))


# ---- full target size through properties ------------------------------------------------
def test_target_1m_elementwise(W, golden_dir):
    """The headline batch (1 M x 1456 B, braided kernel): all 1,048,576 CRCs vs the
    oracle, and the vector's digest vs the reference's own (bench_digests.json)."""
    import hashlib
    import json
    n = 1 << 20
    buf = torch.empty(n * 1456, dtype=torch.uint8, device="cuda")
    W.synth_fill(buf)
    fast = u32_out(n)
    W.crc32_batch_fixed(buf, 1456, 1456, n, fast)
    a = to_u32(fast, n)
    host = buf.cpu().numpy()
    for off in (0, host.size // 2, host.size - (1 << 20)):
        assert np.array_equal(host[off:off + (1 << 20)], O.synth_fill_np(1 << 20, start_byte=off)), off
    want = O.batch_fixed(host, 1456, 1456, n, threads=THREADS)
    bad = np.nonzero(a != want)[0]
    assert bad.size == 0, (bad.size, bad[:5])
    with open(os.path.join(golden_dir, "bench_digests.json")) as f:
        ref = json.load(f)["sha256_by_packets"][str(n)]
    assert hashlib.sha256(a.astype("<u4").tobytes()).hexdigest() == ref
    # the general kernel on the same bytes (different algorithm) agrees too
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * 1456
    lens = torch.full((n,), 1456, dtype=torch.int32, device="cuda")
    gen = u32_out(n)
    W.crc32_batch_var(buf, n * 1456, offs, lens, n, gen)
    assert np.array_equal(to_u32(gen, n), a)
    # idempotence: a second launch gives the same bytes
    W.crc32_batch_fixed(buf, 1456, 1456, n, fast)
    assert np.array_equal(to_u32(fast, n), a)


def test_errors_are_loud(W):
    out = u32_out(4)
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(W.WtpError):
        W.crc32_batch_fixed(buf, 8192, 8192, 4, out)
    with pytest.raises(W.WtpError):
        W.verify_batch(buf, 8, torch.zeros(4, dtype=torch.int32, device="cuda"), 4,
                       torch.zeros(4, dtype=torch.uint8, device="cuda"))


@pytest.mark.parametrize("lead", [16, 32, 48, 64, 80, 96, 112])
def test_fast_path_frame_placements(W, lead):
    # every 16-B base offset modulo 128 exercises a different braid frame placement
    for L, stride in ((1456, 1456), (1456, 1472), (256, 272), (1536, 1536), (16, 16), (1296, 1312)):
        n = 333
        host = O.synth_fill_np(lead + n * stride + 16, start_byte=lead + L)
        d = dev_u8(host)
        out = u32_out(n)
        W.crc32_batch_fixed(d[lead:], stride, L, n, out)
        assert np.array_equal(to_u32(out, n), O.batch_fixed(host[lead:], stride, L, n)), (L, stride)


# ---- size-independent properties at full config sizes -----------------------------------
# CRC-32 is affine over GF(2): for equal-length messages x, y,
#   crc(x ^ y) = crc(x) ^ crc(y) ^ crc(0^len).
# Checked for EVERY packet at C4's per-rank size and for C5's distribution below and past
# 2 GiB (device-only, so nothing is sampled), with crc(0^len) itself pinned to the oracle
# for every length that occurs (1456 x 0x00 -> 0x16BCBC70 is a reference KAT).
def _xor_pair(nbytes, seeds=(0x5EED, 0xC0FFEE)):
    a = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    b = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    import wtp_crc32 as W
    W.synth_fill(a, seed=seeds[0], nbytes=nbytes)
    W.synth_fill(b, seed=seeds[1], nbytes=nbytes)
    c = torch.bitwise_xor(a, b)
    z = torch.zeros_like(a)
    return a, b, c, z


def test_linearity_c4_rank_shard_every_packet(W):
    """C4's per-rank shard, 2,097,152 x 1456 B (3.05 GB; the held-results braided launch):
    crc(A ^ B) == crc(A) ^ crc(B) ^ crc(0) for all 2 M packets, crc(0) == 0x16BCBC70."""
    n = 2_097_152
    bufs = _xor_pair(n * 1456)
    outs = []
    for t in bufs:
        o = u32_out(n)
        W.crc32_batch_fixed(t, 1456, 1456, n, o)
        outs.append(o)
    assert W.LIB.wtp_last_kernel().decode() == "k_fixed_braid<6, 0, CrcHoldBEpi>"
    a, b, c, z = outs
    assert torch.equal(torch.bitwise_xor(torch.bitwise_xor(a, b), z), c)
    zu = to_u32(z, n)
    assert (zu == np.uint32(0x16BCBC70)).all() and O.crc32(bytes(1456)) == 0x16BCBC70
    assert not torch.equal(a, b)
    del bufs


@pytest.mark.parametrize("n", [1 << 20, 17_000_000])
def test_linearity_zipf_packed_every_payload(W, n):
    """C5's Zipf(1.1) lengths, packed: 1 M payloads (one piece launch) and 17 M (2.3 GB: the
    device-cut sub-launches past 2 GiB).  Every payload: crc(A ^ B) == crc(A) ^ crc(B) ^
    crc(0^len), and crc(0^len) equal to the oracle's for each distinct length."""
    lens = O.zipf_lengths(n, s=1.1).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum())
    bufs = _xor_pair(total)
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    outs = []
    for t in bufs:
        o = u32_out(n)
        W.crc32_batch_packed(t, total, do, dl, n, o)
        outs.append(o)
    if total + 64 >= (1 << 31):
        assert W.LIB.wtp_last_kernel().decode().startswith("k_pieces<RangeArrayProvL")
    a, b, c, z = outs
    assert torch.equal(torch.bitwise_xor(torch.bitwise_xor(a, b), z), c)
    zu = to_u32(z, n)
    for L in np.unique(lens):
        first = int(np.argmax(lens == L))
        assert int(zu[first]) == O.crc32(bytes(int(L))), L
    # every payload of one length has the same crc(0^len)
    order = np.argsort(lens, kind="stable")
    ls, zs = lens[order], zu[order]
    starts = np.concatenate([[True], ls[1:] != ls[:-1]])
    assert np.array_equal(zs, np.repeat(zs[starts], np.diff(np.concatenate([np.nonzero(starts)[0], [n]]))))
    del bufs
