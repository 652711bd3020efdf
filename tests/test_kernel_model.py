"""CPU check of the kernels' algebra through tests/kernel_model.py (no GPU needed)."""
import numpy as np
import pytest

import oracle as O
import kernel_model as KM
from kernel_model import Tables, braid_crc, pieces_crc


@pytest.fixture(scope="module")
def T():
    return Tables()


@pytest.mark.parametrize("L", [16, 32, 240, 256, 272, 1280, 1296, 1456, 1536])
def test_braid_model(T, L):
    for seed_off in (0, 77777):
        pkt = O.synth_fill_np(L, start_byte=seed_off + L).tobytes()
        for addr in range(0, 256, 16):  # every frame placement case
            assert braid_crc(T, pkt, addr) == O.crc32(pkt), (L, addr)


@pytest.mark.parametrize("L", [0, 1, 3, 4, 5, 63, 64, 65, 127, 128, 129, 700, 1455, 1456, 1484, 4096])
def test_pieces_model(T, L):
    buf = O.synth_fill_np(L + 200, start_byte=3 * L).tobytes()
    for off in (0, 1, 5, 13, 100):
        if off + L <= len(buf):
            assert pieces_crc(T, buf, off, L) == O.crc32(buf[off:off + L]), (L, off)


@pytest.mark.parametrize("case", ["packed_zipf", "strided_odd", "scattered", "dgram", "edge_start", "big"])
def test_pieces_rounds_model(T, case):
    """Round-level model of k_pieces (piece stream, carry across rounds, speculative
    span prefetch, padded LDS staging) against the oracle."""
    from kernel_model import pieces_rounds
    rng = np.random.default_rng(7)
    if case == "packed_zipf":
        lens = O.zipf_lengths(300, s=1.0)
        offs = np.concatenate([[0], np.cumsum(lens[:-1])]) + 5
    elif case == "strided_odd":
        lens = np.full(40, 1457 - 8, dtype=np.int64)
        offs = 3 + 1457 * np.arange(40)
    elif case == "scattered":
        lens = rng.integers(0, 200, 200)
        offs = rng.permutation(200) * 300 + rng.integers(0, 16, 200)
    elif case == "dgram":
        lens = np.array([1456, 0, 700, 1456, 33, 1456, 1456] * 8)
        offs = 1472 * np.arange(len(lens)) + 16
    elif case == "big":  # 4096-B packets: 64 pieces each, every round one whole packet
        lens = np.array([4096, 4095, 4033, 4096, 1, 4096])
        offs = np.concatenate([[0], np.cumsum(lens[:-1])]) + 9
    else:  # packets at the very start and end of the buffer, lengths 0/1/64/4096
        lens = np.array([1, 64, 0, 4096, 63, 65, 2, 4096, 1456])
        offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    offs = [int(o) for o in offs]
    lens = [int(v) for v in lens]
    nbytes = max(o + v for o, v in zip(offs, lens)) + 7
    buf = O.synth_fill_np(nbytes, start_byte=11).tobytes()
    got, rounds, hits = pieces_rounds(T, buf, offs, lens, rng)
    want = [O.crc32(buf[o:o + v]) for o, v in zip(offs, lens)]
    assert got == want
    if case in ("packed_zipf", "strided_odd"):
        assert hits == rounds - 1  # every round after the first is prefetched


@pytest.mark.parametrize("case", ["zipf", "tiny", "long_4095", "one", "empty_mix"])
def test_stream_model(case):
    """k_stream's algebra (prefix values, block anchors, feed, nibble length shift) on
    packed batches at several view alignments, vs the oracle."""
    import kernel_model as K
    T = K.StreamTables()
    rng = np.random.default_rng(len(case))
    n = {"one": 1, "long_4095": 12}.get(case, 150)
    if case == "zipf":
        lens = O.zipf_lengths(n, s=1.1)
    elif case == "tiny":
        lens = rng.integers(0, 4, n)
    elif case == "long_4095":
        lens = np.full(n, 4095)
    elif case == "one":
        lens = np.array([33])
    else:
        lens = np.where(rng.random(n) < 0.5, 0, rng.integers(1, 300, n))
    for first, view_addr in ((0, 0), (77, 16), (130, 48)):
        offs = first + np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
        buf = O.synth_fill_np(int(offs[-1] + lens[-1]) + 9, start_byte=first).tobytes()
        out, _ = K.stream_wave(T, buf, offs, lens, view_addr=view_addr)
        assert out == [O.crc32(buf[o:o + L]) for o, L in zip(offs, lens)], (case, first)


@pytest.mark.parametrize("G,sb,lead", [(4096, 10**9, 0), (3000, 37, 5), (50_000, 100, 11), (1 << 20, 64, 3)])
def test_cut_ranges_partition_and_views(G, sb, lead):
    """k_cut_ranges (mirrored at small G and sub-batch sizes): the sub-launches partition
    [0, n) in order, none holds more than sb packets, a packed batch's ranges each fit a
    view of G + 4 KiB (nothing outside, so no fallback), and a batch with swapped payloads
    still partitions, its out-of-view packets being exactly those the fallback must redo."""
    rng = np.random.default_rng(G + sb)
    n = 5000
    lens = rng.integers(0, 4097, n).astype(np.int64)
    lens[rng.integers(0, n, 200)] = 0
    offs = np.concatenate([[3], 3 + np.cumsum(lens[:-1])]).astype(np.int64)
    vspan = (lead + int(offs[-1] + lens[-1]) + 15) & ~15
    for broken in (False, True):
        o = offs.copy()
        if broken:
            for b in rng.choice(n - 1, 30, replace=False):
                o[[b, b + 1]] = o[[b + 1, b]]
        rs = KM.cut_ranges(o, n, lead, vspan, G, sb)
        assert len(rs) == -(-vspan // G) + -(-n // sb) - 1
        assert rs[0]["begin"] == 0 and rs[-1]["end"] == n
        assert all(a["end"] == b["begin"] for a, b in zip(rs, rs[1:]))
        assert all(r["end"] - r["begin"] <= sb for r in rs)
        outside = [p for r in rs if r["begin"] < r["end"] for p in KM.range_outside(r, o, lens, lead)]
        if not broken:
            assert not outside and not any(r["bad"] for r in rs)
            for r in rs:
                if r["begin"] < r["end"]:
                    end = max(int(o[p] + lens[p]) for p in range(r["begin"], r["end"])) + lead
                    assert end - r["rebase"] <= G + 4096 + 16
