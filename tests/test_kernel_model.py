"""CPU check of the kernels' algebra through tests/kernel_model.py (no GPU needed)."""
import numpy as np
import pytest

import oracle as O
from kernel_model import LaneTables, Tables, braid_crc, lane_parts, pieces_crc, var_lane_combine, var_lane_group


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




def test_var_lane_model():
    """k_var_lane's part split, frame/mask/braid/fold and part combine algebra: lengths up
    to 4096 B (up to 17 parts), every start alignment, tasks of different sizes in one
    group."""
    LT = LaneTables()
    rng = np.random.default_rng(5)
    view = O.synth_fill_np(16384, start_byte=77).tobytes()
    lens = list(range(1, 40)) + [127, 128, 129, 255, 256, 257, 271, 272, 273, 700, 1455, 1456, 1521, 1536, 4095, 4096]
    for L in lens:
        pk = [(int(o), L) for o in rng.integers(0, 8192, 4)] + [(o, L) for o in range(16)]
        pk += [(int(o), int(l)) for o, l in zip(rng.integers(0, 8192, 3), rng.integers(1, L + 1, 3))]
        tasks = [(vo, l, j, sp, ep) for vo, l in pk for j, sp, ep in lane_parts(vo, l)]
        assert all(((ep - sp) >> 4) <= 16 for *_, sp, ep in tasks)
        vals = var_lane_group(LT, view, tasks)
        k = 0
        for vo, l in pk:
            m = len(lane_parts(vo, l))
            assert var_lane_combine(LT, vo, l, vals[k:k + m]) == O.crc32(view[vo:vo + l]), (vo, l)
            k += m


def test_mixed_model():
    """k_mixed's algebra: end-aligned frames with forward operators only, the short
    (lane per packet) and long (16 lanes, R rows) paths, packets at every start offset
    including the view's first 15 bytes (negative chunk offsets), extra leading rows."""
    from kernel_model import MX_TH, MixedTables, mixed_long_crc, mixed_short_crc
    MT = MixedTables()
    view = O.synth_fill_np(9000, start_byte=5).tobytes()
    rng = np.random.default_rng(9)
    for L in [0, 1, 2, 15, 16, 17, 100, 16 * MX_TH]:
        for s in list(range(0, 18)) + [int(x) for x in rng.integers(0, 8000, 3)]:
            assert mixed_short_crc(MT, view, s, L) == O.crc32(view[s:s + L]), (s, L)
    for L in [4, 5, 17, 65, 129, 255, 256, 257, 700, 1456, 4096]:
        for s in [0, 1, 7, 12, 13, 14, 15, 16, 33] + [int(x) for x in rng.integers(0, 4800, 2)]:
            R = (L + 255) // 256
            for extra in (0, 1):
                assert mixed_long_crc(MT, view, s, L, R + extra) == O.crc32(view[s:s + L]), (s, L, extra)
