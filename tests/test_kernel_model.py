"""CPU check of the kernels' algebra through tests/kernel_model.py (no GPU needed)."""
import numpy as np
import pytest

import oracle as O
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
