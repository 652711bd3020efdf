"""Bit-level CPU model of the two HIP kernels' algorithms (TEST INFRASTRUCTURE).

It mirrors csrc/crc32_kernels.hip step for step — braid tables, x^(-32k) folds,
cross-lane tree, piece windows, segmented scan — using tables built with the oracle's
shift/unshift, so an algebra mistake shows up here, on CPU, before any GPU time.
It is not the product and is never imported by it.
"""
from __future__ import annotations

import numpy as np

import oracle as O

G = 16
BRAID_BLOCK = 256
S = 64


def _word_tables(block: int) -> np.ndarray:
    t = O.table()
    out = np.zeros((4, 256), dtype=np.uint32)
    for k in range(4):
        for e in range(256):
            out[k, e] = O.shift(int(t[e]), block - 1 - k)
    return out


def _operator(f) -> np.ndarray:
    out = np.zeros((4, 256), dtype=np.uint32)
    for k in range(4):
        for b in range(256):
            out[k, b] = f(b << (8 * k))
    return out


def _apply(tab: np.ndarray, v: int) -> int:
    return int(tab[0, v & 255] ^ tab[1, (v >> 8) & 255] ^ tab[2, (v >> 16) & 255] ^ tab[3, v >> 24])


class Tables:
    def __init__(self):
        self.braid = _word_tables(BRAID_BLOCK)
        self.inv = {n: _operator(lambda v, n=n: O.unshift(v, n)) for n in (4, 8, 16, 32, 64, 128)}
        self.s4 = _word_tables(4)
        self.fwd = {d: _operator(lambda v, d=d: O.shift(v, S * d)) for d in (1, 2, 4, 8, 16, 32)}

    @staticmethod
    def init_const(L: int) -> int:
        return O.shift(0xFFFFFFFF, L) ^ 0xFFFFFFFF


def frame_start(st: int, L: int, rows: int) -> int:
    """Frame placement of k_fixed_braid: 128-B aligned if the frame still covers the
    packet end, else 64-B aligned, else right-aligned to the packet end."""
    frame = 256 * rows
    en = st + L
    for a in (128, 64):
        fs = st - st % a
        if fs + frame >= en:
            return fs
    return en - frame


def braid_crc(T: Tables, pkt: bytes, addr: int = 0) -> int:
    """k_fixed_braid for one packet (len % 16 == 0, 16 <= len <= 1536) starting at
    device address `addr` (16-B aligned)."""
    L = len(pkt)
    rows = (L + 255) // 256
    fs = frame_start(addr, L, rows)
    lead = addr - fs
    trail = fs + rows * 256 - (addr + L)  # T: zero bytes after the packet, undone below
    frame = b"\0" * lead + pkt + b"\0" * trail
    assert len(frame) == rows * 256
    B = [[0, 0, 0, 0] for _ in range(G)]
    for i in range(rows):
        for j in range(G):
            c = (i * G + j) * 16
            for k in range(4):
                w = int.from_bytes(frame[c + 4 * k:c + 4 * k + 4], "little")
                B[j][k] = _apply(T.braid, B[j][k] ^ w)
    v = [B[j][0] ^ _apply(T.inv[4], B[j][1]) ^ _apply(T.inv[8], B[j][2] ^ _apply(T.inv[4], B[j][3]))
         for j in range(G)]
    d = 1
    while d < G:
        nv = list(v)
        for j in range(G):
            u = v[j + d] if j + d < G else v[j]
            if j & (2 * d - 1) == 0:
                nv[j] = v[j] ^ _apply(T.inv[16 * d], u)
        v = nv
        d *= 2
    r = v[0]
    t = trail // 16
    for bit, n in ((1, 16), (2, 32), (4, 64), (8, 128)):
        if t & bit:
            r = _apply(T.inv[n], r)
    return r ^ T.init_const(L)


def pieces_crc(T: Tables, buf: bytes, off: int, L: int) -> int:
    """k_pieces for one packet: 64-B windows counted back from the end, segmented scan."""
    K = 1 if L == 0 else (L + S - 1) // S
    vals = []
    for piece in range(K):
        we = off + L - (K - 1 - piece) * S
        ws = we - S
        window = bytearray(S)
        for t in range(S):
            g = ws + t
            if off <= g < off + L:  # bytes before the packet are masked to zero
                window[t] = buf[g]
        c = 0
        for i in range(16):
            c = _apply(T.s4, c ^ int.from_bytes(window[4 * i:4 * i + 4], "little"))
        vals.append(c)
    W = list(vals)
    d = 1
    while d < 64:
        nW = list(W)
        for i in range(K):
            if i >= d:
                nW[i] = _apply(T.fwd[d], W[i - d]) ^ W[i]
        W = nW
        d *= 2
    return W[K - 1] ^ T.init_const(L)
