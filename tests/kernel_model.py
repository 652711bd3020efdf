"""Bit-level CPU model of the two HIP kernels' algorithms (TEST INFRASTRUCTURE).

It mirrors csrc/crc32_kernels.hip step for step — braid tables with the next word
folded into the lookup XOR, the in-lane x^-32 Horner fold, the Horner flush over the
transposition slot (two halves of 8 columns, x^-1024, masked x^-128 trailing steps),
piece windows, segmented scan — using tables built with the oracle's
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
        self.inv = {n: _operator(lambda v, n=n: O.unshift(v, n)) for n in (1, 4, 8, 16, 32, 64, 128)}
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
    # main loop: b <- B ^ w of the current row; b <- T(b) ^ w_next; the last row applies T
    b = [[int.from_bytes(frame[j * 16 + 4 * k:j * 16 + 4 * k + 4], "little") for k in range(4)] for j in range(G)]
    for i in range(1, rows):
        for j in range(G):
            c = (i * G + j) * 16
            for k in range(4):
                w = int.from_bytes(frame[c + 4 * k:c + 4 * k + 4], "little")
                b[j][k] = _apply(T.braid, b[j][k]) ^ w
    # (the last row's advance T is deferred to the flush: it commutes with every x^-k)
    # in-lane fold: v_j = b0 ^ x^-32 (b1 ^ x^-32 (b2 ^ x^-32 b3))
    v = []
    for j in range(G):
        x = _apply(T.inv[4], b[j][3]) ^ b[j][2]
        x = _apply(T.inv[4], x) ^ b[j][1]
        v.append(_apply(T.inv[4], x) ^ b[j][0])
    # flush: lane h takes columns 8h .. 8h+7 (Horner with x^-128), h = 1 moved by
    # x^-1024, both take t masked x^-128 steps (t = trailing zero chunks), then XOR
    t = trail // 16
    tmax = (rows * 256 - L) // 16
    halves = []
    for h in (0, 1):
        acc = v[8 * h + 7]
        for jj in range(6, -1, -1):
            acc = _apply(T.inv[16], acc) ^ v[8 * h + jj]
        if h:
            acc = _apply(T.inv[128], acc)
        for s2 in range(tmax):
            if s2 < t:
                acc = _apply(T.inv[16], acc)
        halves.append(acc)
    return _apply(T.braid, halves[0] ^ halves[1]) ^ T.init_const(L)


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


# ---- k_pieces round structure (staging + lane assignment) --------------------------
PC_CHUNKS = 272
PC_SLOT = 4640
SPAN = 16 * PC_CHUNKS


def stage_addr(chunk: int) -> int:
    return 16 * (chunk + (chunk >> 4))


def pieces_rounds(T: Tables, buf: bytes, offs, lens, rng=None):
    """One wave of k_pieces over packets (offs[i], lens[i]) of `buf` (the 16-B aligned
    view; reads outside it return 0 as the buffer resource does).  Mirrors the round
    loop of csrc/crc32_kernels.hip: the piece stream with carry/skip across rounds, the
    round cut at the first window outside the slot span, the speculative span prefetch
    (hit/miss), lane-contiguous staging into a padded slot that still holds older bytes,
    5 x 16-B window reads, masking, the head-init table, chain and segmented scan.
    Returns (crcs, rounds, hits)."""
    rng = rng or np.random.default_rng(0)
    buf = bytes(buf) + bytes(-len(buf) % 16)  # the host rounds the resource up to 16 B
    nb = len(buf)
    hinit = [O.shift(0xFFFFFFFF, h) for h in range(S + 1)]

    def rd16(o):  # raw buffer load of 16 B at u32 offset o
        o &= 0xFFFFFFFF
        return bytes(16) if o + 16 > nb else buf[o:o + 16]

    def load_span(b16):
        return [rd16(b16 + 16 * c) for c in range(PC_CHUNKS)]

    slot = bytearray(rng.integers(0, 256, PC_SLOT, dtype=np.uint8).tobytes())
    n = len(lens)
    out = [None] * n
    p0 = skip = carry = 0
    spec, x = None, None
    rounds = hits = 0
    while p0 < n:
        navail = min(64, n - p0)
        ks = [1 if lens[p0 + i] == 0 else (int(lens[p0 + i]) + S - 1) // S for i in range(navail)]
        kr = list(ks)
        kr[0] -= skip
        incl = list(np.cumsum(kr))
        lanes = []
        for lane in range(64):
            pk = sum(1 for j in range(navail) if incl[j] <= lane)
            if pk >= navail:
                lanes.append(None)
                continue
            lp = lane - (incl[pk] - kr[pk])
            gp = lp + (skip if pk == 0 else 0)
            off, L, K = int(offs[p0 + pk]), int(lens[p0 + pk]), ks[pk]
            we = off + L - (K - 1 - gp) * S
            lanes.append((pk, lp, gp, off, L, K, we - S, we))
        lo16 = lanes[0][6] & ~15
        total = 64
        for lane, v in enumerate(lanes):
            if v is None or v[6] < lo16 or v[7] - lo16 > SPAN:
                total = lane
                break
        assert total >= 1
        act = lanes[:total]
        hit = spec is not None and all(ws >= spec and we - spec <= SPAN for *_, ws, we in act)
        if hit:
            hits += 1
            sbase = spec
        else:
            x, sbase = load_span(lo16), lo16
        for c in range(PC_CHUNKS):
            a = stage_addr(c)
            assert a + 16 <= PC_SLOT
            slot[a:a + 16] = x[c]
        # next round (prefetch)
        pk_l, lp_l, gp_l, _, _, K_l, _, we_l = act[-1]
        partial = gp_l + 1 < K_l
        p0n = p0 + pk_l + (0 if partial else 1)
        spec = (we_l - S) & ~15 if p0n < n else None
        x = load_span(spec) if spec is not None else None
        vals = []
        for lane, (pk, lp, gp, off, L, K, ws, we) in enumerate(act):
            a = ws & 15
            blk = (ws - sbase) >> 4
            assert blk >= 0 and stage_addr(blk + 4) + 16 <= PC_SLOT
            raw = b"".join(bytes(slot[stage_addr(blk + u):stage_addr(blk + u) + 16]) for u in range(5))
            window = bytearray(raw[a:a + S])
            vf = min(off - ws, 64)
            for t in range(max(vf, 0)):
                window[t] = 0
            c = carry if lane == 0 else 0
            for i in range(16):
                c = _apply(T.s4, c ^ int.from_bytes(window[4 * i:4 * i + 4], "little"))
            if gp == 0:
                c ^= hinit[S - max(vf, 0)]
            vals.append(c)
        W = list(vals)
        d = 1
        while d < 64:
            nW = list(W)
            for i in range(total):
                if act[i][1] >= d:
                    nW[i] = _apply(T.fwd[d], W[i - d]) ^ W[i]
            W = nW
            d *= 2
        for i, (pk, lp, gp, off, L, K, ws, we) in enumerate(act):
            if gp == K - 1:
                out[p0 + pk] = W[i] ^ 0xFFFFFFFF
        carry = W[total - 1] if partial else 0
        skip = gp_l + 1 if partial else 0
        p0 = p0n
        rounds += 1
    return out, rounds, hits


# ---- k_stream: packed mixed-length payloads (payload p+1 starts where p ends) --------
ST_ROUND = 8192  # bytes per wave round: 64 lanes x 128 B
ST_LANE = 128
ST_BLK = 32


def nib_tables(f) -> np.ndarray:
    """A linear operator as 8 nibble tables of 16 words: N[i][e] = f(e << 4i)."""
    out = np.zeros((8, 16), dtype=np.uint32)
    for i in range(8):
        for e in range(16):
            out[i, e] = f(e << (4 * i))
    return out


def nib_apply(N: np.ndarray, v: int) -> int:
    r = 0
    for i in range(8):
        r ^= int(N[i, (v >> (4 * i)) & 15])
    return r


class StreamTables:
    """Tables of k_stream: slice-by-4 (advance 4 B), T256 (shift by one 32-B block),
    scan operators shift by 128 * 2^k B (k = 0..5), and the length shift in four
    3-bit levels: level k, digit j -> shift by j * 8^k bytes (lengths < 4096)."""

    def __init__(self):
        self.s4 = _word_tables(4)
        self.t256 = _operator(lambda v: O.shift(v, ST_BLK))
        self.scan = [nib_tables(lambda v, k=k: O.shift(v, ST_LANE << k)) for k in range(6)]
        self.lenop = [[nib_tables(lambda v, n=j * 8 ** k: O.shift(v, n)) for j in range(8)] for k in range(4)]

    def shift_len(self, v: int, L: int) -> int:
        for k in range(4):
            v = nib_apply(self.lenop[k][(L >> (3 * k)) & 7], v)
        return v


def stream_wave(T: StreamTables, buf: bytes, offs, lens, view_addr: int = 0):
    """One wave of k_stream over packed packets (offs[i+1] == offs[i] + lens[i]) of the
    view `buf` (loads outside it read 0).  Mirrors csrc/crc32_kernels.hip: 8 KiB rounds
    staged lane-contiguously, lane l chains its 128 B as four 32-B blocks (slice-by-4,
    no masking), Horner over the blocks with T256, an inclusive scan over the 64 lanes
    seeded with the round anchor G = P(R), block anchors A = P(block start); per packet
    P(b) = A fed with the t < 32 bytes of its block before b, and
    crc = P(b) ^ shift(P(a) ^ ~0, len) ^ ~0 with P(a) = the previous packet's P(b).
    P(x) = R_0(view[R0 .. x)) for the wave's first round start R0.  Returns (crcs, rounds)."""
    n = len(lens)
    nb = len(buf)

    def rd16(o):  # the host rounds the view up to 16 B: a chunk holding a valid byte is in range
        return bytes(16) if o < 0 or o >= nb else bytes(buf[o:o + 16]).ljust(16, b"\0")

    def le(b, i):
        return int.from_bytes(b[i:i + 4], "little")

    a_lo = int(offs[0])
    R = ((view_addr + a_lo) & ~127) - view_addr
    G = 0
    out = [None] * n
    cur = 0
    cP = None
    rounds = 0
    while cur < n:
        data = b"".join(rd16(R + 16 * c) for c in range(ST_ROUND // 16))
        C, V = [], []
        for l in range(64):
            seg = data[ST_LANE * l:ST_LANE * (l + 1)]
            cs = []
            for j in range(4):
                c = le(seg, ST_BLK * j)
                for k in range(1, 8):
                    c = _apply(T.s4, c) ^ le(seg, ST_BLK * j + 4 * k)
                cs.append(_apply(T.s4, c))
            H = cs[0]
            for j in range(1, 4):
                H = _apply(T.t256, H) ^ cs[j]
            C.append(cs)
            V.append(H)
        I = list(V)
        I[0] ^= nib_apply(T.scan[0], G)
        for k in range(6):
            d = 1 << k
            I = [I[l] ^ nib_apply(T.scan[k], I[l - d]) if l >= d else I[l] for l in range(64)]
        E = [G] + I[:63]
        A = []
        for l in range(64):
            a = [E[l]]
            for j in range(3):
                a.append(_apply(T.t256, a[-1]) ^ C[l][j])
            A.append(a)

        def P(x):
            assert 0 <= x < ST_ROUND
            l, blk, t = x >> 7, (x >> 5) & 3, x & 31
            c = A[l][blk]
            base = ST_LANE * l + ST_BLK * blk
            for k in range(t >> 2):
                c = _apply(T.s4, c ^ le(data, base + 4 * k))
            r = t & 3
            if r:
                y = ((c ^ le(data, base + 4 * (t >> 2))) << (8 * (4 - r))) & 0xFFFFFFFF
                c = (c >> (8 * r)) ^ _apply(T.s4, y)
            return c

        if cP is None:
            cP = P(a_lo - R)
        while cur < n and int(offs[cur]) + int(lens[cur]) - R < ST_ROUND:
            pb = P(int(offs[cur]) + int(lens[cur]) - R)
            out[cur] = pb ^ T.shift_len(cP ^ 0xFFFFFFFF, int(lens[cur])) ^ 0xFFFFFFFF
            cP = pb
            cur += 1
        G = I[63]
        R += ST_ROUND
        rounds += 1
    return out, rounds


# ---- k_cut_ranges: sub-launches of a mixed-length batch past 2 GiB -----
def cut_ranges(offs, n: int, lead: int, vspan: int, G: int, sb: int):
    """Mirror of csrc/crc32_kernels.hip k_cut_ranges: byte cuts (first packet whose view
    offset reaches k*G, binary search, prefix max) merged with count cuts j*sb; one
    (begin, end, rebase, nbytes, bad) per sub-launch, kb + nc - 1 of them."""
    kb = -(-vspan // G)
    nc = -(-n // sb)
    nd = kb + nc - 1
    bcut = [0] * kb
    for k in range(1, kb):
        lo, hi, t = 0, n, k * G
        while lo < hi:
            m = lo + (hi - lo) // 2
            if int(offs[m]) + lead < t:
                lo = m + 1
            else:
                hi = m
        bcut[k] = lo
    cuts, pb, jc, k = [0], 0, sb, 1
    while len(cuts) < nd:
        b = max(bcut[k], pb) if k < kb else None
        c = jc if jc < n else None
        if b is None and c is None:
            cuts.append(n)
            continue
        if c is None or (b is not None and b <= c):
            cuts.append(b)
            pb = b
            k += 1
        else:
            cuts.append(c)
            jc += sb
    cuts.append(n)
    out = []
    for j in range(nd):
        b, e = cuts[j], max(cuts[j + 1], cuts[j])
        d = {"begin": b, "end": e, "rebase": 0, "nbytes": 16, "bad": 0}
        if b < e:
            r = (int(offs[b]) + lead) & ~15
            if r < vspan:
                d["rebase"], d["nbytes"] = r, min(vspan - r, (1 << 31) - 16)
            else:
                d["bad"] = 1
        out.append(d)
    return out


def range_outside(d, offs, lens, lead: int):
    """Packets of one sub-launch that RangeArrayProvL.decode puts outside its view."""
    bad = []
    for p in range(d["begin"], d["end"]):
        o = int(offs[p]) + lead - d["rebase"]
        if not (0 <= o <= d["nbytes"] and int(lens[p]) <= d["nbytes"] - o):
            bad.append(p)
    return bad
