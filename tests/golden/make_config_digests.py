#!/usr/bin/env python3
"""Digests of bench.py's `configs` leg results, computed by the REFERENCE's crc32.

bench.py's configs leg (tools/config_legs.py) runs every BASELINE.json config on the GPU
and checks each row's whole result (not a sample) against a sha256 recorded here.  The
inputs are the synthetic stream (splitmix64 seed 0x5EED, oracle.synth_fill_np, the same
bytes the device generator wtp_synth_fill writes) and, for C5, Zipf lengths
(oracle.zipf_lengths; config_legs.zipf_lengths is the same function, pinned by
tests/test_bench.py).  Every CRC below is the reference's own
cpp/src/common/Crc32.hpp:91-102 (oracle/_ref, compiled here by oracle/Makefile); the wire
headers are the reference's PacketHeader (cpp/src/common/PacketHeader.hpp:5-10), htonl'd as
cpp/src/base/Packet.cpp:40-47 does, type DATA = 2, seq from 0.

    python tests/golden/make_config_digests.py     # build container; ~1 min
Output: tests/golden/config_digests.json (data only).

  c2             u32 CRCs of packets [0, 64 K) (BASELINE configs[1])
  c3_1gib        u32 CRCs of a 1 GiB file chunked at 1456 B: 737,460 full chunks + a 64-B
                 tail (configs[2]; the chunking of cpp/src/base/Sender.cpp:82-92)
  c5_zipf1.1/1.0 u32 CRCs of 1 M packed payloads, Zipf(s) lengths on [1, 1456]
                 (configs[4]; the variable recv_len - 16 of Receiver.cpp:32-33)
  verify_fixup_1m  crc_out of the receiver verify over 1 M DATA datagrams with datagrams
                 0 and n/2 cut to 16 B (payload 0) and n-1 to 1016 B (payload 1000)
  build_1m       the 1 M x 1472-B DATA datagrams of packets [0, 1 M), back to back
  hostbuild_1gib the 737,461 DATA datagrams of the 1 GiB file (last one 16 + 64 B)
"""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (synthetic generator + the compiled reference loader)

P = 1456
U32P = C.POINTER(C.c_uint32)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ref_fixed(ref, buf, n, stride=P, length=P):
    out = np.zeros(n, dtype=np.uint32)
    ref.ref_crc32_batch_fixed_mt(buf.ctypes.data, stride, length, n, out.ctypes.data_as(U32P), min(8, os.cpu_count() or 1))
    return out


def datagrams(ref, payload: np.ndarray, nbytes: int) -> tuple[np.ndarray, np.ndarray]:
    """The DATA datagrams of payload[:nbytes] chunked at 1456 B, seq 0..: full ones as an
    (m, 1472) array, and the last (short) one separately (empty if nbytes % 1456 == 0)."""
    m = nbytes // P
    crc = ref_fixed(ref, payload, m)
    w = np.empty((m, 16 + P), dtype=np.uint8)
    hdr = np.stack([np.full(m, 2, np.uint32), np.arange(m, dtype=np.uint32), np.full(m, P, np.uint32), crc], axis=1)
    w[:, :16] = hdr.astype(">u4").view(np.uint8).reshape(m, 16)
    w[:, 16:] = payload[:m * P].reshape(m, P)
    tail = np.zeros(0, np.uint8)
    if nbytes % P:
        t = payload[m * P:nbytes]
        h = np.array([2, m, t.size, ref.ref_crc32(t.ctypes.data, t.size)], dtype=">u4").view(np.uint8)
        tail = np.concatenate([h, t])
    return w, tail


def main():
    ref = O.ref_lib()
    if ref is None:
        sys.exit("oracle/_ref/libref_crc32.so missing: run `make -C oracle ref` in the build container")
    out = {}
    # C2: 64 K x 1456 B
    n = 65536
    out["c2"] = sha(ref_fixed(ref, O.synth_fill_np(n * P), n).astype("<u4"))
    # C3: 1 GiB chunked at 1456 B
    nb = 1 << 30
    host = O.synth_fill_np(nb)
    m = nb // P
    crc = np.concatenate([ref_fixed(ref, host, m), [ref.ref_crc32(host[m * P:].ctypes.data, nb - m * P)]]).astype("<u4")
    assert crc.size == (nb + P - 1) // P and nb - m * P == 64
    out["c3_1gib"] = sha(crc)
    # host builder over the same 1 GiB
    w, tail = datagrams(ref, host, nb)
    h = hashlib.sha256(w.tobytes())
    h.update(tail.tobytes())
    out["hostbuild_1gib"] = h.hexdigest()
    del w, tail
    # C5: 1 M packed Zipf payloads
    n = 1 << 20
    for s in (1.1, 1.0):
        lens = O.zipf_lengths(n, s=s).astype(np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
        data = O.synth_fill_np(int(lens.sum()))
        c = np.zeros(n, dtype=np.uint32)
        ref.ref_crc32_batch_var(data.ctypes.data, offs.ctypes.data_as(C.POINTER(C.c_uint64)),
                                lens.ctypes.data_as(U32P), n, c.ctypes.data_as(U32P))
        assert int(c[5]) == O.crc32(data[int(offs[5]):int(offs[5]) + int(lens[5])])
        out[f"c5_zipf{s}"] = sha(c.astype("<u4"))
    # device builder and receiver verify over packets [0, 1 M)
    pay = O.synth_fill_np(n * P)
    crc = ref_fixed(ref, pay, n)
    w, _ = datagrams(ref, pay, n * P)
    assert w[1].tobytes() == O.build_datagram(1, pay[P:2 * P].tobytes())
    out["build_1m"] = sha(w)
    del w
    fix = crc.copy()
    fix[0] = fix[n // 2] = ref.ref_crc32(None, 0)
    last = pay[(n - 1) * P:(n - 1) * P + 1000]
    fix[n - 1] = ref.ref_crc32(last.ctypes.data, 1000)
    out["verify_fixup_1m"] = sha(fix.astype("<u4"))
    doc = {"what": "sha256 of bench.py configs-leg results (tools/config_legs.py), every CRC by the reference "
                   "crc32 (cpp/src/common/Crc32.hpp:91-102 via oracle/_ref); see make_config_digests.py",
           "payload": P, "seed": O.SEED, "sha256": out}
    with open(os.path.join(HERE, "config_digests.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
