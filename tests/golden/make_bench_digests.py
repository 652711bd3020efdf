#!/usr/bin/env python3
"""Digests of the full result vectors bench.py produces, computed by the REFERENCE.

bench.py checks its whole CRC vector (not a sample) against these: rank r of an N-rank
run checksums packets [r*n, (r+1)*n) of the global synthetic stream (splitmix64, seed
0x5EED, 1456-B payloads back to back), and rank 0 gathers them, so the vector for N
ranks of n packets is the first N*n packets of the stream.  This script computes those
CRCs with the reference's own cpp/src/common/Crc32.hpp:91-102 (oracle/_ref, compiled
here by oracle/Makefile) and records sha256(little-endian u32 vector) for every prefix
bench.py can produce with its default per-rank sizes (1 M and 2 M = config C4).

    python tests/golden/make_bench_digests.py      # build container; ~5 min on 8 cores
Output: tests/golden/bench_digests.json (data only).
"""
import concurrent.futures as cf
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

PAYLOAD = 1456
CHUNK = 1 << 17  # packets per generation chunk (190 MB)


def main():
    ref = O.ref_lib()
    if ref is None:
        sys.exit("oracle/_ref/libref_crc32.so missing: run `make -C oracle ref` in the build container")
    total = 16 << 20  # 16 M packets: 8 ranks x 2 M (C4)
    marks = sorted({k << 20 for k in (1, 2, 4, 8, 16)})
    h = hashlib.sha256()
    out = {}
    threads = min(8, os.cpu_count() or 1)
    pool = cf.ThreadPoolExecutor(threads)

    def gen(p0, cnt):  # synth in parallel slices (numpy releases the GIL)
        parts = list(pool.map(lambda i: O.synth_fill_np(min(CHUNK // threads + 1, cnt - i) * PAYLOAD,
                                                         start_byte=(p0 + i) * PAYLOAD),
                              range(0, cnt, CHUNK // threads + 1)))
        return np.concatenate(parts)

    for p0 in range(0, total, CHUNK):
        buf = gen(p0, CHUNK)
        crc = np.zeros(CHUNK, dtype=np.uint32)
        ref.ref_crc32_batch_fixed_mt(buf.ctypes.data, PAYLOAD, PAYLOAD, CHUNK,
                                     crc.ctypes.data_as(C.POINTER(C.c_uint32)), threads)
        if p0 == 0:
            assert int(crc[0]) == O.crc32(buf[:PAYLOAD])
        h.update(crc.astype("<u4").tobytes())
        if p0 + CHUNK in marks:
            out[str(p0 + CHUNK)] = h.copy().hexdigest()
            print(p0 + CHUNK, out[str(p0 + CHUNK)], flush=True)
    doc = {"what": "sha256 of the little-endian u32 CRC vector of packets [0, n) of the synthetic stream "
                   "(splitmix64 seed 0x5EED, 1456-B payloads back to back), computed by the reference "
                   "crc32 (cpp/src/common/Crc32.hpp:91-102 via oracle/_ref)",
           "payload": PAYLOAD, "seed": O.SEED, "sha256_by_packets": out}
    with open(os.path.join(HERE, "bench_digests.json"), "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
