#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the REFERENCE itself.

Run in the build container (needs /root/reference and `make -C oracle ref`):
    python tests/golden/make_golden.py

Every expected value below is produced by calling the reference's own
cpp/src/common/Crc32.hpp:91-102 (compiled from where it lies into
oracle/_ref/libref_crc32.so by oracle/Makefile) and cross-checked against
Python's zlib.crc32.  Nothing here is computed by the oracle restatement, so the
oracle is pinned by these vectors rather than by itself.

Outputs (data only):
  golden.json        known answers, per-length vectors, sample-file chunk CRCs,
                     random-batch digest
  input.txt, input2.txt, input3.txt   the reference's sample transfer files
                     (data files; config 1 uses input.txt)
"""
import ctypes as C
import hashlib
import json
import os
import shutil
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_TREE = "/root/reference"
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_crc32.so")
SEED = 0x5EED
CHUNK = 1456  # cpp/src/base/Sender.cpp:20


def splitmix_bytes(nbytes, start=0, seed=SEED):
    """Counter-based payload bytes, SURVEY.md §8d (same definition as the oracle/GPU)."""
    out = bytearray()
    w = start >> 3
    while len(out) < nbytes + (start & 7):
        z = (seed + (w + 1) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
        out += z.to_bytes(8, "little")
        w += 1
    s = start & 7
    return bytes(out[s:s + nbytes])


def main():
    if not os.path.exists(REF_SO):
        sys.exit(f"{REF_SO} missing: run `make -C oracle ref` in the build container")
    ref = C.CDLL(REF_SO)
    ref.ref_crc32.restype = C.c_uint32
    ref.ref_crc32.argtypes = [C.c_char_p, C.c_size_t]

    def rcrc(b: bytes) -> int:
        v = int(ref.ref_crc32(b, len(b)))
        assert v == zlib.crc32(b), "reference and zlib disagree"
        return v

    g = {"generator": "tests/golden/make_golden.py", "source": "reference cpp/src/common/Crc32.hpp:91-102 via oracle/_ref + zlib cross-check",
         "seed": SEED}

    # Known answers
    kats = {
        "123456789": rcrc(b"123456789"),
        "": rcrc(b""),
        "zeros_1456": rcrc(b"\x00" * CHUNK),
        "ones_1456": rcrc(b"\xff" * CHUNK),
        "a": rcrc(b"a"),
        "abc": rcrc(b"abc"),
        "quick_fox": rcrc(b"The quick brown fox jumps over the lazy dog"),
    }
    g["kat"] = {k: f"0x{v:08X}" for k, v in kats.items()}

    # Per-length vectors 0..1456 over the seeded counter-hash payload: message of
    # length L = the first L bytes of the stream starting at byte offset 1000*L.
    per_len = []
    for L in range(CHUNK + 1):
        per_len.append(rcrc(splitmix_bytes(L, start=1000 * L)))
    g["per_length"] = {"rule": "payload(L) = synth bytes [1000*L, 1000*L+L), seed 0x5EED", "crc": per_len}

    # Sample files: the reference sender chunks at 1456 (Sender.cpp:89-90).
    files = {}
    for name in ("input.txt", "input2.txt", "input3.txt"):
        src = os.path.join(REF_TREE, name)
        shutil.copyfile(src, os.path.join(HERE, name))
        data = open(src, "rb").read()
        chunks = [data[i:i + CHUNK] for i in range(0, len(data), CHUNK)]
        files[name] = {"bytes": len(data), "chunk_lens": [len(c) for c in chunks],
                       "crc": [f"0x{rcrc(c):08X}" for c in chunks],
                       "sha256": hashlib.sha256(data).hexdigest()}
    g["files"] = files

    # Random fixed batch: 4096 x 1456 synthetic packets from byte 0.
    n = 4096
    buf = splitmix_bytes(n * CHUNK)
    crcs = [rcrc(buf[i * CHUNK:(i + 1) * CHUNK]) for i in range(n)]
    arr = np.array(crcs, dtype="<u4").tobytes()
    g["batch_4096x1456"] = {"first8": [f"0x{c:08X}" for c in crcs[:8]], "last": f"0x{crcs[-1]:08X}",
                            "sha256_le_u32": hashlib.sha256(arr).hexdigest(),
                            "crc_of_crcs": f"0x{zlib.crc32(arr):08X}"}

    # Mixed-length batch: lengths = 1 + (i*7919) % 1456, packed contiguously from byte 0.
    lens = [1 + (i * 7919) % CHUNK for i in range(2048)]
    total = sum(lens)
    mb = splitmix_bytes(total)
    off = 0
    mcrc = []
    for L in lens:
        mcrc.append(rcrc(mb[off:off + L]))
        off += L
    marr = np.array(mcrc, dtype="<u4").tobytes()
    g["mixed_2048"] = {"rule": "len_i = 1 + (i*7919) % 1456, packed from synth byte 0",
                       "sha256_le_u32": hashlib.sha256(marr).hexdigest(), "first8": [f"0x{c:08X}" for c in mcrc[:8]]}

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
