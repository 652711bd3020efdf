"""Read the gfx950 code object out of a HIP shared library, in pure Python (no ROCm tools
needed, so bench.py can use it on the GPU box): the .hip_fatbin section of the host ELF
holds a Clang offload bundle whose gfx950 entry is an AMDGPU ELF; its symbol table gives
each kernel's machine code.

kernel_code_sha256(lib, pattern) hashes the code bytes of the kernel whose mangled name
matches `pattern`.  bench.py stamps roofline.traffic with it: the committed PMC pass
(profiles/pmc_traffic.json) counts for the kernel it measured and for no other.
"""
from __future__ import annotations

import hashlib
import re
import struct

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf: bytes) -> dict:
    """{name: (offset, size, sh_type, sh_link, sh_entsize, index)} of a little-endian ELF64."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not a little-endian ELF64 file")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stro = hdrs[shstrndx][4]
    out = {}
    for i, h in enumerate(hdrs):
        name_off, sh_type, _fl, _addr, off, size, link, _info, _al, entsize = h
        end = elf.index(b"\0", stro + name_off)
        out[elf[stro + name_off:end].decode()] = (off, size, sh_type, link, entsize, i)
    return out


def gfx950_code_object(lib_path: str) -> bytes:
    blob = open(lib_path, "rb").read()
    secs = _sections(blob)
    if ".hip_fatbin" not in secs:
        raise ValueError(f"{lib_path}: no .hip_fatbin section")
    off, size = secs[".hip_fatbin"][:2]
    fb = blob[off:off + size]
    at = fb.find(_BUNDLE_MAGIC)
    if at < 0:
        raise ValueError(f"{lib_path}: no uncompressed offload bundle")
    p = at + len(_BUNDLE_MAGIC)
    n, = struct.unpack_from("<Q", fb, p)
    p += 8
    for _ in range(n):
        eoff, esize, tlen = struct.unpack_from("<QQQ", fb, p)
        p += 24
        triple = fb[p:p + tlen].decode()
        p += tlen
        if triple.endswith("gfx950"):
            return fb[at + eoff:at + eoff + esize]
    raise ValueError(f"{lib_path}: no gfx950 entry in the offload bundle")


def kernel_symbols(co: bytes) -> dict:
    """{mangled name: (file offset of the code, size)} of the code object's FUNC symbols."""
    secs = _sections(co)
    by_index = {v[5]: v for v in secs.values()}
    symoff, symsize, _t, link, entsize, _i = secs[".symtab"]
    stroff = by_index[link][0]
    out = {}
    for k in range(symsize // entsize):
        name, info, _other, shndx, value, size = struct.unpack_from("<IBBHQQ", co, symoff + k * entsize)
        if info & 0xF != 2 or size == 0 or shndx == 0 or shndx not in by_index:  # STT_FUNC with code
            continue
        end = co.index(b"\0", stroff + name)
        nm = co[stroff + name:end].decode()
        # executable sections of a code object are mapped at their file offset + addr delta
        sh = _section_header(co, shndx)
        out[nm] = (sh["offset"] + (value - sh["addr"]), size)
    return out


def _section_header(elf: bytes, idx: int) -> dict:
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, = struct.unpack_from("<H", elf, 0x3A)
    h = struct.unpack_from("<IIQQQQIIQQ", elf, shoff + idx * shentsize)
    return {"addr": h[3], "offset": h[4], "size": h[5]}


def kernel_code_sha256(lib_path: str, pattern: str) -> dict:
    """sha256 of the machine code of the one kernel whose mangled name matches `pattern`."""
    co = gfx950_code_object(lib_path)
    syms = kernel_symbols(co)
    hits = sorted(n for n in syms if re.search(pattern, n))
    if len(hits) != 1:
        raise ValueError(f"{pattern!r} matches {len(hits)} kernels: {hits[:4]}")
    off, size = syms[hits[0]]
    return {"kernel": hits[0], "code_bytes": size, "sha256": hashlib.sha256(co[off:off + size]).hexdigest()}


# the headline kernel: k_fixed_braid<6 rows, DIAG 0, CrcHoldBEpi> (1456-B payloads; the
# launcher's long-batch epilogue, which 1 M packets use)
HEADLINE_KERNEL = r"k_fixed_braidILi6ELi0ENS0_11CrcHoldBEpiE"

if __name__ == "__main__":
    import json
    import sys
    print(json.dumps(kernel_code_sha256(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else HEADLINE_KERNEL)))
