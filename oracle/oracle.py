"""ctypes front-end for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Loads oracle/liboracle.so (the from-scratch restatement, crc32_oracle.c) and, when
present, oracle/_ref/libref_crc32.so (the reference's own cpp/src/common/Crc32.hpp
compiled in this container).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module; the product path never does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_crc32.so")

SEED = 0x5EED
MAX_PAYLOAD = 1456

_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


def _ptr(a: np.ndarray, t=C.c_void_p):
    return C.cast(a.ctypes.data, t)


def _load_oracle() -> C.CDLL:
    if not os.path.exists(ORACLE_SO):
        raise RuntimeError(f"oracle library missing: {ORACLE_SO} (run `make -C oracle`)")
    lib = C.CDLL(ORACLE_SO)
    lib.oracle_crc32.restype = C.c_uint32
    lib.oracle_crc32.argtypes = [C.c_void_p, C.c_size_t]
    lib.oracle_crc32_raw.restype = C.c_uint32
    lib.oracle_crc32_raw.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
    lib.oracle_crc32_shift.restype = C.c_uint32
    lib.oracle_crc32_shift.argtypes = [C.c_uint32, C.c_uint64]
    lib.oracle_crc32_unshift.restype = C.c_uint32
    lib.oracle_crc32_unshift.argtypes = [C.c_uint32, C.c_uint64]
    lib.oracle_crc32_combine.restype = C.c_uint32
    lib.oracle_crc32_combine.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
    lib.oracle_crc32_table.argtypes = [_u32p]
    lib.oracle_crc32_batch_fixed.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, _u32p]
    lib.oracle_crc32_batch_fixed_mt.restype = C.c_int
    lib.oracle_crc32_batch_fixed_mt.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, _u32p, C.c_int]
    lib.oracle_crc32_batch_var.argtypes = [C.c_void_p, _u64p, _u32p, C.c_size_t, _u32p]
    lib.oracle_verify_datagrams.argtypes = [C.c_void_p, C.c_size_t, _u32p, C.c_size_t, _u8p, _u32p]
    lib.oracle_build_datagram.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, _u8p]
    lib.oracle_synth_word.restype = C.c_uint64
    lib.oracle_synth_word.argtypes = [C.c_uint64, C.c_uint64]
    lib.oracle_synth_fill.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, _u8p]
    return lib


_LIB: C.CDLL | None = None
_REF: C.CDLL | None = None


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = _load_oracle()
    return _LIB


def ref_lib() -> C.CDLL | None:
    """The compiled reference (oracle/_ref), or None when it was not built."""
    global _REF
    if _REF is None and os.path.exists(REF_SO):
        r = C.CDLL(REF_SO)
        r.ref_crc32.restype = C.c_uint32
        r.ref_crc32.argtypes = [C.c_void_p, C.c_size_t]
        r.ref_crc32_batch_fixed.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, _u32p]
        r.ref_crc32_batch_var.argtypes = [C.c_void_p, _u64p, _u32p, C.c_size_t, _u32p]
        r.ref_crc32_batch_fixed_mt.restype = C.c_int
        r.ref_crc32_batch_fixed_mt.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, _u32p, C.c_int]
        _REF = r
    return _REF


# ---- convenience wrappers ---------------------------------------------------------

def crc32(data: bytes | np.ndarray) -> int:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data, dtype=np.uint8)
    return int(lib().oracle_crc32(_ptr(a), a.size))


def table() -> np.ndarray:
    out = np.zeros(256, dtype=np.uint32)
    lib().oracle_crc32_table(_ptr(out, _u32p))
    return out


def shift(v: int, nbytes: int) -> int:
    return int(lib().oracle_crc32_shift(v, nbytes))


def unshift(v: int, nbytes: int) -> int:
    return int(lib().oracle_crc32_unshift(v, nbytes))


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return int(lib().oracle_crc32_combine(crc_a, crc_b, len_b))


def batch_fixed(buf: np.ndarray, stride: int, length: int, n: int, threads: int = 1) -> np.ndarray:
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    if n and (n - 1) * stride + length > buf.size:
        raise ValueError("buffer too small")
    out = np.zeros(n, dtype=np.uint32)
    if threads > 1:
        lib().oracle_crc32_batch_fixed_mt(_ptr(buf), stride, length, n, _ptr(out, _u32p), threads)
    else:
        lib().oracle_crc32_batch_fixed(_ptr(buf), stride, length, n, _ptr(out, _u32p))
    return out


def batch_var(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray) -> np.ndarray:
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = offsets.size
    if n and int((offsets + lengths).max()) > buf.size:
        raise ValueError("buffer too small")
    out = np.zeros(n, dtype=np.uint32)
    lib().oracle_crc32_batch_var(_ptr(buf), _ptr(offsets, _u64p), _ptr(lengths, _u32p), n, _ptr(out, _u32p))
    return out


def verify_datagrams(dgrams: np.ndarray, stride: int, recv_len: np.ndarray):
    dgrams = np.ascontiguousarray(dgrams, dtype=np.uint8)
    recv_len = np.ascontiguousarray(recv_len, dtype=np.uint32)
    n = recv_len.size
    ok = np.zeros(n, dtype=np.uint8)
    crc = np.zeros(n, dtype=np.uint32)
    lib().oracle_verify_datagrams(_ptr(dgrams), stride, _ptr(recv_len, _u32p), n, _ptr(ok, _u8p), _ptr(crc, _u32p))
    return ok, crc


def build_datagram(seq: int, payload: bytes, ptype: int = 2) -> bytes:
    p = np.frombuffer(bytes(payload), dtype=np.uint8)
    out = np.zeros(16 + p.size, dtype=np.uint8)
    lib().oracle_build_datagram(ptype, seq, _ptr(p) if p.size else None, p.size, _ptr(out, _u8p))
    return out.tobytes()


def synth_fill(nbytes: int, start_byte: int = 0, seed: int = SEED) -> np.ndarray:
    out = np.zeros(nbytes, dtype=np.uint8)
    lib().oracle_synth_fill(seed, start_byte, nbytes, _ptr(out, _u8p))
    return out


def synth_fill_np(nbytes: int, start_byte: int = 0, seed: int = SEED) -> np.ndarray:
    """Vectorised numpy version of oracle_synth_fill (same bytes, faster for big buffers)."""
    w0 = start_byte >> 3
    w1 = (start_byte + nbytes + 7) >> 3
    w = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (w + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    s = start_byte - (w0 << 3)
    return b[s:s + nbytes].copy()


def zipf_lengths(n: int, s: float = 1.1, seed: int = SEED, max_len: int = MAX_PAYLOAD) -> np.ndarray:
    """Zipf(s) on [1, max_len] by inverse CDF over splitmix uniforms."""
    k = np.arange(1, max_len + 1, dtype=np.float64)
    pmf = k ** (-s)
    cdf = np.cumsum(pmf)
    cdf /= cdf[-1]
    w = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed ^ 0x21F) + (w + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    idx = np.searchsorted(cdf, u, side="right")
    return np.minimum(idx + 1, max_len).astype(np.uint32)
