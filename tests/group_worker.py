#!/usr/bin/env python3
"""Drives lib/libwtp_group.so from a process WITHOUT torch (its RCCL is /opt/rocm's):
per-rank shards of the global synthetic stream are allocated and filled on their
devices, wtp_group_crc32_fixed_gather checksums and gathers them to the root, and the
gathered u32 vector is written to <out.npy>.  Run by tests/test_gpu_shard.py.

    python tests/group_worker.py <out.npy> <devices,comma,separated> <n_per,comma,separated> <root>
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "a3-reliable-transport_amd", "lib")
PAYLOAD = 1456
SEED = 0x5EED


def main():
    out_path = sys.argv[1]
    devs = [int(x) for x in sys.argv[2].split(",")]
    n_per = [int(x) for x in sys.argv[3].split(",")]
    root = int(sys.argv[4])
    R = len(devs)
    hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
    G = C.CDLL(os.path.join(LIBDIR, "libwtp_group.so"))
    W = C.CDLL(os.path.join(LIBDIR, "libwtp_crc32.so"))
    W.wtp_last_error.restype = C.c_char_p
    W.wtp_synth_fill.argtypes = [C.c_void_p, C.c_uint64, C.c_size_t, C.c_uint64, C.c_void_p]
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    G.wtp_group_create.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
    G.wtp_group_destroy.argtypes = [C.c_void_p]
    G.wtp_group_size.argtypes = [C.c_void_p]
    G.wtp_group_crc32_fixed_gather.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]

    def check(rc, what):
        if rc != 0:
            raise SystemExit(f"{what} failed ({rc}): {W.wtp_last_error().decode()}")

    def dmalloc(dev, nbytes):
        check(hip.hipSetDevice(dev), "hipSetDevice")
        p = C.c_void_p()
        check(hip.hipMalloc(C.byref(p), max(nbytes, 16)), "hipMalloc")
        return p.value

    shards, locals_ = [], []
    start = 0
    for r in range(R):
        sb = dmalloc(devs[r], n_per[r] * PAYLOAD + 64)
        check(W.wtp_synth_fill(sb, start * PAYLOAD, n_per[r] * PAYLOAD, SEED, None), "wtp_synth_fill")
        shards.append(sb)
        locals_.append(dmalloc(devs[r], n_per[r] * 4))
        start += n_per[r]
    total = start
    d_out = dmalloc(devs[root], total * 4)
    g = C.c_void_p()
    dv = (C.c_int * R)(*devs)
    check(G.wtp_group_create(dv, R, C.byref(g)), "wtp_group_create")
    assert G.wtp_group_size(g) == R
    sh = (C.c_void_p * R)(*shards)
    lo = (C.c_void_p * R)(*locals_)
    npr = (C.c_size_t * R)(*n_per)
    check(G.wtp_group_crc32_fixed_gather(g, sh, PAYLOAD, PAYLOAD, npr, lo, d_out, root, None),
          "wtp_group_crc32_fixed_gather")
    for d in set(devs):
        check(hip.hipSetDevice(d), "hipSetDevice")
        check(hip.hipDeviceSynchronize(), "hipDeviceSynchronize")
    host = np.zeros(total, dtype=np.uint32)
    check(hip.hipSetDevice(devs[root]), "hipSetDevice")
    check(hip.hipMemcpy(host.ctypes.data, d_out, total * 4, 2), "hipMemcpy D2H")  # 2 = DeviceToHost
    G.wtp_group_destroy(g)
    np.save(out_path, host)
    print(f"group of {R} on devices {devs}: gathered {total} CRCs to rank {root}")


if __name__ == "__main__":
    main()
