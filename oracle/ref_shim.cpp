// ref_shim.cpp — C-ABI wrapper around the REFERENCE's own CRC header, compiled where
// it lies (/root/reference/cpp/src/common/Crc32.hpp, found through -I in
// oracle/Makefile; nothing is copied).  Output goes to oracle/_ref/ only.
//
// TEST INFRASTRUCTURE ONLY: used to pin the oracle restatement (tests/golden/
// make_golden.py) and as bench.py's cpu_baseline ("kind": "reference").
// The product library never links or loads it.
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

#include "Crc32.hpp"  // reference: cpp/src/common/Crc32.hpp:91-102

extern "C" {

uint32_t ref_crc32(const void *buf, size_t size) { return crc32(buf, size); }

// The reference calls crc32 once per chunk (cpp/src/base/Packet.cpp:36-38); this
// loop is only the batch driver around those calls.
void ref_crc32_batch_fixed(const void *base, size_t stride, size_t len, size_t n, uint32_t *out) {
    const char *b = static_cast<const char *>(base);
    for (size_t i = 0; i < n; ++i) out[i] = crc32(b + i * stride, len);
}

// Payloads at arbitrary offsets/lengths (config C5's packed mixed lengths): one reference
// crc32 call per payload, as the receiver makes one per datagram (Receiver.cpp:32-33).
void ref_crc32_batch_var(const void *base, const uint64_t *offs, const uint32_t *lens, size_t n, uint32_t *out) {
    const char *b = static_cast<const char *>(base);
    for (size_t i = 0; i < n; ++i) out[i] = crc32(b + offs[i], lens[i]);
}

int ref_crc32_batch_fixed_mt(const void *base, size_t stride, size_t len, size_t n, uint32_t *out,
                             int threads) {
    if (threads < 1) threads = 1;
    std::vector<std::thread> th;
    const char *b = static_cast<const char *>(base);
    for (int t = 0; t < threads; ++t) {
        size_t lo = n * size_t(t) / size_t(threads), hi = n * size_t(t + 1) / size_t(threads);
        th.emplace_back([=] {
            for (size_t i = lo; i < hi; ++i) out[i] = crc32(b + i * stride, len);
        });
    }
    for (auto &x : th) x.join();
    return 0;
}

}  // extern "C"
