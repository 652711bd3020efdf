// Crc32.hpp — drop-in for the reference's cpp/src/common/Crc32.hpp.
//
// Keeps the reference call surface  `inline uint32_t crc32(const void *buf, size_t size)`
// (Crc32.hpp:91-102) with identical results — IEEE CRC-32, reflected polynomial
// 0xEDB88320, init/xorout 0xFFFFFFFF, crc32(p, 0) == 0 — for single packets and the
// 0-byte ACK payloads (Sender::isAckValid, cpp/src/base/Sender.cpp:235-237).  The
// table is generated at compile time from the polynomial (the reference's literal table
// at :46-89 is exactly this generator's output); it is const, unlike the reference's
// mutable `static` array, and the header has an include guard.
//
// wtp::crc32_fast (below) is the same function, slice-by-8, for the endpoints' small-batch
// CPU path.
//
// Batches go to the MI355X library through the C-ABI in include/wtp_crc32.h (included
// here so that existing `#include "../common/Crc32.hpp"` sites see it):
//   sender packet build -> wtp_crc32_host_chunked / wtp_crc32_batch_fixed
//   receiver verify     -> wtp_crc32_host_verify  / wtp_crc32_verify_batch
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>

#include "wtp_crc32.h"

namespace wtp::detail {
constexpr std::array<uint32_t, 256> make_crc32_table() {
    std::array<uint32_t, 256> t{};
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        t[b] = c;
    }
    return t;
}
inline constexpr std::array<uint32_t, 256> kCrc32Table = make_crc32_table();
static_assert(kCrc32Table[1] == 0x77073096u && kCrc32Table[255] == 0x2D02EF8Du);

// Slice-by-8: table k advances a byte by k more zero bytes (T_k[b] = T_0[T_{k-1}[b] & 0xFF]
// ^ (T_{k-1}[b] >> 8)), so 8 input bytes cost 8 independent lookups instead of a chain of 8.
constexpr std::array<std::array<uint32_t, 256>, 8> make_crc32_slice8() {
    std::array<std::array<uint32_t, 256>, 8> t{};
    t[0] = make_crc32_table();
    for (int k = 1; k < 8; ++k)
        for (int b = 0; b < 256; ++b) t[k][b] = t[0][t[k - 1][b] & 0xFFu] ^ (t[k - 1][b] >> 8);
    return t;
}
inline constexpr std::array<std::array<uint32_t, 256>, 8> kCrc32Slice8 = make_crc32_slice8();
}  // namespace wtp::detail

inline uint32_t crc32(const void *buf, size_t size) {
    const auto &t = wtp::detail::kCrc32Table;
    const uint8_t *p = static_cast<const uint8_t *>(buf);
    uint32_t c = 0xFFFFFFFFu;
    while (size--) c = t[(c ^ *p++) & 0xFFu] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

namespace wtp {
// The same CRC-32 as crc32() above, 8 bytes per step (slice-by-8): the CPU path for batches
// too small to amortise a GPU call (Checksums::verify_batch), ~4x the byte loop.
inline uint32_t crc32_fast(const void *buf, size_t size) {
    const auto &t = detail::kCrc32Slice8;
    const uint8_t *p = static_cast<const uint8_t *>(buf);
    uint32_t c = 0xFFFFFFFFu;
    for (; size >= 8; size -= 8, p += 8) {
        uint32_t lo, hi;
        __builtin_memcpy(&lo, p, 4);
        __builtin_memcpy(&hi, p + 4, 4);
        lo ^= c;  // little-endian host (x86-64, the GPU box's)
        c = t[7][lo & 0xFFu] ^ t[6][(lo >> 8) & 0xFFu] ^ t[5][(lo >> 16) & 0xFFu] ^ t[4][lo >> 24] ^
            t[3][hi & 0xFFu] ^ t[2][(hi >> 8) & 0xFFu] ^ t[1][(hi >> 16) & 0xFFu] ^ t[0][hi >> 24];
    }
    while (size--) c = t[0][(c ^ *p++) & 0xFFu] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}
static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "crc32_fast reads words little-endian");
}  // namespace wtp
