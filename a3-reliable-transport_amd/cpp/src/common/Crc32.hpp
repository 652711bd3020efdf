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
}  // namespace wtp::detail

inline uint32_t crc32(const void *buf, size_t size) {
    const auto &t = wtp::detail::kCrc32Table;
    const uint8_t *p = static_cast<const uint8_t *>(buf);
    uint32_t c = 0xFFFFFFFFu;
    while (size--) c = t[(c ^ *p++) & 0xFFu] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}
