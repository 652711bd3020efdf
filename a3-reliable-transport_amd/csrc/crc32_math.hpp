// crc32_math.hpp — host-side GF(2) algebra of the reflected CRC-32 used to build the
// device constant tables.  Everything is generated from the polynomial; no table is
// copied from the reference (whose cpp/src/common/Crc32.hpp:46-89 equals
// sarwate_table() below — checked by tests/test_oracle.py against the golden vectors).
//
// Notation: R_c(M) = CRC register after message M from init c, no
// xorout.  crc32(M) = R_{~0}(M) ^ ~0 = R_0(M) ^ shift(~0, |M|) ^ ~0.
//   shift(v, n)   = R_v(0^n)          = v * x^(8n)  mod P
//   unshift(v, n) = v * x^(-8n) mod P  (x is invertible because P(0) = 1)
#pragma once

#include <cstddef>
#include <cstdint>

namespace wtp {

constexpr uint32_t kPoly = 0xEDB88320u;  // reflected 0x04C11DB7, Crc32.hpp:30-34

struct Sarwate {
    uint32_t t[256];
    Sarwate() {
        for (uint32_t b = 0; b < 256; ++b) {
            uint32_t c = b;
            for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
            t[b] = c;
        }
    }
};

inline const Sarwate &sarwate() {
    static const Sarwate s;
    return s;
}

// Byte-at-a-time register update (Crc32.hpp:98-99).
inline uint32_t raw_update(uint32_t c, const uint8_t *p, size_t n) {
    const uint32_t *t = sarwate().t;
    while (n--) c = t[(c ^ *p++) & 0xFFu] ^ (c >> 8);
    return c;
}

inline uint32_t shift_bytes(uint32_t v, uint64_t n) {
    const uint32_t *t = sarwate().t;
    while (n--) v = t[v & 0xFFu] ^ (v >> 8);
    return v;
}

inline uint32_t unshift_bytes(uint32_t v, uint64_t n) {
    for (uint64_t i = 0; i < 8 * n; ++i)
        v = (v & 0x80000000u) ? (((v ^ kPoly) << 1) | 1u) : (v << 1);
    return v;
}

// Linear operator on a 32-bit register as four byte tables:
//   f(v) = op[0][v&255] ^ op[1][(v>>8)&255] ^ op[2][(v>>16)&255] ^ op[3][v>>24].
// `out` receives 1024 words, table k at out[256*k].
template <class F>
inline void make_operator(uint32_t *out, F f) {
    for (int k = 0; k < 4; ++k)
        for (uint32_t b = 0; b < 256; ++b) out[256 * k + b] = f(b << (8 * k));
}

// Word tables for a message word placed at the start of a `block`-byte block:
// wt[256*k + e] = R_0(block with byte k = e, all other bytes 0), k = 0..3.
// block = 4 gives slice-by-4; block = 4N gives the N-braid "advance" tables.
inline void make_word_tables(uint32_t *out, uint64_t block) {
    const uint32_t *t = sarwate().t;
    for (int k = 0; k < 4; ++k)
        for (uint32_t e = 0; e < 256; ++e) out[256 * k + e] = shift_bytes(t[e], block - 1 - (uint64_t)k);
}

// crc32 of a message of length L equals R_0(M) ^ init_const(L).
inline uint32_t init_const(uint64_t len) { return shift_bytes(0xFFFFFFFFu, len) ^ 0xFFFFFFFFu; }

}  // namespace wtp
