// crc32_kernels.hip — CDNA4 (gfx950) kernels for WTP's per-packet CRC-32.
//
// Reference path being replaced (mmheyer/a3-reliable-transport):
//   crc32()  cpp/src/common/Crc32.hpp:91-102 — byte-at-a-time Sarwate loop, one call
//            per DATA payload (Packet.cpp:13 sender build, Receiver.cpp:204 verify).
//
// Two kernel families, both HBM-read-bound integer work (no MFMA):
//
// 1. k_fixed_braid<ROWS> — equal-length payloads whose ends are 16-B aligned (the
//    1456-B DATA chunk case, the receiver's 1472-B ring, the fused packet builder).
//    16 lanes per packet, 4 packets per wave.  Each lane owns 4 interleaved "braids"
//    (CRC streams over every 64th dword of the packet's frame), so the 16 lanes of a
//    packet read 256 contiguous bytes per row with buffer_load_dwordx4 (coalesced, no
//    LDS staging) and every lane carries 4 independent dependency chains.  Per lookup:
//    one v_perm_b32 builds the LDS address and one ds_read_b32 fetches the table word
//    from staggered 8-copy tables (conflict-free whatever the data).  A lane folds its
//    braids in-lane (x^-32 Horner); every 8 rounds a flush combines each packet's 16
//    columns by Horner's rule through an LDS transposition slot.
//
// 2. k_pieces<Prov, Epi> — anything else (mixed lengths, odd strides, unaligned
//    buffers, datagrams that are not full ring slots).  Each packet is cut into pieces of
//    S = 64 bytes counted back from its end (the head piece is shorter); pieces of
//    consecutive packets are packed densely into the 64 lanes of a wave ("wavefront-
//    packed tails"), each lane runs a slice-by-4 chain over its piece, and a segmented
//    inclusive scan with uniform x^(8*64*d) shifts combines the pieces of each packet.
//    Waves get equal piece counts, and rotate their issue priority.
//
// All algebra (tables, operators) is generated on the host in crc32_math.hpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <unordered_map>
#include <string>
#include <vector>

#include "crc32_math.hpp"
#include "wtp_crc32.h"

namespace wtp {

// ------------------------------------------------------------------------------------
// Device constant tables (one block per device, built once on the host)
// ------------------------------------------------------------------------------------
constexpr int kG = 16;                       // lanes per packet in the braided kernel
constexpr int kBraids = 4 * kG;              // 64 braids x 4-byte words
constexpr uint32_t kBraidBlock = 4 * kBraids;  // one row = 256 bytes
#ifndef WTP_PC_S  // piece bytes in the general kernel (128 was an A/B variant; it no
                  // longer compiles: the verify fix-up's LDS static_assert below rejects it)
#define WTP_PC_S 64
#endif
constexpr int kPieceS = WTP_PC_S;
static_assert(kPieceS == 64 || kPieceS == 128, "piece size");
constexpr uint32_t kHinitWords = (kPieceS + 4) & ~3;  // shift(~0, h), h = 0..kPieceS, padded
constexpr uint32_t kMaxVarLen = 4096;
constexpr uint64_t kSubBatch = 1ull << 28;      // packets per general-kernel launch (32-bit store offsets)        // 64 pieces x 64 B: one packet per wave max

constexpr uint32_t OFF_BRAID = 0;            // 4x256 braid word tables (advance 256 B)
constexpr uint32_t OFF_INV = 1024;           // 6 ops: x^-32, x^-64, x^-128, x^-256, x^-512, x^-1024
constexpr uint32_t OFF_S4 = OFF_INV + 6 * 1024;   // 4x256 slice-by-4 word tables
constexpr uint32_t OFF_FWD = OFF_S4 + 1024;       // 6 ops: x^(8*S*d), d = 1..32 (S = kPieceS)
constexpr uint32_t OFF_HINIT = OFF_FWD + 6 * 1024;  // shift(~0, h), h = 0..S (head-piece init)
// k_stream (packed mixed lengths): T256 = shift by one 32-B block; 38 nibble operators
// (8 tables x 16 words each): shift by 128 * 2^k B (k = 0..5, the lane scan), then the
// payload-length shift in four 3-bit levels (level k, digit j: shift by j * 8^k B).
constexpr uint32_t OFF_T256 = OFF_HINIT + kHinitWords;
constexpr uint32_t kStNibOps = 6 + 32;
constexpr uint32_t OFF_NIB = OFF_T256 + 1024;
constexpr uint32_t OFF_X64 = OFF_NIB + kStNibOps * 128;  // x^(8*64): joins the two chains of a 128-B piece
constexpr uint32_t OFF_S8 = OFF_X64 + 1024;  // 4x256 word tables, a word then 4 zero bytes (split piece chains)
constexpr uint32_t TAB_WORDS = OFF_S8 + 1024;

// LDS images (staggered table sets are described at StagKeys below).
constexpr uint32_t kOpBytes = 4096;  // a plain operator: 4 byte tables x 256 words
// k_fixed_braid: region A = {braid tables, x^-32}, region B = {x^-128, x^-1024} (staggered,
// conflict-free), then the 16 waves' 2 KiB transposition slots.
constexpr uint32_t kBraidXpose = 131072;
constexpr uint32_t kBraidLdsWords = (kBraidXpose + 16 * 2048) / 4;  // 163,840 B

namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// Explicit global (address space 1) pointers for the streaming loads: a select between
// two generic pointers defeats address-space inference and degrades to flat_load, which
// also counts on lgkmcnt and serialises with the LDS lookups.
typedef const __attribute__((address_space(1))) uint8_t gu8;
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
// Explicit LDS (address space 3) pointers for the general kernel's staging slots and
// flags: the accesses are ds_* by construction, never flat.
typedef __attribute__((address_space(3))) char lchar;
typedef __attribute__((address_space(3))) u32x4 lu32x4;
typedef __attribute__((address_space(3))) u32x2 lu32x2;
typedef __attribute__((address_space(3))) uint8_t lu8;

// Per-wave phase timestamps for tools/pprobe.hip (built with -DWTP_PROBE=1 there and
// compiled out of the product): slot k of wave (block, wave) gets value v, e.g. a
// 100 MHz s_memrealtime stamp.
#ifndef WTP_PROBE
#define WTP_PROBE 0
#endif
#if WTP_PROBE
__device__ uint64_t *g_probe;
#define PC_PROBE(k, v)                                                                                  \
    do {                                                                                                \
        if (lane == 0u) g_probe[(uint64_t(blockIdx.x) * 16u + wave) * 8u + (k)] = (v);                 \
    } while (0)
#else
#define PC_PROBE(k, v) \
    do {               \
    } while (0)
#endif

__device__ __forceinline__ uint32_t lds_rd(const char *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(lds + byte_addr);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c);
// w ^ f(v) for a linear operator f stored as 4 byte tables (256 words each) at LDS byte
// offset base: each byte address is one v_bfe + one v_lshl_or, the five-way XOR two
// v_bitop3 (the piece kernel's scan levels)
__device__ __forceinline__ uint32_t op_apply_fold(const char *lds, uint32_t base, uint32_t v, uint32_t w) {
    const uint32_t a0 = (__builtin_amdgcn_ubfe(v, 0, 8) << 2) | base;
    const uint32_t a1 = (__builtin_amdgcn_ubfe(v, 8, 8) << 2) | (base + 1024u);
    const uint32_t a2 = (__builtin_amdgcn_ubfe(v, 16, 8) << 2) | (base + 2048u);
    const uint32_t a3 = ((v >> 24) << 2) | (base + 3072u);
    return xor3(xor3(lds_rd(lds, a0), lds_rd(lds, a1), lds_rd(lds, a2)), lds_rd(lds, a3), w);
}

// ---- staggered 8-copy tables (conflict-free with a quarter of the replication) ------
// A "table set" is 4 byte-tables (256 u32 each) of one linear map.  Each 32-lane half of
// a wave is split into 4 groups of 8 lanes; in lookup instruction s, group g reads table
// (s + g) & 3, so the 4 groups always hit 4 different tables, and copy c = lane & 7 of
// table t lives in bank 8t + c: all 32 lanes touch distinct banks whatever the bytes.
// Every lane still XORs one entry of each of the 4 tables, just in a lane-dependent
// order.  Layout: 256-B rows, one per byte value e; two table sets per 64 KiB region:
//   byte address = region*65536 + e*256 + set*128 + t*32 + c*4.
// The per-lane key holds everything but e; v_perm_b32 with a per-lane selector drops the
// data byte t into bits 8..15, so each lookup is one v_perm + one ds_read_b32 (the set
// bit is the instruction's immediate offset).
struct StagKeys {
    uint32_t kA[4], kB[4], sel[4];
    __device__ __forceinline__ explicit StagKeys(uint32_t lane) {
        const uint32_t h = lane & 31u, g = (h >> 3) & 3u, c = h & 7u;
#pragma unroll
        for (uint32_t s = 0; s < 4; ++s) {
            const uint32_t t = (s + g) & 3u;
            kA[s] = (t << 5) | (c << 2);
            kB[s] = kA[s] | (1u << 16);
            sel[s] = 0x0C020000u | ((4u + t) << 8);
        }
    }
};

template <uint32_t OFF>
__device__ __forceinline__ uint32_t stag_apply(const char *lds, const uint32_t (&key)[4], const uint32_t (&sel)[4],
                                               uint32_t x) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, key[0], sel[0]);
    const uint32_t a1 = __builtin_amdgcn_perm(x, key[1], sel[1]);
    const uint32_t a2 = __builtin_amdgcn_perm(x, key[2], sel[2]);
    const uint32_t a3 = __builtin_amdgcn_perm(x, key[3], sel[3]);
    return (lds_rd(lds, a0 + OFF) ^ lds_rd(lds, a1 + OFF)) ^ (lds_rd(lds, a2 + OFF) ^ lds_rd(lds, a3 + OFF));
}

// Fill one table set (1024 words from global: table t at g[256 t]) into the staggered image.
// Store j (of 2048) writes the 16-B half h = j & 1 of table t = (j >> 1) & 3's 8 copies of
// entry e = j >> 3, so each 8-lane ds_write_b128 group covers 128 contiguous bytes (one
// entry per 32 B, lanes 256 B apart, was 8-way bank-conflicted: 3.4 us per launch).
__device__ __forceinline__ uint32_t stag_fill_word(uint32_t j) { return ((j >> 1) & 3u) * 256u + (j >> 3); }
__device__ __forceinline__ uint32_t stag_fill_off(uint32_t j) { return (j >> 3) * 256u + ((j >> 1) & 3u) * 32u + (j & 1u) * 16u; }
__device__ __forceinline__ void fill_stag(char *lds, uint32_t region, uint32_t set, const uint32_t *__restrict__ g) {
    for (uint32_t j = threadIdx.x; j < 2048; j += blockDim.x) {
        const uint32_t v = g[stag_fill_word(j)];
        *reinterpret_cast<u32x4 *>(lds + region * 65536u + set * 128u + stag_fill_off(j)) = u32x4{v, v, v, v};
    }
}

// Staggered fill of NS table sets with every global load of a thread issued before any
// LDS write.  The tables are usually evicted from L2 by the stream between launches, and
// the load-write loop of fill_stag paid one memory latency per word: entry to first
// round took 5.9 us in every braided launch (tools/bprobe.py), a third of a C2 launch.
struct StagSet {
    const uint32_t *g;  // 4 byte tables (1024 words)
    uint32_t off;       // region * 65536 + set * 128
};
// load() issues the loads, store() writes LDS: a kernel issues the table loads before
// its first data loads, since vmcnt completes in order and the table writes would
// otherwise wait for the first round's data (the fill ended 4.4 us after entry).
#ifndef WTP_FILL_X4_PC
#define WTP_FILL_X4_PC 1  // the same for the piece kernel's 1024-thread fill: C5 -0.5..0.8%, 64 K mixed -3% (r06c)
#endif
#ifndef WTP_FILL_X4
#define WTP_FILL_X4 1  // 16-B table loads, each feeding 4 stores (<= 512 threads; 0: one dword per store, A/B builds)
#endif
template <int NS, int THREADS>
struct StagFill {
    static_assert(THREADS <= 1024 && 2048 % THREADS == 0, "StagFill");
    // X4 form: load slot s of a set (512 per set) covers table t = (s >> 1) & 3, entries
    // 4g .. 4g+3 (g = s >> 3), half h = s & 1 of their 8 copies: one 16-B global load, four
    // 16-B LDS stores (each 8-lane group still writes 128 contiguous bytes of one row).
    // A quarter of the prologue's vector memory instructions: C2 (64 K packets) 15.46 ->
    // 14.29 us from a graph, 16 K 7.03 -> 5.98, 1 M 216.5 -> 214.9 (interleaved,
    // profiles/r04fx).  The piece kernel's 1024-thread fill too since round 6 (7 -> 4 loads
    // per thread): C5 1 M 47.4 -> 47.0-47.2 us median, 64 K mixed 19.2 -> 18.6-18.7
    // (interleaved, both library orders, profiles/r06c).
    static constexpr bool kX4 = WTP_FILL_X4 && (THREADS <= 512 || WTP_FILL_X4_PC);
    static constexpr int PER = kX4 ? NS * 512 / THREADS : NS * 2048 / THREADS;  // loads per thread
    typename std::conditional<kX4, u32x4, uint32_t>::type v[PER];
    __device__ __forceinline__ void load(const StagSet (&sets)[NS]) {
        if constexpr (kX4) {
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const uint32_t sidx = (uint32_t(k * THREADS) + threadIdx.x) & 511u;
                if constexpr (THREADS <= 512) {  // one set per k
                    v[k] = *reinterpret_cast<const u32x4 *>(sets[(k * THREADS) >> 9].g + ((sidx >> 1) & 3u) * 256u +
                                                            4u * (sidx >> 3));
                } else {  // the set as an offset from set 0 (a select between pointers would be flat)
                    const uint32_t si = (uint32_t(k * THREADS) + threadIdx.x) >> 9;
                    ptrdiff_t gofs = 0;
#pragma unroll
                    for (int i = 1; i < NS; ++i) gofs = si == uint32_t(i) ? sets[i].g - sets[0].g : gofs;
                    v[k] = *reinterpret_cast<const u32x4 *>(sets[0].g + gofs + ((sidx >> 1) & 3u) * 256u + 4u * (sidx >> 3));
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < PER; ++k)
                v[k] = sets[(k * THREADS) >> 11].g[stag_fill_word((uint32_t(k * THREADS) + threadIdx.x) & 2047u)];
        }
    }
    __device__ __forceinline__ void store(char *lds, const StagSet (&sets)[NS]) const {
        if constexpr (kX4) {
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const uint32_t sidx = (uint32_t(k * THREADS) + threadIdx.x) & 511u;
                uint32_t soff;
                if constexpr (THREADS <= 512) {
                    soff = sets[(k * THREADS) >> 9].off;
                } else {
                    const uint32_t si = (uint32_t(k * THREADS) + threadIdx.x) >> 9;
                    soff = sets[0].off;
#pragma unroll
                    for (int i = 1; i < NS; ++i) soff = si == uint32_t(i) ? sets[i].off : soff;
                }
                const uint32_t base = soff + (sidx >> 3) * 1024u + ((sidx >> 1) & 3u) * 32u + (sidx & 1u) * 16u;
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i)
                    *reinterpret_cast<u32x4 *>(lds + base + i * 256u) = u32x4{v[k][i], v[k][i], v[k][i], v[k][i]};
            }
        } else {
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const uint32_t j = (uint32_t(k * THREADS) + threadIdx.x) & 2047u;
                *reinterpret_cast<u32x4 *>(lds + sets[(k * THREADS) >> 11].off + stag_fill_off(j)) =
                    u32x4{v[k], v[k], v[k], v[k]};
            }
        }
    }
};
template <int NS, int THREADS>
__device__ __forceinline__ void fill_stag_batch(char *lds, const StagSet (&sets)[NS]) {
    StagFill<NS, THREADS> f;
    f.load(sets);
    f.store(lds, sets);
}

// ------------------------------------------------------------------------------------
// 1. braided fixed-length kernel
// ------------------------------------------------------------------------------------
// Packet p occupies base[p*stride, p*stride + len); base, stride and len are multiples
// of 16 and 256*(ROWS-1) < len <= 256*ROWS.  The packet is placed in a frame of ROWS
// rows x 256 B whose start is 128-B aligned when the frame still covers the packet end
// (else 64-B aligned, else right-aligned): each wave instruction then reads four
// line-aligned 256-B segments (right-aligned frames were 4% slower, kbench A/B).  Frame
// bytes before the packet are free zeros (R_0(0^k || M) = R_0(M)); the T = 16t zero
// bytes after it are undone at the flush with x^(-128 t).
__device__ __forceinline__ uint32_t braid_lead(uintptr_t st, uint32_t len, uint32_t frame) {
    const uint32_t l128 = uint32_t(st & 127u), l64 = uint32_t(st & 63u);
    return l128 + len <= frame ? l128 : (l64 + len <= frame ? l64 : frame - len);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// x ^ apply(set, x) folded with the next data word w: xor3(xor3(l0, l1, l2), l3, w).
template <uint32_t OFF>
__device__ __forceinline__ uint32_t stag_apply3x(const char *lds, const uint32_t (&key)[4], const uint32_t (&sel)[4],
                                                 uint32_t x, uint32_t w) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, key[0], sel[0]);
    const uint32_t a1 = __builtin_amdgcn_perm(x, key[1], sel[1]);
    const uint32_t a2 = __builtin_amdgcn_perm(x, key[2], sel[2]);
    const uint32_t a3 = __builtin_amdgcn_perm(x, key[3], sel[3]);
    return xor3(xor3(lds_rd(lds, a0 + OFF), lds_rd(lds, a1 + OFF), lds_rd(lds, a2 + OFF)), lds_rd(lds, a3 + OFF), w);
}

template <uint32_t OFF>
__device__ __forceinline__ uint32_t stag_apply3(const char *lds, const uint32_t (&key)[4], const uint32_t (&sel)[4],
                                                uint32_t x) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, key[0], sel[0]);
    const uint32_t a1 = __builtin_amdgcn_perm(x, key[1], sel[1]);
    const uint32_t a2 = __builtin_amdgcn_perm(x, key[2], sel[2]);
    const uint32_t a3 = __builtin_amdgcn_perm(x, key[3], sel[3]);
    return xor3(lds_rd(lds, a0 + OFF), lds_rd(lds, a1 + OFF), lds_rd(lds, a2 + OFF)) ^ lds_rd(lds, a3 + OFF);
}

// Operator stored as 8 nibble tables of 16 words at LDS byte address `base` (which may
// differ per lane): f(v) = XOR_i N_i[(v >> 4i) & 15].  A table's 16 words sit in 16
// consecutive banks, so a wave-uniform operator never conflicts.
__device__ __forceinline__ uint32_t nib_apply(const char *lds, uint32_t base, uint32_t v) {
    uint32_t l[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) l[i] = lds_rd(lds, base + 64u * i + 4u * __builtin_amdgcn_ubfe(v, 4 * i, 4));
    return xor3(xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5]), l[6] ^ l[7]);
}

// Wave issue priority, rotated (general kernel).  The SIMD arbiter favours the oldest of
// equal-priority waves: with static per-wave work, the four waves sharing a SIMD ran at
// unequal speeds (k_pieces on C5: 2.8 us per round for the oldest, 4.2 us for the
// youngest; tools/pprobe.py) and the launch waited for the youngest while its SIMD ran
// nearly empty.  Each wave steps its priority through 0..3 per round (x = round counter
// + the wave's age rank), so each spends a quarter of its rounds at every level: C5
// 57.6 -> 54.6 us (interleaved A/B, tools/ab_c5.py).  The braided kernel, at the read
// ceiling, lost 1% with it (and 2.5% with dynamic per-workgroup group claims).
__device__ __forceinline__ void rotate_prio(uint32_t x) {
    switch (x & 3u) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// Epilogues of the braided kernel.  A flush hands lane 2P + h (h = 0) the result of
// packet slot q = P & 3 of round k = P >> 2 of its 8-round group; pre() issues, one
// group ahead, the loads put() will need (so a flush never waits on memory).
struct CrcBEpi {  // out[p] = crc
    static constexpr bool kCopy = false;  // see BuildBEpi
    static constexpr bool kFixup = false;  // see VerifyBEpi
    static constexpr int kThreads = 512;  // the launcher's workgroup size (launch_fixed_braid)
    static constexpr int kDepth = 2;      // register sets in the main loop (rounds in flight + 1)
    static constexpr int kDiag = 0;       // DIAG of the production instantiation
    static constexpr int kBound = 1024;   // __launch_bounds__ (kbench A/B builds launch up to 1024)
    static constexpr int kLoadAux = 2;   // rows >= 1 stream (nt); row 0 is temporal (see k_fixed_braid)
    static constexpr bool kHold = false;  // CrcHoldBEpi: results held in LDS, stored in bursts
    static constexpr const char *kName = "CrcBEpi";  // wtp_last_kernel()
    __device__ __forceinline__ uint32_t lead(uint64_t, uint32_t st, uint32_t len, uint32_t frame) const {
        return braid_lead(st, len, frame);
    }
    uint32_t *out;
    uint32_t cinit;  // init_const(len)
    struct Pre {};
    __device__ __forceinline__ void pre(uint64_t, Pre &) const {}
    __device__ __forceinline__ bool listed(bool, const Pre &) const { return false; }
    __device__ __forceinline__ void put(uint64_t p, uint32_t v, bool on, const Pre &) const {
        if (on) out[p] = v ^ cinit;
    }
};
// The same epilogue for long batches (the launcher's rule): k_fixed_braid holds the CRCs in
// LDS and stores them in bursts (see kDump there).
struct CrcHoldBEpi : CrcBEpi {
    static constexpr bool kHold = true;
    static constexpr const char *kName = "CrcHoldBEpi";
};
// Receiver verify over a datagram ring: the kernel runs on base = ring + 16 with the
// ring's "full" payload length len (1456 for a WTP ring: 1472-B datagrams, whatever the
// slot stride, e.g. wReceiver's 1504-B slots that hold a 1500-B recvfrom buffer).
// Datagrams with recv_len == 16 + len are decided here (Receiver.cpp:203-206:
// ntohl(header.checksum) == crc32(payload)).  Every other datagram (short, empty, runt,
// 1473-1500 B, oversize) first gets ok = 0, crc = 0, is counted, and the workgroup's
// fix-up phase (verify_fixup, after its braided rounds) recomputes it with the
// reference's semantics: one launch, no state outside the caller's buffers.
struct VerifyBEpi {
    static constexpr bool kHold = false;  // see CrcBEpi
    static constexpr const char *kName = "VerifyBEpi";
    static constexpr bool kCopy = false;
    static constexpr bool kFixup = true;  // see VerifyBEpi
    static constexpr int kThreads = 512;  // verify_fixup's LDS layout assumes 8 waves
    static constexpr int kDepth = 2;
    static constexpr int kDiag = 0;
    static constexpr int kBound = 1024;
    static constexpr int kLoadAux = 2;   // rows >= 1 stream (nt); row 0 is temporal (see k_fixed_braid)
    __device__ __forceinline__ uint32_t lead(uint64_t, uint32_t st, uint32_t len, uint32_t frame) const {
        return braid_lead(st, len, frame);
    }
    const uint32_t *rl;
    const uint8_t *ring;  // 16-B aligned, stride % 16 == 0: header words are aligned
    uint64_t stride;
    uint8_t *ok;
    uint32_t *crc;  // may be null
    uint32_t *status;
    uint32_t cinit;
    uint64_t n;
    uint32_t full;  // recv_len of the datagrams this pass decides (16 + len)
    struct Pre {
        uint32_t r, h;
    };
    __device__ __forceinline__ void pre(uint64_t p, Pre &q) const {
        typedef const __attribute__((address_space(1))) uint32_t gu32;
        const uint64_t pc = p < n ? p : n - 1;
        q.r = ((gu32 *)rl)[pc];
        q.h = *(gu32 *)((gu8 *)ring + pc * stride + 12);
    }
    // true for a datagram the fix-up phase must finish
    __device__ __forceinline__ bool listed(bool on, const Pre &q) const { return on && q.r != full; }
    __device__ __forceinline__ void put(uint64_t p, uint32_t v, bool on, const Pre &q) const {
        if (!on) return;
        const uint32_t c = v ^ cinit;
        const bool mine = q.r == full;
        ok[p] = mine && bswap32(q.h) == c ? 1 : 0;
        if (crc) crc[p] = mine ? c : 0u;
    }
};

// Fused DATA packet builder (Packet.cpp:9-14,40-47,
// Sender.cpp:187-197): payload p (stride len) -> wire[p*wstride ..) = big-endian
// PacketHeader{DATA, seq0 + p, len, crc} || payload.  kCopy: every 16-B chunk the
// kernel loads is also stored into its wire slot in the same round (one buffer store
// per row, out-of-range offset for chunks outside the packet), so the payload is read
// from HBM once; the header follows at the flush.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t nbytes);
#ifndef WTP_BUILD_THREADS
#define WTP_BUILD_THREADS 128  // fused builder workgroup size (A/B builds: 256, 512)
#endif
#ifndef WTP_BUILD_DIAG
#define WTP_BUILD_DIAG 0
#endif
#ifndef WTP_BUILD_DEPTH
#define WTP_BUILD_DEPTH 2  // fused builder register sets (A/B builds: 3)
#endif
#ifndef WTP_BUILD_SAUX
#define WTP_BUILD_SAUX 2  // cache policy of the builder's wire stores, rows >= 1: nt (A/B builds: 0)
#endif
#ifndef WTP_BUILD_WLEAD
#define WTP_BUILD_WLEAD 1  // frame lead from the wire slot's alignment (0: the source's, A/B builds)
#endif
#ifndef WTP_BUILD_LAUX
#define WTP_BUILD_LAUX 2  // builder loads, rows >= 1 (A/B builds: 0 = temporal)
#endif
#ifndef WTP_BUILD_SAUX0
#define WTP_BUILD_SAUX0 0  // the same for row 0 (it shares a 64-B segment with the header)
#endif
struct BuildBEpi {
    static constexpr bool kHold = false;  // see CrcBEpi
    static constexpr const char *kName = "BuildBEpi";
    static constexpr bool kCopy = true;
    static constexpr bool kFixup = false;  // see VerifyBEpi
    // launched at 128 threads: the bound lets the copy rows keep their registers (at the
    // generic 1024 bound the compiler had 128 VGPRs and spilled 192-240 of them, 484 B of
    // scratch per lane)
    static constexpr int kThreads = WTP_BUILD_THREADS;
    static constexpr int kDepth = WTP_BUILD_DEPTH;
    static constexpr int kDiag = WTP_BUILD_DIAG;  // ablation builds only (wrong CRCs)
    static constexpr int kBound = WTP_BUILD_THREADS;
    static constexpr int kLoadAux = WTP_BUILD_LAUX;
    uint8_t *wire;
    uint64_t wstride;  // multiple of 16
    uint32_t seq0, len;
    uint32_t *wire_len;  // may be null
    uint32_t cinit;
    struct Pre {};
    __device__ __forceinline__ void pre(uint64_t, Pre &) const {}
    // frame lead: with WTP_BUILD_WLEAD the frame rows map to 64-B aligned wire addresses
    // (lead = wire payload address mod 64) when the frame still covers the packet
    __device__ __forceinline__ uint32_t lead(uint64_t p, uint32_t st, uint32_t l, uint32_t frame) const {
        if (WTP_BUILD_WLEAD) {
            const uint32_t w = (uint32_t(reinterpret_cast<uintptr_t>(wire)) + uint32_t(p) * uint32_t(wstride) + 16u) & 63u;
            if (w + l <= frame) return w;
        }
        return braid_lead(st, l, frame);
    }
    // buffer resource over the 4 wire slots of round packets p0 .. p0+3
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t round_rsrc(uint64_t p0) const {
        return make_rsrc(wire + p0 * wstride, uint32_t(4 * wstride));
    }
    __device__ __forceinline__ void copy(__amdgpu_buffer_rsrc_t rs, uint32_t q, int32_t rel, bool valid, u32x4 w,
                                         bool row0) const {
        const uint32_t o = valid ? q * uint32_t(wstride) + 16u + uint32_t(rel) : 0x80000000u;
        // The frame lead follows the wire slot (lead()), so rows >= 1 store whole 64-B
        // segments of the slot and stream (nt); row 0 shares its first segment with the
        // header written at the flush and stays write-back, so L2 merges the two.
        // Interleaved A/B, 1 M x 1456 B -> 1472-B slots (profiles/r03h, r03m): all
        // write-back with the source's frame lead 635.9 us; nt rows >= 1 615.1 / 619.7 us;
        // wire-aligned lead + nt rows >= 1 597.1 us; the same with temporal loads 606.2;
        // nt row 0 too 637.3; wire-aligned, all write-back 631.5.
        if (row0)
            __builtin_amdgcn_raw_buffer_store_b128(w, rs, int(o), 0, WTP_BUILD_SAUX0);
        else
            __builtin_amdgcn_raw_buffer_store_b128(w, rs, int(o), 0, WTP_BUILD_SAUX);
    }
    __device__ __forceinline__ bool listed(bool, const Pre &) const { return false; }
    __device__ __forceinline__ void put(uint64_t p, uint32_t v, bool on, const Pre &) const {
        if (!on) return;
        const u32x4 h = {bswap32(WTP_TYPE_DATA), bswap32(seq0 + uint32_t(p)), bswap32(len), bswap32(v ^ cinit)};
        *reinterpret_cast<u32x4 *>(wire + p * wstride) = h;
        if (wire_len) wire_len[p] = 16u + len;
    }
};

__device__ __forceinline__ void verify_fixup(char *lds, const VerifyBEpi &epi, const uint32_t *gtab, uint32_t nfix,
                                             uint64_t rstep, uint32_t wave, uint32_t lane);

// k_fixed_braid<ROWS> — 16 lanes own one packet, a wave holds 4 packets per round.
//
// Main loop (per round, per lane): ROWS 16-B loads, one per frame row; each dword
// feeds one of the lane's 4 braids (CRC streams over every 64th dword of the frame,
// tables advancing 256 B).  B <- T(B ^ w) with the next row's word folded into the
// lookup XOR.  The 4 braids are folded in-lane, b0 ^ x^-32 (b1 ^ x^-32 (b2 ^ x^-32 b3)),
// giving one column value v_j per lane; the packet's CRC register is T applied to
// XOR_j x^(-128 j) v_j times x^(-128 t) for its t trailing zero chunks (the last row's
// advance T commutes with the x^-k, so it runs once per packet at the flush instead of
// once per braid per round: 16 of 108 lookups per round gone).
//
// Combine (Horner through LDS): each round writes its 64 column values into the wave's
// 2 KiB transposition slot at [k][q][j]; every 8 rounds the flush has lane 2P + h read
// columns 8h .. 8h+7 of packet P = 4k + q (two ds_read_b128), evaluate them by Horner's
// rule with x^-128 (7 applies), move the h = 1 half by x^-1024, apply the trailing-zero
// fix to both halves (t <= 15 masked x^-128 steps, wave-uniform count) and XOR the pair
// (DPP lane ^ 1).  This replaced a 4-level cross-lane tree in which half the lanes of
// each level idled: 6.07 -> 6.43 TB/s.
//
// Loads: all rows go through one buffer resource per round (SGPRs) whose range ends at
// the last byte of packet n-1, so lanes of packets past n and rounds past the end read
// zeros without a request; frame bytes outside a packet (first and last row only) use an
// out-of-range offset, which needs neither a clamp nor zeroing.  Row 0 holds the cache
// line a packet shares with the previous packet's last row: a normal (temporal) load
// keeps it in L2 for that row, every other row streams (nt).  All-nt re-fetched those
// lines (HBM traffic 1.069x algorithmic, 4.7% slower); all-temporal was 8.7% slower.
//
// Power: the MI355X runs this kernel at its board limit; the effective clock under the
// lookups is ~4% below the load-only skeleton's, and the kernel's cycle count is the
// skeleton's (kbench + GRBM_GUI_ACTIVE, profiles/).  Every VALU/LDS instruction in the
// loop therefore costs bandwidth: XORs are v_bitop3_b32 (3-input, new on gfx950), a
// lookup address is one v_perm_b32 into the staggered conflict-free tables, results are
// stored once per 8 rounds (on gfx950 stores share vmcnt with loads), and long batches
// (CrcHoldBEpi) hold them in LDS and store them once per 128 rounds (see kDump).
//
// DIAG (ablation builds only, tools/kbench.hip): bit0 replaces the table lookups by
// XOR/shift, bit1 skips the in-lane fold, bit2 drops the per-round wave-priority rotation;
// access-pattern ablations: bit4 drops the result stores, bit5 loads row 0
// nt as well, bit6 right-aligns every frame to its packet end (lead = frame - len), bit10
// holds the results in LDS for any CRC epilogue (CrcHoldBEpi does without it, see kDump),
// bit11 turns that off.  Production instantiations use DIAG = 0.  (Rejected round-4 forms,
// in git history at commit ba1b383: blocked-8 round order, a workgroup result ring, a
// deferred flush.)
template <int ROWS, int DIAG = 0, class BEpi = CrcBEpi>
__global__ __launch_bounds__(BEpi::kBound) void k_fixed_braid(const uint8_t *__restrict__ base, uint32_t stride,
                                                      uint32_t len, uint64_t n, BEpi epi,
                                                      const uint32_t *__restrict__ gtab) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_w[kBraidLdsWords];
    char *lds = reinterpret_cast<char *>(lds_w);
    constexpr uint32_t kGroup = 8;  // rounds per flush (2 KiB slot per wave)

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    PC_PROBE(0, __builtin_amdgcn_s_memrealtime());
    const uint32_t nwave = blockDim.x >> 6;
    const uint32_t j = lane & (kG - 1);  // braid group (column) within the packet
    const uint32_t q = lane >> 4;        // packet slot within the wave (0..3)
    const StagKeys K(lane);

    constexpr uint32_t kFrame = 256u * ROWS;
    const uint64_t rounds = (n + 3) >> 2;
    // Round order: grid-interleaved, wave (b, w) takes rounds b*nwave + w + i*rstep, so the
    // whole grid moves through the batch as one front.  (A contiguous block of rounds per
    // workgroup, and one per XCD class b % 8, were built in round 4 and measured slower at
    // every size, DESIGN 7.10, as was a translation-prefetch wave; code in git history,
    // commits f56e6d4 and 8c994a0.)
    const uint64_t rstep = uint64_t(gridDim.x) * nwave;
    const uint32_t qoff = q * stride;
    gu8 *const gbase = (gu8 *)base;

    struct Round {
        u32x4 w[ROWS];
        uint32_t lead;
    };
    // Round rr: packets 4rr .. 4rr+3.  rr is wave-uniform.
    auto load_round = [&](uint64_t rr, Round &R) {
        const bool live = rr < rounds;
        const uint64_t p0 = rr * 4;
        gu8 *sb = gbase + (live ? p0 * stride : 0);
        const uint64_t last = live ? n - 1 - p0 : 0;
        const uint32_t nrec = !live ? 0u : (last >= 3 ? 3u * stride + len : uint32_t(last) * stride + len);
        const __amdgpu_buffer_rsrc_t rs = make_rsrc((const void *)sb, nrec);
        const uint32_t lead = (DIAG & 64) ? kFrame - len
                                          : epi.lead(p0 + q, uint32_t(reinterpret_cast<uintptr_t>((const void *)sb)) + qoff, len, kFrame);
        R.lead = lead;
        const uint32_t fo = qoff - lead + j * 16u;
#pragma unroll
        for (int i = 0; i < ROWS; ++i) {
            uint32_t o = fo + uint32_t(i) * 256u;
            if (i == 0 || i == ROWS - 1) {  // may hold frame bytes outside the packet
                const int32_t rel = int32_t(uint32_t(i) * 256u + j * 16u) - int32_t(lead);
                o = (rel >= 0 && rel < int32_t(len)) ? o : 0x80000000u;
            }
            if (i == 0)
                R.w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(o), 0, (DIAG & 32) ? BEpi::kLoadAux : 0));
            else
                R.w[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(o), 0, BEpi::kLoadAux));
        }
    };

    lchar *const xs = (lchar *)(lds + kBraidXpose + wave * 2048u);
    uint32_t k = 0;            // rounds written to the slot since the last flush
    uint64_t rfirst = 0;       // round of slot row 0
    typename BEpi::Pre pre{};  // epilogue loads for the current group
    uint32_t nfix = 0;         // datagrams this wave left to the fix-up phase (verify)
    // Results (CrcHoldBEpi): a flush writes its 32 CRCs into the wave's LDS result buffer (2 KiB
    // at transposition slot 8 + wave, free at 8 waves) instead of storing them, and every
    // 16 flushes (128 rounds) the wave stores the buffer in one burst of two dwordx4 stores
    // per lane.  A 1 M batch then writes its 4 MiB of results near the end of the launch
    // instead of 32 B per wave every 8 rounds among the reads: 1 M x 1456 B alternating
    // between two buffers 232.8 -> 225.9 us, same buffer 221.9 -> 220.5 us (interleaved
    // kbench, profiles/r04r; no stores at all: 221.7 / 219.1).  Waiting for the store acks
    // was not it (deferring the flush past the next loads: neutral, profiles/r04q), nor
    // partial lines (whole-line stores per wave: neutral, profiles/r04o).
    constexpr bool kDump = ((BEpi::kHold && !(DIAG & 2048)) || (DIAG & 1024)) && !BEpi::kCopy && !BEpi::kFixup;
    // (the launcher picks CrcHoldBEpi for long batches only; the buffer needs 8 waves)
    const bool hold = kDump && nwave <= 8;
#ifndef WTP_BR_HOLD
#define WTP_BR_HOLD 16  // flushes held per burst (A/B builds: 4, 8)
#endif
    constexpr uint32_t kHoldG = WTP_BR_HOLD;
    static_assert(kHoldG == 4 || kHoldG == 8 || kHoldG == 16, "hold capacity");
    lchar *const rbuf = (lchar *)(lds + kBraidXpose + (8u + wave) * 2048u);
    uint32_t dgroups = 0;    // flushes held in rbuf
    uint64_t dfirst = 0;     // round of the first held flush's row 0 (this wave)
    auto dump = [&]() {
        if constexpr (kDump) {
            __builtin_amdgcn_wave_barrier();
            // buffer resource from this dump's first packet: its offsets stay below
            // 16 * kHoldG * 8 * rstep (< 2^31) and the range ends at packet n for any n
            const uint64_t pb0 = 4 * dfirst, left = n > pb0 ? n - pb0 : 0;
            const __amdgpu_buffer_rsrc_t ors =
                make_rsrc(epi.out + pb0, left >= (1ull << 29) ? 0x80000000u : uint32_t(4 * left));
#pragma unroll
            for (uint32_t t = 0; t < (kHoldG * 8 + 63) / 64; ++t) {
                const uint32_t si = lane + 64u * t;  // segment: flush si >> 3, row si & 7
                const u32x4 v = *(const lu32x4 *)(rbuf + si * 16u);
                const uint64_t rr = dfirst + (8u * uint64_t(si >> 3) + (si & 7u)) * rstep;
                const uint64_t pb = 4 * rr;
                const uint32_t o = uint32_t(4 * (pb - pb0));
                const bool live = (si >> 3) < dgroups && rr < rounds;
                if (__builtin_amdgcn_ballot_w64(live && pb + 4 > n) == 0) {
                    __builtin_amdgcn_raw_buffer_store_b128(v, ors, live ? int(o) : int(0x80000000u), 0, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b32(v.x, ors, live && pb + 0 < n ? int(o) : int(0x80000000u), 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(v.y, ors, live && pb + 1 < n ? int(o + 4) : int(0x80000000u), 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(v.z, ors, live && pb + 2 < n ? int(o + 8) : int(0x80000000u), 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(v.w, ors, live && pb + 3 < n ? int(o + 12) : int(0x80000000u), 0, 0);
                }
            }
            __builtin_amdgcn_wave_barrier();
            dgroups = 0;
        }
    };
    auto group_packet = [&](uint64_t g0) { return (g0 + uint64_t(lane >> 3) * rstep) * 4 + ((lane >> 1) & 3u); };

    auto flush = [&](uint64_t next_g0, bool more) {
        __builtin_amdgcn_wave_barrier();
        const u32x4 lo = *(const lu32x4 *)(xs + lane * 32u), hi = *(const lu32x4 *)(xs + lane * 32u + 16u);
        uint32_t acc = hi.w;
        acc = stag_apply3x<0>(lds, K.kB, K.sel, acc, hi.z);
        acc = stag_apply3x<0>(lds, K.kB, K.sel, acc, hi.y);
        acc = stag_apply3x<0>(lds, K.kB, K.sel, acc, hi.x);
        acc = stag_apply3x<0>(lds, K.kB, K.sel, acc, lo.w);
        acc = stag_apply3x<0>(lds, K.kB, K.sel, acc, lo.z);
        acc = stag_apply3x<0>(lds, K.kB, K.sel, acc, lo.y);
        acc = stag_apply3x<0>(lds, K.kB, K.sel, acc, lo.x);
        const uint32_t h = lane & 1u;
        {
            const uint32_t y = stag_apply3<128>(lds, K.kB, K.sel, acc);  // x^-1024
            acc = h ? y : acc;
        }
        const uint64_t rr = rfirst + uint64_t(lane >> 3) * rstep;
        const uint64_t p = rr * 4 + ((lane >> 1) & 3u);
        const uint32_t st = uint32_t(reinterpret_cast<uintptr_t>(base)) + uint32_t(p) * stride;
        const uint32_t t = (kFrame - len - ((DIAG & 64) ? kFrame - len : epi.lead(p, st, len, kFrame))) >> 4;
        const uint32_t tmax = (kFrame - len) >> 4;  // wave-uniform
        for (uint32_t s2 = 0; s2 < tmax; ++s2) {
            const uint32_t y = stag_apply3<0>(lds, K.kB, K.sel, acc);  // x^-128
            acc = s2 < t ? y : acc;
        }
        acc ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(acc), 0xB1, 0xF, 0xF, false));  // lane ^ 1
        // the advance T past the last row, deferred from the rounds (it commutes with
        // every x^-k above): once per packet instead of four times per lane per round
        if (!(DIAG & 1)) acc = stag_apply3<0>(lds, K.kA, K.sel, acc);
        const bool on = h == 0 && (lane >> 3) < k && rr < rounds && p < n;
        if constexpr (kDump) {
            if (hold) {  // the buffer sits in the transposition slots of waves 8..15
                if (dgroups == 0) dfirst = rfirst;
                // flush dgroups, row lane >> 3, packet (lane >> 1) & 3: segment 8 dgroups + row
                if (h == 0)
                    *(__attribute__((address_space(3))) uint32_t *)(rbuf + (dgroups * 8u + (lane >> 3)) * 16u +
                                                                     ((lane >> 1) & 3u) * 4u) = acc ^ epi.cinit;
                if (++dgroups == kHoldG) dump();
            } else if (!(DIAG & 16)) {
                epi.put(p, acc, on, pre);
            }
        } else if (!(DIAG & 16)) {
            epi.put(p, acc, on, pre);
        }
        if constexpr (BEpi::kFixup) nfix += uint32_t(__popcll(__ballot(epi.listed(on, pre))));
        if (more) epi.pre(group_packet(next_g0), pre);
        k = 0;
    };

    auto crc_round = [&](uint64_t rr, const Round &R) {
        if constexpr (BEpi::kCopy) {
            const auto crs = epi.round_rsrc(rr * 4);
            const bool qlive = rr * 4 + q < n;
#pragma unroll
            for (int i = 0; i < ROWS; ++i) {
                const int32_t rel = int32_t(uint32_t(i) * 256u + j * 16u) - int32_t(R.lead);
                const bool in = (i == 0 || i == ROWS - 1) ? (rel >= 0 && rel < int32_t(len)) : true;
                epi.copy(crs, q, rel, in && qlive, R.w[i], i == 0);
            }
        }
        uint32_t b0 = R.w[0].x, b1 = R.w[0].y, b2 = R.w[0].z, b3 = R.w[0].w;  // B ^ w of the current row
#pragma unroll
        for (int i = 1; i < ROWS; ++i) {
            const u32x4 w = R.w[i];
            if (DIAG & 1) {
                b0 = (b0 ^ w.x) + (b0 >> 3);
                b1 = (b1 ^ w.y) + (b1 >> 3);
                b2 = (b2 ^ w.z) + (b2 >> 3);
                b3 = (b3 ^ w.w) + (b3 >> 3);
                continue;
            }
            b0 = stag_apply3x<0>(lds, K.kA, K.sel, b0, w.x);
            b1 = stag_apply3x<0>(lds, K.kA, K.sel, b1, w.y);
            b2 = stag_apply3x<0>(lds, K.kA, K.sel, b2, w.z);
            b3 = stag_apply3x<0>(lds, K.kA, K.sel, b3, w.w);
        }
        // braid b = 4j + k holds R_0(frame_b) * x^(32 b) / T (the last row's advance T is
        // applied at the flush): fold with x^-32 (Horner in-lane)
        uint32_t v;
        if (DIAG & 2) {
            v = xor3(b0, b1, b2) ^ b3;
        } else {
            v = stag_apply3x<128>(lds, K.kA, K.sel, b3, b2);
            v = stag_apply3x<128>(lds, K.kA, K.sel, v, b1);
            v = stag_apply3x<128>(lds, K.kA, K.sel, v, b0);
        }
        if (k == 0) rfirst = rr;
        *(__attribute__((address_space(3))) uint32_t *)(xs + k * 256u + lane * 4u) = v;
        if (++k == kGroup) flush(rr + rstep, true);
    };

    uint64_t r = uint64_t(blockIdx.x) * nwave + wave;
    // the first loads are issued before the LDS table fill so the fill overlaps them
    Round A, B;
    // braid tables, x^-32 (region A); x^-128, x^-1024 (region B): their loads go out
    // first, the first round's data loads overlap the LDS writes
    const StagSet sets[4] = {{gtab + OFF_BRAID, 0u},
                             {gtab + OFF_INV + 0 * 1024, 128u},
                             {gtab + OFF_INV + 2 * 1024, 65536u},
                             {gtab + OFF_INV + 5 * 1024, 65536u + 128u}};
    constexpr int kT = BEpi::kThreads;  // the launcher's workgroup size
    StagFill<4, kT> fill;
    const bool batched = blockDim.x == kT;  // other sizes: tools/kbench.hip A/B builds
#ifndef WTP_BR_PROLOGUE_DIAG  // probe builds only: 1 = no table loads, 2 = no table fill at all
#define WTP_BR_PROLOGUE_DIAG 0
#endif
    if (batched && WTP_BR_PROLOGUE_DIAG == 0) fill.load(sets);
    if constexpr (WTP_BR_PROLOGUE_DIAG == 1)
        for (int kk = 0; kk < fill.PER; ++kk) fill.v[kk] = threadIdx.x + kk;
    epi.pre(group_packet(r), pre);
    load_round(r, A);
    PC_PROBE(1, __builtin_amdgcn_s_memrealtime());
    if (WTP_BR_PROLOGUE_DIAG == 2) {
    } else if (batched) {
        fill.store(lds, sets);
    } else {
        for (int q2 = 0; q2 < 4; ++q2) fill_stag(lds, sets[q2].off >> 16, (sets[q2].off >> 7) & 1u, sets[q2].g);
    }
    PC_PROBE(2, __builtin_amdgcn_s_memrealtime());
    __syncthreads();
    PC_PROBE(3, __builtin_amdgcn_s_memrealtime());

    // 2-way unrolled: one round in flight while the previous one is hashed, no register
    // copies between the two sets.  (A variant keeping two rounds in flight, with the
    // per-wave invariants hoisted and 8 rounds unrolled, was 0.7-1.3% slower under
    // sustained load, interleaved A/B; it was 7% faster on 64K-packet batches.)
    // rotating s_setprio per round, offset by the wave's age rank (as in k_pieces): at 8
    // waves per CU +0.9% sustained (kbench x4, profiles/r01i/kbench_512_prio.log; it lost
    // 1% at 16 waves).  DIAG bit2 turns it off for ablations.
    uint32_t prio_round = wave >> 2;
    if constexpr (BEpi::kDepth == 3) {
        // three register sets, two rounds in flight while one is hashed (the fused
        // builder: only 2 waves per CU, so each wave keeps more bytes in flight)
        Round C;
        load_round(r + rstep, B);
        while (r < rounds) {
            if (!(DIAG & 4)) rotate_prio(++prio_round);
            load_round(r + 2 * rstep, C);
            crc_round(r, A);
            r += rstep;
            if (r >= rounds) break;
            load_round(r + 2 * rstep, A);
            crc_round(r, B);
            r += rstep;
            if (r >= rounds) break;
            load_round(r + 2 * rstep, B);
            crc_round(r, C);
            r += rstep;
        }
    } else {
        while (r < rounds) {
            if (!(DIAG & 4)) rotate_prio(++prio_round);
            load_round(r + rstep, B);
            crc_round(r, A);
            if (WTP_PROBE && prio_round == (wave >> 2) + 1) PC_PROBE(4, __builtin_amdgcn_s_memrealtime());
            r += rstep;
            if (r >= rounds) break;
            load_round(r + rstep, A);
            crc_round(r, B);
            r += rstep;
        }
    }
    if (k) flush(0, false);
    if constexpr (kDump) {
        if (dgroups) dump();
    }
    PC_PROBE(5, __builtin_amdgcn_s_memrealtime());
    if constexpr (BEpi::kFixup) verify_fixup(lds, epi, gtab, nfix, rstep, wave, lane);
}

// ------------------------------------------------------------------------------------
// 2. pieces kernel (general shapes)
// ------------------------------------------------------------------------------------
// Epilogues store through buffer resources: lanes without a result use an out-of-range
// offset, so the store is one unconditional instruction (no exec branch, so the
// compiler's vmcnt accounting keeps the round's prefetches in flight).  n < 2^29 (the
// host splits larger batches).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t nbytes);
// Raw metadata words of one packet as loaded by a provider (see the providers below).
struct MetaRaw {
    uint64_t a;
    uint32_t b, c, d;
};
// One sub-launch of a packed batch >= 2 GiB (launch_packed_ranges): packets [begin, end)
// of the caller's arrays, read through a < 2 GiB view that starts `rebase` bytes into the
// 16-B aligned buffer.  Written on the device by k_cut_ranges.  `bad` holds two flags:
// kCutBad, set by k_cut_ranges (an offset past the buffer; fixed before any piece
// sub-launch starts, so every wave of a sub-launch reads the same value), and kRunBad, set
// by the piece kernel when a packet lies outside the view (the offsets were not packed).
// Either one makes the gated k_stream launch recompute the whole batch.
constexpr uint32_t kRunBad = 1u, kCutBad = 2u;
struct RangeDesc {
    uint64_t begin, end, rebase;
    uint32_t nbytes, bad;
};
static_assert(sizeof(RangeDesc) == 32, "RangeDesc");
// providers whose packet range and view are bound on the device (bind(), at kernel entry)
template <class P>
constexpr bool kDevRange = requires { requires P::kDevRange; };  // declared and true
struct CrcEpi {
    static constexpr const char *kName = "CrcEpi";  // wtp_last_kernel()
    uint32_t *out;
    uint32_t n;
    __device__ __forceinline__ void rebase(uint64_t first, uint32_t cnt) {  // a device-bound sub-range
        out += first;
        n = cnt;
    }
    __device__ __forceinline__ void put(uint64_t p, uint32_t crc, bool, uint32_t, bool on) const {
        __builtin_amdgcn_raw_buffer_store_b32(crc, make_rsrc(out, 4 * n), on ? int(4 * p) : int(0x80000000u), 0, 0);
    }
};
// Receiver.cpp:203-206: (int)ntohl(hdr.checksum) == (int)crc32(payload).  aux carries the
// header checksum (host order) from the provider.
struct VerifyEpi {
    static constexpr const char *kName = "VerifyEpi";
    uint8_t *ok;
    uint32_t *crc;  // may be null
    uint32_t n;
    __device__ __forceinline__ void put(uint64_t p, uint32_t c, bool valid, uint32_t want, bool on) const {
        const bool good = valid && want == c;
        __builtin_amdgcn_raw_buffer_store_b8(uint8_t(good ? 1 : 0), make_rsrc(ok, n), on ? int(p) : int(0x80000000u),
                                             0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(valid ? c : 0u, make_rsrc(crc, crc ? 4 * n : 0u),
                                              on ? int(4 * p) : int(0x80000000u), 0, 0);
    }
};

// Buffer resource over [base, base + nbytes) (nbytes rounded up to 16 by the host, so
// every 16-B block that holds a valid byte is in range); out-of-range loads return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)nbytes, 0x00020000);
}
__device__ __forceinline__ u32x4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

// LDS of k_pieces: region 0 holds two staggered table sets (set 0 = slice-by-4, set 1 =
// the x^(8*64) scan operator), then the scan operators x^(8*64*d), d = 2..32, as plain
// 4 KiB tables, the 65-word head-init table, and one staging slot per wave.  A slot
// holds a span of 16-B chunks with 16 B of padding after every 256 B (chunk c at
// 16*(c + c/16)): the windows of consecutive pieces are 64 B apart, and the padding
// spreads their 16-B reads over all bank groups instead of four.
#ifndef WTP_PC_THREADS
#define WTP_PC_THREADS 1024
#endif
constexpr uint32_t kPcThreads = WTP_PC_THREADS, kPcLogT = __builtin_ctz(kPcThreads), kPcWaves = kPcThreads / 64;
constexpr uint32_t kPcWords = uint32_t(kPieceS) / 4;                // window words per lane
constexpr uint32_t kPcNOps = kPieceS == 64 ? 5 : 6;                  // plain scan operators in LDS
constexpr uint32_t kPcOps = 65536;
constexpr uint32_t kPcHinit = kPcOps + kPcNOps * kOpBytes;
// WTP_PC_SPLIT (A/B knob, off): each lane's 64-B window as two interleaved chains (even /
// odd words) over word tables that advance 8 bytes (region 0, set 0 = S8 instead of S4),
// the odd chain's last word through a nibble-table S4 operator (512 B): 8 dependent LDS
// round trips per round instead of 16, for +13 VALU and +4 lookups per lane.  Bit-exact
// (342 GPU tests), but C5 got ~2% slower (46.0 -> 46.9, 45.7 -> 46.6 us, both library
// orders, profiles/r06e): the loop is bound by VALU issue, not by its LDS chain latency.
#ifndef WTP_PC_SPLIT
#define WTP_PC_SPLIT 0
#endif
constexpr uint32_t kPcNib4 = (kPcHinit + 4 * kHinitWords + 15) & ~15u;
constexpr uint32_t kPcStage = WTP_PC_SPLIT ? kPcNib4 + 512 : kPcHinit + 4 * kHinitWords;
constexpr uint32_t kPcChunks = 4 * uint32_t(kPieceS) + 16;  // span chunks a slot holds: 64 pieces + gaps + head slack
constexpr uint32_t kPcSlot = 16 * (kPcChunks + kPcChunks / 16 + 1);  // windows read one chunk past
constexpr uint32_t kPcSpanRegs = (kPcChunks + 63) / 64;     // lane-contiguous 16-B loads per span
constexpr uint32_t kPcFlags = kPcStage + kPcWaves * kPcSlot;  // 64 B per wave: packet-start flags
constexpr uint32_t kPcBal = kPcFlags + kPcWaves * 64;         // wave split: 16 piece sums, 17 u64 starts
constexpr uint32_t kPcSpre = kPcBal + 64 + 17 * 8;       // 17 u32: pieces before each wave's range
// 16 u32: pieces each wave has left, by SIMD (read as one 16-B vector per SIMD, so the
// base is 16-B aligned: pieces_loop takes the LDS base as a pointer, the compiler assumes
// natural alignment, and a misaligned ds_read_b128 here cost C5 3.3 us per launch)
constexpr uint32_t kPcRem = (kPcSpre + 17 * 4 + 15) & ~15u;
constexpr uint32_t kPcLdsWords = (kPcRem + 64) / 4;      // 161,904 B
static_assert(kPcRem % 16 == 0 && kPcStage % 16 == 0 && kPcSlot % 16 == 0 && kPcOps % 16 == 0, "LDS vector alignment");
static_assert(16 * (kPcChunks + kPcChunks / 16 + 1) <= kPcSlot, "staging slot");
static_assert(kPcLdsWords * 4 <= 163840, "LDS");
static_assert(!WTP_PC_SPLIT || kPieceS == 64, "split chains: 64-B pieces");

__device__ __forceinline__ uint32_t stage_addr(uint32_t chunk) { return 16u * (chunk + (chunk >> 4)); }

// Inclusive prefix sum over the wave with DPP (no LDS round trips): Hillis-Steele within
// each 16-lane row (row_shr 1, 2, 4, 8), then row_bcast:15 / row_bcast:31 carry the row
// totals into the rows above.
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v) {
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xF, 0xF, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xF, 0xF, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xF, 0xF, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xF, 0xF, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xA, 0xF, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xC, 0xF, false));
    return v;
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    return uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v))))) |
           (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v >> 32))))) << 32);
}

// Pieces of a packet of payload length len as the main loop counts them (an empty or
// over-long packet is one).  Providers with variable lengths expose load_len(p) (the one
// metadata word the length comes from) and len_of(word).
__device__ __forceinline__ uint32_t pieces_of_len(uint32_t len) {
    return (len == 0 || len > kMaxVarLen) ? 1u : (len + kPieceS - 1) / kPieceS;
}
template <class Prov>
__device__ __forceinline__ uint32_t piece_count(const Prov &prov, uint64_t p) {
    return pieces_of_len(prov.len_of(prov.load_len(p)));
}

// Wave ranges of a workgroup's packets [g0, g1) with equal piece counts (rounds), not
// equal packet counts: with Zipf lengths, equal counts left the busiest wave 1.43x the
// mean number of rounds (C5, s = 1.1) and the launch waited for it.  Each thread owns a
// contiguous sub-range; load() issues the length loads of its first kReg packets (they
// fly while the LDS tables fill), finish() sums their pieces, a block scan places the sub-ranges,
// and the thread whose sub-range holds wave w's target (total * w / waves) walks it, from
// registers, to the first packet at or past the target.  Every thread of the block must
// call finish() (two barriers).  k_pieces runs 1024-thread blocks: the divisions by the
// thread and wave counts are shifts (64-bit divisions by a runtime value cost ~100 VALU
// each, and the target loop had 15 of them).
#ifndef WTP_PC_LEN128
#define WTP_PC_LEN128 1  // wave split: length words by two 16-B loads (0: eight dword loads)
#endif
#ifndef WTP_PC_LAG
#define WTP_PC_LAG 1  // k_pieces: wave priority by work left (0: rotate by round and age)
#endif
static_assert(kPcThreads >= 128 && kPcThreads <= 1024 && (kPcThreads & (kPcThreads - 1)) == 0, "k_pieces block");
// Pieces of packets [p, min(p + 16, b)) from four 16-B length loads issued together (4-B
// aligned offsets; words at or past g1 read 0 and are not counted).  Packets are taken
// while the running count is below `want` (~0u: all; the boundary walk passes the pieces
// left to its target), and *taken (if given) receives how many were.
template <class Prov>
__device__ __forceinline__ uint32_t chunk_pieces(const Prov &prov, uint64_t g1, uint64_t p, uint64_t b, uint32_t want,
                                                 uint32_t *taken) {
    const __amdgpu_buffer_rsrc_t lr = make_rsrc(prov.len_array(), uint32_t(4 * g1));
    u32x4 q[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) q[j] = buf_ld16(lr, uint32_t(4 * (p + 4 * j)));
    const uint32_t w[16] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w,
                            q[2].x, q[2].y, q[2].z, q[2].w, q[3].x, q[3].y, q[3].z, q[3].w};
    uint32_t sum = 0, n = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        const bool step = p + i < b && sum < want;
        sum += step ? pieces_of_len(prov.len_of(w[i])) : 0u;
        n += step ? 1u : 0u;
    }
    if (taken) *taken = n;
    return sum;
}
struct WaveSplit {
    static constexpr uint32_t kReg = 8, kThreads = kPcThreads, kWaves = kThreads / 64;
    uint32_t raw[kReg];  // length words of the first kReg packets of the sub-range
    uint64_t a, b;
    template <class Prov>
    __device__ __forceinline__ void load(const Prov &prov, uint64_t g0, uint64_t g1) {
        const uint64_t R = g1 - g0;
        a = g0 + ((R * threadIdx.x) >> kPcLogT);
        b = g0 + ((R * (threadIdx.x + 1)) >> kPcLogT);
#if WTP_PC_LEN128
        // the sub-range's first 8 length words as two 16-B buffer loads (4-B aligned is
        // enough; words at or past g1 read 0 and are never used): a quarter of the vector
        // memory instructions of 8 dword loads, in the prologue where they queue behind
        // the table loads
        static_assert(kReg == 8, "two 16-B loads");
        const __amdgpu_buffer_rsrc_t lr = make_rsrc(prov.len_array(), uint32_t(4 * g1));
        const u32x4 l0 = buf_ld16(lr, uint32_t(4 * a)), l1 = buf_ld16(lr, uint32_t(4 * a + 16));
        raw[0] = l0.x; raw[1] = l0.y; raw[2] = l0.z; raw[3] = l0.w;
        raw[4] = l1.x; raw[5] = l1.y; raw[6] = l1.z; raw[7] = l1.w;
#else
#pragma unroll
        for (uint32_t j = 0; j < kReg; ++j) raw[j] = prov.load_len(a + j < b ? a + j : g0);  // g0 < g1: valid
#endif
    }
    template <class Prov>
    __device__ __forceinline__ void finish(const Prov &prov, uint64_t g0, uint64_t g1, char *lds, uint32_t wave,
                                           uint32_t lane, uint64_t &lo, uint64_t &hi, uint32_t &wpieces) {
        constexpr uint32_t nw = kWaves;
        const uint64_t m = b - a;
        uint32_t k[kReg], sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < kReg; ++j) {
            k[j] = j < m ? pieces_of_len(prov.len_of(raw[j])) : 0u;
            sum += k[j];
        }
        // > kReg packets per thread (launches of more than 2 M packets): the rest in chunks
        // of 16 length words, four 16-B loads in flight per chunk.  (A dword loop waited on
        // each load: at 15 M packets per launch, ~50 serial loads here and up to ~57 in the
        // boundary walk below cost ~0.1 ms per launch.)  Counts only balance the waves: the
        // ranges stay a partition of [g0, g1) whatever they hold.
        for (uint64_t p = a + kReg; p < b; p += 16) sum += chunk_pieces(prov, g1, p, b, ~0u, nullptr);
        const uint32_t incl = wave_incl_add(sum);
        uint32_t *const wsum = reinterpret_cast<uint32_t *>(lds + kPcBal);
        uint64_t *const starts = reinterpret_cast<uint64_t *>(lds + kPcBal + 64);
        uint32_t *const spre = reinterpret_cast<uint32_t *>(lds + kPcSpre);
        if (lane == 63u) wsum[wave] = incl;
        if (threadIdx.x == 0) {
            starts[0] = g0;
            starts[nw] = g1;
            spre[0] = 0;
        }
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (uint32_t w = 0; w < nw; ++w) {
            const uint32_t v = wsum[w];
            before += w < wave ? v : 0u;
            total += v;
        }
        const uint32_t excl = before + incl - sum;
        for (uint32_t w = 1; w < nw; ++w) {
            const uint32_t target = uint32_t((uint64_t(total) * w) >> (kPcLogT - 6));
            if (target >= excl && target - excl < sum) {
                uint32_t pre = excl;
                uint64_t p = a;
#pragma unroll
                for (uint32_t j = 0; j < kReg; ++j) {
                    const bool step = j < m && pre < target;
                    pre += step ? k[j] : 0u;
                    p += step ? 1u : 0u;
                }
                while (p < b && pre < target) {
                    uint32_t taken = 0;
                    pre += chunk_pieces(prov, g1, p, b, target - pre, &taken);
                    p += taken;
                }
                starts[w] = p;
                spre[w] = pre;
            }
        }
        if (threadIdx.x == 0) spre[nw] = total;
        __syncthreads();
        // Every starts[w] was written above: pieces_of_len() >= 1, so total >= g1 - g0 > 0
        // and each target < total lies in exactly one thread's [excl, excl + sum).  The
        // clamp keeps a wave inside [g0, g1] even if that invariant were ever broken: a
        // round-3 development build counted 0 pieces for small packets, so an all-small
        // workgroup wrote no starts[1..15] and its waves ran over the previous kernel's
        // stale LDS indices (hipErrorIllegalAddress).
        const uint64_t s0 = uniform64(starts[wave]), s1 = uniform64(starts[wave + 1]);
        lo = s0 < g0 ? g0 : (s0 > g1 ? g1 : s0);
        hi = s1 < lo ? lo : (s1 > g1 ? g1 : s1);
        wpieces = uint32_t(__builtin_amdgcn_readfirstlane(int(spre[wave + 1] - spre[wave])));
    }
};

// Lane-contiguous load of kPcChunks 16-B chunks starting at view offset b16 (16-aligned,
// may be negative near the buffer start): 4 full wave instructions + 16 lanes of a
// fifth.  Offsets outside the buffer read 0 without touching memory.
__device__ __forceinline__ void load_span(__amdgpu_buffer_rsrc_t rs, int32_t b16, uint32_t lane,
                                          u32x4 (&x)[kPcSpanRegs]) {
#pragma unroll
    for (uint32_t i = 0; i < kPcSpanRegs; ++i) {
        const uint32_t c = 64u * i + lane;
        x[i] = buf_ld16(rs, c < kPcChunks ? uint32_t(b16) + 16u * c : 0x80000000u);
    }
}

// Span staging by LDS-DMA (WTP_PC_DMA=1): the same slot image as load_span + the
// ds_write_b128 staging below, written by `buffer_load_dwordx4 ... lds` straight from
// memory.  An LDS-DMA instruction writes 64 consecutive 16-B positions (wave-uniform base
// in M0 + 16 * lane), so the per-256-B padding is made on the SOURCE side: position q of
// the slot holds chunk q - q/17 (the inverse of stage_addr; every 17th position is padding
// and receives a duplicate chunk that no window reads).  Positions 0..kPcSlotPos-1: four
// full instructions and 34 lanes of a fifth.  Issued as inline asm, so the compiler keeps
// no count of them: the loop waits for them itself (vmcnt(0) before the slot is read) and
// lets the window reads finish (lgkmcnt(0)) before the next span may overwrite the slot.
#ifndef WTP_PC_DMA
#define WTP_PC_DMA 1  // 0: register staging (load_span + ds_write_b128), the round-3 form (A/B builds)
#endif
constexpr uint32_t kPcSlotPos = kPcSlot / 16;                 // 290 positions of 16 B
constexpr uint32_t kPcDmaRegs = (kPcSlotPos + 63) / 64;       // 5 instructions
static_assert(kPcSlotPos - 64 * (kPcDmaRegs - 1) <= 64, "slot positions");
struct SpanDma {
    uint32_t coff[kPcDmaRegs];  // per lane: 16 * (source chunk of slot position 64 i + lane)
    uint32_t slot;              // LDS byte address of the wave's slot (wave-uniform)
    __device__ __forceinline__ SpanDma(uint32_t slot_addr, uint32_t lane) : slot(slot_addr) {
#pragma unroll
        for (uint32_t i = 0; i < kPcDmaRegs; ++i) {
            const uint32_t q = 64u * i + lane;
            coff[i] = 16u * (q - q / 17u);
        }
    }
    // the span of 16-B chunks from view offset b16 (16-aligned, may be "negative" or past
    // the view: those offsets read 0 without touching memory) into the slot
    __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, int32_t b16, uint32_t lane) const {
        // lgkmcnt(0) first: this wave's window reads of the slot have returned
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (uint32_t i = 0; i < kPcDmaRegs; ++i) {
            const uint32_t voff = uint32_t(b16) + coff[i];
            const uint32_t m0v = slot + 1024u * i;
            uint32_t keep;
            if (i + 1 < kPcDmaRegs || lane < kPcSlotPos - 64u * (kPcDmaRegs - 1))
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                             "s_mov_b32 m0, %0"
                             : "=&s"(keep)
                             : "v"(voff), "s"(rs), "s"(m0v)
                             : "memory");
        }
    }
    // The same, leaving out the chunks that start at or past view byte `lim` (their lanes
    // get an out-of-range offset: no request).  The tail clamp (WTP_PC_TAILCLAMP) below.
    __device__ __forceinline__ void issue_below(__amdgpu_buffer_rsrc_t rs, int32_t b16, uint32_t lane, int32_t lim) const {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (uint32_t i = 0; i < kPcDmaRegs; ++i) {
            const int32_t c0 = b16 + int32_t(coff[i]);
            const uint32_t voff = c0 < lim ? uint32_t(c0) : 0x80000000u;
            const uint32_t m0v = slot + 1024u * i;
            uint32_t keep;
            if (i + 1 < kPcDmaRegs || lane < kPcSlotPos - 64u * (kPcDmaRegs - 1))
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                             "s_mov_b32 m0, %0"
                             : "=&s"(keep)
                             : "v"(voff), "s"(rs), "s"(m0v)
                             : "memory");
        }
    }
    __device__ __forceinline__ static void wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
};

// Maximum over the wave (unsigned; 0 is neutral), by the same DPP steps as wave_incl_add
// (a __shfl_xor ladder here changed how the compiler lowered the loop's other
// shuffles and cost C5 ~2 us per launch).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    auto mx = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
    v = mx(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xF, 0xF, false)));
    v = mx(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xF, 0xF, false)));
    v = mx(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xF, 0xF, false)));
    v = mx(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xF, 0xF, false)));
    v = mx(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xA, 0xF, false)));
    v = mx(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xC, 0xF, false)));
    return uint32_t(__builtin_amdgcn_readlane(int(v), 63));
}

// Tail clamp of the span prefetch: a wave's last rounds used to prefetch a full 4352-B
// span past the end of its last packet, i.e. into the first bytes of the next wave's
// range, which that wave had read ~40 us earlier (its first round), so they came from
// memory twice: ~3.4 KB per wave boundary, 14.1 MB of C5's 26 MB excess read
// (tools/c5_span_model.py, profiles/r05).  When the round's view holds every packet the
// wave has left, the prefetch stops at the end of the last of them.
#ifndef WTP_PC_TAILCLAMP
#define WTP_PC_TAILCLAMP 0  // measured and not shipped: -12.1 MB of reads, +1.5 us
#endif

// The wave's packets form one stream of 64-B pieces (each packet cut into pieces counted
// back from its end, the head piece possibly shorter).  A round takes the next pieces,
// one per lane, up to 64 and up to the first piece whose window falls outside the span
// one LDS slot holds (kPcChunks chunks from the round's first window): packed and
// strided batches always fill all 64 lanes, scattered offsets make shorter rounds.  A
// packet may straddle rounds: its CRC register after its last piece in round r seeds the
// chain of its next piece in round r+1.  Per round a wave
//   1. scans the piece counts of the next 64 packets (metadata prefetched during the
//      previous round) and assigns lane -> (packet, piece);
//   2. stages the span into its LDS slot: it was loaded during the previous round (it
//      starts at most 64 B before that round's last window ends: speculative, exact for
//      packed and strided batches); a miss loads it now.  The span goes from memory
//      straight into the slot by LDS-DMA (SpanDma, 5 instructions of 1 KiB; round 3
//      loaded it into 20 VGPRs and stored it with 5 ds_write_b128: C5 47.9 -> 46.1 us);
//   3. reads each lane's 64-B window from the slot and issues the next round's metadata
//      and span loads;
//   4. runs the slice-by-4 chain over the window (bytes before the packet masked to
//      zero; the head piece adds shift(~0, head length), the CRC's initial value), then a
//      segmented scan with x^(8*64*d) combines each packet's pieces and the lane holding
//      a packet's last piece emits crc = W ^ ~0.
// Loads and stores are branch-free (out-of-range buffer offsets for idle lanes), so the
// prefetches stay in flight across the round.
// Metadata of packets q0 .. q0+63 for one round: lane i loads packet q0 + i (clamped to
// hi - 1: branch-free).  The caller of pieces_loop issues the first round's (raw) before
// its last prologue waits, so that latency overlaps them.
template <class Prov>
__device__ __forceinline__ void pieces_meta(const Prov &prov, uint64_t q0, uint64_t hi, uint32_t lane, MetaRaw &raw,
                                            __amdgpu_buffer_rsrc_t rs) {
    if constexpr (Prov::kGroupLoad) {
        prov.load_group(q0, lane, raw);  // buffer loads: lanes past the arrays read 0
    } else {
        const uint64_t pi = q0 + lane;
        prov.load(pi < hi ? pi : hi - 1, raw, rs);
    }
}

// The piece-stream main loop: packets [lo, hi) of the provider (wpieces = their piece
// total, for the work-left priority of variable-length providers), tables already in LDS
// (PcTables), raw = the first round's metadata (pieces_meta(lo)).  Used by k_pieces and
// by the braided verify's fix-up phase.
template <class Prov, class Epi>
__device__ __forceinline__ void pieces_loop(char *lds, __amdgpu_buffer_rsrc_t rs, const Prov &prov, const Epi &epi,
                                            uint64_t lo, uint64_t hi, uint32_t wpieces, uint32_t *status,
                                            uint32_t wave, uint32_t lane, MetaRaw raw) {
    const StagKeys K(lane);
    lchar *const slot = (lchar *)lds + kPcStage + wave * kPcSlot;
    constexpr int32_t kSpanBytes = int32_t(16 * kPcChunks);
    constexpr int32_t kNoSpan = 0x7FFFF000;  // out of range: loads return 0, no traffic

    auto meta = [&](uint64_t q0) { pieces_meta(prov, q0, hi, lane, raw, rs); };
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the loop entry then matches its back edge

    PC_PROBE(3, __builtin_amdgcn_s_memrealtime());
    uint32_t skip = 0, carry = 0;  // pieces of packet p0 done in earlier rounds, their register
    int32_t spec = kNoSpan;        // view offset of the prefetched span
#if WTP_PC_DMA
    const SpanDma dma(__builtin_amdgcn_readfirstlane(uint32_t(uintptr_t(slot))), lane);
#else
    u32x4 x[kPcSpanRegs];
#endif
    uint32_t nrounds = 0, done = 0;
    hi = uniform64(hi);  // wave-uniform in SGPRs: the round's packet arithmetic stays scalar
    for (uint64_t p0 = uniform64(lo); p0 < hi;) {
        uint64_t off;
        uint32_t len, aux = 0, oslot = 0;
        bool valid;
        prov.decode(raw, off, len, valid, aux, oslot);
        const uint32_t inview = hi - p0 > 64u ? 64u : uint32_t(hi - p0);  // wave-uniform (SALU)
        const bool have = lane < inview;
        if constexpr (kDevRange<Prov>) {
            if (have && !valid) prov.flag_outside();  // not packed: the gated k_stream redoes the batch
        }
        if (have && len > kMaxVarLen) {
            atomicOr(status, 1u);
            len = 0;
            valid = false;
        }
        const uint32_t k = have ? (len == 0 ? 1u : (len + kPieceS - 1) / kPieceS) : 64u;
        const uint32_t kr = k - (lane == 0 ? skip : 0u);  // pieces still to do
        const uint32_t incl = wave_incl_add(kr);
        const uint32_t excl = incl - kr;
        const uint32_t navail = __popcll(__ballot(have));  // packets of the wave left in view
        const uint32_t covered = uint32_t(__builtin_amdgcn_readlane(int(incl), int(navail - 1)));  // pieces in view

        // --- lane -> (packet, piece): flag the first lane of every packet in LDS, then
        // pk = (# flagged lanes <= this lane) - 1 from a ballot ----------------------------
        lu8 *const flags = (lu8 *)lds + kPcFlags + wave * 64u;
        flags[lane] = 0;
        if (have && excl < 64u) flags[excl] = 1;
        __builtin_amdgcn_wave_barrier();
        const bool start = flags[lane] != 0;
        __builtin_amdgcn_wave_barrier();
        const uint64_t starts = __ballot(start);
        uint32_t pk = __builtin_amdgcn_mbcnt_hi(uint32_t(starts >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(starts), 0u)) +
                      (start ? 1u : 0u) - 1u;
        const bool mapped = lane < covered;
        pk = mapped ? pk : 0;
        const uint32_t pex = __shfl(excl, pk);
        const uint32_t pkk = __shfl(k, pk);
        const uint32_t plen = __shfl(len, pk);
        const uint32_t poff = __shfl(uint32_t(off), pk);  // < 2^31: the view is < 2 GiB
        const bool pvalid = __shfl(valid ? 1u : 0u, pk) != 0;
        const uint32_t paux = __shfl(aux, pk);
        const uint64_t pout = Prov::kIndexed ? uint64_t(uint32_t(__shfl(oslot, pk))) : p0 + pk;  // output index
        const uint32_t lp = lane - pex;                  // piece index within this round
        const uint32_t gp = lp + (pk == 0 ? skip : 0u);  // piece index within the packet

        // --- piece window: the 64 bytes ending at this piece's end ----------------------
        const int32_t we = int32_t(poff + plen) - int32_t(pkk - 1 - gp) * kPieceS;
        const int32_t ws = we - kPieceS;
        // the round: lanes up to the first one whose window leaves [lo16, lo16 + span)
        const int32_t lo16 = __builtin_amdgcn_readlane(ws, 0) & ~15;
        const bool out = !mapped || ws < lo16 || we - lo16 > kSpanBytes;
        const uint64_t outm = __ballot(out);
        const uint32_t total = outm ? uint32_t(__builtin_ctzll(outm)) : 64u;  // >= 1: lane 0 fits
        const bool active = lane < total;
        const int32_t vf0 = int32_t(poff) - ws;  // bytes of the window before the packet
        const int32_t vf = active ? (vf0 > kPieceS ? kPieceS : vf0) : kPieceS;

        // --- stage the span ---------------------------------------------------------------
        const bool hit = __ballot(active && (ws < spec || we - spec > kSpanBytes)) == 0;
        int32_t sbase = spec;
#if WTP_PC_DMA
        if (!hit) {
            dma.issue(rs, lo16, lane);  // the miss pays its latency here
            sbase = lo16;
        }
        SpanDma::wait();  // the slot holds the span (prefetched, or just loaded)
#else
        if (!hit) {
            load_span(rs, lo16, lane, x);
            sbase = lo16;
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the miss pays its latency here
        }
#pragma unroll
        for (uint32_t i = 0; i + 1 < kPcSpanRegs; ++i) *(lu32x4 *)(slot + stage_addr(64u * i + lane)) = x[i];
        if (lane < kPcChunks - 64u * (kPcSpanRegs - 1)) *(lu32x4 *)(slot + stage_addr(64u * (kPcSpanRegs - 1) + lane)) = x[kPcSpanRegs - 1];
#endif
        __builtin_amdgcn_wave_barrier();
        // the window's five 16-B blocks, aligned (dword-aligned variants without the
        // rotation below were slower on C5: ds_read2_b32 pairs at the 64-B lane stride
        // conflict 4-way, +13%; unaligned ds_read_b128 from inline asm, which gfx950
        // executes correctly, +39%)
        uint32_t d[kPcWords + 4];
        {
            const uint32_t blk = active ? uint32_t(ws - sbase) >> 4 : 0u;
#pragma unroll
            for (uint32_t u = 0; u < kPcWords / 4 + 1; ++u) {
                const u32x4 y = *(const lu32x4 *)(slot + stage_addr(blk + u));
                d[4 * u + 0] = y.x;
                d[4 * u + 1] = y.y;
                d[4 * u + 2] = y.z;
                d[4 * u + 3] = y.w;
            }
        }
        __builtin_amdgcn_wave_barrier();

        // --- round bookkeeping and the next round's prefetch ------------------------------
        const uint32_t tl = total - 1;
        const uint32_t last_pk = __builtin_amdgcn_readlane(pk, tl);
        const uint32_t last_gp = __builtin_amdgcn_readlane(gp, tl);
        const uint32_t last_k = __builtin_amdgcn_readlane(pkk, tl);
        const int32_t last_we = __builtin_amdgcn_readlane(we, tl);
        const bool partial = last_gp + 1 < last_k;
        const uint64_t p0n = p0 + last_pk + (partial ? 0u : 1u);
        meta(p0n);  // first: the next round waits for these, not for the span
        spec = p0n < hi ? ((last_we - kPieceS) & ~15) : kNoSpan;
#if WTP_PC_DMA
        // (not in the verify fix-up's indexed pass: scattered datagrams, and its kernel has
        // no SGPRs to spare for it)
        if (WTP_PC_TAILCLAMP && !Prov::kIndexed && spec != kNoSpan && hi - p0 <= 64u) {  // wave-uniform: the wave's last packets are all in view
            // end of the bytes any packet still to do can need (lanes from the round's last
            // packet on: a superset of p0n .. hi-1)
            const uint32_t pend = have && lane >= last_pk ? uint32_t(off) + len : 0u;
            dma.issue_below(rs, spec, lane, int32_t(wave_max_u32(pend)));
        } else if (spec != kNoSpan) {
            dma.issue(rs, spec, lane);  // wave-uniform branch
        }
#else
        load_span(rs, spec, lane, x);
#endif

        // rotate left by a>>2 dwords with bit-selects (v_bfi_b32), then funnel by a&3
        const uint32_t a = uint32_t(ws) & 15u;
        const uint32_t m2 = 0u - ((a >> 3) & 1u), m1 = 0u - ((a >> 2) & 1u), sb = a & 3u;
        uint32_t e[kPcWords + 2];
#pragma unroll
        for (int i = 0; i < int(kPcWords) + 2; ++i) e[i] = d[i] ^ ((d[i] ^ d[i + 2]) & m2);
#pragma unroll
        for (int i = 0; i < int(kPcWords) + 1; ++i) e[i] = e[i] ^ ((e[i] ^ e[i + 1]) & m1);

        // one chain per 64 B of the window (128-B pieces: two independent chains, joined
        // below by x^(8*64)); WTP_PC_SPLIT: two interleaved chains per 64 B (below)
        uint32_t c;
        if constexpr (!WTP_PC_SPLIT) {
        constexpr int kChains = int(kPcWords) / 16;
        uint32_t cc[kChains];
        cc[0] = (lane == 0u) ? carry : 0u;  // carry is 0 unless packet p0 continues
        if constexpr (kChains == 2) cc[1] = 0u;
        const int32_t vf8 = 8 * vf;
#pragma unroll
        for (int j = 0; j < 16 * kChains; ++j) {
            const int i = (j % kChains) * 16 + j / kChains;  // interleave the chains
            uint32_t &cj = cc[j % kChains];
            const uint32_t wd = __builtin_amdgcn_alignbyte(e[i + 1], e[i], sb);
            // keep the bytes at window offset >= vf: the low s = clamp(8 vf - 32 i, 0, 32)
            // bits of word i go.  One v_med3 + one v_lshlrev_b64 (the shift unit reads 6
            // bits: word 2j takes the low half of 0xFFFFFFFF << s, word 2j+1 the high half
            // of 0xFFFFFFFF << (s + 32), and s = 32 wraps to a zero high half)
            const int32_t t = vf8 < 32 * i ? 32 * i : (vf8 > 32 * i + 32 ? 32 * i + 32 : vf8);
            const uint64_t k64 = uint64_t(0xFFFFFFFFu) << (uint32_t(t) & 63u);
            const uint32_t keep = (i & 1) ? uint32_t(k64 >> 32) : uint32_t(k64);
            cj = stag_apply3<0>(lds, K.kA, K.sel, __builtin_amdgcn_bitop3_b32(cj, wd, keep, 0x78));  // cj ^ (wd & keep)
        }
        c = cc[0];
        if constexpr (kChains == 2) c = stag_apply3x<128>(lds, K.kA, K.sel, cc[0], cc[1]);  // x^(8*64) * c0 ^ c1
        } else {
            // two chains, 8 dependent steps each: even words advance by S8 (a word then 4
            // zero bytes, the odd word's slot) and end aligned with the window's end; odd
            // words 1..13 likewise, and word 15 by a plain S4 step (nibble tables)
            uint32_t ca = (lane == 0u) ? carry : 0u, cb = 0u;
            const int32_t vf8 = 8 * vf;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t wd = __builtin_amdgcn_alignbyte(e[i + 1], e[i], sb);
                const int32_t t = vf8 < 32 * i ? 32 * i : (vf8 > 32 * i + 32 ? 32 * i + 32 : vf8);
                const uint64_t k64 = uint64_t(0xFFFFFFFFu) << (uint32_t(t) & 63u);
                const uint32_t keep = (i & 1) ? uint32_t(k64 >> 32) : uint32_t(k64);
                if ((i & 1) == 0)
                    ca = stag_apply3<0>(lds, K.kA, K.sel, __builtin_amdgcn_bitop3_b32(ca, wd, keep, 0x78));
                else if (i < 15)
                    cb = stag_apply3<0>(lds, K.kA, K.sel, __builtin_amdgcn_bitop3_b32(cb, wd, keep, 0x78));
                else
                    cb = nib_apply(lds, kPcNib4, __builtin_amdgcn_bitop3_b32(cb, wd, keep, 0x78));
            }
            c = ca ^ cb;
        }
        // head piece: R_~0(head) = R_0(0^vf || head) ^ shift(~0, S - vf)
        const uint32_t hw = lds_rd(lds, kPcHinit + 4u * uint32_t(kPieceS - (vf < 0 ? 0 : vf)));
        c ^= gp == 0u ? hw : 0u;

        // --- segmented inclusive scan: W_i <- W_{i-d} * x^(8*64*d) ^ W_i ---------------
        uint32_t W = c;
        {
            const uint32_t u = __shfl_up(W, 1);
            if constexpr (kPieceS == 64) {  // x^(8*64) is the staggered set 1
                if (lp >= 1u && lane >= 1u) W = stag_apply3x<128>(lds, K.kA, K.sel, u, W);
            } else {  // set 1 joins the chains; x^(8*128) is plain operator 0
                if (lp >= 1u && lane >= 1u) W = op_apply_fold(lds, kPcOps, u, W);
            }
        }
        // levels no lane needs (every packet of the round has < dd pieces in it) are
        // skipped with a wave-uniform branch on the ballot (SGPRs): small-packet rounds
        // stop early
#pragma unroll
        for (uint32_t dd = 2, o = 0; dd < 64; dd <<= 1, ++o) {
            const bool need = lp >= dd && lane >= dd;
            if (__builtin_amdgcn_ballot_w64(need) == 0) break;
            const uint32_t u = __shfl_up(W, dd);
            if (need) W = op_apply_fold(lds, kPcOps + (o + kPcNOps - 5) * kOpBytes, u, W);  // exec-masked: idle lanes issue no lookups
        }
        epi.put(pout, W ^ 0xFFFFFFFFu, pvalid, paux, active && gp == pkk - 1);
        carry = partial ? __builtin_amdgcn_readlane(W, tl) : 0u;
        skip = partial ? last_gp + 1 : 0u;
        p0 = uniform64(p0n);  // keeps the loop-carried packet index in SGPRs
        if (WTP_PROBE && nrounds == 0) PC_PROBE(4, __builtin_amdgcn_s_memrealtime());
        ++nrounds;
        if constexpr (Prov::kVarLen && WTP_PC_LAG) {
            // The SIMD arbiter serves the oldest of equal-priority waves first, so with a
            // fixed rotation the youngest waves still ended ~8 us after the oldest
            // (tools/pprobe.py).  Priority = how many of the SIMD's four waves have less
            // work left than this one (stale reads only blur the ranking).
            done += total;
            const uint32_t left = wpieces > done ? wpieces - done : 0u;
            const uint32_t simd = wave & 3u;
            typedef __attribute__((address_space(3))) uint32_t lu32w;
            if (lane == 0) *(lu32w *)((lchar *)lds + kPcRem + 4u * (4u * simd + (wave >> 2))) = left;
            // lanes 0..3 read the SIMD's four entries; the rank is one ballot's popcount
            const uint32_t other = *(const lu32w *)((lchar *)lds + kPcRem + 16u * simd + 4u * (lane & 3u));
            rotate_prio(uint32_t(__popcll(__builtin_amdgcn_ballot_w64(lane < kPcWaves / 4u && other < left))));
        } else {
            rotate_prio(nrounds + (wave >> 2));
        }
    }
    PC_PROBE(5, __builtin_amdgcn_s_memrealtime());
    PC_PROBE(6, nrounds);
    PC_PROBE(7, hi - lo);
}

// LDS tables of the piece loop: the two staggered sets (slice-by-4, x^(8*64)), the plain
// scan operators x^(8*64*d), d = 2..32, and the head-init table.  load() issues every
// global load (ahead of the caller's other prologue loads: vmcnt completes in order),
// store() writes LDS; a barrier must follow before pieces_loop.
template <int THREADS>
struct PcTables {
    static constexpr uint32_t kOpQ = kPcNOps * 256, kOpPer = (kOpQ + THREADS - 1) / THREADS;
    StagFill<2, THREADS> fill;
    u32x4 q[kOpPer];
    uint32_t hv;
    u32x4 n4;
    __device__ __forceinline__ static void sets(const uint32_t *gtab, StagSet (&s)[2]) {
        s[0] = {gtab + (WTP_PC_SPLIT ? OFF_S8 : OFF_S4), 0u};
        s[1] = {gtab + (kPieceS == 64 ? OFF_FWD : OFF_X64), 128u};  // x^(8*64)
    }
    __device__ __forceinline__ void load(const uint32_t *gtab) {
        StagSet ss[2];
        sets(gtab, ss);
        fill.load(ss);
        const u32x4 *src = reinterpret_cast<const u32x4 *>(gtab + OFF_FWD + 1024 * (6 - kPcNOps));
#pragma unroll
        for (uint32_t k = 0; k < kOpPer; ++k) {
            const uint32_t i = threadIdx.x + k * THREADS;
            q[k] = src[i < kOpQ ? i : 0];
        }
        hv = gtab[OFF_HINIT + (threadIdx.x <= kPieceS ? threadIdx.x : 0)];
        if constexpr (WTP_PC_SPLIT)  // nibble-table S4 (shift by 4 bytes): operator 6 + 4 of OFF_NIB
            n4 = reinterpret_cast<const u32x4 *>(gtab + OFF_NIB + 128 * 10)[threadIdx.x & 31u];
    }
    __device__ __forceinline__ void store(char *lds, const uint32_t *gtab) const {
        StagSet ss[2];
        sets(gtab, ss);
        fill.store(lds, ss);
        u32x4 *dst = reinterpret_cast<u32x4 *>(lds + kPcOps);
#pragma unroll
        for (uint32_t k = 0; k < kOpPer; ++k) {
            const uint32_t i = threadIdx.x + k * THREADS;
            if (i < kOpQ) dst[i] = q[k];
        }
        if (threadIdx.x <= kPieceS) reinterpret_cast<uint32_t *>(lds + kPcHinit)[threadIdx.x] = hv;
        if constexpr (WTP_PC_SPLIT)
            if (threadIdx.x < 32u) reinterpret_cast<u32x4 *>(lds + kPcNib4)[threadIdx.x] = n4;
    }
};

template <class Prov, class Epi>
__global__ __launch_bounds__(kPcThreads) void k_pieces(const uint8_t *__restrict__ base_in, uint32_t nbytes_in,
                                                 Prov prov_in, uint64_t n_in, Epi epi_in,
                                                 const uint32_t *__restrict__ gtab, uint32_t *__restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_w[kPcLdsWords];
    char *lds = reinterpret_cast<char *>(lds_w);
    Prov prov = prov_in;
    Epi epi = epi_in;
    const uint8_t *base = base_in;
    uint32_t nbytes = nbytes_in;
    uint64_t n = n_in;
    if constexpr (kDevRange<Prov>) {
        if (!prov.bind(base, nbytes, n, epi)) return;  // this sub-launch's range is empty
    }
    const uint32_t nw = blockDim.x >> 6;
    const uint64_t tw = uint64_t(gridDim.x) * nw, w0 = uint64_t(blockIdx.x) * nw;
    const uint64_t g0 = n * w0 / tw, g1 = n * (w0 + nw) / tw;  // this workgroup's packets
    if (g0 == g1) return;  // no packets for this block
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(base, nbytes);
    PC_PROBE(0, __builtin_amdgcn_s_memrealtime());
    WaveSplit split;
    PcTables<kPcThreads> tb;
    // every table load first (one memory latency, and ahead of the length loads of the
    // wave split, since vmcnt completes in order; see StagFill).  (Lengths first, tables
    // behind them, the first round's metadata issued before the table stores wait:
    // neutral on C5, 53.4 vs 52.9 us back to back, profiles/r03f/abc5.log.)
    tb.load(gtab);
    if constexpr (Prov::kVarLen) split.load(prov, g0, g1);
    PC_PROBE(1, __builtin_amdgcn_s_memrealtime());
    tb.store(lds, gtab);
    uint64_t lo, hi;
    uint32_t wpieces = 0;  // pieces of this wave's range (variable-length providers)
    if constexpr (Prov::kVarLen) {
        split.finish(prov, g0, g1, lds, wave, lane, lo, hi, wpieces);  // two barriers; LDS outside the tables
    } else {
        lo = n * (w0 + wave) / tw;
        hi = n * (w0 + wave + 1) / tw;
    }
    MetaRaw raw{};
    if (lo < hi) pieces_meta(prov, lo, hi, lane, raw, rs);
    __syncthreads();  // the tables are visible to every wave
    PC_PROBE(2, __builtin_amdgcn_s_memrealtime());

    pieces_loop(lds, rs, prov, epi, lo, hi, wpieces, status, wave, lane, raw);
}

// ------------------------------------------------------------------------------------
// 2a. verify fix-up phase (end of k_fixed_braid<VerifyBEpi>)
// ------------------------------------------------------------------------------------
// The braided verify decides the datagrams of the ring's full length; every other one
// (short, empty, runt, 1473-1500 B in a 1504-B slot, oversize) was given ok = 0, crc = 0
// and counted by its wave's flush (nfix).  Once all waves of the workgroup are past their
// braided rounds, a workgroup that counted none returns (one barrier: the common case
// costs nothing).  Otherwise it rebuilds its LDS for the piece loop (PcTables), rescans
// its own packets in passes of kVfPass, compacts the listed ones into an LDS index list
// and finishes them with pieces_loop (DgramProvL semantics: CRC over [16, recv_len),
// Receiver.cpp:25-35,203-206).  Nothing lives outside the caller's buffers and the
// kernel: no list in global memory, no counters, no second launch, so any number of
// concurrent calls, streams and graph replays are independent.  A rescan that finds a
// different number of datagrams than the flushes counted (the recv_len array changed
// under the kernel) sets status bit 2.
//
// LDS after the braided rounds (the piece layout for 8 waves): tables [0, kPcStage),
// staging slots of waves 0..7, the index list where slots 8..15 of k_pieces would be,
// flags at kPcFlags, control words (per-wave counts, list length) past kPcLdsWords.
constexpr uint32_t kVfWaves = 8;  // the verify launch's 512 threads (VerifyBEpi::kThreads)
constexpr uint32_t kVfList = kPcStage + kVfWaves * kPcSlot;
constexpr uint32_t kVfCap = (kPcFlags - kVfList) / 4;
constexpr uint32_t kVfCtl = (kPcLdsWords * 4 + 15) & ~15u;
constexpr uint32_t kVfPer = 8;                          // packets rescanned per thread and pass
constexpr uint32_t kVfPass = kVfWaves * 64 * kVfPer;   // packets rescanned per pass
// Unconditional: a layout that leaves the fix-up list no room (e.g. the rejected 128-B
// piece variant) must not compile, rather than overwrite the flags with indices.
static_assert(kVfPass <= kVfCap && kVfCtl + 64 <= kBraidLdsWords * 4, "verify fix-up LDS");

// Product builds (a3-reliable-transport_amd/Makefile) take every A/B, probe and ablation
// knob of this file at its shipped value; only tools/build_ab.sh and tools/Makefile (kbench,
// pprobe) define WTP_AB_BUILD to build variants.  A misconfigured product build is a
// compile error, not a library that runs wrong.
#ifndef WTP_AB_BUILD
static_assert(WTP_PC_S == 64 && WTP_PC_THREADS == 1024 && WTP_PC_LEN128 == 1 && WTP_PC_LAG == 1 && WTP_PC_DMA == 1 &&
                  WTP_PC_TAILCLAMP == 0 && WTP_PC_SPLIT == 0,
              "product build: piece-kernel knobs must keep their shipped values");
static_assert(WTP_BR_PROLOGUE_DIAG == 0 && WTP_PROBE == 0, "product build: no probe / prologue ablation");
static_assert(WTP_BR_HOLD == 16 && WTP_FILL_X4 == 1 && WTP_FILL_X4_PC == 1,
              "product build: held results every 16 flushes, 16-B table fill (braided and piece kernels)");
static_assert(WTP_BUILD_THREADS == 128 && WTP_BUILD_DIAG == 0 && WTP_BUILD_DEPTH == 2 && WTP_BUILD_SAUX == 2 &&
                  WTP_BUILD_WLEAD == 1 && WTP_BUILD_LAUX == 2 && WTP_BUILD_SAUX0 == 0,
              "product build: fused-builder knobs must keep their shipped values");
#endif

typedef __attribute__((address_space(3))) uint32_t lu32;

// Datagram list[p] of the ring (lead 0: the ring is 16-B aligned); aux = ntohl(checksum).
struct LdsIdxDgramProv {
    static constexpr const char *kName = "LdsIdxDgramProv";  // wtp_last_kernel()
    static constexpr bool kVarLen = false;
    static constexpr bool kIndexed = true;
    static constexpr bool kGroupLoad = false;
    uint64_t stride;
    const uint32_t *__restrict__ rl;
    const lu32 *list;
    __device__ __forceinline__ void load(uint64_t p, MetaRaw &r, __amdgpu_buffer_rsrc_t rs) const {
        const uint32_t idx = list[p];
        const uint32_t h = uint32_t(uint64_t(idx) * stride + 12);  // 4-B aligned, the view is < 2 GiB
        r.a = idx;
        r.b = rl[idx];
        const u32x2 w = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, int(h), 0, 0));
        r.c = w.x;
        r.d = w.y;
    }
    __device__ __forceinline__ void decode(const MetaRaw &r, uint64_t &off, uint32_t &l, bool &ok, uint32_t &want,
                                           uint32_t &slot) const {
        const uint64_t d = r.a * stride;
        want = bswap32(r.c);  // d + 12 is 4-B aligned
        off = d + 16;
        ok = r.b >= 16 && r.b <= stride;
        l = ok ? r.b - 16 : 0;
        slot = uint32_t(r.a);
    }
};

__device__ __forceinline__ void verify_fixup(char *lds, const VerifyBEpi &epi, const uint32_t *gtab, uint32_t nfix,
                                             uint64_t rstep, uint32_t wave, uint32_t lane) {
    lu32 *const ctl = (lu32 *)((lchar *)lds + kVfCtl);  // [w] = wave w's count, [8] = list length
    const uint32_t nwave = blockDim.x >> 6;
    if (lane == 0) ctl[wave] = nfix;
    __syncthreads();  // every wave is past its braided rounds and flushes
    uint32_t total = 0;
    for (uint32_t w = 0; w < nwave; ++w) total += ctl[w];
    total = __builtin_amdgcn_readfirstlane(total);
    if (total == 0) return;
    typedef __attribute__((address_space(1))) uint32_t gmu32;
    gmu32 *const st = (gmu32 *)epi.status;
    if (nwave != kVfWaves) {  // the host launches 512 threads; anything else cannot hold the list
        if (threadIdx.x == 0) __hip_atomic_fetch_or(st, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    {
        PcTables<kVfWaves * 64> tb;  // overwrites the braid tables: no wave reads them any more
        tb.load(gtab);
        tb.store(lds, gtab);
    }
    const uint64_t n = epi.n;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(epi.ring, uint32_t((n * epi.stride + 15) & ~uint64_t(15)));
    const __amdgpu_buffer_rsrc_t rr = make_rsrc(epi.rl, uint32_t(4 * n));
    lu32 *const list = (lu32 *)((lchar *)lds + kVfList);
    const LdsIdxDgramProv prov{epi.stride, epi.rl, list};
    const VerifyEpi vepi{epi.ok, epi.crc, uint32_t(n)};
    const uint64_t g0 = uint64_t(blockIdx.x) * nwave;  // the workgroup's first round
    uint32_t found = 0;
    // the workgroup's packets in braided order: enumeration index e <-> packet
    // 4 (g0 + (e >> 5) rstep) + (e & 31) (wave (e & 31) >> 2's round of group e >> 5)
    for (uint64_t e0 = 0; 4 * (g0 + (e0 >> 5) * rstep) < n; e0 += kVfPass) {
        if (threadIdx.x == 0) ctl[8] = 0;
        __syncthreads();  // publishes the tables (first pass) and the reset list length
        uint64_t pv[kVfPer];
        uint32_t rv[kVfPer];
#pragma unroll
        for (uint32_t k = 0; k < kVfPer; ++k) {
            const uint64_t e = e0 + k * (kVfWaves * 64) + threadIdx.x;
            pv[k] = 4 * (g0 + (e >> 5) * rstep) + (e & 31u);
            rv[k] = __builtin_amdgcn_raw_buffer_load_b32(rr, pv[k] < n ? int(4 * pv[k]) : int(0x80000000u), 0, 0);
        }
#pragma unroll
        for (uint32_t k = 0; k < kVfPer; ++k) {
            const bool need = pv[k] < n && rv[k] != epi.full;
            const uint64_t m = __ballot(need);
            if (m == 0) continue;  // wave-uniform
            uint32_t b = 0;
            if (lane == 0) b = __hip_atomic_fetch_add(&ctl[8], uint32_t(__popcll(m)), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
            b = __builtin_amdgcn_readfirstlane(b);
            const uint32_t pos = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
            if (need) list[b + pos] = uint32_t(pv[k]);
        }
        __syncthreads();
        const uint32_t c = __builtin_amdgcn_readfirstlane(ctl[8]);
        found += c;
        const uint64_t lo = uint64_t(c) * wave / kVfWaves, hi = uint64_t(c) * (wave + 1) / kVfWaves;
        MetaRaw raw{};
        if (lo < hi) pieces_meta(prov, lo, hi, lane, raw, rs);
        pieces_loop(lds, rs, prov, vepi, lo, hi, 0u, epi.status, wave, lane, raw);
        __syncthreads();  // the next pass rebuilds the list
    }
    if (threadIdx.x == 0 && found != total) __hip_atomic_fetch_or(st, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------
// 2b. stream kernel (packed mixed lengths: payload p+1 starts where payload p ends)
// ------------------------------------------------------------------------------------
// A receive buffer or record file holds its payloads back to back, so a wave can hash
// its region of the byte stream as one uniform stream and read every payload's CRC off
// prefix values:  P(x) = R_0(stream[X0 .. x)) for the wave's start X0, and
//   crc(payload [a, b)) = P(b) ^ shift(P(a) ^ ~0, b - a) ^ ~0
// (R_0(M[a,b)) = P(b) ^ shift(P(a), b - a); the CRC's ~0 init enters as shift(~0, len)).
// Packed, P(a) of payload p is P(b) of payload p-1.  Per round a wave
//   1. stages 8 KiB of the stream into its LDS slot (lane-contiguous 1 KiB loads,
//      prefetched a round ahead); lane l takes bytes [128 l, 128 l + 128);
//   2. chains its four 32-B blocks independently (slice-by-4, no masking, no rotation:
//      the stream is 16-B aligned), combines them by Horner with T256 = shift(., 32 B),
//      scans the 64 lane values with shift(., 128 * 2^k B) seeded with G = P(round
//      start), and stores the four block anchors P(block start) next to its data;
//   3. for the payloads that end in this round (lane i <-> payload q + i), evaluates
//      P(b) = the block anchor fed with the t < 32 bytes of the block before b, takes
//      P(a) from the lane below (lane 0: the previous payload's), and applies the
//      length shift in four 3-bit levels of nibble-table operators.
// Payloads that break the packing (or are >= 4096 B) are found when their metadata is
// decoded; the wave hands them to a lane-per-payload path at its end (correct for any
// offsets, slower), so the entry point is exact for every input.
// Wave ranges inside a workgroup are balanced by bytes + 64 per payload.
constexpr uint32_t kStThreads = 512, kStWaves = kStThreads / 64;
constexpr uint32_t kStRound = 8192;                     // stream bytes per wave round
constexpr uint32_t kStLane = 144;                       // per lane: 128 B of data + 16 B of anchors
constexpr uint32_t kStSlot = 64 * kStLane;              // 9216 B per wave
constexpr uint32_t kStNib = 65536;                      // after region 0 (S4 + T256 staggered)
constexpr uint32_t kStSlots = kStNib + kStNibOps * 512;
constexpr uint32_t kStBal = kStSlots + kStWaves * kStSlot;
constexpr uint32_t kStLdsWords = (kStBal + (kStWaves + 1) * 8) / 4;
constexpr uint32_t kStMaxLen = 4095;  // the length shift has four 3-bit levels
static_assert(kStLdsWords * 4 <= 163840, "k_stream LDS");


// P at round position x (0 <= x < kStRound): lane x/128's anchor for the 32-B block
// holding x, fed with the t = x % 32 block bytes before x (whole words by slice-by-4,
// then the last r = t % 4 bytes as c' = (c >> 8r) ^ T4((c ^ w) << (32 - 8r))).
__device__ __forceinline__ uint32_t st_feed(const char *lds, lchar *slot, const StagKeys &K, uint32_t x) {
    typedef const __attribute__((address_space(3))) uint32_t lu32c;
    const uint32_t l = x >> 7, blk = (x >> 5) & 3u, t = x & 31u;
    lchar *const b = slot + l * kStLane + blk * 32u;
    uint32_t c = *(lu32c *)(slot + l * kStLane + 128u + 4u * blk);
    const u32x4 w0 = *(const lu32x4 *)b, w1 = *(const lu32x4 *)(b + 16);
    const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    const uint32_t nw = t >> 2, r = t & 3u;
    const uint32_t wn = *(lu32c *)(b + 4u * nw);
#pragma unroll
    for (uint32_t k = 0; k < 7; ++k) {
        if (__ballot(k < nw) == 0) break;  // wave-uniform trip count: the largest nw
        const uint32_t y = stag_apply3<0>(lds, K.kA, K.sel, c ^ w[k]);
        c = k < nw ? y : c;
    }
    const uint32_t y = r ? (c ^ wn) << (32u - 8u * r) : 0u;
    return (c >> (8u * r)) ^ stag_apply3<0>(lds, K.kA, K.sel, y);
}

template <int DUMMY = 0>
__global__ __launch_bounds__(kStThreads) void k_stream(const uint8_t *__restrict__ view, uint64_t view_bytes,
                                                     const uint64_t *__restrict__ offs,
                                                     const uint32_t *__restrict__ lens, uint64_t lead, uint64_t n,
                                                     uint32_t *__restrict__ out, const uint32_t *__restrict__ gtab,
                                                     uint32_t *__restrict__ status, const RangeDesc *__restrict__ gate,
                                                     uint32_t ngate) {
    typedef const __attribute__((address_space(1))) uint64_t gu64;
    typedef const __attribute__((address_space(1))) uint32_t gu32;
    // Fallback of launch_packed_ranges: runs only if a piece sub-launch found a packet
    // outside its view (the offsets were not packed); then it redoes the whole batch.
    if (gate) {
        uint32_t any = 0;
        for (uint32_t j = 0; j < ngate; ++j) any |= gate[j].bad;
        if (!any) return;
    }
    __shared__ __attribute__((aligned(16))) uint32_t lds_w[kStLdsWords];
    char *lds = reinterpret_cast<char *>(lds_w);
    const uint64_t g0 = n * blockIdx.x / gridDim.x, g1 = n * (blockIdx.x + 1) / gridDim.x;
    if (g0 == g1) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto off_of = [&](uint64_t p) { return ((gu64 *)offs)[p] + lead; };  // view offset
    auto len_of = [&](uint64_t p) { return ((gu32 *)lens)[p]; };

    // --- wave ranges: boundaries at equal weight (bytes + 64 per payload), found among
    // 512 evenly spaced sample payloads; a prefix max keeps the partition monotone
    // whatever the offsets hold ------------------------------------------------------
    uint64_t *const starts = reinterpret_cast<uint64_t *>(lds + kStBal);
    const uint64_t span = g1 - g0;
    const uint64_t smp = g0 + ((span * threadIdx.x) >> 9);
    if (threadIdx.x <= kStWaves) starts[threadIdx.x] = threadIdx.x == 0 ? g0 : g1;
    uint64_t o0, oe, os;
    {
        // table loads ahead of the sample loads (vmcnt completes in order; see StagFill)
        constexpr uint32_t kNQ = kStNibOps * 32, kNPer = (kNQ + kStThreads - 1) / kStThreads;
        const u32x4 *src = reinterpret_cast<const u32x4 *>(gtab + OFF_NIB);
        const StagSet sets[2] = {{gtab + OFF_S4, 0u}, {gtab + OFF_T256, 128u}};
        StagFill<2, kStThreads> fill;
        fill.load(sets);
        u32x4 q[kNPer];
#pragma unroll
        for (uint32_t k = 0; k < kNPer; ++k) {
            const uint32_t i = threadIdx.x + k * kStThreads;
            q[k] = src[i < kNQ ? i : 0];
        }
        o0 = off_of(g0);
        oe = off_of(g1 - 1) + len_of(g1 - 1);
        os = off_of(smp);
        fill.store(lds, sets);
        u32x4 *dst = reinterpret_cast<u32x4 *>(lds + kStNib);
#pragma unroll
        for (uint32_t k = 0; k < kNPer; ++k) {
            const uint32_t i = threadIdx.x + k * kStThreads;
            if (i < kNQ) dst[i] = q[k];
        }
    }
    __syncthreads();
    {
        const uint64_t wtot = (oe - o0) + 64 * span, wsm = (os - o0) + 64 * (smp - g0);
        for (uint32_t w = 1; w < kStWaves; ++w) {
            const uint64_t m = __ballot(wsm >= (wtot >> 3) * w);
            if (m && lane == uint32_t(__builtin_ctzll(m))) atomicMin(reinterpret_cast<unsigned long long *>(starts + w),
                                                                    (unsigned long long)smp);
        }
    }
    __syncthreads();
    uint64_t lo = starts[0];
    for (uint32_t w = 1; w <= wave; ++w) lo = starts[w] > lo ? starts[w] : lo;
    const uint64_t hi = starts[wave + 1] > lo ? starts[wave + 1] : lo;
    lo = uniform64(lo);
    if (lo >= hi) return;  // no block barrier below this point

    const StagKeys K(lane);
    lchar *const slot = (lchar *)lds_w + kStSlots + wave * kStSlot;
    const uint64_t vabs = uint64_t(reinterpret_cast<uintptr_t>(view));
    const uint64_t vb16 = (view_bytes + 15) & ~uint64_t(15);

    // --- metadata: groups of 64 payloads; lane i of group gs <-> payload gs + i -------
    auto load_group = [&](uint64_t gs, uint64_t &o, uint32_t &l) {
        const uint64_t p = gs + lane, pc = p < hi ? p : hi - 1;
        o = off_of(pc);
        l = len_of(pc);
    };
    uint64_t oA, oB, oC;
    uint32_t lA, lB, lC;
    load_group(lo, oA, lA);
    load_group(lo + 64, oB, lB);
    // (uniform64 widens each half as unsigned: an earlier form OR'ed the int that
    // readfirstlane returns into the 64-bit value, sign-extending the low half, so a wave
    // whose first offset had bit 31 set got a garbage stream base and ran its whole range
    // on the lane-per-payload path: exact, 6-7x slower, e.g. any wave starting between 2
    // and 4 GiB into the buffer)
    const uint64_t o_lo = uniform64(oA);
    const uint64_t wb = ((vabs + o_lo) & ~uint64_t(127)) - vabs;  // X0 (view offset, mod 2^64)
    uint64_t fb = hi;    // first payload that breaks the packing (wave-uniform)
    uint64_t pe = o_lo;  // end of the payload before the group being decoded
    // decode: relative end e (to X0) and length; flags the first payload that is not
    // packed, is >= 4096 B, or lies outside 4 GiB of X0
    auto decode = [&](uint64_t gs, uint64_t o, uint32_t l, uint32_t &e, uint32_t &len) {
        const uint64_t end = o + l;
        const uint32_t plo = uint32_t(__builtin_amdgcn_update_dpp(int(uint32_t(pe)), int(uint32_t(end)), 0x138, 0xF, 0xF, false));
        const uint32_t phi = uint32_t(__builtin_amdgcn_update_dpp(int(uint32_t(pe >> 32)), int(uint32_t(end >> 32)), 0x138, 0xF, 0xF, false));
        const uint64_t prev = uint64_t(plo) | (uint64_t(phi) << 32);  // lane 0: pe (wave_shr:1 keeps old)
        const uint64_t p = gs + lane;
        const bool bad = p < hi && ((p > lo && o != prev) || l > kStMaxLen || end - wb >= (1ull << 32));
        const uint64_t m = __ballot(bad);
        if (m) {
            const uint64_t f = gs + uint64_t(__builtin_ctzll(m));
            fb = f < fb ? f : fb;
        }
        e = uint32_t(end - wb);
        len = l;
        pe = uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(end)), 63))) |
             (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(end >> 32)), 63))) << 32);
    };
    uint32_t eA, nA, eB, nB;
    decode(lo, oA, lA, eA, nA);
    decode(lo + 64, oB, lB, eB, nB);

    // --- stream rounds ------------------------------------------------------------------
    auto load_round = [&](uint64_t rrel, u32x4 (&x)[8]) {
        const int64_t st = int64_t(wb + rrel);
        const uint64_t sp = st < 0 ? 0 : uint64_t(st);
        const int32_t adj = int32_t(st - int64_t(sp));  // <= 0: chunks before the view read 0
        const uint64_t left = sp < vb16 ? vb16 - sp : 0;
        const auto rs = make_rsrc(view + sp, uint32_t(left < 0x7FFFFFF0u ? left : 0x7FFFFFF0u));
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i)
            x[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rs, int(uint32_t(adj) + 16u * (64u * i + lane)), 0, 2));
    };
    u32x4 x[8];
    load_round(0, x);
    uint64_t rrel = 0, gsA = lo;
    uint32_t G = 0, d = 0, cP = 0;
    bool first = true;
    const uint32_t scan0 = kStNib;  // shift by 128 B
    for (;;) {
        // 1. stage (chunk c of the round -> lane c/8's data at 16 (c % 8)) and prefetch
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t c = 64u * i + lane;
            *(lu32x4 *)(slot + kStLane * (c >> 3) + 16u * (c & 7u)) = x[i];
        }
        // group C (the one after B) is (re)issued before the prefetch, so a rotation in
        // this round waits for it with a counted vmcnt that leaves the prefetch in flight
        load_group(gsA + 128, oC, lC);
        load_round(rrel + kStRound, x);
        bool rotated = false;
        __builtin_amdgcn_wave_barrier();
        // 2. chain the lane's four 32-B blocks (independent), Horner, scan, anchors
        uint32_t w[32];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            const u32x4 y = *(const lu32x4 *)(slot + kStLane * lane + 16u * u);
            w[4 * u] = y.x;
            w[4 * u + 1] = y.y;
            w[4 * u + 2] = y.z;
            w[4 * u + 3] = y.w;
        }
        uint32_t cb[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) cb[j] = w[8 * j];
#pragma unroll
        for (uint32_t k = 1; k < 8; ++k)
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) cb[j] = stag_apply3x<0>(lds, K.kA, K.sel, cb[j], w[8 * j + k]);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) cb[j] = stag_apply3<0>(lds, K.kA, K.sel, cb[j]);  // R_0(block j)
        uint32_t V = cb[0];
#pragma unroll
        for (uint32_t j = 1; j < 4; ++j) V = stag_apply3x<128>(lds, K.kA, K.sel, V, cb[j]);  // T256(V) ^ c_j
        const uint32_t gs128 = nib_apply(lds, scan0, G);  // shift(G, 128 B)
        uint32_t I = V ^ (lane == 0 ? gs128 : 0u);
#pragma unroll
        for (uint32_t k = 0; k < 6; ++k) {
            const uint32_t dd = 1u << k;
            const uint32_t y = nib_apply(lds, kStNib + 512u * k, __shfl_up(I, dd));
            I = lane >= dd ? I ^ y : I;
        }
        uint32_t A0 = __shfl_up(I, 1);
        A0 = lane == 0 ? G : A0;
        const uint32_t A1 = stag_apply3x<128>(lds, K.kA, K.sel, A0, cb[0]);
        const uint32_t A2 = stag_apply3x<128>(lds, K.kA, K.sel, A1, cb[1]);
        const uint32_t A3 = stag_apply3x<128>(lds, K.kA, K.sel, A2, cb[2]);
        *(lu32x4 *)(slot + kStLane * lane + 128u) = u32x4{A0, A1, A2, A3};
        const uint32_t Gn = __builtin_amdgcn_readlane(I, 63);
        __builtin_amdgcn_wave_barrier();
        if (first) {  // P(a) of the wave's first payload
            cP = __builtin_amdgcn_readfirstlane(st_feed(lds, slot, K, uint32_t(o_lo - wb)));
            first = false;
        }
        // 3. the payloads that end in this round, 64 at a time (fb can drop when a group
        // is decoded at a rotation, so the end of the fast range is re-read each time)
        for (;;) {
            const uint64_t pend = fb < hi ? fb : hi;
            const uint32_t idx = d + lane;
            const uint32_t src = (idx & 63u) << 2;
            const uint32_t ea = uint32_t(__builtin_amdgcn_ds_bpermute(int(src), int(eA)));
            const uint32_t eb = uint32_t(__builtin_amdgcn_ds_bpermute(int(src), int(eB)));
            const uint32_t na = uint32_t(__builtin_amdgcn_ds_bpermute(int(src), int(nA)));
            const uint32_t nb = uint32_t(__builtin_amdgcn_ds_bpermute(int(src), int(nB)));
            const uint32_t e = idx < 64u ? ea : eb, len = idx < 64u ? na : nb;
            const uint64_t p = gsA + idx;
            const bool ends = p < pend && uint64_t(e) < rrel + kStRound;
            const uint64_t em = __ballot(ends);
            if (em == 0) break;
            const uint32_t m = uint32_t(__popcll(em));  // a prefix of the lanes: ends are sorted
            const uint32_t pb = st_feed(lds, slot, K, ends ? uint32_t(e - uint32_t(rrel)) : 0u);
            uint32_t v = __shfl_up(pb, 1);
            v = (lane == 0 ? cP : v) ^ 0xFFFFFFFFu;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) v = nib_apply(lds, kStNib + 512u * (6u + 8u * k + ((len >> (3 * k)) & 7u)), v);
            const auto ro = make_rsrc(out + gsA + d, 256u);
            __builtin_amdgcn_raw_buffer_store_b32(pb ^ v ^ 0xFFFFFFFFu, ro, ends ? int(4u * lane) : int(0x80000000u), 0, 0);
            cP = __builtin_amdgcn_readlane(pb, m - 1);
            d += m;
            if (d >= 64u) {  // group A done: B -> A, C -> B
                eA = eB;
                nA = nB;
                gsA += 64;
                d -= 64u;
                if (rotated) {  // a second rotation this round (> ~128 short payloads): load C now
                    load_group(gsA + 64, oC, lC);
                    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                }
                decode(gsA + 64, oC, lC, eB, nB);
                rotated = true;
            }
            if (m < 64u) break;
        }
        if (gsA + d >= (fb < hi ? fb : hi)) break;
        G = Gn;
        rrel += kStRound;
    }

    // --- payloads [fb, hi): one lane per payload, 16-B chunks straight from memory
    // (the next chunk prefetched while this one is fed word by word) --------------------
    typedef const __attribute__((address_space(1))) u32x4 gq;
    if (fb < hi && lane == 0) atomicOr(status, 8u);  // informational: this batch left the fast path
    for (uint64_t g = fb; g < hi; g += 64) {
        const uint64_t p = g + lane, pc = p < hi ? p : hi - 1;
        const uint64_t o = off_of(pc);
        const uint32_t l0 = len_of(pc);
        const bool have = p < hi, over = l0 > kMaxVarLen;
        if (have && over) atomicOr(status, 1u);
        const int32_t L = have && !over ? int32_t(l0) : 0;
        const uint64_t a0 = o & ~uint64_t(15);
        const int32_t ld0 = int32_t(o & 15u);
        const uint32_t nq = L ? uint32_t(ld0 + L + 15) >> 4 : 0u;
        auto chunk = [&](uint32_t k) {  // chunk k of the payload, 0 outside the view
            const uint64_t a = a0 + 16ull * k;
            const bool in = k < nq && a + 16 <= vb16;
            gq *const src = in ? (gq *)view + (a >> 4) : (gq *)gtab;  // never an address outside the view
            const u32x4 q = *src;
            return in ? q : u32x4{0u, 0u, 0u, 0u};
        };
        uint32_t c = 0xFFFFFFFFu;
        u32x4 cur = chunk(0);
        for (uint32_t k = 0;; ++k) {
            if (__ballot(k < nq) == 0) break;
            const u32x4 nxt = chunk(k + 1);
            const uint32_t wv[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                // payload bytes [b0, b0 + 4) of this word; feed its bytes in [0, L)
                const int32_t b0 = int32_t(16u * k + 4u * u) - ld0;
                const int32_t s0 = b0 < 0 ? -b0 : 0, e0 = L - b0 < 4 ? L - b0 : 4;
                const int32_t r = e0 - s0;
                const uint32_t rr = r > 0 ? uint32_t(r) : 4u, ss = s0 < 4 ? uint32_t(s0) : 0u;
                const uint32_t yv = wv[u] >> (8u * ss);
                const uint32_t c2 = uint32_t(uint64_t(c) >> (8u * rr)) ^
                                    stag_apply3<0>(lds, K.kA, K.sel, uint32_t(uint64_t(c ^ yv) << (32u - 8u * rr)));
                c = r > 0 && k < nq ? c2 : c;
            }
            cur = nxt;
        }
        const auto ro = make_rsrc(out + g, 256u);
        __builtin_amdgcn_raw_buffer_store_b32(c ^ 0xFFFFFFFFu, ro, have ? int(4u * lane) : int(0x80000000u), 0, 0);
    }
}

// ------------------------------------------------------------------------------------
// 3. fused DATA packet builder
// ------------------------------------------------------------------------------------
// Stage A: copy chunk i into its wire slot after a 16-B header hole; CRC computed on
// the payload with the general kernel, then stage B writes the big-endian header.
__global__ void k_wire_copy(const uint8_t *__restrict__ src, uint64_t total, uint8_t *__restrict__ wire,
                            uint64_t wstride, uint64_t nchunks) {
    const uint64_t per = WTP_MAX_PAYLOAD;
    for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;; t += uint64_t(gridDim.x) * blockDim.x) {
        const uint64_t i = t / (per / 4 + 1);  // 364 dwords + 1 header slot per chunk
        if (i >= nchunks) break;
        const uint64_t w = t % (per / 4 + 1);
        if (w == per / 4) continue;
        const uint64_t so = i * per + w * 4;
        uint8_t *dst = wire + i * wstride + 16 + w * 4;
        if (so + 4 <= total) {
            uint32_t v;
            memcpy(&v, src + so, 4);
            memcpy(dst, &v, 4);
        } else {
            for (uint64_t b = so; b < total && b < so + 4; ++b) dst[b - so] = src[b];
        }
    }
}
// crc and wlen may be the same buffer (the CRCs are staged in d_wire_len, then become the
// lengths): neither is __restrict__, so each thread's crc[i] load stays ahead of its
// wlen[i] store.
__global__ void k_wire_header(const uint32_t *crc, uint64_t total, uint32_t seq0, uint8_t *__restrict__ wire,
                              uint64_t wstride, uint32_t *wlen, uint64_t nchunks) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nchunks;
         i += uint64_t(gridDim.x) * blockDim.x) {
        const uint64_t rem = total - i * WTP_MAX_PAYLOAD;
        const uint32_t len = uint32_t(rem < WTP_MAX_PAYLOAD ? rem : WTP_MAX_PAYLOAD);
        const uint32_t hdr[4] = {bswap32(WTP_TYPE_DATA), bswap32(seq0 + uint32_t(i)), bswap32(len), bswap32(crc[i])};
        memcpy(wire + i * wstride, hdr, 16);
        if (wlen) wlen[i] = 16 + len;
    }
}

// ------------------------------------------------------------------------------------
// 4. synthetic payload fill
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void k_synth(uint8_t *__restrict__ out, uint64_t start, uint64_t nbytes, uint64_t seed) {
    const uint64_t w0 = start >> 3, w1 = (start + nbytes + 7) >> 3;
    for (uint64_t w = w0 + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w < w1;
         w += uint64_t(gridDim.x) * blockDim.x) {
        const uint64_t z = mix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull);
        const uint64_t g0 = w << 3;
        if (g0 >= start && g0 + 8 <= start + nbytes && ((reinterpret_cast<uintptr_t>(out + (g0 - start)) & 7u) == 0)) {
            *reinterpret_cast<uint64_t *>(out + (g0 - start)) = z;
        } else {
            for (uint32_t b = 0; b < 8; ++b) {
                const uint64_t g = g0 + b;
                if (g >= start && g < start + nbytes) out[g - start] = uint8_t(z >> (8 * b));
            }
        }
    }
}

}  // namespace dev

// ------------------------------------------------------------------------------------
// host side: per-device state, error handling, launchers
// ------------------------------------------------------------------------------------
namespace {

thread_local std::string g_err;
thread_local std::string g_kernel;  // wtp_last_kernel(): the calling thread's last launch

void note_kernel(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void note_kernel(const char *fmt, ...) {
    char buf[128];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_kernel = buf;
}

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define WTP_HIP(call)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) return fail(WTP_EHIP, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)

constexpr size_t kStreamScratch = 32768;  // launch_packed_ranges' descriptors (one call)
constexpr unsigned kCaptureSlots = 64;     // descriptor buffers for calls captured into graphs
struct DevState {
    std::once_flag once;
    int rc = WTP_OK;
    std::string err;
    uint32_t *tabs = nullptr;
    uint32_t *status = nullptr;
    int cus = 0;
    std::atomic<int> reserve{0};  // CUs left free of the persistent kernels (wtp_reserve_cus)
    unsigned grid_cus() const { return unsigned(std::max(1, cus - reserve.load(std::memory_order_relaxed))); }
    hipMemPool_t pool = nullptr;  // library-owned stream-ordered pool, never trimmed (builder scratch)
    // Device scratch of fixed size for launch_packed_ranges' descriptors.  Outside graph
    // capture: one buffer per stream, made on the stream's first use and kept (calls on one
    // stream are ordered, so they may share it).  During capture: a slot of `cap`, taken
    // by that one captured call for the life of the process, so two graphs captured on one
    // stream (torch's shared capture stream) never share descriptors when replayed at
    // once; with every slot taken, a captured call takes k_stream instead (exact, no
    // scratch).  Both kinds are plain hipMalloc memory made outside any capture, so a graph
    // bakes in a buffer that outlives it.  (Stream-ordered pool allocations inside a
    // capture replayed wrongly when one graph held several calls: the sub-launches read
    // zeroed descriptors and did nothing; profiles/r05)
    std::mutex smu;
    std::unordered_map<hipStream_t, void *> sbuf;
    uint8_t *cap = nullptr;  // kCaptureSlots x kStreamScratch, made at init
    unsigned cap_used = 0;
};
constexpr int kMaxDev = 64;
DevState g_dev[kMaxDev];

std::vector<uint32_t> host_tables() {
    std::vector<uint32_t> t(TAB_WORDS, 0);
    make_word_tables(&t[OFF_BRAID], kBraidBlock);
    const uint32_t inv_bytes[6] = {4, 8, 16, 32, 64, 128};
    for (int o = 0; o < 6; ++o)
        make_operator(&t[OFF_INV + 1024 * o], [&](uint32_t v) { return unshift_bytes(v, inv_bytes[o]); });
    make_word_tables(&t[OFF_S4], 4);
    for (int o = 0; o < 6; ++o) {
        const uint64_t nb = uint64_t(kPieceS) << o;
        make_operator(&t[OFF_FWD + 1024 * o], [&](uint32_t v) { return shift_bytes(v, nb); });
    }
    for (uint32_t h = 0; h <= uint32_t(kPieceS); ++h) t[OFF_HINIT + h] = shift_bytes(0xFFFFFFFFu, h);
    make_operator(&t[OFF_X64], [](uint32_t v) { return shift_bytes(v, 64); });
    make_word_tables(&t[OFF_S8], 8);
    make_operator(&t[OFF_T256], [](uint32_t v) { return shift_bytes(v, 32); });
    auto nib = [&](uint32_t op, uint64_t nbytes) {
        for (uint32_t i = 0; i < 8; ++i)
            for (uint32_t e = 0; e < 16; ++e) t[OFF_NIB + 128 * op + 16 * i + e] = shift_bytes(e << (4 * i), nbytes);
    };
    for (uint32_t k = 0; k < 6; ++k) nib(k, uint64_t(128) << k);
    for (uint32_t k = 0; k < 4; ++k)
        for (uint32_t j = 0; j < 8; ++j) nib(6 + 8 * k + j, uint64_t(j) << (3 * k));
    return t;
}

int init_device(int dev) {
    if (dev < 0 || dev >= kMaxDev) return fail(WTP_EINVAL, "device %d out of range", dev);
    DevState &s = g_dev[dev];
    std::call_once(s.once, [&] {
        auto setfail = [&](int code, const std::string &m) {
            s.rc = code;
            s.err = m;
        };
        int prev = 0;
        (void)hipGetDevice(&prev);
        auto setup = [&]() {
            if (hipSetDevice(dev) != hipSuccess) return setfail(WTP_ENODEV, "hipSetDevice failed");
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return setfail(WTP_ENODEV, "hipGetDeviceProperties failed");
            if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
                return setfail(WTP_ENODEV, std::string("device is ") + prop.gcnArchName + ", library built for gfx950");
            s.cus = prop.multiProcessorCount;
            std::vector<uint32_t> t = host_tables();
            if (hipMalloc(&s.tabs, t.size() * 4) != hipSuccess) return setfail(WTP_ENOMEM, "hipMalloc(tables) failed");
            if (hipMemcpy(s.tabs, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
                return setfail(WTP_EHIP, "hipMemcpy(tables) failed");
            if (hipMalloc(&s.status, 4) != hipSuccess) return setfail(WTP_ENOMEM, "hipMalloc(status) failed");
            if (hipMemset(s.status, 0, 4) != hipSuccess) return setfail(WTP_EHIP, "hipMemset(status) failed");
            // Scratch of async entry points (the builder's CRCs on its slow path) comes from a
            // library-owned pool whose memory is kept across calls (release threshold max):
            // the default threshold returns it at every synchronisation, and re-mapping it
            // cost ~1 ms per small host-verify call.
            hipMemPoolProps pp{};
            pp.allocType = hipMemAllocationTypePinned;
            pp.location.type = hipMemLocationTypeDevice;
            pp.location.id = dev;
            if (hipMalloc(&s.cap, kCaptureSlots * kStreamScratch) != hipSuccess)
                return setfail(WTP_ENOMEM, "hipMalloc(capture scratch) failed");
            if (hipMemPoolCreate(&s.pool, &pp) != hipSuccess) return setfail(WTP_EHIP, "hipMemPoolCreate failed");
            uint64_t keep = UINT64_MAX;
            if (hipMemPoolSetAttribute(s.pool, hipMemPoolAttrReleaseThreshold, &keep) != hipSuccess)
                return setfail(WTP_EHIP, "hipMemPoolSetAttribute failed");
        };
        setup();
        (void)hipSetDevice(prev);  // the caller's current device, on success and on failure
        (void)hipGetLastError();
    });
    if (s.rc != WTP_OK) return fail(s.rc, "wtp init(device %d): %s", dev, s.err.c_str());
    return WTP_OK;
}

int current(DevState *&s) {
    int dev = 0;
    WTP_HIP(hipGetDevice(&dev));
    int rc = init_device(dev);
    if (rc) return rc;
    s = &g_dev[dev];
    return WTP_OK;
}

// Descriptor scratch (kStreamScratch bytes) for one launch_packed_ranges call on `st`
// (DevState::sbuf / cap).  *out = nullptr: the call is being captured and every capture
// slot is taken; the caller then takes the scratch-free k_stream route.
int stream_scratch(DevState &s, hipStream_t st, void **out) {
    std::lock_guard<std::mutex> g(s.smu);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    WTP_HIP(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone) {
        *out = s.cap_used < kCaptureSlots ? s.cap + kStreamScratch * s.cap_used++ : nullptr;
        return WTP_OK;
    }
    auto it = s.sbuf.find(st);
    if (it != s.sbuf.end()) {
        *out = it->second;
        return WTP_OK;
    }
    void *p = nullptr;
    WTP_HIP(hipMalloc(&p, kStreamScratch));
    s.sbuf.emplace(st, p);
    *out = p;
    return WTP_OK;
}

int launch_check(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WTP_EHIP, "launch %s: %s", what, hipGetErrorString(e));
    return WTP_OK;
}

// Workgroup size of the braided kernel (one workgroup per CU: its LDS tables take the
// CU's 160 KiB).  Interleaved A/B on one box (profiles/r01i/ab_braid_threads.txt):
//   CRC / verify, 1 M x 1456 B: 1024 threads 0.2325 ms, 768 0.2334, 640 0.2286,
//     576 0.2271, 512 0.2219 (86% of HBM peak), 448 0.2289, 384 0.2353, 256 0.2720;
//   fused builder (reads + wire writes): 1024 0.769 ms, 512 0.745, 256 0.680,
//     192 0.667, 128 0.653, 64 1.052.
// Fewer waves per CU keep fewer rows in flight; HBM serves the stream with less
// queueing (and, for the builder, fewer read/write turnarounds) while 8 resp. 2 waves,
// two rounds each, still cover its latency.
// (the sizes are each epilogue's kThreads: CrcBEpi and VerifyBEpi 512, BuildBEpi 128)
static_assert(dev::VerifyBEpi::kThreads == dev::CrcBEpi::kThreads, "one braided grid rule");
static_assert(dev::VerifyBEpi::kThreads == 64 * dev::kVfWaves, "verify fix-up LDS layout");

template <int ROWS, class BEpi>
void launch_braid_rows(dim3 grid, unsigned threads, hipStream_t st, const uint8_t *b, uint64_t stride, uint32_t len,
                       uint64_t n, BEpi epi, const uint32_t *tabs) {
    note_kernel("k_fixed_braid<%d, %d, %s>", ROWS, BEpi::kDiag, BEpi::kName);
    hipLaunchKernelGGL((dev::k_fixed_braid<ROWS, BEpi::kDiag, BEpi>), grid, dim3(threads), 0, st, b,
                       uint32_t(stride), len, n, epi, tabs);
}

// Braided kernel over n packets base[p*stride, +len): base, stride, len multiples of 16,
// 16 <= len <= 1536, stride <= 16 KiB.  The epilogue's cinit is filled in here.
template <class BEpi>
int launch_fixed_braid_rows(DevState &s, const uint8_t *base, uint64_t stride, uint32_t len, uint64_t n, BEpi epi,
                            hipStream_t st, unsigned grid, unsigned threads, int rows);
#ifndef WTP_BR_HOLD_ROUNDS
#define WTP_BR_HOLD_ROUNDS 64  // rounds per wave from which the CRC holds its results (CrcHoldBEpi)
#endif
#ifndef WTP_AB_BUILD
static_assert(WTP_BR_HOLD_ROUNDS == 64, "product build: held results from 64 rounds per wave");
#endif

template <class BEpi>
int launch_fixed_braid(DevState &s, const uint8_t *base, uint64_t stride, uint32_t len, uint64_t n, BEpi epi,
                       hipStream_t st) {
    const int rows = int((len + 255) / 256);
    const unsigned threads = BEpi::kThreads;
    const uint64_t rounds = (n + 3) / 4;
    const uint64_t want = (rounds + threads / 64 - 1) / (threads / 64);
    uint64_t cap = s.grid_cus();
    // Long streaming batches (>= 64 rounds per wave) run one workgroup per XCD fewer than
    // CUs: fewer rows in flight queue less at HBM.  Interleaved A/B, 8 reps
    // (profiles/r02h/ab_reserve2.log): 1 M x 1456 B 220.6 us at 256 workgroups, 218.7 at
    // 252, 217.4 at 248, 217.5-217.7 at 244-232; 2 M 460.6 vs 452.2 us at 248.  Short
    // batches keep every CU (C2: 8 rounds per wave, a ninth would be its tail).
    if (!BEpi::kCopy && s.reserve.load(std::memory_order_relaxed) == 0 && rounds >= 64 * cap * (threads / 64))
        cap -= cap / 32;
    const unsigned grid = unsigned(want < cap ? want : cap);
    epi.cinit = init_const(len);
    if constexpr (std::is_same_v<BEpi, dev::CrcBEpi>) {
        // long batches hold their results in LDS (k_fixed_braid, kDump): short ones store
        // directly, the held form's code was 1.4-1.7% slower on 16 K-64 K packets even with
        // nothing held (profiles/r04u).  The held form's bursts are 16-B stores at
        // out + 16 k: only a 16-B aligned `out` takes it (a torch slice out[1:] is only
        // 4-B aligned; it keeps the direct dword stores).
        if (rounds >= uint64_t(WTP_BR_HOLD_ROUNDS) * grid * (threads / 64) &&
            (reinterpret_cast<uintptr_t>(epi.out) & 15u) == 0) {
            dev::CrcHoldBEpi h;
            static_cast<dev::CrcBEpi &>(h) = epi;
            return launch_fixed_braid_rows(s, base, stride, len, n, h, st, grid, threads, rows);
        }
    }
    return launch_fixed_braid_rows(s, base, stride, len, n, epi, st, grid, threads, rows);
}

template <class BEpi>
int launch_fixed_braid_rows(DevState &s, const uint8_t *base, uint64_t stride, uint32_t len, uint64_t n, BEpi epi,
                            hipStream_t st, unsigned grid, unsigned threads, int rows) {
    switch (rows) {
        case 1: launch_braid_rows<1>(grid, threads, st, base, stride, len, n, epi, s.tabs); break;
        case 2: launch_braid_rows<2>(grid, threads, st, base, stride, len, n, epi, s.tabs); break;
        case 3: launch_braid_rows<3>(grid, threads, st, base, stride, len, n, epi, s.tabs); break;
        case 4: launch_braid_rows<4>(grid, threads, st, base, stride, len, n, epi, s.tabs); break;
        case 5: launch_braid_rows<5>(grid, threads, st, base, stride, len, n, epi, s.tabs); break;
        case 6: launch_braid_rows<6>(grid, threads, st, base, stride, len, n, epi, s.tabs); break;
        default: return fail(WTP_EINVAL, "braid rows %d", rows);
    }
    return launch_check("k_fixed_braid");
}

template <class Prov, class Epi>
int launch_pieces(DevState &s, const uint8_t *base, uint64_t nbytes, Prov prov, uint64_t n, Epi epi,
                  hipStream_t st) {
    // Align the buffer view down to 16 B and round its size up: every 16-B block holding
    // a valid byte is then fully inside the resource (and inside one page).
    const uintptr_t ub = reinterpret_cast<uintptr_t>(base);
    const uint64_t lead = ub & 15u;
    const uint8_t *b16 = base - lead;
    const uint64_t span = (lead + nbytes + 15) & ~uint64_t(15);
    if (span >= (1ull << 31)) return fail(WTP_EINVAL, "general kernel span %llu B >= 2 GiB (split the batch)", (unsigned long long)span);
    const uint64_t waves_want = (n + 63) / 64;
    uint64_t grid = (waves_want + dev::kPcThreads / 64 - 1) / (dev::kPcThreads / 64);
    if (grid > uint64_t(s.grid_cus())) grid = uint64_t(s.grid_cus());
    if (grid == 0) grid = 1;
    note_kernel("k_pieces<%s, %s>", Prov::kName, Epi::kName);
    hipLaunchKernelGGL((dev::k_pieces<Prov, Epi>), dim3(unsigned(grid)), dim3(dev::kPcThreads), 0, st, b16, uint32_t(span),
                       prov, n, epi, s.tabs, s.status);
    return launch_check("k_pieces");
}

// Packed mixed lengths (k_stream): one launch for any n and any buffer size (64-bit
// offsets, per-round buffer resources); the kernel finds its own workgroup ranges.
int launch_stream(DevState &s, const uint8_t *base, uint64_t nbytes, const uint64_t *offs, const uint32_t *lens,
                  uint64_t n, uint32_t *out, hipStream_t st, const dev::RangeDesc *gate = nullptr, uint32_t ngate = 0) {
    const uint64_t lead = reinterpret_cast<uintptr_t>(base) & 15u;
    uint64_t grid = (n + dev::kStWaves * 64 - 1) / (dev::kStWaves * 64);  // >= 64 payloads per wave
    if (grid > uint64_t(s.grid_cus())) grid = uint64_t(s.grid_cus());
    if (grid == 0) grid = 1;
    note_kernel("k_stream");
    hipLaunchKernelGGL((dev::k_stream<0>), dim3(unsigned(grid)), dim3(dev::kStThreads), 0, st, base - lead,
                       lead + nbytes, offs, lens, lead, n, out, s.tabs, s.status, gate, ngate);
    return launch_check("k_stream");
}

}  // namespace

// Offsets handed to k_pieces must be relative to the 16-B aligned view.  The providers
// below add `lead` back.
namespace dev {
// Providers split metadata access in two: load() only issues loads (its results are
// consumed a round later, so no arithmetic may touch them there) and decode() turns the
// raw words into (offset in the view, length, valid, aux, output slot) when the round
// uses them.  count(n) is the number of packets (device-side for the fix-up pass).
struct FixedProvL {
    static constexpr const char *kName = "FixedProvL";  // wtp_last_kernel()
    static constexpr bool kVarLen = false;  // wave ranges balanced by pieces
    static constexpr bool kIndexed = false;
    static constexpr bool kGroupLoad = false;
    uint64_t stride, lead;
    uint32_t len;
    __device__ __forceinline__ void load(uint64_t p, MetaRaw &r, __amdgpu_buffer_rsrc_t) const { r.a = p; }
    __device__ __forceinline__ void decode(const MetaRaw &r, uint64_t &off, uint32_t &l, bool &ok, uint32_t &,
                                           uint32_t &) const {
        off = lead + r.a * stride;
        l = len;
        ok = true;
    }
};
struct ArrayProvL {
    static constexpr const char *kName = "ArrayProvL";  // wtp_last_kernel()
    static constexpr bool kVarLen = true;  // wave ranges balanced by pieces
    static constexpr bool kIndexed = false;
    static constexpr bool kGroupLoad = true;  // load_group: 32-bit buffer offsets, no clamp
    const uint64_t *__restrict__ offs;
    const uint32_t *__restrict__ lens;
    uint64_t lead;
    uint32_t n;  // packets of this launch (< 2^28: the arrays' byte extents fit 32 bits)
    __device__ __forceinline__ void load(uint64_t p, MetaRaw &r, __amdgpu_buffer_rsrc_t) const {
        r.a = reinterpret_cast<const uint32_t *>(offs)[2 * p];  // low dword: the view is < 2 GiB
        r.b = lens[p];
    }
    // packets q0 + lane: one VALU address per array; past n the loads return 0 (the range
    // check covers voffset, so the whole offset goes there, none in soffset)
    __device__ __forceinline__ void load_group(uint64_t q0, uint32_t lane, MetaRaw &r) const {
        const uint32_t pi = uint32_t(q0) + lane;
        r.a = __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(offs, n * 8u), int(pi * 8u), 0, 0);
        r.b = __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(lens, n * 4u), int(pi * 4u), 0, 0);
    }
    __device__ __forceinline__ uint32_t load_len(uint64_t p) const { return lens[p]; }
    __device__ __forceinline__ const uint32_t *len_array() const { return lens; }
    __device__ __forceinline__ uint32_t len_of(uint32_t w) const { return w; }
    __device__ __forceinline__ void decode(const MetaRaw &r, uint64_t &off, uint32_t &l, bool &ok, uint32_t &,
                                           uint32_t &) const {
        off = lead + r.a;
        l = r.b;
        ok = true;
    }
};
// Packed batches >= 2 GiB (launch_packed_ranges): ArrayProvL over one device-bound
// sub-range of the arrays (RangeDesc), 64-bit offsets rebased onto the sub-launch's
// < 2 GiB view.  A packet outside the view (offsets not packed) is flagged, not read.
struct RangeArrayProvL {
    static constexpr const char *kName = "RangeArrayProvL";  // wtp_last_kernel()
    static constexpr bool kVarLen = true;
    static constexpr bool kIndexed = false;
    static constexpr bool kGroupLoad = true;
    static constexpr bool kDevRange = true;
    const uint64_t *__restrict__ offs;  // the caller's arrays (bind() moves them to the range)
    const uint32_t *__restrict__ lens;
    RangeDesc *desc;
    uint64_t lead;        // the caller's base mod 16
    uint64_t rebase = 0;  // bind(): view offset of this launch's resource base
    uint32_t n = 0, vbytes = 0;
    template <class E>
    __device__ __forceinline__ bool bind(const uint8_t *&base, uint32_t &nbytes, uint64_t &nn, E &e) {
        const uint64_t b = desc->begin, en = desc->end;
        // only the cut-time flag: kRunBad may be set by another workgroup mid-launch, and
        // reading it here could let some waves of a block leave before a barrier
        if (b >= en || (desc->bad & kCutBad)) return false;
        rebase = desc->rebase;
        vbytes = desc->nbytes;
        offs += b;
        lens += b;
        n = uint32_t(en - b);  // <= kSubBatch
        base += rebase;
        nbytes = vbytes;
        nn = en - b;
        e.rebase(b, n);
        return true;
    }
    __device__ __forceinline__ void flag_outside() const { atomicOr(&desc->bad, kRunBad); }
    __device__ __forceinline__ void load(uint64_t p, MetaRaw &r, __amdgpu_buffer_rsrc_t) const {
        r.a = offs[p];
        r.b = lens[p];
    }
    __device__ __forceinline__ void load_group(uint64_t q0, uint32_t lane, MetaRaw &r) const {
        const uint32_t pi = uint32_t(q0) + lane;  // past n: 0
        const u32x2 w = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(make_rsrc(offs, n * 8u),
                                                                                        int(pi * 8u), 0, 0));
        r.a = uint64_t(w.x) | (uint64_t(w.y) << 32);
        r.b = __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(lens, n * 4u), int(pi * 4u), 0, 0);
    }
    __device__ __forceinline__ uint32_t load_len(uint64_t p) const { return lens[p]; }
    __device__ __forceinline__ const uint32_t *len_array() const { return lens; }
    __device__ __forceinline__ uint32_t len_of(uint32_t w) const { return w; }
    __device__ __forceinline__ void decode(const MetaRaw &r, uint64_t &off, uint32_t &l, bool &ok, uint32_t &,
                                           uint32_t &) const {
        const uint64_t o = r.a + lead - rebase;  // offset in this launch's view (mod 2^64)
        const bool in = o <= uint64_t(vbytes) && uint64_t(r.b) <= uint64_t(vbytes) - o;
        off = in ? o : 0u;
        l = in ? r.b : 0u;
        ok = in;
    }
};

// Sub-ranges of a packed batch for launch_packed_ranges: cuts where the view offset
// reaches k * G (binary search over the offsets; a prefix max keeps them monotone for
// any offsets) merged with the count cuts j * sb, so every range holds <= sb packets
// and, if packed, its bytes lie within G + 4 KiB < 2 GiB of its first offset.
constexpr uint32_t kMaxRanges = 1024;
__global__ __launch_bounds__(256) void k_cut_ranges(const uint64_t *__restrict__ offs, uint64_t n, uint64_t lead,
                                                    uint64_t vspan, uint64_t G, uint32_t kb, uint64_t sb,
                                                    RangeDesc *__restrict__ desc, uint32_t nd) {
    __shared__ uint64_t bcut[kMaxRanges];
    __shared__ uint64_t cuts[kMaxRanges + 1];
    for (uint32_t k = threadIdx.x + 1; k < kb; k += blockDim.x) {
        const uint64_t t = uint64_t(k) * G;
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t m = lo + (hi - lo) / 2;
            if (offs[m] + lead < t) lo = m + 1;
            else hi = m;
        }
        bcut[k] = lo;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t pb = 0, jc = sb;
        uint32_t k = 1, m = 1;
        cuts[0] = 0;
        while (m < nd) {
            const uint64_t b = k < kb ? (bcut[k] > pb ? bcut[k] : pb) : ~0ull;
            const uint64_t c = jc < n ? jc : ~0ull;
            if (b == ~0ull && c == ~0ull) {  // both lists used up (cannot happen for nd = kb + nc - 1): pad
                cuts[m++] = n;
                continue;
            }
            if (b <= c) {
                cuts[m++] = b;
                pb = b;
                ++k;
            } else {
                cuts[m++] = c;
                jc += sb;
            }
        }
        cuts[nd] = n;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nd; j += blockDim.x) {
        RangeDesc d{};
        d.begin = cuts[j];
        d.end = cuts[j + 1] > cuts[j] ? cuts[j + 1] : cuts[j];
        d.nbytes = 16;
        if (d.begin < d.end) {
            const uint64_t r = (offs[d.begin] + lead) & ~uint64_t(15);
            if (r < vspan) {
                d.rebase = r;
                d.nbytes = uint32_t(vspan - r < (1ull << 31) - 16 ? vspan - r : (1ull << 31) - 16);
            } else {
                d.bad = kCutBad;  // an offset past the buffer: not a packed batch
            }
        }
        desc[j] = d;
    }
}

// Datagram p = view[lead + p*stride, +recv_len[p]): header (16 B) + payload.  aux =
// ntohl(header.checksum): the two dwords covering header bytes 12..15 ride with the
// metadata prefetch (through the view's buffer resource: the second dword may lie past
// the last datagram, reads there return 0 and are never selected) and are
// funnel-shifted at decode.
struct DgramProvL {
    static constexpr const char *kName = "DgramProvL";  // wtp_last_kernel()
    static constexpr bool kVarLen = true;  // wave ranges balanced by pieces
    static constexpr bool kIndexed = false;
    static constexpr bool kGroupLoad = false;
    uint64_t stride, lead;
    const uint32_t *__restrict__ rl;
    __device__ __forceinline__ void load(uint64_t p, MetaRaw &r, __amdgpu_buffer_rsrc_t rs) const {
        const uint32_t h = uint32_t(lead + p * stride + 12) & ~3u;  // the view is < 2 GiB
        r.a = p;
        r.b = rl[p];
        const u32x2 w = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, int(h), 0, 0));
        r.c = w.x;
        r.d = w.y;
    }
    __device__ __forceinline__ uint32_t load_len(uint64_t p) const { return rl[p]; }
    __device__ __forceinline__ const uint32_t *len_array() const { return rl; }
    __device__ __forceinline__ uint32_t len_of(uint32_t r) const { return r >= 16 && r <= stride ? r - 16 : 0u; }
    __device__ __forceinline__ void decode(const MetaRaw &r, uint64_t &off, uint32_t &l, bool &ok, uint32_t &want,
                                           uint32_t &) const {
        const uint64_t d = lead + r.a * stride;
        want = bswap32(__builtin_amdgcn_alignbyte(r.d, r.c, uint32_t(d + 12) & 3u));
        off = d + 16;
        ok = r.b >= 16 && r.b <= stride;
        l = ok ? r.b - 16 : 0;
    }
};
}  // namespace dev

namespace {
// Packed mixed lengths in a buffer >= 2 GiB (wtp_crc32_batch_packed): the piece kernel in
// sub-launches over < 2 GiB views instead of k_stream (C5-like data: 43 vs 57 us per 1 M
// packets).  The host knows neither offsets nor lengths, so the cuts are
// made on the device (k_cut_ranges: view offsets at multiples of G, packet counts at
// multiples of kSubBatch) and each k_pieces sub-launch binds its range from its
// descriptor (RangeArrayProvL); the host launches an upper bound of kb + nc - 1 of them
// (empty ones return at once).  Exact for any offsets: a sub-launch that meets a packet
// outside its view flags its descriptor, and the gated k_stream launch at the end then
// recomputes the whole batch (it returns at once otherwise).  Asynchronous on `st`; the
// descriptors live in the stream's scratch (stream_scratch: calls on one stream are
// ordered, so they may share it).
int launch_packed_ranges(DevState &s, const uint8_t *b, uint64_t base_bytes, const uint64_t *offs,
                         const uint32_t *lens, uint64_t n, uint32_t *out, hipStream_t st) {
    const uint64_t lead = reinterpret_cast<uintptr_t>(b) & 15u;
    const uint8_t *view = b - lead;
    const uint64_t vspan = (lead + base_bytes + 15) & ~uint64_t(15);
    constexpr uint64_t G = (1ull << 31) - (1ull << 16);  // packed: a range spans <= G + 4111 B < 2 GiB - 16
    const uint64_t kb = (vspan + G - 1) / G, nc = (n + kSubBatch - 1) / kSubBatch;
    const uint64_t nd = kb + nc - 1;
    if (nd > dev::kMaxRanges) return launch_stream(s, b, base_bytes, offs, lens, n, out, st);
    static_assert(dev::kMaxRanges * sizeof(dev::RangeDesc) <= kStreamScratch, "descriptor scratch");
    dev::RangeDesc *d = nullptr;
    int rc = stream_scratch(s, st, reinterpret_cast<void **>(&d));
    if (rc) return rc;
    if (!d) return launch_stream(s, b, base_bytes, offs, lens, n, out, st);  // captured, no slot left
    hipLaunchKernelGGL(dev::k_cut_ranges, dim3(1), dim3(256), 0, st, offs, n, lead, vspan, G, uint32_t(kb),
                       uint64_t(kSubBatch), d, uint32_t(nd));
    rc = launch_check("k_cut_ranges");
    const uint64_t per = n < kSubBatch ? n : kSubBatch;  // packets of the largest range: the grid
    uint64_t grid = ((per + 63) / 64 + dev::kPcThreads / 64 - 1) / (dev::kPcThreads / 64);
    if (grid > uint64_t(s.grid_cus())) grid = uint64_t(s.grid_cus());
    for (uint64_t j = 0; j < nd && !rc; ++j) {
        hipLaunchKernelGGL((dev::k_pieces<dev::RangeArrayProvL, dev::CrcEpi>), dim3(unsigned(grid)),
                           dim3(dev::kPcThreads), 0, st, view, uint32_t(0),
                           dev::RangeArrayProvL{offs, lens, d + j, lead}, per, dev::CrcEpi{out, 0}, s.tabs, s.status);
        rc = launch_check("k_pieces");
    }
    if (!rc) rc = launch_stream(s, b, base_bytes, offs, lens, n, out, st, d, uint32_t(nd));
    note_kernel("k_pieces<RangeArrayProvL, CrcEpi> x %llu (+ k_stream if not packed)", (unsigned long long)nd);
    return rc;
}
}  // namespace

}  // namespace wtp

// ======================================================================================
// C ABI
// ======================================================================================
using namespace wtp;

extern "C" {

const char *wtp_version(void) { return "wtp-crc32-mi355x 0.1 (gfx950)"; }

const char *wtp_last_error(void) { return g_err.c_str(); }
const char *wtp_last_kernel(void) { return g_kernel.c_str(); }

int wtp_set_error_(int code, const char *msg) {
    g_err = msg ? msg : "";
    return code;
}

int wtp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int wtp_init(int device) { return init_device(device); }

int wtp_reserve_cus(int device, int ncus) {
    int rc = init_device(device);
    if (rc) return rc;
    DevState &s = g_dev[device];
    if (ncus < 0 || ncus >= s.cus) return fail(WTP_EINVAL, "ncus %d outside [0, %d)", ncus, s.cus);
    s.reserve.store(ncus, std::memory_order_relaxed);
    return WTP_OK;
}

int wtp_device_status(int device, uint32_t *flags, int clear) {
    if (!flags) return fail(WTP_EINVAL, "flags is null");
    int rc = init_device(device);
    if (rc) return rc;
    int prev = 0;
    WTP_HIP(hipGetDevice(&prev));
    WTP_HIP(hipSetDevice(device));
    auto body = [&]() -> int {
        WTP_HIP(hipDeviceSynchronize());
        WTP_HIP(hipMemcpy(flags, g_dev[device].status, 4, hipMemcpyDeviceToHost));
        if (clear) WTP_HIP(hipMemset(g_dev[device].status, 0, 4));
        return WTP_OK;
    };
    rc = body();
    (void)hipSetDevice(prev);  // restored on failure too
    return rc;
}

uint32_t wtp_crc32(const void *buf, size_t size) {
    return raw_update(0xFFFFFFFFu, static_cast<const uint8_t *>(buf), size) ^ 0xFFFFFFFFu;
}

int wtp_crc32_batch_fixed(const void *d_payloads, size_t stride, size_t len, size_t n, uint32_t *d_out,
                          void *stream) {
    if (n == 0) return WTP_OK;
    if (!d_out || (!d_payloads && len > 0)) return fail(WTP_EINVAL, "null pointer");
    if (len > kMaxVarLen) return fail(WTP_EINVAL, "len %zu > %u", len, kMaxVarLen);
    DevState *s = nullptr;
    int rc = current(s);
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint8_t *b = static_cast<const uint8_t *>(d_payloads);
    // braided fast path (stride <= 16 KiB: the range the parity tests cover)
    const bool fast = len >= 16 && len <= 1536 && len % 16 == 0 && stride % 16 == 0 && stride <= 16384 &&
                      reinterpret_cast<uintptr_t>(b) % 16 == 0;
    if (fast) return launch_fixed_braid(*s, b, stride, uint32_t(len), n, dev::CrcBEpi{d_out, 0}, st);
    // general kernel, in sub-batches whose byte span stays < 2 GiB
    const uint64_t per = std::min<uint64_t>(kSubBatch, stride ? std::max<uint64_t>(1, ((1ull << 30) - 4096) / stride) : n);
    for (uint64_t p = 0; p < n; p += per) {
        const uint64_t cnt = std::min<uint64_t>(per, n - p);
        const uint8_t *sb = b + p * stride;
        const uint64_t lead = reinterpret_cast<uintptr_t>(sb) & 15u;
        const uint64_t span = (cnt - 1) * stride + len;
        rc = launch_pieces(*s, sb, span, dev::FixedProvL{stride, lead, uint32_t(len)}, cnt,
                           dev::CrcEpi{d_out + p, uint32_t(cnt)}, st);
        if (rc) return rc;
    }
    return WTP_OK;
}

int wtp_crc32_batch_var(const void *d_base, size_t base_bytes, const uint64_t *d_offsets,
                        const uint32_t *d_lengths, size_t n, uint32_t *d_out, void *stream) {
    if (n == 0) return WTP_OK;
    if (!d_base || !d_offsets || !d_lengths || !d_out) return fail(WTP_EINVAL, "null pointer");
    DevState *s = nullptr;
    int rc = current(s);
    if (rc) return rc;
    const uint8_t *b = static_cast<const uint8_t *>(d_base);
    const uint64_t lead = reinterpret_cast<uintptr_t>(b) & 15u;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // The general kernel addresses a view of < 2 GiB (32-bit buffer offsets).  Larger
    // buffers take launch_packed_ranges: device-cut < 2 GiB sub-launches of the same
    // kernel when the offsets are packed (the common layout even through this entry),
    // else the gated stream kernel (64-bit offsets, exact for any layout) redoes the batch.
    if (((lead + base_bytes + 15) & ~uint64_t(15)) >= (1ull << 31))
        return launch_packed_ranges(*s, b, base_bytes, d_offsets, d_lengths, n, d_out, st);
    for (uint64_t p = 0; p < n; p += kSubBatch) {
        const uint64_t cnt = std::min<uint64_t>(kSubBatch, n - p);
        rc = launch_pieces(*s, b, base_bytes, dev::ArrayProvL{d_offsets + p, d_lengths + p, lead, uint32_t(cnt)}, cnt,
                           dev::CrcEpi{d_out + p, uint32_t(cnt)}, st);
        if (rc) break;
    }
    return rc;
}

int wtp_crc32_batch_packed(const void *d_base, size_t base_bytes, const uint64_t *d_offsets,
                           const uint32_t *d_lengths, size_t n, uint32_t *d_out, void *stream) {
    if (n == 0) return WTP_OK;
    if (!d_base || !d_offsets || !d_lengths || !d_out) return fail(WTP_EINVAL, "null pointer");
    // The piece-stream kernel is the faster one on every distribution measured (C5 Zipf
    // 1.1: 45.6 vs 57.0 us), so below 2 GiB a packed batch takes the same route as
    // wtp_crc32_batch_var, and from 2 GiB on it runs the same kernel in < 2 GiB
    // sub-launches cut on the device (launch_packed_ranges).  WTP_STREAM_KERNEL=1 in the
    // environment forces the stream kernel (tests, measurements).
    const char *force = getenv("WTP_STREAM_KERNEL");
    const bool stream_kernel = force && force[0] == '1';
    const uint64_t lead = reinterpret_cast<uintptr_t>(d_base) & 15u;
    const bool big = ((lead + base_bytes + 15) & ~uint64_t(15)) >= (1ull << 31);
    if (!stream_kernel && !big) return wtp_crc32_batch_var(d_base, base_bytes, d_offsets, d_lengths, n, d_out, stream);
    DevState *s = nullptr;
    int rc = current(s);
    if (rc) return rc;
    if (!stream_kernel)
        return launch_packed_ranges(*s, static_cast<const uint8_t *>(d_base), base_bytes, d_offsets, d_lengths, n,
                                    d_out, static_cast<hipStream_t>(stream));
    return launch_stream(*s, static_cast<const uint8_t *>(d_base), base_bytes, d_offsets, d_lengths, n, d_out,
                         static_cast<hipStream_t>(stream));
}

int wtp_crc32_verify_batch(const void *d_dgrams, size_t stride, const uint32_t *d_recv_len, size_t n,
                           uint8_t *d_ok, uint32_t *d_crc_out, void *stream) {
    if (n == 0) return WTP_OK;
    if (!d_dgrams || !d_recv_len || !d_ok) return fail(WTP_EINVAL, "null pointer");
    if (stride < 16) return fail(WTP_EINVAL, "stride %zu < 16", stride);
    DevState *s = nullptr;
    int rc = current(s);
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint8_t *b = static_cast<const uint8_t *>(d_dgrams);
    // Braided fast path for a 16-B aligned ring: one launch per sub-batch decides every
    // datagram of the ring's full WTP length 16 + min(stride - 16, 1456) (1472 B in
    // wReceiver's 1504-B slots or in a packed 1472-B ring); each workgroup then finishes
    // the rest of its own datagrams (short, empty, 1473-1500 B, malformed) in its fix-up
    // phase (verify_fixup).  No memory outside the caller's buffers, so captures, graph
    // replays and concurrent calls on any streams need nothing from the host.  The
    // sub-batches keep each launch's ring view below 2 GiB (32-bit buffer offsets).
    if (stride % 16 == 0 && stride >= 32 && stride <= 16384 && reinterpret_cast<uintptr_t>(b) % 16 == 0) {
        const uint32_t flen = uint32_t(std::min<size_t>(stride - 16, WTP_MAX_PAYLOAD));
        const uint64_t per = std::min<uint64_t>(kSubBatch, ((1ull << 31) - 4096) / stride);
        for (uint64_t p = 0; p < n && !rc; p += per) {
            const uint64_t cnt = std::min<uint64_t>(per, n - p);
            const uint8_t *sb = b + p * stride;
            rc = launch_fixed_braid(*s, sb + 16, stride, flen, cnt,
                                    dev::VerifyBEpi{d_recv_len + p, sb, stride, d_ok + p,
                                                    d_crc_out ? d_crc_out + p : nullptr, s->status, 0, cnt, 16u + flen},
                                    st);
        }
        return rc;
    }
    const uint64_t per = std::min<uint64_t>(kSubBatch, std::max<uint64_t>(1, (1ull << 30) / stride));
    for (uint64_t p = 0; p < n; p += per) {
        const uint64_t cnt = std::min<uint64_t>(per, n - p);
        const uint8_t *sb = b + p * stride;
        const uint64_t lead = reinterpret_cast<uintptr_t>(sb) & 15u;
        rc = launch_pieces(*s, sb, cnt * stride, dev::DgramProvL{stride, lead, d_recv_len + p}, cnt,
                           dev::VerifyEpi{d_ok + p, d_crc_out ? d_crc_out + p : nullptr, uint32_t(cnt)}, st);
        if (rc) return rc;
    }
    return WTP_OK;
}

int wtp_synth_fill(void *d_out, uint64_t start_byte, size_t nbytes, uint64_t seed, void *stream) {
    if (nbytes == 0) return WTP_OK;
    if (!d_out) return fail(WTP_EINVAL, "null pointer");
    const uint64_t words = (nbytes + 16) / 8;
    uint64_t blocks = (words + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(dev::k_synth, dim3(unsigned(blocks)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<uint8_t *>(d_out), start_byte, uint64_t(nbytes), seed);
    return launch_check("k_synth");
}

int wtp_build_data_packets(const void *d_payloads, size_t total_bytes, uint32_t seq0, void *d_wire,
                           size_t wire_stride, uint32_t *d_wire_len, void *stream) {
    if (total_bytes == 0) return WTP_OK;
    if (!d_payloads || !d_wire) return fail(WTP_EINVAL, "null pointer");
    if (wire_stride < 16 + WTP_MAX_PAYLOAD) return fail(WTP_EINVAL, "wire_stride %zu < 1472", wire_stride);
    DevState *s = nullptr;
    int rc = current(s);
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t nch = (total_bytes + WTP_MAX_PAYLOAD - 1) / WTP_MAX_PAYLOAD;
    const uint64_t full = total_bytes / WTP_MAX_PAYLOAD;
    const uint8_t *pay = static_cast<const uint8_t *>(d_payloads);
    uint8_t *wire = static_cast<uint8_t *>(d_wire);
    // Fused path: the braided kernel reads each full chunk once, copies it into its wire
    // slot and writes the header (16-B aligned buffers and slots).
    const bool fused = reinterpret_cast<uintptr_t>(pay) % 16 == 0 && reinterpret_cast<uintptr_t>(wire) % 16 == 0 &&
                       wire_stride % 16 == 0 && wire_stride <= 16384;
    const uint64_t first = fused ? full : 0;  // chunks [first, nch) take the three-step path
    if (fused && full &&
        (rc = launch_fixed_braid(*s, pay, WTP_MAX_PAYLOAD, WTP_MAX_PAYLOAD, full,
                                 dev::BuildBEpi{wire, wire_stride, seq0, WTP_MAX_PAYLOAD, d_wire_len, 0}, st)))
        return rc;
    const uint64_t nslow = nch - first;
    if (!nslow) return WTP_OK;
    // Three-step path (unaligned buffers, and the short last chunk): copy into the slots,
    // CRC over the slots, then the headers.  CRCs land in d_wire_len first (then become
    // the lengths), else in stream-ordered scratch.
    const uint8_t *spay = pay + first * WTP_MAX_PAYLOAD;
    uint8_t *swire = wire + first * wire_stride;
    const uint64_t stotal = total_bytes - first * WTP_MAX_PAYLOAD;
    uint32_t *crc = d_wire_len ? d_wire_len + first : nullptr;
    uint32_t *tmp = nullptr;
    if (!crc) {
        WTP_HIP(hipMallocFromPoolAsync(reinterpret_cast<void **>(&tmp), nslow * 4, s->pool, st));
        crc = tmp;
    }
    {
        const uint64_t work = nslow * (WTP_MAX_PAYLOAD / 4 + 1);
        uint64_t blocks = (work + 255) / 256;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(dev::k_wire_copy, dim3(unsigned(blocks)), dim3(256), 0, st, spay, stotal, swire,
                           uint64_t(wire_stride), nslow);
        rc = launch_check("k_wire_copy");
    }
    const uint64_t sfull = stotal / WTP_MAX_PAYLOAD;
    const uint64_t tail = stotal - sfull * WTP_MAX_PAYLOAD;
    if (!rc && sfull) rc = wtp_crc32_batch_fixed(swire + 16, wire_stride, WTP_MAX_PAYLOAD, sfull, crc, stream);
    if (!rc && tail) rc = wtp_crc32_batch_fixed(swire + sfull * wire_stride + 16, 0, tail, 1, crc + sfull, stream);
    if (!rc) {
        uint64_t blocks = (nslow + 255) / 256;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(dev::k_wire_header, dim3(unsigned(blocks)), dim3(256), 0, st, crc, stotal,
                           seq0 + uint32_t(first), swire, uint64_t(wire_stride), crc == tmp ? nullptr : crc, nslow);
        rc = launch_check("k_wire_header");
    }
    if (tmp) {
        const hipError_t fe = hipFreeAsync(tmp, st);
        if (!rc && fe != hipSuccess) rc = fail(WTP_EHIP, "hipFreeAsync: %s", hipGetErrorString(fe));
    }
    if (rc) return rc;
    return WTP_OK;
}

}  // extern "C"
