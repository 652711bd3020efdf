// Legacy LDS layout kept for the ablation harness only (tools/kbench.hip): the first
// braided kernel's 32-copy replicated tables (128 KiB per 4-table set).  The product
// kernels use the staggered 8-copy layout (StagKeys in crc32_kernels.hip).
#pragma once
namespace wtp {
// Replicated word tables: byte address t_hi*65536 + e*256 + t_lo*128 + (lane&31)*4 for
// table t = 2*t_hi + t_lo, so a ds_read_b32 by lane L always lands in bank L%32.
constexpr uint32_t kRepBytes = 131072;
constexpr uint32_t kLdsWords = (kRepBytes + 6 * kOpBytes) / 4;  // 155,648 B
namespace dev {
// Copy four 256-entry word tables from global into the replicated LDS image.
__device__ __forceinline__ void fill_replicated(char *lds, const uint32_t *__restrict__ g) {
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) {
        const uint32_t t = i >> 8, e = i & 255u;
        const uint32_t v = g[i];
        u32x4 *dst = reinterpret_cast<u32x4 *>(lds + (t >> 1) * 65536u + e * 256u + (t & 1u) * 128u);
        const u32x4 q = {v, v, v, v};
#pragma unroll
        for (int c = 0; c < 8; ++c) dst[c] = q;
    }
}

__device__ __forceinline__ void fill_ops(char *lds, const uint32_t *__restrict__ g, int nops) {
    u32x4 *dst = reinterpret_cast<u32x4 *>(lds + kRepBytes);
    const u32x4 *src = reinterpret_cast<const u32x4 *>(g);
    for (int i = threadIdx.x; i < nops * 256; i += blockDim.x) dst[i] = src[i];
}

// Per-lane address constants for the replicated tables: byte0 = t_lo<<7 | (lane&31)<<2,
// byte2 = t_hi.  v_perm_b32(x, K_t, sel_t) = K_t.b0 | x.b_t << 8 | K_t.b2 << 16.
struct RepKeys {
    uint32_t k[4];
    __device__ __forceinline__ explicit RepKeys(uint32_t lane) {
        const uint32_t c4 = (lane & 31u) << 2;
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) k[t] = ((t & 1u) << 7) | c4 | ((t >> 1) << 16);
    }
};

// XOR_t table_t[byte_t(x)] through the replicated image (4 v_perm + 4 ds_read_b32).
__device__ __forceinline__ uint32_t rep_word(const char *lds, const RepKeys &K, uint32_t x) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, K.k[0], 0x0C020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(x, K.k[1], 0x0C020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(x, K.k[2], 0x0C020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(x, K.k[3], 0x0C020700u);
    return (lds_rd(lds, a0) ^ lds_rd(lds, a1)) ^ (lds_rd(lds, a2) ^ lds_rd(lds, a3));
}

// Table 3 of the slice-by-4 set is the plain Sarwate table: one byte step.
__device__ __forceinline__ uint32_t rep_byte(const char *lds, const RepKeys &K, uint32_t c, uint32_t b) {
    const uint32_t a = __builtin_amdgcn_perm((c ^ b), K.k[3], 0x0C020400u);
    return lds_rd(lds, a) ^ (c >> 8);
}

}  // namespace dev
}  // namespace wtp
