// kbench.hip — standalone kernel ablation harness (diagnostics only, not the product).
// Builds against the product kernel source and times, in one process with interleaved
// rounds (guide §5.4 rule 24):
//   read_probe   : the HBM read ceiling of this access shape (dwordx4 nt loads + XOR)
//   braid_prod   : the production k_fixed_braid<6>
//   braid_nolut  : same loads/loop, table lookups replaced by XOR/shift (DIAG 1)
//   braid_nofold : production lookups, the in-lane x^-32 fold removed (DIAG 2)
//   braid_skel   : both (DIAG 3): the loop skeleton's loads, flush and stores
//   *_probe      : load-only access shapes (no compute)
// KB_ONLY=a,b,c selects variants, KB_SUSTAIN=... times them back to back (KB_NS launches,
// KB_REPS interleaved rounds).  Variants named var* are checked bit-exact against
// braid_prod.  Output: one line per variant with median/min time and GB/s on 1M x 1456 B.
#include "../a3-reliable-transport_amd/csrc/crc32_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>
#include <functional>
#include <cstring>
#include <unistd.h>
#include <string>

using namespace wtp;
using namespace wtp::dev;

__global__ __launch_bounds__(1024) void k_read_probe(const u32x4 *__restrict__ p, uint64_t n16, uint32_t *out) {
    uint32_t acc = 0;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
        u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Same load pattern as the braid (16 lanes x 16 B per packet row, 4 packets/wave),
// no compute: isolates the access-pattern cost.  NT: nontemporal loads.
template <int ROWS, bool NT, int DEPTH>
__global__ __launch_bounds__(1024) void k_strided_probe(const uint8_t *__restrict__ base, uint64_t stride, uint32_t len,
                                                        uint64_t n, uint32_t *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
    const uint32_t j = lane & 15u, q = lane >> 4;
    constexpr uint32_t kFrame = 256u * ROWS;
    const uint32_t zc = (kFrame - len) >> 4;
    const uint64_t rounds = (n + 3) >> 2;
    const uint64_t rstep = uint64_t(gridDim.x) * nwave;
    uint32_t acc = 0;
    for (uint64_t r = uint64_t(blockIdx.x) * nwave + wave; r < rounds; r += rstep * DEPTH) {
        u32x4 w[DEPTH][ROWS];
#pragma unroll
        for (int dd = 0; dd < DEPTH; ++dd) {
            uint64_t p = (r + dd * rstep) * 4 + q;
            p = p < n ? p : n - 1;
            const uint8_t *fs = base + p * stride + len - kFrame;
#pragma unroll
            for (int i = 0; i < ROWS; ++i) {
                const uint32_t c = uint32_t(i) * 16u + j;
                if (c >= zc) w[dd][i] = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(fs + c * 16u))
                                           : *reinterpret_cast<const u32x4 *>(fs + c * 16u);
                else w[dd][i] = u32x4{0, 0, 0, 0};
            }
        }
#pragma unroll
        for (int dd = 0; dd < DEPTH; ++dd)
#pragma unroll
            for (int i = 0; i < ROWS; ++i) acc ^= w[dd][i].x ^ w[dd][i].y ^ w[dd][i].z ^ w[dd][i].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// One packet per wave: 64 lanes x 16 B = 1 KiB contiguous rows (G = 64 layout), no compute.
template <int DEPTH>
__global__ __launch_bounds__(1024) void k_g64_probe(const uint8_t *__restrict__ base, uint64_t n, uint32_t *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
    const uint64_t rstep = uint64_t(gridDim.x) * nwave;
    uint32_t acc = 0;
    for (uint64_t p = uint64_t(blockIdx.x) * nwave + wave; p < n; p += rstep * DEPTH) {
        u32x4 w[DEPTH][2];
#pragma unroll
        for (int dd = 0; dd < DEPTH; ++dd) {
            uint64_t pp = p + dd * rstep;
            pp = pp < n ? pp : n - 1;
            const uint8_t *fs = base + pp * 1456 + 1456 - 2048;
            w[dd][0] = lane >= 37 ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(fs + lane * 16u)) : u32x4{0,0,0,0};
            w[dd][1] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(fs + 1024 + lane * 16u));
        }
#pragma unroll
        for (int dd = 0; dd < DEPTH; ++dd) acc ^= w[dd][0].x ^ w[dd][0].y ^ w[dd][0].z ^ w[dd][0].w ^ w[dd][1].x ^ w[dd][1].y ^ w[dd][1].z ^ w[dd][1].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Generic braid-shaped load probe: G lanes x 16 B per packet row, 64/G packets per wave,
// ROWS rows, DEPTH rounds in flight.  AL=0: frame right-aligned to the packet end (as the
// production kernel); AL=1: frame start 128-B aligned when it fits, else 64-B aligned.
template <int G, int ROWS, int AL, int DEPTH>
__global__ __launch_bounds__(1024) void k_gprobe(const uint8_t *__restrict__ base, uint64_t n, uint32_t *__restrict__ out) {
    constexpr int PW = 64 / G;
    constexpr uint32_t RB = 16u * G, kFrame = RB * ROWS;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
    const uint32_t j = lane % G, q = lane / G;
    const uint64_t rounds = (n + PW - 1) / PW;
    const uint64_t rstep = uint64_t(gridDim.x) * nwave;
    uint32_t acc = 0;
    for (uint64_t r = uint64_t(blockIdx.x) * nwave + wave; r < rounds; r += rstep * DEPTH) {
        u32x4 w[DEPTH][ROWS];
#pragma unroll
        for (int dd = 0; dd < DEPTH; ++dd) {
            uint64_t p = (r + dd * rstep) * PW + q;
            p = p < n ? p : n - 1;
            const uint64_t st = p * 1456, en = st + 1456;
            uint64_t fs = en - kFrame;
            if (AL) {
                const uint64_t a128 = st & ~uint64_t(127), a64 = st & ~uint64_t(63);
                fs = (a128 + kFrame >= en) ? a128 : a64;
            }
#pragma unroll
            for (int i = 0; i < ROWS; ++i) {
                const uint64_t o = fs + uint64_t(i) * RB + j * 16u;
                if (o >= st && o < en) w[dd][i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base + o));
                else w[dd][i] = u32x4{0, 0, 0, 0};
            }
        }
#pragma unroll
        for (int dd = 0; dd < DEPTH; ++dd)
#pragma unroll
            for (int i = 0; i < ROWS; ++i) acc ^= w[dd][i].x ^ w[dd][i].y ^ w[dd][i].z ^ w[dd][i].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Segment layout probe: 16 lanes per packet, lane j owns the contiguous 96-B segment
// [frame + 96 j, +96) of a right-aligned 1536-B frame; row i loads 16 B at +16 i.
template <int DEPTH>
__global__ __launch_bounds__(1024) void k_seg_probe(const uint8_t *__restrict__ base, uint64_t n, uint32_t *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
    const uint32_t j = lane & 15u, q = lane >> 4;
    const uint64_t rounds = (n + 3) >> 2;
    const uint64_t rstep = uint64_t(gridDim.x) * nwave;
    uint32_t acc = 0;
    for (uint64_t r = uint64_t(blockIdx.x) * nwave + wave; r < rounds; r += rstep * DEPTH) {
        u32x4 w[DEPTH][6];
#pragma unroll
        for (int dd = 0; dd < DEPTH; ++dd) {
            uint64_t p = (r + dd * rstep) * 4 + q;
            p = p < n ? p : n - 1;
            const uint8_t *fs = base + p * 1456 + 1456 - 1536;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const uint32_t o = j * 96u + i * 16u;
                w[dd][i] = o >= 80u ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(fs + o)) : u32x4{0, 0, 0, 0};
            }
        }
#pragma unroll
        for (int dd = 0; dd < DEPTH; ++dd)
#pragma unroll
            for (int i = 0; i < 6; ++i) acc ^= w[dd][i].x ^ w[dd][i].y ^ w[dd][i].z ^ w[dd][i].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Stage-through-LDS probes: a wave's 4 packets (5824 contiguous bytes) are read as six
// contiguous 1 KiB pieces, written to a per-wave 6 KiB LDS slot, and read back in the braid
// layout (lane (q, j), row i <- packet q chunk 16 i + j, right-aligned 1536-B frame).
// DMA = 0: global_load_dwordx4 + ds_write_b128; DMA = 1: global_load_lds_dwordx4.
template <int DMA>
__global__ __launch_bounds__(1024) void k_stage_probe(const uint8_t *__restrict__ base, uint64_t n, uint32_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[16 * 6144];
    const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nwave = blockDim.x >> 6;
    const uint32_t j = lane & 15u, q = lane >> 4;
    uint8_t *slot = stage + wave * 6144;
    const uint64_t rounds = (n + 3) >> 2;
    const uint64_t rstep = uint64_t(gridDim.x) * nwave;
    const uint64_t total = n * 1456;
    gu8 *gb = (gu8 *)base;
    uint32_t acc = 0;
    for (uint64_t r = uint64_t(blockIdx.x) * nwave + wave; r < rounds; r += rstep) {
        const uint64_t r0 = r * 4 * 1456;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            uint64_t o = r0 + uint64_t(i) * 1024 + lane * 16;
            o = o + 16 <= total ? o : 0;
            if (DMA) {
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(gb + o),
                                                 (__attribute__((address_space(3))) void *)(slot + i * 1024), 16, 0, 0);
            } else {
                const u32x4 v = __builtin_nontemporal_load((gu32x4 *)(gb + o));
                *reinterpret_cast<u32x4 *>(slot + i * 1024 + lane * 16) = v;
            }
        }
        if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int32_t o = int32_t(q * 1456u) - 80 + i * 256 + int32_t(j * 16u);
            if (o >= int32_t(q * 1456u)) {
                const u32x4 v = *reinterpret_cast<const u32x4 *>(slot + o);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (acc == 0x12345678u) out[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 20);
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const uint64_t bytes = n * 1456;
    CK(hipSetDevice(0));
    if (wtp_init(0)) { fprintf(stderr, "init: %s\n", wtp_last_error()); return 1; }
    DevState &s = g_dev[0];
    // KB_ALT=1: two n-packet buffers, every launch reads the other one (no launch re-reads
    // what the previous launch read: the streaming case)
    const bool alt = getenv("KB_ALT") && atoi(getenv("KB_ALT"));
    uint8_t *base0, *buf; uint32_t *out;
    CK(hipMalloc(&base0, (alt ? 2 : 1) * bytes + 64));
    CK(hipMalloc(&out, n * 4 + 64));
    if (wtp_synth_fill(base0, 0, (alt ? 2 : 1) * bytes, 0x5EED, nullptr)) return 1;
    buf = base0;
    auto flip = [&] { if (alt) buf = buf == base0 ? base0 + bytes : base0; };
    CK(hipDeviceSynchronize());
    const uint32_t cinit = init_const(1456);
    const uint64_t rounds = (n + 3) / 4;
    const unsigned grid = unsigned(std::min<uint64_t>((rounds + 15) / 16, s.cus));

    struct V { const char *name; std::function<void()> f; std::vector<float> t; };
    std::vector<V> vs;
    vs.push_back({"read_probe_g256x1024", [&] { hipLaunchKernelGGL(k_read_probe, dim3(s.cus), dim3(1024), 0, 0, (const u32x4 *)buf, bytes / 16, out); }, {}});
    vs.push_back({"read_probe_g2048x256", [&] { hipLaunchKernelGGL(k_read_probe, dim3(2048), dim3(256), 0, 0, (const u32x4 *)buf, bytes / 16, out); }, {}});
    vs.push_back({"read_probe_g8192x256", [&] { hipLaunchKernelGGL(k_read_probe, dim3(8192), dim3(256), 0, 0, (const u32x4 *)buf, bytes / 16, out); }, {}});
    vs.push_back({"braid_prod", [&] { hipLaunchKernelGGL(k_fixed_braid<6>, dim3(grid), dim3(1024), 0, 0, buf, 1456u, 1456u, n, CrcBEpi{out, cinit}, s.tabs); }, {}});
#define BD(NAME, DIAG) vs.push_back({NAME, [&] { hipLaunchKernelGGL((k_fixed_braid<6, DIAG>), dim3(grid), dim3(1024), 0, 0, buf, 1456u, 1456u, n, CrcBEpi{out, cinit}, s.tabs); }, {}})
    BD("braid_nolut", 1); BD("braid_nofold", 2); BD("braid_skel", 3);
    // the product's workgroup size (512 threads, 8 waves per CU) and its ablations
    const unsigned grid512 = unsigned(std::min<uint64_t>((rounds + 7) / 8, s.cus));
#define BD5(NAME, DIAG) vs.push_back({NAME, [&] { hipLaunchKernelGGL((k_fixed_braid<6, DIAG>), dim3(grid512), dim3(512), 0, 0, buf, 1456u, 1456u, n, CrcBEpi{out, cinit}, s.tabs); }, {}})
    BD5("braid512_noprio", 4); BD5("braid512_prod", 0); BD5("braid512_nolut", 1); BD5("braid512_nofold", 2); BD5("braid512_skel", 3);
    // access-pattern ablations of the skeleton: no result stores (16), row 0
    // nt (32), right-aligned frames (64)
    BD5("braid512_skel_nost", 3 | 16); BD5("braid512_skel_nt0", 3 | 32); BD5("braid512_skel_ra", 3 | 64);
    BD5("braid512_skel_noprio", 3 | 4); BD5("braid512_skel_all", 3 | 16 | 32 | 64); BD5("varbraid512_ra", 64);
    BD5("braid512_nost", 16);  BD5("varbraid512_direct", 2048); BD5("braid512_skel_hold", 3 | 1024);
    vs.push_back({"varbraid512_hold", [&] { CrcHoldBEpi h; static_cast<CrcBEpi &>(h) = CrcBEpi{out, cinit};
        hipLaunchKernelGGL((k_fixed_braid<6, 0, CrcHoldBEpi>), dim3(grid512), dim3(512), 0, 0, buf, 1456u, 1456u, n, h, s.tabs); }, {}});
    vs.push_back({"read_probe_g256x512", [&] { hipLaunchKernelGGL(k_read_probe, dim3(s.cus), dim3(512), 0, 0, (const u32x4 *)buf, bytes / 16, out); }, {}});
    vs.push_back({"strided_nt_d1", [&] { hipLaunchKernelGGL((k_strided_probe<6, true, 1>), dim3(grid), dim3(1024), 0, 0, buf, 1456ull, 1456u, n, out); }, {}});
    vs.push_back({"strided_nt_d2", [&] { hipLaunchKernelGGL((k_strided_probe<6, true, 2>), dim3(grid), dim3(1024), 0, 0, buf, 1456ull, 1456u, n, out); }, {}});
    vs.push_back({"strided_plain_d2", [&] { hipLaunchKernelGGL((k_strided_probe<6, false, 2>), dim3(grid), dim3(1024), 0, 0, buf, 1456ull, 1456u, n, out); }, {}});
    vs.push_back({"strided_nt_d2_g256x512", [&] { hipLaunchKernelGGL((k_strided_probe<6, true, 2>), dim3(s.cus), dim3(512), 0, 0, buf, 1456ull, 1456u, n, out); }, {}});
    vs.push_back({"strided_nt_d2_g512", [&] { hipLaunchKernelGGL((k_strided_probe<6, true, 2>), dim3(512), dim3(512), 0, 0, buf, 1456ull, 1456u, n, out); }, {}});
    vs.push_back({"g64_d2", [&] { hipLaunchKernelGGL((k_g64_probe<2>), dim3(s.cus), dim3(1024), 0, 0, buf, n, out); }, {}});
    vs.push_back({"g64_d4", [&] { hipLaunchKernelGGL((k_g64_probe<4>), dim3(s.cus), dim3(1024), 0, 0, buf, n, out); }, {}});
    vs.push_back({"g64_d4_g1024x256", [&] { hipLaunchKernelGGL((k_g64_probe<4>), dim3(1024), dim3(256), 0, 0, buf, n, out); }, {}});
#define GP(G, R, AL, D, GR, BL) vs.push_back({"gprobe_G" #G "_R" #R "_al" #AL "_d" #D "_" #GR "x" #BL, [&] { hipLaunchKernelGGL((k_gprobe<G, R, AL, D>), dim3(GR), dim3(BL), 0, 0, buf, n, out); }, {}})
    GP(16, 6, 0, 1, 256, 1024); GP(16, 6, 1, 1, 256, 1024); GP(16, 6, 0, 2, 256, 1024); GP(16, 6, 1, 2, 256, 1024);
    GP(8, 12, 0, 1, 256, 1024); GP(8, 12, 1, 1, 256, 1024); GP(8, 12, 1, 2, 256, 1024);
    GP(32, 3, 0, 2, 256, 1024); GP(32, 3, 1, 2, 256, 1024); GP(32, 3, 1, 4, 256, 1024);
    GP(16, 6, 1, 2, 512, 512); GP(8, 12, 1, 1, 512, 512);
    vs.push_back({"stage_probe_reg", [&] { hipLaunchKernelGGL((k_stage_probe<0>), dim3(s.cus), dim3(1024), 0, 0, buf, n, out); }, {}});
    vs.push_back({"stage_probe_dma", [&] { hipLaunchKernelGGL((k_stage_probe<1>), dim3(s.cus), dim3(1024), 0, 0, buf, n, out); }, {}});
    vs.push_back({"seg_probe_d1", [&] { hipLaunchKernelGGL((k_seg_probe<1>), dim3(s.cus), dim3(1024), 0, 0, buf, n, out); }, {}});
    vs.push_back({"seg_probe_d2", [&] { hipLaunchKernelGGL((k_seg_probe<2>), dim3(s.cus), dim3(1024), 0, 0, buf, n, out); }, {}});
    vs.push_back({"pieces_fixed", [&] {  // general kernel, fixed provider
        launch_pieces(s, buf, bytes, dev::FixedProvL{1456, 0, 1456u}, n, dev::CrcEpi{out, uint32_t(n)}, nullptr); }, {}});

    if (const char *only = getenv("KB_ONLY")) {  // comma-separated exact names; braid_prod always kept first
        std::vector<V> keep;
        std::string o = std::string(",") + only + ",";
        for (auto &v : vs)
            if (!strcmp(v.name, "braid_prod") || o.find(std::string(",") + v.name + ",") != std::string::npos) keep.push_back(v);
        vs.swap(keep);
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (auto &v : vs) { flip(); v.f(); flip(); v.f(); }
    CK(hipDeviceSynchronize());
    for (int r = 0; r < reps; ++r)
        for (auto &v : vs) {
            flip();
            CK(hipEventRecord(a, 0));
            v.f();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            v.t.push_back(ms);
        }
    // sustained: 200 back-to-back launches per selected variant (DVFS steady state)
    if (getenv("KB_SUSTAIN")) {
        // KB_REPS rounds over the selected variants (interleaved A B C A B C ...), NS
        // back-to-back launches each; the summary averages the per-round steady medians.
        const int NS = getenv("KB_NS") ? atoi(getenv("KB_NS")) : 200;
        const int RR = getenv("KB_REPS") ? atoi(getenv("KB_REPS")) : 1;
        std::vector<hipEvent_t> ev(NS + 1);
        for (size_t k = 0; k < ev.size(); ++k) CK(hipEventCreate(&ev[k]));
        std::vector<std::vector<float>> med(vs.size());
        for (int rep = 0; rep < RR; ++rep)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            auto &v = vs[vi];
            if (!strstr(getenv("KB_SUSTAIN"), v.name) && strcmp(getenv("KB_SUSTAIN"), "all")) continue;
            CK(hipDeviceSynchronize());
            usleep(200000);  // let clocks settle between variants
            CK(hipEventRecord(ev[0], 0));
            for (int r = 0; r < NS; ++r) { flip(); v.f(); CK(hipEventRecord(ev[r + 1], 0)); }
            CK(hipDeviceSynchronize());
            std::vector<float> t;
            for (int r = 0; r < NS; ++r) { float ms; CK(hipEventElapsedTime(&ms, ev[r], ev[r + 1])); t.push_back(ms); }
            std::vector<float> tail(t.begin() + NS / 2, t.end());
            std::sort(tail.begin(), tail.end());
            med[vi].push_back(tail[tail.size() / 2]);
            float tot; CK(hipEventElapsedTime(&tot, ev[0], ev[NS]));
            printf("SUSTAIN %-26s all %.1f GB/s | steady median %.4f ms %.1f GB/s | t[0..]=", v.name, bytes * NS / (tot * 1e-3) / 1e9,
                   tail[tail.size() / 2], bytes / (tail[tail.size() / 2] * 1e-3) / 1e9);
            for (int r = 0; r < NS; r += 20) printf("%.0f ", t[r] * 1000);
            printf("us\n");
        }
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            if (med[vi].empty()) continue;
            double m = 0; for (float x : med[vi]) m += x; m /= med[vi].size();
            printf("SUMMARY %-26s steady %.4f ms %.1f GB/s (%.1f%% of 8 TB/s) over %zu rounds\n", vs[vi].name, m, bytes / (m * 1e-3) / 1e9,
                   100.0 * bytes / (m * 1e-3) / 8e12, med[vi].size());
        }
    }
    // back-to-back launches of the production kernel (as bench.py issues them)
    {
        size_t bp = 0;
        for (size_t k = 0; k < vs.size(); ++k) if (!strcmp(vs[k].name, "braid_prod")) bp = k;
        std::vector<hipEvent_t> ev(2 * reps);
        for (size_t k = 0; k < ev.size(); ++k) CK(hipEventCreate(&ev[k]));
        for (int r = 0; r < reps; ++r) {
            flip();
            CK(hipEventRecord(ev[2 * r], 0));
            vs[bp].f();
            CK(hipEventRecord(ev[2 * r + 1], 0));
        }
        CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int r = 0; r < reps; ++r) { float ms; CK(hipEventElapsedTime(&ms, ev[2 * r], ev[2 * r + 1])); t.push_back(ms); }
        std::sort(t.begin(), t.end());
        printf("braid_prod back-to-back: median %.4f ms (%.1f GB/s) min %.4f max %.4f\n", t[t.size() / 2],
               bytes / (t[t.size() / 2] * 1e-3) / 1e9, t[0], t.back());
    }
    {  // correctness of the var* variants against braid_prod (same outputs, bit-exact)
        buf = base0;
        std::vector<uint32_t> ref(n), got(n);
        size_t bp = 0;
        for (size_t k = 0; k < vs.size(); ++k) if (!strcmp(vs[k].name, "braid_prod")) bp = k;
        CK(hipMemset(out, 0, n * 4)); vs[bp].f(); CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), out, n * 4, hipMemcpyDeviceToHost));
        for (auto &v : vs) {
            if (strncmp(v.name, "var", 3)) continue;
            CK(hipMemset(out, 0, n * 4)); v.f(); CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
            uint64_t bad = 0;
            for (uint64_t i = 0; i < n; ++i) bad += ref[i] != got[i];
            printf("CHECK %-20s %s (%llu mismatches)\n", v.name, bad ? "MISMATCH" : "ok", (unsigned long long)bad);
        }
    }
    printf("# n=%llu packets x 1456 B = %.3f GB per launch, grid(braid)=%u, reps=%d, %s\n", (unsigned long long)n, bytes / 1e9, grid, reps,
           alt ? "alternating buffers (KB_ALT)" : "one buffer");
    for (auto &v : vs) {
        std::sort(v.t.begin(), v.t.end());
        const float med = v.t[v.t.size() / 2], mn = v.t[0];
        printf("%-24s median %.4f ms (%.1f GB/s, %.1f%% of 8 TB/s)  min %.4f ms (%.1f GB/s)\n", v.name, med,
               bytes / (med * 1e-3) / 1e9, 100.0 * bytes / (med * 1e-3) / 8e12, mn, bytes / (mn * 1e-3) / 1e9);
    }
    return 0;
}
