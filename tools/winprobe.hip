// Window-load probe for a piece kernel without LDS staging (diagnostic, not the product):
// each lane reads its own 64-B window as four 16-B loads at a byte offset, the windows of
// a wave's 64 lanes lying back to back (lane stride 64 B) with a per-lane jitter of
// 0..63 B, 4 KiB per wave round, streamed over 1.5 GB; XOR-reduced.  Variants: aligned
// (jitter 0), dword-aligned jitter, byte jitter; and the staged reference: lane-contiguous
// 1 KiB loads (what k_pieces' span load does).  Prints GB/s of window bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 0 lane-contiguous 1 KiB per instruction, 1 windows aligned, 2 dword jitter, 3 byte jitter
__global__ __launch_bounds__(1024) void k_win(const uint8_t *base, uint64_t nbytes, uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
    const uint64_t nblk = (nbytes - 8192) / 4096;
    u32x4 acc = {0, 0, 0, 0};
    uint32_t h = lane * 2654435761u;
    for (uint64_t b = wave; b < nblk; b += nwaves) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base + b * 4096), (short)0, 8192, 0x00020000);
        h = h * 1664525u + 1013904223u;
        uint32_t o;
        if (MODE == 0) o = lane * 16u;
        else if (MODE == 1) o = lane * 64u;
        else if (MODE == 2) o = lane * 64u + ((h >> 24) & 60u);
        else o = lane * 64u + ((h >> 24) & 63u);
        const uint32_t st = MODE == 0 ? 1024u : 16u;
        const u32x4 v0 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(o), 0, 0));
        const u32x4 v1 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(o + st), 0, 0));
        const u32x4 v2 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(o + 2 * st), 0, 0));
        const u32x4 v3 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(o + 3 * st), 0, 0));
        acc ^= v0 ^ v1 ^ v2 ^ v3;
    }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int MODE>
static int run(const char *name, const uint8_t *d, uint64_t n, uint32_t *sink) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_win<MODE>, dim3(256), dim3(1024), 0, 0, d, n, sink);
    CK(hipEventRecord(a));
    for (int i = 0; i < 30; ++i) hipLaunchKernelGGL(k_win<MODE>, dim3(256), dim3(1024), 0, 0, d, n, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double bytes = double((n - 8192) / 4096) * 4096.0;
    printf("{\"mode\": \"%s\", \"us\": %.1f, \"GBps\": %.1f}\n", name, ms / 30 * 1e3, bytes / (ms / 30 * 1e-3) / 1e9);
    return 0;
}

int main() {
    const uint64_t n = 1536ull << 20;
    uint8_t *d;
    uint32_t *sink;
    CK(hipMalloc(&d, n + 8192));
    CK(hipMemset(d, 0x3c, n + 8192));
    CK(hipMalloc(&sink, 256 * 1024 * 4));
    for (int rep = 0; rep < 2; ++rep) {
        if (run<0>("lane_contiguous_1KiB", d, n, sink)) return 1;
        if (run<1>("windows_aligned", d, n, sink)) return 1;
        if (run<2>("windows_dword_jitter", d, n, sink)) return 1;
        if (run<3>("windows_byte_jitter", d, n, sink)) return 1;
    }
    return 0;
}
