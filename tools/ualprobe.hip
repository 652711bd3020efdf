// Unaligned 16-B buffer loads: do byte-misaligned buffer_load_dwordx4 stream at the
// aligned rate?  (Diagnostic for a braided mixed-length kernel whose frames end at
// byte-aligned packet ends.)  Reads 1.5 GB as lanes of 16 B at byte offset `mis`
// (0..15) from a 16-B aligned base, nt, 1 KiB per wave instruction, 4 in flight,
// XOR-reduced; prints GB/s per misalignment.  Also checks the loaded bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_rd(const uint8_t *base, uint64_t nbytes, uint32_t mis, uint32_t *sink) {
    const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), (short)0, 0x7FFFFFFF, 0x00020000);
    const uint64_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
    const uint64_t nblk = (nbytes - 64) / 4096;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t b = wave; b < nblk; b += nwaves) {
        const uint64_t o = b * 4096;
        // 1.5 GB does not fit 31-bit offsets: a resource per block start
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base + o), (short)0, 8192, 0x00020000);
        (void)rs0;
        const uint32_t l = uint32_t(lane) * 16u + mis;
        const u32x4 v0 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(l), 0, 2));
        const u32x4 v1 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(l + 1024), 0, 2));
        const u32x4 v2 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(l + 2048), 0, 2));
        const u32x4 v3 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(l + 3072), 0, 2));
        acc ^= v0 ^ v1 ^ v2 ^ v3;
    }
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_check(const uint8_t *base, uint32_t mis, uint32_t *out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), (short)0, 4096, 0x00020000);
    const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(threadIdx.x * 16u + mis), 0, 0));
    out[threadIdx.x * 4 + 0] = v.x;
    out[threadIdx.x * 4 + 1] = v.y;
    out[threadIdx.x * 4 + 2] = v.z;
    out[threadIdx.x * 4 + 3] = v.w;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
    const uint64_t n = 1536ull << 20;
    uint8_t *d;
    uint32_t *sink, *chk;
    CK(hipMalloc(&d, n + 4096));
    CK(hipMalloc(&sink, 256 * 512 * 4));
    CK(hipMalloc(&chk, 64 * 16));
    std::vector<uint8_t> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = uint8_t(i * 7 + 3);
    CK(hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice));
    for (uint32_t mis : {0u, 1u, 3u, 4u, 8u, 13u}) {
        hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d, mis, chk);
        std::vector<uint8_t> g(64 * 16);
        CK(hipMemcpy(g.data(), chk, g.size(), hipMemcpyDeviceToHost));
        bool ok = true;
        for (int i = 0; i < 64 * 16; ++i) ok = ok && g[i] == h[i + mis];
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_rd, dim3(256), dim3(512), 0, 0, d, n, mis, sink);
        CK(hipEventRecord(a));
        for (int i = 0; i < 30; ++i) hipLaunchKernelGGL(k_rd, dim3(256), dim3(512), 0, 0, d, n, mis, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"mis\": %u, \"us\": %.1f, \"GBps\": %.1f, \"bytes_ok\": %s}\n", mis, ms / 30 * 1e3, n / (ms / 30 * 1e-3) / 1e9, ok ? "true" : "false");
    }
    return 0;
}
