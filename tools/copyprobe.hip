// Copy-ceiling probe for the fused DATA builder (diagnostic, not the product).
// Times, on one MI355X, copies with the builder's traffic: 1 M x 1456-B payloads
// (contiguous) -> 1472-B wire slots (payload at +16).  Variants:
//   flat   : contiguous 1456*N bytes -> contiguous, 16 B per lane (the plain copy ceiling)
//   slot   : payload -> slot + 16, 16 B per lane, write-back stores
//   slotnt : the same with nt loads and nt stores
//   slotu4 : slot copy, 4 x 16 B per lane in flight (more bytes per wave before the waits)
//   wslot  : iterate over wire chunks instead: 64-B aligned full-segment stores, loads
//            16-B aligned only (the wire payload sits 16 B into a 64-B aligned slot)
//   wslotnt: the same with nt loads and nt stores
// Prints read+write GB/s per variant (HIP events, 50 launches after 20 warmups).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t kN = 1u << 20, kL = 1456, kW = 1472;

__global__ __launch_bounds__(256) void k_flat(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, uint64_t n16) {
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * 256) d[i] = s[i];
}

template <int NT>
__global__ __launch_bounds__(256) void k_slot(const uint8_t *__restrict__ s, uint8_t *__restrict__ d, uint64_t n16) {
    constexpr uint64_t c = kL / 16;  // 91 chunks per packet
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * 256) {
        const uint64_t p = i / c, k = i - p * c;
        const u32x4 *src = reinterpret_cast<const u32x4 *>(s + i * 16);
        u32x4 *dst = reinterpret_cast<u32x4 *>(d + p * kW + 16 + k * 16);
        if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(src), dst);
        else *dst = *src;
    }
}

// wire chunk m of slot p (m = 1..91 payload, m = 0 header: skipped) <- payload chunk m - 1
template <int NT>
__global__ __launch_bounds__(256) void k_wslot(const uint8_t *__restrict__ s, uint8_t *__restrict__ d, uint64_t nw16) {
    constexpr uint64_t c = kW / 16;  // 92 chunks per slot
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < nw16; i += uint64_t(gridDim.x) * 256) {
        const uint64_t p = i / c, k = i - p * c;
        if (k == 0) continue;
        const u32x4 *src = reinterpret_cast<const u32x4 *>(s + p * kL + (k - 1) * 16);
        u32x4 *dst = reinterpret_cast<u32x4 *>(d + i * 16);
        if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(src), dst);
        else *dst = *src;
    }
}

__global__ __launch_bounds__(256) void k_slot4(const uint8_t *__restrict__ s, uint8_t *__restrict__ d, uint64_t n16) {
    constexpr uint64_t c = kL / 16;
    const uint64_t T = uint64_t(gridDim.x) * 256;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += 4 * T) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t ii = i + u * T;
            if (ii < n16) v[u] = *reinterpret_cast<const u32x4 *>(s + ii * 16);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t ii = i + u * T;
            if (ii < n16) {
                const uint64_t p = ii / c, k = ii - p * c;
                *reinterpret_cast<u32x4 *>(d + p * kW + 16 + k * 16) = v[u];
            }
        }
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <class F>
static double time_ms(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int i = 0; i < 20; ++i) f();
    hipEventRecord(a);
    for (int i = 0; i < 50; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    return ms / 50;
}

int main() {
    uint8_t *s, *d;
    CK(hipMalloc(&s, kN * kL));
    CK(hipMalloc(&d, kN * kW));
    CK(hipMemset(s, 0x5a, kN * kL));
    CK(hipMemset(d, 0, kN * kW));
    const uint64_t n16 = kN * kL / 16;
    const double rw = 2.0 * kN * kL;
    const unsigned grids[] = {1024, 2048, 4096, 8192};
    for (unsigned g : grids) {
        double t;
        t = time_ms([&] { hipLaunchKernelGGL(k_flat, dim3(g), dim3(256), 0, 0, (const u32x4 *)s, (u32x4 *)d, n16); });
        printf("{\"variant\": \"flat\", \"grid\": %u, \"ms\": %.4f, \"GBps_rw\": %.1f}\n", g, t, rw / t / 1e6);
        t = time_ms([&] { hipLaunchKernelGGL(k_slot<0>, dim3(g), dim3(256), 0, 0, s, d, n16); });
        printf("{\"variant\": \"slot\", \"grid\": %u, \"ms\": %.4f, \"GBps_rw\": %.1f}\n", g, t, rw / t / 1e6);
        t = time_ms([&] { hipLaunchKernelGGL(k_slot<1>, dim3(g), dim3(256), 0, 0, s, d, n16); });
        printf("{\"variant\": \"slotnt\", \"grid\": %u, \"ms\": %.4f, \"GBps_rw\": %.1f}\n", g, t, rw / t / 1e6);
        t = time_ms([&] { hipLaunchKernelGGL(k_wslot<0>, dim3(g), dim3(256), 0, 0, s, d, kN * kW / 16); });
        printf("{\"variant\": \"wslot\", \"grid\": %u, \"ms\": %.4f, \"GBps_rw\": %.1f}\n", g, t, rw / t / 1e6);
        t = time_ms([&] { hipLaunchKernelGGL(k_wslot<1>, dim3(g), dim3(256), 0, 0, s, d, kN * kW / 16); });
        printf("{\"variant\": \"wslotnt\", \"grid\": %u, \"ms\": %.4f, \"GBps_rw\": %.1f}\n", g, t, rw / t / 1e6);
        t = time_ms([&] { hipLaunchKernelGGL(k_slot4, dim3(g), dim3(256), 0, 0, s, d, n16); });
        printf("{\"variant\": \"slotu4\", \"grid\": %u, \"ms\": %.4f, \"GBps_rw\": %.1f}\n", g, t, rw / t / 1e6);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
