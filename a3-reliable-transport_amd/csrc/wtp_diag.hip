// wtp_diag.hip — measurement probes for bench.py and tools/ (not part of the drop-in
// boundary; the product library libwtp_crc32.so does not contain them).
//
//   wtp_diag_read_xor : the HBM read ceiling of the box the bench runs on — a plain
//                       streaming read (nt buffer_load_dwordx4, 1 KiB per wave
//                       instruction, 4 in flight per lane) XOR-reduced to one word per
//                       lane, over the same bytes the CRC kernel reads.  bench.py times
//                       it interleaved with the CRC kernel so a slow box and a slow
//                       kernel can be told apart (VERDICT r1 "what's weak" 1).
//   wtp_diag_clock    : effective shader clock: one wave spins on dependent VALU work
//                       and reads s_memtime (shader-clock counter) and s_memrealtime
//                       (constant 100 MHz) before and after.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "wtp_diag.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_read_xor(const uint8_t *__restrict__ base, uint64_t n16, uint32_t *sink) {
    typedef const __attribute__((address_space(1))) u32x4 gu32x4;
    gu32x4 *p = (gu32x4 *)base;
    const uint64_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
    // wave w reads 4 KiB blocks w, w + nwaves, ... : 4 x 1 KiB instructions per block
    const uint64_t nblk = n16 / 256;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t b = wave; b < nblk; b += nwaves) {
        const uint64_t i = b * 256 + lane;
        const u32x4 v0 = __builtin_nontemporal_load(p + i);
        const u32x4 v1 = __builtin_nontemporal_load(p + i + 64);
        const u32x4 v2 = __builtin_nontemporal_load(p + i + 128);
        const u32x4 v3 = __builtin_nontemporal_load(p + i + 192);
        acc ^= v0 ^ v1 ^ v2 ^ v3;
    }
    // ragged tail (< 4 KiB), whole 16-B words only
    for (uint64_t i = nblk * 256 + wave * 64 + lane; i < n16; i += nwaves * 64) acc ^= __builtin_nontemporal_load(p + i);
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) sink[0] = x;  // keeps the loads; (practically) never stores
}

__global__ void k_clock(uint64_t *out, uint32_t iters) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t v = threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i) v = v * 1664525u + 1013904223u;
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = v;
    }
}

}  // namespace

extern "C" {

int wtp_diag_read_xor(const void *d_buf, size_t nbytes, uint32_t *d_sink, unsigned blocks, unsigned threads,
                      void *stream) {
    if (!d_buf || !d_sink || nbytes < 16 || threads == 0 || threads > 512 || threads % 64 || blocks == 0) return -1;
    hipLaunchKernelGGL(k_read_xor, dim3(blocks), dim3(threads), 0, static_cast<hipStream_t>(stream),
                       static_cast<const uint8_t *>(d_buf), uint64_t(nbytes / 16), d_sink);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int wtp_diag_clock(uint64_t *d_out, uint32_t iters, void *stream) {
    if (!d_out) return -1;
    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), d_out, iters);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Timing-only events (hip_runtime_api.h, hipEventDisableSystemFence: "for events that are
// only being used to measure timing ... avoiding the cost of cache writeback and
// invalidation, and the performance impact of those actions on the execution of
// following work").
int wtp_diag_event_create(void **ev) {
    if (!ev) return -1;
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return -2;
    *ev = e;
    return 0;
}

int wtp_diag_event_record(void *ev, void *stream) {
    if (!ev) return -1;
    return hipEventRecord(static_cast<hipEvent_t>(ev), static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -2;
}

int wtp_diag_event_elapsed_ms(void *start, void *end, float *ms) {
    if (!start || !end || !ms) return -1;
    if (hipEventSynchronize(static_cast<hipEvent_t>(end)) != hipSuccess) return -2;
    return hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(end)) == hipSuccess ? 0 : -2;
}

// Make `stream` wait for `ev` (a timing-only event): a cross-stream dependency whose
// record on the producer stream carries no system-scope fence (bench.py --gather-helper).
int wtp_diag_stream_wait(void *stream, void *ev) {
    if (!ev) return -1;
    return hipStreamWaitEvent(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(ev), 0) == hipSuccess ? 0 : -2;
}

int wtp_diag_event_destroy(void *ev) {
    if (!ev) return 0;
    return hipEventDestroy(static_cast<hipEvent_t>(ev)) == hipSuccess ? 0 : -2;
}

}  // extern "C"
