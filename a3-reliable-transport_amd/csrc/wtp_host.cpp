// wtp_host.cpp — host-memory entry points of the C-ABI (include/wtp_crc32.h).
//
// The reference path starts and ends in host memory: wSender reads the whole file into
// a std::vector<char> and checksums it chunk by chunk (cpp/src/base/Sender.cpp:82-92),
// wReceiver checksums each recvfrom() buffer (cpp/src/base/Receiver.cpp:123-131,
// :203-206).  These wrappers move such host batches through the device kernels:
//
//   slab s (<= 64 MiB of payload) on stream s%2:
//     [pageable source: CPU memcpy into library-owned pinned slab]  ->  H2D
//     -> CRC kernel -> D2H of the 32-bit results into pinned memory
//
// Two slabs are in flight, so slab s+1's staging and H2D overlap slab s's kernel and
// D2H.  Pinned sources (e.g. from hipHostMalloc) are copied H2D directly.  The end-to-end
// rate is PCIe-bound; DESIGN.md records the measured figure.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "wtp_crc32.h"

// Defined in crc32_kernels.hip: sets the per-thread message read by wtp_last_error().
extern "C" int wtp_set_error_(int code, const char *msg);

namespace {

constexpr size_t kSlabBytes = 64ull << 20;
constexpr size_t kStageThreads = 6;  // staging-copy threads per pipeline (pageable sources)

int hfail(int code, const char *what, hipError_t e) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return wtp_set_error_(code, buf);
}

#define H_HIP(call)                                                  \
    do {                                                             \
        hipError_t e_ = (call);                                      \
        if (e_ != hipSuccess) return hfail(WTP_EHIP, #call, e_);     \
    } while (0)

struct Pipe {
    std::mutex mu;
    std::once_flag once;
    int rc = WTP_OK;
    hipStream_t st[2] = {nullptr, nullptr};
    uint8_t *pin_in[2] = {nullptr, nullptr};
    uint8_t *dev_in[2] = {nullptr, nullptr};
    uint32_t *pin_aux[2] = {nullptr, nullptr};   // recv_len staging (verify)
    uint32_t *dev_aux[2] = {nullptr, nullptr};
    uint32_t *pin_out[2] = {nullptr, nullptr};   // crc results
    uint32_t *dev_out[2] = {nullptr, nullptr};
    uint8_t *pin_ok[2] = {nullptr, nullptr};
    uint8_t *dev_ok[2] = {nullptr, nullptr};
    void *view_ok0 = nullptr, *view_out0 = nullptr;  // device views of pin_ok[0] / pin_out[0] (zero-copy verify)
    size_t max_pk = 0;                           // packets per slab (results capacity)
    std::once_flag wire_once;                    // the builder's wire slabs, made on first use
    int wire_rc = WTP_OK;
    uint8_t *dev_wire[2] = {nullptr, nullptr};
    uint8_t *pin_wire[2] = {nullptr, nullptr};
};
Pipe g_pipe[64];

int pipe_get(Pipe *&out) {
    int dev = 0;
    H_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return hfail(WTP_EINVAL, "device index", hipSuccess);
    int rc = wtp_init(dev);
    if (rc) return rc;
    Pipe &p = g_pipe[dev];
    std::call_once(p.once, [&p] {
        auto mk = [&p]() -> int {
            p.max_pk = kSlabBytes / 16 + 1;  // worst case: 16-B datagrams / 1-B chunks capped below
            for (int b = 0; b < 2; ++b) {
                H_HIP(hipStreamCreateWithFlags(&p.st[b], hipStreamNonBlocking));
                H_HIP(hipHostMalloc(reinterpret_cast<void **>(&p.pin_in[b]), kSlabBytes, hipHostMallocDefault));
                H_HIP(hipMalloc(reinterpret_cast<void **>(&p.dev_in[b]), kSlabBytes + 64));
                H_HIP(hipHostMalloc(reinterpret_cast<void **>(&p.pin_out[b]), p.max_pk * 4, hipHostMallocDefault));
                H_HIP(hipMalloc(reinterpret_cast<void **>(&p.dev_out[b]), p.max_pk * 4));
                H_HIP(hipHostMalloc(reinterpret_cast<void **>(&p.pin_aux[b]), p.max_pk * 4, hipHostMallocDefault));
                H_HIP(hipMalloc(reinterpret_cast<void **>(&p.dev_aux[b]), p.max_pk * 4));
                H_HIP(hipHostMalloc(reinterpret_cast<void **>(&p.pin_ok[b]), p.max_pk, hipHostMallocDefault));
                H_HIP(hipMalloc(reinterpret_cast<void **>(&p.dev_ok[b]), p.max_pk));
            }
            // the library's own pinned result buffers never move: look their device views
            // up once, not per zero-copy call.  Optional: without them only the
            // zero-copy verify fast path is skipped, so a failed lookup leaves both null and
            // clears the HIP error instead of failing the pipeline
            if (hipHostGetDevicePointer(&p.view_ok0, p.pin_ok[0], 0) != hipSuccess ||
                hipHostGetDevicePointer(&p.view_out0, p.pin_out[0], 0) != hipSuccess) {
                p.view_ok0 = p.view_out0 = nullptr;
                (void)hipGetLastError();
            }
            return WTP_OK;
        };
        p.rc = mk();
    });
    if (p.rc) return hfail(p.rc, "host pipeline setup failed", hipSuccess);
    out = &p;
    return WTP_OK;
}

// Staging copy of a pageable source into a pinned slab, split over a few threads: one
// thread's memcpy (~25 GB/s) is what bounded pageable sources at half the pinned
// rate (C3: 26 vs 52 GiB/s), below the PCIe link.
void stage_copy(void *dst, const void *src, size_t bytes) {
    constexpr size_t kMinPart = 8ull << 20;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t parts = std::min<size_t>({kStageThreads, std::max<size_t>(1, hw / 2), bytes / kMinPart});
    if (parts <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    // ceil(bytes / parts) rounded up to a page, so parts * per >= bytes and the last part
    // copies whatever is left (rounding floor(bytes / parts) up left bytes % parts bytes
    // uncopied whenever floor(bytes / parts) was already page-aligned)
    const size_t per = ((bytes + parts - 1) / parts + 4095) & ~size_t(4095);
    std::vector<std::thread> th;
    th.reserve(parts - 1);
    for (size_t i = 1; i < parts; ++i) {
        const size_t o = i * per;
        if (o >= bytes) break;
        const size_t cnt = i + 1 == parts ? bytes - o : std::min(per, bytes - o);
        th.emplace_back([=] { memcpy(static_cast<uint8_t *>(dst) + o, static_cast<const uint8_t *>(src) + o, cnt); });
    }
    memcpy(dst, src, std::min(per, bytes));
    for (auto &t : th) t.join();
}

bool is_pinned(const void *ptr) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// One slab of work: `in_bytes` host bytes at `src` -> device, then `run` launches the
// kernels on stream st; `finish` copies results out once the slab's stream is done.
struct Slab {
    const uint8_t *src = nullptr;
    size_t in_bytes = 0;
    size_t first = 0, count = 0;  // packet range
    bool live = false;
};

}  // namespace

extern "C" {

// Fixed-geometry host batch (also used by wtp_crc32_host_chunked): payload i =
// h[i*stride, i*stride + len), the last packet may be shorter (tail_len) when
// `tail_len` != len.
// Wait for both pipeline streams (errors ignored: the caller is already failing).  Run
// before any error return from inside a pipelined loop, so no H2D into pin_in / D2H into
// pin_out of this call is still in flight when the mutex is released and the next caller
// reuses those buffers (the library keeps no work past its return, wtp_crc32.h).
static void drain(Pipe *P) {
    for (int b = 0; b < 2; ++b) (void)hipStreamSynchronize(P->st[b]);
    (void)hipGetLastError();
}

static int host_fixed_loop(Pipe *P, const uint8_t *h, bool pinned, size_t stride, size_t len, size_t n,
                           size_t tail_len, uint32_t *h_out) {
    const size_t step = stride ? stride : 1;
    size_t per = std::min(P->max_pk, std::max<size_t>(1, (kSlabBytes - len) / step + 1));
    if (stride == 0) per = std::min(n, P->max_pk);
    Slab slot[2];
    size_t s = 0;
    int rc = WTP_OK;
    for (size_t first = 0; first < n || slot[0].live || slot[1].live; ++s) {
        const int b = int(s & 1);
        Slab &sl = slot[b];
        if (sl.live) {  // retire the slab that used this buffer two steps ago
            H_HIP(hipStreamSynchronize(P->st[b]));
            memcpy(h_out + sl.first, P->pin_out[b], sl.count * 4);
            sl.live = false;
        }
        if (first >= n) continue;
        const size_t cnt = std::min(per, n - first);
        const bool has_tail = (first + cnt == n) && tail_len != len;
        const size_t last_len = has_tail ? tail_len : len;
        const size_t bytes = (cnt - 1) * stride + last_len;
        const uint8_t *src = h + first * stride;
        if (pinned) {
            H_HIP(hipMemcpyAsync(P->dev_in[b], src, bytes, hipMemcpyHostToDevice, P->st[b]));
        } else {
            stage_copy(P->pin_in[b], src, bytes);
            H_HIP(hipMemcpyAsync(P->dev_in[b], P->pin_in[b], bytes, hipMemcpyHostToDevice, P->st[b]));
        }
        const size_t full = has_tail ? cnt - 1 : cnt;
        if (full && (rc = wtp_crc32_batch_fixed(P->dev_in[b], stride, len, full, P->dev_out[b], P->st[b]))) return rc;
        if (has_tail &&
            (rc = wtp_crc32_batch_fixed(P->dev_in[b] + full * stride, 0, tail_len, 1, P->dev_out[b] + full, P->st[b])))
            return rc;
        H_HIP(hipMemcpyAsync(P->pin_out[b], P->dev_out[b], cnt * 4, hipMemcpyDeviceToHost, P->st[b]));
        sl.first = first;
        sl.count = cnt;
        sl.live = true;
        first += cnt;
    }
    return WTP_OK;
}

// Fixed-geometry host batch on the current device (also used by wtp_crc32_host_chunked):
// payload i = h[i*stride, i*stride + len), the last packet may be shorter (tail_len)
// when `tail_len` != len.
static int host_fixed_impl(const void *h_payloads, size_t stride, size_t len, size_t n, size_t tail_len,
                           uint32_t *h_out) {
    if (n == 0) return WTP_OK;
    if (!h_payloads || !h_out) return hfail(WTP_EINVAL, "null pointer", hipSuccess);
    if (len > kSlabBytes || stride > kSlabBytes) return hfail(WTP_EINVAL, "payload/stride larger than a slab", hipSuccess);
    Pipe *P = nullptr;
    int rc = pipe_get(P);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(P->mu);
    rc = host_fixed_loop(P, static_cast<const uint8_t *>(h_payloads), is_pinned(h_payloads), stride, len, n, tail_len,
                         h_out);
    if (rc) drain(P);
    return rc;
}

int wtp_crc32_host_batch_fixed(const void *h_payloads, size_t stride, size_t len, size_t n, uint32_t *h_out) {
    return host_fixed_impl(h_payloads, stride, len, n, len, h_out);
}

int wtp_crc32_host_chunked(const void *h_buf, size_t nbytes, size_t chunk, uint32_t *h_out) {
    if (nbytes == 0) return WTP_OK;
    if (chunk == 0) return hfail(WTP_EINVAL, "chunk == 0", hipSuccess);
    const size_t n = (nbytes + chunk - 1) / chunk;
    const size_t tail = nbytes - (n - 1) * chunk;
    return host_fixed_impl(h_buf, chunk, chunk, n, tail, h_out);
}

static int host_verify_loop(Pipe *P, const uint8_t *h, bool pinned, size_t stride, const uint32_t *h_recv_len,
                            bool lens_pinned, size_t n, uint8_t *h_ok, uint32_t *h_crc_out) {
    const size_t per = std::min(P->max_pk, kSlabBytes / stride);
    Slab slot[2];
    size_t s = 0;
    int rc = WTP_OK;
    for (size_t first = 0; first < n || slot[0].live || slot[1].live; ++s) {
        const int b = int(s & 1);
        Slab &sl = slot[b];
        if (sl.live) {
            H_HIP(hipStreamSynchronize(P->st[b]));
            memcpy(h_ok + sl.first, P->pin_ok[b], sl.count);
            if (h_crc_out) memcpy(h_crc_out + sl.first, P->pin_out[b], sl.count * 4);
            sl.live = false;
        }
        if (first >= n) continue;
        const size_t cnt = std::min(per, n - first);
        const uint8_t *src = h + first * stride;
        const uint32_t *lsrc = h_recv_len + first;
        if (!pinned) {
            stage_copy(P->pin_in[b], src, cnt * stride);
            src = P->pin_in[b];
        }
        if (!lens_pinned) {
            memcpy(P->pin_aux[b], lsrc, cnt * 4);
            lsrc = P->pin_aux[b];
        }
        H_HIP(hipMemcpyAsync(P->dev_in[b], src, cnt * stride, hipMemcpyHostToDevice, P->st[b]));
        H_HIP(hipMemcpyAsync(P->dev_aux[b], lsrc, cnt * 4, hipMemcpyHostToDevice, P->st[b]));
        if ((rc = wtp_crc32_verify_batch(P->dev_in[b], stride, P->dev_aux[b], cnt, P->dev_ok[b], P->dev_out[b], P->st[b])))
            return rc;
        H_HIP(hipMemcpyAsync(P->pin_ok[b], P->dev_ok[b], cnt, hipMemcpyDeviceToHost, P->st[b]));
        H_HIP(hipMemcpyAsync(P->pin_out[b], P->dev_out[b], cnt * 4, hipMemcpyDeviceToHost, P->st[b]));
        sl.first = first;
        sl.count = cnt;
        sl.live = true;
        first += cnt;
    }
    return WTP_OK;
}

// Device address of page-locked host memory (hipHostMalloc / wtp_host_alloc memory is
// mapped into the device's address space), or null for any other pointer.
static void *dev_view(const void *h) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, h) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}

// Host wrapper of the fused DATA builder (wSender --crc gpu; SURVEY.md §8f row 1,
// Packet.cpp:9-14,40-47, Sender.cpp:187-197): slabs of whole 1456-B chunks go H2D
// (pinned sources directly, pageable ones through the staging copy), wtp_build_data_packets
// writes their datagrams into a device wire slab, which comes back D2H straight into a
// pinned h_wire (else through a pinned slab); two slabs in flight.
static int wire_slabs(Pipe *P) {
    std::call_once(P->wire_once, [P] {
        auto mk = [P]() -> int {
            for (int b = 0; b < 2; ++b) {
                H_HIP(hipMalloc(reinterpret_cast<void **>(&P->dev_wire[b]), kSlabBytes));
                H_HIP(hipHostMalloc(reinterpret_cast<void **>(&P->pin_wire[b]), kSlabBytes, hipHostMallocDefault));
            }
            return WTP_OK;
        };
        P->wire_rc = mk();
    });
    return P->wire_rc ? hfail(P->wire_rc, "builder wire slabs", hipSuccess) : WTP_OK;
}

static int host_build_loop(Pipe *P, const uint8_t *h, size_t total, uint32_t seq0, uint8_t *h_wire, size_t ws,
                           uint32_t *h_wire_len) {
    constexpr size_t kChunk = 1456;
    const size_t n = (total + kChunk - 1) / kChunk;
    const bool pin_src = dev_view(h) != nullptr, pin_wire = dev_view(h_wire) != nullptr;
    const bool pin_len = h_wire_len && dev_view(h_wire_len) != nullptr;
    const size_t per = std::min({P->max_pk, kSlabBytes / kChunk, kSlabBytes / ws});
    struct {
        size_t first = 0, count = 0;
        bool live = false;
    } slot[2];
    for (size_t first = 0, s = 0; first < n || slot[0].live || slot[1].live; ++s) {
        const int b = int(s & 1);
        auto &sl = slot[b];
        if (sl.live) {
            H_HIP(hipStreamSynchronize(P->st[b]));
            if (!pin_wire) memcpy(h_wire + sl.first * ws, P->pin_wire[b], sl.count * ws);
            if (h_wire_len && !pin_len) memcpy(h_wire_len + sl.first, P->pin_aux[b], sl.count * 4);
            sl.live = false;
        }
        if (first >= n) continue;
        const size_t cnt = std::min(per, n - first);
        const size_t bytes = first + cnt == n ? total - first * kChunk : cnt * kChunk;
        const uint8_t *src = h + first * kChunk;
        if (!pin_src) {
            stage_copy(P->pin_in[b], src, bytes);
            src = P->pin_in[b];
        }
        H_HIP(hipMemcpyAsync(P->dev_in[b], src, bytes, hipMemcpyHostToDevice, P->st[b]));
        int rc = wtp_build_data_packets(P->dev_in[b], bytes, seq0 + uint32_t(first), P->dev_wire[b], ws,
                                        h_wire_len ? P->dev_aux[b] : nullptr, P->st[b]);
        if (rc) return rc;
        H_HIP(hipMemcpyAsync(pin_wire ? h_wire + first * ws : P->pin_wire[b], P->dev_wire[b], cnt * ws,
                             hipMemcpyDeviceToHost, P->st[b]));
        if (h_wire_len)
            H_HIP(hipMemcpyAsync(pin_len ? h_wire_len + first : P->pin_aux[b], P->dev_aux[b], cnt * 4,
                                 hipMemcpyDeviceToHost, P->st[b]));
        sl.first = first;
        sl.count = cnt;
        sl.live = true;
        first += cnt;
    }
    return WTP_OK;
}

// Small batches from a pinned ring and pinned lengths (wReceiver's window-size batches):
// the kernel reads the ring and the lengths in place over PCIe and writes ok / crc into
// the pipeline's pinned result buffers, so a call is one launch and one synchronisation
// instead of four copies around the launch.  Rings up to kZeroCopyBytes (4 MiB); larger ones
// take the copy pipeline (two slabs in flight), which streams PCIe at the link rate.
constexpr size_t kZeroCopyBytes = size_t(4) << 20;
static bool zero_copy_enabled(const char *var = "WTP_HOST_ZEROCOPY") {
    const char *e = getenv(var);  // 0 disables (A/B measurements, tests)
    return !(e && e[0] == '0');
}

static int host_verify_zero_copy(Pipe *P, const void *dr, size_t stride, const void *dl, size_t n, void *dok,
                                 void *dcrc, uint8_t *h_ok, uint32_t *h_crc_out) {
    int rc = wtp_crc32_verify_batch(dr, stride, static_cast<const uint32_t *>(dl), n, static_cast<uint8_t *>(dok),
                                    static_cast<uint32_t *>(dcrc), P->st[0]);
    if (rc) return rc;
    H_HIP(hipStreamSynchronize(P->st[0]));
    memcpy(h_ok, P->pin_ok[0], n);
    if (h_crc_out) memcpy(h_crc_out, P->pin_out[0], n * 4);
    return WTP_OK;
}

int wtp_crc32_host_verify(const void *h_dgrams, size_t stride, const uint32_t *h_recv_len, size_t n, uint8_t *h_ok,
                          uint32_t *h_crc_out) {
    if (n == 0) return WTP_OK;
    if (!h_dgrams || !h_recv_len || !h_ok) return hfail(WTP_EINVAL, "null pointer", hipSuccess);
    if (stride < 16 || stride > kSlabBytes) return hfail(WTP_EINVAL, "bad datagram stride", hipSuccess);
    Pipe *P = nullptr;
    int rc = pipe_get(P);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(P->mu);
    const void *dr = dev_view(h_dgrams), *dl = dev_view(h_recv_len);
    if (dr && dl && P->view_ok0 && P->view_out0 && n <= P->max_pk && n * stride <= kZeroCopyBytes &&
        zero_copy_enabled()) {
        rc = host_verify_zero_copy(P, dr, stride, dl, n, P->view_ok0, P->view_out0, h_ok, h_crc_out);
    } else {
        // a pinned ring (wReceiver's recvmmsg ring) is copied to the device directly
        rc = host_verify_loop(P, static_cast<const uint8_t *>(h_dgrams), dr != nullptr, stride, h_recv_len,
                              dl != nullptr, n, h_ok, h_crc_out);
    }
    if (rc) drain(P);
    return rc;
}

int wtp_host_build_data_packets(const void *h_payloads, size_t total_bytes, uint32_t seq0, void *h_wire,
                                size_t wire_stride, uint32_t *h_wire_len) {
    if (total_bytes == 0) return WTP_OK;
    if (!h_payloads || !h_wire) return hfail(WTP_EINVAL, "null pointer", hipSuccess);
    if (wire_stride < 16 + 1456 || wire_stride > kSlabBytes) return hfail(WTP_EINVAL, "bad wire stride", hipSuccess);
    Pipe *P = nullptr;
    int rc = pipe_get(P);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(P->mu);
    const void *ds = dev_view(h_payloads);
    void *dw = dev_view(h_wire), *dln = h_wire_len ? dev_view(h_wire_len) : nullptr;
    if (ds && dw && (!h_wire_len || dln) && zero_copy_enabled("WTP_HOST_BUILD_ZEROCOPY")) {
        // pinned both ways: the builder reads the payloads and writes the datagrams across
        // the link itself, both directions at once, no device staging
        rc = wtp_build_data_packets(ds, total_bytes, seq0, dw, wire_stride, static_cast<uint32_t *>(dln), P->st[0]);
        if (!rc) {
            hipError_t e = hipStreamSynchronize(P->st[0]);
            if (e != hipSuccess) rc = hfail(WTP_EHIP, "builder zero copy", e);
        }
        if (rc) drain(P);
        return rc;
    }
    if ((rc = wire_slabs(P))) return rc;
    rc = host_build_loop(P, static_cast<const uint8_t *>(h_payloads), total_bytes, seq0, static_cast<uint8_t *>(h_wire),
                         wire_stride, h_wire_len);
    if (rc) drain(P);
    return rc;
}

// Multi-GPU host path: the chunks of one host buffer split into ndev contiguous ranges,
// one pipeline (and one PCIe link, and one CPU staging thread for pageable sources) per
// device, results written straight into h_out.  Chunks are independent (Crc32.hpp:92-96
// keeps no state across calls), so no collective is needed: each device's slice of h_out
// is disjoint.
int wtp_crc32_host_chunked_multi(const void *h_buf, size_t nbytes, size_t chunk, uint32_t *h_out, const int *devices,
                                 int ndev) {
    if (nbytes == 0) return WTP_OK;
    if (chunk == 0) return hfail(WTP_EINVAL, "chunk == 0", hipSuccess);
    if (!h_buf || !h_out) return hfail(WTP_EINVAL, "null pointer", hipSuccess);
    if (ndev <= 0) ndev = wtp_device_count();
    if (ndev <= 0) return hfail(WTP_ENODEV, "no HIP device", hipSuccess);
    if (ndev > 64) return hfail(WTP_EINVAL, "ndev > 64", hipSuccess);
    const size_t n = (nbytes + chunk - 1) / chunk;
    const size_t tail = nbytes - (n - 1) * chunk;
    const uint8_t *h = static_cast<const uint8_t *>(h_buf);
    int used = int(std::min<size_t>(size_t(ndev), n));
    std::vector<int> rcs(used, WTP_OK);
    std::vector<std::string> msgs(used);
    auto work = [&](int r) {
        const int dev = devices ? devices[r] : r;
        const size_t lo = n * size_t(r) / size_t(used), hi = n * size_t(r + 1) / size_t(used);
        int prev = 0;
        int rc = WTP_OK;
        if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(dev) != hipSuccess) {
            rc = hfail(WTP_ENODEV, "hipSetDevice", hipSuccess);
        } else {
            const bool last = hi == n;
            rc = host_fixed_impl(h + lo * chunk, chunk, chunk, hi - lo, last ? tail : chunk, h_out + lo);
            (void)hipSetDevice(prev);
        }
        rcs[r] = rc;
        if (rc) msgs[r] = std::string("device ") + std::to_string(dev) + ": " + wtp_last_error();
    };
    if (used == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int r = 0; r < used; ++r) th.emplace_back(work, r);
        for (auto &t : th) t.join();
    }
    for (int r = 0; r < used; ++r)
        if (rcs[r]) return wtp_set_error_(rcs[r], msgs[r].c_str());
    return WTP_OK;
}

// Pinned host allocation helpers for callers that want zero-copy staging (wSender --crc
// gpu reads its file straight into such a buffer; wReceiver's recvmmsg ring lives in one).
void *wtp_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}
void wtp_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

}  // extern "C"
