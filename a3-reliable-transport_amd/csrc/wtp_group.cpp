// wtp_group.cpp — several GPUs of one process + RCCL gather of the 32-bit results
// (include/wtp_group.h).  Kept out of libwtp_crc32.so so that the drop-in library has no
// RCCL dependency (Python processes bring their own through torch.distributed).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "wtp_group.h"

extern "C" int wtp_set_error_(int code, const char *msg);

struct wtp_group {
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    bool aborted = false;  // a gather failed inside its RCCL group: communicators aborted
};

namespace {

int gfail(int code, const std::string &m) { return wtp_set_error_(code, m.c_str()); }

// Runs f with device d current, then restores the caller's device.
template <class F>
int on_device(int d, F &&f) {
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) return gfail(WTP_EHIP, "hipGetDevice failed");
    if (hipSetDevice(d) != hipSuccess) return gfail(WTP_ENODEV, "hipSetDevice(" + std::to_string(d) + ") failed");
    const int rc = f();
    (void)hipSetDevice(prev);
    return rc;
}

int nccl_fail(const char *what, ncclResult_t r) {
    return gfail(WTP_EHIP, std::string(what) + ": " + ncclGetErrorString(r));
}

}  // namespace

extern "C" {

int wtp_group_create(const int *devices, int ndev, wtp_group **out) {
    if (!out) return gfail(WTP_EINVAL, "out is null");
    *out = nullptr;
    if (ndev <= 0 || ndev > 64) return gfail(WTP_EINVAL, "ndev must be 1..64");
    auto *g = new wtp_group;
    for (int r = 0; r < ndev; ++r) g->dev.push_back(devices ? devices[r] : r);
    for (int d : g->dev) {
        const int rc = wtp_init(d);
        if (rc) {
            delete g;
            return rc;
        }
    }
    g->comm.resize(ndev);
    int prev = 0;
    (void)hipGetDevice(&prev);
    const ncclResult_t r = ncclCommInitAll(g->comm.data(), ndev, g->dev.data());
    (void)hipSetDevice(prev);
    if (r != ncclSuccess) {
        delete g;
        return nccl_fail("ncclCommInitAll", r);
    }
    *out = g;
    return WTP_OK;
}

void wtp_group_destroy(wtp_group *g) {
    if (!g) return;
    if (!g->aborted)
        for (ncclComm_t c : g->comm) (void)ncclCommDestroy(c);
    delete g;
}

int wtp_group_size(const wtp_group *g) { return g ? int(g->dev.size()) : 0; }

int wtp_group_crc32_fixed_gather(wtp_group *g, const void *const *d_shards, size_t stride, size_t len,
                                 const size_t *n_per, uint32_t *const *d_local, uint32_t *d_out, int root,
                                 void *const *streams) {
    if (!g || !d_shards || !n_per || !d_local || !d_out) return gfail(WTP_EINVAL, "null pointer");
    if (g->aborted) return gfail(WTP_EHIP, "group aborted by an earlier failed gather; destroy and recreate it");
    const int R = int(g->dev.size());
    if (root < 0 || root >= R) return gfail(WTP_EINVAL, "root out of range");
    for (int r = 0; r < R; ++r)
        if (!d_local[r] || (n_per[r] && !d_shards[r])) return gfail(WTP_EINVAL, "null shard or result pointer");
    auto st = [&](int r) { return streams ? static_cast<hipStream_t>(streams[r]) : hipStream_t(nullptr); };
    // 1. every rank checksums its shard (the braided kernel for 1456-B payloads)
    for (int r = 0; r < R; ++r) {
        const int rc = on_device(g->dev[r], [&] {
            return wtp_crc32_batch_fixed(d_shards[r], stride, len, n_per[r], d_local[r], st(r));
        });
        if (rc) return rc;
    }
    // 2. gather to the root, stream-ordered after each rank's kernel.  Every device is
    // made current once before the group opens, so nothing expected can fail between
    // ncclGroupStart and ncclGroupEnd; if an enqueue still fails there, the ops already
    // posted for other ranks would wait for peers that never post theirs, so the
    // communicators are aborted (and the group refuses further use) instead.
    bool equal = true;
    for (int r = 1; r < R; ++r) equal = equal && n_per[r] == n_per[0];
    int prev = 0;
    (void)hipGetDevice(&prev);
    for (int r = 0; r < R; ++r)
        if (hipSetDevice(g->dev[r]) != hipSuccess) {
            (void)hipSetDevice(prev);
            return gfail(WTP_ENODEV, "hipSetDevice(" + std::to_string(g->dev[r]) + ") failed");
        }
    ncclResult_t res = ncclGroupStart();
    if (res != ncclSuccess) return nccl_fail("ncclGroupStart", res);
    int rc = WTP_OK;
    size_t off_root = 0;
    for (int r = 0; r < root; ++r) off_root += n_per[r];
    for (int r = 0; r < R && rc == WTP_OK; ++r) {
        if (hipSetDevice(g->dev[r]) != hipSuccess) {
            rc = gfail(WTP_ENODEV, "hipSetDevice failed");
            break;
        }
        if (equal) {
            res = ncclGather(d_local[r], r == root ? d_out : nullptr, n_per[r], ncclUint32, root, g->comm[r], st(r));
            if (res != ncclSuccess) rc = nccl_fail("ncclGather", res);
        } else if (r != root) {
            if (n_per[r]) res = ncclSend(d_local[r], n_per[r], ncclUint32, root, g->comm[r], st(r));
            if (res != ncclSuccess) rc = nccl_fail("ncclSend", res);
        } else {
            size_t off = 0;
            for (int q = 0; q < R && rc == WTP_OK; ++q) {
                if (q != root && n_per[q]) {
                    res = ncclRecv(d_out + off, n_per[q], ncclUint32, q, g->comm[root], st(root));
                    if (res != ncclSuccess) rc = nccl_fail("ncclRecv", res);
                }
                off += n_per[q];
            }
        }
    }
    res = ncclGroupEnd();
    if (rc == WTP_OK && res != ncclSuccess) rc = nccl_fail("ncclGroupEnd", res);
    if (rc != WTP_OK) {
        for (ncclComm_t c : g->comm) (void)ncclCommAbort(c);
        g->aborted = true;
        (void)hipSetDevice(prev);
        return rc;
    }
    // the root's own shard (ragged path): a device-local copy behind its kernel
    if (rc == WTP_OK && !equal && n_per[root] && hipSetDevice(g->dev[root]) == hipSuccess) {
        if (hipMemcpyAsync(d_out + off_root, d_local[root], n_per[root] * 4, hipMemcpyDeviceToDevice, st(root)) !=
            hipSuccess)
            rc = gfail(WTP_EHIP, "hipMemcpyAsync (root shard) failed");
    }
    (void)hipSetDevice(prev);
    return rc;
}

}  // extern "C"
