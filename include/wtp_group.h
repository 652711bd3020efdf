/*
 * wtp_group.h — several MI355X GPUs of ONE process, with an RCCL communicator
 * (lib/libwtp_group.so; links libwtp_crc32.so and RCCL).
 *
 * For a C/C++ host such as wSender that holds per-device shards of a packet batch
 * itself: every device checksums its own shard with the braided kernel,
 * and the 32-bit results are gathered to one root device over xGMI.  Packets are
 * independent (cpp/src/common/Crc32.hpp:92-96 keeps no state across calls), so the
 * gather is the only exchange step.  Multi-process jobs (one process per GPU) use
 * torch.distributed / RCCL directly instead (a3-reliable-transport_amd/shard.py).
 *
 * Conventions as in wtp_crc32.h: 0 / negative wtp_status, wtp_last_error() for the
 * message, asynchronous on the given streams, no pointers kept past the call.
 */
#ifndef WTP_GROUP_H
#define WTP_GROUP_H

#include <stddef.h>
#include <stdint.h>

#include "wtp_crc32.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wtp_group wtp_group;

/* Communicator over devices[0 .. ndev) (rank r = devices[r]; NULL devices = 0 .. ndev-1),
   tables initialised on every device.  The caller's current device is unchanged. */
int wtp_group_create(const int *devices, int ndev, wtp_group **out);
void wtp_group_destroy(wtp_group *g);
int wtp_group_size(const wtp_group *g);

/* Sharded fixed-length batch + gather.  Shard r lives on rank r's device: n_per[r]
   payloads d_shards[r][i*stride .. i*stride + len) (wtp_crc32_batch_fixed geometry).
   Their CRCs go to d_local[r] (n_per[r] u32 on that device), then to d_out on the root
   rank's device in rank order (sum of n_per entries).  Equal shard sizes use one
   ncclGather; ragged ones grouped ncclSend/ncclRecv.  streams[r] is a hipStream_t of
   rank r's device (streams == NULL or a NULL entry: the null stream).  Every device is
   made current before the RCCL group opens; if an enqueue nevertheless fails inside the
   group, the communicators are aborted (no rank waits for a peer that never posted) and
   every later call on g fails: destroy it and create a new one. */
int wtp_group_crc32_fixed_gather(wtp_group *g, const void *const *d_shards, size_t stride, size_t len,
                                 const size_t *n_per, uint32_t *const *d_local, uint32_t *d_out, int root,
                                 void *const *streams);

#ifdef __cplusplus
}
#endif

#endif /* WTP_GROUP_H */
