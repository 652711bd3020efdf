/*
 * wtp_crc32.h — C-ABI of the MI355X (gfx950) CRC-32 path for WTP.
 *
 * Drop-in boundary for the reference's checksum call surface
 * (mmheyer/a3-reliable-transport):
 *   - inline uint32_t crc32(const void *buf, size_t size)   cpp/src/common/Crc32.hpp:91-102
 *     called from Packet::calculateCheckSum                 cpp/src/base/Packet.cpp:36-38
 *                                                           cpp/src/opt/Packet.cpp:38-40
 *     and from the receiver verify                          cpp/src/base/Receiver.cpp:203-206
 *                                                           cpp/src/opt/Receiver.cpp:208-211
 *   - struct PacketHeader {type, seqNum, length, checksum}   cpp/src/common/PacketHeader.hpp:5-10
 *
 * The reference calls crc32() once per packet on the CPU.  These entry points take
 * whole batches of payloads that are already device-resident (or host buffers, for
 * the *_host_* wrappers) and compute every CRC in one HIP launch.  Results are
 * bit-identical to the reference: IEEE CRC-32, reflected polynomial 0xEDB88320,
 * init 0xFFFFFFFF, xorout 0xFFFFFFFF; crc of an empty payload is 0.
 *
 * Conventions
 *   - Plain pointers and sizes; `stream` is a hipStream_t passed as void* (NULL =
 *     the null stream).  Device entry points are asynchronous on that stream; the
 *     library keeps no pointer past stream completion.
 *   - Return 0 (WTP_OK) on success, a negative wtp_status on failure; never abort.
 *     wtp_last_error() gives a per-thread message for the last failure.
 *   - n == 0 is valid (no launch).  DATA payloads are at most WTP_MAX_PAYLOAD
 *     (1456 = 1500 - 20 IP - 8 UDP - 16 header, README.md:46-47); the kernels accept
 *     any payload up to WTP_MAX_KERNEL_LEN (4096 >= the 1484 bytes a 1500-byte
 *     recvfrom buffer can carry after the header, cpp/src/base/Receiver.cpp:123).
 *   - Device-side data errors (a length > WTP_MAX_KERNEL_LEN in a device array)
 *     cannot be returned by an async call: such packets get crc 0 and set a sticky
 *     per-device flag readable with wtp_device_status().
 */
#ifndef WTP_CRC32_H
#define WTP_CRC32_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WTP_MAX_PAYLOAD 1456u   /* cpp/src/base/Sender.cpp:20 CHUNK_SIZE */
#define WTP_MAX_KERNEL_LEN 4096u
#define WTP_HEADER_BYTES 16u    /* sizeof(PacketHeader), PacketHeader.hpp:5-10 */
#define WTP_TYPE_START 0u       /* cpp/src/base/Packet.hpp:8-13 */
#define WTP_TYPE_END 1u
#define WTP_TYPE_DATA 2u
#define WTP_TYPE_ACK 3u

typedef enum wtp_status {
    WTP_OK = 0,
    WTP_EINVAL = -1,   /* bad argument (null pointer with n > 0, length > max, ...) */
    WTP_EHIP = -2,     /* a HIP runtime call failed */
    WTP_ENOMEM = -3,   /* device or pinned allocation failed */
    WTP_ENODEV = -4    /* no usable gfx950 device */
} wtp_status;

/* Library version string. */
const char *wtp_version(void);

/* Message for the calling thread's last failure ("" if none). */
const char *wtp_last_error(void);

/* Kernel instantiation the calling thread's last launch used, e.g.
   "k_fixed_braid<6, 0, CrcHoldBEpi>" ("" if none).  Diagnostics: bench.py names the
   kernel its roofline measures with it. */
const char *wtp_last_kernel(void);

/* Number of visible HIP devices (0 when none). Does not create a context. */
int wtp_device_count(void);

/* Build the per-device constant tables for `device` now (they are otherwise built
   lazily on first use).  Call before capturing a launch into a hipGraph. */
int wtp_init(int device);

/* Leave `ncus` compute units of `device` free of the library's persistent kernels
   (0 <= ncus < the device's CUs; 0, the default, uses all).  For callers that overlap
   RCCL collectives with CRC launches, e.g. the gather of one batch's results with the
   next batch: a braided workgroup holds all of its CU's LDS, so a collective's
   workgroups can only start on CUs the launch leaves free.  Affects later launches on
   that device from any thread. */
int wtp_reserve_cus(int device, int ncus);

/* Sticky device-side flags of `device`.  Data errors: bit 0, a general-kernel payload
   length was > WTP_MAX_KERNEL_LEN (that payload's result is then 0 / not ok); bit 2, see
   wtp_crc32_verify_batch.  Informational: bit 3, the stream kernel met payloads that
   were not packed (or >= 4096 B) and computed them on its slower per-payload path
   (results exact).  Synchronous; clears the flags when `clear` != 0. */
int wtp_device_status(int device, uint32_t *flags, int clear);

/* ---- CPU reference semantics (single packet) --------------------------------------
   Replaces crc32() of cpp/src/common/Crc32.hpp:91-102 for single packets and 0-byte
   ACK payloads (Sender::isAckValid, cpp/src/base/Sender.cpp:235-237).  Pure C++
   byte-at-a-time table loop; thread-safe. */
uint32_t wtp_crc32(const void *buf, size_t size);

/* ---- device-resident batches (the hot path) ---------------------------------------
   Sender packet build, batched: payload i = d_payloads[i*stride .. i*stride+len).
   Replaces the per-chunk crc32 of Packet(DATA, chunk, seq) in the send loop
   (cpp/src/base/Sender.cpp:88-95 -> Packet.cpp:13).  Fast path (braided CDNA4
   kernel): base % 16 == 0, stride % 16 == 0, len % 16 == 0, 16 <= len <= 1536,
   stride <= 16384; other shapes run the general kernel (len <= WTP_MAX_KERNEL_LEN). */
int wtp_crc32_batch_fixed(const void *d_payloads, size_t stride, size_t len, size_t n,
                          uint32_t *d_out, void *stream);

/* Mixed lengths: payload i = d_base[d_offsets[i] .. d_offsets[i] + d_lengths[i]), any
   order, overlaps allowed.  `base_bytes` = size of the d_base buffer (bounds for the
   loads).  Buffers below 2 GiB run the general (piece-stream) kernel; larger ones take
   the route of wtp_crc32_batch_packed there (the piece kernel in device-cut < 2 GiB
   sub-launches, and the stream kernel, 64-bit offsets, for batches whose offsets turn
   out not to be packed), so there is no size limit.  d_lengths[i] <= WTP_MAX_KERNEL_LEN. */
int wtp_crc32_batch_var(const void *d_base, size_t base_bytes, const uint64_t *d_offsets,
                        const uint32_t *d_lengths, size_t n, uint32_t *d_out, void *stream);

/* Mixed lengths stored back to back (a receive buffer, a record file):
   d_offsets[i+1] == d_offsets[i] + d_lengths[i] (offsets = exclusive prefix sum of the
   lengths, any first offset).  The stream kernel: each wave hashes its region
   of the byte stream once and reads every payload's CRC off prefix values (no per-
   payload windows, masks or padding).  No limit on base_bytes (64-bit offsets) or n.
   Payloads that break the packing, or are longer than 4095 B, are still computed
   exactly on a slower lane-per-payload path, so results are correct for any offsets;
   lengths > WTP_MAX_KERNEL_LEN give crc 0 and set the status flag.
   The library picks the kernel: below 2 GiB the general kernel, the faster one on
   packed batches too (C5: DESIGN.md), so this call then equals wtp_crc32_batch_var; at
   or above 2 GiB the general kernel in sub-launches over < 2 GiB views that the device
   cuts from the offsets; a sub-launch that meets a payload outside its
   view (offsets not packed) flags it and the stream kernel then recomputes the batch,
   so results stay exact for any offsets.  That route keeps its descriptors in device
   scratch: 32 KiB per stream outside graph capture (made on the stream's first such
   call); a call captured into a graph takes one of 64 slots made at init, its own for
   the life of the process, so graphs captured on one stream may be replayed
   concurrently; with every slot taken a captured call runs the stream kernel (exact).
   WTP_STREAM_KERNEL=1 in the environment forces the stream kernel. */
int wtp_crc32_batch_packed(const void *d_base, size_t base_bytes, const uint64_t *d_offsets,
                           const uint32_t *d_lengths, size_t n, uint32_t *d_out, void *stream);

/* Receiver verify, batched (cpp/src/base/Receiver.cpp:25-35 + :203-206): datagram i is
   d_dgrams[i*stride .. i*stride + d_recv_len[i]) = 16-B big-endian PacketHeader ||
   payload.  As in the reference, the CRC covers bytes [16, recv_len) and
   header.length is ignored.  d_ok[i] = 1 iff 16 <= recv_len <= stride and
   ntohl(header.checksum) == crc32(payload), else 0 (drop, no ACK).  A recv_len
   above stride (more than the ring slot holds; recvfrom cannot return it) is
   malformed: ok 0.  d_crc_out may be NULL; otherwise it receives the computed CRCs
   (0 for runts and malformed lengths).  Fast path: a 16-B aligned ring with
   stride % 16 == 0 (e.g. 1472 = header + 1456, or wReceiver's 1504-B slots holding the
   reference's 1500-B receive buffer) runs the braided kernel over the first
   min(stride - 16, 1456) payload bytes of every slot and decides the datagrams of
   exactly that length; in the same launch each workgroup then finishes its other
   datagrams (short, empty, 1473-1500 B, malformed) with the general algorithm.  The
   call uses no memory besides the caller's buffers and keeps no state between calls:
   graph captures, replays on any stream and concurrent calls are independent.  Status
   bit 2 (wtp_device_status): the recv_len array changed while the kernel ran. */
int wtp_crc32_verify_batch(const void *d_dgrams, size_t stride, const uint32_t *d_recv_len,
                           size_t n, uint8_t *d_ok, uint32_t *d_crc_out, void *stream);

/* Fused DATA packet builder (Packet.cpp:9-14,40-47 +
   Sender.cpp:187-197): chunk i = d_payloads[i*1456 ..) of min(1456, total-i*1456)
   bytes -> d_wire[i*wire_stride ..) = htonl{type=2, seq0+i, len, crc} || payload.
   wire_stride >= 16 + 1456.  d_wire_len[i] (may be NULL) = 16 + len. */
int wtp_build_data_packets(const void *d_payloads, size_t total_bytes, uint32_t seq0,
                           void *d_wire, size_t wire_stride, uint32_t *d_wire_len,
                           void *stream);

/* ---- host-memory wrappers (library-owned pinned staging, synchronous) -------------- */

/* Like wtp_crc32_batch_fixed but payloads and results live in host memory. */
int wtp_crc32_host_batch_fixed(const void *h_payloads, size_t stride, size_t len, size_t n,
                               uint32_t *h_out);

/* The wSender path (cpp/src/base/Sender.cpp:82-92): CRC of every `chunk`-byte chunk of
   a host buffer (last chunk may be short).  Pipelined: pinned H2D -> CRC -> D2H,
   double-buffered on two HIP streams.  h_out needs ceil(nbytes/chunk) entries. */
int wtp_crc32_host_chunked(const void *h_buf, size_t nbytes, size_t chunk, uint32_t *h_out);

/* wtp_crc32_host_chunked over several GPUs of this process: the chunks split into ndev
   contiguous ranges, one pinned pipeline (and PCIe link, and staging thread) per device,
   results written straight into h_out (chunks are independent, Crc32.hpp:92-96: no
   collective).  devices = NULL means devices 0 .. ndev-1; ndev <= 0 means every
   visible device.  The calling thread's current device is unchanged on return. */
int wtp_crc32_host_chunked_multi(const void *h_buf, size_t nbytes, size_t chunk, uint32_t *h_out,
                                 const int *devices, int ndev);

/* The wReceiver path, host buffers: same semantics as wtp_crc32_verify_batch.  When the
   ring and recv_len both live in page-locked memory (wtp_host_alloc) and the ring is at
   most 4 MiB, the kernel reads them in place (one launch + one sync per call); other
   batches go through the library's pinned double-buffered copy pipeline.
   WTP_HOST_ZEROCOPY=0 in the environment forces the pipeline. */
int wtp_crc32_host_verify(const void *h_dgrams, size_t stride, const uint32_t *h_recv_len,
                          size_t n, uint8_t *h_ok, uint32_t *h_crc_out);

/* The fused builder from and to host memory (wSender --crc gpu): same layout as
   wtp_build_data_packets; the bytes of a wire slot past its datagram are unspecified.
   Pinned (wtp_host_alloc) payloads and wire buffers move by DMA directly, others through
   the library's pinned slabs; synchronous. */
int wtp_host_build_data_packets(const void *h_payloads, size_t total_bytes, uint32_t seq0,
                                void *h_wire, size_t wire_stride, uint32_t *h_wire_len);

/* Pinned (page-locked) host allocation for zero-copy staging, e.g. wSender reads its
   input file straight into such a buffer.  NULL on failure. */
void *wtp_host_alloc(size_t bytes);
void wtp_host_free(void *p);

/* ---- synthetic inputs (bench / tests) ------------------------------
   d_out[i] = byte (start_byte+i) of the splitmix64 stream for `seed`:
   byte g = (mix64(seed + ((g>>3)+1)*0x9E3779B97F4A7C15) >> (8*(g&7))) & 0xFF. */
int wtp_synth_fill(void *d_out, uint64_t start_byte, size_t nbytes, uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* WTP_CRC32_H */
