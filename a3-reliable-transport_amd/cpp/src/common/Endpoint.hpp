// Endpoint.hpp — shared plumbing of the WTP endpoints (wSender / wReceiver): argument
// parsing for the spec'd flags (README.md:83-89, 120-125), the per-packet log line
// `<type> <seqNum> <length> <checksum>` (README.md:93-99), UDP sockets, and the checksum
// engine that routes whole batches to the MI355X library (--crc gpu) or to the CPU
// crc32() of Crc32.hpp (--crc cpu, the reference's behaviour).
#pragma once

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "Crc32.hpp"
#include "PacketHeader.hpp"

namespace wtp {

struct Args {
    std::map<std::string, std::string> kv;
    Args(int argc, char **argv, const std::map<std::string, std::string> &alias) {
        for (int i = 1; i < argc; ++i) {
            std::string k = argv[i];
            auto it = alias.find(k);
            if (it == alias.end()) throw std::runtime_error("unknown argument " + k);
            if (it->second.rfind("flag:", 0) == 0) {
                kv[it->second.substr(5)] = "1";
                continue;
            }
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + k);
            kv[it->second] = argv[++i];
        }
    }
    std::string get(const std::string &k, const std::string &def = "") const {
        auto it = kv.find(k);
        return it == kv.end() ? def : it->second;
    }
    bool has(const std::string &k) const { return kv.count(k) != 0; }
};

class Log {
   public:
    explicit Log(const std::string &path) : f_(path.empty() ? nullptr : std::fopen(path.c_str(), "w")) {}
    ~Log() {
        if (f_) std::fclose(f_);
    }
    void pkt(const PacketHeader &h) {
        if (f_) {
            std::fprintf(f_, "%u %u %u %u\n", h.type, h.seqNum, h.length, h.checksum);
            std::fflush(f_);
        }
    }

   private:
    FILE *f_;
};

// Checksums for whole batches.  GPU mode goes through the C-ABI; CPU mode is the
// reference's one-call-per-packet crc32().
class Checksums {
   public:
    // Receiver batches of at most this many payload bytes are verified on the CPU in GPU
    // mode (crc32_fast): below it one GPU call (launch + sync + PCIe, ~21 us from C++)
    // costs more than hashing the bytes here.  Measured crossover on the MI355X box:
    // DESIGN.md 5 (tools/verify_crossover.cpp); WTP_VERIFY_CPU_MAX_BYTES overrides it
    // (0 = always the GPU).
    static constexpr size_t kCpuVerifyMaxBytes = 64 * 1024;

    // gpus: devices the sender spreads its file over (0 = every visible device).
    explicit Checksums(const std::string &mode, int gpus = 1)
        : gpu_(mode == "gpu"), gpus_(gpus), cpu_max_(cpu_max_from_env()) {
        if (mode != "gpu" && mode != "cpu") throw std::runtime_error("--crc must be cpu or gpu");
        if (gpu_ && wtp_init(0) != WTP_OK) throw std::runtime_error(std::string("GPU CRC unavailable: ") + wtp_last_error());
    }
    bool gpu() const { return gpu_; }
    size_t cpu_verify_max_bytes() const { return cpu_max_; }

    // Sender build: crc of every kMaxPayload chunk of the file (Sender.cpp:88-92).  With
    // several GPUs the chunks split into one contiguous range per device (one PCIe link
    // each); a pinned buffer (wtp_host_alloc) is copied to the devices without staging.
    std::vector<uint32_t> chunks(const uint8_t *buf, size_t n) const {
        const size_t nch = (n + kMaxPayload - 1) / kMaxPayload;
        std::vector<uint32_t> out(nch);
        if (!nch) return out;
        if (gpu_ && gpus_ != 1) {
            if (wtp_crc32_host_chunked_multi(buf, n, kMaxPayload, out.data(), nullptr, gpus_) != WTP_OK)
                throw std::runtime_error(std::string("wtp_crc32_host_chunked_multi: ") + wtp_last_error());
        } else if (gpu_) {
            if (wtp_crc32_host_chunked(buf, n, kMaxPayload, out.data()) != WTP_OK)
                throw std::runtime_error(std::string("wtp_crc32_host_chunked: ") + wtp_last_error());
        } else {
            for (size_t i = 0; i < nch; ++i) out[i] = crc32(buf + i * kMaxPayload, std::min(kMaxPayload, n - i * kMaxPayload));
        }
        return out;
    }

    // Batched receiver verify (Receiver.cpp:25-35,203-206): datagram
    // i = ring[i*stride, +rl[i]), ok[i] = its CRC over bytes [16, rl[i]) equals the
    // header's checksum.  GPU mode sends the batch to the MI355X in one call when it
    // carries more than cpu_verify_max_bytes() of payload, and hashes it here with
    // crc32_fast otherwise (the window-size batches of config C1); CPU mode is the
    // reference's one byte-loop crc32() per datagram.  All routes give the same ok[].
    // Returns true if the batch went to the GPU.
    bool verify_batch(const uint8_t *ring, size_t stride, const uint32_t *rl, size_t n, uint8_t *ok) const {
        if (!n) return false;
        if (gpu_ && payload_bytes(stride, rl, n) > cpu_max_) {
            if (wtp_crc32_host_verify(ring, stride, rl, n, ok, nullptr) != WTP_OK)
                throw std::runtime_error(std::string("wtp_crc32_host_verify: ") + wtp_last_error());
            return true;
        }
        for (size_t i = 0; i < n; ++i) {
            const uint8_t *d = ring + i * stride;
            const bool shaped = rl[i] >= kHeaderBytes && rl[i] <= stride;
            ok[i] = shaped && get_header(d).checksum == (gpu_ ? crc32_fast(d + kHeaderBytes, rl[i] - kHeaderBytes)
                                                              : crc32(d + kHeaderBytes, rl[i] - kHeaderBytes));
        }
        return false;
    }

   private:
    static size_t payload_bytes(size_t stride, const uint32_t *rl, size_t n) {
        size_t b = 0;
        for (size_t i = 0; i < n; ++i) b += rl[i] > kHeaderBytes ? std::min<size_t>(rl[i], stride) - kHeaderBytes : 0;
        return b;
    }
    // WTP_VERIFY_CPU_MAX_BYTES: a plain decimal byte count (0 = every batch to the GPU).
    // Anything else ("64K", "abc", out of range) is rejected: strtoull would read it as 0,
    // which is a valid setting, so a typo would silently send every batch to the GPU.
    static size_t cpu_max_from_env() {
        const char *e = std::getenv("WTP_VERIFY_CPU_MAX_BYTES");
        if (!e || !*e) return kCpuVerifyMaxBytes;
        char *end = nullptr;
        errno = 0;
        const unsigned long long v = std::strtoull(e, &end, 10);
        // the first character must be a digit: strtoull skips any leading whitespace and sign
        if (errno != 0 || end == e || *end != '\0' || !std::isdigit(static_cast<unsigned char>(*e)))
            throw std::invalid_argument(std::string("WTP_VERIFY_CPU_MAX_BYTES: not a decimal byte count: '") + e + "'");
        return size_t(v);
    }
    bool gpu_;
    int gpus_;
    size_t cpu_max_;
};

// Receive ring for recvmmsg: `slots` datagram slots of kSlot = 1504 bytes in pinned host
// memory (wtp_host_alloc), filled by one recvmmsg call per batch.  Each slot receives
// into kRecv = 1500 bytes, the reference's `char buffer[1500]` (Receiver.cpp:123-125):
// a longer datagram is truncated to 1500 bytes exactly as recvfrom truncates it there,
// and its recv_len is 1500, so verify CRCs the same bytes the reference does.  The slot
// stride is rounded up to a multiple of 16 so the verify kernel's braided fast path takes
// the ring (it decides the 1472-B WTP DATA datagrams; other lengths go to its fix-up pass).
class RecvRing {
   public:
    static constexpr size_t kRecv = 1500;  // Receiver.cpp:123 char buffer[1500]
    static constexpr size_t kSlot = 1504;  // kRecv rounded up to 16
    // pinned: allocate the ring and its recv_len array with wtp_host_alloc (GPU verify:
    // batches up to 4 MiB are read by the kernel in place, larger ones take one DMA per
    // slab); otherwise plain page-aligned memory (CPU verify needs no device).
    RecvRing(size_t slots, bool pinned)
        : n_(slots), buf_(alloc<uint8_t>(slots * kSlot, pinned)), len_(alloc<uint32_t>(slots * 4, pinned)),
          ok_(slots), iov_(slots), msg_(slots), peer_(slots) {
        for (size_t i = 0; i < n_; ++i) {
            iov_[i] = {buf_.get() + i * kSlot, kRecv};
            msg_[i].msg_hdr.msg_iov = &iov_[i];
            msg_[i].msg_hdr.msg_iovlen = 1;
        }
    }
    RecvRing(const RecvRing &) = delete;
    RecvRing &operator=(const RecvRing &) = delete;

    // Block for at least one datagram, take up to `slots` (MSG_WAITFORONE).  Returns the
    // count; 0 on timeout (SO_RCVTIMEO) or EINTR.
    size_t receive(int fd) {
        for (size_t i = 0; i < n_; ++i) {
            msg_[i].msg_hdr.msg_name = &peer_[i];
            msg_[i].msg_hdr.msg_namelen = sizeof(sockaddr_in);
            msg_[i].msg_hdr.msg_flags = 0;
        }
        const int got = ::recvmmsg(fd, msg_.data(), unsigned(n_), MSG_WAITFORONE, nullptr);
        if (got <= 0) return 0;
        for (int i = 0; i < got; ++i) len_.get()[i] = uint32_t(msg_[i].msg_len);  // <= kRecv (truncated like recvfrom)
        return size_t(got);
    }
    uint8_t *slot(size_t i) { return buf_.get() + i * kSlot; }
    uint32_t len(size_t i) const { return len_.get()[i]; }
    const uint32_t *lens() const { return len_.get(); }
    uint8_t *ok() { return ok_.data(); }
    const sockaddr_in &peer(size_t i) const { return peer_[i]; }
    uint8_t *ring() { return buf_.get(); }

   private:
    // Each allocation is owned as soon as it exists, so a failure of the second one (or
    // of anything later in the constructor) frees the first: pinned memory does not leak.
    struct Free {
        bool pinned;
        void operator()(void *p) const {
            if (pinned)
                wtp_host_free(p);
            else
                std::free(p);
        }
    };
    template <class T>
    using Owned = std::unique_ptr<T, Free>;
    template <class T>
    static Owned<T> alloc(size_t bytes, bool pinned) {
        void *p = pinned ? wtp_host_alloc(bytes) : std::aligned_alloc(4096, (bytes + 4095) & ~size_t(4095));
        if (!p) throw std::runtime_error("receive ring allocation failed");
        return Owned<T>(static_cast<T *>(p), Free{pinned});
    }
    size_t n_;
    Owned<uint8_t> buf_;
    Owned<uint32_t> len_;  // recv_len per slot (pinned with the ring)
    std::vector<uint8_t> ok_;
    std::vector<iovec> iov_;
    std::vector<mmsghdr> msg_;
    std::vector<sockaddr_in> peer_;
};

inline int udp_socket() {
    int fd = ::socket(AF_INET, SOCK_DGRAM, 0);
    if (fd < 0) throw std::runtime_error("socket() failed");
    return fd;
}

inline void set_rcv_timeout_ms(int fd, int ms) {
    timeval tv{ms / 1000, (ms % 1000) * 1000};
    if (setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv) < 0) throw std::runtime_error("setsockopt failed");
}

inline sockaddr_in addr_of(const std::string &host, int port) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(uint16_t(port));
    if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) throw std::runtime_error("bad IPv4 address " + host);
    return a;
}

// Build one datagram (header htonl'd, Packet.cpp:40-47 / Sender.cpp:189-194).
inline size_t make_datagram(uint8_t *wire, uint32_t type, uint32_t seq, const uint8_t *payload, uint32_t len,
                            uint32_t checksum) {
    put_header(wire, PacketHeader{type, seq, len, checksum});
    if (len) std::memcpy(wire + kHeaderBytes, payload, len);
    return kHeaderBytes + len;
}

}  // namespace wtp
