// wSender.cpp — WTP sender (go-back-N), config C1 plumbing around the CRC path.
//
//   wSender -h <ip> -p <port> -w <window> -i <input> -o <log> [--crc cpu|gpu] [--gpus N]
//
// Reference behaviour (mmheyer/a3-reliable-transport README.md:62-127, cpp/src/base/
// Sender.cpp): START with a random seqNum until ACKed, DATA seqNums from 0 in chunks of
// 1456 B, cumulative ACKs, a 500 ms timer that resends the whole window when it does not
// advance, END with the START seqNum until ACKed.
//
// The checksum path is the one this repository accelerates: the whole file is read up
// front (as Sender.cpp:82 does; into pinned memory with --crc gpu).  With --crc gpu on one
// device every DATA datagram — header and CRC included (Sender.cpp:187-197) — is built in
// ONE fused pass by wtp_host_build_data_packets into a pinned wire buffer, and sending is
// a pointer into it.  With --gpus N (0 = all) every chunk's CRC is computed in one batch by
// wtp_crc32_host_chunked_multi, and with --crc cpu by the reference's per-packet crc32();
// those two paths write the header per send.  Retransmissions resend the same bytes.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <memory>
#include <random>
#include <vector>

#include "common/Endpoint.hpp"

using namespace wtp;
using Clock = std::chrono::steady_clock;

namespace {

// The input file in one buffer: pinned (wtp_host_alloc) for the GPU path, else heap.
class InputFile {
   public:
    InputFile(const std::string &path, bool pinned) : pinned_(pinned) {
        std::FILE *f = std::fopen(path.c_str(), "rb");
        if (!f) throw std::runtime_error("cannot open " + path);
        long sz = -1;
        if (std::fseek(f, 0, SEEK_END) == 0) {
            sz = std::ftell(f);
            if (std::fseek(f, 0, SEEK_SET) != 0) sz = -1;
        }
        bool ok;
        if (sz >= 0) {  // a regular file: one read into a buffer of its size
            n_ = size_t(sz);
            p_ = alloc(n_);
            ok = p_ && std::fread(p_, 1, n_, f) == n_;
        } else {  // a pipe, /dev/stdin, process substitution: read until EOF
            std::vector<uint8_t> v;
            uint8_t buf[1 << 16];
            size_t got;
            while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + got);
            ok = !std::ferror(f);
            n_ = v.size();
            p_ = alloc(n_);
            ok = ok && p_;
            if (ok && n_) std::memcpy(p_, v.data(), n_);
        }
        std::fclose(f);
        if (!ok) {
            release();
            throw std::runtime_error("cannot read " + path);
        }
    }
    ~InputFile() { release(); }
    InputFile(const InputFile &) = delete;
    InputFile &operator=(const InputFile &) = delete;
    const uint8_t *data() const { return p_; }
    size_t size() const { return n_; }

   private:
    uint8_t *alloc(size_t n) const {
        return static_cast<uint8_t *>(pinned_ ? wtp_host_alloc(n) : std::malloc(n ? n : 1));
    }
    void release() {
        if (pinned_)
            wtp_host_free(p_);
        else
            std::free(p_);
        p_ = nullptr;
    }
    bool pinned_;
    uint8_t *p_ = nullptr;
    size_t n_ = 0;
};

// Every DATA datagram of the file in one pinned buffer, slot i = [i*kSlot, +len(i)),
// built on the device by the fused builder (--crc gpu on one device).
class WireBuffer {
   public:
    static constexpr size_t kSlot = kHeaderBytes + kMaxPayload;  // 1472 = 92 * 16: the braided path
    explicit WireBuffer(const InputFile &file) : n_((file.size() + kMaxPayload - 1) / kMaxPayload) {
        if (!n_) return;
        p_ = static_cast<uint8_t *>(wtp_host_alloc(n_ * kSlot));
        if (!p_) throw std::runtime_error("cannot pin the wire buffer");
        if (wtp_host_build_data_packets(file.data(), file.size(), 0, p_, kSlot, nullptr) != WTP_OK) {
            wtp_host_free(p_);
            throw std::runtime_error(std::string("wtp_host_build_data_packets: ") + wtp_last_error());
        }
    }
    ~WireBuffer() { wtp_host_free(p_); }
    WireBuffer(const WireBuffer &) = delete;
    WireBuffer &operator=(const WireBuffer &) = delete;
    const uint8_t *slot(uint32_t i) const { return p_ + size_t(i) * kSlot; }
    size_t count() const { return n_; }

   private:
    size_t n_;
    uint8_t *p_ = nullptr;
};

struct Conn {
    int fd;
    sockaddr_in peer;
    Log &log;

    void send(const uint8_t *wire, size_t n) {
        ::sendto(fd, wire, n, 0, reinterpret_cast<const sockaddr *>(&peer), sizeof peer);
        log.pkt(get_header(wire));
    }
    // Returns true and the ACK header if a valid ACK arrived before the socket timeout.
    bool recv_ack(PacketHeader &h) {
        uint8_t buf[2048];
        ssize_t n = ::recvfrom(fd, buf, sizeof buf, 0, nullptr, nullptr);
        if (n < ssize_t(kHeaderBytes)) return false;
        h = get_header(buf);
        // ACKs carry no payload; crc32 of an empty payload is 0 (Sender.cpp:235-237)
        if (h.type != ACK || h.checksum != crc32(buf + kHeaderBytes, 0)) return false;
        log.pkt(h);
        return true;
    }
};

// Send a control packet until its ACK (seqNum == seq) arrives.
bool control(Conn &c, uint32_t type, uint32_t seq, int max_tries) {
    uint8_t wire[kHeaderBytes];
    make_datagram(wire, type, seq, nullptr, 0, crc32(nullptr, 0));
    for (int t = 0; t < max_tries; ++t) {
        c.send(wire, sizeof wire);
        const auto deadline = Clock::now() + std::chrono::milliseconds(500);
        PacketHeader h;
        while (Clock::now() < deadline) {
            if (c.recv_ack(h) && h.seqNum == seq) return true;
        }
    }
    return false;
}

}  // namespace

int main(int argc, char **argv) {
    try {
        Args a(argc, argv, {{"-h", "host"}, {"--hostname", "host"}, {"-p", "port"}, {"--port", "port"},
                            {"-w", "window"}, {"--window-size", "window"}, {"-i", "input"}, {"--input-file", "input"},
                            {"-o", "log"}, {"--output-log", "log"}, {"--crc", "crc"}, {"--gpus", "gpus"}});
        const int port = std::stoi(a.get("port", "0"));
        const int window = std::stoi(a.get("window", "0"));
        if (port <= 0 || port > 65535 || window <= 0 || !a.has("host") || !a.has("input")) {
            std::cerr << "usage: wSender -h <ip> -p <port> -w <window> -i <input> -o <log> [--crc cpu|gpu] [--gpus N]\n";
            return 1;
        }
        Checksums crc(a.get("crc", "cpu"), std::stoi(a.get("gpus", "1")));
        Log log(a.get("log"));

        // The whole file up front, as Sender.cpp:82 does; with --crc gpu straight into
        // pinned memory, so the CRC pipeline DMAs it to the device without staging.
        const InputFile file(a.get("input"), crc.gpu());

        // Every DATA datagram built on the device (--crc gpu, one device), else every DATA
        // checksum in one batch (the device path when --crc gpu --gpus N).  The wire buffer
        // pins a second copy of the file (n * 1472 B); if it cannot be pinned or built, or
        // is larger than WTP_WIRE_MAX_BYTES, the sender falls back to the checksum batch
        // (crc.chunks) and writes each header per send, as with --gpus N.
        bool fused = crc.gpu() && std::stoi(a.get("gpus", "1")) == 1;
        std::unique_ptr<WireBuffer> built;
        std::vector<uint32_t> sums;
        if (fused) {
            const char *cap = std::getenv("WTP_WIRE_MAX_BYTES");
            const size_t wire_bytes = ((file.size() + kMaxPayload - 1) / kMaxPayload) * WireBuffer::kSlot;
            try {
                if (cap && *cap && wire_bytes > size_t(std::strtoull(cap, nullptr, 10)))
                    throw std::runtime_error("the wire buffer (" + std::to_string(wire_bytes) +
                                             " B) exceeds WTP_WIRE_MAX_BYTES");
                built = std::make_unique<WireBuffer>(file);
            } catch (const std::exception &e) {
                std::cerr << "wSender: fused build unavailable (" << e.what() << "); using the checksum batch\n";
                fused = false;
            }
        }
        if (!fused) sums = crc.chunks(file.data(), file.size());
        const uint32_t nchunks = uint32_t(fused ? built->count() : sums.size());

        Conn c{udp_socket(), addr_of(a.get("host"), port), log};
        set_rcv_timeout_ms(c.fd, 50);

        std::mt19937 gen(std::random_device{}());
        const uint32_t start_seq = std::uniform_int_distribution<uint32_t>(1, 0xFFFFFFFFu)(gen);
        if (!control(c, START, start_seq, 100)) throw std::runtime_error("START was never acknowledged");

        uint8_t wire[kMaxDatagram];
        auto send_chunk = [&](uint32_t i) {
            const size_t off = size_t(i) * kMaxPayload;
            const uint32_t len = uint32_t(std::min(kMaxPayload, file.size() - off));
            if (fused)
                c.send(built->slot(i), kHeaderBytes + len);
            else
                c.send(wire, make_datagram(wire, DATA, i, file.data() + off, len, sums[i]));
        };

        uint32_t base = 0, next = 0;  // window = [base, next)
        auto timer = Clock::now();
        while (base < nchunks) {
            while (next < nchunks && next - base < uint32_t(window)) send_chunk(next++);
            PacketHeader h;
            if (c.recv_ack(h) && h.seqNum > base && h.seqNum <= next) {  // cumulative ACK
                base = h.seqNum;
                timer = Clock::now();
            } else if (Clock::now() - timer >= std::chrono::milliseconds(500)) {
                for (uint32_t s = base; s < next; ++s) send_chunk(s);  // go-back-N
                timer = Clock::now();
            }
        }
        if (!control(c, END, start_seq, 100)) throw std::runtime_error("END was never acknowledged");
        ::close(c.fd);
        std::cout << "sent " << file.size() << " bytes in " << nchunks << " DATA packets (crc " << (crc.gpu() ? "gpu" : "cpu")
                  << ")\n";
        return 0;
    } catch (const std::exception &e) {
        std::cerr << "wSender: " << e.what() << "\n";
        return 1;
    }
}
