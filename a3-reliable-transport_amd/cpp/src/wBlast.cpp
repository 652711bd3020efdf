// wBlast.cpp — UDP traffic generator for the batched-receive measurement (SURVEY.md
// §8f row 2).  Not part of the WTP protocol: it pre-builds DATA datagrams (16-B
// big-endian PacketHeader || payload, Packet.cpp:40-47) from a file or from the
// synthetic generator and sends them with sendmmsg, cycling, for a fixed time.
//
//   wBlast -h <host> -p <port> [-i <file>] [--seconds S] [--batch N] [--corrupt K]
//
// --corrupt K flips one payload bit in every K-th datagram (the receiver must drop
// exactly those).  Prints one JSON line with what was sent.
#include <time.h>

#include <fstream>
#include <iostream>
#include <iterator>

#include "common/Endpoint.hpp"

using namespace wtp;

namespace {
double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return double(t.tv_sec) + 1e-9 * double(t.tv_nsec);
}
// Byte g of the splitmix64 stream (seed 0x5EED), the same generator as wtp_synth_fill.
uint8_t synth_byte(uint64_t g) {
    uint64_t z = 0x5EEDull + ((g >> 3) + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return uint8_t(z >> (8 * (g & 7)));
}
}  // namespace

int main(int argc, char **argv) {
    try {
        Args a(argc, argv, {{"-h", "host"}, {"-p", "port"}, {"-i", "input"}, {"--seconds", "seconds"},
                            {"--batch", "batch"}, {"--corrupt", "corrupt"}});
        const int port = std::stoi(a.get("port", "0"));
        if (port <= 0 || port > 65535 || !a.has("host")) {
            std::cerr << "usage: wBlast -h <host> -p <port> [-i <file>] [--seconds S] [--batch N] [--corrupt K]\n";
            return 1;
        }
        std::vector<uint8_t> data;
        if (a.has("input")) {
            std::ifstream f(a.get("input"), std::ios::binary);
            if (!f) throw std::runtime_error("cannot open " + a.get("input"));
            data.assign(std::istreambuf_iterator<char>(f), {});
        } else {
            data.resize(kMaxPayload * 4096);
            for (size_t g = 0; g < data.size(); ++g) data[g] = synth_byte(g);
        }
        const size_t nch = (data.size() + kMaxPayload - 1) / kMaxPayload;
        if (!nch) throw std::runtime_error("empty input");
        const uint64_t corrupt = std::stoull(a.get("corrupt", "0"));
        std::vector<uint8_t> wire(nch * kMaxDatagram);
        std::vector<uint32_t> wlen(nch);
        for (size_t i = 0; i < nch; ++i) {
            const uint32_t len = uint32_t(std::min(kMaxPayload, data.size() - i * kMaxPayload));
            const uint8_t *p = data.data() + i * kMaxPayload;
            wlen[i] = uint32_t(make_datagram(wire.data() + i * kMaxDatagram, DATA, uint32_t(i), p, len, crc32(p, len)));
            if (corrupt && i % corrupt == 0 && len) wire[i * kMaxDatagram + kHeaderBytes + (i % len)] ^= 0x20;
        }
        const size_t batch = size_t(std::stoul(a.get("batch", "64")));
        const double seconds = std::stod(a.get("seconds", "2"));
        int fd = udp_socket();
        int big = 16 << 20;
        setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
        sockaddr_in to = addr_of(a.get("host"), port);
        std::vector<iovec> iov(batch);
        std::vector<mmsghdr> msg(batch);
        uint64_t sent = 0, bytes = 0, bad = 0;
        size_t next = 0;
        const double t0 = now_s();
        double t = t0;
        while (t - t0 < seconds) {
            for (size_t k = 0; k < batch; ++k) {
                const size_t i = (next + k) % nch;
                iov[k] = {wire.data() + i * kMaxDatagram, wlen[i]};
                msg[k].msg_hdr = {};
                msg[k].msg_hdr.msg_name = &to;
                msg[k].msg_hdr.msg_namelen = sizeof to;
                msg[k].msg_hdr.msg_iov = &iov[k];
                msg[k].msg_hdr.msg_iovlen = 1;
            }
            const int n = ::sendmmsg(fd, msg.data(), unsigned(batch), 0);
            if (n > 0) {
                for (int k = 0; k < n; ++k) {
                    const size_t i = (next + size_t(k)) % nch;
                    bytes += wlen[i] - kHeaderBytes;
                    bad += (corrupt && i % corrupt == 0 && wlen[i] > kHeaderBytes) ? 1 : 0;
                }
                sent += uint64_t(n);
                next = (next + size_t(n)) % nch;
            }
            t = now_s();
        }
        ::close(fd);
        std::printf("{\"sent\": %llu, \"payload_bytes\": %llu, \"seconds\": %.4f, \"GBps\": %.4f, \"corrupted\": %llu}\n",
                    (unsigned long long)sent, (unsigned long long)bytes, t - t0, double(bytes) / (t - t0) / 1e9,
                    (unsigned long long)bad);
        return 0;
    } catch (const std::exception &e) {
        std::cerr << "wBlast: " << e.what() << "\n";
        return 1;
    }
}
