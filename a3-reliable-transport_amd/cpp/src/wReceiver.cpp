// wReceiver.cpp — WTP receiver, config C1 plumbing around the CRC path.
//
//   wReceiver -p <port> -w <window> -d <output-dir> -o <log> [--crc cpu|gpu] [--once]
//
// Reference behaviour (README.md:98-127, cpp/src/base/Receiver.cpp): one connection at a
// time (START of another connection is ignored while one is open), DATA with a bad
// checksum or seqNum >= expected + window is dropped without an ACK, every accepted
// packet gets a cumulative ACK carrying the next expected seqNum, START/END are ACKed
// with their own seqNum, and connection i is stored as <output-dir>/FILE-i.out.
//
// Checksum verify follows Receiver.cpp:25-35,203-206: the CRC covers datagram bytes
// [16, recv_len) — header.length is not trusted — and is compared with the header's
// checksum; with --crc gpu it runs on the MI355X (wtp_crc32_host_verify).
// Deliberate differences from the reference: buffered
// out-of-order packets are flushed in order, the file goes to -d (not the CWD), ACKs
// are 16-byte datagrams.  --once exits after the first completed connection (tests).
#include <fstream>
#include <iostream>

#include "common/Endpoint.hpp"

using namespace wtp;

int main(int argc, char **argv) {
    try {
        Args a(argc, argv, {{"-p", "port"}, {"--port", "port"}, {"-w", "window"}, {"--window-size", "window"},
                            {"-d", "dir"}, {"--output-dir", "dir"}, {"-o", "log"}, {"--output-log", "log"},
                            {"--crc", "crc"}, {"--once", "flag:once"}});
        const int port = std::stoi(a.get("port", "0"));
        const uint32_t window = uint32_t(std::stoi(a.get("window", "0")));
        if (port <= 0 || port > 65535 || window == 0 || !a.has("dir")) {
            std::cerr << "usage: wReceiver -p <port> -w <window> -d <dir> -o <log> [--crc cpu|gpu] [--once]\n";
            return 1;
        }
        Checksums crc(a.get("crc", "cpu"));
        Log log(a.get("log"));

        int fd = udp_socket();
        sockaddr_in me = addr_of("0.0.0.0", port);
        if (::bind(fd, reinterpret_cast<sockaddr *>(&me), sizeof me) < 0) throw std::runtime_error("bind failed");

        bool open = false;
        uint32_t start_seq = 0, expected = 0;
        int file_no = 0;
        std::ofstream out;
        std::map<uint32_t, std::vector<uint8_t>> pending;  // out-of-order DATA
        uint8_t buf[2048];

        for (;;) {
            sockaddr_in peer{};
            socklen_t plen = sizeof peer;
            const ssize_t n = ::recvfrom(fd, buf, sizeof buf, 0, reinterpret_cast<sockaddr *>(&peer), &plen);
            if (n < ssize_t(kHeaderBytes)) continue;
            if (!crc.verify(buf, size_t(n))) continue;  // corrupted: drop, no ACK, no log
            const PacketHeader h = get_header(buf);
            log.pkt(h);

            uint32_t ack_seq;
            if (h.type == START) {
                if (open && h.seqNum != start_seq) continue;  // another sender mid-connection
                if (!open) {
                    open = true;
                    start_seq = h.seqNum;
                    expected = 0;
                    pending.clear();
                    out.open(a.get("dir") + "/FILE-" + std::to_string(file_no) + ".out", std::ios::binary | std::ios::trunc);
                }
                ack_seq = h.seqNum;
            } else if (h.type == END) {
                if (h.seqNum != start_seq) continue;
                if (!open) {  // duplicate END of the connection just closed: re-ACK it
                    uint8_t ack[kHeaderBytes];
                    make_datagram(ack, ACK, h.seqNum, nullptr, 0, crc32(nullptr, 0));
                    ::sendto(fd, ack, sizeof ack, 0, reinterpret_cast<sockaddr *>(&peer), plen);
                    log.pkt(get_header(ack));
                    continue;
                }
                ack_seq = h.seqNum;
            } else if (h.type == DATA) {
                if (!open || h.seqNum >= expected + window) continue;  // outside the window: drop
                if (h.seqNum >= expected) pending.emplace(h.seqNum, std::vector<uint8_t>(buf + kHeaderBytes, buf + n));
                for (auto it = pending.find(expected); it != pending.end(); it = pending.find(expected)) {
                    out.write(reinterpret_cast<const char *>(it->second.data()), std::streamsize(it->second.size()));
                    pending.erase(it);
                    ++expected;
                }
                ack_seq = expected;
            } else {
                continue;
            }
            uint8_t ack[kHeaderBytes];
            make_datagram(ack, ACK, ack_seq, nullptr, 0, crc32(nullptr, 0));
            ::sendto(fd, ack, sizeof ack, 0, reinterpret_cast<sockaddr *>(&peer), plen);
            log.pkt(get_header(ack));

            if (h.type == END) {
                out.close();
                open = false;
                ++file_no;
                if (a.has("once")) break;
            }
        }
        ::close(fd);
        return 0;
    } catch (const std::exception &e) {
        std::cerr << "wReceiver: " << e.what() << "\n";
        return 1;
    }
}
