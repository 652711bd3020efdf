// wReceiver.cpp — WTP receiver, config C1 plumbing around the CRC path.
//
//   wReceiver -p <port> -w <window> -d <output-dir> -o <log> [--crc cpu|gpu] [--once]
//             [--batch N]
//   wReceiver --bench <seconds> -p <port> [--crc cpu|gpu] [--batch N]
//
// Reference behaviour (README.md:98-127, cpp/src/base/Receiver.cpp): one connection at a
// time (START of another connection is ignored while one is open), DATA with a bad
// checksum or seqNum >= expected + window is dropped without an ACK, every accepted
// packet gets a cumulative ACK carrying the next expected seqNum, START/END are ACKed
// with their own seqNum, and connection i is stored as <output-dir>/FILE-i.out.
//
// Checksum verify follows Receiver.cpp:25-35,123-125,203-206: datagrams are received into
// 1500 bytes (longer ones truncated, as recvfrom into char buffer[1500] does), the CRC
// covers bytes [16, recv_len) — header.length is not trusted — and is compared with the
// header's checksum, for DATA only (START/END are not checked, Receiver.cpp:139-186);
// with --crc gpu it runs on the MI355X (wtp_crc32_host_verify).
// Deliberate differences from the reference: buffered
// out-of-order packets are flushed in order, the file goes to -d (not the CWD), ACKs
// are 16-byte datagrams.  --once exits after the first completed connection (tests).
//
// Batched receive: datagrams arrive through recvmmsg into a pinned
// ring of --batch slots (default: the window size), the whole batch is verified with one
// call (one GPU launch with --crc gpu; batches of at most Checksums::kCpuVerifyMaxBytes
// of payload are hashed on the CPU with crc32_fast instead, where a GPU call's launch and
// sync cost more), then processed in arrival order exactly as one-at-a-time reception
// would.  --bench measures that path alone: it receives DATA datagrams (e.g. from wBlast)
// for the given seconds, verifying each batch on a worker thread while the next one
// arrives, and prints one JSON line with the rate.
#include <time.h>

#include <condition_variable>
#include <fstream>
#include <iostream>
#include <mutex>
#include <thread>

#include "common/Endpoint.hpp"

using namespace wtp;

namespace {

void send_ack(int fd, Log &log, uint32_t seq, const sockaddr_in &peer) {
    uint8_t ack[kHeaderBytes];
    make_datagram(ack, ACK, seq, nullptr, 0, crc32(nullptr, 0));
    ::sendto(fd, ack, sizeof ack, 0, reinterpret_cast<const sockaddr *>(&peer), sizeof peer);
    log.pkt(get_header(ack));
}

double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return double(t.tv_sec) + 1e-9 * double(t.tv_nsec);
}

// Receive + verify throughput (no protocol): prints
// {"datagrams":..,"payload_bytes":..,"seconds":..,"GBps":..,"ok":..,"batches":..,...}
// Two rings alternate: a worker thread verifies batch k (one GPU call with --crc gpu)
// while the main thread receives batch k+1 into the other ring.
int bench(int fd, const Checksums &crc, size_t batch, double seconds) {
    int big = 64 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    set_rcv_timeout_ms(fd, 500);
    RecvRing ring0(batch, crc.gpu()), ring1(batch, crc.gpu());
    RecvRing *rings[2] = {&ring0, &ring1};
    uint64_t dgrams = 0, bytes = 0, good = 0, batches = 0, gpu_batches = 0;
    double t0 = 0, t1 = 0, tverify = 0;

    std::mutex mu;
    std::condition_variable cv;
    RecvRing *job = nullptr;  // batch handed to the worker
    size_t job_n = 0;
    bool busy = false, stop = false;
    std::thread worker([&] {
        for (;;) {
            RecvRing *r;
            size_t n;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return job != nullptr || stop; });
                if (!job) return;
                r = job;
                n = job_n;
            }
            const double tv = now_s();
            const bool on_gpu = crc.verify_batch(r->ring(), RecvRing::kSlot, r->lens(), n, r->ok());
            const double dv = now_s() - tv;
            uint64_t b = 0, g = 0;
            for (size_t i = 0; i < n; ++i) {
                b += r->len(i) > kHeaderBytes ? r->len(i) - kHeaderBytes : 0;
                g += r->ok()[i];
            }
            std::lock_guard<std::mutex> lk(mu);
            tverify += dv;
            dgrams += n;
            bytes += b;
            good += g;
            ++batches;
            gpu_batches += on_gpu ? 1 : 0;
            job = nullptr;
            busy = false;
            cv.notify_all();
        }
    });
    for (int k = 0;; k ^= 1) {
        const size_t got = rings[k]->receive(fd);  // the other ring may be under verify
        const double t = now_s();
        if (got && t0 == 0) t0 = t;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return !busy; });
            if (got) {
                job = rings[k];
                job_n = got;
                busy = true;
                cv.notify_all();
            }
        }
        if (!got && t0 > 0) break;  // the sender stopped
        t1 = now_s();
        if (t0 > 0 && t1 - t0 >= seconds) break;
    }
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !busy; });
        stop = true;
        cv.notify_all();
    }
    worker.join();
    t1 = now_s();
    const double dt = t1 > t0 ? t1 - t0 : 1e-9;
    std::printf("{\"mode\": \"%s\", \"batch_slots\": %zu, \"datagrams\": %llu, \"payload_bytes\": %llu, "
                "\"seconds\": %.4f, \"GBps\": %.4f, \"datagrams_per_s\": %.0f, \"ok\": %llu, \"batches\": %llu, "
                "\"verify_seconds\": %.4f, \"verify_GBps\": %.3f, \"gpu_batches\": %llu, "
                "\"cpu_verify_max_bytes\": %zu, \"overlapped\": true}\n",
                crc.gpu() ? "gpu" : "cpu", batch, (unsigned long long)dgrams, (unsigned long long)bytes, dt,
                double(bytes) / dt / 1e9, double(dgrams) / dt, (unsigned long long)good, (unsigned long long)batches,
                tverify, tverify > 0 ? double(bytes) / tverify / 1e9 : 0.0, (unsigned long long)gpu_batches,
                crc.gpu() ? crc.cpu_verify_max_bytes() : size_t(0));
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    try {
        Args a(argc, argv, {{"-p", "port"}, {"--port", "port"}, {"-w", "window"}, {"--window-size", "window"},
                            {"-d", "dir"}, {"--output-dir", "dir"}, {"-o", "log"}, {"--output-log", "log"},
                            {"--crc", "crc"}, {"--once", "flag:once"}, {"--batch", "batch"},
                            {"--bench", "bench"}});
        const int port = std::stoi(a.get("port", "0"));
        const uint32_t window = uint32_t(std::stoi(a.get("window", "0")));
        const bool benchmode = a.has("bench");
        if (port <= 0 || port > 65535 || (!benchmode && (window == 0 || !a.has("dir")))) {
            std::cerr << "usage: wReceiver -p <port> -w <window> -d <dir> -o <log> [--crc cpu|gpu] [--once] "
                         "[--batch N]\n       wReceiver --bench <seconds> -p <port> [--crc cpu|gpu] [--batch N]\n";
            return 1;
        }
        const size_t batch = size_t(std::stoul(a.get("batch", std::to_string(window ? window : 64))));
        if (batch == 0) throw std::runtime_error("--batch must be > 0");
        Checksums crc(a.get("crc", "cpu"));

        int fd = udp_socket();
        sockaddr_in me = addr_of("0.0.0.0", port);
        if (::bind(fd, reinterpret_cast<sockaddr *>(&me), sizeof me) < 0) throw std::runtime_error("bind failed");
        if (benchmode) {
            const int rc = bench(fd, crc, batch, std::stod(a.get("bench")));
            ::close(fd);
            return rc;
        }
        Log log(a.get("log"));
        RecvRing ring(batch, crc.gpu());

        bool open = false, done = false;
        uint32_t start_seq = 0, expected = 0;
        int file_no = 0;
        std::ofstream out;
        std::map<uint32_t, std::vector<uint8_t>> pending;  // out-of-order DATA

        while (!done) {
            const size_t got = ring.receive(fd);
            crc.verify_batch(ring.ring(), RecvRing::kSlot, ring.lens(), got, ring.ok());
            for (size_t k = 0; k < got && !done; ++k) {
                const uint8_t *buf = ring.slot(k);
                const size_t n = ring.len(k);
                if (n < kHeaderBytes) continue;  // runt: no header (the reference reads past its end)
                const PacketHeader h = get_header(buf);
                // only DATA is CRC-checked, as in the reference (Receiver.cpp:139-206)
                if (h.type == DATA && !ring.ok()[k]) continue;  // corrupted: drop, no ACK, no log
                const sockaddr_in &peer = ring.peer(k);
                log.pkt(h);

                uint32_t ack_seq;
                if (h.type == START) {
                    if (open && h.seqNum != start_seq) continue;  // another sender mid-connection
                    if (!open) {
                        open = true;
                        start_seq = h.seqNum;
                        expected = 0;
                        pending.clear();
                        out.open(a.get("dir") + "/FILE-" + std::to_string(file_no) + ".out",
                                 std::ios::binary | std::ios::trunc);
                    }
                    ack_seq = h.seqNum;
                } else if (h.type == END) {
                    if (h.seqNum != start_seq) continue;
                    if (!open) {  // duplicate END of the connection just closed: re-ACK it
                        send_ack(fd, log, h.seqNum, peer);
                        continue;
                    }
                    ack_seq = h.seqNum;
                } else if (h.type == DATA) {
                    if (!open || h.seqNum >= expected + window) continue;  // outside the window: drop
                    if (h.seqNum >= expected)
                        pending.emplace(h.seqNum, std::vector<uint8_t>(buf + kHeaderBytes, buf + n));
                    for (auto it = pending.find(expected); it != pending.end(); it = pending.find(expected)) {
                        out.write(reinterpret_cast<const char *>(it->second.data()), std::streamsize(it->second.size()));
                        pending.erase(it);
                        ++expected;
                    }
                    ack_seq = expected;
                } else {
                    continue;
                }
                send_ack(fd, log, ack_seq, peer);
                if (h.type == END) {
                    out.close();
                    open = false;
                    ++file_no;
                    if (a.has("once")) done = true;
                }
            }
        }
        ::close(fd);
        return 0;
    } catch (const std::exception &e) {
        std::cerr << "wReceiver: " << e.what() << "\n";
        return 1;
    }
}
