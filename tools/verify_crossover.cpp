// verify_crossover — where a receiver batch is cheaper on the CPU than on the GPU.
//
// Times Checksums::verify_batch (cpp/src/common/Endpoint.hpp, the wReceiver path) on a
// pinned ring of full 1472-B WTP datagrams in 1504-B slots, for batch sizes 1..1024, two
// ways: forced to the CPU (crc32_fast, WTP_VERIFY_CPU_MAX_BYTES huge) and forced to the GPU
// (wtp_crc32_host_verify, WTP_VERIFY_CPU_MAX_BYTES=0).  Median of `reps` calls each,
// interleaved.  One JSON line per batch size; the crossover sets kCpuVerifyMaxBytes.
//   verify_crossover [reps]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common/Endpoint.hpp"

using namespace wtp;

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 400;
    const size_t nmax = 1024, stride = RecvRing::kSlot;
    uint8_t *ring = static_cast<uint8_t *>(wtp_host_alloc(nmax * stride));
    uint32_t *rl = static_cast<uint32_t *>(wtp_host_alloc(nmax * 4));
    if (!ring || !rl) return 2;
    uint64_t x = 0x5EED;
    std::vector<uint8_t> pay(kMaxPayload);
    for (size_t i = 0; i < nmax; ++i) {
        for (auto &b : pay) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            b = uint8_t(x >> 56);
        }
        rl[i] = uint32_t(make_datagram(ring + i * stride, DATA, uint32_t(i), pay.data(), kMaxPayload,
                                       crc32(pay.data(), kMaxPayload)));
    }
    setenv("WTP_VERIFY_CPU_MAX_BYTES", "18446744073709551615", 1);
    const Checksums cpu("gpu");
    setenv("WTP_VERIFY_CPU_MAX_BYTES", "0", 1);
    const Checksums gpu("gpu");
    std::vector<uint8_t> ok(nmax);
    auto once = [&](const Checksums &c, size_t n) {
        const auto t0 = std::chrono::steady_clock::now();
        c.verify_batch(ring, stride, rl, n, ok.data());
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        for (size_t i = 0; i < n; ++i)
            if (!ok[i]) std::exit(3);  // every datagram is intact
        return us;
    };
    for (int w = 0; w < 50; ++w) once(gpu, 64), once(cpu, 64);
    for (size_t n : {1, 2, 4, 8, 10, 16, 24, 32, 48, 64, 96, 128, 192, 256, 512, 1024}) {
        std::vector<double> a, b;
        for (int r = 0; r < reps; ++r) {
            a.push_back(once(cpu, n));
            b.push_back(once(gpu, n));
        }
        std::nth_element(a.begin(), a.begin() + reps / 2, a.end());
        std::nth_element(b.begin(), b.begin() + reps / 2, b.end());
        std::printf("{\"datagrams\": %zu, \"payload_bytes\": %zu, \"cpu_us\": %.2f, \"gpu_us\": %.2f, \"faster\": \"%s\"}\n",
                    n, n * kMaxPayload, a[reps / 2], b[reps / 2], a[reps / 2] <= b[reps / 2] ? "cpu" : "gpu");
        std::fflush(stdout);
    }
    wtp_host_free(ring);
    wtp_host_free(rl);
    return 0;
}
