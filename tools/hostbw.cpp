// hostbw.cpp -- diagnostic: host DRAM bandwidth with T threads (read, write, copy), the ceiling
// under a device group's copy-inclusive batches: an encode moves k rows of every
// block host -> device and m rows back, so host memory sees (k + m) / k bytes per payload byte
// whichever GPU the block goes to.  Usage: hostbw [threads = 16] [MiB per thread = 512]
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 16;
    const size_t per = (argc > 2 ? size_t(std::atol(argv[2])) : 512) << 20;
    std::vector<uint64_t*> a(static_cast<size_t>(T)), b(static_cast<size_t>(T));
    for (int t = 0; t < T; t++) {
        a[size_t(t)] = static_cast<uint64_t*>(std::aligned_alloc(4096, per));
        b[size_t(t)] = static_cast<uint64_t*>(std::aligned_alloc(4096, per));
        std::memset(a[size_t(t)], t + 1, per);
        std::memset(b[size_t(t)], 0, per);
    }
    const size_t n = per / 8;
    auto run = [&](const char* name, double bytes_per_thread, auto body) {
        double best = 1e30;
        for (int rep = 0; rep < 3; rep++) {
            std::vector<std::thread> th;
            const auto t0 = std::chrono::steady_clock::now();
            for (int t = 0; t < T; t++) th.emplace_back([&, t] { body(t); });
            for (auto& x : th) x.join();
            best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        std::printf("%-6s %3d threads  %8.1f GB/s\n", name, T, bytes_per_thread * T / best / 1e9);
    };
    volatile uint64_t sink = 0;
    run("read", double(per), [&](int t) {
        const uint64_t* p = a[size_t(t)];
        uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        for (size_t i = 0; i < n; i += 4) {
            s0 += p[i];
            s1 += p[i + 1];
            s2 += p[i + 2];
            s3 += p[i + 3];
        }
        sink += s0 + s1 + s2 + s3;
    });
    run("write", double(per), [&](int t) { std::memset(b[size_t(t)], t, per); });
    run("copy", 2.0 * double(per), [&](int t) { std::memcpy(b[size_t(t)], a[size_t(t)], per); });
    for (int t = 0; t < T; t++) {
        std::free(a[size_t(t)]);
        std::free(b[size_t(t)]);
    }
    return 0;
}
