// latency.cpp -- per-block call latency of the C-ABI (the Dag Node's per-key Put / Get seam,
// erasure.go:51-93): rsmi_encode_block and a 1-lost-shard rsmi_reconstruct, from pageable
// (std::vector, like Go slices over cgo) and page-locked (rsmi_host_alloc) buffers.
// Diagnostic; prints microseconds per call (median of 200); --threads: coalesced groups from
// concurrent callers (throughput); block sizes
// may be given as arguments.  --sched-spin sets
// hipDeviceScheduleSpin before the first HIP call (the runtime's polling wait), for comparison:
// level with the default (profiles/r04/f), as was the engine polling its stream.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <tuple>
#include <thread>
#include <vector>

#include <emmintrin.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <ucontext.h>
#include <unistd.h>
#include <hip/hip_runtime_api.h>

#include "../include/rsmi.h"

using clk = std::chrono::steady_clock;

template <class F>
static double median_us(F f, int iters = 200) {
    std::vector<double> t;
    for (int i = 0; i < iters; i++) {
        auto a = clk::now();
        if (f() != RSMI_OK) {
            std::fprintf(stderr, "call failed\n");
            std::exit(1);
        }
        t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

// n bytes with streaming (non-temporal) stores: dst lands in memory, not in this core's cache
static void copy_nt(uint8_t* dst, const uint8_t* src, size_t n) {
    size_t i = 0;
    while (i < n && (reinterpret_cast<uintptr_t>(dst + i) & 15)) dst[i] = src[i], i++;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    for (; i < n; i++) dst[i] = src[i];
    _mm_sfence();
}

// ---- crash report: on SIGSEGV/SIGBUS write the faulting address, the PC and
// every stack frame with the /proc/self/maps line that owns it (library + offset), plus the
// mappings that end at or begin at the faulting address, then chain to the previous handler
// (rocprofv3's own stack printer).  Only read(2)/write(2)-level calls on static buffers, apart
// from backtrace(), which is preloaded at install time.
static char g_maps[1 << 20];
static struct sigaction g_prev_segv, g_prev_bus;

static void put_str(const char* s) { (void)!write(2, s, std::strlen(s)); }
static void put_hex(uintptr_t v) {
    char b[19] = "0x";
    for (int i = 0; i < 16; i++) b[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15];
    b[18] = 0;
    put_str(b);
}
static uintptr_t parse_hex(const char*& p) {
    uintptr_t v = 0;
    for (;; p++) {
        const char ch = *p;
        if (ch >= '0' && ch <= '9') v = v * 16 + uintptr_t(ch - '0');
        else if (ch >= 'a' && ch <= 'f') v = v * 16 + uintptr_t(ch - 'a' + 10);
        else break;
    }
    return v;
}
// the maps line containing a (or, with edge, the lines ending or starting exactly at a)
static void describe(const char* what, uintptr_t a, bool edge) {
    put_str(what);
    put_hex(a);
    bool found = false;
    for (const char* line = g_maps; *line;) {
        const char* eol = line;
        while (*eol && *eol != '\n') eol++;
        const char* p = line;
        const uintptr_t lo = parse_hex(p);
        p++;
        const uintptr_t hi = parse_hex(p);
        const bool in = a >= lo && a < hi, at_edge = edge && (hi == a || lo == a);
        if (in || at_edge) {
            put_str(in ? "  in  [+" : (hi == a ? "  ends at it: [" : "  starts at it: ["));
            put_hex(in ? a - lo : 0);
            put_str("] ");
            (void)!write(2, line, size_t(eol - line));
            found = true;
        }
        line = *eol ? eol + 1 : eol;
    }
    if (!found) put_str("  (no mapping)");
    put_str("\n");
}
static void crash_handler(int sig, siginfo_t* si, void* uc) {
    size_t len = 0;
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        for (ssize_t r; len + 1 < sizeof g_maps && (r = read(fd, g_maps + len, sizeof g_maps - 1 - len)) > 0;)
            len += size_t(r);
        close(fd);
    }
    g_maps[len] = 0;
    put_str(sig == SIGSEGV ? "\n=== latency: SIGSEGV ===\n" : "\n=== latency: SIGBUS ===\n");
    describe("fault address ", reinterpret_cast<uintptr_t>(si->si_addr), true);
    const auto* ctx = static_cast<const ucontext_t*>(uc);
    describe("pc            ", uintptr_t(ctx->uc_mcontext.gregs[REG_RIP]), false);
    void* frames[64];
    const int nf = backtrace(frames, 64);
    for (int i = 0; i < nf; i++) describe("frame         ", reinterpret_cast<uintptr_t>(frames[i]), false);
    put_str("=== /proc/self/maps ===\n");
    (void)!write(2, g_maps, len);
    put_str("=== end ===\n");
    const struct sigaction& prev = sig == SIGSEGV ? g_prev_segv : g_prev_bus;
    sigaction(sig, &prev, nullptr);  // chain: the previous handler, or the default action
    raise(sig);
}
static void install_crash_handler() {
    void* warm[1];
    (void)backtrace(warm, 1);  // loads libgcc's unwinder now, not inside the handler
    struct sigaction sa {};
    sa.sa_sigaction = crash_handler;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGBUS, &sa, &g_prev_bus);
}

// T threads, each coding `calls` blocks of B bytes through rsmi_encode_block_coalesced_crcs, in
// place in its own page-locked buffer (block == shards_out, Split by the thread): the coalesced
// groups' throughput, GiB/s of block payload, and how many groups they formed
static void coalesced_threads(int k, int m, size_t B, int T, int calls, int lanes = 1, int clanes = 2, int carry = 1,
                              int wait_us = 0, bool nt = false, int pipe = 1, int flag = 1) {
    // lanes > 1: the threads spread over that many contexts (thread t on context t % lanes);
    // clanes: each context's coalescing lanes (option "coalesce_lanes")
    std::vector<rsmi_ctx*> cs(static_cast<size_t>(lanes));
    for (auto& x : cs) {
        if (rsmi_open(k, m, 0, &x) != RSMI_OK) std::exit(2);
        if (rsmi_set_option(x, "coalesce_lanes", clanes) != RSMI_OK || rsmi_set_option(x, "coalesce_carry", carry) != RSMI_OK ||
            rsmi_set_option(x, "coalesce_us", wait_us) != RSMI_OK || rsmi_set_option(x, "coalesce_pipeline", pipe) != RSMI_OK ||
            rsmi_set_option(x, "coalesce_flag", flag) != RSMI_OK ||
            rsmi_warm(x) != RSMI_OK)
            std::exit(2);
    }
    rsmi_ctx* c = cs[0];
    const size_t n = size_t(k + m), S = rsmi_shard_size(B, k);
    std::vector<uint8_t*> bufs(static_cast<size_t>(T));
    std::vector<std::vector<uint8_t>> blocks(static_cast<size_t>(T), std::vector<uint8_t>(B));
    for (int t = 0; t < T; t++) {
        bufs[size_t(t)] = static_cast<uint8_t*>(rsmi_host_alloc(n * S));
        for (size_t i = 0; i < B; i++) blocks[size_t(t)][i] = uint8_t(i * 31 + size_t(t));
    }
    auto run = [&] {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                std::vector<uint32_t> raw(n);
                for (int i = 0; i < calls; i++) {
                    if (nt) copy_nt(bufs[size_t(t)], blocks[size_t(t)].data(), B);
                    else std::memcpy(bufs[size_t(t)], blocks[size_t(t)].data(), B);
                    if (rsmi_encode_block_coalesced_crcs(cs[size_t(t % lanes)], bufs[size_t(t)], B, bufs[size_t(t)],
                                                         raw.data(), nullptr))
                        std::exit(3);
                }
            });
        for (auto& x : th) x.join();
    };
    run();  // warm: plans, staging, tables
    auto stat = [&](const char* key) {
        long v = 0;
        for (auto* x : cs) v += rsmi_get_stat(x, key);
        return v;
    };
    const long c0 = stat("coalesced_calls"), b0 = stat("coalesced_batches");
    const auto a = std::chrono::steady_clock::now();
    run();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    const long calls_n = stat("coalesced_calls") - c0, batches = stat("coalesced_batches") - b0;
    std::printf("RS(%d,%d) B=%8zu  %2d threads x %d coalesced encodes + CRC-16 in place, %d context(s) x %d lane(s), "
                "carry %d, wait %d us%s, pipeline %d, flag %d: %7.2f GiB/s, %ld calls in %ld groups (%.2f; last kernel %s)\n", k, m, B, T, calls,
                lanes, clanes, carry, wait_us, nt ? ", streaming copies" : "", pipe, flag,
                double(T) * calls * B / sec / 1073741824.0, calls_n, batches, double(batches) / double(calls_n),
                rsmi_last_kernel(c));
    for (auto* p : bufs) rsmi_host_free(p);
    for (auto* x : cs) rsmi_close(x);
}

// One thread, back-to-back in-place host calls of N blocks each (a coalesced group's shape without
// the queue): the rate of the zero-copy kernel + launch + synchronisation against group size.
static void group_sweep() {
    for (auto shape : {std::make_tuple(10, 4, size_t(262144)), std::make_tuple(2, 1, size_t(262144))}) {
        const int k = std::get<0>(shape), m = std::get<1>(shape);
        const size_t B = std::get<2>(shape), n = size_t(k + m), S = rsmi_shard_size(B, k);
        rsmi_ctx* c = nullptr;
        if (rsmi_open(k, m, 0, &c) != RSMI_OK || rsmi_warm(c) != RSMI_OK) std::exit(2);
        for (size_t N : {1, 2, 4, 8, 16, 32, 64, 256}) {
            uint8_t* buf = static_cast<uint8_t*>(rsmi_host_alloc(N * n * S));
            for (size_t i = 0; i < N * n * S; i++) buf[i] = uint8_t(i * 7);
            std::vector<uint32_t> raw(N * n);
            for (int crc = 0; crc < 2; crc++) {
                auto call = [&] {
                    return crc ? rsmi_encode_batch_host_crcs(c, buf, n * S, buf + k * S, n * S, S, N, raw.data(), nullptr)
                               : rsmi_encode_batch_host(c, buf, n * S, buf + k * S, n * S, S, N);
                };
                const int it = int(std::max<size_t>(20, 2048 / N));
                for (int i = 0; i < 5; i++) call();
                const auto a = clk::now();
                for (int i = 0; i < it; i++)
                    if (call() != RSMI_OK) std::exit(3);
                const double us = std::chrono::duration<double, std::micro>(clk::now() - a).count() / it;
                std::printf("RS(%d,%d) B=%zu  %3zu blocks per in-place call%s: %8.1f us per call, %6.2f GiB/s, "
                            "%5.1f GB/s host->device (%s)\n", k, m, B, N, crc ? " + CRC-16" : "          ", us,
                            double(N * B) / us / 1073.741824, double(N * k * S) / us / 1e3, rsmi_last_kernel(c));
            }
            rsmi_host_free(buf);
        }
        rsmi_close(c);
    }
}

int main(int argc, char** argv) {
    install_crash_handler();
    if (argc > 1 && !std::strcmp(argv[1], "--group-sweep")) {
        group_sweep();
        return 0;
    }
    if (argc > 1 && !std::strcmp(argv[1], "--threads")) {
        // one context with 1, 2 or 4 coalescing lanes (one queue), and round 4's spread over 4
        // contexts of one lane each
        // (contexts, lanes, carry, coalesce_us, streaming copies); THREADS_CFG=quick: the first
        // (default) configuration and its variants at 16 threads only
        const bool quick = std::getenv("THREADS_CFG") && !std::strcmp(std::getenv("THREADS_CFG"), "quick");
        if (std::getenv("THREADS_CFG") && !std::strcmp(std::getenv("THREADS_CFG"), "one")) {
            // the default configuration at 16 threads, RS(10,4) 256 KiB only (for a kernel trace)
            coalesced_threads(10, 4, size_t(262144), 16, 128);
            return 0;
        }
        if (std::getenv("THREADS_CFG") && !std::strcmp(std::getenv("THREADS_CFG"), "flag")) {
            // option coalesce_flag off / on: 1 thread (a lone caller's in-place call) and 16 threads,
            // alternated twice
            for (int rep = 0; rep < 2; rep++)
                for (int T : {1, 16})
                    for (int flag : {0, 1})
                        for (auto shape : {std::make_tuple(2, 1, size_t(262144)), std::make_tuple(10, 4, size_t(262144)),
                                           std::make_tuple(10, 4, size_t(4096)), std::make_tuple(16, 4, size_t(4194304))})
                            coalesced_threads(std::get<0>(shape), std::get<1>(shape), std::get<2>(shape), T,
                                              std::get<2>(shape) > (size_t(1) << 20) ? 16 : (T == 1 ? 400 : 128), 1, 2, 1, 0,
                                              false, 1, flag);
            return 0;
        }
        if (std::getenv("THREADS_CFG") && !std::strcmp(std::getenv("THREADS_CFG"), "pipe")) {
            // option coalesce_pipeline off / on at 16 threads, (lanes, carry) pairs, alternated twice
            for (int rep = 0; rep < 2; rep++)
                for (auto cfg : {std::make_pair(2, 1), std::make_pair(1, 1), std::make_pair(1, 3), std::make_pair(2, 3)})
                    for (int pipe : {0, 1})
                        for (auto shape : {std::make_tuple(2, 1, size_t(262144)), std::make_tuple(10, 4, size_t(262144)),
                                           std::make_tuple(16, 4, size_t(4194304))})
                            coalesced_threads(std::get<0>(shape), std::get<1>(shape), std::get<2>(shape), 16,
                                              std::get<2>(shape) > (size_t(1) << 20) ? 16 : 128, 1, cfg.first, cfg.second,
                                              0, false, pipe);
            return 0;
        }
        for (auto cfg : {std::make_tuple(1, 2, 1, 0, false), std::make_tuple(1, 2, 1, 0, true),
                         std::make_tuple(1, 1, 1, 30, false), std::make_tuple(1, 2, 1, 30, false),
                         std::make_tuple(1, 1, 0, 0, false), std::make_tuple(1, 1, 1, 0, false),
                         std::make_tuple(1, 2, 0, 0, false), std::make_tuple(1, 4, 1, 0, false),
                         std::make_tuple(4, 1, 0, 0, false)})
            for (int T : {4, 16}) {
                if (quick && T != 16) continue;
                for (auto shape : {std::make_tuple(2, 1, size_t(262144)), std::make_tuple(10, 4, size_t(262144)),
                                   std::make_tuple(16, 4, size_t(4194304))})
                    coalesced_threads(std::get<0>(shape), std::get<1>(shape), std::get<2>(shape), T,
                                      std::get<2>(shape) > (size_t(1) << 20) ? 16 : 128, std::get<0>(cfg),
                                      std::get<1>(cfg), std::get<2>(cfg), std::get<3>(cfg), std::get<4>(cfg));
            }
        return 0;
    }
    const int k = 10, m = 4, n = k + m;
    std::vector<size_t> sizes;  // block sizes given on the command line, else the default list
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--sched-spin")) {
            if (hipSetDeviceFlags(hipDeviceScheduleSpin) != hipSuccess) return 3;
            std::printf("hipDeviceScheduleSpin\n");
        } else {
            sizes.push_back(std::strtoull(argv[i], nullptr, 10));
        }
    }
    if (sizes.empty()) sizes = {4096, 65536, 262144, 1048576, 4194304};
    rsmi_ctx* c = nullptr;
    if (rsmi_open(k, m, 0, &c) != RSMI_OK) return 2;
    for (size_t B : sizes) {
        const size_t S = rsmi_shard_size(B, k);
        std::mt19937 r(1);
        std::vector<uint8_t> blk(B), out(n * S);
        for (auto& x : blk) x = uint8_t(r());
        uint8_t* pblk = static_cast<uint8_t*>(rsmi_host_alloc(B));
        uint8_t* pout = static_cast<uint8_t*>(rsmi_host_alloc(n * S));
        std::memcpy(pblk, blk.data(), B);
        std::vector<uint8_t> present(n, 1);
        present[0] = 0;
        const double e_pg = median_us([&] { return rsmi_encode_block(c, blk.data(), B, out.data()); });
        const double r_pg = median_us([&] { return rsmi_reconstruct(c, out.data(), S, present.data(), 1); });
        const double e_pin = median_us([&] { return rsmi_encode_block(c, pblk, B, pout); });
        const double r_pin = median_us([&] { return rsmi_reconstruct(c, pout, S, present.data(), 1); });
        std::vector<uint32_t> raw(n);
        const double ec_pg = median_us([&] { return rsmi_encode_block_crc(c, blk.data(), B, out.data(), raw.data()); });
        // the lone DagNode.Put's codec call: Split already in the page-locked (k+m)*S buffer,
        // one in-place encode with every shard's CRC-16
        std::memcpy(pout, blk.data(), B);
        const double ec_inplace = median_us([&] {
            return rsmi_encode_batch_host_crcs(c, pout, n * S, pout + k * S, n * S, S, 1, raw.data(), nullptr);
        });
        // the lone Put's whole codec phase: the Split copy of a block that is not in cache (one
        // of 512 distinct blocks, like tools/bench_dagnode) into the page-locked scratch, then
        // the in-place call; the copy with plain and with streaming stores
        {
            const size_t nblk = 512;
            std::vector<uint8_t> many(nblk * B);
            for (size_t i = 0; i < many.size(); i += 64) many[i] = uint8_t(i >> 6);
            size_t it = 0;
            auto put_phase = [&](bool nt, bool call) {
                return median_us([&] {
                    const uint8_t* src = many.data() + (it++ % nblk) * B;
                    if (nt) copy_nt(pout, src, B);
                    else std::memcpy(pout, src, B);
                    std::memset(pout + B, 0, k * S - B);
                    return call ? rsmi_encode_batch_host_crcs(c, pout, n * S, pout + k * S, n * S, S, 1, raw.data(), nullptr)
                                : RSMI_OK;
                });
            };
            const double cp = put_phase(false, false), cpn = put_phase(true, false);
            const double ph = put_phase(false, true), phn = put_phase(true, true);
            std::printf("B=%8zu  Split copy %.1f us (streaming %.1f) | copy + in-place encode + CRC-16 %.1f us "
                        "(streaming copy %.1f)\n", B, cp, cpn, ph, phn);
        }
        // what the engine pays per pointer lookup (hipPointerGetAttributes) on page-locked and
        // pageable memory
        // the rows-CRC call of GetMany's verify / RepairDataNode (both CRCs of the n rows)
        std::vector<uint32_t> r32(n);
        const double crc_rows = median_us([&] {
            return rsmi_crc_rows_host(c, pout, S, n, S, raw.data(), r32.data());
        });
        const double attr_pin = median_us([&] {
            hipPointerAttribute_t a{};
            return hipPointerGetAttributes(&a, pout) == hipSuccess ? RSMI_OK : RSMI_ERR_DEVICE;
        }, 1000);
        const double attr_pg = median_us([&] {
            hipPointerAttribute_t a{};
            (void)hipPointerGetAttributes(&a, out.data());
            (void)hipGetLastError();
            return RSMI_OK;
        }, 1000);
        std::printf("B=%8zu  encode in place + CRC-16 (lone Put) %8.1f us pinned | CRC-16 + CRC-32 of the rows "
                    "%8.1f us pinned | hipPointerGetAttributes %.2f us pinned, %.2f us pageable\n",
                    B, ec_inplace, crc_rows, attr_pin, attr_pg);
        std::printf("B=%8zu  encode_block %8.1f us pageable %8.1f us pinned | reconstruct(1 lost) %8.1f us pageable "
                    "%8.1f us pinned  (%.2f / %.2f GiB/s pageable) | encode_block_crc %8.1f us pageable\n",
                    B, e_pg, e_pin, r_pg, r_pin, B / e_pg / 1073.741824, B / r_pg / 1073.741824, ec_pg);
        rsmi_host_free(pblk);
        rsmi_host_free(pout);
    }
    // what the rows-CRC read-back replaced: a blocking copy of a few result words after the sync
    void* d = nullptr;
    if (hipMalloc(&d, 4096) != hipSuccess) return 5;
    std::vector<uint8_t> h(256);
    const double d2h = median_us([&] {
        return hipMemcpy(h.data(), d, 56, hipMemcpyDeviceToHost) == hipSuccess ? RSMI_OK : RSMI_ERR_DEVICE;
    });
    std::printf("hipMemcpy device->pageable host, 56 B: %.1f us\n", d2h);
    (void)hipFree(d);
    rsmi_close(c);
    return 0;
}
