// prelaunch_probe.hip -- diagnostic (not part of the product): can a per-block host call hide its
// launch behind the host's staging copy?  A per-block DagNode call copies its rows into
// page-locked memory, then launches one zero-copy kernel and synchronises (~15-20 us of launch and
// wait).  Form B queues the kernel first behind a stream wait on a page-locked flag
// (hipStreamWaitValue32), copies, then releases the flag; form A is the product's order.  The
// kernel XORs the k = 10 data rows of 26 215 B into one output row over PCIe (a 1-row reconstruct
// of a 256 KiB RS(10,4) block).  Every iteration's flag value is new and is always written, so no
// queued wait is ever left pending; a bounded spin on the host (2 s) guards the synchronisation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                  \
        }                                                                                  \
    } while (0)

__global__ __launch_bounds__(256) void xor_rows(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S,
                                                uint32_t k) {
    const uint32_t i = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (i + 4 > S) return;
    uint32_t acc = 0;
    for (uint32_t c = 0; c < k; c++) acc ^= *reinterpret_cast<const uint32_t*>(in + size_t(c) * S + i);
    *reinterpret_cast<uint32_t*>(out + i) = acc;
}

using clk = std::chrono::steady_clock;

int main() {
    const uint32_t k = 10, S = 26216;  // dword-multiple row (the probe's kernel reads dwords)
    const size_t rows = size_t(k) * S;
    std::vector<uint8_t> src(rows);
    for (size_t i = 0; i < rows; i++) src[i] = uint8_t(i * 131 + 7);
    uint8_t* buf = nullptr;
    uint32_t* flag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&buf), rows + S, hipHostMallocPortable));
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocPortable));
    uint8_t *dbuf = nullptr, *dflag = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dbuf), buf, 0));
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), flag, 0));
    *flag = 0;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const dim3 grid((S / 4 + 255) / 256);
    auto check = [&] {
        uint32_t want = 0;
        for (uint32_t c = 0; c < k; c++) want ^= *reinterpret_cast<const uint32_t*>(buf + size_t(c) * S + 4 * 100);
        if (*reinterpret_cast<const uint32_t*>(buf + rows + 4 * 100) != want) {
            std::fprintf(stderr, "wrong result\n");
            std::exit(3);
        }
    };
    uint32_t seq = 0;
    for (int form = 0; form < 2; form++)
        for (int rep = 0; rep < 2; rep++) {
            std::vector<double> t;
            for (int it = 0; it < 300; it++) {
                src[it % rows] ^= 1;  // a different block each time
                const auto a = clk::now();
                if (form == 0) {
                    std::memcpy(buf, src.data(), rows);
                    hipLaunchKernelGGL(xor_rows, grid, dim3(256), 0, st, dbuf, dbuf + rows, S, k);
                    CK(hipStreamSynchronize(st));
                } else {
                    ++seq;
                    CK(hipStreamWaitValue32(st, flag, seq, hipStreamWaitValueEq, 0xFFFFFFFFu));
                    hipLaunchKernelGGL(xor_rows, grid, dim3(256), 0, st, dbuf, dbuf + rows, S, k);
                    std::memcpy(buf, src.data(), rows);
                    __atomic_store_n(flag, seq, __ATOMIC_RELEASE);
                    // bounded wait: the stream must drain within 2 s
                    const auto w0 = clk::now();
                    while (hipStreamQuery(st) == hipErrorNotReady) {
                        if (clk::now() - w0 > std::chrono::seconds(2)) {
                            std::fprintf(stderr, "stream did not drain\n");
                            std::exit(4);
                        }
                    }
                }
                t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
                check();
            }
            std::sort(t.begin(), t.end());
            std::printf("%s: median %.1f us, p10 %.1f, p90 %.1f\n",
                        form == 0 ? "copy, launch, synchronise             " : "wait-queued launch, copy, release flag",
                        t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
        }
    // the same product order with the query loop instead of the blocking wait (A/B of the wait)
    std::vector<double> t;
    for (int it = 0; it < 300; it++) {
        const auto a = clk::now();
        std::memcpy(buf, src.data(), rows);
        hipLaunchKernelGGL(xor_rows, grid, dim3(256), 0, st, dbuf, dbuf + rows, S, k);
        while (hipStreamQuery(st) == hipErrorNotReady) {
        }
        t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
    }
    std::sort(t.begin(), t.end());
    std::printf("copy, launch, poll the stream           : median %.1f us, p10 %.1f, p90 %.1f\n", t[t.size() / 2],
                t[t.size() / 10], t[t.size() * 9 / 10]);
    CK(hipStreamDestroy(st));
    CK(hipHostFree(buf));
    CK(hipHostFree(flag));
    return 0;
}
