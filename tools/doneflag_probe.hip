// doneflag_probe.hip -- diagnostic (not part of the product): how much of a per-block host call's
// ~15-20 us fixed cost is the stream synchronisation?  Form A is the product's order: copy the
// rows into page-locked memory, launch one zero-copy kernel, hipStreamSynchronize.  Form B
// launches a kernel whose last workgroup (a device counter) releases a page-locked completion
// flag at system scope after every workgroup's stores, and the host spins on that flag instead of
// synchronising the stream.  The kernel XORs the k = 10 data rows of 26 216 B into one output row
// over PCIe (a 1-row reconstruct of a 256 KiB RS(10,4) block).  Forms C and D keep the kernel and
// release the flag behind it: a one-thread kernel queued after it, or hipStreamWriteValue32.  Every launch's flag value is new;
// the host spin is bounded (2 s), and the stream is synchronised after each form.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                          \
        }                                                                                          \
    } while (0)

template <bool FLAG>
__global__ __launch_bounds__(256) void xor_rows(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t S,
                                                uint32_t k, uint32_t* ctr, uint32_t* flag, uint32_t seq,
                                                uint32_t target) {
    const uint32_t i = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (i + 4 <= S) {
        uint32_t acc = 0;
        for (uint32_t c = 0; c < k; c++) acc ^= *reinterpret_cast<const uint32_t*>(in + size_t(c) * S + i);
        *reinterpret_cast<uint32_t*>(out + i) = acc;
    }
    if constexpr (FLAG) {
        __syncthreads();  // the workgroup's stores issued
        if (threadIdx.x == 0) {
            // counts every flag launch's workgroups (never reset): this launch ends at target
            const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
            if (old + 1u == target) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// form C: the release as a kernel of its own, queued behind the work
__global__ void set_flag(uint32_t* flag, uint32_t seq) {
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

using clk = std::chrono::steady_clock;

int main() {
    const uint32_t k = 10, S = 26216;
    const size_t rows = size_t(k) * S;
    std::vector<uint8_t> src(rows);
    for (size_t i = 0; i < rows; i++) src[i] = uint8_t(i * 131 + 7);
    uint8_t* buf = nullptr;
    uint32_t* flag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&buf), rows + S, hipHostMallocPortable));
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocPortable));
    uint8_t* dbuf = nullptr;
    uint32_t* dflag = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dbuf), buf, 0));
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), flag, 0));
    uint32_t* ctr = nullptr;
    CK(hipMalloc(reinterpret_cast<void**>(&ctr), 64));
    CK(hipMemset(ctr, 0, 64));
    __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const dim3 grid((S / 4 + 255) / 256);
    auto check = [&] {
        for (uint32_t at : {0u, 100u, S / 4 - 1}) {
            uint32_t want = 0;
            for (uint32_t c = 0; c < k; c++) want ^= *reinterpret_cast<const uint32_t*>(buf + size_t(c) * S + 4 * at);
            if (*reinterpret_cast<const uint32_t*>(buf + rows + 4 * at) != want) {
                std::fprintf(stderr, "wrong result\n");
                std::exit(3);
            }
        }
    };
    uint32_t seq = 0, nflag = 0;  // flag values; launches of the flag-releasing kernel
    const char* names[4] = {"launch, hipStreamSynchronize", "launch, spin on the kernel's flag",
                            "launch + flag kernel, spin", "launch + hipStreamWriteValue32, spin"};
    for (int copy = 1; copy >= 0; copy--)
        for (int rep = 0; rep < 2; rep++)
            for (int form = 0; form < 4; form++) {
                std::vector<double> t, tl;
                for (int it = 0; it < 400; it++) {
                    src[it % rows] ^= 1;
                    std::memset(buf + rows, 0, S);
                    if (form == 1 && nflag + 1 > 0xFFFFFFFFu / grid.x) {
                        std::fprintf(stderr, "counter range\n");
                        std::exit(5);
                    }
                    const auto a = clk::now();
                    if (copy) std::memcpy(buf, src.data(), rows);
                    const auto l0 = clk::now();
                    if (form == 0) {
                        hipLaunchKernelGGL(xor_rows<false>, grid, dim3(256), 0, st, dbuf, dbuf + rows, S, k, ctr, dflag,
                                           0u, 0u);
                        tl.push_back(std::chrono::duration<double, std::micro>(clk::now() - l0).count());
                        CK(hipStreamSynchronize(st));
                    } else {
                        ++seq;
                        if (form == 1) {
                            ++nflag;
                            hipLaunchKernelGGL(xor_rows<true>, grid, dim3(256), 0, st, dbuf, dbuf + rows, S, k, ctr,
                                               dflag, seq, nflag * grid.x);
                        } else {
                            hipLaunchKernelGGL(xor_rows<false>, grid, dim3(256), 0, st, dbuf, dbuf + rows, S, k, ctr,
                                               dflag, 0u, 0u);
                            if (form == 2)
                                hipLaunchKernelGGL(set_flag, dim3(1), dim3(1), 0, st, dflag, seq);
                            else
                                CK(hipStreamWriteValue32(st, flag, seq, 0));
                        }
                        tl.push_back(std::chrono::duration<double, std::micro>(clk::now() - l0).count());
                        const auto w0 = clk::now();
                        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                            if (clk::now() - w0 > std::chrono::seconds(2)) {
                                std::fprintf(stderr, "flag not released\n");
                                CK(hipStreamSynchronize(st));
                                std::exit(4);
                            }
                        }
                    }
                    t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
                    check();
                }
                CK(hipStreamSynchronize(st));
                std::sort(t.begin(), t.end());
                std::sort(tl.begin(), tl.end());
                std::printf("%s%-34s: median %.1f us, p10 %.1f, p90 %.1f (launch call %.1f)\n", copy ? "copy, " : "      ",
                            names[form], t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10], tl[tl.size() / 2]);
            }
    CK(hipStreamDestroy(st));
    CK(hipFree(ctr));
    CK(hipHostFree(buf));
    CK(hipHostFree(flag));
    return 0;
}
