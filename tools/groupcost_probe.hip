// groupcost_probe.hip -- diagnostic (not part of the product): where the fixed cost of a small
// zero-copy coalesced group goes (verdict r5 item 4).  A group kernel shaped like the product's
// table launch (RS(10,4) 256 KiB blocks in page-locked host memory, S = 26 216, one 1 KiB tile per
// wave, 4 waves per workgroup, 6 of the 10 input rows in flight per lane, 4 output rows stored,
// every workgroup's last act the completion-flag release of launch_done) is timed from the host
// and from inside:
//   launch   host: hipLaunchKernelGGL call to return
//   dispatch the launch call's start to the first wave's first instruction (GPU clock mapped to
//            the host clock, below)
//   first    a wave's start to its first input row's arrival (one zero-copy load round trip),
//            median over the waves
//   span     first wave's start to the last wave's end (every store complete)
//   tail     the last wave's end to the host seeing the flag
// The GPU clock (s_memrealtime, 100 MHz) is mapped to the host's steady clock by a calibration
// kernel that writes its clock into fine-grained host memory for ~2 ms (a bounded loop) while the
// host polls: offset = min over samples of (host time - GPU time), i.e. biased by the one-way
// visibility latency (~1 us); the dispatch and tail figures carry that bias with opposite signs.
// The XOR math stands in for the GF(2^8) tables: the memory traffic and geometry are the product's.
// Every launch has a fresh flag value, the host spin is bounded (2 s), and each kernel's loops end
// after a fixed count.
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t gpu_clock() {
    uint64_t t;
    asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}

constexpr int K = 10, M = 4, P = 6;  // input rows, output rows, rows in flight
constexpr uint32_t S = 26216, TILE = 1024, TPB = (S + TILE - 1) / TILE;  // 26 tiles per block

// stamps[w * 4 + 0..2]: wave w's start, first row arrived, end (GPU clock)
__global__ __launch_bounds__(256) void group_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                    uint32_t ntiles, uint64_t* stamps, uint32_t* ctr,
                                                    uint32_t* flag, uint32_t seq) {
    const uint64_t t_start = gpu_clock();
    const uint32_t lane = threadIdx.x & 63, wave = blockIdx.x * 4 + threadIdx.x / 64;
    uint64_t t_first = t_start;
    if (wave < ntiles) {
        const uint32_t blk = wave / TPB, tib = wave % TPB;
        const uint32_t off = tib * TILE + lane * 16;
        const uint32_t o = off + 16 <= S ? off : S - 16;  // the row's last window overlaps (UA)
        const uint8_t* b = in + size_t(blk) * (K + M) * S;
        u32x4 v[P];
#pragma unroll
        for (int c = 0; c < P; c++) v[c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b + size_t(c) * S + o));
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");  // row 0 has arrived
        t_first = gpu_clock();
        u32x4 acc[M] = {};
#pragma unroll
        for (int c = 0; c < K; c++) {
            const u32x4 x = v[c % P];
#pragma unroll
            for (int j = 0; j < M; j++) acc[j] ^= (x << (j + 1)) | (x >> (31 - j));
            if (c + P < K) v[c % P] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b + size_t(c + P) * S + o));
        }
        uint8_t* ob = out + size_t(blk) * (K + M) * S + size_t(K) * S;
#pragma unroll
        for (int j = 0; j < M; j++) __builtin_nontemporal_store(acc[j], reinterpret_cast<u32x4*>(ob + size_t(j) * S + o));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // every wave's stores, system scope
    const uint64_t t_end = gpu_clock();
    if (lane == 0 && wave < ntiles) {
        stamps[wave * 4 + 0] = t_start;
        stamps[wave * 4 + 1] = t_first;
        stamps[wave * 4 + 2] = t_end;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
        if (old + 1u == gridDim.x) {
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// calibration: one thread writes (i, clock) pairs into fine-grained host memory, a fixed count
__global__ void clock_pump(uint64_t* box, uint32_t n) {
    for (uint32_t i = 1; i <= n; i++) {
        const uint64_t t = gpu_clock();
        __hip_atomic_store(box + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(box, uint64_t(i), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_sleep(2);
    }
}

using clk = std::chrono::steady_clock;
static double host_us(clk::time_point t) {
    return std::chrono::duration<double, std::micro>(t.time_since_epoch()).count();
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
    const bool dev_data = argc > 1 && !std::strcmp(argv[1], "--device-data");
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const double gpu_us = 1000.0 / double(rate_khz);  // microseconds per GPU clock tick
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    // clock calibration
    uint64_t* box = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&box), 64, hipHostMallocCoherent | hipHostMallocMapped));
    box[0] = box[1] = 0;
    uint64_t* dbox = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dbox), box, 0));
    const uint32_t npump = 20000;
    hipLaunchKernelGGL(clock_pump, dim3(1), dim3(1), 0, st, dbox, npump);
    double offset = 1e300;  // host us - GPU us
    uint64_t last = 0;
    const auto w0 = clk::now();
    while (last < npump && clk::now() - w0 < std::chrono::seconds(2)) {
        const uint64_t i = __atomic_load_n(box, __ATOMIC_ACQUIRE);
        if (i != last) {
            const double h = host_us(clk::now());
            const uint64_t g = __atomic_load_n(box + 1, __ATOMIC_ACQUIRE);
            if (__atomic_load_n(box, __ATOMIC_ACQUIRE) == i) offset = std::min(offset, h - double(g) * gpu_us);
            last = i;
        }
    }
    CK(hipStreamSynchronize(st));
    std::printf("clock: %d kHz, calibration %s (%llu samples seen)\n", rate_khz,
                last >= npump ? "complete" : "cut short", (unsigned long long)last);
    const uint32_t max_blocks = 16;
    const size_t bytes = size_t(max_blocks) * (K + M) * S;
    uint8_t* host = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&host), bytes, hipHostMallocPortable | hipHostMallocMapped));
    for (size_t i = 0; i < bytes; i++) host[i] = uint8_t(i * 131 + 7);
    uint8_t* data = nullptr;
    if (dev_data) {
        CK(hipMalloc(reinterpret_cast<void**>(&data), bytes));
        CK(hipMemcpy(data, host, bytes, hipMemcpyHostToDevice));
    } else {
        CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&data), host, 0));
    }
    const uint32_t max_tiles = max_blocks * TPB;
    uint64_t* stamps = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&stamps), max_tiles * 4 * 8, hipHostMallocPortable | hipHostMallocMapped));
    uint64_t* dstamps = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dstamps), stamps, 0));
    uint32_t* flag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocCoherent | hipHostMallocMapped));
    uint32_t* dflag = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), flag, 0));
    __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
    uint32_t* ctr = nullptr;
    CK(hipMalloc(reinterpret_cast<void**>(&ctr), 64));
    CK(hipMemset(ctr, 0, 64));
    CK(hipDeviceSynchronize());
    std::printf("%s data, RS(10,4) 256 KiB blocks, medians of 200 launches (us)\n", dev_data ? "device" : "page-locked host");
    std::printf("%6s %8s %8s %9s %8s %8s %8s %8s | %s\n", "blocks", "launch", "dispatch", "1st load", "span", "tail",
                "total", "GB/s", "span = first load + rest");
    uint32_t seq = 0;
    for (uint32_t nb : {1u, 2u, 4u, 8u, 16u}) {
        const uint32_t ntiles = nb * TPB, grid = (ntiles + 3) / 4;
        std::vector<double> launch, dispatch, first, span, tail, total;
        for (int it = 0; it < 220; it++) {
            ++seq;
            const auto t0 = clk::now();
            hipLaunchKernelGGL(group_kernel, dim3(grid), dim3(256), 0, st, data, data, ntiles, dstamps, ctr, dflag, seq);
            const auto t1 = clk::now();
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                if (clk::now() - t1 > std::chrono::seconds(2)) {
                    std::fprintf(stderr, "flag not released\n");
                    CK(hipStreamSynchronize(st));
                    return 4;
                }
            }
            const auto t2 = clk::now();
            CK(hipStreamSynchronize(st));
            if (it < 20) continue;  // warm-up
            uint64_t s0 = ~0ull, e1 = 0;
            std::vector<double> f;
            for (uint32_t w = 0; w < ntiles; w++) {
                s0 = std::min(s0, stamps[w * 4 + 0]);
                e1 = std::max(e1, stamps[w * 4 + 2]);
                f.push_back(double(stamps[w * 4 + 1] - stamps[w * 4 + 0]) * gpu_us);
            }
            const double g0 = double(s0) * gpu_us + offset, g1 = double(e1) * gpu_us + offset;
            launch.push_back(host_us(t1) - host_us(t0));
            dispatch.push_back(g0 - host_us(t0));
            first.push_back(median(f));
            span.push_back(g1 - g0);
            tail.push_back(host_us(t2) - g1);
            total.push_back(host_us(t2) - host_us(t0));
        }
        const double moved = double(nb) * (K + M) * S;
        std::printf("%6u %8.1f %8.1f %9.1f %8.1f %8.1f %8.1f %8.1f |\n", nb, median(launch), median(dispatch), median(first),
                    median(span), median(tail), median(total), moved / median(total) / 1e3);
    }
    CK(hipStreamDestroy(st));
    if (dev_data) CK(hipFree(data));
    CK(hipFree(ctr));
    CK(hipHostFree(host));
    CK(hipHostFree(stamps));
    CK(hipHostFree(flag));
    CK(hipHostFree(box));
    return 0;
}
