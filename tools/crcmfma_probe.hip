// crcmfma_probe.hip -- diagnostic (not part of the product): can the matrix cores fold the
// datanode CRC-16 (howeyc IBM, crc16.hpp) cheaper than the LDS nibble fold the fused encode
// uses?  R(chunk) is GF(2)-linear in the chunk's 128 bits, so a tile's chunk values are a
// GF(2) matrix product.  An MFMA sums integer products; with every product of a set bit and a
// set weight equal to one unit, bit 0 of the count (fp4) or bit 7 of the i8 sum is the parity.
//
//   nib  -- the fused encode's fold (rs_kernels.hip crc_row): quad-relative nibble tables Q in
//           LDS, 32 lookups per 16-byte chunk, two DPP XORs per quad; 16 u16 records per tile.
//   fp4  -- v_mfma_scale_f32_16x16x128_f8f6f4, fp4 (e2m1) operands: the data operand takes one
//           bit per nibble (v & 0x11111111, 0x22.., 0x44.., (v >> 1) & 0x44..: 5 VALU per dword
//           for its 32 bits), weights 2 / 1 / 0.5 so every product is 1.0; 4 MFMAs per 1 KiB.
//   i8   -- v_mfma_i32_16x16x64_i8: one bit per byte (v & (0x01010101 << s)), weights 2^(7-s),
//           every product +-128; 8 MFMAs per 1 KiB.
// MFMA forms: B = the tile's data (column m = lane & 15, k block j = lane >> 4: chunk 16 j + m),
// A = weights (row n = CRC bit), D[n][m] = chunk class m's value relative to the end of chunk
// 48 + m; four ballots of the parity bits are the tile's 32-byte record.
// Every record of a small run is checked against a host byte loop; then each fold runs over
// HBM (384 MiB of rows) and over a cache-resident 2 MiB (its issue-bound rate).  Each wave
// loads its next tile before it folds the current one.
// Usage: crcmfma_probe [iterations = 10]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            std::exit(2);                                                                        \
        }                                                                                        \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- host CRC-16 algebra
static uint16_t T[256];
static void make_table() {
    for (int i = 0; i < 256; i++) {
        uint16_t c = uint16_t(i);
        for (int k = 0; k < 8; k++) c = (c & 1) ? uint16_t((c >> 1) ^ 0xA001) : uint16_t(c >> 1);
        T[i] = c;
    }
}
static uint16_t zshift(uint16_t s, int n) {  // A^n(s): n zero bytes
    for (int i = 0; i < n; i++) s = uint16_t((s >> 8) ^ T[s & 0xFF]);
    return s;
}
static uint16_t host_chunk(const uint8_t* p) {  // R(16 bytes)
    uint16_t s = 0;
    for (int i = 0; i < 16; i++) s = uint16_t((s >> 8) ^ T[(s ^ p[i]) & 0xFF]);
    return s;
}
// contribution of bit b of byte p of a chunk, relative to the chunk's end
static uint16_t contrib(int p, int b) { return zshift(T[1 << b], 15 - p); }

// ---------------------------------------------------------------- kernels
constexpr int kWG = 256, kWave = 64;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// nib: the fused encode's fold; Q[p][h][q][v] u16 (4 KiB) in LDS
__global__ __launch_bounds__(kWG) void fold_nib(const uint8_t* __restrict__ buf, uint64_t ntiles, uint64_t wrap /* mask */,
                                                const uint32_t* __restrict__ q_tbl, uint16_t* __restrict__ rec) {
    __shared__ uint32_t s_q[1024];
    for (int i = threadIdx.x; i < 1024; i += kWG) s_q[i] = q_tbl[i];
    __syncthreads();
    const uint8_t* qt = reinterpret_cast<const uint8_t*>(s_q);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t qq = (lane & 3u) * 0x20202020u;
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    uint64_t t = uint64_t(blockIdx.x) * (kWG / kWave) + threadIdx.x / kWave;
    u32x4 xn = reinterpret_cast<const u32x4*>(buf + ((t < ntiles ? t : 0) & wrap) * 1024)[lane];
    for (; t < ntiles; t += nw) {
        const u32x4 x = xn;  // this tile; the next one's load is in flight during the fold
        xn = reinterpret_cast<const u32x4*>(buf + ((t + nw < ntiles ? t + nw : t) & wrap) * 1024)[lane];
        uint32_t cr = 0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            uint32_t lo = ((x[w] << 1) & 0x1E1E1E1Eu) | qq, hi = ((x[w] >> 3) & 0x1E1E1E1Eu) | qq;
            asm volatile("" : "+v"(lo), "+v"(hi));
            uint32_t l[8];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int p = 4 * w + q;
                l[2 * q] = *reinterpret_cast<const uint16_t*>(qt + 256 * p + ((lo >> (8 * q)) & 0xFF));
                l[2 * q + 1] = *reinterpret_cast<const uint16_t*>(qt + 256 * p + 128 + ((hi >> (8 * q)) & 0xFF));
            }
            cr = xor3(xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5]), xor3(l[6], l[7], cr));
        }
        cr ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(cr), 0xB1, 0xF, 0xF, false));
        cr ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(cr), 0x4E, 0xF, 0xF, false));
        if ((lane & 3u) == 0) rec[t * 16 + lane / 4] = uint16_t(cr);
    }
}

// the four ballots -> lanes 0..7 store the record's 8 dwords
__device__ __forceinline__ void store_ballots(uint64_t b0, uint64_t b1, uint64_t b2, uint64_t b3, uint32_t lane,
                                              uint32_t* rec) {
    const uint64_t b = lane < 2 ? b0 : lane < 4 ? b1 : lane < 6 ? b2 : b3;
    if (lane < 8) rec[lane] = uint32_t(b >> (32 * (lane & 1)));
}

// fp4: W[s] = the weight operand of bit group s for this lane (16 bytes used)
__global__ __launch_bounds__(kWG) void fold_fp4(const uint8_t* __restrict__ buf, uint64_t ntiles, uint64_t wrap /* mask */,
                                                const u32x4* __restrict__ wts, uint32_t* __restrict__ rec) {
    const uint32_t lane = threadIdx.x & 63;
    v8i W[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const u32x4 w = wts[s * 64 + lane];
        W[s] = v8i{int(w[0]), int(w[1]), int(w[2]), int(w[3]), 0, 0, 0, 0};
    }
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    uint64_t t = uint64_t(blockIdx.x) * (kWG / kWave) + threadIdx.x / kWave;
    u32x4 xn = reinterpret_cast<const u32x4*>(buf + ((t < ntiles ? t : 0) & wrap) * 1024)[lane];
    for (; t < ntiles; t += nw) {
        const u32x4 x = xn;  // this tile; the next one's load is in flight during the fold
        xn = reinterpret_cast<const u32x4*>(buf + ((t + nw < ntiles ? t + nw : t) & wrap) * 1024)[lane];
        v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; s++) {
            v8i d;
#pragma unroll
            for (int w = 0; w < 4; w++)
                d[w] = int(s < 3 ? x[w] & (0x11111111u << s) : (x[w] >> 1) & 0x44444444u);
            d[4] = d[5] = d[6] = d[7] = 0;
            acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(W[s], d, acc, 4, 4, 0, 127, 0, 127);
        }
        store_ballots(__builtin_amdgcn_ballot_w64((int(acc[0]) & 1) != 0),
                      __builtin_amdgcn_ballot_w64((int(acc[1]) & 1) != 0),
                      __builtin_amdgcn_ballot_w64((int(acc[2]) & 1) != 0),
                      __builtin_amdgcn_ballot_w64((int(acc[3]) & 1) != 0), lane, rec + t * 8);
    }
}

// i8: W[s] = the weight operand of bit s for this lane
__global__ __launch_bounds__(kWG) void fold_i8(const uint8_t* __restrict__ buf, uint64_t ntiles, uint64_t wrap /* mask */,
                                               const u32x4* __restrict__ wts, uint32_t* __restrict__ rec) {
    const uint32_t lane = threadIdx.x & 63;
    v4i W[8];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const u32x4 w = wts[s * 64 + lane];
        W[s] = v4i{int(w[0]), int(w[1]), int(w[2]), int(w[3])};
    }
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    uint64_t t = uint64_t(blockIdx.x) * (kWG / kWave) + threadIdx.x / kWave;
    u32x4 xn = reinterpret_cast<const u32x4*>(buf + ((t < ntiles ? t : 0) & wrap) * 1024)[lane];
    for (; t < ntiles; t += nw) {
        const u32x4 x = xn;  // this tile; the next one's load is in flight during the fold
        xn = reinterpret_cast<const u32x4*>(buf + ((t + nw < ntiles ? t + nw : t) & wrap) * 1024)[lane];
        v4i acc = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const uint32_t mk = 0x01010101u << s;
            const v4i d = {int(x[0] & mk), int(x[1] & mk), int(x[2] & mk), int(x[3] & mk)};
            acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(W[s], d, acc, 0, 0, 0);
        }
        store_ballots(__builtin_amdgcn_ballot_w64((acc[0] & 0x80) != 0), __builtin_amdgcn_ballot_w64((acc[1] & 0x80) != 0),
                      __builtin_amdgcn_ballot_w64((acc[2] & 0x80) != 0), __builtin_amdgcn_ballot_w64((acc[3] & 0x80) != 0),
                      lane, rec + t * 8);
    }
}

// ---------------------------------------------------------------- host side
// value of class m (chunks m, m+16, m+32, m+48 of a tile) relative to the end of chunk 48 + m
static uint16_t class_value(const uint8_t* tile, int m) {
    uint16_t v = 0;
    for (int j = 0; j < 4; j++) v ^= zshift(host_chunk(tile + 16 * (16 * j + m)), 256 * (3 - j));  // 16 chunks apart
    return v;
}
static uint16_t quad_value(const uint8_t* tile, int q) {
    uint16_t v = 0;
    for (int i = 0; i < 4; i++) v ^= zshift(host_chunk(tile + 16 * (4 * q + i)), 16 * (3 - i));
    return v;
}
static uint16_t record_class(const uint32_t* r, int m) {  // val_m bit n = bit 16(n/4) + m of ballot n%4
    uint16_t v = 0;
    for (int n = 0; n < 16; n++) {
        const uint64_t b = uint64_t(r[2 * (n & 3)]) | (uint64_t(r[2 * (n & 3) + 1]) << 32);
        v |= uint16_t(((b >> (16 * (n >> 2) + m)) & 1) << n);
    }
    return v;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 10;
    make_table();
    // nib tables: Q[p][h][q][v] = A^(16 (3 - q)) (A^(15 - p) (T[v << 4h]))
    std::vector<uint16_t> Q(16 * 2 * 4 * 16);
    for (int p = 0; p < 16; p++)
        for (int h = 0; h < 2; h++)
            for (int q = 0; q < 4; q++)
                for (int v = 0; v < 16; v++)
                    Q[((p * 2 + h) * 4 + q) * 16 + v] = zshift(zshift(T[v << (4 * h)], 15 - p), 16 * (3 - q));
    // fp4 weights: lane l = (j = l >> 4, n = l & 15), nibble e of its 16 bytes = k 32 j + e:
    // data bit b = s + 4 (e & 1) of byte e >> 1 of chunk 16 j + m
    std::vector<uint32_t> w4(4 * 64 * 4, 0), w8(8 * 64 * 4, 0);
    const uint32_t code4[4] = {4, 2, 1, 1};  // 2.0, 1.0, 0.5, 0.5 against data 0.5, 1.0, 2.0, 2.0
    for (int s = 0; s < 4; s++)
        for (int l = 0; l < 64; l++) {
            const int j = l >> 4, n = l & 15;
            for (int e = 0; e < 32; e++) {
                const uint16_t c = zshift(contrib(e >> 1, s + 4 * (e & 1)), 256 * (3 - j));
                if ((c >> n) & 1) w4[(s * 64 + l) * 4 + e / 8] |= code4[s] << (4 * (e % 8));
            }
        }
    for (int s = 0; s < 8; s++)
        for (int l = 0; l < 64; l++) {
            const int j = l >> 4, n = l & 15;
            for (int e = 0; e < 16; e++) {
                const uint16_t c = zshift(contrib(e, s), 256 * (3 - j));
                if ((c >> n) & 1) w8[(s * 64 + l) * 4 + e / 4] |= (s == 0 ? 0x80u : (1u << (7 - s))) << (8 * (e % 4));
            }
        }
    const uint64_t big = 384ull << 20, ntiles = big / 1024, wrap_small = 2048;
    uint8_t *d_buf;
    uint32_t *d_q, *d_w4, *d_w8, *d_rec;
    uint16_t* d_rec16;
    CK(hipMalloc(&d_buf, big));
    CK(hipMalloc(&d_q, Q.size() * 2));
    CK(hipMalloc(&d_w4, w4.size() * 4));
    CK(hipMalloc(&d_w8, w8.size() * 4));
    CK(hipMalloc(&d_rec, 4 * ntiles * 32));
    CK(hipMalloc(&d_rec16, 4 * ntiles * 32));
    CK(hipMemcpy(d_q, Q.data(), Q.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_w4, w4.data(), w4.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_w8, w8.data(), w8.size() * 4, hipMemcpyHostToDevice));
    // random data: a host-generated first 4 MiB (checked), the rest device-filled by copies
    const uint64_t chk_tiles = 4096;
    std::vector<uint8_t> h(chk_tiles * 1024);
    uint64_t st = 0xF11EDA6;
    for (auto& b : h) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        b = uint8_t(st >> 56);
    }
    for (uint64_t off = 0; off < big; off += h.size()) CK(hipMemcpy(d_buf + off, h.data(), h.size(), hipMemcpyHostToDevice));
    const int grid = 256 * 8;
    auto run = [&](int kind, uint64_t nt, uint64_t wrap) {
        if (kind == 0)
            hipLaunchKernelGGL(fold_nib, dim3(grid), dim3(kWG), 0, 0, d_buf, nt, wrap, d_q, d_rec16);
        else if (kind == 1)
            hipLaunchKernelGGL(fold_fp4, dim3(grid), dim3(kWG), 0, 0, d_buf, nt, wrap,
                               reinterpret_cast<const u32x4*>(d_w4), d_rec);
        else
            hipLaunchKernelGGL(fold_i8, dim3(grid), dim3(kWG), 0, 0, d_buf, nt, wrap,
                               reinterpret_cast<const u32x4*>(d_w8), d_rec);
        CK(hipGetLastError());
    };
    const char* names[3] = {"nib", "fp4", "i8"};
    // exactness on the first 4096 tiles
    bool all_ok = true;
    for (int kind = 0; kind < 3; kind++) {
        run(kind, chk_tiles, ~0ull);
        CK(hipDeviceSynchronize());
        uint64_t bad = 0, n = 0;
        if (kind == 0) {
            std::vector<uint16_t> r(chk_tiles * 16);
            CK(hipMemcpy(r.data(), d_rec16, r.size() * 2, hipMemcpyDeviceToHost));
            for (uint64_t t = 0; t < chk_tiles; t++)
                for (int q = 0; q < 16; q++, n++) bad += r[t * 16 + q] != quad_value(h.data() + t * 1024, q);
        } else {
            std::vector<uint32_t> r(chk_tiles * 8);
            CK(hipMemcpy(r.data(), d_rec, r.size() * 4, hipMemcpyDeviceToHost));
            for (uint64_t t = 0; t < chk_tiles; t++)
                for (int m = 0; m < 16; m++, n++) bad += record_class(&r[t * 8], m) != class_value(h.data() + t * 1024, m);
        }
        std::printf("exactness %-4s: %llu values, %llu wrong\n", names[kind], (unsigned long long)n, (unsigned long long)bad);
        all_ok &= bad == 0;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 2; mode++) {
        const uint64_t wrap = mode ? wrap_small - 1 : ~0ull, nt = mode ? 4 * ntiles : ntiles;
        for (int kind = 0; kind < 3; kind++) {
            run(kind, nt, wrap);  // warm
            float best = 1e30f;
            for (int i = 0; i < iters; i++) {
                CK(hipEventRecord(e0));
                run(kind, nt, wrap);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            std::printf("%-6s %-4s %10.1f us  %8.1f GB/s of row bytes (%llu tiles of 1 KiB%s)\n",
                        mode ? "cached" : "hbm", names[kind], best * 1e3, double(nt) * 1024 / (best * 1e-3) / 1e9,
                        (unsigned long long)nt, mode ? ", 2 MiB reused" : "");
        }
    }
    return all_ok ? 0 : 1;
}
