// rs_crc32_kernels.hip -- R(row) of shard rows for the mutcask value checksum (CRC-32 IEEE,
// kv/mutcask/cask.go:73-97; algebra in crc32.hpp), the CRC-32 sibling of
// rs_crc16_rows_kernel (rs_kernels.hip).
//
// Work item = (row, segment of kCrcSegTiles consecutive 1 KiB tiles).  Each lane loads its
// 16-byte chunk of every tile of the segment (all loads in flight first), folds each chunk
// with 32 nibble lookups into 16-entry u32 tables (N: chunk value relative to the chunk's
// end; a wave-wide lookup into one table touches at most 16 dwords in 16 distinct banks, so
// it never conflicts) and carries a running register across the tiles (A^1024 between
// them).  A Hillis-Steele scan over the 64 lanes (A^(16 * 2^j) per level) leaves the
// segment's value, relative to the segment's end, in lane 63.  Lane 63 then moves it to the
// row's end -- forward by S - end for inner segments (A^(2^i) tables, i < 32), backward by
// end - S < 1024 for the last one (A^-(2^i), i < 10) -- and XORs it into the row's word.
// Every power is applied nibble-sliced (8 lookups into 16-entry tables, 512 B per power),
// so all 42 of them sit in LDS next to the fold tables (23 KiB): the end shift is a
// dependent chain of up to 32 applications, and chained L2 reads made it the kernel's
// bottleneck (2.7 TB/s at 26 KB rows with byte-sliced tables in global memory).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "crc32.hpp"
#include "rs_device.hpp"
#include "rs_plan.hpp"

namespace rsmi {

namespace {

// A^(2^i) or A^-(2^i) of s from a nibble-sliced table t[8][16] (512 B): the nibble offsets
// come out of two masked words, as in the chunk fold
__device__ __forceinline__ uint32_t pow_nib(const uint32_t* t, uint32_t s) {
    uint32_t lo = (s << 2) & 0x3C3C3C3Cu, hi = (s >> 2) & 0x3C3C3C3Cu;
    asm volatile("" : "+v"(lo), "+v"(hi));
    const uint8_t* b = reinterpret_cast<const uint8_t*>(t);
    uint32_t l[8];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        l[2 * q] = *reinterpret_cast<const uint32_t*>(b + 128 * q + ((lo >> (8 * q)) & 0xFF));
        l[2 * q + 1] = *reinterpret_cast<const uint32_t*>(b + 128 * q + 64 + ((hi >> (8 * q)) & 0xFF));
    }
    return xor3(xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5]), l[6] ^ l[7]);
}

}  // namespace

// tbl: N[32][16] | PN[32][8][16] | QN[10][8][16] (u32 words, rs_plan.hpp), all staged in LDS
template <bool ALIGNED>
__global__ __launch_bounds__(kWG) void rs_crc32_rows_kernel(const uint32_t* __restrict__ tbl,
                                                            const uint8_t* __restrict__ base, uint64_t bstride,
                                                            uint64_t rpitch, uint32_t nrows, uint64_t S, uint32_t tpb,
                                                            uint32_t nseg, uint64_t nitems, uint32_t* __restrict__ out,
                                                            uint64_t out_bs) {
    __shared__ uint32_t s_tbl[kCrc32TableWords];
    for (int i = threadIdx.x; i < kCrc32TableWords; i += kWG) s_tbl[i] = tbl[i];
    __syncthreads();
    const uint32_t* s_n = s_tbl;
    const uint32_t* sP = s_tbl + kCrc32NWords;
    const uint32_t* sQ = sP + kCrc32Powers * kCrc32PowWords;
    auto lpow = [&](int i, uint32_t s) { return pow_nib(sP + i * kCrc32PowWords, s); };

    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    for (uint64_t it = uint64_t(blockIdx.x) * (kWG / kWave) + wid; it < nitems; it += nw) {
        const uint32_t seg = uint32_t(it % nseg);
        const uint64_t rid = it / nseg;
        const uint64_t b = rid / nrows;
        const uint32_t r = uint32_t(rid - b * nrows);
        const uint8_t* row = base + b * bstride + uint64_t(r) * rpitch;
        const uint32_t t0 = seg * kCrcSegTiles;
        const uint32_t nt = tpb - t0 < uint32_t(kCrcSegTiles) ? tpb - t0 : uint32_t(kCrcSegTiles);
        u32x4 v[kCrcSegTiles];
#pragma unroll
        for (int i = 0; i < kCrcSegTiles; i++)
            if (uint32_t(i) < nt) {
                const uint64_t off = (uint64_t(t0 + i) * kWave + lane) * 16;
                // wave-uniform: only a row's last tile needs the per-lane bounds and masks
                if (ALIGNED && (uint64_t(t0 + i) + 1) * (kWave * 16) <= S)
                    v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + off));
                else
                    v[i] = crc_chunk_load<ALIGNED>(row, off, S);
            }
        uint32_t acc = 0;
        const uint8_t* nb = reinterpret_cast<const uint8_t*>(s_n);
#pragma unroll
        for (int i = 0; i < kCrcSegTiles; i++) {
            if (uint32_t(i) < nt) {
                uint32_t c = 0;
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    // byte offsets 4 x nibble into the 16-entry u32 tables (64 B each)
                    uint32_t lo = (v[i][w] << 2) & 0x3C3C3C3Cu, hi = (v[i][w] >> 2) & 0x3C3C3C3Cu;
                    asm volatile("" : "+v"(lo), "+v"(hi));  // keep the two masks (one extract per offset)
                    uint32_t l[8];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int p = 4 * w + q;
                        l[2 * q] = *reinterpret_cast<const uint32_t*>(nb + 128 * p + ((lo >> (8 * q)) & 0xFF));
                        l[2 * q + 1] = *reinterpret_cast<const uint32_t*>(nb + 128 * p + 64 + ((hi >> (8 * q)) & 0xFF));
                    }
                    c = xor3(c, xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5])) ^ (l[6] ^ l[7]);
                }
                acc = lpow(10, acc) ^ c;  // previous tiles move 1 KiB further from the end
            }
        }
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const uint32_t w = lpow(4 + j, acc);  // 16 * 2^j bytes
            const uint32_t t = __shfl_up(w, 1u << j);
            if (lane >= (1u << j)) acc ^= t;
        }
        if (lane == kWave - 1) {
            const uint64_t seg_end = uint64_t(t0 + nt) * (kWave * 16);
            if (seg_end <= S) {
                uint64_t e = S - seg_end;
                for (int i = 0; e; i++, e >>= 1)
                    if (e & 1) acc = lpow(i, acc);
            } else {
                uint32_t e = uint32_t(seg_end - S);  // < 1024: only the last tile passes S
                for (int i = 0; e; i++, e >>= 1)
                    if (e & 1) acc = pow_nib(sQ + i * kCrc32PowWords, acc);
            }
            atomicXor(out + b * out_bs + r, acc);
        }
    }
}

void* crc32_rows_kernel(bool aligned) {
    return aligned ? reinterpret_cast<void*>(&rs_crc32_rows_kernel<true>)
                   : reinterpret_cast<void*>(&rs_crc32_rows_kernel<false>);
}

}  // namespace rsmi
