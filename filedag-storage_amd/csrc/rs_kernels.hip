// rs_kernels.hip -- CDNA4 (gfx950) Reed-Solomon coding kernels.
//
// One kernel family computes every RS operation the Dag Node needs:
//   out_row[j][x] = XOR_c coef[j][c] * in_row[c][x]      (GF(2^8), poly 0x11D)
// Encode (erasure.go:60, upstream Encode) uses the parity rows of the systematic matrix
// over the k data rows; reconstruct (erasure.go:82/88, ReconstructData/Reconstruct) uses
// the decode rows over the first k present rows.  Positions x are independent, so the
// kernel is a pure HBM stream: read K rows, write MT rows, no reuse across workgroups.
//
// GF multiply without MFMA: a product a*x is linear in the bits of x, so it is the XOR
// of three table lookups on bit fields of x (bits 0-2, 3-5, 6-7).  Each lookup is a
// single v_perm_b32 that selects 4 bytes at once from an 8-byte pool of products, with
// the field values as per-byte selectors.  Per input dword: 5 VALU ops build the three
// selector words (shared by all MT outputs); per (output, input) dword: 3 v_perm_b32 and
// 1.5 v_bitop3_b32 (3-input XOR).  Tables for the current column come from LDS by
// broadcast ds_read_b128 (same address in every lane).
//
// Layout contract (fast path): row r of block b lives at base + b*bstride + r*rstride,
// every base/stride 16-byte aligned, rstride >= roundup(S,16).  A wave owns a "tile" of
// 64*D consecutive 16-byte chunks of one block; lanes past the block's last chunk clamp
// their loads to a valid chunk and skip their stores, and the one partial chunk at the
// end of a row is stored bytewise so no byte at or past S is ever written.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "crc16.hpp"
#include "rs_device.hpp"
#include "rs_plan.hpp"

namespace rsmi {

// Rows in flight per lane for the software pipeline: narrow outputs (MT <= 2) keep every
// input row in flight (registers are cheap there, measured +2.6% on RS(10,4) 1-row
// reconstruct); wide outputs keep a ring of 6.
template <int K, int MT>
constexpr int rows_in_flight() {
    constexpr int cap = MT <= 2 ? 16 : 6;
    return K < cap ? K : cap;
}

// K inputs, MT (<= 4) outputs, one 16-byte chunk per lane per row.
// NT: cache policy, 1 = nontemporal loads and stores (write-heavy tiles), 2 = nontemporal
// loads, default stores (tiles that read at least 4 rows per row written); DESIGN.md §4.
// WPS: waves per SIMD the register allocation must allow.
// UA: rows at any byte alignment and pitch (S >= 16).  A lane's 16-byte window starts at
// min(16*ch, S - 16): the row's last window overlaps the one before it instead of running
// past S, so loads never leave [0, S) and every store is a whole 16-byte window (the
// overlapped bytes get the same value from both lanes).  This serves the Split layout itself
// (rows back to back at pitch S, odd for RS(10,4)) and page-locked host memory read and
// written in place over PCIe.
// CRC (with UA only): also fold every row the tile reads or writes into per-chunk CRC-16
// values (crc16.hpp: R of the chunk's bytes relative to the chunk's end, nibble tables) and
// store them as u16 at crc_out[(block * crc_slots + shard) * tpb * 64 + chunk]; input row c is
// shard in_row[c], output row j is shard crc_out_slot0 + out_row[j].  rs_crc16_combine_kernel
// turns them into R(row).
// Launch geometry: one tile per wave; the loop strides over further tiles only
// when the caller caps the grid (option waves_per_cu).
template <int K, int MT, int NT, int WPS = kMinWavesPerSimd, bool UA = false, bool CRC = false>
__global__ __launch_bounds__(kWG, WPS) void rs_fast_kernel(const RsPlanDev* __restrict__ plan,
                                                       const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                       uint64_t in_bs, uint64_t in_rs, uint64_t out_bs,
                                                       uint64_t out_rs, uint32_t S, uint32_t cpb, uint32_t tpb,
                                                       uint32_t ntiles, const uint32_t* __restrict__ crc_tbl,
                                                       uint16_t* __restrict__ crc_out, uint32_t crc_slots,
                                                       uint32_t crc_out_slot0) {
    static_assert(!CRC || UA, "fused chunk CRCs: unaligned-window kernels only");
    static_assert(NT == 1 || NT == 2, "cache policy 1 or 2");
    __shared__ u32x4 s_tbl[K * kColDwords / 4];
    __shared__ uint32_t s_crc[CRC ? kCrcNWords : 1];
    {
        const uint32_t* src = plan->tbl;
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_tbl);
        for (int i = threadIdx.x; i < K * kColDwords; i += kWG) dst[i] = src[i];
        if constexpr (CRC)
            for (int i = threadIdx.x; i < kCrcNWords; i += kWG) s_crc[i] = crc_tbl[kCrcPWords + i];
    }
    __syncthreads();

    constexpr uint32_t kWavesPerWG = kWG / kWave;
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t nw = gridDim.x * kWavesPerWG;
    uint32_t t = blockIdx.x * kWavesPerWG + wid;
    if (t >= ntiles) return;

    constexpr int P = rows_in_flight<K, MT>();
    uint64_t in_off[K], out_off[MT];
#pragma unroll
    for (int c = 0; c < K; c++) in_off[c] = uint64_t(plan->in_row[c]) * in_rs;
#pragma unroll
    for (int j = 0; j < MT; j++) out_off[j] = uint64_t(plan->out_row[j]) * out_rs;

    // walk this wave's tiles t, t+nw, ... keeping (block, tile-in-block) incrementally
    uint32_t blk = t / tpb;
    uint32_t tib = t - blk * tpb;
    const uint32_t step_b = nw / tpb, step_t = nw - step_b * tpb;

    for (; t < ntiles; t += nw) {
#ifndef RSMI_DIAG_CACHED
        const uint8_t* ib = in + uint64_t(blk) * in_bs;
        uint8_t* ob = out + uint64_t(blk) * out_bs;
#else  // diagnostic build (tools/Makefile diag-cached): tiles wrap onto the first 16
       // blocks (~7 MB, cache-resident), so the kernel's own issue rate (VALU, LDS, waits)
       // is what the launch time shows
        const uint8_t* ib = in + uint64_t(blk & 15) * in_bs;
        uint8_t* ob = out + uint64_t(blk & 15) * out_bs;
#endif
        const uint32_t ch = tib * kWave + lane;
        const uint32_t chl = ch < cpb ? ch : cpb - 1;  // load chunk, clamped: loads stay unconditional
        // UA: byte offset of the lane's 16-byte window
        const uint32_t win = UA ? (chl * 16u < S - 16u ? chl * 16u : S - 16u) : 0u;
        // CRC: leading bytes of the lane's window that belong to the previous chunk (the last
        // window only) count as zero, as per-dword keep masks; branch-free so the folds stay in
        // straight code
        u32x4 keep = {~0u, ~0u, ~0u, ~0u};
        if constexpr (CRC) {
            const int lead = int(chl * 16u - win);
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const int nb = lead - 4 * w;
                keep[w] = nb >= 4 ? 0u : nb <= 0 ? ~0u : ~((1u << (8 * nb)) - 1u);
            }
        }
        uint16_t* crc_tile = nullptr;  // this lane's chunk slot in shard 0 of the tile's block
        if constexpr (CRC) {
            crc_tile = crc_out + uint64_t(blk) * crc_slots * (uint64_t(tpb) * kWave) + ch;
            asm volatile("" : "+v"(crc_tile));
        }
        auto crc_store = [&](u32x4 x, uint32_t shard) {
            if constexpr (CRC) {
                x &= keep;
                const uint8_t* nbt = reinterpret_cast<const uint8_t*>(s_crc);
                uint32_t cr = 0;
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    uint32_t lo = (x[w] << 1) & 0x1E1E1E1Eu, hi = (x[w] >> 3) & 0x1E1E1E1Eu;
                    asm volatile("" : "+v"(lo), "+v"(hi));
                    uint32_t l[8];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int p = 4 * w + q;
                        l[2 * q] = *reinterpret_cast<const uint16_t*>(nbt + 64 * p + ((lo >> (8 * q)) & 0xFF));
                        l[2 * q + 1] = *reinterpret_cast<const uint16_t*>(nbt + 64 * p + 32 + ((hi >> (8 * q)) & 0xFF));
                    }
                    cr = xor3(cr, xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5])) ^ (l[6] ^ l[7]);
                }
                // unconditional: lanes past the row's end own padding slots (chunk pitch
                // tpb * 64), so no branch splits the column loop (a branch there lets the
                // compiler sink every column's GF math past it)
                crc_tile[uint64_t(shard) * (uint64_t(tpb) * kWave)] = uint16_t(cr);
            }
        };
        auto load_col = [&](int c) {
            if constexpr (UA)
                return ld16u<true>(ib + in_off[c] + win);
            else
                return ld16<true>(reinterpret_cast<const u32x4*>(ib + in_off[c]) + chl);
        };

        // Software pipeline over the K input rows: a ring of P rows in flight, one
        // scheduling region per row (sched_barrier) so the compiler cannot hoist every
        // load and table read to the top and blow the 128-VGPR budget.
        u32x4 v[P];
#pragma unroll
        for (int c = 0; c < P; c++) v[c] = load_col(c);

        // acc ^= p1^p2^p3 per column, folded two columns at a time with 3-input XORs:
        // even columns leave p3 pending, odd columns retire it (1.5 VALU per column).
        uint32_t acc[MT][4], pend[MT][4];

        // Opaque per-tile table base: stops LICM from hoisting all K*20 table words out
        // of the tile loop (which would pin ~200 VGPRs and drop occupancy to 1 wave).
        uint32_t tb = 0;
        asm volatile("" : "+v"(tb));
        const u32x4* tbl = s_tbl + tb;
        u32x4 Tn[5];
#pragma unroll
        for (int f = 0; f < 5; f++) Tn[f] = tbl[f];

#pragma unroll
        for (int c = 0; c < K; c++) {
            const int slot = c % P;
            u32x4 T[5];
#pragma unroll
            for (int f = 0; f < 5; f++) T[f] = Tn[f];
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const uint32_t x = u4get(v[slot], w);
                const uint32_t s1 = x & 0x07070707u;
                const uint32_t s2 = (x >> 3) & 0x07070707u;
                const uint32_t s3 = (x >> 6) & 0x03030303u;
#pragma unroll
                for (int j = 0; j < MT; j++) {
                    const uint32_t p1 = __builtin_amdgcn_perm(u4get(T[1], j), u4get(T[0], j), s1);
                    const uint32_t p2 = __builtin_amdgcn_perm(u4get(T[3], j), u4get(T[2], j), s2);
                    const uint32_t p3 = __builtin_amdgcn_perm(u4get(T[4], j), u4get(T[4], j), s3);
                    uint32_t& a = acc[j][w];
                    uint32_t& q = pend[j][w];
                    if (c == 0 && K == 1) {
                        a = xor3(p1, p2, p3);
                    } else if (c == 0) {
                        a = p1 ^ p2;
                        q = p3;
                    } else if (c & 1) {
                        a = xor3(a, p1, p2);
                        a = xor3(a, p3, q);
                    } else if (c == K - 1) {
                        a = xor3(a, p1, p2);
                        a ^= p3;
                    } else {
                        a = xor3(a, p1, p2);
                        q = p3;
                    }
                }
            }
            if constexpr (CRC) crc_store(v[slot], plan->in_row[c]);
            if (c + P < K) v[slot] = load_col(c + P);
            if (c + 1 < K) {
#pragma unroll
                for (int f = 0; f < 5; f++) Tn[f] = tbl[(c + 1) * 5 + f];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // Anchor the results outside the store predicate; otherwise the compiler sinks the
        // whole column pipeline into the `ch < cpb` branch and hoists every table read.
#pragma unroll
        for (int j = 0; j < MT; j++)
#pragma unroll
            for (int w = 0; w < 4; w++) asm volatile("" : "+v"(acc[j][w]));

        if (UA && ch < cpb) {
#pragma unroll
            for (int j = 0; j < MT; j++) {
                const u32x4 o = u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
                st16u<NT == 1>(ob + out_off[j] + win, o);
                if constexpr (CRC) {
                    crc_store(o, crc_out_slot0 + plan->out_row[j]);
                    __builtin_amdgcn_sched_barrier(0);  // one row's 32 table reads in flight at a time
                }
            }
        } else if (!UA && ch < cpb) {
            const uint32_t boff = ch * 16u;
            if (boff + 16u <= S) {
#pragma unroll
                for (int j = 0; j < MT; j++) {
                    const u32x4 o = u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
                    if constexpr (NT == 1)
                        __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(ob + out_off[j]) + ch);
                    else
                        *(reinterpret_cast<u32x4*>(ob + out_off[j]) + ch) = o;
                }
            } else {
                // the row's last, partial chunk (1..15 bytes): whole dwords, then bytes
#pragma unroll
                for (int j = 0; j < MT; j++) {
                    uint8_t* p = ob + out_off[j] + boff;
#pragma unroll
                    for (int w = 0; w < 4; w++) {
                        const uint32_t val = acc[j][w];
                        const uint32_t o = boff + 4u * w;
                        if (o + 4u <= S) {
                            *reinterpret_cast<uint32_t*>(p + 4 * w) = val;
                        } else if (o < S) {
                            p[4 * w] = uint8_t(val);
                            if (o + 1u < S) p[4 * w + 1] = uint8_t(val >> 8);
                            if (o + 2u < S) p[4 * w + 2] = uint8_t(val >> 16);
                        }
                    }
                }
            }
        }

        blk += step_b;
        tib += step_t;
        if (tib >= tpb) {
            tib -= tpb;
            blk++;
        }
    }
}

// Any K (<= 256), MT <= 4, any alignment: one byte-group of 4 per lane, bytewise memory
// access.  Correctness path for layouts the fast kernel does not accept.
__global__ __launch_bounds__(kWG) void rs_generic_kernel(const RsPlanDev* __restrict__ plan, const uint8_t* in,
                                                         uint8_t* out, uint64_t in_bs, uint64_t in_rs,
                                                         uint64_t out_bs, uint64_t out_rs, uint64_t S,
                                                         uint64_t nblocks) {
    __shared__ u32x4 s_tbl[kMaxK * kColDwords / 4];
    const int K = int(plan->k), MT = int(plan->mt);
    {
        const uint32_t* src = plan->tbl;
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_tbl);
        for (int i = threadIdx.x; i < K * kColDwords; i += kWG) dst[i] = src[i];
    }
    __syncthreads();
    const uint64_t groups = (S + 3) / 4;
    for (uint64_t b = blockIdx.y; b < nblocks; b += gridDim.y) {
        for (uint64_t g = uint64_t(blockIdx.x) * kWG + threadIdx.x; g < groups; g += uint64_t(gridDim.x) * kWG) {
            const uint64_t x0 = g * 4;
            const int nb = int(S - x0 < 4 ? S - x0 : 4);
            uint32_t acc[4] = {0, 0, 0, 0};
            for (int c = 0; c < K; c++) {
                const uint8_t* p = in + b * in_bs + uint64_t(plan->in_row[c]) * in_rs + x0;
                uint32_t x = 0;
                for (int i = 0; i < nb; i++) x |= uint32_t(p[i]) << (8 * i);
                const uint32_t s1 = x & 0x07070707u, s2 = (x >> 3) & 0x07070707u, s3 = (x >> 6) & 0x03030303u;
                const u32x4 T0 = s_tbl[c * 5 + 0], T1 = s_tbl[c * 5 + 1], T2 = s_tbl[c * 5 + 2],
                            T3 = s_tbl[c * 5 + 3], T4 = s_tbl[c * 5 + 4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    acc[j] ^= __builtin_amdgcn_perm(u4get(T1, j), u4get(T0, j), s1) ^
                              __builtin_amdgcn_perm(u4get(T3, j), u4get(T2, j), s2) ^
                              __builtin_amdgcn_perm(u4get(T4, j), u4get(T4, j), s3);
                }
            }
            for (int j = 0; j < MT; j++) {
                uint8_t* p = out + b * out_bs + uint64_t(plan->out_row[j]) * out_rs + x0;
                for (int i = 0; i < nb; i++) p[i] = uint8_t(acc[j] >> (8 * i));
            }
        }
    }
}

// Strided byte-row copy on the device (any src/dst alignment): rows x width bytes from
// src (row pitch spitch) to dst (row pitch dpitch).  Host staging uses it to turn the
// contiguous Split layout (pitch S, often odd) into the 16-B-aligned pitched layout and
// back, so PCIe transfers stay linear (odd-width 2-D DMA runs at 3-9 GB/s on MI355X).
// Each thread writes one naturally aligned destination dword; its 4 source bytes are
// funnel-shifted out of the two aligned source dwords that cover them.  A row's first
// and last dwords may be shared with a neighbouring row, so they are written bytewise.
__global__ __launch_bounds__(kWG) void rs_repitch_kernel(const uint8_t* __restrict__ src, uint64_t spitch,
                                                         uint8_t* __restrict__ dst, uint64_t dpitch, uint64_t width,
                                                         uint64_t rows) {
    const uint64_t dw_per_row = (width + 6) / 4 + 1;  // upper bound of dwords a row can touch
    const uint64_t total = dw_per_row * rows;
    for (uint64_t i = uint64_t(blockIdx.x) * kWG + threadIdx.x; i < total; i += uint64_t(gridDim.x) * kWG) {
        const uint64_t r = i / dw_per_row, q = i - r * dw_per_row;
        const uintptr_t drow = reinterpret_cast<uintptr_t>(dst + r * dpitch);
        const uintptr_t a = (drow & ~uintptr_t(3)) + 4 * q;  // aligned destination dword
        if (a >= drow + width) continue;
        const uint8_t* srow = src + r * spitch;
        const int64_t off = int64_t(a) - int64_t(drow);     // row offset of the dword's byte 0
        if (off >= 0 && uint64_t(off) + 4 <= width) {
            const uintptr_t sa = reinterpret_cast<uintptr_t>(srow) + uint64_t(off);
            const uint32_t* p = reinterpret_cast<const uint32_t*>(sa & ~uintptr_t(3));
            const uint32_t sh = uint32_t(sa & 3);
            const uint32_t lo = p[0];
            const uint32_t hi = sh ? p[1] : 0u;  // a second dword only when straddling
            *reinterpret_cast<uint32_t*>(a) = __builtin_amdgcn_alignbyte(hi, lo, sh);
        } else {
            for (int b = 0; b < 4; b++) {
                const int64_t o = off + b;
                if (o >= 0 && uint64_t(o) < width) reinterpret_cast<uint8_t*>(a)[b] = srow[o];
            }
        }
    }
}

void* repitch_kernel() { return reinterpret_cast<void*>(&rs_repitch_kernel); }

// ------------------------------------------------------------------ CRC-16 of shard rows
// R(row) of the datanode entry checksum (crc16.hpp has the algebra).  A wave owns one
// segment of kCrcSegTiles consecutive 1 KiB tiles of one row: each lane loads its 16-byte
// chunk of every tile (all loads in flight first), folds each chunk with positional LDS
// lookups -- 32 nibble lookups in 16-entry tables (every wave-wide lookup reads 8 distinct
// dwords in 8 distinct banks, so it never conflicts) -- and carries a running register
// across the tiles (A^1024 between tiles).  A
// Hillis-Steele scan over the 64 lanes (A^(16*2^j) per level) leaves the segment's value,
// relative to the segment's end, in lane 63; shifting it by (S - segment end) mod 32767
// bytes places it relative to the row's end, and one atomic XOR adds it into the row's
// word.  Bytes at or past S read as zero (zero bytes contribute nothing to R, they only
// move the reference point, which the final shift accounts for).
__device__ __forceinline__ uint32_t crc_pow(const uint16_t* sP, int i, uint32_t s) {
    return uint32_t(sP[i * 512 + (s & 0xFF)]) ^ uint32_t(sP[i * 512 + 256 + (s >> 8)]);
}

__device__ __forceinline__ uint32_t crc_nib_chunk(const uint8_t* nb, const u32x4& v) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        uint32_t lo = (v[w] << 1) & 0x1E1E1E1Eu, hi = (v[w] >> 3) & 0x1E1E1E1Eu;
        asm volatile("" : "+v"(lo), "+v"(hi));
        uint32_t l[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int p = 4 * w + q;
            l[2 * q] = *reinterpret_cast<const uint16_t*>(nb + 64 * p + ((lo >> (8 * q)) & 0xFF));
            l[2 * q + 1] = *reinterpret_cast<const uint16_t*>(nb + 64 * p + 32 + ((hi >> (8 * q)) & 0xFF));
        }
        c = xor3(c, xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5])) ^ (l[6] ^ l[7]);
    }
    return c;
}

template <bool ALIGNED>
__global__ __launch_bounds__(kWG) void rs_crc16_rows_kernel(const uint32_t* __restrict__ tbl,
                                                            const uint8_t* __restrict__ base, uint64_t bstride,
                                                            uint64_t rpitch, uint32_t nrows, uint64_t S, uint32_t tpb,
                                                            uint32_t nseg, uint64_t nitems, uint32_t* __restrict__ out,
                                                            uint64_t out_bs) {
    __shared__ uint32_t s_tbl[kCrcPWords + kCrcNWords];
    for (int i = threadIdx.x; i < kCrcPWords; i += kWG) s_tbl[i] = tbl[i];
    for (int i = threadIdx.x; i < kCrcNWords; i += kWG) s_tbl[kCrcPWords + i] = tbl[kCrcPWords + i];
    __syncthreads();
    const uint16_t* sP = reinterpret_cast<const uint16_t*>(s_tbl);
    const uint8_t* nb = reinterpret_cast<const uint8_t*>(sP + kCrcPWords * 2);  // N[32][16]

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
#pragma unroll
        for (int i = 0; i < kCrcSegTiles; i++) {
            if (uint32_t(i) < nt) {
                const uint32_t c = crc_nib_chunk(nb, v[i]);
                acc = crc_pow(sP, 10, acc) ^ c;  // previous tiles move 1 KiB further from the end
            }
        }
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const uint32_t w = crc_pow(sP, 4 + j, acc);  // 16 * 2^j bytes
            const uint32_t t = __shfl_up(w, 1u << j);
            if (lane >= (1u << j)) acc ^= t;
        }
        const int64_t seg_end = int64_t(t0 + nt) * (kWave * 16);
        int64_t e = (int64_t(S) - seg_end) % int64_t(kCrcOrder);
        if (e < 0) e += kCrcOrder;
#pragma unroll
        for (int i = 0; i < kCrcPowers; i++)
            if ((e >> i) & 1) acc = crc_pow(sP, i, acc);
        if (lane == kWave - 1) atomicXor(out + b * out_bs + r, acc);
    }
}

// The nibble rows pass, software-pipelined, for 16-byte-aligned rows (the default).  A wave
// issues the 8 tile loads of its next item before it folds the current one (two register sets,
// the loop unrolled by two), so its own fold covers the next item's memory latency instead of
// only the other waves on the SIMD.  Loads are unconditional -- chunks past the row's end read
// the row's last chunk and are masked to zero in the fold, and the prefetch past the last item
// re-reads that item -- so no load sits behind a branch and the compiler's vmcnt waits count
// only the older set.
__global__ __launch_bounds__(kWG) void rs_crc16_rows_pipe_kernel(const uint32_t* __restrict__ tbl,
                                                                 const uint8_t* __restrict__ base, uint64_t bstride,
                                                                 uint64_t rpitch, uint32_t nrows, uint64_t S,
                                                                 uint32_t tpb, uint32_t nseg, uint64_t nitems,
                                                                 uint32_t* __restrict__ out, uint64_t out_bs) {
    __shared__ uint32_t s_tbl[kCrcPWords + kCrcNWords];
    for (int i = threadIdx.x; i < kCrcPWords; i += kWG) s_tbl[i] = tbl[i];
    for (int i = threadIdx.x; i < kCrcNWords; i += kWG) s_tbl[kCrcPWords + i] = tbl[kCrcPWords + i];
    __syncthreads();
    const uint16_t* sP = reinterpret_cast<const uint16_t*>(s_tbl);
    const uint8_t* nb = reinterpret_cast<const uint8_t*>(sP + kCrcPWords * 2);

    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    const uint64_t last = (S - 1) / 16 * 16;  // the row's last chunk (S > 0)
    auto issue = [&](uint64_t it, u32x4(&v)[kCrcSegTiles]) {
        const uint32_t seg = uint32_t(it % nseg);
        const uint64_t rid = it / nseg;
        const uint64_t b = rid / nrows;
        const uint32_t r = uint32_t(rid - b * nrows);
        const uint8_t* row = base + b * bstride + uint64_t(r) * rpitch;
#pragma unroll
        for (int i = 0; i < kCrcSegTiles; i++) {
            const uint64_t off = (uint64_t(seg * kCrcSegTiles + i) * kWave + lane) * 16;
            v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + (off < last ? off : last)));
        }
    };
    auto finish = [&](uint64_t it, u32x4(&v)[kCrcSegTiles]) {
        const uint32_t seg = uint32_t(it % nseg);
        const uint64_t rid = it / nseg;
        const uint64_t b = rid / nrows;
        const uint32_t r = uint32_t(rid - b * nrows);
        const uint32_t t0 = seg * kCrcSegTiles;
        const uint32_t nt = tpb - t0 < uint32_t(kCrcSegTiles) ? tpb - t0 : uint32_t(kCrcSegTiles);
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < kCrcSegTiles; i++) {
            if (uint32_t(i) < nt) {
                if ((uint64_t(t0 + i) + 1) * (kWave * 16) > S) {  // wave-uniform: the row's last tile
                    const int64_t valid = int64_t(S) - int64_t((uint64_t(t0 + i) * kWave + lane) * 16);
#pragma unroll
                    for (int w = 0; w < 4; w++) {
                        const int64_t n = valid - 4 * w;
                        v[i][w] &= n >= 4 ? ~0u : n <= 0 ? 0u : (1u << (8 * n)) - 1u;
                    }
                }
                acc = crc_pow(sP, 10, acc) ^ crc_nib_chunk(nb, v[i]);  // earlier tiles move 1 KiB
            }
        }
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const uint32_t w = crc_pow(sP, 4 + j, acc);  // 16 * 2^j bytes
            const uint32_t t = __shfl_up(w, 1u << j);
            if (lane >= (1u << j)) acc ^= t;
        }
        const int64_t seg_end = int64_t(t0 + nt) * (kWave * 16);
        int64_t e = (int64_t(S) - seg_end) % int64_t(kCrcOrder);
        if (e < 0) e += kCrcOrder;
#pragma unroll
        for (int i = 0; i < kCrcPowers; i++)
            if ((e >> i) & 1) acc = crc_pow(sP, i, acc);
        if (lane == kWave - 1) atomicXor(out + b * out_bs + r, acc);
    };
    const uint64_t it0 = uint64_t(blockIdx.x) * (kWG / kWave) + wid;
    if (it0 >= nitems) return;
    const uint64_t itmax = nitems - 1;
    u32x4 va[kCrcSegTiles], vb[kCrcSegTiles];
    issue(it0, va);
    for (uint64_t it = it0;; it += 2 * nw) {
        issue(it + nw < itmax ? it + nw : itmax, vb);
        finish(it, va);
        if (it + nw > itmax) break;
        issue(it + 2 * nw < itmax ? it + 2 * nw : itmax, va);
        finish(it + nw, vb);
        if (it + 2 * nw > itmax) break;
    }
}

// R(row) from the fused kernels' per-chunk values (rs_fast_kernel CRC): one wave per row.
// A wave step covers 512 chunks: lane l loads chunks 8l..8l+7 as one 16-byte load (the chunk
// values are u16), combines them with a depth-3 tree (A^16, A^32, A^64), and its running
// register steps by A^8192 between wave steps; a lane scan then combines the lanes
// (A^(128*2^j)), and lane 63 shifts the total from the 8 KiB grid end to the row end.  Loads
// for 4 wave steps are issued ahead of the dependent chain.  The row's last chunk is relative
// to S (its window ends at S), so it first moves onto the 16-byte grid by A^(16*cpb - S).
// out[row] is written once (host memory allowed).
__global__ __launch_bounds__(kWG) void rs_crc16_combine_kernel(const uint32_t* __restrict__ tbl,
                                                               const uint16_t* __restrict__ chunks, uint32_t cpb,
                                                               uint32_t pitch, uint64_t S, uint64_t nrows,
                                                               uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(128))) uint32_t s_tbl[kCrcPWords];
    for (int i = threadIdx.x; i < kCrcPWords; i += kWG) s_tbl[i] = tbl[i];
    __syncthreads();
    auto pw = [&](int i, uint32_t x) { return crc_pow(reinterpret_cast<const uint16_t*>(s_tbl), i, x); };
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    constexpr uint32_t kStep = kWave * 8;  // chunks per wave step
    const uint32_t T = (cpb + kStep - 1) / kStep;
    const uint32_t lead = uint32_t((uint64_t(cpb) * 16 - S) % kCrcOrder);  // 16*cpb - S < 16
    for (uint64_t r = uint64_t(blockIdx.x) * (kWG / kWave) + wid; r < nrows; r += nw) {
        const uint16_t* rc = chunks + r * pitch;
        uint32_t acc = 0;
        for (uint32_t t0 = 0; t0 < T; t0 += 4) {
            u32x4 v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t g = (t0 + i) * kStep + 8 * lane;
                v[i] = u32x4{0, 0, 0, 0};
                if (t0 + i < T && g < pitch) v[i] = *reinterpret_cast<const u32x4*>(rc + g);  // pitch % 64 == 0
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if (t0 + i >= T) break;
                const uint32_t g = (t0 + i) * kStep + 8 * lane;
                uint32_t c[8];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    c[q] = (v[i][q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
                    if (g + q >= cpb) c[q] = 0;
                }
                if (g <= cpb - 1 && cpb - 1 < g + 8) {  // onto the grid: as if followed by 16*cpb - S zero bytes
                    const uint32_t q = cpb - 1 - g;
                    uint32_t x = 0;
#pragma unroll
                    for (int e = 0; e < 8; e++) x = uint32_t(e) == q ? c[e] : x;
#pragma unroll
                    for (int b = 0; b < 4; b++)
                        if ((lead >> b) & 1) x = pw(b, x);
#pragma unroll
                    for (int e = 0; e < 8; e++) c[e] = uint32_t(e) == q ? x : c[e];
                }
                const uint32_t p0 = pw(4, c[0]) ^ c[1], p1 = pw(4, c[2]) ^ c[3];
                const uint32_t p2 = pw(4, c[4]) ^ c[5], p3 = pw(4, c[6]) ^ c[7];
                const uint32_t x = pw(6, pw(5, p0) ^ p1) ^ (pw(5, p2) ^ p3);
                acc = pw(13, acc) ^ x;  // earlier wave steps move 8 KiB
            }
        }
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const uint32_t w = pw(7 + j, acc);  // 128 * 2^j bytes
            const uint32_t t = __shfl_up(w, 1u << j);
            if (lane >= (1u << j)) acc ^= t;
        }
        uint32_t val = uint32_t(__builtin_amdgcn_readlane(int(acc), kWave - 1));  // uniform: broadcast lookups
        int64_t e = (int64_t(S) - int64_t(T) * (kStep * 16)) % int64_t(kCrcOrder);
        if (e < 0) e += kCrcOrder;
        for (int i = 0; e; i++, e >>= 1)
            if (e & 1) val = pw(i, val);
        if (lane == 0) out[r] = val;
    }
}

void* crc16_combine_kernel() { return reinterpret_cast<void*>(&rs_crc16_combine_kernel); }

// aligned rows: the pipelined pass; any other layout: the plain nibble pass
void* crc16_rows_kernel(bool aligned) {
    return aligned ? reinterpret_cast<void*>(&rs_crc16_rows_pipe_kernel)
                   : reinterpret_cast<void*>(&rs_crc16_rows_kernel<false>);
}

// ------------------------------------------------------------------ dispatch table
// One kernel per (K, MT) and layout, with the cache policy of the shape (auto_cache_policy in
// rsmi_core.cpp): nontemporal stores unless the tile reads at least 4 rows per row it writes.
constexpr int auto_nt(int K, int MT) { return K >= 4 * MT ? 2 : 1; }

template <int K, int MT>
static void fill_km(FastKernelTable& t) {
    constexpr int NT = auto_nt(K, MT);
    t.fn[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, NT>);
    t.ua[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, NT, kMinWavesPerSimd, true>);
    // 2 waves/SIMD: the chunk folds need registers beyond the 128 the streaming kernels keep to
    t.ua_crc[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, NT, 2, true, true>);
}

template <int K>
static void fill_k(FastKernelTable& t) {
    fill_km<K, 1>(t);
    fill_km<K, 2>(t);
    fill_km<K, 3>(t);
    fill_km<K, 4>(t);
}

const FastKernelTable& fast_kernels() {
    static const FastKernelTable t = [] {
        FastKernelTable x{};
        fill_k<1>(x);
        fill_k<2>(x);
        fill_k<3>(x);
        fill_k<4>(x);
        fill_k<5>(x);
        fill_k<6>(x);
        fill_k<8>(x);
        fill_k<10>(x);
        fill_k<12>(x);
        fill_k<16>(x);
        return x;
    }();
    return t;
}

void* generic_kernel() { return reinterpret_cast<void*>(&rs_generic_kernel); }

}  // namespace rsmi
