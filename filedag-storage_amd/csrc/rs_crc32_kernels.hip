// rs_crc32_kernels.hip -- R(row) of shard rows for the mutcask value checksum (CRC-32 IEEE,
// kv/mutcask/cask.go:73-97; algebra in crc32.hpp), the CRC-32 sibling of
// rs_crc16_rows_kernel (rs_kernels.hip).
//
// Work item = (row, up to kCrc32SupGroups segments of kCrc32SegTiles = 8 consecutive 1 KiB
// tiles).  Each lane loads its 16-byte chunk of every tile of a segment and folds each
// chunk with 32 nibble lookups into 16-entry u32 tables (a wave-wide lookup into one table
// touches at most 16 dwords in 16 distinct banks, so it never conflicts).  Tile t of the
// segment has its own tables (NT[t] = A^(1024 * (7 - t)) o N), so every chunk's value comes
// out relative to the end of the segment's 8-tile span with no per-tile shift.  A
// Hillis-Steele scan over the 64 lanes (A^(16 * 2^j) per level) leaves the segment's value in
// lane 63, which moves it to the row's end and XORs it into the row's word.  With
// S = 8192 q + r, inner segment j moves by 8192 (q - j - 1) + r; the last segment's span ends
// at 8192 q (r = 0: the row's end) or 8192 (q + 1) = the row's end + 8192 - r, so it moves by
// r - 8192.  A^r arrives by value (per launch), A^(8192 * 2^i) and A^-8192 from global
// memory, all in column form, one column per lane, applied with a DPP XOR reduction (~10
// instructions, no LDS -- the kernel's binding resource).  Per 8 KiB item: 256 fold lookups +
// 48 scan lookups; the earlier form (a per-tile A^1024 and a chained end shift through
// nibble tables) took ~430.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "crc32.hpp"
#include "rs_device.hpp"
#include "rs_plan.hpp"

namespace rsmi {

namespace {

// A^(16 * 2^j) of s from a nibble-sliced table t[8][16] (512 B): the nibble offsets come out
// of two masked words, as in the chunk fold
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

// M(s) for a matrix M held lane-distributed (lane l < 32 of col holds M's image of 1 << l;
// lanes 32-63 repeat them) and a wave-uniform s: each lane keeps its column if bit l of s is
// set, an XOR scan over each 16-lane row (DPP row_shr 1, 2, 4, 8) leaves the rows' sums in
// lanes 15 and 31.  No SGPR copies of the matrix, no LDS.
__device__ __forceinline__ uint32_t dpp_xor_shr(uint32_t x, int n) {
    switch (n) {  // DPP control must be a constant: row_shr:n = 0x110 + n
        case 1: return x ^ uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, false));
        case 2: return x ^ uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, false));
        case 4: return x ^ uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, false));
        default: return x ^ uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, false));
    }
}

__device__ __forceinline__ uint32_t apply_lanes(uint32_t col, uint32_t s, uint32_t l32) {
    uint32_t x = ((s >> l32) & 1u) ? col : 0u;
    x = dpp_xor_shr(x, 1);
    x = dpp_xor_shr(x, 2);
    x = dpp_xor_shr(x, 4);
    x = dpp_xor_shr(x, 8);
    return uint32_t(__builtin_amdgcn_readlane(int(x), 15)) ^ uint32_t(__builtin_amdgcn_readlane(int(x), 31));
}

// R(chunk) relative to the end of its table set's span: 32 nibble lookups into the 16-entry
// u32 tables t[32][16] (64 B each; byte offsets 4 x nibble)
__device__ __forceinline__ uint32_t crc32_nib_chunk(const uint8_t* t, const u32x4& v) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        uint32_t lo = (v[w] << 2) & 0x3C3C3C3Cu, hi = (v[w] >> 2) & 0x3C3C3C3Cu;
        asm volatile("" : "+v"(lo), "+v"(hi));  // keep the two masks (one extract per offset)
        uint32_t l[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int p = 4 * w + q;
            l[2 * q] = *reinterpret_cast<const uint32_t*>(t + 128 * p + ((lo >> (8 * q)) & 0xFF));
            l[2 * q + 1] = *reinterpret_cast<const uint32_t*>(t + 128 * p + 64 + ((hi >> (8 * q)) & 0xFF));
        }
        c = xor3(c, xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5])) ^ (l[6] ^ l[7]);
    }
    return c;
}

// The item's value -> row word: lane scan (lane 63 ends with the value relative to the end of
// group gl), the shift to the row's end, one atomic XOR.  With S = 8192 q8 + r8, a group gl < q8
// moves by 8192 (q8 - gl - 1) + r8; a group that ends past S (the row's last one, r8 != 0) moves
// back by 8192 (gl - q8 + 1) - r8.  Unaligned rows fold on the memory's grid, where every group
// ends mis bytes earlier than on the row's (and a row may reach into group q8 + 1): mis more.
// The shift of a wave-uniform value relative to the end of group gl to the row's end, then one
// atomic XOR into the row's word (the second half of crc32_item_out).
__device__ __forceinline__ void crc32_shift_out(const uint32_t* sC, uint32_t col_r, uint32_t lane, uint32_t l32,
                                                uint32_t val, uint32_t gl, uint32_t q8, uint32_t mis, uint32_t* word) {
    if (gl < q8) {
        // whole segments, then the remainder r8
        uint32_t a = q8 - gl - 1;
        for (int i = 0; a; i++, a >>= 1)
            if (a & 1) val = apply_lanes(sC[32 * i + l32], val, l32);
    } else {
        for (uint32_t g = q8; g <= gl; g++) val = apply_lanes(sC[32 * kCrc32SegPowers + l32], val, l32);  // A^-8192
    }
    val = apply_lanes(col_r, val, l32);
#pragma unroll
    for (int i = 0; i < kCrc32MisPowers; i++)
        if ((mis >> i) & 1) val = apply_lanes(sC[32 * (kCrc32SegPowers + 1 + i) + l32], val, l32);
    if (lane == 0) atomicXor(word, val);
}

__device__ __forceinline__ void crc32_item_out(const uint32_t* sS, const uint32_t* sC, uint32_t col_r, uint32_t lane,
                                               uint32_t l32, uint32_t acc, uint32_t gl, uint32_t q8, uint32_t mis,
                                               uint32_t* word) {
#pragma unroll
    for (int j = 0; j < kCrc32ScanPowers; j++) {
        const uint32_t w = pow_nib(sS + j * kCrc32PowWords, acc);  // 16 * 2^j bytes
        const uint32_t t = __shfl_up(w, 1u << j);
        if (lane >= (1u << j)) acc ^= t;
    }
    const uint32_t val = uint32_t(__builtin_amdgcn_readlane(int(acc), kWave - 1));  // wave-uniform from here on
    crc32_shift_out(sC, col_r, lane, l32, val, gl, q8, mis, word);
}

// Position of item `it` (nsup items per row): its row, first tile and tile count.
struct Crc32Item {
    uint64_t b;
    uint32_t r, t0, nt;
};
__device__ __forceinline__ Crc32Item crc32_item(uint64_t it, uint32_t nsup, uint32_t nrows, uint32_t tpb) {
    constexpr uint32_t kSup = kCrc32SupGroups * kCrc32SegTiles;
    Crc32Item x;
    uint32_t sup;
    if (it < (uint64_t(1) << 32)) {  // 32-bit divisions (scalar), the common case
        const uint32_t i32 = uint32_t(it), rid = i32 / nsup;
        sup = i32 - rid * nsup;
        const uint32_t b = rid / nrows;
        x.b = b;
        x.r = rid - b * nrows;
    } else {
        sup = uint32_t(it % nsup);
        const uint64_t rid = it / nsup;
        x.b = rid / nrows;
        x.r = uint32_t(rid - x.b * nrows);
    }
    x.t0 = sup * kSup;
    x.nt = tpb - x.t0 < kSup ? tpb - x.t0 : kSup;
    return x;
}

}  // namespace

// LDS staging shared by the rows passes: NT | SN | SG (19 KiB); SC stays in global memory
#define RSMI_CRC32_ROWS_STAGE()                                                                           \
    __shared__ uint32_t s_tbl[kCrc32LdsWords];                                                            \
    for (int i = threadIdx.x; i < kCrc32LdsWords; i += kWG) s_tbl[i] = tbl[i];                            \
    __syncthreads();                                                                                      \
    const uint8_t* nb = reinterpret_cast<const uint8_t*>(s_tbl);                                          \
    const uint32_t* sS = s_tbl + kCrc32FoldWords;                                                         \
    const uint32_t* sG = sS + kCrc32ScanPowers * kCrc32PowWords;                                          \
    const uint32_t* sC = tbl + kCrc32LdsWords;                                                            \
    const uint32_t q8 = uint32_t(S / (kCrc32SegTiles * 1024));                                           \
    const uint32_t l32 = threadIdx.x & 31;                                                                \
    uint32_t col_r = 0; /* A^r8, lane-distributed */                                                      \
    _Pragma("unroll") for (int b_ = 0; b_ < 32; b_++) col_r = l32 == uint32_t(b_) ? sh.col[b_] : col_r;

// tbl: NT[8][32][16] | SN[6][8][16] | SG[8][16] (staged in LDS) | SC[24][32] (rs_plan.hpp).
// An item is up to kCrc32SupGroups 8-tile groups of one row: each group folds through the
// tile-set tables into a value relative to its end, a running register steps by A^8192 (SG)
// between groups, and the scan and the end shift run once per item (8-tile items spent a
// quarter of the pass there).  Software-pipelined as rs_crc16_rows_pipe_kernel: a wave works in
// units of half a group (4 tiles) and issues the loads of its next unit, of this item or its next
// one, before it folds the current one (two register sets of 16 VGPRs, the loop unrolled by two).
// Loads are unconditional: chunks past the row's end re-read the row's last chunk and are masked
// to zero in the fold, and the prefetch past the wave's last unit re-reads that unit.
// UA: rows at any alignment (the Split layout) fold on the memory's 16-byte grid, as the CRC-16
// matrix-core pass does: loads from the aligned chunk at or below the row's first byte (its mis
// leading bytes masked), the launch's tiles per row counting mis + S <= S + 15 bytes, and the end
// shift mis bytes longer.
template <bool UA>
__global__ __launch_bounds__(kWG) void rs_crc32_rows_pipe_kernel(const uint32_t* __restrict__ tbl,
                                                                 const uint8_t* __restrict__ base, uint64_t bstride,
                                                                 uint64_t rpitch, uint32_t nrows, uint64_t S,
                                                                 uint32_t tpb, uint32_t nseg, uint32_t nsup,
                                                                 uint64_t nitems, uint32_t* __restrict__ out,
                                                                 uint64_t out_bs, Crc32Shift sh) {
    RSMI_CRC32_ROWS_STAGE()
    constexpr int kU = kCrc32SegTiles / 2;  // tiles per unit
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    struct Unit {
        uint64_t it;
        Crc32Item x;
        uint32_t h;  // half group within the item
    };
    auto at = [&](uint64_t it) -> Unit { return Unit{it, crc32_item(it, nsup, nrows, tpb), 0}; };
    auto next = [&](const Unit& u) -> Unit {
        if ((u.h + 1) * kU < u.x.nt) return Unit{u.it, u.x, u.h + 1};
        return at(u.it + nw);
    };
    // the row's misalignment (wave-uniform; 0 for aligned rows)
    auto misof = [&](const Crc32Item& x) -> uint32_t {
        const uint8_t* row = base + x.b * bstride + uint64_t(x.r) * rpitch;
        return UA ? uint32_t(__builtin_amdgcn_readfirstlane(int(reinterpret_cast<uintptr_t>(row) & 15u))) : 0u;
    };
    auto issue = [&](const Unit& u, u32x4(&v)[kU]) {
        const uint32_t mis = misof(u.x);
        const uint8_t* rowa = base + u.x.b * bstride + uint64_t(u.x.r) * rpitch - mis;
        const uint64_t last = (S + mis - 1) / 16 * 16;  // the aligned chunk holding the row's last byte
#pragma unroll
        for (int i = 0; i < kU; i++) {
            const uint64_t off = (uint64_t(u.x.t0 + u.h * kU + i) * kWave + lane) * 16;
            v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowa + (off < last ? off : last)));
        }
    };
    uint32_t acc = 0, gs = 0;
    auto finish = [&](const Unit& u, u32x4(&v)[kU]) {
        const Crc32Item& x = u.x;
        const uint32_t u0 = u.h * kU, t0 = x.t0 + u0;
        const uint32_t nt = x.nt - u0 < uint32_t(kU) ? x.nt - u0 : uint32_t(kU);
        const uint8_t* gt = nb + 2048 * kU * (u.h & 1);  // table sets of this half of the group
        const uint32_t mis = misof(x);
        const uint64_t Sm = S + mis;  // the row's end on the memory grid
#pragma unroll
        for (int i = 0; i < kU; i++) {
            if (uint32_t(i) < nt) {
                if ((uint64_t(t0 + i) + 1) * (kWave * 16) > Sm) {  // wave-uniform: the row's last tile
                    const int64_t valid = int64_t(Sm) - int64_t((uint64_t(t0 + i) * kWave + lane) * 16);
#pragma unroll
                    for (int w = 0; w < 4; w++) {
                        const int64_t n = valid - 4 * w;
                        v[i][w] &= n >= 4 ? ~0u : n <= 0 ? 0u : (1u << (8 * n)) - 1u;
                    }
                }
                if (UA && t0 + i == 0 && mis != 0u && lane == 0) {  // the bytes before the row
#pragma unroll
                    for (int w = 0; w < 4; w++) {
                        const int n = int(mis) - 4 * w;
                        v[i][w] &= n >= 4 ? 0u : n <= 0 ? ~0u : ~((1u << (8 * n)) - 1u);
                    }
                }
                gs ^= crc32_nib_chunk(gt + 2048 * i, v[i]);
            }
        }
        const bool item_end = u0 + kU >= x.nt;
        if ((u.h & 1) || item_end) {  // the group is complete
            acc = pow_nib(sG, acc) ^ gs;  // earlier groups move 8 KiB further from the end
            gs = 0;
        }
        if (item_end) {
            crc32_item_out(sS, sC, col_r, lane, l32, acc, (x.t0 + x.nt - 1) / kCrc32SegTiles, q8, mis,
                           out + x.b * out_bs + x.r);
            acc = 0;
        }
    };
    const uint64_t it0 = uint64_t(blockIdx.x) * (kWG / kWave) + wid;
    if (it0 >= nitems) return;
    Unit cur = at(it0);
    u32x4 va[kU], vb[kU];
    issue(cur, va);
    for (;;) {
        Unit nx = next(cur);
        bool more = nx.it < nitems;
        issue(more ? nx : cur, vb);
        finish(cur, va);
        if (!more) break;
        cur = nx;
        nx = next(cur);
        more = nx.it < nitems;
        issue(more ? nx : cur, va);
        finish(cur, vb);
        if (!more) break;
        cur = nx;
    }
}

// The rows pass with the fold on the matrix cores: rs_crc16_rows_mfma_kernel (rs_kernels.hip)
// with a 32-bit register.  B = the tile's data, one data bit per fp4 nibble (forms x & 0x11..,
// 0x22.., 0x44.., (x >> 1) & 0x44..), column m = lane & 15, k block j = lane >> 4; two MFMAs per
// form, A = the weights of CRC bits 0-15 and 16-31 of tile t of an 8-tile group (MW, 64 KiB of
// LDS shared by a workgroup of 8 waves); a group's counts accumulate in two f32 quads (at most
// 4096 per count, exact) and eight ballots give class m's 32-bit value in lane m (chunks m,
// m + 16, m + 32, m + 48 of the group's tiles, relative to the end of chunk 48 + m of tile 7).
// Groups step by A^8192 (SG); at the item's end a 4-level scan over lanes 0..15 (SN, A^(16 2^j))
// takes lane 15 to the end of the item's last group, and crc32_shift_out moves it to the row's
// end.  UA: the memory-grid fold of the CRC-16 pass (loads from the aligned chunk at or below the
// row's first byte, its mis leading bytes masked, the end shift mis bytes longer).
typedef int mfma32_v8i __attribute__((ext_vector_type(8)));
typedef float mfma32_v4f __attribute__((ext_vector_type(4)));

template <bool UA>
__global__ __launch_bounds__(kCrc32MfmaWG) void rs_crc32_rows_mfma_kernel(
    const uint32_t* __restrict__ tbl, const uint8_t* __restrict__ base, uint64_t bstride, uint64_t rpitch,
    uint32_t nrows, uint64_t S, uint32_t tpb, uint32_t nseg, uint32_t nsup, uint64_t nitems,
    uint32_t* __restrict__ out, uint64_t out_bs, Crc32Shift sh) {
    constexpr int kWWords = kCrc32MWWords * kCrc32MfmaTiles / kCrc32SegTiles;  // the staged tiles' weights
    __shared__ u32x4 s_w[kWWords / 4];
    __shared__ uint32_t s_pw[6 * kCrc32PowWords];  // SN[0..3] | SG | SG4
    {
        // half groups: tiles 4..7 of MW weigh a half group's tiles relative to its end
        const u32x4* w = reinterpret_cast<const u32x4*>(tbl + kCrc32MWOff + (kCrc32MWWords - kWWords));
        for (int i = threadIdx.x; i < kWWords / 4; i += kCrc32MfmaWG) s_w[i] = w[i];
        for (int i = threadIdx.x; i < 4 * kCrc32PowWords; i += kCrc32MfmaWG) s_pw[i] = tbl[kCrc32FoldWords + i];
        for (int i = threadIdx.x; i < kCrc32PowWords; i += kCrc32MfmaWG) {
            s_pw[4 * kCrc32PowWords + i] = tbl[kCrc32FoldWords + 6 * kCrc32PowWords + i];
            s_pw[5 * kCrc32PowWords + i] = tbl[kCrc32SG4Off + i];
        }
    }
    __syncthreads();
    const uint32_t* sS = s_pw;
    const uint32_t* sG = s_pw + 4 * kCrc32PowWords;
    const uint32_t* sG4 = s_pw + 5 * kCrc32PowWords;
    const uint32_t* sC = tbl + kCrc32LdsWords;
    const uint32_t q8 = uint32_t(S / (kCrc32SegTiles * 1024));
    const uint32_t l32 = threadIdx.x & 31;
    uint32_t col_r = 0;  // A^r8, lane-distributed
#pragma unroll
    for (int b = 0; b < 32; b++) col_r = l32 == uint32_t(b) ? sh.col[b] : col_r;
    constexpr uint32_t kWaves = kCrc32MfmaWG / kWave;
    const uint32_t lane = threadIdx.x & (kWave - 1), m = lane & 15u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * kWaves;
    for (uint64_t it = uint64_t(blockIdx.x) * kWaves + wid; it < nitems; it += nw) {
        const Crc32Item x = crc32_item(it, nsup, nrows, tpb);
        const uint8_t* row = base + x.b * bstride + uint64_t(x.r) * rpitch;
        const uint32_t mis = UA ? uint32_t(__builtin_amdgcn_readfirstlane(int(reinterpret_cast<uintptr_t>(row) & 15u))) : 0u;
        const uint8_t* rowa = row - mis;
        const uint64_t Sm = mis + S;  // the row's end on the memory grid
        const uint64_t lasta = (Sm - 1) / 16 * 16;
        uint32_t acc = 0;  // lanes 0..15: class m's running value
        for (uint32_t g0 = 0; g0 < x.nt; g0 += kCrc32SegTiles) {
            const uint32_t t0 = x.t0 + g0;
            const uint32_t nt = x.nt - g0 < uint32_t(kCrc32SegTiles) ? x.nt - g0 : uint32_t(kCrc32SegTiles);
            u32x4 v[kCrc32SegTiles];
#pragma unroll
            for (int i = 0; i < kCrc32SegTiles; i++) {
                const uint64_t off = (uint64_t(t0 + i) * kWave + lane) * 16;  // unconditional, clamped
                v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowa + (off < lasta ? off : lasta)));
            }
            uint32_t gval = 0;  // the group's value, relative to its end
#pragma unroll
            for (int hh = 0; hh < kCrc32SegTiles / kCrc32MfmaTiles; hh++) {
            mfma32_v4f c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = hh * kCrc32MfmaTiles; i < (hh + 1) * kCrc32MfmaTiles; i++) {
                if (uint32_t(i) < nt) {
                    u32x4 d = v[i];
                    if ((uint64_t(t0 + i) + 1) * (kWave * 16) > Sm) {  // wave-uniform: the row's last tile
                        const int64_t valid = int64_t(Sm) - int64_t((uint64_t(t0 + i) * kWave + lane) * 16);
#pragma unroll
                        for (int w = 0; w < 4; w++) {
                            const int64_t n = valid - 4 * w;
                            d[w] &= n >= 4 ? ~0u : n <= 0 ? 0u : (1u << (8 * n)) - 1u;
                        }
                    }
                    if (UA && t0 + i == 0 && mis != 0u && lane == 0) {  // the bytes before the row
#pragma unroll
                        for (int w = 0; w < 4; w++) {
                            const int n = int(mis) - 4 * w;
                            d[w] &= n >= 4 ? 0u : n <= 0 ? ~0u : ~((1u << (8 * n)) - 1u);
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        mfma32_v8i bd;
#pragma unroll
                        for (int w = 0; w < 4; w++)
                            bd[w] = int(q < 3 ? d[w] & (0x11111111u << q) : (d[w] >> 1) & 0x44444444u);
                        bd[4] = bd[5] = bd[6] = bd[7] = 0;
                        const int ti = i % kCrc32MfmaTiles;  // the tile's weights (relative to the read-out's end)
                        const u32x4 w0 = s_w[((ti * 4 + q) * 2 + 0) * kWave + lane];
                        const u32x4 w1 = s_w[((ti * 4 + q) * 2 + 1) * kWave + lane];
                        const mfma32_v8i a0 = {int(w0[0]), int(w0[1]), int(w0[2]), int(w0[3]), 0, 0, 0, 0};
                        const mfma32_v8i a1 = {int(w1[0]), int(w1[1]), int(w1[2]), int(w1[3]), 0, 0, 0, 0};
                        c0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a0, bd, c0, 4, 4, 0, 127, 0, 127);
                        c1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a1, bd, c1, 4, 4, 0, 127, 0, 127);
                    }
                }
            }
            // parity bits -> class m's 32-bit value: bit n of half h is bit 16 (n >> 2) + m of
            // ballot n & 3 of that half's accumulator
            uint32_t Y0 = 0, Y1 = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint64_t b0 = __builtin_amdgcn_ballot_w64((int(c0[i]) & 1) != 0);
                const uint64_t b1 = __builtin_amdgcn_ballot_w64((int(c1[i]) & 1) != 0);
                const uint32_t lo0 = uint32_t(b0) >> m, hi0 = uint32_t(b0 >> 32) >> m;
                const uint32_t lo1 = uint32_t(b1) >> m, hi1 = uint32_t(b1 >> 32) >> m;
                Y0 |= ((lo0 & 0x10001u) | ((hi0 & 0x10001u) << 8)) << i;
                Y1 |= ((lo1 & 0x10001u) | ((hi1 & 0x10001u) << 8)) << i;
            }
            const uint32_t val = ((Y0 & 0x0F0Fu) | ((Y0 >> 12) & 0xF0F0u)) |
                                 (((Y1 & 0x0F0Fu) | ((Y1 >> 12) & 0xF0F0u)) << 16);
            gval = (hh == 0 ? 0u : pow_nib(sG4, gval)) ^ val;  // an earlier half moves 4 KiB further
            }
            acc = (g0 == 0 ? 0u : pow_nib(sG, acc)) ^ gval;  // earlier groups move 8 KiB further from the end
        }
        // classes -> the end of the item's last group: lane 15 takes sum_m A^(16 (15 - m)) (class m)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t w = pow_nib(sS + j * kCrc32PowWords, acc);  // 16 * 2^j bytes
            const uint32_t t = __shfl_up(w, 1u << j);
            if (m >= (1u << j)) acc ^= t;
        }
        const uint32_t val = uint32_t(__builtin_amdgcn_readlane(int(acc), 15));  // wave-uniform from here
        crc32_shift_out(sC, col_r, lane, l32, val, (x.t0 + x.nt - 1) / kCrc32SegTiles, q8, mis,
                        out + x.b * out_bs + x.r);
    }
}

void* crc32_rows_mfma_kernel(bool aligned) {
    return aligned ? reinterpret_cast<void*>(&rs_crc32_rows_mfma_kernel<false>)
                   : reinterpret_cast<void*>(&rs_crc32_rows_mfma_kernel<true>);
}

void* crc32_rows_kernel(bool aligned) {
    return aligned ? reinterpret_cast<void*>(&rs_crc32_rows_pipe_kernel<false>)
                   : reinterpret_cast<void*>(&rs_crc32_rows_pipe_kernel<true>);
}

}  // namespace rsmi
