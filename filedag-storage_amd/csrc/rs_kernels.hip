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
#include <type_traits>

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

// A table copied into LDS in two steps: its words are loaded into registers at the kernel's
// start and written to LDS (then one barrier) once the wave's first rows are in flight, so the
// table's latency and the rows' overlap instead of adding up (a per-block call over PCIe is
// latency-bound, tools/latency.cpp).  Every thread of the workgroup takes part.
template <int N>
struct LdsTable {
    static constexpr int kPer = (N + kWG - 1) / kWG;
    uint32_t r[kPer];
    __device__ __forceinline__ void load(const uint32_t* __restrict__ src) {
#pragma unroll
        for (int i = 0; i < kPer; i++) {
            const int x = int(threadIdx.x) + i * kWG;
            r[i] = x < N ? src[x] : 0u;
        }
    }
    __device__ __forceinline__ void store(uint32_t* dst) const {
#pragma unroll
        for (int i = 0; i < kPer; i++) {
            const int x = int(threadIdx.x) + i * kWG;
            if (x < N) dst[x] = r[i];
        }
    }
};

// Block blk's rows: at p + blk * bs, or, over a table of block bases (TB, BlockBases), at the
// table's entry for blk plus the offset p (one scalar load from the kernel arguments per wave).
template <bool TB, class T>
__device__ __forceinline__ T* block_rows(const BasesArg<TB>& bases, T* p, uint32_t blk, uint64_t bs) {
    if constexpr (TB)
        return reinterpret_cast<T*>(uintptr_t(bases.b[blk]) + reinterpret_cast<uintptr_t>(p));
    else
        return p + uint64_t(blk) * bs;
}

// A table launch's completion release (BlockBases::done_flag; every workgroup calls it once, as
// its last act, with all its waves).  Every thread first releases its own stores at system scope
// (buffer_wbl2 + s_waitcnt vmcnt(0) in every wave): the barrier alone does not wait for other
// waves' stores on gfx950 (back-off barrier, and a workgroup-scope release emits no vmcnt wait in
// non-tgsplit mode), so without the per-wave fence waves 1..3 could still have parity or R(shard)
// stores in flight to page-locked host memory when wave 0 counts.  After the barrier, one
// system-scope fetch-add counts the workgroup, and the launch's last workgroup resets the counter
// for the next launch and releases the flag.  A table without a flag (and every table-less
// instantiation) skips all of it.  ISA check: DESIGN.md §4.3.
#ifndef RSMI_FLAG_FENCE  // 0: round 5's release (wave 0 only), for the cost A/B (tools/Makefile variant)
#define RSMI_FLAG_FENCE 1
#endif
template <bool TB>
__device__ __forceinline__ void launch_done(const BasesArg<TB>& bases) {
    if constexpr (TB) {
        if (!bases.done_flag) return;  // kernel argument: uniform over the launch
        if constexpr (RSMI_FLAG_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope, every thread
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t old = __hip_atomic_fetch_add(bases.done_ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
            if (old + 1u == gridDim.x) {
                __hip_atomic_store(bases.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(bases.done_flag, bases.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// K inputs, MT (<= 4) outputs, one 16-byte chunk per lane per row.
// NT: cache policy, 1 = nontemporal loads and stores (write-heavy tiles), 2 = nontemporal
// loads, default stores (tiles that read at least 4 rows per row written); DESIGN.md §4.1.
// WPS: waves per SIMD the register allocation must allow.
// UA: rows at any byte alignment and pitch (S >= 16).  A lane's 16-byte window starts at
// min(16*ch, S - 16): the row's last window overlaps the one before it instead of running
// past S, so loads never leave [0, S) and every store is a whole 16-byte window (the
// overlapped bytes get the same value from both lanes).  This serves the Split layout itself
// (rows back to back at pitch S, odd for RS(10,4)) and page-locked host memory read and
// written in place over PCIe.
// CRC (encode plans only: input row c is shard c, output row j shard K + j): also fold every
// row the tile reads or writes into CRC-16 values (crc16.hpp).  Lane q of each 4-lane quad
// folds its 16-byte chunk with the quad-relative nibble tables Q (relative to the end of the
// quad), two DPP XORs sum the quad, and lane q keeps rows r = q mod 4: one dword store per two
// such rows leaves the tile's record rec[(block * tpb + tile) * ns2 * 64 + s2 * 64 + lane]
// (rows 8 s2 + q and 8 s2 + 4 + q of quad lane / 4, u16 each).  Bytes at or past S count as
// zero (aligned layouts: the row's last chunk is masked).  UA: the row's last window ends at S,
// not on the 16-byte grid, so its chunk stays out of the quad sums and its value (relative to S)
// goes to tail[block * (K + MT) + r].  rs_crc16_combine_kernel turns records and tails into
// R(row).
// Launch geometry: one tile per wave; the loop strides over further tiles only
// when the caller caps the grid (option waves_per_cu).
// TB: the blocks lie where a table of block bases says (BlockBases: a coalesced group of callers'
// own page-locked buffers, one launch for the group); in / out are offsets from each base.
#ifndef RSMI_ROWS_FIRST  // 1: the coding table staged after the first rows are issued (A/B)
#define RSMI_ROWS_FIRST 0
#endif
template <int K, int MT, int NT, int WPS = kMinWavesPerSimd, bool UA = false, bool CRC = false, bool TB = false>
__global__ __launch_bounds__(kFastWG, WPS) void rs_fast_kernel(const RsPlanDev* __restrict__ plan,
                                                       const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                       uint64_t in_bs, uint64_t in_rs, uint64_t out_bs,
                                                       uint64_t out_rs, uint32_t S, uint32_t cpb, uint32_t tpb,
                                                       uint32_t ntiles, const uint32_t* __restrict__ crc_tbl,
                                                       uint32_t* __restrict__ crc_rec, uint32_t* __restrict__ crc_tail,
                                                       BasesArg<TB> bases) {
    static_assert(NT == 1 || NT == 2, "cache policy 1 or 2");
    constexpr int NSH = K + MT;            // CRC: shards of the block (encode plans)
    constexpr int NSL = (NSH + 3) / 4;     // CRC: rows each lane keeps (r = q mod 4)
    __shared__ u32x4 s_tbl[K * kColDwords / 4];
    __shared__ uint32_t s_crc[CRC ? kCrcQWords : 1];
#if RSMI_ROWS_FIRST
    // the coding table is loaded into registers here and written to LDS (stage, one barrier) once
    // the wave's first rows are in flight, so a wave's first HBM loads do not wait for the table's
    // round trip and the barrier
    static_assert(kFastWG == kWG, "LdsTable stages with kWG threads");
    LdsTable<K * kColDwords> lt;
    lt.load(plan->tbl);
    if constexpr (CRC)
        for (int i = threadIdx.x; i < kCrcQWords; i += kFastWG) s_crc[i] = crc_tbl[kCrcQOff + i];
    __builtin_amdgcn_sched_barrier(0);
    bool staged = false;  // wave-uniform: every wave passes the staging barrier exactly once
    auto stage = [&]() {
        if (staged) return;
        lt.store(reinterpret_cast<uint32_t*>(s_tbl));
        __syncthreads();
        staged = true;
    };
#else
    {
        const uint32_t* src = plan->tbl;
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_tbl);
        for (int i = threadIdx.x; i < K * kColDwords; i += kFastWG) dst[i] = src[i];
        if constexpr (CRC)
            for (int i = threadIdx.x; i < kCrcQWords; i += kFastWG) s_crc[i] = crc_tbl[kCrcQOff + i];
    }
    __syncthreads();
    auto stage = [] {};
#endif

    constexpr uint32_t kWavesPerWG = kFastWG / kWave;
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t nw = gridDim.x * kWavesPerWG;
    // UA: workgroups renumbered so each XCD (the dispatcher deals workgroups round-robin over
    // the 8 XCDs) takes one contiguous eighth of the tiles.  A row's 1 KiB tile at an odd address
    // shares its first and last 64-byte lines with the neighbouring tiles; with the neighbours on
    // the same XCD those lines come from one L2 (Split layout: encode +4-5%).
    // Aligned layouts share no lines and keep the plain order (re-measured in round 2: +1.2% on
    // RS(10,4) 256 KiB, -1.3 to -3% on the other BASELINE shapes, profiles/r02/cfg_ab_xcd.txt).
    uint32_t wg = blockIdx.x;
    if (UA && (gridDim.x & 7u) == 0u) wg = (wg & 7u) * (gridDim.x >> 3) + (wg >> 3);
    uint32_t t = wg * kWavesPerWG + wid;
    if constexpr (TB) {
        // a table launch may release a completion flag (launch_done, as every workgroup's last
        // act): its workgroups leave together, waves past the last tile skip the tile loop
        if (wg * kWavesPerWG >= ntiles) {
            launch_done<TB>(bases);
            return;
        }
    } else {
        if (t >= ntiles) {
            stage();  // the workgroup's other waves may have tiles: their barrier needs this one
            return;
        }
    }

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
        const uint8_t* ib = block_rows<TB>(bases, in, blk, in_bs);
        uint8_t* ob = block_rows<TB>(bases, out, blk, out_bs);
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
        // CRC: bytes of the lane's 16-byte chunk that are not part of the row's chunk ch count as
        // zero -- UA: the leading bytes of the row's overlapping last window; aligned: the bytes
        // at or past S of the row's last chunk.  The mask lives in the nibble-offset masks (a
        // zero nibble looks up a zero entry: the tables are linear), so it costs nothing per
        // row, and it is branch-free, so the folds stay in straight code (a branch inside the
        // column loop lets the compiler sink every column's GF math past it).
        uint32_t nm[4];  // per dword: 0x1E in every byte lane that counts
        uint32_t slot[NSL], tl[(NSH + 1) / 2];  // rows kept by this lane; UA: the last chunk's values
        bool in_quad = true;
        if constexpr (CRC) {
            const int lead = UA ? int(chl * 16u - win) : 0;          // UA: bytes before the chunk
            const int valid = UA ? 16 : int(S) - int(chl * 16u);     // aligned: bytes before S
#pragma unroll
            for (int w = 0; w < 4; w++) {
                uint32_t m = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int pos = 4 * w + b;
                    if (pos >= lead && pos < valid) m |= 0x1Eu << (8 * b);
                }
                nm[w] = m;
            }
            in_quad = UA ? ch + 1 < cpb : ch < cpb;  // UA: the last chunk is a tail; lanes past it add nothing
#pragma unroll
            for (int i = 0; i < NSL; i++) slot[i] = 0;
        }
        const uint32_t qq = (lane & 3u) * 0x20202020u;  // byte offset of this lane's table set
        // fold shard r's chunk x into this lane's slot for r (compile-time r after unrolling)
        auto crc_row = [&](const u32x4& x, int r) {
            if constexpr (CRC) {
                const uint8_t* qt = reinterpret_cast<const uint8_t*>(s_crc);
                uint32_t cr = 0;
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    uint32_t lo = ((x[w] << 1) & nm[w]) | qq, hi = ((x[w] >> 3) & nm[w]) | qq;
                    asm volatile("" : "+v"(lo), "+v"(hi));  // one byte extract per offset
                    uint32_t l[8];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int p = 4 * w + q;
                        l[2 * q] = *reinterpret_cast<const uint16_t*>(qt + 256 * p + ((lo >> (8 * q)) & 0xFF));
                        l[2 * q + 1] = *reinterpret_cast<const uint16_t*>(qt + 256 * p + 128 + ((hi >> (8 * q)) & 0xFF));
                    }
                    // 8 lookups and the running value: four 3-input XORs
                    cr = xor3(xor3(l[0], l[1], l[2]), xor3(l[3], l[4], l[5]), xor3(l[6], l[7], cr));
                }
                if constexpr (UA) tl[r / 2] = (r & 1) ? (tl[r / 2] | (cr << 16)) : cr;
                cr = in_quad ? cr : 0u;
                cr ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(cr), 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
                cr ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(cr), 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
                slot[r / 4] = (lane & 3u) == uint32_t(r & 3) ? cr : slot[r / 4];
            }
        };
        // UA4 (read-heavy unaligned tiles): the lane's 16-byte window is loaded from the dword
        // boundary at or below it (a 4-byte-aligned dwordx4 plus the dword after it) and
        // funnel-shifted by the window's byte offset in that dword (v_alignbyte_b32), instead of
        // one byte-aligned 16-byte load: +7% on the Split layout's RS(10,4) 1-row reconstruct
        // (4.78 -> 5.11 TB/s, profiles/r03/ua/ua4_ab.txt).  Every dword loaded holds a byte of the
        // row: the dwordx4 holds the window's first byte, and the extra dword is the one holding its
        // last byte, (p + 15) & ~3.  That is the dword after the dwordx4 when the window is not
        // 4-aligned; when it is (r == 0: a row's last window at S - 16 with S a multiple of 4, as in
        // a page-exact buffer), it is the dwordx4's own last dword again, never the dword at S, and
        // alignbyte with r == 0 ignores it.
        constexpr bool UA4 = UA && (RSMI_UA_DWORD_LOADS == 2 || (NT == 2 && RSMI_UA_DWORD_LOADS == 1));
        uint32_t vx[UA4 ? P : 1];  // UA4: the dword holding each row's window's last byte
        auto load_col = [&](int c) {
            if constexpr (UA4) {
                const uintptr_t p = reinterpret_cast<uintptr_t>(ib + in_off[c] + win);
                const uintptr_t a = p & ~uintptr_t(3);
                vx[c % P] = *reinterpret_cast<const uint32_t*>((p + 15) & ~uintptr_t(3));
                return u32x4(*reinterpret_cast<const u32x4a4*>(a));
            } else if constexpr (UA) {
                // nontemporal loads for write-heavy tiles; read-heavy UA tiles keep the lines
                // they share with their neighbours in the L2
                return ld16u<NT == 1 && RSMI_UA_NT_LOADS>(ib + in_off[c] + win);
            } else {
                return ld16<true>(reinterpret_cast<const u32x4*>(ib + in_off[c]) + chl);
            }
        };
        // UA4: row c's window from its two loads
        auto window = [&](int c, const u32x4& d) -> u32x4 {
            if constexpr (UA4) {
                const uint32_t r = uint32_t(reinterpret_cast<uintptr_t>(ib + in_off[c] + win)) & 3u;
                const uint32_t e = vx[c % P];
                return u32x4{__builtin_amdgcn_alignbyte(d[1], d[0], r), __builtin_amdgcn_alignbyte(d[2], d[1], r),
                             __builtin_amdgcn_alignbyte(d[3], d[2], r), __builtin_amdgcn_alignbyte(e, d[3], r)};
            } else {
                return d;
            }
        };

        // Software pipeline over the K input rows: a ring of P rows in flight, one
        // scheduling region per row (sched_barrier) so the compiler cannot hoist every
        // load and table read to the top and blow the 128-VGPR budget.
        u32x4 v[P];
#pragma unroll
        for (int c = 0; c < P; c++) v[c] = load_col(c);
        stage();  // RSMI_ROWS_FIRST: the table to LDS while the first tile's rows are in flight

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
            if constexpr (UA4) v[slot] = window(c, v[slot]);
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
            if constexpr (CRC) crc_row(v[slot], c);
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

        if constexpr (CRC) {
#pragma unroll
            for (int j = 0; j < MT; j++) crc_row(u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]}, K + j);
            uint32_t* rec = crc_rec + (uint64_t(blk) * tpb + tib) * ((NSL + 1) / 2) * kWave + lane;
#pragma unroll
            for (int i = 0; i < NSL; i += 2) rec[i / 2 * kWave] = slot[i] | (i + 1 < NSL ? slot[i + 1] << 16 : 0u);
            if constexpr (UA) {
                if (ch + 1 == cpb) {
                    uint32_t* tp = crc_tail + uint64_t(blk) * NSH;
#pragma unroll
                    for (int r = 0; r < NSH; r++) tp[r] = (tl[r / 2] >> (16 * (r & 1))) & 0xFFFFu;
                }
            }
        }
        if (UA && ch < cpb) {
#pragma unroll
            for (int j = 0; j < MT; j++) {
                const u32x4 o = u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
                st16u<NT == 1 && RSMI_UA_NT_STORES>(ob + out_off[j] + win, o);
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
    stage();  // a table launch's waves past the last tile (no-op once staged)
    launch_done<TB>(bases);
}

typedef int mfma_v8i __attribute__((ext_vector_type(8)));
typedef float mfma_v4f __attribute__((ext_vector_type(4)));

// A^(2^i)(s) through the nibble-sliced tables P4[i][4][16]
__device__ __forceinline__ uint32_t crc_pow4(const uint16_t* sQ, int i, uint32_t s) {
    const uint16_t* t = sQ + i * 64;
    return xor3(uint32_t(t[s & 15]), uint32_t(t[16 + ((s >> 4) & 15)]), uint32_t(t[32 + ((s >> 8) & 15)])) ^
           uint32_t(t[48 + ((s >> 12) & 15)]);
}

// R(row) of rows 4 p + g (lane l = 16 g + m: class m) of one block from its unit records
// (rs_fused_mfma_kernel): for each unit h a lane gathers its class's 16-bit value from the
// class's four record bytes (one dword load; the loads of 8 units are issued before their power
// steps) and steps its running value by one unit (A^4096 for 4-tile units) before adding it; a
// 4-level scan over the 16 classes (A^(16 * 2^j)) then leaves the row's value relative to the end
// of the last unit in lane 15 of the group, and A^e, e = (S - that end) mod 32767 (column form),
// moves it to the row's end.  out[r] is written once (host memory allowed).
__device__ __forceinline__ void crc16_combine_rows(const uint16_t* sQ, const uint8_t* rec, uint32_t upb, uint32_t nacc,
                                                   uint32_t nsh, const Crc16Shift& sh, uint32_t* out, uint32_t p,
                                                   uint32_t lane) {
    const uint32_t m = lane & 15u, g = lane >> 4;
    const uint32_t r = g + 4u * p, rr = r < nsh ? r : nsh - 1;  // idle lanes repeat a row, store nothing
    const uint32_t sp = 4u * (rr & 1u);
    // the class's four bytes (j = 0..3) of accumulator rr / 2 in unit h
    const uint8_t* rb = rec + (rr >> 1) * kWave + m * 4u;
    uint32_t acc = 0;
    for (uint32_t h0 = 0; h0 < upb; h0 += 8) {
        uint32_t x[8];
#pragma unroll
        for (int hh = 0; hh < 8; hh++) {
            const uint32_t h = h0 + hh < upb ? h0 + hh : upb - 1;
            x[hh] = *reinterpret_cast<const uint32_t*>(rb + uint64_t(h) * nacc * kWave);
        }
#pragma unroll
        for (int hh = 0; hh < 8; hh++) {
            if (h0 + hh >= upb) break;
            const uint32_t y = x[hh] >> sp;
            const uint32_t v = (y & 15u) | ((y >> 4) & 0xF0u) | ((y >> 8) & 0xF00u) | ((y >> 12) & 0xF000u);
            acc = crc_pow4(sQ, 10 + kFusedUnitLog, acc) ^ v;  // earlier units move one unit further
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t w = crc_pow4(sQ, 4 + j, acc);  // 16 * 2^j bytes
        const uint32_t t = __shfl_up(w, 1u << j);
        if (m >= (1u << j)) acc ^= t;
    }
    uint32_t y = 0;  // A^e(acc), column form
#pragma unroll
    for (int bit = 0; bit < 16; bit++) y ^= ((acc >> bit) & 1u) ? sh.col[bit] : 0u;
    if (m == 15 && r < nsh) out[r] = y;
}


// ------------------------------------------------------------------ fused encode + CRC-16, matrix-core fold
// DagNode.Put's device form (node.go:358-408 with server.go:57-80's checksum of every shard):
// the encode of rs_fast_kernel (aligned layouts, encode plans: input row c is shard c, output row
// j shard K + j) with R(shard) of every row it reads and writes folded on the matrix cores
// instead of the nibble tables of the CRC variants above.  R(chunk) is GF(2)-linear in the
// chunk's 128 bits, so a tile's fold is a GF(2) matrix product evaluated as exact fp4 counts
// (v_mfma_scale_f32_16x16x128_f8f6f4, as in rs_crc16_rows_mfma_kernel): B = one data bit per
// nibble (forms x & 0x11111111, & 0x22.., & 0x44.. and (x >> 3) & 0x11111111 -- the encode
// computes x >> 3 for its GF tables anyway), A = the weights of the tile's position in its unit
// (crc16.hpp FW, LDS, loaded once per tile and shared by every row).  Per row and tile: 4
// bitwise ops per dword and 4 MFMAs, against 15 VALU and 8 LDS lookups per dword for the nibble
// fold.
//
// A unit is kFusedUnitTiles = 4 consecutive tiles of one block, coded by the 4 waves of one
// workgroup (one tile each, RSMI_FUSED_COOP) or by one wave, and the counts of a row accumulate
// over the unit's tiles, so the parity is read once per unit.  Two shards share
// one f32 accumulator: the odd shard's MFMAs run with B scale 2^12, and a unit's counts stay
// below 2^11 (4 tiles x 4 MFMAs x 128 products), so count0 + 2^12 count1 < 2^24 is exact in f32
// and the parities are bits 0 and 12 of the integer.  Record of a unit: per accumulator and lane
// l = 16 j + m, a byte whose bits 0-3 / 4-7 = parity of element i of the even / odd shard (CRC
// bit 4 j + i of class m: chunks m, m + 16, m + 32, m + 48 of the unit's tiles, relative to the
// end of chunk 48 + m of its last tile); four accumulators per dword, dword d of the unit at lane
// slot 4 m + j, so a class's four dwords are contiguous for rs_crc16_combine_mfma_kernel.
//
// UA: rows at any alignment and pitch (S >= 16; the Split layout), with the unaligned-window
// loads and stores of rs_fast_kernel's UA form.  The fold needs every lane's bytes at their
// chunk position: only the lane holding a row's last, overlapping window (it starts at S - 16,
// not at 16 ch) differs: its window must move right by d = 16 ch - (S - 16) bytes.  The rows go
// into the fold unshifted, and the row's last tile then adds (window XOR shifted window) of that
// lane alone (the counts only matter mod 2), for the output rows from registers and for the input
// rows from a reload, so the common tiles carry none of it.  Workgroups take XCD-contiguous units,
// as the UA coding kernels do.
// INL (small launches, a block of a few units): the block's last unit to finish combines its
// records into R(row) itself, so the call needs no second launch (below).
// TB: over a table of block bases, as rs_fast_kernel TB (a coalesced group of DagNode.Put
// callers' own page-locked buffers in one launch).
template <int K, int MT, int NT, int WPS, bool UA = false, bool INL = false, bool TB = false>
__global__ __launch_bounds__(kWG, WPS) void rs_fused_mfma_kernel(const RsPlanDev* __restrict__ plan,
                                                              const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                              uint64_t in_bs, uint64_t in_rs, uint64_t out_bs,
                                                              uint64_t out_rs, uint32_t S, uint32_t cpb, uint32_t tpb,
                                                              uint32_t upb, uint32_t nunits,
                                                              const uint32_t* __restrict__ crc_tbl,
                                                              uint8_t* __restrict__ crc_rec, uint32_t* __restrict__ ctr,
                                                              uint32_t* __restrict__ raw, Crc16Shift sh,
                                                              BasesArg<TB> bases) {
    static_assert(NT == 1 || NT == 2, "cache policy 1 or 2");
    constexpr int NSH = K + MT;
    constexpr int NACC = (NSH + 1) / 2;  // two shards per accumulator
    __shared__ u32x4 s_tbl[K * kColDwords / 4];
#ifdef RSMI_FUSED_WSTAGE  // diagnostic: the weights staged in LDS by every workgroup (16 KiB)
    __shared__ u32x4 s_w[kCrcFWWords / 4];
#endif
    // INL: the combine's power tables, staged with the coding tables (off the combine's path)
    __shared__ uint32_t s_p4[INL ? kCrcP4Words : 1];
    // the tables; INL (latency-bound launches): written to LDS once the wave's first rows are in
    // flight (stage, below), else at once
    LdsTable<K * kColDwords> lt;
    lt.load(plan->tbl);
    LdsTable<INL ? kCrcP4Words : 1> lp;
    if constexpr (INL) lp.load(crc_tbl + kCrcP4Off);
    __builtin_amdgcn_sched_barrier(0);
    bool staged = false;  // wave-uniform: every wave passes the staging barrier exactly once
    auto stage = [&]() {
        if (staged) return;
        lt.store(reinterpret_cast<uint32_t*>(s_tbl));
        if constexpr (INL) lp.store(s_p4);
#ifdef RSMI_FUSED_WSTAGE
        const u32x4* w = reinterpret_cast<const u32x4*>(crc_tbl + kCrcFWOff);
        for (int i = threadIdx.x; i < kCrcFWWords / 4; i += kWG) s_w[i] = w[i];
#endif
        __syncthreads();
        staged = true;
    };
    if constexpr (!INL) stage();

    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
#if RSMI_FUSED_COOP
    // a workgroup codes a unit, wave w its tile w: every wave codes one tile, as in the plain
    // encode, and the waves' counts meet in LDS at the end (below); UA: each XCD takes one
    // contiguous eighth of the units (their rows share boundary lines)
    uint32_t u = blockIdx.x;
    if (UA && (gridDim.x & 7u) == 0u) u = (u & 7u) * (gridDim.x >> 3) + (u >> 3);
#else
    const uint32_t u = blockIdx.x * (kWG / kWave) + wid;
#endif
    if (u >= nunits) {
        stage();
        if constexpr (RSMI_FUSED_COOP) launch_done<TB>(bases);
        return;
    }
    const uint32_t blk = u / upb;
    const uint32_t t0 = (u - blk * upb) * kFusedUnitTiles;
    const uint32_t nt = tpb - t0 < uint32_t(kFusedUnitTiles) ? tpb - t0 : uint32_t(kFusedUnitTiles);
#ifndef RSMI_DIAG_CACHED
    const uint8_t* ib = block_rows<TB>(bases, in, blk, in_bs);
    uint8_t* ob = block_rows<TB>(bases, out, blk, out_bs);
#else  // diagnostic build (tools/Makefile diag-cached): the rows of the first 16 blocks only, so
       // the launch time is the kernel's own issue time
    const uint8_t* ib = in + uint64_t(blk & 15) * in_bs;
    uint8_t* ob = out + uint64_t(blk & 15) * out_bs;
#endif

#ifdef RSMI_FUSED_RING  // diagnostic: rows in flight
    constexpr int P = K < RSMI_FUSED_RING ? K : RSMI_FUSED_RING;
#else
    constexpr int P = rows_in_flight<K, MT>();
#endif
    uint64_t in_off[K], out_off[MT];
#pragma unroll
    for (int c = 0; c < K; c++) in_off[c] = uint64_t(plan->in_row[c]) * in_rs;
#pragma unroll
    for (int j = 0; j < MT; j++) out_off[j] = uint64_t(plan->out_row[j]) * out_rs;

    mfma_v4f cacc[NACC];
#pragma unroll
    for (int a = 0; a < NACC; a++) cacc[a] = mfma_v4f{0.f, 0.f, 0.f, 0.f};

    // the output rows of one tile: the lane's chunk ch (UA: its window at byte win)
    auto store_out = [&](uint32_t ch, uint32_t win, const uint32_t (&acc)[MT][4]) {
        if (UA && ch < cpb) {
#pragma unroll
            for (int j = 0; j < MT; j++) st16u<NT == 1>(ob + out_off[j] + win, u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]});
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
    };
    // INL: the output rows are stored after the unit's record is published, so the publish's
    // release waits for the record alone, not for the rows' writes (over PCIe when the call
    // codes page-locked host memory in place); one tile per wave (COOP) keeps them in registers
    constexpr bool kDefer = INL && RSMI_FUSED_COOP && RSMI_FUSED_INL_DEFER;
    uint32_t dacc[kDefer ? MT : 1][4];
    uint32_t dch = ~0u, dwin = 0u;

#if RSMI_FUSED_COOP
    static_assert(kFusedUnitTiles == kWG / kWave, "one tile per wave of the unit's workgroup");
    for (uint32_t i = wid; i < nt; i += kWG / kWave) {
#else
#pragma unroll 1
    for (uint32_t i = 0; i < nt; i++) {
#endif
        const uint32_t ch = (t0 + i) * kWave + lane;
        const uint32_t chl = ch < cpb ? ch : cpb - 1;  // load chunk, clamped: loads stay unconditional
        // UA: byte offset of the lane's 16-byte window (the row's last one overlaps the one before)
        const uint32_t win = UA ? (chl * 16u < S - 16u ? chl * 16u : S - 16u) : 0u;
        const bool last_tile = (t0 + i + 1) * uint32_t(kWave * 16) > S;  // wave-uniform
        // UA: the last window's shift to its chunk position (0 when S is a multiple of 16)
        const uint32_t dsh = UA ? 16u * (cpb - 1u) - (S - 16u) : 0u;
        // wave-uniform: this tile's last window moves
        const bool fix = UA && last_tile && dsh != 0u;
        const bool mine = ch == cpb - 1u;
        // the window's 16 bytes shifted right by dsh bytes (1..15, zero fill): two u64 halves
        auto shifted = [&](const u32x4& x) -> u32x4 {
            const uint64_t lo = uint64_t(x[0]) | (uint64_t(x[1]) << 32), hi = uint64_t(x[2]) | (uint64_t(x[3]) << 32);
            const uint32_t sb = 8u * dsh;
            const uint64_t nlo = sb == 0u ? lo : sb < 64u ? (lo >> sb) | (hi << ((64u - sb) & 63u)) : hi >> ((sb - 64u) & 63u);
            const uint64_t nhi = sb < 64u ? hi >> sb : 0u;
            return u32x4{uint32_t(nlo), uint32_t(nlo >> 32), uint32_t(nhi), uint32_t(nhi >> 32)};
        };
        // the correction that moves the window's bytes to their chunk position: the counts only
        // matter mod 2, so adding (window XOR shifted window), its lane alone, does it
        auto correction = [&](const u32x4& x) -> u32x4 {
            const u32x4 y = shifted(x);
            return u32x4{mine ? x[0] ^ y[0] : 0u, mine ? x[1] ^ y[1] : 0u, mine ? x[2] ^ y[2] : 0u, mine ? x[3] ^ y[3] : 0u};
        };
        // bytes of the lane's chunk that count: those before S (lanes past the row's last chunk,
        // which loaded a clamped chunk, count nothing); all-ones except in a row's last tile
        uint32_t mk[4] = {~0u, ~0u, ~0u, ~0u};
        if (last_tile) {
            const int valid = int(S) - int(ch * 16u);
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const int nb = valid - 4 * w;
                mk[w] = nb >= 4 ? ~0u : nb <= 0 ? 0u : (1u << (8 * nb)) - 1u;
            }
        }
        // this tile position's weights, one operand per bit form, shared by every row
        // (from global memory: the 16 KiB table stays in the L2, and a workgroup that staged it
        // in LDS first would hold its waves' HBM loads back by the staging's latency)
#ifdef RSMI_FUSED_WSTAGE
        const u32x4* wt = s_w + (4 - kFusedUnitTiles + i) * 4 * kWave + lane;
#else
        const u32x4* wt = reinterpret_cast<const u32x4*>(crc_tbl + kCrcFWOff) + (4 - kFusedUnitTiles + i) * 4 * kWave + lane;
#endif
#ifndef RSMI_FUSED_WLDS
        u32x4 W[4];
#pragma unroll
        for (int q = 0; q < 4; q++) W[q] = wt[q * kWave];
#endif
        // one MFMA: bit form q of row r's chunk x into the row's accumulator
        auto crc_mfma = [&](const u32x4& x, int r, int q) {
            mfma_v4f& acc = cacc[r / 2];
#if defined(RSMI_FUSED_DIAG) && RSMI_FUSED_DIAG == 3  // diagnostic: no CRC work at all
            return;
#endif
#if defined(RSMI_FUSED_DIAG) && RSMI_FUSED_DIAG == 1  // diagnostic: the output rows' CRC skipped
            if (r >= K) return;
#endif
            const uint32_t msk = q == 1 ? 0x22222222u : q == 2 ? 0x44444444u : 0x11111111u;
            mfma_v8i bd;
#pragma unroll
            for (int w = 0; w < 4; w++)
                bd[w] = int(__builtin_amdgcn_bitop3_b32(q < 3 ? x[w] : x[w] >> 3, mk[w], msk, 0x80));  // a & b & c
            bd[4] = bd[5] = bd[6] = bd[7] = 0;
#if defined(RSMI_FUSED_DIAG) && RSMI_FUSED_DIAG == 2  // diagnostic: the bit forms without the MFMAs
            acc[0] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, acc[0]) ^ uint32_t(bd[0] ^ bd[1] ^ bd[2] ^ bd[3]));
            return;
#endif
#ifdef RSMI_FUSED_WLDS  // diagnostic: the weights read from LDS for every MFMA instead of held per tile
            const u32x4 Wq = wt[q * kWave];
#else
            const u32x4 Wq = W[q];
#endif
            const mfma_v8i aw = {int(Wq[0]), int(Wq[1]), int(Wq[2]), int(Wq[3]), 0, 0, 0, 0};
            acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(aw, bd, acc, 4, 4, 0, 127, 0,
                                                                   (r & 1) ? 127 + 12 : 127);
        };
        // keep the MFMAs where they are issued: the accumulators are only read after the tile
        // loop, so without an anchor the MFMAs sink to the loop's end and every row's bit forms
        // stay live
        auto anchor = [&](int r) { asm volatile("" : "+v"(cacc[r / 2])); };
        // the tile's body; UA: the row's last tile with S % 16 != 0 moves its last window to its
        // chunk position (a separate copy, so the common tiles carry none of it)
        auto tile_body = [&]() {
            auto load_col = [&](int c) {
                if constexpr (UA)
                    return ld16u<NT == 1>(ib + in_off[c] + win);
                else
                    return ld16<true>(reinterpret_cast<const u32x4*>(ib + in_off[c]) + chl);
            };

            u32x4 v[P];
    #pragma unroll
            for (int c = 0; c < P; c++) v[c] = load_col(c);
            stage();
            uint32_t acc[MT][4], pend[MT][4];
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
    #ifndef RSMI_FUSED_NOIL
                    // form w's MFMA between the GF work of dword w and w + 1: its latency (and the
                    // chain of the row's four MFMAs) hides under this wave's own VALU stream
                    crc_mfma(v[slot], c, w);
                    __builtin_amdgcn_sched_barrier(0);
    #endif
                }
    #ifdef RSMI_FUSED_NOIL  // diagnostic: the row's four MFMAs back to back after its GF work
    #pragma unroll
                for (int q = 0; q < 4; q++) crc_mfma(v[slot], c, q);
    #endif
                anchor(c);
                if (c + P < K) v[slot] = load_col(c + P);
                if (c + 1 < K) {
    #pragma unroll
                    for (int f = 0; f < 5; f++) Tn[f] = tbl[(c + 1) * 5 + f];
                }
                __builtin_amdgcn_sched_barrier(0);
            }
    #pragma unroll
            for (int j = 0; j < MT; j++)
    #pragma unroll
                for (int w = 0; w < 4; w++) asm volatile("" : "+v"(acc[j][w]));
            // the output rows: bit form by bit form, even rows before odd ones, so consecutive MFMAs
            // go to different accumulators wherever two output rows do not share one
    #pragma unroll
            for (int q = 0; q < 4; q++)
    #pragma unroll
                for (int h = 0; h < 2; h++)
    #pragma unroll
                    for (int j = h; j < MT; j += 2) crc_mfma(u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]}, K + j, q);
    #pragma unroll
            for (int j = 0; j < MT; j++) anchor(K + j);
            // UA: every row's last window went in unshifted; correct the output rows' counts here
            // and the input rows' after the stores (reloaded: a shifted copy of every row in flight
            // would not fit the registers)
            if (UA && fix) {
    #pragma unroll
                for (int j = 0; j < MT; j++) {
                    const u32x4 d = correction(u32x4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]});
    #pragma unroll
                    for (int q = 0; q < 4; q++) crc_mfma(d, K + j, q);
                    anchor(K + j);
                }
            }

            if constexpr (kDefer) {
    #pragma unroll
                for (int j = 0; j < MT; j++)
    #pragma unroll
                    for (int w = 0; w < 4; w++) dacc[j][w] = acc[j][w];
                dch = ch;
                dwin = win;
            } else {
                store_out(ch, win, acc);
            }
            if (UA && fix) {
                // an opaque base: the reloads must not be merged with the row loop's loads (that
                // would keep every row's window live through the tile)
                const uint8_t* rb = ib;
                uint32_t rw = win;
                asm volatile("" : "+s"(rb), "+v"(rw));
    #pragma unroll
                for (int c = 0; c < K; c++) {
                    u32x4 x = {0u, 0u, 0u, 0u};
                    if (mine) x = ld16u<NT == 1>(rb + in_off[c] + rw);  // that lane's 16 bytes only
                    const u32x4 d = correction(x);
    #pragma unroll
                    for (int q = 0; q < 4; q++) crc_mfma(d, c, q);
                    anchor(c);  // one reload at a time
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        };
        tile_body();
    }
    stage();  // waves without a tile (the unit's last tiles past the row's end)

    // parities -> the unit's record: byte (accumulator a, lane slot), bits i / 4 + i = element i's
    // parity of shard 2 a / 2 a + 1 (bits 0 and 12 of the exact count)
    auto record = [&](int a, const mfma_v4f& c) {
        uint32_t y = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) y |= (uint32_t(c[e]) & 0x1001u) << e;
        crc_rec[(uint64_t(u) * NACC + a) * kWave + (lane & 15u) * 4u + (lane >> 4)] = uint8_t(y | (y >> 8));
    };
#if RSMI_FUSED_COOP
    // the unit's four tiles meet in LDS (count sums stay below 2^24: exact), and wave w reads out
    // accumulators w, w + 4, ..., so no wave is left with the whole unit's tail
    __shared__ mfma_v4f s_red[kWG / kWave][NACC][kWave];
#pragma unroll
    for (int a = 0; a < NACC; a++) s_red[wid][a][lane] = cacc[a];
    __syncthreads();
    for (int a = int(wid); a < NACC; a += kWG / kWave)
        record(a, s_red[0][a][lane] + s_red[1][a][lane] + s_red[2][a][lane] + s_red[3][a][lane]);
    if constexpr (INL) {
        // The block's last unit to finish combines its records into R(row) (no second launch).
        // Each workgroup publishes its record (fence, then one atomic increment of the block's
        // counter); atomicInc wraps the counter back to 0 at the block's last unit, so the
        // counters are ready for the next launch without a memset.  The agent-scope release writes
        // back the XCD's L2 (the 8 XCDs' L2s are not coherent with each other): per unit of a
        // 4096-block launch that cost 25x the separate combine (8.2 ms against 0.33), so only
        // launches of a few units take this form (rsmi_crc.cpp, kFusedInlineUnits).
        // A block of one unit needs none of it: its own workgroup wrote every record.
#ifndef RSMI_DIAG_INL_NOFENCE  // diagnostic (wrong R for blocks of several units): the publish's cost
        if (upb > 1u) {
            __threadfence();
            __syncthreads();
            __shared__ uint32_t s_last;
            if (threadIdx.x == 0) s_last = atomicInc(ctr + blk, upb - 1) == upb - 1 ? 1u : 0u;
            __syncthreads();
            if (!s_last) {
                if constexpr (kDefer) if (dch != ~0u) store_out(dch, dwin, dacc);
                launch_done<TB>(bases);
                return;
            }
            __threadfence();
        }
#else
        if (u - blk * upb != upb - 1u) {
            if constexpr (kDefer) if (dch != ~0u) store_out(dch, dwin, dacc);
            launch_done<TB>(bases);
            return;
        }
#endif
        if constexpr (kDefer) if (dch != ~0u) store_out(dch, dwin, dacc);
        __syncthreads();
        const uint8_t* rb = crc_rec + uint64_t(blk) * upb * NACC * kWave;
        for (uint32_t p = wid; p < uint32_t(NSH + 3) / 4; p += kWG / kWave)
            crc16_combine_rows(reinterpret_cast<const uint16_t*>(s_p4), rb, upb, NACC, NSH, sh,
                               raw + uint64_t(blk) * NSH, p, lane);
    }
    launch_done<TB>(bases);
#else
#pragma unroll
    for (int a = 0; a < NACC; a++) record(a, cacc[a]);
#endif
}


#ifndef RSMI_TB_UNIT  // rs_kernels_tb.hip: the coding kernels above only
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
// R(row) of the datanode entry checksum (crc16.hpp has the algebra).  A wave owns one item: a
// super-segment of up to kCrcSupGroups groups of kCrcSegTiles = 8 consecutive 1 KiB tiles of
// one row.  Each lane folds its 16-byte chunk of every tile with positional LDS lookups -- 32
// nibble lookups in 16-entry tables (every wave-wide lookup reads 8 distinct dwords in 8
// distinct banks, so it never conflicts).  Tile k of a group uses its own table set G[k]
// (relative to the group's end), so the folds of a group are independent and combine by XOR,
// and a running register carries the groups (A^8192 between them): no dependent power step per
// tile.  A Hillis-Steele scan over the 64 lanes (A^(16*2^j) per level) leaves the item's
// value, relative to the item's end, in lane 63; shifting it by (S - item end) mod 32767 bytes
// places it relative to the row's end, and one atomic XOR adds it into the row's word.  The
// scan and the shift cost about as much as 8 tiles of folding, so items span 32 tiles
// (8-tile items spent 30 % of the pass there).  Powers use nibble-sliced tables
// (P4, conflict-free, 1.9 KiB), so a workgroup stages 12 KiB of LDS.  Bytes at or past S read
// as zero (zero bytes contribute nothing to R, they only move the reference point, which the
// final shift accounts for).
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

// M(s) for a 16x16 matrix held lane-distributed (lane l < 16 of every 16-lane row holds M's
// image of 1 << l) and a wave-uniform s: each lane keeps its column if bit l of s is set, and an
// XOR scan over the 16-lane row (DPP row_shr 1, 2, 4, 8) leaves the image in lane 15.  No LDS.
__device__ __forceinline__ uint32_t crc_apply_cols(uint32_t col, uint32_t s, uint32_t l16) {
    uint32_t x = ((s >> l16) & 1u) ? col : 0u;
    x ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, false));  // row_shr:1
    x ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, false));  // row_shr:2
    x ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, false));  // row_shr:4
    x ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, false));  // row_shr:8
    return uint32_t(__builtin_amdgcn_readlane(int(x), 15));
}

// The item's value -> row word: lane scan, shift to the row's end, one atomic XOR (lane 63).
// The shift is A^d (d = the bytes between the item's end and the last item's end, mod 32767:
// a few power steps, none for the row's last item) and then the launch's A^E (E = S - the last
// item's end) in column form.
__device__ __forceinline__ void crc_item_out(const uint16_t* sQ, uint32_t lane, uint32_t acc, uint64_t item_end,
                                             uint64_t last_end, uint32_t col_e, uint32_t* word) {
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const uint32_t w = crc_pow4(sQ, 4 + j, acc);  // 16 * 2^j bytes
        const uint32_t t = __shfl_up(w, 1u << j);
        if (lane >= (1u << j)) acc ^= t;
    }
    uint32_t val = uint32_t(__builtin_amdgcn_readlane(int(acc), kWave - 1));  // wave-uniform from here
    const uint32_t d = uint32_t((last_end - item_end) % kCrcOrder);
#pragma unroll
    for (int i = 0; i < kCrcPowers; i++)
        if ((d >> i) & 1) val = crc_pow4(sQ, i, val);
    val = crc_apply_cols(col_e, val, lane & 15u);
    if (lane == kWave - 1) atomicXor(word, val);
}

// Position of item `it` (nsup items per row): its row and first tile.
struct CrcItem {
    uint64_t b;
    uint32_t r, t0, nt;  // block, row in block, first tile, tiles in the item
};
__device__ __forceinline__ CrcItem crc_item(uint64_t it, uint32_t nsup, uint32_t nrows, uint32_t tpb) {
    constexpr uint32_t kSup = kCrcSupGroups * kCrcSegTiles;
    CrcItem x;
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
// the byte the item's value is relative to: the end of its last group, counted as 8 tiles
__device__ __forceinline__ uint64_t crc_item_end(const CrcItem& x) {
    return (uint64_t(x.t0) + (x.nt + kCrcSegTiles - 1) / kCrcSegTiles * kCrcSegTiles) * (kWave * 16);
}

// LDS staging shared by the rows passes: P4, then G
#define RSMI_CRC_ROWS_STAGE()                                                                             \
    __shared__ uint32_t s_tbl[kCrcP4Words + kCrcGWords];                                                  \
    for (int i = threadIdx.x; i < kCrcP4Words; i += kWG) s_tbl[i] = tbl[kCrcP4Off + i];                   \
    for (int i = threadIdx.x; i < kCrcGWords; i += kWG) s_tbl[kCrcP4Words + i] = tbl[kCrcGOff + i];       \
    __syncthreads();                                                                                      \
    const uint16_t* sQ = reinterpret_cast<const uint16_t*>(s_tbl);                                        \
    const uint8_t* nb = reinterpret_cast<const uint8_t*>(s_tbl + kCrcP4Words); /* G[8][32][16] */  \
    uint32_t col_e = 0; /* A^E, lane-distributed */                                                    \
    _Pragma("unroll") for (int b_ = 0; b_ < 16; b_++) col_e = (threadIdx.x & 15u) == uint32_t(b_) ? sh.col[b_] : col_e; \
    const uint64_t last_end = (uint64_t(tpb) + kCrcSegTiles - 1) / kCrcSegTiles * kCrcSegTiles * (kWave * 16);

template <bool ALIGNED>
__global__ __launch_bounds__(kWG) void rs_crc16_rows_kernel(const uint32_t* __restrict__ tbl,
                                                            const uint8_t* __restrict__ base, uint64_t bstride,
                                                            uint64_t rpitch, uint32_t nrows, uint64_t S, uint32_t tpb,
                                                            uint32_t nsup, uint64_t nitems, uint32_t* __restrict__ out,
                                                            uint64_t out_bs, Crc16Shift sh) {
    RSMI_CRC_ROWS_STAGE()
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    for (uint64_t it = uint64_t(blockIdx.x) * (kWG / kWave) + wid; it < nitems; it += nw) {
        const CrcItem x = crc_item(it, nsup, nrows, tpb);
        const uint8_t* row = base + x.b * bstride + uint64_t(x.r) * rpitch;
        uint32_t acc = 0;
        for (uint32_t g0 = 0; g0 < x.nt; g0 += kCrcSegTiles) {
            const uint32_t t0 = x.t0 + g0;
            const uint32_t nt = x.nt - g0 < uint32_t(kCrcSegTiles) ? x.nt - g0 : uint32_t(kCrcSegTiles);
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
            uint32_t gs = 0;  // the group's value, relative to the end of its 8th tile
#pragma unroll
            for (int i = 0; i < kCrcSegTiles; i++)
                if (uint32_t(i) < nt) gs ^= crc_nib_chunk(nb + 1024 * i, v[i]);
            acc = crc_pow4(sQ, 13, acc) ^ gs;  // earlier groups move 8 KiB further from the end
        }
        crc_item_out(sQ, lane, acc, crc_item_end(x), last_end, col_e, out + x.b * out_bs + x.r);
    }
}

// The nibble rows pass, software-pipelined, for 16-byte-aligned rows (the default).  A wave
// works in units of half a group (4 tiles) and issues the loads of its next unit (of this item
// or its next one) before it folds the current one (two register sets of 16 VGPRs, the loop
// unrolled by two), so its own fold covers the next unit's memory latency instead of only the
// other waves on the SIMD; half-group units keep the kernel under 64 VGPRs (8 waves per SIMD,
// with 12 KiB of LDS per workgroup).  Loads are unconditional -- chunks past the row's end read
// the row's last chunk and are masked to zero in the fold, and the prefetch past the wave's
// last unit re-reads that unit -- so no load sits behind a branch and the compiler's vmcnt
// waits count only the older set.
__global__ __launch_bounds__(kWG) void rs_crc16_rows_pipe_kernel(const uint32_t* __restrict__ tbl,
                                                                 const uint8_t* __restrict__ base, uint64_t bstride,
                                                                 uint64_t rpitch, uint32_t nrows, uint64_t S,
                                                                 uint32_t tpb, uint32_t nsup, uint64_t nitems,
                                                                 uint32_t* __restrict__ out, uint64_t out_bs,
                                                                 Crc16Shift sh) {
    RSMI_CRC_ROWS_STAGE()
    constexpr int kU = kCrcSegTiles / 2;  // tiles per unit
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    const uint64_t last = (S - 1) / 16 * 16;  // the row's last chunk (S > 0)
    // a unit of work: tiles t0 + 4 h .. t0 + 4 h + 3 of item it (its position computed once per item)
    struct Unit {
        uint64_t it;
        CrcItem x;
        uint32_t h;
    };
    auto at = [&](uint64_t it) -> Unit { return Unit{it, crc_item(it, nsup, nrows, tpb), 0}; };
    auto next = [&](const Unit& u) -> Unit {
        if ((u.h + 1) * kU < u.x.nt) return Unit{u.it, u.x, u.h + 1};
        return at(u.it + nw);
    };
    auto issue = [&](const Unit& u, u32x4(&v)[kU]) {
        const uint8_t* row = base + u.x.b * bstride + uint64_t(u.x.r) * rpitch;
#pragma unroll
        for (int i = 0; i < kU; i++) {
            const uint64_t off = (uint64_t(u.x.t0 + u.h * kU + i) * kWave + lane) * 16;
            v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + (off < last ? off : last)));
        }
    };
    uint32_t acc = 0, gs = 0;
    auto finish = [&](const Unit& u, u32x4(&v)[kU]) {
        const CrcItem& x = u.x;
        const uint32_t u0 = u.h * kU, t0 = x.t0 + u0;
        const uint32_t nt = x.nt - u0 < uint32_t(kU) ? x.nt - u0 : uint32_t(kU);
        const uint8_t* gt = nb + 1024 * kU * (u.h & 1);  // table sets of this half of the group
#pragma unroll
        for (int i = 0; i < kU; i++) {
            if (uint32_t(i) < nt) {
                if ((uint64_t(t0 + i) + 1) * (kWave * 16) > S) {  // wave-uniform: the row's last tile
                    const int64_t valid = int64_t(S) - int64_t((uint64_t(t0 + i) * kWave + lane) * 16);
#pragma unroll
                    for (int w = 0; w < 4; w++) {
                        const int64_t n = valid - 4 * w;
                        v[i][w] &= n >= 4 ? ~0u : n <= 0 ? 0u : (1u << (8 * n)) - 1u;
                    }
                }
                gs ^= crc_nib_chunk(gt + 1024 * i, v[i]);
            }
        }
        const bool item_end = u0 + kU >= x.nt;
        if ((u.h & 1) || item_end) {  // the group is complete
            acc = crc_pow4(sQ, 13, acc) ^ gs;  // earlier groups move 8 KiB further from the end
            gs = 0;
        }
        if (item_end) {
            crc_item_out(sQ, lane, acc, crc_item_end(x), last_end, col_e, out + x.b * out_bs + x.r);
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

// The rows pass with the fold on the matrix cores, aligned rows.  R(chunk) is
// GF(2)-linear in the chunk's 128 bits, so a tile's fold is a GF(2) matrix product; the fp4
// MFMA v_mfma_scale_f32_16x16x128_f8f6f4 sums integer products exactly, and bit 0 of each count
// is the product's bit.  B = the tile's data, one data bit per fp4 nibble (v & 0x11111111,
// 0x22.., 0x44.., (v >> 1) & 0x44..; bit 3 is the e2m1 sign), column m = lane & 15, k block
// j = lane >> 4 (chunk 16 j + m); A = the weights of tile t of an 8-tile group (MW, in LDS,
// one ds_read_b128 per MFMA), row n = CRC bit; every product of a set data bit and a set weight
// is 1.0.  The counts of a whole group accumulate in one f32 quad (at most 4096 per count), so
// the parity is read once per group: four ballots, and lane m (< 16) gathers class m's value
// (chunks m, m + 16, m + 32, m + 48 of the group's tiles, relative to the end of chunk 48 + m
// of tile 7).  Groups step by A^8192 as in the nibble pass; at the item's end a 4-level scan
// over lanes 0..15 (A^(16 * 2^j)) leaves the value relative to the group's end in lane 15, and
// the shift to the row's end is the nibble pass's.  4 MFMAs and 20 VALU per tile fold what the
// nibble tables fold with 32 lookups and ~70 VALU.
//
// UA: rows at any byte alignment (the Split layout: rows back to back at pitch S).  The fold runs
// on the memory's 16-byte grid instead of the row's: the row's bytes are folded where they lie,
// from the aligned chunk at or below the row's first byte (its mis = row & 15 leading bytes, the
// previous row's tail, masked to zero) to the aligned chunk holding its last byte (bytes past it
// masked), so every load is the aligned pass's and no data moves between lanes.  Only the reference
// point changes: an item's value is relative to its end on that grid, mis bytes before its end on
// the row's grid, so the shift to the row's end takes mis bytes more (the launch's tiles per row
// count mis + S bytes, S + 15 at most).
template <bool UA>
__global__ __launch_bounds__(kWG) void rs_crc16_rows_mfma_kernel(const uint32_t* __restrict__ tbl,
                                                                 const uint8_t* __restrict__ base, uint64_t bstride,
                                                                 uint64_t rpitch, uint32_t nrows, uint64_t S,
                                                                 uint32_t tpb, uint32_t nsup, uint64_t nitems,
                                                                 uint32_t* __restrict__ out, uint64_t out_bs,
                                                                 Crc16Shift sh) {
    __shared__ uint32_t s_p4[kCrcP4Words];
    __shared__ u32x4 s_w[kCrcMWWords / 4];
    for (int i = threadIdx.x; i < kCrcP4Words; i += kWG) s_p4[i] = tbl[kCrcP4Off + i];
    for (int i = threadIdx.x; i < kCrcMWWords / 4; i += kWG)
        s_w[i] = reinterpret_cast<const u32x4*>(tbl + kCrcMWOff)[i];
    __syncthreads();
    const uint16_t* sQ = reinterpret_cast<const uint16_t*>(s_p4);
    uint32_t col_e = 0;  // A^E, lane-distributed
#pragma unroll
    for (int b = 0; b < 16; b++) col_e = (threadIdx.x & 15u) == uint32_t(b) ? sh.col[b] : col_e;
    const uint64_t last_end = (uint64_t(tpb) + kCrcSegTiles - 1) / kCrcSegTiles * kCrcSegTiles * (kWave * 16);
    const uint32_t lane = threadIdx.x & (kWave - 1), m = lane & 15u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    for (uint64_t it = uint64_t(blockIdx.x) * (kWG / kWave) + wid; it < nitems; it += nw) {
        const CrcItem x = crc_item(it, nsup, nrows, tpb);
        const uint8_t* row = base + x.b * bstride + uint64_t(x.r) * rpitch;
        // UA: the row's misalignment (wave-uniform), its aligned base and the aligned chunk that
        // holds its last byte
        const uint32_t mis = UA ? uint32_t(__builtin_amdgcn_readfirstlane(int(reinterpret_cast<uintptr_t>(row) & 15u))) : 0u;
        const uint8_t* rowa = row - mis;
        const uint64_t Sm = mis + S;  // the row's end on the memory grid
        const uint64_t lasta = (Sm - 1) / 16 * 16;
        uint32_t acc = 0;  // lanes 0..15: class m's running value
        for (uint32_t g0 = 0; g0 < x.nt; g0 += kCrcSegTiles) {
            const uint32_t t0 = x.t0 + g0;
            const uint32_t nt = x.nt - g0 < uint32_t(kCrcSegTiles) ? x.nt - g0 : uint32_t(kCrcSegTiles);
            u32x4 v[kCrcSegTiles];
#pragma unroll
            for (int i = 0; i < kCrcSegTiles; i++) {
                const uint64_t off = (uint64_t(t0 + i) * kWave + lane) * 16;  // unconditional, clamped
                v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowa + (off < lasta ? off : lasta)));
            }
            mfma_v4f c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < kCrcSegTiles; i++) {
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
                    if (UA && t0 + i == 0 && mis != 0u && lane == 0) {  // UA: the bytes before the row
#pragma unroll
                        for (int w = 0; w < 4; w++) {
                            const int n = int(mis) - 4 * w;  // leading bytes of dword w to drop
                            d[w] &= n >= 4 ? 0u : n <= 0 ? ~0u : ~((1u << (8 * n)) - 1u);
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        mfma_v8i bd;
#pragma unroll
                        for (int w = 0; w < 4; w++)
                            bd[w] = int(q < 3 ? d[w] & (0x11111111u << q) : (d[w] >> 1) & 0x44444444u);
                        bd[4] = bd[5] = bd[6] = bd[7] = 0;
                        const u32x4 wt = s_w[(i * 4 + q) * kWave + lane];
                        const mfma_v8i aw = {int(wt[0]), int(wt[1]), int(wt[2]), int(wt[3]), 0, 0, 0, 0};
                        c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(aw, bd, c, 4, 4, 0, 127, 0, 127);
                    }
                }
            }
            // parity bits -> class m's 16-bit value: bit n of class m is bit 16 (n >> 2) + m of
            // ballot n & 3
            uint32_t Y = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint64_t bl = __builtin_amdgcn_ballot_w64((int(c[i]) & 1) != 0);
                const uint32_t lo = uint32_t(bl) >> m, hi = uint32_t(bl >> 32) >> m;
                Y |= ((lo & 0x10001u) | ((hi & 0x10001u) << 8)) << i;  // n = i, 4 + i (bit 16), 8 + i, 12 + i (bit 24)
            }
            const uint32_t val = (Y & 0x0F0Fu) | ((Y >> 12) & 0xF0F0u);
            acc = crc_pow4(sQ, 13, acc) ^ val;  // earlier groups move 8 KiB further from the end
        }
        // classes -> the group's end: lane 15 takes sum_m A^(16 (15 - m)) (class m)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t w = crc_pow4(sQ, 4 + j, acc);  // 16 * 2^j bytes
            const uint32_t t = __shfl_up(w, 1u << j);
            if (m >= (1u << j)) acc ^= t;
        }
        uint32_t val = uint32_t(__builtin_amdgcn_readlane(int(acc), 15));  // wave-uniform from here
        // UA: the item's end lies mis bytes before its end on the row's grid
        const uint32_t dd = uint32_t((last_end - crc_item_end(x) + mis) % kCrcOrder);
#pragma unroll
        for (int i = 0; i < kCrcPowers; i++)
            if ((dd >> i) & 1) val = crc_pow4(sQ, i, val);
        val = crc_apply_cols(col_e, val, lane & 15u);
        if (lane == kWave - 1) atomicXor(out + x.b * out_bs + x.r, val);
    }
}

void* crc16_rows_mfma_kernel(bool aligned) {
    return aligned ? reinterpret_cast<void*>(&rs_crc16_rows_mfma_kernel<false>)
                   : reinterpret_cast<void*>(&rs_crc16_rows_mfma_kernel<true>);
}

// R(row) from rs_fused_mfma_kernel's unit records: a persistent grid whose waves take items
// (block b, row group p) in turn, lane l = 16 g + m class m of row 4 p + g (the workgroup stages
// the power tables once).  For each unit h
// a lane gathers its class's 16-bit value from the class's four record dwords (one 16-byte load;
// the loads of 8 units are issued before their power steps) and steps its running value by one
// unit (A^4096 for 4-tile units) before adding it; a 4-level scan over the 16 classes (A^(16 * 2^j)) then leaves the
// row's value relative to the end of the last unit (upb units of 1 KiB tiles) in lane 15 of the
// group, and A^e, e = (S - that end) mod 32767 (column form, by value), moves it to the row's end.
// out[block * nsh + r] is written once (host memory allowed).
__global__ __launch_bounds__(kWG) void rs_crc16_combine_mfma_kernel(const uint32_t* __restrict__ tbl,
                                                                    const uint8_t* __restrict__ rec, uint32_t upb,
                                                                    uint32_t nacc, uint32_t nsh, Crc16Shift sh,
                                                                    uint64_t nblocks, uint32_t* __restrict__ out) {
    __shared__ uint32_t s_p4[kCrcP4Words];
    for (int i = threadIdx.x; i < kCrcP4Words; i += kWG) s_p4[i] = tbl[kCrcP4Off + i];
    __syncthreads();
    const uint16_t* sQ = reinterpret_cast<const uint16_t*>(s_p4);
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t npass = (nsh + 3) / 4;  // wave-uniform
    const uint64_t nitems = nblocks * npass, nw = uint64_t(gridDim.x) * (kWG / kWave);
    for (uint64_t it = uint64_t(blockIdx.x) * (kWG / kWave) + wid; it < nitems; it += nw) {
        const uint64_t b = it / npass;
        const uint32_t p = uint32_t(it - b * npass);
        crc16_combine_rows(sQ, rec + b * upb * nacc * kWave, upb, nacc, nsh, sh, out + b * nsh, p, lane);
    }
}

void* crc16_combine_mfma_kernel() { return reinterpret_cast<void*>(&rs_crc16_combine_mfma_kernel); }

// R(row) from the fused encode's tile records (rs_fast_kernel CRC): one wave per block (a
// persistent grid strides over blocks).  Lane l takes quads i = 64 j + l of the block (quad i =
// chunks 4i..4i+3, tile i / 16, record lane 4 (i % 16) + q), loads the quad values of every
// row (two rows per dword, ns2 * 16 bytes), and keeps one running register per row that steps
// by A^4096 (64 quads) between its quads; a lane scan (A^(64 * 2^j)) leaves the sums, relative
// to the end of the last step E = 4096 J bytes, in lane 63.  Lane r then takes row r's sum,
// moves it to the row's end (A^(S - E), mod 32767) and adds the row's tail (UA records: the
// last chunk, folded with its quad position's tables, so moved back by 16 (3 - q) to S).  out[block * nsh + r] is written once (host memory allowed).
template <int NS2>
__global__ __launch_bounds__(kWG) void rs_crc16_combine_kernel(const uint32_t* __restrict__ tbl,
                                                               const uint32_t* __restrict__ rec,
                                                               const uint32_t* __restrict__ tail, uint32_t tpb,
                                                               uint32_t nsh, uint64_t S, uint64_t nblocks,
                                                               uint32_t* __restrict__ out) {
    constexpr int R = 8 * NS2;  // rows carried per lane (padding rows stay zero)
    // nibble-sliced powers (P4, 1.9 KiB, 16-entry tables: conflict-free), 4 lookups per power
    __shared__ uint32_t s_tbl[kCrcP4Words];
    for (int i = threadIdx.x; i < kCrcP4Words; i += kWG) s_tbl[i] = tbl[kCrcP4Off + i];
    __syncthreads();
    auto pw = [&](int i, uint32_t x) { return crc_pow4(reinterpret_cast<const uint16_t*>(s_tbl), i, x); };
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t nw = uint64_t(gridDim.x) * (kWG / kWave);
    const uint32_t nq = 16 * tpb, J = (nq + kWave - 1) / kWave;
    int64_t e = (int64_t(S) - int64_t(J) * 4096) % int64_t(kCrcOrder);
    if (e < 0) e += kCrcOrder;
    const uint32_t qt = uint32_t((S + 15) / 16 - 1) & 3u;            // the tail chunk's lane in its quad
    const uint32_t et = (kCrcOrder - 16 * (3 - qt)) % kCrcOrder;      // A^-(16 (3 - q))
    for (uint64_t b = uint64_t(blockIdx.x) * (kWG / kWave) + wid; b < nblocks; b += nw) {
        uint32_t acc[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = 0;
        const uint32_t* rb = rec + uint64_t(b) * tpb * (NS2 * kWave);
        for (uint32_t j = 0; j < J; j++) {
            const uint32_t i = j * kWave + lane;
            u32x4 v[NS2];
#pragma unroll
            for (int s = 0; s < NS2; s++) {
                v[s] = u32x4{0, 0, 0, 0};
                if (i < nq) v[s] = *reinterpret_cast<const u32x4*>(rb + (i >> 4) * (NS2 * kWave) + s * kWave + (i & 15) * 4);
            }
#pragma unroll
            for (int r = 0; r < R; r++) {
                // row r = 8 s + 4 h + q: dword q of record s, half h
                const uint32_t x = (v[r / 8][r % 4] >> (16 * ((r / 4) & 1))) & 0xFFFFu;
                acc[r] = j ? pw(12, acc[r]) ^ x : x;  // earlier quads of this lane move 4 KiB
            }
        }
#pragma unroll
        for (int l = 0; l < 6; l++) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                const uint32_t w = pw(6 + l, acc[r]);  // 64 * 2^l bytes
                const uint32_t t = __shfl_up(w, 1u << l);
                if (lane >= (1u << l)) acc[r] ^= t;
            }
        }
        uint32_t x = 0;  // lane r: row r's sum
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint32_t s = uint32_t(__builtin_amdgcn_readlane(int(acc[r]), kWave - 1));
            x = lane == uint32_t(r) ? s : x;
        }
        for (int k = 0; k < kCrcPowers; k++)
            if ((e >> k) & 1) x = pw(k, x);
        if (lane < nsh) {
            if (tail) {
                // the tail lane folded with its quad position's tables (relative to S + 16 (3 - q))
                uint32_t y = tail[b * nsh + lane];
                for (int k = 0; k < kCrcPowers; k++)
                    if ((et >> k) & 1) y = pw(k, y);
                x ^= y;
            }
            out[b * nsh + lane] = x;
        }
    }
}

void* crc16_combine_kernel(int ns2) {
    switch (ns2) {
        case 1: return reinterpret_cast<void*>(&rs_crc16_combine_kernel<1>);
        case 2: return reinterpret_cast<void*>(&rs_crc16_combine_kernel<2>);
        case 3: return reinterpret_cast<void*>(&rs_crc16_combine_kernel<3>);
        default: return nullptr;
    }
}

// aligned rows: the pipelined pass; any other layout: the plain nibble pass
void* crc16_rows_kernel(bool aligned) {
    return aligned ? reinterpret_cast<void*>(&rs_crc16_rows_pipe_kernel)
                   : reinterpret_cast<void*>(&rs_crc16_rows_kernel<false>);
}

#endif  // RSMI_TB_UNIT

// ------------------------------------------------------------------ dispatch table
// One kernel per (K, MT) and layout, with the cache policy of the shape (auto_cache_policy in
// rsmi_core.cpp): nontemporal stores unless the tile reads at least 4 rows per row it writes.
constexpr int auto_nt(int K, int MT) { return K >= 4 * MT ? 2 : 1; }
constexpr int ua_nt(int K, int MT) { return RSMI_UA_NT ? RSMI_UA_NT : auto_nt(K, MT); }

#ifdef RSMI_TB_UNIT
// the table-of-bases forms (rs_kernels_tb.hip, its own translation unit so the build compiles it
// beside this one): for the BASELINE shapes' encodes (K = k, MT = m) and their reconstructs of up
// to 4 rows; other shapes code a coalesced group with one launch per block
template <int K, int MT>
static void fill_tb_km(FastKernelTable& t) {
    constexpr int NT = auto_nt(K, MT);
    t.fn_tb[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, NT, kMinWavesPerSimd, false, false, true>);
    t.ua_tb[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, ua_nt(K, MT), kMinWavesPerSimd, true, false, true>);
}
template <int K, int MT>
static void fill_tb_fused(FastKernelTable& t) {
    constexpr int NT = auto_nt(K, MT);
    t.fused_tb[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, false, false, true>);
    t.fused_ua_tb[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, true, false, true>);
    t.fused_inl_tb[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, false, true, true>);
    t.fused_ua_inl_tb[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, true, true, true>);
}
template <int K, int MT>
static void fill_tb_fused_inl(FastKernelTable& t) {
    constexpr int NT = auto_nt(K, MT);
    t.fused_inl_tb[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, false, true, true>);
    t.fused_ua_inl_tb[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, true, true, true>);
}
template <int K>
static void fill_tb_k(FastKernelTable& t) {
    fill_tb_km<K, 1>(t);
    fill_tb_km<K, 2>(t);
    fill_tb_km<K, 3>(t);
    fill_tb_km<K, 4>(t);
}
void fill_table_kernels(FastKernelTable& t) {
    fill_tb_k<2>(t);
    fill_tb_k<4>(t);
    fill_tb_k<10>(t);
    fill_tb_k<16>(t);
    fill_tb_fused<2, 1>(t);
    fill_tb_fused<4, 2>(t);
    fill_tb_fused<10, 4>(t);
    fill_tb_fused<16, 4>(t);
    // the verified reconstructs of a lone degraded read (the survivors' R(row) with the rebuilt
    // rows, one block: the in-kernel combine and its completion flag) of fewer rows than m
    fill_tb_fused_inl<4, 1>(t);
    fill_tb_fused_inl<10, 1>(t);
    fill_tb_fused_inl<10, 2>(t);
    fill_tb_fused_inl<10, 3>(t);
    fill_tb_fused_inl<16, 1>(t);
    fill_tb_fused_inl<16, 2>(t);
    fill_tb_fused_inl<16, 3>(t);
}
#else

template <int K, int MT>
static void fill_km(FastKernelTable& t) {
    constexpr int NT = auto_nt(K, MT);
    t.fn[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, NT>);
    t.ua[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, ua_nt(K, MT), kMinWavesPerSimd, true>);
    t.crc[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, NT, kMinWavesPerSimd, false, true>);
    t.ua_crc[K][MT] = reinterpret_cast<void*>(&rs_fast_kernel<K, MT, NT, kMinWavesPerSimd, true, true>);
    t.fused[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd>);
    t.fused_ua[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, true>);
}

// the in-kernel combine for small launches, for the encode shapes of the BASELINE configs (other
// shapes take the two-launch form)
template <int K, int MT>
static void fill_inl(FastKernelTable& t) {
    constexpr int NT = auto_nt(K, MT);
    t.fused_inl[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, false, true>);
    t.fused_ua_inl[K][MT] = reinterpret_cast<void*>(&rs_fused_mfma_kernel<K, MT, NT, kFusedWavesPerSimd, true, true>);
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
        fill_inl<2, 1>(x);
        fill_inl<4, 2>(x);
        fill_inl<10, 4>(x);
        fill_inl<16, 4>(x);
        fill_table_kernels(x);
        return x;
    }();
    return t;
}

void* generic_kernel() { return reinterpret_cast<void*>(&rs_generic_kernel); }
#endif  // RSMI_TB_UNIT

}  // namespace rsmi
