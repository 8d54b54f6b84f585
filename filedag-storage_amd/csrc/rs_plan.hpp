// rs_plan.hpp -- device-side coding plan shared by the host launcher and the kernels.
#pragma once
#include <cstdint>
#include <type_traits>

namespace rsmi {

constexpr int kWave = 64;       // CDNA wavefront
constexpr int kWG = 256;        // threads per workgroup (4 waves)
#ifndef RSMI_FAST_WG  // threads per workgroup of the coding kernel rs_fast_kernel (A/B builds)
#define RSMI_FAST_WG 256
#endif
constexpr int kFastWG = RSMI_FAST_WG;
constexpr int kMaxK = 256;      // k + m <= 256 (erasure.go:22)
constexpr int kMaxMT = 4;       // outputs per launch tile
constexpr int kColDwords = 20;  // per input column: 5 table fields x 4 outputs
constexpr int kMinWavesPerSimd = 4;  // caps the fast kernels at 128 VGPRs (16 waves/CU)
// unaligned-window tiles: dword-aligned loads funnel-shifted for read-heavy tiles (1, the
// default), for every UA tile (2), or byte-aligned 16-byte loads (0)
#ifndef RSMI_UA_DWORD_LOADS
#define RSMI_UA_DWORD_LOADS 1
#endif
// A/B knobs for the unaligned-window coding kernels (tools/ua_ab.sh, Split layout): the cache
// policy of their instantiations (0: the shape's own, auto_nt; 1 or 2: that one for every UA
// shape), and whether a write-heavy UA tile's stores are nontemporal (1) or default (0)
#ifndef RSMI_UA_NT
#define RSMI_UA_NT 0
#endif
#ifndef RSMI_UA_NT_STORES
#define RSMI_UA_NT_STORES 1
#endif
// ... and whether its loads are nontemporal (1) or default (0)
#ifndef RSMI_UA_NT_LOADS
#define RSMI_UA_NT_LOADS 1
#endif

// One launch tile: MT (<= 4) output rows computed from K input rows.
// tbl[c*20 + f*4 + j] = field-f product word for coefficient coef[j][c] (gf256.hpp
// perm_tables); padded outputs (j >= MT) have all-zero tables.
struct RsPlanDev {
    uint32_t k, mt, pad0[14];
    uint32_t in_row[kMaxK];
    uint32_t out_row[kMaxMT], pad1[12];
    uint32_t tbl[kMaxK * kColDwords];
};

// A coalesced group of blocks that each lie in their own caller's page-locked buffer (concurrent
// DagNode.Put / Get callers, rsmi_coalesce.cpp), coded by one launch: block b's rows start at
// b[b], and the launch's in / out pointers are offsets from there.  Passed by value, so the
// table travels in the kernel arguments (one scalar load per wave, no copy to the device); a
// group of more blocks takes several launches.  The kernels' table-less instantiations take
// NoBases in its place, an unused empty argument that leaves their code unchanged.
// done_flag (the fused encode + CRC-16 with its combine inside, rs_fused_mfma_kernel TB INL): the
// launch's workgroups count themselves in done_ctr as they finish, and the last one releases
// done_seq into the page-locked done_flag, so the caller sees the group's end by polling it
// instead of synchronising the stream (rsmi_coalesce.cpp)
constexpr int kTableBlocks = 64;
struct BlockBases {
    uint64_t b[kTableBlocks];
    uint32_t* done_ctr = nullptr;
    uint32_t* done_flag = nullptr;
    uint32_t done_seq = 0, done_pad = 0;
};
struct NoBases {};
template <bool TB>
using BasesArg = std::conditional_t<TB, BlockBases, NoBases>;

// Instantiated fast kernels, one per (K, MT) with the shape's cache policy (null when K has no
// instantiation): aligned layouts, unaligned-window layouts, and both with the datanode CRC-16
// of every row fused in (encode plans).
struct FastKernelTable {
    void* fn[17][kMaxMT + 1];
    void* ua[17][kMaxMT + 1];
    void* crc[17][kMaxMT + 1];
    void* ua_crc[17][kMaxMT + 1];
    void* fused[17][kMaxMT + 1];     // aligned, the CRC-16 folded on the matrix cores (rs_fused_mfma_kernel)
    void* fused_ua[17][kMaxMT + 1];  // the same on unaligned-window layouts (S >= 16)
    void* fused_inl[17][kMaxMT + 1];     // fused with the combine in the kernel (small launches;
    void* fused_ua_inl[17][kMaxMT + 1];  // null: the two-launch form)
    // the same over a table of block bases (BlockBases; rs_kernels_tb.hip, for the shapes of the
    // BASELINE configs; null: one launch per block)
    void* fn_tb[17][kMaxMT + 1];
    void* ua_tb[17][kMaxMT + 1];
    void* fused_tb[17][kMaxMT + 1];
    void* fused_ua_tb[17][kMaxMT + 1];
    void* fused_inl_tb[17][kMaxMT + 1];
    void* fused_ua_inl_tb[17][kMaxMT + 1];
};
void fill_table_kernels(FastKernelTable& t);  // rs_kernels_tb.hip

const FastKernelTable& fast_kernels();
void* generic_kernel();
void* repitch_kernel();

// CRC-16 of shard rows (crc16.hpp): the device table buffer holds P[15][2][256] (the powers
// A^(2^i), byte-sliced) and N[32][16] (u16); a wave folds kCrcSegTiles 1 KiB tiles of one row
// with one N lookup per nibble (16-entry tables: each wave-wide lookup touches 8 distinct
// banks, so it never conflicts).
constexpr int kCrcSegTiles = 8;   // tiles a wave loads at once (one group)
constexpr int kCrcSupGroups = 4;  // groups per item: the scan and the end shift run once per 32 tiles
constexpr int kCrcPWords = 15 * 2 * 256 / 2;
constexpr int kCrcNWords = 32 * 16 / 2;
constexpr int kCrcQWords = 16 * 2 * 4 * 16 / 2;  // quad-relative nibble tables (fused kernels)
constexpr int kCrcQOff = kCrcPWords + kCrcNWords;
constexpr int kCrcGWords = 8 * 32 * 16 / 2;     // tile-set nibble tables (rows pass)
constexpr int kCrcGOff = kCrcQOff + kCrcQWords;
constexpr int kCrcP4Words = 15 * 4 * 16 / 2;     // nibble-sliced powers (rows pass)
constexpr int kCrcP4Off = kCrcGOff + kCrcGWords;
constexpr int kCrcMWWords = 8 * 4 * 64 * 4;       // fp4 weight operands (matrix-core rows pass)
constexpr int kCrcMWOff = kCrcP4Off + kCrcP4Words;
constexpr int kCrcFWWords = 4 * 4 * 64 * 4;       // fp4 weights of the fused encode + CRC kernel
constexpr int kCrcFWOff = kCrcMWOff + kCrcMWWords;
constexpr int kCrcTableWords = kCrcFWOff + kCrcFWWords;
#ifndef RSMI_FUSED_UNIT
#define RSMI_FUSED_UNIT 4
#endif
#ifndef RSMI_FUSED_COOP  // 1: a workgroup codes a unit (one tile per wave); 0: one wave codes a unit
#define RSMI_FUSED_COOP 1
#endif
// launches of at most this many units combine their records in the fused kernel (one launch
// instead of two; larger ones keep the separate combine, see rs_fused_mfma_kernel INL)
#ifndef RSMI_FUSED_INLINE_UNITS
#define RSMI_FUSED_INLINE_UNITS 64
#endif
constexpr uint32_t kFusedInlineUnits = RSMI_FUSED_INLINE_UNITS;
// 1: such launches store the output rows after the unit's record is published (0: before it)
#ifndef RSMI_FUSED_INL_DEFER
#define RSMI_FUSED_INL_DEFER 1
#endif
// fused encode + CRC on the matrix cores: tiles per wave (one unit), 1, 2 or 4 (the two-shard
// accumulators stay exact up to 4 tiles)
constexpr int kFusedUnitTiles = RSMI_FUSED_UNIT;
constexpr int kFusedUnitLog = kFusedUnitTiles == 4 ? 2 : kFusedUnitTiles == 2 ? 1 : 0;
static_assert(kFusedUnitTiles == 1 << kFusedUnitLog, "unit of 1, 2 or 4 tiles");
#ifndef RSMI_FUSED_WPS
#define RSMI_FUSED_WPS 3
#endif
constexpr int kFusedWavesPerSimd = RSMI_FUSED_WPS;  // its register budget: 168 VGPRs (the row accumulators)
// CRC-32 (crc32.hpp) device tables, u32 words: NT[8][32][16] | SN[6][8][16] (both staged in
// LDS, 19 KiB) | SC[24][32] (column form, read with scalar loads)
constexpr int kCrc32FoldWords = 8 * 32 * 16;
constexpr int kCrc32PowWords = 8 * 16;  // one nibble-sliced power
constexpr int kCrc32LdsWords = kCrc32FoldWords + 7 * kCrc32PowWords;  // NT | SN[6] | SG
#ifndef RSMI_CRC32_FOLD_DEFAULT
#define RSMI_CRC32_FOLD_DEFAULT 1
#endif
constexpr int kCrc32MWOff = kCrc32LdsWords + 24 * 32;       // MW[8][4][2][64][4] (matrix-core pass)
constexpr int kCrc32MWWords = 8 * 4 * 2 * 64 * 4;
// RSMI_CRC32_MFMA_HALF 1: the matrix-core CRC-32 pass reads the parity per half group (4 tiles,
// weights MW[4..7], 32 KiB, the halves joined by A^4096), so 4-wave workgroups stage half the
// weights; 0: per 8-tile group, all 64 KiB staged by 8-wave workgroups
#ifndef RSMI_CRC32_MFMA_HALF
#define RSMI_CRC32_MFMA_HALF 0
#endif
constexpr bool kCrc32MfmaHalf = RSMI_CRC32_MFMA_HALF;
constexpr int kCrc32MfmaWG = kCrc32MfmaHalf ? 256 : 512;
constexpr int kCrc32MfmaTiles = kCrc32MfmaHalf ? 4 : 8;  // tiles per parity read-out
constexpr int kCrc32SG4Off = kCrc32MWOff + kCrc32MWWords;  // SG4[8][16]: A^4096, nibble-sliced
constexpr int kCrc32TableWords = kCrc32SG4Off + 8 * 16;
// per-launch shift to the row's end, column form (crc32.hpp), passed by value: A^(S mod 8192),
// the end of an inner segment moved over whatever of the row follows whole segments
struct Crc32Shift {
    uint32_t col[32];
};
// the CRC-16 rows pass's per-launch shift, column form: A^E with E = (S - end of the row's last
// item) mod 32767, col[b] = A^E(1 << b)
struct Crc16Shift {
    uint32_t col[16];
};
void* crc16_rows_kernel(bool aligned);
void* crc16_rows_mfma_kernel(bool aligned);  // the fold on the matrix cores (unaligned rows: funnel-shifted aligned loads)
void* crc16_combine_kernel(int ns2);  // ns2 = record dwords per lane (rows / 8, rounded up)
void* crc16_combine_mfma_kernel();    // records of rs_fused_mfma_kernel
void* crc32_rows_kernel(bool aligned);
void* crc32_rows_mfma_kernel(bool aligned);  // the fold on the matrix cores (512-thread workgroups)

}  // namespace rsmi
