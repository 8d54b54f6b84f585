// rs_plan.hpp -- device-side coding plan shared by the host launcher and the kernels.
#pragma once
#include <cstdint>

namespace rsmi {

constexpr int kWave = 64;       // CDNA wavefront
constexpr int kWG = 256;        // threads per workgroup (4 waves)
constexpr int kMaxK = 256;      // k + m <= 256 (erasure.go:22)
constexpr int kMaxMT = 4;       // outputs per launch tile
constexpr int kColDwords = 20;  // per input column: 5 table fields x 4 outputs
constexpr int kMinWavesPerSimd = 4;  // caps the fast kernels at 128 VGPRs (16 waves/CU)

// One launch tile: MT (<= 4) output rows computed from K input rows.
// tbl[c*20 + f*4 + j] = field-f product word for coefficient coef[j][c] (gf256.hpp
// perm_tables); padded outputs (j >= MT) have all-zero tables.
struct RsPlanDev {
    uint32_t k, mt, pad0[14];
    uint32_t in_row[kMaxK];
    uint32_t out_row[kMaxMT], pad1[12];
    uint32_t tbl[kMaxK * kColDwords];
};

// Instantiated fast kernels: fn[K][MT][D][NT] (null when K has no instantiation); NT is
// the cache policy (0 default, 1 nontemporal loads + stores, 2 nontemporal loads only).
struct FastKernelTable {
    void* fn[17][kMaxMT + 1][3][5];  // [K][MT][D][cache policy 0..4]
    void* ua[17][kMaxMT + 1][3];  // unaligned-layout variants [K][MT][NT], D = 1
    void* ua_crc[17][kMaxMT + 1];  // the same with fused per-chunk CRC-16 (auto cache policy)
};

// Experimental variants: fn[shape][v], shape 0 = K10/MT4, 1 = K10/MT1 (D=1);
// v 0/1/2 = 4/8/10 rows in flight (NT=1); v 3 = split table source (TS=1; NT 1 for MT4,
// 2 for MT1, the auto policy's choices).
struct ExpKernelTable {
    void* fn[2][5];  // v 4 = 64-bit selector shifts (SH64)
    void* st[2][6];  // buffer stores with the cache bits kStoreAux[v] (option store_aux)
};
constexpr int kStoreAux[6] = {0, 1, 2, 16, 17, 18};

// LDS-DMA staged variants (rs_lds_kernels.hip, option lds_dma): [0] RS(10,4) encode and
// [1] 1-row reconstruct with 4 waves per workgroup, [2]/[3] the same with 2
struct LdsKernelTable {
    void* fn[4];
    int wpg[4];
};

const FastKernelTable& fast_kernels();
const LdsKernelTable& lds_kernels();
const ExpKernelTable& exp_kernels();
void* generic_kernel();
void* repitch_kernel();

// CRC-16 of shard rows (crc16.hpp): the device table buffer holds P[15][2][256], then
// U[16][256], N[32][16], H[22][64] and PH[15][3][64] (u16); a wave folds kCrcSegTiles 1 KiB
// tiles of one row.  Chunk fold: 0 = one U lookup per byte (256-entry tables, bank
// conflicts), 1 = one N lookup per nibble (16-entry tables: each lookup touches 8 distinct
// banks, conflict-free), 2 = one H lookup per six bits (64 u16 = 32 dwords, one per bank of a
// ds_read_b32 half-wave: conflict-free) with powers from PH, also conflict-free (A/B: level
// with 1).
constexpr int kCrcSegTiles = 8;
constexpr int kCrcPWords = 15 * 2 * 256 / 2;
constexpr int kCrcUWords = 16 * 256 / 2;
constexpr int kCrcNWords = 32 * 16 / 2;
constexpr int kCrcHWords = 22 * 64 / 2;
constexpr int kCrcPHWords = 15 * 3 * 64 / 2;
constexpr int kCrcHOff = kCrcPWords + kCrcUWords + kCrcNWords;
constexpr int kCrcTableWords = kCrcHOff + kCrcHWords + kCrcPHWords;
// CRC-32 (crc32.hpp) device tables, u32 words: NT[8][32][16] | SN[6][8][16] (both staged in
// LDS, 19 KiB) | SC[20][32] (column form, read with scalar loads)
constexpr int kCrc32FoldWords = 8 * 32 * 16;
constexpr int kCrc32PowWords = 8 * 16;  // one nibble-sliced power
constexpr int kCrc32LdsWords = kCrc32FoldWords + 6 * kCrc32PowWords;
constexpr int kCrc32TableWords = kCrc32LdsWords + 20 * 32;
// per-launch shift to the row's end, column form (crc32.hpp), passed by value: A^(S mod 8192),
// the end of an inner segment moved over whatever of the row follows whole segments
struct Crc32Shift {
    uint32_t col[32];
};
void* crc16_rows_kernel(bool aligned, int fold);
void* crc16_combine_kernel(bool six);
void* crc32_rows_kernel(bool aligned, bool pipe);

}  // namespace rsmi
