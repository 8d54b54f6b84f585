// crc32.hpp -- CRC-32 IEEE (Go hash/crc32 ChecksumIEEE: reflected polynomial 0xEDB88320,
// register complemented on entry and exit; the same function as zlib's crc32), the value
// checksum of the mutcask KV engine (kv/mutcask/cask.go:73-97: | crc32 (4 B LE) | value |,
// where the datanode's value is its whole entry, server.go:58-75), split into pieces the GPU
// computes in parallel.  Same algebra as crc16.hpp with a 32-bit register:
//   zero byte      A(s) = T[s & 0xFF] ^ (s >> 8)            (linear over GF(2), invertible)
//   raw CRC        R(D) = fold of the byte update over D from s = 0
//   Checksum(D)    = ~(A^|D|(0xFFFFFFFF) ^ R(D)),   R(D1 || D2) = A^|D2|(R(D1)) ^ R(D2)
// No group order is used: forward shifts come from tables of A^(2^i), i < 32 (any 32-bit
// byte count), backward ones (below 8 KiB: a row's last device segment ends up to 8191 bytes
// past the row's end) from tables of A^-(2^i), i < 14.  The host applies them byte-sliced
// (4 lookups).  The device folds with nibble tables (8 lookups per word, 16-entry tables that
// never bank-conflict), and applies its few per-segment shifts in column form (a 32 x 32
// matrix over GF(2) as the images of the 32 basis vectors: 2 VALU per bit, no lookups).
#pragma once
#include <cstddef>
#include <cstdint>

namespace rsmi {

constexpr int kCrc32Powers = 32;    // A^(2^i)
constexpr int kCrc32InvPowers = 14;  // A^-(2^i): backward shifts up to 8192 bytes
constexpr int kCrc32SegTiles = 8;    // device segment: 8 tiles of 1 KiB (rs_crc32_rows_kernel)
constexpr int kCrc32ScanPowers = 6;  // A^(16 * 2^j), j < 6: the 64-lane scan of a tile
constexpr int kCrc32SegPowers = 19;  // A^(8192 * 2^i), i < 19: whole-segment shifts
constexpr int kCrc32SupGroups = 4;   // 8-tile groups per device item (scan and end shift once per item)
constexpr int kCrc32MisPowers = 4;   // A^(2^i), i < 4: an unaligned row's misalignment (< 16 bytes)

struct Crc32Tables {
    uint32_t T[256];                          // reflected 0xEDB88320
    uint32_t N[32][16];                       // nibble tables: N[2p][v] = A^(15-p)(T[v]), N[2p+1][v] = A^(15-p)(T[v << 4])
    uint32_t P[kCrc32Powers][4][256];         // P[i][h][x] = A^(2^i)(x << 8h)
    uint32_t Q[kCrc32InvPowers][4][256];      // Q[i][h][x] = A^-(2^i)(x << 8h)
    // device tables.  NT[t][q][v]: the nibble table N[q] moved 1024 * (7 - t) bytes further
    // from the end, for a chunk in tile t of an 8-tile segment (value relative to the
    // segment's end); SN[j][h][v] = A^(16 * 2^j)(v << 4h), nibble-sliced scan powers;
    // SC[i][b] = A^(8192 * 2^i)(1 << b), column-form segment powers, SC[19] = A^-8192 and
    // SC[20 + i] = A^(2^i), i < 4 (the unaligned pass's shift by the row's misalignment)
    uint32_t NT[kCrc32SegTiles][32][16];
    uint32_t SN[kCrc32ScanPowers][8][16];
    uint32_t SG[8][16];  // A^8192 nibble-sliced: the step between an item's 8-tile groups
    uint32_t SC[kCrc32SegPowers + 1 + kCrc32MisPowers][32];
    // fp4 weight operands of the matrix-core rows pass (rs_crc32_rows_mfma_kernel), the CRC-16
    // pass's MW with a 32-bit register: per tile t of an 8-tile group, bit group s (data bits s
    // and s + 4 of every byte), half h (CRC bits 16 h .. 16 h + 15: one MFMA each), lane
    // l = 16 j + n: nibble e of the lane's 16 bytes weighs data bit s + 4 (e & 1) of byte e >> 1
    // of chunk 16 j + m for CRC bit 16 h + n, relative to the end of chunk 48 + m of the group's
    // tile 7; fp4 codes 2.0 / 1.0 / 0.5 / 0.5 (s = 0..3) against data values 0.5 / 1 / 2 / 2
    uint32_t MW[kCrc32SegTiles][4][2][64][4];
    uint32_t SG4[8][16];  // A^4096 nibble-sliced: the half-group step of the matrix-core pass
    Crc32Tables();
    static uint32_t apply(const uint32_t (&t)[4][256], uint32_t s) {
        return t[0][s & 0xFF] ^ t[1][(s >> 8) & 0xFF] ^ t[2][(s >> 16) & 0xFF] ^ t[3][s >> 24];
    }
    uint32_t shift(uint32_t s, uint64_t n) const;    // A^n(s), n < 2^32
    uint32_t unshift(uint32_t s, uint32_t n) const;  // A^-n(s), n < 8192
    // A^n / A^-n in column form (col[b] = image of 1 << b)
    void shift_columns(uint64_t n, uint32_t (&col)[32]) const;
    void unshift_columns(uint32_t n, uint32_t (&col)[32]) const;
    uint32_t fold(uint32_t s, const uint8_t* p, size_t n) const;
};

const Crc32Tables& crc32_tables();

// Go crc32.ChecksumIEEE(p[0..n))
uint32_t crc32_checksum(const uint8_t* p, size_t n);
// ChecksumIEEE(head || D) given only R(D) and |D|
uint32_t crc32_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len);

}  // namespace rsmi
