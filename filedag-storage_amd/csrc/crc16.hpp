// crc16.hpp -- CRC-16 "IBM" (howeyc/crc16 Checksum(data, IBMTable), the datanode entry
// checksum of dag/node/datanode/server.go:70) split into pieces the GPU can compute in
// parallel.
//
// Notation (reflected register s, 16 bits; T = makeTable(0xA001)):
//   byte update    s' = T[(s ^ b) & 0xFF] ^ (s >> 8)        (howeyc update(), per byte)
//   zero byte      A(s) = T[s & 0xFF] ^ (s >> 8)            (linear over GF(2))
//   raw CRC        R(D) = fold of the byte update over D from s = 0
//   Checksum(D)    = ~fold from s = 0xFFFF = ~(A^|D|(0xFFFF) ^ R(D))
// The byte update is A(s) ^ T[b], so a fold from s0 over D is A^|D|(s0) ^ R(D) and
//   R(D1 || D2) = A^|D2|(R(D1)) ^ R(D2).
// A is invertible with A^32767 = I (x^16+x^15+x^2+1 = (x+1)(x^15+x+1), x^15+x+1 primitive),
// so shifts by negative byte counts are shifts by (n mod 32767).
//
// Device split (rs_kernels.hip rs_crc16_rows_kernel): each lane folds 16-byte chunks with
// positional tables -- R(chunk) = XOR_p U[15-p][b_p], U[p][b] = A^p(T[b]), or by linearity
// the same with one lookup per nibble in 16-entry tables N -- lanes and tiles
// combine with the power tables A^(2^i), and one atomic XOR per (row, segment) lands the
// row's R(D) in a u32.  The host turns R(D) into the datanode checksum with entry_crc().
#pragma once
#include <cstddef>
#include <cstdint>

namespace rsmi {

constexpr int kCrcPowers = 15;  // A^(2^i), i < 15: any exponent mod 32767
constexpr uint32_t kCrcOrder = 32767;

struct Crc16Tables {
    uint16_t T[256];                  // howeyc makeTable(IBM)
    uint16_t U[16][256];              // U[p][b] = A^p(T[b])
    uint16_t N[32][16];               // nibble tables: N[2p][v] = U[15-p][v], N[2p+1][v] = U[15-p][v << 4]
    uint16_t P[kCrcPowers][2][256];   // P[i][0][x] = A^(2^i)(x), P[i][1][x] = A^(2^i)(x << 8)
    // quad-relative nibble tables of the fused encode + CRC kernels: Q[p][h][q][v] =
    // A^(16 (3 - q)) (U[15 - p][v << 4h]) -- lane q of a 4-lane quad folds its chunk relative to
    // the END OF THE QUAD, so the quad's four values combine by plain XOR
    uint16_t Q[16][2][4][16];
    // tile-set nibble tables of the rows pass: G[k] = A^(1024 (7 - k)) (N) -- tile k of an
    // 8-tile group folds relative to the END OF THE GROUP, so the group's tiles combine by XOR
    uint16_t G[8][32][16];
    // nibble-sliced power tables of the rows pass: P4[i][h][v] = A^(2^i)(v << 4h) (16-entry
    // tables never conflict; 1.9 KiB where P takes 15 KiB)
    uint16_t P4[kCrcPowers][4][16];
    // fp4 weight operands of the matrix-core rows pass (rs_crc16_rows_mfma_kernel), per tile t
    // of an 8-tile group, bit group s (data bits s and s + 4 of every byte), lane l = 16 j + n:
    // nibble e of the lane's 16 bytes weighs data bit s + 4 (e & 1) of byte e >> 1 of chunk
    // 16 j + m for CRC bit n, relative to the end of chunk 48 + m of the group's tile 7; fp4
    // codes 2.0 / 1.0 / 0.5 / 0.5 (s = 0..3) against data values 0.5 / 1 / 2 / 2, so every
    // product of a set data bit and a set weight is 1.0
    uint32_t MW[8][4][64][4];
    // fp4 weight operands of the fused encode + CRC kernel (rs_fused_mfma_kernel): a wave codes a
    // unit of 4 consecutive tiles of one block, tile t of the unit weighs like MW[4 + t] (relative
    // to the end of chunk 48 + m of the unit's tile 3), except that bit group 3 arrives as
    // (x >> 3) & 0x11111111 (bit 3 of each nibble moved to bit 0, data value 0.5, so weight 2.0):
    // the encode computes x >> 3 for its GF tables anyway
    uint32_t FW[4][4][64][4];
    Crc16Tables();
    uint16_t pow2(int i, uint16_t s) const { return uint16_t(P[i][0][s & 0xFF] ^ P[i][1][s >> 8]); }
    // A^n(s) for any n >= 0 (reduced mod 32767)
    uint16_t shift(uint16_t s, uint64_t n) const;
    // fold from register s over p[0..n)
    uint16_t fold(uint16_t s, const uint8_t* p, size_t n) const;
};

const Crc16Tables& crc16_tables();

// howeyc Checksum(p, IBMTable)
uint16_t crc16_checksum(const uint8_t* p, size_t n);
// Checksum(head || D) given only R(D) and |D| (head may be empty)
uint16_t crc16_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len);

}  // namespace rsmi
