// crc32.hpp -- CRC-32 IEEE (Go hash/crc32 ChecksumIEEE: reflected polynomial 0xEDB88320,
// register complemented on entry and exit; the same function as zlib's crc32), the value
// checksum of the mutcask KV engine (kv/mutcask/cask.go:73-97: | crc32 (4 B LE) | value |,
// where the datanode's value is its whole entry, server.go:58-75), split into pieces the GPU
// computes in parallel.  Same algebra as crc16.hpp with a 32-bit register:
//   zero byte      A(s) = T[s & 0xFF] ^ (s >> 8)            (linear over GF(2), invertible)
//   raw CRC        R(D) = fold of the byte update over D from s = 0
//   Checksum(D)    = ~(A^|D|(0xFFFFFFFF) ^ R(D)),   R(D1 || D2) = A^|D2|(R(D1)) ^ R(D2)
// No group order is used: forward shifts come from tables of A^(2^i), i < 32 (any 32-bit
// byte count), and the one backward shift the device needs -- a row's last 1 KiB tile ends
// up to 1023 bytes past the row's end -- from tables of A^-(2^i), i < 10.  The host applies
// them byte-sliced (4 lookups); the device nibble-sliced (8 lookups, 512 B per power).
#pragma once
#include <cstddef>
#include <cstdint>

namespace rsmi {

constexpr int kCrc32Powers = 32;    // A^(2^i)
constexpr int kCrc32InvPowers = 10;  // A^-(2^i): backward shifts below 1024 bytes

struct Crc32Tables {
    uint32_t T[256];                          // reflected 0xEDB88320
    uint32_t N[32][16];                       // nibble tables: N[2p][v] = A^(15-p)(T[v]), N[2p+1][v] = A^(15-p)(T[v << 4])
    uint32_t P[kCrc32Powers][4][256];         // P[i][h][x] = A^(2^i)(x << 8h)
    uint32_t Q[kCrc32InvPowers][4][256];      // Q[i][h][x] = A^-(2^i)(x << 8h)
    // nibble-sliced copies for the device (512 B per power, so all of them fit in LDS):
    // PN[i][h][v] = A^(2^i)(v << 4h), QN likewise
    uint32_t PN[kCrc32Powers][8][16];
    uint32_t QN[kCrc32InvPowers][8][16];
    Crc32Tables();
    static uint32_t apply(const uint32_t (&t)[4][256], uint32_t s) {
        return t[0][s & 0xFF] ^ t[1][(s >> 8) & 0xFF] ^ t[2][(s >> 16) & 0xFF] ^ t[3][s >> 24];
    }
    uint32_t shift(uint32_t s, uint64_t n) const;    // A^n(s), n < 2^32
    uint32_t unshift(uint32_t s, uint32_t n) const;  // A^-n(s), n < 1024
    uint32_t fold(uint32_t s, const uint8_t* p, size_t n) const;
};

const Crc32Tables& crc32_tables();

// Go crc32.ChecksumIEEE(p[0..n))
uint32_t crc32_checksum(const uint8_t* p, size_t n);
// ChecksumIEEE(head || D) given only R(D) and |D|
uint32_t crc32_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len);

}  // namespace rsmi
