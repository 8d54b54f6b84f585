// crc_clmul.hpp -- host CRC folding with carry-less multiplies (VPCLMULQDQ, AVX-512) for the
// datanode's reflected CRCs: the entry CRC-16 (howeyc IBM, poly 0x8005 reflected 0xA001,
// dag/node/datanode/server.go:70) and the mutcask value CRC-32 (IEEE 0x04C11DB7,
// kv/mutcask/cask.go:73-97).  The datanode checks its entry CRC on every Get
// (server.go:93-97), byte-serially in the reference; slice-by-8 runs ~4 GiB/s per core.
//
// Algebra (normal-order polynomials; a reflected register holds the coefficients bit-reversed):
// the register after message M from zero is M(x) x^w mod P.  A 16-byte block is a polynomial of
// degree < 128 (bit j of the little-endian block <-> x^(127-j)), so any X congruent to M mod P
// with degree < 128 has the same CRC as M: fold 16-byte accumulators forward by 128 d bits with
//   X x^(128 d) = X_hi x^(128 d + 64) + X_lo x^(128 d) == X_hi K1 + X_lo K2   (mod P)
// (X_hi = the block's first 8 bytes), each product of degree < 96.  A reflected carry-less
// product lands one bit low, so the constants are x^(128 d + 63) and x^(128 d - 1) mod P.  The
// register's start value XORs into the first bytes, and the final 16-byte accumulator and the
// tail (< 16 bytes) run through the byte tables.
#pragma once
#include <cstddef>
#include <cstdint>

namespace rsmi {
namespace host {

// Fold n bytes into the reflected register state s (the state before the bytes, not
// complemented); returns the state after them, or false in *done when the CPU lacks
// VPCLMULQDQ/AVX-512 or n < 256 (the caller then runs its table loop over all n bytes).
// crc16: width 16, normal poly 0x8005; crc32: width 32, normal poly 0x04C11DB7.
uint32_t clmul_crc16(uint32_t s, const uint8_t* p, size_t n, bool* done);
uint32_t clmul_crc32(uint32_t s, const uint8_t* p, size_t n, bool* done);

}  // namespace host
}  // namespace rsmi
