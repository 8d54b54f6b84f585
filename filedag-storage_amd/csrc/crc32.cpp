// crc32.cpp -- host half of the split CRC-32 (see crc32.hpp).
#include "crc32.hpp"

#include <cstdlib>
#include <utility>

namespace rsmi {

namespace {
uint32_t zero_byte(const uint32_t* T, uint32_t s) { return T[s & 0xFF] ^ (s >> 8); }

// byte-sliced table of a linear map given by its values on the 32 basis vectors
void slice(const uint32_t (&col)[32], uint32_t (&t)[4][256]) {
    for (int h = 0; h < 4; h++)
        for (int x = 0; x < 256; x++) {
            uint32_t v = 0;
            for (int b = 0; b < 8; b++)
                if ((x >> b) & 1) v ^= col[8 * h + b];
            t[h][x] = v;
        }
}

void square(const uint32_t (&a)[4][256], uint32_t (&out)[4][256]) {
    for (int h = 0; h < 4; h++)
        for (int x = 0; x < 256; x++) out[h][x] = Crc32Tables::apply(a, Crc32Tables::apply(a, uint32_t(x) << (8 * h)));
}
}  // namespace

Crc32Tables::Crc32Tables() {
    for (int i = 0; i < 256; i++) {
        uint32_t c = uint32_t(i);
        for (int j = 0; j < 8; j++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        T[i] = c;
    }
    // U[p][b] = A^p(T[b]) for the chunk fold; nibbles by linearity in the byte
    uint32_t U[16][256];
    for (int b = 0; b < 256; b++) {
        U[0][b] = T[b];
        for (int p = 1; p < 16; p++) U[p][b] = zero_byte(T, U[p - 1][b]);
    }
    for (int p = 0; p < 16; p++)
        for (int v = 0; v < 16; v++) {
            N[2 * p][v] = U[15 - p][v];
            N[2 * p + 1][v] = U[15 - p][v << 4];
        }
    // A by columns, and its inverse by Gauss-Jordan elimination over GF(2)
    uint32_t a[32], inv[32];
    for (int j = 0; j < 32; j++) a[j] = zero_byte(T, 1u << j);
    {
        // rows of [A | I]: row i holds bit i of every column
        uint32_t rl[32], rr[32];
        for (int i = 0; i < 32; i++) {
            rl[i] = 0;
            for (int j = 0; j < 32; j++) rl[i] |= ((a[j] >> i) & 1u) << j;
            rr[i] = 1u << i;
        }
        for (int col = 0; col < 32; col++) {
            int piv = -1;
            for (int i = col; i < 32; i++)
                if ((rl[i] >> col) & 1) {
                    piv = i;
                    break;
                }
            if (piv < 0) std::abort();  // A is invertible for any CRC polynomial with an x^0 term
            std::swap(rl[col], rl[piv]);
            std::swap(rr[col], rr[piv]);
            for (int i = 0; i < 32; i++)
                if (i != col && ((rl[i] >> col) & 1)) {
                    rl[i] ^= rl[col];
                    rr[i] ^= rr[col];
                }
        }
        for (int j = 0; j < 32; j++) {
            inv[j] = 0;
            for (int i = 0; i < 32; i++) inv[j] |= ((rr[i] >> j) & 1u) << i;
        }
    }
    slice(a, P[0]);
    for (int i = 1; i < kCrc32Powers; i++) square(P[i - 1], P[i]);
    slice(inv, Q[0]);
    for (int i = 1; i < kCrc32InvPowers; i++) square(Q[i - 1], Q[i]);
    for (int t = 0; t < kCrc32SegTiles; t++)
        for (int q = 0; q < 32; q++)
            for (int v = 0; v < 16; v++) NT[t][q][v] = shift(N[q][v], uint64_t(1024) * (kCrc32SegTiles - 1 - t));
    for (int j = 0; j < kCrc32ScanPowers; j++)
        for (int h = 0; h < 8; h++)
            for (int v = 0; v < 16; v++) SN[j][h][v] = apply(P[4 + j], uint32_t(v) << (4 * h));
    for (int h = 0; h < 8; h++)
        for (int v = 0; v < 16; v++) SG[h][v] = apply(P[13], uint32_t(v) << (4 * h));
    for (int h = 0; h < 8; h++)
        for (int v = 0; v < 16; v++) SG4[h][v] = apply(P[12], uint32_t(v) << (4 * h));
    for (int i = 0; i < kCrc32SegPowers; i++) shift_columns(uint64_t(8192) << i, SC[i]);
    unshift_columns(8192, SC[kCrc32SegPowers]);
    for (int i = 0; i < kCrc32MisPowers; i++) shift_columns(uint64_t(1) << i, SC[kCrc32SegPowers + 1 + i]);
    const uint32_t code4[4] = {4, 2, 1, 1};
    for (int t = 0; t < kCrc32SegTiles; t++)
        for (int s = 0; s < 4; s++)
            for (int h = 0; h < 2; h++)
                for (int l = 0; l < 64; l++) {
                    const int j = l >> 4, n = 16 * h + (l & 15);
                    for (int w = 0; w < 4; w++) MW[t][s][h][l][w] = 0;
                    for (int e = 0; e < 32; e++) {
                        // bit s of byte e >> 1's low (e even) or high (e odd) nibble, relative to the
                        // chunk's end (N), then to the end of chunk 48 + m of tile 7
                        const uint32_t c = shift(N[2 * (e >> 1) + (e & 1)][1u << s],
                                                 uint64_t(256 * (3 - j) + 1024 * (kCrc32SegTiles - 1 - t)));
                        if ((c >> n) & 1) MW[t][s][h][l][e / 8] |= code4[s] << (4 * (e % 8));
                    }
                }
    // A^-1 really inverts A, on a basis
    for (int bit = 0; bit < 32; bit++)
        if (apply(Q[0], apply(P[0], 1u << bit)) != (1u << bit)) std::abort();
}

uint32_t Crc32Tables::shift(uint32_t s, uint64_t n) const {
    for (int i = 0; n && i < kCrc32Powers; i++, n >>= 1)
        if (n & 1) s = apply(P[i], s);
    return s;
}

uint32_t Crc32Tables::unshift(uint32_t s, uint32_t n) const {  // n <= 8192
    for (int i = 0; n && i < kCrc32InvPowers; i++, n >>= 1)
        if (n & 1) s = apply(Q[i], s);
    return s;
}

void Crc32Tables::shift_columns(uint64_t n, uint32_t (&col)[32]) const {
    for (int b = 0; b < 32; b++) col[b] = shift(1u << b, n);
}

void Crc32Tables::unshift_columns(uint32_t n, uint32_t (&col)[32]) const {
    for (int b = 0; b < 32; b++) col[b] = unshift(1u << b, n);
}

uint32_t Crc32Tables::fold(uint32_t s, const uint8_t* p, size_t n) const {
    for (size_t i = 0; i < n; i++) s = T[(s ^ p[i]) & 0xFF] ^ (s >> 8);
    return s;
}

const Crc32Tables& crc32_tables() {
    static const Crc32Tables t;
    return t;
}

uint32_t crc32_checksum(const uint8_t* p, size_t n) { return ~crc32_tables().fold(0xFFFFFFFFu, p, n); }

uint32_t crc32_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len) {
    const Crc32Tables& t = crc32_tables();
    return ~(t.shift(t.fold(0xFFFFFFFFu, head, head_len), data_len) ^ raw);
}

}  // namespace rsmi
