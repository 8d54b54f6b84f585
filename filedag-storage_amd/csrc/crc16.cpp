// crc16.cpp -- host half of the split CRC-16 (see crc16.hpp).
#include "crc16.hpp"

#include <cstdlib>

namespace rsmi {

namespace {
uint16_t zero_byte(const uint16_t* T, uint16_t s) { return uint16_t(T[s & 0xFF] ^ (s >> 8)); }
}  // namespace

Crc16Tables::Crc16Tables() {
    for (int i = 0; i < 256; i++) {
        uint16_t c = uint16_t(i);
        for (int j = 0; j < 8; j++) c = (c & 1) ? uint16_t((c >> 1) ^ 0xA001) : uint16_t(c >> 1);
        T[i] = c;
    }
    for (int b = 0; b < 256; b++) {
        U[0][b] = T[b];
        for (int p = 1; p < 16; p++) U[p][b] = zero_byte(T, U[p - 1][b]);
    }
    for (int p = 0; p < 16; p++)
        for (int v = 0; v < 16; v++) {
            N[2 * p][v] = U[15 - p][v];
            N[2 * p + 1][v] = U[15 - p][v << 4];
        }
    // A^(2^0) = A; A^(2^(i+1)) = A^(2^i) applied twice (tables are linear in the byte index)
    for (int x = 0; x < 256; x++) {
        P[0][0][x] = zero_byte(T, uint16_t(x));
        P[0][1][x] = zero_byte(T, uint16_t(x << 8));
    }
    for (int i = 1; i < kCrcPowers; i++)
        for (int h = 0; h < 2; h++)
            for (int x = 0; x < 256; x++) {
                const uint16_t v = P[i - 1][h][x];
                P[i][h][x] = uint16_t(P[i - 1][0][v & 0xFF] ^ P[i - 1][1][v >> 8]);
            }
    for (int p = 0; p < 16; p++)
        for (int h = 0; h < 2; h++)
            for (int q = 0; q < 4; q++)
                for (int v = 0; v < 16; v++) Q[p][h][q][v] = shift(U[15 - p][v << (4 * h)], uint64_t(16 * (3 - q)));
    for (int i = 0; i < kCrcPowers; i++)
        for (int h = 0; h < 4; h++)
            for (int v = 0; v < 16; v++) P4[i][h][v] = pow2(i, uint16_t(v << (4 * h)));
    for (int k = 0; k < 8; k++)
        for (int p = 0; p < 32; p++)
            for (int v = 0; v < 16; v++) G[k][p][v] = shift(N[p][v], uint64_t(1024 * (7 - k)));
    const uint32_t code4[4] = {4, 2, 1, 1};
    for (int t = 0; t < 8; t++)
        for (int s = 0; s < 4; s++)
            for (int l = 0; l < 64; l++) {
                const int j = l >> 4, n = l & 15;
                for (int w = 0; w < 4; w++) MW[t][s][l][w] = 0;
                for (int e = 0; e < 32; e++) {
                    const uint16_t c = shift(U[15 - (e >> 1)][1 << (s + 4 * (e & 1))],
                                             uint64_t(256 * (3 - j) + 1024 * (7 - t)));
                    if ((c >> n) & 1) MW[t][s][l][e / 8] |= code4[s] << (4 * (e % 8));
                }
            }
    const uint32_t fcode4[4] = {4, 2, 1, 4};
    for (int t = 0; t < 4; t++)
        for (int s = 0; s < 4; s++)
            for (int l = 0; l < 64; l++)
                for (int w = 0; w < 4; w++) {
                    uint32_t x = MW[4 + t][s][l][w], y = 0;
                    for (int e = 0; e < 8; e++)
                        if ((x >> (4 * e)) & 0xF) y |= fcode4[s] << (4 * e);
                    FW[t][s][l][w] = y;
                }
    // the group order the negative shifts rely on: A^32767 = I on a basis
    for (int bit = 0; bit < 16; bit++)
        if (shift(uint16_t(1u << bit), kCrcOrder) != uint16_t(1u << bit)) std::abort();
}

uint16_t Crc16Tables::shift(uint16_t s, uint64_t n) const {
    uint32_t e = uint32_t(n % kCrcOrder);
    for (int i = 0; e; i++, e >>= 1)
        if (e & 1) s = pow2(i, s);
    return s;
}

uint16_t Crc16Tables::fold(uint16_t s, const uint8_t* p, size_t n) const {
    for (size_t i = 0; i < n; i++) s = uint16_t(T[(s ^ p[i]) & 0xFF] ^ (s >> 8));
    return s;
}

const Crc16Tables& crc16_tables() {
    static const Crc16Tables t;
    return t;
}

uint16_t crc16_checksum(const uint8_t* p, size_t n) {
    return uint16_t(~crc16_tables().fold(0xFFFF, p, n));
}

uint16_t crc16_entry(const uint8_t* head, size_t head_len, uint32_t raw, size_t data_len) {
    const Crc16Tables& t = crc16_tables();
    const uint16_t s = t.fold(0xFFFF, head, head_len);
    return uint16_t(~(t.shift(s, data_len) ^ uint16_t(raw)));
}

}  // namespace rsmi
