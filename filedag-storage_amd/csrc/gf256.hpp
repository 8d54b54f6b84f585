// gf256.hpp -- host-side GF(2^8) arithmetic and coding-matrix construction for the
// product library (independent of oracle/, which only the tests load).
//
// Semantics follow the codec filedag-storage calls from dag/node/dagnode/erasure.go:37
// (klauspost/reedsolomon v1.11.0): polynomial 0x11D, generator 2,
// systematic matrix = Vandermonde(n x k) x inverse(top k x k), reconstruct from the
// first k present shards in index order.
#pragma once
#include <array>
#include <cstdint>
#include <cstring>
#include <vector>

namespace rsmi {

struct GF256 {
    std::array<uint8_t, 512> exp{};
    std::array<uint8_t, 256> log{};
    GF256() {
        unsigned x = 1;
        for (int i = 0; i < 255; i++) {
            exp[i] = static_cast<uint8_t>(x);
            log[x] = static_cast<uint8_t>(i);
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; i++) exp[i] = exp[i - 255];
    }
    uint8_t mul(uint8_t a, uint8_t b) const {
        if (!a || !b) return 0;
        return exp[log[a] + log[b]];
    }
    uint8_t div(uint8_t a, uint8_t b) const {  // b != 0
        if (!a) return 0;
        int l = int(log[a]) - int(log[b]);
        return exp[l < 0 ? l + 255 : l];
    }
    // galExp: galExp(a,0)=1 (also for a=0), galExp(0,n>0)=0
    uint8_t pow(uint8_t a, int n) const {
        if (n == 0) return 1;
        if (!a) return 0;
        return exp[(int(log[a]) * n) % 255];
    }
};

const GF256& gf();

// Row-major byte matrix.
struct Matrix {
    int rows = 0, cols = 0;
    std::vector<uint8_t> v;
    Matrix() = default;
    Matrix(int r, int c) : rows(r), cols(c), v(size_t(r) * c, 0) {}
    uint8_t& at(int r, int c) { return v[size_t(r) * cols + c]; }
    uint8_t at(int r, int c) const { return v[size_t(r) * cols + c]; }
    const uint8_t* row(int r) const { return v.data() + size_t(r) * cols; }
};

Matrix mat_mul(const Matrix& a, const Matrix& b);
// Gauss-Jordan inverse; returns false when singular.
bool mat_invert(const Matrix& in, Matrix& out);
// n x k systematic encode matrix (A.2).
Matrix build_encode_matrix(int k, int m);

// Field-split product tables for the HIP kernels.  A product a*x is the XOR of three
// lookups on bit fields of x: bits 0-2 (8 entries), bits 3-5 (8 entries), bits 6-7
// (4 entries); each lookup is one v_perm_b32 over byte pools packed into dwords:
//   f0 = a*{0..3}, f1 = a*{4..7}, f2 = a*{0..3}<<3, f3 = a*{4..7}<<3, f4 = a*{0..3}<<6
inline void perm_tables(uint8_t a, uint32_t out[5]) {
    const GF256& g = gf();
    auto pack = [&](int base, int shift) {
        uint32_t w = 0;
        for (int i = 0; i < 4; i++) w |= uint32_t(g.mul(a, uint8_t((base + i) << shift))) << (8 * i);
        return w;
    };
    out[0] = pack(0, 0);
    out[1] = pack(4, 0);
    out[2] = pack(0, 3);
    out[3] = pack(4, 3);
    out[4] = pack(0, 6);
}

}  // namespace rsmi
