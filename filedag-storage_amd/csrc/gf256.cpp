// gf256.cpp -- GF(2^8) matrix algebra for the product library (see gf256.hpp).
#include "gf256.hpp"

namespace rsmi {

const GF256& gf() {
    static const GF256 g;
    return g;
}

Matrix mat_mul(const Matrix& a, const Matrix& b) {
    const GF256& g = gf();
    Matrix r(a.rows, b.cols);
    for (int i = 0; i < a.rows; i++)
        for (int j = 0; j < b.cols; j++) {
            uint8_t acc = 0;
            for (int t = 0; t < a.cols; t++) acc ^= g.mul(a.at(i, t), b.at(t, j));
            r.at(i, j) = acc;
        }
    return r;
}

bool mat_invert(const Matrix& in, Matrix& out) {
    const GF256& g = gf();
    const int n = in.rows;
    if (in.cols != n) return false;
    // work on [in | I]
    Matrix w(n, 2 * n);
    for (int r = 0; r < n; r++) {
        std::memcpy(&w.at(r, 0), in.row(r), size_t(n));
        w.at(r, n + r) = 1;
    }
    for (int r = 0; r < n; r++) {
        if (w.at(r, r) == 0) {
            int s = r + 1;
            while (s < n && w.at(s, r) == 0) s++;
            if (s == n) return false;
            for (int c = 0; c < 2 * n; c++) std::swap(w.at(r, c), w.at(s, c));
        }
        const uint8_t p = w.at(r, r);
        if (p != 1)
            for (int c = 0; c < 2 * n; c++) w.at(r, c) = g.div(w.at(r, c), p);
        for (int o = 0; o < n; o++) {
            if (o == r) continue;
            const uint8_t f = w.at(o, r);
            if (!f) continue;
            for (int c = 0; c < 2 * n; c++) w.at(o, c) ^= g.mul(f, w.at(r, c));
        }
    }
    out = Matrix(n, n);
    for (int r = 0; r < n; r++) std::memcpy(&out.at(r, 0), &w.at(r, n), size_t(n));
    return true;
}

Matrix build_encode_matrix(int k, int m) {
    const GF256& g = gf();
    const int n = k + m;
    Matrix vm(n, k);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) vm.at(r, c) = g.pow(uint8_t(r), c);
    Matrix top(k, k);
    for (int r = 0; r < k; r++) std::memcpy(&top.at(r, 0), vm.row(r), size_t(k));
    Matrix inv;
    mat_invert(top, inv);  // a Vandermonde top square with distinct rows is never singular
    return mat_mul(vm, inv);
}

}  // namespace rsmi
