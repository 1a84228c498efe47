// gf256.hpp -- GF(2^8) arithmetic and dense GF matrices for the host side of
// the engine (matrix construction and k x k inversion; the byte coding itself
// runs on the GPU).
//
// Field: generator polynomial 29 (x^8+x^4+x^3+x^2+1, Galois.java:42), primitive
// element 2, as Galois.java:258-305.  Matrix semantics follow Matrix.java:
// times (:191-208), invert by Gauss-Jordan with the same pivot rule (:271-344).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace rsamd {

class Gf256 {
public:
    static const Gf256 &instance();

    uint8_t mul(uint8_t a, uint8_t b) const {
        if (a == 0 || b == 0) return 0;
        return exp_[log_[a] + log_[b]];
    }
    // a / b; b must be non-zero (Galois.java:213-227 throws for b == 0).
    uint8_t div(uint8_t a, uint8_t b) const {
        if (a == 0) return 0;
        int l = int(log_[a]) - int(log_[b]);
        return exp_[l < 0 ? l + 255 : l];
    }
    // a ** n (Galois.java:238-253): n == 0 -> 1, even for a == 0.
    uint8_t pow(uint8_t a, int n) const {
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp_[(int(log_[a]) * n) % 255];
    }
    const uint8_t *log_table() const { return log_; }
    const uint8_t *exp_table() const { return exp_; }

private:
    Gf256();
    uint8_t log_[256];
    uint8_t exp_[510];
};

// Row-major GF(256) matrix.
class GfMatrix {
public:
    GfMatrix() = default;
    GfMatrix(int rows, int cols) : rows_(rows), cols_(cols), d_(size_t(rows) * cols, 0) {}

    static GfMatrix identity(int n);
    static GfMatrix vandermonde(int rows, int cols);  // V[r][c] = r ** c

    int rows() const { return rows_; }
    int cols() const { return cols_; }
    uint8_t at(int r, int c) const { return d_[size_t(r) * cols_ + c]; }
    uint8_t &at(int r, int c) { return d_[size_t(r) * cols_ + c]; }
    const uint8_t *row(int r) const { return d_.data() + size_t(r) * cols_; }
    const std::vector<uint8_t> &data() const { return d_; }

    GfMatrix times(const GfMatrix &rhs) const;
    GfMatrix select_rows(const std::vector<int> &rows) const;
    GfMatrix top(int n) const;  // first n rows
    // Returns false when singular (Matrix.java:310 "Matrix is singular").
    bool invert(GfMatrix *out) const;

private:
    int rows_ = 0, cols_ = 0;
    std::vector<uint8_t> d_;
};

// Systematic generator matrix of ReedSolomon.buildMatrix (ReedSolomon.java:312-324).
GfMatrix build_generator(int k, int total);

// Kernel form of "multiply by constant c": byte x = x0 | x1<<3 | x2<<6 with
// x0, x1 in [0,8) and x2 in [0,4); c*x = T0[x0] ^ T1[x1] ^ T2[x2].  Each
// table is packed as little-endian bytes so one v_perm_b32 looks up four
// bytes at once: {t0lo, t0hi} = T0[0..7], {t1lo, t1hi} = T1[0..7], t2 = T2[0..3].
struct PermTable {
    uint32_t t0lo, t0hi, t1lo, t1hi, t2;
};
static_assert(sizeof(PermTable) == 20, "PermTable is 5 dwords");
PermTable perm_table(uint8_t c);

}  // namespace rsamd
