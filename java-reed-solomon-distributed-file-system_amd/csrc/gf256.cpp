// gf256.cpp -- see gf256.hpp.
#include "gf256.hpp"

#include <utility>

namespace rsamd {

Gf256::Gf256() {
    // Powers of the primitive element 2 modulo x^8+x^4+x^3+x^2+1 (0x11D):
    // the same walk as Galois.generateLogTable (Galois.java:258-275).
    unsigned b = 1;
    for (int l = 0; l < 255; ++l) {
        log_[b] = uint8_t(l);
        exp_[l] = uint8_t(b);
        exp_[l + 255] = uint8_t(b);  // doubled like Galois.java:285 so log a + log b needs no mod
        b <<= 1;
        if (b & 0x100) b ^= 0x11D;
    }
    log_[0] = 0;  // never read: mul/div/pow test for zero first
}

const Gf256 &Gf256::instance() {
    static const Gf256 g;
    return g;
}

GfMatrix GfMatrix::identity(int n) {
    GfMatrix m(n, n);
    for (int i = 0; i < n; ++i) m.at(i, i) = 1;
    return m;
}

GfMatrix GfMatrix::vandermonde(int rows, int cols) {
    const Gf256 &gf = Gf256::instance();
    GfMatrix m(rows, cols);
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) m.at(r, c) = gf.pow(uint8_t(r), c);
    return m;
}

GfMatrix GfMatrix::times(const GfMatrix &rhs) const {
    const Gf256 &gf = Gf256::instance();
    GfMatrix out(rows_, rhs.cols_);
    for (int r = 0; r < rows_; ++r)
        for (int c = 0; c < rhs.cols_; ++c) {
            uint8_t v = 0;
            for (int i = 0; i < cols_; ++i) v ^= gf.mul(at(r, i), rhs.at(i, c));
            out.at(r, c) = v;
        }
    return out;
}

GfMatrix GfMatrix::select_rows(const std::vector<int> &rows) const {
    GfMatrix out(int(rows.size()), cols_);
    for (size_t i = 0; i < rows.size(); ++i)
        for (int c = 0; c < cols_; ++c) out.at(int(i), c) = at(rows[i], c);
    return out;
}

GfMatrix GfMatrix::top(int n) const {
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    return select_rows(idx);
}

bool GfMatrix::invert(GfMatrix *out) const {
    const Gf256 &gf = Gf256::instance();
    const int n = rows_;
    // Work on [A | I]; pivot search = first lower row with a non-zero entry
    // (Matrix.java:300-307), forward pass then backward pass.
    GfMatrix w(n, 2 * n);
    for (int r = 0; r < n; ++r) {
        for (int c = 0; c < n; ++c) w.at(r, c) = at(r, c);
        w.at(r, n + r) = 1;
    }
    const int W = 2 * n;
    for (int r = 0; r < n; ++r) {
        if (w.at(r, r) == 0) {
            for (int below = r + 1; below < n; ++below)
                if (w.at(below, r) != 0) {
                    for (int c = 0; c < W; ++c) std::swap(w.at(r, c), w.at(below, c));
                    break;
                }
        }
        if (w.at(r, r) == 0) return false;
        if (w.at(r, r) != 1) {
            uint8_t s = gf.div(1, w.at(r, r));
            for (int c = 0; c < W; ++c) w.at(r, c) = gf.mul(w.at(r, c), s);
        }
        for (int below = r + 1; below < n; ++below) {
            uint8_t s = w.at(below, r);
            if (s)
                for (int c = 0; c < W; ++c) w.at(below, c) ^= gf.mul(s, w.at(r, c));
        }
    }
    for (int d = 0; d < n; ++d)
        for (int above = 0; above < d; ++above) {
            uint8_t s = w.at(above, d);
            if (s)
                for (int c = 0; c < W; ++c) w.at(above, c) ^= gf.mul(s, w.at(d, c));
        }
    GfMatrix inv(n, n);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) inv.at(r, c) = w.at(r, n + c);
    *out = std::move(inv);
    return true;
}

GfMatrix build_generator(int k, int total) {
    GfMatrix v = GfMatrix::vandermonde(total, k);
    GfMatrix inv;
    v.top(k).invert(&inv);  // a Vandermonde top square over distinct points is never singular
    return v.times(inv);
}

PermTable perm_table(uint8_t c) {
    const Gf256 &gf = Gf256::instance();
    uint8_t t0[8], t1[8], t2[4];
    for (int j = 0; j < 8; ++j) {
        t0[j] = gf.mul(c, uint8_t(j));
        t1[j] = gf.mul(c, uint8_t(j << 3));
    }
    for (int j = 0; j < 4; ++j) t2[j] = gf.mul(c, uint8_t(j << 6));
    auto pack = [](const uint8_t *b) {
        return uint32_t(b[0]) | uint32_t(b[1]) << 8 | uint32_t(b[2]) << 16 | uint32_t(b[3]) << 24;
    };
    return PermTable{pack(t0), pack(t0 + 4), pack(t1), pack(t1 + 4), pack(t2)};
}

}  // namespace rsamd
