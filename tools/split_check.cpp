// split_check.cpp -- round-5 diagnosis of the r4zx wrong file encode (VERDICT
// r4 item 1): checks, on the CPU and without touching memory, the arithmetic
// that splits a pageable host call into page-locked interior rows / columns
// and staged ends (capi.cpp interior_rows, file_encode_interior,
// file_decode_interior, run_direct_interior), at the r4zx geometry (k=3, m=2,
// block 520, file 2,614,744 B, S = 872,040) and others, for every 8-byte
// view offset 0..4088 of the file and of the shards.  It includes capi.cpp
// itself, so the functions checked are the library's own.
//
// For each placement:
//   * the interior rows [r0, r1) and the staged pieces [0, r0), [r1, rows)
//     cover [0, rows) exactly once, and the pieces' file lengths sum to the
//     file length;
//   * every locked range, rounded to pages as HostRegistration::lock rounds
//     it, lies inside its own array;
//   * the interior's file bytes are all real file bytes (no padding row).
// Round 5 removed the path; this checker builds against the tree before the
// removal (capi.cpp of commit 4f31d22: `git show 4f31d22:java-reed-solomon-
// distributed-file-system_amd/csrc/capi.cpp`), linked with that tree's other
// objects; it prints one line per geometry and exits 1 on any violation
// (profiles/r5/split_check_r5.txt).
#include "../java-reed-solomon-distributed-file-system_amd/csrc/capi.cpp"

#include <cinttypes>
#include <random>

namespace {

int g_fail = 0;
uint64_t g_checked = 0;

bool page_inside(uintptr_t start, size_t n, uintptr_t arr, size_t len) {
    if (n == 0) return true;
    const uintptr_t ps = start & ~uintptr_t(4095), pe = (start + n + 4095) & ~uintptr_t(4095);
    return ps >= arr && pe <= arr + len;
}

void report(const char *what, const char *geom, size_t a, size_t b) {
    if (g_fail++ < 10) std::printf("VIOLATION %s: %s (%zu, %zu)\n", what, geom, a, b);
}

// File encode: arrays = file (per_row k*blk, len file_len) + T shards (per_row blk, len S).
void check_encode(int k, int m, size_t blk, size_t file_len, uintptr_t file, const std::vector<uintptr_t> &sh) {
    const size_t kb = size_t(k) * blk;
    const size_t padded = file_len % kb == 0 ? file_len : file_len / kb * kb + kb, S = padded / k, rows = S / blk;
    std::vector<RowArray> arrays{{reinterpret_cast<const uint8_t *>(file), file_len, kb}};
    for (uintptr_t p : sh) arrays.push_back({reinterpret_cast<const uint8_t *>(p), S, blk});
    size_t r0 = 0, r1 = 0;
    ++g_checked;
    if (!interior_rows(arrays, rows, &r0, &r1)) return;  // staged whole: nothing to check
    if (!(r0 < r1 && r1 <= rows)) report("encode rows out of order", "", r0, r1);
    if (r1 * kb > file_len) report("encode interior past the file", "", r1, file_len);
    for (const RowArray &a : arrays)
        if (!page_inside(reinterpret_cast<uintptr_t>(a.p) + r0 * a.per_row, (r1 - r0) * a.per_row,
                         reinterpret_cast<uintptr_t>(a.p), a.len))
            report("encode lock outside its array", "", r0, r1);
    // file_encode_interior's pieces and their file lengths
    size_t covered = r1 - r0, flen = (r1 - r0) * kb;
    for (const auto &piece : {std::make_pair(size_t(0), r0), std::make_pair(r1, rows)}) {
        const size_t a = piece.first, b = piece.second;
        if (b <= a) continue;
        covered += b - a;
        flen += std::min((b - a) * kb, file_len - a * kb);
    }
    if (covered != rows) report("encode rows not covered once", "", covered, rows);
    if (flen != file_len) report("encode file bytes not covered once", "", flen, file_len);
}

// File decode {0, T-1} (file_decode_interior): survivors per_row blk, len rows_needed*blk;
// rebuilt shards len S; file_out per_row k*blk, len file_size.
void check_decode(int k, int m, size_t blk, size_t file_size, uintptr_t fout, const std::vector<uintptr_t> &sh) {
    const int T = k + m;
    const size_t kb = size_t(k) * blk;
    const size_t padded = file_size % kb == 0 ? file_size : file_size / kb * kb + kb, S = padded / k, rows = S / blk;
    std::vector<int> surv, missing;
    for (int i = 0; i < T; ++i) {
        const bool present = i != 0 && i != T - 1;
        if (present && int(surv.size()) < k) surv.push_back(i);
        if (!present) missing.push_back(i);
    }
    const size_t rows_needed = file_rows_needed(k, S, blk, missing, file_size);
    std::vector<RowArray> arrays;
    for (int i : surv) arrays.push_back({reinterpret_cast<const uint8_t *>(sh[i]), rows_needed * blk, blk});
    for (int i : missing) arrays.push_back({reinterpret_cast<const uint8_t *>(sh[i]), S, blk});
    arrays.push_back({reinterpret_cast<const uint8_t *>(fout), file_size, kb});
    size_t r0 = 0, r1 = 0;
    ++g_checked;
    if (!interior_rows(arrays, rows_needed, &r0, &r1)) return;
    if (!(r0 < r1 && r1 <= rows_needed)) report("decode rows out of order", "", r0, r1);
    for (const RowArray &a : arrays)
        if (a.len && !page_inside(reinterpret_cast<uintptr_t>(a.p) + r0 * a.per_row, (r1 - r0) * a.per_row,
                                  reinterpret_cast<uintptr_t>(a.p), a.len))
            report("decode lock outside its array", "", r0, r1);
    auto fsz = [&](size_t a, size_t b) { return file_size > a * kb ? std::min(file_size - a * kb, (b - a) * kb) : 0; };
    size_t covered = r1 - r0, flen = fsz(r0, r1);
    for (const auto &piece : {std::make_pair(size_t(0), r0), std::make_pair(r1, rows_needed)}) {
        if (piece.second <= piece.first) continue;
        covered += piece.second - piece.first;
        flen += fsz(piece.first, piece.second);
    }
    if (covered != rows_needed) report("decode rows not covered once", "", covered, rows_needed);
    if (flen != file_size) report("decode file bytes not covered once", "", flen, file_size);
}

// run_direct_interior's column split (restated from capi.cpp:222-241, the
// only part of it that is not a call): [lo, hi) locked, [0, lo) and
// [hi, count) staged through the zero-copy buffer.
void check_columns(const std::vector<uintptr_t> &slots, size_t offset, size_t count) {
    constexpr uintptr_t kPage = 4096;
    size_t lo = 0, hi = count;
    ++g_checked;
    for (uintptr_t s : slots) {
        const uintptr_t a = s + offset;
        const uintptr_t first = (a + kPage - 1) & ~(kPage - 1), end = (a + count) & ~(kPage - 1);
        if (end <= first) return;
        lo = std::max<size_t>(lo, first - a);
        hi = std::min<size_t>(hi, end - a);
    }
    if (hi <= lo) return;
    for (uintptr_t s : slots)
        if (!page_inside(s + offset + lo, hi - lo, s + offset, count)) report("columns lock outside", "", lo, hi);
    if (lo + (hi - lo) + (count - hi) != count) report("columns not covered once", "", lo, hi);
}

}  // namespace

int main() {
    std::mt19937_64 rng(4);
    struct G {
        int k, m;
        size_t blk, n;
    };
    // r4zx's case first, then the other test_file_host_random_large cases' shapes
    const G geoms[] = {{3, 2, 520, 2614744}, {4, 2, 1000, 64u << 20}, {4, 2, 4096, 3u << 20},
                       {10, 4, 1024, 5000000}, {2, 1, 8, 300000}, {6, 3, 2048, 1 << 22}};
    for (const G &g : geoms) {
        const int T = g.k + g.m;
        const uint64_t before = g_checked;
        auto base = [](int i) { return uintptr_t(0x7f0000000000ull) + uintptr_t(i) * (uintptr_t(1) << 32); };
        for (size_t fo = 0; fo < 4096; fo += 8) {
            // shards at one common offset (every 8-byte residue), and at random 8-byte offsets
            for (size_t so = 0; so < 4096; so += 8) {
                std::vector<uintptr_t> sh(T);
                for (int i = 0; i < T; ++i) sh[i] = base(i + 1) + so;
                check_encode(g.k, g.m, g.blk, g.n, base(0) + fo, sh);
                check_decode(g.k, g.m, g.blk, g.n, base(0) + fo, sh);
            }
            for (int r = 0; r < 64; ++r) {
                std::vector<uintptr_t> sh(T);
                for (int i = 0; i < T; ++i) sh[i] = base(i + 1) + (rng() % 512) * 8;
                check_encode(g.k, g.m, g.blk, g.n, base(0) + fo, sh);
                check_decode(g.k, g.m, g.blk, g.n, base(0) + fo, sh);
                check_columns(sh, fo, g.n / size_t(g.k));
            }
        }
        std::printf("k=%d m=%d block=%zu n=%zu: %" PRIu64 " placements checked, violations so far %d\n", g.k, g.m,
                    g.blk, g.n, g_checked - before, g_fail);
    }
    std::printf("%s: %" PRIu64 " placements, %d violations\n", g_fail ? "FAIL" : "OK", g_checked, g_fail);
    return g_fail ? 1 : 0;
}
