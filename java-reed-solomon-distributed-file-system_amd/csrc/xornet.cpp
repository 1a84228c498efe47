// xornet.cpp -- see xornet.hpp.
#include "xornet.hpp"

#include <hip/hiprtc.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <tuple>
#include <vector>

#include "gf256.hpp"

namespace rsamd {
namespace {

// Device prelude of every generated kernel.  tr8 transposes 8 dwords as four
// 8x8 bit matrices (row r = dword r, column b = bit b of a byte): afterwards
// dword b holds bit b of every byte, byte j / dword i of the input landing at
// bit 8j + i.  It is an involution, so the same network turns output planes
// back into bytes.  Each stage swaps the off-diagonal blocks of a pair of rows
// with two shift + bit-select (v_bfi_b32) pairs: 48 VALU ops per 32 bytes.
const char *kPrelude = R"(
typedef unsigned int u32;
typedef unsigned long long u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
struct XorNetArgs {
    unsigned char *base;
    const int *in_idx;
    const int *out_idx;
    u64 stripe_stride;
    u64 shard_stride;
    u32 chunks, n_items, cdiv_m, cdiv_s1, cdiv_s2, xcd_span, rot;
    int *mismatch;
};
static __device__ __forceinline__ u32 x3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
static __device__ __forceinline__ u32x4 ld(const unsigned char *p) {
    return __builtin_nontemporal_load((const u32x4 *)p);
}
static __device__ __forceinline__ void st(unsigned char *p, u32x4 v) { __builtin_nontemporal_store(v, (u32x4 *)p); }
// sel(a, b, m) = m ? b : a per bit: v_bitop3_b32 truth table 0xD8 (operand
// bytes 0xF0 / 0xCC / 0xAA).  As a builtin, not the C expression: LLVM rewrites
// (a & ~m) | (b & m) as ((a ^ b) & m) ^ a and distributes the masks into the
// XOR network (1560 instead of 1230 VALU ops for 10+4).
static __device__ __forceinline__ u32 sel(u32 a, u32 b, u32 m) { return __builtin_amdgcn_bitop3_b32(a, b, m, 0xD8); }
#define RS_SW(a, b, s, lo)                                                   \
    {                                                                        \
        const u32 a_ = (a), b_ = (b);                                        \
        (a) = sel(a_, b_ << (s), (lo) << (s));                               \
        (b) = sel(b_, a_ >> (s), (lo));                                      \
    }
static __device__ __forceinline__ void tr8(u32 (&d)[8]) {
    RS_SW(d[0], d[4], 4, 0x0F0F0F0Fu) RS_SW(d[1], d[5], 4, 0x0F0F0F0Fu)
    RS_SW(d[2], d[6], 4, 0x0F0F0F0Fu) RS_SW(d[3], d[7], 4, 0x0F0F0F0Fu)
    RS_SW(d[0], d[2], 2, 0x33333333u) RS_SW(d[1], d[3], 2, 0x33333333u)
    RS_SW(d[4], d[6], 2, 0x33333333u) RS_SW(d[5], d[7], 2, 0x33333333u)
    RS_SW(d[0], d[1], 1, 0x55555555u) RS_SW(d[2], d[3], 1, 0x55555555u)
    RS_SW(d[4], d[5], 1, 0x55555555u) RS_SW(d[6], d[7], 1, 0x55555555u)
}
static __device__ __forceinline__ u32 fdiv(u32 n, u32 m, u32 s1, u32 s2) {
    const u32 t = (u32)(((u64)n * m) >> 32);
    return (t + ((n - t) >> s1)) >> s2;
}
)";

// Operand of the network for one input: 0..7 = plane X[b], 8.. = temporaries.
struct Temp {
    int a, b;
};

// One input's contribution to the 8*nout output planes: for row (p, j) the
// planes b of input i with bit j of row[p][i] * 2^b set.  Pairs of operands
// that recur in >= 3 rows are hoisted into a temporary (one XOR saves about
// half an op per row that uses it).
void input_network(const std::vector<uint8_t> &coef, std::vector<std::vector<int>> *rows, std::vector<Temp> *temps) {
    const Gf256 &gf = Gf256::instance();
    const int nout = int(coef.size());
    rows->assign(size_t(nout) * 8, {});
    for (int p = 0; p < nout; ++p)
        for (int b = 0; b < 8; ++b) {
            const uint8_t col = gf.mul(coef[p], uint8_t(1u << b));
            for (int j = 0; j < 8; ++j)
                if ((col >> j) & 1) (*rows)[size_t(p) * 8 + j].push_back(b);
        }
    temps->clear();
    for (;;) {
        std::map<std::pair<int, int>, int> count;
        for (const auto &r : *rows)
            for (size_t x = 0; x < r.size(); ++x)
                for (size_t y = x + 1; y < r.size(); ++y) ++count[{std::min(r[x], r[y]), std::max(r[x], r[y])}];
        std::pair<int, int> best{-1, -1};
        int best_n = 2;
        for (const auto &kv : count)
            if (kv.second > best_n) {
                best_n = kv.second;
                best = kv.first;
            }
        if (best.first < 0) break;
        const int id = 8 + int(temps->size());
        temps->push_back({best.first, best.second});
        for (auto &r : *rows) {
            auto ia = std::find(r.begin(), r.end(), best.first), ib = std::find(r.begin(), r.end(), best.second);
            if (ia == r.end() || ib == r.end()) continue;
            r.erase(std::remove_if(r.begin(), r.end(), [&](int v) { return v == best.first || v == best.second; }),
                    r.end());
            r.push_back(id);
        }
    }
}

std::string operand(int id, int i) {
    return id < 8 ? "X" + std::to_string(i) + "[" + std::to_string(id) + "]"
                  : "T" + std::to_string(i) + "_" + std::to_string(id - 8);
}

// acc (= or ^=) XOR of terms, folded with 3-input XORs; returns the op count.
int emit_fold(std::ostringstream &o, const std::string &acc, bool init, std::vector<std::string> terms) {
    if (terms.empty()) return 0;
    if (!init) terms.insert(terms.begin(), acc);
    int ops = 0;
    while (terms.size() >= 3) {
        const std::string e = "x3(" + terms[0] + ", " + terms[1] + ", " + terms[2] + ")";
        terms.erase(terms.begin(), terms.begin() + 3);
        terms.insert(terms.begin(), e);
        ++ops;
    }
    std::string e = terms[0];
    if (terms.size() == 2) {
        e = "(" + terms[0] + " ^ " + terms[1] + ")";
        ++ops;
    }
    o << "        " << acc << " = " << e << ";\n";
    return ops;
}

}  // namespace

std::string xornet_source(const uint8_t *rows, int nin, int nout, bool verify, const std::string &name, int *ops_out) {
    std::ostringstream o;
    int ops = 0;
    o << kPrelude;
    o << "extern \"C\" __global__ void __launch_bounds__(64) " << name << "(XorNetArgs a) {\n";
    if (verify) o << "    if (*a.mismatch) return;\n";
    o << "    u32 b = blockIdx.x;\n"
         "    if (a.xcd_span && b < 8u * a.xcd_span) b = (b & 7u) * a.xcd_span + (b >> 3);\n"
         "    const u32 stripe = fdiv(b, a.cdiv_m, a.cdiv_s1, a.cdiv_s2);\n"
         "    u32 chunk = b - stripe * a.chunks;\n"
         "    if (a.rot) {  // stripe * rot < n_items\n"
         "        const u32 p = stripe * a.rot;\n"
         "        chunk += p - fdiv(p, a.cdiv_m, a.cdiv_s1, a.cdiv_s2) * a.chunks;\n"
         "        if (chunk >= a.chunks) chunk -= a.chunks;\n"
         "    }\n"
         "    unsigned char *sb = a.base + (u64)stripe * a.stripe_stride + (u64)chunk * "
      << kXorChunk << "u + threadIdx.x * 16u;\n";
    for (int p = 0; p < nout; ++p)
        o << "    const u64 oo" << p << " = (u64)a.out_idx[" << p << "] * a.shard_stride;\n";
    for (int i = 0; i < nin; ++i)
        o << "    const u64 oi" << i << " = (u64)a.in_idx[" << i << "] * a.shard_stride;\n";
    // Every input's two 16-byte halves are loaded up front (as the vector
    // kernels do): 8 dwords per input in flight per lane.
    for (int i = 0; i < nin; ++i)
        o << "    const u32x4 L" << i << "a = ld(sb + oi" << i << "), L" << i << "b = ld(sb + oi" << i << " + "
          << kXorChunk / 2 << ");\n";
    o << "    u32 A[" << nout << "][8];\n";
    std::vector<bool> init(size_t(nout) * 8, true);
    for (int i = 0; i < nin; ++i) {
        std::vector<uint8_t> coef(nout);
        for (int p = 0; p < nout; ++p) coef[p] = rows[size_t(p) * nin + i];
        std::vector<std::vector<int>> net;
        std::vector<Temp> temps;
        input_network(coef, &net, &temps);
        o << "    {\n        u32 X" << i << "[8] = {L" << i << "a.x, L" << i << "a.y, L" << i << "a.z, L" << i << "a.w, L"
          << i << "b.x, L" << i << "b.y, L" << i << "b.z, L" << i << "b.w};\n        tr8(X" << i << ");\n";
        ops += 48;
        for (size_t t = 0; t < temps.size(); ++t) {
            o << "        const u32 " << operand(8 + int(t), i) << " = " << operand(temps[t].a, i) << " ^ "
              << operand(temps[t].b, i) << ";\n";
            ++ops;
        }
        for (int r = 0; r < nout * 8; ++r) {
            std::vector<std::string> terms;
            for (int id : net[r]) terms.push_back(operand(id, i));
            const std::string acc = "A[" + std::to_string(r / 8) + "][" + std::to_string(r % 8) + "]";
            ops += emit_fold(o, acc, init[r], terms);
            if (!terms.empty()) init[r] = false;
        }
        o << "    }\n";
    }
    for (int r = 0; r < nout * 8; ++r)
        if (init[r]) o << "    A[" << r / 8 << "][" << r % 8 << "] = 0u;\n";
    for (int p = 0; p < nout; ++p) {
        o << "    {\n        u32 Y[8] = {A[" << p << "][0], A[" << p << "][1], A[" << p << "][2], A[" << p
          << "][3], A[" << p << "][4], A[" << p << "][5], A[" << p << "][6], A[" << p << "][7]};\n"
          << "        tr8(Y);\n";
        ops += 48;
        if (verify) {
            o << "        const u32x4 Ha = ld(sb + oo" << p << "), Hb = ld(sb + oo" << p << " + " << kXorChunk / 2
              << ");\n"
                 "        if (Ha.x != Y[0] || Ha.y != Y[1] || Ha.z != Y[2] || Ha.w != Y[3] || Hb.x != Y[4] ||\n"
                 "            Hb.y != Y[5] || Hb.z != Y[6] || Hb.w != Y[7])\n"
                 "            __hip_atomic_fetch_or(a.mismatch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n";
        } else {
            o << "        st(sb + oo" << p << ", u32x4{Y[0], Y[1], Y[2], Y[3]});\n"
              << "        st(sb + oo" << p << " + " << kXorChunk / 2 << ", u32x4{Y[4], Y[5], Y[6], Y[7]});\n";
        }
        o << "    }\n";
    }
    o << "}\n";
    if (ops_out) *ops_out = ops;
    return o.str();
}

namespace {

std::atomic<int> g_compiled{0};

struct Key {
    int dev, nin, nout;
    bool verify;
    std::vector<uint8_t> rows;
    bool operator<(const Key &o) const {
        return std::tie(dev, nin, nout, verify, rows) < std::tie(o.dev, o.nin, o.nout, o.verify, o.rows);
    }
};

struct Entry {
    std::once_flag once;
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    hipError_t status = hipErrorNotReady;
    std::string err;
};

std::mutex g_mu;
std::map<Key, std::unique_ptr<Entry>> g_cache;  // modules live for the process

void compile(const Key &k, Entry *e) {
    const std::string name = "rsamd_xornet";
    const std::string src = xornet_source(k.rows.data(), k.nin, k.nout, k.verify, name);
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "rsamd_xornet.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        e->status = hipErrorInvalidValue;
        e->err = "hiprtcCreateProgram failed";
        return;
    }
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    const hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        e->status = hipErrorInvalidImage;
        e->err = std::string("hiprtc: ") + hiprtcGetErrorString(rc) + ": " + log.substr(0, 2000);
        hiprtcDestroyProgram(&prog);
        return;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    std::vector<char> code(n);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    e->status = hipModuleLoadData(&e->mod, code.data());
    if (e->status != hipSuccess) {
        e->err = "hipModuleLoadData failed";
        return;
    }
    e->status = hipModuleGetFunction(&e->fn, e->mod, name.c_str());
    if (e->status != hipSuccess) e->err = "hipModuleGetFunction failed";
    else g_compiled.fetch_add(1);
}

}  // namespace

hipError_t xornet_function(const uint8_t *rows, int nin, int nout, bool verify, hipFunction_t *fn, std::string *err) {
    int dev = 0;
    hipError_t he = hipGetDevice(&dev);
    if (he != hipSuccess) return he;
    Key k{dev, nin, nout, verify, std::vector<uint8_t>(rows, rows + size_t(nin) * nout)};
    Entry *e;
    {
        std::lock_guard<std::mutex> lock(g_mu);
        auto &slot = g_cache[k];
        if (!slot) slot.reset(new Entry);
        e = slot.get();
    }
    std::call_once(e->once, [&] { compile(k, e); });  // other callers of this key wait; other keys do not
    if (e->status != hipSuccess) {
        if (err) *err = e->err;
        return e->status;
    }
    *fn = e->fn;
    return hipSuccess;
}

hipError_t launch_xornet(hipFunction_t fn, const XorNetArgs &a, hipStream_t s) {
    XorNetArgs arg = a;
    size_t size = sizeof arg;
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &arg, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
    return hipModuleLaunchKernel(fn, a.n_items, 1, 1, 64, 1, 1, 0, s, nullptr, cfg);
}

bool xornet_enabled() {
    static const bool env_on = [] {
        const char *e = std::getenv("RSAMD_XORNET");
        return e && e[0] == '1';
    }();
    return env_on;
}

int xornet_compiled_count() { return g_compiled.load(); }

}  // namespace rsamd
