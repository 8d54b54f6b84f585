// crc_clmul.cpp -- carry-less-multiply folding for the datanode's reflected CRCs (algebra in
// crc_clmul.hpp).  Four 512-bit accumulators (sixteen 16-byte lanes) fold 256 bytes per step
// with VPCLMULQDQ; the lanes then fold into one 16-byte accumulator with per-distance
// constants, whole 16-byte blocks follow one at a time, and the byte table finishes.
#include "crc_clmul.hpp"

#include <atomic>

#include <immintrin.h>

#include <cstring>

namespace rsmi {
namespace host {

namespace {

struct Engine {
    int w;
    uint64_t pfull;      // normal-order polynomial including x^w
    uint32_t t[256];     // reflected byte table
    uint64_t k256[2];    // fold by 256 bytes: x^(2048 + 63), x^(2048 - 1) mod P, reflected
    uint64_t kd[16][2];  // fold by d 16-byte blocks (d >= 1)

    uint64_t xpow(uint64_t n) const {  // x^n mod P, normal order
        uint64_t r = 1;
        for (uint64_t i = 0; i < n; i++) {
            r <<= 1;
            if ((r >> w) & 1) r ^= pfull;
        }
        return r;
    }
    uint64_t refl64(uint64_t r) const {  // bit 63 - d <-> x^d
        uint64_t o = 0;
        for (int d = 0; d < w; d++)
            if ((r >> d) & 1) o |= uint64_t(1) << (63 - d);
        return o;
    }
    Engine(int width, uint64_t poly) : w(width), pfull(poly | (uint64_t(1) << width)) {
        uint32_t rp = 0;  // reflected polynomial (without x^w)
        for (int d = 0; d < w; d++)
            if ((poly >> d) & 1) rp |= 1u << (w - 1 - d);
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int j = 0; j < 8; j++) c = (c & 1) ? (c >> 1) ^ rp : c >> 1;
            t[i] = c;
        }
        k256[0] = refl64(xpow(2048 + 63));
        k256[1] = refl64(xpow(2048 - 1));
        for (int d = 1; d < 16; d++) {
            kd[d][0] = refl64(xpow(128 * uint64_t(d) + 63));
            kd[d][1] = refl64(xpow(128 * uint64_t(d) - 1));
        }
        kd[0][0] = kd[0][1] = 0;
    }
    uint32_t bytes(uint32_t s, const uint8_t* p, size_t n) const {
        for (size_t i = 0; i < n; i++) s = t[(s ^ p[i]) & 0xFF] ^ (s >> 8);
        return s;
    }
};

bool cpu_ok() {
    static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("vpclmulqdq") &&
                           __builtin_cpu_supports("pclmul");
    return ok;
}

__attribute__((target("avx512f,vpclmulqdq,pclmul,sse4.1"))) inline __m128i fold16(__m128i x, __m128i k, __m128i b) {
    return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), b);
}

__attribute__((target("avx512f,vpclmulqdq,pclmul,sse4.1"))) uint32_t fold(const Engine& E, uint32_t s,
                                                                          const uint8_t* p, size_t n) {
    // n >= 256: the register's start value XORs into the first bytes
    __m512i x[4];
    for (int a = 0; a < 4; a++) x[a] = _mm512_loadu_si512(p + 64 * a);
    x[0] = _mm512_xor_si512(x[0], _mm512_zextsi128_si512(_mm_cvtsi32_si128(int(s))));
    const __m512i k = _mm512_broadcast_i32x4(_mm_set_epi64x(int64_t(E.k256[1]), int64_t(E.k256[0])));
    size_t i = 256;
    for (; i + 256 <= n; i += 256) {
        for (int a = 0; a < 4; a++) {
            const __m512i b = _mm512_loadu_si512(p + i + 64 * a);
            x[a] = _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x[a], k, 0x00),
                                             _mm512_clmulepi64_epi128(x[a], k, 0x11), b, 0x96);
        }
    }
    // lane j (16-byte block j of the last 256 bytes) moves forward by 15 - j blocks
    alignas(64) uint8_t lanes[256];
    for (int a = 0; a < 4; a++) _mm512_store_si512(lanes + 64 * a, x[a]);
    __m128i acc = _mm_load_si128(reinterpret_cast<const __m128i*>(lanes + 240));
    for (int j = 0; j < 15; j++) {
        const __m128i kj = _mm_set_epi64x(int64_t(E.kd[15 - j][1]), int64_t(E.kd[15 - j][0]));
        acc = fold16(_mm_load_si128(reinterpret_cast<const __m128i*>(lanes + 16 * j)), kj, acc);
    }
    const __m128i k1 = _mm_set_epi64x(int64_t(E.kd[1][1]), int64_t(E.kd[1][0]));
    for (; i + 16 <= n; i += 16) acc = fold16(acc, k1, _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i)));
    alignas(16) uint8_t last[16];
    _mm_store_si128(reinterpret_cast<__m128i*>(last), acc);
    return E.bytes(E.bytes(0, last, 16), p + i, n - i);
}

const Engine& crc16_engine() {
    static const Engine e(16, 0x8005);
    return e;
}
const Engine& crc32_engine() {
    static const Engine e(32, 0x04C11DB7);
    return e;
}

}  // namespace

// Test switch (tests/test_erasure_host.py): force every length onto the callers' table loops,
// so hosts with VPCLMULQDQ still test the path that CPUs without it take.
std::atomic<int> g_force_tables{0};

uint32_t clmul_crc16(uint32_t s, const uint8_t* p, size_t n, bool* done) {
    *done = n >= 256 && !g_force_tables.load(std::memory_order_relaxed) && cpu_ok();
    return *done ? fold(crc16_engine(), s, p, n) : s;
}

uint32_t clmul_crc32(uint32_t s, const uint8_t* p, size_t n, bool* done) {
    *done = n >= 256 && !g_force_tables.load(std::memory_order_relaxed) && cpu_ok();
    return *done ? fold(crc32_engine(), s, p, n) : s;
}

}  // namespace host
}  // namespace rsmi

// test-only (not in include/rsmi.h): 1 = the datanode CRCs take the slice-by-8 loops at every
// length, 0 = carry-less folding from 256 bytes where the CPU has it (the default)
extern "C" void rsmi_host_crc_force_tables(int on) { rsmi::host::g_force_tables.store(on ? 1 : 0); }
