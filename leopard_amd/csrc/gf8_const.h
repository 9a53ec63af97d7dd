// gf8_const.h -- GF(2^8) in Leopard's Cantor-basis representation, built at
// compile time (constexpr), for kernels whose butterfly multipliers are
// compile-time constants (rs_ff8_bs.hip: bit-sliced tiles, where a multiply by
// a known constant is an XOR network over the 8 bit planes).
//
// The same construction as the host tables (gf_tables.cpp, which the rest of
// the library uses): logs via the LFSR of polynomial 0x11D over the Cantor
// basis (LeopardFF8.cpp:46-48, 158-194), FFT skews by FFTInitialize
// (LeopardFF8.cpp:496-531).  tests/test_cpu_gf8_const.py checks these tables
// and every multiply matrix against the host library's tables, the oracle's and
// the reference's own LogLUT / ExpLUT / FFTSkew (compiled reference, oracle/_ref).
#pragma once

#include <cstdint>

namespace lamd {

struct Gf8Const {
    uint8_t log[256] = {};   // log[x] of the element with Cantor coordinates x; log[0] = 255
    uint8_t exp[256] = {};   // exp[log[x]] = x, exp[255] = exp[0]
    uint8_t skew[255] = {};  // FFT skews as elements (not logs): 0 = the zero skew

    constexpr unsigned add_mod(unsigned a, unsigned b) const {
        const unsigned s = a + b;
        return (s + (s >> 8)) & 255u;
    }
    constexpr unsigned mul_log(unsigned x, unsigned lm) const { return x == 0 ? 0u : exp[add_mod(log[x], lm)]; }
    // x * c for elements x, c
    constexpr unsigned mul(unsigned x, unsigned c) const { return c == 0 ? 0u : mul_log(x, log[c]); }

    constexpr Gf8Const() {
        constexpr uint16_t cantor[8] = {1, 214, 152, 146, 86, 200, 88, 230};
        uint16_t poly_log[256] = {};
        unsigned x = 1;
        for (unsigned e = 0; e < 255; ++e) {
            poly_log[x] = uint16_t(e);
            x <<= 1;
            if (x & 256u) x ^= 0x11Du;
        }
        poly_log[0] = 255;
        uint16_t element[256] = {};
        for (unsigned c = 1; c < 256; ++c) {
            unsigned bit = 0;
            while (!((c >> bit) & 1u)) ++bit;
            element[c] = uint16_t(element[c & (c - 1)] ^ cantor[bit]);
        }
        for (unsigned c = 0; c < 256; ++c) log[c] = uint8_t(poly_log[element[c]]);
        for (unsigned c = 0; c < 256; ++c) exp[log[c]] = uint8_t(c);
        exp[255] = exp[0];
        // skews (as in gf_tables.cpp build_skews, elements until the final log step)
        unsigned sk[255] = {};
        unsigned v[7] = {};
        for (unsigned i = 0; i < 7; ++i) v[i] = 1u << (i + 1);
        for (unsigned lvl = 0; lvl < 7; ++lvl) {
            const unsigned first = (1u << lvl) - 1;
            sk[first] = 0;
            for (unsigned i = lvl; i < 7; ++i) {
                const unsigned span = 1u << (i + 1);
                for (unsigned j = first; j < span; j += 2u << lvl) sk[j + span] = sk[j] ^ v[i];
            }
            v[lvl] = 255u - log[mul_log(v[lvl], log[v[lvl] ^ 1u])];
            for (unsigned i = lvl + 1; i < 7; ++i) v[i] = mul_log(v[i], add_mod(log[v[i] ^ 1u], v[lvl]));
        }
        // sk[] holds elements; the reference converts them to logs (FFTSkew),
        // whose multiply is by exp(log) = the element itself
        for (unsigned i = 0; i < 255; ++i) skew[i] = uint8_t(sk[i]);
    }
};

inline constexpr Gf8Const kGf8{};

// 8 x 8 GF(2) matrix of "multiply by c" on bit planes: bit 8 i + j is bit i of
// (1 << j) * c, so plane i of c * y is the XOR of the planes j of y whose bit is set.
constexpr uint64_t gf8_matrix(unsigned c) {
    uint64_t m = 0;
    for (unsigned j = 0; j < 8; ++j) {
        const unsigned col = kGf8.mul(1u << j, c);
        for (unsigned i = 0; i < 8; ++i)
            if ((col >> i) & 1u) m |= uint64_t(1) << (8 * i + j);
    }
    return m;
}

// Skew element of FFT position `idx` (skew base + group index; the reference's
// FFTSkew[idx], as an element): 0 is the zero skew (XOR-only butterfly).
constexpr unsigned gf8_skew(int idx) { return kGf8.skew[idx]; }

}  // namespace lamd
