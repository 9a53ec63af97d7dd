// Test helper (tests/test_cpu_gf8_const.py): prints the compile-time GF(2^8)
// tables of leopard_amd/csrc/gf8_const.h -- the constants every multiplier of
// the bit-sliced tile (rs_ff8_bs.hip) is compiled from -- as whitespace-separated
// integers: 256 logs, 256 exps, 255 skews (elements), then the 8 x 8 GF(2)
// matrices of multiply-by-c for c = 0 .. 255 as 64-bit integers.
#include <cstdio>

#include "gf8_const.h"

static_assert(lamd::kGf8.log[0] == 255, "log of zero is the modulus");

int main() {
    for (unsigned i = 0; i < 256; ++i) std::printf("%u ", unsigned(lamd::kGf8.log[i]));
    std::printf("\n");
    for (unsigned i = 0; i < 256; ++i) std::printf("%u ", unsigned(lamd::kGf8.exp[i]));
    std::printf("\n");
    for (unsigned i = 0; i < 255; ++i) std::printf("%u ", lamd::gf8_skew(int(i)));
    std::printf("\n");
    for (unsigned c = 0; c < 256; ++c) std::printf("%llu ", static_cast<unsigned long long>(lamd::gf8_matrix(c)));
    std::printf("\n");
    return 0;
}
