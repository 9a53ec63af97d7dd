// gf_tables.h -- host-side construction of the GF(2^8)/GF(2^16) tables that the
// device kernels consume.  Built once in leo_init() (reference: ff8/ff16
// Initialize(), LeopardFF8.cpp:1922-1935, LeopardFF16.cpp:1781-1794).
#pragma once

#include <cstdint>
#include <vector>

namespace lamd {

// One binary extension field in Leopard's Cantor-basis representation.
//   log_of[x]   : discrete log of the element whose Cantor coordinates are x
//                 (log_of[0] == modulus, i.e. "zero"),     LeopardFF8.cpp:158-194
//   exp_of[l]   : inverse map, exp_of[modulus] == exp_of[0]
//   skew[i]     : FFT skew factors as logs (modulus == the zero element),
//                 eq. (28) of Lin-Chung-Han,                LeopardFF8.cpp:496-531
//   log_walsh[i]: FWHT of log_of (log_of[0] := 0),          LeopardFF8.cpp:533-537
class GaloisField {
public:
    GaloisField(unsigned bits, unsigned polynomial, const uint16_t* cantor_basis);

    unsigned bits() const { return bits_; }
    unsigned order() const { return order_; }
    unsigned modulus() const { return modulus_; }

    // Partially reduced mod 2^bits - 1 (the modulus itself stands for 0).
    unsigned add_mod(unsigned a, unsigned b) const {
        unsigned s = a + b;
        return (s + (s >> bits_)) & modulus_;
    }
    unsigned sub_mod(unsigned a, unsigned b) const {
        unsigned d = a - b;
        return (d + (d >> bits_)) & modulus_;
    }
    // x * exp(log_m): the only multiply Leopard ever performs (LeopardFF8.cpp:141-154).
    unsigned mul_log(unsigned x, unsigned log_m) const {
        return x == 0 ? 0u : exp_of[add_mod(log_of[x], log_m)];
    }
    // In-place Walsh-Hadamard transform mod 2^bits - 1 over `n` entries.
    void walsh(uint16_t* v, unsigned n) const;

    std::vector<uint16_t> log_of, exp_of, skew, log_walsh;

private:
    void build_logs(unsigned polynomial, const uint16_t* basis);
    void build_skews();

    unsigned bits_, order_, modulus_;
};

const GaloisField& field8();
const GaloisField& field16();

// Byte-permute multiply tables consumed by v_perm_b32 (see rs_device.h).
//
// FF8, 8 dwords per log value L (entries are products x * exp(L)):
//   [0..1] 8 entries for input bits 0-2     [2..3] bits 3-5
//   [4]    4 entries for input bits 6-7     [5..7] zero padding
// FF16, 24 dwords per log value L (element = lo | hi << 8; every input chunk
// gives a 16-bit product, split into a low-byte table and a high-byte table):
//   chunk lo[0-2]: [0..1] lo-byte, [2..3] hi-byte     chunk lo[3-5]: [4..7]
//   chunk hi[0-2]: [8..11]                             chunk hi[3-5]: [12..15]
//   chunk lo[6-7]: [16] lo-byte, [17] hi-byte          chunk hi[6-7]: [18], [19]
//   [20..23] zero padding
// Both arrays carry one extra all-zero table at index order (multiply by 0).
constexpr unsigned kTab8Dwords = 8;
constexpr unsigned kTab16Dwords = 24;
void build_perm_tables8(const GaloisField& f, std::vector<uint32_t>& out);
void build_perm_tables16(const GaloisField& f, std::vector<uint32_t>& out);

// Butterfly tables indexed by FFT-skew position i (not by log value): entry i
// holds the multiply table of skew[i] and, in dword kSkewFlagDw, 1 when skew[i]
// is the zero element (the butterfly then only XORs, LeopardFF8.cpp:690-708).
// Kernels fetch entry (skew offset + group index) with one scalar load, with no
// dependent skew -> log -> table chain.  order entries (the last is padding).
constexpr unsigned kSkewFlagDw8 = 5;
constexpr unsigned kSkewFlagDw16 = 20;
void build_skew_tables(const GaloisField& f, const std::vector<uint32_t>& perm_tables, unsigned tab_dwords,
                       unsigned flag_dw, std::vector<uint32_t>& out);

// FF8 encoder: the top IFFT layer of chunk c fused with the top FFT layer
// (rs_ff8.hip): entry (T - 1) * 256 + c holds the multiply table (kTab8Dwords)
// of skew-element(m - 1 + c*m + m/2) + skew-element(m/2 - 1), m = 2^T.
constexpr unsigned kFused8Entries = 7 * 256;
void build_fused_top_tables8(const GaloisField& f, const std::vector<uint32_t>& perm_tables,
                             std::vector<uint32_t>& out);

// FF16 encoders: the same fused top layer as a table index (log value, or
// order() for the all-zero table) per (T, chunk c) at fused16_base(T) + c,
// T = 1..15 (65536 >> T chunks each); the kernels read tab16[index].
constexpr unsigned kFused16Entries = 65536;
constexpr unsigned fused16_base(unsigned T) { return 65536u - (131072u >> T); }
void build_fused_top_logs16(const GaloisField& f, std::vector<uint32_t>& out);

// FF16 decoder, n = 256 * 2^H (H = 1..3): the high part of the transform as
// q[t ^ t'] over tile indices (rs_ff16_small.hip), entry high_q16_base(H) + k:
// the log value of q[k], or kHighQZero / kHighQOne.
constexpr unsigned kHighQ16Entries = 14;
constexpr uint32_t kHighQZero = 0xFFFFFFFFu, kHighQOne = 0xFFFFFFFEu;
constexpr unsigned high_q16_base(unsigned H) { return (1u << H) - 2; }
bool build_high_q16(const GaloisField& f, std::vector<uint32_t>& out);

}  // namespace lamd
