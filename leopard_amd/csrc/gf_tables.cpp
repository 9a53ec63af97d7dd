// gf_tables.cpp -- see gf_tables.h.
#include "gf_tables.h"

#include <algorithm>
#include <array>

namespace lamd {

namespace {
// Cantor bases (reference LeopardFF8.cpp:46-48, LeopardFF16.cpp:46-51).
constexpr std::array<uint16_t, 8> kCantor8 = {1, 214, 152, 146, 86, 200, 88, 230};
constexpr std::array<uint16_t, 16> kCantor16 = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                                0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
}  // namespace

GaloisField::GaloisField(unsigned bits, unsigned polynomial, const uint16_t* cantor_basis)
    : bits_(bits), order_(1u << bits), modulus_((1u << bits) - 1) {
    build_logs(polynomial, cantor_basis);
    build_skews();
}

void GaloisField::walsh(uint16_t* v, unsigned n) const {
    for (unsigned half = 1; half < n; half *= 2) {
        for (unsigned base = 0; base < n; base += 2 * half) {
            uint16_t* lo = v + base;
            uint16_t* hi = v + base + half;
            for (unsigned i = 0; i < half; ++i) {
                const unsigned a = lo[i], b = hi[i];
                lo[i] = static_cast<uint16_t>(add_mod(a, b));
                hi[i] = static_cast<uint16_t>(sub_mod(a, b));
            }
        }
    }
}

void GaloisField::build_logs(unsigned polynomial, const uint16_t* basis) {
    // Discrete logs of the polynomial-basis elements via the LFSR x -> x*2.
    std::vector<uint16_t> poly_log(order_);
    unsigned x = 1;
    for (unsigned e = 0; e < modulus_; ++e) {
        poly_log[x] = static_cast<uint16_t>(e);
        x <<= 1;
        if (x & order_) x ^= polynomial;
    }
    poly_log[0] = static_cast<uint16_t>(modulus_);

    // Element with Cantor-basis coordinate vector c is XOR of the selected basis
    // vectors; Leopard's "log" of c is the discrete log of that element.
    log_of.assign(order_, 0);
    exp_of.assign(order_, 0);
    std::vector<uint16_t> element(order_, 0);
    for (unsigned c = 1; c < order_; ++c) {
        const unsigned low = c & (c - 1);       // c with its lowest set bit cleared
        const unsigned bit = __builtin_ctz(c);  // index of that bit
        element[c] = static_cast<uint16_t>(element[low] ^ basis[bit]);
    }
    for (unsigned c = 0; c < order_; ++c) log_of[c] = poly_log[element[c]];
    for (unsigned c = 0; c < order_; ++c) exp_of[log_of[c]] = static_cast<uint16_t>(c);
    exp_of[modulus_] = exp_of[0];
}

void GaloisField::build_skews() {
    // Skew factors of the novel-basis additive FFT (Lin-Chung-Han eq. 28),
    // generated subspace by subspace as the reference does (LeopardFF8.cpp:496-531).
    skew.assign(modulus_, 0);
    const unsigned levels = bits_ - 1;
    std::vector<unsigned> v(levels);
    for (unsigned i = 0; i < levels; ++i) v[i] = 1u << (i + 1);

    for (unsigned lvl = 0; lvl < levels; ++lvl) {
        const unsigned first = (1u << lvl) - 1;
        skew[first] = 0;
        for (unsigned i = lvl; i < levels; ++i) {
            const unsigned span = 1u << (i + 1);
            for (unsigned j = first; j < span; j += 2u << lvl) skew[j + span] = static_cast<uint16_t>(skew[j] ^ v[i]);
        }
        // normalise the remaining subspace generators by this level's vanishing value
        v[lvl] = modulus_ - log_of[mul_log(v[lvl], log_of[v[lvl] ^ 1u])];
        for (unsigned i = lvl + 1; i < levels; ++i) v[i] = mul_log(v[i], add_mod(log_of[v[i] ^ 1u], v[lvl]));
    }
    for (auto& s : skew) s = log_of[s];

    log_walsh.assign(log_of.begin(), log_of.end());
    log_walsh[0] = 0;
    walsh(log_walsh.data(), order_);
}

const GaloisField& field8() {
    static const GaloisField f(8, 0x11D, kCantor8.data());
    return f;
}

const GaloisField& field16() {
    static const GaloisField f(16, 0x1002D, kCantor16.data());
    return f;
}

namespace {
// Pack 4 or 8 table bytes into little-endian dwords.
inline void pack_bytes(const uint8_t* b, unsigned count, uint32_t* out) {
    for (unsigned d = 0; d < (count + 3) / 4; ++d) {
        uint32_t w = 0;
        for (unsigned k = 0; k < 4 && d * 4 + k < count; ++k) w |= uint32_t(b[d * 4 + k]) << (8 * k);
        out[d] = w;
    }
}
}  // namespace

void build_perm_tables8(const GaloisField& f, std::vector<uint32_t>& out) {
    out.assign(size_t(f.order() + 1) * kTab8Dwords, 0);  // + the all-zero table
    for (unsigned L = 0; L < f.order(); ++L) {
        uint32_t* t = &out[size_t(L) * kTab8Dwords];
        uint8_t b[8];
        for (unsigned e = 0; e < 8; ++e) b[e] = static_cast<uint8_t>(f.mul_log(e, L));
        pack_bytes(b, 8, t + 0);
        for (unsigned e = 0; e < 8; ++e) b[e] = static_cast<uint8_t>(f.mul_log(e << 3, L));
        pack_bytes(b, 8, t + 2);
        for (unsigned e = 0; e < 4; ++e) b[e] = static_cast<uint8_t>(f.mul_log(e << 6, L));
        pack_bytes(b, 4, t + 4);
    }
}

void build_perm_tables16(const GaloisField& f, std::vector<uint32_t>& out) {
    out.assign(size_t(f.order() + 1) * kTab16Dwords, 0);  // + the all-zero table
    // (input shift, entries, destination dword) per chunk, in table order
    struct Chunk { unsigned shift, entries, dst; };
    static const Chunk chunks[6] = {{0, 8, 0}, {3, 8, 4}, {8, 8, 8}, {11, 8, 12}, {6, 4, 16}, {14, 4, 18}};
    for (unsigned L = 0; L < f.order(); ++L) {
        uint32_t* t = &out[size_t(L) * kTab16Dwords];
        for (const Chunk& c : chunks) {
            uint8_t lo[8], hi[8];
            for (unsigned e = 0; e < c.entries; ++e) {
                const unsigned p = f.mul_log(e << c.shift, L);
                lo[e] = static_cast<uint8_t>(p);
                hi[e] = static_cast<uint8_t>(p >> 8);
            }
            const unsigned dw = c.entries / 4;  // 2 for full chunks, 1 for 2-bit chunks
            pack_bytes(lo, c.entries, t + c.dst);
            pack_bytes(hi, c.entries, t + c.dst + dw);
        }
    }
}

void build_skew_tables(const GaloisField& f, const std::vector<uint32_t>& perm_tables, unsigned tab_dwords,
                       unsigned flag_dw, std::vector<uint32_t>& out) {
    out.assign(size_t(f.order()) * tab_dwords, 0);
    for (unsigned i = 0; i < f.modulus(); ++i) {
        uint32_t* e = &out[size_t(i) * tab_dwords];
        const unsigned lm = f.skew[i];
        if (lm == f.modulus()) {
            e[flag_dw] = 1;  // zero skew: XOR only
            continue;
        }
        const uint32_t* t = &perm_tables[size_t(lm) * tab_dwords];
        for (unsigned d = 0; d < flag_dw; ++d) e[d] = t[d];
    }
}

void build_fused_top_tables8(const GaloisField& f, const std::vector<uint32_t>& perm_tables,
                             std::vector<uint32_t>& out) {
    out.assign(size_t(kFused8Entries) * kTab8Dwords, 0);
    auto element = [&](unsigned i) { return f.skew[i] == f.modulus() ? 0u : unsigned(f.exp_of[f.skew[i]]); };
    for (unsigned T = 1; T <= 7; ++T) {
        const unsigned m = 1u << T;
        for (unsigned c = 0; c + 1 < f.order() / m; ++c) {
            const unsigned e = element(m - 1 + c * m + m / 2) ^ element(m / 2 - 1);
            if (e == 0) continue;  // multiply by zero: the all-zero table
            const uint32_t* t = &perm_tables[size_t(f.log_of[e]) * kTab8Dwords];
            std::copy(t, t + kTab8Dwords, &out[(size_t(T - 1) * 256 + c) * kTab8Dwords]);
        }
    }
}

void build_fused_top_logs16(const GaloisField& f, std::vector<uint32_t>& out) {
    out.assign(kFused16Entries, f.order());  // default: the all-zero table
    auto element = [&](unsigned i) { return f.skew[i] == f.modulus() ? 0u : unsigned(f.exp_of[f.skew[i]]); };
    for (unsigned T = 1; T <= 15; ++T) {
        const unsigned m = 1u << T;
        for (unsigned c = 0; c + 1 < f.order() / m; ++c) {
            const unsigned e = element(m - 1 + c * m + m / 2) ^ element(m / 2 - 1);
            out[fused16_base(T) + c] = e == 0 ? f.order() : f.log_of[e];
        }
    }
}

// The high part Q = F_hi (I + D_hi) I_hi of the FF16 decoder transform over the
// tiles of 256 positions (rs_ff16_small.hip), n = 256 * 2^H: the decoder's
// skews (base -1) of the high layers depend on the tile index alone, so Q is
// one 2^H x 2^H matrix over the field, applied to the unit vectors here with
// the reference's butterflies (IFFT_DIT2 / FFT_DIT2, LeopardFF16.cpp:629-705,
// 1083-1159; formal derivative :1738-1758 restricted to the high bits).  It is
// an XOR-convolution, Q[t][t'] = q[t ^ t'], which is checked; returns false
// (and leaves the narrow decoder off) if it were not.
bool build_high_q16(const GaloisField& f, std::vector<uint32_t>& out) {
    out.assign(kHighQ16Entries, kHighQZero);
    const unsigned one = f.exp_of[0];
    for (unsigned H = 1; H <= 3; ++H) {
        const unsigned N = 1u << H;
        std::vector<std::vector<unsigned>> Q(N, std::vector<unsigned>(N, 0));
        for (unsigned tp = 0; tp < N; ++tp) {
            std::vector<unsigned> v(N, 0);
            v[tp] = one;
            auto skew_of = [&](unsigned i, unsigned l) {
                const unsigned p = i << 8;
                return unsigned(f.skew[(((p >> l) | 1u) << l) - 1]);
            };
            for (unsigned b = 0; b < H; ++b) {  // IFFT, high layers bottom-up
                const unsigned d = 1u << b;
                for (unsigned i = 0; i < N; ++i) {
                    if (i & d) continue;
                    const unsigned lm = skew_of(i, 8 + b);
                    v[i + d] ^= v[i];
                    if (lm != f.modulus()) v[i] ^= f.mul_log(v[i + d], lm);
                }
            }
            std::vector<unsigned> o(v);  // formal derivative on the high bits (sources unmodified)
            for (unsigned k = 0; k < N; ++k)
                for (unsigned b = 0; b < H; ++b)
                    if (!((k >> b) & 1u)) o[k] ^= v[k | (1u << b)];
            v = o;
            for (unsigned b = H; b-- > 0;) {  // FFT, high layers top-down
                const unsigned d = 1u << b;
                for (unsigned i = 0; i < N; ++i) {
                    if (i & d) continue;
                    const unsigned lm = skew_of(i, 8 + b);
                    if (lm != f.modulus()) v[i] ^= f.mul_log(v[i + d], lm);
                    v[i + d] ^= v[i];
                }
            }
            for (unsigned t = 0; t < N; ++t) Q[t][tp] = v[t];
        }
        for (unsigned t = 0; t < N; ++t)
            for (unsigned tp = 0; tp < N; ++tp)
                if (Q[t][tp] != Q[t ^ tp][0]) return false;
        for (unsigned k = 0; k < N; ++k) {
            const unsigned q = Q[k][0];
            out[high_q16_base(H) + k] = q == 0 ? kHighQZero : q == one ? kHighQOne : unsigned(f.log_of[q]);
        }
    }
    return true;
}

}  // namespace lamd
