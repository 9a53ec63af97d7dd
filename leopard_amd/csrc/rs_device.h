// rs_device.h -- CDNA4 (gfx950) device building blocks of the Reed-Solomon engine.
//
// Data model (reference: SURVEY.md section 0; LeopardFF8.cpp / LeopardFF16.cpp):
//   * every operation acts column-wise: byte j of piece i only meets byte j of
//     other pieces (FF8), or the ALTMAP pair (j, j+32) of a 64-byte block (FF16,
//     LeopardFF16.cpp:315-332);
//   * a "unit" is what one lane holds of one piece per column step: FF8 = one
//     dword (4 elements), FF16 = one dword of low bytes + the matching dword of
//     high bytes 32 bytes further (4 elements);
//   * a lane owns C consecutive units of every piece of its tile (so one piece
//     is one dwordxC load per lane, 256*C contiguous bytes per wave for FF8);
//   * a workgroup owns a tile of 2^T pieces x (64*C) units; the FFT across the
//     pieces runs in registers, 2^(T-H) pieces per lane, with one LDS transpose
//     between the low and the high layer group (2^H waves per workgroup).
//
// GF multiply by a constant: x*c is GF(2)-linear in x, so the input byte is cut
// into 3+3+2-bit chunks and each chunk's contribution is looked up with one
// v_perm_b32 (8-entry byte table held in two dwords).  Tables are per log value
// (gf_tables.h) and are wave-uniform, so they arrive through the scalar cache.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

#define LDEV __device__ __forceinline__

namespace lamd {

LDEV uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
LDEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
LDEV unsigned uniform(unsigned v) { return __builtin_amdgcn_readfirstlane(v); }

// Load through the constant address space: the data (tables, skews, error
// locator, pointer tables) is read-only for the kernel's lifetime, so with a
// wave-uniform address this becomes an s_load into SGPRs via the scalar cache.
LDEV uint32_t cload(const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) uint32_t*)(p);
#else
    return *p;
#endif
}
LDEV uint64_t cload64(const uint64_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) uint64_t*)(p);
#else
    return *p;
#endif
}

template <int B, int E, class Fn>
__host__ __device__ __forceinline__ void static_for(Fn&& fn) {
    if constexpr (B < E) {
        fn(std::integral_constant<int, B>{});
        static_for<B + 1, E>(fn);
    }
}

// ----------------------------------------------------------------- fields ---

struct FF8 {
    static constexpr int kBits = 8;
    static constexpr int kDw = 1;  // dwords per unit
    static constexpr unsigned kModulus = 255;
    static constexpr unsigned kTabDw = 8;
    struct Tab {
        uint32_t a0, a1, b0, b1, c0;
    };
    LDEV static Tab tab(const uint32_t* tabs, unsigned log_m) {
        const uint32_t* p = tabs + log_m * kTabDw;
        return Tab{cload(p), cload(p + 1), cload(p + 2), cload(p + 3), cload(p + 4)};
    }
    LDEV static uint32_t prod(uint32_t y, const Tab& t) {
        const uint32_t s0 = y & 0x07070707u;
        const uint32_t s1 = (y >> 3) & 0x07070707u;
        const uint32_t s2 = (y >> 6) & 0x03030303u;
        return xor3(perm(t.a1, t.a0, s0), perm(t.b1, t.b0, s1), perm(t.c0, t.c0, s2));
    }
    // x ^= y * c
    LDEV static void muladd(uint32_t* x, const uint32_t* y, const Tab& t) {
        const uint32_t s0 = y[0] & 0x07070707u;
        const uint32_t s1 = (y[0] >> 3) & 0x07070707u;
        const uint32_t s2 = (y[0] >> 6) & 0x03030303u;
        x[0] = xor3(x[0], perm(t.a1, t.a0, s0), perm(t.b1, t.b0, s1)) ^ perm(t.c0, t.c0, s2);
    }
    LDEV static void mul(uint32_t* x, const uint32_t* y, const Tab& t) { x[0] = prod(y[0], t); }
};

struct FF16 {
    static constexpr int kBits = 16;
    static constexpr int kDw = 2;  // [0] low bytes of 4 elements, [1] their high bytes
    static constexpr unsigned kModulus = 65535;
    static constexpr unsigned kTabDw = 24;
    struct Tab {
        uint32_t t[20];
    };
    LDEV static Tab tab(const uint32_t* tabs, unsigned log_m) {
        const uint32_t* p = tabs + log_m * kTabDw;
        Tab r;
#pragma unroll
        for (int i = 0; i < 20; ++i) r.t[i] = cload(p + i);
        return r;
    }
    // (pl, ph) = (lo, hi) * c, see gf_tables.h for the table layout
    LDEV static void prod(uint32_t lo, uint32_t hi, const Tab& T, uint32_t& pl, uint32_t& ph) {
        const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
        const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
        const uint32_t* t = T.t;
        pl = xor3(perm(t[1], t[0], a0), perm(t[5], t[4], a1), perm(t[9], t[8], b0));
        pl = xor3(pl, perm(t[13], t[12], b1), perm(t[16], t[16], a2)) ^ perm(t[18], t[18], b2);
        ph = xor3(perm(t[3], t[2], a0), perm(t[7], t[6], a1), perm(t[11], t[10], b0));
        ph = xor3(ph, perm(t[15], t[14], b1), perm(t[17], t[17], a2)) ^ perm(t[19], t[19], b2);
    }
    LDEV static void muladd(uint32_t* x, const uint32_t* y, const Tab& t) {
        uint32_t pl, ph;
        prod(y[0], y[1], t, pl, ph);
        x[0] ^= pl;
        x[1] ^= ph;
    }
    LDEV static void mul(uint32_t* x, const uint32_t* y, const Tab& t) { prod(y[0], y[1], t, x[0], x[1]); }
};

// ------------------------------------------------------------ piece maps ---

// Where piece i lives: a pointer table (caller's scattered buffers) or a slab
// (base + i * stride).  `off` is the byte offset of the current column range.
struct PieceMap {
    const uint64_t* table;
    uint8_t* base;
    uint64_t stride;
    uint64_t off;
    LDEV uint8_t* ptr(unsigned i) const {
        uint8_t* p = table ? reinterpret_cast<uint8_t*>(cload64(table + i)) : base + uint64_t(i) * stride;
        return p + off;
    }
};

// Byte offset of unit q inside a piece.
template <class F>
LDEV uint64_t unit_offset(uint64_t q) {
    if constexpr (F::kDw == 1) return q * 4;
    else return (q >> 3) * 64 + (q & 7) * 4;
}

template <int C>
struct VecT;
template <>
struct VecT<1> { using type = uint32_t; };
template <>
struct VecT<2> { using type = uint2; };
template <>
struct VecT<4> { using type = uint4; };

template <int C>
LDEV void vload(uint32_t* dst, const uint8_t* src) {
    using V = typename VecT<C>::type;
    const V v = *reinterpret_cast<const V*>(src);
    if constexpr (C == 1) dst[0] = v;
    else if constexpr (C == 2) { dst[0] = v.x; dst[1] = v.y; }
    else { dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w; }
}
template <int C>
LDEV void vstore(uint8_t* dst, const uint32_t* src) {
    using V = typename VecT<C>::type;
    V v;
    if constexpr (C == 1) v = src[0];
    else if constexpr (C == 2) { v.x = src[0]; v.y = src[1]; }
    else { v.x = src[0]; v.y = src[1]; v.z = src[2]; v.w = src[3]; }
    *reinterpret_cast<V*>(dst) = v;
}

// One lane's C units of one piece, register layout: for FF8 x[u]; for FF16
// x[2u] = low-byte dword, x[2u+1] = high-byte dword of unit u.
template <class F, int C>
LDEV void load_units(uint32_t* x, const uint8_t* piece, uint64_t q0) {
    if constexpr (F::kDw == 1) {
        vload<C>(x, piece + q0 * 4);
    } else {
        const uint8_t* p = piece + unit_offset<F>(q0);
        uint32_t lo[C], hi[C];
        vload<C>(lo, p);
        vload<C>(hi, p + 32);
#pragma unroll
        for (int u = 0; u < C; ++u) { x[2 * u] = lo[u]; x[2 * u + 1] = hi[u]; }
    }
}
template <class F, int C>
LDEV void store_units(uint8_t* piece, uint64_t q0, const uint32_t* x) {
    if constexpr (F::kDw == 1) {
        vstore<C>(piece + q0 * 4, x);
    } else {
        uint8_t* p = piece + unit_offset<F>(q0);
        uint32_t lo[C], hi[C];
#pragma unroll
        for (int u = 0; u < C; ++u) { lo[u] = x[2 * u]; hi[u] = x[2 * u + 1]; }
        vstore<C>(p, lo);
        vstore<C>(p + 32, hi);
    }
}

// ------------------------------------------------------------- tile engine --

// Global piece index of tile piece tp:  lo_fixed | tp << l0 | hi_fixed.
struct PieceSpace {
    unsigned lo_fixed, l0, hi_fixed;
    LDEV unsigned global(unsigned tp) const { return lo_fixed | (tp << l0) | hi_fixed; }
};

// Skew index of the butterfly on pair (i, i + 2^l), bit l of i clear: the
// group [g, g + 2^(l+1)) containing i uses skew[g + 2^l]   (the layer-by-layer
// form of LeopardFF8.cpp:1111-1114 / 1557-1560).
LDEV unsigned skew_index(unsigned i, unsigned l) { return ((i >> l) | 1u) << l; }

template <class F, int T, int H, int C>
struct Tile {
    static_assert(T - H >= H, "high layout needs T-H >= H");
    static constexpr int NR = 1 << (T - H);  // pieces per lane
    static constexpr int U = C * F::kDw;      // dwords per piece per lane
    static constexpr int NW = 1 << H;         // waves per workgroup
    using Reg = uint32_t[NR][U];

    // tile piece held in register r by wave w.  Layout 0: register index =
    // tile bits [0, T-H); layout 1: register index = tile bits [H, T).
    LDEV static unsigned piece(int lay, int r, unsigned w) {
        return lay == 0 ? (unsigned(r) | (w << (T - H))) : (w | (unsigned(r) << H));
    }

    LDEV static void zero(Reg& x) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int k = 0; k < U; ++k) x[r][k] = 0;
    }
    LDEV static void xor_into(Reg& x, const Reg& y) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int k = 0; k < U; ++k) x[r][k] ^= y[r][k];
    }
    LDEV static void copy(Reg& x, const Reg& y) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int k = 0; k < U; ++k) x[r][k] = y[r][k];
    }

    // One butterfly layer on tile bit L (compile time) in layout LAY.
    //   IFFT (LeopardFF8.cpp:595-666):  y ^= x; x ^= y * skew   (skipped if skew is 0)
    //   FFT  (LeopardFF8.cpp:1319-1390): x ^= y * skew; y ^= x
    template <bool kInverse, int LAY, int L>
    LDEV static void layer(Reg& x, unsigned w, const PieceSpace& ps, const uint32_t* __restrict__ skew,
                           const uint32_t* __restrict__ tabs) {
        constexpr int rb = LAY == 0 ? L : L - H;
        static_assert(rb >= 0 && rb < T - H, "layer not in this layout");
        constexpr int half = 1 << rb;
        const unsigned gl = ps.l0 + L;
#pragma unroll
        for (int g = 0; g < NR; g += 2 * half) {
            const unsigned gp = ps.global(piece(LAY, g, w));
            const unsigned lm = cload(skew + skew_index(gp, gl));
            if (lm != F::kModulus) {
                const typename F::Tab t = F::tab(tabs, lm);
#pragma unroll
                for (int j = 0; j < half; ++j) {
#pragma unroll
                    for (int u = 0; u < C; ++u) {
                        uint32_t* a = &x[g + j][u * F::kDw];
                        uint32_t* b = &x[g + j + half][u * F::kDw];
                        if constexpr (kInverse) {
#pragma unroll
                            for (int k = 0; k < F::kDw; ++k) b[k] ^= a[k];
                            F::muladd(a, b, t);
                        } else {
                            F::muladd(a, b, t);
#pragma unroll
                            for (int k = 0; k < F::kDw; ++k) b[k] ^= a[k];
                        }
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < half; ++j)
#pragma unroll
                    for (int k = 0; k < U; ++k) x[g + j + half][k] ^= x[g + j][k];
            }
        }
    }

    // Move the tile between layouts through LDS (lds: 2^T * 64 * U dwords).
    template <int FROM>
    LDEV static void transpose(Reg& x, unsigned w, unsigned lane, uint32_t* lds) {
        if constexpr (H > 0) {
            __syncthreads();
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                uint32_t* p = lds + (size_t(piece(FROM, r, w)) * 64 + lane) * U;
#pragma unroll
                for (int k = 0; k < U; ++k) p[k] = x[r][k];
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const uint32_t* p = lds + (size_t(piece(1 - FROM, r, w)) * 64 + lane) * U;
#pragma unroll
                for (int k = 0; k < U; ++k) x[r][k] = p[k];
            }
        }
    }

    // IFFT over all tile bits: starts in layout 0, ends in layout 1.
    LDEV static void ifft(Reg& x, unsigned w, unsigned lane, uint32_t* lds, const PieceSpace& ps,
                          const uint32_t* skew, const uint32_t* tabs) {
        static_for<0, T - H>([&](auto L) { layer<true, 0, decltype(L)::value>(x, w, ps, skew, tabs); });
        transpose<0>(x, w, lane, lds);
        static_for<T - H, T>([&](auto L) { layer<true, 1, decltype(L)::value>(x, w, ps, skew, tabs); });
    }

    // FFT over all tile bits: starts in layout 1, ends in layout 0.
    LDEV static void fft(Reg& x, unsigned w, unsigned lane, uint32_t* lds, const PieceSpace& ps,
                         const uint32_t* skew, const uint32_t* tabs) {
        static_for<0, H>([&](auto I) { layer<false, 1, T - 1 - decltype(I)::value>(x, w, ps, skew, tabs); });
        transpose<1>(x, w, lane, lds);
        static_for<0, T - H>([&](auto I) { layer<false, 0, T - H - 1 - decltype(I)::value>(x, w, ps, skew, tabs); });
    }

    // d += sum over tile bits b with bit b of k clear of v[k | 2^b]   (layout 1).
    // This is the tile's share of Leopard's formal derivative; with d = v it is
    // the whole derivative of a transform that fits the tile (closed form of
    // the loop at LeopardFF8.cpp:1890-1899: every source is read before it is
    // modified, so out[k] = v[k] ^ XOR_{b: k_b = 0} v[k | 2^b]).
    LDEV static void derivative_add(Reg& d, const Reg& v, unsigned w, unsigned lane, uint32_t* lds) {
        // register bits (tile bits H .. T-1)
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int b = 0; b < T - H; ++b)
                if (!(r & (1 << b)))
#pragma unroll
                    for (int k = 0; k < U; ++k) d[r][k] ^= v[r | (1 << b)][k];
        // wave bits (tile bits 0 .. H-1) through LDS
        if constexpr (H > 0) {
            __syncthreads();
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                uint32_t* p = lds + (size_t(piece(1, r, w)) * 64 + lane) * U;
#pragma unroll
                for (int k = 0; k < U; ++k) p[k] = v[r][k];
            }
            __syncthreads();
            for (int b = 0; b < H; ++b) {
                if (w & (1u << b)) continue;  // wave-uniform
                const unsigned w2 = w | (1u << b);
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const uint32_t* p = lds + (size_t(piece(1, r, w2)) * 64 + lane) * U;
#pragma unroll
                    for (int k = 0; k < U; ++k) d[r][k] ^= p[k];
                }
            }
        }
    }
};

}  // namespace lamd
