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

// Ablation switches for performance experiments only (tools/ablate.sh builds
// separate libraries with them; the shipped library has LAMD_ABLATE == 0):
// 1 = no butterfly arithmetic, 2 = no LDS transposes, 4 = no piece loads,
// 8 = no piece stores, 16 = fused kernels return at once (launch floor),
// 32 = (unused), 64 = no formal derivative,
// 128 = FF8 decoder: no scale / reveal multiplies, 256 = no table staging.
#ifndef LAMD_ABLATE
#define LAMD_ABLATE 0
#endif
// 1: the library reads the A/B experiment switches (LEO_AMD_FF8_WIDE,
// LEO_AMD_FF8_HALF / SPLIT / INVERT, LEO_AMD_PIPE_MODE) from the environment;
// tools/ builds only.  The shipped library always takes the tested defaults.
#ifndef LAMD_EXPERIMENT_ENV
#define LAMD_EXPERIMENT_ENV 0
#endif
#ifndef LAMD_FF16_PREFETCH
#define LAMD_FF16_PREFETCH 0
#endif
#ifndef LAMD_FF16_INFLIGHT  // GF(2^16) butterflies a wave keeps in flight (scheduling window)
#define LAMD_FF16_INFLIGHT 2
#endif
// 1: every tile exchange and layer takes an opaque copy of the wave index, so
// the per-lane LDS and table addresses derived from it are computed where they
// are used instead of being hoisted and kept live across the transform (for
// kernels whose registers hold more than the tile, e.g. the one-pass decoder's
// accumulators; rs_ff16_one.hip)
#ifndef LAMD_TILE_OPAQUE_W
#define LAMD_TILE_OPAQUE_W 0
#endif
#define LAMD_OPAQUE_W(w)                                        \
    do {                                                        \
        if constexpr (LAMD_TILE_OPAQUE_W) asm volatile("" : "+v"(w)); \
    } while (0)

namespace lamd {

// Native clang vectors, not HIP's uint4/uint2: those are unions wrapped in a
// struct, and a local array of them is not promoted to registers (it lives in
// scratch memory, stored and reloaded around every asm barrier).
using v4u = unsigned __attribute__((ext_vector_type(4)));
using v2u = unsigned __attribute__((ext_vector_type(2)));

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
    static constexpr unsigned kOrder = 256;
    static constexpr int kDw = 1;  // dwords per unit
    static constexpr unsigned kModulus = 255;
    static constexpr unsigned kTabDw = 8;
    static constexpr unsigned kFlagDw = 5;  // skew-indexed tables: 1 = zero skew
    struct Tab {
        uint32_t a0, a1, b0, b1, c0;
    };
    LDEV static Tab tab_at(const uint32_t* p) {
        return Tab{cload(p), cload(p + 1), cload(p + 2), cload(p + 3), cload(p + 4)};
    }
    LDEV static Tab tab(const uint32_t* tabs, unsigned log_m) { return tab_at(tabs + log_m * kTabDw); }
    LDEV static Tab tab_lds(const uint32_t* p) {
        const v4u v = *reinterpret_cast<const v4u*>(p);
        return Tab{v.x, v.y, v.z, v.w, p[4]};
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
    static constexpr unsigned kOrder = 65536;
    static constexpr int kDw = 2;  // [0] low bytes of 4 elements, [1] their high bytes
    static constexpr unsigned kModulus = 65535;
    static constexpr unsigned kTabDw = 24;
    static constexpr unsigned kFlagDw = 20;
    struct Tab {
        uint32_t t[20];
    };
    LDEV static Tab tab_at(const uint32_t* p) {
        Tab r;
#pragma unroll
        for (int i = 0; i < 20; ++i) r.t[i] = cload(p + i);
        return r;
    }
    LDEV static Tab tab(const uint32_t* tabs, unsigned log_m) { return tab_at(tabs + log_m * kTabDw); }
    LDEV static Tab tab_lds(const uint32_t* p) {
        Tab r;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const v4u v = reinterpret_cast<const v4u*>(p)[i];
            r.t[4 * i] = v.x;
            r.t[4 * i + 1] = v.y;
            r.t[4 * i + 2] = v.z;
            r.t[4 * i + 3] = v.w;
        }
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
    // x ^= y * c: the six products of each output byte and x folded by three
    // 3-input XORs (v_bitop3) per output dword.  (v_perm_b32 issues at half the
    // rate of a VOP2 op on gfx950, tools/ubench_isa2.hip: the 12 perms are half
    // of a butterfly's issue time, the selectors and XORs the other half.)
    LDEV static void muladd(uint32_t* x, const uint32_t* y, const Tab& T) {
        const uint32_t lo = y[0], hi = y[1];
        const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
        const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
        const uint32_t* t = T.t;
        x[0] = xor3(x[0], xor3(perm(t[1], t[0], a0), perm(t[5], t[4], a1), perm(t[9], t[8], b0)),
                    xor3(perm(t[13], t[12], b1), perm(t[16], t[16], a2), perm(t[18], t[18], b2)));
        x[1] = xor3(x[1], xor3(perm(t[3], t[2], a0), perm(t[7], t[6], a1), perm(t[11], t[10], b0)),
                    xor3(perm(t[15], t[14], b1), perm(t[17], t[17], a2), perm(t[19], t[19], b2)));
    }
    LDEV static void mul(uint32_t* x, const uint32_t* y, const Tab& t) { prod(y[0], y[1], t, x[0], x[1]); }
    // The six perm selectors of y, for several multiplies of the same y.
    struct Sel {
        uint32_t a0, a1, a2, b0, b1, b2;
    };
    LDEV static Sel sel(const uint32_t* y) {
        const uint32_t lo = y[0], hi = y[1];
        return Sel{lo & 0x07070707u, (lo >> 3) & 0x07070707u, (lo >> 6) & 0x03030303u,
                   hi & 0x07070707u, (hi >> 3) & 0x07070707u, (hi >> 6) & 0x03030303u};
    }
    // x ^= y * c with y's selectors s
    LDEV static void muladd_sel(uint32_t* x, const Sel& s, const Tab& T) {
        const uint32_t* t = T.t;
        x[0] = xor3(x[0], xor3(perm(t[1], t[0], s.a0), perm(t[5], t[4], s.a1), perm(t[9], t[8], s.b0)),
                    xor3(perm(t[13], t[12], s.b1), perm(t[16], t[16], s.a2), perm(t[18], t[18], s.b2)));
        x[1] = xor3(x[1], xor3(perm(t[3], t[2], s.a0), perm(t[7], t[6], s.a1), perm(t[11], t[10], s.b0)),
                    xor3(perm(t[15], t[14], s.b1), perm(t[17], t[17], s.a2), perm(t[19], t[19], s.b2)));
    }
};

// ------------------------------------------------------------ piece maps ---

// Where piece i lives: a pointer table (caller's scattered buffers) or a slab
// (base + i * stride).  `off` is the byte offset of the current column range.
struct PieceMap {
    const uint64_t* table;
    uint8_t* base;
    uint64_t stride;
    uint64_t off;
    // a map known to be a slab (the multi-pass intermediates): no table test
    LDEV uint8_t* slab_ptr(unsigned i) const { return base + uint64_t(i) * stride + off; }
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

// Piece memory is global (HBM): say so, or a pointer chosen at run time
// becomes a flat access, which also counts against lgkmcnt and so makes every
// later scalar-load wait block on the HBM load as well.
#if defined(__HIP_DEVICE_COMPILE__)
template <class V, class P>
LDEV __attribute__((address_space(1))) V* gptr(P* p) {
    return (__attribute__((address_space(1))) V*)(p);
}
#else
template <class V, class P>
LDEV V* gptr(P* p) { return (V*)(p); }
#endif

template <int C>
struct VecT;
template <>
struct VecT<1> { using type = uint32_t; };
template <>
struct VecT<2> { using type = v2u; };
template <>
struct VecT<4> { using type = v4u; };

// Piece loads / stores, plain or nontemporal (nt: streamed past the caches'
// retention).  nt is the default where it was measured faster: the GF(2^8)
// dense tiles (bit-sliced batch +4%, single call 9.9 -> 8.8 us); the GF(2^16)
// passes were equal or slower with it (profiles/r05_v6/ntall_ab.txt), so the
// unit helpers below stay plain unless an experiment build sets LAMD_NT_IO.
#ifndef LAMD_NT_IO
#define LAMD_NT_IO 0
#endif
template <class V, bool kNt = LAMD_NT_IO != 0>
LDEV V gld(const uint8_t* p) {
    if constexpr (kNt) return __builtin_nontemporal_load(gptr<const V>(p));
    else return *gptr<const V>(p);
}
template <class V, bool kNt = LAMD_NT_IO != 0>
LDEV void gst(uint8_t* p, const V& v) {
    if constexpr (kNt) __builtin_nontemporal_store(v, gptr<V>(p));
    else *gptr<V>(p) = v;
}

template <int C>
LDEV void vload(uint32_t* dst, const uint8_t* src) {
    using V = typename VecT<C>::type;
    const V v = gld<V>(src);
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
    gst<V>(dst, v);
}

// One lane's C units of one piece, register layout: for FF8 x[u]; for FF16
// x[2u] = low-byte dword, x[2u+1] = high-byte dword of unit u.
template <class F, int C>
LDEV void load_units(uint32_t* x, const uint8_t* piece, uint64_t q0) {
    if constexpr ((LAMD_ABLATE & 4) != 0) {
        for (int k = 0; k < C * F::kDw; ++k) x[k] = uint32_t(q0) * 2654435761u + uint32_t(uintptr_t(piece));
        return;
    }
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
    if constexpr ((LAMD_ABLATE & 8) != 0) {
        uint32_t acc = 0;
        for (int k = 0; k < C * F::kDw; ++k) acc ^= x[k];
        if (acc == 0x9E3779B9u && q0 == 0x7FFFFFFFull) *reinterpret_cast<uint32_t*>(piece) = acc;  // keep x live
        return;
    }
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

// Butterfly tables of one transform stage.  A stage with skew base `off`
// needs the skew-indexed entries off + cidx for the group indices cidx its tile
// produces (gf_tables.h: build_skew_tables).
//
// LdsSkew8 (FF8, 5-dword tables): the whole 256-entry array is staged once per
// workgroup in LDS (TabStage8, 5 KB) before the first barrier; a stage only
// moves the base.  Tables land in VGPRs (ds_read), so v_perm needs no
// SGPR->VGPR copies and no per-stage refill barrier exists.
//
// GlobalWindow (FF16, 20-dword tables over 65536 entries) reads entries
// straight from the global skew-indexed array through the scalar cache.
// FF8 multiply tables of N entries in LDS, split for a compact footprint (20
// bytes per entry instead of the 32 of the global layout): the four perm dwords
// (a0, a1, b0, b1) of entry i as one 16-byte slot, the fifth (c0) in a second
// array.  Two aligned reads per table (ds_read_b128 + ds_read_b32).
template <unsigned N>
struct LdsTab8 {
    uint32_t* base;
    static constexpr size_t kDwords = 5 * size_t(N);
    LDEV FF8::Tab at(int i) const {
        const v4u v = reinterpret_cast<const v4u*>(base)[i];
        return FF8::Tab{v.x, v.y, v.z, v.w, base[4 * N + i]};
    }
};

struct LdsSkew8 {
    LdsTab8<256> tabs;
    int off = 0;
    LDEV FF8::Tab table(unsigned cidx) const { return tabs.at(off + int(cidx)); }
    LDEV void stage(const uint32_t*, int o) { off = o; }
    // The skew of position j is zero exactly at j = 2^k - 1 (FFTSkew[2^k - 1]
    // = 0, LeopardFF8.cpp:496-538): such a butterfly is the reference's XOR-only
    // form (its multiply-add adds 0).  Wave-uniform.  With skew base -1 (the
    // FFT of every encode, the IFFT of every decode) this is group 0 of every
    // layer: 63 of the 448 butterflies of a 128-point transform.
    LDEV bool zero(unsigned cidx) const {
        const unsigned j = unsigned(off + int(cidx));
        return ((j + 1) & j) == 0;
    }
};
// The same tables with every butterfly multiplied (a zero skew's all-zero
// table adds 0).  The XOR-only shortcut is a wave-uniform branch per group; in
// straight-line tiles (the GF(2^8) dense forms) its two paths cost register
// copies at every merge (~110 v_mov per wave in the 16-pieces-per-lane batch
// tile), more than the multiplies it saves, which are concentrated in the
// waves holding the first positions (the others run every multiply anyway).
struct LdsSkew8NoZero : LdsSkew8 {
    LDEV constexpr bool zero(unsigned) const { return false; }
};
// The dense GF(2^8) tiles (K = R = m, one chunk, PieceSpace{0, 0, 0}): the
// skew base is a compile-time constant, so in the layout that holds the top
// tile bits (kLast: every bit above a layer's bit is a register bit) the skew
// of every butterfly group is known at compile time, and the groups whose skew
// is zero (FFTSkew[2^k - 1] = 0, LeopardFF8.cpp:496-538) compile to the
// reference's XOR-only butterfly with no branch: at skew base -1 that is 7 of
// the 24 multiplies per lane of layers 5, 4, 3 (6 of 16 for layers 4, 5),
// the same in every wave.  In the other layouts a group's skew depends on the
// wave index, so there every butterfly is multiplied (LdsSkew8NoZero).
template <int kOff>
struct LdsSkew8Fixed : LdsSkew8NoZero {
    static constexpr bool kStaticOffset = true;
    static constexpr int kOffset = kOff;
    LDEV FF8::Tab table(unsigned cidx) const { return tabs.at(kOff + int(cidx)); }
};
template <class W, class = void>
struct StaticOffsetOf {
    static constexpr bool value = false;
};
template <class W>
struct StaticOffsetOf<W, std::void_t<decltype(W::kStaticOffset)>> {
    static constexpr bool value = W::kStaticOffset;
};

template <class F>
struct GlobalWindow {
    const uint32_t* sk = nullptr;
    LDEV constexpr bool zero(unsigned) const { return false; }
    LDEV typename F::Tab table(unsigned cidx) const { return F::tab_at(sk + size_t(cidx) * F::kTabDw); }
    LDEV void stage(const uint32_t* sktab, int off) { sk = sktab + ptrdiff_t(off) * ptrdiff_t(F::kTabDw); }
};

// FF16 butterfly tables of one transform stage staged in LDS (Tabs16Stage):
// slot j (1 <= j < 2^T) of a set holds the table of skew position
// base + hi_fixed + (j << l0).  Those are exactly the positions a tile of
// PieceSpace{lo_fixed, l0, hi_fixed} asks for on its layers: for a layer on
// global bit l >= l0, skew_index(i, l) = hi_fixed + (j << l0) with
// j = ((tile piece >> (l - l0)) | 1) << (l - l0).  A table is five
// ds_read_b128 at a wave-uniform address into VGPRs, so v_perm takes both
// table dwords from VGPRs (SGPR tables cost a v_mov per perm pair) and no
// scalar-load round trip sits in front of every butterfly group.
//
// Slot s starts at dword tab16_slot(s): 20 dwords a slot plus 4 dwords of
// padding after every 8th and every 64th slot.  Lane groups that hold
// different pieces (Tile LW < 64) read slots 8, 16, ... or 64, 128, ... apart
// in the same instruction; without the padding those start in the same LDS
// bank (20 * 8 = 160 = 0 mod 32 dwords) and the reads serialise.
__host__ __device__ constexpr unsigned tab16_slot(unsigned s) { return 20u * s + 4u * ((s >> 3) + (s >> 6)); }
constexpr size_t tab16_set_dwords(int T) { return tab16_slot(1u << T); }
struct LdsWindow16 {
    const uint32_t* set;
    unsigned hi_fixed, l0;
    LDEV constexpr bool zero(unsigned) const { return false; }
    LDEV FF16::Tab table(unsigned cidx) const { return FF16::tab_lds(set + tab16_slot((cidx - hi_fixed) >> l0)); }
    LDEV void stage(const uint32_t*, int) {}
};
constexpr size_t kTab16LdsDwords = 20;
// A set staged at skew base kOff with hi_fixed = 0 and l0 = kL0: in the layout
// holding the top tile bits, a group's skew position is known at compile time,
// and the zero-skew groups run the XOR-only butterfly with no branch (as
// LdsSkew8Fixed for GF(2^8)).  At skew base -1 that is group 0 of every layer.
template <int kOff, unsigned kL0>
struct LdsWindow16Static : LdsWindow16 {
    static constexpr bool kStaticOffset = true;
    static constexpr int kOffset = kOff;
    static constexpr unsigned kLowBits = kL0;
};

// Cooperative global -> LDS copy of one set of 2^T FF16 skew tables (see
// LdsWindow16), split like TabStage8: load() issues the global loads (ahead of
// the piece loads), store() writes LDS after the piece loads are in flight.
template <int NT, int T>
struct Tabs16Stage {
    static constexpr unsigned kVec = ((1u << T) - 1) * 5;  // v4u per set (slot 0 unused)
    static constexpr unsigned PER = (kVec + NT - 1) / NT;
    v4u v[PER];
    LDEV void load(const uint32_t* sktab, int base, unsigned hi_fixed, unsigned l0) {
        if constexpr ((LAMD_ABLATE & 256) != 0) return;
        static_for<0, int(PER)>([&](auto I) __attribute__((always_inline)) {
            constexpr unsigned i = decltype(I)::value;
            unsigned e = threadIdx.x + i * NT;
            if constexpr ((i + 1) * NT > kVec) e = e < kVec ? e : kVec - 1;
            const unsigned j = 1 + e / 5, k = e % 5;
            const size_t entry = size_t(int64_t(base) + int64_t(hi_fixed + (j << l0)));
            v[i] = reinterpret_cast<const v4u*>(sktab)[entry * 6 + k];  // 24-dword entries
        });
    }
    LDEV void store(uint32_t* set) const {
        if constexpr ((LAMD_ABLATE & 256) != 0) return;
        static_for<0, int(PER)>([&](auto I) __attribute__((always_inline)) {
            constexpr unsigned i = decltype(I)::value;
            const unsigned e = threadIdx.x + i * NT;
            const unsigned j = 1 + e / 5, k = e % 5;
            if ((i + 1) * NT <= kVec || e < kVec) reinterpret_cast<v4u*>(set)[tab16_slot(j) / 4 + k] = v[i];
        });
    }
};

// Cooperative copy of the FF16 multiply tables of N log values into LDS: slot
// p = the table of log value logs[p] (tab16: 24 dwords per log value; 65536 =
// the all-zero table).  The decoder's per-piece scale and reveal multiplies.
template <int NT, unsigned N>
struct LogTabs16Stage {
    static constexpr unsigned kVec = N * 5;
    static constexpr unsigned PER = (kVec + NT - 1) / NT;
    v4u v[PER];
    LDEV void load(const uint32_t* tabs, const uint32_t* logs) {
        if constexpr ((LAMD_ABLATE & 256) != 0) return;
        static_for<0, int(PER)>([&](auto I) __attribute__((always_inline)) {
            constexpr unsigned i = decltype(I)::value;
            unsigned e = threadIdx.x + i * NT;
            if constexpr ((i + 1) * NT > kVec) e = e < kVec ? e : kVec - 1;
            const unsigned lm = logs[e / 5];
            v[i] = reinterpret_cast<const v4u*>(tabs)[size_t(lm) * 6 + e % 5];
        });
    }
    // slot p (the table of logs[p]) at dword tab16_slot(p), as the skew sets
    LDEV void store(uint32_t* dst) const {
        if constexpr ((LAMD_ABLATE & 256) != 0) return;
        static_for<0, int(PER)>([&](auto I) __attribute__((always_inline)) {
            constexpr unsigned i = decltype(I)::value;
            const unsigned e = threadIdx.x + i * NT;
            if ((i + 1) * NT <= kVec || e < kVec) reinterpret_cast<v4u*>(dst)[tab16_slot(e / 5) / 4 + e % 5] = v[i];
        });
    }
};

// Workgroup-cooperative copy of N global FF8 tables (8-dword entries) into an
// LdsTab8<N>, split so that the global loads are issued first (ahead of the
// piece loads: vmcnt retires in order, so waiting for these does not wait for
// the pieces) and the LDS stores happen after the piece loads are in flight.
template <int NT, unsigned N>
struct TabStage8 {
    static constexpr unsigned PER = (N + NT - 1) / NT;  // entries per thread
    v4u va[PER];
    uint32_t vc[PER];
    LDEV void load(const uint32_t* src) {
        if constexpr ((LAMD_ABLATE & 256) != 0) return;
        static_for<0, int(PER)>([&](auto I) __attribute__((always_inline)) {
            constexpr unsigned i = decltype(I)::value;
            unsigned e = threadIdx.x + i * NT;
            if constexpr ((i + 1) * NT > N) e = e < N ? e : N - 1;  // tail: re-read a valid entry
            va[i] = reinterpret_cast<const v4u*>(src)[2 * e];
            vc[i] = src[8 * e + 4];
        });
    }
    template <unsigned M>
    LDEV void store(LdsTab8<M> dst) const {
        static_assert(M >= N, "destination too small");
        if constexpr ((LAMD_ABLATE & 256) != 0) return;
        static_for<0, int(PER)>([&](auto I) __attribute__((always_inline)) {
            constexpr unsigned i = decltype(I)::value;
            const unsigned e = threadIdx.x + i * NT;
            if ((i + 1) * NT <= N || e < N) {
                reinterpret_cast<v4u*>(dst.base)[e] = va[i];
                dst.base[4 * M + e] = vc[i];
            }
        });
    }
};

// LDS areas used in turn by consecutive tile exchanges (Tile::exchange,
// Tile::derivative_ring).  With two areas an area is rewritten only after the
// barrier of the exchange in between, so an exchange needs one barrier (writes
// -> reads); with one area it also needs one ahead of its writes, but takes
// half the LDS (more workgroups per CU).  The counter is a compile-time
// constant once the transforms are unrolled.
template <size_t kArea, int kAreas>
struct LdsRing {
    static_assert(kAreas == 1 || kAreas == 2, "one or two areas");
    static constexpr bool kPreBarrier = kAreas == 1;
    uint32_t* base;
    unsigned n = 0;
    LDEV uint32_t* next() {
        uint32_t* p = base + (kAreas == 2 ? (n & 1u) * kArea : 0);
        ++n;
        return p;
    }
};

// Global piece index of tile piece tp:  lo_fixed | tp << l0 | hi_fixed.
struct PieceSpace {
    unsigned lo_fixed, l0, hi_fixed;
    LDEV unsigned global(unsigned tp) const { return lo_fixed | (tp << l0) | hi_fixed; }
};

// Pruning predicates.  A butterfly layer on global bit l acts inside aligned
// blocks of 2^(l+1) codeword positions; pred(pos, l + 1) says whether the
// block holding position pos is live.  IFFT: a block with no non-zero input
// stays all-zero, so its butterflies are skipped; FFT: a block holding no
// needed output feeds no needed output, so its butterflies are skipped (the
// reference's FFT_DIT_ErrorBits, LeopardFF8.cpp:1681-1801, generalised to both
// transforms).  Every predicate is wave-uniform (scalar).  The pipelined
// transforms fetch a predicate's raw word with the lookahead of its layer
// (word) and test it when the layer runs (bit).
struct AllLive {
    LDEV constexpr bool operator()(unsigned, unsigned) const { return true; }
    LDEV constexpr uint32_t word(unsigned, unsigned) const { return 1u; }
    LDEV constexpr bool bit(uint32_t, unsigned, unsigned) const { return true; }
};
// Live iff the block starts below `limit` (encoder: inputs [0, K - base),
// outputs [0, R)).
struct BelowLive {
    unsigned limit;
    LDEV bool operator()(unsigned pos, unsigned level) const { return ((pos >> level) << level) < limit; }
    LDEV uint32_t word(unsigned pos, unsigned level) const { return (*this)(pos, level) ? 1u : 0u; }
    LDEV bool bit(uint32_t wd, unsigned, unsigned) const { return wd != 0; }
};
// Occupancy pyramid: level L holds one bit per aligned block of 2^L positions,
// starting at word off(L).  FF8: 256 positions, 20 words, passed by value in
// the kernel arguments.  FF16: 65536 positions in device memory (pyr_offset).
constexpr unsigned pyr8_offset(unsigned L) { return L <= 3 ? 16u - (16u >> L) : 15u + (L - 4); }
constexpr unsigned kPyr8Words = 20;
struct Pyr8Live {
    const uint32_t* w;  // kernel-argument words
    LDEV uint32_t word(unsigned pos, unsigned level) const { return w[pyr8_offset(level) + ((pos >> level) >> 5)]; }
    LDEV bool bit(uint32_t wd, unsigned pos, unsigned level) const { return (wd >> ((pos >> level) & 31)) & 1u; }
    LDEV bool operator()(unsigned pos, unsigned level) const { return bit(word(pos, level), pos, level); }
};

// Skew index of the butterfly on pair (i, i + 2^l), bit l of i clear: the
// group [g, g + 2^(l+1)) containing i uses skew[g + 2^l]   (the layer-by-layer
// form of LeopardFF8.cpp:1111-1114 / 1557-1560).
LDEV unsigned skew_index(unsigned i, unsigned l) { return ((i >> l) | 1u) << l; }

// A tile: 2^T pieces x (64*C) units.  Each lane holds NR = 2^R pieces in
// registers; a "layout" k assigns tile bits [lo(k), lo(k) + R) to the register
// index and the remaining T-R bits, in order, to the wave index (2^(T-R) waves).
// Layouts k = 0 .. NL-1 step upward through the bits (the last one holds the
// top R bits); a butterfly layer on tile bit l runs in a layout holding bit l
// in registers, and an LDS transpose moves the tile between adjacent layouts.
// LW: lanes per tile column strip (64 = a wave per column strip; 32 or 16 when
// the lane groups of a wave hold different pieces: "w" is then the virtual wave
// index (wave and lane group) and "lane" the lane inside its group).
//
// S "split" bits: LDS exchanges (transposes, the formal derivative's wave-bit
// gathers) run in 2^S rounds, one per value of tile bits [T-R, T-R+S), which
// are register bits in both layouts of a two-layout tile; each round moves
// 1/2^S of the tile through an area of 1/2^S the size.  This is what lets two
// GF(2^16) workgroups of 256 pieces share a CU's 160 KiB of LDS, so that one
// workgroup's loads and stores overlap the other's butterflies.
#ifndef LAMD_FF8_KB
#define LAMD_FF8_KB 4  // FF8 butterfly tables read (and live) together per layer batch
#endif
// LGL: the lane group (LW < 64) is the low LGL bits of the virtual wave index
// (0: no lane groups, or lane groups above the wave, as the GF(2^8) encoder's
// lane-group forms).  In a layout whose low lo(k) >= LGL bits come from the
// virtual wave, the lane groups then hold tile bits below every layer of that
// layout, whose butterfly tables are therefore the same for all lane groups:
// they are addressed from the wave-uniform part of the index (scalar address
// arithmetic, no per-lane table addresses kept live).
template <class F, int T, int R, int C, int LW = 64, int S = 0, int LGL = 0>
struct Tile {
    static_assert(R >= 1 && R <= T, "register bits");
    static constexpr int NR = 1 << R;         // pieces per lane
    static constexpr int U = C * F::kDw;      // dwords per piece per lane
    static constexpr int NW = 1 << (T - R);   // waves per workgroup
    static constexpr int NL = (T + R - 1) / R;
    static constexpr int kLast = NL - 1;
    using Reg = uint32_t[NR][U];
    static_assert(S == 0 || (NL == 2 && S <= 2 * R - T), "split bits must be register bits of both layouts");
    static constexpr int kSB = T - R;  // first split bit
    // LDS dwords of one exchange area (a transpose, a derivative gather)
    static constexpr size_t kXchDwords = T > R ? (size_t(1) << (T - S)) * LW * U : 0;
    // area slot of tile piece p: p without its split bits
    LDEV static unsigned compact(unsigned p) {
        if constexpr (S == 0) return p;
        else return (p & ((1u << kSB) - 1)) | ((p >> (kSB + S)) << kSB);
    }
    // split bits of the piece register r holds in layout k (compile time: register bits)
    static constexpr unsigned split_of(int k, int r) {
        return S == 0 ? 0u : (unsigned(r) >> (kSB - (k * R < T - R ? k * R : T - R))) & ((1u << S) - 1);
    }

    static constexpr int lo(int k) { return k * R < T - R ? k * R : T - R; }
    static_assert(S == 0 || split_of(NL - 1, (1 << S) - 1) == (1u << S) - 1, "kLast: split class = low register bits");
    // Layers done in layout k.  FFT: [lo(k), lo(k + 1)) (the last layout up to
    // T), i.e. every layer in the latest layout holding its bit.  IFFT: by
    // default [lo(k - 1) + R, lo(k) + R), every layer in the earliest one; with
    // kLate the FFT's rule, which puts the most layers in the top layout, where
    // a transform at skew base -1 has its zero-skew groups at compile time
    // (LdsSkew8Fixed, LdsWindow16Static; measured: the decoders gain, the
    // encoders' base m - 1 IFFTs lose 2-4% to the other order, r03_v12).
    template <bool kLate>
    static constexpr int ifft_begin(int k) { return kLate ? lo(k) : (k == 0 ? 0 : lo(k - 1) + R); }
    template <bool kLate>
    static constexpr int ifft_end(int k) { return kLate ? (k == NL - 1 ? T : lo(k + 1)) : lo(k) + R; }
    static constexpr int fft_end(int k) { return k == NL - 1 ? T : lo(k + 1); }
    template <class Win>
    static constexpr bool late_ifft() {
        if constexpr (StaticOffsetOf<Win>::value) return Win::kOffset == -1;
        else return false;
    }

    // tile piece held in register r by wave w in layout k
    LDEV static unsigned piece(int k, int r, unsigned w) {
        const int b = lo(k);
        return (w & ((1u << b) - 1)) | (unsigned(r) << b) | ((w >> b) << (b + R));
    }

    LDEV static void zero(Reg& x) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int k = 0; k < U; ++k) x[r][k] = 0;
    }
    // Materialise x here: keeps the compiler from sinking the computation of a
    // register into the (conditional) blocks that consume it, which would keep
    // all of its inputs live until then.
    LDEV static void pin(Reg& x) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int k = 0; k < U; ++k) asm volatile("" : "+v"(x[r][k]));
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
    // win holds the stage's butterfly tables (skew base already applied).
    template <bool kInverse, int LAY, int L, class Win, class Pred>
    LDEV static void layer(Reg& x, unsigned w, const PieceSpace& ps, const Win& win, const Pred& pred) {
        if constexpr ((LAMD_ABLATE & 1) != 0) return;
        LAMD_OPAQUE_W(w);
        constexpr int rb = L - lo(LAY);
        static_assert(rb >= 0 && rb < R, "layer not in this layout");
        constexpr int half = 1 << rb;
        const unsigned gl = ps.l0 + L;
        auto live = [&](int g) { return pred(ps.global(piece(LAY, g, w)), gl + 1); };
        const unsigned wt = [&] {
            if constexpr (LGL > 0 && LGL <= lo(LAY)) return uniform(w);  // lane 0 is lane group 0
            else return w;
        }();
        auto table = [&](int g) {
            // A zero skew has an all-zero table: the multiply-add adds 0, which is
            // the reference's XOR-only butterfly.
            return win.table(skew_index(ps.global(piece(LAY, g, wt)), gl));
        };
        auto zero = [&](int g) { return win.zero(skew_index(ps.global(piece(LAY, g, w)), gl)); };
        // XOR-only butterflies of a zero-skew group (wave-uniform branch): the
        // IFFT's y ^= x; x ^= 0 and the FFT's x ^= 0; y ^= x are both y ^= x.
        auto xor_group = [&](int g) {
#pragma unroll
            for (int j = 0; j < half; ++j)
#pragma unroll
                for (int k = 0; k < U; ++k) x[g + j + half][k] ^= x[g + j][k];
        };
        constexpr int NG = NR / (2 * half);  // groups (distinct skews) per lane in this layer
        auto group = [&](int g, const typename F::Tab& t) {
#pragma unroll
            for (int j = 0; j < half; ++j) {
#pragma unroll
                for (int u = 0; u < C; ++u) {
                    uint32_t* a = &x[g + j][u * F::kDw];
                    uint32_t* b = &x[g + j + half][u * F::kDw];
                    if constexpr (kInverse) {
#pragma unroll
                        for (int k = 0; k < F::kDw; ++k) {
                            b[k] ^= a[k];
                            // Materialise y: otherwise the compiler folds (y ^ x) & mask
                            // into one v_bitop3 (VOP3, ~1.6x the issue cost of the
                            // VOP2 and it replaces; measured 12% per butterfly).
                            if constexpr (F::kDw == 1) asm volatile("" : "+v"(b[k]));
                        }
                        F::muladd(a, b, t);
                    } else {
                        F::muladd(a, b, t);
#pragma unroll
                        for (int k = 0; k < F::kDw; ++k) b[k] ^= a[k];
                    }
                    if constexpr (F::kDw == 2) {
                        // GF(2^16): at most two butterflies in flight (each holds
                        // ~10 temporaries next to a 64-VGPR tile and its table)
#pragma unroll
                        for (int k = 0; k < F::kDw; ++k) asm volatile("" : "+v"(a[k]), "+v"(b[k]));
                        if ((j * C + u) % LAMD_FF16_INFLIGHT == LAMD_FF16_INFLIGHT - 1) __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        };
        if constexpr (F::kDw == 1 && StaticOffsetOf<Win>::value && LAY == kLast) {
            // top layout of a transform at a compile-time skew base: zero-skew
            // groups known at compile time (LdsSkew8Fixed; piece space
            // {0, 0, 0}, wave bits below the layer)
            constexpr int KB = NG < LAMD_FF8_KB ? NG : LAMD_FF8_KB;
            static_for<0, NG / KB>([&](auto BI) {
                constexpr int g0 = decltype(BI)::value * KB;
                typename F::Tab tabs[KB];
                asm volatile("" ::: "memory");
                static_for<0, KB>([&](auto GI) {
                    constexpr int g = (g0 + GI.value) * 2 * half;
                    constexpr unsigned cidx = ((unsigned(g << lo(LAY)) >> L) | 1u) << L;
                    constexpr int j = Win::kOffset + int(cidx);
                    if constexpr (((j + 1) & j) != 0) tabs[GI.value] = win.table(cidx);
                });
                static_for<0, KB>([&](auto GI) {
                    constexpr int g = (g0 + GI.value) * 2 * half;
                    constexpr unsigned cidx = ((unsigned(g << lo(LAY)) >> L) | 1u) << L;
                    constexpr int j = Win::kOffset + int(cidx);
                    if (live(g)) {
                        if constexpr (((j + 1) & j) == 0) xor_group(g);
                        else group(g, tabs[GI.value]);
                    }
                });
                __builtin_amdgcn_sched_barrier(0);
            });
        } else if constexpr (F::kDw == 1) {
            // FF8 (5-dword tables): read every table of the layer, then let the
            // scheduler interleave the layer's independent butterflies (ILP).
            // At most 4 tables (20 VGPRs) live at a time.
            constexpr int KB = NG < LAMD_FF8_KB ? NG : LAMD_FF8_KB;
            static_for<0, NG / KB>([&](auto BI) {
                constexpr int g0 = decltype(BI)::value * KB;
                typename F::Tab tabs[KB];
                // Re-read tables from LDS each time rather than let the compiler
                // keep earlier reads of the same entries live across the transform.
                asm volatile("" ::: "memory");
                static_for<0, KB>([&](auto GI) { tabs[GI.value] = table((g0 + GI.value) * 2 * half); });
                static_for<0, KB>([&](auto GI) {
                    constexpr int g = (g0 + GI.value) * 2 * half;
                    if (live(g)) {
                        if (zero(g)) xor_group(g);
                        else group(g, tabs[GI.value]);
                    }
                });
                __builtin_amdgcn_sched_barrier(0);  // keep the next batch's tables below this one
            });
        } else {
#if LAMD_FF16_PREFETCH
            // FF16: software pipeline, the next group's table read is issued
            // ahead of this group's butterflies (two tables live).
            typename F::Tab next = table(0);
            static_for<0, NG>([&](auto GI) {
                constexpr int g = decltype(GI)::value * 2 * half;
                const typename F::Tab t = next;
                asm volatile("" ::: "memory");
                if constexpr (g + 2 * half < NR) next = table(g + 2 * half);
                __builtin_amdgcn_sched_barrier(0);
                if (live(g)) {
                    group(g, t);
#pragma unroll
                    for (int j = 0; j < 2 * half; ++j)
#pragma unroll
                        for (int k = 0; k < U; ++k) asm volatile("" : "+v"(x[g + j][k]));
                }
                __builtin_amdgcn_sched_barrier(0);
            });
#else
            // FF16 (20-dword tables): one table live at a time, read inside the
            // live branch; the scheduling barrier keeps the compiler from
            // hoisting later groups' table reads (20 VGPRs each) next to a
            // tile that already holds 64.
            static_for<0, NG>([&](auto GI) {
                constexpr int g = decltype(GI)::value * 2 * half;
                asm volatile("" ::: "memory");
                if constexpr (StaticOffsetOf<Win>::value && LAY == kLast) {
                    // LdsWindow16Static: wave bits below the layer, hi_fixed = 0
                    constexpr unsigned cidx = ((unsigned(g << lo(LAY)) >> L) | 1u) << (L + Win::kLowBits);
                    constexpr int j = Win::kOffset + int(cidx);
                    if constexpr (((j + 1) & j) == 0) {
                        if (live(g)) {
                            xor_group(g);
#pragma unroll
                            for (int jj = 0; jj < 2 * half; ++jj)
#pragma unroll
                                for (int k = 0; k < U; ++k) asm volatile("" : "+v"(x[g + jj][k]));
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        return;
                    }
                }
                if (live(g)) {
                    group(g, table(g));
                    // materialise the group's outputs here: otherwise the
                    // arithmetic sinks to its next use and the table stays live
#pragma unroll
                    for (int j = 0; j < 2 * half; ++j)
#pragma unroll
                        for (int k = 0; k < U; ++k) asm volatile("" : "+v"(x[g + j][k]));
                }
                __builtin_amdgcn_sched_barrier(0);
            });
#endif
        }
    }

    // The top IFFT layer of one stage followed by the top FFT layer of the next,
    // on the same pairs (i, i + 2^(T-1)), as one butterfly (layout kLast):
    //   IFFT  y1 = y ^ x, x1 = x ^ c1*y1;  FFT  x2 = x1 ^ c2*y1, y2 = y1 ^ x2
    //   =>    y1 = y ^ x, x2 = x ^ (c1 + c2)*y1, y2 = y1 ^ x2
    // t is the multiply table of the field element c1 + c2 (one group: the top
    // layer has a single skew).  Saves one multiply layer per encode.
    LDEV static void fused_top(Reg& x, const typename F::Tab& t) {
        if constexpr ((LAMD_ABLATE & 1) != 0) return;
        constexpr int half = 1 << (T - 1 - lo(kLast));
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            if (r & half) continue;
#pragma unroll
            for (int u = 0; u < C; ++u) {
                uint32_t* a = &x[r][u * F::kDw];
                uint32_t* b = &x[r + half][u * F::kDw];
#pragma unroll
                for (int k = 0; k < F::kDw; ++k) {
                    b[k] ^= a[k];
                    if constexpr (F::kDw == 1) asm volatile("" : "+v"(b[k]));
                }
                F::muladd(a, b, t);
#pragma unroll
                for (int k = 0; k < F::kDw; ++k) b[k] ^= a[k];
                if constexpr (F::kDw == 2) {  // as in layer(): bounded butterflies in flight
#pragma unroll
                    for (int k = 0; k < F::kDw; ++k) asm volatile("" : "+v"(a[k]), "+v"(b[k]));
                    if ((r * C + u) & 1) __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    }

    // Move the tile from layout FROM to layout TO through LDS (kXchDwords; in
    // 2^S rounds when split).  The rounds read into a second array: a round's
    // TO registers are not the FROM registers written so far (the split bits
    // are different register bits in the two layouts), so reading in place
    // would overwrite values still to be written.  Register allocation turns
    // the copy into renaming: a FROM value dies as it is written, so about one
    // tile stays live.
    template <int FROM, int TO>
    LDEV static void transpose(Reg& x, unsigned w, unsigned lane, uint32_t* lds) {
        if constexpr ((LAMD_ABLATE & 2) != 0) return;
        LAMD_OPAQUE_W(w);
        Reg y;
        static_for<0, (1 << S)>([&](auto Q) {
            constexpr unsigned q = decltype(Q)::value;
            __syncthreads();
            static_for<0, NR>([&](auto RI) {
                constexpr int r = decltype(RI)::value;
                if constexpr (split_of(FROM, r) == q) {
                    uint32_t* p = lds + (size_t(compact(piece(FROM, r, w))) * LW + lane) * U;
#pragma unroll
                    for (int k = 0; k < U; ++k) p[k] = x[r][k];
                }
            });
            __syncthreads();
            static_for<0, NR>([&](auto RI) {
                constexpr int r = decltype(RI)::value;
                if constexpr (split_of(TO, r) == q) {
                    const uint32_t* p = lds + (size_t(compact(piece(TO, r, w))) * LW + lane) * U;
#pragma unroll
                    for (int k = 0; k < U; ++k) y[r][k] = p[k];
                }
            });
        });
        copy(x, y);
    }

    // ------------------------------------------------------------------
    // Pipelined transforms (GF(2^8) kernels: butterfly tables in LDS).
    //  * The tables and predicate words of layer l+1 are read before the
    //    butterflies of layer l, so the LDS / scalar reads overlap butterflies.
    //    After a barrier all waves run in lockstep; reading a layer's tables at
    //    its start stalled every wave on the LDS at once (measured: LDS and
    //    VALU time added up).
    //  * A layer's live-group mask is formed before the next lookahead is
    //    issued: scalar loads return out of order, so a wait on one is a wait on
    //    every outstanding LDS and scalar read (lgkmcnt(0)).
    //  * Exchanges go through an LdsRing (one or two areas).
    static constexpr size_t kAreaDwords = (size_t(1) << T) * LW * U;
    static constexpr int kMaxGroups = NR / 2 > 0 ? NR / 2 : 1;
    struct Look {
        typename F::Tab t[kMaxGroups];
        uint32_t pw[kMaxGroups];
    };

    template <bool kLate>
    static constexpr int ifft_layout(int L) {
        int k = 0;
        while (!(L >= ifft_begin<kLate>(k) && L < ifft_end<kLate>(k))) ++k;
        return k;
    }
    static constexpr int fft_layout(int L) {
        int k = NL - 1;
        while (!(L >= lo(k) && L < fft_end(k))) --k;
        return k;
    }
    static constexpr int groups(int LAY, int L) { return NR / (2 << (L - lo(LAY))); }

    template <int LAY, int L, class Win, class Pred>
    LDEV static void read_look(Look& lk, unsigned w, const PieceSpace& ps, const Win& win, const Pred& pred) {
        constexpr int half = 1 << (L - lo(LAY));
        asm volatile("" ::: "memory");  // keep the reads here (issue point of the lookahead)
        static_for<0, groups(LAY, L)>([&](auto G) {
            constexpr int gi = decltype(G)::value;
            const unsigned pos = ps.global(piece(LAY, gi * 2 * half, w));
            lk.t[gi] = win.table(skew_index(pos, ps.l0 + L));
            lk.pw[gi] = pred.word(pos, ps.l0 + L + 1);
        });
    }
    template <int LAY, int L>
    LDEV static void take_look(Look& cur, const Look& nxt) {
        static_for<0, groups(LAY, L)>([&](auto G) {
            cur.t[decltype(G)::value] = nxt.t[decltype(G)::value];
            cur.pw[decltype(G)::value] = nxt.pw[decltype(G)::value];
        });
    }
    template <int LAY, int L, class Pred>
    LDEV static uint32_t live_mask(const Look& lk, unsigned w, const PieceSpace& ps, const Pred& pred) {
        constexpr int half = 1 << (L - lo(LAY));
        uint32_t mask = 0;
        static_for<0, groups(LAY, L)>([&](auto G) {
            constexpr int gi = decltype(G)::value;
            const unsigned pos = ps.global(piece(LAY, gi * 2 * half, w));
            if (pred.bit(lk.pw[gi], pos, ps.l0 + L + 1)) mask |= 1u << gi;
        });
        asm volatile("" ::"s"(mask));  // formed here, ahead of the next lookahead
        return mask;
    }
    template <bool kInverse, int LAY, int L>
    LDEV static void apply(Reg& x, const Look& lk, uint32_t live) {
        if constexpr ((LAMD_ABLATE & 1) != 0) return;
        constexpr int half = 1 << (L - lo(LAY));
        static_for<0, groups(LAY, L)>([&](auto G) {
            constexpr int gi = decltype(G)::value, g = gi * 2 * half;
            if ((live >> gi) & 1u) {
#pragma unroll
                for (int j = 0; j < half; ++j) {
#pragma unroll
                    for (int u = 0; u < C; ++u) {
                        uint32_t* a = &x[g + j][u * F::kDw];
                        uint32_t* b = &x[g + j + half][u * F::kDw];
                        if constexpr (kInverse) {
#pragma unroll
                            for (int k = 0; k < F::kDw; ++k) {
                                b[k] ^= a[k];
                                if constexpr (F::kDw == 1) asm volatile("" : "+v"(b[k]));
                            }
                            F::muladd(a, b, lk.t[gi]);
                        } else {
                            F::muladd(a, b, lk.t[gi]);
#pragma unroll
                            for (int k = 0; k < F::kDw; ++k) b[k] ^= a[k];
                        }
                    }
                }
            }
        });
    }

    // Transpose from layout FROM to layout TO through the ring's next area.
    template <int FROM, int TO, class Ring>
    LDEV static void exchange(Reg& x, unsigned w, unsigned lane, Ring& ring) {
        static_assert(S == 0, "pipelined exchanges move the whole tile");
        uint32_t* area = ring.next();
        if constexpr ((LAMD_ABLATE & 2) != 0) return;
        if constexpr (Ring::kPreBarrier) __syncthreads();
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            uint32_t* p = area + (size_t(piece(FROM, r, w)) * LW + lane) * U;
#pragma unroll
            for (int k = 0; k < U; ++k) p[k] = x[r][k];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint32_t* p = area + (size_t(piece(TO, r, w)) * LW + lane) * U;
#pragma unroll
            for (int k = 0; k < U; ++k) x[r][k] = p[k];
        }
    }

    template <bool kSkipTop = false, class Ring, class Win, class Pred = AllLive>
    LDEV static void ifft_pl(Reg& x, unsigned w, unsigned lane, Ring& ring, const PieceSpace& ps, const Win& win,
                             const Pred& pred = Pred{}) {
        constexpr int NS = kSkipTop ? T - 1 : T;  // layers computed here
        constexpr bool kL = late_ifft<Win>();
        Look cur, nxt;
        if constexpr (NS > 0) read_look<ifft_layout<kL>(0), 0>(cur, w, ps, win, pred);
        static_for<0, (NS > 0 ? NS : 0)>([&](auto LI) {
            constexpr int L = decltype(LI)::value, k = ifft_layout<kL>(L);
            const uint32_t live = live_mask<k, L>(cur, w, ps, pred);
            if constexpr (L + 1 < NS) read_look<ifft_layout<kL>(L + 1), L + 1>(nxt, w, ps, win, pred);
            apply<true, k, L>(x, cur, live);
            if constexpr (L + 1 < T && ifft_layout<kL>(L + 1) != k) exchange<k, ifft_layout<kL>(L + 1)>(x, w, lane, ring);
            if constexpr (L + 1 < NS) take_look<ifft_layout<kL>(L + 1), L + 1>(cur, nxt);
        });
        if constexpr (NS == 0 && NL > 1) exchange<0, kLast>(x, w, lane, ring);
    }

    template <bool kSkipTop = false, class Ring, class Win, class Pred = AllLive>
    LDEV static void fft_pl(Reg& x, unsigned w, unsigned lane, Ring& ring, const PieceSpace& ps, const Win& win,
                            const Pred& pred = Pred{}) {
        constexpr int top = kSkipTop ? T - 2 : T - 1;  // first layer computed here
        if constexpr (top >= 0) {
            if constexpr (fft_layout(top) != kLast) exchange<kLast, fft_layout(top)>(x, w, lane, ring);
            Look cur, nxt;
            read_look<fft_layout(top), top>(cur, w, ps, win, pred);
            static_for<0, top + 1>([&](auto LI) {
                constexpr int L = top - decltype(LI)::value, k = fft_layout(L);
                const uint32_t live = live_mask<k, L>(cur, w, ps, pred);
                if constexpr (L > 0) read_look<fft_layout(L - 1), L - 1>(nxt, w, ps, win, pred);
                apply<false, k, L>(x, cur, live);
                if constexpr (L > 0 && fft_layout(L - 1) != k) exchange<k, fft_layout(L - 1)>(x, w, lane, ring);
                if constexpr (L > 0) take_look<fft_layout(L - 1), L - 1>(cur, nxt);
            });
            if constexpr (fft_layout(0) != 0) exchange<fft_layout(0), 0>(x, w, lane, ring);
        } else if constexpr (NL > 1) {
            exchange<kLast, 0>(x, w, lane, ring);
        }
    }

    // IFFT over all tile bits: starts in layout 0, ends in layout kLast.
    // kSkipTop: leave out the layer on the top tile bit (fused_top does it).
    template <bool kSkipTop = false, class Win, class Pred = AllLive>
    LDEV static void ifft(Reg& x, unsigned w, unsigned lane, uint32_t* lds, const PieceSpace& ps, const Win& win,
                          const Pred& pred = Pred{}) {
        static_for<0, NL>([&](auto K) {
            constexpr int k = decltype(K)::value;
            constexpr bool kL = late_ifft<Win>();
            constexpr int end = (kSkipTop && k == NL - 1) ? T - 1 : ifft_end<kL>(k);
            static_for<ifft_begin<kL>(k), end>(
                [&](auto L) { layer<true, k, decltype(L)::value>(x, w, ps, win, pred); });
            if constexpr (k + 1 < NL) transpose<k, k + 1>(x, w, lane, lds);
        });
    }

    // FFT over all tile bits: starts in layout kLast, ends in layout 0.
    template <bool kSkipTop = false, class Win, class Pred = AllLive>
    LDEV static void fft(Reg& x, unsigned w, unsigned lane, uint32_t* lds, const PieceSpace& ps, const Win& win,
                         const Pred& pred = Pred{}) {
        static_for<0, NL>([&](auto KI) {
            constexpr int k = NL - 1 - decltype(KI)::value;
            constexpr int end = (kSkipTop && k == NL - 1) ? T - 1 : fft_end(k);
            static_for<lo(k), end>([&](auto LI) {
                constexpr int L = end - 1 - (decltype(LI)::value - lo(k));
                layer<false, k, L>(x, w, ps, win, pred);
            });
            if constexpr (k > 0) transpose<k, k - 1>(x, w, lane, lds);
        });
    }

    // The decoder's top IFFT layer, the formal derivative and the top FFT
    // layer collapse: both top layers use the same skew c (offset -1, group 0),
    // so with (x, y) a pair across the top bit, F_top (I + D_top) I_top maps
    // (x, y) -> (y, x) (the multiplies cancel: y1 = x ^ y, x1 = x ^ c*y1,
    // x2 = x1 ^ y1, x3 = x2 ^ c*y1 = y, y3 = y1 ^ x3 = x), F_top I_top = I, and
    // the lower-bit terms D_low commute with the single-skew top layers:
    //   F (I + D) I = F_low (swap_top + D_low) I_low.
    // This computes v <- swap_top(v) + D_low(v) in layout kLast after an IFFT
    // without its top layer; the FFT then skips its top layer as well.
    // `area`: LDS for the wave-bit terms; pre_barrier: wait for earlier reads.
    // In place, with the exchange split into rounds: round q handles the
    // registers of split class q (ascending q, ascending r inside a class, the
    // pairs (r, r + H) across the top bit together), so every register a term
    // reads is still unmodified: the register terms of class q read classes
    // >= q and higher registers of its own class; the wave-bit terms read the
    // partner waves' originals that round q published in LDS first.
    LDEV static void derivative_swaptop(Reg& v, unsigned w, unsigned lane, uint32_t* area, bool pre_barrier) {
        if constexpr ((LAMD_ABLATE & 64) != 0) return;
        constexpr int H = NR / 2;  // register bit of the top tile bit (kLast holds the top R bits)
        static_for<0, (1 << S)>([&](auto Q) {
            constexpr unsigned q = decltype(Q)::value;
            if constexpr (T > R) {
                if (pre_barrier || q > 0) __syncthreads();
                static_for<0, NR>([&](auto RI) {
                    constexpr int r = decltype(RI)::value;
                    if constexpr (split_of(kLast, r) == q) {
                        uint32_t* p = area + (size_t(compact(piece(kLast, r, w))) * LW + lane) * U;
#pragma unroll
                        for (int k = 0; k < U; ++k) p[k] = v[r][k];
                    }
                });
                __syncthreads();
            }
            static_for<0, H>([&](auto RI) {
                constexpr int r = decltype(RI)::value;
                if constexpr (split_of(kLast, r) == q) {
                    uint32_t lo[U], hi[U];
#pragma unroll
                    for (int k = 0; k < U; ++k) {
                        lo[k] = v[r + H][k];
                        hi[k] = v[r][k];
                    }
#pragma unroll
                    for (int b = 0; b + 1 < R; ++b)
                        if (!(r & (1 << b)))
#pragma unroll
                            for (int k = 0; k < U; ++k) {
                                lo[k] ^= v[r | (1 << b)][k];
                                hi[k] ^= v[(r + H) | (1 << b)][k];
                            }
#pragma unroll
                    for (int k = 0; k < U; ++k) {
                        v[r][k] = lo[k];
                        v[r + H][k] = hi[k];
                    }
                }
            });
            if constexpr (T > R) {
                for (int b = 0; b < T - R; ++b) {
                    if (w & (1u << b)) continue;  // wave-uniform
                    const unsigned w2 = w | (1u << b);
                    static_for<0, NR>([&](auto RI) {
                        constexpr int r = decltype(RI)::value;
                        if constexpr (split_of(kLast, r) == q) {
                            const uint32_t* p = area + (size_t(compact(piece(kLast, r, w2))) * LW + lane) * U;
#pragma unroll
                            for (int k = 0; k < U; ++k) v[r][k] ^= p[k];
                        }
                    });
                }
            }
        });
    }

    // d += sum over tile bits b with bit b of k clear of v[k | 2^b]   (layout kLast,
    // whose registers hold the top R bits and whose wave index is bits [0, T-R)).
    // This is the tile's share of Leopard's formal derivative (closed form of
    // the loop at LeopardFF8.cpp:1890-1899: every source is read before it is
    // modified, so out[k] = v[k] ^ XOR_{b: k_b = 0} v[k | 2^b]).  v is not held
    // as a tile: load(r, out) fetches register r of it, one split class at a
    // time (8 pieces a round at S = 2), so d plus one class fits the VGPR budget.
    template <class LoadFn>
    LDEV static void derivative_add(Reg& d, LoadFn load, unsigned w, unsigned lane, uint32_t* lds) {
        constexpr int NB = NR >> S;  // registers per class: class q = {r : r & (2^S - 1) = q}
        static_for<0, (1 << S)>([&](auto Q) {
            constexpr unsigned q = decltype(Q)::value;
            uint32_t v[NB][U];
            static_for<0, NB>([&](auto I) { load(int(I.value << S | q), v[I.value]); });
            // register terms: v[r'] feeds d[r' - 2^b] for every register bit b set in r'
            static_for<0, NB>([&](auto I) {
                constexpr int rs = int(I.value << S | q);
#pragma unroll
                for (int b = 0; b < R; ++b)
                    if (rs & (1 << b))
#pragma unroll
                        for (int k = 0; k < U; ++k) d[rs ^ (1 << b)][k] ^= v[I.value][k];
            });
            if constexpr (T > R) {
                __syncthreads();
                static_for<0, NB>([&](auto I) {
                    constexpr int r = int(I.value << S | q);
                    uint32_t* p = lds + (size_t(compact(piece(kLast, r, w))) * LW + lane) * U;
#pragma unroll
                    for (int k = 0; k < U; ++k) p[k] = v[I.value][k];
                });
                __syncthreads();
                for (int b = 0; b < T - R; ++b) {
                    if (w & (1u << b)) continue;  // wave-uniform
                    const unsigned w2 = w | (1u << b);
                    static_for<0, NB>([&](auto I) {
                        constexpr int r = int(I.value << S | q);
                        const uint32_t* p = lds + (size_t(compact(piece(kLast, r, w2))) * LW + lane) * U;
#pragma unroll
                        for (int k = 0; k < U; ++k) d[r][k] ^= p[k];
                    });
                }
            }
        });
    }
};

}  // namespace lamd
