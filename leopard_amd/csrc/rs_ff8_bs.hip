// rs_ff8_bs.hip -- bit-sliced GF(2^8) dense tile for gfx950: batches of K = R = m = 128
// codes (the benchmark's 128 + 128 shape), encode and full-loss decode.
//
// Reference path: ReedSolomonEncode (LeopardFF8.cpp:1602-1672) with one chunk,
//   out = FFT_{-1}( IFFT_{m-1}(data) )            (IFFT_DIT / FFT_DIT, :595-666, :1319-1390)
// and its inverse for a full-loss decode of such a code (rs_ff8.hip:
// launch_ff8_decode_full), data = FFT_{m-1}( IFFT_{-1}(recovery) ).
//
// Why bit slices.  In the byte layout of rs_ff8.hip a multiply by a constant c
// costs 3 v_perm_b32 + 5 selector ops + 2 XORs per 4 elements, and the tile is
// bound by VALU issue.  Here a lane holds 32 elements of
// a piece as 8 bit planes (plane k = bit k of 32 elements), so x ^= c * y is
// the 8 x 8 GF(2) matrix of c applied to the planes: plane i of x takes the XOR
// of the planes j of y that row i selects.  Every skew of the dense tile is
// known at compile time (gf8_const.h), so most butterflies compile to a fixed
// XOR network (~4x cheaper than the byte form, tools/ubench_bitslice8.hip).
//
// Tile: ONE wave owns the whole 128-piece transform over a 256-byte column
// strip of every piece.  Lane = 8 * g + l: lane group g (8 groups), lane l of
// the group holds bytes [16 l, 16 l + 16) and [128 + 16 l, 128 + 16 l + 16) of
// the strip (32 elements = 8 dwords -> 8 planes) of 16 pieces:
//   layout 0   (load, IFFT layers 0-2, FFT layers 2-0, store): register r holds
//              piece r | g << 4 (piece bits 0-3 in registers, bits 4-6 = g);
//   layout top (IFFT layers 3-5, fused top layer 6, FFT layers 5-3): register r
//              holds piece g | r << 3 (bits 3-6 in registers, bits 0-2 = g).
// A layer-l butterfly group's skew depends on the piece bits above l only
// (skew index ((i >> l) | 1) << l).  In layout top those are register bits:
// every multiplier is a compile-time constant.  In layout 0 the bits 4-6 come
// from the lane group; the skews are affine in those bits (FFTInitialize builds
// FFTSkew[first + k * 2^(l+1)] as the XOR of one generator per bit of k,
// LeopardFF8.cpp:505-514; checked by static_assert below), so
//   c(g) * y = A * y  ^  sum over bits b of g of  (g_b ? H_b * y : 0)
// with A and H_b compile time and the selection by per-lane masks (v_bitop3).
// The two layouts are exchanged through a wave-private LDS area (no barrier:
// one wave's LDS operations execute in order).  No tables, no workgroup
// barriers: waves are independent, several per SIMD.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "gf8_const.h"
#include "rs_args.h"

namespace lamd {

namespace {

#ifndef LAMD_BS_WAVES
#define LAMD_BS_WAVES 4  // independent tiles (waves) per workgroup
#endif
#ifndef LAMD_BS_OCC
#define LAMD_BS_OCC 2  // waves per SIMD the register budget is sized for
#endif
constexpr int kBsWaves = LAMD_BS_WAVES;
constexpr unsigned kBsBlocksPerCu = 4 * LAMD_BS_OCC / kBsWaves;  // workgroups per CU (LAMD_BS_OCC waves per SIMD)
constexpr unsigned kBsStrip = 256;           // bytes of every piece per wave
constexpr unsigned kBsAreaDw = (128 + 8) * 8 * 2;  // LDS dwords per wave: 136 rows x 8 lanes x 2 planes
#ifndef LAMD_BS_SCHED
#define LAMD_BS_SCHED 1  // 1: a scheduling barrier after every butterfly (bounds the temporaries in flight)
#endif
LDEV void bs_fence() {
    if constexpr (LAMD_BS_SCHED) __builtin_amdgcn_sched_barrier(0);
}
#ifndef LAMD_BS_XFENCE
#define LAMD_BS_XFENCE 1  // transposes between scheduling barriers
#endif
#ifndef LAMD_BS_BFENCE
#define LAMD_BS_BFENCE 1  // butterflies between scheduling barriers
#endif
template <int N>
LDEV void bs_fence_every(int i) {
    if ((i + 1) % N == 0) bs_fence();
}

// ---------------------------------------------------------- bit planes -----

// v_bitop3_b32 truth tables: index = 4 * src0 + 2 * src1 + src2
LDEV uint32_t sel_b(uint32_t a, uint32_t b, uint32_t m) { return __builtin_amdgcn_bitop3_b32(a, b, m, 0xD8); }  // m ? b : a
LDEV uint32_t xor_and(uint32_t a, uint32_t b, uint32_t m) { return __builtin_amdgcn_bitop3_b32(a, b, m, 0x78); }  // a ^ (b & m)

// The transpose's three bit masks in VGPRs: v_bitop3_b32 with an SGPR (or
// literal) operand issues at ~4.2 cycles a wave64 instruction against ~2.5
// with three VGPRs (tools/ubench_issue.hip).
struct XMasks {
    uint32_t m4, m2, m1;
    LDEV XMasks() : m4(0x0F0F0F0Fu), m2(0x33333333u), m1(0x55555555u) {
        asm volatile("" : "+v"(m4), "+v"(m2), "+v"(m1));
    }
};
// Delta-swap stage S on register pairs (lo[i], hi[i]), i = 0, 1, 2, 3: the
// MASK << S bits of lo[i] are exchanged with the MASK bits of hi[i]:
//   lo' = MASK ? lo : hi << S,   hi' = MASK ? lo >> S : hi.
// The shifts run as 64-bit shifts of register pairs (hi[0], hi[1]) and
// (lo[0], lo[1]) (a shift costs ~4 cycles a wave64 instruction whatever its
// width): the bits one dword's shift carries into its neighbour land only where
// the select takes the other operand (MASK has its top S bits clear and MASK << S
// its low S bits).
template <int S>
LDEV void dstage(uint32_t* const (&lo)[4], uint32_t* const (&hi)[4], uint32_t mask) {
    uint32_t hs[4], ls[4];
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
        // raw 64-bit shifts (the compiler would keep the carried bits exact
        // with v_alignbit / v_or pairs)
        v2u h0, l0, h, l;
        h0.x = *hi[i], h0.y = *hi[i + 1];
        l0.x = *lo[i], l0.y = *lo[i + 1];
        asm("v_lshlrev_b64 %0, %1, %2" : "=v"(h) : "i"(S), "v"(h0));
        asm("v_lshrrev_b64 %0, %1, %2" : "=v"(l) : "i"(S), "v"(l0));
        hs[i] = h.x, hs[i + 1] = h.y;
        ls[i] = l.x, ls[i + 1] = l.y;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t a = *lo[i], b = *hi[i];
        *lo[i] = sel_b(hs[i], a, mask);
        *hi[i] = sel_b(b, ls[i], mask);
    }
}
// Exact 8 x 8 bit transpose in each byte lane of 8 dwords: afterwards plane k
// bit (8 p + r) = bit k of byte p of dword r.  An involution (bytes <-> planes).
// The three stages commute (each exchanges one register-index bit with one
// bit-in-byte index bit).
LDEV void transpose8(uint32_t* v, const XMasks& m) {
#ifdef ABL_XPOSE
    return;
#endif
    dstage<4>({&v[0], &v[1], &v[2], &v[3]}, {&v[4], &v[5], &v[6], &v[7]}, m.m4);
    dstage<2>({&v[0], &v[1], &v[4], &v[5]}, {&v[2], &v[3], &v[6], &v[7]}, m.m2);
    dstage<1>({&v[0], &v[4], &v[2], &v[6]}, {&v[1], &v[5], &v[3], &v[7]}, m.m1);
}

LDEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
// acc ^ (XOR of the planes y[j] with bit j of `row` set), as 3-input XORs
template <unsigned row, int J = 0>
LDEV uint32_t fold(uint32_t acc, const uint32_t* y) {
    if constexpr (J >= 8 || (row >> J) == 0) {
        return acc;
    } else if constexpr (((row >> J) & 1u) == 0) {
        return fold<row, J + 1>(acc, y);
    } else {
        constexpr unsigned rest = row & ~((2u << J) - 1u);  // bits above J
        if constexpr (rest == 0) {
            return acc ^ y[J];
        } else {
            constexpr int K = __builtin_ctz(rest);
            return fold<row & ~((2u << K) - 1u), K + 1>(xor3(acc, y[J], y[K]), y);
        }
    }
}
// Keep a value materialised here: the networks are all XORs, and without a
// fence the compiler reassociates them across butterflies and layers into
// long-lived shared subexpressions (200+ VGPRs instead of the tile's 128).
LDEV void pin8(uint32_t* v) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(v[k]));
}

// x ^= M * y (M compile time: the multiply by a constant as an XOR network)
template <uint64_t M>
LDEV void mac(uint32_t* x, const uint32_t* y) {
    static_for<0, 8>([&](auto I) {
        constexpr int i = decltype(I)::value;
        constexpr unsigned row = unsigned(M >> (8 * i)) & 0xFFu;
        if constexpr (row != 0) x[i] = fold<row>(x[i], y);
    });
}
// x ^= (M * y) & g  (g: a per-lane all-ones / all-zeros mask)
template <uint64_t M>
LDEV void mac_masked(uint32_t* x, const uint32_t* y, uint32_t g) {
#ifdef ABL_MASKED
    return;
#endif
    static_for<0, 8>([&](auto I) {
        constexpr int i = decltype(I)::value;
        constexpr unsigned row = unsigned(M >> (8 * i)) & 0xFFu;
        if constexpr (row != 0) {
            constexpr int J = __builtin_ctz(row);
            x[i] = xor_and(x[i], fold<(row & ~(1u << J))>(y[J], y), g);
        }
    });
}

// ------------------------------------------------------------ skews --------

constexpr unsigned sidx(unsigned p, unsigned l) { return ((p >> l) | 1u) << l; }
constexpr unsigned skew_at(int off, unsigned p, unsigned l) { return gf8_skew(off + int(sidx(p, l))); }

// ----------------------------------------------------------- layouts -------

// A layout says which piece-index bit each register-index bit (4) and each
// lane-group bit (3, g = lane >> 3) holds: piece(r, g) = the OR of bit i of r
// at position rb[i] and bit j of g at position gb[j].  Packed into a template
// argument: rb[i] in bits 3 i .. 3 i + 2, gb[j] in bits 12 + 3 j ...
constexpr uint32_t lay(unsigned r0, unsigned r1, unsigned r2, unsigned r3, unsigned g0, unsigned g1, unsigned g2) {
    return r0 | r1 << 3 | r2 << 6 | r3 << 9 | g0 << 12 | g1 << 15 | g2 << 18;
}
constexpr unsigned lay_rb(uint32_t L, unsigned i) { return (L >> (3 * i)) & 7u; }
constexpr unsigned lay_gb(uint32_t L, unsigned j) { return (L >> (12 + 3 * j)) & 7u; }
constexpr unsigned piece_of(uint32_t L, unsigned r, unsigned g) {
    unsigned p = 0;
    for (unsigned i = 0; i < 4; ++i) p |= ((r >> i) & 1u) << lay_rb(L, i);
    for (unsigned j = 0; j < 3; ++j) p |= ((g >> j) & 1u) << lay_gb(L, j);
    return p;
}
constexpr int reg_bit_of(uint32_t L, unsigned pbit) {
    for (unsigned i = 0; i < 4; ++i)
        if (lay_rb(L, i) == pbit) return int(i);
    return -1;
}
constexpr bool lay_ok(uint32_t L) {
    unsigned seen = 0;
    for (unsigned i = 0; i < 4; ++i) seen |= 1u << lay_rb(L, i);
    for (unsigned j = 0; j < 3; ++j) seen |= 1u << lay_gb(L, j);
    return seen == 127u;
}

// A layer-l skew depends on the piece bits above l only (sidx).  Those held
// by lane-group bits make it vary over the wave; it is affine in them
// (FFTInitialize builds FFTSkew[first + k 2^(l+1)] as the XOR of one generator
// per bit of k, LeopardFF8.cpp:505-514), so
//   c(r, g) * y = A_r * y  ^  sum over g bits j above l of  (g_j ? H_j * y : 0)
// with A_r = the skew of piece(r, 0) and H_j = the generator of bit gb[j]: the
// "twist", selected per lane by the all-ones masks G[j] (checked here for every
// layout the kernel uses).
constexpr unsigned twist_at(int off, uint32_t L, unsigned r, unsigned l, unsigned j) {
    const unsigned p = piece_of(L, r, 0);
    return lay_gb(L, j) > l ? skew_at(off, p | (1u << lay_gb(L, j)), l) ^ skew_at(off, p, l) : 0u;
}
constexpr bool affine_ok(uint32_t L, unsigned l) {
    for (int off : {-1, 127})
        for (unsigned r = 0; r < 16; ++r)
            for (unsigned g = 0; g < 8; ++g) {
                unsigned v = skew_at(off, piece_of(L, r, 0), l);
                for (unsigned j = 0; j < 3; ++j)
                    if ((g >> j) & 1u) v ^= twist_at(off, L, r, l, j);
                if (v != skew_at(off, piece_of(L, r, g), l)) return false;
            }
    return true;
}

// Layouts of the tile (LAMD_BS_SWAPS = 1, the default):
//   kLay0 (load / store, layer 0): registers = piece bits 0-3, lane groups 6, 5, 4;
//   kLay1 (layer 1): piece bit 0 <-> 4 exchanged (v_permlane32_swap: g bit 2 is lane bit 5);
//   kLay2 (layer 2): piece bit 1 <-> 5 exchanged (v_permlane16_swap: g bit 1 is lane bit 4);
//   kLayT (layers 3-6): piece bit 2 <-> 6 exchanged through LDS (g bit 0 is lane bit 3).
// Layer l then varies over the lane groups in 3, 2, 1, 0 bits (l = 0, 1, 2, >= 3),
// the fewest any 4-register-bit layout allows: 6 twisted (layer, bit) pairs per
// transform instead of 9.  LAMD_BS_SWAPS = 0 is the round-5 tile: layers 0-2 in
// kLay0 (lane groups 4, 5, 6), one LDS exchange of all three bits to kLayT.
#ifndef LAMD_BS_QUEUE
#define LAMD_BS_QUEUE 1  // tile queues (0: every wave codes tiles i, i + n, i + 2 n, ...)
#endif
#ifndef LAMD_BS_SWAPS
#define LAMD_BS_SWAPS 1
#endif
#if LAMD_BS_SWAPS
constexpr uint32_t kLay0 = lay(0, 1, 2, 3, 6, 5, 4);
constexpr uint32_t kLay1 = lay(4, 1, 2, 3, 6, 5, 0);
constexpr uint32_t kLay2 = lay(4, 5, 2, 3, 6, 1, 0);
constexpr uint32_t kLayT = lay(4, 5, 6, 3, 2, 1, 0);
#else
constexpr uint32_t kLay0 = lay(0, 1, 2, 3, 4, 5, 6);
constexpr uint32_t kLay1 = kLay0;
constexpr uint32_t kLay2 = kLay0;
constexpr uint32_t kLayT = lay(3, 4, 5, 6, 0, 1, 2);
#endif
static_assert(lay_ok(kLay0) && lay_ok(kLay1) && lay_ok(kLay2) && lay_ok(kLayT), "layouts are bit permutations");
static_assert(affine_ok(kLay0, 0) && affine_ok(kLay1, 1) && affine_ok(kLay2, 2), "skews are affine in the lane-group bits");

// ----------------------------------------------------------- butterflies ---

using Reg = uint32_t[16][8];

// Layer L in layout LAY: the pairs (r, r + 2^i) over the register bit i that
// holds piece bit L, restricted to the half of register bit 3 = H (H < 0: all
// 16 registers; the low layers never pair across it, it holds piece bit 3).
template <bool kInverse, int kOff, int L, uint32_t LAY, int H = -1>
LDEV void layer(Reg& x, const uint32_t (&G)[3]) {
    constexpr int ib = reg_bit_of(LAY, L);
    static_assert(ib >= 0, "the layer's bit is a register bit");
    constexpr unsigned half = 1u << ib;
    static_for<0, 16>([&](auto RI) {
        constexpr unsigned r = decltype(RI)::value;
        if constexpr ((r & half) == 0 && (H < 0 || int(r >> 3) == H)) {
            constexpr uint64_t A = gf8_matrix(skew_at(kOff, piece_of(LAY, r, 0), L));
            constexpr uint64_t H0 = gf8_matrix(twist_at(kOff, LAY, r, L, 0));
            constexpr uint64_t H1 = gf8_matrix(twist_at(kOff, LAY, r, L, 1));
            constexpr uint64_t H2 = gf8_matrix(twist_at(kOff, LAY, r, L, 2));
            uint32_t* a = x[r];
            uint32_t* b = x[r + half];
            if constexpr (kInverse) {  // IFFT_DIT2: y ^= x; x ^= y * skew
#pragma unroll
                for (int k = 0; k < 8; ++k) b[k] ^= a[k];
            }
            mac<A>(a, b);
            if constexpr (H0 != 0) mac_masked<H0>(a, b, G[0]);
            if constexpr (H1 != 0) mac_masked<H1>(a, b, G[1]);
            if constexpr (H2 != 0) mac_masked<H2>(a, b, G[2]);
            if constexpr (!kInverse) {  // FFT_DIT2: x ^= y * skew; y ^= x
#pragma unroll
                for (int k = 0; k < 8; ++k) b[k] ^= a[k];
            }
            pin8(a);
            pin8(b);
            bs_fence_every<LAMD_BS_BFENCE>(int(r));
        }
    });
}
// The top IFFT layer (skew base kOffI) and the top FFT layer (kOffF) on the
// same pairs as one butterfly with multiplier c1 + c2 (as Tile::fused_top):
// y1 = y ^ x, x2 = x ^ (c1 + c2) y1, y2 = y1 ^ x2.  Piece bit 6 is a register
// bit of kLayT and the skews of layer 6 are the same for every pair.
template <int kOffI, int kOffF>
LDEV void fused_top(Reg& x) {
    constexpr int ib = reg_bit_of(kLayT, 6);
    constexpr unsigned half = 1u << ib;
    constexpr uint64_t E = gf8_matrix(skew_at(kOffI, 64, 6) ^ skew_at(kOffF, 64, 6));
    static_for<0, 16>([&](auto RI) {
        constexpr unsigned r = decltype(RI)::value;
        if constexpr ((r & half) == 0) {
            uint32_t* a = x[r];
            uint32_t* b = x[r + half];
#pragma unroll
            for (int k = 0; k < 8; ++k) b[k] ^= a[k];
            mac<E>(a, b);
#pragma unroll
            for (int k = 0; k < 8; ++k) b[k] ^= a[k];
            pin8(a);
            pin8(b);
            bs_fence_every<LAMD_BS_BFENCE>(int(r));
        }
    });
}

// --------------------------------------------------------- exchanges -------

// Register bit IB <-> lane-group bit 2 (lane bit 5, v_permlane32_swap) or 1
// (lane bit 4, v_permlane16_swap) on the registers of half H (register bit 3):
// for each pair (R0, R1) over bit IB the swap leaves R0 = [R0 lanes with the
// bit clear, R1 lanes with it clear], R1 = [R0 set, R1 set] -- the two bits
// trade places, as one VALU instruction per dword pair.
template <int IB, int GBIT, int H>
LDEV void swap_lanes(Reg& x) {
    static_assert(GBIT == 1 || GBIT == 2, "permlane swaps exist for lane bits 4 and 5");
#if defined(ABL_XCH) || defined(ABL_SWAP)
    return;
#endif
    static_for<0, 16>([&](auto RI) {
        constexpr unsigned r = decltype(RI)::value;
        if constexpr (((r >> IB) & 1u) == 0 && int(r >> 3) == H) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if constexpr (GBIT == 2) {
                    const auto v = __builtin_amdgcn_permlane32_swap(x[r][k], x[r | (1u << IB)][k], false, false);
                    x[r][k] = v[0];
                    x[r | (1u << IB)][k] = v[1];
                } else {
                    const auto v = __builtin_amdgcn_permlane16_swap(x[r][k], x[r | (1u << IB)][k], false, false);
                    x[r][k] = v[0];
                    x[r | (1u << IB)][k] = v[1];
                }
            }
        }
    });
}

// Layout FROM -> TO through the wave's LDS area, in 4 rounds of 2 planes: every
// register of every lane written at (piece, lane column) in FROM and read back
// at (piece, lane column) in TO.  Byte address of piece p, column l:
//   64 (p + pad(p)) + 8 l,  pad(p) = p >> 4 for the round-5 tile (its lane groups
// hold pieces 16 apart) and 0 otherwise,
// so that the 8 lane groups of one access fall in 4 different 64-byte bank
// windows (two lanes per bank: the minimum for 8-byte accesses).  The
// per-register part is a compile-time offset (the ds instruction's immediate).
constexpr unsigned kBsPad = LAMD_BS_SWAPS ? 0u : 1u;
constexpr unsigned lds_row(unsigned p) { return p + (kBsPad ? (p >> 4) : 0u); }
template <uint32_t FROM, uint32_t TO>
LDEV void exchange(Reg& x, uint8_t* area, unsigned g, unsigned l) {
#if defined(ABL_XCH) || defined(ABL_LDSX)
    return;
#endif
    Reg y;
    // lane parts: the lane-group bits of FROM / TO (disjoint from every register's
    // piece bits, so row(p(r, g)) = row(p(r, 0)) + row part of g when unpadded;
    // padded rows are exact because the round-5 lane bits are the high bits)
    uint8_t* const wbase = area + 64u * lds_row(piece_of(FROM, 0, g)) + 8u * l;
    uint8_t* const rbase = area + 64u * lds_row(piece_of(TO, 0, g)) + 8u * l;
    static_for<0, 4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        static_for<0, 16>([&](auto RI) {
            constexpr unsigned r = decltype(RI)::value;
            v2u v;
            v.x = x[r][2 * q];
            v.y = x[r][2 * q + 1];
            *reinterpret_cast<v2u*>(wbase + 64u * (lds_row(piece_of(FROM, r, 0)) - lds_row(0))) = v;
        });
        // one wave's LDS operations execute in order: the reads below see the
        // writes above, and the next round's writes follow these reads
        asm volatile("" ::: "memory");
        static_for<0, 16>([&](auto RI) {
            constexpr unsigned r = decltype(RI)::value;
            const v2u v = *reinterpret_cast<const v2u*>(rbase + 64u * (lds_row(piece_of(TO, r, 0)) - lds_row(0)));
            y[r][2 * q] = v.x;
            y[r][2 * q + 1] = v.y;
        });
        asm volatile("" ::: "memory");
    });
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int k = 0; k < 8; ++k) x[r][k] = y[r][k];
}

// ---------------------------------------------------------- tile I/O -----

// Where one tile (object, 256-byte column strip) lives for this lane.
#ifndef LAMD_BS_NT
#define LAMD_BS_NT 3  // nontemporal piece loads (1) and stores (2): +4% on the headline (profiles/r05_v6/nt_ab.txt)
#endif
// Where one tile (object, 256-byte column strip) lives for this lane: the
// strip's column in piece 0 of the object's input / output slab (wave-uniform,
// scalar registers), the slab strides (uniform) and the lane's offsets from
// there: its lane group's first piece, piece_of(kLay0, 0, g), plus its two
// 16-byte segments (a segment past the piece's end re-reads segment 0).  Piece
// register r is at column + r * stride + lane offset: the per-register part is
// scalar arithmetic.  kNarrow (every stride in [0, 2^32 / 128)): 32-bit lane
// offsets, so a load or store is one global_*_dwordx4 with a scalar base and
// a 32-bit vector offset (no 64-bit vector address per instruction).
template <bool kNarrow>
struct BsTile {
    using Off = std::conditional_t<kNarrow, uint32_t, int64_t>;
    uint64_t in, out;
    int32_t in_stride, out_stride;
    Off in0, in1, out0, out1;
};
template <bool kNarrow>
LDEV BsTile<kNarrow> bs_tile(const Ff8SlabBatch& b, unsigned t, unsigned strips, unsigned g, unsigned l) {
    using Off = typename BsTile<kNarrow>::Off;
    const unsigned obj = t / strips, strip = t - obj * strips;
    const uint32_t rem = b.nunits * 4u - strip * kBsStrip;  // >= 64 (bytes % 64 == 0)
    const uint32_t o0 = 16u * l, o1 = 128u + 16u * l;
    const uint32_t s0 = o0 + 16u <= rem ? o0 : 0u, s1 = o1 + 16u <= rem ? o1 : 0u;
    BsTile<kNarrow> T;
    T.in_stride = b.in_stride[obj];
    T.out_stride = b.out_stride[obj];
    const uint64_t col = uint64_t(strip) * kBsStrip;
    T.in = b.in_base[obj] + col;
    T.out = b.out_base[obj] + col;
    const Off pg = Off(piece_of(kLay0, 0, g));  // the lane group's pieces: pg | r
    T.in0 = pg * Off(T.in_stride) + s0;
    T.in1 = pg * Off(T.in_stride) + s1;
    T.out0 = pg * Off(T.out_stride) + s0;
    T.out1 = pg * Off(T.out_stride) + s1;
    return T;
}
template <class Off>
LDEV auto bs_addr(uint64_t base_r, Off off) {  // a global (address space 1) pointer
    if constexpr (std::is_same_v<Off, uint32_t>)
        return gptr<v4u>(reinterpret_cast<uint8_t*>(base_r) + uint64_t(off));
    else
        return gptr<v4u>(reinterpret_cast<uint8_t*>(base_r) + off);
}
// One piece register r (piece r | piece_of(kLay0, 0, g)) of a tile: a lane
// group reads 128 contiguous bytes per instruction.
template <bool kNarrow>
LDEV void load_reg(uint32_t* v, const BsTile<kNarrow>& T, int r) {
    const uint64_t base = T.in + uint64_t(int64_t(r) * T.in_stride);
#ifdef ABL_MEM
    v4u v0, v1;
    v0.x = uint32_t(base) + uint32_t(T.in0) + threadIdx.x, v0.y = v0.x * 3, v0.z = v0.x * 5, v0.w = v0.x * 7;
    v1 = v0 * 11u;
#else
#if LAMD_BS_NT & 1
    const v4u v0 = __builtin_nontemporal_load(bs_addr(base, T.in0));
    const v4u v1 = __builtin_nontemporal_load(bs_addr(base, T.in1));
#else
    const v4u v0 = *bs_addr(base, T.in0);
    const v4u v1 = *bs_addr(base, T.in1);
#endif
#endif
    v[0] = v0.x, v[1] = v0.y, v[2] = v0.z, v[3] = v0.w;
    v[4] = v1.x, v[5] = v1.y, v[6] = v1.z, v[7] = v1.w;
}
// Registers R0 .. R1 - 1 of a tile.
template <int R0, int R1 = R0 + 8, bool kNarrow>
LDEV void load_half(Reg& x, const BsTile<kNarrow>& T) {
#pragma unroll
    for (int r = R0; r < R1; ++r) load_reg(x[r], T, r);
}
template <int R0, bool kNarrow>
LDEV void store_half(const Reg& x, const BsTile<kNarrow>& T) {
#pragma unroll
    for (int r = R0; r < R0 + 8; ++r) {
        const uint64_t base = T.out + uint64_t(int64_t(r) * T.out_stride);
        v4u v0, v1;
        v0.x = x[r][0], v0.y = x[r][1], v0.z = x[r][2], v0.w = x[r][3];
        v1.x = x[r][4], v1.y = x[r][5], v1.z = x[r][6], v1.w = x[r][7];
#ifdef ABL_MEM
        const uint32_t acc = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
        if (acc == 0x12345679u && T.in_stride == 7) *gptr<uint32_t>(reinterpret_cast<uint8_t*>(base)) = acc;  // keep the values live
        continue;
#endif
        // A segment past the piece's end was loaded from segment 0 of the
        // strip (always inside: pieces are multiples of 64 bytes), and the
        // transform is column by column, so it holds segment 0's output: it is
        // stored there, the same bytes lane 8 g writes (no branch per store).
        const auto p0 = bs_addr(base, T.out0);
        const auto p1 = bs_addr(base, T.out1);
#if LAMD_BS_NT & 2
        __builtin_nontemporal_store(v0, p0);
        __builtin_nontemporal_store(v1, p1);
#else
        *p0 = v0;
        *p1 = v1;
#endif
    }
}
template <int R0>
LDEV void transpose_half(Reg& x, const XMasks& xm) {
#pragma unroll
    for (int r = R0; r < R0 + 8; ++r) {
        transpose8(x[r], xm);
        pin8(x[r]);
        bs_fence_every<LAMD_BS_XFENCE>(r);
    }
}

#ifdef LAMD_CLOCK
// Diagnostic builds only (tools/bs_clock.py): per wave, (s_memtime,
// s_memrealtime) at entry and exit, for the shader clock under this kernel's
// load and the waves' lifetimes.
__device__ uint64_t* g_bs_clock;
#endif

// -------------------------------------------------------------- kernel -----

// One transform direction's low layers (0-2) on half H, and their inverse order.
template <bool kInverse, int kOff, int H>
LDEV void low_layers(Reg& x, const uint32_t (&G)[3]) {
    if constexpr (kInverse) {
        layer<true, kOff, 0, kLay0, H>(x, G);
        if constexpr (LAMD_BS_SWAPS) swap_lanes<0, 2, H>(x);
        layer<true, kOff, 1, kLay1, H>(x, G);
        if constexpr (LAMD_BS_SWAPS) swap_lanes<1, 1, H>(x);
        layer<true, kOff, 2, kLay2, H>(x, G);
    } else {
        layer<false, kOff, 2, kLay2, H>(x, G);
        if constexpr (LAMD_BS_SWAPS) swap_lanes<1, 1, H>(x);
        layer<false, kOff, 1, kLay1, H>(x, G);
        if constexpr (LAMD_BS_SWAPS) swap_lanes<0, 2, H>(x);
        layer<false, kOff, 0, kLay0, H>(x, G);
    }
}

// Persistent waves: the grid fills the GPU once (kBsBlocksPerCu workgroups of
// kBsWaves independent waves a CU) and wave i codes tiles i, i + n, ... (tile =
// object * strips + strip).  A tile is software-pipelined in halves (register
// bit 3 = piece bit 3 in every low layout, never paired by layers 0-2 or the
// lane swaps): the last FFT layers, transposes and stores of half 0 run, then
// the next tile's half-0 loads are issued into the freed registers while half 1
// computes; at the top of the next tile half 1's loads are in flight while half
// 0 transposes and runs its IFFT layers.  (Deeper prefetch -- part of the next
// tile a whole tile ahead, by LDS-DMA into the unused LDS or into spare VGPRs --
// addresses latency, which is not what binds: the kernel runs at the board's
// power limit, memory and arithmetic each at full clock alone)
template <int kForm, bool kNarrow>
__global__ void __launch_bounds__(64 * kBsWaves) __attribute__((amdgpu_waves_per_eu(LAMD_BS_OCC, LAMD_BS_OCC)))
k_ff8_bs_slab(Ff8SlabBatch b, uint32_t count, uint32_t strips, uint32_t* q, uint32_t* qclear) {
    constexpr int kOffI = kForm == kFormDenseDec ? -1 : 127;  // IFFT skew base
    constexpr int kOffF = kForm == kFormDenseDec ? 127 : -1;  // FFT skew base
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const unsigned wave = threadIdx.x >> 6;
    const unsigned n = gridDim.x * kBsWaves, total = count * strips;
    uint8_t* const area = reinterpret_cast<uint8_t*>(lds + wave * kBsAreaDw);
    // wave-uniform, so that a tile's pointers are scalar loads (off the vector
    // memory counter the piece loads are waited on with)
    unsigned t = __builtin_amdgcn_readfirstlane(blockIdx.x * kBsWaves + wave);
    if (t >= total) return;  // waves share nothing
#ifdef LAMD_CLOCK
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned t0 = t;
#endif
    const unsigned lane = threadIdx.x & 63u, g = lane >> 3, l = lane & 7u;
    // Tile queues (q != null): after the first round (tile = wave index) a wave
    // takes its next tile from the queue of its XCD (workgroups are dealt to
    // the 8 XCDs round robin): tiles n + xq + 8 k, k = that queue's counter.
    // Waves that run faster take more tiles, so all of a launch's waves end
    // within about one tile of each other (a static share left the two waves
    // of a SIMD ending up to ~35% apart, the second one alone at half the issue
    // rate).  One counter set per launch; this launch zeroes the other set, the
    // previous launch's, for the next one (Workspace::bs_queue).
    if (qclear != nullptr && blockIdx.x == 0 && wave == 0 && lane < 8u) qclear[32u * lane] = 0u;
    const unsigned xq = blockIdx.x & 7u;
    uint32_t* const head = q != nullptr ? q + 32u * xq : nullptr;
    const uint32_t G[3] = {(g & 1u) ? ~0u : 0u, (g & 2u) ? ~0u : 0u, (g & 4u) ? ~0u : 0u};
    const XMasks xm;
    Reg x;
    BsTile<kNarrow> cur = bs_tile<kNarrow>(b, t, strips, g, l);
    load_half<0, 8>(x, cur);
    load_half<8, 16>(x, cur);
    for (;;) {
        // the next tile's index, requested a tile ahead (its latency hidden)
        uint32_t kq = 0;
        if (head != nullptr && lane == 0) kq = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifndef ABL_ARITH
        transpose_half<0>(x, xm);
        low_layers<true, kOffI, 0>(x, G);
        transpose_half<8>(x, xm);
        low_layers<true, kOffI, 1>(x, G);
        exchange<kLay2, kLayT>(x, area, g, l);
        layer<true, kOffI, 3, kLayT>(x, G);
        layer<true, kOffI, 4, kLayT>(x, G);
        layer<true, kOffI, 5, kLayT>(x, G);
        fused_top<kOffI, kOffF>(x);
        layer<false, kOffF, 5, kLayT>(x, G);
        layer<false, kOffF, 4, kLayT>(x, G);
        layer<false, kOffF, 3, kLayT>(x, G);
        exchange<kLayT, kLay2>(x, area, g, l);
#else
#pragma unroll
        for (int r = 0; r < 16; ++r) pin8(x[r]);
#endif
        const unsigned tn = head != nullptr ? n + xq + 8u * __builtin_amdgcn_readfirstlane(kq) : t + n;
        const bool more = tn < total;
        const BsTile<kNarrow> nxt = bs_tile<kNarrow>(b, more ? tn : t, strips, g, l);
#ifndef ABL_ARITH
        low_layers<false, kOffF, 0>(x, G);
        transpose_half<0>(x, xm);
#endif
        store_half<0>(x, cur);
        if (more) load_half<0, 8>(x, nxt);
#ifndef ABL_ARITH
        low_layers<false, kOffF, 1>(x, G);
        transpose_half<8>(x, xm);
#endif
        store_half<8>(x, cur);
        if (!more) break;
        load_half<8, 16>(x, nxt);
        t = tn;
        cur = nxt;
    }
#ifdef LAMD_CLOCK
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63u) == 0 && g_bs_clock != nullptr) {  // null unless tools/bs_clock.py set it
        uint64_t* o = g_bs_clock + 4ull * t0;
        o[0] = c0, o[1] = r0, o[2] = c1, o[3] = r1;
    }
#endif
}

}  // namespace

bool ff8_bs_supported(unsigned T, unsigned K, unsigned R, unsigned nchunks) {
    return T == 7 && K == 128 && R == 128 && nchunks == 1;
}

hipError_t launch_ff8_bs_slab(const Ff8SlabBatch& b, unsigned count, int form, hipStream_t s, unsigned cus,
                              uint32_t* q, uint32_t* qclear) {
    if (count == 0 || count > kSlabObjs || (b.nunits * 4u) % 64u != 0 || b.K != 128 || b.R != 128)
        return hipErrorInvalidValue;
    if (form != kFormDenseEnc && form != kFormDenseDec) return hipErrorInvalidValue;
    cus = std::max(cus, 1u);
    uint32_t strips = (b.nunits * 4u + kBsStrip - 1) / kBsStrip;
    uint32_t cnt = count;
    const unsigned total = cnt * strips;
    const unsigned blocks = std::min<unsigned>((total + kBsWaves - 1) / kBsWaves, cus * kBsBlocksPerCu);
    const size_t lds = size_t(kBsWaves) * kBsAreaDw * 4;
#if LAMD_BS_QUEUE == 0
    q = qclear = nullptr;
#endif
    // the 8 queues each serve the workgroups of one XCD (blockIdx.x & 7): every
    // queue needs workgroups, or static assignment (tiles i, i + n, ...); the
    // next launch's set is still cleared (Workspace::bs_queue alternates them)
    if (blocks < 8) q = nullptr;
    void* params[] = {const_cast<Ff8SlabBatch*>(&b), &cnt, &strips, &q, &qclear};
    // 32-bit lane offsets when every slab's lane offsets (up to 127 strides + a
    // strip) fit them
    bool narrow = true;
    for (unsigned o = 0; o < count; ++o)
        for (const int32_t st : {b.in_stride[o], b.out_stride[o]})
            narrow = narrow && st >= 0 && uint64_t(st) * 128u + kBsStrip <= (uint64_t(1) << 32);
    const void* fn = form == kFormDenseDec
                         ? (narrow ? reinterpret_cast<const void*>(&k_ff8_bs_slab<kFormDenseDec, true>)
                                   : reinterpret_cast<const void*>(&k_ff8_bs_slab<kFormDenseDec, false>))
                         : (narrow ? reinterpret_cast<const void*>(&k_ff8_bs_slab<kFormDenseEnc, true>)
                                   : reinterpret_cast<const void*>(&k_ff8_bs_slab<kFormDenseEnc, false>));
    return hipLaunchKernel(fn, dim3(blocks), dim3(64 * kBsWaves), params, lds, s);
}

}  // namespace lamd

#ifdef LAMD_CLOCK
extern "C" __attribute__((visibility("default"))) int leo_amd_debug_bs_clock(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(lamd::g_bs_clock), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif
