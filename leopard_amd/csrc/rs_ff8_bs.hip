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
// lane-group part of a layout-0 skew: bit c of g = piece bit 4 + c
constexpr unsigned twist(int off, unsigned r, unsigned l, unsigned c) {
    return skew_at(off, r | (16u << c), l) ^ skew_at(off, r, l);
}
constexpr bool affine_ok() {
    for (int off : {-1, 127})
        for (unsigned l = 0; l < 3; ++l)
            for (unsigned r = 0; r < 16; ++r)
                for (unsigned g = 0; g < 8; ++g) {
                    unsigned v = skew_at(off, r, l);
                    for (unsigned c = 0; c < 3; ++c)
                        if ((g >> c) & 1u) v ^= twist(off, r, l, c);
                    if (v != skew_at(off, r | (g << 4), l)) return false;
                }
    return true;
}
static_assert(affine_ok(), "layout-0 skews are affine in the lane-group bits");

// ----------------------------------------------------------- butterflies ---

using Reg = uint32_t[16][8];

// Layout 0, layer L in {0, 1, 2}: pairs (r, r + 2^L) of register bits 0-3, in
// the half r = R0 .. R0 + 7 (the pairs never cross halves).
template <bool kInverse, int kOff, int L, int R0>
LDEV void layer_low(Reg& x, const uint32_t (&G)[3]) {
    constexpr int half = 1 << L;
    static_for<R0, R0 + 8>([&](auto RI) {
        constexpr unsigned r = decltype(RI)::value;
        if constexpr ((r & half) == 0) {
            constexpr uint64_t A = gf8_matrix(skew_at(kOff, r, L));
            constexpr uint64_t H0 = gf8_matrix(twist(kOff, r, L, 0));
            constexpr uint64_t H1 = gf8_matrix(twist(kOff, r, L, 1));
            constexpr uint64_t H2 = gf8_matrix(twist(kOff, r, L, 2));
            uint32_t* a = x[r];
            uint32_t* b = x[r + half];
            if constexpr (kInverse) {  // IFFT_DIT2: y ^= x; x ^= y * skew
#pragma unroll
                for (int k = 0; k < 8; ++k) b[k] ^= a[k];
            }
            mac<A>(a, b);
            mac_masked<H0>(a, b, G[0]);
            mac_masked<H1>(a, b, G[1]);
            mac_masked<H2>(a, b, G[2]);
            if constexpr (!kInverse) {  // FFT_DIT2: x ^= y * skew; y ^= x
#pragma unroll
                for (int k = 0; k < 8; ++k) b[k] ^= a[k];
            }
            pin8(a);
            pin8(b);
            bs_fence_every<LAMD_BS_BFENCE>(int((r >> (L + 1)) << L | (r & (half - 1))));
        }
    });
}
// Layout top, layer L in {3, 4, 5}: pairs over register bit L - 3 (piece g | r << 3).
template <bool kInverse, int kOff, int L>
LDEV void layer_top(Reg& x) {
    constexpr int half = 1 << (L - 3);
    static_for<0, 16>([&](auto RI) {
        constexpr unsigned r = decltype(RI)::value;
        if constexpr ((r & half) == 0) {
            constexpr uint64_t A = gf8_matrix(skew_at(kOff, r << 3, L));
            uint32_t* a = x[r];
            uint32_t* b = x[r + half];
            if constexpr (kInverse) {
#pragma unroll
                for (int k = 0; k < 8; ++k) b[k] ^= a[k];
            }
            mac<A>(a, b);
            if constexpr (!kInverse) {
#pragma unroll
                for (int k = 0; k < 8; ++k) b[k] ^= a[k];
            }
            pin8(a);
            pin8(b);
            bs_fence_every<LAMD_BS_BFENCE>(int((r >> (L - 2)) << (L - 3) | (r & (half - 1))));
        }
    });
}
// The top IFFT layer (skew base kOffI) and the top FFT layer (kOffF) on the
// same pairs (r, r + 8) as one butterfly with multiplier c1 + c2 (as
// Tile::fused_top): y1 = y ^ x, x2 = x ^ (c1 + c2) y1, y2 = y1 ^ x2.
template <int kOffI, int kOffF>
LDEV void fused_top(Reg& x) {
    constexpr uint64_t E = gf8_matrix(skew_at(kOffI, 64, 6) ^ skew_at(kOffF, 64, 6));
    static_for<0, 8>([&](auto RI) {
        constexpr unsigned r = decltype(RI)::value;
        uint32_t* a = x[r];
        uint32_t* b = x[r + 8];
#pragma unroll
        for (int k = 0; k < 8; ++k) b[k] ^= a[k];
        mac<E>(a, b);
#pragma unroll
        for (int k = 0; k < 8; ++k) b[k] ^= a[k];
        pin8(a);
        pin8(b);
        bs_fence_every<LAMD_BS_BFENCE>(int(r));
    });
}

// --------------------------------------------------------- exchanges -------

// LDS byte address of piece p, lane l in the wave's area: 64-byte rows of
// 8 lanes x 8 bytes, one pad row after every 16 pieces,
//   64 p + 64 (p >> 4) + 8 l,
// so that the 8 lane groups of a layout-0 access (pieces 16 apart: 1088 g) and
// of a layout-top access (pieces 1 apart: 64 g) fall in 4 different 64-byte
// bank windows (two lanes per bank: the minimum for 8-byte accesses).  The
// per-register part is a compile-time offset (the ds instruction's immediate).
constexpr unsigned off0(unsigned r) { return 64u * r; }                               // layout 0, + lane part 1088 g + 8 l
constexpr unsigned offT(unsigned r) { return 512u * r + 64u * (r >> 1); }            // layout top, + lane part 64 g + 8 l

// Layout 0 -> top (kToTop) or back, in 4 rounds of 2 planes through the wave's area.
template <bool kToTop>
LDEV void exchange(Reg& x, uint8_t* area, unsigned g, unsigned l) {
#ifdef ABL_XCH
    return;
#endif
    Reg y;
    uint8_t* const base0 = area + 1088u * g + 8u * l;
    uint8_t* const baseT = area + 64u * g + 8u * l;
    uint8_t* const wbase = kToTop ? base0 : baseT;
    uint8_t* const rbase = kToTop ? baseT : base0;
    static_for<0, 4>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        static_for<0, 16>([&](auto RI) {
            constexpr unsigned r = decltype(RI)::value;
            v2u v;
            v.x = x[r][2 * q];
            v.y = x[r][2 * q + 1];
            *reinterpret_cast<v2u*>(wbase + (kToTop ? off0(r) : offT(r))) = v;
        });
        // one wave's LDS operations execute in order: the reads below see the
        // writes above, and the next round's writes follow these reads
        asm volatile("" ::: "memory");
        static_for<0, 16>([&](auto RI) {
            constexpr unsigned r = decltype(RI)::value;
            const v2u v = *reinterpret_cast<const v2u*>(rbase + (kToTop ? offT(r) : off0(r)));
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

// -------------------------------------------------------------- kernel -----

// Where one tile (object, 256-byte column strip) lives for this lane.
#ifndef LAMD_BS_PRIO
#define LAMD_BS_PRIO 0
#endif
#ifndef LAMD_BS_NT
#define LAMD_BS_NT 3  // nontemporal piece loads (1) and stores (2): +4% on the headline (profiles/r05_v6/nt_ab.txt)
#endif
struct BsTile {
    const uint8_t* in;   // piece g << 4 of the strip, + lane offset
    uint8_t* out;
    int32_t in_stride, out_stride;
    uint32_t l0, l1;     // offsets of the lane's two 16-byte segments (past the piece's end: segment 0)
};
LDEV BsTile bs_tile(const Ff8SlabBatch& b, unsigned t, unsigned strips, unsigned g, unsigned l) {
    const unsigned obj = t / strips, strip = t - obj * strips;
    const uint32_t rem = b.nunits * 4u - strip * kBsStrip;  // >= 64 (bytes % 64 == 0)
    const uint32_t o0 = 16u * l, o1 = 128u + 16u * l;
    BsTile T;
    T.in_stride = b.in_stride[obj];
    T.out_stride = b.out_stride[obj];
    const uint64_t col = uint64_t(strip) * kBsStrip;
    T.in = reinterpret_cast<const uint8_t*>(b.in_base[obj] + col) + int64_t(g << 4) * T.in_stride;
    T.out = reinterpret_cast<uint8_t*>(b.out_base[obj] + col) + int64_t(g << 4) * T.out_stride;
    T.l0 = o0 + 16u <= rem ? o0 : 0u;
    T.l1 = o1 + 16u <= rem ? o1 : 0u;
    return T;
}
// Pieces r0 .. r0 + 7 (| g << 4) of a tile: a lane group reads 128 contiguous
// bytes per instruction.
template <int R0>
LDEV void load_half(Reg& x, const BsTile& T) {
#pragma unroll
    for (int r = R0; r < R0 + 8; ++r) {
        const uint8_t* p = T.in + int64_t(r) * T.in_stride;
#ifdef ABL_MEM
        v4u v0, v1;
        v0.x = uint32_t(uintptr_t(p)) + threadIdx.x, v0.y = v0.x * 3, v0.z = v0.x * 5, v0.w = v0.x * 7;
        v1 = v0 * 11u;
#else
#if LAMD_BS_NT & 1
        const v4u v0 = __builtin_nontemporal_load(gptr<const v4u>(p + T.l0));
        const v4u v1 = __builtin_nontemporal_load(gptr<const v4u>(p + T.l1));
#else
        const v4u v0 = *gptr<const v4u>(p + T.l0);
        const v4u v1 = *gptr<const v4u>(p + T.l1);
#endif
#endif
        x[r][0] = v0.x, x[r][1] = v0.y, x[r][2] = v0.z, x[r][3] = v0.w;
        x[r][4] = v1.x, x[r][5] = v1.y, x[r][6] = v1.z, x[r][7] = v1.w;
    }
}
template <int R0>
LDEV void store_half(const Reg& x, const BsTile& T) {
#pragma unroll
    for (int r = R0; r < R0 + 8; ++r) {
        uint8_t* p = T.out + int64_t(r) * T.out_stride;
        v4u v0, v1;
        v0.x = x[r][0], v0.y = x[r][1], v0.z = x[r][2], v0.w = x[r][3];
        v1.x = x[r][4], v1.y = x[r][5], v1.z = x[r][6], v1.w = x[r][7];
#ifdef ABL_MEM
        const uint32_t acc = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
        if (acc == 0x12345679u && T.in_stride == 7) *gptr<uint32_t>(p) = acc;  // keep the values live
        continue;
#endif
        // A segment past the piece's end was loaded from segment 0 of the
        // strip (always inside: pieces are multiples of 64 bytes), and the
        // transform is column by column, so it holds segment 0's output: it is
        // stored there, the same bytes lane 8 g writes (no branch per store).
#if LAMD_BS_NT & 2
        __builtin_nontemporal_store(v0, gptr<v4u>(p + T.l0));
        __builtin_nontemporal_store(v1, gptr<v4u>(p + T.l1));
#else
        *gptr<v4u>(p + T.l0) = v0;
        *gptr<v4u>(p + T.l1) = v1;
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

// Persistent waves: the grid fills the GPU once (kBsBlocksPerCu workgroups of
// kBsWaves independent waves a CU) and wave i codes tiles i, i + n, ... (tile =
// object * strips + strip).  A tile is software-pipelined in halves: the low
// layers (0-2) pair registers r and r ^ 1, 2, 4 only, so pieces 0-7 and 8-15 of
// layout 0 are independent there.  The last FFT layers, transposes and stores
// of half 0 run, then the next tile's half-0 loads are issued into the freed
// registers while half 1 computes; at the top of the next tile half 1's loads
// are in flight while half 0 transposes and runs its IFFT layers.
#ifndef LAMD_BS_STAGGER
#define LAMD_BS_STAGGER_BLOCKS 0
#define LAMD_BS_STAGGER 0  // s_sleep 127 (8128 cycles) steps of the second wave of a SIMD (measured: 1, 2, 4 slower)
#endif
template <int kForm>
__global__ void __launch_bounds__(64 * kBsWaves) __attribute__((amdgpu_waves_per_eu(LAMD_BS_OCC, LAMD_BS_OCC)))
k_ff8_bs_slab(Ff8SlabBatch b, uint32_t count, uint32_t strips) {
    constexpr int kOffI = kForm == kFormDenseDec ? -1 : 127;  // IFFT skew base
    constexpr int kOffF = kForm == kFormDenseDec ? 127 : -1;  // FFT skew base
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const unsigned wave = threadIdx.x >> 6;
    const unsigned n = gridDim.x * kBsWaves, total = count * strips;
    uint8_t* const area = reinterpret_cast<uint8_t*>(lds + wave * kBsAreaDw);
    unsigned t = blockIdx.x * kBsWaves + wave;
    if (t >= total) return;  // wave-uniform; waves share nothing
#if LAMD_BS_STAGGER_BLOCKS  // the second half of the grid (the second workgroup of each CU, dispatch order)
    if (blockIdx.x >= gridDim.x / 2 && t + n < total)
#else
    if (wave >= kBsWaves / 2 && t + n < total)
#endif
        for (int i = 0; i < LAMD_BS_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
    const unsigned lane = threadIdx.x & 63u, g = lane >> 3, l = lane & 7u;
    const uint32_t G[3] = {(g & 1u) ? ~0u : 0u, (g & 2u) ? ~0u : 0u, (g & 4u) ? ~0u : 0u};
    const XMasks xm;
    Reg x;
    BsTile cur = bs_tile(b, t, strips, g, l);
    load_half<0>(x, cur);
    load_half<8>(x, cur);
    for (;;) {
#ifndef ABL_ARITH
        transpose_half<0>(x, xm);
        layer_low<true, kOffI, 0, 0>(x, G);
        layer_low<true, kOffI, 1, 0>(x, G);
        layer_low<true, kOffI, 2, 0>(x, G);
        transpose_half<8>(x, xm);
        layer_low<true, kOffI, 0, 8>(x, G);
        layer_low<true, kOffI, 1, 8>(x, G);
        layer_low<true, kOffI, 2, 8>(x, G);
        exchange<true>(x, area, g, l);
        layer_top<true, kOffI, 3>(x);
        layer_top<true, kOffI, 4>(x);
        layer_top<true, kOffI, 5>(x);
        fused_top<kOffI, kOffF>(x);
        layer_top<false, kOffF, 5>(x);
        layer_top<false, kOffF, 4>(x);
        layer_top<false, kOffF, 3>(x);
        exchange<false>(x, area, g, l);
#endif
        const unsigned tn = t + n;
        const bool more = tn < total;
        const BsTile nxt = bs_tile(b, more ? tn : t, strips, g, l);
#ifndef ABL_ARITH
        layer_low<false, kOffF, 2, 0>(x, G);
        layer_low<false, kOffF, 1, 0>(x, G);
        layer_low<false, kOffF, 0, 0>(x, G);
        transpose_half<0>(x, xm);
#endif
        store_half<0>(x, cur);
#if LAMD_BS_PRIO
        __builtin_amdgcn_s_setprio(LAMD_BS_PRIO);  // experiments: issue the next tile's loads ahead of the other wave's arithmetic
#endif
        if (more) load_half<0>(x, nxt);
#if LAMD_BS_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
#ifndef ABL_ARITH
        layer_low<false, kOffF, 2, 8>(x, G);
        layer_low<false, kOffF, 1, 8>(x, G);
        layer_low<false, kOffF, 0, 8>(x, G);
        transpose_half<8>(x, xm);
#endif
        store_half<8>(x, cur);
        if (!more) break;
#if LAMD_BS_PRIO
        __builtin_amdgcn_s_setprio(LAMD_BS_PRIO);
#endif
        load_half<8>(x, nxt);
#if LAMD_BS_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        t = tn;
        cur = nxt;
    }
}

}  // namespace

bool ff8_bs_supported(unsigned T, unsigned K, unsigned R, unsigned nchunks) {
    return T == 7 && K == 128 && R == 128 && nchunks == 1;
}

hipError_t launch_ff8_bs_slab(const Ff8SlabBatch& b, unsigned count, int form, hipStream_t s) {
    if (count == 0 || count > kSlabObjs || (b.nunits * 4u) % 64u != 0 || b.K != 128 || b.R != 128)
        return hipErrorInvalidValue;
    if (form != kFormDenseEnc && form != kFormDenseDec) return hipErrorInvalidValue;
    static int cus[64] = {};  // compute units per device (queried once)
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (cus[dev] == 0) {
        int n = 0;
        e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        cus[dev] = n > 0 ? n : 1;
    }
    uint32_t strips = (b.nunits * 4u + kBsStrip - 1) / kBsStrip;
    uint32_t cnt = count;
    const unsigned total = cnt * strips;
    const unsigned blocks = std::min<unsigned>((total + kBsWaves - 1) / kBsWaves, unsigned(cus[dev]) * kBsBlocksPerCu);
    const size_t lds = size_t(kBsWaves) * kBsAreaDw * 4;
    void* params[] = {const_cast<Ff8SlabBatch*>(&b), &cnt, &strips};
    const void* fn = form == kFormDenseDec ? reinterpret_cast<const void*>(&k_ff8_bs_slab<kFormDenseDec>)
                                           : reinterpret_cast<const void*>(&k_ff8_bs_slab<kFormDenseEnc>);
    return hipLaunchKernel(fn, dim3(blocks), dim3(64 * kBsWaves), params, lds, s);
}

}  // namespace lamd
