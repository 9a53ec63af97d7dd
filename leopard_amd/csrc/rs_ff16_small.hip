// rs_ff16_small.hip -- GF(2^16) kernels for small codes (m <= 256 encode,
// n <= 2048 decode) on narrow column strips, for gfx950.
//
// At 64 KiB pieces a 512-byte column strip per workgroup (the layout of
// rs_kernels.hip) gives 128 strips: too few workgroups to fill 256 CUs, so the
// small-code kernels there split the transform into slab passes and still leave
// SIMDs idle.  Here a workgroup owns a strip of LW units (LW < 64: 16 units =
// two 64-byte ALTMAP blocks = 128 bytes of every piece), and the 64 lanes of a
// wave form 64 / LW lane groups that hold DIFFERENT pieces of the tile (Tile
// LW, rs_device.h: the "virtual wave" index carries the lane-group bits).  So a
// 64 KiB call is 512 workgroups, each running its whole transform:
//   * butterfly tables are staged per workgroup in LDS (Tabs16Stage) and read
//     at a per-lane address (a lane group's pieces sit in different butterfly
//     groups: same ds_read_b128 count as a wave-uniform read);
//   * piece pointers are per lane group (vector address arithmetic).
//
// Encoder (ReedSolomonEncode, LeopardFF16.cpp:1397-1467):
//   work = XOR_c IFFT_m(data chunk c, skew base m - 1 + c m);  out = FFT_m(work, skew base -1)[0, R)
// as one workgroup per strip looping over the chunks, the next chunk's pieces
// loaded while the current chunk's IFFT runs; the top
// IFFT layer of every chunk and the top FFT layer run as one fused butterfly
// (Tile::fused_top, as rs_ff8.hip).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "rs_args.h"

namespace lamd {

#ifdef LAMD_STAMPS
// Diagnostic builds only (tools/build_variant.sh ... -DLAMD_STAMPS): per-wave
// s_memrealtime stamps at phase boundaries, without draining memory
// operations (the prefetch overlap stays as it is).
__device__ uint64_t* g_stamps16;
#define STAMP16(k)                                                                                        \
    do {                                                                                                 \
        const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                            \
        if ((threadIdx.x & 63) == 0)                                                                     \
            g_stamps16[kStampBase + ((uint64_t(blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (k)] = t_; \
    } while (0)
#else
#define STAMP16(k) \
    do {           \
    } while (0)
#endif

namespace {

// Units (8 bytes: 4 ALTMAP elements) of a lane: q = strip * LW + lane; byte
// offset of unit q inside a piece (unit_offset<FF16>).
template <int LW>
struct NarrowCols {
    uint64_t off;  // byte offset of this lane's unit (lanes past the end: the last unit)
    bool live;
};
template <int LW>
LDEV NarrowCols<LW> narrow_cols(uint64_t nunits, unsigned lane, uint64_t strip = blockIdx.x) {
    const uint64_t q = strip * LW + lane;
    const uint64_t ql = q < nunits ? q : nunits - 1;
    return NarrowCols<LW>{unit_offset<FF16>(ql), q < nunits};
}

// Addresses of the pieces idx(r), r < NR, of a caller's map at per-lane
// indices: one wave-uniform table-or-slab decision, every table entry read
// before any piece load is issued (a table read in front of each piece load
// would make each wait for all earlier loads: vmcnt retires in order).
template <int NR, class Idx>
LDEV void lane_ptrs(uint64_t (&pp)[NR], const PieceMap& pm, Idx idx) {
    if (pm.table) {
#pragma unroll
        for (int r = 0; r < NR; ++r) pp[r] = pm.table[idx(r)];
    } else {
#pragma unroll
        for (int r = 0; r < NR; ++r) pp[r] = uint64_t(reinterpret_cast<uintptr_t>(pm.base)) + uint64_t(idx(r)) * pm.stride;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) pp[r] += pm.off;
}
LDEV void ld_unit(uint32_t* x, const uint8_t* piece, uint64_t off) {
    if constexpr ((LAMD_ABLATE & 4) != 0) {  // ablation builds: no piece loads
        x[0] = uint32_t(off) * 2654435761u + uint32_t(uintptr_t(piece));
        x[1] = x[0] ^ 0x5bd1e995u;
        return;
    }
    x[0] = gld<uint32_t>(piece + off);
    x[1] = gld<uint32_t>(piece + off + 32);
}
LDEV void st_unit(uint8_t* piece, uint64_t off, const uint32_t* x) {
    if constexpr ((LAMD_ABLATE & 8) != 0) {  // ablation builds: no piece stores (x kept live)
        if ((x[0] ^ x[1]) == 0x9E3779B9u && off == 0x7FFFFFFFull) *gptr<uint32_t>(piece) = x[0];
        return;
    }
    gst<uint32_t>(piece + off, x[0]);
    gst<uint32_t>(piece + off + 32, x[1]);
}

constexpr int lg2(unsigned v) { return v <= 1 ? 0 : 1 + lg2(v >> 1); }
constexpr int lg_bits(int LW) { return LW == 64 ? 0 : LW == 32 ? 1 : LW == 16 ? 2 : 3; }
template <int T, int R, int LW>
constexpr unsigned threads_n() { return 64u << (T - R - lg_bits(LW)); }

// ------------------------------------------------------------- LDS-DMA --

// 16 bytes per lane from src (per lane) to dst + 16 * lane (dst wave-uniform)
LDEV void dma16(const uint32_t* src, uint32_t* dst) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src),
                                     (__attribute__((address_space(3))) void*)(dst), 16, 0, 0);
#endif
}
LDEV void wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// 16-byte unit u of a table set laid out by tab16_slot (slot s at 5 s + (s >> 3)
// + (s >> 6) units): its slot and its unit inside the slot, or slot ~0u for a
// padding unit.
LDEV unsigned unit_slot(unsigned u, unsigned& k) {
    const unsigned b = u / 329u, r = u - b * 329u;
    const unsigned g = r / 41u, r2 = r - g * 41u;
    if (r == 328u || r2 == 40u) {
        k = 0;
        return ~0u;
    }
    const unsigned i = r2 / 5u;
    k = r2 - i * 5u;
    return 64u * b + 8u * g + i;
}
constexpr unsigned kSetUnits = unsigned(tab16_set_dwords(8) / 4);  // = tab16_slot(256) / 4
static_assert(tab16_slot(256) / 4 == kSetUnits, "skew and log sets have the same footprint");
// The skew set of entries base + s, slot s in [1, 2^T) (Tabs16Stage::load(sktab,
// base, 0, 0)'s entries) by LDS-DMA.  (lane is made opaque: the unit -> slot
// arithmetic is redone at each use instead of being hoisted out of the tile
// loops and kept live.)
template <int NW, int T>
LDEV void dma_skew_set_at(uint32_t* set, const uint32_t* sktab, int base, unsigned wave, unsigned lane) {
    constexpr unsigned kUnits = unsigned(tab16_set_dwords(T) / 4);
    asm volatile("" : "+v"(lane));
    for (unsigned c = wave; c * 64u < kUnits; c += NW) {
        const unsigned u = c * 64u + lane;
        unsigned k;
        unsigned sl = unit_slot(u, k);
        if (sl == ~0u || sl == 0u || sl >= (1u << T)) sl = 1u;  // padding and the unused slot 0: any valid entry
        if (u < kUnits) dma16(sktab + size_t(int64_t(base) + sl) * 24u + k * 4u, set + c * 256u);
    }
}
// skew set of tile hi_fixed >> 8 at skew base -1 (the decoder's)
template <int NW>
LDEV void dma_skew_set(uint32_t* set, const uint32_t* sktab, unsigned hi_fixed, unsigned wave, unsigned lane) {
    dma_skew_set_at<NW, 8>(set, sktab, int(hi_fixed) - 1, wave, lane);
}

// ------------------------------------------------------------------ encode --

#ifndef LAMD_ENC16N_DMA  // 1: the next stage's skew set by LDS-DMA during the current chunk's IFFT (measured slower: 54.7 vs 52.3 us at 1000+200 x 64 KiB, r04_v19)
#define LAMD_ENC16N_DMA 0
#endif
constexpr bool kEncDma = LAMD_ENC16N_DMA;

template <int T, int R, int LW>
LDEV void enc16n_body(const EncArgs& a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    constexpr int G = lg_bits(LW);
    static_assert(T - R - G >= 0, "at least one wave");
    using TL = Tile<FF16, T, R, 1, LW, 0, G>;
    constexpr unsigned NT = threads_n<T, R, LW>();
    constexpr unsigned m = 1u << T;
    constexpr size_t kSet = tab16_set_dwords(T);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    auto set_of = [&](unsigned k) { return lds + TL::kXchDwords + (k & 1u) * kSet; };  // two table sets
    const unsigned wave = uniform(threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & (LW - 1);
    // virtual wave index: the lane group in its low bits.  In layout 0 the lane
    // groups then hold tile bits R, R + 1 and in every later layout bits 0, 1:
    // below every layer of those layouts, so their butterfly tables are the
    // same for all lane groups (a layer on bit l uses the skew of the bits
    // above l); only the layers of layout 0 read per-lane-group tables.
    const unsigned w = (wave << G) | ((threadIdx.x & 63u) >> (6 - G));
    const NarrowCols<LW> cl = narrow_cols<LW>(a.nunits, lane);
    const PieceSpace ps{0, 0, 0};
    typename TL::Reg x, nx, acc;
    // chunk c's pieces base + tp (tp = tile piece of register r in layout 0).
    // Branch-free: a piece past K re-reads piece K - 1 and is dropped at use
    // (take_chunk), as the zero padding of the last chunk (LeopardFF16.cpp:1446-1448).
    auto piece_of = [&](unsigned c, int r) { return c * m + TL::piece(0, r, w); };
    auto load_chunk = [&](typename TL::Reg& dst, unsigned c, auto&& between) {
        uint64_t pp[TL::NR];
        lane_ptrs(pp, a.in, [&](int r) { return min(piece_of(c, r), a.K - 1); });
        between();  // issued after the table reads, before the piece loads
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) ld_unit(dst[r], reinterpret_cast<const uint8_t*>(pp[r]), cl.off);
    };
    auto take_chunk = [&](typename TL::Reg& dst, const typename TL::Reg& src, unsigned c) {
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const bool ok = piece_of(c, r) < a.K;
#pragma unroll
            for (int k = 0; k < TL::U; ++k) dst[r][k] = ok ? src[r][k] : 0u;
        }
    };
    [[maybe_unused]] constexpr uint64_t kStampBase = 0;
    STAMP16(0);
    {
        Tabs16Stage<NT, T> st;
        load_chunk(nx, 0, [&] { st.load(a.sktab, int(m - 1), 0, 0); });  // chunk 0's IFFT skews
        st.store(set_of(0));
        take_chunk(x, nx, 0);
        __syncthreads();
    }
    STAMP16(1);
    TL::zero(acc);
    for (unsigned c = 0;;) {
        const bool more = c + 1 < a.nchunks;
        if (more)  // next chunk's pieces in flight during this chunk's transform
            load_chunk(nx, c + 1, [] {});
        if constexpr (kEncDma) {
            // the next stage's skew set (chunk c + 1's IFFT, or the FFT's) by LDS-DMA
            // into the set chunk c - 1 used (every wave is past that IFFT: the
            // barrier above), landing during this chunk's IFFT
            dma_skew_set_at<int(NT / 64), T>(set_of(c + 1), a.sktab, more ? int(m - 1 + (c + 1) * m) : -1, wave,
                                             threadIdx.x & 63u);
        }
        // an opaque copy of w per chunk: the per-lane table addresses are
        // recomputed in each chunk instead of being hoisted and kept live
        unsigned wc = w;
        asm volatile("" : "+v"(wc));
        TL::template ifft<true>(x, wc, lane, lds, ps, LdsWindow16{set_of(c), 0, 0}, AllLive{});
        TL::fused_top(x, FF16::tab(a.tabs, cload(a.fused + c)));
        TL::xor_into(acc, x);
        STAMP16(2 + (c < 3 ? c : 3));
        if (!more) break;
        ++c;
        if constexpr (!kEncDma) {
            // its tables (L2-resident after the first workgroups: a short wait),
            // into the set chunk c - 2 used (read before the previous barrier)
            Tabs16Stage<NT, T> st;
            st.load(a.sktab, int(m - 1 + c * m), 0, 0);
            st.store(set_of(c));
        }
        take_chunk(x, nx, c);
        if constexpr (kEncDma) wait_dma();
        __syncthreads();
    }
    {
        // FFT tables (skew base -1) into the set the last chunk did not use
        uint32_t* fset = set_of(a.nchunks);
        if constexpr (kEncDma) {
            wait_dma();
        } else {
            Tabs16Stage<NT, T> st;
            st.load(a.sktab, -1, 0, 0);
            st.store(fset);
        }
        __syncthreads();
        TL::template fft<true>(acc, w, lane, lds, ps, LdsWindow16Static<-1, 0>{{fset, 0, 0}}, AllLive{});
    }
    TL::pin(acc);
    STAMP16(6);
    uint64_t pp[TL::NR];
    lane_ptrs(pp, a.out, [&](int r) { return min(TL::piece(0, r, w), a.R - 1); });
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r)
        if (TL::piece(0, r, w) < a.R) st_unit(reinterpret_cast<uint8_t*>(pp[r]), cl.off, acc[r]);
    STAMP16(7);
}

template <int T, int R, int LW>
__global__ void __launch_bounds__((threads_n<T, R, LW>()), 4) k_enc16n(EncArgs a) {
    enc16n_body<T, R, LW>(a);
}
// Batched launch (leo_amd_encode_batch): object blockIdx.y of an array of
// argument blocks in device memory, one grid over every object's strips.
template <int T, int R, int LW>
__global__ void __launch_bounds__((threads_n<T, R, LW>()), 4) k_enc16n_batch(const EncArgs* __restrict__ objs) {
    enc16n_body<T, R, LW>(objs[blockIdx.y]);
}

// Chunk-parallel form of enc16n_body for single calls on few column strips
// (2560-byte pieces: 20 strips of 128 bytes, so the one-kernel form runs 20
// workgroups, each taking its K / m chunks one after the other).  Pass 1, grid
// (strips, chunks): chunk c = blockIdx.y's IFFT and fused top layer (one
// iteration of enc16n_body's chunk loop) into the slab rows c m + slot(r, w);
// pass 2, grid (strips): the XOR of every chunk's rows (TL::xor_into, by
// linearity as in enc16n_body), the FFT, the R outputs.  slot(r, w) = r 2^(T-R)
// + w enumerates the m (register, virtual wave) pairs; both passes use it, so
// the layout the IFFT ends in need not be named.
template <int T, int R, int LW>
LDEV unsigned enc16n_slot(int r, unsigned w) {
    return unsigned(r) * (1u << (T - R)) + w;
}
template <int T, int R, int LW>
__global__ void __launch_bounds__((threads_n<T, R, LW>()), 4) k_enc16n_part(EncArgs a) {
    constexpr int G = lg_bits(LW);
    using TL = Tile<FF16, T, R, 1, LW, 0, G>;
    constexpr unsigned NT = threads_n<T, R, LW>();
    constexpr unsigned m = 1u << T;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const unsigned wave = uniform(threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & (LW - 1);
    const unsigned w = (wave << G) | ((threadIdx.x & 63u) >> (6 - G));
    const unsigned c = blockIdx.y;
    const NarrowCols<LW> cl = narrow_cols<LW>(a.nunits, lane);
    const PieceSpace ps{0, 0, 0};
    uint32_t* const set = lds + TL::kXchDwords;
    typename TL::Reg x;
    {
        uint64_t pp[TL::NR];
        lane_ptrs(pp, a.in, [&](int r) { return min(c * m + TL::piece(0, r, w), a.K - 1); });
        Tabs16Stage<NT, T> st;
        st.load(a.sktab, int(m - 1 + c * m), 0, 0);  // chunk c's IFFT skews
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) ld_unit(x[r], reinterpret_cast<const uint8_t*>(pp[r]), cl.off);
        st.store(set);
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {  // the last chunk's zero padding (LeopardFF16.cpp:1446-1448)
            const bool ok = c * m + TL::piece(0, r, w) < a.K;
#pragma unroll
            for (int k = 0; k < TL::U; ++k) x[r][k] = ok ? x[r][k] : 0u;
        }
        __syncthreads();
    }
    TL::template ifft<true>(x, w, lane, lds, ps, LdsWindow16{set, 0, 0}, AllLive{});
    TL::fused_top(x, FF16::tab(a.tabs, cload(a.fused + c)));
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) st_unit(a.slab_out.slab_ptr(c * m + enc16n_slot<T, R, LW>(r, w)), cl.off, x[r]);
}
template <int T, int R, int LW>
__global__ void __launch_bounds__((threads_n<T, R, LW>()), 4) k_enc16n_comb(EncArgs a) {
    constexpr int G = lg_bits(LW);
    using TL = Tile<FF16, T, R, 1, LW, 0, G>;
    constexpr unsigned NT = threads_n<T, R, LW>();
    constexpr unsigned m = 1u << T;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const unsigned wave = uniform(threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & (LW - 1);
    const unsigned w = (wave << G) | ((threadIdx.x & 63u) >> (6 - G));
    const NarrowCols<LW> cl = narrow_cols<LW>(a.nunits, lane);
    const PieceSpace ps{0, 0, 0};
    uint32_t* const set = lds + TL::kXchDwords;
    Tabs16Stage<NT, T> st;
    st.load(a.sktab, -1, 0, 0);  // FFT skews (base -1)
    typename TL::Reg acc, x;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) ld_unit(acc[r], a.slab_in.slab_ptr(enc16n_slot<T, R, LW>(r, w)), cl.off);
    for (unsigned c = 1; c < a.nchunks; ++c) {
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) ld_unit(x[r], a.slab_in.slab_ptr(c * m + enc16n_slot<T, R, LW>(r, w)), cl.off);
        TL::xor_into(acc, x);
    }
    st.store(set);
    __syncthreads();
    TL::template fft<true>(acc, w, lane, lds, ps, LdsWindow16Static<-1, 0>{{set, 0, 0}}, AllLive{});
    TL::pin(acc);
    uint64_t pp[TL::NR];
    lane_ptrs(pp, a.out, [&](int r) { return min(TL::piece(0, r, w), a.R - 1); });
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r)
        if (TL::piece(0, r, w) < a.R) st_unit(reinterpret_cast<uint8_t*>(pp[r]), cl.off, acc[r]);
}

template <int T, int R, int LW>
hipError_t launch_enc16n(const EncArgs& a, hipStream_t s) {
    using TL = Tile<FF16, T, R, 1, LW, 0, lg_bits(LW)>;
    constexpr size_t lds = (TL::kXchDwords + 2 * tab16_set_dwords(T)) * 4;
    static_assert(lds <= (LW == 16 ? 80 : 160) * 1024, "two (16-unit strips) / one workgroup(s) per CU");
    static hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_enc16n<T, R, LW>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (attr != hipSuccess) return attr;
    void* params[] = {const_cast<EncArgs*>(&a)};
    const unsigned grid = unsigned((a.nunits + LW - 1) / LW);
    return hipLaunchKernel(reinterpret_cast<const void*>(&k_enc16n<T, R, LW>), dim3(grid), dim3(threads_n<T, R, LW>()),
                           params, lds, s);
}


// ------------------------------------------------------------------ decode --
//
// Decoder (ReedSolomonDecode, LeopardFF16.cpp:1652-1775) for n = 2^Tn <= 2048:
//   v = IFFT_n(el * received);  z = FormalDerivative(v);  lost i = FFT_n(z)[m + i] * exp(-el[m + i])
// Positions split into tiles of 256 (low 8 bits) and Tn - 8 high bits t:
//   F (I + D) I = F_lo ( Q + D_lo ) I_lo,    Q = F_hi (I + D_hi) I_hi
// (D_lo commutes with the high layers, F_hi I_hi = I: rs_kernels.hip header).
// Q acts on the tile index alone, the same for every low index; it is the
// XOR-convolution Q[t][t'] = q[t ^ t'] with q[0] = 0, q[1] = 1 (gf_tables.h:
// build_high_q16).  Hence two passes and one intermediate:
//   pass 1 (k_dec16n_lo):  U_t' = IFFT_lo^(t')( el * received tile t' )            -> slab
//   pass 2 (k_dec16n_fin): Z_t = XOR_t' q[t ^ t'] U_t'  ^  D_lo U_t,
//                          lost originals of tile t = FFT_lo^(t)(Z_t) * exp(-el)
// At 1000 + 200: 13 multiplies and 3 XORs per position for the high part (the
// 3-pass form: 14 multiplies, plus a slab written and read).

// bit j of level L of an occupancy pyramid (rs_args.h)
LDEV bool pyr_bit(const uint32_t* pyr, unsigned L, unsigned j) {
    return (cload(pyr + pyr_offset(L) + (j >> 5)) >> (j & 31)) & 1u;
}
constexpr uint32_t kQZero = 0xFFFFFFFFu, kQOne = 0xFFFFFFFEu;  // q entries that are 0 / 1 (else a log value)

template <int R, int LW>
LDEV void dec16n_lo_body(const DecArgs& a, const unsigned y) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    constexpr int T = 8, G = lg_bits(LW);
    using TL = Tile<FF16, T, R, 1, LW, 0, G>;
    constexpr unsigned NT = threads_n<T, R, LW>();
    if (!pyr_bit(a.present_pyr, T, y)) return;  // nothing received in this tile: U_y = 0, pass 2 skips it
    [[maybe_unused]] constexpr uint64_t kStampBase = 0;
    STAMP16(0);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* set = lds + TL::kXchDwords;
    uint32_t* scl = lds;  // the scale tables share the exchange area: used before the first transpose
    const unsigned wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & (LW - 1);
    const unsigned w = (wave << G) | ((threadIdx.x & 63u) >> (6 - G));
    const NarrowCols<LW> cl = narrow_cols<LW>(a.nunits, lane);
    const PieceSpace ps{0, 0, y << T};
    // erasure bits of this lane's pieces: in layout 0 a lane holds NR
    // consecutive positions (tile piece r | w << R), all in one bitmap word
    const uint32_t ew = a.erased_dev[(y << 3) + (w >> (5 - R))];
    Tabs16Stage<NT, T> st;
    LogTabs16Stage<NT, (1u << T)> ls;
    st.load(a.sktab, -1, y << T, 0);
    ls.load(a.tabs, a.scale_logs + (y << T));
    typename TL::Reg x;
    {
        // received pieces: positions [0, R) recovery, [m, m + K) originals
        // (LeopardFF16.cpp:1715-1730); absent ones read the zero page
        auto pos = [&](int r) { return (y << T) + TL::piece(0, r, w); };
        uint64_t pr[TL::NR], po[TL::NR];
        lane_ptrs(pr, a.rec, [&](int r) { return min(pos(r), a.R - 1); });
        lane_ptrs(po, a.orig, [&](int r) { return pos(r) >= a.m ? min(pos(r) - a.m, a.K - 1) : 0u; });
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const unsigned p = pos(r), tp = TL::piece(0, r, w);
            const bool got = !((ew >> (tp & 31)) & 1u) && (p < a.R || (p >= a.m && p < a.m + a.K));
            const uint8_t* src = got ? reinterpret_cast<const uint8_t*>(p < a.R ? pr[r] : po[r]) : a.zeros;
            ld_unit(x[r], src, got ? cl.off : (cl.off & 31));
        }
    }
    st.store(set);
    ls.store(scl);
    __syncthreads();
    STAMP16(1);
    // scale by exp(el[p]) (the zero table for absent positions)
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        asm volatile("" ::: "memory");  // one table live at a time
        const FF16::Tab t = FF16::tab_lds(scl + tab16_slot(TL::piece(0, r, w)));
        FF16::mul(x[r], x[r], t);
#pragma unroll
        for (int k = 0; k < TL::U; ++k) asm volatile("" : "+v"(x[r][k]));
    }
    STAMP16(2);
    TL::ifft(x, w, lane, lds, ps, LdsWindow16{set, y << T, 0}, AllLive{});
    STAMP16(3);
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const uint64_t row = ps.global(TL::piece(TL::kLast, r, w));
        st_unit(a.a_out.base + row * a.a_out.stride + a.a_out.off, cl.off, x[r]);
    }
    STAMP16(4);
}

template <int R, int LW>
__global__ void __launch_bounds__((threads_n<8, R, LW>()), 4) k_dec16n_lo(DecArgs a) {
    dec16n_lo_body<R, LW>(a, blockIdx.y);
}
// batched: tile blockIdx.y of object blockIdx.z (argument blocks in device memory)
template <int R, int LW>
__global__ void __launch_bounds__((threads_n<8, R, LW>()), 4) k_dec16n_lo_batch(const DecArgs* __restrict__ objs) {
    dec16n_lo_body<R, LW>(objs[blockIdx.z], blockIdx.y);
}

// Pass 2 over NZ consecutive output tiles per workgroup: every U tile is read
// once for all of them and its perm selectors are formed once for all of their
// multiplies.  NZ = 2 measured slower than 1 (its registers allow one
// workgroup per CU instead of two: 1000+200 x 64 KiB decode 203 vs 181 us,
// profiles/r03_v4/dec_nz_ab.txt), so the default is 1.  Prefetching U two
// tiles ahead instead of one measured equal (179 vs 180 us) and was dropped.
#ifndef LAMD_DEC16N_NZ  // output tiles per pass-2 workgroup (2 measured slower: occupancy, r03_v4)
#define LAMD_DEC16N_NZ 1
#endif
#ifndef LAMD_DEC16N_FIN_WAVES  // waves per SIMD the pass-2 register budget is cut for
#define LAMD_DEC16N_FIN_WAVES (LAMD_DEC16N_NZ > 1 ? 3 : 4)
#endif
template <int R, int LW, int NZ>
LDEV void dec16n_fin_body(const DecArgs& a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    constexpr int T = 8, G = lg_bits(LW);
    using TL = Tile<FF16, T, R, 1, LW, 0, G>;
    constexpr unsigned NT = threads_n<T, R, LW>();
    constexpr size_t kSet = tab16_set_dwords(T);
    // workgroup i runs on XCD i % 8: the workgroups of one strip (its groups of
    // output tiles) are dealt to one XCD back to back, so the U tiles they all
    // read come from that XCD's L2
    const unsigned ngrp = (a.nout + NZ - 1) / NZ;
    const unsigned j = blockIdx.x >> 3;
    const uint64_t strip = (blockIdx.x & 7u) + 8ull * (j / ngrp);
    if (strip * LW >= a.nunits) return;
    unsigned t[NZ];
    bool live[NZ];
    bool any = false;
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        t[k] = a.tile0 + (j % ngrp) * NZ + k;
        live[k] = t[k] < a.tile0 + a.nout && pyr_bit(a.needed_pyr, T, t[k]);  // tile holds a lost original
        any |= live[k];
    }
    if (!any) return;
    [[maybe_unused]] constexpr uint64_t kStampBase = 1ull << 22;
    STAMP16(0);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* rvl = lds;  // the reveal tables go to the exchange area once an FFT is done with it
    auto fset = [&](int k) { return lds + TL::kXchDwords + size_t(k) * kSet; };
    const unsigned wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & (LW - 1);
    const unsigned w = (wave << G) | ((threadIdx.x & 63u) >> (6 - G));
    const NarrowCols<LW> cl = narrow_cols<LW>(a.nunits, lane, strip);
    // U tile ut in layout kLast (the layout the low IFFT ended in and the FFT starts in)
    auto load_u = [&](typename TL::Reg& u, unsigned ut) {
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const uint64_t row = (ut << T) + TL::piece(TL::kLast, r, w);
            ld_unit(u[r], a.a_in.base + row * a.a_in.stride + a.a_in.off, cl.off);
        }
    };
    // the U tiles read: received data, and q[t ^ ut] != 0 or ut = t (D_lo) for a live output t
    auto wanted = [&](unsigned ut) {
        if (!(ut < a.nlo && pyr_bit(a.present_pyr, T, ut))) return false;
        bool want = false;
#pragma unroll
        for (int k = 0; k < NZ; ++k) want |= live[k] && (ut == t[k] || cload(a.qlog + (t[k] ^ ut)) != kQZero);
        return want;
    };
#pragma unroll
    for (int k = 0; k < NZ; ++k)
        if (live[k]) {
            Tabs16Stage<NT, T> st;
            st.load(a.sktab, -1, t[k] << T, 0);
            st.store(fset(k));
        }
    typename TL::Reg z[NZ], u, nu;
#pragma unroll
    for (int k = 0; k < NZ; ++k) TL::zero(z[k]);
    unsigned ut = 0;
    while (ut < a.nlo && !wanted(ut)) ++ut;
    if (ut < a.nlo) load_u(nu, ut);
    __syncthreads();
    STAMP16(1);
    while (ut < a.nlo) {
        TL::copy(u, nu);
        unsigned next = ut + 1;
        while (next < a.nlo && !wanted(next)) ++next;
        if (next < a.nlo) load_u(nu, next);  // in flight while this tile is folded in
        uint32_t q[NZ];
        unsigned mulmask = 0;
#pragma unroll
        for (int k = 0; k < NZ; ++k) {
            q[k] = live[k] && ut != t[k] ? cload(a.qlog + (t[k] ^ ut)) : kQZero;
            if (q[k] != kQZero && q[k] != kQOne) mulmask |= 1u << k;
        }
        // z_k ^= q_k * U for the outputs in the (wave-uniform) mask, one set of selectors per piece
        static_for<1, (1 << NZ)>([&](auto M) {
            constexpr unsigned mask = decltype(M)::value;
            if (mulmask == mask) {
                FF16::Tab tq[NZ];
                static_for<0, NZ>([&](auto K) {
                    if constexpr ((mask >> K.value) & 1u) tq[K.value] = FF16::tab(a.tabs, q[K.value]);
                });
#pragma unroll
                for (int r = 0; r < TL::NR; ++r) {
                    const FF16::Sel sl = FF16::sel(u[r]);
                    static_for<0, NZ>([&](auto K) {
                        if constexpr ((mask >> K.value) & 1u) FF16::muladd_sel(z[K.value][r], sl, tq[K.value]);
                    });
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        });
#pragma unroll
        for (int k = 0; k < NZ; ++k)
            if (q[k] == kQOne) TL::xor_into(z[k], u);
        // the formal derivative's low bits: D_lo U_t (rs_device.h derivative_add)
#pragma unroll
        for (int k = 0; k < NZ; ++k)
            if (live[k] && ut == t[k])
                TL::derivative_add(z[k], [&](int r, uint32_t* out) { out[0] = u[r][0]; out[1] = u[r][1]; }, w, lane,
                                   lds);
        ut = next;
    }
    STAMP16(2);
    static_for<0, NZ>([&](auto K) {
        constexpr int k = decltype(K)::value;
        if (!live[k]) return;
        const unsigned tk = t[k];
        LogTabs16Stage<NT, (1u << T)> ls;
        ls.load(a.tabs, a.reveal_logs + (tk << T));  // in flight during the FFT
        // (the FFT's first exchange starts with a barrier: the previous output's reveal is done with rvl)
        TL::fft(z[k], w, lane, lds, PieceSpace{0, 0, tk << T}, LdsWindow16{fset(k), tk << T, 0}, AllLive{});
        __syncthreads();  // every wave is past the FFT's last exchange
        STAMP16(3);
        ls.store(rvl);
        // lost original at p = m + i: work[i] = z[p] * exp(-el[p])  (LeopardFF16.cpp:1771-1773)
        auto pos = [&](int r) { return (tk << T) + TL::piece(0, r, w); };
        const uint32_t ew = a.erased_dev[(tk << 3) + (w >> (5 - R))];  // layout 0: one word a lane
        uint64_t po[TL::NR];
        lane_ptrs(po, a.out, [&](int r) { return pos(r) >= a.m ? min(pos(r) - a.m, a.K - 1) : 0u; });
        __syncthreads();
        if (cl.live) {
#pragma unroll
            for (int r = 0; r < TL::NR; ++r) {
                const unsigned p = pos(r), tp = TL::piece(0, r, w);
                if (p >= a.m && p < a.m + a.K && ((ew >> (tp & 31)) & 1u)) {
                    asm volatile("" ::: "memory");
                    uint32_t o[2];
                    FF16::mul(o, z[k][r], FF16::tab_lds(rvl + tab16_slot(tp)));
                    st_unit(reinterpret_cast<uint8_t*>(po[r]), cl.off, o);
                }
            }
        }
    });
    STAMP16(4);
}

// ------------------------------------------------------- one-pass decode --
//
// The same decoder in ONE pass per column strip (no U slab): a workgroup owns
// a strip of LW units of every position and walks the received tiles t' in
// order -- scale, low IFFT, and fold the result straight into the Z
// accumulators of every output tile, which stay in registers for the whole
// kernel -- then runs the low FFT and the reveal of each output tile:
//   for each received tile t':   U = IFFT_lo^(t')( el * received tile t' )
//                                Z_t ^= q[t ^ t'] U   (t != t'),   Z_t ^= D_lo U   (t = t')
//   for each output tile t:      lost originals of t = FFT_lo^(t)(Z_t) * exp(-el)
// (LeopardFF16.cpp:1652-1775; the split F (I + D) I = F_lo (Q + D_lo) I_lo as in
// the two-pass form above).  U is never written to memory: a call reads the
// received pieces once and writes the lost originals once.  NZ output tiles
// (tiles holding a lost original, [tile0, tile0 + nout)) are held per lane
// (NZ * 2^R * 2 dwords); calls with more use the two-pass form.
//
// Tables reach LDS by LDS-DMA (global_load_lds_dwordx4: no registers, no
// per-lane LDS stores): a tile's skew set (the decoder's IFFT and FFT of one
// tile use the same skew positions, base -1, LeopardFF16.cpp:1737, 1764) and
// its 256 scale / reveal tables, whose log values the workgroup keeps in LDS.
// Each tile boundary is one exposed wait (the DMA of the next tables and the
// next pieces' loads); two workgroups per CU cover each other's.

// the multiply tables of log values logs[0, 256) (global memory), slot p =
// position p.  The log values of all of this wave's units are read first and
// the DMAs issued after them: the wait for a log value then covers only the log
// reads (vmcnt retires in order), not DMAs issued before this call.
// sparse: only the slots whose log value is not the zero table's (the reveal
// multiplies of the lost originals); the other slots keep stale bytes and are
// never read.
template <int NW>
LDEV void dma_log_set(uint32_t* dst, const uint32_t* tabs, const uint32_t* logs, unsigned wave, unsigned lane,
                      bool sparse = false) {
    constexpr unsigned kChunks = (kSetUnits + 63) / 64, kPer = (kChunks + NW - 1) / NW;
    asm volatile("" : "+v"(lane));
    uint32_t lg[kPer];
#pragma unroll
    for (unsigned i = 0; i < kPer; ++i) {
        const unsigned u = (wave + i * NW) * 64u + lane;
        unsigned k;
        unsigned p = unit_slot(u < kSetUnits ? u : 0u, k);
        if (p == ~0u) p = 0u;
        lg[i] = logs[p];
    }
    asm volatile("" : "+v"(lane));  // the unit -> slot arithmetic redone below, not kept live
    // every source address before the first DMA: a wait for a log value after a
    // DMA has been issued would wait for that DMA too
    const uint32_t* src[kPer];
    bool go[kPer];
#pragma unroll
    for (unsigned i = 0; i < kPer; ++i) {
        const unsigned c = wave + i * NW, u = c * 64u + lane;
        unsigned k;
        unit_slot(u < kSetUnits ? u : 0u, k);
        src[i] = tabs + size_t(lg[i]) * 24u + k * 4u;
        go[i] = u < kSetUnits && !(sparse && lg[i] == FF16::kOrder);
        asm volatile("" : "+v"(src[i]));
    }
#pragma unroll
    for (unsigned i = 0; i < kPer; ++i) {
        const unsigned c = wave + i * NW;
        if (c < kChunks && go[i]) dma16(src[i], dst + c * 256u);
    }
}
// 4 bytes per lane from src (per lane) to dst + 4 * lane (dst wave-uniform)
LDEV void dma4(const uint32_t* src, uint32_t* dst) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src),
                                     (__attribute__((address_space(3))) void*)(dst), 4, 0, 0);
#endif
}

#ifndef LAMD_DEC16_ONE_WAVES  // waves per SIMD the one-pass decoder's register budget is cut for
#define LAMD_DEC16_ONE_WAVES 4
#endif
// LDS of the one-pass decoder (dwords): the exchange area (transposes; the image
// of the next received tile's pieces between them; the reveal tables), the skew
// set, the scale tables, the next tile's piece addresses
template <int R, int LW>
constexpr size_t one_xch_dwords() {
    constexpr size_t x = Tile<FF16, 8, R, 1, LW, 0, lg_bits(LW)>::kXchDwords;
    return x > tab16_slot(256) ? x : tab16_slot(256);
}
template <int R, int LW>
constexpr size_t one_lds_dwords() {
    return one_xch_dwords<R, LW>() + 2 * tab16_set_dwords(8) + 2 * 256;
}
template <int R, int LW, int NZ>
LDEV void dec16n_one(const DecArgs& a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    constexpr int T = 8, G = lg_bits(LW);
    using TL = Tile<FF16, T, R, 1, LW, 0, G>;
    constexpr unsigned NT = threads_n<T, R, LW>(), NW = NT / 64;
    constexpr size_t kSet = tab16_set_dwords(T);
    constexpr size_t kXch = one_xch_dwords<R, LW>();
    static_assert(LW <= 32 && TL::U == 2, "a DMA lane's unit half is the same in every instruction");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* xch = lds;                 // transposes; the next tile's piece image; the reveal tables
    uint32_t* set = lds + kXch;          // skew tables of the current transform
    uint32_t* stab = set + kSet;         // scale tables of the current received tile
    uint64_t* ptab = reinterpret_cast<uint64_t*>(stab + kSet);  // piece addresses of the next received tile
    const unsigned wave = uniform(threadIdx.x >> 6), lane64 = threadIdx.x & 63u, lane = threadIdx.x & (LW - 1);
    const unsigned w0 = (wave << G) | (lane64 >> (6 - G));
    const uint64_t strip = blockIdx.x;
    const NarrowCols<LW> cl = narrow_cols<LW>(a.nunits, lane, strip);
#ifdef LAMD_STAMPS  // 32 stamps per wave: 0 start, 1 first tile staged, per input tile i 2+3i (scale + IFFT), 3+3i (fold), 4+3i (next tile's wait), 26+k output tile k done
#define STAMP1(k)                                                                                              \
    do {                                                                                                      \
        const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                                 \
        if ((threadIdx.x & 63) == 0) g_stamps16[(2ull << 22) + (uint64_t(blockIdx.x) * NW + wave) * 32 + (k)] = t_; \
    } while (0)
#else
#define STAMP1(k) \
    do {          \
    } while (0)
#endif
    [[maybe_unused]] unsigned ti = 0;
    STAMP1(0);
    // output slots: tile tile0 + k holds a lost original
    unsigned live = 0;
#pragma unroll
    for (int k = 0; k < NZ; ++k)
        if (unsigned(k) < a.nout && pyr_bit(a.needed_pyr, T, a.tile0 + k)) live |= 1u << k;
    // received tiles
    unsigned have = 0;
    for (unsigned y = 0; y < a.nlo; ++y)
        if (pyr_bit(a.present_pyr, T, y)) have |= 1u << y;
    auto next_have = [&](unsigned y) {  // first received tile after y (a.nlo: none)
        const unsigned rest = have & ~((2u << y) - 1u);
        return rest ? unsigned(__builtin_ctz(rest)) : a.nlo;
    };

    // Received pieces of tile yt: positions [0, R) recovery, [m, m + K)
    // originals (LeopardFF16.cpp:1715-1730); 0 = absent (read the zero page).
    // (Addressing slab maps directly in front of each DMA instead, a scalar
    // erasure-word load and a 64-bit multiply per instruction, measured slower:
    // 1000+200 x 64 KiB decode 190 vs 164 us, profiles/r04_v10.)
    auto build_ptab = [&](unsigned yt) {
        for (unsigned tp = threadIdx.x; tp < 256u; tp += NT) {
            const unsigned p = (yt << T) + tp;
            const bool is_rec = p < a.R, is_orig = p >= a.m && p < a.m + a.K;
            const PieceMap& pm = is_rec ? a.rec : a.orig;
            const unsigned idx = is_rec ? p : (is_orig ? p - a.m : 0u);
            // both loads issued before either is used (one latency, not two)
            const uint32_t ew = a.erased_dev[(yt << 3) + (tp >> 5)];
            const uint64_t b = pm.table ? pm.table[idx] : uint64_t(reinterpret_cast<uintptr_t>(pm.base)) + uint64_t(idx) * pm.stride;
            const bool got = !((ew >> (tp & 31u)) & 1u) && (is_rec || is_orig);
            ptab[tp] = got ? b + pm.off : 0ull;
        }
    };
    // The pieces of the tile in ptab into xch by 16-byte LDS-DMA.  Each wave
    // fetches exactly what its own lanes hold in layout 0 (tile pieces
    // r | vw << R of its NG virtual waves vw = NG wave + g), so a wave's own
    // vmcnt covers its reads.  Instruction q of wave W fills 1 KiB: 16-byte slot
    // i = 32 rho + 16 h + KP g + k' holds chunk k = 4 (k' >> 1) + (k' & 1) + 2 h
    // (16 bytes: the low (h = 0) or high (h = 1) bytes of 4 units of 64-byte
    // block k' >> 1) of tile piece (2 q + rho) | (NG W + g) << R.  A read of one
    // register's low (or high) dwords then touches 16 distinct 16-byte bank
    // groups: conflict-free.
    constexpr unsigned NG = 64u / LW, KP = LW / 4u;  // lane groups; low-byte chunks of a strip
    static_assert((LW == 16 || LW == 32) && R == 3 && NG * KP == 16, "16- or 32-unit strips, 8 pieces a lane");
    auto dma_pieces = [&] {
        // a last strip of fewer 64-byte blocks re-reads its last block for the
        // missing ones; those units are never stored
        const unsigned nblk = unsigned(min(uint64_t(LW / 8u), (a.nunits - strip * LW) / 8u));
        const uint64_t sbase = uint64_t(unit_offset<FF16>(strip * LW));
        unsigned ln = lane64;
        asm volatile("" : "+v"(ln));
        const unsigned rho = ln >> 5, h = (ln >> 4) & 1u, g = (ln & 15u) / KP, kp = (ln & 15u) % KP;
        const unsigned blk = min(kp >> 1, nblk - 1u);
        const unsigned k = 4u * blk + (kp & 1u) + 2u * h;
#pragma unroll
        for (unsigned q = 0; q < 4; ++q) {
            const uint64_t base = ptab[(2u * q + rho) | ((wave * NG + g) << R)];
            const uint8_t* src = base ? reinterpret_cast<const uint8_t*>(base) + sbase + 16u * k : a.zeros + 16u * k;
            dma16(reinterpret_cast<const uint32_t*>(src), xch + (wave * 4u + q) * 256u);
        }
    };
    auto read_pieces = [&](typename TL::Reg& x, unsigned w) {
        (void)w;
        const unsigned g = lane64 / LW, l = lane64 % LW;
        const unsigned kp = 2u * (l >> 3) + ((l >> 2) & 1u);
        const uint32_t* base = xch + wave * 1024u + (g * KP + kp) * 4u + (l & 3u);
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const uint32_t* p = base + (r >> 1) * 256 + (r & 1) * 128;
            x[r][0] = p[0];   // h = 0
            x[r][1] = p[64];  // h = 1: 16 slots on
        }
    };

    typename TL::Reg z[NZ], x;
    // first received tile: piece image, skew set and scale tables, one wait
    unsigned y = have ? unsigned(__builtin_ctz(have)) : a.nlo;
    if (y < a.nlo) {
        build_ptab(y);
        __syncthreads();
        dma_log_set<NW>(stab, a.tabs, a.scale_logs + (y << T), wave, lane64);
        dma_skew_set<NW>(set, a.sktab, y << T, wave, lane64);
        dma_pieces();
        wait_dma();
        __syncthreads();
        read_pieces(x, w0);
        const unsigned yn = next_have(y);
        if (yn < a.nlo) build_ptab(yn);  // (every wave's DMAs are issued: ptab is free)
    } else if (live) {
        dma_skew_set<NW>(set, a.sktab, (a.tile0 + unsigned(__builtin_ctz(live))) << T, wave, lane64);
        wait_dma();
        __syncthreads();
    }
    __builtin_amdgcn_sched_barrier(0);  // the accumulators start here, not across the first staging
#pragma unroll
    for (int k = 0; k < NZ; ++k) TL::zero(z[k]);
    STAMP1(1);
    while (y < a.nlo) {
        // an opaque copy of the lane's virtual wave per tile: the per-lane LDS
        // and table addresses derived from it are recomputed in each tile
        // instead of being hoisted out of the loop and kept live (k_enc16n)
        unsigned w = w0;
        asm volatile("" : "+v"(w));
        // scale by exp(el[p]) (the zero table for absent positions)
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            asm volatile("" ::: "memory");  // one table live at a time
            const FF16::Tab t = FF16::tab_lds(stab + tab16_slot(TL::piece(0, r, w)));
            FF16::mul(x[r], x[r], t);
#pragma unroll
            for (int k = 0; k < TL::U; ++k) asm volatile("" : "+v"(x[r][k]));
        }
        TL::ifft(x, w, lane, xch, PieceSpace{0, 0, y << T}, LdsWindow16{set, y << T, 0}, AllLive{});
        const unsigned ynext = next_have(y);
        const unsigned sknext = ynext < a.nlo ? ynext : live ? a.tile0 + unsigned(__builtin_ctz(live)) : ~0u;
        STAMP1(2 + 3 * ti);
        // every wave is past the IFFT: set, stab and xch are free.  The next
        // phase's tables go out now, its pieces once the derivative is done with
        // xch; all of them land during the fold.
        __syncthreads();
        // (Staging them through registers at the tile boundary instead spills 22
        // VGPRs next to the accumulators.)
        if (ynext < a.nlo) dma_log_set<NW>(stab, a.tabs, a.scale_logs + (ynext << T), wave, lane64);
        if (sknext != ~0u) dma_skew_set<NW>(set, a.sktab, sknext << T, wave, lane64);
        asm volatile("" : "+v"(w));  // the fold's addresses: recomputed, not kept from the IFFT
        // the formal derivative's low bits: D_lo U_t for t = y (rs_device.h derivative_add)
        static_for<0, NZ>([&](auto K) {
            constexpr int k = decltype(K)::value;
            if (((live >> k) & 1u) && a.tile0 + k == y) {
                unsigned wd = w;
                asm volatile("" : "+v"(wd));
                TL::derivative_add(z[k], [&](int r, uint32_t* out) { out[0] = x[r][0]; out[1] = x[r][1]; }, wd, lane,
                                   xch);
            }
        });
        if (ynext < a.nlo) {
            __syncthreads();  // every wave is done with xch
            dma_pieces();
        }
        // fold U = x into the other output tiles (every branch is workgroup-uniform)
        static_for<0, NZ>([&](auto K) {
            constexpr int k = decltype(K)::value;
            if (!((live >> k) & 1u)) return;
            const unsigned t = a.tile0 + k;
            if (t == y) return;
            const uint32_t q = cload(a.qlog + (t ^ y));
            if (q == kQZero) return;
            if (q == kQOne) {
                TL::xor_into(z[k], x);
                return;
            }
            // the multiplier's table through the scalar cache (wave-uniform): SGPRs, of
            // which v_perm takes one per instruction, so only one dword of each
            // table pair occupies a VGPR (the LDS copy would hold all 20 in VGPRs
            // next to the 64 accumulator and 16 tile registers)
            const FF16::Tab tq = FF16::tab(a.tabs, q);
#pragma unroll
            for (int r = 0; r < TL::NR; ++r) {
                FF16::muladd(z[k][r], x[r], tq);
                asm volatile("" : "+v"(z[k][r][0]), "+v"(z[k][r][1]));
                __builtin_amdgcn_sched_barrier(0);  // one multiply-add in flight: the table and 80 accumulators are live
            }
        });
        STAMP1(3 + 3 * ti);
        // next received tile: its pieces, scale tables and skew set have landed
        y = ynext;
        wait_dma();
        __syncthreads();
        if (y < a.nlo) {
            read_pieces(x, w);
            const unsigned yn = next_have(y);
            if (yn < a.nlo) build_ptab(yn);  // visible to the DMAs after the IFFT's barriers
        }
        STAMP1(4 + 3 * ti);
        ++ti;
    }
    // output tiles: low FFT, reveal, store the lost originals
    static_for<0, NZ>([&](auto K) {
        constexpr int k = decltype(K)::value;
        if (!((live >> k) & 1u)) return;
        const unsigned tk = a.tile0 + k;
        unsigned w = w0;  // opaque per output tile, as in the tile loop
        asm volatile("" : "+v"(w));
        // the reveal tables of the lost originals (the others are never read),
        // landing during the FFT (stab is free once every wave is past the
        // previous reveal)
        __syncthreads();
        dma_log_set<NW>(stab, a.tabs, a.reveal_logs + (tk << T), wave, lane64, true);
        TL::fft(z[k], w, lane, xch, PieceSpace{0, 0, tk << T}, LdsWindow16{set, tk << T, 0}, AllLive{});
        __syncthreads();  // every wave is past the FFT's last exchange and its last table read
        // the next output tile's skew set
        const unsigned rest = live & ~((2u << k) - 1u);
        if (rest) dma_skew_set<NW>(set, a.sktab, (a.tile0 + unsigned(__builtin_ctz(rest))) << T, wave, lane64);
        // lost original at p = m + i: work[i] = z[p] * exp(-el[p])  (LeopardFF16.cpp:1771-1773)
        auto pos = [&](int r) { return (tk << T) + TL::piece(0, r, w); };
        const uint32_t ew = a.erased_dev[(tk << 3) + (w >> (5 - R))];  // layout 0: one word a lane
        uint64_t po[TL::NR];
        lane_ptrs(po, a.out, [&](int r) { return pos(r) >= a.m ? min(pos(r) - a.m, a.K - 1) : 0u; });
        wait_dma();
        __syncthreads();
        if (cl.live) {
#pragma unroll
            for (int r = 0; r < TL::NR; ++r) {
                const unsigned p = pos(r), tp = TL::piece(0, r, w);
                if (p >= a.m && p < a.m + a.K && ((ew >> (tp & 31)) & 1u)) {
                    asm volatile("" ::: "memory");
                    uint32_t o[2];
                    FF16::mul(o, z[k][r], FF16::tab_lds(stab + tab16_slot(tp)));
                    st_unit(reinterpret_cast<uint8_t*>(po[r]), cl.off, o);
                }
            }
        }
        STAMP1(26 + k);
    });
}
#undef STAMP1

template <int R, int LW, int NZ>
__global__ void __launch_bounds__((threads_n<8, R, LW>()), LAMD_DEC16_ONE_WAVES) k_dec16n_one(DecArgs a) {
    dec16n_one<R, LW, NZ>(a);
}
// Batches (round 5): object blockIdx.y of an array of argument blocks in device
// memory (read through the scalar cache like the kernel arguments), each with
// its own decoder-state slot -- no U slab for batches either.
template <int R, int LW, int NZ>
__global__ void __launch_bounds__((threads_n<8, R, LW>()), LAMD_DEC16_ONE_WAVES)
k_dec16n_one_batch(const DecArgs* __restrict__ objs) {
    dec16n_one<R, LW, NZ>(objs[blockIdx.y]);
}

template <int R, int LW, int NZ>
__global__ void __launch_bounds__((threads_n<8, R, LW>()), LAMD_DEC16N_FIN_WAVES) k_dec16n_fin(DecArgs a) {
    dec16n_fin_body<R, LW, NZ>(a);
}
// batched: object blockIdx.y
template <int R, int LW, int NZ>
__global__ void __launch_bounds__((threads_n<8, R, LW>()), LAMD_DEC16N_FIN_WAVES)
    k_dec16n_fin_batch(const DecArgs* __restrict__ objs) {
    dec16n_fin_body<R, LW, NZ>(objs[blockIdx.y]);
}

template <class Kern>
hipError_t launch16n(Kern* fn, dim3 grid, unsigned threads, size_t lds_bytes, const DecArgs& a, hipStream_t s) {
    const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_bytes));
    if (attr != hipSuccess) return attr;
    void* params[] = {const_cast<DecArgs*>(&a)};
    return hipLaunchKernel(reinterpret_cast<const void*>(fn), grid, dim3(threads), params, lds_bytes, s);
}

#ifndef LAMD_DEC16N_R  // registers bits of the narrow decoder tiles (experiment builds: 2)
#define LAMD_DEC16N_R 3
#endif
constexpr int kDecR = LAMD_DEC16N_R, kDecLW = 16, kDecNZ = LAMD_DEC16N_NZ;
using DecTL = Tile<FF16, 8, kDecR, 1, kDecLW, 0, lg_bits(kDecLW)>;
constexpr size_t kDecLds = (DecTL::kXchDwords + tab16_set_dwords(8)) * 4;
constexpr size_t kDecFinLds = (DecTL::kXchDwords + kDecNZ * tab16_set_dwords(8)) * 4;
static_assert(kDecLds <= 160 * 1024 / 3, "three workgroups per CU");
static_assert(kDecFinLds <= 160 * 1024 / 2, "two workgroups per CU");
static_assert(tab16_slot(256) <= DecTL::kXchDwords, "log tables fit the exchange area");
constexpr int kDecOneNZ = 4;  // output tiles held per lane by the one-pass decoder
#ifndef LAMD_DEC16_ONE_R
#define LAMD_DEC16_ONE_R 3
#endif
constexpr int kDecOneR = LAMD_DEC16_ONE_R;
// Column strips of 16 units (128 bytes, 8-wave workgroups, two per CU) or 32
// units (16-wave workgroups, one per CU: each tile's tables are staged once per
// CU instead of twice).  32 is taken when it makes one full round of 240..256
// workgroups (60-64 KiB pieces): 1000+200 x 64 KiB 150.6 vs 156.8-157.1 us,
// 600+400 133.1 vs 139.6; at 128 KiB (two rounds) the two are equal
// (profiles/r04_v21, r04_v22).  The host takes the one-pass form only from
// 60 KiB pieces (fewer workgroups leave SIMDs idle: at 32 KiB it ran 96.7 us
// against 87.2 for the two passes, at 48 KiB 145.8 against 139.7, at 56 KiB
// 148.6 against 147.1; r04_v22, r04_v23).  With one workgroup per CU its LDS has
// room for a second buffer of tables (each phase's skew set and scale / reveal
// tables staged a whole phase ahead): measured 1-2% slower (152.4-153.4 vs
// 150.9-152.5 us, r04_v24-v26) -- the boundary wait is the pieces', not the
// tables', and the staging moved in front of the IFFT's first barrier.
constexpr size_t kDecOneLds16 = one_lds_dwords<kDecOneR, 16>() * 4;
constexpr size_t kDecOneLds32 = one_lds_dwords<kDecOneR, 32>() * 4;
static_assert(kDecOneLds16 <= 160 * 1024 / 2 && kDecOneLds32 <= 160 * 1024, "two / one workgroup(s) per CU");
}  // namespace

#ifdef LAMD_STAMPS
extern "C" __attribute__((visibility("default"))) int leo_amd_debug_stamps16(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps16), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif

// m = 2^Tm with Tm = 7, 8 (m = 128, 256), narrow strips of 16 units.
bool encode16_small_supported(unsigned Tm) { return Tm == 7 || Tm == 8; }
// m = 128: 32-unit strips (8-wave workgroups instead of 4, the chunk tables
// staged once per 256-byte strip) when that makes one full round of 240..256
// workgroups, as the one-pass decoder: 200+100 x 64 KiB 19.45 vs 20.0 us.  For
// m = 256 (16-wave workgroups, one per CU) it measured slower (53.5 vs 52.6 us
// at 1000+200 x 64 KiB, profiles/r04_v27), so 16-unit strips stay there.
#ifndef LAMD_ENC16N_LW32
#define LAMD_ENC16N_LW32 1
#endif
hipError_t launch_encode16_small(unsigned Tm, const EncArgs& a, hipStream_t s) {
    const uint64_t strips32 = (a.nunits + 31) / 32;
    const bool wide = LAMD_ENC16N_LW32 && strips32 >= 240 && strips32 <= 256;
    switch (Tm) {
        case 7: return wide ? launch_enc16n<7, 3, 32>(a, s) : launch_enc16n<7, 3, 16>(a, s);
        case 8: return launch_enc16n<8, 3, 16>(a, s);
        default: return hipErrorInvalidValue;
    }
}

// The chunk-parallel form (k_enc16n_part + k_enc16n_comb, 16-unit strips) for
// single calls with several chunks on fewer 16-unit strips than CUs; the slab
// (a.slab_out = a.slab_in) holds nchunks x m rows of the piece width.
bool encode16_split_wins(unsigned Tm, unsigned nchunks, uint64_t nunits, unsigned cus) {
    bool win = encode16_small_supported(Tm) && nchunks >= 2 && (nunits + 15) / 16 < cus;
#if LAMD_EXPERIMENT_ENV
    static const int force = [] {
        const char* e = std::getenv("LEO_AMD_ENC16_SPLIT");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    if (force >= 0) win = encode16_small_supported(Tm) && nchunks >= 2 && force == 1;
#endif
    return win;
}
hipError_t launch_encode16_split(unsigned Tm, const EncArgs& a, hipStream_t s) {
    auto go = [&](auto part, auto comb, unsigned threads, size_t lds) {
        for (const void* fn : {reinterpret_cast<const void*>(part), reinterpret_cast<const void*>(comb)}) {
            const hipError_t attr = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
            if (attr != hipSuccess) return attr;
        }
        void* params[] = {const_cast<EncArgs*>(&a)};
        const unsigned strips = unsigned((a.nunits + 15) / 16);
        hipError_t e = hipLaunchKernel(reinterpret_cast<const void*>(part), dim3(strips, a.nchunks), dim3(threads), params,
                                       lds, s);
        if (e != hipSuccess) return e;
        return hipLaunchKernel(reinterpret_cast<const void*>(comb), dim3(strips), dim3(threads), params, lds, s);
    };
    using TL7 = Tile<FF16, 7, 3, 1, 16, 0, lg_bits(16)>;
    using TL8 = Tile<FF16, 8, 3, 1, 16, 0, lg_bits(16)>;
    switch (Tm) {
        case 7: return go(&k_enc16n_part<7, 3, 16>, &k_enc16n_comb<7, 3, 16>, threads_n<7, 3, 16>(),
                          (TL7::kXchDwords + tab16_set_dwords(7)) * 4);
        case 8: return go(&k_enc16n_part<8, 3, 16>, &k_enc16n_comb<8, 3, 16>, threads_n<8, 3, 16>(),
                          (TL8::kXchDwords + tab16_set_dwords(8)) * 4);
        default: return hipErrorInvalidValue;
    }
}

// Batches of `count` objects of one shape: argument blocks in device memory.
hipError_t launch_encode16_small_batch(unsigned Tm, const EncArgs* objs, unsigned count, uint64_t nunits,
                                       hipStream_t s) {
    auto go = [&](auto fn, unsigned threads, size_t lds) {
        const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (attr != hipSuccess) return attr;
        const EncArgs* arg = objs;
        void* params[] = {&arg};
        return hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3(unsigned((nunits + 15) / 16), count),
                               dim3(threads), params, lds, s);
    };
    using TL7 = Tile<FF16, 7, 3, 1, 16, 0, lg_bits(16)>;
    using TL8 = Tile<FF16, 8, 3, 1, 16, 0, lg_bits(16)>;
    switch (Tm) {
        case 7: return go(&k_enc16n_batch<7, 3, 16>, threads_n<7, 3, 16>(), (TL7::kXchDwords + 2 * tab16_set_dwords(7)) * 4);
        case 8: return go(&k_enc16n_batch<8, 3, 16>, threads_n<8, 3, 16>(), (TL8::kXchDwords + 2 * tab16_set_dwords(8)) * 4);
        default: return hipErrorInvalidValue;
    }
}

// n = 2^Tn, 9 <= Tn <= 11 (2 .. 8 tiles of 256 positions)
bool decode16_small_supported(unsigned Tn) { return Tn >= 9 && Tn <= 11; }
hipError_t launch_decode16_small_lo(const DecArgs& a, hipStream_t s) {
    const unsigned strips = unsigned((a.nunits + kDecLW - 1) / kDecLW);
    return launch16n(&k_dec16n_lo<kDecR, kDecLW>, dim3(strips, a.nlo), threads_n<8, kDecR, kDecLW>(), kDecLds, a, s);
}
// one-pass form: at most kDecOneNZ output tiles
#ifndef LAMD_DEC16_ONE  // 0: the two-pass form only (A/B builds)
#define LAMD_DEC16_ONE 1
#endif
bool decode16_one_supported(unsigned nout) { return LAMD_DEC16_ONE && nout <= unsigned(kDecOneNZ); }
hipError_t launch_decode16_one(const DecArgs& a, hipStream_t s) {
    const unsigned strips32 = unsigned((a.nunits + 31) / 32);
    if (strips32 >= 240 && strips32 <= 256)
        return launch16n(&k_dec16n_one<kDecOneR, 32, kDecOneNZ>, dim3(strips32), threads_n<8, kDecOneR, 32>(),
                         kDecOneLds32, a, s);
    const unsigned strips = unsigned((a.nunits + 15) / 16);
    return launch16n(&k_dec16n_one<kDecOneR, 16, kDecOneNZ>, dim3(strips), threads_n<8, kDecOneR, 16>(), kDecOneLds16,
                     a, s);
}
// the one-pass form over `count` objects of one shape (nout <= kDecOneNZ)
hipError_t launch_decode16_one_batch(const DecArgs* objs, unsigned count, uint64_t nunits, hipStream_t s) {
    const unsigned strips = unsigned((nunits + 15) / 16);
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dec16n_one_batch<kDecOneR, 16, kDecOneNZ>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, int(kDecOneLds16));
    if (e != hipSuccess) return e;
    const DecArgs* arg = objs;
    void* params[] = {&arg};
    return hipLaunchKernel(reinterpret_cast<const void*>(&k_dec16n_one_batch<kDecOneR, 16, kDecOneNZ>),
                           dim3(strips, count), dim3(threads_n<8, kDecOneR, 16>()), params, kDecOneLds16, s);
}
// both passes over `count` objects of one shape (same nlo, nout, column count)
hipError_t launch_decode16_small_batch(const DecArgs* objs, unsigned count, uint64_t nunits, unsigned nlo,
                                       unsigned nout, hipStream_t s) {
    const unsigned strips = unsigned((nunits + kDecLW - 1) / kDecLW);
    const DecArgs* arg = objs;
    void* params[] = {&arg};
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dec16n_lo_batch<kDecR, kDecLW>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(kDecLds));
    if (e != hipSuccess) return e;
    e = hipLaunchKernel(reinterpret_cast<const void*>(&k_dec16n_lo_batch<kDecR, kDecLW>), dim3(strips, nlo, count),
                        dim3(threads_n<8, kDecR, kDecLW>()), params, kDecLds, s);
    if (e != hipSuccess) return e;
    const unsigned groups = (strips + 7) / 8;
    const unsigned ngrp = (nout + kDecNZ - 1) / kDecNZ;
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dec16n_fin_batch<kDecR, kDecLW, kDecNZ>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(kDecFinLds));
    if (e != hipSuccess) return e;
    return hipLaunchKernel(reinterpret_cast<const void*>(&k_dec16n_fin_batch<kDecR, kDecLW, kDecNZ>),
                           dim3(groups * 8 * ngrp, count), dim3(threads_n<8, kDecR, kDecLW>()), params, kDecFinLds, s);
}
hipError_t launch_decode16_small_fin(const DecArgs& a, hipStream_t s) {
    const unsigned strips = unsigned((a.nunits + kDecLW - 1) / kDecLW);
    const unsigned groups = (strips + 7) / 8;  // strips dealt 8 at a time, one per XCD
    const unsigned ngrp = (a.nout + kDecNZ - 1) / kDecNZ;
    return launch16n(&k_dec16n_fin<kDecR, kDecLW, kDecNZ>, dim3(groups * 8 * ngrp), threads_n<8, kDecR, kDecLW>(),
                     kDecFinLds, a, s);
}

}  // namespace lamd
