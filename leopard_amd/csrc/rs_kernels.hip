// rs_kernels.hip -- the Reed-Solomon encode/decode kernels for gfx950.
//
// Encoder (reference ReedSolomonEncode, LeopardFF8.cpp:1602-1672):
//   work = XOR_c IFFT_m(data[c*m .. c*m+m), skew + m-1 + c*m);  out = FFT_m(work, skew - 1)[0..R)
// Decoder (reference ReedSolomonDecode, LeopardFF8.cpp:1809-1916):
//   el   = FWHT(LogWalsh * FWHT(erasures))          error locator, as logs
//   v    = IFFT_n(el * received, skew - 1)
//   z    = FormalDerivative(v)
//   lost original i = FFT_n(z)[m + i] * exp(-el[m + i])
//
// Kernel families (T = tile bits, see rs_device.h):
//   k_enc_fused<FF16>         : the whole encode transform in one workgroup tile (m <= 256)
//   (GF(2^8), n <= 256, lives in rs_ff8.hip)
//   k_enc_lo/hi/fin, k_dec_lo/hi/fin : FF16 transforms of 2^9 .. 2^16 pieces as
//     three tile passes: low 8 bits, high bits, low 8 bits again.  The formal
//     derivative is split between the passes with
//        F_lo F_hi (I + D_hi + D_lo) v = F_lo ( F_hi (I + D_hi) v  +  D_lo F_hi v ),
//     valid because D_lo (flips of low bits) commutes with every butterfly of
//     the high layers, whose skew depends only on the high bits of the index.
#include <hip/hip_runtime.h>

#include "rs_args.h"

namespace lamd {

namespace {

constexpr int C = kUnitsPerLane;

// Register bits per lane for a tile of T bits: 8 pieces per lane when that
// gives at most 16 waves (more waves per SIMD hide the butterfly chains'
// latency), otherwise 16 pieces (T = 8: 16 waves of 16 pieces).
constexpr int reg_bits(int T) { return T <= 3 ? T : (T - 3 <= 4 ? 3 : T - 4); }
constexpr int wave_bits(int T) { return T - reg_bits(T); }

// LDS carve-up: the tile transpose area
template <class F, int T>
constexpr size_t tile_lds_dwords() {
    return wave_bits(T) > 0 ? (size_t(1) << T) * 64 * C * F::kDw : 0;  // transposes
}

// Butterfly tables of a kernel: FF16 reads them through the scalar cache (the
// FF8 kernels in rs_ff8.hip stage theirs in LDS).
template <class F, int NT>
struct SkewTables {
    using Win = GlobalWindow<F>;
    static constexpr size_t kLdsDwords = 0;
    LDEV void load(const uint32_t*) {}
    LDEV void publish(uint32_t*) const {}
    LDEV static Win window(uint32_t*) { return Win{}; }
};
LDEV uint64_t lane_units(unsigned lane) { return (uint64_t(blockIdx.x) * 64 + lane) * C; }

// Column addressing of the multi-pass GF(2^16) kernels: workgroup x owns units
// [64x, 64x + 64) = bytes [512x, 512x + 512) of every piece (a unit = the low
// and the high dword of 4 ALTMAP elements, 32 bytes apart).  The strip base is
// wave-uniform and the lane's offset inside it a 32-bit VGPR, so each piece
// access is a global_load/store with an SGPR base: no 64-bit vector address
// per piece (32 pieces a lane).  Lanes past the last unit re-read the last
// valid unit and never store.
struct Cols16 {
    uint64_t strip;  // byte offset of the strip (wave-uniform)
    uint32_t off;    // this lane's byte offset inside the strip
    bool live;
};
LDEV Cols16 cols16(uint64_t nunits, unsigned lane) {
    const uint64_t first = uint64_t(blockIdx.x) * 64;
    const uint64_t left = nunits - first;
    const unsigned l = lane < left ? lane : unsigned(left - 1);
    return Cols16{first * 8, (l >> 3) * 64u + (l & 7u) * 4u, lane < left};
}
// base: wave-uniform address of the strip (piece pointer + strip, or the zero page)
LDEV void ld16(uint32_t* x, const uint8_t* base, uint32_t off) {
    if constexpr ((LAMD_ABLATE & 4) != 0) {  // experiments: no piece loads
        x[0] = off * 2654435761u + uint32_t(uintptr_t(base));
        x[1] = x[0] ^ 0x5bd1e995u;
        return;
    }
    x[0] = gld<uint32_t>(base + off);
    x[1] = gld<uint32_t>(base + off + 32);
}
LDEV void st16(uint8_t* base, uint32_t off, const uint32_t* x) {
    if constexpr ((LAMD_ABLATE & 8) != 0) {  // experiments: no piece stores (keep x live)
        if ((x[0] ^ x[1]) == 0x9E3779B9u && off == 0x7FFFFFFFu) *gptr<uint32_t>(base) = x[0];
        return;
    }
    gst<uint32_t>(base + off, x[0]);
    gst<uint32_t>(base + off + 32, x[1]);
}
// piece i of pm when `ok` (wave-uniform), else zeros from the zero page
LDEV void ld16z(uint32_t* x, const PieceMap& pm, bool ok, unsigned i, const uint8_t* zeros, const Cols16& c) {
    const uint8_t* base = zeros;
    if (ok) base = pm.ptr(i) + c.strip;
    ld16(x, base, c.off);
}

// Strip addresses of the pieces of a caller's piece map (a pointer table or a
// slab, wave-uniform) that a lane's registers r < NR hold, `ok(r)` false: the
// zero page.  The table-or-slab test is made once for all of them, the table
// entries are read back to back (one scalar-load round trip instead of one per
// piece) and the zero-page choice is a select, not a branch: per piece the
// prologue is a few scalar instructions, not a dozen and three branches.
template <int NR, class Idx, class Ok>
LDEV void map_ptrs(const uint8_t* (&pp)[NR], const PieceMap& pm, Idx idx, Ok ok, const uint8_t* zeros,
                   const Cols16& c) {
    uint64_t q[NR];
    if (pm.table) {
#pragma unroll
        for (int r = 0; r < NR; ++r) q[r] = cload64(pm.table + (ok(r) ? idx(r) : 0u));  // entry 0 always exists
    } else {
#pragma unroll
        for (int r = 0; r < NR; ++r) q[r] = uint64_t(reinterpret_cast<uintptr_t>(pm.base)) + uint64_t(idx(r)) * pm.stride;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) pp[r] = ok(r) ? reinterpret_cast<const uint8_t*>(q[r] + pm.off + c.strip) : zeros;
}
// x[r] <- the pieces of a caller's map for r < NR (map_ptrs), in batches of 8
template <class TL, class Idx, class Ok>
LDEV void load_map(typename TL::Reg& x, const PieceMap& pm, Idx idx, Ok ok, const uint8_t* zeros, const Cols16& c) {
    constexpr int B = TL::NR < 8 ? TL::NR : 8;
    static_for<0, TL::NR / B>([&](auto BI) {
        constexpr int r0 = decltype(BI)::value * B;
        const uint8_t* pp[B];
        map_ptrs(pp, pm, [&](int r) { return idx(r0 + r); }, [&](int r) { return ok(r0 + r); }, zeros, c);
#pragma unroll
        for (int r = 0; r < B; ++r) ld16(x[r0 + r], pp[r], c.off);
    });
}

// Piece i of pm when `ok` (wave-uniform), else zeros read from the zero page.
// The choice is made on scalars so the vector code has no branch.
template <class F>
LDEV void load_or_zero(uint32_t* x, const PieceMap& pm, bool ok, unsigned i, const uint8_t* zeros, uint64_t q) {
    const uint8_t* src = zeros;
    uint64_t qq = 0;
    if (ok) { src = pm.ptr(i); qq = q; }
    load_units<F, C>(x, src, qq);
}

// ------------------------------------------------------------------ encode --

template <class F, int T>
__global__ void __launch_bounds__(64 << wave_bits(T), 4) k_enc_fused(EncArgs a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    using TL = Tile<F, T, reg_bits(T), C>;
    constexpr int NT = 64 << wave_bits(T);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* sk_lds = lds + tile_lds_dwords<F, T>();
    SkewTables<F, NT> sk;
    sk.load(a.sktab);
    auto win = sk.window(sk_lds);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t q0 = lane_units(lane);
    const bool live = q0 < a.nunits;
    const uint64_t ql = live ? q0 : a.nunits - C;  // dead lanes re-read a valid unit: loads stay unpredicated
    constexpr unsigned m = 1u << T;
    const PieceSpace ps{0, 0, 0};
    typename TL::Reg acc, x;
    auto load_chunk = [&](unsigned c) {
        const unsigned base = c * m;
        const unsigned cnt = a.K - base < m ? a.K - base : m;
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const unsigned tp = TL::piece(0, r, w);
            load_or_zero<F>(x[r], a.in, tp < cnt, base + tp, a.zeros, ql);
        }
    };
    load_chunk(0);
    sk.publish(sk_lds);
    __syncthreads();
    TL::zero(acc);
    for (unsigned c = 0;;) {
        // IFFT without its top layer, then the fused top (IFFT top + FFT top, as rs_ff8.hip)
        win.stage(a.sktab, int(m - 1 + c * m));
        TL::template ifft<true>(x, w, lane, lds, ps, win, BelowLive{a.K - c * m});
        TL::fused_top(x, F::tab(a.tabs, cload(a.fused + c)));
        TL::xor_into(acc, x);
        if (++c >= a.nchunks) break;
        load_chunk(c);
    }
    win.stage(a.sktab, -1);
    TL::template fft<true>(acc, w, lane, lds, ps, win, BelowLive{a.R});
    TL::pin(acc);
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned tp = TL::piece(0, r, w);
        if (tp < a.R && live) store_units<F, C>(a.out.ptr(tp), q0, acc[r]);
    }
}

// ------------------------------------------------- multi-pass GF(2^16) tiles --
//
// Tiles of the multi-pass transforms: 2^T pieces, 32 pieces per lane in
// registers (R = 5), so a 256-piece tile is 8 waves and its LDS exchanges run
// in 4 rounds through a 32 KiB area (Tile S = 2); with its butterfly tables
// (and the decoder's per-piece scale / reveal tables) staged in LDS that is at
// most 72 KiB, so two workgroups share every CU and one's loads and stores
// overlap the other's butterflies (one 1024-thread, 128 KiB workgroup per CU
// ran load -> butterflies -> store with nothing to overlap: ~35% VALU issue).
constexpr int reg16(int T) { return T <= 5 ? T : 5; }
#ifndef LAMD_SPLIT16
#define LAMD_SPLIT16 2
#endif
constexpr int split16(int T) { return T >= 7 ? LAMD_SPLIT16 : (T == 6 && LAMD_SPLIT16 ? 1 : 0); }
// the multi-chunk encoder pass keeps an accumulator tile as well: 16 pieces per lane
constexpr int reg16_acc(int T) { return T <= 4 ? T : 4; }
constexpr int split16_acc(int T) { return T == 6 ? 1 : 0; }
constexpr unsigned threads16(int T, int R) { return 64u << (T - R); }

template <int T, int R, int S>
using Tile16 = Tile<FF16, T, R, C, 64, S>;

// Waves per SIMD the high passes are compiled for (4: <= 128 VGPRs; 3 gives
// the 32-piece tiles room without spills at one workgroup fewer per CU).
#ifndef LAMD_HI_WAVES
#define LAMD_HI_WAVES 4
#endif

// Pruning inside a multi-pass tile: off by default.  A per-group branch around
// updates of a 64-VGPR tile makes the register allocator copy and spill at
// every merge; every butterfly runs instead (a dead IFFT block is all zero and
// stays zero, a dead FFT block feeds no needed output, so results are the
// same).  Whole tiles are still skipped: the lo passes run only tiles with
// input, the hi passes read zeros for empty low tiles, k_dec_fin returns on
// tiles without a lost original.  LAMD_PRUNE16=1 builds the per-group form.
#ifndef LAMD_PRUNE16
#define LAMD_PRUNE16 0
#endif
template <class P>
LDEV auto prune16(const P& p) {
    if constexpr (LAMD_PRUNE16 != 0) return p;
    else return AllLive{};
}

// LDS carve-up: exchange area, then `sets` butterfly-table sets, then `logs`
// per-piece log-value table slots.
template <int T, int R, int S>
constexpr size_t lds16_dwords(int sets, int logs) {
    return Tile16<T, R, S>::kXchDwords + size_t(sets) * tab16_set_dwords(T) +
           size_t(tab16_slot(logs));
}

// x[r] ^= the units of piece map pm at tile pieces piece(LAY, r, w), loaded in
// batches of 8 pieces (keeps the batch's VGPRs bounded next to a full tile).
template <class TL, int LAY, class PosFn>
LDEV void xor_load(typename TL::Reg& x, const PieceMap& pm, PosFn pos, unsigned w, const Cols16& cl) {
    constexpr int B = TL::NR < 8 ? TL::NR : 8;
    static_for<0, TL::NR / B>([&](auto BI) {
        constexpr int r0 = decltype(BI)::value * B;
        uint32_t y[B][TL::U];
        static_for<0, B>([&](auto I) { ld16(y[I.value], pm.slab_ptr(pos(TL::piece(LAY, r0 + I.value, w))) + cl.strip, cl.off); });
        __builtin_amdgcn_sched_barrier(0);  // one batch of loads in flight at a time
        static_for<0, B>([&](auto I) {
#pragma unroll
            for (int k = 0; k < TL::U; ++k) x[r0 + I.value][k] ^= y[I.value][k];
        });
    });
}

// pass 1: IFFT over the low kLoBits of chunk blockIdx.z -> slab_out[c*m + g]
// (tables: skew base m-1 + c*m, the tile's positions y*256 + j)
template <int R, int S>
__global__ void __launch_bounds__(threads16(kLoBits, R), 4) k_enc_lo(EncArgs a) {
    constexpr int T = kLoBits;
    constexpr int NT = threads16(T, R);
    using TL = Tile16<T, R, S>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* set = lds + TL::kXchDwords;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols16 cl = cols16(a.nunits, lane);
    const bool live = cl.live;
    const unsigned m = 1u << a.Tm;
    const unsigned c = blockIdx.z, base = c * m, y = blockIdx.y;
    const PieceSpace ps{0, 0, y << T};
    Tabs16Stage<NT, T> st;
    st.load(a.sktab, int(m - 1 + base), y << T, 0);
    typename TL::Reg x;
    load_map<TL>(x, a.in, [&](int r) { return base + ps.global(TL::piece(0, r, w)); },
                 [&](int r) { return base + ps.global(TL::piece(0, r, w)) < a.K; }, a.zeros, cl);
    st.store(set);
    __syncthreads();
    TL::ifft(x, w, lane, lds, ps, LdsWindow16{set, y << T, 0}, prune16(BelowLive{a.K - base}));
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned g = ps.global(TL::piece(TL::kLast, r, w));
        st16(a.slab_out.slab_ptr(base + g) + cl.strip, cl.off, x[r]);
    }
}

// pass 2: for every chunk IFFT over the high bits and accumulate; then the
// FFT over the high bits -> slab_out[g].  Tile positions y + (j << 8): the IFFT
// tables of chunk c (skew base m-1 + c*m) and the FFT tables (base -1) are two
// LDS sets.  kMulti: several chunks (T <= 6 then), accumulated in a second tile.
template <int T, int R, int S, bool kMulti>
__global__ void __launch_bounds__(threads16(T, R), LAMD_HI_WAVES) k_enc_hi(EncArgs a) {
    constexpr int NT = threads16(T, R);
    using TL = Tile16<T, R, S>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* iset = lds + TL::kXchDwords;
    uint32_t* fset = iset + tab16_set_dwords(T);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols16 cl = cols16(a.nunits, lane);
    const bool live = cl.live;
    const unsigned m = 1u << a.Tm;
    const PieceSpace ps{blockIdx.y, kLoBits, 0};
    const LdsWindow16 iwin{iset, 0, kLoBits};
    const LdsWindow16Static<-1, kLoBits> fwin{{fset, 0, kLoBits}};  // staged at skew base -1
    typename TL::Reg x;
    auto load_chunk = [&](unsigned c) {
        const unsigned base = c * m;
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const unsigned tp = TL::piece(0, r, w);
            // low tiles that lie entirely past K were all-zero inputs
            const bool ok = base + (tp << kLoBits) < a.K;
            ld16(x[r], ok ? a.slab_in.slab_ptr(base + ps.global(tp)) + cl.strip : a.zeros, cl.off);
        }
    };
    {
        Tabs16Stage<NT, T> si, sf;
        si.load(a.sktab, int(m - 1), 0, kLoBits);
        sf.load(a.sktab, -1, 0, kLoBits);
        load_chunk(0);
        si.store(iset);
        sf.store(fset);
        __syncthreads();
    }
    if constexpr (!kMulti) {
        TL::template ifft<true>(x, w, lane, lds, ps, iwin, prune16(BelowLive{a.K}));
        TL::fused_top(x, FF16::tab(a.tabs, cload(a.fused)));  // top of the m-transform: this pass's top bit
    } else {
        typename TL::Reg acc;
        for (unsigned c = 0;;) {
            TL::template ifft<true>(x, w, lane, lds, ps, iwin, prune16(BelowLive{a.K - c * m}));
            TL::fused_top(x, FF16::tab(a.tabs, cload(a.fused + c)));
            if (c == 0) TL::copy(acc, x);
            else TL::xor_into(acc, x);
            if (++c >= a.nchunks) break;
            Tabs16Stage<NT, T> si;
            si.load(a.sktab, int(m - 1 + c * m), 0, kLoBits);
            load_chunk(c);
            __syncthreads();  // every wave is done with the previous chunk's tables
            si.store(iset);
            __syncthreads();
        }
        TL::copy(x, acc);
    }
    TL::template fft<true>(x, w, lane, lds, ps, fwin, prune16(BelowLive{a.R}));
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned g = ps.global(TL::piece(0, r, w));
        st16(a.slab_out.slab_ptr(g) + cl.strip, cl.off, x[r]);
    }
}

// pass 3: FFT over the low bits, keep outputs g < R.  When m = 2^kLoBits (no
// high pass) the chunk IFFTs of pass 1 are combined here: x = XOR_c U[c*m + g].
template <int R, int S>
__global__ void __launch_bounds__(threads16(kLoBits, R), 4) k_enc_fin(EncArgs a) {
    constexpr int T = kLoBits;
    constexpr int NT = threads16(T, R);
    using TL = Tile16<T, R, S>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* set = lds + TL::kXchDwords;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols16 cl = cols16(a.nunits, lane);
    const bool live = cl.live;
    const unsigned y = blockIdx.y;
    const PieceSpace ps{0, 0, y << T};
    Tabs16Stage<NT, T> st;
    st.load(a.sktab, -1, y << T, 0);
    typename TL::Reg x;
    auto pos = [&](unsigned tp) { return ps.global(tp); };
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) ld16(x[r], a.slab_in.slab_ptr(pos(TL::piece(TL::kLast, r, w))) + cl.strip, cl.off);
    st.store(set);
    __syncthreads();
    if (a.Tm == unsigned(kLoBits))
        for (unsigned c = 1; c < a.nchunks; ++c)
            xor_load<TL, TL::kLast>(x, a.slab_in, [&](unsigned tp) { return (c << T) + pos(tp); }, w, cl);
    TL::fft(x, w, lane, lds, ps, LdsWindow16{set, y << T, 0}, prune16(BelowLive{a.R}));
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned g = ps.global(TL::piece(0, r, w));
        if (g < a.R) st16(a.out.ptr(g) + cl.strip, cl.off, x[r]);
    }
}
// ------------------------------------------------------------------ decode --

LDEV bool bit_set(const uint32_t* bits, unsigned p) { return (cload(bits + (p >> 5)) >> (p & 31)) & 1u; }

// FF16 occupancy pyramid in device memory (rs_args.h: pyr_offset), read through
// the scalar cache; see rs_device.h for the pruning rule.
struct Pyr16Live {
    const uint32_t* pyr;
    LDEV bool operator()(unsigned pos, unsigned level) const {
        const unsigned j = pos >> level;
        return (cload(pyr + pyr_offset(level) + (j >> 5)) >> (j & 31)) & 1u;
    }
};

// Received piece at codeword position p (scaled later by exp(el[p])); zero if
// absent.  Positions: [0, m) recovery (only [0, R) exist), [m, m+K) originals
// (LeopardFF8.cpp:1857-1877).  Branch-free on the vector side: an absent piece
// reads the zero page at unit 0.
#ifndef LAMD_DEC_LO_RUN
#define LAMD_DEC_LO_RUN 1
#endif
LDEV void load_received(uint32_t* x, const DecArgs& a, unsigned p, const Cols16& c) {
    const uint8_t* base = a.zeros;
    if (!bit_set(a.erased_dev, p)) {
        if (p < a.R) base = a.rec.ptr(p) + c.strip;
        else if (p >= a.m && p < a.m + a.K) base = a.orig.ptr(p - a.m) + c.strip;
    }
    ld16(x, base, c.off);
}

// The NR received pieces at positions p0 .. p0 + NR - 1 (a lane's registers
// in layout 0; p0 a multiple of NR <= 32): the erasure bits come from one
// word and every piece pointer is fetched before the first piece load issues.
// (load_received per piece chained an erasure-word scalar load, a wait, a
// branch, a pointer scalar load and a wait in front of each piece load.)
template <int NR, class Reg>
LDEV void load_received_run(Reg& v, const DecArgs& a, unsigned p0, const Cols16& c) {
    static_assert(NR <= 32 && (NR & (NR - 1)) == 0, "positions inside one erasure word");
    const uint32_t ew = cload(a.erased_dev + (p0 >> 5)) >> (p0 & 31);
    const uint8_t* base[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const unsigned p = p0 + unsigned(r);
        const uint8_t* b = a.zeros;
        if (!((ew >> r) & 1u)) {
            if (p < a.R) b = a.rec.ptr(p) + c.strip;
            else if (p >= a.m && p < a.m + a.K) b = a.orig.ptr(p - a.m) + c.strip;
        }
        base[r] = b;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) asm volatile("" : "+s"(base[r]));
#pragma unroll
    for (int r = 0; r < NR; ++r) ld16(v[r], base[r], c.off);
}

// pass 1: scale-on-load + IFFT over the low bits -> a_out[g].  LDS: exchange
// area, the tile's butterfly tables (skew base -1, positions y*256 + j), and
// its 256 scale tables (log value scale_logs[p] = el[p], or the zero table).
template <int R, int S>
__global__ void __launch_bounds__(threads16(kLoBits, R), 4) k_dec_lo(DecArgs a) {
    constexpr int T = kLoBits;
    constexpr int NT = threads16(T, R);
    using TL = Tile16<T, R, S>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* set = lds + TL::kXchDwords;
    uint32_t* scl = set + tab16_set_dwords(T);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols16 cl = cols16(a.nunits, lane);
    const bool live = cl.live;
    const unsigned y = blockIdx.y;
    const PieceSpace ps{0, 0, y << T};
    Tabs16Stage<NT, T> st;
    st.load(a.sktab, -1, y << T, 0);
    LogTabs16Stage<NT, (1u << T)> ls;
    ls.load(a.tabs, a.scale_logs + (y << T));
    typename TL::Reg v;
    static_assert(TL::lo(0) == 0, "layout 0: register r holds position r | w << R");
#if LAMD_DEC_LO_RUN
    load_received_run<TL::NR>(v, a, ps.global(TL::piece(0, 0, w)), cl);
#else
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) load_received(v[r], a, ps.global(TL::piece(0, r, w)), cl);
#endif
    st.store(set);
    ls.store(scl);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        asm volatile("" ::: "memory");  // keeps the compiler from hoisting every table read up here
        const FF16::Tab t = FF16::tab_lds(scl + tab16_slot(TL::piece(0, r, w)));
#pragma unroll
        for (int u = 0; u < C; ++u) FF16::mul(&v[r][u * 2], &v[r][u * 2], t);
#pragma unroll
        for (int k = 0; k < 2 * C; ++k) asm volatile("" : "+v"(v[r][k]));  // one scale table live at a time
    }
    TL::ifft(v, w, lane, lds, ps, LdsWindow16{set, y << T, 0}, prune16(Pyr16Live{a.present_pyr}));
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) st16(a.a_out.slab_ptr(ps.global(TL::piece(TL::kLast, r, w))) + cl.strip, cl.off, v[r]);
}

// pass 2: A = F_hi (I + D_hi) I_hi U over the high bits, computed as
// F_hi' (swap_top + D_hi') I_hi' U without the top layers (Tile::derivative_swaptop).
// The other term of the split derivative needs F_hi(I_hi U) = U, which pass 3
// reads straight from pass 1's slab.  Tables: skew base -1, positions j << 8.
template <int T, int R, int S>
__global__ void __launch_bounds__(threads16(T, R), LAMD_HI_WAVES) k_dec_hi(DecArgs a) {
    constexpr int NT = threads16(T, R);
    using TL = Tile16<T, R, S>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* set = lds + TL::kXchDwords;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols16 cl = cols16(a.nunits, lane);
    const bool live = cl.live;
    const PieceSpace ps{blockIdx.y, kLoBits, 0};
    Tabs16Stage<NT, T> st;
    st.load(a.sktab, -1, 0, kLoBits);
    typename TL::Reg v;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned tp = TL::piece(0, r, w);
        ld16(v[r], tp < a.nlo ? a.a_in.slab_ptr(ps.global(tp)) + cl.strip : a.zeros, cl.off);
    }
    st.store(set);
    __syncthreads();
    const LdsWindow16Static<-1, kLoBits> win{{set, 0, kLoBits}};  // staged at skew base -1
    TL::template ifft<true>(v, w, lane, lds, ps, win, prune16(Pyr16Live{a.present_pyr}));
    TL::derivative_swaptop(v, w, lane, lds, true);
    TL::template fft<true>(v, w, lane, lds, ps, win, prune16(Pyr16Live{a.needed_pyr}));
    // pass 3 reads A only in low tiles holding a lost original: store nothing else
    const Pyr16Live needed{a.needed_pyr};
    if (live)
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const unsigned p = ps.global(TL::piece(0, r, w));
            if (needed(p, kLoBits)) st16(a.a_out.slab_ptr(p) + cl.strip, cl.off, v[r]);
        }
}

// pass 2 when every received piece is in the low half (K = R, every original
// lost; see k_ff8_dec_half in rs_ff8.hip): the high IFFT layers of the low
// half, the fused top layer of the m-transform (encoder chunk 0's table) and the
// high FFT layers with the skews of the high half; A is written at the high
// positions only and pass 3 adds D_lo(U) = 0 there (U has no high tiles).
// Tables: skew base -1, positions j << 8 (low half) and m + (j << 8) (high half).
template <int T, int R, int S>
__global__ void __launch_bounds__(threads16(T, R), LAMD_HI_WAVES) k_dec_hi_half(DecArgs a) {
    constexpr int NT = threads16(T, R);
    using TL = Tile16<T, R, S>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* lset = lds + TL::kXchDwords;
    uint32_t* hset = lset + tab16_set_dwords(T);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols16 cl = cols16(a.nunits, lane);
    const bool live = cl.live;
    const PieceSpace low{blockIdx.y, kLoBits, 0}, high{blockIdx.y, kLoBits, a.m};
    Tabs16Stage<NT, T> sl, sh;
    sl.load(a.sktab, -1, 0, kLoBits);
    sh.load(a.sktab, -1, a.m, kLoBits);
    typename TL::Reg v;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned tp = TL::piece(0, r, w);
        ld16(v[r], tp < a.nlo ? a.a_in.slab_ptr(low.global(tp)) + cl.strip : a.zeros, cl.off);
    }
    sl.store(lset);
    sh.store(hset);
    __syncthreads();
    TL::template ifft<true>(v, w, lane, lds, low, LdsWindow16Static<-1, kLoBits>{{lset, 0, kLoBits}},
                            prune16(Pyr16Live{a.present_pyr}));
    TL::fused_top(v, FF16::tab(a.tabs, cload(a.fused)));
    TL::template fft<true>(v, w, lane, lds, high, LdsWindow16{hset, a.m, kLoBits}, prune16(Pyr16Live{a.needed_pyr}));
    if (live)
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) st16(a.a_out.slab_ptr(high.global(TL::piece(0, r, w))) + cl.strip, cl.off, v[r]);
}

// pass 3: z = A + D_lo(U), FFT over the low bits, reveal lost originals
// (work[i] = z[m + i] * exp(-el[m + i]), LeopardFF8.cpp:1913-1915; the reveal
// tables, log value reveal_logs[p], staged in LDS).  U of a low tile without
// received data is zero and was never written.
template <int R, int S>
__global__ void __launch_bounds__(threads16(kLoBits, R), 4) k_dec_fin(DecArgs a) {
    constexpr int T = kLoBits;
    constexpr int NT = threads16(T, R);
    using TL = Tile16<T, R, S>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const unsigned y = blockIdx.y;
    // skip tiles holding no lost original (uniform across the workgroup)
    if (!((cload(a.needed_pyr + pyr_offset(T) + (y >> 5)) >> (y & 31)) & 1u)) return;
    uint32_t* set = lds + TL::kXchDwords;
    uint32_t* rvl = set + tab16_set_dwords(T);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols16 cl = cols16(a.nunits, lane);
    const bool live = cl.live;
    const PieceSpace ps{0, 0, y << T};
    Tabs16Stage<NT, T> st;
    st.load(a.sktab, -1, y << T, 0);
    LogTabs16Stage<NT, (1u << T)> ls;
    ls.load(a.tabs, a.reveal_logs + (y << T));
    typename TL::Reg z;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) ld16(z[r], a.a_in.slab_ptr(ps.global(TL::piece(TL::kLast, r, w))) + cl.strip, cl.off);
    // output pointers of the lane's lost originals (layout 0: positions p0 + r),
    // fetched here as one batch behind the slab loads: at the stores each was an
    // erasure-word and a pointer scalar load, waited for one after the other
    static_assert(TL::lo(0) == 0, "layout 0: register r holds position r | w << R");
    const unsigned p0 = ps.global(TL::piece(0, 0, w));
    const uint32_t ew = cload(a.erased_dev + (p0 >> 5)) >> (p0 & 31);
    uint8_t* op[TL::NR];
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned p = p0 + unsigned(r);
        op[r] = nullptr;
        if (p >= a.m && p < a.m + a.K && ((ew >> r) & 1u)) op[r] = a.out.ptr(p - a.m) + cl.strip;
    }
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) asm volatile("" : "+s"(op[r]));
    st.store(set);
    ls.store(rvl);
    __syncthreads();
    // U of a tile past the received ones is zero, and so is D_lo(U) (workgroup-uniform)
    if (y < a.nlo)
        TL::derivative_add(z, [&](int r, uint32_t* out) {
            ld16(out, a.b_in.slab_ptr(ps.global(TL::piece(TL::kLast, r, w))) + cl.strip, cl.off);
        }, w, lane, lds);
    TL::fft(z, w, lane, lds, ps, LdsWindow16{set, y << T, 0}, prune16(Pyr16Live{a.needed_pyr}));
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        if (op[r] != nullptr) {
            uint32_t o[2 * C];
            asm volatile("" ::: "memory");
            const FF16::Tab t = FF16::tab_lds(rvl + tab16_slot(TL::piece(0, r, w)));
#pragma unroll
            for (int u = 0; u < C; ++u) FF16::mul(&o[u * 2], &z[r][u * 2], t);
            st16(op[r], cl.off, o);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// FF16 error locator over 65536 positions as a 256 x 256 Walsh-Hadamard
// transform: rows (low 8 bits) / columns (high 8 bits), one wave per line.
struct Mod16 {
    LDEV static unsigned add(unsigned a, unsigned b) { unsigned s = a + b; return s >= 65535u ? s - 65535u : s; }
    LDEV static unsigned sub(unsigned a, unsigned b) { unsigned s = a + 65535u - b; return s >= 65535u ? s - 65535u : s; }
};
LDEV void fwht256(unsigned (&e)[4], unsigned lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned o = __shfl_xor(int(e[j]), d);
            e[j] = (lane & d) ? Mod16::sub(o, e[j]) : Mod16::add(e[j], o);
        }
    const unsigned a0 = Mod16::add(e[0], e[1]), a1 = Mod16::sub(e[0], e[1]);
    const unsigned a2 = Mod16::add(e[2], e[3]), a3 = Mod16::sub(e[2], e[3]);
    e[0] = Mod16::add(a0, a2); e[2] = Mod16::sub(a0, a2);
    e[1] = Mod16::add(a1, a3); e[3] = Mod16::sub(a1, a3);
}

// mode 0: rows of the erasure bitmap -> tmp; mode 1: rows of tmp -> el, plus
// the per-position log values of the decoder's multiplies: scale_logs[p] =
// el[p] for a received piece (LeopardFF8.cpp:1857-1877), reveal_logs[p] =
// kModulus - el[p] for a lost original (:1913-1915), the all-zero table
// (65536) elsewhere.
__global__ void __launch_bounds__(64) k_el16_rows(const uint32_t* erased, uint32_t* tmp, uint32_t* el,
                                                 uint32_t* scale_logs, uint32_t* reveal_logs, int mode, unsigned m,
                                                 unsigned K, unsigned R) {
    const unsigned lane = threadIdx.x, row = blockIdx.x;
    unsigned e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const unsigned p = row * 256 + lane + 64 * j;
        e[j] = mode == 0 ? bit_set(erased, p) : tmp[p];
    }
    fwht256(e, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const unsigned p = row * 256 + lane + 64 * j;
        if (mode == 0) {
            tmp[p] = e[j];
        } else {
            el[p] = e[j];
            const bool lost = bit_set(erased, p);
            const bool orig = p >= m && p < m + K;
            scale_logs[p] = !lost && (p < R || orig) ? e[j] : 65536u;
            reveal_logs[p] = lost && orig ? 65535u - e[j] : 65536u;
        }
    }
}
// columns: FWHT over the high bits, pointwise * LogWalsh mod 65535, FWHT again
__global__ void __launch_bounds__(64) k_el16_cols(uint32_t* tmp, const uint32_t* walsh) {
    const unsigned lane = threadIdx.x, col = blockIdx.x;
    unsigned e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) e[j] = tmp[col + 256 * (lane + 64 * j)];
    fwht256(e, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const unsigned p = col + 256 * (lane + 64 * j);
        e[j] = (e[j] * walsh[p]) % 65535u;
    }
    fwht256(e, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) tmp[col + 256 * (lane + 64 * j)] = e[j];
}

// R == 1 parity paths (leopard.cpp:106-121, 214-231): out = XOR of pieces.
__global__ void __launch_bounds__(256) k_xor_reduce(XorArgs a) {
    const uint64_t q = (uint64_t(blockIdx.x) * 256 + threadIdx.x) * 4;  // dword index
    if (q >= a.ndwords) return;
    v4u acc = v4u{0, 0, 0, 0};
    for (unsigned i = 0; i < a.count; ++i) {
        const uint8_t* p = a.src.ptr(i);
        const v4u v = *gptr<const v4u>(p + q * 4);
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    *gptr<v4u>(a.out.ptr(0) + q * 4) = acc;
}

// ------------------------------------------------------------ dispatching --

unsigned tiles_for(uint64_t nunits) { return unsigned((nunits + kUnitsPerTile - 1) / kUnitsPerTile); }

template <class KernelFn>
hipError_t launch(KernelFn* fn, dim3 grid, unsigned threads, size_t lds_dwords, hipStream_t s, const void* args_ptr) {
    const size_t lds = lds_dwords * 4;
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    void* params[] = {const_cast<void*>(args_ptr)};
    return hipLaunchKernel(reinterpret_cast<const void*>(fn), grid, dim3(threads), params, lds, s);
}

template <class F, int T>
constexpr size_t full_tile_lds() {  // transpose area + staged skew tables
    return tile_lds_dwords<F, T>() + SkewTables<F, (64 << wave_bits(T))>::kLdsDwords;
}

template <class F, int T>
struct EncFusedFn {
    static hipError_t run(const EncArgs& a, hipStream_t s) {
        return launch(&k_enc_fused<F, T>, dim3(tiles_for(a.nunits)), 64u << wave_bits(T), full_tile_lds<F, T>(), s,
                      &a);
    }
};
template <int T, bool kMulti>
struct EncHiFn {
    static hipError_t run(const EncArgs& a, hipStream_t s) {
        constexpr int R = kMulti ? reg16_acc(T) : reg16(T), S = kMulti ? split16_acc(T) : split16(T);
        return launch(&k_enc_hi<T, R, S, kMulti>, dim3(tiles_for(a.nunits), 1u << kLoBits), threads16(T, R),
                      lds16_dwords<T, R, S>(2, 0), s, &a);
    }
};
template <int T>
struct DecHiFn {
    static hipError_t run(const DecArgs& a, hipStream_t s) {
        constexpr int R = reg16(T), S = split16(T);
        return launch(&k_dec_hi<T, R, S>, dim3(tiles_for(a.nunits), 1u << kLoBits), threads16(T, R),
                      lds16_dwords<T, R, S>(1, 0), s, &a);
    }
};
template <int T>
struct DecHiHalfFn {
    static hipError_t run(const DecArgs& a, hipStream_t s) {
        constexpr int R = reg16(T), S = split16(T);
        return launch(&k_dec_hi_half<T, R, S>, dim3(tiles_for(a.nunits), 1u << kLoBits), threads16(T, R),
                      lds16_dwords<T, R, S>(2, 0), s, &a);
    }
};

template <template <int> class Fn, int TMIN, int TMAX, class A>
hipError_t dispatch_T(unsigned T, const A& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<TMIN, TMAX + 1>([&](auto I) {
        if (T == unsigned(decltype(I)::value)) e = Fn<decltype(I)::value>::run(a, s);
    });
    return e;
}
template <int T>
using EncHiSingle = EncHiFn<T, false>;
template <int T>
using EncHiMulti = EncHiFn<T, true>;

constexpr int kLoR = reg16(kLoBits), kLoS = split16(kLoBits);
constexpr unsigned kNarrowGrid = 256;  // workgroups: one per CU of an MI355X

}  // namespace

hipError_t launch_encode_fused16(unsigned T, const EncArgs& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 9>([&](auto I) {
        if (T == unsigned(decltype(I)::value)) e = EncFusedFn<FF16, decltype(I)::value>::run(a, s);
    });
    return e;
}
hipError_t launch_encode_lo(const EncArgs& a, hipStream_t s) {
    const unsigned m = 1u << a.Tm;
    return launch(&k_enc_lo<kLoR, kLoS>, dim3(tiles_for(a.nunits), m >> kLoBits, a.nchunks),
                  threads16(kLoBits, kLoR), lds16_dwords<kLoBits, kLoR, kLoS>(1, 0), s, &a);
}
hipError_t launch_encode_hi(const EncArgs& a, hipStream_t s) {
    if (a.nchunks > 1) return dispatch_T<EncHiMulti, 1, 6>(a.Tm - kLoBits, a, s);
    return dispatch_T<EncHiSingle, 1, 7>(a.Tm - kLoBits, a, s);
}
hipError_t launch_encode_fin(const EncArgs& a, hipStream_t s) {
    const unsigned tiles = (a.R + (1u << kLoBits) - 1) >> kLoBits;
    const dim3 grid(tiles_for(a.nunits), tiles);
    // A grid of at most one workgroup per CU (e.g. R <= 256 on 64 KiB pieces):
    // 16 pieces per lane in 16 waves (the whole 128 KiB exchange area, one
    // workgroup per CU) halve every wave's work where the 32-piece form would
    // leave 3 of 4 wave slots of each SIMD empty.
    if (grid.x * grid.y <= kNarrowGrid)
        return launch(&k_enc_fin<4, 0>, grid, threads16(kLoBits, 4), lds16_dwords<kLoBits, 4, 0>(1, 0), s, &a);
    return launch(&k_enc_fin<kLoR, kLoS>, grid, threads16(kLoBits, kLoR), lds16_dwords<kLoBits, kLoR, kLoS>(1, 0), s,
                  &a);
}
hipError_t launch_decode_lo(const DecArgs& a, hipStream_t s) {
    return launch(&k_dec_lo<kLoR, kLoS>, dim3(tiles_for(a.nunits), a.nlo), threads16(kLoBits, kLoR),
                  lds16_dwords<kLoBits, kLoR, kLoS>(1, 1 << kLoBits), s, &a);
}
hipError_t launch_decode_hi(const DecArgs& a, hipStream_t s) {
    return dispatch_T<DecHiFn, 1, 8>(a.Tn - kLoBits, a, s);
}
hipError_t launch_decode_hi_half(const DecArgs& a, hipStream_t s) {
    return dispatch_T<DecHiHalfFn, 1, 7>(a.Tn - 1 - kLoBits, a, s);
}
hipError_t launch_decode_fin(const DecArgs& a, hipStream_t s) {
    const unsigned n = 1u << a.Tn;
    return launch(&k_dec_fin<kLoR, kLoS>, dim3(tiles_for(a.nunits), n >> kLoBits), threads16(kLoBits, kLoR),
                  lds16_dwords<kLoBits, kLoR, kLoS>(1, 1 << kLoBits), s, &a);
}
hipError_t launch_error_locator16(const uint32_t* erased, const uint32_t* walsh, uint32_t* tmp, uint32_t* el,
                                  uint32_t* scale_logs, uint32_t* reveal_logs, unsigned m, unsigned K, unsigned R,
                                  hipStream_t s) {
    hipLaunchKernelGGL(k_el16_rows, dim3(256), dim3(64), 0, s, erased, tmp, el, scale_logs, reveal_logs, 0, m, K, R);
    hipLaunchKernelGGL(k_el16_cols, dim3(256), dim3(64), 0, s, tmp, walsh);
    hipLaunchKernelGGL(k_el16_rows, dim3(256), dim3(64), 0, s, erased, tmp, el, scale_logs, reveal_logs, 1, m, K, R);
    return hipGetLastError();
}
hipError_t launch_xor_reduce(const XorArgs& a, hipStream_t s) {
    const unsigned blocks = unsigned((a.ndwords / 4 + 255) / 256);
    hipLaunchKernelGGL(k_xor_reduce, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace lamd
