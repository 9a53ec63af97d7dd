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

// pass 1: IFFT over the low kLoBits of chunk blockIdx.z -> slab_out[c*m + g]
template <class F>
__global__ void __launch_bounds__(64 << wave_bits(kLoBits), 4) k_enc_lo(EncArgs a) {
    constexpr int T = kLoBits;
    using TL = Tile<F, T, reg_bits(T), C>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    GlobalWindow<F> win;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t q0 = lane_units(lane);
    const bool live = q0 < a.nunits;
    const uint64_t ql = live ? q0 : a.nunits - C;
    const unsigned m = 1u << a.Tm;
    const unsigned c = blockIdx.z, base = c * m;
    const PieceSpace ps{0, 0, blockIdx.y << T};
    typename TL::Reg x;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned g = ps.global(TL::piece(0, r, w));
        load_or_zero<F>(x[r], a.in, base + g < a.K, base + g, a.zeros, ql);
    }
    win.stage(a.sktab, int(m - 1 + base));
    TL::ifft(x, w, lane, lds, ps, win, BelowLive{a.K - base});
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned g = ps.global(TL::piece(TL::kLast, r, w));
        store_units<F, C>(a.slab_out.ptr(base + g), q0, x[r]);
    }
}

// pass 2: for every chunk IFFT over the high bits and accumulate; then the
// FFT over the high bits -> slab_out[g]
template <class F, int T>
__global__ void __launch_bounds__(64 << wave_bits(T), 4) k_enc_hi(EncArgs a) {
    using TL = Tile<F, T, reg_bits(T), C>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    GlobalWindow<F> win;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t q0 = lane_units(lane);
    const bool live = q0 < a.nunits;
    const uint64_t ql = live ? q0 : a.nunits - C;
    const unsigned m = 1u << a.Tm;
    const PieceSpace ps{blockIdx.y, kLoBits, 0};
    typename TL::Reg acc, x;
    for (unsigned c = 0; c < a.nchunks; ++c) {
        const unsigned base = c * m;
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const unsigned tp = TL::piece(0, r, w);
            // low tiles that lie entirely past K were all-zero inputs
            load_or_zero<F>(x[r], a.slab_in, base + (tp << kLoBits) < a.K, base + ps.global(tp), a.zeros, ql);
        }
        win.stage(a.sktab, int(m - 1 + base));
        TL::template ifft<true>(x, w, lane, lds, ps, win, BelowLive{a.K - base});
        TL::fused_top(x, F::tab(a.tabs, cload(a.fused + c)));  // top of the m-transform: this pass's top bit
        if (c == 0) TL::copy(acc, x);
        else TL::xor_into(acc, x);
    }
    win.stage(a.sktab, -1);
    TL::template fft<true>(acc, w, lane, lds, ps, win, BelowLive{a.R});
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned g = ps.global(TL::piece(0, r, w));
        store_units<F, C>(a.slab_out.ptr(g), q0, acc[r]);
    }
}

// pass 3: FFT over the low bits, keep outputs g < R.  When m = 2^kLoBits (no
// high pass) the chunk IFFTs of pass 1 are combined here: x = XOR_c U[c*m + g].
template <class F>
__global__ void __launch_bounds__(64 << wave_bits(kLoBits), 4) k_enc_fin(EncArgs a) {
    constexpr int T = kLoBits;
    using TL = Tile<F, T, reg_bits(T), C>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    GlobalWindow<F> win;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t q0 = lane_units(lane);
    const bool live = q0 < a.nunits;
    const uint64_t ql = live ? q0 : a.nunits - C;
    const PieceSpace ps{0, 0, blockIdx.y << T};
    typename TL::Reg x;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) load_units<F, C>(x[r], a.slab_in.ptr(ps.global(TL::piece(TL::kLast, r, w))), ql);
    if (a.Tm == unsigned(kLoBits))
        for (unsigned c = 1; c < a.nchunks; ++c) {
            typename TL::Reg y;
#pragma unroll
            for (int r = 0; r < TL::NR; ++r)
                load_units<F, C>(y[r], a.slab_in.ptr((c << T) + ps.global(TL::piece(TL::kLast, r, w))), ql);
            TL::xor_into(x, y);
        }
    win.stage(a.sktab, -1);
    TL::fft(x, w, lane, lds, ps, win, BelowLive{a.R});
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned g = ps.global(TL::piece(0, r, w));
        if (g < a.R) store_units<F, C>(a.out.ptr(g), q0, x[r]);
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

// FF16 decoder state in device memory: erasure bitmap (bit p <=>
// error_locations[p] = 1, LeopardFF8.cpp:1825-1840) and error locator logs.
// Multiply tables by log value come through the scalar cache.
struct State16 {
    const uint32_t* bits;
    const uint32_t* el;
    const uint32_t* tabs;
    LDEV bool erased(unsigned p) const { return bit_set(bits, p); }
    LDEV unsigned loc(unsigned p) const { return cload(el + p); }
    LDEV FF16::Tab table(unsigned lm) const { return FF16::tab(tabs, lm); }
};

// Received piece at codeword position p (to be scaled by exp(el[p])); zero if
// absent.  Positions: [0, m) recovery (only [0, R) exist), [m, m+K) originals
// (LeopardFF8.cpp:1857-1877).  Branch-free on the vector side: an absent piece
// reads the zero page at unit 0 and is scaled through the all-zero table.
// Returns the log of the scale factor.
template <class F, class St>
LDEV unsigned load_received(uint32_t* x, const DecArgs& a, const St& st, unsigned p, uint64_t q) {
    const uint8_t* src = a.zeros;
    unsigned lm = F::kModulus + 1;  // the zero table
    uint64_t qq = 0;
    if (!st.erased(p)) {
        if (p < a.R) { src = a.rec.ptr(p); lm = st.loc(p); qq = q; }
        else if (p >= a.m && p < a.m + a.K) { src = a.orig.ptr(p - a.m); lm = st.loc(p); qq = q; }
    }
    load_units<F, C>(x, src, qq);
    return lm;
}

// Lost original at position p = m + i: work[i] = z[p] * exp(-el[p])  (LeopardFF8.cpp:1913-1915).
template <class F, class St>
LDEV void reveal(const uint32_t* z, const DecArgs& a, const St& st, unsigned p, uint64_t q0) {
    if (p >= a.m && p < a.m + a.K && st.erased(p)) {
        uint32_t y[C * F::kDw];
        const typename F::Tab t = st.table(F::kModulus - st.loc(p));
#pragma unroll
        for (int u = 0; u < C; ++u) F::mul(&y[u * F::kDw], &z[u * F::kDw], t);
        store_units<F, C>(a.out.ptr(p - a.m), q0, y);
    }
}

// pass 1: scale-on-load + IFFT over the low bits -> a_out[g]
template <class F>
__global__ void __launch_bounds__(64 << wave_bits(kLoBits), 4) k_dec_lo(DecArgs a) {
    constexpr int T = kLoBits;
    using TL = Tile<F, T, reg_bits(T), C>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    GlobalWindow<F> win;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t q0 = lane_units(lane);
    const bool live = q0 < a.nunits;
    const uint64_t ql = live ? q0 : a.nunits - C;
    const PieceSpace ps{0, 0, blockIdx.y << T};
    const State16 st{a.erased_dev, a.el, a.tabs};
    typename TL::Reg v;
    // every piece load in flight first, then the scale multiplies (one table
    // live at a time)
    unsigned lm[TL::NR];
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) lm[r] = load_received<F>(v[r], a, st, ps.global(TL::piece(0, r, w)), ql);
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const typename F::Tab t = st.table(lm[r]);
#pragma unroll
        for (int u = 0; u < C; ++u) F::mul(&v[r][u * F::kDw], &v[r][u * F::kDw], t);
        __builtin_amdgcn_sched_barrier(0);
    }
    win.stage(a.sktab, -1);
    TL::ifft(v, w, lane, lds, ps, win, Pyr16Live{a.present_pyr});
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) store_units<F, C>(a.a_out.ptr(ps.global(TL::piece(TL::kLast, r, w))), q0, v[r]);
}

// pass 2: A = F_hi (I + D_hi) I_hi U over the high bits, computed as
// F_hi' (swap_top + D_hi') I_hi' U without the top layers (Tile::derivative_swaptop).
// The other term of the split derivative needs F_hi(I_hi U) = U, which pass 3
// reads straight from pass 1's slab.
template <class F, int T>
__global__ void __launch_bounds__(64 << wave_bits(T), 4) k_dec_hi(DecArgs a) {
    using TL = Tile<F, T, reg_bits(T), C>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    GlobalWindow<F> win;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t q0 = lane_units(lane);
    const bool live = q0 < a.nunits;
    const uint64_t ql = live ? q0 : a.nunits - C;
    const PieceSpace ps{blockIdx.y, kLoBits, 0};
    typename TL::Reg v;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned tp = TL::piece(0, r, w);
        load_or_zero<F>(v[r], a.a_in, tp < a.nlo, ps.global(tp), a.zeros, ql);
    }
    win.stage(a.sktab, -1);
    TL::template ifft<true>(v, w, lane, lds, ps, win, Pyr16Live{a.present_pyr});
    TL::derivative_swaptop(v, w, lane, lds, true);
    TL::template fft<true>(v, w, lane, lds, ps, win, Pyr16Live{a.needed_pyr});
    if (live)
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) store_units<F, C>(a.a_out.ptr(ps.global(TL::piece(0, r, w))), q0, v[r]);
}

// pass 2 when every received piece is in the low half (K = R, every original
// lost; see k_ff8_dec_half in rs_ff8.hip): the high IFFT layers of the low
// half, the fused top layer of the m-transform (encoder chunk 0's table) and the
// high FFT layers with the skews of the high half; A is written at the high
// positions only and pass 3 adds D_lo(U) = 0 there (U has no high tiles).
template <class F, int T>
__global__ void __launch_bounds__(64 << wave_bits(T), 4) k_dec_hi_half(DecArgs a) {
    using TL = Tile<F, T, reg_bits(T), C>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    GlobalWindow<F> win;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t q0 = lane_units(lane);
    const bool live = q0 < a.nunits;
    const uint64_t ql = live ? q0 : a.nunits - C;
    const PieceSpace low{blockIdx.y, kLoBits, 0}, high{blockIdx.y, kLoBits, a.m};
    typename TL::Reg v;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned tp = TL::piece(0, r, w);
        load_or_zero<F>(v[r], a.a_in, tp < a.nlo, low.global(tp), a.zeros, ql);
    }
    win.stage(a.sktab, -1);
    TL::template ifft<true>(v, w, lane, lds, low, win, Pyr16Live{a.present_pyr});
    TL::fused_top(v, F::tab(a.tabs, cload(a.fused)));
    TL::template fft<true>(v, w, lane, lds, high, win, Pyr16Live{a.needed_pyr});
    if (live)
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) store_units<F, C>(a.a_out.ptr(high.global(TL::piece(0, r, w))), q0, v[r]);
}

// pass 3: z = A + D_lo(U), FFT over the low bits, reveal lost originals (U of
// a low tile without received data is zero and was never written)
template <class F>
__global__ void __launch_bounds__(64 << wave_bits(kLoBits), 4) k_dec_fin(DecArgs a) {
    constexpr int T = kLoBits;
    using TL = Tile<F, T, reg_bits(T), C>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    // skip tiles holding no lost original (uniform across the workgroup)
    {
        const unsigned L = T, j = blockIdx.y;
        if (!((cload(a.needed_pyr + pyr_offset(L) + (j >> 5)) >> (j & 31)) & 1u)) return;
    }
    GlobalWindow<F> win;
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t q0 = lane_units(lane);
    const bool live = q0 < a.nunits;
    const uint64_t ql = live ? q0 : a.nunits - C;
    const PieceSpace ps{0, 0, blockIdx.y << T};
    const State16 st{a.erased_dev, a.el, a.tabs};
    typename TL::Reg z;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) load_units<F, C>(z[r], a.a_in.ptr(ps.global(TL::piece(TL::kLast, r, w))), ql);
    win.stage(a.sktab, -1);
    // U of a tile past the received ones is zero, and so is D_lo(U) (workgroup-uniform)
    if (blockIdx.y < a.nlo) {
        typename TL::Reg v;
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) load_units<F, C>(v[r], a.b_in.ptr(ps.global(TL::piece(TL::kLast, r, w))), ql);
        TL::derivative_add(z, v, w, lane, lds);
    }
    TL::fft(z, w, lane, lds, ps, win, Pyr16Live{a.needed_pyr});
    if (!live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        reveal<F>(z[r], a, st, ps.global(TL::piece(0, r, w)), q0);
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

// mode 0: rows of the erasure bitmap -> tmp; mode 1: rows of tmp -> el (u16)
__global__ void __launch_bounds__(64) k_el16_rows(const uint32_t* erased, uint32_t* tmp, uint32_t* el, int mode) {
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
        if (mode == 0) tmp[p] = e[j];
        else el[p] = e[j];
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
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (unsigned i = 0; i < a.count; ++i) {
        const uint8_t* p = a.src.ptr(i);
        const uint4 v = *gptr<const uint4>(p + q * 4);
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    *gptr<uint4>(a.out.ptr(0) + q * 4) = acc;
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
template <class F, int T>
struct EncHiFn {
    static hipError_t run(const EncArgs& a, hipStream_t s) {
        return launch(&k_enc_hi<F, T>, dim3(tiles_for(a.nunits), 1u << kLoBits), 64u << wave_bits(T),
                      full_tile_lds<F, T>(), s, &a);
    }
};
template <class F, int T>
struct DecHiFn {
    static hipError_t run(const DecArgs& a, hipStream_t s) {
        return launch(&k_dec_hi<F, T>, dim3(tiles_for(a.nunits), 1u << kLoBits), 64u << wave_bits(T),
                      full_tile_lds<F, T>(), s, &a);
    }
};

template <class F, int T>
struct DecHiHalfFn {
    static hipError_t run(const DecArgs& a, hipStream_t s) {
        return launch(&k_dec_hi_half<F, T>, dim3(tiles_for(a.nunits), 1u << kLoBits), 64u << wave_bits(T),
                      full_tile_lds<F, T>(), s, &a);
    }
};

template <template <class, int> class Fn, class F, int TMIN, int TMAX, class A>
hipError_t dispatch_T(unsigned T, const A& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<TMIN, TMAX + 1>([&](auto I) {
        if (T == unsigned(decltype(I)::value)) e = Fn<F, decltype(I)::value>::run(a, s);
    });
    return e;
}

}  // namespace

hipError_t launch_encode_fused16(unsigned T, const EncArgs& a, hipStream_t s) {
    return dispatch_T<EncFusedFn, FF16, 1, 8>(T, a, s);
}
hipError_t launch_encode_lo(const EncArgs& a, hipStream_t s) {
    const unsigned m = 1u << a.Tm;
    return launch(&k_enc_lo<FF16>, dim3(tiles_for(a.nunits), m >> kLoBits, a.nchunks), 64u << wave_bits(kLoBits),
                  full_tile_lds<FF16, kLoBits>(), s, &a);
}
hipError_t launch_encode_hi(const EncArgs& a, hipStream_t s) {
    return dispatch_T<EncHiFn, FF16, 1, 8>(a.Tm - kLoBits, a, s);
}
hipError_t launch_encode_fin(const EncArgs& a, hipStream_t s) {
    const unsigned tiles = (a.R + (1u << kLoBits) - 1) >> kLoBits;
    return launch(&k_enc_fin<FF16>, dim3(tiles_for(a.nunits), tiles), 64u << wave_bits(kLoBits),
                  full_tile_lds<FF16, kLoBits>(), s, &a);
}
hipError_t launch_decode_lo(const DecArgs& a, hipStream_t s) {
    return launch(&k_dec_lo<FF16>, dim3(tiles_for(a.nunits), a.nlo), 64u << wave_bits(kLoBits),
                  full_tile_lds<FF16, kLoBits>(), s, &a);
}
hipError_t launch_decode_hi(const DecArgs& a, hipStream_t s) {
    return dispatch_T<DecHiFn, FF16, 1, 8>(a.Tn - kLoBits, a, s);
}
hipError_t launch_decode_hi_half(const DecArgs& a, hipStream_t s) {
    return dispatch_T<DecHiHalfFn, FF16, 1, 7>(a.Tn - 1 - kLoBits, a, s);
}
hipError_t launch_decode_fin(const DecArgs& a, hipStream_t s) {
    const unsigned n = 1u << a.Tn;
    return launch(&k_dec_fin<FF16>, dim3(tiles_for(a.nunits), n >> kLoBits), 64u << wave_bits(kLoBits),
                  full_tile_lds<FF16, kLoBits>(), s, &a);
}
hipError_t launch_error_locator16(const uint32_t* erased, const uint32_t* walsh, uint32_t* tmp, uint32_t* el,
                                  hipStream_t s) {
    hipLaunchKernelGGL(k_el16_rows, dim3(256), dim3(64), 0, s, erased, tmp, el, 0);
    hipLaunchKernelGGL(k_el16_cols, dim3(256), dim3(64), 0, s, tmp, walsh);
    hipLaunchKernelGGL(k_el16_rows, dim3(256), dim3(64), 0, s, erased, tmp, el, 1);
    return hipGetLastError();
}
hipError_t launch_xor_reduce(const XorArgs& a, hipStream_t s) {
    const unsigned blocks = unsigned((a.ndwords / 4 + 255) / 256);
    hipLaunchKernelGGL(k_xor_reduce, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace lamd
