// rs_ff8.hip -- GF(2^8) encode / decode kernels (codeword length n <= 256) for gfx950.
//
// One workgroup = the whole transform (2^T pieces) over one 256-byte column
// strip: 64 lanes x one dword column each, pieces spread over registers and
// waves by the tile engine (rs_device.h).  Reference paths:
//   encode  ReedSolomonEncode  LeopardFF8.cpp:1602-1672
//     work = XOR_c IFFT_m(data chunk c, skew + m-1 + c*m);  out = FFT_m(work, skew - 1)[0, R)
//   decode  ReedSolomonDecode  LeopardFF8.cpp:1809-1916
//     v = IFFT_n(received * exp(el));  z = FormalDerivative(v);  lost i = FFT_n(z)[m+i] * exp(-el[m+i])
//
// Launch data (piece pointers, erasure pyramids, error locator) arrives by
// value in the kernel arguments (rs_args.h), so the prologue is scalar loads of
// kernel arguments and one batch of piece loads.  Butterfly tables are staged
// once per workgroup into LDS (TabStage8).
//
// The encoder runs the top IFFT layer and the top FFT layer as one butterfly
// (Tile::fused_top): c1*y + c2*y = (c1 + c2)*y, one multiply layer fewer.  By
// linearity of the FFT this also holds per chunk when several chunks are
// accumulated (FFT(sum) = F_low(sum of F_top(chunk IFFTs))).
#include <hip/hip_runtime.h>

#include <mutex>

#include "rs_args.h"

namespace lamd {

#ifdef LAMD_STAMPS
// Diagnostic builds only (tools/stamps.sh): per-wave s_memrealtime stamps at
// phase boundaries, each after draining every outstanding memory operation.
__device__ uint64_t* g_stamps;
#define STAMP(k)                                                                                     \
    do {                                                                                             \
        __builtin_amdgcn_s_waitcnt(0);                                                               \
        const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                        \
        if ((threadIdx.x & 63) == 0)                                                                 \
            g_stamps[(uint64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (k)] = t_; \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif

namespace {

#ifndef LAMD_FF8_RB7  // experiment hook: register bits of the 7-bit tile
#define LAMD_FF8_RB7 3
#endif
#ifndef LAMD_FF8_SGPR_TABS  // experiment hook: butterfly tables through the scalar cache
#define LAMD_FF8_SGPR_TABS 0
#endif
#ifndef LAMD_FF8_RB8
#define LAMD_FF8_RB8 4
#endif
constexpr int reg_bits8(int T) {
    return T <= 3 ? T : T == 7 ? LAMD_FF8_RB7 : T == 8 ? LAMD_FF8_RB8 : (T - 3 <= 4 ? 3 : T - 4);
}
constexpr int wave_bits8(int T) { return T - reg_bits8(T); }
constexpr unsigned threads8(int T) { return 64u << wave_bits8(T); }
constexpr size_t tile_dwords8(int T) { return wave_bits8(T) > 0 ? (size_t(1) << T) * 64 : 0; }

// This lane's column inside the workgroup's 64-dword strip.  Lanes past the
// end of the pieces (last strip, B/4 not a multiple of 64) read the last valid
// dword and never store.
struct Cols {
    uint64_t base;      // byte offset of the strip (wave-uniform)
    uint32_t lane_off;  // byte offset of this lane's dword inside the strip
    bool live;
};
LDEV Cols strip_cols(uint32_t nunits, unsigned lane) {
    const uint32_t first = blockIdx.x * 64u;
    const uint32_t left = nunits - first;
    return Cols{uint64_t(first) * 4, (lane < left ? lane : left - 1) * 4, lane < left};
}
// piece pointer (kernel argument, wave-uniform) + strip base stay scalar: the
// access is global_load/store with an SGPR base and the lane's VGPR offset.
LDEV uint32_t gload(uint64_t piece, const Cols& c) {
    return *gptr<const uint32_t>(reinterpret_cast<const uint8_t*>(piece + c.base) + c.lane_off);
}
LDEV void gstore(uint64_t piece, const Cols& c, uint32_t v) {
    *gptr<uint32_t>(reinterpret_cast<uint8_t*>(piece + c.base) + c.lane_off) = v;
}

// --------------------------------------------------------------- encode -----

template <int T, bool kMulti>
__global__ void __launch_bounds__(threads8(T), 4) k_ff8_enc(Ff8EncArgs a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    using TL = Tile<FF8, T, reg_bits8(T), 1>;
    constexpr unsigned m = 1u << T;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const LdsTab8<256> tabs{lds + tile_dwords8(T)};
    STAMP(0);
    TabStage8<threads8(T), 256> stage;
    if constexpr (!LAMD_FF8_SGPR_TABS) stage.load(a.sktab);  // issued ahead of the piece loads
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols cl = strip_cols(a.nunits, lane);
    const PieceSpace ps{0, 0, 0};
    typename TL::Reg x;
    auto load_chunk = [&](unsigned c) {
        const unsigned base = c * m;
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) {
            const unsigned i = base + TL::piece(0, r, w);
            x[r][0] = i < a.K ? gload(a.ptr[i], cl) : 0u;  // past K: zero padding (LeopardFF8.cpp:1631-1634)
        }
    };
    load_chunk(0);
    STAMP(1);
    if constexpr (!LAMD_FF8_SGPR_TABS) {
        stage.store(tabs);
        __syncthreads();
    }
    STAMP(2);
#if LAMD_FF8_SGPR_TABS
    GlobalWindow<FF8> win;
#else
    LdsSkew8 win{tabs};
#endif
    if constexpr (!kMulti) {
        win.stage(a.sktab, int(m - 1));
        TL::template ifft<true>(x, w, lane, lds, ps, win, BelowLive{a.K});
        STAMP(3);
        TL::fused_top(x, FF8::tab_at(a.fused));
        win.stage(a.sktab, -1);
        TL::template fft<true>(x, w, lane, lds, ps, win, BelowLive{a.R});
        STAMP(4);
    } else {
        typename TL::Reg acc;
        for (unsigned c = 0;;) {
            win.stage(a.sktab, int(m - 1 + c * m));
            TL::template ifft<true>(x, w, lane, lds, ps, win, BelowLive{a.K - c * m});
            TL::fused_top(x, FF8::tab_at(a.fused + c * FF8::kTabDw));
            if (c == 0) TL::copy(acc, x);
            else TL::xor_into(acc, x);
            if (++c >= a.nchunks) break;
            load_chunk(c);
        }
        TL::copy(x, acc);
        win.stage(a.sktab, -1);
        TL::template fft<true>(x, w, lane, lds, ps, win, BelowLive{a.R});
    }
    TL::pin(x);
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned tp = TL::piece(0, r, w);
        if (tp < a.R) gstore(a.ptr[a.K + tp], cl, x[r][0]);
    }
    STAMP(5);
}

// --------------------------------------------------------------- decode -----

LDEV unsigned el_at(const Ff8DecArgs& a, unsigned p) { return (a.el[p >> 2] >> ((p & 3) * 8)) & 0xFFu; }

template <int T>
__global__ void __launch_bounds__(threads8(T), 4) k_ff8_dec(Ff8DecArgs a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    using F = FF8;
    using TL = Tile<F, T, reg_bits8(T), 1>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const LdsTab8<256> sk{lds + tile_dwords8(T)};
    const LdsTab8<256> ltab{sk.base + LdsTab8<256>::kDwords};  // by log value
    STAMP(0);
    TabStage8<threads8(T), 256> sk_stage, log_stage;
    sk_stage.load(a.sktab);
    log_stage.load(a.tabs);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols cl = strip_cols(a.nunits, lane);
    const PieceSpace ps{0, 0, 0};
    const Pyr8Live present{a.present}, needed{a.needed};
    typename TL::Reg v;
    // received pieces: positions [0, R) recovery, [m, m + K) originals (LeopardFF8.cpp:1857-1877)
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned p = TL::piece(0, r, w);
        v[r][0] = present(p, 0) ? gload(a.ptr[p], cl) : 0u;
    }
    STAMP(1);
    sk_stage.store(sk);
    log_stage.store(ltab);
    __syncthreads();
    STAMP(2);
    // scale by exp(el) (absent pieces stay zero)
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned p = TL::piece(0, r, w);
        if ((LAMD_ABLATE & 128) == 0 && present(p, 0)) F::mul(v[r], v[r], ltab.at(int(el_at(a, p))));
    }
#if LAMD_FF8_SGPR_TABS
    GlobalWindow<FF8> win;
#else
    LdsSkew8 win{sk};
#endif
    win.stage(a.sktab, -1);
    TL::ifft(v, w, lane, lds, ps, win, present);
    STAMP(3);
    TL::derivative_inplace(v, w, lane, lds);
    STAMP(4);
    TL::fft(v, w, lane, lds, ps, win, needed);
    STAMP(5);
    TL::pin(v);
    if (!cl.live) return;
    // lost original at p = m + i: work[i] = z[p] * exp(-el[p])  (LeopardFF8.cpp:1913-1915)
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned p = TL::piece(0, r, w);
        if (needed(p, 0)) {
            uint32_t y[1] = {v[r][0]};
            if constexpr ((LAMD_ABLATE & 128) == 0) F::mul(y, v[r], ltab.at(int(F::kModulus - el_at(a, p))));
            gstore(a.ptr[p], cl, y[0]);
        }
    }
    STAMP(6);
}

// Opting a kernel into > 64 KiB of LDS is a per-function attribute, set once
// per kernel (Once is a distinct type per kernel instantiation).
template <class Tag>
struct Once {
    static hipError_t set_lds(const void* fn, size_t lds) {
        static std::once_flag once;
        static hipError_t attr = hipSuccess;
        std::call_once(once, [&] { attr = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)); });
        return attr;
    }
};
template <class Tag, class KernelFn, class Args>
hipError_t launch8(KernelFn* fn, unsigned T, const Args& a, size_t lds_dwords, hipStream_t s) {
    const size_t lds = lds_dwords * 4;
    if (lds > 65536) {
        const hipError_t e = Once<Tag>::set_lds(reinterpret_cast<const void*>(fn), lds);
        if (e != hipSuccess) return e;
    }
    void* params[] = {const_cast<Args*>(&a)};
    const dim3 grid((a.nunits + 63) / 64);
    return hipLaunchKernel(reinterpret_cast<const void*>(fn), grid, dim3(threads8(int(T))), params, lds, s);
}

template <int T, bool M>
struct EncTag {};
template <int T>
struct DecTag {};

template <int T>
hipError_t enc_T(const Ff8EncArgs& a, hipStream_t s) {
    constexpr size_t lds = tile_dwords8(T) + LdsTab8<256>::kDwords;
    if (a.nchunks > 1) return launch8<EncTag<T, true>>(&k_ff8_enc<T, true>, T, a, lds, s);
    return launch8<EncTag<T, false>>(&k_ff8_enc<T, false>, T, a, lds, s);
}
template <int T>
hipError_t dec_T(const Ff8DecArgs& a, hipStream_t s) {
    return launch8<DecTag<T>>(&k_ff8_dec<T>, T, a, tile_dwords8(T) + 2 * LdsTab8<256>::kDwords, s);
}

}  // namespace

#ifdef LAMD_STAMPS
extern "C" __attribute__((visibility("default"))) int leo_amd_debug_stamps(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_ff8_encode(unsigned T, const Ff8EncArgs& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 8>([&](auto I) {
        if (T == unsigned(decltype(I)::value)) e = enc_T<decltype(I)::value>(a, s);
    });
    return e;
}

hipError_t launch_ff8_decode(unsigned T, const Ff8DecArgs& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 9>([&](auto I) {
        if (T == unsigned(decltype(I)::value)) e = dec_T<decltype(I)::value>(a, s);
    });
    return e;
}

}  // namespace lamd
