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

#include <cstdlib>
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
#ifdef LAMD_CLOCK
// Diagnostic builds only (tools/clock.py): per workgroup of the slab batch
// kernel, (s_memtime, s_memrealtime) at entry and exit of wave 0, for the
// in-kernel shader clock (MI355X_MICROARCH.md "DVFS give-back" item 6).
__device__ uint64_t* g_clock;
#endif

namespace {

// Register bits per lane of a T-bit tile (the remaining piece bits index the
// wave): 8 pieces per lane up to 16 waves, 16 pieces for the 8-bit decoder
// tile.  The encoder's 7-bit tile also has a 16-pieces-per-lane form (8 waves,
// one LDS transpose per transform instead of two) that wins once every CU runs
// several workgroups (large pieces); with one workgroup per CU the 16-wave form
// hides more latency (measured: 64 KiB pieces 10.5 vs 11.1 us, 1 MiB 87 vs 79 us).
// Tables through the scalar cache instead of LDS measured slower (decode +15%).
constexpr int reg_bits8(int T) { return T <= 3 ? T : (T - 3 <= 4 ? 3 : T - 4); }
constexpr int wide_bits8(int T) { return T == 7 ? 4 : reg_bits8(T); }
constexpr unsigned threads_for(int T, int RB) { return 64u << (T - RB); }
constexpr size_t tile_dwords_for(int T, int RB) { return T > RB ? (size_t(1) << T) * 64 : 0; }
constexpr int wide_dec_bits8(int T) { return T == 8 ? 5 : reg_bits8(T); }
// Batched launches hold many workgroups per CU: their 7- and 8-bit tiles use
// 16 / 32 pieces per lane (8-wave workgroups, one transpose per transform,
// four workgroups per CU).  Measured, 16 objects of 128+128 x 64 KiB per
// batch: 632 GB/s vs 557 with the 16-wave tiles of the single calls and 532
// with 32 pieces per lane (LAMD_BATCH_BITS8 = 3 / 5; 0 = the single-call tiles).
#ifndef LAMD_BATCH_BITS8
#define LAMD_BATCH_BITS8 4
#endif
constexpr int batch_bits8(int T) { return LAMD_BATCH_BITS8 && T >= 7 ? LAMD_BATCH_BITS8 : reg_bits8(T); }

// Transforms: the plain ones (Tile::ifft / fft: one LDS area, two barriers
// per exchange) by default; LAMD_FF8_PIPE=1 builds the pipelined ones
// (Tile::ifft_pl / fft_pl: lookahead of tables and predicate words, two
// exchange areas, one barrier per exchange) for launches of at most one
// workgroup per CU.  Measured on MI355X, 128+128 pieces: pipelined is 3%
// faster for one 64 KiB encode on an idle GPU, but its LDS footprint keeps
// kernels of concurrent calls from sharing a CU (3 calls in flight: 22.6 vs
// 15.8 us per encode+decode step) and at 1 MiB pieces it is 10-15% slower.
#ifndef LAMD_FF8_PIPE
#define LAMD_FF8_PIPE 0
#endif
constexpr bool kPipe8 = LAMD_FF8_PIPE != 0;
constexpr bool pipe8(int NA) { return kPipe8 && NA == 2; }
constexpr int areas8(int NA) { return pipe8(NA) ? 2 : 1; }

constexpr uint32_t kOneWgPerCuUnits = 256 * 64;  // 256 CUs x one 64-dword strip
// Encoder lane groups (k_ff8_enc<..., G>): G = 1, 2 split a wave into 2^G
// column strips of different pieces, so a 64 KiB call runs 2^G workgroups per
// CU.  Bit-exact (tests/test_gpu_parity.py::test_encoder_lane_group_forms) but
// measured slower on MI355X, 128+128 x 64 KiB encode: G = 0 10.4 us, G = 1
// 11.5, G = 2 11.9 (per-workgroup table staging and per-lane-group table reads
// outweigh the phase overlap; profiles/r01_v7/lane_groups_ab.txt), so the
// default stays 0 and LEO_AMD_FF8_G selects the others for experiments.
#ifndef LAMD_PRIO_LOADS
#define LAMD_PRIO_LOADS 0
#endif
// Window of the pruned (non-dense) tiles: LAMD_FF8_ZERO_CHECK=1 keeps the
// XOR-only branch for zero skews (rs_device.h: LdsSkew8NoZero)
#ifndef LAMD_FF8_ZERO_CHECK
#define LAMD_FF8_ZERO_CHECK 0
#endif
#if LAMD_FF8_ZERO_CHECK
struct Skew8Win : LdsSkew8 {};
#else
using Skew8Win = LdsSkew8NoZero;
#endif
#ifndef LAMD_FF8_ENC_G
#define LAMD_FF8_ENC_G 0
#endif
constexpr int kDefaultEncG = LAMD_FF8_ENC_G;

// Piece pointers of the NR pieces a lane holds, fetched as one batch of scalar
// loads: otherwise the compiler sinks each load into the branch that uses it,
// a chain of dependent scalar-load round trips before the piece loads issue.
template <int NR, class Get, class Idx>
LDEV void fetch_ptrs_by(uint64_t (&pp)[NR], Get get, Idx idx) {
#pragma unroll
    for (int r = 0; r < NR; ++r) pp[r] = get(idx(r));
#pragma unroll
    for (int r = 0; r < NR; ++r) asm volatile("" : "+s"(pp[r]));
}
template <int NR, class A, class Idx>
LDEV void fetch_ptrs(uint64_t (&pp)[NR], const A& a, Idx idx) {
    fetch_ptrs_by(pp, [&](unsigned i) { return a.piece(i); }, idx);
}

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
// Strips of LW < 64 dwords (lane groups of a wave hold different pieces): the
// strip index is XCD-major, so the neighbouring strips that share a 128-byte
// line run on one XCD (workgroups are dealt round-robin over the 8 XCDs).
template <int LW>
LDEV Cols strip_cols_lw(uint32_t nunits, unsigned lane) {
    const uint32_t nblk = gridDim.x, b = blockIdx.x;
    const uint32_t s = (nblk & 7u) == 0 ? (b & 7u) * (nblk >> 3) + (b >> 3) : b;
    const uint32_t first = s * uint32_t(LW);
    const uint32_t left = nunits - first;
    return Cols{uint64_t(first) * 4, (lane < left ? lane : left - 1) * 4, lane < left};
}
// piece pointer (kernel argument, wave-uniform) + strip base stay scalar: the
// access is global_load/store with an SGPR base and the lane's VGPR offset.
#ifndef LAMD_FF8_NT
#define LAMD_FF8_NT 1  // nontemporal piece I/O in the byte tiles (see gld in rs_device.h)
#endif
constexpr bool kFf8Nt = LAMD_FF8_NT != 0;
LDEV uint32_t gload(uint64_t piece, const Cols& c) {
    return gld<uint32_t, kFf8Nt>(reinterpret_cast<const uint8_t*>(piece + c.base) + c.lane_off);
}
LDEV void gstore(uint64_t piece, const Cols& c, uint32_t v) {
    gst<uint32_t, kFf8Nt>(reinterpret_cast<uint8_t*>(piece + c.base) + c.lane_off, v);
}
// p: piece pointer with the strip base already added
LDEV uint32_t gload_at(uint64_t p, const Cols& c) {
    return gld<uint32_t, kFf8Nt>(reinterpret_cast<const uint8_t*>(p) + c.lane_off);
}
LDEV void gstore_at(uint64_t p, const Cols& c, uint32_t v) { gst<uint32_t, kFf8Nt>(reinterpret_cast<uint8_t*>(p) + c.lane_off, v); }

// Strip pointers of the NR consecutive pieces first, first + 1, ... (a lane's
// registers in layout 0 hold pieces r | w << RB): a slab view steps by its
// stride (one 64-bit scalar add per piece), a pointer table is read per piece.
template <int NR, class Get>
LDEV void run_ptrs(uint64_t (&pp)[NR], Get get, unsigned first, int32_t stride, bool slab, const Cols& c) {
    if (slab) {
        uint64_t p = get(first) + c.base;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            pp[r] = p;
            p += uint64_t(int64_t(stride));
        }
    } else {
#pragma unroll
        for (int r = 0; r < NR; ++r) pp[r] = get(first + r) + c.base;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) asm volatile("" : "+s"(pp[r]));
}
template <class A>
LDEV int32_t in_stride_of(const A& a) {
    if constexpr (A::kSlab) return a.in_stride;
    else return 0;
}
template <class A>
LDEV int32_t out_stride_of(const A& a) {
    if constexpr (A::kSlab) return a.out_stride;
    else return 0;
}

// --------------------------------------------------------------- encode -----

// A pruning predicate made wave-uniform: live if any lane's block is live (lane
// groups hold different pieces).  Running the butterflies of a dead block is
// harmless: an IFFT block without input stays zero, an FFT block without a
// needed output feeds no needed output.
template <class P>
struct AnyLane {
    P p;
    LDEV bool operator()(unsigned pos, unsigned level) const {
        return __builtin_amdgcn_ballot_w64(p(pos, level)) != 0;
    }
};
template <int G, class P>
LDEV auto lane_pred(const P& p) {
    if constexpr (G == 0) return p;
    else return AnyLane<P>{p};
}

// kForm (Ff8Form): kFormDenseEnc = one chunk with K = R = m (the 128+128
// headline shape): every block of both transforms is live and every tile piece
// is loaded and stored, so the pruning predicates and the per-piece bounds
// tests compile away (they were a third of the kernel's scalar instructions).
// kFormDenseDec = the same tile run as the inverse map, the full-loss decode of
// a K = R = m code (see launch_ff8_decode_full).
template <int T, int RB, bool kMulti, int NA, int G, int kForm = kFormGeneral, class A = Ff8EncArgs>
LDEV void ff8_enc(const A& a) {
    constexpr bool kDense = kForm != kFormGeneral;
    static_assert(!(kDense && kMulti), "dense = one chunk");
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    // G lane-group bits: the wave's 64 lanes hold 2^G column strips of LW lanes
    // for different pieces (virtual wave w = lane group above the real wave), so
    // a workgroup spans LW dwords of every piece and a 64 KiB call fills each CU
    // with 2^G independent workgroups whose load / butterfly / store phases overlap.
    constexpr int LW = 64 >> G;
    using TL = Tile<FF8, T, RB, 1, LW>;
    constexpr unsigned m = 1u << T;
    constexpr size_t kTile = tile_dwords_for(T, RB) >> G;
    constexpr unsigned kThreads = threads_for(T, RB) >> G;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const LdsTab8<256> tabs{lds + areas8(NA) * kTile};
    LdsRing<kTile, areas8(NA)> ring{lds};
    STAMP(0);
    TabStage8<kThreads, 256> stage;
    stage.load(a.sktab);  // issued ahead of the piece loads
    const unsigned wave = uniform(threadIdx.x >> 6);
    const unsigned lane = threadIdx.x & (LW - 1);
    const unsigned w = G == 0 ? wave : (((threadIdx.x & 63u) >> (6 - G)) << (T - RB - G)) | wave;
    const Cols cl = G == 0 ? strip_cols(a.nunits, lane) : strip_cols_lw<LW>(a.nunits, lane);
    const PieceSpace ps{0, 0, 0};
    typename TL::Reg x;
    // input pieces [0, K) and output pieces [0, R) through their own accessors:
    // no per-piece select between the two (a slab view's piece(i) compiles to a
    // dozen scalar instructions per piece, in front of the loads)
    auto in_ptr = [&](unsigned i) { return a.in_piece(i); };
    auto ptrs = [&](uint64_t (&pp)[TL::NR], auto idx) {
        if constexpr (G == 0) fetch_ptrs_by(pp, in_ptr, idx);
        else {
#pragma unroll
            for (int r = 0; r < TL::NR; ++r) pp[r] = a.in_piece(idx(r));  // per lane group
        }
    };
    auto load_chunk = [&](unsigned c) {
        const unsigned base = c * m;  // base + tp < nchunks * m <= K + m - 1 < 256
        uint64_t pp[TL::NR];
        if constexpr (G == 0) {
            static_assert(TL::lo(0) == 0, "layout 0: register r holds piece r | w << RB");
            run_ptrs(pp, in_ptr, base + TL::piece(0, 0, w), in_stride_of(a), A::kSlab, cl);
#pragma unroll
            for (int r = 0; r < TL::NR; ++r) {
                const unsigned i = base + TL::piece(0, r, w);
                if constexpr (kDense) x[r][0] = gload_at(pp[r], cl);
                else x[r][0] = i < a.K ? gload_at(pp[r], cl) : 0u;  // past K: zero padding (LeopardFF8.cpp:1631-1634)
            }
        } else {
            // per-lane pieces: branch-free, padding lanes re-read piece K - 1 and drop it
            // (the exec-masked form of the conditional load in the chunk loop gave
            // wrong results for a partial last chunk, e.g. 40 + 20 pieces)
            ptrs(pp, [&](int r) {
                const unsigned i = base + TL::piece(0, r, w);
                return i < a.K ? i : a.K - 1;
            });
            uint32_t v[TL::NR];
#pragma unroll
            for (int r = 0; r < TL::NR; ++r) v[r] = gload(pp[r], cl);
#pragma unroll
            for (int r = 0; r < TL::NR; ++r) x[r][0] = base + TL::piece(0, r, w) < a.K ? v[r] : 0u;
        }
    };
    // IFFT / FFT of one stage: pipelined (lookahead tables, ring of two LDS areas) or plain
    auto ifft = [&](const auto& win, const auto& pred) {
        if constexpr (pipe8(NA)) TL::template ifft_pl<true>(x, w, lane, ring, ps, win, pred);
        else TL::template ifft<true>(x, w, lane, lds, ps, win, pred);
    };
    auto fft = [&](const auto& win, const auto& pred) {
        if constexpr (pipe8(NA)) TL::template fft_pl<true>(x, w, lane, ring, ps, win, pred);
        else TL::template fft<true>(x, w, lane, lds, ps, win, pred);
    };
#if LAMD_PRIO_LOADS
    __builtin_amdgcn_s_setprio(3);  // experiments: issue this workgroup's loads ahead of other waves' butterflies
#endif
    load_chunk(0);
#if LAMD_PRIO_LOADS
    __builtin_amdgcn_s_setprio(0);
#endif
    // Output piece pointers (pointer-table args): fetched here, behind the
    // piece loads, as one batch -- fetched at the stores they were eight
    // dependent scalar-load round trips after the last butterfly (scalar loads
    // return out of order, so each use waited for every load before it).
    // Dense: out piece j is ptr[m + j], a compile-time offset, so the batch
    // merges into one 16-dword scalar load like the input pointers'.
    uint64_t po[TL::NR];
    if constexpr (G == 0 && !A::kSlab)
        fetch_ptrs_by(po, [&](unsigned j) { return kDense ? a.piece(m + j) : a.out_piece(j); },
                      [&](int r) { return TL::piece(0, r, w); });
    STAMP(1);
    stage.store(tabs);
    __syncthreads();
    STAMP(2);
    Skew8Win win{{tabs}};
    if constexpr (kDense) {
        // encode: IFFT skew base m - 1, FFT base -1; inverse: the other way round
        constexpr int kIfftOff = kForm == kFormDenseDec ? -1 : int(m - 1);
        constexpr int kFftOff = kForm == kFormDenseDec ? int(m - 1) : -1;
        ifft(LdsSkew8Fixed<kIfftOff>{{{tabs}}}, AllLive{});
        TL::fused_top(x, FF8::tab_at(a.fused));
        fft(LdsSkew8Fixed<kFftOff>{{{tabs}}}, AllLive{});
    } else if constexpr (!kMulti) {
        win.stage(nullptr, int(m - 1));
        ifft(win, lane_pred<G>(BelowLive{a.K}));
        STAMP(3);
        TL::fused_top(x, FF8::tab_at(a.fused));
        fft(LdsSkew8Fixed<-1>{{{tabs}}}, lane_pred<G>(BelowLive{a.R}));
        STAMP(4);
    } else {
        typename TL::Reg acc;
        for (unsigned c = 0;;) {
            win.stage(nullptr, int(m - 1 + c * m));
            ifft(win, lane_pred<G>(BelowLive{a.K - c * m}));
            TL::fused_top(x, FF8::tab_at(a.fused + c * FF8::kTabDw));
            if (c == 0) TL::copy(acc, x);
            else TL::xor_into(acc, x);
            if (++c >= a.nchunks) break;
            load_chunk(c);
        }
        TL::copy(x, acc);
        fft(LdsSkew8Fixed<-1>{{{tabs}}}, lane_pred<G>(BelowLive{a.R}));
    }
    TL::pin(x);
    uint64_t pp[TL::NR];
    if constexpr (G == 0 && A::kSlab)
        run_ptrs(pp, [&](unsigned j) { return a.out_piece(j); }, TL::piece(0, 0, w), out_stride_of(a), true, cl);
    else if constexpr (G == 0) {
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) pp[r] = po[r] + cl.base;
    } else {
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) pp[r] = a.out_piece(TL::piece(0, r, w)) + cl.base;  // tp < m: R + tp < 256
    }
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) {
        const unsigned tp = TL::piece(0, r, w);
        if (kDense || tp < a.R) gstore_at(pp[r], cl, x[r][0]);
    }
    STAMP(5);
}

template <int T, int RB, bool kMulti, int NA, int G, int kForm = kFormGeneral>
__global__ void __launch_bounds__(threads_for(T, RB) >> G, 4) k_ff8_enc(Ff8EncArgs a) {
    ff8_enc<T, RB, kMulti, NA, G, kForm>(a);
}
// Batched launch (leo_amd_encode_batch): object blockIdx.y of an array of
// argument blocks in device memory (read through the scalar cache like the
// kernel arguments of k_ff8_enc); one grid over every object's column strips.
template <int T, int RB, bool kMulti, int kForm = kFormGeneral>
__global__ void __launch_bounds__(threads_for(T, RB), 4) k_ff8_enc_batch(const Ff8EncArgs* __restrict__ objs) {
    ff8_enc<T, RB, kMulti, 1, 0, kForm>(objs[blockIdx.y]);
}

// Slab batch (leo_amd_encode_batch / decode_batch on slab-laid objects): the
// argument block of every object is in the kernel arguments, object blockIdx.y.
#ifndef LAMD_SLAB_WAVES
#define LAMD_SLAB_WAVES 4
#endif
template <int T, int RB, bool kMulti, int kForm = kFormGeneral>
__global__ void __launch_bounds__(threads_for(T, RB), LAMD_SLAB_WAVES) k_ff8_enc_slab(Ff8SlabBatch b) {
#ifdef LAMD_CLOCK
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
    ff8_enc<T, RB, kMulti, 1, 0, kForm>(Ff8SlabView(b, blockIdx.y));
#ifdef LAMD_CLOCK
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        uint64_t* o = g_clock + 4ull * (blockIdx.x + uint64_t(blockIdx.y) * gridDim.x);
        o[0] = c0; o[1] = r0; o[2] = c1; o[3] = r1;
    }
#endif
}

// --------------------------------------------------------------- decode -----

// Error locator of the decoders (LeopardFF8.cpp:1845-1853, FWHT :80-130):
//   el = FWHT( LogWalsh * FWHT(erasures) )  mod 255,
// a 256-point Walsh-Hadamard transform mod 255, twice.  k_el8 computes it once
// per erasure pattern (the host caches the result per workspace, keyed by the
// pattern: a repeated pattern launches nothing), one wave per pattern, 4
// positions a lane (p = 4 lane + j: one dword of el bytes per lane), six
// layers across lanes (__shfl_xor) and two in registers.  Fully reduced mod 255
// (the reference reduces partially, 255 standing for 0: the same residues; the
// multiply tables of log 0 and log 255 are the same, x * exp(0) = x * exp(255)).
// The decode kernels read it at their top (ElRegs).
struct Mod8 {
    LDEV static unsigned add(unsigned a, unsigned b) { const unsigned s = a + b; return s >= 255u ? s - 255u : s; }
    LDEV static unsigned sub(unsigned a, unsigned b) { const unsigned s = a + 255u - b; return s >= 255u ? s - 255u : s; }
};
// FWHT_2 {a, b} = {a + b, a - b}: position bits 0, 1 in registers, bits 2..7 = lane bits 0..5
LDEV void fwht256_mod255(unsigned (&e)[4], unsigned lane) {
    const unsigned a0 = Mod8::add(e[0], e[1]), a1 = Mod8::sub(e[0], e[1]);
    const unsigned a2 = Mod8::add(e[2], e[3]), a3 = Mod8::sub(e[2], e[3]);
    e[0] = Mod8::add(a0, a2);
    e[2] = Mod8::sub(a0, a2);
    e[1] = Mod8::add(a1, a3);
    e[3] = Mod8::sub(a1, a3);
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned o = unsigned(__shfl_xor(int(e[j]), d));
            e[j] = (lane & d) ? Mod8::sub(o, e[j]) : Mod8::add(e[j], o);
        }
}
__global__ void __launch_bounds__(64) k_el8(El8Args a) {
    const El8Job& job = a.job[blockIdx.x];
    const unsigned lane = threadIdx.x;
    const uint32_t ebits = (job.erased[lane >> 3] >> ((lane & 7) * 4)) & 0xFu;  // positions 4 lane .. 4 lane + 3
    unsigned e[4], w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        w[j] = a.walsh[4 * lane + j];
        e[j] = (ebits >> j) & 1u;
    }
    fwht256_mod255(e, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) e[j] = (e[j] * w[j]) % 255u;
    fwht256_mod255(e, lane);
    a.out[size_t(job.slot) * 64 + lane] = e[0] | (e[1] << 8) | (e[2] << 16) | (e[3] << 24);
}
// The error locator of this launch's pattern (k_el8's output, one byte per
// position) at a wave-uniform position, through the scalar cache: from the
// argument block when the host passes it by value, else from the workspace slot
// (an LDS copy put an LDS round trip in front of every scale table read).
LDEV uint32_t el_word(const Ff8DecArgs& a, unsigned i) { return a.el_by_value ? a.el_val[i] : cload(a.el + i); }
// The el bytes of a lane's NR layout-0 positions p0 + r (p0 = w << R: NR
// consecutive positions, wave-uniform), read at the top of the kernel so that
// their latency (kernel-argument or scalar-cache reads) overlaps the piece loads
// instead of sitting in front of the first scale multiply.
// (p0 is a multiple of NR: NR < 4 positions share one word.)
template <int NR>
struct ElRegs {
    static constexpr int kW = NR >= 4 ? NR / 4 : 1;
    uint32_t wd[kW];
    unsigned off;
    LDEV void load(const Ff8DecArgs& a, unsigned p0) {
        off = p0 & 3u;
#pragma unroll
        for (int i = 0; i < kW; ++i) wd[i] = el_word(a, (p0 >> 2) + i);
    }
    LDEV unsigned at(int r) const {
        const unsigned q = off + unsigned(r);
        return (wd[q >> 2] >> ((q & 3u) * 8u)) & 0xFFu;
    }
};

// v[r] *= table(log_of(r)) for the pieces with pred(r): the tables of KB pieces
// are read together, then their multiplies run (one LDS round trip per batch).
template <class TL, class LogFn, class PredFn>
LDEV void scale_batched(typename TL::Reg& v, const LdsTab8<256>& ltab, LogFn log_of, PredFn pred) {
    constexpr int KB = TL::NR < 4 ? TL::NR : 4;
    static_for<0, TL::NR / KB>([&](auto BI) {
        constexpr int r0 = decltype(BI)::value * KB;
        FF8::Tab t[KB];
        asm volatile("" ::: "memory");
        static_for<0, KB>([&](auto I) { t[decltype(I)::value] = ltab.at(int(log_of(r0 + decltype(I)::value))); });
        static_for<0, KB>([&](auto I) {
            constexpr int r = r0 + decltype(I)::value;
            if ((LAMD_ABLATE & 128) == 0 && pred(r)) FF8::mul(v[r], v[r], t[decltype(I)::value]);
        });
    });
}

template <int T, int RB, int NA>
LDEV void ff8_dec(const Ff8DecArgs& a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    using F = FF8;
    using TL = Tile<F, T, RB, 1>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const LdsTab8<256> sk{lds + areas8(NA) * tile_dwords_for(T, RB)};
    const LdsTab8<256> ltab{sk.base + LdsTab8<256>::kDwords};  // by log value
    LdsRing<tile_dwords_for(T, RB), areas8(NA)> ring{lds};
    STAMP(0);
    TabStage8<threads_for(T, RB), 256> sk_stage, log_stage;
    sk_stage.load(a.sktab);
    log_stage.load(a.tabs);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols cl = strip_cols(a.nunits, lane);
    const PieceSpace ps{0, 0, 0};
    const Pyr8Live present{a.present}, needed{a.needed};
    auto pos = [&](int r) { return TL::piece(0, r, w); };
    ElRegs<TL::NR> el;
    el.load(a, pos(0));
    typename TL::Reg v;
    // received pieces: positions [0, R) recovery, [m, m + K) originals
    // (LeopardFF8.cpp:1857-1877); a lost original's position holds its output
    // buffer, so these pointers also serve the stores (kept in SGPRs: a second
    // fetch after the butterflies was a scalar-load round trip in front of them)
    uint64_t pp[TL::NR];
    fetch_ptrs(pp, a, pos);
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) v[r][0] = present(pos(r), 0) ? gload(pp[r], cl) : 0u;
    STAMP(1);
    sk_stage.store(sk);
    log_stage.store(ltab);
    __syncthreads();
    STAMP(2);
    // scale by exp(el) (absent pieces stay zero)
    scale_batched<TL>(v, ltab, [&](int r) { return el.at(r); }, [&](int r) { return present(pos(r), 0); });
    // decoder skew base -1 (LeopardFF8.cpp:1880, 1903), piece space {0, 0, 0}
    const LdsSkew8Fixed<-1> win{{{sk}}};
    // IFFT and FFT without their top layers around swap_top + D_low (see
    // Tile::derivative_swaptop): the same map as IFFT, (I + D), FFT
    if constexpr (pipe8(NA)) {
        TL::template ifft_pl<true>(v, w, lane, ring, ps, win, present);
        STAMP(3);
        TL::derivative_swaptop(v, w, lane, ring.next(), decltype(ring)::kPreBarrier);
        STAMP(4);
        TL::template fft_pl<true>(v, w, lane, ring, ps, win, needed);
    } else {
        TL::template ifft<true>(v, w, lane, lds, ps, win, present);
        STAMP(3);
        TL::derivative_swaptop(v, w, lane, lds, true);
        STAMP(4);
        TL::template fft<true>(v, w, lane, lds, ps, win, needed);
    }
    STAMP(5);
    TL::pin(v);
    // lost original at p = m + i: work[i] = z[p] * exp(-el[p])  (LeopardFF8.cpp:1913-1915)
    auto is_needed = [&](int r) { return needed(pos(r), 0); };
    scale_batched<TL>(v, ltab, [&](int r) { return F::kModulus - el.at(r); }, is_needed);
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r)
        if (is_needed(r)) gstore(pp[r], cl, v[r][0]);
    STAMP(6);
}
template <int T, int RB, int NA>
__global__ void __launch_bounds__(threads_for(T, RB), 4) k_ff8_dec(Ff8DecArgs a) {
    ff8_dec<T, RB, NA>(a);
}
template <int T, int RB>
__global__ void __launch_bounds__(threads_for(T, RB), 4) k_ff8_dec_batch(const Ff8DecArgs* __restrict__ objs) {
    ff8_dec<T, RB, 1>(objs[blockIdx.y]);
}

// Decode when every received piece sits in the low half of the positions (no
// original survives; n = 2m, so recovery [0, R) is the low half and the lost
// originals [m, m + K) the high half).  FFT (I + D) IFFT = F_low (swap_top +
// D_low) I_low (Tile::derivative_swaptop), and F_low, D_low, I_low act inside
// each half.  The high half of I_low(v) is zero, so after swap_top + D_low the
// high half holds exactly the low half of I_low(v): the needed outputs are
//   lost i = F_low,high( I_low,low( received * exp(el) ) )[i] * exp(-el[m + i])
// -- an m-point IFFT on the low positions, an m-point FFT with the skews of the
// high positions (the encoder's transform pair with the halves exchanged, so
// the top layers fuse as in the encoder), no derivative, every wave busy (in k_ff8_dec the waves of the
// empty high half idle through the scale and the low IFFT layers).
// kDense: K = R = m and every recovery piece received (full loss of the
// originals, the benchmark's worst case): all low positions present, all high
// ones needed, so the pyramid predicates compile away.
template <int T, int RB, bool kDense = false>
LDEV void ff8_dec_half(const Ff8DecArgs& a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    using F = FF8;
    using TL = Tile<F, T, RB, 1>;
    constexpr unsigned m = 1u << T;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const LdsTab8<256> sk{lds + tile_dwords_for(T, RB)};
    const LdsTab8<256> ltab{sk.base + LdsTab8<256>::kDwords};  // by log value
    TabStage8<threads_for(T, RB), 256> sk_stage, log_stage;
    sk_stage.load(a.sktab);
    log_stage.load(a.tabs);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols cl = strip_cols(a.nunits, lane);
    const PieceSpace low{0, 0, 0}, high{0, 0, m};
    auto pyr = [](const uint32_t* w) {
        if constexpr (kDense) return AllLive{};
        else return Pyr8Live{w};
    };
    const auto present = pyr(a.present), needed = pyr(a.needed);
    auto lpos = [&](int r) { return TL::piece(0, r, w); };
    auto hpos = [&](int r) { return m + TL::piece(0, r, w); };
    ElRegs<TL::NR> el_lo, el_hi;
    el_lo.load(a, lpos(0));
    el_hi.load(a, hpos(0));
    typename TL::Reg v;
    {
        uint64_t pp[TL::NR];
        fetch_ptrs(pp, a, lpos);
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) v[r][0] = present(lpos(r), 0) ? gload(pp[r], cl) : 0u;
    }
    // output pointers now, behind the piece loads (not after the butterflies)
    uint64_t pp[TL::NR];
    fetch_ptrs(pp, a, hpos);
    sk_stage.store(sk);
    log_stage.store(ltab);
    __syncthreads();
    scale_batched<TL>(v, ltab, [&](int r) { return el_lo.at(r); }, [&](int r) { return present(lpos(r), 0); });
    Skew8Win win{{sk}};
    win.stage(nullptr, -1);  // decoder skew base (LeopardFF8.cpp:1880, 1903)
    // both top layers (single skews m/2 - 1 and m + m/2 - 1) as one butterfly
    // with their sum, the encoder's chunk-0 fused table (Tile::fused_top)
    TL::template ifft<true>(v, w, lane, lds, low, LdsSkew8Fixed<-1>{{{sk}}}, present);
    TL::fused_top(v, FF8::tab_at(a.fused));
    TL::template fft<true>(v, w, lane, lds, high, win, needed);
    TL::pin(v);
    auto is_needed = [&](int r) { return needed(hpos(r), 0); };
    scale_batched<TL>(v, ltab, [&](int r) { return F::kModulus - el_hi.at(r); }, is_needed);
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r)
        if (is_needed(r)) gstore(pp[r], cl, v[r][0]);
}
template <int T, int RB, bool kDense>
__global__ void __launch_bounds__(threads_for(T, RB), 4) k_ff8_dec_half(Ff8DecArgs a) {
    ff8_dec_half<T, RB, kDense>(a);
}
template <int T, int RB, bool kDense>
__global__ void __launch_bounds__(threads_for(T, RB), 4) k_ff8_dec_half_batch(const Ff8DecArgs* __restrict__ objs) {
    ff8_dec_half<T, RB, kDense>(objs[blockIdx.y]);
}

// Partial loss with n = 2m (K <= m, some originals received).  The received
// vector splits by linearity into (x, h): x on the low positions (recovery
// pieces), h on the high ones (surviving originals).  With
//   F (I + D) I = F_low (swap_top + D_low) I_low      (Tile::derivative_swaptop)
// and I_low (x, h) = (I_L x, I_H h), the high half -- where every needed output
// lives -- is
//   F_H( I_L x  ^  N(I_H h) )
// with I_L / I_H / F_H the m-point transforms at the skews of the low / high
// positions and N the m-point neighbour sum of the formal derivative (every
// tile bit; LeopardFF8.cpp:1890-1899 restricted to one half).  Three m-point
// transforms on a 2^T tile instead of two n-point ones on a 2^(T+1) tile
// (k_ff8_dec): every wave busy, a third fewer butterflies.
template <int T, int RB>
LDEV void ff8_dec_split(const Ff8DecArgs& a) {
    if constexpr ((LAMD_ABLATE & 16) != 0) return;
    using F = FF8;
    using TL = Tile<F, T, RB, 1>;
    constexpr unsigned m = 1u << T;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const LdsTab8<256> sk{lds + tile_dwords_for(T, RB)};
    const LdsTab8<256> ltab{sk.base + LdsTab8<256>::kDwords};  // by log value
    TabStage8<threads_for(T, RB), 256> sk_stage, log_stage;
    sk_stage.load(a.sktab);
    log_stage.load(a.tabs);
    const unsigned w = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cols cl = strip_cols(a.nunits, lane);
    const PieceSpace low{0, 0, 0}, high{0, 0, m};
    const Pyr8Live present{a.present}, needed{a.needed};
    auto lpos = [&](int r) { return TL::piece(0, r, w); };
    auto hpos = [&](int r) { return m + TL::piece(0, r, w); };
    ElRegs<TL::NR> el_lo, el_hi;
    el_lo.load(a, lpos(0));
    el_hi.load(a, hpos(0));
    typename TL::Reg x, h;
    // high positions: surviving originals in, lost originals out (kept for the stores)
    uint64_t ph[TL::NR];
    fetch_ptrs(ph, a, hpos);
#pragma unroll
    for (int r = 0; r < TL::NR; ++r) h[r][0] = present(hpos(r), 0) ? gload(ph[r], cl) : 0u;
    {
        uint64_t pp[TL::NR];
        fetch_ptrs(pp, a, lpos);
#pragma unroll
        for (int r = 0; r < TL::NR; ++r) x[r][0] = present(lpos(r), 0) ? gload(pp[r], cl) : 0u;
    }
    sk_stage.store(sk);
    log_stage.store(ltab);
    __syncthreads();
    Skew8Win win{{sk}};
    win.stage(nullptr, -1);  // decoder skew base (LeopardFF8.cpp:1880, 1903)
    // y = N(I_H(h * exp(el)))
    scale_batched<TL>(h, ltab, [&](int r) { return el_hi.at(r); }, [&](int r) { return present(hpos(r), 0); });
    TL::template ifft<false>(h, w, lane, lds, high, win, present);
    typename TL::Reg y;
    TL::zero(y);
    TL::derivative_add(y, [&](int r, uint32_t* out) { out[0] = h[r][0]; }, w, lane, lds);
    // x <- I_L(x * exp(el)) ^ y, then F_H
    scale_batched<TL>(x, ltab, [&](int r) { return el_lo.at(r); }, [&](int r) { return present(lpos(r), 0); });
    TL::template ifft<false>(x, w, lane, lds, low, LdsSkew8Fixed<-1>{{{sk}}}, present);
    TL::xor_into(x, y);
    TL::template fft<false>(x, w, lane, lds, high, win, needed);
    TL::pin(x);
    auto is_needed = [&](int r) { return needed(hpos(r), 0); };
    scale_batched<TL>(x, ltab, [&](int r) { return F::kModulus - el_hi.at(r); }, is_needed);
    if (!cl.live) return;
#pragma unroll
    for (int r = 0; r < TL::NR; ++r)
        if (is_needed(r)) gstore(ph[r], cl, x[r][0]);
}
template <int T, int RB>
__global__ void __launch_bounds__(threads_for(T, RB), 4) k_ff8_dec_split(Ff8DecArgs a) {
    ff8_dec_split<T, RB>(a);
}
template <int T, int RB>
__global__ void __launch_bounds__(threads_for(T, RB), 4) k_ff8_dec_split_batch(const Ff8DecArgs* __restrict__ objs) {
    ff8_dec_split<T, RB>(objs[blockIdx.y]);
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
hipError_t launch8(KernelFn* fn, unsigned threads, const Args& a, size_t lds_dwords, hipStream_t s, unsigned lw = 64) {
    const size_t lds = lds_dwords * 4;
    if (lds > 65536) {
        const hipError_t e = Once<Tag>::set_lds(reinterpret_cast<const void*>(fn), lds);
        if (e != hipSuccess) return e;
    }
    void* params[] = {const_cast<Args*>(&a)};
    const dim3 grid((a.nunits + lw - 1) / lw);
    return hipLaunchKernel(reinterpret_cast<const void*>(fn), grid, dim3(threads), params, lds, s);
}
// Batched form: argument blocks in device memory, grid (strips, objects).
template <class Tag, class KernelFn, class Args>
hipError_t launch8_batch(KernelFn* fn, unsigned threads, const Args* objs, unsigned count, uint32_t nunits,
                         size_t lds_dwords, hipStream_t s) {
    const size_t lds = lds_dwords * 4;
    if (lds > 65536) {
        const hipError_t e = Once<Tag>::set_lds(reinterpret_cast<const void*>(fn), lds);
        if (e != hipSuccess) return e;
    }
    const Args* arg = objs;
    void* params[] = {&arg};
    return hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3((nunits + 63) / 64, count), dim3(threads), params,
                           lds, s);
}
template <int T, bool M>
struct EncBatchTag {};
template <int T>
struct DecBatchTag {};
template <int T>
struct DecHalfBatchTag {};
template <int T>
struct DecSplitBatchTag {};

template <int T, int RB, bool M, int NA, int G>
struct EncTag {};
template <int T, int RB, int NA>
struct DecTag {};
template <int T, int RB>
struct DecHalfTag {};
template <int T, int RB>
struct DecSplitTag {};

// Launch shape overrides for experiments (LEO_AMD_FF8_WIDE=1: the wide
// register forms at every size); read once.
bool force_wide() {
#if LAMD_EXPERIMENT_ENV
    static const bool v = [] {
        const char* e = std::getenv("LEO_AMD_FF8_WIDE");
        return e && e[0] == '1';
    }();
    return v;
#else
    return false;  // experiment builds only (LAMD_EXPERIMENT_ENV=1)
#endif
}

// The bit-sliced dense tile (rs_ff8_bs.hip) for K = R = 128 slab batches; the
// byte-layout tile stays selectable for A/B in experiment builds
// (LEO_AMD_FF8_BS=0).
#ifndef LAMD_FF8_BS
#define LAMD_FF8_BS 1
#endif
bool bs_tile_enabled() {
#if LAMD_EXPERIMENT_ENV
    static const bool v = [] {
        const char* e = std::getenv("LEO_AMD_FF8_BS");
        return e ? e[0] == '1' : LAMD_FF8_BS != 0;
    }();
    return v;
#else
    return LAMD_FF8_BS != 0;
#endif
}

// Lane-group bits of the encoder launch (LEO_AMD_FF8_G overrides in experiment
// builds, LAMD_EXPERIMENT_ENV=1: lib/exp/libleopard_amd.so; read once):
// pieces of at most 64 KiB run 64-byte strips (G = 2: four workgroups per CU
// in a 64 KiB call), larger pieces the full-wave strips.
int enc_lane_groups(uint32_t nunits) {
#if LAMD_EXPERIMENT_ENV
    static const int v = [] {
        const char* e = std::getenv("LEO_AMD_FF8_G");
        return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : -1;
    }();
    if (v >= 0) return v;
#endif
    return nunits <= 16384u ? kDefaultEncG : 0;
}

// One chunk with K = R = m: the dense encoder (no pruning predicates).
inline bool enc_dense(unsigned T, const Ff8EncArgs& a) {
    return a.nchunks == 1 && a.K == (1u << T) && a.R == (1u << T);
}

template <int T, int RB, int NA, int G>
hipError_t enc_RBG(const Ff8EncArgs& a, hipStream_t s) {
    constexpr size_t lds = areas8(NA) * (tile_dwords_for(T, RB) >> G) + LdsTab8<256>::kDwords;
    constexpr unsigned threads = threads_for(T, RB) >> G;
    if constexpr (G == 0)
        if (enc_dense(T, a))
            return launch8<EncTag<T, RB, false, NA, 4>>(&k_ff8_enc<T, RB, false, NA, 0, kFormDenseEnc>, threads, a, lds,
                                                         s);
    if (a.nchunks > 1)
        return launch8<EncTag<T, RB, true, NA, G>>(&k_ff8_enc<T, RB, true, NA, G>, threads, a, lds, s, 64u >> G);
    return launch8<EncTag<T, RB, false, NA, G>>(&k_ff8_enc<T, RB, false, NA, G>, threads, a, lds, s, 64u >> G);
}
template <int T, int RB, int NA>
hipError_t enc_RB(const Ff8EncArgs& a, hipStream_t s) {
    if constexpr (NA == 1 && T - RB >= 2 && T > RB) {
        const int g = enc_lane_groups(a.nunits);
        if (g == 2) return enc_RBG<T, RB, NA, 2>(a, s);
        if (g == 1) return enc_RBG<T, RB, NA, 1>(a, s);
    }
    return enc_RBG<T, RB, NA, 0>(a, s);
}
template <int T>
hipError_t enc_T(const Ff8EncArgs& a, hipStream_t s) {
    // wide form once every CU gets >= 4 strips (256 CUs x 4 x 256 B: 256 KiB pieces)
    if constexpr (wide_bits8(T) != reg_bits8(T))
        if (a.nunits >= 65536 || force_wide()) return enc_RB<T, wide_bits8(T), 1>(a, s);
    if constexpr (kPipe8)
        if (a.nunits <= kOneWgPerCuUnits) return enc_RB<T, reg_bits8(T), 2>(a, s);
    return enc_RB<T, reg_bits8(T), 1>(a, s);
}
template <int T, int RB, int NA>
hipError_t dec_RB(const Ff8DecArgs& a, hipStream_t s) {
    constexpr size_t lds = areas8(NA) * tile_dwords_for(T, RB) + 2 * LdsTab8<256>::kDwords + kEl8Dwords;
    return launch8<DecTag<T, RB, NA>>(&k_ff8_dec<T, RB, NA>, threads_for(T, RB), a, lds, s);
}
template <int T>
hipError_t dec_T(const Ff8DecArgs& a, hipStream_t s) {
    if constexpr (wide_dec_bits8(T) != reg_bits8(T))
        if (force_wide()) return dec_RB<T, wide_dec_bits8(T), 1>(a, s);
    if constexpr (kPipe8)
        if (a.nunits <= kOneWgPerCuUnits) return dec_RB<T, reg_bits8(T), 2>(a, s);
    return dec_RB<T, reg_bits8(T), 1>(a, s);
}

template <int T>
hipError_t dec_half_T(const Ff8DecArgs& a, hipStream_t s) {
    constexpr int RB = reg_bits8(T);
    constexpr size_t lds = tile_dwords_for(T, RB) + 2 * LdsTab8<256>::kDwords + kEl8Dwords;
    if (a.dense)
        return launch8<DecHalfTag<T, RB + 16>>(&k_ff8_dec_half<T, RB, true>, threads_for(T, RB), a, lds, s);
    return launch8<DecHalfTag<T, RB>>(&k_ff8_dec_half<T, RB, false>, threads_for(T, RB), a, lds, s);
}
template <int T>
hipError_t dec_split_T(const Ff8DecArgs& a, hipStream_t s) {
    constexpr int RB = reg_bits8(T);
    constexpr size_t lds = tile_dwords_for(T, RB) + 2 * LdsTab8<256>::kDwords + kEl8Dwords;
    return launch8<DecSplitTag<T, RB>>(&k_ff8_dec_split<T, RB>, threads_for(T, RB), a, lds, s);
}

}  // namespace

#ifdef LAMD_CLOCK
extern "C" __attribute__((visibility("default"))) int leo_amd_debug_clock(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_clock), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef LAMD_STAMPS
extern "C" __attribute__((visibility("default"))) int leo_amd_debug_stamps(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_error_locator8(const El8Args& a, unsigned count, hipStream_t s) {
    if (count == 0 || count > kEl8Jobs) return hipErrorInvalidValue;
    void* params[] = {const_cast<El8Args*>(&a)};
    return hipLaunchKernel(reinterpret_cast<const void*>(&k_el8), dim3(count), dim3(64), params, 0, s);
}

hipError_t launch_ff8_encode(unsigned T, const Ff8EncArgs& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 8>([&](auto I) {
        if (T == unsigned(decltype(I)::value)) e = enc_T<decltype(I)::value>(a, s);
    });
    return e;
}

// Full-loss decode of a K = R = m code: with every original lost and every
// recovery piece received, the decoder's map is the inverse of the encoder's
// rec = FFT_{-1}(IFFT_{m-1}(data)) -- a bijection of m pieces, so the
// reference decoder (which returns the unique originals) computes exactly
//   data = FFT_{m-1}(IFFT_{-1}(rec))
// (an IFFT inverts the FFT of the same skew base and vice versa).  That is the
// encoder's tile with the two skew bases exchanged: no error locator, no
// scale / reveal multiplies.  `a` is an encoder block: ptr[0, m) the recovery
// pieces, ptr[m, 2m) the outputs, fused = the encoder's chunk-0 table (the
// fused top layer adds the same two single skews).
hipError_t launch_ff8_decode_full(unsigned Tm, const Ff8EncArgs& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 8>([&](auto I) {
        constexpr int TT = decltype(I)::value;
        if (Tm != unsigned(TT)) return;
        constexpr int RB = wide_bits8(TT);
        const bool wide = RB != reg_bits8(TT) && (a.nunits >= 65536 || force_wide());
        if (wide) {
            constexpr size_t lds = tile_dwords_for(TT, RB) + LdsTab8<256>::kDwords;
            e = launch8<EncTag<TT, RB, false, 1, 5>>(&k_ff8_enc<TT, RB, false, 1, 0, kFormDenseDec>,
                                                     threads_for(TT, RB), a, lds, s);
        } else {
            constexpr int RN = reg_bits8(TT);
            constexpr size_t lds = tile_dwords_for(TT, RN) + LdsTab8<256>::kDwords;
            e = launch8<EncTag<TT, RN, false, 1, 5>>(&k_ff8_enc<TT, RN, false, 1, 0, kFormDenseDec>,
                                                     threads_for(TT, RN), a, lds, s);
        }
    });
    return e;
}

hipError_t launch_ff8_decode_half(unsigned Tm, const Ff8DecArgs& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 8>([&](auto I) {
        if (Tm == unsigned(decltype(I)::value)) e = dec_half_T<decltype(I)::value>(a, s);
    });
    return e;
}

hipError_t launch_ff8_decode_split(unsigned Tm, const Ff8DecArgs& a, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 8>([&](auto I) {
        if (Tm == unsigned(decltype(I)::value)) e = dec_split_T<decltype(I)::value>(a, s);
    });
    return e;
}

hipError_t launch_ff8_encode_batch(unsigned T, const Ff8EncArgs* objs, unsigned count, uint32_t nunits, bool multi,
                                   int form, hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 8>([&](auto I) {
        constexpr int TT = decltype(I)::value, RB = batch_bits8(TT);
        constexpr size_t lds = tile_dwords_for(TT, RB) + LdsTab8<256>::kDwords;
        if (T != unsigned(TT)) return;
        if (form == kFormDenseEnc)
            e = launch8_batch<EncBatchTag<TT + 16, false>>(&k_ff8_enc_batch<TT, RB, false, kFormDenseEnc>,
                                                           threads_for(TT, RB), objs, count, nunits, lds, s);
        else if (form == kFormDenseDec)
            e = launch8_batch<EncBatchTag<TT + 32, false>>(&k_ff8_enc_batch<TT, RB, false, kFormDenseDec>,
                                                           threads_for(TT, RB), objs, count, nunits, lds, s);
        else if (multi)
            e = launch8_batch<EncBatchTag<TT, true>>(&k_ff8_enc_batch<TT, RB, true>, threads_for(TT, RB), objs, count,
                                                     nunits, lds, s);
        else
            e = launch8_batch<EncBatchTag<TT, false>>(&k_ff8_enc_batch<TT, RB, false>, threads_for(TT, RB), objs,
                                                      count, nunits, lds, s);
    });
    return e;
}

hipError_t launch_ff8_encode_slab(unsigned T, const Ff8SlabBatch& b, unsigned count, bool multi, int form,
                                  hipStream_t s, unsigned cus, uint32_t* q, uint32_t* qclear) {
    // dense 128 + 128 forms: the bit-sliced tile (rs_ff8_bs.hip)
    if (form != kFormGeneral && !multi && bs_tile_enabled() && ff8_bs_supported(T, b.K, b.R, b.nchunks))
        return launch_ff8_bs_slab(b, count, form, s, cus, q, qclear);
    hipError_t e = hipErrorInvalidValue;
    static_for<1, 8>([&](auto I) {
        constexpr int TT = decltype(I)::value, RB = batch_bits8(TT);
        constexpr size_t lds = (tile_dwords_for(TT, RB) + LdsTab8<256>::kDwords) * 4;
        if (T != unsigned(TT)) return;
        const void* fn = form == kFormDenseEnc   ? reinterpret_cast<const void*>(&k_ff8_enc_slab<TT, RB, false, kFormDenseEnc>)
                         : form == kFormDenseDec ? reinterpret_cast<const void*>(&k_ff8_enc_slab<TT, RB, false, kFormDenseDec>)
                         : multi                 ? reinterpret_cast<const void*>(&k_ff8_enc_slab<TT, RB, true>)
                                                 : reinterpret_cast<const void*>(&k_ff8_enc_slab<TT, RB, false>);
        static_assert(lds <= 65536, "slab batch tiles fit the default LDS limit");
        void* params[] = {const_cast<Ff8SlabBatch*>(&b)};
        e = hipLaunchKernel(fn, dim3((b.nunits + 63) / 64, count), dim3(threads_for(TT, RB)), params, lds, s);
    });
    return e;
}

hipError_t launch_ff8_decode_batch(unsigned T, const Ff8DecArgs* objs, unsigned count, uint32_t nunits, int mode,
                                   hipStream_t s) {
    hipError_t e = hipErrorInvalidValue;
    if (mode != kDec8General) {
        static_for<1, 8>([&](auto I) {
            constexpr int TT = decltype(I)::value, RB = batch_bits8(TT);
            constexpr size_t lds = tile_dwords_for(TT, RB) + 2 * LdsTab8<256>::kDwords + kEl8Dwords;
            if (T != unsigned(TT)) return;
            if (mode == kDec8Split)
                e = launch8_batch<DecSplitBatchTag<TT>>(&k_ff8_dec_split_batch<TT, RB>, threads_for(TT, RB), objs,
                                                        count, nunits, lds, s);
            else if (mode == kDec8HalfDense)
                e = launch8_batch<DecHalfBatchTag<TT + 16>>(&k_ff8_dec_half_batch<TT, RB, true>, threads_for(TT, RB),
                                                            objs, count, nunits, lds, s);
            else
                e = launch8_batch<DecHalfBatchTag<TT>>(&k_ff8_dec_half_batch<TT, RB, false>, threads_for(TT, RB), objs,
                                                       count, nunits, lds, s);
        });
        return e;
    }
    static_for<1, 9>([&](auto I) {
        constexpr int TT = decltype(I)::value, RB = batch_bits8(TT);
        constexpr size_t lds = tile_dwords_for(TT, RB) + 2 * LdsTab8<256>::kDwords + kEl8Dwords;
        if (T == unsigned(TT))
            e = launch8_batch<DecBatchTag<TT>>(&k_ff8_dec_batch<TT, RB>, threads_for(TT, RB), objs, count, nunits, lds,
                                               s);
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
