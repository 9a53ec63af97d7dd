// rs_ff8_mat.hip -- GF(2^8) codes applied as their coefficient matrix: the
// matrix path for small codes and few losses (single leo_encode / leo_decode
// calls with n <= 256).
//
// Every GF(2^8) encode (LeopardFF8.cpp:1602-1672) and every decode of one
// erasure pattern (LeopardFF8.cpp:1809-1916) is a GF(2^8)-linear map of the
// pieces it reads, the same for every byte column:
//   out_i[c] = XOR_j  M[i][j] * in_j[c]      (i < L outputs, j < N inputs).
// For a decode, the inputs are ALL received pieces (recovery and originals,
// every one the reference's decoder scales and transforms), so the map is the
// reference decoder's own, also on inputs that are not codewords.  The host
// obtains M once per (K, R, erasure pattern) by running the transform kernels
// on unit pieces (piece j = the byte 1 at column j, rs_ff8.hip), and
// k_ff8_mat_tabs turns the L x N products into byte-permute multiply tables.
// The transforms cost ~ n log2 n butterflies in 2 log2 n dependent layers with
// LDS transposes and barriers between them; the matrix costs L x N independent
// multiply-adds per column -- fewer instructions on the critical path of a
// small call, no layers, no exchanges.
//
// k_ff8_mat: a workgroup of W waves (kMatWaves; N <= 16 W) owns a
// 256-byte column strip (a dword per lane) and a group of LB outputs (grid.y =
// output groups, so a call with few column strips still spreads over the
// GPU); wave w multiplies the inputs j = w, w + W, ... into LB per-lane
// accumulators, with the group's tables staged in LDS (broadcast reads; rows
// past L are zero tables, so the inner loop has no branch); then the waves'
// partial sums are XORed through LDS and each output is stored once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "rs_args.h"

namespace lamd {

namespace {

constexpr int kMatWaves = 16;  // most waves per workgroup (inputs split across them)
constexpr int kMatInMax = 16;  // most inputs per wave (KI = 1, 2, 4, 8 or 16)

// C dwords of a piece from byte offset `off`, through a buffer resource of
// `nbytes` bytes: a slot with no piece passes 0 and reads zeros without a
// memory access (no branch).  Cached loads: the workgroups of the other output
// groups of this strip read the same bytes, from the same XCD's L2 (workgroup
// ids y * strips + x, strips a multiple of 8 or close: the groups of strip x
// land on one XCD).
template <int C>
LDEV void mat_load(uint32_t* v, uint64_t base, uint32_t off, uint32_t nbytes) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), short(0), int(nbytes), 0x00020000);
    if constexpr (C == 1) {
        v[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    } else if constexpr (C == 2) {
        const v2u x = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        v[0] = x.x, v[1] = x.y;
    } else {
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
        v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w;
    }
}
template <int C>
LDEV void mat_store(uint64_t base, uint32_t off, const uint32_t* v) {
    using V = typename VecT<C>::type;
    V x;
    if constexpr (C == 1) x = v[0];
    else if constexpr (C == 2) x = V{v[0], v[1]};
    else x = V{v[0], v[1], v[2], v[3]};
    __builtin_nontemporal_store(x, gptr<V>(reinterpret_cast<uint8_t*>(base) + off));
}

// LB outputs per workgroup, C dwords (4 C columns) per lane: one table read
// serves C multiply-adds (the LDS return path, ~1 KiB a wave for a broadcast
// 16-byte read, is what C = 1 runs into on large calls).  KI inputs per wave
// (16 KI >= N): wave w multiplies inputs j = w + 16 k, k < KI; slots j >= N
// hold zero tables and load zeros through an empty buffer range, so the loads
// do not branch (branches there made the compiler wait for every load before
// the first multiply).
template <int LB, int C, int KI>
__global__ void __launch_bounds__(64 * kMatWaves) k_ff8_mat(Ff8MatArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr unsigned W = kMatWaves;  // the launch always runs kMatWaves waves
    constexpr unsigned NP = W * KI;    // table slots per output row
    const unsigned wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const unsigned N = a.N, L = a.L, i0 = blockIdx.y * LB;
    // Memory first, every request before the first wait: the group's tables
    // (slot (i, j) at dwords 8 (i NP + j) .. + 4: an aligned ds_read_b128 and a
    // ds_read_b32; rows i0 + i >= L and slots j >= N are zero tables), then
    // this wave's inputs.
    constexpr unsigned kChunks = LB * NP * 2;  // 16-byte chunks of the staged tables
    constexpr unsigned kTabPer = (kChunks + 64 * W - 1) / (64 * W);
    const unsigned rows = min(L - i0, unsigned(LB));
    const v4u* tsrc = reinterpret_cast<const v4u*>(a.tabs) + size_t(i0) * N * 2;
    const v4u* tzero = reinterpret_cast<const v4u*>(a.tabs) + size_t(L) * N * 2;
    v4u tv[kTabPer];
#pragma unroll
    for (unsigned u = 0; u < kTabPer; ++u) {
        const unsigned e = threadIdx.x + u * 64u * W;
        const unsigned i = e / (NP * 2), j = (e / 2) % NP, h = e & 1u;
        const bool real = e < kChunks && i < rows && j < N;
        // empty slots read the zero entry after the L x N (no branch, no select
        // that would wait for the load)
        tv[u] = real ? tsrc[(i * N + j) * 2 + h] : tzero[h];
    }
    const uint32_t q0 = (blockIdx.x * 64u + lane) * C;  // first dword column of the lane
    const bool live = q0 < a.nunits;                  // nunits is a multiple of 16 (64-byte pieces)
    const uint32_t off = (live ? q0 : a.nunits - C) * 4u;  // dead lanes re-read valid columns, never store
    uint32_t v[KI][C];
    const uint32_t nbytes = a.nunits * 4u;
    uint64_t p[KI];  // piece pointers: one batch of scalar loads, then the piece loads in order
#pragma unroll
    for (int k = 0; k < KI; ++k) p[k] = a.ptr[min(wave + W * k, N - 1)];
#pragma unroll
    for (int k = 0; k < KI; ++k) asm volatile("" : "+s"(p[k]));
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        mat_load<C>(v[k], p[k], off, wave + W * k < N ? nbytes : 0u);
        __builtin_amdgcn_sched_barrier(0);  // issued in k order: the multiplies wait for them in k order
    }
#pragma unroll
    for (unsigned u = 0; u < kTabPer; ++u) {
        const unsigned e = threadIdx.x + u * 64u * W;
        if (e < kChunks) reinterpret_cast<v4u*>(lds)[e] = tv[u];
    }
    // the tables are in LDS; the input loads stay in flight (a __syncthreads
    // would wait for every one of them: its fence covers global memory too)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    uint32_t acc[LB][C];
#pragma unroll
    for (int i = 0; i < LB; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[i][c] = 0;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
        const unsigned j = wave + W * k;
        if (j >= N) break;  // wave-uniform: the rest are empty slots
        uint32_t s0[C], s1[C], s2[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            s0[c] = v[k][c] & 0x07070707u;
            s1[c] = (v[k][c] >> 3) & 0x07070707u;
            s2[c] = (v[k][c] >> 6) & 0x03030303u;
        }
#pragma unroll
        for (int i = 0; i < LB; ++i) {
            const FF8::Tab t = FF8::tab_lds(lds + 8u * (unsigned(i) * NP + j));
#pragma unroll
            for (int c = 0; c < C; ++c)
                acc[i][c] = xor3(acc[i][c], perm(t.a1, t.a0, s0[c]), perm(t.b1, t.b0, s1[c])) ^ perm(t.c0, t.c0, s2[c]);
        }
    }
    // partial sums of the waves -> outputs
    __syncthreads();  // every wave is done with the tables
#pragma unroll
    for (int i = 0; i < LB; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) lds[((wave * LB + i) * C + c) * 64u + lane] = acc[i][c];
    __syncthreads();
    for (unsigned i = wave; i < LB && i0 + i < L; i += W) {
        uint32_t r[C];
#pragma unroll
        for (int c = 0; c < C; ++c) r[c] = 0;
        for (unsigned w = 0; w < W; ++w)
#pragma unroll
            for (int c = 0; c < C; ++c) r[c] ^= lds[((w * LB + i) * C + c) * 64u + lane];
        if (live) mat_store<C>(a.ptr[N + i0 + i], off, r);
    }
}

// unit pieces: piece j (of `pitch` bytes) is the byte 1 at column j
__global__ void k_ff8_unit(uint32_t* out, unsigned n, unsigned pitch) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;  // dword index
    const unsigned dw = pitch / 4;
    if (i >= n * dw) return;
    const unsigned j = i / dw, c = (i % dw) * 4;
    out[i] = (j >= c && j < c + 4) ? (1u << (8 * (j - c))) : 0u;
}

// tables of M[i][j] = byte j of row i: value-indexed multiply tables (vtab, 8
// dwords per element value, entry 0 all zero) copied into entry (i, j)
__global__ void k_ff8_mat_tabs(const uint8_t* rows, unsigned pitch, unsigned L, unsigned N, const uint32_t* vtab,
                               uint32_t* tabs) {
    const unsigned e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e == L * N) {  // the zero entry after the L x N
        v4u* d = reinterpret_cast<v4u*>(tabs + 8u * e);
        d[0] = d[1] = v4u{0u, 0u, 0u, 0u};
    }
    if (e >= L * N) return;
    const unsigned i = e / N, j = e % N;
    const unsigned v = rows[size_t(i) * pitch + j];
    const v4u* s = reinterpret_cast<const v4u*>(vtab + 8u * v);
    v4u* d = reinterpret_cast<v4u*>(tabs + 8u * e);
    d[0] = s[0];
    d[1] = s[1];
}

constexpr size_t ff8_mat_lds_bytes(unsigned lb, unsigned c, unsigned ki, unsigned waves) {
    return std::max<size_t>(size_t(lb) * waves * ki * 32, size_t(waves) * lb * c * 64 * 4);
}

template <int C, int KI>
const void* mat_kernel(unsigned lb) {
    if constexpr (C == 4) {  // LB 8 at 4 dwords a lane is never chosen (register budget)
        return lb == 4 ? reinterpret_cast<const void*>(&k_ff8_mat<4, C, KI>)
             : lb == 2 ? reinterpret_cast<const void*>(&k_ff8_mat<2, C, KI>)
                       : reinterpret_cast<const void*>(&k_ff8_mat<1, C, KI>);
    } else {
        return lb == 8   ? reinterpret_cast<const void*>(&k_ff8_mat<8, C, KI>)
             : lb == 4 ? reinterpret_cast<const void*>(&k_ff8_mat<4, C, KI>)
             : lb == 2 ? reinterpret_cast<const void*>(&k_ff8_mat<2, C, KI>)
                       : reinterpret_cast<const void*>(&k_ff8_mat<1, C, KI>);
    }
}
template <int C>
const void* mat_kernel(unsigned lb, unsigned ki) {
    return ki == 1   ? mat_kernel<C, 1>(lb)
         : ki == 2 ? mat_kernel<C, 2>(lb)
         : ki == 4 ? mat_kernel<C, 4>(lb)
         : ki == 8 ? mat_kernel<C, 8>(lb)
                   : mat_kernel<C, 16>(lb);
}

}  // namespace

bool ff8_mat_supported(unsigned L, unsigned N) {
    return L >= 1 && L <= kFf8MatMaxOut && N >= 1 && N + L <= kFf8Ptrs;
}

// Grid: column strips of 64 C dwords x output groups of LB (below);
// kMatWaves waves with at most kMatInMax inputs each.
hipError_t launch_ff8_mat(const Ff8MatArgs& a, unsigned cus, hipStream_t s) {
    if (!ff8_mat_supported(a.L, a.N) || a.nunits == 0 || a.nunits > (1u << 29)) return hipErrorInvalidValue;
    auto groups = [&](unsigned lb) { return (a.L + lb - 1) / lb; };
    auto strips_of = [&](unsigned c) { return (a.nunits + 64 * c - 1) / (64 * c); };
    // Output groups as wide as L allows, up to 8 (each input load and its
    // selectors serve LB outputs), then the widest lanes that still give every
    // CU a workgroup; a call too small for that at a dword a lane narrows its
    // groups instead (measured, DESIGN.md 7.6: 128+128 x 64 KiB with 16 lost
    // 11.5 us at LB 4 x 4 dwords, 10.8 at 8 x 2; with 8 lost 8.3 at 2 x 4, 7.4
    // at 8 x 1).  LB 8 runs at most 2 dwords a lane (register budget).
    unsigned lb = 8;
    while (lb > 1 && lb / 2 >= a.L) lb /= 2;
    unsigned c = 1;
    if (lb <= 4 && strips_of(4) * groups(lb) >= cus) c = 4;
    else if (strips_of(2) * groups(lb) >= cus) c = 2;
    else
        while (lb > 1 && strips_of(1) * groups(lb) < cus) lb /= 2;
#if LAMD_EXPERIMENT_ENV
    static const int force_c = [] { const char* e = std::getenv("LEO_AMD_MAT_C"); return e ? std::atoi(e) : 0; }();
    if (force_c == 1 || force_c == 2 || force_c == 4) c = unsigned(force_c);
    static const int force_lb = [] { const char* e = std::getenv("LEO_AMD_MAT_LB"); return e ? std::atoi(e) : 0; }();
    if (force_lb == 1 || force_lb == 2 || force_lb == 4 || force_lb == 8) lb = unsigned(force_lb);
    if (c == 4 && lb == 8) lb = 4;
#endif
    const unsigned strips = strips_of(c);
    // every wave of the workgroup in use even for few inputs: a small call is
    // bound by the chain through one wave (measured: 16 waves of 1-2 inputs beat
    // 2 waves of 12), a large one by the total instructions, which W barely changes
    const unsigned waves = kMatWaves;
    static_assert(kMatWaves * kMatInMax >= kFf8Ptrs, "every input has a wave");
    const dim3 grid(strips, groups(lb));
    void* params[] = {const_cast<Ff8MatArgs*>(&a)};
    // inputs per wave: the fewest of 1, 2, 4, 8, 16 that cover N
    unsigned ki = 1;
    while (kMatWaves * ki < a.N) ki *= 2;
    const void* fn = c == 4 ? mat_kernel<4>(lb, ki) : c == 2 ? mat_kernel<2>(lb, ki) : mat_kernel<1>(lb, ki);
    return hipLaunchKernel(fn, grid, dim3(64 * waves), params, ff8_mat_lds_bytes(lb, c, ki, waves), s);
}

hipError_t launch_ff8_unit(uint8_t* out, unsigned n, unsigned pitch, hipStream_t s) {
    if (pitch % 4 != 0 || n > pitch) return hipErrorInvalidValue;
    const unsigned total = n * (pitch / 4);
    hipLaunchKernelGGL(k_ff8_unit, dim3((total + 255) / 256), dim3(256), 0, s, reinterpret_cast<uint32_t*>(out), n,
                       pitch);
    return hipGetLastError();
}

hipError_t launch_ff8_mat_tabs(const uint8_t* rows, unsigned pitch, unsigned L, unsigned N, const uint32_t* vtab,
                               uint32_t* tabs, hipStream_t s) {
    const unsigned total = L * N + 1;
    hipLaunchKernelGGL(k_ff8_mat_tabs, dim3((total + 255) / 256), dim3(256), 0, s, rows, pitch, L, N, vtab, tabs);
    return hipGetLastError();
}

}  // namespace lamd
