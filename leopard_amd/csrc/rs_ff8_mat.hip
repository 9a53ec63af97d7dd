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
constexpr int kMatInMax = 16;  // most inputs per wave (the launch sizes the workgroup for it)

// C dwords of a piece from byte offset `off`: plain (cached) loads -- the
// workgroups of the other output groups of this strip read the same bytes,
// from the same XCD's L2 (workgroup ids y * strips + x, strips a multiple of 8
// or close: the groups of strip x land on one XCD)
template <int C>
LDEV void mat_load(uint32_t* v, uint64_t base, uint32_t off) {
    using V = typename VecT<C>::type;
    const V x = *gptr<const V>(reinterpret_cast<const uint8_t*>(base) + off);
    if constexpr (C == 1) v[0] = x;
    else if constexpr (C == 2) { v[0] = x.x; v[1] = x.y; }
    else { v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; }
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
// 16-byte read, is what C = 1 runs into on large calls).
template <int LB, int C>
__global__ void __launch_bounds__(64 * kMatWaves) k_ff8_mat(Ff8MatArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const unsigned wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63u, W = blockDim.x >> 6;
    const unsigned N = a.N, L = a.L, i0 = blockIdx.y * LB;
    // the group's tables: entry (i, j) at dwords 8 (i N + j) .. + 4 (an aligned
    // ds_read_b128 and a ds_read_b32); rows i0 + i >= L read as zero tables
    {
        const unsigned n4 = LB * N * 2;  // 16-byte chunks
        const v4u* src = reinterpret_cast<const v4u*>(a.tabs) + size_t(i0) * N * 2;
        const unsigned have = (min(L - i0, unsigned(LB))) * N * 2;
        v4u* dst = reinterpret_cast<v4u*>(lds);
        for (unsigned i = threadIdx.x; i < n4; i += blockDim.x) dst[i] = i < have ? src[i] : v4u{0u, 0u, 0u, 0u};
    }
    const uint32_t q0 = (blockIdx.x * 64u + lane) * C;  // first dword column of the lane
    const bool live = q0 < a.nunits;                  // nunits is a multiple of 16 (64-byte pieces)
    const uint32_t off = (live ? q0 : a.nunits - C) * 4u;  // dead lanes re-read valid columns, never store
    // this wave's inputs, every load issued before the first multiply
    uint32_t v[kMatInMax][C];
#pragma unroll
    for (int k = 0; k < kMatInMax; ++k) {
        const unsigned j = wave + W * k;
        if (j < N) mat_load<C>(v[k], a.ptr[j], off);
        else
#pragma unroll
            for (int c = 0; c < C; ++c) v[k][c] = 0;
    }
    __syncthreads();
    uint32_t acc[LB][C];
#pragma unroll
    for (int i = 0; i < LB; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[i][c] = 0;
#pragma unroll
    for (int k = 0; k < kMatInMax; ++k) {
        const unsigned j = wave + W * k;
        if (j >= N) break;  // wave-uniform
        uint32_t s0[C], s1[C], s2[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            s0[c] = v[k][c] & 0x07070707u;
            s1[c] = (v[k][c] >> 3) & 0x07070707u;
            s2[c] = (v[k][c] >> 6) & 0x03030303u;
        }
        FF8::Tab t[LB];
#pragma unroll
        for (int i = 0; i < LB; ++i) t[i] = FF8::tab_lds(lds + 8u * (unsigned(i) * N + j));
#pragma unroll
        for (int i = 0; i < LB; ++i)
#pragma unroll
            for (int c = 0; c < C; ++c)
                acc[i][c] = xor3(acc[i][c], perm(t[i].a1, t[i].a0, s0[c]), perm(t[i].b1, t[i].b0, s1[c])) ^
                            perm(t[i].c0, t[i].c0, s2[c]);
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
    if (e >= L * N) return;
    const unsigned i = e / N, j = e % N;
    const unsigned v = rows[size_t(i) * pitch + j];
    const v4u* s = reinterpret_cast<const v4u*>(vtab + 8u * v);
    v4u* d = reinterpret_cast<v4u*>(tabs + 8u * e);
    d[0] = s[0];
    d[1] = s[1];
}

constexpr size_t ff8_mat_lds_bytes(unsigned lb, unsigned c, unsigned N, unsigned waves) {
    return std::max<size_t>(size_t(lb) * N * 32, size_t(waves) * lb * c * 64 * 4);
}

}  // namespace

bool ff8_mat_supported(unsigned L, unsigned N) {
    return L >= 1 && L <= kFf8MatMaxOut && N >= 1 && N + L <= kFf8Ptrs;
}

// Columns: 4 dwords a lane (1 KiB strips) where that still gives every CU a
// workgroup with outputs in groups of at least 2, else a dword a lane.  Output
// groups of LB = 8 (4 with 4-dword lanes), 4, 2 or 1: the largest that still
// gives every CU a workgroup (a call of few column strips spreads its outputs
// over the GPU; one of many strips shares each input load and its selectors
// among LB outputs); kMatWaves waves with at most kMatInMax inputs each.
hipError_t launch_ff8_mat(const Ff8MatArgs& a, unsigned cus, hipStream_t s) {
    if (!ff8_mat_supported(a.L, a.N) || a.nunits == 0) return hipErrorInvalidValue;
    auto groups = [&](unsigned lb) { return (a.L + lb - 1) / lb; };
    const unsigned strips4 = (a.nunits + 255) / 256;
    unsigned c = strips4 * groups(2) >= cus ? 4u : 1u;
#if LAMD_EXPERIMENT_ENV
    static const int force_c = [] { const char* e = std::getenv("LEO_AMD_MAT_C"); return e ? std::atoi(e) : 0; }();
    if (force_c == 1 || force_c == 2 || force_c == 4) c = unsigned(force_c);
#endif
    const unsigned strips = (a.nunits + 64 * c - 1) / (64 * c);
    unsigned lb = c == 4 ? 4 : 8;
    while (lb > 1 && strips * groups(lb) < cus) lb /= 2;
#if LAMD_EXPERIMENT_ENV
    static const int force_lb = [] { const char* e = std::getenv("LEO_AMD_MAT_LB"); return e ? std::atoi(e) : 0; }();
    if (force_lb == 1 || force_lb == 2 || force_lb == 4 || (force_lb == 8 && c <= 2)) lb = unsigned(force_lb);
#endif
    // every wave of the workgroup in use even for few inputs: a small call is
    // bound by the chain through one wave (measured: 16 waves of 1-2 inputs beat
    // 2 waves of 12), a large one by the total instructions, which W barely changes
    const unsigned waves = kMatWaves;
    static_assert(kMatWaves * kMatInMax >= kFf8Ptrs, "every input has a wave");
    const dim3 grid(strips, groups(lb));
    void* params[] = {const_cast<Ff8MatArgs*>(&a)};
    const void* fn = nullptr;
    if (c == 4)
        fn = lb == 4   ? reinterpret_cast<const void*>(&k_ff8_mat<4, 4>)
             : lb == 2 ? reinterpret_cast<const void*>(&k_ff8_mat<2, 4>)
                       : reinterpret_cast<const void*>(&k_ff8_mat<1, 4>);
    else if (c == 2)
        fn = lb == 8   ? reinterpret_cast<const void*>(&k_ff8_mat<8, 2>)
             : lb == 4 ? reinterpret_cast<const void*>(&k_ff8_mat<4, 2>)
             : lb == 2 ? reinterpret_cast<const void*>(&k_ff8_mat<2, 2>)
                       : reinterpret_cast<const void*>(&k_ff8_mat<1, 2>);
    else
        fn = lb == 8   ? reinterpret_cast<const void*>(&k_ff8_mat<8, 1>)
             : lb == 4 ? reinterpret_cast<const void*>(&k_ff8_mat<4, 1>)
             : lb == 2 ? reinterpret_cast<const void*>(&k_ff8_mat<2, 1>)
                       : reinterpret_cast<const void*>(&k_ff8_mat<1, 1>);
    return hipLaunchKernel(fn, grid, dim3(64 * waves), params, ff8_mat_lds_bytes(lb, c, a.N, waves), s);
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
    const unsigned total = L * N;
    hipLaunchKernelGGL(k_ff8_mat_tabs, dim3((total + 255) / 256), dim3(256), 0, s, rows, pitch, L, N, vtab, tabs);
    return hipGetLastError();
}

}  // namespace lamd
