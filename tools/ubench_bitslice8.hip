// Microbenchmark (performance experiment only, not product code): cost of a
// GF(2^8) butterfly  x ^= c * y; y ^= x  by a wave-uniform constant c on gfx950,
// per 32 elements a lane (8 dwords), in the forms a GF(2^8) tile could use:
//   perm      today's byte layout (FF8::muladd): 3 v_perm_b32 per 4 elements
//   r2 / r3   bit-sliced planes (plane k = bit k of 32 elements), c * y as an
//             8 x 8 GF(2) matrix by the "four Russians" method: the XOR
//             combinations of each group of input planes (2 groups of 4 or
//             3 groups of 3, 3, 2), each output plane = XOR of one combination
//             per group picked by a wave-uniform index (register indexing)
//   mask      bit-sliced, out_i ^= y_j & m_ij with 64 SGPR masks (v_bitop3)
//   fixed     bit-sliced, a compile-time constant (an XOR network)
//   xpose     byte -> plane -> byte transposes of 8 dwords (no multiply)
// The report is SIMD cycles per element at the measured clock.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_bitslice8 tools/ubench_bitslice8.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                          \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            printf("%s: %s\n", #x, hipGetErrorString(e));                 \
            return 1;                                                     \
        }                                                                 \
    } while (0)

#define LDEV __device__ __forceinline__
LDEV uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
LDEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
LDEV uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

constexpr int kConsts = 64;
using v16u = unsigned __attribute__((ext_vector_type(16)));
using v8u = unsigned __attribute__((ext_vector_type(8)));
using v4u = unsigned __attribute__((ext_vector_type(4)));

template <int NU>
struct Data {
    uint32_t x[NU][8], y[NU][8];
    LDEV void init() {
        for (int u = 0; u < NU; ++u)
            for (int k = 0; k < 8; ++k) {
                x[u][k] = threadIdx.x * (7 + k) + u;
                y[u][k] = threadIdx.x * (5 + k) + u * 3;
            }
    }
    LDEV uint32_t fold() const {
        uint32_t acc = 0;
        for (int u = 0; u < NU; ++u)
            for (int k = 0; k < 8; ++k) acc ^= x[u][k] ^ y[u][k];
        return acc;
    }
};

// ---- perm: 5 dwords of tables per constant ----
template <int NU>
__global__ void __launch_bounds__(256) k_perm(const uint32_t* __restrict__ tabs, uint32_t* out, int iters) {
    Data<NU> d;
    d.init();
    for (int it = 0; it < iters; ++it) {
        const uint32_t* t = tabs + (it % kConsts) * 8;
        const uint32_t a0 = uni(t[0]), a1 = uni(t[1]), b0 = uni(t[2]), b1 = uni(t[3]), c0 = uni(t[4]);
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t y = d.y[u][k];
                const uint32_t s0 = y & 0x07070707u, s1 = (y >> 3) & 0x07070707u, s2 = (y >> 6) & 0x03030303u;
                d.x[u][k] = xor3(d.x[u][k], perm(a1, a0, s0), perm(b1, b0, s1)) ^ perm(c0, c0, s2);
                d.y[u][k] ^= d.x[u][k];
            }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = d.fold();
}

// ---- four Russians, 2 groups of 4 planes: indices = 8 bytes (row i: lo nibble group A, hi nibble group B) ----
template <int NU>
__global__ void __launch_bounds__(256) k_r2(const uint32_t* __restrict__ idx, uint32_t* out, int iters) {
    Data<NU> d;
    d.init();
    for (int it = 0; it < iters; ++it) {
        const uint32_t* ix = idx + (it % kConsts) * 8;
        const uint32_t w0 = uni(ix[0]), w1 = uni(ix[1]);
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            v16u ca, cb;
            auto build = [&](v16u& c, const uint32_t* v) {
                c[0] = 0;
                c[1] = v[0];
                c[2] = v[1];
                c[3] = v[0] ^ v[1];
                c[4] = v[2];
                c[5] = v[0] ^ v[2];
                c[6] = v[1] ^ v[2];
                c[7] = xor3(v[0], v[1], v[2]);
                c[8] = v[3];
                c[9] = v[0] ^ v[3];
                c[10] = v[1] ^ v[3];
                c[11] = xor3(v[0], v[1], v[3]);
                c[12] = v[2] ^ v[3];
                c[13] = xor3(v[0], v[2], v[3]);
                c[14] = xor3(v[1], v[2], v[3]);
                c[15] = c[3] ^ c[12];
            };
            build(ca, &d.y[u][0]);
            build(cb, &d.y[u][4]);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t wb = (i < 4 ? w0 : w1) >> ((i & 3) * 8);
                const uint32_t ia = uni(wb & 15u), ib = uni((wb >> 4) & 15u);
                d.x[u][i] = xor3(d.x[u][i], ca[ia], cb[ib]);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = d.fold();
}

// ---- four Russians, 3 groups (planes 0-2, 3-5, 6-7): row i = 3+3+2 index bits ----
template <int NU>
__global__ void __launch_bounds__(256) k_r3(const uint32_t* __restrict__ idx, uint32_t* out, int iters) {
    Data<NU> d;
    d.init();
    for (int it = 0; it < iters; ++it) {
        const uint32_t* ix = idx + (it % kConsts) * 8;
        const uint32_t w0 = uni(ix[0]), w1 = uni(ix[1]);
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            v8u ca, cb;
            v4u cc;
            auto build3 = [&](v8u& c, const uint32_t* v) {
                c[0] = 0;
                c[1] = v[0];
                c[2] = v[1];
                c[3] = v[0] ^ v[1];
                c[4] = v[2];
                c[5] = v[0] ^ v[2];
                c[6] = v[1] ^ v[2];
                c[7] = xor3(v[0], v[1], v[2]);
            };
            build3(ca, &d.y[u][0]);
            build3(cb, &d.y[u][3]);
            cc[0] = 0;
            cc[1] = d.y[u][6];
            cc[2] = d.y[u][7];
            cc[3] = d.y[u][6] ^ d.y[u][7];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t wb = (i < 4 ? w0 : w1) >> ((i & 3) * 8);
                const uint32_t ia = uni(wb & 7u), ib = uni((wb >> 3) & 7u), ic = uni((wb >> 6) & 3u);
                d.x[u][i] = xor3(d.x[u][i], ca[ia], cb[ib]) ^ cc[ic];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = d.fold();
}

// ---- mask: 64 SGPR masks per constant (m_ij = -(bit j of row i)) ----
template <int NU>
__global__ void __launch_bounds__(256) k_mask(const uint32_t* __restrict__ masks, uint32_t* out, int iters) {
    Data<NU> d;
    d.init();
    for (int it = 0; it < iters; ++it) {
        const uint32_t* m = masks + (it % kConsts) * 64;
        uint32_t M[64];
#pragma unroll
        for (int i = 0; i < 64; ++i) M[i] = uni(m[i]);
#pragma unroll
        for (int u = 0; u < NU; ++u) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t a = d.x[u][i];
#pragma unroll
                for (int j = 0; j < 8; ++j) a = __builtin_amdgcn_bitop3_b32(a, d.y[u][j], M[8 * i + j], 0x78);  // a ^ (b & c)
                d.x[u][i] = a;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = d.fold();
}

// ---- fixed: compile-time matrices (rows with 4 ones on average), cycled over 4 ----
template <uint64_t M>
LDEV void fixed_muladd(uint32_t* x, const uint32_t* y) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t a = x[i];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((M >> (8 * i + j)) & 1) a ^= y[j];
        x[i] = a;
    }
}
template <int NU>
__global__ void __launch_bounds__(256) k_fixed(const uint32_t*, uint32_t* out, int iters) {
    Data<NU> d;
    d.init();
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            fixed_muladd<0x9A3C5E71B2D48F06ull>(d.x[u], d.y[u]);
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
            fixed_muladd<0x4D71E29B3A6C85F0ull>(d.x[u], d.y[u]);
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
            fixed_muladd<0xC3B5691E7248DA2Full>(d.x[u], d.y[u]);
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
            fixed_muladd<0x2E8F47A1D5693CB0ull>(d.x[u], d.y[u]);
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = d.fold();
}

// ---- transposes: 8 dwords of bytes <-> 8 bit planes ----
// swap bit groups: a' = (a & ~M) | ((b << s) & M) ... as delta swaps.
template <int S, uint32_t MASK>
LDEV void dswap(uint32_t& a, uint32_t& b) {
    // bits of a at positions in MASK<<S exchange with bits of b at positions MASK
    const uint32_t t = ((a >> S) ^ b) & MASK;
    b ^= t;
    a ^= t << S;
}
LDEV void to_planes(uint32_t* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) dswap<4, 0x0F0F0F0Fu>(v[i + 4], v[i]);
#pragma unroll
    for (int i = 0; i < 8; i += 4)
#pragma unroll
        for (int j = 0; j < 2; ++j) dswap<2, 0x33333333u>(v[i + j + 2], v[i + j]);
#pragma unroll
    for (int i = 0; i < 8; i += 2) dswap<1, 0x55555555u>(v[i + 1], v[i]);
}
// merge form: a' = (a & ~M<<S) | (b << S & M<<S) ... 4 ops a pair (2 shifts, 2 v_bitop3)
template <int S, uint32_t MASK>
LDEV void mswap(uint32_t& a, uint32_t& b) {
    // the same exchange as dswap<S, MASK>(a, b) as two bit selects (v_bitop3
    // truth table 0xD8: src2 ? src1 : src0)
    const uint32_t na = __builtin_amdgcn_bitop3_b32(b << S, a, MASK, 0xD8);  // MASK ? a : b << S
    const uint32_t nb = __builtin_amdgcn_bitop3_b32(b, a >> S, MASK, 0xD8);  // MASK ? a >> S : b
    a = na;
    b = nb;
}
LDEV void to_planes2(uint32_t* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) mswap<4, 0x0F0F0F0Fu>(v[i + 4], v[i]);
#pragma unroll
    for (int i = 0; i < 8; i += 4)
#pragma unroll
        for (int j = 0; j < 2; ++j) mswap<2, 0x33333333u>(v[i + j + 2], v[i + j]);
#pragma unroll
    for (int i = 0; i < 8; i += 2) mswap<1, 0x55555555u>(v[i + 1], v[i]);
}
template <int NU, int F>
__global__ void __launch_bounds__(256) k_xpose(const uint32_t*, uint32_t* out, int iters) {
    Data<NU> d;
    d.init();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            if constexpr (F == 0) to_planes(d.x[u]);
            else to_planes2(d.x[u]);
            d.x[u][0] ^= uint32_t(it);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = d.fold();
}

// ---- per-lane twist (the (B) tile's low layers): x ^= a*y ^ sum_b g_b (H_b*y), a, H_b compile time,
//      g_b per-lane masks ----
template <uint64_t M>
LDEV void fixed_prod(uint32_t* t, const uint32_t* y) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t a = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((M >> (8 * i + j)) & 1) a ^= y[j];
        t[i] = a;
    }
}
template <uint64_t M>
LDEV void masked_muladd(uint32_t* x, const uint32_t* y, uint32_t g) {
    uint32_t t[8];
    fixed_prod<M>(t, y);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_bitop3_b32(x[i], t[i], g, 0x78);  // x ^ (t & g)
}
template <int NU>
__global__ void __launch_bounds__(256) k_twist(const uint32_t*, uint32_t* out, int iters) {
    Data<NU> d;
    d.init();
    const uint32_t g0 = (threadIdx.x & 8) ? ~0u : 0u, g1 = (threadIdx.x & 16) ? ~0u : 0u,
                   g2 = (threadIdx.x & 32) ? ~0u : 0u;
    for (int it = 0; it < iters; it += 2) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            fixed_muladd<0x9A3C5E71B2D48F06ull>(d.x[u], d.y[u]);
            masked_muladd<0x4D71E29B3A6C85F0ull>(d.x[u], d.y[u], g0);
            masked_muladd<0xC3B5691E7248DA2Full>(d.x[u], d.y[u], g1);
            masked_muladd<0x2E8F47A1D5693CB0ull>(d.x[u], d.y[u], g2);
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
            fixed_muladd<0x71B2D48F069A3C5Eull>(d.x[u], d.y[u]);
            masked_muladd<0x3A6C85F04D71E29Bull>(d.x[u], d.y[u], g0);
            masked_muladd<0x7248DA2FC3B5691Eull>(d.x[u], d.y[u], g1);
            masked_muladd<0xD5693CB02E8F47A1ull>(d.x[u], d.y[u], g2);
            for (int k = 0; k < 8; ++k) d.y[u][k] ^= d.x[u][k];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = d.fold();
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 2000;
    std::vector<uint32_t> h(kConsts * 64);
    uint32_t s = 12345;
    for (auto& v : h) v = (s = s * 1664525u + 1013904223u);
    std::vector<uint32_t> hm(kConsts * 64);
    for (size_t i = 0; i < hm.size(); ++i) hm[i] = (h[i] & 1) ? ~0u : 0u;
    uint32_t *tabs, *masks, *out;
    CHECK(hipMalloc(&tabs, h.size() * 4));
    CHECK(hipMalloc(&masks, hm.size() * 4));
    CHECK(hipMalloc(&out, size_t(blocks) * threads * 4));
    CHECK(hipMemcpy(tabs, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(masks, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch, double elems_per_lane_iter) -> int {
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double elems = double(blocks) * threads * iters * elems_per_lane_iter;
        const double simd_cycles = ms * 1e-3 * 2.3e9 * 256 * 4;  // 2.3 GHz measured in-kernel clock, 1024 SIMDs
        printf("%-26s %8.3f ms  %7.2f G elem/s  %6.3f SIMD-cycles/elem  (%6.1f cycles per 32-element butterfly)\n", name,
               ms, elems / (ms * 1e-3) / 1e9, simd_cycles / elems * 64, simd_cycles / elems * 64 * 32);
        return 0;
    };
#define RUN(name, K, buf, per)                                                                              \
    if (run(name, [&] { hipLaunchKernelGGL(K, blocks, threads, 0, 0, buf, out, iters); }, per)) return 1;
    RUN("perm x1", k_perm<1>, tabs, 32.0)
    RUN("perm x2", k_perm<2>, tabs, 64.0)
    RUN("r2 (2x4 four Russians) x1", k_r2<1>, tabs, 32.0)
    RUN("r2 x2", k_r2<2>, tabs, 64.0)
    RUN("r3 (3+3+2 four Russians) x1", k_r3<1>, tabs, 32.0)
    RUN("r3 x2", k_r3<2>, tabs, 64.0)
    RUN("mask (bitop3, SGPR) x1", k_mask<1>, masks, 32.0)
    RUN("mask x2", k_mask<2>, masks, 64.0)
    RUN("fixed (XOR network) x1", k_fixed<1>, tabs, 32.0)
    RUN("fixed x2", k_fixed<2>, tabs, 64.0)
    RUN("xpose delta-swap x1", (k_xpose<1, 0>), tabs, 32.0)
    RUN("xpose delta-swap x2", (k_xpose<2, 0>), tabs, 64.0)
    RUN("xpose merge x1", (k_xpose<1, 1>), tabs, 32.0)
    RUN("xpose merge x2", (k_xpose<2, 1>), tabs, 64.0)
    RUN("twist (fixed + 3 masked) x1", k_twist<1>, tabs, 32.0)
    RUN("twist x2", k_twist<2>, tabs, 64.0)
    return 0;
}
