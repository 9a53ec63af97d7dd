// Microbenchmark (performance experiment only, not product code): cost of a
// GF(2^16) multiply-add by a wave-uniform constant, x ^= c * y, in two data
// layouts on gfx950.
//   perm:      the product's ALTMAP byte layout (FF16::muladd in rs_device.h):
//              12 v_perm_b32 byte-table lookups per 4 elements.
//   bitslice:  16 bit planes per 32 elements (plane k = bit k of 32 elements);
//              c * y is a 16 x 16 GF(2) matrix times the planes, evaluated by
//              the "four Russians" method: per group of 4 input planes the 16
//              XOR combinations, then each output plane = XOR of one combination
//              per group, selected by a wave-uniform 4-bit index (register
//              indexing, no memory).
// Both loops run N multiply-adds per lane with a different constant each time;
// the report is SIMD cycles per element (one element = one 16-bit field value).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_bitslice tools/ubench_bitslice.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            printf("%s: %s\n", #x, hipGetErrorString(e));                               \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }

constexpr int kConsts = 64;  // distinct constants cycled through

// ---------------------------------------------------------------- perm ----
// tabs: kConsts x 20 dwords (random: the cost does not depend on the values)
__global__ void __launch_bounds__(256) k_perm(const uint32_t* __restrict__ tabs, uint32_t* out, int iters) {
    uint32_t x[8][2], y[8][2];
    for (int u = 0; u < 8; ++u) {
        x[u][0] = threadIdx.x * 7 + u;
        x[u][1] = threadIdx.x * 13 + u;
        y[u][0] = threadIdx.x * 5 + u * 3;
        y[u][1] = threadIdx.x * 11 + u * 9;
    }
    for (int it = 0; it < iters; ++it) {
        const uint32_t* t = tabs + (it % kConsts) * 20;  // uniform: scalar loads
        uint32_t T[20];
#pragma unroll
        for (int i = 0; i < 20; ++i) T[i] = __builtin_amdgcn_readfirstlane(t[i]);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t lo = y[u][0], hi = y[u][1];
            const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
            const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
            x[u][0] = xor3(x[u][0], xor3(perm(T[1], T[0], a0), perm(T[5], T[4], a1), perm(T[9], T[8], b0)),
                           xor3(perm(T[13], T[12], b1), perm(T[16], T[16], a2), perm(T[18], T[18], b2)));
            x[u][1] = xor3(x[u][1], xor3(perm(T[3], T[2], a0), perm(T[7], T[6], a1), perm(T[11], T[10], b0)),
                           xor3(perm(T[15], T[14], b1), perm(T[17], T[17], a2), perm(T[19], T[19], b2)));
            // butterfly partner update (as in an FFT layer): y ^= x
            y[u][0] ^= x[u][0];
            y[u][1] ^= x[u][1];
        }
    }
    uint32_t acc = 0;
    for (int u = 0; u < 8; ++u) acc ^= x[u][0] ^ x[u][1] ^ y[u][0] ^ y[u][1];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// ------------------------------------------------------------ bitslice ----
// idx: kConsts x 8 dwords = 64 nibbles: nibble (j * 4 + g) selects the
// combination of group g for output plane j.
template <int NU>
__global__ void __launch_bounds__(256) k_bitslice(const uint32_t* __restrict__ idx, uint32_t* out, int iters) {
    uint32_t x[NU][16], y[NU][16];
    for (int u = 0; u < NU; ++u)
        for (int k = 0; k < 16; ++k) {
            x[u][k] = threadIdx.x * (7 + k) + u;
            y[u][k] = threadIdx.x * (5 + k) + u * 3;
        }
    for (int it = 0; it < iters; ++it) {
        const uint32_t* ix = idx + (it % kConsts) * 8;
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = __builtin_amdgcn_readfirstlane(ix[i]);
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            // one 16-entry array per group (register indexing needs each array
            // promoted to a vector of VGPRs; a [4][16] array stays in scratch)
            uint32_t c0[16], c1[16], c2[16], c3[16];
            auto build = [&](uint32_t* c, const uint32_t* v) {
                c[0] = 0;
                c[1] = v[0];
                c[2] = v[1];
                c[3] = v[0] ^ v[1];
                c[4] = v[2];
                c[5] = v[0] ^ v[2];
                c[6] = v[1] ^ v[2];
                c[7] = c[3] ^ v[2];
                c[8] = v[3];
#pragma unroll
                for (int q = 9; q < 16; ++q) c[q] = c[q - 8] ^ v[3];
            };
            build(c0, &y[u][0]);
            build(c1, &y[u][4]);
            build(c2, &y[u][8]);
            build(c3, &y[u][12]);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t wj = w[j >> 1] >> ((j & 1) * 16);
                const uint32_t i0 = __builtin_amdgcn_readfirstlane(wj & 15u);
                const uint32_t i1 = __builtin_amdgcn_readfirstlane((wj >> 4) & 15u);
                const uint32_t i2 = __builtin_amdgcn_readfirstlane((wj >> 8) & 15u);
                const uint32_t i3 = __builtin_amdgcn_readfirstlane((wj >> 12) & 15u);
                x[u][j] = xor3(x[u][j], c0[i0], c1[i1]) ^ c2[i2] ^ c3[i3];
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) y[u][k] ^= x[u][k];
        }
    }
    uint32_t acc = 0;
    for (int u = 0; u < NU; ++u)
        for (int k = 0; k < 16; ++k) acc ^= x[u][k] ^ y[u][k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 2000;
    std::vector<uint32_t> h(kConsts * 20);
    uint32_t s = 12345;
    for (auto& v : h) v = (s = s * 1664525u + 1013904223u);
    uint32_t *tabs, *idx, *out;
    CHECK(hipMalloc(&tabs, h.size() * 4));
    CHECK(hipMalloc(&idx, h.size() * 4));
    CHECK(hipMalloc(&out, size_t(blocks) * threads * 4));
    CHECK(hipMemcpy(tabs, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    int clk_khz = 0;
    CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
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
        const double simd_cycles = ms * 1e-3 * 2.4e9 * 256 * 4;  // at 2.4 GHz, 1024 SIMDs
        printf("%-28s %8.3f ms  %7.3f G mul-add elems/s  %6.3f SIMD-cycles/elem (at 2.4 GHz; rated clock %d MHz)\n",
               name, ms, elems / (ms * 1e-3) / 1e9, simd_cycles / elems * 64, clk_khz / 1000);
        return 0;
    };
    if (run("perm (ALTMAP bytes)", [&] { hipLaunchKernelGGL(k_perm, blocks, threads, 0, 0, tabs, out, iters); }, 32.0))
        return 1;
    if (run("bitslice four-Russians x1", [&] { hipLaunchKernelGGL(k_bitslice<1>, blocks, threads, 0, 0, idx, out, iters); }, 32.0))
        return 1;
    if (run("bitslice four-Russians x2", [&] { hipLaunchKernelGGL(k_bitslice<2>, blocks, threads, 0, 0, idx, out, iters); }, 64.0))
        return 1;
    return 0;
}
