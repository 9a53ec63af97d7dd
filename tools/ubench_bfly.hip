// Register-only microbenchmark of the FF8 butterfly (v_perm GF multiply +
// xor3) on gfx950: cycles per butterfly per SIMD at several waves per SIMD.
// Performance experiment only; not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -o ubench_bfly tools/ubench_bfly.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

struct Tab { uint32_t a0, a1, b0, b1, c0; };

__device__ __forceinline__ void muladd(uint32_t& x, uint32_t y, const Tab& t) {
    const uint32_t s0 = y & 0x07070707u;
    const uint32_t s1 = (y >> 3) & 0x07070707u;
    const uint32_t s2 = (y >> 6) & 0x03030303u;
    x = xor3(x, perm(t.a1, t.a0, s0), perm(t.b1, t.b0, s1)) ^ perm(t.c0, t.c0, s2);
}

// MODE 0: IFFT-style butterflies (y ^= x; x ^= y*c), 8 independent pairs
// MODE 1: only the xor part (no multiply): cost of the rest
template <int MODE>
__global__ void k(uint32_t* out, const uint32_t* tabs, int iters) {
    uint32_t v[16];
    for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 2654435761u + i * 40503u;
    const unsigned lane = threadIdx.x & 63;
    Tab t[4];
    for (int g = 0; g < 4; ++g) {
        const uint32_t* p = tabs + ((lane + g) & 7) * 8;
        t[g] = Tab{p[0], p[1], p[2], p[3], p[4]};
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t& a = v[j];
            uint32_t& b = v[j + 8];
            b ^= a;
            if constexpr (MODE == 0) muladd(a, b, t[j & 3]);
            else a ^= b + 0x9E3779B9u;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t& a = v[2 * j];
            uint32_t& b = v[2 * j + 1];
            b ^= a;
            if constexpr (MODE == 0) muladd(a, b, t[(j + 1) & 3]);
            else a ^= b + 0x7F4A7C15u;
        }
    }
    uint32_t acc = 0;
    for (int i = 0; i < 16; ++i) acc ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    int cus = 0;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    cus = prop.multiProcessorCount;
    const int clock_khz = prop.clockRate;
    uint32_t *out, *tabs;
    CHECK(hipMalloc(&out, 64u << 20));
    CHECK(hipMalloc(&tabs, 4096));
    CHECK(hipMemset(tabs, 0x35, 4096));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int iters = 2000;
    printf("CUs=%d clock=%d MHz\n", cus, clock_khz / 1000);
    for (int mode = 0; mode < 2; ++mode) {
        for (int wps : {1, 2, 4, 8}) {  // waves per SIMD
            const int threads = 256;     // 4 waves per block, one per SIMD
            const int blocks = cus * wps;
            auto fn = mode == 0 ? k<0> : k<1>;
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(threads), 0, 0, out, tabs, 10);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(threads), 0, 0, out, tabs, iters);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            // butterflies per SIMD: waves per SIMD * iters * 16
            const double bf_per_simd = double(wps) * iters * 16;
            const double ns_per_bf = ms * 1e6 / bf_per_simd;
            printf("mode=%d waves/SIMD=%d  %.3f ms  %.3f ns per butterfly per SIMD (%.2f cyc @2.4GHz)\n", mode, wps, ms,
                   ns_per_bf, ns_per_bf * 2.4);
        }
    }
    return 0;
}
