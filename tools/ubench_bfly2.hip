// Butterfly instruction-sequence variants on gfx950 (performance experiment
// only): cycles per IFFT butterfly (y ^= x; x ^= y * c) per SIMD, 16 values per
// lane (8 independent butterflies per layer), at 2 / 4 / 8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_bfly2 tools/ubench_bfly2.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

struct Tab { uint32_t a0, a1, b0, b1, c0; };

template <int V>
__device__ __forceinline__ void muladd(uint32_t& x, uint32_t y, const Tab& t, uint32_t m7, uint32_t m3) {
    if constexpr (V == 0) {  // as the library writes it (compiler fuses (x^y)&M into bitop3)
        const uint32_t s0 = y & 0x07070707u, s1 = (y >> 3) & 0x07070707u, s2 = (y >> 6) & 0x03030303u;
        x = xor3(x, perm(t.a1, t.a0, s0), perm(t.b1, t.b0, s1)) ^ perm(t.c0, t.c0, s2);
    } else if constexpr (V == 1 || V == 2) {  // y materialised first: all-VOP2 selector extraction
        asm volatile("" : "+v"(y));
        const uint32_t M7 = V == 1 ? 0x07070707u : m7, M3 = V == 1 ? 0x03030303u : m3;
        const uint32_t s0 = y & M7, s1 = (y >> 3) & M7, s2 = (y >> 6) & M3;
        x = xor3(x, perm(t.a1, t.a0, s0), perm(t.b1, t.b0, s1)) ^ perm(t.c0, t.c0, s2);
    } else if constexpr (V == 3) {  // 2 perms only (wrong math, cost probe)
        asm volatile("" : "+v"(y));
        const uint32_t s0 = y & 0x07070707u, s1 = (y >> 4) & 0x07070707u;
        x = xor3(x, perm(t.a1, t.a0, s0), perm(t.b1, t.b0, s1));
    } else if constexpr (V == 4) {  // plain xors instead of xor3
        asm volatile("" : "+v"(y));
        const uint32_t s0 = y & 0x07070707u, s1 = (y >> 3) & 0x07070707u, s2 = (y >> 6) & 0x03030303u;
        uint32_t p0 = perm(t.a1, t.a0, s0), p1 = perm(t.b1, t.b0, s1), p2 = perm(t.c0, t.c0, s2);
        asm volatile("" : "+v"(p0), "+v"(p1), "+v"(p2));
        x ^= p0; x ^= p1; x ^= p2;
    }
}

template <int V>
__global__ void __launch_bounds__(256) k(uint32_t* out, const uint32_t* tabs, int iters) {
    uint32_t v[16];
    for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 2654435761u + i * 40503u;
    const unsigned lane = threadIdx.x & 63;
    Tab t[4];
    for (int g = 0; g < 4; ++g) {
        const uint32_t* p = tabs + ((lane + g) & 7) * 8;
        t[g] = Tab{p[0], p[1], p[2], p[3], p[4]};
    }
    uint32_t m7, m3;  // masks forced into SGPRs
    asm volatile("s_mov_b32 %0, 0x7070707" : "=s"(m7));
    asm volatile("s_mov_b32 %0, 0x3030303" : "=s"(m3));
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t& a = v[j];
            uint32_t& b = v[j + 8];
            b ^= a;
            muladd<V>(a, b, t[j & 3], m7, m3);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t& a = v[2 * j];
            uint32_t& b = v[2 * j + 1];
            b ^= a;
            muladd<V>(a, b, t[(j + 1) & 3], m7, m3);
        }
    }
    uint32_t acc = 0;
    for (int i = 0; i < 16; ++i) acc ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int V>
int run(uint32_t* out, uint32_t* tabs, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int wps : {2, 4, 8}) {
        const int blocks = cus * wps, iters = 2000;
        hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, out, tabs, 10);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, out, tabs, iters);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double bf = double(wps) * iters * 16;
        printf("variant=%d waves/SIMD=%d  %.2f cyc/butterfly/SIMD @2.4GHz\n", V, wps, ms * 1e6 / bf * 2.4);
    }
    return 0;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    uint32_t *out, *tabs;
    CHECK(hipMalloc(&out, 64u << 20));
    CHECK(hipMalloc(&tabs, 4096));
    CHECK(hipMemset(tabs, 0x35, 4096));
    const int cus = prop.multiProcessorCount;
    run<0>(out, tabs, cus);
    run<1>(out, tabs, cus);
    run<2>(out, tabs, cus);
    run<3>(out, tabs, cus);
    run<4>(out, tabs, cus);
    return 0;
}
