// GF(2^16) butterfly throughput on gfx950 (performance experiment only): the
// FF16 IFFT butterfly of rs_device.h (y ^= x; x ^= y * c, 12 v_perm_b32 per 4
// elements) in registers, tables in VGPRs, no memory.  Reports SIMD cycles per
// wave-butterfly at several waves per SIMD, to separate VALU issue capacity
// from the multi-pass kernels' latency / memory stalls.
//   hipcc --offload-arch=gfx950 -O3 -I leopard_amd/csrc -o tools/bin/ubench_ff16 tools/ubench_ff16.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "rs_device.h"

using namespace lamd;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// NR pieces per lane, 2 dwords each; ITERS x (NR/2 butterflies) per launch.
template <int NR, int INFL>
__global__ void __launch_bounds__(256) k_bfly(uint32_t* out, const uint32_t* tabs, int iters) {
    uint32_t x[NR][2];
    for (int i = 0; i < NR; ++i) { x[i][0] = threadIdx.x * 2654435761u + i * 40503u; x[i][1] = x[i][0] * 7u + 3u; }
    FF16::Tab t;
    for (int i = 0; i < 20; ++i) t.t[i] = tabs[(threadIdx.x & 7) * 24 + i];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < NR / 2; ++j) {
            uint32_t* a = x[2 * j];
            uint32_t* b = x[2 * j + 1];
            b[0] ^= a[0];
            b[1] ^= a[1];
            FF16::muladd(a, b, t);
            asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]));
            if (j % INFL == INFL - 1) __builtin_amdgcn_sched_barrier(0);
        }
        // rotate pairings so the next iteration depends on this one
        uint32_t s0 = x[0][0], s1 = x[0][1];
#pragma unroll
        for (int i = 0; i + 1 < NR; ++i) { x[i][0] = x[i + 1][0]; x[i][1] = x[i + 1][1]; }
        x[NR - 1][0] = s0; x[NR - 1][1] = s1;
    }
    uint32_t acc = 0;
    for (int i = 0; i < NR; ++i) acc ^= x[i][0] ^ x[i][1];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NR, int INFL>
int run(uint32_t* out, const uint32_t* tabs, int waves_per_simd) {
    const int iters = 2000;
    const int blocks = 256 * waves_per_simd;  // 256-thread blocks: 4 waves = one per SIMD
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_bfly<NR, INFL>), dim3(blocks), dim3(256), 0, 0, out, tabs, 10);
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((k_bfly<NR, INFL>), dim3(blocks), dim3(256), 0, 0, out, tabs, iters);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double cycles = ms * 1e-3 * 2.4e9;  // at 2.4 GHz
    const double bfly_per_simd = double(iters) * (NR / 2) * waves_per_simd;  // wave-butterflies per SIMD
    printf("NR=%2d inflight=%d waves/SIMD=%d: %.1f SIMD cycles per wave-butterfly (%.1f us)\n", NR, INFL,
           waves_per_simd, cycles / bfly_per_simd, ms * 1e3);
    return 0;
}

int main() {
    uint32_t *out, *tabs;
    CHECK(hipMalloc(&out, 256 * 8 * 256 * 4 * 4));
    CHECK(hipMalloc(&tabs, 8 * 24 * 4));
    uint32_t h[8 * 24];
    for (int i = 0; i < 8 * 24; ++i) h[i] = (i * 0x9E3779B9u) & 0x07070707u;  // any bytes: cost probe
    CHECK(hipMemcpy(tabs, h, sizeof(h), hipMemcpyHostToDevice));
    for (int w : {1, 2, 4, 8}) run<16, 2>(out, tabs, w);
    for (int w : {1, 2, 4}) run<32, 2>(out, tabs, w);
    for (int w : {2, 4}) run<32, 1>(out, tabs, w);
    for (int w : {2, 4}) run<32, 4>(out, tabs, w);
    return 0;
}
