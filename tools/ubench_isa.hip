// Per-instruction VALU throughput on gfx950 (performance experiment only):
// cycles per wave-instruction per SIMD for the ops a GF(2^8)/GF(2^16) butterfly
// uses, at 2 and 8 waves per SIMD, 16 independent chains per wave.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_isa tools/ubench_isa.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, int iters, uint32_t seed) {
    uint32_t v[16], a = seed ^ threadIdx.x, b = seed * 3u + threadIdx.x, c = 0x07070707u;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 2654435761u + i;
    for (int it = 0; it < iters; ++it) {
#define OPX(i)                                                                                             \
    if constexpr (OP == 0) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a), "v"(b));      \
    if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b)); \
    if constexpr (OP == 2) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(a));                   \
    if constexpr (OP == 3) asm volatile("v_and_b32 %0, 0x7070707, %0" : "+v"(v[i]));                     \
    if constexpr (OP == 4) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v[i]));                         \
    if constexpr (OP == 5) asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[i]) : "v"(c));                   \
    if constexpr (OP == 6) asm volatile("v_bfe_u32 %0, %0, 3, 3" : "+v"(v[i]));                          \
    if constexpr (OP == 7) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));      \
    if constexpr (OP == 8) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "s"(a), "v"(b));      \
    if constexpr (OP == 9) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));    \
    if constexpr (OP == 10) asm volatile("v_mov_b32_dpp %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(v[i])); \
    if constexpr (OP == 11) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(v[i]), "+v"(a));          \
    if constexpr (OP == 12) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(v[i]) : "v"(a));
        REP16(OPX)
    }
    uint32_t acc = a;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static const char* names[] = {"v_perm_b32", "v_bitop3_b32", "v_xor_b32", "v_and_b32 lit", "v_lshrrev_b32",
                              "v_and_b32 reg", "v_bfe_u32", "v_add3_u32", "v_perm sgpr", "v_and_or_b32",
                              "v_mov_dpp ror8", "v_permlane32_swap", "v_lshl_or_b32"};

template <int OP>
int run(uint32_t* out, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int wps : {1, 2, 8}) {
        const int blocks = cus * wps, iters = 4000;
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 10, 1u);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double inst_per_simd = double(wps) * iters * 16;
        printf("%-18s waves/SIMD=%d  %6.2f cyc/inst/SIMD @2.4GHz\n", names[OP], wps, ms * 1e6 / inst_per_simd * 2.4);
    }
    return 0;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    uint32_t* out;
    CHECK(hipMalloc(&out, 64u << 20));
    int cus = prop.multiProcessorCount;
    run<0>(out, cus); run<1>(out, cus); run<2>(out, cus); run<3>(out, cus); run<4>(out, cus);
    run<5>(out, cus); run<6>(out, cus); run<7>(out, cus); run<8>(out, cus); run<9>(out, cus);
    run<10>(out, cus); run<11>(out, cus); run<12>(out, cus);
    return 0;
}
