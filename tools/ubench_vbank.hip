// Microbenchmark (performance experiment only): does the VGPR bank of a
// VOP3's three sources (register index mod 4) change its issue rate on gfx950?
// 8 independent v_bitop3_b32 chains on fixed registers, sources in one bank vs
// in three banks, at 1, 2 and 4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_vbank tools/ubench_vbank.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                  \
    do {                                                          \
        hipError_t e = (x);                                       \
        if (e != hipSuccess) {                                    \
            printf("%s: %s\n", #x, hipGetErrorString(e));         \
            return 1;                                             \
        }                                                         \
    } while (0)

#define S8(A, B, C)                                                                               \
    "v_bitop3_b32 v" #A "0, v" #A "0, v" #B "0, v" #C "0 bitop3:0x96\n"                          \
    "v_bitop3_b32 v" #A "4, v" #A "4, v" #B "4, v" #C "4 bitop3:0x96\n"                          \
    "v_bitop3_b32 v" #A "8, v" #A "8, v" #B "8, v" #C "8 bitop3:0x96\n"
// same bank: dst/src0 v{10,14,18,...}, src1 v{40,...}, src2 v{70,...}: all index = 2 mod 4 / 0 mod 4
constexpr int kIters = 2048;

template <int MODE>
__global__ void __launch_bounds__(256) k_bank(uint32_t* out, uint64_t* clk) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
        if constexpr (MODE == 0)  // sources in one bank (index mod 4 equal)
            asm volatile(
                "v_bitop3_b32 v10, v10, v40, v70 bitop3:0x96\n v_bitop3_b32 v14, v14, v44, v74 bitop3:0x96\n"
                "v_bitop3_b32 v18, v18, v48, v78 bitop3:0x96\n v_bitop3_b32 v22, v22, v52, v82 bitop3:0x96\n"
                "v_bitop3_b32 v26, v26, v56, v86 bitop3:0x96\n v_bitop3_b32 v30, v30, v60, v90 bitop3:0x96\n"
                "v_bitop3_b32 v34, v34, v64, v94 bitop3:0x96\n v_bitop3_b32 v38, v38, v68, v98 bitop3:0x96\n"
                ::: "v10", "v14", "v18", "v22", "v26", "v30", "v34", "v38", "v40", "v44", "v48", "v52", "v56", "v60",
                "v64", "v68", "v70", "v74", "v78", "v82", "v86", "v90", "v94", "v98");
        if constexpr (MODE == 1)  // sources in three banks
            asm volatile(
                "v_bitop3_b32 v10, v10, v41, v71 bitop3:0x96\n v_bitop3_b32 v14, v14, v45, v75 bitop3:0x96\n"
                "v_bitop3_b32 v18, v18, v49, v79 bitop3:0x96\n v_bitop3_b32 v22, v22, v53, v83 bitop3:0x96\n"
                "v_bitop3_b32 v26, v26, v57, v87 bitop3:0x96\n v_bitop3_b32 v30, v30, v61, v91 bitop3:0x96\n"
                "v_bitop3_b32 v34, v34, v65, v95 bitop3:0x96\n v_bitop3_b32 v38, v38, v69, v99 bitop3:0x96\n"
                ::: "v10", "v14", "v18", "v22", "v26", "v30", "v34", "v38", "v41", "v45", "v49", "v53", "v57", "v61",
                "v65", "v69", "v71", "v75", "v79", "v83", "v87", "v91", "v95", "v99");
        if constexpr (MODE == 2)  // v_xor_b32, both sources one bank
            asm volatile(
                "v_xor_b32 v10, v10, v40\n v_xor_b32 v14, v14, v44\n v_xor_b32 v18, v18, v48\n v_xor_b32 v22, v22, v52\n"
                "v_xor_b32 v26, v26, v56\n v_xor_b32 v30, v30, v60\n v_xor_b32 v34, v34, v64\n v_xor_b32 v38, v38, v68\n"
                ::: "v10", "v14", "v18", "v22", "v26", "v30", "v34", "v38", "v40", "v44", "v48", "v52", "v56", "v60",
                "v64", "v68");
        if constexpr (MODE == 3)  // v_xor_b32, two banks
            asm volatile(
                "v_xor_b32 v10, v10, v41\n v_xor_b32 v14, v14, v45\n v_xor_b32 v18, v18, v49\n v_xor_b32 v22, v22, v53\n"
                "v_xor_b32 v26, v26, v57\n v_xor_b32 v30, v30, v61\n v_xor_b32 v34, v34, v65\n v_xor_b32 v38, v38, v69\n"
                ::: "v10", "v14", "v18", "v22", "v26", "v30", "v34", "v38", "v41", "v45", "v49", "v53", "v57", "v61",
                "v65", "v69");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) clk[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = threadIdx.x;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* out;
    uint64_t* clk;
    CHECK(hipMalloc(&out, size_t(cus) * 4 * 256 * 4));
    CHECK(hipMalloc(&clk, size_t(cus) * 4 * 4 * 8));
    static uint64_t h[256 * 4 * 4 * 4];
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const char* names[] = {"v_bitop3 3 sources, one bank", "v_bitop3 3 sources, 3 banks", "v_xor 2 sources, one bank",
                           "v_xor 2 sources, 2 banks"};
    auto run = [&](int mode, auto kern) -> int {
        for (int wps : {1, 2, 4}) {
            const int blocks = cus * wps;
            hipLaunchKernelGGL(kern, blocks, 256, 0, 0, out, clk);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(kern, blocks, 256, 0, 0, out, clk);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            CHECK(hipMemcpy(h, clk, size_t(blocks) * 4 * 8, hipMemcpyDeviceToHost));
            double cyc = 0;
            for (int i = 0; i < blocks * 4; ++i) cyc += double(h[i]);
            cyc /= blocks * 4;
            const double instr = double(kIters) * 8;
            printf("%-32s waves/SIMD=%d: %6.2f wave-cycles/instr, %5.2f SIMD-cycles/instr (wall, 2.3 GHz)\n",
                   names[mode], wps, cyc / instr, ms * 1e-3 * 2.3e9 / (instr * wps));
        }
        return 0;
    };
    if (run(0, k_bank<0>) || run(1, k_bank<1>) || run(2, k_bank<2>) || run(3, k_bank<3>)) return 1;
    return 0;
}
