// Microbenchmark (performance experiment only): VALU issue cost on gfx950 at
// 1, 2, 3 and 4 waves per SIMD for the instruction forms of the bit-sliced
// GF(2^8) tile (rs_ff8_bs.hip): v_xor_b32 (VOP2), v_bitop3_b32 with three
// VGPR sources, v_bitop3_b32 with an SGPR source, each in C independent chains;
// and the lane exchanges (v_permlane16/32_swap, DPP row_ror:8 forms).
// Reports SIMD cycles per instruction (wall time x clock / instructions per
// SIMD) and per-wave cycles per instruction (s_memtime inside the kernel).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_issue tools/ubench_issue.hip
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

constexpr int kIters = 4096;

template <int OP, int C>
__global__ void __launch_bounds__(256) k_issue(uint32_t* out, uint64_t* clk, uint32_t s) {
    uint32_t v[C], w[C];
#pragma unroll
    for (int i = 0; i < C; ++i) {
        v[i] = threadIdx.x * (i + 3);
        w[i] = threadIdx.x ^ (i * 77);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int i = 0; i < C; ++i) {
                if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(w[i]));
                if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(w[i]), "v"(w[(i + 1) % C]));
                if constexpr (OP == 2) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x78" : "+v"(v[i]) : "v"(w[i]), "s"(s));
                if constexpr (OP == 3) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(v[i]));
                // lane exchanges (chains >= 4: no DPP / permlane read-after-write hazard inside a chain)
                if constexpr (OP == 4) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(v[i]), "+v"(w[i]));
                if constexpr (OP == 5) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(v[i]), "+v"(w[i]));
                if constexpr (OP == 6) asm volatile("v_cndmask_b32_dpp %0, %1, %0, vcc row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(v[i]) : "v"(w[i]));
                if constexpr (OP == 7) asm volatile("v_mov_b32_dpp %0, %1 row_ror:8 row_mask:0xf bank_mask:0xf" : "=v"(v[i]) : "v"(w[(i + 1) % C]));
                if constexpr (OP == 8) asm volatile("v_xor_b32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(v[i]) : "v"(w[i]));
            }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) acc ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) clk[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
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
    auto run = [&](const char* name, auto kern, int chains) -> int {
        for (int wps = 1; wps <= 4; ++wps) {
            const int blocks = cus * wps;  // 256 threads = one wave on each SIMD per block
            hipLaunchKernelGGL(kern, blocks, 256, 0, 0, out, clk, 0x0F0F0F0Fu);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(kern, blocks, 256, 0, 0, out, clk, 0x0F0F0F0Fu);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            CHECK(hipMemcpy(h, clk, size_t(blocks) * 4 * 8, hipMemcpyDeviceToHost));
            double cyc = 0;
            for (int i = 0; i < blocks * 4; ++i) cyc += double(h[i]);
            cyc /= blocks * 4;
            const double instr = double(kIters) * 8 * chains;  // per wave
            printf("%-34s chains=%d waves/SIMD=%d: %6.2f wave-cycles/instr, %5.2f SIMD-cycles/instr (wall, 2.3 GHz)\n",
                   name, chains, wps, cyc / instr, ms * 1e-3 * 2.3e9 / (instr * wps));
        }
        return 0;
    };
#define R(name, OP, C) if (run(name, k_issue<OP, C>, C)) return 1;
    R("v_xor_b32", 0, 1) R("v_xor_b32", 0, 2) R("v_xor_b32", 0, 4) R("v_xor_b32", 0, 8)
    R("v_bitop3_b32 (3 VGPR)", 1, 1) R("v_bitop3_b32 (3 VGPR)", 1, 2) R("v_bitop3_b32 (3 VGPR)", 1, 4) R("v_bitop3_b32 (3 VGPR)", 1, 8)
    R("v_bitop3_b32 (2 VGPR + SGPR)", 2, 1) R("v_bitop3_b32 (2 VGPR + SGPR)", 2, 4) R("v_bitop3_b32 (2 VGPR + SGPR)", 2, 8)
    R("v_lshlrev_b32", 3, 1) R("v_lshlrev_b32", 3, 4) R("v_lshlrev_b32", 3, 8)
    R("v_permlane32_swap_b32", 4, 4) R("v_permlane32_swap_b32", 4, 8)
    R("v_permlane16_swap_b32", 5, 4) R("v_permlane16_swap_b32", 5, 8)
    R("v_cndmask_b32_dpp row_ror:8", 6, 4) R("v_cndmask_b32_dpp row_ror:8", 6, 8)
    R("v_mov_b32_dpp row_ror:8", 7, 4) R("v_mov_b32_dpp row_ror:8", 7, 8)
    R("v_xor_b32_dpp row_ror:8", 8, 4) R("v_xor_b32_dpp row_ror:8", 8, 8)
    return 0;
}
