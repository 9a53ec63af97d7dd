// Throughput of single VALU instruction kinds on gfx950 (performance experiment
// only): SIMD cycles per wave64 instruction, 8 independent chains per lane, at
// 4 waves per SIMD.  Decides how to price v_perm_b32 against plain VOP2 ops in
// the GF multiply.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_isa2 tools/ubench_isa2.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ unsigned long long g_clk[2];

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, int iters, uint32_t s) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t v[8], w[8];
    for (int i = 0; i < 8; ++i) { v[i] = threadIdx.x * 2654435761u + i; w[i] = v[i] * 3u + 0x07060504u; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (OP == 0) v[i] = __builtin_amdgcn_perm(w[i], v[i], w[(i + 1) & 7] & 0x07070707u ^ 0x07070707u);
                if constexpr (OP == 1) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(v[i]) : "v"(w[i]), "v"(w[(i + 3) & 7]));
                if constexpr (OP == 2) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(w[i]));
                if constexpr (OP == 3) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(v[i]) : "v"(w[i]), "v"(w[(i + 3) & 7]));
                if constexpr (OP == 4) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v[i]));
                if constexpr (OP == 5) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(v[i]) : "s"(s), "v"(w[(i + 3) & 7]));
                if constexpr (OP == 6) asm volatile("v_and_or_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(w[i]), "v"(w[(i + 3) & 7]));
                if constexpr (OP == 7) asm volatile("v_bfe_u32 %0, %0, 3, 3" : "+v"(v[i]));
                if constexpr (OP == 8) asm volatile("v_lshl_or_b32 %0, %1, 3, %0" : "+v"(v[i]) : "v"(w[i]));
                if constexpr (OP == 9) asm volatile("v_pk_add_u16 %0, %1, %0" : "+v"(v[i]) : "v"(w[i]));
                if constexpr (OP == 10) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(w[i]));
                if constexpr (OP == 11) {  // one 64-bit shift of a register pair (the pair counts as one instruction)
                    uint64_t p = (uint64_t(w[i]) << 32) | v[i];
                    asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(p));
                    v[i] = uint32_t(p);
                    w[i] = uint32_t(p >> 32);
                }
                if constexpr (OP == 12) asm volatile("v_alignbit_b32 %0, %0, %1, 3" : "+v"(v[i]) : "v"(w[i]));
            }
        }
    }
    uint32_t acc = 0;
    for (int i = 0; i < 8; ++i) acc ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - c0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int OP>
int run(uint32_t* out, const char* name) {
    const int iters = 4000, wps = 4;
    const int blocks = 256 * wps;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 10, 5u);
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double cycles = ms * 1e-3 * 2.4e9;
    const double instr_per_simd = double(iters) * 16 * 8 * wps;
    unsigned long long clk[2];
    CHECK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk)));
    const double ghz = double(clk[0]) / (double(clk[1]) / 100e6) / 1e9;  // s_memrealtime: 100 MHz
    printf("%-28s %.2f SIMD cycles per wave64 instruction (2.4 GHz basis); in-kernel clock %.2f GHz -> %.2f cycles\n",
           name, cycles / instr_per_simd, ghz, cycles / instr_per_simd * ghz / 2.4);
    return 0;
}

int main() {
    uint32_t* out;
    CHECK(hipMalloc(&out, 256 * 8 * 256 * 4));
    run<2>(out, "v_xor_b32");
    run<4>(out, "v_lshrrev_b32");
    run<1>(out, "v_perm_b32 (vgpr, vgpr)");
    run<5>(out, "v_perm_b32 (sgpr, vgpr)");
    run<3>(out, "v_bitop3_b32");
    run<6>(out, "v_and_or_b32");
    run<7>(out, "v_bfe_u32");
    run<8>(out, "v_lshl_or_b32");
    run<9>(out, "v_pk_add_u16");
    run<10>(out, "v_cndmask_b32");
    run<0>(out, "perm+and+xor (compiled)");
    run<11>(out, "v_lshrrev_b64");
    run<12>(out, "v_alignbit_b32");
    return 0;
}
