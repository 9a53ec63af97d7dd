// Memory-pattern microbenchmark (performance experiment only, not part of the
// library): copy 128 pieces x B bytes (slab) with the access shapes a
// Reed-Solomon tile kernel could use, and report GB/s of (read + write) bytes.
//   wide   : wave = 16 pieces x 64 dword columns (256-B segments per piece)
//   narrow8: wave = 128 pieces x 8 columns  (lane = 3 column bits + 3 piece bits, 32-B segments)
//   narrow16: wave = 128 pieces x 16 columns (lane = 4 column bits + 2 piece bits, 64-B segments)
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_mem tools/ubench_mem.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef __attribute__((address_space(1))) uint32_t gu32;

// grid: (B/256 column strips) x (128/16 piece blocks); block = 64 threads
__global__ void __launch_bounds__(256) k_wide(const uint32_t* in, uint32_t* out, uint64_t stride_dw) {
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t col = uint64_t(blockIdx.x) * 64 + lane;
    const unsigned p0 = (blockIdx.y * 4 + w) * 16;
    uint32_t v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = ((const gu32*)in)[(p0 + r) * stride_dw + col];
#pragma unroll
    for (int r = 0; r < 16; ++r) ((gu32*)out)[(p0 + r) * stride_dw + col] = v[r] ^ 0x5A5A5A5Au;
}

// one wave = 128 pieces x 8 columns; 4 waves per block = 32 adjacent columns
__global__ void __launch_bounds__(256) k_narrow8(const uint32_t* in, uint32_t* out, uint64_t stride_dw) {
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t col = (uint64_t(blockIdx.x) * 4 + w) * 8 + (lane & 7);
    const unsigned pl = lane >> 3;
    uint32_t v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = ((const gu32*)in)[(r * 8 + pl) * stride_dw + col];
#pragma unroll
    for (int r = 0; r < 16; ++r) ((gu32*)out)[(r * 8 + pl) * stride_dw + col] = v[r] ^ 0x5A5A5A5Au;
}

// one wave = 128 pieces x 16 columns; 2 waves per block = 32 adjacent columns
__global__ void __launch_bounds__(128) k_narrow16(const uint32_t* in, uint32_t* out, uint64_t stride_dw) {
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t col = (uint64_t(blockIdx.x) * 2 + w) * 16 + (lane & 15);
    const unsigned pl = lane >> 4;
    uint32_t v[32];
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = ((const gu32*)in)[(r * 4 + pl) * stride_dw + col];
#pragma unroll
    for (int r = 0; r < 32; ++r) ((gu32*)out)[(r * 4 + pl) * stride_dw + col] = v[r] ^ 0x5A5A5A5Au;
}

int main() {
    for (uint64_t B : {65536ull, 1048576ull}) {
        const int sets = B == 65536 ? 16 : 2;
        const uint64_t slab = 128 * B;
        uint8_t *in, *out;
        CHECK(hipMalloc(&in, slab * sets));
        CHECK(hipMalloc(&out, slab * sets));
        CHECK(hipMemset(in, 1, slab * sets));
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        const uint64_t sdw = B / 4;
        for (int kind = 0; kind < 3; ++kind) {
            auto launch = [&](int s) {
                const uint32_t* i = (const uint32_t*)(in + s * slab);
                uint32_t* o = (uint32_t*)(out + s * slab);
                if (kind == 0) hipLaunchKernelGGL(k_wide, dim3(B / 256, 2), dim3(256), 0, 0, i, o, sdw);
                else if (kind == 1) hipLaunchKernelGGL(k_narrow8, dim3(B / 128), dim3(256), 0, 0, i, o, sdw);
                else hipLaunchKernelGGL(k_narrow16, dim3(B / 128), dim3(128), 0, 0, i, o, sdw);
            };
            for (int it = 0; it < 200; ++it) launch(it % sets);
            CHECK(hipDeviceSynchronize());
            const int n = 200;
            CHECK(hipEventRecord(e0));
            for (int it = 0; it < n; ++it) launch(it % sets);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / n;
            printf("B=%7llu %-9s %8.2f us/call  %7.1f GB/s (read+write)\n", (unsigned long long)B,
                   kind == 0 ? "wide" : kind == 1 ? "narrow8" : "narrow16", us, 2.0 * slab / us / 1e3);
        }
        CHECK(hipFree(in));
        CHECK(hipFree(out));
    }
    return 0;
}
