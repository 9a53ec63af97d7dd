// Host-link bandwidth probe (performance experiment only): DMA copies and
// kernels reading / writing pinned host memory in place, alone and together.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/pcie_probe tools/pcie_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void copy_k(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        dst[i] = src[i];
}

int main() {
    const size_t bytes = 64ull << 20, n = bytes / 16;
    void *h_in, *h_out, *d_a, *d_b;
    CHECK(hipHostMalloc(&h_in, bytes, hipHostMallocMapped));
    CHECK(hipHostMalloc(&h_out, bytes, hipHostMallocMapped));
    CHECK(hipMalloc(&d_a, bytes));
    CHECK(hipMalloc(&d_b, bytes));
    hipStream_t s1, s2;
    CHECK(hipStreamCreate(&s1));
    CHECK(hipStreamCreate(&s2));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](const char* name, double moved, auto fn) {
        fn();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a, 0));
        for (int i = 0; i < 5; ++i) fn();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("%-44s %7.1f GB/s\n", name, moved * 5 / (ms * 1e-3) / 1e9);
        return 0;
    };
    void *dh_in, *dh_out;
    CHECK(hipHostGetDevicePointer(&dh_in, h_in, 0));
    CHECK(hipHostGetDevicePointer(&dh_out, h_out, 0));
    timeit("DMA H2D", bytes, [&] { (void)hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s1); });
    timeit("DMA D2H", bytes, [&] { (void)hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s1); });
    timeit("DMA H2D + D2H concurrently (sum)", 2.0 * bytes, [&] {
        (void)hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s1);
        (void)hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s2);
    });
    for (int blocks : {256, 1024, 4096}) {
        char name[64];
        snprintf(name, sizeof(name), "kernel reads host (%d blocks)", blocks);
        timeit(name, bytes, [&] { hipLaunchKernelGGL(copy_k, dim3(blocks), dim3(256), 0, s1, (const uint4*)dh_in, (uint4*)d_a, n); });
        snprintf(name, sizeof(name), "kernel writes host (%d blocks)", blocks);
        timeit(name, bytes, [&] { hipLaunchKernelGGL(copy_k, dim3(blocks), dim3(256), 0, s1, (const uint4*)d_b, (uint4*)dh_out, n); });
        snprintf(name, sizeof(name), "kernel host->host (%d blocks, sum)", blocks);
        timeit(name, 2.0 * bytes, [&] { hipLaunchKernelGGL(copy_k, dim3(blocks), dim3(256), 0, s1, (const uint4*)dh_in, (uint4*)dh_out, n); });
    }
    timeit("kernel reads host + DMA D2H concurrently (sum)", 2.0 * bytes, [&] {
        hipLaunchKernelGGL(copy_k, dim3(1024), dim3(256), 0, s1, (const uint4*)dh_in, (uint4*)d_a, n);
        (void)hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s2);
    });
    // 2-D copies of column slices (128 pieces x 16 KiB of 64 KiB rows) from
    // hipHostRegister'ed malloc memory: the staging-free host pipeline's copies.
    {
        const size_t rows = 128, pitch = 65536, width = 16384;
        void* hreg = malloc(rows * pitch);
        void* hreg2 = malloc(rows * pitch);
        memset(hreg, 1, rows * pitch);
        memset(hreg2, 2, rows * pitch);
        CHECK(hipHostRegister(hreg, rows * pitch, hipHostRegisterMapped));
        CHECK(hipHostRegister(hreg2, rows * pitch, hipHostRegisterMapped));
        void *dreg, *dreg2;
        CHECK(hipHostGetDevicePointer(&dreg, hreg, 0));
        CHECK(hipHostGetDevicePointer(&dreg2, hreg2, 0));
        const size_t n8 = rows * pitch / 16;
        timeit("kernel reads registered malloc 8 MiB", double(rows * pitch), [&] {
            hipLaunchKernelGGL(copy_k, dim3(512), dim3(256), 0, s1, (const uint4*)dreg, (uint4*)d_a, n8); });
        timeit("kernel writes registered malloc 8 MiB", double(rows * pitch), [&] {
            hipLaunchKernelGGL(copy_k, dim3(512), dim3(256), 0, s1, (const uint4*)d_b, (uint4*)dreg2, n8); });
        timeit("kernel read + write registered, 2 streams (sum)", 2.0 * rows * pitch, [&] {
            hipLaunchKernelGGL(copy_k, dim3(512), dim3(256), 0, s1, (const uint4*)dreg, (uint4*)d_a, n8);
            hipLaunchKernelGGL(copy_k, dim3(512), dim3(256), 0, s2, (const uint4*)d_b, (uint4*)dreg2, n8); });
        timeit("2D H2D 128 x 16 KiB (registered)", double(rows * width), [&] {
            (void)hipMemcpy2DAsync(d_a, width, hreg, pitch, width, rows, hipMemcpyHostToDevice, s1); });
        timeit("2D D2H 128 x 16 KiB (registered)", double(rows * width), [&] {
            (void)hipMemcpy2DAsync(hreg2, pitch, d_b, width, width, rows, hipMemcpyDeviceToHost, s1); });
        timeit("2D H2D + D2H concurrently (sum)", 2.0 * rows * width, [&] {
            (void)hipMemcpy2DAsync(d_a, width, hreg, pitch, width, rows, hipMemcpyHostToDevice, s1);
            (void)hipMemcpy2DAsync(hreg2, pitch, d_b, width, width, rows, hipMemcpyDeviceToHost, s2); });
        timeit("2D H2D 128 x 64 KiB whole rows (registered)", double(rows * pitch), [&] {
            (void)hipMemcpy2DAsync(d_a, pitch, hreg, pitch, pitch, rows, hipMemcpyHostToDevice, s1); });
        timeit("linear H2D 8 MiB (registered)", double(rows * pitch), [&] {
            (void)hipMemcpyAsync(d_a, hreg, rows * pitch, hipMemcpyHostToDevice, s1); });
        timeit("per-row H2D 128 x 16 KiB (registered)", double(rows * width), [&] {
            for (size_t r = 0; r < rows; ++r)
                (void)hipMemcpyAsync((char*)d_a + r * width, (char*)hreg + r * pitch, width, hipMemcpyHostToDevice, s1); });
    }
    return 0;
}
