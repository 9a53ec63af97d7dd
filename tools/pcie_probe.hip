// Host-link bandwidth probe (performance experiment only): DMA copies and
// kernels reading / writing pinned host memory in place, alone and together.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/pcie_probe tools/pcie_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

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
    return 0;
}
