// GPU-side dispatch cost of back-to-back launches on one stream (performance
// experiment only): empty kernels with the FF8 single-call shape (256 x 1024
// threads), varying kernel-argument size, dynamic LDS and block size.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/ubench_launch tools/ubench_launch.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Small { unsigned long long p; };
struct Big { unsigned long long p[500]; };  // ~4 KB
struct Mid { unsigned long long p[270]; };  // ~2.1 KB, like Ff8EncArgs

__global__ void k_small(Small a) { if (a.p == 1234567) ((int*)a.p)[threadIdx.x] = 0; }
__global__ void k_mid(Mid a) { if (a.p[0] == 1234567) ((int*)a.p[0])[threadIdx.x] = 0; }
__global__ void k_big(Big a) { if (a.p[0] == 1234567) ((int*)a.p[0])[threadIdx.x] = 0; }
__global__ void k_lds(Small a) {
    extern __shared__ int lds[];
    if (a.p == 1234567) { lds[threadIdx.x] = 1; __syncthreads(); ((int*)a.p)[threadIdx.x] = lds[threadIdx.x ^ 1]; }
}
__global__ void spin(long long cycles) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    Small sm{0};
    Big bg{};
    Mid md{};
    CHECK(hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 10; ++i) launch();
        CHECK(hipStreamSynchronize(s));
        hipLaunchKernelGGL(spin, dim3(1), dim3(1), 0, s, 20000000LL);  // host queues everything behind it
        CHECK(hipEventRecord(a, s));
        const int n = 200;
        for (int i = 0; i < n; ++i) launch();
        CHECK(hipEventRecord(b, s));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("%-52s %7.2f us/launch\n", name, ms * 1e3 / n);
        return 0;
    };
    run("empty 256 x 1024, 8 B args", [&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, s, sm); });
    run("empty 256 x 1024, 2.1 KB args", [&] { hipLaunchKernelGGL(k_mid, dim3(256), dim3(1024), 0, s, md); });
    run("empty 256 x 1024, 4 KB args", [&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(1024), 0, s, bg); });
    run("empty 256 x 512, 4 KB args", [&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, s, bg); });
    run("empty 256 x 256, 8 B args", [&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, sm); });
    run("empty 1 x 64, 8 B args", [&] { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, sm); });
    run("empty 256 x 1024, 8 B args, 40 KB LDS", [&] { hipLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 40 * 1024, s, sm); });
    run("empty 256 x 1024, 8 B args, 100 KB LDS", [&] { hipLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 100 * 1024, s, sm); });
    run("empty 4096 x 512, 8 B args", [&] { hipLaunchKernelGGL(k_small, dim3(4096), dim3(512), 0, s, sm); });
    return 0;
}
