// Host copy rates on the GPU box (diagnostics for the pageable host path,
// DESIGN.md section 4): gather / scatter between pageable buffers and pinned
// (hipHostMalloc) staging memory with 1..16 threads, memcpy vs non-temporal
// stores, plus SDMA H2D / D2H from pinned and pageable memory.
// build: hipcc --offload-arch=gfx950 -O3 -mavx2 -o tools/hostcopy_probe tools/hostcopy_probe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void copy_nt(uint8_t* dst, const uint8_t* src, size_t n) {
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i*)(src + i));
        __m256i b = _mm256_loadu_si256((const __m256i*)(src + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i*)(src + i + 64));
        __m256i d = _mm256_loadu_si256((const __m256i*)(src + i + 96));
        _mm256_stream_si256((__m256i*)(dst + i), a);
        _mm256_stream_si256((__m256i*)(dst + i + 32), b);
        _mm256_stream_si256((__m256i*)(dst + i + 64), c);
        _mm256_stream_si256((__m256i*)(dst + i + 96), d);
    }
    std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

// pieces: `np` pieces of `len` bytes at `src` (stride len) -> dst, split over t threads
static double run(int t, bool nt, uint8_t* dst, const uint8_t* src, size_t total, int reps) {
    const size_t part = 1 << 20;
    const size_t nparts = (total + part - 1) / part;
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
        std::atomic<size_t> next{0};
        const double t0 = now();
        std::vector<std::thread> th;
        auto work = [&] {
            for (size_t i = next.fetch_add(1); i < nparts; i = next.fetch_add(1)) {
                const size_t o = i * part, n = std::min(part, total - o);
                if (nt) copy_nt(dst + o, src + o, n);
                else std::memcpy(dst + o, src + o, n);
            }
        };
        for (int k = 1; k < t; ++k) th.emplace_back(work);
        work();
        for (auto& x : th) x.join();
        best = std::min(best, now() - t0);
    }
    return total / best / 1e9;
}

int main() {
    const size_t total = size_t(128) << 16;  // 128 pieces x 64 KiB = one encode's inputs
    uint8_t *pin, *dev;
    if (hipHostMalloc((void**)&pin, total, hipHostMallocDefault) != hipSuccess) return 1;
    if (hipMalloc((void**)&dev, total) != hipSuccess) return 1;
    uint8_t* a = (uint8_t*)aligned_alloc(4096, total);
    uint8_t* b = (uint8_t*)aligned_alloc(4096, total);
    std::memset(a, 1, total);
    std::memset(b, 2, total);
    std::memset(pin, 3, total);
    std::printf("8 MiB copies, GB/s (best of 20)\n");
    for (int t : {1, 2, 4, 8, 12, 16}) {
        std::printf("threads %2d: pageable->pageable memcpy %6.1f nt %6.1f | pageable->pinned memcpy %6.1f nt %6.1f | "
                    "pinned->pageable memcpy %6.1f nt %6.1f\n",
                    t, run(t, false, b, a, total, 20), run(t, true, b, a, total, 20), run(t, false, pin, a, total, 20),
                    run(t, true, pin, a, total, 20), run(t, false, a, pin, total, 20), run(t, true, a, pin, total, 20));
    }
    hipStream_t s;
    hipStreamCreate(&s);
    auto sdma = [&](void* d, const void* src, hipMemcpyKind k) {
        double best = 1e30;
        for (int r = 0; r < 20; ++r) {
            hipStreamSynchronize(s);
            const double t0 = now();
            hipMemcpyAsync(d, src, total, k, s);
            hipStreamSynchronize(s);
            best = std::min(best, now() - t0);
        }
        return total / best / 1e9;
    };
    std::printf("SDMA 8 MiB: H2D pinned %.1f, H2D pageable %.1f, D2H pinned %.1f, D2H pageable %.1f GB/s\n",
                sdma(dev, pin, hipMemcpyHostToDevice), sdma(dev, a, hipMemcpyHostToDevice),
                sdma(pin, dev, hipMemcpyDeviceToHost), sdma(a, dev, hipMemcpyDeviceToHost));
    // hipHostRegister cost of one 8 MiB pageable buffer (register + unregister)
    double best = 1e30;
    for (int r = 0; r < 10; ++r) {
        const double t0 = now();
        if (hipHostRegister(a, total, hipHostRegisterMapped) != hipSuccess) return 2;
        const double t1 = now();
        hipHostUnregister(a);
        best = std::min(best, t1 - t0);
    }
    std::printf("hipHostRegister 8 MiB: %.1f us\n", best * 1e6);
    return 0;
}
