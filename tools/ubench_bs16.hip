// GF(2^16) multiply-add by a wave-uniform RUNTIME constant in bit-sliced form
// on gfx950 (performance experiment only): a lane holds
// 32 elements as 16 bit planes, x ^= M_c * y with M_c the 16 x 16 GF(2) matrix
// of the multiply by c, by four Russians: the 16 XOR combinations of each
// group of 4 input planes (11 XORs a group, in VGPRs), then every output plane
// XORs one combination of each group, picked by the wave-uniform nibble of its
// matrix row (a dynamically indexed VGPR read, v_movrels with the index in M0).
// A second form, the alpha chain (muladd_chain), uses the field structure.
// Against the byte-table form of rs_device.h (FF16::muladd: 12 v_perm_b32 per 4
// elements), same registers-only loop as tools/ubench_ff16.hip.  Reports SIMD
// cycles per 32 elements and checks the bit-sliced map against the host.
//   hipcc --offload-arch=gfx950 -O3 -I leopard_amd/csrc -o tools/bin/ubench_bs16 tools/ubench_bs16.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rs_device.h"

using namespace lamd;

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("%s: %s\n", #x, hipGetErrorString(e));                          \
            return 1;                                                              \
        }                                                                          \
    } while (0)

// x ^= M * y, rows: nib[i] = the 4 nibbles of row i of M (bit j of the row =
// input plane j), wave-uniform (SGPRs)
typedef uint32_t v16u __attribute__((ext_vector_type(16)));
__device__ __forceinline__ void muladd_bs16(uint32_t* x, const uint32_t* y, const uint32_t* rows) {
    v16u T[4];  // vector registers: a uniform index reads them with v_movrels / gpr-index mode
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const uint32_t* p = y + 4 * g;
        v16u t;
        t[0] = 0;
        t[1] = p[0];
        t[2] = p[1];
        t[3] = p[0] ^ p[1];
        t[4] = p[2];
        t[5] = t[1] ^ p[2];
        t[6] = t[2] ^ p[2];
        t[7] = t[3] ^ p[2];
        t[8] = p[3];
        t[9] = t[1] ^ p[3];
        t[10] = t[2] ^ p[3];
        t[11] = t[3] ^ p[3];
        t[12] = t[4] ^ p[3];
        t[13] = t[5] ^ p[3];
        t[14] = t[6] ^ p[3];
        t[15] = t[7] ^ p[3];
        T[g] = t;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t r = __builtin_amdgcn_readfirstlane(rows[i]);
        const uint32_t a = T[0][r & 15u], b = T[1][(r >> 4) & 15u], c = T[2][(r >> 8) & 15u], d = T[3][(r >> 12) & 15u];
        x[i] = __builtin_amdgcn_bitop3_b32(x[i], a, b, 0x96) ^ c ^ d;
    }
}

// The same map by the field structure: c y = XOR over the set bits k of c of
// alpha^k y, alpha^k y by the chain z <- alpha z (a plane rotation and 3 XORs:
// x^16 + x^5 + x^3 + x^2 + 1, the reference's 0x1002D), each set bit one
// wave-uniform branch of 16 XORs.  cbits: the constant's 16 bits (uniform).
__device__ __forceinline__ void muladd_chain(uint32_t* x, const uint32_t* y, uint32_t cbits) {
    uint32_t z[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = y[i];
    const uint32_t c = __builtin_amdgcn_readfirstlane(cbits);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if ((c >> k) & 1u) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] ^= z[i];
        }
        if (k < 15) {
            const uint32_t t = z[15];
#pragma unroll
            for (int i = 15; i > 0; --i) z[i] = z[i - 1];
            z[0] = t;
            z[2] ^= t;
            z[3] ^= t;
            z[5] ^= t;
        }
    }
}

// NS element sets of 2 pieces (x, y: 16 planes each) per lane; the butterfly
// y ^= x; x ^= M y, ITERS times, rotating the sets
template <int NS>
__global__ void __launch_bounds__(256) k_bs16(uint32_t* out, const uint32_t* rows_in, int iters) {
    uint32_t x[NS][2][16];
    for (int s = 0; s < NS; ++s)
        for (int k = 0; k < 2; ++k)
            for (int i = 0; i < 16; ++i) x[s][k][i] = (threadIdx.x + 1) * 2654435761u ^ (s * 977u + k * 131u + i * 40503u);
    uint32_t rows[16];
    for (int i = 0; i < 16; ++i) rows[i] = rows_in[i];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[s][1][i] ^= x[s][0][i];
            muladd_bs16(x[s][0], x[s][1], rows);
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(x[s][0][i]), "+v"(x[s][1][i]));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    uint32_t acc = 0;
    for (int s = 0; s < NS; ++s)
        for (int i = 0; i < 16; ++i) acc ^= x[s][0][i] * (i + 1) ^ x[s][1][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NS>
__global__ void __launch_bounds__(256) k_chain(uint32_t* out, const uint32_t* c_in, int iters) {
    uint32_t x[NS][2][16];
    for (int s = 0; s < NS; ++s)
        for (int k = 0; k < 2; ++k)
            for (int i = 0; i < 16; ++i) x[s][k][i] = (threadIdx.x + 1) * 2654435761u ^ (s * 977u + k * 131u + i * 40503u);
    const uint32_t c = c_in[0];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[s][1][i] ^= x[s][0][i];
            muladd_chain(x[s][0], x[s][1], c + it);  // a different constant every iteration
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(x[s][0][i]), "+v"(x[s][1][i]));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    uint32_t acc = 0;
    for (int s = 0; s < NS; ++s)
        for (int i = 0; i < 16; ++i) acc ^= x[s][0][i] * (i + 1) ^ x[s][1][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// one multiply-add for the check: x = x0 ^ M * y
__global__ void k_check(uint32_t* xo, const uint32_t* xi, const uint32_t* yi, const uint32_t* rows) {
    uint32_t x[16], y[16];
    for (int i = 0; i < 16; ++i) x[i] = xi[i * 64 + threadIdx.x], y[i] = yi[i * 64 + threadIdx.x];
    muladd_bs16(x, y, rows);
    for (int i = 0; i < 16; ++i) xo[i * 64 + threadIdx.x] = x[i];
}

// the byte-table form, as tools/ubench_ff16.hip: 2 dwords (4 elements) per piece
template <int NR>
__global__ void __launch_bounds__(256) k_bytes(uint32_t* out, const uint32_t* tabs, int iters) {
    uint32_t x[NR][2];
    for (int i = 0; i < NR; ++i) {
        x[i][0] = threadIdx.x * 2654435761u + i * 40503u;
        x[i][1] = x[i][0] * 7u + 3u;
    }
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
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    uint32_t acc = 0;
    for (int i = 0; i < NR; ++i) acc ^= x[i][0] ^ x[i][1];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <class F>
double time_ms(F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch(10);
    (void)hipEventRecord(a);
    launch(2000);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t *out, *rows, *tabs, *xi, *yi, *xo;
    CHECK(hipMalloc(&out, 1 << 24));
    CHECK(hipMalloc(&rows, 64));
    CHECK(hipMalloc(&tabs, 4096));
    CHECK(hipMalloc(&xi, 4096));
    CHECK(hipMalloc(&yi, 4096));
    CHECK(hipMalloc(&xo, 4096));
    std::vector<uint32_t> hr(16), ht(1024), hx(1024), hy(1024), ho(1024);
    srand(7);
    for (auto& v : hr) v = uint32_t(rand()) & 0xFFFFu;
    for (auto& v : ht) v = uint32_t(rand()) * 2654435761u;
    for (auto& v : hx) v = uint32_t(rand()) * 2246822519u;
    for (auto& v : hy) v = uint32_t(rand()) * 3266489917u;
    CHECK(hipMemcpy(rows, hr.data(), 64, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(tabs, ht.data(), 4096, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(xi, hx.data(), 4096, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(yi, hy.data(), 4096, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, xo, xi, yi, rows);
    CHECK(hipMemcpy(ho.data(), xo, 4096, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 16; ++i) {
            uint32_t want = hx[i * 64 + l];
            for (int j = 0; j < 16; ++j)
                if ((hr[i] >> j) & 1u) want ^= hy[j * 64 + l];
            bad += want != ho[i * 64 + l];
        }
    printf("bit-sliced map check: %s (%d wrong planes)\n", bad ? "FAIL" : "ok", bad);
    const double ghz = 2.4;
    for (int wps : {1, 2, 4}) {
        const int blocks = 256 * wps;  // 256-thread blocks: one wave per SIMD each, 1024 SIMDs
        const double ms_bs = time_ms([&](int it) { hipLaunchKernelGGL(k_bs16<2>, dim3(blocks), dim3(256), 0, 0, out, rows, it); });
        const double ms_ch = time_ms([&](int it) { hipLaunchKernelGGL(k_chain<2>, dim3(blocks), dim3(256), 0, 0, out, rows, it); });
        const double ms_by = time_ms([&](int it) { hipLaunchKernelGGL(k_bytes<16>, dim3(blocks), dim3(256), 0, 0, out, tabs, it); });
        // cycles per SIMD per 32-element multiply-add (wave-wide): bit-sliced 2 sets per iteration;
        // byte form 8 butterflies of 4 elements = 32 elements per iteration
        const double cyc_bs = ms_bs * 1e-3 * ghz * 1e9 / (2000.0 * 2 * wps);
        const double cyc_by = ms_by * 1e-3 * ghz * 1e9 / (2000.0 * wps);
        const double cyc_ch = ms_ch * 1e-3 * ghz * 1e9 / (2000.0 * 2 * wps);
        printf("waves/SIMD %d: SIMD cycles per 32-element mul-add: four Russians %.1f (%.2fx), alpha chain %.1f (%.2fx), "
               "byte tables %.1f\n", wps, cyc_bs, cyc_by / cyc_bs, cyc_ch, cyc_by / cyc_ch, cyc_by);
    }
    return bad ? 1 : 0;
}
