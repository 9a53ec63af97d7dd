/*
 * A plain C caller of the drop-in ABI, written the way a user of the reference
 * library calls it (reference tests/benchmark.cpp:384-385, 421-428, 472-479):
 * include "leopard.h", leo_init(), leo_encode_work_count / leo_encode on
 * caller-owned host buffers, drop originals, leo_decode, check the rebuilt
 * pieces.  Compiled with gcc against include/leopard.h and linked against
 * libleopard_amd.so or libleopard_amd.a (tests/test_cpu_c_abi.py).
 *
 * usage: leo_c_caller K R B LOSSES
 * prints "init <code>", the validation results, and on a GPU
 * "recovery_fnv <hex>" and "decode ok" (exit 0), or exits non-zero on failure.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "leopard.h"

static uint64_t fnv1a64(const uint8_t* p, size_t n, uint64_t h) {
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001B3ull;
    }
    return h;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s K R B LOSSES\n", argv[0]);
        return 2;
    }
    const unsigned K = (unsigned)atoi(argv[1]), R = (unsigned)atoi(argv[2]), L = (unsigned)atoi(argv[4]);
    const uint64_t B = (uint64_t)atoll(argv[3]);

    /* argument checks come before the initialisation check (leopard.cpp:131-140) */
    const void* one[1] = {0};
    void* wone[1] = {0};
    printf("check invalid_size %d\n", (int)leo_encode(63, 4, 2, 4, one, wone));
    printf("check invalid_counts %d\n", (int)leo_encode(64, 4, 5, 4, one, wone));
    printf("check invalid_input %d\n", (int)leo_encode(64, 4, 2, 4, NULL, wone));
    printf("result_string %s\n", leo_result_string(Leopard_InvalidCounts));

    const int init = leo_init();
    printf("init %d\n", init);
    if (init != Leopard_Success) return init == Leopard_Platform ? 3 : 1; /* 3: no usable GPU */

    const unsigned wc = leo_encode_work_count(K, R), dwc = leo_decode_work_count(K, R);
    uint8_t** orig = calloc(K, sizeof(uint8_t*));
    void** work = calloc(wc, sizeof(void*));
    void** dwork = calloc(dwc, sizeof(void*));
    const void** dorig = calloc(K, sizeof(void*));
    const void** drec = calloc(R, sizeof(void*));
    for (unsigned i = 0; i < K; ++i) {
        orig[i] = malloc(B);
        for (uint64_t j = 0; j < B; ++j) orig[i][j] = (uint8_t)(i * 131u + j * 7u + 3u + (j >> 8) * 29u);
    }
    for (unsigned i = 0; i < wc; ++i) work[i] = malloc(B);
    for (unsigned i = 0; i < dwc; ++i) dwork[i] = malloc(B);

    LeopardResult r = leo_encode(B, K, R, wc, (const void* const*)orig, work);
    printf("encode %d\n", (int)r);
    if (r != Leopard_Success) return 1;
    uint64_t h = 0xCBF29CE484222325ull;
    for (unsigned i = 0; i < R; ++i) h = fnv1a64((const uint8_t*)work[i], B, h);
    printf("recovery_fnv %016llx\n", (unsigned long long)h);

    /* lose originals 0, 2, 4, ... (L of them); keep the first L recovery pieces */
    for (unsigned i = 0; i < K; ++i) dorig[i] = orig[i];
    unsigned lost = 0;
    for (unsigned i = 0; i < K && lost < L; i += 2, ++lost) dorig[i] = NULL;
    for (unsigned i = 0; i < R; ++i) drec[i] = i < lost ? work[i] : NULL;
    r = leo_decode(B, K, R, dwc, dorig, drec, dwork);
    printf("decode %d\n", (int)r);
    if (r != Leopard_Success) return 1;
    for (unsigned i = 0; i < K; ++i)
        if (!dorig[i] && memcmp(dwork[i], orig[i], B) != 0) {
            printf("decode mismatch at %u\n", i);
            return 1;
        }
    printf("decode ok\n");
    return 0;
}
