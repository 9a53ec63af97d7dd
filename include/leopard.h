/*
 * leopard.h -- drop-in C ABI of the MI355X-native Leopard-RS engine.
 *
 * Every declaration below keeps the exact name, argument list, argument
 * meaning, return codes and version macro of the reference interface
 * (catid/leopard v2, /root/reference/leopard.h), so existing callers relink
 * against libleopard_amd.so unchanged:
 *
 *   leo_init_ / leo_init()   <- reference leopard.h:105-106   (leopard.cpp:49-69)
 *   LeopardResult            <- reference leopard.h:113-124
 *   leo_result_string        <- reference leopard.h:127       (leopard.cpp:74-88)
 *   leo_encode_work_count    <- reference leopard.h:143-145   (leopard.cpp:94-103)
 *   leo_encode               <- reference leopard.h:180-186   (leopard.cpp:123-197)
 *   leo_decode_work_count    <- reference leopard.h:202-204   (leopard.cpp:203-212)
 *   leo_decode               <- reference leopard.h:227-234   (leopard.cpp:233-344)
 *
 * Buffers may be host memory (the reference's contract: the call stages them
 * through the GPU and returns when results are back in host memory) or HIP
 * device memory (detected from the first piece pointer; all pieces of one call
 * must be of the same kind).  See leopard_amd.h for stream/async control.
 */
#ifndef LEOPARD_AMD_LEOPARD_H
#define LEOPARD_AMD_LEOPARD_H

#define LEO_VERSION 2

#if defined(_WIN32)
#define LEO_EXPORT __declspec(dllexport)
#else
#define LEO_EXPORT __attribute__((visibility("default")))
#endif

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One-time initialisation: builds the GF(2^8)/GF(2^16) tables and checks that
 * a gfx950 device is present.  0 on success; Leopard_InvalidInput for a
 * version mismatch; Leopard_Platform when no supported GPU is visible. */
LEO_EXPORT int leo_init_(int version);
#define leo_init() leo_init_(LEO_VERSION)

typedef enum LeopardResultT {
    Leopard_Success = 0,
    Leopard_NeedMoreData = -1,   /* fewer surviving pieces than lost originals */
    Leopard_TooMuchData = -2,    /* NextPow2(NextPow2(R) + K) > 65536 */
    Leopard_InvalidSize = -3,    /* buffer_bytes zero or not a multiple of 64 */
    Leopard_InvalidCounts = -4,  /* R == 0, R > K, or wrong work_count */
    Leopard_InvalidInput = -5,   /* null pointer array */
    Leopard_Platform = -6,       /* no supported GPU / HIP failure */
    Leopard_CallInitialize = -7, /* leo_init() not called */
} LeopardResult;

LEO_EXPORT const char* leo_result_string(LeopardResult result);

/* Number of work_data buffers leo_encode() needs: R if K == 1, 1 if R == 1,
 * else 2 * NextPow2(R).  No validation (as the reference). */
LEO_EXPORT unsigned leo_encode_work_count(unsigned original_count, unsigned recovery_count);

/* Recovery pieces -> work_data[0 .. recovery_count).  buffer_bytes is a
 * multiple of 64; recovery_count <= original_count. */
LEO_EXPORT LeopardResult leo_encode(
    uint64_t buffer_bytes,
    unsigned original_count,
    unsigned recovery_count,
    unsigned work_count,
    const void* const* const original_data,
    void** work_data);

/* Number of work_data buffers leo_decode() needs: K if K == 1 or R == 1, else
 * NextPow2(NextPow2(R) + K). */
LEO_EXPORT unsigned leo_decode_work_count(unsigned original_count, unsigned recovery_count);

/* Lost pieces are NULL in original_data / recovery_data.  Each lost original i
 * is rebuilt into work_data[i]; with no loss, all originals are copied to
 * work_data[0 .. original_count). */
LEO_EXPORT LeopardResult leo_decode(
    uint64_t buffer_bytes,
    unsigned original_count,
    unsigned recovery_count,
    unsigned work_count,
    const void* const* const original_data,
    const void* const* const recovery_data,
    void** work_data);

#ifdef __cplusplus
}
#endif

#endif /* LEOPARD_AMD_LEOPARD_H */
