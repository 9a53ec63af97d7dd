/*
 * leopard_amd.h -- MI355X-specific extensions of the Leopard C ABI.
 *
 * None of these is needed for drop-in use (include/leopard.h is the contract);
 * they let a GPU-resident caller avoid the synchronous host-memory semantics of
 * the reference (leopard.h:180-234 return only when results are written).
 */
#ifndef LEOPARD_AMD_EXT_H
#define LEOPARD_AMD_EXT_H

#include "leopard.h"

#ifdef __cplusplus
extern "C" {
#endif

/* HIP stream used by the calling thread's leo_encode/leo_decode on device
 * memory (a hipStream_t passed as void*; NULL = the legacy default stream).
 * Per thread. */
LEO_EXPORT void leo_amd_set_stream(void* hip_stream);

/* Scratch: the library keeps per (calling thread, device, stream) scratch --
 * a device arena, pinned staging, and for host-memory calls a pinned ring with
 * two streams -- and keeps at most 8 of them per thread (least recently used
 * freed first).  A thread's scratch is freed when the thread exits.  This call
 * frees the calling thread's scratch for `hip_stream` on every device, after
 * the work this library queued on that stream has finished; call it before
 * destroying a stream used with leo_amd_set_stream.  (void*)-1 frees the
 * calling thread's scratch of every stream. */
LEO_EXPORT void leo_amd_release_stream(void* hip_stream);

/* 1: device-resident calls return after enqueueing work on the stream (the
 * caller orders later reads on that stream).  0 (default): every call
 * synchronises, like the reference.  Host-memory calls are always synchronous.
 * Per thread. */
LEO_EXPORT void leo_amd_set_async(int async_enable);

/* Device ordinal the calling thread's calls run on (default: the current HIP
 * device at call time).  -1 restores the default.  Per thread. */
LEO_EXPORT void leo_amd_set_device(int device);

/* Host-memory calls of the calling thread split their columns into `ranges`
 * 64-byte-aligned ranges, range i coded on device i % device_count by its own
 * worker thread over that device's PCIe link; the call returns when all are
 * done.  -1 = one range per device; 0 = the LEO_AMD_FANOUT environment value
 * (default 1, no split).  At most one range per 4 KiB of columns.  Device
 * pointers are not affected.  Per thread. */
LEO_EXPORT void leo_amd_set_fanout(int ranges);

/* Encode/decode a column range of every piece: identical to leo_encode /
 * leo_decode over bytes [byte_offset, byte_offset + slice_bytes) of each
 * piece (both multiples of 64).  This is how independent GPUs shard one object
 * by 64-byte column blocks without any collective (each GPU owns a slice). */
LEO_EXPORT LeopardResult leo_amd_encode_slice(
    uint64_t buffer_bytes, uint64_t byte_offset, uint64_t slice_bytes,
    unsigned original_count, unsigned recovery_count, unsigned work_count,
    const void* const* const original_data, void** work_data);

LEO_EXPORT LeopardResult leo_amd_decode_slice(
    uint64_t buffer_bytes, uint64_t byte_offset, uint64_t slice_bytes,
    unsigned original_count, unsigned recovery_count, unsigned work_count,
    const void* const* const original_data, const void* const* const recovery_data,
    void** work_data);

/* Batches: object_count independent objects of one shape (same buffer_bytes,
 * counts and work_count), each with exactly the semantics of one leo_encode /
 * leo_decode call; original_data[o], recovery_data[o], work_data[o] are object
 * o's pointer arrays.  Every object is validated first: the first failing
 * object's result is returned and nothing runs.  Device-resident GF(2^8)
 * objects (n <= 256) on one device are coded by ONE kernel launch over every
 * object's columns -- a single 64 KiB-piece object gives each CU one
 * workgroup, a batch fills the GPU; other batches run object by object.
 * Decoding objects may have different erasure patterns. */
LEO_EXPORT LeopardResult leo_amd_encode_batch(
    unsigned object_count, uint64_t buffer_bytes, unsigned original_count, unsigned recovery_count,
    unsigned work_count, const void* const* const* original_data, void** const* work_data);

LEO_EXPORT LeopardResult leo_amd_decode_batch(
    unsigned object_count, uint64_t buffer_bytes, unsigned original_count, unsigned recovery_count,
    unsigned work_count, const void* const* const* original_data, const void* const* const* recovery_data,
    void** const* work_data);

/* Caller-registered host memory: pins [ptr, ptr + bytes) and maps it for
 * every device.  leo_encode / leo_decode calls whose host pieces all lie in
 * registered ranges run the kernels on them in place (reads and writes over
 * PCIe, no staging copies); other host pieces go through the pinned staging
 * pipeline.  The range must stay allocated until leo_amd_unregister_host(ptr)
 * (the contract of hipHostRegister and RDMA memory registration).
 * Returns Leopard_Platform when the runtime refuses the registration. */
LEO_EXPORT LeopardResult leo_amd_register_host(void* ptr, uint64_t bytes);
LEO_EXPORT LeopardResult leo_amd_unregister_host(void* ptr);

/* Number of HIP devices usable by the library (0 when none / not gfx950). */
LEO_EXPORT int leo_amd_device_count(void);

/* Host-side tables, for conformance tests (no GPU needed).  field: 8 or 16.
 * which: 0 = log (Cantor basis), 1 = exp, 2 = FFT skew (as logs), 3 = LogWalsh.
 * Copies up to `capacity` uint16 entries into out; returns the table length,
 * or a negative LeopardResult. */
LEO_EXPORT int leo_amd_table(int field, int which, uint16_t* out, unsigned capacity);

/* Human-readable description of the last error on the calling thread. */
LEO_EXPORT const char* leo_amd_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* LEOPARD_AMD_EXT_H */
