// leopard_amd.cpp -- the drop-in C ABI (include/leopard.h) over the gfx950 kernels.
//
// Replaces the reference's leopard.cpp dispatch (leopard.cpp:49-344): same
// validation order, result codes, work counts and edge paths (K == 1, R == 1,
// no loss), with the codec bodies (ReedSolomonEncode/Decode) running as HIP
// kernels instead of ff8::/ff16:: SIMD loops.  There is no CPU fallback: with no
// usable GPU leo_init() returns Leopard_Platform and every call fails loudly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <immintrin.h>

#include "../../include/leopard.h"
#include "../../include/leopard_amd.h"
#include "gf_tables.h"
#include "rs_args.h"

namespace lamd {
namespace {

// ------------------------------------------------------------ thread state --

struct ThreadState {
    hipStream_t stream = nullptr;
    bool async = false;
    int device = -1;
    int fanout = 0;               // leo_amd_set_fanout (0 = LEO_AMD_FANOUT, default 1)
    bool fanout_worker = false;   // this thread runs one range of a fanned-out call
    std::string last_error;
};
thread_local ThreadState tls;

void set_error(const char* what, hipError_t e) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    tls.last_error = buf;
}

// A/B switches of the performance experiments (tools/): read from the
// environment only in builds with LAMD_EXPERIMENT_ENV=1.  The shipped library
// (Makefile default) ignores them and always takes the default paths, which
// are the ones the tests cover.
bool experiment_off(const char* name) {
#if LAMD_EXPERIMENT_ENV
    const char* e = std::getenv(name);
    return e && e[0] == '0';
#else
    (void)name;
    return false;
#endif
}

#define HIP_OK(expr, what)                         \
    do {                                           \
        hipError_t e_ = (expr);                    \
        if (e_ != hipSuccess) {                    \
            set_error(what, e_);                   \
            return Leopard_Platform;               \
        }                                          \
    } while (0)

// ----------------------------------------------------- per-device resources --

struct DeviceTables {
    uint32_t* tab8 = nullptr;   // (256 + 1) x 8 dwords
    uint32_t* tab16 = nullptr;  // (65536 + 1) x 24 dwords
    uint32_t* sktab8 = nullptr;   // skew-indexed butterfly tables, 256 x 8 dwords
    uint32_t* sktab16 = nullptr;  // 65536 x 24 dwords
    uint32_t* fused8 = nullptr;  // fused top-layer tables of the FF8 encoder
    uint32_t* fused16 = nullptr;  // fused top-layer table indices of the FF16 encoders
    uint32_t* walsh8 = nullptr;
    uint32_t* walsh16 = nullptr;
    uint32_t* qlog16 = nullptr;  // high part of the small FF16 decoder (gf_tables.h: build_high_q16)
    uint8_t* zeros = nullptr;   // zero page
    hipStream_t svc = nullptr;  // library-owned stream for releasing workspace memory
    // Library-owned stream-ordered memory pool of the workspaces: trimming it
    // (release_device_memory) never touches the application's own cached
    // stream-ordered memory in the device's default pool.
    hipMemPool_t pool = nullptr;
    unsigned cus = 0;  // compute units (grid sizing of persistent kernels and launch-form rules)
    uint32_t* vtab8 = nullptr;  // FF8 multiply tables by element value (entry 0 all zero; matrix path)
    bool ready = false;
};

// Coefficient matrices of the GF(2^8) matrix path (rs_ff8_mat.hip), per device,
// by (kind, K, R, erasure bitmap): the tables of M[i][j] for L outputs x N
// inputs.  Entries are written once, on the stream of the call that first needs
// them (event `ready` after the writes), and never rewritten or freed while the
// process runs: a later call on another stream waits for `ready` on the device
// (or not at all once it has completed), and no call ever reads an entry that
// another call could be changing.  At most kMatCacheBytes of tables a device;
// past that, new patterns take the transform kernels.
struct MatEntry {
    uint32_t* tabs = nullptr;
    unsigned L = 0, N = 0;
    hipEvent_t ready = nullptr;
    hipStream_t stream = nullptr;
    std::atomic<bool> done{false};
};
struct MatCache {
    std::mutex mu;
    std::map<std::vector<uint32_t>, std::unique_ptr<MatEntry>> entries;
    size_t bytes = 0;
};
constexpr size_t kMatCacheBytes = 64ull << 20;

// Bytes of freed stream-ordered memory the library's pool keeps per device.
constexpr uint64_t kPoolKeepBytes = 256ull << 20;

std::mutex g_mu;
bool g_initialized = false;
int g_device_count = 0;
std::vector<DeviceTables> g_dev;
std::vector<std::unique_ptr<MatCache>> g_mat;  // per device
std::vector<uint32_t> g_h_vtab8;  // FF8 tables by element value (matrix path)
std::vector<uint32_t> g_h_tab8, g_h_tab16, g_h_sktab8, g_h_sktab16, g_h_fused8, g_h_fused16, g_h_walsh8, g_h_walsh16,
    g_h_qlog16;
bool g_q16_ok = false;  // the high part is an XOR-convolution (always; checked at init)

template <class T>
hipError_t upload(T** dst, const std::vector<T>& src) {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(dst), src.size() * sizeof(T));
    if (e != hipSuccess) return e;
    return hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
}

LeopardResult ensure_device(int dev, DeviceTables** out) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (dev < 0 || dev >= int(g_dev.size())) {
        tls.last_error = "device ordinal out of range";
        return Leopard_Platform;
    }
    DeviceTables& d = g_dev[dev];
    if (!d.ready) {
        HIP_OK(upload(&d.tab8, g_h_tab8), "upload FF8 tables");
        HIP_OK(upload(&d.vtab8, g_h_vtab8), "upload FF8 value tables");
        HIP_OK(upload(&d.tab16, g_h_tab16), "upload FF16 tables");
        HIP_OK(upload(&d.sktab8, g_h_sktab8), "upload FF8 skew tables");
        HIP_OK(upload(&d.sktab16, g_h_sktab16), "upload FF16 skew tables");
        HIP_OK(upload(&d.fused8, g_h_fused8), "upload FF8 fused tables");
        HIP_OK(upload(&d.fused16, g_h_fused16), "upload FF16 fused indices");
        HIP_OK(upload(&d.walsh8, g_h_walsh8), "upload FF8 LogWalsh");
        HIP_OK(upload(&d.walsh16, g_h_walsh16), "upload FF16 LogWalsh");
        HIP_OK(upload(&d.qlog16, g_h_qlog16), "upload FF16 high-part table");
        HIP_OK(hipMalloc(reinterpret_cast<void**>(&d.zeros), 4096), "zero page");
        HIP_OK(hipMemset(d.zeros, 0, 4096), "zero page");
        HIP_OK(hipStreamCreateWithFlags(&d.svc, hipStreamNonBlocking), "service stream");
        int cus = 0;
        HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "compute unit count");
        d.cus = cus > 0 ? unsigned(cus) : 1u;
        hipMemPoolProps props;
        std::memset(&props, 0, sizeof(props));
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        HIP_OK(hipMemPoolCreate(&d.pool, &props), "workspace memory pool");
        // Freed blocks up to kPoolKeepBytes stay in the pool for reuse (a call's
        // scratch, the ring, small direct rows); above that the pool returns
        // memory to the device at the next synchronisation, so one-off large
        // allocations (direct rows of a big host call, an arena replaced by a
        // larger one) are not held idle against the application's own
        // allocations.  release_device_memory trims the rest.
        uint64_t keep = kPoolKeepBytes;
        HIP_OK(hipMemPoolSetAttribute(d.pool, hipMemPoolAttrReleaseThreshold, &keep), "pool release threshold");
        d.ready = true;
    }
    *out = &d;
    return Leopard_Success;
}

// Set by an atexit handler (registered in leo_init after the HIP runtime is
// up, so it runs before the runtime's own teardown): workspaces destroyed
// after it leave their memory to process teardown instead of calling into a
// runtime that may be half gone.
std::atomic<bool> g_exiting{false};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

// Stream-ordered allocation from the library's pool of device dev.
hipError_t pool_alloc(void** p, size_t bytes, int dev, hipStream_t s) {
    return hipMallocFromPoolAsync(p, bytes, g_dev[dev].pool, s);
}

// Frees stream-ordered allocations that nothing uses any more on the device's
// service stream and trims the library's pool (only its own: the application's
// allocations are elsewhere), so that the memory is free again (hipMemGetInfo)
// when this returns.
void release_device_memory(int dev, std::initializer_list<void*> ptrs) {
    hipStream_t svc = dev >= 0 && dev < int(g_dev.size()) ? g_dev[dev].svc : nullptr;
    bool any = false;
    for (void* p : ptrs)
        if (p) {
            (void)hipFreeAsync(p, svc);
            any = true;
        }
    if (!any) return;
    (void)hipStreamSynchronize(svc);
    if (svc && g_dev[dev].pool) (void)hipMemPoolTrimTo(g_dev[dev].pool, 0);
}

// Scratch of one (thread, device, stream): device arena plus a pinned host
// staging area for pointer tables / bitmaps.  Keyed by stream as well as by
// device: the kernels of a call read the arena after the call returns (async
// mode), and only calls on the same stream are ordered after them, so two
// streams must never share one arena.
//
// Lifetime: a thread keeps at most kMaxWorkspaces of them (least recently used
// evicted first) and releases all of them when it exits.  Device memory is
// allocated and freed stream-ordered on the workspace's stream (growth never
// synchronises the device), and `last_use` -- recorded on the stream after
// every call that used the workspace's memory -- is waited for before a
// workspace is freed, so release is safe even after the caller destroyed the
// stream.  (The reference holds no per-call state at all)
// Events that only order work (a slot's reuse, a workspace's release, one
// stream's wait for another): completion without the system-scope fence a
// default event adds, which writes back and invalidates the caches and held
// back the next kernel of a back-to-back stream by ~5.5 us (a decode call
// marks its workspace use; profiles/r04_v13/ff8trace).  Events after which the
// host reads what the device wrote keep the fence.
#ifndef LAMD_ORDER_EVENT_FLAGS
#define LAMD_ORDER_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
constexpr unsigned kOrderEvent = LAMD_ORDER_EVENT_FLAGS;

struct Workspace {
    int dev = -1;
    hipStream_t stream = nullptr;
    uint8_t* dbuf = nullptr;
    size_t dsize = 0;
    hipEvent_t last_use = nullptr;
    bool touched = false;  // the current call enqueued work that uses this workspace's memory
    // Pinned staging ring for small host->device uploads (pointer tables,
    // batch argument blocks, decoder state): a slot is rewritten only after
    // the copy issued from it kBack uploads ago has completed, so back-to-back
    // async calls do not wait for each other's copies.
    static constexpr int kStageSlots = 8;
    struct StageSlot {
        uint8_t* host = nullptr;
        size_t size = 0;
        hipEvent_t done = nullptr;
        bool pending = false;
    };
    StageSlot stage[kStageSlots];
    unsigned stage_next = 0;
    // Host-memory pipeline ring: two slots of `slot_bytes` in pinned host memory
    // and in device memory, one stream and two events per slot.
    uint8_t* ring_host = nullptr;
    uint8_t* ring_host_dev = nullptr;  // device address of ring_host (mapped pinned memory)
    uint8_t* ring_dev = nullptr;
    size_t slot_bytes = 0;
    hipStream_t pipe_stream[2] = {nullptr, nullptr};
    hipEvent_t in_done[2] = {nullptr, nullptr};
    hipEvent_t out_done[2] = {nullptr, nullptr};
    // GF(2^16) decoder states kept on the device across calls (allocations of
    // their own, so the arena above can be reused by every other call), one
    // per erasure pattern in kDec16Slots slots: erasure bitmap, the two
    // occupancy pyramids, the error locator and its FWHT scratch, the scale /
    // reveal log values.  A slot's key is the (K, R, bitmap) it was built for:
    // a repeated pattern re-uploads nothing and skips the error-locator
    // launches.  A new pattern takes the next slot the current call does not
    // use (a batch holds one per object); slots are rewritten only by later
    // work on this workspace's stream.
    struct Dec16Slot {
        uint8_t* mem = nullptr;
        std::vector<uint32_t> key;
        uint64_t stamp = 0;
    };
    static constexpr unsigned kDec16Slots = 16;
    Dec16Slot dec16[kDec16Slots];
    uint64_t dec16_call = 0;
    unsigned dec16_next = 0;
    // Device rows of a host call staged by direct SDMA copies (run_host_direct),
    // and the side streams its column slices run on (with their events).
    uint8_t* direct = nullptr;
    size_t direct_size = 0;
    static constexpr int kSideStreams = 3;
    hipStream_t side[kSideStreams] = {nullptr, nullptr, nullptr};
    hipEvent_t side_ev[kSideStreams + 1] = {nullptr, nullptr, nullptr, nullptr};
    // GF(2^8) error locators by erasure pattern (k_el8's outputs): kEl8Slots
    // slots of 256 bytes on the device.  A pattern seen before launches
    // nothing; a new one takes the next slot that the current call does not
    // use.  Slots are rewritten only by later work on this workspace's stream,
    // so every decode enqueued earlier has read its slot by then.
    struct El8Key {
        uint32_t e[8];
        bool operator==(const El8Key& o) const { return std::memcmp(e, o.e, sizeof(e)) == 0; }
    };
    struct El8Hash {
        size_t operator()(const El8Key& k) const {
            uint64_t h = 1469598103934665603ull;
            for (uint32_t v : k.e) h = (h ^ v) * 1099511628211ull;
            return size_t(h);
        }
    };
    // Tile queues of the bit-sliced batch kernel (rs_ff8_bs.hip): two sets of
    // kBsQueueDw counters; launch i on this stream takes set i & 1 and zeroes
    // the other one, which launch i - 1 used and has finished with (stream order).
    uint32_t* bsq = nullptr;
    unsigned bsq_launches = 0;
    LeopardResult bs_queue(uint32_t** use, uint32_t** clear) {
        touched = true;
        if (!bsq) {
            HIP_OK(pool_alloc(reinterpret_cast<void**>(&bsq), 2 * kBsQueueDw * 4, dev, stream), "allocate tile queues");
            HIP_OK(hipMemsetAsync(bsq, 0, 2 * kBsQueueDw * 4, stream), "clear tile queues");
        }
        *use = bsq + (bsq_launches & 1u) * kBsQueueDw;
        *clear = bsq + ((bsq_launches + 1) & 1u) * kBsQueueDw;
        ++bsq_launches;
        return Leopard_Success;
    }
    static constexpr unsigned kEl8Slots = 512;
    uint32_t* el8 = nullptr;
    std::unordered_map<El8Key, unsigned, El8Hash> el8_map;
    std::vector<El8Key> el8_key;     // pattern of each slot
    std::vector<uint64_t> el8_stamp;  // the call that last used each slot
    std::vector<uint8_t> el8_valid;
    uint64_t el8_call = 0;
    unsigned el8_next = 0;
    // Host copies of the slots (read back once per pattern, pinned): a single
    // call whose pattern's locator is on the host passes it by value and reads
    // no workspace memory, so it needs no completion marker after it (a marker
    // between back-to-back kernels cost ~1.3 us a call, profiles/r04_v15).
    // el8_state: 0 device only, 1 read-back pending (event el8_evi), 2 on the
    // host.  el8_epoch tells a pending read-back of a slot's previous pattern
    // from one of its current pattern.
    static constexpr int kEl8Events = 4;
    uint8_t* el8_host = nullptr;
    std::vector<uint8_t> el8_state, el8_evi;
    std::vector<uint32_t> el8_epoch;
    hipEvent_t el8_ev[kEl8Events] = {};
    std::vector<std::pair<unsigned, uint32_t>> el8_ev_slots[kEl8Events];  // (slot, epoch) per pending event

    ~Workspace() { release(); }
    // Waits for the work that may still use this workspace, then frees it.
    void release() {
        if (g_exiting.load()) return;  // process teardown: the runtime may already be gone
        DeviceGuard guard(dev);
        if (last_use) (void)hipEventSynchronize(last_use);
        for (int s = 0; s < 2; ++s)
            if (pipe_stream[s]) (void)hipStreamSynchronize(pipe_stream[s]);
        for (StageSlot& sl : stage) {
            if (sl.pending) (void)hipEventSynchronize(sl.done);
            if (sl.host) (void)hipHostFree(sl.host);
            if (sl.done) (void)hipEventDestroy(sl.done);
            sl = StageSlot{};
        }
        release_device_memory(dev, {dbuf, ring_dev, direct, el8, bsq});
        if (el8_host) (void)hipHostFree(el8_host);
        el8_host = nullptr;
        for (int e = 0; e < kEl8Events; ++e) {
            if (el8_ev[e]) (void)hipEventDestroy(el8_ev[e]);
            el8_ev[e] = nullptr;
            el8_ev_slots[e].clear();
        }
        el8_state.clear();
        el8_evi.clear();
        el8_epoch.clear();
        for (Dec16Slot& d : dec16) {
            release_device_memory(dev, {d.mem});
            d = Dec16Slot{};
        }
        el8 = nullptr;
        bsq = nullptr;
        bsq_launches = 0;
        el8_map.clear();
        el8_key.clear();
        el8_stamp.clear();
        el8_valid.clear();
        if (ring_host) (void)hipHostFree(ring_host);
        for (int s = 0; s < 2; ++s) {
            if (pipe_stream[s]) (void)hipStreamDestroy(pipe_stream[s]);
            if (in_done[s]) (void)hipEventDestroy(in_done[s]);
            if (out_done[s]) (void)hipEventDestroy(out_done[s]);
            pipe_stream[s] = nullptr;
            in_done[s] = out_done[s] = nullptr;
        }
        for (int i = 0; i < kSideStreams; ++i)
            if (side[i]) {
                (void)hipStreamSynchronize(side[i]);
                (void)hipStreamDestroy(side[i]);
                side[i] = nullptr;
            }
        for (hipEvent_t& e : side_ev)
            if (e) {
                (void)hipEventDestroy(e);
                e = nullptr;
            }
        if (last_use) (void)hipEventDestroy(last_use);
        dbuf = ring_dev = ring_host = ring_host_dev = direct = nullptr;
        last_use = nullptr;
        dsize = slot_bytes = direct_size = 0;
    }
    // Called at the end of every call: marks where the work of this call that
    // uses the workspace's memory ends on the stream.
    LeopardResult mark_use(hipStream_t s) {
#ifdef LAMD_X_NO_MARK  // A/B only: what the per-call event costs (unsafe release)
        touched = false;
#endif
        if (!touched) return Leopard_Success;
        touched = false;
        if (!last_use) HIP_OK(hipEventCreateWithFlags(&last_use, kOrderEvent), "event");
#ifdef LAMD_X_TRACE_MARK
        std::fprintf(stderr, "mark_use\n");
#endif
        HIP_OK(hipEventRecord(last_use, s), "record workspace use");
        return Leopard_Success;
    }
    LeopardResult reserve_ring(size_t bytes_per_slot) {
        for (int s = 0; s < 2; ++s) {
            if (!pipe_stream[s]) HIP_OK(hipStreamCreateWithFlags(&pipe_stream[s], hipStreamNonBlocking), "stream");
            if (!in_done[s]) HIP_OK(hipEventCreateWithFlags(&in_done[s], kOrderEvent), "event");
            if (!out_done[s]) HIP_OK(hipEventCreateWithFlags(&out_done[s], hipEventDisableTiming), "event");
        }
        if (bytes_per_slot <= slot_bytes) return Leopard_Success;
        if (ring_dev) {
            // the ring is used only by its own two streams (the host pipeline
            // waits for both before returning, so this is normally a no-op)
            for (int s = 0; s < 2; ++s) HIP_OK(hipStreamSynchronize(pipe_stream[s]), "sync before ring growth");
            HIP_OK(hipFreeAsync(ring_dev, pipe_stream[0]), "free ring");
            HIP_OK(hipHostFree(ring_host), "free pinned ring");
            ring_dev = ring_host = ring_host_dev = nullptr;
            slot_bytes = 0;
        }
        const size_t want = (bytes_per_slot + 4095) / 4096 * 4096;
        HIP_OK(pool_alloc(reinterpret_cast<void**>(&ring_dev), 2 * want, dev, pipe_stream[0]), "allocate device ring");
        // both pipe streams use it: the second one waits for the allocation
        HIP_OK(hipEventRecord(in_done[0], pipe_stream[0]), "record ring allocation");
        HIP_OK(hipStreamWaitEvent(pipe_stream[1], in_done[0], 0), "order ring allocation");
        HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&ring_host), 2 * want, hipHostMallocDefault), "pinned ring");
        HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ring_host_dev), ring_host, 0), "map pinned ring");
        slot_bytes = want;
        return Leopard_Success;
    }
    // Device arena of at least `bytes`, stream-ordered: a grown arena replaces
    // the old one after this stream's earlier work (no device synchronisation).
    LeopardResult reserve_device(size_t bytes) {
        touched = true;
        if (bytes <= dsize) return Leopard_Success;
        const size_t want = std::max(bytes, dsize * 2);
        if (dbuf) HIP_OK(hipFreeAsync(dbuf, stream), "free scratch");
        dbuf = nullptr;
        dsize = 0;
        HIP_OK(pool_alloc(reinterpret_cast<void**>(&dbuf), want, dev, stream), "allocate scratch");
        dsize = want;
        return Leopard_Success;
    }
    // The decoder-state slot of pattern `key` for the current call (++dec16_call
    // first): *fresh when it must be built.  Fails when every slot is taken by
    // the current call (callers keep to kDec16Slots patterns a call).
    LeopardResult dec16_slot(std::vector<uint32_t>& key, size_t bytes, unsigned* idx, bool* fresh) {
        touched = true;
        for (unsigned i = 0; i < kDec16Slots; ++i)
            if (dec16[i].mem && dec16[i].key == key) {
                dec16[i].stamp = dec16_call;
                *idx = i;
                *fresh = false;
                return Leopard_Success;
            }
        unsigned tries = 0;
        while (dec16[dec16_next].stamp == dec16_call && tries++ < kDec16Slots) dec16_next = (dec16_next + 1) % kDec16Slots;
        if (tries > kDec16Slots) {
            tls.last_error = "too many erasure patterns in one call";
            return Leopard_InvalidInput;
        }
        Dec16Slot& d = dec16[dec16_next];
        if (!d.mem) HIP_OK(pool_alloc(reinterpret_cast<void**>(&d.mem), bytes, dev, stream), "allocate decoder state");
        d.key.swap(key);
        d.stamp = dec16_call;
        *idx = dec16_next;
        *fresh = true;
        dec16_next = (dec16_next + 1) % kDec16Slots;
        return Leopard_Success;
    }
    // Starts a call's use of the error-locator cache (slots it takes stay put until the next call).
    void el8_begin() { ++el8_call; }
    // The device error locator of erasure bitmap `erased` (8 words): a cached
    // slot, or a new slot whose computation is appended to `jobs` (flush_el8
    // launches them, ahead of the decode kernels).
    // The caller marks the workspace touched when a kernel reads the slot.
    LeopardResult el8_slot(const uint32_t* erased, std::vector<El8Job>& jobs, const uint32_t** out,
                           unsigned* slot_out = nullptr) {
        if (!el8) {
            touched = true;
            HIP_OK(pool_alloc(reinterpret_cast<void**>(&el8), size_t(kEl8Slots) * 256, dev, stream),
                   "allocate error locators");
            HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&el8_host), size_t(kEl8Slots) * 256, hipHostMallocDefault),
                   "pinned error locators");
            el8_key.assign(kEl8Slots, El8Key{});
            el8_stamp.assign(kEl8Slots, 0);
            el8_valid.assign(kEl8Slots, 0);
            el8_state.assign(kEl8Slots, 0);
            el8_evi.assign(kEl8Slots, 0);
            el8_epoch.assign(kEl8Slots, 0);
        }
        El8Key k;
        std::memcpy(k.e, erased, sizeof(k.e));
        unsigned slot;
        const auto it = el8_map.find(k);
        if (it != el8_map.end()) {
            slot = it->second;
        } else {
            unsigned tries = 0;
            while (el8_stamp[el8_next] == el8_call && tries++ < kEl8Slots) el8_next = (el8_next + 1) % kEl8Slots;
            if (tries > kEl8Slots) {  // callers split their work into <= kEl8Slots patterns per call
                tls.last_error = "too many erasure patterns in one call";
                return Leopard_InvalidInput;
            }
            slot = el8_next;
            el8_next = (el8_next + 1) % kEl8Slots;
            if (el8_valid[slot]) el8_map.erase(el8_key[slot]);
            el8_key[slot] = k;
            el8_valid[slot] = 1;
            el8_state[slot] = 0;
            ++el8_epoch[slot];
            el8_map.emplace(k, slot);
            touched = true;  // k_el8 writes the slot
            El8Job j;
            std::memcpy(j.erased, erased, sizeof(j.erased));
            j.slot = slot;
            jobs.push_back(j);
        }
        el8_stamp[slot] = el8_call;
        *out = el8 + size_t(slot) * 64;
        if (slot_out) *slot_out = slot;
        return Leopard_Success;
    }
    // The host copy of slot's locator, if it has arrived (never waits).
    bool el8_value(unsigned slot, uint32_t* out) {
        if (el8_state[slot] == 1) {
            const int e = el8_evi[slot];
            if (hipEventQuery(el8_ev[e]) != hipSuccess) return false;
            for (const auto& se : el8_ev_slots[e])
                if (el8_epoch[se.first] == se.second && el8_state[se.first] == 1) el8_state[se.first] = 2;
            el8_ev_slots[e].clear();
        }
        if (el8_state[slot] != 2) return false;
        std::memcpy(out, el8_host + size_t(slot) * 256, 256);
        return true;
    }
    // Queues the read-back of slot's locator (after the work that writes it),
    // if one of the read-back events is free.
    LeopardResult el8_readback(unsigned slot, hipStream_t s) {
        if (el8_state[slot] != 0) return Leopard_Success;
        int e = -1;
        for (int i = 0; i < kEl8Events && e < 0; ++i) {
            if (!el8_ev[i]) {
                // the host reads what the copy wrote: a default (system-fenced) event
                HIP_OK(hipEventCreateWithFlags(&el8_ev[i], hipEventDisableTiming), "event");
                e = i;
            } else if (el8_ev_slots[i].empty() || hipEventQuery(el8_ev[i]) == hipSuccess) {
                for (const auto& se : el8_ev_slots[i])
                    if (el8_epoch[se.first] == se.second && el8_state[se.first] == 1) el8_state[se.first] = 2;
                el8_ev_slots[i].clear();
                e = i;
            }
        }
        if (e < 0) return Leopard_Success;  // all busy: a later call of this pattern tries again
        touched = true;
        HIP_OK(hipMemcpyAsync(el8_host + size_t(slot) * 256, el8 + size_t(slot) * 64, 256, hipMemcpyDeviceToHost, s),
               "read back error locator");
        HIP_OK(hipEventRecord(el8_ev[e], s), "record read-back");
        el8_ev_slots[e].emplace_back(slot, el8_epoch[slot]);
        el8_state[slot] = 1;
        el8_evi[slot] = uint8_t(e);
        return Leopard_Success;
    }
    // A slot whose computation failed to launch holds nothing valid.
    void el8_forget(unsigned slot) {
        if (slot < el8_valid.size() && el8_valid[slot]) {
            el8_map.erase(el8_key[slot]);
            el8_valid[slot] = 0;
        }
    }
    // Device rows for run_host_direct, stream-ordered like the arena.
    LeopardResult reserve_direct(size_t bytes) {
        touched = true;
        if (bytes <= direct_size) return Leopard_Success;
        if (direct) HIP_OK(hipFreeAsync(direct, stream), "free direct rows");
        direct = nullptr;
        direct_size = 0;
        HIP_OK(pool_alloc(reinterpret_cast<void**>(&direct), bytes, dev, stream), "allocate direct rows");
        direct_size = bytes;
        return Leopard_Success;
    }
    // Copies `bytes` from host memory src (or, with src == nullptr, lets
    // fill(host) write them) through the next ring slot into device memory dst,
    // ordered on stream s.
    template <class Fill>
    LeopardResult upload(void* dst, size_t bytes, hipStream_t s, Fill&& fill) {
        touched = true;
        StageSlot& sl = stage[stage_next];
        stage_next = (stage_next + 1) % kStageSlots;
        if (sl.pending) {
            HIP_OK(hipEventSynchronize(sl.done), "wait staging slot");
            sl.pending = false;
        }
        if (!sl.done) HIP_OK(hipEventCreateWithFlags(&sl.done, kOrderEvent), "event");
        if (bytes > sl.size) {
            if (sl.host) HIP_OK(hipHostFree(sl.host), "free staging");
            sl.host = nullptr;
            const size_t want = std::max<size_t>(bytes, std::max<size_t>(sl.size * 2, 1 << 16));
            HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&sl.host), want, hipHostMallocDefault), "pinned staging");
            sl.size = want;
        }
        fill(sl.host);
        HIP_OK(hipMemcpyAsync(dst, sl.host, bytes, hipMemcpyHostToDevice, s), "upload");
        HIP_OK(hipEventRecord(sl.done, s), "record staging");
        sl.pending = true;
        return Leopard_Success;
    }
    LeopardResult upload(void* dst, const void* src, size_t bytes, hipStream_t s) {
        return upload(dst, bytes, s, [&](uint8_t* h) { std::memcpy(h, src, bytes); });
    }
};
// The calling thread's workspaces, most recently used first; released when the
// thread exits.  At most kMaxWorkspaces are kept: one API call uses at most
// three (its own and the host pipeline's two slot streams), always the most
// recently used ones, so eviction never frees one that a call in progress holds.
constexpr size_t kMaxWorkspaces = 8;
struct WorkspaceList {
    std::vector<std::unique_ptr<Workspace>> list;
    ~WorkspaceList() { list.clear(); }
};
thread_local WorkspaceList tws;

// Frees workspace i (waiting for its work) and the workspaces of the host
// pipeline streams it owned (those streams are destroyed with it).
void drop_workspace(size_t i) {
    auto& l = tws.list;
    const hipStream_t ps[2 + Workspace::kSideStreams] = {l[i]->pipe_stream[0], l[i]->pipe_stream[1], l[i]->side[0],
                                                        l[i]->side[1], l[i]->side[2]};
    l.erase(l.begin() + i);
    for (hipStream_t p : ps)
        for (size_t j = 0; p && j < l.size();)
            if (l[j]->stream == p) l.erase(l.begin() + j);
            else ++j;
}

Workspace& workspace(int dev, hipStream_t stream) {
    auto& l = tws.list;
    for (size_t i = 0; i < l.size(); ++i)
        if (l[i]->dev == dev && l[i]->stream == stream) {
            std::rotate(l.begin(), l.begin() + i, l.begin() + i + 1);
            return *l.front();
        }
    l.insert(l.begin(), std::make_unique<Workspace>());
    l.front()->dev = dev;
    l.front()->stream = stream;
    while (l.size() > kMaxWorkspaces) drop_workspace(l.size() - 1);  // least recently used
    return *l.front();
}

// Drops the calling thread's workspaces of `stream` (every device), or all of
// them (leo_amd_release_stream).
void release_workspaces(hipStream_t stream, bool all) {
    auto& l = tws.list;
    for (size_t i = 0; i < l.size();) {
        if (all || l[i]->stream == stream) {
            drop_workspace(i);  // may remove entries before i as well
            i = 0;
        } else {
            ++i;
        }
    }
}

// ------------------------------------------------------------ call helpers --

unsigned next_pow2(unsigned n) {
    unsigned p = 1;
    while (p < n) p <<= 1;
    return p;
}
unsigned log2u(unsigned n) {
    unsigned t = 0;
    while ((1u << t) < n) ++t;
    return t;
}

enum class MemKind { Device, Host };

// Pointer kind from the first non-null pointer (all pieces of a call must agree).
MemKind classify(const void* p, int* dev) {
    hipPointerAttribute_t attr;
    std::memset(&attr, 0, sizeof(attr));
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return MemKind::Host;
    }
    if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) {
        *dev = attr.device;
        return MemKind::Device;
    }
    return MemKind::Host;
}

// Builds a PieceMap: a slab (base + i*stride) when the non-null pointers are
// equally spaced, else a device pointer table written into `tables` (pinned
// staging, uploaded by the caller).
struct MapBuilder {
    std::vector<uint64_t> staged;  // host image of all tables of this call
    struct Pending {
        PieceMap* map;
        size_t index;
    };
    std::vector<Pending> pending;

    void build(PieceMap& pm, const void* const* ptrs, unsigned count, uint64_t off) {
        pm = PieceMap{nullptr, nullptr, 0, off};
        int i0 = -1, i1 = -1;
        for (unsigned i = 0; i < count; ++i) {
            if (!ptrs[i]) continue;
            if (i0 < 0) i0 = int(i);
            else { i1 = int(i); break; }
        }
        if (i0 < 0) return;  // nothing present; never dereferenced
        int64_t stride = 0;
        bool slab = true;
        const int64_t p0 = int64_t(reinterpret_cast<uintptr_t>(ptrs[i0]));
        if (i1 >= 0) {
            const int64_t d = int64_t(reinterpret_cast<uintptr_t>(ptrs[i1])) - p0;
            if (d % (i1 - i0) != 0) slab = false;
            else stride = d / (i1 - i0);
        }
        for (unsigned i = unsigned(i0); slab && i < count; ++i)
            if (ptrs[i] && int64_t(reinterpret_cast<uintptr_t>(ptrs[i])) != p0 + (int64_t(i) - i0) * stride) slab = false;
        if (slab) {
            pm.base = reinterpret_cast<uint8_t*>(uintptr_t(p0 - int64_t(i0) * stride));
            pm.stride = uint64_t(stride);
            return;
        }
        const size_t at = staged.size();
        for (unsigned i = 0; i < count; ++i) staged.push_back(uint64_t(reinterpret_cast<uintptr_t>(ptrs[i])));
        pending.push_back({&pm, at});
    }
    size_t bytes() const { return staged.size() * sizeof(uint64_t); }
    // Enqueues the upload of the tables into dev (through the staging ring).
    LeopardResult flush(Workspace& ws, uint64_t* dev, hipStream_t s) {
        if (staged.empty()) return Leopard_Success;
        LeopardResult r = ws.upload(dev, staged.data(), bytes(), s);
        if (r != Leopard_Success) return r;
        for (auto& p : pending) p.map->table = dev + p.index;
        return Leopard_Success;
    }
};

// Pieces of at most this many bytes count as narrow columns for the small
// GF(2^16) kernels (rs_ff16_small.hip): 256 KiB = 2048 strips of 128 bytes.
constexpr uint64_t kNarrowColumnsMax = 256 << 10;
constexpr uint64_t kOnePassMinBytes = 60 << 10;  // the single-pass GF(2^16) decoder from here (rs_ff16_small.hip)

// Columns per GF(2^8) launch: its argument block counts dword columns in 32 bits.
constexpr uint64_t kFf8MaxLaunchBytes = 1ull << 32;

// Column range processed per pass sequence of the multi-pass FF16 kernels:
// keep the intermediates (pieces x slice) around the 256 MiB Infinity Cache.
uint64_t mall_budget() {
    static const uint64_t v = [] {
        const char* e = std::getenv("LEO_AMD_SLICE_MB");  // tuning experiments
        const long mb = e ? std::atol(e) : 3072;
        return uint64_t(std::max(1L, mb)) << 20;
    }();
    return v;
}
uint64_t mall_slice(uint64_t bytes, uint64_t slab_pieces) {
    const uint64_t budget = mall_budget();
    uint64_t slice = budget / std::max<uint64_t>(slab_pieces, 1);
    slice = std::max<uint64_t>(slice / 512 * 512, 512);  // whole FF16 tiles (64 units x 8 B)
    return std::min(slice, bytes);
}

struct Call {
    int dev = 0;
    DeviceTables* t = nullptr;
    Workspace* ws = nullptr;
    hipStream_t s = nullptr;
};

LeopardResult begin_call(int dev, Call& c) {
    LeopardResult r = ensure_device(dev, &c.t);
    if (r != Leopard_Success) return r;
    c.dev = dev;
    c.s = tls.stream;
    c.ws = &workspace(dev, c.s);
    return Leopard_Success;
}

LeopardResult finish(const Call& c, bool force_sync) {
    HIP_OK(hipGetLastError(), "kernel launch");
    if (c.ws) {
        const LeopardResult r = c.ws->mark_use(c.s);
        if (r != Leopard_Success) return r;
    }
    if (force_sync || !tls.async) HIP_OK(hipStreamSynchronize(c.s), "stream synchronize");
    return Leopard_Success;
}

// --------------------------------------------------------------- encode ----

// ------------------------------------------------------------ matrix path --
// Small GF(2^8) codes and few losses (rs_ff8_mat.hip): the call applied as its
// L x N coefficient matrix, built once per (K, R, erasure pattern) from the
// transform kernels' own outputs on unit pieces.  LEO_AMD_FF8_MATRIX=0 turns it
// off (A/B experiments); read once.
bool ff8_matrix_enabled() {
    static const bool v = !experiment_off("LEO_AMD_FF8_MATRIX");
    return v;
}
thread_local bool tls_mat_gen = false;  // building a matrix: the transform kernels, never the matrix path
// Where the matrix runs (measured crossovers): at most
// kMatMaxEntries coefficients, and L N bytes (the matrix's multiply-adds) at
// most kMatMaxWork where the transform path is slow for its work -- the split
// decoder (n = 2m, its three transforms and 128 scale multiplies) and encoders
// that run three or more chunks one after the other -- or any call of at most
// kMatSmallBytes; kMatMaxWorkOther otherwise.  Decodes (their transform path
// runs the error locator, two or three transforms and the scale multiplies):
// kMatMaxWorkDec.
constexpr unsigned kMatMaxEntries = 4096;
constexpr uint64_t kMatMaxWork = 1ull << 27;
constexpr uint64_t kMatMaxWorkOther = 1ull << 25;
constexpr uint64_t kMatMaxWorkDec = 3ull << 27;
constexpr uint64_t kMatSmallBytes = 16ull << 10;
bool use_matrix(unsigned L, unsigned N, uint64_t bytes, bool slow_transform, bool decode) {
    const uint64_t work = uint64_t(L) * N * bytes;
    uint64_t cap = decode ? kMatMaxWorkDec : slow_transform || bytes <= kMatSmallBytes ? kMatMaxWork : kMatMaxWorkOther;
#if LAMD_EXPERIMENT_ENV
    // A/B of the crossovers: LEO_AMD_MAT_WORK=s sets both caps to 2^s
    static const int work_log2 = [] { const char* e = std::getenv("LEO_AMD_MAT_WORK"); return e ? std::atoi(e) : 0; }();
    if (work_log2 > 0 && work_log2 < 40) cap = 1ull << work_log2;
#endif
    return !tls_mat_gen && ff8_matrix_enabled() && L >= 1 && uint64_t(L) * N <= kMatMaxEntries && work <= cap &&
           ff8_mat_supported(L, N);
}
LeopardResult encode_matrix(Call& c, uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                            void** work, bool* done);
bool slab_of(const void* const* p, unsigned n, uint64_t& base, int32_t& stride);

// Single dense 128 + 128 calls (encode, or the full-loss decode) on pieces of at
// least kBsSingleMinBytes whose inputs and outputs are slabs: the bit-sliced
// batch tile with one object (rs_ff8_bs.hip; its persistent grid has a tile for
// every wave from 2048 256-byte strips on).  Smaller calls keep the byte tile,
// whose 16-wave workgroups finish one strip sooner.  *done: launched.
constexpr uint64_t kBsSingleMinBytes = 512ull << 10;
LeopardResult dense_single_bs(Call& c, uint64_t bytes, uint64_t off, unsigned m, const void* const* in,
                              void* const* out, int form, bool* done) {
    *done = false;
    uint64_t ib = 0, ob = 0;
    int32_t is = 0, os = 0;
    static const bool enabled = !experiment_off("LEO_AMD_FF8_BS_SINGLE");  // A/B experiments only
    if (!enabled || m != 128 || bytes < kBsSingleMinBytes || bytes / 4 > 0xFFFFFFFFull || !ff8_bs_supported(7, m, m, 1) ||
        !slab_of(in, m, ib, is) || !slab_of(const_cast<const void* const*>(out), m, ob, os))
        return Leopard_Success;
    Ff8SlabBatch b;
    std::memset(&b, 0, sizeof(b));
    b.in_base[0] = ib + off;
    b.in_stride[0] = is;
    b.out_base[0] = ob + off;
    b.out_stride[0] = os;
    b.sktab = c.t->sktab8;
    b.fused = c.t->fused8 + size_t(6) * 256 * kTab8Dwords;  // T = 7, chunk 0
    b.K = b.R = m;
    b.nchunks = 1;
    b.nunits = uint32_t(bytes / 4);
    uint32_t *q = nullptr, *qclear = nullptr;
    const LeopardResult r = c.ws->bs_queue(&q, &qclear);
    if (r != Leopard_Success) return r;
    HIP_OK(launch_ff8_encode_slab(7, b, 1, false, form, c.s, c.t->cus, q, qclear), "bit-sliced single call");
    *done = true;
    return Leopard_Success;
}
LeopardResult decode_matrix(Call& c, uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                            const void* const* rec, void** work, bool* done);

// GF(2^8) encoder argument block of one object: columns [off, off + bytes)
// of every piece (bytes <= kFf8MaxLaunchBytes).
void fill_enc8(Ff8EncArgs& a, const DeviceTables* t, unsigned K, unsigned R, const void* const* orig, void** work,
               uint64_t off, uint64_t bytes) {
    const unsigned m = next_pow2(R);
    std::memset(&a, 0, sizeof(a));
    for (unsigned i = 0; i < K; ++i) a.ptr[i] = uint64_t(reinterpret_cast<uintptr_t>(orig[i])) + off;
    for (unsigned i = 0; i < R; ++i) a.ptr[K + i] = uint64_t(reinterpret_cast<uintptr_t>(work[i])) + off;
    a.sktab = t->sktab8;
    a.fused = t->fused8 + size_t(log2u(m) - 1) * 256 * kTab8Dwords;
    a.K = K;
    a.R = R;
    a.nchunks = (K + m - 1) / m;
    a.nunits = uint32_t(bytes / 4);
}

// Device-resident encode of pieces [off, off + bytes) (reference:
// leo_encode -> ff8|ff16::ReedSolomonEncode, leopard.cpp:162-197).
LeopardResult encode_device(Call& c, uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                            void** work) {
    const unsigned m = next_pow2(R);
    const unsigned n = next_pow2(m + K);
    const bool ff16 = n > 256;
    const unsigned Tm = log2u(m);
    const unsigned nchunks = (K + m - 1) / m;

    if (!ff16) {  // n <= 256: one fused kernel, launch data by value (rs_ff8.hip)
        // small codes: the coefficient matrix (use_matrix)
        if (K == R && nchunks == 1) {  // dense 128 + 128 on large pieces: the bit-sliced tile
            bool done = false;
            const LeopardResult r = dense_single_bs(c, bytes, off, m, orig, work, kFormDenseEnc, &done);
            if (r != Leopard_Success || done) return r;
        }
        if (use_matrix(R, K, bytes, nchunks >= 3, false) && (nchunks >= 2 || bytes <= kMatSmallBytes)) {
            bool done = false;
            const LeopardResult r = encode_matrix(c, bytes, off, K, R, orig, work, &done);
            if (r != Leopard_Success || done) return r;
        }
        Ff8EncArgs a;
        // one launch per <= 4 GiB of columns (the kernel counts dword columns in 32 bits)
        for (uint64_t pos = 0; pos < bytes; pos += kFf8MaxLaunchBytes) {
            fill_enc8(a, c.t, K, R, orig, work, off + pos, std::min(kFf8MaxLaunchBytes, bytes - pos));
            HIP_OK(launch_ff8_encode(Tm, a, c.s), "encode kernel");
        }
        return Leopard_Success;
    }

    EncArgs a;
    std::memset(&a, 0, sizeof(a));
    MapBuilder mb;
    mb.build(a.in, orig, K, off);
    mb.build(a.out, work, R, off);
    a.sktab = ff16 ? c.t->sktab16 : c.t->sktab8;
    a.tabs = ff16 ? c.t->tab16 : c.t->tab8;
    a.zeros = c.t->zeros;
    a.fused = c.t->fused16 + fused16_base(Tm);
    a.K = K;
    a.R = R;
    a.Tm = Tm;
    a.nchunks = nchunks;
    const unsigned unit_bytes = ff16 ? 8 : 4;

    // Multi-pass for m > 2^kLoBits; also for m = 2^kLoBits with several chunks
    // on narrow columns, where the single-tile kernel's one workgroup per
    // 512-byte strip leaves CUs idle: pass 1 runs the chunk IFFTs in parallel
    // workgroups and pass 3 combines them (no high pass).
    // Narrow columns with m <= 256: one workgroup per 128-byte strip runs the
    // whole encode (rs_ff16_small.hip), enough workgroups to fill the GPU.
    const bool narrow = ff16 && encode16_small_supported(Tm) && bytes <= kNarrowColumnsMax;
    const bool chunk_parallel = !narrow && ff16 && Tm == kLoBits && nchunks > 1 && bytes / 8 < 1024 * 64;
    const bool multipass = !narrow && ((ff16 && Tm > kLoBits) || chunk_parallel);
    uint64_t slice = bytes, slab_bytes = 0;
    if (multipass) {
        const uint64_t slab_pieces = uint64_t(nchunks) * m + m;
        slice = mall_slice(bytes, slab_pieces);
        slab_bytes = slab_pieces * slice;
    }
    // narrow columns, several chunks, fewer 16-unit strips than CUs: the chunk
    // IFFTs in parallel workgroups through a slab of nchunks x m rows
    const bool split = narrow && encode16_split_wins(Tm, nchunks, bytes / unit_bytes, c.t->cus);
    if (split) slab_bytes = uint64_t(nchunks) * m * bytes;
    const size_t table_bytes = (mb.bytes() + 255) / 256 * 256;
    LeopardResult r = c.ws->reserve_device(table_bytes + slab_bytes);
    if (r != Leopard_Success) return r;
    r = mb.flush(*c.ws, reinterpret_cast<uint64_t*>(c.ws->dbuf), c.s);
    if (r != Leopard_Success) return r;

    if (narrow) {
        a.nunits = bytes / unit_bytes;
        if (split) {
            a.slab_out = a.slab_in = PieceMap{nullptr, c.ws->dbuf + table_bytes, bytes, 0};
            HIP_OK(launch_encode16_split(Tm, a, c.s), "encode kernels");
        } else {
            HIP_OK(launch_encode16_small(Tm, a, c.s), "encode kernel");
        }
        return Leopard_Success;
    }
    if (!multipass) {
        a.nunits = bytes / unit_bytes;
        HIP_OK(launch_encode_fused16(Tm, a, c.s), "encode kernel");
        return Leopard_Success;
    }
    uint8_t* U = c.ws->dbuf + table_bytes;
    uint8_t* V = U + uint64_t(nchunks) * m * slice;
    for (uint64_t pos = 0; pos < bytes; pos += slice) {
        const uint64_t len = std::min(slice, bytes - pos);
        EncArgs b = a;
        b.in.off = off + pos;
        b.out.off = off + pos;
        b.slab_out = PieceMap{nullptr, U, slice, 0};
        b.nunits = len / unit_bytes;
        HIP_OK(launch_encode_lo(b, c.s), "encode pass 1");
        if (!chunk_parallel) {
            b.slab_in = PieceMap{nullptr, U, slice, 0};
            b.slab_out = PieceMap{nullptr, V, slice, 0};
            HIP_OK(launch_encode_hi(b, c.s), "encode pass 2");
            b.slab_in = PieceMap{nullptr, V, slice, 0};
        } else {
            b.slab_in = PieceMap{nullptr, U, slice, 0};
        }
        HIP_OK(launch_encode_fin(b, c.s), "encode pass 3");
    }
    return Leopard_Success;
}

// XOR of `count` pieces into out (R == 1 paths).
LeopardResult xor_device(Call& c, uint64_t bytes, uint64_t off, const void* const* src, unsigned count, void* out) {
    XorArgs a;
    std::memset(&a, 0, sizeof(a));
    MapBuilder mb;
    mb.build(a.src, src, count, off);
    void* outs[1] = {out};
    mb.build(a.out, outs, 1, off);
    a.count = count;
    a.ndwords = bytes / 4;
    LeopardResult r = c.ws->reserve_device((mb.bytes() + 255) / 256 * 256);
    if (r != Leopard_Success) return r;
    r = mb.flush(*c.ws, reinterpret_cast<uint64_t*>(c.ws->dbuf), c.s);
    if (r != Leopard_Success) return r;
    HIP_OK(launch_xor_reduce(a, c.s), "xor kernel");
    return Leopard_Success;
}

// --------------------------------------------------------------- decode ----

// LEO_AMD_FF8_HALF=0 turns the half-position decoders (FF8 kernel, FF16 pass 2)
// off (A/B experiments); read once.
bool ff8_half_decoder_enabled() {
    static const bool v = !experiment_off("LEO_AMD_FF8_HALF");
    return v;
}

// LEO_AMD_FF8_SPLIT=0 turns the split partial-loss decoder off (A/B); read once.
bool ff8_split_decoder_enabled() {
    static const bool v = !experiment_off("LEO_AMD_FF8_SPLIT");
    return v;
}

// GF(2^8) erasure bitmap over 256 positions: error_locations[] = 1 at lost
// recoveries, [R, m) and lost originals (LeopardFF8.cpp:1825-1840).
void erasures8(unsigned K, unsigned R, unsigned m, const void* const* orig, const void* const* rec, uint32_t* erased) {
    std::memset(erased, 0, 8 * sizeof(uint32_t));
    auto set = [&](unsigned p) { erased[p >> 5] |= 1u << (p & 31); };
    for (unsigned i = 0; i < R; ++i)
        if (!rec[i]) set(i);
    for (unsigned i = R; i < m; ++i) set(i);
    for (unsigned i = 0; i < K; ++i)
        if (!orig[i]) set(m + i);
}

// GF(2^8) decoder argument block of one object (columns [off, off + bytes));
// returns the decoder kind (kDec8*): with n = 2m, the half-position decoder
// when no original survives (every received piece in the low half of the
// positions, every output in the high half; k_ff8_dec_half), the split decoder
// when some do (k_ff8_dec_split); otherwise the general n-point decoder.
int fill_dec8(Ff8DecArgs& a, const DeviceTables* t, unsigned K, unsigned R, const void* const* orig,
              const void* const* rec, void** work, uint64_t off, uint64_t bytes, const uint32_t* el) {
    const unsigned m = next_pow2(R);
    const unsigned Tn = log2u(next_pow2(m + K));
    std::memset(&a, 0, sizeof(a));
    uint32_t erased[8];
    erasures8(K, R, m, orig, rec, erased);
    auto addr = [&](const void* p) { return uint64_t(reinterpret_cast<uintptr_t>(p)) + off; };
    for (unsigned i = 0; i < R; ++i)
        if (rec[i]) a.ptr[i] = addr(rec[i]);
    for (unsigned i = 0; i < K; ++i) a.ptr[m + i] = addr(orig[i] ? orig[i] : work[i]);  // lost: its slot carries the output
    // The pyramids depend only on (K, R, erasure pattern); the last pattern is
    // cached per thread (repeated patterns are the common case).
    struct PyrCache {
        unsigned K = 0, R = 0;
        uint32_t erased[8] = {~0u};
        uint32_t present[kPyr8Words], needed[kPyr8Words];
    };
    thread_local PyrCache pc;
    if (pc.K != K || pc.R != R || std::memcmp(pc.erased, erased, sizeof(pc.erased)) != 0) {
        auto mark = [](uint32_t* pyr, unsigned p) {
            for (unsigned L = 0; L <= 8; ++L) {
                const unsigned j = p >> L;
                pyr[pyr8_offset(L) + (j >> 5)] |= 1u << (j & 31);
            }
        };
        std::memset(pc.present, 0, sizeof(pc.present));
        std::memset(pc.needed, 0, sizeof(pc.needed));
        for (unsigned i = 0; i < R; ++i)
            if (rec[i]) mark(pc.present, i);
        for (unsigned i = 0; i < K; ++i) mark(orig[i] ? pc.present : pc.needed, m + i);
        pc.K = K;
        pc.R = R;
        std::memcpy(pc.erased, erased, sizeof(pc.erased));
    }
    std::memcpy(a.present, pc.present, sizeof(a.present));
    std::memcpy(a.needed, pc.needed, sizeof(a.needed));
    a.el = el;  // this pattern's error locator (k_el8, cached per workspace)
    a.sktab = t->sktab8;
    a.tabs = t->tab8;
    a.K = K;
    a.R = R;
    a.m = m;
    a.nunits = uint32_t(bytes / 4);
    bool any_orig = false;
    for (unsigned i = 0; i < K; ++i) any_orig |= orig[i] != nullptr;
    const bool two_halves = Tn >= 2 && 2 * m == (1u << Tn);
    // some originals received: the split decoder (k_ff8_dec_split) when n = 2m
    if (any_orig) return two_halves && ff8_split_decoder_enabled() ? kDec8Split : kDec8General;
    const bool half = two_halves && ff8_half_decoder_enabled();
    if (!half) return kDec8General;
    a.fused = t->fused8 + size_t(Tn - 2) * 256 * kTab8Dwords;  // T = Tn - 1, chunk 0
    bool all_rec = K == m && R == m;
    for (unsigned i = 0; i < R && all_rec; ++i) all_rec = rec[i] != nullptr;
    a.dense = all_rec ? 1u : 0u;
    return all_rec ? kDec8HalfDense : kDec8Half;
}

// Launches the queued error-locator computations (k_el8, kEl8Jobs patterns a launch).
LeopardResult flush_el8(Workspace& ws, const DeviceTables* t, std::vector<El8Job>& jobs, hipStream_t s) {
    for (size_t i = 0; i < jobs.size(); i += kEl8Jobs) {
        El8Args a;
        std::memset(&a, 0, sizeof(a));
        const unsigned n = unsigned(std::min<size_t>(kEl8Jobs, jobs.size() - i));
        std::memcpy(a.job, jobs.data() + i, n * sizeof(El8Job));
        a.walsh = t->walsh8;
        a.out = ws.el8;
        const hipError_t e = launch_error_locator8(a, n, s);
        if (e != hipSuccess) {
            for (const El8Job& j : jobs) ws.el8_forget(j.slot);
            jobs.clear();
            set_error("error locator kernel", e);
            return Leopard_Platform;
        }
    }
    jobs.clear();
    return Leopard_Success;
}

// LEO_AMD_FF8_INVERT=0 turns the inverse full-loss decoder off (A/B); read once.
bool ff8_invert_enabled() {
    static const bool v = !experiment_off("LEO_AMD_FF8_INVERT");
    return v;
}

// Full loss of a K = R = m code (every original lost, every recovery piece
// received; the benchmark's worst case at 128+128): the decoder is the inverse
// of the encoder's transform pair (launch_ff8_decode_full, rs_ff8.hip).
bool full_loss_square(unsigned K, unsigned R, const void* const* orig, const void* const* rec) {
    if (K < 2 || K != R || next_pow2(R) != R || !ff8_invert_enabled()) return false;
    for (unsigned i = 0; i < K; ++i)
        if (orig[i] || !rec[i]) return false;
    return true;
}
void fill_dec8_full(Ff8EncArgs& a, const DeviceTables* t, unsigned m, const void* const* rec, void** work,
                    uint64_t off, uint64_t bytes) {
    std::memset(&a, 0, sizeof(a));
    for (unsigned i = 0; i < m; ++i) {
        a.ptr[i] = uint64_t(reinterpret_cast<uintptr_t>(rec[i])) + off;
        a.ptr[m + i] = uint64_t(reinterpret_cast<uintptr_t>(work[i])) + off;
    }
    a.sktab = t->sktab8;
    a.fused = t->fused8 + size_t(log2u(m) - 1) * 256 * kTab8Dwords;  // encoder chunk 0 of this m
    a.K = a.R = m;
    a.nchunks = 1;
    a.nunits = uint32_t(bytes / 4);
}

LeopardResult decode_device8(Call& c, uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                             const void* const* rec, void** work) {
    const unsigned Tn = log2u(next_pow2(next_pow2(R) + K));
    if (full_loss_square(K, R, orig, rec)) {
        bool done = false;
        LeopardResult r = dense_single_bs(c, bytes, off, R, rec, work, kFormDenseDec, &done);
        if (r != Leopard_Success || done) return r;
        Ff8EncArgs e;
        for (uint64_t pos = 0; pos < bytes; pos += kFf8MaxLaunchBytes) {
            fill_dec8_full(e, c.t, R, rec, work, off + pos, std::min(kFf8MaxLaunchBytes, bytes - pos));
            HIP_OK(launch_ff8_decode_full(Tn - 1, e, c.s), "decode kernel");
        }
        return Leopard_Success;
    }
    {  // few losses of a small code: the coefficient matrix
        unsigned L = 0, N = 0;
        for (unsigned i = 0; i < R; ++i) N += rec[i] != nullptr;
        for (unsigned i = 0; i < K; ++i) (orig[i] ? N : L) += 1;
        if (use_matrix(L, N, bytes, true, true)) {
            bool done = false;
            const LeopardResult r = decode_matrix(c, bytes, off, K, R, orig, rec, work, &done);
            if (r != Leopard_Success || done) return r;
        }
    }
    // the error locator of this pattern (computed on the device once per pattern)
    uint32_t erased[8];
    erasures8(K, R, next_pow2(R), orig, rec, erased);
    c.ws->el8_begin();
    std::vector<El8Job> jobs;
    const uint32_t* el = nullptr;
    unsigned slot = 0;
    LeopardResult r = c.ws->el8_slot(erased, jobs, &el, &slot);
    if (r != Leopard_Success) return r;
    if ((r = flush_el8(*c.ws, c.t, jobs, c.s)) != Leopard_Success) return r;
    // the locator by value once the host holds it; until then the slot (and a
    // read-back of it for the calls after this one)
    uint32_t elv[kFf8Ptrs / 4];
    const bool by_value = c.ws->el8_value(slot, elv);
#ifdef LAMD_X_TRACE_MARK
    std::fprintf(stderr, "el8 slot %u state %d by_value %d\n", slot, int(c.ws->el8_state[slot]), int(by_value));
#endif
    if (!by_value) {
        c.ws->touched = true;
        if ((r = c.ws->el8_readback(slot, c.s)) != Leopard_Success) return r;
    }
    Ff8DecArgs a;
    for (uint64_t pos = 0; pos < bytes; pos += kFf8MaxLaunchBytes) {  // see encode_device
        const int mode =
            fill_dec8(a, c.t, K, R, orig, rec, work, off + pos, std::min(kFf8MaxLaunchBytes, bytes - pos), el);
        if (by_value) {
            std::memcpy(a.el_val, elv, sizeof(elv));
            a.el_by_value = 1;
        }
        HIP_OK(mode == kDec8General ? launch_ff8_decode(Tn, a, c.s)
               : mode == kDec8Split ? launch_ff8_decode_split(Tn - 1, a, c.s)
                                    : launch_ff8_decode_half(Tn - 1, a, c.s),
               "decode kernel");
    }
    return Leopard_Success;
}

// The matrix entry of `key` (L outputs x N inputs) for this call, built now by
// gen(units, rows, pitch) when new: gen runs the transform kernels on N unit
// pieces (piece j = the byte 1 at column j, `pitch` bytes each) into L rows,
// byte j of row i = M[i][j].  *out stays null when the cache is full.
template <class Gen>
LeopardResult mat_entry(Call& c, std::vector<uint32_t>&& key, unsigned L, unsigned N, Gen&& gen,
                        const MatEntry** out) {
    *out = nullptr;
    MatCache& mc = *g_mat[c.dev];
    std::lock_guard<std::mutex> lk(mc.mu);  // generation is a few launches, once per pattern
    auto it = mc.entries.find(key);
    if (it != mc.entries.end()) {
        MatEntry& e = *it->second;
        if (!e.done.load(std::memory_order_acquire)) {
            if (hipEventQuery(e.ready) == hipSuccess) e.done.store(true, std::memory_order_release);
            else HIP_OK(hipStreamWaitEvent(c.s, e.ready, 0), "wait for matrix");  // built on another stream
        }
        *out = &e;
        return Leopard_Success;
    }
    const size_t tab_bytes = (size_t(L) * N + 1) * 32;  // + one zero entry (k_ff8_mat's empty slots)
    if (mc.bytes + tab_bytes > kMatCacheBytes) return Leopard_Success;
    constexpr unsigned kPitch = kFf8Ptrs;  // >= N columns, a multiple of 64 bytes
    LeopardResult r = c.ws->reserve_device(size_t(N + L) * kPitch);
    if (r != Leopard_Success) return r;
    uint8_t* units = c.ws->dbuf;
    uint8_t* rows = units + size_t(N) * kPitch;
    HIP_OK(launch_ff8_unit(units, N, kPitch, c.s), "unit pieces");
    tls_mat_gen = true;
    r = gen(units, rows, kPitch);
    tls_mat_gen = false;
    if (r != Leopard_Success) return r;
    std::unique_ptr<MatEntry> e(new MatEntry);
    HIP_OK(pool_alloc(reinterpret_cast<void**>(&e->tabs), tab_bytes, c.dev, c.s), "allocate matrix");
    HIP_OK(launch_ff8_mat_tabs(rows, kPitch, L, N, c.t->vtab8, e->tabs, c.s), "matrix tables");
    HIP_OK(hipEventCreateWithFlags(&e->ready, kOrderEvent), "event");
    HIP_OK(hipEventRecord(e->ready, c.s), "record matrix");
    e->L = L;
    e->N = N;
    e->stream = c.s;
    mc.bytes += tab_bytes;
    *out = e.get();
    mc.entries.emplace(std::move(key), std::move(e));
    return Leopard_Success;
}

// out[i] = XOR_j M[i][j] * in[j] over columns [off, off + bytes) (one launch:
// use_matrix keeps L N bytes <= kMatMaxWork, far below 2^32 dword columns).
LeopardResult mat_apply(Call& c, const MatEntry& e, const std::vector<uint64_t>& in, const std::vector<uint64_t>& out,
                        uint64_t bytes, uint64_t off) {
    Ff8MatArgs a;
    std::memset(&a, 0, sizeof(a));
    for (unsigned j = 0; j < e.N; ++j) a.ptr[j] = in[j] + off;
    for (unsigned i = 0; i < e.L; ++i) a.ptr[e.N + i] = out[i] + off;
    a.tabs = e.tabs;
    a.N = e.N;
    a.L = e.L;
    a.nunits = uint32_t(bytes / 4);
    HIP_OK(launch_ff8_mat(a, c.t->cus, c.s), "matrix kernel");
    return Leopard_Success;
}

// Encode: recovery j = XOR_i G[j][i] * original i (G depends on K and R only).
LeopardResult encode_matrix(Call& c, uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                            void** work, bool* done) {
    *done = false;
    const MatEntry* e = nullptr;
    LeopardResult r = mat_entry(c, {0u, K, R}, R, K,
                                [&](uint8_t* units, uint8_t* rows, unsigned pitch) {
                                    std::vector<const void*> o(K);
                                    std::vector<void*> w(R);
                                    for (unsigned i = 0; i < K; ++i) o[i] = units + size_t(i) * pitch;
                                    for (unsigned j = 0; j < R; ++j) w[j] = rows + size_t(j) * pitch;
                                    return encode_device(c, pitch, 0, K, R, o.data(), w.data());
                                },
                                &e);
    if (r != Leopard_Success || !e) return r;
    std::vector<uint64_t> in(K), out(R);
    for (unsigned i = 0; i < K; ++i) in[i] = uint64_t(reinterpret_cast<uintptr_t>(orig[i]));
    for (unsigned j = 0; j < R; ++j) out[j] = uint64_t(reinterpret_cast<uintptr_t>(work[j]));
    r = mat_apply(c, *e, in, out, bytes, off);
    *done = r == Leopard_Success;
    return r;
}

// Decode of one erasure pattern: lost original i = XOR_j D[i][j] * received j,
// over every received piece (recovery pieces in index order, then originals):
// the transform decoder's own map (rs_ff8.hip kernels on unit pieces), also on
// inputs that are not codewords.
LeopardResult decode_matrix(Call& c, uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                            const void* const* rec, void** work, bool* done) {
    *done = false;
    std::vector<uint64_t> in, out;
    for (unsigned i = 0; i < R; ++i)
        if (rec[i]) in.push_back(uint64_t(reinterpret_cast<uintptr_t>(rec[i])));
    for (unsigned i = 0; i < K; ++i) {
        if (orig[i]) in.push_back(uint64_t(reinterpret_cast<uintptr_t>(orig[i])));
        else out.push_back(uint64_t(reinterpret_cast<uintptr_t>(work[i])));
    }
    const unsigned N = unsigned(in.size()), L = unsigned(out.size());
    uint32_t erased[8];
    erasures8(K, R, next_pow2(R), orig, rec, erased);
    std::vector<uint32_t> key{1u, K, R};
    key.insert(key.end(), erased, erased + 8);
    const MatEntry* e = nullptr;
    LeopardResult r = mat_entry(c, std::move(key), L, N,
                                [&](uint8_t* units, uint8_t* rows, unsigned pitch) {
                                    std::vector<const void*> ou(K), ru(R);
                                    std::vector<void*> wu(K);
                                    unsigned j = 0, l = 0;
                                    for (unsigned i = 0; i < R; ++i)
                                        ru[i] = rec[i] ? units + size_t(j++) * pitch : nullptr;
                                    for (unsigned i = 0; i < K; ++i) {
                                        ou[i] = orig[i] ? units + size_t(j++) * pitch : nullptr;
                                        wu[i] = orig[i] ? nullptr : rows + size_t(l++) * pitch;
                                    }
                                    return decode_device8(c, pitch, 0, K, R, ou.data(), ru.data(), wu.data());
                                },
                                &e);
    if (r != Leopard_Success || !e) return r;
    r = mat_apply(c, *e, in, out, bytes, off);
    *done = r == Leopard_Success;
    return r;
}

// GF(2^16) decoder state of one erasure pattern (a workspace slot): erasure
// bitmap over 65536 positions, occupancy pyramids for pruning (received data /
// lost originals), the error locator and the per-position log values of the
// scale and reveal multiplies -- uploaded and computed on the device only when
// the slot is new for this pattern.  Fills a's shape and state fields.
constexpr size_t kDec16Bitmap = 65536 / 32;
constexpr size_t kDec16OffPyr = kDec16Bitmap * 4;
constexpr size_t kDec16OffTmp = kDec16OffPyr + (2 * kPyrWords * 4 + 255) / 256 * 256;
constexpr size_t kDec16OffEl = kDec16OffTmp + 65536 * 4;
constexpr size_t kDec16OffSl = kDec16OffEl + 65536 * 4;
constexpr size_t kDec16OffRl = kDec16OffSl + 65536 * 4;
constexpr size_t kDec16Bytes = kDec16OffRl + 65536 * 4;
LeopardResult dec16_state(Call& c, unsigned K, unsigned R, const void* const* orig, const void* const* rec,
                          DecArgs& a) {
    const unsigned m = next_pow2(R);
    const unsigned n = next_pow2(m + K);
    // error_locations[] = 1 at lost recoveries, [R, m), lost originals (LeopardFF8.cpp:1825-1840)
    std::vector<uint32_t> key(2 + kDec16Bitmap, 0);
    key[0] = K;
    key[1] = R;
    uint32_t* erased = key.data() + 2;
    auto set = [&](unsigned p) { erased[p >> 5] |= 1u << (p & 31); };
    for (unsigned i = 0; i < R; ++i)
        if (!rec[i]) set(i);
    for (unsigned i = R; i < m; ++i) set(i);
    for (unsigned i = 0; i < K; ++i)
        if (!orig[i]) set(m + i);
    const unsigned words = (std::max(n, 256u) + 31) / 32;
    std::vector<uint32_t> bitmap(erased, erased + words);
    Workspace& ws = *c.ws;
    unsigned si = 0;
    bool fresh = false;
    LeopardResult r = ws.dec16_slot(key, kDec16Bytes, &si, &fresh);
    if (r != Leopard_Success) return r;
    uint8_t* st = ws.dec16[si].mem;
    if (fresh) {
        ws.dec16[si].key.clear();  // stays invalid unless the uploads and launches below succeed
        r = ws.upload(st, kDec16OffTmp, c.s, [&](uint8_t* h) {
            std::memset(h, 0, kDec16OffTmp);
            std::memcpy(h, bitmap.data(), bitmap.size() * 4);
            uint32_t* pp = reinterpret_cast<uint32_t*>(h + kDec16OffPyr);
            uint32_t* pn = pp + kPyrWords;
            auto mark = [](uint32_t* pyr, unsigned p) {
                for (unsigned L = 0; L <= 16; ++L) {
                    const unsigned j = p >> L;
                    pyr[pyr_offset(L) + (j >> 5)] |= 1u << (j & 31);
                }
            };
            for (unsigned i = 0; i < R; ++i)
                if (rec[i]) mark(pp, i);
            for (unsigned i = 0; i < K; ++i) mark(orig[i] ? pp : pn, m + i);
        });
        if (r != Leopard_Success) return r;
        HIP_OK(launch_error_locator16(reinterpret_cast<uint32_t*>(st), c.t->walsh16,
                                      reinterpret_cast<uint32_t*>(st + kDec16OffTmp),
                                      reinterpret_cast<uint32_t*>(st + kDec16OffEl),
                                      reinterpret_cast<uint32_t*>(st + kDec16OffSl),
                                      reinterpret_cast<uint32_t*>(st + kDec16OffRl), m, K, R, c.s),
               "error locator");
        ws.dec16[si].key.assign(2 + kDec16Bitmap, 0);
        ws.dec16[si].key[0] = K;
        ws.dec16[si].key[1] = R;
        std::copy(bitmap.begin(), bitmap.end(), ws.dec16[si].key.begin() + 2);
    }
    a.sktab = c.t->sktab16;
    a.tabs = c.t->tab16;
    a.zeros = c.t->zeros;
    a.walsh = c.t->walsh16;
    a.K = K;
    a.R = R;
    a.m = m;
    a.Tn = log2u(n);
    a.el = reinterpret_cast<uint32_t*>(st + kDec16OffEl);
    a.scale_logs = reinterpret_cast<uint32_t*>(st + kDec16OffSl);
    a.reveal_logs = reinterpret_cast<uint32_t*>(st + kDec16OffRl);
    a.erased_dev = reinterpret_cast<uint32_t*>(st);
    a.present_pyr = reinterpret_cast<uint32_t*>(st + kDec16OffPyr);
    a.needed_pyr = a.present_pyr + kPyrWords;
    return Leopard_Success;
}

LeopardResult decode_device(Call& c, uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                            const void* const* rec, void** work) {
    const unsigned m = next_pow2(R);
    const unsigned n = next_pow2(m + K);
    const bool ff16 = n > 256;
    const unsigned Tn = log2u(n);
    if (!ff16) return decode_device8(c, bytes, off, K, R, orig, rec, work);

    DecArgs a;
    std::memset(&a, 0, sizeof(a));
    MapBuilder mb;
    mb.build(a.orig, orig, K, off);
    mb.build(a.rec, rec, R, off);
    mb.build(a.out, work, K, off);
    Workspace& ws = *c.ws;

    // Narrow columns and n <= 2048: the two-pass narrow-strip decoder
    // (rs_ff16_small.hip), whose only intermediate is U (tiles with received data).
    const unsigned ntiles_in = (m + K + (1u << kLoBits) - 1) >> kLoBits;
    const bool narrow = g_q16_ok && decode16_small_supported(Tn) && bytes <= kNarrowColumnsMax;
    // few output tiles and pieces of at least kOnePassMinBytes (60 KiB: below
    // that the one-pass grid leaves SIMDs idle and measured slower, 32 KiB
    // 96.7 vs 87.2 us, rs_ff16_small.hip): the one-pass form (no U slab);
    // narrower calls keep the two passes, whose grids also spread over the tiles
    const bool one_pass = narrow && bytes >= kOnePassMinBytes &&
                          decode16_one_supported(((m + K - 1) >> kLoBits) - (m >> kLoBits) + 1);
    const uint64_t slab_pieces = one_pass ? 0 : narrow ? uint64_t(ntiles_in) << kLoBits : 2ull * n;  // U (+ A, multi-pass)
    const uint64_t slice = narrow ? bytes : mall_slice(bytes, slab_pieces);
    const size_t table_bytes = (mb.bytes() + 255) / 256 * 256;
    const size_t off_slab = table_bytes;
    LeopardResult r = ws.reserve_device(off_slab + slab_pieces * slice);
    if (r != Leopard_Success) return r;
    r = mb.flush(ws, reinterpret_cast<uint64_t*>(ws.dbuf), c.s);  // piece tables (if any)
    if (r != Leopard_Success) return r;
    ++ws.dec16_call;
    if ((r = dec16_state(c, K, R, orig, rec, a)) != Leopard_Success) return r;
    a.nlo = (m + K + (1u << kLoBits) - 1) >> kLoBits;
    // No original survives and n = 2m: the received pieces fill only the low half
    // (k_dec_hi_half); pass 1 then runs the recovery tiles only.
    bool any_orig = false;
    for (unsigned i = 0; i < K; ++i) any_orig |= orig[i] != nullptr;
    const bool half = !any_orig && Tn >= kLoBits + 2 && 2 * m == n && ff8_half_decoder_enabled();
    if (half) {
        a.nlo = (R + (1u << kLoBits) - 1) >> kLoBits;
        a.fused = c.t->fused16 + fused16_base(Tn - 1);
    }

    if (narrow) {
        a.nlo = ntiles_in;
        a.qlog = c.t->qlog16 + high_q16_base(Tn - kLoBits);
        a.tile0 = m >> kLoBits;
        a.nout = ((m + K - 1) >> kLoBits) - a.tile0 + 1;
        a.nunits = bytes / 8;
        if (one_pass) {  // no intermediate at all
            HIP_OK(launch_decode16_one(a, c.s), "decode");
            return Leopard_Success;
        }
        a.a_out = a.a_in = PieceMap{nullptr, ws.dbuf + off_slab, bytes, 0};
        HIP_OK(launch_decode16_small_lo(a, c.s), "decode pass 1");
        HIP_OK(launch_decode16_small_fin(a, c.s), "decode pass 2");
        return Leopard_Success;
    }
    uint8_t* A = ws.dbuf + off_slab;
    uint8_t* Uu = A + uint64_t(n) * slice;
    for (uint64_t pos = 0; pos < bytes; pos += slice) {
        const uint64_t len = std::min(slice, bytes - pos);
        DecArgs b = a;
        b.orig.off = off + pos;
        b.rec.off = off + pos;
        b.out.off = off + pos;
        b.nunits = len / 8;
        b.a_out = PieceMap{nullptr, Uu, slice, 0};
        HIP_OK(launch_decode_lo(b, c.s), "decode pass 1");
        b.a_in = PieceMap{nullptr, Uu, slice, 0};
        b.a_out = PieceMap{nullptr, A, slice, 0};
        HIP_OK(half ? launch_decode_hi_half(b, c.s) : launch_decode_hi(b, c.s), "decode pass 2");
        b.a_in = PieceMap{nullptr, A, slice, 0};
        b.b_in = PieceMap{nullptr, Uu, slice, 0};
        HIP_OK(launch_decode_fin(b, c.s), "decode pass 3");
    }
    return Leopard_Success;
}

// ---------------------------------------------------- host-memory pipeline --

// Host (pageable) pieces are the reference's contract: caller-owned buffers in,
// results in host memory on return.  The columns are cut into slices that flow
// through a two-slot ring: host threads gather one slice of every input piece
// into pinned memory, one H2D copy, the kernels, one D2H copy, host threads
// scatter the outputs.  Slot j & 1 has its own stream, so the gather of slice
// j, the copies and kernels of slice j - 1 and the scatter of slice j - 1 overlap.

// Fixed pool of host copy threads (LEO_AMD_HOST_THREADS, default min(8, cores)).
class CpuPool {
public:
    static CpuPool& get() {
        static CpuPool* pool = new CpuPool();  // never destroyed: detached workers outlive static teardown
        return *pool;
    }
    // fn(i) for every i in [0, count), on the workers and the calling thread.
    void run(unsigned count, const std::function<void(unsigned)>& fn) {
        if (workers_ == 0 || count <= 1) {
            for (unsigned i = 0; i < count; ++i) fn(i);
            return;
        }
        std::lock_guard<std::mutex> call(call_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            count_ = count;
            next_.store(0);
            busy_ = workers_;
            ++gen_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return busy_ == 0; });
        fn_ = nullptr;
    }

private:
    CpuPool() {
        unsigned n = std::min(8u, std::max(1u, std::thread::hardware_concurrency()));
        if (const char* e = std::getenv("LEO_AMD_HOST_THREADS")) n = unsigned(std::max(1, std::atoi(e)));
        workers_ = n - 1;
        for (unsigned i = 0; i < workers_; ++i) std::thread([this] { loop(); }).detach();
    }
    void drain() {
        for (unsigned i = next_.fetch_add(1); i < count_; i = next_.fetch_add(1)) (*fn_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
            }
            drain();
            std::lock_guard<std::mutex> lk(mu_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* fn_ = nullptr;
    unsigned count_ = 0, workers_ = 0, busy_ = 0;
    std::atomic<unsigned> next_{0};
    uint64_t gen_ = 0;
};

struct CopyJob {
    uint8_t* dst;
    const uint8_t* src;
    uint64_t len;
};

// Copy with non-temporal stores: the staging copies move every byte once and
// neither side is read again soon, so streaming stores skip the read-for-
// ownership of each destination line (a third of the memory traffic of a
// cached copy) and leave the caches alone.  AVX2 when the CPU has it.
__attribute__((target("avx2"))) void copy_stream_avx2(uint8_t* dst, const uint8_t* src, uint64_t n) {
    const uint64_t head = std::min<uint64_t>(n, (32 - (reinterpret_cast<uintptr_t>(dst) & 31)) & 31);
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    uint64_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
        const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
    }
    std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();  // the streamed lines are visible before the copy engine or the caller reads them
}
void copy_stream(uint8_t* dst, const uint8_t* src, uint64_t n) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2 && n >= 4096) copy_stream_avx2(dst, src, n);
    else std::memcpy(dst, src, n);
}

// Copy of every job, split into <= 1 MiB parts spread over the pool.
void parallel_copy(const std::vector<CopyJob>& jobs) {
    constexpr uint64_t kPart = 1 << 20;
    std::vector<CopyJob> parts;
    for (const CopyJob& j : jobs)
        for (uint64_t o = 0; o < j.len; o += kPart) parts.push_back({j.dst + o, j.src + o, std::min(kPart, j.len - o)});
    CpuPool::get().run(unsigned(parts.size()), [&](unsigned i) { copy_stream(parts[i].dst, parts[i].src, parts[i].len); });
}

// Device work for one slice: inputs are rows [0, nin) of `din`, outputs rows
// [0, nout) of `dout`, row stride `stride`, `len` bytes per row.
using SliceFn = std::function<LeopardResult(Call&, uint64_t len, uint8_t* din, uint8_t* dout, uint64_t stride)>;

constexpr int kDefaultPipeMode = 0;

// Bytes per ring slot (inputs + outputs of one slice); LEO_AMD_SLOT_MB overrides.
uint64_t pipe_slot_budget() {
    static const uint64_t v = [] {
        const char* e = std::getenv("LEO_AMD_SLOT_MB");
        const long mb = e ? std::atol(e) : 32;
        return uint64_t(std::max(1L, mb)) << 20;
    }();
    return v;
}

// How a ring slot reaches the kernels (LEO_AMD_PIPE_MODE, read once):
//   0  SDMA: H2D copy of the inputs, kernels on device memory, D2H copy of the outputs;
//   1  SDMA H2D of the inputs; the kernels write the outputs straight into the
//      pinned slot over PCIe (no D2H copy: kernel stores reach ~53 GB/s, the
//      D2H SDMA engine ~30);
//   2  the kernels read the inputs from and write the outputs to the pinned slot
//      over PCIe (no SDMA copies at all).
int pipe_mode() {
#if LAMD_EXPERIMENT_ENV
    static const int v = [] {
        const char* e = std::getenv("LEO_AMD_PIPE_MODE");
        return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : kDefaultPipeMode;
    }();
    return v;
#else
    return kDefaultPipeMode;
#endif
}

// Pieces that follow each other at one stride (rows of one caller array): a
// run is one copy (1-D when the stride is the piece length, else 2-D).
struct HostRun {
    uint64_t first, count, stride;
};
constexpr uint64_t kRunMaxGap = 1ull << 20;  // bytes between two rows of one run
template <class P>
std::vector<HostRun> host_runs(const std::vector<P>& v, uint64_t bytes) {
    std::vector<HostRun> runs;
    for (uint64_t i = 0; i < v.size(); ++i) {
        if (!runs.empty()) {
            HostRun& b = runs.back();
            const uint8_t* prev = v[i - 1];
            const uint8_t* cur = v[i];
            if (cur > prev) {
                const uint64_t d = uint64_t(cur - prev);
                // a run's first pair sets its stride: only pitches that leave a
                // small gap (rows of one array, or of a wider one) start a run,
                // never two unrelated allocations far apart
                if (d >= bytes && (b.count == 1 ? d - bytes <= kRunMaxGap : d == b.stride)) {
                    b.stride = d;
                    ++b.count;
                    continue;
                }
            }
        }
        runs.push_back({i, 1, bytes});
    }
    return runs;
}
constexpr size_t kDirectMaxRuns = 16;                 // more runs: the gather / scatter ring
constexpr uint64_t kDirectMaxBytes = 8ull << 30;      // device rows of one direct call
constexpr uint64_t kDirectKeepBytes = 256ull << 20;   // direct rows kept for the next call (larger: freed)
// Column slices of a direct call, one stream each (<= 4).  Measured on the
// pageable 128+128 x 64 KiB encode: 4 slices 16.1-16.6 GB/s, 1 slice 22.4-22.5
// (512+512: 22.3-22.5 vs 24.2-24.5, profiles/r04_v9/host.txt): the strided 2-D
// copies of a slice move less per SDMA command than one whole-row copy, and the
// copy engines, not the overlap, bound the call.  One slice stays the default.
#ifndef LAMD_DIRECT_SLICES
#define LAMD_DIRECT_SLICES 1
#endif
constexpr unsigned kDirectSlices = LAMD_DIRECT_SLICES;
static_assert(kDirectSlices >= 1 && kDirectSlices <= 4, "one stream per slice: the call's and three side streams");
constexpr uint64_t kDirectSliceMinBytes = 4ull << 20;  // smaller calls: one slice

// Host pieces that form a few row runs (the usual caller layout: pieces are
// rows of one or a few arrays) go straight between the caller's pageable
// memory and device rows by SDMA, one copy per run: no host copies at all.
// The copy engines read and write pageable memory at the PCIe rate (53 GB/s
// each way, profiles/r03_v2/hostcopy.txt), where the gather / scatter ring is
// bound by host memcpy.  Returns Leopard_Success with *done = false when the
// layout does not qualify.
LeopardResult run_host_direct(Call& c, uint64_t bytes, const std::vector<const uint8_t*>& hin,
                              const std::vector<uint8_t*>& hout, const SliceFn& fn, bool* done) {
    *done = false;
    const uint64_t nin = hin.size(), nout = hout.size(), rows = nin + nout;
    if (rows * bytes > kDirectMaxBytes) return Leopard_Success;
    const std::vector<HostRun> rin = host_runs(hin, bytes), rout = host_runs(hout, bytes);
    if (rin.size() + rout.size() > kDirectMaxRuns) return Leopard_Success;
    Workspace& ws = *c.ws;
    LeopardResult r = ws.reserve_direct(rows * bytes);
    if (r != Leopard_Success) {  // no room for the rows: the ring (bounded slots) does the call
        (void)hipGetLastError();
        tls.last_error.clear();
        return Leopard_Success;
    }
    uint8_t* din = ws.direct;
    uint8_t* dout = ws.direct + nin * bytes;
    // Column slices, slice j on its own stream: upload, kernels, download.  One
    // slice's upload then overlaps an earlier slice's kernels and download
    // (PCIe carries both directions at once), where a single slice runs
    // upload -> kernels -> download back to back.  The downloads are enqueued
    // after every upload (a pageable download may hold the enqueueing thread).
    const unsigned nsl = rows * bytes >= kDirectSliceMinBytes && bytes >= 4096 * kDirectSlices ? kDirectSlices : 1;
    const uint64_t sw = nsl == 1 ? bytes : ((bytes + nsl - 1) / nsl + 63) / 64 * 64;  // slice width
    std::vector<Call> cj(nsl, c);
    if (nsl > 1) {
        for (hipEvent_t& e : ws.side_ev)
            if (!e) HIP_OK(hipEventCreateWithFlags(&e, kOrderEvent), "event");
        HIP_OK(hipEventRecord(ws.side_ev[0], c.s), "record direct rows");  // the rows' allocation and earlier work
        for (unsigned j = 1; j < nsl; ++j) {
            hipStream_t& st = ws.side[j - 1];
            if (!st) HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
            HIP_OK(hipStreamWaitEvent(st, ws.side_ev[0], 0), "order side stream");
        }
    }
    for (unsigned j = 0; j < nsl; ++j) {
        if (j > 0) {
            cj[j].s = ws.side[j - 1];
            cj[j].ws = &workspace(c.dev, cj[j].s);  // scratch of its own (GF(2^16) intermediates)
        }
        const uint64_t o = uint64_t(j) * sw, len = std::min(sw, bytes - o);
        for (const HostRun& run : rin) {
            uint8_t* dst = din + run.first * bytes + o;
            if (nsl == 1 && run.stride == bytes)
                HIP_OK(hipMemcpyAsync(dst, hin[run.first], run.count * bytes, hipMemcpyHostToDevice, cj[j].s),
                       "upload rows");
            else
                HIP_OK(hipMemcpy2DAsync(dst, bytes, hin[run.first] + o, run.stride, len, run.count,
                                        hipMemcpyHostToDevice, cj[j].s),
                       "upload rows");
        }
        if ((r = fn(cj[j], len, din + o, dout + o, bytes)) != Leopard_Success) return r;
        HIP_OK(hipGetLastError(), "kernel launch");
        if (j > 0 && (r = cj[j].ws->mark_use(cj[j].s)) != Leopard_Success) return r;
    }
    for (unsigned j = 0; j < nsl; ++j) {
        const uint64_t o = uint64_t(j) * sw, len = std::min(sw, bytes - o);
        for (const HostRun& run : rout) {
            const uint8_t* src = dout + run.first * bytes + o;
            if (nsl == 1 && run.stride == bytes)
                HIP_OK(hipMemcpyAsync(hout[run.first], src, run.count * bytes, hipMemcpyDeviceToHost, cj[j].s),
                       "download rows");
            else
                HIP_OK(hipMemcpy2DAsync(hout[run.first] + o, run.stride, src, bytes, len, run.count,
                                        hipMemcpyDeviceToHost, cj[j].s),
                       "download rows");
        }
    }
    for (unsigned j = 1; j < nsl; ++j) {  // the call's stream waits for every slice
        HIP_OK(hipEventRecord(ws.side_ev[j], cj[j].s), "record slice");
        HIP_OK(hipStreamWaitEvent(c.s, ws.side_ev[j], 0), "join slice");
    }
    if (ws.direct_size > kDirectKeepBytes) {  // large rows do not stay with the thread: freed after this call's copies
        HIP_OK(hipFreeAsync(ws.direct, c.s), "free direct rows");
        ws.direct = nullptr;
        ws.direct_size = 0;
    }
    *done = true;
    return Leopard_Success;
}

// hin: host input pieces (call offset applied); hout: host output pieces.
// Slot j & 1 runs on its own stream with its own scratch (per-stream workspaces).
LeopardResult run_host_pipeline(Call& c, uint64_t bytes, const std::vector<const uint8_t*>& hin,
                                const std::vector<uint8_t*>& hout, const SliceFn& fn) {
    bool direct = false;
    LeopardResult r = run_host_direct(c, bytes, hin, hout, fn, &direct);
    if (r != Leopard_Success || direct) return r;
    const uint64_t nin = hin.size(), nout = hout.size(), rows = nin + nout;
    uint64_t slice = bytes;
    if (rows * bytes > pipe_slot_budget())  // >= 4 KiB slices even when that outgrows the budget
        slice = std::max<uint64_t>(pipe_slot_budget() / rows / 64 * 64, std::min<uint64_t>(bytes, 4096));
    if (rows * bytes > (4ull << 20)) slice = std::min<uint64_t>(slice, (bytes / 4 + 63) / 64 * 64);  // >= 4 slices
    const uint64_t in_bytes = nin * slice, slot = rows * slice;
    r = c.ws->reserve_ring(slot);
    if (r != Leopard_Success) return r;
    Workspace& ws = *c.ws;
    const unsigned nslices = unsigned((bytes + slice - 1) / slice);
    const int mode = pipe_mode();
    auto len_of = [&](unsigned j) { return std::min(slice, bytes - uint64_t(j) * slice); };
    auto scatter = [&](unsigned j) -> LeopardResult {
        const unsigned s = j & 1;
        HIP_OK(hipEventSynchronize(ws.out_done[s]), "wait slice output");
        const uint8_t* pin = ws.ring_host + s * ws.slot_bytes + in_bytes;
        std::vector<CopyJob> jobs;
        for (uint64_t i = 0; i < nout; ++i) jobs.push_back({hout[i] + uint64_t(j) * slice, pin + i * slice, len_of(j)});
        parallel_copy(jobs);
        return Leopard_Success;
    };
    for (unsigned j = 0; j < nslices; ++j) {
        const unsigned s = j & 1;
        uint8_t* pin = ws.ring_host + s * ws.slot_bytes;
        uint8_t* dev = ws.ring_dev + s * ws.slot_bytes;
        const uint64_t pos = uint64_t(j) * slice, len = len_of(j);
        if (j >= 2) HIP_OK(hipEventSynchronize(ws.in_done[s]), "wait slot input");
        std::vector<CopyJob> jobs;
        for (uint64_t i = 0; i < nin; ++i) jobs.push_back({pin + i * slice, hin[i] + pos, len});
        parallel_copy(jobs);
        Call cs = c;
        cs.s = ws.pipe_stream[s];
        cs.ws = &workspace(c.dev, cs.s);  // GF(2^16) scratch must not be shared between the two streams
        uint8_t* mapped = ws.ring_host_dev + s * ws.slot_bytes;  // the pinned slot as the kernels see it
        if (mode != 2) {
            HIP_OK(hipMemcpyAsync(dev, pin, in_bytes, hipMemcpyHostToDevice, cs.s), "slice upload");
            HIP_OK(hipEventRecord(ws.in_done[s], cs.s), "record upload");
        }
        r = mode == 0 ? fn(cs, len, dev, dev + in_bytes, slice)
            : mode == 1 ? fn(cs, len, dev, mapped + in_bytes, slice)
                        : fn(cs, len, mapped, mapped + in_bytes, slice);
        if (r != Leopard_Success) return r;
        HIP_OK(hipGetLastError(), "kernel launch");
        if ((r = cs.ws->mark_use(cs.s)) != Leopard_Success) return r;
        if (mode == 0)
            HIP_OK(hipMemcpyAsync(pin + in_bytes, dev + in_bytes, nout * slice, hipMemcpyDeviceToHost, cs.s),
                   "slice download");
        if (mode == 2) HIP_OK(hipEventRecord(ws.in_done[s], cs.s), "record input use");  // kernels read the slot
        HIP_OK(hipEventRecord(ws.out_done[s], cs.s), "record download");
        if (j >= 1 && (r = scatter(j - 1)) != Leopard_Success) return r;
    }
    return scatter(nslices - 1);
}

// ------------------------------------------------ registered host memory --

// Caller-registered host memory (leo_amd_register_host): pinned and mapped
// into every device's address space, so kernels read the caller's pieces and
// write the results in place over PCIe -- no staging copies.  The caller keeps
// a registered range alive until it unregisters it (the contract of
// hipHostRegister / RDMA memory registration).
struct HostReg {
    uintptr_t base;
    uint64_t size;
    uintptr_t dbase;  // device address of base
};
std::mutex g_reg_mu;
std::map<uintptr_t, HostReg> g_regs;

// Device addresses of ptrs[i] + [off, off + bytes) when every non-null piece
// lies in one registered range; else false.
bool map_registered(const void* const* ptrs, unsigned count, uint64_t off, uint64_t bytes, std::vector<void*>& out) {
    out.assign(count, nullptr);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    if (g_regs.empty()) return false;
    for (unsigned i = 0; i < count; ++i) {
        if (!ptrs[i]) continue;
        const uintptr_t p = reinterpret_cast<uintptr_t>(ptrs[i]);
        auto it = g_regs.upper_bound(p);
        if (it == g_regs.begin()) return false;
        --it;
        const HostReg& r = it->second;
        if (p + off + bytes > r.base + r.size) return false;
        out[i] = reinterpret_cast<void*>(r.dbase + (p - r.base));
    }
    return true;
}

// ------------------------------------------------------ multi-GPU fan-out --

// A host-memory call (the reference's contract: caller-owned host buffers)
// can split its columns over several GPUs, each staging or reading its range
// over its own PCIe link.  Range i runs on device
// i % device_count on fan-out worker i, a persistent thread that keeps its own
// per-device workspaces; the call returns when every range is done.
class FanoutPool {
public:
    static FanoutPool& get() {
        static FanoutPool* pool = new FanoutPool();  // never destroyed (detached workers)
        return *pool;
    }
    void run(unsigned n, const std::function<void(unsigned)>& fn) {
        std::lock_guard<std::mutex> call(call_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            while (workers_ < n) {
                const unsigned id = workers_++;
                const uint64_t seen = gen_;
                std::thread([this, id, seen] { loop(id, seen); }).detach();
            }
            fn_ = &fn;
            n_ = n;
            pending_ = n;
            ++gen_;
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return pending_ == 0; });
        fn_ = nullptr;
    }

private:
    void loop(unsigned id, uint64_t seen) {
        for (;;) {
            const std::function<void(unsigned)>* fn = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (id >= n_) continue;
                fn = fn_;
            }
            (*fn)(id);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_all();
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* fn_ = nullptr;
    unsigned workers_ = 0, n_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
};

// Ranges a host-memory call of `bytes` columns is split into: the thread's
// leo_amd_set_fanout value, else LEO_AMD_FANOUT (default 1; -1 = every
// device), at most one range per 4 KiB of columns.
unsigned fanout_ranges(uint64_t bytes) {
    static const int env = [] {
        const char* e = std::getenv("LEO_AMD_FANOUT");
        return e ? std::atoi(e) : 1;
    }();
    int n = tls.fanout != 0 ? tls.fanout : env;
    if (n < 0) n = std::max(1, g_device_count);
    const uint64_t cap = std::max<uint64_t>(1, bytes / 4096);
    return unsigned(std::min<uint64_t>(std::max(n, 1), cap));
}

// fn(len, off) for each of n 64-byte-aligned column ranges of [0, bytes), one
// per fan-out worker; returns the first failure (its error text moves to the
// calling thread).
LeopardResult fanout(unsigned n, uint64_t bytes, const std::function<LeopardResult(uint64_t, uint64_t)>& fn) {
    const uint64_t blocks = bytes / 64;
    std::vector<LeopardResult> res(n, Leopard_Success);
    std::vector<std::string> err(n);
    const int ndev = std::max(1, g_device_count);
    FanoutPool::get().run(n, [&](unsigned i) {
        const uint64_t b0 = blocks * i / n, b1 = blocks * (i + 1) / n;
        tls.device = int(i % unsigned(ndev));
        tls.stream = nullptr;
        tls.async = false;
        tls.fanout_worker = true;
        res[i] = b1 > b0 ? fn((b1 - b0) * 64, b0 * 64) : Leopard_Success;
        if (res[i] != Leopard_Success) err[i] = tls.last_error;
    });
    for (unsigned i = 0; i < n; ++i)
        if (res[i] != Leopard_Success) {
            tls.last_error = err[i];
            return res[i];
        }
    return Leopard_Success;
}

LeopardResult encode_any(uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig, void** work);
LeopardResult decode_any(uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                         const void* const* rec, void** work);

int pick_device(const void* first, MemKind* kind) {
    int dev = -1;
    *kind = classify(first, &dev);
    if (*kind == MemKind::Device) return dev;
    if (tls.device >= 0) return tls.device;
    int cur = 0;
    (void)hipGetDevice(&cur);
    return cur;
}

// A NULL destination for a piece the call must write (recovery piece j < R on
// encode, the work piece of a lost original on decode).  The reference would
// write through it (leopard.cpp:123-344 validates only the arrays); here it is
// Leopard_InvalidInput, decided where the work is done: per column range on
// the fan-out workers, whose failure then reaches the caller.
LeopardResult missing_output(void* const* outs, unsigned count, const void* const* lost_if) {
    for (unsigned i = 0; i < count; ++i)
        if (!outs[i] && (!lost_if || !lost_if[i])) {
            char buf[96];
            std::snprintf(buf, sizeof(buf), "work_data[%u] is NULL but the call writes it", i);
            tls.last_error = buf;
            return Leopard_InvalidInput;
        }
    return Leopard_Success;
}

LeopardResult encode_any(uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig, void** work) {
    MemKind kind;
    const int dev = pick_device(orig[0], &kind);
    DeviceGuard guard(dev);
    Call c;
    LeopardResult r = begin_call(dev, c);
    if (r != Leopard_Success) return r;

    if (kind == MemKind::Device) {
        if ((r = missing_output(work, R, nullptr)) != Leopard_Success) return r;
        if (K == 1) {  // leopard.cpp:144-149
            for (unsigned i = 0; i < R; ++i)
                HIP_OK(hipMemcpyAsync(static_cast<uint8_t*>(work[i]) + off, static_cast<const uint8_t*>(orig[i]) + off,
                                      bytes, hipMemcpyDeviceToDevice, c.s),
                       "copy");
        } else if (R == 1) {  // leopard.cpp:152-160
            r = xor_device(c, bytes, off, orig, K, work[0]);
        } else {
            r = encode_device(c, bytes, off, K, R, orig, work);
        }
        if (r != Leopard_Success) return r;
        return finish(c, false);
    }

    // host memory (leopard.cpp:143-149: K == 1 is a copy)
    if (K == 1) {
        if ((r = missing_output(work, R, nullptr)) != Leopard_Success) return r;
        std::vector<CopyJob> jobs;
        for (unsigned i = 0; i < R; ++i)
            jobs.push_back({static_cast<uint8_t*>(work[i]) + off, static_cast<const uint8_t*>(orig[i]) + off, bytes});
        parallel_copy(jobs);
        return Leopard_Success;
    }
    if (!tls.fanout_worker) {  // columns over several GPUs
        const unsigned nr = fanout_ranges(bytes);
        if (nr > 1)
            return fanout(nr, bytes, [&](uint64_t len, uint64_t o) { return encode_any(len, off + o, K, R, orig, work); });
    }
    if ((r = missing_output(work, R, nullptr)) != Leopard_Success) return r;
    // Device work of one column slice staged as dense rows: inputs = the K
    // originals, outputs = the R recovery pieces.
    const SliceFn slice_fn = [&](Call& cs, uint64_t len, uint8_t* din, uint8_t* dout, uint64_t stride) {
        std::vector<const void*> di(K);
        std::vector<void*> dw(R);
        for (unsigned i = 0; i < K; ++i) di[i] = din + i * stride;
        for (unsigned i = 0; i < R; ++i) dw[i] = dout + i * stride;
        if (R == 1) return xor_device(cs, len, 0, di.data(), K, dw[0]);
        return encode_device(cs, len, 0, K, R, di.data(), dw.data());
    };
    {  // caller-registered host memory: the kernels run on it in place
        std::vector<void*> di, dw;
        if (map_registered(orig, K, off, bytes, di) && map_registered(work, R, off, bytes, dw)) {
            r = R == 1 ? xor_device(c, bytes, off, const_cast<const void* const*>(di.data()), K, dw[0])
                       : encode_device(c, bytes, off, K, R, const_cast<const void* const*>(di.data()), dw.data());
            if (r != Leopard_Success) return r;
            return finish(c, true);
        }
    }
    std::vector<const uint8_t*> hin(K);
    std::vector<uint8_t*> hout(R);
    for (unsigned i = 0; i < K; ++i) hin[i] = static_cast<const uint8_t*>(orig[i]) + off;
    for (unsigned i = 0; i < R; ++i) hout[i] = static_cast<uint8_t*>(work[i]) + off;
    r = run_host_pipeline(c, bytes, hin, hout, slice_fn);
    if (r != Leopard_Success) return r;
    return finish(c, true);
}

LeopardResult decode_any(uint64_t bytes, uint64_t off, unsigned K, unsigned R, const void* const* orig,
                         const void* const* rec, void** work) {
    unsigned lost = 0, lost_i = 0, got = 0, got_i = 0;
    for (unsigned i = 0; i < K; ++i)
        if (!orig[i]) { ++lost; lost_i = i; }
    for (unsigned i = 0; i < R; ++i)
        if (rec[i]) { ++got; got_i = i; }
    if (got < lost) return Leopard_NeedMoreData;  // leopard.cpp:275-276

    const void* first = nullptr;
    for (unsigned i = 0; i < K && !first; ++i) first = orig[i];
    for (unsigned i = 0; i < R && !first; ++i) first = rec[i];
    if (!first) first = work[0];
    MemKind kind;
    const int dev = pick_device(first, &kind);
    DeviceGuard guard(dev);
    Call c;
    LeopardResult r = begin_call(dev, c);
    if (r != Leopard_Success) return r;

    // K == 1 copies recovery_data[last received] (leopard.cpp:279-283); with no
    // recovery received the reference would read NULL, we copy the original.
    const void* k1_src = K == 1 ? (rec[got_i] ? rec[got_i] : orig[0]) : nullptr;

    if (kind == MemKind::Device) {
        if ((r = missing_output(work, K == 1 ? 1 : K, K == 1 || lost == 0 ? nullptr : orig)) != Leopard_Success)
            return r;
        if (K == 1) {  // leopard.cpp:279-283
            HIP_OK(hipMemcpyAsync(static_cast<uint8_t*>(work[0]) + off, static_cast<const uint8_t*>(k1_src) + off,
                                  bytes, hipMemcpyDeviceToDevice, c.s),
                   "copy");
        } else if (lost == 0) {  // leopard.cpp:286-291
            for (unsigned i = 0; i < K; ++i)
                HIP_OK(hipMemcpyAsync(static_cast<uint8_t*>(work[i]) + off, static_cast<const uint8_t*>(orig[i]) + off,
                                      bytes, hipMemcpyDeviceToDevice, c.s),
                       "copy");
        } else if (R == 1) {  // leopard.cpp:294-303
            std::vector<const void*> src;
            src.push_back(rec[0]);
            for (unsigned i = 0; i < K; ++i)
                if (orig[i]) src.push_back(orig[i]);
            r = xor_device(c, bytes, off, src.data(), unsigned(src.size()), work[lost_i]);
        } else {
            r = decode_device(c, bytes, off, K, R, orig, rec, work);
        }
        if (r != Leopard_Success) return r;
        return finish(c, false);
    }

    // host memory: K == 1 and zero loss are copies (leopard.cpp:279-291)
    if (K == 1 || lost == 0) {
        if ((r = missing_output(work, K == 1 ? 1 : K, nullptr)) != Leopard_Success) return r;
        std::vector<CopyJob> jobs;
        if (K == 1) jobs.push_back({static_cast<uint8_t*>(work[0]) + off, static_cast<const uint8_t*>(k1_src) + off, bytes});
        else
            for (unsigned i = 0; i < K; ++i)
                jobs.push_back({static_cast<uint8_t*>(work[i]) + off, static_cast<const uint8_t*>(orig[i]) + off, bytes});
        parallel_copy(jobs);
        return Leopard_Success;
    }
    if (!tls.fanout_worker) {  // columns over several GPUs
        const unsigned nr = fanout_ranges(bytes);
        if (nr > 1)
            return fanout(nr, bytes,
                          [&](uint64_t len, uint64_t o) { return decode_any(len, off + o, K, R, orig, rec, work); });
    }
    if ((r = missing_output(work, K, orig)) != Leopard_Success) return r;
    // Device work of one column slice staged as dense rows: inputs = received
    // recoveries, then received originals (so the R == 1 XOR sources form one
    // slab); outputs = lost originals in order.
    std::vector<int> in_row_rec(R, -1), in_row_orig(K, -1), out_row(K, -1);
    int nin = 0, nout = 0;
    for (unsigned i = 0; i < R; ++i)
        if (rec[i]) in_row_rec[i] = nin++;
    for (unsigned i = 0; i < K; ++i) {
        if (orig[i]) in_row_orig[i] = nin++;
        else out_row[i] = nout++;
    }
    const SliceFn slice_fn = [&](Call& cs, uint64_t len, uint8_t* din, uint8_t* dout, uint64_t stride) {
        if (R == 1) {  // leopard.cpp:294-303
            std::vector<const void*> src;
            for (int j = 0; j < nin; ++j) src.push_back(din + j * stride);
            return xor_device(cs, len, 0, src.data(), unsigned(src.size()), dout);
        }
        std::vector<const void*> dorig(K, nullptr), drec(R, nullptr);
        std::vector<void*> dwork(K, nullptr);
        for (unsigned i = 0; i < R; ++i)
            if (in_row_rec[i] >= 0) drec[i] = din + in_row_rec[i] * stride;
        for (unsigned i = 0; i < K; ++i) {
            if (in_row_orig[i] >= 0) dorig[i] = din + in_row_orig[i] * stride;
            else dwork[i] = dout + out_row[i] * stride;
        }
        return decode_device(cs, len, 0, K, R, dorig.data(), drec.data(), dwork.data());
    };
    {  // caller-registered host memory: the kernels run on it in place
        std::vector<void*> dorig, drec, dwork;
        std::vector<const void*> wl(K, nullptr);  // only the work pieces of lost originals are written
        for (unsigned i = 0; i < K; ++i)
            if (!orig[i]) wl[i] = work[i];
        if (map_registered(orig, K, off, bytes, dorig) && map_registered(rec, R, off, bytes, drec) &&
            map_registered(wl.data(), K, off, bytes, dwork)) {
            if (R == 1) {  // leopard.cpp:294-303
                std::vector<const void*> src;
                src.push_back(drec[0]);
                for (unsigned i = 0; i < K; ++i)
                    if (orig[i]) src.push_back(dorig[i]);
                r = xor_device(c, bytes, off, src.data(), unsigned(src.size()), dwork[lost_i]);
            } else {
                r = decode_device(c, bytes, off, K, R, const_cast<const void* const*>(dorig.data()),
                                  const_cast<const void* const*>(drec.data()), dwork.data());
            }
            if (r != Leopard_Success) return r;
            return finish(c, true);
        }
    }
    std::vector<const uint8_t*> hin;
    std::vector<uint8_t*> hout;
    for (unsigned i = 0; i < R; ++i)
        if (rec[i]) hin.push_back(static_cast<const uint8_t*>(rec[i]) + off);
    for (unsigned i = 0; i < K; ++i) {
        if (orig[i]) hin.push_back(static_cast<const uint8_t*>(orig[i]) + off);
        else hout.push_back(static_cast<uint8_t*>(work[i]) + off);
    }
    r = run_host_pipeline(c, bytes, hin, hout, slice_fn);
    if (r != Leopard_Success) return r;
    return finish(c, true);
}

// Validation shared by leo_encode / leo_amd_encode_slice (leopard.cpp:131-140, 162-166).
LeopardResult check_encode(uint64_t bytes, unsigned K, unsigned R, unsigned work_count, const void* const* orig,
                           void** work) {
    if (bytes == 0 || bytes % 64 != 0) return Leopard_InvalidSize;
    if (R == 0 || R > K) return Leopard_InvalidCounts;
    if (!orig || !work) return Leopard_InvalidInput;
    if (!g_initialized) return Leopard_CallInitialize;
    if (K == 1 || R == 1) return Leopard_Success;
    const unsigned m = next_pow2(R);
    const unsigned n = next_pow2(m + K);
    if (work_count != m * 2) return Leopard_InvalidCounts;
    if (n > 65536) return Leopard_TooMuchData;
    return Leopard_Success;
}

// leopard.cpp:242-252, 305-309 (NeedMoreData is decided later, after counting).
LeopardResult check_decode(uint64_t bytes, unsigned K, unsigned R, unsigned work_count, const void* const* orig,
                           const void* const* rec, void** work) {
    if (bytes == 0 || bytes % 64 != 0) return Leopard_InvalidSize;
    if (R == 0 || R > K) return Leopard_InvalidCounts;
    if (!orig || !rec || !work) return Leopard_InvalidInput;
    if (!g_initialized) return Leopard_CallInitialize;
    return Leopard_Success;
}

LeopardResult decode_checked(uint64_t bytes, uint64_t off, unsigned K, unsigned R, unsigned work_count,
                             const void* const* orig, const void* const* rec, void** work) {
    // the general path needs work_count == n (leopard.cpp:305-309); edge paths do not
    unsigned lost = 0, got = 0;
    for (unsigned i = 0; i < K; ++i) lost += orig[i] == nullptr;
    for (unsigned i = 0; i < R; ++i) got += rec[i] != nullptr;
    if (got < lost) return Leopard_NeedMoreData;
    if (K != 1 && lost != 0 && R != 1) {
        const unsigned m = next_pow2(R);
        const unsigned n = next_pow2(m + K);
        if (work_count != n) return Leopard_InvalidCounts;
        if (n > 65536) return Leopard_TooMuchData;
    }
    return decode_any(bytes, off, K, R, orig, rec, work);
}

// ------------------------------------------------------------- batches ----

// leo_amd_encode_batch / leo_amd_decode_batch: `count` independent objects of
// one shape, each with exactly the semantics of one leo_encode / leo_decode.
// Device-resident GF(2^8) objects on one device run as ONE launch over every
// object's column strips (argument blocks uploaded through the staging ring),
// so a batch of small objects fills the GPU where a single 64 KiB-piece call
// gives each CU one workgroup; anything else runs object by object.
//
// The one-launch path is taken only when every piece the kernel touches (every
// input read and every output written, of every object) lies in device memory
// of that one device.  Pieces are checked against the allocation ranges
// already seen (hipMemGetAddressRange), so a slab-laid object costs two range
// checks and a batch a handful of runtime queries.
struct RangeCache {
    struct Range {
        uintptr_t lo, hi;
        int dev;
    };
    std::vector<Range> seen;
    // [p, p + len) inside one device allocation of device dev
    bool on(const void* p, uint64_t len, int dev) {
        if (!p) return false;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        for (const Range& x : seen)
            if (a >= x.lo && a < x.hi) return x.dev == dev && a + len <= x.hi;
        int d = -1;
        if (classify(p, &d) != MemKind::Device) return false;
        void* base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        const uintptr_t lo = reinterpret_cast<uintptr_t>(base);
        seen.push_back({lo, lo + size, d});
        return d == dev && a + len <= lo + size;
    }
    // every non-null piece of p[0, n)
    bool all_on(const void* const* p, unsigned n, uint64_t len, int dev) {
        for (unsigned i = 0; i < n; ++i)
            if (p[i] && !on(p[i], len, dev)) return false;
        return true;
    }
};

// Pieces p[0, n) equally spaced (a slab) with a stride that fits a signed
// 32-bit integer (Ff8SlabBatch): base and stride (two's complement).
bool slab_of(const void* const* p, unsigned n, uint64_t& base, int32_t& stride) {
    base = uint64_t(reinterpret_cast<uintptr_t>(p[0]));
    const int64_t s = n > 1 ? int64_t(uint64_t(reinterpret_cast<uintptr_t>(p[1])) - base) : 0;
    if (s < INT32_MIN || s > INT32_MAX) return false;
    stride = int32_t(s);
    for (unsigned i = 0; i < n; ++i)
        if (!p[i] || uint64_t(reinterpret_cast<uintptr_t>(p[i])) != base + uint64_t(int64_t(i) * s)) return false;
    return true;
}
// the bytes a slab of n pieces of `len` bytes spans, inside one allocation of dev
bool slab_on(RangeCache& rc, uint64_t base, int32_t stride, unsigned n, uint64_t len, int dev) {
    const int64_t span = int64_t(n - 1) * stride;
    const uint64_t lo = base + uint64_t(std::min<int64_t>(0, span));
    const uint64_t hi = base + uint64_t(std::max<int64_t>(0, span)) + len;
    return rc.on(reinterpret_cast<const void*>(uintptr_t(lo)), hi - lo, dev);
}

// Batch of objects whose `nin` inputs and `nout` outputs are slabs on device
// dev: launches of up to kSlabObjs objects with every argument by value (no
// upload in front of the kernel).  Returns false (nothing launched) when some
// object is not slab-laid there.
bool run_slab_batch8(int dev, RangeCache& rc, unsigned count, uint64_t bytes, unsigned T, unsigned K, unsigned R,
                     unsigned nin, unsigned nout, const void* const* const* ins, void* const* const* outs, bool multi,
                     int form, LeopardResult* res) {
    std::vector<uint64_t> ib(count), ob(count);
    std::vector<int32_t> is(count), os(count);
    for (unsigned o = 0; o < count; ++o)
        if (!slab_of(ins[o], nin, ib[o], is[o]) ||
            !slab_of(const_cast<const void* const*>(outs[o]), nout, ob[o], os[o]) ||
            !slab_on(rc, ib[o], is[o], nin, bytes, dev) || !slab_on(rc, ob[o], os[o], nout, bytes, dev))
            return false;
    *res = [&]() -> LeopardResult {
        DeviceGuard guard(dev);
        Call c;
        LeopardResult r = begin_call(dev, c);
        if (r != Leopard_Success) return r;
        const unsigned m = next_pow2(R);
        Ff8SlabBatch b;
        std::memset(&b, 0, sizeof(b));
        b.sktab = c.t->sktab8;
        b.fused = c.t->fused8 + size_t(T - 1) * 256 * kTab8Dwords;
        b.K = K;
        b.R = R;
        b.nchunks = (K + m - 1) / m;
        b.nunits = uint32_t(bytes / 4);
        for (unsigned o0 = 0; o0 < count; o0 += kSlabObjs) {
            const unsigned n = std::min(kSlabObjs, count - o0);
            for (unsigned j = 0; j < n; ++j) {
                b.in_base[j] = ib[o0 + j];
                b.in_stride[j] = is[o0 + j];
                b.out_base[j] = ob[o0 + j];
                b.out_stride[j] = os[o0 + j];
            }
            uint32_t *q = nullptr, *qclear = nullptr;
            if (form != kFormGeneral && !multi && ff8_bs_supported(T, K, R, b.nchunks) &&
                (r = c.ws->bs_queue(&q, &qclear)) != Leopard_Success)
                return r;
            HIP_OK(launch_ff8_encode_slab(T, b, n, multi, form, c.s, c.t->cus, q, qclear), "slab batch kernel");
        }
        return finish(c, false);
    }();
    return true;
}

// prep(c): work enqueued on the call's stream ahead of the batch kernel.
template <class Args, class Fill, class Launch, class Prep>
LeopardResult run_batch8(int dev, unsigned count, Fill fill, Launch launch, Prep prep) {
    DeviceGuard guard(dev);
    Call c;
    LeopardResult r = begin_call(dev, c);
    if (r != Leopard_Success) return r;
    if ((r = prep(c)) != Leopard_Success) return r;
    const size_t bytes = size_t(count) * sizeof(Args);
    r = c.ws->reserve_device(bytes);
    if (r != Leopard_Success) return r;
    Args* dargs = reinterpret_cast<Args*>(c.ws->dbuf);
    int kind = INT32_MAX;  // the least specialised kind over the objects
    r = c.ws->upload(dargs, bytes, c.s, [&](uint8_t* h) {
        Args* ha = reinterpret_cast<Args*>(h);
        for (unsigned o = 0; o < count; ++o) kind = std::min(kind, fill(ha[o], c.t, o));
    });
    if (r != Leopard_Success) return r;
    HIP_OK(launch(dargs, kind, c.s), "batch kernel");
    return finish(c, false);
}
template <class Args, class Fill, class Launch>
LeopardResult run_batch8(int dev, unsigned count, Fill fill, Launch launch) {
    return run_batch8<Args>(dev, count, fill, launch, [](Call&) { return Leopard_Success; });
}
// objects (erasure patterns: one error-locator slot each) per batched GF(2^8) decode launch
constexpr unsigned kDecBatchChunk = Workspace::kEl8Slots / 2;

// GF(2^16) batches on narrow strips (pieces <= 256 KiB): the encoder for
// m = 128, 256 (k_enc16n) and the two-pass decoder for n <= 2048 run one grid
// per kernel over every object (blockIdx.y / .z = object, argument blocks
// uploaded through the staging ring), so a batch of small objects fills the
// GPU where one call of 2560-byte pieces is 20 column strips.
bool narrow_encode16(unsigned K, unsigned R, uint64_t bytes) {
    const unsigned m = next_pow2(R), n = next_pow2(m + K);
    return K > 1 && R > 1 && n > 256 && encode16_small_supported(log2u(m)) && bytes <= kNarrowColumnsMax;
}
bool narrow_decode16(unsigned K, unsigned R, uint64_t bytes) {
    const unsigned m = next_pow2(R), n = next_pow2(m + K);
    return n > 256 && g_q16_ok && decode16_small_supported(log2u(n)) && bytes <= kNarrowColumnsMax;
}

LeopardResult encode_batch16(int dev, unsigned count, uint64_t bytes, unsigned K, unsigned R,
                             const void* const* const* orig, void** const* work) {
    DeviceGuard guard(dev);
    Call c;
    LeopardResult r = begin_call(dev, c);
    if (r != Leopard_Success) return r;
    const unsigned m = next_pow2(R), Tm = log2u(m);
    std::vector<EncArgs> args(count);  // sized up front: mb keeps pointers to the maps
    MapBuilder mb;
    for (unsigned o = 0; o < count; ++o) {
        EncArgs& a = args[o];
        std::memset(&a, 0, sizeof(a));
        mb.build(a.in, orig[o], K, 0);
        mb.build(a.out, work[o], R, 0);
        a.sktab = c.t->sktab16;
        a.tabs = c.t->tab16;
        a.zeros = c.t->zeros;
        a.fused = c.t->fused16 + fused16_base(Tm);
        a.K = K;
        a.R = R;
        a.Tm = Tm;
        a.nchunks = (K + m - 1) / m;
        a.nunits = bytes / 8;
    }
    const size_t table_bytes = (mb.bytes() + 255) / 256 * 256;
    if ((r = c.ws->reserve_device(table_bytes + count * sizeof(EncArgs))) != Leopard_Success) return r;
    if ((r = mb.flush(*c.ws, reinterpret_cast<uint64_t*>(c.ws->dbuf), c.s)) != Leopard_Success) return r;
    EncArgs* dargs = reinterpret_cast<EncArgs*>(c.ws->dbuf + table_bytes);
    if ((r = c.ws->upload(dargs, args.data(), count * sizeof(EncArgs), c.s)) != Leopard_Success) return r;
    HIP_OK(launch_encode16_small_batch(Tm, dargs, count, bytes / 8, c.s), "batch encode kernel");
    return finish(c, false);
}

// Decoder: objects in chunks of kDec16Slots (each object's erasure pattern
// holds a decoder-state slot for the chunk).  At most kDecOneNZ output tiles:
// the one-pass kernel over every object of a chunk in one grid (no
// intermediate).  Otherwise the two passes with a U slab per object, at most
// kBatch16SlabBytes of slabs a chunk, and only for pieces under
// kOnePassMinBytes (larger pieces decode object by object).
constexpr uint64_t kBatch16SlabBytes = 256ull << 20;
// One-pass batch when its grid (16-unit strips x objects) gives every CU at
// least kBatch16OneWgsPerCu workgroups; below that the two-pass form's grids
// (one workgroup per strip and tile) keep more SIMDs busy (16 objects of
// 2560-byte pieces: 9.56 vs 8.07 us per object, profiles/r05_v2).
// LEO_AMD_DEC16_BATCH_ONE=0/1 forces either form in experiment builds.
constexpr uint64_t kBatch16OneWgsPerCu = 4;
bool batch16_one_pass(unsigned count, uint64_t bytes, unsigned cus) {
#if LAMD_EXPERIMENT_ENV
    static const int force = [] {
        const char* e = std::getenv("LEO_AMD_DEC16_BATCH_ONE");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    if (force >= 0) return force == 1;
#endif
    const uint64_t wgs = (bytes / 8 + 15) / 16 * count;
    return wgs >= kBatch16OneWgsPerCu * cus;
}
LeopardResult decode_batch16(int dev, unsigned count, uint64_t bytes, unsigned K, unsigned R,
                             const void* const* const* orig, const void* const* const* rec, void** const* work) {
    DeviceGuard guard(dev);
    Call c;
    LeopardResult r = begin_call(dev, c);
    if (r != Leopard_Success) return r;
    Workspace& ws = *c.ws;
    const unsigned m = next_pow2(R), n = next_pow2(m + K), Tn = log2u(n);
    const unsigned ntiles_in = (m + K + (1u << kLoBits) - 1) >> kLoBits;
    const unsigned tile0 = m >> kLoBits, nout = ((m + K - 1) >> kLoBits) - tile0 + 1;
    // one pass (round 5): no U slab, one grid (strips, objects); two passes otherwise
    const bool one = decode16_one_supported(nout) && batch16_one_pass(count, bytes, c.t->cus);
    const uint64_t slab = one ? 0 : (uint64_t(ntiles_in) << kLoBits) * bytes;  // U of one object
    const unsigned per_chunk =
        one ? Workspace::kDec16Slots
            : unsigned(std::max<uint64_t>(1, std::min<uint64_t>(Workspace::kDec16Slots, kBatch16SlabBytes / slab)));
    for (unsigned o0 = 0; o0 < count; o0 += per_chunk) {
        const unsigned nb = std::min(per_chunk, count - o0);
        ++ws.dec16_call;
        std::vector<DecArgs> args(nb);
        MapBuilder mb;
        for (unsigned o = 0; o < nb; ++o) {
            DecArgs& a = args[o];
            std::memset(&a, 0, sizeof(a));
            mb.build(a.orig, orig[o0 + o], K, 0);
            mb.build(a.rec, rec[o0 + o], R, 0);
            mb.build(a.out, work[o0 + o], K, 0);
            if ((r = dec16_state(c, K, R, orig[o0 + o], rec[o0 + o], a)) != Leopard_Success) return r;
            a.nlo = ntiles_in;
            a.qlog = c.t->qlog16 + high_q16_base(Tn - kLoBits);
            a.tile0 = tile0;
            a.nout = nout;
            a.nunits = bytes / 8;
        }
        const size_t table_bytes = (mb.bytes() + 255) / 256 * 256;
        const size_t args_bytes = (nb * sizeof(DecArgs) + 255) / 256 * 256;
        if ((r = ws.reserve_device(table_bytes + args_bytes + nb * slab)) != Leopard_Success) return r;
        if ((r = mb.flush(ws, reinterpret_cast<uint64_t*>(ws.dbuf), c.s)) != Leopard_Success) return r;
        for (unsigned o = 0; o < nb; ++o)
            args[o].a_out = args[o].a_in = PieceMap{nullptr, ws.dbuf + table_bytes + args_bytes + o * slab, bytes, 0};
        DecArgs* dargs = reinterpret_cast<DecArgs*>(ws.dbuf + table_bytes);
        if ((r = ws.upload(dargs, args.data(), nb * sizeof(DecArgs), c.s)) != Leopard_Success) return r;
        if (one)
            HIP_OK(launch_decode16_one_batch(dargs, nb, bytes / 8, c.s), "batch decode kernel");
        else
            HIP_OK(launch_decode16_small_batch(dargs, nb, bytes / 8, ntiles_in, nout, c.s), "batch decode kernels");
    }
    return finish(c, false);
}

LeopardResult encode_batch(unsigned count, uint64_t bytes, unsigned K, unsigned R, unsigned work_count,
                           const void* const* const* orig, void** const* work) {
    if (!orig || !work) return Leopard_InvalidInput;
    for (unsigned o = 0; o < count; ++o) {
        LeopardResult r = check_encode(bytes, K, R, work_count, orig[o], work[o]);
        if (r != Leopard_Success) return r;
        // every recovery piece is written (the one-launch path stores through each)
        if ((r = missing_output(work[o], R, nullptr)) != Leopard_Success) return r;
    }
    if (count == 0) return Leopard_Success;
    const unsigned m = next_pow2(R), n = next_pow2(m + K);
    MemKind kind = MemKind::Host;
    const int dev = K > 1 && R > 1 && n <= 256 && bytes <= kFf8MaxLaunchBytes ? pick_device(orig[0][0], &kind) : -1;
    if (kind == MemKind::Device) {
        const unsigned Tm = log2u(m);
        const bool multi = (K + m - 1) / m > 1;
        const int form = K == m && R == m ? kFormDenseEnc : kFormGeneral;
        RangeCache rc;
        LeopardResult res;
        if (run_slab_batch8(dev, rc, count, bytes, Tm, K, R, K, R, orig, work, multi, form, &res)) return res;
        bool on_dev = true;
        for (unsigned o = 0; o < count && on_dev; ++o)
            on_dev = rc.all_on(orig[o], K, bytes, dev) && rc.all_on(const_cast<const void* const*>(work[o]), R, bytes, dev);
        if (on_dev)
            return run_batch8<Ff8EncArgs>(
                dev, count,
                [&](Ff8EncArgs& a, const DeviceTables* t, unsigned o) {
                    fill_enc8(a, t, K, R, orig[o], work[o], 0, bytes);
                    return 0;
                },
                [&](const Ff8EncArgs* d, int, hipStream_t s) {
                    return launch_ff8_encode_batch(Tm, d, count, uint32_t(bytes / 4), multi, form, s);
                });
    }
    if (narrow_encode16(K, R, bytes)) {
        MemKind k16 = MemKind::Host;
        const int d16 = pick_device(orig[0][0], &k16);
        if (k16 == MemKind::Device) {
            RangeCache rc;
            bool on_dev = true;
            for (unsigned o = 0; o < count && on_dev; ++o)
                on_dev = rc.all_on(orig[o], K, bytes, d16) &&
                         rc.all_on(const_cast<const void* const*>(work[o]), R, bytes, d16);
            if (on_dev) return encode_batch16(d16, count, bytes, K, R, orig, work);
        }
    }
    for (unsigned o = 0; o < count; ++o) {
        const LeopardResult r = encode_any(bytes, 0, K, R, orig[o], work[o]);
        if (r != Leopard_Success) return r;
    }
    return Leopard_Success;
}

LeopardResult decode_batch(unsigned count, uint64_t bytes, unsigned K, unsigned R, unsigned work_count,
                           const void* const* const* orig, const void* const* const* rec, void** const* work) {
    if (!orig || !rec || !work) return Leopard_InvalidInput;
    bool general = true;  // every object takes the general decoder (no edge path)
    for (unsigned o = 0; o < count; ++o) {
        LeopardResult r = check_decode(bytes, K, R, work_count, orig[o], rec[o], work[o]);
        if (r != Leopard_Success) return r;
        unsigned lost = 0, got = 0;
        for (unsigned i = 0; i < K; ++i) lost += orig[o][i] == nullptr;
        for (unsigned i = 0; i < R; ++i) got += rec[o][i] != nullptr;
        if (got < lost) return Leopard_NeedMoreData;
        if (K == 1 || lost == 0 || R == 1) {
            general = false;
        } else {
            const unsigned n = next_pow2(next_pow2(R) + K);
            if (work_count != n) return Leopard_InvalidCounts;
            if (n > 65536) return Leopard_TooMuchData;
        }
    }
    if (count == 0) return Leopard_Success;
    const unsigned m = next_pow2(R), n = next_pow2(m + K);
    MemKind kind = MemKind::Host;
    int dev = -1;
    if (general && n <= 256 && bytes <= kFf8MaxLaunchBytes) {
        const void* first = nullptr;  // the device rule of decode_any
        for (unsigned i = 0; i < K && !first; ++i) first = orig[0][i];
        for (unsigned i = 0; i < R && !first; ++i) first = rec[0][i];
        dev = pick_device(first, &kind);
    }
    if (kind == MemKind::Device) {
        const unsigned Tn = log2u(n);
        bool full = true;  // every object a full loss of a K = R = m code: the inverse encoder tile
        for (unsigned o = 0; o < count && full; ++o) full = full_loss_square(K, R, orig[o], rec[o]);
        RangeCache rc;
        LeopardResult res;
        if (full && run_slab_batch8(dev, rc, count, bytes, Tn - 1, m, m, m, m, rec, work, false, kFormDenseDec, &res))
            return res;
        // inputs: received originals and recoveries; outputs: the work pieces of lost originals
        bool on_dev = true;
        for (unsigned o = 0; o < count && on_dev; ++o) {
            on_dev = rc.all_on(orig[o], K, bytes, dev) && rc.all_on(rec[o], R, bytes, dev);
            for (unsigned i = 0; i < K && on_dev; ++i)
                if (!orig[o][i]) on_dev = rc.on(work[o][i], bytes, dev);
        }
        if (on_dev && full)
            return run_batch8<Ff8EncArgs>(
                dev, count,
                [&](Ff8EncArgs& a, const DeviceTables* t, unsigned o) {
                    fill_dec8_full(a, t, m, rec[o], work[o], 0, bytes);
                    return 0;
                },
                [&](const Ff8EncArgs* d, int, hipStream_t s) {
                    return launch_ff8_encode_batch(Tn - 1, d, count, uint32_t(bytes / 4), false, kFormDenseDec, s);
                });
        if (on_dev) {
            for (unsigned o0 = 0; o0 < count; o0 += kDecBatchChunk) {
                const unsigned nb = std::min(kDecBatchChunk, count - o0);
                std::vector<const uint32_t*> els(nb);
                const LeopardResult r = run_batch8<Ff8DecArgs>(
                    dev, nb,
                    [&](Ff8DecArgs& a, const DeviceTables* t, unsigned o) {
                        return fill_dec8(a, t, K, R, orig[o0 + o], rec[o0 + o], work[o0 + o], 0, bytes, els[o]);
                    },
                    [&](const Ff8DecArgs* d, int mode, hipStream_t s) {
                        return launch_ff8_decode_batch(mode != kDec8General ? Tn - 1 : Tn, d, nb, uint32_t(bytes / 4),
                                                       mode, s);
                    },
                    [&](Call& c) -> LeopardResult {  // the error locators of the new patterns, one launch
                        c.ws->el8_begin();
                        c.ws->touched = true;  // the batch's kernels read the slots
                        std::vector<El8Job> jobs;
                        for (unsigned o = 0; o < nb; ++o) {
                            uint32_t erased[8];
                            erasures8(K, R, m, orig[o0 + o], rec[o0 + o], erased);
                            const LeopardResult re = c.ws->el8_slot(erased, jobs, &els[o]);
                            if (re != Leopard_Success) return re;
                        }
                        return flush_el8(*c.ws, c.t, jobs, c.s);
                    });
                if (r != Leopard_Success) return r;
            }
            return Leopard_Success;
        }
    }
    if (general && narrow_decode16(K, R, bytes)) {
        const void* first = nullptr;  // the device rule of decode_any
        for (unsigned i = 0; i < K && !first; ++i) first = orig[0][i];
        for (unsigned i = 0; i < R && !first; ++i) first = rec[0][i];
        MemKind k16 = MemKind::Host;
        const int d16 = pick_device(first, &k16);
        if (k16 == MemKind::Device) {
            RangeCache rc;
            bool on_dev = true;
            for (unsigned o = 0; o < count && on_dev; ++o) {
                on_dev = rc.all_on(orig[o], K, bytes, d16) && rc.all_on(rec[o], R, bytes, d16);
                for (unsigned i = 0; i < K && on_dev; ++i)
                    if (!orig[o][i]) on_dev = rc.on(work[o][i], bytes, d16);
            }
            const unsigned m16 = next_pow2(R);
            const unsigned nout16 = ((m16 + K - 1) >> kLoBits) - (m16 >> kLoBits) + 1;
            DeviceTables* t16 = nullptr;
            if (on_dev) {
                const LeopardResult rt = ensure_device(d16, &t16);
                if (rt != Leopard_Success) return rt;
            }
            // the two-pass batch keeps a U slab per object: only for pieces under
            // kOnePassMinBytes, where a single object does not fill the GPU
            if (on_dev && ((decode16_one_supported(nout16) && batch16_one_pass(count, bytes, t16->cus)) ||
                           bytes < kOnePassMinBytes))
                return decode_batch16(d16, count, bytes, K, R, orig, rec, work);
        }
    }
    for (unsigned o = 0; o < count; ++o) {
        const LeopardResult r = decode_any(bytes, 0, K, R, orig[o], rec[o], work[o]);
        if (r != Leopard_Success) return r;
    }
    return Leopard_Success;
}

}  // namespace
}  // namespace lamd

using namespace lamd;

extern "C" {

LEO_EXPORT int leo_init_(int version) {
    if (version != LEO_VERSION) return Leopard_InvalidInput;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_initialized) return Leopard_Success;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        tls.last_error = "no HIP device visible";
        return Leopard_Platform;
    }
    for (int d = 0; d < count; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) != hipSuccess) return Leopard_Platform;
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            tls.last_error = std::string("unsupported GPU architecture ") + prop.gcnArchName;
            return Leopard_Platform;
        }
    }
    const GaloisField& f8 = field8();
    const GaloisField& f16 = field16();
    build_perm_tables8(f8, g_h_tab8);
    g_h_vtab8.assign(256 * kTab8Dwords, 0u);  // entry v = the table of log_of[v]; entry 0 stays zero
    for (unsigned v = 1; v < 256; ++v)
        std::copy_n(g_h_tab8.begin() + size_t(f8.log_of[v]) * kTab8Dwords, kTab8Dwords,
                    g_h_vtab8.begin() + size_t(v) * kTab8Dwords);
    build_perm_tables16(f16, g_h_tab16);
    build_skew_tables(f8, g_h_tab8, kTab8Dwords, kSkewFlagDw8, g_h_sktab8);
    build_skew_tables(f16, g_h_tab16, kTab16Dwords, kSkewFlagDw16, g_h_sktab16);
    build_fused_top_tables8(f8, g_h_tab8, g_h_fused8);
    build_fused_top_logs16(f16, g_h_fused16);
    g_h_walsh8.assign(f8.log_walsh.begin(), f8.log_walsh.end());
    g_h_walsh16.assign(f16.log_walsh.begin(), f16.log_walsh.end());
    g_q16_ok = build_high_q16(f16, g_h_qlog16);
    g_dev.assign(count, DeviceTables{});
    g_mat.clear();
    for (int i = 0; i < count; ++i) g_mat.emplace_back(new MatCache);
    g_device_count = count;
    g_initialized = true;
    std::atexit([] { g_exiting.store(true); });  // after the runtime's own registration: runs before its teardown
    return Leopard_Success;
}

LEO_EXPORT const char* leo_result_string(LeopardResult result) {
    switch (result) {
        case Leopard_Success: return "Operation succeeded";
        case Leopard_NeedMoreData: return "Not enough recovery data received";
        case Leopard_TooMuchData: return "Buffer counts are too high";
        case Leopard_InvalidSize: return "Buffer size must be a multiple of 64 bytes";
        case Leopard_InvalidCounts: return "Invalid counts provided";
        case Leopard_InvalidInput: return "A function parameter was invalid";
        case Leopard_Platform: return "Platform is unsupported";
        case Leopard_CallInitialize: return "Call leo_init() first";
    }
    return "Unknown";
}

LEO_EXPORT unsigned leo_encode_work_count(unsigned original_count, unsigned recovery_count) {
    if (original_count == 1) return recovery_count;
    if (recovery_count == 1) return 1;
    return next_pow2(recovery_count) * 2;
}

LEO_EXPORT unsigned leo_decode_work_count(unsigned original_count, unsigned recovery_count) {
    if (original_count == 1 || recovery_count == 1) return original_count;
    const unsigned m = next_pow2(recovery_count);
    return next_pow2(m + original_count);
}

LEO_EXPORT LeopardResult leo_encode(uint64_t buffer_bytes, unsigned original_count, unsigned recovery_count,
                                    unsigned work_count, const void* const* const original_data, void** work_data) {
    LeopardResult r = check_encode(buffer_bytes, original_count, recovery_count, work_count, original_data, work_data);
    if (r != Leopard_Success) return r;
    return encode_any(buffer_bytes, 0, original_count, recovery_count, original_data, work_data);
}

LEO_EXPORT LeopardResult leo_decode(uint64_t buffer_bytes, unsigned original_count, unsigned recovery_count,
                                    unsigned work_count, const void* const* const original_data,
                                    const void* const* const recovery_data, void** work_data) {
    LeopardResult r = check_decode(buffer_bytes, original_count, recovery_count, work_count, original_data,
                                   recovery_data, work_data);
    if (r != Leopard_Success) return r;
    return decode_checked(buffer_bytes, 0, original_count, recovery_count, work_count, original_data, recovery_data,
                          work_data);
}

LEO_EXPORT LeopardResult leo_amd_encode_slice(uint64_t buffer_bytes, uint64_t byte_offset, uint64_t slice_bytes,
                                              unsigned original_count, unsigned recovery_count, unsigned work_count,
                                              const void* const* const original_data, void** work_data) {
    if (slice_bytes == 0 || slice_bytes % 64 || byte_offset % 64 || byte_offset + slice_bytes > buffer_bytes)
        return Leopard_InvalidSize;
    LeopardResult r = check_encode(buffer_bytes, original_count, recovery_count, work_count, original_data, work_data);
    if (r != Leopard_Success) return r;
    return encode_any(slice_bytes, byte_offset, original_count, recovery_count, original_data, work_data);
}

LEO_EXPORT LeopardResult leo_amd_decode_slice(uint64_t buffer_bytes, uint64_t byte_offset, uint64_t slice_bytes,
                                              unsigned original_count, unsigned recovery_count, unsigned work_count,
                                              const void* const* const original_data,
                                              const void* const* const recovery_data, void** work_data) {
    if (slice_bytes == 0 || slice_bytes % 64 || byte_offset % 64 || byte_offset + slice_bytes > buffer_bytes)
        return Leopard_InvalidSize;
    LeopardResult r = check_decode(buffer_bytes, original_count, recovery_count, work_count, original_data,
                                   recovery_data, work_data);
    if (r != Leopard_Success) return r;
    return decode_checked(slice_bytes, byte_offset, original_count, recovery_count, work_count, original_data,
                          recovery_data, work_data);
}

LEO_EXPORT LeopardResult leo_amd_encode_batch(unsigned object_count, uint64_t buffer_bytes, unsigned original_count,
                                              unsigned recovery_count, unsigned work_count,
                                              const void* const* const* original_data, void** const* work_data) {
    return encode_batch(object_count, buffer_bytes, original_count, recovery_count, work_count, original_data,
                        work_data);
}

LEO_EXPORT LeopardResult leo_amd_decode_batch(unsigned object_count, uint64_t buffer_bytes, unsigned original_count,
                                              unsigned recovery_count, unsigned work_count,
                                              const void* const* const* original_data,
                                              const void* const* const* recovery_data, void** const* work_data) {
    return decode_batch(object_count, buffer_bytes, original_count, recovery_count, work_count, original_data,
                        recovery_data, work_data);
}

LEO_EXPORT LeopardResult leo_amd_register_host(void* ptr, uint64_t bytes) {
    if (!ptr || bytes == 0) return Leopard_InvalidInput;
    hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) {
        set_error("hipHostRegister", e);
        return Leopard_Platform;
    }
    void* d = nullptr;
    e = hipHostGetDevicePointer(&d, ptr, 0);
    if (e != hipSuccess) {
        set_error("hipHostGetDevicePointer", e);
        (void)hipHostUnregister(ptr);
        return Leopard_Platform;
    }
    std::lock_guard<std::mutex> lk(g_reg_mu);
    const uintptr_t b = reinterpret_cast<uintptr_t>(ptr);
    g_regs[b] = HostReg{b, bytes, reinterpret_cast<uintptr_t>(d)};
    return Leopard_Success;
}

LEO_EXPORT LeopardResult leo_amd_unregister_host(void* ptr) {
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        if (g_regs.erase(reinterpret_cast<uintptr_t>(ptr)) == 0) return Leopard_InvalidInput;
    }
    const hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) {
        set_error("hipHostUnregister", e);
        return Leopard_Platform;
    }
    return Leopard_Success;
}

LEO_EXPORT void leo_amd_set_stream(void* hip_stream) { tls.stream = static_cast<hipStream_t>(hip_stream); }
LEO_EXPORT void leo_amd_set_async(int async_enable) { tls.async = async_enable != 0; }
LEO_EXPORT void leo_amd_set_device(int device) { tls.device = device; }
LEO_EXPORT void leo_amd_set_fanout(int ranges) { tls.fanout = ranges; }
LEO_EXPORT void leo_amd_release_stream(void* hip_stream) {
    release_workspaces(static_cast<hipStream_t>(hip_stream), hip_stream == reinterpret_cast<void*>(intptr_t(-1)));
}

LEO_EXPORT int leo_amd_device_count(void) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return count;
}

LEO_EXPORT int leo_amd_table(int field, int which, uint16_t* out, unsigned capacity) {
    if ((field != 8 && field != 16) || which < 0 || which > 3 || !out) return Leopard_InvalidInput;
    const GaloisField& f = field == 8 ? field8() : field16();
    const std::vector<uint16_t>& v = which == 0 ? f.log_of : which == 1 ? f.exp_of : which == 2 ? f.skew : f.log_walsh;
    std::memcpy(out, v.data(), std::min<size_t>(capacity, v.size()) * sizeof(uint16_t));
    return int(v.size());
}

LEO_EXPORT const char* leo_amd_last_error(void) { return tls.last_error.c_str(); }

}  // extern "C"
