// rs_args.h -- kernel argument blocks shared by the host dispatcher and kernels.
#pragma once

#include <cstdint>

#include "rs_device.h"

namespace lamd {

// Tile bits of the "low" passes of a multi-pass FF16 transform (2^8 pieces per
// workgroup tile; the remaining high bits form the second tile).
constexpr unsigned kLoBits = 8;

// Occupancy pyramid over 65536 codeword positions: level L (0..16) has one bit
// per aligned block of 2^L positions, set when any position in the block is set.
// Level L starts at word pyr_offset(L).
__host__ __device__ inline unsigned pyr_offset(unsigned L) { return L <= 12 ? 4096u - (4096u >> L) : 4095u + (L - 12); }
constexpr unsigned kPyrWords = 4100;

struct EncArgs {
    PieceMap in;        // originals (K)
    PieceMap out;       // recovery destinations (R)
    PieceMap slab_in;   // multi-pass intermediate read
    PieceMap slab_out;  // multi-pass intermediate write
    const uint32_t* sktab;  // butterfly tables indexed by skew position (gf_tables.h)
    const uint32_t* tabs;   // multiply tables by log value; entry kModulus+1 is all zero
    const uint8_t* zeros;   // >= 256 zero bytes
    const uint32_t* fused;  // FF16: fused top-layer table index per chunk of this m (gf_tables.h)
    unsigned K, R, Tm, nchunks;
    uint64_t nunits;  // column units in this launch
};

struct DecArgs {
    PieceMap orig, rec, out;
    PieceMap a_in, b_in, a_out;  // multi-pass intermediates (FF16 decode: U, A)
    const uint32_t* sktab;
    const uint32_t* tabs;
    const uint8_t* zeros;
    const uint32_t* walsh;  // FF16 LogWalsh
    const uint32_t* present_pyr;  // FF16: "any received data" pyramid over positions
    const uint32_t* needed_pyr;   // FF16: "any lost original" pyramid over positions
    const uint32_t* el;          // FF16: precomputed error locator logs
    const uint32_t* erased_dev;  // FF16: erasure bitmap over positions [0, n)
    const uint32_t* fused;       // FF16 half-position pass 2: fused top-layer table index of this m
    const uint32_t* scale_logs;  // FF16: log value of the scale multiply per position (65536 = zero table)
    const uint32_t* reveal_logs; // FF16: log value of the reveal multiply per position
    unsigned K, R, m, Tn, nlo;   // nlo: number of non-zero low tiles
    uint64_t nunits;
    // narrow-strip decoder (n <= 2048, rs_ff16_small.hip): the high part of the
    // transform as the matrix q[t ^ t'] over 256-position tiles (gf_tables.h:
    // build_high_q16), and the tiles holding originals [tile0, tile0 + nout)
    const uint32_t* qlog;
    unsigned tile0, nout;
};

// GF(2^8) kernels (codeword length n <= 256).  Everything a launch needs travels
// by value in the kernel arguments (< 4 KiB), so a wave's prologue is one batch
// of scalar loads with no pointer-chasing or branching on piece maps.
constexpr unsigned kFf8Ptrs = 256;
struct Ff8EncArgs {
    uint64_t ptr[kFf8Ptrs];  // [0, K) originals, [K, K + R) recovery outputs (launch's column base applied)
    const uint32_t* sktab;   // skew-indexed butterfly tables, 8 dwords per entry
    const uint32_t* fused;   // fused top-layer tables of this m, entry c for chunk c (8 dwords)
    unsigned K, R, nchunks;
    uint32_t nunits;         // dword columns per piece in this launch
    __host__ __device__ uint64_t piece(unsigned i) const { return ptr[i]; }
    static constexpr bool kSlab = false;
    __host__ __device__ uint64_t in_piece(unsigned i) const { return ptr[i]; }       // i < K
    __host__ __device__ uint64_t out_piece(unsigned j) const { return ptr[K + j]; }  // j < R
};
// Batches whose objects keep their pieces in slabs (piece i at base + i *
// stride, the usual layout of a caller's buffer): the whole batch travels by
// value in the kernel arguments -- no argument upload in front of the launch.
// Encoder tile view (Ff8SlabView): pieces [0, K) = in slab, [K, K + R) = out slab.
// Strides are signed 32-bit (the host falls back to pointer tables otherwise):
// a piece address is one 32 x 32 -> 64-bit scalar multiply and a 64-bit add.
constexpr unsigned kSlabObjs = 64;
struct Ff8SlabBatch {
    uint64_t in_base[kSlabObjs], out_base[kSlabObjs];  // column base of the launch applied
    int32_t in_stride[kSlabObjs], out_stride[kSlabObjs];
    const uint32_t* sktab;
    const uint32_t* fused;
    unsigned K, R, nchunks;
    uint32_t nunits;
};
// One object of a slab batch with the interface of Ff8EncArgs (rs_ff8.hip: ff8_enc).
struct Ff8SlabView {
    uint64_t in_base, out_base;
    int32_t in_stride, out_stride;
    const uint32_t* sktab;
    const uint32_t* fused;
    unsigned K, R, nchunks;
    uint32_t nunits;
    __host__ __device__ Ff8SlabView(const Ff8SlabBatch& b, unsigned o)
        : in_base(b.in_base[o]), out_base(b.out_base[o]), in_stride(b.in_stride[o]), out_stride(b.out_stride[o]),
          sktab(b.sktab), fused(b.fused), K(b.K), R(b.R), nchunks(b.nchunks), nunits(b.nunits) {}
    static constexpr bool kSlab = true;  // piece i + 1 = piece i + stride
    __host__ __device__ uint64_t piece(unsigned i) const { return i < K ? in_piece(i) : out_piece(i - K); }
    __host__ __device__ uint64_t in_piece(unsigned i) const { return in_base + uint64_t(int64_t(i) * in_stride); }
    __host__ __device__ uint64_t out_piece(unsigned j) const { return out_base + uint64_t(int64_t(j) * out_stride); }
};
struct Ff8DecArgs {
    uint64_t ptr[kFf8Ptrs];        // position p: received piece / output of a lost original / 0
    uint32_t present[kPyr8Words];  // pyramid of received positions (Pyr8Live)
    uint32_t needed[kPyr8Words];   // pyramid of lost originals
    const uint32_t* el;            // error locator of this pattern, one byte per position (k_el8's output)
    uint32_t el_val[kFf8Ptrs / 4]; // the same bytes by value (el_by_value): a single call whose pattern's
    uint32_t el_by_value;          //   locator the host already holds reads no workspace memory
    const uint32_t* sktab;
    const uint32_t* tabs;          // multiply tables by log value; entry 256 is all zero
    const uint32_t* fused;         // k_ff8_dec_half: fused top-layer table of this m (= encoder chunk 0's)
    unsigned K, R, m;
    uint32_t nunits;
    uint32_t dense;                // half decoder with K = R = m, every recovery received (host-side dispatch)
    __host__ __device__ uint64_t piece(unsigned i) const { return ptr[i]; }
};
// GF(2^8) codes applied as their coefficient matrix (rs_ff8_mat.hip): output
// i = XOR_j M[i][j] * input j, for L <= kFf8MatMaxOut outputs and N inputs
// (N + L <= kFf8Ptrs); tabs: L x N byte-permute multiply tables, 8 dwords per
// entry (FF8::Tab in dwords 0-4), row-major by output, then one all-zero entry.
constexpr unsigned kFf8MatMaxOut = 32;
struct Ff8MatArgs {
    uint64_t ptr[kFf8Ptrs];  // [0, N) inputs, [N, N + L) outputs (column base applied)
    const uint32_t* tabs;
    unsigned N, L;
    uint32_t nunits;         // dword columns in this launch
};
// GF(2^8) error locators of up to kEl8Jobs erasure patterns in one launch
// (k_el8): job i writes the 256 el bytes of bitmap erased (LeopardFF8.cpp:
// 1825-1840) to out + 64 * slot dwords.
constexpr unsigned kEl8Jobs = 64;
struct El8Job {
    uint32_t erased[kFf8Ptrs / 32];
    uint32_t slot;
};
struct El8Args {
    El8Job job[kEl8Jobs];
    const uint32_t* walsh;  // LogWalsh (256 entries)
    uint32_t* out;
};
// GF(2^8) decoder kinds of one argument block (fill_dec8, launch_ff8_decode_batch)
// (ordered from the least specialised: a batch runs the minimum over its objects;
// the split decoder also handles the half kinds, with no high-half input)
constexpr int kDec8General = 0, kDec8Split = 1, kDec8Half = 2, kDec8HalfDense = 3;
// LDS dwords of the GF(2^8) error locator in the decode kernels (one byte per position)
constexpr size_t kEl8Dwords = kFf8Ptrs / 4;
// Forms of the GF(2^8) encoder tile (k_ff8_enc): general (pruned, chunked),
// dense encode (one chunk, K = R = m), dense inverse (full-loss decode of a
// K = R = m code, launch_ff8_decode_full).
constexpr int kFormGeneral = 0, kFormDenseEnc = 1, kFormDenseDec = 2;

struct XorArgs {
    PieceMap src;
    unsigned count;
    PieceMap out;
    uint64_t ndwords;
};

// Launchers (rs_kernels.hip).  Return hipSuccess or the launch error.
hipError_t launch_decode_hi_half(const DecArgs& a, hipStream_t s);
hipError_t launch_ff8_decode_half(unsigned Tm, const Ff8DecArgs& a, hipStream_t s);
hipError_t launch_ff8_decode_split(unsigned Tm, const Ff8DecArgs& a, hipStream_t s);
hipError_t launch_encode_fused16(unsigned T, const EncArgs& a, hipStream_t s);
hipError_t launch_encode_lo(const EncArgs& a, hipStream_t s);
hipError_t launch_encode_hi(const EncArgs& a, hipStream_t s);
hipError_t launch_encode_fin(const EncArgs& a, hipStream_t s);
hipError_t launch_decode_lo(const DecArgs& a, hipStream_t s);
hipError_t launch_decode_hi(const DecArgs& a, hipStream_t s);
hipError_t launch_decode_fin(const DecArgs& a, hipStream_t s);
hipError_t launch_error_locator16(const uint32_t* erased, const uint32_t* walsh, uint32_t* tmp, uint32_t* el,
                                  uint32_t* scale_logs, uint32_t* reveal_logs, unsigned m, unsigned K, unsigned R,
                                  hipStream_t s);
hipError_t launch_xor_reduce(const XorArgs& a, hipStream_t s);
// Small GF(2^16) codes on narrow column strips (rs_ff16_small.hip)
bool encode16_small_supported(unsigned Tm);
hipError_t launch_encode16_small(unsigned Tm, const EncArgs& a, hipStream_t s);
// the chunk-parallel form for single calls of few column strips (chunk IFFTs in
// parallel workgroups into the slab a.slab_out = a.slab_in of nchunks x m rows,
// then their XOR, the FFT and the outputs)
bool encode16_split_wins(unsigned Tm, unsigned nchunks, uint64_t nunits, unsigned cus);
hipError_t launch_encode16_split(unsigned Tm, const EncArgs& a, hipStream_t s);
// decode, n = 2^Tn with 9 <= Tn <= 11: pass 1 (scale + low IFFT of every tile
// with received data -> slab a_out), pass 2 (high part + D_lo + low FFT +
// reveal of every tile holding a lost original, slab a_in = pass 1's)
bool decode16_small_supported(unsigned Tn);
hipError_t launch_decode16_small_lo(const DecArgs& a, hipStream_t s);
hipError_t launch_decode16_small_fin(const DecArgs& a, hipStream_t s);
// batches of `count` objects of one shape, argument blocks in device memory
// (object = blockIdx.y; pass 1 of the decoder: blockIdx.z)
hipError_t launch_encode16_small_batch(unsigned Tm, const EncArgs* objs, unsigned count, uint64_t nunits,
                                       hipStream_t s);
hipError_t launch_decode16_small_batch(const DecArgs* objs, unsigned count, uint64_t nunits, unsigned nlo,
                                       unsigned nout, hipStream_t s);
// one pass (scale + low IFFT per received tile folded into per-lane Z
// accumulators, then low FFT + reveal per output tile) when nout is small
bool decode16_one_supported(unsigned nout);
hipError_t launch_decode16_one(const DecArgs& a, hipStream_t s);
hipError_t launch_decode16_one_batch(const DecArgs* objs, unsigned count, uint64_t nunits, hipStream_t s);
hipError_t launch_ff8_encode(unsigned T, const Ff8EncArgs& a, hipStream_t s);
hipError_t launch_ff8_decode(unsigned T, const Ff8DecArgs& a, hipStream_t s);
hipError_t launch_error_locator8(const El8Args& a, unsigned count, hipStream_t s);
// Batched GF(2^8) launches: `count` argument blocks in device memory (same T,
// column count and chunk structure), one grid (strips x objects).  For the
// decoder, mode = the least specialised kDec8* kind over the objects (T is the
// half tile's bits for the half kinds, as for launch_ff8_decode_half).
hipError_t launch_ff8_encode_batch(unsigned T, const Ff8EncArgs* objs, unsigned count, uint32_t nunits, bool multi,
                                   int form, hipStream_t s);
hipError_t launch_ff8_decode_full(unsigned Tm, const Ff8EncArgs& a, hipStream_t s);
// Slab batches (count <= kSlabObjs objects, arguments by value): the encoder
// tile (form as launch_ff8_encode_batch; kFormDenseDec = full-loss decodes of
// K = R = m codes, in = received recovery slab, out = outputs).
// q / qclear: the bit-sliced tile's queue counters for this launch and the set
// to zero for the next one (Workspace::bs_queue; null: static tile assignment).
// cus: the device's compute units (sizes the bit-sliced kernel's persistent grid).
hipError_t launch_ff8_encode_slab(unsigned T, const Ff8SlabBatch& b, unsigned count, bool multi, int form,
                                  hipStream_t s, unsigned cus, uint32_t* q = nullptr, uint32_t* qclear = nullptr);
hipError_t launch_ff8_decode_batch(unsigned T, const Ff8DecArgs* objs, unsigned count, uint32_t nunits, int mode,
                                   hipStream_t s);
// Bit-sliced dense tile (rs_ff8_bs.hip): slab batches of K = R = 128 codes,
// form kFormDenseEnc or kFormDenseDec (the encoder's inverse, full loss).
bool ff8_bs_supported(unsigned T, unsigned K, unsigned R, unsigned nchunks);
// Tile queues of the bit-sliced kernel: 8 counters (one per XCD), 128 bytes apart.
constexpr unsigned kBsQueueDw = 8 * 32;
hipError_t launch_ff8_bs_slab(const Ff8SlabBatch& b, unsigned count, int form, hipStream_t s, unsigned cus,
                              uint32_t* q, uint32_t* qclear);

// Matrix path (rs_ff8_mat.hip): the kernel, unit pieces (piece j = byte 1 at
// column j, `pitch` bytes each) and the conversion of the L rows of products
// (byte j of row i = M[i][j]) into tables, through vtab (value-indexed tables).
bool ff8_mat_supported(unsigned L, unsigned N);
hipError_t launch_ff8_mat(const Ff8MatArgs& a, unsigned cus, hipStream_t s);
hipError_t launch_ff8_unit(uint8_t* out, unsigned n, unsigned pitch, hipStream_t s);
hipError_t launch_ff8_mat_tabs(const uint8_t* rows, unsigned pitch, unsigned L, unsigned N, const uint32_t* vtab,
                               uint32_t* tabs, hipStream_t s);

// Units per lane chosen for each kernel family (the host sizes grids with it).
constexpr int kUnitsPerLane = 1;
constexpr unsigned kUnitsPerTile = 64 * kUnitsPerLane;

}  // namespace lamd
