/*
 * leo_oracle.c -- CPU restatement of Leopard-RS (catid/leopard v2) encode/decode.
 *
 * *** TEST INFRASTRUCTURE ONLY. ***
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this file's shared object, and only as the checker / CPU baseline.  The
 * product library (leopard_amd/, libleopard_amd.so) never links or calls it.
 *
 * It restates the reference's math in plain scalar C, written from the
 * reference's algorithm description (not its SIMD code):
 *   - fields, log/exp tables, Cantor basis .......... LeopardFF8.cpp:46-48,158-194
 *                                                      LeopardFF16.cpp:46-51,164-197
 *   - AddMod / SubMod / MultiplyLog .................. LeopardFF8.cpp:58-73,141-154
 *   - FWHT (mod 2^r-1) ............................... LeopardFF8.cpp:80-130
 *   - FFT skew + LogWalsh ............................ LeopardFF8.cpp:496-538, LeopardFF16.cpp:530-572
 *   - IFFT/FFT butterflies, layer drivers ............ LeopardFF8.cpp:595-816,1088-1262,1319-1596
 *   - ReedSolomonEncode / ReedSolomonDecode .......... LeopardFF8.cpp:1602-1672,1809-1916
 *                                                      LeopardFF16.cpp:1397-1467,1652-1775
 *   - leo_* dispatch, edge paths, error codes ........ leopard.cpp:94-344
 *   - FF16 ALTMAP element layout (lo byte j, hi byte j+32 of a 64-byte block)
 *                                                      LeopardFF16.cpp:315-332
 *
 * Parity of this restatement is pinned against the reference library compiled
 * from /root/reference by oracle/Makefile (oracle/_ref/libleopard_ref.so) and
 * against the committed fixtures under tests/golden/ (tests/golden/gen_golden.py).
 *
 * Exported C ABI (ctypes): orc_init, orc_encode_work_count, orc_decode_work_count,
 * orc_encode, orc_decode, orc_table (debug access to the tables).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_NEED_MORE_DATA (-1)
#define ORC_TOO_MUCH_DATA (-2)
#define ORC_INVALID_SIZE (-3)
#define ORC_INVALID_COUNTS (-4)
#define ORC_INVALID_INPUT (-5)
#define ORC_CALL_INITIALIZE (-7)

typedef struct {
    unsigned bits, order, modulus, poly;
    uint16_t *log_tab; /* Cantor-basis log: LogLUT */
    uint16_t *exp_tab; /* inverse: ExpLUT (modulus entry wraps to 0) */
    uint16_t *skew;    /* FFTSkew[modulus] as logs */
    uint16_t *walsh;   /* LogWalsh[order] */
} field_t;

static field_t F8, F16;
static int g_ready = 0;
static uint8_t *g_mul8; /* g_mul8[log_m * 256 + x] = x * exp(log_m) (FF8 only, speed) */

static const uint16_t kBasis8[8] = {1, 214, 152, 146, 86, 200, 88, 230};
static const uint16_t kBasis16[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                      0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

/* partially reduced modular add/sub (LeopardFF8.cpp:58-73): kModulus is a valid "zero" */
static inline unsigned add_mod(const field_t *f, unsigned a, unsigned b) {
    unsigned s = a + b;
    return (s + (s >> f->bits)) & f->modulus;
}
static inline unsigned sub_mod(const field_t *f, unsigned a, unsigned b) {
    unsigned d = a - b;
    return (d + (d >> f->bits)) & f->modulus;
}
/* a * exp(log_b), a a field element, log_b a (partially reduced) log (LeopardFF8.cpp:141-154) */
static inline unsigned mul_log(const field_t *f, unsigned a, unsigned log_b) {
    if (a == 0) return 0;
    return f->exp_tab[add_mod(f, f->log_tab[a], log_b)];
}

/* Walsh-Hadamard transform mod 2^r-1 over `order` entries (LeopardFF8.cpp:80-130).
 * Every layer is a butterfly (a,b)->(a+b,a-b); layers commute, so order is free. */
static void fwht(const field_t *f, uint16_t *v, unsigned order) {
    for (unsigned d = 1; d < order; d <<= 1)
        for (unsigned g = 0; g < order; g += 2 * d)
            for (unsigned i = g; i < g + d; ++i) {
                unsigned a = v[i], b = v[i + d];
                v[i] = (uint16_t)add_mod(f, a, b);
                v[i + d] = (uint16_t)sub_mod(f, a, b);
            }
}

static int field_build(field_t *f, unsigned bits, unsigned poly, const uint16_t *basis) {
    f->bits = bits;
    f->order = 1u << bits;
    f->modulus = f->order - 1;
    f->poly = poly;
    f->log_tab = (uint16_t *)calloc(f->order, 2);
    f->exp_tab = (uint16_t *)calloc(f->order, 2);
    f->skew = (uint16_t *)calloc(f->modulus, 2);
    f->walsh = (uint16_t *)calloc(f->order, 2);
    if (!f->log_tab || !f->exp_tab || !f->skew || !f->walsh) return 0;

    /* 1) discrete log in the standard (LFSR) representation, stored in exp_tab */
    uint16_t *dlog = f->exp_tab;
    unsigned st = 1;
    for (unsigned i = 0; i < f->modulus; ++i) {
        dlog[st] = (uint16_t)i;
        st <<= 1;
        if (st >= f->order) st ^= poly;
    }
    dlog[0] = (uint16_t)f->modulus;
    /* 2) element with Cantor-basis coordinates i, then its discrete log */
    uint16_t *cant = f->log_tab;
    cant[0] = 0;
    for (unsigned b = 0; b < bits; ++b) {
        unsigned w = 1u << b;
        for (unsigned j = 0; j < w; ++j) cant[j + w] = cant[j] ^ basis[b];
    }
    for (unsigned i = 0; i < f->order; ++i) f->log_tab[i] = dlog[cant[i]];
    /* 3) inverse map */
    for (unsigned i = 0; i < f->order; ++i) f->exp_tab[f->log_tab[i]] = (uint16_t)i;
    f->exp_tab[f->modulus] = f->exp_tab[0];

    /* FFT skew factors, eq.(28) of Lin-Chung-Han (LeopardFF8.cpp:496-538) */
    unsigned t[16];
    for (unsigned i = 1; i < bits; ++i) t[i - 1] = 1u << i;
    for (unsigned mm = 0; mm + 1 < bits; ++mm) {
        unsigned step = 1u << (mm + 1);
        f->skew[(1u << mm) - 1] = 0;
        for (unsigned i = mm; i + 1 < bits; ++i) {
            unsigned s = 1u << (i + 1);
            for (unsigned j = (1u << mm) - 1; j < s; j += step) f->skew[j + s] = f->skew[j] ^ (uint16_t)t[i];
        }
        t[mm] = f->modulus - f->log_tab[mul_log(f, t[mm], f->log_tab[t[mm] ^ 1])];
        for (unsigned i = mm + 1; i + 1 < bits; ++i) {
            unsigned sum = add_mod(f, f->log_tab[t[i] ^ 1], t[mm]);
            t[i] = mul_log(f, t[i], sum);
        }
    }
    for (unsigned i = 0; i < f->modulus; ++i) f->skew[i] = f->log_tab[f->skew[i]];

    for (unsigned i = 0; i < f->order; ++i) f->walsh[i] = f->log_tab[i];
    f->walsh[0] = 0;
    fwht(f, f->walsh, f->order);
    return 1;
}

int orc_init(void) {
    if (g_ready) return ORC_OK;
    if (!field_build(&F8, 8, 0x11D, kBasis8)) return -6;
    if (!field_build(&F16, 16, 0x1002D, kBasis16)) return -6;
    g_mul8 = (uint8_t *)malloc(256 * 256);
    for (unsigned lm = 0; lm < 256; ++lm)
        for (unsigned x = 0; x < 256; ++x) g_mul8[lm * 256 + x] = (uint8_t)mul_log(&F8, x, lm);
    g_ready = 1;
    return ORC_OK;
}

/* table export for tests: which = 0 log, 1 exp, 2 skew, 3 walsh */
int orc_table(int ff16, int which, uint16_t *out) {
    if (!g_ready) return ORC_CALL_INITIALIZE;
    const field_t *f = ff16 ? &F16 : &F8;
    const uint16_t *src = which == 0 ? f->log_tab : which == 1 ? f->exp_tab : which == 2 ? f->skew : f->walsh;
    unsigned n = which == 2 ? f->modulus : f->order;
    memcpy(out, src, n * 2u);
    return (int)n;
}

/* ---------------------------------------------------------------- buffers -- */
/* One "piece" is `bytes` bytes.  FF8 elements are bytes; FF16 element j of a
 * 64-byte block is b[j] | b[j+32] << 8 (ALTMAP, LeopardFF16.cpp:315-332). */

static void buf_xor(uint8_t *x, const uint8_t *y, uint64_t bytes) {
    for (uint64_t i = 0; i < bytes; ++i) x[i] ^= y[i];
}

/* x ^= y * exp(log_m)   (skipped by callers when the skew is "zero") */
static void buf_muladd(const field_t *f, uint8_t *x, const uint8_t *y, unsigned log_m, uint64_t bytes) {
    if (f->bits == 8) {
        const uint8_t *t = g_mul8 + log_m * 256u;
        for (uint64_t i = 0; i < bytes; ++i) x[i] ^= t[y[i]];
        return;
    }
    for (uint64_t blk = 0; blk < bytes; blk += 64)
        for (unsigned j = 0; j < 32; ++j) {
            unsigned e = y[blk + j] | ((unsigned)y[blk + j + 32] << 8);
            unsigned p = mul_log(f, e, log_m);
            x[blk + j] ^= (uint8_t)p;
            x[blk + j + 32] ^= (uint8_t)(p >> 8);
        }
}

/* x = y * exp(log_m)  (mul_mem: log_m == modulus multiplies by one) */
static void buf_mul(const field_t *f, uint8_t *x, const uint8_t *y, unsigned log_m, uint64_t bytes) {
    memset(x, 0, bytes);
    buf_muladd(f, x, y, log_m, bytes);
}

/* Butterflies (LeopardFF8.cpp:595-666 IFFT, 1319-1390 FFT).  A skew equal to
 * kModulus encodes the zero element: the multiply is skipped. */
static void ifft_bfly(const field_t *f, uint8_t *x, uint8_t *y, unsigned log_m, uint64_t bytes) {
    buf_xor(y, x, bytes);
    if (log_m != f->modulus) buf_muladd(f, x, y, log_m, bytes);
}
static void fft_bfly(const field_t *f, uint8_t *x, uint8_t *y, unsigned log_m, uint64_t bytes) {
    if (log_m != f->modulus) buf_muladd(f, x, y, log_m, bytes);
    buf_xor(y, x, bytes);
}

/* IFFT over `size` pieces, layers dist = 1,2,4,...; the pair (i, i+dist) in the
 * group starting at g uses skew[g + dist]  (LeopardFF8.cpp:1088-1262: the
 * radix-4 driver uses log_m01=skew[r+dist], log_m23=skew[r+3dist],
 * log_m02=skew[r+2dist], which is this rule applied layer by layer).
 * Groups entirely at or beyond `trunc` hold zeros and are skipped. */
static void ifft(const field_t *f, uint8_t **w, unsigned size, unsigned trunc, const uint16_t *skew, uint64_t bytes) {
    for (unsigned d = 1; d < size; d <<= 1)
        for (unsigned g = 0; g < size; g += 2 * d) {
            if (g >= trunc) continue; /* all-zero group stays zero */
            unsigned lm = skew[g + d];
            for (unsigned i = g; i < g + d; ++i) ifft_bfly(f, w[i], w[i + d], lm, bytes);
        }
}

/* FFT over `size` pieces, layers dist = size/2 ... 1, same skew rule
 * (LeopardFF8.cpp:1544-1596); outputs at index >= trunc are not needed. */
static void fft(const field_t *f, uint8_t **w, unsigned size, unsigned trunc, const uint16_t *skew, uint64_t bytes) {
    for (unsigned d = size >> 1; d >= 1; d >>= 1)
        for (unsigned g = 0; g < trunc && g < size; g += 2 * d) {
            unsigned lm = skew[g + d];
            for (unsigned i = g; i < g + d; ++i) fft_bfly(f, w[i], w[i + d], lm, bytes);
        }
}

static unsigned next_pow2(unsigned n) {
    unsigned p = 1;
    while (p < n) p <<= 1;
    return p;
}

unsigned orc_encode_work_count(unsigned k, unsigned r) {
    if (k == 1) return r;
    if (r == 1) return 1;
    return next_pow2(r) * 2;
}
unsigned orc_decode_work_count(unsigned k, unsigned r) {
    if (k == 1 || r == 1) return k;
    unsigned m = next_pow2(r);
    return next_pow2(m + k);
}

/* ReedSolomonEncode (LeopardFF8.cpp:1602-1672): work[0..m) = XOR over chunks c
 * of IFFT_m(data[c*m..], skew + m-1 + c*m), then FFT_m(work, skew - 1) and the
 * first R outputs are the recovery pieces. */
static void rs_encode(const field_t *f, uint64_t bytes, unsigned k, unsigned r, unsigned m, const uint8_t *const *data,
                      uint8_t **work) {
    for (unsigned c = 0; c * m < k; ++c) {
        unsigned cnt = k - c * m < m ? k - c * m : m;
        uint8_t **dst = c == 0 ? work : work + m;
        for (unsigned i = 0; i < m; ++i) {
            if (i < cnt) memcpy(dst[i], data[c * m + i], bytes);
            else memset(dst[i], 0, bytes);
        }
        ifft(f, dst, m, cnt, f->skew + m - 1 + c * m, bytes);
        if (c > 0)
            for (unsigned i = 0; i < m; ++i) buf_xor(work[i], dst[i], bytes);
    }
    fft(f, work, m, r, f->skew - 1, bytes);
}

/* ReedSolomonDecode (LeopardFF8.cpp:1809-1916). */
static void rs_decode(const field_t *f, uint64_t bytes, unsigned k, unsigned r, unsigned m, unsigned n,
                      const uint8_t *const *orig, const uint8_t *const *rec, uint8_t **work) {
    uint16_t *el = (uint16_t *)calloc(f->order, 2);
    for (unsigned i = 0; i < r; ++i)
        if (!rec[i]) el[i] = 1;
    for (unsigned i = r; i < m; ++i) el[i] = 1;
    for (unsigned i = 0; i < k; ++i)
        if (!orig[i]) el[m + i] = 1;
    /* error locator: FWHT, pointwise * LogWalsh mod (2^r-1), FWHT */
    fwht(f, el, f->order);
    for (unsigned i = 0; i < f->order; ++i) el[i] = (uint16_t)(((unsigned)el[i] * f->walsh[i]) % f->modulus);
    fwht(f, el, f->order);

    for (unsigned i = 0; i < m; ++i) {
        if (i < r && rec[i]) buf_mul(f, work[i], rec[i], el[i], bytes);
        else memset(work[i], 0, bytes);
    }
    for (unsigned i = 0; i < k; ++i) {
        if (orig[i]) buf_mul(f, work[m + i], orig[i], el[m + i], bytes);
        else memset(work[m + i], 0, bytes);
    }
    for (unsigned i = m + k; i < n; ++i) memset(work[i], 0, bytes);

    ifft(f, work, n, m + k, f->skew - 1, bytes);

    /* formal derivative (LeopardFF8.cpp:1890-1899): for i=1..n-1, with
     * w = lowest set bit of i, work[i-w+j] ^= work[i+j] for j < w. */
    for (unsigned i = 1; i < n; ++i) {
        unsigned w = i & (~i + 1);
        for (unsigned j = 0; j < w; ++j) buf_xor(work[i - w + j], work[i + j], bytes);
    }

    fft(f, work, n, m + k, f->skew - 1, bytes);

    for (unsigned i = 0; i < k; ++i)
        if (!orig[i]) buf_mul(f, work[i], work[i + m], f->modulus - el[i + m], bytes);
    free(el);
}

/* leo_encode dispatch restated (leopard.cpp:123-197) */
int orc_encode(uint64_t bytes, unsigned k, unsigned r, unsigned work_count, const void *const *orig, void **work) {
    if (bytes == 0 || bytes % 64 != 0) return ORC_INVALID_SIZE;
    if (r == 0 || r > k) return ORC_INVALID_COUNTS;
    if (!orig || !work) return ORC_INVALID_INPUT;
    if (!g_ready) return ORC_CALL_INITIALIZE;
    if (k == 1) {
        for (unsigned i = 0; i < r; ++i) memcpy(work[i], orig[i], bytes);
        return ORC_OK;
    }
    if (r == 1) { /* parity of all originals (leopard.cpp:106-121) */
        memcpy(work[0], orig[0], bytes);
        for (unsigned i = 1; i < k; ++i) buf_xor((uint8_t *)work[0], (const uint8_t *)orig[i], bytes);
        return ORC_OK;
    }
    unsigned m = next_pow2(r), n = next_pow2(m + k);
    if (work_count != 2 * m) return ORC_INVALID_COUNTS;
    if (n <= 256) rs_encode(&F8, bytes, k, r, m, (const uint8_t *const *)orig, (uint8_t **)work);
    else if (n <= 65536) rs_encode(&F16, bytes, k, r, m, (const uint8_t *const *)orig, (uint8_t **)work);
    else return ORC_TOO_MUCH_DATA;
    return ORC_OK;
}

/* leo_decode dispatch restated (leopard.cpp:233-344) */
int orc_decode(uint64_t bytes, unsigned k, unsigned r, unsigned work_count, const void *const *orig,
               const void *const *rec, void **work) {
    if (bytes == 0 || bytes % 64 != 0) return ORC_INVALID_SIZE;
    if (r == 0 || r > k) return ORC_INVALID_COUNTS;
    if (!orig || !rec || !work) return ORC_INVALID_INPUT;
    if (!g_ready) return ORC_CALL_INITIALIZE;
    unsigned lost = 0, lost_i = 0, got = 0, got_i = 0;
    for (unsigned i = 0; i < k; ++i)
        if (!orig[i]) { ++lost; lost_i = i; }
    for (unsigned i = 0; i < r; ++i)
        if (rec[i]) { ++got; got_i = i; }
    if (got < lost) return ORC_NEED_MORE_DATA;
    if (k == 1) {
        memcpy(work[0], rec[got_i], bytes);
        return ORC_OK;
    }
    if (lost == 0) {
        for (unsigned i = 0; i < k; ++i) memcpy(work[i], orig[i], bytes);
        return ORC_OK;
    }
    if (r == 1) { /* leopard.cpp:214-231 */
        memcpy(work[lost_i], rec[0], bytes);
        for (unsigned i = 0; i < k; ++i)
            if (orig[i]) buf_xor((uint8_t *)work[lost_i], (const uint8_t *)orig[i], bytes);
        return ORC_OK;
    }
    unsigned m = next_pow2(r), n = next_pow2(m + k);
    if (work_count != n) return ORC_INVALID_COUNTS;
    if (n <= 256)
        rs_decode(&F8, bytes, k, r, m, n, (const uint8_t *const *)orig, (const uint8_t *const *)rec, (uint8_t **)work);
    else if (n <= 65536)
        rs_decode(&F16, bytes, k, r, m, n, (const uint8_t *const *)orig, (const uint8_t *const *)rec,
                  (uint8_t **)work);
    else return ORC_TOO_MUCH_DATA;
    return ORC_OK;
}
