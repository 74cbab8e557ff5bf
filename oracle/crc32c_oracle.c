/* oracle/crc32c_oracle.c -- CPU restatement of Consus's CRC32C hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so, and only as the
 * checker / the timed CPU baseline -- never as the thing measured or shipped.
 * The product library (consus_amd/lib/libconsus_crc32c.so) never links it.
 *
 * What is restated (all file:line references are into rescrv/Consus):
 *   - consus::crc32c(init, data, n)            common/crc32c.h:40-41, common/crc32c.cc:122-126
 *     init is a previous CRC *output*: it is pre-inverted and the result
 *     post-inverted (CRC_FFs, common/crc32c.cc:31,41,47,52,79), so calls chain.
 *   - crc32_sse42_quads                         common/crc32c.cc:50-81
 *     crc32b up to 8-byte alignment, crc32q body, crc32b tail.
 *   - crc32_software + crc32c_sb8_64_bit        common/crc32c.cc:40-48, 594-634
 *     Intel slicing-by-8 with a 4-byte alignment prologue.  The reference
 *     passes the size_t length through a uint32_t parameter (:598), so
 *     n >= 4 GiB is silently taken mod 2^32; restated as-is.
 *   - tables crc_tableil8_o32..o88              common/crc32c.cc:153..531
 *     generated here from the reflected polynomial 0x82F63B78 with the
 *     recurrence T_k[i] = (T_{k-1}[i] >> 8) ^ T_0[T_{k-1}[i] & 0xFF];
 *     o(32+8k) == T_k (checked against the compiled reference in tests).
 *   - choose_crc32c dispatch                    common/crc32c.cc:101-120
 *
 * Pinning: tests/test_oracle.py checks this file against RFC 3720 B.4
 * known answers, the CRC-32C check value, and against the reference itself
 * compiled from /root/reference/common/crc32c.cc (oracle/_ref, built by
 * oracle/Makefile), including the committed golden fixtures in tests/golden/.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "splitmix.h"

#define ORACLE_POLY 0x82F63B78u
#define CRC_FFS 0xFFFFFFFFu

static uint32_t g_tab[16][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void oracle_make_tables(void)
{
    for (unsigned i = 0; i < 256; ++i)
    {
        uint32_t c = i;
        for (int b = 0; b < 8; ++b)
            c = (c & 1) ? (c >> 1) ^ ORACLE_POLY : (c >> 1);
        g_tab[0][i] = c;
    }
    for (int k = 1; k < 16; ++k)
        for (unsigned i = 0; i < 256; ++i)
            g_tab[k][i] = (g_tab[k - 1][i] >> 8) ^ g_tab[0][g_tab[k - 1][i] & 0xFF];
}

static inline void tables(void) { pthread_once(&g_once, oracle_make_tables); }

/* Export T_0..T_15 (16 x 256 u32) for table-parity tests. */
void oracle_tables(uint32_t* out)
{
    tables();
    memcpy(out, g_tab, sizeof(g_tab));
}

/* Definition: one bit at a time, reflected, poly 0x82F63B78. */
uint32_t oracle_crc32c_bitwise(uint32_t init, const uint8_t* p, size_t n)
{
    uint32_t c = init ^ CRC_FFS;
    for (size_t i = 0; i < n; ++i)
    {
        c ^= p[i];
        for (int b = 0; b < 8; ++b)
            c = (c & 1) ? (c >> 1) ^ ORACLE_POLY : (c >> 1);
    }
    return c ^ CRC_FFS;
}

/* Restates crc32c_sb8_64_bit (common/crc32c.cc:594-634). */
static uint32_t sb8_body(uint32_t crc, const uint8_t* p, uint32_t length, uint32_t init_bytes)
{
    const uint32_t running = ((length - init_bytes) / 8) * 8;
    const uint32_t end_bytes = length - init_bytes - running;
    for (uint32_t i = 0; i < init_bytes; ++i)
        crc = g_tab[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    for (uint32_t i = 0; i < running / 8; ++i)
    {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        p += 8;
        crc ^= lo;
        crc = g_tab[7][crc & 0xFF] ^ g_tab[6][(crc >> 8) & 0xFF] ^
              g_tab[5][(crc >> 16) & 0xFF] ^ g_tab[4][crc >> 24] ^
              g_tab[3][hi & 0xFF] ^ g_tab[2][(hi >> 8) & 0xFF] ^
              g_tab[1][(hi >> 16) & 0xFF] ^ g_tab[0][hi >> 24];
    }
    for (uint32_t i = 0; i < end_bytes; ++i)
        crc = g_tab[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
    return crc;
}

/* Restates crc32_software (common/crc32c.cc:40-48): 4-byte alignment
 * prologue computed from the pointer value, length truncated to uint32_t. */
uint32_t oracle_crc32c_sb8(uint32_t init, const uint8_t* p, size_t n)
{
    tables();
    const uintptr_t x = (uintptr_t)p;
    uint32_t pro = (uint32_t)(((x + 3) & ~(uintptr_t)3) - x);
    if (pro > n) pro = (uint32_t)n;
    return sb8_body(init ^ CRC_FFS, p, (uint32_t)n, pro) ^ CRC_FFS;
}

/* Restates crc32_sse42_quads (common/crc32c.cc:50-81) with the SSE4.2
 * intrinsics that compile to the same crc32b / crc32q instructions. */
__attribute__((target("sse4.2")))
uint32_t oracle_crc32c_sse42(uint32_t init, const uint8_t* p, size_t n)
{
    uint64_t crc = init ^ CRC_FFS;
    const uintptr_t x = (uintptr_t)p;
    const size_t align = ((x + 7) & ~(uintptr_t)7) - x;
    const size_t pro = align > n ? n : align;
    const size_t body = (n - pro) >> 3;
    const size_t tail = n - (body << 3) - pro;
    for (size_t i = 0; i < pro; ++i)
        crc = __builtin_ia32_crc32qi((uint32_t)crc, p[i]);
    const uint8_t* q = p + pro;
    for (size_t i = 0; i < body; ++i)
    {
        uint64_t w;
        memcpy(&w, q + 8 * i, 8);
        crc = __builtin_ia32_crc32di(crc, w);
    }
    const size_t off = n - tail;
    for (size_t i = 0; i < tail; ++i)
        crc = __builtin_ia32_crc32qi((uint32_t)crc, p[off + i]);
    return (uint32_t)(crc ^ CRC_FFS);
}

int oracle_has_sse42(void)
{
    __builtin_cpu_init();
    return __builtin_cpu_supports("sse4.2") ? 1 : 0;
}

/* consus::crc32c as dispatched by choose_crc32c (common/crc32c.cc:101-126). */
uint32_t oracle_crc32c(uint32_t init, const uint8_t* p, size_t n)
{
    return oracle_has_sse42() ? oracle_crc32c_sse42(init, p, n)
                              : oracle_crc32c_sb8(init, p, n);
}

/* ---- shift-by-zeros operator and combine ------------------------------
 * Z_n(s): the register after feeding n zero bytes to a raw (un-inverted)
 * CRC register s.  crc32c(0, A||B) == Z_{|B|}(crc32c(0, A)) ^ crc32c(0, B),
 * which is what chaining consus::crc32c(crc32c(0, A), B) computes
 * (common/crc32c.cc:122-126 semantics). */
static uint32_t gf2_times(const uint32_t* mat, uint32_t vec)
{
    uint32_t sum = 0;
    for (int i = 0; vec; ++i, vec >>= 1)
        if (vec & 1) sum ^= mat[i];
    return sum;
}

static void gf2_square(uint32_t* sq, const uint32_t* mat)
{
    for (int i = 0; i < 32; ++i) sq[i] = gf2_times(mat, mat[i]);
}

uint32_t oracle_shift(uint32_t s, uint64_t nbytes)
{
    uint32_t odd[32], even[32];
    /* operator for one zero bit */
    odd[0] = ORACLE_POLY;
    for (int i = 1; i < 32; ++i) odd[i] = 1u << (i - 1);
    gf2_square(even, odd); /* 2 bits */
    gf2_square(odd, even); /* 4 bits */
    /* now odd = 4 bits; squaring once more gives one byte */
    uint32_t* cur = odd;
    uint32_t* nxt = even;
    gf2_square(nxt, cur); /* 8 bits = 1 byte */
    { uint32_t* t = cur; cur = nxt; nxt = t; }
    while (nbytes)
    {
        if (nbytes & 1) s = gf2_times(cur, s);
        nbytes >>= 1;
        if (!nbytes) break;
        gf2_square(nxt, cur);
        uint32_t* t = cur; cur = nxt; nxt = t;
    }
    return s;
}

uint32_t oracle_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    return oracle_shift(crc_a, len_b) ^ crc_b;
}

/* ---- batch helpers (threads split contiguous record ranges) ------------ */
struct batch_job {
    const uint8_t* base;
    const uint64_t* off;
    const uint32_t* len;
    size_t stride, flen;
    const uint32_t* inits;
    uint32_t* out;
    size_t lo, hi;
};

static void* batch_worker(void* arg)
{
    struct batch_job* j = (struct batch_job*)arg;
    for (size_t i = j->lo; i < j->hi; ++i)
    {
        const uint32_t init = j->inits ? j->inits[i] : 0;
        if (j->off)
            j->out[i] = oracle_crc32c(init, j->base + j->off[i], j->len[i]);
        else
            j->out[i] = oracle_crc32c(init, j->base + i * j->stride, j->flen);
    }
    return NULL;
}

static void run_batch(struct batch_job proto, size_t count, int threads)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    struct batch_job jobs[256];
    for (int t = 0; t < threads; ++t)
    {
        jobs[t] = proto;
        jobs[t].lo = count * (size_t)t / (size_t)threads;
        jobs[t].hi = count * (size_t)(t + 1) / (size_t)threads;
        pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

void oracle_crc32c_batch(const uint8_t* base, const uint64_t* off, const uint32_t* len,
                         const uint32_t* inits, size_t count, uint32_t* out, int threads)
{
    tables();
    struct batch_job p = {base, off, len, 0, 0, inits, out, 0, 0};
    run_batch(p, count, threads);
}

void oracle_crc32c_fixed(const uint8_t* base, size_t stride, size_t length,
                         const uint32_t* inits, size_t count, uint32_t* out, int threads)
{
    tables();
    struct batch_job p = {base, NULL, NULL, stride, length, inits, out, 0, 0};
    run_batch(p, count, threads);
}

/* Digest of a CRC vector: crc32c(0, little-endian bytes of crcs[0..n)) and
 * the XOR of all entries (SURVEY.md section 8(c) "Digests"). */
uint32_t oracle_digest(const uint32_t* crcs, size_t n, uint32_t* xor_out)
{
    uint32_t x = 0;
    for (size_t i = 0; i < n; ++i) x ^= crcs[i];
    if (xor_out) *xor_out = x;
    return oracle_crc32c(0, (const uint8_t*)crcs, n * sizeof(uint32_t));
}

void oracle_fill(uint8_t* dst, size_t nbytes, uint64_t seed, uint64_t byte_offset)
{
    oracle_fill_stream(dst, nbytes, seed, byte_offset);
}

/* Batch-CRC callback with the signature of consus::durable_log_batch_crc /
 * mi_dlog_batch_crc, so CPU tests can run the durable log's host logic
 * (segments, watermark, framing, replay) with the oracle as the engine. */
int oracle_dlog_batch(void* ctx, const void* base, const uint64_t* off, const uint32_t* len,
                      size_t count, uint64_t total, uint32_t* out)
{
    (void)ctx;
    (void)total;
    oracle_crc32c_batch((const uint8_t*)base, off, len, NULL, count, out, 1);
    return 0;
}
