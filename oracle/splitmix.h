/* oracle/splitmix.h -- synthetic-input definition shared by the oracle and
 * the reference driver (TEST INFRASTRUCTURE ONLY; see oracle/README.md).
 *
 * The benchmark inputs of BASELINE.json configs 2-4 are defined in SURVEY.md
 * section 8(d): u64 word j of the batch is splitmix64(seed ^ j), stored
 * little-endian, j counted from the start of the whole (unsharded) batch.
 * The product library has its own device/host generator
 * (consus_amd/csrc/workload.cc); tests check the two agree byte for byte.
 */
#ifndef CONSUS_ORACLE_SPLITMIX_H
#define CONSUS_ORACLE_SPLITMIX_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t oracle_splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Fill bytes [byte_offset, byte_offset + nbytes) of the virtual stream
 * defined by `seed` into dst.  byte_offset need not be word aligned. */
static inline void oracle_fill_stream(uint8_t* dst, size_t nbytes,
                                      uint64_t seed, uint64_t byte_offset)
{
    size_t i = 0;
    while (i < nbytes)
    {
        const uint64_t pos = byte_offset + i;
        const uint64_t word = oracle_splitmix64(seed ^ (pos >> 3));
        const unsigned k = (unsigned)(pos & 7);
        size_t take = 8 - k;
        if (take > nbytes - i) take = nbytes - i;
        uint8_t w[8];
        for (int b = 0; b < 8; ++b) w[b] = (uint8_t)(word >> (8 * b));
        memcpy(dst + i, w + k, take);
        i += take;
    }
}

#endif
