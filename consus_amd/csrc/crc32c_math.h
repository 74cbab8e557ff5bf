// consus_amd/csrc/crc32c_math.h -- GF(2) operator algebra for CRC-32C.
//
// Host-side table construction for the HIP kernels.  Nothing here touches
// record payloads: these are the constant operators the kernels stage in LDS.
//
// Conventions (reflected CRC-32C, polynomial 0x82F63B78, the one consus::crc32c
// computes -- common/crc32c.cc:31-48, table model comment at :139-151):
//   raw register s, byte update      s' = T0[(s ^ b) & 0xFF] ^ (s >> 8)
//   Z_n(s)  = register after n zero bytes are fed to s (linear in s)
//   T_k[b]  = Z_{k+1}(b)            (slice-by-16 table k; reference o(32+8k) == T_k)
//   G^n_j[b] = Z_n(b << 8j)         ("fold" table set for a shift of n bytes)
// Identities used by the kernels (derivations in DESIGN.md section 3):
//   raw(A || B)            = Z_|B|(raw(A)) ^ raw(B)
//   raw(0^k || A)          = raw(A)                (leading zeros are free)
//   crc32c(init, A)        = ~raw(A with ~init XORed into its first 4 bytes), |A| >= 4
//   crc32c(0, A||B)        = Z_|B|(crc32c(0, A)) ^ crc32c(0, B)   (combine)
#pragma once

#include <stdint.h>
#include <string.h>

namespace mi_crc {

constexpr uint32_t kPoly = 0x82F63B78u;

// 32x32 GF(2) matrix stored as 32 column images (image of bit i).
struct Op32
{
    uint32_t col[32];

    uint32_t apply(uint32_t v) const
    {
        uint32_t r = 0;
        for (int i = 0; v; ++i, v >>= 1)
            if (v & 1u) r ^= col[i];
        return r;
    }

    Op32 then(const Op32& after) const  // after o this
    {
        Op32 r;
        for (int i = 0; i < 32; ++i) r.col[i] = after.apply(col[i]);
        return r;
    }

    static Op32 identity()
    {
        Op32 r;
        for (int i = 0; i < 32; ++i) r.col[i] = 1u << i;
        return r;
    }

    // Z_1: one zero byte.
    static Op32 zero_byte()
    {
        Op32 r;
        for (int i = 0; i < 32; ++i)
        {
            uint32_t c = 1u << i;
            for (int b = 0; b < 8; ++b) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
            r.col[i] = c;
        }
        return r;
    }
};

// Inverse of an invertible operator (Gauss-Jordan over GF(2)).  Z_n is
// invertible because x is a unit modulo the CRC polynomial.  Returns false if
// the matrix is singular.
inline bool invert(const Op32& m, Op32* inv)
{
    // rows[i] = (row i of M) | (row i of I) << 32, bit j of the low half = M[i][j]
    uint64_t rows[32];
    for (int i = 0; i < 32; ++i)
    {
        uint64_t r = 0;
        for (int j = 0; j < 32; ++j)
            if ((m.col[j] >> i) & 1u) r |= uint64_t(1) << j;
        rows[i] = r | (uint64_t(1) << (32 + i));
    }
    for (int c = 0; c < 32; ++c)
    {
        int piv = -1;
        for (int i = c; i < 32; ++i)
            if ((rows[i] >> c) & 1u)
            {
                piv = i;
                break;
            }
        if (piv < 0) return false;
        const uint64_t t = rows[c];
        rows[c] = rows[piv];
        rows[piv] = t;
        for (int i = 0; i < 32; ++i)
            if (i != c && ((rows[i] >> c) & 1u)) rows[i] ^= rows[c];
    }
    for (int j = 0; j < 32; ++j)
    {
        uint32_t col = 0;
        for (int i = 0; i < 32; ++i)
            if ((rows[i] >> (32 + j)) & 1u) col |= 1u << i;
        inv->col[j] = col;
    }
    return true;
}

// Z_n by square-and-multiply over the 2^k-byte operators.
inline Op32 zeros_op(uint64_t nbytes)
{
    Op32 result = Op32::identity();
    Op32 p = Op32::zero_byte();
    while (nbytes)
    {
        if (nbytes & 1u) result = result.then(p);
        nbytes >>= 1;
        if (nbytes) p = p.then(p);
    }
    return result;
}

inline uint32_t shift_bytes(uint32_t s, uint64_t nbytes) { return zeros_op(nbytes).apply(s); }

// Operator tables: out[j][b] = z(b << 8j), j = 0..3 -- four 256-entry tables.
inline void make_op_tables(uint32_t out[4][256], const Op32& z)
{
    for (int j = 0; j < 4; ++j)
        for (uint32_t b = 0; b < 256; ++b) out[j][b] = z.apply(b << (8 * j));
}

// G^n_j[b] = Z_n(b << 8j).
inline void make_fold_tables(uint32_t out[4][256], uint64_t nbytes)
{
    make_op_tables(out, zeros_op(nbytes));
}

// Slice-by-16 tables T_0..T_15.
inline void make_slice16_tables(uint32_t out[16][256])
{
    for (uint32_t i = 0; i < 256; ++i)
    {
        uint32_t c = i;
        for (int b = 0; b < 8; ++b) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
        out[0][i] = c;
    }
    for (int k = 1; k < 16; ++k)
        for (uint32_t i = 0; i < 256; ++i)
            out[k][i] = (out[k - 1][i] >> 8) ^ out[0][out[k - 1][i] & 0xFFu];
}

}  // namespace mi_crc
