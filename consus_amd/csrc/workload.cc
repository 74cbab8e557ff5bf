// consus_amd/csrc/workload.cc -- synthetic record batches of BASELINE.json
// configs 3 and 5.  Host-side input generation only (the
// payload bytes themselves are generated on the device by mi_fill_splitmix64).
//
// Config 3 lengths: L_i = max(64, 64*k_i - j_i), k_i in 1..1024 Zipf with
// P(k) ~ k^-1.2, j_i uniform in 0..63.  Integer-only so that every host
// (and tests/golden/make_golden.py, which restates it in Python) agrees:
//   r_k   = floor((k^6 * 2^50)^(1/5))  = floor(k^1.2 * 2^10)   (exact iroot)
//   w_k   = floor(2^40 / r_k),  W_k = w_1 + ... + w_k
//   u_i   = splitmix64(seed ^ 2i),  v_i = splitmix64(seed ^ (2i+1))
//   k_i   = 1 + #{k : W_k <= u_i mod W_1024},  j_i = v_i & 63
#include <stddef.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "../../include/consus_crc32c.h"

namespace {

uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

using u128 = unsigned __int128;

uint64_t iroot5(u128 x)
{
    uint64_t lo = 0, hi = uint64_t(1) << 26;  // (2^110)^(1/5) = 2^22 < 2^26
    while (lo < hi)
    {
        const uint64_t mid = (lo + hi + 1) / 2;
        const u128 m = mid;
        if (m * m * m * m * m <= x)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

const std::vector<uint64_t>& zipf_cdf()
{
    static std::vector<uint64_t> cdf;
    static std::once_flag once;
    std::call_once(once, [] {
        cdf.resize(1024);
        uint64_t acc = 0;
        for (uint64_t k = 1; k <= 1024; ++k)
        {
            const u128 k6 = u128(k) * k * k * k * k * k;
            const uint64_t r = iroot5(k6 << 50);
            acc += (uint64_t(1) << 40) / r;
            cdf[k - 1] = acc;
        }
    });
    return cdf;
}

}  // namespace

extern "C" {

// Lengths of records [first, first + count) of the config-3 stream `seed`.
void mi_workload_zipf_lengths(uint64_t seed, uint64_t first, size_t count, uint32_t* out)
{
    const std::vector<uint64_t>& cdf = zipf_cdf();
    const uint64_t total = cdf.back();
    for (size_t n = 0; n < count; ++n)
    {
        const uint64_t i = first + n;
        const uint64_t x = splitmix64(seed ^ (2 * i)) % total;
        const uint64_t j = splitmix64(seed ^ (2 * i + 1)) & 63u;
        size_t lo = 0, hi = 1023;  // first k-1 with cdf > x
        while (lo < hi)
        {
            const size_t mid = (lo + hi) / 2;
            if (cdf[mid] > x)
                hi = mid;
            else
                lo = mid + 1;
        }
        const uint64_t k = lo + 1;
        const uint64_t L = 64 * k - j;
        out[n] = uint32_t(L < 64 ? 64 : L);
    }
}

}  // extern "C"
