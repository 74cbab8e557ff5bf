// oracle/ref_driver.cc -- exports the REFERENCE implementation itself.
//
// TEST INFRASTRUCTURE ONLY (see oracle/crc32c_oracle.c header).  This driver
// is compiled by oracle/Makefile together with the unmodified reference TU
// /root/reference/common/crc32c.cc (pulled in by #include from where it lies;
// no reference source is copied into this repository).  The result,
// oracle/_ref/libref_crc32c.so, is git-ignored and travels to the GPU box as a
// prebuilt file, where bench.py times it as the CPU baseline
// ("cpu_baseline.kind": "reference") and tests use it as the parity anchor.
//
// Including the .cc gives this TU access to its file-static functions:
//   crc32_software      common/crc32c.cc:40-48
//   crc32_sse42_quads   common/crc32c.cc:50-81
//   crc32c_func         common/crc32c.cc:120 (the static-init dispatch choice)
//   crc_tableil8_o32..o88  common/crc32c.cc:153-585
#include "common/crc32c.cc"

#include <algorithm>
#include <thread>
#include <vector>

#include "splitmix.h"

#define REF_EXPORT extern "C" __attribute__((visibility("default")))

REF_EXPORT uint32_t ref_crc32c(uint32_t init, const unsigned char* p, size_t n)
{
    return consus::crc32c(init, p, n);
}

REF_EXPORT uint32_t ref_crc32c_sw(uint32_t init, const unsigned char* p, size_t n)
{
    return crc32_software(init, p, n);
}

REF_EXPORT uint32_t ref_crc32c_hw(uint32_t init, const unsigned char* p, size_t n)
{
    return crc32_sse42_quads(init, p, n);
}

REF_EXPORT int ref_dispatch_is_sse42(void)
{
    return crc32c_func == crc32_sse42_quads ? 1 : 0;
}

REF_EXPORT void ref_tables(uint32_t* out /* 8 x 256 */)
{
    const uint32_t* t[8] = {crc_tableil8_o32, crc_tableil8_o40, crc_tableil8_o48,
                            crc_tableil8_o56, crc_tableil8_o64, crc_tableil8_o72,
                            crc_tableil8_o80, crc_tableil8_o88};
    for (int k = 0; k < 8; ++k)
        std::copy(t[k], t[k] + 256, out + 256 * k);
}

template <typename F>
static void parallel_ranges(size_t count, int threads, F f)
{
    threads = std::max(1, std::min(threads, 256));
    if (threads == 1)
    {
        f(size_t(0), count);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
    {
        const size_t lo = count * size_t(t) / size_t(threads);
        const size_t hi = count * size_t(t + 1) / size_t(threads);
        th.emplace_back([=] { f(lo, hi); });
    }
    for (auto& x : th) x.join();
}

// Fixed-stride batch through the reference API (what a record-batching
// caller of consus::crc32c would do), one contiguous record range per thread.
REF_EXPORT void ref_crc32c_fixed_mt(const unsigned char* base, size_t stride, size_t len,
                                    const uint32_t* inits, size_t count, uint32_t* out,
                                    int threads)
{
    parallel_ranges(count, threads, [=](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i)
            out[i] = consus::crc32c(inits ? inits[i] : 0, base + i * stride, len);
    });
}

REF_EXPORT void ref_crc32c_batch_mt(const unsigned char* base, const uint64_t* off,
                                    const uint32_t* len, const uint32_t* inits, size_t count,
                                    uint32_t* out, int threads)
{
    parallel_ranges(count, threads, [=](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i)
            out[i] = consus::crc32c(inits ? inits[i] : 0, base + off[i], len[i]);
    });
}

// Per-record CRCs of the splitmix64-defined fixed-stride batch
//  without materialising it: each thread
// generates 4 MiB windows of records and hashes them with the reference.
REF_EXPORT void ref_crc32c_splitmix_fixed(uint64_t seed, size_t rec_len, uint64_t first_rec,
                                          size_t count, uint32_t* out, int threads)
{
    parallel_ranges(count, threads, [=](size_t lo, size_t hi) {
        const size_t per = std::max<size_t>(1, (size_t(4) << 20) / std::max<size_t>(rec_len, 1));
        std::vector<unsigned char> buf(per * rec_len + 8);
        for (size_t i = lo; i < hi; i += per)
        {
            const size_t n = std::min(per, hi - i);
            oracle_fill_stream(buf.data(), n * rec_len, seed, (first_rec + i) * rec_len);
            for (size_t r = 0; r < n; ++r)
                out[i + r] = consus::crc32c(0, buf.data() + r * rec_len, rec_len);
        }
    });
}

// One CRC over bytes [byte_off, byte_off + nbytes) of the splitmix64 stream
// `seed`, generated and hashed in 4 MiB pieces chained through init
// (common/crc32c.cc:122-126: init is a previous CRC): the single-record
// golden of bench.py --config single.
REF_EXPORT uint32_t ref_crc32c_splitmix_stream(uint64_t seed, uint64_t byte_off, uint64_t nbytes)
{
    const size_t piece = size_t(4) << 20;
    std::vector<unsigned char> buf(piece + 8);
    uint32_t crc = 0;
    for (uint64_t done = 0; done < nbytes;)
    {
        const size_t n = size_t(std::min<uint64_t>(piece, nbytes - done));
        oracle_fill_stream(buf.data(), n, seed, byte_off + done);
        crc = consus::crc32c(crc, buf.data(), n);
        done += n;
    }
    return crc;
}

// Per-record CRCs of records [base_off + offsets[i], +lengths[i]) of the
// splitmix64 stream `seed` (config 3: packed Zipf-length records), generated
// on the fly per record.
REF_EXPORT void ref_crc32c_splitmix_var(uint64_t seed, const uint64_t* offsets,
                                        const uint32_t* lengths, size_t count, uint32_t* out,
                                        int threads)
{
    parallel_ranges(count, threads, [=](size_t lo, size_t hi) {
        std::vector<unsigned char> buf;
        for (size_t i = lo; i < hi; ++i)
        {
            if (buf.size() < lengths[i] + size_t(8)) buf.resize(lengths[i] + size_t(8));
            oracle_fill_stream(buf.data(), lengths[i], seed, offsets[i]);
            out[i] = consus::crc32c(0, buf.data(), lengths[i]);
        }
    });
}
