// tools/flush_probe.cc -- per-flush cost of the durable log's GPU batch (dev
// tool): frames of 42-1024 B entries staged back to back
// in mapped pinned memory (as the log's arena), checksummed through the
// entry points the log uses, median of REPS calls per flush size.
//
//   flush_probe [REPS]
//
// Columns: frames and bytes per flush; us per call of mi_crc32c_batch_multi
// (the log's default engine), of mi_crc32c_batch, of the same batch staged
// by copy commands (MI_CRC32C_ZERO_COPY=0), of the direct kernel with its LDS
// table image (MI_CRC32C_DIRECT_LITE=0), of the default form waited for by a
// stream sync (MI_CRC32C_DONE_WORD=0), of a one-record round trip (16 B),
// the bound 'round trip + bytes / 55 GB/s', and the engine's CPU path on the
// calling thread (MI_CRC32C_CPU: crc32q, what the durable log routes flushes
// below its host_batch_max to; round 5).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <vector>

#include "consus_crc32c.h"

namespace {

double median_us(int reps, const std::function<void()>& f)
{
    std::vector<double> t(reps);
    for (int i = 0; i < 20; ++i) f();
    for (int i = 0; i < reps; ++i)
    {
        const auto a = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

}  // namespace

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 1000;
    mi_crc32c_set_gpu_min(0);
    if (mi_crc32c_init(0) != MI_CRC32C_OK)
    {
        fprintf(stderr, "no device: %s\n", mi_crc32c_last_error());
        return 1;
    }
    const size_t cap = size_t(8) << 20;
    void* p = nullptr;
    if (mi_host_malloc_pinned(&p, cap) != MI_CRC32C_OK) return 1;
    unsigned char* arena = static_cast<unsigned char*>(p);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < cap; ++i)
    {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        arena[i] = (unsigned char)x;
    }
    printf("%7s %9s %10s %10s %10s %10s %10s %10s %10s %10s\n", "frames", "bytes", "multi_us",
           "batch_us", "copy_us", "lds_us", "sync_us", "empty_us", "bound_us", "cpu_us");
    for (size_t frames : {1, 16, 64, 128, 270, 384, 512, 640, 768, 1024, 2048, 4096, 8192})
    {
        std::vector<uint64_t> off(frames);
        std::vector<uint32_t> len(frames);
        std::vector<uint32_t> out(frames), out2(frames);
        uint64_t at = 0, total = 0;
        for (size_t i = 0; i < frames; ++i)
        {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            const uint32_t entry = 42 + uint32_t(x % 983);
            off[i] = at;
            len[i] = 16 + entry;  // header + entry; the 4-B CRC slot follows
            at += 16 + entry + 4;
            total += len[i];
        }
        const double multi = median_us(reps, [&] {
            mi_crc32c_batch_multi(arena, off.data(), len.data(), nullptr, frames, total, out.data(),
                                  MI_CRC32C_FALLBACK, nullptr, 0, 0);
        });
        const double batch = median_us(reps, [&] {
            mi_crc32c_batch(arena, off.data(), len.data(), nullptr, frames, total, out2.data(),
                            MI_CRC32C_FALLBACK);
        });
        if (memcmp(out.data(), out2.data(), frames * 4)) printf("MISMATCH multi/batch\n");
        setenv("MI_CRC32C_ZERO_COPY", "0", 1);
        const double copy = median_us(reps, [&] {
            mi_crc32c_batch(arena, off.data(), len.data(), nullptr, frames, total, out2.data(),
                            MI_CRC32C_FALLBACK);
        });
        unsetenv("MI_CRC32C_ZERO_COPY");
        if (memcmp(out.data(), out2.data(), frames * 4)) printf("MISMATCH copy\n");
        setenv("MI_CRC32C_DIRECT_LITE", "0", 1);
        const double lds = median_us(reps, [&] {
            mi_crc32c_batch(arena, off.data(), len.data(), nullptr, frames, total, out2.data(),
                            MI_CRC32C_FALLBACK);
        });
        unsetenv("MI_CRC32C_DIRECT_LITE");
        if (memcmp(out.data(), out2.data(), frames * 4)) printf("MISMATCH lds\n");
        setenv("MI_CRC32C_DONE_WORD", "0", 1);
        const double sync = median_us(reps, [&] {
            mi_crc32c_batch(arena, off.data(), len.data(), nullptr, frames, total, out2.data(),
                            MI_CRC32C_FALLBACK);
        });
        unsetenv("MI_CRC32C_DONE_WORD");
        if (memcmp(out.data(), out2.data(), frames * 4)) printf("MISMATCH sync\n");
        const uint64_t o16 = 0;
        const uint32_t l16 = 16;
        uint32_t c16 = 0;
        const double empty = median_us(reps, [&] {
            mi_crc32c_batch(arena, &o16, &l16, nullptr, 1, 16, &c16, MI_CRC32C_FALLBACK);
        });
        const double cpu = median_us(reps, [&] {
            mi_crc32c_batch(arena, off.data(), len.data(), nullptr, frames, total, out2.data(),
                            MI_CRC32C_CPU);
        });
        if (memcmp(out.data(), out2.data(), frames * 4)) printf("MISMATCH cpu\n");
        printf("%7zu %9llu %10.2f %10.2f %10.2f %10.2f %10.2f %10.2f %10.2f %10.2f\n", frames,
               (unsigned long long)at, multi, batch, copy, lds, sync, empty,
               empty + double(at) / 55e3, cpu);
        fflush(stdout);
    }
    mi_crc32c_stats_t st;
    mi_crc32c_stats(&st);
    printf("gpu_calls %llu zero_copy_batches %llu fallback_calls %llu\n",
           (unsigned long long)st.gpu_calls, (unsigned long long)st.zero_copy_batches,
           (unsigned long long)st.fallback_calls);
    mi_host_free_pinned(p);
    return st.fallback_calls ? 1 : 0;
}
