// tools/route_probe.cc -- latency of one consus::crc32c call on host bytes,
// through the GPU engine and through the engine's CPU path, by size (dev
// tool; sets the size-routing default, include/consus_crc32c.h
// mi_crc32c_set_gpu_min).
//
//   route_probe [REPS]      prints one line per size: median us of each path
//
// Both paths are the library's own (mi_crc32c with the threshold forced to
// 0 = GPU, or to 2^64-1 = CPU); results are compared with each other.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "consus_crc32c.h"

namespace {

double now_us()
{
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

double median_us(const unsigned char* p, size_t n, int reps, uint32_t* crc)
{
    std::vector<double> t(reps);
    for (int i = 0; i < 5; ++i) *crc = mi_crc32c(0, p, n);
    for (int i = 0; i < reps; ++i)
    {
        const double t0 = now_us();
        *crc = mi_crc32c(0, p, n);
        t[i] = now_us() - t0;
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

}  // namespace

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    if (mi_crc32c_init(0) != MI_CRC32C_OK)
    {
        fprintf(stderr, "no device: %s\n", mi_crc32c_last_error());
        return 1;
    }
    const size_t maxn = size_t(64) << 20;
    std::vector<unsigned char> buf(maxn);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < maxn; ++i)
    {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        buf[i] = (unsigned char)x;
    }
    int bad = 0;
    printf("%10s %12s %12s %10s\n", "bytes", "gpu_us", "cpu_us", "faster");
    for (size_t n = 16; n <= maxn; n *= 4)
    {
        uint32_t cg = 0, cc = 0;
        const int r = n >= (size_t(16) << 20) ? std::max(reps / 20, 5) : reps;
        mi_crc32c_set_gpu_min(0);
        const double g = median_us(buf.data() + 3, n - 3, r, &cg);
        mi_crc32c_set_gpu_min(UINT64_MAX);
        const double c = median_us(buf.data() + 3, n - 3, r, &cc);
        if (cg != cc) ++bad;
        printf("%10zu %12.2f %12.2f %10s%s\n", n - 3, g, c, g < c ? "gpu" : "cpu",
               cg == cc ? "" : "  MISMATCH");
        fflush(stdout);
    }
    mi_crc32c_stats_t st;
    mi_crc32c_stats(&st);
    printf("gpu_calls %llu host_routed_calls %llu fallback_calls %llu\n",
           (unsigned long long)st.gpu_calls, (unsigned long long)st.host_routed_calls,
           (unsigned long long)st.fallback_calls);
    return bad || st.fallback_calls ? 1 : 0;
}
