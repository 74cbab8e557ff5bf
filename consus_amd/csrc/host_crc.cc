// consus_amd/csrc/host_crc.cc -- the engine's CPU path (see host_crc.h).
//
// Used after an engine failure, and for single host calls below the GPU
// threshold (size routing, api.cc).  Same arithmetic as consus::crc32c
// (reflected CRC-32C, poly 0x82F63B78; common/crc32c.cc:122-126): the SSE4.2
// crc32 instruction over 8-byte words where the host has it, a byte-wise
// table otherwise.
#include "host_crc.h"

#include <atomic>
#include <cstring>

#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

#include "../../include/consus_crc32c.h"

namespace mi_host {
namespace {

struct Table
{
    uint32_t t[256];
    Table()
    {
        for (uint32_t b = 0; b < 256; ++b)
        {
            uint32_t s = b;
            for (int k = 0; k < 8; ++k) s = (s >> 1) ^ (0x82F63B78u & (0u - (s & 1u)));
            t[b] = s;
        }
    }
};

uint32_t raw_table(uint32_t s, const uint8_t* p, size_t n)
{
    static const Table tab;
    while (n--) s = tab.t[(s ^ *p++) & 0xFFu] ^ (s >> 8);
    return s;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t raw_hw(uint32_t s, const uint8_t* p, size_t n)
{
    while (n && (uintptr_t(p) & 7u))
    {
        s = _mm_crc32_u8(s, *p++);
        --n;
    }
    uint64_t s64 = s;
    for (; n >= 8; n -= 8, p += 8)
    {
        uint64_t w;
        std::memcpy(&w, p, 8);
        s64 = _mm_crc32_u64(s64, w);
    }
    s = uint32_t(s64);
    while (n--) s = _mm_crc32_u8(s, *p++);
    return s;
}

bool have_sse42()
{
    static const bool ok = __builtin_cpu_supports("sse4.2");
    return ok;
}
#endif

std::atomic<uint64_t> g_gpu_calls{0}, g_fb_calls{0}, g_fb_bytes{0}, g_sharded{0}, g_sorted{0},
    g_routed_calls{0}, g_routed_bytes{0}, g_zero_copy{0}, g_hint_overflow{0},
    g_host_batches{0}, g_host_batch_bytes{0}, g_sorted_one{0}, g_window{0};
std::atomic<int> g_fb_status{0};
std::atomic<int> g_multi_ranges{0};
std::atomic<int> g_multi_devs[MI_CRC32C_MAX_DEVICES];

}  // namespace

uint32_t crc32c(uint32_t init, const void* p, size_t n)
{
    if (n == 0) return init;
    const uint8_t* b = static_cast<const uint8_t*>(p);
#if defined(__x86_64__)
    if (have_sse42()) return ~raw_hw(~init, b, n);
#endif
    return ~raw_table(~init, b, n);
}

void batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
           const uint32_t* inits, size_t count, uint32_t* out)
{
    const uint8_t* b = static_cast<const uint8_t*>(base);
    for (size_t i = 0; i < count; ++i)
        out[i] = crc32c(inits ? inits[i] : 0u, lengths[i] ? b + offsets[i] : b, lengths[i]);
}

void batch_fixed(const void* base, uint64_t stride, uint64_t length, const uint32_t* inits,
                 size_t count, uint32_t* out)
{
    const uint8_t* b = static_cast<const uint8_t*>(base);
    for (size_t i = 0; i < count; ++i)
        out[i] = crc32c(inits ? inits[i] : 0u, b + i * stride, size_t(length));
}

void note_fallback(int status, uint64_t bytes)
{
    g_fb_calls.fetch_add(1, std::memory_order_relaxed);
    g_fb_bytes.fetch_add(bytes, std::memory_order_relaxed);
    g_fb_status.store(status, std::memory_order_relaxed);
}

void note_gpu_call() { g_gpu_calls.fetch_add(1, std::memory_order_relaxed); }
void note_sharded_call() { g_sharded.fetch_add(1, std::memory_order_relaxed); }
void note_sorted_batch(bool one_launch)
{
    g_sorted.fetch_add(1, std::memory_order_relaxed);
    if (one_launch) g_sorted_one.fetch_add(1, std::memory_order_relaxed);
}
void note_window_batch() { g_window.fetch_add(1, std::memory_order_relaxed); }
void note_zero_copy_batch() { g_zero_copy.fetch_add(1, std::memory_order_relaxed); }
void note_hint_overflow() { g_hint_overflow.fetch_add(1, std::memory_order_relaxed); }
void note_host_batch(uint64_t bytes)
{
    g_host_batches.fetch_add(1, std::memory_order_relaxed);
    g_host_batch_bytes.fetch_add(bytes, std::memory_order_relaxed);
}
void note_host_routed(uint64_t bytes)
{
    g_routed_calls.fetch_add(1, std::memory_order_relaxed);
    g_routed_bytes.fetch_add(bytes, std::memory_order_relaxed);
}
void note_multi(int ranges, const int* devices)
{
    for (int i = 0; i < MI_CRC32C_MAX_DEVICES; ++i)
        g_multi_devs[i].store(i < ranges ? devices[i] : -1, std::memory_order_relaxed);
    g_multi_ranges.store(ranges, std::memory_order_relaxed);
}

}  // namespace mi_host

extern "C" {

void mi_crc32c_stats(mi_crc32c_stats_t* out)
{
    if (!out) return;
    out->gpu_calls = mi_host::g_gpu_calls.load();
    out->fallback_calls = mi_host::g_fb_calls.load();
    out->fallback_bytes = mi_host::g_fb_bytes.load();
    out->sharded_calls = mi_host::g_sharded.load();
    out->host_routed_calls = mi_host::g_routed_calls.load();
    out->host_routed_bytes = mi_host::g_routed_bytes.load();
    out->sorted_batches = mi_host::g_sorted.load();
    out->zero_copy_batches = mi_host::g_zero_copy.load();
    out->hint_overflows = mi_host::g_hint_overflow.load();
    out->host_batches = mi_host::g_host_batches.load();
    out->host_batch_bytes = mi_host::g_host_batch_bytes.load();
    out->sorted_one_launch = mi_host::g_sorted_one.load();
    out->window_batches = mi_host::g_window.load();
    out->last_fallback_status = mi_host::g_fb_status.load();
    const int ranges = mi_host::g_multi_ranges.load();
    out->last_multi_ranges = ranges;
    for (int i = 0; i < MI_CRC32C_MAX_DEVICES; ++i)
        out->last_multi_devices[i] = i < ranges ? mi_host::g_multi_devs[i].load() : -1;
}

void mi_crc32c_stats_reset(void)
{
    mi_host::g_gpu_calls.store(0);
    mi_host::g_fb_calls.store(0);
    mi_host::g_fb_bytes.store(0);
    mi_host::g_sharded.store(0);
    mi_host::g_sorted.store(0);
    mi_host::g_zero_copy.store(0);
    mi_host::g_hint_overflow.store(0);
    mi_host::g_host_batches.store(0);
    mi_host::g_host_batch_bytes.store(0);
    mi_host::g_sorted_one.store(0);
    mi_host::g_window.store(0);
    mi_host::g_routed_calls.store(0);
    mi_host::g_routed_bytes.store(0);
    mi_host::g_fb_status.store(0);
    mi_host::g_multi_ranges.store(0);
}

}  // extern "C"
