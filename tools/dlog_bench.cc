// tools/dlog_bench.cc -- throughput of the batching durable-log front-end
// (include/txman/durable_log.h; reference txman/durable_log.cc:187-242 append,
// :287-347 flush) driven the way txman drives it: T network threads call
// append() concurrently (txman/main.cc:191-193), then the caller waits for the
// watermark to cover every record (daemon::durable, durable_log::wait).
//
//   dlog_bench DIR THREADS APPENDS_PER_THREAD MIN_ENTRY MAX_ENTRY [SEGMENT_BYTES]
//
// Entry lengths are uniform in [MIN_ENTRY, MAX_ENTRY] from a splitmix64
// stream, entry bytes are slices of one splitmix64 pool.  After the timed
// region the log is closed and replayed (a GPU-verified scan of both segment
// files): every record must come back, in recno order, byte-exact.
// Prints one JSON line.
//
// Engines of the flush thread's batch CRC: the GPU (default; flushes below
// the log's host_batch_max take the flush thread's CPU, MI_DLOG_HOST_BATCH_MAX
// overrides); with REF_CRC_SO=path/to/oracle/_ref/libref_crc32c.so the
// reference common/crc32c.cc itself (compiled unmodified, bench.py's CPU
// leg), called per frame on the flush thread -- the same front-end with a
// CPU checksum, timed in the same run.  With REF_SCHEME=1 as well, the
// reference's own placement instead (txman/durable_log.cc:215-218): every
// appender computes its frame's CRC with the reference function on its own
// thread, outside any lock, and the flush thread checksums nothing.
//
// DLOG_ENTRY=zipf: entry lengths from the configs[2] distribution (Zipf,
// 64 B - 64 KiB, mi_workload_zipf_lengths) instead of uniform in
// [MIN_ENTRY, MAX_ENTRY].
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "consus_crc32c.h"
#include "txman/durable_log.h"

namespace {

uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef uint32_t (*ref_crc32c_fn)(uint32_t, const unsigned char*, size_t);
ref_crc32c_fn g_ref = nullptr;

int ref_batch(void*, const void* base, const uint64_t* off, const uint32_t* len, size_t n, uint64_t,
              uint32_t* out)
{
    const unsigned char* b = static_cast<const unsigned char*>(base);
    for (size_t i = 0; i < n; ++i) out[i] = g_ref(0, b + off[i], len[i]);
    return 0;
}

double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Replay
{
    const std::vector<uint32_t>* len;  // entry length of recno r (1-based) at r - 1
    const std::vector<uint64_t>* at;   // pool offset of recno r's entry
    const unsigned char* pool;
    uint64_t next = 0;
    uint64_t bad = 0;
};

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 6)
    {
        fprintf(stderr,
                "usage: %s DIR THREADS APPENDS_PER_THREAD MIN_ENTRY MAX_ENTRY [SEGMENT_BYTES "
                "[FSYNC_DELAY_US]]\n",
                argv[0]);
        return 2;
    }
    const std::string dir = argv[1];
    const int threads = atoi(argv[2]);
    const uint64_t per = strtoull(argv[3], nullptr, 10);
    uint32_t lo = uint32_t(atoi(argv[4])), hi = uint32_t(atoi(argv[5]));
    const size_t seg = argc > 6 ? size_t(strtoull(argv[6], nullptr, 10)) : 0;
    // a slower disk than tmpfs: every fsync also sleeps this long
    const uint32_t fsync_delay = argc > 7 ? uint32_t(strtoul(argv[7], nullptr, 10)) : 0;
    // diagnosis only: FAKE_CRC=1 replaces the GPU batch with a no-op (CRCs
    // left zero, replay not checked) to time the front-end alone
    const bool fake = getenv("FAKE_CRC") && atoi(getenv("FAKE_CRC"));
    const bool ref_scheme = getenv("REF_SCHEME") && atoi(getenv("REF_SCHEME"));
    const bool zipf = getenv("DLOG_ENTRY") && !strcmp(getenv("DLOG_ENTRY"), "zipf");
    if (zipf) lo = 64, hi = 65536;
    if (threads < 1 || per < 1 || hi < lo)
    {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    // entry pool: 64 MiB of splitmix64 bytes; entry k of thread t starts at a
    // stream-chosen offset
    const size_t pool_bytes = (64u << 20) + hi;
    std::vector<unsigned char> pool(pool_bytes);
    for (size_t i = 0; i < pool_bytes / 8; ++i)
    {
        const uint64_t w = splitmix64(0xD106ull ^ i);
        memcpy(&pool[i * 8], &w, 8);
    }
    std::vector<std::vector<uint32_t>> lens(threads, std::vector<uint32_t>(per));
    std::vector<std::vector<uint64_t>> offs(threads, std::vector<uint64_t>(per));
    uint64_t entry_bytes = 0;
    // configs[2]'s lengths: thread t takes records t*per .. of the stream
    if (zipf)
        for (int t = 0; t < threads; ++t)
            mi_workload_zipf_lengths(0x5EED, uint64_t(t) * per, per, lens[t].data());
    for (int t = 0; t < threads; ++t)
        for (uint64_t k = 0; k < per; ++k)
        {
            const uint64_t r = splitmix64((uint64_t(t) << 40) ^ k ^ 0x5EEDull);
            if (!zipf) lens[t][k] = lo + uint32_t(r % (hi - lo + 1));
            offs[t][k] = (r >> 20) % (pool_bytes - hi);
            entry_bytes += lens[t][k];
        }

    std::vector<std::pair<size_t, double>> g_link;  // (bytes, us) of pinned-to-device copies
    std::vector<std::pair<size_t, double>> g_cpu;   // (bytes, us) of the CPU path's batch
    const char* ref_so = getenv("REF_CRC_SO");
    if (ref_so && *ref_so)
    {
        void* h = dlopen(ref_so, RTLD_NOW | RTLD_LOCAL);
        g_ref = h ? reinterpret_cast<ref_crc32c_fn>(dlsym(h, "ref_crc32c")) : nullptr;
        if (!g_ref)
        {
            fprintf(stderr, "REF_CRC_SO=%s: %s\n", ref_so, dlerror());
            return 2;
        }
    }
    // the floor of one flush's GPU batch: the round trip of a one-frame batch
    // from mapped pinned memory through the log's engine entry point
    double empty_us = 0;
    // DLOG_NO_PROBES=1: skip these one-off probes (repeated runs of a bench)
    if (!g_ref && !fake && !(getenv("DLOG_NO_PROBES") && atoi(getenv("DLOG_NO_PROBES"))))
    {
        void* pin = nullptr;
        if (mi_host_malloc_pinned(&pin, 4096) == MI_CRC32C_OK)
        {
            memset(pin, 7, 4096);
            const uint64_t o = 0;
            const uint32_t l = 64;
            uint32_t c = 0;
            std::vector<double> t;
            for (int i = 0; i < 220; ++i)
            {
                const double a = now();
                mi_crc32c_batch_multi(pin, &o, &l, nullptr, 1, 64, &c, MI_CRC32C_FALLBACK, nullptr,
                                      0, 0);
                if (i >= 20) t.push_back((now() - a) * 1e6);
            }
            std::sort(t.begin(), t.end());
            empty_us = t[t.size() / 2];
            mi_host_free_pinned(pin);
        }
        // the host link as a flush sees it: a synchronous copy of n bytes of
        // pinned memory to the device, median of 40, at flush-like sizes
        void* hp = nullptr;
        void* dp = nullptr;
        const size_t big = size_t(16) << 20;
        if (mi_host_malloc_pinned(&hp, big) == MI_CRC32C_OK && mi_dev_malloc(&dp, big) == MI_CRC32C_OK)
        {
            memset(hp, 3, big);
            for (size_t n : {size_t(64) << 10, size_t(256) << 10, size_t(1) << 20, size_t(4) << 20,
                             size_t(16) << 20})
            {
                std::vector<double> t;
                for (int i = 0; i < 45; ++i)
                {
                    const double a = now();
                    mi_memcpy(dp, hp, n, MI_MEMCPY_H2D);
                    if (i >= 5) t.push_back((now() - a) * 1e6);
                }
                std::sort(t.begin(), t.end());
                g_link.push_back({n, t[t.size() / 2]});
            }
        }
        // the flush thread's CPU path as a routed flush sees it: frames of
        // the run's entry sizes checksummed by mi_crc32c_batch(MI_CRC32C_CPU)
        if (hp)
        {
            const unsigned char* b = static_cast<const unsigned char*>(hp);
            for (size_t n : {size_t(64) << 10, size_t(256) << 10, size_t(1) << 20, size_t(4) << 20})
            {
                std::vector<uint64_t> o;
                std::vector<uint32_t> l;
                for (uint64_t at = 0, k = 0; at < n; ++k)
                {
                    const uint32_t e = std::min<uint64_t>(
                        16 + (zipf ? 4700 : (lo + hi) / 2) + 4, n - at);
                    o.push_back(at);
                    l.push_back(e > 4 ? e - 4 : e);
                    at += e;
                }
                std::vector<uint32_t> c(o.size());
                std::vector<double> t;
                for (int i = 0; i < 25; ++i)
                {
                    const double a = now();
                    mi_crc32c_batch(b, o.data(), l.data(), nullptr, o.size(), 0, c.data(), MI_CRC32C_CPU);
                    if (i >= 5) t.push_back((now() - a) * 1e6);
                }
                std::sort(t.begin(), t.end());
                g_cpu.push_back({n, t[t.size() / 2]});
            }
        }
        if (dp) mi_dev_free(dp);
        if (hp) mi_host_free_pinned(hp);
    }
    consus::durable_log log(seg);
    // watchdog: a stage that takes more than DLOG_STAGE_LIMIT s (default 60)
    // prints where the run is and the log's counters, then ends the process
    std::atomic<int> stage{0};
    static const char* const kStage[] = {"open", "append", "durable", "monitor", "replay", "close",
                                         "done"};
    std::atomic<bool> wd_stop{false};
    const double wd_limit = getenv("DLOG_STAGE_LIMIT") ? atof(getenv("DLOG_STAGE_LIMIT")) : 60.0;
    std::thread watchdog([&] {
        int last = -1;
        double since = now();
        while (!wd_stop.load())
        {
            usleep(100000);
            const int st = stage.load();
            if (st != last) last = st, since = now();
            if (now() - since > wd_limit)
            {
                double f[6], m[6];
                log.flush_seconds(f);
                log.flush_max_seconds(m);
                char st_line[512];
                log.debug_state(st_line, sizeof st_line);
                fprintf(stderr,
                        "dlog_bench: stage '%s' exceeded %.0f s: durable %lld, flushes %llu, frames "
                        "flushed %llu, error %d; flush s: wait %.3f walk %.3f crc %.3f patch %.3f "
                        "pwrite %.3f fsync %.3f; max us: %.0f %.0f %.0f %.0f %.0f %.0f\n"
                        "dlog_bench: state: %s\n",
                        kStage[st], wd_limit, (long long)log.durable(),
                        (unsigned long long)log.flushes(),
                        (unsigned long long)log.frames_flushed(), log.error(), f[0], f[1], f[2],
                        f[3], f[4], f[5], m[0] * 1e6, m[1] * 1e6, m[2] * 1e6, m[3] * 1e6,
                        m[4] * 1e6, m[5] * 1e6, st_line);
                fflush(stderr);
                _exit(3);
            }
        }
    });
    if (g_ref && ref_scheme)
    {
        // the reference scheme: the appenders checksum, the flush thread
        // does not (the batch engine stays the default: the replay's scan)
        log.set_append_crc_for_testing(g_ref);
    }
    else if (g_ref)
        log.set_batch_crc_for_testing(ref_batch, nullptr);
    if (fake)
        log.set_batch_crc_for_testing(
            [](void*, const void*, const uint64_t*, const uint32_t*, size_t n, uint64_t,
               uint32_t* out) {
                memset(out, 0, n * 4);
                return 0;
            },
            nullptr);
    log.set_fsync_delay_for_testing(fsync_delay);
    // DLOG_PINNED=0/1: ordinary or pinned staging arenas whatever the engine
    // (an injected engine defaults to ordinary memory, the GPU batch to pinned)
    if (const char* e = getenv("DLOG_PINNED")) log.set_pinned_arenas_for_testing(atoi(e) != 0);
    // DLOG_SINK=1: no pwrite, no fsync (storage faster than the front-end);
    // nothing to replay then
    const bool sink = getenv("DLOG_SINK") && atoi(getenv("DLOG_SINK"));
    if (sink) log.set_sink_for_testing(true);
    const double t_open = now();
    if (!log.open(dir))
    {
        fprintf(stderr, "open(%s) failed: %s\n", dir.c_str(), strerror(log.error()));
        return 1;
    }
    // recno -> (thread, k) so the replay can be checked
    const uint64_t total = uint64_t(threads) * per;
    std::vector<uint32_t> rec_len(total);
    std::vector<uint64_t> rec_at(total);
    // each appender records its recnos in its own array and the recno-indexed
    // tables are filled after the timed region: stores indexed by recno from
    // every thread would share cache lines (consecutive recnos belong to
    // different threads) and bench the bookkeeping's false sharing, not the log
    std::vector<std::vector<int64_t>> got(threads, std::vector<int64_t>(per, 0));
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::atomic<uint64_t> failures{0};
    std::vector<std::thread> ths;
    // durability latency: every 64th append's return time against the first
    // watermark the monitor sees that covers it (commit latency of txman)
    std::vector<std::vector<std::pair<int64_t, double>>> samples(threads);
    std::vector<std::pair<double, int64_t>> marks;
    std::atomic<bool> stop{false};
    for (int t = 0; t < threads; ++t)
        ths.emplace_back([&, t] {
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            for (uint64_t k = 0; k < per; ++k)
            {
                const int64_t r = log.append(&pool[offs[t][k]], lens[t][k]);
                if (r <= 0 || uint64_t(r) > total)
                {
                    failures.fetch_add(1);
                    continue;
                }
                if ((k & 63) == 0) samples[t].emplace_back(r, now());
                got[t][k] = r;
            }
        });
    std::thread monitor([&] {
        int64_t w = log.durable();
        while (!stop.load())
        {
            w = log.wait(w);
            marks.emplace_back(now(), w);
            if (log.error()) break;
        }
    });
    while (ready.load() < threads) std::this_thread::yield();
    const double t0 = now();
    stage.store(1);
    go.store(true, std::memory_order_release);
    for (auto& th : ths) th.join();
    const double t_appended = now();
    stage.store(2);
    int64_t x = log.durable();
    while (x <= int64_t(total) && !log.error()) x = log.wait(x);
    const double t_durable = now();
    stage.store(3);
    stop.store(true);
    log.wake();
    monitor.join();
    stage.store(4);
    for (int t = 0; t < threads; ++t)
        for (uint64_t k = 0; k < per; ++k)
            if (const int64_t r = got[t][k]; r > 0 && uint64_t(r) <= total)
            {
                rec_len[r - 1] = lens[t][k];
                rec_at[r - 1] = offs[t][k];
            }
    std::vector<double> lat;
    double worst = -1, worst_at = 0;  // the longest wait and when (s after the start) it began
    for (const auto& v : samples)
        for (const auto& [r, ta] : v)
        {
            // first mark whose watermark exceeds r (marks are in watermark order)
            auto it = std::upper_bound(marks.begin(), marks.end(), r,
                                       [](int64_t rr, const std::pair<double, int64_t>& m) {
                                           return rr < m.second;
                                       });
            if (it != marks.end())
            {
                lat.push_back(std::max(0.0, it->first - ta) * 1e6);
                if (lat.back() > worst) worst = lat.back(), worst_at = ta - t0;
            }
        }
    std::sort(lat.begin(), lat.end());
    auto pct = [&](double q) { return lat.empty() ? 0.0 : lat[size_t(q * (lat.size() - 1))]; };
    const uint64_t flushes = log.flushes(), frames = log.frames_flushed();
    const uint64_t host_flushes = log.host_flushes();
    const int err = log.error();
    double fs[6], fm[6];
    log.flush_seconds(fs);
    log.flush_max_seconds(fm);
    // DLOG_TIMELINE=path: the per-flush timeline (durable_log::flush_timeline)
    // as text, after a header line with the run's own marks, all in seconds
    // since open(): appends started, appends returned, everything durable
    if (const char* tp = getenv("DLOG_TIMELINE"))
        if (FILE* f = fopen(tp, "w"))
        {
            std::vector<double> rows(size_t(1 << 14) * 7);
            const size_t nr = log.flush_timeline(rows.data(), size_t(1) << 14);
            fprintf(f, "# start %.6f appended %.6f durable %.6f\n", t0 - t_open, t_appended - t_open,
                    t_durable - t_open);
            fprintf(f, "# sealed checksummed queued write_start write_end synced bytes\n");
            for (size_t i = 0; i < nr; ++i)
                fprintf(f, "%.6f %.6f %.6f %.6f %.6f %.6f %.0f\n", rows[i * 7], rows[i * 7 + 1],
                        rows[i * 7 + 2], rows[i * 7 + 3], rows[i * 7 + 4], rows[i * 7 + 5],
                        rows[i * 7 + 6]);
            fclose(f);
        }

    // the replay: every record back, in order, byte-exact
    Replay rp{&rec_len, &rec_at, pool.data()};
    const int64_t n = fake || sink ? int64_t(total) : log.replay(
        [](void* p, const unsigned char* data, size_t len) {
            Replay* r = static_cast<Replay*>(p);
            const uint64_t i = r->next++;
            if (i >= r->len->size() || len != (*r->len)[i] ||
                memcmp(data, r->pool + (*r->at)[i], len) != 0)
                ++r->bad;
        },
        &rp);
    stage.store(5);
    log.close();
    stage.store(6);
    wd_stop.store(true);
    watchdog.join();
    const uint64_t frame_bytes = entry_bytes + total * 20;
    std::string link = "{";
    for (size_t i = 0; i < g_link.size(); ++i)
    {
        char b[64];
        snprintf(b, sizeof b, "%s\"%zu\": %.2f", i ? ", " : "", g_link[i].first, g_link[i].second);
        link += b;
    }
    link += "}";
    std::string cpu = "{";
    for (size_t i = 0; i < g_cpu.size(); ++i)
    {
        char b[64];
        snprintf(b, sizeof b, "%s\"%zu\": %.2f", i ? ", " : "", g_cpu[i].first, g_cpu[i].second);
        cpu += b;
    }
    cpu += "}";
    printf("{\"sink\": %s, \"engine\": \"%s\", \"entries\": \"%s\", \"host_flushes\": %llu, \"cpu_batch_us\": %s, \"link_us\": %s, \"empty_batch_us\": %.2f, \"threads\": %d, \"appends\": %llu, \"entry_bytes\": %llu, \"frame_bytes\": %llu, "
           "\"append_s\": %.6f, \"durable_s\": %.6f, \"appends_per_s\": %.1f, "
           "\"frame_GiB_per_s\": %.4f, \"flushes\": %llu, \"frames_flushed\": %llu, "
           "\"failures\": %llu, \"error\": %d, \"replayed\": %lld, \"replay_bad\": %llu, "
           "\"flush_s\": {\"copy_wait\": %.4f, \"walk\": %.4f, \"batch_crc\": %.4f, "
           "\"patch\": %.4f, \"pwrite\": %.4f, \"fsync\": %.4f}, "
           "\"flush_max_us\": {\"copy_wait\": %.1f, \"walk\": %.1f, \"batch_crc\": %.1f, "
           "\"patch\": %.1f, \"pwrite\": %.1f, \"fsync\": %.1f}, "
           "\"durable_latency_us\": {\"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f, "
           "\"max_at_s\": %.4f, \"samples\": %zu}}\n",
           sink ? "true" : "false", fake ? "none" : g_ref ? (ref_scheme ? "reference-scheme" : "reference-cpu") : "gpu",
           zipf ? "zipf 64 B - 64 KiB" : "uniform", (unsigned long long)host_flushes, cpu.c_str(), link.c_str(),
           empty_us, threads,
           (unsigned long long)total,
           (unsigned long long)entry_bytes,
           (unsigned long long)frame_bytes, t_appended - t0, t_durable - t0,
           double(total) / (t_durable - t0), double(frame_bytes) / (t_durable - t0) / (1u << 30),
           (unsigned long long)flushes, (unsigned long long)frames,
           (unsigned long long)failures.load(), err, (long long)n, (unsigned long long)rp.bad,
           fs[0], fs[1], fs[2], fs[3], fs[4], fs[5], fm[0] * 1e6, fm[1] * 1e6, fm[2] * 1e6,
           fm[3] * 1e6, fm[4] * 1e6, fm[5] * 1e6, pct(0.5), pct(0.99),
           lat.empty() ? 0.0 : lat.back(), worst_at, lat.size());
    return (failures.load() || err || n != int64_t(total) || rp.bad) ? 1 : 0;
}
