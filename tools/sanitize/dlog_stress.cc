// tools/sanitize/dlog_stress.cc -- drives the host code of the engine under a
// sanitizer (tools/sanitize/Makefile): the durable log's lock-free
// reservation protocol, flush and sync threads (consus_amd/csrc/durable_log.cc;
// reference concurrency txman/durable_log.cc:187-242), the multi-device
// worker pool and the CPU fallback (api.cc, host_crc.cc).
//
//   1. 8 appenders x 3000 entries (42 B - 9 KiB, every 97th one larger than
//      the staging arena) into logs with small staging buffers (2 KiB,
//      16 KiB, 256 KiB: most flushes cut a full segment), wait for the
//      watermark, replay: every record byte-exact, in order;
//   2. close() while 4 appenders keep appending;
//   3. 4 threads at once calling the total drop-in, FALLBACK batches and
//      multi-device batches (forced split), checked against a bitwise CRC.
// Exits 0 and prints "stress ok" when every check holds.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "consus_crc32c.h"
#include "txman/durable_log.h"

namespace {

std::atomic<int> g_fail{0};

void check(bool ok, const char* what)
{
    if (!ok && g_fail.fetch_add(1) == 0) fprintf(stderr, "stress check failed: %s\n", what);
}

uint32_t bitwise_crc(uint32_t init, const unsigned char* p, size_t n)
{
    uint32_t s = ~init;
    for (size_t i = 0; i < n; ++i)
    {
        s ^= p[i];
        for (int k = 0; k < 8; ++k) s = (s >> 1) ^ (0x82F63B78u & (0u - (s & 1u)));
    }
    return ~s;
}

uint64_t mix(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

std::string entry_for(unsigned t, unsigned i, size_t cap)
{
    const uint64_t h = mix(uint64_t(t) << 32 | i);
    size_t n = 42 + h % 9000;
    if (i % 97 == 13) n = cap + h % 5000;  // larger than the staging arena
    std::string e(n, '\0');
    for (size_t k = 0; k < n; ++k) e[k] = char(mix(h + k) & 0xFF);
    return e;
}

struct Replayed
{
    std::vector<std::string> v;
};

void on_entry(void* p, const unsigned char* e, size_t n)
{
    static_cast<Replayed*>(p)->v.emplace_back(reinterpret_cast<const char*>(e), n);
}

void wait_for(consus::durable_log& log, int64_t upto)
{
    int64_t x = log.durable();
    while (x <= upto && log.error() == 0) x = log.wait(x);
}

void stress_appenders(const std::string& dir, size_t cap)
{
    consus::durable_log log(cap);
    check(log.open(dir), "open");
    const unsigned threads = 8, per = 3000;
    std::mutex mu;
    std::map<int64_t, std::string> got;
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
            std::vector<std::pair<int64_t, std::string>> mine;
            for (unsigned i = 0; i < per; ++i)
            {
                std::string e = entry_for(t, i, cap);
                const int64_t r = log.append(e.data(), e.size());
                check(r > 0, "append");
                mine.emplace_back(r, std::move(e));
            }
            std::lock_guard<std::mutex> hold(mu);
            for (auto& m : mine) got.emplace(m.first, std::move(m.second));
        });
    for (auto& t : ts) t.join();
    const int64_t n = int64_t(threads) * per;
    check(int64_t(got.size()) == n && got.begin()->first == 1 && got.rbegin()->first == n,
          "record numbers 1..n, each once");
    wait_for(log, n);
    check(log.error() == 0, "no log error");
    log.close();
    Replayed rp;
    check(log.replay(on_entry, &rp) == n, "replay count");
    bool same = int64_t(rp.v.size()) == n;
    for (int64_t r = 1; same && r <= n; ++r) same = rp.v[size_t(r - 1)] == got[r];
    check(same, "replayed entries byte-exact in record order");
}

void stress_close(const std::string& dir)
{
    consus::durable_log log(size_t(1) << 15);
    check(log.open(dir), "open (close test)");
    std::atomic<bool> stop{false};
    int64_t before = 0;
    for (int i = 0; i < 50; ++i) before = log.append("xxxxxxxxxxxxxxxx", 16);
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t)
        ts.emplace_back([&] {
            while (!stop.load() && log.append("yyyyyyyyyyyyyyyyyyyyyyyyy", 25) > 0)
            {
            }
        });
    log.close();
    stop.store(true);
    for (auto& t : ts) t.join();
    check(log.durable() > before, "close drained the records reserved before it");
    check(log.append("late", 4) < 0, "append after close fails");
}

void stress_engine_calls()
{
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t)
        ts.emplace_back([t] {
            std::vector<unsigned char> buf(1 << 20);
            for (size_t k = 0; k < buf.size(); ++k) buf[k] = (unsigned char)(mix(t * 7919 + k));
            std::vector<uint64_t> off;
            std::vector<uint32_t> len, want;
            for (uint64_t o = 0; o + 9000 < buf.size(); o += 9000)
            {
                off.push_back(o + (o % 13));
                len.push_back(uint32_t(o % 8000));
            }
            for (size_t i = 0; i < off.size(); ++i)
                want.push_back(bitwise_crc(0, buf.data() + off[i], len[i]));
            for (int rep = 0; rep < 6; ++rep)
            {
                std::vector<uint32_t> out(off.size());
                check(mi_crc32c(0, buf.data() + 5, 1000) == bitwise_crc(0, buf.data() + 5, 1000),
                      "drop-in");
                check(mi_crc32c_batch(buf.data(), off.data(), len.data(), nullptr, off.size(), 0,
                                      out.data(), MI_CRC32C_FALLBACK) == MI_CRC32C_OK &&
                          out == want,
                      "fallback batch");
                const int devs[3] = {0, 1, 0};
                out.assign(off.size(), 0);
                check(mi_crc32c_batch_multi(buf.data(), off.data(), len.data(), nullptr,
                                            off.size(), 0, out.data(), MI_CRC32C_FALLBACK, devs, 3,
                                            1) == MI_CRC32C_OK &&
                          out == want,
                      "multi-device batch");
            }
        });
    for (auto& t : ts) t.join();
}

}  // namespace

int main(int argc, char** argv)
{
    char tmpl[] = "/tmp/dlog_stress_XXXXXX";
    const char* root = argc > 1 ? argv[1] : mkdtemp(tmpl);
    if (!root)
    {
        perror("mkdtemp");
        return 2;
    }
    const std::string r(root);
    if (argc > 1 && mkdir(root, 0700) < 0 && errno != EEXIST)
    {
        perror("mkdir");
        return 2;
    }
    int k = 0;
    for (size_t cap : {size_t(2048), size_t(16384), size_t(256) << 10})
        stress_appenders(r + "/a" + std::to_string(k++), cap);
    stress_close(r + "/c");
    stress_engine_calls();
    std::string cmd = "rm -rf '" + r + "'";
    if (system(cmd.c_str()) != 0) fprintf(stderr, "cleanup of %s failed\n", root);
    mi_crc32c_stats_t st;
    mi_crc32c_stats(&st);
    if (g_fail.load()) return 1;
    printf("stress ok gpu_calls=%llu fallback_calls=%llu sharded_calls=%llu\n",
           (unsigned long long)st.gpu_calls, (unsigned long long)st.fallback_calls,
           (unsigned long long)st.sharded_calls);
    return 0;
}
