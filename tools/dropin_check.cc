// tools/dropin_check.cc -- the drop-in boundary exercised from C++ the way
// Consus's own code uses it, linked against libconsus_crc32c.so only
// (no Python, no oracle):
//   * consus::crc32c as durable_log::append calls it (txman/durable_log.cc:
//     215-218): chained over the 16-byte header, then the entry;
//   * the check value and the n == 0 contract (common/crc32c.cc:122-126);
//   * consus::durable_log open / append / wait / replay / close in a
//     temporary directory, and the frame bytes on disk.
// Prints "dropin ok gpu_calls=G fallback_calls=F" and exits 0, or names the
// first failed check and exits 1.  Without a usable GPU every check must still
// pass (the drop-in is total, as the reference is) with F > 0; on the GPU the
// test asserts F == 0.
// Built by consus_amd/csrc/Makefile; run by tests/test_dropin_cpp.py.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "common/crc32c.h"
#include "consus_crc32c.h"
#include "txman/durable_log.h"

namespace {

int g_fail = 0;

void check(bool ok, const char* what)
{
    if (!ok && !g_fail)
    {
        fprintf(stderr, "dropin check failed: %s\n", what);
        g_fail = 1;
    }
}

void be64(uint64_t v, unsigned char* p)
{
    for (int i = 7; i >= 0; --i, v >>= 8) p[i] = static_cast<unsigned char>(v);
}

struct Replayed
{
    std::vector<std::string> entries;
};

void on_entry(void* p, const unsigned char* e, size_t n)
{
    static_cast<Replayed*>(p)->entries.emplace_back(reinterpret_cast<const char*>(e), n);
}

}  // namespace

int main()
{
    const unsigned char digits[] = "123456789";
    check(consus::crc32c(0, digits, 9) == 0xE3069283u, "check value");
    check(consus::crc32c(0x12345678u, digits, 0) == 0x12345678u, "n == 0 returns init");
    check(consus::crc32c(consus::crc32c(0, digits, 4), digits + 4, 5) == 0xE3069283u,
          "chaining through init");

    // the frame CRC exactly as durable_log::append computes it
    unsigned char hdr[16];
    be64(1, hdr);
    be64(5, hdr + 8);
    const unsigned char hello[] = "hello";
    const uint32_t crc = consus::crc32c(consus::crc32c(0, hdr, 16), hello, 5);
    check(crc == 0x189BA4C0u, "frame crc (golden frame_example)");

    char dir[] = "/tmp/dropin_check_XXXXXX";
    if (!mkdtemp(dir))
    {
        perror("mkdtemp");
        return 1;
    }
    const std::string d(dir);
    {
        consus::durable_log log;
        check(log.open(d + "/log"), "open");
        const char* entries[] = {"hello", "", "a somewhat longer third entry"};
        int64_t last = 0;
        for (const char* e : entries)
        {
            const int64_t r = log.append(e, strlen(e));
            check(r == last + 1, "append returns consecutive record numbers");
            last = r;
        }
        int64_t x = log.durable();
        while (x <= last && log.error() == 0) x = log.wait(x);
        check(log.error() == 0 && x > last, "watermark passes the last record");
        log.close();
        Replayed rp;
        check(log.replay(on_entry, &rp) == 3, "replay count");
        check(rp.entries.size() == 3 && rp.entries[0] == "hello" && rp.entries[1].empty() &&
                  rp.entries[2] == entries[2],
              "replayed entries");
    }
    // frame 1 on disk: [recno BE][len BE]["hello"][crc BE]
    FILE* f = fopen((d + "/log/file_a").c_str(), "rb");
    unsigned char frame[25] = {};
    const size_t got = f ? fread(frame, 1, sizeof(frame), f) : 0;
    if (f) fclose(f);
    const unsigned char want_crc[4] = {0x18, 0x9B, 0xA4, 0xC0};
    check(got == 25 && memcmp(frame, hdr, 16) == 0 && memcmp(frame + 16, hello, 5) == 0 &&
              memcmp(frame + 21, want_crc, 4) == 0,
          "frame bytes on disk");
    for (const char* n : {"/log/file_a", "/log/file_b", "/log/LOCK"}) unlink((d + n).c_str());
    rmdir((d + "/log").c_str());
    rmdir(dir);
    mi_crc32c_stats_t st;
    mi_crc32c_stats(&st);
    if (!g_fail)
        printf("dropin ok gpu_calls=%llu fallback_calls=%llu\n",
               (unsigned long long)st.gpu_calls, (unsigned long long)st.fallback_calls);
    return g_fail;
}
