// consus_amd/csrc/durable_log.cc -- the record-batching durable log.
//
// Re-implements txman/durable_log.cc (rescrv/Consus) around the MI355X CRC
// engine; see include/txman/durable_log.h for the contract.  Kept from the
// reference: two segment files, record numbers from 1 in append order, a
// flush thread with all signals blocked (:287-347) that fsyncs one segment
// while appends go to the other, and the watermark "every recno < x is
// durable" (:421-440).  Changed: append() reserves (record number, staging
// offset) with one fetch-and-add on the active segment instead of two
// m_mtx sections (:195-213, :232-239) -- under 8 appending threads the lock
// hand-offs cut throughput ~9x -- and stages the frame in pinned memory; the
// flush thread checksums each sealed segment in one GPU batch (read in place
// from the mapped staging arena), a writer thread pwrites it while the next
// segment is checksummed (the arena rotates through a third, spare one), and
// a sync thread fsyncs it and publishes the watermark.

#include "../../include/txman/durable_log.h"

#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <new>

#include "../../include/consus_crc32c.h"
#include "../../include/consus_durable_log.h"
#include "host_crc.h"

using consus::durable_log;

namespace {

constexpr size_t kHeader = 2 * sizeof(uint64_t);  // RECORD_HEADER_SIZE, txman/durable_log.cc:54
constexpr size_t kTrailer = sizeof(uint32_t);
constexpr size_t kDefaultCapacity = size_t(64) << 20;

void pack64be(uint64_t v, unsigned char* p)
{
    for (int i = 0; i < 8; ++i) p[i] = (unsigned char)(v >> (56 - 8 * i));
}

void pack32be(uint32_t v, unsigned char* p)
{
    for (int i = 0; i < 4; ++i) p[i] = (unsigned char)(v >> (24 - 8 * i));
}

uint64_t unpack64be(const unsigned char* p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return v;
}

uint32_t unpack32be(const unsigned char* p)
{
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) v = (v << 8) | p[i];
    return v;
}

// The default batch engine: the GPU, sharded over the configured devices for
// large segments (mi_crc32c_batch_multi applies the amortisation threshold),
// completed on the engine's CPU path if the GPU fails (MI_CRC32C_FALLBACK:
// the log never turns an engine failure into EIO; the fallback is counted in
// mi_crc32c_stats).
int gpu_batch(void* ctx, const void* base, const uint64_t* off, const uint32_t* len, size_t n,
              uint64_t total, uint32_t* out)
{
    const auto* o = static_cast<const consus::durable_log_options*>(ctx);
    const int gpus = o ? o->gpus : 0;
    if (gpus == 1)
        return mi_crc32c_batch(base, off, len, nullptr, n, total, out, MI_CRC32C_FALLBACK);
    return mi_crc32c_batch_multi(base, off, len, nullptr, n, total, out, MI_CRC32C_FALLBACK,
                                 nullptr, gpus, o ? o->shard_min_bytes : 0);
}

// Frames longer than this are checksummed one by one (single-buffer path)
// rather than inside a batch, whose lengths are 32-bit.
constexpr uint64_t kBatchFrameMax = uint64_t(1) << 30;

// Flushes below this many frame bytes are checksummed on the flush thread's
// CPU (the engine's crc32q loop, MI_CRC32C_CPU): the GPU batch's floor (a
// launch, zero-copy reads over PCIe and the completion word, ~11.5 us) costs
// more there than the CPU loop (~19 GB/s on the GPU box's EPYC 9575F).
// Measured per flush size with tools/flush_probe, medians of 1,000
// (profiles/r05_flush_probe.txt): 215 KB 19.6 us GPU / 10.9 CPU, 429 KB
// 25.6 / 21.9, 569 KB 29.9 / 29.2, 1.12 MB 44.3 / 58.6; they cross near
// 550 KB.
constexpr uint64_t kHostBatchMaxDefault = uint64_t(512) << 10;

uint64_t host_batch_max(const consus::durable_log_options& o)
{
    if (const char* e = std::getenv("MI_DLOG_HOST_BATCH_MAX"))
        return std::strtoull(e, nullptr, 10);
    return o.host_batch_max < 0 ? kHostBatchMaxDefault : uint64_t(o.host_batch_max);
}

bool pwrite_all(int fd, const unsigned char* p, size_t n, off_t off)
{
    while (n)
    {
        const ssize_t w = ::pwrite(fd, p, n, off);
        if (w < 0)
        {
            if (errno == EINTR) continue;
            return false;
        }
        p += w;
        n -= size_t(w);
        off += w;
    }
    return true;
}

struct Frame
{
    uint64_t recno;
    uint64_t offset;  // of the frame in the file / buffer
    uint64_t length;  // of the entry
};

// Parse frames by their length chain and verify every CRC: frames up to
// kBatchFrameMax in one batch, longer ones one by one (`single`).  Returns the
// number of leading complete, CRC-valid frames, or -1 if the engine failed.
// A torn tail or the first bad CRC ends the scan.
template <typename Single>
int64_t scan_frames(const unsigned char* buf, uint64_t size, consus::durable_log_batch_crc fn,
                    void* ctx, Single single, std::vector<Frame>* frames, uint64_t* valid_bytes)
{
    std::vector<uint64_t> offs, recnos, lens;
    std::vector<uint32_t> stored;
    uint64_t pos = 0;
    while (size - pos >= kHeader + kTrailer)
    {
        const uint64_t recno = unpack64be(buf + pos);
        const uint64_t len = unpack64be(buf + pos + 8);
        if (len > size - pos - kHeader - kTrailer) break;  // torn
        offs.push_back(pos);
        lens.push_back(kHeader + len);
        stored.push_back(unpack32be(buf + pos + kHeader + len));
        recnos.push_back(recno);
        pos += kHeader + len + kTrailer;
    }
    std::vector<uint32_t> crcs(offs.size());
    std::vector<uint64_t> boffs;
    std::vector<uint32_t> blens;
    std::vector<size_t> which;
    uint64_t total = 0;
    for (size_t i = 0; i < offs.size(); ++i)
    {
        if (lens[i] > kBatchFrameMax)
        {
            crcs[i] = single(buf + offs[i], lens[i]);
            continue;
        }
        boffs.push_back(offs[i]);
        blens.push_back(uint32_t(lens[i]));
        which.push_back(i);
        total += lens[i];
    }
    std::vector<uint32_t> bcrcs(boffs.size());
    if (!boffs.empty() &&
        fn(ctx, buf, boffs.data(), blens.data(), boffs.size(), total, bcrcs.data()) != 0)
        return -1;
    for (size_t j = 0; j < which.size(); ++j) crcs[which[j]] = bcrcs[j];
    size_t good = 0;
    uint64_t bytes = 0;
    while (good < offs.size() && crcs[good] == stored[good])
    {
        if (frames) frames->push_back(Frame{recnos[good], offs[good], lens[good] - kHeader});
        bytes += lens[good] + kTrailer;
        ++good;
    }
    if (valid_bytes) *valid_bytes = bytes;
    return int64_t(good);
}

// A batch engine whose failures the engine's CPU path completes (counted).
struct Chained
{
    consus::durable_log_batch_crc fn;
    void* ctx;
};

int batch_or_host(void* c, const void* base, const uint64_t* off, const uint32_t* len, size_t n,
                  uint64_t total, uint32_t* out)
{
    const auto* ch = static_cast<const Chained*>(c);
    if (ch->fn(ch->ctx, base, off, len, n, total, out) == 0) return 0;
    mi_host::batch(base, off, len, nullptr, n, out);
    mi_host::note_fallback(MI_CRC32C_EHIP, total);
    return 0;
}

// One frame's CRC on the engine's single-buffer path (completes on the CPU
// path if the GPU fails).
uint32_t single_crc(const unsigned char* p, uint64_t n)
{
    uint32_t c = 0;
    if (mi_crc32c_buffer(0, p, size_t(n), &c, MI_CRC32C_FALLBACK) != MI_CRC32C_OK)
    {
        c = mi_host::crc32c(0, p, size_t(n));
        mi_host::note_fallback(MI_CRC32C_EINVAL, n);
    }
    return c;
}

bool read_file(int dirfd, const char* name, std::vector<unsigned char>* out)
{
    const int fd = dirfd >= 0 ? openat(dirfd, name, O_RDONLY) : ::open(name, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) < 0)
    {
        ::close(fd);
        return false;
    }
    out->resize(size_t(st.st_size));
    size_t got = 0;
    while (got < out->size())
    {
        const ssize_t r = ::pread(fd, out->data() + got, out->size() - got, off_t(got));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) break;
        got += size_t(r);
    }
    ::close(fd);
    out->resize(got);
    return true;
}

}  // namespace

// Reservation word of a segment: bit 63 = sealed (no more appends), bits
// 40..62 = frames reserved, bits 0..39 = staged bytes reserved.  An append
// takes its slot with one fetch-and-add (under 8-16 appending threads a
// compare-and-swap loop measured half the append rate), so frames sit back
// to back in the arena in reservation order and frame i has record number
// base + i.  When the segment fills, the adds past the end fail and the
// first failure marks the cut.
constexpr uint64_t kSealed = uint64_t(1) << 63;
constexpr int kIdxShift = 40;
constexpr uint64_t kUsedMask = (uint64_t(1) << kIdxShift) - 1;
constexpr uint64_t kMaxFrames = (uint64_t(1) << (63 - kIdxShift)) - 1;
constexpr unsigned kDoneShards = 16;
// at_slot(i) of a frame staged outside the arena (see segment::ext)
constexpr uint64_t kExternal = uint64_t(1) << 63;

struct durable_log::segment
{
    int fd = -1;
    unsigned char* arena = nullptr;  // frames staged since the last flush
    size_t cap = 0;
    uint64_t file_size = 0;          // bytes already written to the file (flush thread)
    uint64_t base = 0;               // record number of frame 0; set before unsealing
    // staging offset of frame i, written by its appender at at_slot(i): the
    // flush thread reads the offsets as 8 sequential streams instead of
    // walking the frames' length chain (a dependent cache miss per frame:
    // 150 ns, 58 % of the flush thread under 8 appenders).  Consecutive frames
    // land in 8 different regions, so concurrent appenders rarely write the
    // same cache line.
    uint64_t* at = nullptr;
    uint64_t slots = 0;              // capacity in frames (a multiple of 8)
    uint64_t& at_slot(uint64_t i) { return at[(i & 7) * (slots >> 3) + (i >> 3)]; }
    alignas(64) std::atomic<uint64_t> word{kSealed};  // every append's one atomic: own line
    // (index << 40) | offset of the first reservation that did not fit
    alignas(64) std::atomic<uint64_t> cut{~uint64_t(0)};
    std::atomic<uint64_t> failed{0};  // reservations that did not fit
    // frames whose bytes are fully staged, counted in per-thread shards on
    // lines of their own (a single counter was a second contended line per
    // append); the flush thread sums them
    struct alignas(64) Shard
    {
        std::atomic<uint64_t> n{0};
    };
    Shard done[kDoneShards];
    uint64_t done_total() const
    {
        uint64_t t = 0;
        for (const Shard& d : done) t += d.n.load(std::memory_order_acquire);
        return t;
    }
    void done_reset()
    {
        for (Shard& d : done) d.n.store(0);
    }
    // Frames too large for the staging arena (more than half of it) take a
    // slot and a record number like any other (0 arena bytes reserved) but
    // are staged in a buffer of their own, listed here until the flush
    // writes them in record order between the arena's frames.
    struct External
    {
        uint64_t idx;
        unsigned char* frame;  // header, entry, room for the CRC; null: malloc failed
        uint64_t bytes;        // 0 when frame is null
        uint64_t charged;      // bytes charged to durable_log::m_ext_bytes
    };
    std::mutex ext_mu;
    std::vector<External> ext;
    bool pinned = false;  // arena from mi_host_malloc_pinned (else malloc)
};

// A checksummed segment handed from the flush thread to the writer: its
// arena (the segment itself has moved on to the spare arena) with the frames
// at [0, used), the external frames and the arena offsets they precede, and
// where they go in which file.  Frees what it still holds.
struct durable_log::write_job
{
    durable_log* log = nullptr;
    unsigned char* arena = nullptr;
    bool arena_pinned = false;
    uint64_t used = 0;
    std::vector<segment::External> ext;
    std::vector<uint64_t> ext_at;
    int fd = -1;
    uint64_t file_off = 0;
    uint64_t upto = 0;    // watermark once written and synced
    uint64_t frames = 0;
    size_t row = SIZE_MAX;  // flush_timeline row
    void release_ext()
    {
        for (segment::External& x : ext)
        {
            free(x.frame);
            log->release_external(x.charged);
        }
        ext.clear();
    }
    ~write_job() { release_ext(); }
};

static unsigned done_shard()
{
    static std::atomic<unsigned> next{0};
    thread_local const unsigned k = next.fetch_add(1) % kDoneShards;
    return k;
}

namespace {
consus::durable_log_options with_capacity(size_t cap)
{
    consus::durable_log_options o;
    o.segment_capacity = cap;
    return o;
}
}  // namespace

durable_log::durable_log() : durable_log(durable_log_options()) {}

durable_log::durable_log(size_t segment_capacity) : durable_log(with_capacity(segment_capacity)) {}

durable_log::durable_log(const durable_log_options& options)
    : m_path()
    , m_dir(-1)
    , m_lock_fd(-1)
    , m_mtx()
    , m_cond()
    , m_flush()
    , m_error(0)
    , m_wakeup(false)
    , m_opened(false)
    , m_capacity(options.segment_capacity ? options.segment_capacity : kDefaultCapacity)
    , m_opts(options)
    , m_segment_a(nullptr)
    , m_segment_b(nullptr)
    , m_active(nullptr)
    , m_switch_gen(0)
    , m_flush_phase(0)
    , m_slow_waiters(0)
    , m_append_hook(nullptr)
    , m_append_hook_ctx(nullptr)
    , m_durable(1)
    , m_flush_idle(false)
    , m_crc(gpu_batch)
    , m_crc_ctx(&m_opts)
    , m_host_max(host_batch_max(options))
    , m_host_flushes(0)
    , m_append_crc(nullptr)
    , m_ext_malloc_fail(false)
    , m_pinned(true)
    , m_flushes(0)
    , m_frames_flushed(0)
    , m_spare(nullptr)
    , m_spare_pinned(false)
    , m_stop_writer(false)
    , m_stop(false)
    , m_fsync_delay_us(0)
    , m_sink(false)
    , m_ext_bytes(0)
    , m_ext_peak(0)
{
    for (auto& t : m_flush_ns) t.store(0);
    for (auto& t : m_flush_max_ns) t.store(0);
    m_flush = std::thread(&durable_log::flush, this);
    m_writer = std::thread(&durable_log::writer, this);
    m_sync = std::thread(&durable_log::sync, this);
}

durable_log::~durable_log() throw()
{
    close();
    if (m_flush.joinable()) m_flush.join();
    {
        std::lock_guard<std::mutex> hold(m_mtx);
        m_stop_writer = true;  // the writer drains its job first
        m_cond.notify_all();
    }
    if (m_writer.joinable()) m_writer.join();
    {
        std::lock_guard<std::mutex> hold(m_mtx);
        m_stop = true;
        m_cond.notify_all();
    }
    if (m_sync.joinable()) m_sync.join();
    for (write_job* j : m_jobs)
    {
        if (j->arena) j->arena_pinned ? (void)mi_host_free_pinned(j->arena) : free(j->arena);
        delete j;
    }
    if (m_spare) m_spare_pinned ? (void)mi_host_free_pinned(m_spare) : free(m_spare);
    for (segment* s : {m_segment_a, m_segment_b})
    {
        if (!s) continue;
        if (s->fd >= 0) ::close(s->fd);
        delete[] s->at;
        if (s->arena)
        {
            if (s->pinned)
                mi_host_free_pinned(s->arena);
            else
                free(s->arena);
        }
        for (segment::External& x : s->ext) free(x.frame);
        delete s;
    }
    if (m_lock_fd >= 0) ::close(m_lock_fd);
    if (m_dir >= 0) ::close(m_dir);
}

void durable_log::set_batch_crc_for_testing(durable_log_batch_crc fn, void* ctx)
{
    std::lock_guard<std::mutex> hold(m_mtx);
    if (m_opened) return;
    m_crc = fn ? fn : gpu_batch;
    m_crc_ctx = fn ? ctx : &m_opts;
    m_pinned = !fn;
}

void durable_log::set_pinned_arenas_for_testing(bool pinned)
{
    std::lock_guard<std::mutex> hold(m_mtx);
    if (!m_opened) m_pinned = pinned;
}

// Rows of the flush timeline kept (a bench run flushes a few thousand times).
constexpr size_t kTimelineRows = 1 << 14;

double durable_log::since_open() const
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - m_t_open).count();
}

// Under m_mtx.
void durable_log::mark(size_t row, int col, double v)
{
    if (row < m_timeline.size() / 7) m_timeline[row * 7 + size_t(col)] = v;
}

size_t durable_log::flush_timeline(double* out, size_t max_rows)
{
    std::lock_guard<std::mutex> hold(m_mtx);
    const size_t n = std::min(max_rows, m_timeline.size() / 7);
    std::copy(m_timeline.begin(), m_timeline.begin() + ptrdiff_t(n * 7), out);
    return n;
}

void durable_log::set_append_crc_for_testing(uint32_t (*fn)(uint32_t, const unsigned char*, size_t))
{
    std::lock_guard<std::mutex> hold(m_mtx);
    if (m_opened) return;
    m_append_crc = fn;
}

void durable_log::set_external_malloc_failure_for_testing(bool fail) { m_ext_malloc_fail = fail; }

uint64_t durable_log::host_flushes() const { return m_host_flushes; }

uint64_t durable_log::flushes() const { return m_flushes; }
uint64_t durable_log::frames_flushed() const { return m_frames_flushed; }

void durable_log::flush_seconds(double out[6]) const
{
    for (int i = 0; i < 6; ++i) out[i] = double(m_flush_ns[i].load()) * 1e-9;
}

void durable_log::flush_max_seconds(double out[6]) const
{
    for (int i = 0; i < 6; ++i) out[i] = double(m_flush_max_ns[i].load()) * 1e-9;
}

void durable_log::note_phase(int phase, uint64_t ns)
{
    m_flush_ns[phase] += ns;
    uint64_t m = m_flush_max_ns[phase].load(std::memory_order_relaxed);
    while (ns > m && !m_flush_max_ns[phase].compare_exchange_weak(m, ns, std::memory_order_relaxed))
    {
    }
}

void durable_log::set_sink_for_testing(bool sink)
{
    std::lock_guard<std::mutex> hold(m_mtx);
    if (!m_opened) m_sink = sink;
}

void durable_log::set_fsync_delay_for_testing(uint32_t microseconds)
{
    m_fsync_delay_us.store(microseconds);
}

void durable_log::set_append_hook_for_testing(void (*fn)(void*, int), void* ctx)
{
    std::lock_guard<std::mutex> hold(m_mtx);
    if (m_opened) return;
    m_append_hook = fn;
    m_append_hook_ctx = ctx;
}

void durable_log::debug_state(char* buf, size_t n)
{
    if (!buf || !n) return;
    static const char* const phases[] = {"start",     "idle",        "sealing", "wait-copies",
                                         "prepare",   "wait-spare",  "stopped"};
    std::lock_guard<std::mutex> hold(m_mtx);
    const segment* act = m_active.load();
    const int ph = m_flush_phase.load();
    uint64_t w = 0, staged = 0, failed = 0, base = 0;
    if (act)
    {
        w = act->word.load();
        staged = act->done_total();
        failed = act->failed.load();
        base = act->base;
    }
    snprintf(buf, n,
             "flush=%s active=%s sealed=%d frames=%llu bytes=%llu staged=%llu failed=%llu "
             "base=%llu switches=%llu flush_idle=%d spare=%d jobs=%zu pending=%zu "
             "append_slow=%d error=%d durable=%llu",
             ph >= 0 && ph <= 6 ? phases[ph] : "?",
             !act ? "none" : act == m_segment_a ? "a" : "b", int((w & kSealed) != 0),
             (unsigned long long)((w & ~kSealed) >> kIdxShift),
             (unsigned long long)(w & kUsedMask), (unsigned long long)staged,
             (unsigned long long)failed, (unsigned long long)base,
             (unsigned long long)m_switch_gen.load(), int(m_flush_idle.load()),
             int(m_spare != nullptr), m_jobs.size(), m_pending.size(), m_slow_waiters.load(),
             m_error.load(), (unsigned long long)m_durable.load());
}

bool durable_log::open(const std::string& dir)
{
    std::lock_guard<std::mutex> hold(m_mtx);
    m_path = dir;
    struct stat st;
    int ret = stat(m_path.c_str(), &st);
    if (ret < 0 && errno == ENOENT)
    {
        if (mkdir(m_path.c_str(), S_IRWXU) < 0)
        {
            m_error = errno;
            return false;
        }
        ret = stat(m_path.c_str(), &st);
    }
    if (ret < 0)
    {
        m_error = errno;
        return false;
    }
    if (!S_ISDIR(st.st_mode))
    {
        m_error = errno = ENOTDIR;
        return false;
    }
    m_dir = ::open(m_path.c_str(), O_RDONLY);
    if (m_dir < 0)
    {
        m_error = errno;
        return false;
    }
    m_lock_fd = openat(m_dir, "LOCK", O_RDWR | O_CREAT, S_IRUSR | S_IWUSR);
    if (m_lock_fd < 0 || flock(m_lock_fd, LOCK_EX | LOCK_NB) < 0)
    {
        m_error = errno;
        return false;
    }
    // As the reference (:157-159): the segments are truncated, no rotation.
    const int file_a = openat(m_dir, "file_a", O_WRONLY | O_CREAT | O_TRUNC, S_IRUSR | S_IWUSR);
    const int file_b = openat(m_dir, "file_b", O_WRONLY | O_CREAT | O_TRUNC, S_IRUSR | S_IWUSR);
    if (file_a < 0 || file_b < 0)
    {
        if (file_a >= 0) ::close(file_a);
        if (file_b >= 0) ::close(file_b);
        return false;
    }
    segment* segs[2] = {new segment, new segment};
    const int fds[2] = {file_a, file_b};
    // the third arena: a checksummed segment's bytes go to the writer in
    // their arena while the segment continues in this one
    {
        void* p = nullptr;
        if (m_pinned && mi_host_malloc_pinned(&p, m_capacity) == MI_CRC32C_OK)
            m_spare_pinned = true;
        else
            p = malloc(m_capacity);
        m_spare = static_cast<unsigned char*>(p);
    }
    // at most one frame per 20 staged bytes, and headroom below the
    // reservation word's frame field (no carry into the sealed bit)
    const uint64_t frames = std::min<uint64_t>(m_capacity / (kHeader + kTrailer) + 1,
                                               kMaxFrames / 2);
    bool ok = true;
    for (int i = 0; i < 2; ++i)
    {
        segs[i]->fd = fds[i];
        segs[i]->cap = m_capacity;
        void* p = nullptr;
        // pinned staging lets the GPU batch DMA the segment in place; without
        // a usable device the log still works from ordinary memory (its CRCs
        // then come from the engine's CPU path)
        if (m_pinned && mi_host_malloc_pinned(&p, m_capacity) == MI_CRC32C_OK)
            segs[i]->pinned = true;
        else
            p = malloc(m_capacity);
        segs[i]->arena = static_cast<unsigned char*>(p);
        segs[i]->slots = (frames + 7) & ~uint64_t(7);
        segs[i]->at = new (std::nothrow) uint64_t[segs[i]->slots];
        ok = ok && p && segs[i]->at;
    }
    if (!ok || !m_spare)
    {
        if (m_spare) m_spare_pinned ? (void)mi_host_free_pinned(m_spare) : free(m_spare);
        m_spare = nullptr;
        m_error = ENOMEM;
        for (segment* s : segs)
        {
            if (s->arena) s->pinned ? (void)mi_host_free_pinned(s->arena) : free(s->arena);
            delete[] s->at;
            ::close(s->fd);
            delete s;
        }
        errno = ENOMEM;
        return false;
    }
    m_segment_a = segs[0];
    m_segment_b = segs[1];
    m_t_open = std::chrono::steady_clock::now();
    m_segment_a->base = 1;  // record numbers start at 1 (:151)
    m_segment_a->word.store(0);
    m_active.store(m_segment_a);
    m_opened = true;
    m_cond.notify_all();
    return true;
}

void durable_log::close()
{
    std::unique_lock<std::mutex> hold(m_mtx);
    if (m_error == 0 && m_active.load())
    {
        // Deviation (stronger than the reference, :172-177): every record
        // reserved before close() was called is made durable before the log
        // shuts down.  The bound is read once, so appenders that keep going
        // cannot hold close() up; their later records may or may not be
        // flushed, as with the reference, whose close() drops them all.
        const segment* act = m_active.load();
        const uint64_t ub = act->base + ((act->word.load() & ~kSealed) >> kIdxShift);
        m_cond.wait(hold, [&] { return m_error != 0 || m_durable.load() >= ub; });
    }
    if (m_error == 0) m_error = -1;
    m_cond.notify_all();
}

int64_t durable_log::append(const char* entry, size_t entry_sz)
{
    return append(reinterpret_cast<const unsigned char*>(entry), entry_sz);
}

int64_t durable_log::append(const unsigned char* entry, size_t entry_sz)
{
    if (entry_sz > UINT64_MAX - kHeader - kTrailer)
    {
        errno = EMSGSIZE;
        return -1;
    }
    const uint64_t frame = kHeader + entry_sz + kTrailer;
    // Frames of more than half the staging arena are staged outside it
    // (segment::External), so an entry of any size is accepted, as by the
    // reference (txman/durable_log.cc:187-242).  Their bytes are charged
    // before the frame takes a record number and released once the flush
    // has written it, so they wait for room like a full arena does.
    const bool external = frame > m_capacity / 2;
    const uint64_t arena_bytes = external ? 0 : frame;
    if (external && !charge_external(frame)) return -1;
    bool charged = external;  // released by the flush from here on, or below on failure
    struct Uncharge
    {
        durable_log* log;
        const bool& charged;
        uint64_t bytes;
        ~Uncharge()
        {
            if (charged) log->release_external(bytes);
        }
    } uncharge{this, charged, frame};
    while (true)
    {
        if (const int e = m_error.load())
        {
            errno = e;
            return -1;
        }
        // the generation first: switch_to_next stores m_active before it
        // bumps the generation, so seg is the segment of generation `gen` or
        // a later one, and a switch away from seg always moves it past gen
        const uint64_t gen = m_switch_gen.load(std::memory_order_acquire);
        segment* seg = m_active.load(std::memory_order_acquire);
        if (!seg)
        {
            errno = EBADF;
            return -1;
        }
        if (m_append_hook) m_append_hook(m_append_hook_ctx, 0);
        // record number and staging offset in one step (txman/durable_log.cc:
        // 195-213 takes m_mtx for the same reservation)
        const uint64_t w = seg->word.fetch_add((uint64_t(1) << kIdxShift) | arena_bytes);
        if (!(w & kSealed))
        {
            const uint64_t idx = w >> kIdxShift, at = w & kUsedMask;
            if (at + arena_bytes <= seg->cap && idx < seg->slots)
            {
                if (idx == 0 && m_flush_idle.load())
                {
                    std::lock_guard<std::mutex> hold(m_mtx);  // the flush thread sleeps for this frame
                    m_cond.notify_all();
                }
                // encode_header (txman/durable_log.cc:57-61) and the entry
                const uint64_t recno = seg->base + idx;
                unsigned char* p = !external ? seg->arena + at
                                   : m_ext_malloc_fail.load() ? nullptr
                                   : static_cast<unsigned char*>(malloc(frame));
                if (p)
                {
                    pack64be(recno, p);
                    pack64be(entry_sz, p + 8);
                    if (entry_sz) memcpy(p + kHeader, entry, entry_sz);
                    // the reference scheme (bench hook): this thread's CRC
                    if (m_append_crc)
                        pack32be(m_append_crc(0, p, kHeader + entry_sz), p + kHeader + entry_sz);
                }
                if (external)
                {
                    // written in record order, just before the arena bytes
                    // reserved after it (its slot holds that arena offset);
                    // the flush releases its charge (a failed malloc's too)
                    std::lock_guard<std::mutex> hold(seg->ext_mu);
                    seg->ext.push_back(segment::External{idx, p, p ? frame : 0, frame});
                    seg->at_slot(idx) = at | kExternal;
                    charged = false;
                }
                else
                    seg->at_slot(idx) = at;
                seg->done[done_shard()].n.fetch_add(1, std::memory_order_release);
                if (!p)
                {
                    // out of memory for a record that already holds a record
                    // number: fatal for the log, as an I/O error is in the
                    // reference (txman/durable_log.cc:226-230)
                    std::lock_guard<std::mutex> hold(m_mtx);
                    if (m_error == 0) m_error = ENOMEM;
                    m_cond.notify_all();
                    errno = ENOMEM;
                    return -1;
                }
                return int64_t(recno);
            }
            // Full.  `used` only grows, so every reservation from this one on
            // fails too: the valid frames are the prefix before the first
            // failure, which the flush thread reads from `cut` once every
            // reservation it sealed is accounted for (staged or failed).
            uint64_t c = seg->cut.load();
            while (idx < (c >> kIdxShift) &&
                   !seg->cut.compare_exchange_weak(c, (idx << kIdxShift) | at))
            {
            }
            seg->failed.fetch_add(1, std::memory_order_release);
        }
        // sealed (the flush thread is switching segments) or full
        if (m_append_hook) m_append_hook(m_append_hook_ctx, 1);
        const int64_t r = append_slow(seg, gen);
        if (r < 0) return r;
    }
}

// The active segment is full or being sealed: wake the flush thread and wait
// until it has switched appends to the other segment (backpressure when both
// staging buffers are in use, as the reference's writers wait on its flush).
// A segment sealed or filled at generation `gen` is always followed by a
// switch (the flush thread seals only the active segment, and switches away
// from it once its reservations are accounted for), so waiting for the
// generation to move cannot block forever.  Waiting for m_active != seg could:
// two switches (seg -> other -> seg) between this appender's failed
// reservation and its wait bring seg back, empty, and with no other appender
// the flush thread then sleeps on it for good.  txman/durable_log.cc:195-213
// never waits for a switch (its segment files are unbounded); here the
// staging arenas are bounded, so a full one is backpressure.
int64_t durable_log::append_slow(segment* seg, uint64_t gen)
{
    std::unique_lock<std::mutex> hold(m_mtx);
    // wake the flush thread only if seg is still the one to switch away from
    if (m_switch_gen.load() == gen && m_active.load() == seg) m_cond.notify_all();
    ++m_slow_waiters;
    m_cond.wait(hold, [&] { return m_error != 0 || m_switch_gen.load() != gen; });
    --m_slow_waiters;
    if (m_error != 0)
    {
        errno = m_error;
        return -1;
    }
    return 0;
}

int64_t durable_log::durable()
{
    return int64_t(m_durable.load());
}

int64_t durable_log::wait(int64_t prev_ub)
{
    std::unique_lock<std::mutex> hold(m_mtx);
    while (true)
    {
        const int64_t x = int64_t(m_durable.load());
        if (m_error == 0 && x <= prev_ub && !m_wakeup)
            m_cond.wait(hold);
        else
        {
            m_wakeup = false;
            return x;
        }
    }
}

void durable_log::wake()
{
    std::lock_guard<std::mutex> hold(m_mtx);
    m_wakeup = true;
    m_cond.notify_all();
}

int durable_log::error()
{
    std::lock_guard<std::mutex> hold(m_mtx);
    return m_error;
}

// External frames (more than half an arena) are bounded together, as staged
// arena bytes are: by both arenas' capacity, but at least 16 MiB (a small
// arena would otherwise admit one such frame per flush).  An append over the
// bound waits for the flush to write earlier ones.  A single frame larger
// than the bound is admitted when none is staged, so an entry of any size is
// still accepted.
constexpr uint64_t kExternalMinBudget = uint64_t(16) << 20;

bool durable_log::charge_external(uint64_t bytes)
{
    const uint64_t budget = std::max<uint64_t>(2 * uint64_t(m_capacity), kExternalMinBudget);
    uint64_t cur = m_ext_bytes.load();
    while (true)
    {
        if (cur == 0 || cur + bytes <= budget)
        {
            if (!m_ext_bytes.compare_exchange_weak(cur, cur + bytes)) continue;
            uint64_t peak = m_ext_peak.load();
            while (cur + bytes > peak && !m_ext_peak.compare_exchange_weak(peak, cur + bytes))
            {
            }
            return true;
        }
        std::unique_lock<std::mutex> hold(m_mtx);
        m_cond.notify_all();  // the flush thread: a staged frame is waiting
        m_cond.wait(hold, [&] {
            cur = m_ext_bytes.load();
            return m_error != 0 || cur == 0 || cur + bytes <= budget;
        });
        if (m_error != 0)
        {
            errno = m_error;
            return false;
        }
    }
}

uint64_t durable_log::external_bytes_peak() const { return m_ext_peak.load(); }

void durable_log::release_external(uint64_t bytes)
{
    m_ext_bytes.fetch_sub(bytes);
    std::lock_guard<std::mutex> hold(m_mtx);
    m_cond.notify_all();
}

// The batch CRC of n staged frames through the configured engine.  The
// default engine completes engine failures on the CPU path itself; if an
// injected test engine fails, the engine's CPU path completes the batch here
// (counted in mi_crc32c_stats), so a failed checksum never fails the log.
int durable_log::batch_crc(const unsigned char* base, const uint64_t* offs, const uint32_t* lens,
                           size_t n, uint64_t total, uint32_t* out)
{
    // below the GPU/CPU crossover: the flush thread's CPU (counted)
    if (m_crc == gpu_batch && total < m_host_max &&
        mi_crc32c_batch(base, offs, lens, nullptr, n, total, out, MI_CRC32C_CPU) == MI_CRC32C_OK)
    {
        m_host_flushes.fetch_add(1, std::memory_order_relaxed);
        return 0;
    }
    if (m_crc(m_crc_ctx, base, offs, lens, n, total, out) == 0) return 0;
    mi_host::batch(base, offs, lens, nullptr, n, out);
    mi_host::note_fallback(MI_CRC32C_EHIP, total);
    return 0;
}

// CRC of one frame's header + entry (`length` bytes) staged on its own.
uint32_t durable_log::frame_crc(const unsigned char* frame, uint64_t length)
{
    if (m_crc != gpu_batch && length <= kBatchFrameMax)
    {
        const uint64_t off = 0;
        const uint32_t len = uint32_t(length);
        uint32_t c = 0;
        batch_crc(frame, &off, &len, 1, length, &c);
        return c;
    }
    return single_crc(frame, length);
}

// Checksum the segment's n frames -- the arena's in one batch, external ones
// one by one -- and patch the CRCs in; fill `job` with what the writer needs
// to write them in record order at the end of the file.  Arena frames sit
// back to back from offset 0; their offsets come from the slots.
int durable_log::prepare_segment(segment* seg, uint64_t& n, uint64_t& used, write_job* job)
{
    auto t = std::chrono::steady_clock::now();
    auto lap = [&](int phase) {
        const auto u = std::chrono::steady_clock::now();
        note_phase(phase, uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(u - t).count()));
        t = u;
    };
    job->log = this;
    {
        std::lock_guard<std::mutex> hold(seg->ext_mu);
        job->ext.swap(seg->ext);
    }
    std::vector<segment::External>& ext = job->ext;
    std::sort(ext.begin(), ext.end(),
              [](const segment::External& x, const segment::External& y) { return x.idx < y.idx; });
    // frames past the cut were never handed out (their appenders retried)
    while (!ext.empty() && ext.back().idx >= n)
    {
        free(ext.back().frame);
        release_external(ext.back().charged);
        ext.pop_back();
    }
    // A frame whose staging malloc failed put the log into ENOMEM: nothing
    // from it on reaches the file (no record-number gap on disk), so the
    // segment ends at its slot.
    for (size_t j = 0; j < ext.size(); ++j)
        if (!ext[j].frame)
        {
            n = ext[j].idx;
            used = seg->at_slot(ext[j].idx) & ~kExternal;
            for (size_t k = j; k < ext.size(); ++k)
            {
                free(ext[k].frame);
                release_external(ext[k].charged);
            }
            ext.resize(j);
            break;
        }
    job->ext_at.resize(ext.size());
    for (size_t j = 0; j < ext.size(); ++j) job->ext_at[j] = seg->at_slot(ext[j].idx) & ~kExternal;
    if (n)
    {
        m_offs.resize(n);
        m_lens.resize(n);
        m_crcs.resize(n);
        uint64_t k = 0, total = 0;
        for (uint64_t i = 0; i < n; ++i)
        {
            const uint64_t a = seg->at_slot(i);
            if (!(a & kExternal)) m_offs[k++] = a;
        }
        for (uint64_t i = 0; i < k; ++i)
        {
            const uint64_t end = i + 1 < k ? m_offs[i + 1] : used;
            if (end < m_offs[i] + kHeader + kTrailer) return EIO;  // offsets must tile the bytes
            m_lens[i] = uint32_t(end - m_offs[i] - kTrailer);
            total += m_lens[i];
        }
        lap(1);
        // (with the append-CRC bench hook every frame already holds its CRC)
        if (k && !m_append_crc)
            batch_crc(seg->arena, m_offs.data(), m_lens.data(), size_t(k), total, m_crcs.data());
        if (!m_append_crc)
            for (segment::External& x : ext)
                pack32be(frame_crc(x.frame, x.bytes - kTrailer), x.frame + x.bytes - kTrailer);
        lap(2);
        // crc32c(crc32c(0, header, 16), entry) == crc32c(0, header || entry),
        // stored big-endian after the entry (txman/durable_log.cc:215-224)
        if (!m_append_crc)
            for (uint64_t i = 0; i < k; ++i) pack32be(m_crcs[i], seg->arena + m_offs[i] + m_lens[i]);
        lap(3);
    }
    uint64_t bytes = used;
    for (const segment::External& x : ext) bytes += x.bytes;
    job->used = used;
    job->fd = seg->fd;
    job->file_off = seg->file_size;
    job->upto = seg->base + n;
    job->frames = n;
    seg->file_size += bytes;
    return 0;
}

// The writer's half: the job's frames in record order at its file offset.
int durable_log::write_out(write_job* job)
{
    const auto t = std::chrono::steady_clock::now();
    if (m_sink)  // bench hook: storage faster than anything else here
    {
        job->release_ext();
        return 0;
    }
    uint64_t at = 0, file = job->file_off;
    for (size_t j = 0; j < job->ext.size(); ++j)
    {
        const segment::External& x = job->ext[j];
        const uint64_t upto = job->ext_at[j];
        if (upto > at && !pwrite_all(job->fd, job->arena + at, upto - at, off_t(file))) return errno;
        file += upto - at;
        at = upto;
        if (x.bytes && !pwrite_all(job->fd, x.frame, x.bytes, off_t(file))) return errno;
        file += x.bytes;
    }
    if (job->used > at &&
        !pwrite_all(job->fd, job->arena + at, job->used - at, off_t(file)))
        return errno;
    job->release_ext();
    note_phase(4, uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                  std::chrono::steady_clock::now() - t)
                                  .count()));
    return 0;
}

// The writer thread: write each checksummed segment, give its arena back as
// the spare, and hand the fsync to the sync thread (at most one written
// segment waits for it, so appends stay throttled by the disk).  It runs
// beside the flush thread, which meanwhile checksums the next segment.
void durable_log::writer()
{
    sigset_t ss;
    if (sigfillset(&ss) == 0) pthread_sigmask(SIG_BLOCK, &ss, nullptr);
    std::unique_lock<std::mutex> hold(m_mtx);
    while (true)
    {
        m_cond.wait(hold, [&] { return m_stop_writer || !m_jobs.empty(); });
        if (m_jobs.empty()) return;  // m_stop_writer, nothing left to write
        write_job* job = m_jobs.front();
        m_jobs.erase(m_jobs.begin());
        mark(job->row, 3, since_open());
        hold.unlock();
        const int e = m_error.load() > 0 ? 0 : write_out(job);
        hold.lock();
        mark(job->row, 4, since_open());
        m_spare = job->arena;  // free again: the next sealed segment may take it
        m_spare_pinned = job->arena_pinned;
        job->arena = nullptr;
        if (e && (m_error == 0 || m_error == -1)) m_error = e;
        m_cond.notify_all();
        if (m_error == 0 || m_error == -1)
        {
            m_cond.wait(hold, [&] { return (m_error != 0 && m_error != -1) || m_pending.empty(); });
            if (m_error == 0 || m_error == -1)
            {
                m_pending.push_back(synced{job->fd, job->upto, job->frames, job->row});
                m_cond.notify_all();
            }
        }
        hold.unlock();
        delete job;  // frees external frames a failed write left behind
        hold.lock();
    }
}

// The sync thread: fsync each written segment in turn and publish its
// watermark (in write order, so the watermark only grows).  It runs beside
// the flush thread, which meanwhile checksums and writes the next segment.
void durable_log::sync()
{
    sigset_t ss;
    if (sigfillset(&ss) == 0) pthread_sigmask(SIG_BLOCK, &ss, nullptr);
    std::unique_lock<std::mutex> hold(m_mtx);
    while (true)
    {
        m_cond.wait(hold, [&] { return m_stop || !m_pending.empty(); });
        if (m_pending.empty()) return;  // m_stop
        const synced job = m_pending.front();
        hold.unlock();
        const auto t = std::chrono::steady_clock::now();
        int e = m_sink ? 0 : fsync(job.fd) < 0 ? errno : 0;
        if (const uint32_t us = m_fsync_delay_us.load()) usleep(us);
        note_phase(5, uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                      std::chrono::steady_clock::now() - t)
                                      .count()));
        hold.lock();
        m_pending.erase(m_pending.begin());
        if (e)
        {
            if (m_error == 0) m_error = e;
        }
        else if (m_error == 0 || m_error == -1)
        {
            m_durable.store(job.upto);
            mark(job.row, 5, since_open());
            ++m_flushes;
            m_frames_flushed += job.frames;
        }
        m_cond.notify_all();
    }
}

// Appends move to the other segment (its previous flush is complete: there
// is one flush thread); its record numbers continue after seg's n frames.
// Called with m_mtx held.
void durable_log::switch_to_next(segment* seg, uint64_t n)
{
    segment* next = seg == m_segment_a ? m_segment_b : m_segment_a;
    next->base = seg->base + n;
    next->done_reset();
    next->failed.store(0);
    next->cut.store(~uint64_t(0));
    next->word.store(0);  // unsealed, empty: appends may reserve in it
    m_active.store(next);
    m_switch_gen.fetch_add(1);  // after m_active: see append()
    m_cond.notify_all();  // appenders waiting for room
}

// The flush thread's first GPU batch creates its engine context (stream,
// pinned staging, completion counter; ~10-15 ms once).  Done once the log is
// open, before the first frame can wait for it: inside the first flush it
// was the p99 of the durability latency (7-14 ms against < 1 ms with the CPU
// checksum, round 3).  One 64-B record of the spare arena (pinned, unused
// until the first flush returns it to the writer) per device the flush may
// use, result ignored; no fallback flag, so a host without a device counts
// nothing.
void durable_log::warm_up()
{
    const unsigned char* arena = nullptr;
    {
        std::unique_lock<std::mutex> hold(m_mtx);
        m_cond.wait(hold, [&] { return m_opened || m_error != 0; });
        if (m_error != 0 || m_crc != gpu_batch || !m_spare || !m_spare_pinned) return;
        arena = m_spare;
    }
    const uint64_t off = 0;
    const uint32_t len = 64;
    uint32_t out = 0;
    if (m_opts.gpus == 1)
    {
        (void)mi_crc32c_batch(arena, &off, &len, nullptr, 1, len, &out, 0);
        return;
    }
    // A sharded flush runs its extra ranges on the engine's worker threads,
    // each with its own per-thread, per-device context: warm all of them
    // through the same entry point and device list (one 64-B record per
    // device, forced to split with a 1-byte shard minimum).
    const int nd = std::max(mi_crc32c_device_count(), 1);
    std::vector<uint64_t> offs(size_t(nd), 0);
    std::vector<uint32_t> lens(size_t(nd), len);
    std::vector<uint32_t> outs(size_t(nd), 0);
    (void)mi_crc32c_batch_multi(arena, offs.data(), lens.data(), nullptr, size_t(nd),
                                uint64_t(len) * uint64_t(nd), outs.data(), 0, nullptr,
                                m_opts.gpus, 1);
}

// The flush thread (txman/durable_log.cc:287-347): wait for a first staged
// frame, seal the active segment and switch appends to the other one (whose
// previous flush is complete: there is one flush thread), wait for the
// sealed segment's in-flight copies, then checksum, write and fsync it and
// publish the watermark.
void durable_log::flush()
{
    sigset_t ss;
    if (sigfillset(&ss) < 0 || pthread_sigmask(SIG_BLOCK, &ss, nullptr) != 0)
    {
        std::lock_guard<std::mutex> hold(m_mtx);
        m_error = errno;
        m_cond.notify_all();
        return;
    }
    warm_up();
    while (true)
    {
        segment* seg = nullptr;
        uint64_t n = 0, used = 0;
        bool exact = true;
        size_t row = SIZE_MAX;  // flush_timeline row of this flush
        {
            std::unique_lock<std::mutex> hold(m_mtx);
            m_flush_phase.store(1);
            while (true)
            {
                if (m_error != 0)
                {
                    m_flush_phase.store(6);
                    return;
                }
                seg = m_active.load();
                if (seg)
                {
                    // sleep only while the active segment is empty; an append
                    // that takes frame 0 wakes us (seq_cst: it sees the flag or
                    // we see its frame)
                    m_flush_idle.store(true);
                    if (((seg->word.load() & ~kSealed) >> kIdxShift) != 0) break;
                }
                m_cond.wait(hold);
            }
            m_flush_idle.store(false);
            m_flush_phase.store(2);
            // seal.  Unless the segment filled up, every reservation taken
            // so far is valid, so appends move to the other segment at once,
            // before the copies into this one finish.
            const uint64_t w = seg->word.fetch_or(kSealed);
            n = w >> kIdxShift;
            used = w & kUsedMask;
            exact = used <= seg->cap && n <= seg->slots;
            if (exact) switch_to_next(seg, n);
            if (m_timeline.size() / 7 < kTimelineRows)
            {
                row = m_timeline.size() / 7;
                m_timeline.resize(m_timeline.size() + 7, 0.0);
                mark(row, 0, since_open());
            }
        }
        // every reservation taken before the seal finishes: its frame is
        // staged, or it did not fit (and its appender retries elsewhere)
        m_flush_phase.store(3);
        const auto t_wait = std::chrono::steady_clock::now();
        for (int spins = 0; seg->done_total() + seg->failed.load(std::memory_order_acquire) != n;
             ++spins)
        {
            if (spins < 1024)
                std::this_thread::yield();
            else
                usleep(20);
        }
        note_phase(0, uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                      std::chrono::steady_clock::now() - t_wait)
                                      .count()));
        if (!exact)
        {
            // the segment filled up: the valid frames end at the first
            // reservation that did not fit
            const uint64_t cut = seg->cut.load();
            if ((cut >> kIdxShift) < n)
            {
                n = cut >> kIdxShift;
                used = cut & kUsedMask;
            }
            std::lock_guard<std::mutex> hold(m_mtx);
            switch_to_next(seg, n);
        }
        m_flush_phase.store(4);
        auto* job = new write_job;
        const int e = prepare_segment(seg, n, used, job);
        const double t_prepared = since_open();
        {
            std::unique_lock<std::mutex> hold(m_mtx);
            job->row = row;
            mark(row, 1, t_prepared);
            {
                uint64_t bytes = job->used;
                for (const segment::External& x : job->ext) bytes += x.bytes;
                mark(row, 6, double(bytes));
            }
            if (e)
            {
                m_error = e;
                m_flush_phase.store(6);
                m_cond.notify_all();
                hold.unlock();
                delete job;
                return;
            }
            m_flush_phase.store(5);
            // hand the bytes to the writer in their arena; the segment takes
            // the spare one (back from the writer's previous job) before it
            // can be active again
            m_cond.wait(hold, [&] { return m_error != 0 || m_spare != nullptr; });
            if (m_error != 0)
            {
                m_flush_phase.store(6);
                hold.unlock();
                delete job;
                return;
            }
            job->arena = seg->arena;
            job->arena_pinned = seg->pinned;
            seg->arena = m_spare;
            seg->pinned = m_spare_pinned;
            m_spare = nullptr;
            m_jobs.push_back(job);
            mark(row, 2, since_open());
            m_cond.notify_all();
        }
    }
}

// The reference declares replay (txman/durable_log.h:64) but never defines it
// (TODO:2-3).  Here: scan both segment files, verify every frame's CRC on the
// GPU (one batch per file), and hand the valid entries to f in record-number
// order.  Returns the number of records replayed, or -1 with errno set.
int64_t durable_log::replay(void (*f)(void*, const unsigned char*, size_t), void* p)
{
    durable_log_batch_crc fn;
    void* ctx;
    int dirfd;
    {
        std::lock_guard<std::mutex> hold(m_mtx);
        fn = m_crc;
        ctx = m_crc_ctx;
        dirfd = m_dir;
    }
    if (dirfd < 0)
    {
        errno = EBADF;
        return -1;
    }
    std::vector<unsigned char> bufs[2];
    std::vector<Frame> frames[2];
    const char* names[2] = {"file_a", "file_b"};
    for (int i = 0; i < 2; ++i)
    {
        if (!read_file(dirfd, names[i], &bufs[i])) return -1;
        Chained ch{fn, ctx};
        if (scan_frames(bufs[i].data(), bufs[i].size(), batch_or_host, &ch, single_crc,
                        &frames[i], nullptr) < 0)
        {
            errno = EIO;
            return -1;
        }
    }
    size_t ia = 0, ib = 0;
    int64_t n = 0;
    while (ia < frames[0].size() || ib < frames[1].size())
    {
        const bool take_a = ib >= frames[1].size() ||
                            (ia < frames[0].size() && frames[0][ia].recno < frames[1][ib].recno);
        const int s = take_a ? 0 : 1;
        const Frame& fr = take_a ? frames[0][ia++] : frames[1][ib++];
        if (f) f(p, bufs[s].data() + fr.offset + kHeader, fr.length);
        ++n;
    }
    return n;
}

// ---- C ABI ------------------------------------------------------------------
struct mi_dlog
{
    explicit mi_dlog(const consus::durable_log_options& o) : log(o) {}
    durable_log log;
};

extern "C" {

mi_dlog* mi_dlog_create(size_t segment_capacity)
{
    return new mi_dlog(with_capacity(segment_capacity));
}
mi_dlog* mi_dlog_create_ex(size_t segment_capacity, int gpus, uint64_t shard_min_bytes)
{
    consus::durable_log_options o;
    o.segment_capacity = segment_capacity;
    o.gpus = gpus;
    o.shard_min_bytes = shard_min_bytes;
    return new mi_dlog(o);
}
void mi_dlog_destroy(mi_dlog* l) { delete l; }
int mi_dlog_open(mi_dlog* l, const char* dir)
{
    if (!l || !dir)
    {
        errno = EINVAL;
        return 0;
    }
    return l->log.open(dir) ? 1 : 0;
}
void mi_dlog_close(mi_dlog* l) { l->log.close(); }
int64_t mi_dlog_append(mi_dlog* l, const void* entry, size_t sz)
{
    if (!l || (!entry && sz))
    {
        errno = EINVAL;
        return -1;
    }
    return l->log.append(static_cast<const unsigned char*>(entry), sz);
}
int64_t mi_dlog_durable(mi_dlog* l) { return l->log.durable(); }
int64_t mi_dlog_wait(mi_dlog* l, int64_t prev_ub) { return l->log.wait(prev_ub); }
void mi_dlog_wake(mi_dlog* l) { l->log.wake(); }
int mi_dlog_error(mi_dlog* l) { return l->log.error(); }
int64_t mi_dlog_replay(mi_dlog* l, void (*f)(void*, const unsigned char*, size_t), void* p)
{
    return l->log.replay(f, p);
}
uint64_t mi_dlog_flushes(mi_dlog* l) { return l->log.flushes(); }
uint64_t mi_dlog_host_flushes(mi_dlog* l) { return l->log.host_flushes(); }
mi_dlog* mi_dlog_create_opts(size_t segment_capacity, int gpus, uint64_t shard_min_bytes,
                             int64_t host_batch_max)
{
    consus::durable_log_options o;
    o.segment_capacity = segment_capacity;
    o.gpus = gpus;
    o.shard_min_bytes = shard_min_bytes;
    o.host_batch_max = host_batch_max;
    return new mi_dlog(o);
}
void mi_dlog_set_append_crc_for_testing(mi_dlog* l,
                                        uint32_t (*fn)(uint32_t, const unsigned char*, size_t))
{
    l->log.set_append_crc_for_testing(fn);
}
void mi_dlog_set_external_malloc_failure_for_testing(mi_dlog* l, int fail)
{
    l->log.set_external_malloc_failure_for_testing(fail != 0);
}
uint64_t mi_dlog_frames_flushed(mi_dlog* l) { return l->log.frames_flushed(); }
uint64_t mi_dlog_external_peak(mi_dlog* l) { return l->log.external_bytes_peak(); }
void mi_dlog_flush_seconds(mi_dlog* l, double out[6]) { l->log.flush_seconds(out); }
void mi_dlog_flush_max_seconds(mi_dlog* l, double out[6]) { l->log.flush_max_seconds(out); }
void mi_dlog_set_batch_crc_for_testing(mi_dlog* l, mi_dlog_batch_crc fn, void* ctx)
{
    l->log.set_batch_crc_for_testing(fn, ctx);
}
void mi_dlog_set_fsync_delay_for_testing(mi_dlog* l, uint32_t microseconds)
{
    l->log.set_fsync_delay_for_testing(microseconds);
}
void mi_dlog_set_append_hook_for_testing(mi_dlog* l, void (*fn)(void*, int), void* ctx)
{
    l->log.set_append_hook_for_testing(fn, ctx);
}
void mi_dlog_debug_state(mi_dlog* l, char* buf, size_t n) { l->log.debug_state(buf, n); }

int64_t mi_dlog_scan_file(const char* path, uint64_t* valid_bytes, uint64_t* recnos,
                          uint64_t* offsets, size_t max_frames)
{
    std::vector<unsigned char> buf;
    if (!read_file(-1, path, &buf)) return -1;
    std::vector<Frame> frames;
    const int64_t n =
        scan_frames(buf.data(), buf.size(), gpu_batch, nullptr, single_crc, &frames, valid_bytes);
    if (n < 0) return -1;
    for (size_t i = 0; i < frames.size() && i < max_frames; ++i)
    {
        if (recnos) recnos[i] = frames[i].recno;
        if (offsets) offsets[i] = frames[i].offset;
    }
    return n;
}

}  // extern "C"
