// consus_amd/csrc/durable_log.cc -- the record-batching durable log.
//
// Re-implements txman/durable_log.cc (rescrv/Consus) around the MI355X CRC
// engine; see include/txman/durable_log.h for the contract.  Control flow
// follows the reference: segment choice (select_segment_write / _fsync,
// :349-419), record-number reservation under the mutex (:195-213), a flush
// thread with all signals blocked (:287-347) and the watermark
// (durable_lock_held_elsewhere, :421-440).  The data path differs: frames are
// staged in pinned memory and checksummed per flushed segment in one GPU
// batch, then written with one pwrite and fsynced.
#include "../../include/txman/durable_log.h"

#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>

#include "../../include/consus_crc32c.h"
#include "../../include/consus_durable_log.h"

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

int gpu_batch(void*, const void* base, const uint64_t* off, const uint32_t* len, size_t n,
              uint64_t total, uint32_t* out)
{
    return mi_crc32c_batch(base, off, len, nullptr, n, total, out, 0);
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
    uint32_t length;  // of the entry
};

// Parse frames by their length chain and verify every CRC in one batch.
// Returns the number of leading complete, CRC-valid frames, or -1 if the
// engine failed.  A torn tail or the first bad CRC ends the scan.
int64_t scan_frames(const unsigned char* buf, uint64_t size, consus::durable_log_batch_crc fn,
                    void* ctx, std::vector<Frame>* frames, uint64_t* valid_bytes)
{
    std::vector<uint64_t> offs;
    std::vector<uint32_t> lens, stored;
    std::vector<uint64_t> recnos;
    uint64_t pos = 0, total = 0;
    while (size - pos >= kHeader + kTrailer)
    {
        const uint64_t recno = unpack64be(buf + pos);
        const uint64_t len = unpack64be(buf + pos + 8);
        if (len > size - pos - kHeader - kTrailer || len > UINT32_MAX - kHeader) break;  // torn
        offs.push_back(pos);
        lens.push_back(uint32_t(kHeader + len));
        stored.push_back(unpack32be(buf + pos + kHeader + len));
        recnos.push_back(recno);
        total += kHeader + len;
        pos += kHeader + len + kTrailer;
    }
    std::vector<uint32_t> crcs(offs.size());
    if (!offs.empty() && fn(ctx, buf, offs.data(), lens.data(), offs.size(), total, crcs.data()) != 0)
        return -1;
    size_t good = 0;
    uint64_t bytes = 0;
    while (good < offs.size() && crcs[good] == stored[good])
    {
        if (frames) frames->push_back(Frame{recnos[good], offs[good], lens[good] - uint32_t(kHeader)});
        bytes += lens[good] + kTrailer;
        ++good;
    }
    if (valid_bytes) *valid_bytes = bytes;
    return int64_t(good);
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

struct durable_log::segment
{
    int fd = -1;
    unsigned char* arena = nullptr;  // staged frames since the last flush
    size_t cap = 0;
    uint64_t used = 0;
    uint64_t offset_next_write = 0;
    uint64_t offset_last_fsync = 0;
    uint64_t recno_last_write = 0;
    uint64_t recno_last_fsync = 0;
    int32_t ongoing_writes = 0;
    std::condition_variable done_writing;
    bool syncing = false;
    std::vector<uint64_t> frame_off;  // arena offset of each staged frame
    std::vector<uint32_t> frame_len;  // header + entry bytes covered by its CRC
};

durable_log::durable_log() : durable_log(kDefaultCapacity) {}

durable_log::durable_log(size_t segment_capacity)
    : m_path()
    , m_dir(-1)
    , m_lock_fd(-1)
    , m_mtx()
    , m_cond()
    , m_flush()
    , m_error(0)
    , m_wakeup(false)
    , m_opened(false)
    , m_next_entry(1)
    , m_capacity(segment_capacity ? segment_capacity : kDefaultCapacity)
    , m_segment_a(nullptr)
    , m_segment_b(nullptr)
    , m_crc(gpu_batch)
    , m_crc_ctx(nullptr)
    , m_pinned(true)
    , m_flushes(0)
    , m_frames_flushed(0)
{
    m_flush = std::thread(&durable_log::flush, this);
}

durable_log::~durable_log() throw()
{
    close();
    if (m_flush.joinable()) m_flush.join();
    for (segment* s : {m_segment_a, m_segment_b})
    {
        if (!s) continue;
        if (s->fd >= 0) ::close(s->fd);
        if (s->arena)
        {
            if (m_pinned)
                mi_host_free_pinned(s->arena);
            else
                free(s->arena);
        }
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
    m_crc_ctx = ctx;
    m_pinned = !fn;
}

uint64_t durable_log::flushes() const { return m_flushes; }
uint64_t durable_log::frames_flushed() const { return m_frames_flushed; }

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
    for (int i = 0; i < 2; ++i)
    {
        segs[i]->fd = fds[i];
        segs[i]->cap = m_capacity;
        void* p = nullptr;
        if (m_pinned)
        {
            if (mi_host_malloc_pinned(&p, m_capacity) != MI_CRC32C_OK) p = nullptr;
        }
        else
            p = malloc(m_capacity);
        if (!p)
        {
            m_error = ENOMEM;
            for (segment* s : segs)
            {
                if (s->arena) m_pinned ? (void)mi_host_free_pinned(s->arena) : free(s->arena);
                ::close(s->fd);
                delete s;
            }
            errno = ENOMEM;
            return false;
        }
        segs[i]->arena = static_cast<unsigned char*>(p);
    }
    m_segment_a = segs[0];
    m_segment_b = segs[1];
    m_opened = true;
    m_cond.notify_all();
    return true;
}

void durable_log::close()
{
    std::unique_lock<std::mutex> hold(m_mtx);
    if (m_error == 0 && m_segment_a && m_segment_b)
    {
        // Deviation (stronger than the reference): staged frames are flushed
        // before the log shuts down, so close() never drops appended records.
        m_cond.wait(hold, [&] {
            return m_error != 0 || (m_segment_a->offset_next_write == m_segment_a->offset_last_fsync &&
                                    m_segment_b->offset_next_write == m_segment_b->offset_last_fsync &&
                                    m_segment_a->ongoing_writes == 0 &&
                                    m_segment_b->ongoing_writes == 0);
        });
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
    const uint64_t frame = kHeader + entry_sz + kTrailer;
    segment* seg = nullptr;
    uint64_t at = 0;
    uint64_t recno = 0;
    {
        std::unique_lock<std::mutex> hold(m_mtx);
        if (!m_error && (!m_segment_a || frame > m_capacity || entry_sz > UINT32_MAX - kHeader))
        {
            errno = m_segment_a ? EMSGSIZE : EBADF;
            return -1;
        }
        while (true)
        {
            if (m_error)
            {
                errno = m_error;
                return -1;
            }
            seg = select_segment_write();
            if (seg && seg->used + frame > seg->cap)
            {
                segment* other = seg == m_segment_a ? m_segment_b : m_segment_a;
                seg = (!other->syncing && other->used + frame <= other->cap) ? other : nullptr;
            }
            if (seg) break;
            m_cond.notify_all();  // both staging buffers full: wait for a flush
            m_cond.wait(hold);
        }
        recno = m_next_entry++;
        at = seg->used;
        seg->used += frame;
        seg->offset_next_write += frame;
        seg->recno_last_write = recno;
        seg->frame_off.push_back(at);
        seg->frame_len.push_back(uint32_t(kHeader + entry_sz));
        ++seg->ongoing_writes;
    }
    // encode_header (txman/durable_log.cc:57-61) and the entry, outside the lock
    unsigned char* p = seg->arena + at;
    pack64be(recno, p);
    pack64be(entry_sz, p + 8);
    if (entry_sz) memcpy(p + kHeader, entry, entry_sz);
    {
        std::lock_guard<std::mutex> hold(m_mtx);
        if (--seg->ongoing_writes == 0)
        {
            seg->done_writing.notify_all();
            m_cond.notify_all();
        }
    }
    return int64_t(recno);
}

int64_t durable_log::durable()
{
    std::lock_guard<std::mutex> hold(m_mtx);
    return durable_lock_held_elsewhere();
}

int64_t durable_log::wait(int64_t prev_ub)
{
    std::unique_lock<std::mutex> hold(m_mtx);
    while (true)
    {
        const int64_t x = durable_lock_held_elsewhere();
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

int durable_log::flush_segment(segment* seg, const std::vector<uint64_t>& offs,
                               const std::vector<uint32_t>& lens, uint64_t used, uint64_t file_off)
{
    if (!offs.empty())
    {
        std::vector<uint32_t> crcs(offs.size());
        uint64_t total = 0;
        for (uint32_t l : lens) total += l;
        if (m_crc(m_crc_ctx, seg->arena, offs.data(), lens.data(), offs.size(), total,
                  crcs.data()) != 0)
            return EIO;
        // crc32c(crc32c(0, header, 16), entry) == crc32c(0, header || entry),
        // stored big-endian after the entry (txman/durable_log.cc:215-224)
        for (size_t i = 0; i < offs.size(); ++i) pack32be(crcs[i], seg->arena + offs[i] + lens[i]);
    }
    if (used && !pwrite_all(seg->fd, seg->arena, used, off_t(file_off))) return errno;
    if (fsync(seg->fd) < 0) return errno;
    return 0;
}

void durable_log::flush()
{
    sigset_t ss;
    if (sigfillset(&ss) < 0 || pthread_sigmask(SIG_BLOCK, &ss, nullptr) != 0)
    {
        std::lock_guard<std::mutex> hold(m_mtx);
        m_error = errno;
        return;
    }
    std::vector<uint64_t> offs;
    std::vector<uint32_t> lens;
    while (true)
    {
        uint64_t offset_saved, recno_saved, used, file_off;
        segment* seg = nullptr;
        {
            std::unique_lock<std::mutex> hold(m_mtx);
            while (m_error == 0 && !(seg = select_segment_fsync())) m_cond.wait(hold);
            if (m_error != 0) break;
            seg->syncing = true;
            seg->done_writing.wait(hold, [&] { return seg->ongoing_writes == 0; });
            offset_saved = seg->offset_next_write;
            recno_saved = seg->recno_last_write;
            used = seg->used;
            file_off = offset_saved - used;
            offs.swap(seg->frame_off);
            lens.swap(seg->frame_len);
            seg->frame_off.clear();
            seg->frame_len.clear();
        }
        const int e = flush_segment(seg, offs, lens, used, file_off);
        {
            std::lock_guard<std::mutex> hold(m_mtx);
            if (e) m_error = e;
            seg->syncing = false;
            if (!e)
            {
                seg->offset_last_fsync = offset_saved;
                seg->recno_last_fsync = recno_saved;
                seg->used = 0;
                ++m_flushes;
                m_frames_flushed += offs.size();
            }
            m_cond.notify_all();
        }
        offs.clear();
        lens.clear();
    }
}

durable_log::segment* durable_log::select_segment_write()
{
    segment* a = m_segment_a;
    segment* b = m_segment_b;
    const uint64_t a_unflushed = a->offset_next_write - a->offset_last_fsync;
    const uint64_t b_unflushed = b->offset_next_write - b->offset_last_fsync;
    if (a_unflushed < b_unflushed && !a->syncing) return a;
    if (a_unflushed > b_unflushed && !b->syncing) return b;
    if (!a->syncing) return a;
    if (!b->syncing) return b;
    return nullptr;
}

durable_log::segment* durable_log::select_segment_fsync()
{
    segment* a = m_segment_a;
    segment* b = m_segment_b;
    if (!a || !b) return nullptr;
    const uint64_t a_unflushed = a->offset_next_write - a->offset_last_fsync;
    const uint64_t b_unflushed = b->offset_next_write - b->offset_last_fsync;
    if (a_unflushed < b_unflushed) return b;
    if (a_unflushed > b_unflushed) return a;
    if (a_unflushed > 0) return a;
    if (b_unflushed > 0) return b;
    return nullptr;
}

int64_t durable_log::durable_lock_held_elsewhere()
{
    segment* a = m_segment_a;
    segment* b = m_segment_b;
    if (!a || !b) return 1;
    if (a->recno_last_fsync > b->recno_last_fsync) std::swap(a, b);
    if (a->offset_next_write - a->offset_last_fsync > 0) return int64_t(a->recno_last_fsync + 1);
    return int64_t(b->recno_last_fsync + 1);
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
        if (scan_frames(bufs[i].data(), bufs[i].size(), fn, ctx, &frames[i], nullptr) < 0)
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
    explicit mi_dlog(size_t cap) : log(cap) {}
    durable_log log;
};

extern "C" {

mi_dlog* mi_dlog_create(size_t segment_capacity) { return new mi_dlog(segment_capacity); }
void mi_dlog_destroy(mi_dlog* l) { delete l; }
int mi_dlog_open(mi_dlog* l, const char* dir) { return l->log.open(dir) ? 1 : 0; }
void mi_dlog_close(mi_dlog* l) { l->log.close(); }
int64_t mi_dlog_append(mi_dlog* l, const void* entry, size_t sz)
{
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
uint64_t mi_dlog_frames_flushed(mi_dlog* l) { return l->log.frames_flushed(); }
void mi_dlog_set_batch_crc_for_testing(mi_dlog* l, mi_dlog_batch_crc fn, void* ctx)
{
    l->log.set_batch_crc_for_testing(fn, ctx);
}

int64_t mi_dlog_scan_file(const char* path, uint64_t* valid_bytes, uint64_t* recnos,
                          uint64_t* offsets, size_t max_frames)
{
    std::vector<unsigned char> buf;
    if (!read_file(-1, path, &buf)) return -1;
    std::vector<Frame> frames;
    const int64_t n = scan_frames(buf.data(), buf.size(), gpu_batch, nullptr, &frames, valid_bytes);
    if (n < 0) return -1;
    for (size_t i = 0; i < frames.size() && i < max_frames; ++i)
    {
        if (recnos) recnos[i] = frames[i].recno;
        if (offsets) offsets[i] = frames[i].offset;
    }
    return n;
}

}  // extern "C"
