// include/txman/durable_log.h -- drop-in replacement for Consus's
// txman/durable_log.h with a record-batching front-end for the MI355X
// CRC-32C engine.
//
// replaces: class consus::durable_log, txman/durable_log.h:53-93
// Same public interface and the same contracts:
//   * append() returns the record number at once (1, 2, ...), or -1 with errno
//     set after an I/O error (txman/durable_log.cc:187-242);
//   * the on-disk frame is [recno u64 BE][len u64 BE][entry][crc u32 BE] with
//     crc = consus::crc32c(consus::crc32c(0, header, 16), entry, len)
//     (txman/durable_log.cc:54-61, 215-224), in two alternating segment files
//     file_a / file_b created (truncated) by open() (:157-169);
//   * durable() / wait() report the watermark "every recno < x is durable"
//     (:421-440); one segment is fsynced while appends go to the other one
//     (:287-419).
// What changes: append() reserves its record number and staging offset with
// one fetch-and-add on the active segment (no lock on the append path),
// copies the frame into the segment's staging buffer (pinned host memory)
// and defers its CRC; the flush thread computes the CRCs
// of every staged frame of the segment in ONE GPU batch
// (mi_crc32c_batch), patches them in and writes the segment with one pwrite;
// a sync thread fsyncs it and only then publishes the watermark -- so the
// watermark still covers only records whose CRC bytes are on disk.  The
// fsync of one segment overlaps the CRC and write of the next (at most one
// written segment waits for its fsync).
// Errors: as in the reference, whose flush thread stops at the first error
// (:226-230, :287-347), the first error -- an I/O error, or ENOMEM when an
// oversized frame's own staging buffer cannot be allocated -- stops the log:
// later appends fail, segments not yet fsynced are dropped, and the
// watermark never passes the record that failed.
// replay() -- declared but never defined by the reference (:64, TODO:2-3) --
// is implemented as a GPU-verified scan of both segment files.
#ifndef consus_txman_log_h_
#define consus_txman_log_h_

#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

// consus
#include "namespace.h"

BEGIN_CONSUS_NAMESPACE

// CRC engine for a batch of frames (default: the GPU, mi_crc32c_batch_multi).
typedef int (*durable_log_batch_crc)(void* ctx, const void* base, const uint64_t* offsets,
                                     const uint32_t* lengths, size_t count, uint64_t total_bytes,
                                     uint32_t* out);

// Tuning knobs (the reference has none: txman/main.cc:84-117 parses only
// daemon flags; these map onto the same flag style, e.g. --log-segment-mb).
struct durable_log_options
{
    size_t segment_capacity = 0;   // bytes of staged frames per segment; 0 = 64 MiB
    int gpus = 0;                  // devices one flush may shard over: 0 = every usable
                                   // gfx950 device, 1 = the engine's default device only
    uint64_t shard_min_bytes = 0;  // per-device share below which a flush stays on fewer
                                   // devices; 0 = the engine's measured default (4 MiB)
    int64_t host_batch_max = -1;   // a flush whose frames total fewer bytes is checksummed
                                   // on the flush thread's CPU (crc32q, MI_CRC32C_CPU):
                                   // -1 = the measured GPU/CPU crossover
                                   // (kHostBatchMaxDefault in durable_log.cc), 0 = never;
                                   // the environment's MI_DLOG_HOST_BATCH_MAX overrides
};

// As in the reference, the class sits in Consus's hidden-visibility namespace
// (namespace.h:4-5).  The reference compiles durable_log.cc into the txman
// executable; here libconsus_crc32c.so carries it (with the mi_dlog_* C ABI),
// so the class alone is given default visibility to be linkable from it.
class __attribute__((visibility("default"))) durable_log
{
    public:
        durable_log();
        explicit durable_log(size_t segment_capacity);
        explicit durable_log(const durable_log_options& options);
        ~durable_log() throw ();

    public:
        bool open(const std::string& dir);
        void close();
        int64_t append(const char* entry, size_t entry_sz);
        int64_t append(const unsigned char* entry, size_t entry_sz);
        int64_t replay(void (*f)(void*, const unsigned char*, size_t), void* p);
        int64_t durable();
        int64_t wait(int64_t prev_ub);
        void wake();
        int error();

    public:
        // Test hook: run the host logic with another batch engine (CPU tests
        // inject the oracle).  Must be called before open().
        void set_batch_crc_for_testing(durable_log_batch_crc fn, void* ctx);
        // Counters for tests and tuning.
        uint64_t flushes() const;
        uint64_t frames_flushed() const;
        // Seconds spent per phase: copy wait, frame walk, batch CRC, CRC
        // patch, pwrite (flush thread), fsync (sync thread).
        void flush_seconds(double out[6]) const;
        // the longest single occurrence of each phase (same order), seconds
        void flush_max_seconds(double out[6]) const;
        // Test hook: every fsync also sleeps this long (a slow disk on tmpfs).
        void set_fsync_delay_for_testing(uint32_t microseconds);
        // Bench hook (call before open): the writer and the sync thread skip
        // pwrite and fsync (storage faster than the appenders and the
        // checksum), so the log's rate is its front-end's; the files stay
        // empty (no replay).
        void set_sink_for_testing(bool sink);
        // Most bytes of oversized frames (staged outside the arenas) held at
        // once: at most max(2 x segment capacity, 16 MiB, the largest such
        // frame).
        uint64_t external_bytes_peak() const;
        // Test hook (call before open): every append calls fn(ctx, point) at
        // point 0, after it has read the active segment and before it
        // reserves in it, and at point 1, after a reservation that failed
        // (segment sealed or full) and before it waits for the flush thread
        // to switch segments.  A test parks one appender there while the
        // flush thread switches segments under it.
        void set_append_hook_for_testing(void (*fn)(void* ctx, int point), void* ctx);
        // Bench hook (call before open): the reference's checksum placement
        // (txman/durable_log.cc:215-218) -- every appender computes its
        // frame's CRC with fn(0, header || entry) on its own thread, outside
        // any lock, and stores it in the frame; the flush thread then
        // checksums nothing.  bench.py's durable-log leg times the reference
        // common/crc32c.cc this way beside the batch engines.
        void set_append_crc_for_testing(uint32_t (*fn)(uint32_t, const unsigned char*, size_t));
        // Test hook: the staging malloc of an oversized frame fails (ENOMEM).
        void set_external_malloc_failure_for_testing(bool fail);
        // Flushes checksummed on the flush thread's CPU (below host_batch_max).
        uint64_t host_flushes() const;
        // Test hook (call before open): stage frames in pinned (true) or
        // ordinary (false) memory whatever the batch engine (an injected
        // engine defaults to ordinary memory, the GPU batch to pinned).
        void set_pinned_arenas_for_testing(bool pinned);
        // Bench hook: one row per flushed segment, up to max_rows, of 7
        // values -- seconds since open() when it was sealed, checksummed
        // (CRCs patched in), handed to the writer, written from, written to,
        // synced, and its bytes.  Returns the rows written.
        size_t flush_timeline(double* out, size_t max_rows);
        // One line of the log's internal state (flush-thread phase, the
        // active segment's reservation word, queued jobs, appenders waiting
        // for a switch) for watchdogs; writes at most n bytes, NUL included.
        void debug_state(char* buf, size_t n);

    private:
        struct segment;
        struct write_job;                   // a checksummed segment's bytes for the writer
        struct synced                       // a written segment awaiting fsync
        {
            int fd;
            uint64_t upto;                  // watermark once it is synced
            uint64_t frames;
            size_t row;                     // its flush_timeline row
        };
        void flush();
        void warm_up();
        void writer();
        void sync();
        int64_t append_slow(segment* seg, uint64_t gen);
        void switch_to_next(segment* seg, uint64_t n);
        int prepare_segment(segment* seg, uint64_t& nframes, uint64_t& used, write_job* job);
        int write_out(write_job* job);
        bool charge_external(uint64_t bytes);
        void release_external(uint64_t bytes);
        int batch_crc(const unsigned char* base, const uint64_t* offs, const uint32_t* lens,
                      size_t n, uint64_t total, uint32_t* out);
        uint32_t frame_crc(const unsigned char* frame, uint64_t length);

    private:
        std::string m_path;
        int m_dir;
        int m_lock_fd;
        std::mutex m_mtx;               // flush hand-offs, waiters; never on the append fast path
        std::condition_variable m_cond;
        std::thread m_flush;
        std::thread m_writer;           // pwrites checksummed segments (beside the next CRC)
        std::thread m_sync;             // fsyncs written segments, publishes the watermark
        std::atomic<int> m_error;
        bool m_wakeup;
        bool m_opened;
        size_t m_capacity;
        durable_log_options m_opts;
        segment* m_segment_a;
        segment* m_segment_b;
        std::atomic<segment*> m_active;      // the segment appends reserve in
        // segment switches so far, bumped after m_active is stored: an
        // appender that saw generation g and a sealed or full segment waits
        // for a generation != g (waiting on m_active != seg was ABA-prone:
        // two switches bring the same segment back)
        std::atomic<uint64_t> m_switch_gen;
        std::atomic<int> m_flush_phase;      // what the flush thread is doing (debug_state)
        std::atomic<int> m_slow_waiters;     // appenders waiting for a switch (debug_state)
        void (*m_append_hook)(void*, int);   // test hook, set before open()
        void* m_append_hook_ctx;
        std::atomic<uint64_t> m_durable;     // every recno below it is on disk
        std::atomic<bool> m_flush_idle;      // the flush thread sleeps for a first frame
        durable_log_batch_crc m_crc;
        void* m_crc_ctx;
        uint64_t m_host_max;                 // flushes below this many bytes: the CPU path
        std::atomic<uint64_t> m_host_flushes;
        uint32_t (*m_append_crc)(uint32_t, const unsigned char*, size_t);  // bench hook
        std::atomic<bool> m_ext_malloc_fail;  // test hook
        bool m_pinned;
        std::atomic<uint64_t> m_flushes;
        std::atomic<uint64_t> m_frames_flushed;
        std::atomic<uint64_t> m_flush_ns[6];
        std::atomic<uint64_t> m_flush_max_ns[6];
        void note_phase(int phase, uint64_t ns);
        std::vector<uint64_t> m_offs;   // flush thread: the sealed segment's frames
        std::vector<uint32_t> m_lens;
        std::vector<uint32_t> m_crcs;
        std::vector<synced> m_pending;  // under m_mtx: at most one written, unsynced segment
        std::vector<write_job*> m_jobs; // under m_mtx: at most one segment for the writer
        unsigned char* m_spare;         // under m_mtx: the third staging arena, free (null:
        bool m_spare_pinned;            //   the writer holds it)
        bool m_stop_writer;             // under m_mtx: the destructor ends the writer thread
        bool m_stop;                    // under m_mtx: the destructor ends the sync thread
        std::atomic<uint32_t> m_fsync_delay_us;
        bool m_sink;                    // bench hook: no pwrite, no fsync
        // bytes of frames staged outside the arenas (entries of more than
        // half a segment), both segments together; bounded like the arenas
        std::atomic<uint64_t> m_ext_bytes;
        std::atomic<uint64_t> m_ext_peak;
        // flush_timeline: rows of 7 (under m_mtx), times from m_t_open
        std::vector<double> m_timeline;
        std::chrono::steady_clock::time_point m_t_open;
        double since_open() const;
        void mark(size_t row, int col, double v);

    private:
        durable_log(const durable_log&);
        durable_log& operator = (const durable_log&);
};

END_CONSUS_NAMESPACE

#endif // consus_txman_log_h_
