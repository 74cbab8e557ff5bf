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
//     (:421-440); the flush thread fsyncs the segment with the most unflushed
//     bytes while appends go to the other one (:287-419).
// What changes: append() copies the frame into the segment's staging buffer
// (pinned host memory) and defers its CRC; the flush thread computes the CRCs
// of every staged frame of the segment in ONE GPU batch
// (mi_crc32c_batch), patches them in, writes the segment with one pwrite and
// fsyncs it before publishing the watermark -- so the watermark still covers
// only records whose CRC bytes are on disk.
// replay() -- declared but never defined by the reference (:64, TODO:2-3) --
// is implemented as a GPU-verified scan of both segment files.
#ifndef consus_txman_log_h_
#define consus_txman_log_h_

#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace consus {

// CRC engine for a batch of frames (default: the GPU, mi_crc32c_batch).
typedef int (*durable_log_batch_crc)(void* ctx, const void* base, const uint64_t* offsets,
                                     const uint32_t* lengths, size_t count, uint64_t total_bytes,
                                     uint32_t* out);

class durable_log
{
    public:
        durable_log();
        explicit durable_log(size_t segment_capacity);
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

    private:
        struct segment;
        void flush();
        segment* select_segment_write();
        segment* select_segment_fsync();
        int64_t durable_lock_held_elsewhere();
        int flush_segment(segment* seg, const std::vector<uint64_t>& offs,
                          const std::vector<uint32_t>& lens, uint64_t used, uint64_t file_off);

    private:
        std::string m_path;
        int m_dir;
        int m_lock_fd;
        std::mutex m_mtx;
        std::condition_variable m_cond;
        std::thread m_flush;
        int m_error;
        bool m_wakeup;
        bool m_opened;
        uint64_t m_next_entry;
        size_t m_capacity;
        segment* m_segment_a;
        segment* m_segment_b;
        durable_log_batch_crc m_crc;
        void* m_crc_ctx;
        bool m_pinned;
        std::atomic<uint64_t> m_flushes;
        std::atomic<uint64_t> m_frames_flushed;

    private:
        durable_log(const durable_log&);
        durable_log& operator = (const durable_log&);
};

}  // namespace consus

#endif // consus_txman_log_h_
