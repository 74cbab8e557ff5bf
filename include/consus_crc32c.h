/* include/consus_crc32c.h -- C ABI of the MI355X CRC-32C engine
 * (libconsus_crc32c.so).
 *
 * This is the drop-in boundary for Consus's durable-log checksum path.  Every
 * entry point computes exactly what consus::crc32c computes
 * (common/crc32c.h:40-41, common/crc32c.cc:122-126): reflected CRC-32C
 * (Castagnoli, poly 0x82F63B78), `init` is a previous CRC *output* (pre- and
 * post-inverted), n == 0 returns init.  Results are bit-identical to the
 * reference on every input.  The checksums are computed by the HIP kernels on
 * the GPU.  The drop-in `mi_crc32c` / `consus::crc32c` is total, as the
 * reference is: if the engine fails (no usable gfx950 device, a HIP error, an
 * input beyond the engine's limits) the call is completed by the engine's own
 * CPU path and counted in mi_crc32c_stats().  Status-returning calls return
 * the failure, unless called with MI_CRC32C_FALLBACK on host memory, in which
 * case they complete on the CPU path too (and count it).
 *
 * Plain C types only; the caller owns every buffer.  Pointers are host
 * pointers unless MI_CRC32C_DEVICE is passed, in which case every pointer
 * argument of that call is a device pointer on the engine's device.  All
 * calls are thread-safe: each calling thread gets its own HIP stream and
 * workspaces.
 */
#ifndef CONSUS_CRC32C_H
#define CONSUS_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define MI_CRC32C_OK 0
#define MI_CRC32C_EINVAL (-22)  /* bad argument (null pointer with count > 0, ...) */
#define MI_CRC32C_ENODEV (-19)  /* no usable gfx950 device */
#define MI_CRC32C_ENOMEM (-12)  /* device or pinned allocation failed */
#define MI_CRC32C_EHIP (-5)     /* a HIP runtime call failed; see mi_crc32c_last_error() */
#define MI_CRC32C_ERCCL (-71)   /* an RCCL call failed */
#define MI_CRC32C_ERANGE (-34)  /* input beyond the GPU engine's limits (>= 2^31 records,
                                   device addresses >= 2^47, > 2^32 planned pieces) */

/* ---- flags -------------------------------------------------------------- */
#define MI_CRC32C_DEVICE 0x1u   /* pointer arguments are device pointers */
#define MI_CRC32C_ASYNC 0x2u    /* DEVICE only: return once enqueued on the
                                   calling thread's stream (mi_crc32c_stream_sync) */
#define MI_CRC32C_PLANNED 0x4u  /* mi_crc32c_batch on host memory: always take the
                                   planned path (plan -> chunks -> finalize), even
                                   for a batch of short records small enough for
                                   the one-launch direct kernel (tests, tuning) */
#define MI_CRC32C_FALLBACK 0x8u /* host memory only: if the GPU engine fails, complete the
                                   call on the engine's CPU path (counted in
                                   mi_crc32c_stats) instead of returning the failure.
                                   Bad arguments (MI_CRC32C_EINVAL) still fail. */
#define MI_CRC32C_CPU 0x10u     /* mi_crc32c_batch[_multi] on host memory: hash on the
                                   engine's CPU path (crc32q) by the caller's choice, no
                                   GPU involved -- the durable log sends flushes below its
                                   measured GPU/CPU crossover this way (counted in
                                   host_batches / host_batch_bytes, not as a fallback) */

/* ---- engine ------------------------------------------------------------- */
/* Select the device and upload the operator tables.  Idempotent; called
 * implicitly with device 0 by the first compute call.
 * replaces: the static-init dispatch choose_crc32c (common/crc32c.cc:101-120) */
int mi_crc32c_init(int device);
const char* mi_crc32c_strerror(int status);
/* Message of the last failure on the calling thread ("" if none). */
const char* mi_crc32c_last_error(void);
/* Number of usable (gfx950) devices; does not initialise them. */
int mi_crc32c_device_count(void);
/* PCI bus id ("0000:05:00.0") of HIP device `device` into buf (len bytes);
 * identifies which physical GPU a rank runs on. */
int mi_crc32c_device_pci_bus_id(int device, char* buf, int len);
/* The HIP stream (hipStream_t) the calling thread's work is enqueued on. */
void* mi_crc32c_stream(void);
int mi_crc32c_stream_sync(void);

/* Counters of the whole process.  The GPU parity tests assert that
 * fallback_calls and host_routed_calls stay 0: they certify the HIP kernels,
 * not the CPU path. */
#define MI_CRC32C_MAX_DEVICES 16
typedef struct mi_crc32c_stats_t
{
    uint64_t gpu_calls;           /* compute calls completed by the HIP kernels */
    uint64_t fallback_calls;      /* calls (or shards) completed by the CPU path after an
                                     engine failure */
    uint64_t fallback_bytes;      /* bytes the CPU path hashed after engine failures */
    uint64_t sharded_calls;       /* multi-device calls split over more than one range */
    uint64_t host_routed_calls;   /* single host calls below the GPU threshold answered by the
                                     CPU path by design (mi_crc32c_set_gpu_min) */
    int32_t last_fallback_status; /* engine status that forced the last fallback (0: none) */
    int32_t last_multi_ranges;    /* ranges of the last multi-device call (0: none yet) */
    uint64_t sorted_batches;      /* variable-length batches hashed by the sorted path */
    uint64_t host_routed_bytes;   /* bytes of those routed calls */
    int32_t last_multi_devices[MI_CRC32C_MAX_DEVICES]; /* device ordinal of each range of the
                                     last multi-device call, in range order (-1: unused) */
    uint64_t zero_copy_batches;   /* host batches the kernels read in place from mapped
                                     pinned memory (mi_host_malloc_pinned) */
    uint64_t hint_overflows;      /* asynchronous device batches whose total_bytes hint
                                     understated their records (reported by the next
                                     mi_crc32c_stream_sync, which then fails) */
    uint64_t host_batches;        /* batches hashed on the CPU path by the caller's choice
                                     (MI_CRC32C_CPU: durable-log flushes below the
                                     crossover) */
    uint64_t host_batch_bytes;    /* bytes of those batches */
    uint64_t sorted_one_launch;   /* sorted batches hashed in one launch (grid barrier) */
    uint64_t window_batches;      /* variable-length batches hashed by the window path
                                     (mid-size device batches, one launch) */
} mi_crc32c_stats_t;
void mi_crc32c_stats(mi_crc32c_stats_t* out);
void mi_crc32c_stats_reset(void);

/* Size routing of single host calls: mi_crc32c /
 * consus::crc32c and mi_crc32c_buffer on HOST memory with n < gpu_min bytes
 * are answered by the engine's CPU path, without a GPU round trip; larger
 * ones, every batch and every device buffer go to the GPU.  The default is
 * the crossover measured on MI355X; env
 * MI_CRC32C_GPU_MIN (bytes) overrides it at load, this call at run time
 * (0 = every call on the GPU, as the GPU parity tests run).  Returns the
 * previous value. */
uint64_t mi_crc32c_set_gpu_min(uint64_t gpu_min);
uint64_t mi_crc32c_gpu_min(void);

/* ---- the drop-in -------------------------------------------------------- */
/* Same signature and semantics as consus::crc32c; never fails (engine failures
 * complete on the CPU path, counted in mi_crc32c_stats).
 * replaces: uint32_t consus::crc32c(uint32_t init, const unsigned char* data, size_t n)
 *           common/crc32c.h:40-41, common/crc32c.cc:122-126 */
uint32_t mi_crc32c(uint32_t init, const void* data, size_t n);

/* Status-returning single-buffer form; `data` host or device per flags,
 * `out` always a host pointer. */
int mi_crc32c_buffer(uint32_t init, const void* data, size_t n, uint32_t* out, unsigned flags);

/* ---- batches: the durable-log record-batching path ---------------------- */
/* Record i is the byte range [base + offsets[i], base + offsets[i] + lengths[i]);
 * out[i] = consus::crc32c(inits ? inits[i] : 0, that range).
 * Ranges may be unaligned, empty, unordered or overlapping.  total_bytes is
 * the sum of lengths if the caller knows it (0 = unknown: with DEVICE arrays
 * the engine then reads the plan size back once); it must not understate
 * the sum.  With DEVICE arrays and an understated hint no device access goes
 * out of bounds; a synchronous call detects it and recomputes the batch on
 * the path that reads its plan size back (exact results, slower); with
 * MI_CRC32C_ASYNC the contents of out[] are then unspecified.
 * replaces: the per-record call pair crc32c(crc32c(0, header, 16), entry, n)
 *           in durable_log::append, txman/durable_log.cc:215-218 */
int mi_crc32c_batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                    const uint32_t* inits, size_t count, uint64_t total_bytes, uint32_t* out,
                    unsigned flags);

/* Fixed-stride records: record i = [base + i*stride, +length). */
int mi_crc32c_batch_fixed(const void* base, uint64_t stride, uint64_t length,
                          const uint32_t* inits, size_t count, uint32_t* out, unsigned flags);

/* ---- multi-device host batches ------------------------- */
/* The batch is cut into contiguous record ranges of about equal bytes
 * (mi_crc32c_balanced_ranges), one per device, and each range is staged over
 * its own device's PCIe link and hashed there, concurrently (one persistent
 * worker thread per extra device).  Only as many devices are used as keep
 * every range >= shard_min_bytes (0 = the measured default, 4 MiB;
 * env MI_CRC32C_SHARD_MIN overrides the default), so small batches stay on
 * one device.  devices/ndev: the ordinals to use (a list may repeat an
 * ordinal: two ranges on one device, two streams); devices NULL = the
 * list in env MI_CRC32C_DEVICES ("0,1,2,3") if set, else the usable devices;
 * ndev > 0 then caps how many are used, ndev <= 0 = all of them.  Host memory only: device-resident
 * records are hashed where they live (mi_crc32c_batch with MI_CRC32C_DEVICE).
 * Flags: MI_CRC32C_FALLBACK (per range), MI_CRC32C_PLANNED.
 * replaces: the per-record crc32c calls of durable_log::append
 *           (txman/durable_log.cc:215-218) for a whole flushed segment. */
int mi_crc32c_batch_multi(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                          const uint32_t* inits, size_t count, uint64_t total_bytes,
                          uint32_t* out, unsigned flags, const int* devices, int ndev,
                          uint64_t shard_min_bytes);
/* Fixed-stride records, equal record counts per device. */
int mi_crc32c_batch_fixed_multi(const void* base, uint64_t stride, uint64_t length,
                                const uint32_t* inits, size_t count, uint32_t* out,
                                unsigned flags, const int* devices, int ndev,
                                uint64_t shard_min_bytes);
/* The split rule: bounds[0..k] with bounds[0] = 0, bounds[k] = count; range r
 * = records [bounds[r], bounds[r+1]) ends at the first record whose inclusive
 * prefix sum of lengths reaches ceil(total * r / k). */
void mi_crc32c_balanced_ranges(const uint32_t* lengths, size_t count, int k, uint64_t total,
                               size_t* bounds);

/* crc32c(0, A || B) from crc_a = crc32c(0, A), crc_b = crc32c(0, B) and |B|
 * (the chaining identity of common/crc32c.cc:122-126).  Pure operator math. */
uint32_t mi_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
int mi_crc32c_combine_batch(const uint32_t* crc_a, const uint32_t* crc_b, const uint64_t* len_b,
                            size_t count, uint32_t* out, unsigned flags);

/* ---- streaming host segments (H2D -> CRC -> D2H overlapped) ------------- */
/* A pipeline of `depth` slots, each with pinned staging for one segment of
 * up to max_segment_bytes and max_records records, on its own HIP stream.
 * submit() enqueues H2D + kernels + D2H of the CRCs and returns a ticket;
 * wait() blocks until that ticket's CRCs are in host_out.  Submitting into a
 * busy slot waits for that slot's previous ticket first.
 * Buffer ownership: a PAGEABLE host_segment is copied into the slot's pinned
 * staging before submit() returns, so the caller may reuse it at once.  A
 * PINNED host_segment (mi_host_malloc_pinned, hipHostMalloc) is DMA'd in place
 * -- no extra copy, which is what makes a pinned producer fast -- so it must
 * stay allocated and unmodified until wait(ticket) returns; the CRCs are of
 * the bytes the DMA reads.  offsets/lengths/inits are copied by submit(). */
typedef struct mi_crc32c_pipeline mi_crc32c_pipeline;
int mi_crc32c_pipeline_create(size_t max_segment_bytes, size_t max_records, int depth,
                              mi_crc32c_pipeline** out);
int mi_crc32c_pipeline_submit(mi_crc32c_pipeline* p, const void* host_segment, size_t bytes,
                              const uint64_t* offsets, const uint32_t* lengths,
                              const uint32_t* inits, size_t count, uint32_t* host_out,
                              uint64_t* ticket);
int mi_crc32c_pipeline_wait(mi_crc32c_pipeline* p, uint64_t ticket);
int mi_crc32c_pipeline_destroy(mi_crc32c_pipeline* p);

/* ---- device memory and synthetic inputs --------------------------------- */
/* For callers without their own allocator (tests, bench, the durable log). */
int mi_dev_malloc(void** p, size_t bytes);
int mi_dev_free(void* p);
int mi_host_malloc_pinned(void** p, size_t bytes);
int mi_host_free_pinned(void* p);
#define MI_MEMCPY_H2D 1
#define MI_MEMCPY_D2H 2
#define MI_MEMCPY_D2D 3
int mi_memcpy(void* dst, const void* src, size_t bytes, int kind); /* synchronous */
int mi_memset(void* dev, int value, size_t bytes);
/* bytes [byte_offset, byte_offset + nbytes) of the splitmix64 stream of `seed`
 * (SURVEY.md 8(d)); dev 8-byte aligned, byte_offset a multiple of 8. */
int mi_fill_splitmix64(void* dev, size_t nbytes, uint64_t seed, uint64_t byte_offset);

/* Host-side synthetic record lengths of BASELINE.json config 3 (Zipf 64 B -
 * 64 KiB; definition in consus_amd/csrc/workload.cc).  No device needed. */
void mi_workload_zipf_lengths(uint64_t seed, uint64_t first, size_t count, uint32_t* out);

/* ---- timing on the calling thread's stream ------------------------------ */
int mi_timer_start(void);
int mi_timer_stop(float* elapsed_ms); /* synchronizes the stream */

/* ---- multi-GPU: RCCL over xGMI ------------------------------------------ */
#define MI_COMM_ID_BYTES 128
int mi_comm_unique_id(unsigned char id[MI_COMM_ID_BYTES]);
int mi_comm_init(const unsigned char id[MI_COMM_ID_BYTES], int nranks, int rank);
/* recv[r * count + i] = send_of_rank_r[i]; device pointers, calling thread's stream */
int mi_comm_allgather_u32(const uint32_t* dev_send, size_t count, uint32_t* dev_recv);
/* ranks of the communicator as RCCL counts them (ncclCommCount), this rank
 * (ncclCommUserRank) and its device (ncclCommCuDevice) */
int mi_comm_info(int* nranks, int* rank, int* device);
int mi_comm_destroy(void);

#ifdef __cplusplus
}
#endif

#endif /* CONSUS_CRC32C_H */
