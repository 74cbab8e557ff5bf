// consus_amd/csrc/engine.hip -- host side of the MI355X CRC-32C engine:
// the C ABI of include/consus_crc32c.h.
//
// Owns: device selection and the operator-table image (uploaded once),
// one HIP stream + grow-only workspaces per calling thread (the reference
// function is called concurrently by N txman worker threads,
// txman/durable_log.cc:215-218 runs outside m_mtx), staging of host batches,
// the streaming pipeline, and the RCCL communicator.
//
// No CRC over payload bytes is ever computed on the host here: every checksum
// comes from the kernels in crc32c_kernels.hip.  Host code only does
// operator algebra (table construction, combine of finished CRCs).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/consus_crc32c.h"
#include "crc32c_kernels.h"
#include "crc32c_math.h"
#include "engine_internal.h"
#include "host_crc.h"

using namespace mi_crc;
using mi_eng::fail;
using mi_eng::kMaxDevices;

namespace {

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(MI_CRC32C_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Host batches whose packed inputs fit this take one staging copy.
constexpr uint64_t kPackMax = uint64_t(4) << 20;
constexpr uint64_t kPackInPlace = uint64_t(512) << 10;
constexpr uint64_t kZeroCopyMax = uint64_t(8) << 10;  // packed inputs read in place by the GPU
// completion word of synchronous direct launches: pin_small word, and how
// long the host spins on it before it blocks in a stream sync
constexpr int kDoneWord = 16;
constexpr int kDoneSpinUs = 1000;
// ... and up to which batch size (bytes hashed) it beats the stream sync:
// above ~2 MB the sync returned 5-14 us sooner (tools/flush_probe, 3 rounds:
// 4,096 frames / 2.28 MB 78.7-83.2 us vs 84.3-88.0; 8,192 / 4.56 MB
// 138.5-146.0 vs 152.4-159.7; 2,048 / 1.13 MB still 1-2 us slower;
// profiles/r03_done_word_crossover.txt)
constexpr uint64_t kDoneWordMaxBytes = uint64_t(2) << 20;

// MI_CRC32C_DONE_WORD=0: synchronous direct launches wait in a stream sync
// instead of spinning on their completion word (A/B; read per batch).
bool done_word_disabled()
{
    const char* e = std::getenv("MI_CRC32C_DONE_WORD");
    return e && !std::strcmp(e, "0");
}
// Device buffers from this size take launch_single (fixed-record kernel on
// the 4 KiB chunks + a two-level combine tree) instead of the variable path.
constexpr uint64_t kSingleMin = 64 * 1024;

struct DeviceState
{
    int ordinal = -1;
    int cus = 0;
    uint32_t* d_tables = nullptr;  // kTabWords
    uint32_t* d_pow2 = nullptr;    // 48 x 1024: G^{2^k}
    Op32 pow2_ops[64];             // host copies for mi_crc32c_combine
    uint32_t crc0 = 0;             // crc32c(0, 4096 zero bytes): chunk CRC -> raw register
    std::string arch;
    // thread contexts of this process that have run the sorted path on the
    // device: the one-launch (grid-barrier) form only while it is 1
    std::atomic<int> sorted_users{0};
};

std::mutex g_mu;
std::atomic<DeviceState*> g_devs[kMaxDevices];  // per ordinal, built on first use
std::atomic<int> g_default{-1};                 // the process's default device

// Fault injection for the fallback tests (read once): MI_CRC32C_FAULT=init
// makes every device fail to initialise (as on a host without a usable GPU);
// =compute initialises normally but fails every compute call with EHIP (a
// HIP error at run time).  Unset in production.
enum Fault { kFaultNone = 0, kFaultInit = 1, kFaultCompute = 2 };
int fault_mode()
{
    static const int mode = [] {
        const char* e = std::getenv("MI_CRC32C_FAULT");
        if (!e) return int(kFaultNone);
        if (!std::strcmp(e, "init")) return int(kFaultInit);
        if (!std::strcmp(e, "compute")) return int(kFaultCompute);
        return int(kFaultNone);
    }();
    return mode;
}

bool is_gfx950(int device, std::string* arch = nullptr)
{
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
    {
        (void)hipGetLastError();
        return false;
    }
    if (arch) *arch = prop.gcnArchName;
    return std::string(prop.gcnArchName).find("gfx950") != std::string::npos;
}

// Builds the operator tables of `device` (once per device); the caller holds g_mu.
int build_device(int device)
{
    if (fault_mode() == kFaultInit)
        return fail(MI_CRC32C_ENODEV, "fault injected (MI_CRC32C_FAULT=init)");
    int n = 0;
    if (device < 0 || device >= kMaxDevices || hipGetDeviceCount(&n) != hipSuccess || n <= device)
    {
        (void)hipGetLastError();
        return fail(MI_CRC32C_ENODEV, "no HIP device " + std::to_string(device));
    }
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    std::string arch = prop.gcnArchName;
    if (arch.find("gfx950") == std::string::npos)
        return fail(MI_CRC32C_ENODEV, "device " + std::to_string(device) + " is " + arch +
                                          "; this engine is built for gfx950 (MI355X) only");
    auto* d = new DeviceState;
    d->ordinal = device;
    d->cus = prop.multiProcessorCount;
    d->arch = arch;
    // Operator-table image (crc32c_math.h): G^{128}, T_0..T_15, G^{32}, G^{64}, G^{4096}.
    std::vector<uint32_t> img(kTabWords);
    make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabMain]), kRowBytes);
    make_slice16_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabT]));
    make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZ32]), 32);
    make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZ64]), 64);
    make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZChunk]), kChunk);
    make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZLong]),
                     uint64_t(kLongBlock) * kChunk);
    for (int b = 0; b < 10; ++b)
        make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZC2 + b * 1024]),
                         uint64_t(kChunk) << b);
    for (int b = 0; b < 13; ++b)
        make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabP2 + b * 1024]),
                         uint64_t(1) << b);
    for (int k = 1; k <= 32; ++k)
        make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZRows + (k - 1) * 1024]),
                         uint64_t(kRowBytes) * k);
    for (uint32_t k = 1; k < kWinShifts; ++k)
        make_fold_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZWin + (k - 1) * 1024]),
                         uint64_t(512) * k);
    {
        Op32 inv;
        if (!invert(zeros_op(kRowBytes), &inv))
        {
            delete d;
            return fail(MI_CRC32C_EHIP, "Z_128 is not invertible (table construction bug)");
        }
        make_op_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZInv128]), inv);
        // Z_{-m} = Z_{-128} o Z_{128-m}, m = 0..127 (m = 0: the identity)
        for (int m = 0; m < kRowBytes; ++m)
            make_op_tables(reinterpret_cast<uint32_t(*)[256]>(&img[kTabZNeg + m * 1024]),
                           m ? zeros_op(uint64_t(kRowBytes - m)).then(inv) : Op32::identity());
    }
    {
        // lane-fold tables: 6-bit slices of the team fold's six shifts (chunk 5 holds bits 30-31)
        const uint64_t shifts[kLaneOps] = {16, 12, 8, 4, 32, 64, kRowBytes, 512, 1024};
        for (int k = 0; k < kLaneOps; ++k)
        {
            const Op32 z = zeros_op(shifts[k]);
            for (int c = 0; c < 6; ++c)
                for (uint32_t i = 0; i < 64; ++i)
                    img[kTabLane + (k * 6 + c) * 64 + i] = z.apply(c < 5 ? i << (6 * c) : (i & 3u) << 30);
        }
    }
    {
        // F[n] = Z_n(~0): the register a zero init reaches after n bytes of zeros
        const uint32_t* t0 = &img[kTabT];
        uint32_t f = 0xFFFFFFFFu;
        for (int n = 0; n <= int(kChunk); ++n)
        {
            img[kTabFInit + n] = f;
            f = t0[f & 0xFFu] ^ (f >> 8);
        }
    }
    d->crc0 = ~img[kTabFInit + kChunk];
    std::vector<uint32_t> pow2(48 * 1024);
    Op32 p = Op32::zero_byte();
    for (int k = 0; k < 64; ++k)
    {
        d->pow2_ops[k] = p;
        if (k < 48)
            for (int j = 0; j < 4; ++j)
                for (uint32_t b = 0; b < 256; ++b) pow2[k * 1024 + j * 256 + b] = p.apply(b << (8 * j));
        p = p.then(p);
    }
    hipError_t e = hipMalloc(&d->d_tables, img.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&d->d_pow2, pow2.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(d->d_tables, img.data(), img.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d->d_pow2, pow2.data(), pow2.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = configure_kernels();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess)
    {
        delete d;
        return fail(MI_CRC32C_EHIP, std::string("table upload: ") + hipGetErrorString(e));
    }
    g_devs[device].store(d);
    return MI_CRC32C_OK;
}

// The state of `device` (-1 = the default device), initialised on first use.
DeviceState* device_state(int device, int* status)
{
    if (device < 0)
    {
        device = g_default.load();
        if (device < 0)
        {
            std::lock_guard<std::mutex> lock(g_mu);
            if (g_default.load() < 0) g_default.store(0);
            device = g_default.load();
        }
    }
    if (device >= kMaxDevices)
    {
        *status = fail(MI_CRC32C_ENODEV, "device ordinal " + std::to_string(device) + " >= 16");
        return nullptr;
    }
    if (DeviceState* d = g_devs[device].load()) return d;
    std::lock_guard<std::mutex> lock(g_mu);
    if (DeviceState* d = g_devs[device].load()) return d;
    *status = build_device(device);
    return g_devs[device].load();
}

// mi_crc32c_init: the default device is chosen once per process.
int init_device(int device)
{
    {
        std::lock_guard<std::mutex> lock(g_mu);
        const int cur = g_default.load();
        if (cur >= 0 && device >= 0 && cur != device)
            return fail(MI_CRC32C_EINVAL, "engine already initialised on another device");
        if (cur < 0) g_default.store(device < 0 ? 0 : device);
    }
    int st = MI_CRC32C_OK;
    return device_state(-1, &st) ? MI_CRC32C_OK : st;
}

DeviceState* dev_or_init(int* status) { return device_state(-1, status); }

// Grow-only device buffer.
struct DevBuf
{
    void* p = nullptr;
    size_t cap = 0;
    int reserve(size_t bytes)
    {
        if (bytes <= cap) return MI_CRC32C_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 4096);
        want = want + want / 4;
        if (hipMalloc(&p, want) != hipSuccess)
            return fail(MI_CRC32C_ENOMEM, "hipMalloc(" + std::to_string(want) + ") failed");
        cap = want;
        return MI_CRC32C_OK;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T* as() const { return static_cast<T*>(p); }
};

struct PinBuf
{
    void* p = nullptr;
    void* dev = nullptr;  // the device's address of the same bytes (mapped pinned memory)
    size_t cap = 0;
    int reserve(size_t bytes)
    {
        if (bytes <= cap) return MI_CRC32C_OK;
        release();
        // powers of two from 64 KiB: pinning costs milliseconds, and a
        // durable log's flushes grow a few percent at a time (each regrowth
        // was a multi-ms stall of the flush thread: the p99 durability
        // latency of round 3's first dlog runs)
        size_t want = size_t(64) << 10;
        while (want < bytes) want <<= 1;
        if (hipHostMalloc(&p, want, hipHostMallocMapped) != hipSuccess)
        {
            p = nullptr;
            return fail(MI_CRC32C_ENOMEM, "hipHostMalloc(" + std::to_string(want) + ") failed");
        }
        if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess)
        {
            (void)hipGetLastError();
            dev = nullptr;  // no device mapping: callers stage through a copy
        }
        cap = want;
        return MI_CRC32C_OK;
    }
    template <typename T>
    T* as() const { return static_cast<T*>(p); }
    void release()
    {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        dev = nullptr;
        cap = 0;
    }
};

// Per-(thread or pipeline slot) execution context.
struct Ctx
{
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
    DevBuf data, off, len, inits, out;  // staging of host batches
    DevBuf items, partial, first_pos, int_pos, last_pos, blk, longs;
    DevBuf srt_cost, srt_ctrl, srt_items;  // sorted path (launch_sorted)
    DevBuf win_acc;                        // window path: acc64[count], acc[count], cnt[count], kept zero
    DevBuf done_ctr;                    // direct kernel's completion counter (DoneSignal)
    uint32_t done_seq = 0;
    PinBuf pin_small;                   // plan-size read-back; word kDoneWord: completion word
    PinBuf pin_stage, pin_out;          // packed small host batches: inputs, CRCs
    int ordinal = -1;
    // set by the last device batch: where its overflow shows when a caller's
    // size hint was too small (sorted path: ctrl[1] != 0; piece path: the
    // plan's item total > plan_cap)
    uint32_t* sorted_ctrl = nullptr;
    // an asynchronous sorted batch ran since the last stream sync: its
    // overflow (understated size hint) sits in the sticky ctrl[2]
    bool async_sorted_unchecked = false;
    // the sticky word as earlier asynchronous batches left it, read
    // before a synchronous batch ran on the stream (which may set and clear
    // the word itself); reported by the next stream sync
    bool async_overflow_latched = false;
    // the one-launch sorted form: this context counted in its device's
    // sorted_users, and the barrier counter's value before the next launch
    std::atomic<int>* sorted_users = nullptr;
    uint32_t bar_base = 0;
    bool force_unfused = false;  // the retry after a timed-out barrier
    uint32_t bar_tag = 0;        // ctrl[3] if the last one-launch batch's barrier timed out
    uint32_t* plan_total = nullptr;
    uint64_t plan_cap = 0;

    int open(int dev)
    {
        ordinal = dev;
        HIP_TRY(hipSetDevice(dev));
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreate(&ev0));
        HIP_TRY(hipEventCreate(&ev1));
        HIP_TRY(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        int st;
        if ((st = done_ctr.reserve(64))) return st;
        HIP_TRY(hipMemset(done_ctr.p, 0, 64));
        return pin_small.reserve(4096);
    }
    // The completion word of the next synchronous direct launch of `bytes`
    // (false: the pinned page has no device mapping, or the batch is larger
    // than kDoneWordMaxBytes; then the caller syncs the stream).
    bool next_signal(DoneSignal* s, uint64_t bytes)
    {
        if (!pin_small.dev || !done_ctr.p || bytes > kDoneWordMaxBytes || done_word_disabled())
            return false;
        volatile uint32_t* h = pin_small.as<uint32_t>() + kDoneWord;
        *h = 0;
        if (++done_seq == 0) done_seq = 1;
        *s = DoneSignal{done_ctr.as<uint32_t>(), static_cast<uint32_t*>(pin_small.dev) + kDoneWord,
                        done_seq};
        return true;
    }
    // Wait for the launch that carries `s` (or, without one, the stream):
    // spin on the completion word for up to kDoneSpinUs, then block in a stream
    // sync, which also reports any fault of the launch.
    int wait_direct(bool signalled)
    {
        if (signalled)
        {
            const volatile uint32_t* h = pin_small.as<uint32_t>() + kDoneWord;
            const auto t0 = std::chrono::steady_clock::now();
            for (uint32_t n = 0;; ++n)
            {
                if (*h == done_seq)
                {
                    std::atomic_thread_fence(std::memory_order_acquire);
                    return MI_CRC32C_OK;
                }
                __builtin_ia32_pause();
                if ((n & 255u) == 255u &&
                    std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kDoneSpinUs))
                    break;
            }
        }
        HIP_TRY(hipStreamSynchronize(stream));
        if (signalled && *static_cast<const volatile uint32_t*>(pin_small.as<uint32_t>() +
                                                                kDoneWord) != done_seq)
        {
            // The launch finished without storing its word: its counter did
            // not end at the grid size (a launch cut short), and only the
            // last workgroup resets it.  Zero it here, so the next launch's
            // last workgroup cannot fire before every CRC is stored.
            HIP_TRY(hipMemsetAsync(done_ctr.p, 0, 64, stream));
            HIP_TRY(hipStreamSynchronize(stream));
        }
        return MI_CRC32C_OK;
    }
    // Waits for the stream's work, then frees every buffer, event and the stream.
    void release()
    {
        if (stream) (void)hipStreamSynchronize(stream);
        if (sorted_users) sorted_users->fetch_sub(1);
        sorted_users = nullptr;
        for (DevBuf* b : {&data, &off, &len, &inits, &out, &items, &partial, &first_pos, &int_pos,
                          &last_pos, &blk, &longs, &srt_cost,
                          &srt_ctrl, &srt_items, &win_acc, &done_ctr})
            b->release();
        for (PinBuf* b : {&pin_small, &pin_stage, &pin_out}) b->release();
        for (hipEvent_t* e : {&ev0, &ev1, &done})
            if (*e)
            {
                (void)hipEventDestroy(*e);
                *e = nullptr;
            }
        if (stream) (void)hipStreamDestroy(stream);
        stream = nullptr;
    }
};

// One context per (calling thread, device), released when the thread exits
// (a durable log's flush thread lives as long as the log is open; its
// workspaces go with it; the multi-device workers of api.cc live as long as
// the process).
struct ThreadCtx
{
    Ctx* c[kMaxDevices] = {};
    ~ThreadCtx()
    {
        for (Ctx*& x : c)
            if (x)
            {
                (void)hipSetDevice(x->ordinal);
                x->release();
                delete x;
                x = nullptr;
            }
    }
};
thread_local ThreadCtx t_ctx;

// The calling thread's context on `dev` (-1 = default device); makes `dev`
// the thread's current HIP device (allocations go there).
Ctx* thread_ctx_on(int dev, DeviceState** dout, int* status)
{
    DeviceState* d = device_state(dev, status);
    if (!d) return nullptr;
    if (dout) *dout = d;
    // The caller (or a library beside us, e.g. torch) may have made another
    // device current on this thread since our last call: check every time,
    // allocations follow the current device.
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != d->ordinal)
    {
        if (hipSetDevice(d->ordinal) != hipSuccess)
        {
            *status = fail(MI_CRC32C_EHIP, "hipSetDevice(" + std::to_string(d->ordinal) + ")");
            return nullptr;
        }
    }
    if (Ctx* c = t_ctx.c[d->ordinal]) return c;
    auto* c = new Ctx;
    *status = c->open(d->ordinal);
    if (*status != MI_CRC32C_OK)
    {
        c->release();
        delete c;
        return nullptr;
    }
    t_ctx.c[d->ordinal] = c;
    return c;
}

Ctx* thread_ctx(int* status) { return thread_ctx_on(-1, nullptr, status); }

// The device's address of host bytes in mapped pinned memory (hipHostMalloc
// with hipHostMallocMapped, e.g. a durable-log staging arena), else null.
const uint8_t* mapped_device_ptr(const void* p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess)
    {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return static_cast<const uint8_t*>(a.devicePointer) +
           (static_cast<const uint8_t*>(p) - static_cast<const uint8_t*>(a.hostPointer));
}

// The device's address of the span [p, p + n) if ALL of it is in mapped
// pinned memory, read through one contiguous device mapping; else null (the
// batch is then staged by a CPU copy, which only needs the span readable).
// Checking the first byte alone let a span that runs from a mapped buffer
// into pageable memory reach the kernel, which would then read past the
// mapping.  Both ends must be mapped, at device addresses the
// same distance apart, and the span must lie inside ONE device allocation:
// when the runtime reports the allocation's range, that range bounds it;
// when it does not -- hipHostRegister'ed memory, for which ROCm 7.2 reports
// the size with a null base (tools/zc_probe.py:
// profiles/r04_zero_copy_pointer_probe.txt) -- two registered regions with a
// pageable gap between them would pass the two-end check, so every page of
// the span is checked instead.
const uint8_t* mapped_span_device_ptr(const uint8_t* p, uint64_t n)
{
    const uint8_t* d0 = mapped_device_ptr(p);
    if (!d0 || n <= 1) return d0;
    const uint8_t* d1 = mapped_device_ptr(p + (n - 1));
    if (!d1 || d1 < d0 || uint64_t(d1 - d0) != n - 1) return nullptr;
    hipDeviceptr_t pbase = nullptr;
    size_t psize = 0;
    if (hipMemGetAddressRange(&pbase, &psize, const_cast<uint8_t*>(d0)) == hipSuccess && pbase)
    {
        const uint8_t* b = static_cast<const uint8_t*>(pbase);
        return d0 < b || uint64_t(d1 - b) >= psize ? nullptr : d0;
    }
    (void)hipGetLastError();
    // no allocation range: every page between the two ends, mapped at the
    // same distance.  One runtime query per page, so the walk is capped
    // (sparse records across a multi-GiB registered buffer cost
    // hundreds of thousands of queries per batch); a longer span is staged
    // by a CPU copy, which is correct, only slower.
    constexpr uint64_t kPage = 4096;
    constexpr uint64_t kWalkMaxBytes = 2 * kDirectMaxBytes + (uint64_t(64) << 20);  // a 64 MiB segment
    if (n > kWalkMaxBytes) return nullptr;
    const uintptr_t first = (reinterpret_cast<uintptr_t>(p) | (kPage - 1)) + 1;
    for (uintptr_t q = first; q < reinterpret_cast<uintptr_t>(p) + n; q += kPage)
    {
        const uint8_t* dq = mapped_device_ptr(reinterpret_cast<const uint8_t*>(q));
        if (dq != d0 + (q - reinterpret_cast<uintptr_t>(p))) return nullptr;
    }
    return d0;
}

// All of [p, p + n) is pinned host memory of one mapping, so a copy engine
// may read it in place (pinned-but-unmapped spans take the CPU copy: correct,
// only slower).
bool is_pinned_span(const void* p, uint64_t n)
{
    return mapped_span_device_ptr(static_cast<const uint8_t*>(p), n) != nullptr;
}

uint32_t apply_zeros(const DeviceState* d, uint32_t s, uint64_t n)
{
    for (int k = 0; n && k < 64; ++k, n >>= 1)
        if (n & 1u) s = d->pow2_ops[k].apply(s);
    return s;
}

// MI_CRC32C_VARPATH=pieces|sorted: the variable-length path for batches the
// direct kernel does not take.  Default (round 4): the sorted path whenever
// the batch's total bytes are known, its pieces sized by sorted_piece_log2
// (with 4-16 KiB pieces it beats the piece path at every size: 1 MiB 0.029
// against 0.056 ms, 64 MiB 0.038 against 0.138, 512 MiB 0.119 against
// 0.186); the piece path when the total is not given (its plan reads the
// item count back).  "pieces" forces the piece path (tests), "sorted" is the
// default made explicit.
int varpath_forced()
{
    // read per batch (not cached) so that a test can switch paths in-process
    const char* e = std::getenv("MI_CRC32C_VARPATH");
    if (e && !std::strcmp(e, "pieces")) return 1;
    if (e && !std::strcmp(e, "sorted")) return 2;
    if (e && !std::strcmp(e, "window")) return 3;
    return 0;
}

// The window path (one launch, crc32c_kernels.hip "window path") takes device
// batches of at most kWinMaxCount records and kWinMaxBytes bytes (total
// given); MI_CRC32C_VARPATH=window forces it up to kWinMaxCount records,
// =sorted / =pieces never.  MI_CRC32C_WIN_MAX_BYTES overrides the size bound
// (probes; read per batch), MI_CRC32C_WIN_MAX_COUNT the record bound (up to
// kWinMaxCountBig).  configs[2] records cut to 16 / 20 / 24 / 28 MiB (3811 /
// 4727 / 5687 / 6513 records): 15.9 / 16.8 / 24.3 / 26.5 us against the
// sorted path's 24.7 / 25.4 / 25.7 / 26.3 (profiles/r05_window_block768.txt).
constexpr uint64_t kWinMaxBytes = 26ull << 20;
bool window_path(uint64_t count, uint64_t total_bytes)
{
    const int f = varpath_forced();
    uint64_t maxc = kWinMaxCount;  // MI_CRC32C_WIN_MAX_COUNT (probes), up to kWinMaxCountBig
    if (const char* e = std::getenv("MI_CRC32C_WIN_MAX_COUNT"))
        maxc = std::min<uint64_t>(kWinMaxCountBig, std::strtoull(e, nullptr, 10));
    if (!total_bytes || count > maxc || f == 1 || f == 2) return false;
    if (f == 3) return true;
    uint64_t cap = kWinMaxBytes;
    if (const char* e = std::getenv("MI_CRC32C_WIN_MAX_BYTES")) cap = std::strtoull(e, nullptr, 10);
    return total_bytes <= cap;
}

// A device buffer of at least `bytes` whose new allocations are zeroed (on the
// stream, before any later work on it).
int reserve_zeroed(DevBuf& b, size_t bytes, hipStream_t stream)
{
    if (bytes <= b.cap) return MI_CRC32C_OK;
    int st;
    if ((st = b.reserve(bytes))) return st;
    HIP_TRY(hipMemsetAsync(b.p, 0, b.cap, stream));
    return MI_CRC32C_OK;
}

// Piece size of the sorted path by batch size.  A team hashes one item (a
// whole record, or a piece of a longer one) serially, a few rows in flight,
// so the largest item bounds a small batch: 64 KiB pieces made every batch
// of 1-512 MiB take 0.13-0.19 ms.  Smaller pieces cost a fold and a combine
// each, which the full configs[2] batch pays for.  Measured on the final
// round-4 kernel (tools/mid_probe.py, configs[2] records cut to size, ms per
// device batch; profiles/r04_sorted_piece_sweep.txt, last session):
//   batch     1 MiB  16 MiB  64 MiB  256 MiB  512 MiB
//   2 KiB     .020   .024    .034    .071     .126
//   4 KiB     .023   .026    .031    .067     .111
//   8 KiB     .029   .030    .034    .065     .110
//   16 KiB    .041   .043    .045    .064     .107
// and earlier (64 KiB pieces, round-3 kernel): 1 GiB .250, 2 GiB .392
// against .209/.378 at 16 KiB; the full configs[2] 4.9 GB is fastest with
// 64 KiB pieces (.813 against .853 at 16 KiB).
// (4 against 2, ms per device batch: 1 MiB .027/.029, 16 MiB .031/.034,
// 256 MiB .072/.074, 1 GiB .207/.218, 2 GiB .391/.395;
// profiles/r04_sorted_ring_sweep.txt)
// Re-measured on the round-5 kernel (4-row ring, us per batch;
// profiles/r05_sorted_piece_sweep_recheck.txt):
//   batch     32 MiB  64 MiB  96 MiB  128 MiB  160 MiB  192 MiB  256 MiB
//   2 KiB     27.3    35.5    41.8    50.6     57.0     63.4
//   4 KiB     27.4    31.5    37.6    45.9     52.6     58.9
//   8 KiB     31.5    34.6    37.9    41.1     47.3     53.0     66.0
//   16 KiB    43.0    43.8    46.5    46.1     48.1     53.1     63.6
// so 8 KiB pieces from 112 MiB (128 MiB: 41.1 against 45.9) to 224 MiB.
// And above (us per batch, 16 / 32 / 64 KiB pieces with the 4- or 2-row ring):
//   batch     512 MiB          1 GiB            2 GiB            3 GiB
//   16 KiB    107.9 / 112.7    191.2 / 198.6    366.3 / 366.3    551.4 / 543.0
//   32 KiB    106.9 / 127.4    192.2 / 199.0    359.9 / 354.4    538.0 / 522.7
//   64 KiB    124.8 / 181.1    196.6 / 237.8    354.9 / 374.6    534.0 / 517.9
// so 32 KiB pieces with the 2-row ring from 1.5 GiB to 3 GiB.
constexpr int kSortRingSmall = 4;

uint32_t sorted_piece_log2(uint64_t total_bytes)
{
    if (total_bytes < (uint64_t(32) << 20)) return 11;
    if (total_bytes < (uint64_t(112) << 20)) return 12;
    if (total_bytes < (uint64_t(224) << 20)) return 13;
    if (total_bytes < (uint64_t(3) << 29)) return 14;
    if (total_bytes < (uint64_t(3) << 30)) return 15;
    return kSortPieceLog2;
}

// Rows in flight per wave in the sorted kernel's hash loop: 32 and 64 KiB
// pieces (batches from 1.5 GiB, the full configs[2] batch; HBM-bound) take
// the 2-row ring, smaller pieces (where a wave has a group or two) a deeper one.
// MI_CRC32C_SORT_RING=2|4 overrides (A/B, tests).
int sorted_ring(uint32_t plog)
{
    if (const char* e = std::getenv("MI_CRC32C_SORT_RING"))
    {
        const int r = std::atoi(e);
        if (r == 2 || r == 4) return r;
    }
    return plog < 15 ? kSortRingSmall : 2;
}

// Records spanning at most this many 128-B rows are hashed one per lane
// (lane items); MI_CRC32C_SORT_LANE_ROWS=0..3
// overrides (0: every item takes a team).
uint32_t sorted_lane_rows()
{
    if (const char* e = std::getenv("MI_CRC32C_SORT_LANE_ROWS"))
        return uint32_t(std::max(0, std::min(int(kSortLaneRowsMax), std::atoi(e))));
    return kSortLaneRows;
}

// The one-launch sorted form (a grid barrier, crc32c_kernels.hip
// sorted_fused_costs) needs every workgroup resident: one per CU, so at most
// `cus` of them, and no second barrier launch sharing the CUs -- so only
// while this is the process's one context that runs the sorted path on the
// device.  Measured slower than the two launches (round 5, interleaved on one
// box: configs[2] 0.7708-0.7732 ms against 0.7678-0.7690; 16 / 64 / 256 MiB
// 26.7 / 34.1 / 67.7 us against 24.9 / 31.5 / 63.6; profiles/r05_fused_ab.txt):
// the barrier's fan-in of 256 agent-scope adds on one word plus the
// write-through drain cost more than the cost kernel's launch.  Off unless
// MI_CRC32C_SORT_FUSED=1 (A/B, tests; read per batch).
bool fused_ok(DeviceState* d, const Ctx* c, int grid)
{
    if (c->force_unfused) return false;
    const char* e = std::getenv("MI_CRC32C_SORT_FUSED");
    if (!e || std::strcmp(e, "1")) return false;
    return grid <= d->cus && d->sorted_users.load() == 1;
}

// The sorted path (crc32c_kernels.hip, "sorted path"): whole records per team.
int run_sorted(DeviceState* d, Ctx* c, const void* base, const uint64_t* off, const uint32_t* len,
               const uint32_t* inits, size_t count, uint64_t total_bytes, uint32_t* out)
{
    uint32_t plog = sorted_piece_log2(total_bytes);
    if (const char* e = std::getenv("MI_CRC32C_SORT_PIECE_LOG2"))
        plog = uint32_t(std::max(9, std::min(int(kSortPieceLog2), std::atoi(e))));
    // MI_CRC32C_SORTED_GRID=k: k workgroups instead of one per CU (tests: one
    // workgroup puts every item of a small batch into one sorted list)
    int grid = d->cus;
    if (const char* e = std::getenv("MI_CRC32C_SORTED_GRID"))
        grid = std::max(1, std::min(8 * grid, std::atoi(e)));
    const uint64_t cap = sorted_item_cap(count, total_bytes, plog, grid);
    int st;
    if ((st = c->srt_cost.reserve(uint64_t(sorted_blocks(count)) * 8)) ||
        (st = reserve_zeroed(c->srt_ctrl, 64 * 4, c->stream)) ||
        (st = c->srt_items.reserve(cap * 20)))
        return st;
    // descriptors, then the fold values by slot
    uint8_t* const ib = c->srt_items.as<uint8_t>();
    if (!c->sorted_users)
    {
        c->sorted_users = &d->sorted_users;
        c->sorted_users->fetch_add(1);
    }
    SortedWorkspace ws{c->srt_cost.as<uint64_t>(), c->srt_ctrl.as<uint32_t>(),
                       reinterpret_cast<uint4*>(ib), cap,
                       reinterpret_cast<uint32_t*>(ib + cap * 16), plog, sorted_ring(plog),
                       sorted_lane_rows(), fused_ok(d, c, grid) ? 1 : 0, c->bar_base};
    // MI_CRC32C_SORT_BARRIER_SKEW=1 (tests): the kernel waits for one arrival
    // more than the grid has, so every workgroup's wait times out
    const char* skew = std::getenv("MI_CRC32C_SORT_BARRIER_SKEW");
    if (ws.fused && skew && !std::strcmp(skew, "1")) ws.bar_base += 1;
    HIP_TRY(launch_sorted(base, off, len, inits, count, ws, out, d->d_tables, d->d_pow2, grid,
                          c->stream));
    c->bar_tag = ws.fused ? ws.bar_base + uint32_t(grid) + 1u : 0u;
    if (ws.fused) c->bar_base += uint32_t(grid);
    c->sorted_ctrl = ws.ctrl;
    mi_host::note_sorted_batch(ws.fused != 0);
    return MI_CRC32C_OK;
}

int run_window(DeviceState* d, Ctx* c, const void* base, const uint64_t* off, const uint32_t* len,
               const uint32_t* inits, size_t count, uint64_t total_bytes, uint32_t* out)
{
    int st;
    if ((st = reserve_zeroed(c->win_acc, count * 16, c->stream)) ||
        (st = reserve_zeroed(c->srt_ctrl, 64 * 4, c->stream)))
        return st;
    uint64_t* acc64 = c->win_acc.as<uint64_t>();
    uint32_t* acc = reinterpret_cast<uint32_t*>(acc64 + count);
    // MI_CRC32C_WIN_BLOCK=64|256|768, MI_CRC32C_WIN_ROWS=4|8|16: the workgroup and
    // the window (A/B, tests; default by count and size)
    uint32_t block = 0, rows = 0;
    if (const char* e = std::getenv("MI_CRC32C_WIN_BLOCK")) block = std::atoi(e) == 64 ? 64u : std::atoi(e) == int(kWinBlockBig) ? kWinBlockBig : 256u;
    if (const char* e = std::getenv("MI_CRC32C_WIN_ROWS"))
        rows = std::atoi(e) == 4 ? 4u : std::atoi(e) == 8 ? 8u : 16u;
    HIP_TRY(launch_window(base, off, len, inits, count, total_bytes, out, acc64, acc, acc + count,
                          d->d_tables, d->d_pow2, c->srt_ctrl.as<uint32_t>(), 8 * d->cus, block, rows,
                          c->stream));
    // more than 2^31 windows (an understated hint) set ctrl[1] and
    // the sticky ctrl[2]; the batch is then checked as a sorted batch is
    // (a synchronous one recomputed on the plan path, an asynchronous one
    // reported at the next stream sync)
    c->sorted_ctrl = c->srt_ctrl.as<uint32_t>();
    c->bar_tag = 0;
    mi_host::note_window_batch();
    return MI_CRC32C_OK;
}

// MI_CRC32C_ZERO_COPY=0: host batches in mapped pinned memory are staged by
// copy commands instead of read in place (A/B and tests; read per batch)
bool zero_copy_disabled()
{
    const char* e = std::getenv("MI_CRC32C_ZERO_COPY");
    return e && !std::strcmp(e, "0");
}

// MI_CRC32C_DIRECT_LITE=0 / 1: the direct kernel's LDS-free form never /
// always (tests cover both; default: by size, kLiteMaxBytes).  Read per batch.
int direct_lite_mode()
{
    const char* e = std::getenv("MI_CRC32C_DIRECT_LITE");
    if (!e || !*e) return -1;
    return std::strcmp(e, "0") ? 1 : 0;
}

// MI_CRC32C_PLAN_SCAN=1: plans always take the separate scan pass (which
// only plans of more than 16M records need), so tests exercise both forms.
bool plan_scan_forced()
{
    static const bool v = [] {
        const char* e = std::getenv("MI_CRC32C_PLAN_SCAN");
        return e && !std::strcmp(e, "1");
    }();
    return v;
}

// ---- the variable-length pipeline on device-resident arrays -------------
// All pointers device pointers; enqueued on c->stream.  `total_bytes` bounds
// the plan size (0 = unknown -> one read-back).
int run_var(DeviceState* d, Ctx* c, const void* base, const uint64_t* off, const uint32_t* len,
            const uint32_t* inits, size_t count, uint64_t total_bytes, uint32_t* out,
            uint64_t max_len = UINT64_MAX)  // longest record if known (host batches)
{
    if (count == 0) return MI_CRC32C_OK;
    if (count >= (1ull << 31)) return fail(MI_CRC32C_ERANGE, "count >= 2^31 records");
    // items pack addresses in 41 bits (crc32c_kernels.h: Item); user-space and
    // GPU virtual addresses are below 2^47
    if (uintptr_t(base) >= (kItemMaxAddr >> 1)) return fail(MI_CRC32C_ERANGE, "address above 2^47");
    // small batches of short records: one launch, no plan (a durable-log
    // flush, one host call); a team hashes a record's rows serially, so only
    // when the longest record is known to be short
    if (max_len <= kDirectMaxRecord && total_bytes <= kDirectMaxBytes && count <= kDirectMaxCount)
    {
        HIP_TRY(launch_direct(base, off, len, inits, count, total_bytes, out, d->d_tables,
                              d->d_pow2, d->cus, c->stream, nullptr, direct_lite_mode()));
        return MI_CRC32C_OK;
    }
    if (window_path(count, total_bytes))
        return run_window(d, c, base, off, len, inits, count, total_bytes, out);
    if (total_bytes && count < kSortedMaxCount && varpath_forced() != 1)
        return run_sorted(d, c, base, off, len, inits, count, total_bytes, out);
    const uint32_t nb = var_plan_blocks(count);
    int st;
    if ((st = c->blk.reserve((kBins * size_t(nb) + kPlanHdrWords) * 4)) ||
        (st = c->first_pos.reserve(count * 4)) || (st = c->int_pos.reserve(count * 4)) ||
        (st = c->last_pos.reserve(count * 4)) || (st = c->longs.reserve(count * 4)))
        return st;
    uint64_t cap = total_bytes ? total_bytes / kChunk + 2 * uint64_t(count) + 1
                               : std::max<uint64_t>(c->items.cap / sizeof(Item), 2 * count + 1);
    for (int attempt = 0; attempt < 2; ++attempt)
    {
        if (cap >= (1ull << 32)) return fail(MI_CRC32C_ERANGE, "plan exceeds 2^32 chunks");
        if ((st = c->items.reserve(cap * sizeof(Item))) || (st = c->partial.reserve(cap * 4)))
            return st;
        cap = std::min<uint64_t>(c->items.cap / sizeof(Item), c->partial.cap / 4);
        VarWorkspace ws{c->blk.as<uint32_t>(),       c->items.as<Item>(),
                        c->partial.as<uint32_t>(),   c->first_pos.as<uint32_t>(),
                        c->int_pos.as<uint32_t>(),   c->last_pos.as<uint32_t>(),
                        c->longs.as<uint32_t>(),     cap};
        HIP_TRY(launch_var_plan(base, off, len, count, ws, c->stream, plan_scan_forced()));
        if (!total_bytes)
        {
            uint32_t* h = c->pin_small.as<uint32_t>();
            HIP_TRY(hipMemcpyAsync(h, plan_hdr(c->blk.as<uint32_t>(), nb) + kPlanHdrTotal, 4,
                                   hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            if (*h > cap)
            {
                cap = *h;
                continue;
            }
        }
        const uint64_t want_grid = (cap + (kBlock / kTeam) - 1) / (kBlock / kTeam);
        const int grid = int(std::min<uint64_t>(uint64_t(d->cus), std::max<uint64_t>(want_grid, 1)));
        if (total_bytes)
        {
            c->plan_total = plan_hdr(c->blk.as<uint32_t>(), nb) + kPlanHdrTotal;
            c->plan_cap = cap;
        }
        HIP_TRY(launch_var_chunks(inits, count, ws, d->d_tables, grid, c->stream));
        HIP_TRY(launch_var_finalize(base, off, len, inits, count, ws, out, d->d_tables, d->d_pow2,
                                    c->stream));
        return MI_CRC32C_OK;
    }
    return fail(MI_CRC32C_EHIP, "plan size did not converge");
}

bool fixed_fast_ok(const void* base, uint64_t stride, uint64_t length)
{
    return (uintptr_t(base) % 16) == 0 && (stride % 16) == 0 && (length % 16) == 0 &&
           length >= 16 && length <= (1ull << 30) && stride >= length;
}

int run_fixed(DeviceState* d, Ctx* c, const void* base, uint64_t stride, uint64_t length,
              const uint32_t* inits, size_t count, uint32_t* out)
{
    if (count == 0) return MI_CRC32C_OK;
    if (fixed_fast_ok(base, stride, length))
    {
        HIP_TRY(launch_fixed(base, stride, uint32_t(length), inits, count, out, d->d_tables,
                             d->cus, c->stream));
        return MI_CRC32C_OK;
    }
    int st;
    if ((st = c->off.reserve(count * 8)) || (st = c->len.reserve(count * 4))) return st;
    HIP_TRY(launch_make_fixed_records(c->off.as<uint64_t>(), c->len.as<uint32_t>(), count, stride,
                                      uint32_t(length), c->stream));
    return run_var(d, c, base, c->off.as<uint64_t>(), c->len.as<uint32_t>(), inits, count,
                   length * count, out);
}

int finish(Ctx* c, unsigned flags)
{
    if ((flags & MI_CRC32C_DEVICE) && (flags & MI_CRC32C_ASYNC)) return MI_CRC32C_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MI_CRC32C_OK;
}

}  // namespace

// ==========================================================================
extern "C" {

int mi_crc32c_init(int device) { return init_device(device); }

int mi_crc32c_device_pci_bus_id(int device, char* buf, int len)
{
    if (!buf || len < 13) return fail(MI_CRC32C_EINVAL, "buffer too small for a PCI bus id");
    HIP_TRY(hipDeviceGetPCIBusId(buf, len, device));
    return MI_CRC32C_OK;
}

void* mi_crc32c_stream(void)
{
    int st = 0;
    Ctx* c = thread_ctx(&st);
    return c ? static_cast<void*>(c->stream) : nullptr;
}

int mi_crc32c_stream_sync(void)
{
    int st = 0;
    Ctx* c = thread_ctx(&st);
    if (!c) return st;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->async_sorted_unchecked || c->async_overflow_latched)
    {
        // an asynchronous sorted (or window) batch whose
        // total_bytes hint understated its records left out[] incomplete (no
        // access went out of bounds); the kernel's sticky word says so, read
        // and cleared here (or latched by a synchronous batch since)
        uint32_t* w = c->pin_small.as<uint32_t>() + 2;
        *w = 0;
        if (c->async_sorted_unchecked)
        {
            HIP_TRY(hipMemcpyAsync(w, c->srt_ctrl.as<uint32_t>() + 2, 4, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
        }
        const bool latched = c->async_overflow_latched;
        c->async_sorted_unchecked = c->async_overflow_latched = false;
        if (*w || latched)
        {
            HIP_TRY(hipMemsetAsync(c->srt_ctrl.as<uint32_t>() + 2, 0, 4, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            mi_host::note_hint_overflow();
            return fail(MI_CRC32C_EINVAL,
                        "an asynchronous sorted batch left out[] incomplete: its total_bytes "
                        "hint understated the sum of its lengths, or its one-launch grid barrier "
                        "timed out (another barrier launch held CUs)");
        }
    }
    return MI_CRC32C_OK;
}

}  // extern "C"

namespace mi_eng {

// The usable (gfx950) devices, probed once per process: every multi-device
// call (each durable-log flush) asks, and a property query per device per
// call cost microseconds.
int usable_devices(int* ordinals, int max)
{
    if (fault_mode() == kFaultInit) return 0;
    struct Found
    {
        int n = 0;
        int ord[kMaxDevices];
    };
    static const Found found = [] {
        Found f;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess)
        {
            (void)hipGetLastError();
            return f;
        }
        for (int i = 0; i < n && i < kMaxDevices; ++i)
            if (is_gfx950(i)) f.ord[f.n++] = i;
        return f;
    }();
    const int k = std::min(found.n, max);
    for (int i = 0; i < k; ++i) ordinals[i] = found.ord[i];
    return k;
}

int batch(int dev, const void* base, const uint64_t* offsets, const uint32_t* lengths,
          const uint32_t* inits, size_t count, uint64_t total_bytes, uint32_t* out,
          unsigned flags)
{
    if (count == 0) return MI_CRC32C_OK;
    if (!offsets || !lengths || !out) return fail(MI_CRC32C_EINVAL, "null array with count > 0");
    if (fault_mode() == kFaultCompute)
        return fail(MI_CRC32C_EHIP, "fault injected (MI_CRC32C_FAULT=compute)");
    int st = 0;
    DeviceState* d = nullptr;
    Ctx* c = thread_ctx_on(dev, &d, &st);
    if (!c) return st;
    if (flags & MI_CRC32C_DEVICE)
    {
        // before a synchronous batch, the sticky word as the
        // unchecked asynchronous batches left it (pin_small word 8), latched
        // once this batch's sync has read it; the word is then free for this
        // batch's own overflow, which is recovered here
        const bool pre = !(flags & MI_CRC32C_ASYNC) && c->async_sorted_unchecked;
        uint32_t* pre_w = c->pin_small.as<uint32_t>() + 8;
        if (pre)
            HIP_TRY(hipMemcpyAsync(pre_w, c->srt_ctrl.as<uint32_t>() + 2, 4, hipMemcpyDeviceToHost,
                                   c->stream));
        auto latch = [&]() {
            if (!pre) return MI_CRC32C_OK;
            c->async_overflow_latched |= *pre_w != 0;
            c->async_sorted_unchecked = false;
            HIP_TRY(hipMemsetAsync(c->srt_ctrl.as<uint32_t>() + 2, 0, 4, c->stream));
            return MI_CRC32C_OK;
        };
        c->sorted_ctrl = c->plan_total = nullptr;
        if ((st = run_var(d, c, base, offsets, lengths, inits, count, total_bytes, out)))
            return st;
        if (flags & MI_CRC32C_ASYNC) c->async_sorted_unchecked |= c->sorted_ctrl != nullptr;
        if ((flags & MI_CRC32C_ASYNC) || (!c->sorted_ctrl && !c->plan_total))
        {
            if ((st = finish(c, flags))) return st;
            return latch();
        }
        // Synchronous batch sized by the caller's hint: if the hint understated
        // the sum of lengths, the workspace overflowed and out[] is incomplete
        // (sorted path: a workgroup found no room for its descriptors; piece
        // path: the plan exceeded its capacity).  Then hash the batch again
        // with the plan size read back (total_bytes = 0): exact, slower.
        uint32_t* flag = c->pin_small.as<uint32_t>() + 4;  // ctrl[0..3] / the plan total
        HIP_TRY(hipMemcpyAsync(flag, c->sorted_ctrl ? c->sorted_ctrl : c->plan_total,
                               c->sorted_ctrl ? 16 : 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if ((st = latch())) return st;
        // the one-launch form's barrier timed out (ctrl[3] holds this launch's
        // tag, bar_base after it + 1): hash the batch again with two launches
        if (c->sorted_ctrl && c->bar_tag && flag[3] == c->bar_tag)
        {
            // ctrl[3], and this batch's sticky ctrl[2] (an unchecked
            // asynchronous batch's state was latched above)
            HIP_TRY(hipMemsetAsync(c->sorted_ctrl + 2, 0, 8, c->stream));
            c->force_unfused = true;
            if ((st = run_var(d, c, base, offsets, lengths, inits, count, total_bytes, out))) return st;
            c->force_unfused = false;
            HIP_TRY(hipMemcpyAsync(flag, c->sorted_ctrl, 16, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
        }
        const bool overflow = c->sorted_ctrl ? flag[1] != 0 : flag[0] > c->plan_cap;
        if (!overflow) return MI_CRC32C_OK;
        // the sticky word (ctrl[2]) is for asynchronous batches: this one is
        // recovered here.  The earlier asynchronous batches' state was latched
        // before this batch ran, so the word is cleared.
        if (c->sorted_ctrl) HIP_TRY(hipMemsetAsync(c->sorted_ctrl + 2, 0, 4, c->stream));
        if ((st = run_var(d, c, base, offsets, lengths, inits, count, 0, out))) return st;
        return finish(c, flags);
    }
    // Host batch: stage the spanned bytes, rebased offsets, lengths, inits.
    uint64_t lo = UINT64_MAX, hi = 0, total = 0, maxlen = 0;
    for (size_t i = 0; i < count; ++i)
    {
        if (offsets[i] > UINT64_MAX - lengths[i])
            return fail(MI_CRC32C_EINVAL, "record end overflows 64 bits");
        if (lengths[i] == 0) continue;
        lo = std::min<uint64_t>(lo, offsets[i]);
        hi = std::max<uint64_t>(hi, offsets[i] + lengths[i]);
        total += lengths[i];
        maxlen = std::max<uint64_t>(maxlen, lengths[i]);
    }
    if (lo == UINT64_MAX) lo = hi = 0;
    if (hi > lo && !base) return fail(MI_CRC32C_EINVAL, "null base");
    const uint64_t maxlen_arg = (flags & MI_CRC32C_PLANNED) ? UINT64_MAX : maxlen;
    // Bytes already in mapped pinned memory (a durable-log flush: the staging
    // arena is mapped) and a batch the one-launch direct kernel takes: the
    // kernel reads the records where they lie, over PCIe (zero-copy), and
    // the offsets, lengths and CRCs through mapped pinned staging too -- one
    // launch and one sync, no copy command.  (Two copy commands around the
    // kernel cost ~40 us more per 550 KB flush: DESIGN.md section 7.)
    if (hi > lo && maxlen_arg <= kDirectMaxRecord && total <= kDirectMaxBytes &&
        count <= kDirectMaxCount && !zero_copy_disabled())
    {
        if (const uint8_t* zsrc = mapped_span_device_ptr(static_cast<const uint8_t*>(base) + lo,
                                                         hi - lo))
        {
            const uint64_t meta_bytes = uint64_t(count) * (inits ? 16 : 12);
            if ((st = c->pin_stage.reserve(meta_bytes + 16)) || (st = c->pin_out.reserve(count * 4)))
                return st;
            if (c->pin_stage.dev && c->pin_out.dev)
            {
                uint8_t* hp = c->pin_stage.as<uint8_t>();
                uint64_t* ho = reinterpret_cast<uint64_t*>(hp);
                for (size_t i = 0; i < count; ++i) ho[i] = lengths[i] ? offsets[i] - lo : 0;
                std::memcpy(hp + count * 8, lengths, count * 4);
                if (inits) std::memcpy(hp + count * 12, inits, count * 4);
                const uint8_t* sp = static_cast<const uint8_t*>(c->pin_stage.dev);
                DoneSignal sig;
                const bool signalled = c->next_signal(&sig, total);
                HIP_TRY(launch_direct(zsrc, reinterpret_cast<const uint64_t*>(sp),
                                      reinterpret_cast<const uint32_t*>(sp + count * 8),
                                      inits ? reinterpret_cast<const uint32_t*>(sp + count * 12)
                                            : nullptr,
                                      count, total, static_cast<uint32_t*>(c->pin_out.dev),
                                      d->d_tables, d->d_pow2, d->cus, c->stream,
                                      signalled ? &sig : nullptr, direct_lite_mode()));
                if ((st = c->wait_direct(signalled))) return st;
                std::memcpy(out, c->pin_out.p, count * 4);
                mi_host::note_zero_copy_batch();
                return MI_CRC32C_OK;
            }
        }
    }
    // Small batches (a consus::crc32c call, a durable-log flush): offsets,
    // lengths, inits -- and the bytes, unless they already sit in pinned
    // memory -- packed into one pinned staging buffer and moved with ONE
    // copy; the CRCs come back into pinned memory.  Each pageable
    // hipMemcpyAsync costs a staging round trip of its own.
    const uint64_t meta = uint64_t(count) * (inits ? 16 : 12);
    // bytes already pinned are DMA'd in place only when large: below ~512 KiB a
    // CPU copy into the packed buffer beats a second copy command (measured:
    // 400 frames, 227 KB: 50 us packed vs 54 us with the bytes DMA'd in place)
    const bool src_pinned = hi - lo > kPackInPlace &&
                            is_pinned_span(static_cast<const uint8_t*>(base) + lo, hi - lo);
    const uint64_t data_at = (meta + 127) & ~uint64_t(127);
    const uint64_t packed = data_at + (src_pinned ? 0 : hi - lo);
    if (packed <= kPackMax)
    {
        if ((st = c->pin_stage.reserve(packed + 16)) || (st = c->pin_out.reserve(count * 4)) ||
            (st = c->off.reserve(packed + 16)) || (st = c->out.reserve(count * 4)) ||
            (src_pinned && (st = c->data.reserve(hi - lo + 16))))
            return st;
        uint8_t* hp = c->pin_stage.as<uint8_t>();
        uint64_t* ho = reinterpret_cast<uint64_t*>(hp);
        for (size_t i = 0; i < count; ++i) ho[i] = lengths[i] ? offsets[i] - lo : 0;
        std::memcpy(hp + count * 8, lengths, count * 4);
        if (inits) std::memcpy(hp + count * 12, inits, count * 4);
        if (!src_pinned && hi > lo)
            std::memcpy(hp + data_at, static_cast<const uint8_t*>(base) + lo, hi - lo);
        // Tiny batches of short records (a single consus::crc32c call): the
        // direct kernel reads the packed inputs and writes the CRCs in mapped
        // pinned memory, no copy commands at all (one launch + one sync).
        if (packed <= kZeroCopyMax && !src_pinned && maxlen_arg <= kDirectMaxRecord &&
            c->pin_stage.dev && c->pin_out.dev)
        {
            const uint8_t* sp = static_cast<const uint8_t*>(c->pin_stage.dev);
            DoneSignal sig;
            const bool signalled = c->next_signal(&sig, total);
            HIP_TRY(launch_direct(sp + data_at, reinterpret_cast<const uint64_t*>(sp),
                                  reinterpret_cast<const uint32_t*>(sp + count * 8),
                                  inits ? reinterpret_cast<const uint32_t*>(sp + count * 12)
                                        : nullptr,
                                  count, total, static_cast<uint32_t*>(c->pin_out.dev),
                                  d->d_tables, d->d_pow2, d->cus, c->stream,
                                  signalled ? &sig : nullptr, direct_lite_mode()));
            if ((st = c->wait_direct(signalled))) return st;
            std::memcpy(out, c->pin_out.p, count * 4);
            return MI_CRC32C_OK;
        }
        uint8_t* dp = c->off.as<uint8_t>();
        HIP_TRY(hipMemcpyAsync(dp, hp, packed, hipMemcpyHostToDevice, c->stream));
        const uint8_t* dbase = dp + data_at;
        if (src_pinned)
        {
            HIP_TRY(hipMemcpyAsync(c->data.p, static_cast<const uint8_t*>(base) + lo, hi - lo,
                                   hipMemcpyHostToDevice, c->stream));
            dbase = c->data.as<uint8_t>();
        }
        if ((st = run_var(d, c, dbase, reinterpret_cast<const uint64_t*>(dp),
                          reinterpret_cast<const uint32_t*>(dp + count * 8),
                          inits ? reinterpret_cast<const uint32_t*>(dp + count * 12) : nullptr,
                          count, total, c->out.as<uint32_t>(), maxlen_arg)))
            return st;
        HIP_TRY(hipMemcpyAsync(c->pin_out.p, c->out.p, count * 4, hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        std::memcpy(out, c->pin_out.p, count * 4);
        return MI_CRC32C_OK;
    }
    std::vector<uint64_t> reb(count);
    for (size_t i = 0; i < count; ++i) reb[i] = lengths[i] ? offsets[i] - lo : 0;
    if ((st = c->data.reserve(hi - lo + 16)) || (st = c->off.reserve(count * 8)) ||
        (st = c->len.reserve(count * 4)) || (st = c->out.reserve(count * 4)) ||
        (inits && (st = c->inits.reserve(count * 4))))
        return st;
    if (hi > lo)
        HIP_TRY(hipMemcpyAsync(c->data.p, static_cast<const uint8_t*>(base) + lo, hi - lo,
                               hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->off.p, reb.data(), count * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->len.p, lengths, count * 4, hipMemcpyHostToDevice, c->stream));
    if (inits)
        HIP_TRY(hipMemcpyAsync(c->inits.p, inits, count * 4, hipMemcpyHostToDevice, c->stream));
    if ((st = run_var(d, c, c->data.p, c->off.as<uint64_t>(), c->len.as<uint32_t>(),
                      inits ? c->inits.as<uint32_t>() : nullptr, count, total,
                      c->out.as<uint32_t>(), maxlen_arg)))
        return st;
    HIP_TRY(hipMemcpyAsync(out, c->out.p, count * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MI_CRC32C_OK;
}

int batch_fixed(int dev, const void* base, uint64_t stride, uint64_t length,
                const uint32_t* inits, size_t count, uint32_t* out, unsigned flags)
{
    if (count == 0) return MI_CRC32C_OK;
    if (!out || (!base && length)) return fail(MI_CRC32C_EINVAL, "null pointer with count > 0");
    if (length > 0xFFFFFFFFull) return fail(MI_CRC32C_EINVAL, "fixed length >= 4 GiB");
    uint64_t span = 0;  // bytes from the first record's start to the last one's end
    if (length && (__builtin_mul_overflow(uint64_t(count - 1), stride, &span) ||
                   __builtin_add_overflow(span, length, &span)))
        return fail(MI_CRC32C_EINVAL, "batch span overflows 64 bits");
    if (fault_mode() == kFaultCompute)
        return fail(MI_CRC32C_EHIP, "fault injected (MI_CRC32C_FAULT=compute)");
    int st = 0;
    DeviceState* d = nullptr;
    Ctx* c = thread_ctx_on(dev, &d, &st);
    if (!c) return st;
    if (flags & MI_CRC32C_DEVICE)
    {
        if ((st = run_fixed(d, c, base, stride, length, inits, count, out))) return st;
        return finish(c, flags);
    }
    if ((st = c->data.reserve(span + 16)) || (st = c->out.reserve(count * 4)) ||
        (inits && (st = c->inits.reserve(count * 4))))
        return st;
    if (span) HIP_TRY(hipMemcpyAsync(c->data.p, base, span, hipMemcpyHostToDevice, c->stream));
    if (inits)
        HIP_TRY(hipMemcpyAsync(c->inits.p, inits, count * 4, hipMemcpyHostToDevice, c->stream));
    if ((st = run_fixed(d, c, c->data.p, stride, length, inits ? c->inits.as<uint32_t>() : nullptr,
                        count, c->out.as<uint32_t>())))
        return st;
    HIP_TRY(hipMemcpyAsync(out, c->out.p, count * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MI_CRC32C_OK;
}

int buffer(int dev, uint32_t init, const void* data, size_t n, uint32_t* out, unsigned flags)
{
    if (!out) return fail(MI_CRC32C_EINVAL, "null out");
    if (n == 0)
    {
        *out = init;
        return MI_CRC32C_OK;
    }
    if (!data) return fail(MI_CRC32C_EINVAL, "null data");
    if (fault_mode() == kFaultCompute)
        return fail(MI_CRC32C_EHIP, "fault injected (MI_CRC32C_FAULT=compute)");
    int st = 0;
    DeviceState* d = nullptr;
    Ctx* c = thread_ctx_on(dev, &d, &st);
    if (!c) return st;
    // Device buffers of >= kSingleMin bytes (up to 64 GiB): launch_single.
    // Otherwise pieces of <= 16 MiB computed as one batch (one long-path record each,
    // so a 4 GiB buffer keeps 256 workgroups of long_finalize busy) and
    // joined with the combine identity crc(0, A||B) = Z_|B|(crc(0, A)) ^
    // crc(0, B); init goes into piece 0.
    constexpr uint64_t kPiece = 16ull << 20;
    const size_t np = size_t((n + kPiece - 1) / kPiece);
    if (np >= (1ull << 31)) return fail(MI_CRC32C_ERANGE, "buffer too large");
    std::vector<uint64_t> off(np), after(np);
    std::vector<uint32_t> len(np), ini(np, 0), res(np);
    for (size_t i = 0; i < np; ++i)
    {
        off[i] = i * kPiece;
        len[i] = uint32_t(std::min<uint64_t>(kPiece, n - i * kPiece));
        after[i] = n - off[i] - len[i];
    }
    ini[0] = init;
    if ((flags & MI_CRC32C_DEVICE) && n >= kSingleMin)
    {
        // head up to the next 4 KiB boundary (>= 4 bytes, so ~init lands in
        // it), 4 KiB chunks through the fixed-record kernel, tail < 4 KiB
        uint64_t h = (kChunk - uintptr_t(data) % kChunk) % kChunk;
        if (h < 4) h += kChunk;
        const uint64_t m = (n - h) / kChunk;
        const uint32_t t = uint32_t(n - h - m * kChunk);
        if (m + 2 <= (1ull << 24) - (1ull << 14))  // launch_single's limits
        {
            if ((st = c->out.reserve((m + kSingleVals + 1) * 4))) return st;
            uint32_t* crcs = c->out.as<uint32_t>();
            uint32_t* dres = crcs + m + kSingleVals;
            HIP_TRY(launch_single(data, h, m, t, init, d->crc0, crcs, crcs + m, dres,
                                  d->d_tables, d->d_pow2, d->cus, c->stream));
            uint32_t* hr = c->pin_small.as<uint32_t>();
            HIP_TRY(hipMemcpyAsync(hr, dres, 4, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            *out = *hr;
            return MI_CRC32C_OK;
        }
    }
    if (flags & MI_CRC32C_DEVICE)
    {
        DevBuf& d_after = c->data;  // device staging unused on the device path
        if ((st = c->off.reserve(np * 8)) || (st = c->len.reserve(np * 4)) ||
            (st = c->inits.reserve(np * 4)) || (st = c->out.reserve(np * 4 + 4)) ||
            (st = d_after.reserve(np * 8)))
            return st;
        HIP_TRY(hipMemcpyAsync(c->off.p, off.data(), np * 8, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(c->len.p, len.data(), np * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(c->inits.p, ini.data(), np * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(d_after.p, after.data(), np * 8, hipMemcpyHostToDevice, c->stream));
        if ((st = run_var(d, c, data, c->off.as<uint64_t>(), c->len.as<uint32_t>(),
                          c->inits.as<uint32_t>(), np, n, c->out.as<uint32_t>())))
            return st;
        uint32_t* dres = c->out.as<uint32_t>() + np;
        HIP_TRY(launch_chain(c->out.as<uint32_t>(), d_after.as<uint64_t>(), uint32_t(np), dres,
                             d->d_pow2, c->stream));
        uint32_t* h = c->pin_small.as<uint32_t>();
        HIP_TRY(hipMemcpyAsync(h, dres, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        *out = *h;
        return MI_CRC32C_OK;
    }
    if ((st = batch(dev, data, off.data(), len.data(), ini.data(), np, n, res.data(), 0)))
        return st;
    uint32_t acc = 0;
    for (size_t i = 0; i < np; ++i) acc ^= apply_zeros(d, res[i], after[i]);
    *out = acc;
    return MI_CRC32C_OK;
}

}  // namespace mi_eng

extern "C" {

uint32_t mi_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    static const Op32* ops = [] {
        static Op32 o[64];
        Op32 p = Op32::zero_byte();
        for (int k = 0; k < 64; ++k)
        {
            o[k] = p;
            p = p.then(p);
        }
        return o;
    }();
    uint32_t s = crc_a;
    for (int k = 0; len_b && k < 64; ++k, len_b >>= 1)
        if (len_b & 1u) s = ops[k].apply(s);
    return s ^ crc_b;
}

int mi_crc32c_combine_batch(const uint32_t* crc_a, const uint32_t* crc_b, const uint64_t* len_b,
                            size_t count, uint32_t* out, unsigned flags)
{
    if (count == 0) return MI_CRC32C_OK;
    if (!crc_a || !crc_b || !len_b || !out) return fail(MI_CRC32C_EINVAL, "null array");
    int st = 0;
    DeviceState* d = nullptr;
    Ctx* c = thread_ctx_on(-1, &d, &st);
    if (!c) return st;
    if (flags & MI_CRC32C_DEVICE)
    {
        HIP_TRY(launch_combine(crc_a, crc_b, len_b, count, out, d->d_pow2, c->stream));
        return finish(c, flags);
    }
    if ((st = c->inits.reserve(count * 4)) || (st = c->out.reserve(count * 4)) ||
        (st = c->off.reserve(count * 8)) || (st = c->len.reserve(count * 4)))
        return st;
    HIP_TRY(hipMemcpyAsync(c->inits.p, crc_a, count * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->len.p, crc_b, count * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->off.p, len_b, count * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(launch_combine(c->inits.as<uint32_t>(), c->len.as<uint32_t>(), c->off.as<uint64_t>(),
                           count, c->out.as<uint32_t>(), d->d_pow2, c->stream));
    HIP_TRY(hipMemcpyAsync(out, c->out.p, count * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MI_CRC32C_OK;
}

// ---- streaming pipeline ----------------------------------------------------
}  // extern "C"

struct mi_crc32c_pipeline
{
    struct Slot
    {
        Ctx ctx;
        PinBuf seg, meta, res;   // pinned: segment bytes, offsets+lengths+inits, crcs
        DevBuf dseg, dmeta;      // device: segment bytes, offsets+lengths+inits
        uint64_t ticket = 0;     // ticket in flight (0 = none)
        uint32_t* host_out = nullptr;
        size_t count = 0;
    };
    std::vector<Slot> slots;
    DeviceState* dev = nullptr;  // the device the slots' streams and buffers live on
    size_t max_bytes = 0, max_records = 0;
    uint64_t next_ticket = 1;
    std::mutex mu;
};

namespace {

int slot_complete(mi_crc32c_pipeline::Slot& s)
{
    if (!s.ticket) return MI_CRC32C_OK;
    HIP_TRY(hipEventSynchronize(s.ctx.done));
    if (s.host_out && s.count) std::memcpy(s.host_out, s.res.p, s.count * 4);
    s.ticket = 0;
    s.host_out = nullptr;
    return MI_CRC32C_OK;
}


}  // namespace

extern "C" {

int mi_crc32c_pipeline_create(size_t max_segment_bytes, size_t max_records, int depth,
                              mi_crc32c_pipeline** out)
{
    if (!out || depth < 1 || depth > 16 || max_records == 0)
        return fail(MI_CRC32C_EINVAL, "bad pipeline arguments");
    int st = 0;
    DeviceState* d = dev_or_init(&st);
    if (!d) return st;
    auto* p = new mi_crc32c_pipeline;
    p->dev = d;
    p->slots.resize(size_t(depth));
    p->max_bytes = max_segment_bytes;
    p->max_records = max_records;
    for (auto& s : p->slots)
    {
        if ((st = s.ctx.open(d->ordinal)) || (st = s.seg.reserve(max_segment_bytes + 16)) ||
            (st = s.meta.reserve(max_records * 16)) || (st = s.res.reserve(max_records * 4)) ||
            (st = s.dseg.reserve(max_segment_bytes + 16)) ||
            (st = s.dmeta.reserve(max_records * 16)) || (st = s.ctx.out.reserve(max_records * 4)))
        {
            mi_crc32c_pipeline_destroy(p);
            return st;
        }
    }
    *out = p;
    return MI_CRC32C_OK;
}

int mi_crc32c_pipeline_submit(mi_crc32c_pipeline* p, const void* host_segment, size_t bytes,
                              const uint64_t* offsets, const uint32_t* lengths,
                              const uint32_t* inits, size_t count, uint32_t* host_out,
                              uint64_t* ticket)
{
    if (!p || bytes > p->max_bytes || count > p->max_records || (count && (!offsets || !lengths)) ||
        (bytes && !host_segment) || (count && !host_out))
        return fail(MI_CRC32C_EINVAL, "segment exceeds pipeline limits or null pointer");
    // validated before a ticket is taken: a refused segment leaves no trace
    uint64_t total = 0, maxlen = 0;
    for (size_t i = 0; i < count; ++i)
    {
        if (lengths[i] && (offsets[i] > bytes || lengths[i] > bytes - offsets[i]))
            return fail(MI_CRC32C_EINVAL, "record outside segment");
        total += lengths[i];
        maxlen = std::max<uint64_t>(maxlen, lengths[i]);
    }
    std::lock_guard<std::mutex> lock(p->mu);
    DeviceState* d = p->dev;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != d->ordinal) HIP_TRY(hipSetDevice(d->ordinal));
    const uint64_t t = p->next_ticket++;
    auto& s = p->slots[t % p->slots.size()];
    int st;
    if ((st = slot_complete(s))) return st;
    const void* src = host_segment;
    if (bytes && !is_pinned_span(host_segment, bytes))
    {
        std::memcpy(s.seg.p, host_segment, bytes);
        src = s.seg.p;
    }
    uint8_t* meta = s.meta.as<uint8_t>();
    std::memcpy(meta, offsets, count * 8);
    std::memcpy(meta + count * 8, lengths, count * 4);
    if (inits) std::memcpy(meta + count * 12, inits, count * 4);
    Ctx& c = s.ctx;
    if (bytes) HIP_TRY(hipMemcpyAsync(s.dseg.p, src, bytes, hipMemcpyHostToDevice, c.stream));
    HIP_TRY(hipMemcpyAsync(s.dmeta.p, meta, count * (inits ? 16 : 12), hipMemcpyHostToDevice,
                           c.stream));
    uint8_t* dm = s.dmeta.as<uint8_t>();
    if ((st = run_var(d, &c, s.dseg.p, reinterpret_cast<uint64_t*>(dm),
                      reinterpret_cast<uint32_t*>(dm + count * 8),
                      inits ? reinterpret_cast<uint32_t*>(dm + count * 12) : nullptr, count, total,
                      c.out.as<uint32_t>(), maxlen)))
        return st;
    HIP_TRY(hipMemcpyAsync(s.res.p, c.out.p, count * 4, hipMemcpyDeviceToHost, c.stream));
    HIP_TRY(hipEventRecord(c.done, c.stream));
    s.ticket = t;
    s.host_out = host_out;
    s.count = count;
    if (ticket) *ticket = t;
    return MI_CRC32C_OK;
}

int mi_crc32c_pipeline_wait(mi_crc32c_pipeline* p, uint64_t ticket)
{
    if (!p) return fail(MI_CRC32C_EINVAL, "null pipeline");
    std::lock_guard<std::mutex> lock(p->mu);
    auto& s = p->slots[ticket % p->slots.size()];
    if (s.ticket != ticket) return MI_CRC32C_OK;  // already completed
    return slot_complete(s);
}

int mi_crc32c_pipeline_destroy(mi_crc32c_pipeline* p)
{
    if (!p) return MI_CRC32C_OK;
    int rc = MI_CRC32C_OK;
    for (auto& s : p->slots)
    {
        if (s.ctx.stream && s.ticket) rc = slot_complete(s);
        s.ctx.release();
        for (DevBuf* b : {&s.dseg, &s.dmeta}) b->release();
        for (PinBuf* b : {&s.seg, &s.meta, &s.res}) b->release();
    }
    delete p;
    return rc;
}

// ---- memory helpers ---------------------------------------------------------
int mi_dev_malloc(void** p, size_t bytes)
{
    int st = 0;
    if (!p) return fail(MI_CRC32C_EINVAL, "null out pointer");
    if (!thread_ctx(&st)) return st;  // makes the default device current
    if (hipMalloc(p, std::max<size_t>(bytes, 1)) != hipSuccess)
        return fail(MI_CRC32C_ENOMEM, "hipMalloc(" + std::to_string(bytes) + ") failed");
    return MI_CRC32C_OK;
}

int mi_dev_free(void* p)
{
    if (p) HIP_TRY(hipFree(p));
    return MI_CRC32C_OK;
}

int mi_host_malloc_pinned(void** p, size_t bytes)
{
    int st = 0;
    if (!p) return fail(MI_CRC32C_EINVAL, "null out pointer");
    if (!dev_or_init(&st)) return st;
    // mapped (and portable: every device's address space), so batches over
    // these bytes can be read in place by the kernels (zero-copy)
    if (hipHostMalloc(p, std::max<size_t>(bytes, 1), hipHostMallocMapped | hipHostMallocPortable) !=
        hipSuccess)
        return fail(MI_CRC32C_ENOMEM, "hipHostMalloc(" + std::to_string(bytes) + ") failed");
    return MI_CRC32C_OK;
}

int mi_host_free_pinned(void* p)
{
    if (p) HIP_TRY(hipHostFree(p));
    return MI_CRC32C_OK;
}

int mi_memcpy(void* dst, const void* src, size_t bytes, int kind)
{
    int st = 0;
    Ctx* c = thread_ctx(&st);
    if (!c) return st;
    const hipMemcpyKind k = kind == MI_MEMCPY_H2D   ? hipMemcpyHostToDevice
                            : kind == MI_MEMCPY_D2H ? hipMemcpyDeviceToHost
                                                    : hipMemcpyDeviceToDevice;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, k, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MI_CRC32C_OK;
}

int mi_memset(void* dev, int value, size_t bytes)
{
    int st = 0;
    Ctx* c = thread_ctx(&st);
    if (!c) return st;
    HIP_TRY(hipMemsetAsync(dev, value, bytes, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MI_CRC32C_OK;
}

int mi_fill_splitmix64(void* dev, size_t nbytes, uint64_t seed, uint64_t byte_offset)
{
    if ((uintptr_t(dev) & 7u) || (byte_offset & 7u))
        return fail(MI_CRC32C_EINVAL, "fill needs 8-byte alignment");
    int st = 0;
    Ctx* c = thread_ctx(&st);
    if (!c) return st;
    HIP_TRY(launch_fill_splitmix(dev, nbytes, seed, byte_offset, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MI_CRC32C_OK;
}

int mi_timer_start(void)
{
    int st = 0;
    Ctx* c = thread_ctx(&st);
    if (!c) return st;
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    return MI_CRC32C_OK;
}

int mi_timer_stop(float* elapsed_ms)
{
    int st = 0;
    Ctx* c = thread_ctx(&st);
    if (!c) return st;
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    HIP_TRY(hipEventSynchronize(c->ev1));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (elapsed_ms) *elapsed_ms = ms;
    return MI_CRC32C_OK;
}

// ---- RCCL ---------------------------------------------------------------------
static ncclComm_t g_comm = nullptr;

int mi_comm_unique_id(unsigned char id[MI_COMM_ID_BYTES])
{
    static_assert(sizeof(ncclUniqueId) <= MI_COMM_ID_BYTES, "unique id size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(MI_CRC32C_ERCCL, ncclGetErrorString(r));
    std::memset(id, 0, MI_COMM_ID_BYTES);
    std::memcpy(id, &u, sizeof(u));
    return MI_CRC32C_OK;
}

int mi_comm_init(const unsigned char id[MI_COMM_ID_BYTES], int nranks, int rank)
{
    int st = 0;
    if (!thread_ctx(&st)) return st;
    if (g_comm) return fail(MI_CRC32C_EINVAL, "communicator already initialised");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&g_comm, nranks, u, rank);
    if (r != ncclSuccess) return fail(MI_CRC32C_ERCCL, ncclGetErrorString(r));
    return MI_CRC32C_OK;
}

int mi_comm_allgather_u32(const uint32_t* dev_send, size_t count, uint32_t* dev_recv)
{
    int st = 0;
    Ctx* c = thread_ctx(&st);
    if (!c) return st;
    if (!g_comm) return fail(MI_CRC32C_EINVAL, "no communicator");
    const ncclResult_t r = ncclAllGather(dev_send, dev_recv, count, ncclUint32, g_comm, c->stream);
    if (r != ncclSuccess) return fail(MI_CRC32C_ERCCL, ncclGetErrorString(r));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MI_CRC32C_OK;
}

int mi_comm_info(int* nranks, int* rank, int* device)
{
    if (!g_comm) return fail(MI_CRC32C_EINVAL, "no communicator");
    ncclResult_t r = ncclSuccess;
    if (nranks && (r = ncclCommCount(g_comm, nranks)) != ncclSuccess)
        return fail(MI_CRC32C_ERCCL, ncclGetErrorString(r));
    if (rank && (r = ncclCommUserRank(g_comm, rank)) != ncclSuccess)
        return fail(MI_CRC32C_ERCCL, ncclGetErrorString(r));
    if (device && (r = ncclCommCuDevice(g_comm, device)) != ncclSuccess)
        return fail(MI_CRC32C_ERCCL, ncclGetErrorString(r));
    return MI_CRC32C_OK;
}

int mi_comm_destroy(void)
{
    if (g_comm)
    {
        ncclCommDestroy(g_comm);
        g_comm = nullptr;
    }
    return MI_CRC32C_OK;
}

}  // extern "C"
