// consus_amd/csrc/api.cc -- the compute entry points of the C ABI
// (include/consus_crc32c.h) above the HIP engine (engine.hip):
//
//   * argument checks and the per-thread error message;
//   * size routing: single host calls below the GPU threshold
//     (mi_crc32c_set_gpu_min) are answered by the CPU path without a GPU
//     round trip, counted as host_routed_calls;
//   * totality: the drop-in mi_crc32c / consus::crc32c never fails, as the
//     reference cannot (common/crc32c.cc:122-126).  When the engine reports a
//     failure (no usable device, a HIP error, an input beyond its limits) the
//     call is completed by the engine's own CPU path (host_crc.cc) and
//     counted in mi_crc32c_stats.  Status-returning calls do the same only
//     with MI_CRC32C_FALLBACK (the durable log passes it); otherwise they
//     return the status;
//   * multi-device sharding of host batches (mi_crc32c_batch[_fixed]_multi):
//     contiguous record ranges balanced by bytes, one per device, each
//     staged over that device's own PCIe link by a persistent worker thread
//     (SURVEY.md 8(e)), only when every shard amortises the hand-off.
//
// Host-only C++: also linked, with an engine stub, into the sanitizer builds
// of tools/sanitize/ (ThreadSanitizer, AddressSanitizer + UBSan).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/consus_crc32c.h"
#include "engine_internal.h"
#include "host_crc.h"

namespace mi_eng {

thread_local std::string t_err;

int fail(int status, const std::string& msg)
{
    t_err = msg;
    return status;
}

}  // namespace mi_eng

namespace {

using mi_eng::fail;

// Per-range amortisation threshold of the multi-device entry points.
// Measured on MI355X (tools/shard_probe.py, profiles/r02_shard_overhead.txt):
// a host batch of 4 KiB records costs 0.114 / 0.157 / 0.424 / 1.28 ms on one
// device at 1 / 4 / 16 / 64 MiB (pageable memory, 52-56 GB/s from 64 MiB up),
// and the split itself (worker hand-off, a second stream and staging) adds
// 2-15 us.  A range of >= 4 MiB therefore carries >= 0.157 ms of link time,
// of which a split costs < 10 %.  MI_CRC32C_SHARD_MIN (bytes) overrides it.
constexpr uint64_t kShardMinDefault = uint64_t(4) << 20;

uint64_t shard_min(uint64_t arg)
{
    if (arg) return arg;
    static const uint64_t env = [] {
        const char* e = std::getenv("MI_CRC32C_SHARD_MIN");
        return e ? std::strtoull(e, nullptr, 0) : 0ull;
    }();
    return env ? env : kShardMinDefault;
}

// Single host calls below this many bytes are answered on the CPU (size
// routing).  Measured on MI355X + EPYC 9575F (tools/route_probe.cc,
// profiles/r03_route_probe.txt): a GPU round trip of
// one host call costs 17 us at 16 B, 21 us at 4 KiB, 117 us at 1 MiB and
// 154 us at 4 MiB (pageable staging); the CPU path runs at ~13 GiB/s (0.03 us
// at 16 B, 78 us at 1 MiB, 313 us at 4 MiB).  They cross near 1.7 MiB.
constexpr uint64_t kGpuMinDefault = uint64_t(3) << 19;  // 1.5 MiB

std::atomic<uint64_t>& gpu_min_word()
{
    static std::atomic<uint64_t> w{[] {
        const char* e = std::getenv("MI_CRC32C_GPU_MIN");
        return e ? uint64_t(std::strtoull(e, nullptr, 0)) : kGpuMinDefault;
    }()};
    return w;
}

// A failure the CPU path can stand in for: anything but a bad argument.
bool engine_failure(int st) { return st != MI_CRC32C_OK && st != MI_CRC32C_EINVAL; }

uint64_t sum_lengths(const uint32_t* lengths, size_t count)
{
    uint64_t t = 0;
    for (size_t i = 0; i < count; ++i) t += lengths[i];
    return t;
}

// ---- persistent workers for multi-device calls -----------------------------
// One worker per extra shard, created on first use and kept for the life of
// the process, so each keeps its HIP streams and staging buffers (engine.hip
// keeps one context per thread and device) from call to call.  One
// multi-device call runs at a time.
class Workers
{
  public:
    // Runs jobs[0] on the calling thread and jobs[1..] on workers; waits for
    // all of them before returning, even if jobs[0] throws (the workers hold
    // pointers into `jobs`).  Jobs catch their own exceptions (guarded()).
    void run(std::vector<std::function<void()>>& jobs)
    {
        std::lock_guard<std::mutex> call(m_call);
        while (m_ws.size() + 1 < jobs.size()) m_ws.emplace_back(new Worker);
        size_t posted = 0;
        struct JoinAll
        {
            Workers* w;
            const size_t* n;
            ~JoinAll()
            {
                for (size_t j = 0; j < *n; ++j) w->m_ws[j]->join();
            }
        } join_all{this, &posted};
        for (size_t j = 1; j < jobs.size(); ++j, ++posted) m_ws[j - 1]->post(&jobs[j]);
        jobs[0]();
    }

  private:
    struct Worker
    {
        std::mutex mu;
        std::condition_variable cv;
        std::function<void()>* job = nullptr;
        bool busy = false;
        Worker()
        {
            std::thread([this] { loop(); }).detach();  // lives as long as the process
        }
        void post(std::function<void()>* j)
        {
            std::lock_guard<std::mutex> hold(mu);
            job = j;
            busy = true;
            cv.notify_all();
        }
        void join()
        {
            std::unique_lock<std::mutex> hold(mu);
            cv.wait(hold, [&] { return !busy; });
        }
        void loop()
        {
            std::unique_lock<std::mutex> hold(mu);
            while (true)
            {
                cv.wait(hold, [&] { return job != nullptr; });
                std::function<void()>* j = job;
                hold.unlock();
                (*j)();
                hold.lock();
                job = nullptr;
                busy = false;
                cv.notify_all();
            }
        }
    };
    std::mutex m_call;
    std::vector<Worker*> m_ws;  // never destroyed: detached threads wait on them
};

Workers& workers()
{
    static Workers* w = new Workers;  // leaked on purpose (see Workers)
    return *w;
}

// A job body that never lets an exception escape (it would cross the C ABI,
// or kill a worker thread): std::bad_alloc maps to ENOMEM, anything else to
// EHIP, recorded in the job's status slot.
template <typename F>
void guarded(int& status, std::string& msg, F&& body)
{
    try
    {
        body();
    }
    catch (const std::bad_alloc&)
    {
        status = MI_CRC32C_ENOMEM;
        msg = "out of host memory";
    }
    catch (const std::exception& e)
    {
        status = MI_CRC32C_EHIP;
        msg = e.what();
    }
    catch (...)
    {
        status = MI_CRC32C_EHIP;
        msg = "unknown exception";
    }
}

// MI_CRC32C_DEVICES="0,1,2,3": the device list multi-device calls use when
// the caller names none (an ordinal may repeat: two ranges on one device).
int env_devices(int* out)
{
    const char* e = std::getenv("MI_CRC32C_DEVICES");
    if (!e || !*e) return -1;
    int n = 0;
    for (const char* p = e; *p && n < mi_eng::kMaxDevices;)
    {
        char* end = nullptr;
        const long v = std::strtol(p, &end, 10);
        if (end == p) break;
        if (v >= 0 && v < mi_eng::kMaxDevices) out[n++] = int(v);
        p = *end == ',' ? end + 1 : end;
    }
    return n;
}

// The devices a multi-device call may use.
int pick_devices(const int* devices, int ndev, int* out)
{
    if (devices && ndev > 0)
    {
        const int n = std::min(ndev, mi_eng::kMaxDevices);
        for (int i = 0; i < n; ++i) out[i] = devices[i];
        return n;
    }
    int n = env_devices(out);
    if (n < 0) n = mi_eng::usable_devices(out, mi_eng::kMaxDevices);
    return ndev > 0 ? std::min(n, ndev) : n;
}

// MI_CRC32C_CPU: the engine's CPU path by the caller's choice (host memory
// only), counted apart from fallbacks.
int host_batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
               const uint32_t* inits, size_t count, uint64_t total_bytes, uint32_t* out,
               unsigned flags)
{
    if (flags & MI_CRC32C_DEVICE)
        return fail(MI_CRC32C_EINVAL, "MI_CRC32C_CPU takes host memory, not device pointers");
    if (count == 0) return MI_CRC32C_OK;
    if (!offsets || !lengths || !out) return fail(MI_CRC32C_EINVAL, "null array with count > 0");
    for (size_t i = 0; i < count; ++i)
        if (offsets[i] > UINT64_MAX - lengths[i])
            return fail(MI_CRC32C_EINVAL, "record end overflows 64 bits");
    const uint64_t total = total_bytes ? total_bytes : sum_lengths(lengths, count);
    if (!base && total) return fail(MI_CRC32C_EINVAL, "null base");
    mi_host::batch(base, offsets, lengths, inits, count, out);
    mi_host::note_host_batch(total);
    return MI_CRC32C_OK;
}

}  // namespace

extern "C" {

// Contiguous record ranges with about equal byte sums (consus_amd/shard.py
// balanced_ranges): range r ends at the first record whose inclusive prefix
// sum reaches ceil(total * r / k).  bounds has k + 1 entries.
void mi_crc32c_balanced_ranges(const uint32_t* lengths, size_t count, int k, uint64_t total,
                               size_t* bounds)
{
    if (k < 1 || !bounds) return;
    bounds[0] = 0;
    uint64_t pref = 0;
    size_t i = 0;
    for (int r = 1; r < k; ++r)
    {
        const uint64_t target = (total * uint64_t(r) + uint64_t(k) - 1) / uint64_t(k);
        // first i with pref(i inclusive) >= target
        while (i < count && pref + lengths[i] < target) pref += lengths[i++];
        size_t cut = i < count ? i + 1 : count;
        cut = std::max(cut, bounds[r - 1]);
        bounds[r] = std::min(cut, count);
    }
    bounds[k] = count;
}

const char* mi_crc32c_strerror(int status)
{
    switch (status)
    {
        case MI_CRC32C_OK: return "ok";
        case MI_CRC32C_EINVAL: return "invalid argument";
        case MI_CRC32C_ENODEV: return "no usable gfx950 device";
        case MI_CRC32C_ENOMEM: return "out of memory";
        case MI_CRC32C_EHIP: return "HIP runtime error";
        case MI_CRC32C_ERCCL: return "RCCL error";
        case MI_CRC32C_ERANGE: return "input beyond the GPU engine's limits";
        default: return "unknown status";
    }
}

const char* mi_crc32c_last_error(void) { return mi_eng::t_err.c_str(); }

int mi_crc32c_device_count(void)
{
    int ords[mi_eng::kMaxDevices];
    return mi_eng::usable_devices(ords, mi_eng::kMaxDevices);
}

uint64_t mi_crc32c_set_gpu_min(uint64_t gpu_min) { return gpu_min_word().exchange(gpu_min); }

uint64_t mi_crc32c_gpu_min(void) { return gpu_min_word().load(std::memory_order_relaxed); }

int mi_crc32c_buffer(uint32_t init, const void* data, size_t n, uint32_t* out, unsigned flags)
{
    if (!(flags & MI_CRC32C_DEVICE) && n && n < gpu_min_word().load(std::memory_order_relaxed))
    {
        if (!out || !data) return fail(MI_CRC32C_EINVAL, "null pointer");
        *out = mi_host::crc32c(init, data, n);
        mi_host::note_host_routed(n);
        return MI_CRC32C_OK;
    }
    const int st = mi_eng::buffer(-1, init, data, n, out, flags);
    if (st == MI_CRC32C_OK)
    {
        if (n) mi_host::note_gpu_call();
        return st;
    }
    if (!(flags & MI_CRC32C_FALLBACK) || (flags & MI_CRC32C_DEVICE) || !engine_failure(st))
        return st;
    *out = mi_host::crc32c(init, data, n);
    mi_host::note_fallback(st, n);
    return MI_CRC32C_OK;
}

uint32_t mi_crc32c(uint32_t init, const void* data, size_t n)
{
    if (n == 0) return init;
    // too small to pay a GPU round trip: the CPU path, by design (counted)
    if (n < gpu_min_word().load(std::memory_order_relaxed))
    {
        mi_host::note_host_routed(n);
        return mi_host::crc32c(init, data, n);
    }
    uint32_t out = 0;
    const int st = mi_eng::buffer(-1, init, data, n, &out, 0);
    if (st == MI_CRC32C_OK)
    {
        mi_host::note_gpu_call();
        return out;
    }
    // The reference function cannot fail: complete the call on the CPU path.
    mi_host::note_fallback(st, n);
    return mi_host::crc32c(init, data, n);
}

int mi_crc32c_batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                    const uint32_t* inits, size_t count, uint64_t total_bytes, uint32_t* out,
                    unsigned flags)
{
    if (flags & MI_CRC32C_CPU)
        return host_batch(base, offsets, lengths, inits, count, total_bytes, out, flags);
    const int st = mi_eng::batch(-1, base, offsets, lengths, inits, count, total_bytes, out, flags);
    if (st == MI_CRC32C_OK)
    {
        if (count) mi_host::note_gpu_call();
        return st;
    }
    if (!(flags & MI_CRC32C_FALLBACK) || (flags & MI_CRC32C_DEVICE) || !engine_failure(st))
        return st;
    mi_host::batch(base, offsets, lengths, inits, count, out);
    mi_host::note_fallback(st, total_bytes ? total_bytes : sum_lengths(lengths, count));
    return MI_CRC32C_OK;
}

int mi_crc32c_batch_fixed(const void* base, uint64_t stride, uint64_t length,
                          const uint32_t* inits, size_t count, uint32_t* out, unsigned flags)
{
    const int st = mi_eng::batch_fixed(-1, base, stride, length, inits, count, out, flags);
    if (st == MI_CRC32C_OK)
    {
        if (count) mi_host::note_gpu_call();
        return st;
    }
    if (!(flags & MI_CRC32C_FALLBACK) || (flags & MI_CRC32C_DEVICE) || !engine_failure(st))
        return st;
    mi_host::batch_fixed(base, stride, length, inits, count, out);
    mi_host::note_fallback(st, uint64_t(count) * length);
    return MI_CRC32C_OK;
}

int mi_crc32c_batch_multi(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                          const uint32_t* inits, size_t count, uint64_t total_bytes,
                          uint32_t* out, unsigned flags, const int* devices, int ndev,
                          uint64_t shard_min_bytes)
{
    if (count == 0) return MI_CRC32C_OK;
    if (flags & MI_CRC32C_CPU)
        return host_batch(base, offsets, lengths, inits, count, total_bytes, out, flags);
    if (flags & MI_CRC32C_DEVICE)
        return fail(MI_CRC32C_EINVAL,
                    "multi-device batches take host memory: device-resident records are hashed "
                    "on the device that holds them (mi_crc32c_batch)");
    if (!offsets || !lengths || !out || (!base && total_bytes))
        return fail(MI_CRC32C_EINVAL, "null array with count > 0");
    int devs[mi_eng::kMaxDevices];
    const int nd = pick_devices(devices, ndev, devs);
    const uint64_t total = total_bytes ? total_bytes : sum_lengths(lengths, count);
    const uint64_t per = shard_min(shard_min_bytes);
    int k = int(std::min<uint64_t>(uint64_t(std::max(nd, 1)), std::max<uint64_t>(total / per, 1)));
    k = int(std::min<uint64_t>(uint64_t(k), count));
    if (nd == 0)
    {
        const int st = fail(MI_CRC32C_ENODEV, "no usable gfx950 device");
        if (!(flags & MI_CRC32C_FALLBACK)) return st;
        mi_host::batch(base, offsets, lengths, inits, count, out);
        mi_host::note_fallback(st, total);
        return MI_CRC32C_OK;
    }
    std::vector<size_t> bounds(size_t(k) + 1);
    mi_crc32c_balanced_ranges(lengths, count, k, total, bounds.data());
    std::vector<int> status(static_cast<size_t>(k), MI_CRC32C_OK);
    std::vector<std::string> msgs(static_cast<size_t>(k));
    std::vector<std::function<void()>> jobs;
    for (int j = 0; j < k; ++j)
        jobs.emplace_back([&, j] { guarded(status[size_t(j)], msgs[size_t(j)], [&] {
            const size_t lo = bounds[size_t(j)], n = bounds[size_t(j) + 1] - lo;
            if (n == 0) return;
            const uint64_t bytes = sum_lengths(lengths + lo, n);
            int st = mi_eng::batch(devs[j], base, offsets + lo, lengths + lo,
                                   inits ? inits + lo : nullptr, n, bytes, out + lo,
                                   flags & ~unsigned(MI_CRC32C_FALLBACK));
            if (st != MI_CRC32C_OK && (flags & MI_CRC32C_FALLBACK) && engine_failure(st))
            {
                mi_host::batch(base, offsets + lo, lengths + lo, inits ? inits + lo : nullptr, n,
                               out + lo);
                mi_host::note_fallback(st, bytes);
                st = MI_CRC32C_OK;
            }
            else if (st == MI_CRC32C_OK)
                mi_host::note_gpu_call();
            status[size_t(j)] = st;
            if (st != MI_CRC32C_OK) msgs[size_t(j)] = mi_eng::t_err;
        }); });
    mi_host::note_multi(k, devs);
    if (k == 1)
        jobs[0]();
    else
    {
        mi_host::note_sharded_call();
        workers().run(jobs);
    }
    for (int j = 0; j < k; ++j)
        if (status[size_t(j)] != MI_CRC32C_OK) return fail(status[size_t(j)], msgs[size_t(j)]);
    return MI_CRC32C_OK;
}

int mi_crc32c_batch_fixed_multi(const void* base, uint64_t stride, uint64_t length,
                                const uint32_t* inits, size_t count, uint32_t* out,
                                unsigned flags, const int* devices, int ndev,
                                uint64_t shard_min_bytes)
{
    if (count == 0) return MI_CRC32C_OK;
    if (flags & MI_CRC32C_DEVICE)
        return fail(MI_CRC32C_EINVAL,
                    "multi-device batches take host memory: device-resident records are hashed "
                    "on the device that holds them (mi_crc32c_batch_fixed)");
    if (!out || (!base && length)) return fail(MI_CRC32C_EINVAL, "null pointer with count > 0");
    int devs[mi_eng::kMaxDevices];
    const int nd = pick_devices(devices, ndev, devs);
    const uint64_t total = uint64_t(count) * length;
    const uint64_t per = shard_min(shard_min_bytes);
    int k = int(std::min<uint64_t>(uint64_t(std::max(nd, 1)), std::max<uint64_t>(total / per, 1)));
    k = int(std::min<uint64_t>(uint64_t(k), count));
    if (nd == 0)
    {
        const int st = fail(MI_CRC32C_ENODEV, "no usable gfx950 device");
        if (!(flags & MI_CRC32C_FALLBACK)) return st;
        mi_host::batch_fixed(base, stride, length, inits, count, out);
        mi_host::note_fallback(st, total);
        return MI_CRC32C_OK;
    }
    std::vector<int> status(static_cast<size_t>(k), MI_CRC32C_OK);
    std::vector<std::string> msgs(static_cast<size_t>(k));
    std::vector<std::function<void()>> jobs;
    const uint8_t* b = static_cast<const uint8_t*>(base);
    for (int j = 0; j < k; ++j)
        jobs.emplace_back([&, j] { guarded(status[size_t(j)], msgs[size_t(j)], [&] {
            const size_t lo = count * size_t(j) / size_t(k), hi = count * size_t(j + 1) / size_t(k);
            if (hi == lo) return;
            int st = mi_eng::batch_fixed(devs[j], b + lo * stride, stride, length,
                                         inits ? inits + lo : nullptr, hi - lo, out + lo,
                                         flags & ~unsigned(MI_CRC32C_FALLBACK));
            if (st != MI_CRC32C_OK && (flags & MI_CRC32C_FALLBACK) && engine_failure(st))
            {
                mi_host::batch_fixed(b + lo * stride, stride, length, inits ? inits + lo : nullptr,
                                     hi - lo, out + lo);
                mi_host::note_fallback(st, uint64_t(hi - lo) * length);
                st = MI_CRC32C_OK;
            }
            else if (st == MI_CRC32C_OK)
                mi_host::note_gpu_call();
            status[size_t(j)] = st;
            if (st != MI_CRC32C_OK) msgs[size_t(j)] = mi_eng::t_err;
        }); });
    mi_host::note_multi(k, devs);
    if (k == 1)
        jobs[0]();
    else
    {
        mi_host::note_sharded_call();
        workers().run(jobs);
    }
    for (int j = 0; j < k; ++j)
        if (status[size_t(j)] != MI_CRC32C_OK) return fail(status[size_t(j)], msgs[size_t(j)]);
    return MI_CRC32C_OK;
}

}  // extern "C"
