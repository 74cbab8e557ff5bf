// tools/sanitize/engine_stub.cc -- stand-in for the HIP engine (engine.hip)
// in the sanitizer builds of the host code (ThreadSanitizer, AddressSanitizer
// + UBSan; tools/sanitize/Makefile).  Sanitizers cannot instrument the GPU
// side, so the host layers above it -- api.cc (fallback, multi-device
// workers), host_crc.cc and durable_log.cc (the lock-free reservation
// protocol, flush and sync threads) -- are linked against this stub:
//
//   STUB_ENGINE=fail (default): every device call fails as without a GPU, so
//       every checksum takes the counted CPU fallback;
//   STUB_ENGINE=ok: the stub plays a working device (it answers with the
//       engine's CPU arithmetic), so the no-fallback paths run, including the
//       multi-device worker threads (STUB_DEVICES devices, default 4).
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../consus_amd/csrc/engine_internal.h"
#include "../../consus_amd/csrc/host_crc.h"
#include "../../include/consus_crc32c.h"

namespace {

bool ok_mode()
{
    static const bool ok = [] {
        const char* e = std::getenv("STUB_ENGINE");
        return e && !std::strcmp(e, "ok");
    }();
    return ok;
}

int no_device() { return mi_eng::fail(MI_CRC32C_ENODEV, "sanitizer build: no GPU engine"); }

}  // namespace

namespace mi_eng {

int usable_devices(int* ordinals, int max)
{
    if (!ok_mode()) return 0;
    const char* e = std::getenv("STUB_DEVICES");
    const int n = std::min(max, e ? std::atoi(e) : 4);
    for (int i = 0; i < n; ++i) ordinals[i] = i;
    return n;
}

int buffer(int, uint32_t init, const void* data, size_t n, uint32_t* out, unsigned flags)
{
    if (!out || (n && !data)) return fail(MI_CRC32C_EINVAL, "null pointer");
    if (!ok_mode() || (flags & MI_CRC32C_DEVICE)) return no_device();
    *out = mi_host::crc32c(init, data, n);
    return MI_CRC32C_OK;
}

int batch(int, const void* base, const uint64_t* offsets, const uint32_t* lengths,
          const uint32_t* inits, size_t count, uint64_t, uint32_t* out, unsigned flags)
{
    if (count == 0) return MI_CRC32C_OK;
    if (!offsets || !lengths || !out) return fail(MI_CRC32C_EINVAL, "null array");
    if (!ok_mode() || (flags & MI_CRC32C_DEVICE)) return no_device();
    mi_host::batch(base, offsets, lengths, inits, count, out);
    return MI_CRC32C_OK;
}

int batch_fixed(int, const void* base, uint64_t stride, uint64_t length, const uint32_t* inits,
                size_t count, uint32_t* out, unsigned flags)
{
    if (count == 0) return MI_CRC32C_OK;
    if (!out) return fail(MI_CRC32C_EINVAL, "null out");
    if (!ok_mode() || (flags & MI_CRC32C_DEVICE)) return no_device();
    mi_host::batch_fixed(base, stride, length, inits, count, out);
    return MI_CRC32C_OK;
}

}  // namespace mi_eng

extern "C" {

// the durable log stages in pinned memory when the engine provides it
int mi_host_malloc_pinned(void** p, size_t)
{
    if (p) *p = nullptr;
    return no_device();
}

int mi_host_free_pinned(void* p)
{
    std::free(p);
    return MI_CRC32C_OK;
}

}  // extern "C"
