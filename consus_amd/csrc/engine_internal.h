// consus_amd/csrc/engine_internal.h -- seam between the C ABI layer (api.cc:
// argument checks, CPU fallback after engine failures, multi-device
// sharding, statistics) and the HIP engine (engine.hip: devices, streams,
// staging, kernel launches).  Internal to libconsus_crc32c.so.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>

namespace mi_eng {

constexpr int kMaxDevices = 16;

// Record `msg` as the calling thread's last error; returns status.
int fail(int status, const std::string& msg);

// Ordinals of the usable (gfx950) devices, at most `max`; returns how many.
// Does not initialise them.
int usable_devices(int* ordinals, int max);

// Compute entry points on device `dev` (-1 = the process's default device,
// see mi_crc32c_init).  Same arguments and statuses as the C ABI functions
// of the same name; no CPU fallback here.
int buffer(int dev, uint32_t init, const void* data, size_t n, uint32_t* out, unsigned flags);
int batch(int dev, const void* base, const uint64_t* offsets, const uint32_t* lengths,
          const uint32_t* inits, size_t count, uint64_t total_bytes, uint32_t* out,
          unsigned flags);
int batch_fixed(int dev, const void* base, uint64_t stride, uint64_t length,
                const uint32_t* inits, size_t count, uint32_t* out, unsigned flags);

}  // namespace mi_eng
