// consus_amd/csrc/host_crc.h -- the engine's own CPU path for CRC-32C.
//
// Runs when the GPU engine cannot (a HIP call failed, no usable gfx950
// device) -- it is what makes the drop-in total, as the reference function is
// (common/crc32c.cc:122-126 cannot fail) -- and for single host calls too
// small to pay a GPU round trip (size routing, mi_crc32c_set_gpu_min).  Every
// use is counted (mi_crc32c_stats: fallback_calls, host_routed_calls); the GPU
// parity tests run with the routing threshold at 0 and assert both counts stay
// 0, so they certify the HIP kernels, never this path.  Product code,
// independent of the test oracle under oracle/.
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace mi_host {

// consus::crc32c(init, p, n): reflected CRC-32C, init is a previous CRC output.
uint32_t crc32c(uint32_t init, const void* p, size_t n);

// Record i = [base + offsets[i], + lengths[i]); out[i] = crc32c(inits ? inits[i] : 0, record).
void batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
           const uint32_t* inits, size_t count, uint32_t* out);

// Record i = [base + i * stride, + length).
void batch_fixed(const void* base, uint64_t stride, uint64_t length, const uint32_t* inits,
                 size_t count, uint32_t* out);

// Bookkeeping of fallbacks (engine status that forced it, bytes hashed on the CPU).
void note_fallback(int status, uint64_t bytes);
void note_gpu_call();
void note_sharded_call();
void note_sorted_batch(bool one_launch = false);
void note_window_batch();
void note_zero_copy_batch();
void note_hint_overflow();
void note_host_batch(uint64_t bytes);
void note_host_routed(uint64_t bytes);
void note_multi(int ranges, const int* devices);

}  // namespace mi_host
