// tools/zerocopy_probe.hip -- round-trip latency of a small host call with the
// kernel reading and writing mapped pinned host memory (zero-copy) against
// the staged path (H2D copy, kernel on device memory, D2H copy), on one
// stream (dev tool).  Checks every result.
//   hipcc --offload-arch=gfx950 -O2 -o tools/zerocopy_probe tools/zerocopy_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                      \
    do                                                                                \
    {                                                                                 \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess)                                                         \
        {                                                                             \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

// one workgroup: XOR of the n/4 words -> out[0]
__global__ void xor_words(const uint32_t* __restrict__ in, uint32_t n_words, uint32_t* out)
{
    __shared__ uint32_t sh[256];
    uint32_t x = 0;
    for (uint32_t i = threadIdx.x; i < n_words; i += blockDim.x) x ^= in[i];
    sh[threadIdx.x] = x;
    __syncthreads();
    for (uint32_t s = 128; s; s >>= 1)
    {
        if (threadIdx.x < s) sh[threadIdx.x] ^= sh[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = sh[0];
}

int main()
{
    const size_t cap = size_t(1) << 20;
    void *h_in = nullptr, *h_out = nullptr, *d_in_map = nullptr, *d_out_map = nullptr;
    CHECK(hipHostMalloc(&h_in, cap, hipHostMallocMapped));
    CHECK(hipHostMalloc(&h_out, 4096, hipHostMallocMapped));
    CHECK(hipHostGetDevicePointer(&d_in_map, h_in, 0));
    CHECK(hipHostGetDevicePointer(&d_out_map, h_out, 0));
    std::printf("mapped: host %p -> device %p (%s)\n", h_in, d_in_map,
                h_in == d_in_map ? "same VA" : "different VA");
    void *d_in = nullptr, *d_out = nullptr;
    CHECK(hipMalloc(&d_in, cap));
    CHECK(hipMalloc(&d_out, 4096));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<uint8_t> src(cap);
    for (size_t i = 0; i < cap; ++i) src[i] = uint8_t(i * 2654435761u >> 13);
    uint32_t sink = 0;
    for (size_t n : {size_t(16), size_t(1024), size_t(16384), size_t(262144), size_t(1) << 20})
    {
        uint32_t want = 0;
        for (size_t i = 0; i + 4 <= n; i += 4)
        {
            uint32_t w;
            std::memcpy(&w, src.data() + i, 4);
            want ^= w;
        }
        std::vector<double> tz, ts;
        for (int it = 0; it < 300; ++it)
        {
            // zero-copy: CPU copies into mapped pinned memory, the kernel reads it
            // over PCIe and writes its result straight to host memory
            auto t0 = std::chrono::steady_clock::now();
            std::memcpy(h_in, src.data(), n);
            hipLaunchKernelGGL(xor_words, dim3(1), dim3(256), 0, s,
                               static_cast<const uint32_t*>(d_in_map), uint32_t(n / 4),
                               static_cast<uint32_t*>(d_out_map));
            CHECK(hipStreamSynchronize(s));
            const uint32_t gz = *static_cast<volatile uint32_t*>(h_out);
            auto t1 = std::chrono::steady_clock::now();
            // staged: H2D, kernel on device memory, D2H
            std::memcpy(h_in, src.data(), n);
            CHECK(hipMemcpyAsync(d_in, h_in, n, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(xor_words, dim3(1), dim3(256), 0, s,
                               static_cast<const uint32_t*>(d_in), uint32_t(n / 4),
                               static_cast<uint32_t*>(d_out));
            CHECK(hipMemcpyAsync(h_out, d_out, 4, hipMemcpyDeviceToHost, s));
            CHECK(hipStreamSynchronize(s));
            const uint32_t gs = *static_cast<volatile uint32_t*>(h_out);
            auto t2 = std::chrono::steady_clock::now();
            if (gz != want || gs != want)
            {
                std::fprintf(stderr, "MISMATCH n=%zu zero-copy %08x staged %08x want %08x\n", n,
                             gz, gs, want);
                return 1;
            }
            sink ^= gz;
            tz.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            ts.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
        }
        std::nth_element(tz.begin(), tz.begin() + tz.size() / 2, tz.end());
        std::nth_element(ts.begin(), ts.begin() + ts.size() / 2, ts.end());
        std::printf("n=%8zu  zero-copy %7.1f us   staged %7.1f us  (median of 300)\n", n,
                    tz[tz.size() / 2], ts[ts.size() / 2]);
    }
    CHECK(hipStreamDestroy(s));
    CHECK(hipFree(d_in));
    CHECK(hipFree(d_out));
    CHECK(hipHostFree(h_in));
    CHECK(hipHostFree(h_out));
    return sink == 0x12345678u ? 2 : 0;
}
