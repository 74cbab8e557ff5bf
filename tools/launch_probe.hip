// tools/launch_probe.hip -- where a one-record GPU batch's ~18 us round trip
// goes (dev tool): median us of REPS calls of
//
//   empty       an empty kernel, hipStreamSynchronize
//   lds152      an empty kernel asking for 152 KiB of LDS (as the record kernels)
//   stage       the same kernel reading 152 KiB of tables into LDS
//   flag        empty kernel that stores a sequence number into mapped pinned
//               memory; the host spins on it (no hipStreamSynchronize)
//   flag+sync   as flag, then hipStreamSynchronize (already complete)
//   event       empty kernel, hipEventRecord + hipEventSynchronize
//   launch      hipLaunchKernel alone (host time of the enqueue)
//   spin-*      the same with hipDeviceScheduleSpin set before first use
//
//   launch_probe [REPS] [spin]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <vector>

namespace {

constexpr uint32_t kLds = 155648;

__global__ void empty_kernel() {}

__global__ __launch_bounds__(1024, 1) void lds_kernel(const uint32_t* __restrict__ t, uint32_t* o,
                                                      int stage)
{
    extern __shared__ uint32_t s[];
    if (stage)
    {
        for (uint32_t i = threadIdx.x; i < kLds / 4; i += blockDim.x) s[i] = t[i];
        __syncthreads();
        if (threadIdx.x == 0 && s[7] == 0xFFFFFFFFu && s[99] == 1u) o[0] = 1;  // keep the loads
    }
}

__global__ void flag_kernel(volatile uint32_t* flag, uint32_t seq)
{
    if (threadIdx.x == 0)
    {
        __threadfence_system();
        flag[0] = seq;
    }
}

double median_us(int reps, const std::function<void()>& f)
{
    std::vector<double> t(reps);
    for (int i = 0; i < 50; ++i) f();
    for (int i = 0; i < reps; ++i)
    {
        const auto a = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

#define CK(x)                                                                      \
    do                                                                             \
    {                                                                              \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess)                                                      \
        {                                                                          \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

}  // namespace

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 2000;
    const bool spin = argc > 2 && !strcmp(argv[2], "spin");
    if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    CK(hipSetDevice(0));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&lds_kernel),
                           hipFuncAttributeMaxDynamicSharedMemorySize, int(kLds)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *tab = nullptr, *o = nullptr;
    CK(hipMalloc(&tab, kLds));
    CK(hipMemset(tab, 0, kLds));
    CK(hipMalloc(&o, 64));
    void* hp = nullptr;
    CK(hipHostMalloc(&hp, 4096, hipHostMallocMapped | hipHostMallocPortable));
    volatile uint32_t* hflag = static_cast<volatile uint32_t*>(hp);
    uint32_t* dflag = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), hp, 0));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    uint32_t seq = 0;
    long spins_total = 0;

    const double t_empty = median_us(reps, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CK(hipStreamSynchronize(s));
    });
    const double t_lds = median_us(reps, [&] {
        hipLaunchKernelGGL(lds_kernel, dim3(1), dim3(1024), kLds, s, tab, o, 0);
        CK(hipStreamSynchronize(s));
    });
    const double t_stage = median_us(reps, [&] {
        hipLaunchKernelGGL(lds_kernel, dim3(1), dim3(1024), kLds, s, tab, o, 1);
        CK(hipStreamSynchronize(s));
    });
    const double t_stage3 = median_us(reps, [&] {
        hipLaunchKernelGGL(lds_kernel, dim3(3), dim3(1024), kLds, s, tab, o, 1);
        CK(hipStreamSynchronize(s));
    });
    auto wait_flag = [&](uint32_t want) {
        const auto a = std::chrono::steady_clock::now();
        while (*hflag != want)
        {
            ++spins_total;
            if (std::chrono::steady_clock::now() - a > std::chrono::seconds(2))
            {
                CK(hipStreamSynchronize(s));
                if (*hflag != want)
                {
                    fprintf(stderr, "flag never arrived\n");
                    exit(1);
                }
            }
        }
    };
    const double t_flag = median_us(reps, [&] {
        ++seq;
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, dflag, seq);
        wait_flag(seq);
    });
    CK(hipStreamSynchronize(s));
    const double t_flag_sync = median_us(reps, [&] {
        ++seq;
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, dflag, seq);
        wait_flag(seq);
        CK(hipStreamSynchronize(s));
    });
    const double t_event = median_us(reps, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CK(hipEventRecord(ev, s));
        CK(hipEventSynchronize(ev));
    });
    const double t_launch = median_us(reps, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    });
    CK(hipStreamSynchronize(s));
    // a query-poll loop instead of the blocking sync
    const double t_query = median_us(reps, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        while (hipStreamQuery(s) == hipErrorNotReady)
        {
        }
    });
    printf("%s empty %.2f lds152 %.2f stage %.2f stage3wg %.2f flag %.2f flag+sync %.2f event %.2f "
           "launch %.2f query %.2f (us, median of %d)\n",
           spin ? "spin" : "auto", t_empty, t_lds, t_stage, t_stage3, t_flag, t_flag_sync, t_event,
           t_launch, t_query, reps);
    CK(hipHostFree(hp));
    return 0;
}
