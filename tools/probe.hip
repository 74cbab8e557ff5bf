// tools/probe.hip -- HBM read-ceiling calibration kernels (development tool,
// not part of the product library).  Each probe reads a device buffer with a
// given access pattern and XOR-reduces it (trivial compute), so its rate is
// the memory-side ceiling for that pattern on this MI355X.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p)
{
    if (NT)
    {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *p;
}

// Contiguous: every wave-instruction reads 1 KiB contiguous; U loads in flight.
template <bool NT, int U>
__global__ __launch_bounds__(256) void probe_stream(const uint4* __restrict__ p, uint64_t n16,
                                                    uint32_t* __restrict__ sink)
{
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t nth = uint64_t(gridDim.x) * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + (U - 1) * nth < n16; i += U * nth)
    {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(p + i + u * nth);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += nth) acc ^= ld<NT>(p + i).x;
    if (acc == 0x12345678u) sink[tid & 1023] = acc;
}

// The fixed kernel's access pattern: 8-lane teams, 128-B rows, record stride
// 4 KiB, 16 loads per lane per step, persistent grid of 1024-thread blocks.
template <bool NT>
__global__ __launch_bounds__(1024, 1) void probe_team(const uint8_t* __restrict__ base,
                                                      uint64_t count, uint32_t* __restrict__ sink,
                                                      uint32_t skew = 0)
{
    base += skew;
    const uint32_t tl = threadIdx.x & 7u;
    const uint64_t team = (uint64_t(blockIdx.x) * 1024 + threadIdx.x) / 8;
    const uint64_t nteams = uint64_t(gridDim.x) * 1024 / 8;
    uint32_t acc = 0;
    for (uint64_t rec = team; rec < count; rec += nteams)
    {
        const uint8_t* r = base + rec * 4096 + tl * 16;
        for (int g = 0; g < 4; g += 2)
        {
            uint4 v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                v[k] = ld<NT>(reinterpret_cast<const uint4*>(r + g * 1024 + k * 128));
#pragma unroll
            for (int k = 0; k < 16; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// TEAM-lane teams: rows of 16*TEAM bytes, record stride 4 KiB, 16 loads per step.
template <int TEAM>
__global__ __launch_bounds__(1024, 1) void probe_teamN(const uint8_t* __restrict__ base,
                                                       uint64_t count, uint32_t* __restrict__ sink)
{
    constexpr int ROW = 16 * TEAM;
    const uint32_t tl = threadIdx.x & (TEAM - 1);
    const uint64_t team = (uint64_t(blockIdx.x) * 1024 + threadIdx.x) / TEAM;
    const uint64_t nteams = uint64_t(gridDim.x) * 1024 / TEAM;
    uint32_t acc = 0;
    for (uint64_t rec = team; rec < count; rec += nteams)
    {
        const uint8_t* r = base + rec * 4096 + tl * 16;
        for (int g = 0; g < 4096 / ROW; g += 16)
        {
            uint4 v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                v[k] = ld<true>(reinterpret_cast<const uint4*>(r + (g + k) * ROW));
#pragma unroll
            for (int k = 0; k < 16; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}


// The team pattern with each cache-policy flag set on the 16-B loads (inline
// asm: the compiler does not track these loads, so an explicit vmcnt(0)
// precedes the use).
#define MI_PROBE_POLICY(NAME, FLAGS)                                                             \
    __global__ __launch_bounds__(1024, 1) void NAME(const uint8_t* __restrict__ base,            \
                                                    uint64_t count, uint32_t* __restrict__ sink) \
    {                                                                                            \
        const uint32_t tl = threadIdx.x & 7;                                                     \
        const uint64_t team = (uint64_t(blockIdx.x) * 1024 + threadIdx.x) / 8;                   \
        const uint64_t nteams = uint64_t(gridDim.x) * 1024 / 8;                                  \
        uint32_t acc = 0;                                                                        \
        for (uint64_t rec = team; rec < count; rec += nteams)                                    \
        {                                                                                        \
            const uint8_t* r = base + rec * 4096 + tl * 16;                                      \
            for (int g = 0; g < 4; g += 2)                                                       \
            {                                                                                    \
                u32x4 v[16];                                                                     \
                _Pragma("unroll") for (int k = 0; k < 16; ++k)                                   \
                    asm volatile("global_load_dwordx4 %0, %1, off " FLAGS                        \
                                 : "=v"(v[k]) : "v"(r + g * 1024 + k * 128) : "memory");          \
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                 \
                _Pragma("unroll") for (int k = 0; k < 16; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w; \
            }                                                                                    \
        }                                                                                        \
        if (acc == 0x12345678u) sink[threadIdx.x] = acc;                                         \
    }
MI_PROBE_POLICY(probe_pol_none, "")
MI_PROBE_POLICY(probe_pol_nt, "nt")
MI_PROBE_POLICY(probe_pol_sc1, "sc1")
MI_PROBE_POLICY(probe_pol_sc0sc1, "sc0 sc1")
MI_PROBE_POLICY(probe_pol_ntsc1, "sc1 nt")
MI_PROBE_POLICY(probe_pol_ntsc0sc1, "sc0 sc1 nt")
MI_PROBE_POLICY(probe_pol_sc0nt, "sc0 nt")
MI_PROBE_POLICY(probe_pol_sc0, "sc0")

// The fixed kernel's pipeline with no compute: D groups of 8 rows in flight
// per team, each consumed (XOR) when it lands (vmcnt(8 (D - 1))) and its
// buffer refilled with the group D ahead (records strided by the team count,
// 4 groups per 4 KiB record).  Explicit asm loads + waits, the waits tied to
// the consumed registers so nothing is hoisted above them.
template <int D>
__global__ __launch_bounds__(1024, 1) void probe_pipe(const uint8_t* __restrict__ base,
                                                      uint64_t count, uint32_t* __restrict__ sink)
{
    const uint32_t tl = threadIdx.x & 7;
    const uint64_t team = (uint64_t(blockIdx.x) * 1024 + threadIdx.x) / 8;
    const uint64_t nteams = uint64_t(gridDim.x) * 1024 / 8;
    const uint64_t recs = (count - (team & ~uint64_t(7)) + nteams - 1) / nteams;  // per team
    const uint64_t ngroups = recs * 4;
    auto gaddr = [&](uint64_t q) {
        uint64_t rec = team + (q >> 2) * nteams;
        if (rec >= count) rec = count - 1;
        return base + rec * 4096 + (q & 3) * 1024 + tl * 16;
    };
    u32x4 buf[D][8];
    uint32_t acc = 0;
#pragma unroll
    for (int d = 0; d < D; ++d)
    {
        const uint8_t* p = gaddr(d);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(buf[d][k]) : "v"(p + k * 128) : "memory");
    }
    for (uint64_t q = 0; q < ngroups; q += D)
    {
#pragma unroll
        for (int d = 0; d < D; ++d)
        {
            asm volatile("s_waitcnt vmcnt(%8)"
                         : "+v"(buf[d][0]), "+v"(buf[d][1]), "+v"(buf[d][2]), "+v"(buf[d][3]),
                           "+v"(buf[d][4]), "+v"(buf[d][5]), "+v"(buf[d][6]), "+v"(buf[d][7])
                         : "n"(8 * (D - 1)) : "memory");
#pragma unroll
            for (int k = 0; k < 8; ++k) acc ^= buf[d][k].x ^ buf[d][k].y ^ buf[d][k].z ^ buf[d][k].w;
            const uint8_t* p = gaddr(q + d + D);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(buf[d][k]) : "v"(p + k * 128) : "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// probe_pipe<2> with an XCD-contiguous record map: workgroups are dealt to
// the 8 XCDs round-robin (b % 8), so workgroup b is renumbered to
// (b % 8) * (grid / 8) + b / 8 and each XCD sweeps one contiguous eighth of
// the records instead of interleaved 128-record stretches.
__global__ __launch_bounds__(1024, 1) void probe_pipe_xcd(const uint8_t* __restrict__ base,
                                                          uint64_t count, uint32_t* __restrict__ sink)
{
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t vb = (b % 8) * (G / 8) + b / 8;
    const uint32_t tl = threadIdx.x & 7;
    const uint64_t team = (uint64_t(vb) * 1024 + threadIdx.x) / 8;
    const uint64_t nteams = uint64_t(G) * 1024 / 8;
    // contiguous: team t owns records [t * per, (t + 1) * per)
    const uint64_t per = count / nteams;
    u32x4 buf[2][8];
    uint32_t acc = 0;
    auto gaddr = [&](uint64_t q) {
        uint64_t rec = team * per + (q >> 2);
        if (rec >= count) rec = count - 1;
        return base + rec * 4096 + (q & 3) * 1024 + tl * 16;
    };
    const uint64_t ngroups = per * 4;
#pragma unroll
    for (int d = 0; d < 2; ++d)
    {
        const uint8_t* p = gaddr(d);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(buf[d][k]) : "v"(p + k * 128) : "memory");
    }
    for (uint64_t q = 0; q < ngroups; q += 2)
    {
#pragma unroll
        for (int d = 0; d < 2; ++d)
        {
            asm volatile("s_waitcnt vmcnt(8)"
                         : "+v"(buf[d][0]), "+v"(buf[d][1]), "+v"(buf[d][2]), "+v"(buf[d][3]),
                           "+v"(buf[d][4]), "+v"(buf[d][5]), "+v"(buf[d][6]), "+v"(buf[d][7])
                         :: "memory");
#pragma unroll
            for (int k = 0; k < 8; ++k) acc ^= buf[d][k].x ^ buf[d][k].y ^ buf[d][k].z ^ buf[d][k].w;
            const uint8_t* p = gaddr(q + d + 2);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(buf[d][k]) : "v"(p + k * 128) : "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

}  // namespace

extern "C" float probe_run(int which, const void* buf, uint64_t bytes, int grid, int reps,
                           uint32_t* sink)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const uint4* p = static_cast<const uint4*>(buf);
    const uint64_t n16 = bytes / 16;
    auto launch = [&] {
        switch (which)
        {
            case 0: hipLaunchKernelGGL((probe_stream<false, 8>), dim3(grid), dim3(256), 0, 0, p, n16, sink); break;
            case 1: hipLaunchKernelGGL((probe_stream<true, 8>), dim3(grid), dim3(256), 0, 0, p, n16, sink); break;
            case 2: hipLaunchKernelGGL((probe_stream<false, 16>), dim3(grid), dim3(256), 0, 0, p, n16, sink); break;
            case 3: hipLaunchKernelGGL((probe_team<false>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096, sink, 0u); break;
            case 4: hipLaunchKernelGGL((probe_team<true>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096, sink, 0u); break;
            case 5: hipLaunchKernelGGL((probe_team<true>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096 - 1, sink, 16u); break;
            case 6: hipLaunchKernelGGL((probe_team<true>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096 - 1, sink, 64u); break;
            case 7: hipLaunchKernelGGL((probe_team<true>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096 - 1, sink, 80u); break;
            case 8: hipLaunchKernelGGL((probe_teamN<4>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096, sink); break;
            case 9: hipLaunchKernelGGL((probe_teamN<8>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096, sink); break;
            case 10: hipLaunchKernelGGL((probe_teamN<16>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096, sink); break;
            case 11: hipLaunchKernelGGL((probe_teamN<2>), dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096, sink); break;
#define MI_CASE(N, K) case N: hipLaunchKernelGGL(K, dim3(grid), dim3(1024), 0, 0, static_cast<const uint8_t*>(buf), bytes / 4096, sink); break;
            MI_CASE(20, probe_pol_none) MI_CASE(21, probe_pol_nt) MI_CASE(22, probe_pol_sc1)
            MI_CASE(23, probe_pol_sc0sc1) MI_CASE(24, probe_pol_ntsc1) MI_CASE(25, probe_pol_ntsc0sc1)
            MI_CASE(26, probe_pol_sc0nt) MI_CASE(27, probe_pol_sc0)
            MI_CASE(30, probe_pipe<1>) MI_CASE(31, probe_pipe<2>) MI_CASE(32, probe_pipe<3>)
            MI_CASE(33, probe_pipe_xcd)
#undef MI_CASE
        }
    };
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms / reps;
}
