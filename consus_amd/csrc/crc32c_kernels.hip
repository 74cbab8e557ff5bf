// consus_amd/csrc/crc32c_kernels.hip -- CDNA4 (gfx950) CRC-32C kernels.
//
// Re-implements the per-record checksum of consus::crc32c
// (common/crc32c.h:40-41, common/crc32c.cc:122-126) for batches of
// independent durable-log records (txman/durable_log.cc:215-218).
// Bit-exact with the reference; parity tests in tests/test_gpu_parity.py.
//
// Work decomposition:
//   * a "team" of 8 lanes owns one record (or one 4 KiB chunk of one);
//     a row is 128 contiguous bytes, 16 B per lane (global_load_dwordx4),
//     so each wave-wide load moves 8 full 128-B lines;
//   * each lane keeps 4 independent raw-CRC chains V_q, one per dword of its
//     16-B column, with stride 32 dwords: V <- Z_128(V) ^ d.  Z_128 is applied
//     with 4 lookups into "fold" tables staged in LDS in a bank-private layout
//     (each of the 32 lanes of a ds_read_b32 group owns its own bank, so the
//     lookups are conflict-free whatever the data), addressed by ONE v_perm_b32
//     per lookup;
//   * at the end of a record the 32 chains of a team are folded with the
//     slice-by-16 tables and a 3-level lane tree (Z_16, Z_32, Z_64).
// No MFMA: this is a GF(2) scan; the bound is HBM read bandwidth.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "crc32c_kernels.h"

namespace mi_crc {

extern __shared__ __attribute__((aligned(16))) char smem[];

// The record kernels declare no static LDS, so the dynamic image starts at
// LDS address 0 (checked by tests/test_build.py on the ISA metadata) and a
// table byte offset IS the ds_read address: no base add per lookup.
typedef __attribute__((address_space(3))) const uint32_t lds_u32;

__device__ __forceinline__ uint32_t lds32(uint32_t byte_addr)
{
    return *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(byte_addr));
}

// a ^ b ^ c in one CDNA4 v_bitop3_b32 (truth table 0x96); hipcc does not
// form it from two v_xor_b32 by itself.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Stage the table image into LDS: G^{128} replicated 32x bank-private, then
// T_0..T_15, G^{32}, G^{64} verbatim.  Byte address of G^{128}_t[b] for the
// lane whose ds_read_b32 group position is c (= lane & 31):
//   (t >> 1) * 65536 + b * 256 + (t & 1) * 128 + c * 4   ->  bank == c.
// Every record kernel runs kBlock threads: all loads are issued first, then
// all stores (one L2 round trip per thread, not one per iteration).  The two
// halves are separate so that a kernel can issue the loads early and store
// later (the sorted kernel: its LDS holds the descriptor list until then).
struct TableRegs
{
    static constexpr uint32_t NM = 1024u * 8u / kBlock;   // G^{128} entries x 8 quads
    static constexpr uint32_t NT = (4096u + 2048u) / 4u;  // T_0..15, G^32, G^64 as uint4
    static constexpr uint32_t NTI = (NT + kBlock - 1) / kBlock;
    uint32_t v[NM];
    uint4 t[NTI];
};
static_assert(1024u * 8u % kBlock == 0, "table staging shape");

__device__ __forceinline__ void stage_tables_load(TableRegs& r, const uint32_t* __restrict__ g)
{
    const uint4* src = reinterpret_cast<const uint4*>(g + kTabT);
#pragma unroll
    for (uint32_t k = 0; k < TableRegs::NM; ++k) r.v[k] = g[kTabMain + ((threadIdx.x + k * kBlock) >> 3)];
#pragma unroll
    for (uint32_t k = 0; k < TableRegs::NTI; ++k)
    {
        const uint32_t i = threadIdx.x + k * kBlock;
        r.t[k] = i < TableRegs::NT ? src[i] : make_uint4(0, 0, 0, 0);
    }
}

__device__ __forceinline__ void stage_tables_store(const TableRegs& r)
{
#pragma unroll
    for (uint32_t k = 0; k < TableRegs::NM; ++k)
    {
        const uint32_t i = threadIdx.x + k * kBlock;
        const uint32_t e = i >> 3;          // t * 256 + b
        const uint32_t c4 = (i & 7u) * 4u;  // first of 4 consecutive copies
        const uint32_t tb = e >> 8, b = e & 255u;
        const uint32_t addr = (tb >> 1) * 65536u + b * 256u + (tb & 1u) * 128u + c4 * 4u;
        *reinterpret_cast<uint4*>(smem + kLdsMain + addr) = make_uint4(r.v[k], r.v[k], r.v[k], r.v[k]);
    }
    uint4* dst = reinterpret_cast<uint4*>(smem + kLdsT);
#pragma unroll
    for (uint32_t k = 0; k < TableRegs::NTI; ++k)
    {
        const uint32_t i = threadIdx.x + k * kBlock;
        if (i < TableRegs::NT) dst[i] = r.t[k];
    }
    __syncthreads();
}

__device__ __forceinline__ void stage_tables(const uint32_t* __restrict__ g)
{
    TableRegs r;
    stage_tables_load(r, g);
    stage_tables_store(r);
}

// Lane info for the v_perm address builder: byte0 = c*4, byte1 = c*4 + 128,
// byte2 = 0, byte3 = 1 (the 64 KiB half for tables 2 and 3).
__device__ __forceinline__ uint32_t lane_info()
{
    const uint32_t c4 = (threadIdx.x & 31u) * 4u;
    return c4 | ((c4 + 128u) << 8) | (1u << 24);
}

// Z_128 lookups (row_update): v_perm_b32 builds {lane byte, v.byte_t, half
// bit, 0} = the LDS byte address of G^{128}_t[v.byte_t] in this lane's
// private bank.  Selector bytes 0-3 pick v (src1), 4-7 pick li (src0),
// 0x0C gives 0x00.

// Z_{4m}(v) from the slice-by-16 tables: byte j uses T_{4m-1-j}.
template <int M>
__device__ __forceinline__ uint32_t zT(uint32_t v)
{
    constexpr uint32_t k0 = kLdsT + (4 * M - 1) * 1024;
    return xor3(lds32(k0 + ((v & 0xFFu) << 2)), lds32(k0 - 1024 + ((v >> 6) & 0x3FCu)),
                lds32(k0 - 2048 + ((v >> 14) & 0x3FCu))) ^
           lds32(k0 - 3072 + ((v >> 22) & 0x3FCu));
}

// Z_n(v) from a G^n table set at LDS byte offset `base` (byte j uses G_j).
__device__ __forceinline__ uint32_t zG(uint32_t base, uint32_t v)
{
    return xor3(lds32(base + ((v & 0xFFu) << 2)), lds32(base + 1024 + ((v >> 6) & 0x3FCu)),
                lds32(base + 2048 + ((v >> 14) & 0x3FCu))) ^
           lds32(base + 3072 + ((v >> 22) & 0x3FCu));
}

// Z_n(v) for a per-lane n in 0..16 from the slice-by-16 tables: byte j of v
// leaves the register after n - j zero bytes (T_{n-1-j}), bytes j >= n shift
// down by n bytes.
__device__ __forceinline__ uint32_t zT_n(uint32_t v, uint32_t n)
{
    uint32_t x = n >= 4 ? 0u : v >> (8 * n);
#pragma unroll
    for (int j = 0; j < 4; ++j)
    {
        const int32_t t = int32_t(n) - 1 - j;
        const uint32_t e = lds32(kLdsT + uint32_t(max(t, 0)) * 1024u + ((v >> (8 * j)) & 0xFFu) * 4u);
        x ^= t >= 0 ? e : 0u;
    }
    return x;
}

// One 128-B row: each lane folds its 16 bytes into its four chains.
// All 16 addresses, then all 16 lookups, then the XORs, so a wave keeps 16
// conflict-free ds_read_b32 in flight per row.
__device__ __forceinline__ void row_update(uint32_t (&V)[4], const uint4 d, uint32_t li)
{
    uint32_t a[16], r[16];
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
        a[4 * q + 0] = __builtin_amdgcn_perm(li, V[q], 0x0C060004u);
        a[4 * q + 1] = __builtin_amdgcn_perm(li, V[q], 0x0C060105u);
        a[4 * q + 2] = __builtin_amdgcn_perm(li, V[q], 0x0C070204u);
        a[4 * q + 3] = __builtin_amdgcn_perm(li, V[q], 0x0C070305u);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
        r[i] = lds32(kLdsMain + a[i]);
    V[0] = xor3(xor3(r[0], r[1], r[2]), r[3], d.x);
    V[1] = xor3(xor3(r[4], r[5], r[6]), r[7], d.y);
    V[2] = xor3(xor3(r[8], r[9], r[10]), r[11], d.z);
    V[3] = xor3(xor3(r[12], r[13], r[14]), r[15], d.w);
}

// The first row of a record meets all-zero chains, whose lookups are all
// G[0] = 0: the update is the row itself (saves the row's 16 lookups, 16
// address builds and 8 XORs: one row in 32 of a 4 KiB record).
__device__ __forceinline__ void row_first(uint32_t (&V)[4], const uint4 d)
{
    V[0] = d.x;
    V[1] = d.y;
    V[2] = d.z;
    V[3] = d.w;
}

// Fold a team's 32 chains into the raw CRC of the team's bytes, assuming the
// last processed row ends exactly at the end of those bytes.  Valid in lane
// (lane & 7) == 0 of the team.  DESIGN.md section 3 (lane-parallel CRC of one row):
//   raw = XOR_L Z_{16(7-L)}( Z16 V0 ^ Z12 V1 ^ Z8 V2 ^ Z4 V3 )_L
// v from lane + N of the same 16-lane DPP row (row_shl:N); a team's lane 0
// (lane 0 or 8 of a row) reads lanes 1..7 of its own team.  A DPP operand
// costs nothing beside its v_xor; __shfl_xor is a ds_bpermute round trip
// (measured: 0.657 vs 0.657-0.665 ms on the headline batch).
template <int N>
__device__ __forceinline__ uint32_t from_lane_up(uint32_t v)
{
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x100 + N, 0xF, 0xF, true));
}

__device__ __forceinline__ uint32_t team_fold(const uint32_t (&V)[4])
{
    const uint32_t x = zT<4>(V[0]) ^ zT<3>(V[1]) ^ zT<2>(V[2]) ^ zT<1>(V[3]);
    const uint32_t y = zT<4>(x) ^ from_lane_up<1>(x);
    const uint32_t w = zG(kLdsZ32, y) ^ from_lane_up<2>(y);
    return zG(kLdsZ64, w) ^ from_lane_up<4>(w);
}

// The same fold without LDS tables (the headline kernel's): every Z_n of the fold is
// six 64-entry tables of 6-bit slices (kTabLane), each held one entry per lane
// in a VGPR and read with ds_bpermute, a crossbar permute that touches no LDS
// bank.  The shared slice-by-16 tables cannot be made bank-private (24 KiB of
// them beside the 128 KiB G^{128} image), so their random lookups conflict
// 3.5-way on average; these cannot conflict.  The permute uses address bits
// 7:2 only, so each slice's address is one shift.  Costs 36 VGPRs.
struct LaneTabs
{
    uint32_t t[6 * kLaneOps];
};
// the first N of the 42 (36: the fold's six operators; 42: and Z_128)
template <int N = 36>
__device__ __forceinline__ void load_lane_tabs(LaneTabs& L, const uint32_t* __restrict__ tables)
{
    const uint32_t* p = tables + kTabLane + (threadIdx.x & 63u);
#pragma unroll
    for (int k = 0; k < N; ++k) L.t[k] = p[k * 64];
}
__device__ __forceinline__ uint32_t bperm(uint32_t addr, uint32_t tab)
{
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(addr), int(tab)));
}
template <int K>
__device__ __forceinline__ uint32_t zL(const LaneTabs& L, uint32_t v)
{
    const uint32_t* z = L.t + 6 * K;
    return xor3(xor3(bperm(v << 2, z[0]), bperm(v >> 4, z[1]), bperm(v >> 10, z[2])),
                bperm(v >> 16, z[3]), bperm(v >> 22, z[4])) ^
           bperm(v >> 28, z[5]);
}
// Every lane of the wave must be active (ds_bpermute reads inactive lanes as 0).
__device__ __forceinline__ uint32_t team_fold_lane(const uint32_t (&V)[4], const LaneTabs& L)
{
    const uint32_t x = zL<0>(L, V[0]) ^ zL<1>(L, V[1]) ^ zL<2>(L, V[2]) ^ zL<3>(L, V[3]);
    const uint32_t y = zL<0>(L, x) ^ from_lane_up<1>(x);
    const uint32_t w = zL<4>(L, y) ^ from_lane_up<2>(y);
    return zL<5>(L, w) ^ from_lane_up<4>(w);
}

// The row update through the Z_128 lane tables (no LDS image): six
// permutes per chain instead of four bank-private lookups.  Wave-uniform
// control flow only (inactive lanes would read as 0); `act` keeps the chains
// of a team whose record has ended, `first` starts them.
__device__ __forceinline__ void row_update_lane(uint32_t (&V)[4], const uint4 d, const LaneTabs& L,
                                                bool act, bool first)
{
    const uint32_t n0 = zL<6>(L, V[0]) ^ d.x, n1 = zL<6>(L, V[1]) ^ d.y;
    const uint32_t n2 = zL<6>(L, V[2]) ^ d.z, n3 = zL<6>(L, V[3]) ^ d.w;
    V[0] = act ? (first ? d.x : n0) : V[0];
    V[1] = act ? (first ? d.y : n1) : V[1];
    V[2] = act ? (first ? d.z : n2) : V[2];
    V[3] = act ? (first ? d.w : n3) : V[3];
}

// Record bytes are read exactly once: non-temporal loads (global_load_dwordx4
// ... nt) keep them from displacing L2/MALL lines.  Measured on MI355X with
// this kernel's access pattern (tools/probe.py): 7.07 TB/s nt vs 6.19 TB/s
// with default-policy loads.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4_t make_u32x4(const uint4& v)
{
    u32x4_t r = {v.x, v.y, v.z, v.w};
    return r;
}

__device__ __forceinline__ uint4 load16(const uint8_t* p)
{
    // explicitly global: a pointer rebuilt from an integer (Item::bits) would
    // otherwise be FLAT, and FLAT loads also count in lgkmcnt, so every wait
    // for an LDS lookup would drain the prefetched rows too
    typedef const __attribute__((address_space(1))) u32x4_t* gptr;
    const u32x4_t v = __builtin_nontemporal_load((gptr)(uintptr_t)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// A record's first and last rows share their 128-B lines with the
// neighbouring records (packed back to back), which another team reads later.
// The sorted kernel reads a group's edge rows (its first rows, up to the last
// row in which an item starts, and its last row) with the default policy
// instead of nt.  Round 4 A/B on configs[2], 3 interleaved rounds on one box:
// 0.786-0.806 ms against 0.827-0.828 with every row nt; PMC FETCH_SIZE is
// unchanged (2.475e6 against 2.478e6 KB x 2 per step), so the gain is in the
// latency of those rows, not in HBM bytes (profiles/r04_sorted_edge_loads_ab.txt).
__device__ __forceinline__ uint4 load16_edge(const uint8_t* p)
{
    typedef const __attribute__((address_space(1))) u32x4_t* gptr;
    const u32x4_t v = *((gptr)(uintptr_t)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// ---------------------------------------------------------------------------
// Fixed-stride batches: record i = [base + i*stride, +len), base and stride
// 16-byte aligned, len a multiple of 16 (other shapes take the variable path).
// Persistent grid (one 1024-thread workgroup per CU, 152 KiB LDS); team t
// handles records t, t + nteams, ...  Each step issues two groups (16 KiB
// per wave, 16 dwordx4 per lane) and consumes them in the same step, so the
// compiler's vmcnt accounting stays exact (no loop-carried loads, which it
// would drain with vmcnt(0)); 16 waves per CU keep >= 128 KiB in flight.
// ---------------------------------------------------------------------------
template <bool PADDED, bool INITS>
__global__ __launch_bounds__(kBlock, 1) void crc32c_fixed_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, uint32_t len, uint32_t groups,
    const uint32_t* __restrict__ inits, uint64_t init_stride, uint64_t count,
    uint32_t* __restrict__ out, const uint32_t* __restrict__ tables)
{
    stage_tables(tables);

    const uint32_t tl = threadIdx.x & (kTeam - 1);
    const uint32_t li = lane_info();
    const uint64_t team = (uint64_t(blockIdx.x) * kBlock + threadIdx.x) / kTeam;
    const uint64_t nteams = uint64_t(gridDim.x) * kBlock / kTeam;
    const uint64_t team0 = team & ~uint64_t(7);  // first team of this wave
    const uint64_t iters = team0 < count ? (count - team0 + nteams - 1) / nteams : 0;

    // Byte offset (from the record start) of this lane's column in row 0 of
    // group 0; negative in the leading pad when len is not a multiple of 1 KiB.
    const int32_t pad = int32_t(groups * kGroupBytes) - int32_t(len);
    const int32_t col0 = int32_t(tl) * 16 - pad;
    // Row/lane holding the record's first dword (where ~init is folded in).
    const uint32_t r0 = uint32_t(pad) / kRowBytes;
    const bool init_lane = tl == (uint32_t(pad) % kRowBytes) / 16u;

    for (uint64_t it = 0; it < iters; ++it)
    {
        // Teams past the end re-hash the last record (loads stay
        // unconditional) and do not store.
        const uint64_t rec_raw = team + it * nteams;
        const uint64_t rec = rec_raw < count ? rec_raw : count - 1;
        const uint8_t* rbase = base + rec * stride;
        uint32_t init_word = INITS ? inits[rec * init_stride] : 0u;  // inverted at use
        uint32_t V[4] = {0, 0, 0, 0};
        for (uint32_t g = 0; g < groups; g += 2)
        {
            // Both groups are always loaded (a lone group re-reads itself) so
            // the compiler counts 16 outstanding loads at the first use.
            const bool two = g + 1 < groups;
            const uint32_t gb = two ? g + 1 : g;
            uint4 A[kGroupRows], B[kGroupRows];
#pragma unroll
            for (int r = 0; r < kGroupRows; ++r)
            {
                const int32_t o = col0 + int32_t(g) * kGroupBytes + r * kRowBytes;
                A[r] = load16(PADDED && o < 0 ? rbase : rbase + o);
            }
#pragma unroll
            for (int r = 0; r < kGroupRows; ++r)
            {
                const int32_t o = col0 + int32_t(gb) * kGroupBytes + r * kRowBytes;
                B[r] = load16(PADDED && o < 0 ? rbase : rbase + o);
            }
            __builtin_amdgcn_sched_barrier(0);  // all 16 loads issue before any use
            // keep the init word's wait behind the data loads (no hoisting)
            if (INITS) asm volatile("" : "+v"(init_word));
            if (PADDED)
            {
#pragma unroll
                for (int r = 0; r < kGroupRows; ++r)
                {
                    const int32_t o = col0 + int32_t(g) * kGroupBytes + r * kRowBytes;
                    if (o < 0) A[r] = make_uint4(0, 0, 0, 0);
                }
            }
            const uint32_t x = (g == 0 && init_lane) ? ~init_word : 0u;  // ~0 = 0xFFFFFFFF for init 0
            if (PADDED)
            {
#pragma unroll
                for (int r = 0; r < kGroupRows; ++r)
                    if (uint32_t(r) == r0) A[r].x ^= x;
            }
            else
                A[0].x ^= x;
#pragma unroll
            for (int r = 0; r < kGroupRows; ++r) row_update(V, A[r], li);
            if (two)
            {
#pragma unroll
                for (int r = 0; r < kGroupRows; ++r) row_update(V, B[r], li);
            }
        }
        const uint32_t raw = team_fold(V);
        if (tl == 0 && rec_raw < count) out[rec] = ~raw;
    }
}

// Software-pipelined fast path for records of exactly G KiB (G even), the
// shape of the headline batch (4 KiB).  A record's rows are loaded in
// sub-groups of Q rows into NB rotating buffers: NB - 1 sub-groups (of this
// record or the next one) are in flight while one is folded, so a wave
// always has (NB - 1) * Q KiB of loads outstanding, Q * NB rows of buffer
// VGPRs.  The loop body is straight-line per record and every buffer's role
// is the same in every record (NB divides the sub-groups per record), so the
// loop-carried loads are the same on every path into the header and the
// compiler's vmcnt accounting stays exact.
// Shape (MI355X, 1M x 4 KiB, tools/ab.py, 6 interleaved rounds per build,
// medians): Q = 1 row, NB = 4 (71 VGPRs) 0.640-0.648 ms; Q = 1, NB = 8
// 0.642-0.648; Q = 1, NB = 2 0.645-0.652; Q = 2, NB = 4 0.651-0.657; Q = 4,
// NB = 4 0.655-0.666; the former Q = 8, NB = 2 (two 8-row groups, 126 VGPRs)
// 0.652-0.669.  Issuing one row ahead of each row's folding spreads the loads
// evenly through the lookups; the depth beyond 3 rows changes nothing.
// Dropping the sched_barrier costs 1 % (Q = 1, NB = 4: 0.649-0.655).
// Issuing the first record's rows before the table staging was neutral
// (0.636-0.658 vs 0.634-0.658 ms, 6 interleaved rounds).
constexpr int kPipeRows = 1, kPipeBufs = 4;
template <int G, bool INITS>
__device__ __forceinline__ void fixed_pipe(const uint8_t* __restrict__ base, uint64_t stride,
                                           const uint32_t* __restrict__ inits,
                                           uint64_t init_stride, uint64_t count,
                                           uint32_t* __restrict__ out,
                                           const uint32_t* __restrict__ tables)
{
    constexpr int Q = kPipeRows, NB = kPipeBufs;
    constexpr int SG = G * kGroupRows / Q;  // sub-groups per record
    static_assert(G * kGroupRows % Q == 0 && SG % NB == 0 && NB >= 2, "pipeline shape");
    const uint32_t tl = threadIdx.x & (kTeam - 1);
    const uint32_t li = lane_info();
    const uint64_t team = (uint64_t(blockIdx.x) * kBlock + threadIdx.x) / kTeam;
    const uint64_t nteams = uint64_t(gridDim.x) * kBlock / kTeam;
    const uint64_t team0 = team & ~uint64_t(7);  // the wave's first team: iters is wave-uniform
    const uint64_t iters = team0 < count ? (count - team0 + nteams - 1) / nteams : 0;

    auto rec_of = [&](uint64_t it) {
        const uint64_t r = team + it * nteams;
        return r < count ? r : count - 1;
    };
    auto load_sub = [&](uint4 (&buf)[Q], uint64_t rec, int q) {
        const uint8_t* p = base + rec * stride + tl * 16 + q * Q * kRowBytes;
#pragma unroll
        for (int r = 0; r < Q; ++r) buf[r] = load16(p + r * kRowBytes);
    };

    uint4 bufs[NB][Q];
    uint64_t rec = iters ? rec_of(0) : 0;
    uint32_t init_word = 0;
    stage_tables(tables);  // every thread reaches the barrier
    LaneTabs lt;
    load_lane_tabs(lt, tables);
    if (iters == 0) return;
    if (INITS) init_word = inits[rec * init_stride];
#pragma unroll
    for (int q = 0; q < NB - 1; ++q) load_sub(bufs[q], rec, q);
    for (uint64_t it = 0; it < iters; ++it)
    {
        const uint64_t next = rec_of(it + 1);
        uint32_t V[4] = {0, 0, 0, 0};
        uint32_t next_init = 0;
#pragma unroll
        for (int q = 0; q < SG; ++q)
        {
            const int qa = q + NB - 1;  // the sub-group issued now
            if (qa < SG)
                load_sub(bufs[qa % NB], rec, qa);
            else
            {
                load_sub(bufs[qa % NB], next, qa - SG);
                if (INITS && qa == SG) next_init = inits[next * init_stride];
            }
            // Keep the loads ahead of this sub-group's folding (the scheduler
            // would otherwise sink them into it to save registers).
            __builtin_amdgcn_sched_barrier(0);
            uint4(&cur)[Q] = bufs[q % NB];
            if (q == 0) cur[0].x ^= tl == 0 ? ~init_word : 0u;
#pragma unroll
            for (int r = 0; r < Q; ++r)
            {
                if (q == 0 && r == 0)
                    row_first(V, cur[0]);
                else
                    row_update(V, cur[r], li);
            }
        }
        const uint32_t raw = team_fold_lane(V, lt);
        if (tl == 0 && team + it * nteams < count) out[rec] = ~raw;
        rec = next;
        if (INITS) init_word = next_init;
    }
}

template <int G, bool INITS>
__global__ __launch_bounds__(kBlock, 1) void crc32c_fixed_pipe_kernel(
    const uint8_t* __restrict__ base, uint64_t stride, const uint32_t* __restrict__ inits,
    uint64_t init_stride, uint64_t count, uint32_t* __restrict__ out,
    const uint32_t* __restrict__ tables)
{
    fixed_pipe<G, INITS>(base, stride, inits, init_stride, count, out, tables);
}

// The same code over launch_single's 4 KiB chunks of one record, under a
// name of its own so that a profile tells it apart from record batches.
__global__ __launch_bounds__(kBlock, 1) void crc32c_span_chunk_kernel(
    const uint8_t* __restrict__ base, uint64_t count, uint32_t* __restrict__ out,
    const uint32_t* __restrict__ tables)
{
    fixed_pipe<4, false>(base, kChunk, tables + kTabZero, 0, count, out, tables);
}

hipError_t launch_fixed(const void* base, uint64_t stride, uint32_t len, const uint32_t* inits,
                        uint64_t count, uint32_t* out, const uint32_t* tables, int grid,
                        hipStream_t stream)
{
    const uint32_t* zero_word = tables + kTabZero;
    if (count == 0) return hipSuccess;
    const uint32_t groups = (len + kGroupBytes - 1) / kGroupBytes;
    const uint64_t need = (count + (kBlock / kTeam) - 1) / (kBlock / kTeam);
    if (uint64_t(grid) > need) grid = int(need);
    const bool padded = len != groups * kGroupBytes;
    const uint32_t* ipp = inits ? inits : tables + kTabZero;
    const uint64_t isp = inits ? 1 : 0;
    const uint8_t* bp = static_cast<const uint8_t*>(base);
#define MI_LAUNCH_PIPE(GG, I)                                                                 \
    hipLaunchKernelGGL((crc32c_fixed_pipe_kernel<GG, I>), dim3(grid), dim3(kBlock), kLdsBytes, \
                       stream, bp, stride, ipp, isp, count, out, tables)
    if (!padded && (groups == 4 || groups == 2))
    {
        if (groups == 4 && inits)
            MI_LAUNCH_PIPE(4, true);
        else if (groups == 4)
            MI_LAUNCH_PIPE(4, false);
        else if (inits)
            MI_LAUNCH_PIPE(2, true);
        else
            MI_LAUNCH_PIPE(2, false);
        return hipGetLastError();
    }
#undef MI_LAUNCH_PIPE
    const uint32_t* ip = inits ? inits : zero_word;
    const uint64_t is = inits ? 1 : 0;
    const uint8_t* b = static_cast<const uint8_t*>(base);
#define MI_LAUNCH_FIXED(P, I)                                                                   \
    hipLaunchKernelGGL((crc32c_fixed_kernel<P, I>), dim3(grid), dim3(kBlock), kLdsBytes, stream, \
                       b, stride, len, groups, ip, is, count, out, tables)
    if (padded && inits)
        MI_LAUNCH_FIXED(true, true);
    else if (padded)
        MI_LAUNCH_FIXED(true, false);
    else if (inits)
        MI_LAUNCH_FIXED(false, true);
    else
        MI_LAUNCH_FIXED(false, false);
#undef MI_LAUNCH_FIXED
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Variable-length batches: plan -> pieces -> finalize.
//   plan:     a record [a, E) is cut at the multiples of 4 KiB of the address
//             space into n pieces (first, n-2 interior full chunks, last);
//             pieces are bucketed by their 1-KiB group count (4 first) so the
//             8 teams of a wave get equal work.  Every team window is 128-B
//             aligned in memory (a 16-B skew of the rows costs 16 % of HBM
//             bandwidth, tools/probe.py).
//   pieces:   one team per piece -> R = raw(window) = Z_m(raw(piece)).
//   finalize: one thread per record: Horner from ~init over its pieces,
//             undoing the last piece's m trailing zeros with
//             Z_{-m} = Z_{-128} o Z_{128-m}; records < 32 B byte-serially.
// ---------------------------------------------------------------------------
// Plan blocks: 1024 threads x 4 consecutive records.  The per-block bin
// counts live in blk[bin * nblocks + block]; the plan header follows them
// (plan_hdr): bin starts [0, kBins), total items, long-record count.
constexpr uint32_t kPlanThreads = 1024;
constexpr uint32_t kPlanPer = 4;
constexpr uint32_t kPlanRecs = kPlanThreads * kPlanPer;
constexpr uint32_t kHdrTotal = kPlanHdrTotal;
constexpr uint32_t kHdrLongs = kBins + 1;
constexpr uint32_t kHdrGrab = kBins + 2;  // chunk kernel's shared-pool cursor
static_assert(kHdrGrab < kPlanHdrWords, "plan header size");

uint32_t var_plan_blocks(uint64_t count)
{
    return uint32_t((count + kPlanRecs - 1) / kPlanRecs);
}

__device__ __forceinline__ uint32_t* plan_hdr_d(uint32_t* blk, uint32_t nblocks)
{
    return blk + kBins * nblocks;
}

struct RecShape
{
    uint64_t a, E;  // record bytes [a, E) (absolute addresses)
    uint64_t k0;    // chunk index of the first piece
    uint32_t n;     // pieces; 0 = short record (finalize hashes it byte-serially)
};

__device__ __forceinline__ RecShape rec_shape(uint64_t a, uint32_t L)
{
    RecShape s{a, a + L, a / kChunk, 0};
    if (L >= uint32_t(kSmallRecord)) s.n = uint32_t((s.E - 1) / kChunk - s.k0 + 1);
    return s;
}

__device__ __forceinline__ uint64_t piece_start(const RecShape& s, uint32_t i)
{
    const uint64_t c = (s.k0 + i) * kChunk;
    return c > s.a ? c : s.a;
}

__device__ __forceinline__ uint64_t piece_end(const RecShape& s, uint32_t i)
{
    const uint64_t c = (s.k0 + i + 1) * kChunk;
    return c < s.E ? c : s.E;
}

__device__ __forceinline__ Item make_item(uint64_t w, uint32_t lenw, uint32_t m)
{
    return Item{((w >> 7) << kItemAddrShift) | (uint64_t(lenw) << kItemLenShift) | m};
}

__device__ __forceinline__ Item piece_item(const RecShape& s, uint32_t i)
{
    const uint64_t ps = piece_start(s, i), pe = piece_end(s, i);
    const uint64_t w = (pe + kRowBytes - 1) & ~uint64_t(kRowBytes - 1);
    return make_item(w, uint32_t(w - ps), uint32_t(w - pe));
}

// Interior piece j (0-based) of a record whose first piece is in chunk k0.
__device__ __forceinline__ Item interior_item(uint64_t k0, uint32_t j)
{
    return make_item((k0 + 2 + j) * kChunk, kChunk, 0);
}

// bins 0, 1, 2 = 4, 3, 2 groups of 8 rows; 3 + (8 - R) = one group, R rows
__device__ __forceinline__ uint32_t piece_bin(const RecShape& s, uint32_t i)
{
    const uint64_t ps = piece_start(s, i), pe = piece_end(s, i);
    const uint64_t w = (pe + kRowBytes - 1) & ~uint64_t(kRowBytes - 1);
    const uint32_t rows = uint32_t((w - (ps & ~uint64_t(kRowBytes - 1))) / kRowBytes);
    return rows > kGroupRows ? 4 - (rows + kGroupRows - 1) / kGroupRows : 3 + (kGroupRows - rows);
}

// One thread's bin counts over its kPlanPer records without dynamically
// indexed arrays: bin 0 in c0, bins 1..10 in 4-bit fields of cn (a record
// adds at most 2 to a bin, so a thread's count is <= 8).
struct ThreadCounts
{
    uint32_t c0 = 0;
    uint64_t cn = 0;
    __device__ void add(uint32_t bin)
    {
        if (bin == 0)
            c0 += 1;
        else
            cn += uint64_t(1) << (4 * (bin - 1));
    }
    // first, interior (bin 0), last
    __device__ void add_record(const RecShape& s)
    {
        if (s.n == 0) return;
        add(piece_bin(s, 0));
        if (s.n >= 2)
        {
            c0 += s.n - 2;
            add(piece_bin(s, s.n - 1));
        }
    }
};

// Bin counts packed for block-wide sums/scans: bin 0 in its own word (a
// block holds < 2^32 pieces of it), bins 1..10 two per word in 16-bit fields
// (<= 8 per thread: <= 8192 per block).
constexpr int kPacked = 6;

__device__ __forceinline__ void pack_counts(const ThreadCounts& t, uint32_t p[kPacked])
{
    p[0] = t.c0;
#pragma unroll
    for (int w = 1; w < kPacked; ++w)
        p[w] = uint32_t((t.cn >> (8 * (w - 1))) & 0xFu) |
               (uint32_t((t.cn >> (8 * (w - 1) + 4)) & 0xFu) << 16);
}

__device__ __forceinline__ void unpack_counts(const uint32_t p[kPacked], uint32_t c[kBins])
{
    c[0] = p[0];
#pragma unroll
    for (int w = 1; w < kPacked; ++w)
    {
        c[2 * w - 1] = p[w] & 0xFFFFu;
        c[2 * w] = p[w] >> 16;
    }
}

__global__ __launch_bounds__(kPlanThreads) void plan_count_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, uint64_t count, uint32_t* __restrict__ blk, uint32_t nblocks)
{
    __shared__ uint32_t sh[kPlanThreads / 64][kPacked];
    const uint64_t r0 = (uint64_t(blockIdx.x) * kPlanThreads + threadIdx.x) * kPlanPer;
    ThreadCounts tc;
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q)
        if (r0 + q < count) tc.add_record(rec_shape(uint64_t(base) + off[r0 + q], len[r0 + q]));
    uint32_t p[kPacked];
    pack_counts(tc, p);
#pragma unroll
    for (int w = 0; w < kPacked; ++w)
        for (int d = 32; d >= 1; d >>= 1) p[w] += __shfl_xor(p[w], d);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (lane == 0)
        for (int w = 0; w < kPacked; ++w) sh[wave][w] = p[w];
    __syncthreads();
    if (threadIdx.x == 0)
    {
        uint32_t t[kPacked] = {};
        for (uint32_t v = 0; v < kPlanThreads / 64; ++v)
            for (int w = 0; w < kPacked; ++w) t[w] += sh[v][w];
        uint32_t bc[kBins];
        unpack_counts(t, bc);
        for (uint32_t b = 0; b < kBins; ++b) blk[b * nblocks + blockIdx.x] = bc[b];
        if (blockIdx.x == 0)
        {
            plan_hdr_d(blk, nblocks)[kHdrLongs] = 0;      // plan_scatter appends
            plan_hdr_d(blk, nblocks)[kHdrGrab] = 0;       // chunk kernel pool cursor
        }
    }
}

// One workgroup turns the bin-major block counts into bases in place: the
// exclusive scan of the flat array [bin][block] is exactly "items of earlier
// bins + items of this bin in earlier blocks".  Tiles of 16K entries are
// staged through LDS (loads and stores coalesced; index padded one word per
// 32 against bank conflicts), each thread scans 16 consecutive entries.  The
// header gets the bin starts and the item total.
constexpr uint32_t kScanPer = 16;
constexpr uint32_t kScanTile = 1024 * kScanPer;

__device__ __forceinline__ uint32_t scan_slot(uint32_t i) { return i + (i >> 5); }

__global__ __launch_bounds__(1024) void plan_scan_kernel(uint32_t* __restrict__ blk,
                                                         uint32_t nblocks)
{
    __shared__ uint32_t tile[kScanTile + kScanTile / 32];
    __shared__ uint32_t sh[16];
    __shared__ uint32_t carry;
    const uint32_t n = kBins * nblocks;
    uint32_t* hdr = plan_hdr_d(blk, nblocks);
    if (threadIdx.x == 0) carry = 0;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    for (uint32_t base = 0; base < n; base += kScanTile)
    {
        const uint32_t cnt = min(kScanTile, n - base);
        for (uint32_t i = threadIdx.x; i < kScanTile; i += 1024)
            tile[scan_slot(i)] = i < cnt ? blk[base + i] : 0u;
        __syncthreads();
        uint32_t v[kScanPer], sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < kScanPer; ++j)
        {
            v[j] = tile[scan_slot(threadIdx.x * kScanPer + j)];
            sum += v[j];
        }
        uint32_t x = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1)
        {
            const uint32_t y = __shfl_up(x, d);
            if (lane >= uint32_t(d)) x += y;
        }
        if (lane == 63) sh[wave] = x;
        __syncthreads();
        uint32_t run = carry + x - sum, tot = 0;
        for (uint32_t w = 0; w < 16; ++w)
        {
            if (w < wave) run += sh[w];
            tot += sh[w];
        }
#pragma unroll
        for (uint32_t j = 0; j < kScanPer; ++j)
        {
            tile[scan_slot(threadIdx.x * kScanPer + j)] = run;
            run += v[j];
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < cnt; i += 1024)
        {
            const uint32_t e = tile[scan_slot(i)];
            blk[base + i] = e;
            if ((base + i) % nblocks == 0) hdr[(base + i) / nblocks] = e;  // bin start
        }
        if (threadIdx.x == 0) carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) hdr[kHdrTotal] = carry;
}

// Each block derives its base in every bin from the per-block counts and
// hands its threads their slots.  Up to kScanFreeBlocks plan blocks (16M
// records) no scan pass runs: wave b < kBins sums bin b over all blocks and
// over the blocks before this one (11 x nblocks words, L2-resident), the bin
// starts are the exclusive scan of the totals, and block 0 publishes the
// plan header.  Larger plans run plan_scan_kernel first (scanned = true: blk
// holds the bases).  Interior runs of every length are written here, by the
// whole wave, 64 items per store; long records (> kLongChunks interior
// pieces) are also listed for the finalize's block-wide fold.
constexpr uint32_t kScanFreeBlocks = 4096;

__global__ __launch_bounds__(kPlanThreads) void plan_scatter_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, uint64_t count, uint32_t* __restrict__ blk,
    uint32_t nblocks, Item* __restrict__ items, uint64_t item_cap,
    uint32_t* __restrict__ first_pos, uint32_t* __restrict__ int_pos,
    uint32_t* __restrict__ last_pos, uint32_t* __restrict__ longs, bool scanned)
{
    __shared__ uint32_t bin_base[kBins];
    __shared__ uint32_t bin_tot[kBins];
    __shared__ uint32_t slot[kBins][kPlanThreads];
    __shared__ uint32_t sh[kPlanThreads / 64][kPacked];
    __shared__ bool over;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t* hdr = plan_hdr_d(blk, nblocks);
    if (scanned)
    {
        if (hdr[kHdrTotal] > item_cap) return;  // host re-plans (uniform)
        if (threadIdx.x < kBins) bin_base[threadIdx.x] = blk[threadIdx.x * nblocks + blockIdx.x];
    }
    else
    {
        if (wave < kBins)
        {
            uint32_t tot = 0, pre = 0;
            for (uint32_t j = lane; j < nblocks; j += 64)
            {
                const uint32_t c = blk[wave * nblocks + j];
                tot += c;
                pre += j < blockIdx.x ? c : 0u;
            }
            for (int d = 32; d >= 1; d >>= 1)
            {
                tot += __shfl_xor(tot, d);
                pre += __shfl_xor(pre, d);
            }
            if (lane == 0)
            {
                bin_tot[wave] = tot;
                bin_base[wave] = pre;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0)
        {
            uint32_t start = 0;
            for (uint32_t b = 0; b < kBins; ++b)
            {
                if (blockIdx.x == 0) hdr[b] = start;
                bin_base[b] += start;
                start += bin_tot[b];
            }
            if (blockIdx.x == 0) hdr[kHdrTotal] = start;
            over = start > item_cap;
        }
        __syncthreads();
        if (over) return;  // host re-plans (uniform)
    }

    // this thread's records and their counts (overlaps the loads above)
    const uint64_t r0 = (uint64_t(blockIdx.x) * kPlanThreads + threadIdx.x) * kPlanPer;
    RecShape srec[kPlanPer];
    ThreadCounts tc;
#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q)
    {
        srec[q] = RecShape{0, 0, 0, 0};
        if (r0 + q < count)
        {
            srec[q] = rec_shape(uint64_t(base) + off[r0 + q], len[r0 + q]);
            tc.add_record(srec[q]);
        }
    }
    // block exclusive scan of the packed counts
    uint32_t p[kPacked], x[kPacked];
    pack_counts(tc, p);
#pragma unroll
    for (int w = 0; w < kPacked; ++w)
    {
        x[w] = p[w];
        for (int d = 1; d < 64; d <<= 1)
        {
            const uint32_t y = __shfl_up(x[w], d);
            if (lane >= uint32_t(d)) x[w] += y;
        }
    }
    if (lane == 63)
        for (int w = 0; w < kPacked; ++w) sh[wave][w] = x[w];
    __syncthreads();
    uint32_t ex[kPacked];
#pragma unroll
    for (int w = 0; w < kPacked; ++w)
    {
        uint32_t acc = x[w] - p[w];
        for (uint32_t v = 0; v < wave; ++v) acc += sh[v][w];
        ex[w] = acc;
    }
    // this thread's next free slot per bin, in LDS (bank = thread, whatever the bin)
    {
        uint32_t e[kBins];
        unpack_counts(ex, e);
#pragma unroll
        for (uint32_t b = 0; b < kBins; ++b) slot[b][threadIdx.x] = bin_base[b] + e[b];
    }
    auto take = [&](uint32_t b, uint32_t n) {
        const uint32_t v = slot[b][threadIdx.x];
        slot[b][threadIdx.x] = v + n;
        return v;
    };

#pragma unroll
    for (uint32_t q = 0; q < kPlanPer; ++q)
    {
        const RecShape& s = srec[q];
        const uint64_t r = r0 + q;
        uint32_t nint_w = 0, ip = 0;  // interior run this lane hands to its wave
        if (r < count && s.n != 0)
        {
            // bin 0 holds, in order: first (if bin 0), interior pieces, last (if bin 0)
            const uint32_t fp = take(piece_bin(s, 0), 1);
            items[fp] = piece_item(s, 0);
            first_pos[r] = fp;
            if (s.n >= 2)
            {
                const uint32_t nint = s.n - 2;
                ip = take(0, nint);
                int_pos[r] = ip;
                if (nint > kLongChunks) longs[atomicAdd(hdr + kHdrLongs, 1u)] = uint32_t(r);
                nint_w = nint;
                const uint32_t lp = take(piece_bin(s, s.n - 1), 1);
                items[lp] = piece_item(s, s.n - 1);
                last_pos[r] = lp;
            }
        }
        // interior runs: the whole wave writes each lane's run, 64 items per store
        uint64_t pending = __builtin_amdgcn_ballot_w64(nint_w != 0);
        while (pending)
        {
            const int l = __builtin_ctzll(pending);
            pending &= pending - 1;
            // readlane returns int: go through uint32_t so the halves zero-extend
            const uint32_t n_l = uint32_t(__builtin_amdgcn_readlane(int(nint_w), l));
            const uint32_t ip_l = uint32_t(__builtin_amdgcn_readlane(int(ip), l));
            const uint32_t k0_lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(s.k0)), l));
            const uint32_t k0_hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(s.k0 >> 32)), l));
            const uint64_t k0_l = uint64_t(k0_lo) | (uint64_t(k0_hi) << 32);
            for (uint32_t j = lane; j < n_l; j += 64) items[ip_l + j] = interior_item(k0_l, j);
        }
    }
}

hipError_t launch_var_plan(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                           uint64_t count, const VarWorkspace& ws, hipStream_t stream,
                           bool force_scan)
{
    const uint32_t nb = var_plan_blocks(count);
    const uint8_t* b = static_cast<const uint8_t*>(base);
    hipLaunchKernelGGL(plan_count_kernel, dim3(nb), dim3(kPlanThreads), 0, stream, b, offsets,
                       lengths, count, ws.blk, nb);
    const bool scanned = force_scan || nb > kScanFreeBlocks;
    if (scanned) hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(1024), 0, stream, ws.blk, nb);
    hipLaunchKernelGGL(plan_scatter_kernel, dim3(nb), dim3(kPlanThreads), 0, stream, b, offsets,
                       lengths, count, ws.blk, nb, ws.items, ws.item_cap, ws.first_pos,
                       ws.int_pos, ws.last_pos, ws.longs, scanned);
    return hipGetLastError();
}

// Byte masks of one 16-B block, word q: keep bytes >= b (b in 0..16) or
// bytes < c (c in 0..16).  64-bit shifts make the 0- and 32-bit edge cases
// branch-free (a shift by 32 empties the word).
__device__ __forceinline__ uint32_t keep_from(int32_t b, int q)
{
    const uint32_t s = uint32_t(min(max(b - 4 * q, 0), 4)) * 8u;
    return uint32_t(~uint64_t(0) << s);
}

__device__ __forceinline__ uint32_t keep_below(int32_t c, int q)
{
    const uint32_t s = uint32_t(min(max(c - 4 * q, 0), 4)) * 8u;
    return uint32_t((uint64_t(0xFFFFFFFFu) << s) >> 32);
}

__device__ __forceinline__ uint4 mask_from(uint4 d, int32_t b)
{
    return make_uint4(d.x & keep_from(b, 0), d.y & keep_from(b, 1), d.z & keep_from(b, 2),
                      d.w & keep_from(b, 3));
}

__device__ __forceinline__ uint4 mask_below(uint4 d, int32_t c)
{
    return make_uint4(d.x & keep_below(c, 0), d.y & keep_below(c, 1), d.z & keep_below(c, 2),
                      d.w & keep_below(c, 3));
}

// One piece as a lane sees it.  Window coordinates: the window is G groups
// of 8 rows ending at the item's 128-aligned end; the piece occupies window
// bytes [s0, G*1024 - m).
//   p0   this lane's 16 B of window row 0
//   x    16*lane - s0: offset of that block from the piece start.  A block of
//        group 0 lying wholly before the piece is loaded from a zero block
//        instead (no read before the piece, nothing to mask).
//   rsb  the one row/byte where the piece starts inside this lane's block
//        ((row << 4) | byte, or 0xFF..: none): that block keeps bytes >= byte
//   ce   bytes of this lane's block in the LAST row that belong to the
//        piece (0..16); the rest is masked
struct ChunkView
{
    const uint8_t* p0;
    int32_t x;
    int32_t rsb;
    int32_t ce;
};

template <int G>
__device__ __forceinline__ ChunkView view_of(const Item& it, uint32_t tl)
{
    constexpr int32_t W = G * int32_t(kGroupBytes);
    const int32_t lenw = int32_t((it.bits >> kItemLenShift) & 0x1FFFu);
    const int32_t m = int32_t(it.bits & 0x7Fu);
    const int32_t s0 = W - lenw;
    ChunkView v;
    v.p0 = reinterpret_cast<const uint8_t*>((it.bits >> kItemAddrShift) << 7) - W + tl * 16;
    v.x = int32_t(tl) * 16 - s0;
    v.rsb = ((s0 & 15) != 0 && ((s0 >> 4) & 7) == int32_t(tl)) ? (((s0 >> 7) << 4) | (s0 & 15))
                                                               : 0x7FFFFFFF;
    v.ce = min(max(W - m - (W - int32_t(kRowBytes)) - int32_t(tl) * 16, 0), 16);
    return v;
}

// Items [lo, hi) all have G groups (the plan bins them).  Same discipline as
// crc32c_fixed_pipe_kernel: every group's 8 loads are unconditional and
// issued (sched_barrier) while the previous group is folded; item
// descriptors run ahead, so the loop-carried loads are identical on every
// path and vmcnt stays exact.  Masking is per block, not per row: group-0
// blocks before the piece read zeros, the start block is masked only in the
// row where some team of the wave has one (a wave-uniform ballot), and the
// last row is masked to the piece end.  For odd G two items are unrolled
// per iteration so the A/B buffers alternate.
template <int G>
__device__ __forceinline__ void chunk_bin(const Item* __restrict__ items, uint32_t lo, uint32_t hi,
                                          uint32_t* __restrict__ partial, uint32_t team,
                                          uint32_t team0, uint32_t nteams, uint32_t tl,
                                          uint32_t li, const uint8_t* zero16)
{
    if (hi <= lo || lo + team0 >= hi) return;
    constexpr int U = (G % 2 == 0) ? 1 : 2;  // items per loop iteration
    const uint32_t iters_items = (hi - lo - team0 + nteams - 1) / nteams;
    const uint32_t iters = (iters_items + U - 1) / U;
    auto idx_of = [&](uint32_t k) {
        const uint32_t i = lo + team + k * nteams;
        return i < hi ? i : hi - 1;
    };
    auto load_group = [&](uint4 (&buf)[kGroupRows], const ChunkView& v, int g) {
#pragma unroll
        for (int r = 0; r < kGroupRows; ++r)
        {
            const int32_t o = g * int32_t(kGroupBytes) + r * int32_t(kRowBytes);
            if (g == 0)
                buf[r] = load16(v.x + o > -16 ? v.p0 + o : zero16);
            else
                buf[r] = load16(v.p0 + o);
        }
    };

    // Descriptors run LA items ahead of the data: two for short pieces, one
    // for 3-4 group pieces (whose own time covers the descriptor's latency;
    // the extra registers would spill).
    constexpr uint32_t LA = G >= 3 ? 1 : 2;
    uint4 A[kGroupRows], B[kGroupRows];
    ChunkView cur = view_of<G>(items[idx_of(0)], tl);
    Item nit = LA == 2 ? items[idx_of(1)] : Item{};
    load_group(A, cur, 0);
    uint32_t k = 0;
    for (uint32_t iter = 0; iter < iters; ++iter)
    {
#pragma unroll
        for (int u = 0; u < U; ++u, ++k)
        {
            const Item nnit = items[idx_of(k + LA)];
            if (LA == 1) nit = nnit;
            ChunkView nxt = cur;
            uint32_t V[4] = {0, 0, 0, 0};
            bool fresh = true;  // wave-uniform: no row folded yet
#pragma unroll
            for (int g = 0; g < G; ++g)
            {
                const int parity = (u * G + g) % 2;  // buffer holding group g
                uint4(&bc)[kGroupRows] = parity == 0 ? A : B;
                uint4(&bn)[kGroupRows] = parity == 0 ? B : A;
                if (g + 1 < G)
                    load_group(bn, cur, g + 1);
                else
                {
                    nxt = view_of<G>(nit, tl);
                    load_group(bn, nxt, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int r = 0; r < kGroupRows; ++r)
                {
                    uint4 d = bc[r];
                    if (g == 0)
                    {
                        // rows before every team's piece leave V = 0: skip them
                        // (one-group pieces are sorted by row count, so this is common)
                        if (G == 1 && !__builtin_amdgcn_ballot_w64(cur.x + r * int32_t(kRowBytes) > -16))
                            continue;
                        const bool start_here = (cur.rsb >> 4) == r;
                        if (__builtin_amdgcn_ballot_w64(start_here))
                            d = mask_from(d, start_here ? (cur.rsb & 15) : 0);
                    }
                    if (g == G - 1 && r == kGroupRows - 1) d = mask_below(d, cur.ce);
                    // the window's first row, or (one-group pieces) the first
                    // row some team of the wave needs: the chains are still zero
                    if (g == 0 && (r == 0 || (G == 1 && fresh)))
                        row_first(V, d);
                    else
                        row_update(V, d, li);
                    if (G == 1) fresh = false;
                }
            }
            const uint32_t raw = team_fold(V);
            const uint32_t i = lo + team + k * nteams;
            if (tl == 0 && i < hi) partial[i] = raw;
            cur = nxt;
            nit = nnit;
        }
    }
}

// All bins in one launch with wave roles.  Measured on config 3 (MI355X):
// the 4-group pieces are HBM-bound and reach the same rate with 4 waves per
// CU as with 16, while the short pieces are bound by per-item latency and
// want as many waves as possible; run one after the other they cost the sum
// of the two, run side by side on every CU (4 "lead" waves on the 4-group
// pieces, 12 on the rest) they overlap.  A batch with only one kind gives
// every wave to it.  Item assignment is static except for a tail pool of
// 4-group pieces that waves of both roles drain when their own share is done,
// one atomic per 128-piece wave grab: a queue with one atomic per piece on a
// single address serialised (~12 ns/atomic chip-wide) into a 2x slower step.
constexpr uint32_t kLeadWaves = 4;
constexpr uint32_t kLeadAuto = ~0u;  // lead_override: pick from the plan (any value > 16)

// Shared pool (cfg 3, MI355X, same-box A/B): the last 30 % of the 4-group
// pieces, grabbed 128 at a time (16 per team): 0.892-0.896 ms per step
// against 0.904-0.929 with every piece statically assigned; 15-50 % pools
// and 32/64-piece grabs gain less, 256-piece grabs lose (coarse tail).
constexpr uint32_t kShareFrac = 30;  // % of the 4-group pieces in the shared pool
constexpr uint32_t kGrab = 128;      // pool pieces per wave grab

__global__ __launch_bounds__(kBlock, 1) void crc32c_chunk_kernel(
    const Item* __restrict__ items, uint32_t* __restrict__ blk, uint32_t nblocks,
    uint32_t* __restrict__ partial, uint64_t item_cap, const uint32_t* __restrict__ tables,
    uint32_t lead_override)
{
    uint32_t* hdr = blk + kBins * nblocks;  // plan_hdr
    const uint32_t n_items = hdr[kHdrTotal];
    if (n_items > item_cap || n_items == 0) return;
    // bins: [hdr[0], hdr[1]) 4 groups, [hdr[1], hdr[2]) 3, [hdr[2], hdr[3]) 2,
    // [hdr[3], n_items) one group of 8..1 rows
    const uint32_t b0 = hdr[0], b1 = hdr[1], b2 = hdr[2], b3 = hdr[3];
    const uint32_t lead = lead_override <= 16 ? lead_override
                          : b1 == b0          ? 0u
                          : n_items == b1     ? 16u
                                              : kLeadWaves;
    stage_tables(tables);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64u);
    const uint32_t tl = threadIdx.x & (kTeam - 1);
    const uint32_t tw = (threadIdx.x & 63u) / kTeam;
    const uint32_t li = lane_info();
    const uint8_t* zero16 = reinterpret_cast<const uint8_t*>(tables + kTabZero);
    // With both roles present, the last kShareFrac % of the 4-group pieces
    // form a pool that every wave drains once its static share is done, so
    // neither role idles while the other finishes.
    const bool mixed = lead != 0 && lead != 16;
    const uint32_t split = mixed ? b1 - uint32_t(uint64_t(b1 - b0) * kShareFrac / 100u) : b1;
    if (wave < lead)
    {
        const uint32_t team = (blockIdx.x * lead + wave) * kTeam + tw;
        const uint32_t nteams = gridDim.x * lead * kTeam;
        chunk_bin<4>(items, b0, split, partial, team, team & ~7u, nteams, tl, li, zero16);
    }
    else
    {
        const uint32_t rest = 16u - lead;
        const uint32_t team = (blockIdx.x * rest + (wave - lead)) * kTeam + tw;
        const uint32_t nteams = gridDim.x * rest * kTeam;
        chunk_bin<3>(items, b1, b2, partial, team, team & ~7u, nteams, tl, li, zero16);
        chunk_bin<2>(items, b2, b3, partial, team, team & ~7u, nteams, tl, li, zero16);
        chunk_bin<1>(items, b3, n_items, partial, team, team & ~7u, nteams, tl, li, zero16);
    }
    // one relaxed atomic per wave grab; every wave leaves once the pool is empty
    while (split < b1)
    {
        uint32_t got = 0;
        if ((threadIdx.x & 63u) == 0)
            got = __hip_atomic_fetch_add(hdr + kHdrGrab, kGrab, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t lo = split + __builtin_amdgcn_readfirstlane(got);
        if (lo >= b1) break;
        chunk_bin<4>(items, lo, min(lo + kGrab, b1), partial, tw, 0u, 64u / kTeam, tl, li, zero16);
    }
}

hipError_t launch_var_chunks(const uint32_t* inits, uint64_t count, const VarWorkspace& ws,
                             const uint32_t* tables, int grid, hipStream_t stream)
{
    if (count == 0) return hipSuccess;
    (void)inits;  // applied by the finalize kernels
    hipLaunchKernelGGL(crc32c_chunk_kernel, dim3(grid), dim3(kBlock), kLdsBytes, stream, ws.items,
                       ws.blk, var_plan_blocks(count), ws.partial, ws.item_cap, tables,
                       kLeadAuto);
    return hipGetLastError();
}

// Z_n(v) through a G^n table set (LDS or global).
__device__ __forceinline__ uint32_t zglob(const uint32_t* g, uint32_t v)
{
    return g[v & 0xFFu] ^ g[256 + ((v >> 8) & 0xFFu)] ^ g[512 + ((v >> 16) & 0xFFu)] ^
           g[768 + (v >> 24)];
}

// Z_n for n < 2^13 through the G^{2^k} tables.
__device__ __forceinline__ uint32_t zbits(const uint32_t* p2, uint32_t v, uint32_t n)
{
    for (int k = 0; n; ++k, n >>= 1)
        if (n & 1u) v = zglob(p2 + k * 1024, v);
    return v;
}

// Z_{-m}, 0 <= m < 128: Z_{-128} o Z_{128-m}.
__device__ __forceinline__ uint32_t zneg(const uint32_t* p2, const uint32_t* zinv, uint32_t v,
                                        uint32_t m)
{
    return m ? zglob(zinv, zbits(p2, v, kRowBytes - m)) : v;
}

// Register after a record's first piece: the seed ~init shifted across the
// piece's window, `sx` = Z_{w-a}(~init), XORed with R0 and the trailing m
// zeros undone.  window [.., w), piece [a, pe), m = w - pe, R0 = Z_m(raw(piece)):
// state = Z_{pe-a}(~init) ^ raw(piece) = Z_{-m}(sx ^ R0).
__device__ __forceinline__ uint32_t first_piece_state(const RecShape& s, const uint32_t* p2,
                                                      const uint32_t* zinv, uint32_t sx,
                                                      uint32_t R0)
{
    const uint64_t pe = piece_end(s, 0);
    const uint64_t w = (pe + kRowBytes - 1) & ~uint64_t(kRowBytes - 1);
    return zneg(p2, zinv, sx ^ R0, uint32_t(w - pe));
}

// Z_{w-a}(~init) for the first piece (w - a <= 4096): with no inits, one
// load from F = Z_n(~0) (issued before the partials arrive); else the shift.
__device__ __forceinline__ uint32_t first_seed(const RecShape& s, const uint32_t* p2,
                                               const uint32_t* __restrict__ finit,
                                               const uint32_t* __restrict__ inits, uint64_t r)
{
    const uint64_t pe = piece_end(s, 0);
    const uint32_t n = uint32_t(((pe + kRowBytes - 1) & ~uint64_t(kRowBytes - 1)) - s.a);
    return inits ? zbits(p2, ~inits[r], n) : finit[n];
}

// Register after the last piece (n >= 2) from the state before it.  The
// piece starts on a chunk boundary, so its window is 128 k bytes (k <= 32):
// one G^{128 k} table set (global, L2-resident) instead of a bit-serial shift.
__device__ __forceinline__ uint32_t last_piece_state(const RecShape& s, const uint32_t* p2,
                                                     const uint32_t* zinv,
                                                     const uint32_t* __restrict__ zrows,
                                                     uint32_t x, uint32_t R)
{
    const uint64_t ps = piece_start(s, s.n - 1), pe = s.E;
    const uint64_t w = (pe + kRowBytes - 1) & ~uint64_t(kRowBytes - 1);
    const uint32_t k = uint32_t(w - ps) / kRowBytes;
    return zneg(p2, zinv, zglob(zrows + (k - 1) * 1024, x) ^ R, uint32_t(w - pe));
}

// One thread per record: Horner from ~init over its pieces (see the section
// comment); records < 32 B byte-serially.
constexpr uint32_t kFinBlock = 512;
__global__ __launch_bounds__(kFinBlock) void crc32c_finalize_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ inits, uint64_t count,
    const uint32_t* __restrict__ partial, const uint32_t* __restrict__ first_pos,
    const uint32_t* __restrict__ int_pos, const uint32_t* __restrict__ last_pos,
    uint32_t* __restrict__ out, const uint32_t* __restrict__ tables,
    const uint32_t* __restrict__ counters, uint64_t item_cap,
    const uint32_t* __restrict__ longs, const uint32_t* __restrict__ pow2)
{
    // a plan larger than the workspace (an understated total_bytes hint) was
    // not scattered: leave out[] alone rather than read unwritten positions
    if (counters[kHdrTotal] > item_cap) return;
    __shared__ uint32_t t0[256];
    __shared__ uint32_t zc[1024];
    __shared__ uint32_t zinv[1024];
    __shared__ uint32_t p2[7 * 1024];  // G^{2^k}, k < 7: the Z_{128-m} of zneg
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) t0[i] = tables[kTabT + i];
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x)
    {
        zc[i] = tables[kTabZChunk + i];
        zinv[i] = tables[kTabZInv128 + i];
    }
    for (uint32_t i = threadIdx.x; i < 7 * 1024; i += blockDim.x) p2[i] = tables[kTabP2 + i];
    __syncthreads();
    // persistent grid: the tables are staged once per workgroup
    for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < count;
         r += uint64_t(gridDim.x) * blockDim.x)
    {
        const uint8_t* p = base + off[r];
        const uint32_t L = len[r];
        uint32_t c = ~(inits ? inits[r] : 0u);
        const RecShape s = rec_shape(uint64_t(p), L);
        if (s.n == 0)
        {
            for (uint32_t i = 0; i < L; ++i) c = t0[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
        }
        else
        {
            if (s.n >= 2 && s.n - 2 > kLongChunks) continue;  // the block-wide fold below
            const uint32_t sx = first_seed(s, tables + kTabP2, tables + kTabFInit, inits, r);
            c = first_piece_state(s, p2, zinv, sx, partial[first_pos[r]]);
            if (s.n >= 2)
            {
                const uint32_t ip = int_pos[r];
                for (uint32_t j = 0; j + 2 < s.n; ++j) c = zglob(zc, c) ^ partial[ip + j];
                c = last_piece_state(s, p2, zinv, tables + kTabZRows, c, partial[last_pos[r]]);
            }
        }
        out[r] = ~c;
    }
    // Long records (listed by plan_scatter_kernel), one workgroup each:
    // their interior run contributes XOR_jj Z_{C jj}(p[ip + nint - 1 - jj]).
    // Thread t folds jj = t + 512 q by Horner with Z_{512 C}, shifts by
    // Z_{C t} (G^{C 2^b}, b < 9) and the workgroup XOR-reduces; thread 0 adds
    // the first piece carried by Z_{C nint} and the last piece.  Their tables
    // are read from global memory (L2): long records are rare.
    const uint32_t nlong = counters[kHdrLongs];
    if (blockIdx.x >= nlong) return;
    static_assert(kFinBlock == 512, "long fold stride: Z_{512 C} = G^{C 2^9}");
    __shared__ uint32_t red[kFinBlock / 64];
    const uint32_t t = threadIdx.x;
    const uint32_t* zs = tables + kTabZC2 + 9 * 1024;
    for (uint32_t k = blockIdx.x; k < nlong; k += gridDim.x)
    {
        const uint32_t r = longs[k];
        const RecShape s = rec_shape(uint64_t(base) + off[r], len[r]);
        const uint32_t nint = s.n - 2;
        const uint32_t ip = int_pos[r];
        uint32_t acc = 0;
        if (t < nint)
        {
            const uint32_t n_t = (nint - t + kFinBlock - 1) / kFinBlock;
            for (uint32_t q = n_t; q-- > 0;)
                acc = zglob(zs, acc) ^ partial[ip + nint - 1 - (t + q * kFinBlock)];
#pragma unroll 1
            for (int b = 0; b < 9; ++b)
                if (t & (1u << b)) acc = zglob(tables + kTabZC2 + b * 1024, acc);
        }
        for (int d = 32; d >= 1; d >>= 1) acc ^= __shfl_xor(acc, d);
        if ((t & 63) == 0) red[t >> 6] = acc;
        __syncthreads();
        if (t == 0)
        {
            uint32_t c = 0;
            for (int w = 0; w < kFinBlock / 64; ++w) c ^= red[w];
            uint32_t h = first_piece_state(s, p2, zinv, first_seed(s, tables + kTabP2, tables + kTabFInit, inits, r),
                                           partial[first_pos[r]]);
            uint64_t n = uint64_t(nint) * kChunk;  // bytes of the interior run
#pragma unroll 1
            for (int b = 0; n && b < 48; ++b, n >>= 1)
                if (n & 1u) h = zglob(pow2 + b * 1024, h);
            c ^= h;
            out[r] = ~last_piece_state(s, p2, zinv, tables + kTabZRows, c, partial[last_pos[r]]);
        }
        __syncthreads();
    }
}

hipError_t launch_var_finalize(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                               const uint32_t* inits, uint64_t count, const VarWorkspace& ws,
                               uint32_t* out, const uint32_t* tables, const uint32_t* pow2,
                               hipStream_t stream)
{
    if (count == 0) return hipSuccess;
    const uint8_t* b = static_cast<const uint8_t*>(base);
    // four 512-thread workgroups per CU fit the 37 KB of tables each stages
    const uint64_t fin_blocks = (count + kFinBlock - 1) / kFinBlock;
    hipLaunchKernelGGL(crc32c_finalize_kernel, dim3(uint32_t(fin_blocks < 1024 ? fin_blocks : 1024)),
                       dim3(kFinBlock), 0,
                       stream, b, offsets, lengths, inits, count, ws.partial, ws.first_pos,
                       ws.int_pos, ws.last_pos, out, tables,
                       plan_hdr(ws.blk, var_plan_blocks(count)), ws.item_cap, ws.longs, pow2);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Small batches (a durable-log flush, one consus::crc32c call on host data):
// one launch instead of plan + chunks + finalize.  Team t of the grid takes
// records t, t + nteams, ...; a record [a, E) is read as the 128-B rows that
// cover it, bytes outside it masked to zero (leading zeros are free; the
// m = ceil128(E) - E trailing ones are undone with one Z_{-m} table), folded
// by the row update and team fold of the fixed kernel, and finished with the
// seed: crc = ~(Z_L(~init) ^ raw).  Rows go 8 at a time (one load group).
// ---------------------------------------------------------------------------
// LITE (batches up to kLiteMaxBytes): one-wave workgroups (launch bound 256), no LDS; the
// row update and the fold go through the lane tables (row_update_lane,
// team_fold_lane), 42 VGPRs loaded from L2 beside the first record's reads,
// instead of a 152 KiB LDS image staged by every workgroup before any
// record is read.  Same rows, masks and finish.
template <bool LITE>
__global__ __launch_bounds__(LITE ? kLiteBlock : kBlock, 1) void crc32c_direct_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ inits, uint64_t count,
    uint32_t* __restrict__ out, const uint32_t* __restrict__ tables,
    const uint32_t* __restrict__ pow2, DoneSignal sig)
{
    const uint32_t B = LITE ? blockDim.x : uint32_t(kBlock);
    const uint32_t tl = threadIdx.x & (kTeam - 1);
    const uint32_t li = lane_info();
    const uint64_t team = (uint64_t(blockIdx.x) * B + threadIdx.x) / kTeam;
    const uint64_t nteams = uint64_t(gridDim.x) * B / kTeam;
    const uint64_t team0 = team & ~uint64_t(7);  // first team of this wave
    const uint64_t iters = team0 < count ? (count - team0 + nteams - 1) / nteams : 0;
    const uint8_t* zero16 = reinterpret_cast<const uint8_t*>(tables + kTabZero);
    // the first record's offset and length are loaded before the table
    // staging, so their latency (a PCIe round trip when they sit in mapped
    // pinned memory: a durable-log flush) overlaps it
    uint64_t nx_off = 0;
    uint32_t nx_len = 0;
    if (iters)
    {
        const uint64_t r0 = team < count ? team : count - 1;
        nx_off = off[r0];
        nx_len = team < count ? len[r0] : 0u;
    }
    LaneTabs lt;
    if constexpr (LITE)
        load_lane_tabs<42>(lt, tables);  // the fold operators and Z_128
    else
        stage_tables(tables);
    for (uint64_t it = 0; it < iters; ++it)
    {
        const uint64_t r_raw = team + it * nteams;
        const bool live = r_raw < count;
        const uint64_t r = live ? r_raw : count - 1;
        const uint32_t L = nx_len;
        const uint64_t a = uint64_t(base) + nx_off, E = a + L;
        if (it + 1 < iters)
        {
            const uint64_t rn_raw = r_raw + nteams;
            const uint64_t rn = rn_raw < count ? rn_raw : count - 1;
            nx_off = off[rn];
            nx_len = rn_raw < count ? len[rn] : 0u;
        }
        const uint64_t w0 = a & ~uint64_t(kRowBytes - 1);
        const uint64_t w1 = (E + kRowBytes - 1) & ~uint64_t(kRowBytes - 1);
        const uint32_t rows = uint32_t((w1 - w0) / kRowBytes);
        // groups of 8 rows, two buffers: group g + 1 is in flight while g is
        // folded.  The wave runs as many groups as its longest record needs;
        // rows past a record's end load a zero block and are not folded, so
        // every load is unconditional and the vmcnt counts stay exact.
        uint32_t rmax = rows;
        for (int dlt = 32; dlt >= 1; dlt >>= 1) rmax = max(rmax, uint32_t(__shfl_xor(int(rmax), dlt)));
        const uint32_t ngw = (rmax + kGroupRows - 1) / kGroupRows;
        auto load_group = [&](uint4 (&buf)[kGroupRows], uint32_t g) {
#pragma unroll
            for (int k = 0; k < kGroupRows; ++k)
            {
                const uint32_t row = g * kGroupRows + k;
                const uint64_t bs = w0 + uint64_t(row) * kRowBytes + tl * 16;
                buf[k] = load16(row < rows ? reinterpret_cast<const uint8_t*>(bs) : zero16);
            }
        };
        uint32_t V[4] = {0, 0, 0, 0};
        // only the first row starts before the record and only the last one
        // runs past it: this lane keeps bytes >= f0 of the first, < bl of the last
        const int32_t f0 = min(max(int32_t(a - w0) - int32_t(tl) * 16, 0), 16);
        const int32_t bl = min(max(int32_t(E + kRowBytes - w1) - int32_t(tl) * 16, 0), 16);
        auto fold_group = [&](const uint4 (&buf)[kGroupRows], uint32_t g) {
#pragma unroll
            for (int k = 0; k < kGroupRows; ++k)
            {
                const uint32_t row = g * kGroupRows + k;
                if constexpr (LITE)
                {
                    if (row >= rmax) break;  // wave-uniform
                    uint4 d = buf[k];
                    if (row == 0) d = mask_from(d, f0);
                    if (row + 1 == rows) d = mask_below(d, bl);
                    row_update_lane(V, d, lt, row < rows, row == 0);
                }
                else
                {
                    if (row >= rows) break;
                    uint4 d = buf[k];
                    if (row == 0) d = mask_from(d, f0);
                    if (row + 1 == rows) d = mask_below(d, bl);
                    if (row == 0)
                        row_first(V, d);
                    else
                        row_update(V, d, li);
                }
            }
        };
        uint4 A[kGroupRows], B[kGroupRows];
        load_group(A, 0);
        for (uint32_t g = 0; g < ngw; g += 2)
        {
            load_group(B, g + 1);
            __builtin_amdgcn_sched_barrier(0);
            fold_group(A, g);
            load_group(A, g + 2);
            __builtin_amdgcn_sched_barrier(0);
            fold_group(B, g + 1);
        }
        uint32_t W;  // every lane of the wave takes part
        if constexpr (LITE)
            W = team_fold_lane(V, lt);
        else
            W = team_fold(V);
        if (tl == 0 && live)
        {
            const uint32_t raw = zglob(tables + kTabZNeg + uint32_t(w1 - E) * 1024, W);
            const uint32_t init = inits ? inits[r] : 0u;
            uint32_t seed;
            if (init == 0 && L <= uint32_t(kChunk))
                seed = tables[kTabFInit + L];  // Z_L(~0)
            else
            {
                seed = ~init;
                uint32_t n = L;
                for (int k = 0; n; ++k, n >>= 1)
                    if (n & 1u) seed = zglob(pow2 + k * 1024, seed);
            }
            out[r] = ~(seed ^ raw);
        }
    }
    if (sig.counter)
    {
        // each thread's CRC stores reach the system before its workgroup
        // counts itself done; the last one to count publishes seq
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0 && atomicAdd(sig.counter, 1u) == gridDim.x - 1)
        {
            atomicExch(sig.counter, 0u);  // ready for the next launch on the stream
            __threadfence_system();
            *reinterpret_cast<volatile uint32_t*>(sig.flag) = sig.seq;
        }
    }
}

hipError_t launch_direct(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                         const uint32_t* inits, uint64_t count, uint64_t total_bytes, uint32_t* out,
                         const uint32_t* tables, const uint32_t* pow2, int grid,
                         hipStream_t stream, const DoneSignal* signal, int lite)
{
    if (count == 0) return hipSuccess;
    const DoneSignal sig = signal ? *signal : DoneSignal{nullptr, nullptr, 0};
    if (lite < 0) lite = total_bytes <= kLiteMaxBytes;
    if (lite)
    {
        // one-wave workgroups (8 teams): a flush's records spread over as many
        // CUs as it has waves, so more of its PCIe reads are in flight at once
        // (round 3 A/B, profiles/r03_lite_wg_ab.txt: a 270-frame
        // zero-copy flush 17.3-18.7 us against 18.9-19.8 with 256-thread
        // workgroups, never slower up to 8,192 frames); up to 16 per CU
        constexpr uint32_t wg = kLiteWG;
        const uint64_t need = (count + (wg / kTeam) - 1) / (wg / kTeam);
        const uint64_t g = std::min<uint64_t>(need, uint64_t(grid) * (4 * kLiteBlock / wg));
        hipLaunchKernelGGL(crc32c_direct_kernel<true>, dim3(uint32_t(g)), dim3(wg), 0, stream,
                           static_cast<const uint8_t*>(base), offsets, lengths, inits, count, out,
                           tables, pow2, sig);
        return hipGetLastError();
    }
    const uint64_t need = (count + (kBlock / kTeam) - 1) / (kBlock / kTeam);
    if (uint64_t(grid) > need) grid = int(need);
    hipLaunchKernelGGL(crc32c_direct_kernel<false>, dim3(grid), dim3(kBlock), kLdsBytes, stream,
                       static_cast<const uint8_t*>(base), offsets, lengths, inits, count, out,
                       tables, pow2, sig);
    return hipGetLastError();
}

// Offsets/lengths for a fixed-stride batch the fast kernel cannot take
// (unaligned base/stride or a length that is not a multiple of 16).
__global__ __launch_bounds__(256) void make_fixed_records_kernel(uint64_t* __restrict__ off,
                                                                 uint32_t* __restrict__ len,
                                                                 uint64_t count, uint64_t stride,
                                                                 uint32_t length)
{
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= count) return;
    off[i] = i * stride;
    len[i] = length;
}

hipError_t launch_make_fixed_records(uint64_t* off, uint32_t* len, uint64_t count, uint64_t stride,
                                     uint32_t length, hipStream_t stream)
{
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(make_fixed_records_kernel, dim3(uint32_t((count + 255) / 256)), dim3(256),
                       0, stream, off, len, count, stride, length);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// combine: out[i] = Z_{len_b[i]}(crc_a[i]) ^ crc_b[i]  (crc32c(0, A||B) from
// crc32c(0, A), crc32c(0, B) and |B|).  pow2_tables holds G^{2^k}, k = 0..47.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void crc32c_combine_kernel(
    const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
    const uint64_t* __restrict__ nb, uint64_t count, uint32_t* __restrict__ out,
    const uint32_t* __restrict__ pow2)
{
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint32_t s = a[i];
    uint64_t n = nb[i];
    for (int k = 0; n && k < 48; ++k, n >>= 1)
    {
        if (n & 1u)
        {
            const uint32_t* g = pow2 + k * 1024;
            s = g[s & 0xFFu] ^ g[256 + ((s >> 8) & 0xFFu)] ^ g[512 + ((s >> 16) & 0xFFu)] ^
                g[768 + (s >> 24)];
        }
    }
    out[i] = s ^ b[i];
}

// One CRC from consecutive pieces: out = XOR_i Z_{after_i}(crc_i), after_i
// = bytes of the pieces behind piece i (identity 1 of DESIGN.md section 3,
// applied to every piece at once instead of a serial Horner chain).  One
// workgroup; G^{2^k} tables from global memory.
__global__ __launch_bounds__(1024) void crc32c_chain_kernel(const uint32_t* __restrict__ crcs,
                                                            const uint64_t* __restrict__ after,
                                                            uint32_t np, uint32_t* __restrict__ out,
                                                            const uint32_t* __restrict__ pow2)
{
    __shared__ uint32_t red[16];
    uint32_t acc = 0;
    for (uint32_t i = threadIdx.x; i < np; i += blockDim.x)
    {
        uint32_t s = crcs[i];
        uint64_t n = after[i];
        for (int k = 0; n && k < 48; ++k, n >>= 1)
            if (n & 1u) s = zglob(pow2 + k * 1024, s);
        acc ^= s;
    }
    for (int d = 32; d >= 1; d >>= 1) acc ^= __shfl_xor(acc, d);
    if ((threadIdx.x & 63u) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        uint32_t r = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; ++w) r ^= red[w];
        out[0] = r;
    }
}

hipError_t launch_chain(const uint32_t* crcs, const uint64_t* after, uint32_t np, uint32_t* out,
                        const uint32_t* pow2_tables, hipStream_t stream)
{
    if (np == 0) return hipSuccess;
    hipLaunchKernelGGL(crc32c_chain_kernel, dim3(1), dim3(1024), 0, stream, crcs, after, np, out,
                       pow2_tables);
    return hipGetLastError();
}

hipError_t launch_combine(const uint32_t* crc_a, const uint32_t* crc_b, const uint64_t* len_b,
                          uint64_t count, uint32_t* out, const uint32_t* pow2_tables,
                          hipStream_t stream)
{
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(crc32c_combine_kernel, dim3(uint32_t((count + 255) / 256)), dim3(256), 0,
                       stream, crc_a, crc_b, len_b, count, out, pow2_tables);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// One large device buffer (consus::crc32c(init, data, n), common/crc32c.cc:
// 122-126, on a device pointer).  The buffer [a, a + n) is cut as
//   head      [a, E)            4 <= h = E - a < 4100 bytes, E 4 KiB-aligned
//   interior  m chunks of 4 KiB from E (crc32c_span_chunk_kernel, init 0)
//   tail      t < 4096 bytes
// and joined with raw-register algebra:
//   raw(chunk j) = crc_j ^ crc0,  crc0 = crc32c(0, 4096 zero bytes)
//   s = raw(head window, ~init XORed into bytes a..a+3)
//   s = Z_{4096 m}(s) ^ raw(interior);  s = Z_t(s) ^ raw(tail);  crc = ~s
// raw(interior) is a two-level tree: single_tree_kernel folds S = 1024 R
// consecutive chunk CRCs per workgroup (strided Horner over R per thread, then a
// 1024-leaf tree of 4 KiB leaves, thread t taking chunks t + 1024 r);
// single_join_kernel
// (one workgroup) trees the per-workgroup values the same way and adds head
// and tail, each hashed by the whole workgroup from a zero-masked window.
// The chunk index space is padded with zero chunks at the FRONT (leading
// zeros are free), so every tree is full.
// ---------------------------------------------------------------------------
constexpr uint32_t kSingleStaged = 36;  // G^{2^k}, k < 36, staged by single_join_kernel

// Tree of the 1024 values of a workgroup: leaf i spans `unit` bytes (unit =
// 2^k0); returns the raw register of the concatenation in thread 0.  `zt(l, v)`
// applies Z_{unit 2^l}.
template <typename ZT>
__device__ __forceinline__ uint32_t block_tree(uint32_t x, ZT zt, uint32_t* sh)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
#pragma unroll
    for (int l = 0; l < 6; ++l) x = zt(l, x) ^ __shfl_xor(x, 1 << l);
    if (lane == 0) sh[wave] = x;
    __syncthreads();
    if (wave == 0)
    {
        x = lane < 16 ? sh[lane] : 0u;
#pragma unroll
        for (int l = 6; l < 10; ++l) x = zt(l, x) ^ __shfl_xor(x, 1 << (l - 6));
    }
    return x;
}

// Raw register of the window [w, w + 1024 * B) of bytes, B = 4 or 8 per thread,
// keeping only bytes in [lo, hi) (others read as zero, none is loaded) and
// XORing `x4` (little-endian) into bytes [x_at, x_at + 4).  T = T_0..T_15
// (global); p2[l] = G^{B 2^l} (LDS), l < 10.
template <int B>
__device__ __forceinline__ uint32_t window_raw(uint64_t w, uint64_t lo, uint64_t hi, uint64_t x_at,
                                               uint32_t x4, const uint32_t* __restrict__ T,
                                               const uint32_t (*p2)[1024], uint32_t* sh)
{
    const uint64_t p = w + uint64_t(threadIdx.x) * B;
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < B; ++i)
    {
        const uint64_t q = p + i;
        uint32_t byte = (q >= lo && q < hi) ? *reinterpret_cast<const uint8_t*>(q) : 0u;
        if (q >= x_at && q < x_at + 4) byte ^= (x4 >> (8 * (q - x_at))) & 0xFFu;
        r ^= T[(B - 1 - i) * 256 + byte];  // byte i is followed by B - 1 - i bytes
    }
    return block_tree(r, [&](int l, uint32_t v) { return zglob(p2[l], v); }, sh);
}

// Workgroups [0, nblocks): the interior tree.  Workgroup nblocks: the head
// (the 8 KiB window ending at E = a + h, ~init in the record's first 4
// bytes); nblocks + 1: the tail (the 4 KiB window ending at the buffer end).
// Results: vals[0, nblocks), vals[1024] = head, vals[1025] = tail.
__global__ __launch_bounds__(1024) void single_tree_kernel(
    const uint32_t* __restrict__ crcs, uint64_t pad, uint32_t crc0, uint32_t log_r,
    uint64_t a, uint64_t h, uint64_t m, uint32_t t, uint32_t init,
    const uint32_t* __restrict__ tables, const uint32_t* __restrict__ pow2,
    uint32_t* __restrict__ vals)
{
    __shared__ uint32_t tab[11][1024];
    __shared__ uint32_t sh[16];
    const uint32_t nblocks = gridDim.x - 2;
    if (blockIdx.x >= nblocks)
    {
        const bool head = blockIdx.x == nblocks;
        const int k0 = head ? 3 : 2;  // G^{8 2^l} / G^{4 2^l}
        for (uint32_t i = threadIdx.x; i < 10 * 1024; i += 1024)
            tab[i >> 10][i & 1023] = pow2[k0 * 1024 + i];
        __syncthreads();
        const uint64_t E = a + h, b = E + m * kChunk;
        const uint32_t* T = tables + kTabT;
        uint32_t x = 0;
        if (head)
            x = window_raw<8>(E - 8192, a, E, a, ~init, T, tab, sh);
        else if (t)
            x = window_raw<4>(b + t - 4096, b, b + t, 0, 0, T, tab, sh);
        if (threadIdx.x == 0) vals[head ? 1024 : 1025] = x;
        return;
    }
    // tab[0] = Z_{4096 * 1024}, the thread's stride; tab[1 + l] = Z_{4096 * 2^l}
    for (uint32_t i = threadIdx.x; i < 1024; i += 1024) tab[0][i] = pow2[22 * 1024 + i];
    for (uint32_t i = threadIdx.x; i < 10 * 1024; i += 1024)
        tab[1 + (i >> 10)][i & 1023] = pow2[12 * 1024 + i];
    // thread t takes virtual chunks b S + t + 1024 r (coalesced); chunk v < pad is zero.
    // Its Horner value H_t (stride Z_{4096 * 1024}) enters the span's raw register
    // as Z_{4096 (1023 - t)}(H_t): a 1024-leaf tree of 4 KiB leaves.
    const uint32_t R = 1u << log_r;
    const uint64_t v0 = uint64_t(blockIdx.x) * (1024u << log_r) + threadIdx.x;
    uint32_t v[16];
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r)
    {
        const uint64_t c = v0 + uint64_t(r) * 1024;
        v[r] = (r < R && c >= pad) ? crcs[c - pad] ^ crc0 : 0u;
    }
    __syncthreads();
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r)
        if (r < R) acc = zglob(tab[0], acc) ^ v[r];
    acc = block_tree(acc, [&](int l, uint32_t x) { return zglob(tab[1 + l], x); }, sh);
    if (threadIdx.x == 0) vals[blockIdx.x] = acc;
}

// One workgroup: tree of the interior workgroups' values (leaf i =
// workgroup i - (1024 - nblocks)), then s = Z_t(Z_{4096 m}(head) ^ interior)
// ^ tail and crc = ~s.  G^{2^k}, k < kSingleStaged, staged in LDS.
__global__ __launch_bounds__(1024) void single_join_kernel(uint64_t m, uint32_t t,
                                                          uint32_t nblocks, uint32_t log_s,
                                                          const uint32_t* __restrict__ vals,
                                                          const uint32_t* __restrict__ pow2,
                                                          uint32_t* __restrict__ out)
{
    extern __shared__ uint32_t p2s[];  // kSingleStaged x 1024
    __shared__ uint32_t sh[16];
    uint32_t(*p2)[1024] = reinterpret_cast<uint32_t(*)[1024]>(p2s);
    for (uint32_t i = threadIdx.x; i < kSingleStaged * 1024; i += 1024) p2s[i] = pow2[i];
    const uint32_t bv = threadIdx.x >= 1024 - nblocks ? vals[threadIdx.x - (1024 - nblocks)] : 0u;
    __syncthreads();
    const uint32_t xi = block_tree(bv, [&](int l, uint32_t v) { return zglob(p2[log_s + l], v); }, sh);
    if (threadIdx.x == 0)
    {
        uint32_t s = vals[1024];
        for (int k = 0; k < int(kSingleStaged) - 12; ++k)
            if ((m >> k) & 1u) s = zglob(p2[12 + k], s);
        s ^= xi;
        for (int k = 0; k < 12; ++k)
            if ((t >> k) & 1u) s = zglob(p2[k], s);
        out[0] = ~(s ^ vals[1025]);
    }
}

hipError_t launch_single(const void* data, uint64_t h, uint64_t m, uint32_t t, uint32_t init,
                         uint32_t crc0, uint32_t* crcs, uint32_t* vals, uint32_t* out,
                         const uint32_t* tables, const uint32_t* pow2, int grid,
                         hipStream_t stream)
{
    // S = 1024 R chunks per tree workgroup: about 256 workgroups up to
    // R = 16, then up to 1024.  Each stages 44 KB of tables, so fewer is
    // cheaper, but each folds R chunk CRCs serially; measured for one 4 GiB
    // record (rocprof, 36 calls): 15.2 us at ~128 workgroups (R = 16),
    // 10.6 at ~256 (R = 4), 12.7 at ~1024 (R = 1).
    uint32_t log_r = 0;
    while (log_r < 4 && (uint64_t(256) << (10 + log_r)) < m + 2) ++log_r;
    const uint64_t S = uint64_t(1024) << log_r;
    const uint64_t M = (m + 2 + S - 1) / S * S;  // leading chunks [0, M - m) are zero
    const uint32_t nblocks = uint32_t(M / S);
    // the join's top tree level G^{4096 S 2^9} must be staged; Z_{4096 m} needs m < 2^24
    if (m == 0 || nblocks > 1024 || 22 + log_r + 9 >= kSingleStaged || (m >> 24) != 0)
        return hipErrorInvalidValue;
    const uint8_t* base = static_cast<const uint8_t*>(data) + h;
    const uint64_t need = (m + (kBlock / kTeam) - 1) / (kBlock / kTeam);
    if (uint64_t(grid) > need) grid = int(need);
    hipLaunchKernelGGL(crc32c_span_chunk_kernel, dim3(grid), dim3(kBlock), kLdsBytes, stream, base,
                       m, crcs, tables);
    hipLaunchKernelGGL(single_tree_kernel, dim3(nblocks + 2), dim3(1024), 0, stream, crcs, M - m,
                       crc0, log_r, uint64_t(data), h, m, t, init, tables, pow2, vals);
    hipLaunchKernelGGL(single_join_kernel, dim3(1), dim3(1024), kSingleStaged * 4096, stream, m,
                       t, nblocks, 22 + log_r, vals, pow2, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Variable-length batches, sorted path: one team per
// whole record, records binned by row count inside each workgroup's share.
//   sorted_cost_kernel:   per block of 1,024 records, the sum of the records'
//       costs (rows plus a fold allowance per item).  Records shorter than
//       4 B are finished here byte-serially; split records get out[r] = ~0.
//   crc32c_sorted_kernel: with C the total cost and G workgroups, workgroup b
//       takes the items whose cost starts in [C b / G, C (b + 1) / G), a
//       contiguous run of records.  It bins them by row count (largest
//       first; items of <= lrows rows after them, by 16-B block count),
//       builds the 16-B descriptor list in LDS (before the tables are
//       staged there) and writes it to the workspace in list order.  Its 16
//       waves take groups of 8 team items (one per team) from an LDS
//       counter, largest first (LPT).  A team hashes its item's 128-B rows
//       right-aligned to the group's row count (padded to a multiple of the
//       ring): ~init is XORed into the record's first 4 bytes (identity 3),
//       bytes outside the item are masked, rows before it are read from a
//       zero block, and crc = ~Z_{-m}(fold), m = ceil128(E) - E (in the loop
//       for the 4-row ring, else by a finish pass in record order).  Then
//       the lane items, 64 per grab, one per lane: slice-by-16 over the
//       blocks, no fold, no finish.
//   Records longer than a piece (2-64 KiB, by batch size) are cut into
//   pieces from their end; each piece XORs Z_{E - pe}(raw(piece)) into
//   out[r] (identity 1).
// No plan/finalize passes over the items: one small launch, then the hash.
// ---------------------------------------------------------------------------
constexpr uint64_t kSortPiece = 65536;                            // bytes per piece of a split record
// rows of the largest item: a 64 KiB + 3 B head piece at an unaligned start (514)
constexpr uint32_t kSortRows = uint32_t(kSortPiece / kRowBytes) + 2;
// Lane items (round 4): whole records and heads spanning at most lrows <=
// kSortLaneRowsMax rows are hashed one per lane (slice-by-16 over the 16-B
// blocks they touch), binned by block count K after the team items:
// bin = kSortRows - rows for team items, kSortRows - lrows + 8 lrows - K for
// lane items (K <= 8 lrows).
constexpr uint32_t kSortBins = kSortRows + 7 * kSortLaneRowsMax;
// rows per ring of the sorted kernel: a template parameter (2 for 64 KiB pieces;
// 4 measured slower there: profiles/r03_sorted_wave_roles_ab.txt)
// XCD-weighted shares: workgroup b runs on XCD b % 8 (round-robin dispatch),
// and in every timeline measured (round 2's stamped builds, 5 GPU sessions,
// profiles/r02_sorted_stamps_timeline.txt)
// the odd XCDs finished configs[2] 10-30 us after the even ones with equal
// shares.  Even workgroups take kSortXcdw/1000 more cost, odd ones as much
// less (A/B against equal shares: 0.878-0.905 ms vs 0.885-0.916 at 20;
// 15 is the default, 0 turns it off).
// (round 4, with the edge-row policy: 0 / 30 measured 0.796-0.797 /
// 0.792-0.793 ms against 0.788-0.791 at 15, profiles/r04_configs2_variants_ab.txt;
// round 5, final kernel: 0 / 30 0.772-0.774 / 0.768-0.769 against 0.765 at
// 15, profiles/r05_xcd_weight_lane_rows_ab.txt; MI_SORT_XCDW builds A/B variants)
#ifndef MI_SORT_XCDW
#define MI_SORT_XCDW 15
#endif
constexpr uint32_t kSortXcdw = MI_SORT_XCDW;
#ifndef MI_SORT_FOLD_COST
#define MI_SORT_FOLD_COST 2
#endif
constexpr uint32_t kSortFold = MI_SORT_FOLD_COST;            // cost allowance per item, in rows (fold, masks)
constexpr uint32_t kSortPer = 1;             // records per thread of a cost block
constexpr uint32_t kSortRecs = kPlanThreads * kSortPer;
constexpr uint32_t kSortMulti = 0x80000000u;  // descriptor flag: a piece of a split record
constexpr uint32_t kSortFirst = 0x40000000u;  // ... its first piece (carries the init)
constexpr uint32_t kSortRecMask = 0x3FFFFFFFu;
constexpr uint32_t kSortNone = 0xFFFFFFFFu;   // team without an item
constexpr uint32_t kSortJJNone = 0xFFFFu;     // descriptor: the piece's E - pe not held (read off/len)
#ifndef MI_SORT_JJ
#define MI_SORT_JJ 1  // A/B builds: 0 = every piece's shift from off[] / len[] (round 5)
#endif

uint32_t sorted_blocks(uint64_t count) { return uint32_t((count + kSortRecs - 1) / kSortRecs); }

struct SortCost
{
    uint64_t cost;       // all the record's items
    uint32_t n;          // items (pieces); 0: finished by sorted_cost_kernel (L < 4)
    uint32_t c_int;      // cost of every piece but the last (in cost order: the full pieces)
    uint32_t rows_full;  // rows of every piece but the last
    uint32_t rows_last;  // rows of the last piece in cost order: the head
    uint32_t blk_last;   // 16-B blocks the head touches (lane items)
};

// Pieces are cut from the record's END (round 4): the full pieces are
// [E - P (j + 1), E - P j), so a piece's part of the record CRC is
// Z_{P j}(raw(piece)), a shift by popcount(j) table lookups (cut from the
// start, the shift was E - pe = any length: up to 17 dependent L2 lookup
// rounds per piece, which small batches of 4 KiB pieces waited for).  The
// head [a, E - P (n - 1)) takes what is left, at least 4 bytes so that the
// ~init word stays inside it (a shorter remainder joins the next piece: the
// head then has up to P + 3 bytes).  In piece order the full pieces come
// first (piece i < n - 1 is the full piece ending P (n - 2 - i) before E) and
// the head last, so every piece but the last in that order costs c_int.
__device__ __forceinline__ SortCost sort_cost(uint64_t a, uint32_t L, uint32_t plog)
{
    SortCost s{0, 0, 0, 0, 0, 0};
    if (L < 4) return s;
    const uint64_t piece = uint64_t(1) << plog;
    s.n = uint32_t((uint64_t(L) + piece - 1) >> plog);
    if (s.n > 1 && uint64_t(L) - (uint64_t(s.n - 1) << plog) < 4) --s.n;  // head >= 4 bytes
    const uint64_t E = a + L;
    s.rows_full = uint32_t(piece / kRowBytes) + ((E & (kRowBytes - 1)) ? 1u : 0u);
    const uint64_t he = E - (uint64_t(s.n - 1) << plog);  // the head's end
    s.rows_last = uint32_t(((he + kRowBytes - 1) >> 7) - (a >> 7));
    s.blk_last = uint32_t(((he + 15) >> 4) - (a >> 4));
    s.c_int = s.rows_full + kSortFold;
    s.cost = uint64_t(s.n - 1) * s.c_int + s.rows_last + kSortFold;
    return s;
}

// The record's last item (in cost order) is a lane item.
__device__ __forceinline__ bool sort_is_lane(const SortCost& s, uint32_t lrows)
{
    return s.rows_last <= lrows;
}

// Bin of the last item: team items by rows (largest first), then lane items
// by 16-B blocks (largest first).
__device__ __forceinline__ uint32_t sort_key(const SortCost& s, uint32_t lrows)
{
    return sort_is_lane(s, lrows) ? kSortRows + 7 * lrows - s.blk_last : kSortRows - s.rows_last;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), l));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), l));
    return uint64_t(lo) | (uint64_t(hi) << 32);
}

// Two or four cost blocks per launch block, every load issued first, gave
// kernel minimums of 6.2 and 6.5 us against 7.2 but did not move the step
// (5 interleaved rounds, profiles/r02_sorted_cost_kernel_ab.txt).  Round 5,
// on the current hash kernel: two per launch block took configs[2] (1,024
// cost blocks) 1-2 us faster (better in 7 of 8 interleaved pairs) and 64 /
// 256 MiB batches (15-58 cost blocks) 0.3-0.5 us slower; four was mixed
// (profiles/r05_cost_blocks_ab.txt).  So X = 2 from 512 cost blocks on.
template <uint32_t X>
__global__ __launch_bounds__(kPlanThreads) void sorted_cost_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ inits, uint64_t count,
    uint64_t* __restrict__ blk_cost, uint32_t* __restrict__ ctrl, uint32_t* __restrict__ out,
    const uint32_t* __restrict__ tables, uint32_t plog)
{
    static_assert(kSortPer == 1, "one record per thread and cost block");
    __shared__ uint64_t sh[X][kPlanThreads / 64];
    uint64_t av[X];
    uint32_t Lv[X];
#pragma unroll
    for (uint32_t x = 0; x < X; ++x)
    {
        const uint64_t r = (uint64_t(blockIdx.x) * X + x) * kPlanThreads + threadIdx.x;
        av[x] = r < count ? off[r] : 0;
        Lv[x] = r < count ? len[r] : 4u;  // past the end: no cost, no store
    }
#pragma unroll
    for (uint32_t x = 0; x < X; ++x)
    {
        const uint64_t r = (uint64_t(blockIdx.x) * X + x) * kPlanThreads + threadIdx.x;
        uint64_t c = 0;
        if (r < count)
        {
            const uint8_t* p = base + av[x];
            const uint32_t L = Lv[x];
            if (L < 4)
            {
                uint32_t h = ~(inits ? inits[r] : 0u);
                for (uint32_t i = 0; i < L; ++i) h = tables[kTabT + ((h ^ p[i]) & 0xFFu)] ^ (h >> 8);
                out[r] = ~h;
            }
            else
            {
                const SortCost sc = sort_cost(uint64_t(p), L, plog);
                c = sc.cost;
                if (sc.n > 1) out[r] = ~0u;  // the pieces XOR their parts in
            }
        }
        for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
        if ((threadIdx.x & 63u) == 0) sh[x][threadIdx.x >> 6] = c;
    }
    __syncthreads();
    if (threadIdx.x < X)
    {
        const uint32_t x = threadIdx.x;
        uint64_t t = 0;
        for (uint32_t w = 0; w < kPlanThreads / 64; ++w) t += sh[x][w];
        const uint64_t cb = uint64_t(blockIdx.x) * X + x;
        if (cb * kPlanThreads < count) blk_cost[cb] = t;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
    {
        ctrl[1] = 0;  // overflow flag
    }
}


// Full pieces one workgroup's share can hold: its items are those whose cost
// starts in [T_b, T_b+1), at most C (1000 + w) / (1000 G) + 2 wide (the
// XCD-weighted share, rounding included), and full pieces cost c_f = P/128 +
// kSortFold or more each.  The host sizes the workspace with an upper bound
// of C (total/128 + 4 items); the kernel places workgroup b's full pieces at
// b x sorted_fpw(C, ...) from the exact C.
__host__ __device__ inline uint64_t sorted_fpw(uint64_t C, uint32_t plog, uint64_t grid)
{
    const uint64_t share = C / (1000 * grid) * (1000 + kSortXcdw) +
                           (C % (1000 * grid)) * (1000 + kSortXcdw) / (1000 * grid) + 2;
    return share / ((uint64_t(1) << plog) / kRowBytes + kSortFold) + 3;
}

// LDS of the sorted kernel beyond the table image.
struct SortShared
{
    uint32_t bins[kSortBins];  // whole records / last pieces per bin, then bin bases
    uint32_t fbins[2];         // full pieces of split records with 513 / 512 rows
    uint32_t n_items;
    uint32_t n_full;           // full pieces (listed first: the largest items)
    uint32_t full_base;        // their slots: items[count + full_base ...]
    uint32_t next_group;
    uint32_t next_lane;        // lane items taken (64 per grab)
    uint32_t teams_done;       // waves whose team groups are done (finish overlap)
    uint32_t next_fin;         // finish-pass records taken
    uint32_t lane_base;        // the first lane item's position among the last pieces
    uint32_t bound[4];         // (record, piece) of the first item and of the end
    uint32_t blk[2];           // cost blocks holding the two targets (nb: none)
    uint32_t bar_ok;           // fused launch: the grid barrier completed
    uint32_t sink;             // prefetch results' sink (never written in practice)
    uint64_t pre[2];           // cost before those blocks
    uint64_t target[2];
    uint64_t total;            // the batch's total cost C
    uint64_t wsum[kBlock / 64];
    uint32_t zinv[1024];       // Z_{-128} (the finish, in the loop or after it)
};
constexpr uint32_t kLdsSorted = kLdsBytes + uint32_t((sizeof(SortShared) + 255) & ~size_t(255));
static_assert(kLdsSorted <= 163840, "sorted kernel LDS");
static_assert(kSortRecs == 2 * 512, "sort_resolve: 512 threads x 2 records per cost block");

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x)
{
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
    {
        const uint64_t y = __shfl_up(x, d);
        if (lane >= uint32_t(d)) x += y;
    }
    return x;
}

// Exclusive prefix of v over the 1024-thread workgroup, and the total.
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t* wsum, uint64_t& total)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t x = wave_incl_scan64(v);
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (uint32_t w = 0; w < kBlock / 64; ++w)
    {
        const uint64_t s = wsum[w];
        pre += w < wave ? s : 0;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

// Wave 0: the total cost C, the targets C b / G and C (b + 1) / G, and the
// cost blocks holding them.  Each lane takes 16 consecutive blocks per round;
// up to 1,024 blocks (1M records) the costs stay in registers, so the total
// and the search cost one round trip.
__device__ __forceinline__ void sort_find_blocks(const uint64_t* __restrict__ blk_cost, uint32_t nb,
                                                 uint64_t count, SortShared& S)
{
    constexpr uint32_t K = 16;
    const uint32_t lane = threadIdx.x & 63u;
    const bool one_round = nb <= 64 * K;
    uint64_t v[K], tot = 0;
    for (uint32_t c0 = 0; c0 < nb; c0 += 64 * K)
    {
#pragma unroll
        for (uint32_t k = 0; k < K; ++k)
        {
            const uint32_t j = c0 + lane * K + k;
            // sc1 loads: in a fused launch other workgroups stored these
            // costs (sc1, write-through) before the grid barrier
            v[k] = j < nb ? __hip_atomic_load(blk_cost + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        }
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) tot += v[k];
    }
    for (int d = 32; d >= 1; d >>= 1) tot += __shfl_xor(tot, d);
    const uint64_t G = gridDim.x, b = blockIdx.x;
    uint64_t T[2];
    T[0] = tot / G * b + (tot % G) * b / G;
    T[1] = b + 1 == G ? tot : tot / G * (b + 1) + (tot % G) * (b + 1) / G;
    if (kSortXcdw && !(G & 1))
    {
        // T(x) = C (1000 x + w (x & 1)) / (1000 G): share 1 + w/1000 for even
        // b, 1 - w/1000 for odd b; T(G) = C exactly
        auto at = [&](uint64_t x) {
            return x >= G ? tot : uint64_t(double(tot) * (double(x) * 1000.0 + kSortXcdw * double(x & 1)) /
                                           (double(G) * 1000.0));
        };
        T[0] = at(b);
        T[1] = at(b + 1);
    }
    if (lane == 0) S.total = tot;
    if (lane == 0)
        for (int h = 0; h < 2; ++h)
        {
            S.blk[h] = nb;  // past the end unless found
            S.pre[h] = 0;
            S.target[h] = T[h];
            S.bound[2 * h] = uint32_t(count);
            S.bound[2 * h + 1] = 0;
        }
    bool found[2] = {false, false};
    uint64_t carry = 0;
    for (uint32_t c0 = 0; c0 < nb && !(found[0] && found[1]); c0 += 64 * K)
    {
        uint64_t sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < K; ++k)
        {
            const uint32_t j = c0 + lane * K + k;
            if (!one_round)
                v[k] = j < nb ? __hip_atomic_load(blk_cost + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
            sum += v[k];
        }
        const uint64_t incl = carry + wave_incl_scan64(sum), excl = incl - sum;
#pragma unroll
        for (int h = 0; h < 2; ++h)
        {
            const bool mine = !found[h] && excl <= T[h] && T[h] < incl;
            if (mine)
            {
                uint64_t p = excl;
                uint32_t k = 0;
                while (p + v[k] <= T[h]) p += v[k++];  // stops inside this lane's run
                S.blk[h] = c0 + lane * K + k;
                S.pre[h] = p;
            }
            found[h] = found[h] || __builtin_amdgcn_ballot_w64(mine) != 0;
        }
        carry = readlane64(incl, 63);
    }
}

// The first item (record, piece) whose cost starts at or after each target:
// threads 512 h .. 512 h + 511 resolve target h inside its cost block (two
// records per thread), both at once.  Result in bound[2 h], bound[2 h + 1].
__device__ __forceinline__ void sort_resolve(const uint8_t* base, const uint64_t* off,
                                             const uint32_t* len, uint64_t count, uint32_t nb,
                                             SortShared& S, uint32_t plog)
{
    const uint32_t h = threadIdx.x >> 9, t = threadIdx.x & 511u;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t j = S.blk[h];
    const uint64_t r0 = uint64_t(j) * kSortRecs + 2 * t;
    SortCost sc[2];
    uint64_t mine = 0;
#pragma unroll
    for (uint32_t q = 0; q < 2; ++q)
    {
        sc[q] = SortCost{0, 0, 0, 0, 0, 0};
        if (j < nb && r0 + q < count)
            sc[q] = sort_cost(uint64_t(base) + off[r0 + q], len[r0 + q], plog);
        mine += sc[q].cost;
    }
    const uint64_t x = wave_incl_scan64(mine);
    if (lane == 63) S.wsum[wave] = x;
    __syncthreads();
    uint64_t start = x - mine;
    for (uint32_t w = 8 * h; w < wave; ++w) start += S.wsum[w];
    const uint64_t tl = S.target[h] - S.pre[h];
#pragma unroll
    for (uint32_t q = 0; q < 2; ++q)
    {
        if (sc[q].cost && start <= tl && tl < start + sc[q].cost)
        {
            const uint64_t i = (tl - start + sc[q].c_int - 1) / sc[q].c_int;  // first piece at/after
            S.bound[2 * h] = uint32_t(i < sc[q].n ? r0 + q : r0 + q + 1);
            S.bound[2 * h + 1] = uint32_t(i < sc[q].n ? i : 0);
        }
        start += sc[q].cost;
    }
    __syncthreads();
}

// Lanes of the wave (among `active` ones) with the same 10-bit key: one
// ballot per key bit (no contended LDS atomics when most keys repeat).
__device__ __forceinline__ uint64_t match_key10(uint32_t key, bool active)
{
    uint64_t eq = __builtin_amdgcn_ballot_w64(active);
#pragma unroll
    for (int b = 0; b < 10; ++b)
    {
        const bool bit = (key >> b) & 1u;
        const uint64_t m = __builtin_amdgcn_ballot_w64(bit);
        eq &= bit ? m : ~m;
    }
    return eq;
}

// A team's view of its item within the group window [w1 - 128 n, w1) of n rows.
struct SortView
{
    uint64_t p0;     // this lane's 16 B in window row 0
    int32_t f;       // the item's first row (n - rows)
    int32_t lo, hi;  // rows in which this lane reads item bytes (lo > hi: none)
    uint4 kf;        // row f: keep masks (bytes from the item start on)
    uint4 xf;        // row f: ~init over the record's first 4 bytes (0: none)
    uint32_t xs;     // row f + 1, dword 0: the init word's spill (0: none)
    uint4 ke;        // row n - 1: keep masks (bytes before the item end)
    uint32_t m;      // bytes masked after the item in the last row
    uint32_t recf;   // record | flags, kSortNone: no item
    uint32_t slot;   // the item's descriptor slot (whole records)
    uint32_t jj;     // a piece's E - pe in pieces (kSortJJNone: not held)
};


__device__ __forceinline__ uint64_t sort_addr(const uint4& d)
{
    return uint64_t(d.x) | (uint64_t(d.y & 0xFFFFu) << 32);
}

__device__ __forceinline__ uint32_t sort_rows(const uint4& d)
{
    const uint64_t ps = sort_addr(d);
    return d.z ? uint32_t(((ps + d.z + kRowBytes - 1) >> 7) - (ps >> 7)) : 0u;
}

// ~init placed at byte offset q of a 16-B block (q in -3..15), dword k.
__device__ __forceinline__ uint32_t init_dword(uint32_t ninit, int32_t q, int k)
{
    const int32_t dd = 4 * k - q;  // init byte 0 sits dd bytes before this dword
    const uint32_t s = uint32_t(min(max(32 + 8 * dd, 0), 63));
    const uint32_t x = uint32_t((uint64_t(ninit) << 32) >> s);
    return (dd > -4 && dd < 4) ? x : 0u;
}

// The masks depend on the record's init, loaded here (when there is an init
// array) and consumed a group later (sort_view runs for the NEXT group).
// 32-bit window arithmetic (an item spans < 2^17 bytes); one 64-bit add for
// the row pointer.  The init word: (hi:lo) = ~init << 8 (q & 3) goes to
// dwords q>>2 and q>>2 + 1 of the lane's block (q = the record's first byte
// there, -3..15), or to row f + 1 (lane 0, q >= 125).  (Against five 64-bit
// shifts per view: SQ_INSTS_VALU -9 % on the < 256 B class.)
__device__ __forceinline__ SortView sort_view(const uint4& d, int32_t n, uint32_t tl,
                                              const uint32_t* __restrict__ inits,
                                              const uint32_t* __restrict__ ones_word)
{
    SortView v;
    const uint32_t L = d.z;
    const int32_t s0 = int32_t(d.x & (kRowBytes - 1));
    const int32_t se = s0 + int32_t(L);
    const int32_t rows = L ? (se + int32_t(kRowBytes) - 1) >> 7 : 0;
    v.recf = L ? d.w : kSortNone;
    v.jj = d.y >> 16;
    v.f = n - rows;
    const uint64_t ps = sort_addr(d);
    v.p0 = ps + int64_t(int32_t(uint32_t(rows - n) * kRowBytes + tl * 16u) - s0);
    const int32_t q = s0 - int32_t(tl) * 16;
    const int32_t bs = min(max(q, 0), 16);
    const int32_t ce = min(max(se - (rows - 1) * int32_t(kRowBytes) - int32_t(tl) * 16, 0), 16);
    v.lo = L ? v.f + (bs >= 16 ? 1 : 0) : n;
    v.hi = L ? n - 1 - (ce == 0 ? 1 : 0) : -1;
    v.m = uint32_t(rows * int32_t(kRowBytes) - se);
    v.kf = make_uint4(keep_from(bs, 0), keep_from(bs, 1), keep_from(bs, 2), keep_from(bs, 3));
    v.ke = make_uint4(keep_below(ce, 0), keep_below(ce, 1), keep_below(ce, 2), keep_below(ce, 3));
    const bool with_init = L && (!(d.w & kSortMulti) || (d.w & kSortFirst));
    // With an init array: one load per lane (all ones, i.e. ~init = 0, where
    // no init word goes in).  Without one (a uniform kernel argument): no load
    // and no wait, ~init is all ones where the init word goes in, 0 elsewhere
    // (round 3 A/B, profiles/r03_sorted_initskip_ab.txt: -1.5 to -2 us per
    // configs[2] step).
    const uint32_t ninit = inits ? ~*(!with_init ? ones_word : inits + (d.w & kSortRecMask))
                                 : (with_init ? 0xFFFFFFFFu : 0u);
    const uint64_t sh = uint64_t(ninit) << ((uint32_t(q) & 3u) * 8u);
    const uint32_t xl = uint32_t(sh), xh = uint32_t(sh >> 32);
    const int32_t qd = q >> 2;  // arithmetic: -1 for q in -3..-1
    v.xf = make_uint4(qd == 0 ? xl : qd == -1 ? xh : 0u, qd == 1 ? xl : qd == 0 ? xh : 0u,
                      qd == 2 ? xl : qd == 1 ? xh : 0u, qd == 3 ? xl : qd == 2 ? xh : 0u);
    v.xs = q >= int32_t(kRowBytes) - 3 ? xh : 0u;
    return v;
}

// The raw-CRC step over one 16-B block x (the state already XORed into its
// first word) of which only bytes 0 .. t-1 are data (bytes >= t are zero;
// t = 1..16): byte p goes through T_{t-1-p}; for t < 4 the state bytes
// past the data shift down.  Lookups of p >= t read some other LDS word
// (T_{t-1-p} < T_0: the G^{128} image) and are dropped.
__device__ __forceinline__ uint32_t lane_tail_step(const uint4& x, uint32_t t)
{
    uint32_t r = t < 4u ? x.x >> (8u * t) : 0u;
    const uint32_t tb = kLdsT + (t - 1u) * 1024u;  // T_{t-1}
#pragma unroll
    for (int p = 0; p < 16; ++p)
    {
        const uint32_t wv = p < 4 ? x.x : p < 8 ? x.y : p < 12 ? x.z : x.w;
        const uint32_t v = lds32(tb - uint32_t(p) * 1024u + ((wv >> (8 * (p & 3))) & 0xFFu) * 4u);
        r ^= int32_t(t) - 1 - p >= 0 ? v : 0u;
    }
    return r;
}

__device__ __forceinline__ uint32_t zshift48(const uint32_t* __restrict__ pow2, uint32_t v, uint64_t n)
{
    for (int k = 0; n && k < 48; ++k, n >>= 1)
        if (n & 1u) v = zglob(pow2 + k * 1024, v);
    return v;
}

// Z_{P jj}(v), a piece's shift to its record's end: one lookup in the Z_{512 k}
// sets when P jj / 512 < 256 (4-16 KiB pieces of records up to 128 KiB),
// else popcount lookups in the G^{2^k} sets.
__device__ __forceinline__ uint32_t zshift_piece(const uint32_t* __restrict__ tables,
                                                 const uint32_t* __restrict__ pow2, uint32_t v, uint64_t n)
{
    const uint64_t k = n >> 9;
    if ((n & 511u) == 0 && k - 1 < uint64_t(kWinShifts - 1)) return zglob(tables + kTabZWin + (k - 1) * 1024u, v);
    return zshift48(pow2, v, n);
}

// One-launch form (round 5, VERDICT r4 Next 1a): the work of
// sorted_cost_kernel done by the hash kernel's own workgroups, then a grid
// barrier, so the batch needs no second launch.  Workgroup b computes cost
// blocks b, b + G, ... (up to four per round, every load issued first),
// stores each block's sum and every split record's ~0 (the identity its
// pieces XOR into) with write-through (sc1) stores, drains them (vmcnt(0),
// every wave), and arrives at the barrier: one agent-scope add per workgroup
// on a monotonic counter (ctrl[32]; this launch's arrivals take it from
// bar_base to bar_base + G), polled with sc1 loads (MI355X_MICROARCH.md,
// inter-workgroup visibility, the table's first row: sc1 stores, one atomic
// add per workgroup, sc1 loads of the handed-off words -- sort_find_blocks
// reads the block costs with sc1 loads; the pieces' XORs are memory-side
// atomics, after the barrier).  The engine launches this form only when the
// grid fits one workgroup per CU and no other thread's context of the
// process uses the sorted path on the device (two barrier launches sharing
// the CUs could wait on each other); even so the wait is bounded: after
// kSortBarrierTicks the workgroup stores ctrl[3] = bar_base + G + 1 (and the
// sticky ctrl[2]) and returns, and the host recomputes the batch with the two
// launches (a synchronous batch) or reports it at the next stream sync.
constexpr uint64_t kSortBarrierTicks = 5000000;  // 50 ms at s_memrealtime's 100 MHz
template <typename SS>
__device__ __forceinline__ bool sorted_fused_costs(const uint8_t* base, const uint64_t* off,
                                                   const uint32_t* len, const uint32_t* inits,
                                                   uint64_t count, uint64_t* blk_cost, uint32_t nb,
                                                   uint32_t* ctrl, uint32_t* out,
                                                   const uint32_t* tables, uint32_t plog,
                                                   uint32_t bar_base, SS& S)
{
    constexpr uint32_t CX = 4;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t G = gridDim.x;
    // per-wave sums in the table image's LDS (free until the binning)
    uint64_t* const wsum = reinterpret_cast<uint64_t*>(smem);
    for (uint64_t j0 = blockIdx.x; j0 < nb; j0 += CX * G)
    {
        uint64_t av[CX];
        uint32_t Lv[CX];
#pragma unroll
        for (uint32_t x = 0; x < CX; ++x)
        {
            const uint64_t r = (j0 + x * G) * kSortRecs + threadIdx.x;
            const bool in = j0 + x * G < nb && r < count;
            av[x] = in ? off[r] : 0;
            Lv[x] = in ? len[r] : 0;
        }
#pragma unroll
        for (uint32_t x = 0; x < CX; ++x)
        {
            const uint64_t r = (j0 + x * G) * kSortRecs + threadIdx.x;
            const bool in = j0 + x * G < nb && r < count;
            uint64_t c = 0;
            if (in)
            {
                const uint8_t* p = base + av[x];
                const uint32_t L = Lv[x];
                if (L < 4)
                {
                    uint32_t h = ~(inits ? inits[r] : 0u);
                    for (uint32_t i = 0; i < L; ++i) h = tables[kTabT + ((h ^ p[i]) & 0xFFu)] ^ (h >> 8);
                    out[r] = ~h;
                }
                else
                {
                    const SortCost sc = sort_cost(uint64_t(p), L, plog);
                    c = sc.cost;
                    if (sc.n > 1) __hip_atomic_store(out + r, ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
            if (lane == 0) wsum[x * 16 + wave] = c;
        }
        __syncthreads();
        if (threadIdx.x < CX && j0 + threadIdx.x * G < nb)
        {
            uint64_t t = 0;
            for (uint32_t w = 0; w < kBlock / 64; ++w) t += wsum[threadIdx.x * 16 + w];
            __hip_atomic_store(blk_cost + j0 + threadIdx.x * G, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(ctrl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // overflow flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 stores written through
    __syncthreads();
    if (threadIdx.x == 0)
    {
        __hip_atomic_fetch_add(ctrl + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = true;
        while (uint32_t(__hip_atomic_load(ctrl + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - bar_base) <
               uint32_t(G))
        {
            if (__builtin_amdgcn_s_memrealtime() - t0 > kSortBarrierTicks)
            {
                ok = false;
                __hip_atomic_store(ctrl + 3, bar_base + uint32_t(G) + 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(ctrl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        S.bar_ok = ok;
    }
    __syncthreads();
    return S.bar_ok != 0;
}

// Phase stamps of the sorted kernel (dev builds only: tools/build_variant.sh
// TAG -DMI_SORT_STAMP=1, read by tools/sort_stamps.py through
// mi_debug_sort_stamps): lane 0 of every wave of workgroups < 256 stores
// s_memrealtime (100 MHz) at 8 points -- entry, cost blocks found,
// boundaries resolved, binning pass done, first group (tables staged), team
// groups done, lane items done, finish done.  Off in the product build.
#ifndef MI_SORT_STAMP
#define MI_SORT_STAMP 0
#endif
#ifndef MI_SORT_LANE_BLOCKS
#define MI_SORT_LANE_BLOCKS 16
#endif
#ifndef MI_SORT_FIN_OVERLAP
#define MI_SORT_FIN_OVERLAP 1
#endif
#ifndef MI_SORT_PREFETCH
#define MI_SORT_PREFETCH 1
#endif
// Timing ablation (dev builds only, wrong CRCs for the records it skips):
// MI_SORT_ABL_LANE=1 leaves the lane items unhashed, to bound what any faster
// lane phase could return (profiles/r06_lane_phase_ablation.txt).
#ifndef MI_SORT_ABL_LANE
#define MI_SORT_ABL_LANE 0
#endif
#if MI_SORT_STAMP
__device__ uint64_t g_sort_stamp[256 * 16 * 8];
// where each workgroup ran: HW_ID (cu, sh, se fields) and XCC_ID (round 6)
__device__ uint32_t g_sort_hw[256 * 2];
#define SORT_STAMP(k)                                                                        \
    do                                                                                       \
    {                                                                                        \
        if ((threadIdx.x & 63u) == 0 && blockIdx.x < 256)                                    \
            g_sort_stamp[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 + (k)] =                 \
                __builtin_amdgcn_s_memrealtime();                                            \
    } while (0)
#else
#define SORT_STAMP(k) \
    do                \
    {                 \
    } while (0)
#endif

template <int RB>
__global__ __launch_bounds__(kBlock, 1) void crc32c_sorted_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ inits, uint64_t count,
    uint64_t* __restrict__ blk_cost, uint32_t nb, uint32_t* __restrict__ ctrl,
    uint4* __restrict__ items, uint64_t item_cap, uint32_t* __restrict__ wr, uint32_t* __restrict__ out,
    const uint32_t* __restrict__ tables, const uint32_t* __restrict__ pow2, uint32_t plog,
    uint32_t lrows, int fused, uint32_t bar_base)
{
    SortShared& S = *reinterpret_cast<SortShared*>(smem + kLdsBytes);
    const uint64_t piece = uint64_t(1) << plog;
    const uint32_t rows_max = uint32_t(piece / kRowBytes) + 1;  // rows of a full piece, unaligned
    const uint32_t lane = threadIdx.x & 63u;
    if (threadIdx.x < kSortBins) S.bins[threadIdx.x] = 0;
    if (threadIdx.x < 2) S.fbins[threadIdx.x] = 0;
    if (threadIdx.x == 0) S.next_group = 0;
    if (threadIdx.x == 0) S.next_lane = 0;
    if (threadIdx.x == 0) S.teams_done = 0;
    if (threadIdx.x == 0) S.next_fin = 0;
    // small batches finish each whole record right after its fold (below):
    // Z_{-128} is staged with the tables
    // whole records finished in the loop (RB = 4, small batches) or by the
    // finish pass (RB = 2, configs[2]: in the loop it measured 0.829-0.831
    // ms against 0.788-0.791, profiles/r04_configs2_variants_ab.txt)
    constexpr bool INLOOP = RB >= 4;
    if (INLOOP || MI_SORT_FIN_OVERLAP) S.zinv[threadIdx.x] = tables[kTabZInv128 + threadIdx.x];
    // (1) Wave 0: the two targets and the cost blocks holding them.  (The
    // tables reach the LDS later, at the stage_tables_store() call after the
    // binning has written the descriptor list out: until then their LDS holds
    // the list, so no table lookup may come before that call.)
    SORT_STAMP(0);
#if MI_SORT_STAMP
    if (threadIdx.x == 0 && blockIdx.x < 256)
    {
        g_sort_hw[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);       // HW_REG_HW_ID
        g_sort_hw[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    }
#endif
    if (fused && !sorted_fused_costs(base, off, len, inits, count, blk_cost, nb, ctrl, out, tables,
                                     plog, bar_base, S))
        return;  // the grid barrier timed out: ctrl[3] tells the host (below)
    if (threadIdx.x < 64)
        sort_find_blocks(blk_cost, nb, count, S);
#if MI_SORT_PREFETCH
    else
    {
        // (round 5) While wave 0 searches the cost blocks, the other waves
        // read the middle of this workgroup's likely record range (the
        // record-count share: a cost share is near it) so that the binning
        // pass's offset and length loads hit L2.
        const uint64_t per = count / gridDim.x;
        const uint64_t r0 = uint64_t(blockIdx.x) * per + per / 8;
        const uint64_t re = r0 + per - per / 4;
        constexpr uint32_t PF = 4;  // records per thread, every load issued first
        uint64_t o[PF];
        uint32_t l[PF];
#pragma unroll
        for (uint32_t u = 0; u < PF; ++u)
        {
            const uint64_t r = r0 + threadIdx.x - 64 + u * (kBlock - 64);
            o[u] = r < re ? off[r] : 0;
            l[u] = r < re ? len[r] : 0;
        }
        uint64_t acc = 0;
#pragma unroll
        for (uint32_t u = 0; u < PF; ++u) acc += o[u] + l[u];
        if (acc == 0x5A5A5A5A5A5A5A5Aull) S.sink = uint32_t(acc);
    }
#endif
    __syncthreads();
    SORT_STAMP(1);
    // The tables are staged after the binning (step 3), which uses their LDS
    // to put the descriptors in list order first.
    constexpr uint32_t kLdsZInv = kLdsBytes + uint32_t(offsetof(SortShared, zinv));
    // (2) Exact (record, piece) boundaries of this workgroup's items.
    sort_resolve(base, off, len, count, nb, S, plog);
    SORT_STAMP(2);

    // (3) Bin the items by row count, largest first.  Whole records and the
    // last pieces of split records go to this workgroup's slots of the
    // record-indexed list, items[rlo ...] (a record has one last piece, so the
    // ranges never overlap); the full 64 KiB pieces of split records, 512 or
    // 513 rows, to slots taken from ctrl[0] past items[count] and are listed
    // first.  Ranks come from returning LDS atomics: one per distinct row
    // count of a wave (match_key10).  Up to 8 records per thread the ranks
    // stay in registers and the descriptors are written after the bin scan;
    // larger ranges take a second pass over the records.
    const uint32_t rlo = S.bound[0], klo0 = S.bound[1], rhi = S.bound[2], khi0 = S.bound[3];
    const uint64_t rend = min(uint64_t(rhi) + (khi0 ? 1u : 0u), count);
    constexpr uint32_t U = 4, CH = 2;  // records per thread per chunk, chunks held
    const bool held = rend <= uint64_t(rlo) + U * CH * kBlock;
    struct RecInfo
    {
        SortCost s;
        uint32_t klo, nf;
        bool last;
    };
    auto info = [&](uint64_t r, uint64_t a, uint32_t L) {
        RecInfo f;
        f.s = sort_cost(a, L, plog);  // L = 0 past rend: no items
        f.klo = r == rlo ? klo0 : 0u;
        const uint32_t khi = r == rhi ? khi0 : f.s.n;
        const uint32_t lim = f.s.n ? f.s.n - 1 : 0u;  // pieces before the last
        f.nf = min(khi, lim) > f.klo ? min(khi, lim) - f.klo : 0u;
        f.last = f.s.n != 0 && f.klo < khi && khi == f.s.n;
        return f;
    };
    // one returning atomic per full-piece run and per wave leader of a row
    // count; returns (full rank or cursor, last-piece rank or cursor)
    auto take = [&](const RecInfo& f, uint32_t& rf, uint32_t& rl) {
        rf = f.nf ? atomicAdd(&S.fbins[f.s.rows_full == rows_max ? 0 : 1], f.nf) : 0u;
        const uint32_t key = sort_key(f.s, lrows);
        const uint64_t eq = match_key10(key, f.last);
        const uint32_t rank = uint32_t(__builtin_popcountll(eq & ((uint64_t(1) << lane) - 1)));
        uint32_t b0 = 0;
        if (f.last && rank == 0) b0 = atomicAdd(&S.bins[key], uint32_t(__builtin_popcountll(eq)));
        b0 = uint32_t(__shfl(int(b0), f.last ? int(__builtin_ctzll(eq)) : int(lane)));
        rl = b0 + rank;
    };
    // piece k in cost order: k < n - 1 the full piece ending P (n - 2 - k)
    // before E, k = n - 1 the head (carries the init)
    auto desc = [&](uint64_t r, uint64_t a, uint32_t L, const RecInfo& f, uint32_t k) {
        const uint64_t E = a + L;
        const bool head = k + 1 == f.s.n;
        const uint64_t pe = E - (uint64_t(head ? f.s.n - 1 : f.s.n - 2 - k) << plog);
        const uint64_t ps = head ? a : pe - piece;
        // a piece's E - pe = P jj: jj in the top 16 bits of the address word
        // (addresses are < 2^48), so its shift needs no off/len reads (kSortJJNone: read them)
        const uint64_t jj = (E - pe) >> plog;
        const uint32_t jw = f.s.n > 1 && MI_SORT_JJ ? uint32_t(min(jj, uint64_t(kSortJJNone))) << 16
                                                    : uint32_t(kSortJJNone) << 16;
        return make_uint4(uint32_t(ps), uint32_t(ps >> 32) | jw, uint32_t(pe - ps),
                          uint32_t(r) | (f.s.n > 1 ? kSortMulti : 0u) | (head ? kSortFirst : 0u));
    };
    uint4* const fullv = items + count;
    uint4* const lastv = items + rlo;
    // absolute slots: full run at fpos, last piece at lpos
    // Descriptors go out with non-temporal stores: the ~2 MB of them per XCD
    // then do not sit dirty in the XCD's 4 MB L2 through the hash phase
    // (measured: prologue 8 us longer, step 8-10 us shorter).  The group loop
    // reads them two groups ahead (non-temporal loads there: neutral).
    auto put = [&](uint4* dst, const uint4& dv) {
        __builtin_nontemporal_store(make_u32x4(dv), reinterpret_cast<u32x4_t*>(dst));
    };
    // Up to kLdsBytes / 16 items, the descriptors go to LDS at their list
    // position (the table image's space: the tables are staged after), and
    // then out in list order, whole lines: scattered 16-B stores cost the
    // configs[2] prologue 19 us (profiles/r04_sorted_prologue_phases.txt).
    uint4* const stage_lds = reinterpret_cast<uint4*>(smem);
    bool staged = false;
    uint32_t stage_nf = 0;
    auto put_full = [&](uint32_t pos, const uint4& dv) {
        if (staged) stage_lds[pos] = dv;
        else put(fullv + S.full_base + pos, dv);
    };
    auto put_last = [&](uint32_t pos, const uint4& dv) {
        if (staged) stage_lds[stage_nf + pos] = dv;
        else put(lastv + pos, dv);
    };
    auto place = [&](uint64_t r, uint64_t a, uint32_t L, const RecInfo& f, uint32_t fpos, uint32_t lpos) {
        for (uint32_t i = 0; i < f.nf; ++i) put_full(fpos + i, desc(r, a, L, f, f.klo + i));
        if (f.last) put_last(lpos, desc(r, a, L, f, f.s.n - 1));
    };
    uint64_t ha[CH][U];
    uint32_t hL[CH][U], hf[CH][U], hl[CH][U];
    auto pass = [&](bool second) {
        for (uint32_t c = 0;; ++c)
        {
            const uint64_t c0 = uint64_t(rlo) + threadIdx.x + uint64_t(c) * U * kBlock;
            if (c0 >= rend) break;
            uint64_t av[U];
            uint32_t Lv[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
            {
                const uint64_t r = c0 + u * kBlock;
                av[u] = r < rend ? uint64_t(base) + off[r] : 0;
                Lv[u] = r < rend ? len[r] : 0;
            }
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
            {
                const uint64_t r = c0 + u * kBlock;
                const RecInfo f = info(r, av[u], Lv[u]);
                uint32_t rf, rl;
                take(f, rf, rl);
                if (second)
                    place(r, av[u], Lv[u], f, rf, rl);  // the bins hold cursors now
                else if (held)
#pragma unroll
                    for (uint32_t cc = 0; cc < CH; ++cc)
                        if (cc == c)
                        {
                            ha[cc][u] = av[u];
                            hL[cc][u] = Lv[u];
                            hf[cc][u] = rf;
                            hl[cc][u] = rl;
                        }
            }
        }
    };
    pass(false);
    __syncthreads();
    SORT_STAMP(3);
    // (round 6) The table image's global loads go out now, beside the bin
    // scan, the placement and the list's copy-out; they reach the LDS once
    // the list has left it (32 / 64 MiB batches 0.4-0.8 us faster, configs[2]
    // unchanged: profiles/r06_early_table_loads_ab.txt)
    TableRegs tregs;
    stage_tables_load(tregs, tables);
    {
        const uint32_t c = threadIdx.x < kSortBins ? S.bins[threadIdx.x] : 0u;
        uint64_t total;
        const uint32_t e = uint32_t(block_excl_scan64(c, S.wsum, total));
        if (threadIdx.x < kSortBins) S.bins[threadIdx.x] = e;
        if (threadIdx.x == kSortRows - lrows) S.lane_base = e;  // lane items follow the team items
        if (threadIdx.x == 0)
        {
            // full pieces go to this workgroup's own region of fpw slots
            // (sorted_fpw; round 3 took them from a global cursor: a round
            // trip in the prologue).  Every workgroup computes the same fpw
            // from the same C, so an understated total_bytes (workspace too
            // small) stops all of them alike.
            const uint32_t nf = S.fbins[0] + S.fbins[1];
            const uint64_t fpw = sorted_fpw(S.total, plog, gridDim.x);
            const uint32_t fb = uint32_t(blockIdx.x * fpw);
            S.n_full = nf;
            S.n_items = nf + uint32_t(total);
            if (nf > fpw || count + uint64_t(gridDim.x) * fpw > item_cap)
            {
                ctrl[1] = 1;  // workspace too small (understated total_bytes): out[] left alone
                ctrl[2] = 1;  // sticky: an asynchronous batch's is reported at the next stream sync
                S.n_items = 0;
            }
            S.full_base = fb;
            if (!held)  // cursors for the second pass
            {
                S.fbins[1] = S.fbins[0];
                S.fbins[0] = 0;
            }
        }
    }
    __syncthreads();
    const uint32_t n_items = S.n_items, n_full = S.n_full;
    staged = n_items <= kLdsBytes / 16;
    stage_nf = n_full;
    if (n_items)
    {
        if (held)
        {
            const uint32_t f513 = S.fbins[0];
#pragma unroll
            for (uint32_t c = 0; c < CH; ++c)
#pragma unroll
                for (uint32_t u = 0; u < U; ++u)
                {
                    const uint64_t r = uint64_t(rlo) + threadIdx.x + (uint64_t(c) * U + u) * kBlock;
                    if (r < rend)
                    {
                        const RecInfo f = info(r, ha[c][u], hL[c][u]);
                        const uint32_t fpos = (f.s.rows_full == rows_max ? 0u : f513) + hf[c][u];
                        place(r, ha[c][u], hL[c][u], f, fpos,
                              f.last ? S.bins[sort_key(f.s, lrows)] + hl[c][u] : 0u);
                    }
                }
        }
        else
            pass(true);
    }
    __syncthreads();
    if (n_items == 0) return;
    if (staged)
    {
        // list order out: full pieces to their region, the rest after rlo
        for (uint32_t i = threadIdx.x; i < n_items; i += kBlock)
            put(i < n_full ? fullv + S.full_base + i : lastv + (i - n_full), stage_lds[i]);
        __syncthreads();
    }
    stage_tables_store(tregs);  // ends with a barrier
    SORT_STAMP(4);
    // team items first, lane items (positions n_long ..) after them
    const uint32_t n_long = n_full + S.lane_base;

    // (4) Groups of 8 team items, largest first, one LDS grab per group.
    const uint32_t n_groups = (n_long + 7) / 8;
    const uint32_t tl = threadIdx.x & (kTeam - 1);
    const uint32_t tw = lane / kTeam;
    const uint32_t li = lane_info();
    const uint8_t* zero16 = reinterpret_cast<const uint8_t*>(tables + kTabZero);
    const uint32_t* ones_word = tables + kTabFInit;  // Z_0(~0) = 0xFFFFFFFF
    const uint32_t* zneg = tables + kTabZNeg;
    // A whole record's fold value goes to out[] right after its fold; the
    // finish pass after the loop applies Z_{-m} from LDS tables.  (Round 2-3
    // applied it in the loop from the 512 KB global Z_{-m} table, one lookup
    // per lane a group later: 4M scattered L2 lines per configs[2] step,
    // 10 us of it; profiles/r03_sorted_late_finish_ab.txt.)  Only a piece of
    // a split record still takes that lookup in the loop: its part,
    // Z_{E-pe}(raw(piece)), is XORed into out[] a group later.
    uint32_t pz = 0;               // this lane's Z_{-m} entry of the pending piece
    uint32_t p_recf = kSortNone;   // the pending piece's record | flags
    uint64_t p_pe = 0;             // its end (lane 0)
    uint32_t p_jj = kSortJJNone;   // its E - pe in pieces (kSortJJNone: from off/len)
    bool p_multi = false;          // wave-uniform: some team has a pending piece
    auto flush = [&]() {
        if (!p_multi) return;
        uint32_t v = pz;
        v ^= from_lane_up<1>(v);
        v ^= from_lane_up<2>(v);  // lane 0: Z_{-m}(fold) = raw(piece)
        if (tl == 0 && p_recf != kSortNone)
        {
            // this piece's part: Z_{E - pe}(raw(piece)), E the record's end
            const uint32_t rec = p_recf & kSortRecMask;
            if (p_jj != kSortJJNone)
            {
                // E - pe from the descriptor: no dependent off/len reads
                if (p_jj) v = zshift_piece(tables, pow2, v, uint64_t(p_jj) << plog);
            }
            else
            {
                const uint64_t a_rec = uint64_t(base) + off[rec];
                const uint32_t L_rec = len[rec];
                v = zshift48(pow2, v, a_rec + L_rec - p_pe);
            }
            __hip_atomic_fetch_xor(out + rec, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    auto grab = [&]() {
        uint32_t g = 0;
        if (lane == 0) g = atomicAdd(&S.next_group, 1u);
        return uint32_t(__builtin_amdgcn_readfirstlane(int(g)));
    };
    const uint4* const listF = items + count + S.full_base;  // full pieces first
    const uint4* const listL = items + rlo - n_full;          // then the rest
    auto load_desc = [&](uint32_t g) {
        const uint32_t i = g * 8 + tw;
        const uint4* p = (g < n_groups && i < n_long) ? (i < n_full ? listF : listL) + i
                                                       : reinterpret_cast<const uint4*>(zero16);
        return *p;
    };
    // Uniform shape of a group: n rows (its largest item, padded to an even
    // count with a leading zero row), the first row of that item, the last
    // row in which some team's item starts (or its init word spills into),
    // and the first row from which every lane reads item bytes (n: never, in
    // a group with teams but no item).  The list is descending except where
    // the 512-row full pieces meet the 513-row whole records (the full
    // pieces are listed first), so the largest and smallest item are taken
    // over the group's teams, not from its first and last.
    struct Shape
    {
        int32_t n, fmin, fedge, fast;
    };
    auto shape_of = [&](const uint4& d, uint32_t g) {
        Shape s{0, 0, 0, 0};
        if (g >= n_groups) return s;
        const uint32_t tlast = min(7u, n_long - 1 - g * 8);
        const int rv = int(sort_rows(d));
        int32_t rmax = 0, rmin = int32_t(kSortRows);
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t)
        {
            const int32_t x = __builtin_amdgcn_readlane(rv, int(t * kTeam));
            rmax = t <= tlast ? max(rmax, x) : rmax;
            rmin = t <= tlast ? min(rmin, x) : rmin;
        }
        s.n = (rmax + RB - 1) & ~(RB - 1);
        s.fmin = s.n - rmax;
        s.fedge = s.n - rmin + 1;
        s.fast = tlast == 7 ? s.fedge + 1 : s.n;
        return s;
    };
    auto row_ptr = [&](const SortView& v, int32_t r, bool fast) {
        const uint8_t* p = reinterpret_cast<const uint8_t*>(v.p0 + uint64_t(uint32_t(r)) * kRowBytes);
        if (!fast) p = (r >= v.lo && r <= v.hi) ? p : zero16;
        return p;
    };

    // (5) Lane items, 64 per grab, one per lane (lane
    // items).  A lane hashes the 16-B aligned blocks its item touches with
    // the slice-by-16 tables: bytes before the item are zeroed (leading zeros
    // leave the zero raw state at zero), ~init is XORed over its first 4
    // bytes, and the last block, holding t = 1..16 of the item's bytes, takes
    // the t-byte form of the step, so the state is the item's raw CRC with no
    // finish.  The list is ordered by block count, so the lanes of a wave run
    // about the same number of steps.  Blocks are read with the default
    // policy: a block's line is shared with the neighbouring records.
    // blocks of one lane item loaded at once (a multiple of 4; the rest of a
    // longer item takes another round)
    constexpr int32_t kLaneBlocks = MI_SORT_LANE_BLOCKS;
    auto lane_items = [&]() {
        if (MI_SORT_ABL_LANE) return;
        const uint32_t n_lane = n_items - n_long;
        const uint4* const listLane = listL + n_long;
        auto grab64 = [&]() {
            uint32_t c = 0;
            if (lane == 0) c = atomicAdd(&S.next_lane, 64u);
            return uint32_t(__builtin_amdgcn_readfirstlane(int(c)));
        };
        auto ldesc = [&](uint32_t c) {
            return c + lane < n_lane ? listLane[c + lane] : make_uint4(0, 0, 0, 0);
        };
        // Latency (round 5): a grab used to be three dependent global round
        // trips or more (its descriptors, then its blocks four at a time,
        // then the last block).  Now the next grab's descriptors are loaded
        // while this grab is hashed, and all of an item's blocks are issued at
        // once (up to 16 before the last: an item of <= 2 rows touches <= 17
        // blocks), the last block first; they are hashed four at a time, up
        // to the wave's largest item (the list is ordered by block count).
        uint32_t c0 = grab64();
        uint4 d = ldesc(c0);
        while (c0 < n_lane)
        {
            const uint32_t c1 = grab64();
            const uint4 d1 = ldesc(c1);
            const bool act = c0 + lane < n_lane;
            const uint64_t a = sort_addr(d);
            const uint64_t e = a + d.z;
            const uint32_t q = uint32_t(a) & 15u;
            const int32_t K = act ? int32_t(((e + 15) >> 4) - (a >> 4)) : 0;  // blocks, >= 1
            const uint32_t t = ((uint32_t(e) - 1u) & 15u) + 1u;                // item bytes' end in the last block
            const uint32_t rec = d.w & kSortRecMask;
            const uint8_t* const pb = reinterpret_cast<const uint8_t*>(a & ~uint64_t(15));
            const int32_t nb = K - 1;  // blocks before the last
            uint4 xl = load16_edge(act ? pb + 16 * (K - 1) : zero16);
            const bool with_init = !(d.w & kSortMulti) || (d.w & kSortFirst);
            const uint32_t ninit = !with_init ? 0u : inits ? (act ? ~inits[rec] : 0u) : 0xFFFFFFFFu;
            const uint64_t shi = uint64_t(ninit) << ((q & 3u) * 8u);
            const uint32_t xlo = uint32_t(shi), xhi = uint32_t(shi >> 32);
            const uint32_t qd = q >> 2;
            const uint4 xf = make_uint4(qd == 0 ? xlo : 0u, qd == 1 ? xlo : qd == 0 ? xhi : 0u,
                                        qd == 2 ? xlo : qd == 1 ? xhi : 0u, qd == 3 ? xlo : qd == 2 ? xhi : 0u);
            const uint32_t xs = qd == 3 ? xhi : 0u;  // the init word's spill into block 1
            const uint4 kf = make_uint4(keep_from(int32_t(q), 0), keep_from(int32_t(q), 1),
                                        keep_from(int32_t(q), 2), keep_from(int32_t(q), 3));
            uint32_t st = 0;
            for (int32_t j = 0; __builtin_amdgcn_ballot_w64(j < nb) != 0; j += kLaneBlocks)
            {
                uint4 w[kLaneBlocks];
#pragma unroll
                for (int u = 0; u < int(kLaneBlocks); ++u)
                {
                    w[u] = make_uint4(0, 0, 0, 0);
                    if (__builtin_amdgcn_ballot_w64(j + u < nb) != 0)  // wave-uniform
                        w[u] = load16_edge(j + u < nb ? pb + 16 * (j + u) : zero16);
                }
#pragma unroll
                for (int u4 = 0; u4 < int(kLaneBlocks); u4 += 4)
                {
                    if (__builtin_amdgcn_ballot_w64(j + u4 < nb) == 0) break;
#pragma unroll
                    for (int u = u4; u < u4 + 4; ++u)
                    {
                        uint4 x = w[u];
                        if (j + u == 0)
                        {
                            x.x = __builtin_amdgcn_bitop3_b32(x.x, kf.x, xf.x, 0x6A);
                            x.y = __builtin_amdgcn_bitop3_b32(x.y, kf.y, xf.y, 0x6A);
                            x.z = __builtin_amdgcn_bitop3_b32(x.z, kf.z, xf.z, 0x6A);
                            x.w = __builtin_amdgcn_bitop3_b32(x.w, kf.w, xf.w, 0x6A);
                        }
                        if (j + u == 1) x.x ^= xs;
                        const uint32_t sn = zT<4>(st ^ x.x) ^ zT<3>(x.y) ^ zT<2>(x.z) ^ zT<1>(x.w);
                        st = j + u < nb ? sn : st;
                    }
                }
            }
            // the last block: bytes >= t zeroed, then the t-byte step
            {
                uint4 x = xl;
                const bool first = K == 1;
                x.x = first ? __builtin_amdgcn_bitop3_b32(x.x, kf.x, xf.x, 0x6A) : x.x;
                x.y = first ? __builtin_amdgcn_bitop3_b32(x.y, kf.y, xf.y, 0x6A) : x.y;
                x.z = first ? __builtin_amdgcn_bitop3_b32(x.z, kf.z, xf.z, 0x6A) : x.z;
                x.w = first ? __builtin_amdgcn_bitop3_b32(x.w, kf.w, xf.w, 0x6A) : x.w;
                x.x ^= K == 2 ? xs : 0u;
                x = mask_below(x, int32_t(t));
                x.x ^= st;
                st = lane_tail_step(x, t);
            }
            if (act)
            {
                if (!(d.w & kSortMulti))
                    out[rec] = ~st;
                else
                {
                    // the head of a split record: Z_{E - pe}(raw(head)), E the record's end
                    const uint32_t jj = d.y >> 16;
                    const uint64_t sh = jj != kSortJJNone ? uint64_t(jj) << plog
                                                          : uint64_t(base) + off[rec] + len[rec] - e;
                    __hip_atomic_fetch_xor(out + rec, jj != kSortJJNone ? zshift_piece(tables, pow2, st, sh)
                                                                        : zshift48(pow2, st, sh),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            c0 = c1;
            d = d1;
        }
    };
    uint32_t g_cur = grab();
    uint4 d_cur = load_desc(g_cur);
    uint32_t g_nxt = grab();
    uint4 d_nxt = load_desc(g_nxt);
    Shape shA = shape_of(d_cur, g_cur);
    SortView vA = sort_view(d_cur, shA.n, tl, inits, ones_word);
    const uint32_t slot0 = rlo - n_full + tw;  // slot of list position i: slot0 + 8 g (whole records)
    vA.slot = slot0 + g_cur * 8;
    Shape shB{0, 0, 0, 0};
    SortView vB = vA;
    const SortView& cur0 = vA;
    // Row ring of RB buffers: row r of a group sits in b[r % RB]; each row
    // step issues row r + RB - 1 (this group's, or one of the next group's
    // first rows) before folding row r.  Groups are padded to a multiple of
    // RB rows, so the roles never change.  RB = 2 (kSortRing): one row in
    // flight per wave while another folds (measured on the headline batch:
    // one row ahead costs < 1 % against three; here it keeps the padding to
    // half a row per group).  RB = 4 serves small batches (pieces below
    // 64 KiB), where a wave has only a group or two of up to 33 rows, so the
    // rows in flight per wave, not the HBM, bound it; it finishes whole
    // records in the loop (no finish pass).  RB = 8 (128 VGPRs once the
    // finish pass is gone) measured no faster than 4 at 1 MiB - 2 GiB
    // (round 4, profiles/r04_sorted_ring_sweep.txt).
    uint4 b[RB];
#pragma unroll
    for (int j = 0; j < RB - 1; ++j) b[j] = load16_edge(row_ptr(cur0, j, false));
    if (RB == 2 && shA.n == 2) b[1] = load16_edge(row_ptr(cur0, 1, false));
    __builtin_amdgcn_sched_barrier(0);
    // One group: hash `cur` (shape sh) while the next group's view is built
    // into `nxt`.  The loop runs it twice per iteration with the two views
    // swapped (round 2 A/B: profiles/r02_sorted_view32_pingpong_ab.txt), so the ~20 registers of a view are never
    // copied at the back edge.
    auto step = [&](const SortView& cur, const Shape& sh, SortView& nxt, Shape& shn) {
        // A 2-row group runs no body loop: its row 1 was issued at the end of
        // the previous step, into b[1] once that step's last row was folded
        // (see below), a whole fold, finish and group header ahead.
        const bool pre = RB == 2 && sh.n == 2;
        const uint32_t g_nn = grab();
        const uint4 d_nn = load_desc(g_nn);
        shn = shape_of(d_nxt, g_nxt);
        nxt = sort_view(d_nxt, shn.n, tl, inits, ones_word);
        nxt.slot = slot0 + g_nxt * 8;
        uint32_t V[4] = {0, 0, 0, 0};
        const int32_t n = sh.n, fmin = sh.fmin, fedge = sh.fedge, fast = sh.fast;
        // General row: padding skip, start mask and init word (rows up to
        // fedge), end mask (row n - 1), zero-block reads.  Used for the first
        // rows and the last RB of a group; the rows between take the body
        // loop below: all lanes read item bytes, nothing to mask.
        auto gen_row = [&](uint4 d, int32_t r) {
            if (r < fmin) return;  // the padding row: V stays 0
            if (r <= fedge)
            {
                // row f: (d & keep) ^ ~init in one v_bitop3 per dword (truth
                // table index S0 S1 S2 = d keep x, MSB first: 0x6A)
                const bool at_f = r == cur.f;
                d.x = at_f ? __builtin_amdgcn_bitop3_b32(d.x, cur.kf.x, cur.xf.x, 0x6A) : d.x;
                d.y = at_f ? __builtin_amdgcn_bitop3_b32(d.y, cur.kf.y, cur.xf.y, 0x6A) : d.y;
                d.z = at_f ? __builtin_amdgcn_bitop3_b32(d.z, cur.kf.z, cur.xf.z, 0x6A) : d.z;
                d.w = at_f ? __builtin_amdgcn_bitop3_b32(d.w, cur.kf.w, cur.xf.w, 0x6A) : d.w;
                d.x ^= r == cur.f + 1 ? cur.xs : 0u;
            }
            if (r == n - 1)
            {
                d.x &= cur.ke.x;
                d.y &= cur.ke.y;
                d.z &= cur.ke.z;
                d.w &= cur.ke.w;
            }
            if (r == fmin)
                row_first(V, d);  // the largest item starts here; every other team's row is zero
            else
                row_update(V, d, li);
        };
        // body rows [hend, n - RB): after every team's first row and init
        // word (full groups only: a partial group has teams without items)
        const int32_t hend = fast < n ? min(n - RB, (fedge + RB) & ~(RB - 1)) : n - RB;
        int32_t r = 0;
        for (; r < hend; r += RB)
        {
#pragma unroll
            for (int j = 0; j < RB; ++j)
            {
                {
                    const int32_t rr = r + j + RB - 1;
                    const uint8_t* pp = row_ptr(cur, rr, false);
                    b[(j + RB - 1) % RB] = rr <= fedge ? load16_edge(pp) : load16(pp);
                }
                __builtin_amdgcn_sched_barrier(0);
                gen_row(b[j], r + j);
            }
        }
        {
            const uint8_t* pr = reinterpret_cast<const uint8_t*>(cur.p0);
            for (; r < n - RB; r += RB)
            {
#pragma unroll
                for (int j = 0; j < RB; ++j)
                {
                    b[(j + RB - 1) % RB] = load16(pr + uint32_t(r + j + RB - 1) * uint32_t(kRowBytes));
                    __builtin_amdgcn_sched_barrier(0);
                    row_update(V, b[j], li);
                }
            }
        }
        // the last RB rows: row n - 1, then the next group's first rows
#pragma unroll
        for (int j = 0; j < RB; ++j)
        {
            if (!(j == 0 && pre))
                b[(j + RB - 1) % RB] = load16_edge(j == 0 ? row_ptr(cur, n - 1, false) : row_ptr(nxt, j - 1, false));
            __builtin_amdgcn_sched_barrier(0);
            gen_row(b[j], n - RB + j);
        }
        // the next group's row 1 if it has two rows (b[1] is free now)
        if (RB == 2 && shn.n == 2) b[1] = load16_edge(row_ptr(nxt, 1, false));
        const uint32_t W = team_fold(V);
        flush();  // the previous group's split-record pieces
        {
            const bool multi = cur.recf != kSortNone && (cur.recf & kSortMulti);
            // whole records: the fold value by slot, eight consecutive words per
            // group (stores to out[rec] here hit a line per record, scattered:
            // 8-11 us of the configs[2] step, profiles/r03_sorted_late_finish_ab.txt)
            if (!INLOOP)
            {
                if (tl == 0 && cur.recf != kSortNone && !multi) wr[cur.slot] = W;
            }
            else if (cur.recf != kSortNone && !multi)
            {
                // small batches (RB >= 4): a wave has a group or two, so the
                // finish pass's two dependent global reads per record cost
                // more than finishing here: crc = ~Z_{-m}(W) from LDS tables
                const uint32_t m = cur.m & 127u, nn = 128u - m;
                uint32_t t = zT_n(W, nn & 15u);
                t = (nn & 16u) ? zT<4>(t) : t;
                t = (nn & 32u) ? zG(kLdsZ32, t) : t;
                t = (nn & 64u) ? zG(kLdsZ64, t) : t;
                t = zG(kLdsZInv, t);
                if (tl == 0) out[cur.recf & kSortRecMask] = ~(m ? t : W);
            }
            p_multi = __builtin_amdgcn_ballot_w64(multi) != 0;
            if (p_multi)
            {
                // fold value from the team's lane 0 to lanes 0..3 (quad_perm [0,0,0,0])
                const uint32_t Wq = uint32_t(__builtin_amdgcn_mov_dpp(int(W), 0x00, 0xF, 0xF, false));
                const uint32_t q = tl & 3u;
                uint32_t pz_new = zneg[(cur.m & 127u) * 1024u + q * 256u + ((Wq >> (8 * q)) & 0xFFu)];
                // an opaque definition: without it the loop-carried copy of pz at
                // the loop header waited for this load every group
                asm volatile("" : "+v"(pz_new));
                pz = pz_new;
            }
            p_recf = multi ? cur.recf : kSortNone;
            p_pe = cur.p0 + uint64_t(n) * kRowBytes - cur.m;
            p_jj = cur.jj;
        }
        g_nxt = g_nn;
        d_nxt = d_nn;
    };
    // twice per iteration with the two views swapped: the ~20 registers of a
    // view are never copied at the back edge (~60 v_mov per group before)
    while (shA.n > 0)
    {
        step(vA, shA, vB, shB);
        if (shB.n <= 0) break;
        step(vB, shB, vA, shA);
    }
    flush();
#if MI_SORT_FIN_OVERLAP
    // this wave's fold values (wr) are stored: count it done for the finish
    // pass, which starts when every wave's team groups are, beside the other
    // waves' lane items
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) atomicAdd(&S.teams_done, 1u);
#endif
    SORT_STAMP(5);
    lane_items();
    SORT_STAMP(6);
    if (INLOOP) return;  // whole records were finished in the loop
    // Finish pass, in list order (round 5): a whole record's fold value W
    // (wr at its slot, eight consecutive words per group) is Z_m(raw) of its
    // bytes, m = ceil128(E) - E; crc = ~Z_{-m}(W).  The team items past the
    // full pieces -- whole records and the heads of split records, which
    // their XORs finished -- sit at list positions n_full .. n_long - 1: their
    // descriptors at items[rlo + k] and their fold values at wr[rlo + k],
    // both read in order, together (rounds 3-4 read off[], len[] and the slot
    // left in out[r] in record order, then wr[slot]: two dependent round
    // trips, and the binning pass stored every slot).  The CRCs go to out[rec],
    // scattered inside the workgroup's record range.
#if MI_SORT_FIN_OVERLAP
    // (round 5) No workgroup barrier: a wave whose lane items are done waits
    // for every wave's team groups only (their wr stores), then takes records
    // 256 at a time while other waves may still hash lane items.
    while (__hip_atomic_load(&S.teams_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < kBlock / 64)
        __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    constexpr uint32_t FU = 4;
    const uint32_t n_whole = n_long - n_full;
    const uint4* const dl = items + rlo;
    for (;;)
    {
        uint32_t c0 = 0;
        if (lane == 0) c0 = atomicAdd(&S.next_fin, FU * 64u);
        c0 = uint32_t(__builtin_amdgcn_readfirstlane(int(c0)));
        if (c0 >= n_whole) break;
        uint4 dv[FU];
        uint32_t wv[FU];
#pragma unroll
        for (uint32_t u = 0; u < FU; ++u)
        {
            const uint32_t k = c0 + u * 64 + lane;
            dv[u] = k < n_whole ? dl[k] : make_uint4(0, 0, 0, kSortMulti);
            wv[u] = k < n_whole ? wr[uint64_t(rlo) + k] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < FU; ++u)
        {
            const uint64_t ps = sort_addr(dv[u]);
            const uint32_t m = uint32_t(0u - uint32_t(ps + dv[u].z)) & 127u;
            uint32_t v = wv[u];
            const uint32_t n = 128u - m;
            uint32_t t = zT_n(v, n & 15u);
            t = (n & 16u) ? zT<4>(t) : t;
            t = (n & 32u) ? zG(kLdsZ32, t) : t;
            t = (n & 64u) ? zG(kLdsZ64, t) : t;
            t = zG(kLdsZInv, t);
            v = m ? t : v;
            if (!(dv[u].w & kSortMulti)) out[dv[u].w & kSortRecMask] = ~v;
        }
    }
#else
    S.zinv[threadIdx.x] = tables[kTabZInv128 + threadIdx.x];
    __syncthreads();  // the workgroup's own stores are visible to it past the barrier
    constexpr uint32_t FU = 4;
    const uint32_t n_whole = n_long - n_full;
    const uint4* const dl = items + rlo;
    for (uint32_t k0 = threadIdx.x; k0 < n_whole; k0 += FU * kBlock)
    {
        uint4 dv[FU];
        uint32_t wv[FU];
#pragma unroll
        for (uint32_t u = 0; u < FU; ++u)
        {
            const uint32_t k = k0 + u * kBlock;
            dv[u] = k < n_whole ? dl[k] : make_uint4(0, 0, 0, kSortMulti);
            wv[u] = k < n_whole ? wr[uint64_t(rlo) + k] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < FU; ++u)
        {
            const uint64_t ps = sort_addr(dv[u]);
            const uint32_t m = uint32_t(0u - uint32_t(ps + dv[u].z)) & 127u;
            uint32_t v = wv[u];
            const uint32_t n = 128u - m;
            uint32_t t = zT_n(v, n & 15u);
            t = (n & 16u) ? zT<4>(t) : t;
            t = (n & 32u) ? zG(kLdsZ32, t) : t;
            t = (n & 64u) ? zG(kLdsZ64, t) : t;
            t = zG(kLdsZInv, t);
            v = m ? t : v;
            if (!(dv[u].w & kSortMulti)) out[dv[u].w & kSortRecMask] = ~v;
        }
    }
#endif
    SORT_STAMP(7);
}

#if MI_SORT_STAMP
extern "C" __attribute__((visibility("default"))) int mi_debug_sort_stamps(uint64_t* host, size_t n)
{
    n = n < sizeof(g_sort_stamp) / 8 ? n : sizeof(g_sort_stamp) / 8;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sort_stamp), n * 8) == hipSuccess ? 0 : -5;
}
extern "C" __attribute__((visibility("default"))) int mi_debug_sort_hw(uint32_t* host, size_t n)
{
    n = n < sizeof(g_sort_hw) / 4 ? n : sizeof(g_sort_hw) / 4;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sort_hw), n * 4) == hipSuccess ? 0 : -5;
}
#endif

// Slots for one workgroup's full pieces: items whose cost starts in its share
// (at most C (1000 + w) / (1000 G) + 1, the XCD-weighted share) are at least
// c_f = P/128 + kSortFold apart when they are full pieces, so a share holds
// at most share / c_f + 1 of them; C <= total/128 + 4 items bounds the total
// cost (rows <= len/128 + 2 per item, + kSortFold).
uint64_t sorted_full_per_wg(uint64_t count, uint64_t total_bytes, uint32_t plog, int grid)
{
    const uint64_t items = count + (total_bytes >> plog) + 1;
    return sorted_fpw(total_bytes / kRowBytes + 4 * items, plog, uint64_t(grid));
}

hipError_t launch_sorted(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                         const uint32_t* inits, uint64_t count, const SortedWorkspace& ws,
                         uint32_t* out, const uint32_t* tables, const uint32_t* pow2, int grid,
                         hipStream_t stream)
{
    if (count == 0) return hipSuccess;
    const uint32_t nb = sorted_blocks(count);
    const uint8_t* b = static_cast<const uint8_t*>(base);
    if (!ws.fused)
    {
        const uint32_t X = nb >= 512 ? 2u : 1u;
        auto ck = X == 2 ? sorted_cost_kernel<2> : sorted_cost_kernel<1>;
        hipLaunchKernelGGL(ck, dim3((nb + X - 1) / X), dim3(kPlanThreads), 0, stream, b, offsets,
                           lengths, inits, count, ws.blk_cost, ws.ctrl, out, tables, ws.plog);
    }
    auto k = ws.ring == 4 ? crc32c_sorted_kernel<4> : crc32c_sorted_kernel<2>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), kLdsSorted, stream, b, offsets, lengths, inits,
                       count, ws.blk_cost, nb, ws.ctrl, ws.items, ws.item_cap, ws.wr, out, tables,
                       pow2, ws.plog, ws.lane_rows, ws.fused, ws.bar_base);
    return hipGetLastError();
}

uint64_t sorted_item_cap(uint64_t count, uint64_t total_bytes, uint32_t plog, int grid)
{
    return count + uint64_t(grid) * sorted_full_per_wg(count, total_bytes, plog, grid);
}

// ---------------------------------------------------------------------------
// Window path (round 5, VERDICT r4 Next 4): mid-size device batches in ONE
// launch, no cost kernel, no LDS table image.  A record [a, E) covers the
// 128-B rows [Rs, Re); it is cut into windows of R rows (R = 4, 8 or 16)
// counted back from its end: window k = rows [Re - R (k + 1), Re - R k) within
// [Rs, Re) (K = ceil((L + 127) / 128 R) windows: an upper bound taken from the
// length alone, so the last may be empty).  A team (8 lanes) hashes one
// window: its R rows are issued at once (R dwordx4 per lane in flight) and
// folded through the lane tables (ds_bpermute; the sorted kernel's 152 KiB LDS
// image took 3.7 us to stage on a 1 MiB batch) as independent chains of 4
// rows, joined with Z_512 and Z_1024 (a 16-row chain measured 3.8 us of a
// 1 MiB batch's 13.1, profiles/r05_window_parts.txt).  The team's fold value W
// is the raw state of the window's bytes as of row Re - R k; Z_{128 R k}(W)
// (the Z_{512 j} L2 table, zshift48 past it) moves it to row Re.  ~init rides
// in the record's first four bytes (the sorted kernel's init word; a record
// of < 4 bytes takes the seed Z_L(~init) instead).  The windows of a record
// that fall in one wave are XORed there (team leaders' values through 16
// permutes); a record within one wave is finished by its first team:
// crc = ~Z_{-m}(XOR), m = 128 Re - E.  A record over several waves (segments)
// XORs each segment's value into the low half of a 64-bit word acc64[r] and
// its segment bit into the high half in ONE atomic; the segment that
// completes the mask finishes the record and zeroes the word (three dependent
// device-scope atomics per window measured 1.8 / 4.8 / 17 us of a 1 / 4 /
// 16 MiB batch).  Records of more than 32 segments take the acc / cnt form
// (XOR, acq_rel count, swap).  All workspace words are zero between launches.
// Tasks (r, window) are numbered by a prefix over the record lengths that
// every workgroup computes for itself in LDS (count <= kWinMaxCountBig): no
// second launch, no grid barrier.  Workgroups of 64, 256 or 768 threads
// (launch_window's rule; 768: one per CU, looping).  A grid smaller than the
// task count (understated total) loops; it never fails.
// ---------------------------------------------------------------------------
#ifndef MI_WIN_SKIP
#define MI_WIN_SKIP 0  // A/B timing builds only (wrong CRCs): 1 no combine, 2 no lookups, 4 no fold
#endif
__device__ __forceinline__ uint32_t wave_min32(uint32_t x)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) x = min(x, uint32_t(__shfl_xor(int(x), d)));
    return x;
}

// Windows of a record of L bytes, computed in 64 bits: a record of close to
// 4 GiB wrapped the 32-bit sum to 0 windows.
template <uint32_t R>
__device__ __forceinline__ uint32_t win_count(uint32_t L)
{
    return uint32_t((uint64_t(L) + kRowBytes - 1 + R * kRowBytes - 1) / (R * kRowBytes));
}
// Tasks a launch may number: task indices, the round cursor and the records'
// first tasks stay in 32 bits below it.  A batch with more (only with a
// total_bytes hint understated ~80,000-fold: 2^31 windows are >= 1 TiB of
// records) stores ctrl[1] = ctrl[2] = 1 and hashes nothing, as the sorted
// path does when its workspace overflows: the engine recomputes a
// synchronous batch on the plan path and reports an asynchronous one at the
// next stream sync.
constexpr uint64_t kWinMaxTasks = uint64_t(1) << 31;

// B threads per workgroup (64, 256, kWinBlockBig), R rows per window (4, 8, 16)
template <uint32_t B, uint32_t R>
__global__ __launch_bounds__(B) void crc32c_window_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ inits, uint32_t count,
    uint32_t* __restrict__ out, uint64_t* __restrict__ acc64, uint32_t* __restrict__ acc,
    uint32_t* __restrict__ cnt, const uint32_t* __restrict__ tables, const uint32_t* __restrict__ pow2,
    uint32_t* __restrict__ ctrl)
{
    // LDS: first task of each record, wave sums (64-bit, 8-B aligned)
    uint32_t* const s_pre = reinterpret_cast<uint32_t*>(smem);
    uint64_t* const s_wsum = reinterpret_cast<uint64_t*>(smem + ((size_t(count) * 4 + 7) & ~size_t(7)));
    LaneTabs lt;
    load_lane_tabs<6 * kLaneOps>(lt, tables);
    // (1) windows per record, from the lengths alone (an empty record: one
    // task, which stores init)
    for (uint32_t i = threadIdx.x; i < count; i += B) s_pre[i] = win_count<R>(len[i]);
    __syncthreads();
    // (2) exclusive prefix: a contiguous run of records per thread
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    // an odd run length: the runs of a wave's lanes start in distinct LDS banks
    // (a run of 16 made every read a 32-way conflict: 11,822 records in
    // 768-thread workgroups took 6-7 us more, profiles/r05_window_small_records.txt)
    const uint32_t per = ((count + B - 1) / B) | 1u;
    const uint32_t i0 = min(count, threadIdx.x * per), i1 = min(count, i0 + per);
    uint64_t own = 0;
    for (uint32_t i = i0; i < i1; ++i) own += s_pre[i];
    const uint64_t x = wave_incl_scan64(own);
    if (lane == 63) s_wsum[wave] = x;
    __syncthreads();
    uint64_t run64 = x - own, ntask64 = 0;
#pragma unroll
    for (uint32_t w = 0; w < B / 64; ++w)
    {
        const uint64_t s = s_wsum[w];
        run64 += w < wave ? s : 0u;
        ntask64 += s;
    }
    if (ntask64 > kWinMaxTasks)  // workgroup-uniform, and the same in every workgroup
    {
        if (blockIdx.x == 0 && threadIdx.x == 0)
        {
            ctrl[1] = 1;
            ctrl[2] = 1;  // sticky: an asynchronous batch's is reported at the next stream sync
        }
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ctrl[1] = 0;
    const uint32_t ntask = uint32_t(ntask64);
    uint32_t run = uint32_t(run64);
    for (uint32_t i = i0; i < i1; ++i)
    {
        const uint32_t c = s_pre[i];
        s_pre[i] = run;
        run += c;
    }
    __syncthreads();

    // (3) one window per team per round; the round loop is wave-uniform (the
    // lane-table permutes need every lane of the wave)
    const uint32_t tl = threadIdx.x & (kTeam - 1);
    const uint32_t team = threadIdx.x / kTeam;
    const uint32_t tw = team & 7u;  // team within the wave
    constexpr uint32_t kTeamsPerWg = B / kTeam;
    const uint8_t* zero16 = reinterpret_cast<const uint8_t*>(tables + kTabZero);
    for (uint32_t t0 = blockIdx.x * kTeamsPerWg; t0 + wave * 8 < ntask; t0 += gridDim.x * kTeamsPerWg)
    {
        const uint32_t t = t0 + team;
        const bool live = t < ntask;
        // the record: the last r with pre[r] <= t (pre[0] = 0)
        uint32_t lo = 0, hi = count - 1;
        while (live && lo < hi)
        {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_pre[mid] <= t)
                lo = mid;
            else
                hi = mid - 1;
        }
        const uint32_t r = lo;
        const uint32_t p0 = s_pre[r];
        const uint32_t K = (r + 1 < count ? s_pre[r + 1] : ntask) - p0;
        const uint32_t k = live ? K - 1 - (t - p0) : 0u;  // windows from the record's end
        const uint64_t a = uint64_t(base) + off[r];
        const uint32_t L = live ? len[r] : 0u;
        const uint32_t ninit = inits ? ~inits[r] : 0xFFFFFFFFu;
        const uint64_t E = a + L;
        const int64_t Rs = int64_t(a >> 7), Re = int64_t((E + kRowBytes - 1) >> 7);
        const int64_t row0 = Re - int64_t(R) * (int64_t(k) + 1);  // window row 0
        // first row of this team's bytes in the window; the wave folds from
        // its teams' smallest
        const uint32_t ist = L ? uint32_t(min(max(Rs - row0, int64_t(0)), int64_t(R))) : R;
        const uint32_t imin = wave_min32(ist);
        uint4 w[R];
#pragma unroll
        for (int i = 0; i < int(R); ++i)
        {
            const bool in = uint32_t(i) >= ist;
            const uint64_t p = uint64_t(row0 + i) * kRowBytes + tl * 16u;
            w[i] = make_uint4(0, 0, 0, 0);
            if (uint32_t(i) >= imin)  // wave-uniform
                w[i] = load16_edge(in ? reinterpret_cast<const uint8_t*>(p) : zero16);
        }
        // edges: bytes before a in row Rs, the init word (rows Rs, Rs + 1),
        // bytes from E on in row Re - 1
        const int64_t lb = int64_t(a) - (Rs * kRowBytes + int64_t(tl) * 16);  // a within this lane's block of row Rs
        const int32_t f0 = int32_t(min(max(lb, int64_t(0)), int64_t(16)));
        const int32_t be = int32_t(min(max(int64_t(E) - ((Re - 1) * kRowBytes + int64_t(tl) * 16), int64_t(0)), int64_t(16)));
        const bool with_init = L >= 4;
        // chains of four rows
        uint32_t V[R / 4][4] = {};
#pragma unroll
        for (int i = 0; i < int(R); ++i)
        {
            if (uint32_t(i) < imin) continue;  // wave-uniform
            uint4 d = w[i];
            const int64_t row = row0 + i;
            if (row == Rs) d = mask_from(d, f0);
            if (with_init && (row == Rs || row == Rs + 1))
            {
                const int32_t q = int32_t(lb - (row - Rs) * kRowBytes);
                d.x ^= init_dword(ninit, q, 0);
                d.y ^= init_dword(ninit, q, 1);
                d.z ^= init_dword(ninit, q, 2);
                d.w ^= init_dword(ninit, q, 3);
            }
            if (row == Re - 1) d = mask_below(d, be);
            if (MI_WIN_SKIP & 4)
            {
                V[i >> 2][0] ^= d.x; V[i >> 2][1] ^= d.y; V[i >> 2][2] ^= d.z; V[i >> 2][3] ^= d.w;
            }
            else
                row_update_lane(V[i >> 2], d, lt, true, false);
        }
        uint32_t U[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {
            if constexpr (R == 4)
            {
                U[q] = V[0][q];
                continue;
            }
            const uint32_t lo8 = zL<7>(lt, V[0][q]) ^ V[1][q];  // Z_512: rows 0-7 as of row 7
            if constexpr (R == 16)
            {
                const uint32_t hi8 = zL<7>(lt, V[2][q]) ^ V[3][q];  // rows 8-15 as of row 15
                U[q] = zL<8>(lt, lo8) ^ hi8;                          // Z_1024
            }
            else
                U[q] = lo8;
        }
        const uint32_t W = team_fold_lane(U, lt);
        // this window's value as of row Re (team leaders; 0 for no record)
        uint32_t T = live && L ? W : 0u;
        if (k && !(MI_WIN_SKIP & 2))
        {
            const uint32_t kb = k * (R / 4);  // shift in 512 B
            T = kb < kWinShifts ? zglob(tables + kTabZWin + (kb - 1) * 1024u, T)
                                : zshift48(pow2, T, uint64_t(k) * R * kRowBytes);
        }
        // XOR over this wave's windows of the same record
        const uint32_t rr = live ? r : 0xFFFFFFFFu;
        uint32_t seg = 0;
        bool lead = true;
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j)
        {
            const uint32_t rj = uint32_t(__shfl(int(rr), int(8 * j)));
            const uint32_t Tj = uint32_t(__shfl(int(T), int(8 * j)));
            seg ^= rj == rr ? Tj : 0u;
            lead = lead && !(j < tw && rj == rr);
        }
        if (tl == 0 && live && lead)
        {
            bool fin = true;
            if (L == 0)
                out[r] = ~ninit;  // crc32c(init, "", 0) = init
            else
            {
                const uint32_t wf = p0 >> 3, wl = (p0 + K - 1) >> 3;  // the record's first and last waves
                const uint32_t nseg = wl - wf + 1;
                if (nseg > 1 && !(MI_WIN_SKIP & 1))
                {
                    if (nseg <= 32)
                    {
                        const uint32_t sb = 1u << ((t >> 3) - wf);
                        const uint64_t old = __hip_atomic_fetch_xor(acc64 + r, (uint64_t(sb) << 32) | seg,
                                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t full = nseg == 32 ? 0xFFFFFFFFu : (1u << nseg) - 1u;
                        fin = (uint32_t(old >> 32) | sb) == full;
                        if (fin)
                        {
                            seg ^= uint32_t(old);
                            __hip_atomic_store(acc64 + r, uint64_t(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                    else
                    {
                        __hip_atomic_fetch_xor(acc + r, seg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t seen = __hip_atomic_fetch_add(cnt + r, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                        fin = seen == nseg - 1;
                        if (fin)
                        {
                            seg = __hip_atomic_exchange(acc + r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(cnt + r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                }
                if (fin)
                {
                    const uint32_t m = uint32_t(uint64_t(Re) * kRowBytes - E);
                    uint32_t v = (MI_WIN_SKIP & 2) ? seg : zglob(tables + kTabZNeg + m * 1024u, seg);
                    if (!with_init) v ^= zbits(tables + kTabP2, ninit, L);  // seed Z_L(~init)
                    out[r] = ~v;
                }
            }
        }
    }
}

size_t window_lds_bytes(uint32_t count) { return ((size_t(count) * 4 + 7) & ~size_t(7)) + 8 * (kWinBlockBig / 64); }

uint64_t window_grid(uint64_t count, uint64_t total_bytes, int grid_cap, uint32_t block, uint32_t rows)
{
    // windows <= L / 2048 + 1.07 per record (win_count)
    const uint64_t bound = total_bytes / (rows * kRowBytes) + (17 * count) / 16 + 1;
    const uint64_t g = (bound + block / kTeam - 1) / (block / kTeam);
    return std::max<uint64_t>(1, std::min<uint64_t>(g, uint64_t(grid_cap)));
}

hipError_t launch_window(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                         const uint32_t* inits, uint64_t count, uint64_t total_bytes, uint32_t* out,
                         uint64_t* acc64, uint32_t* acc, uint32_t* cnt, const uint32_t* tables,
                         const uint32_t* pow2, uint32_t* ctrl, int grid_cap, uint32_t block,
                         uint32_t rows, hipStream_t stream)
{
    if (count == 0) return hipSuccess;
    if (count > kWinMaxCountBig) return hipErrorInvalidValue;
    // 4-row windows up to 12 waves of them per CU (grid_cap / 8 = the CUs),
    // then 8: configs[2] records cut to 1 / 2 / 4 / 8 / 16 MiB took 7.2 / 8.4
    // / 9.3 / 12.6 / 21.5 us with 4 rows, 8.7 / 9.7 / 10.2 / 13.8 / 17.4 with 8,
    // 12.0 / 12.8 / 13.8 / 15.0 / 20.3 with 16 (profiles/r05_window_rows.txt)
    const uint64_t cus = uint64_t(grid_cap) / 8;
    if (rows == 0) rows = window_grid(count, total_bytes, 1 << 30, 64, 4) <= 12 * cus ? 4u : 8u;
    // One-wave workgroups spread a small batch's lane-table permutes over as
    // many CUs as it has waves; four-wave ones read the lengths fewer times;
    // one twelve-wave workgroup per CU (kWinBlockBig) builds the prefix once
    // per CU, which pays once the windows fill most of the CUs' teams: 4-row
    // windows above 48 per CU, 8-row ones from 64 up to ~1.1 rounds of 96 per
    // CU (a second round costs ~11 us).  configs[2] cut to 8 / 16 / 20 MiB:
    // 11.6 / 15.9 / 16.8 us against 12.6 / 17.5 / 20.0 with four-wave
    // workgroups; at 4 / 12 / 24 MiB the four-wave ones were faster
    // (profiles/r05_window_block768.txt)
    if (block == 0)
    {
        const uint64_t w = window_grid(count, total_bytes, 1 << 30, kTeam, rows);  // windows
        const bool big = rows == 4 ? w > 48 * cus : (w > 64 * cus && w <= 108 * cus);
        block = big ? kWinBlockBig : count <= kWinSmallCount ? 64u : kWinBlockMax;
    }
    // kWinBlockBig workgroups: one per CU (grid_cap / 8), looping over the windows
    const uint32_t g = uint32_t(window_grid(count, total_bytes, block == kWinBlockBig ? grid_cap / 8 : grid_cap,
                                            block, rows));
    auto k = block == 64             ? (rows == 4   ? crc32c_window_kernel<64, 4>
                                        : rows == 8 ? crc32c_window_kernel<64, 8>
                                                    : crc32c_window_kernel<64, 16>)
             : block == kWinBlockBig ? (rows == 4   ? crc32c_window_kernel<kWinBlockBig, 4>
                                        : rows == 8 ? crc32c_window_kernel<kWinBlockBig, 8>
                                                    : crc32c_window_kernel<kWinBlockBig, 16>)
                                     : (rows == 4   ? crc32c_window_kernel<kWinBlockMax, 4>
                                        : rows == 8 ? crc32c_window_kernel<kWinBlockMax, 8>
                                                    : crc32c_window_kernel<kWinBlockMax, 16>);
    hipLaunchKernelGGL(k, dim3(g), dim3(block), window_lds_bytes(uint32_t(count)), stream,
                       static_cast<const uint8_t*>(base), offsets, lengths, inits, uint32_t(count),
                       out, acc64, acc, cnt, tables, pow2, ctrl);
    return hipGetLastError();
}

// Allow the 152 KiB dynamic LDS image on the two persistent kernels.
hipError_t configure_kernels()
{
    const void* k[] = {reinterpret_cast<const void*>(&crc32c_fixed_pipe_kernel<4, false>),
                       reinterpret_cast<const void*>(&crc32c_span_chunk_kernel),
                       reinterpret_cast<const void*>(&crc32c_fixed_pipe_kernel<4, true>),
                       reinterpret_cast<const void*>(&crc32c_fixed_pipe_kernel<2, false>),
                       reinterpret_cast<const void*>(&crc32c_fixed_pipe_kernel<2, true>),
                       reinterpret_cast<const void*>(&crc32c_fixed_kernel<false, false>),
                       reinterpret_cast<const void*>(&crc32c_fixed_kernel<false, true>),
                       reinterpret_cast<const void*>(&crc32c_fixed_kernel<true, false>),
                       reinterpret_cast<const void*>(&crc32c_fixed_kernel<true, true>)};
    hipError_t e = hipSuccess;
    for (const void* f : k)
        if (e == hipSuccess)
            e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_chunk_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&crc32c_direct_kernel<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&single_join_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kSingleStaged * 4096);
    const void* kw[] = {reinterpret_cast<const void*>(&crc32c_window_kernel<64, 4>),
                        reinterpret_cast<const void*>(&crc32c_window_kernel<kWinBlockMax, 4>),
                        reinterpret_cast<const void*>(&crc32c_window_kernel<64, 8>),
                        reinterpret_cast<const void*>(&crc32c_window_kernel<64, 16>),
                        reinterpret_cast<const void*>(&crc32c_window_kernel<kWinBlockMax, 8>),
                        reinterpret_cast<const void*>(&crc32c_window_kernel<kWinBlockMax, 16>),
                        reinterpret_cast<const void*>(&crc32c_window_kernel<kWinBlockBig, 4>),
                        reinterpret_cast<const void*>(&crc32c_window_kernel<kWinBlockBig, 8>),
                        reinterpret_cast<const void*>(&crc32c_window_kernel<kWinBlockBig, 16>)};
    for (const void* f : kw)
        if (e == hipSuccess)
            e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    int(window_lds_bytes(kWinMaxCountBig)));
    const void* ks[] = {reinterpret_cast<const void*>(&crc32c_sorted_kernel<2>),
                        reinterpret_cast<const void*>(&crc32c_sorted_kernel<4>)};
    for (const void* f : ks)
        if (e == hipSuccess)
            e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsSorted);
    return e;
}

// ---------------------------------------------------------------------------
// Synthetic input: u64 word j of the stream = splitmix64(seed ^ j).
// dst must be 8-byte aligned and byte_offset a multiple of 8.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_splitmix_kernel(uint8_t* __restrict__ dst,
                                                            uint64_t nbytes, uint64_t seed,
                                                            uint64_t word0)
{
    const uint64_t nwords = nbytes / 8;
    const uint64_t npairs = nwords / 2;
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t step = uint64_t(gridDim.x) * blockDim.x;
    for (; i < npairs; i += step)
    {
        ulonglong2 v;
        v.x = splitmix64(seed ^ (word0 + 2 * i));
        v.y = splitmix64(seed ^ (word0 + 2 * i + 1));
        reinterpret_cast<ulonglong2*>(dst)[i] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
    {
        for (uint64_t w = npairs * 2; w < nwords; ++w)
            reinterpret_cast<uint64_t*>(dst)[w] = splitmix64(seed ^ (word0 + w));
        const uint64_t tail = nbytes & 7u;
        if (tail)
        {
            const uint64_t v = splitmix64(seed ^ (word0 + nwords));
            for (uint64_t k = 0; k < tail; ++k) dst[nwords * 8 + k] = uint8_t(v >> (8 * k));
        }
    }
}

hipError_t launch_fill_splitmix(void* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset,
                                hipStream_t stream)
{
    if (nbytes == 0) return hipSuccess;
    const uint64_t pairs = nbytes / 16 + 1;
    uint64_t grid = (pairs + 255) / 256;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(uint32_t(grid)), dim3(256), 0, stream,
                       static_cast<uint8_t*>(dst), nbytes, seed, byte_offset / 8);
    return hipGetLastError();
}

}  // namespace mi_crc
