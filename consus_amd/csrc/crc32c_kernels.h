// consus_amd/csrc/crc32c_kernels.h -- launch interface of the CDNA4 kernels.
//
// Internal to libconsus_crc32c.so; the public boundary is include/consus_crc32c.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mi_crc {

// Geometry of the record kernels.
constexpr int kTeam = 8;                    // lanes per record ("team")
constexpr int kRowBytes = 16 * kTeam;       // one row = 16 B per lane = 128 B
constexpr int kGroupRows = 8;               // rows per software-pipelined group
constexpr int kGroupBytes = kRowBytes * kGroupRows;  // 1 KiB
constexpr int kChunk = 4096;                // variable-length work unit
constexpr int kBlock = 1024;                // threads per workgroup (16 waves)
constexpr int kSmallRecord = 32;            // records shorter than this are finished byte-serially
constexpr uint32_t kLongChunks = 64;        // records with more interior chunks take the long path
// Plan bins: 0, 1, 2 = pieces of 4, 3, 2 groups; 3 + (8 - R) = one group of R rows (R = 8..1)
constexpr uint32_t kBins = 11;
constexpr int kLongBlock = 1024;            // threads per long record

// Global table image uploaded once per device (u32 words).
constexpr int kTabMain = 0;                 // G^{128}_j, 4 x 256  (row fold, replicated bank-private in LDS)
constexpr int kTabT = 1024;                 // T_0..T_15, 16 x 256 (slice-by-16)
constexpr int kTabZ32 = kTabT + 4096;       // G^{32}_j
constexpr int kTabZ64 = kTabZ32 + 1024;     // G^{64}_j
constexpr int kTabZChunk = kTabZ64 + 1024;  // G^{4096}_j (chunk combine)
constexpr int kTabZLong = kTabZChunk + 1024;   // G^{1024*4096} (long-record stride)
constexpr int kTabZC2 = kTabZLong + 1024;      // G^{4096*2^b}, b = 0..9
constexpr int kTabP2 = kTabZC2 + 10 * 1024;    // G^{2^k}, k = 0..12 (shifts up to 4 KiB)
constexpr int kTabZInv128 = kTabP2 + 13 * 1024; // Z_{-128} = (Z_128)^{-1}
constexpr int kTabZero = kTabZInv128 + 1024;    // 4 zero words (init 0 when inits == nullptr)
constexpr int kTabFInit = kTabZero + 4;         // Z_n(0xFFFFFFFF), n = 0..4096 (init 0 seeds)
constexpr int kTabZRows = kTabFInit + 4100;     // G^{128 k}, k = 1..32 (last-piece shifts)
constexpr int kTabZNeg = kTabZRows + 32 * 1024; // Z_{-m} = (Z_m)^{-1}, m = 0..127 (direct kernel)
constexpr int kTabLane = kTabZNeg + 128 * 1024; // Z_16, Z_12, Z_8, Z_4, Z_32, Z_64, Z_128, Z_512,
                                                 // Z_1024 as six 64-entry tables each:
                                                 // [op][c][i] = Z(i << 6c) (lane fold; Z_128: the
                                                 // LDS-free row update; Z_512, Z_1024: the window
                                                 // path's chain joins)
constexpr int kLaneOps = 9;
constexpr int kTabZWin = kTabLane + kLaneOps * 6 * 64;  // G^{512 k}, k = 1..255 (window path)
constexpr uint32_t kWinShifts = 256;
constexpr int kTabWords = kTabZWin + (kWinShifts - 1) * 1024;

// LDS image of the record kernels (bytes).
constexpr uint32_t kLdsMain = 0;            // 128 KiB bank-private G^{128}
constexpr uint32_t kLdsT = 131072;          // 16 KiB
constexpr uint32_t kLdsZ32 = kLdsT + 16384;
constexpr uint32_t kLdsZ64 = kLdsZ32 + 4096;
constexpr uint32_t kLdsBytes = kLdsZ64 + 4096;  // 155648

// One unit of variable-length work ("piece"): the part of a record inside one
// 4 KiB-aligned chunk of the address space.  A team hashes the 128-B-aligned
// window [wend - G KiB, wend), wend = the piece end rounded up to 128, with
// the bytes before the piece start and the m bytes after its end masked.
// Packed in 8 bytes: wend >> 7 (41 bits: addresses below 2^48), the window
// length wend - piece start (13 bits, <= 4096 + 127) and m (7 bits).
struct Item
{
    uint64_t bits;
};
constexpr uint32_t kItemAddrShift = 20;
constexpr uint32_t kItemLenShift = 7;
constexpr uint64_t kItemMaxAddr = uint64_t(1) << 48;

hipError_t configure_kernels();

hipError_t launch_fixed(const void* base, uint64_t stride, uint32_t len, const uint32_t* inits,
                        uint64_t count, uint32_t* out, const uint32_t* tables, int grid,
                        hipStream_t stream);

// Variable-length pipeline.  `ws_*` are engine-owned device workspaces.
struct VarWorkspace
{
    uint32_t* blk;        // kBins * nblocks block counts, then the plan header (plan_hdr)
    Item* items;          // capacity `item_cap`
    uint32_t* partial;    // capacity `item_cap`
    uint32_t* first_pos;  // count: item of the record's first piece
    uint32_t* int_pos;    // count: first interior (full 4 KiB) piece
    uint32_t* last_pos;   // count: item of the last piece (records with >= 2 pieces)
    uint32_t* longs;      // count (records on the long path)
    uint64_t item_cap;
};

// Small batches: one launch, one team per record, no plan (launch_direct).
constexpr uint64_t kDirectMaxCount = 1u << 18;   // records
constexpr uint64_t kDirectMaxBytes = 32ull << 20;  // sum of lengths
constexpr uint64_t kDirectMaxRecord = 16u << 10;   // longest record (128 rows for one team;
                                                   // the planned path wins above ~32 KiB)
// Batches of at most kLiteMaxBytes (a durable-log flush) take the LDS-free
// form: one-wave workgroups, no 152 KiB table staging.
constexpr uint64_t kLiteMaxBytes = 2ull << 20;
constexpr int kLiteBlock = 256;   // launch bound of the LDS-free form
constexpr uint32_t kLiteWG = 64;  // ... and the workgroup it is launched with
// Completion word: when `signal` is set, the last workgroup to finish stores
// `seq` to signal->flag (mapped host memory) after every CRC is visible
// system-wide, so the host may spin on it instead of a stream sync.
struct DoneSignal
{
    uint32_t* counter;  // device word, 0 between launches
    uint32_t* flag;     // mapped pinned host word (device address)
    uint32_t seq;
};
hipError_t launch_direct(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                         const uint32_t* inits, uint64_t count, uint64_t total_bytes, uint32_t* out,
                         const uint32_t* tables, const uint32_t* pow2, int grid,
                         hipStream_t stream, const DoneSignal* signal = nullptr,
                         int lite = -1);  // -1: by size; 0 / 1: force (tests)

// force_scan: run the separate scan pass even for plans that do not need it
// (MI_CRC32C_PLAN_SCAN=1, so the tests cover both plan forms).
hipError_t launch_var_plan(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                           uint64_t count, const VarWorkspace& ws, hipStream_t stream,
                           bool force_scan);
hipError_t launch_var_chunks(const uint32_t* inits, uint64_t count, const VarWorkspace& ws,
                             const uint32_t* tables, int grid, hipStream_t stream);
hipError_t launch_var_finalize(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                               const uint32_t* inits, uint64_t count, const VarWorkspace& ws,
                               uint32_t* out, const uint32_t* tables, const uint32_t* pow2,
                               hipStream_t stream);
uint32_t var_plan_blocks(uint64_t count);
// Plan header after the kBins x blocks counts: bin starts, total items, long records.
constexpr uint32_t kPlanHdrTotal = kBins;
constexpr uint32_t kPlanHdrWords = kBins + 4;
inline uint32_t* plan_hdr(uint32_t* blk, uint32_t nblocks) { return blk + kBins * nblocks; }

// Sorted path (launch_sorted): whole records per team, binned by row count
// inside each workgroup's cost-balanced share; two launches, no plan/finalize.
struct SortedWorkspace
{
    uint64_t* blk_cost;  // sorted_blocks(count)
    uint32_t* ctrl;      // 4 words: item cursor, overflow flag
    uint4* items;        // item_cap 16-B descriptors
    uint64_t item_cap;   // sorted_item_cap(count, total_bytes)
    uint32_t* wr;        // item_cap words: a whole record's fold value, by descriptor slot
    uint32_t plog;       // log2 of the piece records longer than it are cut into (9..16)
    int ring;            // rows per ring of the hash loop: 2 or 4
    uint32_t lane_rows;  // records spanning <= this many rows are lane items (0..kSortLaneRowsMax)
    // One launch (round 5): the hash kernel computes the cost blocks itself
    // and meets at a grid barrier (every workgroup resident: one per CU);
    // ctrl[32] counts arrivals, bar_base = its value before this launch.
    int fused;
    uint32_t bar_base;
};
constexpr uint64_t kSortedMaxCount = 1ull << 30;
uint32_t sorted_blocks(uint64_t count);
constexpr uint32_t kSortPieceLog2 = 16;  // 64 KiB pieces (the default)
// Lane items: whole records and heads spanning at most this many 128-B rows
// are hashed one per lane (crc32c_sorted_kernel).  configs[2], 3 interleaved
// rounds on one box: 0.783-0.786 ms at 2 rows against 0.788-0.789 at 3 and
// 0.792-0.799 with teams only (profiles/r04_sorted_lane_items_ab.txt).
constexpr uint32_t kSortLaneRows = 2;
constexpr uint32_t kSortLaneRowsMax = 3;
uint64_t sorted_item_cap(uint64_t count, uint64_t total_bytes, uint32_t plog, int grid);
uint64_t sorted_full_per_wg(uint64_t count, uint64_t total_bytes, uint32_t plog, int grid);
hipError_t launch_sorted(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                         const uint32_t* inits, uint64_t count, const SortedWorkspace& ws,
                         uint32_t* out, const uint32_t* tables, const uint32_t* pow2, int grid,
                         hipStream_t stream);

// Window path (launch_window): mid-size batches of at most kWinMaxCount
// records in one launch; each record cut into windows of 4, 8 or 16 rows from
// its end, one per team.  acc64 / acc / cnt: count words each, zero before
// and after.  ctrl: the sorted path's control words; ctrl[1] = 1 (and the
// sticky ctrl[2]) when the batch numbers more than 2^31 windows, which only
// a total_bytes hint understated by a factor ~80,000 lets through (nothing
// is hashed then; the engine recovers as for the sorted path's overflow).
constexpr uint32_t kWinBlockMax = 256;   // workgroup of batches above kWinSmallCount records
constexpr uint32_t kWinSmallCount = 768;  // ... and one wave per workgroup up to it
constexpr uint32_t kWinMaxCount = 8192;     // the engine's record bound (MI_CRC32C_WIN_MAX_COUNT: probes)
constexpr uint32_t kWinBlockBig = 768;      // one workgroup per CU (12 waves) for batches that fill the CUs
constexpr uint32_t kWinMaxCountBig = 16384; // the LDS prefix's bound (64 KiB)
size_t window_lds_bytes(uint32_t count);
uint64_t window_grid(uint64_t count, uint64_t total_bytes, int grid_cap, uint32_t block, uint32_t rows);
hipError_t launch_window(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                         const uint32_t* inits, uint64_t count, uint64_t total_bytes, uint32_t* out,
                         uint64_t* acc64, uint32_t* acc, uint32_t* cnt, const uint32_t* tables,
                         const uint32_t* pow2, uint32_t* ctrl, int grid_cap,
                         uint32_t block,  // 0: by count; 64, 256
                         uint32_t rows,   // rows per window, 0: by size; 4, 8, 16
                         hipStream_t stream);

hipError_t launch_chain(const uint32_t* crcs, const uint64_t* after, uint32_t np, uint32_t* out,
                        const uint32_t* pow2_tables, hipStream_t stream);
hipError_t launch_combine(const uint32_t* crc_a, const uint32_t* crc_b, const uint64_t* len_b,
                          uint64_t count, uint32_t* out, const uint32_t* pow2_tables,
                          hipStream_t stream);

// One device buffer: head h bytes, m 4 KiB chunks (m + 2 <= 2^24), tail t;
// crcs: m words, vals: kSingleVals words, out: 1 word (all device).
constexpr uint32_t kSingleVals = 1026;
hipError_t launch_single(const void* data, uint64_t h, uint64_t m, uint32_t t, uint32_t init,
                         uint32_t crc0, uint32_t* crcs, uint32_t* vals, uint32_t* out,
                         const uint32_t* tables, const uint32_t* pow2, int grid,
                         hipStream_t stream);

hipError_t launch_make_fixed_records(uint64_t* off, uint32_t* len, uint64_t count, uint64_t stride,
                                     uint32_t length, hipStream_t stream);

hipError_t launch_fill_splitmix(void* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset,
                                hipStream_t stream);

}  // namespace mi_crc
