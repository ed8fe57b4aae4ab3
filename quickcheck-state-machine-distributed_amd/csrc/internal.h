// internal.h -- declarations shared by the search kernels and the C-ABI host.
//
// The cascade of one check call (api.hip), four launches on one stream:
//
//   stage 0   compact_search<G32>  every history; <= 32 events, <= 8 pids,
//                                  compact values; one history per lane with
//                                  a node budget          (csrc/compact.hip)
//   stage 0w  compact_search<G64>  the histories stage 0 cannot hold, <= 64
//                                  events                 (csrc/compact.hip)
//   heavy     wave_search          the histories over the stage-0 / 0w
//                                  budgets (both lists, one launch): one
//                                  wavefront per history, scalar DFS, LDS
//                                  memo (csrc/wave.hip) -- or, for a long
//                                  list, memo_search: one lane per history
//                                  with an exact-count memo (csrc/memo.hip);
//                                  heavy_mode 2 (default) picks by the last
//                                  call's count
//   giants    giant_search         everything else: the split stage (one
//                                  history over many lanes), the ordered
//                                  combine, the batch totals (csrc/split.hip)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "qsmd.h"
#include "qsmd_gen.h"

namespace qsmd {

// Batch totals, accumulated per call into kBuckets buckets of one cache line
// each (a block adds its counts to bucket blockIdx % kBuckets: the blocks of
// one bucket share an XCD) and summed by the giant stage's last block.
enum { T_CHECKED = 0, T_LIN, T_NONLIN, T_ERR, T_ENC, T_BUDGET, T_SKIPPED, T_NODES, T_N };
constexpr uint32_t kBuckets = 64;
constexpr uint32_t kBucketWords = 16;        // 128 B per bucket

// The per-call counters (u32, zeroed when the workspace is allocated and
// restored by the giant stage's last block at the end of every call).
enum Cnt : uint32_t {
    C_DEFER = 0,        // stage 0 -> stage 0w list
    C_HEAVY32,          // stage 0 over its budget -> heavy stage (G32)
    C_HEAVY64,          // stage 0w over its budget -> heavy stage (G64)
    C_GIANT,            // -> giant stage
    C_TIMED,            // the time limit fired
    C_FIRST_FAIL,       // QSMD_FLAG_EARLY_EXIT_BATCH: first failing history (idle = ~0u)
    C_NEXT32,           // heavy stage queue heads
    C_NEXT64,
    C_TASKS0,           // giant stage: tasks per variant
    C_TASKS1,
    C_TQ0,              // giant stage: task queue heads
    C_TQ1,
    C_GNEXT,            // giant stage: frontier queue head
    C_GDONE,            // giants whose frontier finished
    C_TDONE,            // tasks finished
    C_CNEXT,            // combine queue head
    C_CDONE,            // giants combined
    C_XNEXT,            // early-exit fixup queue head
    C_XDONE,            // fixup chunks finished
    C_EXIT,             // giant-stage blocks finished
    C_WIDE,             // stage 0w -> wave mode's wide list (or, in lane mode, on to the giant stage)
    C_TAIL,             // lane mode -> the wave-mode tail launch (searches past tail_cap iterations)
    C_ZERO,             // always 0 (the tail launch's empty lists)
    C_KHIST = 32,       // heavy_sort: histories per predicted-work key (kKeys)
    C_KCUR = 48,        // heavy_sort: each key's fill cursor
    C_N = 64
};

// Stage 0's heavy list in kShards shards: a group of 64 appends to shard
// (group % kShards), whose counter sits kShardStride words (256 B) from the
// next one (its deferred list the same way, the counter one word after the
// heavy list's: kDeferShardWord).  One counter for the whole batch serialised the appends (one
// returning atomic per wavefront on one address): lone stage 0 at node
// budget 20 took 0.171 ms with it and 0.105 ms without any append.  Shard k
// holds at most ceil(groups / kShards) groups' histories, so shard k's
// entries are list[k * cap .. k * cap + count_k), cap = that bound x 64.
// Consumers see one list through list_total / list_at (index order: shard
// 0's entries, then shard 1's, ...).
// words of a saved stage-0 search state (LaneDFS::save / restore, lane.h)
constexpr uint32_t kResumeWords = 20;
constexpr uint32_t kKeys = 16;     // heavy_sort's key classes (a key past 15 counts as 15)
constexpr uint32_t kSortChunkHost = 256;   // heavy_sort: entries per workgroup and pass (memo.hip kSortChunk)
constexpr uint32_t kShards = 16;
constexpr uint32_t kShardStride = 64;
constexpr uint32_t kDeferShardWord = 1;   // stage 0's deferred list: shard k's counter at [k * kShardStride + 1]

__host__ __device__ inline uint64_t shard_cap(uint64_t n_hist) {
    return ((n_hist + 63) / 64 + kShards - 1) / kShards * 64;
}
// cap == 0: a plain list of *count entries
__device__ __forceinline__ uint32_t list_total(const uint32_t* count, uint32_t cap) {
    if (!cap) return *count;
    uint32_t t = 0;
#pragma unroll
    for (uint32_t k = 0; k < kShards; ++k) t += count[k * kShardStride];
    return t;
}
// the position in `list` of entry idx
__device__ __forceinline__ uint64_t list_pos(const uint32_t* count, uint32_t cap, uint64_t idx) {
    if (!cap) return idx;
    for (uint32_t k = 0; k < kShards; ++k) {
        const uint32_t c = count[k * kShardStride];
        if (idx < c) return (uint64_t)k * cap + idx;
        idx -= c;
    }
    return 0u;   // (idx >= list_total: not reached)
}
__device__ __forceinline__ uint32_t list_at(const uint32_t* list, const uint32_t* count, uint32_t cap, uint64_t idx) {
    return list[list_pos(count, cap, idx)];
}

// Workspace header: counters, buckets (normal and early-exit recount), the
// heavy list's shard counters, and the probe snapshot the last block copies
// for the host.
constexpr size_t kOffCnt = 0;
constexpr size_t kOffBuckets = 256;
constexpr size_t kOffXBuckets = kOffBuckets + (size_t)kBuckets * kBucketWords * 8;
constexpr size_t kOffShards = kOffXBuckets + (size_t)kBuckets * kBucketWords * 8;
constexpr size_t kWsHeader = kOffShards + (size_t)kShards * kShardStride * 4;

// Everything one search launch needs (passed by value).
struct SearchArgs {
    const qsmd_hdr* hdr;
    const uint2* events;          // qsmd_event viewed as {lo word, val}
    uint64_t n_hist;
    uint64_t n_events;            // bound for every ev_off + n_ev
    // list mode: histories are list[0 .. *list_count), else 0 .. n_hist
    // (list_shard_cap > 0: a sharded list, list_total / list_at)
    const uint32_t* list;
    const uint32_t* list_count;
    uint32_t list_shard_cap;
    // histories this stage cannot hold go to defer_list
    uint32_t* defer_list;
    uint32_t* defer_count;
    uint32_t defer_shard_cap;     // > 0: defer_list / defer_count sharded like the heavy list (stage 0)
    // histories over the stage's node budget go to heavy_list (searched
    // again from the root by the heavy stage); null = no stage budget
    uint32_t* heavy_list;
    uint32_t* heavy_count;
    uint32_t heavy_shard_cap;     // > 0: heavy_list / heavy_count sharded (kShards)
    uint32_t* heavy_state;        // stage 0: a heavy history's search state at the budget, slot k x
                                  // heavy_state_cap + (its position in shard k), kResumeWords words each;
                                  // positions past heavy_state_cap save nothing (the heavy stage starts
                                  // those at the root); null = no saved states
    uint32_t heavy_state_cap;
    // stage 0, long heavy lists: a heavy history's predicted work (its
    // untried candidates on the stack, LaneDFS::untried_above, saturated at
    // 255) at its heavy-list position; memo.hip's heavy_sort orders the
    // list by it, so histories of like remaining work share a wavefront
    // (null: none)
    uint8_t* heavy_key;
    uint64_t stage0_budget;
    uint32_t flags;
    uint32_t model_id;
    uint64_t max_nodes;           // 0 = unbounded
    uint64_t time_limit;          // s_memrealtime ticks (100 MHz), 0 = none
    // initial model (model0): Bank exists + balances / Ticket just + n (val[0])
    uint32_t m0_exists;
    uint32_t m0_just;
    uint32_t m0_small;            // every model0 value within 19-bit signed (compact stages)
    uint32_t m0_wave;             // every model0 value within +-2^24 (wave mode's wide list)
    int64_t m0_val[QSMD_BANK_MAX_ACCOUNTS];
    // outputs
    uint8_t* status;
    uint64_t* nodes;              // may be null
    uint8_t* witness;             // may be null
    unsigned long long* buckets;  // [kBuckets][kBucketWords]
    uint32_t* timed_out;          // set to 1 if the time limit fired
    // QSMD_FLAG_EARLY_EXIT_BATCH: smallest index of a history found
    // non-linearisable (or raising); histories above it may stop early and
    // are reported SKIPPED by the giant stage's fixup.  Null when the flag is off.
    uint32_t* first_fail;
    // histories a stage hands on to the giant stage (split search)
    uint32_t* giant_list;
    uint32_t* giant_count;
    // diagnostic build only (tools/diag/compact_diag.patch with
    // QSMD_DIAG_STAGE0=2, stage0_stamps_ptr): stage 0 writes 8 x u64 per
    // group (phase stamps, DFS iterations, the workgroup's entry and exit)
    unsigned long long* stamps;
};

// qsmd_ctx::probe_host slots: [C_DEFER, C_HEAVY32, C_HEAVY64, C_GIANT,
// C_TIMED] of the last finished call, then its wide-list count
constexpr int kProbeWide = 5;
constexpr int kProbeBudget = 6;   // the call's stage-0 budget and batch size (api.hip: the automatic budget)
constexpr int kProbeN = 7;
constexpr int kProbeWritten = 8;  // 1 once a call's giant stage wrote the probe (never reset)
constexpr int kProbeTail = 9;     // the lane-mode searches handed to the wave-mode tail launch
constexpr int kProbeSlots = 10;

// Histories per early-exit fixup chunk of the giant stage (a workgroup takes
// one at a time; a wavefront marks ~0.33 us per row of 64, so short chunks
// spread a small batch's fixup over more workgroups; api.hip sizes the grid
// by them)
constexpr uint32_t kFixupChunk = 512;

// internal status: the search was handed to a later stage (not a result)
constexpr int QSMD_STATUS_HANDED_OFF = 0x40;
constexpr int QSMD_STATUS_TO_TAIL = 0x41;     // lane mode: on to the wave-mode tail launch (internal)

// ------------------------------------------------------------ giant stage
// One history searched by many lanes.  The frontier phase
// runs the reference DFS with a cut at depth D: every node reached at depth
// D roots a task (its subtree), listed in the reference's DFS order with the
// number of nodes the reference counts up to and including that node.  The
// task phase searches the subtrees in parallel; the combine phase folds them
// back in DFS order, so verdict, node count and witness are exactly those of
// the single DFS.
enum { SPLIT_VARIANTS = 2 };          // 0: <= 64 events, <= 8 pids; 1: <= 128 events
constexpr uint32_t kTaskWitness = 64; // bytes per task witness row (<= 64 levels)

struct GiantRec {
    uint32_t h;             // history index
    uint32_t variant;       // SPLIT_VARIANTS index
    uint32_t first;         // first task, index into the variant's task region
    uint32_t n_tasks;
    uint32_t depth;         // cut depth D
    uint32_t term_status;   // how the search above the cut ended (NONLIN = exhausted)
    uint64_t term_nodes;    // nodes counted above the cut when it ended
    uint32_t min_win;       // smallest local task index that decided (LIN / MODEL_ERROR)
    uint32_t pad;
};

struct SplitArgs {
    SearchArgs s;                 // histories, model0, flags, per-history outputs
    uint32_t* cnt;                // the call's counters (Cnt)
    uint32_t* shards;             // the heavy list's shard counters (kShards x kShardStride)
    const uint32_t* giant_list;   // giant g = history giant_list[g]
    const uint32_t* giant_count;
    GiantRec* giants;
    qsmd_task* tasks;             // [SPLIT_VARIANTS][task_cap]
    uint32_t task_cap;
    uint32_t target;              // wanted tasks per giant (0 = no split: searched whole)
    uint32_t max_tasks;           // tasks per giant at most
    uint32_t max_depth;           // cut depth at most (<= QSMD_SPLIT_MAX_DEPTH)
    uint64_t whole_cap;           // iterations of the whole search before the cut (0 = none)
    uint8_t* task_status;         // [SPLIT_VARIANTS][task_cap]
    uint64_t* task_nodes;
    uint8_t* task_witness;        // [SPLIT_VARIANTS][task_cap][kTaskWitness] or null
    unsigned long long* memo;     // QSMD_FLAG_MEMO table (8 x u64 per entry), the exact memo's, or null
    uint64_t memo_mask;           // entries - 1
    uint32_t memo_exact;          // 1: exact-count memo (16 x u64 per entry, epoch-tagged)
    uint32_t memo_epoch;          // this call's tag in either table (24 bits)
    uint32_t external_tasks;      // tasks given by the caller (qsmd_check_tasks)
    uint32_t early;               // QSMD_FLAG_EARLY_EXIT_BATCH: the fixup phase runs
    qsmd_totals* totals;          // the call's totals (device), written by the last block
    uint32_t* probe_host;         // pinned host copy of counters [0..3] (null = none)
    uint32_t probe_budget;        // -> probe_host[kProbeBudget]: the call's stage-0 budget (saturated)
    uint32_t* debug;              // diagnostic: pinned host [grid][4] phase / progress (null = none)
    uint64_t stall_ticks;         // diagnostic (giant_stall_us): the first frontier chunk starts this late
};

// Ordered fold of task results (reference DFS order); shared by the combine
// phase and qsmd_combine_tasks.  Returns the status, sets nodes and the
// winning task (-1 if the decision came from above the cut).
__host__ __device__ inline int combine_tasks(uint32_t term_status, uint64_t term_nodes, const qsmd_task* tasks,
                                             const uint8_t* st, const uint64_t* nd, uint64_t n,
                                             uint64_t max_nodes, uint64_t* nodes_out, int64_t* winner) {
    const uint64_t limit = max_nodes ? max_nodes : ~0ull;
    uint64_t sum = 0;
    *winner = -1;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t s = st[i];
        if (s == QSMD_STATUS_SKIPPED || s == QSMD_STATUS_BUDGET || s > QSMD_STATUS_SKIPPED) {
            *nodes_out = max_nodes && s == QSMD_STATUS_BUDGET ? max_nodes : tasks[i].top_before + sum;
            return s == QSMD_STATUS_SKIPPED ? QSMD_STATUS_SKIPPED : QSMD_STATUS_BUDGET;
        }
        uint64_t total;
        if (__builtin_add_overflow(tasks[i].top_before + sum, nd[i], &total) || total > limit) {
            *nodes_out = limit;              // (a count beyond 2^64 - 1: the budget of u64)
            return QSMD_STATUS_BUDGET;
        }
        sum += nd[i];
        if (s == QSMD_STATUS_LINEARISABLE || s == QSMD_STATUS_MODEL_ERROR) {
            *nodes_out = total;
            *winner = (int64_t)i;
            return (int)s;
        }
    }
    if (term_status == QSMD_STATUS_BUDGET) {
        *nodes_out = max_nodes ? max_nodes : term_nodes + sum;
        return QSMD_STATUS_BUDGET;
    }
    uint64_t total;
    if (__builtin_add_overflow(term_nodes, sum, &total) || total > limit) {
        *nodes_out = limit;
        return QSMD_STATUS_BUDGET;
    }
    *nodes_out = total;
    return (int)term_status;
}

// ------------------------------------------------------------ heavy stage
// wave_search (csrc/wave.hip): one wavefront per history of list32 (<= 32
// events), list64 (<= 64 events) and list_wide (<= 128 events, <= 8 pids;
// the rest of it goes on to the giant stage), the DFS in wave-uniform
// registers with an LDS state memo per wavefront; histories it cannot finish
// within explore_cap iterations go to the giant stage.
struct WaveArgs {
    SearchArgs s;
    const uint32_t* list32;       // (sharded: cap32 > 0, list_total / list_at)
    const uint32_t* count32;
    uint32_t cap32;
    const uint32_t* list64;
    const uint32_t* count64;
    const uint32_t* list_wide;    // stage 0w's deferred histories (> 64 events or wide values); null = every history
    const uint32_t* count_wide;
    uint64_t explore_cap;         // iterations per heavy history before the giant stage (0 = none)
    uint64_t explore_cap_wide;    // the same for the wide list
    uint32_t memo_min_rem;        // nodes with at most this many events left are not memoised
    uint32_t memo_mode;           // QSMD_FLAG_MEMO: a memo hit counts nothing (explored nodes)
    uint32_t buckets;             // LDS memo table: buckets of 64 words (a power of two)
    uint32_t wide128;             // a second launch searches the wide list's 65..128-event histories
    uint32_t dag_states;          // state-DAG capacity per wavefront (0 = DFS only; <= 4095)
    uint32_t dag_items;           // its capacity in (state, candidate) items (<= 65535)
    uint32_t* dbg;                // diagnostic (dag_debug_ptr): the DAG arrays of history dbg_h, or null
    uint32_t dbg_h;
    unsigned long long* stats;    // diagnostic: DFS iterations [max, sum], s_memtime cycles [max, sum], nodes sum,
                                  // DAG-searched histories, their s_memtime cycles max
};
// grid 0: no u64 launch (no history of <= 64 events in the call)
hipError_t launch_wave(const WaveArgs& p, uint32_t grid, uint32_t grid128, hipStream_t s);

// memo_search (csrc/memo.hip): per-lane search of a compact stage's heavy
// histories (s.list / s.list_count) with an exact-count state memo; one
// private table of `entries` (power of two) entries per lane slot of the grid
struct MemoArgs {
    SearchArgs s;
    uint32_t* table;              // grid * 64 * entries * (8 | 16) u32
    uint32_t entries;
    uint32_t memo_after;          // no memo probe / insert before a search has counted this many nodes
    const uint32_t* resume;       // G32 list: stage 0's saved states (SearchArgs::heavy_state), or null
    uint32_t resume_cap;          // their slots per shard (SearchArgs::heavy_state_cap)
    uint32_t lds_entries;         // LDS tables (lds_tables): entries per lane, a power of two <= 64
    uint32_t epoch;               // this call's tag (24 bits)
    uint64_t giant_cap;           // > 0: a search past this many iterations goes to s.giant_list
    const uint32_t* order;        // G32 list: positions in heavy-key order (heavy_sort), or null: list order
    uint64_t tail_cap;            // > 0: a search past this many iterations goes to tail_list (wave mode)
    uint32_t* tail_list;
    uint32_t* tail_count;
    unsigned long long* stats;    // diagnostic (memo_stats_ptr): 8 x u64 per group of the launch, or null
    uint64_t stats_groups;        // groups the stats buffer holds
    const uint32_t* fwd_list;     // appended to s.giant_list as they are (stage 0w's wide list)
    const uint32_t* fwd_count;
};
// lds_tables: the G32 memo tables in LDS (ignored with `wide`; only after
// memo_lds_accepted said yes for p32.lds_entries).  start / stop: events
// the launch records at the kernel's start and end
hipError_t launch_memo(const MemoArgs& p32, const MemoArgs& p64, uint32_t grid, bool wide, bool lds_tables,
                       hipStream_t s, hipEvent_t start, hipEvent_t stop);
bool memo_lds_accepted(uint32_t model_id, uint32_t lds_entries, size_t cap);
// stage 0's heavy list (shards: kShards counters, cap entries each) ordered
// by heavy_key, highest first, into order (positions); cnt: the counters
// (C_KHIST, C_KCUR zero on entry; finish_call restores them)
hipError_t launch_heavy_sort(const uint32_t* shards, uint32_t cap, const uint8_t* key, uint32_t* cnt,
                             uint32_t* order, uint32_t grid, hipStream_t s);

hipError_t launch_gen(const qsmd_gen_params& p, uint64_t first, uint64_t n_hist, uint32_t ev_base, qsmd_hdr* hdr,
                      qsmd_event* events, uint8_t* bug_out, hipStream_t s);

// csrc/wellformed.hip; rank[pid] = position of pid in the `pids` list, 0xFF = not listed
hipError_t launch_wellformed(const qsmd_hdr* hdr, uint64_t n_hist, const uint2* events, uint64_t n_events,
                             const uint8_t* rank, qsmd_wf* out, uint32_t grid, hipStream_t s);

// Early exit: relaxed agent-scope read (a stale value only delays skipping).
__device__ __forceinline__ bool beyond_first_fail(const SearchArgs& a, uint32_t h) {
    return a.first_fail && h > __hip_atomic_load(a.first_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void note_failure(const SearchArgs& a, uint32_t h, int status) {
    if (a.first_fail && (status == QSMD_STATUS_NONLINEARISABLE || status == QSMD_STATUS_MODEL_ERROR))
        atomicMin(a.first_fail, h);
}

// Add a block's counts (one value per lane 0..T_N-1, zero elsewhere) to its
// bucket: one agent-scope atomic per non-zero count.
__device__ __forceinline__ void bucket_add(unsigned long long* buckets, uint32_t block, uint32_t k, uint64_t v) {
    if (v) __hip_atomic_fetch_add(buckets + (uint64_t)(block % kBuckets) * kBucketWords + k, (unsigned long long)v,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Stage 0 (csrc/compact.hip): <= 32 events, <= 8 pids, 19-bit values; the
// launch records `start` / `stop` at the kernel's start and end.
hipError_t launch_compact(const SearchArgs& a, uint32_t grid, hipStream_t s, hipEvent_t start, hipEvent_t stop);
// Stage 0w (csrc/compact.hip, G64): <= 64 events, <= 8 pids, 13/25-bit values, list mode.
hipError_t launch_compact64(const SearchArgs& a, uint32_t grid, hipStream_t s);

// Giant stage (csrc/split.hip): one launch for the frontier, task, combine
// and fixup phases and the totals; frontier-only and task-only launches for
// the split-search entry points.
hipError_t launch_giants(const SplitArgs& p, uint32_t grid, hipStream_t s);
hipError_t launch_frontier_only(int variant, const SplitArgs& p, hipStream_t s);
hipError_t launch_tasks_only(int variant, const SplitArgs& p, uint32_t grid, hipStream_t s);

// A kernel's dynamic-LDS limit (hipFuncAttributeMaxDynamicSharedMemorySize)
// raised once per device to the largest size launched so far: the
// attribute persists, and setting it before every launch cost host time on
// the per-call path.  `cache`: one slot per device, zero-initialised.
constexpr int kAttrDevices = 64;
inline hipError_t ensure_dyn_lds(const void* fn, std::atomic<int>* cache, size_t lds) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kAttrDevices) dev = -1;
    if (dev >= 0 && cache[dev].load(std::memory_order_relaxed) >= (int)lds) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e == hipSuccess && dev >= 0) {
        int cur = cache[dev].load(std::memory_order_relaxed);
        while (cur < (int)lds && !cache[dev].compare_exchange_weak(cur, (int)lds)) {
        }
    }
    return e;
}

}  // namespace qsmd
