// internal.h -- declarations shared by the search kernels and the C-ABI host.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qsmd.h"
#include "qsmd_gen.h"

namespace qsmd {

// Per-block partial totals, reduced into qsmd_totals by reduce_totals().
enum { T_CHECKED = 0, T_LIN, T_NONLIN, T_ERR, T_ENC, T_BUDGET, T_SKIPPED, T_NODES, T_N };

// Everything one search launch needs (passed by value).
struct SearchArgs {
    const qsmd_hdr* hdr;
    const uint2* events;          // qsmd_event viewed as {lo word, val}
    uint64_t n_hist;
    uint64_t n_events;            // bound for every ev_off + n_ev
    // list mode: histories are list[0 .. *list_count), else 0 .. n_hist
    const uint32_t* list;
    const uint32_t* list_count;
    // overflow: histories this stage cannot hold go to defer_list
    uint32_t* defer_list;
    uint32_t* defer_count;
    // stage 0: histories over the stage-0 node budget go to heavy_list
    // (searched again from scratch by the refill stage, whose queue head is
    // queue_head); null heavy_list = no stage-0 budget
    uint32_t* heavy_list;
    uint32_t* heavy_count;
    uint32_t* queue_head;
    uint64_t stage0_budget;
    uint32_t refill_min;          // refill stage: idle lanes before a refill (0 = 8)
    uint32_t flags;
    uint32_t model_id;
    uint64_t max_nodes;           // 0 = unbounded
    uint64_t time_limit;          // s_memrealtime ticks (100 MHz), 0 = none
    // initial model (model0): Bank exists + balances / Ticket just + n (val[0])
    uint32_t m0_exists;
    uint32_t m0_just;
    uint32_t m0_small;            // every model0 value within 19-bit signed (stage 0)
    int64_t m0_val[QSMD_BANK_MAX_ACCOUNTS];
    // outputs
    uint8_t* status;
    uint64_t* nodes;              // may be null
    uint8_t* witness;             // may be null
    unsigned long long* partials; // [gridDim.x][T_N]
    uint32_t* timed_out;          // set to 1 if the time limit fired
    unsigned long long* stamps;   // diagnostic phase timings (null in production)
    // QSMD_FLAG_EARLY_EXIT_BATCH: smallest index of a history found
    // non-linearisable (or raising); histories above it may stop early and
    // are reported SKIPPED by early_exit_fixup.  Null when the flag is off.
    uint32_t* first_fail;
    // split stage (csrc/split.hip): a history whose per-lane search reaches
    // split_budget nodes (< max_nodes) is appended to giant_list and searched
    // again by many lanes.  Null giant_list = no split.
    uint32_t* giant_list;
    uint32_t* giant_count;
    uint64_t split_budget;
    // adaptive cascade probe: histories whose search counted more than
    // probe_nodes nodes (null = no probe)
    uint32_t* probe;
    uint64_t probe_nodes;
    // straggler cut (compact stages with a heavy list): once a wavefront has
    // run cut_min iterations and at most cut_k of its lanes still search,
    // those lanes stop and their histories go to the heavy list (searched
    // again from the root there); cut_count counts them.  0 = off.
    uint32_t cut_k;
    uint32_t cut_min;
    uint32_t* cut_count;
};

// internal status: the search was handed to a later stage (not a result)
constexpr int QSMD_STATUS_HANDED_OFF = 0x40;

// The per-lane node limit of a stage, and whether reaching it hands the
// history to the split stage (rather than being the caller's BUDGET).
__device__ __forceinline__ bool split_enabled(const SearchArgs& a) {
    return a.giant_list && a.split_budget && (!a.max_nodes || a.split_budget < a.max_nodes);
}
__device__ __forceinline__ uint64_t stage_limit(const SearchArgs& a) {
    return split_enabled(a) ? a.split_budget : (a.max_nodes ? a.max_nodes : ~0ull);
}
__device__ __forceinline__ bool to_split(const SearchArgs& a, int status, uint64_t nodes) {
    return status == QSMD_STATUS_BUDGET && split_enabled(a) && nodes >= a.split_budget;
}

// ------------------------------------------------------------ split stage
// One history searched by many lanes.  The frontier kernel
// runs the reference DFS with a cut at depth D: every node reached at depth D
// roots a task (its subtree), listed in the reference's DFS order with the
// number of nodes the reference counts up to and including that node.  The
// task kernel searches the subtrees in parallel; the combine kernel folds
// them back in DFS order, so verdict, node count and witness are exactly
// those of the single DFS.
enum { SPLIT_VARIANTS = 2 };          // 0: <= 64 events, <= 8 pids; 1: <= 128 events
constexpr uint32_t kTaskWitness = 64; // bytes per task witness row (<= 64 levels)

struct GiantRec {
    uint32_t h;             // history index
    uint32_t variant;       // SPLIT_VARIANTS index, ~0u = not (yet) handled
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
    const uint32_t* giant_list;   // giant g = history giant_list[g]
    const uint32_t* giant_count;
    GiantRec* giants;
    qsmd_task* tasks;             // [SPLIT_VARIANTS][task_cap]
    uint32_t* task_count;         // [SPLIT_VARIANTS]
    uint32_t* queue_head;         // [SPLIT_VARIANTS]
    uint32_t task_cap;
    uint32_t target;              // wanted tasks per giant
    uint32_t max_tasks;           // tasks per giant at most
    uint32_t max_depth;           // cut depth at most (<= QSMD_SPLIT_MAX_DEPTH)
    uint8_t* task_status;         // [SPLIT_VARIANTS][task_cap]
    uint64_t* task_nodes;
    uint8_t* task_witness;        // [SPLIT_VARIANTS][task_cap][kTaskWitness] or null
    unsigned long long* memo;     // QSMD_FLAG_MEMO table (8 x u64 per entry), the exact memo's, or null
    uint64_t memo_mask;           // entries - 1
    uint32_t memo_exact;          // 1: exact-count memo (16 x u64 per entry, epoch-tagged)
    uint32_t memo_epoch;          // exact memo: this call's tag (24 bits)
    uint32_t external_tasks;      // tasks given by the caller (qsmd_check_tasks)
};

// Ordered fold of task results (reference DFS order); shared by the combine
// kernel and qsmd_combine_tasks.  Returns the status, sets nodes and the
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

// ------------------------------------------------------------ spread stage
// Dynamic split of the compact-domain histories that exceed the stage-0
// node budget (csrc/spread.hip).  A task is a region of one history's
// reference DFS tree: the subtrees of the remaining candidates `cand` of the
// node reached by the prefix path[0..depth).  Tasks are keyed by their place
// in the reference's DFS order (spread.hip, key digits), so the verdict and
// node count of the single DFS are a fold over the task results in key order.
struct SpreadTask {             // 64 B, 8 x u64 (published with agent-scope stores)
    uint32_t g;                 // heavy-history index (history = heavy_list[g])
    uint32_t cand;              // remaining candidates at the base node (~0u: root)
    uint8_t depth;              // prefix length = base depth
    uint8_t found;              // the base node already had a child before `cand`
    uint8_t status;             // result: QSMD_STATUS_*, or SPREAD_SPLIT / SPREAD_CAP
    uint8_t wdepth;             // LINEARISABLE: witness path length (path[] = the full path)
    uint32_t pad;
    uint64_t key_hi, key_lo;    // DFS-order key
    uint64_t nodes;             // result: nodes this task counted
    uint8_t path[16];           // prefix (and, on LINEARISABLE, the full witness path)
    uint64_t ready;             // = the call's epoch once the record is published
};
static_assert(sizeof(SpreadTask) == 64, "SpreadTask is 64 B");
enum : uint8_t { SPREAD_SPLIT = 6, SPREAD_CAP = 7 };

struct SpreadHist {             // per heavy history
    uint64_t min_hi, min_lo;    // smallest key of a deciding task
    uint64_t sum;               // nodes of the tasks up to and including the decider
    uint64_t explored;          // nodes explored by every task (speculation cap)
    uint32_t flags;             // 1: incomplete (cap) 2: early-exit skip 4: time limit
    uint32_t win_status;
    uint64_t pad;
};

struct SpreadArgs {
    SearchArgs s;                 // histories, model0, flags, per-history outputs
    const uint32_t* heavy_list;
    const uint32_t* heavy_count;
    SpreadTask* tasks;
    uint32_t cap;                 // task capacity
    uint32_t epoch;               // ready-flag value of this call
    SpreadHist* hist;
    unsigned long long* ad;       // (allocated << 32) | done
    uint32_t* head;               // next task slot to take
    uint64_t task_budget;         // nodes a task searches before it splits
    uint64_t explore_cap;         // per-history speculation cap (0 = none)
    uint32_t min_pending;         // split only while fewer tasks than this wait
    uint32_t min_count;           // run only when at least this many histories came (auto mode)
    unsigned long long* stamps;   // diagnostic task timeline (null in production)
    uint32_t* redo_list;          // histories to search again exactly (cap hit)
    uint32_t* redo_count;
};

hipError_t launch_spread(const SpreadArgs& p, uint32_t grid, hipStream_t s);

// ------------------------------------------------------------ coop stage
// One wavefront per heavy compact history (csrc/coop.hip).
struct CoopArgs {
    SearchArgs s;                 // histories, model0, flags, outputs; partials [grid]
    const uint32_t* heavy_list;
    const uint32_t* heavy_count;
    uint32_t* next;               // next heavy history to take (zeroed per call)
    uint64_t budget;              // nodes a task searches before it may split
    uint64_t explore_cap;         // per-history speculation cap (0 = none)
    uint32_t* redo_list;          // histories to search again exactly (cap hit)
    uint32_t* redo_count;
    unsigned long long* stats;    // diagnostic: 8 x u64 per workgroup (null in production)
    uint32_t max_count;           // run only when at most this many histories came (auto mode)
};

hipError_t launch_coop(const CoopArgs& p, uint32_t grid, hipStream_t s);
hipError_t launch_coop64(const CoopArgs& p, uint32_t grid, hipStream_t s);
hipError_t launch_prep(uint32_t* cnt, qsmd_totals* totals, hipStream_t s);
hipError_t launch_gen(const qsmd_gen_params& p, uint64_t first, uint64_t n_hist, uint32_t ev_base, qsmd_hdr* hdr,
                      qsmd_event* events, uint8_t* bug_out, hipStream_t s);

// memo stage (csrc/memo.hip): per-lane search of a compact stage's heavy
// histories (s.list / s.list_count) with an exact-count state memo; one
// private table of `entries` (power of two) entries per lane slot of the grid
struct MemoArgs {
    SearchArgs s;
    uint32_t* table;              // grid * 64 * entries * (8 | 16) u32
    uint32_t entries;
    uint32_t epoch;               // this call's tag (24 bits)
    unsigned long long* stats;    // diagnostic: iterations, hits, inserts, max per history (null = off)
    uint64_t giant_cap;           // > 0: a search past this many iterations goes to s.giant_list
    uint32_t min_rem;             // states with at most this many events left are not memoised
};
hipError_t launch_memo(const MemoArgs& p, uint32_t grid, bool wide, hipStream_t s);

// ------------------------------------------------------------ group stage
// Stage 0 with in-wavefront sharing (csrc/group.hip).  Per-wavefront scratch
// (global memory, touched by its own wavefront only): the task pool and the
// task records of the group's shared history.
struct GroupScratch {
    static constexpr uint32_t kPool = 64, kRec = 256;
    uint32_t cand[kPool], meta[kPool], rem[kPool], model[kPool], stk[4][kPool];
    uint64_t khi[kPool], klo[kPool];
    int32_t bal[QSMD_BANK_MAX_ACCOUNTS][kPool];
    uint64_t rkhi[kRec], rklo[kRec], rnodes[kRec];
};

struct GroupArgs {
    SearchArgs s;                 // histories, outputs, defer list (-> stage 1); partials [grid]
    GroupScratch* scratch;        // [grid]
    uint32_t* group_next;         // group counter (zeroed per call)
    uint64_t task_budget;         // nodes a shared task searches before it may split
    uint32_t share_idle;          // idle lanes needed to start sharing
    uint32_t share_nodes;         // nodes an own search must have counted to be shared
    uint64_t explore_cap;         // per-history speculation cap (0 = none)
    uint32_t* redo_list;          // shared histories to search again exactly (cap hit)
    uint32_t* redo_count;
    unsigned long long* stats;    // diagnostic: 8 x u64 per workgroup (null in production)
    unsigned long long* debug;    // diagnostic: 256 x u64 per workgroup (null in production)
};

hipError_t launch_group(const GroupArgs& p, uint32_t grid, hipStream_t s);

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

hipError_t launch_early_exit_fixup(uint8_t* status, uint64_t* nodes, uint64_t n, const uint32_t* first_fail,
                                   unsigned long long* partials, uint32_t grid, hipStream_t s);

// Stage 0 (csrc/compact.hip): <= 32 events, <= 8 pids, 19-bit values.
hipError_t launch_compact(const SearchArgs& a, uint32_t grid, hipStream_t s);
// Stage 0w (csrc/compact.hip, G64): <= 64 events, <= 8 pids, 13/25-bit values, list mode.
hipError_t launch_compact64(const SearchArgs& a, uint32_t grid, hipStream_t s);
// Stage 0b (csrc/compact.hip): persistent refill search over the heavy list.
hipError_t launch_refill(const SearchArgs& a, uint32_t grid, hipStream_t s);
// Stages 1 and 2 (csrc/search.hip): list mode over the deferred histories.
hipError_t launch_stage(int stage, const SearchArgs& a, uint32_t grid, hipStream_t s);
uint32_t stage_lanes(int stage);
uint32_t stage_max_events(int stage);

hipError_t launch_reduce(const unsigned long long* partials, uint64_t n_blocks,
                         qsmd_totals* totals, hipStream_t s);

// Split stage (csrc/split.hip).
hipError_t launch_frontier(int variant, const SplitArgs& p, uint32_t grid, hipStream_t s);
hipError_t launch_tasks(int variant, const SplitArgs& p, uint32_t grid, hipStream_t s);
hipError_t launch_combine(const SplitArgs& p, uint32_t grid, hipStream_t s);
uint32_t split_lanes(int variant);

}  // namespace qsmd
