// internal.h -- declarations shared by the search kernels and the C-ABI host.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qsmd.h"

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
};

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
// Stage 0b (csrc/compact.hip): persistent refill search over the heavy list.
hipError_t launch_refill(const SearchArgs& a, uint32_t grid, hipStream_t s);
// Stages 1 and 2 (csrc/search.hip): list mode over the deferred histories.
hipError_t launch_stage(int stage, const SearchArgs& a, uint32_t grid, hipStream_t s);
uint32_t stage_lanes(int stage);
uint32_t stage_max_events(int stage);

hipError_t launch_reduce(const unsigned long long* partials, uint64_t n_blocks,
                         qsmd_totals* totals, hipStream_t s);

}  // namespace qsmd
