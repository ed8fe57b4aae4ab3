// compact.hip -- the search kernels for compact histories: stage 0 (<= 32
// events, <= 8 pids, every value within the compressed encoding) -- every
// history of the reference's own properties (2 clients, suffix <= 6,
// src/QuickCheckHelpers.hs:74) and of the 4x16 / 2x10 benchmark
// configurations -- and stage 0w (<= 64 events, the 6x24 configuration).
//
// The reference search (src/Linearisability.hs:25-69 over the Lemma L1
// event bitset) runs as a per-lane state machine (LaneDFS, lane.h) for a
// divergent 64-lane wavefront where each lane runs its own DFS:
//   * per node, addresses come from registers (pids bit-sliced into three
//     masks P0/P1/P2), so a node costs one LDS round trip for the candidate
//     invocation + its response and (Bank) one for the two balances;
//   * the DFS stack lives in registers: 8 bits per level (candidate index +
//     the two pre-op "account exists" bits Bank's undo needs), 16 levels in
//     4 VGPRs.  The TicketDispenser model needs no undo record at all: it is
//     a function of (depth, mask of levels that applied Reset);
//   * the model's post/next are table lookups and predicated arithmetic, not
//     branches; Bank balances (i32) are the only model state in LDS;
//   * LDS per wavefront: the history (one u32 per event) + Bank balances,
//     [slot][lane] (bank = lane: conflict-free for any per-lane index).
//
// 64 histories per wavefront, staged together (coalesced 16-B loads for
// packed batches), each searched with a node budget: a wavefront runs as
// long as its slowest lane, so a history that exceeds the budget is appended
// to the heavy list (csrc/memo.hip searches it with the exact-count memo).
// Histories outside the stage's bounds go to the next stage through a
// wave-aggregated append to the defer list.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"

// (Diagnostic builds -- stage 0 without its search, per-group phase stamps,
// no heavy-list append -- are a patch applied to a copy of this file by
// tools/build_variant.sh: tools/diag/compact_diag.patch.)

namespace qsmd {

// Run one lane's search to its end (status), with the early-exit and time
// limit checks every 1024 iterations.
template <class DFS>
__device__ __forceinline__ int run_search(DFS& dfs, const SearchArgs& a, const uint32_t* evc,
                                          int32_t (*s_bal)[C_LANES], int lane, uint64_t limit, uint32_t h,
                                          uint64_t t0) {
    int status = -1;
    while (true) {
        // 1024 steps between the checks (the inner loop's only test is the
        // step's one exit, see LaneDFS::step)
        // (a wavefront-uniform counter: the loop runs while any lane
        // searches, the finished lanes masked off)
        for (uint32_t k = 0; k < 1024u; ++k) {
            if (status < 0) status = dfs.template step<C_LANES>(a, evc, s_bal, lane, limit);
            if (__ballot(status < 0) == 0ull) break;
        }
        if (status >= 0) break;
        if (beyond_first_fail(a, h)) {
            status = QSMD_STATUS_SKIPPED;
        } else if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
            atomicOr(a.timed_out, 1u);
            status = QSMD_STATUS_BUDGET;
            dfs.last_j = 32u;          // (no untried candidate: LaneDFS::save)
        }
        if (status >= 0) break;
    }
    return dfs.finish(status);
}

// Stage the histories of the `fresh` lanes (history h) into their LDS
// columns and classify them: returns -2 (deferred to the next stage), -1
// (dfs initialised: search it) or a final status (encode error, the empty
// history, skipped).  When all 64 lanes are fresh with one common length
// and back-to-back events, the block stages coalesced (stage_packed).
// Every lane of the wavefront calls it (the deferral append is a ballot).
template <uint32_t MODEL, class G>
__device__ __forceinline__ int stage_fresh(const SearchArgs& a, bool fresh, uint32_t h, uint32_t (*s_ev)[C_LANES],
                                           int32_t (*s_bal)[C_LANES], int lane, LaneDFS<MODEL, G>& dfs,
                                           qsmd_hdr& H, uint32_t shard) {
    using M = typename G::M;
    if (fresh) H = a.hdr[h];
    else H = qsmd_hdr{0, 0, 0, 0, 0, 0};
    const uint32_t n_ev = H.n_ev, n_pid = H.n_pid;
    const bool enc_ok = fresh && H.model_id == MODEL && n_ev <= QSMD_MAX_EVENTS && n_pid <= QSMD_MAX_PIDS &&
                        (uint64_t)H.ev_off + n_ev <= a.n_events;
    const bool small = enc_ok && n_ev <= (uint32_t)G::EV && n_pid <= 8u && a.m0_small;

    StagedT<M> s{0, 0, 0, 0, 0, true, true};
    // a block: the fresh histories (a prefix of the lanes) with the first
    // one's length, back to back
    const uint64_t F = __ballot(fresh);
    const uint32_t N0 = __builtin_amdgcn_readfirstlane(n_ev);
    const uint32_t off0 = __builtin_amdgcn_readfirstlane(H.ev_off);
    const bool lane_uni = small && n_ev == N0 && H.ev_off == off0 + (uint32_t)lane * N0;
    const bool packed = F != 0ull && __ballot(fresh && !lane_uni) == 0ull && N0 > 0u;
    if (packed) stage_packed<MODEL, G>(a, N0, off0, (uint32_t)__builtin_popcountll(F), s_ev, lane);
    else if (small) stage_lane<MODEL, G>(a, H, s_ev, lane);
    if (small) finish_lane<MODEL, G>(s_ev, lane, n_ev, n_pid, a.events + H.ev_off, s);
    s.ok = s.ok && enc_ok;

    const bool defer = enc_ok && (!small || (s.ok && !s.fits));
    // -> the next stage (stage 0: the group's shard, as the heavy list's --
    // one counter for the batch serialised a wide batch's appends)
    if constexpr (G::EV == 32)
        wave_append(defer, h, a.defer_list + (uint64_t)shard * a.defer_shard_cap,
                    a.defer_count + shard * kShardStride, lane);
    else
        wave_append(defer, h, a.defer_list, a.defer_count, lane);
    if (!fresh || defer) return -2;          // (dfs untouched: the lane may be searching)
    dfs.depth = 0;
    dfs.nodes = 0;
    if (!s.ok) return QSMD_STATUS_ENCODE_ERROR;
    if (n_ev == 0) return QSMD_STATUS_LINEARISABLE;                 // src/Linearisability.hs:59
    if (beyond_first_fail(a, h)) return QSMD_STATUS_SKIPPED;
    dfs.init(s, a, s_bal, lane);
    return -1;
}

// G32: direct over [0, n_hist) (stage 0).  G64: the same search for
// histories of 33..64 events (u64 masks, 16 KB of LDS), run in list mode over
// the histories stage 0 deferred (a.list).
template <uint32_t MODEL, class G = G32>
__global__ __launch_bounds__(C_LANES, G::EV == 32 ? 4 : 2) void compact_search(SearchArgs a) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    __shared__ uint32_t s_ev[G::EV][C_LANES];
    __shared__ int32_t s_bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][C_LANES];

    const int lane = threadIdx.x;
    // (stage 0 runs over the whole batch; stage 0w over stage 0's sharded
    // deferred list, or the whole batch when stage 0 did not run)
    const uint64_t total = G::EV == 32 || !a.list ? a.n_hist : (uint64_t)list_total(a.list_count, a.list_shard_cap);
    if ((uint64_t)blockIdx.x * C_LANES >= total) return;   // (stage 0w of a call that deferred nothing)
    WaveCounters cnt;
    const uint64_t t0 = a.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t user_limit = a.max_nodes ? a.max_nodes : ~0ull;
    const bool tiered = a.stage0_budget < user_limit && a.heavy_list != nullptr;
    const uint64_t limit = tiered ? a.stage0_budget : user_limit;

    // groups of 64 histories, grid-stride
    for (uint64_t base = (uint64_t)blockIdx.x * C_LANES; base < total; base += (uint64_t)gridDim.x * C_LANES) {
        const uint64_t idx = base + lane;
        const bool active = idx < total;
        const uint32_t h = !active ? 0u
                         : G::EV == 32 || !a.list ? (uint32_t)idx : list_at(a.list, a.list_count, a.list_shard_cap, idx);
        const uint32_t shard = (uint32_t)((base / C_LANES) % kShards);
        qsmd_hdr H;
        LaneDFS<MODEL, G> dfs;
        int status = stage_fresh<MODEL, G>(a, active, h, s_ev, s_bal, lane, dfs, H, shard);
        const bool live = status != -2;     // (-2: no history here, or handed to the next stage)
        const bool search = status == -1;
        const uint32_t n_ev = H.n_ev;
        // the general path (pid masks): finish_lane does not pair (lane.h)
        if (search) status = run_search(dfs, a, &s_ev[0][lane], s_bal, lane, limit, h, t0);
        note_failure(a, h, status);
        // over the stage budget (not the caller's): searched again by the heavy stage
        const bool heavy = tiered && status == QSMD_STATUS_BUDGET && dfs.nodes >= limit;
        if (a.heavy_shard_cap) {    // (stage 0: the group's shard, internal.h)
            const uint32_t k = shard;
            const uint32_t at = wave_append(heavy, h, a.heavy_list + (uint64_t)k * a.heavy_shard_cap,
                                            a.heavy_count + k * kShardStride, lane);
            if constexpr (G::EV == 32) {
                if (heavy && a.heavy_state && at < a.heavy_state_cap)
                    dfs.save(a.heavy_state + ((uint64_t)k * a.heavy_state_cap + at) * kResumeWords, s_bal, lane);
                // (long lists: the predicted work, by which the heavy stage's
                // groups are formed -- internal.h heavy_key)
                if (heavy && a.heavy_key) {
                    const uint32_t u = dfs.untried_above();
                    a.heavy_key[(uint64_t)k * a.heavy_shard_cap + at] = (uint8_t)(u < 255u ? u : 255u);
                }
            }
        } else {
            wave_append(heavy, h, a.heavy_list, a.heavy_count, lane);
        }
        const bool out = live && !heavy;
        if (out) {
            a.status[h] = (uint8_t)status;
            if (a.nodes) a.nodes[h] = dfs.nodes;
            if (a.witness && status == QSMD_STATUS_LINEARISABLE) dfs.write_witness(a.witness + H.ev_off, n_ev);
        }
        cnt.add(out, status, dfs.nodes);    // (every lane: the status counts are ballots)
    }
    cnt.flush(a.buckets, lane);
}


hipError_t launch_compact64(const SearchArgs& a, uint32_t grid, hipStream_t s) {
    if (a.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL((compact_search<QSMD_MODEL_BANK, G64>), dim3(grid), dim3(C_LANES), 0, s, a);
    else
        hipLaunchKernelGGL((compact_search<QSMD_MODEL_TICKET, G64>), dim3(grid), dim3(C_LANES), 0, s, a);
    return hipGetLastError();
}

// start / stop: events the launch itself records at the kernel's start and
// end (the per-call stage-0 timing: no launch gap inside the interval)
hipError_t launch_compact(const SearchArgs& a, uint32_t grid, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    if (a.model_id == QSMD_MODEL_BANK)
        hipExtLaunchKernelGGL((compact_search<QSMD_MODEL_BANK, G32>), dim3(grid), dim3(C_LANES), 0, s, start, stop,
                              0u, a);
    else
        hipExtLaunchKernelGGL((compact_search<QSMD_MODEL_TICKET, G32>), dim3(grid), dim3(C_LANES), 0, s, start, stop,
                              0u, a);
    return hipGetLastError();
}

}  // namespace qsmd
