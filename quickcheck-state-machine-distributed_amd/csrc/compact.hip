// compact.hip -- the search kernels for small histories (<= 32 events, <= 8
// pids, every value within 19-bit signed): every history of the reference's
// own properties (2 clients, suffix <= 6, src/QuickCheckHelpers.hs:74) and of
// the 4x16 / 2x10 benchmark configurations.
//
// Same search as csrc/search.hip (src/Linearisability.hs:25-69 over the
// Lemma L1 event bitset), as a per-lane state machine (LaneDFS) for a
// divergent 64-lane wavefront where each lane runs its own DFS:
//   * per node, addresses come from registers (pids bit-sliced into three
//     masks P0/P1/P2), so a node costs one LDS round trip for the candidate
//     invocation + its response and (Bank) one for the two balances;
//   * the DFS stack lives in registers: 8 bits per level (candidate index +
//     the two pre-op "account exists" bits Bank's undo needs), 16 levels in
//     4 VGPRs.  The TicketDispenser model needs no undo record at all: it is
//     a function of (depth, mask of levels that applied Reset) -- after the
//     last Reset the model is Just (#TakeTickets since), before any Reset it
//     is model0 advanced by `succ <$>` once per level;
//   * the model's post/next are table lookups and predicated arithmetic, not
//     branches; Bank balances (i32) are the only model state in LDS;
//   * LDS per wavefront: the history (one u32 per event) + Bank balances,
//     [slot][lane] (bank = lane: conflict-free for any per-lane index).
//
// Two kernels share LaneDFS (heavy-tailed search sizes are the enemy of a
// SIMT wavefront, which runs as long as its slowest lane):
//   compact_search  (stage 0)  64 histories per wavefront, staged together
//                   (coalesced 16-B loads for packed batches), each searched
//                   with a node budget; a history that exceeds the budget is
//                   appended to the `heavy` list.
//   refill_search   (stage 0b) persistent wavefronts over the heavy list:
//                   a lane that finishes pulls the next history (wave-
//                   aggregated atomic on a queue head) and stages it into its
//                   own LDS column, so lanes stay busy while long searches
//                   run.
// Histories outside the stage-0 bounds go to stage 1 (search.hip) through a
// wave-aggregated append to the deferred list.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"

namespace qsmd {

// -------------------------------------------------------------- stage 0

// Run one lane's search to its end (status), with the early-exit and time
// limit checks every 1024 iterations.
template <int MODE, class DFS>
__device__ __forceinline__ int run_search(DFS& dfs, const SearchArgs& a, const uint32_t* evc,
                                          int32_t (*s_bal)[C_LANES], int lane, uint64_t limit, uint32_t h,
                                          uint64_t t0) {
    int status;
    uint32_t iter = 0;
    do {                                 // one exit (see LaneDFS::step)
        status = dfs.template step<C_LANES, MODE>(a, evc, s_bal, lane, limit);
        ++iter;
        if (a.cut_k && (iter & 3u) == 0u && iter >= a.cut_min) {   // straggler cut (wave-uniform test)
            const uint64_t live = __ballot(status < 0);
            if ((uint32_t)__builtin_popcountll(live) <= a.cut_k && status < 0) status = QSMD_STATUS_HANDED_OFF;
        }
        if ((iter & 1023u) == 0u && status < 0) {
            if (beyond_first_fail(a, h)) {
                status = QSMD_STATUS_SKIPPED;
            } else if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                atomicOr(a.timed_out, 1u);
                status = QSMD_STATUS_BUDGET;
            }
        }
    } while (status < 0);
    return status;
}

// STAMP = diagnostic build: lane 0 accumulates s_memtime deltas of the
// phases (header+staging, search, output, groups) into a.stamps[block][0..3]
// and records its residency (realtime start/end, HW_ID, XCC_ID) in [4..7].
//
// G64: the same search for histories of 33..64 events (u64 masks, 16 KB of
// LDS), run in list mode over the histories stage 0 deferred (a.list).
template <uint32_t MODEL, bool STAMP, class G = G32>
__global__ __launch_bounds__(C_LANES, G::EV == 32 ? 4 : 2) void compact_search(SearchArgs a) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    using M = typename G::M;
    __shared__ uint32_t s_ev[G::EV][C_LANES];
    __shared__ int32_t s_bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][C_LANES];

    const int lane = threadIdx.x;
    const uint64_t total = a.list ? (uint64_t)*a.list_count : a.n_hist;
    Counters cnt;
    const uint64_t t0 = a.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t user_limit = a.max_nodes ? a.max_nodes : ~0ull;
    const bool tiered = a.stage0_budget < user_limit && a.heavy_list != nullptr;
    const uint64_t limit = tiered ? a.stage0_budget : user_limit;
    uint64_t st_acc[4] = {0, 0, 0, 0}, ts_a = 0, ts_b = 0;
    const uint64_t rt0 = STAMP ? __builtin_amdgcn_s_memrealtime() : 0;

    // groups of 64 histories: this block's first, then (a.queue_head set)
    // dynamically from a counter fetched one group ahead, else grid-stride
    uint32_t next = 0;
    if (a.queue_head && lane == 0) next = atomicAdd(a.queue_head, 1u) + gridDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * C_LANES; base < total;) {
        if constexpr (STAMP) ts_a = __builtin_amdgcn_s_memtime();
        const uint64_t idx = base + lane;
        const bool active = idx < total;
        const uint32_t h = active ? (a.list ? a.list[idx] : (uint32_t)idx) : 0u;
        qsmd_hdr H;
        if (active) H = a.hdr[h];
        else H = qsmd_hdr{0, 0, 0, 0, 0, 0};
        const uint32_t n_ev = H.n_ev, n_pid = H.n_pid;
        const bool enc_ok = active && H.model_id == MODEL && n_ev <= QSMD_MAX_EVENTS &&
                            n_pid <= QSMD_MAX_PIDS && (uint64_t)H.ev_off + n_ev <= a.n_events;
        const bool small = enc_ok && n_ev <= (uint32_t)G::EV && n_pid <= 8u && a.m0_small;

        StagedT<M> s{0, 0, 0, 0, 0, true, true, false};
        const uint32_t N0 = __builtin_amdgcn_readfirstlane(n_ev);
        const uint32_t off0 = __builtin_amdgcn_readfirstlane(H.ev_off);
        const bool lane_uni = active && small && n_ev == N0 && H.ev_off == off0 + (uint32_t)lane * N0;
        const bool packed = __ballot(!lane_uni) == 0ull && N0 > 0u;
        if (packed) stage_packed<MODEL, G>(a, N0, off0, s_ev, lane);
        else if (small) stage_lane<MODEL, G>(a, H, s_ev, lane);
        if (small) finish_lane<G>(s_ev, lane, n_ev, n_pid, s);
        s.ok = s.ok && enc_ok;

        const bool defer = enc_ok && (!small || (s.ok && !s.fits));
        if constexpr (STAMP) {
            ts_b = __builtin_amdgcn_s_memtime();
            st_acc[0] += ts_b - ts_a;
        }
        wave_append(defer, h, a.defer_list, a.defer_count, lane);   // -> stage 1
        // the next group (uniform): counted ahead, or grid-stride
        uint64_t base_next;
        if (a.queue_head) {
            base_next = (uint64_t)(uint32_t)__shfl((int)next, 0, 64) * C_LANES;
            if (lane == 0 && base_next < total) next = atomicAdd(a.queue_head, 1u) + gridDim.x;
        } else {
            base_next = base + (uint64_t)gridDim.x * C_LANES;
        }
        if (!active || defer) {
            base = base_next;
            continue;
        }

        int status = -1;
        LaneDFS<MODEL, G> dfs;
        dfs.depth = 0;
        dfs.nodes = 0;
        bool search = false;
        if (!s.ok) {
            status = QSMD_STATUS_ENCODE_ERROR;
        } else if (n_ev == 0) {
            status = QSMD_STATUS_LINEARISABLE;                       // :59
        } else if (beyond_first_fail(a, h)) {
            status = QSMD_STATUS_SKIPPED;
        } else {
            dfs.init(s, a, s_bal, lane);
            search = true;
        }
        // one specialised loop per wavefront: paired when every searched
        // history of the wavefront is paired
        if (__ballot(search && !s.paired) == 0ull) {
            if (search) status = run_search<M_PAIRED>(dfs, a, &s_ev[0][lane], s_bal, lane, limit, h, t0);
        } else {
            if (search) status = run_search<M_GENERAL>(dfs, a, &s_ev[0][lane], s_bal, lane, limit, h, t0);
        }
        note_failure(a, h, status);
        if constexpr (STAMP) {
            ts_a = __builtin_amdgcn_s_memtime();
            st_acc[1] += ts_a - ts_b;
        }
        // over the stage-0 budget (not the caller's): restart in the refill stage
        // (or cut as a straggler)
        const bool cut = status == QSMD_STATUS_HANDED_OFF;
        const bool heavy = (tiered && status == QSMD_STATUS_BUDGET && dfs.nodes >= limit) || cut;
        wave_append(heavy, h, a.heavy_list, a.heavy_count, lane);
        if (a.cut_count) {
            const uint64_t cm = __ballot(cut);
            if (cm && lane == __builtin_ctzll(cm)) atomicAdd(a.cut_count, (uint32_t)__builtin_popcountll(cm));
        }
        if (heavy) {
            base = base_next;
            continue;
        }

        a.status[h] = (uint8_t)status;
        if (a.nodes) a.nodes[h] = dfs.nodes;
        if (a.witness && status == QSMD_STATUS_LINEARISABLE) dfs.write_witness(a.witness + H.ev_off, n_ev);
        cnt.add(status, dfs.nodes);
        if (a.probe) {                            // adaptive cascade (api.hip): long searches
            const uint64_t pm = __ballot(dfs.nodes > a.probe_nodes);
            if (pm && lane == __builtin_ctzll(pm)) atomicAdd(a.probe, (uint32_t)__builtin_popcountll(pm));
        }
        if constexpr (STAMP) {
            st_acc[2] += __builtin_amdgcn_s_memtime() - ts_a;
            st_acc[3] += 1;
        }
        base = base_next;
    }
    if constexpr (STAMP) {
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) a.stamps[(uint64_t)blockIdx.x * 8 + k] = st_acc[k];
            // residency: realtime (100 MHz) at start / end, HW_ID, XCC_ID
            a.stamps[(uint64_t)blockIdx.x * 8 + 4] = rt0;
            a.stamps[(uint64_t)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_memrealtime();
            a.stamps[(uint64_t)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            a.stamps[(uint64_t)blockIdx.x * 8 + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        }
    }
    cnt.flush(a.partials, lane);
}

// ------------------------------------------------------------- stage 0b

// Persistent wavefronts over the heavy list (*a.list_count entries of
// a.list, head counter a.queue_head).  Idle lanes refill together once at
// least kRefillMin of them are idle (or no lane is busy), with one atomic per
// wavefront; each refilled lane stages its history into its own LDS column.
//
// Direct mode (a.list == null): the same loop over histories 0 .. n_hist-1 as
// a persistent replacement of compact_search; each refilled lane validates
// and stages its own history (deferring the ones stage 0 cannot hold), so a
// lane never waits for the slowest lane of a 64-history group.
template <uint32_t MODEL>
__global__ __launch_bounds__(C_LANES) void refill_search(SearchArgs a) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    __shared__ uint32_t s_ev[C_MAXEV][C_LANES];
    __shared__ int32_t s_bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][C_LANES];

    const int lane = threadIdx.x;
    const bool direct = a.list == nullptr;
    const uint32_t kRefillMin = a.refill_min ? a.refill_min : 8u;
    const uint32_t count = direct ? (uint32_t)a.n_hist : *a.list_count;
    Counters cnt;
    const uint64_t t0 = a.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t limit = stage_limit(a);
    bool busy = false, exhausted = false;
    uint32_t h = 0, iter = 0, n_ev = 0, ev_off = 0;
    LaneDFS<MODEL> dfs;
    dfs.depth = 0;
    dfs.nodes = 0;
    for (;;) {
        const uint64_t idle = __ballot(!busy);
        const uint64_t busy_m = __ballot(busy);
        if (!exhausted && idle && (__builtin_popcountll(idle) >= kRefillMin || busy_m == 0)) {
            const int leader = __builtin_ctzll(idle);
            const uint32_t want = (uint32_t)__builtin_popcountll(idle);
            uint32_t first = 0;
            if (lane == leader) first = atomicAdd(a.queue_head, want);
            first = __shfl(first, leader, 64);
            if (first + want >= count) exhausted = true;
            if (!busy) {
                const uint32_t idx = first + lane_prefix(idle);
                const uint32_t hh = idx < count ? (direct ? idx : a.list[idx]) : 0u;
                if (idx < count && !beyond_first_fail(a, hh)) {   // else: early_exit_fixup
                    h = hh;
                    const qsmd_hdr H = a.hdr[h];
                    n_ev = H.n_ev;
                    ev_off = H.ev_off;
                    bool enc_ok = true, small = true;
                    if (direct) {                             // stage 0's checks
                        enc_ok = H.model_id == MODEL && n_ev <= QSMD_MAX_EVENTS && H.n_pid <= QSMD_MAX_PIDS &&
                                 (uint64_t)ev_off + n_ev <= a.n_events;
                        small = enc_ok && n_ev <= (uint32_t)C_MAXEV && H.n_pid <= 8u && a.m0_small;
                    }
                    Staged s{0u, 0u, 0u, 0u, 0u, true, true, false};
                    if (small) {                              // (list mode: validated by stage 0)
                        stage_lane<MODEL>(a, H, s_ev, lane);
                        finish_lane(s_ev, lane, n_ev, H.n_pid, s);
                    }
                    if (enc_ok && (!small || (s.ok && !s.fits))) {
                        a.defer_list[atomicAdd(a.defer_count, 1u)] = h;        // -> stage 1
                    } else if (!enc_ok || !s.ok || n_ev == 0) {
                        const int st = n_ev == 0 && enc_ok ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_ENCODE_ERROR;
                        a.status[h] = (uint8_t)st;
                        if (a.nodes) a.nodes[h] = 0;
                        cnt.add(st, 0);
                    } else {
                        dfs.init(s, a, s_bal, lane);
                        busy = true;
                    }
                }
            }
        }
        if (exhausted && __ballot(busy) == 0) break;
        if (busy) {
            int status = dfs.template step<C_LANES, M_LANE>(a, &s_ev[0][lane], s_bal, lane, limit);
            if (status < 0 && ((iter + 1u) & 1023u) == 0u && beyond_first_fail(a, h))
                status = QSMD_STATUS_SKIPPED;
            if (status < 0 && time_up(a, t0, iter)) {
                atomicOr(a.timed_out, 1u);
                status = QSMD_STATUS_BUDGET;
            }
            if (status >= 0 && to_split(a, status, dfs.nodes)) {   // -> split stage
                a.giant_list[atomicAdd(a.giant_count, 1u)] = h;
                busy = false;
            } else if (status >= 0) {
                note_failure(a, h, status);
                a.status[h] = (uint8_t)status;
                if (a.nodes) a.nodes[h] = dfs.nodes;
                if (a.witness && status == QSMD_STATUS_LINEARISABLE) dfs.write_witness(a.witness + ev_off, n_ev);
                cnt.add(status, dfs.nodes);
                busy = false;
            }
        }
    }
    cnt.flush(a.partials, lane);
}

hipError_t launch_compact64(const SearchArgs& a, uint32_t grid, hipStream_t s) {
    if (a.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL((compact_search<QSMD_MODEL_BANK, false, G64>), dim3(grid), dim3(C_LANES), 0, s, a);
    else
        hipLaunchKernelGGL((compact_search<QSMD_MODEL_TICKET, false, G64>), dim3(grid), dim3(C_LANES), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_compact(const SearchArgs& a, uint32_t grid, hipStream_t s) {
    const bool bank = a.model_id == QSMD_MODEL_BANK;
    if (a.stamps) {
        if (bank) hipLaunchKernelGGL((compact_search<QSMD_MODEL_BANK, true>), dim3(grid), dim3(C_LANES), 0, s, a);
        else hipLaunchKernelGGL((compact_search<QSMD_MODEL_TICKET, true>), dim3(grid), dim3(C_LANES), 0, s, a);
    } else {
        if (bank) hipLaunchKernelGGL((compact_search<QSMD_MODEL_BANK, false>), dim3(grid), dim3(C_LANES), 0, s, a);
        else hipLaunchKernelGGL((compact_search<QSMD_MODEL_TICKET, false>), dim3(grid), dim3(C_LANES), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_refill(const SearchArgs& a, uint32_t grid, hipStream_t s) {
    if (a.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL(refill_search<QSMD_MODEL_BANK>, dim3(grid), dim3(C_LANES), 0, s, a);
    else
        hipLaunchKernelGGL(refill_search<QSMD_MODEL_TICKET>, dim3(grid), dim3(C_LANES), 0, s, a);
    return hipGetLastError();
}

}  // namespace qsmd
