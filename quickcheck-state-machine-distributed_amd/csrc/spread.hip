// spread.hip -- the spread stage: dynamic split of the compact-domain
// histories (<= 32 events, <= 8 pids) whose search exceeds the stage-0 node
// budget.
//
// A wavefront runs as long as its slowest lane, and one lane searches one
// history at ~0.5 us per node, so a history of 10^4..10^5 nodes (the 4x16
// Bank batch with injected bugs) or the rare 10^2-node one in a batch of
// 10^6 sets the length of the whole launch.  This stage searches such a
// history with as many lanes as its tree can feed, with no static frontier:
//
//   task       a region of the reference DFS tree (src/Linearisability.hs:
//              52-69): the subtrees of the remaining candidates `cand` of the
//              node N reached by the prefix path[0..depth).  The root task of
//              a history is the whole tree.
//   split      a lane that has counted `task_budget` nodes in its task stops
//              and publishes what it has not searched as range tasks, one per
//              level between its base and its current node N: at each level
//              the candidates after the one the path went through (at N: the
//              untried candidates, including the one it was about to count).
//              Its own result is "no decision in the part searched, k nodes".
//   key        every task carries its place in the reference's DFS order: a
//              digit string, digit i = 2*(j+1) for a path step through
//              candidate event j at level i, and 2*c+1 at the task's own
//              level for "candidates c, c+1, ... of this node".  Keys compare
//              lexicographically (a prefix first); a task's explored nodes
//              come after every task of smaller key and before every task of
//              larger key.
//   fold       the reference stops at the first deciding node (a success, or
//              Map.! raising).  Its node count is therefore the sum of the
//              nodes of every task whose key is below the deciding task's,
//              plus the decider's own count -- or the sum of all when nothing
//              decides (non-linearisable).  Three grid-stride passes over the
//              tasks (min key, then sum) and one per history.
//   cancel     a task that decides lowers its history's minimum key; tasks
//              whose key is above it stop (they lie after the decision in DFS
//              order and cannot change the result).
//
// Work distribution: a persistent grid; idle lanes take task slots with one
// atomic per wavefront, wait for the slot to be published, stage the
// history into their LDS column (per-lane staging, lane.h), replay the
// prefix (transitions only) and search.  Termination: the packed word
// ad = (allocated << 32) | done; a split adds its k children and its own
// completion in ONE atomic, so done == allocated holds only when no task is
// running and none is unpublished.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"

namespace qsmd {

namespace {

constexpr uint32_t kRootCand = ~0u;
constexpr uint32_t kNullTask = ~0u;     // g of a slot whose block did not fit the capacity

__device__ __forceinline__ uint64_t ld_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, uint64_t v) {
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long* words(SpreadTask* t) {
    return reinterpret_cast<unsigned long long*>(t);
}

// key digit i of a path/range (7 bits): hi holds digits 0..8, lo 9..15
__device__ __forceinline__ void key_put(uint64_t& hi, uint64_t& lo, uint32_t i, uint64_t d) {
    if (i < 9u) hi |= d << (56u - 7u * i);
    else lo |= d << (56u - 7u * (i - 9u));
}

__device__ __forceinline__ bool key_less(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah < bh || (ah == bh && al < bl);
}

// Events removed at level d of the current path (the candidate's pid: its
// last removed invocation and response -- the restore of a backtrack).
template <uint32_t MODEL>
__device__ __forceinline__ uint32_t removed_at(const LaneDFS<MODEL>& dfs, const uint32_t* evc, uint32_t rem,
                                               uint32_t j) {
    if (dfs.paired) return (1u << j) | (1u << c_r(evc[j * C_LANES]));
    const uint32_t gone = ~rem & dfs.same_pid(j);
    return (1u << (31 - __builtin_clz(gone & dfs.INV))) | (1u << (31 - __builtin_clz(gone & dfs.RESP)));
}

// Walk the levels base..D of the lane's current position from the deepest
// up, calling emit(level, cand, found) for every non-empty remaining range.
// At level D (the current node) the range is the untried candidates plus
// `extra` (the candidate whose node the budget did not count).
template <uint32_t MODEL, typename F>
__device__ __forceinline__ void for_each_range(const LaneDFS<MODEL>& dfs, const uint32_t* evc, uint32_t extra,
                                               F&& emit) {
    uint32_t rem = dfs.rem;
    const uint32_t top = dfs.cand | extra;
    if (top) emit(dfs.depth, top, dfs.found);
    for (uint32_t l = dfs.depth; l-- > dfs.base;) {
        const uint32_t j = dfs.stk.get(l, dfs.depth) & 31u;
        rem |= removed_at(dfs, evc, rem, j);
        const uint32_t c = cands(rem, dfs.INV, dfs.RESP) & mask_above(j, 0u);
        if (c) emit(l, c, 1u);
    }
}

// diagnostic timeline (p.stamps, 4 x u64 per task slot): s_memrealtime at
// slot assignment, task start, search start (after staging + replay), end
__device__ __forceinline__ void stamp(const SpreadArgs& p, uint32_t slot, int k) {
    if (p.stamps && slot < p.cap) p.stamps[(uint64_t)slot * 4 + k] = __builtin_amdgcn_s_memrealtime();
}

struct Lane {
    uint32_t phase;      // 0 idle, 1 waiting for `slot`, 2 searching `slot`, 3 finished
    uint32_t slot, g, h;
    uint64_t key_hi, key_lo, limit;
};

}  // namespace

// ---------------------------------------------------------------- kernels

// Root task per heavy history, per-history records, counters.
__device__ __forceinline__ uint32_t spread_count(const SpreadArgs& p) {
    const uint32_t n = *p.heavy_count;
    return n >= p.min_count ? n : 0u;           // auto mode: few histories go to the coop stage
}

__global__ void spread_init_kernel(SpreadArgs p) {
    const uint32_t n = spread_count(p);
    const uint32_t n_root = n < p.cap ? n : p.cap;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < n; g += gridDim.x * blockDim.x) {
        SpreadHist& r = p.hist[g];
        r.min_hi = ~0ull;
        r.min_lo = ~0ull;
        r.sum = 0;
        r.explored = 0;
        r.flags = g < n_root ? 0u : 1u;            // beyond the task capacity: searched again exactly
        r.win_status = QSMD_STATUS_NONLINEARISABLE;
        if (g < n_root) {
            SpreadTask t{};
            t.g = g;
            t.cand = kRootCand;
            t.status = QSMD_STATUS_SKIPPED;
            t.ready = p.epoch;
            p.tasks[g] = t;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *p.ad = (unsigned long long)n_root << 32;
        *p.head = 0;
    }
}

template <uint32_t MODEL>
__global__ __launch_bounds__(C_LANES) void spread_search(SpreadArgs p) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    __shared__ uint32_t s_ev[C_MAXEV][C_LANES];
    __shared__ int32_t s_bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][C_LANES];
    const SearchArgs& a = p.s;
    const int lane = threadIdx.x;
    const uint32_t* evc = &s_ev[0][lane];
    const uint32_t refill_min = a.refill_min ? a.refill_min : 8u;
    const uint64_t t0 = a.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    LaneDFS<MODEL> dfs;
    dfs.depth = 0;
    dfs.nodes = 0;
    Lane L{0u, 0u, 0u, 0u, 0ull, 0ull, 0ull};
    uint32_t backoff = 1u, tick = 0u, my_done = 0u;

    // task result: record, explored count, the history's minimum deciding key, done += 1
    auto finish = [&](int st) {
        stamp(p, L.slot, 3);
        SpreadTask* t = p.tasks + L.slot;
        t->status = (uint8_t)st;
        t->nodes = dfs.nodes;
        if (st == QSMD_STATUS_LINEARISABLE) {
            t->wdepth = (uint8_t)dfs.depth;
            for (uint32_t d = 0; d < dfs.depth; ++d) t->path[d] = (uint8_t)(dfs.stk.get(d, dfs.depth) & 31u);
        }
        if (p.explore_cap && dfs.nodes)
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.hist[L.g].explored), dfs.nodes);
        if (st == QSMD_STATUS_LINEARISABLE || st == QSMD_STATUS_MODEL_ERROR)
            atomicMin(reinterpret_cast<unsigned long long*>(&p.hist[L.g].min_hi), L.key_hi);
        if (st == QSMD_STATUS_BUDGET) atomicOr(&p.hist[L.g].flags, 4u);
        if (st == SPREAD_CAP) atomicOr(&p.hist[L.g].flags, 1u);
        if (st == QSMD_STATUS_SKIPPED && beyond_first_fail(a, L.h)) atomicOr(&p.hist[L.g].flags, 2u);
        ++my_done;                               // flushed once the wavefront is idle
        L.phase = 0u;
    };

    // publish the unsearched rest of the task as range tasks, when idle
    // lanes want work (fewer than p.min_pending tasks wait); false = search on
    auto split = [&]() -> bool {
        const unsigned long long v0 = ld_agent(p.ad);
        const uint32_t hd = __hip_atomic_load(p.head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t alloc0 = (uint32_t)(v0 >> 32);
        if (alloc0 > hd && alloc0 - hd >= p.min_pending) return false;
        const uint32_t extra = 1u << dfs.last_j;
        uint32_t k = 0;
        for_each_range(dfs, evc, extra, [&](uint32_t, uint32_t, uint32_t) { ++k; });
        // children + own completion in one add
        const unsigned long long v = atomicAdd(p.ad, ((unsigned long long)k << 32) + 1ull);
        const uint32_t first = (uint32_t)(v >> 32);
        const bool room = first + k <= p.cap;
        uint32_t i = 0;
        uint8_t path[16];
        for (uint32_t d = 0; d < 16u; ++d) path[d] = d < dfs.depth ? (uint8_t)(dfs.stk.get(d, dfs.depth) & 31u) : 0u;
        for_each_range(dfs, evc, extra, [&](uint32_t lvl, uint32_t c, uint32_t found) {
            if (first + i < p.cap) {
                unsigned long long* w = words(p.tasks + first + i);
                if (room) {
                    uint64_t hi = 0, lo = 0;
                    uint32_t pw[4] = {0u, 0u, 0u, 0u};
                    for (uint32_t d = 0; d < lvl; ++d) {
                        key_put(hi, lo, d, 2ull * (path[d] + 1u));
                        pw[d >> 2] |= (uint32_t)path[d] << ((d & 3u) * 8u);
                    }
                    key_put(hi, lo, lvl, 2ull * __builtin_ctz(c) + 1ull);
                    st_agent(w + 0, (uint64_t)L.g | ((uint64_t)c << 32));
                    st_agent(w + 1, (uint64_t)lvl | ((uint64_t)found << 8) | ((uint64_t)QSMD_STATUS_SKIPPED << 16));
                    st_agent(w + 2, hi);
                    st_agent(w + 3, lo);
                    st_agent(w + 4, 0ull);
                    st_agent(w + 5, (uint64_t)pw[0] | ((uint64_t)pw[1] << 32));
                    st_agent(w + 6, (uint64_t)pw[2] | ((uint64_t)pw[3] << 32));
                } else {
                    st_agent(w + 0, (uint64_t)kNullTask);          // a slot of a block that did not fit
                }
            }
            ++i;
        });
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (uint32_t q = 0; q < k; ++q)
            if (first + q < p.cap) st_agent(words(p.tasks + first + q) + 7, p.epoch);
        if (!room) {
            // the block's null slots count as done; this task is not: undo its completion
            atomicAdd(p.ad, (unsigned long long)k - 1ull);
            return false;
        }
        stamp(p, L.slot, 3);
        SpreadTask* t = p.tasks + L.slot;     // this task: "no decision in the part searched"
        t->status = SPREAD_SPLIT;
        t->nodes = dfs.nodes;
        if (p.explore_cap)
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.hist[L.g].explored), dfs.nodes);
        L.phase = 0u;
        return true;
    };

    // start the task in slot L.slot (published): record, stage, replay
    auto start = [&]() {
        stamp(p, L.slot, 1);
        unsigned long long* w = words(p.tasks + L.slot);
        const uint64_t w0 = ld_agent(w + 0), w1 = ld_agent(w + 1);
        L.g = (uint32_t)w0;
        if (L.g == kNullTask) {                  // counted as done by its producer
            L.phase = 0u;
            return;
        }
        L.key_hi = ld_agent(w + 2);
        L.key_lo = ld_agent(w + 3);
        const uint64_t w5 = ld_agent(w + 5), w6 = ld_agent(w + 6);
        const uint32_t cand = (uint32_t)(w0 >> 32), depth = (uint32_t)w1 & 0xFFu,
                       found = (uint32_t)(w1 >> 8) & 0xFFu;
        L.h = p.heavy_list[L.g];
        L.phase = 2u;
        L.limit = p.task_budget;
        dfs.nodes = 0;
        dfs.depth = 0;
        const uint64_t mh = ld_agent(reinterpret_cast<unsigned long long*>(&p.hist[L.g].min_hi));
        const bool capped = p.explore_cap &&
                            ld_agent(reinterpret_cast<unsigned long long*>(&p.hist[L.g].explored)) > p.explore_cap;
        if (beyond_first_fail(a, L.h) || L.key_hi > mh) {
            finish(QSMD_STATUS_SKIPPED);
        } else if (capped) {
            finish(SPREAD_CAP);
        } else {
            const qsmd_hdr H = a.hdr[L.h];
            Staged s{0u, 0u, 0u, 0u, 0u, true, true, false};
            stage_lane<MODEL>(a, H, s_ev, lane);
            finish_lane(s_ev, lane, H.n_ev, H.n_pid, s);
            dfs.init(s, a, s_bal, lane);
            // replay the prefix: transitions only, nothing counted
            for (uint32_t d = 0; d < depth; ++d) {
                const uint32_t j = d < 8u ? (uint32_t)(w5 >> (8u * d)) & 0xFFu
                                          : (uint32_t)(w6 >> (8u * (d - 8u))) & 0xFFu;
                dfs.cand = 1u << j;
                (void)dfs.template step<C_LANES, M_LANE>(a, evc, s_bal, lane, ~0ull);
            }
            dfs.nodes = 0;
            dfs.base = depth;
            if (cand != kRootCand) {
                dfs.cand = cand;
                dfs.found = found;
            }
            stamp(p, L.slot, 2);
        }
    };

    // Polls are software-pipelined: the counters and ready flags loaded at
    // the end of one iteration are used at the start of the next, so the
    // searching lanes of the wavefront do not wait for them.
    unsigned long long nx_ad = 0, nx_ready = 0;
    uint32_t nx_head = 0, grab_first = 0, grab_n = 0;
    bool polled = false;
    for (;;) {
        ++tick;
        const uint64_t busy = __ballot(L.phase == 2u);
        if (busy == 0ull && __ballot(my_done != 0u)) {   // flush the completions: one add per wavefront
            const uint32_t tot = (uint32_t)wave_sum64(my_done);
            my_done = 0u;
            if (lane == 0) atomicAdd(p.ad, (unsigned long long)tot);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            polled = false;                      // re-poll after the flush
        }
        // consume a poll once it has had time to land: every iteration while
        // no lane searches, else every 8th (issued 7 iterations earlier)
        if (polled && (busy == 0ull || (tick & 7u) == 0u)) {
            polled = false;
            const unsigned long long v = nx_ad;
            const uint32_t alloc = (uint32_t)(v >> 32), done = (uint32_t)v;
            // ---- the grab issued last iteration: slots for the idle lanes
            if (grab_n) {
                const uint32_t gf = __shfl(grab_first, 0, 64);
                const uint64_t idle = __ballot(L.phase == 0u);
                const uint32_t k = lane_prefix(idle);
                if (L.phase == 0u && k < grab_n) {
                    L.slot = gf + k;
                    L.phase = 1u;
                    stamp(p, L.slot, 0);
                }
                backoff = 1u;
            }
            // ---- waiting lanes: start a published task, or finish for good
            if (L.phase == 1u) {
                if (L.slot < alloc && L.slot >= p.cap) {
                    L.phase = 0u;                        // a null slot beyond the capacity
                } else if (L.slot < alloc && nx_ready == p.epoch) {
                    start();
                } else if (done == alloc && L.slot >= alloc) {
                    L.phase = 3u;                        // nothing can be published any more
                } else if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > 2 * a.time_limit) {
                    atomicOr(a.timed_out, 1u);           // safety net: never spin for ever
                    L.phase = 3u;
                }
            }
            // ---- idle lanes: take allocated slots (one atomic per wavefront)
            const uint64_t idle = __ballot(L.phase == 0u);
            grab_n = 0;
            if (idle) {
                const uint32_t avail = alloc > nx_head ? alloc - nx_head : 0u;
                if (avail && (busy == 0ull || __builtin_popcountll(idle) >= refill_min)) {
                    grab_n = min((uint32_t)__builtin_popcountll(idle), avail);
                    if (lane == 0) grab_first = atomicAdd(p.head, grab_n);
                } else if (!avail && done == alloc) {
                    if (L.phase == 0u) L.phase = 3u;
                }
            }
        }
        // ---- issue the polls for the next iteration
        const uint64_t want = __ballot(L.phase == 0u || L.phase == 1u);
        if (want && !polled && (busy == 0ull || (tick & 7u) == 1u || __ballot(L.phase == 2u) == 0ull)) {
            polled = true;
            nx_ad = ld_agent(p.ad);
            nx_head = __hip_atomic_load(p.head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            nx_ready = (L.phase == 1u && L.slot < p.cap) ? ld_agent(words(p.tasks + L.slot) + 7) : 0ull;
        }
        // ---- searching lanes: one DFS iteration
        if (L.phase == 2u) {
            int st = dfs.template step<C_LANES, M_LANE>(a, evc, s_bal, lane, L.limit);
            if ((tick & 63u) == 0u && st < 0) {          // wave-synchronous: one round trip per 64
                const uint64_t mh = ld_agent(reinterpret_cast<unsigned long long*>(&p.hist[L.g].min_hi));
                if (L.key_hi > mh || beyond_first_fail(a, L.h)) st = QSMD_STATUS_SKIPPED;
                else if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                    atomicOr(a.timed_out, 1u);
                    st = QSMD_STATUS_BUDGET;
                }
            }
            if (st == QSMD_STATUS_BUDGET && dfs.nodes >= L.limit) {
                // task budget reached: split, or search on
                const bool capped = p.explore_cap &&
                                    ld_agent(reinterpret_cast<unsigned long long*>(&p.hist[L.g].explored)) +
                                            dfs.nodes > p.explore_cap;
                if (capped) {
                    finish(SPREAD_CAP);
                } else if (!split()) {
                    dfs.cand |= 1u << dfs.last_j;
                    L.limit += p.task_budget;
                }
            } else if (st >= 0) {
                finish(st);
            }
        }
        if (__ballot(L.phase != 3u) == 0ull) break;
        if (__ballot(L.phase == 2u) == 0ull) {          // nothing to search: back off
            for (uint32_t q = 0; q < backoff; ++q) __builtin_amdgcn_s_sleep(8);
            backoff = backoff < 16u ? 2u * backoff : 16u;
        }
    }
}

// fold pass A / B: the smallest key of a deciding task, per history
__global__ void spread_fold_min(SpreadArgs p, int pass) {
    const uint32_t n = min((uint32_t)(*p.ad >> 32), p.cap);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const SpreadTask& t = p.tasks[i];
        if (t.g == kNullTask) continue;
        if (t.status != QSMD_STATUS_LINEARISABLE && t.status != QSMD_STATUS_MODEL_ERROR) continue;
        SpreadHist& r = p.hist[t.g];
        if (pass == 0) atomicMin(reinterpret_cast<unsigned long long*>(&r.min_hi), t.key_hi);
        else if (t.key_hi == r.min_hi) atomicMin(reinterpret_cast<unsigned long long*>(&r.min_lo), t.key_lo);
    }
}

// fold pass C: nodes of every task up to the decider; the decider's status
// and witness; flags of tasks before it
__global__ void spread_fold_sum(SpreadArgs p) {
    const uint32_t n = min((uint32_t)(*p.ad >> 32), p.cap);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const SpreadTask& t = p.tasks[i];
        if (t.g == kNullTask) continue;
        SpreadHist& r = p.hist[t.g];
        const bool win = t.key_hi == r.min_hi && t.key_lo == r.min_lo &&
                         (t.status == QSMD_STATUS_LINEARISABLE || t.status == QSMD_STATUS_MODEL_ERROR);
        if (!win && !key_less(t.key_hi, t.key_lo, r.min_hi, r.min_lo)) continue;
        atomicAdd(reinterpret_cast<unsigned long long*>(&r.sum), t.nodes);
        if (t.status == SPREAD_CAP) atomicOr(&r.flags, 1u);
        if (t.status == QSMD_STATUS_SKIPPED) atomicOr(&r.flags, 2u);
        if (t.status == QSMD_STATUS_BUDGET) atomicOr(&r.flags, 4u);
        if (win) {
            r.win_status = t.status;
            const uint32_t h = p.heavy_list[t.g];
            if (p.s.witness && t.status == QSMD_STATUS_LINEARISABLE) {
                const qsmd_hdr H = p.s.hdr[h];
                uint8_t* w = p.s.witness + H.ev_off;
                for (uint32_t d = 0; d < t.wdepth; ++d) w[d] = t.path[d];
                if (t.wdepth < H.n_ev) w[t.wdepth] = QSMD_WITNESS_END;
            }
        }
    }
}

// per history: status, nodes, counters (partials[gridDim.x]); a history the
// speculation cap left incomplete goes to the redo list
__global__ void spread_final(SpreadArgs p) {
    const uint32_t n = spread_count(p);
    uint32_t c[T_N] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t nodes_sum = 0;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < n; g += gridDim.x * blockDim.x) {
        const SpreadHist& r = p.hist[g];
        const uint32_t h = p.heavy_list[g];
        int st;
        uint64_t nd = r.sum;
        if (r.flags & 2u) {
            st = QSMD_STATUS_SKIPPED;
            nd = 0;
        } else if (r.flags & 4u) {
            st = QSMD_STATUS_BUDGET;
            if (p.s.max_nodes) nd = p.s.max_nodes;
        } else if (r.flags & 1u) {
            p.redo_list[atomicAdd(p.redo_count, 1u)] = h;
            continue;
        } else {
            st = (int)r.win_status;
            if (p.s.max_nodes && nd > p.s.max_nodes) {
                st = QSMD_STATUS_BUDGET;
                nd = p.s.max_nodes;
            }
        }
        note_failure(p.s, h, st);
        p.s.status[h] = (uint8_t)st;
        if (p.s.nodes) p.s.nodes[h] = nd;
        if (st != QSMD_STATUS_SKIPPED) {
            c[T_LIN] += st == QSMD_STATUS_LINEARISABLE;
            c[T_NONLIN] += st == QSMD_STATUS_NONLINEARISABLE;
            c[T_ERR] += st == QSMD_STATUS_MODEL_ERROR;
            c[T_BUDGET] += st == QSMD_STATUS_BUDGET;
            nodes_sum += nd;
        }
    }
    // block reduction into this block's partials row
    __shared__ unsigned long long red[T_N];
    if (threadIdx.x < T_N) red[threadIdx.x] = 0;
    __syncthreads();
    atomicAdd(&red[T_LIN], (unsigned long long)c[T_LIN]);
    atomicAdd(&red[T_NONLIN], (unsigned long long)c[T_NONLIN]);
    atomicAdd(&red[T_ERR], (unsigned long long)c[T_ERR]);
    atomicAdd(&red[T_BUDGET], (unsigned long long)c[T_BUDGET]);
    atomicAdd(&red[T_NODES], (unsigned long long)nodes_sum);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long* row = p.s.partials + (uint64_t)blockIdx.x * T_N;
        row[T_CHECKED] = red[T_LIN] + red[T_NONLIN] + red[T_ERR];
        row[T_LIN] = red[T_LIN];
        row[T_NONLIN] = red[T_NONLIN];
        row[T_ERR] = red[T_ERR];
        row[T_ENC] = 0;
        row[T_BUDGET] = red[T_BUDGET];
        row[T_SKIPPED] = 0;
        row[T_NODES] = red[T_NODES];
    }
}

constexpr uint32_t kFoldGrid = 128, kFoldBlock = 256;

// spread_final's grid (its partials rows)
uint32_t spread_final_grid() { return 64; }   // = kSpreadFinalGrid (api.hip)

hipError_t launch_spread(const SpreadArgs& p, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(spread_init_kernel, dim3(64), dim3(256), 0, s, p);
    if (p.s.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL(spread_search<QSMD_MODEL_BANK>, dim3(grid), dim3(C_LANES), 0, s, p);
    else
        hipLaunchKernelGGL(spread_search<QSMD_MODEL_TICKET>, dim3(grid), dim3(C_LANES), 0, s, p);
    // (pass A, the minimum key_hi of the deciders, was taken by the search itself)
    hipLaunchKernelGGL(spread_fold_min, dim3(kFoldGrid), dim3(kFoldBlock), 0, s, p, 1);
    hipLaunchKernelGGL(spread_fold_sum, dim3(kFoldGrid), dim3(kFoldBlock), 0, s, p);
    hipLaunchKernelGGL(spread_final, dim3(spread_final_grid()), dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace qsmd
