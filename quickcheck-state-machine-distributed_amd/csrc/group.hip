// group.hip -- stage 0 with in-wavefront work sharing (the default first
// stage for histories of at most 32 events and 8 pids).
//
// compact_search (compact.hip) runs one history per lane and a wavefront
// as long as its slowest lane: in the 4x16 Bank batch the mean history needs
// 16.4 nodes but the slowest of 64 needs 26, and one group in ~3000 holds a
// history of 100..274 nodes, which alone sets the end of the launch; in the
// batch with injected bugs a group can hold a 10^4..10^5-node history.
// group_search keeps the per-lane search of compact_search and adds:
//
//   * persistent wavefronts pulling 64-history groups from a counter (the
//     next group's index is fetched while the current one is searched);
//   * sharing: once a group has >= share_idle idle lanes and a lane whose
//     search has counted >= share_nodes nodes, that lane's history becomes
//     the group's shared history: the lane hands everything it has not
//     searched to a task pool (one range task per level of its path, each
//     with the node's exact state, restored level by level with the DFS's
//     own undo) and every idle lane searches pool tasks, splitting its task
//     again (every task_budget nodes) while lanes are idle and the pool is
//     empty.  The verdict and the reference's node count come back by the
//     ordered fold of coop.hip (task keys in DFS order; records below every
//     running and pending key fold into a running sum);
//   * one shared history at a time; when it is done, the next long one.
//
// Pool and records live in a per-wavefront scratch block in global memory
// (only its own wavefront touches it), so LDS stays at compact_search's
// 10 KB and the occupancy at 4 wavefronts per SIMD.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"

namespace qsmd {

namespace {

// task key digit i (7 bits): hi holds digits 0..8, lo 9..15 (coop.hip)
__device__ __forceinline__ void gkey_put(uint64_t& hi, uint64_t& lo, uint32_t i, uint64_t d) {
    if (i < 9u) hi |= d << (56u - 7u * i);
    else lo |= d << (56u - 7u * (i - 9u));
}
__device__ __forceinline__ bool gkey_less(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah < bh || (ah == bh && al < bl);
}
__device__ __forceinline__ void gwave_min_key(uint64_t& hi, uint64_t& lo) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t oh = __shfl_xor(hi, off, 64), ol = __shfl_xor(lo, off, 64);
        if (gkey_less(oh, ol, hi, lo)) {
            hi = oh;
            lo = ol;
        }
    }
}
__device__ __forceinline__ uint32_t gwave_excl_scan(uint32_t v, int lane) {
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x - v;
}
// scratch loads bypass the CU's L1: pool slots and records are rewritten by
// other lanes of the wavefront after a lane may have cached them
template <typename T>
__device__ __forceinline__ T nc(const T* p) {
    return __builtin_nontemporal_load(p);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {   // (readfirstlane returns int: no sign extension)
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}
__device__ __forceinline__ uint32_t gwave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
    return v;
}

}  // namespace

template <uint32_t MODEL, int MODE>
__device__ __forceinline__ void group_loop(const GroupArgs& p, LaneDFS<MODEL>& dfs, bool busy, uint32_t h_own,
                                           uint32_t (*s_ev)[C_LANES], int32_t (*s_bal)[C_LANES],
                                           uint8_t* s_path, GroupScratch* sc, int lane, uint64_t t0,
                                           Counters& cnt) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    constexpr uint32_t P = GroupScratch::kPool, R = GroupScratch::kRec;
    const SearchArgs& a = p.s;
    const uint64_t user_limit = a.max_nodes ? a.max_nodes : ~0ull;
    bool own = busy;                       // searching its own history (else a shared task)
    uint32_t col = (uint32_t)lane;         // LDS column of the history searched
    uint64_t khi = 0, klo = 0, limit = user_limit;
    // the shared history (wave-uniform)
    bool sh = false;
    uint32_t sh_lane = 0, sh_h = 0, sINV = 0, sRESP = 0, sP0 = 0, sP1 = 0, sP2 = 0;
    bool s_paired = false;
    uint32_t pool_n = 0, rec_n = 0, best_status = 0, best_depth = 0;
    uint64_t best_hi = 0, best_lo = 0, prefix_sum = 0, explored = 0;
    bool timed = false, skipped = false, incomplete = false;
    uint32_t tick = 0;

    // fold the records below min(every running / pending key, best decider)
    // into prefix_sum, drop the ones above the best decider
    auto compact = [&]() {
        uint64_t mh = (busy && !own) ? khi : ~0ull, ml = (busy && !own) ? klo : ~0ull;
        for (uint32_t i = lane; i < pool_n; i += 64)
            if (gkey_less(nc(&sc->khi[i]), nc(&sc->klo[i]), mh, ml)) {
                mh = nc(&sc->khi[i]);
                ml = nc(&sc->klo[i]);
            }
        gwave_min_key(mh, ml);
        if (gkey_less(best_hi, best_lo, mh, ml)) {
            mh = best_hi;
            ml = best_lo;
        }
        uint32_t kept = 0;
        uint64_t folded = 0;
        for (uint32_t c0 = 0; c0 < rec_n; c0 += 64) {
            const uint32_t i = c0 + lane;
            const bool in = i < rec_n;
            uint64_t rh = 0, rl = 0, rn = 0;
            if (in) {
                rh = nc(&sc->rkhi[i]);
                rl = nc(&sc->rklo[i]);
                rn = nc(&sc->rnodes[i]);
            }
            const bool below = in && gkey_less(rh, rl, mh, ml);
            const bool after = in && gkey_less(best_hi, best_lo, rh, rl);
            const bool keep = in && !below && !after;
            folded += below ? rn : 0ull;
            const uint64_t km = __ballot(keep);
            if (keep) {
                const uint32_t d = kept + lane_prefix(km);
                sc->rkhi[d] = rh;
                sc->rklo[d] = rl;
                sc->rnodes[d] = rn;
            }
            kept += (uint32_t)__builtin_popcountll(km);
        }
        prefix_sum = uni64(prefix_sum + wave_sum64(folded));
        rec_n = uni(kept);
    };

    // hand the rest of this lane's search (from its current node up to its
    // base) to the pool at index first + (k - 1 - i), i = 0 deepest
    auto emit_ranges = [&](uint32_t first, uint32_t k, uint32_t extra) {
        uint32_t i = 0;
        auto emit = [&](uint32_t c) {
            const uint32_t e = first + (k - 1u - i);
            ++i;
            uint64_t hi = 0, lo = 0;
            for (uint32_t d = 0; d < dfs.depth; ++d) gkey_put(hi, lo, d, 2ull * ((dfs.stk.get(d, dfs.depth) & 31u) + 1u));
            gkey_put(hi, lo, dfs.depth, 2ull * __builtin_ctz(c) + 1ull);
            sc->khi[e] = hi;
            sc->klo[e] = lo;
            sc->cand[e] = c;
            sc->meta[e] = dfs.depth | ((uint32_t)dfs.found << 8);
            sc->rem[e] = dfs.rem;
            if constexpr (BANK) {
                sc->model[e] = (dfs.ex & 0xFFu) | ((dfs.neg & 0xFFu) << 8);
#pragma unroll
                for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) sc->bal[q][e] = s_bal[q][lane];
            } else {
                sc->model[e] = dfs.RS;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) sc->stk[q][e] = dfs.stk.w[q];
        };
        const uint32_t* evc = &s_ev[0][col];
        const uint32_t top = dfs.cand | extra;
        if (top) emit(top);
        while (dfs.depth > dfs.base) {
            const uint32_t j = dfs.template undo<C_LANES, MODE>(evc, s_bal, lane);
            dfs.found = 1u;
            const uint32_t c = cands(dfs.rem, dfs.INV, dfs.RESP) & mask_above(j, 0u);
            if (c) emit(c);
        }
    };
    // number of ranges emit_ranges would write
    auto count_ranges = [&](uint32_t extra) -> uint32_t {
        const uint32_t* evc = &s_ev[0][col];
        uint32_t r = dfs.rem, k = (dfs.cand | extra) ? 1u : 0u;
        for (uint32_t l = dfs.depth; l-- > dfs.base;) {
            const uint32_t j = dfs.stk.get(l, dfs.depth) & 31u;
            if (dfs.template is_paired<MODE>()) {
                r |= (1u << j) | (1u << c_r(evc[j * C_LANES]));
            } else {
                const uint32_t gone = ~r & dfs.same_pid(j);
                r |= (1u << (31 - __builtin_clz(gone & dfs.INV))) | (1u << (31 - __builtin_clz(gone & dfs.RESP)));
            }
            k += (cands(r, dfs.INV, dfs.RESP) & mask_above(j, 0u)) ? 1u : 0u;
        }
        return k;
    };

    for (;;) {
        ++tick;
        // ---- idle lanes take pending tasks of the shared history (LIFO)
        if (sh && pool_n) {
            const uint64_t idle = __ballot(!busy);
            const uint32_t take = min((uint32_t)__builtin_popcountll(idle), pool_n);
            if (take) {
                const uint32_t k = lane_prefix(idle);
                if (!busy && k < take) {
                    const uint32_t e = pool_n - 1u - k;
                    khi = nc(&sc->khi[e]);
                    klo = nc(&sc->klo[e]);
                    if (!gkey_less(best_hi, best_lo, khi, klo)) {     // else: after the decider
                        dfs.INV = sINV;
                        dfs.RESP = sRESP;
                        dfs.P0 = sP0;
                        dfs.P1 = sP1;
                        dfs.P2 = sP2;
                        dfs.ALL = sINV | sRESP;
                        dfs.paired = s_paired;
                        const uint32_t meta = nc(&sc->meta[e]);
                        dfs.cand = nc(&sc->cand[e]);
                        dfs.depth = meta & 0xFFu;
                        dfs.base = dfs.depth;
                        dfs.found = (meta >> 8) & 1u;
                        dfs.rem = nc(&sc->rem[e]);
                        const uint32_t mdl = nc(&sc->model[e]);
                        if constexpr (BANK) {
                            dfs.ex = mdl & 0xFFu;
                            dfs.neg = (mdl >> 8) & 0xFFu;
#pragma unroll
                            for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) s_bal[q][lane] = nc(&sc->bal[q][e]);
                        } else {
                            dfs.RS = mdl;
                        }
#pragma unroll
                        for (int q = 0; q < 4; ++q) dfs.stk.w[q] = nc(&sc->stk[q][e]);
                        dfs.nodes = 0;
                        limit = p.task_budget;
                        col = sh_lane;
                        busy = true;
                    }
                }
                pool_n -= take;
            }
        }
        // ---- the shared history is done: fold, result
        if (sh && pool_n == 0u && __ballot(busy && !own) == 0ull) {
            int status;
            uint64_t nodes = 0;
            if (skipped) {
                status = QSMD_STATUS_SKIPPED;
            } else if (timed) {
                status = QSMD_STATUS_BUDGET;
                nodes = a.max_nodes;
            } else if (incomplete) {
                status = -1;
            } else {
                uint64_t part = 0;
                for (uint32_t i = lane; i < rec_n; i += 64) {
                    const uint64_t rh = nc(&sc->rkhi[i]), rl = nc(&sc->rklo[i]);
                    if (gkey_less(rh, rl, best_hi, best_lo) || (rh == best_hi && rl == best_lo)) part += nc(&sc->rnodes[i]);
                }
                nodes = uni64(prefix_sum + wave_sum64(part));
                status = (int)best_status;
                if (a.max_nodes && nodes > a.max_nodes) {
                    status = QSMD_STATUS_BUDGET;
                    nodes = a.max_nodes;
                }
            }
            if (lane == 0) {
                if (status < 0) {
                    p.redo_list[atomicAdd(p.redo_count, 1u)] = sh_h;
                } else {
                    note_failure(a, sh_h, status);
                    a.status[sh_h] = (uint8_t)status;
                    if (a.nodes) a.nodes[sh_h] = nodes;
                    cnt.add(status, nodes);
                }
            }
            if (status == QSMD_STATUS_LINEARISABLE && a.witness) {
                const qsmd_hdr H = a.hdr[sh_h];
                if ((uint32_t)lane < H.n_ev) {
                    uint8_t* w = a.witness + H.ev_off;
                    if ((uint32_t)lane < best_depth) w[lane] = s_path[lane];
                    else if ((uint32_t)lane == best_depth) w[lane] = QSMD_WITNESS_END;
                }
            }
            if (p.stats && lane == 0) {
                unsigned long long* q = p.stats + (uint64_t)blockIdx.x * 8;
                q[0] += 1;
                q[1] += nodes;
            }
            sh = false;
        }
        const uint64_t busy_m = __ballot(busy);
        if (!busy_m) break;

        // ---- one DFS iteration on every busy lane
        int st = -1;
        if (busy) {
            st = dfs.template step<C_LANES, MODE>(a, &s_ev[0][col], s_bal, lane, limit);
            if (!own && st < 0 && gkey_less(best_hi, best_lo, khi, klo)) st = QSMD_STATUS_SKIPPED;   // cancelled
        }
        if ((tick & 1023u) == 0u) {      // early exit / time limit (own searches)
            if (busy && own && st < 0) {
                if (beyond_first_fail(a, h_own)) {
                    st = QSMD_STATUS_SKIPPED;
                } else if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                    atomicOr(a.timed_out, 1u);
                    st = QSMD_STATUS_BUDGET;
                }
            }
        }
        // ---- own search finished: its result
        if (busy && own && st >= 0) {
            note_failure(a, h_own, st);
            a.status[h_own] = (uint8_t)st;
            if (a.nodes) a.nodes[h_own] = dfs.nodes;
            if (a.witness && st == QSMD_STATUS_LINEARISABLE) {
                const qsmd_hdr H = a.hdr[h_own];
                dfs.write_witness(a.witness + H.ev_off, H.n_ev);
            }
            cnt.add(st, dfs.nodes);
            busy = false;
            own = false;
        }
        // ---- shared tasks: budget / split, records, the best decider
        if (sh) {
            if ((tick & 63u) == 0u) {
                if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                    timed = true;
                    if (lane == 0) atomicOr(a.timed_out, 1u);
                }
                if (beyond_first_fail(a, sh_h)) skipped = true;
                if (p.explore_cap && explored + wave_sum64((busy && !own) ? dfs.nodes : 0ull) > p.explore_cap)
                    incomplete = true;
                if (timed || skipped || incomplete) {     // stop the shared history's tasks
                    if (busy && !own) {
                        busy = false;
                        st = -1;
                    }
                    pool_n = 0;
                }
            }
            const bool mine = busy && !own;
            const bool at_budget = mine && st == QSMD_STATUS_BUDGET && dfs.nodes >= limit;
            const bool hungry = __ballot(!busy) != 0ull && pool_n == 0u;
            uint32_t k_ranges = 0;
            if (at_budget && hungry) k_ranges = count_ranges(1u << dfs.last_j);
            uint32_t off = 0, tot = 0;
            if (__ballot(k_ranges != 0u)) {
                off = gwave_excl_scan(k_ranges, lane);
                tot = uni((uint32_t)__shfl((int)(off + k_ranges), 63, 64));
            }
            const uint32_t running = (uint32_t)__builtin_popcountll(__ballot(mine));
            if (tot && rec_n + running + pool_n + tot > R) compact();
            const bool room = rec_n + running + pool_n + tot <= R && pool_n + tot <= P;
            bool split_done = false;
            if (at_budget && hungry && room && k_ranges) {
                emit_ranges(pool_n + off, k_ranges, 1u << dfs.last_j);
                split_done = true;
            } else if (at_budget) {
                dfs.cand |= 1u << dfs.last_j;    // search on
                limit += p.task_budget;
            }
            if (tot && room) pool_n = uni(pool_n + tot);
            const bool fin = mine && (split_done || (st >= 0 && st != QSMD_STATUS_BUDGET && st != QSMD_STATUS_SKIPPED));
            const bool decided = mine && (st == QSMD_STATUS_LINEARISABLE || st == QSMD_STATUS_MODEL_ERROR);
            if (p.explore_cap) explored = uni64(explored + wave_sum64(fin ? dfs.nodes : 0ull));
            const uint64_t fm = __ballot(fin);
            if (fm) {                            // records (room is kept for every task)
                if (fin) {
                    const uint32_t i = rec_n + lane_prefix(fm);
                    sc->rkhi[i] = khi;
                    sc->rklo[i] = klo;
                    sc->rnodes[i] = dfs.nodes;
                }
                rec_n = uni(rec_n + (uint32_t)__builtin_popcountll(fm));
            }
            if (__ballot(decided)) {
                uint64_t dh = decided ? khi : ~0ull, dl = decided ? klo : ~0ull;
                gwave_min_key(dh, dl);
                dh = uni64(dh);
                dl = uni64(dl);
                if (p.debug && lane == 0) {
                    unsigned long long* dbg = p.debug + (uint64_t)blockIdx.x * 256;
                    const uint32_t c = (uint32_t)dbg[200];
                    if (c < 20) {
                        dbg[201 + c * 2] = dh;
                        dbg[202 + c * 2] = dl;
                        dbg[200] = c + 1;
                    }
                }
                if (gkey_less(dh, dl, best_hi, best_lo)) {
                    best_hi = dh;
                    best_lo = dl;
                    const bool me = decided && khi == dh && klo == dl;
                    const int w = __builtin_ctzll(__ballot(me));
                    best_status = uni((uint32_t)__shfl(st, w, 64));
                    best_depth = uni((uint32_t)__shfl((int)dfs.depth, w, 64));
                    if (me && st == QSMD_STATUS_LINEARISABLE)
                        for (uint32_t d = 0; d < dfs.depth; ++d) s_path[d] = (uint8_t)(dfs.stk.get(d, dfs.depth) & 31u);
                }
            }
            if (mine && (fin || st == QSMD_STATUS_SKIPPED)) busy = false;
        }
        // ---- start sharing: a long own search while lanes are idle
        if (!sh && __builtin_popcountll(__ballot(!busy)) >= p.share_idle) {
            // (not at a node whose candidates are used up: its next step
            // decides a leaf's success or backtracks, which a range cannot carry)
            const bool cand_v = busy && own && dfs.nodes >= p.share_nodes && dfs.cand != 0u;
            if (__ballot(cand_v)) {
                const uint32_t key = cand_v ? (min((uint32_t)dfs.nodes, 0x3FFFFFFu) << 6) | (uint32_t)lane : 0u;
                const int v = (int)uni(gwave_max_u32(key) & 63u);
                sh_lane = (uint32_t)v;
                sh_h = uni((uint32_t)__shfl((int)h_own, v, 64));
                sINV = uni((uint32_t)__shfl((int)dfs.INV, v, 64));
                sRESP = uni((uint32_t)__shfl((int)dfs.RESP, v, 64));
                sP0 = uni((uint32_t)__shfl((int)dfs.P0, v, 64));
                sP1 = uni((uint32_t)__shfl((int)dfs.P1, v, 64));
                sP2 = uni((uint32_t)__shfl((int)dfs.P2, v, 64));
                s_paired = uni((uint32_t)__shfl((int)dfs.paired, v, 64)) != 0u;
                best_hi = best_lo = ~0ull;
                best_status = QSMD_STATUS_NONLINEARISABLE;
                best_depth = 0;
                prefix_sum = 0;
                timed = skipped = incomplete = false;
                uint32_t k = 0;
                if (lane == v) {
                    // the victim's search so far is the root task's record
                    // (key 0); the rest goes to the pool
                    k = count_ranges(0u);
                    sc->rkhi[0] = 0;
                    sc->rklo[0] = 0;
                    sc->rnodes[0] = dfs.nodes;
                    if (p.debug) {
                        unsigned long long* dbg = p.debug + (uint64_t)blockIdx.x * 256;
                        dbg[0] = dfs.nodes;
                        dbg[1] = dfs.depth | ((uint64_t)dfs.found << 8) | ((uint64_t)k << 16) | ((uint64_t)dfs.cand << 32);
                        dbg[2] = dfs.rem | ((uint64_t)dfs.paired << 32);
                        for (int q = 0; q < 4; ++q) dbg[3 + q] = dfs.stk.w[q];
                    }
                    emit_ranges(0u, k, 0u);
                    if (p.debug) {
                        unsigned long long* dbg = p.debug + (uint64_t)blockIdx.x * 256;
                        for (uint32_t e = 0; e < k && e < 20; ++e) {
                            dbg[8 + e * 4] = sc->khi[e];
                            dbg[9 + e * 4] = sc->klo[e];
                            dbg[10 + e * 4] = sc->cand[e] | ((uint64_t)sc->meta[e] << 32);
                            dbg[11 + e * 4] = sc->rem[e];
                        }
                    }
                    busy = false;
                    own = false;
                }
                explored = uni64(__shfl(dfs.nodes, v, 64));
                pool_n = uni((uint32_t)__shfl((int)k, v, 64));
                rec_n = 1;
                sh = true;
                if (p.stats && lane == 0) p.stats[(uint64_t)blockIdx.x * 8 + 2] += 1;
            }
        }
    }
}

template <uint32_t MODEL>
__global__ __launch_bounds__(C_LANES) void group_search(GroupArgs p) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    __shared__ uint32_t s_ev[C_MAXEV][C_LANES];
    __shared__ int32_t s_bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][C_LANES];
    __shared__ uint8_t s_path[16];
    const SearchArgs& a = p.s;
    const int lane = threadIdx.x;
    GroupScratch* sc = p.scratch + blockIdx.x;
    const uint64_t total = a.n_hist;
    const uint32_t n_groups = (uint32_t)((total + C_LANES - 1) / C_LANES);
    Counters cnt;
    const uint64_t t0 = a.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    // group order: this block's first group, then the counter (fetched ahead)
    uint32_t g = blockIdx.x, next = 0;
    if (lane == 0) next = atomicAdd(p.group_next, 1u) + gridDim.x;
    while (g < n_groups) {
        const uint64_t idx = (uint64_t)g * C_LANES + lane;
        const bool active = idx < total;
        const uint32_t h = (uint32_t)idx;
        qsmd_hdr H;
        if (active) H = a.hdr[h];
        else H = qsmd_hdr{0, 0, 0, 0, 0, 0};
        const uint32_t n_ev = H.n_ev, n_pid = H.n_pid;
        const bool enc_ok = active && H.model_id == MODEL && n_ev <= QSMD_MAX_EVENTS &&
                            n_pid <= QSMD_MAX_PIDS && (uint64_t)H.ev_off + n_ev <= a.n_events;
        const bool small = enc_ok && n_ev <= (uint32_t)C_MAXEV && n_pid <= 8u && a.m0_small;

        Staged s{0u, 0u, 0u, 0u, 0u, true, true, false};
        const uint32_t N0 = __builtin_amdgcn_readfirstlane(n_ev);
        const uint32_t off0 = __builtin_amdgcn_readfirstlane(H.ev_off);
        const bool lane_uni = active && small && n_ev == N0 && H.ev_off == off0 + (uint32_t)lane * N0;
        const bool packed = __ballot(!lane_uni) == 0ull && N0 > 0u;
        if (packed) stage_packed<MODEL>(a, N0, off0, s_ev, lane);
        else if (small) stage_lane<MODEL>(a, H, s_ev, lane);
        if (small) finish_lane(s_ev, lane, n_ev, n_pid, s);
        s.ok = s.ok && enc_ok;
        const bool defer = enc_ok && (!small || (s.ok && !s.fits));
        wave_append(defer, h, a.defer_list, a.defer_count, lane);   // -> stage 1

        LaneDFS<MODEL> dfs;
        dfs.depth = 0;
        dfs.nodes = 0;
        bool search = false;
        if (active && !defer) {
            int status = -1;
            if (!s.ok) status = QSMD_STATUS_ENCODE_ERROR;
            else if (n_ev == 0) status = QSMD_STATUS_LINEARISABLE;   // :59
            else if (beyond_first_fail(a, h)) status = QSMD_STATUS_SKIPPED;
            else search = true;
            if (!search) {
                a.status[h] = (uint8_t)status;
                if (a.nodes) a.nodes[h] = 0;
                cnt.add(status, 0);
            }
        }
        if (search) dfs.init(s, a, s_bal, lane);
        // one loop, the pairing mode is a per-lane flag (uniform in practice)
        group_loop<MODEL, M_LANE>(p, dfs, search, h, s_ev, s_bal, s_path, sc, lane, t0, cnt);
        g = (uint32_t)__shfl((int)next, 0, 64);
        if (lane == 0 && g < n_groups) next = atomicAdd(p.group_next, 1u) + gridDim.x;
    }
    cnt.flush(a.partials, lane);
}

hipError_t launch_group(const GroupArgs& p, uint32_t grid, hipStream_t s) {
    if (p.s.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL(group_search<QSMD_MODEL_BANK>, dim3(grid), dim3(C_LANES), 0, s, p);
    else
        hipLaunchKernelGGL(group_search<QSMD_MODEL_TICKET>, dim3(grid), dim3(C_LANES), 0, s, p);
    return hipGetLastError();
}

}  // namespace qsmd
