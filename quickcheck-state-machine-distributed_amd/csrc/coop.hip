// coop.hip -- the cooperative stage: one wavefront searches one heavy
// compact history (<= 32 events, <= 8 pids) with all 64 lanes.
//
// Stage 0 searches one history per lane with a node budget; the few
// histories over it (a wavefront runs as long as its slowest lane, and one
// lane does ~1 node per us, so a 10^2..10^5-node history would hold a whole
// wavefront and the launch with it) come here.  A wavefront takes one heavy
// history at a time, stages it once into LDS (shared by its lanes) and
// searches the reference DFS tree (src/Linearisability.hs:52-69) with every
// lane:
//
//   task    a region of the tree: the candidates `cand` of the node N at
//           depth `depth`, with N's exact search state (remaining events,
//           model, path).  The root task is the whole tree.
//   split   a lane whose task has counted `budget` more nodes while other
//           lanes are idle and the pool is empty hands the rest of its task
//           to the pool: one range task per level between its base and its
//           current node (the untried candidates of that node), each with
//           the node's state, restored level by level with the DFS's own
//           exact undo.  No replay, no global memory.
//   key     a task's place in the reference's DFS order: digit i =
//           2*(j+1) for a path step through candidate event j, 2*c+1 at the
//           task's level for "candidates c, c+1, ... of this node" (keys
//           compare lexicographically, a prefix first).
//   fold    the reference stops at the first deciding node (a success, or
//           Map.! raising).  Its node count = nodes of every task whose key
//           is below the decider's + the decider's own; when nothing decides,
//           the sum of all.  Finished tasks are recorded (key, nodes) in LDS;
//           a record below every running and pending task's key can never be
//           after a future decider and is folded into a running sum, so the
//           record array stays small.
//   cancel  a lane whose task key is above the best decider so far stops at
//           once; pending tasks above it are dropped.
//
// All scheduling is wave-synchronous (ballots, prefix counts, LDS); the only
// global atomic is the one that hands out the next heavy history.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"

namespace qsmd {

namespace {

constexpr int kPool = 64;          // pending range tasks per wavefront
constexpr int kRec = 256;          // task records per history

// task key: digit i of DB bits, DPW digits per u64 word, compared
// lexicographically (G32: 16 digits of 7 bits in 2 words; G64: 32 digits of
// 8 bits in 4 words -- a path digit 2(j+1) reaches 2*EV)
template <class G>
struct CKey {
    static constexpr int NK = G::EV == 32 ? 2 : 4;
    static constexpr uint32_t DB = G::EV == 32 ? 7u : 8u;
    static constexpr uint32_t DPW = 64u / DB;
    uint64_t w[NK];
    __device__ __forceinline__ void clear(uint64_t v) {
#pragma unroll
        for (int q = 0; q < NK; ++q) w[q] = v;
    }
    __device__ __forceinline__ void put(uint32_t i, uint64_t d) {
        const uint32_t k = i / DPW, sh = 64u - DB * (i % DPW + 1u);
#pragma unroll
        for (int q = 0; q < NK; ++q)
            if ((uint32_t)q == k) w[q] |= d << sh;
    }
    __device__ __forceinline__ bool less(const CKey& b) const {
#pragma unroll
        for (int q = 0; q < NK; ++q)
            if (w[q] != b.w[q]) return w[q] < b.w[q];
        return false;
    }
    __device__ __forceinline__ bool operator==(const CKey& b) const {
        bool e = true;
#pragma unroll
        for (int q = 0; q < NK; ++q) e = e && w[q] == b.w[q];
        return e;
    }
};

// wave-wide minimum of a key (every lane gets it)
template <class K>
__device__ __forceinline__ void wave_min_key(K& k) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        K o;
#pragma unroll
        for (int q = 0; q < K::NK; ++q) o.w[q] = __shfl_xor(k.w[q], off, 64);
        if (o.less(k)) k = o;
    }
}

// exclusive prefix sum over the wavefront
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, int lane) {
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x - v;
}

template <class G>
struct Pool {              // pending range tasks (LDS)
    using M = typename G::M;
    using K = CKey<G>;
    M cand[kPool];
    uint32_t meta[kPool];  // depth | found << 8
    M rem[kPool];
    uint32_t model[kPool]; // Bank: ex | neg << 8; Ticket: RS
    uint32_t stk[G::LEVELS / 4][kPool];
    uint64_t key[K::NK][kPool];
    int32_t bal[QSMD_BANK_MAX_ACCOUNTS][kPool];
    __device__ __forceinline__ K get_key(uint32_t e) const {
        K k;
#pragma unroll
        for (int q = 0; q < K::NK; ++q) k.w[q] = key[q][e];
        return k;
    }
    __device__ __forceinline__ void set_key(uint32_t e, const K& k) {
#pragma unroll
        for (int q = 0; q < K::NK; ++q) key[q][e] = k.w[q];
    }
};

template <class G>
struct Recs {              // finished tasks of the current history (LDS)
    using K = CKey<G>;
    uint64_t key[K::NK][kRec];
    uint64_t nodes[kRec];
    __device__ __forceinline__ K get_key(uint32_t e) const {
        K k;
#pragma unroll
        for (int q = 0; q < K::NK; ++q) k.w[q] = key[q][e];
        return k;
    }
    __device__ __forceinline__ void set_key(uint32_t e, const K& k) {
#pragma unroll
        for (int q = 0; q < K::NK; ++q) key[q][e] = k.w[q];
    }
};

}  // namespace

template <uint32_t MODEL, int MODE, class G>
__device__ __forceinline__ void coop_history(const CoopArgs& p, uint32_t h, const StagedT<typename G::M>& s,
                                             uint32_t* s_hist, int32_t (*s_bal)[C_LANES], Pool<G>& pool,
                                             Recs<G>& rec, uint8_t* s_path, int lane, uint64_t t0, Counters& cnt);

// G: the geometry (G32: <= 32 events, stage 0's heavy histories; G64: <= 64
// events, stage 0w's)
template <uint32_t MODEL, class G>
__global__ __launch_bounds__(C_LANES) void coop_search(CoopArgs p) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    using M = typename G::M;
    __shared__ uint32_t s_hist[G::EV];
    __shared__ int32_t s_bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][C_LANES];
    __shared__ Pool<G> pool;
    __shared__ Recs<G> rec;
    __shared__ uint8_t s_path[G::LEVELS];
    const int lane = threadIdx.x;
    const uint64_t t0 = p.s.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t n_heavy = *p.heavy_count;
    const uint32_t count = n_heavy <= p.max_count ? n_heavy : 0u;   // auto mode: many go to spread
    Counters cnt;
    uint32_t next = ~0u;
    if (count) {
        if (lane == 0) next = atomicAdd(p.next, 1u);
        next = __shfl(next, 0, 64);
    }
    while (next < count) {
        const uint32_t g = next;
        if (lane == 0) next = atomicAdd(p.next, 1u);      // prefetch the next history
        const uint32_t h = p.heavy_list[g];
        // stage the history once (shared by the lanes): one event per lane
        const qsmd_hdr H = p.s.hdr[h];
        if ((uint32_t)lane < H.n_ev) {
            const uint2 x = p.s.events[H.ev_off + lane];
            s_hist[lane] = compress<MODEL, G>(x.x, (int32_t)x.y);
        }
        // paired?  (every lane evaluates the same history; lane 0 writes the pairs)
        StagedT<M> s{0, 0, 0, 0, 0, true, true, false};
        finish_shared<G>(s_hist, lane == 0, H.n_ev, H.n_pid, s);
        if (s.paired)
            coop_history<MODEL, M_PAIRED, G>(p, h, s, s_hist, s_bal, pool, rec, s_path, lane, t0, cnt);
        else
            coop_history<MODEL, M_GENERAL, G>(p, h, s, s_hist, s_bal, pool, rec, s_path, lane, t0, cnt);
        next = __shfl(next, 0, 64);
    }
    cnt.flush(p.s.partials, lane);
}

template <uint32_t MODEL, int MODE, class G>
__device__ __forceinline__ void coop_history(const CoopArgs& p, uint32_t h, const StagedT<typename G::M>& s,
                                             uint32_t* s_hist, int32_t (*s_bal)[C_LANES], Pool<G>& pool,
                                             Recs<G>& rec, uint8_t* s_path, int lane, uint64_t t0, Counters& cnt) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    using M = typename G::M;
    using K = CKey<G>;
    constexpr uint32_t JM = (uint32_t)G::EV - 1u;
    const SearchArgs& a = p.s;
    const qsmd_hdr H = a.hdr[h];
    LaneDFS<MODEL, G> dfs;
    dfs.init(s, a, s_bal, lane);                 // every lane: masks, model0 (the root's state)
    bool busy = lane == 0;                       // lane 0 starts the root task
    K key, best;
    key.clear(0ull);
    best.clear(~0ull);
    uint64_t limit = p.budget;
    uint32_t pool_n = 0, rec_n = 0;              // wave-uniform
    uint64_t best_nodes = 0, prefix_sum = 0, explored = 0;
    uint32_t best_status = QSMD_STATUS_NONLINEARISABLE, best_depth = 0;
    bool incomplete = false, timed = false, skipped = false;
    uint32_t tick = 0, st_splits = 0, st_nosplit = 0, st_compact = 0, st_tasks = 0;

    // record the finished task of every lane with `done` (wave-synchronous)
    auto record = [&](bool done, uint64_t nodes) {
        const uint64_t m = __ballot(done);
        if (!m) return;
        const uint32_t k = lane_prefix(m);
        if (done) {
            const uint32_t i = rec_n + k;        // room is kept for every running lane
            rec.set_key(i, key);
            rec.nodes[i] = nodes;
        }
        rec_n += (uint32_t)__builtin_popcountll(m);
    };

    // fold the records below min(every running / pending key, best decider)
    // into prefix_sum, drop the ones above the best decider
    auto compact = [&]() {
        K mk;
        if (busy) mk = key;
        else mk.clear(~0ull);
        for (uint32_t i = lane; i < pool_n; i += 64) {
            const K pk = pool.get_key(i);
            if (pk.less(mk)) mk = pk;
        }
        wave_min_key(mk);
        if (best.less(mk)) mk = best;
        uint32_t kept = 0;
        uint64_t folded = 0;
        for (uint32_t c0 = 0; c0 < rec_n; c0 += 64) {
            const uint32_t i = c0 + lane;
            const bool in = i < rec_n;
            K rk;
            rk.clear(0ull);
            uint64_t rn = 0;
            if (in) {
                rk = rec.get_key(i);
                rn = rec.nodes[i];
            }
            const bool below = in && rk.less(mk);
            const bool after = in && best.less(rk);
            const bool keep = in && !below && !after;
            folded += below ? rn : 0ull;
            const uint64_t km = __ballot(keep);
            if (keep) {                          // in place, in order (kept <= i)
                const uint32_t d = kept + lane_prefix(km);
                rec.set_key(d, rk);
                rec.nodes[d] = rn;
            }
            kept += (uint32_t)__builtin_popcountll(km);
        }
        prefix_sum += wave_sum64(folded);
        rec_n = kept;
    };

    for (;;) {
        ++tick;
        // ---- idle lanes take pending tasks (LIFO: the deepest ranges of the
        // last split, i.e. the smallest keys, first)
        {
            const uint64_t idle = __ballot(!busy);
            const uint32_t take = min((uint32_t)__builtin_popcountll(idle), pool_n);
            if (take) {
                const uint32_t k = lane_prefix(idle);
                if (!busy && k < take) {
                    const uint32_t e = pool_n - 1u - k;
                    key = pool.get_key(e);
                    if (!best.less(key)) {       // else: after the decider, dropped
                        const uint32_t meta = pool.meta[e];
                        dfs.cand = pool.cand[e];
                        dfs.depth = meta & 0xFFu;
                        dfs.base = dfs.depth;
                        dfs.found = (meta >> 8) & 1u;
                        dfs.rem = pool.rem[e];
                        const uint32_t mdl = pool.model[e];
                        if constexpr (BANK) {
                            dfs.ex = mdl & 0xFFu;
                            dfs.neg = (mdl >> 8) & 0xFFu;
#pragma unroll
                            for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) s_bal[q][lane] = pool.bal[q][e];
                        } else {
                            dfs.RS = mdl;
                        }
#pragma unroll
                        for (int q = 0; q < G::LEVELS / 4; ++q) dfs.stk.w[q] = pool.stk[q][e];
                        dfs.nodes = 0;
                        limit = p.budget;
                        busy = true;
                    }
                }
                pool_n -= take;
            }
        }
        const uint64_t busy_m = __ballot(busy);
        if (!busy_m) break;                      // nothing runs, nothing waits: done
        // ---- one DFS iteration on every busy lane
        int st = -1;
        if (busy) {
            st = dfs.template step<1, MODE>(a, s_hist, s_bal, lane, limit);
            if (st < 0 && best.less(key)) st = QSMD_STATUS_SKIPPED;   // cancelled
        }
        if ((tick & 63u) == 0u) {
            if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                timed = true;
                if (lane == 0) atomicOr(a.timed_out, 1u);
            }
            if (beyond_first_fail(a, h)) skipped = true;
            if (p.explore_cap && explored + wave_sum64(busy ? dfs.nodes : 0ull) > p.explore_cap) incomplete = true;
            if (timed || skipped || incomplete) break;
        }
        // ---- task budget reached: split when lanes are idle and nothing waits
        const bool at_budget = busy && st == QSMD_STATUS_BUDGET && dfs.nodes >= limit;
        const bool hungry = __ballot(!busy) != 0ull && pool_n == 0u;
        uint32_t k_ranges = 0;
        if (at_budget && hungry) {
            // ranges: the current node's untried candidates (+ the one the
            // budget did not count), then each ancestor level's later ones
            M r = dfs.rem;
            k_ranges = (dfs.cand | ((M)1 << dfs.last_j)) ? 1u : 0u;
            for (uint32_t l = dfs.depth; l-- > dfs.base;) {
                const uint32_t j = dfs.stk.get(l, dfs.depth) & JM;
                if (MODE == M_PAIRED) {
                    r |= ((M)1 << j) | ((M)1 << c_r<G>(s_hist[j]));
                } else {
                    const M gone = ~r & dfs.same_pid(j);
                    r |= ((M)1 << m_hibit(gone & dfs.INV)) | ((M)1 << m_hibit(gone & dfs.RESP));
                }
                k_ranges += (cands(r, dfs.INV, dfs.RESP) & mask_above(j, (M)0)) ? 1u : 0u;
            }
        }
        uint32_t off = 0, tot = 0;
        if (__ballot(k_ranges != 0u)) {
            off = wave_excl_scan(k_ranges, lane);
            tot = __shfl(off + k_ranges, 63, 64);
        }
        // room: pool entries, and a record for every task that may still
        // finish (running, pending, new)
        const uint32_t running = (uint32_t)__builtin_popcountll(busy_m);
        if (tot && rec_n + running + pool_n + tot > (uint32_t)kRec) {
            compact();
            ++st_compact;
        }
        const bool room = rec_n + running + pool_n + tot <= (uint32_t)kRec && pool_n + tot <= (uint32_t)kPool;
        bool split_done = false;
        if (at_budget && hungry && room && k_ranges) {
            // emit: entry index pool_n + off + (k_ranges - 1 - i), i = 0 at
            // the deepest level (popped first)
            uint32_t i = 0;
            auto emit = [&](M c) {
                const uint32_t e = pool_n + off + (k_ranges - 1u - i);
                ++i;
                K k;
                k.clear(0ull);
                for (uint32_t d = 0; d < dfs.depth; ++d) k.put(d, 2ull * ((dfs.stk.get(d, dfs.depth) & JM) + 1u));
                k.put(dfs.depth, 2ull * m_ctz(c) + 1ull);
                pool.set_key(e, k);
                pool.cand[e] = c;
                pool.meta[e] = dfs.depth | ((uint32_t)dfs.found << 8);
                pool.rem[e] = dfs.rem;
                if constexpr (BANK) {
                    pool.model[e] = (dfs.ex & 0xFFu) | ((dfs.neg & 0xFFu) << 8);
#pragma unroll
                    for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) pool.bal[q][e] = s_bal[q][lane];
                } else {
                    pool.model[e] = dfs.RS;
                }
#pragma unroll
                for (int q = 0; q < G::LEVELS / 4; ++q) pool.stk[q][e] = dfs.stk.w[q];
            };
            const M top = dfs.cand | ((M)1 << dfs.last_j);
            if (top) emit(top);
            while (dfs.depth > dfs.base) {
                const uint32_t j = dfs.template undo<1, MODE>(s_hist, s_bal, lane);
                dfs.found = 1u;
                const M c = cands(dfs.rem, dfs.INV, dfs.RESP) & mask_above(j, (M)0);
                if (c) emit(c);
            }
            split_done = true;
        } else if (at_budget) {
            dfs.cand |= (M)1 << dfs.last_j;      // search on
            limit += p.budget;
        }
        if (tot && room) {
            pool_n += tot;                       // the ranges of the lanes that split
            ++st_splits;
        } else if (tot) {
            ++st_nosplit;
        }
        // ---- finished tasks: records, the best decider
        // (a BUDGET return is always a task budget: the caller's max_nodes is
        // applied by the fold)
        const bool fin = busy && (split_done || (st >= 0 && st != QSMD_STATUS_BUDGET && st != QSMD_STATUS_SKIPPED));
        const bool decided = busy && (st == QSMD_STATUS_LINEARISABLE || st == QSMD_STATUS_MODEL_ERROR);
        if (p.explore_cap) explored += wave_sum64(fin ? dfs.nodes : 0ull);
        st_tasks += (uint32_t)__builtin_popcountll(__ballot(fin));
        record(fin, dfs.nodes);
        if (__ballot(decided)) {
            K dk;
            if (decided) dk = key;
            else dk.clear(~0ull);
            wave_min_key(dk);
            if (dk.less(best)) {
                best = dk;
                const bool me = decided && key == dk;
                const uint64_t mm = __ballot(me);
                const int w = __builtin_ctzll(mm);
                best_nodes = __shfl(dfs.nodes, w, 64);
                best_status = (uint32_t)__shfl(st, w, 64);
                best_depth = (uint32_t)__shfl(dfs.depth, w, 64);
                if (me && st == QSMD_STATUS_LINEARISABLE)
                    for (uint32_t d = 0; d < dfs.depth; ++d) s_path[d] = (uint8_t)(dfs.stk.get(d, dfs.depth) & JM);
            }
        }
        if (busy && (fin || st == QSMD_STATUS_SKIPPED)) busy = false;
    }

    // ---- fold: records up to the best decider
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
            const K rk = rec.get_key(i);
            if (!best.less(rk)) part += rec.nodes[i];
        }
        nodes = prefix_sum + wave_sum64(part);
        status = (int)best_status;
        if (a.max_nodes && nodes > a.max_nodes) {
            status = QSMD_STATUS_BUDGET;
            nodes = a.max_nodes;
        }
    }
    if (lane == 0) {
        if (status < 0) {
            p.redo_list[atomicAdd(p.redo_count, 1u)] = h;
        } else {
            note_failure(a, h, status);
            a.status[h] = (uint8_t)status;
            if (a.nodes) a.nodes[h] = nodes;
            if (status != QSMD_STATUS_SKIPPED) cnt.add(status, nodes);
        }
    }
    if (status == QSMD_STATUS_LINEARISABLE && a.witness && (uint32_t)lane < H.n_ev) {
        uint8_t* w = a.witness + H.ev_off;
        if ((uint32_t)lane < best_depth) w[lane] = s_path[lane];
        else if ((uint32_t)lane == best_depth) w[lane] = QSMD_WITNESS_END;
    }
    (void)best_nodes;
    if (p.stats && lane == 0) {
        unsigned long long* q = p.stats + (uint64_t)blockIdx.x * 8;
        q[0] += 1;
        q[1] += tick;
        q[2] += st_splits;
        q[3] += st_nosplit;
        q[4] += st_compact;
        q[5] += st_tasks;
        q[6] = q[6] > tick ? q[6] : tick;
        q[7] += nodes;
    }
}

hipError_t launch_coop(const CoopArgs& p, uint32_t grid, hipStream_t s) {
    if (p.s.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL((coop_search<QSMD_MODEL_BANK, G32>), dim3(grid), dim3(C_LANES), 0, s, p);
    else
        hipLaunchKernelGGL((coop_search<QSMD_MODEL_TICKET, G32>), dim3(grid), dim3(C_LANES), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_coop64(const CoopArgs& p, uint32_t grid, hipStream_t s) {
    if (p.s.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL((coop_search<QSMD_MODEL_BANK, G64>), dim3(grid), dim3(C_LANES), 0, s, p);
    else
        hipLaunchKernelGGL((coop_search<QSMD_MODEL_TICKET, G64>), dim3(grid), dim3(C_LANES), 0, s, p);
    return hipGetLastError();
}

}  // namespace qsmd
