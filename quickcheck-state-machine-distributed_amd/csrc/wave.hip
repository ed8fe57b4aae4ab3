// wave.hip -- the heavy stage: one wavefront searches one history with all
// 64 lanes and a state memo shared by the lanes in LDS (BASELINE north star
// (a)-(c)).
//
// Stages 0 / 0w search one history per lane with a node budget; the few
// histories over it (a wavefront runs as long as its slowest lane, so a long
// search would hold 63 idle lanes and the launch with them) come here.  A
// wavefront takes one heavy history at a time, stages it once into LDS
// (shared by its lanes) and searches the reference DFS tree
// (src/Linearisability.hs:52-69) with every lane:
//
//   task    a region of the tree: the candidates `cand` of the node N at
//           depth `depth`, with N's exact search state (remaining events,
//           model, path).  The root task is the whole tree.
//   split   a lane whose task has counted `budget` more nodes while other
//           lanes are idle and the pool is empty hands the rest of its task
//           to the pool: one range task per level between its base and its
//           current node (the untried candidates of that node), each with
//           the node's state, restored level by level with the DFS's own
//           exact undo.  Idle lanes take pending tasks by ballot + prefix
//           count; the deepest ranges (smallest keys) first.
//   key     a task's place in the reference's DFS order: digit i =
//           2*(j+1) for a path step through candidate event j, 2*c+1 at the
//           task's level for "candidates c, c+1, ... of this node" (keys
//           compare lexicographically, a prefix first).
//   fold    the reference stops at the first deciding node (a success, or
//           Map.! raising).  Its node count = nodes of every task whose key
//           is below the decider's + the decider's own; when nothing decides,
//           the sum of all.  Finished tasks are recorded (key, nodes) in LDS;
//           a record below every running and pending task's key can never be
//           after a future decider and is folded into a running sum.
//   cancel  a lane whose task key is above the best decider so far stops at
//           once; pending tasks above it are dropped.
//   memo    the subtree below a node depends only on its state S =
//           (remaining events, model) (SURVEY.md §8a Lemma L1), so its
//           outcome and node count are a function of S.  A subtree that a
//           lane searched to its end inside its own task (no split below it)
//           without deciding has failed; the lane records (S, count) in the
//           wavefront's LDS table, and any lane entering a node whose S is
//           recorded adds the count and treats the subtree as failed.  Keys
//           are the full state (no hash-only match), so counts, verdicts and
//           witnesses stay the reference's exactly; only the work shrinks.
//
// All scheduling is wave-synchronous (ballots, prefix counts, LDS); the only
// global atomic is the one that hands out the next heavy history.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"

namespace qsmd {

namespace {

constexpr int kPool = 64;                  // pending range tasks per wavefront
constexpr int kRec = 256;                  // task records per history
constexpr uint32_t kMemoEntries = 512;     // LDS memo entries per wavefront (power of two)
constexpr uint32_t kMemoW = 8;             // words per entry (SoA: word w of entry e at w * E + e)
constexpr uint32_t kTagValid = 0x80000000u;
constexpr uint32_t kTagClaim = 0x40000000u;

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

template <class G>
struct WaveLds {
    uint32_t hist[G::EV];                              // the history, compressed (lane.h)
    int32_t bal[QSMD_BANK_MAX_ACCOUNTS][C_LANES];      // Bank balances [account][lane]
    uint32_t entry[G::LEVELS][C_LANES];                // node count (low 32 bits) on entering a level
    Pool<G> pool;
    Recs<G> rec;
    uint8_t path[G::LEVELS];                           // the best witness path
};

__device__ __forceinline__ uint32_t wmix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    h *= 0x846CA68Bu;
    h ^= h >> 16;
    return h;
}

// The memo key of a lane's current node: tag (valid | model flags), the
// remaining events, the model (Bank: balances of the existing accounts as
// i16, absent = 0; Ticket: n).  ok = false: the state is outside the key
// encoding (a balance beyond i16) and is not memoised.
struct WKey {
    uint32_t tag, rem_lo, rem_hi, m[4], slot;
    bool ok;
};

template <uint32_t MODEL, class G>
__device__ __forceinline__ WKey wave_key(const LaneDFS<MODEL, G>& d, const SearchArgs& a,
                                         int32_t (*s_bal)[C_LANES], int lane) {
    WKey k;
    k.ok = true;
    k.rem_lo = (uint32_t)d.rem;
    k.rem_hi = G::EV == 64 ? (uint32_t)((uint64_t)d.rem >> 32) : 0u;
    if constexpr (MODEL == QSMD_MODEL_BANK) {
        const uint32_t ex = d.ex;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int32_t b0 = ((ex >> (2 * q)) & 1u) ? s_bal[2 * q][lane] : 0;
            const int32_t b1 = ((ex >> (2 * q + 1)) & 1u) ? s_bal[2 * q + 1][lane] : 0;
            k.ok = k.ok && b0 == (int32_t)(int16_t)b0 && b1 == (int32_t)(int16_t)b1;
            k.m[q] = ((uint32_t)b0 & 0xFFFFu) | ((uint32_t)b1 << 16);
        }
        k.tag = kTagValid | (ex & 0xFFu);
    } else {
        // the model after levels 0 .. depth-1 (LaneDFS::try_next's formula)
        const uint32_t just = d.RS ? 1u : a.m0_just;
        const int32_t n = d.RS ? (int32_t)(d.depth - 1u - (31u - __builtin_clz(d.RS | 1u)))
                               : (int32_t)a.m0_val[0] + (a.m0_just ? (int32_t)d.depth : 0);
        k.m[0] = just ? (uint32_t)n : 0u;
        k.m[1] = k.m[2] = k.m[3] = 0u;
        k.tag = kTagValid | just;
    }
    uint32_t h = wmix(k.rem_lo ^ 0x9E3779B9u);
    h = wmix(h ^ k.rem_hi ^ k.tag);
#pragma unroll
    for (int q = 0; q < 4; ++q) h = wmix(h ^ k.m[q]);
    k.slot = h & (kMemoEntries - 1u);
    return k;
}

__device__ __forceinline__ bool wave_lookup(const uint32_t* tab, const WKey& k, uint32_t& count) {
    const uint32_t s = k.slot;
    constexpr uint32_t E = kMemoEntries;
    const bool hit = tab[s] == k.tag && tab[E + s] == k.rem_lo && tab[2 * E + s] == k.rem_hi &&
                     tab[4 * E + s] == k.m[0] && tab[5 * E + s] == k.m[1] && tab[6 * E + s] == k.m[2] &&
                     tab[7 * E + s] == k.m[3];
    count = tab[3 * E + s];
    return hit;
}

// Lanes inserting into one slot in the same instruction: the first CAS of
// the tag word claims the slot, the others leave it (a cache entry lost, no
// result changes); the winner writes the key and count, the tag last.
__device__ __forceinline__ void wave_insert(uint32_t* tab, const WKey& k, uint32_t count, int lane) {
    const uint32_t s = k.slot;
    constexpr uint32_t E = kMemoEntries;
    const uint32_t cur = __hip_atomic_load(&tab[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    const uint32_t mine = kTagClaim | (uint32_t)lane;
    const uint32_t old = atomicCAS(&tab[s], cur, mine);
    if (old == cur) {
        tab[E + s] = k.rem_lo;
        tab[2 * E + s] = k.rem_hi;
        tab[3 * E + s] = count;
        tab[4 * E + s] = k.m[0];
        tab[5 * E + s] = k.m[1];
        tab[6 * E + s] = k.m[2];
        tab[7 * E + s] = k.m[3];
        __hip_atomic_store(&tab[s], k.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
}

// One DFS iteration of a lane (LaneDFS::step) with the memo hooks: on
// leaving a node entered inside the current task, record its subtree; on
// entering a node, reuse a recorded subtree.
template <uint32_t MODEL, class G, int MODE>
__device__ __forceinline__ int wave_step(LaneDFS<MODEL, G>& d, const SearchArgs& a, const uint32_t* hist,
                                         int32_t (*s_bal)[C_LANES], int lane, uint64_t limit, uint32_t* entry,
                                         bool& skip, uint32_t* tab, uint32_t min_rem) {
    using M = typename G::M;
    const bool empty = d.cand == (M)0;
    const bool term = empty & ((d.found == 0u) | (d.depth == d.base));
    int status = !term ? -1
                       : ((!d.found && d.depth > 0) ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_NONLINEARISABLE);
    if (empty & !term) {
        // leaving the node at depth d.depth (> base): its subtree was searched
        // to the end by this lane and failed (counts exact below 2^32)
        if (!skip && d.nodes <= 0xFFFFFFFFull && (uint32_t)__builtin_popcountll((uint64_t)d.rem) > min_rem) {
            const WKey k = wave_key<MODEL, G>(d, a, s_bal, lane);
            if (k.ok) wave_insert(tab, k, (uint32_t)d.nodes - entry[(d.depth - 1u) * C_LANES], lane);
        }
        skip = false;
        const uint32_t j = d.template undo<1, MODE>(hist, s_bal, lane);
        d.cand = cands(d.rem, d.INV, d.RESP) & mask_above(j, (M)0);
        d.found = 1u;
    }
    if (d.cand) {
        const uint32_t dep0 = d.depth;
        status = d.template try_next<1, MODE>(a, hist, s_bal, lane, limit);
        if (d.depth > dep0 && status < 0 &&
            (uint32_t)__builtin_popcountll((uint64_t)d.rem) > min_rem) {   // entered a new node (the search goes on)
            entry[dep0 * C_LANES] = (uint32_t)d.nodes;
            const WKey k = wave_key<MODEL, G>(d, a, s_bal, lane);
            uint32_t c = 0;
            if (k.ok && wave_lookup(tab, k, c)) {
                d.nodes += c;                     // the subtree's nodes, counted; it failed
                d.cand = (M)0;
                d.found = 1u;
                skip = true;
            }
        }
    }
    return status;
}

}  // namespace

template <uint32_t MODEL, int MODE, class G>
__device__ void wave_history(const WaveArgs& p, uint32_t h, const qsmd_hdr& H, const StagedT<typename G::M>& s,
                             WaveLds<G>& L, uint32_t* tab, int lane, uint64_t t0, Counters& cnt) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    using M = typename G::M;
    using K = CKey<G>;
    constexpr uint32_t JM = (uint32_t)G::EV - 1u;
    const SearchArgs& a = p.s;
    Pool<G>& pool = L.pool;
    Recs<G>& rec = L.rec;
    LaneDFS<MODEL, G> dfs;
    dfs.init(s, a, L.bal, lane);                 // every lane: masks, model0 (the root's state)
    bool busy = lane == 0;                       // lane 0 starts the root task
    bool skip = false;
    K key, best;
    key.clear(0ull);
    best.clear(~0ull);
    uint64_t limit = p.budget;
    uint32_t pool_n = 0, rec_n = 0;              // wave-uniform
    uint64_t prefix_sum = 0, explored = 0;
    uint32_t best_status = QSMD_STATUS_NONLINEARISABLE, best_depth = 0, work = 0;
    bool incomplete = false, timed = false, skipped = false, overflow = false;
    uint32_t tick = 0, n_splits = 0;
    const uint64_t c0 = p.stats ? __builtin_amdgcn_s_memtime() : 0;

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
            overflow |= __builtin_add_overflow(folded, below ? rn : 0ull, &folded);
            const uint64_t km = __ballot(keep);
            if (keep) {                          // in place, in order (kept <= i)
                const uint32_t d = kept + lane_prefix(km);
                rec.set_key(d, rk);
                rec.nodes[d] = rn;
            }
            kept += (uint32_t)__builtin_popcountll(km);
        }
        // (a sum beyond 2^64 - 1 anywhere: the giant stage reports it)
        const uint64_t f = wave_sum64(folded);
        overflow |= __ballot(f < folded) != 0ull;
        overflow |= __builtin_add_overflow(prefix_sum, f, &prefix_sum);
        overflow = __ballot(overflow) != 0ull;
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
                            for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) L.bal[q][lane] = pool.bal[q][e];
                        } else {
                            dfs.RS = mdl;
                        }
#pragma unroll
                        for (int q = 0; q < G::LEVELS / 4; ++q) dfs.stk.w[q] = pool.stk[q][e];
                        dfs.nodes = 0;
                        limit = p.budget;
                        skip = false;
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
            st = wave_step<MODEL, G, MODE>(dfs, a, L.hist, L.bal, lane, limit, &L.entry[0][lane], skip, tab,
                                           p.memo_min_rem);
            ++work;
            if (st < 0 && best.less(key)) st = QSMD_STATUS_SKIPPED;   // cancelled
        }
        if ((tick & 63u) == 0u) {
            if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                timed = true;
                if (lane == 0) atomicOr(a.timed_out, 1u);
            }
            if (beyond_first_fail(a, h)) skipped = true;
            if (p.explore_cap && explored + wave_sum64(work) > p.explore_cap) incomplete = true;
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
                    r |= ((M)1 << j) | ((M)1 << c_r<G>(L.hist[j]));
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
        if (tot && rec_n + running + pool_n + tot > (uint32_t)kRec) compact();
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
                    for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) pool.bal[q][e] = L.bal[q][lane];
                } else {
                    pool.model[e] = dfs.RS;
                }
#pragma unroll
                for (int q = 0; q < G::LEVELS / 4; ++q) pool.stk[q][e] = dfs.stk.w[q];
            };
            const M top = dfs.cand | ((M)1 << dfs.last_j);
            if (top) emit(top);
            while (dfs.depth > dfs.base) {
                const uint32_t j = dfs.template undo<1, MODE>(L.hist, L.bal, lane);
                dfs.found = 1u;
                const M c = cands(dfs.rem, dfs.INV, dfs.RESP) & mask_above(j, (M)0);
                if (c) emit(c);
            }
            split_done = true;
        } else if (at_budget) {
            dfs.cand |= (M)1 << dfs.last_j;      // search on (a memo hit may have jumped past the limit)
            limit = dfs.nodes + p.budget;
        }
        if (tot && room) {
            pool_n += tot;                       // the ranges of the lanes that split
            ++n_splits;
        }
        // ---- finished tasks: records, the best decider
        // (a BUDGET return is always a task budget: the caller's max_nodes is
        // applied by the fold)
        const bool fin = busy && (split_done || (st >= 0 && st != QSMD_STATUS_BUDGET && st != QSMD_STATUS_SKIPPED));
        const bool decided = busy && (st == QSMD_STATUS_LINEARISABLE || st == QSMD_STATUS_MODEL_ERROR);
        if (p.explore_cap && __ballot(fin)) {
            explored += wave_sum64(fin ? work : 0u);
            work = fin ? 0u : work;
        }
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
                best_status = (uint32_t)__shfl(st, w, 64);
                best_depth = (uint32_t)__shfl(dfs.depth, w, 64);
                if (me && st == QSMD_STATUS_LINEARISABLE)
                    for (uint32_t d = 0; d < dfs.depth; ++d) L.path[d] = (uint8_t)(dfs.stk.get(d, dfs.depth) & JM);
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
    } else if (incomplete || overflow) {
        status = QSMD_STATUS_HANDED_OFF;
    } else {
        uint64_t part = 0;
        bool ovf = false;
        for (uint32_t i = lane; i < rec_n; i += 64) {
            const K rk = rec.get_key(i);
            if (!best.less(rk)) ovf |= __builtin_add_overflow(part, rec.nodes[i], &part);
        }
        const uint64_t sum = wave_sum64(part);
        ovf |= __ballot(ovf || sum < part) != 0ull;
        ovf |= __builtin_add_overflow(prefix_sum, sum, &nodes);
        status = ovf ? QSMD_STATUS_HANDED_OFF : (int)best_status;
        if (!ovf && a.max_nodes && nodes > a.max_nodes) {
            status = QSMD_STATUS_BUDGET;
            nodes = a.max_nodes;
        }
    }
    if (p.stats && lane == 0) {                  // diagnostic
        unsigned long long* q = p.stats + (uint64_t)blockIdx.x * 8;
        q[0] += 1;
        q[1] += tick;
        q[2] += __builtin_amdgcn_s_memtime() - c0;
        q[3] += n_splits;
        q[4] = q[4] > tick ? q[4] : tick;
        q[7] += nodes;
    }
    if (lane == 0) {
        if (status == QSMD_STATUS_HANDED_OFF) {  // the giant stage searches it again, from the root
            a.giant_list[atomicAdd(a.giant_count, 1u)] = h;
        } else {
            note_failure(a, h, status);
            a.status[h] = (uint8_t)status;
            if (a.nodes) a.nodes[h] = nodes;
            cnt.add(status, nodes);
        }
    }
    if (status == QSMD_STATUS_LINEARISABLE && a.witness && (uint32_t)lane < H.n_ev) {
        uint8_t* w = a.witness + H.ev_off;
        if ((uint32_t)lane < best_depth) w[lane] = L.path[lane];
        else if ((uint32_t)lane == best_depth) w[lane] = QSMD_WITNESS_END;
    }
}

// One list (G32: stage 0's heavy histories; G64: stage 0w's): a wavefront
// takes one history at a time from the queue head.
template <uint32_t MODEL, class G>
__device__ __forceinline__ void wave_list(const WaveArgs& p, const uint32_t* list, const uint32_t* count_p,
                                          uint32_t* head, WaveLds<G>& L, uint32_t* tab, int lane, uint64_t t0,
                                          Counters& cnt) {
    using M = typename G::M;
    const uint32_t count = *count_p;
    if (count == 0u) return;
    uint32_t next = 0;
    if (lane == 0) next = atomicAdd(head, 1u);
    next = __shfl(next, 0, 64);
    while (next < count) {
        const uint32_t g = next;
        if (lane == 0) next = atomicAdd(head, 1u);      // prefetch the next history
        const uint32_t h = list[g];
        const qsmd_hdr H = p.s.hdr[h];
        // the history once, shared by the lanes: one event per lane
        if ((uint32_t)lane < H.n_ev) {
            const uint2 x = p.s.events[H.ev_off + lane];
            L.hist[lane] = compress<MODEL, G>(x.x, (int32_t)x.y);
        }
        // a clear memo (entries of the previous history must not match)
        for (uint32_t i = (uint32_t)lane * 4u; i < kMemoW * kMemoEntries; i += 256u)
            *reinterpret_cast<uint4*>(tab + i) = make_uint4(0u, 0u, 0u, 0u);
        __builtin_amdgcn_wave_barrier();
        StagedT<M> s{0, 0, 0, 0, 0, true, true, false};
        finish_shared<G>(L.hist, lane == 0, H.n_ev, H.n_pid, s);
        __builtin_amdgcn_wave_barrier();
        if (H.n_ev == 0u || beyond_first_fail(p.s, h)) {   // (stages 0 / 0w never send an empty one)
            const int st = H.n_ev == 0u ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_SKIPPED;
            if (lane == 0) {
                p.s.status[h] = (uint8_t)st;
                if (p.s.nodes) p.s.nodes[h] = 0;
                cnt.add(st, 0);
            }
        } else if (s.paired) {
            wave_history<MODEL, M_PAIRED, G>(p, h, H, s, L, tab, lane, t0, cnt);
        } else {
            wave_history<MODEL, M_GENERAL, G>(p, h, H, s, L, tab, lane, t0, cnt);
        }
        next = __shfl(next, 0, 64);
    }
}

template <uint32_t MODEL>
__global__ __launch_bounds__(C_LANES) void wave_search(WaveArgs p) {
    __shared__ union {
        WaveLds<G32> g32;
        WaveLds<G64> g64;
    } u;
    __shared__ __attribute__((aligned(16))) uint32_t tab[kMemoW * kMemoEntries];
    const int lane = threadIdx.x;
    const uint64_t t0 = p.s.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    Counters cnt;
    wave_list<MODEL, G32>(p, p.list32, p.count32, p.next32, u.g32, tab, lane, t0, cnt);
    wave_list<MODEL, G64>(p, p.list64, p.count64, p.next64, u.g64, tab, lane, t0, cnt);
    cnt.flush(p.s.buckets, lane);
}

hipError_t launch_wave(const WaveArgs& p, uint32_t grid, hipStream_t s) {
    if (p.s.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL(wave_search<QSMD_MODEL_BANK>, dim3(grid), dim3(C_LANES), 0, s, p);
    else
        hipLaunchKernelGGL(wave_search<QSMD_MODEL_TICKET>, dim3(grid), dim3(C_LANES), 0, s, p);
    return hipGetLastError();
}

}  // namespace qsmd
