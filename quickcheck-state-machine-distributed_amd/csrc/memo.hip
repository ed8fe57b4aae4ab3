// memo.hip -- the memo stage: per-lane search with an exact-count state memo
// (north star (c)), for the histories the compact stages stop at their node
// budget.
//
// The reference (src/Linearisability.hs:52-69) evaluates a subtree
// `any' (step model') (interleavings es')` that depends only on the state
// S = (remaining events es', model') (Lemma L1).  Its outcome and its node
// count are therefore a function of S.  The search stops at the first
// success (any / && short-circuit up to the root) or the first Map.! error,
// so any subtree that is searched to its end before the search ends has
// failed; a later visit to the same S (another interleaving of the same
// operations reaching the same model) would fail again after counting the
// same nodes.  The memo stage records, on leaving such a subtree, (S, its
// node count) and, on entering a state it holds, adds the count and treats
// the subtree as failed without searching it.  Verdicts, node counts and
// witnesses stay the reference's exactly (a witness path never passes a
// failed subtree); only the work changes: 10^4-node Bank histories with
// injected bugs take ~10^2 explored nodes.
//
// Table: one private table per lane (the lane's slot in the grid), T
// direct-mapped entries in HBM, keyed by the history index and the call's
// epoch (stale entries never match, nothing is cleared per call) and the
// full state: remaining-event mask and model (Bank: existing accounts and
// their balances as i16; Ticket: Just n).  A state outside that encoding
// (a balance beyond i16, a count beyond u32) is simply not recorded.  One
// writer and reader per table: plain loads and stores, no atomics.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"


namespace qsmd {

namespace {

// entry: G32 8 x u32 (32 B), G64 16 x u32 (64 B)
//   [0] history index  [1] epoch (24 bits) | ex << 24   [2] rem (lo)  [3] count
//   [4..7] model: Bank 8 x i16 balances (existing accounts, else 0);
//          Ticket [4] = just | n << 1
//   G64: [8] rem (hi)
template <class G>
struct MemoEntry {
    static constexpr int W = G::EV == 32 ? 8 : 16;
};

template <uint32_t MODEL, class G>
struct LaneKey {
    uint32_t w1, rem_lo, rem_hi, m[4];
    uint32_t slot;
};

// The memo's slot hash: slot = the top log2(entries) bits of one
// multiplicative hash (they see every input bit): product >> sh,
// sh = 32 - log2(entries) (entries >= 2).
struct SlotHash {
    uint32_t sh;
};

// Whether every state a search of this call can reach has a memo key: the
// key holds balances (Bank) or the counter (Ticket) as i16, and a compact
// history of at most G::LEVELS operations with values of 9 bits (c_ival)
// moves an account by at most 256 per operation, so a model0 within
// +-(32767 - 256 LEVELS) keeps every reachable state in range.  Checked once
// per call (wave-uniform) instead of per node; a call outside it runs the
// memo stage without the memo (exact either way).
template <uint32_t MODEL, class G>
__device__ __forceinline__ bool keys_fit(const SearchArgs& a) {
    constexpr int64_t lim = 32767 - 256 * G::LEVELS;
    bool ok = true;
    if constexpr (MODEL == QSMD_MODEL_BANK) {
#pragma unroll
        for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q)
            ok = ok && (!((a.m0_exists >> q) & 1u) || (a.m0_val[q] >= -lim && a.m0_val[q] <= lim));
    } else {
        ok = !a.m0_just || (a.m0_val[0] >= -lim && a.m0_val[0] <= lim);
    }
    return ok;
}

// The key of the lane's current state (the node at depth dfs.depth) in two
// parts: the model's raw words (Bank: the eight balances, read from LDS; an
// absent account holds 0 there -- LaneDFS: created from 0, restored to 0 by
// undo -- so they are read unconditionally), then the key and its slot.
// The caller has checked keys_fit.
template <uint32_t MODEL>
struct KeyRaw {
    uint32_t b[MODEL == QSMD_MODEL_BANK ? QSMD_BANK_MAX_ACCOUNTS : 1];
};

template <uint32_t MODEL, class G>
__device__ __forceinline__ KeyRaw<MODEL> memo_key_raw(int32_t (*s_bal)[C_LANES], int lane) {
    KeyRaw<MODEL> r;
    if constexpr (MODEL == QSMD_MODEL_BANK) {
#pragma unroll
        for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) r.b[q] = (uint32_t)s_bal[q][lane];
    } else {
        r.b[0] = 0u;
    }
    return r;
}

// Bank: LaneDFS::fold of the raw balances (the XOR over accounts q of
// balance q rotated right by 4q; undo / try_next keep it from here on)
template <uint32_t MODEL>
__device__ __forceinline__ uint32_t fold_of(const KeyRaw<MODEL>& r) {
    uint32_t f = 0u;
    if constexpr (MODEL == QSMD_MODEL_BANK) {
#pragma unroll
        for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) f ^= __builtin_amdgcn_alignbit(r.b[q], r.b[q], 4u * q);
    }
    return f;
}

// The Ticket model's key word: the model after the levels 0 .. depth-1 (the
// formula of LaneDFS::try_next), just | n << 1
template <uint32_t MODEL>
__device__ __forceinline__ uint32_t ticket_word(uint32_t RS, uint32_t depth, const SearchArgs& a) {
    const uint32_t just = RS ? 1u : a.m0_just;
    const int32_t n = RS ? (int32_t)(depth - 1u - (31u - __builtin_clz(RS | 1u)))
                         : (int32_t)a.m0_val[0] + (a.m0_just ? (int32_t)depth : 0);
    return just | (just ? ((uint32_t)n & 0xFFFFu) << 1 : 0u);
}

// The slot of a state from registers: the model's word (Bank: the balances'
// fold and the existing accounts; Ticket: the key word) rotated into the
// remaining set, then one multiplicative hash (one quarter-rate multiply)
template <uint32_t MODEL, class G>
__device__ __forceinline__ uint32_t memo_slot(uint32_t fold, typename G::M rem, uint32_t ex, uint32_t RS,
                                              uint32_t depth, const SearchArgs& a, SlotHash sh) {
    const uint32_t v = MODEL == QSMD_MODEL_BANK ? fold ^ ex : ticket_word<MODEL>(RS, depth, a);
    uint32_t t = (uint32_t)rem ^ __builtin_amdgcn_alignbit(v, v, 13);
    if constexpr (G::EV == 64) {
        const uint32_t hi = (uint32_t)((uint64_t)rem >> 32);
        t ^= __builtin_amdgcn_alignbit(hi, hi, 7);
    }
    return (t * 0x9E3779B1u) >> sh.sh;
}

template <uint32_t MODEL, class G>
__device__ __forceinline__ LaneKey<MODEL, G> memo_key_of(const KeyRaw<MODEL>& r, uint32_t fold, typename G::M rem,
                                                         uint32_t ex, uint32_t RS, uint32_t depth,
                                                         const SearchArgs& a, uint32_t epoch, SlotHash sh) {
    LaneKey<MODEL, G> k;
    k.rem_lo = (uint32_t)rem;
    k.rem_hi = G::EV == 64 ? (uint32_t)((uint64_t)rem >> 32) : 0u;
    if constexpr (MODEL == QSMD_MODEL_BANK) {
        // two i16 halves per word by one v_perm
#pragma unroll
        for (int q = 0; q < 4; ++q) k.m[q] = __builtin_amdgcn_perm(r.b[2 * q + 1], r.b[2 * q], 0x05040100u);
    } else {
        ex = 0u;
        k.m[0] = ticket_word<MODEL>(RS, depth, a);
        k.m[1] = k.m[2] = k.m[3] = 0u;
    }
    k.w1 = (epoch & 0xFFFFFFu) | (ex << 24);
    k.slot = memo_slot<MODEL, G>(fold, rem, ex, RS, depth, a, sh);
    return k;
}

template <uint32_t MODEL, class G>
__device__ __forceinline__ LaneKey<MODEL, G> memo_key(const LaneDFS<MODEL, G>& d, const SearchArgs& a,
                                                      int32_t (*s_bal)[C_LANES], int lane, uint32_t epoch,
                                                      SlotHash sh) {
    return memo_key_of<MODEL, G>(memo_key_raw<MODEL, G>(s_bal, lane), d.fold, d.rem, d.ex, d.RS, d.depth, a, epoch,
                                 sh);
}

template <uint32_t MODEL, class G>
__device__ __forceinline__ bool memo_lookup(const uint32_t* tab, const LaneKey<MODEL, G>& k, uint32_t h,
                                            uint32_t& count) {
    // the whole entry in one round trip: both 16-B loads issued before any
    // compare (with && the compiler loaded word 0, compared, then the rest,
    // then the count -- two or three dependent HBM round trips per probe)
    const uint4* e = reinterpret_cast<const uint4*>(tab + (uint64_t)k.slot * MemoEntry<G>::W);
    uint4 x0 = e[0], x1 = e[1];
    asm volatile("" : "+v"(x0.x), "+v"(x0.y), "+v"(x0.z), "+v"(x0.w), "+v"(x1.x), "+v"(x1.y), "+v"(x1.z),
                 "+v"(x1.w));
    bool hit = (x0.x == h) & (x0.y == k.w1) & (x0.z == k.rem_lo) & (x1.x == k.m[0]) & (x1.y == k.m[1]) &
               (x1.z == k.m[2]) & (x1.w == k.m[3]);
    if constexpr (G::EV == 64) hit = hit & (e[2].x == k.rem_hi);
    count = x0.w;
    return hit;
}

template <uint32_t MODEL, class G>
__device__ __forceinline__ void memo_insert(uint32_t* tab, const LaneKey<MODEL, G>& k, uint32_t h, uint32_t count) {
    uint4* e = reinterpret_cast<uint4*>(tab + (uint64_t)k.slot * MemoEntry<G>::W);
    e[0] = make_uint4(h, k.w1, k.rem_lo, count);
    e[1] = make_uint4(k.m[0], k.m[1], k.m[2], k.m[3]);
    if constexpr (G::EV == 64) e[2] = make_uint4(k.rem_hi, 0u, 0u, 0u);
}

// The LDS table (G32, a short heavy list): lds_entries (<= 64) direct-mapped entries
// per lane, word w of entry e at col[(e * 8 + w) * 64] (each lane its own
// bank); an LDS probe instead of an HBM round trip per node.  128 KB per
// workgroup: one wavefront per CU, chosen only when the heavy groups fit
// the CUs (api.hip); fewer entries per lane (knob memo_lds_entries) leave
// the CU's LDS to other work.  Word 0 holds the history index; kNoHistory = empty.
constexpr uint32_t kNoHistory = 0xFFFFFFFFu;
// an entry count never recorded (a level entered by stage 0 before a resume)
constexpr uint32_t kNoEntry = 0xFFFFFFFFu;

template <uint32_t MODEL, class G>
__device__ __forceinline__ bool memo_lookup_lds(const uint32_t* col, const LaneKey<MODEL, G>& k, uint32_t h,
                                                uint32_t& count) {
    // every word read before any compare (one LDS round trip, see memo_lookup)
    const uint32_t* e = col + k.slot * 8u * C_LANES;
    bool hit = (e[0] == h) & (e[1 * C_LANES] == k.w1) & (e[2 * C_LANES] == k.rem_lo) & (e[4 * C_LANES] == k.m[0]);
    if constexpr (MODEL == QSMD_MODEL_BANK)
        hit = hit & (e[5 * C_LANES] == k.m[1]) & (e[6 * C_LANES] == k.m[2]) & (e[7 * C_LANES] == k.m[3]);
    count = e[3 * C_LANES];
    return hit;
}

template <uint32_t MODEL, class G>
__device__ __forceinline__ void memo_insert_lds(uint32_t* col, const LaneKey<MODEL, G>& k, uint32_t h, uint32_t count) {
    uint32_t* e = col + k.slot * 8u * C_LANES;
    e[0] = h;
    e[1 * C_LANES] = k.w1;
    e[2 * C_LANES] = k.rem_lo;
    e[3 * C_LANES] = count;
    e[4 * C_LANES] = k.m[0];
    if constexpr (MODEL == QSMD_MODEL_BANK) {
        e[5 * C_LANES] = k.m[1];
        e[6 * C_LANES] = k.m[2];
        e[7 * C_LANES] = k.m[3];
    }
}

// The slots this lane has written for its current history, as 64 bits
// (slot & 63: a set bit means "maybe written").  An entry can only match
// when the lane wrote it for this history in this call (the key holds the
// history index and the call's epoch), so a probe of a clear bit is a miss
// without the HBM round trip -- most probes: a heavy search finds ~1 % of
// its states in the table.
struct Written {
    uint64_t m;
    __device__ __forceinline__ void clear() { m = 0ull; }
    __device__ __forceinline__ void set(uint32_t slot) { m |= 1ull << (slot & 63u); }
    __device__ __forceinline__ bool maybe(uint32_t slot) const { return (m >> (slot & 63u)) & 1ull; }
};

// Diagnostic (ST) records per group: kMemoStatsWords u64 (tools/memo_stats.py).
//   [0..2] realtime at start / staged / end  [3] max DFS iterations over the
//   lanes  [4] their sum  [5] memo hits  [6] histories  [7] shader cycles of
//   the search loop (max over the lanes)
//   [8..11] shader cycles the wavefront spent in the iteration's phases, each
//   drained of its memory operations before its end stamp (so latency lands
//   in the phase that issued it): [8] backtrack (entry count, memo count,
//   undo) [9] try_next [10] memo slot [11] HBM probe (the key's balances and
//   the entry)  [12] wave iterations in which some lane's LaneDFS::fold
//   differs from its balances' (a consistency check: 0)
//   [13] wave iterations with a backtrack [14] with an HBM probe [15] wave
//   iterations
constexpr uint32_t kMemoStatsWords = 16;

// One wavefront per workgroup: phase clocks in LDS, added by one lane
// (the first active one of the block that stamps).
struct PhaseClock {
    uint64_t acc[8];
    __device__ __forceinline__ uint64_t start() {
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t t = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        return t;
    }
    __device__ __forceinline__ void stop(int k, uint64_t t0, int lane) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0);
        const uint64_t t = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        if (lane == (int)__builtin_ctzll(__ballot(1))) acc[k] += t - t0;
    }
    __device__ __forceinline__ void count(int k, bool any, int lane) {
        if (lane == (int)__builtin_ctzll(__ballot(1)) && any) acc[k] += 1;
    }
};

// One DFS iteration with the memo (LaneDFS::step plus the two hooks).
// entry: the lane's column of node counts at entry, per level; tab: the
// lane's HBM table, or (LT) its LDS column.  keyed: every reachable state
// has a key (keys_fit), so a failed subtree is recorded from the heavy
// stage's start; memo (the search has counted memo_after nodes): probes.
template <uint32_t MODEL, class G, bool LT, bool ST>
__device__ __forceinline__ int memo_step(LaneDFS<MODEL, G>& d, const SearchArgs& a, const uint32_t* evc,
                                         int32_t (*s_bal)[C_LANES], int lane, uint64_t limit, uint32_t* tab,
                                         uint32_t h, uint32_t epoch, SlotHash sh, uint32_t* entry, bool& skip,
                                         bool keyed, uint64_t memo_after, Written& wr, PhaseClock* ph) {
    using M = typename G::M;
    // a short search runs as the plain DFS (no HBM probe per node); the memo
    // joins once the search has counted memo_after nodes.  Failed subtrees
    // are recorded from the start (entry counts are kept from the start): a
    // node that fails before the memo joins is found by the probes after.
    const bool memo = keyed & (d.nodes >= memo_after);
    const bool empty = d.cand == (M)0;
    const bool term = empty & ((d.found == 0u) | (d.depth == d.base));
    int status = !term ? -1
                       : ((!d.found && d.depth > 0) ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_NONLINEARISABLE);
    uint64_t t0 = 0;
    if constexpr (ST) {
        ph->count(5, __ballot(empty & !term) != 0ull, lane);
        ph->count(7, true, lane);
    }
    if (empty & !term) {
        if constexpr (ST) t0 = ph->start();
        // leaving the node at depth d.depth: its subtree was searched to the
        // end and failed (counts kept mod 2^32: exact while the running count
        // is below 2^32).  The key (the node's balances, before the undo),
        // the level's entry count and the undo's first read are issued
        // together: one LDS round trip instead of three in a row
        uint32_t ent = entry[(d.depth - 1u) * C_LANES];
        KeyRaw<MODEL> raw = memo_key_raw<MODEL, G>(s_bal, lane);
        const M rem0 = d.rem;
        const uint32_t ex0 = d.ex, RS0 = d.RS, dep0 = d.depth, fold0 = d.fold;
        const uint32_t j = d.template undo<C_LANES, true>(evc, s_bal, lane);
        // (the key's reads complete here, not sunk into the branch below: the
        // compiler issues them beside the undo's)
        if constexpr (MODEL == QSMD_MODEL_BANK)
            asm volatile("" : "+v"(ent), "+v"(raw.b[0]), "+v"(raw.b[1]), "+v"(raw.b[2]), "+v"(raw.b[3]),
                         "+v"(raw.b[4]), "+v"(raw.b[5]), "+v"(raw.b[6]), "+v"(raw.b[7]));
        const bool rec = keyed & !skip & (d.nodes <= 0xFFFFFFFFull) & (ent != kNoEntry);
        const uint32_t cnt = (uint32_t)d.nodes - ent;
        skip = false;
        d.cand = cands(d.rem, d.INV, d.RESP) & mask_above(j, (M)0);
        d.found = 1u;
        if (rec) {
            const LaneKey<MODEL, G> k = memo_key_of<MODEL, G>(raw, fold0, rem0, ex0, RS0, dep0, a, epoch, sh);
            if constexpr (LT) {
                memo_insert_lds<MODEL, G>(tab, k, h, cnt);
            } else {
                memo_insert<MODEL, G>(tab, k, h, cnt);
                wr.set(k.slot);
            }
        }
        if constexpr (ST) ph->stop(0, t0, lane);
    }
    if (d.cand) {
        const uint32_t dep0 = d.depth;
        if constexpr (ST) t0 = ph->start();
        status = d.template try_next<C_LANES, true>(a, evc, s_bal, lane, limit);
        if constexpr (ST) {
            ph->stop(1, t0, lane);
            if constexpr (MODEL == QSMD_MODEL_BANK)
                ph->count(4, __ballot(fold_of<MODEL>(memo_key_raw<MODEL, G>(s_bal, lane)) != d.fold) != 0ull, lane);
        }
        // the count at entry of the node a descent enters: stored whether or
        // not this try descended (the slot belongs to the current node's
        // next child, read only on leaving a child entered after this store)
        entry[dep0 * C_LANES] = (uint32_t)d.nodes;
        if (memo && d.depth > dep0 && status < 0) {
            uint32_t cnt = 0;
            bool hit = false;
            if constexpr (LT) {
                if constexpr (ST) t0 = ph->start();
                const LaneKey<MODEL, G> k = memo_key<MODEL, G>(d, a, s_bal, lane, epoch, sh);
                if constexpr (ST) ph->stop(2, t0, lane);
                hit = memo_lookup_lds<MODEL, G>(tab, k, h, cnt);
            } else {
                // the slot from registers; the key's balances only for a
                // probe of a slot this lane wrote for this history
                if constexpr (ST) t0 = ph->start();
                const uint32_t slot = memo_slot<MODEL, G>(d.fold, d.rem, d.ex, d.RS, d.depth, a, sh);
                if constexpr (ST) ph->stop(2, t0, lane);
                if constexpr (ST) ph->count(6, __ballot(wr.maybe(slot)) != 0ull, lane);
                if (wr.maybe(slot)) {
                    if constexpr (ST) t0 = ph->start();
                    const LaneKey<MODEL, G> k = memo_key<MODEL, G>(d, a, s_bal, lane, epoch, sh);
                    hit = memo_lookup<MODEL, G>(tab, k, h, cnt);
                    if constexpr (ST) ph->stop(3, t0, lane);
                }
            }
            if (hit) {
                if (d.nodes + cnt > limit) {      // the budget falls inside that subtree
                    d.nodes = limit;
                    status = QSMD_STATUS_BUDGET;
                } else {
                    d.nodes += cnt;               // the subtree's nodes, counted; it failed
                    d.cand = (M)0;
                    d.found = 1u;
                    skip = true;
                }
            }
        }
    }
    return status;
}

}  // namespace

namespace {

template <uint32_t MODEL, class G>
struct MemoLds {
    uint32_t ev[G::EV][C_LANES];
    int32_t bal[MODEL == QSMD_MODEL_BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][C_LANES];
    uint32_t entry[G::LEVELS][C_LANES];   // node count at entry, per level
};

// One group of 64 histories of p's list (from index base); every history of
// the list fits geometry G (a compact stage staged it before).
// ST: diagnostic build of the loop, one record per group in p.stats
// (kMemoStatsWords: see PhaseClock).
template <uint32_t MODEL, class G, bool LT, bool ST>
__device__ __forceinline__ void memo_group(const MemoArgs& p, uint64_t base, MemoLds<MODEL, G>& L, uint32_t* lcol,
                                           Counters& cnt, uint64_t t0, int lane, unsigned long long* q) {
    using M = typename G::M;
    const SearchArgs& a = p.s;
    const uint64_t total = list_total(a.list_count, a.list_shard_cap);
    const uint64_t limit = a.max_nodes ? a.max_nodes : ~0ull;
    uint32_t* tab;
    SlotHash sh;
    if constexpr (LT) {
        tab = lcol;
        sh.sh = 32u - (uint32_t)__builtin_ctz(p.lds_entries);
    } else {
        tab = p.table + ((uint64_t)blockIdx.x * C_LANES + (uint64_t)lane) * (uint64_t)p.entries *
                            (uint64_t)MemoEntry<G>::W;
        sh.sh = 32u - (uint32_t)__builtin_ctz(p.entries);
    }
    // a call with a model0 some reachable state has no key for: no memo
    const bool keyed = keys_fit<MODEL, G>(a);
    const uint64_t memo_after = (uint64_t)p.memo_after;
    const uint64_t idx = base + lane;
    const bool active = idx < total;
    uint64_t r0 = 0, c0 = 0;
    uint32_t hits = 0;
    if constexpr (ST) r0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t pos = !active ? 0u : (p.order ? (uint64_t)p.order[idx] : list_pos(a.list_count, a.list_shard_cap, idx));
    const uint32_t h = active ? a.list[pos] : 0u;
    qsmd_hdr H;
    if (active) H = a.hdr[h];
    else H = qsmd_hdr{0, 0, 0, 0, 0, 0};
    StagedT<M> s{0, 0, 0, 0, 0, true, true};
    if (active) {
        stage_lane<MODEL, G>(a, H, L.ev, lane);
        finish_lane<MODEL, G>(L.ev, lane, H.n_ev, H.n_pid, a.events + H.ev_off, s);
    }
    if constexpr (ST) {
        c0 = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
            q[0] = r0;
            q[1] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (!active) return;
    int status = -1;
    LaneDFS<MODEL, G> dfs;
    dfs.depth = 0;
    dfs.nodes = 0;
    bool search = false;
    if (!s.ok || !s.fits) {
        status = QSMD_STATUS_ENCODE_ERROR;   // cannot happen: the list came from a compact stage
    } else if (H.n_ev == 0) {
        status = QSMD_STATUS_LINEARISABLE;
    } else if (beyond_first_fail(a, h)) {
        status = QSMD_STATUS_SKIPPED;
    } else {
        dfs.init(s, a, L.bal, lane);
        search = true;
        if constexpr (G::EV == 32) {
            // go on from stage 0's state at its budget (the nodes it counted
            // stay counted); the levels entered there have no entry count,
            // so they are never recorded in the memo when they fail
            // (the saved state's slot: shard k = pos / cap, its position in the
            // shard pos % cap; none past resume_cap)
            const uint32_t cap = a.list_shard_cap;
            const uint64_t within = cap ? pos % cap : pos;
            if (p.resume && within < p.resume_cap) {
                dfs.restore(p.resume + ((cap ? pos / cap : 0u) * p.resume_cap + within) * kResumeWords, L.bal, lane);
                for (uint32_t d = 0; d < dfs.depth; ++d) L.entry[d][lane] = kNoEntry;
            }
        }
        dfs.fold = fold_of<MODEL>(memo_key_raw<MODEL, G>(L.bal, lane));
    }
    if (search) {
        bool skip = false;
        // the iteration count is the wavefront's (its lanes start together and
        // a lane steps in every iteration until it stops), so the hand-off
        // cap and the checks every 1024 iterations sit outside the inner loop
        uint64_t iter = 0;
        // (past tail_cap: the wave-mode tail launch searches it from the
        // root -- its state DAG of ~17 levels costs less than hundreds of
        // lane iterations; past giant_cap: the giant stage)
        const uint64_t gcap = p.giant_cap ? p.giant_cap : ~0ull;
        const uint64_t tcap = p.tail_cap && p.tail_list ? p.tail_cap : ~0ull;
        const uint64_t cap = gcap < tcap ? gcap : tcap;
        uint32_t lane_iter = 0;   // (ST only)
        Written wr;
        wr.clear();
        PhaseClock* ph = nullptr;
        if constexpr (ST) {
            __shared__ PhaseClock phc;
            ph = &phc;
            if (lane == (int)__builtin_ctzll(__ballot(1)))
                for (int k = 0; k < 8; ++k) phc.acc[k] = 0;
        }
        // nothing outstanding at the loop's entry: otherwise the compiler
        // waits for the memo insert's stores inside the loop (vmcnt counts
        // them), a store round trip on every backtrack
        __builtin_amdgcn_s_waitcnt(0);
        while (true) {
            const uint64_t span = cap - iter < 1024u ? cap - iter : 1024u;
            uint64_t k = 0;
            while (k < span) {
                if (status < 0) {
                    const bool was = skip;
                    status = memo_step<MODEL, G, LT, ST>(dfs, a, &L.ev[0][lane], L.bal, lane, limit, tab, h,
                                                         p.epoch, sh, &L.entry[0][lane], skip, keyed, memo_after, wr, ph);
                    if constexpr (ST) {
                        hits += (!was && skip) ? 1u : 0u;
                        ++lane_iter;
                    }
                }
                ++k;
                if (__ballot(status < 0) == 0ull) break;
            }
            iter += k;
            if (__ballot(status < 0) == 0ull) break;
            if (iter >= cap) {
                if (status < 0) status = iter >= tcap && tcap < gcap ? QSMD_STATUS_TO_TAIL : QSMD_STATUS_HANDED_OFF;
                break;
            }
            if (status < 0) {   // every 1024 iterations
                if (beyond_first_fail(a, h)) {
                    status = QSMD_STATUS_SKIPPED;
                } else if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                    atomicOr(a.timed_out, 1u);
                    status = QSMD_STATUS_BUDGET;
                }
            }
        }
        if constexpr (ST) {
            atomicMax(q + 3, (unsigned long long)lane_iter);
            atomicAdd(q + 4, (unsigned long long)lane_iter);
            atomicAdd(q + 5, (unsigned long long)hits);
            atomicMax(q + 7, (unsigned long long)(__builtin_amdgcn_s_memtime() - c0));
            if (lane == (int)__builtin_ctzll(__ballot(1)))
                for (int k = 0; k < 8; ++k) atomicAdd(q + 8 + k, (unsigned long long)ph->acc[k]);
        }
    }
    if constexpr (ST) {
        atomicAdd(q + 6, 1ull);
        atomicMax(q + 2, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    if (status == QSMD_STATUS_HANDED_OFF) {      // the giant stage searches it (exact, from the root)
        a.giant_list[atomicAdd(a.giant_count, 1u)] = h;
        return;
    }
    if (status == QSMD_STATUS_TO_TAIL) {         // the tail launch searches it (exact, from the root)
        p.tail_list[atomicAdd(p.tail_count, 1u)] = h;
        return;
    }
    note_failure(a, h, status);
    a.status[h] = (uint8_t)status;
    if (a.nodes) a.nodes[h] = dfs.nodes;
    if (a.witness && status == QSMD_STATUS_LINEARISABLE) dfs.write_witness(a.witness + H.ev_off, H.n_ev);
    cnt.add(status, dfs.nodes);
}

}  // namespace

// The heavy stage in lane mode, one launch for both lists: the groups of
// p32's list (stage 0's heavy histories, <= 32 events) then those of p64's
// (stage 0w's, <= 64 events), grid-stride.  The LDS (dynamic) holds one
// group of either geometry when `wide`, else G32 only (14 KB instead of 26:
// twice the resident wavefronts when the last call had no G64 history in the
// heavy stage); without it a G64 group goes to the giant stage, which
// searches any history exactly from the root.  LT (never with `wide`): the
// G32 memo tables in LDS after the group (a short list: the heavy stage's
// time is one search's DFS chain, and the HBM probe was half of it).
//
// With the folded tail (api.hip fold: the last call deferred nothing) no
// stage 0w runs: p64's list is stage 0's deferred list, which without `wide`
// goes on to the giant list.
template <uint32_t MODEL, bool LT>
__global__ __launch_bounds__(C_LANES, LT ? 1 : 3) void memo_search(MemoArgs p32, MemoArgs p64, uint32_t wide) {
    extern __shared__ uint32_t lds[];
    const int lane = threadIdx.x;
    const uint64_t n32 = (list_total(p32.s.list_count, p32.s.list_shard_cap) + 63u) / 64u,
                   n64 = (list_total(p64.s.list_count, p64.s.list_shard_cap) + 63u) / 64u;
    Counters cnt;
    const uint64_t t0 = p32.s.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t* lcol = nullptr;
    if constexpr (LT) {
        lcol = lds + sizeof(MemoLds<MODEL, G32>) / 4u + lane;
        for (uint32_t e = 0; e < p32.lds_entries; ++e) lcol[e * 8u * C_LANES] = kNoHistory;
    }
    // stage 0w's wide list goes on to the giant stage (wave mode searches it)
    const uint32_t nf = *p32.fwd_count;
    for (uint32_t b = blockIdx.x * C_LANES; b < nf; b += gridDim.x * C_LANES) {
        const bool in = b + (uint32_t)lane < nf;
        wave_append(in, in ? p32.fwd_list[b + lane] : 0u, p32.s.giant_list, p32.s.giant_count, lane);
    }
    for (uint64_t grp = blockIdx.x; grp < n32 + n64; grp += gridDim.x) {
        unsigned long long* q =
            p32.stats && grp < p32.stats_groups ? p32.stats + grp * kMemoStatsWords : nullptr;
        if (grp < n32) {
            auto& L = *reinterpret_cast<MemoLds<MODEL, G32>*>(lds);
            if (q) memo_group<MODEL, G32, LT, true>(p32, grp * 64u, L, lcol, cnt, t0, lane, q);
            else memo_group<MODEL, G32, LT, false>(p32, grp * 64u, L, lcol, cnt, t0, lane, q);
        } else if (!LT && wide) {
            auto& L = *reinterpret_cast<MemoLds<MODEL, G64>*>(lds);
            if (q) memo_group<MODEL, G64, false, true>(p64, (grp - n32) * 64u, L, lcol, cnt, t0, lane, q);
            else memo_group<MODEL, G64, false, false>(p64, (grp - n32) * 64u, L, lcol, cnt, t0, lane, q);
        } else {
            const uint64_t idx = (grp - n32) * 64u + lane;
            const bool in = idx < list_total(p64.s.list_count, p64.s.list_shard_cap);
            wave_append(in, in ? list_at(p64.s.list, p64.s.list_count, p64.s.list_shard_cap, idx) : 0u,
                        p64.s.giant_list, p64.s.giant_count, lane);
        }
    }
    cnt.flush(p32.s.buckets, lane);
}

// ---------------------------------------------------------------- heavy_sort
// Stage 0's heavy list ordered by predicted work (SearchArgs::heavy_key:
// the untried candidates on the stack at the budget, correlation 0.84 with
// a search's remaining lane iterations on config 3, tools/heavy_predictor.py),
// highest key first, so the heavy stage's groups of 64 hold searches of like
// length: lane utilisation 0.34 -> 0.49 on config 3.  Two launches, a
// counting sort: per-key counts (each workgroup counts its share in LDS,
// then one global atomic per key), then every workgroup reserves its range
// of each key's run with one atomic per key and writes its positions there.
// The order within a key follows the workgroups' reservations; the results
// do not depend on it (each history's search is independent).  Workgroup x
// of shard k takes that shard's entries x*256 .. x*256+255, grid-stride.
constexpr uint32_t kSortChunk = kSortChunkHost;

__device__ __forceinline__ uint32_t key_class(uint8_t key) { return key < kKeys - 1u ? key : kKeys - 1u; }

__global__ __launch_bounds__(kSortChunk) void heavy_count(const uint32_t* shards, uint32_t cap, const uint8_t* key,
                                                          uint32_t* cnt) {
    __shared__ uint32_t hist[kKeys];
    const uint32_t t = threadIdx.x, k = blockIdx.y;
    if (t < kKeys) hist[t] = 0u;
    __syncthreads();
    const uint32_t n = shards[k * kShardStride];
    for (uint32_t i = blockIdx.x * kSortChunk + t; i < n; i += gridDim.x * kSortChunk)
        atomicAdd(&hist[key_class(key[(uint64_t)k * cap + i])], 1u);
    __syncthreads();
    if (t < kKeys && hist[t]) atomicAdd(cnt + C_KHIST + t, hist[t]);
}

__global__ __launch_bounds__(kSortChunk) void heavy_scatter(const uint32_t* shards, uint32_t cap, const uint8_t* key,
                                                            uint32_t* cnt, uint32_t* order) {
    __shared__ uint32_t start[kKeys], hist[kKeys];
    const uint32_t t = threadIdx.x, k = blockIdx.y;
    const uint32_t n = shards[k * kShardStride];
    // each key's run: the keys above it first
    if (t < kKeys) {
        uint32_t p = 0u;
        for (uint32_t b = kKeys - 1u; b > t; --b) p += cnt[C_KHIST + b];
        start[t] = p;
    }
    for (uint32_t base = blockIdx.x * kSortChunk; base < n; base += gridDim.x * kSortChunk) {
        if (t < kKeys) hist[t] = 0u;
        __syncthreads();
        const uint32_t i = base + t;
        const uint32_t b = i < n ? key_class(key[(uint64_t)k * cap + i]) : 0u;
        const uint32_t rank = i < n ? atomicAdd(&hist[b], 1u) : 0u;
        __syncthreads();
        if (t < kKeys && hist[t]) hist[t] = start[t] + atomicAdd(cnt + C_KCUR + t, hist[t]);
        __syncthreads();
        if (i < n) order[hist[b] + rank] = k * cap + i;
        __syncthreads();
    }
}

hipError_t launch_heavy_sort(const uint32_t* shards, uint32_t cap, const uint8_t* key, uint32_t* cnt,
                             uint32_t* order, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(heavy_count, dim3(grid, kShards), dim3(kSortChunk), 0, s, shards, cap, key, cnt);
    hipLaunchKernelGGL(heavy_scatter, dim3(grid, kShards), dim3(kSortChunk), 0, s, shards, cap, key, cnt, order);
    return hipGetLastError();
}

template <uint32_t MODEL>
static size_t memo_lds_bytes(uint32_t lds_entries) {
    return sizeof(MemoLds<MODEL, G32>) + (size_t)lds_entries * 8u * C_LANES * 4u;
}

template <uint32_t MODEL, bool LT>
static hipError_t launch_memo_t(const MemoArgs& p32, const MemoArgs& p64, uint32_t grid, bool wide, hipStream_t s,
                                hipEvent_t start, hipEvent_t stop) {
    const size_t lds = LT ? memo_lds_bytes<MODEL>(p32.lds_entries)
                          : (wide ? sizeof(MemoLds<MODEL, G64>) : sizeof(MemoLds<MODEL, G32>));
    hipExtLaunchKernelGGL((memo_search<MODEL, LT>), dim3(grid), dim3(C_LANES), lds, s, start, stop, 0u, p32, p64,
                          wide ? 1u : 0u);
    return hipGetLastError();
}

// Whether the LDS tables of `lds_entries` per lane can launch: their size
// within `cap` (0 = the device's limit; a lower cap is a diagnostic knob,
// memo_lds_cap, that makes the refusal happen on gfx950) and the kernel's
// dynamic-LDS limit raised to it.  The host decides before it sizes the
// tables, so a refusal runs the HBM tables it then allocates.
bool memo_lds_accepted(uint32_t model_id, uint32_t lds_entries, size_t cap) {
    const bool bank = model_id == QSMD_MODEL_BANK;
    const size_t lds = bank ? memo_lds_bytes<QSMD_MODEL_BANK>(lds_entries) : memo_lds_bytes<QSMD_MODEL_TICKET>(lds_entries);
    if (cap && lds > cap) return false;
    static std::atomic<int> set_b[kAttrDevices], set_t[kAttrDevices];
    const hipError_t e = bank ? ensure_dyn_lds(reinterpret_cast<const void*>(&memo_search<QSMD_MODEL_BANK, true>), set_b, lds)
                              : ensure_dyn_lds(reinterpret_cast<const void*>(&memo_search<QSMD_MODEL_TICKET, true>), set_t, lds);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return true;
}

// lds_tables (with !wide): the caller has checked memo_lds_accepted
hipError_t launch_memo(const MemoArgs& p32, const MemoArgs& p64, uint32_t grid, bool wide, bool lds_tables,
                       hipStream_t s, hipEvent_t start, hipEvent_t stop) {
    const bool bank = p32.s.model_id == QSMD_MODEL_BANK;
    if (lds_tables && !wide)
        return bank ? launch_memo_t<QSMD_MODEL_BANK, true>(p32, p64, grid, wide, s, start, stop)
                    : launch_memo_t<QSMD_MODEL_TICKET, true>(p32, p64, grid, wide, s, start, stop);
    return bank ? launch_memo_t<QSMD_MODEL_BANK, false>(p32, p64, grid, wide, s, start, stop)
                : launch_memo_t<QSMD_MODEL_TICKET, false>(p32, p64, grid, wide, s, start, stop);
}

}  // namespace qsmd
