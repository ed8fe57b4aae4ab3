// split.h -- the giant stage's device code (included by split.hip only, whose
// kernels launch it; with lane mode's folded tail, api.hip `fold`, stage 0's
// deferred histories reach it straight from the heavy stage's forward list):
// every history the compact and heavy stages hand on (beyond their geometry,
// or over their work caps), searched by one lane or split over many
// (SURVEY.md §8e); then the totals.
//
// One launch per call (giant_search), phases chained inside it by counters:
//
//   frontier  one lane per giant (pulled in chunks of 64).  First the whole
//             reference DFS (src/Linearisability.hs:52-69, Lemma L1 state)
//             in the lane, for at most whole_cap iterations (with the exact
//             memo below when on): most giants end there.  Otherwise the DFS
//             is cut at depth D: a node reached at depth D (a passed
//             postcondition, i.e. a `step` that recurses) is not expanded but
//             recorded as a task -- its path and the number of nodes the
//             reference has counted up to and including it.  D is the
//             smallest depth giving `target` tasks (count-only passes, then
//             one emitting pass into a contiguous reserved range).
//   tasks     (after every frontier) idle lanes pull tasks with one atomic per
//             wavefront.  A lane replays the task's path (transitions only,
//             nothing counted), then searches the subtree below it
//             (`any' (step ...)`: no children = True).  A task that decides
//             (True, or Map.! raising) lowers the giant's min_win; tasks
//             after it are skipped.
//   combine   (after every task) one lane per giant folds the task results in
//             DFS order (combine_tasks, internal.h): the reference's count is
//             nodes above the cut up to the deciding task + all nodes of the
//             subtrees before it + that subtree's count.
//   fixup     (QSMD_FLAG_EARLY_EXIT_BATCH, after the combine) histories after
//             the first failing one become SKIPPED; the totals are recounted.
//   finish    the last workgroup sums the buckets into the call's totals and
//             restores the counters for the next call.  With no giant (the
//             common case) every other workgroup returns at once and
//             workgroup 0 finishes.
// A phase waits (polling an agent-scope counter) only on work that running
// workgroups have already taken, so the chain cannot deadlock.
//
// Memo (north star (c)): with QSMD_FLAG_MEMO, a subtree root state (remaining
// events, model) that was fully searched without success is inserted into an
// open-addressing table in HBM; a lane that reaches a state in the table
// skips its subtree.  A state's outcome is a function of the state alone
// (Lemma L1; post and next read only the model), so pruning never changes a
// verdict.  Entries are 8 x u64: word 0 = tag (giant id, hash, ready bit),
// words 1-7 = the exact key; writers store the key with agent-scope (sc1)
// stores, drain them, then set the ready bit; readers compare every key word,
// so a stale or torn read can only miss.
//
// Generic DFS (GenDFS) over MaskT event bitsets, history in LDS [slot][lane];
// two variants: <= 64 events / <= 8 pids (u64 masks, 64 lanes) and <= 128
// events / <= 128 pids (128-bit masks, 16 lanes of the wavefront).
#pragma once

#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"
#include "mask.h"
#include "models.h"

namespace qsmd {

namespace {

constexpr int kDescended = -2;   // step(): descended into a new node

__device__ __forceinline__ uint32_t sp_lane_prefix(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

__device__ __forceinline__ uint64_t ld_sc1(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned long long* p, uint64_t v) {
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// --------------------------------------------------------------- memo table
constexpr int kMemoKey = 7;       // key words per entry (after the tag)
constexpr int kMemoProbe = 16;

struct MemoKey {
    uint64_t w[kMemoKey];
    uint64_t tag, hash;
    bool ok;                      // false: state not representable (no memo)
};

struct Memo {
    unsigned long long* tab;
    uint64_t mask;
    uint32_t epoch = 0;           // exact memo: the call's tag

    // ---- exact-count memo (csrc/memo.hip's argument, shared by the split
    // stage's lanes): 16 x u64 per entry = [tag | key 7 | count]; tag =
    // epoch24 << 40 | (giant + 1) << 8 | hash7 << 1 | ready.  Writers claim an
    // empty or stale (older epoch) slot by CAS, store key and count with
    // agent-scope (sc1) stores, drain them, then set the ready bit; readers use
    // sc1 loads (the protocol of the QSMD_FLAG_MEMO table) and take a count
    // only under a ready, matching tag
    // and all seven key words.
    __device__ uint64_t xtag(const MemoKey& k, uint32_t id) const {
        return ((uint64_t)(epoch & 0xFFFFFFu) << 40) | ((uint64_t)(id + 1u) << 8) | ((k.hash >> 56) & 0xFEull);
    }
    __device__ bool stale(uint64_t t) const { return t != 0 && (uint32_t)(t >> 40) != (epoch & 0xFFFFFFu); }
    __device__ bool xlookup(const MemoKey& k, uint32_t id, uint64_t* count) const {
        const uint64_t want = xtag(k, id);
        for (int i = 0; i < kMemoProbe; ++i) {
            unsigned long long* e = tab + ((k.hash + (uint64_t)i) & mask) * 16u;
            const uint64_t t = ld_sc1(e);
            if (t == 0 || stale(t)) return false;   // an insert would have taken this slot
            if (t != (want | 1ull)) continue;
            bool eq = true;
#pragma unroll
            for (int q = 0; q < kMemoKey; ++q) eq = eq & (ld_sc1(e + 1 + q) == k.w[q]);
            if (eq) {
                *count = ld_sc1(e + 8);
                return true;
            }
        }
        return false;
    }
    __device__ void xinsert(const MemoKey& k, uint32_t id, uint64_t count) const {
        const uint64_t want = xtag(k, id);
        for (int i = 0; i < kMemoProbe; ++i) {
            unsigned long long* e = tab + ((k.hash + (uint64_t)i) & mask) * 16u;
            uint64_t t = ld_sc1(e);
            while (t == 0 || stale(t)) {
                const uint64_t old = atomicCAS(e, (unsigned long long)t, (unsigned long long)want);
                if (old == t) {
#pragma unroll
                    for (int q = 0; q < kMemoKey; ++q) st_sc1(e + 1 + q, k.w[q]);
                    st_sc1(e + 8, count);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // key and count land before the bit
                    __hip_atomic_fetch_or(e, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    return;
                }
                t = old;                             // taken meanwhile: look at what is there now
            }
            if ((t | 1ull) == (want | 1ull)) {
                if (!(t & 1ull)) return;             // being written (likely this very key)
                bool eq = true;
#pragma unroll
                for (int q = 0; q < kMemoKey; ++q) eq = eq & (ld_sc1(e + 1 + q) == k.w[q]);
                if (eq) return;                      // present (the same count: a function of the state)
            }
        }
    }

    // ---- QSMD_FLAG_MEMO table: 8 x u64 per entry = [tag | key 7]; tag =
    // epoch24 << 40 | k.tag (the giant | hash7), the same claim / ready
    // protocol; entries of an older call (epoch) count as empty, so the table
    // is cleared only when allocated (and when the 24-bit epochs wrap)
    __device__ uint64_t mtag(const MemoKey& k) const { return ((uint64_t)(epoch & 0xFFFFFFu) << 40) | k.tag; }
    __device__ bool lookup(const MemoKey& k) const {
        const uint64_t want = mtag(k);
        for (int i = 0; i < kMemoProbe; ++i) {
            const unsigned long long* e = tab + ((k.hash + (uint64_t)i) & mask) * 8u;
            const uint64_t t = ld_sc1(e);
            if (t == 0 || stale(t)) return false;
            if ((t | 1ull) != (want | 1ull) || !(t & 1ull)) continue;
            bool eq = true;
#pragma unroll
            for (int q = 0; q < kMemoKey; ++q) eq = eq & (ld_sc1(e + 1 + q) == k.w[q]);
            if (eq) return true;
        }
        return false;
    }

    __device__ void insert(const MemoKey& k) const {
        const uint64_t want = mtag(k);
        for (int i = 0; i < kMemoProbe; ++i) {
            unsigned long long* e = tab + ((k.hash + (uint64_t)i) & mask) * 8u;
            uint64_t t = ld_sc1(e);
            while (t == 0 || stale(t)) {
                const uint64_t old = atomicCAS(e, (unsigned long long)t, (unsigned long long)want);
                if (old == t) {
#pragma unroll
                    for (int q = 0; q < kMemoKey; ++q) st_sc1(e + 1 + q, k.w[q]);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_fetch_or(e, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    return;
                }
                t = old;
            }
            if ((t | 1ull) == (want | 1ull)) {
                if (!(t & 1ull)) return;          // being written (likely this very key)
                bool eq = true;
#pragma unroll
                for (int q = 0; q < kMemoKey; ++q) eq = eq & (ld_sc1(e + 1 + q) == k.w[q]);
                if (eq) return;
            }
        }
    }
};

// ----------------------------------------------------------- generic DFS

template <uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
struct GLds {
    static constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    static constexpr int MAXD = MAXEV / 2;
    uint2 ev[MAXEV][LANES];
    MaskT pm[MAXPID][LANES];
    uint32_t meta[MAXD][LANES];                         // j | pre-op model bits
    int64_t undo[BANK ? 1 : MAXD][LANES];               // Ticket: pre-op n
    int64_t bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][LANES];
    uint64_t ent[MAXD][LANES];                          // exact memo: nodes counted on entering level d
};

template <typename MaskT> __device__ __forceinline__ uint64_t mask_lo(const MaskT& m) { return (uint64_t)m; }
template <typename MaskT> __device__ __forceinline__ uint64_t mask_hi(const MaskT&) { return 0ull; }
template <> __device__ __forceinline__ uint64_t mask_lo<M128>(const M128& m) { return m.lo; }
template <> __device__ __forceinline__ uint64_t mask_hi<M128>(const M128& m) { return m.hi; }

template <uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
struct GenDFS {
    using Ops = MaskOps<MaskT>;
    using Lds = GLds<MODEL, MaskT, MAXEV, MAXPID, LANES>;
    static constexpr bool BANK = MODEL == QSMD_MODEL_BANK;

    MaskT INV, RESP, rem, cand;
    uint32_t depth, base, found, skip_ins, n_ev;
    uint64_t nodes;
    BankState bank;
    TicketState tick;

    // Stage history H into the lane's LDS column and validate it.
    __device__ bool load(const SearchArgs& a, const qsmd_hdr& H, Lds& s, int lane) {
        n_ev = H.n_ev;
        const uint32_t n_pid = H.n_pid;
        INV = MaskT{};
        RESP = MaskT{};
        bool ok = H.model_id == MODEL && n_ev <= (uint32_t)MAXEV && n_pid <= (uint32_t)MAXPID &&
                  (uint64_t)H.ev_off + n_ev <= a.n_events;
        if (!ok) return false;
        for (uint32_t p = 0; p < n_pid; ++p) s.pm[p][lane] = MaskT{};
        const uint2* evp = a.events + H.ev_off;
        for (uint32_t e0 = 0; e0 < n_ev; e0 += 8) {
            uint2 xs[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) xs[k] = e0 + k < n_ev ? evp[e0 + k] : make_uint2(0u, 0u);
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t e = e0 + k;
                if (e >= n_ev) break;
                const Ev ev{xs[k].x, (int32_t)xs[k].y};
                const uint32_t p = ev.pid();
                ok = ok && p < n_pid && valid_event<MODEL>(ev);
                s.ev[e][lane] = xs[k];
                const MaskT bit = Ops::bit((int)e);
                if (ev.is_resp()) RESP |= bit; else INV |= bit;
                if (p < n_pid) s.pm[p][lane] = s.pm[p][lane] | bit;
            }
        }
        return ok;
    }

    __device__ __forceinline__ MaskT candidates(const MaskT& r) const {
        const MaskT rr = r & RESP;
        const int R = Ops::any(rr) ? Ops::ctz(rr) : Ops::BITS;
        return r & INV & Ops::below(R);
    }

    // model0 and the root of the search
    __device__ void init(const SearchArgs& a, Lds& s, int lane) {
        bank = BankState{a.m0_exists, 0u};
        tick = TicketState{a.m0_just, a.m0_val[0]};
        if constexpr (BANK) {
#pragma unroll
            for (int c = 0; c < QSMD_BANK_MAX_ACCOUNTS; ++c) {
                const bool ex = (a.m0_exists >> c) & 1u;
                const int64_t v = ex ? a.m0_val[c] : 0;
                s.bal[c][lane] = v;
                bank.neg |= (ex && v < 0) ? (1u << c) : 0u;
            }
        }
        rem = INV | RESP;
        cand = candidates(rem);
        depth = 0;
        base = 0;
        found = 0;
        skip_ins = 0;
        nodes = 0;
    }

    // Push level `depth` for child j (its response r) and apply the
    // transition (Left inv; Right is the identity for both models).
    __device__ __forceinline__ void descend(uint32_t j, const Ev& ej, const MaskT& pm, int r, Lds& s, int lane) {
        if constexpr (BANK) {
            s.meta[depth][lane] = j | (bank.exists << 8) | (bank.neg << 16);
            const uint32_t code = ej.code();
            if (code != QSMD_BANK_CHECK_BALANCE) {
                const int ia = (int)ej.a();
                const int64_t m = ej.val;
                const bool ex_a = (bank.exists >> ia) & 1u;
                const int64_t bal_a = s.bal[ia][lane];
                int64_t na;
                if (code == QSMD_BANK_OPEN_ACCOUNT) na = ex_a ? bal_a : 0;
                else if (code == QSMD_BANK_DEPOSIT) na = ex_a ? bal_a + m : m;
                else na = ex_a ? bal_a - m : m;          // Withdraw / Transfer's withdraw
                s.bal[ia][lane] = na;
                bank.exists |= 1u << ia;
                bank.neg = (bank.neg & ~(1u << ia)) | (na < 0 ? (1u << ia) : 0u);
                if (code == QSMD_BANK_TRANSFER) {
                    const int ib = (int)ej.b();
                    const bool ex_b = (bank.exists >> ib) & 1u;
                    const int64_t nb = ex_b ? s.bal[ib][lane] + m : m;
                    s.bal[ib][lane] = nb;
                    bank.exists |= 1u << ib;
                    bank.neg = (bank.neg & ~(1u << ib)) | (nb < 0 ? (1u << ib) : 0u);
                }
            }
        } else {
            s.meta[depth][lane] = j | (tick.just << 8);
            s.undo[depth][lane] = tick.n;
            ticket_apply(tick, ej);
        }
        ++depth;
        rem &= ~(Ops::lowest(rem & pm & INV) | Ops::bit(r));
        cand = candidates(rem);
        found = 0;
    }

    // Pop level depth-1 and restore its state exactly; the remaining
    // candidates of that level are the ones after j.
    __device__ __forceinline__ void backtrack(Lds& s, int lane) {
        --depth;
        const uint32_t meta = s.meta[depth][lane];
        const uint32_t j = meta & 0xFFu;
        const uint2 xj = s.ev[j][lane];
        const Ev ej{xj.x, (int32_t)xj.y};
        const MaskT gone = ~rem & s.pm[ej.pid()][lane];
        rem |= Ops::bit(Ops::msb(gone & INV)) | Ops::bit(Ops::msb(gone & RESP));
        if constexpr (BANK) {
            const uint32_t code = ej.code();
            if (code != QSMD_BANK_CHECK_BALANCE) {
                const uint32_t pre_ex = (meta >> 8) & 0xFFu;
                const int ia = (int)ej.a();
                const int64_t m = ej.val;
                if (code == QSMD_BANK_TRANSFER) {
                    const int ib = (int)ej.b();
                    const bool exb_mid = ((pre_ex | (1u << ia)) >> ib) & 1u;
                    s.bal[ib][lane] = exb_mid ? s.bal[ib][lane] - m : 0;
                }
                const int64_t delta = code == QSMD_BANK_DEPOSIT ? m : code == QSMD_BANK_OPEN_ACCOUNT ? 0 : -m;
                s.bal[ia][lane] = ((pre_ex >> ia) & 1u) ? s.bal[ia][lane] - delta : 0;
                bank.exists = pre_ex;
                bank.neg = (meta >> 16) & 0xFFu;
            }
        } else {
            tick.just = (meta >> 8) & 1u;
            tick.n = s.undo[depth][lane];
        }
        cand = candidates(rem) & ~Ops::below((int)j + 1);
        found = 1;
    }

    // Follow a recorded choice without evaluating or counting it.
    __device__ __forceinline__ void replay(uint32_t j, Lds& s, int lane) {
        const uint2 xj = s.ev[j][lane];
        const Ev ej{xj.x, (int32_t)xj.y};
        const MaskT pm = s.pm[ej.pid()][lane];
        const MaskT rr = rem & pm & RESP;
        descend(j, ej, pm, Ops::ctz(rr), s, lane);
    }

    // The state key (remaining events, model) for the memo table.
    __device__ MemoKey key(uint32_t id, Lds& s, int lane) const {
        MemoKey k;
        k.ok = true;
        k.w[0] = mask_lo(rem);
        k.w[1] = mask_hi(rem);
        if constexpr (BANK) {
            k.w[2] = bank.exists;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t b0 = ((bank.exists >> (2 * q)) & 1u) ? s.bal[2 * q][lane] : 0;
                const int64_t b1 = ((bank.exists >> (2 * q + 1)) & 1u) ? s.bal[2 * q + 1][lane] : 0;
                k.ok = k.ok && b0 == (int64_t)(int32_t)b0 && b1 == (int64_t)(int32_t)b1;
                k.w[3 + q] = (uint64_t)(uint32_t)(int32_t)b0 | ((uint64_t)(uint32_t)(int32_t)b1 << 32);
            }
        } else {
            k.w[2] = tick.just;
            k.w[3] = tick.just ? (uint64_t)tick.n : 0ull;
            k.w[4] = k.w[5] = k.w[6] = 0;
        }
        uint64_t h = mix64(0x51ED5EEDull + id);
#pragma unroll
        for (int q = 0; q < kMemoKey; ++q) h = mix64(h ^ k.w[q]);
        k.hash = h;
        k.tag = ((uint64_t)(id + 1u) << 8) | ((h >> 56) & 0xFEull);   // (id + 1 < 2^32: below the epoch)
        return k;
    }

    // One DFS iteration.  Returns -1 (continue), kDescended (a node passed
    // its postcondition and was entered), or the final QSMD_STATUS_*.
    // MEMO: 0 none, 1 QSMD_FLAG_MEMO (skip known-failing states: explored
    // counts), 2 exact-count memo (add the recorded subtree count: the
    // reference's counts)
    template <int MEMO>
    __device__ int step(Lds& s, int lane, uint64_t limit, const Memo& memo, uint32_t id) {
        if (!Ops::any(cand)) {
            // no children: a leaf => True (any' []), the root => False (any []);
            // a subtree rooted at depth base > 0 is an inner node of the tree
            if (!found || depth == base) {
                if constexpr (MEMO != 0) {
                    if (found && depth > 0 && !skip_ins) {   // a task root that failed
                        const MemoKey k = key(id, s, lane);
                        if (k.ok) {
                            if constexpr (MEMO == 2) memo.xinsert(k, id, nodes);   // the task counted its subtree
                            else memo.insert(k);
                        }
                    }
                }
                return (!found && depth > 0) ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_NONLINEARISABLE;
            }
            if constexpr (MEMO != 0) {
                if (!skip_ins) {
                    const MemoKey k = key(id, s, lane);      // this state failed
                    if (k.ok) {
                        if constexpr (MEMO == 2) memo.xinsert(k, id, nodes - s.ent[depth - 1][lane]);
                        else memo.insert(k);
                    }
                }
                skip_ins = 0;
            }
            backtrack(s, lane);
            return -1;
        }
        const uint32_t j = (uint32_t)Ops::ctz(cand);
        cand = Ops::clear_lowest(cand);
        const uint2 xj = s.ev[j][lane];
        const Ev ej{xj.x, (int32_t)xj.y};
        const MaskT pm = s.pm[ej.pid()][lane];
        const MaskT rr = rem & pm & RESP;
        if (!Ops::any(rr)) return -1;                  // findResponse => []: no child
        found = 1;
        if (nodes >= limit) return QSMD_STATUS_BUDGET;
        ++nodes;
        const int r = Ops::ctz(rr);
        const uint2 xr = s.ev[r][lane];
        const Ev er{xr.x, (int32_t)xr.y};
        int post;
        if constexpr (BANK) post = bank_post(bank, ej, er, s.bal[ej.a()][lane]);
        else post = ticket_post(tick, ej, er);
        if (post == POST_ERROR) return QSMD_STATUS_MODEL_ERROR;
        if (post == POST_FALSE) return -1;
        descend(j, ej, pm, r, s, lane);
        if constexpr (MEMO == 1) {
            const MemoKey k = key(id, s, lane);
            if (k.ok && memo.lookup(k)) {              // known to fail: skip the subtree
                cand = MaskT{};
                found = 1;
                skip_ins = 1;
            }
        } else if constexpr (MEMO == 2) {
            s.ent[depth - 1][lane] = nodes;
            const MemoKey k = key(id, s, lane);
            uint64_t c = 0, sum = 0;
            if (k.ok && memo.xlookup(k, id, &c)) {     // searched before: its count, failed
                if (__builtin_add_overflow(nodes, c, &sum) || sum > limit) {
                    nodes = limit;                     // the budget falls inside that subtree
                    return QSMD_STATUS_BUDGET;
                }
                nodes = sum;
                cand = MaskT{};
                found = 1;
                skip_ins = 1;
            }
        }
        return kDescended;
    }

    // Abandon the node just entered as if its subtree had failed (the cut).
    __device__ __forceinline__ void prune() {
        cand = MaskT{};
        found = 1;
        skip_ins = 1;
    }

    __device__ void path_to(uint8_t* w, uint32_t len, Lds& s, int lane) const {
        for (uint32_t d = 0; d < depth && d < len; ++d) w[d] = (uint8_t)(s.meta[d][lane] & 0xFFu);
        if (depth < len) w[depth] = QSMD_WITNESS_END;
    }
};

__device__ __forceinline__ bool sp_time_up(const SearchArgs& a, uint64_t t0, uint32_t iter) {
    return a.time_limit && ((iter & 1023u) == 0u) && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit;
}

template <int MAXEV, int MAXPID>
__device__ __forceinline__ bool fits_variant(const qsmd_hdr& H) {
    return H.n_ev <= (uint32_t)MAXEV && H.n_pid <= (uint32_t)MAXPID;
}
// variant of a history: the first that holds it (0: <= 64 events, <= 8 pids)
__device__ __forceinline__ uint32_t variant_of(const qsmd_hdr& H) {
    return fits_variant<64, 8>(H) ? 0u : 1u;
}

}  // namespace

namespace {

// ---------------------------------------------------------------- frontier

// Search above the cut.  Returns the terminal status; count = tasks reached
// (written to out[0..) when out != null); top = nodes counted.
template <uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
__device__ int top_search(GenDFS<MODEL, MaskT, MAXEV, MAXPID, LANES>& d,
                          GLds<MODEL, MaskT, MAXEV, MAXPID, LANES>& s, const SearchArgs& a, int lane,
                          uint32_t cut, uint64_t limit, uint32_t g, uint32_t max_count, qsmd_task* out,
                          uint32_t& count, uint64_t t0) {
    const Memo none{nullptr, 0};
    d.init(a, s, lane);
    count = 0;
    uint32_t iter = 0;
    for (;;) {
        const int st = d.template step<0>(s, lane, limit, none, 0);
        if (st == kDescended) {
            if (d.depth == cut) {
                if (out && count < max_count) {
                    qsmd_task t;
                    t.hist = g;
                    t.depth = (uint16_t)cut;
                    t.reserved = 0;
                    t.top_before = d.nodes;
#pragma unroll
                    for (int q = 0; q < QSMD_SPLIT_MAX_DEPTH; ++q)
                        t.path[q] = (uint32_t)q < cut ? (uint8_t)(s.meta[q][lane] & 0xFFu) : (uint8_t)0;
                    out[count] = t;
                }
                ++count;
                d.prune();
            }
            continue;
        }
        if (st >= 0) return st;
        if (sp_time_up(a, t0, ++iter)) {
            atomicOr(a.timed_out, 1u);
            return QSMD_STATUS_BUDGET;
        }
    }
}

// The whole search in one lane, for at most `cap` iterations (0 = none):
// MEMO 0 plain, 1 QSMD_FLAG_MEMO, 2 exact-count memo.  Returns the status,
// or -1 when the cap was reached first.
template <int MEMO, uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
__device__ int whole_search(GenDFS<MODEL, MaskT, MAXEV, MAXPID, LANES>& d,
                            GLds<MODEL, MaskT, MAXEV, MAXPID, LANES>& s, const SearchArgs& a, int lane,
                            uint64_t limit, const Memo& memo, uint32_t g, uint64_t cap, uint64_t t0) {
    d.init(a, s, lane);
    uint64_t iter = 0;
    for (;;) {
        const int st = d.template step<MEMO>(s, lane, limit, memo, g);
        if (st >= 0) return st;
        ++iter;
        if (cap && iter >= cap) return -1;
        if (sp_time_up(a, t0, (uint32_t)iter)) {
            atomicOr(a.timed_out, 1u);
            return QSMD_STATUS_BUDGET;
        }
    }
}

// One giant (history p.giant_list[g], of `variant`) in this lane: the whole
// search first (p.whole_cap iterations; unbounded without a split), then
// the cut into tasks.  Writes p.giants[g].
template <uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
__device__ void frontier_one(const SplitArgs& p, uint32_t g, uint32_t h, const qsmd_hdr& H, uint32_t variant,
                             GLds<MODEL, MaskT, MAXEV, MAXPID, LANES>& s, int lane, uint64_t t0) {
    using DFS = GenDFS<MODEL, MaskT, MAXEV, MAXPID, LANES>;
    const SearchArgs& a = p.s;
    const uint64_t limit = a.max_nodes ? a.max_nodes : ~0ull;
    GiantRec G;
    G.h = h;
    G.variant = variant;
    G.first = 0;
    G.n_tasks = 0;
    G.depth = 0;
    G.term_status = QSMD_STATUS_ENCODE_ERROR;
    G.term_nodes = 0;
    G.min_win = ~0u;
    G.pad = 0;
    DFS d;
    if (!d.load(a, H, s, lane)) {
        p.giants[g] = G;
        return;
    }
    if (d.n_ev == 0) {
        G.term_status = QSMD_STATUS_LINEARISABLE;                 // :59
        p.giants[g] = G;
        return;
    }
    Memo memo{p.memo, p.memo_mask};
    memo.epoch = p.memo_epoch;
    const bool split = p.target != 0;
    if (!split || p.whole_cap) {
        // the whole search in this lane (exact memo when on; most giants end here)
        const uint64_t cap = split ? p.whole_cap : 0;
        const int st = !p.memo ? whole_search<0>(d, s, a, lane, limit, memo, g, cap, t0)
                     : p.memo_exact ? whole_search<2>(d, s, a, lane, limit, memo, g, cap, t0)
                                    : whole_search<1>(d, s, a, lane, limit, memo, g, cap, t0);
        if (st >= 0) {
            G.term_status = (uint32_t)st;
            G.term_nodes = d.nodes;
            if (a.witness && st == QSMD_STATUS_LINEARISABLE) d.path_to(a.witness + H.ev_off, d.n_ev, s, lane);
            p.giants[g] = G;
            return;
        }
    }
    // past the cap: the cut (top_search re-initialises the search)
    const uint32_t dmax = min(min(p.max_depth, (uint32_t)QSMD_SPLIT_MAX_DEPTH), d.n_ev / 2u);
    uint32_t cut = 1, count = 0;
    for (;; ++cut) {
        top_search(d, s, a, lane, cut, limit, g, 0, nullptr, count, t0);
        if (count > p.max_tasks && cut > 1) { --cut; break; }
        if (count >= p.target || cut >= dmax) break;
    }
    // reserve a contiguous range; on overflow search the whole history here
    qsmd_task* region = p.tasks + (uint64_t)variant * p.task_cap;
    uint32_t first = ~0u;
    top_search(d, s, a, lane, cut, limit, g, 0, nullptr, count, t0);
    if (count <= p.max_tasks) {
        first = atomicAdd(&p.cnt[C_TASKS0 + variant], count);
        if ((uint64_t)first + count > p.task_cap) {
            // out of task slots: mark the part of the range below the cap as holes
            for (uint64_t q = first; q < p.task_cap && q < (uint64_t)first + count; ++q) region[q].hist = ~0u;
            first = ~0u;
        }
    }
    int st;
    if (first != ~0u) {
        uint32_t emitted = 0;
        st = top_search(d, s, a, lane, cut, limit, g, count, region + first, emitted, t0);
        G.first = first;
        G.n_tasks = count;
        G.depth = cut;
    } else {
        // no task slots left: the whole search here
        st = !p.memo ? whole_search<0>(d, s, a, lane, limit, memo, g, 0, t0)
           : p.memo_exact ? whole_search<2>(d, s, a, lane, limit, memo, g, 0, t0)
                          : whole_search<1>(d, s, a, lane, limit, memo, g, 0, t0);
    }
    G.term_status = (uint32_t)st;
    G.term_nodes = d.nodes;
    if (a.witness && st == QSMD_STATUS_LINEARISABLE) d.path_to(a.witness + H.ev_off, d.n_ev, s, lane);
    p.giants[g] = G;
}

// ------------------------------------------------------------------- tasks

// Persistent task search of one variant by the LANES lanes of this
// wavefront that call it; returns the tasks this wavefront took (holes and
// skipped ones included).
template <uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
__device__ uint32_t task_loop(const SplitArgs& p, uint32_t variant, GLds<MODEL, MaskT, MAXEV, MAXPID, LANES>& s,
                              int lane, uint64_t t0, uint32_t* head) {
    using DFS = GenDFS<MODEL, MaskT, MAXEV, MAXPID, LANES>;
    constexpr uint32_t kRefillMin = LANES >= 64 ? 8u : 2u;
    const SearchArgs& a = p.s;
    const uint32_t count = min(__hip_atomic_load(&p.cnt[C_TASKS0 + variant], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT), p.task_cap);
    const qsmd_task* tasks = p.tasks + (uint64_t)variant * p.task_cap;
    uint8_t* t_status = p.task_status + (uint64_t)variant * p.task_cap;
    uint64_t* t_nodes = p.task_nodes + (uint64_t)variant * p.task_cap;
    uint8_t* t_wit = p.task_witness ? p.task_witness + (uint64_t)variant * p.task_cap * kTaskWitness : nullptr;
    Memo memo{p.memo, p.memo_mask};
    memo.epoch = p.memo_epoch;
    const bool use_memo = p.memo != nullptr;
    const bool exact = use_memo && p.memo_exact;
    const uint64_t limit = a.max_nodes ? a.max_nodes : ~0ull;

    bool busy = false, exhausted = count == 0;
    uint32_t idx = 0, g = 0, local = 0, h = 0, iter = 0, taken = 0;
    DFS d;
    d.depth = 0;
    d.nodes = 0;
    for (;;) {
        const uint64_t idle = __ballot(!busy);
        const uint64_t busy_m = __ballot(busy);
        if (exhausted && busy_m == 0) break;
        if (!exhausted && idle && (__builtin_popcountll(idle) >= kRefillMin || busy_m == 0)) {
            const int leader = __builtin_ctzll(idle);
            const uint32_t want = (uint32_t)__builtin_popcountll(idle);
            uint32_t first = 0;
            if (lane == leader) first = atomicAdd(head, want);
            first = __shfl(first, leader, LANES);
            if (first + want >= count) exhausted = true;
            taken += first >= count ? 0u : min(want, count - first);
            if (!busy) {
                idx = first + sp_lane_prefix(idle);
                if (idx < count && tasks[idx].hist != ~0u) {   // ~0u: a hole (frontier overflow)
                    const qsmd_task T = tasks[idx];   // path bytes re-read below (no scratch)
                    g = T.hist;
                    const GiantRec* G = p.giants + g;
                    h = p.external_tasks ? 0u : G->h;
                    local = idx - G->first;
                    const uint32_t mw = __hip_atomic_load(&G->min_win, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (local > mw || beyond_first_fail(a, h)) {
                        t_status[idx] = QSMD_STATUS_SKIPPED;
                        t_nodes[idx] = 0;
                    } else {
                        d.load(a, a.hdr[h], s, lane);         // validated by the frontier
                        d.init(a, s, lane);
                        for (uint32_t q = 0; q < T.depth; ++q) d.replay(tasks[idx].path[q], s, lane);
                        d.base = T.depth;
                        busy = true;
                        iter = 0;
                        if (use_memo && T.depth > 0) {           // root state known to fail
                            const MemoKey k = d.key(g, s, lane);
                            uint64_t c = 0;
                            if (exact ? (k.ok && memo.xlookup(k, g, &c)) : (k.ok && memo.lookup(k))) {
                                t_status[idx] = QSMD_STATUS_NONLINEARISABLE;
                                t_nodes[idx] = c;                // exact: the subtree's count
                                busy = false;
                            }
                        }
                    }
                }
            }
        }
        if (busy) {
            int st = exact ? d.template step<2>(s, lane, limit, memo, g)
                     : use_memo ? d.template step<1>(s, lane, limit, memo, g)
                                : d.template step<0>(s, lane, limit, memo, g);
            if (st < 0 && ((++iter & 1023u) == 0u)) {
                const uint32_t mw = __hip_atomic_load(&p.giants[g].min_win, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
                if (local > mw || beyond_first_fail(a, h)) st = QSMD_STATUS_SKIPPED;
                else if (sp_time_up(a, t0, iter)) {
                    atomicOr(a.timed_out, 1u);
                    st = QSMD_STATUS_BUDGET;
                }
            }
            if (st >= 0) {
                t_status[idx] = (uint8_t)st;
                t_nodes[idx] = st == QSMD_STATUS_SKIPPED ? 0ull : d.nodes;
                if (st == QSMD_STATUS_LINEARISABLE || st == QSMD_STATUS_MODEL_ERROR)
                    atomicMin(&p.giants[g].min_win, local);
                if (t_wit && st == QSMD_STATUS_LINEARISABLE)
                    d.path_to(t_wit + (uint64_t)idx * kTaskWitness, kTaskWitness, s, lane);
                busy = false;
            }
        }
    }
    return taken;
}

// ----------------------------------------------------------------- combine

// Fold giant g's tasks into its history's outputs; returns the status.
// stale: a phase wait of this workgroup gave up (wait_for's safety net), so
// the giant's frontier record or task results may be unfinished: BUDGET.
[[maybe_unused]] __device__ int combine_one(const SplitArgs& p, uint32_t g, uint64_t& nodes, bool stale) {
    const SearchArgs& a = p.s;
    const uint32_t h = p.giant_list[g];
    nodes = 0;
    if (stale) {
        a.status[h] = QSMD_STATUS_BUDGET;
        if (a.nodes) a.nodes[h] = a.max_nodes;
        nodes = a.max_nodes;
        return QSMD_STATUS_BUDGET;
    }
    const GiantRec G = p.giants[g];
    const uint64_t base = (uint64_t)G.variant * p.task_cap + G.first;
    int64_t win = -1;
    const int st = combine_tasks(G.term_status, G.term_nodes, p.tasks + base, p.task_status + base,
                                 p.task_nodes + base, G.n_tasks, a.max_nodes, &nodes, &win);
    note_failure(a, h, st);
    a.status[h] = (uint8_t)st;
    if (a.nodes) a.nodes[h] = nodes;
    if (a.witness && win >= 0 && st == QSMD_STATUS_LINEARISABLE) {
        const uint8_t* row = p.task_witness + (base + (uint64_t)win) * kTaskWitness;
        const qsmd_hdr H = a.hdr[h];
        for (uint32_t q = 0; q < H.n_ev && q < kTaskWitness; ++q) {
            a.witness[H.ev_off + q] = row[q];
            if (row[q] == QSMD_WITNESS_END) break;
        }
    }
    return st;
}

// ------------------------------------------------------- phase hand-offs

// After this workgroup's stores: add v to a phase counter (release).
__device__ __forceinline__ void publish_add(uint32_t* ctr, uint32_t v, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (lane == 0 && v) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(ctr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// A poll of a counter other workgroups update: a global (not flat) sc1
// load, which bypasses this CU's L1 (a flat load may be served by a stale
// L1 line, e.g. the counters' line read at kernel start, and spin forever).
__device__ __forceinline__ uint32_t poll_u32(const uint32_t* c) {
    using gptr = const __attribute__((address_space(1))) uint32_t*;
    return __hip_atomic_load((gptr)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until a phase counter reaches target (acquire).  A safety net bounds
// the wait by twice the call's time limit (a stuck phase then reports
// through timed_out instead of holding the GPU); returns true when it gave
// up -- the phase before may still be running in another workgroup (one
// that started late), so what this workgroup combines afterwards is BUDGET.
__device__ __forceinline__ bool wait_for(const uint32_t* ctr, uint32_t target, const SearchArgs& a, uint64_t t0) {
    uint32_t polls = 0;
    bool gave_up = false;
    while (poll_u32(ctr) < target) {
        __builtin_amdgcn_s_sleep(8);
        if ((++polls & 63u) == 0u) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // (and the L1 refreshed now and then)
            if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > 2 * a.time_limit) {
                atomicOr(a.timed_out, 2u);
                gave_up = true;
                break;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    return gave_up;
}

__device__ __forceinline__ uint32_t ld_cnt(const uint32_t* c) { return poll_u32(c); }

// The call's last act: totals from the buckets, the probe snapshot for the
// host, every counter and bucket restored for the next call.
__device__ __forceinline__ void finish_call(const SplitArgs& p, int lane) {
    unsigned long long* bk = p.s.buckets;
    unsigned long long* xb = bk + (size_t)kBuckets * kBucketWords;   // early-exit recount
    const unsigned long long* src = p.early ? xb : bk;
    uint64_t v[T_N];
#pragma unroll
    for (int k = 0; k < T_N; ++k) v[k] = lane < (int)kBuckets ? src[(uint64_t)lane * kBucketWords + k] : 0ull;
#pragma unroll
    for (int k = 0; k < T_N; ++k) v[k] = wave_sum64(v[k]);
    if (p.totals && lane < T_N) {
        uint64_t t = 0;
#pragma unroll
        for (int k = 0; k < T_N; ++k) t = lane == k ? v[k] : t;
        reinterpret_cast<unsigned long long*>(p.totals)[lane] = t;
    }
    // (stage 0's heavy and deferred lists: the sums of their shard counters)
    const uint64_t heavy32 = wave_sum64(p.shards && lane < (int)kShards ? p.shards[lane * kShardStride] : 0u);
    const uint64_t defer = wave_sum64(p.shards && lane < (int)kShards ? p.shards[lane * kShardStride + kDeferShardWord]
                                                                        : 0u);
    if (p.probe_host && lane <= (int)C_TIMED)
        p.probe_host[lane] = !p.shards ? p.cnt[lane]
                           : lane == (int)C_HEAVY32 ? (uint32_t)heavy32
                           : lane == (int)C_DEFER   ? (uint32_t)defer + p.cnt[C_DEFER]
                                                    : p.cnt[lane];
    if (p.probe_host && lane == kProbeWide) p.probe_host[kProbeWide] = p.cnt[C_WIDE];
    if (p.probe_host && lane == kProbeBudget) p.probe_host[kProbeBudget] = p.probe_budget;
    if (p.probe_host && lane == kProbeN) p.probe_host[kProbeN] = (uint32_t)p.s.n_hist;
    if (p.probe_host && lane == kProbeTail) p.probe_host[kProbeTail] = p.cnt[C_TAIL];
    if (p.probe_host && lane == kProbeWritten) p.probe_host[kProbeWritten] = 1u;
    // restore: buckets (and the early-exit ones), then the counters
    for (uint32_t i = (uint32_t)lane; i < kBuckets * kBucketWords; i += 64u) {
        bk[i] = 0ull;
        if (p.early) xb[i] = 0ull;
    }
    if (lane < (int)C_N) p.cnt[lane] = lane == (int)C_FIRST_FAIL ? 0xFFFFFFFFu : 0u;
    if (p.shards && lane < (int)kShards) {
        p.shards[lane * kShardStride] = 0u;
        p.shards[lane * kShardStride + kDeferShardWord] = 0u;
    }
}

}  // namespace

// ------------------------------------------------------------------ kernels

namespace {
template <uint32_t MODEL>
struct GiantLds {
    union {
        GLds<MODEL, uint64_t, 64, 8, 64> v0;
        GLds<MODEL, M128, 128, 128, 16> v1;
    };
};
}  // namespace

__device__ __forceinline__ void beat(const SplitArgs& p, int lane, uint32_t k, uint32_t v) {
    if (p.debug && lane == 0)
        __hip_atomic_store(p.debug + (uint64_t)blockIdx.x * 4 + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The frontier, task and combine phases (n_g > 0 giants).
template <uint32_t MODEL>
__device__ __forceinline__ void giant_phases(const SplitArgs& p, uint32_t n_g, GiantLds<MODEL>& u, uint64_t t0) {
    const SearchArgs& a = p.s;
    const int lane = threadIdx.x;
    uint32_t* cnt = p.cnt;
    // ---- frontier: chunks of 64 giants; variant 0 on all lanes, then variant
    // 1 in four rounds of 16 lanes
    for (;;) {
        uint32_t c0 = 0;
        if (lane == 0) c0 = atomicAdd(cnt + C_GNEXT, 64u);
        c0 = __shfl(c0, 0, 64);
        if (c0 >= n_g) break;
        if (p.stall_ticks && c0 == 0u) {        // diagnostic: the first chunk's workgroup starts late
            while (__builtin_amdgcn_s_memrealtime() - t0 < p.stall_ticks) __builtin_amdgcn_s_sleep(127);
        }
        const uint32_t g = c0 + (uint32_t)lane;
        const bool in = g < n_g;
        uint32_t h = 0;
        qsmd_hdr H{0, 0, 0, 0, 0, 0};
        if (in) {
            h = p.giant_list[g];
            H = a.hdr[h];
        }
        const uint32_t var = variant_of(H);
        if (in && var == 0u) frontier_one<MODEL, uint64_t, 64, 8, 64>(p, g, h, H, 0u, u.v0, lane, t0);
        __syncthreads();
        for (uint32_t r = 0; r < 4u; ++r) {
            if (in && var == 1u && (uint32_t)lane / 16u == r)
                frontier_one<MODEL, M128, 128, 128, 16>(p, g, h, H, 1u, u.v1, lane & 15, t0);
            __syncthreads();
        }
        publish_add(cnt + C_GDONE, min(64u, n_g - c0), lane);
        beat(p, lane, 1, c0 + 1);
    }
    beat(p, lane, 0, 2);
    // ---- tasks (every frontier done: the task lists are complete)
    bool stale = wait_for(cnt + C_GDONE, n_g, a, t0);
    beat(p, lane, 0, 3);
    uint32_t took = task_loop<MODEL, uint64_t, 64, 8, 64>(p, 0u, u.v0, lane, t0, cnt + C_TQ0);
    __syncthreads();
    if (lane < 16) {
        const uint32_t t1 = task_loop<MODEL, M128, 128, 128, 16>(p, 1u, u.v1, lane, t0, cnt + C_TQ1);
        took += lane == 0 ? t1 : 0u;
    }
    took = __shfl(took, 0, 64);
    publish_add(cnt + C_TDONE, took, lane);
    beat(p, lane, 0, 4);
    beat(p, lane, 2, took);
    // ---- combine (every task done)
    const uint32_t n_tasks = min(ld_cnt(cnt + C_TASKS0), p.task_cap) + min(ld_cnt(cnt + C_TASKS1), p.task_cap);
    stale |= wait_for(cnt + C_TDONE, n_tasks, a, t0);
    beat(p, lane, 0, 5);
    Counters cc;
    for (;;) {
        uint32_t c0 = 0;
        if (lane == 0) c0 = atomicAdd(cnt + C_CNEXT, 64u);
        c0 = __shfl(c0, 0, 64);
        if (c0 >= n_g) break;
        const uint32_t g = c0 + (uint32_t)lane;
        if (g < n_g) {
            uint64_t nodes = 0;
            const int st = combine_one(p, g, nodes, stale);
            cc.add(st, nodes);
        }
        publish_add(cnt + C_CDONE, min(64u, n_g - c0), lane);
    }
    cc.flush(a.buckets, lane);
}

// The giant stage's work (a call with giants or the early exit): out of
// line, so that a call without giants -- nearly every call -- runs the
// kernel's short path alone (the functions below take the arguments by
// reference; from the kernel's own parameter that made a private copy of
// them, ~400 B per lane, at every launch)
template <uint32_t MODEL>
__device__ __noinline__ void giant_work(const SplitArgs& p, uint32_t n_g, GiantLds<MODEL>& u) {
    const SearchArgs& a = p.s;
    const int lane = threadIdx.x;
    uint32_t* cnt = p.cnt;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    beat(p, lane, 0, 1);
    // (no giant: an early-exit call goes straight to the fixup -- the giant
    // count is final here, every stage that appends ran before this launch,
    // and without a frontier there are no tasks; the phases' queue and
    // done-counter atomics in every workgroup cost ~60 us per call)
    if (n_g) giant_phases<MODEL>(p, n_g, u, t0);
    // ---- early exit: every history after the first failing one is SKIPPED,
    // and the totals are recounted from the final outputs
    if (p.early) {
        if (n_g) (void)wait_for(cnt + C_CDONE, n_g, a, t0);
        const uint32_t ff = ld_cnt(a.first_fail);
        Counters xc;
        uint64_t skipped = 0;
        constexpr uint32_t kChunk = kFixupChunk;
        uint8_t* const st_out = a.status;
        uint64_t* const nd_out = a.nodes;
        const uint64_t n_hist = a.n_hist;
        for (;;) {
            uint32_t c0 = 0;
            if (lane == 0) c0 = atomicAdd(cnt + C_XNEXT, 1u);
            const uint64_t b0 = (uint64_t)__shfl(c0, 0, 64) * kChunk;
            if (b0 >= n_hist) break;
            // the histories up to the first failure counted (loads only),
            // then the rest marked (stores only), the pointers and bounds
            // in registers: a byte store may alias the argument block the
            // loop read them from, and vmcnt counts stores too, so each
            // reload waited for the row's stores (a 4096-history chunk ~33 us)
            const uint64_t e0 = min(n_hist, b0 + kChunk);
            const uint64_t keep = min(e0, (uint64_t)ff + 1u);
            for (uint64_t hh = b0 + (uint64_t)lane; hh < keep; hh += 64) xc.add(st_out[hh], nd_out ? nd_out[hh] : 0ull);
            for (uint64_t hh = max(b0, keep) + (uint64_t)lane; hh < e0; hh += 64) {
                st_out[hh] = QSMD_STATUS_SKIPPED;
                if (nd_out) nd_out[hh] = 0;
                ++skipped;
            }
        }
        xc.flush(a.buckets + (size_t)kBuckets * kBucketWords, lane);
        const uint64_t sk = wave_sum64(skipped);
        bucket_add(a.buckets + (size_t)kBuckets * kBucketWords, blockIdx.x, T_SKIPPED, lane == 0 ? sk : 0ull);
    }
    beat(p, lane, 0, 6);
    // ---- the last workgroup out finishes the call
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t last = 0;
    if (lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicAdd(cnt + C_EXIT, 1u) == gridDim.x - 1u;
    }
    if (__shfl(last, 0, 64)) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        finish_call(p, lane);
    }
}


}  // namespace qsmd
