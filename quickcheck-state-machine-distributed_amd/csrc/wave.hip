// wave.hip -- the heavy stage in wave mode: one wavefront per history, the
// DFS in wave-uniform (scalar) registers.
//
// The heavy histories are the few whose search exceeds the compact stages'
// node budget (config 2: ~1200 of 1M, 40..320 reference nodes each).  In
// lane mode (csrc/memo.hip) a lane runs one of them, and every DFS step is
// a chain of dependent LDS round trips (the candidate's event, its response,
// the balances, the memo probe) that a lone wavefront cannot hide: ~2900
// cycles per step, so the list's longest search sets the stage's time.
// Here the whole wavefront owns one history and nothing on the DFS chain
// touches memory:
//   * event e of the history sits in lane e (e - 64: a second register) of
//     two VGPRs, its lo word and its value, read at a wave-uniform index with
//     v_readlane (an SGPR result);
//   * Bank balances sit in lanes 0..7 of a VGPR (v_readlane / v_writelane at
//     the account index), the DFS stack and the per-level node counts in lane
//     d of two more VGPRs; event masks, the remaining-event set, the model's
//     small parts and the node count are scalars;
//   * so a candidate try (src/Linearisability.hs:25-69 at one node:
//     takeInvocations, findResponse, filter1, postcondition, transition) is
//     straight scalar code, ~10x shorter than the lane-mode step's memory
//     chain.
// The state memo (north star (c)) is exact-count, as in lane mode: a state
// S = (remaining events, model) is recorded with the nodes its subtree
// counted when the search leaves it (it failed: the search goes on), and a
// later entry into S adds that count and backtracks (memo.hip explains why
// verdict, count and witness stay the reference's).  With QSMD_FLAG_MEMO
// (explored-node counts) a hit adds nothing and every state is recorded.
// The table is the wavefront's own, in LDS: buckets of 64 words, one word
// per lane, holding 8 entries of 8 words (<= 64 events) or 4 of 16 (<= 128),
// so a probe is ONE ds_read_b32 across the wavefront and a ballot of the 64
// word compares finds a matching entry.  Entries carry a per-history epoch:
// nothing is cleared between histories.
//
// Three lists, one launch: the heavy lists of stages 0 and 0w (<= 32 and
// <= 64 events) and the histories stage 0w deferred (beyond 64 events, or
// values beyond the compact encoding): those with <= 128 events, <= 8 pids
// and values within 2^24 (no i32 overflow in any balance) run here with
// 128-bit masks, the rest go to the giant stage, as does every search past
// its iteration cap (the split stage searches it again from the root).
// Lane mode keeps the long heavy lists (config 3: ~285k heavy histories,
// where 64 searches per wavefront instruction win); the host picks by the
// last call's heavy count (api.hip, heavy_mode 2).
#include <hip/hip_runtime.h>

#include "internal.h"
#include "lane.h"
#include "mask.h"

namespace qsmd {

namespace {

constexpr uint32_t kEpochMax = 0xFFFFFFu;    // 24-bit entry tags (word 2 = ex | epoch << 8)
constexpr int32_t kWideValue = 1 << 24;      // wide-list values (and model0) within +-2^24: no i32 overflow

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int32_t rli(int32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
// (a lane write as a compare + select on the lane id: hipcc emits v_writelane)
__device__ __forceinline__ uint32_t wl(uint32_t v, uint32_t x, uint32_t l) { return threadIdx.x == l ? x : v; }
__device__ __forceinline__ int32_t wli(int32_t v, int32_t x, uint32_t l) { return threadIdx.x == l ? x : v; }

// ---- scalar event-mask helpers: u64 (<= 64 events) and M128 (<= 128)
__device__ __forceinline__ bool mnz(uint64_t m) { return m != 0ull; }
__device__ __forceinline__ bool mnz(const M128& m) { return (m.lo | m.hi) != 0ull; }
__device__ __forceinline__ uint32_t mctz(uint64_t m) { return (uint32_t)__builtin_ctzll(m); }
__device__ __forceinline__ uint32_t mctz(const M128& m) {
    return m.lo ? (uint32_t)__builtin_ctzll(m.lo) : 64u + (uint32_t)__builtin_ctzll(m.hi);
}
__device__ __forceinline__ uint32_t mhibit(uint64_t m) { return 63u - (uint32_t)__builtin_clzll(m); }
__device__ __forceinline__ uint32_t mhibit(const M128& m) {
    return m.hi ? 127u - (uint32_t)__builtin_clzll(m.hi) : 63u - (uint32_t)__builtin_clzll(m.lo);
}
__device__ __forceinline__ uint32_t mpop(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }
__device__ __forceinline__ uint32_t mpop(const M128& m) {
    return (uint32_t)(__builtin_popcountll(m.lo) + __builtin_popcountll(m.hi));
}
template <typename M> __device__ __forceinline__ M mbit(uint32_t j);
template <> __device__ __forceinline__ uint64_t mbit<uint64_t>(uint32_t j) { return 1ull << j; }
template <> __device__ __forceinline__ M128 mbit<M128>(uint32_t j) {
    return mk128(j < 64u ? 1ull << (j & 63u) : 0ull, j < 64u ? 0ull : 1ull << (j & 63u));
}
__device__ __forceinline__ uint64_t mlowest(uint64_t m) { return m & (0ull - m); }
// per-lane select, word by word (a select of whole M128 objects goes through scratch)
__device__ __forceinline__ uint64_t msel(bool c, uint64_t a, uint64_t b) { return c ? a : b; }
__device__ __forceinline__ M128 msel(bool c, const M128& a, const M128& b) {
    return mk128(c ? a.lo : b.lo, c ? a.hi : b.hi);
}
__device__ __forceinline__ M128 mlowest(const M128& m) { return MaskOps<M128>::lowest(m); }
// the bits above j
__device__ __forceinline__ uint64_t mabove(uint32_t j, uint64_t) { return ~1ull << j; }
__device__ __forceinline__ M128 mabove(uint32_t j, const M128&) { return ~MaskOps<M128>::below((int)j + 1); }
// takeInvocations (src/Linearisability.hs:25-28): remaining invocations
// below the lowest remaining response
__device__ __forceinline__ uint64_t mcands(uint64_t rem, uint64_t INV, uint64_t RESP) {
    const uint64_t rr = rem & RESP;
    return rem & INV & ((rr & (0ull - rr)) - 1ull);
}
__device__ __forceinline__ M128 mcands(const M128& rem, const M128& INV, const M128& RESP) {
    const M128 rr = rem & RESP;
    return rem & INV & MaskOps<M128>::below(mnz(rr) ? (int)mctz(rr) : 128);
}

template <typename M> struct Geo;
template <> struct Geo<uint64_t> { static constexpr uint32_t NW = 1, EW = 8; };     // events / 64, entry words
template <> struct Geo<M128> { static constexpr uint32_t NW = 2, EW = 16; };

// The reference DFS of one history, wave-uniform (every member is a scalar;
// the per-event / per-account / per-level arrays are lanes of VGPRs).
template <uint32_t MODEL, typename M>
struct WaveDFS {
    static constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    static constexpr uint32_t NW = Geo<M>::NW, EW = Geo<M>::EW;
    M INV, RESP;
    M rem, cand;
    uint64_t nodes;
    uint64_t RS;            // Ticket: levels whose operation was a Reset
    uint32_t depth, ex, neg, found;
    // Bank, for the memo key (kept as the balances change): wacc = accounts
    // whose balance is beyond i16, mh = XOR of per-account hashes
    uint32_t wacc, mh;
    // lanes: lo / val / pidv = event e (lane e % 64 of word e / 64; pidv =
    // its pid, 0xFF past the history), bal = account q (lane q), kb = the
    // balances as i16 pairs in the memo key's lane layout (lane l with
    // l % EW = 4 + q holds accounts 2q, 2q + 1), stk = the undo record of
    // level d (lane d: j | ex_a << 7 | ex_b << 8), ent = the node count at
    // entry of level d (lane d)
    uint32_t lo[NW], pidv[NW];
    int32_t val[NW];
    int32_t bal;
    uint32_t kb;
    uint32_t stk, ent;

    __device__ static __forceinline__ uint32_t acc_hash(uint32_t c, int32_t v) {
        return ((uint32_t)v * 0x9E3779B1u) ^ ((c + 1u) * 0x85EBCA77u) ^ ((uint32_t)v >> 7);
    }
    // account c := v (old: its balance before), the key parts with it
    __device__ __forceinline__ void set_bal(uint32_t c, int32_t old, int32_t v) {
        bal = wli(bal, v, c);
        const uint32_t w = threadIdx.x % EW, sh = (c & 1u) * 16u;
        const uint32_t keep = 0xFFFF0000u >> sh;
        kb = w == 4u + (c >> 1) ? (kb & keep) | (((uint32_t)v & 0xFFFFu) << sh) : kb;
        const bool fits = v == (int32_t)(int16_t)v;
        wacc = (wacc & ~(1u << c)) | (fits ? 0u : 1u << c);
        mh ^= acc_hash(c, old) ^ acc_hash(c, v);
    }

    __device__ __forceinline__ uint32_t ev_lo(uint32_t e) const {
        if constexpr (NW == 1) {
            return rl(lo[0], e);
        } else {
            const uint32_t x0 = rl(lo[0], e & 63u), x1 = rl(lo[1], e & 63u);
            return e < 64u ? x0 : x1;
        }
    }
    __device__ __forceinline__ int32_t ev_val(uint32_t e) const {
        if constexpr (NW == 1) {
            return rli(val[0], e);
        } else {
            const int32_t x0 = rli(val[0], e & 63u), x1 = rli(val[1], e & 63u);
            return e < 64u ? x0 : x1;
        }
    }
    // the events of the pid of event j: one lane compare per event register
    __device__ __forceinline__ M same_pid(uint32_t j) const {
        const uint32_t p = ev_lo(j) & 0x7Fu;
        if constexpr (NW == 1) return __ballot(pidv[0] == p);
        else return mk128(__ballot(pidv[0] == p), __ballot(pidv[1] == p));
    }

    // Undo the last level exactly (remaining events, model); returns its candidate.
    __device__ __forceinline__ uint32_t undo() {
        --depth;
        const uint32_t st = rl(stk, depth);
        const uint32_t j = st & 127u;
        const M gone = ~rem & same_pid(j);
        rem |= mbit<M>(mhibit(gone & INV)) | mbit<M>(mhibit(gone & RESP));
        if constexpr (BANK) {
            const uint32_t lj = ev_lo(j);
            const int32_t m = ev_val(j);
            const uint32_t code = (lj >> 8) & 0xFFu, ia = (lj >> 16) & 7u, ib = (lj >> 24) & 7u;
            const uint32_t pa = (st >> 7) & 1u, pb = (st >> 8) & 1u;
            const bool tr = code == QSMD_BANK_TRANSFER;
            const int32_t ba = rli(bal, ia), bb = rli(bal, ib);
            const int32_t rb = (pb || ia == ib) ? bb - m : 0;      // Transfer's deposit on b undone
            const int32_t cur_a = (tr && ia == ib) ? rb : ba;
            const int32_t ra = pa ? cur_a - bank_sign(code) * m : 0;
            if (tr) set_bal(ib, bb, rb);                           // (Transfer only)
            set_bal(ia, (tr && ia == ib) ? rb : ba, ra);           // last (ia == ib)
            ex = (ex & ~((1u << ia) | ((tr ? 1u : 0u) << ib))) | (pa << ia) | ((tr ? pb : 0u) << ib);
            neg = 0u;   // the parent held the invariant (a step descends only then)
        } else {
            RS &= ~(1ull << depth);
        }
        return j;
    }

    // Ticket model at the current depth: Just (#TT since the last Reset), or
    // model0 advanced by succ <$> once per level
    __device__ __forceinline__ void ticket_model(const SearchArgs& a, uint32_t& just, int32_t& n) const {
        just = RS ? 1u : a.m0_just;
        n = RS ? (int32_t)(depth - 1u - (63u - (uint32_t)__builtin_clzll(RS | 1ull)))
               : (int32_t)a.m0_val[0] + (a.m0_just ? (int32_t)depth : 0);
    }

    // Try the next candidate of the current node (LaneDFS::try_next, scalar):
    // -1 to go on, or QSMD_STATUS_BUDGET / QSMD_STATUS_MODEL_ERROR.
    __device__ __forceinline__ int try_next(const SearchArgs& a, uint64_t limit) {
        const uint32_t j = mctz(cand);
        cand &= ~mbit<M>(j);
        const M pm = same_pid(j);
        const M rr = rem & pm & RESP;
        const bool has = mnz(rr);                                  // findResponse => [] : no child
        const uint32_t r = has ? mctz(rr) : j;
        const uint32_t lj = ev_lo(j), lr = ev_lo(r);
        const int32_t m = ev_val(j), rv = ev_val(r);
        const uint32_t code = (lj >> 8) & 0xFFu, rc = (lr >> 8) & 0xFFu;
        const bool over = has && nodes >= limit;
        bool ok, err = false;
        uint32_t stw = j;
        if constexpr (BANK) {
            const uint32_t ia = (lj >> 16) & 7u, ib = (lj >> 24) & 7u;
            const int32_t bal_a = rli(bal, ia), bal_b = rli(bal, ib);
            const uint32_t ex_a = (ex >> ia) & 1u, ex_b = (ex >> ib) & 1u;
            // post (test/Bank.hs:118-131): invariant && the expected response
            const bool tr = code == QSMD_BANK_TRANSFER, chk = code == QSMD_BANK_CHECK_BALANCE;
            const bool same = ia == ib;
            const uint32_t sel = (code == QSMD_BANK_OPEN_ACCOUNT || bal_a >= m) ? ex_a : 0u;
            const uint32_t exp = (kBankExp2 >> (code * 6u + sel * 3u)) & 7u;
            const bool inv_ok = neg == 0u;
            err = has && inv_ok && chk && rc == QSMD_BANK_BALANCE && !ex_a;   // Map.! raises
            ok = has && !over && inv_ok && !err && rc == exp && (!chk || rv == bal_a);
            stw = j | (ex_a << 7) | (ex_b << 8);
            if (ok) {
                // next' (test/Bank.hs:92-101): insertWith on a, then Transfer's deposit on b
                const int32_t sa = bank_sign(code);
                const int32_t na = (ex_a ? bal_a : 0) + (ex_a ? sa : (sa & 1)) * m;
                const int32_t bo = same ? na : bal_b;
                const int32_t fb = tr ? (((ex_b != 0u) || same) ? bo : 0) + m : bo;
                set_bal(ia, bal_a, na);
                if (tr) set_bal(ib, same ? na : bal_b, fb);
                const int32_t va = same ? fb : na;
                ex |= ((chk ? 0u : 1u) << ia) | ((tr ? 1u : 0u) << ib);
                neg = (va | fb) < 0 ? 1u : 0u;
            }
        } else {
            // TicketDispenser (test/TicketDispenser.hs:81-102)
            uint32_t just;
            int32_t tn;
            ticket_model(a, just, tn);
            const bool tt = code == QSMD_TICKET_TAKE_TICKET;
            ok = has && !over && (tt ? (rc == QSMD_TICKET_NUMBER && just != 0u && rv == tn + 1)
                                     : rc == QSMD_TICKET_OK);
            if (ok && !tt) RS |= 1ull << depth;
        }
        const bool counted = has && !over;
        nodes += counted ? 1u : 0u;
        found |= counted ? 1u : 0u;
        if (ok) {
            stk = wl(stk, stw, depth);
            ++depth;
            const M fi = rem & pm & INV;                           // filter1: the pid's first invocation
            rem &= ~(mlowest(fi) | mbit<M>(r));
            cand = mcands(rem, INV, RESP);
            found = 0u;
        }
        return over ? QSMD_STATUS_BUDGET : (err ? QSMD_STATUS_MODEL_ERROR : -1);
    }
};

// The memo key of the current state in lane layout: lane l holds word l % EW
// of an entry: 0, 1 rem bits 0-63, 2 ex | epoch << 8, 3 count, 4..7 model
// (Bank balances as i16 pairs, Ticket just | n << 1), and for 128-bit masks
// 8, 9 rem bits 64-127 (10..15 zero).  `ok` false when the state does not
// fit (a balance beyond i16): not recorded, not looked up.
struct WKey {
    uint32_t vec;       // this lane's word
    uint32_t bucket;
    bool ok;
};

template <uint32_t MODEL, typename M>
__device__ __forceinline__ WKey wave_key(const WaveDFS<MODEL, M>& d, const SearchArgs& a, uint32_t epoch,
                                         uint32_t bucket_mask, int lane) {
    constexpr uint32_t EW = Geo<M>::EW;
    bool ok = true;
    uint32_t mw, mhash;                           // the model: lanes 4..7 (Bank: d.kb), its hash
    if constexpr (MODEL == QSMD_MODEL_BANK) {
        ok = d.wacc == 0u;
        mw = d.kb;
        mhash = d.mh;
    } else {
        uint32_t just;
        int32_t n;
        d.ticket_model(a, just, n);
        const uint32_t m0 = just | (just ? (uint32_t)n << 1 : 0u);
        mw = ((uint32_t)lane % EW) == 4u ? m0 : 0u;
        mhash = m0 * 0x9E3779B1u;
    }
    uint32_t r0, r1, r2 = 0u, r3 = 0u;
    if constexpr (Geo<M>::NW == 1) {
        r0 = (uint32_t)d.rem;
        r1 = (uint32_t)(d.rem >> 32);
    } else {
        r0 = (uint32_t)d.rem.lo;
        r1 = (uint32_t)(d.rem.lo >> 32);
        r2 = (uint32_t)d.rem.hi;
        r3 = (uint32_t)(d.rem.hi >> 32);
    }
    const uint32_t w2 = (MODEL == QSMD_MODEL_BANK ? d.ex : 0u) | (epoch << 8);
    uint32_t hsh = (r0 * 0x9E3779B1u) ^ ((r1 ^ w2) * 0x85EBCA77u) ^ mhash ^ ((r2 ^ (r3 << 16 | r3 >> 16)) * 0x27D4EB2Fu);
    hsh ^= (hsh >> 16) ^ (hsh >> 24);
    const uint32_t w = (uint32_t)lane % EW;
    uint32_t x = w == 0u ? r0 : (w == 1u ? r1 : (w == 2u ? w2 : 0u));
    x = (w >= 4u && w < 8u) ? mw : x;
    if constexpr (EW == 16) {
        x = w == 8u ? r2 : x;
        x = w == 9u ? r3 : x;
    }
    return WKey{x, hsh & bucket_mask, ok};
}

// One probe: the bucket's entries (one word per lane); the count of the
// matching entry, if any.  Group g of EW bits of the ballot = entry g.
template <uint32_t EW>
__device__ __forceinline__ bool wave_lookup(const uint32_t* tab, const WKey& k, int lane, uint32_t& count) {
    constexpr uint64_t ONES = EW == 8 ? 0x0101010101010101ull : 0x0001000100010001ull;
    constexpr uint64_t HIGH = ONES << (EW - 1u);
    const uint32_t w = tab[k.bucket * 64u + (uint32_t)lane];
    const uint64_t eq = __ballot(w == k.vec) | (ONES << 3);   // word 3 (the count) is not compared
    const uint64_t z = ~eq;                                    // a zero group: every word matched
    const uint64_t t = (z - ONES) & ~z & HIGH;
    if (t == 0ull) return false;
    const uint32_t e = (uint32_t)__builtin_ctzll(t) / EW;      // the lowest flagged group is exact
    count = rl(w, e * EW + 3u);
    return true;
}

template <uint32_t EW>
__device__ __forceinline__ void wave_insert(uint32_t* tab, const WKey& k, uint32_t count, uint32_t victim,
                                            int lane) {
    if (((uint32_t)lane / EW) == (victim % (64u / EW)))
        tab[k.bucket * 64u + (uint32_t)lane] = ((uint32_t)lane % EW) == 3u ? count : k.vec;
}

// ---------------------------------------------------------------- state DAG
// The subtree below a node is a function of its state S = (remaining events,
// model) (Lemma L1), so the reference's search tree folds into a DAG of
// states: level d holds the states after d operations (popcount(rem) = n_ev -
// 2d, so an edge always goes one level down and equal states meet only within
// a level).  The wavefront builds it level by level -- a level's states in
// lanes, then its (state, candidate) items in lanes: findResponse, filter1,
// postcondition, transition; the children deduplicated by full-key compare --
// and folds it back from the deepest level:
//   g(S) = over S's children in candidate order: +1 node each (the step
//          call); a raising postcondition decides (MODEL_ERROR); a True one
//          adds the child's count and decides when g(child) does (True or
//          raise); no child at all: True (any' []), or False at the root (any).
// That is exactly the DFS's accumulation (src/Linearisability.hs:59-69): the
// node count, verdict and -- by following the deciding child from the root --
// the witness are the reference's, with every state evaluated once.  With
// QSMD_FLAG_MEMO the count is the explored-node count of the DFS that prunes
// known-failing states (oracle/ref_cpu.c): the decision path's evaluated
// children plus, once each, every state below a failed earlier sibling.
// Histories whose DAG does not fit (a level wider than 64 states or items,
// more than the capacity in states or items) run the DFS below instead.
enum : uint32_t { G_F = 0u, G_T = 1u, G_ERR = 2u, G_SAT = 4u, G_MARK = 8u };

template <typename M> struct DagGeo;
template <> struct DagGeo<uint64_t> { static constexpr uint32_t NM = 2; };
template <> struct DagGeo<M128> { static constexpr uint32_t NM = 4; };

__device__ __forceinline__ void mwords(uint64_t m, uint32_t* w) {
    w[0] = (uint32_t)m;
    w[1] = (uint32_t)(m >> 32);
}
__device__ __forceinline__ void mwords(const M128& m, uint32_t* w) {
    w[0] = (uint32_t)m.lo;
    w[1] = (uint32_t)(m.lo >> 32);
    w[2] = (uint32_t)m.hi;
    w[3] = (uint32_t)(m.hi >> 32);
}
template <typename M> __device__ __forceinline__ M mfrom(const uint32_t* w);
template <> __device__ __forceinline__ uint64_t mfrom<uint64_t>(const uint32_t* w) {
    return w[0] | (uint64_t)w[1] << 32;
}
template <> __device__ __forceinline__ M128 mfrom<M128>(const uint32_t* w) {
    return mk128(w[0] | (uint64_t)w[1] << 32, w[2] | (uint64_t)w[3] << 32);
}

// The wavefront's DAG arrays in LDS (the keys stay in lanes).
constexpr uint32_t kDagSlots = 1024;   // dedup table: a level's children by key hash
struct DagLds {
    uint32_t* sitem;   // [SC]: first item | item count << 16
    uint32_t* glo;     // [SC]: g count, low / high word
    uint32_t* ghi;
    uint32_t* gfl;     // [SC]: g result | G_SAT | G_MARK
    uint32_t* item;    // [IC]: child | post << 12 | j << 14 (child 0xFFF: none)
    uint32_t* evlo;    // [128]: event lo words
    int32_t* evval;    // [128]: event values
    uint32_t* tab;     // [kDagSlots]: lowest lane holding a child of that hash slot (~0u: none)
    uint32_t* path;    // [128]: the deciding path's candidate per depth
};

template <uint32_t MODEL, typename M>
struct DagKey {
    static constexpr uint32_t NM = DagGeo<M>::NM;
    static constexpr uint32_t MWD = MODEL == QSMD_MODEL_BANK ? 9u : 2u;
    static constexpr uint32_t KW = NM + MWD;   // key words: rem, then the model (Bank: ex, 8 balances; Ticket: just, n)
};

template <uint32_t MODEL, typename M>
__host__ __device__ constexpr size_t dag_lds_bytes(uint32_t SC, uint32_t IC) {
    return (size_t)SC * 16u + (size_t)IC * 4u + 128u * 8u + kDagSlots * 4u + 128u * 4u;
}

template <uint32_t MODEL, typename M>
__device__ __forceinline__ DagLds dag_carve(uint32_t* base, uint32_t SC, uint32_t IC) {
    DagLds L;
    L.sitem = base;
    L.glo = L.sitem + SC;
    L.ghi = L.glo + SC;
    L.gfl = L.ghi + SC;
    L.item = L.gfl + SC;
    L.evlo = L.item + IC;
    L.evval = reinterpret_cast<int32_t*>(L.evlo + 128);
    L.tab = reinterpret_cast<uint32_t*>(L.evval + 128);
    L.path = L.tab + kDagSlots;
    return L;
}


// A key's 32-bit hash: independent products folded together (a short chain)
template <uint32_t KW>
__device__ __forceinline__ uint32_t dag_hash(const uint32_t* kw, uint32_t used) {
    constexpr uint32_t C[4] = {0x9E3779B1u, 0x85EBCA77u, 0xC2B2AE3Du, 0x27D4EB2Fu};
    uint32_t h[4] = {0x165667B1u, 0xD3A2646Cu, 0xFD7046C5u, 0xB55A4F09u};
#pragma unroll
    for (uint32_t k = 0; k < KW; ++k)
        if (k < used) h[k & 3u] ^= __builtin_rotateleft32(kw[k] * C[k & 3u], 5u * k);
    uint32_t x = (h[0] ^ h[1]) + (h[2] ^ h[3]);
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    return x;
}

// The DAG search of the staged history (d: events in lanes, INV / RESP);
// QSMD_STATUS_* or -1 when the DAG does not fit.  Witness path in L.path.
template <uint32_t MODEL, typename M>
__device__ int dag_history(const WaveArgs& p, const SearchArgs& a, const WaveDFS<MODEL, M>& d, uint32_t n_ev,
                           uint32_t n_pid, const DagLds& L, uint32_t SC, uint32_t IC, int lane, uint64_t& nodes_out,
                           uint32_t& path_len) {
    using K = DagKey<MODEL, M>;
    constexpr uint32_t NM = K::NM, KW = K::KW;
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    const uint32_t ul = (uint32_t)lane;
    // events into LDS, the per-pid invocation / response masks (scalars)
#pragma unroll
    for (uint32_t w = 0; w < Geo<M>::NW; ++w) {
        const uint32_t e = ul + 64u * w;
        if (e < n_ev) {
            L.evlo[e] = d.lo[w];
            L.evval[e] = d.val[w];
        }
    }
    for (uint32_t i = ul; i < kDagSlots; i += 64u) L.tab[i] = ~0u;
    // the events of pid q: one lane compare per event register (a ballot,
    // recomputed where needed: the masks of 8 pids would not stay in SGPRs;
    // called in uniform control flow only, every lane active)
    auto pid_ev = [&](uint32_t q) -> M {
        if constexpr (Geo<M>::NW == 1) return __ballot(d.pidv[0] == q);
        else return mk128(__ballot(d.pidv[0] == q), __ballot(d.pidv[1] == q));
    };
    // ---- forward: the levels.  A level's states live in lanes (SM: which
    // ones; kw: the key, sid: the state id); its items (one per candidate
    // with a response, in candidate order per state) in lanes 0..total-1;
    // the leaders of the children's dedup become the next level's state lanes
    uint32_t kw[KW];
    mwords(d.INV | d.RESP, kw);
    if constexpr (BANK) {
        kw[NM] = a.m0_exists;
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) kw[NM + 1 + q] = (uint32_t)(int32_t)a.m0_val[q];
    } else {
        kw[NM] = a.m0_just;
        kw[NM + 1] = (uint32_t)(int32_t)a.m0_val[0];
    }
    // Bank: the accounts the history (or model0) can touch; the balances of
    // the others stay 0 in every key, so the loops over key words stop at
    // `used` (wave-uniform)
    uint32_t n_acc = 8u, used = KW;
    if constexpr (BANK) {
        uint32_t touched = a.m0_exists;
#pragma unroll
        for (uint32_t w = 0; w < Geo<M>::NW; ++w) {
            const uint32_t lo = d.lo[w];
            const bool inv = d.pidv[w] != 0xFFu && !(lo & 0x80u);
            const uint32_t bits = inv ? (1u << ((lo >> 16) & 7u)) |
                                            (((lo >> 8) & 0xFFu) == QSMD_BANK_TRANSFER ? 1u << ((lo >> 24) & 7u) : 0u)
                                      : 0u;
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) touched |= __ballot((bits >> q) & 1u) ? 1u << q : 0u;
        }
        n_acc = touched ? 32u - (uint32_t)__builtin_clz(touched) : 1u;
        used = NM + 1u + n_acc;
    }
    // level boundaries in lanes: lane d of lv0 (d < 64) / lv1 (64 + d) = the first state of level d
    uint32_t lv0 = ul == 1u ? 1u : 0u, lv1 = 0u;
    uint64_t SM = 1ull;                                     // the root, in lane 0
    uint64_t leaf_or_err = 0ull;                            // a leaf below the root or a raising step seen
    uint32_t sid = 0u;
    uint32_t n_states = 1u, n_items = 0u, nlev = 1u;
    bool fit = true;
    const bool timing = p.stats != nullptr;
    uint64_t tph[5] = {0, 0, 0, 0, 0}, tprev = timing ? __builtin_amdgcn_s_memtime() : 0ull;
    auto tick = [&](int k) {
        if (timing) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            tph[k] += t - tprev;
            tprev = t;
        }
    };
    auto flush_stats = [&](uint32_t levels) {               // (the diagnostic counters, lane 0)
        tick(4);
        if (timing && ul == 0) {
#pragma unroll
            for (int k = 0; k < 5; ++k) atomicAdd(p.stats + 8 + k, (unsigned long long)tph[k]);
            atomicAdd(p.stats + 13, (unsigned long long)levels);
        }
    };
    while (true) {
        // state lanes: the candidates with a response (takeInvocations, findResponse)
        const bool sl = (SM >> ul) & 1ull;
        const M rem = mfrom<M>(kw);
        const M C = mcands(rem, d.INV, d.RESP);
        M V{};
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {              // (the ballots in uniform control flow)
            if (q >= n_pid) break;
            const M pq = pid_ev(q);
            V = msel(mnz(rem & pq & d.RESP), V | (C & pq), V);
        }
        V = msel(sl, V, M{});
        const uint32_t deg = mpop(V);
        // the items' offsets: a prefix sum of deg over the lanes, from ballots of its bits
        uint32_t excl = 0u, total = 0u;
        if (__builtin_popcountll(SM) == 1) {                // one state: its items start the level
            total = rl(deg, (uint32_t)__builtin_ctzll(SM));
        } else {
            for (uint32_t b = 0; b < 8; ++b) {
                const uint64_t bm = __ballot((deg >> b) != 0u);
                if (!bm) break;
                const uint64_t bb = __ballot((deg >> b) & 1u);
                excl += lane_prefix(bb) << b;
                total += (uint32_t)__builtin_popcountll(bb) << b;
            }
        }
        if (total > 64u || n_items + total > IC) { fit = false; break; }
        if (sl) L.sitem[sid] = (n_items + excl) | deg << 16;
        leaf_or_err |= __ballot(sl && deg == 0u && sid != 0u);
        tick(0);
        if (total == 0u) break;                             // every state of the level is a leaf
        // item lane i: its state lane (the last with items at or below i), the
        // t-th candidate of that state
        const bool il = ul < total;
        const uint64_t withi = SM & __ballot(deg != 0u);
        uint32_t skw[KW], vw[NM], e0 = 0u;
        uint32_t vv[NM];
        mwords(V, vv);
        if (__builtin_popcountll(withi) == 1) {             // one state with items: its key is uniform
            const uint32_t l = (uint32_t)__builtin_ctzll(withi);
#pragma unroll
            for (uint32_t k = 0; k < KW; ++k) skw[k] = k < used ? rl(kw[k], l) : 0u;
#pragma unroll
            for (uint32_t k = 0; k < NM; ++k) vw[k] = rl(vv[k], l);
        } else {
            uint32_t src = 0u;
            for (uint64_t m = withi; m; m &= m - 1ull) {
                const uint32_t l = (uint32_t)__builtin_ctzll(m);
                const uint32_t e = rl(excl, l);
                src = ul >= e ? l : src;
                e0 = ul >= e ? e : e0;
            }
#pragma unroll
            for (uint32_t k = 0; k < KW; ++k) {
                if (k < used) skw[k] = (uint32_t)__shfl((int)kw[k], (int)src, 64);
                else skw[k] = 0u;
            }
#pragma unroll
            for (uint32_t k = 0; k < NM; ++k) vw[k] = (uint32_t)__shfl((int)vv[k], (int)src, 64);
        }
        M Vs = mfrom<M>(vw);
        for (uint32_t t = il ? ul - e0 : 0u; t; --t) Vs &= ~mlowest(Vs);
        const uint32_t j = il ? mctz(Vs) : 0u;
        // its pid's masks: response r (findResponse) and first invocation fi (filter1)
        M Pj = pid_ev(0);
        const M jb = mbit<M>(j);
#pragma unroll
        for (uint32_t q = 1; q < 8; ++q) {
            if (q >= n_pid) break;
            const M pq = pid_ev(q);
            Pj = msel(mnz(pq & jb), pq, Pj);
        }
        const M PIj = Pj & d.INV, PRj = Pj & d.RESP;
        const M rems = mfrom<M>(skw);
        const M rr = rems & PRj;
        const uint32_t r = mnz(rr) ? mctz(rr) : j, fi = mctz(rems & PIj);
        const uint32_t lj = L.evlo[j], lr = L.evlo[r];
        const int32_t m = L.evval[j], rv = L.evval[r];
        const uint32_t code = (lj >> 8) & 0xFFu, rc = (lr >> 8) & 0xFFu;
        uint32_t res;
        if constexpr (BANK) {
            const uint32_t ex = skw[NM];
            const uint32_t ia = (lj >> 16) & 7u, ib = (lj >> 24) & 7u;
            int32_t bal_a = 0, bal_b = 0;
            bool neg = false;
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) {
                if (q < n_acc) {
                    const int32_t bq = (int32_t)skw[NM + 1 + q];
                    bal_a = q == ia ? bq : bal_a;
                    bal_b = q == ib ? bq : bal_b;
                    neg = neg || (((ex >> q) & 1u) && bq < 0);
                }
            }
            const uint32_t ex_a = (ex >> ia) & 1u, ex_b = (ex >> ib) & 1u;
            // post (test/Bank.hs:118-131): the invariant, then the expected response
            const bool tr = code == QSMD_BANK_TRANSFER, chk = code == QSMD_BANK_CHECK_BALANCE;
            const bool same = ia == ib;
            const uint32_t sel = (code == QSMD_BANK_OPEN_ACCOUNT || bal_a >= m) ? ex_a : 0u;
            const uint32_t exp = (kBankExp2 >> (code * 6u + sel * 3u)) & 7u;
            const bool err = !neg && chk && rc == QSMD_BANK_BALANCE && !ex_a;   // Map.! raises
            const bool ok = !neg && !err && rc == exp && (!chk || rv == bal_a);
            res = err ? G_ERR : (ok ? G_T : G_F);
            // next' (test/Bank.hs:92-101)
            const int32_t sa = bank_sign(code);
            const int32_t na = (ex_a ? bal_a : 0) + (ex_a ? sa : (sa & 1)) * m;
            const int32_t bo = same ? na : bal_b;
            const int32_t fb = tr ? (((ex_b != 0u) || same) ? bo : 0) + m : bo;
            skw[NM] = ex | ((chk ? 0u : 1u) << ia) | ((tr ? 1u : 0u) << ib);
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) {
                if (q < n_acc) {
                    uint32_t v = skw[NM + 1 + q];
                    v = q == ia ? (uint32_t)na : v;
                    v = (tr && q == ib) ? (uint32_t)fb : v;
                    skw[NM + 1 + q] = v;
                }
            }
        } else {
            // TicketDispenser (test/TicketDispenser.hs:81-102)
            const uint32_t just = skw[NM];
            const int32_t tn = (int32_t)skw[NM + 1];
            const bool tt = code == QSMD_TICKET_TAKE_TICKET;
            const bool ok = tt ? (rc == QSMD_TICKET_NUMBER && just != 0u && rv == tn + 1) : rc == QSMD_TICKET_OK;
            res = ok ? G_T : G_F;
            skw[NM] = 1u;
            skw[NM + 1] = tt ? (uint32_t)(tn + 1) : 0u;
        }
        {   // the child's remaining events: the pid's first invocation and its response gone
            uint32_t w2[NM];
            mwords(rems & ~(mbit<M>(fi) | mbit<M>(r)), w2);
#pragma unroll
            for (uint32_t k = 0; k < NM; ++k) skw[k] = w2[k];
        }
        tick(1);
        // children: one state per distinct key.  Lanes meet in a hash slot;
        // its lowest lane leads when the full keys agree; the rest (a slot
        // shared by different keys) go through a leader loop
        const bool isT = il && res == G_T;
        leaf_or_err |= __ballot(il && res == G_ERR);
        uint32_t child = 0xFFFu;
        uint64_t LM = 0ull;
        uint64_t pending = __ballot(isT);
        // with one parent state, the first pending lane's group by direct
        // compare (often every child: a shared pid's candidates); then hash
        // slots when more than 2 lanes remain, then the leader loop
        auto lead_one = [&]() {
            const uint32_t ldr = (uint32_t)__builtin_ctzll(pending);
            bool e2 = true;
#pragma unroll
            for (uint32_t k = 0; k < KW; ++k)
                if (k < used) e2 = e2 && skw[k] == rl(skw[k], ldr);
            const uint64_t same = __ballot(e2) & pending;
            child = (same >> ul) & 1ull ? n_states : child;
            ++n_states;
            LM |= 1ull << ldr;
            pending &= ~same;
        };
        if (pending && __builtin_popcountll(withi) == 1) lead_one();   // (one parent: often one child)
        if (__builtin_popcountll(pending) > 2) {
            const bool pl = (pending >> ul) & 1ull;
            const uint32_t slot = dag_hash<KW>(skw, used) >> 22;
            if (pl) atomicMin(&L.tab[slot], ul);
            __syncthreads();
            const uint32_t w = pl ? L.tab[slot] : ul;
            bool eq = true;
#pragma unroll
            for (uint32_t k = 0; k < KW; ++k)
                if (k < used) eq = eq && skw[k] == (uint32_t)__shfl((int)skw[k], (int)w, 64);
            const uint64_t lm = __ballot(pl && w == ul);
            if (pl && eq) child = n_states + (uint32_t)__builtin_popcountll(lm & ((1ull << w) - 1ull));
            n_states += (uint32_t)__builtin_popcountll(lm);
            LM |= lm;
            if (pl) L.tab[slot] = ~0u;                      // (every lane of the slot has read it)
            pending = __ballot(pl && !eq);
        }
        while (pending) lead_one();
        if (n_states > SC) { fit = false; break; }
        if (il) L.item[n_items + ul] = child | res << 12 | j << 14;
        n_items += total;
        lv0 = ul == nlev + 1u ? n_states : lv0;
        lv1 = ul + 64u == nlev + 1u ? n_states : lv1;
        // the next level: the leaders, with their children's keys
        SM = LM;
        sid = child;
#pragma unroll
        for (uint32_t k = 0; k < KW; ++k) kw[k] = skw[k];
        tick(2);
        if (!LM) break;                                     // no new state: the last level
        ++nlev;
    }
    __syncthreads();
    if (!fit) return -1;

    auto lvl_at = [&](uint32_t k) { return k < 64u ? rl(lv0, k) : rl(lv1, k - 64u); };
    const uint64_t limit = a.max_nodes ? a.max_nodes : ~0ull;
    if (p.memo_mode && !leaf_or_err) {
        // QSMD_FLAG_MEMO without a leaf or a raising step: every state fails,
        // and the pruning DFS evaluates each state's children once: n_items
        path_len = 0u;
        flush_stats(nlev);
        nodes_out = (uint64_t)n_items > limit ? limit : n_items;
        return (uint64_t)n_items > limit ? QSMD_STATUS_BUDGET : QSMD_STATUS_NONLINEARISABLE;
    }
    // ---- backward: g of every state, deepest level first (a state's items
    // and their children's g read 4 at a time, then folded in order)
    for (int lv = (int)nlev - 1; lv >= 0; --lv) {
        const uint32_t b0 = lvl_at((uint32_t)lv), b1 = lvl_at((uint32_t)lv + 1u);
        const uint32_t s = b0 + ul;
        if (s < b1) {
            const uint32_t xi = L.sitem[s];
            const uint32_t off = xi & 0xFFFFu, deg = xi >> 16;
            uint64_t c = 0ull;
            uint32_t res = deg ? G_F : (s ? G_T : G_F), sat = 0u;
            bool done = false;
            for (uint32_t base = 0; base < deg && !done; base += 4u) {
                uint32_t it[4], cl[4], chh[4], cf[4];
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t) it[t] = base + t < deg ? L.item[off + base + t] : 0u;
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t) {
                    const bool tc = ((it[t] >> 12) & 3u) == G_T && base + t < deg;
                    const uint32_t ch = tc ? it[t] & 0xFFFu : 0u;
                    cl[t] = tc ? L.glo[ch] : 0u;
                    chh[t] = tc ? L.ghi[ch] : 0u;
                    cf[t] = tc ? L.gfl[ch] : G_F;
                }
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t) {
                    if (done || base + t >= deg) continue;
                    const uint32_t post = (it[t] >> 12) & 3u;
                    c += 1ull;
                    if (post == G_ERR) {
                        res = G_ERR;
                        done = true;
                    } else if (post == G_T) {
                        uint64_t sum;
                        sat |= (cf[t] & G_SAT) |
                               (__builtin_add_overflow(c, cl[t] | (uint64_t)chh[t] << 32, &sum) ? G_SAT : 0u);
                        c = sum;
                        if ((cf[t] & 3u) != G_F) {
                            res = cf[t] & 3u;
                            done = true;
                        }
                    }
                }
            }
            L.glo[s] = (uint32_t)c;
            L.ghi[s] = (uint32_t)(c >> 32);
            L.gfl[s] = res | sat;
        }
        __syncthreads();
    }
    tick(3);
    const uint32_t f0 = L.gfl[0];
    const uint32_t res0 = f0 & 3u;
    const bool memo = p.memo_mode != 0u;
    // ---- the deciding path (the witness; QSMD_FLAG_MEMO: its evaluated
    // children, and the failed earlier siblings marked)
    uint64_t mcount = 0ull;
    path_len = 0u;
    if (res0 == G_T || memo) {
        uint32_t s = 0u;
        while (true) {
            const uint32_t xi = L.sitem[s];
            const uint32_t off = xi & 0xFFFFu, deg = xi >> 16;
            if (deg == 0u) break;
            uint32_t it = 0u, post = G_F, ch = 0u, cf = G_F;
            if (ul < deg) {
                it = L.item[off + ul];
                post = (it >> 12) & 3u;
                ch = post == G_T ? it & 0xFFFu : 0u;
                cf = post == G_T ? (L.gfl[ch] & 3u) : G_F;
            }
            const uint64_t dec = __ballot(ul < deg && (post == G_ERR || cf != G_F));
            const uint32_t k = dec ? (uint32_t)__builtin_ctzll(dec) : deg;
            mcount += dec ? k + 1u : deg;
            if (memo && ul < k && post == G_T) L.gfl[ch] = L.gfl[ch] | G_MARK;
            if (!dec) break;
            const uint32_t itk = rl(it, k);
            if (((itk >> 12) & 3u) == G_ERR) break;
            if (ul == 0) L.path[path_len] = (itk >> 14) & 127u;
            ++path_len;
            s = itk & 0xFFFu;
        }
        __syncthreads();
    }
    if (memo) {
        // the marked states' subtrees, level by level: each state counted once
        uint64_t part = 0ull;
        for (uint32_t lv = 1; lv < nlev; ++lv) {
            const uint32_t b0 = lvl_at(lv), b1 = lvl_at(lv + 1u);
            const uint32_t s = b0 + ul;
            if (s < b1 && (L.gfl[s] & G_MARK)) {
                const uint32_t xi = L.sitem[s];
                const uint32_t off = xi & 0xFFFFu, deg = xi >> 16;
                part += deg;
                for (uint32_t t = 0; t < deg; ++t) {
                    const uint32_t it = L.item[off + t];
                    if (((it >> 12) & 3u) == G_T) {
                        const uint32_t ch = it & 0xFFFu;
                        L.gfl[ch] = L.gfl[ch] | G_MARK;
                    }
                }
            }
            __syncthreads();
        }
        mcount += wave_sum64(part);
    }
    const uint64_t c0 = L.glo[0] | (uint64_t)L.ghi[0] << 32;
    const uint64_t n = memo ? mcount : c0;
    __syncthreads();
    flush_stats(nlev);
    if ((!memo && (f0 & G_SAT)) || n > limit) {
        nodes_out = limit;
        return QSMD_STATUS_BUDGET;
    }
    nodes_out = n;
    return res0 == G_T ? QSMD_STATUS_LINEARISABLE : (res0 == G_ERR ? QSMD_STATUS_MODEL_ERROR
                                                                   : QSMD_STATUS_NONLINEARISABLE);
}

// ---------------------------------------------------------------- chains
// A TicketDispenser history whose state DAG is a chain: at every level the
// candidates whose step is True all lead to one state (config 4's
// adversarial 8 x 64 history on one shared pid: every pending TakeTicket is
// a True candidate with the same successor -- filter1 and findResponse take
// the pid's first remaining invocation and response whichever candidate is
// tried -- so 64 levels of one state each).  A level is scalar work on the
// event masks: a candidate's step depends only on its pid's first remaining
// response (findResponse), its own request (TakeTicket / Reset) and the
// uniform state (rem, Just n), so per pid the True candidates are the pid's
// candidates among the TakeTickets or the Resets, whichever the response
// answers (test/TicketDispenser.hs:99-102).  No LDS, no per-lane step, no
// dedup table, no backward pass over LDS arrays.  Counts
// (src/Linearisability.hs:59-69): along a chain, a state's False candidates
// have no child and its True ones all enter the next state, so
//   * a chain ending at a leaf (any' [] = True) is decided by each state's
//     first True candidate: per state the candidates up to it;
//   * a chain ending at a state whose candidates are all False fails
//     everywhere: QSMD_FLAG_MEMO (each state's children once) counts every
//     candidate of every state, the exhaustive DFS g(S) = deg(S) + nT(S) *
//     g(next), folded from the bottom (past 2^64: BUDGET).
// Returns -1 when the history is not such a chain (two True candidates of a
// level with different successors): the DAG takes it from the root.
template <typename M>
__device__ int ticket_chain(const SearchArgs& a, const WaveDFS<QSMD_MODEL_TICKET, M>& d, uint32_t n_pid,
                            bool memo_mode, uint64_t& nodes_out, uint32_t& path_len, uint32_t& pathv) {
    constexpr uint32_t NW = Geo<M>::NW;
    auto pid_ev = [&](uint32_t q) -> M {                // (uniform control flow: every lane active)
        if constexpr (NW == 1) return __ballot(d.pidv[0] == q);
        else return mk128(__ballot(d.pidv[0] == q), __ballot(d.pidv[1] == q));
    };
    const M ALL = d.INV | d.RESP;
    // the TakeTicket requests (every other request of a valid history is a Reset)
    M TT;
    if constexpr (NW == 1) TT = __ballot(((d.lo[0] >> 8) & 0xFFu) == QSMD_TICKET_TAKE_TICKET) & d.INV;
    else TT = mk128(__ballot(((d.lo[0] >> 8) & 0xFFu) == QSMD_TICKET_TAKE_TICKET),
                    __ballot(((d.lo[1] >> 8) & 0xFFu) == QSMD_TICKET_TAKE_TICKET)) & d.INV;
    const M RS = d.INV & ~TT;
    M rem = ALL;
    uint32_t just = a.m0_just;
    int32_t n = (int32_t)a.m0_val[0];
    uint64_t along = 0ull, items = 0ull;
    uint32_t lvl = 0u, degv = 0u, ntv = 0u;
    int status;
    while (true) {
        const M C = mcands(rem, d.INV, d.RESP);         // takeInvocations
        // per pid: its first remaining response (findResponse) decides every
        // candidate of the pid -- TakeTicket True iff it is Number (n + 1)
        // under Just n, Reset True iff it is Ok (test/TicketDispenser.hs:99-102)
        M IT{}, T{};
        for (uint32_t q = 0; q < 8; ++q) {
            if (q >= n_pid) break;
            const M P = n_pid == 1u ? ALL : pid_ev(q);
            const M rr = rem & P & d.RESP;
            if (!mnz(rr)) continue;                     // no response: no child, not a node
            const uint32_t rq = mctz(rr);
            const uint32_t rc = (d.ev_lo(rq) >> 8) & 0xFFu;
            const int32_t rv = d.ev_val(rq);
            const M Cq = C & P;
            IT |= Cq;
            const bool ok_tt = rc == QSMD_TICKET_NUMBER && just != 0u && rv == n + 1;
            const bool ok_rs = rc == QSMD_TICKET_OK;
            T |= Cq & ((ok_tt ? TT : M{}) | (ok_rs ? RS : M{}));
        }
        const uint32_t deg = mpop(IT);
        if (deg == 0u) {                                // any' [] = True; the root: any [] = False
            status = lvl ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_NONLINEARISABLE;
            break;
        }
        const uint32_t nt = mpop(T);
        items += deg;
        degv = wl(degv, deg, lvl);
        ntv = wl(ntv, nt, lvl);
        if (nt == 0u) {                                 // every candidate False: the chain fails
            status = QSMD_STATUS_NONLINEARISABLE;
            break;
        }
        // the first True candidate (the DFS's choice) and its successor: the
        // pid's first remaining invocation and response gone (filter1,
        // findResponse), TakeTicket succ <$>, Reset Just 0
        // (test/TicketDispenser.hs:81-84).  Every True candidate must lead
        // there: one pid, and one successor model
        const uint32_t j = mctz(T);
        along += mpop(IT & MaskOps<M>::below((int)j)) + 1u;
        pathv = wl(pathv, j, lvl);
        const M Pj = n_pid == 1u ? ALL : pid_ev(d.ev_lo(j) & 0x7Fu);
        const bool tj = mnz(TT & mbit<M>(j));
        if (mnz(T & ~Pj) || (mnz(T & TT) && mnz(T & RS) && n + 1 != 0)) return -1;   // two successors
        rem &= ~(mlowest(rem & Pj & d.INV) | mlowest(rem & Pj & d.RESP));
        n = tj ? n + 1 : 0;
        just = 1u;
        ++lvl;
    }
    const uint64_t limit = a.max_nodes ? a.max_nodes : ~0ull;
    uint64_t c = status == QSMD_STATUS_LINEARISABLE ? along : items;
    bool sat = false;
    if (status == QSMD_STATUS_NONLINEARISABLE && !memo_mode && lvl > 0u) {
        // exhaustive: each True candidate searches the failing state below again
        uint64_t g = rl(degv, lvl);
        for (int k = (int)lvl - 1; k >= 0 && !sat; --k) {
            uint64_t x;
            sat = __builtin_mul_overflow((uint64_t)rl(ntv, (uint32_t)k), g, &x) ||
                  __builtin_add_overflow(x, (uint64_t)rl(degv, (uint32_t)k), &g);
        }
        c = g;
    }
    path_len = status == QSMD_STATUS_LINEARISABLE ? lvl : 0u;
    if (sat || c > limit) {
        nodes_out = limit;
        return QSMD_STATUS_BUDGET;
    }
    nodes_out = c;
    return status;
}

// The chain of a history on ONE pid (the reference's own TicketDispenser
// histories: every event on the test process's pid, test/TicketDispenser.hs:
// 302-309), level-parallel.  With one pid, level k's state has lost the
// first k invocations and the first k responses whichever candidates were
// tried (filter1 / findResponse), so its candidates are the invocations of
// rank >= k before the k-th response, and that response decides them all:
// Number v makes exactly the TakeTickets True (when v = n_k + 1 under Just
// n_k), Ok exactly the Resets (test/TicketDispenser.hs:99-102).  Every True
// candidate enters the same state, so the DAG is always a chain, and the
// model at level k > 0 is Just v or Just 0 from response k-1 (:81-84).
// Lane k evaluates level k at once; the first level without a True
// candidate or without candidates ends the chain, and the counts are
// ticket_chain's (below).  scratch: >= 256 words of the wavefront's LDS.
template <typename M>
__device__ int ticket_shared_chain(const SearchArgs& a, const WaveDFS<QSMD_MODEL_TICKET, M>& d, uint32_t n_ev,
                                   bool memo_mode, uint32_t* scratch, int lane, uint64_t& nodes_out,
                                   uint32_t& path_len, uint32_t& pathv) {
    constexpr uint32_t NW = Geo<M>::NW;
    const uint32_t ul = (uint32_t)lane;
    M TT;
    if constexpr (NW == 1) TT = __ballot(((d.lo[0] >> 8) & 0xFFu) == QSMD_TICKET_TAKE_TICKET) & d.INV;
    else TT = mk128(__ballot(((d.lo[0] >> 8) & 0xFFu) == QSMD_TICKET_TAKE_TICKET),
                    __ballot(((d.lo[1] >> 8) & 0xFFu) == QSMD_TICKET_TAKE_TICKET)) & d.INV;
    const M RS = d.INV & ~TT;
    // the k-th invocation's position, the k-th response's position, code and
    // value, by rank (event lanes scatter them into LDS)
    uint32_t* inv_at = scratch;
    uint32_t* resp_at = scratch + 64;
    uint32_t* resp_code = scratch + 128;
    int32_t* resp_val = reinterpret_cast<int32_t*>(scratch + 192);
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
        const uint32_t e = ul + 64u * w;
        const M below = MaskOps<M>::below((int)e);
        const bool inv = e < n_ev && mnz(d.INV & mbit<M>(e)), resp = e < n_ev && mnz(d.RESP & mbit<M>(e));
        const uint32_t ri = mpop(d.INV & below), rr = mpop(d.RESP & below);
        if (inv && ri < 64u) inv_at[ri] = e;
        if (resp && rr < 64u) {
            resp_at[rr] = e;
            resp_code[rr] = (d.lo[w] >> 8) & 0xFFu;
            resp_val[rr] = d.val[w];
        }
    }
    __syncthreads();
    const uint32_t nI = mpop(d.INV), nR = mpop(d.RESP);
    const uint32_t k = ul;
    const bool hasR = k < nR;
    const uint32_t I = k < nI ? inv_at[k] : 128u;
    const uint32_t R = hasR ? resp_at[k] : 0u;
    const uint32_t rc = hasR ? resp_code[k] : 0u;
    const int32_t rv = hasR ? resp_val[k] : 0;
    __syncthreads();                                    // (the scratch is free again)
    // the model at level k: model0, then Just (response k-1's Number) or Just 0
    const uint32_t prc = (uint32_t)__shfl((int)rc, (int)(k ? k - 1u : 0u), 64);
    const int32_t prv = __shfl(rv, (int)(k ? k - 1u : 0u), 64);
    const uint32_t just = k ? 1u : a.m0_just;
    const int32_t n = k ? (prc == QSMD_TICKET_NUMBER ? prv : 0) : (int32_t)a.m0_val[0];
    // candidates: invocations of rank >= k (positions >= I) before position R
    const M W = hasR ? d.INV & ~MaskOps<M>::below((int)I) & MaskOps<M>::below((int)R) : M{};
    const bool tt_ok = rc == QSMD_TICKET_NUMBER && just != 0u && rv == n + 1;
    const M T = tt_ok ? W & TT : (rc == QSMD_TICKET_OK ? W & RS : M{});
    const uint32_t deg = mpop(W), nt = mpop(T);
    const uint32_t j = mnz(T) ? mctz(T) : 0u;
    const uint32_t idx = mnz(T) ? mpop(W & MaskOps<M>::below((int)j)) : 0u;
    const uint64_t stop = __ballot(deg == 0u || nt == 0u);
    const uint32_t L = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;   // the chain's last level
    const uint32_t degL = L < 64u ? rl(deg, L) : 0u;
    int status = degL ? QSMD_STATUS_NONLINEARISABLE : (L ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_NONLINEARISABLE);
    const uint64_t along = wave_sum64(k < L ? (uint64_t)idx + 1u : 0ull);
    const uint64_t items = wave_sum64(k <= L ? (uint64_t)deg : 0ull);
    pathv = j;
    uint64_t c = status == QSMD_STATUS_LINEARISABLE ? along : items;
    bool sat = false;
    if (degL && !memo_mode && L > 0u) {                 // exhaustive: g = deg + nT g(next), from the bottom
        uint64_t g = degL;
        for (int q = (int)L - 1; q >= 0 && !sat; --q) {
            uint64_t x;
            sat = __builtin_mul_overflow((uint64_t)rl(nt, (uint32_t)q), g, &x) ||
                  __builtin_add_overflow(x, (uint64_t)rl(deg, (uint32_t)q), &g);
        }
        c = g;
    }
    const uint64_t limit = a.max_nodes ? a.max_nodes : ~0ull;
    path_len = status == QSMD_STATUS_LINEARISABLE ? L : 0u;
    if (sat || c > limit) {
        nodes_out = limit;
        return QSMD_STATUS_BUDGET;
    }
    nodes_out = c;
    return status;
}

__device__ __forceinline__ void clear_table(uint32_t* tab, uint32_t buckets, int lane) {
    // every word 0xFFFFFFFF (word 2 never matches), 16 B per lane and store
    uint4* t4 = reinterpret_cast<uint4*>(tab);
    for (uint32_t k = (uint32_t)lane; k < buckets * 16u; k += 64u) t4[k] = make_uint4(~0u, ~0u, ~0u, ~0u);
}

// One history h (its header H) searched by the whole wavefront (wide: from
// stage 0w's deferred list).
template <uint32_t MODEL, typename M>
__device__ __forceinline__ void wave_history(const WaveArgs& p, uint32_t h, const qsmd_hdr& H, bool wide,
                                             uint32_t* tab, uint32_t epoch, uint32_t& victim, int lane, uint64_t t0,
                                             Counters& cnt, uint32_t* dag_base) {
    constexpr uint32_t NW = Geo<M>::NW, EW = Geo<M>::EW;
    const SearchArgs& a = p.s;
    const uint64_t limit = a.max_nodes ? a.max_nodes : ~0ull;
    const uint32_t n_ev = H.n_ev;
    WaveDFS<MODEL, M> d;
    // staging: lane l loads events l (and l + 64): coalesced 8-B loads
    bool bad = false, big = false;
    uint64_t resp[NW], all[NW];
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
        const uint32_t e = (uint32_t)lane + 64u * w;
        const bool in = e < n_ev;
        const uint2 x = in ? a.events[H.ev_off + e] : make_uint2(0u, 0u);
        d.lo[w] = x.x;
        d.val[w] = (int32_t)x.y;
        const uint32_t pid = x.x & 0x7Fu;
        d.pidv[w] = in ? pid : 0xFFu;
        bad = bad || (in && (!valid_bits<MODEL>(x.x) || pid >= H.n_pid));
        big = big || (in && (x.x & 0x80u) == 0u && ((int32_t)x.y >= kWideValue || (int32_t)x.y <= -kWideValue));
        resp[w] = __ballot(in && (x.x & 0x80u));
        all[w] = __ballot(in);
    }
    M ALL;
    if constexpr (NW == 1) {
        d.RESP = resp[0];
        ALL = all[0];
    } else {
        d.RESP = mk128(resp[0], resp[1]);
        ALL = mk128(all[0], all[1]);
    }
    d.INV = ALL & ~d.RESP;
    d.rem = ALL;
    d.cand = mcands(d.rem, d.INV, d.RESP);
    d.depth = 0u;
    d.found = 0u;
    d.nodes = 0ull;
    d.RS = 0ull;
    d.stk = 0u;
    d.ent = 0u;
    d.ex = a.m0_exists;
    const bool e_q = (uint32_t)lane < QSMD_BANK_MAX_ACCOUNTS && ((a.m0_exists >> (uint32_t)lane) & 1u);
    d.bal = 0;
    d.neg = __ballot(e_q && (int32_t)a.m0_val[lane & 7] < 0) != 0ull ? 1u : 0u;
    d.kb = 0u;
    d.wacc = 0u;
    d.mh = 0u;
#pragma unroll
    for (uint32_t q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) {
        d.mh ^= WaveDFS<MODEL, M>::acc_hash(q, 0);
        if constexpr (MODEL == QSMD_MODEL_BANK)
            if ((a.m0_exists >> q) & 1u) d.set_bal(q, 0, (int32_t)a.m0_val[q]);
    }

    int status = -1;
    if (__ballot(bad) != 0ull) {
        status = QSMD_STATUS_ENCODE_ERROR;
    } else if (wide && __ballot(big) != 0ull) {
        status = QSMD_STATUS_HANDED_OFF;         // values the i32 model may overflow on: the giant stage
    } else if (n_ev == 0u) {
        status = QSMD_STATUS_LINEARISABLE;
    } else if (beyond_first_fail(a, h)) {
        status = QSMD_STATUS_SKIPPED;
    }
    const uint64_t c0 = p.stats ? __builtin_amdgcn_s_memtime() : 0ull;
    if (status < 0 && dag_base) {                    // a chain, else the state DAG when it fits
        const DagLds L = dag_carve<MODEL, M>(dag_base, p.dag_states, p.dag_items);
        uint64_t dn = 0ull;
        uint32_t plen = 0u, pathv = 0u;
        int ds = -1;
        bool chain = false;
        if constexpr (MODEL == QSMD_MODEL_TICKET) {
            ds = H.n_pid == 1u ? ticket_shared_chain<M>(a, d, n_ev, p.memo_mode != 0u, L.tab, lane, dn, plen, pathv)
                               : ticket_chain<M>(a, d, H.n_pid, p.memo_mode != 0u, dn, plen, pathv);
            chain = ds >= 0;
        }
        if (ds < 0) ds = dag_history<MODEL, M>(p, a, d, n_ev, H.n_pid, L, p.dag_states, p.dag_items, lane, dn, plen);
        if (ds >= 0) {
            if (p.stats && lane == 0) {
                const unsigned long long cyc = __builtin_amdgcn_s_memtime() - c0;
                atomicAdd(p.stats + 5, 1ull);
                atomicMax(p.stats + 6, cyc);
                atomicAdd(p.stats + 7, cyc);
            }
            if (lane == 0) {
                note_failure(a, h, ds);
                a.status[h] = (uint8_t)ds;
                if (a.nodes) a.nodes[h] = dn;
                cnt.add(ds, dn);
            }
            if (p.dbg && h == p.dbg_h) {             // diagnostic: the DAG arrays of one history
                const uint32_t* src = dag_base;
                const uint32_t nw = (uint32_t)(dag_lds_bytes<MODEL, M>(p.dag_states, p.dag_items) / 4u);
                for (uint32_t i = (uint32_t)lane; i < nw; i += 64u) p.dbg[16 + i] = src[i];
                if (lane == 0) {
                    p.dbg[0] = (uint32_t)ds;
                    p.dbg[1] = (uint32_t)dn;
                    p.dbg[2] = p.dag_states;
                    p.dbg[3] = p.dag_items;
                }
            }
            if (a.witness && ds == QSMD_STATUS_LINEARISABLE) {
                uint8_t* w = a.witness + H.ev_off;
                if (chain) {                         // (a chain of <= 64 levels: lane k holds level k's)
                    if ((uint32_t)lane < plen) w[lane] = (uint8_t)pathv;
                    if (lane == 0 && plen < n_ev) w[plen] = QSMD_WITNESS_END;
                } else {
                    for (uint32_t k = (uint32_t)lane; k <= plen && k < n_ev; k += 64u)
                        w[k] = k < plen ? (uint8_t)L.path[k] : QSMD_WITNESS_END;
                }
            }
            __syncthreads();                         // (L.path read before the next history reuses it)
            return;
        }
    }
    if (status < 0 && dag_base) {
        // the DAG did not fit and its arrays share the LDS with the memo
        // table (wave_lds: one region, the larger of the two): clear it
        clear_table(tab, p.buckets, lane);
        __syncthreads();
    }
    bool skip = false;
    uint32_t iter = 0;
    const uint32_t min_rem = p.memo_min_rem;
    const bool counts = !p.memo_mode;            // exact counts (else QSMD_FLAG_MEMO: explored nodes)
    const uint32_t cap = (uint32_t)min(wide ? p.explore_cap_wide : p.explore_cap, 0xFFFFFFFFull);
    while (status < 0) {
        const bool empty = !mnz(d.cand);
        if (empty && (d.found == 0u || d.depth == 0u)) {
            // no children: a leaf => True (any' []), the root => False (any [])
            status = (d.found == 0u && d.depth > 0u) ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_NONLINEARISABLE;
            break;
        }
        if (empty) {
            // leaving the node at depth d.depth: its subtree was searched to the end and failed
            if (!skip && (!counts || d.nodes <= 0xFFFFFFFFull) && mpop(d.rem) > min_rem) {
                const WKey k = wave_key<MODEL, M>(d, a, epoch, p.buckets - 1u, lane);
                if (k.ok) wave_insert<EW>(tab, k, counts ? (uint32_t)d.nodes - rl(d.ent, d.depth - 1u) : 0u,
                                          victim++, lane);
            }
            skip = false;
            const uint32_t j = d.undo();
            d.cand = mcands(d.rem, d.INV, d.RESP) & mabove(j, d.rem);
            d.found = 1u;
        }
        if (mnz(d.cand)) {
            const uint32_t dep0 = d.depth;
            status = d.try_next(a, limit);
            if (d.depth > dep0 && status < 0) {                // entered a new node (the search goes on)
                d.ent = wl(d.ent, (uint32_t)d.nodes, dep0);
                if (mpop(d.rem) > min_rem) {
                    const WKey k = wave_key<MODEL, M>(d, a, epoch, p.buckets - 1u, lane);
                    uint32_t c = 0;
                    if (k.ok && wave_lookup<EW>(tab, k, lane, c)) {
                        if (counts && d.nodes + c > limit) {   // the budget falls inside that subtree
                            d.nodes = limit;
                            status = QSMD_STATUS_BUDGET;
                        } else {
                            d.nodes += counts ? c : 0u;        // its nodes, counted; it failed
                            d.cand = M{};
                            d.found = 1u;
                            skip = true;
                        }
                    }
                }
            }
        }
        ++iter;
        if (status < 0) {
            if (cap && iter >= cap) {
                status = QSMD_STATUS_HANDED_OFF;
            } else if ((iter & 1023u) == 0u) {
                if (beyond_first_fail(a, h)) {
                    status = QSMD_STATUS_SKIPPED;
                } else if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                    if (lane == 0) atomicOr(a.timed_out, 1u);
                    status = QSMD_STATUS_BUDGET;
                }
            }
        }
    }
    if (p.stats && lane == 0) {
        const uint64_t cyc = __builtin_amdgcn_s_memtime() - c0;
        atomicMax(p.stats + 0, (unsigned long long)iter);
        atomicAdd(p.stats + 1, (unsigned long long)iter);
        atomicMax(p.stats + 2, (unsigned long long)cyc);
        atomicAdd(p.stats + 3, (unsigned long long)cyc);
        atomicAdd(p.stats + 4, (unsigned long long)d.nodes);
    }
    if (status == QSMD_STATUS_HANDED_OFF) {          // the giant stage searches it (exact, from the root)
        if (lane == 0) a.giant_list[atomicAdd(a.giant_count, 1u)] = h;
        return;
    }
    if (lane == 0) {
        note_failure(a, h, status);
        a.status[h] = (uint8_t)status;
        if (a.nodes) a.nodes[h] = d.nodes;
        cnt.add(status, d.nodes);
    }
    if (a.witness && status == QSMD_STATUS_LINEARISABLE) {
        uint8_t* w = a.witness + H.ev_off;
        if ((uint32_t)lane < d.depth) w[lane] = (uint8_t)(d.stk & 127u);
        else if ((uint32_t)lane == d.depth && d.depth < n_ev) w[lane] = QSMD_WITNESS_END;
    }
}

}  // namespace

// The three lists (stage 0's heavy, stage 0w's heavy, stage 0w's wide), one
// history per wavefront, grid-stride; two kernels so that each holds one mask
// width in its scalar registers: u64 (list32, list64 and the wide list's
// histories of <= 64 events) and, when p.wide128, M128 (the wide list's
// 65..128-event histories).  A wide history neither takes (> 128 events, > 8
// pids, model0 values beyond +-2^24) goes to the giant stage, once.
template <uint32_t MODEL, typename M>
__global__ __launch_bounds__(C_LANES) void wave_search(WaveArgs p) {
    constexpr bool W128 = Geo<M>::NW == 2;
    extern __shared__ uint32_t tab[];
    const int lane = threadIdx.x;
    // (list_wide null: every history of the batch is on the wide list -- the
    // host entry's routing when none fits the compact stages)
    const uint32_t n32 = W128 ? 0u : list_total(p.count32, p.cap32), n64 = W128 ? 0u : *p.count64;
    const uint32_t nw = p.list_wide ? *p.count_wide : (uint32_t)p.s.n_hist;
    const uint64_t t0 = p.s.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    Counters cnt;
    uint32_t* dag = p.dag_states ? tab : nullptr;   // (the DAG arrays over the memo table: wave_lds)
    clear_table(tab, p.buckets, lane);
    uint32_t epoch = 0u, victim = 0u;
    for (uint32_t i = blockIdx.x; i < n32 + n64 + nw; i += gridDim.x) {
        const uint32_t h = i < n32 ? list_at(p.list32, p.count32, p.cap32, i)
                         : (i < n32 + n64 ? p.list64[i - n32]
                                          : (p.list_wide ? p.list_wide[i - n32 - n64] : i - n32 - n64));
        const qsmd_hdr H = p.s.hdr[h];
        const bool wide = i >= n32 + n64;
        if (wide) {
            // (no list: the M128 launch alone takes the batch; a <= 64-event
            // history there has more than 8 pids and goes on to the giant stage)
            const bool mine = W128 ? (H.n_ev > 64u || !p.list_wide) : (H.n_ev <= 64u || !p.wide128);
            if (!mine) continue;
            // the batch unlisted: no compact stage checked the header (the
            // wide list's come validated by stage 0w); a wrong model or an
            // event range outside the batch is ENCODE_ERROR, never read
            if (!p.list_wide && H.n_ev <= QSMD_MAX_EVENTS && H.n_pid <= QSMD_MAX_PIDS &&
                (H.model_id != MODEL || (uint64_t)H.ev_off + H.n_ev > p.s.n_events)) {
                if (lane == 0) {
                    p.s.status[h] = (uint8_t)QSMD_STATUS_ENCODE_ERROR;
                    if (p.s.nodes) p.s.nodes[h] = 0ull;
                    cnt.add(QSMD_STATUS_ENCODE_ERROR, 0ull);
                }
                continue;
            }
            if (H.n_ev > (W128 || !p.wide128 ? 128u : 64u) || H.n_ev > 64u * Geo<M>::NW || H.n_pid > 8u ||
                !p.s.m0_wave) {                  // the giant stage's
                if (lane == 0) p.s.giant_list[atomicAdd(p.s.giant_count, 1u)] = h;
                continue;
            }
        }
        if (++epoch == kEpochMax) {                  // tags exhausted: clear, start over
            clear_table(tab, p.buckets, lane);
            epoch = 1u;
        }
        wave_history<MODEL, M>(p, h, H, wide, tab, epoch, victim, lane, t0, cnt, dag);
    }
    cnt.flush(p.s.buckets, lane);
}

// dynamic LDS of one workgroup: the memo table and the DAG arrays in one
// region (a history runs the DFS, with the memo, only when its DAG did not
// fit, and the table is cleared then), so a config-2 call's ~2300 heavy
// histories are resident at once (16 workgroups per CU; with the two regions
// side by side, 9 per CU: two rounds)
template <uint32_t MODEL, typename M>
static size_t wave_lds(const WaveArgs& p) {
    const size_t memo = (size_t)p.buckets * 64u * 4u;
    const size_t dag = p.dag_states ? dag_lds_bytes<MODEL, M>(p.dag_states, p.dag_items) : 0u;
    return memo > dag ? memo : dag;
}

constexpr size_t kMaxLds = 160u * 1024u;   // gfx950: LDS per workgroup at most

template <uint32_t MODEL, typename M>
static hipError_t launch_one(WaveArgs p, uint32_t grid, hipStream_t s) {
    while (p.dag_states && wave_lds<MODEL, M>(p) > kMaxLds) {   // a DAG capacity beyond the LDS: halved
        p.dag_states = (p.dag_states / 2u) & ~1u;
        p.dag_items = 4u * p.dag_states;
    }
    const size_t lds = wave_lds<MODEL, M>(p);
    if (lds > 64u * 1024u) {
        static std::atomic<int> set[kAttrDevices];
        const hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&wave_search<MODEL, M>), set, lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((wave_search<MODEL, M>), dim3(grid), dim3(C_LANES), lds, s, p);
    return hipGetLastError();
}

hipError_t launch_wave(const WaveArgs& p, uint32_t grid, uint32_t grid128, hipStream_t s) {
    hipError_t e = hipSuccess;
    if (grid)                                               // (0: no <= 64-event history in the call)
        e = p.s.model_id == QSMD_MODEL_BANK ? launch_one<QSMD_MODEL_BANK, uint64_t>(p, grid, s)
                                            : launch_one<QSMD_MODEL_TICKET, uint64_t>(p, grid, s);
    if (e != hipSuccess || !p.wide128) return e;
    return p.s.model_id == QSMD_MODEL_BANK ? launch_one<QSMD_MODEL_BANK, M128>(p, grid128, s)
                                           : launch_one<QSMD_MODEL_TICKET, M128>(p, grid128, s);
}

}  // namespace qsmd
