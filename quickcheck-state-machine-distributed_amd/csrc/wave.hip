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

// One history h (its header H) searched by the whole wavefront (wide: from
// stage 0w's deferred list).
template <uint32_t MODEL, typename M>
__device__ __forceinline__ void wave_history(const WaveArgs& p, uint32_t h, const qsmd_hdr& H, bool wide,
                                             uint32_t* tab, uint32_t epoch, uint32_t& victim, int lane, uint64_t t0,
                                             Counters& cnt) {
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
    bool skip = false;
    uint32_t iter = 0;
    const uint64_t c0 = p.stats ? __builtin_amdgcn_s_memtime() : 0ull;
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

__device__ __forceinline__ void clear_table(uint32_t* tab, uint32_t buckets, int lane) {
    for (uint32_t b = 0; b < buckets; ++b) tab[b * 64u + (uint32_t)lane] = 0xFFFFFFFFu;   // word 2 never matches
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
    const uint32_t n32 = W128 ? 0u : *p.count32, n64 = W128 ? 0u : *p.count64, nw = *p.count_wide;
    const uint64_t t0 = p.s.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    Counters cnt;
    clear_table(tab, p.buckets, lane);
    uint32_t epoch = 0u, victim = 0u;
    for (uint32_t i = blockIdx.x; i < n32 + n64 + nw; i += gridDim.x) {
        const uint32_t h = i < n32 ? p.list32[i] : (i < n32 + n64 ? p.list64[i - n32] : p.list_wide[i - n32 - n64]);
        const qsmd_hdr H = p.s.hdr[h];
        const bool wide = i >= n32 + n64;
        if (wide) {
            const bool mine = W128 ? H.n_ev > 64u : (H.n_ev <= 64u || !p.wide128);
            if (!mine) continue;
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
        wave_history<MODEL, M>(p, h, H, wide, tab, epoch, victim, lane, t0, cnt);
    }
    cnt.flush(p.s.buckets, lane);
}

hipError_t launch_wave(const WaveArgs& p, uint32_t grid, uint32_t grid128, hipStream_t s) {
    const size_t lds = (size_t)p.buckets * 64u * 4u;
    if (p.s.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL((wave_search<QSMD_MODEL_BANK, uint64_t>), dim3(grid), dim3(C_LANES), lds, s, p);
    else
        hipLaunchKernelGGL((wave_search<QSMD_MODEL_TICKET, uint64_t>), dim3(grid), dim3(C_LANES), lds, s, p);
    if (p.wide128) {
        if (p.s.model_id == QSMD_MODEL_BANK)
            hipLaunchKernelGGL((wave_search<QSMD_MODEL_BANK, M128>), dim3(grid128), dim3(C_LANES), lds, s, p);
        else
            hipLaunchKernelGGL((wave_search<QSMD_MODEL_TICKET, M128>), dim3(grid128), dim3(C_LANES), lds, s, p);
    }
    return hipGetLastError();
}

}  // namespace qsmd
