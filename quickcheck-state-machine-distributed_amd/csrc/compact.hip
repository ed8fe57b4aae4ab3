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
#include "models.h"

namespace qsmd {

namespace {

constexpr int C_MAXEV = 32;
constexpr int C_LANES = 64;
constexpr int C_CHUNK = 16;
constexpr int32_t V19_MIN = -(1 << 18), V19_MAX = (1 << 18) - 1;

// compressed event: pid 3 | resp 1 | code 3 | a 3 | b 3 | val 19 (signed)
__device__ __forceinline__ uint32_t c_code(uint32_t w) { return (w >> 4) & 7u; }
__device__ __forceinline__ uint32_t c_a(uint32_t w) { return (w >> 7) & 7u; }
__device__ __forceinline__ uint32_t c_b(uint32_t w) { return (w >> 10) & 7u; }
__device__ __forceinline__ int32_t c_val(uint32_t w) { return (int32_t)w >> 13; }

__device__ __forceinline__ uint32_t below32(uint32_t r) { return (uint32_t)((1ull << r) - 1ull); }

// candidates: remaining invocations before the first remaining response
// (takeInvocations, src/Linearisability.hs:25-28); branch-free
__device__ __forceinline__ uint32_t cands(uint32_t rem, uint32_t INV, uint32_t RESP) {
    const uint32_t R = (uint32_t)__builtin_ctzll((uint64_t)(rem & RESP) | (1ull << 32));
    return rem & INV & below32(R);
}

// Expected Bank response constructor of `post` (test/Bank.hs:118-131) as a
// table lookup, index = code*4 + ex_a*2 + ge (3 bits per entry):
//   Open: ex_a ? AccountAlreadyExists : AccountCreated   Deposit: DepositMade
//   Withdraw: ge ? WithdrawalMade : InsufficientFunds    CheckBalance: Balance
//   Transfer: ge ? TransferMade : InsufficientFunds
constexpr uint64_t bank_exp_table() {
    uint64_t t = 0;
    for (uint32_t code = 0; code < 5; ++code)
        for (uint32_t exa = 0; exa < 2; ++exa)
            for (uint32_t ge = 0; ge < 2; ++ge) {
                uint32_t e = QSMD_BANK_INSUFFICIENT_FUNDS;
                if (code == QSMD_BANK_OPEN_ACCOUNT) e = exa ? QSMD_BANK_ACCOUNT_ALREADY_EXISTS : QSMD_BANK_ACCOUNT_CREATED;
                else if (code == QSMD_BANK_DEPOSIT) e = QSMD_BANK_DEPOSIT_MADE;
                else if (code == QSMD_BANK_WITHDRAW) e = ge ? QSMD_BANK_WITHDRAWAL_MADE : QSMD_BANK_INSUFFICIENT_FUNDS;
                else if (code == QSMD_BANK_CHECK_BALANCE) e = QSMD_BANK_BALANCE;
                else e = ge ? QSMD_BANK_TRANSFER_MADE : QSMD_BANK_INSUFFICIENT_FUNDS;
                t |= (uint64_t)e << (3 * (code * 4 + exa * 2 + ge));
            }
    return t;
}
constexpr uint64_t kBankExp = bank_exp_table();
// per request code: sign of the step on account a (Deposit +1, Withdraw and
// Transfer -1, Open / CheckBalance 0); an absent account is created with the
// money exactly when the sign is non-zero (insertWith, test/Bank.hs:96-97)
constexpr uint32_t kBankNeg = (1u << QSMD_BANK_WITHDRAW) | (1u << QSMD_BANK_TRANSFER);
constexpr uint32_t kBankPos = (1u << QSMD_BANK_DEPOSIT);

__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// include/qsmd.h encoding rules, branch-free.
template <uint32_t MODEL>
__device__ __forceinline__ bool valid_bits(uint32_t lo) {
    const uint32_t c = (lo >> 8) & 0xFFu, ea = (lo >> 16) & 0xFFu, eb = lo >> 24;
    if constexpr (MODEL == QSMD_MODEL_TICKET) {
        return c <= 1u;
    } else {
        const bool resp = (lo & 0x80u) != 0u;
        const bool inv_ok = (c <= QSMD_BANK_TRANSFER) & (ea < 8u) & ((c != QSMD_BANK_TRANSFER) | (eb < 8u));
        return resp ? (c <= QSMD_BANK_BALANCE) : inv_ok;
    }
}

// The DFS stack: 16 levels x 8 bits in 4 VGPRs.  Selection goes through an
// empty asm so hipcc keeps it a register select (it otherwise turns the
// select tree into a scratch-memory indexed load).
struct Stack16 {
    uint32_t w[4];
    __device__ __forceinline__ uint32_t word(uint32_t d) const {
        uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3];
        asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
        const uint32_t k = d >> 2;
        const uint32_t lo = (k & 1u) ? x1 : x0, hi = (k & 1u) ? x3 : x2;
        return (k & 2u) ? hi : lo;
    }
    __device__ __forceinline__ uint32_t get(uint32_t d) const {
        return (word(d) >> ((d & 3u) * 8u)) & 0xFFu;
    }
    __device__ __forceinline__ void put(uint32_t d, uint32_t v) {
        const uint32_t k = d >> 2, sh = (d & 3u) * 8u;
        const uint32_t keep = ~(0xFFu << sh), ins = v << sh;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) w[q] = (q == k) ? ((w[q] & keep) | ins) : w[q];
    }
};

// ------------------------------------------------------------------ staging

struct Staged {
    uint32_t INV, RESP, P0, P1, P2;
    bool ok, fits;
};

__device__ __forceinline__ uint32_t compress(uint32_t lo, int32_t val) {
    return (lo & 7u) | (((lo >> 7) & 1u) << 3) | (((lo >> 8) & 7u) << 4) | (((lo >> 16) & 7u) << 7) |
           (((lo >> 24) & 7u) << 10) | ((uint32_t)val << 13);
}

// One lane stages its own history: C_CHUNK loads in flight (index clamped
// into the history, no exec-masked branches), compress into its LDS column,
// build the register masks.
template <uint32_t MODEL>
__device__ __forceinline__ void stage_lane(const SearchArgs& a, const qsmd_hdr& H, uint32_t (*s_ev)[C_LANES],
                                           int lane, Staged& s) {
    const uint32_t n_ev = H.n_ev, n_pid = H.n_pid;
    if (n_ev == 0) return;
    const uint2* evp = a.events + H.ev_off;
    const uint32_t last = n_ev - 1u;
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < n_ev; c0 += C_CHUNK) {
        uint2 x[C_CHUNK];
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)C_CHUNK; ++k) {
            const uint32_t e = c0 + k;
            x[k] = evp[e < last ? e : last];
        }
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)C_CHUNK; ++k) {
            const uint32_t e = c0 + k;
            const uint32_t lo = x[k].x;
            const int32_t val = (int32_t)x[k].y;
            const bool in = e < n_ev;
            const uint32_t p = lo & 0x7Fu;
            s.ok = s.ok & (!in | ((p < n_pid) & valid_bits<MODEL>(lo)));
            s.fits = s.fits & (!in | ((val >= V19_MIN) & (val <= V19_MAX)));
            s_ev[e][lane] = compress(lo, val);
            const uint32_t bit = in ? (1u << e) : 0u;
            const uint32_t resp = (lo >> 7) & 1u;
            s.RESP |= resp ? bit : 0u;
            s.INV |= resp ? 0u : bit;
            s.P0 |= (p & 1u) ? bit : 0u;
            s.P1 |= (p & 2u) ? bit : 0u;
            s.P2 |= (p & 4u) ? bit : 0u;
        }
    }
}

// The whole wavefront stages 64 histories packed back to back with one
// common length N0 starting at event off0: the 64*N0-event block is read
// with fully coalesced 16-byte loads (a per-lane history walk touches 64
// cache lines per wave instruction), each event is validated, compressed and
// scattered to its history's lane column, then every lane builds its masks
// from LDS.  Requires all 64 lanes active.
template <uint32_t MODEL>
__device__ __forceinline__ void stage_packed(const SearchArgs& a, uint32_t N0, uint32_t off0, uint32_t n_ev,
                                             uint32_t n_pid, uint32_t (*s_ev)[C_LANES], uint32_t* s_flag,
                                             int lane, Staged& s) {
    s_flag[lane] = 0u;
    const float invN = 1.0f / (float)N0;
    // history of block event g (exact for g < 2^11)
    auto hist_of = [&](uint32_t g) -> uint32_t { return (uint32_t)(((float)g + 0.5f) * invN) & 63u; };
    // n_pid of that history: the cross-lane read runs with every lane active
    // (ds_bpermute from an inactive source lane returns 0)
    auto npid_of = [&](uint32_t hh) -> uint32_t { return (uint32_t)__shfl((int)n_pid, (int)hh, 64); };
    auto put_event = [&](uint32_t g, uint32_t hh, uint32_t np, uint32_t lo, int32_t val) {
        const uint32_t e = g - hh * N0;
        const uint32_t p = lo & 0x7Fu;
        const bool vok = (p < np) & valid_bits<MODEL>(lo);
        const bool vfit = (val >= V19_MIN) & (val <= V19_MAX);
        s_ev[e][hh] = compress(lo, val);
        if (!(vok & vfit)) atomicOr(&s_flag[hh], vok ? 2u : 1u);
    };
    const uint32_t total_ev = 64u * N0;
    if ((off0 & 1u) == 0u) {
        const uint4* blk = reinterpret_cast<const uint4*>(a.events + off0);
        for (uint32_t k0 = 0; k0 < total_ev / 2u; k0 += 4u * 64u) {
            uint4 x[4];
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t q = k0 + u * 64u + (uint32_t)lane;
                x[u] = q < total_ev / 2u ? blk[q] : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t q = k0 + u * 64u + (uint32_t)lane;
                const uint32_t h0 = hist_of(2u * q), h1 = hist_of(2u * q + 1u);
                const uint32_t np0 = npid_of(h0), np1 = npid_of(h1);
                if (q < total_ev / 2u) {
                    put_event(2u * q, h0, np0, x[u].x, (int32_t)x[u].y);
                    put_event(2u * q + 1u, h1, np1, x[u].z, (int32_t)x[u].w);
                }
            }
        }
    } else {
        const uint2* blk = a.events + off0;
        for (uint32_t k0 = 0; k0 < total_ev; k0 += 8u * 64u) {
            uint2 x[8];
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t g = k0 + u * 64u + (uint32_t)lane;
                x[u] = g < total_ev ? blk[g] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t g = k0 + u * 64u + (uint32_t)lane;
                const uint32_t hh = hist_of(g);
                const uint32_t np = npid_of(hh);
                if (g < total_ev) put_event(g, hh, np, x[u].x, (int32_t)x[u].y);
            }
        }
    }
    const uint32_t fl = s_flag[lane];
    s.ok = s.ok & ((fl & 1u) == 0u);
    s.fits = s.fits & ((fl & 2u) == 0u);
#pragma unroll
    for (uint32_t e = 0; e < (uint32_t)C_MAXEV; ++e) {
        const uint32_t cw = s_ev[e][lane];
        const uint32_t bit = e < n_ev ? (1u << e) : 0u;
        const uint32_t resp = (cw >> 3) & 1u;
        s.RESP |= resp ? bit : 0u;
        s.INV |= resp ? 0u : bit;
        s.P0 |= (cw & 1u) ? bit : 0u;
        s.P1 |= (cw & 2u) ? bit : 0u;
        s.P2 |= (cw & 4u) ? bit : 0u;
    }
}

// --------------------------------------------------------------- the DFS

// Per-lane search state (registers) over the history in LDS column `lane`.
// step() runs one iteration: an optional backtrack followed by one
// candidate try; it returns -1 to continue or the final QSMD_STATUS_*
// (QSMD_STATUS_BUDGET = `limit` nodes reached before a decision).
template <uint32_t MODEL>
struct LaneDFS {
    static constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    uint32_t INV, RESP, P0, P1, P2, ALL;
    uint32_t rem, cand, depth, ex, neg, RS, found;
    uint32_t base;          // depth of the search root (0; the task depth in split_search)
    uint64_t nodes;
    Stack16 stk;

    // events whose pid equals the pid of event j (bit-sliced compare)
    __device__ __forceinline__ uint32_t same_pid(uint32_t j) const {
        const uint32_t m0 = 0u - ((P0 >> j) & 1u), m1 = 0u - ((P1 >> j) & 1u), m2 = 0u - ((P2 >> j) & 1u);
        return ~((P0 ^ m0) | (P1 ^ m1) | (P2 ^ m2)) & ALL;
    }

    __device__ __forceinline__ void init(const Staged& s, const SearchArgs& a, int32_t (*s_bal)[C_LANES],
                                         int lane) {
        INV = s.INV; RESP = s.RESP; P0 = s.P0; P1 = s.P1; P2 = s.P2;
        ALL = INV | RESP;
        rem = ALL;
        cand = cands(rem, INV, RESP);
        depth = 0; found = 0; nodes = 0; RS = 0; base = 0;
        stk.w[0] = stk.w[1] = stk.w[2] = stk.w[3] = 0u;
        ex = a.m0_exists; neg = 0;
        if constexpr (BANK) {
#pragma unroll
            for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) {
                const bool e = (ex >> q) & 1u;
                const int32_t v = e ? (int32_t)a.m0_val[q] : 0;
                s_bal[q][lane] = v;
                neg |= (e && v < 0) ? (1u << q) : 0u;
            }
        }
    }

    // evc[e * STRIDE] = compressed event e (the lane's LDS column: STRIDE = 64;
    // a history shared by the wavefront: STRIDE = 1)
    template <int STRIDE>
    __device__ __forceinline__ int step(const SearchArgs& a, const uint32_t* evc,
                                        int32_t (*s_bal)[C_LANES], int lane, uint64_t limit) {
        if (!cand) {
            // no children: a leaf => True (any' []), the root => False (any []);
            // a subtree rooted at depth base > 0 is an inner node of the reference tree
            if (!found || depth == base)
                return (!found && depth > 0) ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_NONLINEARISABLE;
            // ---- backtrack: restore the parent level exactly
            --depth;
            const uint32_t st = stk.get(depth);
            const uint32_t j = st & 31u;
            const uint32_t gone = ~rem & same_pid(j);
            rem |= (1u << (31 - __builtin_clz(gone & INV))) | (1u << (31 - __builtin_clz(gone & RESP)));
            if constexpr (BANK) {
                const uint32_t cj = evc[j * STRIDE];
                const uint32_t code = c_code(cj), ia = c_a(cj), ib = c_b(cj);
                const int32_t m = c_val(cj);
                const uint32_t pa = (st >> 5) & 1u, pb = (st >> 6) & 1u;
                const uint32_t tr = code == QSMD_BANK_TRANSFER ? 1u : 0u;
                const int32_t ba = s_bal[ia][lane], bb = s_bal[ib][lane];
                // undo Transfer's deposit on b, then the step on a
                const int32_t rb = (pb | (ia == ib)) ? bb - m : 0;
                const int32_t cur_a = (tr & (ia == ib)) ? rb : ba;
                const int32_t sa = (int32_t)((kBankPos >> code) & 1u) - (int32_t)((kBankNeg >> code) & 1u);
                const int32_t ra = pa ? cur_a - sa * m : 0;
                const int32_t fb = tr ? rb : bb;
                s_bal[ib][lane] = fb;                  // a no-op unless Transfer
                s_bal[ia][lane] = ra;                  // written last (ia == ib)
                ex = (ex & ~((1u << ia) | (tr << ib))) | (pa << ia) | ((tr & pb) << ib);
                const int32_t vb = ia == ib ? ra : fb;
                neg &= ~((1u << ia) | (1u << ib));
                neg |= ((ra < 0) ? ((ex >> ia) & 1u) : 0u) << ia;
                neg |= ((vb < 0) ? ((ex >> ib) & 1u) : 0u) << ib;
            } else {
                RS &= ~(1u << depth);
            }
            cand = cands(rem, INV, RESP) & ~below32(j + 1u);
            found = 1u;
            if (!cand) return -1;
        }
        // ---- try the next candidate: straight-line, predicated
        const uint32_t j = (uint32_t)__builtin_ctz(cand);
        cand &= cand - 1u;
        const uint32_t pmj = same_pid(j);
        const uint32_t rr = rem & pmj & RESP;
        const bool has = rr != 0u;             // findResponse => [] : no child
        const uint32_t r = (uint32_t)__builtin_ctz(rr | 0x80000000u);
        const uint32_t cj = evc[j * STRIDE], cr = evc[r * STRIDE];
        const uint32_t code = c_code(cj), rc = c_code(cr);
        const int32_t m = c_val(cj), rv = c_val(cr);
        bool ok, err;
        uint32_t stw;
        if constexpr (BANK) {
            const uint32_t ia = c_a(cj), ib = c_b(cj);
            const int32_t bal_a = s_bal[ia][lane], bal_b = s_bal[ib][lane];
            const uint32_t ex_a = (ex >> ia) & 1u, ex_b = (ex >> ib) & 1u;
            // post (test/Bank.hs:118-131): invariant && expected response
            const uint32_t tr = code == QSMD_BANK_TRANSFER ? 1u : 0u;
            const bool chk = code == QSMD_BANK_CHECK_BALANCE;
            const uint32_t ge = (ex_a & (bal_a >= m ? 1u : 0u));   // lookup >= Just m
            const uint32_t exp = (uint32_t)(kBankExp >> (3u * (code * 4u + ex_a * 2u + ge))) & 7u;
            const bool inv_ok = neg == 0u;
            err = has & inv_ok & chk & (rc == QSMD_BANK_BALANCE) & !ex_a;   // Map.! raises
            ok = has & inv_ok & (rc == exp) & (!chk | (rv == bal_a));
            // next' (test/Bank.hs:92-101) on a, then Transfer's deposit on b;
            // stored unconditionally (the old values when !ok)
            stw = j | (ex_a << 5) | (ex_b << 6);
            const int32_t sa = (int32_t)((kBankPos >> code) & 1u) - (int32_t)((kBankNeg >> code) & 1u);
            const int32_t na = ex_a ? bal_a + sa * m : (sa != 0 ? m : 0);
            const uint32_t ex1 = ex | ((chk ? 0u : 1u) << ia);
            const int32_t bo = ia == ib ? na : bal_b;
            const int32_t nb = ((ex1 >> ib) & 1u) ? bo + m : m;
            const int32_t fb = tr ? nb : bo;
            s_bal[ia][lane] = ok ? na : bal_a;
            s_bal[ib][lane] = ok ? fb : bal_b;
            const uint32_t ex2 = ex1 | (tr << ib);
            const int32_t va = ia == ib ? fb : na;
            uint32_t neg2 = neg & ~((1u << ia) | (1u << ib));
            neg2 |= ((va < 0) ? ((ex2 >> ia) & 1u) : 0u) << ia;
            neg2 |= ((fb < 0) ? ((ex2 >> ib) & 1u) : 0u) << ib;
            ex = ok ? ex2 : ex;
            neg = ok ? neg2 : neg;
        } else {
            // model at this depth: Just (#TT since the last Reset), or model0
            // advanced by succ <$> once per level
            const uint32_t m0_just = a.m0_just;
            const int32_t m0_n = (int32_t)a.m0_val[0];
            const uint32_t just = RS ? 1u : m0_just;
            const int32_t tn = RS ? (int32_t)(depth - 1u - (31u - __builtin_clz(RS | 1u)))
                                  : m0_n + (m0_just ? (int32_t)depth : 0);
            // postcondition (test/TicketDispenser.hs:99-102)
            const bool tt = code == QSMD_TICKET_TAKE_TICKET;
            err = false;
            ok = has & (tt ? (rc == QSMD_TICKET_NUMBER) & (just != 0u) & (rv == tn + 1) : rc == QSMD_TICKET_OK);
            stw = j;
            RS |= ((ok & !tt) ? 1u : 0u) << depth;   // transition: Reset => Just 0
        }
        // budget before the node is counted, then Map.! (rare exit)
        const bool over = has & (nodes >= limit);
        if (over | err) {
            nodes += over ? 0u : 1u;
            return over ? QSMD_STATUS_BUDGET : QSMD_STATUS_MODEL_ERROR;
        }
        nodes += has ? 1u : 0u;
        found |= has ? 1u : 0u;
        // descend on success
        stk.put(ok ? depth : 64u, stw);
        depth += ok ? 1u : 0u;
        const uint32_t fi = rem & pmj & INV;
        const uint32_t rem2 = rem & ~((fi & (0u - fi)) | (1u << r));
        rem = ok ? rem2 : rem;
        cand = ok ? cands(rem2, INV, RESP) : cand;
        found = ok ? 0u : found;
        return -1;
    }

    __device__ __forceinline__ void write_witness(uint8_t* w, uint32_t n_ev) const {
        for (uint32_t d = 0; d < depth; ++d) w[d] = (uint8_t)(stk.get(d) & 31u);
        if (depth < n_ev) w[depth] = QSMD_WITNESS_END;
    }
};

__device__ __forceinline__ bool time_up(const SearchArgs& a, uint64_t t0, uint32_t& iter) {
    return a.time_limit && ((++iter & 1023u) == 0u) && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit;
}

// Wave-aggregated append of h to list (one atomic per wavefront).
__device__ __forceinline__ void wave_append(bool pred, uint32_t h, uint32_t* list, uint32_t* count, int lane) {
    const uint64_t dm = __ballot(pred);
    if (dm) {
        const int leader = __builtin_ctzll(dm);
        uint32_t slot = 0;
        if (lane == leader) slot = atomicAdd(count, (uint32_t)__builtin_popcountll(dm));
        slot = __shfl(slot, leader, 64);
        if (pred) list[slot + lane_prefix(dm)] = h;
    }
}

struct Counters {
    uint32_t lin = 0, nonlin = 0, err = 0, enc = 0, budget = 0;
    uint64_t nodes = 0;
    __device__ __forceinline__ void add(int status, uint64_t n) {
        if (status == QSMD_STATUS_SKIPPED) return;     // counted by early_exit_fixup
        lin += status == QSMD_STATUS_LINEARISABLE;
        nonlin += status == QSMD_STATUS_NONLINEARISABLE;
        err += status == QSMD_STATUS_MODEL_ERROR;
        enc += status == QSMD_STATUS_ENCODE_ERROR;
        budget += status == QSMD_STATUS_BUDGET;
        nodes += n;
    }
    __device__ __forceinline__ void flush(unsigned long long* partials, int lane) const {
        const uint64_t t_lin = wave_sum64(lin), t_non = wave_sum64(nonlin), t_err = wave_sum64(err),
                       t_enc = wave_sum64(enc), t_bud = wave_sum64(budget), t_nodes = wave_sum64(nodes);
        if (lane == 0) {
            unsigned long long* p = partials + (uint64_t)blockIdx.x * T_N;
            p[T_CHECKED] = t_lin + t_non + t_err;
            p[T_LIN] = t_lin;
            p[T_NONLIN] = t_non;
            p[T_ERR] = t_err;
            p[T_ENC] = t_enc;
            p[T_BUDGET] = t_bud;
            p[T_SKIPPED] = 0;
            p[T_NODES] = t_nodes;
        }
    }
};

}  // namespace

// -------------------------------------------------------------- stage 0

// STAMP = diagnostic build: lane 0 accumulates s_memtime deltas of the
// phases (header+staging, search, output, groups) into a.stamps[block][0..3]
// and records its residency (realtime start/end, HW_ID, XCC_ID) in [4..7].
template <uint32_t MODEL, bool STAMP>
__global__ __launch_bounds__(C_LANES) void compact_search(SearchArgs a) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    __shared__ uint32_t s_ev[C_MAXEV][C_LANES];
    __shared__ int32_t s_bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][C_LANES];
    __shared__ uint32_t s_flag[C_LANES];

    const int lane = threadIdx.x;
    const uint64_t total = a.n_hist;
    Counters cnt;
    const uint64_t t0 = a.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t user_limit = a.max_nodes ? a.max_nodes : ~0ull;
    const bool tiered = a.stage0_budget < user_limit && a.heavy_list != nullptr;
    const uint64_t limit = tiered ? a.stage0_budget : user_limit;
    uint64_t st_acc[4] = {0, 0, 0, 0}, ts_a = 0, ts_b = 0;
    const uint64_t rt0 = STAMP ? __builtin_amdgcn_s_memrealtime() : 0;

    for (uint64_t base = (uint64_t)blockIdx.x * C_LANES; base < total;
         base += (uint64_t)gridDim.x * C_LANES) {
        if constexpr (STAMP) ts_a = __builtin_amdgcn_s_memtime();
        const uint64_t idx = base + lane;
        const bool active = idx < total;
        const uint32_t h = (uint32_t)idx;
        qsmd_hdr H;
        if (active) H = a.hdr[h];
        else H = qsmd_hdr{0, 0, 0, 0, 0, 0};
        const uint32_t n_ev = H.n_ev, n_pid = H.n_pid;
        const bool enc_ok = active && H.model_id == MODEL && n_ev <= QSMD_MAX_EVENTS &&
                            n_pid <= QSMD_MAX_PIDS && (uint64_t)H.ev_off + n_ev <= a.n_events;
        const bool small = enc_ok && n_ev <= (uint32_t)C_MAXEV && n_pid <= 8u && a.m0_small;

        Staged s{0u, 0u, 0u, 0u, 0u, enc_ok, small};
        const uint32_t N0 = __builtin_amdgcn_readfirstlane(n_ev);
        const uint32_t off0 = __builtin_amdgcn_readfirstlane(H.ev_off);
        const bool lane_uni = active && small && n_ev == N0 && H.ev_off == off0 + (uint32_t)lane * N0;
        const bool packed = __ballot(!lane_uni) == 0ull && N0 > 0u;
        if (packed) stage_packed<MODEL>(a, N0, off0, n_ev, n_pid, s_ev, s_flag, lane, s);
        else if (small) stage_lane<MODEL>(a, H, s_ev, lane, s);

        const bool defer = enc_ok && (!small || (s.ok && !s.fits));
        if constexpr (STAMP) {
            ts_b = __builtin_amdgcn_s_memtime();
            st_acc[0] += ts_b - ts_a;
        }
        wave_append(defer, h, a.defer_list, a.defer_count, lane);   // -> stage 1
        if (!active || defer) continue;

        int status = -1;
        LaneDFS<MODEL> dfs;
        dfs.depth = 0;
        dfs.nodes = 0;
        if (!s.ok) {
            status = QSMD_STATUS_ENCODE_ERROR;
        } else if (n_ev == 0) {
            status = QSMD_STATUS_LINEARISABLE;                       // :59
        } else if (beyond_first_fail(a, h)) {
            status = QSMD_STATUS_SKIPPED;
        } else {
            dfs.init(s, a, s_bal, lane);
            uint32_t iter = 0;
            while ((status = dfs.template step<C_LANES>(a, &s_ev[0][lane], s_bal, lane, limit)) < 0) {
                if (((iter + 1u) & 1023u) == 0u && beyond_first_fail(a, h)) {
                    status = QSMD_STATUS_SKIPPED;
                    break;
                }
                if (time_up(a, t0, iter)) {
                    atomicOr(a.timed_out, 1u);
                    status = QSMD_STATUS_BUDGET;
                    break;
                }
            }
        }
        note_failure(a, h, status);
        if constexpr (STAMP) {
            ts_a = __builtin_amdgcn_s_memtime();
            st_acc[1] += ts_a - ts_b;
        }
        // over the stage-0 budget (not the caller's): restart in the refill stage
        const bool heavy = tiered && status == QSMD_STATUS_BUDGET && dfs.nodes >= limit;
        wave_append(heavy, h, a.heavy_list, a.heavy_count, lane);
        if (heavy) continue;

        a.status[h] = (uint8_t)status;
        if (a.nodes) a.nodes[h] = dfs.nodes;
        if (a.witness && status == QSMD_STATUS_LINEARISABLE) dfs.write_witness(a.witness + H.ev_off, n_ev);
        cnt.add(status, dfs.nodes);
        if constexpr (STAMP) {
            st_acc[2] += __builtin_amdgcn_s_memtime() - ts_a;
            st_acc[3] += 1;
        }
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
                    Staged s{0u, 0u, 0u, 0u, 0u, true, true};
                    if (small) stage_lane<MODEL>(a, H, s_ev, lane, s);   // (list mode: validated by stage 0)
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
            int status = dfs.template step<C_LANES>(a, &s_ev[0][lane], s_bal, lane, limit);
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
