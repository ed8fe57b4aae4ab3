// lane.h -- the per-lane search machinery shared by the compact-domain
// kernels (csrc/compact.hip: stages 0 and 0w; csrc/memo.hip: the heavy
// stage in lane mode): the compressed event format, the staging paths, and LaneDFS, the reference
// DFS (src/Linearisability.hs:25-69 over the Lemma L1 event bitset) as a
// per-lane state machine for histories of at most 32 (G32) or 64 (G64)
// events and 8 pids.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "internal.h"
#include "models.h"

namespace qsmd {

namespace {


constexpr int C_MAXEV = 32;
constexpr int C_LANES = 64;
constexpr int C_CHUNK = 16;
constexpr int32_t V19_MIN = -(1 << 18), V19_MAX = (1 << 18) - 1;   // model0 values (api.hip m0_small)

// compressed event (one u32 per event, LDS [event][lane]):
//   invocation  pid 3 | 0 | code 3 | 0 (5 bits) | a 3 | 0 (5) | b 3 | val 9 (signed)
//   response    pid 3 | 1 | code 3 | val 25 (signed)
// (the invocation's fields where lo >> 4 puts them; Bank money in the
// reference comes from QuickCheck's getPositive at sizes <= 100,
// test/Bank.hs:139-144)
// Staging writes a marker instead of an event it cannot hold: an invocation
// with code 7 (not an encodable event: ENCODE_ERROR) or code 6 (a value
// outside the ranges above: the history goes to the next stage), or code 6
// with bit 7 set (an event with a field of 8 or more -- an encode error, or
// a legal event with junk in a field its constructor does not use -- that
// finish_lane classifies from the raw event: ENCODE_ERROR or the next stage).
constexpr int32_t IVAL_BITS = 9, RVAL_BITS = 25;
constexpr uint32_t MARK_BAD = 0x70u, MARK_WIDE = 0x60u, MARK_SUSP = 0xE0u;
// the illegal (resp, code) pairs of a model, bit resp | code << 1: Bank
// invocations 0..4 and every response code 0..7 are legal, Ticket 0..1 both
template <uint32_t MODEL>
constexpr uint32_t kCodeBad = (MODEL == QSMD_MODEL_TICKET ? 0xFu : 0xABFFu) ^ 0xFFFFu;
// Geometry of a compact stage: <= 32 events (u32 event masks, 16 levels,
// stack entries j 5 bits) or <= 64 events (u64, 32 levels, j 6 bits).  The
// event words are the same.
struct G32 {
    using M = uint32_t;
    static constexpr int EV = 32, RB = 5, IVB = IVAL_BITS, LEVELS = 16;
};
struct G64 {
    using M = uint64_t;
    static constexpr int EV = 64, RB = 6, IVB = IVAL_BITS, LEVELS = 32;
};

__device__ __forceinline__ uint32_t c_code(uint32_t w) { return (w >> 4) & 7u; }
__device__ __forceinline__ uint32_t c_a(uint32_t w) { return (w >> 12) & 7u; }
__device__ __forceinline__ uint32_t c_b(uint32_t w) { return (w >> 20) & 7u; }
template <class G = G32>
__device__ __forceinline__ int32_t c_ival(uint32_t w) { return (int32_t)w >> (32 - G::IVB); }
__device__ __forceinline__ int32_t c_rval(uint32_t w) { return (int32_t)w >> (32 - RVAL_BITS); }

__device__ __forceinline__ uint32_t below32(uint32_t r) { return (uint32_t)((1ull << r) - 1ull); }

__device__ __forceinline__ uint64_t below64(uint32_t r) { return r >= 64u ? ~0ull : (1ull << r) - 1ull; }
__device__ __forceinline__ uint32_t mask_below(uint32_t r, uint32_t) { return below32(r); }
__device__ __forceinline__ uint64_t mask_below(uint32_t r, uint64_t) { return below64(r); }
__device__ __forceinline__ uint32_t m_ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
__device__ __forceinline__ uint32_t m_ctz(uint64_t x) { return (uint32_t)__builtin_ctzll(x); }
__device__ __forceinline__ uint32_t m_hibit(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }
__device__ __forceinline__ uint32_t m_hibit(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }
// the highest set bit of x != 0 as a mask (v_ffbh + one shift)
__device__ __forceinline__ uint32_t m_topbit(uint32_t x) { return 0x80000000u >> __builtin_clz(x); }
__device__ __forceinline__ uint64_t m_topbit(uint64_t x) { return 0x8000000000000000ull >> __builtin_clzll(x); }

// candidates: remaining invocations before the first remaining response
// (takeInvocations, src/Linearisability.hs:25-28); branch-free
// ((rr & -rr) - 1: the bits below the lowest remaining response; all ones
// when none remains)
__device__ __forceinline__ uint32_t cands(uint32_t rem, uint32_t INV, uint32_t RESP) {
    const uint32_t rr = rem & RESP;
    return rem & INV & ((rr & (0u - rr)) - 1u);
}
__device__ __forceinline__ uint64_t cands(uint64_t rem, uint64_t INV, uint64_t RESP) {
    const uint64_t rr = rem & RESP;
    return rem & INV & ((rr & (0ull - rr)) - 1ull);
}
// the bits above j (j < width)
__device__ __forceinline__ uint32_t mask_above(uint32_t j, uint32_t) { return ~1u << j; }
__device__ __forceinline__ uint64_t mask_above(uint32_t j, uint64_t) { return ~1ull << j; }

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
// The same table folded to 3 bits x (code, sel) with sel = exists a for
// OpenAccount and lookup a >= Just m otherwise (a 30-bit word: one v_bfe).
constexpr uint32_t bank_exp2_table() {
    uint32_t t = 0;
    for (uint32_t code = 0; code < 5; ++code)
        for (uint32_t sel = 0; sel < 2; ++sel) {
            // Open: sel = exists a; otherwise sel = ge (which implies exists a)
            const uint32_t exa = sel, ge = code == QSMD_BANK_OPEN_ACCOUNT ? 0u : sel;
            t |= (uint32_t)((kBankExp >> (3 * (code * 4 + exa * 2 + ge))) & 7u) << (code * 6 + sel * 3);
        }
    return t;
}
constexpr uint32_t kBankExp2 = bank_exp2_table();
// per request code, the sign of the step on account a as a 2-bit signed
// field (Deposit +1, Withdraw and Transfer -1, Open / CheckBalance 0)
constexpr uint32_t kBankSign = (1u << (2 * QSMD_BANK_DEPOSIT)) | (3u << (2 * QSMD_BANK_WITHDRAW)) |
                               (3u << (2 * QSMD_BANK_TRANSFER));
__device__ __forceinline__ int32_t bank_sign(uint32_t code) {
    return __builtin_amdgcn_sbfe((int32_t)kBankSign, code * 2u, 2u);
}

// (x & m) | y as one v_and_or_b32 (hipcc makes two of them two ands and an or3)
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t m, uint32_t y) {
    uint32_t d;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(d) : "v"(x), "s"(m), "v"(y));
    return d;
}

// (x << s) | y as one v_lshl_or_b32 (hipcc merges two of them into
// shifts and an or3)
__device__ __forceinline__ uint32_t lshl_or(uint32_t x, uint32_t s, uint32_t y) {
    uint32_t d;
    asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(d) : "v"(x), "v"(s), "v"(y));
    return d;
}

__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// include/qsmd.h encoding rules, branch-free (the pid range is checked
// against the header's n_pid by finish_lane).  As bit tests on the event's
// lo word (kp | code << 8 | a << 16 | b << 24): pid < 8 = bits 3-6 clear;
// Ticket code <= 1 = bits 9-15 clear; Bank response code <= 7 = bits 11-15
// clear; Bank request code <= 4, account a < 8 = bits 19-23 clear, and for a
// Transfer b < 8 = bits 27-31 clear.
template <uint32_t MODEL>
__device__ __forceinline__ bool valid_bits(uint32_t lo) {
    if constexpr (MODEL == QSMD_MODEL_TICKET) {
        return (lo & 0xFE78u) == 0u;
    } else {
        // a request is bad when (code << 5 | b >> 3) > (Transfer << 5): code > 4,
        // or a Transfer with b >= 8
        const bool resp = (lo & 0x80u) != 0u;
        const uint32_t bits = lo & (resp ? 0xF878u : 0x00F80078u);
        const uint32_t req = resp ? 0u : ((((lo >> 8) & 0xFFu) << 5) | (lo >> 27));
        return (bits | (req > (QSMD_BANK_TRANSFER << 5) ? 1u : 0u)) == 0u;
    }
}

// The compressed word of one event, or a marker.  For a `plain` event --
// pid, code, a and b each below 8, the only events encoders write -- the
// invocation is lo >> 4 with the pid put back in its low bits (a bit
// insert) and the value above, the response keeps the low 7 bits, and a
// legal code is one table bit; a value fits when the word's value field
// sign-extends back to it.  Anything else is MARK_SUSP, classified from the
// raw event by finish_lane (an encode error, or a legal event for the next
// stage: junk in a field its constructor does not use, a value too wide).
template <uint32_t MODEL, class G = G32>
__device__ __forceinline__ uint32_t compress(uint32_t lo, int32_t val) {
    static_assert(32 - G::IVB == 23 && 32 - RVAL_BITS == 7, "value field shifts");
    uint32_t t;                                                       // pid | resp << 3 | code << 4 | a << 12 | b << 20
    asm("v_bfi_b32 %0, 7, %1, %2" : "=v"(t) : "v"(lo), "v"(lo >> 4));   // (hipcc emits and + and_or)
    const uint32_t sh = 23u - (__builtin_amdgcn_ubfe(lo, 7u, 1u) << 4);   // response: 7
    // a plain invocation's t is below 2^23; a response keeps pid | 1 | code
    const uint32_t w = ((uint32_t)val << sh) | __builtin_amdgcn_ubfe(t, 0u, sh);
    const bool fit = ((int32_t)w >> sh) == val;
    // (resp | code << 1 | code bit 3 << 4: bit 11 is in the field mask too)
    const uint32_t bad = __builtin_amdgcn_ubfe(kCodeBad<MODEL> | 0xFFFF0000u, __builtin_amdgcn_ubfe(lo, 7u, 5u), 1u);
    const bool plain = ((lo & 0xF8F8F878u) | bad) == 0u;
    return (plain & fit) ? w : MARK_SUSP;
}

// The DFS stack: LEVELS entries x 8 bits in NW VGPRs, kept as a shift
// register -- the top entry is byte 0, a push shifts every word up by one byte
// (v_alignbit), a pop down -- so push and pop cost one instruction per word
// and no indexing.  Entry d of a stack of depth n is byte n - 1 - d (get()),
// used off the hot path only; there the selection goes through an empty asm
// so hipcc keeps it a register select (it otherwise turns the select tree
// into a scratch-memory indexed load).
template <int NW>
struct StackN {
    uint32_t w[NW];
    __device__ __forceinline__ uint32_t word(uint32_t k) const {
        if constexpr (NW == 4) {
            uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3];
            asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
            const uint32_t lo = (k & 1u) ? x1 : x0, hi = (k & 1u) ? x3 : x2;
            return (k & 2u) ? hi : lo;
        } else {
            uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4], x5 = w[5], x6 = w[6], x7 = w[7];
            asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
            asm volatile("" : "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
            const uint32_t a0 = (k & 1u) ? x1 : x0, a1 = (k & 1u) ? x3 : x2, a2 = (k & 1u) ? x5 : x4,
                           a3 = (k & 1u) ? x7 : x6;
            const uint32_t b0 = (k & 2u) ? a1 : a0, b1 = (k & 2u) ? a3 : a2;
            return (k & 4u) ? b1 : b0;
        }
    }
    // entry d (from the bottom) of a stack holding n entries
    __device__ __forceinline__ uint32_t get(uint32_t d, uint32_t n) const {
        const uint32_t pos = n - 1u - d;
        return (word(pos >> 2) >> ((pos & 3u) * 8u)) & 0xFFu;
    }
    __device__ __forceinline__ uint32_t top() const { return w[0] & 0xFFu; }
    __device__ __forceinline__ void pop() {
#pragma unroll
        for (int q = 0; q + 1 < NW; ++q) w[q] = __builtin_amdgcn_alignbit(w[q + 1], w[q], 8u);
        w[NW - 1] >>= 8;
    }
    // push v (< 256) when c: one v_perm per word with a per-lane byte
    // selector (the shifted word when c, the word itself otherwise)
    // (in place, top word first: no temporaries)
    __device__ __forceinline__ void push_if(bool c, uint32_t v) {
        const uint32_t keep = 0x07060504u;
        const uint32_t sel0 = c ? 0x06050400u : keep, sel = c ? 0x06050403u : keep;
#pragma unroll
        for (int q = NW - 1; q >= 1; --q) w[q] = __builtin_amdgcn_perm(w[q], w[q - 1], sel);
        w[0] = __builtin_amdgcn_perm(w[0], v, sel0);
    }
};

template <class M>
struct StagedT {
    M INV, RESP, P0, P1, P2;
    bool ok, fits;
};
using Staged = StagedT<uint32_t>;

// One lane stages its own history: C_CHUNK loads in flight (index clamped
// into the history, no exec-masked branches), compress into its LDS column.
template <uint32_t MODEL, class G = G32>
__device__ __forceinline__ void stage_lane(const SearchArgs& a, const qsmd_hdr& H, uint32_t (*s_ev)[C_LANES],
                                           int lane) {
    const uint32_t n_ev = H.n_ev;
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
        for (uint32_t k = 0; k < (uint32_t)C_CHUNK; ++k)
            if (c0 + k < n_ev) s_ev[c0 + k][lane] = compress<MODEL, G>(x[k].x, (int32_t)x[k].y);
    }
}

// The whole wavefront stages 64 histories packed back to back with one
// common length N0 starting at event off0: the 64*N0-event block is read
// with fully coalesced 16-byte loads (a per-lane history walk touches 64
// cache lines per wave instruction), each event is compressed and written
// to its history's lane column.
__device__ __forceinline__ uint32_t magic_div(uint32_t N0) { return (uint32_t)(0xFFFFFFFFull / N0) + 1u; }

// The block's loads go 4 x 16 B per lane at a time (the stage is bound by
// VALU issue, not by these round trips: 8 or 16 at a time measured no
// faster).  A power-of-two length (the common packed batch) maps block event
// g to its history (= column) by a shift.
template <uint32_t MODEL, class G, bool POW2>
__device__ __forceinline__ void stage_packed_body(const SearchArgs& a, uint32_t N0, uint32_t off0, uint32_t nh,
                                                  uint32_t (*s_ev)[C_LANES], int lane) {
    // history of block event g: exact for g < 2^16 (g * N0 < 2^21 << 2^32)
    const uint32_t mg = POW2 ? 0u : magic_div(N0);
    const uint32_t sh = POW2 ? (uint32_t)__builtin_ctz(N0) : 0u;
    auto col_of = [&](uint32_t g, uint32_t& e) {
        const uint32_t hh = POW2 ? g >> sh : __umulhi(g, mg);
        e = POW2 ? g & (N0 - 1u) : g - hh * N0;
        return hh;
    };
    constexpr uint32_t U = 4;
    const uint32_t total_ev = nh * N0;
    if (((off0 | total_ev) & 1u) == 0u) {         // 16-B aligned start, whole 16-B pairs
        const uint4* blk = reinterpret_cast<const uint4*>(a.events + off0);
        const uint32_t nq = total_ev / 2u;
        const uint32_t e_lane = POW2 ? (2u * (uint32_t)lane) & (N0 - 1u) : 0u;
        const uint32_t c_lane = POW2 ? (2u * (uint32_t)lane) >> sh : 0u;
        // U x 64 pairs per step: full steps without per-element guards, then the rest
        auto step = [&](uint32_t k0, auto guard) {
            constexpr bool GUARD = decltype(guard)::value;
            uint4 x[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint32_t q = k0 + u * 64u + (uint32_t)lane;
                // non-temporal: the events are read once per call (they
                // need not displace the memo tables and saved states in L2;
                // the driver's command 8.66 vs 8.63e9 over 8 rounds, 200
                // steps 9.87-9.93 vs 9.83-9.89e9, tools/gpu/archive/r05_nt.sh)
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                if (!GUARD || q < nq) {
                    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(&blk[q]));
                    x[u] = make_uint4(v.x, v.y, v.z, v.w);
                } else {
                    x[u] = make_uint4(0u, 0u, 0u, 0u);
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint32_t q = k0 + u * 64u + (uint32_t)lane;
                uint32_t e0, e1, c0, c1;
                if constexpr (POW2) {
                    // an even power-of-two length N0 <= 64: both events of the
                    // pair in one history (one ds_write2 per pair), the event
                    // index the lane's own constant (2 (k0 + 64 u) is a multiple
                    // of N0) and the column a wave-uniform part plus the lane's
                    e0 = e_lane;
                    e1 = e_lane + 1u;
                    c0 = ((2u * (k0 + u * 64u)) >> sh) + c_lane;
                    c1 = c0;
                } else {
                    c0 = col_of(2u * q, e0);
                    c1 = col_of(2u * q + 1u, e1);
                }
                if (!GUARD || q < nq) {
                    s_ev[e0][c0] = compress<MODEL, G>(x[u].x, (int32_t)x[u].y);
                    s_ev[e1][c1] = compress<MODEL, G>(x[u].z, (int32_t)x[u].w);
                }
            }
        };
        uint32_t k0 = 0;
        for (; k0 + U * 64u <= nq; k0 += U * 64u) step(k0, std::false_type{});
        if (k0 < nq) step(k0, std::true_type{});
    } else {
        const uint2* blk = a.events + off0;
        auto step = [&](uint32_t k0, auto guard) {
            constexpr bool GUARD = decltype(guard)::value;
            uint2 x[2u * U];
#pragma unroll
            for (uint32_t u = 0; u < 2u * U; ++u) {
                const uint32_t g = k0 + u * 64u + (uint32_t)lane;
                x[u] = (!GUARD || g < total_ev) ? blk[g] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < 2u * U; ++u) {
                const uint32_t g = k0 + u * 64u + (uint32_t)lane;
                uint32_t e;
                const uint32_t c = col_of(g, e);
                if (!GUARD || g < total_ev) s_ev[e][c] = compress<MODEL, G>(x[u].x, (int32_t)x[u].y);
            }
        };
        uint32_t k0 = 0;
        for (; k0 + 2u * U * 64u <= total_ev; k0 += 2u * U * 64u) step(k0, std::false_type{});
        if (k0 < total_ev) step(k0, std::true_type{});
    }
}

// nh histories packed back to back with one common length N0 from event
// off0, history hh to column hh
template <uint32_t MODEL, class G = G32>
__device__ __forceinline__ void stage_packed(const SearchArgs& a, uint32_t N0, uint32_t off0, uint32_t nh,
                                             uint32_t (*s_ev)[C_LANES], int lane) {
    if ((N0 & (N0 - 1u)) == 0u && N0 >= 2u) stage_packed_body<MODEL, G, true>(a, N0, off0, nh, s_ev, lane);
    else stage_packed_body<MODEL, G, false>(a, N0, off0, nh, s_ev, lane);
}

// Per lane, over its own column (evp: its raw events, read only for a
// MARK_SUSP): the encoding checks (markers, pid < n_pid) and the register masks (RESP / INV, the pid bit slices), 8 events
// at a time with the event index wave-uniform (the calling lanes' longest
// history bounds the loop: no indexed registers, no per-event branches).
// No pairing: the compact stages search every history on the general path
// (pid masks), which costs less per DFS step than pairing the invocations
// at staging costs per event (A/B in flight, config 2: 6.44e9 vs 6.10e9
// histories/s).  Words beyond n_ev (stale) are masked out by ALL.
template <uint32_t MODEL, class G = G32>
__device__ __forceinline__ void finish_lane(uint32_t (*s_ev)[C_LANES], int lane, uint32_t n_ev, uint32_t n_pid,
                                            const uint2* evp, StagedT<typename G::M>& s) {
    using M = typename G::M;
    constexpr uint32_t U = 8;
    // a ballot max: the callers may be a subset of the wavefront
    const uint32_t n_cl = min(n_ev, (uint32_t)G::EV);
    uint32_t n_max = 0;
#pragma unroll
    for (int b = 6; b >= 0; --b) {
        const uint32_t t = n_max | (1u << b);
        n_max = __ballot(n_cl >= t) ? t : n_max;
    }
    const M ALL = mask_below(n_ev, (M)0);
    // Per 8 events: their low nibbles (pid bits 0-2, resp bit 3) packed 4
    // bits apart, then split into the 4 bit planes by shifts (8 bits each);
    // the marker test (an invocation with code 6 or 7: bits 5 and 6 set, bit
    // 3 clear) as one bit per event.  BAD / WIDE apart only when some lane
    // of the wavefront has a marker (injected inputs; never in a clean batch).
    M RESP = 0, P0 = 0, P1 = 0, P2 = 0, MK = 0;
    auto plane8 = [](uint32_t nib, uint32_t b) {   // bits b, b+4, ..., b+28 -> bits 0..7
        uint32_t t = (nib >> b) & 0x11111111u;
        t = (t | (t >> 3)) & 0x03030303u;
        t = (t | (t >> 6)) & 0x000F000Fu;
        return (t | (t >> 12)) & 0xFFu;
    };
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < n_max; c0 += U) {
        uint32_t W[U];
#pragma unroll
        for (uint32_t k = 0; k < U; ++k) W[k] = s_ev[c0 + k][lane];
        // the low bytes of the even / odd events, four to a word (v_perm;
        // selector 0x0C = a zero byte): x0 = [w0, w2, w4, w6], x1 = [w1, w3, w5, w7]
        const uint32_t x0 = __builtin_amdgcn_perm(W[2], W[0], 0x0C0C0400u) |
                            __builtin_amdgcn_perm(W[6], W[4], 0x04000C0Cu);
        const uint32_t x1 = __builtin_amdgcn_perm(W[3], W[1], 0x0C0C0400u) |
                            __builtin_amdgcn_perm(W[7], W[5], 0x04000C0Cu);
        const uint32_t nib = (x0 & 0x0F0F0F0Fu) | ((x1 & 0x0F0F0F0Fu) << 4);    // event k at bits 4k..4k+3
        // marker bytes (bits 5, 6 set, 3 clear) at bit 6 of each byte, then
        // one bit per event: m has events 0, 1 at bits 0, 1, 2, 3 at 8, 9, ...
        const uint32_t y0 = x0 & (x0 << 1) & ~(x0 << 3) & 0x40404040u;
        const uint32_t y1 = x1 & (x1 << 1) & ~(x1 << 3) & 0x40404040u;
        const uint32_t m = (y0 >> 6) | (y1 >> 5);
        const uint32_t z = m | (m >> 6);                                         // events 0-3 at 0-3, 4-7 at 16-19
        const uint32_t mk = (z & 0xFu) | ((z >> 12) & 0xF0u);
        RESP |= (M)plane8(nib, 3) << c0;
        P0 |= (M)plane8(nib, 0) << c0;
        P1 |= (M)plane8(nib, 1) << c0;
        P2 |= (M)plane8(nib, 2) << c0;
        MK |= (M)mk << c0;
    }
    M BAD = 0, WIDE = 0;
    if (__ballot((MK & ALL) != (M)0)) {
#pragma unroll 1
        for (uint32_t e = 0; e < n_max; ++e) {
            uint32_t mkw = s_ev[e][lane] & 0xF8u;
            // (a MARK_SUSP event: illegal => ENCODE_ERROR, legal => the next stage)
            if (mkw == MARK_SUSP && e < n_ev) mkw = valid_bits<MODEL>(evp[e].x) ? MARK_WIDE : MARK_BAD;
            BAD |= (M)(mkw == MARK_BAD ? 1u : 0u) << e;
            WIDE |= (M)(mkw == MARK_WIDE ? 1u : 0u) << e;
        }
    }
    RESP &= ALL;
    P0 &= ALL;
    P1 &= ALL;
    P2 &= ALL;
    // events whose pid is >= n_pid (pid q's events from the bit slices)
    M GEP = 0;
#pragma unroll
    for (uint32_t q = 0; q < 8u; ++q) {
        const M pq = ((q & 1u) ? P0 : ~P0) & ((q & 2u) ? P1 : ~P1) & ((q & 4u) ? P2 : ~P2) & ALL;
        GEP |= q >= n_pid ? pq : (M)0;
    }
    s.INV = ALL & ~RESP;
    s.RESP = RESP;
    s.P0 = P0;
    s.P1 = P1;
    s.P2 = P2;
    s.ok = ((BAD & ALL) | GEP) == (M)0;
    s.fits = (WIDE & ALL) == (M)0;
}

// --------------------------------------------------------------- the DFS

// Per-lane search state (registers) over the history in LDS column `lane`.
// step() runs one iteration: an optional backtrack followed by one
// candidate try; it returns -1 to continue or the final QSMD_STATUS_*
// (QSMD_STATUS_BUDGET = `limit` nodes reached before a decision).  Any pid
// pattern: the response and the removed invocation come from the
// bit-sliced pid masks.

template <uint32_t MODEL, class G = G32>
struct LaneDFS {
    static constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    using M = typename G::M;
    static constexpr uint32_t JM = (uint32_t)G::EV - 1u;   // event index mask of a stack entry
    static constexpr uint32_t JB = (uint32_t)G::RB;        // stack entry: j | ex_a << JB | ex_b << JB+1
    M INV, RESP, P0, P1, P2, ALL;
    M rem, cand;
    uint32_t depth, ex, RS, found;
    int32_t neg;            // < 0: some existing balance is negative (the invariant fails)
    uint32_t base;          // depth of the search root (0; the task depth in split_search)
    uint32_t last_j;        // candidate of the most recent try (the one a BUDGET return did not count;
                            // 32: none -- a BUDGET from the time limit, compact.hip run_search)
    uint64_t nodes;
    StackN<G::LEVELS / 4> stk;
    // (Bank, the memo stage's slot hash: memo.hip) the XOR over accounts q of
    // balance q rotated right by 4q, kept by undo / try_next when FOLD -- the
    // probe's slot from registers, the balances read only for a probe that
    // can hit.  Unused (and not computed) by the compact stages.
    uint32_t fold;

    // events whose pid equals the pid of event j (bit-sliced compare); the
    // bits beyond the history are not cleared -- every use ANDs the result
    // with INV or RESP (u32: each slice's bit j sign-extended by one v_bfe_i32,
    // then two 3-input logic ops)
    __device__ __forceinline__ M same_pid(uint32_t j) const {
        if constexpr (sizeof(M) == 4) {
            const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int32_t)P0, j, 1u);
            const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int32_t)P1, j, 1u);
            const uint32_t m2 = (uint32_t)__builtin_amdgcn_sbfe((int32_t)P2, j, 1u);
            return ~((P0 ^ m0) | (P1 ^ m1) | (P2 ^ m2));
        } else {
            const M m0 = (M)0 - ((P0 >> j) & (M)1), m1 = (M)0 - ((P1 >> j) & (M)1), m2 = (M)0 - ((P2 >> j) & (M)1);
            return ~((P0 ^ m0) | (P1 ^ m1) | (P2 ^ m2));
        }
    }

    __device__ __forceinline__ void init(const StagedT<M>& s, const SearchArgs& a, int32_t (*s_bal)[C_LANES],
                                         int lane) {
        INV = s.INV; RESP = s.RESP; P0 = s.P0; P1 = s.P1; P2 = s.P2;
        ALL = INV | RESP;
        rem = ALL;
        cand = cands(rem, INV, RESP);
        depth = 0; found = 0; nodes = 0; RS = 0; base = 0;
#pragma unroll
        for (int q = 0; q < G::LEVELS / 4; ++q) stk.w[q] = 0u;
        ex = a.m0_exists; neg = 0;
        if constexpr (BANK) {
#pragma unroll
            for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) {
                const bool e = (ex >> q) & 1u;
                const int32_t v = e ? (int32_t)a.m0_val[q] : 0;
                s_bal[q][lane] = v;
                neg |= (e && v < 0) ? v : 0;
            }
        }
    }

    // evc[e * STRIDE] = compressed event e (the lane's LDS column: STRIDE = 64;
    // a history shared by the wavefront: STRIDE = 1)
    // Undo the last level: restore the parent node's state exactly
    // (remaining events, model); returns the candidate the level went through.
    template <int STRIDE, bool FOLD = false>
    __device__ __forceinline__ uint32_t undo(const uint32_t* evc, int32_t (*s_bal)[C_LANES], int lane) {
        --depth;
        const uint32_t st = stk.top();
        stk.pop();
        const uint32_t j = st & JM;
        const uint32_t cj = BANK ? evc[j * STRIDE] : 0u;
        const M gone = ~rem & same_pid(j);
        rem |= m_topbit(gone & INV) | m_topbit(gone & RESP);
        if constexpr (BANK) {
            const uint32_t code = c_code(cj), ia = c_a(cj), ib = c_b(cj);
            const int32_t m = c_ival<G>(cj);
            // -(exists a), -(exists b) before the step (the stack entry's bits)
            const int32_t pam = __builtin_amdgcn_sbfe((int32_t)st, JB, 1u);
            const int32_t pbm = __builtin_amdgcn_sbfe((int32_t)st, JB + 1u, 1u);
            const bool tr = code == QSMD_BANK_TRANSFER, same = ia == ib;
            int32_t ba = s_bal[ia][lane], bb = s_bal[ib][lane];
            // both reads in flight together: without this the compiler sinks
            // ba's read into a branch on the pre-op `exists a` bit, a second
            // serial LDS round trip per backtrack
            asm volatile("" : "+v"(ba), "+v"(bb));
            // undo Transfer's deposit on b, then the step on a
            const int32_t rb = (bb - m) & (pbm | (same ? -1 : 0));
            const int32_t cur_a = (tr & same) ? rb : ba;
            const int32_t ra = (cur_a - bank_sign(code) * m) & pam;
            const int32_t fb = tr ? rb : bb;
            s_bal[ib][lane] = fb;                  // a no-op unless Transfer
            s_bal[ia][lane] = ra;                  // written last (ia == ib)
            if constexpr (FOLD) {
                const uint32_t da = (uint32_t)(ba ^ ra), db = same ? 0u : (uint32_t)(bb ^ fb);
                fold ^= __builtin_amdgcn_alignbit(da, da, ia << 2) ^ __builtin_amdgcn_alignbit(db, db, ib << 2);
            }
            // the existence bits of a (and b for Transfer) back to the stack's
            const uint32_t A = 1u << ia, B = tr ? 1u << ib : 0u;
            ex = (ex & ~A) | (A & (uint32_t)pam);
            ex = (ex & ~B) | (B & (uint32_t)pbm);
            // the parent held the invariant (a step descends only when it
            // holds, test/Bank.hs:118), so no existing balance was negative
            neg = 0;
        } else {
            RS &= ~(1u << depth);
        }
        return j;
    }

    // step()'s return for a search that ended (a leaf or the exhausted
    // root): finish() turns it into the outcome once, after the loop
    static constexpr int kTerm = 64;
    __device__ __forceinline__ int finish(int status) const {
        return status != kTerm ? status
                               : ((!found && depth > 0) ? QSMD_STATUS_LINEARISABLE : QSMD_STATUS_NONLINEARISABLE);
    }

    template <int STRIDE>
    __device__ __forceinline__ int step(const SearchArgs& a, const uint32_t* evc,
                                        int32_t (*s_bal)[C_LANES], int lane, uint64_t limit) {
        // one exit at the end (no early returns: the state stays in place
        // across the two halves instead of being copied between paths)
        // no children: a leaf => True (any' []), the root => False (any []);
        // a subtree rooted at depth base > 0 is an inner node of the reference tree
        const bool empty = cand == (M)0;
        const bool term = empty & ((found == 0u) | (depth == base));
        int status = term ? kTerm : -1;    // (the outcome itself: finish())
        if (empty & !term) {
            // ---- backtrack: restore the parent level exactly
            const uint32_t j = undo<STRIDE>(evc, s_bal, lane);
            cand = cands(rem, INV, RESP) & mask_above(j, (M)0);
            found = 1u;
        }
        if (cand) status = try_next<STRIDE>(a, evc, s_bal, lane, limit);
        return status;
    }

    // ---- try the next candidate: straight-line, predicated
    template <int STRIDE, bool FOLD = false>
    __device__ __forceinline__ int try_next(const SearchArgs& a, const uint32_t* evc,
                                            int32_t (*s_bal)[C_LANES], int lane, uint64_t limit) {
        const uint32_t j = m_ctz(cand);
        cand &= cand - (M)1;
        last_j = j;
        const uint32_t cj = evc[j * STRIDE];
        const M pmj = same_pid(j);
        const M rr = rem & pmj & RESP;
        const bool has = rr != (M)0;           // findResponse => [] : no child
        const uint32_t r = m_ctz(rr | ((M)1 << JM));
        const uint32_t cr = evc[r * STRIDE];
        const uint32_t code = c_code(cj), rc = c_code(cr);
        const int32_t m = c_ival<G>(cj), rv = c_rval(cr);
        // budget before the node is counted (a BUDGET return leaves the state
        // untouched, so the search can go on with a larger limit)
        const bool over = has & (nodes >= limit);
        bool ok, err;
        uint32_t stw;
        if constexpr (BANK) {
            const uint32_t ia = c_a(cj), ib = c_b(cj);
            const int32_t bal_a = s_bal[ia][lane], bal_b = s_bal[ib][lane];
            // exm = -(exists a): one v_bfe_i32 serves the test, the stack
            // entry and the masked balance below
            const int32_t exm = __builtin_amdgcn_sbfe((int32_t)ex, ia, 1u);
            const bool ex_a = exm != 0;
            const int32_t exbm = __builtin_amdgcn_sbfe((int32_t)ex, ib, 1u);   // -(exists b)
            // post (test/Bank.hs:118-131): invariant && expected response
            const bool tr = code == QSMD_BANK_TRANSFER;
            const bool chk = code == QSMD_BANK_CHECK_BALANCE;
            const bool same = ia == ib;
            // expected constructor: kBankExp2[code][exists a (Open) / lookup a >= Just m]
            const bool sel = ex_a & ((code == QSMD_BANK_OPEN_ACCOUNT) | (bal_a >= m));
            const uint32_t exp = __builtin_amdgcn_ubfe(kBankExp2, code * 6u + (sel ? 3u : 0u), 3u);
            const bool inv_ok = neg >= 0;
            err = has & inv_ok & chk & (rc == QSMD_BANK_BALANCE) & !ex_a;   // Map.! raises
            // a raising step never descends (an absent account's stored 0
            // would otherwise match `Balance 0`)
            ok = has & !over & inv_ok & !err & (rc == exp) & (!chk | (rv == bal_a));
            // next' (test/Bank.hs:92-101) on a (an absent account is created
            // with m exactly when the step's sign is non-zero: insertWith),
            // then Transfer's deposit on b; stored unconditionally (the old
            // values when !ok)
            stw = and_or((uint32_t)exbm, 2u << JB, and_or((uint32_t)exm, 1u << JB, j));
            const int32_t sa = bank_sign(code);
            const int32_t na = (bal_a & exm) + (sa & (exm | 1)) * m;
            const int32_t bo = same ? na : bal_b;
            // Transfer: b (0 when absent; the stepped a when b == a) + m
            const int32_t fb = tr ? (same ? na : (bal_b & exbm)) + m : bo;
            s_bal[ia][lane] = ok ? na : bal_a;
            s_bal[ib][lane] = ok ? fb : bal_b;
            const int32_t va = same ? fb : na;     // a's value after the step
            if constexpr (FOLD) {
                const uint32_t da = (uint32_t)(bal_a ^ va), db = same ? 0u : (uint32_t)(bal_b ^ fb);
                const uint32_t df =
                    __builtin_amdgcn_alignbit(da, da, ia << 2) ^ __builtin_amdgcn_alignbit(db, db, ib << 2);
                fold ^= ok ? df : 0u;
            }
            ex = lshl_or((ok & !chk) ? 1u : 0u, ia, ex);
            ex = lshl_or((ok & tr) ? 1u : 0u, ib, ex);
            // ok => the invariant held before the step and absent accounts
            // hold 0: the child breaks it iff a or b went negative (the sign
            // of va | fb)
            neg = ok ? (va | fb) : neg;
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
            ok = has & !over & (tt ? (rc == QSMD_TICKET_NUMBER) & (just != 0u) & (rv == tn + 1) : rc == QSMD_TICKET_OK);
            stw = j;
            RS |= ((ok & !tt) ? 1u : 0u) << depth;   // transition: Reset => Just 0
        }
        // counted unless over the budget (a BUDGET return leaves the state as
        // it was); Map.! ends the search (the state after it is not used)
        const bool cnt = has & !over;
        nodes += cnt ? 1u : 0u;
        found |= cnt ? 1u : 0u;
        // descend on success (ok implies !over)
        stk.push_if(ok, stw);
        depth += ok ? 1u : 0u;
        const M fi = rem & pmj & INV;
        const M rem2 = rem & ~((fi & ((M)0 - fi)) | ((M)1 << r));
        rem = ok ? rem2 : rem;
        cand = ok ? cands(rem2, INV, RESP) : cand;
        found = ok ? 0u : found;
        return over ? QSMD_STATUS_BUDGET : (err ? QSMD_STATUS_MODEL_ERROR : -1);
    }

    // The candidates not tried yet at the levels above the current node (the
    // stack's ancestors: each level's remaining set replayed upward as undo
    // restores it) -- a predictor of the search's remaining work
    // (tools/heavy_predictor.py: correlation 0.84 with a heavy search's
    // remaining iterations on config 3)
    __device__ __forceinline__ uint32_t untried_above() const {
        StackN<G::LEVELS / 4> s = stk;
        M r = rem;
        uint32_t u = 0;
        for (uint32_t d = depth; d > base; --d) {
            const uint32_t j = s.top() & JM;
            s.pop();
            const M gone = ~r & same_pid(j);
            r |= m_topbit(gone & INV) | m_topbit(gone & RESP);
            const M c = cands(r, INV, RESP) & mask_above(j, (M)0);
            if constexpr (sizeof(M) == 4) u += (uint32_t)__builtin_popcount(c);
            else u += (uint32_t)__builtin_popcountll(c);
        }
        return u;
    }

    __device__ __forceinline__ void write_witness(uint8_t* w, uint32_t n_ev) const {
        for (uint32_t d = 0; d < depth; ++d) w[d] = (uint8_t)(stk.get(d, depth) & JM);
        if (depth < n_ev) w[depth] = QSMD_WITNESS_END;
    }

    // The search state at a stage budget (a BUDGET return: nothing moved but
    // the untried candidate last_j, dropped from cand), for the heavy stage
    // to go on from instead of the root (G32 only: kResumeWords words --
    // rem, cand, depth, found, ex, neg, RS, nodes, the stack, the balances)
    __device__ __forceinline__ void save(uint32_t* r, int32_t (*s_bal)[C_LANES], int lane) const {
        static_assert(sizeof(M) == 4 && G::LEVELS / 4 == 4, "G32");
        uint4* q = reinterpret_cast<uint4*>(r);
        q[0] = make_uint4(rem, cand | (last_j < 32u ? 1u << last_j : 0u), depth, found);
        q[1] = make_uint4(ex, (uint32_t)neg, RS, (uint32_t)nodes);
        q[2] = make_uint4(stk.w[0], stk.w[1], stk.w[2], stk.w[3]);
        if constexpr (BANK) {
            q[3] = make_uint4((uint32_t)s_bal[0][lane], (uint32_t)s_bal[1][lane], (uint32_t)s_bal[2][lane],
                              (uint32_t)s_bal[3][lane]);
            q[4] = make_uint4((uint32_t)s_bal[4][lane], (uint32_t)s_bal[5][lane], (uint32_t)s_bal[6][lane],
                              (uint32_t)s_bal[7][lane]);
        }
    }
    // (after init() from the staged history)
    __device__ __forceinline__ void restore(const uint32_t* r, int32_t (*s_bal)[C_LANES], int lane) {
        static_assert(sizeof(M) == 4 && G::LEVELS / 4 == 4, "G32");
        const uint4* q = reinterpret_cast<const uint4*>(r);
        const uint4 a = q[0], b = q[1], c = q[2];
        rem = a.x; cand = a.y; depth = a.z; found = a.w;
        ex = b.x; neg = (int32_t)b.y; RS = b.z; nodes = b.w;
        stk.w[0] = c.x; stk.w[1] = c.y; stk.w[2] = c.z; stk.w[3] = c.w;
        if constexpr (BANK) {
            const uint4 d = q[3], e = q[4];
            s_bal[0][lane] = (int32_t)d.x; s_bal[1][lane] = (int32_t)d.y;
            s_bal[2][lane] = (int32_t)d.z; s_bal[3][lane] = (int32_t)d.w;
            s_bal[4][lane] = (int32_t)e.x; s_bal[5][lane] = (int32_t)e.y;
            s_bal[6][lane] = (int32_t)e.z; s_bal[7][lane] = (int32_t)e.w;
        }
    }
};

// Wave-aggregated append of h to list (one atomic per wavefront).
// Returns the lane's slot (meaningful where pred).
__device__ __forceinline__ uint32_t wave_append(bool pred, uint32_t h, uint32_t* list, uint32_t* count, int lane) {
    const uint64_t dm = __ballot(pred);
    uint32_t at = 0;
    if (dm) {
        const int leader = __builtin_ctzll(dm);
        uint32_t slot = 0;
        if (lane == leader) slot = atomicAdd(count, (uint32_t)__builtin_popcountll(dm));
        slot = __shfl(slot, leader, 64);
        at = slot + lane_prefix(dm);
        if (pred) list[at] = h;
    }
    return at;
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
    // the wavefront's counts into its bucket (lane k adds count k: one
    // atomic instruction per wavefront)
    __device__ __forceinline__ void flush(unsigned long long* buckets, int lane) const {
        const uint64_t t_lin = wave_sum64(lin), t_non = wave_sum64(nonlin), t_err = wave_sum64(err),
                       t_enc = wave_sum64(enc), t_bud = wave_sum64(budget), t_nodes = wave_sum64(nodes);
        const uint64_t v = lane == T_CHECKED ? t_lin + t_non + t_err
                         : lane == T_LIN     ? t_lin
                         : lane == T_NONLIN  ? t_non
                         : lane == T_ERR     ? t_err
                         : lane == T_ENC     ? t_enc
                         : lane == T_BUDGET  ? t_bud
                         : lane == T_NODES   ? t_nodes
                                             : 0ull;
        bucket_add(buckets, blockIdx.x, (uint32_t)lane, v);
    }
};

// The same totals for a wavefront whose lanes all reach the count together
// (the compact stages): the status counts as ballots into wave-uniform
// scalars, only the node count summed over the lanes at the flush (one
// reduction instead of six).
struct WaveCounters {
    uint32_t lin = 0, nonlin = 0, err = 0, enc = 0, budget = 0;
    uint64_t nodes = 0;
    // out: this lane's history is final here (SKIPPED: counted by early_exit_fixup)
    __device__ __forceinline__ void add(bool out, int status, uint64_t n) {
        lin += (uint32_t)__builtin_popcountll(__ballot(out && status == QSMD_STATUS_LINEARISABLE));
        nonlin += (uint32_t)__builtin_popcountll(__ballot(out && status == QSMD_STATUS_NONLINEARISABLE));
        err += (uint32_t)__builtin_popcountll(__ballot(out && status == QSMD_STATUS_MODEL_ERROR));
        enc += (uint32_t)__builtin_popcountll(__ballot(out && status == QSMD_STATUS_ENCODE_ERROR));
        budget += (uint32_t)__builtin_popcountll(__ballot(out && status == QSMD_STATUS_BUDGET));
        nodes += (out && status != QSMD_STATUS_SKIPPED) ? n : 0ull;
    }
    __device__ __forceinline__ void flush(unsigned long long* buckets, int lane) const {
        const uint64_t t_nodes = wave_sum64(nodes);
        const uint64_t v = lane == T_CHECKED ? (uint64_t)lin + nonlin + err
                         : lane == T_LIN     ? lin
                         : lane == T_NONLIN  ? nonlin
                         : lane == T_ERR     ? err
                         : lane == T_ENC     ? enc
                         : lane == T_BUDGET  ? budget
                         : lane == T_NODES   ? t_nodes
                                             : 0ull;
        bucket_add(buckets, blockIdx.x, (uint32_t)lane, v);
    }
};

}  // namespace

}  // namespace qsmd
