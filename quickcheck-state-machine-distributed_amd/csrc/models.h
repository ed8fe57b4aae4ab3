// models.h -- device functors for the model closures the reference passes to
// `linearisable` (src/Linearisability.hs:54-55).
//
//   Bank            next' / invariant / post     test/Bank.hs:92-131
//   TicketDispenser transition / postcondition   test/TicketDispenser.hs:81-102
//
// The search keeps the model in registers (small parts) and LDS (Bank
// balances, one i64 per account per lane, laid out [account][lane] so that
// any per-lane account index is bank-conflict free).  Every transition is
// undone exactly on backtrack from a compact per-level undo record, so the
// DFS never copies a model.  All arithmetic is integer and exact.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qsmd.h"

namespace qsmd {

// Post-condition outcome.
enum : int { POST_FALSE = 0, POST_TRUE = 1, POST_ERROR = 2 };

// Decoded event (include/qsmd.h qsmd_event packed as uint2).
struct Ev {
    uint32_t lo;   // kp | code << 8 | a << 16 | b << 24
    int32_t val;
    __device__ __forceinline__ uint32_t pid() const { return lo & 0x7Fu; }
    __device__ __forceinline__ bool is_resp() const { return (lo & 0x80u) != 0; }
    __device__ __forceinline__ uint32_t code() const { return (lo >> 8) & 0xFFu; }
    __device__ __forceinline__ uint32_t a() const { return (lo >> 16) & 0xFFu; }
    __device__ __forceinline__ uint32_t b() const { return lo >> 24; }
};

// Validation of one event for a model (include/qsmd.h encoding rules).
template <uint32_t MODEL>
__device__ __forceinline__ bool valid_event(const Ev& e) {
    const uint32_t c = e.code();
    if constexpr (MODEL == QSMD_MODEL_TICKET) {
        return c <= 1u;
    } else {
        if (e.is_resp()) return c <= QSMD_BANK_BALANCE;
        return c <= QSMD_BANK_TRANSFER && e.a() < QSMD_BANK_MAX_ACCOUNTS &&
               (c != QSMD_BANK_TRANSFER || e.b() < QSMD_BANK_MAX_ACCOUNTS);
    }
}

// ---------------------------------------------------------------- Ticket
// Model `Maybe Int`: just (bool) + n (i64).  Undo of Reset needs the old
// model: the undo record is {old just, old n}.
struct TicketState {
    uint32_t just;
    int64_t n;
};

__device__ __forceinline__ int ticket_post(const TicketState& m, const Ev& inv, const Ev& resp) {
    // postcondition m TakeTicket (Number i) = Just i == (succ <$> m)
    // postcondition _ Reset Ok = True ; _ = False     (TicketDispenser.hs:99-102)
    const uint32_t ic = inv.code(), rc = resp.code();
    const bool tt = ic == QSMD_TICKET_TAKE_TICKET && rc == QSMD_TICKET_NUMBER &&
                    m.just && (int64_t)resp.val == m.n + 1;
    const bool rs = ic == QSMD_TICKET_RESET && rc == QSMD_TICKET_OK;
    return (tt || rs) ? POST_TRUE : POST_FALSE;
}

__device__ __forceinline__ void ticket_apply(TicketState& m, const Ev& inv) {
    // transition m (Left TakeTicket) = succ <$> m ; (Left Reset) = Just 0
    if (inv.code() == QSMD_TICKET_TAKE_TICKET) {
        m.n += m.just ? 1 : 0;
    } else {
        m.just = 1u;
        m.n = 0;
    }
}

// ---------------------------------------------------------------- Bank
// Model `Map acc Money`: `exists` bitmask (<= 8 accounts) in a register,
// balances in LDS (0 when absent), and `neg` = bitmask of existing accounts
// with a negative balance, so `invariant` (Bank.hs:103-104) is `neg == 0`.
struct BankState {
    uint32_t exists;
    uint32_t neg;
};

// Expected response constructor of `post` for a request, given the
// pre-state (test/Bank.hs:118-131).  CheckBalance is handled separately.
__device__ __forceinline__ uint32_t bank_expected(uint32_t code, bool ex_a, int64_t bal_a, int64_t m) {
    const bool ge = ex_a && bal_a >= m;               // M.lookup acc model >= Just money
    uint32_t exp = QSMD_BANK_INSUFFICIENT_FUNDS;
    if (code == QSMD_BANK_OPEN_ACCOUNT)
        exp = ex_a ? QSMD_BANK_ACCOUNT_ALREADY_EXISTS : QSMD_BANK_ACCOUNT_CREATED;
    else if (code == QSMD_BANK_DEPOSIT)
        exp = QSMD_BANK_DEPOSIT_MADE;
    else if (code == QSMD_BANK_WITHDRAW)
        exp = ge ? QSMD_BANK_WITHDRAWAL_MADE : QSMD_BANK_INSUFFICIENT_FUNDS;
    else if (code == QSMD_BANK_TRANSFER)
        exp = ge ? QSMD_BANK_TRANSFER_MADE : QSMD_BANK_INSUFFICIENT_FUNDS;
    else
        exp = QSMD_BANK_BALANCE;
    return exp;
}

// post model req resp.  bal_a = balance of req's account (0 if absent).
__device__ __forceinline__ int bank_post(const BankState& m, const Ev& inv, const Ev& resp, int64_t bal_a) {
    if (m.neg != 0u) return POST_FALSE;               // invariant model && ...
    const uint32_t code = inv.code(), rc = resp.code();
    const bool ex_a = (m.exists >> inv.a()) & 1u;
    const uint32_t exp = bank_expected(code, ex_a, bal_a, (int64_t)inv.val);
    if (rc != exp) return POST_FALSE;
    if (code == QSMD_BANK_CHECK_BALANCE) {
        // resp == Balance (model M.! acc): Map.! raises on a missing key
        if (!ex_a) return POST_ERROR;
        return (int64_t)resp.val == bal_a ? POST_TRUE : POST_FALSE;
    }
    return POST_TRUE;
}

}  // namespace qsmd
