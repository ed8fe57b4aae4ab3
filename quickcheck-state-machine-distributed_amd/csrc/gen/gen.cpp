// gen.cpp -- seeded synthetic history generator (include/qsmd_gen.h).
//
// Restates the reference's history producer: the deterministic scheduler of
// src/Scheduler.hs:105-186 (one mailbox per (client, server) pair, each pair
// alternates request / response, one uniformly chosen ready event per tick),
// the sequential prefix of test/Bank.hs:264-269 and
// test/TicketDispenser.hs:292-305, and the generators test/Bank.hs:133-146 /
// test/TicketDispenser.hs:108-112.  The "implementation" answering requests is
// the model itself executed at each operation's linearisation point, so every
// history without an injected bug is linearisable.
#include "qsmd_gen.h"

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct Rng {  // xoshiro256** seeded by splitmix64
    uint64_t s[4];
    static uint64_t splitmix(uint64_t& x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    Rng(uint64_t seed, uint64_t index) {
        uint64_t x = seed ^ (index * 0xD1B54A32D192ED03ull);
        for (auto& v : s) v = splitmix(x);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
        s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    uint32_t below(uint32_t n) { return n ? (uint32_t)((next() >> 32) * n >> 32) : 0; }
    double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct Op {
    uint8_t pid, code, a, b;
    int32_t val;
    uint8_t rcode;
    int32_t rval;
};

// Sequential specification state (the model, executed).
struct Spec {
    uint32_t exists = 0;
    int64_t bal[QSMD_BANK_MAX_ACCOUNTS] = {};
    bool just = false;
    int64_t n = 0;
};

// Execute one request against the spec; fills the response (test/Bank.hs:92-131,
// test/TicketDispenser.hs:81-102: the response is the one `post` accepts).
void execute(uint32_t model, Spec& s, Op& op) {
    if (model == QSMD_MODEL_TICKET) {
        if (op.code == QSMD_TICKET_RESET) {
            s.just = true; s.n = 0;
            op.rcode = QSMD_TICKET_OK; op.rval = 0;
        } else {
            if (s.just) s.n += 1;
            op.rcode = QSMD_TICKET_NUMBER; op.rval = (int32_t)s.n;
        }
        return;
    }
    const int a = op.a;
    const bool ex = (s.exists >> a) & 1u;
    op.rval = 0;
    switch (op.code) {
    case QSMD_BANK_OPEN_ACCOUNT:
        if (ex) { op.rcode = QSMD_BANK_ACCOUNT_ALREADY_EXISTS; }
        else { s.exists |= 1u << a; s.bal[a] = 0; op.rcode = QSMD_BANK_ACCOUNT_CREATED; }
        break;
    case QSMD_BANK_DEPOSIT:
        s.bal[a] = ex ? s.bal[a] + op.val : op.val; s.exists |= 1u << a;
        op.rcode = QSMD_BANK_DEPOSIT_MADE;
        break;
    case QSMD_BANK_WITHDRAW:
    case QSMD_BANK_TRANSFER: {
        const bool ok = ex && s.bal[a] >= op.val;
        s.bal[a] = ex ? s.bal[a] - op.val : op.val; s.exists |= 1u << a;
        if (op.code == QSMD_BANK_TRANSFER) {
            const int b = op.b;
            const bool exb = (s.exists >> b) & 1u;
            s.bal[b] = exb ? s.bal[b] + op.val : op.val; s.exists |= 1u << b;
            op.rcode = ok ? QSMD_BANK_TRANSFER_MADE : QSMD_BANK_INSUFFICIENT_FUNDS;
        } else {
            op.rcode = ok ? QSMD_BANK_WITHDRAWAL_MADE : QSMD_BANK_INSUFFICIENT_FUNDS;
        }
        break;
    }
    case QSMD_BANK_CHECK_BALANCE:
        if (ex) { op.rcode = QSMD_BANK_BALANCE; op.rval = (int32_t)s.bal[a]; }
        else { op.rcode = QSMD_BANK_ACCOUNT_DOESNT_EXIST; }
        break;
    }
}

// Bank request for account a, drawn when the request is sent, respecting the
// preconditions of test/Bank.hs:106-116 on the current state (the suchThat
// retry of src/QuickCheckHelpers.hs:39,72).  Weights test/Bank.hs:136-146.
void bank_request(Rng& r, const qsmd_gen_params& p, const Spec& s, uint8_t a, Op& op) {
    const uint32_t C = p.n_clients, mmax = p.money_max ? p.money_max : 100;
    op.a = a; op.b = a; op.val = 0;
    const bool ex = (s.exists >> a) & 1u;
    if (!ex) { op.code = QSMD_BANK_OPEN_ACCOUNT; return; }
    const int64_t bal = s.bal[a];
    for (;;) {
        uint32_t w = r.below(24);   // Open 1, Deposit 5, Withdraw 5, Transfer 8, Check 5
        if (w < 1) continue;        // Open: precondition notMember fails (all open)
        if (w < 6) { op.code = QSMD_BANK_DEPOSIT; op.val = 1 + (int32_t)r.below(mmax); return; }
        if (w < 11) {
            if (bal < 1) continue;
            op.code = QSMD_BANK_WITHDRAW;
            op.val = 1 + (int32_t)r.below((uint32_t)(bal < mmax ? bal : mmax));
            return;
        }
        if (w < 19) {
            if (bal < 1 || C < 2) continue;
            op.code = QSMD_BANK_TRANSFER;
            op.val = 1 + (int32_t)r.below((uint32_t)(bal < mmax ? bal : mmax));
            uint32_t b = r.below(C - 1);
            op.b = (uint8_t)(b >= a ? b + 1 : b);
            return;
        }
        op.code = QSMD_BANK_CHECK_BALANCE; return;
    }
}

uint8_t ticket_request(Rng& r, const Spec& s) {   // test/TicketDispenser.hs:108-112
    if (!s.just) return QSMD_TICKET_RESET;
    return r.below(9) == 0 ? QSMD_TICKET_RESET : QSMD_TICKET_TAKE_TICKET;
}

void gen_one(const qsmd_gen_params& p, uint64_t index, qsmd_event* ev, uint8_t* bug) {
    Rng r(p.seed, index);
    const uint32_t C = p.n_clients, K = p.n_ops;
    const bool ticket = p.model_id == QSMD_MODEL_TICKET;
    const bool shared = p.pid_mode == QSMD_GEN_PID_SHARED;
    const uint32_t overlap = p.overlap ? p.overlap : C;
    Spec s;
    int ne = 0;
    auto emit_inv = [&](const Op& o) {
        ev[ne++] = qsmd_event{(uint8_t)(shared ? 0 : o.pid), o.code, o.a, o.b, o.val};
    };
    auto emit_resp = [&](const Op& o) {
        ev[ne++] = qsmd_event{(uint8_t)(QSMD_EV_RESP | (shared ? 0 : o.pid)), o.rcode, 0, 0, o.rval};
    };

    // ---- sequential prefix (SchedulerSequential)
    uint32_t prefix = p.prefix_ops;
    if (!ticket && prefix < C) prefix = C;
    if (prefix > K) prefix = K;
    for (uint32_t i = 0; i < prefix; ++i) {
        Op o{};
        if (ticket) {
            o.pid = 0; o.code = ticket_request(r, s);
        } else {
            uint8_t a = (uint8_t)(i < C ? i : r.below(C));
            o.pid = a;
            bank_request(r, p, s, a, o);
        }
        execute(p.model_id, s, o);
        emit_inv(o); emit_resp(o);
    }

    // ---- concurrent suffix
    const uint32_t S = K - prefix;
    // Which client issues each suffix request (Ticket: alternate like
    // `zip (cycle [True, False]) suffix`, test/TicketDispenser.hs:300-305;
    // Bank: the request's account, uniform).
    std::vector<uint8_t> owner(S);
    for (uint32_t i = 0; i < S; ++i) owner[i] = (uint8_t)(ticket ? i % C : r.below(C));
    std::vector<uint32_t> queued(C, 0);
    for (uint32_t i = 0; i < S; ++i) queued[owner[i]]++;
    std::vector<Op> cur(C);
    std::vector<uint8_t> st(C, 0);   // 0 idle, 1 invoked, 2 executed
    uint32_t outstanding = 0, done = 0;
    std::vector<uint32_t> act;
    act.reserve(3 * C);
    while (done < S) {
        act.clear();
        for (uint32_t c = 0; c < C; ++c) {
            if (st[c] == 0 && queued[c] && outstanding < overlap) act.push_back(c * 3 + 0);
            if (st[c] == 1) act.push_back(c * 3 + 1);
            if (st[c] == 2) act.push_back(c * 3 + 2);
        }
        const uint32_t pick = act[r.below((uint32_t)act.size())];
        const uint32_t c = pick / 3, what = pick % 3;
        Op& o = cur[c];
        if (what == 0) {
            o = Op{};
            o.pid = (uint8_t)c;
            if (ticket) o.code = ticket_request(r, s);
            else bank_request(r, p, s, (uint8_t)c, o);
            emit_inv(o);
            queued[c]--; outstanding++;
            if (p.lin_policy == QSMD_GEN_LIN_AT_INVOKE) { execute(p.model_id, s, o); st[c] = 2; }
            else st[c] = 1;
        } else if (what == 1) {
            execute(p.model_id, s, o);
            st[c] = 2;
        } else {
            emit_resp(o);
            st[c] = 0; outstanding--; done++;
        }
    }

    // ---- bug injection (a corrupted Balance/Number value or two swapped
    //      responses)
    uint8_t has_bug = 0;
    if (p.p_bug > 0 && r.unit() < p.p_bug && ne > 0) {
        const int first = (int)(2 * prefix);
        std::vector<int> vals, resps;
        for (int e = first; e < ne; ++e) {
            if (!(ev[e].kp & QSMD_EV_RESP)) continue;
            resps.push_back(e);
            const bool valued = ticket ? ev[e].code == QSMD_TICKET_NUMBER
                                       : ev[e].code == QSMD_BANK_BALANCE;
            if (valued) vals.push_back(e);
        }
        if (!vals.empty() && (resps.size() < 2 || r.below(2) == 0)) {
            const int e = vals[r.below((uint32_t)vals.size())];
            const int32_t d = 1 + (int32_t)r.below(3);
            ev[e].val += r.below(2) ? d : -d;
            has_bug = 1;
        } else if (resps.size() >= 2) {
            const int e1 = resps[r.below((uint32_t)resps.size())];
            int e2 = resps[r.below((uint32_t)resps.size())];
            if (e2 == e1) e2 = resps[(std::find(resps.begin(), resps.end(), e1) - resps.begin() + 1) % resps.size()];
            std::swap(ev[e1].code, ev[e2].code);
            std::swap(ev[e1].val, ev[e2].val);
            has_bug = 1;
        }
    }
    if (bug) *bug = has_bug;
}

}  // namespace

extern "C" int qsmd_gen_batch(const qsmd_gen_params* p, uint64_t first, uint64_t n_hist,
                              uint32_t ev_base, qsmd_hdr* hdr, qsmd_event* events,
                              uint8_t* bug_out, int n_threads) {
    if (!p || !hdr || !events) return QSMD_ERR_ARG;
    if (p->model_id != QSMD_MODEL_BANK && p->model_id != QSMD_MODEL_TICKET) return QSMD_ERR_ARG;
    if (p->n_clients < 1 || p->n_clients > QSMD_BANK_MAX_ACCOUNTS) return QSMD_ERR_ARG;
    if (p->n_ops < 1 || 2 * p->n_ops > QSMD_MAX_EVENTS) return QSMD_ERR_ARG;
    if (p->model_id == QSMD_MODEL_BANK && p->n_ops < p->n_clients) return QSMD_ERR_ARG;
    const uint32_t per = 2 * p->n_ops;
    if (n_threads < 1) n_threads = 1;
    auto work = [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i) {
            qsmd_hdr& h = hdr[i];
            std::memset(&h, 0, sizeof(h));
            h.ev_off = ev_base + (uint32_t)(i * per);
            h.n_ev = (uint16_t)per;
            h.n_pid = (uint8_t)(p->pid_mode == QSMD_GEN_PID_SHARED ? 1 : p->n_clients);
            h.model_id = (uint8_t)p->model_id;
            h.tag = (uint32_t)(first + i);
            gen_one(*p, first + i, events + i * per, bug_out ? bug_out + i : nullptr);
        }
    };
    if (n_threads == 1 || n_hist < 1024) { work(0, n_hist); return 0; }
    std::vector<std::thread> th;
    const uint64_t chunk = (n_hist + n_threads - 1) / n_threads;
    for (int t = 0; t < n_threads; ++t) {
        const uint64_t lo = t * chunk, hi = std::min<uint64_t>(n_hist, lo + chunk);
        if (lo >= hi) break;
        th.emplace_back(work, lo, hi);
    }
    for (auto& x : th) x.join();
    return 0;
}
