// gen.hip -- on-device synthetic history generation.
//
// The device restatement of the seeded generator (csrc/gen/gen.cpp,
// include/qsmd_gen.h): one history per lane, the same per-history RNG stream
// (xoshiro256** seeded by splitmix64 from (seed, global index)), the same
// scheduler-policy delivery (src/Scheduler.hs:105-186), sequential prefix,
// request distributions (test/Bank.hs:133-146, test/TicketDispenser.hs:108-112)
// and bug injection, so a batch generated here is byte-identical to the host
// generator's (tests/test_gpu_gen.py).  Removes host generation and the
// host-to-device copy from 10M-history runs.  Every history has exactly
// 2 * n_ops events at ev_base + i * 2 * n_ops.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "qsmd_gen.h"

namespace qsmd {

namespace {

struct DRng {
    uint64_t s[4];
    __device__ static uint64_t splitmix(uint64_t& x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    __device__ DRng(uint64_t seed, uint64_t index) {
        uint64_t x = seed ^ (index * 0xD1B54A32D192ED03ull);
        for (int q = 0; q < 4; ++q) s[q] = splitmix(x);
    }
    __device__ static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    __device__ uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    __device__ uint32_t below(uint32_t n) { return n ? (uint32_t)((next() >> 32) * n >> 32) : 0u; }
    __device__ double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct DOp {
    uint8_t pid, code, a, b;
    int32_t val;
    uint8_t rcode;
    int32_t rval;
};

struct DSpec {
    uint32_t exists;
    int64_t bal[QSMD_BANK_MAX_ACCOUNTS];
    bool just;
    int64_t n;
};

// the spec executed at the linearisation point (test/Bank.hs:92-131,
// test/TicketDispenser.hs:81-102: the response `post` accepts)
__device__ void d_execute(uint32_t model, DSpec& s, DOp& op) {
    if (model == QSMD_MODEL_TICKET) {
        if (op.code == QSMD_TICKET_RESET) {
            s.just = true;
            s.n = 0;
            op.rcode = QSMD_TICKET_OK;
            op.rval = 0;
        } else {
            if (s.just) s.n += 1;
            op.rcode = QSMD_TICKET_NUMBER;
            op.rval = (int32_t)s.n;
        }
        return;
    }
    const int a = op.a;
    const bool ex = (s.exists >> a) & 1u;
    op.rval = 0;
    if (op.code == QSMD_BANK_OPEN_ACCOUNT) {
        if (ex) {
            op.rcode = QSMD_BANK_ACCOUNT_ALREADY_EXISTS;
        } else {
            s.exists |= 1u << a;
            s.bal[a] = 0;
            op.rcode = QSMD_BANK_ACCOUNT_CREATED;
        }
    } else if (op.code == QSMD_BANK_DEPOSIT) {
        s.bal[a] = ex ? s.bal[a] + op.val : op.val;
        s.exists |= 1u << a;
        op.rcode = QSMD_BANK_DEPOSIT_MADE;
    } else if (op.code == QSMD_BANK_WITHDRAW || op.code == QSMD_BANK_TRANSFER) {
        const bool ok = ex && s.bal[a] >= op.val;
        s.bal[a] = ex ? s.bal[a] - op.val : op.val;
        s.exists |= 1u << a;
        if (op.code == QSMD_BANK_TRANSFER) {
            const int b = op.b;
            const bool exb = (s.exists >> b) & 1u;
            s.bal[b] = exb ? s.bal[b] + op.val : op.val;
            s.exists |= 1u << b;
            op.rcode = ok ? QSMD_BANK_TRANSFER_MADE : QSMD_BANK_INSUFFICIENT_FUNDS;
        } else {
            op.rcode = ok ? QSMD_BANK_WITHDRAWAL_MADE : QSMD_BANK_INSUFFICIENT_FUNDS;
        }
    } else {                                     // CheckBalance
        if (ex) {
            op.rcode = QSMD_BANK_BALANCE;
            op.rval = (int32_t)s.bal[a];
        } else {
            op.rcode = QSMD_BANK_ACCOUNT_DOESNT_EXIST;
        }
    }
}

// a request for account a under the preconditions (test/Bank.hs:106-116,
// the suchThat retry of src/QuickCheckHelpers.hs:39,72), weights :136-146
__device__ void d_bank_request(DRng& r, const qsmd_gen_params& p, const DSpec& s, uint8_t a, DOp& op) {
    const uint32_t C = p.n_clients, mmax = p.money_max ? p.money_max : 100u;
    op.a = a;
    op.b = a;
    op.val = 0;
    const bool ex = (s.exists >> a) & 1u;
    if (!ex) {
        op.code = QSMD_BANK_OPEN_ACCOUNT;
        return;
    }
    const int64_t bal = s.bal[a];
    for (;;) {
        const uint32_t w = r.below(24);          // Open 1, Deposit 5, Withdraw 5, Transfer 8, Check 5
        if (w < 1) continue;
        if (w < 6) {
            op.code = QSMD_BANK_DEPOSIT;
            op.val = 1 + (int32_t)r.below(mmax);
            return;
        }
        if (w < 11) {
            if (bal < 1) continue;
            op.code = QSMD_BANK_WITHDRAW;
            op.val = 1 + (int32_t)r.below((uint32_t)(bal < (int64_t)mmax ? bal : (int64_t)mmax));
            return;
        }
        if (w < 19) {
            if (bal < 1 || C < 2) continue;
            op.code = QSMD_BANK_TRANSFER;
            op.val = 1 + (int32_t)r.below((uint32_t)(bal < (int64_t)mmax ? bal : (int64_t)mmax));
            const uint32_t b = r.below(C - 1);
            op.b = (uint8_t)(b >= a ? b + 1 : b);
            return;
        }
        op.code = QSMD_BANK_CHECK_BALANCE;
        return;
    }
}

__device__ uint8_t d_ticket_request(DRng& r, const DSpec& s) {
    if (!s.just) return QSMD_TICKET_RESET;
    return r.below(9) == 0 ? QSMD_TICKET_RESET : QSMD_TICKET_TAKE_TICKET;
}

__device__ void d_put(qsmd_event* ev, int e, uint8_t kp, uint8_t code, uint8_t a, uint8_t b, int32_t val) {
    qsmd_event x;
    x.kp = kp;
    x.code = code;
    x.a = a;
    x.b = b;
    x.val = val;
    ev[e] = x;
}

}  // namespace

__global__ __launch_bounds__(64) void gen_kernel(qsmd_gen_params p, uint64_t first, uint64_t n_hist,
                                                uint32_t ev_base, qsmd_hdr* hdr, qsmd_event* events,
                                                uint8_t* bug_out) {
    const uint64_t i = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (i >= n_hist) return;
    const uint32_t per = 2u * p.n_ops;
    qsmd_hdr H;
    H.ev_off = ev_base + (uint32_t)(i * per);
    H.n_ev = (uint16_t)per;
    H.n_pid = (uint8_t)(p.pid_mode == QSMD_GEN_PID_SHARED ? 1u : p.n_clients);
    H.model_id = (uint8_t)p.model_id;
    H.tag = (uint32_t)(first + i);
    H.reserved = 0u;
    hdr[i] = H;
    qsmd_event* ev = events + i * per;

    DRng r(p.seed, first + i);
    const uint32_t C = p.n_clients, K = p.n_ops;
    const bool ticket = p.model_id == QSMD_MODEL_TICKET;
    const bool shared = p.pid_mode == QSMD_GEN_PID_SHARED;
    const uint32_t overlap = p.overlap ? p.overlap : C;
    DSpec s;
    s.exists = 0u;
    for (int q = 0; q < QSMD_BANK_MAX_ACCOUNTS; ++q) s.bal[q] = 0;
    s.just = false;
    s.n = 0;
    int ne = 0;
    auto emit_inv = [&](const DOp& o) { d_put(ev, ne++, (uint8_t)(shared ? 0 : o.pid), o.code, o.a, o.b, o.val); };
    auto emit_resp = [&](const DOp& o) {
        d_put(ev, ne++, (uint8_t)(QSMD_EV_RESP | (shared ? 0 : o.pid)), o.rcode, 0, 0, o.rval);
    };

    // ---- sequential prefix (SchedulerSequential)
    uint32_t prefix = p.prefix_ops;
    if (!ticket && prefix < C) prefix = C;
    if (prefix > K) prefix = K;
    for (uint32_t k = 0; k < prefix; ++k) {
        DOp o{};
        if (ticket) {
            o.pid = 0;
            o.code = d_ticket_request(r, s);
        } else {
            const uint8_t a = (uint8_t)(k < C ? k : r.below(C));
            o.pid = a;
            d_bank_request(r, p, s, a, o);
        }
        d_execute(p.model_id, s, o);
        emit_inv(o);
        emit_resp(o);
    }

    // ---- concurrent suffix (one uniformly chosen ready event per tick)
    const uint32_t S = K - prefix;
    uint8_t owner[QSMD_MAX_EVENTS / 2];
    for (uint32_t k = 0; k < S; ++k) owner[k] = (uint8_t)(ticket ? k % C : r.below(C));
    uint32_t queued[QSMD_BANK_MAX_ACCOUNTS] = {};
    for (uint32_t k = 0; k < S; ++k) queued[owner[k]]++;
    DOp cur[QSMD_BANK_MAX_ACCOUNTS];
    uint8_t st[QSMD_BANK_MAX_ACCOUNTS] = {};      // 0 idle, 1 invoked, 2 executed
    uint32_t outstanding = 0, done = 0;
    uint32_t act[3 * QSMD_BANK_MAX_ACCOUNTS];
    while (done < S) {
        uint32_t n_act = 0;
        for (uint32_t c = 0; c < C; ++c) {
            if (st[c] == 0 && queued[c] && outstanding < overlap) act[n_act++] = c * 3 + 0;
            if (st[c] == 1) act[n_act++] = c * 3 + 1;
            if (st[c] == 2) act[n_act++] = c * 3 + 2;
        }
        const uint32_t pick = act[r.below(n_act)];
        const uint32_t c = pick / 3, what = pick % 3;
        DOp& o = cur[c];
        if (what == 0) {
            o = DOp{};
            o.pid = (uint8_t)c;
            if (ticket) o.code = d_ticket_request(r, s);
            else d_bank_request(r, p, s, (uint8_t)c, o);
            emit_inv(o);
            queued[c]--;
            outstanding++;
            if (p.lin_policy == QSMD_GEN_LIN_AT_INVOKE) {
                d_execute(p.model_id, s, o);
                st[c] = 2;
            } else {
                st[c] = 1;
            }
        } else if (what == 1) {
            d_execute(p.model_id, s, o);
            st[c] = 2;
        } else {
            emit_resp(o);
            st[c] = 0;
            outstanding--;
            done++;
        }
    }

    // ---- bug injection (a corrupted Balance/Number value or two swapped responses)
    uint8_t has_bug = 0;
    if (p.p_bug > 0 && r.unit() < p.p_bug && ne > 0) {
        const int first_e = (int)(2 * prefix);
        uint8_t vals[QSMD_MAX_EVENTS / 2], resps[QSMD_MAX_EVENTS / 2];
        uint32_t n_vals = 0, n_resps = 0;
        for (int e = first_e; e < ne; ++e) {
            const qsmd_event x = ev[e];
            if (!(x.kp & QSMD_EV_RESP)) continue;
            resps[n_resps++] = (uint8_t)e;
            const bool valued = ticket ? x.code == QSMD_TICKET_NUMBER : x.code == QSMD_BANK_BALANCE;
            if (valued) vals[n_vals++] = (uint8_t)e;
        }
        if (n_vals && (n_resps < 2 || r.below(2) == 0)) {
            const int e = vals[r.below(n_vals)];
            const int32_t d = 1 + (int32_t)r.below(3);
            qsmd_event x = ev[e];
            x.val += r.below(2) ? d : -d;
            ev[e] = x;
            has_bug = 1;
        } else if (n_resps >= 2) {
            const uint32_t k1 = r.below(n_resps);
            uint32_t k2 = r.below(n_resps);
            if (k2 == k1) k2 = (k1 + 1) % n_resps;
            const int e1 = resps[k1], e2 = resps[k2];
            qsmd_event x1 = ev[e1], x2 = ev[e2];
            const uint8_t c1 = x1.code;
            const int32_t v1 = x1.val;
            x1.code = x2.code;
            x1.val = x2.val;
            x2.code = c1;
            x2.val = v1;
            ev[e1] = x1;
            ev[e2] = x2;
            has_bug = 1;
        }
    }
    if (bug_out) bug_out[i] = has_bug;
}

hipError_t launch_gen(const qsmd_gen_params& p, uint64_t first, uint64_t n_hist, uint32_t ev_base, qsmd_hdr* hdr,
                      qsmd_event* events, uint8_t* bug_out, hipStream_t s) {
    const uint64_t grid = (n_hist + 63) / 64;
    hipLaunchKernelGGL(gen_kernel, dim3((uint32_t)grid), dim3(64), 0, s, p, first, n_hist, ev_base, hdr, events,
                       bug_out);
    return hipGetLastError();
}

}  // namespace qsmd
