// compact.hip -- stage 0 of the search cascade: the hot kernel for small
// histories (<= 32 events, <= 8 pids, every value within 19-bit signed), i.e.
// every history of the reference's own properties (2 clients, suffix <= 6,
// src/QuickCheckHelpers.hs:74) and of the 4x16 Bank benchmark.
//
// Same search as csrc/search.hip (src/Linearisability.hs:25-69 over the
// Lemma L1 event bitset), re-laid out for latency: the only per-node LDS
// traffic is ONE round trip that fetches the candidate invocation and its
// response together (both addresses are computed in registers first: the pid
// of every event is kept as 4-bit nibbles in 4 VGPRs and the per-pid event
// masks in 8 VGPRs), and the model (Bank balances as i32, Ticket Maybe Int)
// lives entirely in registers, indexed by unrolled select trees.  LDS holds
// only the history (one u32 per event, [event][lane]) and one u32 per DFS
// level ([level][lane]): 12 KiB per wavefront.  Histories outside these
// bounds are deferred to stage 1 (search.hip) with a wave-aggregated append.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "models.h"

namespace qsmd {

namespace {

constexpr int C_MAXEV = 32;
constexpr int C_MAXD = C_MAXEV / 2;
constexpr int C_LANES = 64;
constexpr int32_t V19_MIN = -(1 << 18), V19_MAX = (1 << 18) - 1;

// compressed event: pid 3 | resp 1 | code 3 | a 3 | b 3 | val 19 (signed)
__device__ __forceinline__ uint32_t c_code(uint32_t w) { return (w >> 4) & 7u; }
__device__ __forceinline__ uint32_t c_a(uint32_t w) { return (w >> 7) & 7u; }
__device__ __forceinline__ uint32_t c_b(uint32_t w) { return (w >> 10) & 7u; }
__device__ __forceinline__ int32_t c_val(uint32_t w) { return (int32_t)w >> 13; }

// v[i] for a per-lane i, as a VGPR select tree.  The empty asm makes each
// element an opaque register value: without it hipcc folds the select tree
// back into a dynamically indexed private array (scratch memory).
template <typename T>
__device__ __forceinline__ T sel8(const T (&v)[8], uint32_t i) {
    T x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        x[q] = v[q];
        asm volatile("" : "+v"(x[q]));
    }
    const T a0 = (i & 1u) ? x[1] : x[0], a1 = (i & 1u) ? x[3] : x[2];
    const T a2 = (i & 1u) ? x[5] : x[4], a3 = (i & 1u) ? x[7] : x[6];
    const T b0 = (i & 2u) ? a1 : a0, b1 = (i & 2u) ? a3 : a2;
    return (i & 4u) ? b1 : b0;
}

template <typename T>
__device__ __forceinline__ void put8(T (&v)[8], uint32_t i, T x) {
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) v[q] = (q == i) ? x : v[q];
}

__device__ __forceinline__ uint32_t below32(uint32_t r) { return r >= 32u ? ~0u : (1u << r) - 1u; }

__device__ __forceinline__ uint32_t cands(uint32_t rem, uint32_t INV, uint32_t RESP) {
    const uint32_t rr = rem & RESP;
    const uint32_t R = rr ? (uint32_t)__builtin_ctz(rr) : 32u;
    return rem & INV & below32(R);
}

__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace

template <uint32_t MODEL>
__global__ __launch_bounds__(C_LANES) void compact_search(SearchArgs a) {
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;
    __shared__ uint32_t s_ev[C_MAXEV][C_LANES];
    __shared__ uint32_t s_st[C_MAXD][C_LANES];

    const int lane = threadIdx.x;
    const uint64_t total = a.n_hist;
    uint32_t c_lin = 0, c_nonlin = 0, c_err = 0, c_enc = 0, c_budget = 0;
    uint64_t c_nodes = 0;
    const uint64_t t0 = a.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;

    for (uint64_t base = (uint64_t)blockIdx.x * C_LANES; base < total;
         base += (uint64_t)gridDim.x * C_LANES) {
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

        // ---- stage the history: 16 independent 8-byte loads in flight per
        //      chunk, then (branch-free) compress into LDS and build the
        //      register masks.  Pids are kept bit-sliced: P0/P1/P2 hold bit
        //      0/1/2 of every event's pid, so "events with the pid of event
        //      j" is a handful of VALU ops (same_pid below), no table.
        uint32_t INV = 0, RESP = 0, P0 = 0, P1 = 0, P2 = 0;
        bool ok = enc_ok, fits = small;
        if (small) {
            const uint2* evp = a.events + H.ev_off;
#pragma unroll
            for (int c = 0; c < C_MAXEV / 16; ++c) {
                uint2 x[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const uint32_t e = (uint32_t)(c * 16 + k);
                    x[k] = e < n_ev ? evp[e] : make_uint2(0u, 0u);
                }
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const uint32_t e = (uint32_t)(c * 16 + k);
                    const bool in = e < n_ev;
                    const Ev ev{x[k].x, (int32_t)x[k].y};
                    const uint32_t p = ev.pid();
                    ok = ok & (!in | ((p < n_pid) & valid_event<MODEL>(ev)));
                    fits = fits & (!in | ((ev.val >= V19_MIN) & (ev.val <= V19_MAX)));
                    const uint32_t resp = ev.is_resp() ? 1u : 0u;
                    s_ev[e][lane] = (p & 7u) | (resp << 3) | ((ev.code() & 7u) << 4) |
                                    ((ev.a() & 7u) << 7) | ((ev.b() & 7u) << 10) |
                                    ((uint32_t)ev.val << 13);
                    const uint32_t bit = in ? (1u << e) : 0u;
                    RESP |= resp ? bit : 0u;
                    INV |= resp ? 0u : bit;
                    P0 |= (p & 1u) ? bit : 0u;
                    P1 |= (p & 2u) ? bit : 0u;
                    P2 |= (p & 4u) ? bit : 0u;
                }
            }
        }
        const uint32_t ALL = INV | RESP;
        // events whose pid equals the pid of event j (bit-sliced compare)
        auto same_pid = [&](uint32_t j) -> uint32_t {
            const uint32_t m0 = 0u - ((P0 >> j) & 1u), m1 = 0u - ((P1 >> j) & 1u),
                           m2 = 0u - ((P2 >> j) & 1u);
            return ~((P0 ^ m0) | (P1 ^ m1) | (P2 ^ m2)) & ALL;
        };
        const bool defer = enc_ok && (!small || (ok && !fits));

        // ---- overflow to stage 1 (wave-aggregated append)
        const uint64_t dm = __ballot(defer);
        if (dm) {
            const int leader = __builtin_ctzll(dm);
            uint32_t slot = 0;
            if (lane == leader) slot = atomicAdd(a.defer_count, (uint32_t)__builtin_popcountll(dm));
            slot = __shfl(slot, leader, 64);
            if (defer) a.defer_list[slot + lane_prefix(dm)] = h;
        }
        if (!active || defer) continue;

        int status = -1;
        uint64_t nodes = 0;
        uint32_t depth = 0;
        if (!ok) {
            status = QSMD_STATUS_ENCODE_ERROR;
        } else if (n_ev == 0) {
            status = QSMD_STATUS_LINEARISABLE;                       // :59
        } else {
            // ---- model in registers
            uint32_t ex = a.m0_exists, neg = 0;
            int32_t bal[8];
            uint32_t just = a.m0_just;
            int32_t tn = (int32_t)a.m0_val[0];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                bal[q] = ((ex >> q) & 1u) ? (int32_t)a.m0_val[q] : 0;
                neg |= (((ex >> q) & 1u) && bal[q] < 0) ? (1u << q) : 0u;
            }

            uint32_t rem = INV | RESP;
            uint32_t cand = cands(rem, INV, RESP);
            bool found = false;
            uint32_t iter = 0;
            for (;;) {
                if (!cand) {
                    if (!found) {        // no children: leaf => True, root => False
                        status = depth == 0 ? QSMD_STATUS_NONLINEARISABLE : QSMD_STATUS_LINEARISABLE;
                        break;
                    }
                    if (depth == 0) { status = QSMD_STATUS_NONLINEARISABLE; break; }
                    // ---- backtrack
                    --depth;
                    const uint32_t st = s_st[depth][lane];
                    const uint32_t j = st & 31u;
                    const uint32_t cj = s_ev[j][lane];
                    const uint32_t pmj = same_pid(j);
                    const uint32_t gone = ~rem & pmj;
                    rem |= (1u << (31 - __builtin_clz(gone & INV))) |
                           (1u << (31 - __builtin_clz(gone & RESP)));
                    if constexpr (BANK) {
                        const uint32_t code = c_code(cj);
                        if (code != QSMD_BANK_CHECK_BALANCE) {
                            const uint32_t ia = c_a(cj), ib = c_b(cj);
                            const int32_t m = c_val(cj);
                            const uint32_t pa = (st >> 5) & 1u, pb = (st >> 6) & 1u;
                            if (code == QSMD_BANK_TRANSFER) {
                                const bool mid = pb || ia == ib;
                                put8(bal, ib, mid ? sel8(bal, ib) - m : 0);
                            }
                            const int32_t delta = code == QSMD_BANK_DEPOSIT ? m
                                                : code == QSMD_BANK_OPEN_ACCOUNT ? 0 : -m;
                            put8(bal, ia, pa ? sel8(bal, ia) - delta : 0);
                            ex = (ex & ~(1u << ia)) | (pa << ia);
                            if (code == QSMD_BANK_TRANSFER) ex = (ex & ~(1u << ib)) | (pb << ib);
                            const int32_t va = sel8(bal, ia), vb = sel8(bal, ib);
                            neg = (neg & ~((1u << ia) | (1u << ib))) |
                                  ((((ex >> ia) & 1u) && va < 0) ? (1u << ia) : 0u) |
                                  ((((ex >> ib) & 1u) && vb < 0) ? (1u << ib) : 0u);
                        }
                    } else {
                        just = (st >> 5) & 1u;
                        tn = (int32_t)st >> 6;
                    }
                    cand = cands(rem, INV, RESP) & ~below32(j + 1u);
                    found = true;
                    continue;
                }
                if (a.time_limit && ((++iter & 1023u) == 0u) &&
                    __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                    atomicOr(a.timed_out, 1u);
                    status = QSMD_STATUS_BUDGET;
                    break;
                }
                // ---- next candidate: addresses from registers, one LDS round trip
                const uint32_t j = (uint32_t)__builtin_ctz(cand);
                cand &= cand - 1u;
                const uint32_t pmj = same_pid(j);
                const uint32_t rr = rem & pmj & RESP;
                if (!rr) continue;                    // findResponse => []: no child
                found = true;
                if (a.max_nodes && nodes >= a.max_nodes) { status = QSMD_STATUS_BUDGET; break; }
                ++nodes;
                const uint32_t r = (uint32_t)__builtin_ctz(rr);
                const uint32_t cj = s_ev[j][lane];
                const uint32_t cr = s_ev[r][lane];
                const uint32_t code = c_code(cj), rc = c_code(cr);
                const int32_t m = c_val(cj), rv = c_val(cr);
                uint32_t stw;
                if constexpr (BANK) {
                    // post (test/Bank.hs:118-131)
                    const uint32_t ia = c_a(cj), ib = c_b(cj);
                    const bool ex_a = (ex >> ia) & 1u;
                    const int32_t bal_a = sel8(bal, ia);
                    if (neg) continue;                            // invariant model
                    const uint32_t exp = bank_expected(code, ex_a, bal_a, m);
                    if (rc != exp) continue;
                    if (code == QSMD_BANK_CHECK_BALANCE) {
                        if (!ex_a) { status = QSMD_STATUS_MODEL_ERROR; break; }   // Map.!
                        if (rv != bal_a) continue;
                    }
                    // descend: next' (test/Bank.hs:92-101)
                    const uint32_t pb = (ex >> ib) & 1u;
                    stw = j | ((ex_a ? 1u : 0u) << 5) | (pb << 6);
                    if (code != QSMD_BANK_CHECK_BALANCE) {
                        int32_t na;
                        if (code == QSMD_BANK_OPEN_ACCOUNT) na = ex_a ? bal_a : 0;
                        else if (code == QSMD_BANK_DEPOSIT) na = ex_a ? bal_a + m : m;
                        else na = ex_a ? bal_a - m : m;       // Withdraw / Transfer's withdraw
                        put8(bal, ia, na);
                        ex |= 1u << ia;
                        if (code == QSMD_BANK_TRANSFER) {
                            const bool ex_b = (ex >> ib) & 1u;
                            put8(bal, ib, ex_b ? sel8(bal, ib) + m : m);
                            ex |= 1u << ib;
                        }
                        const int32_t va = sel8(bal, ia), vb = sel8(bal, ib);
                        neg = (neg & ~((1u << ia) | (1u << ib))) |
                              ((((ex >> ia) & 1u) && va < 0) ? (1u << ia) : 0u) |
                              ((((ex >> ib) & 1u) && vb < 0) ? (1u << ib) : 0u);
                    }
                } else {
                    // postcondition (test/TicketDispenser.hs:99-102)
                    const bool tt = code == QSMD_TICKET_TAKE_TICKET && rc == QSMD_TICKET_NUMBER &&
                                    just && rv == tn + 1;
                    const bool rs = code == QSMD_TICKET_RESET && rc == QSMD_TICKET_OK;
                    if (!(tt || rs)) continue;
                    stw = j | (just << 5) | ((uint32_t)tn << 6);
                    if (code == QSMD_TICKET_TAKE_TICKET) tn += (int32_t)just;   // succ <$> m
                    else { just = 1u; tn = 0; }                                 // Just 0
                }
                s_st[depth][lane] = stw;
                ++depth;
                const uint32_t fi = rem & pmj & INV;
                rem &= ~((fi & (0u - fi)) | (1u << r));
                cand = cands(rem, INV, RESP);
                found = false;
            }
        }

        a.status[h] = (uint8_t)status;
        if (a.nodes) a.nodes[h] = nodes;
        if (a.witness && status == QSMD_STATUS_LINEARISABLE) {
            uint8_t* w = a.witness + H.ev_off;
            for (uint32_t d = 0; d < depth; ++d) w[d] = (uint8_t)(s_st[d][lane] & 31u);
            if (depth < n_ev) w[depth] = QSMD_WITNESS_END;
        }
        c_lin += status == QSMD_STATUS_LINEARISABLE;
        c_nonlin += status == QSMD_STATUS_NONLINEARISABLE;
        c_err += status == QSMD_STATUS_MODEL_ERROR;
        c_enc += status == QSMD_STATUS_ENCODE_ERROR;
        c_budget += status == QSMD_STATUS_BUDGET;
        c_nodes += nodes;
    }

    const uint64_t t_lin = wave_sum64(c_lin), t_non = wave_sum64(c_nonlin), t_err = wave_sum64(c_err),
                   t_enc = wave_sum64(c_enc), t_bud = wave_sum64(c_budget), t_nodes = wave_sum64(c_nodes);
    if (lane == 0) {
        unsigned long long* p = a.partials + (uint64_t)blockIdx.x * T_N;
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

hipError_t launch_compact(const SearchArgs& a, uint32_t grid, hipStream_t s) {
    if (a.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL(compact_search<QSMD_MODEL_BANK>, dim3(grid), dim3(C_LANES), 0, s, a);
    else
        hipLaunchKernelGGL(compact_search<QSMD_MODEL_TICKET>, dim3(grid), dim3(C_LANES), 0, s, a);
    return hipGetLastError();
}

}  // namespace qsmd
