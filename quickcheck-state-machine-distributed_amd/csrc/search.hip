// search.hip -- the linearisability search on gfx950 (MI355X).
//
// Restates src/Linearisability.hs:25-69 (advancedtelematic/
// quickcheck-state-machine-distributed) as an explicit-stack DFS over the
// counter state of SURVEY.md §8a Lemma L1, encoded as an event bitset:
//
//   rem        remaining events of the history (bit e = event e)
//   R          first remaining response          (takeInvocations, :25-28)
//   candidates remaining invocations before R, ascending position  (:40)
//   child(j)   pid p = pid(j): removes the FIRST remaining invocation of p
//              (filter1, :41,:47-50) and the FIRST remaining response of p
//              (findResponse, :30-34); the node is Operation p inv_j resp.
//   step       postcondition && any' children, any' [] = True  (:63-69)
//   root       [] => True; plain `any`, no roots => False       (:59-61)
//
// One node = one `step` evaluation; the count is exact for the reference's
// lazy left-to-right short-circuit order (candidates are tried in ascending
// position, the first success ends the search).
//
// Layout: ONE HISTORY PER LANE.  A workgroup is one wavefront of 64 lanes;
// each lane's history, pid masks and DFS stack live in LDS laid out
// [slot][lane], so every per-lane random index is bank-conflict free
// (bank = lane-determined).  Histories that exceed a stage's capacity are
// appended (wave-aggregated atomics) to a deferred list that the next stage
// consumes in list mode without a host round trip:
//   stage 0: <= 32 events, <= 8 pids, u32 masks, 64 lanes  (the 4x16 Bank bench)
//   stage 1: <= 64 events, <= 8 pids, u64 masks, 64 lanes
//   stage 2: <= 128 events, <= 128 pids, 128-bit masks, 16 lanes
#include <hip/hip_runtime.h>

#include "internal.h"
#include "mask.h"
#include "models.h"

namespace qsmd {

__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int W>
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, W);
    return v;
}

template <uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
__global__ __launch_bounds__(LANES) void lane_search(SearchArgs a) {
    using Ops = MaskOps<MaskT>;
    constexpr int MAXD = MAXEV / 2;
    constexpr bool BANK = MODEL == QSMD_MODEL_BANK;

    __shared__ uint2 s_ev[MAXEV][LANES];
    __shared__ MaskT s_pm[MAXPID][LANES];
    __shared__ MaskT s_cand[MAXD][LANES];
    __shared__ uint32_t s_meta[MAXD][LANES];
    __shared__ int64_t s_undo[BANK ? 1 : MAXD][LANES];
    __shared__ int64_t s_bal[BANK ? QSMD_BANK_MAX_ACCOUNTS : 1][LANES];

    const int lane = threadIdx.x;
    const bool list_mode = a.list != nullptr;
    const uint64_t total = list_mode ? (uint64_t)*a.list_count : a.n_hist;

    uint32_t c_lin = 0, c_nonlin = 0, c_err = 0, c_enc = 0, c_budget = 0;
    uint64_t c_nodes = 0;
    const uint64_t t0 = a.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t limit = stage_limit(a);

    for (uint64_t base = (uint64_t)blockIdx.x * LANES; base < total;
         base += (uint64_t)gridDim.x * LANES) {
        const uint64_t idx = base + lane;
        const bool active = idx < total;
        const uint32_t h = active ? (list_mode ? a.list[idx] : (uint32_t)idx) : 0u;

        qsmd_hdr H;
        if (active) H = a.hdr[h];
        else H = qsmd_hdr{0, 0, 0, 0, 0, 0};
        const uint32_t n_ev = H.n_ev, n_pid = H.n_pid;
        const bool enc_ok = active && H.model_id == MODEL && n_ev <= QSMD_MAX_EVENTS &&
                            n_pid <= QSMD_MAX_PIDS && (uint64_t)H.ev_off + n_ev <= a.n_events;
        const bool defer = enc_ok && (n_ev > (uint32_t)MAXEV || n_pid > (uint32_t)MAXPID);

        // ---- overflow to the next stage (wave-aggregated append)
        const uint64_t dm = __ballot(defer);
        if (dm) {
            const int leader = __builtin_ctzll(dm);
            uint32_t slot = 0;
            if (lane == leader) slot = atomicAdd(a.defer_count, (uint32_t)__builtin_popcountll(dm));
            slot = __shfl(slot, leader, LANES);
            if (defer) a.defer_list[slot + lane_prefix(dm)] = h;
        }
        if (!active || defer) continue;

        int status = -1;
        uint64_t nodes = 0;
        int depth = 0;

        // ---- stage the history into LDS, validate, build masks
        MaskT INV{}, RESP{};
        bool ok = enc_ok;
        if (ok) {
            for (uint32_t p = 0; p < n_pid; ++p) s_pm[p][lane] = MaskT{};
            const uint2* evp = a.events + H.ev_off;
            for (uint32_t e0 = 0; e0 < n_ev; e0 += 8) {
                uint2 xs[8];                       // 8 independent loads in flight
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k)
                    xs[k] = e0 + k < n_ev ? evp[e0 + k] : make_uint2(0u, 0u);
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint32_t e = e0 + k;
                    if (e >= n_ev) break;
                    const uint2 x = xs[k];
                    const Ev ev{x.x, (int32_t)x.y};
                    const uint32_t p = ev.pid();
                    ok = ok && p < n_pid && valid_event<MODEL>(ev);
                    s_ev[e][lane] = x;
                    const MaskT bit = Ops::bit((int)e);
                    if (ev.is_resp()) RESP |= bit; else INV |= bit;
                    if (p < n_pid) s_pm[p][lane] = s_pm[p][lane] | bit;
                }
            }
        }
        if (!ok) {
            status = QSMD_STATUS_ENCODE_ERROR;
        } else if (n_ev == 0) {
            status = QSMD_STATUS_LINEARISABLE;                     // :59
        } else if (beyond_first_fail(a, h)) {
            status = QSMD_STATUS_SKIPPED;                          // early exit
        } else {
            // ---- model0
            BankState bank{a.m0_exists, 0u};
            TicketState tick{a.m0_just, a.m0_val[0]};
            if constexpr (BANK) {
#pragma unroll
                for (int c = 0; c < QSMD_BANK_MAX_ACCOUNTS; ++c) {
                    const bool ex = (a.m0_exists >> c) & 1u;
                    const int64_t v = ex ? a.m0_val[c] : 0;
                    s_bal[c][lane] = v;
                    bank.neg |= (ex && v < 0) ? (1u << c) : 0u;
                }
            }

            // ---- DFS
            MaskT rem = INV | RESP;
            auto candidates = [&](const MaskT& r) -> MaskT {
                const MaskT rr = r & RESP;
                const int R = Ops::any(rr) ? Ops::ctz(rr) : Ops::BITS;
                return r & INV & Ops::below(R);
            };
            MaskT cand = candidates(rem);
            bool found = false;
            uint32_t iter = 0;
            for (;;) {
                if (!Ops::any(cand)) {
                    if (!found) {           // no children: leaf => True; root => False
                        status = depth == 0 ? QSMD_STATUS_NONLINEARISABLE : QSMD_STATUS_LINEARISABLE;
                        break;
                    }
                    if (depth == 0) { status = QSMD_STATUS_NONLINEARISABLE; break; }
                    // ---- backtrack: restore the parent level
                    --depth;
                    cand = s_cand[depth][lane];
                    const uint32_t meta = s_meta[depth][lane];
                    const uint2 xj = s_ev[meta & 0xFFu][lane];
                    const Ev ej{xj.x, (int32_t)xj.y};
                    const MaskT gone = ~rem & s_pm[ej.pid()][lane];
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
                                s_bal[ib][lane] = exb_mid ? s_bal[ib][lane] - m : 0;
                            }
                            const int64_t delta = code == QSMD_BANK_DEPOSIT ? m
                                                : code == QSMD_BANK_OPEN_ACCOUNT ? 0 : -m;
                            s_bal[ia][lane] = ((pre_ex >> ia) & 1u) ? s_bal[ia][lane] - delta : 0;
                            bank.exists = pre_ex;
                            bank.neg = (meta >> 16) & 0xFFu;
                        }
                    } else {
                        tick.just = (meta >> 8) & 1u;
                        tick.n = s_undo[depth][lane];
                    }
                    found = true;
                    continue;
                }
                if (((++iter & 1023u) == 0u)) {
                    if (beyond_first_fail(a, h)) { status = QSMD_STATUS_SKIPPED; break; }
                    if (a.time_limit && __builtin_amdgcn_s_memrealtime() - t0 > a.time_limit) {
                        atomicOr(a.timed_out, 1u);
                        status = QSMD_STATUS_BUDGET;
                        break;
                    }
                }
                // ---- next candidate of this level
                const int j = Ops::ctz(cand);
                cand = Ops::clear_lowest(cand);
                const uint2 xj = s_ev[j][lane];
                const Ev ej{xj.x, (int32_t)xj.y};
                const MaskT pm = s_pm[ej.pid()][lane];
                const MaskT rr = rem & pm & RESP;
                if (!Ops::any(rr)) continue;            // findResponse => []: no child
                found = true;
                if (nodes >= limit) { status = QSMD_STATUS_BUDGET; break; }
                ++nodes;
                const int r = Ops::ctz(rr);
                const uint2 xr = s_ev[r][lane];
                const Ev er{xr.x, (int32_t)xr.y};

                int post;
                int64_t bal_a = 0;
                if constexpr (BANK) {
                    bal_a = s_bal[ej.a()][lane];
                    post = bank_post(bank, ej, er, bal_a);
                } else {
                    post = ticket_post(tick, ej, er);
                }
                if (post == POST_ERROR) { status = QSMD_STATUS_MODEL_ERROR; break; }
                if (post == POST_FALSE) continue;

                // ---- descend: push this level, apply transition (Left inv; Right is id)
                s_cand[depth][lane] = cand;
                if constexpr (BANK) {
                    s_meta[depth][lane] = (uint32_t)j | (bank.exists << 8) | (bank.neg << 16);
                    const uint32_t code = ej.code();
                    if (code != QSMD_BANK_CHECK_BALANCE) {
                        const int ia = (int)ej.a();
                        const int64_t m = ej.val;
                        const bool ex_a = (bank.exists >> ia) & 1u;
                        int64_t na;
                        if (code == QSMD_BANK_OPEN_ACCOUNT) na = ex_a ? bal_a : 0;
                        else if (code == QSMD_BANK_DEPOSIT) na = ex_a ? bal_a + m : m;
                        else na = ex_a ? bal_a - m : m;      // Withdraw / Transfer's withdraw
                        s_bal[ia][lane] = na;
                        bank.exists |= 1u << ia;
                        bank.neg = (bank.neg & ~(1u << ia)) | (na < 0 ? (1u << ia) : 0u);
                        if (code == QSMD_BANK_TRANSFER) {
                            const int ib = (int)ej.b();
                            const bool ex_b = (bank.exists >> ib) & 1u;
                            const int64_t nb = ex_b ? s_bal[ib][lane] + m : m;
                            s_bal[ib][lane] = nb;
                            bank.exists |= 1u << ib;
                            bank.neg = (bank.neg & ~(1u << ib)) | (nb < 0 ? (1u << ib) : 0u);
                        }
                    }
                } else {
                    s_meta[depth][lane] = (uint32_t)j | (tick.just << 8);
                    s_undo[depth][lane] = tick.n;
                    ticket_apply(tick, ej);
                }
                ++depth;
                const MaskT first_inv = Ops::lowest(rem & pm & INV);
                rem &= ~(first_inv | Ops::bit(r));
                cand = candidates(rem);
                found = false;
            }
        }

        // ---- outputs (over the split budget: searched again by the split stage)
        if (to_split(a, status, nodes)) {
            a.giant_list[atomicAdd(a.giant_count, 1u)] = h;
            continue;
        }
        note_failure(a, h, status);
        a.status[h] = (uint8_t)status;
        if (a.nodes) a.nodes[h] = nodes;
        if (a.witness && status == QSMD_STATUS_LINEARISABLE) {
            uint8_t* w = a.witness + H.ev_off;
            for (int d = 0; d < depth; ++d) w[d] = (uint8_t)(s_meta[d][lane] & 0xFFu);
            if ((uint32_t)depth < n_ev) w[depth] = QSMD_WITNESS_END;
        }
        if (status == QSMD_STATUS_SKIPPED) continue;           // counted by early_exit_fixup
        c_lin += status == QSMD_STATUS_LINEARISABLE;
        c_nonlin += status == QSMD_STATUS_NONLINEARISABLE;
        c_err += status == QSMD_STATUS_MODEL_ERROR;
        c_enc += status == QSMD_STATUS_ENCODE_ERROR;
        c_budget += status == QSMD_STATUS_BUDGET;
        c_nodes += nodes;
    }

    // ---- per-block partial totals (one wave per block)
    const uint64_t t_lin = wave_sum<LANES>(c_lin), t_non = wave_sum<LANES>(c_nonlin),
                   t_err = wave_sum<LANES>(c_err), t_enc = wave_sum<LANES>(c_enc),
                   t_bud = wave_sum<LANES>(c_budget), t_nodes = wave_sum<LANES>(c_nodes);
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

// QSMD_FLAG_EARLY_EXIT_BATCH: histories after the first non-linearisable
// (or raising) one are SKIPPED, whatever a search kernel wrote for them, and
// the totals are recounted from the final status / nodes arrays.
__global__ __launch_bounds__(64) void early_exit_fixup_kernel(uint8_t* status, uint64_t* nodes, uint64_t n,
                                                             const uint32_t* first_fail,
                                                             unsigned long long* partials) {
    const uint32_t ff = *first_fail;
    uint64_t c[T_N] = {};
    for (uint64_t h = (uint64_t)blockIdx.x * 64 + threadIdx.x; h < n; h += (uint64_t)gridDim.x * 64) {
        if (h > ff) {
            status[h] = QSMD_STATUS_SKIPPED;
            nodes[h] = 0;
            c[T_SKIPPED] += 1;
            continue;
        }
        const uint32_t st = status[h];
        c[T_LIN] += st == QSMD_STATUS_LINEARISABLE;
        c[T_NONLIN] += st == QSMD_STATUS_NONLINEARISABLE;
        c[T_ERR] += st == QSMD_STATUS_MODEL_ERROR;
        c[T_ENC] += st == QSMD_STATUS_ENCODE_ERROR;
        c[T_BUDGET] += st == QSMD_STATUS_BUDGET;
        c[T_NODES] += nodes[h];
    }
    c[T_CHECKED] = c[T_LIN] + c[T_NONLIN] + c[T_ERR];
#pragma unroll
    for (int k = 0; k < T_N; ++k) {
        const uint64_t s = wave_sum<64>(c[k]);
        if (threadIdx.x == 0) partials[(uint64_t)blockIdx.x * T_N + k] = s;
    }
}

hipError_t launch_early_exit_fixup(uint8_t* status, uint64_t* nodes, uint64_t n, const uint32_t* first_fail,
                                   unsigned long long* partials, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(early_exit_fixup_kernel, dim3(grid), dim3(64), 0, s, status, nodes, n, first_fail, partials);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void reduce_totals_kernel(const unsigned long long* partials,
                                                            uint64_t n_blocks, qsmd_totals* totals) {
    __shared__ unsigned long long acc[T_N][256];
    unsigned long long v[T_N] = {};
    for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < n_blocks;
         b += (uint64_t)gridDim.x * 256) {
#pragma unroll
        for (int k = 0; k < T_N; ++k) v[k] += partials[b * T_N + k];
    }
#pragma unroll
    for (int k = 0; k < T_N; ++k) acc[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
#pragma unroll
            for (int k = 0; k < T_N; ++k) acc[k][threadIdx.x] += acc[k][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x < T_N) {
        unsigned long long* t = reinterpret_cast<unsigned long long*>(totals);
        atomicAdd(&t[threadIdx.x], acc[threadIdx.x][0]);
    }
}

// One launch instead of three memsets before a call: the 32 stage counters
// (counter 6 = first failing history = none), and the totals the reduce
// kernel accumulates into.
__global__ __launch_bounds__(64) void prep_kernel(uint32_t* cnt, unsigned long long* totals) {
    const uint32_t t = threadIdx.x;
    if (t < 32u) cnt[t] = t == 6u ? 0xFFFFFFFFu : 0u;
    if (t < (uint32_t)T_N) totals[t] = 0ull;
}

hipError_t launch_prep(uint32_t* cnt, qsmd_totals* totals, hipStream_t s) {
    hipLaunchKernelGGL(prep_kernel, dim3(1), dim3(64), 0, s, cnt, reinterpret_cast<unsigned long long*>(totals));
    return hipGetLastError();
}

// ------------------------------------------------------------------ launch

namespace {
template <uint32_t MODEL>
hipError_t launch_model(int stage, const SearchArgs& a, uint32_t grid, hipStream_t s) {
    switch (stage) {
    case 0:
        hipLaunchKernelGGL((lane_search<MODEL, uint32_t, 32, 8, 64>), dim3(grid), dim3(64), 0, s, a);
        break;
    case 1:
        hipLaunchKernelGGL((lane_search<MODEL, uint64_t, 64, 8, 64>), dim3(grid), dim3(64), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL((lane_search<MODEL, M128, 128, 128, 16>), dim3(grid), dim3(16), 0, s, a);
        break;
    }
    return hipGetLastError();
}
}  // namespace

uint32_t stage_lanes(int stage) { return stage < 2 ? 64u : 16u; }
uint32_t stage_max_events(int stage) { return stage == 0 ? 32u : stage == 1 ? 64u : 128u; }

hipError_t launch_stage(int stage, const SearchArgs& a, uint32_t grid, hipStream_t s) {
    if (a.model_id == QSMD_MODEL_BANK) return launch_model<QSMD_MODEL_BANK>(stage, a, grid, s);
    return launch_model<QSMD_MODEL_TICKET>(stage, a, grid, s);
}

hipError_t launch_reduce(const unsigned long long* partials, uint64_t n_blocks,
                         qsmd_totals* totals, hipStream_t s) {
    uint32_t grid = (uint32_t)((n_blocks + 255) / 256);
    if (grid > 64) grid = 64;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(reduce_totals_kernel, dim3(grid), dim3(256), 0, s, partials, n_blocks, totals);
    return hipGetLastError();
}

}  // namespace qsmd
