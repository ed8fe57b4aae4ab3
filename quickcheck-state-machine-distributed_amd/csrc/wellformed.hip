// wellformed.hip -- batched `wellformed` (src/Linearisability.hs:97-135):
// the O(n) check the reference runs on each history before the search
// (test/Bank.hs:281-283), over the same SoA as the search.
//
//   wellformed pids history = allRight [ isSequential (processSubhistory p h) | p <- pids ]
//
// i.e. each listed pid's subhistory must be sequential, and the result is
// the first error in `pids` order.  isSequential on one pid's subsequence
// e0 e1 e2 ...:
//   e0 a response                       -> FirstEventIsntInvocation e0
//   then pairs (e2k, e2k+1):  L R -> go on;  L L -> InvocationFollowedByInvocation
//                             R R -> ResponseFollowedByResponse;  R L -> ResponseFollowedByInvocation
//   a last unpaired e2k:      L -> fine;  R -> LoneResponse
// (InvocationFollowedByNonMatchingResponse compares pids of one subhistory,
// which are equal, so wellformed never yields it.)
//
// One history per lane, all pids in one pass over the events: a u16 state per
// (pid, lane) in LDS [pid][lane] (started, odd position, pending kind,
// done, pending event index); the error kept is the one of the pid with the
// smallest rank in `pids`.  HBM-bound: 16 B header + 8 B per event in, 8 B out.
#include <hip/hip_runtime.h>

#include "internal.h"

namespace qsmd {

namespace {

constexpr int WF_LANES = 64;
constexpr int WF_MAXPID = QSMD_MAX_PIDS;
enum : uint32_t { S_STARTED = 1, S_ODD = 2, S_PEND_R = 4, S_DONE = 8 };

}  // namespace

__global__ __launch_bounds__(WF_LANES) void wellformed_kernel(const qsmd_hdr* hdr, uint64_t n_hist,
                                                             const uint2* events, uint64_t n_events,
                                                             const uint8_t* rank_in, qsmd_wf* out) {
    __shared__ uint16_t s_st[WF_MAXPID][WF_LANES];
    __shared__ uint8_t s_rank[WF_MAXPID];
    const int lane = threadIdx.x;
    for (int p = lane; p < WF_MAXPID; p += WF_LANES) s_rank[p] = rank_in ? rank_in[p] : (uint8_t)p;
    __syncthreads();
    for (uint64_t h = (uint64_t)blockIdx.x * WF_LANES + lane; h - lane < n_hist;
         h += (uint64_t)gridDim.x * WF_LANES) {
        if (h >= n_hist) continue;
        const qsmd_hdr H = hdr[h];
        const uint32_t n_ev = H.n_ev, n_pid = H.n_pid;
        qsmd_wf r{0u, 0u, 0u, 0u, 0u};
        if (n_ev > QSMD_MAX_EVENTS || n_pid > QSMD_MAX_PIDS || (uint64_t)H.ev_off + n_ev > n_events) {
            r.code = QSMD_WF_ENCODE_ERROR;
            out[h] = r;
            continue;
        }
        for (uint32_t p = 0; p < n_pid; ++p) s_st[p][lane] = 0;
        uint32_t best = 0xFFu;                 // rank of the pid of the error kept
        const uint2* evp = events + H.ev_off;
        for (uint32_t c0 = 0; c0 < n_ev; c0 += 16) {
            uint2 x[16];
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) {
                const uint32_t e = c0 + k;
                x[k] = evp[e < n_ev ? e : n_ev - 1];
            }
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) {
                const uint32_t e = c0 + k;
                if (e >= n_ev) break;
                const uint32_t kp = x[k].x & 0xFFu, p = kp & QSMD_EV_PID_MASK, resp = kp >> 7;
                if (p >= n_pid) {
                    r.code = QSMD_WF_ENCODE_ERROR;
                    best = 0u;
                    continue;
                }
                const uint32_t rk = s_rank[p];
                if (rk == 0xFFu || rk >= best) continue;   // not listed, or an earlier-ranked error exists
                uint32_t st = s_st[p][lane];
                if (st & S_DONE) continue;
                uint32_t code = 0, e0 = 0;
                if (!(st & S_STARTED)) {
                    if (resp) {
                        code = QSMD_WF_FIRST_EVENT_ISNT_INVOCATION;
                        e0 = e;
                    } else {
                        st = S_STARTED | S_ODD | (e << 8);
                    }
                } else if (st & S_ODD) {                   // e is e(2k+1); e(2k) is pending
                    const uint32_t pend = st >> 8;
                    const bool pr = (st & S_PEND_R) != 0u;
                    if (!pr && resp) st = S_STARTED;       // L R: the pair is done
                    else {
                        code = !pr ? QSMD_WF_INVOCATION_FOLLOWED_BY_INVOCATION
                                   : (resp ? QSMD_WF_RESPONSE_FOLLOWED_BY_RESPONSE
                                           : QSMD_WF_RESPONSE_FOLLOWED_BY_INVOCATION);
                        e0 = pend;
                    }
                } else {                                   // e is e(2k), k >= 1
                    st = S_STARTED | S_ODD | (resp ? S_PEND_R : 0u) | (e << 8);
                }
                if (code) {
                    st |= S_DONE;
                    if (rk < best) {
                        best = rk;
                        r.code = (uint8_t)code;
                        r.pid = (uint8_t)p;
                        r.ev0 = (uint16_t)e0;
                        r.ev1 = (uint16_t)(code == QSMD_WF_FIRST_EVENT_ISNT_INVOCATION ? e0 : e);
                    }
                }
                s_st[p][lane] = (uint16_t)st;
            }
            if (r.code == QSMD_WF_ENCODE_ERROR) break;
        }
        if (r.code != QSMD_WF_ENCODE_ERROR) {
            // a last unpaired response: LoneResponse
            for (uint32_t p = 0; p < n_pid; ++p) {
                const uint32_t st = s_st[p][lane], rk = s_rank[p];
                if (rk != 0xFFu && rk < best && !(st & S_DONE) && (st & S_ODD) && (st & S_PEND_R)) {
                    best = rk;
                    r.code = QSMD_WF_LONE_RESPONSE;
                    r.pid = (uint8_t)p;
                    r.ev0 = r.ev1 = (uint16_t)(st >> 8);
                }
            }
        }
        out[h] = r;
    }
}

hipError_t launch_wellformed(const qsmd_hdr* hdr, uint64_t n_hist, const uint2* events, uint64_t n_events,
                             const uint8_t* rank, qsmd_wf* out, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(wellformed_kernel, dim3(grid), dim3(WF_LANES), 0, s, hdr, n_hist, events, n_events, rank, out);
    return hipGetLastError();
}

}  // namespace qsmd
