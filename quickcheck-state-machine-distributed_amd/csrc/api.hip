// api.hip -- the C ABI of include/qsmd.h: context, workspace, stage cascade.
//
// Replaces the call `linearisable transition postcondition model0 hist`
// (src/Linearisability.hs:52-69) made once per history at test/Bank.hs:285,
// test/TicketDispenser.hs:253 and :320 with one batched call.  The model
// closures are selected by model_id (device functors, csrc/models.h).
//
// One call = four launches on one stream (internal.h): stage 0, stage 0w,
// the heavy stage, the giant stage.  No host round trip, no memset: the
// giant stage's last workgroup restores the call's counters and buckets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <mutex>
#include <string>
#include <vector>

#include "internal.h"
#include "qsmd_gen.h"

#include "qsmd.h"

using namespace qsmd;

struct qsmd_ctx {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::string err;
    // workspace (device): header (counters, buckets) + lists + giant records + tasks
    char* ws = nullptr;
    size_t ws_bytes = 0;
    bool ws_dirty = true;              // the header must be restored before the next call
    // staging for the host-memory entry point: device buffer and its pinned
    // host mirror (one copy in, one copy out per call)
    char* io = nullptr;
    size_t io_bytes = 0;
    char* pin = nullptr;
    size_t pin_bytes = 0;
    // small host calls: a mapped, coherent host buffer the kernels read and
    // write directly (no copy in or out)
    char* zc = nullptr;
    char* zc_dev = nullptr;
    // the calls of this context are ordered: each waits for the previous one
    // (whatever its stream), and buffers are freed only once it is done
    hipEvent_t done_ev = nullptr;
    // A call on a caller's stream records the completion event, so that the
    // context's later waits (quiesce, qsmd_close, a call on another stream)
    // never name a stream the caller may have destroyed since; a call on the
    // context's own stream (the host entry, which also waits for it before
    // returning) does not need it
    bool done_last = false;            // the last call recorded done_ev
    hipStream_t last_stream = nullptr;
    bool in_flight = false;
    bool any_call = false;             // a check call was enqueued
    bool probe_valid = false;          // a check call finished: probe_host holds real counts
    // timing: per call, events at stage 0's start and end, after the last
    // launch, and at the heavy stage's start and end, recorded on the launch
    // stream (a ring of kTimingSlots)
    std::vector<hipEvent_t> ev;        // kSlotEvents per slot
    std::vector<uint8_t> ev_no0;       // per slot: 1 stage 0 skipped (its end event not recorded), 2 no heavy events
    uint64_t n_calls = 0;              // calls recorded since the last reset
    bool timed = false;
    // the per-call timing events above are recorded (from qsmd_timing_reset
    // on, or knob timing_events): three event packets per call that a lone
    // caller pays ~13 us a call for (one call at a time 4.32 vs 4.59e9 with
    // and without, tools/gpu/r04_tev.sh), so off until asked for
    bool timing = false;
    uint64_t time_limit_ms = 120000;   // safety net per search launch
    uint64_t stage0_max_grid = 65536;  // tuning: cap on stage-0 workgroups (grid-stride beyond)
    uint64_t stage0_budget = 32;       // stage-0 node budget before the heavy stage (when not automatic)
    // automatic stage-0 budget (until a budget is set): 24, or 16 while the
    // last finished call's stage 0 sent few histories to the heavy stage --
    // one call at a time on config 2: 4.78 vs 4.59e9 (the heavy list long
    // enough for lane mode, whose tail is no longer than wave mode's, behind
    // a shorter stage 0); config 3's bug-laden batches keep 24 (their heavy
    // fraction at 16 is far above the threshold; 24 vs 32 with the ordered
    // groups and the tail launch: 1.55 vs 1.49e9, profiles/r06/xbudget)
    bool s0_auto = true;
    uint64_t stage0w_budget = 32;      // stage-0w node budget before the heavy stage (when not automatic)
    // automatic stage-0w budget (until one is set): 24 when the heavy stage
    // runs in lane mode, 48 in wave mode -- config 5 (100k 6x24, 3 calls in
    // flight): lane mode 9.0 / 11.2 / 10.6 / 9.6e8 at 16 / 24 / 32 / 48, wave
    // mode 7.4 / 10.7 / 10.1 / 9.2e8 at 32 / 48 / 64 / 96, and its lone call
    // shortest in wave mode at 48 (profiles/r06/config5/)
    bool s0w_auto = true;
    uint64_t split_budget = 1024;      // giant stage: whole-search iterations = 16x, heavy-stage cap = 64x
    uint64_t wave_grid = 0;            // heavy stage, wave mode: workgroups (0 = from the last call's heavy count)
    uint64_t wave_min_rem = 4;         // heavy stage, wave mode: nodes with at most this many events left skip the memo
    uint64_t dag_states = 128;         // heavy stage, wave mode: state-DAG capacity per wavefront (0 = DFS only)
    uint32_t* dag_dbg = nullptr;       // diagnostic (dag_debug_ptr / dag_debug_hist)
    uint64_t dag_dbg_h = 0;
    unsigned long long* wave_stats = nullptr;   // diagnostic (wave_stats_ptr): 16 x u64 (include/qsmd.h)
    unsigned long long* memo_stats = nullptr;   // diagnostic (memo_stats_ptr): 16 x u64 per heavy-stage group
    uint64_t memo_stats_groups = 0;             // (memo_stats_groups)
    uint32_t memo_lds = 1;                      // heavy-stage memo tables in LDS: 0 never, 1 short lists, 2 always
    uint64_t giant_grid = 0;           // giant stage workgroups (0 = 2 per CU)
    uint64_t giant_stall_us = 0;       // diagnostic: the giant stage's first frontier chunk starts this late
    unsigned long long* s0_stamps = nullptr;    // diagnostic (stage0_stamps_ptr): 8 x u64 per stage-0 workgroup
    // heavy stage: one wavefront per history (wave_search, csrc/wave.hip)
    // unless the last finished call sent more than wave_max histories there
    // (then one lane per history, memo_search, csrc/memo.hip); heavy_mode
    // 0 / 1 forces wave / lane mode, 2 (default) picks
    uint64_t heavy_mode = 2;
    uint64_t wave_max = 16384;
    // lane mode's folded tail: a call whose predecessor deferred nothing to
    // stage 0w launches no stage 0w (what stage 0 defers goes on to the giant
    // stage through the heavy stage); 0 = every call launches it.  With calls
    // in flight each launch of a call's chain waits for dispatch behind the
    // other streams' stage 0 (round 4's trace: the empty stage 0w 25 us a call
    // on average, 4 us alone)
    uint64_t fold = 1;
    uint32_t* probe_host = nullptr;    // pinned: [defer, heavy32, heavy64, giant, timed] of the last finished call
    uint32_t* debug_host = nullptr;    // QSMD_SYNC_STAGES: giant-stage heartbeat (pinned)
    // lane mode's tables: one per lane slot of the memo grid
    // heavy stage (lane mode): workgroups at most (0 = 32 per CU, so a long
    // heavy list gets one workgroup per group of 64 histories and the
    // dispatcher starts each group as soon as a slot frees: config 3's heavy
    // stage alone 1.34 -> 1.09 ms against 12 per CU with grid-stride groups,
    // tools/gpu/r06_c3sweep.sh); one table each
    uint64_t memo_grid = 0;
    uint64_t mt_entries = 128;
    uint64_t memo_after = 32;          // lane mode: the memo joins a search after this many nodes
    // lane mode's tail: a search still running after tail_cap wavefront
    // iterations goes to a wave-mode launch after the heavy stage (one
    // wavefront per history, the state DAG from the root), when the last
    // call's heavy list had at least tail_min histories (a throughput-bound
    // list whose longest searches set the stage's end); 0 = never
    uint64_t tail_cap = 256;
    uint64_t tail_min = 65536;
    // the same long lists: the heavy stage forms its groups in order of
    // predicted work (stage 0's heavy_key, memo.hip heavy_sort); 0 = never
    uint64_t heavy_buckets = 1;
    // lane mode: stage 0's saved search states (80 B each), slots per heavy-
    // list shard: from the last call's heavy count (2x, at least 1024; an
    // eighth of the batch before the first call), or the knob resume_cap.  A
    // heavy history past its shard's slots starts again at the root, and a
    // buffer that cannot be had means no resume at all (the same results)
    char* rs = nullptr;
    size_t rs_bytes = 0;
    uint64_t resume_cap = 0;
    uint32_t memo_lds_entries = 64;             // LDS tables: entries per lane (power of two, 4..64)
    uint64_t memo_lds_cap = 0;                  // diagnostic: LDS-table bytes accepted at most (0 = the device's)
    char* mt = nullptr;
    size_t mt_bytes = 0;
    uint32_t mt_epoch = 0;
    // giant stage: exact-count memo (HBM, shared by the giants of a call)
    uint64_t split_xmemo = 1;
    char* xm = nullptr;
    size_t xm_bytes = 0;
    uint32_t xm_epoch = 0;
    // QSMD_FLAG_MEMO table (device), allocated on first use
    unsigned long long* memo = nullptr;
    uint64_t memo_entries = 1ull << 22;
    uint64_t memo_alloc = 0;
    uint32_t memo_epoch = 0;
    // split-search entry points: their own device buffers
    char* sx = nullptr;
    size_t sx_bytes = 0;
    uint8_t* wf_rank_host = nullptr;   // wellformed: pid rank table (pinned) and its device copy
    char* wf_rank_dev = nullptr;
    size_t wf_rank_bytes = 0;
};

namespace {

constexpr uint32_t kStage0wGrid = 1024;
constexpr size_t kZeroCopyBytes = 64 * 1024;   // host calls this small run on a mapped host buffer
constexpr uint64_t kTimingSlots = 1024;
constexpr uint64_t kSlotEvents = 5;      // stage 0 start / end, call end, heavy start / end
constexpr uint64_t kXMemoEntries = 1ull << 22;   // giant stage exact memo: 512 MB (shared by all giants of a call)
constexpr uint32_t kTaskCap = 1u << 19;  // tasks per variant per call (beyond: searched unsplit)
constexpr uint32_t kSplitTarget = 256;   // tasks wanted per giant history
constexpr uint32_t kSplitMaxTasks = 4096;
constexpr uint32_t kTaskGrid[SPLIT_VARIANTS] = {1024, 512};   // qsmd_check_tasks

int fail(qsmd_ctx* c, int code, const char* what, hipError_t e = hipSuccess) {
    if (c) {
        char buf[256];
        if (e != hipSuccess) std::snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
        else std::snprintf(buf, sizeof buf, "%s", what);
        c->err = buf;
    }
    return code;
}

// The context's own stream (host entry points, device calls given no
// stream), created on first use: a caller that always passes its streams
// (bench.py's calls in flight) leaves no idle stream sharing the device's
// hardware queues with the ones it uses.  A blocking stream: a caller that
// passes NULL (torch's default stream is handle 0) gets its calls ordered
// after the work it enqueued on the legacy default stream (a fill or copy of
// the inputs), as HIP orders any blocking stream with that one.
hipStream_t ctx_stream(qsmd_ctx* c) {
    if (!c->stream && hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess) {
        (void)hipGetLastError();
        c->stream = nullptr;
    }
    return c->stream;
}

// QSMD_SYNC_STAGES=1 (diagnostic): synchronise after every launch of the
// cascade and print its time and the counters to stderr.
static bool sync_stages() {
    static const bool on = [] {
        const char* e = std::getenv("QSMD_SYNC_STAGES");
        return e && e[0] == '1';
    }();
    return on;
}

#define HIP_TRY(c, expr, what)                                  \
    do {                                                        \
        hipError_t _e = (expr);                                 \
        if (_e != hipSuccess) return fail((c), QSMD_ERR_DEVICE, (what), _e); \
    } while (0)

size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// Wait until the context's previous call is done (its buffers may be in use):
// its completion event (a call on a caller's stream), or the context's own
// stream -- never the whole device, which would wait for other contexts,
// torch kernels and RCCL's streams too, and never a caller's stream, which
// the caller may destroy once its own work on it is done.
void quiesce(qsmd_ctx* c) {
    if (c->in_flight) {
        if (c->done_last) (void)hipEventSynchronize(c->done_ev);
        else (void)hipStreamSynchronize(c->last_stream);
        c->in_flight = false;
    }
}

// A call on stream s: the previous call of this context (on another
// stream) comes first -- its completion event, or a host wait for the
// context's own stream.
static hipError_t order_after_previous(qsmd_ctx* c, hipStream_t s) {
    if (!c->in_flight || (c->last_stream == s && !c->done_last)) return hipSuccess;
    if (c->done_last) return c->last_stream == s ? hipSuccess : hipStreamWaitEvent(s, c->done_ev, 0);
    const hipError_t e = hipStreamSynchronize(c->last_stream);
    if (e == hipSuccess) c->in_flight = false;
    return e;
}

// Grow a device buffer to at least `need` bytes (1.5x steps); the previous
// call of the context finishes before the old buffer is freed.  Returns
// whether it reallocated (the contents are then undefined).
int grow(qsmd_ctx* c, char** buf, size_t* cap, size_t need, bool* realloc_out = nullptr) {
    if (realloc_out) *realloc_out = false;
    if (*cap >= need) return QSMD_OK;
    const size_t old = *cap;
    if (*buf) {
        quiesce(c);
        (void)hipFree(*buf);
        *buf = nullptr;
        *cap = 0;
    }
    const size_t sz = std::max(need, old + old / 2);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(buf), sz);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(c, QSMD_ERR_NOMEM, "hipMalloc", e);
    }
    *cap = sz;
    if (realloc_out) *realloc_out = true;
    return QSMD_OK;
}

bool in_i32(int64_t v) { return v >= INT32_MIN && v <= INT32_MAX; }

void stage_done(const char* name, hipStream_t s, const uint32_t* cnt) {
    if (!sync_stages()) return;
    static auto t_prev = std::chrono::steady_clock::now();
    const hipError_t e = hipStreamSynchronize(s);
    uint32_t h[C_N] = {};
    (void)hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost);
    {   // stage 0's heavy list: its shard counters (internal.h)
        uint32_t sh[kShards * kShardStride];
        (void)hipMemcpy(sh, reinterpret_cast<const char*>(cnt) - kOffCnt + kOffShards, sizeof sh,
                        hipMemcpyDeviceToHost);
        for (uint32_t k = 0; k < kShards; ++k) {
            h[C_HEAVY32] += sh[k * kShardStride];
            h[C_DEFER] += sh[k * kShardStride + kDeferShardWord];
        }
    }
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[qsmd] %-8s %s %.3f ms  defer %u heavy %u/%u giants %u timed %u tasks %u/%u\n", name,
                 hipGetErrorString(e), std::chrono::duration<double, std::milli>(t - t_prev).count(), h[C_DEFER],
                 h[C_HEAVY32], h[C_HEAVY64], h[C_GIANT], h[C_TIMED], h[C_TASKS0], h[C_TASKS1]);
    t_prev = std::chrono::steady_clock::now();
}

int fill_model0(qsmd_ctx* c, uint32_t model_id, const void* model0, SearchArgs& a) {
    a.m0_exists = 0;
    a.m0_just = 0;
    a.m0_small = 1;
    a.m0_wave = 1;
    for (auto& v : a.m0_val) v = 0;
    if (!model0) return QSMD_OK;
    if (model_id == QSMD_MODEL_BANK) {
        const auto* m = static_cast<const qsmd_bank_model*>(model0);
        if (m->exists >> QSMD_BANK_MAX_ACCOUNTS) return fail(c, QSMD_ERR_ARG, "model0: account >= 8");
        for (int i = 0; i < QSMD_BANK_MAX_ACCOUNTS; ++i) {
            const bool ex = (m->exists >> i) & 1u;
            if (!in_i32(m->balance[i]) || (!ex && m->balance[i] != 0))
                return fail(c, QSMD_ERR_ARG, "model0: balance outside int32 or set on an absent account");
            a.m0_val[i] = m->balance[i];
        }
        a.m0_exists = m->exists;
    } else {
        const auto* m = static_cast<const qsmd_ticket_model*>(model0);
        if (m->is_just > 1 || !in_i32(m->n)) return fail(c, QSMD_ERR_ARG, "model0: bad Maybe Int");
        a.m0_just = m->is_just;
        a.m0_val[0] = m->is_just ? m->n : 0;
    }
    a.m0_wave = 1;
    for (int64_t v : a.m0_val) {
        if (v < -(1 << 18) || v >= (1 << 18)) a.m0_small = 0;   // compact stages hold 19-bit values
        if (v <= -(1 << 24) || v >= (1 << 24)) a.m0_wave = 0;   // wave mode's wide list: +-2^24
    }
    return QSMD_OK;
}

}  // namespace

extern "C" {

uint32_t qsmd_abi_version(void) { return QSMD_ABI_VERSION; }

const char* qsmd_last_error(const qsmd_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int qsmd_open(qsmd_ctx** out, int device) {
    if (!out) return QSMD_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return QSMD_ERR_DEVICE;
    if (device < 0 || device >= n) return QSMD_ERR_ARG;
    auto* c = new qsmd_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        return QSMD_ERR_DEVICE;
    }
    c->ev.resize(kSlotEvents * kTimingSlots, nullptr);
    c->ev_no0.assign(kTimingSlots, 0);
    for (auto& e : c->ev) {
        if (hipEventCreate(&e) != hipSuccess) { qsmd_close(c); return QSMD_ERR_DEVICE; }
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
    if (hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->probe_host), 64,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        qsmd_close(c);
        return QSMD_ERR_DEVICE;
    }
    std::memset(c->probe_host, 0, 64);
    *out = c;
    return QSMD_OK;
}

void qsmd_close(qsmd_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    quiesce(c);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->ws) (void)hipFree(c->ws);
    if (c->sx) (void)hipFree(c->sx);
    if (c->mt) (void)hipFree(c->mt);
    if (c->rs) (void)hipFree(c->rs);
    if (c->xm) (void)hipFree(c->xm);
    if (c->memo) (void)hipFree(c->memo);
    if (c->io) (void)hipFree(c->io);
    if (c->pin) (void)hipHostFree(c->pin);
    if (c->zc) (void)hipHostFree(c->zc);
    for (auto e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->done_ev) (void)hipEventDestroy(c->done_ev);
    if (c->probe_host) (void)hipHostFree(c->probe_host);
    if (c->wf_rank_host) (void)hipHostFree(c->wf_rank_host);
    if (c->wf_rank_dev) (void)hipFree(c->wf_rank_dev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

static constexpr uint64_t kAutoLo = 16, kAutoHi = 24;

// the stage-0 budget of this call: the set one, or (automatic) from the last
// finished call's probe -- at 16, back to 24 once more than 1 in 5 of its
// histories went on to the heavy stage; at 24, down to 16 while fewer than 1
// in 50 did (the gap between the two keeps a batch from alternating)
static uint64_t stage0_budget_of(const qsmd_ctx* c, const uint32_t* hint) {
    if (!c->s0_auto) return c->stage0_budget;
    if (!c->probe_valid) return kAutoHi;
    const uint64_t heavy = hint[1], n = hint[kProbeN], last = hint[kProbeBudget];
    if (!n) return last == kAutoLo ? kAutoLo : kAutoHi;
    if (last == kAutoLo) return heavy * 5 > n ? kAutoHi : kAutoLo;
    return heavy * 50 < n ? kAutoLo : kAutoHi;
}

int qsmd_set_stage0_budget(qsmd_ctx* c, uint64_t nodes) {
    if (!c) return QSMD_ERR_ARG;
    c->stage0_budget = nodes;
    c->s0_auto = false;
    return QSMD_OK;
}

int qsmd_set_param(qsmd_ctx* c, const char* name, uint64_t value) {
    if (!c || !name) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const std::string n(name);
    if (n == "stage0_budget") {
        c->stage0_budget = value;
        c->s0_auto = false;
    } else if (n == "stage0_budget_auto") {
        if (value > 1) return fail(c, QSMD_ERR_ARG, "stage0_budget_auto: 0 or 1");
        c->s0_auto = value != 0;
    } else if (n == "stage0w_budget") {
        c->stage0w_budget = value;
        c->s0w_auto = false;
    } else if (n == "stage0w_budget_auto") {
        if (value > 1) return fail(c, QSMD_ERR_ARG, "stage0w_budget_auto: 0 or 1");
        c->s0w_auto = value != 0;
    } else if (n == "stage0_grid") {
        if (value == 0 || value > 0x7FFFFFFFull) return fail(c, QSMD_ERR_ARG, "bad grid");
        c->stage0_max_grid = value;
    } else if (n == "split_budget") {
        c->split_budget = value;
    } else if (n == "split_xmemo") {
        c->split_xmemo = value ? 1 : 0;
    } else if (n == "wave_grid") {
        if (value > 65536) return fail(c, QSMD_ERR_ARG, "wave_grid in 0..65536");
        c->wave_grid = value;
    } else if (n == "giant_grid") {
        if (value > 65536) return fail(c, QSMD_ERR_ARG, "giant_grid in 0..65536");
        c->giant_grid = value;
    } else if (n == "giant_stall_us") {     // diagnostic (tests of the phase-wait safety net)
        if (value > 10000000ull) return fail(c, QSMD_ERR_ARG, "giant_stall_us in 0..10^7");
        c->giant_stall_us = value;
    } else if (n == "dag_states") {
        if (value > 4095) return fail(c, QSMD_ERR_ARG, "dag_states in 0..4095 (0 = the DFS only)");
        c->dag_states = value;
    } else if (n == "dag_debug_ptr") {      // diagnostic: device buffer (16 + DAG LDS words) for one history
        c->dag_dbg = reinterpret_cast<uint32_t*>(value);
    } else if (n == "stage0_stamps_ptr") {  // diagnostic build (tools/diag/compact_diag.patch, QSMD_DIAG_STAGE0=2): 8 x u64 per workgroup
        c->s0_stamps = reinterpret_cast<unsigned long long*>(value);
    } else if (n == "dag_debug_hist") {
        c->dag_dbg_h = value;
    } else if (n == "wave_min_rem") {
        c->wave_min_rem = std::min<uint64_t>(value, 0xFFFFFFFFull);
    } else if (n == "wave_stats_ptr") {     // diagnostic: device buffer of 16 x u64 (zeroed by the caller)
        c->wave_stats = reinterpret_cast<unsigned long long*>(value);
    } else if (n == "memo_stats_ptr") {     // diagnostic: device buffer of 16 x u64 per heavy-stage group (zeroed)
        c->memo_stats = reinterpret_cast<unsigned long long*>(value);
    } else if (n == "memo_stats_groups") {
        c->memo_stats_groups = value;
    } else if (n == "memo_lds_entries") {
        if (value < 4 || value > 64 || (value & (value - 1)))
            return fail(c, QSMD_ERR_ARG, "memo_lds_entries: a power of two in 4..64");
        c->memo_lds_entries = (uint32_t)value;
    } else if (n == "timing_events") {     // 0: no per-call timing events (qsmd_timing_read / last_kernel_ms)
        if (value > 1) return fail(c, QSMD_ERR_ARG, "timing_events: 0 or 1");
        c->timing = value != 0;
    } else if (n == "memo_after") {
        c->memo_after = value;
    } else if (n == "tail_cap") {
        c->tail_cap = value;
    } else if (n == "tail_min") {
        c->tail_min = value;
    } else if (n == "heavy_buckets") {
        if (value > 1) return fail(c, QSMD_ERR_ARG, "heavy_buckets: 0 or 1");
        c->heavy_buckets = value;
    } else if (n == "memo_lds_cap") {       // diagnostic: force the LDS-refused path (the HBM tables)
        c->memo_lds_cap = value;
    } else if (n == "memo_lds") {
        if (value > 2) return fail(c, QSMD_ERR_ARG, "memo_lds: 0 = HBM tables, 1 = LDS for short lists, 2 = LDS");
        c->memo_lds = (uint32_t)value;
    } else if (n == "resume_cap") {          // lane mode: saved-state slots per heavy-list shard (0 = auto)
        c->resume_cap = value;
    } else if (n == "fold") {
        if (value > 1) return fail(c, QSMD_ERR_ARG, "fold: 0 or 1");
        c->fold = value;
    } else if (n == "heavy_mode") {
        if (value > 2) return fail(c, QSMD_ERR_ARG, "heavy_mode: 0 = wave, 1 = lane, 2 = auto");
        c->heavy_mode = value;
    } else if (n == "wave_max") {
        c->wave_max = value;
    } else if (n == "memo_grid") {
        if (value > 65536) return fail(c, QSMD_ERR_ARG, "memo_grid in 0..65536 (0 = 32 per CU)");
        if (value != c->memo_grid && c->mt) {
            quiesce(c);
            (void)hipFree(c->mt);
            c->mt = nullptr;
            c->mt_bytes = 0;
        }
        c->memo_grid = value;
    } else if (n == "memo_lane_entries") {
        if (value < 2 || value > 65536 || (value & (value - 1)))
            return fail(c, QSMD_ERR_ARG, "memo_lane_entries: a power of two in 2..65536");
        if (value != c->mt_entries && c->mt) {
            quiesce(c);
            (void)hipFree(c->mt);
            c->mt = nullptr;
            c->mt_bytes = 0;
        }
        c->mt_entries = value;
    } else {
        return fail(c, QSMD_ERR_ARG, "unknown parameter");
    }
    return QSMD_OK;
}

int qsmd_set_split_budget(qsmd_ctx* c, uint64_t nodes) {
    if (!c) return QSMD_ERR_ARG;
    c->split_budget = nodes;
    return QSMD_OK;
}

int qsmd_set_memo_capacity(qsmd_ctx* c, uint64_t entries) {
    if (!c || entries < 1024 || (entries & (entries - 1)) || entries > (1ull << 32)) return QSMD_ERR_ARG;
    c->memo_entries = entries;
    return QSMD_OK;
}

int qsmd_set_stage0_grid(qsmd_ctx* c, uint64_t max_blocks) {
    if (!c || max_blocks == 0 || max_blocks > 0x7FFFFFFFull) return QSMD_ERR_ARG;
    c->stage0_max_grid = max_blocks;
    return QSMD_OK;
}

int qsmd_set_time_limit_ms(qsmd_ctx* c, uint64_t ms) {
    if (!c) return QSMD_ERR_ARG;
    c->time_limit_ms = ms;
    return QSMD_OK;
}

// The QSMD_FLAG_MEMO table and this call's epoch (entries are only valid
// within one call: an entry of another epoch counts as empty, so the table is
// cleared when allocated and when the 24-bit epochs wrap, not per call).
static int memo_prepare(qsmd_ctx* c, hipStream_t s, unsigned long long** out, uint32_t* epoch) {
    if (c->memo_alloc != c->memo_entries) {
        if (c->memo) {
            quiesce(c);
            (void)hipStreamSynchronize(s);
            (void)hipFree(c->memo);
            c->memo = nullptr;
            c->memo_alloc = 0;
        }
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&c->memo), c->memo_entries * 64);
        if (e != hipSuccess) return fail(c, QSMD_ERR_NOMEM, "hipMalloc memo table", e);
        c->memo_alloc = c->memo_entries;
        HIP_TRY(c, hipMemsetAsync(c->memo, 0, c->memo_alloc * 64, s), "memset memo table");
    }
    if (((++c->memo_epoch) & 0xFFFFFFu) == 0u) {   // 24-bit tags wrapped: clear
        HIP_TRY(c, hipMemsetAsync(c->memo, 0, c->memo_alloc * 64, s), "memset memo table");
        ++c->memo_epoch;
    }
    *out = c->memo;
    *epoch = c->memo_epoch;
    return QSMD_OK;
}

// A tail stage's grid: one workgroup per 64 histories the last call sent
// there, between `floor` and `cap` (cap before the first call).
static uint64_t tail_grid(uint64_t floor, uint64_t cap, uint64_t last) {
    if (last == 0xFFFFFFFFull || last > 0xFFFFFFFFull) return cap;
    return std::min<uint64_t>(cap, std::max<uint64_t>(floor, (last + 63) / 64));
}

// Lane mode's HBM memo tables for a heavy-stage grid of `grid` workgroups
// (one private table per lane slot: grid x 64 x entries x (32 + 64) B),
// grown on demand and cleared once when (re)allocated -- entries are tagged
// by call epoch, never cleared per call.  False when the device cannot hold
// them: the call then runs the heavy stage in wave mode (the same results).
static bool lane_tables(qsmd_ctx* c, hipStream_t s, uint64_t grid) {
    const size_t need = (size_t)grid * 64 * c->mt_entries * (32 + 64);
    if (c->mt_bytes >= need) return true;
    bool re = false;
    // (with headroom: the grid follows the last call's heavy count, and a
    // stream of distinct batches moves it a little every call -- sized to
    // the count alone, the tables grew, were cleared and waited for the
    // context's last call in the middle of a caller's stream of calls:
    // 4.8 vs 8.8e9 histories/s over five resident batches, tools/gpu/archive/r05_rot2.sh)
    if (grow(c, &c->mt, &c->mt_bytes, need + need / 2, &re) != QSMD_OK &&
        grow(c, &c->mt, &c->mt_bytes, need, &re) != QSMD_OK) {
        (void)hipGetLastError();
        return false;
    }
    if (hipMemsetAsync(c->mt, 0, c->mt_bytes, s) != hipSuccess) {
        (void)hipFree(c->mt);
        c->mt = nullptr;
        c->mt_bytes = 0;
        return false;
    }
    return true;
}

// QSMD_SYNC_STAGES=1 (diagnostic): the giant stage's per-workgroup phase
// records (pinned, mapped) and a heartbeat on stderr while it runs
static uint32_t* giant_debug_buffer(qsmd_ctx* c, uint64_t gg) {
    if (!c->debug_host)
        (void)hipHostMalloc(reinterpret_cast<void**>(&c->debug_host), 65536 * 16,
                            hipHostMallocMapped | hipHostMallocCoherent);
    if (c->debug_host) std::memset(c->debug_host, 0, gg * 16);
    return c->debug_host;
}

static void giant_heartbeat(qsmd_ctx* c, hipStream_t s, uint64_t gg) {
    if (!c->debug_host) return;
    for (int it = 0; hipStreamQuery(s) == hipErrorNotReady && it <= 150; ++it) {
        usleep(200000);
        uint32_t hist[8] = {};
        uint64_t took = 0;
        for (uint64_t b = 0; b < gg; ++b) {
            const uint32_t ph = c->debug_host[b * 4];
            hist[ph < 8 ? ph : 7]++;
            took += c->debug_host[b * 4 + 2];
        }
        std::fprintf(stderr, "[qsmd] giants t=%.1fs phases 0:%u 1:%u 2:%u 3:%u 4:%u 5:%u 6:%u took %llu\n",
                     0.2 * (it + 1), hist[0], hist[1], hist[2], hist[3], hist[4], hist[5], hist[6],
                     (unsigned long long)took);
    }
}

// route (known only to the host entry, which sees the headers): kSkip0 = no
// history fits stage 0, kSkip0w = none fits stage 0w either (every history
// goes straight to the wide list: one wave-mode launch and the giant stage)
enum : uint32_t { kSkip0 = 1u, kSkip0w = 2u };

// wave mode's launch arguments but the lists, the LDS table size and the
// M128 launch (the heavy stage's wave mode and lane mode's tail launch)
static WaveArgs wave_args(const qsmd_ctx* c, const SearchArgs& a, uint32_t flags, uint64_t cap, bool split) {
    WaveArgs wp{};
    wp.s = a;
    wp.explore_cap = cap;
    wp.explore_cap_wide = split ? 16 * c->split_budget : 0;   // (the giant stage's whole-search cap)
    wp.stats = c->wave_stats;
    wp.memo_min_rem = (uint32_t)c->wave_min_rem;
    wp.dag_states = (uint32_t)(c->dag_states & ~1ull);   // (even: the DAG's LDS arrays stay 8-B aligned)
    wp.dag_items = 4u * wp.dag_states;
    wp.dbg = c->dag_dbg;
    wp.dbg_h = (uint32_t)c->dag_dbg_h;
    wp.memo_mode = (flags & QSMD_FLAG_MEMO) ? 1u : 0u;
    return wp;
}

static int check_device_locked(qsmd_ctx* c, uint32_t model_id, const qsmd_hdr* hdr, uint64_t n_hist,
                               const qsmd_event* events, uint64_t n_events, const void* model0,
                               uint32_t flags, uint64_t max_nodes, uint8_t* status, uint64_t* nodes,
                               uint8_t* witness, qsmd_totals* totals, hipStream_t s, uint32_t route = 0u) {
    if (model_id != QSMD_MODEL_BANK && model_id != QSMD_MODEL_TICKET)
        return fail(c, QSMD_ERR_ARG, "unknown model_id");
    if (n_hist && (!hdr || !status)) return fail(c, QSMD_ERR_ARG, "null hdr/status");
    if (n_hist > 0xFFFFFFFFull) return fail(c, QSMD_ERR_ARG, "n_hist > 2^32-1");
    const bool early = (flags & QSMD_FLAG_EARLY_EXIT_BATCH) != 0;
    SearchArgs a{};
    int rc = fill_model0(c, model_id, model0, a);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");

    // the previous call of this context may run on another stream
    HIP_TRY(c, order_after_previous(c, s), "order after the previous call");
    // the tail launches' grids from the last finished call's list sizes (a
    // hint: every tail kernel is grid-stride, any grid gives the same
    // results); none before a call has finished (the giant stage's last
    // block sets the probe's written flag)
    if (!c->probe_valid && c->any_call && __atomic_load_n(&c->probe_host[kProbeWritten], __ATOMIC_ACQUIRE))
        c->probe_valid = true;
    uint32_t hint[kProbeSlots];
    for (int i = 0; i < kProbeSlots; ++i) hint[i] = c->probe_valid ? c->probe_host[i] : 0xFFFFFFFFu;
    const uint64_t budget0 = stage0_budget_of(c, hint);
    // the automatic budget just went down: the last call's heavy count (at
    // the higher budget) undercounts this one's -- size the tail for a long
    // list (a caller that runs ahead enqueues many calls on that stale hint)
    if (c->s0_auto && c->probe_valid && budget0 < hint[kProbeBudget])
        hint[1] = std::max<uint32_t>(hint[1], (uint32_t)std::min<uint64_t>(n_hist / 4, 0xFFFFFFFEull));
    // heavy-stage mode: lane mode (64 searches per wavefront instruction) for
    // a long heavy list, wave mode (one search per wavefront, its DFS chain
    // ~10x shorter) for a short one -- by the last finished call's count;
    // and lane mode for a list of short searches of any length: one where
    // under a fifth of the batch went on (configs 1, 2, 5's shape; one call
    // at a time lane mode took config 2 on 300 / 2k / 100k / 1M histories at
    // budget 20 in 0.049 / 0.070 / 0.100 / 0.195 ms against wave mode's
    // 0.092 / 0.094 / 0.113 / 0.485, config 1 6.9 vs 5.7e9), not a
    // bug-laden batch's (config 3 on 10k: wave mode 0.128 against 0.48 ms --
    // the longest of a few thousand long searches), nor one with wide
    // histories (lane mode hands those to the giant stage);
    // profiles/r06/wavemax/
    const uint64_t heavy_hint = c->probe_valid ? (uint64_t)hint[1] + hint[2] : 0ull;
    const bool short_searches = c->probe_valid && heavy_hint > 0 && 5ull * heavy_hint < hint[kProbeN] &&
                                hint[kProbeWide] == 0u;
    if (c->heavy_mode == 1) route &= ~kSkip0w;   // (lane mode forced: the wide list goes on to the giant stage)
    bool lane = !(route & kSkip0w) &&
                (c->heavy_mode == 1 || (c->heavy_mode == 2 && (heavy_hint > c->wave_max || short_searches)));
    // lane mode's memo tables in LDS (one wavefront per CU) when the last
    // call's heavy groups fit the CUs, else in HBM (one table per lane slot)
    const bool wide = hint[2] != 0u;   // G64 groups in the launch only when the last call had some
    const uint64_t g32 = c->probe_valid ? ((uint64_t)hint[1] + 63u) / 64u : ~0ull;
    bool lt = c->memo_lds == 2 || (c->memo_lds == 1 && g32 <= (uint64_t)c->n_cu);
    // (an LDS size the device refuses: the HBM tables, allocated below)
    const uint32_t lds_entries = (uint32_t)std::min<uint64_t>(c->memo_lds_entries, c->mt_entries);
    if (lane && lt && !wide && !memo_lds_accepted(model_id, lds_entries, c->memo_lds_cap)) lt = false;
    // (LDS tables: one workgroup per CU, so no idle workgroups beyond
    // twice the groups expected -- they would hold CUs the next call's
    // stage 0 could use)
    const uint64_t mg = lt && !wide ? std::min<uint64_t>(c->n_cu, 2 * std::min<uint64_t>(g32, c->n_cu) + 8)
                                    : (c->probe_valid ? tail_grid(8, c->memo_grid ? c->memo_grid : 32ull * c->n_cu,
                                                                  heavy_hint + heavy_hint / 4)
                                                      : (uint64_t)c->n_cu);   // (no hint: grid-stride)
    if (lane && !(lt && !wide)) lane = lane_tables(c, s, mg);
    // the folded tail (lane mode, ctx.fold): the last call deferred nothing
    // to stage 0w and this one has a normal route -- no stage-0w launch
    const bool fold = lane && c->fold && c->probe_valid && route == 0u && !sync_stages() &&
                      hint[0] == 0u && hint[2] == 0u;
    // lane mode's wave-mode tail launch (ctx.tail_cap): for a long heavy list
    // (a list of at least tail_min and a fifth of the last batch: config 3's
    // ~33 %, not config 2's 1.6 % at budget 20 or 9.6 % at the automatic 16,
    // whose longest searches end before tail_cap -- the tail launch alone
    // costs a lone call ~5 us, profiles/r06/inflight1.txt; tail_min 0: any list)
    const bool long_list = c->probe_valid && (c->tail_min == 0 || (heavy_hint >= c->tail_min &&
                                                                   5ull * heavy_hint >= hint[kProbeN]));
    const bool tail = lane && c->tail_cap && long_list && c->dag_states;
    // ... and its heavy list in order of predicted work
    const bool buckets = lane && c->heavy_buckets && long_list && !(route & kSkip0);

    // ---- workspace: header, lists, giant records, tasks
    const bool want_w = (flags & QSMD_FLAG_WITNESS) && witness;
    const uint64_t n_tk = (uint64_t)SPLIT_VARIANTS * kTaskCap;
    const size_t lst = align_up(n_hist * 4 + 4);
    const size_t off_l0 = kWsHeader;                     // stage 0 -> stage 0w
    const uint64_t cap32 = shard_cap(n_hist);            // stage 0's heavy and deferred lists: kShards shards (internal.h)
    const size_t off_h32 = off_l0 + align_up(kShards * cap32 * 4 + 4);   // heavy lists
    const size_t off_h64 = off_h32 + align_up(kShards * cap32 * 4 + 4);
    const size_t off_lw = off_h64 + lst;                 // stage 0w's deferred (wide) histories
    const size_t off_lg = off_lw + lst;                  // giants
    const size_t off_lt = off_lg + lst;                  // lane mode -> the wave-mode tail launch
    const size_t off_ko = off_lt + lst;                  // heavy_sort: keys (u8 per heavy-list slot), order
    const size_t off_gr = off_ko + (buckets ? align_up(kShards * cap32) + lst : 0);
    const size_t off_tk = off_gr + align_up(n_hist * sizeof(GiantRec));
    const size_t off_ts = off_tk + align_up(n_tk * sizeof(qsmd_task));
    const size_t off_tn = off_ts + align_up(n_tk);
    const size_t off_tw = off_tn + align_up(n_tk * 8);
    const size_t off_nd = off_tw + (want_w ? align_up(n_tk * kTaskWitness) : 0);   // nodes if the caller has none
    const size_t off_tot = off_nd + (early && !nodes ? align_up(n_hist * 8) : 0);
    const size_t need = off_tot + align_up(sizeof(qsmd_totals));
    bool re = false;
    rc = grow(c, &c->ws, &c->ws_bytes, need, &re);
    if (rc) return rc;
    if (re || c->ws_dirty) {   // counters 0 (first failing history: none), buckets 0
        HIP_TRY(c, hipMemsetAsync(c->ws, 0, kWsHeader, s), "memset header");
        HIP_TRY(c, hipMemsetAsync(c->ws + kOffCnt + 4 * C_FIRST_FAIL, 0xFF, 4, s), "memset header");
    }
    uint32_t* cnt = reinterpret_cast<uint32_t*>(c->ws + kOffCnt);
    qsmd_totals* tot = totals ? totals : reinterpret_cast<qsmd_totals*>(c->ws + off_tot);
    uint32_t* l0 = reinterpret_cast<uint32_t*>(c->ws + off_l0);
    uint32_t* h32 = reinterpret_cast<uint32_t*>(c->ws + off_h32);
    uint32_t* shards = reinterpret_cast<uint32_t*>(c->ws + kOffShards);
    // stage 0's saved states (lane mode): their own buffer, slots per shard capped
    uint64_t rs_cap = 0;
    uint32_t* states = nullptr;
    if (lane) {
        rs_cap = c->resume_cap ? c->resume_cap
                               : (c->probe_valid ? std::max<uint64_t>(1024, 2ull * hint[1] / kShards) : cap32 / 8);
        rs_cap = std::min<uint64_t>(std::max<uint64_t>(rs_cap, 1), cap32);
        const size_t rs_need = (size_t)kShards * rs_cap * kResumeWords * 4;
        if (c->rs_bytes >= rs_need || grow(c, &c->rs, &c->rs_bytes, rs_need + rs_need / 2) == QSMD_OK ||
            grow(c, &c->rs, &c->rs_bytes, rs_need) == QSMD_OK) {   // (headroom: see lane_tables)
            states = reinterpret_cast<uint32_t*>(c->rs);
        } else {
            (void)hipGetLastError();
            c->err.clear();
        }
    }
    uint32_t* h64 = reinterpret_cast<uint32_t*>(c->ws + off_h64);
    uint32_t* lw = reinterpret_cast<uint32_t*>(c->ws + off_lw);
    uint32_t* lg = reinterpret_cast<uint32_t*>(c->ws + off_lg);
    uint32_t* lt_list = reinterpret_cast<uint32_t*>(c->ws + off_lt);
    uint8_t* hkey = buckets ? reinterpret_cast<uint8_t*>(c->ws + off_ko) : nullptr;
    uint32_t* horder = buckets ? reinterpret_cast<uint32_t*>(c->ws + off_ko + align_up(kShards * cap32)) : nullptr;
    if (early && !nodes) nodes = reinterpret_cast<uint64_t*>(c->ws + off_nd);

    a.hdr = hdr;
    a.events = reinterpret_cast<const uint2*>(events);
    a.n_hist = n_hist;
    a.n_events = n_events;
    a.flags = flags;
    a.model_id = model_id;
    a.max_nodes = max_nodes;
    a.time_limit = c->time_limit_ms * 100000ull;   // 100 MHz s_memrealtime
    a.status = status;
    a.nodes = nodes;
    a.witness = (flags & QSMD_FLAG_WITNESS) ? witness : nullptr;
    a.buckets = reinterpret_cast<unsigned long long*>(c->ws + kOffBuckets);
    a.timed_out = cnt + C_TIMED;
    a.first_fail = early ? cnt + C_FIRST_FAIL : nullptr;
    a.giant_list = lg;
    a.giant_count = cnt + C_GIANT;
    const bool split = c->split_budget && (!max_nodes || c->split_budget < max_nodes);

    // ---- the giant stage's arguments: the split search, the combine, (the
    // fixup), the totals
    SplitArgs p{};
    p.s = a;
    p.cnt = cnt;
    p.shards = shards;
    p.giant_list = lg;
    p.giant_count = cnt + C_GIANT;
    p.giants = reinterpret_cast<GiantRec*>(c->ws + off_gr);
    p.tasks = reinterpret_cast<qsmd_task*>(c->ws + off_tk);
    p.task_cap = kTaskCap;
    p.target = split ? kSplitTarget : 0u;
    p.max_tasks = kSplitMaxTasks;
    p.max_depth = QSMD_SPLIT_MAX_DEPTH;
    p.whole_cap = split ? 16 * c->split_budget : 0;
    p.task_status = reinterpret_cast<uint8_t*>(c->ws + off_ts);
    p.task_nodes = reinterpret_cast<uint64_t*>(c->ws + off_tn);
    p.task_witness = want_w ? reinterpret_cast<uint8_t*>(c->ws + off_tw) : nullptr;
    p.early = early ? 1u : 0u;
    p.totals = tot;
    p.probe_host = c->probe_host;
    // the budget stage 0 runs with (a0.stage0_budget below: capped below
    // 2^31), 0xFFFFFFFF when it has none (budget 0: stage 0 searches every
    // history to its end) -- qsmd_get_param("stage0_budget_last")
    p.probe_budget = budget0 ? (uint32_t)std::min<uint64_t>(budget0, 0x7FFFFFFFull) : 0xFFFFFFFFu;
    p.stall_ticks = c->giant_stall_us * 100ull;   // 100 MHz s_memrealtime
    if (flags & QSMD_FLAG_MEMO) {
        rc = memo_prepare(c, s, &p.memo, &p.memo_epoch);
        if (rc) return rc;
        p.memo_mask = c->memo_alloc - 1;
    } else if (c->split_xmemo) {        // exact-count memo for the giants (the reference's counts)
        const size_t xneed = (size_t)kXMemoEntries * 128;
        if (c->xm_bytes < xneed) {
            rc = grow(c, &c->xm, &c->xm_bytes, xneed);
            if (rc) return rc;
            HIP_TRY(c, hipMemsetAsync(c->xm, 0, c->xm_bytes, s), "memset exact memo");
        }
        if (((++c->xm_epoch) & 0xFFFFFFu) == 0u) {   // 24-bit tags wrapped: clear
            HIP_TRY(c, hipMemsetAsync(c->xm, 0, c->xm_bytes, s), "memset exact memo");
            ++c->xm_epoch;
        }
        p.memo = reinterpret_cast<unsigned long long*>(c->xm);
        p.memo_mask = kXMemoEntries - 1;
        p.memo_exact = 1;
        p.memo_epoch = c->xm_epoch;
    }
    c->ws_dirty = true;                 // until the giant stage is enqueued
    hipEvent_t* evs = &c->ev[kSlotEvents * (c->n_calls % kTimingSlots)];
    const bool tm = c->timing;
    // ---- stage 0: every history, <= 32 events
    SearchArgs a0 = a;
    a0.list = nullptr;
    a0.list_count = nullptr;
    a0.defer_list = l0;
    a0.defer_count = shards + kDeferShardWord;
    a0.defer_shard_cap = (uint32_t)cap32;
    a0.heavy_list = h32;
    a0.heavy_count = shards;
    a0.heavy_shard_cap = (uint32_t)cap32;
    a0.heavy_state = states;                 // (lane mode goes on from them)
    a0.heavy_state_cap = (uint32_t)rs_cap;
    a0.heavy_key = hkey;
    // (below 2^31: a saved state keeps its node count in 32 bits)
    a0.stage0_budget = budget0 ? std::min<uint64_t>(budget0, 0x7FFFFFFFull) : ~0ull;
    a0.stamps = c->s0_stamps;
    const uint64_t n_groups = std::max<uint64_t>((n_hist + 63) / 64, 1);
    stage_done("start", s, cnt);
    if (!(route & kSkip0)) {           // (the events at the kernel's start and end)
        HIP_TRY(c, launch_compact(a0, (uint32_t)std::min<uint64_t>(n_groups, c->stage0_max_grid), s,
                                  tm ? evs[0] : nullptr, tm ? evs[1] : nullptr),
                "stage 0 launch");
    } else if (tm) {                   // (no stage-0 end event: one packet less before the first kernel)
        HIP_TRY(c, hipEventRecord(evs[0], s), "hipEventRecord");
    }
    if (tm) c->ev_no0[c->n_calls % kTimingSlots] = ((route & kSkip0) ? 1u : 0u) | (lane ? 0u : 2u);
    stage_done("stage0", s, cnt);
    // ---- stage 0w: the rest, <= 64 events (beyond: the giant stage)
    SearchArgs aw = a;
    aw.list = (route & kSkip0) ? nullptr : l0;               // (null: every history of the batch)
    aw.list_count = (route & kSkip0) ? nullptr : shards + kDeferShardWord;
    aw.list_shard_cap = (route & kSkip0) ? 0u : (uint32_t)cap32;
    aw.defer_list = lw;                      // (wave mode searches most of them; the rest: giants)
    aw.defer_count = cnt + C_WIDE;
    aw.heavy_list = h64;
    aw.heavy_count = cnt + C_HEAVY64;
    const uint64_t budget0w = c->s0w_auto ? (lane ? 24u : 48u) : c->stage0w_budget;
    aw.stage0_budget = budget0w ? budget0w : ~0ull;
    if (!(route & kSkip0w) && !fold)
        HIP_TRY(c, launch_compact64(aw, (uint32_t)((route & kSkip0) ? std::min<uint64_t>(n_groups, kStage0wGrid)
                                                                    : (hint[0] == 0u ? 8u   // (last call: none)
                                                                                     : tail_grid(2ull * c->n_cu, kStage0wGrid,
                                                                                                 hint[0]))),
                                    s), "stage 0w launch");
    stage_done("stage0w", s, cnt);
    // ---- heavy stage: histories over the stage budgets
    const uint64_t cap = split ? 64 * c->split_budget : 0;
    if (lane) {
        if (((++c->mt_epoch) & 0xFFFFFFu) == 0u && c->mt) {   // 24-bit tags wrapped: clear
            HIP_TRY(c, hipMemsetAsync(c->mt, 0, c->mt_bytes, s), "memset memo tables");
            ++c->mt_epoch;
        }
        const uint64_t slots = mg * 64 * c->mt_entries;
        MemoArgs mp[2]{};
        for (int w = 0; w < 2; ++w) {
            mp[w].s = a;
            // (folded: no stage 0w ran, G64 groups are stage 0's deferred histories)
            mp[w].s.list = w ? (fold ? l0 : h64) : h32;
            mp[w].s.list_count = w ? (fold ? shards + kDeferShardWord : cnt + C_HEAVY64) : shards;
            mp[w].s.list_shard_cap = w && !fold ? 0u : (uint32_t)cap32;
            mp[w].table = reinterpret_cast<uint32_t*>(c->mt + (w ? slots * 32 : 0));
            mp[w].entries = (uint32_t)c->mt_entries;
            mp[w].memo_after = (uint32_t)std::min<uint64_t>(c->memo_after, 0xFFFFFFFFull);
            mp[w].resume = w ? nullptr : states;
            mp[w].resume_cap = (uint32_t)rs_cap;
            mp[w].lds_entries = lds_entries;
            mp[w].epoch = c->mt_epoch;
            mp[w].giant_cap = cap;
            mp[w].order = w ? nullptr : horder;
            mp[w].tail_cap = tail ? c->tail_cap : 0u;
            mp[w].tail_list = tail ? lt_list : nullptr;
            mp[w].tail_count = cnt + C_TAIL;
            mp[w].stats = c->memo_stats;
            mp[w].stats_groups = c->memo_stats ? c->memo_stats_groups : 0;
            mp[w].fwd_list = lw;                 // stage 0w's deferred histories: on to the giant stage
            mp[w].fwd_count = cnt + C_WIDE;
        }
        if (buckets) {   // (workgroups per shard for the last call's count; grid-stride beyond)
            const uint64_t per = ((uint64_t)hint[1] / kShards + kSortChunkHost - 1) / kSortChunkHost;
            HIP_TRY(c, launch_heavy_sort(shards, (uint32_t)cap32, hkey, cnt, horder,
                                         (uint32_t)std::min<uint64_t>(std::max<uint64_t>(per, 1), 64), s),
                    "heavy sort launch");
        }
        HIP_TRY(c, launch_memo(mp[0], mp[1], (uint32_t)mg, wide, lt, s, tm ? evs[3] : nullptr,
                               tm ? evs[4] : nullptr), "memo launch");
        stage_done("lane", s, cnt);
        if (tail) {
            // the tail: the lane-mode searches past tail_cap, one wavefront
            // each (the list as wave mode's G32 list; the others empty)
            WaveArgs wt = wave_args(c, a, flags, cap, split);
            wt.list32 = lt_list;
            wt.count32 = cnt + C_TAIL;
            wt.cap32 = 0u;
            wt.list64 = lt_list;
            wt.count64 = cnt + C_ZERO;
            wt.list_wide = lt_list;
            wt.count_wide = cnt + C_ZERO;
            wt.buckets = 32u;
            wt.wide128 = 0u;
            const uint64_t nt = hint[kProbeTail] == 0xFFFFFFFFu ? 4ull * c->n_cu : hint[kProbeTail];
            const uint64_t gt = c->wave_grid ? c->wave_grid
                                             : std::min<uint64_t>(16ull * c->n_cu, std::max<uint64_t>(64, nt + nt / 4));
            HIP_TRY(c, launch_wave(wt, (uint32_t)gt, 0u, s), "tail launch");
            stage_done("tail", s, cnt);
        }
    } else {
        WaveArgs wp = wave_args(c, a, flags, cap, split);
        wp.list32 = h32;
        wp.count32 = shards;
        wp.cap32 = (uint32_t)cap32;
        wp.list64 = h64;
        wp.count64 = cnt + C_HEAVY64;
        wp.list_wide = (route & kSkip0w) ? nullptr : lw;
        wp.count_wide = cnt + C_WIDE;
        // LDS memo table: 8 KB per wavefront (256 entries of <= 64 events),
        // 64 KB when the last call had wide histories (1024 entries of <= 128)
        const uint64_t wide_hint = (route & kSkip0w) ? n_hist : (c->probe_valid ? (uint64_t)hint[kProbeWide] : 0ull);
        wp.buckets = wide_hint ? 256u : 32u;
        // one workgroup per history the last call sent here (+ 25 %), at
        // least 64 and at most 16 per CU (grid-stride beyond)
        // the 65..128-event launch when the last call had wide histories
        wp.wide128 = wide_hint ? 1u : 0u;
        const uint64_t nh = heavy_hint + wide_hint;
        const uint64_t g = c->wave_grid ? c->wave_grid
                         : std::min<uint64_t>(16ull * c->n_cu,
                                              c->probe_valid ? std::max<uint64_t>(64, nh + nh / 4) : 4ull * c->n_cu);
        const uint64_t g128 = std::min<uint64_t>(16ull * c->n_cu, std::max<uint64_t>(8, wide_hint + wide_hint / 4));
        HIP_TRY(c, launch_wave(wp, (route & kSkip0w) ? 0u : (uint32_t)g, (uint32_t)g128, s), "wave launch");
        stage_done("wave", s, cnt);
    }
    {
        // (2 per CU when the last call had giants, or when folded: stage 0's
        // deferred histories, however many this call has, go straight to the
        // giant stage -- the short path of a call without giants costs the
        // same on 64 or 512 workgroups, profiles/r06/c3c4/giant_grid_split_budget.txt; an
        // early exit without them: one workgroup per fixup chunk, at least 8
        // and at most 2 per CU -- every workgroup of the launch takes the
        // fixup's queue and exit atomics, 2 per CU made a 4096-history call's
        // giant stage ~65 us)
        const uint64_t gg = c->giant_grid ? c->giant_grid
                          : (hint[3] || (fold && !early) ? 2ull * c->n_cu
                                     : (early ? std::min<uint64_t>(2ull * c->n_cu,
                                                                   std::max<uint64_t>(8, (n_hist + kFixupChunk - 1) / kFixupChunk))
                                              : 64ull));
        if (sync_stages()) p.debug = giant_debug_buffer(c, gg);
        HIP_TRY(c, launch_giants(p, (uint32_t)gg, s), "giant launch");
        if (sync_stages()) giant_heartbeat(c, s, gg);
    }
    stage_done("giants", s, cnt);
    c->ws_dirty = false;
    if (tm) HIP_TRY(c, hipEventRecord(evs[2], s), "hipEventRecord");
    const bool own = s == c->stream;
    if (!own) HIP_TRY(c, hipEventRecord(c->done_ev, s), "hipEventRecord");
    c->done_last = !own;
    c->last_stream = s;
    c->in_flight = true;
    c->any_call = true;
    if (tm) {                           // (untimed calls leave the timing ring as it was)
        c->n_calls++;
        c->timed = true;
    }
    return QSMD_OK;
}

int qsmd_check_batch_device(qsmd_ctx* c, uint32_t model_id, const qsmd_hdr* hdr_dev, uint64_t n_hist,
                            const qsmd_event* events_dev, uint64_t n_events, const void* model0_host,
                            uint32_t flags, uint64_t max_nodes, uint8_t* status_dev, uint64_t* nodes_dev,
                            uint8_t* witness_dev, qsmd_totals* totals_dev, void* stream) {
    if (!c) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx_stream(c);
    if (!s) return fail(c, QSMD_ERR_DEVICE, "hipStreamCreate");
    return check_device_locked(c, model_id, hdr_dev, n_hist, events_dev, n_events, model0_host, flags,
                               max_nodes, status_dev, nodes_dev, witness_dev, totals_dev, s);
}

// Grow the pinned host mirror of the io buffer (the previous call is done
// with it: the host entry point synchronises before it returns).
static int grow_pinned(qsmd_ctx* c, size_t need) {
    if (c->pin_bytes >= need) return QSMD_OK;
    quiesce(c);
    if (c->pin) (void)hipHostFree(c->pin);
    c->pin = nullptr;
    c->pin_bytes = 0;
    const size_t sz = std::max(need, (size_t)64 * 1024);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&c->pin), sz, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(c, QSMD_ERR_NOMEM, "hipHostMalloc", e);
    }
    c->pin_bytes = sz;
    return QSMD_OK;
}

int qsmd_check_batch(qsmd_ctx* c, uint32_t model_id, const qsmd_hdr* hdr, uint64_t n_hist,
                     const qsmd_event* events, uint64_t n_events, const void* model0, uint32_t flags,
                     uint64_t max_nodes, uint8_t* status_out, uint64_t* nodes_out, uint8_t* witness_out,
                     qsmd_totals* totals_out) {
    if (!c) return QSMD_ERR_ARG;
    if (n_hist && (!hdr || !status_out)) return fail(c, QSMD_ERR_ARG, "null hdr/status");
    if (n_events && !events) return fail(c, QSMD_ERR_ARG, "null events");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    hipStream_t s = ctx_stream(c);
    if (!s) return fail(c, QSMD_ERR_DEVICE, "hipStreamCreate");
    HIP_TRY(c, order_after_previous(c, s), "order after the previous call");
    const bool want_w = (flags & QSMD_FLAG_WITNESS) && witness_out;
    // io layout: [hdr | events | witness] copied in, [witness | status | nodes | totals] copied out
    const size_t o_hdr = 0;
    const size_t o_ev = o_hdr + align_up(n_hist * sizeof(qsmd_hdr), 16);
    const size_t o_w = o_ev + align_up(n_events * sizeof(qsmd_event), 16);
    const size_t o_st = o_w + align_up(want_w ? n_events : 0, 16);
    const size_t o_nd = o_st + align_up(n_hist, 16);
    const size_t o_tot = o_nd + align_up(n_hist * 8, 16);
    const size_t need = o_tot + align_up(sizeof(qsmd_totals), 16);
    // a small call (the per-history drop-in's) runs on a mapped host buffer:
    // the kernels read headers and events and store the outputs over the bus
    // (plain loads and stores only), so no copy precedes or follows them
    if (need <= kZeroCopyBytes && !c->zc) {
        if (hipHostMalloc(reinterpret_cast<void**>(&c->zc), kZeroCopyBytes,
                          hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void**>(&c->zc_dev), c->zc, 0) != hipSuccess) {
            (void)hipGetLastError();
            if (c->zc) (void)hipHostFree(c->zc);
            c->zc = nullptr;
            c->zc_dev = nullptr;
        }
    }
    const bool zero_copy = need <= kZeroCopyBytes && c->zc_dev != nullptr;
    int rc = QSMD_OK;
    if (!zero_copy) {
        rc = grow(c, &c->io, &c->io_bytes, need);
        if (rc) return rc;
        rc = grow_pinned(c, need);
        if (rc) return rc;
    }
    char* host = zero_copy ? c->zc : c->pin;               // the host side of the buffer
    char* dev = zero_copy ? c->zc_dev : c->io;             // the kernels' side
    if (n_hist) std::memcpy(host + o_hdr, hdr, n_hist * sizeof(qsmd_hdr));
    if (n_events) std::memcpy(host + o_ev, events, n_events * sizeof(qsmd_event));
    if (want_w) std::memset(host + o_w, 0xFF, n_events);
    auto* d_hdr = reinterpret_cast<qsmd_hdr*>(dev + o_hdr);
    auto* d_ev = reinterpret_cast<qsmd_event*>(dev + o_ev);
    auto* d_st = reinterpret_cast<uint8_t*>(dev + o_st);
    auto* d_nd = reinterpret_cast<uint64_t*>(dev + o_nd);
    auto* d_w = reinterpret_cast<uint8_t*>(dev + o_w);
    auto* d_tot = reinterpret_cast<qsmd_totals*>(dev + o_tot);
    if (o_st && !zero_copy) HIP_TRY(c, hipMemcpyAsync(c->io, c->pin, o_st, hipMemcpyHostToDevice, s), "H2D inputs");
    // routing from the headers: skip the compact stages no history fits
    bool fits0 = false, fits0w = false;
    for (uint64_t i = 0; i < n_hist && !fits0; ++i) {
        const bool few = hdr[i].n_pid <= 8u;
        fits0 = fits0 || (few && hdr[i].n_ev <= 32u);
        fits0w = fits0w || (few && hdr[i].n_ev <= 64u);
    }
    const uint32_t route = n_hist == 0 ? 0u : (fits0 ? 0u : kSkip0) | (fits0w || fits0 ? 0u : kSkip0w);
    rc = check_device_locked(c, model_id, d_hdr, n_hist, d_ev, n_events, model0, flags, max_nodes, d_st, d_nd,
                             want_w ? d_w : nullptr, d_tot, s, route);
    if (rc) {
        // kernels enqueued before the failure may still read the inputs and
        // write the outputs in zc / pin: done before the next call writes there
        (void)hipStreamSynchronize(s);
        return rc;
    }
    if (!zero_copy)
        HIP_TRY(c, hipMemcpyAsync(c->pin + o_w, c->io + o_w, need - o_w, hipMemcpyDeviceToHost, s), "D2H outputs");
    HIP_TRY(c, hipStreamSynchronize(s), "hipStreamSynchronize");
    c->in_flight = false;
    if (n_hist) std::memcpy(status_out, host + o_st, n_hist);
    if (n_hist && nodes_out) std::memcpy(nodes_out, host + o_nd, n_hist * 8);
    if (want_w) std::memcpy(witness_out, host + o_w, n_events);
    if (totals_out) std::memcpy(totals_out, host + o_tot, sizeof(qsmd_totals));
    return QSMD_OK;
}

static int wellformed_locked(qsmd_ctx* c, const qsmd_hdr* hdr, uint64_t n_hist, const qsmd_event* events,
                             uint64_t n_events, const uint8_t* pids, uint32_t n_pids, qsmd_wf* out,
                             hipStream_t s) {
    if (n_hist && (!hdr || !out)) return fail(c, QSMD_ERR_ARG, "null hdr/out");
    if (pids && n_pids > QSMD_MAX_PIDS) return fail(c, QSMD_ERR_ARG, "more than 128 pids");
    // rank table: in the context's pinned buffer, copied in order on the stream
    if (!c->wf_rank_host &&
        hipHostMalloc(reinterpret_cast<void**>(&c->wf_rank_host), QSMD_MAX_PIDS, hipHostMallocDefault) != hipSuccess)
        return fail(c, QSMD_ERR_NOMEM, "hipHostMalloc");
    HIP_TRY(c, hipStreamSynchronize(s), "hipStreamSynchronize");   // the pinned table may be in flight
    quiesce(c);
    for (int p = 0; p < QSMD_MAX_PIDS; ++p) c->wf_rank_host[p] = pids ? 0xFF : (uint8_t)p;
    if (pids)
        for (uint32_t i = 0; i < n_pids; ++i) {
            if (pids[i] >= QSMD_MAX_PIDS || c->wf_rank_host[pids[i]] != 0xFF)
                return fail(c, QSMD_ERR_ARG, "pids: index >= 128 or repeated");
            c->wf_rank_host[pids[i]] = (uint8_t)i;
        }
    int rc = grow(c, &c->wf_rank_dev, &c->wf_rank_bytes, QSMD_MAX_PIDS);
    if (rc) return rc;
    HIP_TRY(c, hipMemcpyAsync(c->wf_rank_dev, c->wf_rank_host, QSMD_MAX_PIDS, hipMemcpyHostToDevice, s), "H2D rank");
    if (!n_hist) return QSMD_OK;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n_hist + 63) / 64, 65536);
    HIP_TRY(c, launch_wellformed(hdr, n_hist, reinterpret_cast<const uint2*>(events), n_events,
                                 reinterpret_cast<const uint8_t*>(c->wf_rank_dev), out, grid, s),
            "wellformed launch");
    return QSMD_OK;
}

int qsmd_gen_batch_device(qsmd_ctx* c, const qsmd_gen_params* p, uint64_t first, uint64_t n_hist, uint32_t ev_base,
                          qsmd_hdr* hdr_dev, qsmd_event* events_dev, uint8_t* bug_dev, void* stream) {
    if (!c) return QSMD_ERR_ARG;
    // the parameter checks of qsmd_gen_batch (csrc/gen/gen.cpp)
    if (!p || (n_hist && (!hdr_dev || !events_dev))) return fail(c, QSMD_ERR_ARG, "null params/buffers");
    if (p->model_id != QSMD_MODEL_BANK && p->model_id != QSMD_MODEL_TICKET) return fail(c, QSMD_ERR_ARG, "model_id");
    if (p->n_clients < 1 || p->n_clients > QSMD_BANK_MAX_ACCOUNTS) return fail(c, QSMD_ERR_ARG, "n_clients");
    if (p->n_ops < 1 || 2 * p->n_ops > QSMD_MAX_EVENTS) return fail(c, QSMD_ERR_ARG, "n_ops");
    if (p->model_id == QSMD_MODEL_BANK && p->n_ops < p->n_clients) return fail(c, QSMD_ERR_ARG, "n_ops < n_clients");
    if ((uint64_t)ev_base + n_hist * 2ull * p->n_ops > 0xFFFFFFFFull) return fail(c, QSMD_ERR_ARG, "ev_off beyond u32");
    if (n_hist == 0) return QSMD_OK;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(c, launch_gen(*p, first, n_hist, ev_base, hdr_dev, events_dev, bug_dev,
                          stream ? static_cast<hipStream_t>(stream) : ctx_stream(c)), "gen launch");
    return QSMD_OK;
}

int qsmd_wellformed_batch_device(qsmd_ctx* c, const qsmd_hdr* hdr_dev, uint64_t n_hist, const qsmd_event* events_dev,
                                 uint64_t n_events, const uint8_t* pids, uint32_t n_pids, qsmd_wf* out_dev,
                                 void* stream) {
    if (!c) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    return wellformed_locked(c, hdr_dev, n_hist, events_dev, n_events, pids, n_pids, out_dev,
                             stream ? static_cast<hipStream_t>(stream) : ctx_stream(c));
}

int qsmd_wellformed_batch(qsmd_ctx* c, const qsmd_hdr* hdr, uint64_t n_hist, const qsmd_event* events,
                          uint64_t n_events, const uint8_t* pids, uint32_t n_pids, qsmd_wf* out) {
    if (!c) return QSMD_ERR_ARG;
    if (n_hist && (!hdr || !out)) return fail(c, QSMD_ERR_ARG, "null hdr/out");
    if (n_events && !events) return fail(c, QSMD_ERR_ARG, "null events");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    hipStream_t s = ctx_stream(c);
    if (!s) return fail(c, QSMD_ERR_DEVICE, "hipStreamCreate");
    const size_t o_ev = align_up(n_hist * sizeof(qsmd_hdr));
    const size_t o_out = o_ev + align_up(n_events * sizeof(qsmd_event));
    int rc = grow(c, &c->io, &c->io_bytes, o_out + align_up(n_hist * sizeof(qsmd_wf)));
    if (rc) return rc;
    auto* d_hdr = reinterpret_cast<qsmd_hdr*>(c->io);
    auto* d_ev = reinterpret_cast<qsmd_event*>(c->io + o_ev);
    auto* d_out = reinterpret_cast<qsmd_wf*>(c->io + o_out);
    if (n_hist) HIP_TRY(c, hipMemcpyAsync(d_hdr, hdr, n_hist * sizeof(qsmd_hdr), hipMemcpyHostToDevice, s), "H2D hdr");
    if (n_events) HIP_TRY(c, hipMemcpyAsync(d_ev, events, n_events * sizeof(qsmd_event), hipMemcpyHostToDevice, s), "H2D events");
    rc = wellformed_locked(c, d_hdr, n_hist, d_ev, n_events, pids, n_pids, d_out, s);
    if (rc) return rc;
    if (n_hist) HIP_TRY(c, hipMemcpyAsync(out, d_out, n_hist * sizeof(qsmd_wf), hipMemcpyDeviceToHost, s), "D2H out");
    HIP_TRY(c, hipStreamSynchronize(s), "hipStreamSynchronize");
    return QSMD_OK;
}


int qsmd_last_kernel_ms(qsmd_ctx* c, float* ms) {
    if (!c || !ms) return QSMD_ERR_ARG;
    if (!c->timed || c->n_calls == 0) return fail(c, QSMD_ERR_ARG, "no timed check call yet (qsmd_timing_reset first)");
    hipEvent_t* evs = &c->ev[kSlotEvents * ((c->n_calls - 1) % kTimingSlots)];
    HIP_TRY(c, hipEventSynchronize(evs[2]), "hipEventSynchronize");
    HIP_TRY(c, hipEventElapsedTime(ms, evs[0], evs[2]), "hipEventElapsedTime");
    return QSMD_OK;
}

int qsmd_timing_reset(qsmd_ctx* c) {
    if (!c) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    c->n_calls = 0;
    c->timing = true;
    return QSMD_OK;
}

int qsmd_timing_read_stages(qsmd_ctx* c, float* stage0_ms, float* heavy_ms, float* call_ms, uint64_t max,
                            uint64_t* n_out) {
    if (!c || !n_out) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const uint64_t n = std::min<uint64_t>(std::min<uint64_t>(c->n_calls, kTimingSlots), max);
    const uint64_t first = c->n_calls - n;
    for (uint64_t i = 0; i < n; ++i) {
        hipEvent_t* evs = &c->ev[kSlotEvents * ((first + i) % kTimingSlots)];
        const uint8_t no = c->ev_no0[(first + i) % kTimingSlots];
        HIP_TRY(c, hipEventSynchronize(evs[2]), "hipEventSynchronize");
        if (stage0_ms) {
            if (no & 1u) stage0_ms[i] = 0.0f;   // (no stage 0 in that call)
            else HIP_TRY(c, hipEventElapsedTime(&stage0_ms[i], evs[0], evs[1]), "elapsed");
        }
        if (heavy_ms) {
            if (no & 2u) heavy_ms[i] = -1.0f;   // (the heavy stage in wave mode: not timed)
            else HIP_TRY(c, hipEventElapsedTime(&heavy_ms[i], evs[3], evs[4]), "elapsed");
        }
        if (call_ms) HIP_TRY(c, hipEventElapsedTime(&call_ms[i], evs[0], evs[2]), "elapsed");
    }
    *n_out = n;
    return QSMD_OK;
}

int qsmd_timing_read(qsmd_ctx* c, float* stage0_ms, float* call_ms, uint64_t max, uint64_t* n_out) {
    return qsmd_timing_read_stages(c, stage0_ms, nullptr, call_ms, max, n_out);
}

int qsmd_get_param(qsmd_ctx* c, const char* name, uint64_t* out) {
    if (!c || !name || !out) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const std::string n(name);
    if (n == "stage0_budget_last") {         // the stage-0 budget of the most recent finished call
                                             // (0xFFFFFFFF: none, stage 0 searched every history to its end)
        quiesce(c);
        if (!__atomic_load_n(&c->probe_host[kProbeWritten], __ATOMIC_ACQUIRE))
            return fail(c, QSMD_ERR_ARG, "stage0_budget_last: no finished check call");
        *out = c->probe_host[kProbeBudget];
    } else if (n == "stage0_budget") {       // the set budget, 0 while automatic
        *out = c->s0_auto ? 0 : c->stage0_budget;
    } else if (n == "stage0w_budget_auto") {
        *out = c->s0w_auto ? 1u : 0u;
    } else if (n == "resume_cap") {
        *out = c->resume_cap;
    } else if (n == "fold") {
        *out = c->fold;
    } else if (n == "heavy_mode") {
        *out = c->heavy_mode;
    } else if (n == "memo_after") {
        *out = c->memo_after;
    } else if (n == "tail_cap") {
        *out = c->tail_cap;
    } else if (n == "tail_min") {
        *out = c->tail_min;
    } else if (n == "heavy_buckets") {
        *out = c->heavy_buckets;
    } else {
        return fail(c, QSMD_ERR_ARG, "unknown parameter");
    }
    return QSMD_OK;
}

int qsmd_probe_read(qsmd_ctx* c, uint32_t* out4) {
    if (!c || !out4) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    quiesce(c);
    for (int i = 0; i < 4; ++i) out4[i] = c->probe_host[i];
    return QSMD_OK;
}

int qsmd_timed_out(qsmd_ctx* c, int* out) {
    if (!c || !out) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    quiesce(c);
    *out = c->probe_host[C_TIMED] != 0u ? 1 : 0;
    return QSMD_OK;
}

// ------------------------------------------------------------ split search

static bool split_hdr_ok(const qsmd_hdr* h, uint64_t n_events) {
    return h->n_ev <= QSMD_MAX_EVENTS && h->n_pid <= QSMD_MAX_PIDS && (uint64_t)h->ev_off + h->n_ev <= n_events;
}

static uint32_t split_variant(const qsmd_hdr* h) { return (h->n_ev <= 64 && h->n_pid <= 8) ? 0u : 1u; }

int qsmd_split_frontier(qsmd_ctx* c, uint32_t model_id, const qsmd_hdr* hdr, const qsmd_event* events,
                        uint64_t n_events, const void* model0, uint32_t flags, uint64_t max_nodes,
                        uint32_t min_tasks, qsmd_task* tasks_out, uint64_t max_tasks, qsmd_frontier* fr,
                        uint8_t* witness_out) {
    if (!c) return QSMD_ERR_ARG;
    if (!hdr || !fr || (max_tasks && !tasks_out) || (n_events && !events))
        return fail(c, QSMD_ERR_ARG, "null argument");
    if (model_id != QSMD_MODEL_BANK && model_id != QSMD_MODEL_TICKET) return fail(c, QSMD_ERR_ARG, "unknown model_id");
    if (max_tasks > (1ull << 24)) return fail(c, QSMD_ERR_ARG, "max_tasks > 2^24");
    std::lock_guard<std::mutex> g(c->mu);
    SearchArgs a{};
    int rc = fill_model0(c, model_id, model0, a);
    if (rc) return rc;
    std::memset(fr, 0, sizeof *fr);
    if (!split_hdr_ok(hdr, n_events) || hdr->model_id != model_id) {
        fr->status = QSMD_STATUS_ENCODE_ERROR;
        return QSMD_OK;
    }
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    hipStream_t s = ctx_stream(c);
    if (!s) return fail(c, QSMD_ERR_DEVICE, "hipStreamCreate");
    quiesce(c);
    const uint64_t cap = std::max<uint64_t>(max_tasks, 1);
    const uint32_t v = split_variant(hdr);
    const size_t o_hdr = 0, o_cnt = 256, o_gl = 512, o_gr = 768;
    const size_t o_ev = 1024;
    const size_t o_tk = o_ev + align_up(n_events * sizeof(qsmd_event));
    const size_t o_w = o_tk + align_up(SPLIT_VARIANTS * cap * sizeof(qsmd_task));
    const size_t need = o_w + align_up(QSMD_MAX_EVENTS);
    rc = grow(c, &c->sx, &c->sx_bytes, need);
    if (rc) return rc;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(c->sx + o_cnt);
    const uint32_t one = 1;
    HIP_TRY(c, hipMemcpyAsync(c->sx + o_hdr, hdr, sizeof *hdr, hipMemcpyHostToDevice, s), "H2D hdr");
    if (n_events)
        HIP_TRY(c, hipMemcpyAsync(c->sx + o_ev, events, n_events * sizeof(qsmd_event), hipMemcpyHostToDevice, s), "H2D events");
    HIP_TRY(c, hipMemsetAsync(cnt, 0, 4 * C_N, s), "memset counters");
    HIP_TRY(c, hipMemsetAsync(c->sx + o_gl, 0, 4, s), "memset giant list");
    HIP_TRY(c, hipMemcpyAsync(cnt + C_GIANT, &one, 4, hipMemcpyHostToDevice, s), "H2D giant count");
    a.hdr = reinterpret_cast<const qsmd_hdr*>(c->sx + o_hdr);
    a.events = reinterpret_cast<const uint2*>(c->sx + o_ev);
    a.n_hist = 1;
    a.n_events = n_events;
    a.flags = flags;
    a.model_id = model_id;
    a.max_nodes = max_nodes;
    a.time_limit = c->time_limit_ms * 100000ull;
    a.timed_out = cnt + C_TIMED;
    a.witness = witness_out ? reinterpret_cast<uint8_t*>(c->sx + o_w) : nullptr;
    SplitArgs p{};
    p.s = a;
    p.cnt = cnt;
    p.giant_list = reinterpret_cast<const uint32_t*>(c->sx + o_gl);
    p.giant_count = cnt + C_GIANT;
    p.giants = reinterpret_cast<GiantRec*>(c->sx + o_gr);
    p.tasks = reinterpret_cast<qsmd_task*>(c->sx + o_tk);
    p.task_cap = (uint32_t)cap;
    p.target = std::max<uint32_t>(min_tasks, 1);
    p.max_tasks = (uint32_t)max_tasks;
    p.max_depth = QSMD_SPLIT_MAX_DEPTH;
    p.whole_cap = 0;                      // cut at once (the caller distributes the tasks)
    HIP_TRY(c, launch_frontier_only((int)v, p, s), "frontier launch");
    GiantRec G{};
    HIP_TRY(c, hipMemcpyAsync(&G, p.giants, sizeof G, hipMemcpyDeviceToHost, s), "D2H giant");
    HIP_TRY(c, hipStreamSynchronize(s), "hipStreamSynchronize");
    if (G.n_tasks)
        HIP_TRY(c, hipMemcpy(tasks_out, p.tasks + (uint64_t)G.variant * cap + G.first, G.n_tasks * sizeof(qsmd_task),
                             hipMemcpyDeviceToHost), "D2H tasks");
    if (witness_out && G.term_status == QSMD_STATUS_LINEARISABLE && hdr->n_ev)
        HIP_TRY(c, hipMemcpy(witness_out, c->sx + o_w, hdr->n_ev, hipMemcpyDeviceToHost), "D2H witness");
    fr->status = G.term_status;
    fr->depth = G.depth;
    fr->top_nodes = G.term_nodes;
    fr->n_tasks = G.n_tasks;
    return QSMD_OK;
}

int qsmd_check_tasks(qsmd_ctx* c, uint32_t model_id, const qsmd_hdr* hdr, const qsmd_event* events,
                     uint64_t n_events, const void* model0, uint32_t flags, uint64_t max_nodes,
                     const qsmd_task* tasks, uint64_t n_tasks, uint8_t* status_out, uint64_t* nodes_out,
                     uint8_t* witness_out) {
    if (!c) return QSMD_ERR_ARG;
    if (!hdr || (n_tasks && (!tasks || !status_out)) || (n_events && !events))
        return fail(c, QSMD_ERR_ARG, "null argument");
    if (model_id != QSMD_MODEL_BANK && model_id != QSMD_MODEL_TICKET) return fail(c, QSMD_ERR_ARG, "unknown model_id");
    if (n_tasks > (1ull << 24)) return fail(c, QSMD_ERR_ARG, "n_tasks > 2^24");
    if (hdr->model_id != model_id || !split_hdr_ok(hdr, n_events)) return fail(c, QSMD_ERR_ARG, "bad history header");
    for (uint64_t i = 0; i < n_tasks; ++i) {
        if (tasks[i].hist != 0 || tasks[i].depth > QSMD_SPLIT_MAX_DEPTH || 2u * tasks[i].depth > hdr->n_ev)
            return fail(c, QSMD_ERR_ARG, "bad task (hist must be 0, depth <= 16)");
        for (uint32_t d = 0; d < tasks[i].depth; ++d)
            if (tasks[i].path[d] >= hdr->n_ev) return fail(c, QSMD_ERR_ARG, "bad task path");
    }
    std::lock_guard<std::mutex> g(c->mu);
    SearchArgs a{};
    int rc = fill_model0(c, model_id, model0, a);
    if (rc) return rc;
    if (!n_tasks) return QSMD_OK;
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    hipStream_t s = ctx_stream(c);
    if (!s) return fail(c, QSMD_ERR_DEVICE, "hipStreamCreate");
    quiesce(c);
    const uint32_t v = split_variant(hdr);
    const uint64_t n = n_tasks;
    const bool want_w = witness_out != nullptr;
    const size_t o_hdr = 0, o_cnt = 256, o_gr = 512;
    const size_t o_ev = 1024;
    const size_t o_tk = o_ev + align_up(n_events * sizeof(qsmd_event));
    const size_t o_ts = o_tk + align_up(SPLIT_VARIANTS * n * sizeof(qsmd_task));
    const size_t o_tn = o_ts + align_up(SPLIT_VARIANTS * n);
    const size_t o_tw = o_tn + align_up(SPLIT_VARIANTS * n * 8);
    const size_t need = o_tw + (want_w ? align_up(SPLIT_VARIANTS * n * kTaskWitness) : 0);
    rc = grow(c, &c->sx, &c->sx_bytes, need);
    if (rc) return rc;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(c->sx + o_cnt);
    GiantRec G{};
    G.h = 0;
    G.variant = v;
    G.first = 0;
    G.n_tasks = (uint32_t)n;
    G.term_status = QSMD_STATUS_NONLINEARISABLE;
    G.min_win = ~0u;
    uint32_t counts[C_N] = {};
    counts[C_TASKS0 + v] = (uint32_t)n;
    HIP_TRY(c, hipMemcpyAsync(c->sx + o_hdr, hdr, sizeof *hdr, hipMemcpyHostToDevice, s), "H2D hdr");
    if (n_events)
        HIP_TRY(c, hipMemcpyAsync(c->sx + o_ev, events, n_events * sizeof(qsmd_event), hipMemcpyHostToDevice, s), "H2D events");
    HIP_TRY(c, hipMemcpyAsync(cnt, counts, sizeof counts, hipMemcpyHostToDevice, s), "H2D counters");
    HIP_TRY(c, hipMemcpyAsync(c->sx + o_gr, &G, sizeof G, hipMemcpyHostToDevice, s), "H2D giant");
    auto* d_tk = reinterpret_cast<qsmd_task*>(c->sx + o_tk);
    HIP_TRY(c, hipMemcpyAsync(d_tk + v * n, tasks, n * sizeof(qsmd_task), hipMemcpyHostToDevice, s), "H2D tasks");
    a.hdr = reinterpret_cast<const qsmd_hdr*>(c->sx + o_hdr);
    a.events = reinterpret_cast<const uint2*>(c->sx + o_ev);
    a.n_hist = 1;
    a.n_events = n_events;
    a.flags = flags;
    a.model_id = model_id;
    a.max_nodes = max_nodes;
    a.time_limit = c->time_limit_ms * 100000ull;
    a.timed_out = cnt + C_TIMED;
    SplitArgs p{};
    p.s = a;
    p.cnt = cnt;
    p.giants = reinterpret_cast<GiantRec*>(c->sx + o_gr);
    p.tasks = d_tk;
    p.task_cap = (uint32_t)n;
    p.task_status = reinterpret_cast<uint8_t*>(c->sx + o_ts);
    p.task_nodes = reinterpret_cast<uint64_t*>(c->sx + o_tn);
    p.task_witness = want_w ? reinterpret_cast<uint8_t*>(c->sx + o_tw) : nullptr;
    p.external_tasks = 1;
    if (flags & QSMD_FLAG_MEMO) {
        rc = memo_prepare(c, s, &p.memo, &p.memo_epoch);
        if (rc) return rc;
        p.memo_mask = c->memo_alloc - 1;
    }
    HIP_TRY(c, launch_tasks_only((int)v, p, kTaskGrid[v], s), "task launch");
    HIP_TRY(c, hipMemcpyAsync(status_out, p.task_status + v * n, n, hipMemcpyDeviceToHost, s), "D2H status");
    if (nodes_out)
        HIP_TRY(c, hipMemcpyAsync(nodes_out, p.task_nodes + v * n, n * 8, hipMemcpyDeviceToHost, s), "D2H nodes");
    if (want_w)
        HIP_TRY(c, hipMemcpyAsync(witness_out, p.task_witness + v * n * kTaskWitness, n * kTaskWitness,
                                  hipMemcpyDeviceToHost, s), "D2H witness");
    HIP_TRY(c, hipStreamSynchronize(s), "hipStreamSynchronize");
    return QSMD_OK;
}

int qsmd_combine_tasks(const qsmd_frontier* fr, const qsmd_task* tasks, const uint8_t* status,
                       const uint64_t* nodes, uint64_t n_tasks, uint64_t max_nodes, uint8_t* status_out,
                       uint64_t* nodes_out, int64_t* winner_out) {
    if (!fr || !status_out || !nodes_out || !winner_out || (n_tasks && (!tasks || !status || !nodes)))
        return QSMD_ERR_ARG;
    *status_out = (uint8_t)combine_tasks(fr->status, fr->top_nodes, tasks, status, nodes, n_tasks, max_nodes,
                                         nodes_out, winner_out);
    return QSMD_OK;
}

}  // extern "C"
