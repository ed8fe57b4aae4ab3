// api.hip -- the C ABI of include/qsmd.h: context, workspace, stage cascade.
//
// Replaces the call `linearisable transition postcondition model0 hist`
// (src/Linearisability.hs:52-69) made once per history at test/Bank.hs:285,
// test/TicketDispenser.hs:253 and :320 with one batched call.  The model
// closures are selected by model_id (device functors, csrc/models.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
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
    // workspace (device)
    char* ws = nullptr;
    size_t ws_bytes = 0;
    // staging for the host-memory entry point (device)
    char* io = nullptr;
    size_t io_bytes = 0;
    // timing: per call, events before stage 0, after stage 0 and after the
    // final reduction, recorded on the launch stream (a ring of kTimingSlots)
    std::vector<hipEvent_t> ev;          // 3 per slot
    uint64_t n_calls = 0;                // calls recorded since the last reset
    bool timed = false;
    uint64_t time_limit_ms = 120000;   // safety net per search launch
    uint64_t stage0_max_grid = 65536;  // tuning: cap on stage-0 workgroups (grid-stride beyond)
    unsigned long long* stamps = nullptr;   // diagnostic: stage-0 phase timings
    uint64_t stage0_budget = 0;        // stage-0 node budget before the heavy stages (0 = none)
    // adaptive cascade (default): each call probes how many of its histories
    // needed more than kAutoBudget nodes; while the last probe read back says
    // they are common (>= 1 in kAutoFrac), calls run stage 0 with that budget
    // and the heavy stages, else without (no heavy-stage launches).  Only the
    // speed changes, never a result.  An explicit stage-0 budget turns it off.
    bool stage0_auto = true;
    bool auto_heavy = false;
    bool probe_pending = false;
    uint64_t probe_n_hist = 0;
    uint32_t* probe_host = nullptr;    // pinned copy of the 32 stage counters of the probing call
    bool probe_spread = false;         // that call had a heavy list
    hipEvent_t probe_ev = nullptr;
    uint8_t* wf_rank_host = nullptr;   // wellformed: pid rank table (pinned) and its device copy
    char* wf_rank_dev = nullptr;
    size_t wf_rank_bytes = 0;
    uint64_t split_budget = 1024;      // per-lane node budget before the split stage (0 = none)
    uint64_t stage0_persistent = 0;    // > 0: stage 0 = persistent refill_search (direct) with this grid
    uint64_t refill_min = 8;           // refill kernels: idle lanes before a wavefront refills
    uint64_t spread_budget = 1024;     // spread stage: nodes a task searches before it splits
    uint64_t spread_grid = 1024;       // spread stage: persistent wavefronts
    uint64_t spread_pending = 1024;    // spread stage: split only while fewer tasks wait
    uint64_t heavy_stage = 2;          // histories over the stage-0 budget: 0 = coop, 1 = spread,
                                       // 2 = auto (coop for at most coop_max of them, else spread)
    uint64_t coop_max = 4096;
    uint64_t stage0_kernel = 0;        // 0 = compact_search, 1 = group_search (in-wave sharing)
    uint64_t stage0_dynamic = 0;       // compact_search: groups from a counter (persistent grid)
    uint64_t memo_stage = 1;           // heavy histories: the memo stage (exact-count state memo, csrc/memo.hip)
    uint64_t mt_entries = 256;         // memo stage: table entries per lane (power of two)
    uint64_t memo_min_rem = 0;         // memo stage: states with at most this many events left are not memoised
    uint64_t memo_grid = 2048;         // memo stage: workgroups (table slots = memo_grid * 64)
    char* mt = nullptr;                // memo stage tables: [G32 region][G64 region]
    size_t mt_bytes = 0;
    uint32_t mt_epoch = 0;
    unsigned long long* memo_stats = nullptr;   // diagnostic (memo_stats_ptr)
    uint64_t cut_k = 0;                // straggler cut: lanes still searching when a wave cuts them (0 = off)
    uint64_t cut_min = 16;             // ... after this many iterations
    uint64_t split_xmemo = 1;          // split stage: exact-count memo for the giants' tasks
    char* xm = nullptr;                // its table (kXMemoEntries x 128 B, epoch-tagged)
    size_t xm_bytes = 0;
    uint32_t xm_epoch = 0;
    uint64_t rerun_budget = 0;         // stage 0 budget before the lane re-run (stage 0r); 0 = none
    uint64_t stage0w = 1;              // 33..64-event histories in the compact kernel (else stage 1)
    uint64_t stage0w_budget = 32;      // stage 0w: nodes per history before the memo stage (coop64 without it; 0 = none)
    uint64_t coop64_grid = 512;        // coop64: persistent wavefronts over stage 0w's heavy histories
    uint64_t group_grid = 4096;        // group_search: persistent wavefronts (cap)
    uint64_t group_budget = 16;        // group_search: nodes a shared task searches before it may split
    uint64_t share_idle = 16;          // group_search: idle lanes that start sharing
    uint64_t share_nodes = 32;         // group_search: nodes a search must have counted to be shared
    unsigned long long* group_stats = nullptr;
    unsigned long long* group_debug = nullptr;
    uint64_t coop_grid = 2048;         // coop stage: persistent wavefronts
    uint64_t coop_budget = 16;         // coop stage: nodes a task searches before it may split
    uint64_t spread_cap = 1ull << 22;  // spread stage: task records per call (64 B each)
    uint32_t epoch = 0;                // spread stage: ready-flag value of the current call
    unsigned long long* spread_stamps = nullptr;   // diagnostic: spread task timeline
    char* spt = nullptr;               // spread task records (own buffer: zeroed once, then
    size_t spt_bytes = 0;              // told apart by the epoch of their ready flag)
    const SpreadHist* last_sp_hist = nullptr;   // diagnostics of the last spread launch
    const uint32_t* last_sp_count = nullptr;
    const unsigned long long* last_sp_ad = nullptr;
    // QSMD_FLAG_MEMO table (device), allocated on first use
    unsigned long long* memo = nullptr;
    uint64_t memo_entries = 1ull << 22;
    uint64_t memo_alloc = 0;
    // split-search entry points: their own device buffers
    char* sx = nullptr;
    size_t sx_bytes = 0;
};

namespace {

constexpr uint32_t kStage0wGrid = 1024;
constexpr uint32_t kRerunGrid = 4096;    // stage 0r (list mode, grid-stride)  // list-mode stages: grid-stride
constexpr uint32_t kStage1Grid = 256;   // rare: values beyond the compact encoding
constexpr uint32_t kStage2Grid = 512;   // 65..128 events / > 8 pids (16 lanes per workgroup)
constexpr uint64_t C_LANES_HOST = 64;     // lanes per wavefront (gfx950)
constexpr uint32_t kRedoGrid = 64;      // exact re-search of spread histories the speculation cap cut
constexpr uint32_t kSpreadFinalGrid = 64;
constexpr uint64_t kAutoProbe = 256;     // adaptive cascade: a long search counts more nodes than this
constexpr uint64_t kAutoBudget = 64;     // ... and the stage-0 budget when long searches are common
constexpr uint64_t kQuietBudget = 512;   // ... and outside heavy mode, with the memo stage
constexpr uint64_t kQuietMemoGrid = 256; // memo-stage grid outside heavy mode
constexpr uint64_t kAutoFrac = 1000;     // ... i.e. at least 1 history in kAutoFrac needs more
constexpr uint64_t kTimingSlots = 1024;
constexpr uint32_t kFrontierGrid = 256;  // split stage: one lane per giant history, grid-stride
constexpr uint32_t kTaskGrid[SPLIT_VARIANTS] = {1024, 512};   // persistent task wavefronts
constexpr uint32_t kCombineGrid = 64;
constexpr uint64_t kXMemoEntries = 1ull << 22;   // split stage exact memo: 512 MB (shared by all giants of a call)
constexpr uint32_t kTaskCap = 1u << 19;  // tasks per variant per call (beyond: searched unsplit)
constexpr uint32_t kSplitTarget = 256;   // tasks wanted per giant history
constexpr uint32_t kSplitMaxTasks = 4096;

int fail(qsmd_ctx* c, int code, const char* what, hipError_t e = hipSuccess) {
    if (c) {
        char buf[256];
        if (e != hipSuccess) std::snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
        else std::snprintf(buf, sizeof buf, "%s", what);
        c->err = buf;
    }
    return code;
}

#define HIP_TRY(c, expr, what)                                  \
    do {                                                        \
        hipError_t _e = (expr);                                 \
        if (_e != hipSuccess) return fail((c), QSMD_ERR_DEVICE, (what), _e); \
    } while (0)

size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

int grow(qsmd_ctx* c, char** buf, size_t* cap, size_t need) {
    if (*cap >= need) return QSMD_OK;
    if (*buf) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(*buf);
        *buf = nullptr;
        *cap = 0;
    }
    size_t sz = std::max(need, *cap * 3 / 2);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(buf), sz);
    if (e != hipSuccess) return fail(c, QSMD_ERR_NOMEM, "hipMalloc", e);
    *cap = sz;
    return QSMD_OK;
}

bool in_i32(int64_t v) { return v >= INT32_MIN && v <= INT32_MAX; }

int fill_model0(qsmd_ctx* c, uint32_t model_id, const void* model0, SearchArgs& a) {
    a.m0_exists = 0;
    a.m0_just = 0;
    a.m0_small = 1;
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
    for (int64_t v : a.m0_val)
        if (v < -(1 << 18) || v >= (1 << 18)) a.m0_small = 0;   // stage 0 holds 19-bit values
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
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return QSMD_ERR_DEVICE;
    }
    c->ev.resize(3 * kTimingSlots, nullptr);
    for (auto& e : c->ev) {
        if (hipEventCreate(&e) != hipSuccess) { qsmd_close(c); return QSMD_ERR_DEVICE; }
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
    if (hipEventCreateWithFlags(&c->probe_ev, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->probe_host), 128, hipHostMallocDefault) != hipSuccess) {
        qsmd_close(c);
        return QSMD_ERR_DEVICE;
    }
    *out = c;
    return QSMD_OK;
}

void qsmd_close(qsmd_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->ws) (void)hipFree(c->ws);
    if (c->sx) (void)hipFree(c->sx);
    if (c->spt) (void)hipFree(c->spt);
    if (c->mt) (void)hipFree(c->mt);
    if (c->xm) (void)hipFree(c->xm);
    if (c->memo) (void)hipFree(c->memo);
    if (c->io) (void)hipFree(c->io);
    for (auto e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->probe_ev) (void)hipEventDestroy(c->probe_ev);
    if (c->probe_host) (void)hipHostFree(c->probe_host);
    if (c->wf_rank_host) (void)hipHostFree(c->wf_rank_host);
    if (c->wf_rank_dev) (void)hipFree(c->wf_rank_dev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int qsmd_diag_stamps(qsmd_ctx* c, void* stamps_dev) {
    if (!c) return QSMD_ERR_ARG;
    c->stamps = static_cast<unsigned long long*>(stamps_dev);
    return QSMD_OK;
}

int qsmd_spread_stats(qsmd_ctx* c, uint64_t* out4) {
    if (!c || !out4) return QSMD_ERR_ARG;
    for (int i = 0; i < 4; ++i) out4[i] = 0;
    if (!c->last_sp_hist) return QSMD_OK;
    HIP_TRY(c, hipDeviceSynchronize(), "sync");
    uint32_t n = 0;
    unsigned long long ad = 0;
    HIP_TRY(c, hipMemcpy(&n, c->last_sp_count, 4, hipMemcpyDeviceToHost), "D2H");
    HIP_TRY(c, hipMemcpy(&ad, c->last_sp_ad, 8, hipMemcpyDeviceToHost), "D2H");
    std::vector<SpreadHist> h(n);
    if (n) HIP_TRY(c, hipMemcpy(h.data(), c->last_sp_hist, n * sizeof(SpreadHist), hipMemcpyDeviceToHost), "D2H");
    out4[0] = n;
    out4[1] = ad >> 32;
    for (const auto& r : h) {
        out4[2] += r.explored;
        out4[3] += r.sum;
    }
    return QSMD_OK;
}

int qsmd_set_stage0_budget(qsmd_ctx* c, uint64_t nodes) {
    if (!c) return QSMD_ERR_ARG;
    c->stage0_budget = nodes;
    c->stage0_auto = false;
    return QSMD_OK;
}

int qsmd_set_param(qsmd_ctx* c, const char* name, uint64_t value) {
    if (!c || !name) return QSMD_ERR_ARG;
    const std::string n(name);
    if (n == "stage0_persistent_grid") {
        if (value > 0x7FFFFFFFull) return fail(c, QSMD_ERR_ARG, "grid too large");
        c->stage0_persistent = value;
    } else if (n == "refill_min") {
        if (value < 1 || value > 64) return fail(c, QSMD_ERR_ARG, "refill_min in 1..64");
        c->refill_min = value;
    } else if (n == "spread_budget") {
        if (value < 1) return fail(c, QSMD_ERR_ARG, "spread_budget >= 1");
        c->spread_budget = value;
    } else if (n == "spread_pending") {
        c->spread_pending = std::min<uint64_t>(value, 0xFFFFFFFFull);
    } else if (n == "spread_stamps_ptr") {   // diagnostic: device buffer of 4 x u64 per task slot
        c->spread_stamps = reinterpret_cast<unsigned long long*>(value);
    } else if (n == "stage0_kernel") {
        if (value > 1) return fail(c, QSMD_ERR_ARG, "stage0_kernel: 0 = compact, 1 = group");
        c->stage0_kernel = value;
    } else if (n == "memo_stage") {
        c->memo_stage = value ? 1 : 0;
    } else if (n == "memo_lane_entries") {
        if (value < 2 || value > 65536 || (value & (value - 1)))
            return fail(c, QSMD_ERR_ARG, "memo_lane_entries: a power of two in 2..65536");
        c->mt_entries = value;
    } else if (n == "memo_min_rem") {
        c->memo_min_rem = std::min<uint64_t>(value, 128);
    } else if (n == "memo_grid") {
        if (value < 1 || value > 65536) return fail(c, QSMD_ERR_ARG, "memo_grid in 1..65536");
        c->memo_grid = value;
    } else if (n == "memo_stats_ptr") {     // diagnostic: device buffer of 3 x u64 (iterations, hits, inserts)
        c->memo_stats = reinterpret_cast<unsigned long long*>(value);
    } else if (n == "cut_k") {
        if (value > 63) return fail(c, QSMD_ERR_ARG, "cut_k in 0..63");
        c->cut_k = value;
    } else if (n == "cut_min") {
        c->cut_min = std::min<uint64_t>(value, 0xFFFFFFFFull);
    } else if (n == "split_xmemo") {
        c->split_xmemo = value ? 1 : 0;
    } else if (n == "rerun_budget") {
        c->rerun_budget = value;
    } else if (n == "stage0w") {
        c->stage0w = value ? 1 : 0;
    } else if (n == "stage0w_budget") {
        c->stage0w_budget = value;
    } else if (n == "coop64_grid") {
        if (value < 1 || value > 65536) return fail(c, QSMD_ERR_ARG, "coop64_grid in 1..65536");
        c->coop64_grid = value;
    } else if (n == "stage0_dynamic") {
        c->stage0_dynamic = value ? 1 : 0;
    } else if (n == "group_grid") {
        if (value < 1 || value > 65536) return fail(c, QSMD_ERR_ARG, "group_grid in 1..65536");
        c->group_grid = value;
    } else if (n == "group_budget") {
        if (value < 1) return fail(c, QSMD_ERR_ARG, "group_budget >= 1");
        c->group_budget = value;
    } else if (n == "share_idle") {
        if (value < 1 || value > 64) return fail(c, QSMD_ERR_ARG, "share_idle in 1..64");
        c->share_idle = value;
    } else if (n == "share_nodes") {
        c->share_nodes = std::min<uint64_t>(value, 0xFFFFFFFFull);
    } else if (n == "group_debug_ptr") {    // diagnostic: device buffer of 256 x u64 per block
        c->group_debug = reinterpret_cast<unsigned long long*>(value);
    } else if (n == "group_stats_ptr") {    // diagnostic: device buffer of 8 x u64 per group_search block
        c->group_stats = reinterpret_cast<unsigned long long*>(value);
    } else if (n == "heavy_stage") {
        if (value > 2) return fail(c, QSMD_ERR_ARG, "heavy_stage: 0 = coop, 1 = spread, 2 = auto");
        c->heavy_stage = value;
    } else if (n == "coop_max") {
        c->coop_max = std::min<uint64_t>(value, 0xFFFFFFFFull);
    } else if (n == "coop_grid") {
        if (value < 1 || value > 65536) return fail(c, QSMD_ERR_ARG, "coop_grid in 1..65536");
        c->coop_grid = value;
    } else if (n == "coop_budget") {
        if (value < 1) return fail(c, QSMD_ERR_ARG, "coop_budget >= 1");
        c->coop_budget = value;
    } else if (n == "spread_grid") {
        if (value < 1 || value > 65536) return fail(c, QSMD_ERR_ARG, "spread_grid in 1..65536");
        c->spread_grid = value;
    } else if (n == "spread_cap") {
        if (value < 1024 || value > 0xFFFFFFF0ull) return fail(c, QSMD_ERR_ARG, "spread_cap in 1024..2^32-16");
        c->spread_cap = value;
    } else if (n == "split_budget") {
        c->split_budget = value;
    } else if (n == "stage0_budget") {
        c->stage0_budget = value;
        c->stage0_auto = false;
    } else if (n == "stage0_auto") {
        c->stage0_auto = value != 0;
    } else if (n == "stage0_grid") {
        if (value == 0 || value > 0x7FFFFFFFull) return fail(c, QSMD_ERR_ARG, "bad grid");
        c->stage0_max_grid = value;
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

// The memo table, cleared for this call (entries are only valid within one).
static int memo_prepare(qsmd_ctx* c, hipStream_t s, unsigned long long** out) {
    if (c->memo_alloc != c->memo_entries) {
        if (c->memo) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(c->memo);
            c->memo = nullptr;
            c->memo_alloc = 0;
        }
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&c->memo), c->memo_entries * 64);
        if (e != hipSuccess) return fail(c, QSMD_ERR_NOMEM, "hipMalloc memo table", e);
        c->memo_alloc = c->memo_entries;
    }
    HIP_TRY(c, hipMemsetAsync(c->memo, 0, c->memo_alloc * 64, s), "memset memo table");
    *out = c->memo;
    return QSMD_OK;
}

static int check_device_locked(qsmd_ctx* c, uint32_t model_id, const qsmd_hdr* hdr, uint64_t n_hist,
                               const qsmd_event* events, uint64_t n_events, const void* model0,
                               uint32_t flags, uint64_t max_nodes, uint8_t* status, uint64_t* nodes,
                               uint8_t* witness, qsmd_totals* totals, hipStream_t s) {
    if (model_id != QSMD_MODEL_BANK && model_id != QSMD_MODEL_TICKET)
        return fail(c, QSMD_ERR_ARG, "unknown model_id");
    if (n_hist && (!hdr || !status)) return fail(c, QSMD_ERR_ARG, "null hdr/status");
    if (n_hist > 0xFFFFFFFFull) return fail(c, QSMD_ERR_ARG, "n_hist > 2^32-1");
    const bool early = (flags & QSMD_FLAG_EARLY_EXIT_BATCH) != 0;
    SearchArgs a{};
    int rc = fill_model0(c, model_id, model0, a);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");

    // ---- workspace: defer lists, counters, partials, internal totals
    const bool persistent = c->stage0_persistent != 0;
    const bool grp = c->stage0_kernel == 1 && !persistent;   // group_search (in-wave sharing)
    const uint64_t n_groups = std::max<uint64_t>((n_hist + 63) / 64, 1);
    const uint64_t g0 = persistent ? c->stage0_persistent
                        : grp      ? std::min<uint64_t>(n_groups, c->group_grid)
                                   : std::min<uint64_t>(n_groups, c->stage0_max_grid);
    // stage-0 node budget (compact_search): the histories over it go to the
    // heavy stages (and the ones a speculation cap cut to an exact
    // re-search, kRedoGrid); group_search shares them in-wave instead
    // adaptive cascade: the decision of the last probe that has landed
    if (c->stage0_auto && c->probe_pending && hipEventQuery(c->probe_ev) == hipSuccess) {
        // heavy-list entries (minus the cut stragglers) + long finished searches
        const uint64_t heavy = c->probe_spread ? c->probe_host[4] : 0u;
        const uint64_t longs = heavy - std::min<uint64_t>(heavy, c->probe_host[28]) + c->probe_host[22];
        c->auto_heavy = longs * kAutoFrac >= std::max<uint64_t>(c->probe_n_hist, 1);
        c->probe_pending = false;
    }
    // memo tables first: if the device cannot hold them, this context runs
    // without the memo stage (coop / spread take the heavy histories: the
    // same results, more work)
    const uint64_t mt_slots = c->memo_grid * C_LANES_HOST * c->mt_entries;
    if (c->memo_stage && c->mt_bytes < (size_t)mt_slots * (32 + 64)) {
        if (grow(c, &c->mt, &c->mt_bytes, (size_t)mt_slots * (32 + 64)) != QSMD_OK) {
            (void)hipGetLastError();     // clear the allocation error: later launches check it
            c->memo_stage = 0;
            c->err = "memo tables do not fit on the device: memo stage off for this context";
        } else {
            HIP_TRY(c, hipMemsetAsync(c->mt, 0, c->mt_bytes, s), "memset memo tables");
        }
    }
    // (with the memo stage, a call that is not in heavy mode still sends the
    // histories over min(split budget, 512) nodes to it: it searches most of
    // them in far fewer nodes, and hands the rest to the split stage)
    const uint64_t quiet0 = c->memo_stage ? std::min<uint64_t>(c->split_budget, kQuietBudget) : 0;
    const uint64_t budget0 = c->stage0_auto ? (c->auto_heavy ? kAutoBudget : quiet0) : c->stage0_budget;
    const bool probe = c->stage0_auto && !grp && !persistent && !c->probe_pending;
    const bool spread = !grp && budget0 && !persistent && (!max_nodes || budget0 < max_nodes);
    const bool grp_redo = grp && max_nodes;
    const bool memo0 = spread && c->memo_stage;       // heavy histories -> the memo stage
    const bool coop = spread && !memo0 && c->heavy_stage != 1;
    const bool use_spread = spread && !memo0 && c->heavy_stage != 0;
    // memo grids: outside heavy mode few histories reach the memo stage
    const uint64_t g_m0 = (c->stage0_auto && !c->auto_heavy) ? std::min<uint64_t>(c->memo_grid, kQuietMemoGrid)
                                                               : c->memo_grid;
    const uint64_t g_mw = c->memo_grid;
    const uint64_t g_heavy = memo0 ? g_m0 : (coop ? c->coop_grid : 0) + (use_spread ? kSpreadFinalGrid : 0);
    const uint64_t g0b = spread ? g_heavy + (memo0 ? 0 : kRedoGrid) : (grp_redo ? kRedoGrid : 0);
    const uint64_t gfx = early ? std::min<uint64_t>(std::max<uint64_t>((n_hist + 63) / 64, 1), 4096) : 0;
    const bool split = c->split_budget && (!max_nodes || c->split_budget < max_nodes);
    const bool want_w = (flags & QSMD_FLAG_WITNESS) && witness;
    const uint64_t gsp = split ? kCombineGrid : 0;
    // stage 0r: stage 0 stops every history at rerun_budget nodes (wavefronts
    // then run as long as that, not as their slowest lane); the ones over it
    // are searched again from the root, packed, in list mode, with what stage
    // 0 would otherwise have done (probe, heavy budget, split)
    const bool rerun = c->rerun_budget && !grp && !persistent && (!max_nodes || c->rerun_budget < max_nodes);
    const uint64_t gr = rerun ? std::min<uint64_t>(n_groups, kRerunGrid) : 0;
    const uint64_t g0r = g0 + gr;
    const uint64_t gw0 = c->stage0w ? kStage0wGrid : 0;   // stage 0w: 33..64-event compact
    // stage 0w over its node budget: coop64 (+ an exact redo when no split takes the capped ones)
    const bool heavy_w = gw0 && c->stage0w_budget && (!max_nodes || c->stage0w_budget < max_nodes);
    const bool memo_w = heavy_w && c->memo_stage;
    const uint64_t gwh = memo_w ? g_mw : heavy_w ? c->coop64_grid + (split ? 0 : kRedoGrid) : 0;
    const uint64_t gw = gw0 + gwh;
    const uint64_t n_part = g0r + g0b + gw + kStage1Grid + kStage2Grid + gsp + gfx;
    // counters (32 x u32, zeroed by prep_kernel; [6] = none):
    //   [0] stage-0 defer list, [1] stage-1 defer list, [2] timed out, [3] never written,
    //   [4] heavy list, [5] heavy queue head, [6] first failing history, [7] giant list,
    //   [8..9] tasks per variant, [10..11] task queue heads, [12] persistent head,
    //   [13..14] redo list / head, [16..17] spread ad, [18] spread head, [19] coop next,
    //   [20] group next, [21] dynamic stage-0 head, [22] probe (long finished searches),
    //   [23] stage-0w defer list, [24..26] stage-0w heavy list / coop64 next / redo list,
    //   [27] stage-0r list, [28] straggler cuts
    const size_t off_cnt = 0;
    const size_t off_tot = 256;                                        // qsmd_totals
    const size_t off_l0 = 512;
    const size_t off_l1 = off_l0 + align_up(n_hist * 4 + 4);
    const size_t off_lh = off_l1 + align_up(n_hist * 4 + 4);
    const size_t off_lw = off_lh + align_up(n_hist * 4 + 4);
    const size_t off_lr = off_lw + (gw0 ? align_up(n_hist * 4 + 4) : 0);         // stage 0r list
    const size_t off_lwh = off_lr + (rerun ? align_up(n_hist * 4 + 4) : 0);      // stage 0w heavy
    const size_t off_lwr = off_lwh + (heavy_w ? align_up(n_hist * 4 + 4) : 0);   // coop64 redo
    const size_t off_lg = off_lwr + (heavy_w && !split ? align_up(n_hist * 4 + 4) : 0);
    const size_t off_nd = off_lg + (split ? align_up(n_hist * 4 + 4) : 0);   // nodes if the caller has none
    const size_t off_gr = off_nd + (early && !nodes ? align_up(n_hist * 8) : 0);
    const size_t off_tk = off_gr + (split ? align_up(n_hist * sizeof(GiantRec)) : 0);
    const uint64_t n_tk = split ? (uint64_t)SPLIT_VARIANTS * kTaskCap : 0;
    const size_t off_ts = off_tk + align_up(n_tk * sizeof(qsmd_task));
    const size_t off_tn = off_ts + align_up(n_tk);
    const size_t off_tw = off_tn + align_up(n_tk * 8);
    const size_t off_sh = off_tw + (want_w ? align_up(n_tk * kTaskWitness) : 0);
    const uint64_t sp_cap = use_spread ? c->spread_cap : 0;
    const size_t off_sr = off_sh + (spread ? align_up(n_hist * sizeof(SpreadHist)) : 0);
    const size_t off_gs = off_sr + ((spread || grp_redo) ? align_up(n_hist * 4 + 4) : 0);
    const size_t off_part = off_gs + (grp ? align_up(g0 * sizeof(GroupScratch)) : 0);
    const size_t need = off_part + align_up(n_part * T_N * 8);
    rc = grow(c, &c->ws, &c->ws_bytes, need);
    if (rc) return rc;
    if (sp_cap && c->spt_bytes < sp_cap * sizeof(SpreadTask)) {
        rc = grow(c, &c->spt, &c->spt_bytes, sp_cap * sizeof(SpreadTask));
        if (rc) return rc;
        HIP_TRY(c, hipMemsetAsync(c->spt, 0, c->spt_bytes, s), "memset spread tasks");
    }
    const bool mt_used = memo0 || memo_w;
    if (mt_used && ((++c->mt_epoch) & 0xFFFFFFu) == 0u) {   // 24-bit tags wrapped: clear
        HIP_TRY(c, hipMemsetAsync(c->mt, 0, c->mt_bytes, s), "memset memo tables");
        ++c->mt_epoch;
    }
    uint32_t* cnt = reinterpret_cast<uint32_t*>(c->ws + off_cnt);
    qsmd_totals* tot = totals ? totals : reinterpret_cast<qsmd_totals*>(c->ws + off_tot);
    uint32_t* l0 = reinterpret_cast<uint32_t*>(c->ws + off_l0);
    uint32_t* l1 = reinterpret_cast<uint32_t*>(c->ws + off_l1);
    uint32_t* lh = reinterpret_cast<uint32_t*>(c->ws + off_lh);
    unsigned long long* part = reinterpret_cast<unsigned long long*>(c->ws + off_part);
    if (early && !nodes) nodes = reinterpret_cast<uint64_t*>(c->ws + off_nd);

    HIP_TRY(c, launch_prep(cnt, tot, s), "prep launch");
    a.first_fail = early ? cnt + 6 : nullptr;

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
    a.timed_out = cnt + 2;
    a.refill_min = (uint32_t)c->refill_min;
    uint32_t* lg = reinterpret_cast<uint32_t*>(c->ws + off_lg);
    if (split) {
        a.giant_list = lg;
        a.giant_count = cnt + 7;
        a.split_budget = c->split_budget;
    }

    hipEvent_t* evs = &c->ev[3 * (c->n_calls % kTimingSlots)];
    HIP_TRY(c, hipEventRecord(evs[0], s), "hipEventRecord");
    // stage 0: direct over [0, n_hist)
    SearchArgs a0 = a;
    a0.list = nullptr;
    a0.list_count = nullptr;
    a0.defer_list = l0;
    a0.defer_count = cnt + 0;
    a0.partials = part;
    a0.stamps = c->stamps;
    if (probe && !c->auto_heavy) {      // not in heavy mode: count the long searches
        a0.probe = cnt + 22;
        a0.probe_nodes = kAutoProbe;
    }
    if (spread) {                       // stage 0 -> spread (-> exact redo)
        a0.heavy_list = lh;
        a0.heavy_count = cnt + 4;
        a0.stage0_budget = budget0;
        if (memo0 && c->cut_k) {        // stragglers -> the memo stage as well
            a0.cut_k = (uint32_t)c->cut_k;
            a0.cut_min = (uint32_t)c->cut_min;
            a0.cut_count = cnt + 28;
        }
    } else if (split) {                 // stage 0 -> split
        a0.heavy_list = lg;
        a0.heavy_count = cnt + 7;
        a0.stage0_budget = c->split_budget;
    }
    if (persistent) {                   // persistent lanes, each refilled with its own history
        SearchArgs ad = a;
        ad.list = nullptr;
        ad.defer_list = l0;
        ad.defer_count = cnt + 0;
        ad.queue_head = cnt + 12;
        ad.partials = part;
        HIP_TRY(c, launch_refill(ad, (uint32_t)g0, s), "stage 0 (persistent) launch");
    } else {
        if (grp) {
            GroupArgs gp{};
            gp.s = a0;
            gp.s.heavy_list = nullptr;
            gp.s.giant_list = nullptr;
            gp.scratch = reinterpret_cast<GroupScratch*>(c->ws + off_gs);
            gp.group_next = cnt + 20;
            gp.task_budget = c->group_budget;
            gp.share_idle = (uint32_t)c->share_idle;
            gp.share_nodes = (uint32_t)c->share_nodes;
            gp.explore_cap = max_nodes ? 16 * max_nodes + 64 * c->group_budget : 0;
            gp.redo_list = reinterpret_cast<uint32_t*>(c->ws + off_sr);
            gp.redo_count = cnt + 13;
            gp.stats = c->group_stats;
            gp.debug = c->group_debug;
            HIP_TRY(c, launch_group(gp, (uint32_t)g0, s), "stage 0 (group) launch");
        } else if (rerun) {
            SearchArgs ab = a0;          // stage 0 with the re-run budget
            ab.probe = nullptr;
            ab.heavy_list = reinterpret_cast<uint32_t*>(c->ws + off_lr);
            ab.heavy_count = cnt + 27;
            ab.stage0_budget = c->rerun_budget;
            ab.queue_head = c->stage0_dynamic ? cnt + 21 : nullptr;
            HIP_TRY(c, launch_compact(ab, (uint32_t)g0, s), "stage 0 launch");
            a0.list = ab.heavy_list;     // stage 0r: the rest as stage 0 would have
            a0.list_count = ab.heavy_count;
            a0.stamps = nullptr;
            a0.partials = part + g0 * T_N;
            HIP_TRY(c, launch_compact(a0, (uint32_t)gr, s), "stage 0r launch");
        } else {
            a0.queue_head = c->stage0_dynamic ? cnt + 21 : nullptr;
            HIP_TRY(c, launch_compact(a0, (uint32_t)g0, s), "stage 0 launch");
        }
    }
    HIP_TRY(c, hipEventRecord(evs[1], s), "hipEventRecord");
    // stage 0b: histories over the stage-0 node budget: one wavefront per
    // history (coop), or the global dynamic split (spread)
    if (memo0) {
        MemoArgs mp{};
        mp.s = a;
        mp.s.giant_list = nullptr;
        mp.s.list = lh;
        mp.s.list_count = cnt + 4;
        mp.s.partials = part + g0r * T_N;
        if (split) {                    // the ones the memo does not tame: -> split
            mp.s.giant_list = lg;
            mp.s.giant_count = cnt + 7;
            mp.giant_cap = c->split_budget;
        }
        mp.table = reinterpret_cast<uint32_t*>(c->mt);
        mp.entries = (uint32_t)c->mt_entries;
        mp.min_rem = (uint32_t)c->memo_min_rem;
        mp.epoch = c->mt_epoch;
        mp.stats = c->memo_stats;
        HIP_TRY(c, launch_memo(mp, (uint32_t)g_m0, false, s), "memo launch");
        c->last_sp_hist = nullptr;
    }
    if (coop) {
        CoopArgs cp{};
        cp.s = a;
        cp.s.giant_list = nullptr;
        cp.s.partials = part + g0r * T_N;
        cp.heavy_list = lh;
        cp.heavy_count = cnt + 4;
        cp.next = cnt + 19;
        cp.budget = c->coop_budget;
        cp.explore_cap = max_nodes ? 16 * max_nodes + 64 * c->coop_budget : 0;
        cp.redo_list = reinterpret_cast<uint32_t*>(c->ws + off_sr);
        cp.redo_count = cnt + 13;
        cp.stats = c->spread_stamps;
        cp.max_count = c->heavy_stage == 2 ? (uint32_t)c->coop_max : 0xFFFFFFFFu;
        HIP_TRY(c, launch_coop(cp, (uint32_t)c->coop_grid, s), "coop launch");
        c->last_sp_hist = nullptr;
    }
    if (use_spread) {
        SpreadArgs sp{};
        sp.s = a;
        sp.s.giant_list = nullptr;      // the spread stage holds every compact history
        sp.s.partials = part + (g0r + (coop ? c->coop_grid : 0)) * T_N;
        sp.heavy_list = lh;
        sp.min_count = c->heavy_stage == 2 ? (uint32_t)c->coop_max + 1u : 0u;
        sp.heavy_count = cnt + 4;
        sp.tasks = reinterpret_cast<SpreadTask*>(c->spt);
        sp.cap = (uint32_t)sp_cap;
        if (++c->epoch == 0) ++c->epoch;
        sp.epoch = c->epoch;
        sp.hist = reinterpret_cast<SpreadHist*>(c->ws + off_sh);
        sp.ad = reinterpret_cast<unsigned long long*>(cnt + 16);
        sp.head = cnt + 18;
        sp.task_budget = c->spread_budget;
        sp.min_pending = (uint32_t)c->spread_pending;
        sp.stamps = c->spread_stamps;
        sp.explore_cap = max_nodes ? 16 * max_nodes + 4 * c->spread_budget : 0;
        sp.redo_list = reinterpret_cast<uint32_t*>(c->ws + off_sr);
        sp.redo_count = cnt + 13;
        HIP_TRY(c, launch_spread(sp, (uint32_t)c->spread_grid, s), "spread launch");
        c->last_sp_hist = sp.hist;
        c->last_sp_count = sp.heavy_count;
        c->last_sp_ad = sp.ad;
    }
    if ((spread && !memo0) || grp_redo) {
        SearchArgs ar = a;              // exact per-lane search, no split
        ar.giant_list = nullptr;
        ar.list = reinterpret_cast<uint32_t*>(c->ws + off_sr);
        ar.list_count = cnt + 13;
        ar.queue_head = cnt + 14;
        ar.partials = part + (g0r + g_heavy) * T_N;
        HIP_TRY(c, launch_refill(ar, kRedoGrid, s), "redo launch");
    }
    // stage 0w: histories with 33..64 events in the compact layout (u64 masks)
    uint32_t* l1_in = l0;
    uint32_t* l1_cnt = cnt + 0;
    if (gw0) {
        SearchArgs aw = a;
        aw.list = l0;
        aw.list_count = cnt + 0;
        aw.defer_list = reinterpret_cast<uint32_t*>(c->ws + off_lw);
        aw.defer_count = cnt + 23;
        aw.partials = part + (g0r + g0b) * T_N;
        uint32_t* lwh = reinterpret_cast<uint32_t*>(c->ws + off_lwh);
        if (heavy_w) {                  // over the budget: -> coop64
            aw.heavy_list = lwh;
            aw.heavy_count = cnt + 24;
            aw.stage0_budget = c->stage0w_budget;
            if (memo_w && c->cut_k) {   // stragglers -> the memo stage as well
                aw.cut_k = (uint32_t)c->cut_k;
                aw.cut_min = (uint32_t)c->cut_min;
            }
        } else if (split) {             // as stage 0 without a budget: -> split
            aw.heavy_list = lg;
            aw.heavy_count = cnt + 7;
            aw.stage0_budget = c->split_budget;
        }
        HIP_TRY(c, launch_compact64(aw, (uint32_t)gw0, s), "stage 0w launch");
        if (memo_w) {
            MemoArgs mp{};
            mp.s = a;
            mp.s.giant_list = nullptr;
            mp.s.list = lwh;
            mp.s.list_count = cnt + 24;
            mp.s.partials = part + (g0r + g0b + gw0) * T_N;
            mp.table = reinterpret_cast<uint32_t*>(c->mt + (size_t)mt_slots * 32);
            mp.entries = (uint32_t)c->mt_entries;
            mp.min_rem = (uint32_t)c->memo_min_rem;
            mp.epoch = c->mt_epoch;
            mp.stats = c->memo_stats;
            HIP_TRY(c, launch_memo(mp, (uint32_t)g_mw, true, s), "memo64 launch");
        } else if (heavy_w) {
            // one wavefront per heavy history; one that explores more than the
            // cap goes to the split stage (giants), or to an exact per-lane redo
            CoopArgs cp{};
            cp.s = a;
            cp.s.giant_list = nullptr;
            cp.s.partials = part + (g0r + g0b + gw0) * T_N;
            cp.heavy_list = lwh;
            cp.heavy_count = cnt + 24;
            cp.next = cnt + 25;
            cp.budget = c->coop_budget;
            cp.max_count = 0xFFFFFFFFu;
            cp.stats = c->spread_stamps;    // diagnostic counters (spread_stamps_ptr)
            if (split) {
                cp.explore_cap = 64 * c->split_budget;
                if (max_nodes) cp.explore_cap = std::min<uint64_t>(cp.explore_cap, 16 * max_nodes + 64 * c->coop_budget);
                cp.redo_list = lg;
                cp.redo_count = cnt + 7;
            } else {
                cp.explore_cap = max_nodes ? 16 * max_nodes + 64 * c->coop_budget : 0;
                cp.redo_list = reinterpret_cast<uint32_t*>(c->ws + off_lwr);
                cp.redo_count = cnt + 26;
            }
            HIP_TRY(c, launch_coop64(cp, (uint32_t)c->coop64_grid, s), "coop64 launch");
            if (!split) {
                SearchArgs ar = a;      // exact per-lane search, no budget
                ar.giant_list = nullptr;
                ar.list = cp.redo_list;
                ar.list_count = cp.redo_count;
                ar.defer_list = aw.defer_list;      // never written: stage 0w held them
                ar.defer_count = aw.defer_count;
                ar.partials = part + (g0r + g0b + gw0 + c->coop64_grid) * T_N;
                HIP_TRY(c, launch_compact64(ar, kRedoGrid, s), "coop64 redo launch");
            }
        }
        l1_in = aw.defer_list;
        l1_cnt = aw.defer_count;
    }
    // stage 1: histories with 33..64 events (wide values)
    SearchArgs a1 = a;
    a1.list = l1_in;
    a1.list_count = l1_cnt;
    a1.defer_list = l1;
    a1.defer_count = cnt + 1;
    a1.partials = part + (g0r + g0b + gw) * T_N;
    HIP_TRY(c, launch_stage(1, a1, kStage1Grid, s), "stage 1 launch");
    // stage 2: up to 128 events / 128 pids
    SearchArgs a2 = a;
    a2.list = l1;
    a2.list_count = cnt + 1;
    a2.defer_list = l0;            // never written: stage 2 holds every valid history
    a2.defer_count = cnt + 3;
    a2.partials = part + (g0r + g0b + gw + kStage1Grid) * T_N;
    HIP_TRY(c, launch_stage(2, a2, kStage2Grid, s), "stage 2 launch");
    if (split) {
        SplitArgs p{};
        p.s = a;
        p.s.partials = part + (g0r + g0b + gw + kStage1Grid + kStage2Grid) * T_N;
        p.giant_list = lg;
        p.giant_count = cnt + 7;
        p.giants = reinterpret_cast<GiantRec*>(c->ws + off_gr);
        p.tasks = reinterpret_cast<qsmd_task*>(c->ws + off_tk);
        p.task_count = cnt + 8;
        p.queue_head = cnt + 10;
        p.task_cap = kTaskCap;
        p.target = kSplitTarget;
        p.max_tasks = kSplitMaxTasks;
        p.max_depth = QSMD_SPLIT_MAX_DEPTH;
        p.task_status = reinterpret_cast<uint8_t*>(c->ws + off_ts);
        p.task_nodes = reinterpret_cast<uint64_t*>(c->ws + off_tn);
        p.task_witness = want_w ? reinterpret_cast<uint8_t*>(c->ws + off_tw) : nullptr;
        if (flags & QSMD_FLAG_MEMO) {
            rc = memo_prepare(c, s, &p.memo);
            if (rc) return rc;
            p.memo_mask = c->memo_alloc - 1;
        } else if (c->split_xmemo) {    // exact-count memo for the giants' tasks (the reference's counts)
            const size_t need = (size_t)kXMemoEntries * 128;
            if (c->xm_bytes < need) {
                rc = grow(c, &c->xm, &c->xm_bytes, need);
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
        for (int v = 0; v < SPLIT_VARIANTS; ++v)
            HIP_TRY(c, launch_frontier(v, p, kFrontierGrid, s), "frontier launch");
        for (int v = 0; v < SPLIT_VARIANTS; ++v)
            HIP_TRY(c, launch_tasks(v, p, kTaskGrid[v], s), "task launch");
        HIP_TRY(c, launch_combine(p, kCombineGrid, s), "combine launch");
    }
    if (early) {
        unsigned long long* pf = part + (g0r + g0b + gw + kStage1Grid + kStage2Grid + gsp) * T_N;
        HIP_TRY(c, launch_early_exit_fixup(status, nodes, n_hist, cnt + 6, pf, (uint32_t)gfx, s), "fixup launch");
        HIP_TRY(c, launch_reduce(pf, gfx, tot, s), "reduce launch");
    } else {
        HIP_TRY(c, launch_reduce(part, n_part, tot, s), "reduce launch");
    }
    HIP_TRY(c, hipEventRecord(evs[2], s), "hipEventRecord");
    if (probe) {                        // heavy mode: the heavy list is the probe
        // long searches: finished ones over kAutoProbe nodes + the ones over the budget
        // (one copy of the 32 stage counters: [4] heavy list, [22] long finished, [28] cut)
        HIP_TRY(c, hipMemcpyAsync(c->probe_host, cnt, 128, hipMemcpyDeviceToHost, s), "probe read-back");
        c->probe_spread = spread;
        HIP_TRY(c, hipEventRecord(c->probe_ev, s), "hipEventRecord");
        c->probe_pending = true;
        c->probe_n_hist = n_hist;
    }
    c->n_calls++;
    c->timed = true;
    return QSMD_OK;
}

int qsmd_check_batch_device(qsmd_ctx* c, uint32_t model_id, const qsmd_hdr* hdr_dev, uint64_t n_hist,
                            const qsmd_event* events_dev, uint64_t n_events, const void* model0_host,
                            uint32_t flags, uint64_t max_nodes, uint8_t* status_dev, uint64_t* nodes_dev,
                            uint8_t* witness_dev, qsmd_totals* totals_dev, void* stream) {
    if (!c) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    return check_device_locked(c, model_id, hdr_dev, n_hist, events_dev, n_events, model0_host, flags,
                               max_nodes, status_dev, nodes_dev, witness_dev, totals_dev, s);
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
    hipStream_t s = c->stream;
    const bool want_w = (flags & QSMD_FLAG_WITNESS) && witness_out;
    const size_t o_hdr = 0;
    const size_t o_ev = o_hdr + align_up(n_hist * sizeof(qsmd_hdr));
    const size_t o_st = o_ev + align_up(n_events * sizeof(qsmd_event));
    const size_t o_nd = o_st + align_up(n_hist);
    const size_t o_w = o_nd + align_up(n_hist * 8);
    const size_t o_tot = o_w + align_up(want_w ? n_events : 0);
    const size_t need = o_tot + align_up(sizeof(qsmd_totals));
    int rc = grow(c, &c->io, &c->io_bytes, need);
    if (rc) return rc;
    auto* d_hdr = reinterpret_cast<qsmd_hdr*>(c->io + o_hdr);
    auto* d_ev = reinterpret_cast<qsmd_event*>(c->io + o_ev);
    auto* d_st = reinterpret_cast<uint8_t*>(c->io + o_st);
    auto* d_nd = reinterpret_cast<uint64_t*>(c->io + o_nd);
    auto* d_w = reinterpret_cast<uint8_t*>(c->io + o_w);
    auto* d_tot = reinterpret_cast<qsmd_totals*>(c->io + o_tot);
    if (n_hist) HIP_TRY(c, hipMemcpyAsync(d_hdr, hdr, n_hist * sizeof(qsmd_hdr), hipMemcpyHostToDevice, s), "H2D hdr");
    if (n_events) HIP_TRY(c, hipMemcpyAsync(d_ev, events, n_events * sizeof(qsmd_event), hipMemcpyHostToDevice, s), "H2D events");
    if (want_w) HIP_TRY(c, hipMemsetAsync(d_w, 0xFF, n_events, s), "memset witness");
    rc = check_device_locked(c, model_id, d_hdr, n_hist, d_ev, n_events, model0, flags, max_nodes, d_st, d_nd,
                             want_w ? d_w : nullptr, d_tot, s);
    if (rc) return rc;
    if (n_hist) HIP_TRY(c, hipMemcpyAsync(status_out, d_st, n_hist, hipMemcpyDeviceToHost, s), "D2H status");
    if (n_hist && nodes_out) HIP_TRY(c, hipMemcpyAsync(nodes_out, d_nd, n_hist * 8, hipMemcpyDeviceToHost, s), "D2H nodes");
    if (want_w) HIP_TRY(c, hipMemcpyAsync(witness_out, d_w, n_events, hipMemcpyDeviceToHost, s), "D2H witness");
    qsmd_totals t{};
    HIP_TRY(c, hipMemcpyAsync(&t, d_tot, sizeof t, hipMemcpyDeviceToHost, s), "D2H totals");
    HIP_TRY(c, hipStreamSynchronize(s), "hipStreamSynchronize");
    if (totals_out) *totals_out = t;
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
                          stream ? static_cast<hipStream_t>(stream) : c->stream), "gen launch");
    return QSMD_OK;
}

int qsmd_wellformed_batch_device(qsmd_ctx* c, const qsmd_hdr* hdr_dev, uint64_t n_hist, const qsmd_event* events_dev,
                                 uint64_t n_events, const uint8_t* pids, uint32_t n_pids, qsmd_wf* out_dev,
                                 void* stream) {
    if (!c) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    return wellformed_locked(c, hdr_dev, n_hist, events_dev, n_events, pids, n_pids, out_dev,
                             stream ? static_cast<hipStream_t>(stream) : c->stream);
}

int qsmd_wellformed_batch(qsmd_ctx* c, const qsmd_hdr* hdr, uint64_t n_hist, const qsmd_event* events,
                          uint64_t n_events, const uint8_t* pids, uint32_t n_pids, qsmd_wf* out) {
    if (!c) return QSMD_ERR_ARG;
    if (n_hist && (!hdr || !out)) return fail(c, QSMD_ERR_ARG, "null hdr/out");
    if (n_events && !events) return fail(c, QSMD_ERR_ARG, "null events");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    hipStream_t s = c->stream;
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
    if (!c->timed || c->n_calls == 0) return fail(c, QSMD_ERR_ARG, "no check call yet");
    hipEvent_t* evs = &c->ev[3 * ((c->n_calls - 1) % kTimingSlots)];
    HIP_TRY(c, hipEventSynchronize(evs[2]), "hipEventSynchronize");
    HIP_TRY(c, hipEventElapsedTime(ms, evs[0], evs[2]), "hipEventElapsedTime");
    return QSMD_OK;
}

int qsmd_timing_reset(qsmd_ctx* c) {
    if (!c) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    c->n_calls = 0;
    return QSMD_OK;
}

int qsmd_timing_read(qsmd_ctx* c, float* stage0_ms, float* call_ms, uint64_t max, uint64_t* n_out) {
    if (!c || !n_out) return QSMD_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const uint64_t n = std::min<uint64_t>(std::min<uint64_t>(c->n_calls, kTimingSlots), max);
    const uint64_t first = c->n_calls - n;
    for (uint64_t i = 0; i < n; ++i) {
        hipEvent_t* evs = &c->ev[3 * ((first + i) % kTimingSlots)];
        HIP_TRY(c, hipEventSynchronize(evs[2]), "hipEventSynchronize");
        if (stage0_ms) HIP_TRY(c, hipEventElapsedTime(&stage0_ms[i], evs[0], evs[1]), "elapsed");
        if (call_ms) HIP_TRY(c, hipEventElapsedTime(&call_ms[i], evs[0], evs[2]), "elapsed");
    }
    *n_out = n;
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
    hipStream_t s = c->stream;
    const uint64_t cap = std::max<uint64_t>(max_tasks, 1);
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
    HIP_TRY(c, hipMemsetAsync(cnt, 0, 64, s), "memset counters");
    HIP_TRY(c, hipMemsetAsync(c->sx + o_gl, 0, 4, s), "memset giant list");
    HIP_TRY(c, hipMemcpyAsync(cnt + 7, &one, 4, hipMemcpyHostToDevice, s), "H2D giant count");
    a.hdr = reinterpret_cast<const qsmd_hdr*>(c->sx + o_hdr);
    a.events = reinterpret_cast<const uint2*>(c->sx + o_ev);
    a.n_hist = 1;
    a.n_events = n_events;
    a.flags = flags;
    a.model_id = model_id;
    a.max_nodes = max_nodes;
    a.time_limit = c->time_limit_ms * 100000ull;
    a.timed_out = cnt + 2;
    a.witness = witness_out ? reinterpret_cast<uint8_t*>(c->sx + o_w) : nullptr;
    SplitArgs p{};
    p.s = a;
    p.giant_list = reinterpret_cast<const uint32_t*>(c->sx + o_gl);
    p.giant_count = cnt + 7;
    p.giants = reinterpret_cast<GiantRec*>(c->sx + o_gr);
    p.tasks = reinterpret_cast<qsmd_task*>(c->sx + o_tk);
    p.task_count = cnt + 8;
    p.queue_head = cnt + 10;
    p.task_cap = (uint32_t)cap;
    p.target = std::max<uint32_t>(min_tasks, 1);
    p.max_tasks = (uint32_t)max_tasks;
    p.max_depth = QSMD_SPLIT_MAX_DEPTH;
    for (int v = 0; v < SPLIT_VARIANTS; ++v) HIP_TRY(c, launch_frontier(v, p, 1, s), "frontier launch");
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
    hipStream_t s = c->stream;
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
    uint32_t counts[16] = {};
    counts[8 + v] = (uint32_t)n;
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
    a.timed_out = cnt + 2;
    SplitArgs p{};
    p.s = a;
    p.giants = reinterpret_cast<GiantRec*>(c->sx + o_gr);
    p.tasks = d_tk;
    p.task_count = cnt + 8;
    p.queue_head = cnt + 10;
    p.task_cap = (uint32_t)n;
    p.task_status = reinterpret_cast<uint8_t*>(c->sx + o_ts);
    p.task_nodes = reinterpret_cast<uint64_t*>(c->sx + o_tn);
    p.task_witness = want_w ? reinterpret_cast<uint8_t*>(c->sx + o_tw) : nullptr;
    p.external_tasks = 1;
    if (flags & QSMD_FLAG_MEMO) {
        rc = memo_prepare(c, s, &p.memo);
        if (rc) return rc;
        p.memo_mask = c->memo_alloc - 1;
    }
    HIP_TRY(c, launch_tasks((int)v, p, kTaskGrid[v], s), "task launch");
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
