/*
 * qsmd.h -- C ABI of the MI355X-native linearisability checker.
 *
 * Drop-in boundary for ONE function of advancedtelematic/
 * quickcheck-state-machine-distributed:
 *
 *   linearisable :: Eq pid
 *                => (model -> Either inv resp -> model)      -- transition
 *                -> (model -> inv -> resp -> Bool)           -- postcondition
 *                -> model -> History pid inv resp -> Bool
 *   (src/Linearisability.hs:52-69, exported at :1-7; History at :18)
 *
 * The reference has no FFI; its callers are test/Bank.hs:285,
 * test/TicketDispenser.hs:253 and :320, one call per history.  The binding a
 * Haskell maintainer adds (`foreign import ccall safe "qsmd_check_batch"`) is
 * shown in INTEGRATION.md.  Every entry point below is plain C: caller-owned
 * buffers, plain pointers and sizes, no C++ or torch types.
 *
 * Semantics are bit-exact with the reference search:
 *   - same verdict for every history;
 *   - `nodes` = number of `step` evaluations (src/Linearisability.hs:63) of the
 *     reference's lazy left-to-right short-circuit DFS (exhaustive mode);
 *   - model exceptions (Bank `Map.!`, test/Bank.hs:128) surface as
 *     QSMD_STATUS_MODEL_ERROR exactly when the reference would raise them.
 */
#ifndef QSMD_H
#define QSMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QSMD_ABI_VERSION 3u

/* ---------------------------------------------------------------- layout */

/* One history = one header (16 B) + n_ev events (8 B each) stored
 * contiguously at events[ev_off .. ev_off + n_ev).  Replaces the boxed list
 * `[(pid, Either inv resp)]` of src/Linearisability.hs:18. */
typedef struct qsmd_hdr {
    uint32_t ev_off;    /* index of the first event in the events array      */
    uint16_t n_ev;      /* number of events (<= QSMD_MAX_EVENTS)             */
    uint8_t  n_pid;     /* number of distinct dense pids used (<= 128)       */
    uint8_t  model_id;  /* QSMD_MODEL_* (must equal the call's model_id)     */
    uint32_t tag;       /* caller's tag, ignored by the checker              */
    uint32_t reserved;  /* must be 0                                         */
} qsmd_hdr;

/* One event.  kp = (kind << 7) | pid with kind 0 = Left inv, 1 = Right resp
 * (src/Linearisability.hs:18); pid is the dense per-history pid (the
 * marshaller maps `Eq pid` values to 0..n_pid-1 in order of first use). */
typedef struct qsmd_event {
    uint8_t kp;
    uint8_t code;       /* constructor code, model specific (below)          */
    uint8_t a;          /* Bank: account (dense, < QSMD_BANK_MAX_ACCOUNTS)   */
    uint8_t b;          /* Bank Transfer: destination account                */
    int32_t val;        /* Bank money / Balance; Ticket Number               */
} qsmd_event;

#define QSMD_EV_RESP      0x80u
#define QSMD_EV_PID_MASK  0x7Fu

#define QSMD_MAX_EVENTS   128   /* 64 operations (SURVEY.md §8b encode limit) */
#define QSMD_MAX_PIDS     128

/* ---------------------------------------------------------------- models */

#define QSMD_MODEL_TICKET 1u    /* test/TicketDispenser.hs:51-102          */
#define QSMD_MODEL_BANK   2u    /* test/Bank.hs:41-131                     */

/* TicketDispenser Request / Response (test/TicketDispenser.hs:51-63) */
#define QSMD_TICKET_TAKE_TICKET 0u
#define QSMD_TICKET_RESET       1u
#define QSMD_TICKET_NUMBER      0u   /* Number Int  (val)                  */
#define QSMD_TICKET_OK          1u

/* BankRequestF / BankResponse (test/Bank.hs:44-73) */
#define QSMD_BANK_OPEN_ACCOUNT   0u  /* a                                  */
#define QSMD_BANK_DEPOSIT        1u  /* a, val = money                     */
#define QSMD_BANK_WITHDRAW       2u  /* a, val = money                     */
#define QSMD_BANK_CHECK_BALANCE  3u  /* a                                  */
#define QSMD_BANK_TRANSFER       4u  /* a = from, val = money, b = to      */

#define QSMD_BANK_ACCOUNT_CREATED        0u
#define QSMD_BANK_DEPOSIT_MADE           1u
#define QSMD_BANK_WITHDRAWAL_MADE        2u
#define QSMD_BANK_TRANSFER_MADE          3u
#define QSMD_BANK_ACCOUNT_ALREADY_EXISTS 4u
#define QSMD_BANK_ACCOUNT_DOESNT_EXIST   5u
#define QSMD_BANK_INSUFFICIENT_FUNDS     6u
#define QSMD_BANK_BALANCE                7u  /* Balance Money (val)         */

#define QSMD_BANK_MAX_ACCOUNTS 8

/* Initial models (the `model0` argument).  NULL = the reference's initModel:
 * Nothing (test/TicketDispenser.hs:73-74) / M.empty (test/Bank.hs:86-87). */
typedef struct qsmd_ticket_model {
    uint32_t is_just;   /* 0 = Nothing, 1 = Just n                          */
    uint32_t reserved;
    int64_t  n;         /* must lie in int32 range                          */
} qsmd_ticket_model;

typedef struct qsmd_bank_model {
    uint32_t exists;    /* bit a set <=> account a is a key of the Map      */
    uint32_t reserved;
    int64_t  balance[QSMD_BANK_MAX_ACCOUNTS];  /* int32 range; 0 if absent  */
} qsmd_bank_model;

/* -------------------------------------------------------------- results */

#define QSMD_STATUS_NONLINEARISABLE 0u  /* linearisable ... == False        */
#define QSMD_STATUS_LINEARISABLE    1u  /* == True                          */
#define QSMD_STATUS_MODEL_ERROR     2u  /* reference raises (Map.!)         */
#define QSMD_STATUS_ENCODE_ERROR    3u  /* unknown code, pid/account range, */
                                        /* > QSMD_MAX_EVENTS, bad model_id  */
#define QSMD_STATUS_BUDGET          4u  /* max_nodes reached, undecided     */
#define QSMD_STATUS_SKIPPED         5u  /* QSMD_FLAG_EARLY_EXIT_BATCH       */

#define QSMD_FLAG_EXHAUSTIVE       1u  /* reference search, exact counts    */
#define QSMD_FLAG_MEMO             2u  /* prune known-failing states        */
#define QSMD_FLAG_WITNESS          4u  /* fill witness_out                  */
#define QSMD_FLAG_EARLY_EXIT_BATCH 8u  /* stop at first non-linearisable    */

/* Witness: for a LINEARISABLE history i, witness_out[hdr[i].ev_off + d] is
 * the (history-local) index of the invocation event chosen at depth d of the
 * successful path; the list ends at the first 0xFF (or at n_ev).  Replay:
 * at each step the operation is (pid p of that event, its inv, the first
 * remaining response of p) -- SURVEY.md §8a Lemma L1.  witness_out has as
 * many bytes as the events array. */
#define QSMD_WITNESS_END 0xFFu

typedef struct qsmd_totals {
    uint64_t checked;           /* histories with a decided status         */
    uint64_t linearisable;
    uint64_t nonlinearisable;
    uint64_t model_errors;
    uint64_t encode_errors;
    uint64_t budget;
    uint64_t skipped;
    uint64_t nodes;             /* sum of per-history node counts          */
} qsmd_totals;

/* -------------------------------------------------------------- context */

typedef struct qsmd_ctx qsmd_ctx;

/* Return codes: 0 = ok, < 0 = API / device error (qsmd_last_error). */
#define QSMD_OK              0
#define QSMD_ERR_ARG        -1
#define QSMD_ERR_DEVICE     -2
#define QSMD_ERR_NOMEM      -3
#define QSMD_ERR_UNSUPPORTED -4

/* Bind a context to one HIP device (one process per GPU).  SURVEY.md §8b
 * proposed a device mask; a context serves exactly one device instead, and a
 * process drives several GPUs with one context per device. */
int  qsmd_open(qsmd_ctx** out, int device);
void qsmd_close(qsmd_ctx* ctx);
const char* qsmd_last_error(const qsmd_ctx* ctx);
uint32_t qsmd_abi_version(void);

/* Threading and streams.  Every entry point of one context serialises on the
 * context's mutex, and the check calls of one context are ordered: a call on
 * a stream other than the previous call's first waits (on the device) for
 * that call, because they share the context's device workspace.  Calls that
 * should overlap use one context each (bench.py keeps calls in flight that
 * way).  Contexts share no device state.  A device call on a caller's stream
 * records a completion event on it, and the context's later waits (its next
 * call on another stream, qsmd_close, qsmd_probe_read, qsmd_timed_out, a knob
 * that reallocates) wait for that event, never for the caller's stream or the
 * whole device: the caller may destroy its stream once its own work on it is
 * done. */

/* Check a batch held in HOST memory (the drop-in for one call per history;
 * n_hist = 1 is valid).  Buffers are copied in and out; the library keeps no
 * pointer after return.  max_nodes = 0 means unbounded.  nodes_out,
 * witness_out, totals_out and model0 may be NULL.  Synchronous. */
int qsmd_check_batch(qsmd_ctx* ctx, uint32_t model_id,
                     const qsmd_hdr* hdr, uint64_t n_hist,
                     const qsmd_event* events, uint64_t n_events,
                     const void* model0, uint32_t flags, uint64_t max_nodes,
                     uint8_t* status_out, uint64_t* nodes_out,
                     uint8_t* witness_out, qsmd_totals* totals_out);

/* Same, with every buffer already resident in device memory (HBM) and work
 * enqueued on `stream` (a hipStream_t, NULL = the context's stream, a
 * blocking stream: ordered after the caller's work on the legacy default
 * stream, as HIP orders blocking streams): two to five kernel launches, no
 * host round trip.  totals_dev (device, may be NULL)
 * receives the qsmd_totals of the batch.  Asynchronous: synchronise the
 * stream before reading outputs. */
int qsmd_check_batch_device(qsmd_ctx* ctx, uint32_t model_id,
                            const qsmd_hdr* hdr_dev, uint64_t n_hist,
                            const qsmd_event* events_dev, uint64_t n_events,
                            const void* model0_host, uint32_t flags,
                            uint64_t max_nodes,
                            uint8_t* status_dev, uint64_t* nodes_dev,
                            uint8_t* witness_dev, qsmd_totals* totals_dev,
                            void* stream);

/* Safety net: a search launch whose lanes run longer than this wall time
 * stops and reports QSMD_STATUS_BUDGET for the unfinished histories (default
 * 120000 ms; 0 disables).  Not part of the reference semantics. */
int qsmd_set_time_limit_ms(qsmd_ctx* ctx, uint64_t ms);

/* Tuning knob: cap on the number of workgroups of the first search stage
 * (beyond it each workgroup loops over several groups of 64 histories).
 * Default 65536.  Does not change any result. */
int qsmd_set_stage0_grid(qsmd_ctx* ctx, uint64_t max_blocks);

/* Tuning knob: node budget of the first search stage (0 = none).  A history
 * whose search needs more nodes goes on in the heavy stage (one lane per
 * history with an exact-count state memo, from the saved search state; or
 * one wavefront per history), so one long search does not hold 63 idle
 * lanes.  Default (until set; knob "stage0_budget_auto" 1 restores it):
 * automatic -- 24, or 16 while the context's last finished call sent fewer
 * than 1 in 50 histories to the heavy stage, back to 24 above 1 in 5.
 * Results are unchanged. */
int qsmd_set_stage0_budget(qsmd_ctx* ctx, uint64_t nodes);

/* Tuning knobs by name (none changes a result):
 *   "stage0_budget"     as qsmd_set_stage0_budget
 *   "stage0_budget_auto" 1: the automatic stage-0 budget (the default)
 *   "stage0w_budget"    the same for 33..64-event histories (default: automatic,
 *                       24 when the heavy stage runs in lane mode, 48 in
 *                       wave mode; "stage0w_budget_auto" 1 restores it)
 *   "stage0_grid"       as qsmd_set_stage0_grid
 *   "split_budget"      as qsmd_set_split_budget
 *   "split_xmemo"       1 (default): the giant stage's exact-count memo
 *   "heavy_mode"        2 (default): the heavy stage in lane mode (one lane
 *                       per history, a private memo table per lane) when the
 *                       last finished call sent more than "wave_max"
 *                       (default 16384) histories there, or sent under a
 *                       fifth of its batch and had no wide (65..128-event)
 *                       history; else wave mode (one wavefront per history,
 *                       the state DAG or the DFS in wave-uniform registers,
 *                       an LDS memo per wavefront); 0: always wave mode; 1:
 *                       always lane mode
 *   "memo_lds"          lane mode's memo tables: 1 (default) in LDS when the
 *                       last finished call's heavy histories fit one
 *                       workgroup per CU, else in HBM; 0: always HBM (an
 *                       LDS-table workgroup holds a CU); 2: always LDS
 *   "memo_lds_entries"  the LDS tables' entries per lane, a power of two in
 *                       4..64 (default 64: 128 KB per workgroup; 16: 32 KB)
 *   "memo_grid", "memo_lane_entries"  lane mode: workgroups at most (0 = 12
 *                       per CU), entries per lane (HBM tables: grid x 64 x
 *                       entries x 96 B, grown on demand; the LDS tables hold
 *                       min(memo_lds_entries, entries))
 *   "wave_grid"         wave mode workgroups (0 = the last call's heavy count
 *                       + 25 %, at most 16 per CU; grid-stride beyond)
 *   "wave_min_rem"      wave mode: no memo probe at nodes with at most this
 *                       many remaining events (default 4)
 *   "dag_states"        wave mode: capacity in states of the per-wavefront
 *                       state DAG (default 128, items 4x that; 0 = the DFS
 *                       for every history); a history whose DAG does not fit
 *                       runs the DFS.  A TicketDispenser history whose DAG is
 *                       a chain (every history on one pid) runs as one
 *                       (scalar mask work, no DAG arrays) unless it is 0
 *   "memo_after"        lane mode: the memo probes a search's nodes after
 *                       it counted this many (default 32; its failed
 *                       subtrees are recorded from the start)
 *   "tail_cap", "tail_min"  lane mode: a search still running after tail_cap
 *                       wavefront iterations (default 256; 0 = never) goes to
 *                       a wave-mode launch after the heavy stage and is
 *                       searched there from the root (the state DAG), when
 *                       the last finished call sent at least tail_min
 *                       (default 65536) histories, and a fifth of its batch,
 *                       to the heavy stage (tail_min 0: whatever it sent)
 *   "heavy_buckets"     1 (default): for the same long lists, the heavy
 *                       stage forms its groups of 64 in order of predicted
 *                       work (stage 0 records each heavy history's untried
 *                       candidates on its stack; a counting sort orders the
 *                       list); 0: in list order
 *   "resume_cap"        lane mode: stage 0's saved search states, slots per
 *                       heavy-list shard (0 = automatic: twice the last
 *                       call's heavy count per shard, at least 1024); a heavy
 *                       history past them starts again at the root
 *   "fold"              lane mode: 1 (default) no stage-0w launch after a
 *                       call that deferred nothing to it (the heavy stage
 *                       takes what stage 0 defers on to the giant stage);
 *                       0: every call launches it
 *   "timing_events"     1: record the per-call timing events (qsmd_timing_read,
 *                       qsmd_last_kernel_ms); 0 (default until
 *                       qsmd_timing_reset): none
 *   "giant_grid"        giant stage workgroups (0 = 2 per CU, or 64 when the
 *                       last finished call had no giant history and lane
 *                       mode's fold does not apply)
 *   "wave_stats_ptr", "memo_stats_ptr", "memo_stats_groups"  diagnostics:
 *                       device buffers: wave mode 16 x u64 (DFS iterations
 *                       max / sum, s_memtime cycles max / sum, nodes sum per
 *                       DFS-searched history; DAG-searched histories, their
 *                       cycles max / sum, per-phase cycles, levels;
 *                       tools/wave_stats.py), lane mode per-group
 *                       records (tools/memo_stats.py)
 *   "giant_stall_us"    diagnostic: the workgroup of the giant stage's first
 *                       frontier chunk starts this late (tests of the time
 *                       limit's phase-wait safety net: a giant combined by a
 *                       workgroup that gave up waiting is BUDGET) */
int qsmd_set_param(qsmd_ctx* ctx, const char* name, uint64_t value);

/* Read a knob ("stage0_budget": 0 while automatic, "stage0w_budget_auto", "fold",
 * "heavy_mode", "memo_after", "resume_cap", "tail_cap", "tail_min", "heavy_buckets") or
 * "stage0_budget_last": the stage-0 budget the most recent
 * finished check call ran with (the automatic one included; waits for the
 * context's last call). */
int qsmd_get_param(qsmd_ctx* ctx, const char* name, uint64_t* out);

/* Tuning knob (default 1024): histories the compact stages cannot hold go to
 * the giant stage, which first searches each one in a lane for 16 x this
 * many iterations and otherwise splits it over many lanes (see "Split
 * search" below); the heavy stage hands it a history after 64 x this many
 * iterations.  0 disables the split (every search runs to its end in one
 * lane or wavefront).  Results are unchanged. */
int qsmd_set_split_budget(qsmd_ctx* ctx, uint64_t nodes);

/* QSMD_FLAG_MEMO: the giant stage keeps a table in HBM of search states
 * (remaining events, model) known to fail, shared by every lane searching the
 * same history, and prunes a subtree whose root state is in it.  Verdicts
 * and witnesses are unchanged; node counts of the giant stage's histories
 * become "nodes explored" (fewer than the reference's, and not reproducible
 * from run to run).  Capacity in entries of 64 B, a power of two (default
 * 1 << 22 = 256 MiB, allocated on first use). */
int qsmd_set_memo_capacity(qsmd_ctx* ctx, uint64_t entries);

/* ----------------------------------------------------------- split search
 *
 * One very large history searched by many GPUs.  The
 * reference DFS (src/Linearisability.hs:52-69) is cut at depth `depth`:
 * every node it reaches at that depth (a passed postcondition, i.e. a `step`
 * that recurses) roots a task, its subtree.  Tasks come in the reference's
 * DFS order, each with the number of nodes the reference counts up to and
 * including its root.  Searching the tasks anywhere, in any order, and
 * folding the results in task order (qsmd_combine_tasks) gives the verdict,
 * exhaustive node count and witness of the single search. */
#define QSMD_SPLIT_MAX_DEPTH 16

typedef struct qsmd_task {
    uint32_t hist;          /* history index in the batch (0 for this API)   */
    uint16_t depth;         /* prefix length d (<= QSMD_SPLIT_MAX_DEPTH)     */
    uint16_t reserved;
    uint64_t top_before;    /* reference nodes up to and including the root  */
    uint8_t  path[QSMD_SPLIT_MAX_DEPTH];  /* invocation event chosen at each */
                                          /* prefix level (witness indices)  */
} qsmd_task;

typedef struct qsmd_frontier {
    uint32_t status;        /* the search above the cut: NONLINEARISABLE =   */
                            /* exhausted (the tasks decide); LINEARISABLE /  */
                            /* MODEL_ERROR = decided after top_nodes unless  */
                            /* a task decides first; BUDGET; ENCODE_ERROR    */
    uint32_t depth;         /* cut depth chosen                              */
    uint64_t top_nodes;     /* nodes counted above the cut                   */
    uint64_t n_tasks;
} qsmd_frontier;

/* Cut the search of ONE history (hdr[0]) at the smallest depth that yields
 * at least min_tasks tasks (at most max_tasks, depth <= 16).  witness_out
 * (n_ev bytes, may be NULL) receives the path when the search above the cut
 * ends LINEARISABLE. */
int qsmd_split_frontier(qsmd_ctx* ctx, uint32_t model_id, const qsmd_hdr* hdr,
                        const qsmd_event* events, uint64_t n_events,
                        const void* model0, uint32_t flags, uint64_t max_nodes,
                        uint32_t min_tasks, qsmd_task* tasks_out, uint64_t max_tasks,
                        qsmd_frontier* frontier_out, uint8_t* witness_out);

/* Search the subtrees of tasks[0..n_tasks) of history hdr[0] (tasks in DFS
 * order; any subset of a frontier, kept in order).  Per task: status
 * LINEARISABLE = the subtree holds a linearisation, NONLINEARISABLE = it
 * does not, MODEL_ERROR, BUDGET, SKIPPED = not searched because an earlier
 * task of this call decided; nodes = nodes of the subtree below its root
 * up to its decision; witness_out (n_tasks x 64 B, may be NULL) = the full
 * path of a LINEARISABLE task.  QSMD_FLAG_MEMO applies. */
int qsmd_check_tasks(qsmd_ctx* ctx, uint32_t model_id, const qsmd_hdr* hdr,
                     const qsmd_event* events, uint64_t n_events,
                     const void* model0, uint32_t flags, uint64_t max_nodes,
                     const qsmd_task* tasks, uint64_t n_tasks,
                     uint8_t* status_out, uint64_t* nodes_out, uint8_t* witness_out);

/* Fold task results in DFS order (host only, no device).  winner_out = index
 * of the deciding task, -1 when the decision came from above the cut. */
int qsmd_combine_tasks(const qsmd_frontier* frontier, const qsmd_task* tasks,
                       const uint8_t* status, const uint64_t* nodes, uint64_t n_tasks,
                       uint64_t max_nodes, uint8_t* status_out, uint64_t* nodes_out,
                       int64_t* winner_out);

/* ------------------------------------------------------------ wellformed
 *
 * Batched `wellformed pids history` (src/Linearisability.hs:97-135; call
 * site test/Bank.hs:281-283): every listed pid's subhistory must be
 * sequential; the result is the first NotSequential error in `pids` order,
 * as the constructor code, the pid and the history-local indices of the
 * events it names (ev0 = the first, ev1 = the second; equal when it names
 * one).  InvocationFollowedByNonMatchingResponse compares the pids of one
 * subhistory, which are equal, so wellformed never returns it. */
typedef struct qsmd_wf {
    uint8_t  code;      /* QSMD_WF_*                                         */
    uint8_t  pid;       /* dense pid of the failing subhistory               */
    uint16_t ev0;
    uint16_t ev1;
    uint16_t reserved;
} qsmd_wf;

#define QSMD_WF_OK                                         0u
#define QSMD_WF_FIRST_EVENT_ISNT_INVOCATION                1u
#define QSMD_WF_INVOCATION_FOLLOWED_BY_INVOCATION          2u
#define QSMD_WF_INVOCATION_FOLLOWED_BY_NON_MATCHING_RESPONSE 3u
#define QSMD_WF_RESPONSE_FOLLOWED_BY_RESPONSE              4u
#define QSMD_WF_RESPONSE_FOLLOWED_BY_INVOCATION            5u
#define QSMD_WF_LONE_RESPONSE                              6u
#define QSMD_WF_ENCODE_ERROR                               0xFEu

/* pids: the `pids` list as dense pid indices (< 128, each at most once),
 * applied to every history; NULL = all pids in order 0, 1, 2, ...
 * Host buffers, synchronous. */
int qsmd_wellformed_batch(qsmd_ctx* ctx, const qsmd_hdr* hdr, uint64_t n_hist,
                          const qsmd_event* events, uint64_t n_events,
                          const uint8_t* pids, uint32_t n_pids, qsmd_wf* out);
/* Same on device-resident hdr / events / out, enqueued on `stream`. */
int qsmd_wellformed_batch_device(qsmd_ctx* ctx, const qsmd_hdr* hdr_dev, uint64_t n_hist,
                                 const qsmd_event* events_dev, uint64_t n_events,
                                 const uint8_t* pids, uint32_t n_pids, qsmd_wf* out_dev,
                                 void* stream);

/* Device time (ms, HIP events on the launch stream) of the search kernels of
 * the most recent timed check call, measured once that stream has completed.
 * Timing is off until qsmd_timing_reset (or knob "timing_events" 1): the
 * events are three packets per call on the caller's stream. */
int qsmd_last_kernel_ms(qsmd_ctx* ctx, float* ms_out);

/* Per-call device timings since the last reset, which also turns timing on
 * (at most the last 1024 calls):
 * stage0_ms[i] = the first (dominant) search kernel (0 when the host entry
 * skipped stage 0: no history of the call fitted it), call_ms[i] = every
 * kernel of call i.  Synchronises on the recorded events. */
int qsmd_timing_reset(qsmd_ctx* ctx);
int qsmd_timing_read(qsmd_ctx* ctx, float* stage0_ms, float* call_ms, uint64_t max,
                     uint64_t* n_out);
/* The same with heavy_ms[i] = the heavy-stage kernel of call i in lane mode
 * (events the launch records at its start and end; -1 in wave mode).  Any of
 * the three arrays may be NULL. */
int qsmd_timing_read_stages(qsmd_ctx* ctx, float* stage0_ms, float* heavy_ms, float* call_ms,
                            uint64_t max, uint64_t* n_out);

/* Diagnostic: out4 = [histories stage 0 passed to stage 0w, heavy histories
 * of stage 0, heavy histories of stage 0w, giants] of the most recent check
 * call (waits for it). */
int qsmd_probe_read(qsmd_ctx* ctx, uint32_t* out4);

/* Whether the time limit (qsmd_set_time_limit_ms) fired in the most recent
 * check call (waits for it): *out = 1 when some of its QSMD_STATUS_BUDGET
 * results come from the time limit rather than max_nodes, else 0. */
int qsmd_timed_out(qsmd_ctx* ctx, int* out);

#ifdef __cplusplus
}
#endif

#endif /* QSMD_H */
